// buffer_ops.cpp -- TEST FIXTURE: ManagedBuffer<T>::fill (reference include/cpp/vkt/
// ManagedBuffer.hpp:257, reached by Array1D/2D/3D::fill) with element types of 1 to 300 bytes,
// compiled against the public C++ header like a user's translation unit.  Under the GPU
// policy fill() migrates the buffer to HBM and calls MemsetRange (vktHipMemsetRange's
// kernels), which repeats the element bytes over the buffer.
#include "volkit.hpp"
#include "volkit_hip.h"

#include <cstdint>
#include <cstring>

namespace
{
    template <int N>
    struct Elem
    {
        uint8_t b[N];
    };

    template <class T>
    struct FillableBuffer : vkt::ManagedBuffer<T>
    {
        explicit FillableBuffer(std::size_t n) : vkt::ManagedBuffer<T>(n) {}
        using vkt::ManagedBuffer<T>::fill;
        T* raw()
        {
            this->migrate();
            return this->data_;
        }
    };

    template <int N>
    int fillAndRead(std::size_t count, uint8_t const* pattern, uint8_t* out)
    {
        vkt::ExecutionPolicy saved = vkt::GetThreadExecutionPolicy();
        vkt::ExecutionPolicy gpu = saved;
        gpu.device = vkt::ExecutionPolicy::Device::GPU;
        vkt::SetThreadExecutionPolicy(gpu);
        int rc = 0;
        {
            FillableBuffer<Elem<N>> buf(count);   // allocated in HBM (GPU policy)
            Elem<N> value;
            std::memcpy(value.b, pattern, N);
            buf.fill(value);
            vkt::Memcpy(out, buf.raw(), count * N, vkt::CopyKind::DeviceToHost);
        }
        vkt::SetThreadExecutionPolicy(saved);
        return rc;
    }
} // namespace

extern "C" {

// Fills `count` elements of `elemBytes` bytes each with `pattern` through ManagedBuffer::fill
// on the GPU and copies the buffer to `out` (count * elemBytes bytes).  Returns -100 for an
// element size this fixture does not instantiate.
int vktt_managed_fill(int elemBytes, size_t count, uint8_t const* pattern, uint8_t* out)
{
    switch (elemBytes)
    {
    case 1: return fillAndRead<1>(count, pattern, out);
    case 2: return fillAndRead<2>(count, pattern, out);
    case 3: return fillAndRead<3>(count, pattern, out);
    case 4: return fillAndRead<4>(count, pattern, out);
    case 8: return fillAndRead<8>(count, pattern, out);
    case 16: return fillAndRead<16>(count, pattern, out);
    case 17: return fillAndRead<17>(count, pattern, out);
    case 256: return fillAndRead<256>(count, pattern, out);
    case 300: return fillAndRead<300>(count, pattern, out);
    default: return -100;
    }
}

// ManagedBuffer<uint32_t>::fill under the GPU policy on a buffer allocated under the CPU policy
// whose migration to HBM fails (test knob memory.fail_next_alloc): the buffer stays in host
// memory (the same pointer), and fill() must write the pattern there -- the host pattern loop
// of MemsetRange_serial (reference src/vkt/Memory_serial.hpp:24-37) -- not launch the pattern
// kernel on the pageable pointer.  Copies the host bytes to `out` (count * 4 bytes).
// Returns 0, or -1 when the buffer moved (the knob did not fail the allocation), -2 when the
// buffer is not host-resident after fill().
int vktt_fill_after_failed_migration(size_t count, uint32_t pattern, uint8_t* out)
{
    vkt::ExecutionPolicy saved = vkt::GetThreadExecutionPolicy();
    vkt::ExecutionPolicy cpu = saved, gpu = saved;
    cpu.device = vkt::ExecutionPolicy::Device::CPU;
    gpu.device = vkt::ExecutionPolicy::Device::GPU;
    vkt::SetThreadExecutionPolicy(cpu);
    int rc = 0;
    {
        FillableBuffer<uint32_t> buf(count);   // host memory (CPU policy)
        uint32_t* const host = buf.raw();
        std::memset(host, 0xEE, count * 4);
        vktHipSetTuningKnob("memory.fail_next_alloc", 1);
        vkt::SetThreadExecutionPolicy(gpu);
        buf.fill(pattern);                     // migrate() fails: the bytes stay on the host
        vkt::SetThreadExecutionPolicy(cpu);
        vktHipSetTuningKnob("memory.fail_next_alloc", 0);
        if (!buf.residentOn(cpu))
            rc = -2;
        else if (buf.raw() != host)
            rc = -1;
        else
            std::memcpy(out, host, count * 4);
    }
    vkt::SetThreadExecutionPolicy(saved);
    return rc;
}

} // extern "C"
