// HipContext.cpp -- process-wide HIP context: device, compute/copy streams, errors, timing.
//
// Realises the design intent of the reference's declared-but-undefined CUDA context API
// (reference include/c/vkt/CudaContext.h:17-65: async execution flag, compute and copy
// stream ids) as the vktHip* runtime functions of include/volkit_hip.h.

#include "Runtime.hpp"

#include <rocprofiler-sdk-roctx/roctx.h>
#include "volkit_hip.h"

#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <algorithm>
#include <mutex>
#include <vector>

namespace vkt
{
namespace rt
{
    namespace
    {
        struct Context
        {
            std::mutex mutex;
            bool initialised = false;
            int device = -1;              // requested device, -1 = current at first use
            hipStream_t ownCompute = nullptr;
            hipStream_t userCompute = nullptr;
            bool userStreamSet = false;
            hipStream_t copy = nullptr;
            hipStream_t userCopy = nullptr;
            bool userCopySet = false;
            std::atomic<int> async{1};
            std::atomic<int> timing{0};
        };

        Context& ctx()
        {
            static Context* c = new Context;   // intentionally leaked: no teardown-order issues
            return *c;
        }

        thread_local std::string tlsLastError;
        thread_local float tlsLastKernelMs = 0.f;

        int logLevelFromEnv()
        {
            char const* s = std::getenv("VKT_LOG_LEVEL");
            if (s == nullptr)
                return 2;
            return std::atoi(s);
        }

        void initLocked(Context& c)
        {
            if (c.initialised)
                return;
            if (c.device >= 0)
                (void)hipSetDevice(c.device);
            else
                (void)hipGetDevice(&c.device);
            // Blocking streams: they synchronise with the NULL stream, so user code that
            // hipMemcpy's from getData() pointers sees finished kernels, exactly as with the
            // reference's legacy-default-stream launches.
            (void)hipStreamCreateWithFlags(&c.ownCompute, hipStreamDefault);
            (void)hipStreamCreateWithFlags(&c.copy, hipStreamDefault);
            c.initialised = true;
        }
    } // namespace

    LogStream::~LogStream()
    {
        static int const threshold = logLevelFromEnv();
        if (static_cast<int>(level_) > threshold)
            return;
        static char const* const tag[] = {"\033[1;31m[volkit error]\033[0m ", "\033[1;33m[volkit warning]\033[0m ",
                                          "[volkit] "};
        std::string msg = tag[static_cast<int>(level_)] + stream_.str() + "\n";
        std::fwrite(msg.data(), 1, msg.size(), stdout);
        std::fflush(stdout);
    }

    hipStream_t computeStream()
    {
        Context& c = ctx();
        std::lock_guard<std::mutex> lock(c.mutex);
        initLocked(c);
        return c.userStreamSet ? c.userCompute : c.ownCompute;
    }

    hipStream_t copyStream()
    {
        Context& c = ctx();
        std::lock_guard<std::mutex> lock(c.mutex);
        initLocked(c);
        return c.userCopySet ? c.userCopy : c.copy;
    }

    bool asyncExecution() { return ctx().async.load() != 0; }

    int device()
    {
        Context& c = ctx();
        std::lock_guard<std::mutex> lock(c.mutex);
        initLocked(c);
        return c.device;
    }

    void setLastError(std::string const& msg) { tlsLastError = msg; }

    namespace
    {
        thread_local std::string tlsMigrationFailure;
    }

    void noteMigrationFailure(std::string const& msg)
    {
        tlsMigrationFailure = msg;
        (void)fail(msg.c_str());
    }

    std::string takeMigrationFailure()
    {
        std::string m;
        m.swap(tlsMigrationFailure);
        return m;
    }

    vktError explainFailure(vktError e, char const* name)
    {
        std::string const m = takeMigrationFailure();
        if (e != vktNoError && !m.empty())
            setLastError(std::string(name) + ": " + m);
        return e;
    }

    vktError check(hipError_t err, char const* what)
    {
        if (err == hipSuccess)
            return vktNoError;
        std::string msg = std::string(what) + ": " + hipGetErrorString(err);
        setLastError(msg);
        VKT_LOG(LogLevel::Error) << msg;
        return vktInvalidValue;
    }

    vktError fail(char const* what)
    {
        setLastError(what);
        VKT_LOG(LogLevel::Error) << what;
        return vktInvalidValue;
    }

    vktError finishLaunch(char const* what)
    {
        vktError e = check(hipGetLastError(), what);
        if (e != vktNoError)
            return e;
        if (!asyncExecution())
            return check(hipStreamSynchronize(computeStream()), what);
        return vktNoError;
    }

    void* StreamScratch::acquire(std::size_t bytes, hipStream_t stream)
    {
        m_.lock();
        if (pending_ && (stream != last_ || cap_ < bytes))   // growing frees the old buffer
        {
            (void)check(hipEventSynchronize(done_), "hipEventSynchronize(scratch)");
            pending_ = false;
        }
        if (!done_ && check(hipEventCreateWithFlags(&done_, hipEventDisableTiming), "hipEventCreate") != vktNoError)
        {
            m_.unlock();
            return nullptr;
        }
        if (cap_ < bytes)
        {
            if (p_)
                (void)check(hipFree(p_), "hipFree(scratch)");
            p_ = nullptr;
            cap_ = 0;
            if (check(hipMalloc(&p_, bytes), "hipMalloc(scratch)") != vktNoError)
            {
                p_ = nullptr;
                m_.unlock();
                return nullptr;
            }
            cap_ = bytes;
        }
        return p_;
    }

    void StreamScratch::release(hipStream_t stream)
    {
        if (check(hipEventRecord(done_, stream), "hipEventRecord(scratch)") == vktNoError)
        {
            pending_ = true;
            last_ = stream;
        }
        m_.unlock();
    }

    bool kernelTimingEnabled() { return ctx().timing.load() != 0; }

    namespace
    {
        struct KnobDef
        {
            char const* name;
            int64_t def;
        };
        constexpr KnobDef kKnobs[] = {
            {"pointwise.padded_rows", 1},
            {"pointwise.max_quanta_per_launch", int64_t(1) << 20},
            {"pointwise.general", 1},
            {"pointwise.merge_sectors", 1},
            {"pointwise.general_32bit", 1},
            {"histogram.packed16", 2},
            {"histogram.mulshift", 1},
            {"histogram.p16_step", 1},
            {"pointwise.u8_pairs", 1},
            {"render.bricks", 1},
            {"decompose.aligned_lds", 5},
            {"decompose.stage_words", 6},
            {"pointwise.u8_wide", 1},
            {"pointwise.f32_halves", 1},
            {"pointwise.f32_wide", 2},
            {"aggregates.codes", 3},
            {"reduce.u8_rows16", 1},
            {"decompose.grid", 1},
            {"memory.pool", 1},
            {"memory.arena", 1},
            {"aggregates.moments", 7},
            {"memory.arena_chunk_mib", 0},
            {"decompose.block", 256},
            {"pointwise.dword_shift", 1},
            {"aggregates.moments_pipe", 1},
            {"decompose.batch", 0},
            {"decompose.gather", 0},
            {"decompose.pipe", 0},
            {"decompose.pair", 0},
            {"memory.fail_next_alloc", 0},
            {"comm.test_stall_ms", 0},
            {"pointwise.row_kernel", 3},
            {"pointwise.row_lds", 5632},
            {"pointwise.u8_unroll", 2},
            {"pointwise.u16_unroll", 1},
            {"pointwise.row_lds_u8", 0},
            {"pointwise.row_swizzle", 0},
            {"pointwise.rows_kernel", 3},
            {"transform.shape", 0},
            {"decompose.direct", 1},
            {"resample.prefetch", 0},
            {"resample.any_rows", 1},
            {"histogram.pair_tiles", 1},
            {"resample.lds_pad", 1},
            {"decompose.row_image", 2},
            {"resample.dst_rows", 1},
            {"histogram.u16_codes", 2},
            {"histogram.partials", 1},
        };
        static_assert(sizeof(kKnobs) / sizeof(kKnobs[0]) == static_cast<size_t>(Knob::Count), "knob table");
        std::atomic<int64_t> gKnobs[static_cast<int>(Knob::Count)] = {{kKnobs[0].def}, {kKnobs[1].def},
                                                                  {kKnobs[2].def}, {kKnobs[3].def},
                                                                  {kKnobs[4].def}, {kKnobs[5].def},
                                                                  {kKnobs[6].def}, {kKnobs[7].def},
                                                                  {kKnobs[8].def}, {kKnobs[9].def},
                                                                  {kKnobs[10].def}, {kKnobs[11].def},
                                                                  {kKnobs[12].def}, {kKnobs[13].def},
                                                                  {kKnobs[14].def}, {kKnobs[15].def},
                                                                  {kKnobs[16].def}, {kKnobs[17].def},
                                                                  {kKnobs[18].def}, {kKnobs[19].def},
                                                                  {kKnobs[20].def}, {kKnobs[21].def},
                                                                  {kKnobs[22].def}, {kKnobs[23].def},
                                                                  {kKnobs[24].def}, {kKnobs[25].def},
                                                                  {kKnobs[26].def}, {kKnobs[27].def},
                                                                  {kKnobs[28].def}, {kKnobs[29].def},
                                                                  {kKnobs[30].def}, {kKnobs[31].def},
                                                                  {kKnobs[32].def}, {kKnobs[33].def},
                                                                  {kKnobs[34].def}, {kKnobs[35].def},
                                                                  {kKnobs[36].def}, {kKnobs[37].def},
                                                                  {kKnobs[38].def}, {kKnobs[39].def},
                                                                  {kKnobs[40].def}, {kKnobs[41].def},
                                                                  {kKnobs[42].def}, {kKnobs[43].def},
                                                                  {kKnobs[44].def}, {kKnobs[45].def},
                                                                  {kKnobs[46].def}, {kKnobs[47].def}};
    } // namespace

    int64_t knob(Knob k) { return gKnobs[static_cast<int>(k)].load(std::memory_order_relaxed); }

    bool takeKnobCount(Knob k)
    {
        std::atomic<int64_t>& a = gKnobs[static_cast<int>(k)];
        int64_t v = a.load();
        while (v > 0)
            if (a.compare_exchange_weak(v, v - 1))
                return true;
        return false;
    }

    // Every backend call is also a roctx range named after the reference's backend function
    // (e.g. "SumRange_hip"), so `rocprofv3 --marker-trace` attributes kernels to API calls.
    ScopedKernelTimer::ScopedKernelTimer(char const* name, bool log)
        : name_(name), active_(log || kernelTimingEnabled()), log_(log)
    {
        roctxRangePushA(name);
        if (!active_)
            return;
        hipStream_t s = computeStream();
        if (hipEventCreate(&start_) != hipSuccess || hipEventCreate(&stop_) != hipSuccess)
        {
            active_ = false;
            return;
        }
        (void)hipEventRecord(start_, s);
    }

    ScopedKernelTimer::~ScopedKernelTimer()
    {
        struct Pop
        {
            ~Pop() { roctxRangePop(); }
        } pop;
        if (!active_)
            return;
        (void)hipEventRecord(stop_, computeStream());
        (void)hipEventSynchronize(stop_);
        float ms = 0.f;
        (void)hipEventElapsedTime(&ms, start_, stop_);
        tlsLastKernelMs = ms;
        (void)hipEventDestroy(start_);
        (void)hipEventDestroy(stop_);
        if (log_)
            VKT_LOG(LogLevel::Info) << "Device: GPU (HIP, gfx950), algorithm: " << name_
                                    << ", time elapsed: " << ms * 1e-3f << " sec.";
    }

} // rt
} // vkt

using namespace vkt;

extern "C" {

vktError vktHipSetDevice(int32_t dev)
{
    rt::Context& c = rt::ctx();
    std::lock_guard<std::mutex> lock(c.mutex);
    if (c.initialised && c.device != dev)
        return rt::fail("vktHipSetDevice: the HIP context is already initialised on another device");
    c.device = dev;
    return rt::check(hipSetDevice(dev), "hipSetDevice");
}

vktError vktHipGetDevice(int32_t* dev)
{
    if (dev == nullptr)
        return rt::fail("vktHipGetDevice: null pointer");
    *dev = rt::device();
    return vktNoError;
}

vktError vktHipSetAsyncExecution(int32_t async)
{
    rt::ctx().async.store(async != 0);
    return vktNoError;
}

vktError vktHipGetAsyncExecution(int32_t* async)
{
    if (async == nullptr)
        return rt::fail("vktHipGetAsyncExecution: null pointer");
    *async = rt::ctx().async.load();
    return vktNoError;
}

namespace
{
    // Work queued on the stream being replaced stays ordered before everything queued on its
    // successor (the successor waits for the old tail): the library's later calls, its allocator's
    // reuse of freed buffers (runtime/Memory.cpp drains on the current streams) and a context
    // destroying the old stream all see it finished.
    vktError chainStreams(hipStream_t from, hipStream_t to)
    {
        if (from == to)
            return vktNoError;
        hipEvent_t ev = nullptr;
        VKT_HIP_TRY(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        vktError e = rt::check(hipEventRecord(ev, from), "hipEventRecord(stream switch)");
        if (e == vktNoError)
            e = rt::check(hipStreamWaitEvent(to, ev, 0), "hipStreamWaitEvent(stream switch)");
        (void)hipEventDestroy(ev);
        return e;
    }
} // namespace

vktError vktHipSetComputeStream(void* stream)
{
    rt::Context& c = rt::ctx();
    std::lock_guard<std::mutex> lock(c.mutex);
    rt::initLocked(c);
    hipStream_t const old = c.userStreamSet ? c.userCompute : c.ownCompute;
    hipStream_t const next = stream != nullptr ? static_cast<hipStream_t>(stream) : c.ownCompute;
    vktError const e = chainStreams(old, next);
    c.userCompute = static_cast<hipStream_t>(stream);
    c.userStreamSet = stream != nullptr;
    return e;
}

vktError vktHipGetComputeStream(void** stream)
{
    if (stream == nullptr)
        return rt::fail("vktHipGetComputeStream: null pointer");
    *stream = rt::computeStream();
    return vktNoError;
}

vktError vktHipSetCopyStream(void* stream)
{
    rt::Context& c = rt::ctx();
    std::lock_guard<std::mutex> lock(c.mutex);
    rt::initLocked(c);
    hipStream_t const old = c.userCopySet ? c.userCopy : c.copy;
    hipStream_t const next = stream != nullptr ? static_cast<hipStream_t>(stream) : c.copy;
    vktError const e = chainStreams(old, next);
    c.userCopy = static_cast<hipStream_t>(stream);
    c.userCopySet = stream != nullptr;
    return e;
}

vktError vktHipGetCopyStream(void** stream)
{
    if (stream == nullptr)
        return rt::fail("vktHipGetCopyStream: null pointer");
    *stream = rt::copyStream();
    return vktNoError;
}

vktError vktHipSynchronize(void)
{
    VKT_HIP_TRY(hipStreamSynchronize(rt::computeStream()));
    VKT_HIP_TRY(hipStreamSynchronize(rt::copyStream()));
    return vktNoError;
}

const char* vktHipGetLastErrorString(void) { return rt::tlsLastError.c_str(); }

vktError vktHipSetKernelTiming(int32_t enable)
{
    rt::ctx().timing.store(enable != 0);
    return vktNoError;
}

vktError vktHipGetLastKernelMs(float* ms)
{
    if (ms == nullptr)
        return rt::fail("vktHipGetLastKernelMs: null pointer");
    *ms = rt::tlsLastKernelMs;
    return vktNoError;
}

// Scope for a kernel the caller launches itself on the compute stream (the device-functor
// Transform templates of include/volkit_transform.hpp): the same policy check, roctx range,
// printPerformance timer and launch/async handling as the library's own entry points.
struct vktHipKernelScope_impl
{
    explicit vktHipKernelScope_impl(char const* n, bool log) : name(n), timer(n, log) {}
    char const* name;
    vkt::rt::ScopedKernelTimer timer;
};

vktError vktHipKernelScopeBegin(char const* name, vktHipKernelScope* scope, void** stream)
{
    if (name == nullptr || scope == nullptr || stream == nullptr)
        return rt::fail("vktHipKernelScopeBegin: null pointer");
    *scope = nullptr;
    vkt::ExecutionPolicy ep = vkt::GetThreadExecutionPolicy();
    if (ep.device != vkt::ExecutionPolicy::Device::GPU)
        return rt::fail((std::string(name) + ": CPU execution policy (volkit-amd implements the GPU backend only; "
                                              "set ExecutionPolicy::Device::GPU)").c_str());
    *stream = rt::computeStream();
    *scope = new vktHipKernelScope_impl(name, ep.printPerformance != vkt::False);
    return vktNoError;
}

vktError vktHipKernelScopeEnd(vktHipKernelScope scope)
{
    if (scope == nullptr)
        return rt::fail("vktHipKernelScopeEnd: null scope");
    vktError e = rt::finishLaunch(scope->name);
    delete scope;   // stops the timer, pops the roctx range
    return e;
}

vktError vktHipSetTuningKnob(char const* name, int64_t value)
{
    if (name == nullptr)
        return rt::fail("vktHipSetTuningKnob: null name");
    for (size_t i = 0; i < static_cast<size_t>(rt::Knob::Count); ++i)
        if (std::strcmp(name, rt::kKnobs[i].name) == 0)
        {
            if (value <= 0 && i == static_cast<size_t>(rt::Knob::PointwiseMaxQuanta))
                value = rt::kKnobs[i].def;
            rt::gKnobs[i].store(value < 0 ? rt::kKnobs[i].def : value);
            return vktNoError;
        }
    return rt::fail((std::string("vktHipSetTuningKnob: unknown knob ") + name).c_str());
}

vktError vktHipGetTuningKnob(char const* name, int64_t* value)
{
    if (name == nullptr || value == nullptr)
        return rt::fail("vktHipGetTuningKnob: null pointer");
    for (size_t i = 0; i < static_cast<size_t>(rt::Knob::Count); ++i)
        if (std::strcmp(name, rt::kKnobs[i].name) == 0)
        {
            *value = rt::gKnobs[i].load(std::memory_order_relaxed);
            return vktNoError;
        }
    return rt::fail((std::string("vktHipGetTuningKnob: unknown knob ") + name).c_str());
}

vktError vktHipReportError(char const* message)
{
    return rt::fail(message != nullptr ? message : "vktHipReportError");
}

// ---- context handles (reference include/c/vkt/CudaContext.h:17-65, declared there and never
//      defined): a set of streams + the async flag, bound to the process's backend by
//      vktHipContextMakeCurrent (one HIP context per process -- the library's model).
struct vktHipContext_impl
{
    std::vector<hipStream_t> streams;
    std::vector<char> owned;   // created by the context (destroyed with it)
    int32_t compute = 0, copy = 0;
    int32_t async = 1;
};

namespace
{
    std::mutex gCtxMutex;
    vktHipContext gCurrent = nullptr;

    vktError applyLocked(vktHipContext c)
    {
        vktHipSetAsyncExecution(c->async);
        vktError e = vktHipSetComputeStream(c->streams[static_cast<size_t>(c->compute)]);
        return e != vktNoError ? e : vktHipSetCopyStream(c->streams[static_cast<size_t>(c->copy)]);
    }

    vktError changed(vktHipContext c);

    // Destroys an owned stream the context no longer uses: when the context is current it is
    // first unbound (the backend rebound to the context's remaining ids, which also orders its
    // queued work before theirs) and synchronised, so no caller enqueues on a destroyed handle
    // (ADVICE r3).
    vktError retire(hipStream_t s, bool owned)
    {
        if (!owned)
            return vktNoError;
        VKT_HIP_TRY(hipStreamSynchronize(s));
        VKT_HIP_TRY(hipStreamDestroy(s));
        return vktNoError;
    }

    vktError resize(vktHipContext c, int32_t n)
    {
        (void)vkt::rt::device();   // streams of the library's device
        if (static_cast<int32_t>(c->streams.size()) > n)
        {
            std::vector<hipStream_t> doomed(c->streams.begin() + n, c->streams.end());
            std::vector<char> owned(c->owned.begin() + n, c->owned.end());
            c->compute = std::min(c->compute, n - 1);
            c->copy = std::min(c->copy, n - 1);
            vktError e = changed(c);   // rebind to surviving streams first
            for (size_t i = 0; i < doomed.size() && e == vktNoError; ++i)
                e = retire(doomed[i], owned[i] != 0);
            c->streams.resize(static_cast<size_t>(n));
            c->owned.resize(static_cast<size_t>(n));
            if (e != vktNoError)
                return e;
        }
        while (static_cast<int32_t>(c->streams.size()) < n)
        {
            hipStream_t s = nullptr;
            // blocking streams, like the library's own (ordered with the legacy NULL stream)
            VKT_HIP_TRY(hipStreamCreateWithFlags(&s, hipStreamDefault));
            c->streams.push_back(s);
            c->owned.push_back(1);
        }
        c->compute = std::min(c->compute, n - 1);
        c->copy = std::min(c->copy, n - 1);
        return vktNoError;
    }

    vktError changed(vktHipContext c)
    {
        return c == gCurrent ? applyLocked(c) : vktNoError;
    }
} // namespace

vktError vktHipContextCreate(vktHipContext* context)
{
    if (context == nullptr)
        return rt::fail("vktHipContextCreate: null pointer");
    auto* c = new vktHipContext_impl;
    std::lock_guard<std::mutex> lock(gCtxMutex);
    vktError e = resize(c, 2);   // stream 0: compute, stream 1: copy
    if (e != vktNoError)
    {
        delete c;
        *context = nullptr;
        return e;
    }
    c->copy = 1;
    *context = c;
    return vktNoError;
}

vktError vktHipContextDestroy(vktHipContext context)
{
    if (context == nullptr)
        return vktNoError;
    std::lock_guard<std::mutex> lock(gCtxMutex);
    if (context == gCurrent)
    {
        // back to the library's own streams before the context's streams go away
        VKT_HIP_TRY(hipStreamSynchronize(rt::computeStream()));
        VKT_HIP_TRY(hipStreamSynchronize(rt::copyStream()));
        vktHipSetComputeStream(nullptr);
        vktHipSetCopyStream(nullptr);
        gCurrent = nullptr;
    }
    for (size_t i = 0; i < context->streams.size(); ++i)
        if (context->owned[i])
            (void)hipStreamDestroy(context->streams[i]);
    delete context;
    return vktNoError;
}

vktError vktHipContextMakeCurrent(vktHipContext context)
{
    std::lock_guard<std::mutex> lock(gCtxMutex);
    gCurrent = context;
    if (context == nullptr)
    {
        vktHipSetComputeStream(nullptr);
        return vktHipSetCopyStream(nullptr);
    }
    return applyLocked(context);
}

vktError vktHipContextSetAsyncExecution(vktHipContext context, int32_t async)
{
    if (context == nullptr)
        return rt::fail("vktHipContextSetAsyncExecution: null context");
    std::lock_guard<std::mutex> lock(gCtxMutex);
    context->async = async != 0;
    return changed(context);
}

vktError vktHipContextGetAsyncExecution(vktHipContext context, int32_t* async)
{
    if (context == nullptr || async == nullptr)
        return rt::fail("vktHipContextGetAsyncExecution: null pointer");
    *async = context->async;
    return vktNoError;
}

vktError vktHipContextSetNumStreams(vktHipContext context, int32_t numStreams)
{
    if (context == nullptr || numStreams < 1)
        return rt::fail("vktHipContextSetNumStreams: null context or numStreams < 1");
    std::lock_guard<std::mutex> lock(gCtxMutex);
    vktError e = resize(context, numStreams);
    return e != vktNoError ? e : changed(context);
}

vktError vktHipContextGetNumStreams(vktHipContext context, int32_t* numStreams)
{
    if (context == nullptr || numStreams == nullptr)
        return rt::fail("vktHipContextGetNumStreams: null pointer");
    *numStreams = static_cast<int32_t>(context->streams.size());
    return vktNoError;
}

vktError vktHipContextSetStream(vktHipContext context, int32_t streamId, void* stream)
{
    if (context == nullptr || streamId < 0 || streamId >= static_cast<int32_t>(context->streams.size()) || !stream)
        return rt::fail("vktHipContextSetStream: null context / stream or stream id out of range");
    std::lock_guard<std::mutex> lock(gCtxMutex);
    size_t const i = static_cast<size_t>(streamId);
    hipStream_t const old = context->streams[i];
    bool const owned = context->owned[i] != 0;
    context->streams[i] = static_cast<hipStream_t>(stream);
    context->owned[i] = 0;   // the caller's stream: not destroyed by the context
    vktError const e = changed(context);   // rebind (current context) before the old one goes
    vktError const r = old != context->streams[i] ? retire(old, owned) : vktNoError;
    return e != vktNoError ? e : r;
}

vktError vktHipContextGetStream(vktHipContext context, int32_t streamId, void** stream)
{
    if (context == nullptr || stream == nullptr || streamId < 0 ||
        streamId >= static_cast<int32_t>(context->streams.size()))
        return rt::fail("vktHipContextGetStream: null pointer or stream id out of range");
    *stream = context->streams[static_cast<size_t>(streamId)];
    return vktNoError;
}

vktError vktHipContextSetComputeStreamId(vktHipContext context, int32_t streamId)
{
    if (context == nullptr || streamId < 0 || streamId >= static_cast<int32_t>(context->streams.size()))
        return rt::fail("vktHipContextSetComputeStreamId: null context or stream id out of range");
    std::lock_guard<std::mutex> lock(gCtxMutex);
    context->compute = streamId;
    return changed(context);
}

vktError vktHipContextGetComputeStreamId(vktHipContext context, int32_t* streamId)
{
    if (context == nullptr || streamId == nullptr)
        return rt::fail("vktHipContextGetComputeStreamId: null pointer");
    *streamId = context->compute;
    return vktNoError;
}

vktError vktHipContextSetCopyStreamId(vktHipContext context, int32_t streamId)
{
    if (context == nullptr || streamId < 0 || streamId >= static_cast<int32_t>(context->streams.size()))
        return rt::fail("vktHipContextSetCopyStreamId: null context or stream id out of range");
    std::lock_guard<std::mutex> lock(gCtxMutex);
    context->copy = streamId;
    return changed(context);
}

vktError vktHipContextGetCopyStreamId(vktHipContext context, int32_t* streamId)
{
    if (context == nullptr || streamId == nullptr)
        return rt::fail("vktHipContextGetCopyStreamId: null pointer");
    *streamId = context->copy;
    return vktNoError;
}

} // extern "C"
