// Policy.cpp -- per-thread execution policy and the managed-resource registry.
//
// Execution policy: reference src/vkt/ExecutionPolicy.cpp:17-35 keeps an unlocked global
// unordered_map<thread::id, policy> (a data race under concurrent Set/Get).
// A thread_local gives the same observable semantics -- per calling thread, default
// {CPU, Serial, CUDA(=GPU backend), false}, not inherited by child threads -- without the race.
// Extension: VKT_DEFAULT_DEVICE=GPU makes Device::GPU the initial device of every thread.
//
// Resource registry: reference src/vkt/ManagedResource.cpp:16-40 (monotonic uint32 handles
// over an unlocked map); here guarded by a mutex.

#include "Runtime.hpp"

#include <cstdlib>
#include <cstring>
#include <mutex>
#include <unordered_map>

namespace vkt
{
    namespace
    {
        // Initial policy of every thread: the reference's default {CPU, Serial, CUDA, false},
        // unless VKT_DEFAULT_DEVICE=GPU asks for the GPU device -- then unmodified reference
        // programs, which never set a policy, run their algorithms on this GPU backend.
        ExecutionPolicy initialPolicy()
        {
            static ExecutionPolicy const p = [] {
                ExecutionPolicy e;
                char const* d = std::getenv("VKT_DEFAULT_DEVICE");
                if (d != nullptr && (std::strcmp(d, "GPU") == 0 || std::strcmp(d, "gpu") == 0))
                    e.device = ExecutionPolicy::Device::GPU;
                return e;
            }();
            return p;
        }

        // Constant-initialised (no per-access TLS init guard) with a lazy first-use flag:
        // GetThreadExecutionPolicy runs on every getData()/migrate() of every volume.
        struct TlsPolicy
        {
            ExecutionPolicy policy;
            bool init;
        };
        thread_local TlsPolicy tlsPolicy{ExecutionPolicy{}, false};

        ExecutionPolicy& threadPolicy()
        {
            TlsPolicy& t = tlsPolicy;
            if (!t.init)
            {
                t.policy = initialPolicy();
                t.init = true;
            }
            return t.policy;
        }

        std::mutex& registryMutex()
        {
            static std::mutex* m = new std::mutex;
            return *m;
        }

        std::unordered_map<ResourceHandle, ManagedResource>& registry()
        {
            static auto* r = new std::unordered_map<ResourceHandle, ManagedResource>;
            return *r;
        }

        ResourceHandle nextHandle = 0;
    } // namespace

    void SetThreadExecutionPolicy(ExecutionPolicy policy) { threadPolicy() = policy; }

    ExecutionPolicy GetThreadExecutionPolicy() { return threadPolicy(); }

    ResourceHandle RegisterManagedResource(ManagedResource resource)
    {
        std::lock_guard<std::mutex> lock(registryMutex());
        ResourceHandle h = nextHandle++;
        registry()[h] = resource;
        return h;
    }

    void UnregisterManagedResource(ResourceHandle handle)
    {
        std::lock_guard<std::mutex> lock(registryMutex());
        registry().erase(handle);
    }

    ManagedResource GetManagedResource(ResourceHandle handle)
    {
        std::lock_guard<std::mutex> lock(registryMutex());
        auto it = registry().find(handle);
        return it == registry().end() ? nullptr : it->second;
    }
} // vkt

extern "C" {

// C mapping follows reference src/vkt/ExecutionPolicy.cpp:44-118, including its quirk
// that only the Serial host API and the CUDA(=GPU backend) device API are translated;
// other values fall back to the C++ defaults.
void vktSetThreadExecutionPolicy(vktExecutionPolicy_t policy)
{
    vkt::ExecutionPolicy p;
    if (policy.device == vktExecutionPolicyDeviceCPU)
        p.device = vkt::ExecutionPolicy::Device::CPU;
    else if (policy.device == vktExecutionPolicyDeviceGPU)
        p.device = vkt::ExecutionPolicy::Device::GPU;
    if (policy.hostApi == vktExecutionPolicyHostAPISerial)
        p.hostApi = vkt::ExecutionPolicy::HostAPI::Serial;
    if (policy.deviceApi == vktExecutionPolicyDeviceAPICUDA)
        p.deviceApi = vkt::ExecutionPolicy::DeviceAPI::CUDA;
    p.printPerformance = policy.printPerformance == VKT_TRUE ? vkt::True : vkt::False;
    vkt::SetThreadExecutionPolicy(p);
}

vktExecutionPolicy_t vktGetThreadExecutionPolicy(void)
{
    vkt::ExecutionPolicy p = vkt::GetThreadExecutionPolicy();
    vktExecutionPolicy_t out{};
    out.device = p.device == vkt::ExecutionPolicy::Device::GPU ? vktExecutionPolicyDeviceGPU
                                                               : vktExecutionPolicyDeviceCPU;
    out.hostApi = vktExecutionPolicyHostAPISerial;
    out.deviceApi = vktExecutionPolicyDeviceAPICUDA;
    out.printPerformance = p.printPerformance == vkt::True ? VKT_TRUE : VKT_FALSE;
    return out;
}

vktResourceHandle vktRegisterManagedResource(vktManagedResource resource)
{
    return vkt::RegisterManagedResource(resource);
}

void vktUnregisterManagedResource(vktResourceHandle handle) { vkt::UnregisterManagedResource(handle); }

vktManagedResource vktGetManagedResource(vktResourceHandle handle) { return vkt::GetManagedResource(handle); }

} // extern "C"
