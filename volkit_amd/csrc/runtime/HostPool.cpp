// HostPool.cpp -- persistent host worker threads for parallelFor (runtime/HostPool.hpp).
//
// Workers sleep on a condition variable between jobs; a job is (fn, n, chunk) with an atomic
// cursor that the workers and the caller advance.  The caller returns when every worker that
// joined the job has left it (so no worker straddles two jobs).  One job at a time (try_lock:
// a concurrent or nested call runs serially).

#include "HostPool.hpp"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdlib>
#include <mutex>
#include <thread>
#include <vector>

namespace vkt
{
namespace rt
{
namespace
{
    class Pool
    {
    public:
        explicit Pool(int threads)
        {
            for (int i = 1; i < threads; ++i)
                workers_.emplace_back([this] { loop(); });
        }

        ~Pool()
        {
            {
                std::lock_guard<std::mutex> g(m_);
                stop_ = true;
            }
            cv_.notify_all();
            for (std::thread& t : workers_)
                t.join();
        }

        int threads() const { return static_cast<int>(workers_.size()) + 1; }

        bool run(size_t n, size_t chunk, std::function<void(size_t, size_t)> const& fn)
        {
            std::unique_lock<std::mutex> busy(job_, std::try_to_lock);
            if (!busy.owns_lock())
                return false;
            int dev = 0;
            (void)hipGetDevice(&dev);
            size_t const chunks = (n + chunk - 1) / chunk;
            {
                std::lock_guard<std::mutex> g(m_);
                fn_ = &fn;
                n_ = n;
                chunk_ = chunk;
                chunks_ = chunks;
                device_ = dev;
                next_.store(0);
                ++generation_;
            }
            cv_.notify_all();
            work(&fn);
            std::unique_lock<std::mutex> g(m_);
            fn_ = nullptr;   // no worker joins any more
            doneCv_.wait(g, [&] { return active_ == 0; });
            return true;
        }

    private:
        // take chunks until none is left (fn: the job's function, read under the lock)
        void work(std::function<void(size_t, size_t)> const* fn)
        {
            for (;;)
            {
                size_t const c = next_.fetch_add(1);
                if (c >= chunks_)
                    return;
                size_t const b = c * chunk_, e = std::min(n_, b + chunk_);
                (*fn)(b, e);
            }
        }

        void loop()
        {
            uint64_t seen = 0;
            int dev = -1;
            for (;;)
            {
                std::function<void(size_t, size_t)> const* fn = nullptr;
                {
                    std::unique_lock<std::mutex> g(m_);
                    cv_.wait(g, [&] { return stop_ || generation_ != seen; });
                    if (stop_)
                        return;
                    seen = generation_;
                    if (fn_ == nullptr)
                        continue;
                    if (device_ != dev)
                    {
                        (void)hipSetDevice(device_);
                        dev = device_;
                    }
                    ++active_;
                    fn = fn_;
                }
                work(fn);
                std::lock_guard<std::mutex> g(m_);
                if (--active_ == 0)
                    doneCv_.notify_all();
            }
        }

        std::vector<std::thread> workers_;
        std::mutex job_;                       // one job at a time
        std::mutex m_;
        std::condition_variable cv_, doneCv_;
        bool stop_ = false;
        uint64_t generation_ = 0;
        std::function<void(size_t, size_t)> const* fn_ = nullptr;
        size_t n_ = 0, chunk_ = 1, chunks_ = 0;
        int device_ = 0;
        int active_ = 0;                       // workers inside the current job
        std::atomic<size_t> next_{0};
    };

    Pool& pool()
    {
        static Pool p(hostThreads());
        return p;
    }
} // namespace

int hostThreads()
{
    static int const n = [] {
        if (char const* s = std::getenv("VKT_HOST_THREADS"))
        {
            int const v = std::atoi(s);
            if (v >= 1)
                return std::min(v, 64);
        }
        unsigned const hw = std::thread::hardware_concurrency();
        return static_cast<int>(std::max(1u, std::min(16u, hw)));
    }();
    return n;
}

void parallelFor(size_t n, size_t minChunk, std::function<void(size_t, size_t)> const& fn)
{
    if (n == 0)
        return;
    size_t const chunk = std::max<size_t>(std::max<size_t>(minChunk, 1), (n + 4 * hostThreads() - 1) / (4 * hostThreads()));
    if (hostThreads() <= 1 || n <= chunk || !pool().run(n, chunk, fn))
        fn(0, n);
}

} // rt
} // vkt
