// gc_alloc.hip -- the library's device / pinned-host allocator: a per-device cache of
// freed blocks, keyed by exact size.
//
// A colouring from a resident CSR (rank partition, hub index, rounds,
// validation) allocates ~60 buffers per graph handle; hipMalloc of a large buffer costs
// tens of microseconds to milliseconds and hipFree synchronises the device.  Handles that
// are created and destroyed repeatedly (bench.py's timed step, the CLI's two runs, the
// tests) therefore get their buffers back from this cache: a freed block is parked under
// (device, size) and handed to the next request of exactly that size.  The cache is
// released on a failed allocation (then retried) and by gc_release_cache().
//
// Callers free a block only when no queued work still uses it (every free site follows a
// stream synchronisation), so a parked block is idle by construction.
#include <hip/hip_runtime.h>

#include <stdio.h>
#include <stdlib.h>

#include <chrono>
#include <map>
#include <mutex>
#include <unordered_map>

#include "gc_engine.h"

namespace {

struct Block {
    size_t bytes;
    int device;
    bool host;
};

struct Cache {
    std::mutex mu;
    std::unordered_map<void*, Block> live;                   // handed out
    std::multimap<std::pair<long long, size_t>, void*> idle;  // (device or -1 for host, bytes) -> block
    size_t idle_bytes = 0;
};

// GC_ALLOC_TRACE=1: every hipMalloc / hipFree this allocator makes (cache misses, and frees
// past the idle cap) of 16 MB or more, with its host time, on stderr
bool trace_on() {
    static const bool on = getenv("GC_ALLOC_TRACE") != nullptr;
    return on;
}

struct TraceClock {
    const char* what;
    size_t bytes;
    std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
    TraceClock(const char* w, size_t b) : what(w), bytes(b) {}
    ~TraceClock() {
        if (!trace_on() || bytes < ((size_t)16 << 20)) return;
        const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        fprintf(stderr, "[gc alloc] %-9s %10.1f MB %9.3f ms\n", what, (double)bytes / 1048576.0, ms);
    }
};

Cache& cache() {
    static Cache* c = new Cache();  // never destroyed: frees at process exit would race the runtime's teardown
    return *c;
}

void release_locked(Cache& c) {
    TraceClock tc("release", c.idle_bytes);
    int dev0 = 0;
    hipGetDevice(&dev0);
    for (auto& kv : c.idle) {
        if (kv.first.first < 0) {
            hipHostFree(kv.second);
        } else {
            hipSetDevice((int)kv.first.first);
            hipFree(kv.second);
        }
    }
    c.idle.clear();
    c.idle_bytes = 0;
    hipSetDevice(dev0);
}

hipError_t alloc(void** p, size_t bytes, bool host) {
    if (bytes == 0) bytes = 1;
    int dev = 0;
    hipGetDevice(&dev);
    const long long key = host ? -1 : dev;
    Cache& c = cache();
    {
        std::lock_guard<std::mutex> lk(c.mu);
        auto it = c.idle.find({key, bytes});
        if (it != c.idle.end()) {
            *p = it->second;
            c.idle.erase(it);
            c.idle_bytes -= bytes;
            c.live[*p] = Block{bytes, dev, host};
            return hipSuccess;
        }
    }
    hipError_t e;
    {
        TraceClock tc(host ? "hostalloc" : "malloc", bytes);
        e = host ? hipHostMalloc(p, bytes, hipHostMallocDefault) : hipMalloc(p, bytes);
    }
    if (e != hipSuccess) {  // the cache may hold what is missing: give it back and retry once
        (void)hipGetLastError();
        std::lock_guard<std::mutex> lk(c.mu);
        release_locked(c);
        e = host ? hipHostMalloc(p, bytes, hipHostMallocDefault) : hipMalloc(p, bytes);
        if (e != hipSuccess) return e;
    }
    std::lock_guard<std::mutex> lk(c.mu);
    c.live[*p] = Block{bytes, dev, host};
    return hipSuccess;
}

}  // namespace

hipError_t gc_dmalloc(void** p, size_t bytes) { return alloc(p, bytes, false); }
hipError_t gc_hmalloc(void** p, size_t bytes) { return alloc(p, bytes, true); }

// Parked bytes beyond this are freed at once.  The library's default is 64 GB: parked blocks
// are idle memory of this process only (an allocation of ours that fails gives the whole cache
// back and retries, but torch in the same process or other processes sharing the GPU cannot
// reach them), so the default stays conservative.  Two settings raise it:
//   GC_ALLOC_IDLE_CAP_GB=G       a cap of G GB;
//   GC_ALLOC_IDLE_RESERVE_GB=R   the device's memory less R GB (at least 64 GB) -- bench.py's
//                                one-process-per-GPU runs set R = 48.
// Why bench.py opts in: a fixed 64 GB was below one R-MAT-28 handle's buffers (~110 GB: the
// partitioned CSR, the hub transpose and its hlow copies, the work lists), so every step's
// destroy freed ~40 GB with hipFree -- which returns at once -- and the next large hipMalloc
// waited ~3 s for that memory (GC_ALLOC_TRACE=1, profiles/r05/a: "malloc 1024 MB 3123 ms"):
// R-MAT-28's bench step 2.93 s against 1.77 s without it.  Half of the memory fixed the
// one-GPU step but not the multi-GPU one, whose shard state adds its in-rows and replicas
// (~1.75 s stalls a step, profiles/r05/w).
static size_t idle_cap() {
    static size_t cap = 0;
    if (!cap) {
        size_t freeb = 0, total = 0;
        const size_t floor = (size_t)64 << 30;
        const char* env = getenv("GC_ALLOC_IDLE_CAP_GB");
        const char* res = getenv("GC_ALLOC_IDLE_RESERVE_GB");
        if (env && atoll(env) > 0) {
            cap = (size_t)atoll(env) << 30;
        } else if (res && atoll(res) >= 0) {
            const size_t reserve = (size_t)atoll(res) << 30;
            cap = (hipMemGetInfo(&freeb, &total) == hipSuccess && total > floor + reserve) ? total - reserve : floor;
        } else {
            cap = floor;
        }
    }
    return cap;
}

hipError_t gc_dfree(void* p) {
    if (!p) return hipSuccess;
    Cache& c = cache();
    std::lock_guard<std::mutex> lk(c.mu);
    auto it = c.live.find(p);
    if (it == c.live.end()) return hipFree(p);  // not ours (never expected)
    const Block b = it->second;
    c.live.erase(it);
    if (c.idle_bytes + b.bytes > idle_cap()) {
        TraceClock tc("free", b.bytes);
        return b.host ? hipHostFree(p) : hipFree(p);
    }
    c.idle.insert({{b.host ? -1 : b.device, b.bytes}, p});
    c.idle_bytes += b.bytes;
    return hipSuccess;
}

extern "C" int gc_release_cache(void) {
    Cache& c = cache();
    std::lock_guard<std::mutex> lk(c.mu);
    release_locked(c);
    return GC_OK;
}

// one-off buffers (generators): not cached; a failure releases the cache and retries once
hipError_t gc_raw_malloc(void** p, size_t bytes) {
    hipError_t e = hipMalloc(p, bytes ? bytes : 1);
    if (e == hipSuccess) return e;
    (void)hipGetLastError();
    gc_release_cache();
    return hipMalloc(p, bytes ? bytes : 1);
}

size_t gc_cache_idle_bytes(void) {
    Cache& c = cache();
    std::lock_guard<std::mutex> lk(c.mu);
    return c.idle_bytes;
}
