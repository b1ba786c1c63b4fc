// Device scratch allocator of the kernel library and the native runtime:
// hipMalloc'd blocks cached in a size-keyed free list, reuse ordered by HIP
// events (a block freed on stream f and taken on stream s makes s wait for
// the free's event; same-stream reuse is ordered by the stream itself).
//
// Why not the stream-ordered pool (hipMallocAsync): on this stack the FIRST
// kernel reads of freshly mapped pool memory returned stale lines (zeros)
// for data that a previous kernel or copy of the same stream had written --
// the native 2 x 1 potrf's received diagonal tile read as zero by the
// triangular inverse (tools/probe/scal_probe.cc; SLATE_AMD_NATIVE_NOPOOL
// runs were clean).  hipMalloc'd memory never showed it.
#pragma once
#include <cstdlib>
#include <map>
#include <mutex>
#include <unordered_map>
#include <unordered_set>

#include "common.hpp"

namespace slate_hip {

struct DevBlock {
    void* p;
    hipStream_t s;
    hipEvent_t ev;
};

struct DevAlloc {
    std::mutex mu;
    std::multimap<size_t, DevBlock> free_;        // rounded size -> block
    std::unordered_map<void*, size_t> size_;      // live and cached blocks
    std::unordered_set<void*> cached_;            // blocks in free_ (double-free check)
    size_t reserved = 0;
};

inline DevAlloc& dev_allocator() {
    static DevAlloc* a = new DevAlloc();          // never destroyed: blocks may outlive static teardown
    return *a;
}

inline size_t dev_round(size_t b) {
    if (b <= 4096) return (b + 255) & ~(size_t)255;
    size_t p = 4096;
    while (p * 2 <= b) p *= 2;
    const size_t step = p / 8;
    return (b + step - 1) / step * step;
}

// Reuse order: a block freed on the same stream (ordered by the stream), then
// a block of another stream whose free has already completed; only when the
// cache holds more than dev_cap() bytes does a stream wait on another stream's
// pending free -- otherwise the panel and update streams of a lookahead
// driver would be chained through their scratch (a false dependency that
// serialises them).
inline size_t dev_cap() {
    static const size_t cap = [] {
        const char* e = std::getenv("SLATE_AMD_DEVALLOC_CAP_MB");
        return (size_t)(e ? std::atoll(e) : 16384) << 20;
    }();
    return cap;
}

inline size_t dev_trim_locked(DevAlloc& A) {
    size_t freed = 0;
    for (auto& kv : A.free_) {
        HIP_CHECK(hipEventSynchronize(kv.second.ev));
        HIP_CHECK(hipEventDestroy(kv.second.ev));
        HIP_CHECK(hipFree(kv.second.p));
        A.size_.erase(kv.second.p);
        A.cached_.erase(kv.second.p);
        A.reserved -= kv.first;
        freed += kv.first;
    }
    A.free_.clear();
    return freed;
}

inline void* dev_alloc(size_t bytes, hipStream_t s) {
    if (bytes == 0) return nullptr;
    DevAlloc& A = dev_allocator();
    const size_t r = dev_round(bytes);
    std::lock_guard<std::mutex> g(A.mu);
    auto take = [&](std::multimap<size_t, DevBlock>::iterator it, bool wait) {
        DevBlock b = it->second;
        A.free_.erase(it);
        A.cached_.erase(b.p);
        if (wait) HIP_CHECK(hipStreamWaitEvent(s, b.ev, 0));
        HIP_CHECK(hipEventDestroy(b.ev));
        return b.p;
    };
    const auto lo = A.free_.lower_bound(r);
    for (auto it = lo; it != A.free_.end() && it->first < 2 * r; ++it)
        if (it->second.s == s) return take(it, false);
    for (auto it = lo; it != A.free_.end() && it->first < 2 * r; ++it)
        if (hipEventQuery(it->second.ev) == hipSuccess) return take(it, false);
    if (A.reserved + r > dev_cap())
        for (auto it = lo; it != A.free_.end() && it->first < 2 * r; ++it) return take(it, true);
    void* p = nullptr;
    if (hipMalloc(&p, r) != hipSuccess) {
        // out of device memory: give every cached block back to the driver
        // (each waited for: its last user may still be running) and retry once
        (void)hipGetLastError();
        dev_trim_locked(A);
        p = nullptr;
        HIP_CHECK(hipMalloc(&p, r));
    }
    A.size_[p] = r;
    A.reserved += r;
    return p;
}

// Release every cached (free) block to the driver; live blocks are kept.
// Called on hipMalloc failure and by the native runtime's finalize().
inline size_t dev_trim() {
    DevAlloc& A = dev_allocator();
    std::lock_guard<std::mutex> g(A.mu);
    return dev_trim_locked(A);
}

inline void dev_free(void* p, hipStream_t s) {
    if (!p) return;
    DevAlloc& A = dev_allocator();
    std::lock_guard<std::mutex> g(A.mu);
    auto it = A.size_.find(p);
    if (it == A.size_.end()) throw std::invalid_argument("dev_free: unknown block");
    if (!A.cached_.insert(p).second) throw std::logic_error("dev_free: block freed twice");
    hipEvent_t ev;
    HIP_CHECK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    HIP_CHECK(hipEventRecord(ev, s));
    A.free_.insert({it->second, DevBlock{p, s, ev}});
}

}  // namespace slate_hip
