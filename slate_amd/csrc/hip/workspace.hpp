// Per-stream grow-only device workspaces for multi-kernel launchers
// (trsm, trtri, potrf tile, getrf panel).  Reuse on the same stream is safe by
// stream order; different streams get different buffers; growth returns the
// old buffer to the event-ordered cache of devalloc.hpp.  Avoids an
// allocation per call on the factorization critical path.
#pragma once
#include <mutex>
#include <unordered_map>
#include "common.hpp"
#include "devalloc.hpp"

namespace slate_hip {

// workspace slots (one buffer per stream per slot)
enum { WS_X = 0, WS_W = 1, WS_T = 2, WS_I = 3, WS_QW = 4, WS_QW2 = 5, WS_P = 6, WS_L = 7, WS_C = 8, WS_QF = 9, WS_PM = 10 };

struct WsKey {
    hipStream_t s; int slot;
    bool operator==(const WsKey& o) const { return s == o.s && slot == o.slot; }
};
struct WsHash {
    size_t operator()(const WsKey& k) const { return std::hash<void*>()((void*)k.s) ^ (size_t)k.slot * 7919; }
};

inline void* workspace(hipStream_t s, size_t bytes, int slot) {
    static std::mutex mu;
    static std::unordered_map<WsKey, std::pair<void*, size_t>, WsHash> cache;
    std::lock_guard<std::mutex> g(mu);
    auto& e = cache[WsKey{s, slot}];
    if (e.second < bytes) {
        if (e.first) dev_free(e.first, s);
        size_t nb = std::max(bytes, e.second * 2);
        e.first = dev_alloc(nb, s);
        e.second = nb;
    }
    return e.first;
}

}  // namespace slate_hip
