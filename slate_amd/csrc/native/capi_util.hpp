// Shared helpers of the native C / LAPACK / ScaLAPACK ABI units
// (capi_native.hip, capi_lapack.hip, capi_handles.hip).  Not installed.
#pragma once
#include <algorithm>
#include <cstring>
#include <complex>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "native_rt.hpp"

namespace slate_amd {
namespace native {
namespace capi {

namespace sn = slate_amd::native;

constexpr int ERR_INTERNAL = -1000000;
// message of the last runtime error of this thread (slate_amd_last_error)
inline thread_local std::string g_err;

// process grid of the LAPACK-style host-array routines: 1 x WORLD_SIZE, or
// SLATE_AMD_NATIVE_GRID=PxQ
inline void grid_of(int& p, int& q) {
    const int ws = sn::size();
    p = 1;
    q = ws;
    if (const char* g = std::getenv("SLATE_AMD_NATIVE_GRID")) {
        int a = 0, b = 0;
        if (std::sscanf(g, "%dx%d", &a, &b) == 2 && a * b == ws) { p = a; q = b; }
    }
}

inline int64_t nb_of(int64_t n) {
    if (const char* e = std::getenv("SLATE_AMD_NATIVE_NB")) return std::max<int64_t>(16, std::atoll(e));
    return n >= 8192 ? 512 : (n >= 1024 ? 256 : 64);
}

template <typename F>
int64_t guarded(F&& f) {
    try {
        return (int64_t)f();
    } catch (const std::exception& e) {
        g_err = e.what();
        return ERR_INTERNAL;
    }
}

inline char up(char c) { return (c >= 'a' && c <= 'z') ? (char)(c - 32) : c; }

template <typename T> T cj(T x) { return x; }
template <typename R> std::complex<R> cj(std::complex<R> x) { return std::conj(x); }

// op(a) (rows x cols of the RESULT) into a new column-major array
template <typename T>
std::vector<T> host_op(char op, i64 rows, i64 cols, const T* a, i64 lda) {
    std::vector<T> r((size_t)rows * cols);
    for (i64 j = 0; j < cols; ++j)
        for (i64 i = 0; i < rows; ++i)
            r[i + j * rows] = op == 'N' ? a[i + j * lda] : op == 'T' ? a[j + i * lda] : cj(a[j + i * lda]);
    return r;
}

inline sn::Op op_of(char c) {
    c = up(c);
    return c == 'N' ? sn::Op::NoTrans : c == 'T' ? sn::Op::Trans : sn::Op::ConjTrans;
}
inline sn::Uplo uplo_of(char c) { return up(c) == 'U' ? sn::Uplo::Upper : sn::Uplo::Lower; }
inline sn::Diag diag_of(char c) { return up(c) == 'U' ? sn::Diag::Unit : sn::Diag::NonUnit; }
inline sn::Side side_of(char c) { return up(c) == 'R' ? sn::Side::Right : sn::Side::Left; }

// A ScaLAPACK-style 2D block-cyclic layout (mb x nb blocks, source process
// (rsrc, csrc), p x q grid in column- or row-major rank order); also the
// layout of a native matrix (mb = nb, rsrc = csrc = 0, column-major).
struct ScalLay {
    i64 M, N, mb, nb, lld;
    int rsrc, csrc, p, q;
    bool rowmaj;
    int orow(i64 gi) const { return (int)((gi / mb + rsrc) % p); }
    int ocol(i64 gj) const { return (int)((gj / nb + csrc) % q); }
    static i64 g2l(i64 g, i64 b, int np) { return (g / (b * np)) * b + g % b; }
    int rank_of(int r, int c) const { return rowmaj ? r * q + c : r + c * p; }
    void coords(int rank, int& r, int& c) const {
        if (rowmaj) { r = rank / q; c = rank % q; } else { r = rank % p; c = rank / p; }
    }
};
// move the m x n sub-matrix at (i0, j0) of the ScaLAPACK layout L (host local
// array a of this rank) to / from the aligned native matrix B (host local
// array b, leading dimension ldb)
template <typename T>
void scal_move(const ScalLay& L, i64 i0, i64 j0, i64 m, i64 n, T* a, const sn::Storage& B, T* b, i64 ldb,
               bool to_native) {
    const int me = sn::rank(), ws = sn::size();
    int myr, myc;
    L.coords(me, myr, myc);
    const bool in_grid = me < L.p * L.q;
    const int P = B.p, Q = B.q, bpr = B.pr, bpc = B.pc;
    const i64 bnb = B.nb;
    // source-layout side: my local elements of the sub-matrix, column-major
    std::vector<std::vector<T>> sbuf((size_t)ws);
    std::vector<size_t> cnt_src((size_t)ws, 0), cnt_dst((size_t)ws, 0);
    auto src_walk = [&](auto&& f) {
        if (!in_grid) return;
        for (i64 sj = 0; sj < n; ++sj) {
            const i64 gj = j0 + sj;
            if (L.ocol(gj) != myc) continue;
            const i64 lj = ScalLay::g2l(gj, L.nb, L.q);
            const int dc = (int)((sj / bnb) % Q);
            for (i64 si = 0; si < m; ++si) {
                const i64 gi = i0 + si;
                if (L.orow(gi) != myr) continue;
                const int d = (int)((si / bnb) % P) + dc * P;
                f(d, a + ScalLay::g2l(gi, L.mb, L.p) + lj * L.lld);
            }
        }
    };
    // native side: my local elements of B, column-major over the sub-matrix
    auto dst_walk = [&](auto&& f) {
        for (i64 lj = 0; lj < B.nloc; ++lj) {
            const i64 sj = sn::l2g(lj, bnb, Q, bpc);
            const int sc = L.ocol(j0 + sj);
            for (i64 li = 0; li < B.mloc; ++li) {
                const i64 si = sn::l2g(li, bnb, P, bpr);
                f(L.rank_of(L.orow(i0 + si), sc), b + li + lj * ldb);
            }
        }
    };
    // pack (values in canonical order), self part copied directly
    std::vector<std::vector<T>> rbuf((size_t)ws);
    if (to_native) {
        src_walk([&](int d, T* x) { sbuf[d].push_back(*x); });
        dst_walk([&](int s, T*) { ++cnt_dst[s]; });
        for (int r = 0; r < ws; ++r) rbuf[r].resize(cnt_dst[r]);
    } else {
        dst_walk([&](int s, T* x) { sbuf[s].push_back(*x); });
        src_walk([&](int d, T*) { ++cnt_src[d]; });
        for (int r = 0; r < ws; ++r) rbuf[r].resize(cnt_src[r]);
    }
    rbuf[me] = sbuf[me];
    if (ws > 1) {
        sn::Comm* w = sn::world_comm();
        hipStream_t st = sn::rt().main;
        size_t tot = 0;
        std::vector<size_t> soff((size_t)ws), roff((size_t)ws);
        for (int r = 0; r < ws; ++r) { soff[r] = tot; tot += sbuf[r].size() * sizeof(T); }
        const size_t sb = tot;
        for (int r = 0; r < ws; ++r) { roff[r] = tot; tot += rbuf[r].size() * sizeof(T); }
        sn::Scratch d(std::max<size_t>(tot, 64), st);
        std::vector<char> h(std::max<size_t>(sb, 1));
        for (int r = 0; r < ws; ++r)
            if (!sbuf[r].empty()) std::memcpy(h.data() + soff[r], sbuf[r].data(), sbuf[r].size() * sizeof(T));
        if (sb) sn::upload(d.p, h.data(), sb, st);
        std::vector<sn::P2P> ops;
        for (int r = 0; r < ws; ++r) {
            if (r == me) continue;
            if (!sbuf[r].empty()) ops.push_back({true, r, static_cast<char*>(d.p) + soff[r], sbuf[r].size() * sizeof(T)});
            if (!rbuf[r].empty()) ops.push_back({false, r, static_cast<char*>(d.p) + roff[r], rbuf[r].size() * sizeof(T)});
        }
        if (!ops.empty()) w->exchange(ops, st);
        std::vector<char> hr(std::max<size_t>(tot - sb, 1));
        if (tot > sb) NHIP(hipMemcpyAsync(hr.data(), static_cast<char*>(d.p) + sb, tot - sb, hipMemcpyDeviceToHost, st));
        NHIP(hipStreamSynchronize(st));
        for (int r = 0; r < ws; ++r)
            if (r != me && !rbuf[r].empty())
                std::memcpy(rbuf[r].data(), hr.data() + (roff[r] - sb), rbuf[r].size() * sizeof(T));
    }
    std::vector<size_t> pos((size_t)ws, 0);
    if (to_native) dst_walk([&](int s, T* x) { *x = rbuf[s][pos[s]++]; });
    else src_walk([&](int d, T* x) { *x = rbuf[d][pos[d]++]; });
}

}  // namespace capi
}  // namespace native
}  // namespace slate_amd
