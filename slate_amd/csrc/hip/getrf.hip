// LU panel factorization with partial pivoting on gfx950 -- the GPU panel
// SLATE does not have (its getrf panel always runs on the host,
// src/getrf.cc:95, src/internal/Tile_getrf.hh:160-447).
//
// Recursive (Toledo) on the panel columns so almost all flops are MFMA
// GEMMs / blocked TRSMs:
//     getrf(A) = getrf(A_left); laswp(A_right); trsm; gemm; getrf(A22); laswp(A_left)
//
// Base case (<= 32 columns): one launch per column over many workgroups
// and NO intra-kernel synchronisation (no fences, atomics or grid barriers;
// release/acquire fences cost microseconds each on gfx950):
//   launch j: every workgroup (a) reduces the per-workgroup arg-max
//   partials that launch j-1 left in a parity buffer -> pivot p of column
//   j-1 and the winning candidate row (also left there); (b) applies the
//   row interchange j-1 <-> p on the rows it owns (the old row j-1 was saved
//   by launch j-1, so no two workgroups read a row another one writes);
//   (c) eliminates column j-1 on its rows with the whole row segment held in
//   registers; (d) publishes its local arg-max of column j plus that row and
//   (owner of row j) the current row j.
// Kernel boundaries order the columns, so the panel is stream-ordered
// (graph-capturable, no host sync, no co-residency assumption).
#include <atomic>
#include <cstdlib>
#include <string>
#include <type_traits>
#include "common.hpp"
#include "kernels.hpp"
#include "launchers.hpp"

namespace slate_hip {

namespace {
constexpr int NBB = 32;          // base-case width
constexpr int NTH = 256;         // threads per workgroup (one row each per chunk)
constexpr int MAXG = 128;        // max workgroups per base launch (candidate rows staged in LDS)

template <typename T>
struct PanelBuf {                // one parity half of the device workspace
    double val[MAXG];
    i64 idx[MAXG];
    T cand[MAXG][NBB];
    T diag[NBB];
};
constexpr size_t PANEL_BYTES = 2 * sizeof(PanelBuf<zcplx>);

// (v, i) beats (w, k): NaN wins, then larger, then lower index
template <typename R>
__device__ inline bool beats(R v, i64 i, R w, i64 k) {
    return (v != v && w == w) || v > w || (v == w && i < k);
}
template <typename X>
__device__ inline X xshfl(X v, int o) {
    static_assert(sizeof(X) % 4 == 0, "");
    union U { X x; int w[sizeof(X) / 4]; } a, b;
    a.x = v;
    #pragma unroll
    for (int k = 0; k < (int)(sizeof(X) / 4); ++k) b.w[k] = __shfl_xor(a.w[k], o, 64);
    return b.x;
}
template <typename R>
__device__ inline void wave_argmax(R& v, i64& i, int& g) {
    #pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        R w = xshfl(v, o);
        i64 k = xshfl(i, o);
        int h = __shfl_xor(g, o, 64);
        if (beats(w, k, v, i)) { v = w; i = k; g = h; }
    }
}
}  // namespace

// One launch per column j of the base block [c0, c1) (plus a final j = c1):
//   prologue: every load this launch needs is issued at once -- this
//     thread's row segment, launch j-1's arg-max partials, ALL candidate rows
//     (<= 128 x 32, staged in LDS) and the saved row j-1;
//   (a) pivot of column j-1 = reduction of the partials (wave shuffles);
//   (b) row interchange: the pivot row comes from LDS, the owner of row p
//     takes the saved old row j-1 -- no workgroup reads a row another writes;
//   (c) elimination of column j-1 in registers;
//   (d) arg-max of column j on the updated registers, the winning row and
//     row j are published from registers (no global re-read).
// Only two dependent global round trips per launch; ordering between columns
// comes from kernel boundaries (no fences, atomics or grid barriers).
template <typename T>
__global__ void __launch_bounds__(NTH)
getrf_base_step(i64 m, int c0, int c1, int j, T* A, i64 lda, i64* ipiv, i64 ioff, i64* info,
                i64 info_off, void* work, double thr, bool nopiv) {
    using R = typename scalar_traits<T>::real;
    __shared__ T candL[MAXG * NBB];
    __shared__ T prow[NBB], drow[NBB], orow[NBB];
    __shared__ R wv[NTH / 64];
    __shared__ i64 wi[NTH / 64];
    __shared__ int wg[NTH / 64];
    __shared__ i64 s_p;
    __shared__ int s_gw, s_bt;
    PanelBuf<T>* pb = reinterpret_cast<PanelBuf<T>*>(work);
    const int G = gridDim.x, g = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const i64 rows_per = (m + G - 1) / G;
    const i64 r0 = (i64)g * rows_per, r1 = min(m, r0 + rows_per);
    const int w = c1 - c0;
    const int pc = j - 1;
    const bool first = (j == c0), last = (j >= c1);
    const bool single = rows_per <= NTH;            // one row per thread: full register path
    // ---------------- prologue: issue every independent load, partials first
    // (the compiler then waits for them with vmcnt(N) while the row loads
    // are still in flight)
    R pv = R(-1); i64 pidx = pc; int pg = -1;
    constexpr int PER = MAXG * NBB / NTH;
    T cv[PER];
    T dv = s_zero(T());
    if (!first) {
        PanelBuf<T>& in = pb[pc & 1];
        if (!nopiv && tid < G) { pv = (R)in.val[tid]; pidx = in.idx[tid]; pg = tid; }
        if (tid < w) dv = in.diag[tid];
        // unconditional loads from clamped (always valid) addresses: a
        // load under a runtime select makes hipcc wait for each one
        #pragma unroll
        for (int k = 0; k < PER; ++k) {
            const int e = tid + k * NTH, q = min(e / NBB, G - 1);
            cv[k] = in.cand[q][e % NBB];
        }
    }
    const i64 i0 = r0 + tid;
    T a[NBB];
    const bool mine = single && i0 < r1 && (first ? i0 >= j : i0 > pc);
    {
        const i64 ir = mine ? i0 : 0;
        #pragma unroll
        for (int c = 0; c < NBB; ++c) a[c] = A[ir + (i64)(c0 + min(c, w - 1)) * lda];
    }
    if (!first) {
        if (tid < w) drow[tid] = dv;
        #pragma unroll
        for (int k = 0; k < PER; ++k) {
            const int e = tid + k * NTH, q = e / NBB, c = e % NBB;
            if (q < G && c < w) candL[q * NBB + c] = cv[k];
        }
    }
    // ---------------- (a) pivot of column j-1
    i64 p = pc;
    if (!first) {
        if (!nopiv) {
            wave_argmax(pv, pidx, pg);
            if (lane == 0) { wv[wid] = pv; wi[wid] = pidx; wg[wid] = pg; }
        }
        __syncthreads();
        if (tid == 0) {
            int gw = -1;
            i64 pp = pc;
            if (!nopiv) {
                R bv = wv[0]; i64 bi = wi[0]; gw = wg[0];
                for (int k = 1; k < NTH / 64; ++k)
                    if (beats(wv[k], wi[k], bv, bi)) { bv = wv[k]; bi = wi[k]; gw = wg[k]; }
                pp = bi;
                if (gw < 0) pp = pc;
                else if (thr < 1.0) {
                    R dj = s_abs1(drow[pc - c0]);
                    if (dj == dj && (double)dj >= thr * (double)bv) { pp = pc; gw = -1; }
                }
                if (pp == pc) gw = -1;
            }
            s_p = pp; s_gw = gw;
        }
        __syncthreads();
        p = s_p;
        const int gw = s_gw;
        if (tid < w) prow[tid] = (gw < 0) ? drow[tid] : candL[gw * NBB + tid];
        __syncthreads();
        if (g == 0 && tid == 0) {
            if (ipiv) ipiv[pc] = p + ioff;
            if (s_is_zero(prow[pc - c0]) && info)
                atomicCAS(reinterpret_cast<unsigned long long*>(info), 0ull,
                          (unsigned long long)(pc + 1 + info_off));
        }
        // (b) new row pc = pivot row (its owner writes it)
        if (pc >= r0 && pc < r1 && tid < w) A[pc + (i64)(c0 + tid) * lda] = prow[tid];
    }
    const T u = first ? s_zero(T()) : prow[pc - c0];
    const bool uz = s_is_zero(u);
    R best = R(-1); i64 bi = j;
    if (single) {
        if (mine && !first) {
            const bool isp = (i0 == p) && p != pc;
            if (isp) {
                #pragma unroll
                for (int c = 0; c < NBB; ++c) if (c < w) a[c] = drow[c];
            }
            // (c) eliminate column pc (compile-time indices only: no scratch)
            T l = s_zero(T());
            #pragma unroll
            for (int c = 0; c < NBB; ++c) if (c0 + c == pc) l = a[c];
            if (!uz) l = s_div(l, u);
            #pragma unroll
            for (int c = 0; c < NBB; ++c) {
                if (c0 + c == pc) a[c] = l;
                else if (c < w && c0 + c > pc) a[c] = s_sub(a[c], s_mul(l, prow[c]));
            }
            #pragma unroll
            for (int c = 0; c < NBB; ++c)
                if (c < w && (isp || c0 + c >= pc)) A[i0 + (i64)(c0 + c) * lda] = a[c];
        }
        if (mine && !last && !nopiv) {
            T aj = s_zero(T());
            #pragma unroll
            for (int c = 0; c < NBB; ++c) if (c0 + c == j) aj = a[c];
            best = s_abs1(aj); bi = i0;
        }
    } else {
        // many rows per thread (very tall panels): loop; the winning row is
        // re-read from memory below
        for (i64 i = r0 + tid; i < r1; i += NTH) {
            if (first ? i < j : i <= pc) continue;
            T b[NBB];
            const bool isp = !first && i == p && p != pc;
            #pragma unroll
            for (int c = 0; c < NBB; ++c) if (c < w) b[c] = A[i + (i64)(c0 + c) * lda];
            if (isp) {
                #pragma unroll
                for (int c = 0; c < NBB; ++c) if (c < w) b[c] = drow[c];
            }
            if (!first) {
                T l = s_zero(T());
                #pragma unroll
                for (int c = 0; c < NBB; ++c) if (c0 + c == pc) l = b[c];
                if (!uz) l = s_div(l, u);
                #pragma unroll
                for (int c = 0; c < NBB; ++c) {
                    if (c0 + c == pc) b[c] = l;
                    else if (c < w && c0 + c > pc) b[c] = s_sub(b[c], s_mul(l, prow[c]));
                }
                #pragma unroll
                for (int c = 0; c < NBB; ++c)
                    if (c < w && (isp || c0 + c >= pc)) A[i + (i64)(c0 + c) * lda] = b[c];
            }
            if (!last && !nopiv) {
                T aj = s_zero(T());
                #pragma unroll
                for (int c = 0; c < NBB; ++c) if (c0 + c == j) aj = b[c];
                R v = s_abs1(aj);
                if (beats(v, i, best, bi)) { best = v; bi = i; }
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    if (last) return;
    // ---------------- (d) arg-max of column j, publish winner row and row j
    PanelBuf<T>& out = pb[j & 1];
    if (single && mine && i0 == j) {
        #pragma unroll
        for (int c = 0; c < NBB; ++c) if (c < w) out.diag[c] = a[c];
    }
    if (!single) {
        __syncthreads();                       // rows stored by other threads of this block
        if (j >= r0 && j < r1 && tid < w) out.diag[tid] = A[j + (i64)(c0 + tid) * lda];
    }
    if (nopiv) {
        if (tid == 0) { out.val[g] = -1.0; out.idx[g] = j; }
        return;
    }
    int bt = tid;
    wave_argmax(best, bi, bt);
    if (lane == 0) { wv[wid] = best; wi[wid] = bi; wg[wid] = bt; }
    __syncthreads();
    if (tid == 0) {
        R bv = wv[0]; i64 bb = wi[0]; int t = wg[0];
        for (int k = 1; k < NTH / 64; ++k)
            if (beats(wv[k], wi[k], bv, bb)) { bv = wv[k]; bb = wi[k]; t = wg[k]; }
        out.val[g] = (double)bv;
        out.idx[g] = bb;
        wi[0] = bb;
        s_bt = (bv >= R(0) || bv != bv) ? t : -1;
    }
    __syncthreads();
    if (single) {
        if (tid == s_bt) {
            #pragma unroll
            for (int c = 0; c < NBB; ++c) if (c < w) orow[c] = a[c];
        }
    } else if (s_bt >= 0 && tid < w) {
        orow[tid] = A[wi[0] + (i64)(c0 + tid) * lda];
    }
    __syncthreads();
    if (s_bt >= 0 && tid < w) out.cand[g][tid] = orow[tid];
}

// ---------------------------------------------------------------------------
// Persistent base case (fp64, partial pivoting): ONE launch factors all
// (<= 32) columns of a base block.  G <= 64 co-resident workgroups of 512
// threads each hold R rows of the block per thread (R = 1: m <= 32768,
// R = 2: m <= 65536) in registers for the whole launch; per column the only
// cross-CU traffic is
//   publish: local arg-max (value, row) + the winning row + (owner) row j,
//            all write-through (sc1) stores, drained, then ONE agent-scope
//            atomic add per workgroup on a column counter;
//   gather : one lane polls the counter (sc1 loads, bounded spin), then the
//            partials and the winning row are read with sc1 loads.
// (MI355X_MICROARCH.md "Valid forms", first row of the sc1 hand-off table.)
// Replaces w+1 launches of getrf_base_step (one per column, each re-reading
// the block from memory): the column chain is the critical path of getrf.
//
// Co-residency is not guaranteed (another process or a long kernel can hold
// the CUs), so the launch ends by CONSENSUS on one state word:
//   0 running -> 1 committed : the last workgroup to finish the column loop
//                              (all G finished: nobody can abort any more)
//   0 running -> 2 aborted   : a workgroup whose bounded spin ran out
// Workgroups write the block back only when the state is 1.  On 2 the block
// is untouched and the workgroup that won the abort CAS factors it alone
// (single-workgroup global-memory LU, same pivoting rule): the result is
// always correct, only slower; g_lu_fallbacks counts such launches.
constexpr int PG = 64;           // max workgroups (one per CU on the reserved CUs)
constexpr int PT2 = 512;         // threads per workgroup
// Launch words: cnt = column arrivals, state = 0/1/2 (above), done = loop
// completions.  One 32-byte slot per base launch of a panel, all zeroed by ONE
// memset per panel (not a memset dispatch before every launch).
constexpr int MAXL = 256;        // base launches per panel (N <= MAXL * NBB)
struct LaunchWords {
    unsigned long long cnt, state, done, pad;
};
struct PersistBuf {
    double val[2][PG];
    i64 idx[2][PG];
    double cand[2][PG][NBB];
    double diag[2][NBB];
    LaunchWords lw[MAXL];
};

// tools only: per-phase shader-clock totals of workgroup 0 (lu_persist_profile)
__device__ int g_lu_prof_on = 0;
__device__ unsigned long long g_lu_prof[8];
// failure handling: number of launches that fell back to the one-workgroup
// LU, and a test knob that forces the abort path
__device__ unsigned long long g_lu_fallbacks = 0;
__device__ int g_lu_force_abort = 0;

// wave arg-max of (|value|, row) with a 32-bit row: 3 dwords per shuffle
// round instead of 5
__device__ inline void wave_argmax32(double& v, int& i) {
    #pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const double w = xshfl(v, o);
        const int k = __shfl_xor(i, o, 64);
        if (beats(w, (i64)k, v, (i64)i)) { v = w; i = k; }
    }
}

// Wave arg-max with DPP row permutations (quad xor 1, xor 2, half-row and
// row mirror: every lane of a 16-lane row then holds the row's winner) and
// four v_readlane of the row winners -- no LDS-crossbar (ds_bpermute)
// round trips.  Returns the wave winner in every lane (uniform).
template <int CTRL>
__device__ inline int dpp_i(int x) { return __builtin_amdgcn_update_dpp(0, x, CTRL, 0xF, 0xF, false); }
template <int CTRL>
__device__ inline double dpp_d(double x) {
    const unsigned long long u = __builtin_bit_cast(unsigned long long, x);
    const int lo = dpp_i<CTRL>((int)(u & 0xffffffffu)), hi = dpp_i<CTRL>((int)(u >> 32));
    return __builtin_bit_cast(double, ((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}
template <int CTRL>
__device__ inline void dpp_argmax_step(double& v, int& i, int& g) {
    const double w = dpp_d<CTRL>(v);
    const int k = dpp_i<CTRL>(i), h = dpp_i<CTRL>(g);
    if (beats(w, (i64)k, v, (i64)i)) { v = w; i = k; g = h; }
}
__device__ inline double rdlane_d(double x, int l) {
    const unsigned long long u = __builtin_bit_cast(unsigned long long, x);
    const unsigned lo = __builtin_amdgcn_readlane((int)(u & 0xffffffffu), l);
    const unsigned hi = __builtin_amdgcn_readlane((int)(u >> 32), l);
    return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}
__device__ inline void wave_argmax_dpp(double& v, int& i, int& g) {
    dpp_argmax_step<0xB1>(v, i, g);      // quad_perm [1,0,3,2]
    dpp_argmax_step<0x4E>(v, i, g);      // quad_perm [2,3,0,1]
    dpp_argmax_step<0x141>(v, i, g);     // row_half_mirror
    dpp_argmax_step<0x140>(v, i, g);     // row_mirror
    double bv = rdlane_d(v, 0);
    int bi = __builtin_amdgcn_readlane(i, 0), bg = __builtin_amdgcn_readlane(g, 0);
    #pragma unroll
    for (int r = 1; r < 4; ++r) {
        const double w = rdlane_d(v, 16 * r);
        const int k = __builtin_amdgcn_readlane(i, 16 * r), h = __builtin_amdgcn_readlane(g, 16 * r);
        if (beats(w, (i64)k, bv, (i64)bi)) { bv = w; bi = k; bg = h; }
    }
    v = bv; i = bi; g = bg;
}

__device__ inline double ld_sc1(const double* p) {
    return __builtin_bit_cast(double, __hip_atomic_load(reinterpret_cast<const unsigned long long*>(p),
                                                        __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
__device__ inline i64 ld_sc1(const i64* p) {
    return (i64)__hip_atomic_load(reinterpret_cast<const unsigned long long*>(p), __ATOMIC_RELAXED,
                                  __HIP_MEMORY_SCOPE_AGENT);
}
__device__ inline void st_sc1(double* p, double v) {
    __hip_atomic_store(reinterpret_cast<unsigned long long*>(p), __builtin_bit_cast(unsigned long long, v),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ inline void st_sc1(i64* p, i64 v) {
    __hip_atomic_store(reinterpret_cast<unsigned long long*>(p), (unsigned long long)v, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}
__device__ inline unsigned long long ld_state(const LaunchWords* lw) {
    return __hip_atomic_load(&lw->state, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// CAS running -> to; true if this caller decided the state
__device__ inline bool decide(LaunchWords* lw, unsigned long long to) {
    unsigned long long exp = 0;
    return __hip_atomic_compare_exchange_strong(&lw->state, &exp, to, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT);
}

// Apply the w interchanges piv_s of the block to the OTHER columns of the
// panel (left: factored L, right: not yet factored); workgroup g of G owns
// columns g, g + G, ...  tr_s/ts_s/prv_s/s_nt are LDS scratch.
__device__ void persist_other_cols(double* Ap, i64 lda, const int* piv_s, int* prv_s, int* tr_s, int* ts_s,
                                   int& s_nt, int w, int N, int cabs, int g, int G) {
    const int tid = threadIdx.x;
    if (tid == 0) s_nt = w;
    if (tid < w) prv_s[tid] = -1;
    __syncthreads();
    if (tid < w && piv_s[tid] != tid && piv_s[tid] < w) atomicMax(&prv_s[piv_s[tid]], tid);
    __syncthreads();
    if (tid < w) {
        // parallel fold (see laswp_setup_kernel): the row finally at j came
        // from piv_s[j] just before swap j; prv_s[t] = last swap before t
        // that targets row t
        auto chain = [&](int t) -> int {
            while (prv_s[t] >= 0) t = prv_s[t];
            return t;
        };
        const int q = tid, r = piv_s[q];
        int src;
        if (r == q) {
            src = chain(q);
        } else {
            int kk = -1;
            for (int x = q - 1; x >= 0; --x)
                if (piv_s[x] == r) { kk = x; break; }
            src = (kk < 0) ? r : chain(kk);
        }
        tr_s[q] = q;
        ts_s[q] = src;
        if (r >= w) {
            bool last = true;
            for (int x = q + 1; x < w; ++x)
                if (piv_s[x] == r) { last = false; break; }
            if (last) {
                const int sl = atomicAdd(&s_nt, 1);
                tr_s[sl] = r;
                ts_s[sl] = chain(q);
            }
        }
    }
    __syncthreads();
    const int nt = s_nt, nother = N - w;
    if (g >= nother) return;
    const int mycols = (nother - g + G - 1) / G;
    const int cpc = max(1, PT2 / nt);                   // whole columns per chunk
    for (int k0 = 0; k0 < mycols; k0 += cpc) {
        const int e = tid, t = e % nt, kk = k0 + e / nt;
        const bool act = (e / nt) < cpc && kk < mycols;
        double v = 0.0;
        i64 dst = 0;
        if (act) {
            const int o = g + kk * G;
            const i64 col = o < cabs ? o : o + w;
            v = Ap[ts_s[t] + col * lda];
            dst = tr_s[t] + col * lda;
        }
        __syncthreads();
        if (act) Ap[dst] = v;
        __syncthreads();
    }
}

// The abort path: one workgroup factors the m x w block in global memory
// with the same pivot rule (NaN wins, larger |a|, lower row on ties,
// threshold pivoting) and reports pivots/info like the persistent path.
__device__ void persist_fallback(i64 m, int w, double* A, i64 lda, int* piv_s, double thr, int& zero_at) {
    __shared__ double fv[PT2 / 64];
    __shared__ int fi[PT2 / 64];
    __shared__ int s_piv;
    const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    for (int j = 0; j < w; ++j) {
        double v = -1.0;
        int bi = j;
        for (i64 i = j + tid; i < m; i += PT2) {
            const double x = fabs(A[i + (i64)j * lda]);
            if (beats(x, i, v, (i64)bi)) { v = x; bi = (int)i; }
        }
        wave_argmax32(v, bi);
        if (lane == 0) { fv[wid] = v; fi[wid] = bi; }
        __syncthreads();
        if (tid == 0) {
            double bv = fv[0]; int bb = fi[0];
            for (int k = 1; k < PT2 / 64; ++k)
                if (beats(fv[k], (i64)fi[k], bv, (i64)bb)) { bv = fv[k]; bb = fi[k]; }
            int p = bb;
            if (!(bv >= 0.0) && !(bv != bv)) p = j;
            if (thr < 1.0 && p != j) {
                const double dj = fabs(A[j + (i64)j * lda]);
                if (dj == dj && dj >= thr * bv) p = j;
            }
            s_piv = p;
            piv_s[j] = p;
        }
        __syncthreads();
        const int p = s_piv;
        if (p != j && tid < w) {
            const double t = A[j + (i64)tid * lda];
            A[j + (i64)tid * lda] = A[p + (i64)tid * lda];
            A[p + (i64)tid * lda] = t;
        }
        __syncthreads();
        const double u = A[j + (i64)j * lda];
        if (tid == 0 && u == 0.0 && zero_at < 0) zero_at = j;
        for (i64 i = j + 1 + tid; i < m; i += PT2) {
            double l = A[i + (i64)j * lda];
            if (u != 0.0) l = l / u;
            A[i + (i64)j * lda] = l;
            for (int c = j + 1; c < w; ++c) A[i + (i64)c * lda] -= l * A[j + (i64)c * lda];
        }
        __syncthreads();
    }
}

template <int R>
__global__ void __launch_bounds__(PT2)
getrf_base_persist(i64 m, int w, double* __restrict__ A, i64 lda, i64* ipiv, i64 ioff, i64* info, i64 info_off,
                   PersistBuf* pb, LaunchWords* lw, double thr, int N, int cabs) {
    __shared__ double wv[2 * (PT2 / 64)];          // wave partials, per column parity
    __shared__ i64 wi[2 * (PT2 / 64)];
    __shared__ double prow[NBB], drow[NBB], qrow[NBB], ud_s[NBB];
    __shared__ double candL[PG][NBB];
    __shared__ i64 s_p;
    __shared__ int s_gw, s_abort, s_won, s_zero;
    __shared__ int piv_s[NBB], prv_s[NBB], tr_s[2 * NBB], ts_s[2 * NBB], s_nt;
    const int G = gridDim.x, g = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const i64 rbase = (i64)g * PT2 * R;
    double a[R][NBB];
    #pragma unroll
    for (int r = 0; r < R; ++r) {
        const i64 i = rbase + r * PT2 + tid;
        const i64 ir = i < m ? i : 0;
        #pragma unroll
        for (int c = 0; c < NBB; ++c) a[r][c] = A[ir + (i64)min(c, w - 1) * lda];
    }
    if (tid == 0) { s_abort = 0; s_won = 0; }
    int zero_at = -1;
    const bool prof = g_lu_prof_on && g == 0 && tid == 0;
    unsigned long long tl = prof ? clock64() : 0, ph[5] = {0, 0, 0, 0, 0};
#define LSTAMP(k) do { if (prof) { const unsigned long long t_ = clock64(); ph[k] += t_ - tl; tl = t_; } } while (0)
    // w in a VGPR: per-lane compares give v_cndmask selects instead of 32
    // uniform branches per column-indexed loop
    int wv_; asm volatile("v_mov_b32 %0, %1" : "=v"(wv_) : "s"(w));
    for (int j = 0; j < w; ++j) {
        const int par = j & 1;
        int jv; asm volatile("v_mov_b32 %0, %1" : "=v"(jv) : "s"(j));
        // ---- local arg-max of column j over unpivoted rows (i >= j); the
        //      raw column value is kept for the elimination below
        double v = -1.0;
        int bi = (int)(rbase + tid);                  // rows < 2^31
        double aj[R];
        #pragma unroll
        for (int r = 0; r < R; ++r) {
            const i64 i = rbase + r * PT2 + tid;
            double x = 0.0;
            #pragma unroll
            for (int c = 0; c < NBB; ++c) x = (c == jv) ? a[r][c] : x;
            aj[r] = x;
            const double vr = (i < m && i >= j) ? fabs(x) : -1.0;
            if (r == 0 || beats(vr, i, v, (i64)bi)) { v = vr; bi = (int)i; }
        }
        {
            int dummy = 0;
            wave_argmax_dpp(v, bi, dummy);
        }
        // winner's thread (and register slot): row - rbase = slot * PT2 + thread
        if (lane == 0) { wv[par * 8 + wid] = v; wi[par * 8 + wid] = bi; }
        __syncthreads();
        // every thread reduces the 8 wave partials (LDS broadcast reads): the
        // winning thread publishes without a second barrier
        double bv = wv[par * 8];
        int bb = (int)wi[par * 8];
        #pragma unroll
        for (int k = 1; k < PT2 / 64; ++k) {
            const double x = wv[par * 8 + k];
            const int y = (int)wi[par * 8 + k];
            if (beats(x, (i64)y, bv, (i64)bb)) { bv = x; bb = y; }
        }
        const int s_bt_ = bb - (int)rbase;
        LSTAMP(0);                                      // local arg-max
        // ---- publish the winning row (+ its value and row index) and (owner)
        //      row j, write-through
        #pragma unroll
        for (int r = 0; r < R; ++r) {
            if (tid + r * PT2 == s_bt_) {
                #pragma unroll
                for (int c = 0; c < NBB; ++c) st_sc1(&pb->cand[par][g][c], a[r][c]);   // all NBB: no uniform branches
                st_sc1(&pb->val[par][g], bv);
                st_sc1(&pb->idx[par][g], (i64)bb);
            }
            if (rbase + r * PT2 + tid == j) {
                #pragma unroll
                for (int c = 0; c < NBB; ++c) st_sc1(&pb->diag[par][c], a[r][c]);
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        LSTAMP(1);                                      // publish + drain
        if (tid == 0) {
            __hip_atomic_fetch_add(&lw->cnt, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const unsigned long long target = (unsigned long long)(j + 1) * G;
            int spins = 0;
            const bool force = g_lu_force_abort && g == 0 && j == 0;
            while (force || __hip_atomic_load(&lw->cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
                if (force || ++spins > (1 << 22)) {     // not co-resident: abort, never hang
                    s_won = decide(lw, 2) ? 1 : 0;
                    s_abort = 1;
                    break;
                }
                if ((spins & 255) == 0 && ld_state(lw) == 2) { s_abort = 1; break; }
                __builtin_amdgcn_s_sleep(1);
            }
        }
        LSTAMP(2);                                      // arrive + poll
        __syncthreads();
        if (s_abort) break;
        // ---- global pivot: every candidate row, the partials and row j are
        //      fetched in ONE round of sc1 loads (no dependent second trip)
        {
            double cv[PG * NBB / PT2];
            #pragma unroll
            for (int k = 0; k < PG * NBB / PT2; ++k) {
                const int e = tid + k * PT2, q = min(e / NBB, G - 1), c = e % NBB;
                cv[k] = ld_sc1(&pb->cand[par][q][c]);
            }
            if (tid < w) drow[tid] = ld_sc1(&pb->diag[par][tid]);
            #pragma unroll
            for (int k = 0; k < PG * NBB / PT2; ++k) {
                const int e = tid + k * PT2, q = e / NBB, c = e % NBB;
                if (q < G) candL[q][c] = cv[k];
            }
        }
        if (wid == 0) {
            double pv = -1.0; int pi = j; int pg = -1;
            if (lane < G) { pv = ld_sc1(&pb->val[par][lane]); pi = (int)ld_sc1(&pb->idx[par][lane]); pg = lane; }
            wave_argmax_dpp(pv, pi, pg);
            if (lane == 0) {
                i64 p = pi;
                int gw = pg;
                if (!(pv >= 0.0) && !(pv != pv)) { p = j; gw = -1; }
                if (thr < 1.0 && gw >= 0) {
                    const double dj = fabs(drow[j]);
                    if (dj == dj && dj >= thr * pv) { p = j; gw = -1; }
                }
                if (p == j) gw = -1;
                s_p = p; s_gw = gw;
            }
        }
        __syncthreads();
        LSTAMP(3);                                      // gather + global arg-max
        const i64 p = s_p;
        const int gw = s_gw;
        // pivot row, and its trailing part (columns j < c < w; zeros elsewhere)
        // as the multiplier row of the elimination
        if (tid < NBB) {
            const double x = (tid < w) ? ((gw < 0) ? drow[tid] : candL[gw][tid]) : 0.0;
            prow[tid] = x;
            qrow[tid] = (tid > j && tid < w) ? x : 0.0;
        }
        __syncthreads();
        const double u = prow[j];
        if (tid == 0) {
            piv_s[j] = (int)p;
            ud_s[j] = u;
            if (u == 0.0 && zero_at < 0) zero_at = j;     // first exactly-zero pivot (reported at the end)
        }
        // ---- interchange rows j <-> p and eliminate column j (registers).
        // The L entry stays UNSCALED in the register (qrow[j] = 0, so the
        // update below leaves column j and every factored column untouched:
        // 32 FMAs per row, no per-column selects); the write-back divides by
        // the pivot ud_s[c] -- bitwise the l = x / u used here.
        #pragma unroll
        for (int r = 0; r < R; ++r) {
            const i64 i = rbase + r * PT2 + tid;
            if (i < m && i >= j) {
                if (i == j) {
                    #pragma unroll
                    for (int c = 0; c < NBB; ++c) a[r][c] = (c < wv_) ? prow[c] : a[r][c];
                } else {
                    double x = aj[r];
                    if (i == p) {
                        #pragma unroll
                        for (int c = 0; c < NBB; ++c) a[r][c] = (c < wv_) ? drow[c] : a[r][c];
                        x = drow[j];
                    }
                    const double l = (u != 0.0) ? x / u : x;
                    #pragma unroll
                    for (int c = 0; c < NBB; ++c) a[r][c] = fma(-l, qrow[c], a[r][c]);
                }
            }
        }
        LSTAMP(4);                                      // interchange + elimination
    }
#undef LSTAMP
    if (prof) {
        #pragma unroll
        for (int k = 0; k < 5; ++k) g_lu_prof[k] += ph[k];
    }
    // ---- consensus: commit (every workgroup finished the loop) or abort
    if (tid == 0 && !s_abort) {
        const unsigned long long before =
            __hip_atomic_fetch_add(&lw->done, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (before + 1 == (unsigned long long)G) decide(lw, 1);
        int spins = 0;
        while (ld_state(lw) == 0) {
            if (++spins > (1 << 22)) { s_won = decide(lw, 2) ? 1 : 0; break; }
            __builtin_amdgcn_s_sleep(1);
        }
        s_abort = ld_state(lw) == 2 ? 1 : 0;
    }
    __syncthreads();
    if (s_abort) {
        if (!s_won) return;                             // block untouched: the winner redoes it alone
        if (tid == 0) { s_zero = -1; atomicAdd(&g_lu_fallbacks, 1ull); }
        __syncthreads();
        int zf = -1;
        persist_fallback(m, w, A, lda, piv_s, thr, zf);
        if (tid == 0) s_zero = zf;
        __syncthreads();
        if (ipiv && tid < w) ipiv[tid] = piv_s[tid] + ioff;
        if (tid == 0 && s_zero >= 0 && info)
            atomicCAS(reinterpret_cast<unsigned long long*>(info), 0ull, (unsigned long long)(s_zero + 1 + info_off));
        if (N > w) persist_other_cols(A - (i64)cabs * lda, lda, piv_s, prv_s, tr_s, ts_s, s_nt, w, N, cabs, 0, 1);
        return;
    }
    // pivots and info once per launch (global stores kept out of the column loop)
    if (g == 0) {
        if (ipiv && tid < w) ipiv[tid] = piv_s[tid] + ioff;
        if (tid == 0 && zero_at >= 0 && info)
            atomicCAS(reinterpret_cast<unsigned long long*>(info), 0ull, (unsigned long long)(zero_at + 1 + info_off));
    }
    // write-back: L entries (row below the column) scaled by their pivot now
    #pragma unroll
    for (int r = 0; r < R; ++r) {
        const i64 i = rbase + r * PT2 + tid;
        if (i < m) {
            #pragma unroll
            for (int c = 0; c < NBB; ++c) {
                if (c < w) {
                    double x = a[r][c];
                    const double d = ud_s[c];
                    if (i > c && d != 0.0) x = x / d;
                    A[i + (i64)c * lda] = x;
                }
            }
        }
    }
    // ---- the same w interchanges on every OTHER column of the panel, so the
    // recursion needs no laswp.  Every workgroup knows the whole swap sequence.
    if (N <= w) return;
    __syncthreads();
    persist_other_cols(A - (i64)cabs * lda, lda, piv_s, prv_s, tr_s, ts_s, s_nt, w, N, cabs, g, G);
}

// ---------------------------------------------------------------------------
// Tagged persistent base case (fp64, partial pivoting) -- ONE hand-off per
// column instead of three.  getrf_base_persist publishes (drain) -> arrives
// on a counter -> polls -> gathers: three dependent memory round trips plus
// five barriers per column (~7 us).  Here every workgroup's per-column record
// (winning row, |value|, row index) is written as 8-byte DATA-TAGGED granules
// {tag = column epoch : 32-bit payload} (MI355X_MICROARCH.md hand-off table,
// handoff-1to1 / R2: the data IS the flag -- no drain, no counter, no
// fence).  Every workgroup sweeps the G records (each wave a few of them)
// until every tag carries this column's epoch, assembles the candidates in
// LDS, and picks the pivot redundantly (deterministic: same choice
// everywhere).  The column loop is unrolled over the 32 columns, so column
// j of the register-resident rows is a compile-time register (no per-column
// select chains) and the elimination only touches the columns right of j.
// A double travels as two granules (low / high word); 2-slot parity is safe
// because a workgroup writes column j+2's record only after every workgroup
// published j+1, i.e. after everyone consumed column j.
// Epochs are unique per launch (a host counter advanced by w + 2 per launch;
// never 0), so no slot ever needs zeroing.
struct TagRec {                  // one workgroup's record of one column
    unsigned long long g[68];    // [2c] / [2c+1] = lo / hi word of row value c; [64..65] |v|; [66] row
    unsigned long long pad[4];
};
struct TagBuf {
    TagRec rec[2][PG];
    unsigned long long diag[2][64];   // row j (its owner): lo / hi words
};

__device__ inline void st_tag(unsigned long long* p, unsigned ep, unsigned v) {
    __hip_atomic_store(p, ((unsigned long long)ep << 32) | v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ inline unsigned long long ld_tag(const unsigned long long* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ inline unsigned lo32(double x) { return (unsigned)(__builtin_bit_cast(unsigned long long, x) & 0xffffffffu); }
__device__ inline unsigned hi32(double x) { return (unsigned)(__builtin_bit_cast(unsigned long long, x) >> 32); }
__device__ inline double mk_d(unsigned lo, unsigned hi) {
    return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}

template <int R>
__global__ void __launch_bounds__(PT2)
getrf_base_tag(i64 m, int w, double* __restrict__ A, i64 lda, i64* ipiv, i64 ioff, i64* info, i64 info_off,
               TagBuf* tb, LaunchWords* lw, double thr, int N, int cabs, unsigned ep0) {
    __shared__ double wv[PT2 / 64];
    __shared__ int wi[PT2 / 64];
    // parity double-buffered: column j+1's sweep fills one half while
    // late waves still eliminate column j from the other
    __shared__ double candL[2][PG][NBB + 1];
    __shared__ double pvL[2][PG];
    __shared__ int piL[2][PG];
    __shared__ double drowL[2][NBB];
    __shared__ double stg[2][NBB];          // staged winner row / next diagonal row
    __shared__ double ud_s[NBB];
    __shared__ int s_abort, s_won, s_zero;
    __shared__ int piv_s[NBB], prv_s[NBB], tr_s[2 * NBB], ts_s[2 * NBB], s_nt;
    const int G = gridDim.x, g = blockIdx.x, tid = threadIdx.x, lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const i64 rbase = (i64)g * PT2 * R;
    double a[R][NBB];
    #pragma clang loop unroll(full)
    for (int r = 0; r < R; ++r) {
        const i64 i = rbase + r * PT2 + tid;
        const i64 ir = i < m ? i : 0;
        #pragma clang loop unroll(full)
        for (int c = 0; c < NBB; ++c) a[r][c] = A[ir + (i64)min(c, w - 1) * lda];
    }
    if (tid == 0) { s_abort = 0; s_won = 0; }
    int zero_at = -1;
    const bool prof = g_lu_prof_on && g == 0 && tid == 0;
    unsigned long long tl = prof ? clock64() : 0, ph[5] = {0, 0, 0, 0, 0};
#define TSTAMP(k) do { if (prof) { const unsigned long long t_ = clock64(); ph[k] += t_ - tl; tl = t_; } } while (0)
    // local arg-max of column JJ over rows i >= JJ, block winner (bv, bb)
    // uniform after the barrier
#define TAG_ARGMAX(JJ)                                                                       \
    double bv, v = -1.0;                                                                     \
    int bb, bi = (int)(rbase + tid);                                                          \
    _Pragma("clang loop unroll(full)") for (int r = 0; r < R; ++r) {                                          \
        const i64 i = rbase + r * PT2 + tid;                                                  \
        const double vr = (i < m && i >= (JJ)) ? fabs(a[r][(JJ)]) : -1.0;                    \
        if (r == 0 || beats(vr, i, v, (i64)bi)) { v = vr; bi = (int)i; }                      \
    }                                                                                        \
    { int dummy = 0; wave_argmax_dpp(v, bi, dummy); }                                        \
    if (lane == 0) { wv[wid] = v; wi[wid] = bi; }                                            \
    __syncthreads();                                                                         \
    bv = wv[0]; bb = wi[0];                                                                  \
    _Pragma("clang loop unroll(full)") for (int k = 1; k < PT2 / 64; ++k)                                     \
        if (beats(wv[k], (i64)wi[k], bv, (i64)bb)) { bv = wv[k]; bb = wi[k]; }
    // the staged rows (stg) go out as tagged granules, one or two per lane:
    // wave 0 the winning row and (|v|, row), wave 1 the row JJ (its owner)
#define TAG_PUBLISH(JJ)                                                                      \
    {                                                                                        \
        const int par_ = (JJ) & 1;                                                           \
        const unsigned ep_ = ep0 + (unsigned)(JJ) + 1u;                                      \
        const bool own_d = (JJ) >= rbase && (JJ) < rbase + (i64)R * PT2;                      \
        if (wid == 0) {                                                                      \
            const double x = stg[0][lane >> 1];                                              \
            st_tag(&tb->rec[par_][g].g[lane], ep_, (lane & 1) ? hi32(x) : lo32(x));          \
            if (lane < 2) st_tag(&tb->rec[par_][g].g[64 + lane], ep_, lane ? hi32(bv) : lo32(bv)); \
            if (lane == 2) st_tag(&tb->rec[par_][g].g[66], ep_, (unsigned)bb);               \
        } else if (wid == 1 && own_d) {                                                      \
            const double x = stg[1][lane >> 1];                                              \
            st_tag(&tb->diag[par_][lane], ep_, (lane & 1) ? hi32(x) : lo32(x));              \
        }                                                                                    \
    }
    __syncthreads();                                   // s_abort / s_won initialised
    // ---- column 0: arg-max, stage, publish
    if (w > 0) {
        TAG_ARGMAX(0)
        #pragma clang loop unroll(full)
        for (int r = 0; r < R; ++r) {
            const i64 i = rbase + r * PT2 + tid;
            if (i == bb) {
                #pragma clang loop unroll(full)
                for (int c = 0; c < NBB; ++c) stg[0][c] = a[r][c];
            }
            if (i == 0) {
                #pragma clang loop unroll(full)
                for (int c = 0; c < NBB; ++c) stg[1][c] = a[r][c];
            }
        }
        __syncthreads();
        TAG_PUBLISH(0)
    }
    TSTAMP(1);
    // fully unrolled: j is a compile-time constant in every copy, so a[r][j]
    // is a fixed register and the elimination touches columns > j only.
    // Per column: sweep(j) -> pivot(j) -> interchange, multipliers and
    // column j+1 only -> arg-max(j+1) -> the two publishing rows finish
    // their elimination, are staged and go out -> everyone else finishes
    // the elimination of column j while the records are in flight.
    #pragma clang loop unroll(full)
    for (int j = 0; j < NBB; ++j) {
        if (j < w && !s_abort) {
            const int par = j & 1;
            const unsigned ep = ep0 + (unsigned)j + 1u;
            // ---- sweep: wave q polls records q, q + 8, ...; wave (G % 8) also
            //      the row-j record.  Each lane owns one row granule (+ lanes
            //      0..2 the value / index granules) of each of its records.
            {
                const bool dwave = wid == (G & 7);
                int spins = 0;
                const bool force = g_lu_force_abort && g == 0 && j == 0;
                for (;;) {
                    bool ok = true;
                    for (int q = wid; q < G; q += PT2 / 64) {
                        const unsigned long long x = ld_tag(&tb->rec[par][q].g[lane]);
                        const unsigned long long y = lane < 3 ? ld_tag(&tb->rec[par][q].g[64 + lane])
                                                              : ((unsigned long long)ep << 32);
                        ok &= (unsigned)(x >> 32) == ep && (unsigned)(y >> 32) == ep;
                        // lanes 2c / 2c + 1 hold lo / hi of value c
                        const unsigned o = (unsigned)__shfl_xor((int)(unsigned)x, 1, 64);
                        if ((lane & 1) == 0) candL[par][q][lane >> 1] = mk_d((unsigned)x, o);
                        const unsigned y1 = (unsigned)__shfl((int)(unsigned)y, 1, 64);
                        if (lane == 0) pvL[par][q] = mk_d((unsigned)y, y1);
                        if (lane == 2) piL[par][q] = (int)(unsigned)y;
                    }
                    if (dwave) {
                        const unsigned long long x = ld_tag(&tb->diag[par][lane]);
                        ok &= (unsigned)(x >> 32) == ep;
                        const unsigned o = (unsigned)__shfl_xor((int)(unsigned)x, 1, 64);
                        if ((lane & 1) == 0) drowL[par][lane >> 1] = mk_d((unsigned)x, o);
                    }
                    if (__all(ok) && !force) break;
                    if (force || ++spins > (1 << 20)) {           // not co-resident: abort, never hang
                        if (lane == 0) {
                            if (decide(lw, 2)) s_won = 1;
                            s_abort = 1;
                        }
                        break;
                    }
                    if ((spins & 255) == 0 && ld_state(lw) == 2) {
                        if (lane == 0) s_abort = 1;
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                }
            }
            __syncthreads();
            TSTAMP(2);
            if (!s_abort) {
                // ---- global pivot, redundantly in every wave (DPP over the G partials)
                double pv = -1.0;
                int pi = j, pg = -1;
                if (lane < G) { pv = pvL[par][lane]; pi = piL[par][lane]; pg = lane; }
                wave_argmax_dpp(pv, pi, pg);
                i64 p = pi;
                int gw = pg;
                const double* drow = drowL[par];
                if (!(pv >= 0.0) && !(pv != pv)) { p = j; gw = -1; }
                if (thr < 1.0 && gw >= 0) {
                    const double dj = fabs(drow[j]);
                    if (dj == dj && dj >= thr * pv) { p = j; gw = -1; }
                }
                if (p == j) gw = -1;
                const double* prow = gw < 0 ? drow : &candL[par][gw][0];
                const double u = prow[j];
                if (tid == 0) {
                    piv_s[j] = (int)p;
                    ud_s[j] = u;
                }
                if (u == 0.0 && zero_at < 0) zero_at = j;
                TSTAMP(3);
                // ---- interchange rows j <-> p, multipliers, column j+1 only
                double lsv[R];
                bool pend[R];
                #pragma clang loop unroll(full)
                for (int r = 0; r < R; ++r) {
                    const i64 i = rbase + r * PT2 + tid;
                    pend[r] = false;
                    lsv[r] = 0.0;
                    if (i < m && i >= j) {
                        if (i == j) {
                            #pragma clang loop unroll(full)
                            for (int c = 0; c < NBB; ++c) a[r][c] = prow[c];
                        } else {
                            if (i == p) {
                                #pragma clang loop unroll(full)
                                for (int c = 0; c < NBB; ++c) a[r][c] = drow[c];
                            }
                            const double l = (u != 0.0) ? a[r][j] / u : a[r][j];
                            a[r][j] = l;
                            lsv[r] = l;
                            if (j + 1 < NBB) a[r][j + 1] = fma(-l, prow[j + 1], a[r][j + 1]);
                            pend[r] = true;
                        }
                    }
                }
                if (j + 1 < w) {
                    TAG_ARGMAX(j + 1)
                    // the winner and the owner of row j+1 finish their rows now
                    #pragma clang loop unroll(full)
                    for (int r = 0; r < R; ++r) {
                        const i64 i = rbase + r * PT2 + tid;
                        if (pend[r] && (i == bb || i == j + 1)) {
                            #pragma clang loop unroll(full)
                            for (int c = j + 2; c < NBB; ++c) a[r][c] = fma(-lsv[r], prow[c], a[r][c]);
                            pend[r] = false;
                        }
                        if (i == bb) {
                            #pragma clang loop unroll(full)
                            for (int c = 0; c < NBB; ++c) stg[0][c] = a[r][c];
                        }
                        if (i == j + 1) {
                            #pragma clang loop unroll(full)
                            for (int c = 0; c < NBB; ++c) stg[1][c] = a[r][c];
                        }
                    }
                    __syncthreads();
                    TAG_PUBLISH(j + 1)
                }
                // ---- everyone else: the rest of column j's elimination,
                //      overlapping the records' flight
                #pragma clang loop unroll(full)
                for (int r = 0; r < R; ++r) {
                    if (pend[r]) {
                        #pragma clang loop unroll(full)
                        for (int c = j + 2; c < NBB; ++c) a[r][c] = fma(-lsv[r], prow[c], a[r][c]);
                    }
                }
            }
            TSTAMP(4);
        }
    }
#undef TAG_ARGMAX
#undef TAG_PUBLISH
#undef TSTAMP
    if (prof) {
        #pragma unroll
        for (int k = 0; k < 5; ++k) g_lu_prof[k] += ph[k];
    }
    // ---- consensus: commit (every workgroup finished the loop) or abort
    if (tid == 0 && !s_abort) {
        const unsigned long long before =
            __hip_atomic_fetch_add(&lw->done, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (before + 1 == (unsigned long long)G) decide(lw, 1);
        int spins = 0;
        while (ld_state(lw) == 0) {
            if (++spins > (1 << 22)) { s_won = decide(lw, 2) ? 1 : 0; break; }
            __builtin_amdgcn_s_sleep(1);
        }
        s_abort = ld_state(lw) == 2 ? 1 : 0;
    }
    __syncthreads();
    if (s_abort) {
        if (!s_won) return;                             // block untouched: the winner redoes it alone
        if (tid == 0) { s_zero = -1; atomicAdd(&g_lu_fallbacks, 1ull); }
        __syncthreads();
        int zf = -1;
        persist_fallback(m, w, A, lda, piv_s, thr, zf);
        if (tid == 0) s_zero = zf;
        __syncthreads();
        if (ipiv && tid < w) ipiv[tid] = piv_s[tid] + ioff;
        if (tid == 0 && s_zero >= 0 && info)
            atomicCAS(reinterpret_cast<unsigned long long*>(info), 0ull, (unsigned long long)(s_zero + 1 + info_off));
        if (N > w) persist_other_cols(A - (i64)cabs * lda, lda, piv_s, prv_s, tr_s, ts_s, s_nt, w, N, cabs, 0, 1);
        return;
    }
    if (g == 0) {
        if (ipiv && tid < w) ipiv[tid] = piv_s[tid] + ioff;
        if (tid == 0 && zero_at >= 0 && info)
            atomicCAS(reinterpret_cast<unsigned long long*>(info), 0ull, (unsigned long long)(zero_at + 1 + info_off));
    }
    // write-back (L already scaled in the column loop)
    #pragma unroll
    for (int r = 0; r < R; ++r) {
        const i64 i = rbase + r * PT2 + tid;
        if (i < m) {
            #pragma unroll
            for (int c = 0; c < NBB; ++c)
                if (c < w) A[i + (i64)c * lda] = a[r][c];
        }
    }
    if (N <= w) return;
    __syncthreads();
    persist_other_cols(A - (i64)cabs * lda, lda, piv_s, prv_s, tr_s, ts_s, s_nt, w, N, cabs, g, G);
}

// the persistent form needs every row in a register slot of a co-resident
// workgroup: m <= PG * PT2 rows; fp64 partial pivoting only
// Panel-wide context of the recursion: N = panel width; full = the base
// case applies its interchanges to all N columns (persistent kernel), so the
// recursion levels skip their laswp calls.
struct PanelCtx {
    i64 N;
    bool full;
    mutable int launch;          // next base launch's LaunchWords slot
};

template <typename T>
static bool persist_ok(i64 m, bool nopiv) {
    return std::is_same<T, double>::value && !nopiv && m <= (i64)PG * PT2 * 4 && m >= 1 &&
           (m <= (i64)PG * PT2 * 2 || [] { const char* e = std::getenv("SLATE_AMD_LU_RPT"); return e && std::atoi(e) == 4; }());
}

template <typename T>
static void base(i64 m, int c0, int c1, T* A, i64 lda, i64* ipiv, i64 ioff, i64* info, i64 info_off,
                 void* w, double thr, bool nopiv, hipStream_t s, const PanelCtx& ctx, i64 cabs) {
    if constexpr (std::is_same<T, double>::value) {
        if (ctx.full) {
            PersistBuf* pb = reinterpret_cast<PersistBuf*>(static_cast<char*>(w) + PANEL_BYTES);
            // launch words: zeroed once per panel (getrf_panel_ws); a panel
            // with more than MAXL base launches wraps and re-zeroes
            if (ctx.launch >= MAXL) {
                HIP_CHECK(hipMemsetAsync(pb->lw, 0, sizeof(pb->lw), s));
                ctx.launch = 0;
            }
            LaunchWords* lw = pb->lw + ctx.launch++;
            // rows per thread: 2 by default (SLATE_AMD_LU_RPT = 1 / 2 / 4):
            // half the workgroups of one row per thread -- half the arrivals
            // per column and half the CUs the panel stream reserves (dgetrf
            // n = 32768 on one MI355X: 36.1 TF/s with 2 rows / 32 reserved
            // CUs vs 34.0 with 1 row / 64; 4 rows spill: 21)
            static const int rpt = [] {
                const char* e = std::getenv("SLATE_AMD_LU_RPT");
                const int v = e ? std::atoi(e) : 2;
                return (v == 2 || v == 4) ? v : 1;
            }();
            // short panels (the panel-bound tail of a factorization): one row
            // per thread while that still fits the 32 reserved CUs, m <= 32 *
            // 512 (SLATE_AMD_LU_RPT1_ROWS; measured 0 / 8192 / 16384 / 24576:
            // 36.2 / 36.9 / 37.5 / 33.5 TF/s)
            static const i64 rpt1_rows = [] {
                const char* e = std::getenv("SLATE_AMD_LU_RPT1_ROWS");
                return e ? (i64)std::atoll(e) : (i64)32 * PT2;
            }();
            // tagged one-hand-off form (SLATE_AMD_LU_PANEL=counter: the
            // counter/gather form above)
            static const bool tagged = [] {
                const char* e = std::getenv("SLATE_AMD_LU_PANEL");
                return !e || std::string(e) != "counter";
            }();
            if (tagged && rpt != 4) {
                TagBuf* tb = reinterpret_cast<TagBuf*>(reinterpret_cast<char*>(pb) + sizeof(PersistBuf));
                static std::atomic<unsigned> g_ep{1};
                unsigned ep0 = g_ep.fetch_add((unsigned)(NBB + 2));
                if (ep0 == 0 || ep0 + (unsigned)(NBB + 2) < ep0) ep0 = g_ep.fetch_add((unsigned)(NBB + 2));
                if (m <= rpt1_rows && m <= (i64)PG * PT2) {
                    const int G = (int)((m + PT2 - 1) / PT2);
                    hipLaunchKernelGGL(getrf_base_tag<1>, dim3(G), dim3(PT2), 0, s, m, c1, A, lda, ipiv, ioff,
                                       info, info_off, tb, lw, thr, (int)ctx.N, (int)cabs, ep0);
                } else {
                    const int G = (int)((m + 2 * PT2 - 1) / (2 * PT2));
                    hipLaunchKernelGGL(getrf_base_tag<2>, dim3(G), dim3(PT2), 0, s, m, c1, A, lda, ipiv, ioff,
                                       info, info_off, tb, lw, thr, (int)ctx.N, (int)cabs, ep0);
                }
                HIP_LAUNCH_CHECK();
                return;
            }
            if (rpt != 4 && m <= rpt1_rows && m <= (i64)PG * PT2) {
                const int G = (int)((m + PT2 - 1) / PT2);
                hipLaunchKernelGGL(getrf_base_persist<1>, dim3(G), dim3(PT2), 0, s, m, c1, A, lda, ipiv, ioff,
                                   info, info_off, pb, lw, thr, (int)ctx.N, (int)cabs);
            } else if (rpt == 4 && m <= (i64)PG * PT2 * 4) {
                const int G = (int)((m + 4 * PT2 - 1) / (4 * PT2));
                hipLaunchKernelGGL(getrf_base_persist<4>, dim3(G), dim3(PT2), 0, s, m, c1, A, lda, ipiv, ioff,
                                   info, info_off, pb, lw, thr, (int)ctx.N, (int)cabs);
            } else if (rpt == 1 && m <= (i64)PG * PT2) {
                const int G = (int)((m + PT2 - 1) / PT2);
                hipLaunchKernelGGL(getrf_base_persist<1>, dim3(G), dim3(PT2), 0, s, m, c1, A, lda, ipiv, ioff,
                                   info, info_off, pb, lw, thr, (int)ctx.N, (int)cabs);
            } else {
                const int G = (int)((m + 2 * PT2 - 1) / (2 * PT2));
                hipLaunchKernelGGL(getrf_base_persist<2>, dim3(G), dim3(PT2), 0, s, m, c1, A, lda, ipiv, ioff,
                                   info, info_off, pb, lw, thr, (int)ctx.N, (int)cabs);
            }
            HIP_LAUNCH_CHECK();
            return;
        }
    }
    int G = (int)std::min<i64>(MAXG, std::max<i64>(1, (m + NTH - 1) / NTH));
    for (int j = c0; j <= c1; ++j)
        hipLaunchKernelGGL(getrf_base_step<T>, dim3(G), dim3(NTH), 0, s, m, c0, c1, j, A, lda, ipiv, ioff,
                           info, info_off, w, thr, nopiv);
    HIP_LAUNCH_CHECK();
}

template <typename T>
static void gemm_T(char ta, char tb, i64 m, i64 n, i64 k, double alpha, const T* A, i64 lda,
                   const T* B, i64 ldb, double beta, T* C, i64 ldc, hipStream_t s) {
    GemmCall c;
    c.transA = ta; c.transB = tb; c.m = m; c.n = n; c.k = k;
    c.alpha_re = alpha; c.beta_re = beta;
    c.A = A; c.lda = lda; c.B = B; c.ldb = ldb; c.C = C; c.ldc = ldc;
    if constexpr (scalar_traits<T>::is_complex) gemm_complex<T>(c, s);
    else gemm_real<T>(c, s);
}

// ipiv entries are written relative to the TOP of the outermost panel
// (ioff = row offset of this sub-panel); laswp at this level subtracts ioff.

template <typename T>
static void rec(i64 m, i64 n, T* A, i64 lda, i64* ipiv, i64 ioff, i64* info, i64 info_off, void* w,
                double thr, bool nopiv, hipStream_t s, const PanelCtx& ctx, i64 cabs) {
    if (n <= NBB) {
        base<T>(m, 0, (int)n, A, lda, ipiv, ioff, info, info_off, w, thr, nopiv, s, ctx, cabs);
        return;
    }
    i64 n1 = ((n / 2 + NBB - 1) / NBB) * NBB;
    if (n1 >= n) n1 = n - NBB;
    rec<T>(m, n1, A, lda, ipiv, ioff, info, info_off, w, thr, nopiv, s, ctx, cabs);
    T* A12 = A + n1 * lda;
    if (!nopiv && !ctx.full) laswp_off<T>(n - n1, A12, lda, 0, n1, ipiv, ioff, s);
    trsm<T>('L', 'L', 'N', 'U', n1, n - n1, s_from_real(T(), 1), A, lda, A12, lda, s);
    if (m > n1)
        gemm_T<T>('N', 'N', m - n1, n - n1, n1, -1.0, A + n1, lda, A12, lda, 1.0, A12 + n1, lda, s);
    if (m > n1) {
        rec<T>(m - n1, n - n1, A12 + n1, lda, ipiv ? ipiv + n1 : nullptr, ioff + n1, info, info_off + n1, w,
               thr, nopiv, s, ctx, cabs + n1);
        if (!nopiv && !ctx.full) laswp_off<T>(n1, A, lda, n1, std::min(m, n), ipiv, ioff, s);
    }
}

template <typename T>
void getrf_panel_ws(i64 m, i64 n, T* A, i64 lda, i64* ipiv, i64* info, double thr, bool nopiv,
                    void* work, hipStream_t s) {
    void* w = work;
    if (info) HIP_CHECK(hipMemsetAsync(info, 0, sizeof(i64), s));
    if (m <= 0 || n <= 0) return;
    const i64 k = std::min(m, n);
    // SLATE_AMD_LU_PERSIST=0 disables the persistent base case (diagnostics)
    static const bool persist_env = [] { const char* e = std::getenv("SLATE_AMD_LU_PERSIST"); return !e || e[0] != '0'; }();
    const PanelCtx ctx{n, persist_env && persist_ok<T>(m, nopiv), 0};
    if (ctx.full) {
        PersistBuf* pb = reinterpret_cast<PersistBuf*>(static_cast<char*>(w) + PANEL_BYTES);
        HIP_CHECK(hipMemsetAsync(pb->lw, 0, sizeof(pb->lw), s));
    }
    rec<T>(m, k, A, lda, ipiv, 0, info, 0, w, thr, nopiv, s, ctx, 0);
    if (n > k) {   // wide panel: U12 = L11^{-1} P A12
        if (!nopiv && !ctx.full) laswp_off<T>(n - k, A + k * lda, lda, 0, k, ipiv, 0, s);
        trsm<T>('L', 'L', 'N', 'U', k, n - k, s_from_real(T(), 1), A, lda, A + k * lda, lda, s);
    }
}

// tools: enable (1) / disable (0) the per-phase clocks of the persistent
// base case and read the totals accumulated so far (then reset them)
void lu_persist_profile(int enable, unsigned long long* out) {
    unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (out) HIP_CHECK(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_lu_prof), sizeof(z)));
    HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_lu_prof), z, sizeof(z)));
    HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_lu_prof_on), &enable, sizeof(int)));
}

size_t getrf_work_bytes() { return PANEL_BYTES + sizeof(PersistBuf) + sizeof(TagBuf); }

// failure handling of the persistent base case (tests/tools): number of
// launches that fell back to the one-workgroup LU; force = 1 makes every
// following launch take the abort path
unsigned long long lu_persist_fallbacks(int force) {
    unsigned long long v = 0;
    HIP_CHECK(hipMemcpyFromSymbol(&v, HIP_SYMBOL(g_lu_fallbacks), sizeof(v)));
    if (force >= 0) HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_lu_force_abort), &force, sizeof(int)));
    return v;
}

#define INST(T) \
    template void getrf_panel_ws<T>(i64, i64, T*, i64, i64*, i64*, double, bool, void*, hipStream_t);
INST(float) INST(double) INST(ccplx) INST(zcplx)
#undef INST

}  // namespace slate_hip
