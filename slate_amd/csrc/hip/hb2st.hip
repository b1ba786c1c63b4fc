// Hermitian band -> tridiagonal bulge chasing on the GPU (stage 2 of the
// two-stage eigensolver; SLATE runs it on host threads, src/hb2st.cc and
// internal_hebr.cc hebr1/hebr2/hebr3).
//
// Same task graph as the host pipeline (csrc/host/eig.cpp hb2st_mt): task t
// of sweep j generates the Householder reflector that annihilates column
// `col` below row s = e_prev + 1 and applies it two-sidedly over the window
// [col + 1, e + b]; sweep j may run task t once sweep j-1 has completed
// min(t + D, all) tasks, which keeps every pair of overlapping tasks in the
// sequential order (the result equals the sequential chase up to the
// floating-point summation order inside a task).
//
// MI355X mapping: one persistent workgroup (256 threads) per concurrently
// chased sweep.  Workgroups take sweeps in increasing order from an atomic
// ticket, so a workgroup only ever waits on a sweep taken earlier by a
// running workgroup: no co-residency assumption, no deadlock.  The
// dependency is a per-sweep progress counter published with an agent-scope
// release and polled with an agent-scope acquire (cross-XCD visible).
// Inside a task: the reflector by one wave (lanes over the k <= b rows),
// the left update one wave per column (lanes over rows: coalesced), the
// right update one thread per row.  The matrix is a dense n x n
// column-major copy holding both triangles (only the band is non-zero).
#include <algorithm>
#include <cstdlib>
#include <cstring>

#include "common.hpp"
#include "kernels.hpp"

namespace slate_hip {

namespace {
constexpr int HMAXB = 128;
// bytes of the LDS staging buffer: SLATE_AMD_HB2ST_LDS (KB, 32..152),
// default 128: the 3b-wide window of b = 64 is one chunk (96 KB: two)
inline i64 hb_lds_bytes() {
    static const i64 v = [] {
        const char* e = std::getenv("SLATE_AMD_HB2ST_LDS");
        const i64 kb = e ? std::atoll(e) : 128;
        return std::min<i64>(152, std::max<i64>(32, kb)) * 1024;
    }();
    return v;
}
}

__global__ void hb_copy_tail(const unsigned* __restrict__ src, unsigned* __restrict__ dst) { *dst = *src; }

// Working-copy transfers by KERNEL, not hipMemcpyAsync: a copy-engine write
// into A is not seen by a later kernel that still holds A's old lines in an
// XCD's L2 (the band buffer is typically a reused cached block; its pre-chase
// contents were read back instead of the chased band -- native heev probe,
// profiles/r6).  A kernel's stores take the normal write-back path.
__global__ void __launch_bounds__(256)
hb_copy_words(const unsigned long long* __restrict__ src, unsigned long long* __restrict__ dst, size_t nw) {
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < nw; i += (size_t)gridDim.x * 256) dst[i] = src[i];
}
inline void hb_copy(void* dst, const void* src, size_t bytes, hipStream_t s) {
    const size_t nw = bytes / 8;            // element sizes 4 / 8 / 16: pad odd fp32 counts below
    if (nw) {
        const unsigned g = (unsigned)std::min<size_t>((nw + 255) / 256, 8192);
        hipLaunchKernelGGL(hb_copy_words, dim3(g), dim3(256), 0, s, static_cast<const unsigned long long*>(src),
                           static_cast<unsigned long long*>(dst), nw);
    }
    if (bytes % 8)                          // one trailing 4-byte word (fp32, odd count)
        hipLaunchKernelGGL(hb_copy_tail, dim3(1), dim3(1), 0, s, static_cast<const unsigned*>(src) + 2 * nw,
                           static_cast<unsigned*>(dst) + 2 * nw);
    HIP_LAUNCH_CHECK();
}

// 2-D block moves between global memory and LDS: lanes run along the rows
// (coalesced), waves along the columns; the (row group, column) pair index
// is wave-uniform, so the index arithmetic stays on the scalar unit, and U
// global loads are in flight before the LDS writes (a plain loop waits for
// each load in turn: the window then streams at a few GB/s).
template <int U, int NW, typename F>
__device__ inline void for_pairs(int nrow, int ncol, int lane, int w, F&& body) {
    const int npr = (nrow + 63) >> 6;                     // row groups of 64
    const int ncw = (ncol - w + NW - 1) / NW;              // this wave's columns
    const int tot = ncw * npr;
    for (int base = 0; base < tot; base += U) body(base, npr, min(U, tot - base));
    (void)lane;
}

template <typename T, int NW, typename Src, typename Dst>
__device__ inline void move2d(int nrow, int ncol, int lane, int w, Src src, Dst dst) {
    constexpr int U = 12;
    for_pairs<U, NW>(nrow, ncol, lane, w, [&](int base, int npr, int cnt) {
        T tmp[U];
        #pragma unroll
        for (int u = 0; u < U; ++u) {
            if (u < cnt) {
                const int p = base + u, c = w + NW * (p / npr), r = lane + 64 * (p % npr);
                if (r < nrow) tmp[u] = src(r, c);
            }
        }
        #pragma unroll
        for (int u = 0; u < U; ++u) {
            if (u < cnt) {
                const int p = base + u, c = w + NW * (p / npr), r = lane + 64 * (p % npr);
                if (r < nrow) dst(r, c) = tmp[u];
            }
        }
    });
}

// xor shuffle inside a quad of lanes (any scalar type)
template <typename T>
__device__ inline T quad_xor(T v, int m) {
    if constexpr (scalar_traits<T>::is_complex) return T{__shfl_xor(v.re, m, 64), __shfl_xor(v.im, m, 64)};
    else return __shfl_xor(v, m, 64);
}

template <typename T, int HT>
__global__ void __launch_bounds__(HT)
hb2st_kernel(i64 n, int b, T* __restrict__ A, i64 lda, T* __restrict__ V, T* __restrict__ tauv,
             i64* __restrict__ rowv, i64* __restrict__ lenv, const i64* __restrict__ sweep_ptr,
             const i64* __restrict__ ntask, int* ticket, int* done, i64 nsw, int D, i64* prof, i64 HLDS,
             int fused) {
    using R = typename scalar_traits<T>::real;
    __shared__ T v[HMAXB];
    extern __shared__ unsigned char hb_smem[];
    T* L = reinterpret_cast<T*>(hb_smem);           // staging buffer, HLDS bytes
    __shared__ T s_tau;
    __shared__ R s_beta;
    __shared__ int s_j;
    const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform (SGPR): w-derived branches stay scalar
    auto At = [&](i64 r, i64 c) -> T& { return A[r + c * lda]; };
    // optional per-phase shader-clock totals (prof != nullptr: tools only)
    i64 ph[5] = {0, 0, 0, 0, 0};
    i64 tl = clock64();
#define HSTAMP(i) do { if (prof && tid == 0) { const i64 t_ = clock64(); ph[i] += t_ - tl; tl = t_; } } while (0)
    for (;;) {
        if (tid == 0) s_j = atomicAdd(ticket, 1);
        __syncthreads();
        const i64 j = s_j;
        __syncthreads();
        if (j >= nsw) {
            if (prof && tid == 0)
                for (int i = 0; i < 5; ++i) atomicAdd(reinterpret_cast<unsigned long long*>(prof + i),
                                                      (unsigned long long)ph[i]);
            return;
        }
        const i64 nt = ntask[j];
        i64 s = j + 1, e = min(j + (i64)b, n - 1), col = j;
        // sweep-resident window (fused & 16): the previous task's final row
        // block is still in L; this task takes its reflector column and the
        // first d0 = k_prev - 1 columns of its row block from there (the
        // conjugate transpose of the previous block's columns s..e), and
        // loads only its diagonal block and the bulge columns.  The previous
        // task's stores are then drained just before this task's early
        // publication instead of at its own end.
        bool prev_ok = false;
        i64 p_lo = 0;
        int p_k = 0, p_KPf = 0;
        for (i64 t = 0; t < nt; ++t) {
            if (j > 0) {
                // early mode (fused & 8): done[j-1] = u + 1 says sweep j-1
                // finished tasks < u and PUBLISHED task u's annihilated
                // entries (see below); task t needs tasks <= t+1 finished and
                // task t+2 published (all tasks if sweep j-1 has no t+2)
                const i64 ntp = ntask[j - 1];
                const i64 need = (fused & 8) ? (ntp == 0 ? 0 : (t + 2 < ntp ? t + 3 : ntp + 1))
                                             : min(t + (i64)D, ntp);
                // poll with relaxed loads (an acquire per poll would invalidate
                // the XCD's L2 every time, thrashing the working sweeps), then
                // ONE acquire fence
                if (tid == 0)
                    while (__hip_atomic_load(&done[j - 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < need)
                        __builtin_amdgcn_s_sleep(2);
                __syncthreads();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");   // every wave sees the producer's writes
            }
            HSTAMP(0);
            if (t > 0) { s = e + 1; e = min(e + (i64)b, n - 1); }
            const int k = (int)(e - s + 1);
            const i64 lo = col + 1, hi = min(n - 1, e + (i64)b);
            // LDS pitch of the staged row block: the next value = 4 (mod 32)
            // doubles >= k + 1, so the left update's (column, quad-lane) pairs
            // of a half-wave hit 32 distinct bank pairs (the odd pitch k + 1,
            // SLATE_AMD_HB2ST_PITCH=odd, collides col + q: ~3-way; PMC 55.6 %
            // bank-conflict cycles; dsyevd n = 16384: 4.01 -> 3.88 s)
            const int KPf = ((fused & 2) && sizeof(T) == 8) ? (k + 1) + (((4 - (k + 1)) % 32) + 32) % 32 : k + 1;
            const bool one_chunk = fused && (hi - lo + 1) <= min<i64>(HT, HLDS / ((i64)KPf * (i64)sizeof(T)));
            const bool fuse = one_chunk && (fused & 1);
            // fused path: the row block A(s..e, lo..hi) does not depend on the
            // reflector, so its load is issued BEFORE wave 0 loads the column
            // -- one memory round trip per task instead of two in sequence
            // (a task whose reflector turns out trivial just drops it)
            // wave 0 issues its column loads (k <= 128 rows: two per lane)
            // before its share of the row block, so both are in flight at once
            T xc[HMAXB / 64];
            const bool reuse = (fused & 16) && fuse && prev_ok && b <= 64 && k <= 64 && p_k <= 64;
            const int nc = (int)(hi - lo + 1);
            if (reuse) {
                constexpr int NBR = (64 * 64 + HT - 1) / HT;
                const int cb = (int)(s - p_lo), d0 = p_k - 1;    // d0 = s - lo
                if (w == 0) {
                    #pragma unroll
                    for (int u = 0; u < HMAXB / 64; ++u) {
                        const int r = lane + 64 * u;
                        xc[u] = (r < k) ? s_conj(L[(cb + r) * p_KPf]) : s_zero(T());
                    }
                }
                T br[NBR];
                #pragma unroll
                for (int q = 0; q < NBR; ++q) {
                    const int idx = tid + q * HT, r = 1 + idx / k, cc = idx % k;
                    br[q] = (r < p_k) ? L[(cb + cc) * p_KPf + r] : s_zero(T());
                }
                __syncthreads();                                   // every read of the previous block done
                #pragma unroll
                for (int q = 0; q < NBR; ++q) {
                    const int idx = tid + q * HT, r = 1 + idx / k, cc = idx % k;
                    if (r < p_k) L[(r - 1) * KPf + cc] = s_conj(br[q]);   // A(s + cc, lo + r - 1)
                }
                T* Ab = &At(s, lo + d0);
                move2d<T, HT / 64>(k, nc - d0, lane, w, [&](int r, int c) -> T { return Ab[r + c * lda]; },
                                   [&](int r, int c) -> T& { return L[(c + d0) * KPf + r]; });
            } else {
                if (w == 0) {
                    #pragma unroll
                    for (int u = 0; u < HMAXB / 64; ++u) {
                        const int r = lane + 64 * u;
                        xc[u] = (r < k) ? At(s + r, col) : s_zero(T());
                    }
                }
                if (fuse) {
                    T* Ab = &At(s, lo);
                    move2d<T, HT / 64>(k, nc, lane, w, [&](int r, int c) -> T { return Ab[r + c * lda]; },
                                       [&](int r, int c) -> T& { return L[c * KPf + r]; });
                }
            }
            // ---- reflector (wave 0): x = A(s..e, col)
            if (w == 0) {
                T x0 = s_zero(T());
                R xn2 = 0;
                for (int r = lane; r < k; r += 64) {
                    const T x = xc[r >> 6];
                    v[r] = x;
                    if (r == 0) x0 = x;
                    else xn2 += s_real(s_mul(s_conj(x), x));
                }
                xn2 = wave_sum(xn2);
                x0 = wave_sum(x0);                              // only lane 0 contributed
                const R ar = s_real(x0);
                R ai = 0;
                if constexpr (scalar_traits<T>::is_complex) ai = x0.im;
                T tau;
                R beta;
                bool trivial = (xn2 == R(0) && ai == R(0));
                if (trivial) {
                    tau = s_zero(T());
                    beta = ar;
                } else {
                    beta = -copysign(sqrt(ar * ar + ai * ai + xn2), ar);
                    if constexpr (scalar_traits<T>::is_complex) tau = T{(beta - ar) / beta, -ai / beta};
                    else tau = (beta - ar) / beta;
                }
                // v = x / (alpha - beta), v[0] = 1
                T den = x0;
                if constexpr (scalar_traits<T>::is_complex) den.re -= beta;
                else den -= beta;
                for (int r = lane; r < k; r += 64) {
                    if (r == 0) v[0] = s_from_real(T(), R(1));
                    else if (!trivial) v[r] = s_div(v[r], den);
                }
                if (lane == 0) { s_tau = tau; s_beta = beta; }
            }
            if (fused & 8) {
                // Early publication.  Task (j+1, t-2) -- the one that waits
                // for this task -- shares exactly two entries with it:
                // A(s, col) and A(col, s) (its window is [col' .. s] with
                // col' = col - b + 1; this task writes rows s..e / columns
                // lo = col + 1.. of its row block, their mirror and the
                // column below/right of (s, col)).  So once this column is
                // read and those two entries hold beta, the next sweep may
                // go.  Every wave first drains its stores (the previous
                // task's, deferred) -- a barrier alone does not.
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __syncthreads();
                if (tid == 0) {
                    At(s, col) = s_from_real(T(), s_beta);
                    At(col, s) = s_from_real(T(), s_beta);
                    __hip_atomic_store(&done[j], (int)(t + 1), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
                }
            } else {
                __syncthreads();
            }
            HSTAMP(1);
            const T tau = s_tau;
            if (!s_is_zero(tau) && fuse) {
                // ---- fused two-sided update (A Hermitian, both triangles):
                // ONE load of the row block A(s..e, lo..hi); left update
                // H^H A on it; the right update A H only changes columns
                // s..e, i.e. inside the block just the k x k diagonal block
                // (a thread per row); the rest of A' = H^H A H in columns
                // s..e is the conjugate transpose of the row block (A' is
                // Hermitian), stored as the mirror of its off-diagonal part.
                const T ct = s_conj(tau);
                const int d0 = (int)(s - lo);
                T* Ab = &At(s, lo);
                // (the row block was staged before the reflector; the
                // barrier after the reflector covers its LDS writes)
                // left: four lanes per column (rows q, q + 4, ...), partial
                // dot products combined by two xor shuffles inside the quad
                for (int e = tid; e < 4 * nc; e += HT) {
                    T* Lc = L + (e >> 2) * KPf;
                    const int q = e & 3;
                    T p0 = s_zero(T()), p1 = s_zero(T());
                    int r = q;
                    for (; r + 4 < k; r += 8) {
                        p0 = s_add(p0, s_mul(s_conj(v[r]), Lc[r]));
                        p1 = s_add(p1, s_mul(s_conj(v[r + 4]), Lc[r + 4]));
                    }
                    if (r < k) p0 = s_add(p0, s_mul(s_conj(v[r]), Lc[r]));
                    T acc = s_add(p0, p1);
                    acc = s_add(acc, quad_xor(acc, 1));
                    acc = s_add(acc, quad_xor(acc, 2));
                    acc = s_mul(ct, acc);
                    for (r = q; r < k; r += 4) Lc[r] = s_sub(Lc[r], s_mul(v[r], acc));
                }
                __syncthreads();
                HSTAMP(2);
                // right on the diagonal block: four lanes per row
                for (int e = tid; e < 4 * k; e += HT) {
                    T* Ld = L + (i64)d0 * KPf + (e >> 2);   // row e/4 of the diagonal block
                    const int q = e & 3;
                    T p0 = s_zero(T()), p1 = s_zero(T());
                    int c = q;
                    for (; c + 4 < k; c += 8) {
                        p0 = s_add(p0, s_mul(Ld[c * KPf], v[c]));
                        p1 = s_add(p1, s_mul(Ld[(c + 4) * KPf], v[c + 4]));
                    }
                    if (c < k) p0 = s_add(p0, s_mul(Ld[c * KPf], v[c]));
                    T y = s_add(p0, p1);
                    y = s_add(y, quad_xor(y, 1));
                    y = s_add(y, quad_xor(y, 2));
                    y = s_mul(y, tau);
                    for (c = q; c < k; c += 4) Ld[c * KPf] = s_sub(Ld[c * KPf], s_mul(y, s_conj(v[c])));
                }
                __syncthreads();
                move2d<T, HT / 64>(k, nc, lane, w, [&](int r, int c) -> T { return L[c * KPf + r]; },
                                   [&](int r, int c) -> T& { return Ab[r + c * lda]; });
                // mirror: A(lo + q, s + r) = conj(A'(s + r, lo + q)) for the rows
                // q outside the diagonal block (above it, then below it)
                move2d<T, HT / 64>(d0, k, lane, w, [&](int q, int r) -> T { return s_conj(L[q * KPf + r]); },
                                   [&](int q, int r) -> T& { return At(lo + q, s + r); });
                const int nb2 = nc - d0 - k;
                move2d<T, HT / 64>(nb2, k, lane, w,
                                   [&](int q, int r) -> T { return s_conj(L[(d0 + k + q) * KPf + r]); },
                                   [&](int q, int r) -> T& { return At(e + 1 + q, s + r); });
                __syncthreads();
            } else if (!s_is_zero(tau)) {
                // ---- left: A(s..e, c) -= v (conj(tau) v^H A(s..e, c)), c in [lo, hi].
                // Column chunks staged in LDS (one bulk coalesced load: every
                // load in flight at once), a wave per column, bulk store.
                const T ct = s_conj(tau);
                // thread per column over LDS columns padded to k + 1 (no
                // per-column wave reductions: a shuffle tree per column is a
                // chain of LDS-crossbar round trips)
                const int KP = k + 1;
                const i64 cw = max<i64>(1, min<i64>(min<i64>(hi - lo + 1, HT),
                                                   HLDS / ((i64)KP * (i64)sizeof(T))));
                for (i64 c0 = lo; c0 <= hi; c0 += cw) {
                    const int nc = (int)min<i64>(cw, hi - c0 + 1);
                    T* Ab = &At(s, c0);
                    move2d<T, HT / 64>(k, nc, lane, w, [&](int r, int c) -> T { return Ab[r + c * lda]; },
                              [&](int r, int c) -> T& { return L[c * KP + r]; });
                    __syncthreads();
                    if (tid < nc) {
                        // unrolled by 8 with independent partial sums: the LDS
                        // reads of a group are in flight together
                        T* Lc = L + tid * KP;
                        T part[8];
                        #pragma unroll
                        for (int u = 0; u < 8; ++u) part[u] = s_zero(T());
                        int r = 0;
                        for (; r + 8 <= k; r += 8) {
                            #pragma unroll
                            for (int u = 0; u < 8; ++u) part[u] = s_add(part[u], s_mul(s_conj(v[r + u]), Lc[r + u]));
                        }
                        for (; r < k; ++r) part[0] = s_add(part[0], s_mul(s_conj(v[r]), Lc[r]));
                        T acc = s_zero(T());
                        #pragma unroll
                        for (int u = 0; u < 8; ++u) acc = s_add(acc, part[u]);
                        acc = s_mul(ct, acc);
                        r = 0;
                        for (; r + 8 <= k; r += 8) {
                            #pragma unroll
                            for (int u = 0; u < 8; ++u) Lc[r + u] = s_sub(Lc[r + u], s_mul(v[r + u], acc));
                        }
                        for (; r < k; ++r) Lc[r] = s_sub(Lc[r], s_mul(v[r], acc));
                    }
                    __syncthreads();
                    move2d<T, HT / 64>(k, nc, lane, w, [&](int r, int c) -> T { return L[c * KP + r]; },
                              [&](int r, int c) -> T& { return Ab[r + c * lda]; });
                    __syncthreads();
                }
                HSTAMP(2);
                // ---- right: A(r, s..e) -= (tau A(r, s..e) v) v^H, r in [lo, hi]:
                // row chunks staged in LDS ([c][r]: a thread per row reads
                // consecutive banks)
                const i64 rw = max<i64>(1, min<i64>(hi - lo + 1, min<i64>(HT, HLDS / ((i64)k * (i64)sizeof(T)))));
                for (i64 r0 = lo; r0 <= hi; r0 += rw) {
                    const int nr = (int)min<i64>(rw, hi - r0 + 1);
                    T* Ab = &At(r0, s);
                    move2d<T, HT / 64>(nr, k, lane, w, [&](int r, int c) -> T { return Ab[r + c * lda]; },
                              [&](int r, int c) -> T& { return L[c * nr + r]; });
                    __syncthreads();
                    if (tid < nr) {
                        T part[8];
                        #pragma unroll
                        for (int u = 0; u < 8; ++u) part[u] = s_zero(T());
                        int c = 0;
                        for (; c + 8 <= k; c += 8) {
                            #pragma unroll
                            for (int u = 0; u < 8; ++u) part[u] = s_add(part[u], s_mul(L[(c + u) * nr + tid], v[c + u]));
                        }
                        for (; c < k; ++c) part[0] = s_add(part[0], s_mul(L[c * nr + tid], v[c]));
                        T y = s_zero(T());
                        #pragma unroll
                        for (int u = 0; u < 8; ++u) y = s_add(y, part[u]);
                        y = s_mul(y, tau);
                        c = 0;
                        for (; c + 8 <= k; c += 8) {
                            #pragma unroll
                            for (int u = 0; u < 8; ++u)
                                L[(c + u) * nr + tid] = s_sub(L[(c + u) * nr + tid], s_mul(y, s_conj(v[c + u])));
                        }
                        for (; c < k; ++c) L[c * nr + tid] = s_sub(L[c * nr + tid], s_mul(y, s_conj(v[c])));
                    }
                    __syncthreads();
                    move2d<T, HT / 64>(nr, k, lane, w, [&](int r, int c) -> T { return L[c * nr + r]; },
                              [&](int r, int c) -> T& { return Ab[r + c * lda]; });
                    __syncthreads();
                }
            }
            __syncthreads();
            HSTAMP(3);
            // ---- annihilated column / row, reflector slot
            const R beta = s_beta;
            const i64 slot = sweep_ptr[j] + t;
            // (early mode: (s, col) was stored at publication and may since
            // have been updated by sweep j+1 -- not rewritten)
            for (int r = ((fused & 8) ? 1 : 0) + tid; r < k; r += HT) {
                const T val = (r == 0) ? s_from_real(T(), beta) : s_zero(T());
                At(s + r, col) = val;
                At(col, s + r) = val;
            }
            for (int r = tid; r < b; r += HT) V[slot * b + r] = (r < k) ? v[r] : s_zero(T());
            if (tid == 0) { tauv[slot] = tau; rowv[slot] = s; lenv[slot] = k; }
            const bool publish = !(fused & 8) || t + 1 == nt;
            // the next task of this sweep reads back what this one stored
            // unless it takes it from L; early mode drains at the next
            // publication (or here, at the sweep's last task)
            if (publish || !(fused & 16) || !fuse) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (tid == 0 && publish)                             // one release: writes back this XCD's L2
                __hip_atomic_store(&done[j], (int)((fused & 8) ? nt + 1 : t + 1), __ATOMIC_RELEASE,
                                   __HIP_MEMORY_SCOPE_AGENT);
            HSTAMP(4);
            prev_ok = fuse;
            p_lo = lo; p_k = k; p_KPf = KPf;
            col = s;
        }
    }
}

template <typename T>
void hb2st_device(i64 n, int b, T* A, i64 lda, T* V, T* tau, i64* row, i64* len, const i64* sweep_ptr,
                  const i64* ntask, int* work, i64 nsw, int nwg, hipStream_t s, i64* prof, i64 extent) {
    if (nsw <= 0) return;
    if (b > HMAXB) throw std::invalid_argument("hb2st_device: bandwidth > 128");
    // work = [ticket, done[0..nsw)] zero-initialised by the caller
    // The chase hands windows between workgroups on different XCDs: with
    // the default (L2-cached, non-coherent across XCDs) memory every hand-off
    // writes back and invalidates a whole L2.  SLATE_AMD_HB2ST_MEM=uncached
    // (default) or finegrained runs on a coherent working copy instead.
    static const int mode = [] {
        const char* e = getenv("SLATE_AMD_HB2ST_MEM");
        if (!e || !strcmp(e, "uncached")) return 2;
        return strcmp(e, "finegrained") == 0 ? 1 : 0;
    }();
    T* W = A;
    const size_t bytes = sizeof(T) * (extent > 0 ? (size_t)extent : (size_t)lda * (size_t)n);
    if (mode) {
        HIP_CHECK(hipExtMallocWithFlags(reinterpret_cast<void**>(&W), bytes,
                                        mode == 2 ? hipDeviceMallocUncached : hipDeviceMallocFinegrained));
        hb_copy(W, A, bytes, s);
    }
    // threads per workgroup: the task's window moves are latency bound (loads
    // in flight per workgroup), SLATE_AMD_HB2ST_THREADS = 256 | 512 | 1024;
    // dsyevd n = 16384, b = 64: chase 3.93 / 2.78 / 2.61 s
    static const int threads = [] {
        const char* e = getenv("SLATE_AMD_HB2ST_THREADS");
        const int v = e ? atoi(e) : 1024;
        return (v == 256 || v == 512) ? v : 1024;
    }();
    auto launch = [&](auto kern, int ht) {
        const i64 HLDS = hb_lds_bytes();
        // SLATE_AMD_HB2ST_FUSED=0: separate left / right passes (4 window moves per task instead of 3)
        const int fused = [] {
            const char* e = getenv("SLATE_AMD_HB2ST_FUSED");
            const char* pt = getenv("SLATE_AMD_HB2ST_PITCH");
            const char* ea = getenv("SLATE_AMD_HB2ST_EARLY");
            const char* ru = getenv("SLATE_AMD_HB2ST_REUSE");
            const int early = (ea && ea[0] == '0') ? 0 : 8;                           // early publication
            return ((e && e[0] == '0') ? 0 : 1) | ((pt && pt[0] == 'o') ? 0 : 2) |  // default: 4 (mod 32)
                   early | ((early && !(ru && ru[0] == '0')) ? 16 : 0);              // sweep-resident window
        }();
        HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)HLDS));
        // lag: sweep j runs task t once sweep j-1 finished t + lag tasks.
        // Task t of sweep j touches rows/columns [j+1+(t-1)b, j+(t+2)b]; task
        // t' of sweep j-1 touches [j+(t'-1)b, j-1+(t'+2)b]: they share
        // indices only for t' <= t + 3, and at t' = t + 3 only index
        // j+(t+2)b, which the two tasks use in disjoint rows / columns
        // (sweep j: rows s..e <= j+(t+1)b of column hi and their mirror;
        // sweep j-1: rows >= j+(t+3)b of its column col' = hi) -- so lag 3
        // keeps the sequential order (SLATE_AMD_HB2ST_LAG, default 3; 4 was
        // the conservative choice of round 2)
        const int lag = [] {
            const char* e = getenv("SLATE_AMD_HB2ST_LAG");
            const int v = e ? atoi(e) : 3;
            return v < 3 ? 3 : v;
        }();
        hipLaunchKernelGGL(kern, dim3((unsigned)nwg), dim3(ht), HLDS, s, n, b, W, lda, V, tau, row, len,
                           sweep_ptr, ntask, work, work + 1, nsw, lag, prof, HLDS, fused);
    };
    if (threads == 1024) launch(hb2st_kernel<T, 1024>, 1024);
    else if (threads == 512) launch(hb2st_kernel<T, 512>, 512);
    else launch(hb2st_kernel<T, 256>, 256);
    HIP_LAUNCH_CHECK();
    if (mode) {
        hb_copy(A, W, bytes, s);
        HIP_CHECK(hipStreamSynchronize(s));
        HIP_CHECK(hipFree(W));
    }
}

// ---------------------------------------------------------------- tb2bd
// Upper band -> upper bidiagonal (SVD stage 2; SLATE src/tb2bd.cc with
// internal_gebr.cc gebr1/2/3 on host threads).  Same task graph as the
// host pipeline (csrc/host/eig.cpp tb2bd_mt): task t of sweep j generates
// the right reflector that annihilates row `row` beyond column cs and
// applies it to the rows of columns cs..ce, then the left reflector that
// annihilates column cs below the diagonal and applies it to the columns
// of rows cs..re.  Sweep j runs task t once sweep j-1 has completed
// min(t + 4, all) tasks (see tb2bd_device).  The windows are the exact non-zero extents:
// columns cs..ce hold rows [row, ce] (band + the fill of the previous left
// reflector), rows cs..re hold columns [cs, re + b].
template <typename T, int HT>
__global__ void __launch_bounds__(HT)
tb2bd_kernel(i64 n, int b, T* __restrict__ A, i64 lda, T* __restrict__ UV, T* __restrict__ Utau,
             i64* __restrict__ Urow, i64* __restrict__ Ulen, T* __restrict__ VV, T* __restrict__ Vtau,
             i64* __restrict__ Vrow, i64* __restrict__ Vlen, const i64* __restrict__ sweep_ptr,
             const i64* __restrict__ ntask, int* ticket, int* done, i64 nsw, int D, i64 HLDS) {
    using R = typename scalar_traits<T>::real;
    __shared__ T v[HMAXB];
    extern __shared__ unsigned char hb_smem[];
    T* L = reinterpret_cast<T*>(hb_smem);
    __shared__ T s_tau;
    __shared__ R s_beta;
    __shared__ int s_j;
    const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform (SGPR): w-derived branches stay scalar
    auto At = [&](i64 r, i64 c) -> T& { return A[r + c * lda]; };
    // Householder generator on v[0..k) (wave 0): v <- v / (v0 - beta), v0 = 1
    auto hgen = [&](int k) {
        T x0 = s_zero(T());
        R xn2 = 0;
        for (int r = lane; r < k; r += 64) {
            const T x = v[r];
            if (r == 0) x0 = x;
            else xn2 += s_real(s_mul(s_conj(x), x));
        }
        xn2 = wave_sum(xn2);
        x0 = wave_sum(x0);
        const R ar = s_real(x0);
        R ai = 0;
        if constexpr (scalar_traits<T>::is_complex) ai = x0.im;
        T tau;
        R beta;
        const bool trivial = (xn2 == R(0) && ai == R(0));
        if (trivial) {
            tau = s_zero(T());
            beta = ar;
        } else {
            beta = -copysign(sqrt(ar * ar + ai * ai + xn2), ar);
            if constexpr (scalar_traits<T>::is_complex) tau = T{(beta - ar) / beta, -ai / beta};
            else tau = (beta - ar) / beta;
        }
        T den = x0;
        if constexpr (scalar_traits<T>::is_complex) den.re -= beta;
        else den -= beta;
        for (int r = lane; r < k; r += 64) {
            if (r == 0) v[0] = s_from_real(T(), R(1));
            else if (!trivial) v[r] = s_div(v[r], den);
        }
        if (lane == 0) { s_tau = tau; s_beta = beta; }
    };
    for (;;) {
        if (tid == 0) s_j = atomicAdd(ticket, 1);
        __syncthreads();
        const i64 j = s_j;
        __syncthreads();
        if (j >= nsw) return;
        const i64 nt = ntask[j];
        i64 cs = j + 1, ce = min(j + (i64)b, n - 1), row = j;
        for (i64 t = 0; t < nt; ++t) {
            if (j > 0) {
                const i64 need = min(t + (i64)D, ntask[j - 1]);
                if (tid == 0)
                    while (__hip_atomic_load(&done[j - 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < need)
                        __builtin_amdgcn_s_sleep(2);
                __syncthreads();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            }
            if (t > 0) { cs = ce + 1; ce = min(cs + (i64)b - 1, n - 1); }
            const int k = (int)(ce - cs + 1);
            const i64 slot = sweep_ptr[j] + t;
            // ---- right reflector: x = conj(A(row, cs..ce))
            if (w == 0) {
                for (int c = lane; c < k; c += 64) v[c] = s_conj(At(row, cs + c));
                hgen(k);
            }
            __syncthreads();
            {
                const T tau = s_tau;
                const i64 lo = row, hi = ce;                 // rows holding columns cs..ce
                if (!s_is_zero(tau)) {
                    // A(r, cs..ce) -= (tau A(r, cs..ce) v) v^H, a thread per row
                    const i64 rw = max<i64>(1, min<i64>(hi - lo + 1, min<i64>(HT, HLDS / ((i64)k * (i64)sizeof(T)))));
                    for (i64 r0 = lo; r0 <= hi; r0 += rw) {
                        const int nr = (int)min<i64>(rw, hi - r0 + 1);
                        T* Ab = &At(r0, cs);
                        move2d<T, HT / 64>(nr, k, lane, w, [&](int r, int c) -> T { return Ab[r + c * lda]; },
                                           [&](int r, int c) -> T& { return L[c * nr + r]; });
                        __syncthreads();
                        // four lanes per row (columns q, q + 4, ...), quad reductions
                        for (int e = tid; e < 4 * nr; e += HT) {
                            const int rr = e >> 2, q = e & 3;
                            T y = s_zero(T());
                            for (int c = q; c < k; c += 4) y = s_add(y, s_mul(L[c * nr + rr], v[c]));
                            y = s_add(y, quad_xor(y, 1));
                            y = s_add(y, quad_xor(y, 2));
                            y = s_mul(y, tau);
                            for (int c = q; c < k; c += 4)
                                L[c * nr + rr] = s_sub(L[c * nr + rr], s_mul(y, s_conj(v[c])));
                        }
                        __syncthreads();
                        move2d<T, HT / 64>(nr, k, lane, w, [&](int r, int c) -> T { return L[c * nr + r]; },
                                           [&](int r, int c) -> T& { return Ab[r + c * lda]; });
                        __syncthreads();
                    }
                }
                for (int c = tid; c < k; c += HT) At(row, cs + c) = c == 0 ? s_from_real(T(), s_beta) : s_zero(T());
                for (int c = tid; c < b; c += HT) VV[slot * b + c] = c < k ? v[c] : s_zero(T());
                if (tid == 0) { Vtau[slot] = tau; Vrow[slot] = cs; Vlen[slot] = k; }
            }
            __syncthreads();
            // ---- left reflector: x = A(cs..re, cs)
            const i64 rs = cs, re = min(min(cs + (i64)b - 1, n - 1), ce);
            const int kr = (int)(re - rs + 1);
            if (w == 0) {
                for (int r = lane; r < kr; r += 64) v[r] = At(rs + r, cs);
                hgen(kr);
            }
            __syncthreads();
            {
                const T tau = s_tau;
                const i64 lo = cs, hi = min(n - 1, re + (i64)b);   // columns holding rows rs..re
                if (!s_is_zero(tau)) {
                    const T ct = s_conj(tau);
                    const int KP = kr + 1;
                    const i64 cw = max<i64>(1, min<i64>(min<i64>(hi - lo + 1, HT), HLDS / ((i64)KP * (i64)sizeof(T))));
                    for (i64 c0 = lo; c0 <= hi; c0 += cw) {
                        const int nc = (int)min<i64>(cw, hi - c0 + 1);
                        T* Ab = &At(rs, c0);
                        move2d<T, HT / 64>(kr, nc, lane, w, [&](int r, int c) -> T { return Ab[r + c * lda]; },
                                           [&](int r, int c) -> T& { return L[c * KP + r]; });
                        __syncthreads();
                        // four lanes per column (rows q, q + 4, ...), quad reductions
                        for (int e = tid; e < 4 * nc; e += HT) {
                            T* Lc = L + (e >> 2) * KP;
                            const int q = e & 3;
                            T acc = s_zero(T());
                            for (int r = q; r < kr; r += 4) acc = s_add(acc, s_mul(s_conj(v[r]), Lc[r]));
                            acc = s_add(acc, quad_xor(acc, 1));
                            acc = s_add(acc, quad_xor(acc, 2));
                            acc = s_mul(ct, acc);
                            for (int r = q; r < kr; r += 4) Lc[r] = s_sub(Lc[r], s_mul(v[r], acc));
                        }
                        __syncthreads();
                        move2d<T, HT / 64>(kr, nc, lane, w, [&](int r, int c) -> T { return L[c * KP + r]; },
                                           [&](int r, int c) -> T& { return Ab[r + c * lda]; });
                        __syncthreads();
                    }
                }
                for (int r = tid; r < kr; r += HT) At(rs + r, cs) = r == 0 ? s_from_real(T(), s_beta) : s_zero(T());
                for (int r = tid; r < b; r += HT) UV[slot * b + r] = r < kr ? v[r] : s_zero(T());
                if (tid == 0) { Utau[slot] = tau; Urow[slot] = rs; Ulen[slot] = kr; }
            }
            row = rs;
            // every wave drains its stores before the flag (a barrier alone
            // waits for LDS traffic only)
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (tid == 0)
                __hip_atomic_store(&done[j], (int)(t + 1), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

template <typename T>
void tb2bd_device(i64 n, int b, T* A, i64 lda, T* UV, T* Utau, i64* Urow, i64* Ulen, T* VV, T* Vtau, i64* Vrow,
                  i64* Vlen, const i64* sweep_ptr, const i64* ntask, int* work, i64 nsw, int nwg, hipStream_t s) {
    if (nsw <= 0) return;
    if (b > HMAXB) throw std::invalid_argument("tb2bd_device: bandwidth > 128");
    // work = [ticket, done[0..nsw)] zero-initialised by the caller; the
    // chase runs on an uncached working copy (cross-XCD hand-offs, as hb2st)
    T* W = nullptr;
    const size_t bytes = sizeof(T) * (size_t)lda * (size_t)n;
    HIP_CHECK(hipExtMallocWithFlags(reinterpret_cast<void**>(&W), bytes, hipDeviceMallocUncached));
    hb_copy(W, A, bytes, s);
    // 1024 threads (the window moves are latency bound, as hb2st); lag 4:
    // with the exact windows task t of sweep j stays inside
    // [j + (t - 1) b + 1, j + (t + 2) b] and sweep j-1's tasks from t + 4 on
    // start at j + (t + 3) b (SLATE_AMD_TB2BD_LAG overrides, >= 4)
    constexpr int HT = 1024;
    static const int lag = [] {
        const char* e = std::getenv("SLATE_AMD_TB2BD_LAG");
        return std::max(4, e ? std::atoi(e) : 4);
    }();
    auto kern = tb2bd_kernel<T, HT>;
    const i64 HLDS = hb_lds_bytes();
    HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)HLDS));
    hipLaunchKernelGGL(kern, dim3((unsigned)nwg), dim3(HT), HLDS, s, n, b, W, lda, UV, Utau, Urow, Ulen, VV, Vtau,
                       Vrow, Vlen, sweep_ptr, ntask, work, work + 1, nsw, lag, HLDS);
    HIP_LAUNCH_CHECK();
    hb_copy(A, W, bytes, s);
    HIP_CHECK(hipStreamSynchronize(s));
    HIP_CHECK(hipFree(W));
}

#define INST(T) \
    template void tb2bd_device<T>(i64, int, T*, i64, T*, T*, i64*, i64*, T*, T*, i64*, i64*, const i64*, \
                                  const i64*, int*, i64, int, hipStream_t);
INST(float) INST(double) INST(ccplx) INST(zcplx)
#undef INST

#define INST(T) \
    template void hb2st_device<T>(i64, int, T*, i64, T*, T*, i64*, i64*, const i64*, const i64*, int*, i64, int, \
                                  hipStream_t, i64*, i64);
INST(float) INST(double) INST(ccplx) INST(zcplx)
#undef INST

}  // namespace slate_hip
