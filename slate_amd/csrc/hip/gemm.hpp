// MFMA GEMM for gfx950:  C = alpha * op(A) * op(B) + beta * C
//
// Real types (float, double) use one v_mfma_{f64,f32}_16x16x4 per 16x16x4
// sub-product; complex types use four real MFMAs per complex product on
// split re/im fragments.  Column-major storage throughout (LAPACK/ScaLAPACK
// convention, SLATE tiles).
//
// Design (MI355X-first, not a port of any vendor kernel):
//  * 256-thread workgroups = 4 waves laid out 2x2 over a BMxBN macro tile;
//    each wave owns a (BM/2)x(BN/2) sub-tile = (BM/32)x(BN/32) MFMA tiles.
//  * operands staged global -> registers -> LDS, double-buffered, one barrier
//    per BK step; next tile's global loads issued before the current MFMAs
//    (guide T14, write-after-compute).
//  * two LDS images per operand depending on the contiguous dimension of the
//    source: "MK" [BK][R+16] for row-contiguous sources (16-element pad puts
//    the k and k+1 rows of one ds_read_b64 half-wave in disjoint bank halves)
//    and "KM" [R][BK+1] for k-contiguous sources (odd pad: conflict-free
//    strided fragment reads).
//  * MFMA operands are swapped (D^T = op(B)^T op(A)^T) so the accumulator's
//    lane index runs along m: epilogue stores are 16 consecutive elements of
//    a column (coalesced for column-major C).
//  * XCD-aware bijective block remap + grouped tile order for L2 reuse.
//  * optional triangular output mask (TriMask) evaluated in global
//    coordinates of a 2D block-cyclic matrix, so herk/syrk trailing updates
//    of a distributed matrix are ONE launch on the rank's local buffer.
#pragma once
#include "common.hpp"

namespace slate_hip {

template <typename T> struct mfma_real;
template <> struct mfma_real<double> {
    using acc_t = d4;
    static constexpr int VEC = 2;  // elements per 16-byte vector
    __device__ static inline acc_t mma(double x, double y, acc_t c) {
        return __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, c, 0, 0, 0);
    }
    // row (within the 16x16 D tile) held by (lane, reg)
    __device__ static inline int drow(int lane, int r) { return (lane >> 4) + 4 * r; }
};
template <> struct mfma_real<float> {
    using acc_t = f4;
    static constexpr int VEC = 4;
    __device__ static inline acc_t mma(float x, float y, acc_t c) {
        return __builtin_amdgcn_mfma_f32_16x16x4f32(x, y, c, 0, 0, 0);
    }
    __device__ static inline int drow(int lane, int r) { return 4 * (lane >> 4) + r; }
};

// remap 4: the kept blocks of a lower-masked output form a staircase (block
// row r keeps block columns [0, ncol[r]), ncol non-decreasing); the grid
// covers only those, in the grouped column-major order
constexpr int GEMM_STAIR_MAX = 512;
constexpr int GEMM_STAIR_GROUPS = 128;   // remap 4: at most this many row groups

template <typename T>
struct GemmArgs {
    i64 m, n, k;
    T alpha, beta;
    const T* A; i64 lda; i64 strideA;
    const T* B; i64 ldb; i64 strideB;
    T* C; i64 ldc; i64 strideC;
    const T* const* Aptrs;  // optional pointer arrays (batched over tiles)
    const T* const* Bptrs;
    T* const* Cptrs;
    int vecA, vecB;          // 16-byte vector loads allowed
    int group_m;             // tile-order group size
    int remap;               // 0: plain order; 1: XCD-chunked grouped order (full output);
                             // 3: the same with row-interleaved groups (triangular masks);
                             // 2: compact lower triangle of 8x8 super-tiles (set by launch_real)
    TriMask mask;
    const int* gate;         // optional device predicate (GemmCall::gate)
    unsigned short ncol[GEMM_STAIR_MAX];   // remap 4: kept block columns per block row
    unsigned gpre[GEMM_STAIR_GROUPS + 1];  // remap 4: kept blocks before each row group
};

// remap 4: kept block lin (grouped column-major order over the staircase) ->
// (bm, bn).  A group of G block rows holds gpre[g + 1] - gpre[g] blocks
// (prefix sums filled by the launcher); inside it column c is kept by the
// rows with ncol > c -- the group's last k rows -- and the blocks before
// column c number F(c) = sum_r min(ncol[r], c).  Both searches are binary
// (O(log) scalar loads per block: the former linear walk cost up to
// gn * G dependent loads per workgroup, measurable on tall local blocks).
template <typename GA>
__device__ inline void stair_block(const GA& a, int lin, int gm, int& bm, int& bn) {
    const int G = a.group_m;
    const int ng = (gm + G - 1) / G;
    int lo = 0, hi = ng - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if ((int)a.gpre[mid] <= lin) lo = mid;
        else hi = mid - 1;
    }
    int rem = lin - (int)a.gpre[lo];
    const int r0 = lo * G, r1 = min(gm, r0 + G);
    auto F = [&](int c) {
        int f = 0;
        for (int r = r0; r < r1; ++r) f += min((int)a.ncol[r], c);
        return f;
    };
    int cl = 0, ch = (int)a.ncol[r1 - 1] - 1;
    while (cl < ch) {
        const int mid = (cl + ch + 1) >> 1;
        if (F(mid) <= rem) cl = mid;
        else ch = mid - 1;
    }
    rem -= F(cl);
    int k = 0;
    for (int r = r0; r < r1; ++r) k += (int)a.ncol[r] > cl;
    bm = rem < k ? r1 - k + rem : gm;    // gm: out of range (never for lin < total)
    bn = cl;
}

// ---------------------------------------------------------------------------
// Operand loader: stages an R x BK slab of op(X) into LDS.
//   ROWC = true : source contiguous along R (element (r,k) at X[r + k*ld]) -> MK image
//   ROWC = false: source contiguous along k (element (r,k) at X[k + r*ld]) -> KM image
template <typename T>
struct alignas(16) Vec16 { T e[16 / sizeof(T)]; };

template <typename T, int R, int BK, bool ROWC, int NT, bool CONJ = false>
struct Stage {
    static constexpr int VEC = 16 / sizeof(T);
    // KM image of 8-byte elements with BK = 8: no pad, XOR swizzle of k by
    // 2 * ((r >> 2) & 3) -- the 32 lanes of a ds_read_b64 group (16 rows x
    // 2 k's) then cover all 64 banks (the odd pad left 2-way conflicts:
    // 11-14 % of LDS cycles in the NN GEMM, profiles/pmc_hot_kernels.md)
    static constexpr bool SWZ = !ROWC && sizeof(T) == 8 && BK == 8;
    static constexpr int PADM = (sizeof(T) == 16) ? 8 : 16, PADK = SWZ ? 0 : 1;
    static constexpr int LDS_ELEMS = ROWC ? BK * (R + PADM) : R * (BK + PADK);
    __device__ static inline int kswz(int r, int k) { return SWZ ? (k ^ (2 * ((r >> 2) & 3))) : k; }
    static constexpr int NVEC = R * BK / VEC;
    static constexpr int PER_THREAD = NVEC / NT;
    static_assert(NVEC % NT == 0, "tile not divisible by threads");
    Vec16<T> reg[PER_THREAD];

    __device__ inline void load(const T* __restrict__ X, i64 ld, i64 r0, i64 k0,
                                i64 Rdim, i64 Kdim, bool vec_ok, int tid) {
        const bool full = vec_ok && (r0 + R <= Rdim) && (k0 + BK <= Kdim);
        #pragma unroll
        for (int i = 0; i < PER_THREAD; ++i) {
            int v = tid + i * NT;
            int r, kk;
            if (ROWC) { kk = v / (R / VEC); r = (v % (R / VEC)) * VEC; }
            else      { r = v / (BK / VEC); kk = (v % (BK / VEC)) * VEC; }
            if (full) {
                const T* p = ROWC ? X + (r0 + r) + (k0 + kk) * ld
                                  : X + (k0 + kk) + (r0 + r) * ld;
                reg[i] = *reinterpret_cast<const Vec16<T>*>(p);
            } else {
                #pragma unroll
                for (int e = 0; e < VEC; ++e) {
                    i64 rr = r0 + r + (ROWC ? e : 0);
                    i64 kq = k0 + kk + (ROWC ? 0 : e);
                    T val = s_zero(T());
                    if (rr < Rdim && kq < Kdim)
                        val = ROWC ? X[rr + kq * ld] : X[kq + rr * ld];
                    reg[i].e[e] = val;
                }
            }
            if constexpr (CONJ) {
                #pragma unroll
                for (int e = 0; e < VEC; ++e) reg[i].e[e] = s_conj(reg[i].e[e]);
            }
        }
    }
    __device__ inline void store(T* lds, int tid) const {
        #pragma unroll
        for (int i = 0; i < PER_THREAD; ++i) {
            int v = tid + i * NT;
            if (ROWC) {
                int kk = v / (R / VEC), r = (v % (R / VEC)) * VEC;
                *reinterpret_cast<Vec16<T>*>(lds + kk * (R + PADM) + r) = reg[i];
            } else {
                int r = v / (BK / VEC), kk = (v % (BK / VEC)) * VEC;
                if constexpr (SWZ) {
                    // kk even, the swizzle even: the pair stays adjacent
                    *reinterpret_cast<Vec16<T>*>(lds + r * BK + kswz(r, kk)) = reg[i];
                } else {
                    T* p = lds + r * (BK + PADK) + kk;
                    #pragma unroll
                    for (int e = 0; e < VEC; ++e) p[e] = reg[i].e[e];
                }
            }
        }
    }
    // fragment element (r, k) from the LDS image
    __device__ static inline T frag(const T* lds, int r, int k) {
        return ROWC ? lds[k * (R + PADM) + r] : lds[r * (BK + PADK) + kswz(r, k)];
    }
};

// PF: operand prefetch depth in K steps.  1: the next step's global loads
// are issued at the top of the current step (one register set);
// 2: two steps ahead (two register sets, main loop unrolled by two so every
// set is statically indexed) -- a whole step more latency cover for the
// L2-missing operand loads of the wide trailing updates.
template <typename T, bool TA, bool TB, int BM, int BN, int BK, bool PTRS, int WVM = 2, int WVN = 2, int OCC = 2,
          int PF = 1>
__global__ void __launch_bounds__(64 * WVM * WVN, OCC)
gemm_real_kernel(GemmArgs<T> a) {
    using MF = mfma_real<T>;
    using acc_t = typename MF::acc_t;
    if (a.gate && *a.gate == 0) return;
    constexpr int NT = 64 * WVM * WVN;
    constexpr int WM = BM / WVM, WN = BN / WVN;
    constexpr int MI = WM / 16, NI = WN / 16;
    // op(A) (m x k): !TA -> A stored m x k col-major, contiguous along m.
    using SA = Stage<T, BM, BK, !TA, NT>;
    // op(B) (k x n): !TB -> B stored k x n col-major, contiguous along k.
    using SB = Stage<T, BN, BK, TB, NT>;
    constexpr int LA = SA::LDS_ELEMS, LB = SB::LDS_ELEMS;
    __shared__ T smem[2 * (LA + LB)];

    const int batch = blockIdx.y;
    const T* A; const T* B; T* C;
    if constexpr (PTRS) { A = a.Aptrs[batch]; B = a.Bptrs[batch]; C = a.Cptrs[batch]; }
    else { A = a.A + batch * a.strideA; B = a.B + batch * a.strideB; C = a.C + batch * a.strideC; }

    const int gm = (int)((a.m + BM - 1) / BM), gn = (int)((a.n + BN - 1) / BN);
    int bm, bn;
    if (a.remap == 4) {
        stair_block(a, xcd_remap(blockIdx.x, gridDim.x), gm, bm, bn);
        if (bm >= gm || bn >= gn) return;
    } else if (a.remap == 2) {
        // compact lower triangle (launcher checked that no tile above the
        // diagonal holds a kept element): the grid covers only the 8 x 8
        // super-tiles I >= J, column by column, so the XCD chunks stay
        // balanced and each chunk is a run of whole super-tiles (L2 reuse of
        // 8 A and 8 B tiles per 64 outputs).
        const int lin = xcd_remap(blockIdx.x, gridDim.x);
        const int s = lin >> 6, w = lin & 63;
        const int gsm = (gm + 7) >> 3;
        int J = 0, rem = s;
        while (rem >= gsm - J) { rem -= gsm - J; ++J; }
        bm = (J + rem) * 8 + (w & 7);
        bn = J * 8 + (w >> 3);
        if (bm >= gm || bn >= gn) return;
    } else {
        const int nblk = gm * gn;
        int lin = a.remap ? xcd_remap(blockIdx.x, nblk) : (int)blockIdx.x;
        // grouped ordering: GROUP block-rows swept column by column
        const int G = a.group_m;
        int grp = lin / (G * gn);
        int first = grp * G;
        int gsz = min(gm - first, G);
        int inner = lin - grp * G * gn;
        bm = first + inner % gsz; bn = inner / gsz;
        // remap 3 (triangular masks): the grouped rows interleaved over the
        // whole range, so every XCD chunk holds a balanced share of kept blocks
        if (a.remap == 3) bm = row_interleave(bm, gm, G);
    }
    const i64 m0 = (i64)bm * BM, n0 = (i64)bn * BN;
    if (a.mask.skip_block(m0, min(m0 + BM, a.m), n0, min(n0 + BN, a.n))) return;

    const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wid / WVN, wn = wid % WVN;

    acc_t acc[MI][NI];
    #pragma unroll
    for (int i = 0; i < MI; ++i)
        #pragma unroll
        for (int j = 0; j < NI; ++j)
            #pragma unroll
            for (int r = 0; r < 4; ++r) acc[i][j][r] = T(0);

    SA sa; SB sb;
    const i64 K = a.k;
    const int nk = (int)((K + BK - 1) / BK);
    auto compute = [&](const T* la, const T* lb) {
        #pragma unroll
        for (int kk = 0; kk < BK / 4; ++kk) {
            const int kq = kk * 4 + (lane >> 4);
            T ya[MI], xb[NI];
            #pragma unroll
            for (int i = 0; i < MI; ++i) ya[i] = SA::frag(la, wm * WM + i * 16 + (lane & 15), kq);
            #pragma unroll
            for (int j = 0; j < NI; ++j) xb[j] = SB::frag(lb, wn * WN + j * 16 + (lane & 15), kq);
            #pragma unroll
            for (int i = 0; i < MI; ++i)
                #pragma unroll
                for (int j = 0; j < NI; ++j) acc[i][j] = MF::mma(xb[j], ya[i], acc[i][j]);
        }
    };
    if (nk > 0) {
        sa.load(A, a.lda, m0, 0, a.m, K, a.vecA, tid);
        sb.load(B, a.ldb, n0, 0, a.n, K, a.vecB, tid);
        sa.store(smem, tid);
        sb.store(smem + LA, tid);
    }
    if constexpr (PF == 1) {
        __syncthreads();
        for (int kt = 0; kt < nk; ++kt) {
            T* cur = smem + (kt & 1) * (LA + LB);
            T* nxt = smem + ((kt + 1) & 1) * (LA + LB);
            const bool more = kt + 1 < nk;
            if (more) {
                sa.load(A, a.lda, m0, (i64)(kt + 1) * BK, a.m, K, a.vecA, tid);
                sb.load(B, a.ldb, n0, (i64)(kt + 1) * BK, a.n, K, a.vecB, tid);
            }
            compute(cur, cur + LA);
            if (more) {
                sa.store(nxt, tid);
                sb.store(nxt + LA, tid);
            }
            __syncthreads();
        }
    } else {
        SA sa2; SB sb2;
        if (nk > 1) {
            sa2.load(A, a.lda, m0, (i64)BK, a.m, K, a.vecA, tid);
            sb2.load(B, a.ldb, n0, (i64)BK, a.n, K, a.vecB, tid);
        }
        __syncthreads();
        // step kt: (na, nb_) hold step kt + 1 (in flight), (fa, fb) are free
        // (their step is in LDS already) and take step kt + 2
        auto step = [&](int kt, SA& na, SB& nb_, SA& fa, SB& fb) {
            T* cur = smem + (kt & 1) * (LA + LB);
            T* nxt = smem + ((kt + 1) & 1) * (LA + LB);
            if (kt + 2 < nk) {
                fa.load(A, a.lda, m0, (i64)(kt + 2) * BK, a.m, K, a.vecA, tid);
                fb.load(B, a.ldb, n0, (i64)(kt + 2) * BK, a.n, K, a.vecB, tid);
            }
            compute(cur, cur + LA);
            if (kt + 1 < nk) {
                na.store(nxt, tid);
                nb_.store(nxt + LA, tid);
            }
            __syncthreads();
        };
        int kt = 0;
        for (; kt + 1 < nk; kt += 2) {
            step(kt, sa2, sb2, sa, sb);
            step(kt + 1, sa, sb, sa2, sb2);
        }
        if (kt < nk) step(kt, sa2, sb2, sa, sb);
    }

    // epilogue
    const bool full = a.mask.full_block(m0, min(m0 + BM, a.m), n0, min(n0 + BN, a.n))
                      && m0 + BM <= a.m && n0 + BN <= a.n;
    const T alpha = a.alpha, beta = a.beta;
    const bool beta0 = (beta == T(0));
    #pragma unroll
    for (int i = 0; i < MI; ++i) {
        const i64 m = m0 + wm * WM + i * 16 + (lane & 15);
        #pragma unroll
        for (int j = 0; j < NI; ++j) {
            #pragma unroll
            for (int r = 0; r < 4; ++r) {
                const i64 n = n0 + wn * WN + j * 16 + MF::drow(lane, r);
                if (full || (m < a.m && n < a.n && a.mask.keep(m, n))) {
                    T* pc = C + m + n * a.ldc;
                    T v = alpha * acc[i][j][r];
                    if (!beta0) v += beta * *pc;
                    *pc = v;
                }
            }
        }
    }
}

}  // namespace slate_hip

namespace slate_hip {

// Complex GEMM: four real MFMAs per complex multiply-accumulate on split
// re/im fragments (no 3M trick: keeps the LAPACK error bound).
template <typename T, char TA, char TB, int BM, int BN, int BK, bool PTRS>
__global__ void __launch_bounds__(256, 2)
gemm_complex_kernel(GemmArgs<T> a) {
    using R = typename scalar_traits<T>::real;
    using MF = mfma_real<R>;
    using acc_t = typename MF::acc_t;
    if (a.gate && *a.gate == 0) return;
    constexpr int NT = 256;
    constexpr int WM = BM / 2, WN = BN / 2;
    constexpr int MI = WM / 16, NI = WN / 16;
    using SA = Stage<T, BM, BK, TA == 'N', NT, TA == 'C'>;
    using SB = Stage<T, BN, BK, TB != 'N', NT, TB == 'C'>;
    constexpr int LA = SA::LDS_ELEMS, LB = SB::LDS_ELEMS;
    __shared__ T smem[2 * (LA + LB)];

    const int batch = blockIdx.y;
    const T* A; const T* B; T* C;
    if constexpr (PTRS) { A = a.Aptrs[batch]; B = a.Bptrs[batch]; C = a.Cptrs[batch]; }
    else { A = a.A + batch * a.strideA; B = a.B + batch * a.strideB; C = a.C + batch * a.strideC; }

    const int gm = (int)((a.m + BM - 1) / BM), gn = (int)((a.n + BN - 1) / BN);
    int lin = a.remap ? xcd_remap(blockIdx.x, gm * gn) : (int)blockIdx.x;
    const int G = a.group_m;
    int grp = lin / (G * gn), first = grp * G, gsz = min(gm - first, G);
    int inner = lin - grp * G * gn;
    const int bm = a.remap == 3 ? row_interleave(first + inner % gsz, gm, G) : first + inner % gsz, bn = inner / gsz;
    const i64 m0 = (i64)bm * BM, n0 = (i64)bn * BN;
    if (a.mask.skip_block(m0, min(m0 + BM, a.m), n0, min(n0 + BN, a.n))) return;

    const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wid >> 1, wn = wid & 1;
    acc_t are[MI][NI], aim[MI][NI];
    #pragma unroll
    for (int i = 0; i < MI; ++i)
        #pragma unroll
        for (int j = 0; j < NI; ++j)
            #pragma unroll
            for (int r = 0; r < 4; ++r) { are[i][j][r] = R(0); aim[i][j][r] = R(0); }

    SA sa; SB sb;
    const i64 K = a.k;
    const int nk = (int)((K + BK - 1) / BK);
    if (nk > 0) {
        sa.load(A, a.lda, m0, 0, a.m, K, a.vecA, tid);
        sb.load(B, a.ldb, n0, 0, a.n, K, a.vecB, tid);
        sa.store(smem, tid);
        sb.store(smem + LA, tid);
    }
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
        T* cur = smem + (kt & 1) * (LA + LB);
        T* nxt = smem + ((kt + 1) & 1) * (LA + LB);
        const bool more = kt + 1 < nk;
        if (more) {
            sa.load(A, a.lda, m0, (i64)(kt + 1) * BK, a.m, K, a.vecA, tid);
            sb.load(B, a.ldb, n0, (i64)(kt + 1) * BK, a.n, K, a.vecB, tid);
        }
        #pragma unroll
        for (int kk = 0; kk < BK / 4; ++kk) {
            const int kq = kk * 4 + (lane >> 4);
            T ya[MI], xb[NI];
            #pragma unroll
            for (int i = 0; i < MI; ++i) ya[i] = SA::frag(cur, wm * WM + i * 16 + (lane & 15), kq);
            #pragma unroll
            for (int j = 0; j < NI; ++j) xb[j] = SB::frag(cur + LA, wn * WN + j * 16 + (lane & 15), kq);
            #pragma unroll
            for (int i = 0; i < MI; ++i)
                #pragma unroll
                for (int j = 0; j < NI; ++j) {
                    are[i][j] = MF::mma(xb[j].re, ya[i].re, are[i][j]);
                    are[i][j] = MF::mma(-xb[j].im, ya[i].im, are[i][j]);
                    aim[i][j] = MF::mma(xb[j].re, ya[i].im, aim[i][j]);
                    aim[i][j] = MF::mma(xb[j].im, ya[i].re, aim[i][j]);
                }
        }
        if (more) { sa.store(nxt, tid); sb.store(nxt + LA, tid); }
        __syncthreads();
    }
    const T alpha = a.alpha, beta = a.beta;
    const bool beta0 = s_is_zero(beta);
    #pragma unroll
    for (int i = 0; i < MI; ++i) {
        const i64 m = m0 + wm * WM + i * 16 + (lane & 15);
        #pragma unroll
        for (int j = 0; j < NI; ++j)
            #pragma unroll
            for (int r = 0; r < 4; ++r) {
                const i64 n = n0 + wn * WN + j * 16 + MF::drow(lane, r);
                if (m < a.m && n < a.n && a.mask.keep(m, n)) {
                    T* pc = C + m + n * a.ldc;
                    T v = s_mul(alpha, T{are[i][j][r], aim[i][j][r]});
                    if (!beta0) v = s_add(v, s_mul(beta, *pc));
                    *pc = v;
                }
            }
    }
}

}  // namespace slate_hip
