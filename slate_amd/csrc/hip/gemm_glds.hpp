// fp64 MFMA GEMM with LDS-DMA staging for gfx950:  C = alpha op(A) op(B) + beta C
//
// The production fp64 kernel of gemm.hpp stages operands global -> VGPR ->
// LDS with one K step (BK = 8) in flight.  This one streams both operands
// straight into LDS with global_load_lds_dwordx4 (no VGPR destination, no
// ds_write pass) through an S-stage ring of BK = 16 slabs, so S - 1 K steps
// of loads are in flight across each barrier: one raw s_barrier per K step,
// a counted vmcnt (never 0 inside the loop), and the MFMA chain of 64-cycle
// v_mfma_f64_16x16x4 never waits on an L2 miss.
//
// LDS images (one 1 KiB wave-instruction chunk = 128 doubles, written
// lane-linear; the swizzle lives on the SOURCE address and on the read, the
// same involution on both sides):
//  * MK, source contiguous along the tile's rows r (element (r, k) at
//    X[r + k ld]): image [k][R], element r of row k at r ^ 16 (k & 1) -- the
//    k and k + 1 groups of one ds_read_b64 half-wave sit in opposite 128-byte
//    halves of the bank row;
//  * KM, source contiguous along k (element (r, k) at X[k + r ld]): image
//    [r][16], element k of row r at k ^ 2 ((r >> 1) & 7) -- 16 rows at one k
//    land on 16 distinct 8-byte slots, and k + 1 on the other 16.
// Tile edges in m / n clamp the source row (the duplicated rows feed only
// outputs the epilogue never stores); K must be a multiple of 16 and both
// operands 16-byte aligned with even leading dimensions (launcher checks;
// the register-staged kernel takes every other case).
#pragma once
#include "gemm.hpp"

namespace slate_hip {

template <int R, bool MK>
struct GldsImg {
    static constexpr int BK = 16;
    static constexpr int ELEMS = R * BK;
    static constexpr int CHUNKS = ELEMS / 128;
    __device__ static inline int idx(int r, int k) {
        if constexpr (MK) return k * R + (r ^ ((k & 1) << 4));
        else return r * BK + (k ^ (((r >> 1) & 7) << 1));
    }
    // (r, k) of the first element of the 16-byte pair lane `lane` of chunk c stages
    __device__ static inline void src_of(int c, int lane, int& r, int& k) {
        const int p = c * 128 + 2 * lane;
        if constexpr (MK) {
            k = p / R;
            r = (p % R) ^ ((k & 1) << 4);
        } else {
            r = p >> 4;
            k = (p & 15) ^ (((r >> 1) & 7) << 1);
        }
    }
    // issue this wave's share of the slab (rows r0.., k0..k0+15) into img
    template <int NW>
    __device__ static inline void load(const double* __restrict__ X, i64 ld, i64 r0, i64 k0, i64 Rdim, double* img,
                                       int wid, int lane) {
        static_assert(CHUNKS % NW == 0, "slab chunks not divisible by waves");
        constexpr int PER = CHUNKS / NW;
        #pragma unroll
        for (int i = 0; i < PER; ++i) {
            const int c = wid * PER + i;
            int r, k;
            src_of(c, lane, r, k);
            i64 rr = r0 + r;
            const double* p;
            if constexpr (MK) {
                if (rr >= Rdim) rr = (Rdim - 1) & ~(i64)1;
                p = X + rr + (k0 + k) * ld;
            } else {
                if (rr >= Rdim) rr = Rdim - 1;
                p = X + (k0 + k) + rr * ld;
            }
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)p,
                                             (__attribute__((address_space(3))) void*)(img + c * 128), 16, 0, 0);
        }
    }
};

// s_waitcnt vmcnt(N) with lgkm / exp left alone (gfx9 encoding)
template <int N>
__device__ inline void wait_vmcnt() {
    static_assert(N >= 0 && N < 64, "vmcnt range");
    __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

template <int BM, int BN, bool TA, bool TB, int S>
constexpr size_t glds_lds_bytes() {
    return (size_t)S * (GldsImg<BM, !TA>::ELEMS + GldsImg<BN, TB>::ELEMS) * sizeof(double);
}

template <bool TA, bool TB, int BM, int BN, int WVM, int WVN, int S, int OCC, int PRIO = 0>
__global__ void __launch_bounds__(64 * WVM * WVN, OCC) gemm_f64_glds_kernel(GemmArgs<double> a) {
    using MF = mfma_real<double>;
    using acc_t = typename MF::acc_t;
    constexpr int BK = 16, NW = WVM * WVN;
    constexpr int WM = BM / WVM, WN = BN / WVN, MI = WM / 16, NI = WN / 16;
    using IA = GldsImg<BM, !TA>;
    using IB = GldsImg<BN, TB>;
    constexpr int LA = IA::ELEMS, LS = IA::ELEMS + IB::ELEMS;
    constexpr int L = (IA::CHUNKS + IB::CHUNKS) / NW;   // glds instructions per wave per K step
    static_assert(S >= 2 && S <= 4, "stages");
    extern __shared__ __align__(16) double smem[];

    if (a.gate && *a.gate == 0) return;
    const int batch = blockIdx.y;
    const double* A = a.A + batch * a.strideA;
    const double* B = a.B + batch * a.strideB;
    double* C = a.C + batch * a.strideC;

    const int gm = (int)((a.m + BM - 1) / BM), gn = (int)((a.n + BN - 1) / BN);
    int bm, bn;
    if (a.remap == 4) {
        stair_block(a, xcd_remap(blockIdx.x, gridDim.x), gm, bm, bn);
        if (bm >= gm || bn >= gn) return;
    } else if (a.remap == 2) {
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
        const int lin = a.remap ? xcd_remap(blockIdx.x, nblk) : (int)blockIdx.x;
        const int G = a.group_m;
        const int grp = lin / (G * gn), first = grp * G, gsz = min(gm - first, G);
        const int inner = lin - grp * G * gn;
        bm = first + inner % gsz;
        bn = inner / gsz;
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
            for (int r = 0; r < 4; ++r) acc[i][j][r] = 0.0;

    const int nk = (int)(a.k / BK);
    auto issue = [&](int kt) {
        double* st = smem + (kt % S) * LS;
        IA::template load<NW>(A, a.lda, m0, (i64)kt * BK, a.m, st, wid, lane);
        IB::template load<NW>(B, a.ldb, n0, (i64)kt * BK, a.n, st + LA, wid, lane);
    };
    #pragma unroll
    for (int s = 0; s < S - 1; ++s)
        if (s < nk) issue(s);
    for (int kt = 0; kt < nk; ++kt) {
        // my loads of step kt landed (later steps may stay in flight) ...
        if (kt + S - 2 < nk) wait_vmcnt<(S - 2) * L>();
        else if constexpr (S > 2) {
            if (kt + 1 < nk) wait_vmcnt<L>();     // S = 4 tail: one later step in flight
            else wait_vmcnt<0>();
        } else wait_vmcnt<0>();
        // ... everyone's landed, and everyone finished reading step kt - 1's stage
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        if (kt + S - 1 < nk) issue(kt + S - 1);
        const double* la = smem + (kt % S) * LS;
        const double* lb = la + LA;
        if constexpr (PRIO) __builtin_amdgcn_s_setprio(1);
        #pragma unroll
        for (int kk = 0; kk < BK / 4; ++kk) {
            const int kq = kk * 4 + (lane >> 4);
            double ya[MI], xb[NI];
            #pragma unroll
            for (int i = 0; i < MI; ++i) ya[i] = la[IA::idx(wm * WM + i * 16 + (lane & 15), kq)];
            #pragma unroll
            for (int j = 0; j < NI; ++j) xb[j] = lb[IB::idx(wn * WN + j * 16 + (lane & 15), kq)];
            #pragma unroll
            for (int i = 0; i < MI; ++i)
                #pragma unroll
                for (int j = 0; j < NI; ++j) acc[i][j] = MF::mma(xb[j], ya[i], acc[i][j]);
        }
        if constexpr (PRIO) __builtin_amdgcn_s_setprio(0);
    }

    const bool full = a.mask.full_block(m0, min(m0 + BM, a.m), n0, min(n0 + BN, a.n)) && m0 + BM <= a.m &&
                      n0 + BN <= a.n;
    const double alpha = a.alpha, beta = a.beta;
    const bool beta0 = (beta == 0.0);
    #pragma unroll
    for (int i = 0; i < MI; ++i) {
        const i64 m = m0 + wm * WM + i * 16 + (lane & 15);
        #pragma unroll
        for (int j = 0; j < NI; ++j)
            #pragma unroll
            for (int r = 0; r < 4; ++r) {
                const i64 n = n0 + wn * WN + j * 16 + MF::drow(lane, r);
                if (full || (m < a.m && n < a.n && a.mask.keep(m, n))) {
                    double* pc = C + m + n * a.ldc;
                    double v = alpha * acc[i][j][r];
                    if (!beta0) v += beta * *pc;
                    *pc = v;
                }
            }
    }
}

}  // namespace slate_hip
