// Latency-optimised fp64 kernels of the Cholesky panel on gfx950:
//
//   potrf_lds   ONE workgroup (512 threads, one CU) factors a lower n <= 512
//               tile: left-looking over 32-wide column blocks; the block
//               column (<= 512 x 32) lives in LDS (131 KB of the 160 KB), the
//               left-looking update A(c0:, J) -= L(c0:, :c0) L(J, :c0)^T runs
//               on the f64 MFMA (operands streamed from L2, where this CU just
//               wrote them), the 16-wide diagonal sub-blocks are factored by
//               256 threads, one element each (one barrier per column, the
//               inverse one column behind), and the rows below are solved on
//               the MFMA against that inverse.  One
//               launch replaces the 4 x (potrf_small + trsm + herk) chain of
//               potrf.hip (measured 870 us for n = 512 on MI355X) and leaves
//               every other CU to the trailing update.
//   tri_inv32   inverses of the 32 x 32 diagonal blocks of a lower triangle
//               (one wave per block, column-per-lane substitution).
//   trsm_rlt    X L^T = alpha B for a tall B (the Cholesky panel solve,
//               src/internal/internal_trsm.cc:244 in the reference): every
//               workgroup owns 64 rows, walks 32-column blocks,
//               R = alpha B_J - X_{<J} L_{J,<J}^T (MFMA, K = 32 J) and
//               X_J = R inv(L_JJ)^T (MFMA against tri_inv32's output): every
//               flop on the matrix cores, one launch, no copy-back.
#include <cstdlib>
#include <cstring>
#include "common.hpp"
#include "kernels.hpp"
#include "launchers.hpp"
#include "workspace.hpp"

namespace slate_hip {

namespace {
constexpr int PN = 512;          // largest tile of potrf_lds
constexpr int PB = 32;           // block-column width
constexpr int PT = 512;          // threads of potrf_lds (8 waves: 256-VGPR budget)
constexpr int PLD = PN + 1;      // LDS column stride (doubles)

__device__ inline d4 mma(double x, double y, d4 c) { return __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, c, 0, 0, 0); }
// 1/sqrt(d) for d > 0: hardware estimate + two Newton steps (full fp64)
__device__ inline double rsq_f64(double d) {
    double r = __builtin_amdgcn_rsq(d);
    r = r * (1.5 - 0.5 * d * r * r);
    return r * (1.5 - 0.5 * d * r * r);
}
}  // namespace

// acc[t] += sum_k X(r, k) Y(c, k) over k in [0, K), for one
// 16-row strip (rows xr) and NT 16-column tiles (rows yr[t] of Y); lane
// layout of the f64 MFMA: operand element (lane & 15, k + (lane >> 4)).
// 32-k chunks double-buffered in registers: 24 loads per lane in flight
// while the previous chunk's MFMAs issue.  Requires K % 32 == 0.
typedef unsigned int u2v __attribute__((ext_vector_type(2)));
// raw buffer descriptor on a wave-uniform base (32-bit offsets: every operand
// region here spans < 2 GiB from its base)
__device__ inline __amdgpu_buffer_rsrc_t rsrc_of(const double* p) {
    const uintptr_t a = (uintptr_t)p;
    const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)a);
    const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(a >> 32));
    return __builtin_amdgcn_make_buffer_rsrc((void*)(((uintptr_t)hi << 32) | lo), 0, 0x7fffffff, 0x00020000);
}
__device__ inline double bld(__amdgpu_buffer_rsrc_t r, int voff, int soff) {
    return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, voff, soff, 0));
}

// acc[s][t] += sum_k X(xr[s], k) Y(yr[t], k), k in [0, K), K % (8 U) == 0:
// NS 16-row strips of X against NT 16-row tiles of Y, per-lane rows xr/yr
// relative to wave-uniform bases.  Chunks of U k-steps (of 4) are
// double-buffered in registers: one chunk's loads are in flight while the
// previous chunk's NS*NT*U MFMAs issue.
template <int NS, int NT, int U>
__device__ inline void strip_update(d4 (&acc)[NS][NT], const double* Xb, const int (&xr)[NS], i64 ldx,
                                    const double* Yb, const int (&yr)[NT], i64 ldy, int K, int lane) {
    const int kq = lane >> 4;
    const __amdgpu_buffer_rsrc_t rx = rsrc_of(Xb), ry = rsrc_of(Yb);
    int vx[NS], vy[NT];
    #pragma unroll
    for (int s = 0; s < NS; ++s) vx[s] = (int)((xr[s] + kq * ldx) * 8);
    #pragma unroll
    for (int t = 0; t < NT; ++t) vy[t] = (int)((yr[t] + kq * ldy) * 8);
    double a[2][NS][U], b[2][NT][U];
    auto load = [&](int buf, int k) {
        #pragma unroll
        for (int u = 0; u < U; ++u) {
            #pragma unroll
            for (int s = 0; s < NS; ++s) a[buf][s][u] = bld(rx, vx[s], (int)((k + 4 * u) * ldx * 8));
            #pragma unroll
            for (int t = 0; t < NT; ++t) b[buf][t][u] = bld(ry, vy[t], (int)((k + 4 * u) * ldy * 8));
        }
    };
    auto comp = [&](int buf) {
        #pragma unroll
        for (int u = 0; u < U; ++u)
            #pragma unroll
            for (int s = 0; s < NS; ++s)
                #pragma unroll
                for (int t = 0; t < NT; ++t) acc[s][t] = mma(b[buf][t][u], a[buf][s][u], acc[s][t]);
    };
    if (K <= 0) return;
    load(0, 0);
    int k = 0;
    for (; k + 4 * U < K; k += 8 * U) {
        load(1, k + 4 * U);
        comp(0);
        if (k + 8 * U < K) load(0, k + 8 * U);
        comp(1);
    }
    if (k < K) comp(0);
}

// ---------------------------------------------------------------- potrf_lds
__global__ void __launch_bounds__(PT)
potrf_lds_kernel(int n, double* __restrict__ A, i64 lda, i64* info, i64 info_off, i64* prof, const int* gate,
                 const double* floorp) {
    // gate: device predicate (0 = skip the launch); floorp: regularised mode
    // -- a pivot <= *floorp is replaced by *floorp instead of failing (the
    // CholeskyQR fallback, qr_fast.hip)
    if (gate && *gate == 0) return;
    const double pfloor = floorp ? *floorp : 0.0;
    __shared__ double P[PB * PLD];          // P[c * PLD + r] = A(c0 + r, c0 + c)
    __shared__ double Li[16][17];            // inverse of the current 16 x 16 diagonal sub-block
    __shared__ double Ld[16][17];            // its Cholesky factor (row-major, zero above)
    __shared__ double Dd[16][17];            // working copy of the sub-block
    __shared__ double Xf[16][17];            // final rows of the inverse
    __shared__ double rdl[16];               // 1 / L(j, j)
    __shared__ int s_fail;
    const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform (SGPR): w-derived branches stay scalar
    if (tid == 0) s_fail = 0;
    // optional per-phase shader-clock totals (prof != nullptr: tools only)
    i64 ph[6] = {0, 0, 0, 0, 0, 0};
    i64 tlast = clock64();
    const i64 t0 = tlast, w0 = wall_clock64();
#define STAMP(i) do { if (prof && tid == 0) { const i64 t_ = clock64(); ph[i] += t_ - tlast; tlast = t_; } } while (0)
    const int lr = tid;                                   // one row per thread, 32 columns
    // raw A values of the next block column, loaded one block ahead: plain
    // loads survive the barriers of the factorization phases (no LDS-DMA in
    // flight), so their latency hides behind them
    double v[PB];
    auto fetch = [&](int cn) {
        const int jbn = min(PB, n - cn), Mn = n - cn;
        const __amdgpu_buffer_rsrc_t rs = rsrc_of(A + cn + (i64)cn * lda);   // 32-bit offsets: one VGPR
        const int vo = min(lr, Mn - 1) * 8;
        #pragma unroll
        for (int c = 0; c < PB; ++c) v[c] = bld(rs, vo, (int)((i64)min(c, jbn - 1) * lda * 8));
    };
    fetch(0);
    for (int c0 = 0; c0 < n; c0 += PB) {
        const int jb = min(PB, n - c0), M = n - c0;
        // ---- stage the block column (lower part)
        #pragma unroll
        for (int c = 0; c < PB; ++c)
            if (c < jb && lr < M && lr >= c) P[c * PLD + lr] = v[c];
        __syncthreads();
        STAMP(0);
        // ---- left-looking update by the factored columns [0, c0)
        if (c0 > 0) {
            // strip pairs (2s, 2s+1) x both 16-column tiles per wave
            for (int sp = w; 32 * sp < M; sp += PT / 64) {
                const int xr[2] = {min(32 * sp + (lane & 15), M - 1), min(32 * sp + 16 + (lane & 15), M - 1)};
                const int yr[2] = {min(lane & 15, M - 1), min(16 + (lane & 15), M - 1)};
                d4 acc[2][2];
                #pragma unroll
                for (int u = 0; u < 2; ++u)
                    #pragma unroll
                    for (int t = 0; t < 2; ++t) acc[u][t] = d4{0, 0, 0, 0};
                strip_update<2, 2, 4>(acc, A + c0, xr, lda, A + c0, yr, lda, c0, lane);
                #pragma unroll
                for (int u = 0; u < 2; ++u)
                    #pragma unroll
                    for (int t = 0; t < 2; ++t)
                        #pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            const int m = 32 * sp + 16 * u + (lane & 15), c = 16 * t + (lane >> 4) + 4 * r;
                            if (m < M && c < jb && m >= c) P[c * PLD + m] -= acc[u][t][r];
                        }
            }
            __syncthreads();
        }
        STAMP(1);
        if (c0 + PB < n) fetch(c0 + PB);                  // in flight through the phases below
        // ---- factor the block column in LDS, 16 columns at a time:
        //  (1) 256 threads: 16 x 16 diagonal sub-block -> L_qq and inv(L_qq);
        //  (2) every wave: rows below, X = P inv(L_qq)^T on the MFMA;
        //  (3) first half only: P(:, 16:32) -= X X(16:32, :)^T on the MFMA.
        for (int q0 = 0; q0 < jb; q0 += 16) {
            const int wq = min(16, jb - q0);
            {
                // thread (di, dc) < 256 owns element (di, dc): right-looking
                // Cholesky two columns per barrier (2x2 diagonal step, rank-2
                // update); the inverse (forward substitution on I) runs one
                // pair behind, final rows going to Xf (no row is read and
                // written in the same interval)
                const bool act = tid < 256;
                const int di = tid & 15, dc = (tid >> 4) & 15;
                if (act) {
                    Dd[di][dc] = (di < wq && dc <= di) ? P[(q0 + dc) * PLD + q0 + di] : (di == dc ? 1.0 : 0.0);
                    Li[di][dc] = (di == dc) ? 1.0 : 0.0;
                }
                __syncthreads();
                double myl = 0.0;
                int fail = 0;
                #pragma unroll 1
                for (int j = 0; j <= 16; j += 2) {
                    if (act && j > 0) {
                        // substitution steps j-2, j-1 (their L columns were
                        // written in the previous interval; issued first: its LDS reads
                        // do not wait behind this interval's writes)
                        const double x2 = Li[j - 2][dc] * rdl[j - 2];
                        const double x1 = (Li[j - 1][dc] - Ld[j - 1][j - 2] * x2) * rdl[j - 1];
                        if (di == j - 2) Xf[di][dc] = x2;
                        else if (di == j - 1) Xf[di][dc] = x1;
                        else if (di >= j) Li[di][dc] -= Ld[di][j - 2] * x2 + Ld[di][j - 1] * x1;
                    }
                    if (act && j < 16) {
                        double d0 = Dd[j][j];
                        const double d10 = Dd[j + 1][j], d11 = Dd[j + 1][j + 1];
                        const double a0 = Dd[di][j], a1 = Dd[di][j + 1], b0 = Dd[dc][j], b1 = Dd[dc][j + 1];
                        if (j < wq && !(d0 > pfloor)) {
                            if (pfloor > 0.0) d0 = pfloor;
                            else { if (!fail) fail = c0 + q0 + j + 1; d0 = 1.0; }
                        }
                        const double i0 = rsq_f64(d0), s0 = d0 * i0;          // 1 / L(j, j), L(j, j)
                        const double l10 = d10 * i0;
                        double e = d11 - l10 * l10;
                        if (j + 1 < wq && !(e > pfloor)) {
                            if (pfloor > 0.0) e = pfloor;
                            else { if (!fail) fail = c0 + q0 + j + 2; e = 1.0; }
                        }
                        const double i1 = rsq_f64(e), s1 = e * i1;
                        const double ld0 = a0 * i0, ld1 = (a1 - ld0 * l10) * i1;   // L(di, j), L(di, j+1)
                        const double lc0 = b0 * i0, lc1 = (b1 - lc0 * l10) * i1;   // L(dc, j), L(dc, j+1)
                        if (dc == j) {
                            myl = di > j ? ld0 : (di == j ? s0 : 0.0);
                            Ld[di][j] = myl;
                        } else if (dc == j + 1) {
                            myl = di > j + 1 ? ld1 : (di == j + 1 ? s1 : 0.0);
                            Ld[di][j + 1] = myl;
                        } else if (dc > j + 1 && di >= dc) {
                            Dd[di][dc] -= ld0 * lc0 + ld1 * lc1;
                        }
                        if (tid == 0) { rdl[j] = i0; rdl[j + 1] = i1; }
                    }
                    __syncthreads();
                }
                if (act && di < wq && dc <= di) P[(q0 + dc) * PLD + q0 + di] = myl;
                if (tid == 0 && fail && !s_fail) s_fail = fail;
            }
            __syncthreads();
            STAMP(2);
            // (2) strips of 16 rows below the sub-block: X = P(:, q0:q0+16) inv^T
            const int rb0 = q0 + wq;                          // first row below
            const int nstrip = (M - rb0 + 15) / 16;
            for (int st = w; st < nstrip; st += PT / 64) {
                const int rb = rb0 + 16 * st;
                const int rr = rb + (lane & 15);
                const bool ok = rr < M;
                double a[4];
                #pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int k = 4 * u + (lane >> 4);
                    a[u] = (ok && k < wq) ? P[(q0 + k) * PLD + rr] : 0.0;
                }
                d4 acc = {0, 0, 0, 0};
                #pragma unroll
                for (int u = 0; u < 4; ++u) acc = mma(Xf[lane & 15][4 * u + (lane >> 4)], a[u], acc);
                #pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int c = (lane >> 4) + 4 * r;
                    if (ok && c < wq) P[(q0 + c) * PLD + rr] = acc[r];
                }
            }
            __syncthreads();
            STAMP(3);
            // (3) second half of the block column by the first
            if (q0 == 0 && jb > 16) {
                const int ns3 = (M - 16 + 15) / 16;
                for (int st = w; st < ns3; st += PT / 64) {
                    const int rr = 16 + 16 * st + (lane & 15);
                    const bool ok = rr < M;
                    d4 acc = {0, 0, 0, 0};
                    #pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        const int k = 4 * u + (lane >> 4);
                        const double a = ok ? P[k * PLD + rr] : 0.0;
                        acc = mma(P[k * PLD + 16 + (lane & 15)], a, acc);
                    }
                    #pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int c = (lane >> 4) + 4 * r;
                        if (ok && 16 + c < jb) P[(16 + c) * PLD + rr] -= acc[r];
                    }
                }
                __syncthreads();
                STAMP(4);
            }
        }
        // ---- write back (lower part); the next update reads it from L2
        #pragma unroll 8
        for (int c = 0; c < PB; ++c)
            if (c < jb && lr < M && lr >= c) A[(c0 + lr) + (i64)(c0 + c) * lda] = P[c * PLD + lr];
        __syncthreads();
        STAMP(5);
    }
#undef STAMP
    if (prof && tid == 0) {
        for (int i = 0; i < 6; ++i) prof[i] = ph[i];
        prof[6] = clock64() - t0;
        prof[7] = wall_clock64() - w0;
    }
    if (tid == 0 && s_fail && info)
        atomicCAS(reinterpret_cast<unsigned long long*>(info), 0ull, (unsigned long long)(s_fail + info_off));
}

// ---------------------------------------------------------------- tri_inv32
// Winv[b] (32 x 32, column-major, zero above the diagonal) = inv(L_bb).
__global__ void __launch_bounds__(64)
tri_inv32_kernel(int n, const double* __restrict__ L, i64 ldl, double* __restrict__ Winv, bool unit,
                 const int* gate) {
    if (gate && *gate == 0) return;
    __shared__ double S[32][33];            // S[r][c] = L(c0 + r, c0 + c)
    const int b = blockIdx.x, c0 = 32 * b, jb = min(32, n - c0), t = threadIdx.x;
    if (t < 32) {
        #pragma unroll 8
        for (int c = 0; c < 32; ++c) {
            double v = (t == c) ? 1.0 : 0.0;
            if (t < jb && c < jb && t >= c && !(unit && t == c)) v = L[(c0 + t) + (i64)(c0 + c) * ldl];
            S[t][c] = v;
        }
    }
    __syncthreads();
    if (t >= 32) return;
    const int c = t;                          // column of the inverse
    double x[32];
    #pragma unroll
    for (int r = 0; r < 32; ++r) {
        double acc = (r == c) ? 1.0 : 0.0;
        #pragma unroll
        for (int l = 0; l < r; ++l)
            if (l >= c) acc -= S[r][l] * x[l];
        x[r] = (r >= c) ? acc / S[r][r] : 0.0;
    }
    double* W = Winv + (i64)b * 1024;
    #pragma unroll
    for (int r = 0; r < 32; ++r) W[r + 32 * c] = x[r];
}

// ---------------------------------------------------------------- trsm_rlt
// X L^T = alpha B (B: m x n, L: n x n lower), X overwrites B.  Eight waves
// per 64-row block: wave (s, t) owns rows 16 s.. and, of each 32-column
// block, the 16 columns 16 t..: twice the waves of one-wave-per-strip, so
// each SIMD has four to hide the operand latency of the long K loops.
constexpr int TBM = 64;
__global__ void __launch_bounds__(512)
trsm_rlt_kernel(i64 m, int n, double alpha, const double* __restrict__ L, i64 ldl, const double* __restrict__ Winv,
                double* __restrict__ B, i64 ldb, const int* gate) {
    if (gate && *gate == 0) return;
    // row pitch = 16 mod 32 doubles: the two k rows of one ds_read_b64 lane
    // group land in opposite bank halves (an odd pitch left 2-way conflicts:
    // 33 % of LDS cycles, profiles/pmc_hot_kernels.md)
    __shared__ double R[32][TBM + 16];      // R[c][r]
    const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform (SGPR): w-derived branches stay scalar
    const int st = w & 3, tt = w >> 2;       // row strip, column tile
    const i64 r0 = (i64)blockIdx.x * TBM;
    const int mr = (int)min((i64)TBM, m - r0);
    const int ml = 16 * st + (lane & 15);    // this lane's row within the block (MFMA m index)
    const i64 rx = r0 + min(ml, mr - 1);     // clamped (valid) row for loads
    for (int c0 = 0; c0 < n; c0 += 32) {
        const int jb = min(32, n - c0);
        d4 acc1[1][1] = {{d4{0, 0, 0, 0}}};
        if (c0 > 0) {
            const int xr[1] = {(int)(rx - r0)};
            const int yr[1] = {min(16 * tt + (lane & 15), n - 1 - c0)};
            strip_update<1, 1, 8>(acc1, B + r0, xr, ldb, L + c0, yr, ldl, c0, lane);
        }
        #pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int c = 16 * tt + (lane >> 4) + 4 * r;
            double v = 0.0;
            if (ml < mr && c < jb) v = alpha * B[(r0 + ml) + (i64)(c0 + c) * ldb] - acc1[0][0][r];
            R[c][ml] = v;
        }
        __syncthreads();
        // X_J(:, tile tt) = R inv(L_JJ)^T
        const double* W = Winv + (i64)(c0 / 32) * 1024;
        d4 x = {0, 0, 0, 0};
        #pragma unroll
        for (int k = 0; k < 32; k += 4) {
            const int kk = k + (lane >> 4);
            x = mma(W[(16 * tt + (lane & 15)) + 32 * kk], R[kk][ml], x);
        }
        #pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int c = 16 * tt + (lane >> 4) + 4 * r;
            if (ml < mr && c < jb) B[(r0 + ml) + (i64)(c0 + c) * ldb] = x[r];
        }
        __syncthreads();
    }
}

// ---------------------------------------------------------------- trsm_rlt_ks
// The same solve with the K range of every strip update split over KS waves
// (partial sums reduced through LDS) and RS = 8 / (2 KS) row strips of 16
// per workgroup: per-step latency, not flops, bounds the whole-width kernel
// above (a 64-row block walks n / 32 steps whose strip updates are chains
// of K / 32 dependent load -> MFMA rounds: ~150 us at n = 512 for ANY
// m <= 16384 on MI355X, tools/r5/trsm_probe.py), so a KS-way split shortens
// every chain KS times and the grid holds KS times as many workgroups.
template <int KS>
__global__ void __launch_bounds__(512, 2)
trsm_rlt_ks_kernel(i64 m, int n, double alpha, const double* __restrict__ L, i64 ldl,
                   const double* __restrict__ Winv, double* __restrict__ B, i64 ldb, const int* gate) {
    constexpr int RS = 4 / KS, BM = 16 * RS;
    if (gate && *gate == 0) return;
    __shared__ double R[32][BM + 16];                       // R[c][r] (pitch 16 mod 32, see above)
    __shared__ d4 red[KS > 1 ? (KS - 1) * RS * 2 : 1][64];  // partial sums of the waves kh > 0
    const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int st = w % RS, tt = (w / RS) & 1, kh = w / (2 * RS);
    const i64 r0 = (i64)blockIdx.x * BM;
    const int mr = (int)min((i64)BM, m - r0);
    const int ml = 16 * st + (lane & 15);
    const i64 rx = r0 + min(ml, mr - 1);
    for (int c0 = 0; c0 < n; c0 += 32) {
        const int jb = min(32, n - c0);
        d4 acc1[1][1] = {{d4{0, 0, 0, 0}}};
        if (c0 > 0) {
            // this wave's share of K = c0, in whole 32-wide chunks (strip_update
            // with U = 8 consumes k in steps of 32)
            const int nc = c0 / 32, k0 = 32 * ((nc * kh) / KS), k1 = 32 * ((nc * (kh + 1)) / KS);
            if (k1 > k0) {
                const int xr[1] = {(int)(rx - r0)};
                const int yr[1] = {min(16 * tt + (lane & 15), n - 1 - c0)};
                strip_update<1, 1, 8>(acc1, B + r0 + (i64)k0 * ldb, xr, ldb, L + c0 + (i64)k0 * ldl, yr, ldl,
                                      k1 - k0, lane);
            }
        }
        if (KS > 1) {
            if (kh > 0) red[((kh - 1) * 2 + tt) * RS + st][lane] = acc1[0][0];
            __syncthreads();
            if (kh == 0) {
                #pragma unroll
                for (int h = 1; h < KS; ++h) {
                    const d4 v = red[((h - 1) * 2 + tt) * RS + st][lane];
                    #pragma unroll
                    for (int r = 0; r < 4; ++r) acc1[0][0][r] += v[r];
                }
            }
        }
        if (kh == 0) {
            #pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int c = 16 * tt + (lane >> 4) + 4 * r;
                double v = 0.0;
                if (ml < mr && c < jb) v = alpha * B[(r0 + ml) + (i64)(c0 + c) * ldb] - acc1[0][0][r];
                R[c][ml] = v;
            }
        }
        __syncthreads();
        if (kh == 0) {
            const double* W = Winv + (i64)(c0 / 32) * 1024;
            d4 x = {0, 0, 0, 0};
            #pragma unroll
            for (int k = 0; k < 32; k += 4) {
                const int kk = k + (lane >> 4);
                x = mma(W[(16 * tt + (lane & 15)) + 32 * kk], R[kk][ml], x);
            }
            #pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int c = 16 * tt + (lane >> 4) + 4 * r;
                if (ml < mr && c < jb) B[(r0 + ml) + (i64)(c0 + c) * ldb] = x[r];
            }
        }
        __syncthreads();
    }
}

// ---------------------------------------------------------------- trsm_lln
// L X = alpha B (L: m x m lower, B: m x n), X overwrites B -- the U rows of
// LU (L unit lower) and the forward solves.  Every workgroup owns 64 columns
// of B and walks 32-row blocks: R = alpha B_I - L_{I,<I} X_{<I} (MFMA,
// K = 32 I, the solved rows re-read from L2), X_I = inv(L_II) R (MFMA
// against tri_inv32's output).  One launch instead of the inverse + GEMM +
// copy chain of trsm.hip.
constexpr int TBN = 64;
__global__ void __launch_bounds__(256)
trsm_lln_kernel(int m, i64 n, double alpha, const double* __restrict__ L, i64 ldl, const double* __restrict__ Winv,
                double* __restrict__ B, i64 ldb) {
    __shared__ double R[32][TBN + 16];      // R[i][c] (pitch: see trsm_rlt_kernel)
    const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform (SGPR): w-derived branches stay scalar
    const i64 cb = (i64)blockIdx.x * TBN;
    const int nc = (int)min((i64)TBN, n - cb);
    const int cl = 16 * w + (lane & 15);     // this lane's column (MFMA m index)
    const int cx = min(cl, nc - 1);          // clamped (valid) column for loads
    double* Bc = B + cb * ldb;
    for (int r0 = 0; r0 < m; r0 += 32) {
        const int jb = min(32, m - r0);
        d4 acc2[1][2] = {{d4{0, 0, 0, 0}, d4{0, 0, 0, 0}}};
        if (r0 > 0) {
            const int xr[1] = {(int)(cx * ldb)};
            const int yr[2] = {min(lane & 15, m - 1 - r0), min(16 + (lane & 15), m - 1 - r0)};
            strip_update<1, 2, 8>(acc2, Bc, xr, 1, L + r0, yr, ldl, r0, lane);
        }
        d4 (&acc)[2] = acc2[0];
        #pragma unroll
        for (int t = 0; t < 2; ++t)
            #pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int i = 16 * t + (lane >> 4) + 4 * q;
                double v = 0.0;
                if (cl < nc && i < jb) v = alpha * Bc[(r0 + i) + (i64)cl * ldb] - acc[t][q];
                R[i][cl] = v;
            }
        __syncthreads();
        // X_I = inv(L_II) R
        const double* W = Winv + (i64)(r0 / 32) * 1024;
        d4 x[2] = {d4{0, 0, 0, 0}, d4{0, 0, 0, 0}};
        #pragma unroll
        for (int k = 0; k < 32; k += 4) {
            const int kk = k + (lane >> 4);
            const double rv = R[kk][cl];
            #pragma unroll
            for (int t = 0; t < 2; ++t) x[t] = mma(W[(16 * t + (lane & 15)) + 32 * kk], rv, x[t]);
        }
        #pragma unroll
        for (int t = 0; t < 2; ++t)
            #pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int i = 16 * t + (lane >> 4) + 4 * q;
                if (cl < nc && i < jb) Bc[(r0 + i) + (i64)cl * ldb] = x[t][q];
            }
        __syncthreads();
    }
}

// ---------------------------------------------------------------- launchers
// SLATE_AMD_POTRF_TILE=lds: the one-CU kernel above; default: the
// multi-workgroup blocked kernel of potrf_mc.hip
static bool tile_mc() {
    static const bool mc = [] {
        const char* e = std::getenv("SLATE_AMD_POTRF_TILE");
        return !(e && std::strcmp(e, "lds") == 0);
    }();
    return mc;
}

bool potrf_fast(int n, double* A, i64 lda, i64* info, i64 info_off, hipStream_t s, const int* gate,
                const double* floorp) {
    if (n <= 0 || n > PN) return false;
    if (tile_mc()) return potrf_mc(n, A, lda, info, info_off, s, gate, floorp);
    return potrf_lds(n, A, lda, info, info_off, s, gate, floorp);
}

bool potrf_lds(int n, double* A, i64 lda, i64* info, i64 info_off, hipStream_t s, const int* gate,
               const double* floorp) {
    if (n <= 0 || n > PN) return false;
    hipLaunchKernelGGL(potrf_lds_kernel, dim3(1), dim3(PT), 0, s, n, A, lda, info, info_off, (i64*)nullptr, gate,
                       floorp);
    HIP_LAUNCH_CHECK();
    return true;
}

// tools: phase totals (shader clocks: load, update, diag, solve, half, writeback,
// total) and wall-clock ticks (100 MHz) of one potrf_lds launch
void potrf_lds_profile(int n, double* A, i64 lda, i64* info, i64* prof, hipStream_t s) {
    hipLaunchKernelGGL(potrf_lds_kernel, dim3(1), dim3(PT), 0, s, n, A, lda, info, (i64)0, prof, (const int*)nullptr,
                       (const double*)nullptr);
    HIP_LAUNCH_CHECK();
}

bool trsm_rlt_fast(i64 m, i64 n, double alpha, const double* L, i64 ldl, double* B, i64 ldb, bool unit,
                   hipStream_t s, const int* gate) {
    if (m <= 0 || n <= 0) return true;
    if (n > 1024) return false;
    const int nbj = (int)((n + 31) / 32);
    double* W = static_cast<double*>(workspace(s, sizeof(double) * (size_t)nbj * 1024, WS_C));
    hipLaunchKernelGGL(tri_inv32_kernel, dim3(nbj), dim3(64), 0, s, (int)n, L, ldl, W, unit, gate);
    HIP_LAUNCH_CHECK();
    // K splits of the strip updates (1: the whole-width kernel, 64-row
    // blocks; 2: 32-row blocks; 4: 16-row blocks).  Default by m, measured
    // alone at n = 512 (tools/r5/trsm_probe.py, profiles/r5/trsm_ks.txt):
    // m = 4096: 185 / 131 / 99 us, 8192: 175 / 121 / 123, 16384: 185 / 185
    // / 221, 32256: 309 / 334 / 410.  SLATE_AMD_TRSM_KS=1|2|4 overrides.
    const int ks = [m] {      // read per launch: tests toggle it
        const char* e = std::getenv("SLATE_AMD_TRSM_KS");
        const int v = e ? std::atoi(e) : (m <= 6144 ? 4 : m <= 12288 ? 2 : 1);
        return (v == 2 || v == 4) ? v : 1;
    }();
    if (ks == 2)
        hipLaunchKernelGGL(trsm_rlt_ks_kernel<2>, dim3((unsigned)((m + 31) / 32)), dim3(512), 0, s, m, (int)n, alpha,
                           L, ldl, (const double*)W, B, ldb, gate);
    else if (ks == 4)
        hipLaunchKernelGGL(trsm_rlt_ks_kernel<4>, dim3((unsigned)((m + 15) / 16)), dim3(512), 0, s, m, (int)n, alpha,
                           L, ldl, (const double*)W, B, ldb, gate);
    else
        hipLaunchKernelGGL(trsm_rlt_kernel, dim3((unsigned)((m + TBM - 1) / TBM)), dim3(512), 0, s, m, (int)n, alpha,
                           L, ldl, (const double*)W, B, ldb, gate);
    HIP_LAUNCH_CHECK();
    return true;
}

// L X = alpha B for m <= 64 rows (the bottom levels of the recursive LU
// panel: 32 x 32 and 64 x 64 solves), ONE launch and no triangular inverse:
// four lanes per right-hand side column hold its rows q, q + 4, ... in
// registers; x_k is broadcast inside the quad by a DPP quad_perm (k is a
// compile-time index of the unrolled loop) and L comes from LDS.  Replaces
// tri_inv32 + trsm_lln (~28 us per call at these sizes).
template <int CTRL>
__device__ inline double qbcast(double x) {
    const unsigned long long u = __builtin_bit_cast(unsigned long long, x);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)(u & 0xffffffffu), CTRL, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(u >> 32), CTRL, 0xF, 0xF, false);
    return __builtin_bit_cast(double, ((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}
template <int K, int RPT>
__device__ inline void small_lln_step(double (&b)[RPT], int q, int m, const double (*Ls)[65], bool unit) {
    if constexpr (K < 4 * RPT) {
        if (K < m) {
            constexpr int own = K & 3, reg = K >> 2;
            if (!unit && q == own) b[reg] = b[reg] / Ls[K][K];
            const double xk = qbcast<own * 0x55>(b[reg]);   // quad_perm [own, own, own, own]
            #pragma unroll
            for (int r = 0; r < RPT; ++r) {
                const int i = q + 4 * r;
                if (i > K && i < m) b[r] = fma(-Ls[i][K], xk, b[r]);
            }
            small_lln_step<K + 1, RPT>(b, q, m, Ls, unit);
        }
    }
}
__global__ void __launch_bounds__(256)
trsm_lln_small_kernel(int m, i64 n, double alpha, const double* __restrict__ L, i64 ldl, double* __restrict__ B,
                      i64 ldb, int unit) {
    __shared__ double Ls[64][65];
    const int tid = threadIdx.x;
    for (int e = tid; e < m * m; e += 256) {
        const int i = e % m, k = e / m;
        Ls[i][k] = (i >= k) ? L[i + (i64)k * ldl] : 0.0;
    }
    __syncthreads();
    constexpr int RPT = 16;
    const i64 c = (i64)blockIdx.x * 64 + (tid >> 2);
    const int q = tid & 3;
    const bool col = c < n;
    double b[RPT];
    #pragma unroll
    for (int r = 0; r < RPT; ++r) {
        const int i = q + 4 * r;
        b[r] = (col && i < m) ? alpha * B[i + c * ldb] : 0.0;
    }
    small_lln_step<0, RPT>(b, q, m, Ls, unit != 0);
    if (!col) return;
    #pragma unroll
    for (int r = 0; r < RPT; ++r) {
        const int i = q + 4 * r;
        if (i < m) B[i + c * ldb] = b[r];
    }
}

bool trsm_lln_fast(i64 m, i64 n, double alpha, const double* L, i64 ldl, double* B, i64 ldb, bool unit,
                   hipStream_t s) {
    if (m <= 0 || n <= 0) return true;
    if (m > 1024) return false;
    if (m <= 64) {
        hipLaunchKernelGGL(trsm_lln_small_kernel, dim3((unsigned)((n + 63) / 64)), dim3(256), 0, s, (int)m, n, alpha,
                           L, ldl, B, ldb, unit ? 1 : 0);
        HIP_LAUNCH_CHECK();
        return true;
    }
    const int nbj = (int)((m + 31) / 32);
    double* W = static_cast<double*>(workspace(s, sizeof(double) * (size_t)nbj * 1024, WS_C));
    hipLaunchKernelGGL(tri_inv32_kernel, dim3(nbj), dim3(64), 0, s, (int)m, L, ldl, W, unit, (const int*)nullptr);
    HIP_LAUNCH_CHECK();
    hipLaunchKernelGGL(trsm_lln_kernel, dim3((unsigned)((n + TBN - 1) / TBN)), dim3(256), 0, s, (int)m, n, alpha, L,
                       ldl, (const double*)W, B, ldb);
    HIP_LAUNCH_CHECK();
    return true;
}

}  // namespace slate_hip
