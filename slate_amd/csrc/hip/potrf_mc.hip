// Multi-workgroup fp64 tile Cholesky (n <= 512) for gfx950 -- the diagonal
// tile of the distributed potrf (reference: src/internal/internal_potrf.cc:56-81,
// a vendor lapack::potrf call per tile) and the Gram factor of the
// CholeskyQR panel (qr_fast.hip).
//
// potrf_lds (chol_fast.hip) factors a 512 tile on ONE compute unit; its
// left-looking update alone is n^3/3 flops on one CU's matrix core
// (>= 145 us at the fp64 MFMA peak), so it cannot go below ~150 us however it
// is tuned, and the 8-GPU factorization has 64 of them in a chain.  Here the
// tile is cut into 64 x 64 blocks and factored right-looking by two kinds of
// launches per block step k (at most 2 nbk - 1 launches):
//
//   P_k  workgroup 0: Cholesky of A_kk (64 x 64).  Row = lane, each of the
//        four waves keeps 16 columns in registers; two columns are
//        eliminated per step (2 x 2 pivot block, rank-2 update) with one
//        workgroup barrier, the owner of the next pair updating and
//        factoring it before the bulk update (one-step lookahead).  Then
//        the four waves invert the four 16 x 16 diagonal blocks of L_kk
//        (one column per lane, forward substitution) into a workspace.
//        workgroups 1..: the solve of the PREVIOUS panel, A_{i,k-1} L^-T,
//        for every block row i >= k (stored; see U).
//   U_k  one workgroup per trailing block (i, j), k < j <= i: each of the
//        four waves solves its 16-row strip of X_i = A_ik L_kk^-T (and X_j)
//        in registers -- blocked substitution, 16-column blocks, every
//        product on the f64 MFMA against the 16 x 16 inverses -- then
//        A_ij -= X_i X_j^T (MFMA, X_j exchanged through LDS).  The solved
//        panel is NOT written here (other workgroups of the launch still
//        read A_ik); P_{k+1} writes it.
//
// Critical path per step: P (64-column elimination + inverses) -> U of the
// block (k+1, k+1) -> P_{k+1}.  Optional gate (device predicate, 0 = skip
// the launch) and pivot floor (regularised Cholesky: pivots <= *floor are
// replaced by *floor) serve the CholeskyQR fallback of qr_fast.hip.
#include <cstdlib>
#include <cstring>
#include "common.hpp"
#include "kernels.hpp"
#include "workspace.hpp"

namespace slate_hip {

namespace {
constexpr int PB = 64;                   // block size
constexpr int LDL = 80;                  // LDS pitch (doubles): 2 * 80 = 32 (mod 64) -> conflict-free fragments
constexpr int NTH = 256;                 // threads (4 waves)

__device__ inline d4 mma(double x, double y, d4 c) { return __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, c, 0, 0, 0); }

__device__ inline double rsq64(double d) {
    double r = __builtin_amdgcn_rsq(d);
    r = r * (1.5 - 0.5 * d * r * r);
    return r * (1.5 - 0.5 * d * r * r);
}

__device__ inline double rdlane(double v, int lane) {
    const unsigned long long u = __builtin_bit_cast(unsigned long long, v);
    const unsigned lo = __builtin_amdgcn_readlane((unsigned)u, lane);
    const unsigned hi = __builtin_amdgcn_readlane((unsigned)(u >> 32), lane);
    return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}

// Ls (col-major, pitch LDL) <- lower part of the factored block L (64 x 64,
// rows/cols >= kb: identity), Is <- the four 16 x 16 inverses (col-major).
// (kb = 64 here: every factored block except the last, which nobody loads).
// All 20 loads per thread are issued before the first LDS store.
__device__ inline void load_factor(const double* __restrict__ L, i64 lda, int kb, const double* __restrict__ Winv,
                                   double* Ls, double* Is, int tid) {
    double v[PB * PB / NTH], iv[4];
    const int r = tid & 63, c0 = tid >> 6;        // column c0 + 4 q
    #pragma unroll
    for (int q = 0; q < PB * PB / NTH; ++q) v[q] = L[r + (i64)(c0 + 4 * q) * lda];
    #pragma unroll
    for (int q = 0; q < 4; ++q) iv[q] = Winv[tid + q * NTH];
    #pragma unroll
    for (int q = 0; q < PB * PB / NTH; ++q) {
        const int c = c0 + 4 * q;
        Ls[c * LDL + r] = (r >= c && r < kb && c < kb) ? v[q] : (r == c ? 1.0 : 0.0);
    }
    #pragma unroll
    for (int q = 0; q < 4; ++q) Is[tid + q * NTH] = iv[q];
}

// Prefetch of a 64-row block strip in the MFMA accumulator layout: wave w,
// lane l, tile J, reg r holds B(16 w + (l & 15), 16 J + (l >> 4) + 4 r);
// rows >= mrows and columns >= ncols read as zero.  All 16 loads issue at
// once (the kernels are latency-bound: one dependent load per tile costs a
// full L2 / HBM round trip each).
__device__ inline void strip_load(d4 (&V)[4], const double* __restrict__ B, i64 ldb, int mrows, int ncols, int w,
                                  int lane) {
    const int m = 16 * w + (lane & 15), kq = lane >> 4;
    #pragma unroll
    for (int J = 0; J < 4; ++J)
        #pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int c = 16 * J + kq + 4 * r;
            V[J][r] = (m < mrows && c < ncols) ? B[m + (i64)c * ldb] : 0.0;
        }
}

// One wave: X (rows 16 w .., all 64 columns) = B L^-T with B preloaded
// (strip_load): blocked substitution over 16-column blocks, R_J = B_J -
// X_{<J} L_{J,<J}^T and X_J = R_J inv(L_JJ)^T, every product on the f64
// MFMA.  X[J] has the accumulator layout of B.
__device__ inline void strip_solve(d4 (&X)[4], const d4 (&Bv)[4], int lane, const double* Ls, const double* Is) {
    const int kq = lane >> 4;
    #pragma unroll
    for (int J = 0; J < 4; ++J) {
        d4 S = {0, 0, 0, 0};
        #pragma unroll
        for (int I = 0; I < J; ++I)
            #pragma unroll
            for (int s = 0; s < 4; ++s)
                S = mma(Ls[(16 * I + 4 * s + kq) * LDL + 16 * J + (lane & 15)], X[I][s], S);
        d4 R;
        #pragma unroll
        for (int r = 0; r < 4; ++r) R[r] = Bv[J][r] - S[r];
        d4 Y = {0, 0, 0, 0};
        #pragma unroll
        for (int s = 0; s < 4; ++s) Y = mma(Is[J * 256 + (4 * s + kq) * 16 + (lane & 15)], R[s], Y);
        X[J] = Y;
    }
}

// C (strip, accumulator layout) -= X_i X_j^T with X_j (all 64 rows) in LDS
// Xq (col-major, pitch LDL)
__device__ inline void strip_syrk(d4 (&C)[4], const d4 (&Xi)[4], const double* Xq, int lane) {
    const int kq = lane >> 4;
    #pragma unroll
    for (int T = 0; T < 4; ++T) {
        d4 S = {0, 0, 0, 0};
        #pragma unroll
        for (int K = 0; K < 4; ++K)
            #pragma unroll
            for (int s = 0; s < 4; ++s)
                S = mma(Xq[(16 * K + 4 * s + kq) * LDL + 16 * T + (lane & 15)], Xi[K][s], S);
        #pragma unroll
        for (int r = 0; r < 4; ++r) C[T][r] -= S[r];
    }
}

// X (strip of wave w, accumulator layout) -> LDS, col-major pitch LDL
__device__ inline void strip_to_lds(double* Xq, const d4 (&X)[4], int w, int lane) {
    #pragma unroll
    for (int J = 0; J < 4; ++J)
        #pragma unroll
        for (int r = 0; r < 4; ++r) Xq[(16 * J + (lane >> 4) + 4 * r) * LDL + 16 * w + (lane & 15)] = X[J][r];
}
}  // namespace

// ---------------------------------------------------------------- step k
// Workgroups of launch k (k = 0 .. nbk; launch nbk only stores the last
// panel):
//   [0]            k < nbk: A_kk -= X_k X_k^T (panel k-1, k >= 1), then the
//                  Cholesky of A_kk and the inverses of its 16 x 16 blocks;
//   [1, 1 + nS)    k >= 2: store the solved panel k-2, block row k-1+b;
//   [1 + nS, ...)  1 <= k < nbk: A_ij -= X_i X_j^T by panel k-1 for the
//                  blocks k <= j <= i < nbk other than (k, k).
// Panel k-1 is read unsolved by this launch (X recomputed where needed), so
// it is stored solved only by launch k+1.
__global__ void __launch_bounds__(NTH, 1)
potrf_mc_step_kernel(int n, double* __restrict__ A, i64 lda, int k, double* __restrict__ W, i64* info, i64 info_off,
                     const int* gate, const double* floorp, i64* prof) {
    if (gate && *gate == 0) return;
    // tools only (prof != nullptr): 100 MHz wall-clock stamps per phase
#define PSTAMP(i) do { if (prof && threadIdx.x == 0) prof[k * 512 + blockIdx.x * 8 + (i)] = wall_clock64(); } while (0)
    PSTAMP(0);
    __shared__ double Ls[PB * LDL];          // L of panel p, then X_j / A_kk
    __shared__ double Is[4 * 256];
    __shared__ double2 pb[2][PB];
    __shared__ int sfail;
    const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform (SGPR): w-derived branches stay scalar
    const int nbk = (n + PB - 1) / PB;
    const int nS = (k >= 2) ? nbk - (k - 1) : 0;
    const int b = blockIdx.x;
    const int has0 = k < nbk ? 1 : 0;
    if (b >= has0 && b < has0 + nS) {
        // ---- store the solved panel k-2, block row i
        const int pp = k - 2, i = pp + 1 + (b - has0);
        const int c0 = PB * pp, r0 = PB * i;
        const int mrows = min(PB, n - r0);
        double* B = A + r0 + (i64)c0 * lda;
        d4 Bv[4];
        strip_load(Bv, B, lda, mrows, PB, w, lane);
        load_factor(A + c0 + (i64)c0 * lda, lda, PB, W + (i64)pp * 1024, Ls, Is, tid);
        __syncthreads();
        PSTAMP(1);
        d4 X[4];
        strip_solve(X, Bv, lane, Ls, Is);
        PSTAMP(2);
        const int m = 16 * w + (lane & 15);
        if (m < mrows) {
            #pragma unroll
            for (int J = 0; J < 4; ++J)
                #pragma unroll
                for (int r = 0; r < 4; ++r) B[m + (i64)(16 * J + (lane >> 4) + 4 * r) * lda] = X[J][r];
        }
        return;
    }
    // ---- update of block (i, j) by panel p = k-1 (WG 0: the block (k, k))
    int i = k, j = k;
    if (b > 0) {
        const int t = b - has0 - nS + 1;             // triangle index over k <= j <= i, (k, k) = 0
        int ii = (int)((sqrtf(8.0f * t + 1.0f) - 1.0f) * 0.5f);
        while ((ii + 1) * (ii + 2) / 2 <= t) ++ii;
        while (ii * (ii + 1) / 2 > t) --ii;
        i = k + ii;
        j = k + (t - ii * (ii + 1) / 2);
    }
    const int ri = PB * i, rj = PB * j;
    const int mi = min(PB, n - ri), mj = min(PB, n - rj);
    d4 C[4];
    strip_load(C, A + ri + (i64)rj * lda, lda, mi, mj, w, lane);
    if (k >= 1) {
        const int p = k - 1, c0 = PB * p;
        d4 Bi[4], Bj[4];
        strip_load(Bi, A + ri + (i64)c0 * lda, lda, mi, PB, w, lane);
        if (i != j) strip_load(Bj, A + rj + (i64)c0 * lda, lda, mj, PB, w, lane);
        load_factor(A + c0 + (i64)c0 * lda, lda, PB, W + (i64)p * 1024, Ls, Is, tid);
        __syncthreads();
        PSTAMP(1);
        d4 Xi[4], Xj[4];
        strip_solve(Xi, Bi, lane, Ls, Is);
        if (i != j) strip_solve(Xj, Bj, lane, Ls, Is);
        PSTAMP(2);
        __syncthreads();                         // every wave done reading L_p
        strip_to_lds(Ls, i != j ? Xj : Xi, w, lane);
        __syncthreads();
        strip_syrk(C, Xi, Ls, lane);
        PSTAMP(3);
        if (b > 0) {
            const int m = 16 * w + (lane & 15), kq = lane >> 4;
            double* Cg = A + ri + (i64)rj * lda;
            if (m < mi) {
                #pragma unroll
                for (int T = 0; T < 4; ++T)
                    #pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int cc = 16 * T + kq + 4 * r;
                        if (cc < mj && (i != j || m >= cc)) Cg[m + (i64)cc * lda] = C[T][r];
                    }
            }
            return;
        }
        __syncthreads();                         // every wave done reading X from Ls
    }
    // ---- WG 0: Cholesky of the updated A_kk (C strips -> LDS -> columns)
    const int c0 = PB * k;
    const int kb = mi;
    double* Akk = A + c0 + (i64)c0 * lda;
    const double pfloor = floorp ? *floorp : 0.0;
    strip_to_lds(Ls, C, w, lane);
    __syncthreads();
    // wave w keeps columns 16 w .. 16 w + 15 of every row (row = lane) in
    // registers; step s eliminates columns j = 2 s, j + 1.  The owner of the
    // NEXT pair updates those two columns first, computes their pivots and
    // publishes L(:, j'), L(:, j'+1) to the other pb slot; then every wave
    // applies the rank-2 update of step s to the rest of its columns.  One
    // workgroup barrier per step.  Both pivots of a pair come from
    // independent reciprocal square roots: 1 / L(j+1, j+1) = sqrt(d0) /
    // sqrt(d0 d11 - d10^2).
    const int l = lane;
    double a[16];
    #pragma unroll
    for (int cc = 0; cc < 16; ++cc) {
        const int c = 16 * w + cc;
        a[cc] = (l < kb && c < kb) ? Ls[c * LDL + l] : (l == c ? 1.0 : 0.0);
    }
    int fail = 0;
    PSTAMP(4);
    auto pivot = [&](int jp, int jj) {
        double d0 = rdlane(a[jj], jp), d10 = rdlane(a[jj], jp + 1), d11 = rdlane(a[jj + 1], jp + 1);
        double i0, i1, l10, s0, s1;
        const double det = fma(d0, d11, -d10 * d10);
        if (d0 > pfloor && det > pfloor * d0) {
            i0 = rsq64(d0);
            const double rd = rsq64(det);           // independent of i0
            s0 = d0 * i0;
            l10 = d10 * i0;
            i1 = s0 * rd;
            s1 = det * rd * i0;                     // sqrt(det / d0)
        } else {
            if (!(d0 > pfloor)) {
                if (pfloor > 0.0) d0 = pfloor;
                else { if (!fail && jp < kb) fail = c0 + jp + 1; d0 = 1.0; }
            }
            i0 = rsq64(d0); s0 = d0 * i0; l10 = d10 * i0;
            double e = d11 - l10 * l10;
            if (!(e > pfloor)) {
                if (pfloor > 0.0) e = pfloor;
                else { if (!fail && jp + 1 < kb) fail = c0 + jp + 2; e = 1.0; }
            }
            i1 = rsq64(e); s1 = e * i1;
        }
        const double lj = a[jj] * i0;
        const double lj1 = (a[jj + 1] - lj * l10) * i1;
        if (l == jp) { a[jj] = s0; a[jj + 1] = 0.0; }
        else if (l == jp + 1) { a[jj] = l10; a[jj + 1] = s1; }
        else if (l > jp + 1) { a[jj] = lj; a[jj + 1] = lj1; }
        else { a[jj] = 0.0; a[jj + 1] = 0.0; }
        return (l > jp + 1) ? make_double2(lj, lj1) : make_double2(0.0, 0.0);
    };
    if (w == 0) pb[0][l] = pivot(0, 0);
    __syncthreads();
    #pragma unroll
    for (int st = 0; st < PB / 2; ++st) {
        const int jp = 2 * st, bb = st & 1;
#define SSTAMP(ph) do { if (prof && k == 1 && st < 24 && (tid & 63) == 0) prof[16 * 512 + (w * 24 + st) * 2 + (ph)] = clock64(); } while (0)
        SSTAMP(0);
        const double2 me = pb[bb][l];                    // L(l, jp), L(l, jp+1)
        const int jn = jp + 2;
        if (jn < PB && w == (jn >> 4)) {
            const int jj = jn & 15;
            const double2 p0 = pb[bb][jn], p1 = pb[bb][jn + 1];
            a[jj] -= me.x * p0.x + me.y * p0.y;
            a[jj + 1] -= me.x * p1.x + me.y * p1.y;
            double2 pc[16];
            #pragma unroll
            for (int cc = 0; cc < 16; ++cc)
                if (cc > jj + 1) pc[cc] = pb[bb][16 * w + cc];
            pb[bb ^ 1][l] = pivot(jn, jj);
            #pragma unroll
            for (int cc = 0; cc < 16; ++cc) {
                if (cc <= jj + 1) continue;
                a[cc] -= me.x * pc[cc].x + me.y * pc[cc].y;
            }
        } else if (16 * w + 15 > jp + 1) {
            // every read issued up front; the (wave-uniform) column mask is a
            // 0 / 1 factor, not a branch -- a branch per column made the
            // compiler sink each LDS read into it and wait for it alone
            double2 pc[16];
            #pragma unroll
            for (int cc = 0; cc < 16; ++cc) pc[cc] = pb[bb][16 * w + cc];
            #pragma unroll
            for (int cc = 0; cc < 16; ++cc) {
                const double f = (16 * w + cc > jp + 1) ? 1.0 : 0.0;
                a[cc] -= f * (me.x * pc[cc].x + me.y * pc[cc].y);
            }
        }
        SSTAMP(1);
        __syncthreads();
#undef SSTAMP
    }
    PSTAMP(5);
    // L (lower) -> tile and LDS copy (for the inverses)
    #pragma unroll
    for (int cc = 0; cc < 16; ++cc) {
        const int c = 16 * w + cc;
        const double v = (c <= l) ? a[cc] : 0.0;
        Ls[c * LDL + l] = v;
        if (l < kb && c < kb && c <= l) Akk[l + (i64)c * lda] = v;
    }
    // first failing column over the waves, then one CAS (a later step may
    // already have recorded an earlier tile's failure: keep that)
    if (tid == 0) sfail = 0x7fffffff;
    __syncthreads();
    if (fail && lane == 0) atomicMin(&sfail, fail);
    __syncthreads();
    if (tid == 0 && sfail != 0x7fffffff && info)
        atomicCAS(reinterpret_cast<unsigned long long*>(info), 0ull, (unsigned long long)(sfail + info_off));
    // inverse of diagonal block w: lane c < 16 computes column c (the 64
    // diagonal reciprocals first, one division per lane, so the
    // substitution chain multiplies)
    __shared__ double rdg[PB];
    if (tid < PB) rdg[tid] = 1.0 / Ls[tid * LDL + tid];
    __syncthreads();
    if (lane < 16) {
        const int c = lane, o = 16 * w;
        double x[16];
        #pragma unroll
        for (int r = 0; r < 16; ++r) {
            double acc = (r == c) ? 1.0 : 0.0;
            #pragma unroll
            for (int q = 0; q < r; ++q) acc -= Ls[(o + q) * LDL + o + r] * x[q];
            x[r] = (r >= c) ? acc * rdg[o + r] : 0.0;
        }
        double* Wo = W + (i64)k * 1024 + w * 256;
        #pragma unroll
        for (int r = 0; r < 16; ++r) Wo[c * 16 + r] = x[r];
    }
    PSTAMP(6);
#undef PSTAMP
}

// ---------------------------------------------------------------- launcher
// tools: per-launch / per-workgroup phase stamps (<= 9 launches x 64 WGs x 8)
static i64* g_prof = nullptr;
void potrf_mc_set_prof(i64* p) { g_prof = p; }

bool potrf_mc(int n, double* A, i64 lda, i64* info, i64 info_off, hipStream_t s, const int* gate,
              const double* floorp) {
    if (n <= 0 || n > 512) return false;
    const int nbk = (n + PB - 1) / PB;
    double* W = static_cast<double*>(workspace(s, sizeof(double) * (size_t)nbk * 1024, WS_PM));
    for (int k = 0; k <= nbk; ++k) {
        const int has0 = k < nbk ? 1 : 0;
        const int nS = (k >= 2) ? nbk - (k - 1) : 0;
        const int r = nbk - k;
        const int nU = (k >= 1 && k < nbk) ? r * (r + 1) / 2 - 1 : 0;
        const int g = has0 + nS + nU;
        if (g == 0) continue;
        hipLaunchKernelGGL(potrf_mc_step_kernel, dim3(g), dim3(NTH), 0, s, n, A, lda, k, W, info, info_off, gate,
                           floorp, g_prof);
        HIP_LAUNCH_CHECK();
    }
    return true;
}

}  // namespace slate_hip
