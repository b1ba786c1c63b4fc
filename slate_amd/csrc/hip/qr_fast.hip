// Tall-panel fp64 QR on gfx950: shifted CholeskyQR3 + Householder
// reconstruction.  The output has exactly the form of the recursive
// Householder panel of geqrf.hip -- R on/above the diagonal, unit-lower
// reflectors below it, tau, the compact-WY T and the explicit V -- so the
// trailing update, unmqr and every other consumer of geqrf_panel_ws are
// unchanged.
//
//   CholeskyQR2 (shifted CholeskyQR3 when the second factor shows that the
//   first pass did not reach orthogonality):
//       G = A^T A (+ s I)        split-K MFMA GEMM (gemm_launch.hpp)
//       G = L L^T                potrf_lds, one CU (chol_fast.hip)
//       A = A L^-T               trsm_rlt (chol_fast.hip)
//       R = L^T R                trmm
//   Householder reconstruction of the orthonormal Q (m x b):
//       Q1 - S = Y1 U            LU without pivoting, s_j = -sign(u_jj)
//                                (every |u_jj| >= 1), lu_hr below, one CU
//       Y2 = Q2 U^-1             trsm_rlt against U^T
//       T  = -U S Y1^-T          trsm_rlt against the unit-lower Y1
//       R <- S R, V = [Y1; Y2], tau = diag(T)
// The column-by-column Householder panel is latency-bound (two grid-wide
// launches per column, each re-reading the panel); this one is GEMM-shaped:
// a handful of launches that stream the panel ~8 times.
//
// The reference has no such panel: its geqrf panel is host Householder
// (src/geqrf.cc:96-160 -> internal::geqrf, src/internal/Tile_geqrf.hh:97-330).
// Methods: shifted CholeskyQR3 (Fukaya, Kannan, Nakatsukasa, Yamamoto,
// Yanagisawa, SISC 2020); Householder reconstruction (Ballard, Demmel,
// Grigori, Jacquelin, Knight, Nguyen, IPDPS 2014).
//
// Breakdown is decided on the device, never read back to the host:
// CholeskyQR2 runs first; a check kernel sets a flag when one of its
// Cholesky factorizations failed or its second factor is not I to 1e-3.
// Every kernel of the fallback reads that flag and exits at once when it is
// 0 (a few microseconds per skipped launch).  The fallback restores the panel
// from a copy, adds a random perturbation E with ||E||_F = 10 u ||A||_F
// (within the backward error of Householder QR) and runs shifted CholeskyQR3
// with a pivot floor u tr(G) in each Cholesky: E makes an exactly
// rank-deficient panel (a zero or repeated column) full rank, the shift
// bounds the condition number of the first Q, the floor keeps the Gram
// Cholesky of nearly dependent columns finite.  Measured in double precision
// (numpy model of the same steps, 4096 x 64): zero / repeated columns,
// rank 10 and an all-zero panel all give ||Q^T Q - I|| <= 7e-14 and
// ||QR - A|| / ||A|| <= 1.2e-15; without the floor the rank-10 panel gives
// NaN, without E a zero column stays a zero column of Q.  So the panel never
// needs a host decision, and the sequence is graph-capturable.
#include <cstdlib>
#include <cstring>
#include "common.hpp"
#include "kernels.hpp"
#include "launchers.hpp"
#include "workspace.hpp"
#include "../include/philox.hpp"

namespace slate_hip {

namespace {
constexpr int HB = 256;          // widest panel of the fast path
constexpr int HT = 1024;         // threads of lu_hr
__device__ inline d4 mma_hr(double x, double y, d4 c) { return __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, c, 0, 0, 0); }
}  // namespace

// G(i, i) += c * trace(G)   (trace(A^T A) = ||A||_F^2); optionally saves the
// trace and the pivot floor u * trace for the regularised Cholesky
__global__ void __launch_bounds__(256)
qf_shift_kernel(int b, double* G, i64 ldg, double c, double* tr_out, double* floor_out, const int* gate) {
    if (gate && *gate == 0) return;
    __shared__ double red[256];
    const int t = threadIdx.x;
    double s = 0;
    for (int i = t; i < b; i += 256) s += G[i + (i64)i * ldg];
    red[t] = s;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if (t < o) red[t] += red[t + o];
        __syncthreads();
    }
    const double sh = c * red[0];
    if (t == 0 && tr_out) *tr_out = red[0];
    if (t == 0 && floor_out) *floor_out = red[0] * 0x1p-53;
    if (sh != 0.0)
        for (int i = t; i < b; i += 256) G[i + (i64)i * ldg] += sh;
}

// A = Bk + E, E(i, j) uniform in [-s, s), s = 10 u ||Bk||_F / sqrt(m b / 3)
// (so ||E||_F ~ 10 u ||Bk||_F; 10 u if Bk = 0).  *tr0 = ||Bk||_F^2.
__global__ void __launch_bounds__(256)
qf_perturb_kernel(i64 m, int b, const double* __restrict__ Bk, i64 ldk, double* __restrict__ A, i64 lda,
                  const double* tr0, const int* gate) {
    if (gate && *gate == 0) return;
    const double t = *tr0;
    const double nrm = t > 0.0 ? sqrt(t) : 1.0;
    const double sc = 10.0 * 0x1p-53 * nrm / sqrt((double)m * b / 3.0);
    const i64 i = (i64)blockIdx.x * 256 + threadIdx.x;
    if (i >= m) return;
    for (int j = blockIdx.y; j < b; j += gridDim.y) {
        double u0, u1;
        slate_rng::uniform2(0x5eedc0ffeeull, i, j, 7u, u0, u1);
        A[i + (i64)j * lda] = Bk[i + (i64)j * ldk] + sc * (2.0 * u0 - 1.0);
    }
}

// Ro = L^T R (L lower b x b in the lower part of G, R upper): one thread per
// output element, one workgroup per column
__global__ void __launch_bounds__(256)
qf_ltmul_kernel(int b, const double* __restrict__ L, i64 ldl, const double* __restrict__ R, i64 ldr,
                double* __restrict__ Ro, i64 ldo, const int* gate) {
    if (gate && *gate == 0) return;
    const int j = blockIdx.x;
    for (int i = threadIdx.x; i < b; i += 256) {
        double acc = 0.0;
        for (int k = i; k <= j; ++k) acc += L[k + (i64)i * ldl] * R[k + (i64)j * ldr];
        Ro[i + (i64)j * ldo] = (i <= j) ? acc : 0.0;
    }
}

// R = L^T (upper, zero below)
__global__ void __launch_bounds__(256)
qf_rt_kernel(int b, const double* L, i64 ldl, double* R, i64 ldr, const int* gate) {
    if (gate && *gate == 0) return;
    const int j = blockIdx.x;
    for (int i = threadIdx.x; i < b; i += 256) R[i + (i64)j * ldr] = (i <= j) ? L[j + (i64)i * ldl] : 0.0;
}

// flag = one of the npass Cholesky factorizations failed, or the last
// factor L is not I to within tol (max |L - I| over the lower triangle; NaN
// fails): the Q it produced was not yet orthonormal
__global__ void __launch_bounds__(256)
qf_check_kernel(int b, const double* L, i64 ldl, const i64* info, int npass, double tol, int* flag) {
    __shared__ int bad;
    if (threadIdx.x == 0) {
        int f = 0;
        for (int p = 0; p < npass; ++p) f |= info[p] != 0;
        bad = f;
    }
    __syncthreads();
    for (int e = threadIdx.x; e < b * b; e += 256) {
        const int i = e % b, j = e / b;
        if (i >= j && !(fabs(L[i + (i64)j * ldl] - (i == j ? 1.0 : 0.0)) < tol)) atomicOr(&bad, 1);
    }
    __syncthreads();
    if (threadIdx.x == 0) *flag = bad;
}

// LU without pivoting of Q1 - S in place (b x b, b <= 256), s_j = -sign of
// the current pivot, so u_jj = d + sign(d) and |u_jj| >= 1 (Q1 is a block of
// an orthonormal matrix: no growth).  One workgroup, per 32-column block:
//   (a) rows one per thread in registers, one barrier per column (the pivot
//       row is broadcast through LDS, double-buffered);
//   (b) U12 = L11^-1 A12, one column per thread (L11 broadcast from LDS);
//   (c) A22 -= L21 U12 on the MFMA, both operands from LDS.
__global__ void __launch_bounds__(HT) lu_hr_kernel(int b, double* __restrict__ A, i64 lda, double* __restrict__ sgn) {
    __shared__ double Ls[32][HB + 1];       // Ls[k][r] = L(j0 + r, j0 + k), r < M
    __shared__ double Us[32][HB + 1];       // Us[k][c] = U(j0 + k, j0 + 32 + c)
    __shared__ double rb[2][32];
    const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
    for (int j0 = 0; j0 < b; j0 += 32) {
        const int jb = min(32, b - j0), M = b - j0, N2 = b - j0 - jb;
        // ---- (a) panel: thread r owns row j0 + r
        const int r = tid;
        const bool own = r < M;
        double a[32];
        #pragma unroll
        for (int c = 0; c < 32; ++c) a[c] = (own && c < jb) ? A[(j0 + r) + (i64)(j0 + c) * lda] : 0.0;
        #pragma unroll
        for (int c = 0; c < 32; ++c) {
            if (c < jb) {
                if (r == c) {
                    #pragma unroll
                    for (int cc = 0; cc < 32; ++cc) rb[c & 1][cc] = a[cc];
                }
                __syncthreads();
                const double d = rb[c & 1][c];
                const double u = d + (d >= 0.0 ? 1.0 : -1.0);
                if (own && r > c) {
                    const double l = a[c] / u;
                    a[c] = l;
                    #pragma unroll
                    for (int cc = c + 1; cc < 32; ++cc) a[cc] -= l * rb[c & 1][cc];
                } else if (r == c) {
                    a[c] = u;
                    sgn[j0 + c] = d >= 0.0 ? -1.0 : 1.0;
                }
            }
        }
        if (own) {
            #pragma unroll
            for (int c = 0; c < 32; ++c)
                if (c < jb) {
                    A[(j0 + r) + (i64)(j0 + c) * lda] = a[c];
                    Ls[c][r] = a[c];
                }
        }
        __syncthreads();
        if (N2 <= 0) break;                 // (jb == 32 below)
        // ---- (b) U12 = L11^-1 A12 (unit lower), thread per column
        if (tid < N2) {
            const i64 col = (i64)(j0 + 32 + tid) * lda;
            double x[32];
            #pragma unroll
            for (int c = 0; c < 32; ++c) x[c] = A[(j0 + c) + col];
            #pragma unroll
            for (int k = 0; k < 32; ++k)
                #pragma unroll
                for (int i = k + 1; i < 32; ++i) x[i] -= Ls[k][i] * x[k];
            #pragma unroll
            for (int c = 0; c < 32; ++c) {
                A[(j0 + c) + col] = x[c];
                Us[c][tid] = x[c];
            }
        }
        __syncthreads();
        // ---- (c) A22 -= L21 U12: 16 x 16 tiles over the 16 waves
        const int nt = (N2 + 15) / 16;
        for (int t = w; t < nt * nt; t += HT / 64) {
            const int ti = t % nt, tj = t / nt;
            const int rr = min(16 * ti + (lane & 15), N2 - 1), cc = min(16 * tj + (lane & 15), N2 - 1);
            d4 acc = {0, 0, 0, 0};
            #pragma unroll
            for (int k = 0; k < 32; k += 4) {
                const int kk = k + (lane >> 4);
                acc = mma_hr(Us[kk][cc], Ls[kk][32 + rr], acc);
            }
            // acc[q] = C(row 16 ti + (lane & 15), col 16 tj + (lane >> 4) + 4 q)
            const int row = 16 * ti + (lane & 15);
            #pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int col = 16 * tj + (lane >> 4) + 4 * q;
                if (row < N2 && col < N2) A[(j0 + 32 + row) + (i64)(j0 + 32 + col) * lda] -= acc[q];
            }
        }
        __syncthreads();
    }
}

// The top b x b block holds Y1 (strict lower) and U (upper) from lu_hr:
//   Ut = U^T (lower, for Y2 = Q2 U^-1),  Tm = -U S (upper, zero below),
//   top upper part <- S R.  Every element is read and written by one thread.
__global__ void __launch_bounds__(256)
qf_top_kernel(int b, double* A, i64 lda, const double* sgn, const double* R, i64 ldr, double* Ut, i64 ldu,
              double* Tm, i64 ldt) {
    const int j = blockIdx.x;
    for (int i = threadIdx.x; i < b; i += 256) {
        if (i <= j) {
            const double u = A[i + (i64)j * lda];
            Ut[j + (i64)i * ldu] = u;
            Tm[i + (i64)j * ldt] = -u * sgn[j];
            A[i + (i64)j * lda] = sgn[i] * R[i + (i64)j * ldr];
        } else {
            Ut[j + (i64)i * ldu] = 0.0;
            Tm[i + (i64)j * ldt] = 0.0;
        }
    }
}

__global__ void qf_tau_kernel(int b, const double* Tm, i64 ldt, double* tau) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i < b) tau[i] = Tm[i + (i64)i * ldt];
}

static void gemm_d(char ta, char tb, i64 m, i64 n, i64 k, double alpha, const double* A, i64 lda, const double* B,
                   i64 ldb, double beta, double* C, i64 ldc, hipStream_t s, const int* gate = nullptr) {
    GemmCall c;
    c.transA = ta; c.transB = tb; c.m = m; c.n = n; c.k = k;
    c.alpha_re = alpha; c.beta_re = beta;
    c.A = A; c.lda = lda; c.B = B; c.ldb = ldb; c.C = C; c.ldc = ldc;
    c.gate = gate;
    gemm_real<double>(c, s);
}

static bool cholqr_enabled() {
    static const bool on = [] {
        const char* e = std::getenv("SLATE_AMD_QR_PANEL");
        return !(e && std::strcmp(e, "householder") == 0);
    }();
    return on;
}

bool geqrf_cholqr(i64 m, i64 b, double* A, i64 lda, double* tau, double* Tm, i64 ldt, double* V, i64 ldv,
                  hipStream_t s) {
    if (b < 16 || b > HB || m < 8 * b || !cholqr_enabled()) return false;
    const size_t mb = (size_t)m * b, bb = (size_t)b * b;
    double* Bk = static_cast<double*>(workspace(s, sizeof(double) * (mb + 4 * bb + b + 8) + 64, WS_QF));
    double* G = Bk + mb;
    double* Rm = G + bb;
    double* Rm2 = Rm + bb;
    double* Ut = Rm2 + bb;
    double* sgn = Ut + bb;
    double* tr0 = sgn + b;                      // ||A||_F^2 of the panel
    double* pfloor = tr0 + 1;                   // pivot floor of the fallback Cholesky
    i64* inf = reinterpret_cast<i64*>(pfloor + 1);
    int* flag = reinterpret_cast<int*>(inf + 4);
    gecopy<double, double>('G', 'N', m, b, A, lda, Bk, m, s);
    zero_words(inf, 4, s);
    // ---- CholeskyQR2 (always): G = A^T A, G = L L^T, A = A L^-T, R = L^T R
    auto gram = [&](const int* gate) { gemm_d('T', 'N', b, b, m, 1.0, A, lda, A, lda, 0.0, G, b, s, gate); };
    gram(nullptr);
    hipLaunchKernelGGL(qf_shift_kernel, dim3(1), dim3(256), 0, s, (int)b, G, (i64)b, 0.0, tr0, (double*)nullptr,
                       (const int*)nullptr);
    HIP_LAUNCH_CHECK();
    potrf_fast((int)b, G, b, inf + 0, 0, s);
    trsm_rlt_fast(m, b, 1.0, G, b, A, lda, false, s);
    hipLaunchKernelGGL(qf_rt_kernel, dim3((unsigned)b), dim3(256), 0, s, (int)b, (const double*)G, (i64)b, Rm, (i64)b,
                       (const int*)nullptr);
    HIP_LAUNCH_CHECK();
    gram(nullptr);
    potrf_fast((int)b, G, b, inf + 1, 0, s);
    trsm_rlt_fast(m, b, 1.0, G, b, A, lda, false, s);
    trmm<double>('L', 'L', 'T', 'N', b, b, 1.0, G, b, Rm, b, s);
    // flag = CholeskyQR2 not enough (a Cholesky failed, or the second factor
    // is not I to 1e-3: kappa(A) too large for two passes)
    hipLaunchKernelGGL(qf_check_kernel, dim3(1), dim3(256), 0, s, (int)b, (const double*)G, (i64)b,
                       (const i64*)inf, 2, 1e-3, flag);
    HIP_LAUNCH_CHECK();
    // ---- fallback, gated on the flag: perturbed shifted CholeskyQR3 with a
    //      pivot floor (see the header); R ping-pongs Rm -> Rm2 -> Rm
    {
        const int* g = flag;
        hipLaunchKernelGGL(qf_perturb_kernel, dim3((unsigned)((m + 255) / 256), (unsigned)std::min<i64>(b, 64)),
                           dim3(256), 0, s, m, (int)b, (const double*)Bk, (i64)m, A, lda, (const double*)tr0, g);
        HIP_LAUNCH_CHECK();
        const double shift = 11.0 * ((double)m * b + (double)b * (b + 1)) * 0x1p-53;
        for (int p = 0; p < 3; ++p) {
            gram(g);
            hipLaunchKernelGGL(qf_shift_kernel, dim3(1), dim3(256), 0, s, (int)b, G, (i64)b, p == 0 ? shift : 0.0,
                               (double*)nullptr, pfloor, g);
            HIP_LAUNCH_CHECK();
            potrf_fast((int)b, G, b, inf + 2, 0, s, g, pfloor);
            trsm_rlt_fast(m, b, 1.0, G, b, A, lda, false, s, g);
            if (p == 0) {
                hipLaunchKernelGGL(qf_rt_kernel, dim3((unsigned)b), dim3(256), 0, s, (int)b, (const double*)G, (i64)b,
                                   Rm, (i64)b, g);
            } else {
                const double* Rin = (p == 1) ? Rm : Rm2;
                double* Rout = (p == 1) ? Rm2 : Rm;
                hipLaunchKernelGGL(qf_ltmul_kernel, dim3((unsigned)b), dim3(256), 0, s, (int)b, (const double*)G,
                                   (i64)b, Rin, (i64)b, Rout, (i64)b, g);
            }
            HIP_LAUNCH_CHECK();
        }
    }
    // ---- Householder reconstruction
    hipLaunchKernelGGL(lu_hr_kernel, dim3(1), dim3(HT), 0, s, (int)b, A, lda, sgn);
    HIP_LAUNCH_CHECK();
    hipLaunchKernelGGL(qf_top_kernel, dim3((unsigned)b), dim3(256), 0, s, (int)b, A, lda, (const double*)sgn,
                       (const double*)Rm, (i64)b, Ut, (i64)b, Tm, ldt);
    HIP_LAUNCH_CHECK();
    trsm_rlt_fast(m - b, b, 1.0, Ut, b, A + b, lda, false, s);      // Y2 = Q2 U^-1
    trsm_rlt_fast(b, b, 1.0, A, lda, Tm, ldt, true, s);             // T = -U S Y1^-T
    hipLaunchKernelGGL(qf_tau_kernel, dim3((unsigned)((b + 255) / 256)), dim3(256), 0, s, (int)b,
                       (const double*)Tm, ldt, tau);
    HIP_LAUNCH_CHECK();
    v_explicit<double>(m, b, A, lda, V, ldv, s);
    return true;
}

}  // namespace slate_hip
