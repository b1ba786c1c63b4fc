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
// Breakdown (numerically rank-deficient panel: a Cholesky fails or the
// last factor is not ~I) is detected on the device and read back once per
// attempt; the panel is then restored from a copy and the caller runs the
// Householder panel instead.
#include <cstdlib>
#include <cstring>
#include "common.hpp"
#include "kernels.hpp"
#include "launchers.hpp"
#include "workspace.hpp"

namespace slate_hip {

namespace {
constexpr int HB = 256;          // widest panel of the fast path
constexpr int HT = 1024;         // threads of lu_hr
__device__ inline d4 mma_hr(double x, double y, d4 c) { return __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, c, 0, 0, 0); }
}  // namespace

// G(i, i) += c * trace(G)   (trace(A^T A) = ||A||_F^2)
__global__ void __launch_bounds__(256) qf_shift_kernel(int b, double* G, i64 ldg, double c) {
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
    for (int i = t; i < b; i += 256) G[i + (i64)i * ldg] += sh;
}

// R = L^T (upper, zero below)
__global__ void __launch_bounds__(256) qf_rt_kernel(int b, const double* L, i64 ldl, double* R, i64 ldr) {
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
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
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
                   i64 ldb, double beta, double* C, i64 ldc, hipStream_t s) {
    GemmCall c;
    c.transA = ta; c.transB = tb; c.m = m; c.n = n; c.k = k;
    c.alpha_re = alpha; c.beta_re = beta;
    c.A = A; c.lda = lda; c.B = B; c.ldb = ldb; c.C = C; c.ldc = ldc;
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
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    HIP_CHECK(hipStreamIsCapturing(s, &cs));
    if (cs != hipStreamCaptureStatusNone) return false;     // the breakdown check reads back to the host
    static thread_local int* hflag = nullptr;
    if (!hflag) HIP_CHECK(hipHostMalloc((void**)&hflag, sizeof(int), hipHostMallocDefault));
    const size_t mb = (size_t)m * b, bb = (size_t)b * b;
    double* Bk = static_cast<double*>(workspace(s, sizeof(double) * (mb + 3 * bb + b) + 64, WS_QF));
    double* G = Bk + mb;
    double* Rm = G + bb;
    double* Ut = Rm + bb;
    double* sgn = Ut + bb;
    i64* inf = reinterpret_cast<i64*>(sgn + b);
    int* flag = reinterpret_cast<int*>(inf + 4);
    gecopy<double, double>('G', 'N', m, b, A, lda, Bk, m, s);
    // one CholeskyQR pass: G = A^T A (+ shift I), G = L L^T, A = A L^-T, R = L^T R
    auto pass = [&](int p, bool first, double shift) {
        gemm_d('T', 'N', b, b, m, 1.0, A, lda, A, lda, 0.0, G, b, s);
        if (shift > 0) {
            hipLaunchKernelGGL(qf_shift_kernel, dim3(1), dim3(256), 0, s, (int)b, G, (i64)b, shift);
            HIP_LAUNCH_CHECK();
        }
        potrf_fast((int)b, G, b, inf + p, 0, s);
        trsm_rlt_fast(m, b, 1.0, G, b, A, lda, false, s);
        if (first) {
            hipLaunchKernelGGL(qf_rt_kernel, dim3((unsigned)b), dim3(256), 0, s, (int)b, (const double*)G, (i64)b,
                               Rm, (i64)b);
            HIP_LAUNCH_CHECK();
        } else {
            trmm<double>('L', 'L', 'T', 'N', b, b, 1.0, G, b, Rm, b, s);
        }
    };
    // breakdown / orthogonality check of the last pass, read back to the host
    auto failed = [&](int npass, double tol) {
        hipLaunchKernelGGL(qf_check_kernel, dim3(1), dim3(256), 0, s, (int)b, (const double*)G, (i64)b,
                           (const i64*)inf, npass, tol, flag);
        HIP_LAUNCH_CHECK();
        HIP_CHECK(hipMemcpyAsync(hflag, flag, sizeof(int), hipMemcpyDeviceToHost, s));
        HIP_CHECK(hipStreamSynchronize(s));
        return *hflag != 0;
    };
    // CholeskyQR2 first: enough when kappa(A) << u^-1/2, recognised by the
    // second factor being I to 1e-3 (then the final Q is orthonormal to O(u));
    // otherwise restart from the copy with shifted CholeskyQR3
    HIP_CHECK(hipMemsetAsync(inf, 0, 4 * sizeof(i64), s));
    pass(0, true, 0.0);
    pass(1, false, 0.0);
    if (failed(2, 1e-3)) {
        gecopy<double, double>('G', 'N', m, b, Bk, m, A, lda, s);
        HIP_CHECK(hipMemsetAsync(inf, 0, 4 * sizeof(i64), s));
        pass(0, true, 11.0 * ((double)m * b + (double)b * (b + 1)) * 0x1p-53);
        pass(1, false, 0.0);
        pass(2, false, 0.0);
        if (failed(3, 1e-3)) {
            gecopy<double, double>('G', 'N', m, b, Bk, m, A, lda, s);
            return false;
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
