// Triangular solve / multiply for gfx950 (replaces blas::batch::trsm /
// blas::batch::trmm device calls, src/internal/internal_trsm.cc:244,
// internal_trmm.cc:243).
//
// Blocked along the triangular dimension in KB-wide diagonal blocks:
//  * a "small" kernel solves (or multiplies by) one KB x KB diagonal block
//    for ALL right-hand sides at once: the block lives in LDS, every thread
//    owns one RHS vector in registers (fully unrolled, static indexing);
//  * the off-diagonal coupling is one MFMA GEMM launch per block.
// So a 512-wide triangle with any number of RHS is 8 small launches + 7
// GEMMs, all stream-ordered (no host sync).
#include "common.hpp"
#include "kernels.hpp"
#include "launchers.hpp"

namespace slate_hip {

namespace {
template <typename T> constexpr int kb_of() { return sizeof(T) >= 16 ? 32 : 64; }
}

// op(A) element (r, c) of a column-major A
template <typename T>
__device__ inline T opA(const T* A, i64 lda, char trans, int r, int c) {
    if (trans == 'N') return A[r + (i64)c * lda];
    T v = A[c + (i64)r * lda];
    return trans == 'C' ? s_conj(v) : v;
}

// MODE 0 = solve, 1 = multiply.
template <typename T, int KB, int MODE>
__global__ void __launch_bounds__(256)
tri_small_kernel(char side, bool lower_eff, char trans, bool unit, int kb, i64 nrhs,
                 const T* __restrict__ A, i64 lda, T* __restrict__ B, i64 ldb, T alpha) {
    __shared__ T As[KB][KB + 1];  // As[r][c] = op(A)(r, c)
    for (int idx = threadIdx.x; idx < kb * kb; idx += blockDim.x) {
        int r = idx % kb, c = idx / kb;
        bool in_tri = lower_eff ? (r >= c) : (r <= c);
        T v = in_tri ? opA(A, lda, trans, r, c) : s_zero(T());
        if (r == c && unit) v = s_from_real(T(), 1);
        As[r][c] = v;
    }
    __syncthreads();
    const i64 v = (i64)blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= nrhs) return;
    T x[KB];
    // Left: RHS vector = column v of B (kb x nrhs); Right: row v of B (nrhs x kb)
    #pragma unroll
    for (int j = 0; j < KB; ++j)
        x[j] = (j < kb) ? s_mul(alpha, side == 'L' ? B[j + v * ldb] : B[v + (i64)j * ldb]) : s_zero(T());
    // Left: op(A) x = b  -> forward if lower.  Right: x op(A) = b, i.e.
    // op(A)^T x = b -> forward if upper.
    const bool forward = (side == 'L') ? lower_eff : !lower_eff;
    if (MODE == 0) {
        if (forward) {
            #pragma unroll
            for (int j = 0; j < KB; ++j) {
                if (j < kb) {
                    T s = x[j];
                    #pragma unroll
                    for (int l = 0; l < KB; ++l)
                        if (l < j) s = s_sub(s, s_mul(side == 'L' ? As[j][l] : As[l][j], x[l]));
                    x[j] = s_div(s, As[j][j]);
                }
            }
        } else {
            #pragma unroll
            for (int j = KB - 1; j >= 0; --j) {
                if (j < kb) {
                    T s = x[j];
                    #pragma unroll
                    for (int l = 0; l < KB; ++l)
                        if (l > j && l < kb) s = s_sub(s, s_mul(side == 'L' ? As[j][l] : As[l][j], x[l]));
                    x[j] = s_div(s, As[j][j]);
                }
            }
        }
    } else {
        // multiply: y_j = sum_l M(j, l) x_l with M = op(A) (left) or op(A)^T (right)
        T y[KB];
        #pragma unroll
        for (int j = 0; j < KB; ++j) {
            T s = s_zero(T());
            #pragma unroll
            for (int l = 0; l < KB; ++l)
                if (j < kb && l < kb) s = s_add(s, s_mul(side == 'L' ? As[j][l] : As[l][j], x[l]));
            y[j] = s;
        }
        #pragma unroll
        for (int j = 0; j < KB; ++j) x[j] = y[j];
    }
    #pragma unroll
    for (int j = 0; j < KB; ++j)
        if (j < kb) {
            if (side == 'L') B[j + v * ldb] = x[j];
            else B[v + (i64)j * ldb] = x[j];
        }
}

template <typename T>
static void small(int mode, char side, bool lower_eff, char trans, bool unit, int kb, i64 nrhs,
                  const T* A, i64 lda, T* B, i64 ldb, T alpha, hipStream_t s) {
    constexpr int KB = kb_of<T>();
    if (nrhs <= 0 || kb <= 0) return;
    dim3 grid((unsigned)((nrhs + 255) / 256));
    if (mode == 0)
        hipLaunchKernelGGL((tri_small_kernel<T, KB, 0>), grid, dim3(256), 0, s, side, lower_eff, trans, unit, kb,
                           nrhs, A, lda, B, ldb, alpha);
    else
        hipLaunchKernelGGL((tri_small_kernel<T, KB, 1>), grid, dim3(256), 0, s, side, lower_eff, trans, unit, kb,
                           nrhs, A, lda, B, ldb, alpha);
    HIP_LAUNCH_CHECK();
}

template <typename T>
static void gemm_T(char ta, char tb, i64 m, i64 n, i64 k, double ar, double ai, const T* A, i64 lda,
                   const T* B, i64 ldb, double br, double bi, T* C, i64 ldc, hipStream_t s) {
    GemmCall c;
    c.transA = ta; c.transB = tb; c.m = m; c.n = n; c.k = k;
    c.alpha_re = ar; c.alpha_im = ai; c.beta_re = br; c.beta_im = bi;
    c.A = A; c.lda = lda; c.B = B; c.ldb = ldb; c.C = C; c.ldc = ldc;
    if constexpr (scalar_traits<T>::is_complex) gemm_complex<T>(c, s);
    else gemm_real<T>(c, s);
}

// pointer to op(A) sub-block starting at op-coordinates (r, c)
template <typename T>
static const T* opblk(const T* A, i64 lda, char trans, i64 r, i64 c) {
    return trans == 'N' ? A + r + c * lda : A + c + r * lda;
}

template <typename T>
void trsm(char side, char uplo, char trans, char diag, i64 m, i64 n, T alpha,
          const T* A, i64 lda, T* B, i64 ldb, hipStream_t s) {
    if (m <= 0 || n <= 0) return;
    constexpr int KB = kb_of<T>();
    const bool lower_eff = (uplo == 'L') == (trans == 'N');
    const bool unit = diag == 'U';
    const i64 kt = side == 'L' ? m : n;       // triangular dimension
    const i64 nrhs = side == 'L' ? n : m;
    const i64 nblk = (kt + KB - 1) / KB;
    const bool forward = (side == 'L') ? lower_eff : !lower_eff;
    const T one = s_from_real(T(), 1);
    for (i64 b = 0; b < nblk; ++b) {
        const i64 kbi = forward ? b : nblk - 1 - b;
        const i64 k0 = kbi * KB, kb = std::min<i64>(KB, kt - k0);
        const T a = (b == 0) ? alpha : one;
        T* Bk = side == 'L' ? B + k0 : B + k0 * ldb;
        if (b == 0 && !s_is_zero(s_sub(alpha, one))) {
            // scale the not-yet-touched part by alpha once (the small solve
            // scales its own block)
            // handled by passing alpha to every gemm's beta below
        }
        small<T>(0, side, lower_eff, trans, unit, (int)kb, nrhs, opblk(A, lda, trans, k0, k0), lda, Bk, ldb, a, s);
        // coupling update of the remaining blocks
        const T beta = (b == 0) ? alpha : one;
        const double br = s_real(beta);
        double bi = 0;
        if constexpr (scalar_traits<T>::is_complex) bi = beta.im;
        if (side == 'L') {
            if (forward && k0 + kb < m) {
                i64 r0 = k0 + kb;
                gemm_T<T>(trans, 'N', m - r0, n, kb, -1, 0, opblk(A, lda, trans, r0, k0), lda, Bk, ldb,
                          br, bi, B + r0, ldb, s);
            } else if (!forward && k0 > 0) {
                gemm_T<T>(trans, 'N', k0, n, kb, -1, 0, opblk(A, lda, trans, 0, k0), lda, Bk, ldb,
                          br, bi, B, ldb, s);
            }
        } else {
            // X op(A) = B: columns of B;  B_rest -= X_k * op(A)(k, rest)
            if (forward && k0 + kb < n) {
                i64 c0 = k0 + kb;
                gemm_T<T>('N', trans, m, n - c0, kb, -1, 0, Bk, ldb, opblk(A, lda, trans, k0, c0), lda,
                          br, bi, B + c0 * ldb, ldb, s);
            } else if (!forward && k0 > 0) {
                gemm_T<T>('N', trans, m, k0, kb, -1, 0, Bk, ldb, opblk(A, lda, trans, k0, 0), lda,
                          br, bi, B, ldb, s);
            }
        }
    }
}

template <typename T>
void trmm(char side, char uplo, char trans, char diag, i64 m, i64 n, T alpha,
          const T* A, i64 lda, T* B, i64 ldb, hipStream_t s) {
    if (m <= 0 || n <= 0) return;
    constexpr int KB = kb_of<T>();
    const bool lower_eff = (uplo == 'L') == (trans == 'N');
    const bool unit = diag == 'U';
    const i64 kt = side == 'L' ? m : n;
    const i64 nrhs = side == 'L' ? n : m;
    const i64 nblk = (kt + KB - 1) / KB;
    // order so that the blocks a block depends on are still unmodified:
    // Left lower: last->first; Left upper: first->last;
    // Right lower: first->last; Right upper: last->first.
    const bool first_to_last = (side == 'L') ? !lower_eff : lower_eff;
    const double ar = s_real(alpha);
    double ai = 0;
    if constexpr (scalar_traits<T>::is_complex) ai = alpha.im;
    const T one = s_from_real(T(), 1);
    for (i64 b = 0; b < nblk; ++b) {
        const i64 kbi = first_to_last ? b : nblk - 1 - b;
        const i64 k0 = kbi * KB, kb = std::min<i64>(KB, kt - k0);
        T* Bk = side == 'L' ? B + k0 : B + k0 * ldb;
        small<T>(1, side, lower_eff, trans, unit, (int)kb, nrhs, opblk(A, lda, trans, k0, k0), lda, Bk, ldb,
                 alpha, s);
        (void)one;
        if (side == 'L') {
            if (lower_eff && k0 > 0)        // B_k += alpha op(A)(k, <k) B_<k
                gemm_T<T>(trans, 'N', kb, n, k0, ar, ai, opblk(A, lda, trans, k0, 0), lda, B, ldb, 1, 0, Bk, ldb, s);
            else if (!lower_eff && k0 + kb < m)
                gemm_T<T>(trans, 'N', kb, n, m - k0 - kb, ar, ai, opblk(A, lda, trans, k0, k0 + kb), lda,
                          B + k0 + kb, ldb, 1, 0, Bk, ldb, s);
        } else {
            if (lower_eff && k0 + kb < n)   // B_k += alpha B_>k op(A)(>k, k)
                gemm_T<T>('N', trans, m, kb, n - k0 - kb, ar, ai, B + (k0 + kb) * ldb, ldb,
                          opblk(A, lda, trans, k0 + kb, k0), lda, 1, 0, Bk, ldb, s);
            else if (!lower_eff && k0 > 0)
                gemm_T<T>('N', trans, m, kb, k0, ar, ai, B, ldb, opblk(A, lda, trans, 0, k0), lda, 1, 0, Bk, ldb, s);
        }
    }
}

#define INST(T) \
    template void trsm<T>(char, char, char, char, i64, i64, T, const T*, i64, T*, i64, hipStream_t); \
    template void trmm<T>(char, char, char, char, i64, i64, T, const T*, i64, T*, i64, hipStream_t);
INST(float) INST(double) INST(ccplx) INST(zcplx)
#undef INST

}  // namespace slate_hip
