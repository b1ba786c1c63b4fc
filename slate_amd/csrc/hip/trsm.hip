// Triangular inverse / solve / multiply for gfx950 (replaces the vendor
// blas::batch::trsm / trmm and lapack::trtri device calls,
// src/internal/internal_trsm.cc:244, internal_trmm.cc:243).
//
// All FLOPs go to the MFMA GEMM:
//   tri_inv(A)   ONE launch inverts every 64x64 diagonal block (one workgroup
//                per block, block in LDS, one column of the inverse per
//                thread held in registers, fully unrolled), then log2(n/64)
//                doubling levels, each two STRIDED-BATCHED GEMMs over all
//                block pairs:  W21 = -W22 (A21 W11).
//   trsm         kt <= 1024: W = inv(A) + ONE GEMM X = op(W) B (or B op(W)) +
//                copy back; larger: the same per 1024-block with GEMM
//                coupling updates (blocked forward/backward substitution).
//   trmm         diagonal blocks extracted once, then GEMMs into a workspace.
// Workspaces come from the per-stream cache (workspace.hpp): no host sync,
// no per-call allocation on the critical path.
#include <type_traits>
#include "common.hpp"
#include "kernels.hpp"
#include "launchers.hpp"
#include "workspace.hpp"

namespace slate_hip {

namespace {
constexpr int KB = 64;       // diagonal-block size of the inverse kernel
constexpr int BIG = 1024;    // largest triangle inverted as a whole
}

// W(b) = inv(D_b) (INV) or D_b with the other triangle zeroed (unit diag
// applied) for the b-th KB x KB diagonal block of the stored triangle.
// Output written at W + b*KB*(ldw+1) (i.e. on the diagonal of an n x n W).
template <typename T> constexpr int kbinv() { return scalar_traits<T>::is_complex ? 32 : 64; }

template <typename T, bool INV, int KB = 64>
__global__ void __launch_bounds__(KB)
tri_diag_kernel(char uplo, bool unit, i64 n, const T* __restrict__ A, i64 lda, T* __restrict__ W, i64 ldw,
                bool strip) {
    __shared__ T L[KB][KB + 1];
    const int b = blockIdx.x;
    const i64 k0 = (i64)b * KB;
    const int kb = (int)min((i64)KB, n - k0);
    const bool lower = uplo == 'L';
    const int j = threadIdx.x;
    // coalesced: thread j reads row j of every column
    for (int c = 0; c < KB; ++c) {
        const int r = j;
        T v = s_zero(T());
        if (r < kb && c < kb) {
            bool in = lower ? r >= c : r <= c;
            if (in) v = A[k0 + r + (k0 + c) * lda];
            if (r == c && unit) v = s_from_real(T(), 1);
        }
        if (r == c && r >= kb) v = s_from_real(T(), 1);
        L[r][c] = v;
    }
    __shared__ T dinv[KB];
    __syncthreads();
    dinv[j] = s_div(s_from_real(T(), 1), L[j][j]);
    __syncthreads();
    T* Wb = strip ? W + k0 : W + k0 + k0 * ldw;   // strip: kt x KB stack of blocks
    if (!INV) {
        if (j < kb)
            for (int c = 0; c < kb; ++c) Wb[j + (i64)c * ldw] = L[j][c];
        return;
    }
    if constexpr (scalar_traits<T>::is_complex) {
        // complex: column j of inv(L) kept in LDS (register arrays of complex
        // values spill); row-oriented substitution
        __shared__ T X[KB][KB + 1];
        if (lower) {
            for (int i = 0; i < KB; ++i) {
                T sacc = (i == j) ? s_from_real(T(), 1) : s_zero(T());
                for (int l = j; l < i; ++l) sacc = s_sub(sacc, s_mul(L[i][l], X[l][j]));
                X[i][j] = (i < j) ? s_zero(T()) : s_mul(sacc, dinv[i]);
            }
        } else {
            for (int i = KB - 1; i >= 0; --i) {
                T sacc = (i == j) ? s_from_real(T(), 1) : s_zero(T());
                for (int l = i + 1; l <= j; ++l) sacc = s_sub(sacc, s_mul(L[i][l], X[l][j]));
                X[i][j] = (i > j) ? s_zero(T()) : s_mul(sacc, dinv[i]);
            }
        }
        __syncthreads();
        if (j < kb)
            for (int c = 0; c < kb; ++c) Wb[j + (i64)c * ldw] = X[j][c];
    } else {
        // column j of inv(L), column-oriented substitution, x in registers
        T x[KB];
        #pragma unroll
        for (int i = 0; i < KB; ++i) x[i] = (i == j) ? s_from_real(T(), 1) : s_zero(T());
        if (lower) {
            #pragma unroll
            for (int l = 0; l < KB; ++l) {
                x[l] = s_mul(x[l], dinv[l]);
                const T xl = x[l];
                #pragma unroll
                for (int i = l + 1; i < KB; ++i) x[i] = s_sub(x[i], s_mul(L[i][l], xl));
            }
        } else {
            #pragma unroll
            for (int l = KB - 1; l >= 0; --l) {
                x[l] = s_mul(x[l], dinv[l]);
                const T xl = x[l];
                #pragma unroll
                for (int i = 0; i < l; ++i) x[i] = s_sub(x[i], s_mul(L[i][l], xl));
            }
        }
        // transpose through LDS for a coalesced store
        __syncthreads();
        #pragma unroll
        for (int r = 0; r < KB; ++r) L[r][j] = x[r];
        __syncthreads();
        if (j < kb)
            for (int c = 0; c < kb; ++c) Wb[j + (i64)c * ldw] = L[j][c];
    }
}

template <typename T>
static void gemm_T(char ta, char tb, i64 m, i64 n, i64 k, T alpha, const T* A, i64 lda,
                   const T* B, i64 ldb, T beta, T* C, i64 ldc, hipStream_t s,
                   i64 batch = 1, i64 sA = 0, i64 sB = 0, i64 sC = 0) {
    if (m <= 0 || n <= 0 || batch <= 0) return;
    GemmCall c;
    c.transA = ta; c.transB = tb; c.m = m; c.n = n; c.k = k;
    c.A = A; c.lda = lda; c.B = B; c.ldb = ldb; c.C = C; c.ldc = ldc;
    c.batch = batch; c.strideA = sA; c.strideB = sB; c.strideC = sC;
    if constexpr (scalar_traits<T>::is_complex) {
        c.alpha_re = alpha.re; c.alpha_im = alpha.im; c.beta_re = beta.re; c.beta_im = beta.im;
        gemm_complex<T>(c, s);
    } else {
        c.alpha_re = alpha; c.beta_re = beta;
        gemm_real<T>(c, s);
    }
}

// W (n x n, ld ldw) = inv(A) for the stored triangle of A.  The other
// triangle of W is set to zero.
template <typename T>
void tri_inv(char uplo, char diag, i64 n, const T* A, i64 lda, T* W, i64 ldw, hipStream_t s) {
    if (n <= 0) return;
    const T zero = s_zero(T()), one = s_from_real(T(), 1), mone = s_from_real(T(), -1);
    geset<T>('G', n, n, zero, zero, W, ldw, s);
    constexpr int KI = kbinv<T>();
    const i64 nblk = (n + KI - 1) / KI;
    hipLaunchKernelGGL((tri_diag_kernel<T, true, KI>), dim3((unsigned)nblk), dim3(KI), 0, s, uplo, diag == 'U', n, A,
                       lda, W, ldw, false);
    HIP_LAUNCH_CHECK();
    const bool lower = uplo == 'L';
    T* Tmp = static_cast<T*>(workspace(s, sizeof(T) * (size_t)n * KI * 2 + sizeof(T) * n * n / 2 + 64, WS_T));
    for (i64 b = KI; b < n; b *= 2) {
        // pairs [k0, k0+b) | [k0+b, k0+2b): full pairs are batched
        const i64 npair = n / (2 * b);
        auto pair = [&](i64 k0, i64 b2, i64 batch) {
            // b2 = size of the second block (may be ragged)
            const i64 str = 2 * b * (lda + 1), strw = 2 * b * (ldw + 1), strt = b * b2;
            if (lower) {
                // T = A21 W11 (b2 x b), W21 = -W22 T
                gemm_T<T>('N', 'N', b2, b, b, one, A + (k0 + b) + k0 * lda, lda, W + k0 + k0 * ldw, ldw, zero,
                          Tmp, b2, s, batch, str, strw, strt);
                gemm_T<T>('N', 'N', b2, b, b2, mone, W + (k0 + b) + (k0 + b) * ldw, ldw, Tmp, b2, zero,
                          W + (k0 + b) + k0 * ldw, ldw, s, batch, strw, strt, strw);
            } else {
                // T = A12 W22 (b x b2), W12 = -W11 T
                gemm_T<T>('N', 'N', b, b2, b2, one, A + k0 + (k0 + b) * lda, lda, W + (k0 + b) + (k0 + b) * ldw,
                          ldw, zero, Tmp, b, s, batch, str, strw, strt);
                gemm_T<T>('N', 'N', b, b2, b, mone, W + k0 + k0 * ldw, ldw, Tmp, b, zero,
                          W + k0 + (k0 + b) * ldw, ldw, s, batch, strw, strt, strw);
            }
        };
        if (npair > 0) pair(0, b, npair);
        const i64 k0 = npair * 2 * b;
        if (k0 + b < n) pair(k0, n - k0 - b, 1);   // ragged last pair
    }
}

// pointer to op(A) sub-block starting at op-coordinates (r, c)
template <typename T>
static const T* opblk(const T* A, i64 lda, char trans, i64 r, i64 c) {
    return trans == 'N' ? A + r + c * lda : A + c + r * lda;
}

// X L^T = alpha B, L n x n lower (the Cholesky panel), recursively halved
// over the columns: X1 = alpha B1 L11^{-T}; B2 = alpha B2 - X1 L21^T (one
// MFMA GEMM); X2 = B2 L22^{-T} -- the blocked-inverse strip kernel only on
// the <= 128-column leaves.  Opt-in (SLATE_AMD_TRSM_RLT_REC=1): measured on
// MI355X, dpotrf n = 32768 (the panel solve sharing the GPU with the
// trailing GEMM) 58.4 TF/s with it against 59.1 with the whole-width strip
// kernel (profiles/r5/potrf_trsm_rec.txt).
static bool trsm_rlt_rec(i64 m, i64 n, double alpha, const double* L, i64 ldl, double* B, i64 ldb, bool unit,
                         char trans, hipStream_t s) {
    static const bool on = [] {
        const char* e = std::getenv("SLATE_AMD_TRSM_RLT_REC");
        return e && e[0] == '1';
    }();
    if (!on || n <= 128 || m < 1024) return trsm_rlt_fast(m, n, alpha, L, ldl, B, ldb, unit, s);
    const i64 n1 = ((n / 2 + 63) / 64) * 64;
    if (!trsm_rlt_rec(m, n1, alpha, L, ldl, B, ldb, unit, trans, s)) return false;
    gemm_T<double>('N', trans, m, n - n1, n1, -1.0, B, ldb, L + n1, ldl, alpha, B + n1 * ldb, ldb, s);
    return trsm_rlt_rec(m, n - n1, 1.0, L + n1 + n1 * ldl, ldl, B + n1 * ldb, ldb, unit, trans, s);
}

template <typename T>
void trsm(char side, char uplo, char trans, char diag, i64 m, i64 n, T alpha,
          const T* A, i64 lda, T* B, i64 ldb, hipStream_t s) {
    if (m <= 0 || n <= 0) return;
    if constexpr (std::is_same<T, double>::value) {
        // X L^T = alpha B (the Cholesky panel): blocked-inverse MFMA kernel
        if (side == 'R' && uplo == 'L' && trans != 'N' &&
            trsm_rlt_rec(m, n, alpha, A, lda, B, ldb, diag == 'U', trans, s))
            return;
        // L X = alpha B (LU's U rows, forward solves): one-launch MFMA kernel
        if (side == 'L' && uplo == 'L' && trans == 'N' && trsm_lln_fast(m, n, alpha, A, lda, B, ldb, diag == 'U', s))
            return;
    }
    const bool lower_eff = (uplo == 'L') == (trans == 'N');
    const i64 kt = side == 'L' ? m : n;
    const i64 nblk = (kt + BIG - 1) / BIG;
    const bool forward = (side == 'L') ? lower_eff : !lower_eff;
    const T one = s_from_real(T(), 1), zero = s_zero(T()), mone = s_from_real(T(), -1);
    const i64 bw = std::min<i64>(BIG, kt);
    T* Winv = static_cast<T*>(workspace(s, sizeof(T) * (size_t)bw * bw * nblk, WS_W));
    T* X = static_cast<T*>(workspace(s, sizeof(T) * (size_t)m * n, WS_X));
    const i64 ldx = m;
    for (i64 b = 0; b < nblk; ++b) {
        const i64 k0 = b * BIG, kb = std::min<i64>(BIG, kt - k0);
        tri_inv<T>(uplo, diag, kb, A + k0 + k0 * lda, lda, Winv + b * bw * bw, bw, s);
    }
    for (i64 b = 0; b < nblk; ++b) {
        const i64 kbi = forward ? b : nblk - 1 - b;
        const i64 k0 = kbi * BIG, kb = std::min<i64>(BIG, kt - k0);
        const T a = (b == 0) ? alpha : one;
        const T* Dinv = Winv + kbi * bw * bw;
        if (side == 'L') {
            gemm_T<T>(trans, 'N', kb, n, kb, a, Dinv, bw, B + k0, ldb, zero, X + k0, ldx, s);
            if (forward && k0 + kb < m)
                gemm_T<T>(trans, 'N', m - k0 - kb, n, kb, mone, opblk(A, lda, trans, k0 + kb, k0), lda,
                          X + k0, ldx, a, B + k0 + kb, ldb, s);
            else if (!forward && k0 > 0)
                gemm_T<T>(trans, 'N', k0, n, kb, mone, opblk(A, lda, trans, 0, k0), lda, X + k0, ldx,
                          a, B, ldb, s);
        } else {
            gemm_T<T>('N', trans, m, kb, kb, a, B + k0 * ldb, ldb, Dinv, bw, zero, X + k0 * ldx, ldx, s);
            if (forward && k0 + kb < n)
                gemm_T<T>('N', trans, m, n - k0 - kb, kb, mone, X + k0 * ldx, ldx,
                          opblk(A, lda, trans, k0, k0 + kb), lda, a, B + (k0 + kb) * ldb, ldb, s);
            else if (!forward && k0 > 0)
                gemm_T<T>('N', trans, m, k0, kb, mone, X + k0 * ldx, ldx, opblk(A, lda, trans, k0, 0), lda,
                          a, B, ldb, s);
        }
    }
    gecopy<T, T>('G', 'N', m, n, X, ldx, B, ldb, s);
}

template <typename T>
void trmm(char side, char uplo, char trans, char diag, i64 m, i64 n, T alpha,
          const T* A, i64 lda, T* B, i64 ldb, hipStream_t s) {
    if (m <= 0 || n <= 0) return;
    const bool lower_eff = (uplo == 'L') == (trans == 'N');
    const i64 kt = side == 'L' ? m : n;
    const i64 nblk = (kt + KB - 1) / KB;
    const T zero = s_zero(T()), one = s_from_real(T(), 1);
    T* Wd = static_cast<T*>(workspace(s, sizeof(T) * (size_t)kt * KB + 64, WS_W));
    T* X = static_cast<T*>(workspace(s, sizeof(T) * (size_t)m * n, WS_X));
    const i64 ldx = m;
    // diagonal blocks (other triangle zeroed, unit diag applied) as a kt x KB strip
    hipLaunchKernelGGL((tri_diag_kernel<T, false>), dim3((unsigned)nblk), dim3(KB), 0, s, uplo, diag == 'U', kt, A,
                       lda, Wd, kt, true);
    HIP_LAUNCH_CHECK();
    for (i64 b = 0; b < nblk; ++b) {
        const i64 k0 = b * KB, kb = std::min<i64>(KB, kt - k0);
        const T* D = Wd + k0;
        if (side == 'L') {
            gemm_T<T>(trans, 'N', kb, n, kb, alpha, D, kt, B + k0, ldb, zero, X + k0, ldx, s);
            if (lower_eff && k0 > 0)
                gemm_T<T>(trans, 'N', kb, n, k0, alpha, opblk(A, lda, trans, k0, 0), lda, B, ldb, one, X + k0, ldx, s);
            else if (!lower_eff && k0 + kb < m)
                gemm_T<T>(trans, 'N', kb, n, m - k0 - kb, alpha, opblk(A, lda, trans, k0, k0 + kb), lda,
                          B + k0 + kb, ldb, one, X + k0, ldx, s);
        } else {
            gemm_T<T>('N', trans, m, kb, kb, alpha, B + k0 * ldb, ldb, D, kt, zero, X + k0 * ldx, ldx, s);
            if (lower_eff && k0 + kb < n)
                gemm_T<T>('N', trans, m, kb, n - k0 - kb, alpha, B + (k0 + kb) * ldb, ldb,
                          opblk(A, lda, trans, k0 + kb, k0), lda, one, X + k0 * ldx, ldx, s);
            else if (!lower_eff && k0 > 0)
                gemm_T<T>('N', trans, m, kb, k0, alpha, B, ldb, opblk(A, lda, trans, 0, k0), lda, one,
                          X + k0 * ldx, ldx, s);
        }
    }
    gecopy<T, T>('G', 'N', m, n, X, ldx, B, ldb, s);
}

// Full triangular inverse in place (trtri).
template <typename T>
void trtri(char uplo, char diag, i64 n, T* A, i64 lda, i64* info, hipStream_t s) {
    if (info) HIP_CHECK(hipMemsetAsync(info, 0, sizeof(i64), s));
    if (n <= 0) return;
    if (n <= BIG) {
        T* W = static_cast<T*>(workspace(s, sizeof(T) * (size_t)n * n, WS_I));
        tri_inv<T>(uplo, diag, n, A, lda, W, n, s);
        gecopy<T, T>(uplo, 'N', n, n, W, n, A, lda, s);
        return;
    }
    T* I = nullptr;
    I = static_cast<T*>(dev_alloc(sizeof(T) * n * n, s));
    geset<T>('G', n, n, s_zero(T()), s_from_real(T(), 1), I, n, s);
    trsm<T>('L', uplo, 'N', diag, n, n, s_from_real(T(), 1), A, lda, I, n, s);
    gecopy<T, T>(uplo, 'N', n, n, I, n, A, lda, s);
    dev_free(I, s);
}

#define INST(T) \
    template void trsm<T>(char, char, char, char, i64, i64, T, const T*, i64, T*, i64, hipStream_t); \
    template void trmm<T>(char, char, char, char, i64, i64, T, const T*, i64, T*, i64, hipStream_t); \
    template void trtri<T>(char, char, i64, T*, i64, i64*, hipStream_t); \
    template void tri_inv<T>(char, char, i64, const T*, i64, T*, i64, hipStream_t);
INST(float) INST(double) INST(ccplx) INST(zcplx)
#undef INST

}  // namespace slate_hip
