// Tile Cholesky (potrf) for gfx950 -- the panel kernel of the distributed
// potrf (replaces the vendor `lapack::potrf` device call of
// src/internal/internal_potrf.cc:72).
//
// n <= NS (128 real / 64 complex-double): ONE workgroup of 1024 threads
// factors the block resident in LDS (right-looking, one barrier pair per
// column) -- ~10 us for 128x128 fp64.
// Larger tiles: blocked right-looking with NS-wide diagonal blocks:
//   potrf_small(A_kk) -> trsm(A_{>k,k}) by inverse-diagonal-block MFMA GEMMs
//   -> masked MFMA GEMM (herk) of the trailing triangle.
// info (1-based first non-positive pivot, 0 on success) is kept in a device
// int64 (first failure wins via atomicCAS) so the DAG never syncs the host.
#include <type_traits>
#include "common.hpp"
#include "kernels.hpp"
#include "launchers.hpp"

namespace slate_hip {

namespace {
template <typename T> constexpr int ns_of() { return sizeof(T) >= 16 ? 64 : 128; }
constexpr int NT = 256;
constexpr int IB = 32;

// broadcast lane `src` (wave-uniform) of v: v_readlane on each 32-bit word
template <typename T>
__device__ inline T shfl(T v, int src) {
    static_assert(sizeof(T) % 4 == 0, "");
    union U { T t; int w[sizeof(T) / 4]; } u, r;
    u.t = v;
    #pragma unroll
    for (int k = 0; k < (int)(sizeof(T) / 4); ++k) r.w[k] = __builtin_amdgcn_readlane(u.w[k], src);
    return r.t;
}
template <typename R>
__device__ inline R shfl_real(R v, int src) {
    union U { R t; int w[sizeof(R) / 4]; } u, r;
    u.t = v;
    #pragma unroll
    for (int k = 0; k < (int)(sizeof(R) / 4); ++k) r.w[k] = __builtin_amdgcn_readlane(u.w[k], src);
    return r.t;
}
}  // namespace

// Block resident in LDS (column-major with one-element pad), IB = 32 inner
// blocking:  (1) the 32x32 diagonal block is factored by ONE wave in
// registers (lane i owns row i, rows broadcast with __shfl, no barriers);
// (2) the panel below is solved row-per-thread against it (broadcast LDS
// reads); (3) the trailing lower triangle is updated in 4x4 register blocks.
// Three barriers per 32 columns.
template <typename T, int NS, bool UPPER>
__global__ void __launch_bounds__(NT)
potrf_small_kernel(int n, T* __restrict__ A, i64 lda, i64* info, i64 info_off) {
    using R = typename scalar_traits<T>::real;
    constexpr int LD = NS + 1;
    __shared__ T S[NS * LD];       // S[c * LD + r] = L(r, c)
    __shared__ int s_fail;
    const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    // 2-D thread map (no integer division), loads batched by unrolling
    {
        constexpr int CPI = NT / NS;           // columns per pass
        const int r = tid % NS, cb = tid / NS;
        if (UPPER) {
            // row r of the stored upper triangle is column r of L
            #pragma unroll 8
            for (int c = cb; c < NS; c += CPI)
                if (c < n && r < n && r >= c) S[c * LD + r] = s_conj(A[c + (i64)r * lda]);
        } else {
            #pragma unroll 8
            for (int c = cb; c < NS; c += CPI)
                if (c < n && r < n && r >= c) S[c * LD + r] = A[r + (i64)c * lda];
        }
    }
    if (tid == 0) s_fail = 0;
    __syncthreads();
    for (int k0 = 0; k0 < n; k0 += IB) {
        const int kb = min(IB, n - k0);
        // ---- (1) diagonal block: wave 0, lane i owns row k0+i
        if (wid == 0) {
            T row[IB];
            #pragma unroll
            for (int c = 0; c < IB; ++c)
                row[c] = (lane < kb && c <= lane) ? S[(k0 + c) * LD + k0 + lane] : s_zero(T());
            int fail = 0;
            #pragma unroll
            for (int j = 0; j < IB; ++j) {
                if (j < kb && !fail) {
                    R d = s_real(row[j]);
                    #pragma unroll
                    for (int l = 0; l < IB; ++l)
                        if (l < j) d -= s_real(s_mul(row[l], s_conj(row[l])));
                    R dj = shfl_real(d, j);
                    if (!(dj > R(0))) { fail = k0 + j + 1; }
                    R sq = dj > R(0) ? sqrt(dj) : dj;
                    T rj[IB];
                    #pragma unroll
                    for (int l = 0; l < IB; ++l) rj[l] = shfl(row[l], j);
                    if (lane == j) row[j] = s_from_real(T(), sq);
                    if (lane > j && lane < kb) {
                        T sacc = row[j];
                        #pragma unroll
                        for (int l = 0; l < IB; ++l)
                            if (l < j) sacc = s_sub(sacc, s_mul(row[l], s_conj(rj[l])));
                        row[j] = s_mul(sacc, s_from_real(T(), R(1) / sq));
                    }
                }
            }
            if (lane < kb) {
                #pragma unroll
                for (int c = 0; c < IB; ++c)
                    if (c <= lane) S[(k0 + c) * LD + k0 + lane] = row[c];
            }
            if (lane == 0 && fail) s_fail = fail;
        }
        __syncthreads();
        if (s_fail) break;
        // ---- (2) panel: x D^H = a, one row per thread
        const int r0 = k0 + kb, m = n - r0;
        __shared__ T rdiag[IB];
        if (tid < kb) rdiag[tid] = s_div(s_from_real(T(), 1), S[(k0 + tid) * LD + k0 + tid]);
        __syncthreads();
        for (int i = tid; i < m; i += NT) {
            T x[IB];
            #pragma unroll
            for (int j = 0; j < IB; ++j) {
                if (j < kb) {
                    T sacc = S[(k0 + j) * LD + r0 + i];
                    #pragma unroll
                    for (int l = 0; l < IB; ++l)
                        if (l < j) sacc = s_sub(sacc, s_mul(x[l], s_conj(S[(k0 + l) * LD + k0 + j])));
                    x[j] = s_mul(sacc, rdiag[j]);
                } else {
                    x[j] = s_zero(T());
                }
            }
            #pragma unroll
            for (int j = 0; j < IB; ++j)
                if (j < kb) S[(k0 + j) * LD + r0 + i] = x[j];
        }
        __syncthreads();
        // ---- (3) trailing lower triangle, 4x4 blocks
        const int nbk = (m + 3) / 4;
        const int total = nbk * (nbk + 1) / 2;
        for (int t = tid; t < total; t += NT) {
            int bi = (int)((sqrtf(8.f * t + 1.f) - 1.f) * 0.5f);
            while ((bi + 1) * (bi + 2) / 2 <= t) ++bi;
            while (bi * (bi + 1) / 2 > t) --bi;
            const int bj = t - bi * (bi + 1) / 2;
            const int i0 = r0 + bi * 4, j0 = r0 + bj * 4;
            T acc[4][4];
            #pragma unroll
            for (int u = 0; u < 4; ++u)
                #pragma unroll
                for (int v = 0; v < 4; ++v) acc[u][v] = s_zero(T());
            #pragma unroll 4
            for (int l = 0; l < kb; ++l) {
                const T* col = S + (k0 + l) * LD;
                T ri[4], rc[4];
                #pragma unroll
                for (int u = 0; u < 4; ++u) {
                    ri[u] = (i0 + u < n) ? col[i0 + u] : s_zero(T());
                    rc[u] = (j0 + u < n) ? s_conj(col[j0 + u]) : s_zero(T());
                }
                #pragma unroll
                for (int u = 0; u < 4; ++u)
                    #pragma unroll
                    for (int v = 0; v < 4; ++v) acc[u][v] = s_add(acc[u][v], s_mul(ri[u], rc[v]));
            }
            #pragma unroll
            for (int v = 0; v < 4; ++v)
                #pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int ii = i0 + u, jj = j0 + v;
                    if (ii < n && jj < n && ii >= jj) S[jj * LD + ii] = s_sub(S[jj * LD + ii], acc[u][v]);
                }
        }
        __syncthreads();
    }
    {
        constexpr int CPI = NT / NS;
        const int r = tid % NS, cb = tid / NS;
        #pragma unroll 8
        for (int c = cb; c < NS; c += CPI)
            if (c < n && r < n && r >= c) {
                if (UPPER) A[c + (i64)r * lda] = s_conj(S[c * LD + r]);
                else A[r + (i64)c * lda] = S[c * LD + r];
            }
    }
    if (tid == 0 && s_fail && info)
        atomicCAS(reinterpret_cast<unsigned long long*>(info), 0ull, (unsigned long long)(s_fail + info_off));
}

template <typename T>
static void small(char uplo, int n, T* A, i64 lda, i64* info, i64 off, hipStream_t s) {
    constexpr int NS = ns_of<T>();
    if (uplo == 'U')
        hipLaunchKernelGGL((potrf_small_kernel<T, NS, true>), dim3(1), dim3(NT), 0, s, n, A, lda, info, off);
    else
        hipLaunchKernelGGL((potrf_small_kernel<T, NS, false>), dim3(1), dim3(NT), 0, s, n, A, lda, info, off);
    HIP_LAUNCH_CHECK();
}

template <typename T>
static void herk_lower(char uplo, i64 n, i64 k, const T* P, i64 ldp, T* C, i64 ldc, hipStream_t s) {
    // C -= P P^H (Lower) or C -= P^H P (Upper, P stored k x n), stored triangle only
    GemmCall c;
    c.m = n; c.n = n; c.k = k;
    c.alpha_re = -1; c.beta_re = 1;
    const char ct = scalar_traits<T>::is_complex ? 'C' : 'T';
    if (uplo == 'L') { c.transA = 'N'; c.transB = ct; }
    else { c.transA = ct; c.transB = 'N'; }
    c.A = P; c.lda = ldp; c.B = P; c.ldb = ldp; c.C = C; c.ldc = ldc;
    c.mask.mode = uplo == 'L' ? 1 : 2;
    if constexpr (scalar_traits<T>::is_complex) gemm_complex<T>(c, s);
    else gemm_real<T>(c, s);
}

template <typename T>
void potrf_tile(char uplo, int n, T* A, i64 lda, i64* info, hipStream_t s) {
    if (info) zero_words(info, 1, s);
    if (n <= 0) return;
    if constexpr (std::is_same<T, double>::value) {
        if (uplo == 'L') {
            // diagonal blocks (<= 512) by the one-CU LDS kernel, panel by the
            // blocked-inverse MFMA trsm, trailing triangle by the masked GEMM
            static const int DB = [] {
                const char* e = getenv("SLATE_AMD_POTRF_DIAG");
                const int v = e ? atoi(e) : 512;   // standalone 256 is faster (487 vs 567 us) but dpotrf n=32768 end to end: 52.4 (512) vs 50.8 TF/s (256)
                return (v >= 32 && v <= 512 && v % 32 == 0) ? v : 256;
            }();
            for (int k0 = 0; k0 < n; k0 += DB) {
                const int kb = std::min(DB, n - k0);
                T* Akk = A + k0 + (i64)k0 * lda;
                potrf_fast(kb, Akk, lda, info, k0, s);
                const int m = n - k0 - kb;
                if (m <= 0) break;
                T* P = A + (k0 + kb) + (i64)k0 * lda;
                trsm_rlt_fast(m, kb, 1.0, Akk, lda, P, lda, false, s);
                herk_lower<T>('L', m, kb, P, lda, A + (k0 + kb) + (i64)(k0 + kb) * lda, lda, s);
            }
            return;
        }
    }
    constexpr int NS = ns_of<T>();
    const char ct = scalar_traits<T>::is_complex ? 'C' : 'T';
    const T one = s_from_real(T(), 1);
    for (int k0 = 0; k0 < n; k0 += NS) {
        const int kb = std::min(NS, n - k0);
        T* Akk = A + k0 + (i64)k0 * lda;
        small<T>(uplo, kb, Akk, lda, info, k0, s);
        const int m = n - k0 - kb;
        if (m <= 0) break;
        if (uplo == 'L') {
            T* P = A + (k0 + kb) + (i64)k0 * lda;               // m x kb below the block
            trsm<T>('R', 'L', ct, 'N', m, kb, one, Akk, lda, P, lda, s);
            herk_lower<T>('L', m, kb, P, lda, A + (k0 + kb) + (i64)(k0 + kb) * lda, lda, s);
        } else {
            T* P = A + k0 + (i64)(k0 + kb) * lda;               // kb x m right of the block
            trsm<T>('L', 'U', ct, 'N', kb, m, one, Akk, lda, P, lda, s);
            herk_lower<T>('U', m, kb, P, lda, A + (k0 + kb) + (i64)(k0 + kb) * lda, lda, s);
        }
    }
}

template void potrf_tile<float>(char, int, float*, i64, i64*, hipStream_t);
template void potrf_tile<double>(char, int, double*, i64, i64*, hipStream_t);
template void potrf_tile<ccplx>(char, int, ccplx*, i64, i64*, hipStream_t);
template void potrf_tile<zcplx>(char, int, zcplx*, i64, i64*, hipStream_t);

}  // namespace slate_hip
