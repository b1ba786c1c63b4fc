// Single-tile Cholesky (potrf) for gfx950 -- the panel kernel of the
// distributed potrf (replaces the vendor `lapack::potrf` device call of
// src/internal/internal_potrf.cc:72).
//
// One 512-thread workgroup factors an n x n tile held in global memory
// (L2-resident: a 512^2 fp64 tile is 2 MiB < 4 MiB XCD L2), right-looking
// with IB = 16 column blocks:
//   1. the 16x16 diagonal block is factored by ONE wave in registers
//      (lane i owns row i; row j broadcast with __shfl) -- no barriers;
//   2. the panel below is solved row-per-thread against the diagonal block
//      (broadcast LDS reads) and staged k-major in LDS;
//   3. the trailing lower triangle is updated with 4x4 register blocks per
//      thread from the LDS panel (lower-triangle block enumeration, so no
//      thread works on the strictly-upper part).
// Upper is handled as the conjugate transpose of Lower (accessor swap).
// info (1-based first non-positive pivot, 0 on success) is written to a
// device int64 so the factorization DAG never syncs the host.
#include "common.hpp"
#include "kernels.hpp"

namespace slate_hip {

namespace {
constexpr int IB = 16;
constexpr int NT = 512;

template <typename T, bool UPPER>
struct Acc {
    T* A; i64 lda;
    __device__ inline T get(i64 i, i64 j) const {
        return UPPER ? s_conj(A[j + i * lda]) : A[i + j * lda];
    }
    __device__ inline void set(i64 i, i64 j, T v) const {
        if (UPPER) A[j + i * lda] = s_conj(v); else A[i + j * lda] = v;
    }
};

template <typename T>
__device__ inline T shfl(T v, int src) {
    if constexpr (scalar_traits<T>::is_complex) {
        T r;
        r.re = __shfl(v.re, src, 64);
        r.im = __shfl(v.im, src, 64);
        return r;
    } else {
        return __shfl(v, src, 64);
    }
}
}  // namespace

template <typename T, bool UPPER>
__global__ void __launch_bounds__(NT)
potrf_tile_kernel(int n, T* __restrict__ Aptr, i64 lda, i64* info, int lds_panel_rows) {
    using R = typename scalar_traits<T>::real;
    extern __shared__ __align__(16) unsigned char smem_raw[];
    T* Dl = reinterpret_cast<T*>(smem_raw);                 // IB x IB (row-major [r][c])
    T* Lp = Dl + IB * IB;                                    // [IB][lds_panel_rows] k-major panel
    __shared__ int s_fail;
    const Acc<T, UPPER> a{Aptr, lda};
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    if (tid == 0) s_fail = 0;
    __syncthreads();

    for (int k0 = 0; k0 < n; k0 += IB) {
        const int kb = min(IB, n - k0);
        // ---- 1. diagonal block in wave 0 registers ---------------------
        if (wid == 0) {
            T row[IB];
            #pragma unroll
            for (int c = 0; c < IB; ++c)
                row[c] = (lane < kb && c <= lane) ? a.get(k0 + lane, k0 + c) : s_zero(T());
            int fail = 0;
            #pragma unroll
            for (int j = 0; j < IB; ++j) {
                if (j < kb) {
                    // lane j: d = row[j] - sum_{l<j} |row[l]|^2 ; broadcast row j
                    R d = s_real(row[j]);
                    #pragma unroll
                    for (int l = 0; l < IB; ++l)
                        if (l < j) { T v = row[l]; d -= s_real(s_mul(v, s_conj(v))); }
                    R dj = __shfl(d, j, 64);
                    if (!(dj > R(0))) { if (!fail) fail = k0 + j + 1; dj = R(1); }
                    R sq = sqrt(dj);
                    T rj[IB];
                    #pragma unroll
                    for (int l = 0; l < IB; ++l) rj[l] = shfl(row[l], j);
                    if (lane == j) row[j] = s_from_real(T(), sq);
                    if (lane > j && lane < kb) {
                        T s = row[j];
                        #pragma unroll
                        for (int l = 0; l < IB; ++l)
                            if (l < j) s = s_sub(s, s_mul(row[l], s_conj(rj[l])));
                        row[j] = s_mul(s, s_from_real(T(), R(1) / sq));
                    }
                }
            }
            if (lane < kb) {
                #pragma unroll
                for (int c = 0; c < IB; ++c) {
                    if (c <= lane) a.set(k0 + lane, k0 + c, row[c]);
                    Dl[lane * IB + c] = (c <= lane) ? row[c] : s_zero(T());
                }
            }
            if (lane == 0 && fail && !s_fail) s_fail = fail;
        }
        __syncthreads();
        if (s_fail) break;
        // ---- 2. panel solve: x * D^H = a (row per thread) ------------------
        const int r0 = k0 + kb, m = n - r0;
        for (int i = tid; i < m; i += NT) {
            T x[IB];
            #pragma unroll
            for (int j = 0; j < IB; ++j) {
                if (j < kb) {
                    T s = a.get(r0 + i, k0 + j);
                    #pragma unroll
                    for (int l = 0; l < IB; ++l)
                        if (l < j) s = s_sub(s, s_mul(x[l], s_conj(Dl[j * IB + l])));
                    x[j] = s_div(s, Dl[j * IB + j]);
                } else {
                    x[j] = s_zero(T());
                }
            }
            #pragma unroll
            for (int j = 0; j < IB; ++j) {
                if (j < kb) a.set(r0 + i, k0 + j, x[j]);
                if (i < lds_panel_rows) Lp[j * lds_panel_rows + i] = x[j];
            }
        }
        __syncthreads();
        // ---- 3. trailing update, lower triangle, 4x4 blocks ------------------
        const int nbk = (m + 3) / 4;
        const int total = nbk * (nbk + 1) / 2;
        const bool in_lds = m <= lds_panel_rows;
        for (int t = tid; t < total; t += NT) {
            int bi = (int)((sqrtf(8.f * t + 1.f) - 1.f) * 0.5f);
            while ((bi + 1) * (bi + 2) / 2 <= t) ++bi;
            while (bi * (bi + 1) / 2 > t) --bi;
            const int bc = t - bi * (bi + 1) / 2;
            const int i0 = bi * 4, c0 = bc * 4;
            T acc[4][4];
            #pragma unroll
            for (int u = 0; u < 4; ++u)
                #pragma unroll
                for (int v = 0; v < 4; ++v) acc[u][v] = s_zero(T());
            for (int l = 0; l < kb; ++l) {
                T ri[4], rc[4];
                #pragma unroll
                for (int u = 0; u < 4; ++u) {
                    int ii = i0 + u, cc = c0 + u;
                    if (in_lds) {
                        ri[u] = ii < m ? Lp[l * lds_panel_rows + ii] : s_zero(T());
                        rc[u] = cc < m ? s_conj(Lp[l * lds_panel_rows + cc]) : s_zero(T());
                    } else {
                        ri[u] = ii < m ? a.get(r0 + ii, k0 + l) : s_zero(T());
                        rc[u] = cc < m ? s_conj(a.get(r0 + cc, k0 + l)) : s_zero(T());
                    }
                }
                #pragma unroll
                for (int u = 0; u < 4; ++u)
                    #pragma unroll
                    for (int v = 0; v < 4; ++v) acc[u][v] = s_add(acc[u][v], s_mul(ri[u], rc[v]));
            }
            #pragma unroll
            for (int v = 0; v < 4; ++v) {
                const int cc = c0 + v;
                if (cc >= m) continue;
                #pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int ii = i0 + u;
                    if (ii < m && ii >= cc) a.set(r0 + ii, r0 + cc, s_sub(a.get(r0 + ii, r0 + cc), acc[u][v]));
                }
            }
        }
        __syncthreads();
    }
    if (tid == 0 && info) *info = s_fail;
}

template <typename T>
void potrf_tile(char uplo, int n, T* A, i64 lda, i64* info, hipStream_t s) {
    if (n <= 0) {
        if (info) HIP_CHECK(hipMemsetAsync(info, 0, sizeof(i64), s));
        return;
    }
    // stage the panel in LDS when it fits (<= 128 KiB total)
    const size_t budget = 128 * 1024 - IB * IB * sizeof(T);
    int rows = (int)std::min<size_t>((size_t)n, budget / (IB * sizeof(T)));
    size_t shmem = (IB * IB + (size_t)IB * rows) * sizeof(T);
    if (uplo == 'U')
        hipLaunchKernelGGL((potrf_tile_kernel<T, true>), dim3(1), dim3(NT), shmem, s, n, A, lda, info, rows);
    else
        hipLaunchKernelGGL((potrf_tile_kernel<T, false>), dim3(1), dim3(NT), shmem, s, n, A, lda, info, rows);
    HIP_LAUNCH_CHECK();
}

template void potrf_tile<float>(char, int, float*, i64, i64*, hipStream_t);
template void potrf_tile<double>(char, int, double*, i64, i64*, hipStream_t);
template void potrf_tile<ccplx>(char, int, ccplx*, i64, i64*, hipStream_t);
template void potrf_tile<zcplx>(char, int, zcplx*, i64, i64*, hipStream_t);

}  // namespace slate_hip
