// Local norm contributions for gfx950 (device_genorm.cu,
// device_henorm.cu, device_synorm.cu, device_trnorm.cu; one kernel family
// with uplo / diag / hermitian flags instead of four copies).
//
// Column pass: one workgroup per column (grid-strided), 256 threads reduce
// over the column's rows -> colout[j] = max|a| ('M'), sum|a| ('1'), or the
// LAPACK (scale, sumsq) pair ('F', 2 values per column).  For symmetric /
// Hermitian storage the mirrored off-diagonal contribution of a one-/inf-norm
// is atomically added to rowout[i].  Row pass ('I' of a general or
// trapezoidal block): threads own rows, columns split over grid.y chunks,
// atomicAdd of each chunk's partial row sum.  The caller (distributed
// driver) maps local columns/rows to global indices and all-reduces.
#include "common.hpp"
#include "kernels.hpp"

namespace slate_hip {

namespace {
__device__ inline bool keep(char uplo, i64 i, i64 j) {
    return uplo == 'L' ? i >= j : (uplo == 'U' ? i <= j : true);
}
template <typename R> __device__ inline R nanmax(R a, R b) { return (a != a || b > a) ? (b != b ? b : (a != a ? a : b)) : a; }
template <typename R> __device__ inline R nmax(R a, R b) {
    if (a != a) return a;
    if (b != b) return b;
    return a > b ? a : b;
}
template <typename R>
__device__ inline void ssq_add(R& scale, R& sumsq, R v) {
    if (v != R(0)) {
        if (scale < v) { sumsq = R(1) + sumsq * (scale / v) * (scale / v); scale = v; }
        else sumsq += (v / scale) * (v / scale);
    } else if (v != v) { scale = v; }
}
template <typename R>
__device__ inline void ssq_combine(R& s1, R& q1, R s2, R q2) {
    if (s2 != s2 || s1 != s1) { s1 = s1 != s1 ? s1 : s2; return; }
    if (s1 >= s2) { if (s1 > 0) q1 += q2 * (s2 / s1) * (s2 / s1); }
    else { q1 = q2 + q1 * (s1 / s2) * (s1 / s2); s1 = s2; }
}
}  // namespace

template <typename T, typename R>
__global__ void __launch_bounds__(256)
norm_col_kernel(char norm, char uplo, bool unit, int herm, i64 m, i64 n, const T* A, i64 lda,
                R* colout, R* rowout) {
    __shared__ R s1[256], s2[256];
    for (i64 j = blockIdx.x; j < n; j += gridDim.x) {
        R acc = 0, sc = 0, sq = 1;
        for (i64 i = threadIdx.x; i < m; i += 256) {
            if (!keep(uplo, i, j)) continue;
            // herm 2: Hermitian -- only the real part of the diagonal is referenced (LAPACK lanhe)
            R v = (i == j && unit) ? R(1) : (i == j && herm == 2) ? fabs(s_real(A[i + j * lda])) : s_abs(A[i + j * lda]);
            if (norm == 'M') acc = nmax(acc, v);
            else if (norm == 'F') {
                R w = (herm && i != j) ? v : v;
                ssq_add(sc, sq, w);
                if (herm && i != j) ssq_add(sc, sq, w);
            } else {
                acc += v;
                if (herm && i != j) atomicAdd(&rowout[i], v);
            }
        }
        s1[threadIdx.x] = (norm == 'F') ? sc : acc;
        s2[threadIdx.x] = sq;
        __syncthreads();
        for (int o = 128; o > 0; o >>= 1) {
            if (threadIdx.x < o) {
                if (norm == 'M') s1[threadIdx.x] = nmax(s1[threadIdx.x], s1[threadIdx.x + o]);
                else if (norm == 'F') {
                    R a = s1[threadIdx.x], b = s2[threadIdx.x];
                    ssq_combine(a, b, s1[threadIdx.x + o], s2[threadIdx.x + o]);
                    s1[threadIdx.x] = a; s2[threadIdx.x] = b;
                } else s1[threadIdx.x] += s1[threadIdx.x + o];
            }
            __syncthreads();
        }
        if (threadIdx.x == 0) {
            if (norm == 'F') { colout[2 * j] = s1[0]; colout[2 * j + 1] = s2[0]; }
            else colout[j] = s1[0];
        }
        __syncthreads();
    }
}

template <typename T, typename R>
__global__ void norm_row_kernel(char uplo, bool unit, i64 m, i64 n, const T* A, i64 lda, R* rowout, i64 chunk) {
    i64 i = (i64)blockIdx.x * 256 + threadIdx.x;
    if (i >= m) return;
    i64 j0 = (i64)blockIdx.y * chunk, j1 = min(n, j0 + chunk);
    R acc = 0;
    for (i64 j = j0; j < j1; ++j) {
        if (!keep(uplo, i, j)) continue;
        acc += (i == j && unit) ? R(1) : s_abs(A[i + j * lda]);
    }
    if (acc != R(0) || acc != acc) atomicAdd(&rowout[i], acc);
}

template <typename T, typename R>
void genorm(char norm, char uplo, char diag, int herm, i64 m, i64 n, const T* A, i64 lda, R* out,
            hipStream_t s) {
    // out layout: [ colout (n, or 2n for 'F') | rowout (m) ]  -- zeroed by caller
    if (m <= 0 || n <= 0) return;
    const bool unit = diag == 'U';
    R* colout = out;
    R* rowout = out + (norm == 'F' ? 2 * n : n);
    if (norm == 'I' && !herm) {
        i64 chunk = 256;
        dim3 grid((unsigned)((m + 255) / 256), (unsigned)((n + chunk - 1) / chunk));
        hipLaunchKernelGGL((norm_row_kernel<T, R>), grid, dim3(256), 0, s, uplo, unit, m, n, A, lda, rowout, chunk);
    } else {
        char nm = (norm == 'I') ? '1' : norm;
        unsigned g = (unsigned)std::min<i64>(n, 65535);
        hipLaunchKernelGGL((norm_col_kernel<T, R>), dim3(g), dim3(256), 0, s, nm, uplo, unit, herm, m, n, A, lda,
                           colout, rowout);
    }
    HIP_LAUNCH_CHECK();
}

template void genorm<float, float>(char, char, char, int, i64, i64, const float*, i64, float*, hipStream_t);
template void genorm<double, double>(char, char, char, int, i64, i64, const double*, i64, double*, hipStream_t);
template void genorm<ccplx, float>(char, char, char, int, i64, i64, const ccplx*, i64, float*, hipStream_t);
template void genorm<zcplx, double>(char, char, char, int, i64, i64, const zcplx*, i64, double*, hipStream_t);

}  // namespace slate_hip
