// On-device matrix generation (slate_matgen, matgen/*.cc): every rank fills
// its local block-cyclic buffer from the counter-based Philox stream keyed
// by GLOBAL (i, j) -- identical values to the host generator, independent
// of the grid -- without ever staging the matrix through the host.
#include "common.hpp"
#include "kernels.hpp"
#include "philox.hpp"

namespace slate_hip {

template <typename T>
__global__ void matgen_kernel(int kind, uint64_t seed, i64 mloc, i64 nloc, T* A, i64 lda, i64 m, i64 n,
                              i64 mb, int p, int pr, i64 nb, int q, int pc, i64 row0, i64 col0, double scale) {
    i64 li = (i64)blockIdx.x * 256 + threadIdx.x;
    if (li >= mloc) return;
    const i64 gi = local_to_global(li, mb, p, pr) + row0;
    for (i64 lj = blockIdx.y; lj < nloc; lj += gridDim.y) {
        const i64 gj = local_to_global(lj, nb, q, pc) + col0;
        double re, im;
        slate_rng::entry(kind, seed, gi, gj, m, n, scalar_traits<T>::is_complex, re, im);
        re *= scale; im *= scale;
        if constexpr (scalar_traits<T>::is_complex) {
            T v; v.re = (typename scalar_traits<T>::real)re; v.im = (typename scalar_traits<T>::real)im;
            A[li + lj * lda] = v;
        } else {
            A[li + lj * lda] = (T)re;
        }
    }
}

template <typename T>
void matgen(int kind, uint64_t seed, i64 mloc, i64 nloc, T* A, i64 lda, i64 m, i64 n,
            i64 mb, int p, int pr, i64 nb, int q, int pc, i64 row0, i64 col0, double scale, hipStream_t s) {
    if (mloc <= 0 || nloc <= 0) return;
    dim3 grid((unsigned)((mloc + 255) / 256), (unsigned)std::min<i64>(nloc, 8192));
    hipLaunchKernelGGL(matgen_kernel<T>, grid, dim3(256), 0, s, kind, seed, mloc, nloc, A, lda, m, n, mb, p, pr,
                       nb, q, pc, row0, col0, scale);
    HIP_LAUNCH_CHECK();
}

#define INST(T) template void matgen<T>(int, uint64_t, i64, i64, T*, i64, i64, i64, i64, int, int, i64, int, int, \
                                         i64, i64, double, hipStream_t);
INST(float) INST(double) INST(ccplx) INST(zcplx)
#undef INST

}  // namespace slate_hip
