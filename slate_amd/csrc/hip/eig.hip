// Back-transformation of the bulge-chasing reflectors on gfx950 (replaces
// SLATE's unmtr_hb2st / unmbr_tb2bd host+device mix, src/unmtr_hb2st.cc,
// internal_unmtr_hb2st.cc).
//
// The reflectors of one sweep act on disjoint row ranges, so a whole sweep
// is one launch: grid = (reflectors of the sweep) x (column chunks), one
// wave per column (lanes along the reflector's rows -> coalesced loads),
// v staged in LDS.  Sweeps are applied last-to-first (Z := H Z).
#include "common.hpp"
#include "kernels.hpp"

namespace slate_hip {

namespace {
constexpr int RW = 4;        // waves per workgroup (one column each at a time)
constexpr int RCOLS = 64;    // columns per workgroup
}

template <typename T>
__global__ void __launch_bounds__(64 * RW)
apply_refl_kernel(i64 ncols, T* Z, i64 ldz, const T* V, i64 b, const T* tau, const i64* row, const i64* len,
                  i64 first, int conj_tau) {
    extern __shared__ unsigned char smem_raw[];
    T* vs = reinterpret_cast<T*>(smem_raw);
    const i64 k = first + blockIdx.x;
    const i64 r0 = row[k], L = len[k];
    T t = tau[k];
    if (conj_tau) t = s_conj(t);
    if (s_is_zero(t)) return;
    for (i64 i = threadIdx.x; i < L; i += 64 * RW) vs[i] = V[k * b + i];
    __syncthreads();
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const i64 c0 = (i64)blockIdx.y * RCOLS;
    const i64 c1 = min(ncols, c0 + RCOLS);
    for (i64 c = c0 + wv; c < c1; c += RW) {
        T* z = Z + r0 + c * ldz;
        T w = s_zero(T());
        for (i64 i = lane; i < L; i += 64) w = s_add(w, s_mul(s_conj(vs[i]), z[i]));
        w = wave_sum(w);
        w = s_mul(t, w);
        for (i64 i = lane; i < L; i += 64) z[i] = s_sub(z[i], s_mul(vs[i], w));
    }
}

template <typename T>
void apply_refl_batch(i64 ncols, T* Z, i64 ldz, const T* V, i64 b, const T* tau, const i64* row, const i64* len,
                      i64 first, i64 count, bool conj_tau, hipStream_t s) {
    if (count <= 0 || ncols <= 0) return;
    dim3 grid((unsigned)count, (unsigned)((ncols + RCOLS - 1) / RCOLS));
    hipLaunchKernelGGL(apply_refl_kernel<T>, grid, dim3(64 * RW), sizeof(T) * b, s, ncols, Z, ldz, V, b, tau,
                       row, len, first, conj_tau ? 1 : 0);
    HIP_LAUNCH_CHECK();
}

#define INST(T) \
    template void apply_refl_batch<T>(i64, T*, i64, const T*, i64, const T*, const i64*, const i64*, i64, i64, \
                                      bool, hipStream_t);
INST(float) INST(double) INST(ccplx) INST(zcplx)
#undef INST

}  // namespace slate_hip
