// Host launchers for the MFMA GEMM kernels (see gemm.hpp); instantiated per
// dtype in gemm_{s,d,c,z}.hip so the builds run in parallel.
#pragma once
#include "gemm.hpp"
#include "launchers.hpp"

namespace slate_hip {

template <typename T, bool TA, bool TB, bool PTRS>
static void launch_real(const GemmArgs<T>& a, int batch, hipStream_t s) {
    // 128x128 macro tile, 8 waves (2x4) each 64x32, BK = 8: measured best of
    // the tile sweep in tools/exp/gemm_variants.hip on MI355X (more resident
    // waves per SIMD hide the f64 MFMA / LDS latency better than deeper K).
    constexpr int BM = 128, BN = 128, BK = (sizeof(T) == 8) ? 8 : 16;
    constexpr int WVM = 2, WVN = (sizeof(T) == 8) ? 4 : 2;
    i64 gm = (a.m + BM - 1) / BM, gn = (a.n + BN - 1) / BN;
    if (gm == 0 || gn == 0 || batch == 0) return;
    dim3 grid((unsigned)(gm * gn), (unsigned)batch);
    hipLaunchKernelGGL((gemm_real_kernel<T, TA, TB, BM, BN, BK, PTRS, WVM, WVN>), grid, dim3(64 * WVM * WVN), 0, s, a);
    HIP_LAUNCH_CHECK();
}

template <typename T>
static void dispatch_real(bool ta, bool tb, bool ptrs, const GemmArgs<T>& a, int batch, hipStream_t s) {
    if (ptrs) {
        if (!ta && !tb) launch_real<T, false, false, true>(a, batch, s);
        else if (!ta && tb) launch_real<T, false, true, true>(a, batch, s);
        else if (ta && !tb) launch_real<T, true, false, true>(a, batch, s);
        else launch_real<T, true, true, true>(a, batch, s);
    } else {
        if (!ta && !tb) launch_real<T, false, false, false>(a, batch, s);
        else if (!ta && tb) launch_real<T, false, true, false>(a, batch, s);
        else if (ta && !tb) launch_real<T, true, false, false>(a, batch, s);
        else launch_real<T, true, true, false>(a, batch, s);
    }
}

static inline bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

template <typename T>
void gemm_real(const GemmCall& c, hipStream_t s) {
    GemmArgs<T> a{};
    a.m = c.m; a.n = c.n; a.k = c.k;
    a.alpha = (T)c.alpha_re; a.beta = (T)c.beta_re;
    a.A = (const T*)c.A; a.lda = c.lda; a.strideA = c.strideA;
    a.B = (const T*)c.B; a.ldb = c.ldb; a.strideB = c.strideB;
    a.C = (T*)c.C; a.ldc = c.ldc; a.strideC = c.strideC;
    a.Aptrs = (const T* const*)c.Aptrs; a.Bptrs = (const T* const*)c.Bptrs; a.Cptrs = (T* const*)c.Cptrs;
    const int VEC = 16 / sizeof(T);
    const bool ptrs = c.Aptrs != nullptr;
    // vector loads need 16-byte aligned columns; pointer-array batches are
    // checked conservatively by the caller via c.vec_ok.
    a.vecA = c.vec_ok && (c.lda % VEC == 0) && (ptrs || (aligned16(c.A) && c.strideA % VEC == 0));
    a.vecB = c.vec_ok && (c.ldb % VEC == 0) && (ptrs || (aligned16(c.B) && c.strideB % VEC == 0));
    a.group_m = 8;
    a.mask = c.mask;
    a.remap = c.mask.mode == 0 ? 1 : 0;
    if (c.m <= 0 || c.n <= 0) return;
    dispatch_real<T>(c.transA != 'N', c.transB != 'N', ptrs, a, (int)c.batch, s);
}


}  // namespace slate_hip

namespace slate_hip {

template <typename T, char TA, char TB, bool PTRS>
static void launch_cplx(const GemmArgs<T>& a, int batch, hipStream_t s) {
    constexpr int BM = 64, BN = 64, BK = 16;
    i64 gm = (a.m + BM - 1) / BM, gn = (a.n + BN - 1) / BN;
    if (gm == 0 || gn == 0 || batch == 0) return;
    dim3 grid((unsigned)(gm * gn), (unsigned)batch);
    hipLaunchKernelGGL((gemm_complex_kernel<T, TA, TB, BM, BN, BK, PTRS>), grid, dim3(256), 0, s, a);
    HIP_LAUNCH_CHECK();
}

template <typename T, bool PTRS>
static void dispatch_cplx(char ta, char tb, const GemmArgs<T>& a, int batch, hipStream_t s) {
#define SLATE_CPLX_CASE(X, Y) if (ta == X && tb == Y) return launch_cplx<T, X, Y, PTRS>(a, batch, s);
    SLATE_CPLX_CASE('N', 'N') SLATE_CPLX_CASE('N', 'T') SLATE_CPLX_CASE('N', 'C')
    SLATE_CPLX_CASE('T', 'N') SLATE_CPLX_CASE('T', 'T') SLATE_CPLX_CASE('T', 'C')
    SLATE_CPLX_CASE('C', 'N') SLATE_CPLX_CASE('C', 'T') SLATE_CPLX_CASE('C', 'C')
#undef SLATE_CPLX_CASE
    throw std::invalid_argument("gemm: bad trans");
}

template <typename T>
void gemm_complex(const GemmCall& c, hipStream_t s) {
    using R = typename scalar_traits<T>::real;
    GemmArgs<T> a{};
    a.m = c.m; a.n = c.n; a.k = c.k;
    a.alpha = T{(R)c.alpha_re, (R)c.alpha_im}; a.beta = T{(R)c.beta_re, (R)c.beta_im};
    a.A = (const T*)c.A; a.lda = c.lda; a.strideA = c.strideA;
    a.B = (const T*)c.B; a.ldb = c.ldb; a.strideB = c.strideB;
    a.C = (T*)c.C; a.ldc = c.ldc; a.strideC = c.strideC;
    a.Aptrs = (const T* const*)c.Aptrs; a.Bptrs = (const T* const*)c.Bptrs; a.Cptrs = (T* const*)c.Cptrs;
    const int VEC = 16 / sizeof(T);
    const bool ptrs = c.Aptrs != nullptr;
    a.vecA = c.vec_ok && (c.lda % VEC == 0) && (ptrs || (aligned16(c.A) && c.strideA % VEC == 0));
    a.vecB = c.vec_ok && (c.ldb % VEC == 0) && (ptrs || (aligned16(c.B) && c.strideB % VEC == 0));
    a.group_m = 8;
    a.mask = c.mask;
    a.remap = c.mask.mode == 0 ? 1 : 0;
    if (c.m <= 0 || c.n <= 0) return;
    if (ptrs) dispatch_cplx<T, true>(c.transA, c.transB, a, (int)c.batch, s);
    else dispatch_cplx<T, false>(c.transA, c.transB, a, (int)c.batch, s);
}


}  // namespace slate_hip
