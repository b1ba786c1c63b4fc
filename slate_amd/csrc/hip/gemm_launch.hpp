// Host launchers for the MFMA GEMM kernels (see gemm.hpp); instantiated per
// dtype in gemm_{s,d,c,z}.hip so the builds run in parallel.
#pragma once
#include <cstdlib>
#include "gemm.hpp"
#include "gemm_glds.hpp"
#include "launchers.hpp"
#include "workspace.hpp"

namespace slate_hip {

// ---------------------------------------------------------------- split-K
// Tall-skinny reductions (V^H C in QR, Gram matrices, the k = m reductions
// of the panel recursions) have a few output tiles and a very long k: one
// workgroup per tile would leave the chip idle.  Split k into chunks
// computed as a strided batch into a workspace, then one deterministic
// reduction kernel (fixed summation order -> bit-reproducible results).
template <typename T>
__global__ void splitk_reduce_kernel(i64 m, i64 n, int ks, const T* __restrict__ W, T alpha, T beta, T* C,
                                     i64 ldc, const int* gate) {
    if (gate && *gate == 0) return;
    const i64 i = (i64)blockIdx.x * 256 + threadIdx.x;
    if (i >= m) return;
    const i64 mn = m * n;
    for (i64 j = blockIdx.y; j < n; j += gridDim.y) {
        T acc = W[i + j * m];
        for (int s = 1; s < ks; ++s) acc = s_add(acc, W[s * mn + i + j * m]);
        T v = s_mul(alpha, acc);
        if (!s_is_zero(beta)) v = s_add(v, s_mul(beta, C[i + j * ldc]));
        C[i + j * ldc] = v;
    }
}

// below this many 128 x 128 tiles (x batch) fp64 GEMMs use 64 x 64 tiles:
// the trailing updates near the end of a factorization would otherwise leave
// each CU with one or two workgroups, too few waves to hide the MFMA / LDS
// latency (measured: masked 4096^2 x 512 update at 29 TF/s with 128 x 128).
// SLATE_AMD_GEMM_SMALL overrides (0 = always 128 x 128).
static inline i64 gemm_small_tiles() {
    static const i64 v = [] {
        const char* e = std::getenv("SLATE_AMD_GEMM_SMALL");
        return e ? (i64)std::atoll(e) : (i64)2048;
    }();
    return v;
}

template <typename T, typename Launch>
static bool gemm_splitk(const GemmCall& c, int tile, hipStream_t s, Launch&& launch) {
    if (!c.allow_split || c.batch != 1 || c.Aptrs || c.mask.mode != 0) return false;
    const i64 tiles = ((c.m + tile - 1) / tile) * ((c.n + tile - 1) / tile);
    // (b) fp64 outputs of at most 512 64 x 64 tiles (the 64 x 64 kernel: one
    // or two workgroups per CU) with a long K, e.g. the 64-row V^H Z products
    // of the eigensolver back-transforms (64 x 16384 x K, K up to n): split K
    // until there are ~1024 workgroups; the m n ks partial-sum traffic is
    // small next to the 2 m n k flops once k >= 4096
    const i64 t64 = ((c.m + 63) / 64) * ((c.n + 63) / 64);
    const bool wide = std::is_same<T, double>::value && t64 <= 512 && c.k >= 4096 && tiles < gemm_small_tiles();
    if (!wide && (tiles >= 256 || c.k < 2048 || c.k < 8 * std::max(c.m, c.n))) return false;
    i64 ks = wide ? std::min<i64>(c.k / 1024, (1024 + t64 - 1) / t64)
                  : std::min<i64>(c.k / 512, (512 + tiles - 1) / tiles);
    if (ks < 2) return false;
    const i64 kc = ((c.k + ks - 1) / ks + 63) / 64 * 64;
    const i64 full = c.k / kc, rem = c.k - full * kc;
    ks = full + (rem > 0 ? 1 : 0);
    T* W = static_cast<T*>(workspace(s, sizeof(T) * (size_t)c.m * c.n * ks, WS_P));
    GemmCall p = c;
    p.allow_split = false;
    p.alpha_re = 1; p.alpha_im = 0; p.beta_re = 0; p.beta_im = 0;
    p.C = W; p.ldc = c.m; p.strideC = c.m * c.n;
    p.k = kc; p.batch = full;
    const i64 sa = (c.transA == 'N') ? kc * c.lda : kc;
    const i64 sb = (c.transB == 'N') ? kc : kc * c.ldb;
    p.strideA = sa; p.strideB = sb;
    launch(p);
    if (rem > 0) {
        GemmCall r = p;
        r.batch = 1; r.k = rem; r.strideA = r.strideB = r.strideC = 0;
        r.A = static_cast<const T*>(c.A) + full * sa;
        r.B = static_cast<const T*>(c.B) + full * sb;
        r.C = W + full * c.m * c.n;
        launch(r);
    }
    T alpha, beta;
    if constexpr (scalar_traits<T>::is_complex) {
        using R = typename scalar_traits<T>::real;
        alpha = T{(R)c.alpha_re, (R)c.alpha_im}; beta = T{(R)c.beta_re, (R)c.beta_im};
    } else {
        alpha = (T)c.alpha_re; beta = (T)c.beta_re;
    }
    dim3 grid((unsigned)((c.m + 255) / 256), (unsigned)std::min<i64>(c.n, 1024));
    hipLaunchKernelGGL(splitk_reduce_kernel<T>, grid, dim3(256), 0, s, c.m, c.n, (int)ks, W, alpha, beta,
                       static_cast<T*>(c.C), c.ldc, c.gate);
    HIP_LAUNCH_CHECK();
    return true;
}


// Lower-triangular masks (the potrf/herk trailing updates) launch only the
// 8 x 8 super-tiles on or below the tile diagonal, XCD-remapped (remap = 2 in
// gemm_real_kernel).  Valid when no tile with bm < bn holds a kept element:
// global rows and columns grow with local ones, so it suffices that tile
// (min(bn - 1, gm - 1), bn) is empty for every bn >= 1 (exact host check,
// covers block-cyclic grids with p <= q such as 2 x 4).  Returns the block
// count, or 0 if not eligible.  SLATE_AMD_GEMM_TRI=0 disables it.  Measured
// (tools/exp/gemm_trimask.py, 128 x 128 tiles, k = 512): 31744 x 30720
// 59.0 -> 59.6 TF/s, 8192 x 7168 53.3 -> 54.7 TF/s; used for the 128 x 128
// variant only.
// triangular-masked launches that are not the compact triangle: XCD chunks
// over row-interleaved groups (3, balanced and L2-local) or the plain order
// (0); SLATE_AMD_GEMM_MASK_REMAP overrides
static inline int gemm_mask_remap() {
    static const int v = [] {
        const char* e = std::getenv("SLATE_AMD_GEMM_MASK_REMAP");
        return e ? std::atoi(e) : 3;
    }();
    return v;
}

// tile-order group height (block rows swept together); SLATE_AMD_GEMM_GROUP overrides 8
static inline int gemm_group() {
    static const int v = [] {
        const char* e = std::getenv("SLATE_AMD_GEMM_GROUP");
        const int g = e ? std::atoi(e) : 8;
        return g >= 1 ? g : 8;
    }();
    return v;
}

static inline bool gemm_tri_enabled() {
    const char* e = std::getenv("SLATE_AMD_GEMM_TRI");  // read per launch: tests and sweeps toggle it
    return !(e && e[0] == '0');
}

template <typename T>
static i64 tri_blocks(const GemmArgs<T>& a, int BM, int BN) {
    const TriMask& k = a.mask;
    if (!gemm_tri_enabled() || k.mode != 1 || BM != BN) return 0;
    const i64 gm = (a.m + BM - 1) / BM, gn = (a.n + BN - 1) / BN;
    for (i64 bn = 1; bn < gn; ++bn) {
        const i64 bm = std::min(bn - 1, gm - 1);
        const i64 r0 = bm * BM, c0 = bn * BN;
        if (!k.skip_block(r0, std::min(r0 + BM, a.m), c0, std::min(c0 + BN, a.n))) return 0;
    }
    const i64 gsm = (gm + 7) / 8, gsn = (gn + 7) / 8;
    i64 sup = 0;
    for (i64 J = 0; J < std::min(gsm, gsn); ++J) sup += gsm - J;
    return sup * 64;
}

// fp64 with K % 16 == 0 and 16-byte aligned operands: the LDS-DMA staged
// kernel (gemm_glds.hpp), 128 x 128 x 16, 2 x 4 waves, two LDS stages, two
// workgroups per CU.  Measured on MI355X against the register-staged kernel
// (tools/exp/dgemm_glds_r5.hip, profiles/r5/dgemm_glds.txt): 31744^2 x 512
// NT 61.1 -> 67.1 TF/s, x 1024 NT 63.8 -> 69.7, NN x 512 62.6 -> 65.8,
// 16384^2 x 4096 NN 68.9 -> 70.6, NT 65.3 -> 71.3; bit-identical results.
// SLATE_AMD_GEMM_GLDS=0 selects the register-staged kernel.
static inline bool gemm_glds_enabled() {
    static const bool v = [] {
        const char* e = std::getenv("SLATE_AMD_GEMM_GLDS");
        return !(e && e[0] == '0');
    }();
    return v;
}

// BM = 128: 128 x 128 tiles, NN on 4 x 2 waves (+0.7 % at 16384^2 x 4096 /
// 31744^2 x 512), else 2 x 4; BM = 64: 64 x 64 tiles on 2 x 2 waves, four
// workgroups per CU -- for outputs of fewer than 512 128 x 128 tiles
// (1024^2 x 1024: 15 -> 45 TF/s, 2048^2: 59 -> 64; profiles/r5/dgemm_glds_small.txt)
template <bool TA, bool TB, int BM>
static void launch_glds(const GemmArgs<double>& a, i64 nblk, int batch, hipStream_t s) {
    constexpr int BN = BM, WVM = BM == 64 ? 2 : (!TA && !TB) ? 4 : 2, WVN = BM == 64 ? 2 : 8 / WVM, S = 2,
                  OCC = BM == 64 ? 4 : 2;
    auto K = gemm_f64_glds_kernel<TA, TB, BM, BN, WVM, WVN, S, OCC>;
    constexpr size_t lds = glds_lds_bytes<BM, BN, TA, TB, S>();
    static const bool attr = [&] {
        return hipFuncSetAttribute((const void*)K, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) ==
               hipSuccess;
    }();
    (void)attr;
    hipLaunchKernelGGL(K, dim3((unsigned)nblk, (unsigned)batch), dim3(64 * WVM * WVN), lds, s, a);
    HIP_LAUNCH_CHECK();
}

// remap 4 (gemm.hpp stair_block): a lower mask whose kept blocks per block
// row are a prefix (block-cyclic lower triangles of a rank's local block:
// global rows and columns grow with local ones); the grid then holds only
// the kept blocks, so the resident workgroups stay within a few tile groups
// (L2 reuse) instead of spreading over every group the skipped blocks race
// through.  Measured on MI355X, the 2x4 dpotrf trailing update of rank 0
// (15872 x 7168 x 512, 47 % kept): see profiles/r5/masked_gemm_stair.txt.
// Returns the kept block count (0: not eligible).  SLATE_AMD_GEMM_STAIR=0
// disables.
template <typename T>
static i64 stair_blocks(GemmArgs<T>& a, int BM, int BN, int batch) {
    static const bool on = [] {
        const char* e = std::getenv("SLATE_AMD_GEMM_STAIR");
        return !(e && e[0] == '0');
    }();
    const TriMask& k = a.mask;
    if (!on || k.mode != 1 || batch != 1) return 0;
    const i64 gm = (a.m + BM - 1) / BM, gn = (a.n + BN - 1) / BN;
    const int G = a.group_m >= 1 ? a.group_m : 1;
    if (gm > GEMM_STAIR_MAX || gn > 65535 || gm * gn < 256 || (gm + G - 1) / G > GEMM_STAIR_GROUPS) return 0;
    i64 total = 0, prev = 0;
    for (i64 r = 0; r < gm; ++r) {
        const i64 r0 = r * BM, r1 = std::min(r0 + BM, a.m);
        // first skipped block column (skips are monotone in bn: gcol grows)
        i64 lo = 0, hi = gn;
        while (lo < hi) {
            const i64 mid = (lo + hi) / 2;
            const i64 c0 = mid * BN;
            if (k.skip_block(r0, r1, c0, std::min(c0 + BN, a.n))) hi = mid;
            else lo = mid + 1;
        }
        if (lo < prev) return 0;     // not a staircase
        a.ncol[r] = (unsigned short)lo;
        if (r % G == 0) a.gpre[r / G] = (unsigned)total;
        prev = lo;
        total += lo;
    }
    a.gpre[(gm + G - 1) / G] = (unsigned)total;
    return total;
}

template <typename T, bool TA, bool TB, bool PTRS>
static void launch_real(const GemmArgs<T>& a0, int batch, hipStream_t s) {
    GemmArgs<T> a = a0;
    if constexpr (sizeof(T) == 8) {
        const i64 g128 = ((a.m + 127) / 128) * ((a.n + 127) / 128) * batch;
        if (!PTRS && g128 < 512 && a.k > 0 && a.k % 16 == 0 && a.vecA && a.vecB && gemm_glds_enabled()) {
            const i64 gm = (a.m + 63) / 64, gn = (a.n + 63) / 64;
            if (gm == 0 || gn == 0 || batch == 0) return;
            i64 nb64 = gm * gn;
            if (i64 t = stair_blocks(a, 64, 64, batch)) { a.remap = 4; nb64 = t; }
            launch_glds<TA, TB, 64>(a, nb64, batch, s);
            return;
        }
        if (g128 < gemm_small_tiles() && !(a.k > 0 && a.k % 16 == 0 && a.vecA && a.vecB && gemm_glds_enabled())) {
            constexpr int BM = 64, BN = 64, BK = 8;
            const i64 gm = (a.m + BM - 1) / BM, gn = (a.n + BN - 1) / BN;
            if (gm == 0 || gn == 0 || batch == 0) return;
            // no compact triangle here: measured 4096 x 3072 x 512 masked,
            // 52.9 TF/s full grid vs 50.7 compact (tools/exp/gemm_trimask.py)
            hipLaunchKernelGGL((gemm_real_kernel<T, TA, TB, BM, BN, BK, PTRS, 2, 2>), dim3((unsigned)(gm * gn), (unsigned)batch),
                               dim3(256), 0, s, a);
            HIP_LAUNCH_CHECK();
            return;
        }
    }
    // 128x128 macro tile, 8 waves (2x4) each 64x32, BK = 8: measured best of
    // the tile sweep in tools/exp/gemm_variants.hip on MI355X (more resident
    // waves per SIMD hide the f64 MFMA / LDS latency better than deeper K).
    constexpr int BM = 128, BN = 128, BK = (sizeof(T) == 8) ? 8 : 16;
    constexpr int WVM = 2, WVN = (sizeof(T) == 8) ? 4 : 2;
    i64 gm = (a.m + BM - 1) / BM, gn = (a.n + BN - 1) / BN;
    if (gm == 0 || gn == 0 || batch == 0) return;
    i64 nblk = gm * gn;
    {
        // the exact staircase when it launches clearly fewer blocks than the
        // compact 8 x 8 super-tile triangle (block-cyclic grids: 3248 vs
        // 5824 blocks for the 2x4 step above; a one-rank triangle: ~3 %)
        const i64 t = tri_blocks(a, BM, BN);
        GemmArgs<T> b = a;
        const i64 t2 = stair_blocks(b, BM, BN, batch);
        if (t2 && (!t || t2 < t - t / 8)) { a = b; a.remap = 4; nblk = t2; }
        else if (t) { a.remap = 2; nblk = t; }
    }
    if constexpr (sizeof(T) == 8 && !PTRS) {
        if (a.k > 0 && a.k % 16 == 0 && a.vecA && a.vecB && gemm_glds_enabled()) {
            launch_glds<TA, TB, 128>(a, nblk, batch, s);
            return;
        }
    }
    // Two register stages for fp64 NN (tools/exp/gemm_pf_r5.hip on MI355X:
    // 31744^2 x 512 59.2 -> 62.9 TF/s, 16384^2 x 4096 63.5 -> 68.4 TF/s); the
    // NT form loses with it (61.3 -> 56.3 TF/s), so it keeps one.
    constexpr int PF = (sizeof(T) == 8 && !TA && !TB) ? 2 : 1;
    dim3 grid((unsigned)nblk, (unsigned)batch);
    hipLaunchKernelGGL((gemm_real_kernel<T, TA, TB, BM, BN, BK, PTRS, WVM, WVN, 2, PF>), grid, dim3(64 * WVM * WVN), 0, s,
                       a);
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
    if (c.m > 0 && c.n > 0 && gemm_splitk<T>(c, 128, s, [&](const GemmCall& p) { gemm_real<T>(p, s); }))
        return;
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
    a.group_m = gemm_group();
    a.mask = c.mask;
    a.remap = c.mask.mode == 0 ? 1 : gemm_mask_remap();
    a.gate = c.gate;
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
    if (c.m > 0 && c.n > 0 && gemm_splitk<T>(c, 64, s, [&](const GemmCall& p) { gemm_complex<T>(p, s); }))
        return;
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
    a.group_m = gemm_group();
    a.mask = c.mask;
    a.remap = c.mask.mode == 0 ? 1 : gemm_mask_remap();
    a.gate = c.gate;
    if (c.m <= 0 || c.n <= 0) return;
    if (ptrs) dispatch_cplx<T, true>(c.transA, c.transB, a, (int)c.batch, s);
    else dispatch_cplx<T, false>(c.transA, c.transB, a, (int)c.batch, s);
}


}  // namespace slate_hip
