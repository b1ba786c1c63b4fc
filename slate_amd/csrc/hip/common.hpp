// Common definitions for the CDNA4 (gfx950) HIP kernels of slate_amd.
//
// Everything here is written for one target only: MI355X / gfx950
// (64-lane wavefronts, MFMA f64/f32 16x16x4, 160 KiB LDS per CU, 8 XCDs).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdexcept>
#include <string>

namespace slate_hip {

using i64 = int64_t;

typedef double d4 __attribute__((ext_vector_type(4)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef double d2 __attribute__((ext_vector_type(2)));
typedef float f2v __attribute__((ext_vector_type(2)));

// Plain POD complex types (layout-compatible with std::complex / torch complex).
struct zcplx { double re, im; };
struct ccplx { float re, im; };

#define HIP_CHECK(expr)                                                        \
    do {                                                                       \
        hipError_t _e = (expr);                                                \
        if (_e != hipSuccess)                                                  \
            throw std::runtime_error(std::string("HIP error: ") +              \
                                     hipGetErrorString(_e) + " at " +          \
                                     __FILE__ + ":" + std::to_string(__LINE__)); \
    } while (0)

#define HIP_LAUNCH_CHECK() HIP_CHECK(hipGetLastError())

// Zero n 8-byte words with a kernel instead of hipMemsetAsync: inside a
// hipGraph capture a memset becomes a memset node, and on this runtime such
// nodes replay with stale parameters (the potrf info words came back as
// bytes 0x08 / 0x10 after the first replay, tools/probe/graph_time.py);
// kernel nodes replay exactly.
__global__ void zero_words_kernel(unsigned long long* p, long long n);
inline void zero_words(void* p, long long n, hipStream_t s) {
    if (n <= 0) return;
    hipLaunchKernelGGL(zero_words_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s,
                       static_cast<unsigned long long*>(p), n);
    HIP_LAUNCH_CHECK();
}

// ---------------------------------------------------------------------------
// Scalar helpers usable for real and complex element types.
template <typename T> struct scalar_traits;
template <> struct scalar_traits<float> {
    using real = float; static constexpr bool is_complex = false;
};
template <> struct scalar_traits<double> {
    using real = double; static constexpr bool is_complex = false;
};
template <> struct scalar_traits<ccplx> {
    using real = float; static constexpr bool is_complex = true;
};
template <> struct scalar_traits<zcplx> {
    using real = double; static constexpr bool is_complex = true;
};

__host__ __device__ inline float  s_zero(float)  { return 0.f; }
__host__ __device__ inline double s_zero(double) { return 0.0; }
__host__ __device__ inline ccplx  s_zero(ccplx)  { return {0.f, 0.f}; }
__host__ __device__ inline zcplx  s_zero(zcplx)  { return {0.0, 0.0}; }

__host__ __device__ inline float  s_add(float a, float b)   { return a + b; }
__host__ __device__ inline double s_add(double a, double b) { return a + b; }
__host__ __device__ inline ccplx  s_add(ccplx a, ccplx b)   { return {a.re + b.re, a.im + b.im}; }
__host__ __device__ inline zcplx  s_add(zcplx a, zcplx b)   { return {a.re + b.re, a.im + b.im}; }

__host__ __device__ inline float  s_sub(float a, float b)   { return a - b; }
__host__ __device__ inline double s_sub(double a, double b) { return a - b; }
__host__ __device__ inline ccplx  s_sub(ccplx a, ccplx b)   { return {a.re - b.re, a.im - b.im}; }
__host__ __device__ inline zcplx  s_sub(zcplx a, zcplx b)   { return {a.re - b.re, a.im - b.im}; }

__host__ __device__ inline float  s_mul(float a, float b)   { return a * b; }
__host__ __device__ inline double s_mul(double a, double b) { return a * b; }
__host__ __device__ inline ccplx  s_mul(ccplx a, ccplx b) {
    return {a.re * b.re - a.im * b.im, a.re * b.im + a.im * b.re};
}
__host__ __device__ inline zcplx  s_mul(zcplx a, zcplx b) {
    return {a.re * b.re - a.im * b.im, a.re * b.im + a.im * b.re};
}

__host__ __device__ inline float  s_conj(float a)  { return a; }
__host__ __device__ inline double s_conj(double a) { return a; }
__host__ __device__ inline ccplx  s_conj(ccplx a)  { return {a.re, -a.im}; }
__host__ __device__ inline zcplx  s_conj(zcplx a)  { return {a.re, -a.im}; }

__host__ __device__ inline float  s_real(float a)  { return a; }
__host__ __device__ inline double s_real(double a) { return a; }
__host__ __device__ inline float  s_real(ccplx a)  { return a.re; }
__host__ __device__ inline double s_real(zcplx a)  { return a.re; }

__host__ __device__ inline float  s_from_real(float, float r)   { return r; }
__host__ __device__ inline double s_from_real(double, double r) { return r; }
__host__ __device__ inline ccplx  s_from_real(ccplx, float r)   { return {r, 0.f}; }
__host__ __device__ inline zcplx  s_from_real(zcplx, double r)  { return {r, 0.0}; }

__host__ __device__ inline bool s_is_zero(float a)  { return a == 0.f; }
__host__ __device__ inline bool s_is_zero(double a) { return a == 0.0; }
__host__ __device__ inline bool s_is_zero(ccplx a)  { return a.re == 0.f && a.im == 0.f; }
__host__ __device__ inline bool s_is_zero(zcplx a)  { return a.re == 0.0 && a.im == 0.0; }

__device__ inline float  s_abs(float a)  { return fabsf(a); }
__device__ inline double s_abs(double a) { return fabs(a); }
__device__ inline float  s_abs(ccplx a)  { return hypotf(a.re, a.im); }
__device__ inline double s_abs(zcplx a)  { return hypot(a.re, a.im); }

// |re| + |im| (LAPACK cabs1) used for pivot search.
__device__ inline float  s_abs1(float a)  { return fabsf(a); }
__device__ inline double s_abs1(double a) { return fabs(a); }
__device__ inline float  s_abs1(ccplx a)  { return fabsf(a.re) + fabsf(a.im); }
__device__ inline double s_abs1(zcplx a)  { return fabs(a.re) + fabs(a.im); }

__device__ inline float  s_div(float a, float b)   { return a / b; }
__device__ inline double s_div(double a, double b) { return a / b; }
template <typename C, typename R>
__device__ inline C s_div_c(C a, C b) {
    // Smith's algorithm.
    R ar = a.re, ai = a.im, br = b.re, bi = b.im;
    if (fabs((double)br) >= fabs((double)bi)) {
        R r = bi / br, d = br + bi * r;
        return {(ar + ai * r) / d, (ai - ar * r) / d};
    } else {
        R r = br / bi, d = bi + br * r;
        return {(ar * r + ai) / d, (ai * r - ar) / d};
    }
}
__device__ inline ccplx s_div(ccplx a, ccplx b) { return s_div_c<ccplx, float>(a, b); }
__device__ inline zcplx s_div(zcplx a, zcplx b) { return s_div_c<zcplx, double>(a, b); }

// Wave-level (64 lanes) reductions.
template <typename R>
__device__ inline R wave_sum(R v) {
    #pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ inline zcplx wave_sum(zcplx v) { return zcplx{wave_sum(v.re), wave_sum(v.im)}; }
__device__ inline ccplx wave_sum(ccplx v) { return ccplx{wave_sum(v.re), wave_sum(v.im)}; }
template <typename R>
__device__ inline R wave_max(R v) {
    #pragma unroll
    for (int o = 32; o > 0; o >>= 1) { R w = __shfl_xor(v, o, 64); v = (w > v || w != w) ? w : v; }
    return v;
}

// Global index of a local row/col of a 2D block-cyclic distributed matrix.
// local index l (counting from the first local tile) -> global index.
__host__ __device__ inline i64 local_to_global(i64 l, i64 nb, int p, int pr) {
    i64 lt = l / nb;
    return (lt * p + pr) * nb + (l - lt * nb);
}

// Triangular/trapezoidal output mask for updates of a (possibly
// block-cyclic) Hermitian/triangular matrix: only elements with
// global_row >= global_col (Lower) or <= (Upper) are written.
struct TriMask {
    int mode = 0;          // 0 = full, 1 = lower (row >= col), 2 = upper (row <= col)
    int p = 1, pr = 0;     // process-grid rows / this rank's row
    int q = 1, pc = 0;     // process-grid cols / this rank's col
    i64 nb = 1 << 30;      // tile size (for block-cyclic mapping)
    i64 row_off = 0;       // local row of C(0,0) in this rank's local matrix
    i64 col_off = 0;       // local col of C(0,0)
    i64 diag_off = 0;      // global (row - col) offset: keep row - col >= -diag_off
    __host__ __device__ inline i64 grow(i64 r) const { return local_to_global(r + row_off, nb, p, pr); }
    __host__ __device__ inline i64 gcol(i64 c) const { return local_to_global(c + col_off, nb, q, pc); }
    __host__ __device__ inline bool keep(i64 r, i64 c) const {
        if (mode == 0) return true;
        i64 gr = grow(r), gc = gcol(c);
        return mode == 1 ? (gr + diag_off >= gc) : (gr <= gc + diag_off);
    }
    // true if no element of the block [r0,r1) x [c0,c1) is kept.
    __host__ __device__ inline bool skip_block(i64 r0, i64 r1, i64 c0, i64 c1) const {
        if (mode == 0) return false;
        if (mode == 1) return grow(r1 - 1) + diag_off < gcol(c0);
        return grow(r0) > gcol(c1 - 1) + diag_off;
    }
    // true if every element of the block is kept.
    __host__ __device__ inline bool full_block(i64 r0, i64 r1, i64 c0, i64 c1) const {
        if (mode == 0) return true;
        if (mode == 1) return grow(r0) + diag_off >= gcol(c1 - 1);
        return grow(r1 - 1) <= gcol(c0) + diag_off;
    }
};

// XCD-aware bijective remap of a 1-D block id: blocks b and b+8 share an
// XCD (round-robin dispatch), so give each XCD a contiguous chunk of the
// logical tile order (see guide T1, bijective variant).
// Bijective interleave of n rows in chunks of G: row b = q G + t -> t-th
// chunk (of ceil / floor n / G rows) + q.  Consecutive rows of a tile group
// land spread over the whole range: a group of a triangular-masked launch
// then holds long and short block rows alike (balanced XCD chunks).
__device__ inline int row_interleave(int b, int n, int G) {
    if (n <= G) return b;
    const int q = n / G, r = n % G;
    const int t = b % G, idx = b / G;
    const int base = (t < r) ? t * (q + 1) : r * (q + 1) + (t - r) * q;
    return base + idx;
}

__device__ inline int xcd_remap(int b, int nblocks) {
    const int NX = 8;
    if (nblocks < NX) return b;
    int q = nblocks / NX, r = nblocks % NX;
    int xcd = b % NX, idx = b / NX;
    int base = (xcd < r) ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
    return base + idx;
}

}  // namespace slate_hip
