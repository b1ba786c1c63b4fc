// Host -> device and device -> device byte copies of the native runtime BY
// KERNEL.  A copy-engine write into device memory whose lines a kernel on
// another XCD read earlier was not seen by the next kernel on this stack
// (gfx950: eight XCDs with their own L2): the first potrf_grid of a process
// got a received diagonal tile with stale lines in the triangular inverse
// (tools/probe/scal_probe.cc, profiles/r4/native_first_call.md).  A kernel
// that reads the source and stores the destination keeps every write on the
// normal L2 write-back / invalidate path of kernel boundaries.
#include <cstring>
#include <mutex>
#include <vector>

#include "native_rt.hpp"

namespace slate_amd {
namespace native {

__global__ void __launch_bounds__(256)
copy_words_kernel(const unsigned long long* __restrict__ src, unsigned long long* __restrict__ dst, size_t nw) {
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < nw; i += (size_t)gridDim.x * 256) dst[i] = src[i];
}

__global__ void __launch_bounds__(256)
copy_bytes_kernel(const unsigned char* __restrict__ src, unsigned char* __restrict__ dst, size_t nb) {
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < nb; i += (size_t)gridDim.x * 256) dst[i] = src[i];
}

static void launch_copy(void* d, const void* s, size_t bytes, hipStream_t st) {
    if (!bytes) return;
    const bool words = ((reinterpret_cast<uintptr_t>(d) | reinterpret_cast<uintptr_t>(s) | bytes) & 7) == 0;
    const size_t n = words ? bytes / 8 : bytes;
    const unsigned g = (unsigned)std::min<size_t>((n + 255) / 256, 4096);
    if (words)
        hipLaunchKernelGGL(copy_words_kernel, dim3(g), dim3(256), 0, st,
                           static_cast<const unsigned long long*>(s), static_cast<unsigned long long*>(d), n);
    else
        hipLaunchKernelGGL(copy_bytes_kernel, dim3(g), dim3(256), 0, st, static_cast<const unsigned char*>(s),
                           static_cast<unsigned char*>(d), n);
    NHIP(hipGetLastError());
}

// pinned staging buffer (grown on demand; one upload at a time: the caller's
// stream is synchronised before the buffer is reused)
static std::mutex g_pin_mu;
static void* g_pin = nullptr;
static size_t g_pin_cap = 0;

void upload(void* d, const void* h, size_t bytes, hipStream_t s) {
    if (!bytes) {
        NHIP(hipStreamSynchronize(s));
        return;
    }
    std::lock_guard<std::mutex> g(g_pin_mu);
    if (g_pin_cap < bytes) {
        if (g_pin) NHIP(hipHostFree(g_pin));
        g_pin_cap = std::max(bytes, (size_t)1 << 20);
        NHIP(hipHostMalloc(&g_pin, g_pin_cap, hipHostMallocDefault));
    }
    std::memcpy(g_pin, h, bytes);
    void* dp = nullptr;
    NHIP(hipHostGetDevicePointer(&dp, g_pin, 0));
    launch_copy(d, dp, bytes, s);
    NHIP(hipStreamSynchronize(s));
}

void dcopy(void* d, const void* s, size_t bytes, hipStream_t st) { launch_copy(d, s, bytes, st); }

__global__ void __launch_bounds__(256) zero_words_kernel(unsigned long long* __restrict__ d, size_t nw) {
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < nw; i += (size_t)gridDim.x * 256) d[i] = 0ull;
}
__global__ void __launch_bounds__(256) zero_bytes_kernel(unsigned char* __restrict__ d, size_t nb) {
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < nb; i += (size_t)gridDim.x * 256) d[i] = 0;
}

void dzero(void* d, size_t bytes, hipStream_t st) {
    if (!bytes || !d) return;
    const bool words = ((reinterpret_cast<uintptr_t>(d) | bytes) & 7) == 0;
    const size_t n = words ? bytes / 8 : bytes;
    const unsigned g = (unsigned)std::min<size_t>((n + 255) / 256, 4096);
    if (words)
        hipLaunchKernelGGL(zero_words_kernel, dim3(g), dim3(256), 0, st, static_cast<unsigned long long*>(d), n);
    else
        hipLaunchKernelGGL(zero_bytes_kernel, dim3(g), dim3(256), 0, st, static_cast<unsigned char*>(d), n);
    NHIP(hipGetLastError());
}

// dst[:, didx[c]] = src[:, sidx[c]], columns of mw 4-byte words
__global__ void __launch_bounds__(256)
copy_cols_kernel(const unsigned* __restrict__ src, i64 lds, const i64* __restrict__ sidx, unsigned* __restrict__ dst,
                 i64 ldd, const i64* __restrict__ didx, i64 mw, i64 ncols) {
    for (i64 c = blockIdx.y; c < ncols; c += gridDim.y) {
        const unsigned* a = src + sidx[c] * lds;
        unsigned* b = dst + didx[c] * ldd;
        for (i64 i = (i64)blockIdx.x * 256 + threadIdx.x; i < mw; i += (i64)gridDim.x * 256) b[i] = a[i];
    }
}

void copy_cols(void* dst, i64 ldd, const i64* didx, const void* src, i64 lds, const i64* sidx, i64 m, size_t esize,
               i64 ncols, hipStream_t s) {
    if (ncols <= 0 || m <= 0) return;
    const size_t w = esize / 4;
    std::vector<i64> h(2 * (size_t)ncols);
    std::memcpy(h.data(), sidx, sizeof(i64) * ncols);
    std::memcpy(h.data() + ncols, didx, sizeof(i64) * ncols);
    Scratch ix(sizeof(i64) * h.size(), s);
    upload(ix.p, h.data(), sizeof(i64) * h.size(), s);
    const i64 mw = m * (i64)w;
    const unsigned gx = (unsigned)std::min<i64>((mw + 255) / 256, 64), gy = (unsigned)std::min<i64>(ncols, 16384);
    hipLaunchKernelGGL(copy_cols_kernel, dim3(gx, gy), dim3(256), 0, s, static_cast<const unsigned*>(src),
                       lds * (i64)w, ix.as<i64>(), static_cast<unsigned*>(dst), ldd * (i64)w, ix.as<i64>() + ncols, mw,
                       ncols);
    NHIP(hipGetLastError());
    NHIP(hipStreamSynchronize(s));
}

}  // namespace native
}  // namespace slate_amd
