// Hermitian band -> tridiagonal bulge chasing on the GPU (stage 2 of the
// two-stage eigensolver; SLATE runs it on host threads, src/hb2st.cc and
// internal_hebr.cc hebr1/hebr2/hebr3).
//
// Same task graph as the host pipeline (csrc/host/eig.cpp hb2st_mt): task t
// of sweep j generates the Householder reflector that annihilates column
// `col` below row s = e_prev + 1 and applies it two-sidedly over the window
// [col + 1, e + b]; sweep j may run task t once sweep j-1 has completed
// min(t + D, all) tasks, which keeps every pair of overlapping tasks in the
// sequential order (the result equals the sequential chase up to the
// floating-point summation order inside a task).
//
// MI355X mapping: one persistent workgroup (256 threads) per concurrently
// chased sweep.  Workgroups take sweeps in increasing order from an atomic
// ticket, so a workgroup only ever waits on a sweep taken earlier by a
// running workgroup: no co-residency assumption, no deadlock.  The
// dependency is a per-sweep progress counter published with an agent-scope
// release and polled with an agent-scope acquire (cross-XCD visible).
// Inside a task: the reflector by one wave (lanes over the k <= b rows),
// the left update one wave per column (lanes over rows: coalesced), the
// right update one thread per row.  The matrix is a dense n x n
// column-major copy holding both triangles (only the band is non-zero).
#include <cstdlib>
#include <cstring>

#include "common.hpp"
#include "kernels.hpp"

namespace slate_hip {

namespace {
constexpr int HT = 256;   // threads per workgroup
constexpr int HMAXB = 128;
constexpr i64 HLDS = 96 * 1024;   // bytes of the LDS staging buffer
}

template <typename T>
__global__ void __launch_bounds__(HT)
hb2st_kernel(i64 n, int b, T* __restrict__ A, i64 lda, T* __restrict__ V, T* __restrict__ tauv,
             i64* __restrict__ rowv, i64* __restrict__ lenv, const i64* __restrict__ sweep_ptr,
             const i64* __restrict__ ntask, int* ticket, int* done, i64 nsw, int D) {
    using R = typename scalar_traits<T>::real;
    __shared__ T v[HMAXB];
    extern __shared__ unsigned char hb_smem[];
    T* L = reinterpret_cast<T*>(hb_smem);           // staging buffer, HLDS bytes
    __shared__ T s_tau;
    __shared__ R s_beta;
    __shared__ int s_j;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    auto At = [&](i64 r, i64 c) -> T& { return A[r + c * lda]; };
    for (;;) {
        if (tid == 0) s_j = atomicAdd(ticket, 1);
        __syncthreads();
        const i64 j = s_j;
        __syncthreads();
        if (j >= nsw) return;
        const i64 nt = ntask[j];
        i64 s = j + 1, e = min(j + (i64)b, n - 1), col = j;
        for (i64 t = 0; t < nt; ++t) {
            if (j > 0) {
                const i64 need = min(t + (i64)D, ntask[j - 1]);
                // poll with relaxed loads (an acquire per poll would invalidate
                // the XCD's L2 every time, thrashing the working sweeps), then
                // ONE acquire fence
                if (tid == 0)
                    while (__hip_atomic_load(&done[j - 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < need)
                        __builtin_amdgcn_s_sleep(2);
                __syncthreads();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");   // every wave sees the producer's writes
            }
            if (t > 0) { s = e + 1; e = min(e + (i64)b, n - 1); }
            const int k = (int)(e - s + 1);
            // ---- reflector (wave 0): x = A(s..e, col)
            if (w == 0) {
                T x0 = s_zero(T());
                R xn2 = 0;
                for (int r = lane; r < k; r += 64) {
                    const T x = At(s + r, col);
                    v[r] = x;
                    if (r == 0) x0 = x;
                    else xn2 += s_real(s_mul(s_conj(x), x));
                }
                xn2 = wave_sum(xn2);
                x0 = wave_sum(x0);                              // only lane 0 contributed
                const R ar = s_real(x0);
                R ai = 0;
                if constexpr (scalar_traits<T>::is_complex) ai = x0.im;
                T tau;
                R beta;
                bool trivial = (xn2 == R(0) && ai == R(0));
                if (trivial) {
                    tau = s_zero(T());
                    beta = ar;
                } else {
                    beta = -copysign(sqrt(ar * ar + ai * ai + xn2), ar);
                    if constexpr (scalar_traits<T>::is_complex) tau = T{(beta - ar) / beta, -ai / beta};
                    else tau = (beta - ar) / beta;
                }
                // v = x / (alpha - beta), v[0] = 1
                T den = x0;
                if constexpr (scalar_traits<T>::is_complex) den.re -= beta;
                else den -= beta;
                for (int r = lane; r < k; r += 64) {
                    if (r == 0) v[0] = s_from_real(T(), R(1));
                    else if (!trivial) v[r] = s_div(v[r], den);
                }
                if (lane == 0) { s_tau = tau; s_beta = beta; }
            }
            __syncthreads();
            const T tau = s_tau;
            const i64 lo = col + 1, hi = min(n - 1, e + (i64)b);
            if (!s_is_zero(tau)) {
                // ---- left: A(s..e, c) -= v (conj(tau) v^H A(s..e, c)), c in [lo, hi].
                // Column chunks staged in LDS (one bulk coalesced load: every
                // load in flight at once), a wave per column, bulk store.
                const T ct = s_conj(tau);
                const i64 cw = max<i64>(1, min<i64>(hi - lo + 1, HLDS / ((i64)k * (i64)sizeof(T))));
                for (i64 c0 = lo; c0 <= hi; c0 += cw) {
                    const int nc = (int)min<i64>(cw, hi - c0 + 1);
                    for (int idx = tid; idx < k * nc; idx += HT) {
                        const int r = idx % k, c = idx / k;
                        L[idx] = At(s + r, c0 + c);
                    }
                    __syncthreads();
                    for (int c = w; c < nc; c += HT / 64) {
                        T acc = s_zero(T());
                        for (int r = lane; r < k; r += 64) acc = s_add(acc, s_mul(s_conj(v[r]), L[c * k + r]));
                        acc = s_mul(ct, wave_sum(acc));
                        for (int r = lane; r < k; r += 64) L[c * k + r] = s_sub(L[c * k + r], s_mul(v[r], acc));
                    }
                    __syncthreads();
                    for (int idx = tid; idx < k * nc; idx += HT) {
                        const int r = idx % k, c = idx / k;
                        At(s + r, c0 + c) = L[idx];
                    }
                    __syncthreads();
                }
                // ---- right: A(r, s..e) -= (tau A(r, s..e) v) v^H, r in [lo, hi]:
                // row chunks staged in LDS ([c][r]: a thread per row reads
                // consecutive banks)
                const i64 rw = max<i64>(1, min<i64>(hi - lo + 1, min<i64>(HT, HLDS / ((i64)k * (i64)sizeof(T)))));
                for (i64 r0 = lo; r0 <= hi; r0 += rw) {
                    const int nr = (int)min<i64>(rw, hi - r0 + 1);
                    for (int idx = tid; idx < k * nr; idx += HT) {
                        const int r = idx % nr, c = idx / nr;
                        L[idx] = At(r0 + r, s + c);
                    }
                    __syncthreads();
                    if (tid < nr) {
                        T y = s_zero(T());
                        for (int c = 0; c < k; ++c) y = s_add(y, s_mul(L[c * nr + tid], v[c]));
                        y = s_mul(y, tau);
                        for (int c = 0; c < k; ++c) L[c * nr + tid] = s_sub(L[c * nr + tid], s_mul(y, s_conj(v[c])));
                    }
                    __syncthreads();
                    for (int idx = tid; idx < k * nr; idx += HT) {
                        const int r = idx % nr, c = idx / nr;
                        At(r0 + r, s + c) = L[idx];
                    }
                    __syncthreads();
                }
            }
            __syncthreads();
            // ---- annihilated column / row, reflector slot
            const R beta = s_beta;
            const i64 slot = sweep_ptr[j] + t;
            for (int r = tid; r < k; r += HT) {
                const T val = (r == 0) ? s_from_real(T(), beta) : s_zero(T());
                At(s + r, col) = val;
                At(col, s + r) = val;
            }
            for (int r = tid; r < b; r += HT) V[slot * b + r] = (r < k) ? v[r] : s_zero(T());
            if (tid == 0) { tauv[slot] = tau; rowv[slot] = s; lenv[slot] = k; }
            __syncthreads();                                    // all waves' stores issued and complete
            if (tid == 0)                                        // one release: writes back this XCD's L2
                __hip_atomic_store(&done[j], (int)(t + 1), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
            col = s;
        }
    }
}

template <typename T>
void hb2st_device(i64 n, int b, T* A, i64 lda, T* V, T* tau, i64* row, i64* len, const i64* sweep_ptr,
                  const i64* ntask, int* work, i64 nsw, int nwg, hipStream_t s) {
    if (nsw <= 0) return;
    if (b > HMAXB) throw std::invalid_argument("hb2st_device: bandwidth > 128");
    // work = [ticket, done[0..nsw)] zero-initialised by the caller
    static bool attr = false;
    if (!attr) {
        HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&hb2st_kernel<T>),
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)HLDS));
        attr = true;
    }
    // The chase hands windows between workgroups on different XCDs: with
    // the default (L2-cached, non-coherent across XCDs) memory every hand-off
    // writes back and invalidates a whole L2.  SLATE_AMD_HB2ST_MEM=uncached
    // (default) or finegrained runs on a coherent working copy instead.
    static const int mode = [] {
        const char* e = getenv("SLATE_AMD_HB2ST_MEM");
        if (!e || !strcmp(e, "uncached")) return 2;
        return strcmp(e, "finegrained") == 0 ? 1 : 0;
    }();
    T* W = A;
    const size_t bytes = sizeof(T) * (size_t)lda * (size_t)n;
    if (mode) {
        HIP_CHECK(hipExtMallocWithFlags(reinterpret_cast<void**>(&W), bytes,
                                        mode == 2 ? hipDeviceMallocUncached : hipDeviceMallocFinegrained));
        HIP_CHECK(hipMemcpyAsync(W, A, bytes, hipMemcpyDeviceToDevice, s));
    }
    hipLaunchKernelGGL(hb2st_kernel<T>, dim3((unsigned)nwg), dim3(HT), HLDS, s, n, b, W, lda, V, tau, row, len,
                       sweep_ptr, ntask, work, work + 1, nsw, 4);
    HIP_LAUNCH_CHECK();
    if (mode) {
        HIP_CHECK(hipMemcpyAsync(A, W, bytes, hipMemcpyDeviceToDevice, s));
        HIP_CHECK(hipStreamSynchronize(s));
        HIP_CHECK(hipFree(W));
    }
}

#define INST(T) \
    template void hb2st_device<T>(i64, int, T*, i64, T*, T*, i64*, i64*, const i64*, const i64*, int*, i64, int, \
                                  hipStream_t);
INST(float) INST(double) INST(ccplx) INST(zcplx)
#undef INST

}  // namespace slate_hip
