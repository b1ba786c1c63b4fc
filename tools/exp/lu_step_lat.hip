// Latency breakdown of the LU base-step kernel on gfx950: launch N back-to-back
// dependent launches of each variant and time them with hipEvents.
#include <cstdio>
#include <vector>
#include "../../slate_amd/csrc/hip/getrf.hip"

using namespace slate_hip;

__global__ void k_empty(double* A) { if (threadIdx.x == 9999) A[0] = 1; }

__global__ void __launch_bounds__(256) k_rows(double* A, long lda, int w) {
    long i = (long)blockIdx.x * 256 + threadIdx.x;
    double a[32];
    #pragma unroll
    for (int c = 0; c < 32; ++c) if (c < w) a[c] = A[i + c * lda];
    #pragma unroll
    for (int c = 0; c < 32; ++c) if (c < w) A[i + c * lda] = a[c] * 1.0000001;
}

__global__ void __launch_bounds__(256) k_rows_reduce(double* A, long lda, int w, double* part) {
    __shared__ double sv[256];
    long i = (long)blockIdx.x * 256 + threadIdx.x;
    double a[32];
    double pv = threadIdx.x < gridDim.x ? part[threadIdx.x] : -1;
    #pragma unroll
    for (int c = 0; c < 32; ++c) if (c < w) a[c] = A[i + c * lda];
    sv[threadIdx.x] = pv;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) { if (threadIdx.x < o) sv[threadIdx.x] = fmax(sv[threadIdx.x], sv[threadIdx.x + o]); __syncthreads(); }
    double m = sv[0];
    #pragma unroll
    for (int c = 0; c < 32; ++c) if (c < w) A[i + c * lda] = a[c] - m * 1e-30;
    if (threadIdx.x == 0) part[blockIdx.x] = fabs(a[1]);
}

int main() {
    const long m = 32768, lda = 32768;
    const int n = 32;
    double* A; void* work; long* ipiv; long* info;
    HIP_CHECK(hipMalloc(&A, sizeof(double) * lda * n));
    HIP_CHECK(hipMalloc(&work, getrf_work_bytes()));
    HIP_CHECK(hipMalloc(&ipiv, sizeof(long) * n));
    HIP_CHECK(hipMalloc(&info, sizeof(long)));
    HIP_CHECK(hipMemset(work, 0, getrf_work_bytes()));
    std::vector<double> h(lda * n);
    for (size_t i = 0; i < h.size(); ++i) h[i] = (double)((i * 2654435761u) % 1000) / 1000.0 - 0.5;
    HIP_CHECK(hipMemcpy(A, h.data(), sizeof(double) * h.size(), hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    const int REP = 330;
    auto timeit = [&](const char* name, auto&& launch) {
        for (int r = 0; r < 10; ++r) launch(r);
        hipDeviceSynchronize();
        hipEventRecord(e0);
        for (int r = 0; r < REP; ++r) launch(r);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1);
        printf("%-28s %8.2f us / launch\n", name, ms * 1000.f / REP);
    };
    for (int G : {128, 32}) {
        long mm = (long)G * 256;
        printf("G = %d (m = %ld)\n", G, mm);
        timeit("empty", [&](int) { hipLaunchKernelGGL(k_empty, dim3(G), dim3(256), 0, 0, A); });
        timeit("rows load/store", [&](int) { hipLaunchKernelGGL(k_rows, dim3(G), dim3(256), 0, 0, A, lda, 32); });
        timeit("rows + partial reduce", [&](int) {
            hipLaunchKernelGGL(k_rows_reduce, dim3(G), dim3(256), 0, 0, A, lda, 32, (double*)work); });
        timeit("getrf_base_step", [&](int r) {
            int j = r % 33;
            hipLaunchKernelGGL(getrf_base_step<double>, dim3(G), dim3(256), 0, 0, mm, 0, 32, j, A, lda, ipiv, 0L,
                               info, 0L, work, 1.0, false); });
    }
    return 0;
}
