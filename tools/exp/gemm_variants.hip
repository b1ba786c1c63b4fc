// Tile-shape / occupancy exploration for the fp64 MFMA GEMM (standalone).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/exp/gemm_variants.hip -o tools/exp/gv.bin
#include "../../slate_amd/csrc/hip/gemm.hpp"
#include <vector>
#include <cstdio>
#include <random>
using namespace slate_hip;

template <bool TA, bool TB, int BM, int BN, int BK, int WVM, int WVN, int OCC>
float run(GemmArgs<double> a, int reps) {
    int gm = (a.m + BM - 1) / BM, gn = (a.n + BN - 1) / BN;
    dim3 grid(gm * gn, 1);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    hipLaunchKernelGGL((gemm_real_kernel<double, TA, TB, BM, BN, BK, false, WVM, WVN, OCC>), grid, dim3(64 * WVM * WVN), 0, 0, a);
    hipEventRecord(e0);
    for (int r = 0; r < reps; ++r)
        hipLaunchKernelGGL((gemm_real_kernel<double, TA, TB, BM, BN, BK, false, WVM, WVN, OCC>), grid, dim3(64 * WVM * WVN), 0, 0, a);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    return ms / reps;
}

int main() {
    const long N = 24576;
    double *A, *B, *C;
    hipMalloc(&A, N * 2048 * 8); hipMalloc(&B, N * 2048 * 8); hipMalloc(&C, N * N * 8);
    std::vector<double> h(N * 2048);
    std::mt19937_64 g(1); std::uniform_real_distribution<double> d(-1, 1);
    for (auto& x : h) x = d(g);
    hipMemcpy(A, h.data(), N * 2048 * 8, hipMemcpyHostToDevice);
    hipMemcpy(B, h.data(), N * 2048 * 8, hipMemcpyHostToDevice);
    hipMemset(C, 0, N * N * 8);
    auto mk = [&](long m, long n, long k, bool tb) {
        GemmArgs<double> a{}; a.m = m; a.n = n; a.k = k; a.alpha = -1; a.beta = 1;
        a.A = A; a.lda = m; a.B = B; a.ldb = tb ? n : k; a.C = C; a.ldc = m;
        a.vecA = a.vecB = 1; a.group_m = 8; a.remap = 1; return a; };
    for (long k : {512L, 1024L}) {
        double fl = 2.0 * N * N * k;
#define V(TA, TB, BM, BN, BK, WM, WN, OCC) { auto a = mk(N, N, k, TB); float ms = run<TA, TB, BM, BN, BK, WM, WN, OCC>(a, 4); \
        printf("%ldx%ldx%ld TA=%d TB=%d %dx%dx%d waves %dx%d occ %d: %.3f ms %.2f TF\n", N, N, k, TA, TB, BM, BN, BK, WM, WN, OCC, ms, fl / ms / 1e9); fflush(stdout); }
        V(false, true, 128, 128, 8, 2, 4, 2)
        V(false, true, 128, 128, 16, 2, 4, 2)
        V(false, true, 128, 128, 8, 2, 2, 2)
        V(false, true, 128, 128, 16, 2, 2, 2)
        V(false, true, 256, 128, 8, 4, 2, 1)
        V(false, true, 256, 128, 16, 4, 2, 1)
        V(false, true, 128, 256, 8, 2, 4, 1)
        V(false, true, 256, 256, 8, 4, 4, 1)
        V(false, true, 256, 256, 16, 4, 4, 1)
        V(false, false, 128, 128, 8, 2, 4, 2)
        V(false, false, 256, 128, 8, 4, 2, 1)
    }
    return 0;
}
