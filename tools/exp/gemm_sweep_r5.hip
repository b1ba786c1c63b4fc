// Tile / wave-layout / occupancy sweep of the fp64 MFMA GEMM at the potrf
// trailing-update shape (NT, k = 512) and a long-K NN shape, against the
// 77.4 TF/s bare-MFMA ceiling (profiles/r5/mfma_peak.txt).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/exp/gemm_sweep_r5.hip -o tools/exp/gemm_sweep_r5.bin
#include "../../slate_amd/csrc/hip/gemm.hpp"
#include <algorithm>
#include <cstdio>
#include <random>
#include <vector>
using namespace slate_hip;

template <bool TA, bool TB, int BM, int BN, int BK, int WVM, int WVN, int OCC>
float run(GemmArgs<double> a, int reps) {
    int gm = (a.m + BM - 1) / BM, gn = (a.n + BN - 1) / BN;
    dim3 grid(gm * gn, 1);
    auto K = gemm_real_kernel<double, TA, TB, BM, BN, BK, false, WVM, WVN, OCC>;
    hipLaunchKernelGGL(K, grid, dim3(64 * WVM * WVN), 0, 0, a);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    hipEventRecord(e0);
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(K, grid, dim3(64 * WVM * WVN), 0, 0, a);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    return ms / reps;
}

int main() {
    const long N = 32768, KMAX = 4096;
    double *A, *B, *C;
    hipMalloc(&A, N * KMAX * 8); hipMalloc(&B, N * KMAX * 8); hipMalloc(&C, N * N * 8);
    {
        std::vector<double> h(N * 64);
        std::mt19937_64 g(1); std::uniform_real_distribution<double> d(-1, 1);
        for (auto& x : h) x = d(g);
        for (long off = 0; off < N * KMAX; off += N * 64) {
            hipMemcpy(A + off, h.data(), N * 64 * 8, hipMemcpyHostToDevice);
            hipMemcpy(B + off, h.data(), N * 64 * 8, hipMemcpyHostToDevice);
        }
        for (long off = 0; off < N * N; off += N * 64) hipMemcpy(C + off, h.data(), N * 64 * 8, hipMemcpyHostToDevice);
    }
    auto mk = [&](long m, long n, long k, bool tb, double alpha, double beta) {
        GemmArgs<double> a{}; a.m = m; a.n = n; a.k = k; a.alpha = alpha; a.beta = beta;
        a.A = A; a.lda = m; a.B = B; a.ldb = tb ? n : k; a.C = C; a.ldc = N;
        a.vecA = a.vecB = 1; a.group_m = 8; a.remap = 1; return a; };
    struct Shape { long m, n, k; bool tb; const char* what; };
    const Shape shapes[] = {
        {31744, 31744, 512, true, "trailing NT k=512"},
        {16384, 16384, 4096, true, "NT k=4096"},
        {16384, 16384, 4096, false, "NN k=4096"},
    };
    for (const auto& s : shapes) {
        auto a = mk(s.m, s.n, s.k, s.tb, -1.0, 1.0);
        const double fl = 2.0 * s.m * s.n * s.k;
        const int reps = std::max(2, (int)(3e12 / fl));
#define V(BM, BN, BK, WM, WN, OCC) { float ms = s.tb ? run<false, true, BM, BN, BK, WM, WN, OCC>(a, reps) \
                                                   : run<false, false, BM, BN, BK, WM, WN, OCC>(a, reps); \
        printf("%-20s %ldx%ldx%ld %3dx%3dx%2d waves %dx%d occ %d: %8.3f ms %6.2f TF\n", s.what, s.m, s.n, s.k, \
               BM, BN, BK, WM, WN, OCC, ms, fl / ms / 1e9); fflush(stdout); }
        V(128, 128, 8, 2, 4, 2)
        V(128, 128, 16, 2, 4, 2)
        V(128, 128, 8, 4, 2, 2)
        V(128, 128, 8, 2, 2, 2)
        V(128, 128, 16, 2, 2, 2)
        V(256, 128, 8, 4, 2, 1)
        V(128, 256, 8, 2, 4, 1)
        V(256, 128, 16, 4, 2, 1)
        V(128, 128, 8, 2, 4, 3)
        V(128, 128, 8, 2, 4, 2)
#undef V
    }
    return 0;
}
