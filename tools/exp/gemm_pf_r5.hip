// Prefetch depth (PF 1 / 2) and tile-order group size of the production fp64
// GEMM (128 x 128 x 8, 2 x 4 waves) at the potrf / getrf trailing shapes.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/exp/gemm_pf_r5.hip -o tools/exp/gemm_pf_r5.bin
#include "../../slate_amd/csrc/hip/gemm.hpp"
#include <algorithm>
#include <cstdio>
#include <random>
#include <vector>
using namespace slate_hip;

template <bool TA, bool TB, int BM, int BN, int BK, int WVM, int WVN, int OCC, int PF>
float run(GemmArgs<double> a, int reps) {
    int gm = (a.m + BM - 1) / BM, gn = (a.n + BN - 1) / BN;
    dim3 grid(gm * gn, 1);
    auto K = gemm_real_kernel<double, TA, TB, BM, BN, BK, false, WVM, WVN, OCC, PF>;
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
        {31744, 31744, 1024, true, "trailing NT k=1024"},
        {16384, 16384, 512, true, "trailing NT 16k k=512"},
        {31744, 31744, 512, false, "trailing NN k=512"},
        {16384, 16384, 4096, false, "NN k=4096"},
    };
    for (const auto& s : shapes) {
        const double fl = 2.0 * s.m * s.n * s.k;
        const int reps = std::max(2, (int)(3e12 / fl));
        for (int g : {8, 4, 16}) {
            auto a = mk(s.m, s.n, s.k, s.tb, -1.0, 1.0);
            a.group_m = g;
#define V(PF) { float ms = s.tb ? run<false, true, 128, 128, 8, 2, 4, 2, PF>(a, reps) \
                                : run<false, false, 128, 128, 8, 2, 4, 2, PF>(a, reps); \
            printf("%-22s %ldx%ldx%ld group %2d PF %d: %8.3f ms %6.2f TF\n", s.what, s.m, s.n, s.k, g, PF, ms, \
                   fl / ms / 1e9); fflush(stdout); }
            V(1) V(2) V(1) V(2)
#undef V
        }
    }
    return 0;
}
