// Round-6 fp64 GEMM tile study at the potrf trailing shape (NT, k = 512 /
// 1024, beta = 1) and a square NN dgemm: the production LDS-DMA kernel
// (gemm_glds.hpp, 128 x 128, 2 x 4 waves, S2, occ 2) against 64 x 64-per-wave
// variants (4 waves per 128 x 128, 8 waves per 256 x 128 / 128 x 256), the
// group size of the tile order, s_setprio, and rocBLAS dgemm as the vendor
// reference point (measurement only -- the library never calls rocBLAS).
// Numerics: every variant against the production kernel at ragged shapes.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/exp/dgemm_r6.hip -lrocblas -o tools/exp/dgemm_r6.bin
#include "../../slate_amd/csrc/hip/gemm_glds.hpp"
#include <rocblas/rocblas.h>
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <random>
#include <string>
#include <vector>
using namespace slate_hip;

typedef void (*launch_t)(const GemmArgs<double>&);

static float timed(launch_t launch, const GemmArgs<double>& a, int reps) {
    launch(a);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    for (int r = 0; r < reps; ++r) launch(a);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    hipEventDestroy(e0);
    hipEventDestroy(e1);
    return ms / reps;
}

template <bool TB, int BM, int BN, int WVM, int WVN, int S, int OCC, int PRIO = 0, int G = 8>
void glds_launch(const GemmArgs<double>& a0) {
    GemmArgs<double> a = a0;
    a.group_m = G;
    auto K = gemm_f64_glds_kernel<false, TB, BM, BN, WVM, WVN, S, OCC, PRIO>;
    constexpr size_t lds = glds_lds_bytes<BM, BN, false, TB, S>();
    static bool init = false;
    if (!init) {
        hipFuncSetAttribute((const void*)K, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        init = true;
    }
    const int gm = (a.m + BM - 1) / BM, gn = (a.n + BN - 1) / BN;
    hipLaunchKernelGGL(K, dim3(gm * gn, 1), dim3(64 * WVM * WVN), lds, 0, a);
}

static rocblas_handle g_rb;
template <bool TB>
void rocblas_launch(const GemmArgs<double>& a) {
    const double al = a.alpha, be = a.beta;
    rocblas_dgemm(g_rb, rocblas_operation_none, TB ? rocblas_operation_transpose : rocblas_operation_none, a.m, a.n,
                  a.k, &al, a.A, a.lda, a.B, a.ldb, &be, a.C, a.ldc);
}

struct Var { const char* name; launch_t nt; launch_t nn; };

int main(int argc, char** argv) {
    rocblas_create_handle(&g_rb);
    rocblas_set_pointer_mode(g_rb, rocblas_pointer_mode_host);
    const long N = 32768, KMAX = 4096;
    double *A, *B, *C, *C2;
    hipMalloc(&A, N * KMAX * 8);
    hipMalloc(&B, N * KMAX * 8);
    hipMalloc(&C, N * N * 8);
    hipMalloc(&C2, 4096L * 4096 * 8);
    {
        std::vector<double> h(N * 64);
        std::mt19937_64 g(1);
        std::uniform_real_distribution<double> d(-1, 1);
        for (auto& x : h) x = d(g);
        for (long off = 0; off < N * KMAX; off += N * 64) {
            hipMemcpy(A + off, h.data(), N * 64 * 8, hipMemcpyHostToDevice);
            for (long i = 0; i < 7; ++i) std::swap(h[i * 1000], h[i * 1000 + 500]);
            hipMemcpy(B + off, h.data(), N * 64 * 8, hipMemcpyHostToDevice);
        }
        for (long off = 0; off < N * N; off += N * 64) hipMemcpy(C + off, h.data(), N * 64 * 8, hipMemcpyHostToDevice);
    }
    const Var vars[] = {
        {"prod 128x128 2x4 S2 o2 G8", glds_launch<true, 128, 128, 2, 4, 2, 2>, glds_launch<false, 128, 128, 4, 2, 2, 2>},
        {"128x128 2x4 S2 o2 G16", glds_launch<true, 128, 128, 2, 4, 2, 2, 0, 16>,
         glds_launch<false, 128, 128, 4, 2, 2, 2, 0, 16>},
        {"128x128 2x4 S2 o2 prio", glds_launch<true, 128, 128, 2, 4, 2, 2, 1>,
         glds_launch<false, 128, 128, 4, 2, 2, 2, 1>},
        {"128x128 2x2 S2 o2", glds_launch<true, 128, 128, 2, 2, 2, 2>, glds_launch<false, 128, 128, 2, 2, 2, 2>},
        {"128x128 2x2 S2 o2 prio", glds_launch<true, 128, 128, 2, 2, 2, 2, 1>,
         glds_launch<false, 128, 128, 2, 2, 2, 2, 1>},
        {"128x128 2x2 S3 o1", glds_launch<true, 128, 128, 2, 2, 3, 1>, glds_launch<false, 128, 128, 2, 2, 3, 1>},
        {"256x128 4x2 S2 o1", glds_launch<true, 256, 128, 4, 2, 2, 1>, glds_launch<false, 256, 128, 4, 2, 2, 1>},
        {"128x256 2x4 S2 o1", glds_launch<true, 128, 256, 2, 4, 2, 1>, glds_launch<false, 128, 256, 2, 4, 2, 1>},
        {"rocblas dgemm", rocblas_launch<true>, rocblas_launch<false>},
    };
    const int nvars = sizeof(vars) / sizeof(vars[0]);
    auto mk = [&](long m, long n, long k, bool tb, double alpha, double beta, double* c, long ldc) {
        GemmArgs<double> a{};
        a.m = m; a.n = n; a.k = k; a.alpha = alpha; a.beta = beta;
        a.A = A; a.lda = m + (m & 1); a.B = B; a.ldb = tb ? n + (n & 1) : k; a.C = c; a.ldc = ldc;
        a.vecA = a.vecB = 1; a.group_m = 8; a.remap = 1;
        return a;
    };
    {
        struct Sh { long m, n, k; } sh[] = {{1000, 777, 256}, {129, 1, 16}, {4096, 4096, 512}, {333, 2049, 1024}};
        std::vector<double> h1(4096L * 4096), h2(4096L * 4096);
        for (const auto& s : sh)
            for (int tb = 0; tb < 2; ++tb) {
                const long ldc = 4096;
                hipMemcpy(C2, C, ldc * s.n * 8, hipMemcpyDeviceToDevice);
                auto a = mk(s.m, s.n, s.k, tb, -1.0, 0.5, C2, ldc);
                (tb ? vars[0].nt : vars[0].nn)(a);
                hipDeviceSynchronize();
                hipMemcpy(h1.data(), C2, ldc * s.n * 8, hipMemcpyDeviceToHost);
                for (int v = 1; v < nvars; ++v) {
                    hipMemcpy(C2, C, ldc * s.n * 8, hipMemcpyDeviceToDevice);
                    a = mk(s.m, s.n, s.k, tb, -1.0, 0.5, C2, ldc);
                    (tb ? vars[v].nt : vars[v].nn)(a);
                    hipError_t e = hipDeviceSynchronize();
                    hipMemcpy(h2.data(), C2, ldc * s.n * 8, hipMemcpyDeviceToHost);
                    double md = 0, mx = 0, outside = 0;
                    for (long j = 0; j < s.n; ++j)
                        for (long i = 0; i < ldc; ++i) {
                            const double x = h1[i + j * ldc], y = h2[i + j * ldc];
                            if (i < s.m) { md = std::max(md, std::fabs(x - y)); mx = std::max(mx, std::fabs(x)); }
                            else outside = std::max(outside, std::fabs(x - y));
                        }
                    printf("check %-26s %s %5ldx%5ldx%5ld rel %.3e outside %.1e %s\n", vars[v].name, tb ? "NT" : "NN",
                           s.m, s.n, s.k, md / mx, outside, e == hipSuccess ? "ok" : hipGetErrorString(e));
                    fflush(stdout);
                }
            }
    }
    struct Shape { long m, n, k; bool tb; const char* what; };
    const Shape shapes[] = {
        {31744, 31744, 512, true, "trailing NT k=512"},
        {31744, 31744, 1024, true, "trailing NT k=1024"},
        {16384, 16384, 512, true, "trailing NT 16k k=512"},
        {16384, 16384, 4096, false, "NN k=4096"},
    };
    for (const auto& s : shapes) {
        const double fl = 2.0 * s.m * s.n * s.k;
        const int reps = std::max(5, (int)(1e12 / fl));
        auto a = mk(s.m, s.n, s.k, s.tb, -1.0, 1.0, C, N);
        for (int round = 0; round < 2; ++round)
            for (const auto& v : vars) {
                const float ms = timed(s.tb ? v.nt : v.nn, a, reps);
                printf("%-22s %ldx%ldx%ld %-26s: %8.3f ms %6.2f TF\n", s.what, s.m, s.n, s.k, v.name, ms, fl / ms / 1e9);
                fflush(stdout);
            }
    }
    rocblas_destroy_handle(g_rb);
    return 0;
}
