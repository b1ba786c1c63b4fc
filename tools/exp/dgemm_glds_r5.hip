// LDS-DMA staged fp64 GEMM (csrc/hip/gemm_glds.hpp) against the production
// register-staged kernel (gemm.hpp, 128 x 128 x 8, 2 x 4 waves): numerics at
// ragged shapes, then interleaved timings at the potrf / getrf / dgemm shapes.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/exp/dgemm_glds_r5.hip -o tools/exp/dgemm_glds_r5.bin
#include "../../slate_amd/csrc/hip/gemm_glds.hpp"
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <random>
#include <string>
#include <vector>
using namespace slate_hip;

static float timed(void (*launch)(const GemmArgs<double>&), const GemmArgs<double>& a, int reps) {
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

template <bool TB, int PF>
void ref_launch(const GemmArgs<double>& a) {
    const int gm = (a.m + 127) / 128, gn = (a.n + 127) / 128;
    hipLaunchKernelGGL((gemm_real_kernel<double, false, TB, 128, 128, 8, false, 2, 4, 2, PF>), dim3(gm * gn, 1),
                       dim3(512), 0, 0, a);
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

struct Var { const char* name; void (*nt)(const GemmArgs<double>&); void (*nn)(const GemmArgs<double>&); };

template <bool TB>
void small_launch(const GemmArgs<double>& a) {
    const int gm = (a.m + 63) / 64, gn = (a.n + 63) / 64;
    hipLaunchKernelGGL((gemm_real_kernel<double, false, TB, 64, 64, 8, false, 2, 2, 2, 1>), dim3(gm * gn, 1), dim3(256),
                       0, 0, a);
}

int main(int argc, char** argv) {
    const bool small = argc > 1 && std::string(argv[1]) == "small";
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
    const Var big_vars[] = {
        {"glds 128x128 2x4 S2 occ2", glds_launch<true, 128, 128, 2, 4, 2, 2>, glds_launch<false, 128, 128, 4, 2, 2, 2>},
    };
    const Var small_vars[] = {
        {"64x64 register-staged", small_launch<true>, small_launch<false>},
        {"glds 128x128 2x4 S2 occ2", glds_launch<true, 128, 128, 2, 4, 2, 2>, glds_launch<false, 128, 128, 4, 2, 2, 2>},
        {"glds 64x64 2x2 S2 occ4", glds_launch<true, 64, 64, 2, 2, 2, 4>, glds_launch<false, 64, 64, 2, 2, 2, 4>},
        {"glds 64x64 2x2 S3 occ3", glds_launch<true, 64, 64, 2, 2, 3, 3>, glds_launch<false, 64, 64, 2, 2, 3, 3>},
        {"glds 128x64 2x2 S2 occ3", glds_launch<true, 128, 64, 2, 2, 2, 3>, glds_launch<false, 128, 64, 2, 2, 2, 3>},
    };
    const Var* vars_p = small ? small_vars : big_vars;
    const int nvars = small ? 5 : 1;
    struct VarList { const Var* b; const Var* e; const Var* begin() const { return b; } const Var* end() const { return e; } };
    const VarList vars{vars_p, vars_p + nvars};
    auto mk = [&](long m, long n, long k, bool tb, double alpha, double beta, double* c, long ldc) {
        GemmArgs<double> a{};
        a.m = m; a.n = n; a.k = k; a.alpha = alpha; a.beta = beta;
        a.A = A; a.lda = m + (m & 1); a.B = B; a.ldb = tb ? n + (n & 1) : k; a.C = c; a.ldc = ldc;
        a.vecA = a.vecB = 1; a.group_m = 8; a.remap = 1;
        return a;
    };
    // numerics: ragged m / n, both transposes, beta != 0, against the production kernel
    {
        struct Sh { long m, n, k; } sh[] = {{1000, 777, 256}, {129, 1, 16}, {4096, 4096, 512}, {333, 2049, 1024}};
        std::vector<double> h1(4096L * 4096), h2(4096L * 4096);
        for (const auto& s : sh)
            for (int tb = 0; tb < 2; ++tb) {
                const long ldc = 4096;
                for (const auto& v : vars) {
                    hipMemcpy(C2, C, ldc * s.n * 8, hipMemcpyDeviceToDevice);
                    auto a = mk(s.m, s.n, s.k, tb, -1.0, 0.5, C2, ldc);
                    if (tb) ref_launch<true, 1>(a); else ref_launch<false, 1>(a);
                    hipDeviceSynchronize();
                    hipMemcpy(h1.data(), C2, ldc * s.n * 8, hipMemcpyDeviceToHost);
                    hipMemcpy(C2, C, ldc * s.n * 8, hipMemcpyDeviceToDevice);
                    a = mk(s.m, s.n, s.k, tb, -1.0, 0.5, C2, ldc);
                    (tb ? v.nt : v.nn)(a);
                    hipError_t e = hipDeviceSynchronize();
                    hipMemcpy(h2.data(), C2, ldc * s.n * 8, hipMemcpyDeviceToHost);
                    double md = 0, mx = 0, outside = 0;
                    for (long j = 0; j < s.n; ++j)
                        for (long i = 0; i < ldc; ++i) {
                            const double x = h1[i + j * ldc], y = h2[i + j * ldc];
                            if (i < s.m) { md = std::max(md, std::fabs(x - y)); mx = std::max(mx, std::fabs(x)); }
                            else outside = std::max(outside, std::fabs(x - y));
                        }
                    printf("check %-26s %s %5ldx%5ldx%5ld rel %.3e outside %.1e %s\n", v.name, tb ? "NT" : "NN", s.m,
                           s.n, s.k, md / mx, outside, e == hipSuccess ? "ok" : hipGetErrorString(e));
                    fflush(stdout);
                }
            }
    }
    struct Shape { long m, n, k; bool tb; const char* what; };
    const Shape big_shapes[] = {
        {31744, 31744, 512, true, "trailing NT k=512"},
        {16384, 16384, 4096, false, "NN k=4096"},
    };
    const Shape small_shapes[] = {
        {8192, 8192, 1024, true, "tail NT 8192 k=1024"},
        {4096, 4096, 1024, true, "tail NT 4096 k=1024"},
        {2048, 2048, 1024, true, "tail NT 2048 k=1024"},
        {1024, 1024, 1024, true, "tail NT 1024 k=1024"},
        {4096, 4096, 512, true, "tail NT 4096 k=512"},
        {32768, 512, 512, true, "column NT 32768x512"},
        {16384, 1024, 1024, true, "column NT 16384x1024"},
        {32768, 1024, 512, true, "lookahead NT 32768x1024"},
        {8192, 8192, 512, false, "tail NN 8192 k=512"},
        {4096, 4096, 512, false, "tail NN 4096 k=512"},
        {32768, 512, 512, false, "column NN 32768x512"},
    };
    struct ShapeList { const Shape* b; const Shape* e; const Shape* begin() const { return b; } const Shape* end() const { return e; } };
    const ShapeList shapes = small ? ShapeList{small_shapes, small_shapes + 11} : ShapeList{big_shapes, big_shapes + 2};
    for (const auto& s : shapes) {
        const double fl = 2.0 * s.m * s.n * s.k;
        const int reps = std::max(5, (int)(1e12 / fl));
        auto a = mk(s.m, s.n, s.k, s.tb, -1.0, 1.0, C, N);
        for (int round = 0; round < 2; ++round) {
            float ms = timed(s.tb ? ref_launch<true, 1> : ref_launch<false, 2>, a, reps);
            printf("%-20s %ldx%ldx%ld %-26s: %8.3f ms %6.2f TF\n", s.what, s.m, s.n, s.k, "production", ms,
                   fl / ms / 1e9);
            for (const auto& v : vars) {
                ms = timed(s.tb ? v.nt : v.nn, a, reps);
                printf("%-20s %ldx%ldx%ld %-26s: %8.3f ms %6.2f TF\n", s.what, s.m, s.n, s.k, v.name, ms,
                       fl / ms / 1e9);
                fflush(stdout);
            }
        }
    }
    return 0;
}
