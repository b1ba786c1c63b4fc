// Python-free C++ use of slate_amd (include/slate_amd/slate_native.hh,
// libslate_amd_native.so): Cholesky, LU, GEMM and norms on a 2D block-cyclic
// grid, checked against host references; then the LAPACK-style C ABI; then
// an optional timing of potrf (argv[2] = n).  Prints "check <name> <value>"
// lines (relative residuals) and "time potrf n=.. <ms> <TF/s>".
//
//   ./ex_native [PxQ] [n_bench]          (one process per GPU; torchrun env)
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "slate_amd/slate_native.hh"

namespace sn = slate_amd::native;

extern "C" {
int slate_native_dpotrf(char uplo, int64_t n, double* a, int64_t lda);
int slate_native_dgesv(int64_t n, int64_t nrhs, double* a, int64_t lda, int64_t* ipiv, double* b, int64_t ldb);
const char* slate_native_last_error(void);
}

static double fro(const std::vector<double>& v) {
    double s = 0;
    for (double x : v) s += x * x;
    return std::sqrt(s);
}

int main(int argc, char** argv) {
    int p = 1, q = 1;
    if (argc > 1) std::sscanf(argv[1], "%dx%d", &p, &q);
    const int64_t nbench = argc > 2 ? std::atoll(argv[2]) : 0;
    try {
        sn::initialize();
        const int me = sn::rank();
        auto report = [&](const char* what, double v) {
            if (me == 0) std::printf("check %s %.3e\n", what, v);
            std::fflush(stdout);
        };
        const int64_t n = 700, nb = 64, nrhs = 3;

        // ---- potrf: || L L^T - A || / || A ||
        sn::HermitianMatrix<double> A(sn::Uplo::Lower, n, nb, p, q);
        A.generate(sn::Gen::HermitianPositiveDefinite, 7);
        std::vector<double> a0((size_t)n * n), l((size_t)n * n);
        A.to_host(a0.data(), n);
        int64_t info = sn::potrf(A);
        A.to_host(l.data(), n);
        std::vector<double> r((size_t)n * n, 0.0);
        for (int64_t j = 0; j < n; ++j)
            for (int64_t i = j; i < n; ++i) {
                double s = 0;
                for (int64_t k = 0; k <= j; ++k) s += l[i + k * n] * l[j + k * n];
                r[i + j * n] = s - a0[i + j * n];
            }
        std::vector<double> a0l((size_t)n * n, 0.0);
        for (int64_t j = 0; j < n; ++j)
            for (int64_t i = j; i < n; ++i) a0l[i + j * n] = a0[i + j * n];
        report(info ? "potrf-FAILED" : "potrf", fro(r) / fro(a0l));

        // ---- gemm: C = A B - C0 on the grid vs host
        const int64_t m2 = 300, k2 = 200, n2 = 250;
        sn::Matrix<double> GA(m2, k2, nb, p, q), GB(k2, n2, nb, p, q), GC(m2, n2, nb, p, q);
        GA.generate(sn::Gen::Random, 1);
        GB.generate(sn::Gen::Random, 2);
        GC.generate(sn::Gen::Random, 3);
        std::vector<double> ha((size_t)m2 * k2), hb((size_t)k2 * n2), hc((size_t)m2 * n2), hc1((size_t)m2 * n2);
        GA.to_host(ha.data(), m2);
        GB.to_host(hb.data(), k2);
        GC.to_host(hc.data(), m2);
        sn::gemm(2.0, GA, GB, -1.0, GC);
        GC.to_host(hc1.data(), m2);
        double err = 0, ref = 0;
        for (int64_t j = 0; j < n2; ++j)
            for (int64_t i = 0; i < m2; ++i) {
                double s = 0;
                for (int64_t k = 0; k < k2; ++k) s += ha[i + k * m2] * hb[k + j * k2];
                const double want = 2.0 * s - hc[i + j * m2];
                err += (hc1[i + j * m2] - want) * (hc1[i + j * m2] - want);
                ref += want * want;
            }
        report("gemm", std::sqrt(err / ref));

        // ---- norms against the host
        double mx = 0, fr = 0;
        for (double x : ha) { mx = std::fmax(mx, std::fabs(x)); fr += x * x; }
        report("norm_max", std::fabs(sn::norm(sn::Norm::Max, GA) - mx) / mx);
        report("norm_fro", std::fabs(sn::norm(sn::Norm::Fro, GA) - std::sqrt(fr)) / std::sqrt(fr));

        // ---- getrf on a 1 x (p q) grid: || P A - L U || via a solve
        sn::Matrix<double> G(n, n, nb, 1, p * q);
        G.generate(sn::Gen::Random, 5);
        std::vector<double> g0((size_t)n * n), lu((size_t)n * n);
        G.to_host(g0.data(), n);
        std::vector<int64_t> ipiv;
        info = sn::getrf(G, ipiv);
        G.to_host(lu.data(), n);
        // x = random, b = A x; solve with the factors on the host
        std::vector<double> x(n), b(n, 0.0), y;
        for (int64_t i = 0; i < n; ++i) x[i] = std::sin(1.0 + i);
        for (int64_t j = 0; j < n; ++j)
            for (int64_t i = 0; i < n; ++i) b[i] += g0[i + j * n] * x[j];
        y = b;
        for (int64_t i = 0; i < (int64_t)ipiv.size(); ++i) std::swap(y[i], y[ipiv[i]]);
        for (int64_t j = 0; j < n; ++j)
            for (int64_t i = j + 1; i < n; ++i) y[i] -= lu[i + j * n] * y[j];
        for (int64_t j = n - 1; j >= 0; --j) {
            y[j] /= lu[j + j * n];
            for (int64_t i = 0; i < j; ++i) y[i] -= lu[i + j * n] * y[j];
        }
        double ex = 0, nx = 0;
        for (int64_t i = 0; i < n; ++i) { ex += (y[i] - x[i]) * (y[i] - x[i]); nx += x[i] * x[i]; }
        report(info ? "getrf-FAILED" : "getrf", std::sqrt(ex / nx));

        if (p * q == 1) {
            // ---- posv / gesv (one rank) and the C ABI
            sn::HermitianMatrix<double> S(sn::Uplo::Lower, n, nb);
            S.generate(sn::Gen::HermitianPositiveDefinite, 9);
            std::vector<double> s0((size_t)n * n);
            S.to_host(s0.data(), n);
            sn::Matrix<double> B(n, nrhs, nb);
            B.generate(sn::Gen::Random, 10);
            std::vector<double> b0((size_t)n * nrhs), xs((size_t)n * nrhs);
            B.to_host(b0.data(), n);
            info = sn::posv(S, B);
            B.to_host(xs.data(), n);
            double rr = 0, rb = 0;
            for (int64_t c = 0; c < nrhs; ++c)
                for (int64_t i = 0; i < n; ++i) {
                    double s = 0;
                    for (int64_t j = 0; j < n; ++j) {
                        const double aij = i >= j ? s0[i + j * n] : s0[j + i * n];
                        s += aij * xs[j + c * n];
                    }
                    rr += (s - b0[i + c * n]) * (s - b0[i + c * n]);
                    rb += b0[i + c * n] * b0[i + c * n];
                }
            report(info ? "posv-FAILED" : "posv", std::sqrt(rr / rb));

            std::vector<double> ca = g0, cb = b;
            std::vector<int64_t> cpiv(n);
            const int ci = slate_native_dgesv(n, 1, ca.data(), n, cpiv.data(), cb.data(), n);
            double ce = 0;
            for (int64_t i = 0; i < n; ++i) ce += (cb[i] - x[i]) * (cb[i] - x[i]);
            report(ci ? "capi_dgesv-FAILED" : "capi_dgesv", std::sqrt(ce / nx));

            std::vector<double> cs = s0;
            const int cpi = slate_native_dpotrf('L', n, cs.data(), n);
            double cd = 0;
            for (int64_t i = 0; i < n; ++i) cd += (cs[i + i * n] - l[i + i * n]) * (cs[i + i * n] - l[i + i * n]);
            (void)cd;
            report(cpi ? "capi_dpotrf-FAILED" : "capi_dpotrf_info", (double)cpi);
        }

        if (nbench > 0) {
            sn::HermitianMatrix<double> T(sn::Uplo::Lower, nbench, 512, p, q);
            for (int it = 0; it < 3; ++it) {
                T.generate(sn::Gen::HermitianPositiveDefinite, 11);
                const auto t0 = std::chrono::steady_clock::now();
                info = sn::potrf(T);
                const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
                const double tf = (double)nbench * nbench * nbench / 3.0 / (ms * 1e-3) / 1e12;
                if (me == 0) std::printf("time potrf n=%lld %.2f ms %.2f TF/s info=%lld\n", (long long)nbench, ms, tf,
                                         (long long)info);
                std::fflush(stdout);
            }
        }
        sn::finalize();
    } catch (const std::exception& e) {
        std::fprintf(stderr, "ex_native: %s\n", e.what());
        return 1;
    }
    return 0;
}
