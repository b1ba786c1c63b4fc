// C++ API of slate_amd (include/slate_amd/slate_amd.hh) on a process grid:
// every check computes a relative residual with library routines only and
// prints "rank r: <check> <value>"; the caller asserts value < 1e-10.
// Start one process per rank (RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT);
// argv[1] = "PxQ" (default 1x1).
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <numeric>

#include "slate_amd/slate_amd.hh"

namespace sa = slate_amd;
using M = sa::Matrix<double>;
using H = sa::HermitianMatrix<double>;

static int rank_id() { const char* r = getenv("RANK"); return r ? atoi(r) : 0; }

int main(int argc, char** argv) {
    int p = 1, q = 1;
    if (argc > 1) sscanf(argv[1], "%dx%d", &p, &q);
    const int me = rank_id();
    const int64_t n = 96, nb = 16, nrhs = 5;
    auto report = [&](const char* what, double v) { printf("rank %d: %s %.3e\n", me, what, v); fflush(stdout); };
    try {
        sa::set_option("Lookahead", "2");

        // posv: A X = B, residual by hemm
        H A(sa::Uplo::Lower, n, nb, p, q), A0(sa::Uplo::Lower, n, nb, p, q);
        A.generate(sa::Gen::HermitianPositiveDefinite, 3);
        A0.generate(sa::Gen::HermitianPositiveDefinite, 3);
        M B(n, nrhs, nb, p, q), B0(n, nrhs, nb, p, q);
        B.generate(sa::Gen::Random, 4);
        B0.generate(sa::Gen::Random, 4);
        int64_t info = sa::posv(A, B);
        sa::hemm(sa::Side::Left, 1.0, A0, B, -1.0, B0);
        report(info ? "posv-FAILED" : "posv", sa::norm(sa::Norm::Fro, B0) / (sa::norm(sa::Norm::Fro, A0) * sa::norm(sa::Norm::Fro, B)));

        // gesv + getri on a general matrix
        M G(n, n, nb, p, q), G0(n, n, nb, p, q), X(n, nrhs, nb, p, q), X0(n, nrhs, nb, p, q);
        G.generate(sa::Gen::Random, 5);
        G0.generate(sa::Gen::Random, 5);
        X.generate(sa::Gen::Random, 6);
        X0.generate(sa::Gen::Random, 6);
        sa::Pivots piv;
        info = sa::gesv(G, piv, X);
        sa::gemm(1.0, G0, X, -1.0, X0);
        report(info ? "gesv-FAILED" : "gesv", sa::norm(sa::Norm::Fro, X0) / (sa::norm(sa::Norm::Fro, G0) * sa::norm(sa::Norm::Fro, X)));
        info = sa::getri(G, piv);
        M I(n, n, nb, p, q);
        sa::set(0.0, 1.0, I);
        sa::gemm(1.0, G0, G, -1.0, I);                   // A inv(A) - I
        report(info ? "getri-FAILED" : "getri", sa::norm(sa::Norm::Fro, I) / (sa::norm(sa::Norm::Fro, G0) * sa::norm(sa::Norm::Fro, G)));

        // trmm then trsm round trip on the Cholesky factor
        M C(n, nrhs, nb, p, q), C0(n, nrhs, nb, p, q);
        C.generate(sa::Gen::Random, 7);
        C0.generate(sa::Gen::Random, 7);
        auto L = sa::triangular(sa::Uplo::Lower, sa::Diag::NonUnit, A);
        sa::trmm(sa::Side::Left, 2.0, L, C);
        sa::trsm(sa::Side::Left, 0.5, L, C);
        sa::add(-1.0, C0, 1.0, C);
        report("trmm_trsm", sa::norm(sa::Norm::Fro, C) / sa::norm(sa::Norm::Fro, C0));

        // herk vs gemm with a conjugate-transposed view
        M W(n, 24, nb, p, q);
        W.generate(sa::Gen::Random, 8);
        H K(sa::Uplo::Lower, n, nb, p, q);
        sa::set(0.0, 0.0, K);
        sa::herk(1.0, W, 0.0, K);
        M Kg(n, n, nb, p, q);
        sa::gemm(1.0, W, sa::conj_transpose(W), 0.0, Kg);
        report("herk", std::fabs(sa::norm(sa::Norm::Fro, K) - sa::norm(sa::Norm::Fro, Kg)) / sa::norm(sa::Norm::Fro, Kg));

        // least squares: A^H (A x - b) = 0
        const int64_t m = 2 * n;
        M T(m, n, nb, p, q), T0(m, n, nb, p, q), BX(m, nrhs, nb, p, q), R(m, nrhs, nb, p, q);
        T.generate(sa::Gen::Random, 9);
        T0.generate(sa::Gen::Random, 9);
        BX.generate(sa::Gen::Random, 10);
        R.generate(sa::Gen::Random, 10);
        sa::TriangularFactors tf;
        info = sa::gels(T, tf, BX);
        M Xs = BX.sub(0, n / nb - 1, 0, BX.nt() - 1);
        sa::gemm(1.0, T0, Xs, -1.0, R);                  // A x - b
        M N(n, nrhs, nb, p, q);
        sa::gemm(1.0, sa::conj_transpose(T0), R, 0.0, N);
        report(info ? "gels-FAILED" : "gels", sa::norm(sa::Norm::Fro, N) / (sa::norm(sa::Norm::Fro, T0) * sa::norm(sa::Norm::Fro, R)));

        // spectra: sum w^2 = ||A||_F^2, sum s^2 = ||G0||_F^2
        H E(sa::Uplo::Lower, n, nb, p, q);
        E.generate(sa::Gen::HermitianPositiveDefinite, 11);
        const double ef = sa::norm(sa::Norm::Fro, E);
        auto w = sa::heev(E);
        double sw = 0;
        for (double x : w) sw += x * x;
        report("heev", std::fabs(std::sqrt(sw) - ef) / ef);
        M S(n, n, nb, p, q);
        S.generate(sa::Gen::Random, 12);
        const double sf = sa::norm(sa::Norm::Fro, S);
        auto sv = sa::svd_vals(S);
        double ss = 0;
        for (double x : sv) ss += x * x;
        report("svd_vals", std::fabs(std::sqrt(ss) - sf) / sf);

        // mixed precision with iteration count
        M Gm(n, n, nb, p, q), Gm0(n, n, nb, p, q), Bm(n, nrhs, nb, p, q), Bm0(n, nrhs, nb, p, q), Xm(n, nrhs, nb, p, q);
        Gm.generate(sa::Gen::Random, 13);
        Gm0.generate(sa::Gen::Random, 13);
        Bm.generate(sa::Gen::Random, 14);
        Bm0.generate(sa::Gen::Random, 14);
        sa::Pivots pm;
        int64_t iter = -1;
        info = sa::gesv_mixed(Gm, pm, Bm, Xm, &iter);
        sa::gemm(1.0, Gm0, Xm, -1.0, Bm0);
        report(info ? "gesv_mixed-FAILED" : "gesv_mixed", sa::norm(sa::Norm::Fro, Bm0) / (sa::norm(sa::Norm::Fro, Gm0) * sa::norm(sa::Norm::Fro, Xm)));
        printf("rank %d: gesv_mixed iterations %lld\n", me, (long long)iter);
    } catch (const sa::Exception& e) {
        printf("rank %d: exception %s\n", me, e.what());
        return 1;
    }
    sa::finalize();
    return 0;
}
