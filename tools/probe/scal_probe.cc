// Reproduces the ScaLAPACK-layer Cholesky flow (local arrays -> Matrix ->
// potrf -> local arrays -> potrs) on a p x q grid and checks each stage on
// the host: factor || L L^T - A || / || A ||, then the solve.
//   scal_probe PxQ n nb
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "slate_amd/slate_native.hh"

namespace sn = slate_amd::native;

static int64_t l2g(int64_t l, int64_t nb, int p, int pr) { return ((l / nb) * p + pr) * nb + l % nb; }
static double sym(int64_t i, int64_t j, int64_t n) { return i == j ? (double)n : 1.0 / (1.0 + std::llabs(i - j)); }

int main(int argc, char** argv) {
    int p = 2, q = 2;
    if (argc > 1) std::sscanf(argv[1], "%dx%d", &p, &q);
    const int64_t n = argc > 2 ? std::atoll(argv[2]) : 384, nb = argc > 3 ? std::atoll(argv[3]) : 32;
    sn::initialize();
    const int me = sn::rank(), pr = me % p, pc = me / p;
    const int warm = argc > 4 ? std::atoi(argv[4]) : 0;
    if (warm == 1) {                                  // warm-up factorization first
        sn::HermitianMatrix<double> W(sn::Uplo::Lower, 4 * nb * p, nb, p, q);
        W.generate(sn::Gen::HermitianPositiveDefinite, 1);
        sn::potrf(W);
    } else if (warm == 2) {                           // one-tile potrf
        sn::HermitianMatrix<double> W(sn::Uplo::Lower, nb, nb, p, q);
        W.generate(sn::Gen::HermitianPositiveDefinite, 1);
        sn::potrf(W);
    } else if (warm == 3) {                           // SUMMA gemm
        sn::Matrix<double> X1(2 * nb * p, 2 * nb * q, nb, p, q), X2(2 * nb * q, 2 * nb, nb, p, q),
            X3(2 * nb * p, 2 * nb, nb, p, q);
        X1.generate(sn::Gen::Random, 1);
        X2.generate(sn::Gen::Random, 2);
        sn::gemm(1.0, X1, X2, 0.0, X3);
    } else if (warm == 4) {                           // norm (world all-reduce)
        sn::Matrix<double> X1(2 * nb * p, 2 * nb * q, nb, p, q);
        X1.generate(sn::Gen::Random, 1);
        sn::norm(sn::Norm::Fro, X1);
    } else if (warm == 5) {                           // two-tile potrf
        sn::HermitianMatrix<double> W(sn::Uplo::Lower, 2 * nb, nb, p, q);
        W.generate(sn::Gen::HermitianPositiveDefinite, 1);
        sn::potrf(W);
    }
    sn::Matrix<double> G(n, n, nb, p, q);
    const int64_t mloc = G.mloc(), nloc = G.nloc(), ld = std::max<int64_t>(mloc, 1);
    std::vector<double> a((size_t)ld * std::max<int64_t>(nloc, 1));
    for (int64_t lj = 0; lj < nloc; ++lj)
        for (int64_t li = 0; li < mloc; ++li) a[li + lj * ld] = sym(l2g(li, nb, p, pr), l2g(lj, nb, q, pc), n);
    for (int rep = 0; rep < 3; ++rep) {
        G.from_local_host(a.data(), ld);
        sn::HermitianMatrix<double> H(sn::Uplo::Lower, n, nb, p, q);
        sn::copy(sn::Op::NoTrans, G, H);
        const int64_t info = sn::potrf(H);
        std::vector<double> L((size_t)n * n);
        H.to_host(L.data(), n);
        double e = 0, w = 0;
        for (int64_t j = 0; j < n; j += 3)
            for (int64_t i = j; i < n; i += 2) {
                double s = 0;
                for (int64_t k = 0; k <= j; ++k) s += L[i + k * n] * L[j + k * n];
                e += (s - sym(i, j, n)) * (s - sym(i, j, n));
                w += sym(i, j, n) * sym(i, j, n);
            }
        // solve with the factor as returned
        sn::Matrix<double> B(n, 3, nb, p, q), X(n, 3, nb, p, q);
        B.generate(sn::Gen::Random, 9);
        sn::copy(sn::Op::NoTrans, B, X);
        sn::potrs(H, X);
        std::vector<double> b((size_t)n * 3), x((size_t)n * 3);
        B.to_host(b.data(), n);
        X.to_host(x.data(), n);
        double re = 0, rw = 0;
        for (int c = 0; c < 3; ++c)
            for (int64_t i = 0; i < n; ++i) {
                double s = 0;
                for (int64_t j = 0; j < n; ++j) s += sym(i, j, n) * x[j + c * n];
                re += (s - b[i + c * n]) * (s - b[i + c * n]);
                rw += b[i + c * n] * b[i + c * n];
            }
        if (me == 0)
            std::printf("rep %d info=%lld factor %.3e solve %.3e\n", rep, (long long)info, std::sqrt(e / w),
                        std::sqrt(re / rw));
        std::fflush(stdout);
    }
    sn::finalize();
    return 0;
}
