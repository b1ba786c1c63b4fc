// Probe of the native library's building blocks against host references:
// trsm (lower / upper, NoTrans / ConjTrans), gemm with one column, potrs.
//   native_probe n nb
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "slate_amd/slate_native.hh"

namespace sn = slate_amd::native;

static double relres(const std::vector<double>& A, char uplo, char tr, int64_t n, const std::vector<double>& x,
                     const std::vector<double>& b) {
    // || op(tri(A)) x - b || / || b ||
    double e = 0, w = 0;
    for (int64_t i = 0; i < n; ++i) {
        double s = 0;
        for (int64_t j = 0; j < n; ++j) {
            const int64_t r = tr == 'N' ? i : j, c = tr == 'N' ? j : i;
            const bool in = uplo == 'L' ? r >= c : r <= c;
            if (in) s += A[r + c * n] * x[j];
        }
        e += (s - b[i]) * (s - b[i]);
        w += b[i] * b[i];
    }
    return std::sqrt(e / w);
}

int main(int argc, char** argv) {
    const int64_t n = argc > 1 ? std::atoll(argv[1]) : 8192, nb = argc > 2 ? std::atoll(argv[2]) : 512;
    sn::initialize();
    sn::Matrix<double> A(n, n, nb), V(n, 1, nb), X(n, 1, nb);
    A.generate(sn::Gen::DiagDominant, 3);
    V.generate(sn::Gen::Random, 4);
    std::vector<double> a((size_t)n * n), v(n), x(n);
    A.to_host(a.data(), n);
    V.to_host(v.data(), n);
    for (char uplo : {'L', 'U'})
        for (char tr : {'N', 'C'}) {
            sn::copy(sn::Op::NoTrans, V, X);
            sn::trsm(sn::Side::Left, uplo == 'L' ? sn::Uplo::Lower : sn::Uplo::Upper,
                     tr == 'N' ? sn::Op::NoTrans : sn::Op::ConjTrans, sn::Diag::NonUnit, 1.0, A, X);
            X.to_host(x.data(), n);
            std::printf("trsm %c%c n=%lld nb=%lld: %.3e\n", uplo, tr, (long long)n, (long long)nb,
                        relres(a, uplo, tr, n, x, v));
        }
    // gemm with one column, beta = 1
    sn::copy(sn::Op::NoTrans, V, X);
    sn::gemm(-1.0, A, V, 1.0, X);                    // X = V - A V
    X.to_host(x.data(), n);
    double e = 0, w = 0;
    for (int64_t i = 0; i < n; ++i) {
        double s = v[i];
        for (int64_t j = 0; j < n; ++j) s -= a[i + j * n] * v[j];
        e += (s - x[i]) * (s - x[i]);
        w += s * s;
    }
    std::printf("gemm n1 beta1: %.3e\n", std::sqrt(e / w));
    // potrf + potrs on the same matrix made HPD
    sn::HermitianMatrix<double> H(sn::Uplo::Lower, n, nb);
    H.generate(sn::Gen::HermitianPositiveDefinite, 7);
    std::vector<double> h((size_t)n * n);
    H.to_host(h.data(), n);
    const int64_t info = sn::potrf(H);
    std::vector<double> l((size_t)n * n);
    H.to_host(l.data(), n);
    // || L L^T v - H v || / || H v ||
    std::vector<double> t(n, 0.0), y(n, 0.0), hv(n, 0.0);
    for (int64_t j = 0; j < n; ++j)
        for (int64_t i = j; i < n; ++i) t[j] += l[i + j * n] * v[i];
    for (int64_t j = 0; j < n; ++j)
        for (int64_t i = j; i < n; ++i) y[i] += l[i + j * n] * t[j];
    for (int64_t j = 0; j < n; ++j)
        for (int64_t i = 0; i < n; ++i) hv[i] += h[i + j * n] * v[j];
    e = w = 0;
    for (int64_t i = 0; i < n; ++i) { e += (y[i] - hv[i]) * (y[i] - hv[i]); w += hv[i] * hv[i]; }
    std::printf("potrf LL^T v info=%lld: %.3e\n", (long long)info, std::sqrt(e / w));
    sn::finalize();
    return 0;
}
