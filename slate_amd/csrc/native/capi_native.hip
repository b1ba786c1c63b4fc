// C ABI of the native runtime (no Python): LAPACK-style entry points on
// global column-major host arrays, for C / Fortran applications
// (reference: lapack_api/lapack_potrf.cc etc. wrap the C++ drivers the same
// way).  With several ranks (torchrun environment) every rank passes the
// same global array; the matrix is distributed 1 x WORLD_SIZE (potrf: the
// grid of SLATE_AMD_NATIVE_GRID=PxQ if set) and the result gathered back.
// Return value: LAPACK info, or -1000 on a runtime error (message from
// slate_native_last_error()).
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "slate_amd/slate_native.hh"

namespace sn = slate_amd::native;

namespace {
std::string g_err;

void grid_of(int& p, int& q) {
    const int ws = sn::size();
    p = 1; q = ws;
    if (const char* g = std::getenv("SLATE_AMD_NATIVE_GRID")) {
        int a = 0, b = 0;
        if (std::sscanf(g, "%dx%d", &a, &b) == 2 && a * b == ws) { p = a; q = b; }
    }
}

int64_t nb_of(int64_t n) {
    if (const char* e = std::getenv("SLATE_AMD_NATIVE_NB")) return std::max<int64_t>(16, std::atoll(e));
    return n >= 8192 ? 512 : (n >= 1024 ? 256 : 64);
}

template <typename F>
int guarded(F&& f) {
    try {
        return (int)f();
    } catch (const std::exception& e) {
        g_err = e.what();
        return -1000;
    }
}
}  // namespace

extern "C" {

const char* slate_native_last_error(void) { return g_err.c_str(); }
int slate_native_initialize(void) { return guarded([] { sn::initialize(); return 0; }); }
void slate_native_finalize(void) { sn::finalize(); }

int slate_native_dpotrf(char uplo, int64_t n, double* a, int64_t lda) {
    return guarded([&]() -> int64_t {
        int p, q;
        grid_of(p, q);
        std::vector<double> t;
        if (uplo == 'U' || uplo == 'u') {          // factor A^T = L L^T, return U = L^T
            t.resize((size_t)n * n);
            for (int64_t j = 0; j < n; ++j)
                for (int64_t i = 0; i < n; ++i) t[i + j * n] = a[j + i * lda];
        }
        sn::HermitianMatrix<double> A(sn::Uplo::Lower, n, nb_of(n), p, q);
        if (t.empty()) A.from_host(a, lda); else A.from_host(t.data(), n);
        const int64_t info = sn::potrf(A);
        if (t.empty()) {
            std::vector<double> r((size_t)n * n);
            A.to_host(r.data(), n);
            for (int64_t j = 0; j < n; ++j)
                for (int64_t i = j; i < n; ++i) a[i + j * lda] = r[i + j * n];
        } else {
            A.to_host(t.data(), n);
            for (int64_t j = 0; j < n; ++j)
                for (int64_t i = j; i < n; ++i) a[j + i * lda] = t[i + j * n];
        }
        return info;
    });
}

int slate_native_dgetrf(int64_t m, int64_t n, double* a, int64_t lda, int64_t* ipiv) {
    return guarded([&]() -> int64_t {
        sn::Matrix<double> A(m, n, nb_of(std::max(m, n)), 1, sn::size());
        A.from_host(a, lda);
        std::vector<int64_t> piv;
        const int64_t info = sn::getrf(A, piv);
        A.to_host(a, lda);
        for (size_t i = 0; i < piv.size(); ++i) ipiv[i] = piv[i] + 1;     // LAPACK: 1-based
        return info;
    });
}

int slate_native_dgesv(int64_t n, int64_t nrhs, double* a, int64_t lda, int64_t* ipiv, double* b, int64_t ldb) {
    return guarded([&]() -> int64_t {
        if (sn::size() != 1) throw sn::Error("slate_native_dgesv: one rank");
        const int64_t nb = nb_of(n);
        sn::Matrix<double> A(n, n, nb), B(n, nrhs, nb);
        A.from_host(a, lda);
        B.from_host(b, ldb);
        std::vector<int64_t> piv;
        const int64_t info = sn::gesv(A, piv, B);
        A.to_host(a, lda);
        B.to_host(b, ldb);
        for (size_t i = 0; i < piv.size(); ++i) ipiv[i] = piv[i] + 1;
        return info;
    });
}

int slate_native_dposv(char uplo, int64_t n, int64_t nrhs, double* a, int64_t lda, double* b, int64_t ldb) {
    return guarded([&]() -> int64_t {
        if (sn::size() != 1) throw sn::Error("slate_native_dposv: one rank");
        if (uplo != 'L' && uplo != 'l') throw sn::Error("slate_native_dposv: uplo = 'L'");
        const int64_t nb = nb_of(n);
        sn::HermitianMatrix<double> A(sn::Uplo::Lower, n, nb);
        sn::Matrix<double> B(n, nrhs, nb);
        A.from_host(a, lda);
        B.from_host(b, ldb);
        const int64_t info = sn::posv(A, B);
        B.to_host(b, ldb);
        std::vector<double> r((size_t)n * n);
        A.to_host(r.data(), n);
        for (int64_t j = 0; j < n; ++j)
            for (int64_t i = j; i < n; ++i) a[i + j * lda] = r[i + j * n];
        return info;
    });
}

int slate_native_dgemm(int64_t m, int64_t n, int64_t k, double alpha, const double* a, int64_t lda, const double* b,
                       int64_t ldb, double beta, double* c, int64_t ldc) {
    return guarded([&]() -> int64_t {
        int p, q;
        grid_of(p, q);
        const int64_t nb = nb_of(std::max({m, n, k}));
        sn::Matrix<double> A(m, k, nb, p, q), B(k, n, nb, p, q), C(m, n, nb, p, q);
        A.from_host(a, lda);
        B.from_host(b, ldb);
        C.from_host(c, ldc);
        sn::gemm(alpha, A, B, beta, C);
        C.to_host(c, ldc);
        return 0;
    });
}

double slate_native_dlange(char norm, int64_t m, int64_t n, const double* a, int64_t lda) {
    double r = -1.0;
    const int rc = guarded([&]() -> int64_t {
        int p, q;
        grid_of(p, q);
        sn::Matrix<double> A(m, n, nb_of(std::max(m, n)), p, q);
        A.from_host(a, lda);
        const char k = (norm == 'm' || norm == 'M') ? 'M' : (norm == 'i' || norm == 'I') ? 'I'
                     : (norm == 'f' || norm == 'F' || norm == 'e' || norm == 'E') ? 'F' : '1';
        r = sn::norm((sn::Norm)k, A);
        return 0;
    });
    return rc == 0 ? r : -1.0;
}

}  // extern "C"
