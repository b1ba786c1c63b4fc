// LAPACK-style host-array entry points of the native library, second set
// (reference lapack_api/lapack_{trmm,syrk,herk,syr2k,her2k,symm,hemm,getri,
// potri,lansy,lanhe,lantr}.cc).  Same
// conventions as capi_native.hip: by-value slate_?xxx (int64 dimensions,
// LAPACK info returned), Fortran aliases slate_?xxx_ by reference, complex
// arrays interleaved (re, im) and complex scalars by pointer to (re, im);
// with several ranks every rank passes the same global arrays, the matrix is
// distributed over all ranks (1 x WORLD_SIZE or SLATE_AMD_NATIVE_GRID) and
// the result gathered back to every rank.  No Python anywhere.
#include <algorithm>
#include <cmath>
#include <complex>
#include <vector>

#include "capi_util.hpp"

namespace sn = slate_amd::native;
using sn::i64;
using namespace slate_amd::native::capi;

namespace {

// write the uplo triangle of r (n x n, ld n) into c (ld ldc); the other
// triangle of c is not referenced (LAPACK semantics)
template <typename T>
void put_triangle(char uplo, i64 n, const std::vector<T>& r, T* c, i64 ldc) {
    for (i64 j = 0; j < n; ++j)
        for (i64 i = 0; i < n; ++i)
            if ((uplo == 'L' && i >= j) || (uplo == 'U' && i <= j)) c[i + j * ldc] = r[i + j * n];
}

// B = alpha op(A) B (Left) or alpha B op(A) (Right), A triangular
template <typename T>
int64_t h_trmm(char side, char uplo, char ta, char diag, i64 m, i64 n, T alpha, const T* a, i64 lda, T* b, i64 ldb) {
    side = up(side);
    uplo = up(uplo);
    ta = up(ta);
    diag = up(diag);
    if (side != 'L' && side != 'R') return -1;
    if (uplo != 'L' && uplo != 'U') return -2;
    if (ta != 'N' && ta != 'T' && ta != 'C') return -3;
    if (diag != 'N' && diag != 'U') return -4;
    if (m < 0) return -5;
    if (n < 0) return -6;
    const i64 na = side == 'L' ? m : n;
    if (lda < std::max<i64>(1, na)) return -9;
    if (ldb < std::max<i64>(1, m)) return -11;
    if (m == 0 || n == 0) return 0;
    return guarded([&]() -> int64_t {
        int p, q;
        grid_of(p, q);
        const i64 nb = nb_of(std::max(m, n));
        // complex Trans: op(A) = A^T = conj(A)^H -- conjugate the host copy
        std::vector<T> Ah = host_op<T>('N', na, na, a, lda);
        if (ta == 'T' && sn::is_cplx<T>())
            for (auto& x : Ah) x = cj(x);
        const sn::Op op = ta == 'N' ? sn::Op::NoTrans : sn::Op::ConjTrans;
        sn::Matrix<T> A(na, na, nb, p, q), B(m, n, nb, p, q);
        A.from_host(Ah.data(), na);
        B.from_host(b, ldb);
        sn::trmm(side_of(side), uplo_of(uplo), op, diag_of(diag), alpha, A, B);
        B.to_host(b, ldb);
        return 0;
    });
}

// C = alpha op(A) op(A)^{H|T} + beta C           (two = false: herk / syrk)
// C = alpha op(A) op(B)^H + conj(alpha) op(B) op(A)^H + beta C   (two: her2k / syr2k)
template <typename T, bool HERM, bool TWO>
int64_t h_rank(char uplo, char trans, i64 n, i64 k, T alpha, const T* a, i64 lda, const T* b, i64 ldb, T beta, T* c,
               i64 ldc) {
    uplo = up(uplo);
    trans = up(trans);
    if (uplo != 'L' && uplo != 'U') return -1;
    const char tr_ok = HERM ? 'C' : 'T';
    if (trans != 'N' && trans != tr_ok && !(trans == 'T' && !sn::is_cplx<T>()) &&
        !(trans == 'C' && !sn::is_cplx<T>()))
        return -2;
    if (n < 0) return -3;
    if (k < 0) return -4;
    const i64 ar = trans == 'N' ? n : k;
    if (lda < std::max<i64>(1, ar)) return -7;
    if (TWO && ldb < std::max<i64>(1, ar)) return -9;
    if (ldc < std::max<i64>(1, n)) return TWO ? -12 : -10;
    if (n == 0) return 0;
    return guarded([&]() -> int64_t {
        int p, q;
        grid_of(p, q);
        const i64 nb = nb_of(std::max(n, k));
        const i64 kk = std::max<i64>(k, 1);
        const i64 rows = trans == 'N' ? n : kk, cols = trans == 'N' ? kk : n;
        sn::Matrix<T> A(rows, cols, nb, p, q), B(rows, cols, nb, p, q);
        if (k) A.from_host(a, lda);
        if (TWO && k) B.from_host(b, ldb);
        sn::HermitianMatrix<T> C(uplo_of(uplo), n, nb, p, q);
        C.from_host(c, ldc);
        const sn::Op op = trans == 'N' ? sn::Op::NoTrans : (HERM ? sn::Op::ConjTrans : sn::Op::Trans);
        const T al = k ? alpha : T(0);
        if constexpr (HERM && !TWO) sn::herk<T>(op, std::real(al), A, std::real(beta), C);
        else if constexpr (HERM && TWO) sn::her2k<T>(op, al, A, B, std::real(beta), C);
        else if constexpr (!HERM && !TWO) sn::syrk<T>(op, al, A, beta, C);
        else sn::syr2k<T>(op, al, A, B, beta, C);
        std::vector<T> r((size_t)n * n);
        C.to_host(r.data(), n);
        put_triangle(uplo, n, r, c, ldc);
        return 0;
    });
}

// C = alpha A B + beta C (Left) or alpha B A + beta C (Right), A Hermitian / symmetric
template <typename T, bool HERM>
int64_t h_xmm(char side, char uplo, i64 m, i64 n, T alpha, const T* a, i64 lda, const T* b, i64 ldb, T beta, T* c,
              i64 ldc) {
    side = up(side);
    uplo = up(uplo);
    if (side != 'L' && side != 'R') return -1;
    if (uplo != 'L' && uplo != 'U') return -2;
    if (m < 0) return -3;
    if (n < 0) return -4;
    const i64 na = side == 'L' ? m : n;
    if (lda < std::max<i64>(1, na)) return -7;
    if (ldb < std::max<i64>(1, m)) return -9;
    if (ldc < std::max<i64>(1, m)) return -12;
    if (m == 0 || n == 0) return 0;
    return guarded([&]() -> int64_t {
        int p, q;
        grid_of(p, q);
        const i64 nb = nb_of(std::max(m, n));
        sn::HermitianMatrix<T> A(uplo_of(uplo), na, nb, p, q);
        A.from_host(a, lda);
        sn::Matrix<T> B(m, n, nb, p, q), C(m, n, nb, p, q);
        B.from_host(b, ldb);
        C.from_host(c, ldc);
        if constexpr (HERM) sn::hemm<T>(side_of(side), alpha, A, B, beta, C);
        else sn::symm<T>(side_of(side), alpha, A, B, beta, C);
        C.to_host(c, ldc);
        return 0;
    });
}

// A^-1 from getrf's factors (ipiv 1-based, LAPACK)
template <typename T>
int64_t h_getri(i64 n, T* a, i64 lda, const int64_t* ipiv) {
    if (n < 0) return -1;
    if (lda < std::max<i64>(1, n)) return -3;
    if (n == 0) return 0;
    return guarded([&]() -> int64_t {
        int p, q;
        grid_of(p, q);
        sn::Matrix<T> A(n, n, nb_of(n), p, q);
        A.from_host(a, lda);
        // LAPACK: info > 0 when U(i, i) is exactly zero (singular)
        for (i64 i = 0; i < n; ++i)
            if (a[i + i * lda] == T(0)) return i + 1;
        std::vector<int64_t> piv((size_t)n);
        for (i64 i = 0; i < n; ++i) piv[i] = ipiv[i] - 1;
        sn::getri(A, piv);
        A.to_host(a, lda);
        return 0;
    });
}

// A^-1 of a Hermitian positive definite matrix from potrf's factor (uplo)
template <typename T>
int64_t h_potri(char uplo, i64 n, T* a, i64 lda) {
    uplo = up(uplo);
    if (uplo != 'L' && uplo != 'U') return -1;
    if (n < 0) return -2;
    if (lda < std::max<i64>(1, n)) return -4;
    if (n == 0) return 0;
    return guarded([&]() -> int64_t {
        for (i64 i = 0; i < n; ++i)
            if (a[i + i * lda] == T(0)) return i + 1;
        int p, q;
        grid_of(p, q);
        sn::HermitianMatrix<T> A(uplo_of(uplo), n, nb_of(n), p, q);
        A.from_host(a, lda);
        sn::potri(A);
        std::vector<T> r((size_t)n * n);
        A.to_host(r.data(), n);
        put_triangle(uplo, n, r, a, lda);
        return 0;
    });
}

inline sn::Norm norm_of(char c) {
    c = up(c);
    return c == 'M' ? sn::Norm::Max : c == 'I' ? sn::Norm::Inf : (c == 'F' || c == 'E') ? sn::Norm::Fro : sn::Norm::One;
}

// norms of a Hermitian / symmetric matrix from its uplo triangle
template <typename T, bool HERM>
double h_lan_sym(char norm, char uplo, i64 n, const T* a, i64 lda) {
    if (n == 0) return 0.0;
    double r = -1.0;
    const int64_t rc = guarded([&]() -> int64_t {
        int p, q;
        grid_of(p, q);
        sn::HermitianMatrix<T> A(uplo_of(up(uplo)), n, nb_of(n), p, q);
        A.from_host(a, lda);
        r = HERM ? sn::norm<T>(norm_of(norm), A) : sn::norm_symmetric<T>(norm_of(norm), A);
        return 0;
    });
    return rc == 0 ? r : -1.0;
}

// norms of an m x n upper / lower trapezoid (LAPACK lantr); a square
// pad carries the trapezoid (zero columns / rows contribute nothing; with a
// unit diagonal the padded ones are removed from the Frobenius sum)
template <typename T>
double h_lantr(char norm, char uplo, char diag, i64 m, i64 n, const T* a, i64 lda) {
    if (m == 0 || n == 0) return 0.0;
    double r = -1.0;
    const int64_t rc = guarded([&]() -> int64_t {
        int p, q;
        grid_of(p, q);
        const i64 k = std::max(m, n);
        std::vector<T> sq((size_t)k * k, T(0));
        for (i64 j = 0; j < n; ++j)
            for (i64 i = 0; i < m; ++i) sq[i + j * k] = a[i + j * lda];
        sn::Matrix<T> A(k, k, nb_of(k), p, q);
        A.from_host(sq.data(), k);
        const sn::Norm nk = norm_of(norm);
        r = sn::norm_triangular<T>(nk, uplo_of(up(uplo)), diag_of(up(diag)), A);
        const i64 extra = k - std::min(m, n);
        if (up(diag) == 'U' && extra > 0) {
            if (nk == sn::Norm::Fro) r = std::sqrt(std::max(0.0, r * r - (double)extra));
        }
        return 0;
    });
    return rc == 0 ? r : -1.0;
}

// condition estimates from host factors (reference lapack_api/lapack_gecon.cc,
// _pocon.cc, _trcon.cc): rcond through the native estimators
template <typename T>
int64_t h_con(char kind, char norm, char uplo, char diag, i64 n, const T* a, i64 lda, double anorm, T* rcond) {
    if (n < 0) return -2;
    if (lda < std::max<i64>(1, n)) return -4;
    if (n == 0) { *rcond = T(1); return 0; }
    return guarded([&]() -> int64_t {
        int p, q;
        grid_of(p, q);
        const sn::Norm nk = up(norm) == 'I' ? sn::Norm::Inf : sn::Norm::One;
        double rc = 0;
        if (kind == 'G') {
            sn::Matrix<T> A(n, n, nb_of(n), p, q);
            A.from_host(a, lda);
            rc = sn::gecondest<T>(nk, A, anorm);
        } else if (kind == 'P') {
            // the Cholesky factor as Lower storage (Upper: its conjugate transpose)
            std::vector<T> l = up(uplo) == 'U' ? host_op<T>('C', n, n, a, lda) : std::vector<T>(a, a + 0);
            sn::HermitianMatrix<T> L(sn::Uplo::Lower, n, nb_of(n), p, q);
            if (up(uplo) == 'U') L.from_host(l.data(), n);
            else L.from_host(a, lda);
            rc = sn::pocondest<T>(nk, L, anorm);
        } else {
            sn::Matrix<T> A(n, n, nb_of(n), p, q);
            A.from_host(a, lda);
            rc = sn::trcondest<T>(nk, uplo_of(uplo), diag_of(diag), A);
        }
        *rcond = T(rc);
        return 0;
    });
}

}  // namespace

extern "C" {

#define SN_LAPACK2_R(X, T)                                                                                      \
    int slate_##X##trmm(char side, char uplo, char ta, char diag, int64_t m, int64_t n, T alpha, const T* a,   \
                        int64_t lda, T* b, int64_t ldb) {                                                      \
        return (int)h_trmm<T>(side, uplo, ta, diag, m, n, alpha, a, lda, b, ldb);                              \
    }                                                                                                          \
    int slate_##X##syrk(char uplo, char trans, int64_t n, int64_t k, T alpha, const T* a, int64_t lda, T beta,  \
                        T* c, int64_t ldc) {                                                                   \
        return (int)h_rank<T, false, false>(uplo, trans, n, k, alpha, a, lda, nullptr, 1, beta, c, ldc);       \
    }                                                                                                          \
    int slate_##X##syr2k(char uplo, char trans, int64_t n, int64_t k, T alpha, const T* a, int64_t lda,        \
                         const T* b, int64_t ldb, T beta, T* c, int64_t ldc) {                                  \
        return (int)h_rank<T, false, true>(uplo, trans, n, k, alpha, a, lda, b, ldb, beta, c, ldc);            \
    }                                                                                                          \
    int slate_##X##symm(char side, char uplo, int64_t m, int64_t n, T alpha, const T* a, int64_t lda,          \
                        const T* b, int64_t ldb, T beta, T* c, int64_t ldc) {                                   \
        return (int)h_xmm<T, false>(side, uplo, m, n, alpha, a, lda, b, ldb, beta, c, ldc);                    \
    }                                                                                                          \
    int slate_##X##getri(int64_t n, T* a, int64_t lda, const int64_t* ipiv) {                                   \
        return (int)h_getri<T>(n, a, lda, ipiv);                                                               \
    }                                                                                                          \
    int slate_##X##potri(char uplo, int64_t n, T* a, int64_t lda) { return (int)h_potri<T>(uplo, n, a, lda); } \
    double slate_##X##lansy(char norm, char uplo, int64_t n, const T* a, int64_t lda) {                        \
        return h_lan_sym<T, false>(norm, uplo, n, a, lda);                                                     \
    }                                                                                                          \
    double slate_##X##lantr(char norm, char uplo, char diag, int64_t m, int64_t n, const T* a, int64_t lda) {  \
        return h_lantr<T>(norm, uplo, diag, m, n, a, lda);                                                     \
    }                                                                                                          \
    void slate_##X##trmm_(const char* side, const char* uplo, const char* ta, const char* diag,                \
                          const int64_t* m, const int64_t* n, const T* alpha, const T* a, const int64_t* lda,  \
                          T* b, const int64_t* ldb) {                                                          \
        h_trmm<T>(*side, *uplo, *ta, *diag, *m, *n, *alpha, a, *lda, b, *ldb);                                 \
    }                                                                                                          \
    void slate_##X##syrk_(const char* uplo, const char* trans, const int64_t* n, const int64_t* k,             \
                          const T* alpha, const T* a, const int64_t* lda, const T* beta, T* c,                 \
                          const int64_t* ldc) {                                                                \
        h_rank<T, false, false>(*uplo, *trans, *n, *k, *alpha, a, *lda, nullptr, 1, *beta, c, *ldc);           \
    }                                                                                                          \
    void slate_##X##syr2k_(const char* uplo, const char* trans, const int64_t* n, const int64_t* k,            \
                           const T* alpha, const T* a, const int64_t* lda, const T* b, const int64_t* ldb,     \
                           const T* beta, T* c, const int64_t* ldc) {                                          \
        h_rank<T, false, true>(*uplo, *trans, *n, *k, *alpha, a, *lda, b, *ldb, *beta, c, *ldc);               \
    }                                                                                                          \
    void slate_##X##symm_(const char* side, const char* uplo, const int64_t* m, const int64_t* n,              \
                          const T* alpha, const T* a, const int64_t* lda, const T* b, const int64_t* ldb,      \
                          const T* beta, T* c, const int64_t* ldc) {                                           \
        h_xmm<T, false>(*side, *uplo, *m, *n, *alpha, a, *lda, b, *ldb, *beta, c, *ldc);                       \
    }                                                                                                          \
    void slate_##X##getri_(const int64_t* n, T* a, const int64_t* lda, const int64_t* ipiv, int64_t* info) {    \
        *info = h_getri<T>(*n, a, *lda, ipiv);                                                                 \
    }                                                                                                          \
    void slate_##X##potri_(const char* uplo, const int64_t* n, T* a, const int64_t* lda, int64_t* info) {      \
        *info = h_potri<T>(*uplo, *n, a, *lda);                                                                \
    }                                                                                                          \
    double slate_##X##lansy_(const char* norm, const char* uplo, const int64_t* n, const T* a,                 \
                             const int64_t* lda) {                                                             \
        return h_lan_sym<T, false>(*norm, *uplo, *n, a, *lda);                                                 \
    }                                                                                                          \
    double slate_##X##lantr_(const char* norm, const char* uplo, const char* diag, const int64_t* m,           \
                             const int64_t* n, const T* a, const int64_t* lda) {                               \
        return h_lantr<T>(*norm, *uplo, *diag, *m, *n, a, *lda);                                               \
    }
SN_LAPACK2_R(s, float)
SN_LAPACK2_R(d, double)
#undef SN_LAPACK2_R

// complex: interleaved arrays (R*), complex scalars by pointer to (re, im)
#define SN_LAPACK2_C(X, R)                                                                                      \
    int slate_##X##trmm(char side, char uplo, char ta, char diag, int64_t m, int64_t n, const R* alpha,        \
                        const R* a, int64_t lda, R* b, int64_t ldb) {                                          \
        using T = std::complex<R>;                                                                             \
        return (int)h_trmm<T>(side, uplo, ta, diag, m, n, T(alpha[0], alpha[1]), reinterpret_cast<const T*>(a), \
                              lda, reinterpret_cast<T*>(b), ldb);                                              \
    }                                                                                                          \
    int slate_##X##syrk(char uplo, char trans, int64_t n, int64_t k, const R* alpha, const R* a, int64_t lda,  \
                        const R* beta, R* c, int64_t ldc) {                                                    \
        using T = std::complex<R>;                                                                             \
        return (int)h_rank<T, false, false>(uplo, trans, n, k, T(alpha[0], alpha[1]),                         \
                                            reinterpret_cast<const T*>(a), lda, nullptr, 1,                    \
                                            T(beta[0], beta[1]), reinterpret_cast<T*>(c), ldc);                \
    }                                                                                                          \
    int slate_##X##syr2k(char uplo, char trans, int64_t n, int64_t k, const R* alpha, const R* a, int64_t lda, \
                         const R* b, int64_t ldb, const R* beta, R* c, int64_t ldc) {                          \
        using T = std::complex<R>;                                                                             \
        return (int)h_rank<T, false, true>(uplo, trans, n, k, T(alpha[0], alpha[1]),                           \
                                           reinterpret_cast<const T*>(a), lda, reinterpret_cast<const T*>(b),  \
                                           ldb, T(beta[0], beta[1]), reinterpret_cast<T*>(c), ldc);            \
    }                                                                                                          \
    int slate_##X##herk(char uplo, char trans, int64_t n, int64_t k, R alpha, const R* a, int64_t lda, R beta, \
                        R* c, int64_t ldc) {                                                                   \
        using T = std::complex<R>;                                                                             \
        return (int)h_rank<T, true, false>(uplo, trans, n, k, T(alpha), reinterpret_cast<const T*>(a), lda,    \
                                           nullptr, 1, T(beta), reinterpret_cast<T*>(c), ldc);                 \
    }                                                                                                          \
    int slate_##X##her2k(char uplo, char trans, int64_t n, int64_t k, const R* alpha, const R* a, int64_t lda, \
                         const R* b, int64_t ldb, R beta, R* c, int64_t ldc) {                                 \
        using T = std::complex<R>;                                                                             \
        return (int)h_rank<T, true, true>(uplo, trans, n, k, T(alpha[0], alpha[1]),                            \
                                          reinterpret_cast<const T*>(a), lda, reinterpret_cast<const T*>(b),   \
                                          ldb, T(beta), reinterpret_cast<T*>(c), ldc);                         \
    }                                                                                                          \
    int slate_##X##symm(char side, char uplo, int64_t m, int64_t n, const R* alpha, const R* a, int64_t lda,   \
                        const R* b, int64_t ldb, const R* beta, R* c, int64_t ldc) {                           \
        using T = std::complex<R>;                                                                             \
        return (int)h_xmm<T, false>(side, uplo, m, n, T(alpha[0], alpha[1]), reinterpret_cast<const T*>(a),    \
                                    lda, reinterpret_cast<const T*>(b), ldb, T(beta[0], beta[1]),              \
                                    reinterpret_cast<T*>(c), ldc);                                             \
    }                                                                                                          \
    int slate_##X##hemm(char side, char uplo, int64_t m, int64_t n, const R* alpha, const R* a, int64_t lda,   \
                        const R* b, int64_t ldb, const R* beta, R* c, int64_t ldc) {                           \
        using T = std::complex<R>;                                                                             \
        return (int)h_xmm<T, true>(side, uplo, m, n, T(alpha[0], alpha[1]), reinterpret_cast<const T*>(a),     \
                                   lda, reinterpret_cast<const T*>(b), ldb, T(beta[0], beta[1]),               \
                                   reinterpret_cast<T*>(c), ldc);                                              \
    }                                                                                                          \
    int slate_##X##getri(int64_t n, R* a, int64_t lda, const int64_t* ipiv) {                                   \
        return (int)h_getri<std::complex<R>>(n, reinterpret_cast<std::complex<R>*>(a), lda, ipiv);             \
    }                                                                                                          \
    int slate_##X##potri(char uplo, int64_t n, R* a, int64_t lda) {                                             \
        return (int)h_potri<std::complex<R>>(uplo, n, reinterpret_cast<std::complex<R>*>(a), lda);             \
    }                                                                                                          \
    double slate_##X##lansy(char norm, char uplo, int64_t n, const R* a, int64_t lda) {                        \
        return h_lan_sym<std::complex<R>, false>(norm, uplo, n, reinterpret_cast<const std::complex<R>*>(a),   \
                                                 lda);                                                         \
    }                                                                                                          \
    double slate_##X##lanhe(char norm, char uplo, int64_t n, const R* a, int64_t lda) {                        \
        return h_lan_sym<std::complex<R>, true>(norm, uplo, n, reinterpret_cast<const std::complex<R>*>(a),    \
                                                lda);                                                          \
    }                                                                                                          \
    double slate_##X##lantr(char norm, char uplo, char diag, int64_t m, int64_t n, const R* a, int64_t lda) {  \
        return h_lantr<std::complex<R>>(norm, uplo, diag, m, n, reinterpret_cast<const std::complex<R>*>(a),   \
                                        lda);                                                                  \
    }
SN_LAPACK2_C(c, float)
SN_LAPACK2_C(z, double)
#undef SN_LAPACK2_C


#define SN_CON(X, T)                                                                                            \
    int slate_##X##gecon(char norm, int64_t n, const T* a, int64_t lda, T anorm, T* rcond) {                   \
        return (int)h_con<T>('G', norm, 'L', 'N', n, a, lda, (double)anorm, rcond);                            \
    }                                                                                                          \
    int slate_##X##pocon(char uplo, int64_t n, const T* a, int64_t lda, T anorm, T* rcond) {                   \
        return (int)h_con<T>('P', '1', uplo, 'N', n, a, lda, (double)anorm, rcond);                            \
    }                                                                                                          \
    int slate_##X##trcon(char norm, char uplo, char diag, int64_t n, const T* a, int64_t lda, T* rcond) {      \
        return (int)h_con<T>('T', norm, uplo, diag, n, a, lda, 0.0, rcond);                                    \
    }
SN_CON(s, float)
SN_CON(d, double)
#undef SN_CON

// Fortran-callable aliases of the C ABI (c_api.h: every argument by reference)
int slate_dsgesv(int64_t n, int64_t nrhs, double* a, int64_t lda, int64_t* ipiv, const double* b, int64_t ldb,
                 double* x, int64_t ldx, int* iter);
void slate_dsgesv_(const int64_t* n, const int64_t* nrhs, double* a, const int64_t* lda, int64_t* ipiv,
                   const double* b, const int64_t* ldb, double* x, const int64_t* ldx, int64_t* iter, int64_t* info) {
    int it = 0;
    *info = slate_dsgesv(*n, *nrhs, a, *lda, ipiv, b, *ldb, x, *ldx, &it);
    if (iter) *iter = it;
}
void slate_dsyev(const char* jobz, const char* uplo, const int* n, double* a, const int* lda, double* w, double* work,
                 const int* lwork, int* info);
void slate_dsyevd(const char* jobz, const char* uplo, const int* n, double* a, const int* lda, double* w,
                  double* work, const int* lwork, int* iwork, const int* liwork, int* info);
void slate_dsyev_(const char* jobz, const char* uplo, const int64_t* n, double* a, const int64_t* lda, double* w,
                  int64_t* info) {
    const int nn = (int)*n, ll = (int)*lda, lw = 1;
    int inf = 0;
    double wk = 0;
    slate_dsyev(jobz, uplo, &nn, a, &ll, w, &wk, &lw, &inf);
    *info = inf;
}
void slate_dsyevd_(const char* jobz, const char* uplo, const int64_t* n, double* a, const int64_t* lda, double* w,
                   int64_t* info) {
    const int nn = (int)*n, ll = (int)*lda, lw = 1, liw = 1;
    int inf = 0, iw = 0;
    double wk = 0;
    slate_dsyevd(jobz, uplo, &nn, a, &ll, w, &wk, &lw, &iw, &liw, &inf);
    *info = inf;
}
}  // extern "C"
