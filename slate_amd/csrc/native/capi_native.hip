// C / Fortran ABI of the native runtime -- no Python anywhere.  The same
// symbols and signatures as include/slate_amd/c_api.h, so a C, C++ or
// Fortran application links -lslate_amd_native instead of -lslate_amd_c:
//
//   * LAPACK-style host-array routines (reference lapack_api/lapack_*.cc):
//     slate_{s,d}{gemm,potrf,potrs,posv,getrf,getrs,gesv,trsm,gels} +
//     Fortran aliases slate_?xxx_ (by reference), complex slate_{c,z}potrf,
//     slate_{c,z}gesv, slate_zposv (interleaved re/im), slate_dlange.  With
//     several ranks every rank passes the same global array; the matrix is
//     distributed over all ranks (1 x WORLD_SIZE, or SLATE_AMD_NATIVE_GRID=PxQ)
//     and the result is gathered back to every rank.
//   * ScaLAPACK (reference scalapack_api/scalapack_*.cc):
//     p{s,d,c,z}{potrf,posv,getrf,gesv,potrs,getrs,gemm,trsm,gels,lange}_
//     on the caller's LOCAL block-cyclic arrays (9-int descriptors), with a
//     minimal BLACS (Cblacs_* / blacs_*_, numroc_, descinit_) over the native
//     runtime's ranks.  Operands are any sub-matrix A(ia:ia+m-1, ja:ja+n-1)
//     of a descriptor (any MB / NB, RSRC / CSRC, row- or column-major grid):
//     whole aligned matrices are a local copy, the rest is redistributed
//     point to point (scal_move).
//   * slate_native_* (the earlier entry points; int return = info).
//
// info: 0 = success, > 0 numerical failure, < 0 illegal argument,
// SLATE_AMD_ERR_INTERNAL (-1000000) on a runtime error (message from
// slate_amd_last_error()).
#include <algorithm>
#include <complex>
#include <cstdio>
#include <cstring>
#include <map>
#include <memory>
#include <cstdlib>
#include <string>
#include <vector>

#include "../hip/kernels.hpp"
#include "native_rt.hpp"

namespace sn = slate_amd::native;
using sn::i64;

#include "capi_util.hpp"
using namespace slate_amd::native::capi;

namespace {
// ------------------------------------------------------------ host arrays
template <typename T>
int64_t h_potrf(char uplo, i64 n, T* a, i64 lda) {
    uplo = up(uplo);
    if (uplo != 'L' && uplo != 'U') return -1;
    if (n < 0) return -2;
    if (lda < std::max<i64>(1, n)) return -4;
    if (n == 0) return 0;
    return guarded([&]() -> int64_t {
        int p, q;
        grid_of(p, q);
        sn::HermitianMatrix<T> A(sn::Uplo::Lower, n, nb_of(n), p, q);
        std::vector<T> t;
        if (uplo == 'U') {            // factor A^H = L L^H (Lower), return U = L^H
            t = host_op<T>('C', n, n, a, lda);
            A.from_host(t.data(), n);
        } else {
            A.from_host(a, lda);
        }
        const int64_t info = sn::potrf(A);
        std::vector<T> r((size_t)n * n);
        A.to_host(r.data(), n);
        for (i64 j = 0; j < n; ++j)
            for (i64 i = j; i < n; ++i) {
                if (uplo == 'L') a[i + j * lda] = r[i + j * n];
                else a[j + i * lda] = cj(r[i + j * n]);
            }
        return info;
    });
}

// Lower factor of a (uplo) Cholesky factor held in a host array
template <typename T>
std::vector<T> lower_factor(char uplo, i64 n, const T* a, i64 lda) {
    std::vector<T> L((size_t)n * n, T(0));
    for (i64 j = 0; j < n; ++j)
        for (i64 i = j; i < n; ++i) L[i + j * n] = up(uplo) == 'L' ? a[i + j * lda] : cj(a[j + i * lda]);
    return L;
}

template <typename T>
int64_t h_potrs(char uplo, i64 n, i64 nrhs, const T* a, i64 lda, T* b, i64 ldb) {
    if (up(uplo) != 'L' && up(uplo) != 'U') return -1;
    if (n < 0) return -2;
    if (nrhs < 0) return -3;
    if (lda < std::max<i64>(1, n)) return -5;
    if (ldb < std::max<i64>(1, n)) return -7;
    if (n == 0 || nrhs == 0) return 0;
    return guarded([&]() -> int64_t {
        int p, q;
        grid_of(p, q);
        const i64 nb = nb_of(n);
        sn::HermitianMatrix<T> A(sn::Uplo::Lower, n, nb, p, q);
        sn::Matrix<T> B(n, nrhs, nb, p, q);
        const std::vector<T> L = lower_factor(uplo, n, a, lda);
        A.from_host(L.data(), n);
        B.from_host(b, ldb);
        sn::potrs(A, B);
        B.to_host(b, ldb);
        return 0;
    });
}

template <typename T>
int64_t h_posv(char uplo, i64 n, i64 nrhs, T* a, i64 lda, T* b, i64 ldb) {
    if (up(uplo) != 'L' && up(uplo) != 'U') return -1;
    if (n < 0) return -2;
    if (nrhs < 0) return -3;
    if (lda < std::max<i64>(1, n)) return -5;
    if (ldb < std::max<i64>(1, n)) return -7;
    const int64_t info = h_potrf<T>(uplo, n, a, lda);
    if (info != 0) return info;
    return h_potrs<T>(uplo, n, nrhs, a, lda, b, ldb);
}

// LAPACK dsposv / zcposv and dsgesv / zcgesv: A unchanged unless the
// working-precision fallback ran (then it holds the factors), X = A^-1 B
template <typename T>
int64_t h_posv_mixed(char uplo, i64 n, i64 nrhs, T* a, i64 lda, const T* b, i64 ldb, T* x, i64 ldx, int* iter) {
    uplo = up(uplo);
    if (uplo != 'L' && uplo != 'U') return -1;
    if (n < 0) return -2;
    if (nrhs < 0) return -3;
    if (lda < std::max<i64>(1, n)) return -5;
    if (ldb < std::max<i64>(1, n)) return -7;
    if (ldx < std::max<i64>(1, n)) return -9;
    if (n == 0 || nrhs == 0) return 0;
    return guarded([&]() -> int64_t {
        int p, q;
        grid_of(p, q);
        const i64 nb = nb_of(n);
        sn::Matrix<T> G(n, n, nb, p, q);
        G.from_host(a, lda);
        sn::HermitianMatrix<T> A(sn::Uplo::Lower, n, nb, p, q);
        if (uplo == 'U') sn::copy(sn::Op::ConjTrans, G, A);       // the stored upper triangle, as lower
        else sn::copy(sn::Op::NoTrans, G, A);
        sn::Matrix<T> B(n, nrhs, nb, p, q), X(n, nrhs, nb, p, q);
        B.from_host(b, ldb);
        const int64_t info = sn::posv_mixed(A, B, X, *iter);
        X.to_host(x, ldx);
        if (*iter < 0) {                                          // fallback: A holds the Cholesky factor
            if (uplo == 'U') {
                sn::copy(sn::Op::ConjTrans, A, G);
                std::vector<T> f((size_t)n * n);
                G.to_host(f.data(), n);
                for (i64 j = 0; j < n; ++j)
                    for (i64 i = 0; i <= j; ++i) a[i + j * lda] = f[i + j * n];
            } else {
                std::vector<T> f((size_t)n * n);
                A.to_host(f.data(), n);
                for (i64 j = 0; j < n; ++j)
                    for (i64 i = j; i < n; ++i) a[i + j * lda] = f[i + j * n];
            }
        }
        return info;
    });
}

template <typename T>
int64_t h_gesv_mixed(i64 n, i64 nrhs, T* a, i64 lda, int64_t* ipiv, const T* b, i64 ldb, T* x, i64 ldx, int* iter) {
    if (n < 0) return -1;
    if (nrhs < 0) return -2;
    if (lda < std::max<i64>(1, n)) return -4;
    if (ldb < std::max<i64>(1, n)) return -7;
    if (ldx < std::max<i64>(1, n)) return -9;
    if (n == 0 || nrhs == 0) return 0;
    return guarded([&]() -> int64_t {
        int p, q;
        grid_of(p, q);
        const i64 nb = nb_of(n);
        sn::Matrix<T> A(n, n, nb, p, q), B(n, nrhs, nb, p, q), X(n, nrhs, nb, p, q);
        A.from_host(a, lda);
        B.from_host(b, ldb);
        std::vector<int64_t> piv;
        const int64_t info = sn::gesv_mixed(A, piv, B, X, *iter);
        X.to_host(x, ldx);
        if (*iter < 0) A.to_host(a, lda);
        for (size_t i = 0; i < piv.size(); ++i) ipiv[i] = piv[i] + 1;
        return info;
    });
}

template <typename T>
int64_t h_getrf(i64 m, i64 n, T* a, i64 lda, int64_t* ipiv) {
    if (m < 0) return -1;
    if (n < 0) return -2;
    if (lda < std::max<i64>(1, m)) return -4;
    if (m == 0 || n == 0) return 0;
    return guarded([&]() -> int64_t {
        int p, q;
        grid_of(p, q);
        sn::Matrix<T> A(m, n, nb_of(std::max(m, n)), p, q);
        A.from_host(a, lda);
        std::vector<int64_t> piv;
        const int64_t info = sn::getrf(A, piv);
        A.to_host(a, lda);
        for (size_t i = 0; i < piv.size(); ++i) ipiv[i] = piv[i] + 1;     // LAPACK: 1-based
        return info;
    });
}

template <typename T>
int64_t h_getrs(char trans, i64 n, i64 nrhs, const T* a, i64 lda, const int64_t* ipiv, T* b, i64 ldb) {
    trans = up(trans);
    if (trans != 'N' && trans != 'T' && trans != 'C') return -1;
    if (n < 0) return -2;
    if (nrhs < 0) return -3;
    if (lda < std::max<i64>(1, n)) return -5;
    if (ldb < std::max<i64>(1, n)) return -8;
    if (n == 0 || nrhs == 0) return 0;
    return guarded([&]() -> int64_t {
        int p, q;
        grid_of(p, q);
        const i64 nb = nb_of(n);
        sn::Matrix<T> A(n, n, nb, p, q), B(n, nrhs, nb, p, q);
        A.from_host(a, lda);
        B.from_host(b, ldb);
        std::vector<int64_t> piv((size_t)n);
        for (i64 i = 0; i < n; ++i) piv[i] = ipiv[i] - 1;
        sn::Op op = op_of(trans);
        if (op == sn::Op::Trans && sn::is_cplx<T>()) {
            // A^T x = b  <=>  A^H conj(x) = conj(b)
            std::vector<T> cb = host_op<T>('N', n, nrhs, b, ldb);
            for (auto& x : cb) x = cj(x);
            B.from_host(cb.data(), n);
            sn::getrs(sn::Op::ConjTrans, A, piv, B);
            B.to_host(cb.data(), n);
            for (i64 j = 0; j < nrhs; ++j)
                for (i64 i = 0; i < n; ++i) b[i + j * ldb] = cj(cb[i + j * n]);
            return 0;
        }
        sn::getrs(op == sn::Op::Trans ? sn::Op::ConjTrans : op, A, piv, B);
        B.to_host(b, ldb);
        return 0;
    });
}

template <typename T>
int64_t h_gesv(i64 n, i64 nrhs, T* a, i64 lda, int64_t* ipiv, T* b, i64 ldb) {
    if (n < 0) return -1;
    if (nrhs < 0) return -2;
    if (lda < std::max<i64>(1, n)) return -4;
    if (ldb < std::max<i64>(1, n)) return -7;
    if (n == 0) return 0;
    return guarded([&]() -> int64_t {
        int p, q;
        grid_of(p, q);
        const i64 nb = nb_of(n);
        sn::Matrix<T> A(n, n, nb, p, q), B(n, std::max<i64>(nrhs, 1), nb, p, q);
        A.from_host(a, lda);
        if (nrhs) B.from_host(b, ldb);
        std::vector<int64_t> piv;
        const int64_t info = nrhs ? sn::gesv(A, piv, B) : sn::getrf(A, piv);
        A.to_host(a, lda);
        if (nrhs) B.to_host(b, ldb);
        for (size_t i = 0; i < piv.size(); ++i) ipiv[i] = piv[i] + 1;
        return info;
    });
}

template <typename T>
int64_t h_gemm(char ta, char tb, i64 m, i64 n, i64 k, T alpha, const T* a, i64 lda, const T* b, i64 ldb, T beta,
               T* c, i64 ldc) {
    ta = up(ta);
    tb = up(tb);
    if (ta != 'N' && ta != 'T' && ta != 'C') return -1;
    if (tb != 'N' && tb != 'T' && tb != 'C') return -2;
    if (m < 0) return -3;
    if (n < 0) return -4;
    if (k < 0) return -5;
    if (lda < std::max<i64>(1, ta == 'N' ? m : k)) return -8;
    if (ldb < std::max<i64>(1, tb == 'N' ? k : n)) return -10;
    if (ldc < std::max<i64>(1, m)) return -13;
    if (m == 0 || n == 0) return 0;
    return guarded([&]() -> int64_t {
        int p, q;
        grid_of(p, q);
        const i64 nb = nb_of(std::max({m, n, k}));
        // op() applied on the host copy (the operands are host arrays anyway)
        const std::vector<T> ao = host_op<T>(ta, m, k, a, lda);
        const std::vector<T> bo = host_op<T>(tb, k, n, b, ldb);
        sn::Matrix<T> A(m, std::max<i64>(k, 1), nb, p, q), B(std::max<i64>(k, 1), n, nb, p, q), C(m, n, nb, p, q);
        if (k) {
            A.from_host(ao.data(), m);
            B.from_host(bo.data(), k);
        }
        C.from_host(c, ldc);
        sn::gemm(k ? alpha : T(0), A, B, beta, C);
        C.to_host(c, ldc);
        return 0;
    });
}

// B = alpha op(A)^{-1} B (Left) or alpha B op(A)^{-1} (Right)
template <typename T>
int64_t h_trsm(char side, char uplo, char ta, char diag, i64 m, i64 n, T alpha, const T* a, i64 lda, T* b,
               i64 ldb) {
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
        // Right: X op(A) = alpha B  <=>  op(A)^H X^H = conj(alpha) B^H
        // complex Left Trans: op(A) = A^T = conj(A^H): solve on conj(A)
        std::vector<T> Ah((size_t)na * na);
        for (i64 j = 0; j < na; ++j)
            for (i64 i = 0; i < na; ++i) Ah[i + j * na] = a[i + j * lda];
        char opc = ta;
        const bool right = side == 'R';
        if (right) opc = ta == 'N' ? 'C' : ta == 'C' ? 'N' : 'X';     // X: conj(A) NoTrans
        else if (ta == 'T' && sn::is_cplx<T>()) opc = 'Y';             // Y: conj(A) ConjTrans
        else if (ta == 'T') opc = 'C';
        if (opc == 'X' || opc == 'Y') {
            for (auto& x : Ah) x = cj(x);
            opc = opc == 'X' ? 'N' : 'C';
        }
        if (right && ta == 'T' && !sn::is_cplx<T>()) opc = 'N';
        sn::Matrix<T> A(na, na, nb, p, q);
        A.from_host(Ah.data(), na);
        const i64 bm = right ? n : m, bn = right ? m : n;
        std::vector<T> Bh = right ? host_op<T>('C', bm, bn, b, ldb) : host_op<T>('N', bm, bn, b, ldb);
        sn::Matrix<T> B(bm, bn, nb, p, q);
        B.from_host(Bh.data(), bm);
        sn::trsm(sn::Side::Left, uplo == 'L' ? sn::Uplo::Lower : sn::Uplo::Upper,
                 opc == 'N' ? sn::Op::NoTrans : sn::Op::ConjTrans, diag == 'U' ? sn::Diag::Unit : sn::Diag::NonUnit,
                 right ? cj(alpha) : alpha, A, B);
        B.to_host(Bh.data(), bm);
        for (i64 j = 0; j < n; ++j)
            for (i64 i = 0; i < m; ++i) b[i + j * ldb] = right ? cj(Bh[j + i * bm]) : Bh[i + j * bm];
        return 0;
    });
}

// least squares, trans = 'N', m >= n: X in the top n rows of b
template <typename T>
int64_t h_gels(char trans, i64 m, i64 n, i64 nrhs, T* a, i64 lda, T* b, i64 ldb) {
    if (up(trans) != 'N') return -1;
    if (m < 0) return -2;
    if (n < 0 || n > m) return -3;
    if (nrhs < 0) return -4;
    if (lda < std::max<i64>(1, m)) return -6;
    if (ldb < std::max<i64>(1, m)) return -8;
    if (m == 0 || n == 0 || nrhs == 0) return 0;
    return guarded([&]() -> int64_t {
        const int q = sn::size();                 // 1 x P: geqrf distributes columns
        const i64 nb = nb_of(std::max(m, n));
        sn::Matrix<T> A(m, n, nb, 1, q), B(m, nrhs, nb, 1, q);
        A.from_host(a, lda);
        B.from_host(b, ldb);
        sn::gels(A, B);
        A.to_host(a, lda);
        B.to_host(b, ldb);
        return 0;
    });
}

template <typename T>
double h_lange(char norm, i64 m, i64 n, const T* a, i64 lda) {
    if (m == 0 || n == 0) return 0.0;
    double r = -1.0;
    const int64_t rc = guarded([&]() -> int64_t {
        int p, q;
        grid_of(p, q);
        sn::Matrix<T> A(m, n, nb_of(std::max(m, n)), p, q);
        A.from_host(a, lda);
        const char k = up(norm) == 'M' ? 'M' : up(norm) == 'I' ? 'I' : (up(norm) == 'F' || up(norm) == 'E') ? 'F' : '1';
        r = sn::norm((sn::Norm)k, A);
        return 0;
    });
    return rc == 0 ? r : -1.0;
}

// ------------------------------------------------------------ BLACS / ScaLAPACK
struct Ctx {
    int p = 1, q = 1;
    bool row_major = false;
};
std::vector<Ctx>& contexts() {
    static std::vector<Ctx> c;
    return c;
}

const Ctx& ctx_of(int ctxt) {
    auto& c = contexts();
    if (ctxt < 0 || ctxt >= (int)c.size()) throw sn::Error("BLACS: unknown context " + std::to_string(ctxt));
    return c[ctxt];
}

// ---- ScaLAPACK operands.  The whole-matrix, aligned case (ia = ja = 1,
// sizes equal to the descriptor's, MB = NB, RSRC = CSRC = 0, column-major
// grid) is a local copy of the caller's array.  Anything else -- a
// sub-matrix A(ia:ia+m-1, ja:ja+n-1) at any offset, MB != NB, a non-zero
// source process, a row-major BLACS grid (reference
// scalapack_api/scalapack_slate.hh:81-120 takes the same operands) -- is
// redistributed into an aligned m x n native matrix (tile NB, column-major
// grid) and back: each rank sends the values it owns straight to their new
// owner, in a canonical order (global column-major over the elements a
// source / destination pair shares), so only values travel.
ScalLay scal_lay(const int* desc) {
    const Ctx& c = ctx_of(desc[1]);
    return ScalLay{desc[2], desc[3], desc[4], desc[5], desc[8], desc[6], desc[7], c.p, c.q, c.row_major};
}
struct SubInfo {
    std::weak_ptr<sn::Storage> st;
    std::vector<int> desc;
    i64 i0, j0;                 // 0-based origin of the sub-matrix
};
std::map<const sn::Storage*, SubInfo>& sub_registry() {
    static std::map<const sn::Storage*, SubInfo> r;
    return r;
}
const SubInfo* sub_of(const sn::Storage* s) {
    auto& r = sub_registry();
    auto it = r.find(s);
    if (it == r.end()) return nullptr;
    auto sp = it->second.st.lock();
    if (!sp || sp.get() != s) { r.erase(it); return nullptr; }
    return &it->second;
}
bool scal_aligned(const int* desc, i64 m, i64 n, int ia, int ja) {
    const Ctx& c = ctx_of(desc[1]);
    return ia == 1 && ja == 1 && desc[2] == m && desc[3] == n && desc[4] == desc[5] && desc[6] == 0 && desc[7] == 0 &&
           !(c.row_major && c.p > 1 && c.q > 1);
}

// a native matrix over a ScaLAPACK operand (any sub-matrix, see above)
template <typename T>
sn::Matrix<T> scal_matrix(const int* desc, i64 m, i64 n, int ia, int ja, const T* a) {
    if (ia < 1 || ja < 1 || ia - 1 + m > desc[2] || ja - 1 + n > desc[3])
        throw sn::Error("native ScaLAPACK: sub-matrix outside the descriptor's matrix");
    if (desc[4] < 1 || desc[5] < 1) throw sn::Error("native ScaLAPACK: bad block sizes");
    const Ctx& c = ctx_of(desc[1]);
    if (scal_aligned(desc, m, n, ia, ja)) {
        sn::Matrix<T> A(m, n, desc[5], c.p, c.q);
        if (A.mloc() > desc[8]) throw sn::Error("native ScaLAPACK: lld smaller than the local rows");
        if (A.mloc() && A.nloc()) A.from_local_host(a, desc[8]);
        return A;
    }
    const ScalLay L = scal_lay(desc);
    sn::Matrix<T> A(m, n, desc[5], c.p, c.q);
    const sn::Storage& S = *A.storage();
    std::vector<T> loc((size_t)std::max<i64>(S.mloc, 1) * std::max<i64>(S.nloc, 1));
    scal_move<T>(L, ia - 1, ja - 1, m, n, const_cast<T*>(a), S, loc.data(), std::max<i64>(S.mloc, 1), true);
    if (A.mloc() && A.nloc()) A.from_local_host(loc.data(), std::max<i64>(S.mloc, 1));
    sub_registry()[A.storage().get()] = SubInfo{A.storage(), std::vector<int>(desc, desc + 9), ia - 1, ja - 1};
    return A;
}
// the native result back into the caller's array: exactly the elements of
// the sub-matrix change
template <typename T>
void scal_back(const sn::Matrix<T>& A, const int* desc, T* a) {
    const SubInfo* si = sub_of(A.storage().get());
    if (!si) {
        if (A.mloc() && A.nloc()) A.to_local_host(a, desc[8]);
        return;
    }
    const sn::Storage& S = *A.storage();
    std::vector<T> loc((size_t)std::max<i64>(S.mloc, 1) * std::max<i64>(S.nloc, 1));
    if (A.mloc() && A.nloc()) A.to_local_host(loc.data(), std::max<i64>(S.mloc, 1));
    scal_move<T>(scal_lay(si->desc.data()), si->i0, si->j0, A.m(), A.n(), a, S, loc.data(), std::max<i64>(S.mloc, 1),
                 false);
}
// dst's uplo triangle (global, diagonal included) := src's (same distribution)
template <typename T>
void tri_into(char uplo, const sn::Matrix<T>& src, sn::Matrix<T>& dst) {
    const sn::Storage& S = *dst.storage();
    if (!S.mloc || !S.nloc) return;
    slate_hip::TriMask mk;
    mk.mode = uplo == 'L' ? 1 : 2;
    mk.p = S.p; mk.pr = S.pr; mk.q = S.q; mk.pc = S.pc; mk.nb = S.nb;
    slate_hip::gecopy_mask_merge<sn::K<T>>(mk, S.mloc, S.nloc, sn::kp(src.data()), src.lld(), sn::kp(dst.data()),
                                           S.lld, sn::rt().main);
    NHIP(hipStreamSynchronize(sn::rt().main));
}
template <typename T>
sn::HermitianMatrix<T> scal_herm(const int* desc, i64 n, int ia, int ja, const T* a) {
    sn::Matrix<T> G = scal_matrix<T>(desc, n, n, ia, ja, a);
    sn::HermitianMatrix<T> H(sn::Uplo::Lower, n, G.nb(), G.p(), G.q());
    sn::copy(sn::Op::NoTrans, G, H);
    return H;
}

// ScaLAPACK ipiv (tied to the descriptor's matrix): entry of local row li of
// the global row ia-1+k = 1-based global row that row was swapped with
// (ia-1 + the sub-matrix pivot + 1); <-> the 0-based sub-matrix sequence of
// the native driver, replicated over the process columns
template <typename T>
void ipiv_to_local(const sn::Matrix<T>& A, const int* desc, int ia, const std::vector<int64_t>& piv, int* ipiv) {
    const ScalLay L = scal_lay(desc);
    int myr, myc;
    L.coords(sn::rank(), myr, myc);
    if (sn::rank() >= L.p * L.q) return;
    for (size_t k = 0; k < piv.size(); ++k) {
        const i64 g = ia - 1 + (i64)k;
        if (L.orow(g) == myr) ipiv[ScalLay::g2l(g, L.mb, L.p)] = (int)(ia + piv[k]);
    }
}
template <typename T>
std::vector<int64_t> ipiv_from_local(const sn::Matrix<T>& A, const int* desc, int ia, int ja, i64 k,
                                     const int* ipiv) {
    const ScalLay L = scal_lay(desc);
    int myr, myc;
    L.coords(sn::rank(), myr, myc);
    std::vector<int64_t> g((size_t)std::max<i64>(k, 1), 0);
    if (sn::rank() < L.p * L.q && myc == L.ocol(ja - 1))      // the panel's process column
        for (i64 kk = 0; kk < k; ++kk) {
            const i64 gi = ia - 1 + kk;
            if (L.orow(gi) == myr) g[kk] = ipiv[ScalLay::g2l(gi, L.mb, L.p)] - ia;
        }
    if (sn::size() > 1) {       // one owner per entry: a sum over the world
        sn::Scratch d(sizeof(int64_t) * g.size(), sn::rt().main);
        sn::upload(d.p, g.data(), sizeof(int64_t) * g.size(), sn::rt().main);
        sn::world_comm()->allreduce(d.p, g.size(), sn::DT::I64, 's', sn::rt().main);
        NHIP(hipMemcpyAsync(g.data(), d.p, sizeof(int64_t) * g.size(), hipMemcpyDeviceToHost, sn::rt().main));
        NHIP(hipStreamSynchronize(sn::rt().main));
    }
    g.resize((size_t)k);
    (void)A;
    return g;
}

template <typename T>
int p_potrf(char uplo, int n, T* a, int ia, int ja, const int* desca) {
    uplo = up(uplo);
    if (uplo != 'L' && uplo != 'U') return -1;
    if (n == 0) return 0;
    return (int)guarded([&]() -> int64_t {
        // the factor as Lower storage (Upper: L = U^H), then only the uplo
        // triangle of the caller's sub-matrix changes
        sn::Matrix<T> G = scal_matrix<T>(desca, n, n, ia, ja, a);
        sn::HermitianMatrix<T> A(sn::Uplo::Lower, n, G.nb(), G.p(), G.q());
        sn::copy(uplo == 'U' ? sn::Op::ConjTrans : sn::Op::NoTrans, G, A);
        const int64_t info = sn::potrf(A);
        if (uplo == 'U') {
            sn::Matrix<T> Ut(n, n, G.nb(), G.p(), G.q());
            sn::copy(sn::Op::ConjTrans, A, Ut);
            tri_into<T>('U', Ut, G);
        } else {
            tri_into<T>('L', A, G);
        }
        scal_back(G, desca, a);
        return info;
    });
}

template <typename T>
int p_potrs(char uplo, int n, int nrhs, const T* a, int ia, int ja, const int* desca, T* b, int ib, int jb,
            const int* descb) {
    uplo = up(uplo);
    if (uplo != 'L' && uplo != 'U') return -1;
    if (n == 0 || nrhs == 0) return 0;
    return (int)guarded([&]() -> int64_t {
        sn::HermitianMatrix<T> A = scal_herm<T>(desca, n, ia, ja, a);
        if (uplo == 'U') {
            sn::Matrix<T> U = scal_matrix<T>(desca, n, n, ia, ja, a);
            sn::Matrix<T> Lg(n, n, A.nb(), A.p(), A.q());
            sn::copy(sn::Op::ConjTrans, U, Lg);
            sn::copy(sn::Op::NoTrans, Lg, A);
        }
        sn::Matrix<T> B = scal_matrix<T>(descb, n, nrhs, ib, jb, b);
        sn::potrs(A, B);
        scal_back(B, descb, b);
        return 0;
    });
}

template <typename T>
int p_posv(char uplo, int n, int nrhs, T* a, int ia, int ja, const int* desca, T* b, int ib, int jb,
           const int* descb) {
    const int info = p_potrf<T>(uplo, n, a, ia, ja, desca);
    if (info != 0) return info;
    return p_potrs<T>(uplo, n, nrhs, a, ia, ja, desca, b, ib, jb, descb);
}

// p?gesv_mixed (reference scalapack_api/scalapack_gesv_mixed.cc): factor in
// the lower precision, refine in the working one; X = A^-1 B, B unchanged
template <typename T>
int p_gesv_mixed(int n, int nrhs, T* a, int ia, int ja, const int* desca, int* ipiv, const T* b, int ib, int jb,
                 const int* descb, T* x, int ix, int jx, const int* descx, int* iter) {
    if (n < 0) return -1;
    if (nrhs < 0) return -2;
    *iter = 0;
    if (n == 0 || nrhs == 0) return 0;
    return (int)guarded([&]() -> int64_t {
        sn::Matrix<T> A = scal_matrix<T>(desca, n, n, ia, ja, a);
        sn::Matrix<T> B = scal_matrix<T>(descb, n, nrhs, ib, jb, b);
        sn::Matrix<T> X = scal_matrix<T>(descx, n, nrhs, ix, jx, x);
        if (B.nb() != A.nb() || X.nb() != A.nb() || B.p() != A.p() || X.p() != A.p() || B.q() != A.q() ||
            X.q() != A.q())
            throw sn::Error("native p?gesv_mixed: B and X must have A's block size and grid");
        std::vector<int64_t> piv;
        int it = 0;
        const int64_t info = sn::gesv_mixed<T>(A, piv, B, X, it);
        *iter = it;
        scal_back(X, descx, x);
        if (it < 0) {            // the working-precision fallback factored A (LAPACK dsgesv semantics)
            scal_back(A, desca, a);
            ipiv_to_local(A, desca, ia, piv, ipiv);
        }
        return info;
    });
}

template <typename T>
int p_getrf(int m, int n, T* a, int ia, int ja, const int* desca, int* ipiv) {
    if (m == 0 || n == 0) return 0;
    return (int)guarded([&]() -> int64_t {
        sn::Matrix<T> A = scal_matrix<T>(desca, m, n, ia, ja, a);
        std::vector<int64_t> piv;
        const int64_t info = sn::getrf(A, piv);
        scal_back(A, desca, a);
        ipiv_to_local(A, desca, ia, piv, ipiv);
        return info;
    });
}

template <typename T>
int p_getrs(char trans, int n, int nrhs, const T* a, int ia, int ja, const int* desca, const int* ipiv, T* b,
            int ib, int jb, const int* descb) {
    trans = up(trans);
    if (trans != 'N' && trans != 'T' && trans != 'C') return -1;
    if (n == 0 || nrhs == 0) return 0;
    return (int)guarded([&]() -> int64_t {
        sn::Matrix<T> A = scal_matrix<T>(desca, n, n, ia, ja, a);
        sn::Matrix<T> B = scal_matrix<T>(descb, n, nrhs, ib, jb, b);
        const std::vector<int64_t> piv = ipiv_from_local(A, desca, ia, ja, n, ipiv);
        if (trans == 'T' && sn::is_cplx<T>()) throw sn::Error("native pgetrs: trans = 'T' of a complex matrix");
        sn::getrs(trans == 'N' ? sn::Op::NoTrans : sn::Op::ConjTrans, A, piv, B);
        scal_back(B, descb, b);
        return 0;
    });
}

template <typename T>
int p_gesv(int n, int nrhs, T* a, int ia, int ja, const int* desca, int* ipiv, T* b, int ib, int jb,
           const int* descb) {
    if (n == 0) return 0;
    return (int)guarded([&]() -> int64_t {
        sn::Matrix<T> A = scal_matrix<T>(desca, n, n, ia, ja, a);
        std::vector<int64_t> piv;
        int64_t info;
        if (nrhs) {
            sn::Matrix<T> B = scal_matrix<T>(descb, n, nrhs, ib, jb, b);
            info = sn::gesv(A, piv, B);
            scal_back(B, descb, b);
        } else {
            info = sn::getrf(A, piv);
        }
        scal_back(A, desca, a);
        ipiv_to_local(A, desca, ia, piv, ipiv);
        return info;
    });
}

template <typename T>
void p_gemm(char ta, char tb, int m, int n, int k, T alpha, const T* a, int ia, int ja, const int* desca, const T* b,
            int ib, int jb, const int* descb, T beta, T* c, int ic, int jc, const int* descc) {
    ta = up(ta);
    tb = up(tb);
    if (m == 0 || n == 0) return;
    const int64_t rc = guarded([&]() -> int64_t {
        sn::Matrix<T> A = scal_matrix<T>(desca, ta == 'N' ? m : k, ta == 'N' ? k : m, ia, ja, a);
        sn::Matrix<T> B = scal_matrix<T>(descb, tb == 'N' ? k : n, tb == 'N' ? n : k, ib, jb, b);
        sn::Matrix<T> C = scal_matrix<T>(descc, m, n, ic, jc, c);
        sn::gemm(op_of(ta), op_of(tb), alpha, A, B, beta, C);
        scal_back(C, descc, c);
        return 0;
    });
    if (rc != 0) std::fprintf(stderr, "slate_amd native p?gemm_: %s\n", g_err.c_str());
}

// conj(A) in place (host round trip of the local block: compat path only)
template <typename T>
void conj_inplace(sn::Matrix<T>& A) {
    if constexpr (sn::is_cplx<T>()) {
        if (!A.mloc() || !A.nloc()) return;
        std::vector<T> h((size_t)A.mloc() * A.nloc());
        A.to_local_host(h.data(), A.mloc());
        for (auto& x : h) x = std::conj(x);
        A.from_local_host(h.data(), A.mloc());
    }
}

// B = alpha op(A)^{-1} B (Left) or alpha B op(A)^{-1} (Right), TRANSA N / T / C.
// The native solve is Left with NoTrans / ConjTrans: a complex Trans solves
// with conj(A) and ConjTrans (A^T = conj(A)^H); Right: X op(A) = alpha B <=>
// op(A)^H X^H = conj(alpha) B^H
template <typename T>
void p_trsm(char side, char uplo, char ta, char diag, int m, int n, T alpha, const T* a, int ia, int ja,
            const int* desca, T* b, int ib, int jb, const int* descb) {
    side = up(side);
    uplo = up(uplo);
    ta = up(ta);
    diag = up(diag);
    if (m == 0 || n == 0) return;
    const int64_t rc = guarded([&]() -> int64_t {
        if (side != 'L' && side != 'R') throw sn::Error("native p?trsm_: SIDE must be L or R");
        if (uplo != 'L' && uplo != 'U') throw sn::Error("native p?trsm_: UPLO must be L or U");
        if (ta != 'N' && ta != 'T' && ta != 'C') throw sn::Error("native p?trsm_: TRANSA must be N, T or C");
        if (diag != 'N' && diag != 'U') throw sn::Error("native p?trsm_: DIAG must be N or U");
        const bool right = side == 'R';
        const int na = right ? n : m;
        sn::Matrix<T> A = scal_matrix<T>(desca, na, na, ia, ja, a);
        sn::Matrix<T> B = scal_matrix<T>(descb, m, n, ib, jb, b);
        // effective left operation on A: 'N', 'C', or conj(A) with 'N' / 'C'
        char opc;
        bool conjA = false;
        if (!right) {
            opc = ta == 'N' ? 'N' : 'C';
            conjA = ta == 'T' && sn::is_cplx<T>();
        } else {
            opc = ta == 'N' ? 'C' : 'N';            // (op A)^H
            conjA = ta == 'T' && sn::is_cplx<T>();  // (A^T)^H = conj(A)
        }
        if (conjA) conj_inplace(A);
        const sn::Uplo ul = uplo == 'L' ? sn::Uplo::Lower : sn::Uplo::Upper;
        const sn::Diag dg = diag == 'U' ? sn::Diag::Unit : sn::Diag::NonUnit;
        const sn::Op op = opc == 'N' ? sn::Op::NoTrans : sn::Op::ConjTrans;
        if (!right) {
            sn::trsm(sn::Side::Left, ul, op, dg, alpha, A, B);
            scal_back(B, descb, b);
        } else {
            sn::Matrix<T> Bh(n, m, B.nb(), B.p(), B.q());
            sn::copy(sn::Op::ConjTrans, B, Bh);
            sn::trsm(sn::Side::Left, ul, op, dg, sn::conj_of(alpha), A, Bh);
            sn::copy(sn::Op::ConjTrans, Bh, B);
            scal_back(B, descb, b);
        }
        return 0;
    });
    if (rc != 0) std::fprintf(stderr, "slate_amd native p?trsm_: %s\n", g_err.c_str());
}

// p?gels_ on any BLACS grid (p > 1: TSQR panels -- R in A's upper triangle
// as ScaLAPACK's, the entries below it hold the TSQR tree's local reflectors,
// not ScaLAPACK's Householder vectors); lwork = -1 is a workspace query (the
// library allocates its own: returns 1)
template <typename T>
int p_gels(char trans, int m, int n, int nrhs, T* a, int ia, int ja, const int* desca, T* b, int ib, int jb,
           const int* descb, T* work, int lwork) {
    if (lwork == -1) {
        if (work) work[0] = T(1);
        return 0;
    }
    if (up(trans) != 'N') return -1;
    if (n > m) return -3;
    if (m == 0 || n == 0 || nrhs == 0) return 0;
    return (int)guarded([&]() -> int64_t {
        sn::Matrix<T> A = scal_matrix<T>(desca, m, n, ia, ja, a);
        sn::Matrix<T> B = scal_matrix<T>(descb, m, nrhs, ib, jb, b);
        sn::gels(A, B);
        scal_back(A, desca, a);
        scal_back(B, descb, b);
        return 0;
    });
}

template <typename T>
sn::HermitianMatrix<T> scal_tri(const int* desc, i64 n, int ia, int ja, const T* a, char uplo) {
    sn::Matrix<T> G = scal_matrix<T>(desc, n, n, ia, ja, a);
    sn::HermitianMatrix<T> H(uplo == 'U' ? sn::Uplo::Upper : sn::Uplo::Lower, n, G.nb(), G.p(), G.q());
    sn::copy(sn::Op::NoTrans, G, H);
    return H;
}

// C(uplo) *= beta on the caller's sub-matrix (k = 0 rank updates)
template <typename T>
void scal_scale_tri(const int* desc, int n, int ic, int jc, char uplo, T beta, T* c) {
    const ScalLay L = scal_lay(desc);
    int myr, myc;
    L.coords(sn::rank(), myr, myc);
    if (sn::rank() >= L.p * L.q) return;
    for (i64 sj = 0; sj < n; ++sj) {
        const i64 gj = jc - 1 + sj;
        if (L.ocol(gj) != myc) continue;
        const i64 lj = ScalLay::g2l(gj, L.nb, L.q);
        for (i64 si = 0; si < n; ++si) {
            const i64 gi = ic - 1 + si;
            if (L.orow(gi) != myr || (uplo == 'L' ? si < sj : si > sj)) continue;
            c[ScalLay::g2l(gi, L.mb, L.p) + lj * L.lld] *= beta;
        }
    }
}

// p?potri_: the inverse from the Cholesky factor, over the uplo triangle
template <typename T>
int p_potri(char uplo, int n, T* a, int ia, int ja, const int* desca) {
    uplo = up(uplo);
    if (uplo != 'L' && uplo != 'U') return -1;
    if (n == 0) return 0;
    return (int)guarded([&]() -> int64_t {
        sn::Matrix<T> G = scal_matrix<T>(desca, n, n, ia, ja, a);
        sn::HermitianMatrix<T> L(sn::Uplo::Lower, n, G.nb(), G.p(), G.q());
        sn::copy(uplo == 'U' ? sn::Op::ConjTrans : sn::Op::NoTrans, G, L);   // U = L^H: the factor as lower
        sn::potri(L);
        sn::Matrix<T> R(n, n, G.nb(), G.p(), G.q());
        sn::copy(uplo == 'U' ? sn::Op::ConjTrans : sn::Op::NoTrans, L, R);
        tri_into<T>(uplo, R, G);
        scal_back(G, desca, a);
        return 0;
    });
}

// p?getri_: the inverse from the LU factors and ScaLAPACK pivots; lwork /
// liwork = -1 are workspace queries (the library allocates its own)
template <typename T>
int p_getri(int n, T* a, int ia, int ja, const int* desca, const int* ipiv, T* work, int lwork, int* iwork,
            int liwork) {
    if (lwork == -1 || liwork == -1) {
        if (work) work[0] = T(1);
        if (iwork) iwork[0] = 1;
        return 0;
    }
    if (n == 0) return 0;
    return (int)guarded([&]() -> int64_t {
        sn::Matrix<T> A = scal_matrix<T>(desca, n, n, ia, ja, a);
        const std::vector<int64_t> piv = ipiv_from_local(A, desca, ia, ja, n, ipiv);
        sn::getri(A, piv);
        scal_back(A, desca, a);
        return 0;
    });
}

// p?syrk_ / p?herk_ / p?syr2k_ / p?her2k_ (whole matrices, ia = ja = 1)
template <typename T>
void p_rank_k(bool herm, bool two, char uplo, char trans, int n, int k, T alpha, const T* a, int ia, int ja,
              const int* desca, const T* b, int ib, int jb, const int* descb, T beta, T* c, int ic, int jc,
              const int* descc) {
    uplo = up(uplo);
    trans = up(trans);
    if (n == 0) return;
    const int64_t rc = guarded([&]() -> int64_t {
        if (k == 0 || alpha == T(0)) {
            if (beta != T(1)) scal_scale_tri<T>(descc, n, ic, jc, uplo, beta, c);
            return 0;
        }
        const bool nt = trans == 'N';
        const sn::Op op = nt ? sn::Op::NoTrans : (herm ? sn::Op::ConjTrans : sn::Op::Trans);
        sn::Matrix<T> A = scal_matrix<T>(desca, nt ? n : k, nt ? k : n, ia, ja, a);
        sn::HermitianMatrix<T> C = scal_tri<T>(descc, n, ic, jc, c, uplo);
        using R = sn::real_t<T>;
        if (two) {
            sn::Matrix<T> B = scal_matrix<T>(descb, nt ? n : k, nt ? k : n, ib, jb, b);
            if (herm) sn::her2k(op, alpha, A, B, (R)std::real(beta), C);
            else sn::syr2k(op, alpha, A, B, beta, C);
        } else if (herm) {
            sn::herk(op, (R)std::real(alpha), A, (R)std::real(beta), C);
        } else {
            sn::syrk(op, alpha, A, beta, C);
        }
        scal_back(C, descc, c);
        return 0;
    });
    if (rc != 0) std::fprintf(stderr, "slate_amd native p?%s_: %s\n", two ? (herm ? "her2k" : "syr2k") : (herm ? "herk" : "syrk"),
                              g_err.c_str());
}

// p?symm_ / p?hemm_
template <typename T>
void p_xmm(bool herm, char side, char uplo, int m, int n, T alpha, const T* a, int ia, int ja, const int* desca,
           const T* b, int ib, int jb, const int* descb, T beta, T* c, int ic, int jc, const int* descc) {
    side = up(side);
    uplo = up(uplo);
    if (m == 0 || n == 0) return;
    const int64_t rc = guarded([&]() -> int64_t {
        const int na = side == 'L' ? m : n;
        sn::HermitianMatrix<T> A = scal_tri<T>(desca, na, ia, ja, a, uplo);
        sn::Matrix<T> B = scal_matrix<T>(descb, m, n, ib, jb, b);
        sn::Matrix<T> C = scal_matrix<T>(descc, m, n, ic, jc, c);
        const sn::Side sd = side == 'L' ? sn::Side::Left : sn::Side::Right;
        if (herm) sn::hemm(sd, alpha, A, B, beta, C);
        else sn::symm(sd, alpha, A, B, beta, C);
        scal_back(C, descc, c);
        return 0;
    });
    if (rc != 0) std::fprintf(stderr, "slate_amd native p?%s_: %s\n", herm ? "hemm" : "symm", g_err.c_str());
}

template <typename T>
void p_trmm(char side, char uplo, char ta, char diag, int m, int n, T alpha, const T* a, int ia, int ja,
            const int* desca, T* b, int ib, int jb, const int* descb) {
    side = up(side);
    uplo = up(uplo);
    ta = up(ta);
    if (m == 0 || n == 0) return;
    const int64_t rc = guarded([&]() -> int64_t {
        const int na = side == 'L' ? m : n;
        sn::Matrix<T> A = scal_matrix<T>(desca, na, na, ia, ja, a);
        sn::Matrix<T> B = scal_matrix<T>(descb, m, n, ib, jb, b);
        sn::trmm(side == 'L' ? sn::Side::Left : sn::Side::Right, uplo == 'L' ? sn::Uplo::Lower : sn::Uplo::Upper,
                 op_of(ta), up(diag) == 'U' ? sn::Diag::Unit : sn::Diag::NonUnit, alpha, A, B);
        scal_back(B, descb, b);
        return 0;
    });
    if (rc != 0) std::fprintf(stderr, "slate_amd native p?trmm_: %s\n", g_err.c_str());
}

// p?lansy_ / p?lanhe_ / p?lantr_ (square triangular)
template <typename T>
double p_lan_struct(int kind, char norm, char uplo, char diag, int n, const T* a, int ia, int ja, const int* desca) {
    if (n == 0) return 0.0;
    double r = -1.0;
    const int64_t rc = guarded([&]() -> int64_t {
        const char k = up(norm) == 'M' ? 'M' : up(norm) == 'I' ? 'I' : (up(norm) == 'F' || up(norm) == 'E') ? 'F' : '1';
        const sn::Uplo ul = up(uplo) == 'U' ? sn::Uplo::Upper : sn::Uplo::Lower;
        if (kind == 0) {
            sn::Matrix<T> A = scal_matrix<T>(desca, n, n, ia, ja, a);
            r = sn::norm_triangular((sn::Norm)k, ul, up(diag) == 'U' ? sn::Diag::Unit : sn::Diag::NonUnit, A);
        } else {
            sn::HermitianMatrix<T> A = scal_tri<T>(desca, n, ia, ja, a, up(uplo));
            r = kind == 1 ? sn::norm((sn::Norm)k, A) : sn::norm_symmetric((sn::Norm)k, A);
        }
        return 0;
    });
    if (rc != 0) std::fprintf(stderr, "slate_amd native p?lan*_: %s\n", g_err.c_str());
    return r;
}

template <typename T>
double p_lange(char norm, int m, int n, const T* a, int ia, int ja, const int* desca) {
    if (m == 0 || n == 0) return 0.0;
    double r = -1.0;
    const int64_t rc = guarded([&]() -> int64_t {
        sn::Matrix<T> A = scal_matrix<T>(desca, m, n, ia, ja, a);
        const char k = up(norm) == 'M' ? 'M' : up(norm) == 'I' ? 'I' : (up(norm) == 'F' || up(norm) == 'E') ? 'F' : '1';
        r = sn::norm((sn::Norm)k, A);
        return 0;
    });
    if (rc != 0) std::fprintf(stderr, "slate_amd native p?lange_: %s\n", g_err.c_str());
    return r;
}

}  // namespace

// ---- condition estimates (reference lapack_api/lapack_gecon.cc, pocon, trcon
// and scalapack_api/scalapack_gecon.cc, pocon, trcon)
inline sn::Norm cond_norm(char norm) {
    norm = up(norm);
    if (norm == '1' || norm == 'O') return sn::Norm::One;
    if (norm == 'I') return sn::Norm::Inf;
    throw sn::Error("condition estimate: NORM must be '1', 'O' or 'I'");
}
template <typename T>
int h_gecon(char norm, i64 n, const T* a, i64 lda, double anorm, double* rcond) {
    if (n < 0) return -2;
    if (lda < std::max<i64>(1, n)) return -4;
    return (int)guarded([&]() -> int64_t {
        int p, q;
        grid_of(p, q);
        sn::Matrix<T> A(n, n, nb_of(n), p, q);
        A.from_host(a, lda);
        *rcond = sn::gecondest(cond_norm(norm), A, anorm);
        return 0;
    });
}
template <typename T>
int h_pocon(char uplo, i64 n, const T* a, i64 lda, double anorm, double* rcond) {
    uplo = up(uplo);
    if (uplo != 'L' && uplo != 'U') return -1;
    if (lda < std::max<i64>(1, n)) return -4;
    return (int)guarded([&]() -> int64_t {
        int p, q;
        grid_of(p, q);
        const i64 nb = nb_of(n);
        sn::Matrix<T> G(n, n, nb, p, q);
        G.from_host(a, lda);
        sn::HermitianMatrix<T> L(sn::Uplo::Lower, n, nb, p, q);
        sn::copy(uplo == 'U' ? sn::Op::ConjTrans : sn::Op::NoTrans, G, L);
        *rcond = sn::pocondest(sn::Norm::One, L, anorm);
        return 0;
    });
}
template <typename T>
int h_trcon(char norm, char uplo, char diag, i64 n, const T* a, i64 lda, double* rcond) {
    uplo = up(uplo);
    diag = up(diag);
    if (uplo != 'L' && uplo != 'U') return -2;
    if (diag != 'N' && diag != 'U') return -3;
    if (lda < std::max<i64>(1, n)) return -6;
    return (int)guarded([&]() -> int64_t {
        int p, q;
        grid_of(p, q);
        sn::Matrix<T> A(n, n, nb_of(n), p, q);
        A.from_host(a, lda);
        *rcond = sn::trcondest(cond_norm(norm), uplo == 'L' ? sn::Uplo::Lower : sn::Uplo::Upper,
                               diag == 'U' ? sn::Diag::Unit : sn::Diag::NonUnit, A);
        return 0;
    });
}
template <typename T>
int p_gecon(char norm, int n, const T* a, int ia, int ja, const int* desca, double anorm, double* rcond) {
    if (n == 0) { *rcond = 1.0; return 0; }
    return (int)guarded([&]() -> int64_t {
        sn::Matrix<T> A = scal_matrix<T>(desca, n, n, ia, ja, a);
        *rcond = sn::gecondest(cond_norm(norm), A, anorm);
        return 0;
    });
}
template <typename T>
int p_pocon(char uplo, int n, const T* a, int ia, int ja, const int* desca, double anorm, double* rcond) {
    uplo = up(uplo);
    if (uplo != 'L' && uplo != 'U') return -1;
    if (n == 0) { *rcond = 1.0; return 0; }
    return (int)guarded([&]() -> int64_t {
        sn::Matrix<T> G = scal_matrix<T>(desca, n, n, ia, ja, a);
        sn::HermitianMatrix<T> L(sn::Uplo::Lower, n, G.nb(), G.p(), G.q());
        sn::copy(uplo == 'U' ? sn::Op::ConjTrans : sn::Op::NoTrans, G, L);
        *rcond = sn::pocondest(sn::Norm::One, L, anorm);
        return 0;
    });
}
template <typename T>
int p_trcon(char norm, char uplo, char diag, int n, const T* a, int ia, int ja, const int* desca, double* rcond) {
    uplo = up(uplo);
    diag = up(diag);
    if (uplo != 'L' && uplo != 'U') return -2;
    if (diag != 'N' && diag != 'U') return -3;
    if (n == 0) { *rcond = 1.0; return 0; }
    return (int)guarded([&]() -> int64_t {
        sn::Matrix<T> A = scal_matrix<T>(desca, n, n, ia, ja, a);
        *rcond = sn::trcondest(cond_norm(norm), uplo == 'L' ? sn::Uplo::Lower : sn::Uplo::Upper,
                               diag == 'U' ? sn::Diag::Unit : sn::Diag::NonUnit, A);
        return 0;
    });
}

// ---- Hermitian eigenproblem (reference lapack_api/lapack_heev.cc,
// lapack_heevd.cc, scalapack_api/scalapack_heev.cc, scalapack_heevd.cc): the
// native two-stage solver behind both the QR-named and the D&C-named entry
// points.  LAPACK-style: jobz = 'V' overwrites A with the eigenvectors (LAPACK
// semantics); ScaLAPACK: the eigenvectors into Z(iz:, jz:), W on every rank.
template <typename T>
sn::HermitianMatrix<T> herm_lower_of(const sn::Matrix<T>& G, char uplo) {
    sn::HermitianMatrix<T> H(sn::Uplo::Lower, G.n(), G.nb(), G.p(), G.q());
    sn::copy(uplo == 'U' ? sn::Op::ConjTrans : sn::Op::NoTrans, G, H);     // the stored triangle as lower
    return H;
}
template <typename T>
int h_heev(char jobz, char uplo, i64 n, T* a, i64 lda, sn::real_t<T>* w) {
    jobz = up(jobz);
    uplo = up(uplo);
    if (jobz != 'N' && jobz != 'V') return -1;
    if (uplo != 'L' && uplo != 'U') return -2;
    if (n < 0) return -3;
    if (lda < std::max<i64>(1, n)) return -5;
    if (n == 0) return 0;
    return (int)guarded([&]() -> int64_t {
        int p, q;
        grid_of(p, q);
        sn::Matrix<T> G(n, n, nb_of(n), p, q);
        G.from_host(a, lda);
        sn::HermitianMatrix<T> H = herm_lower_of(G, uplo);
        std::vector<sn::real_t<T>> lam;
        if (jobz == 'V') {
            sn::Matrix<T> Z(n, n, G.nb(), p, q);
            sn::heev(H, lam, Z);
            Z.to_host(a, lda);
        } else {
            sn::heev(H, lam);
        }
        std::copy(lam.begin(), lam.end(), w);
        return 0;
    });
}
template <typename T>
int p_heev(char jobz, char uplo, int n, const T* a, int ia, int ja, const int* desca, sn::real_t<T>* w, T* z,
           int iz, int jz, const int* descz) {
    jobz = up(jobz);
    uplo = up(uplo);
    if (jobz != 'N' && jobz != 'V') return -1;
    if (uplo != 'L' && uplo != 'U') return -2;
    if (n == 0) return 0;
    return (int)guarded([&]() -> int64_t {
        sn::Matrix<T> G = scal_matrix<T>(desca, n, n, ia, ja, a);
        sn::HermitianMatrix<T> H = herm_lower_of(G, uplo);
        std::vector<sn::real_t<T>> lam;
        if (jobz == 'V') {
            sn::Matrix<T> Z = scal_matrix<T>(descz, n, n, iz, jz, z);
            if (Z.nb() != G.nb() || Z.p() != G.p() || Z.q() != G.q())
                throw sn::Error("native p?heev: Z must have A's block size and grid");
            sn::heev(H, lam, Z);
            scal_back(Z, descz, z);
        } else {
            sn::heev(H, lam);
        }
        std::copy(lam.begin(), lam.end(), w);
        return 0;
    });
}

// ---- SVD (reference lapack_api/lapack_gesvd.cc, scalapack_api/scalapack_gesvd.cc):
// jobu / jobvt 'N' (none), 'V' or 'S' (the min(m, n) singular vectors);
// 'A' (full square factors) only when m == n (LAPACK) and 'O' is not offered
inline bool svd_job(char j, bool& want) {
    j = up(j);
    want = j == 'V' || j == 'S' || j == 'A';
    return j == 'N' || j == 'V' || j == 'S' || j == 'A';
}
template <typename T>
int h_gesvd(char jobu, char jobvt, i64 m, i64 n, T* a, i64 lda, sn::real_t<T>* sv, T* u, i64 ldu, T* vt, i64 ldvt) {
    bool wu = false, wv = false;
    if (!svd_job(jobu, wu)) return -1;
    if (!svd_job(jobvt, wv)) return -2;
    if ((up(jobu) == 'A' && m > n) || (up(jobvt) == 'A' && n > m)) return -1;
    if (m < 0) return -3;
    if (n < 0) return -4;
    if (lda < std::max<i64>(1, m)) return -6;
    const i64 k = std::min(m, n);
    if (wu && ldu < std::max<i64>(1, m)) return -9;
    if (wv && ldvt < std::max<i64>(1, k)) return -11;
    if (k == 0) return 0;
    return (int)guarded([&]() -> int64_t {
        int p, q;
        grid_of(p, q);
        const i64 nb = nb_of(std::max(m, n));
        sn::Matrix<T> A(m, n, nb, p, q);
        A.from_host(a, lda);
        std::vector<sn::real_t<T>> S;
        if (wu || wv) {
            sn::Matrix<T> U(m, k, nb, p, q), VH(k, n, nb, p, q);
            sn::svd(A, S, U, VH);
            if (wu) U.to_host(u, ldu);
            if (wv) VH.to_host(vt, ldvt);
        } else {
            sn::svd(A, S);
        }
        std::copy(S.begin(), S.end(), sv);
        return 0;
    });
}
template <typename T>
int p_gesvd(char jobu, char jobvt, int m, int n, const T* a, int ia, int ja, const int* desca, sn::real_t<T>* sv,
            T* u, int iu, int ju, const int* descu, T* vt, int ivt, int jvt, const int* descvt) {
    bool wu = false, wv = false;
    if (!svd_job(jobu, wu) || up(jobu) == 'A') return -1;
    if (!svd_job(jobvt, wv) || up(jobvt) == 'A') return -2;
    const int k = std::min(m, n);
    if (k == 0) return 0;
    return (int)guarded([&]() -> int64_t {
        sn::Matrix<T> A = scal_matrix<T>(desca, m, n, ia, ja, a);
        std::vector<sn::real_t<T>> S;
        if (wu || wv) {
            sn::Matrix<T> U = wu ? scal_matrix<T>(descu, m, k, iu, ju, u) : sn::Matrix<T>(m, k, A.nb(), A.p(), A.q());
            sn::Matrix<T> VH = wv ? scal_matrix<T>(descvt, k, n, ivt, jvt, vt) : sn::Matrix<T>(k, n, A.nb(), A.p(), A.q());
            if (U.nb() != A.nb() || VH.nb() != A.nb()) throw sn::Error("native p?gesvd: U / VT must have A's block size");
            sn::svd(A, S, U, VH);
            if (wu) scal_back(U, descu, u);
            if (wv) scal_back(VH, descvt, vt);
        } else {
            sn::svd(A, S);
        }
        std::copy(S.begin(), S.end(), sv);
        return 0;
    });
}

extern "C" {

void pdsgesv_(const int* n, const int* nrhs, double* a, const int* ia, const int* ja, const int* desca, int* ipiv,
              const double* b, const int* ib, const int* jb, const int* descb, double* x, const int* ix,
              const int* jx, const int* descx, int* iter, int* info) {
    *info = p_gesv_mixed<double>(*n, *nrhs, a, *ia, *ja, desca, ipiv, b, *ib, *jb, descb, x, *ix, *jx, descx, iter);
}
void pzcgesv_(const int* n, const int* nrhs, std::complex<double>* a, const int* ia, const int* ja,
              const int* desca, int* ipiv, const std::complex<double>* b, const int* ib, const int* jb,
              const int* descb, std::complex<double>* x, const int* ix, const int* jx, const int* descx, int* iter,
              int* info) {
    *info = p_gesv_mixed<std::complex<double>>(*n, *nrhs, a, *ia, *ja, desca, ipiv, b, *ib, *jb, descb, x, *ix, *jx,
                                               descx, iter);
}

const char* slate_amd_last_error(void) { return g_err.c_str(); }
int slate_amd_initialize(void) { return (int)guarded([] { sn::initialize(); return 0; }); }
void slate_amd_finalize(void) { sn::finalize(); }

// ---- LAPACK-style, by value
#define SN_LAPACK(X, T)                                                                                         \
    int slate_##X##potrf(char uplo, int64_t n, T* a, int64_t lda) { return (int)h_potrf<T>(uplo, n, a, lda); }  \
    int slate_##X##potrs(char uplo, int64_t n, int64_t nrhs, const T* a, int64_t lda, T* b, int64_t ldb) {      \
        return (int)h_potrs<T>(uplo, n, nrhs, a, lda, b, ldb);                                                 \
    }                                                                                                          \
    int slate_##X##posv(char uplo, int64_t n, int64_t nrhs, T* a, int64_t lda, T* b, int64_t ldb) {            \
        return (int)h_posv<T>(uplo, n, nrhs, a, lda, b, ldb);                                                  \
    }                                                                                                          \
    int slate_##X##getrf(int64_t m, int64_t n, T* a, int64_t lda, int64_t* ipiv) {                             \
        return (int)h_getrf<T>(m, n, a, lda, ipiv);                                                            \
    }                                                                                                          \
    int slate_##X##getrs(char trans, int64_t n, int64_t nrhs, const T* a, int64_t lda, const int64_t* ipiv,    \
                         T* b, int64_t ldb) {                                                                  \
        return (int)h_getrs<T>(trans, n, nrhs, a, lda, ipiv, b, ldb);                                          \
    }                                                                                                          \
    int slate_##X##gesv(int64_t n, int64_t nrhs, T* a, int64_t lda, int64_t* ipiv, T* b, int64_t ldb) {       \
        return (int)h_gesv<T>(n, nrhs, a, lda, ipiv, b, ldb);                                                  \
    }                                                                                                          \
    int slate_##X##gemm(char ta, char tb, int64_t m, int64_t n, int64_t k, T alpha, const T* a, int64_t lda,   \
                        const T* b, int64_t ldb, T beta, T* c, int64_t ldc) {                                  \
        return (int)h_gemm<T>(ta, tb, m, n, k, alpha, a, lda, b, ldb, beta, c, ldc);                           \
    }                                                                                                          \
    int slate_##X##trsm(char side, char uplo, char ta, char diag, int64_t m, int64_t n, T alpha, const T* a,   \
                        int64_t lda, T* b, int64_t ldb) {                                                      \
        return (int)h_trsm<T>(side, uplo, ta, diag, m, n, alpha, a, lda, b, ldb);                              \
    }                                                                                                          \
    double slate_##X##lange(char norm, int64_t m, int64_t n, const T* a, int64_t lda) {                        \
        return h_lange<T>(norm, m, n, a, lda);                                                                 \
    }                                                                                                          \
    int slate_##X##gels(char trans, int64_t m, int64_t n, int64_t nrhs, T* a, int64_t lda, T* b, int64_t ldb) { \
        return (int)h_gels<T>(trans, m, n, nrhs, a, lda, b, ldb);                                             \
    }                                                                                                          \
    void slate_##X##gels_(const char* trans, const int64_t* m, const int64_t* n, const int64_t* nrhs, T* a,     \
                          const int64_t* lda, T* b, const int64_t* ldb, int64_t* info) {                      \
        *info = h_gels<T>(*trans, *m, *n, *nrhs, a, *lda, b, *ldb);                                            \
    }                                                                                                          \
    void slate_##X##potrf_(const char* uplo, const int64_t* n, T* a, const int64_t* lda, int64_t* info) {      \
        *info = h_potrf<T>(*uplo, *n, a, *lda);                                                                \
    }                                                                                                          \
    void slate_##X##potrs_(const char* uplo, const int64_t* n, const int64_t* nrhs, const T* a,                \
                           const int64_t* lda, T* b, const int64_t* ldb, int64_t* info) {                     \
        *info = h_potrs<T>(*uplo, *n, *nrhs, a, *lda, b, *ldb);                                                \
    }                                                                                                          \
    void slate_##X##posv_(const char* uplo, const int64_t* n, const int64_t* nrhs, T* a, const int64_t* lda,   \
                          T* b, const int64_t* ldb, int64_t* info) {                                          \
        *info = h_posv<T>(*uplo, *n, *nrhs, a, *lda, b, *ldb);                                                 \
    }                                                                                                          \
    void slate_##X##getrf_(const int64_t* m, const int64_t* n, T* a, const int64_t* lda, int64_t* ipiv,        \
                           int64_t* info) {                                                                    \
        *info = h_getrf<T>(*m, *n, a, *lda, ipiv);                                                             \
    }                                                                                                          \
    void slate_##X##getrs_(const char* trans, const int64_t* n, const int64_t* nrhs, const T* a,               \
                           const int64_t* lda, const int64_t* ipiv, T* b, const int64_t* ldb, int64_t* info) { \
        *info = h_getrs<T>(*trans, *n, *nrhs, a, *lda, ipiv, b, *ldb);                                         \
    }                                                                                                          \
    void slate_##X##gesv_(const int64_t* n, const int64_t* nrhs, T* a, const int64_t* lda, int64_t* ipiv,      \
                          T* b, const int64_t* ldb, int64_t* info) {                                          \
        *info = h_gesv<T>(*n, *nrhs, a, *lda, ipiv, b, *ldb);                                                  \
    }                                                                                                          \
    void slate_##X##gemm_(const char* ta, const char* tb, const int64_t* m, const int64_t* n,                  \
                          const int64_t* k, const T* alpha, const T* a, const int64_t* lda, const T* b,        \
                          const int64_t* ldb, const T* beta, T* c, const int64_t* ldc) {                       \
        h_gemm<T>(*ta, *tb, *m, *n, *k, *alpha, a, *lda, b, *ldb, *beta, c, *ldc);                             \
    }                                                                                                          \
    void slate_##X##trsm_(const char* side, const char* uplo, const char* ta, const char* diag,                \
                          const int64_t* m, const int64_t* n, const T* alpha, const T* a, const int64_t* lda,  \
                          T* b, const int64_t* ldb) {                                                          \
        h_trsm<T>(*side, *uplo, *ta, *diag, *m, *n, *alpha, a, *lda, b, *ldb);                                 \
    }                                                                                                          \
    double slate_##X##lange_(const char* norm, const int64_t* m, const int64_t* n, const T* a,                 \
                             const int64_t* lda) {                                                             \
        return h_lange<T>(*norm, *m, *n, a, *lda);                                                             \
    }
SN_LAPACK(s, float)
SN_LAPACK(d, double)
#undef SN_LAPACK

// complex, interleaved (re, im) pairs through pointers to the real type
#define SN_LAPACK_C(X, R)                                                                                       \
    int slate_##X##potrf(char uplo, int64_t n, R* a, int64_t lda) {                                            \
        return (int)h_potrf<std::complex<R>>(uplo, n, reinterpret_cast<std::complex<R>*>(a), lda);            \
    }                                                                                                          \
    int slate_##X##posv(char uplo, int64_t n, int64_t nrhs, R* a, int64_t lda, R* b, int64_t ldb) {            \
        return (int)h_posv<std::complex<R>>(uplo, n, nrhs, reinterpret_cast<std::complex<R>*>(a), lda,        \
                                            reinterpret_cast<std::complex<R>*>(b), ldb);                       \
    }                                                                                                          \
    int slate_##X##getrf(int64_t m, int64_t n, R* a, int64_t lda, int64_t* ipiv) {                             \
        return (int)h_getrf<std::complex<R>>(m, n, reinterpret_cast<std::complex<R>*>(a), lda, ipiv);         \
    }                                                                                                          \
    int slate_##X##gesv(int64_t n, int64_t nrhs, R* a, int64_t lda, int64_t* ipiv, R* b, int64_t ldb) {       \
        return (int)h_gesv<std::complex<R>>(n, nrhs, reinterpret_cast<std::complex<R>*>(a), lda, ipiv,        \
                                            reinterpret_cast<std::complex<R>*>(b), ldb);                       \
    }                                                                                                          \
    int slate_##X##gemm(char ta, char tb, int64_t m, int64_t n, int64_t k, const R* alpha, const R* a,         \
                        int64_t lda, const R* b, int64_t ldb, const R* beta, R* c, int64_t ldc) {              \
        using C = std::complex<R>;                                                                             \
        return (int)h_gemm<C>(ta, tb, m, n, k, C(alpha[0], alpha[1]), reinterpret_cast<const C*>(a), lda,     \
                              reinterpret_cast<const C*>(b), ldb, C(beta[0], beta[1]), reinterpret_cast<C*>(c), \
                              ldc);                                                                            \
    }                                                                                                          \
    double slate_##X##lange(char norm, int64_t m, int64_t n, const R* a, int64_t lda) {                        \
        return h_lange<std::complex<R>>(norm, m, n, reinterpret_cast<const std::complex<R>*>(a), lda);        \
    }                                                                                                          \
    int slate_##X##gels(char trans, int64_t m, int64_t n, int64_t nrhs, R* a, int64_t lda, R* b, int64_t ldb) { \
        return (int)h_gels<std::complex<R>>(trans, m, n, nrhs, reinterpret_cast<std::complex<R>*>(a), lda,    \
                                            reinterpret_cast<std::complex<R>*>(b), ldb);                       \
    }
SN_LAPACK_C(c, float)
SN_LAPACK_C(z, double)
#undef SN_LAPACK_C

// ---- mixed precision, LAPACK names (dsposv, dsgesv, zcposv, zcgesv), by value
int slate_dsposv(char uplo, int64_t n, int64_t nrhs, double* a, int64_t lda, const double* b, int64_t ldb, double* x,
                 int64_t ldx, int* iter) {
    return (int)h_posv_mixed<double>(uplo, n, nrhs, a, lda, b, ldb, x, ldx, iter);
}
int slate_dsgesv(int64_t n, int64_t nrhs, double* a, int64_t lda, int64_t* ipiv, const double* b, int64_t ldb,
                 double* x, int64_t ldx, int* iter) {
    return (int)h_gesv_mixed<double>(n, nrhs, a, lda, ipiv, b, ldb, x, ldx, iter);
}
int slate_zcposv(char uplo, int64_t n, int64_t nrhs, double* a, int64_t lda, const double* b, int64_t ldb,
                 double* x, int64_t ldx, int* iter) {
    using Z = std::complex<double>;
    return (int)h_posv_mixed<Z>(uplo, n, nrhs, reinterpret_cast<Z*>(a), lda, reinterpret_cast<const Z*>(b), ldb,
                                reinterpret_cast<Z*>(x), ldx, iter);
}
int slate_zcgesv(int64_t n, int64_t nrhs, double* a, int64_t lda, int64_t* ipiv, const double* b, int64_t ldb,
                 double* x, int64_t ldx, int* iter) {
    using Z = std::complex<double>;
    return (int)h_gesv_mixed<Z>(n, nrhs, reinterpret_cast<Z*>(a), lda, ipiv, reinterpret_cast<const Z*>(b), ldb,
                                reinterpret_cast<Z*>(x), ldx, iter);
}

// ---- BLACS over the native runtime's ranks
void Cblacs_pinfo(int* mypnum, int* nprocs) {
    sn::initialize();
    *mypnum = sn::rank();
    *nprocs = sn::size();
}
void Cblacs_get(int, int, int* val) { *val = 0; }
void Cblacs_gridinit(int* ctxt, const char* order, int nprow, int npcol) {
    Ctx c;
    c.p = nprow;
    c.q = npcol;
    c.row_major = order && (order[0] == 'R' || order[0] == 'r');
    contexts().push_back(c);
    *ctxt = (int)contexts().size() - 1;
}
void Cblacs_gridinfo(int ctxt, int* nprow, int* npcol, int* myrow, int* mycol) {
    auto& cs = contexts();
    if (ctxt < 0 || ctxt >= (int)cs.size()) { *nprow = *npcol = *myrow = *mycol = -1; return; }
    const Ctx& c = cs[ctxt];
    const int r = sn::rank();
    *nprow = c.p;
    *npcol = c.q;
    if (r >= c.p * c.q) { *myrow = *mycol = -1; return; }
    *myrow = c.row_major ? r / c.q : r % c.p;
    *mycol = c.row_major ? r % c.q : r / c.p;
}
void Cblacs_pcoord(int ctxt, int pnum, int* prow, int* pcol) {
    const Ctx& c = contexts().at(ctxt);
    *prow = c.row_major ? pnum / c.q : pnum % c.p;
    *pcol = c.row_major ? pnum % c.q : pnum / c.p;
}
void Cblacs_gridexit(int) {}
void Cblacs_exit(int) {}
void blacs_pinfo_(int* mypnum, int* nprocs) { Cblacs_pinfo(mypnum, nprocs); }
void blacs_get_(const int* ctxt, const int* what, int* val) { Cblacs_get(*ctxt, *what, val); }
void blacs_gridinit_(int* ctxt, const char* order, const int* nprow, const int* npcol) {
    Cblacs_gridinit(ctxt, order, *nprow, *npcol);
}
void blacs_gridinfo_(const int* ctxt, int* nprow, int* npcol, int* myrow, int* mycol) {
    Cblacs_gridinfo(*ctxt, nprow, npcol, myrow, mycol);
}
void blacs_gridexit_(const int*) {}
void blacs_exit_(const int*) {}

int numroc_(const int* n, const int* nb, const int* iproc, const int* isrcproc, const int* nprocs) {
    const int mydist = (*nprocs + *iproc - *isrcproc) % *nprocs;
    return (int)sn::numroc(*n, *nb, mydist, *nprocs);
}
void descinit_(int* desc, const int* m, const int* n, const int* mb, const int* nb, const int* irsrc,
               const int* icsrc, const int* ictxt, const int* lld, int* info) {
    desc[0] = 1; desc[1] = *ictxt; desc[2] = *m; desc[3] = *n; desc[4] = *mb; desc[5] = *nb;
    desc[6] = *irsrc; desc[7] = *icsrc; desc[8] = *lld;
    *info = (*m < 0) ? -2 : (*n < 0) ? -3 : (*mb < 1) ? -4 : (*nb < 1) ? -5 : 0;
}

// ---- ScaLAPACK (complex arrays as std::complex<R> / interleaved pairs)
#define SN_SCAL(X, T)                                                                                          \
    void p##X##potrf_(const char* uplo, const int* n, T* a, const int* ia, const int* ja, const int* desca,   \
                      int* info) {                                                                         \
        *info = p_potrf<T>(*uplo, *n, a, *ia, *ja, desca);                                                 \
    }                                                                                                      \
    void p##X##potrs_(const char* uplo, const int* n, const int* nrhs, const T* a, const int* ia,             \
                      const int* ja, const int* desca, T* b, const int* ib, const int* jb, const int* descb,  \
                      int* info) {                                                                         \
        *info = p_potrs<T>(*uplo, *n, *nrhs, a, *ia, *ja, desca, b, *ib, *jb, descb);                      \
    }                                                                                                      \
    void p##X##posv_(const char* uplo, const int* n, const int* nrhs, T* a, const int* ia, const int* ja,    \
                     const int* desca, T* b, const int* ib, const int* jb, const int* descb, int* info) {     \
        *info = p_posv<T>(*uplo, *n, *nrhs, a, *ia, *ja, desca, b, *ib, *jb, descb);                       \
    }                                                                                                      \
    void p##X##getrf_(const int* m, const int* n, T* a, const int* ia, const int* ja, const int* desca,      \
                      int* ipiv, int* info) {                                                              \
        *info = p_getrf<T>(*m, *n, a, *ia, *ja, desca, ipiv);                                              \
    }                                                                                                      \
    void p##X##getrs_(const char* trans, const int* n, const int* nrhs, const T* a, const int* ia,           \
                      const int* ja, const int* desca, const int* ipiv, T* b, const int* ib, const int* jb,  \
                      const int* descb, int* info) {                                                       \
        *info = p_getrs<T>(*trans, *n, *nrhs, a, *ia, *ja, desca, ipiv, b, *ib, *jb, descb);               \
    }                                                                                                      \
    void p##X##gesv_(const int* n, const int* nrhs, T* a, const int* ia, const int* ja, const int* desca,    \
                     int* ipiv, T* b, const int* ib, const int* jb, const int* descb, int* info) {            \
        *info = p_gesv<T>(*n, *nrhs, a, *ia, *ja, desca, ipiv, b, *ib, *jb, descb);                        \
    }                                                                                                      \
    void p##X##gemm_(const char* ta, const char* tb, const int* m, const int* n, const int* k, const T* alpha, \
                     const T* a, const int* ia, const int* ja, const int* desca, const T* b, const int* ib,   \
                     const int* jb, const int* descb, const T* beta, T* c, const int* ic, const int* jc,      \
                     const int* descc) {                                                                   \
        p_gemm<T>(*ta, *tb, *m, *n, *k, *alpha, a, *ia, *ja, desca, b, *ib, *jb, descb, *beta, c, *ic, *jc,  \
                  descc);                                                                                  \
    }                                                                                                      \
    void p##X##gels_(const char* t, const int* m, const int* n, const int* nrhs, T* a, const int* ia,        \
                     const int* ja, const int* desca, T* b, const int* ib, const int* jb, const int* descb,   \
                     T* work, const int* lwork, int* info) {                                               \
        *info = p_gels<T>(*t, *m, *n, *nrhs, a, *ia, *ja, desca, b, *ib, *jb, descb, work, *lwork);        \
    }                                                                                                      \
    void p##X##trsm_(const char* side, const char* uplo, const char* ta, const char* diag, const int* m,     \
                     const int* n, const T* alpha, const T* a, const int* ia, const int* ja, const int* desca, \
                     T* b, const int* ib, const int* jb, const int* descb) {                                \
        p_trsm<T>(*side, *uplo, *ta, *diag, *m, *n, *alpha, a, *ia, *ja, desca, b, *ib, *jb, descb);        \
    }
SN_SCAL(s, float)
SN_SCAL(d, double)
SN_SCAL(c, std::complex<float>)
SN_SCAL(z, std::complex<double>)
#undef SN_SCAL

// ---- ScaLAPACK BLAS-3 on triangles / symmetric / Hermitian matrices
#define SN_SCAL3(X, T)                                                                                         \
    void p##X##syrk_(const char* uplo, const char* trans, const int* n, const int* k, const T* alpha,        \
                     const T* a, const int* ia, const int* ja, const int* desca, const T* beta, T* c,          \
                     const int* ic, const int* jc, const int* descc) {                                       \
        p_rank_k<T>(false, false, *uplo, *trans, *n, *k, *alpha, a, *ia, *ja, desca, nullptr, 1, 1, nullptr, \
                    *beta, c, *ic, *jc, descc);                                                            \
    }                                                                                                      \
    void p##X##syr2k_(const char* uplo, const char* trans, const int* n, const int* k, const T* alpha,       \
                      const T* a, const int* ia, const int* ja, const int* desca, const T* b, const int* ib,  \
                      const int* jb, const int* descb, const T* beta, T* c, const int* ic, const int* jc,     \
                      const int* descc) {                                                                  \
        p_rank_k<T>(false, true, *uplo, *trans, *n, *k, *alpha, a, *ia, *ja, desca, b, *ib, *jb, descb,     \
                    *beta, c, *ic, *jc, descc);                                                            \
    }                                                                                                      \
    void p##X##symm_(const char* side, const char* uplo, const int* m, const int* n, const T* alpha,        \
                     const T* a, const int* ia, const int* ja, const int* desca, const T* b, const int* ib,   \
                     const int* jb, const int* descb, const T* beta, T* c, const int* ic, const int* jc,      \
                     const int* descc) {                                                                   \
        p_xmm<T>(false, *side, *uplo, *m, *n, *alpha, a, *ia, *ja, desca, b, *ib, *jb, descb, *beta, c, *ic,  \
                 *jc, descc);                                                                              \
    }                                                                                                      \
    void p##X##trmm_(const char* side, const char* uplo, const char* ta, const char* diag, const int* m,     \
                     const int* n, const T* alpha, const T* a, const int* ia, const int* ja, const int* desca, \
                     T* b, const int* ib, const int* jb, const int* descb) {                                \
        p_trmm<T>(*side, *uplo, *ta, *diag, *m, *n, *alpha, a, *ia, *ja, desca, b, *ib, *jb, descb);        \
    }                                                                                                      \
    void p##X##potri_(const char* uplo, const int* n, T* a, const int* ia, const int* ja, const int* desca,   \
                      int* info) {                                                                         \
        *info = p_potri<T>(*uplo, *n, a, *ia, *ja, desca);                                                 \
    }                                                                                                      \
    void p##X##getri_(const int* n, T* a, const int* ia, const int* ja, const int* desca, const int* ipiv,  \
                      T* work, const int* lwork, int* iwork, const int* liwork, int* info) {                \
        *info = p_getri<T>(*n, a, *ia, *ja, desca, ipiv, work, *lwork, iwork, *liwork);                    \
    }
SN_SCAL3(s, float)
SN_SCAL3(d, double)
SN_SCAL3(c, std::complex<float>)
SN_SCAL3(z, std::complex<double>)
#undef SN_SCAL3
#define SN_SCAL3H(X, T, R)                                                                                     \
    void p##X##herk_(const char* uplo, const char* trans, const int* n, const int* k, const R* alpha,        \
                     const T* a, const int* ia, const int* ja, const int* desca, const R* beta, T* c,          \
                     const int* ic, const int* jc, const int* descc) {                                       \
        p_rank_k<T>(true, false, *uplo, *trans, *n, *k, T(*alpha), a, *ia, *ja, desca, nullptr, 1, 1,       \
                    nullptr, T(*beta), c, *ic, *jc, descc);                                                \
    }                                                                                                      \
    void p##X##her2k_(const char* uplo, const char* trans, const int* n, const int* k, const T* alpha,       \
                      const T* a, const int* ia, const int* ja, const int* desca, const T* b, const int* ib,  \
                      const int* jb, const int* descb, const R* beta, T* c, const int* ic, const int* jc,     \
                      const int* descc) {                                                                  \
        p_rank_k<T>(true, true, *uplo, *trans, *n, *k, *alpha, a, *ia, *ja, desca, b, *ib, *jb, descb,      \
                    T(*beta), c, *ic, *jc, descc);                                                         \
    }                                                                                                      \
    void p##X##hemm_(const char* side, const char* uplo, const int* m, const int* n, const T* alpha,        \
                     const T* a, const int* ia, const int* ja, const int* desca, const T* b, const int* ib,   \
                     const int* jb, const int* descb, const T* beta, T* c, const int* ic, const int* jc,      \
                     const int* descc) {                                                                   \
        p_xmm<T>(true, *side, *uplo, *m, *n, *alpha, a, *ia, *ja, desca, b, *ib, *jb, descb, *beta, c, *ic,   \
                 *jc, descc);                                                                              \
    }
SN_SCAL3H(c, std::complex<float>, float)
SN_SCAL3H(z, std::complex<double>, double)
#undef SN_SCAL3H
float pslange_(const char* norm, const int* m, const int* n, const float* a, const int* ia, const int* ja,
               const int* desca, float*) {
    return (float)p_lange<float>(*norm, *m, *n, a, *ia, *ja, desca);
}
double pdlange_(const char* norm, const int* m, const int* n, const double* a, const int* ia, const int* ja,
                const int* desca, double*) {
    return p_lange<double>(*norm, *m, *n, a, *ia, *ja, desca);
}
float pclange_(const char* norm, const int* m, const int* n, const std::complex<float>* a, const int* ia,
               const int* ja, const int* desca, float*) {
    return (float)p_lange<std::complex<float>>(*norm, *m, *n, a, *ia, *ja, desca);
}
double pzlange_(const char* norm, const int* m, const int* n, const std::complex<double>* a, const int* ia,
                const int* ja, const int* desca, double*) {
    return p_lange<std::complex<double>>(*norm, *m, *n, a, *ia, *ja, desca);
}

// p?geadd_ (sub(C) = beta sub(C) + alpha op(sub(A)); op = N), p?laset_, p?lacpy_ (uplo 'G')
#define SN_AUX(X, T)                                                                                           \
    void p##X##geadd_(const char* trans, const int* m, const int* n, const T* alpha, const T* a, const int* ia, \
                      const int* ja, const int* desca, const T* beta, T* c, const int* ic, const int* jc,     \
                      const int* descc) {                                                                  \
        if (*m == 0 || *n == 0) return;                                                                    \
        const int64_t rc = guarded([&]() -> int64_t {                                                      \
            if (up(*trans) != 'N') throw sn::Error("native p?geadd_: trans = 'N' only");                  \
            sn::Matrix<T> A = scal_matrix<T>(desca, *m, *n, *ia, *ja, a);                                   \
            sn::Matrix<T> C = scal_matrix<T>(descc, *m, *n, *ic, *jc, c);                                   \
            sn::add(*alpha, A, *beta, C);                                                                  \
            scal_back(C, descc, c);                                                                        \
            return 0;                                                                                      \
        });                                                                                                \
        if (rc != 0) std::fprintf(stderr, "slate_amd native p?geadd_: %s\n", g_err.c_str());              \
    }                                                                                                      \
    void p##X##laset_(const char* uplo, const int* m, const int* n, const T* alpha, const T* beta, T* a,     \
                      const int* ia, const int* ja, const int* desca) {                                    \
        if (*m == 0 || *n == 0) return;                                                                    \
        const int64_t rc = guarded([&]() -> int64_t {                                                      \
            if (up(*uplo) != 'G' && up(*uplo) != 'A') throw sn::Error("native p?laset_: uplo = 'G' only"); \
            sn::Matrix<T> A = scal_matrix<T>(desca, *m, *n, *ia, *ja, a);                                   \
            sn::set(*alpha, *beta, A);                                                                     \
            scal_back(A, desca, a);                                                                        \
            return 0;                                                                                      \
        });                                                                                                \
        if (rc != 0) std::fprintf(stderr, "slate_amd native p?laset_: %s\n", g_err.c_str());              \
    }                                                                                                      \
    void p##X##lacpy_(const char* uplo, const int* m, const int* n, const T* a, const int* ia, const int* ja, \
                      const int* desca, T* b, const int* ib, const int* jb, const int* descb) {             \
        if (*m == 0 || *n == 0) return;                                                                    \
        const int64_t rc = guarded([&]() -> int64_t {                                                      \
            if (up(*uplo) != 'G' && up(*uplo) != 'A') throw sn::Error("native p?lacpy_: uplo = 'G' only"); \
            sn::Matrix<T> A = scal_matrix<T>(desca, *m, *n, *ia, *ja, a);                                   \
            sn::Matrix<T> B = scal_matrix<T>(descb, *m, *n, *ib, *jb, b);                                   \
            sn::copy(sn::Op::NoTrans, A, B);                                                               \
            scal_back(B, descb, b);                                                                        \
            return 0;                                                                                      \
        });                                                                                                \
        if (rc != 0) std::fprintf(stderr, "slate_amd native p?lacpy_: %s\n", g_err.c_str());              \
    }
SN_AUX(s, float)
SN_AUX(d, double)
SN_AUX(c, std::complex<float>)
SN_AUX(z, std::complex<double>)
#undef SN_AUX

#define SN_LAN(X, T, R)                                                                                        \
    R p##X##lansy_(const char* norm, const char* uplo, const int* n, const T* a, const int* ia, const int* ja, \
                   const int* desca, R*) {                                                                   \
        return (R)p_lan_struct<T>(2, *norm, *uplo, 'N', *n, a, *ia, *ja, desca);                            \
    }                                                                                                        \
    R p##X##lantr_(const char* norm, const char* uplo, const char* diag, const int* m, const int* n,          \
                   const T* a, const int* ia, const int* ja, const int* desca, R*) {                         \
        if (*m != *n) {                                                                                      \
            g_err = "native p?lantr_: square matrices only";                                                 \
            return (R)-1;                                                                                    \
        }                                                                                                    \
        return (R)p_lan_struct<T>(0, *norm, *uplo, *diag, *n, a, *ia, *ja, desca);                          \
    }
SN_LAN(s, float, float)
SN_LAN(d, double, double)
SN_LAN(c, std::complex<float>, float)
SN_LAN(z, std::complex<double>, double)
#undef SN_LAN
float pclanhe_(const char* norm, const char* uplo, const int* n, const std::complex<float>* a, const int* ia,
               const int* ja, const int* desca, float*) {
    return (float)p_lan_struct<std::complex<float>>(1, *norm, *uplo, 'N', *n, a, *ia, *ja, desca);
}
double pzlanhe_(const char* norm, const char* uplo, const int* n, const std::complex<double>* a, const int* ia,
                const int* ja, const int* desca, double*) {
    return p_lan_struct<std::complex<double>>(1, *norm, *uplo, 'N', *n, a, *ia, *ja, desca);
}

// ---- earlier native entry points (kept)
const char* slate_native_last_error(void) { return g_err.c_str(); }
int slate_native_initialize(void) { return slate_amd_initialize(); }
void slate_native_finalize(void) { sn::finalize(); }
int slate_native_dpotrf(char uplo, int64_t n, double* a, int64_t lda) { return (int)h_potrf<double>(uplo, n, a, lda); }
int slate_native_dgetrf(int64_t m, int64_t n, double* a, int64_t lda, int64_t* ipiv) {
    return (int)h_getrf<double>(m, n, a, lda, ipiv);
}
int slate_native_dgesv(int64_t n, int64_t nrhs, double* a, int64_t lda, int64_t* ipiv, double* b, int64_t ldb) {
    return (int)h_gesv<double>(n, nrhs, a, lda, ipiv, b, ldb);
}
int slate_native_dposv(char uplo, int64_t n, int64_t nrhs, double* a, int64_t lda, double* b, int64_t ldb) {
    return (int)h_posv<double>(uplo, n, nrhs, a, lda, b, ldb);
}
int slate_native_dgemm(int64_t m, int64_t n, int64_t k, double alpha, const double* a, int64_t lda, const double* b,
                       int64_t ldb, double beta, double* c, int64_t ldc) {
    return (int)h_gemm<double>('N', 'N', m, n, k, alpha, a, lda, b, ldb, beta, c, ldc);
}
double slate_native_dlange(char norm, int64_t m, int64_t n, const double* a, int64_t lda) {
    return h_lange<double>(norm, m, n, a, lda);
}

// ---- condition estimates: LAPACK-style (host arrays, reference
// lapack_api/lapack_gecon.cc: slate_?gecon etc.) and ScaLAPACK
#define SN_COND(X, T, R)                                                                                        \
    void slate_##X##gecon_(const char* norm, const int64_t* n, const T* a, const int64_t* lda, const R* anorm,  \
                           R* rcond, T* work, int64_t* iwork, int64_t* info) {                                  \
        (void)work; (void)iwork;                                                                                \
        double rc = 0;                                                                                          \
        *info = h_gecon<T>(*norm, *n, a, *lda, (double)*anorm, &rc);                                            \
        *rcond = (R)rc;                                                                                         \
    }                                                                                                           \
    void slate_##X##pocon_(const char* uplo, const int64_t* n, const T* a, const int64_t* lda, const R* anorm,  \
                           R* rcond, T* work, int64_t* iwork, int64_t* info) {                                  \
        (void)work; (void)iwork;                                                                                \
        double rc = 0;                                                                                          \
        *info = h_pocon<T>(*uplo, *n, a, *lda, (double)*anorm, &rc);                                            \
        *rcond = (R)rc;                                                                                         \
    }                                                                                                           \
    void slate_##X##trcon_(const char* norm, const char* uplo, const char* diag, const int64_t* n, const T* a,  \
                           const int64_t* lda, R* rcond, T* work, int64_t* iwork, int64_t* info) {             \
        (void)work; (void)iwork;                                                                                \
        double rc = 0;                                                                                          \
        *info = h_trcon<T>(*norm, *uplo, *diag, *n, a, *lda, &rc);                                              \
        *rcond = (R)rc;                                                                                         \
    }                                                                                                           \
    void p##X##gecon_(const char* norm, const int* n, const T* a, const int* ia, const int* ja,                 \
                      const int* desca, const R* anorm, R* rcond, T* work, const int* lwork, void* iwork,       \
                      const int* liwork, int* info) {                                                           \
        if ((lwork && *lwork == -1) || (liwork && *liwork == -1)) {                                            \
            if (work) work[0] = T(1);                                                                           \
            *info = 0;                                                                                          \
            return;                                                                                             \
        }                                                                                                       \
        double rc = 0;                                                                                          \
        *info = p_gecon<T>(*norm, *n, a, *ia, *ja, desca, (double)*anorm, &rc);                                 \
        *rcond = (R)rc;                                                                                         \
    }                                                                                                           \
    void p##X##pocon_(const char* uplo, const int* n, const T* a, const int* ia, const int* ja,                 \
                      const int* desca, const R* anorm, R* rcond, T* work, const int* lwork, void* iwork,       \
                      const int* liwork, int* info) {                                                           \
        if ((lwork && *lwork == -1) || (liwork && *liwork == -1)) {                                            \
            if (work) work[0] = T(1);                                                                           \
            *info = 0;                                                                                          \
            return;                                                                                             \
        }                                                                                                       \
        double rc = 0;                                                                                          \
        *info = p_pocon<T>(*uplo, *n, a, *ia, *ja, desca, (double)*anorm, &rc);                                 \
        *rcond = (R)rc;                                                                                         \
    }                                                                                                           \
    void p##X##trcon_(const char* norm, const char* uplo, const char* diag, const int* n, const T* a,           \
                      const int* ia, const int* ja, const int* desca, R* rcond, T* work, const int* lwork,     \
                      void* iwork, const int* liwork, int* info) {                                              \
        if ((lwork && *lwork == -1) || (liwork && *liwork == -1)) {                                            \
            if (work) work[0] = T(1);                                                                           \
            *info = 0;                                                                                          \
            return;                                                                                             \
        }                                                                                                       \
        double rc = 0;                                                                                          \
        *info = p_trcon<T>(*norm, *uplo, *diag, *n, a, *ia, *ja, desca, &rc);                                   \
        *rcond = (R)rc;                                                                                         \
    }
// ---- eigenproblem exports: LAPACK-style (reference names slate_?syev /
// ?heev / ?syevd / ?heevd, by reference) and ScaLAPACK p?syev(d)_ / p?heev(d)_
#define SN_EIG_R(X, T)                                                                                          \
    void slate_##X##syev(const char* jobz, const char* uplo, const int* n, T* a, const int* lda, T* w, T* work,  \
                         const int* lwork, int* info) {                                                         \
        if (*lwork == -1) { work[0] = T(1); *info = 0; return; }                                                \
        *info = h_heev<T>(*jobz, *uplo, *n, a, *lda, w);                                                        \
    }                                                                                                           \
    void slate_##X##syevd(const char* jobz, const char* uplo, const int* n, T* a, const int* lda, T* w, T* work, \
                          const int* lwork, int* iwork, const int* liwork, int* info) {                         \
        if (*lwork == -1 || *liwork == -1) { work[0] = T(1); iwork[0] = 1; *info = 0; return; }                 \
        *info = h_heev<T>(*jobz, *uplo, *n, a, *lda, w);                                                        \
    }                                                                                                           \
    void p##X##syev_(const char* jobz, const char* uplo, const int* n, const T* a, const int* ia, const int* ja, \
                     const int* desca, T* w, T* z, const int* iz, const int* jz, const int* descz, T* work,     \
                     const int* lwork, int* info) {                                                             \
        if (*lwork == -1) { work[0] = T(1); *info = 0; return; }                                                \
        *info = p_heev<T>(*jobz, *uplo, *n, a, *ia, *ja, desca, w, z, *iz, *jz, descz);                         \
    }                                                                                                           \
    void p##X##syevd_(const char* jobz, const char* uplo, const int* n, const T* a, const int* ia,             \
                      const int* ja, const int* desca, T* w, T* z, const int* iz, const int* jz,                \
                      const int* descz, T* work, const int* lwork, int* iwork, const int* liwork, int* info) {   \
        if (*lwork == -1 || *liwork == -1) { work[0] = T(1); iwork[0] = 1; *info = 0; return; }                 \
        *info = p_heev<T>(*jobz, *uplo, *n, a, *ia, *ja, desca, w, z, *iz, *jz, descz);                         \
    }
#define SN_EIG_C(X, T, R)                                                                                       \
    void slate_##X##heev(const char* jobz, const char* uplo, const int* n, T* a, const int* lda, R* w, T* work,  \
                         const int* lwork, R* rwork, int* info) {                                               \
        (void)rwork;                                                                                            \
        if (*lwork == -1) { work[0] = T(1); *info = 0; return; }                                                \
        *info = h_heev<T>(*jobz, *uplo, *n, a, *lda, w);                                                        \
    }                                                                                                           \
    void slate_##X##heevd(const char* jobz, const char* uplo, const int* n, T* a, const int* lda, R* w, T* work, \
                          const int* lwork, R* rwork, const int* lrwork, int* iwork, const int* liwork,         \
                          int* info) {                                                                          \
        if (*lwork == -1 || *lrwork == -1 || *liwork == -1) {                                                   \
            work[0] = T(1); rwork[0] = R(1); iwork[0] = 1; *info = 0; return;                                   \
        }                                                                                                       \
        *info = h_heev<T>(*jobz, *uplo, *n, a, *lda, w);                                                        \
    }                                                                                                           \
    void p##X##heev_(const char* jobz, const char* uplo, const int* n, const T* a, const int* ia, const int* ja, \
                     const int* desca, R* w, T* z, const int* iz, const int* jz, const int* descz, T* work,     \
                     const int* lwork, R* rwork, const int* lrwork, int* info) {                                \
        if (*lwork == -1 || *lrwork == -1) { work[0] = T(1); rwork[0] = R(1); *info = 0; return; }              \
        *info = p_heev<T>(*jobz, *uplo, *n, a, *ia, *ja, desca, w, z, *iz, *jz, descz);                         \
    }                                                                                                           \
    void p##X##heevd_(const char* jobz, const char* uplo, const int* n, const T* a, const int* ia,             \
                      const int* ja, const int* desca, R* w, T* z, const int* iz, const int* jz,                \
                      const int* descz, T* work, const int* lwork, R* rwork, const int* lrwork, int* iwork,     \
                      const int* liwork, int* info) {                                                           \
        if (*lwork == -1 || *lrwork == -1 || *liwork == -1) {                                                   \
            work[0] = T(1); rwork[0] = R(1); iwork[0] = 1; *info = 0; return;                                   \
        }                                                                                                       \
        *info = p_heev<T>(*jobz, *uplo, *n, a, *ia, *ja, desca, w, z, *iz, *jz, descz);                         \
    }
#define SN_SVD_R(X, T)                                                                                          \
    void slate_##X##gesvd(const char* jobu, const char* jobvt, const int* m, const int* n, T* a, const int* lda,   \
                          T* s, T* u, const int* ldu, T* vt, const int* ldvt, T* work, const int* lwork, int* info) { \
        if (*lwork == -1) { work[0] = T(1); *info = 0; return; }                                                \
        *info = h_gesvd<T>(*jobu, *jobvt, *m, *n, a, *lda, s, u, *ldu, vt, *ldvt);                              \
    }                                                                                                           \
    void p##X##gesvd_(const char* jobu, const char* jobvt, const int* m, const int* n, const T* a, const int* ia, \
                      const int* ja, const int* desca, T* s, T* u, const int* iu, const int* ju, const int* descu, \
                      T* vt, const int* ivt, const int* jvt, const int* descvt, T* work, const int* lwork,       \
                      int* info) {                                                                              \
        if (*lwork == -1) { work[0] = T(1); *info = 0; return; }                                                \
        *info = p_gesvd<T>(*jobu, *jobvt, *m, *n, a, *ia, *ja, desca, s, u, *iu, *ju, descu, vt, *ivt, *jvt,     \
                           descvt);                                                                             \
    }
#define SN_SVD_C(X, T, R)                                                                                       \
    void slate_##X##gesvd(const char* jobu, const char* jobvt, const int* m, const int* n, T* a, const int* lda,   \
                          R* s, T* u, const int* ldu, T* vt, const int* ldvt, T* work, const int* lwork, R* rwork, \
                          int* info) {                                                                          \
        (void)rwork;                                                                                            \
        if (*lwork == -1) { work[0] = T(1); *info = 0; return; }                                                \
        *info = h_gesvd<T>(*jobu, *jobvt, *m, *n, a, *lda, s, u, *ldu, vt, *ldvt);                              \
    }                                                                                                           \
    void p##X##gesvd_(const char* jobu, const char* jobvt, const int* m, const int* n, const T* a, const int* ia, \
                      const int* ja, const int* desca, R* s, T* u, const int* iu, const int* ju, const int* descu, \
                      T* vt, const int* ivt, const int* jvt, const int* descvt, T* work, const int* lwork,       \
                      R* rwork, int* info) {                                                                    \
        (void)rwork;                                                                                            \
        if (*lwork == -1) { work[0] = T(1); *info = 0; return; }                                                \
        *info = p_gesvd<T>(*jobu, *jobvt, *m, *n, a, *ia, *ja, desca, s, u, *iu, *ju, descu, vt, *ivt, *jvt,     \
                           descvt);                                                                             \
    }
SN_SVD_R(s, float)
SN_SVD_R(d, double)
SN_SVD_C(c, std::complex<float>, float)
SN_SVD_C(z, std::complex<double>, double)
#undef SN_SVD_R
#undef SN_SVD_C

SN_EIG_R(s, float)
SN_EIG_R(d, double)
SN_EIG_C(c, std::complex<float>, float)
SN_EIG_C(z, std::complex<double>, double)
#undef SN_EIG_R
#undef SN_EIG_C

SN_COND(s, float, float)
SN_COND(d, double, double)
SN_COND(c, std::complex<float>, float)
SN_COND(z, std::complex<double>, double)
#undef SN_COND

}  // extern "C"
