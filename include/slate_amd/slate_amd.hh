// slate_amd C++ API: distributed tiled matrices and the dense linear algebra
// routines on them, for C++ applications (SLATE's public C++ interface,
// include/slate/slate.hh:41-1367 and the matrix classes of
// include/slate/Matrix.hh / HermitianMatrix.hh / TriangularMatrix.hh).
//
// Header-only, over the handle C API of c_api.h: link -lslate_amd_native
// (the Python-free native library, csrc/native/capi_handles.hip; the
// CPython-backed -lslate_amd_c is deprecated).  One
// process per GPU; the p x q grid spans every rank started with RANK /
// WORLD_SIZE / MASTER_ADDR / MASTER_PORT (torchrun convention).  A matrix
// object owns a handle; sub-matrix and transposed views share the parent's
// storage (its tiles live on the rank's GPU, 2D block-cyclic, nb x nb).
//
//   slate_amd::Matrix<double> A(n, n, nb, p, q);
//   A.generate(slate_amd::Gen::Random, 7);
//   slate_amd::Pivots piv;
//   int64_t info = slate_amd::gesv(A, piv, B);
//
// Errors of the runtime throw slate_amd::Exception (message from
// slate_amd_last_error()); numerical failures are returned as LAPACK info.
#ifndef SLATE_AMD_HH
#define SLATE_AMD_HH

#include <complex>
#include <cstdint>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "c_api.h"

namespace slate_amd {

class Exception : public std::runtime_error {
public:
    explicit Exception(const std::string& what) : std::runtime_error(what) {}
};

namespace detail {
inline bool failed(double v) { return v <= SLATE_AMD_ERR_INTERNAL + 0.5 && v >= SLATE_AMD_ERR_INIT - 0.5; }
inline int64_t check(int64_t v, const char* where) {
    if (v == SLATE_AMD_ERR_INTERNAL || v == SLATE_AMD_ERR_INIT) {
        const char* e = slate_amd_last_error();
        throw Exception(std::string(where) + ": " + (e ? e : "runtime error"));
    }
    return v;
}
inline double checkd(double v, const char* where) {
    if (failed(v)) check((int64_t)v, where);
    return v;
}
template <typename T> struct code;
template <> struct code<float> { static constexpr char value = 's'; };
template <> struct code<double> { static constexpr char value = 'd'; };
template <> struct code<std::complex<float>> { static constexpr char value = 'c'; };
template <> struct code<std::complex<double>> { static constexpr char value = 'z'; };
}  // namespace detail

enum class Uplo : char { Lower = 'L', Upper = 'U' };
enum class Diag : char { NonUnit = 'N', Unit = 'U' };
enum class Side : char { Left = 'L', Right = 'R' };
enum class Op : char { NoTrans = 'N', Trans = 'T', ConjTrans = 'C' };
enum class Norm : char { One = '1', Inf = 'I', Fro = 'F', Max = 'M' };
enum class Gen : int { Random = 0, HermitianPositiveDefinite = 1, Normal = 2 };

// Library-wide options (SLATE's Options map), e.g.
// set_option("Lookahead", "2"), set_option("MethodLU", "CALU").
inline void set_option(const std::string& name, const std::string& value) {
    detail::check(slate_amd_set_option(name.c_str(), value.c_str()), "set_option");
}
inline void clear_options() { detail::check(slate_amd_clear_options(), "clear_options"); }
inline void finalize() { slate_amd_finalize(); }

// Move-only owner of one handle of the C API.
class Handle {
public:
    Handle() = default;
    explicit Handle(int64_t h, const char* where) : h_(detail::check(h, where)) {}
    Handle(Handle&& o) noexcept : h_(std::exchange(o.h_, 0)) {}
    Handle& operator=(Handle&& o) noexcept {
        if (this != &o) { reset(); h_ = std::exchange(o.h_, 0); }
        return *this;
    }
    Handle(const Handle&) = delete;
    Handle& operator=(const Handle&) = delete;
    ~Handle() { reset(); }
    int64_t get() const { return h_; }
    explicit operator bool() const { return h_ != 0; }

private:
    void reset() {
        if (h_) slate_amd_matrix_destroy(h_);
        h_ = 0;
    }
    int64_t h_ = 0;
};

class Pivots {
public:
    Pivots() : h_(slate_amd_pivots_create(), "Pivots") {}
    int64_t handle() const { return h_.get(); }

private:
    Handle h_;
};

class TriangularFactors {
public:
    TriangularFactors() : h_(slate_amd_tfactors_create(), "TriangularFactors") {}
    int64_t handle() const { return h_.get(); }

private:
    Handle h_;
};

// Base of the typed matrices: a handle plus its global shape.
template <typename T>
class BaseMatrix {
public:
    using value_type = T;
    int64_t handle() const { return h_.get(); }
    int64_t m() const { int64_t a, b; detail::check(slate_amd_matrix_dims(handle(), &a, &b), "m"); return a; }
    int64_t n() const { int64_t a, b; detail::check(slate_amd_matrix_dims(handle(), &a, &b), "n"); return b; }
    int64_t mt() const { int64_t a, b; detail::check(slate_amd_matrix_tiles(handle(), &a, &b), "mt"); return a; }
    int64_t nt() const { int64_t a, b; detail::check(slate_amd_matrix_tiles(handle(), &a, &b), "nt"); return b; }
    // This rank's local block (ScaLAPACK layout: column-major mloc x nloc).
    std::pair<int64_t, int64_t> local_size() const {
        int64_t a = 0, b = 0;
        detail::check(slate_amd_matrix_local_size(handle(), &a, &b), "local_size");
        return {a, b};
    }
    std::vector<T> get_local() const {
        auto [ml, nl] = local_size();
        std::vector<T> v((size_t)(ml * nl));
        if (!v.empty()) detail::check(slate_amd_matrix_get_local(handle(), v.data(), ml), "get_local");
        return v;
    }
    void set_local(const std::vector<T>& v) {
        auto [ml, nl] = local_size();
        if ((int64_t)v.size() != ml * nl) throw Exception("set_local: size mismatch");
        if (!v.empty()) detail::check(slate_amd_matrix_set_local(handle(), v.data(), ml), "set_local");
    }
    void generate(Gen kind, int64_t seed) {
        detail::check(slate_amd_matrix_generate(handle(), (int)kind, seed), "generate");
    }

protected:
    BaseMatrix() = default;
    explicit BaseMatrix(Handle&& h) : h_(std::move(h)) {}
    Handle h_;
};

template <typename T>
class Matrix : public BaseMatrix<T> {
public:
    Matrix() = default;
    // m x n general matrix, nb x nb tiles, p x q grid (2D block-cyclic)
    Matrix(int64_t m, int64_t n, int64_t nb, int p, int q)
        : BaseMatrix<T>(Handle(slate_amd_matrix_create('G', detail::code<T>::value, m, n, nb, p, q), "Matrix")) {}
    // tiles [i1, i2] x [j1, j2], sharing storage (slate::Matrix::sub)
    Matrix sub(int64_t i1, int64_t i2, int64_t j1, int64_t j2) const {
        return Matrix(Handle(slate_amd_matrix_sub(this->handle(), i1, i2, j1, j2), "sub"));
    }
    // adopt a handle of the C API (views made by slate_amd_matrix_sub/_op)
    explicit Matrix(Handle&& h) : BaseMatrix<T>(std::move(h)) {}
};

// SLATE's transpose(A) / conj_transpose(A): views, no data movement
template <typename T>
Matrix<T> transpose(const Matrix<T>& A) { return Matrix<T>(Handle(slate_amd_matrix_op(A.handle(), 'T'), "transpose")); }
template <typename T>
Matrix<T> conj_transpose(const Matrix<T>& A) {
    return Matrix<T>(Handle(slate_amd_matrix_op(A.handle(), 'C'), "conj_transpose"));
}

template <typename T>
class HermitianMatrix : public BaseMatrix<T> {
public:
    HermitianMatrix() = default;
    HermitianMatrix(Uplo uplo, int64_t n, int64_t nb, int p, int q)
        : BaseMatrix<T>(Handle(slate_amd_matrix_create((char)uplo, detail::code<T>::value, n, n, nb, p, q),
                               "HermitianMatrix")), uplo_(uplo) {}
    Uplo uplo() const { return uplo_; }

private:
    Uplo uplo_ = Uplo::Lower;
};
template <typename T> using SymmetricMatrix = HermitianMatrix<T>;

// Triangular view (uplo, diag) of a general or Hermitian matrix's storage.
template <typename T>
struct TriangularView {
    Uplo uplo;
    Diag diag;
    const BaseMatrix<T>& A;
};
template <typename T>
TriangularView<T> triangular(Uplo uplo, Diag diag, const BaseMatrix<T>& A) { return {uplo, diag, A}; }

// ------------------------------------------------------------- BLAS-3
template <typename T>
void gemm(double alpha, const BaseMatrix<T>& A, const BaseMatrix<T>& B, double beta, BaseMatrix<T>& C) {
    detail::check(slate_amd_gemm(alpha, A.handle(), B.handle(), beta, C.handle()), "gemm");
}
template <typename T>
void trsm(Side side, double alpha, TriangularView<T> A, BaseMatrix<T>& B) {
    detail::check(slate_amd_trsm((char)side, (char)A.uplo, (char)A.diag, alpha, A.A.handle(), B.handle()), "trsm");
}
template <typename T>
void trmm(Side side, double alpha, TriangularView<T> A, BaseMatrix<T>& B) {
    detail::check(slate_amd_trmm((char)side, (char)A.uplo, (char)A.diag, alpha, A.A.handle(), B.handle()), "trmm");
}
template <typename T>
void herk(double alpha, const BaseMatrix<T>& A, double beta, HermitianMatrix<T>& C) {
    detail::check(slate_amd_herk(alpha, A.handle(), beta, C.handle()), "herk");
}
template <typename T>
void her2k(double alpha, const BaseMatrix<T>& A, const BaseMatrix<T>& B, double beta, HermitianMatrix<T>& C) {
    detail::check(slate_amd_her2k(alpha, A.handle(), B.handle(), beta, C.handle()), "her2k");
}
template <typename T>
void hemm(Side side, double alpha, const HermitianMatrix<T>& A, const BaseMatrix<T>& B, double beta,
          BaseMatrix<T>& C) {
    detail::check(slate_amd_hemm((char)side, alpha, A.handle(), B.handle(), beta, C.handle()), "hemm");
}
template <typename T>
void syrk(double alpha, const BaseMatrix<T>& A, double beta, HermitianMatrix<T>& C) { herk(alpha, A, beta, C); }

// ------------------------------------------------------------- Cholesky
template <typename T> int64_t potrf(HermitianMatrix<T>& A) { return detail::check(slate_amd_potrf(A.handle()), "potrf"); }
template <typename T> void potrs(const HermitianMatrix<T>& A, BaseMatrix<T>& B) {
    detail::check(slate_amd_potrs(A.handle(), B.handle()), "potrs");
}
template <typename T> int64_t posv(HermitianMatrix<T>& A, BaseMatrix<T>& B) {
    return detail::check(slate_amd_posv(A.handle(), B.handle()), "posv");
}
template <typename T> int64_t potri(HermitianMatrix<T>& A) { return detail::check(slate_amd_potri(A.handle()), "potri"); }
template <typename T> int64_t trtri(TriangularView<T> A) {
    return detail::check(slate_amd_trtri((char)A.uplo, (char)A.diag, A.A.handle()), "trtri");
}
template <typename T>
int64_t posv_mixed(HermitianMatrix<T>& A, BaseMatrix<T>& B, BaseMatrix<T>& X, int64_t* iter = nullptr) {
    int64_t it = 0;
    const int64_t info = detail::check(slate_amd_posv_mixed(A.handle(), B.handle(), X.handle(), &it), "posv_mixed");
    if (iter) *iter = it;
    return info;
}

// ------------------------------------------------------------- LU
template <typename T> int64_t getrf(Matrix<T>& A, Pivots& piv) {
    return detail::check(slate_amd_getrf(A.handle(), piv.handle()), "getrf");
}
template <typename T> void getrs(const Matrix<T>& A, const Pivots& piv, BaseMatrix<T>& B) {
    detail::check(slate_amd_getrs(A.handle(), piv.handle(), B.handle()), "getrs");
}
template <typename T> int64_t gesv(Matrix<T>& A, Pivots& piv, BaseMatrix<T>& B) {
    return detail::check(slate_amd_gesv(A.handle(), piv.handle(), B.handle()), "gesv");
}
template <typename T> int64_t getri(Matrix<T>& A, const Pivots& piv) {
    return detail::check(slate_amd_getri(A.handle(), piv.handle()), "getri");
}
template <typename T> int64_t gesv_nopiv(Matrix<T>& A, BaseMatrix<T>& B) {
    return detail::check(slate_amd_gesv_nopiv(A.handle(), B.handle()), "gesv_nopiv");
}
template <typename T> int64_t gesv_rbt(Matrix<T>& A, BaseMatrix<T>& B) {
    return detail::check(slate_amd_gesv_rbt(A.handle(), B.handle()), "gesv_rbt");
}
template <typename T>
int64_t gesv_mixed(Matrix<T>& A, Pivots& piv, BaseMatrix<T>& B, BaseMatrix<T>& X, int64_t* iter = nullptr) {
    int64_t it = 0;
    const int64_t info =
        detail::check(slate_amd_gesv_mixed(A.handle(), piv.handle(), B.handle(), X.handle(), &it), "gesv_mixed");
    if (iter) *iter = it;
    return info;
}
template <typename T>
int64_t gesv_mixed_gmres(Matrix<T>& A, Pivots& piv, BaseMatrix<T>& B, BaseMatrix<T>& X, int64_t* iter = nullptr) {
    int64_t it = 0;
    const int64_t info = detail::check(
        slate_amd_gesv_mixed_gmres(A.handle(), piv.handle(), B.handle(), X.handle(), &it), "gesv_mixed_gmres");
    if (iter) *iter = it;
    return info;
}

// ------------------------------------------------------------- indefinite
template <typename T> int64_t hesv(HermitianMatrix<T>& A, BaseMatrix<T>& B) {
    return detail::check(slate_amd_hesv(A.handle(), B.handle()), "hesv");
}

// ------------------------------------------------------------- QR / LQ
template <typename T> int64_t geqrf(Matrix<T>& A, TriangularFactors& T_) {
    return detail::check(slate_amd_geqrf(A.handle(), T_.handle()), "geqrf");
}
template <typename T> int64_t gelqf(Matrix<T>& A, TriangularFactors& T_) {
    return detail::check(slate_amd_gelqf(A.handle(), T_.handle()), "gelqf");
}
template <typename T>
void unmqr(Side side, Op op, const Matrix<T>& A, const TriangularFactors& T_, BaseMatrix<T>& C) {
    detail::check(slate_amd_unmqr((char)side, (char)op, A.handle(), T_.handle(), C.handle()), "unmqr");
}
template <typename T>
void unmlq(Side side, Op op, const Matrix<T>& A, const TriangularFactors& T_, BaseMatrix<T>& C) {
    detail::check(slate_amd_unmlq((char)side, (char)op, A.handle(), T_.handle(), C.handle()), "unmlq");
}
template <typename T> int64_t gels(Matrix<T>& A, TriangularFactors& T_, BaseMatrix<T>& BX) {
    return detail::check(slate_amd_gels_t(A.handle(), T_.handle(), BX.handle()), "gels");
}

// ------------------------------------------------------------- spectra
template <typename T>
std::vector<double> heev(HermitianMatrix<T>& A, Matrix<T>* Z = nullptr) {
    std::vector<double> w((size_t)A.n());
    detail::check(slate_amd_heev(A.handle(), w.data(), Z ? Z->handle() : 0), "heev");
    return w;
}
template <typename T>
std::vector<double> hegv(int64_t itype, HermitianMatrix<T>& A, HermitianMatrix<T>& B, Matrix<T>* Z = nullptr) {
    std::vector<double> w((size_t)A.n());
    detail::check(slate_amd_hegv(itype, A.handle(), B.handle(), w.data(), Z ? Z->handle() : 0), "hegv");
    return w;
}
template <typename T>
std::vector<double> svd_vals(Matrix<T>& A) {
    const int64_t k = std::min(A.m(), A.n());
    std::vector<double> s((size_t)k);
    detail::check(slate_amd_svd_vals(A.handle(), s.data()), "svd_vals");
    return s;
}

// ------------------------------------------------------------- auxiliary
template <typename T> double norm(Norm nrm, const BaseMatrix<T>& A) {
    return detail::checkd(slate_amd_norm((char)nrm, A.handle()), "norm");
}
template <typename T> void add(double alpha, const BaseMatrix<T>& A, double beta, BaseMatrix<T>& B) {
    detail::check(slate_amd_add(alpha, A.handle(), beta, B.handle()), "add");
}
template <typename T> void copy(const BaseMatrix<T>& A, BaseMatrix<T>& B) {
    detail::check(slate_amd_copy(A.handle(), B.handle()), "copy");
}
template <typename T> void scale(double numer, double denom, BaseMatrix<T>& A) {
    detail::check(slate_amd_scale(numer, denom, A.handle()), "scale");
}
template <typename T> void set(double offdiag, double diag, BaseMatrix<T>& A) {
    detail::check(slate_amd_set(offdiag, diag, A.handle()), "set");
}
template <typename T> double gecondest(Norm nrm, const Matrix<T>& A, const Pivots& piv, double anorm) {
    return detail::checkd(slate_amd_gecondest((char)nrm, A.handle(), piv.handle(), anorm), "gecondest");
}
template <typename T> double pocondest(Norm nrm, const HermitianMatrix<T>& A, double anorm) {
    return detail::checkd(slate_amd_pocondest((char)nrm, A.handle(), anorm), "pocondest");
}

}  // namespace slate_amd

#endif
