// Native handle-based C API (include/slate_amd/c_api.h, "Distributed
// matrices by opaque handle"): slate_amd_matrix_create / _potrf / _gemm /
// ... over the native C++ drivers of libslate_amd_native.so -- no Python
// runtime.  Reference: src/c_api/wrappers.cc:13-456 (SLATE's generated
// slate_Matrix_create_* / slate_<routine>_c<type> bindings over the C++
// templates) and include/slate/c_api/*.h.
//
// A handle is an int64 id in a process-local registry.  A matrix handle
// owns (shares) a native Matrix<T> of one of the four element types plus its
// kind ('G' general, 'L' / 'U' Hermitian with that stored triangle) and an
// op flag ('N', or 'T' / 'C' for the transposed views of
// slate_amd_matrix_op, which share the parent's storage).  Operands that a
// driver takes as op(A) directly (gemm, copy, trsm, trmm, herk, her2k) use
// the op flag as is; every other routine materialises a transposed view
// once.  Scalars are real (complex matrices take real alpha / beta), as in
// the CPython-era C API this replaces (csrc/capi/capi.cpp, deprecated).
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "capi_util.hpp"

namespace slate_amd {
namespace native {
namespace capi {
namespace {

struct Handle {
    int what = 0;                  // 0 matrix, 1 pivots, 2 QR / LQ factors
    char dtype = 'd', kind = 'G', op = 'N';
    std::shared_ptr<void> mat;     // Matrix<T>
    std::vector<int64_t> piv;
    std::shared_ptr<void> fac;     // QRFactors<T> / LQFactors<T>
    bool lq = false;
    char fac_dt = 0;
};

std::mutex g_mu;
std::map<int64_t, std::shared_ptr<Handle>> g_reg;
int64_t g_next = 1;
Options g_opts;

int64_t put(std::shared_ptr<Handle> h) {
    std::lock_guard<std::mutex> lk(g_mu);
    const int64_t id = g_next++;
    g_reg[id] = std::move(h);
    return id;
}

Handle& get(int64_t id, int what = 0) {
    std::lock_guard<std::mutex> lk(g_mu);
    auto it = g_reg.find(id);
    if (it == g_reg.end()) throw Error("slate_amd handle " + std::to_string(id) + " does not exist");
    if (it->second->what != what)
        throw Error("slate_amd handle " + std::to_string(id) + " is not a " +
                    (what == 0 ? "matrix" : what == 1 ? "pivots" : "tfactors") + " handle");
    return *it->second;
}

template <typename F>
auto dispatch(char dt, F&& f) {
    switch (dt) {
        case 's': return f(float{});
        case 'd': return f(double{});
        case 'c': return f(std::complex<float>{});
        case 'z': return f(std::complex<double>{});
    }
    throw Error(std::string("slate_amd: unknown dtype '") + dt + "'");
}

template <typename T>
Matrix<T>& base(Handle& h) {
    return *static_cast<Matrix<T>*>(h.mat.get());
}

// the handle's matrix as op(A): its storage (op 'N') or a transposed copy
template <typename T>
Matrix<T> value(Handle& h) {
    Matrix<T>& A = base<T>(h);
    if (h.op == 'N') return A;
    Matrix<T> B(A.n(), A.m(), A.nb(), A.p(), A.q());
    copy<T>(op_of(h.op), A, B);
    return B;
}

// an output operand: it must be a plain (non-transposed) handle
template <typename T>
Matrix<T>& out(Handle& h) {
    if (h.op != 'N') throw Error("slate_amd: a transposed view cannot be an output");
    return base<T>(h);
}

Uplo uplo_h(const Handle& h) { return h.kind == 'U' ? Uplo::Upper : Uplo::Lower; }

template <typename T>
HermitianMatrix<T> herm(Handle& h) {
    return HermitianMatrix<T>(uplo_h(h), value<T>(h));
}

template <typename T>
Op op_h(const Handle& h) {
    if (h.op == 'N') return Op::NoTrans;
    if (h.op == 'C' || !is_cplx<T>()) return is_cplx<T>() ? Op::ConjTrans : Op::Trans;
    return Op::Trans;
}

void same_type(const Handle& a, const Handle& b) {
    if (a.dtype != b.dtype) throw Error("slate_amd: operands of different element types");
}

template <typename T>
void put_reals(double* w, const std::vector<real_t<T>>& v) {
    if (w)
        for (size_t i = 0; i < v.size(); ++i) w[i] = (double)v[i];
}

// C op(Q) from the left-only drivers: C op(Q) = (op(Q)^H C^H)^H
template <typename T, typename Apply>
void apply_right(Op op, Matrix<T>& C, Apply&& left) {
    Matrix<T> Ch(C.n(), C.m(), C.nb(), C.p(), C.q());
    copy<T>(Op::ConjTrans, C, Ch);
    left(op == Op::NoTrans ? Op::ConjTrans : Op::NoTrans, Ch);
    copy<T>(Op::ConjTrans, Ch, C);
}

template <typename T> constexpr bool is_hi() {
    return std::is_same<T, double>::value || std::is_same<T, std::complex<double>>::value;
}

}  // namespace
}  // namespace capi
}  // namespace native
}  // namespace slate_amd

using namespace slate_amd::native;
using namespace slate_amd::native::capi;

typedef int64_t slate_amd_matrix_t;
typedef int64_t slate_amd_pivots_t;
typedef int64_t slate_amd_tfactors_t;

#define G(...) (int)guarded([&]() -> int64_t { __VA_ARGS__ })
#define TYPED(h, ...) dispatch((h).dtype, [&](auto tag_) -> int64_t { using T = decltype(tag_); __VA_ARGS__ })

extern "C" {

slate_amd_matrix_t slate_amd_matrix_create(char kind, char dtype, int64_t m, int64_t n, int64_t nb, int p, int q) {
    return guarded([&]() -> int64_t {
        auto h = std::make_shared<Handle>();
        h->kind = up(kind);
        h->dtype = (char)(dtype | 0x20);
        if (h->kind != 'G' && h->kind != 'L' && h->kind != 'U') throw Error("slate_amd_matrix_create: kind G, L or U");
        if (h->kind != 'G' && m != n) throw Error("slate_amd_matrix_create: a Hermitian matrix is square");
        dispatch(h->dtype, [&](auto tag_) -> int64_t {
            using T = decltype(tag_);
            h->mat = std::make_shared<Matrix<T>>(m, n, nb, p, q);
            return 0;
        });
        return put(h);
    });
}

int slate_amd_matrix_destroy(slate_amd_matrix_t A) {
    return G({
        std::lock_guard<std::mutex> lk(g_mu);
        g_reg.erase(A);
        return 0;
    });
}

int slate_amd_matrix_local_size(slate_amd_matrix_t A, int64_t* mloc, int64_t* nloc) {
    return G({
        Handle& h = get(A);
        TYPED(h, {
            Matrix<T>& M = base<T>(h);
            *mloc = M.mloc();
            *nloc = M.nloc();
            return 0;
        });
        return 0;
    });
}

int slate_amd_matrix_get_local(slate_amd_matrix_t A, void* dst, int64_t ld) {
    return G({
        Handle& h = get(A);
        return TYPED(h, {
            base<T>(h).to_local_host(static_cast<T*>(dst), ld);
            return 0;
        });
    });
}

int slate_amd_matrix_set_local(slate_amd_matrix_t A, const void* src, int64_t ld) {
    return G({
        Handle& h = get(A);
        return TYPED(h, {
            base<T>(h).from_local_host(static_cast<const T*>(src), ld);
            return 0;
        });
    });
}

int slate_amd_matrix_generate(slate_amd_matrix_t A, int kind, int64_t seed) {
    return G({
        Handle& h = get(A);
        const Gen g = kind == 1 ? Gen::HermitianPositiveDefinite : kind == 3 ? Gen::DiagDominant : Gen::Random;
        return TYPED(h, {
            base<T>(h).generate(g, (uint64_t)seed);
            return 0;
        });
    });
}

slate_amd_pivots_t slate_amd_pivots_create(void) {
    return guarded([&]() -> int64_t {
        auto h = std::make_shared<Handle>();
        h->what = 1;
        return put(h);
    });
}
int slate_amd_pivots_destroy(slate_amd_pivots_t piv) { return slate_amd_matrix_destroy(piv); }

slate_amd_tfactors_t slate_amd_tfactors_create(void) {
    return guarded([&]() -> int64_t {
        auto h = std::make_shared<Handle>();
        h->what = 2;
        return put(h);
    });
}
int slate_amd_tfactors_destroy(slate_amd_tfactors_t T) { return slate_amd_matrix_destroy(T); }

double slate_amd_norm(char nrm, slate_amd_matrix_t A) {
    double r = -1;
    const int rc = G({
        Handle& h = get(A);
        const char c = up(nrm);
        const Norm k = c == '1' || c == 'O' ? Norm::One : c == 'I' ? Norm::Inf : c == 'F' || c == 'E' ? Norm::Fro
                                                                                                   : Norm::Max;
        return TYPED(h, {
            if (h.kind != 'G') r = norm<T>(k, herm<T>(h));
            else r = norm<T>(k, value<T>(h));
            return 0;
        });
    });
    return rc ? (double)rc : r;
}

int slate_amd_gemm(double alpha, slate_amd_matrix_t A, slate_amd_matrix_t B, double beta, slate_amd_matrix_t C) {
    return G({
        Handle &ha = get(A), &hb = get(B), &hc = get(C);
        same_type(ha, hb);
        same_type(ha, hc);
        return TYPED(ha, {
            gemm<T>(op_h<T>(ha), op_h<T>(hb), T(alpha), base<T>(ha), base<T>(hb), T(beta), out<T>(hc), g_opts);
            return 0;
        });
    });
}

int slate_amd_potrf(slate_amd_matrix_t A) {
    return G({
        Handle& h = get(A);
        return TYPED(h, {
            HermitianMatrix<T> H(uplo_h(h), out<T>(h));
            return potrf<T>(H, g_opts);
        });
    });
}

int slate_amd_potrs(slate_amd_matrix_t A, slate_amd_matrix_t B) {
    return G({
        Handle &ha = get(A), &hb = get(B);
        same_type(ha, hb);
        return TYPED(ha, { return potrs<T>(herm<T>(ha), out<T>(hb), g_opts); });
    });
}

int slate_amd_posv(slate_amd_matrix_t A, slate_amd_matrix_t B) {
    return G({
        Handle &ha = get(A), &hb = get(B);
        same_type(ha, hb);
        return TYPED(ha, {
            HermitianMatrix<T> H(uplo_h(ha), out<T>(ha));
            return posv<T>(H, out<T>(hb), g_opts);
        });
    });
}

int slate_amd_getrf(slate_amd_matrix_t A, slate_amd_pivots_t piv) {
    return G({
        Handle &ha = get(A), &hp = get(piv, 1);
        return TYPED(ha, { return getrf<T>(out<T>(ha), hp.piv, g_opts); });
    });
}

int slate_amd_getrs(slate_amd_matrix_t A, slate_amd_pivots_t piv, slate_amd_matrix_t B) {
    return G({
        Handle &ha = get(A), &hp = get(piv, 1), &hb = get(B);
        same_type(ha, hb);
        // a transposed view of the factors solves op(A) X = B
        return TYPED(ha, { return getrs<T>(op_h<T>(ha), base<T>(ha), hp.piv, out<T>(hb), g_opts); });
    });
}

int slate_amd_gesv(slate_amd_matrix_t A, slate_amd_pivots_t piv, slate_amd_matrix_t B) {
    return G({
        Handle &ha = get(A), &hp = get(piv, 1), &hb = get(B);
        same_type(ha, hb);
        return TYPED(ha, { return gesv<T>(out<T>(ha), hp.piv, out<T>(hb), g_opts); });
    });
}

int slate_amd_gels(slate_amd_matrix_t A, slate_amd_matrix_t BX) {
    return G({
        Handle &ha = get(A), &hb = get(BX);
        same_type(ha, hb);
        return TYPED(ha, { return gels<T>(out<T>(ha), out<T>(hb), g_opts); });
    });
}

int slate_amd_heev(slate_amd_matrix_t A, double* w, slate_amd_matrix_t Z) {
    return G({
        Handle& ha = get(A);
        return TYPED(ha, {
            HermitianMatrix<T> H = herm<T>(ha);
            std::vector<real_t<T>> lam;
            int64_t info;
            if (Z) {
                Handle& hz = get(Z);
                same_type(ha, hz);
                info = heev<T>(H, lam, out<T>(hz), g_opts);
            } else {
                info = heev<T>(H, lam, g_opts);
            }
            put_reals<T>(w, lam);
            return info;
        });
    });
}

// ---- options and views
int slate_amd_set_option(const char* name, const char* value) {
    return G({
        std::string k(name ? name : ""), v(value ? value : "");
        for (auto& c : k) c = (char)std::tolower(c);
        k.erase(std::remove(k.begin(), k.end(), '_'), k.end());
        const int iv = std::atoi(v.c_str());
        if (k == "lookahead") g_opts.lookahead = iv;
        else if (k == "innerblocking" || k == "ib") g_opts.inner_blocking = iv;
        else if (k == "maxiterations") g_opts.max_iterations = iv;
        else if (k == "depth") g_opts.depth = iv;
        else if (k == "restart") g_opts.restart = iv;
        else if (k == "pivotthreshold") g_opts.pivot_threshold = std::atof(v.c_str());
        // other SLATE options (Target, MethodLU, ...) select paths that this
        // library fixes per routine: accepted and ignored
        return 0;
    });
}

int slate_amd_clear_options(void) {
    g_opts = Options{};
    return 0;
}

slate_amd_matrix_t slate_amd_matrix_sub(slate_amd_matrix_t A, int64_t i1, int64_t i2, int64_t j1, int64_t j2) {
    return guarded([&]() -> int64_t {
        Handle& h = get(A);
        if (h.op != 'N') throw Error("slate_amd_matrix_sub: sub-matrix of a transposed view");
        auto v = std::make_shared<Handle>(h);
        TYPED(h, {
            v->mat = std::make_shared<Matrix<T>>(base<T>(h).sub(i1, i2 + 1, j1, j2 + 1));
            return 0;
        });
        // an off-diagonal block of a Hermitian matrix is a general matrix
        if (i1 != j1 || i2 != j2) v->kind = 'G';
        return put(v);
    });
}

slate_amd_matrix_t slate_amd_matrix_op(slate_amd_matrix_t A, char op) {
    return guarded([&]() -> int64_t {
        Handle& h = get(A);
        auto v = std::make_shared<Handle>(h);
        const char o = up(op);
        if (o != 'T' && o != 'C' && o != 'N') throw Error("slate_amd_matrix_op: op N, T or C");
        // op(op(A)): N stays, T T = N, C C = N, T C = conj (not a view here)
        if (o == 'N') v->op = h.op;
        else if (h.op == 'N') v->op = o;
        else if (h.op == o) v->op = 'N';
        else throw Error("slate_amd_matrix_op: the conjugate of a matrix is not a view");
        return put(v);
    });
}

int slate_amd_matrix_dims(slate_amd_matrix_t A, int64_t* m, int64_t* n) {
    return G({
        Handle& h = get(A);
        return TYPED(h, {
            Matrix<T>& M = base<T>(h);
            *m = h.op == 'N' ? M.m() : M.n();
            *n = h.op == 'N' ? M.n() : M.m();
            return 0;
        });
    });
}

int slate_amd_matrix_tiles(slate_amd_matrix_t A, int64_t* mt, int64_t* nt) {
    int64_t m = 0, n = 0;
    const int rc = slate_amd_matrix_dims(A, &m, &n);
    if (rc) return rc;
    return G({
        Handle& h = get(A);
        return TYPED(h, {
            const int64_t nb = base<T>(h).nb();
            *mt = (m + nb - 1) / nb;
            *nt = (n + nb - 1) / nb;
            return 0;
        });
    });
}

// ---- BLAS-3
int slate_amd_trsm(char side, char uplo, char diag, double alpha, slate_amd_matrix_t A, slate_amd_matrix_t B) {
    return G({
        Handle &ha = get(A), &hb = get(B);
        same_type(ha, hb);
        // op(A) triangular with uplo / diag given for op(A): a transposed
        // view stores the opposite triangle
        const bool tr = ha.op != 'N';
        const Uplo u = uplo_of(uplo);
        const Uplo us = tr ? (u == Uplo::Lower ? Uplo::Upper : Uplo::Lower) : u;
        return TYPED(ha, {
            trsm<T>(side_of(side), us, op_h<T>(ha), diag_of(diag), T(alpha), base<T>(ha), out<T>(hb), g_opts);
            return 0;
        });
    });
}

int slate_amd_trmm(char side, char uplo, char diag, double alpha, slate_amd_matrix_t A, slate_amd_matrix_t B) {
    return G({
        Handle &ha = get(A), &hb = get(B);
        same_type(ha, hb);
        const bool tr = ha.op != 'N';
        const Uplo u = uplo_of(uplo);
        const Uplo us = tr ? (u == Uplo::Lower ? Uplo::Upper : Uplo::Lower) : u;
        return TYPED(ha, {
            trmm<T>(side_of(side), us, op_h<T>(ha), diag_of(diag), T(alpha), base<T>(ha), out<T>(hb), g_opts);
            return 0;
        });
    });
}

int slate_amd_herk(double alpha, slate_amd_matrix_t A, double beta, slate_amd_matrix_t C) {
    return G({
        Handle &ha = get(A), &hc = get(C);
        same_type(ha, hc);
        return TYPED(ha, {
            HermitianMatrix<T> H(uplo_h(hc), out<T>(hc));
            const Op o = ha.op == 'N' ? Op::NoTrans : Op::ConjTrans;
            if (ha.op == 'T' && is_cplx<T>()) throw Error("slate_amd_herk: a transposed (not conjugated) complex view");
            herk<T>(o, (real_t<T>)alpha, base<T>(ha), (real_t<T>)beta, H, g_opts);
            return 0;
        });
    });
}

int slate_amd_her2k(double alpha, slate_amd_matrix_t A, slate_amd_matrix_t B, double beta, slate_amd_matrix_t C) {
    return G({
        Handle &ha = get(A), &hb = get(B), &hc = get(C);
        same_type(ha, hb);
        same_type(ha, hc);
        return TYPED(ha, {
            HermitianMatrix<T> H(uplo_h(hc), out<T>(hc));
            her2k<T>(Op::NoTrans, T(alpha), value<T>(ha), value<T>(hb), (real_t<T>)beta, H, g_opts);
            return 0;
        });
    });
}

int slate_amd_hemm(char side, double alpha, slate_amd_matrix_t A, slate_amd_matrix_t B, double beta,
                   slate_amd_matrix_t C) {
    return G({
        Handle &ha = get(A), &hb = get(B), &hc = get(C);
        same_type(ha, hb);
        same_type(ha, hc);
        return TYPED(ha, {
            hemm<T>(side_of(side), T(alpha), herm<T>(ha), value<T>(hb), T(beta), out<T>(hc), g_opts);
            return 0;
        });
    });
}

// ---- factorizations, solves, inverses
int slate_amd_potri(slate_amd_matrix_t A) {
    return G({
        Handle& h = get(A);
        return TYPED(h, {
            HermitianMatrix<T> H(uplo_h(h), out<T>(h));
            return potri<T>(H, g_opts);
        });
    });
}

int slate_amd_trtri(char uplo, char diag, slate_amd_matrix_t A) {
    return G({
        Handle& h = get(A);
        return TYPED(h, { return trtri<T>(uplo_of(uplo), diag_of(diag), out<T>(h), g_opts); });
    });
}

int slate_amd_getri(slate_amd_matrix_t A, slate_amd_pivots_t piv) {
    return G({
        Handle &ha = get(A), &hp = get(piv, 1);
        return TYPED(ha, { return getri<T>(out<T>(ha), hp.piv, g_opts); });
    });
}

int slate_amd_geqrf(slate_amd_matrix_t A, slate_amd_tfactors_t Tf) {
    return G({
        Handle &ha = get(A), &ht = get(Tf, 2);
        return TYPED(ha, {
            auto f = std::make_shared<QRFactors<T>>();
            const int64_t info = geqrf<T>(out<T>(ha), *f, g_opts);
            ht.fac = f;
            ht.lq = false;
            ht.fac_dt = ha.dtype;
            return info;
        });
    });
}

int slate_amd_gelqf(slate_amd_matrix_t A, slate_amd_tfactors_t Tf) {
    return G({
        Handle &ha = get(A), &ht = get(Tf, 2);
        return TYPED(ha, {
            auto f = std::make_shared<LQFactors<T>>();
            const int64_t info = gelqf<T>(out<T>(ha), *f, g_opts);
            ht.fac = f;
            ht.lq = true;
            ht.fac_dt = ha.dtype;
            return info;
        });
    });
}

static int apply_q(bool lq, char side, char op, slate_amd_matrix_t A, slate_amd_tfactors_t Tf, slate_amd_matrix_t C) {
    return G({
        Handle &ha = get(A), &ht = get(Tf, 2), &hc = get(C);
        same_type(ha, hc);
        if (!ht.fac || ht.lq != lq || ht.fac_dt != ha.dtype)
            throw Error(std::string("slate_amd_") + (lq ? "unmlq" : "unmqr") + ": factors of a matching " +
                        (lq ? "gelqf" : "geqrf") + " expected");
        return TYPED(ha, {
            Matrix<T>& Cm = out<T>(hc);
            const Matrix<T>& Am = base<T>(ha);
            Op o = op_of(op);
            if (o == Op::Trans && is_cplx<T>()) throw Error("slate_amd_unmqr: op T of a complex Q (use C)");
            if (o == Op::Trans) o = Op::ConjTrans;
            auto left = [&](Op oo, Matrix<T>& X) {
                if (lq) unmlq<T>(oo, Am, *static_cast<LQFactors<T>*>(ht.fac.get()), X, g_opts);
                else unmqr<T>(oo, Am, *static_cast<QRFactors<T>*>(ht.fac.get()), X, g_opts);
            };
            if (up(side) == 'L') left(o, Cm);
            else apply_right<T>(o, Cm, left);
            return 0;
        });
    });
}

int slate_amd_unmqr(char side, char op, slate_amd_matrix_t A, slate_amd_tfactors_t T, slate_amd_matrix_t C) {
    return apply_q(false, side, op, A, T, C);
}
int slate_amd_unmlq(char side, char op, slate_amd_matrix_t A, slate_amd_tfactors_t T, slate_amd_matrix_t C) {
    return apply_q(true, side, op, A, T, C);
}

int slate_amd_gels_t(slate_amd_matrix_t A, slate_amd_tfactors_t Tf, slate_amd_matrix_t BX) {
    return G({
        (void)get(Tf, 2);
        return slate_amd_gels(A, BX);
    });
}

int slate_amd_hesv(slate_amd_matrix_t A, slate_amd_matrix_t B) {
    return G({
        Handle &ha = get(A), &hb = get(B);
        same_type(ha, hb);
        return TYPED(ha, {
            HermitianMatrix<T> H(uplo_h(ha), out<T>(ha));
            return hesv<T>(H, out<T>(hb), g_opts);
        });
    });
}

}  // extern "C"

template <bool GMRES>
static int gesv_mx(slate_amd_matrix_t A, slate_amd_pivots_t piv, slate_amd_matrix_t B, slate_amd_matrix_t X,
                   int64_t* iter) {
    return G({
        Handle &ha = get(A), &hp = get(piv, 1), &hb = get(B), &hx = get(X);
        same_type(ha, hb);
        same_type(ha, hx);
        return TYPED(ha, {
            if constexpr (is_hi<T>()) {
                int it = 0;
                const int64_t info = GMRES ? gesv_mixed_gmres<T>(out<T>(ha), hp.piv, out<T>(hb), out<T>(hx), it, g_opts)
                                           : gesv_mixed<T>(out<T>(ha), hp.piv, out<T>(hb), out<T>(hx), it, g_opts);
                if (iter) *iter = it;
                return info;
            } else {
                throw Error("slate_amd_gesv_mixed: double / complex<double> matrices only");
            }
        });
    });
}

template <bool GMRES>
static int posv_mx(slate_amd_matrix_t A, slate_amd_matrix_t B, slate_amd_matrix_t X, int64_t* iter) {
    return G({
        Handle &ha = get(A), &hb = get(B), &hx = get(X);
        same_type(ha, hb);
        same_type(ha, hx);
        return TYPED(ha, {
            if constexpr (is_hi<T>()) {
                int it = 0;
                HermitianMatrix<T> H(uplo_h(ha), out<T>(ha));
                const int64_t info = GMRES ? posv_mixed_gmres<T>(H, out<T>(hb), out<T>(hx), it, g_opts)
                                           : posv_mixed<T>(H, out<T>(hb), out<T>(hx), it, g_opts);
                if (iter) *iter = it;
                return info;
            } else {
                throw Error("slate_amd_posv_mixed: double / complex<double> matrices only");
            }
        });
    });
}

extern "C" {

int slate_amd_gesv_mixed(slate_amd_matrix_t A, slate_amd_pivots_t piv, slate_amd_matrix_t B, slate_amd_matrix_t X,
                         int64_t* iter) {
    return gesv_mx<false>(A, piv, B, X, iter);
}
int slate_amd_gesv_mixed_gmres(slate_amd_matrix_t A, slate_amd_pivots_t piv, slate_amd_matrix_t B,
                               slate_amd_matrix_t X, int64_t* iter) {
    return gesv_mx<true>(A, piv, B, X, iter);
}
int slate_amd_posv_mixed(slate_amd_matrix_t A, slate_amd_matrix_t B, slate_amd_matrix_t X, int64_t* iter) {
    return posv_mx<false>(A, B, X, iter);
}
int slate_amd_posv_mixed_gmres(slate_amd_matrix_t A, slate_amd_matrix_t B, slate_amd_matrix_t X, int64_t* iter) {
    return posv_mx<true>(A, B, X, iter);
}

int slate_amd_gesv_rbt(slate_amd_matrix_t A, slate_amd_matrix_t B) {
    return G({
        Handle &ha = get(A), &hb = get(B);
        same_type(ha, hb);
        return TYPED(ha, { return gesv_rbt<T>(out<T>(ha), out<T>(hb), g_opts); });
    });
}

int slate_amd_gesv_nopiv(slate_amd_matrix_t A, slate_amd_matrix_t B) {
    return G({
        Handle &ha = get(A), &hb = get(B);
        same_type(ha, hb);
        return TYPED(ha, { return gesv_nopiv<T>(out<T>(ha), out<T>(hb), g_opts); });
    });
}

// ---- spectra
int slate_amd_svd_vals(slate_amd_matrix_t A, double* s) {
    return G({
        Handle& ha = get(A);
        return TYPED(ha, {
            Matrix<T> M = value<T>(ha);
            std::vector<real_t<T>> sv;
            const int64_t info = svd<T>(M, sv, g_opts);
            put_reals<T>(s, sv);
            return info;
        });
    });
}

int slate_amd_hegv(int64_t itype, slate_amd_matrix_t A, slate_amd_matrix_t B, double* w, slate_amd_matrix_t Z) {
    return G({
        Handle &ha = get(A), &hb = get(B);
        same_type(ha, hb);
        return TYPED(ha, {
            HermitianMatrix<T> HA(uplo_h(ha), out<T>(ha)), HB(uplo_h(hb), out<T>(hb));
            std::vector<real_t<T>> lam;
            int64_t info;
            if (Z) {
                Handle& hz = get(Z);
                same_type(ha, hz);
                info = hegv<T>(itype, HA, HB, lam, out<T>(hz), g_opts);
            } else {
                info = hegv<T>(itype, HA, HB, lam, g_opts);
            }
            put_reals<T>(w, lam);
            return info;
        });
    });
}

// ---- auxiliary
int slate_amd_add(double alpha, slate_amd_matrix_t A, double beta, slate_amd_matrix_t B) {
    return G({
        Handle &ha = get(A), &hb = get(B);
        same_type(ha, hb);
        return TYPED(ha, {
            add<T>(T(alpha), value<T>(ha), T(beta), out<T>(hb));
            return 0;
        });
    });
}

int slate_amd_copy(slate_amd_matrix_t A, slate_amd_matrix_t B) {
    return G({
        Handle &ha = get(A), &hb = get(B);
        same_type(ha, hb);
        return TYPED(ha, {
            copy<T>(op_h<T>(ha), base<T>(ha), out<T>(hb));
            return 0;
        });
    });
}

int slate_amd_scale(double numer, double denom, slate_amd_matrix_t A) {
    return G({
        Handle& h = get(A);
        return TYPED(h, {
            scale<T>((real_t<T>)numer, (real_t<T>)denom, out<T>(h));
            return 0;
        });
    });
}

int slate_amd_set(double offdiag, double diag, slate_amd_matrix_t A) {
    return G({
        Handle& h = get(A);
        return TYPED(h, {
            set<T>(T(offdiag), T(diag), out<T>(h));
            return 0;
        });
    });
}

double slate_amd_gecondest(char nrm, slate_amd_matrix_t A, slate_amd_pivots_t piv, double anorm) {
    double r = -1;
    const int rc = G({
        Handle& ha = get(A);
        (void)get(piv, 1);
        const Norm k = up(nrm) == 'I' ? Norm::Inf : Norm::One;
        return TYPED(ha, {
            r = gecondest<T>(k, base<T>(ha), anorm, g_opts);
            return 0;
        });
    });
    return rc ? (double)rc : r;
}

double slate_amd_pocondest(char nrm, slate_amd_matrix_t A, double anorm) {
    double r = -1;
    const int rc = G({
        Handle& ha = get(A);
        const Norm k = up(nrm) == 'I' ? Norm::Inf : Norm::One;
        return TYPED(ha, {
            r = pocondest<T>(k, herm<T>(ha), anorm, g_opts);
            return 0;
        });
    });
    return rc ? (double)rc : r;
}

}  // extern "C"
