// DEPRECATED (round 6): libslate_amd_native.so now exports every symbol of
// this library (LAPACK-style, ScaLAPACK, BLACS and the matrix handles,
// csrc/native/capi_*.hip) without a Python runtime; link -lslate_amd_native.
// This CPython-embedding ABI stays only for the host-target (CPU) path.
//
// C ABI of slate_amd (include/slate_amd/c_api.h): embeds the CPython
// runtime that drives the framework and forwards each call, with raw
// pointers passed as integers, to slate_amd.compat.capi_bridge.call().
// Replaces the reference's generated C wrappers (src/c_api/wrappers.cc)
// and Fortran-callable LAPACK API (lapack_api/).
#include <Python.h>

#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>

#include "../../../include/slate_amd/c_api.h"

namespace {

std::mutex g_mu;
PyObject* g_call = nullptr;       // capi_bridge.call            (LAPACK-style)
PyObject* g_scal = nullptr;       // capi_bridge.scalapack_call  (p?xxx_)
PyObject* g_blacs = nullptr;      // capi_bridge.blacs           (Cblacs_*)
PyObject* g_handle = nullptr;     // capi_bridge.handle          (matrix handles)
bool g_owned = false;
thread_local std::string g_err;

bool ensure() {
    std::lock_guard<std::mutex> lk(g_mu);
    if (g_call) return true;
    if (!Py_IsInitialized()) {
        Py_InitializeEx(0);
        g_owned = true;
    }
    PyGILState_STATE st = PyGILState_Ensure();
    PyObject* mod = PyImport_ImportModule("slate_amd.compat.capi_bridge");
    if (!mod) {
        PyErr_Print();
        g_err = "cannot import slate_amd.compat.capi_bridge (is slate_amd on PYTHONPATH?)";
        PyGILState_Release(st);
        // the thread that initialised the interpreter still holds the GIL:
        // release it on the failure path too, or a later call from another
        // thread deadlocks in PyGILState_Ensure
        if (g_owned) { PyEval_SaveThread(); g_owned = false; }
        return false;
    }
    g_call = PyObject_GetAttrString(mod, "call");
    g_scal = PyObject_GetAttrString(mod, "scalapack_call");
    g_blacs = PyObject_GetAttrString(mod, "blacs");
    g_handle = PyObject_GetAttrString(mod, "handle");
    Py_DECREF(mod);
    PyGILState_Release(st);
    if (g_owned) PyEval_SaveThread();   // release the GIL held by the init thread
    return g_call != nullptr;
}

// fmt: Py_BuildValue format of the arguments after the routine name
template <typename... A>
double invoke_on(PyObject** fn, const char* name, const char* fmt, A... args) {
    if (!ensure()) return SLATE_AMD_ERR_INIT;
    PyGILState_STATE st = PyGILState_Ensure();
    std::string f = std::string("(s") + fmt + ")";
    PyObject* targs = Py_BuildValue(f.c_str(), name, args...);
    PyObject* r = targs ? PyObject_CallObject(*fn, targs) : nullptr;
    Py_XDECREF(targs);
    double out = SLATE_AMD_ERR_INTERNAL;
    if (!r) {
        PyObject *t, *v, *tb;
        PyErr_Fetch(&t, &v, &tb);
        PyObject* s = v ? PyObject_Str(v) : nullptr;
        g_err = s ? PyUnicode_AsUTF8(s) : "unknown error";
        Py_XDECREF(s);
        if (std::getenv("SLATE_AMD_CAPI_TRACEBACK")) {   // full Python traceback on stderr
            PyErr_Restore(t, v, tb);                       // steals the references
            PyErr_Print();
        } else {
            Py_XDECREF(t); Py_XDECREF(v); Py_XDECREF(tb);
        }
    } else {
        out = PyFloat_Check(r) ? PyFloat_AsDouble(r) : (double)PyLong_AsLongLong(r);
        Py_DECREF(r);
    }
    PyGILState_Release(st);
    return out;
}

template <typename... A>
double invoke(const char* name, const char* fmt, A... args) { return invoke_on(&g_call, name, fmt, args...); }

inline long long P(const void* p) { return (long long)(uintptr_t)p; }
inline int I(double v) { return (int)v; }

}  // namespace

extern "C" {

int slate_amd_initialize(void) { return ensure() ? 0 : -1; }

void slate_amd_finalize(void) {
    std::lock_guard<std::mutex> lk(g_mu);
    if (g_call) {
        PyGILState_STATE st = PyGILState_Ensure();
        Py_CLEAR(g_call);
        PyGILState_Release(st);
    }
}

const char* slate_amd_last_error(void) { return g_err.c_str(); }

#define SLATE_AMD_REAL(X, T)                                                                                 \
    int slate_##X##gemm(char ta, char tb, int64_t m, int64_t n, int64_t k, T alpha, const T* a, int64_t lda, \
                        const T* b, int64_t ldb, T beta, T* c, int64_t ldc) {                                 \
        return I(invoke(#X "gemm", "CCLLLdLLLLdLL", (int)ta, (int)tb, (long long)m, (long long)n,             \
                        (long long)k, (double)alpha, P(a), (long long)lda, P(b), (long long)ldb,              \
                        (double)beta, P(c), (long long)ldc));                                                  \
    }                                                                                                        \
    int slate_##X##potrf(char uplo, int64_t n, T* a, int64_t lda) {                                          \
        return I(invoke(#X "potrf", "CLLL", (int)uplo, (long long)n, P(a), (long long)lda));                 \
    }                                                                                                        \
    int slate_##X##potri(char uplo, int64_t n, T* a, int64_t lda) {                                          \
        return I(invoke(#X "potri", "CLLL", (int)uplo, (long long)n, P(a), (long long)lda));                 \
    }                                                                                                        \
    int slate_##X##potrs(char uplo, int64_t n, int64_t nrhs, const T* a, int64_t lda, T* b, int64_t ldb) {   \
        return I(invoke(#X "potrs", "CLLLLLL", (int)uplo, (long long)n, (long long)nrhs, P(a), (long long)lda, \
                        P(b), (long long)ldb));                                                               \
    }                                                                                                        \
    int slate_##X##posv(char uplo, int64_t n, int64_t nrhs, T* a, int64_t lda, T* b, int64_t ldb) {          \
        return I(invoke(#X "posv", "CLLLLLL", (int)uplo, (long long)n, (long long)nrhs, P(a), (long long)lda,  \
                        P(b), (long long)ldb));                                                               \
    }                                                                                                        \
    int slate_##X##getrf(int64_t m, int64_t n, T* a, int64_t lda, int64_t* ipiv) {                           \
        return I(invoke(#X "getrf", "LLLLL", (long long)m, (long long)n, P(a), (long long)lda, P(ipiv)));     \
    }                                                                                                        \
    int slate_##X##getrs(char t, int64_t n, int64_t nrhs, const T* a, int64_t lda, const int64_t* ipiv, T* b, \
                         int64_t ldb) {                                                                        \
        return I(invoke(#X "getrs", "CLLLLLLL", (int)t, (long long)n, (long long)nrhs, P(a), (long long)lda,   \
                        P(ipiv), P(b), (long long)ldb));                                                      \
    }                                                                                                        \
    int slate_##X##gesv(int64_t n, int64_t nrhs, T* a, int64_t lda, int64_t* ipiv, T* b, int64_t ldb) {      \
        return I(invoke(#X "gesv", "LLLLLLL", (long long)n, (long long)nrhs, P(a), (long long)lda, P(ipiv),    \
                        P(b), (long long)ldb));                                                               \
    }                                                                                                        \
    int slate_##X##trsm(char side, char uplo, char ta, char diag, int64_t m, int64_t n, T alpha, const T* a,  \
                        int64_t lda, T* b, int64_t ldb) {                                                      \
        return I(invoke(#X "trsm", "CCCCLLdLLLL", (int)side, (int)uplo, (int)ta, (int)diag, (long long)m,      \
                        (long long)n, (double)alpha, P(a), (long long)lda, P(b), (long long)ldb));            \
    }                                                                                                        \
    int slate_##X##gels(char t, int64_t m, int64_t n, int64_t nrhs, T* a, int64_t lda, T* b, int64_t ldb) {  \
        return I(invoke(#X "gels", "CLLLLLLL", (int)t, (long long)m, (long long)n, (long long)nrhs, P(a),      \
                        (long long)lda, P(b), (long long)ldb));                                               \
    }

SLATE_AMD_REAL(s, float)
SLATE_AMD_REAL(d, double)
#undef SLATE_AMD_REAL

int slate_zpotrf(char uplo, int64_t n, double* a, int64_t lda) {
    return I(invoke("zpotrf", "CLLL", (int)uplo, (long long)n, P(a), (long long)lda));
}
int slate_zposv(char uplo, int64_t n, int64_t nrhs, double* a, int64_t lda, double* b, int64_t ldb) {
    return I(invoke("zposv", "CLLLLLL", (int)uplo, (long long)n, (long long)nrhs, P(a), (long long)lda, P(b),
                    (long long)ldb));
}
int slate_zgesv(int64_t n, int64_t nrhs, double* a, int64_t lda, int64_t* ipiv, double* b, int64_t ldb) {
    return I(invoke("zgesv", "LLLLLLL", (long long)n, (long long)nrhs, P(a), (long long)lda, P(ipiv), P(b),
                    (long long)ldb));
}
int slate_cpotrf(char uplo, int64_t n, float* a, int64_t lda) {
    return I(invoke("cpotrf", "CLLL", (int)uplo, (long long)n, P(a), (long long)lda));
}
int slate_cgesv(int64_t n, int64_t nrhs, float* a, int64_t lda, int64_t* ipiv, float* b, int64_t ldb) {
    return I(invoke("cgesv", "LLLLLLL", (long long)n, (long long)nrhs, P(a), (long long)lda, P(ipiv), P(b),
                    (long long)ldb));
}
int slate_dsyev(char jobz, char uplo, int64_t n, double* a, int64_t lda, double* w) {
    return I(invoke("dsyev", "CCLLLL", (int)jobz, (int)uplo, (long long)n, P(a), (long long)lda, P(w)));
}
int slate_dgesvd(char jobu, char jobvt, int64_t m, int64_t n, double* a, int64_t lda, double* s, double* u,
                 int64_t ldu, double* vt, int64_t ldvt) {
    return I(invoke("dgesvd", "CCLLLLLLLLL", (int)jobu, (int)jobvt, (long long)m, (long long)n, P(a),
                    (long long)lda, P(s), P(u), (long long)ldu, P(vt), (long long)ldvt));
}
double slate_dlange(char norm, int64_t m, int64_t n, const double* a, int64_t lda) {
    return invoke("dlange", "CLLLL", (int)norm, (long long)m, (long long)n, P(a), (long long)lda);
}

// Fortran-callable aliases
void slate_dpotrf_(const char* uplo, const int64_t* n, double* a, const int64_t* lda, int64_t* info) {
    *info = slate_dpotrf(*uplo, *n, a, *lda);
}
void slate_dgesv_(const int64_t* n, const int64_t* nrhs, double* a, const int64_t* lda, int64_t* ipiv, double* b,
                  const int64_t* ldb, int64_t* info) {
    *info = slate_dgesv(*n, *nrhs, a, *lda, ipiv, b, *ldb);
}
void slate_dgemm_(const char* ta, const char* tb, const int64_t* m, const int64_t* n, const int64_t* k,
                  const double* alpha, const double* a, const int64_t* lda, const double* b, const int64_t* ldb,
                  const double* beta, double* c, const int64_t* ldc) {
    slate_dgemm(*ta, *tb, *m, *n, *k, *alpha, a, *lda, b, *ldb, *beta, c, *ldc);
}
void slate_dposv_(const char* uplo, const int64_t* n, const int64_t* nrhs, double* a, const int64_t* lda,
                  double* b, const int64_t* ldb, int64_t* info) {
    *info = slate_dposv(*uplo, *n, *nrhs, a, *lda, b, *ldb);
}
void slate_dgetrf_(const int64_t* m, const int64_t* n, double* a, const int64_t* lda, int64_t* ipiv,
                   int64_t* info) {
    *info = slate_dgetrf(*m, *n, a, *lda, ipiv);
}
void slate_dgetrs_(const char* t, const int64_t* n, const int64_t* nrhs, const double* a, const int64_t* lda,
                   const int64_t* ipiv, double* b, const int64_t* ldb, int64_t* info) {
    *info = slate_dgetrs(*t, *n, *nrhs, a, *lda, ipiv, b, *ldb);
}
void slate_dpotrs_(const char* uplo, const int64_t* n, const int64_t* nrhs, const double* a, const int64_t* lda,
                   double* b, const int64_t* ldb, int64_t* info) {
    *info = slate_dpotrs(*uplo, *n, *nrhs, a, *lda, b, *ldb);
}
void slate_dpotri_(const char* uplo, const int64_t* n, double* a, const int64_t* lda, int64_t* info) {
    *info = slate_dpotri(*uplo, *n, a, *lda);
}
void slate_dtrsm_(const char* side, const char* uplo, const char* ta, const char* diag, const int64_t* m,
                  const int64_t* n, const double* alpha, const double* a, const int64_t* lda, double* b,
                  const int64_t* ldb) {
    slate_dtrsm(*side, *uplo, *ta, *diag, *m, *n, *alpha, a, *lda, b, *ldb);
}
void slate_dgels_(const char* t, const int64_t* m, const int64_t* n, const int64_t* nrhs, double* a,
                  const int64_t* lda, double* b, const int64_t* ldb, int64_t* info) {
    *info = slate_dgels(*t, *m, *n, *nrhs, a, *lda, b, *ldb);
}
void slate_dsyev_(const char* jobz, const char* uplo, const int64_t* n, double* a, const int64_t* lda, double* w,
                  int64_t* info) {
    *info = slate_dsyev(*jobz, *uplo, *n, a, *lda, w);
}
double slate_dlange_(const char* norm, const int64_t* m, const int64_t* n, const double* a, const int64_t* lda) {
    return slate_dlange(*norm, *m, *n, a, *lda);
}
void slate_sgemm_(const char* ta, const char* tb, const int64_t* m, const int64_t* n, const int64_t* k,
                  const float* alpha, const float* a, const int64_t* lda, const float* b, const int64_t* ldb,
                  const float* beta, float* c, const int64_t* ldc) {
    slate_sgemm(*ta, *tb, *m, *n, *k, *alpha, a, *lda, b, *ldb, *beta, c, *ldc);
}
void slate_spotrf_(const char* uplo, const int64_t* n, float* a, const int64_t* lda, int64_t* info) {
    *info = slate_spotrf(*uplo, *n, a, *lda);
}
void slate_sgesv_(const int64_t* n, const int64_t* nrhs, float* a, const int64_t* lda, int64_t* ipiv, float* b,
                  const int64_t* ldb, int64_t* info) {
    *info = slate_sgesv(*n, *nrhs, a, *lda, ipiv, b, *ldb);
}

// --------------------------------------------- round-3 LAPACK-style ABI
// lapack_api/lapack_{trmm,syrk,syr2k,symm,getri,lansy,lantr,gecon,pocon,
// trcon,heevd,gesv_mixed,hemm,herk,her2k,lanhe}.cc.  Condition numbers and
// iteration counts are written to output pointers, info is returned.
#define SLATE_AMD_REAL2(X, T)                                                                                \
    int slate_##X##trmm(char side, char uplo, char ta, char diag, int64_t m, int64_t n, T alpha, const T* a,  \
                        int64_t lda, T* b, int64_t ldb) {                                                      \
        return I(invoke(#X "trmm", "CCCCLLdLLLL", (int)side, (int)uplo, (int)ta, (int)diag, (long long)m,      \
                        (long long)n, (double)alpha, P(a), (long long)lda, P(b), (long long)ldb));            \
    }                                                                                                        \
    int slate_##X##syrk(char uplo, char tr, int64_t n, int64_t k, T alpha, const T* a, int64_t lda, T beta,  \
                        T* c, int64_t ldc) {                                                                   \
        return I(invoke(#X "syrk", "CCLLdLLdLL", (int)uplo, (int)tr, (long long)n, (long long)k, (double)alpha, \
                        P(a), (long long)lda, (double)beta, P(c), (long long)ldc));                           \
    }                                                                                                        \
    int slate_##X##syr2k(char uplo, char tr, int64_t n, int64_t k, T alpha, const T* a, int64_t lda,         \
                         const T* b, int64_t ldb, T beta, T* c, int64_t ldc) {                                 \
        return I(invoke(#X "syr2k", "CCLLddLLLLdLL", (int)uplo, (int)tr, (long long)n, (long long)k,           \
                        (double)alpha, 0.0, P(a), (long long)lda, P(b), (long long)ldb, (double)beta, P(c),    \
                        (long long)ldc));                                                                     \
    }                                                                                                        \
    int slate_##X##symm(char side, char uplo, int64_t m, int64_t n, T alpha, const T* a, int64_t lda,        \
                        const T* b, int64_t ldb, T beta, T* c, int64_t ldc) {                                  \
        return I(invoke(#X "symm", "CCLLddLLLLddLL", (int)side, (int)uplo, (long long)m, (long long)n,         \
                        (double)alpha, 0.0, P(a), (long long)lda, P(b), (long long)ldb, (double)beta, 0.0,     \
                        P(c), (long long)ldc));                                                               \
    }                                                                                                        \
    int slate_##X##getri(int64_t n, T* a, int64_t lda, const int64_t* ipiv) {                                \
        return I(invoke(#X "getri", "LLLL", (long long)n, P(a), (long long)lda, P(ipiv)));                    \
    }                                                                                                        \
    double slate_##X##lansy(char norm, char uplo, int64_t n, const T* a, int64_t lda) {                      \
        return invoke(#X "lansy", "CCLLL", (int)norm, (int)uplo, (long long)n, P(a), (long long)lda);         \
    }                                                                                                        \
    double slate_##X##lantr(char norm, char uplo, char diag, int64_t m, int64_t n, const T* a, int64_t lda) { \
        return invoke(#X "lantr", "CCCLLLL", (int)norm, (int)uplo, (int)diag, (long long)m, (long long)n, P(a), \
                      (long long)lda);                                                                        \
    }                                                                                                        \
    int slate_##X##gecon(char norm, int64_t n, const T* a, int64_t lda, T anorm, T* rcond) {                 \
        return I(invoke(#X "gecon", "CLLLdL", (int)norm, (long long)n, P(a), (long long)lda, (double)anorm,   \
                        P(rcond)));                                                                           \
    }                                                                                                        \
    int slate_##X##pocon(char uplo, int64_t n, const T* a, int64_t lda, T anorm, T* rcond) {                 \
        return I(invoke(#X "pocon", "CLLLdL", (int)uplo, (long long)n, P(a), (long long)lda, (double)anorm,   \
                        P(rcond)));                                                                           \
    }                                                                                                        \
    int slate_##X##trcon(char norm, char uplo, char diag, int64_t n, const T* a, int64_t lda, T* rcond) {    \
        return I(invoke(#X "trcon", "CCCLLLL", (int)norm, (int)uplo, (int)diag, (long long)n, P(a),            \
                        (long long)lda, P(rcond)));                                                           \
    }                                                                                                        \
    int slate_##X##syevd(char jobz, char uplo, int64_t n, T* a, int64_t lda, T* w) {                         \
        return I(invoke(#X "syevd", "CCLLLL", (int)jobz, (int)uplo, (long long)n, P(a), (long long)lda, P(w))); \
    }

SLATE_AMD_REAL2(s, float)
SLATE_AMD_REAL2(d, double)
#undef SLATE_AMD_REAL2

int slate_dsgesv(int64_t n, int64_t nrhs, double* a, int64_t lda, int64_t* ipiv, double* b, int64_t ldb, double* x,
                 int64_t ldx, int64_t* iter) {
    return I(invoke("dgesv_mixed", "LLLLLLLLLL", (long long)n, (long long)nrhs, P(a), (long long)lda, P(ipiv), P(b),
                    (long long)ldb, P(x), (long long)ldx, P(iter)));
}

// complex<double> (interleaved re, im); complex scalars by pointer to (re, im)
int slate_zhemm(char side, char uplo, int64_t m, int64_t n, const double* alpha, const double* a, int64_t lda,
                const double* b, int64_t ldb, const double* beta, double* c, int64_t ldc) {
    return I(invoke("zhemm", "CCLLddLLLLddLL", (int)side, (int)uplo, (long long)m, (long long)n, alpha[0], alpha[1],
                    P(a), (long long)lda, P(b), (long long)ldb, beta[0], beta[1], P(c), (long long)ldc));
}
int slate_zherk(char uplo, char tr, int64_t n, int64_t k, double alpha, const double* a, int64_t lda, double beta,
                double* c, int64_t ldc) {
    return I(invoke("zherk", "CCLLdLLdLL", (int)uplo, (int)tr, (long long)n, (long long)k, alpha, P(a),
                    (long long)lda, beta, P(c), (long long)ldc));
}
int slate_zher2k(char uplo, char tr, int64_t n, int64_t k, const double* alpha, const double* a, int64_t lda,
                 const double* b, int64_t ldb, double beta, double* c, int64_t ldc) {
    return I(invoke("zher2k", "CCLLddLLLLdLL", (int)uplo, (int)tr, (long long)n, (long long)k, alpha[0], alpha[1],
                    P(a), (long long)lda, P(b), (long long)ldb, beta, P(c), (long long)ldc));
}
double slate_zlanhe(char norm, char uplo, int64_t n, const double* a, int64_t lda) {
    return invoke("zlanhe", "CCLLL", (int)norm, (int)uplo, (long long)n, P(a), (long long)lda);
}
int slate_zheevd(char jobz, char uplo, int64_t n, double* a, int64_t lda, double* w) {
    return I(invoke("zheevd", "CCLLLL", (int)jobz, (int)uplo, (long long)n, P(a), (long long)lda, P(w)));
}

// Fortran-callable aliases (all arguments by reference)
void slate_dtrmm_(const char* side, const char* uplo, const char* ta, const char* diag, const int64_t* m,
                  const int64_t* n, const double* alpha, const double* a, const int64_t* lda, double* b,
                  const int64_t* ldb) {
    slate_dtrmm(*side, *uplo, *ta, *diag, *m, *n, *alpha, a, *lda, b, *ldb);
}
void slate_dsyrk_(const char* uplo, const char* tr, const int64_t* n, const int64_t* k, const double* alpha,
                  const double* a, const int64_t* lda, const double* beta, double* c, const int64_t* ldc) {
    slate_dsyrk(*uplo, *tr, *n, *k, *alpha, a, *lda, *beta, c, *ldc);
}
void slate_dsyr2k_(const char* uplo, const char* tr, const int64_t* n, const int64_t* k, const double* alpha,
                   const double* a, const int64_t* lda, const double* b, const int64_t* ldb, const double* beta,
                   double* c, const int64_t* ldc) {
    slate_dsyr2k(*uplo, *tr, *n, *k, *alpha, a, *lda, b, *ldb, *beta, c, *ldc);
}
void slate_dsymm_(const char* side, const char* uplo, const int64_t* m, const int64_t* n, const double* alpha,
                  const double* a, const int64_t* lda, const double* b, const int64_t* ldb, const double* beta,
                  double* c, const int64_t* ldc) {
    slate_dsymm(*side, *uplo, *m, *n, *alpha, a, *lda, b, *ldb, *beta, c, *ldc);
}
void slate_dgetri_(const int64_t* n, double* a, const int64_t* lda, const int64_t* ipiv, int64_t* info) {
    *info = slate_dgetri(*n, a, *lda, ipiv);
}
double slate_dlansy_(const char* norm, const char* uplo, const int64_t* n, const double* a, const int64_t* lda) {
    return slate_dlansy(*norm, *uplo, *n, a, *lda);
}
double slate_dlantr_(const char* norm, const char* uplo, const char* diag, const int64_t* m, const int64_t* n,
                     const double* a, const int64_t* lda) {
    return slate_dlantr(*norm, *uplo, *diag, *m, *n, a, *lda);
}
void slate_dgecon_(const char* norm, const int64_t* n, const double* a, const int64_t* lda, const double* anorm,
                   double* rcond, int64_t* info) {
    *info = slate_dgecon(*norm, *n, a, *lda, *anorm, rcond);
}
void slate_dpocon_(const char* uplo, const int64_t* n, const double* a, const int64_t* lda, const double* anorm,
                   double* rcond, int64_t* info) {
    *info = slate_dpocon(*uplo, *n, a, *lda, *anorm, rcond);
}
void slate_dtrcon_(const char* norm, const char* uplo, const char* diag, const int64_t* n, const double* a,
                   const int64_t* lda, double* rcond, int64_t* info) {
    *info = slate_dtrcon(*norm, *uplo, *diag, *n, a, *lda, rcond);
}
void slate_dsyevd_(const char* jobz, const char* uplo, const int64_t* n, double* a, const int64_t* lda, double* w,
                   int64_t* info) {
    *info = slate_dsyevd(*jobz, *uplo, *n, a, *lda, w);
}
void slate_dsgesv_(const int64_t* n, const int64_t* nrhs, double* a, const int64_t* lda, int64_t* ipiv, double* b,
                   const int64_t* ldb, double* x, const int64_t* ldx, int64_t* iter, int64_t* info) {
    *info = slate_dsgesv(*n, *nrhs, a, *lda, ipiv, b, *ldb, x, *ldx, iter);
}

// ------------------------------------------------------------------ BLACS
// Minimal BLACS over torch.distributed (no MPI here): the process grid of a
// context is created by Cblacs_gridinit over the world of ranks started with
// RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT (torchrun convention).
void Cblacs_pinfo(int* mypnum, int* nprocs) {
    const double v = invoke_on(&g_blacs, "init", "");
    const long long x = (long long)v;
    *mypnum = (int)(x / 100000);
    *nprocs = (int)(x % 100000);
}
void Cblacs_get(int /*ctxt*/, int /*what*/, int* val) { *val = 0; }
void Cblacs_gridinit(int* ctxt, const char* order, int nprow, int npcol) {
    const char o = (order && (order[0] == 'R' || order[0] == 'r')) ? 'R' : 'C';
    *ctxt = (int)invoke_on(&g_blacs, "gridinit", "iii", (int)o, nprow, npcol);
}
void Cblacs_gridinfo(int ctxt, int* nprow, int* npcol, int* myrow, int* mycol) {
    const long long x = (long long)invoke_on(&g_blacs, "gridinfo", "i", ctxt);
    *mycol = (int)(x % 10000);
    *myrow = (int)((x / 10000) % 10000);
    *npcol = (int)((x / 100000000) % 10000);
    *nprow = (int)(x / 1000000000000LL);
}
void Cblacs_gridexit(int) {}
void Cblacs_exit(int) {}

int numroc_(const int* n, const int* nb, const int* iproc, const int* isrcproc, const int* nprocs) {
    const int mydist = (*nprocs + *iproc - *isrcproc) % *nprocs;
    const int nblocks = *n / *nb;
    int num = (nblocks / *nprocs) * *nb;
    const int extra = nblocks % *nprocs;
    if (mydist < extra) num += *nb;
    else if (mydist == extra) num += *n % *nb;
    return num;
}
void descinit_(int* desc, const int* m, const int* n, const int* mb, const int* nb, const int* irsrc,
               const int* icsrc, const int* ictxt, const int* lld, int* info) {
    desc[0] = 1; desc[1] = *ictxt; desc[2] = *m; desc[3] = *n; desc[4] = *mb; desc[5] = *nb;
    desc[6] = *irsrc; desc[7] = *icsrc; desc[8] = *lld;
    *info = (*m < 0) ? -2 : (*n < 0) ? -3 : (*mb < 1) ? -4 : (*nb < 1) ? -5 : 0;
}

// -------------------------------------------------------------- ScaLAPACK
// p?xxx_ interposers (SLATE scalapack_api/scalapack_*.cc): Fortran calling
// convention, 32-bit integers, descriptors of 9 ints.
#define D9 "(iiiiiiiii)"
#define DV(d) d[0], d[1], d[2], d[3], d[4], d[5], d[6], d[7], d[8]

#define SLATE_AMD_SCALAPACK_REAL(X, T)                                                                     \
    void p##X##potrf_(const char* uplo, const int* n, T* a, const int* ia, const int* ja, const int* desca,   \
                      int* info) {                                                                         \
        *info = I(invoke_on(&g_scal, "p" #X "potrf", "CiLii" D9, (int)*uplo, *n, P(a), *ia, *ja, DV(desca)));  \
    }                                                                                                      \
    void p##X##potrs_(const char* uplo, const int* n, const int* nrhs, const T* a, const int* ia,             \
                      const int* ja, const int* desca, T* b, const int* ib, const int* jb, const int* descb,  \
                      int* info) {                                                                         \
        *info = I(invoke_on(&g_scal, "p" #X "potrs", "CiiLii" D9 "Lii" D9, (int)*uplo, *n, *nrhs, P(a), *ia,   \
                            *ja, DV(desca), P(b), *ib, *jb, DV(descb)));                                    \
    }                                                                                                      \
    void p##X##posv_(const char* uplo, const int* n, const int* nrhs, T* a, const int* ia, const int* ja,    \
                     const int* desca, T* b, const int* ib, const int* jb, const int* descb, int* info) {     \
        *info = I(invoke_on(&g_scal, "p" #X "posv", "CiiLii" D9 "Lii" D9, (int)*uplo, *n, *nrhs, P(a), *ia,    \
                            *ja, DV(desca), P(b), *ib, *jb, DV(descb)));                                    \
    }                                                                                                      \
    void p##X##getrf_(const int* m, const int* n, T* a, const int* ia, const int* ja, const int* desca,      \
                      int* ipiv, int* info) {                                                              \
        *info = I(invoke_on(&g_scal, "p" #X "getrf", "iiLii" D9 "L", *m, *n, P(a), *ia, *ja, DV(desca),      \
                            P(ipiv)));                                                                      \
    }                                                                                                      \
    void p##X##getrs_(const char* t, const int* n, const int* nrhs, const T* a, const int* ia, const int* ja, \
                      const int* desca, const int* ipiv, T* b, const int* ib, const int* jb,                 \
                      const int* descb, int* info) {                                                       \
        *info = I(invoke_on(&g_scal, "p" #X "getrs", "CiiLii" D9 "LLii" D9, (int)*t, *n, *nrhs, P(a), *ia,     \
                            *ja, DV(desca), P(ipiv), P(b), *ib, *jb, DV(descb)));                           \
    }                                                                                                      \
    void p##X##gesv_(const int* n, const int* nrhs, T* a, const int* ia, const int* ja, const int* desca,    \
                     int* ipiv, T* b, const int* ib, const int* jb, const int* descb, int* info) {           \
        *info = I(invoke_on(&g_scal, "p" #X "gesv", "iiLii" D9 "LLii" D9, *n, *nrhs, P(a), *ia, *ja,          \
                            DV(desca), P(ipiv), P(b), *ib, *jb, DV(descb)));                                \
    }                                                                                                      \
    void p##X##gemm_(const char* ta, const char* tb, const int* m, const int* n, const int* k,                \
                     const T* alpha, const T* a, const int* ia, const int* ja, const int* desca, const T* b,  \
                     const int* ib, const int* jb, const int* descb, const T* beta, T* c, const int* ic,      \
                     const int* jc, const int* descc) {                                                    \
        invoke_on(&g_scal, "p" #X "gemm", "CCiiidLii" D9 "Lii" D9 "dLii" D9, (int)*ta, (int)*tb, *m, *n, *k,   \
                  (double)*alpha, P(a), *ia, *ja, DV(desca), P(b), *ib, *jb, DV(descb), (double)*beta, P(c),   \
                  *ic, *jc, DV(descc));                                                                    \
    }                                                                                                      \
    void p##X##trsm_(const char* side, const char* uplo, const char* ta, const char* diag, const int* m,     \
                     const int* n, const T* alpha, const T* a, const int* ia, const int* ja, const int* desca, \
                     T* b, const int* ib, const int* jb, const int* descb) {                                \
        invoke_on(&g_scal, "p" #X "trsm", "CCCCiidLii" D9 "Lii" D9, (int)*side, (int)*uplo, (int)*ta,          \
                  (int)*diag, *m, *n, (double)*alpha, P(a), *ia, *ja, DV(desca), P(b), *ib, *jb, DV(descb));    \
    }                                                                                                      \
    T p##X##lange_(const char* norm, const int* m, const int* n, const T* a, const int* ia, const int* ja,   \
                   const int* desca, T* /*work*/) {                                                        \
        return (T)invoke_on(&g_scal, "p" #X "lange", "CiiLii" D9, (int)*norm, *m, *n, P(a), *ia, *ja,          \
                            DV(desca));                                                                     \
    }

SLATE_AMD_SCALAPACK_REAL(s, float)
SLATE_AMD_SCALAPACK_REAL(d, double)
#undef SLATE_AMD_SCALAPACK_REAL

// complex: the factorizations / solves (alpha-free), interleaved (re, im)
#define SLATE_AMD_SCALAPACK_CPLX(X, R)                                                                     \
    void p##X##potrf_(const char* uplo, const int* n, R* a, const int* ia, const int* ja, const int* desca,   \
                      int* info) {                                                                         \
        *info = I(invoke_on(&g_scal, "p" #X "potrf", "CiLii" D9, (int)*uplo, *n, P(a), *ia, *ja, DV(desca)));  \
    }                                                                                                      \
    void p##X##getrf_(const int* m, const int* n, R* a, const int* ia, const int* ja, const int* desca,      \
                      int* ipiv, int* info) {                                                              \
        *info = I(invoke_on(&g_scal, "p" #X "getrf", "iiLii" D9 "L", *m, *n, P(a), *ia, *ja, DV(desca),      \
                            P(ipiv)));                                                                      \
    }                                                                                                      \
    void p##X##gesv_(const int* n, const int* nrhs, R* a, const int* ia, const int* ja, const int* desca,    \
                     int* ipiv, R* b, const int* ib, const int* jb, const int* descb, int* info) {           \
        *info = I(invoke_on(&g_scal, "p" #X "gesv", "iiLii" D9 "LLii" D9, *n, *nrhs, P(a), *ia, *ja,          \
                            DV(desca), P(ipiv), P(b), *ib, *jb, DV(descb)));                                \
    }                                                                                                      \
    void p##X##posv_(const char* uplo, const int* n, const int* nrhs, R* a, const int* ia, const int* ja,    \
                     const int* desca, R* b, const int* ib, const int* jb, const int* descb, int* info) {     \
        *info = I(invoke_on(&g_scal, "p" #X "posv", "CiiLii" D9 "Lii" D9, (int)*uplo, *n, *nrhs, P(a), *ia,    \
                            *ja, DV(desca), P(b), *ib, *jb, DV(descb)));                                    \
    }

SLATE_AMD_SCALAPACK_CPLX(c, float)
SLATE_AMD_SCALAPACK_CPLX(z, double)
#undef SLATE_AMD_SCALAPACK_CPLX

// ------------------------------------- round-3 ScaLAPACK interposers
// scalapack_api/scalapack_{trmm,syrk,syr2k,symm,potri,getri,lansy,lantr,
// gecon,pocon,trcon,syev,syevd,gesvd,gels,gesv_mixed}.cc (+ the complex
// herk / her2k / hemm / lanhe / heev / heevd).  Workspace queries
// (lwork = -1) return a workspace size of 1 (the library allocates its own).
#define QUERY(lw, work, info)                                                                              \
    if (*(lw) == -1) { if (work) (work)[0] = 1; *(info) = 0; return; }

#define SLATE_AMD_SCALAPACK_REAL2(X, T)                                                                    \
    void p##X##trmm_(const char* side, const char* uplo, const char* ta, const char* diag, const int* m,     \
                     const int* n, const T* alpha, const T* a, const int* ia, const int* ja, const int* desca, \
                     T* b, const int* ib, const int* jb, const int* descb) {                                \
        invoke_on(&g_scal, "p" #X "trmm", "CCCCiidLii" D9 "Lii" D9, (int)*side, (int)*uplo, (int)*ta,          \
                  (int)*diag, *m, *n, (double)*alpha, P(a), *ia, *ja, DV(desca), P(b), *ib, *jb, DV(descb));    \
    }                                                                                                      \
    void p##X##syrk_(const char* uplo, const char* tr, const int* n, const int* k, const T* alpha,            \
                     const T* a, const int* ia, const int* ja, const int* desca, const T* beta, T* c,          \
                     const int* ic, const int* jc, const int* descc) {                                     \
        invoke_on(&g_scal, "p" #X "syrk", "CCiidLii" D9 "dLii" D9, (int)*uplo, (int)*tr, *n, *k,               \
                  (double)*alpha, P(a), *ia, *ja, DV(desca), (double)*beta, P(c), *ic, *jc, DV(descc));        \
    }                                                                                                      \
    void p##X##syr2k_(const char* uplo, const char* tr, const int* n, const int* k, const T* alpha,           \
                      const T* a, const int* ia, const int* ja, const int* desca, const T* b, const int* ib,    \
                      const int* jb, const int* descb, const T* beta, T* c, const int* ic, const int* jc,     \
                      const int* descc) {                                                                  \
        invoke_on(&g_scal, "p" #X "syr2k", "CCiiddLii" D9 "Lii" D9 "dLii" D9, (int)*uplo, (int)*tr, *n, *k,    \
                  (double)*alpha, 0.0, P(a), *ia, *ja, DV(desca), P(b), *ib, *jb, DV(descb), (double)*beta,    \
                  P(c), *ic, *jc, DV(descc));                                                              \
    }                                                                                                      \
    void p##X##symm_(const char* side, const char* uplo, const int* m, const int* n, const T* alpha,          \
                     const T* a, const int* ia, const int* ja, const int* desca, const T* b, const int* ib,     \
                     const int* jb, const int* descb, const T* beta, T* c, const int* ic, const int* jc,      \
                     const int* descc) {                                                                   \
        invoke_on(&g_scal, "p" #X "symm", "CCiiddLii" D9 "Lii" D9 "ddLii" D9, (int)*side, (int)*uplo, *m, *n,  \
                  (double)*alpha, 0.0, P(a), *ia, *ja, DV(desca), P(b), *ib, *jb, DV(descb), (double)*beta,    \
                  0.0, P(c), *ic, *jc, DV(descc));                                                         \
    }                                                                                                      \
    void p##X##potri_(const char* uplo, const int* n, T* a, const int* ia, const int* ja, const int* desca,   \
                      int* info) {                                                                         \
        *info = I(invoke_on(&g_scal, "p" #X "potri", "CiLii" D9, (int)*uplo, *n, P(a), *ia, *ja, DV(desca)));  \
    }                                                                                                      \
    void p##X##getri_(const int* n, T* a, const int* ia, const int* ja, const int* desca, const int* ipiv,    \
                      T* work, const int* lwork, int* iwork, const int* liwork, int* info) {               \
        (void)iwork; (void)liwork;                                                                         \
        QUERY(lwork, work, info)                                                                            \
        *info = I(invoke_on(&g_scal, "p" #X "getri", "iLii" D9 "L", *n, P(a), *ia, *ja, DV(desca), P(ipiv)));  \
    }                                                                                                      \
    T p##X##lansy_(const char* norm, const char* uplo, const int* n, const T* a, const int* ia, const int* ja, \
                   const int* desca, T* /*work*/) {                                                        \
        return (T)invoke_on(&g_scal, "p" #X "lansy", "CCiLii" D9, (int)*norm, (int)*uplo, *n, P(a), *ia, *ja,   \
                            DV(desca));                                                                     \
    }                                                                                                      \
    T p##X##lantr_(const char* norm, const char* uplo, const char* diag, const int* m, const int* n,          \
                   const T* a, const int* ia, const int* ja, const int* desca, T* /*work*/) {              \
        return (T)invoke_on(&g_scal, "p" #X "lantr", "CCCiiLii" D9, (int)*norm, (int)*uplo, (int)*diag, *m,     \
                            *n, P(a), *ia, *ja, DV(desca));                                                 \
    }                                                                                                      \
    void p##X##gecon_(const char* norm, const int* n, const T* a, const int* ia, const int* ja,              \
                      const int* desca, const T* anorm, T* rcond, T* work, const int* lwork, int* iwork,      \
                      const int* liwork, int* info) {                                                      \
        (void)iwork; (void)liwork;                                                                         \
        QUERY(lwork, work, info)                                                                            \
        *info = I(invoke_on(&g_scal, "p" #X "gecon", "CiLii" D9 "dL", (int)*norm, *n, P(a), *ia, *ja,          \
                            DV(desca), (double)*anorm, P(rcond)));                                          \
    }                                                                                                      \
    void p##X##pocon_(const char* uplo, const int* n, const T* a, const int* ia, const int* ja,              \
                      const int* desca, const T* anorm, T* rcond, T* work, const int* lwork, int* iwork,      \
                      const int* liwork, int* info) {                                                      \
        (void)iwork; (void)liwork;                                                                         \
        QUERY(lwork, work, info)                                                                            \
        *info = I(invoke_on(&g_scal, "p" #X "pocon", "CiLii" D9 "dL", (int)*uplo, *n, P(a), *ia, *ja,          \
                            DV(desca), (double)*anorm, P(rcond)));                                          \
    }                                                                                                      \
    void p##X##trcon_(const char* norm, const char* uplo, const char* diag, const int* n, const T* a,         \
                      const int* ia, const int* ja, const int* desca, T* rcond, T* work, const int* lwork,    \
                      int* iwork, const int* liwork, int* info) {                                          \
        (void)iwork; (void)liwork;                                                                         \
        QUERY(lwork, work, info)                                                                            \
        *info = I(invoke_on(&g_scal, "p" #X "trcon", "CCCiLii" D9 "L", (int)*norm, (int)*uplo, (int)*diag, *n, \
                            P(a), *ia, *ja, DV(desca), P(rcond)));                                          \
    }                                                                                                      \
    void p##X##syev_(const char* jobz, const char* uplo, const int* n, T* a, const int* ia, const int* ja,    \
                     const int* desca, T* w, T* z, const int* iz, const int* jz, const int* descz, T* work,   \
                     const int* lwork, int* info) {                                                        \
        QUERY(lwork, work, info)                                                                            \
        *info = I(invoke_on(&g_scal, "p" #X "syev", "CCiLii" D9 "LLii" D9, (int)*jobz, (int)*uplo, *n, P(a),    \
                            *ia, *ja, DV(desca), P(w), P(z), *iz, *jz, DV(descz)));                         \
    }                                                                                                      \
    void p##X##syevd_(const char* jobz, const char* uplo, const int* n, T* a, const int* ia, const int* ja,   \
                      const int* desca, T* w, T* z, const int* iz, const int* jz, const int* descz, T* work,  \
                      const int* lwork, int* iwork, const int* liwork, int* info) {                        \
        (void)iwork; (void)liwork;                                                                         \
        QUERY(lwork, work, info)                                                                            \
        *info = I(invoke_on(&g_scal, "p" #X "syevd", "CCiLii" D9 "LLii" D9, (int)*jobz, (int)*uplo, *n, P(a),   \
                            *ia, *ja, DV(desca), P(w), P(z), *iz, *jz, DV(descz)));                         \
    }                                                                                                      \
    void p##X##gesvd_(const char* jobu, const char* jobvt, const int* m, const int* n, T* a, const int* ia,  \
                      const int* ja, const int* desca, T* s, T* u, const int* iu, const int* ju,              \
                      const int* descu, T* vt, const int* ivt, const int* jvt, const int* descvt, T* work,    \
                      const int* lwork, int* info) {                                                       \
        QUERY(lwork, work, info)                                                                            \
        *info = I(invoke_on(&g_scal, "p" #X "gesvd", "CCiiLii" D9 "LLii" D9 "Lii" D9, (int)*jobu, (int)*jobvt,  \
                            *m, *n, P(a), *ia, *ja, DV(desca), P(s), P(u), *iu, *ju, DV(descu), P(vt), *ivt,   \
                            *jvt, DV(descvt)));                                                             \
    }                                                                                                      \
    void p##X##gels_(const char* t, const int* m, const int* n, const int* nrhs, T* a, const int* ia,        \
                     const int* ja, const int* desca, T* b, const int* ib, const int* jb, const int* descb,   \
                     T* work, const int* lwork, int* info) {                                               \
        QUERY(lwork, work, info)                                                                            \
        *info = I(invoke_on(&g_scal, "p" #X "gels", "CiiiLii" D9 "Lii" D9, (int)*t, *m, *n, *nrhs, P(a), *ia,  \
                            *ja, DV(desca), P(b), *ib, *jb, DV(descb)));                                    \
    }

SLATE_AMD_SCALAPACK_REAL2(s, float)
SLATE_AMD_SCALAPACK_REAL2(d, double)
#undef SLATE_AMD_SCALAPACK_REAL2

void pdsgesv_(const int* n, const int* nrhs, double* a, const int* ia, const int* ja, const int* desca, int* ipiv,
              double* b, const int* ib, const int* jb, const int* descb, double* x, const int* ix, const int* jx,
              const int* descx, int* iter, int* info) {
    *info = I(invoke_on(&g_scal, "pdgesv_mixed", "iiLii" D9 "LLii" D9 "Lii" D9 "L", *n, *nrhs, P(a), *ia, *ja,
                        DV(desca), P(ipiv), P(b), *ib, *jb, DV(descb), P(x), *ix, *jx, DV(descx), P(iter)));
}

// complex<double> (interleaved): Hermitian BLAS-3, norms, eigenvalues
void pzherk_(const char* uplo, const char* tr, const int* n, const int* k, const double* alpha, const double* a,
             const int* ia, const int* ja, const int* desca, const double* beta, double* c, const int* ic,
             const int* jc, const int* descc) {
    invoke_on(&g_scal, "pzherk", "CCiidLii" D9 "dLii" D9, (int)*uplo, (int)*tr, *n, *k, *alpha, P(a), *ia, *ja,
              DV(desca), *beta, P(c), *ic, *jc, DV(descc));
}
void pzher2k_(const char* uplo, const char* tr, const int* n, const int* k, const double* alpha, const double* a,
              const int* ia, const int* ja, const int* desca, const double* b, const int* ib, const int* jb,
              const int* descb, const double* beta, double* c, const int* ic, const int* jc, const int* descc) {
    invoke_on(&g_scal, "pzher2k", "CCiiddLii" D9 "Lii" D9 "dLii" D9, (int)*uplo, (int)*tr, *n, *k, alpha[0],
              alpha[1], P(a), *ia, *ja, DV(desca), P(b), *ib, *jb, DV(descb), *beta, P(c), *ic, *jc, DV(descc));
}
void pzhemm_(const char* side, const char* uplo, const int* m, const int* n, const double* alpha, const double* a,
             const int* ia, const int* ja, const int* desca, const double* b, const int* ib, const int* jb,
             const int* descb, const double* beta, double* c, const int* ic, const int* jc, const int* descc) {
    invoke_on(&g_scal, "pzhemm", "CCiiddLii" D9 "Lii" D9 "ddLii" D9, (int)*side, (int)*uplo, *m, *n, alpha[0],
              alpha[1], P(a), *ia, *ja, DV(desca), P(b), *ib, *jb, DV(descb), beta[0], beta[1], P(c), *ic, *jc,
              DV(descc));
}
double pzlanhe_(const char* norm, const char* uplo, const int* n, const double* a, const int* ia, const int* ja,
                const int* desca, double* /*work*/) {
    return invoke_on(&g_scal, "pzlanhe", "CCiLii" D9, (int)*norm, (int)*uplo, *n, P(a), *ia, *ja, DV(desca));
}
void pzheevd_(const char* jobz, const char* uplo, const int* n, double* a, const int* ia, const int* ja,
              const int* desca, double* w, double* z, const int* iz, const int* jz, const int* descz, double* work,
              const int* lwork, double* rwork, const int* lrwork, int* iwork, const int* liwork, int* info) {
    (void)rwork; (void)lrwork; (void)iwork; (void)liwork;
    QUERY(lwork, work, info)
    *info = I(invoke_on(&g_scal, "pzheevd", "CCiLii" D9 "LLii" D9, (int)*jobz, (int)*uplo, *n, P(a), *ia, *ja,
                        DV(desca), P(w), P(z), *iz, *jz, DV(descz)));
}
#undef QUERY

// ------------------------------------------------------ matrix handles
slate_amd_matrix_t slate_amd_matrix_create(char kind, char dtype, int64_t m, int64_t n, int64_t nb, int p, int q) {
    return (slate_amd_matrix_t)invoke_on(&g_handle, "create", "iiLLLii", (int)kind, (int)dtype, (long long)m,
                                         (long long)n, (long long)nb, p, q);
}
int slate_amd_matrix_destroy(slate_amd_matrix_t h) { return I(invoke_on(&g_handle, "destroy", "L", (long long)h)); }
int slate_amd_matrix_local_size(slate_amd_matrix_t h, int64_t* mloc, int64_t* nloc) {
    const double v = invoke_on(&g_handle, "local_size", "L", (long long)h);
    if (v < 0) return I(v);
    const long long x = (long long)v;
    *mloc = x / 1000000000LL;
    *nloc = x % 1000000000LL;
    return 0;
}
int slate_amd_matrix_get_local(slate_amd_matrix_t h, void* dst, int64_t ld) {
    return I(invoke_on(&g_handle, "get_local", "LLL", (long long)h, P(dst), (long long)ld));
}
int slate_amd_matrix_set_local(slate_amd_matrix_t h, const void* src, int64_t ld) {
    return I(invoke_on(&g_handle, "set_local", "LLL", (long long)h, P(src), (long long)ld));
}
int slate_amd_matrix_generate(slate_amd_matrix_t h, int kind, int64_t seed) {
    return I(invoke_on(&g_handle, "generate", "LiL", (long long)h, kind, (long long)seed));
}
slate_amd_pivots_t slate_amd_pivots_create(void) {
    return (slate_amd_pivots_t)invoke_on(&g_handle, "pivots_create", "");
}
int slate_amd_pivots_destroy(slate_amd_pivots_t h) { return I(invoke_on(&g_handle, "destroy", "L", (long long)h)); }
double slate_amd_norm(char norm, slate_amd_matrix_t A) {
    return invoke_on(&g_handle, "norm", "Li", (long long)A, (int)norm);
}
int slate_amd_gemm(double alpha, slate_amd_matrix_t A, slate_amd_matrix_t B, double beta, slate_amd_matrix_t C) {
    return I(invoke_on(&g_handle, "gemm", "dLLdL", alpha, (long long)A, (long long)B, beta, (long long)C));
}
int slate_amd_potrf(slate_amd_matrix_t A) { return I(invoke_on(&g_handle, "potrf", "L", (long long)A)); }
int slate_amd_posv(slate_amd_matrix_t A, slate_amd_matrix_t B) {
    return I(invoke_on(&g_handle, "posv", "LL", (long long)A, (long long)B));
}
int slate_amd_getrf(slate_amd_matrix_t A, slate_amd_pivots_t piv) {
    return I(invoke_on(&g_handle, "getrf", "LL", (long long)A, (long long)piv));
}
int slate_amd_getrs(slate_amd_matrix_t A, slate_amd_pivots_t piv, slate_amd_matrix_t B) {
    return I(invoke_on(&g_handle, "getrs", "LLL", (long long)A, (long long)piv, (long long)B));
}
int slate_amd_gesv(slate_amd_matrix_t A, slate_amd_pivots_t piv, slate_amd_matrix_t B) {
    return I(invoke_on(&g_handle, "gesv", "LLL", (long long)A, (long long)piv, (long long)B));
}
int slate_amd_gels(slate_amd_matrix_t A, slate_amd_matrix_t BX) {
    return I(invoke_on(&g_handle, "geqrf_gels", "LL", (long long)A, (long long)BX));
}
int slate_amd_heev(slate_amd_matrix_t A, double* w, slate_amd_matrix_t Z) {
    return I(invoke_on(&g_handle, "heev", "LLL", (long long)A, P(w), (long long)Z));
}

// ---- options, views and the wider routine set
#define H_(x) (long long)(x)
int slate_amd_set_option(const char* name, const char* value) {
    return I(invoke_on(&g_handle, "set_option", "ss", name, value));
}
int slate_amd_clear_options(void) { return I(invoke_on(&g_handle, "clear_options", "")); }
slate_amd_matrix_t slate_amd_matrix_sub(slate_amd_matrix_t A, int64_t i1, int64_t i2, int64_t j1, int64_t j2) {
    return (slate_amd_matrix_t)invoke_on(&g_handle, "sub", "LLLLL", H_(A), H_(i1), H_(i2), H_(j1), H_(j2));
}
slate_amd_matrix_t slate_amd_matrix_op(slate_amd_matrix_t A, char op) {
    return (slate_amd_matrix_t)invoke_on(&g_handle, "op_view", "Li", H_(A), (int)op);
}
static int split_pair(double v, int64_t* a, int64_t* b) {
    if (v < 0) return I(v);
    const long long x = (long long)v;
    *a = x / 1000000000LL;
    *b = x % 1000000000LL;
    return 0;
}
int slate_amd_matrix_dims(slate_amd_matrix_t A, int64_t* m, int64_t* n) {
    return split_pair(invoke_on(&g_handle, "dims", "L", H_(A)), m, n);
}
int slate_amd_matrix_tiles(slate_amd_matrix_t A, int64_t* mt, int64_t* nt) {
    return split_pair(invoke_on(&g_handle, "tiles", "L", H_(A)), mt, nt);
}
slate_amd_tfactors_t slate_amd_tfactors_create(void) {
    return (slate_amd_tfactors_t)invoke_on(&g_handle, "tfactors_create", "");
}
int slate_amd_tfactors_destroy(slate_amd_tfactors_t T) { return slate_amd_matrix_destroy(T); }
int slate_amd_trsm(char side, char uplo, char diag, double alpha, slate_amd_matrix_t A, slate_amd_matrix_t B) {
    return I(invoke_on(&g_handle, "trsm", "iiidLL", (int)side, (int)uplo, (int)diag, alpha, H_(A), H_(B)));
}
int slate_amd_trmm(char side, char uplo, char diag, double alpha, slate_amd_matrix_t A, slate_amd_matrix_t B) {
    return I(invoke_on(&g_handle, "trmm", "iiidLL", (int)side, (int)uplo, (int)diag, alpha, H_(A), H_(B)));
}
int slate_amd_herk(double alpha, slate_amd_matrix_t A, double beta, slate_amd_matrix_t C) {
    return I(invoke_on(&g_handle, "herk", "dLdL", alpha, H_(A), beta, H_(C)));
}
int slate_amd_her2k(double alpha, slate_amd_matrix_t A, slate_amd_matrix_t B, double beta, slate_amd_matrix_t C) {
    return I(invoke_on(&g_handle, "her2k", "dLLdL", alpha, H_(A), H_(B), beta, H_(C)));
}
int slate_amd_hemm(char side, double alpha, slate_amd_matrix_t A, slate_amd_matrix_t B, double beta,
                   slate_amd_matrix_t C) {
    return I(invoke_on(&g_handle, "hemm", "idLLdL", (int)side, alpha, H_(A), H_(B), beta, H_(C)));
}
int slate_amd_potrs(slate_amd_matrix_t A, slate_amd_matrix_t B) {
    return I(invoke_on(&g_handle, "potrs", "LL", H_(A), H_(B)));
}
int slate_amd_potri(slate_amd_matrix_t A) { return I(invoke_on(&g_handle, "potri", "L", H_(A))); }
int slate_amd_trtri(char uplo, char diag, slate_amd_matrix_t A) {
    return I(invoke_on(&g_handle, "trtri", "iiL", (int)uplo, (int)diag, H_(A)));
}
int slate_amd_getri(slate_amd_matrix_t A, slate_amd_pivots_t piv) {
    return I(invoke_on(&g_handle, "getri", "LL", H_(A), H_(piv)));
}
int slate_amd_geqrf(slate_amd_matrix_t A, slate_amd_tfactors_t T) {
    return I(invoke_on(&g_handle, "geqrf", "LL", H_(A), H_(T)));
}
int slate_amd_gelqf(slate_amd_matrix_t A, slate_amd_tfactors_t T) {
    return I(invoke_on(&g_handle, "gelqf", "LL", H_(A), H_(T)));
}
int slate_amd_unmqr(char side, char op, slate_amd_matrix_t A, slate_amd_tfactors_t T, slate_amd_matrix_t C) {
    return I(invoke_on(&g_handle, "unmqr", "iiLLL", (int)side, (int)op, H_(A), H_(T), H_(C)));
}
int slate_amd_unmlq(char side, char op, slate_amd_matrix_t A, slate_amd_tfactors_t T, slate_amd_matrix_t C) {
    return I(invoke_on(&g_handle, "unmlq", "iiLLL", (int)side, (int)op, H_(A), H_(T), H_(C)));
}
int slate_amd_gels_t(slate_amd_matrix_t A, slate_amd_tfactors_t T, slate_amd_matrix_t BX) {
    return I(invoke_on(&g_handle, "gels_t", "LLL", H_(A), H_(T), H_(BX)));
}
int slate_amd_hesv(slate_amd_matrix_t A, slate_amd_matrix_t B) {
    return I(invoke_on(&g_handle, "hesv", "LL", H_(A), H_(B)));
}
int slate_amd_gesv_mixed(slate_amd_matrix_t A, slate_amd_pivots_t piv, slate_amd_matrix_t B, slate_amd_matrix_t X,
                         int64_t* iter) {
    return I(invoke_on(&g_handle, "gesv_mixed", "LLLLL", H_(A), H_(piv), H_(B), H_(X), P(iter)));
}
int slate_amd_gesv_mixed_gmres(slate_amd_matrix_t A, slate_amd_pivots_t piv, slate_amd_matrix_t B,
                               slate_amd_matrix_t X, int64_t* iter) {
    return I(invoke_on(&g_handle, "gesv_mixed_gmres", "LLLLL", H_(A), H_(piv), H_(B), H_(X), P(iter)));
}
int slate_amd_posv_mixed(slate_amd_matrix_t A, slate_amd_matrix_t B, slate_amd_matrix_t X, int64_t* iter) {
    return I(invoke_on(&g_handle, "posv_mixed", "LLLL", H_(A), H_(B), H_(X), P(iter)));
}
int slate_amd_posv_mixed_gmres(slate_amd_matrix_t A, slate_amd_matrix_t B, slate_amd_matrix_t X, int64_t* iter) {
    return I(invoke_on(&g_handle, "posv_mixed_gmres", "LLLL", H_(A), H_(B), H_(X), P(iter)));
}
int slate_amd_gesv_rbt(slate_amd_matrix_t A, slate_amd_matrix_t B) {
    return I(invoke_on(&g_handle, "gesv_rbt", "LL", H_(A), H_(B)));
}
int slate_amd_gesv_nopiv(slate_amd_matrix_t A, slate_amd_matrix_t B) {
    return I(invoke_on(&g_handle, "gesv_nopiv", "LL", H_(A), H_(B)));
}
int slate_amd_svd_vals(slate_amd_matrix_t A, double* s) {
    return I(invoke_on(&g_handle, "svd_vals", "LL", H_(A), P(s)));
}
int slate_amd_hegv(int64_t itype, slate_amd_matrix_t A, slate_amd_matrix_t B, double* w, slate_amd_matrix_t Z) {
    return I(invoke_on(&g_handle, "hegv", "LLLLL", H_(itype), H_(A), H_(B), P(w), H_(Z)));
}
int slate_amd_add(double alpha, slate_amd_matrix_t A, double beta, slate_amd_matrix_t B) {
    return I(invoke_on(&g_handle, "add", "dLdL", alpha, H_(A), beta, H_(B)));
}
int slate_amd_copy(slate_amd_matrix_t A, slate_amd_matrix_t B) {
    return I(invoke_on(&g_handle, "copy", "LL", H_(A), H_(B)));
}
int slate_amd_scale(double numer, double denom, slate_amd_matrix_t A) {
    return I(invoke_on(&g_handle, "scale", "ddL", numer, denom, H_(A)));
}
int slate_amd_set(double offdiag, double diag, slate_amd_matrix_t A) {
    return I(invoke_on(&g_handle, "set", "ddL", offdiag, diag, H_(A)));
}
double slate_amd_gecondest(char norm, slate_amd_matrix_t A, slate_amd_pivots_t piv, double anorm) {
    return invoke_on(&g_handle, "gecondest", "iLLd", (int)norm, H_(A), H_(piv), anorm);
}
double slate_amd_pocondest(char norm, slate_amd_matrix_t A, double anorm) {
    return invoke_on(&g_handle, "pocondest", "iLd", (int)norm, H_(A), anorm);
}
#undef H_

}  // extern "C"
