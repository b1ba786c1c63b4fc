// C ABI of slate_amd (include/slate_amd/c_api.h): embeds the CPython
// runtime that drives the framework and forwards each call, with raw
// pointers passed as integers, to slate_amd.compat.capi_bridge.call().
// Replaces the reference's generated C wrappers (src/c_api/wrappers.cc)
// and Fortran-callable LAPACK API (lapack_api/).
#include <Python.h>

#include <cstdint>
#include <cstring>
#include <mutex>
#include <string>

#include "../../../include/slate_amd/c_api.h"

namespace {

std::mutex g_mu;
PyObject* g_call = nullptr;
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
    Py_DECREF(mod);
    PyGILState_Release(st);
    if (g_owned) PyEval_SaveThread();   // release the GIL held by the init thread
    return g_call != nullptr;
}

// fmt: Py_BuildValue format of the arguments after the routine name
template <typename... A>
double invoke(const char* name, const char* fmt, A... args) {
    if (!ensure()) return SLATE_AMD_ERR_INIT;
    PyGILState_STATE st = PyGILState_Ensure();
    std::string f = std::string("(s") + fmt + ")";
    PyObject* targs = Py_BuildValue(f.c_str(), name, args...);
    PyObject* r = targs ? PyObject_CallObject(g_call, targs) : nullptr;
    Py_XDECREF(targs);
    double out = SLATE_AMD_ERR_INTERNAL;
    if (!r) {
        PyObject *t, *v, *tb;
        PyErr_Fetch(&t, &v, &tb);
        PyObject* s = v ? PyObject_Str(v) : nullptr;
        g_err = s ? PyUnicode_AsUTF8(s) : "unknown error";
        Py_XDECREF(s); Py_XDECREF(t); Py_XDECREF(v); Py_XDECREF(tb);
    } else {
        out = PyFloat_Check(r) ? PyFloat_AsDouble(r) : (double)PyLong_AsLongLong(r);
        Py_DECREF(r);
    }
    PyGILState_Release(st);
    return out;
}

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

}  // extern "C"
