/* slate_amd C API (the reference's generated C bindings,
 * src/c_api/wrappers.cc, include/slate/c_api/*.h, and the Fortran-callable
 * LAPACK API, lapack_api/).
 *
 * Link with -lslate_amd_c (built in-tree as slate_amd/libslate_amd_c.so).
 * The library embeds the Python runtime of slate_amd: call
 * slate_amd_initialize() once (it is also called lazily), and
 * slate_amd_finalize() at exit.  Arrays are column-major with leading
 * dimension ld*; complex arrays are interleaved (re, im) pairs.  Every
 * routine returns LAPACK's info: 0 = success, > 0 = numerical failure
 * (e.g. the first non-positive pivot), -i = argument i was illegal.
 * Failures of the runtime itself use two reserved codes far outside the
 * argument range, SLATE_AMD_ERR_INIT (the runtime could not be started)
 * and SLATE_AMD_ERR_INTERNAL (an exception inside the library); the message
 * is then in slate_amd_last_error().
 *
 * Each routine also has a Fortran-callable alias with a trailing
 * underscore and all arguments by reference (e.g. slate_dpotrf_).
 */
#ifndef SLATE_AMD_C_API_H
#define SLATE_AMD_C_API_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SLATE_AMD_ERR_INIT (-1000001)
#define SLATE_AMD_ERR_INTERNAL (-1000000)

int slate_amd_initialize(void);
void slate_amd_finalize(void);
const char* slate_amd_last_error(void);

#define SLATE_AMD_DECL(X, T)                                                                                \
    int slate_##X##gemm(char transa, char transb, int64_t m, int64_t n, int64_t k, T alpha, const T* a,   \
                        int64_t lda, const T* b, int64_t ldb, T beta, T* c, int64_t ldc);                   \
    int slate_##X##potrf(char uplo, int64_t n, T* a, int64_t lda);                                         \
    int slate_##X##potrs(char uplo, int64_t n, int64_t nrhs, const T* a, int64_t lda, T* b, int64_t ldb);  \
    int slate_##X##posv(char uplo, int64_t n, int64_t nrhs, T* a, int64_t lda, T* b, int64_t ldb);         \
    int slate_##X##getrf(int64_t m, int64_t n, T* a, int64_t lda, int64_t* ipiv);                          \
    int slate_##X##getrs(char trans, int64_t n, int64_t nrhs, const T* a, int64_t lda, const int64_t* ipiv, \
                         T* b, int64_t ldb);                                                               \
    int slate_##X##gesv(int64_t n, int64_t nrhs, T* a, int64_t lda, int64_t* ipiv, T* b, int64_t ldb);     \
    int slate_##X##trsm(char side, char uplo, char transa, char diag, int64_t m, int64_t n, T alpha,       \
                        const T* a, int64_t lda, T* b, int64_t ldb);                                        \
    int slate_##X##gels(char trans, int64_t m, int64_t n, int64_t nrhs, T* a, int64_t lda, T* b,           \
                        int64_t ldb);                                                                       \
    int slate_##X##potri(char uplo, int64_t n, T* a, int64_t lda);

/* real types: T is the element type; complex: interleaved pairs passed as
 * pointers to the real type and alpha/beta as (re, im) via the _c variants */
SLATE_AMD_DECL(s, float)
SLATE_AMD_DECL(d, double)
#undef SLATE_AMD_DECL

/* complex (interleaved) */
int slate_zpotrf(char uplo, int64_t n, double* a, int64_t lda);
int slate_zposv(char uplo, int64_t n, int64_t nrhs, double* a, int64_t lda, double* b, int64_t ldb);
int slate_zgesv(int64_t n, int64_t nrhs, double* a, int64_t lda, int64_t* ipiv, double* b, int64_t ldb);
int slate_cpotrf(char uplo, int64_t n, float* a, int64_t lda);
int slate_cgesv(int64_t n, int64_t nrhs, float* a, int64_t lda, int64_t* ipiv, float* b, int64_t ldb);

/* eigen / SVD (real) */
int slate_dsyev(char jobz, char uplo, int64_t n, double* a, int64_t lda, double* w);
int slate_dgesvd(char jobu, char jobvt, int64_t m, int64_t n, double* a, int64_t lda, double* s, double* u,
                 int64_t ldu, double* vt, int64_t ldvt);
double slate_dlange(char norm, int64_t m, int64_t n, const double* a, int64_t lda);

/* Fortran-callable aliases (by reference) */
void slate_dpotrf_(const char* uplo, const int64_t* n, double* a, const int64_t* lda, int64_t* info);
void slate_dgesv_(const int64_t* n, const int64_t* nrhs, double* a, const int64_t* lda, int64_t* ipiv,
                  double* b, const int64_t* ldb, int64_t* info);
void slate_dgemm_(const char* ta, const char* tb, const int64_t* m, const int64_t* n, const int64_t* k,
                  const double* alpha, const double* a, const int64_t* lda, const double* b, const int64_t* ldb,
                  const double* beta, double* c, const int64_t* ldc);

#ifdef __cplusplus
}
#endif
#endif
