/* slate_amd C API (the reference's generated C bindings,
 * src/c_api/wrappers.cc, include/slate/c_api/*.h, and the Fortran-callable
 * LAPACK API, lapack_api/).
 *
 * Link with -lslate_amd_native (slate_amd/libslate_amd_native.so: every
 * symbol below, no Python runtime).  The CPython-embedding
 * slate_amd/libslate_amd_c.so exports the same names and is deprecated.
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

void slate_dposv_(const char* uplo, const int64_t* n, const int64_t* nrhs, double* a, const int64_t* lda,
                  double* b, const int64_t* ldb, int64_t* info);
void slate_dgetrf_(const int64_t* m, const int64_t* n, double* a, const int64_t* lda, int64_t* ipiv,
                   int64_t* info);
void slate_dgetrs_(const char* trans, const int64_t* n, const int64_t* nrhs, const double* a, const int64_t* lda,
                   const int64_t* ipiv, double* b, const int64_t* ldb, int64_t* info);
void slate_dpotrs_(const char* uplo, const int64_t* n, const int64_t* nrhs, const double* a, const int64_t* lda,
                   double* b, const int64_t* ldb, int64_t* info);
void slate_dpotri_(const char* uplo, const int64_t* n, double* a, const int64_t* lda, int64_t* info);
void slate_dtrsm_(const char* side, const char* uplo, const char* transa, const char* diag, const int64_t* m,
                  const int64_t* n, const double* alpha, const double* a, const int64_t* lda, double* b,
                  const int64_t* ldb);
void slate_dgels_(const char* trans, const int64_t* m, const int64_t* n, const int64_t* nrhs, double* a,
                  const int64_t* lda, double* b, const int64_t* ldb, int64_t* info);
void slate_dsyev_(const char* jobz, const char* uplo, const int64_t* n, double* a, const int64_t* lda, double* w,
                  int64_t* info);
double slate_dlange_(const char* norm, const int64_t* m, const int64_t* n, const double* a, const int64_t* lda);
void slate_sgemm_(const char* ta, const char* tb, const int64_t* m, const int64_t* n, const int64_t* k,
                  const float* alpha, const float* a, const int64_t* lda, const float* b, const int64_t* ldb,
                  const float* beta, float* c, const int64_t* ldc);
void slate_spotrf_(const char* uplo, const int64_t* n, float* a, const int64_t* lda, int64_t* info);
void slate_sgesv_(const int64_t* n, const int64_t* nrhs, float* a, const int64_t* lda, int64_t* ipiv, float* b,
                  const int64_t* ldb, int64_t* info);

/* LAPACK-style routines added in round 3 (lapack_api/lapack_trmm.cc, _syrk,
 * _syr2k, _symm, _getri, _lansy, _lantr, _gecon, _pocon, _trcon, _heevd,
 * _gesv_mixed, _hemm, _herk, _her2k, _lanhe).  Return LAPACK info; the
 * condition numbers / refinement iterations go to the output pointers. */
#define SLATE_AMD_DECL2(X, T)                                                                                \
    int slate_##X##trmm(char side, char uplo, char ta, char diag, int64_t m, int64_t n, T alpha, const T* a,  \
                        int64_t lda, T* b, int64_t ldb);                                                      \
    int slate_##X##syrk(char uplo, char trans, int64_t n, int64_t k, T alpha, const T* a, int64_t lda, T beta, \
                        T* c, int64_t ldc);                                                                   \
    int slate_##X##syr2k(char uplo, char trans, int64_t n, int64_t k, T alpha, const T* a, int64_t lda,       \
                         const T* b, int64_t ldb, T beta, T* c, int64_t ldc);                                 \
    int slate_##X##symm(char side, char uplo, int64_t m, int64_t n, T alpha, const T* a, int64_t lda,         \
                        const T* b, int64_t ldb, T beta, T* c, int64_t ldc);                                  \
    int slate_##X##getri(int64_t n, T* a, int64_t lda, const int64_t* ipiv);                                  \
    double slate_##X##lansy(char norm, char uplo, int64_t n, const T* a, int64_t lda);                        \
    double slate_##X##lantr(char norm, char uplo, char diag, int64_t m, int64_t n, const T* a, int64_t lda);  \
    int slate_##X##gecon(char norm, int64_t n, const T* a, int64_t lda, T anorm, T* rcond);                  \
    int slate_##X##pocon(char uplo, int64_t n, const T* a, int64_t lda, T anorm, T* rcond);                  \
    int slate_##X##trcon(char norm, char uplo, char diag, int64_t n, const T* a, int64_t lda, T* rcond);     \
    int slate_##X##syevd(char jobz, char uplo, int64_t n, T* a, int64_t lda, T* w);
SLATE_AMD_DECL2(s, float)
SLATE_AMD_DECL2(d, double)
#undef SLATE_AMD_DECL2
int slate_dsgesv(int64_t n, int64_t nrhs, double* a, int64_t lda, int64_t* ipiv, double* b, int64_t ldb, double* x,
                 int64_t ldx, int64_t* iter);
/* complex<double>, interleaved (re, im); complex scalars by pointer */
int slate_zhemm(char side, char uplo, int64_t m, int64_t n, const double* alpha, const double* a, int64_t lda,
                const double* b, int64_t ldb, const double* beta, double* c, int64_t ldc);
int slate_zherk(char uplo, char trans, int64_t n, int64_t k, double alpha, const double* a, int64_t lda, double beta,
                double* c, int64_t ldc);
int slate_zher2k(char uplo, char trans, int64_t n, int64_t k, const double* alpha, const double* a, int64_t lda,
                 const double* b, int64_t ldb, double beta, double* c, int64_t ldc);
double slate_zlanhe(char norm, char uplo, int64_t n, const double* a, int64_t lda);
int slate_zheevd(char jobz, char uplo, int64_t n, double* a, int64_t lda, double* w);

/* ------------------------------------------------------------------
 * ScaLAPACK interface (SLATE scalapack_api/): p?xxx_ with the Fortran
 * calling convention, 32-bit integers and 9-int descriptors
 * [dtype, ctxt, m, n, mb, nb, rsrc, csrc, lld]; any global offsets ia/ja
 * (1-based); rsrc = csrc = 0.  Each rank passes its local array.  Process
 * grids come from the minimal BLACS below, over the ranks started with
 * RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT (torchrun convention). */
void Cblacs_pinfo(int* mypnum, int* nprocs);
void Cblacs_get(int ctxt, int what, int* val);
void Cblacs_gridinit(int* ctxt, const char* order, int nprow, int npcol);
void Cblacs_gridinfo(int ctxt, int* nprow, int* npcol, int* myrow, int* mycol);
void Cblacs_gridexit(int ctxt);
void Cblacs_exit(int notdone);
int numroc_(const int* n, const int* nb, const int* iproc, const int* isrcproc, const int* nprocs);
void descinit_(int* desc, const int* m, const int* n, const int* mb, const int* nb, const int* irsrc,
               const int* icsrc, const int* ictxt, const int* lld, int* info);

#define SLATE_AMD_PDECL(X, T)                                                                                \
    void p##X##potrf_(const char* uplo, const int* n, T* a, const int* ia, const int* ja, const int* desca,   \
                      int* info);                                                                          \
    void p##X##posv_(const char* uplo, const int* n, const int* nrhs, T* a, const int* ia, const int* ja,    \
                     const int* desca, T* b, const int* ib, const int* jb, const int* descb, int* info);      \
    void p##X##getrf_(const int* m, const int* n, T* a, const int* ia, const int* ja, const int* desca,      \
                      int* ipiv, int* info);                                                               \
    void p##X##gesv_(const int* n, const int* nrhs, T* a, const int* ia, const int* ja, const int* desca,    \
                     int* ipiv, T* b, const int* ib, const int* jb, const int* descb, int* info);
SLATE_AMD_PDECL(s, float)
SLATE_AMD_PDECL(d, double)
SLATE_AMD_PDECL(c, float)   /* complex: interleaved (re, im) */
SLATE_AMD_PDECL(z, double)
#undef SLATE_AMD_PDECL
#define SLATE_AMD_PDECL_R(X, T)                                                                              \
    void p##X##potrs_(const char* uplo, const int* n, const int* nrhs, const T* a, const int* ia,             \
                      const int* ja, const int* desca, T* b, const int* ib, const int* jb, const int* descb,  \
                      int* info);                                                                          \
    void p##X##getrs_(const char* trans, const int* n, const int* nrhs, const T* a, const int* ia,           \
                      const int* ja, const int* desca, const int* ipiv, T* b, const int* ib, const int* jb,  \
                      const int* descb, int* info);                                                        \
    void p##X##gemm_(const char* transa, const char* transb, const int* m, const int* n, const int* k,        \
                     const T* alpha, const T* a, const int* ia, const int* ja, const int* desca, const T* b,  \
                     const int* ib, const int* jb, const int* descb, const T* beta, T* c, const int* ic,      \
                     const int* jc, const int* descc);                                                     \
    void p##X##trsm_(const char* side, const char* uplo, const char* transa, const char* diag, const int* m, \
                     const int* n, const T* alpha, const T* a, const int* ia, const int* ja, const int* desca, \
                     T* b, const int* ib, const int* jb, const int* descb);                                 \
    T p##X##lange_(const char* norm, const int* m, const int* n, const T* a, const int* ia, const int* ja,   \
                   const int* desca, T* work);
SLATE_AMD_PDECL_R(s, float)
SLATE_AMD_PDECL_R(d, double)
#undef SLATE_AMD_PDECL_R

/* ScaLAPACK interposers added in round 3 (scalapack_api/scalapack_trmm.cc,
 * _syrk, _syr2k, _symm, _potri, _getri, _lansy, _lantr, _gecon, _pocon,
 * _trcon, _syev, _syevd, _gesvd, _gels, _gesv_mixed; complex _herk, _her2k,
 * _hemm, _lanhe, _heevd).  Workspace queries (lwork = -1) return 1. */
#define SLATE_AMD_PDECL2(X, T)                                                                               \
    void p##X##trmm_(const char* side, const char* uplo, const char* ta, const char* diag, const int* m,     \
                     const int* n, const T* alpha, const T* a, const int* ia, const int* ja, const int* desca, \
                     T* b, const int* ib, const int* jb, const int* descb);                                 \
    void p##X##syrk_(const char* uplo, const char* tr, const int* n, const int* k, const T* alpha,            \
                     const T* a, const int* ia, const int* ja, const int* desca, const T* beta, T* c,          \
                     const int* ic, const int* jc, const int* descc);                                      \
    void p##X##syr2k_(const char* uplo, const char* tr, const int* n, const int* k, const T* alpha,           \
                      const T* a, const int* ia, const int* ja, const int* desca, const T* b, const int* ib,    \
                      const int* jb, const int* descb, const T* beta, T* c, const int* ic, const int* jc,     \
                      const int* descc);                                                                   \
    void p##X##symm_(const char* side, const char* uplo, const int* m, const int* n, const T* alpha,          \
                     const T* a, const int* ia, const int* ja, const int* desca, const T* b, const int* ib,     \
                     const int* jb, const int* descb, const T* beta, T* c, const int* ic, const int* jc,      \
                     const int* descc);                                                                    \
    void p##X##potri_(const char* uplo, const int* n, T* a, const int* ia, const int* ja, const int* desca,   \
                      int* info);                                                                          \
    void p##X##getri_(const int* n, T* a, const int* ia, const int* ja, const int* desca, const int* ipiv,    \
                      T* work, const int* lwork, int* iwork, const int* liwork, int* info);                \
    T p##X##lansy_(const char* norm, const char* uplo, const int* n, const T* a, const int* ia, const int* ja, \
                   const int* desca, T* work);                                                             \
    T p##X##lantr_(const char* norm, const char* uplo, const char* diag, const int* m, const int* n,          \
                   const T* a, const int* ia, const int* ja, const int* desca, T* work);                   \
    void p##X##gecon_(const char* norm, const int* n, const T* a, const int* ia, const int* ja,              \
                      const int* desca, const T* anorm, T* rcond, T* work, const int* lwork, int* iwork,      \
                      const int* liwork, int* info);                                                       \
    void p##X##pocon_(const char* uplo, const int* n, const T* a, const int* ia, const int* ja,              \
                      const int* desca, const T* anorm, T* rcond, T* work, const int* lwork, int* iwork,      \
                      const int* liwork, int* info);                                                       \
    void p##X##trcon_(const char* norm, const char* uplo, const char* diag, const int* n, const T* a,         \
                      const int* ia, const int* ja, const int* desca, T* rcond, T* work, const int* lwork,    \
                      int* iwork, const int* liwork, int* info);                                           \
    void p##X##syev_(const char* jobz, const char* uplo, const int* n, T* a, const int* ia, const int* ja,    \
                     const int* desca, T* w, T* z, const int* iz, const int* jz, const int* descz, T* work,   \
                     const int* lwork, int* info);                                                         \
    void p##X##syevd_(const char* jobz, const char* uplo, const int* n, T* a, const int* ia, const int* ja,   \
                      const int* desca, T* w, T* z, const int* iz, const int* jz, const int* descz, T* work,  \
                      const int* lwork, int* iwork, const int* liwork, int* info);                         \
    void p##X##gesvd_(const char* jobu, const char* jobvt, const int* m, const int* n, T* a, const int* ia,  \
                      const int* ja, const int* desca, T* s, T* u, const int* iu, const int* ju,              \
                      const int* descu, T* vt, const int* ivt, const int* jvt, const int* descvt, T* work,    \
                      const int* lwork, int* info);                                                        \
    void p##X##gels_(const char* t, const int* m, const int* n, const int* nrhs, T* a, const int* ia,        \
                     const int* ja, const int* desca, T* b, const int* ib, const int* jb, const int* descb,   \
                     T* work, const int* lwork, int* info);
SLATE_AMD_PDECL2(s, float)
SLATE_AMD_PDECL2(d, double)
#undef SLATE_AMD_PDECL2
void pdsgesv_(const int* n, const int* nrhs, double* a, const int* ia, const int* ja, const int* desca, int* ipiv,
              double* b, const int* ib, const int* jb, const int* descb, double* x, const int* ix, const int* jx,
              const int* descx, int* iter, int* info);
void pzherk_(const char* uplo, const char* tr, const int* n, const int* k, const double* alpha, const double* a,
             const int* ia, const int* ja, const int* desca, const double* beta, double* c, const int* ic,
             const int* jc, const int* descc);
void pzher2k_(const char* uplo, const char* tr, const int* n, const int* k, const double* alpha, const double* a,
              const int* ia, const int* ja, const int* desca, const double* b, const int* ib, const int* jb,
              const int* descb, const double* beta, double* c, const int* ic, const int* jc, const int* descc);
void pzhemm_(const char* side, const char* uplo, const int* m, const int* n, const double* alpha, const double* a,
             const int* ia, const int* ja, const int* desca, const double* b, const int* ib, const int* jb,
             const int* descb, const double* beta, double* c, const int* ic, const int* jc, const int* descc);
double pzlanhe_(const char* norm, const char* uplo, const int* n, const double* a, const int* ia, const int* ja,
                const int* desca, double* work);
void pzheevd_(const char* jobz, const char* uplo, const int* n, double* a, const int* ia, const int* ja,
              const int* desca, double* w, double* z, const int* iz, const int* jz, const int* descz, double* work,
              const int* lwork, double* rwork, const int* lrwork, int* iwork, const int* liwork, int* info);

/* ------------------------------------------------------------------
 * Distributed matrices by opaque handle (SLATE's slate_Matrix_create_* /
 * slate_potrf_* C API, src/c_api/wrappers.cc).  kind: 'G' general,
 * 'L' / 'U' Hermitian with that stored triangle; dtype 's','d','c','z';
 * p x q process grid over all ranks; tiles nb x nb, 2D block-cyclic.
 * The local data of this rank (mloc x nloc, column-major) is exchanged with
 * host memory by get/set_local (device-resident under Target::Devices). */
typedef int64_t slate_amd_matrix_t;
typedef int64_t slate_amd_pivots_t;
slate_amd_matrix_t slate_amd_matrix_create(char kind, char dtype, int64_t m, int64_t n, int64_t nb, int p, int q);
int slate_amd_matrix_destroy(slate_amd_matrix_t A);
int slate_amd_matrix_local_size(slate_amd_matrix_t A, int64_t* mloc, int64_t* nloc);
int slate_amd_matrix_get_local(slate_amd_matrix_t A, void* dst, int64_t ld);
int slate_amd_matrix_set_local(slate_amd_matrix_t A, const void* src, int64_t ld);
/* kind 0: uniform random, 1: Hermitian positive definite, 2: normal */
int slate_amd_matrix_generate(slate_amd_matrix_t A, int kind, int64_t seed);
slate_amd_pivots_t slate_amd_pivots_create(void);
int slate_amd_pivots_destroy(slate_amd_pivots_t piv);
double slate_amd_norm(char norm, slate_amd_matrix_t A);
int slate_amd_gemm(double alpha, slate_amd_matrix_t A, slate_amd_matrix_t B, double beta, slate_amd_matrix_t C);
int slate_amd_potrf(slate_amd_matrix_t A);
int slate_amd_posv(slate_amd_matrix_t A, slate_amd_matrix_t B);
int slate_amd_getrf(slate_amd_matrix_t A, slate_amd_pivots_t piv);
int slate_amd_getrs(slate_amd_matrix_t A, slate_amd_pivots_t piv, slate_amd_matrix_t B);
int slate_amd_gesv(slate_amd_matrix_t A, slate_amd_pivots_t piv, slate_amd_matrix_t B);
int slate_amd_gels(slate_amd_matrix_t A, slate_amd_matrix_t BX);
int slate_amd_heev(slate_amd_matrix_t A, double* w, slate_amd_matrix_t Z);

/* Options applied to every later handle call (SLATE's per-call Options map,
 * include/slate/types.hh:32-81): name as in slate::Option ("Lookahead",
 * "MethodLU", "Target", "InnerBlocking", "MaxIterations", ...), value as
 * text ("2", "CALU", "devices", "true"). */
int slate_amd_set_option(const char* name, const char* value);
int slate_amd_clear_options(void);
/* Views sharing the parent's storage: tiles [i1, i2] x [j1, j2] (inclusive,
 * as slate::Matrix::sub), and the transposed ('T') / conjugate-transposed
 * ('C') view.  Destroy views like matrices (the storage stays alive while
 * any handle refers to it). */
slate_amd_matrix_t slate_amd_matrix_sub(slate_amd_matrix_t A, int64_t i1, int64_t i2, int64_t j1, int64_t j2);
slate_amd_matrix_t slate_amd_matrix_op(slate_amd_matrix_t A, char op);
int slate_amd_matrix_dims(slate_amd_matrix_t A, int64_t* m, int64_t* n);
int slate_amd_matrix_tiles(slate_amd_matrix_t A, int64_t* mt, int64_t* nt);
typedef int64_t slate_amd_tfactors_t;      /* QR/LQ block-reflector factors */
slate_amd_tfactors_t slate_amd_tfactors_create(void);
int slate_amd_tfactors_destroy(slate_amd_tfactors_t T);
/* BLAS-3 (real scalars; complex matrices accept real alpha/beta).  A of
 * trsm/trmm is read as triangular (uplo, diag 'N'/'U'); A of hemm and C of
 * herk/her2k as Hermitian (their handle's stored triangle; general handles
 * as Lower). */
int slate_amd_trsm(char side, char uplo, char diag, double alpha, slate_amd_matrix_t A, slate_amd_matrix_t B);
int slate_amd_trmm(char side, char uplo, char diag, double alpha, slate_amd_matrix_t A, slate_amd_matrix_t B);
int slate_amd_herk(double alpha, slate_amd_matrix_t A, double beta, slate_amd_matrix_t C);
int slate_amd_her2k(double alpha, slate_amd_matrix_t A, slate_amd_matrix_t B, double beta, slate_amd_matrix_t C);
int slate_amd_hemm(char side, double alpha, slate_amd_matrix_t A, slate_amd_matrix_t B, double beta,
                   slate_amd_matrix_t C);
/* factorizations, solves, inverses */
int slate_amd_potrs(slate_amd_matrix_t A, slate_amd_matrix_t B);
int slate_amd_potri(slate_amd_matrix_t A);
int slate_amd_trtri(char uplo, char diag, slate_amd_matrix_t A);
int slate_amd_getri(slate_amd_matrix_t A, slate_amd_pivots_t piv);
int slate_amd_geqrf(slate_amd_matrix_t A, slate_amd_tfactors_t T);
int slate_amd_gelqf(slate_amd_matrix_t A, slate_amd_tfactors_t T);
int slate_amd_unmqr(char side, char op, slate_amd_matrix_t A, slate_amd_tfactors_t T, slate_amd_matrix_t C);
int slate_amd_unmlq(char side, char op, slate_amd_matrix_t A, slate_amd_tfactors_t T, slate_amd_matrix_t C);
int slate_amd_gels_t(slate_amd_matrix_t A, slate_amd_tfactors_t T, slate_amd_matrix_t BX);
int slate_amd_hesv(slate_amd_matrix_t A, slate_amd_matrix_t B);
int slate_amd_gesv_mixed(slate_amd_matrix_t A, slate_amd_pivots_t piv, slate_amd_matrix_t B, slate_amd_matrix_t X,
                         int64_t* iter);
int slate_amd_gesv_mixed_gmres(slate_amd_matrix_t A, slate_amd_pivots_t piv, slate_amd_matrix_t B,
                               slate_amd_matrix_t X, int64_t* iter);
int slate_amd_posv_mixed(slate_amd_matrix_t A, slate_amd_matrix_t B, slate_amd_matrix_t X, int64_t* iter);
int slate_amd_posv_mixed_gmres(slate_amd_matrix_t A, slate_amd_matrix_t B, slate_amd_matrix_t X, int64_t* iter);
int slate_amd_gesv_rbt(slate_amd_matrix_t A, slate_amd_matrix_t B);
int slate_amd_gesv_nopiv(slate_amd_matrix_t A, slate_amd_matrix_t B);
/* spectra (s, w: host arrays of min(m, n) / n reals) */
int slate_amd_svd_vals(slate_amd_matrix_t A, double* s);
int slate_amd_hegv(int64_t itype, slate_amd_matrix_t A, slate_amd_matrix_t B, double* w, slate_amd_matrix_t Z);
/* auxiliary */
int slate_amd_add(double alpha, slate_amd_matrix_t A, double beta, slate_amd_matrix_t B);
int slate_amd_copy(slate_amd_matrix_t A, slate_amd_matrix_t B);
int slate_amd_scale(double numer, double denom, slate_amd_matrix_t A);
int slate_amd_set(double offdiag, double diag, slate_amd_matrix_t A);
double slate_amd_gecondest(char norm, slate_amd_matrix_t A, slate_amd_pivots_t piv, double anorm);
double slate_amd_pocondest(char norm, slate_amd_matrix_t A, double anorm);

#ifdef __cplusplus
}
#endif
#endif
