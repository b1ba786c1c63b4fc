/* ScaLAPACK / LAPACK symbols of libslate_amd_native.so from plain C: no
 * Python, no MPI.  BLACS grid over the native runtime's ranks (torchrun-style
 * RANK / WORLD_SIZE env), local block-cyclic arrays, then pdpotrf_ +
 * pdpotrs_, pdgesv_, pdgetrf_ + pdgetrs_, pzgesv_, pdgemm_, pdlange_ and
 * the LAPACK-style slate_dgetrf_ / slate_dgetrs_.  Each rank checks its own
 * part of the solution against the known x and prints
 * "check r<rank> <name> <value>".
 *
 *   ./ex_native_scalapack [PxQ]
 * (reference: scalapack_api/example_pdgetrf.c exercises the same interface) */
#include <complex.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

void Cblacs_pinfo(int* mypnum, int* nprocs);
void Cblacs_get(int ctxt, int what, int* val);
void Cblacs_gridinit(int* ctxt, const char* order, int nprow, int npcol);
void Cblacs_gridinfo(int ctxt, int* nprow, int* npcol, int* myrow, int* mycol);
void Cblacs_gridexit(int ctxt);
int numroc_(const int* n, const int* nb, const int* iproc, const int* isrcproc, const int* nprocs);
void descinit_(int* desc, const int* m, const int* n, const int* mb, const int* nb, const int* irsrc,
               const int* icsrc, const int* ictxt, const int* lld, int* info);
void pdpotrf_(const char* uplo, const int* n, double* a, const int* ia, const int* ja, const int* desca, int* info);
void pdpotrs_(const char* uplo, const int* n, const int* nrhs, const double* a, const int* ia, const int* ja,
              const int* desca, double* b, const int* ib, const int* jb, const int* descb, int* info);
void pdgesv_(const int* n, const int* nrhs, double* a, const int* ia, const int* ja, const int* desca, int* ipiv,
             double* b, const int* ib, const int* jb, const int* descb, int* info);
void pdgetrf_(const int* m, const int* n, double* a, const int* ia, const int* ja, const int* desca, int* ipiv,
              int* info);
void pdgetrs_(const char* trans, const int* n, const int* nrhs, const double* a, const int* ia, const int* ja,
              const int* desca, const int* ipiv, double* b, const int* ib, const int* jb, const int* descb,
              int* info);
void pzgesv_(const int* n, const int* nrhs, double complex* a, const int* ia, const int* ja, const int* desca,
             int* ipiv, double complex* b, const int* ib, const int* jb, const int* descb, int* info);
void pdgemm_(const char* ta, const char* tb, const int* m, const int* n, const int* k, const double* alpha,
             const double* a, const int* ia, const int* ja, const int* desca, const double* b, const int* ib,
             const int* jb, const int* descb, const double* beta, double* c, const int* ic, const int* jc,
             const int* descc);
double pdlange_(const char* norm, const int* m, const int* n, const double* a, const int* ia, const int* ja,
                const int* desca, double* work);
void slate_dgetrf_(const int64_t* m, const int64_t* n, double* a, const int64_t* lda, int64_t* ipiv, int64_t* info);
void slate_dgetrs_(const char* trans, const int64_t* n, const int64_t* nrhs, const double* a, const int64_t* lda,
                   const int64_t* ipiv, double* b, const int64_t* ldb, int64_t* info);
const char* slate_amd_last_error(void);
void pdsgesv_(const int* n, const int* nrhs, double* a, const int* ia, const int* ja, const int* desca, int* ipiv,
              const double* b, const int* ib, const int* jb, const int* descb, double* x, const int* ix,
              const int* jx, const int* descx, int* iter, int* info);
void pdsyrk_(const char* uplo, const char* trans, const int* n, const int* k, const double* alpha, const double* a,
             const int* ia, const int* ja, const int* desca, const double* beta, double* c, const int* ic,
             const int* jc, const int* descc);
void pdtrmm_(const char* side, const char* uplo, const char* ta, const char* diag, const int* m, const int* n,
             const double* alpha, const double* a, const int* ia, const int* ja, const int* desca, double* b,
             const int* ib, const int* jb, const int* descb);
void pdpotri_(const char* uplo, const int* n, double* a, const int* ia, const int* ja, const int* desca, int* info);
void pdgetri_(const int* n, double* a, const int* ia, const int* ja, const int* desca, const int* ipiv, double* work,
              const int* lwork, int* iwork, const int* liwork, int* info);
void pdsymm_(const char* side, const char* uplo, const int* m, const int* n, const double* alpha, const double* a,
             const int* ia, const int* ja, const int* desca, const double* b, const int* ib, const int* jb,
             const int* descb, const double* beta, double* c, const int* ic, const int* jc, const int* descc);
void pdlaset_(const char* uplo, const int* m, const int* n, const double* alpha, const double* beta, double* a,
              const int* ia, const int* ja, const int* desca);
void pdlacpy_(const char* uplo, const int* m, const int* n, const double* a, const int* ia, const int* ja,
              const int* desca, double* b, const int* ib, const int* jb, const int* descb);
void pdgeadd_(const char* trans, const int* m, const int* n, const double* alpha, const double* a, const int* ia,
              const int* ja, const int* desca, const double* beta, double* c, const int* ic, const int* jc,
              const int* descc);
void pztrsm_(const char* side, const char* uplo, const char* ta, const char* diag, const int* m, const int* n,
             const double complex* alpha, const double complex* a, const int* ia, const int* ja, const int* desca,
             double complex* b, const int* ib, const int* jb, const int* descb);
void pdtrsm_(const char* side, const char* uplo, const char* ta, const char* diag, const int* m, const int* n,
             const double* alpha, const double* a, const int* ia, const int* ja, const int* desca, double* b,
             const int* ib, const int* jb, const int* descb);
void pdgecon_(const char* norm, const int* n, const double* a, const int* ia, const int* ja, const int* desca,
              const double* anorm, double* rcond, double* work, const int* lwork, int* iwork, const int* liwork,
              int* info);
void pdpocon_(const char* uplo, const int* n, const double* a, const int* ia, const int* ja, const int* desca,
              const double* anorm, double* rcond, double* work, const int* lwork, int* iwork, const int* liwork,
              int* info);
void pdtrcon_(const char* norm, const char* uplo, const char* diag, const int* n, const double* a, const int* ia,
              const int* ja, const int* desca, double* rcond, double* work, const int* lwork, int* iwork,
              const int* liwork, int* info);
double pdlansy_(const char* norm, const char* uplo, const int* n, const double* a, const int* ia, const int* ja,
                const int* desca, double* work);
void pdsyevd_(const char* jobz, const char* uplo, const int* n, double* a, const int* ia, const int* ja,
              const int* desca, double* w, double* z, const int* iz, const int* jz, const int* descz, double* work,
              const int* lwork, int* iwork, const int* liwork, int* info);
void pdgesvd_(const char* jobu, const char* jobvt, const int* m, const int* n, double* a, const int* ia,
              const int* ja, const int* desca, double* s, double* u, const int* iu, const int* ju, const int* descu,
              double* vt, const int* ivt, const int* jvt, const int* descvt, double* work, const int* lwork,
              int* info);
void pdgels_(const char* trans, const int* m, const int* n, const int* nrhs, double* a, const int* ia, const int* ja,
             const int* desca, double* b, const int* ib, const int* jb, const int* descb, double* work,
             const int* lwork, int* info);
void slate_amd_finalize(void);

static int g_rank;
static int l2g(int l, int nb, int p, int pr) { return ((l / nb) * p + pr) * nb + l % nb; }
/* global entries: SPD (sym), general diagonally dominant (gen), solution */
static double sym(int i, int j, int n) { return i == j ? (double)n : 1.0 / (1.0 + abs(i - j)); }
static double gen(int i, int j, int n) { return i == j ? (double)n : sin(0.7 * i + 0.3 * j); }
static double xs(int i, int c) { return cos(0.1 * i + c); }

static void check(const char* what, double v) {
    printf("check r%d %s %.3e\n", g_rank, what, v);
    fflush(stdout);
}

int main(int argc, char** argv) {
    int p = 1, q = 1;
    if (argc > 1) sscanf(argv[1], "%dx%d", &p, &q);
    int me, np, ctxt, nprow, npcol, pr, pc, info, zero = 0, one = 1;
    Cblacs_pinfo(&me, &np);
    g_rank = me;
    if (p * q != np) { fprintf(stderr, "grid %dx%d != %d ranks\n", p, q, np); return 2; }
    Cblacs_get(-1, 0, &ctxt);
    Cblacs_gridinit(&ctxt, "Col", p, q);
    Cblacs_gridinfo(ctxt, &nprow, &npcol, &pr, &pc);
    const int n = 384, nb = 32, nrhs = 3;
    const int mloc = numroc_(&n, &nb, &pr, &zero, &p), nloc = numroc_(&n, &nb, &pc, &zero, &q);
    const int rloc = numroc_(&nrhs, &nb, &pc, &zero, &q);
    int lld = mloc > 1 ? mloc : 1;
    int desca[9], descb[9];
    descinit_(desca, &n, &n, &nb, &nb, &zero, &zero, &ctxt, &lld, &info);
    descinit_(descb, &n, &nrhs, &nb, &nb, &zero, &zero, &ctxt, &lld, &info);
    double* a = malloc(sizeof(double) * lld * (nloc > 0 ? nloc : 1));
    double* b = malloc(sizeof(double) * lld * (rloc > 0 ? rloc : 1));
    int* ipiv = malloc(sizeof(int) * (mloc + nb));

#define FILL_A(f)                                                                                  \
    for (int lj = 0; lj < nloc; ++lj)                                                              \
        for (int li = 0; li < mloc; ++li) a[li + lj * lld] = f(l2g(li, nb, p, pr), l2g(lj, nb, q, pc), n);
#define FILL_B(f)                                                                                  \
    for (int lc = 0; lc < rloc; ++lc)                                                              \
        for (int li = 0; li < mloc; ++li) {                                                        \
            const int gi = l2g(li, nb, p, pr), c = l2g(lc, nb, q, pc);                             \
            double s = 0;                                                                          \
            for (int j = 0; j < n; ++j) s += f(gi, j, n) * xs(j, c);                               \
            b[li + lc * lld] = s;                                                                  \
        }
#define ERR_B()                                                                                    \
    ({                                                                                             \
        double e = 0, w = 0;                                                                       \
        for (int lc = 0; lc < rloc; ++lc)                                                          \
            for (int li = 0; li < mloc; ++li) {                                                    \
                const double t = xs(l2g(li, nb, p, pr), l2g(lc, nb, q, pc));                       \
                e += (b[li + lc * lld] - t) * (b[li + lc * lld] - t);                              \
                w += t * t;                                                                        \
            }                                                                                      \
        w > 0 ? sqrt(e / w) : sqrt(e);                                                             \
    })

    /* Cholesky + solve */
    FILL_A(sym);
    FILL_B(sym);
    pdpotrf_("L", &n, a, &one, &one, desca, &info);
    if (info) printf("pdpotrf info %d (%s)\n", info, slate_amd_last_error());
    pdpotrs_("L", &n, &nrhs, a, &one, &one, desca, b, &one, &one, descb, &info);
    check(info ? "pdpotrs-FAILED" : "pdpotrs", ERR_B());
    /* upper storage */
    FILL_A(sym);
    FILL_B(sym);
    pdpotrf_("U", &n, a, &one, &one, desca, &info);
    pdpotrs_("U", &n, &nrhs, a, &one, &one, desca, b, &one, &one, descb, &info);
    check(info ? "pdpotrs_upper-FAILED" : "pdpotrs_upper", ERR_B());

    /* aux: pdlaset_ (0.5 off the diagonal, 3 on it), pdlacpy_, pdgeadd_ (C = 2 A - C = A) */
    {
        const double h = 0.5, three = 3.0, two = 2.0, m1 = -1.0;
        double* c2 = calloc((size_t)lld * (nloc > 0 ? nloc : 1), sizeof(double));
        pdlaset_("G", &n, &n, &h, &three, a, &one, &one, desca);
        pdlacpy_("G", &n, &n, a, &one, &one, desca, c2, &one, &one, desca);
        pdgeadd_("N", &n, &n, &two, a, &one, &one, desca, &m1, c2, &one, &one, desca);
        double ae = 0;
        for (int lj = 0; lj < nloc; ++lj)
            for (int li = 0; li < mloc; ++li) {
                const double want = l2g(li, nb, p, pr) == l2g(lj, nb, q, pc) ? 3.0 : 0.5;
                ae = fmax(ae, fabs(c2[li + lj * lld] - want));
            }
        check("pdlaset_lacpy_geadd", ae);
        free(c2);
    }

    /* inverses: x = A^-1 (A x) through pdsymm_ / pdgemm_ */
    {
        double* t = calloc((size_t)lld * (rloc > 0 ? rloc : 1), sizeof(double));
        const double a1 = 1.0, b0 = 0.0;
        int lw = -1, liw = -1;
        double wq;
        int iwq;
        FILL_A(sym);
        FILL_B(sym);
        pdpotrf_("L", &n, a, &one, &one, desca, &info);
        pdpotri_("L", &n, a, &one, &one, desca, &info);
        pdsymm_("L", "L", &n, &nrhs, &a1, a, &one, &one, desca, b, &one, &one, descb, &b0, t, &one, &one, descb);
        memcpy(b, t, sizeof(double) * lld * (rloc > 0 ? rloc : 1));
        check(info ? "pdpotri-FAILED" : "pdpotri", ERR_B());
        FILL_A(gen);
        FILL_B(gen);
        pdgetrf_(&n, &n, a, &one, &one, desca, ipiv, &info);
        pdgetri_(&n, a, &one, &one, desca, ipiv, &wq, &lw, &iwq, &liw, &info);   /* workspace query */
        lw = 1;
        liw = 1;
        pdgetri_(&n, a, &one, &one, desca, ipiv, &wq, &lw, &iwq, &liw, &info);
        pdgemm_("N", "N", &n, &nrhs, &n, &a1, a, &one, &one, desca, b, &one, &one, descb, &b0, t, &one, &one, descb);
        memcpy(b, t, sizeof(double) * lld * (rloc > 0 ? rloc : 1));
        check(info ? "pdgetri-FAILED" : "pdgetri", ERR_B());
        free(t);
    }

    /* condition estimates against the exact 1-norm condition number from the
     * inverse: the estimate of ||A^-1||_1 is a lower bound, in practice within
     * a factor 3 (LAPACK lacn2) -- pass if 1 <= rcond_est / rcond <= 3 */
    {
        int lw = 1, liw = 1, iwq;
        double wq, rc = 0, rc2 = 0;
        FILL_A(gen);
        const double an = pdlange_("1", &n, &n, a, &one, &one, desca, NULL);
        pdgetrf_(&n, &n, a, &one, &one, desca, ipiv, &info);
        pdgecon_("1", &n, a, &one, &one, desca, &an, &rc, &wq, &lw, &iwq, &liw, &info);
        pdgetri_(&n, a, &one, &one, desca, ipiv, &wq, &lw, &iwq, &liw, &info);
        double ratio = rc * an * pdlange_("1", &n, &n, a, &one, &one, desca, NULL);
        check("pdgecon", (ratio >= 1.0 - 1e-12 && ratio <= 3.0) ? 0.0 : ratio);
        FILL_A(sym);
        const double sn_ = pdlange_("1", &n, &n, a, &one, &one, desca, NULL);
        pdpotrf_("L", &n, a, &one, &one, desca, &info);
        pdpocon_("L", &n, a, &one, &one, desca, &sn_, &rc2, &wq, &lw, &iwq, &liw, &info);
        pdpotri_("L", &n, a, &one, &one, desca, &info);
        ratio = rc2 * sn_ * pdlansy_("1", "L", &n, a, &one, &one, desca, NULL);
        check("pdpocon", (ratio >= 1.0 - 1e-12 && ratio <= 3.0) ? 0.0 : ratio);
        FILL_A(gen);
        double rt = 0;
        pdtrcon_("1", "U", "N", &n, a, &one, &one, desca, &rt, &wq, &lw, &iwq, &liw, &info);
        check("pdtrcon", (rt > 0.0 && rt <= 1.0 && info == 0) ? 0.0 : 1.0 + rt);
    }

    /* pdsyevd_: A Z = Z diag(w) (the product by pdgemm_), W ascending on every rank */
    {
        double* z = malloc(sizeof(double) * lld * (nloc > 0 ? nloc : 1));
        double* az = malloc(sizeof(double) * lld * (nloc > 0 ? nloc : 1));
        double* w = malloc(sizeof(double) * n);
        const double a1 = 1.0, b0 = 0.0;
        int lw = -1, liw = -1, iwq;
        double wq;
        FILL_A(gen);
        for (int lj = 0; lj < nloc; ++lj)            /* symmetric: the lower triangle of gen mirrored */
            for (int li = 0; li < mloc; ++li) {
                const int gi = l2g(li, nb, p, pr), gj = l2g(lj, nb, q, pc);
                a[li + lj * lld] = gi >= gj ? gen(gi, gj, n) : gen(gj, gi, n);
            }
        pdsyevd_("V", "L", &n, a, &one, &one, desca, w, z, &one, &one, desca, &wq, &lw, &iwq, &liw, &info);
        lw = liw = 1;
        pdsyevd_("V", "L", &n, a, &one, &one, desca, w, z, &one, &one, desca, &wq, &lw, &iwq, &liw, &info);
        pdgemm_("N", "N", &n, &n, &n, &a1, a, &one, &one, desca, z, &one, &one, desca, &b0, az, &one, &one, desca);
        double ee = 0, an = pdlange_("F", &n, &n, a, &one, &one, desca, NULL);
        int sorted = 1;
        for (int i = 1; i < n; ++i) sorted = sorted && w[i - 1] <= w[i];
        for (int lj = 0; lj < nloc; ++lj)
            for (int li = 0; li < mloc; ++li) {
                const double r = az[li + lj * lld] - z[li + lj * lld] * w[l2g(lj, nb, q, pc)];
                ee += r * r;
            }
        check(info || !sorted ? "pdsyevd-FAILED" : "pdsyevd", sqrt(ee) / (an * n));
        free(z); free(az); free(w);
    }

    /* pdgesvd_: A = U diag(s) VT on the whole n x n matrix (A U-check via pdgemm_) */
    {
        double* u = malloc(sizeof(double) * lld * (nloc > 0 ? nloc : 1));
        double* vt = malloc(sizeof(double) * lld * (nloc > 0 ? nloc : 1));
        double* us = malloc(sizeof(double) * lld * (nloc > 0 ? nloc : 1));
        double* sv = malloc(sizeof(double) * n);
        const double a1 = 1.0, b0 = 0.0;
        int lw = -1;
        double wq;
        FILL_A(gen);
        pdgesvd_("V", "V", &n, &n, a, &one, &one, desca, sv, u, &one, &one, desca, vt, &one, &one, desca, &wq, &lw,
                 &info);
        lw = 1;
        pdgesvd_("V", "V", &n, &n, a, &one, &one, desca, sv, u, &one, &one, desca, vt, &one, &one, desca, &wq, &lw,
                 &info);
        for (int lj = 0; lj < nloc; ++lj)
            for (int li = 0; li < mloc; ++li) us[li + lj * lld] = u[li + lj * lld] * sv[l2g(lj, nb, q, pc)];
        pdgemm_("N", "N", &n, &n, &n, &a1, us, &one, &one, desca, vt, &one, &one, desca, &b0, a, &one, &one, desca);
        double ee = 0, ww = 0;
        int desc_ok = 1;
        for (int i = 1; i < n; ++i) desc_ok = desc_ok && sv[i - 1] >= sv[i];
        for (int lj = 0; lj < nloc; ++lj)
            for (int li = 0; li < mloc; ++li) {
                const double t = gen(l2g(li, nb, p, pr), l2g(lj, nb, q, pc), n);
                ee += (a[li + lj * lld] - t) * (a[li + lj * lld] - t);
                ww += t * t;
            }
        check(info || !desc_ok ? "pdgesvd-FAILED" : "pdgesvd", sqrt(ee / ww));
        free(u); free(vt); free(us); free(sv);
    }

    /* LU */
    FILL_A(gen);
    FILL_B(gen);
    pdgesv_(&n, &nrhs, a, &one, &one, desca, ipiv, b, &one, &one, descb, &info);
    if (info) printf("pdgesv info %d (%s)\n", info, slate_amd_last_error());
    check(info ? "pdgesv-FAILED" : "pdgesv", ERR_B());
    FILL_A(gen);
    FILL_B(gen);
    pdgetrf_(&n, &n, a, &one, &one, desca, ipiv, &info);
    pdgetrs_("N", &n, &nrhs, a, &one, &one, desca, ipiv, b, &one, &one, descb, &info);
    check(info ? "pdgetrs-FAILED" : "pdgetrs", ERR_B());
    /* mixed precision: single-precision LU, double refinement (X = A^-1 B, B kept) */
    {
        FILL_A(gen);
        FILL_B(gen);
        double* x = malloc(sizeof(double) * lld * (rloc > 0 ? rloc : 1));
        int iter = -100;
        pdsgesv_(&n, &nrhs, a, &one, &one, desca, ipiv, b, &one, &one, descb, x, &one, &one, descb, &iter, &info);
        if (info) printf("pdsgesv info %d (%s)\n", info, slate_amd_last_error());
        memcpy(b, x, sizeof(double) * lld * (rloc > 0 ? rloc : 1));
        check(info || iter < 0 ? "pdsgesv-FAILED" : "pdsgesv", ERR_B());
        free(x);
    }

    /* least squares through QR (TSQR panels when p > 1): a consistent square system */
    {
        int lw = -1;
        double wq;
        FILL_A(gen);
        FILL_B(gen);
        pdgels_("N", &n, &n, &nrhs, a, &one, &one, desca, b, &one, &one, descb, &wq, &lw, &info);
        lw = 1;
        pdgels_("N", &n, &n, &nrhs, a, &one, &one, desca, b, &one, &one, descb, &wq, &lw, &info);
        check(info ? "pdgels-FAILED" : "pdgels", ERR_B());
    }

    /* norm and gemm: C = A^T A (one column block checked) */
    FILL_A(gen);
    double nrm = pdlange_("F", &n, &n, a, &one, &one, desca, NULL), want = 0;
    for (int j = 0; j < n; ++j)
        for (int i = 0; i < n; ++i) want += gen(i, j, n) * gen(i, j, n);
    check("pdlange_fro", fabs(nrm - sqrt(want)) / sqrt(want));
    double* c = calloc((size_t)lld * (nloc > 0 ? nloc : 1), sizeof(double));
    const double alpha = 1.0, beta = 0.0;
    pdgemm_("T", "N", &n, &n, &n, &alpha, a, &one, &one, desca, a, &one, &one, desca, &beta, c, &one, &one, desca);
    double ge = 0, gw = 0;
    for (int lj = 0; lj < nloc; lj += 3)
        for (int li = 0; li < mloc; li += 3) {
            const int gi = l2g(li, nb, p, pr), gj = l2g(lj, nb, q, pc);
            double s = 0;
            for (int k = 0; k < n; ++k) s += gen(k, gi, n) * gen(k, gj, n);
            ge += (c[li + lj * lld] - s) * (c[li + lj * lld] - s);
            gw += s * s;
        }
    check("pdgemm_tn", gw > 0 ? sqrt(ge / gw) : sqrt(ge));

    /* pdsyrk_: C(lower) = 2 A^T A - C; the upper triangle must stay untouched */
    for (int lj = 0; lj < nloc; ++lj)
        for (int li = 0; li < mloc; ++li) c[li + lj * lld] = 1.0;
    {
        const double two = 2.0, m1 = -1.0;
        pdsyrk_("L", "T", &n, &n, &two, a, &one, &one, desca, &m1, c, &one, &one, desca);
        double se = 0, sw = 0;
        for (int lj = 0; lj < nloc; lj += 3)
            for (int li = 0; li < mloc; li += 3) {
                const int gi = l2g(li, nb, p, pr), gj = l2g(lj, nb, q, pc);
                double s = 1.0;
                if (gi >= gj) {
                    s = -1.0;
                    for (int k = 0; k < n; ++k) s += 2.0 * gen(k, gi, n) * gen(k, gj, n);
                }
                se += (c[li + lj * lld] - s) * (c[li + lj * lld] - s);
                sw += s * s;
            }
        check("pdsyrk_lower", sw > 0 ? sqrt(se / sw) : sqrt(se));
    }
    /* pdtrmm_: B = U B (U = the upper triangle of gen, non-unit) */
    FILL_A(gen);
    for (int lc = 0; lc < rloc; ++lc)
        for (int li = 0; li < mloc; ++li) b[li + lc * lld] = xs(l2g(li, nb, p, pr), l2g(lc, nb, q, pc));
    {
        const double a1 = 1.0;
        pdtrmm_("L", "U", "N", "N", &n, &nrhs, &a1, a, &one, &one, desca, b, &one, &one, descb);
        double te = 0, tw = 0;
        for (int lc = 0; lc < rloc; ++lc)
            for (int li = 0; li < mloc; ++li) {
                const int gi = l2g(li, nb, p, pr), cc = l2g(lc, nb, q, pc);
                double s = 0;
                for (int j = gi; j < n; ++j) s += gen(gi, j, n) * xs(j, cc);
                te += (b[li + lc * lld] - s) * (b[li + lc * lld] - s);
                tw += s * s;
            }
        check("pdtrmm_lun", tw > 0 ? sqrt(te / tw) : sqrt(te));
    }

    /* sub-matrix operands (ia = ja = nb + 1, size not a multiple of nb;
     * reference scalapack_api/scalapack_slate.hh:81-120): the result must
     * match the sub-problem and nothing outside the sub-matrix may change */
    {
        const int o = nb + 1, ms = n - nb - 21, o0 = o - 1;
        const double a1 = 1.0, b0 = 0.0;
        double* c3 = malloc(sizeof(double) * lld * (nloc > 0 ? nloc : 1));
        FILL_A(gen);
        for (int k = 0; k < lld * nloc; ++k) c3[k] = 7.0;
        pdgemm_("T", "N", &ms, &ms, &ms, &a1, a, &o, &o, desca, a, &o, &o, desca, &b0, c3, &o, &o, desca);
        double se = 0, sw = 0, out = 0;
        for (int lj = 0; lj < nloc; ++lj)
            for (int li = 0; li < mloc; ++li) {
                const int gi = l2g(li, nb, p, pr), gj = l2g(lj, nb, q, pc);
                const double v = c3[li + lj * lld];
                if (gi >= o0 && gi < o0 + ms && gj >= o0 && gj < o0 + ms) {
                    if ((li + lj) % 5) continue;
                    double t = 0;
                    for (int k = 0; k < ms; ++k) t += gen(o0 + k, gi, n) * gen(o0 + k, gj, n);
                    se += (v - t) * (v - t);
                    sw += t * t;
                } else {
                    out = fmax(out, fabs(v - 7.0));
                }
            }
        check("pdgemm_sub", (sw > 0 ? sqrt(se / sw) : sqrt(se)) + out);
        /* pdpotrf_ + pdpotrs_ on A(o:o+ms-1, o:o+ms-1), B(o:o+ms-1, 1:nrhs) */
        FILL_A(sym);
        for (int lc = 0; lc < rloc; ++lc)
            for (int li = 0; li < mloc; ++li) {
                const int gi = l2g(li, nb, p, pr), cc = l2g(lc, nb, q, pc);
                double t = -5.0;                       /* rows outside the sub-matrix: sentinel */
                if (gi >= o0 && gi < o0 + ms) {
                    t = 0;
                    for (int j = 0; j < ms; ++j) t += sym(gi, o0 + j, n) * xs(o0 + j, cc);
                }
                b[li + lc * lld] = t;
            }
        pdpotrf_("L", &ms, a, &o, &o, desca, &info);
        int one_ = 1;
        pdpotrs_("L", &ms, &nrhs, a, &o, &o, desca, b, &o, &one_, descb, &info);
        double pe = 0, pw = 0, pout = 0;
        for (int lc = 0; lc < rloc; ++lc)
            for (int li = 0; li < mloc; ++li) {
                const int gi = l2g(li, nb, p, pr), cc = l2g(lc, nb, q, pc);
                if (gi >= o0 && gi < o0 + ms) {
                    const double t = xs(gi, cc);
                    pe += (b[li + lc * lld] - t) * (b[li + lc * lld] - t);
                    pw += t * t;
                } else {
                    pout = fmax(pout, fabs(b[li + lc * lld] + 5.0));
                }
            }
        /* the strict upper triangle and everything outside the sub-matrix: untouched */
        for (int lj = 0; lj < nloc; ++lj)
            for (int li = 0; li < mloc; ++li) {
                const int gi = l2g(li, nb, p, pr), gj = l2g(lj, nb, q, pc);
                const int inside = gi >= o0 && gi < o0 + ms && gj >= o0 && gj < o0 + ms;
                if (!inside || gi < gj) pout = fmax(pout, fabs(a[li + lj * lld] - sym(gi, gj, n)));
            }
        check(info ? "pdpotrs_sub-FAILED" : "pdpotrs_sub", (pw > 0 ? sqrt(pe / pw) : sqrt(pe)) + pout);
        /* pdgetrf_ + pdgetrs_ on the same sub-matrix (ipiv tied to A) */
        FILL_A(gen);
        for (int lc = 0; lc < rloc; ++lc)
            for (int li = 0; li < mloc; ++li) {
                const int gi = l2g(li, nb, p, pr), cc = l2g(lc, nb, q, pc);
                double t = -5.0;
                if (gi >= o0 && gi < o0 + ms) {
                    t = 0;
                    for (int j = 0; j < ms; ++j) t += gen(gi, o0 + j, n) * xs(o0 + j, cc);
                }
                b[li + lc * lld] = t;
            }
        pdgetrf_(&ms, &ms, a, &o, &o, desca, ipiv, &info);
        pdgetrs_("N", &ms, &nrhs, a, &o, &o, desca, ipiv, b, &o, &one_, descb, &info);
        pe = pw = pout = 0;
        for (int lc = 0; lc < rloc; ++lc)
            for (int li = 0; li < mloc; ++li) {
                const int gi = l2g(li, nb, p, pr), cc = l2g(lc, nb, q, pc);
                if (gi >= o0 && gi < o0 + ms) {
                    const double t = xs(gi, cc);
                    pe += (b[li + lc * lld] - t) * (b[li + lc * lld] - t);
                    pw += t * t;
                } else {
                    pout = fmax(pout, fabs(b[li + lc * lld] + 5.0));
                }
            }
        check(info ? "pdgetrs_sub-FAILED" : "pdgetrs_sub", (pw > 0 ? sqrt(pe / pw) : sqrt(pe)) + pout);
        free(c3);
    }

    /* pdtrsm_ Right: X U = B (U = the upper triangle of gen) on an nrhs x n
     * right-hand side stored in the columns of an n x n array */
    {
        const double a1 = 1.0;
        const int nr = 40;                 /* rows of X */
        double* xb = malloc(sizeof(double) * lld * (nloc > 0 ? nloc : 1));
        FILL_A(gen);
        for (int lj = 0; lj < nloc; ++lj)
            for (int li = 0; li < mloc; ++li) {
                const int gi = l2g(li, nb, p, pr), gj = l2g(lj, nb, q, pc);
                double t = 0;
                if (gi < nr)
                    for (int k = 0; k <= gj; ++k) t += xs(k, gi) * gen(k, gj, n);
                xb[li + lj * lld] = t;
            }
        pdtrsm_("R", "U", "N", "N", &nr, &n, &a1, a, &one, &one, desca, xb, &one, &one, desca);
        double te = 0, tw = 0;
        for (int lj = 0; lj < nloc; ++lj)
            for (int li = 0; li < mloc; ++li) {
                const int gi = l2g(li, nb, p, pr), gj = l2g(lj, nb, q, pc);
                if (gi >= nr) continue;
                const double t = xs(gj, gi);
                te += (xb[li + lj * lld] - t) * (xb[li + lj * lld] - t);
                tw += t * t;
            }
        check("pdtrsm_right", tw > 0 ? sqrt(te / tw) : sqrt(te));
        free(xb);
    }

    /* complex LU */
    double complex* za = malloc(sizeof(double complex) * lld * (nloc > 0 ? nloc : 1));
    double complex* zb = malloc(sizeof(double complex) * lld * (rloc > 0 ? rloc : 1));
    for (int lj = 0; lj < nloc; ++lj)
        for (int li = 0; li < mloc; ++li) {
            const int gi = l2g(li, nb, p, pr), gj = l2g(lj, nb, q, pc);
            za[li + lj * lld] = gen(gi, gj, n) + I * 0.5 * gen(gj, gi, n);
        }
    for (int lc = 0; lc < rloc; ++lc)
        for (int li = 0; li < mloc; ++li) {
            const int gi = l2g(li, nb, p, pr), cc = l2g(lc, nb, q, pc);
            double complex s = 0;
            for (int j = 0; j < n; ++j) s += (gen(gi, j, n) + I * 0.5 * gen(j, gi, n)) * (xs(j, cc) + I * xs(j, cc + 7));
            zb[li + lc * lld] = s;
        }
    pzgesv_(&n, &nrhs, za, &one, &one, desca, ipiv, zb, &one, &one, descb, &info);
    double ze = 0, zw = 0;
    for (int lc = 0; lc < rloc; ++lc)
        for (int li = 0; li < mloc; ++li) {
            const int gi = l2g(li, nb, p, pr), cc = l2g(lc, nb, q, pc);
            const double complex t = xs(gi, cc) + I * xs(gi, cc + 7);
            ze += cabs(zb[li + lc * lld] - t) * cabs(zb[li + lc * lld] - t);
            zw += cabs(t) * cabs(t);
        }
    check(info ? "pzgesv-FAILED" : "pzgesv", zw > 0 ? sqrt(ze / zw) : sqrt(ze));
    /* pztrsm_ TRANSA = 'T' (no conjugation): L^T X = B, L = the lower triangle of za */
    for (int lj = 0; lj < nloc; ++lj)
        for (int li = 0; li < mloc; ++li) {
            const int gi = l2g(li, nb, p, pr), gj = l2g(lj, nb, q, pc);
            za[li + lj * lld] = gen(gi, gj, n) + I * 0.5 * gen(gj, gi, n);
        }
    for (int lc = 0; lc < rloc; ++lc)
        for (int li = 0; li < mloc; ++li) {
            const int gi = l2g(li, nb, p, pr), cc = l2g(lc, nb, q, pc);
            double complex s = 0;
            for (int k = gi; k < n; ++k)       /* (L^T)(gi, k) = L(k, gi), k >= gi */
                s += (gen(k, gi, n) + I * 0.5 * gen(gi, k, n)) * (xs(k, cc) + I * xs(k, cc + 7));
            zb[li + lc * lld] = s;
        }
    {
        const double complex z1 = 1.0;
        pztrsm_("L", "L", "T", "N", &n, &nrhs, &z1, za, &one, &one, desca, zb, &one, &one, descb);
        ze = zw = 0;
        for (int lc = 0; lc < rloc; ++lc)
            for (int li = 0; li < mloc; ++li) {
                const int gi = l2g(li, nb, p, pr), cc = l2g(lc, nb, q, pc);
                const double complex t = xs(gi, cc) + I * xs(gi, cc + 7);
                ze += cabs(zb[li + lc * lld] - t) * cabs(zb[li + lc * lld] - t);
                zw += cabs(t) * cabs(t);
            }
        check("pztrsm_trans", zw > 0 ? sqrt(ze / zw) : sqrt(ze));
    }

    /* LAPACK-style on the global array (every rank the same) */
    {
        const int64_t N = 256, NR = 1, L = 256;
        double* ga = malloc(sizeof(double) * N * N);
        double* gb = malloc(sizeof(double) * N);
        int64_t* gp = malloc(sizeof(int64_t) * N);
        int64_t inf = 0;
        for (int j = 0; j < N; ++j)
            for (int i = 0; i < N; ++i) ga[i + j * N] = gen(i, j, (int)N);
        for (int i = 0; i < N; ++i) {
            double s = 0;
            for (int j = 0; j < N; ++j) s += gen(i, j, (int)N) * xs(j, 0);
            gb[i] = s;
        }
        slate_dgetrf_(&N, &N, ga, &L, gp, &inf);
        slate_dgetrs_("N", &N, &NR, ga, &L, gp, gb, &L, &inf);
        double e = 0, w = 0;
        for (int i = 0; i < N; ++i) { e += (gb[i] - xs(i, 0)) * (gb[i] - xs(i, 0)); w += xs(i, 0) * xs(i, 0); }
        check(inf ? "slate_dgetrf_-FAILED" : "slate_dgetrf_", sqrt(e / w));
        free(ga); free(gb); free(gp);
    }
    Cblacs_gridexit(ctxt);
    free(a); free(b); free(c); free(za); free(zb); free(ipiv);
    slate_amd_finalize();
    return 0;
}
