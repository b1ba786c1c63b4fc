/* LAPACK-style BLAS-3, inverse and norm symbols of libslate_amd_native.so
 * from plain C (no Python, no MPI): slate_?trmm, ?syrk, ?syr2k, ?symm,
 * ?getri, ?potri, ?lansy, ?lantr (s, d, c, z) and the complex ?herk,
 * ?her2k, ?hemm, ?lanhe -- the reference's lapack_api/lapack_{trmm,syrk,
 * syr2k,symm,getri,potri,lansy,lantr,herk,her2k,hemm,lanhe}.cc.  Every
 * result is compared with a naive triple loop on the host and printed as
 * "check <name> <relative error>".  With several ranks (torchrun-style env)
 * every rank passes the same arrays and gets the same result.
 *
 *   ./ex_native_lapack [n] */
#include <complex.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

int slate_dtrmm(char side, char uplo, char ta, char diag, int64_t m, int64_t n, double alpha, const double* a,
                int64_t lda, double* b, int64_t ldb);
int slate_dsyrk(char uplo, char trans, int64_t n, int64_t k, double alpha, const double* a, int64_t lda, double beta,
                double* c, int64_t ldc);
int slate_dsyr2k(char uplo, char trans, int64_t n, int64_t k, double alpha, const double* a, int64_t lda,
                 const double* b, int64_t ldb, double beta, double* c, int64_t ldc);
int slate_dsymm(char side, char uplo, int64_t m, int64_t n, double alpha, const double* a, int64_t lda,
                const double* b, int64_t ldb, double beta, double* c, int64_t ldc);
int slate_dgetrf(int64_t m, int64_t n, double* a, int64_t lda, int64_t* ipiv);
int slate_dgetri(int64_t n, double* a, int64_t lda, const int64_t* ipiv);
int slate_dpotrf(char uplo, int64_t n, double* a, int64_t lda);
int slate_dpotri(char uplo, int64_t n, double* a, int64_t lda);
double slate_dlansy(char norm, char uplo, int64_t n, const double* a, int64_t lda);
double slate_dlantr(char norm, char uplo, char diag, int64_t m, int64_t n, const double* a, int64_t lda);
int slate_strmm(char side, char uplo, char ta, char diag, int64_t m, int64_t n, float alpha, const float* a,
                int64_t lda, float* b, int64_t ldb);
int slate_ssyrk(char uplo, char trans, int64_t n, int64_t k, float alpha, const float* a, int64_t lda, float beta,
                float* c, int64_t ldc);
int slate_zherk(char uplo, char trans, int64_t n, int64_t k, double alpha, const double* a, int64_t lda, double beta,
                double* c, int64_t ldc);
int slate_zher2k(char uplo, char trans, int64_t n, int64_t k, const double* alpha, const double* a, int64_t lda,
                 const double* b, int64_t ldb, double beta, double* c, int64_t ldc);
int slate_zhemm(char side, char uplo, int64_t m, int64_t n, const double* alpha, const double* a, int64_t lda,
                const double* b, int64_t ldb, const double* beta, double* c, int64_t ldc);
int slate_ztrmm(char side, char uplo, char ta, char diag, int64_t m, int64_t n, const double* alpha, const double* a,
                int64_t lda, double* b, int64_t ldb);
int slate_zgetrf(int64_t m, int64_t n, double* a, int64_t lda, int64_t* ipiv);
int slate_zgetri(int64_t n, double* a, int64_t lda, const int64_t* ipiv);
double slate_zlanhe(char norm, char uplo, int64_t n, const double* a, int64_t lda);
double slate_clantr(char norm, char uplo, char diag, int64_t m, int64_t n, const float* a, int64_t lda);
int slate_dgecon(char norm, int64_t n, const double* a, int64_t lda, double anorm, double* rcond);
int slate_dtrcon(char norm, char uplo, char diag, int64_t n, const double* a, int64_t lda, double* rcond);
void slate_dsyev_(const char* jobz, const char* uplo, const int64_t* n, double* a, const int64_t* lda, double* w,
                  int64_t* info);
const char* slate_amd_last_error(void);

static int g_fail = 0;
static void check(const char* what, double v, double tol) {
    int ok = v == v && v <= tol;
    printf("check %s %.3e%s\n", what, v, ok ? "" : " FAILED");
    if (!ok) g_fail = 1;
}
static double rnd(int i, int j, int s) { return sin(0.37 * i + 0.71 * j + 1.3 * s); }

/* naive C = alpha op(A) op(B) + beta C, double, op 'N' / 'T' */
static void ref_gemm(char ta, char tb, int m, int n, int k, double alpha, const double* a, int lda, const double* b,
                     int ldb, double beta, double* c, int ldc) {
    for (int j = 0; j < n; ++j)
        for (int i = 0; i < m; ++i) {
            double s = 0;
            for (int l = 0; l < k; ++l)
                s += (ta == 'N' ? a[i + l * lda] : a[l + i * lda]) * (tb == 'N' ? b[l + j * ldb] : b[j + l * ldb]);
            c[i + j * ldc] = alpha * s + beta * c[i + j * ldc];
        }
}
static double rel(const double* x, const double* y, int m, int n, int ldx, int ldy, char tri) {
    double e = 0, w = 0;
    for (int j = 0; j < n; ++j)
        for (int i = 0; i < m; ++i) {
            if ((tri == 'L' && i < j) || (tri == 'U' && i > j)) continue;
            double d = x[i + j * ldx] - y[i + j * ldy];
            e += d * d;
            w += y[i + j * ldy] * y[i + j * ldy];
        }
    return w > 0 ? sqrt(e / w) : sqrt(e);
}
static double zrel(const double complex* x, const double complex* y, int m, int n, char tri) {
    double e = 0, w = 0;
    for (int j = 0; j < n; ++j)
        for (int i = 0; i < m; ++i) {
            if ((tri == 'L' && i < j) || (tri == 'U' && i > j)) continue;
            e += pow(cabs(x[i + j * m] - y[i + j * m]), 2);
            w += pow(cabs(y[i + j * m]), 2);
        }
    return w > 0 ? sqrt(e / w) : sqrt(e);
}

int main(int argc, char** argv) {
    const int n = argc > 1 ? atoi(argv[1]) : 200, k = n / 2 + 3;
    const double eps = 1e-12;
    double* A = malloc(sizeof(double) * n * n);
    double* B = malloc(sizeof(double) * n * n);
    double* C = malloc(sizeof(double) * n * n);
    double* R = malloc(sizeof(double) * n * n);
    double* T = malloc(sizeof(double) * n * n);
    int64_t* ipiv = malloc(sizeof(int64_t) * n);
    for (int j = 0; j < n; ++j)
        for (int i = 0; i < n; ++i) {
            A[i + j * n] = rnd(i, j, 1) + (i == j ? n : 0);
            B[i + j * n] = rnd(i, j, 2);
            C[i + j * n] = rnd(i, j, 3);
        }
    /* trmm: B = 0.5 A^T B, A lower non-unit */
    memcpy(R, B, sizeof(double) * n * n);
    memcpy(T, A, sizeof(double) * n * n);
    for (int j = 0; j < n; ++j)
        for (int i = 0; i < j; ++i) T[i + j * n] = 0;
    {
        double* W = calloc((size_t)n * n, sizeof(double));
        ref_gemm('T', 'N', n, n, n, 0.5, T, n, R, n, 0.0, W, n);
        int info = slate_dtrmm('L', 'L', 'T', 'N', n, n, 0.5, A, n, R, n);
        check(info ? "slate_dtrmm-FAILED" : "slate_dtrmm_llt", rel(R, W, n, n, n, n, 'G'), eps);
        /* right side, upper, unit: R = B A_u (A_u: unit upper of A) */
        memcpy(R, B, sizeof(double) * n * n);
        memcpy(T, A, sizeof(double) * n * n);
        for (int j = 0; j < n; ++j)
            for (int i = j; i < n; ++i) T[i + j * n] = i == j ? 1.0 : 0.0;
        ref_gemm('N', 'N', n, n, n, 1.0, R, n, T, n, 0.0, W, n);
        info = slate_dtrmm('R', 'U', 'N', 'U', n, n, 1.0, A, n, R, n);
        check(info ? "slate_dtrmm-FAILED" : "slate_dtrmm_run", rel(R, W, n, n, n, n, 'G'), eps);
        free(W);
    }
    /* syrk: C(lower) = -1 A A^T + 2 C, A n x k */
    memcpy(R, C, sizeof(double) * n * n);
    memcpy(T, C, sizeof(double) * n * n);
    ref_gemm('N', 'T', n, n, k, -1.0, B, n, B, n, 2.0, T, n);
    int info = slate_dsyrk('L', 'N', n, k, -1.0, B, n, 2.0, R, n);
    {
        /* the upper triangle must be untouched */
        double up = 0;
        for (int j = 0; j < n; ++j)
            for (int i = 0; i < j; ++i) up += fabs(R[i + j * n] - C[i + j * n]);
        check(info ? "slate_dsyrk-FAILED" : "slate_dsyrk_ln", rel(R, T, n, n, n, n, 'L') + up, eps);
    }
    /* syr2k: C(upper) = A^T B + B^T A + 0.5 C, A, B k x n */
    memcpy(R, C, sizeof(double) * n * n);
    memcpy(T, C, sizeof(double) * n * n);
    ref_gemm('T', 'N', n, n, k, 1.0, A, n, B, n, 0.5, T, n);
    ref_gemm('T', 'N', n, n, k, 1.0, B, n, A, n, 1.0, T, n);
    info = slate_dsyr2k('U', 'T', n, k, 1.0, A, n, B, n, 0.5, R, n);
    check(info ? "slate_dsyr2k-FAILED" : "slate_dsyr2k_ut", rel(R, T, n, n, n, n, 'U'), eps);
    /* symm: C = A_sym B + C, A from its lower triangle, side L */
    memcpy(T, A, sizeof(double) * n * n);
    for (int j = 0; j < n; ++j)
        for (int i = 0; i < j; ++i) T[i + j * n] = A[j + i * n];
    memcpy(R, C, sizeof(double) * n * n);
    {
        double* W = malloc(sizeof(double) * n * n);
        memcpy(W, C, sizeof(double) * n * n);
        ref_gemm('N', 'N', n, n, n, 1.0, T, n, B, n, 1.0, W, n);
        info = slate_dsymm('L', 'L', n, n, 1.0, A, n, B, n, 1.0, R, n);
        check(info ? "slate_dsymm-FAILED" : "slate_dsymm_ll", rel(R, W, n, n, n, n, 'G'), eps);
        /* getri: A^-1 A = I */
        memcpy(R, A, sizeof(double) * n * n);
        info = slate_dgetrf(n, n, R, n, ipiv);
        int info2 = slate_dgetri(n, R, n, ipiv);
        ref_gemm('N', 'N', n, n, n, 1.0, R, n, A, n, 0.0, W, n);
        double e = 0;
        for (int j = 0; j < n; ++j)
            for (int i = 0; i < n; ++i) e = fmax(e, fabs(W[i + j * n] - (i == j)));
        check(info || info2 ? "slate_dgetri-FAILED" : "slate_dgetri", e, 1e-10);
        /* potri: SPD S = T (symmetric) + n I already diagonally dominant */
        memcpy(R, T, sizeof(double) * n * n);
        info = slate_dpotrf('L', n, R, n);
        info2 = slate_dpotri('L', n, R, n);
        for (int j = 0; j < n; ++j)
            for (int i = 0; i < j; ++i) R[i + j * n] = R[j + i * n];
        ref_gemm('N', 'N', n, n, n, 1.0, R, n, T, n, 0.0, W, n);
        e = 0;
        for (int j = 0; j < n; ++j)
            for (int i = 0; i < n; ++i) e = fmax(e, fabs(W[i + j * n] - (i == j)));
        check(info || info2 ? "slate_dpotri-FAILED" : "slate_dpotri", e, 1e-10);
        free(W);
    }
    /* lansy / lantr */
    {
        double one = 0, fro = 0, mx = 0;
        for (int j = 0; j < n; ++j) {
            double cs = 0;
            for (int i = 0; i < n; ++i) {
                cs += fabs(T[i + j * n]);
                fro += T[i + j * n] * T[i + j * n];
                mx = fmax(mx, fabs(T[i + j * n]));
            }
            one = fmax(one, cs);
        }
        check("slate_dlansy_one", fabs(slate_dlansy('1', 'L', n, A, n) - one) / one, eps);
        check("slate_dlansy_fro", fabs(slate_dlansy('F', 'L', n, A, n) - sqrt(fro)) / sqrt(fro), eps);
        check("slate_dlansy_max", fabs(slate_dlansy('M', 'L', n, A, n) - mx) / mx, eps);
        /* upper trapezoid m x n (m < n), unit diagonal */
        const int m = n - 7;
        double inf = 0, f2 = 0;
        for (int i = 0; i < m; ++i) {
            double rs = 0;
            for (int j = i; j < n; ++j) {
                double v = j == i ? 1.0 : A[i + j * n];
                rs += fabs(v);
                f2 += v * v;
            }
            inf = fmax(inf, rs);
        }
        check("slate_dlantr_inf", fabs(slate_dlantr('I', 'U', 'U', m, n, A, n) - inf) / inf, eps);
        check("slate_dlantr_fro", fabs(slate_dlantr('F', 'U', 'U', m, n, A, n) - sqrt(f2)) / sqrt(f2), eps);
    }
    /* single precision spot checks */
    {
        float* As = malloc(sizeof(float) * n * n);
        float* Cs = malloc(sizeof(float) * n * n);
        for (int i = 0; i < n * n; ++i) { As[i] = (float)B[i]; Cs[i] = (float)C[i]; }
        memcpy(T, C, sizeof(double) * n * n);
        ref_gemm('N', 'T', n, n, k, 1.0, B, n, B, n, 1.0, T, n);
        info = slate_ssyrk('L', 'N', n, k, 1.0f, As, n, 1.0f, Cs, n);
        for (int i = 0; i < n * n; ++i) R[i] = Cs[i];
        check(info ? "slate_ssyrk-FAILED" : "slate_ssyrk_ln", rel(R, T, n, n, n, n, 'L'), 1e-5);
        free(As);
        free(Cs);
    }
    /* complex: herk, her2k, hemm, trmm (ConjTrans), getri, lanhe */
    {
        double complex* Z = malloc(sizeof(double complex) * n * n);
        double complex* W = malloc(sizeof(double complex) * n * n);
        double complex* Y = malloc(sizeof(double complex) * n * n);
        double complex* H = malloc(sizeof(double complex) * n * n);
        for (int j = 0; j < n; ++j)
            for (int i = 0; i < n; ++i) {
                Z[i + j * n] = rnd(i, j, 4) + I * rnd(i, j, 5);
                H[i + j * n] = i == j ? (double complex)(n + rnd(i, i, 6)) : rnd(i, j, 7) + I * rnd(i, j, 8);
            }
        /* herk lower: Y = Z(:, 0:k) Z(:, 0:k)^H * 1 + 0 */
        for (int j = 0; j < n; ++j)
            for (int i = 0; i < n; ++i) {
                double complex s = 0;
                for (int l = 0; l < k; ++l) s += Z[i + l * n] * conj(Z[j + l * n]);
                W[i + j * n] = s;
                Y[i + j * n] = 7.0;
            }
        info = slate_zherk('L', 'N', n, k, 1.0, (double*)Z, n, 0.0, (double*)Y, n);
        check(info ? "slate_zherk-FAILED" : "slate_zherk_ln", zrel(Y, W, n, n, 'L'), eps);
        /* her2k upper, ConjTrans: alpha Z^H H + conj(alpha) H^H Z over k rows */
        const double al[2] = {0.5, -0.25};
        const double complex alc = 0.5 - 0.25 * I;
        for (int j = 0; j < n; ++j)
            for (int i = 0; i < n; ++i) {
                double complex s = 0;
                for (int l = 0; l < k; ++l)
                    s += alc * conj(Z[l + i * n]) * H[l + j * n] + conj(alc) * conj(H[l + i * n]) * Z[l + j * n];
                W[i + j * n] = s + 2.0 * (i == j ? 1.0 : 0.0);
                Y[i + j * n] = i == j ? 1.0 : 0.0;
            }
        info = slate_zher2k('U', 'C', n, k, al, (double*)Z, n, (double*)H, n, 2.0, (double*)Y, n);
        check(info ? "slate_zher2k-FAILED" : "slate_zher2k_uc", zrel(Y, W, n, n, 'U'), eps);
        /* hemm right: Y = Z Hf, Hf Hermitian from H's lower triangle */
        const double one[2] = {1.0, 0.0}, zero[2] = {0.0, 0.0};
        for (int j = 0; j < n; ++j)
            for (int i = 0; i < n; ++i) {
                double complex s = 0;
                for (int l = 0; l < n; ++l) {
                    double complex h = l >= j ? H[l + j * n] : conj(H[j + l * n]);
                    if (l == j) h = creal(h);
                    s += Z[i + l * n] * h;
                }
                W[i + j * n] = s;
            }
        info = slate_zhemm('R', 'L', n, n, one, (double*)H, n, (double*)Z, n, zero, (double*)Y, n);
        check(info ? "slate_zhemm-FAILED" : "slate_zhemm_rl", zrel(Y, W, n, n, 'G'), eps);
        /* trmm left lower ConjTrans non-unit: Y = L^H Z */
        for (int j = 0; j < n; ++j)
            for (int i = 0; i < n; ++i) {
                double complex s = 0;
                for (int l = i; l < n; ++l) s += conj(H[l + i * n]) * Z[l + j * n];
                W[i + j * n] = s;
            }
        memcpy(Y, Z, sizeof(double complex) * n * n);
        info = slate_ztrmm('L', 'L', 'C', 'N', n, n, one, (double*)H, n, (double*)Y, n);
        check(info ? "slate_ztrmm-FAILED" : "slate_ztrmm_llc", zrel(Y, W, n, n, 'G'), eps);
        /* getri */
        memcpy(Y, H, sizeof(double complex) * n * n);
        info = slate_zgetrf(n, n, (double*)Y, n, ipiv);
        int info2 = slate_zgetri(n, (double*)Y, n, ipiv);
        double e = 0;
        for (int j = 0; j < n; ++j)
            for (int i = 0; i < n; ++i) {
                double complex s = 0;
                for (int l = 0; l < n; ++l) s += Y[i + l * n] * H[l + j * n];
                e = fmax(e, cabs(s - (i == j)));
            }
        check(info || info2 ? "slate_zgetri-FAILED" : "slate_zgetri", e, 1e-10);
        /* lanhe one-norm from the lower triangle */
        double onen = 0;
        for (int j = 0; j < n; ++j) {
            double cs = 0;
            for (int i = 0; i < n; ++i) {
                double complex h = i >= j ? H[i + j * n] : conj(H[j + i * n]);
                if (i == j) h = creal(h);
                cs += cabs(h);
            }
            onen = fmax(onen, cs);
        }
        check("slate_zlanhe_one", fabs(slate_zlanhe('O', 'L', n, (double*)H, n) - onen) / onen, eps);
        /* clantr max of a lower non-unit trapezoid (single complex) */
        float complex* Hc = malloc(sizeof(float complex) * n * n);
        double mx = 0;
        for (int j = 0; j < n; ++j)
            for (int i = 0; i < n; ++i) {
                Hc[i + j * n] = (float complex)H[i + j * n];
                if (i >= j && j < n - 5) mx = fmax(mx, cabsf(Hc[i + j * n]));
            }
        check("slate_clantr_max", fabs(slate_clantr('M', 'L', 'N', n, n - 5, (float*)Hc, n) - mx) / mx, 1e-6);
        free(Hc);
        free(Z);
        free(W);
        free(Y);
        free(H);
    }
    /* condition estimates (slate_dgecon / slate_dtrcon) against the exact
     * rcond from the inverse; the Fortran alias slate_dsyev_ by its trace */
    {
        double* F = malloc(sizeof(double) * n * n);
        double* G = malloc(sizeof(double) * n * n);
        double anorm = 0;
        for (int j = 0; j < n; ++j) {
            double cs = 0;
            for (int i = 0; i < n; ++i) {
                F[i + j * n] = rnd(i, j, 7) + (i == j ? 3.0 : 0.0);
                cs += fabs(F[i + j * n]);
            }
            anorm = fmax(anorm, cs);
        }
        memcpy(G, F, sizeof(double) * n * n);
        slate_dgetrf(n, n, F, n, ipiv);
        double rc = -1;
        const int ci = slate_dgecon('1', n, F, n, anorm, &rc);
        slate_dgetri(n, F, n, ipiv);
        double inorm = 0;
        for (int j = 0; j < n; ++j) {
            double cs = 0;
            for (int i = 0; i < n; ++i) cs += fabs(F[i + j * n]);
            inorm = fmax(inorm, cs);
        }
        const double ratio = rc * anorm * inorm;
        check("slate_dgecon_ratio", (ci == 0 && ratio >= 0.999 && ratio <= 3.0) ? 0.0 : 1.0, 0.5);
        /* a unit upper triangle: rcond in (0, 1] */
        double rt = -1;
        const int ti = slate_dtrcon('1', 'U', 'U', n, G, n, &rt);
        check("slate_dtrcon_range", (ti == 0 && rt > 0 && rt <= 1.0) ? 0.0 : 1.0, 0.5);
        /* dsyev_: eigenvalues of the symmetric part sum to its trace */
        for (int j = 0; j < n; ++j)
            for (int i = 0; i < n; ++i) F[i + j * n] = 0.5 * (G[i + j * n] + G[j + i * n]);
        double tr = 0;
        for (int i = 0; i < n; ++i) tr += F[i + i * n];
        double* w = malloc(sizeof(double) * n);
        int64_t nn = n, info = -1;
        slate_dsyev_("N", "L", &nn, F, &nn, w, &info);
        double sw = 0;
        for (int i = 0; i < n; ++i) sw += w[i];
        check("slate_dsyev_trace", info == 0 ? fabs(sw - tr) / fabs(tr) : 1.0, 1e-10);
        free(w);
        free(G);
        free(F);
    }
    if (g_fail) fprintf(stderr, "last error: %s\n", slate_amd_last_error());
    printf(g_fail ? "ex_native_lapack: FAILED\n" : "ex_native_lapack: all checks passed\n");
    free(A);
    free(B);
    free(C);
    free(R);
    free(T);
    free(ipiv);
    return g_fail;
}
