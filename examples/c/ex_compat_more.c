/* The LAPACK-style and ScaLAPACK C entry points added in round 3 (SLATE's
 * lapack_api/ and scalapack_api/ routine set): each check prints
 * "rank r: <name> <relative error>" and the test driver asserts < 1e-9
 * (condition numbers: within a factor 3 of the exact value; "info=" lines
 * must read 0).  argv[1] = "PxQ" grid for the ScaLAPACK part (default 1x1),
 * one process per rank (RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT). */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "slate_amd/c_api.h"

static int me = 0;
static void report(const char* what, double v) { printf("rank %d: %s %.3e\n", me, what, v); fflush(stdout); }

static double rnd(int i, int j, int s) { return sin(0.37 * i + 1.13 * j + 0.71 * s) + 0.1 * cos(3.1 * i * j + s); }

/* ---------------------------------------------------------- LAPACK-style */
static void lapack_part(void) {
    const int n = 48, k = 20;
    double *S = malloc(sizeof(double) * n * n), *B = malloc(sizeof(double) * n * n), *C = malloc(sizeof(double) * n * n);
    double *R = malloc(sizeof(double) * n * n), *A = malloc(sizeof(double) * n * n), *X = malloc(sizeof(double) * n * n);
    for (int j = 0; j < n; ++j)
        for (int i = 0; i < n; ++i) {
            S[i + j * n] = rnd(i > j ? i : j, i > j ? j : i, 1) + (i == j ? n : 0);   /* symmetric, SPD */
            A[i + j * n] = rnd(i, j, 2) + (i == j ? 4.0 : 0.0);
            B[i + j * n] = rnd(i, j, 3);
        }
    /* dsymm: C = S B (lower triangle of S referenced) */
    memset(C, 0, sizeof(double) * n * n);
    int info = slate_dsymm('L', 'L', n, n, 1.0, S, n, B, n, 0.0, C, n);
    double e = 0, r = 0;
    for (int j = 0; j < n; ++j)
        for (int i = 0; i < n; ++i) {
            double s = 0;
            for (int l = 0; l < n; ++l) s += S[i + l * n] * B[l + j * n];
            e += (C[i + j * n] - s) * (C[i + j * n] - s); r += s * s;
        }
    report(info ? "dsymm-FAILED" : "dsymm", sqrt(e / r));
    /* dsyrk: C = B(:, :k) B(:, :k)^T (lower) */
    memset(C, 0, sizeof(double) * n * n);
    info = slate_dsyrk('L', 'N', n, k, 1.0, B, n, 0.0, C, n);
    e = 0; r = 0;
    for (int j = 0; j < n; ++j)
        for (int i = j; i < n; ++i) {
            double s = 0;
            for (int l = 0; l < k; ++l) s += B[i + l * n] * B[j + l * n];
            e += (C[i + j * n] - s) * (C[i + j * n] - s); r += s * s;
        }
    report(info ? "dsyrk-FAILED" : "dsyrk", sqrt(e / r));
    /* dtrmm then dtrsm round trip with the lower triangle of A */
    memcpy(X, B, sizeof(double) * n * n);
    info = slate_dtrmm('L', 'L', 'N', 'N', n, n, 1.0, A, n, X, n);
    info |= slate_dtrsm('L', 'L', 'N', 'N', n, n, 1.0, A, n, X, n);
    e = 0; r = 0;
    for (int i = 0; i < n * n; ++i) { e += (X[i] - B[i]) * (X[i] - B[i]); r += B[i] * B[i]; }
    report(info ? "dtrmm-FAILED" : "dtrmm", sqrt(e / r));
    /* dgetrf + dgetri: A inv(A) = I; dgecon against the exact 1-norm rcond */
    memcpy(R, A, sizeof(double) * n * n);
    int64_t ipiv[64];
    info = slate_dgetrf(n, n, R, n, ipiv);
    double anorm = slate_dlange('1', n, n, A, n), rcond = 0;
    info |= slate_dgecon('1', n, R, n, anorm, &rcond);
    info |= slate_dgetri(n, R, n, ipiv);
    e = 0;
    double ainv1 = 0;
    for (int j = 0; j < n; ++j) {
        double cs = 0;
        for (int i = 0; i < n; ++i) {
            double s = 0;
            for (int l = 0; l < n; ++l) s += A[i + l * n] * R[l + j * n];
            e += (s - (i == j)) * (s - (i == j));
            cs += fabs(R[i + j * n]);
        }
        if (cs > ainv1) ainv1 = cs;
    }
    report(info ? "dgetri-FAILED" : "dgetri", sqrt(e / n));
    const double exact = 1.0 / (anorm * ainv1);
    report("dgecon_ratio_err", rcond >= exact / 3 && rcond <= 3 * exact ? 0.0 : 1.0);
    /* dlansy / dlantr against direct sums */
    double mx = 0;
    for (int i = 0; i < n * n; ++i) mx = fmax(mx, fabs(S[i]));
    report("dlansy", fabs(slate_dlansy('M', 'L', n, S, n) - mx) / mx);
    double fr = 0;
    for (int j = 0; j < n; ++j)
        for (int i = 0; i <= j; ++i) fr += A[i + j * n] * A[i + j * n];
    report("dlantr", fabs(slate_dlantr('F', 'U', 'N', n, n, A, n) - sqrt(fr)) / sqrt(fr));
    /* dsyevd: S V = V diag(w) */
    double* w = malloc(sizeof(double) * n);
    memcpy(R, S, sizeof(double) * n * n);
    info = slate_dsyevd('V', 'L', n, R, n, w);
    e = 0;
    for (int j = 0; j < n; ++j)
        for (int i = 0; i < n; ++i) {
            double s = 0;
            for (int l = 0; l < n; ++l) s += S[i + l * n] * R[l + j * n];
            e += (s - w[j] * R[i + j * n]) * (s - w[j] * R[i + j * n]);
        }
    report(info ? "dsyevd-FAILED" : "dsyevd", sqrt(e) / w[n - 1]);
    /* dsgesv: mixed precision solve */
    memcpy(R, A, sizeof(double) * n * n);
    int64_t iter = 0;
    memcpy(C, B, sizeof(double) * n * n);
    info = slate_dsgesv(n, 2, R, n, ipiv, C, n, X, n, &iter);
    e = 0; r = 0;
    for (int j = 0; j < 2; ++j)
        for (int i = 0; i < n; ++i) {
            double s = 0;
            for (int l = 0; l < n; ++l) s += A[i + l * n] * X[l + j * n];
            e += (s - B[i + j * n]) * (s - B[i + j * n]); r += B[i + j * n] * B[i + j * n];
        }
    report(info ? "dsgesv-FAILED" : "dsgesv", sqrt(e / r));
    /* zherk + zlanhe */
    double* Z = malloc(sizeof(double) * 2 * n * k);
    double* H = calloc(2 * n * n, sizeof(double));
    for (int i = 0; i < n * k; ++i) { Z[2 * i] = rnd(i, 1, 4); Z[2 * i + 1] = rnd(i, 2, 5); }
    info = slate_zherk('L', 'N', n, k, 1.0, Z, n, 0.0, H, n);
    e = 0; r = 0;
    for (int j = 0; j < n; ++j)
        for (int i = j; i < n; ++i) {
            double sr = 0, si = 0;
            for (int l = 0; l < k; ++l) {
                const double ar = Z[2 * (i + l * n)], ai = Z[2 * (i + l * n) + 1];
                const double br = Z[2 * (j + l * n)], bi = -Z[2 * (j + l * n) + 1];
                sr += ar * br - ai * bi; si += ar * bi + ai * br;
            }
            const double dr = H[2 * (i + j * n)] - sr, di = H[2 * (i + j * n) + 1] - si;
            e += dr * dr + di * di; r += sr * sr + si * si;
        }
    report(info ? "zherk-FAILED" : "zherk", sqrt(e / r));
    double hm = 0;
    for (int j = 0; j < n; ++j)
        for (int i = j; i < n; ++i) hm = fmax(hm, hypot(H[2 * (i + j * n)], H[2 * (i + j * n) + 1]));
    report("zlanhe", fabs(slate_zlanhe('M', 'L', n, H, n) - hm) / hm);
    free(S); free(B); free(C); free(R); free(A); free(X); free(w); free(Z); free(H);
}

/* ---------------------------------------------------------- ScaLAPACK */
static int pr, pc, p, q;
static int lrows(int m, int nb) { int z = 0; return numroc_(&m, &nb, &pr, &z, &p); }
static int lcols(int n, int nb) { int z = 0; return numroc_(&n, &nb, &pc, &z, &q); }
static int g_of(int l, int nb, int np, int ip) { return ((l / nb) * np + ip) * nb + l % nb; }

static void scalapack_part(int ctxt) {
    const int n = 40, nb = 8, izero = 0, ione = 1;
    const int ml = lrows(n, nb), nl = lcols(n, nb), lld = ml > 1 ? ml : 1;
    int desc[9], info;
    descinit_(desc, &n, &n, &nb, &nb, &izero, &izero, &ctxt, &lld, &info);
    double *A = calloc((size_t)lld * (nl ? nl : 1), sizeof(double)), *S = calloc((size_t)lld * (nl ? nl : 1), sizeof(double));
    double *B = calloc((size_t)lld * (nl ? nl : 1), sizeof(double)), *C = calloc((size_t)lld * (nl ? nl : 1), sizeof(double));
    for (int lj = 0; lj < nl; ++lj)
        for (int li = 0; li < ml; ++li) {
            const int i = g_of(li, nb, p, pr), j = g_of(lj, nb, q, pc);
            A[li + lj * lld] = rnd(i, j, 2) + (i == j ? 6.0 : 0.0);
            S[li + lj * lld] = rnd(i > j ? i : j, i > j ? j : i, 1) + (i == j ? n : 0);
            B[li + lj * lld] = rnd(i, j, 3);
        }
    const double one = 1.0, zero = 0.0;
    /* pdsymm + pdgemm cross-check: C = S B two ways */
    pdsymm_("L", "L", &n, &n, &one, S, &ione, &ione, desc, B, &ione, &ione, desc, &zero, C, &ione, &ione, desc);
    double* D = calloc((size_t)lld * (nl ? nl : 1), sizeof(double));
    double* Sf = calloc((size_t)lld * (nl ? nl : 1), sizeof(double));
    for (int lj = 0; lj < nl; ++lj)
        for (int li = 0; li < ml; ++li) {
            const int i = g_of(li, nb, p, pr), j = g_of(lj, nb, q, pc);
            Sf[li + lj * lld] = rnd(i > j ? i : j, i > j ? j : i, 1) + (i == j ? n : 0);
        }
    pdgemm_("N", "N", &n, &n, &n, &one, Sf, &ione, &ione, desc, B, &ione, &ione, desc, &zero, D, &ione, &ione, desc);
    const double minus = -1.0;
    for (int i = 0; i < lld * nl; ++i) D[i] -= C[i];
    double dn = pdlange_("F", &n, &n, D, &ione, &ione, desc, NULL), cn = pdlange_("F", &n, &n, C, &ione, &ione, desc, NULL);
    report("pdsymm", dn / cn);
    (void)minus;
    /* pdtrmm + pdtrsm round trip */
    memcpy(D, B, sizeof(double) * lld * nl);
    pdtrmm_("L", "U", "N", "N", &n, &n, &one, A, &ione, &ione, desc, D, &ione, &ione, desc);
    pdtrsm_("L", "U", "N", "N", &n, &n, &one, A, &ione, &ione, desc, D, &ione, &ione, desc);
    for (int i = 0; i < lld * nl; ++i) D[i] -= B[i];
    report("pdtrmm", pdlange_("F", &n, &n, D, &ione, &ione, desc, NULL) / pdlange_("F", &n, &n, B, &ione, &ione, desc, NULL));
    /* pdsyrk vs pdgemm: C = B B^T, lower */
    memset(C, 0, sizeof(double) * lld * nl);
    pdsyrk_("L", "N", &n, &n, &one, B, &ione, &ione, desc, &zero, C, &ione, &ione, desc);
    pdgemm_("N", "T", &n, &n, &n, &one, B, &ione, &ione, desc, B, &ione, &ione, desc, &zero, D, &ione, &ione, desc);
    double e = 0;
    for (int lj = 0; lj < nl; ++lj)
        for (int li = 0; li < ml; ++li)
            if (g_of(li, nb, p, pr) >= g_of(lj, nb, q, pc)) e = fmax(e, fabs(C[li + lj * lld] - D[li + lj * lld]));
    report("pdsyrk", e / pdlange_("M", &n, &n, D, &ione, &ione, desc, NULL));
    /* pdgetrf + pdgetri: A inv(A) - I; pdgecon */
    memcpy(C, A, sizeof(double) * lld * nl);
    int* ipiv = calloc((size_t)ml + nb, sizeof(int));
    pdgetrf_(&n, &n, C, &ione, &ione, desc, ipiv, &info);
    double anorm = pdlange_("1", &n, &n, A, &ione, &ione, desc, NULL), rcond = 0, wq = 0;
    int lw = -1, liw = -1, iwq = 0;
    pdgecon_("1", &n, C, &ione, &ione, desc, &anorm, &rcond, &wq, &lw, &iwq, &liw, &info);   /* workspace query */
    lw = 1; liw = 1;
    pdgecon_("1", &n, C, &ione, &ione, desc, &anorm, &rcond, &wq, &lw, &iwq, &liw, &info);
    printf("rank %d: pdgecon info=%d rcond=%.3e\n", me, info, rcond);
    pdgetri_(&n, C, &ione, &ione, desc, ipiv, &wq, &lw, &iwq, &liw, &info);
    pdgemm_("N", "N", &n, &n, &n, &one, A, &ione, &ione, desc, C, &ione, &ione, desc, &zero, D, &ione, &ione, desc);
    for (int lj = 0; lj < nl; ++lj)
        for (int li = 0; li < ml; ++li)
            if (g_of(li, nb, p, pr) == g_of(lj, nb, q, pc)) D[li + lj * lld] -= 1.0;
    report(info ? "pdgetri-FAILED" : "pdgetri", pdlange_("F", &n, &n, D, &ione, &ione, desc, NULL) / sqrt((double)n));
    /* pdpotrf + pdpotri: S inv(S) - I (lower triangle of inv(S) mirrored) */
    memcpy(C, S, sizeof(double) * lld * nl);
    pdpotrf_("L", &n, C, &ione, &ione, desc, &info);
    pdpotri_("L", &n, C, &ione, &ione, desc, &info);
    printf("rank %d: pdpotri info=%d\n", me, info);
    /* pdlansy / pdlantr */
    const double sm = pdlansy_("M", "L", &n, S, &ione, &ione, desc, NULL);
    const double sf = pdlange_("M", &n, &n, Sf, &ione, &ione, desc, NULL);
    report("pdlansy", fabs(sm - sf) / sf);
    /* pdsyev: eigenvalues only, then with vectors (pdsyevd) */
    double *w = calloc(n, sizeof(double)), *w2 = calloc(n, sizeof(double));
    memcpy(C, S, sizeof(double) * lld * nl);
    lw = 1;
    pdsyev_("N", "L", &n, C, &ione, &ione, desc, w, NULL, &ione, &ione, desc, &wq, &lw, &info);
    memcpy(C, S, sizeof(double) * lld * nl);
    pdsyevd_("V", "L", &n, C, &ione, &ione, desc, w2, D, &ione, &ione, desc, &wq, &lw, &iwq, &liw, &info);
    double we = 0;
    for (int i = 0; i < n; ++i) we = fmax(we, fabs(w[i] - w2[i]));
    report(info ? "pdsyevd-FAILED" : "pdsyevd", we / w[n - 1]);
    /* pdsgesv */
    int nrhs = 2, iter = 0;
    const int nrl = lcols(nrhs, nb), lldb = lld;
    double *Bx = calloc((size_t)lldb * (nrl ? nrl : 1), sizeof(double)), *Xx = calloc((size_t)lldb * (nrl ? nrl : 1), sizeof(double));
    int descb[9];
    descinit_(descb, &n, &nrhs, &nb, &nb, &izero, &izero, &ctxt, &lldb, &info);
    for (int lj = 0; lj < nrl; ++lj)
        for (int li = 0; li < ml; ++li) Bx[li + lj * lldb] = rnd(g_of(li, nb, p, pr), g_of(lj, nb, q, pc), 9);
    memcpy(C, A, sizeof(double) * lld * nl);
    pdsgesv_(&n, &nrhs, C, &ione, &ione, desc, ipiv, Bx, &ione, &ione, descb, Xx, &ione, &ione, descb, &iter, &info);
    /* residual A x - b */
    double* Rr = calloc((size_t)lldb * (nrl ? nrl : 1), sizeof(double));
    memcpy(Rr, Bx, sizeof(double) * lldb * (nrl ? nrl : 1));
    pdgemm_("N", "N", &n, &nrhs, &n, &one, A, &ione, &ione, desc, Xx, &ione, &ione, descb, &minus, Rr, &ione, &ione, descb);
    report(info ? "pdsgesv-FAILED" : "pdsgesv",
           pdlange_("F", &n, &nrhs, Rr, &ione, &ione, descb, NULL) / pdlange_("F", &n, &nrhs, Bx, &ione, &ione, descb, NULL));
    free(A); free(S); free(B); free(C); free(D); free(Sf); free(ipiv); free(w); free(w2); free(Bx); free(Xx); free(Rr);
}

int main(int argc, char** argv) {
    int gp = 1, gq = 1;
    if (argc > 1) sscanf(argv[1], "%dx%d", &gp, &gq);
    int np = 1;
    Cblacs_pinfo(&me, &np);
    if (me == 0) lapack_part();
    int ctxt;
    Cblacs_get(0, 0, &ctxt);
    Cblacs_gridinit(&ctxt, "C", gp, gq);
    Cblacs_gridinfo(ctxt, &p, &q, &pr, &pc);
    scalapack_part(ctxt);
    slate_amd_finalize();
    return 0;
}
