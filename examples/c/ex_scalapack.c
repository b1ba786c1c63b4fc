/* ScaLAPACK-style and handle-based C API of slate_amd on a process grid.
 *
 * Start one process per rank with RANK / WORLD_SIZE / MASTER_ADDR /
 * MASTER_PORT set (torchrun convention; a single process needs none).
 * argv[1] = "PxQ" grid (default 1 x WORLD_SIZE).
 *
 *  1. Cblacs_* + descinit_ + numroc_, then pdposv_ and pdgesv_ on
 *     sub-matrices that start INSIDE a tile (ia = ja = 5, nb = 8), and
 *     pdgemm_ on whole matrices; every check is local (known solution).
 *  2. the handle API: gesv on generated matrices, residual by gemm + norm.
 * Prints one "rank r: ..." line per check; the caller greps them.
 */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "slate_amd/c_api.h"

static double aval(int i, int j, int n) { /* symmetric, diagonally dominant */
    return (i == j) ? 2.0 * n + i : 1.0 / (1.0 + i + j);
}

int main(int argc, char** argv) {
    int rank, size, ctxt, p, q, pr, pc, info, zero = 0, one = 1;
    Cblacs_pinfo(&rank, &size);
    p = 1; q = size;
    if (argc > 1) sscanf(argv[1], "%dx%d", &p, &q);
    Cblacs_get(0, 0, &ctxt);
    Cblacs_gridinit(&ctxt, "Col", p, q);
    Cblacs_gridinfo(ctxt, &p, &q, &pr, &pc);

    /* global N x N matrix, sub-problem of size n at (ia, ja) = (5, 5) */
    const int N = 48, nb = 8, n = 40, ia = 5, nrhs = 3;
    int mloc = numroc_(&N, &nb, &pr, &zero, &p), nloc = numroc_(&N, &nb, &pc, &zero, &q);
    int nrl = numroc_(&nrhs, &nb, &pc, &zero, &q);
    int lld = mloc > 1 ? mloc : 1, desca[9], descb[9];
    descinit_(desca, &N, &N, &nb, &nb, &zero, &zero, &ctxt, &lld, &info);
    descinit_(descb, &N, &nrhs, &nb, &nb, &zero, &zero, &ctxt, &lld, &info);
    double* A = calloc((size_t)lld * (nloc > 0 ? nloc : 1), sizeof(double));
    double* B = calloc((size_t)lld * (nrl > 0 ? nrl : 1), sizeof(double));
    int* ipiv = calloc((size_t)mloc + nb, sizeof(int));
    for (int solver = 0; solver < 2; ++solver) {
        /* A(i, j) global; B = A_sub * ones on the sub-matrix rows */
        for (int lj = 0; lj < nloc; ++lj) {
            int j = ((lj / nb) * q + pc) * nb + lj % nb;
            for (int li = 0; li < mloc; ++li) {
                int i = ((li / nb) * p + pr) * nb + li % nb;
                A[li + (size_t)lj * lld] = aval(i, j, N) + (solver ? 0.25 * (i > j) : 0.0);
            }
        }
        for (int lj = 0; lj < nrl; ++lj)
            for (int li = 0; li < mloc; ++li) {
                int i = ((li / nb) * p + pr) * nb + li % nb;
                double s = 0;
                if (i >= ia - 1 && i < ia - 1 + n)
                    for (int j = ia - 1; j < ia - 1 + n; ++j) s += aval(i, j, N) + (solver ? 0.25 * (i > j) : 0.0);
                B[li + (size_t)lj * lld] = s;
            }
        if (solver == 0) pdposv_("L", &n, &nrhs, A, &ia, &ia, desca, B, &ia, &one, descb, &info);
        else pdgesv_(&n, &nrhs, A, &ia, &ia, desca, ipiv, B, &ia, &one, descb, &info);
        double err = 0;
        for (int lj = 0; lj < nrl; ++lj)
            for (int li = 0; li < mloc; ++li) {
                int i = ((li / nb) * p + pr) * nb + li % nb;
                if (i >= ia - 1 && i < ia - 1 + n) err = fmax(err, fabs(B[li + (size_t)lj * lld] - 1.0));
            }
        printf("rank %d: %s info=%d maxerr=%.3e\n", rank, solver ? "pdgesv" : "pdposv", info, err);
    }

    /* pdgemm_: C = A * ones(N, nrhs), A(i, j) = i + 1  ->  C(i, :) = N (i + 1) */
    for (int lj = 0; lj < nloc; ++lj)
        for (int li = 0; li < mloc; ++li)
            A[li + (size_t)lj * lld] = ((li / nb) * p + pr) * nb + li % nb + 1.0;
    double* O = calloc((size_t)lld * (nrl > 0 ? nrl : 1), sizeof(double));
    int desco[9];
    int lldo = lld;
    descinit_(desco, &N, &nrhs, &nb, &nb, &zero, &zero, &ctxt, &lldo, &info);
    for (int k = 0; k < lld * nrl; ++k) O[k] = 1.0;
    const double al = 1.0, be = 0.0;
    pdgemm_("N", "N", &N, &nrhs, &N, &al, A, &one, &one, desca, O, &one, &one, desco, &be, B, &one, &one, descb);
    double gerr = 0;
    for (int lj = 0; lj < nrl; ++lj)
        for (int li = 0; li < mloc; ++li) {
            int i = ((li / nb) * p + pr) * nb + li % nb;
            gerr = fmax(gerr, fabs(B[li + (size_t)lj * lld] - (double)N * (i + 1)));
        }
    printf("rank %d: pdgemm maxerr=%.3e\n", rank, gerr);

    /* handle API */
    const int64_t hn = 64;
    slate_amd_matrix_t hA = slate_amd_matrix_create('G', 'd', hn, hn, 16, p, q);
    slate_amd_matrix_t hA0 = slate_amd_matrix_create('G', 'd', hn, hn, 16, p, q);
    slate_amd_matrix_t hB = slate_amd_matrix_create('G', 'd', hn, 4, 16, p, q);
    slate_amd_matrix_t hB0 = slate_amd_matrix_create('G', 'd', hn, 4, 16, p, q);
    slate_amd_matrix_generate(hA, 0, 11);
    slate_amd_matrix_generate(hA0, 0, 11);
    slate_amd_matrix_generate(hB, 0, 12);
    slate_amd_matrix_generate(hB0, 0, 12);
    int64_t ml, nl;
    slate_amd_matrix_local_size(hA, &ml, &nl);
    double* loc = calloc((size_t)(ml > 0 ? ml : 1) * (nl > 0 ? nl : 1), sizeof(double));
    slate_amd_matrix_get_local(hA, loc, ml > 0 ? ml : 1);   /* round trip through host memory */
    slate_amd_matrix_set_local(hA, loc, ml > 0 ? ml : 1);
    slate_amd_pivots_t piv = slate_amd_pivots_create();
    info = slate_amd_gesv(hA, piv, hB);
    slate_amd_gemm(1.0, hA0, hB, -1.0, hB0);              /* B0 := A0 X - B0 */
    double r = slate_amd_norm('F', hB0);
    printf("rank %d: handle gesv info=%d residual=%.3e\n", rank, info, r);
    slate_amd_pivots_destroy(piv);
    slate_amd_matrix_destroy(hA); slate_amd_matrix_destroy(hA0);
    slate_amd_matrix_destroy(hB); slate_amd_matrix_destroy(hB0);
    free(A); free(B); free(O); free(ipiv); free(loc);
    Cblacs_gridexit(ctxt);
    slate_amd_finalize();
    return 0;
}
