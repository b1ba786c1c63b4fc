/* C API example / test: Cholesky solve and LU solve through libslate_amd_c. */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

#include "slate_amd/c_api.h"

int main(void) {
    const int64_t n = 50, nrhs = 2;
    double *A = malloc(sizeof(double) * n * n), *A0 = malloc(sizeof(double) * n * n);
    double *B = malloc(sizeof(double) * n * nrhs), *B0 = malloc(sizeof(double) * n * nrhs);
    int64_t* ipiv = malloc(sizeof(int64_t) * n);
    srand(1);
    for (int64_t j = 0; j < n; ++j)
        for (int64_t i = 0; i < n; ++i) A0[i + j * n] = (i == j ? n : 0) + (double)rand() / RAND_MAX - 0.5;
    for (int64_t i = 0; i < n * nrhs; ++i) B0[i] = (double)rand() / RAND_MAX;
    if (slate_amd_initialize() != 0) { printf("init failed: %s\n", slate_amd_last_error()); return 2; }
    /* LU solve */
    for (int64_t i = 0; i < n * n; ++i) A[i] = A0[i];
    for (int64_t i = 0; i < n * nrhs; ++i) B[i] = B0[i];
    int info = slate_dgesv(n, nrhs, A, n, ipiv, B, n);
    double err = 0;
    for (int64_t c = 0; c < nrhs; ++c)
        for (int64_t i = 0; i < n; ++i) {
            double s = -B0[i + c * n];
            for (int64_t k = 0; k < n; ++k) s += A0[i + k * n] * B[k + c * n];
            err = fmax(err, fabs(s));
        }
    printf("dgesv info=%d residual=%.3e\n", info, err);
    /* SPD solve: A0 A0^T + n I */
    double* S = malloc(sizeof(double) * n * n);
    for (int64_t j = 0; j < n; ++j)
        for (int64_t i = 0; i < n; ++i) {
            double s = (i == j) ? n : 0;
            for (int64_t k = 0; k < n; ++k) s += A0[i + k * n] * A0[j + k * n];
            S[i + j * n] = s;
            A[i + j * n] = s;
        }
    for (int64_t i = 0; i < n * nrhs; ++i) B[i] = B0[i];
    int info2 = slate_dposv('L', n, nrhs, A, n, B, n);
    double err2 = 0;
    for (int64_t c = 0; c < nrhs; ++c)
        for (int64_t i = 0; i < n; ++i) {
            double s = -B0[i + c * n];
            for (int64_t k = 0; k < n; ++k) s += S[i + k * n] * B[k + c * n];
            err2 = fmax(err2, fabs(s));
        }
    printf("dposv info=%d residual=%.3e\n", info2, err2);
    double nrm = slate_dlange('F', n, n, S, n);
    printf("dlange F = %.6e\n", nrm);
    slate_amd_finalize();
    return (info == 0 && info2 == 0 && err < 1e-9 && err2 < 1e-8) ? 0 : 1;
}
