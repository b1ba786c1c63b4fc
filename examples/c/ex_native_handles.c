/* The handle-based C API of libslate_amd_native.so (include/slate_amd/c_api.h,
 * "Distributed matrices by opaque handle"; reference src/c_api/wrappers.cc)
 * on a p x q grid, without Python.  Every check is a relative residual
 * computed through the API itself (copies, gemm, norms), printed as
 * "check <name> <value>"; the last line is "all checks passed" when every
 * value is below its tolerance.
 *
 *   ./ex_native_handles [PxQ]    (one process per rank, torchrun-style env;
 *                                 SLATE_AMD_NATIVE_TRANSPORT=host lets the
 *                                 ranks of a grid share one GPU)
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "slate_amd/c_api.h"

static int g_fail = 0, g_me = 0;

static void report(const char* name, double v, double tol) {
    if (g_me == 0) printf("check %s %.3e\n", name, v);
    if (!(v < tol)) {
        g_fail = 1;
        if (g_me == 0) printf("  FAILED (tol %.1e): %s\n", tol, slate_amd_last_error());
    }
    fflush(stdout);
}

#define M(kind, dt, m, n) slate_amd_matrix_create(kind, dt, m, n, nb, p, q)

/* || B0 - op(A0) X || / (|| A0 || || X ||), max norms */
static double solve_resid(slate_amd_matrix_t A0, slate_amd_matrix_t X, slate_amd_matrix_t B0, char dt,
                          int64_t nb, int p, int q) {
    int64_t m, n;
    slate_amd_matrix_dims(B0, &m, &n);
    slate_amd_matrix_t R = M('G', dt, m, n);
    slate_amd_copy(B0, R);
    slate_amd_gemm(-1.0, A0, X, 1.0, R);
    const double r = slate_amd_norm('1', R) / (slate_amd_norm('1', A0) * slate_amd_norm('1', X));
    slate_amd_matrix_destroy(R);
    return r;
}

int main(int argc, char** argv) {
    int p = 1, q = 1;
    if (argc > 1) sscanf(argv[1], "%dx%d", &p, &q);
    int nprocs = 1;
    Cblacs_pinfo(&g_me, &nprocs);
    if (slate_amd_initialize() != 0) {
        fprintf(stderr, "init: %s\n", slate_amd_last_error());
        return 1;
    }
    const int64_t n = 192, nrhs = 4, nb = 32;
    const double eps = 2.2e-16;
    const double tol = 1e3 * eps;
    if (g_me == 0) printf("native handles: %d ranks, grid %dx%d\n", nprocs, p, q);

    /* ---- posv (Lower Hermitian handle), potrs, potri */
    {
        slate_amd_matrix_t A = M('L', 'd', n, n), A0 = M('L', 'd', n, n), B = M('G', 'd', n, nrhs),
                           B0 = M('G', 'd', n, nrhs), Af = M('G', 'd', n, n);
        slate_amd_matrix_generate(A, 1, 3);
        slate_amd_matrix_generate(A0, 1, 3);
        slate_amd_matrix_generate(B, 0, 4);
        slate_amd_copy(B, B0);
        /* the full Hermitian A0 for the residual: hemm(A0, I) */
        slate_amd_matrix_t I = M('G', 'd', n, n);
        slate_amd_set(0.0, 1.0, I);
        slate_amd_hemm('L', 1.0, A0, I, 0.0, Af);
        const int info = slate_amd_posv(A, B);
        report(info ? "posv-FAILED" : "posv", solve_resid(Af, B, B0, 'd', nb, p, q), tol);
        slate_amd_copy(B0, B);
        slate_amd_potrs(A, B);
        report("potrs", solve_resid(Af, B, B0, 'd', nb, p, q), tol);
        slate_amd_matrix_t P = M('G', 'd', n, n);
        report("pocondest", slate_amd_pocondest('1', A, slate_amd_norm('1', Af)) > 0 ? 0.0 : 1.0, 0.5);
        slate_amd_potri(A);
        /* || A0 inv(A0) - I ||: the inverse's stored triangle expanded by hemm */
        slate_amd_hemm('R', 1.0, A, Af, 0.0, P);
        slate_amd_add(-1.0, I, 1.0, P);
        report("potri", slate_amd_norm('1', P) / n, tol);
        slate_amd_matrix_destroy(P);
        slate_amd_matrix_destroy(I);
        slate_amd_matrix_destroy(A);
        slate_amd_matrix_destroy(A0);
        slate_amd_matrix_destroy(B);
        slate_amd_matrix_destroy(B0);
        slate_amd_matrix_destroy(Af);
    }
    /* ---- gesv / getrs with a transposed view / getri / gecondest (z) */
    {
        slate_amd_matrix_t A = M('G', 'z', n, n), A0 = M('G', 'z', n, n), B = M('G', 'z', n, nrhs),
                           B0 = M('G', 'z', n, nrhs);
        slate_amd_pivots_t piv = slate_amd_pivots_create();
        slate_amd_matrix_generate(A, 0, 5);
        slate_amd_copy(A, A0);
        slate_amd_matrix_generate(B, 0, 6);
        slate_amd_copy(B, B0);
        const int info = slate_amd_gesv(A, piv, B);
        report(info ? "zgesv-FAILED" : "zgesv", solve_resid(A0, B, B0, 'z', nb, p, q), tol);
        /* A^H X = B with the same factors: a conjugate-transposed view */
        slate_amd_copy(B0, B);
        slate_amd_matrix_t Ah = slate_amd_matrix_op(A, 'C'), A0h = slate_amd_matrix_op(A0, 'C');
        slate_amd_getrs(Ah, piv, B);
        report("zgetrs_conj", solve_resid(A0h, B, B0, 'z', nb, p, q), tol);
        const double rc = slate_amd_gecondest('1', A, piv, slate_amd_norm('1', A0));
        report("zgecondest", rc > 0 && rc <= 1 ? 0.0 : 1.0, 0.5);
        slate_amd_getri(A, piv);
        slate_amd_matrix_t P = M('G', 'z', n, n), I = M('G', 'z', n, n);
        slate_amd_set(0.0, 1.0, I);
        slate_amd_gemm(1.0, A0, A, 0.0, P);
        slate_amd_add(-1.0, I, 1.0, P);
        report("zgetri", slate_amd_norm('1', P) / (n * slate_amd_norm('1', A0) * slate_amd_norm('1', A)), tol);
        slate_amd_matrix_destroy(Ah);
        slate_amd_matrix_destroy(A0h);
        slate_amd_matrix_destroy(P);
        slate_amd_matrix_destroy(I);
        slate_amd_pivots_destroy(piv);
        slate_amd_matrix_destroy(A);
        slate_amd_matrix_destroy(A0);
        slate_amd_matrix_destroy(B);
        slate_amd_matrix_destroy(B0);
    }
    /* ---- gemm with transposed views, trsm / trmm round trip, herk vs gemm */
    {
        const int64_t k = 96;
        slate_amd_matrix_t A = M('G', 'd', k, n), B = M('G', 'd', n, k), C = M('G', 'd', n, n),
                           C2 = M('G', 'd', n, n), At = M('G', 'd', n, k);
        slate_amd_matrix_generate(A, 0, 7);
        slate_amd_matrix_generate(B, 0, 8);
        slate_amd_matrix_t Av = slate_amd_matrix_op(A, 'T');       /* n x k view */
        slate_amd_copy(Av, At);                                      /* materialised A^T */
        slate_amd_matrix_t Bv = slate_amd_matrix_op(B, 'T');       /* k x n view */
        slate_amd_gemm(1.0, Av, Bv, 0.0, C);                        /* A^T B^T */
        slate_amd_gemm(1.0, At, Bv, 0.0, C2);
        slate_amd_add(-1.0, C, 1.0, C2);
        report("gemm_views", slate_amd_norm('M', C2) / slate_amd_norm('M', C), tol);
        /* herk: C = A^T A on the Lower triangle against gemm */
        slate_amd_matrix_t H = M('L', 'd', n, n), G2 = M('G', 'd', n, n), I = M('G', 'd', n, n), Hf = M('G', 'd', n, n);
        slate_amd_herk(1.0, Av, 0.0, H);
        slate_amd_gemm(1.0, Av, A, 0.0, G2);
        slate_amd_set(0.0, 1.0, I);
        slate_amd_hemm('L', 1.0, H, I, 0.0, Hf);
        slate_amd_add(-1.0, G2, 1.0, Hf);
        report("herk", slate_amd_norm('M', Hf) / slate_amd_norm('M', G2), tol);
        /* trmm then trsm with the same triangle: identity */
        slate_amd_matrix_t T = M('G', 'd', n, n), X = M('G', 'd', n, k), X0 = M('G', 'd', n, k);
        slate_amd_matrix_generate(T, 0, 9);
        slate_amd_set(0.0, (double)n, I);
        slate_amd_add(1.0, I, 1.0, T);                              /* well-conditioned diagonal */
        slate_amd_copy(At, X);
        slate_amd_copy(At, X0);
        slate_amd_trmm('L', 'U', 'N', 2.0, T, X);
        slate_amd_trsm('L', 'U', 'N', 0.5, T, X);
        slate_amd_add(-1.0, X0, 1.0, X);
        report("trmm_trsm", slate_amd_norm('M', X) / slate_amd_norm('M', X0), tol);
        slate_amd_matrix_destroy(Av);
        slate_amd_matrix_destroy(Bv);
        slate_amd_matrix_destroy(A);
        slate_amd_matrix_destroy(B);
        slate_amd_matrix_destroy(C);
        slate_amd_matrix_destroy(C2);
        slate_amd_matrix_destroy(At);
        slate_amd_matrix_destroy(H);
        slate_amd_matrix_destroy(G2);
        slate_amd_matrix_destroy(I);
        slate_amd_matrix_destroy(Hf);
        slate_amd_matrix_destroy(T);
        slate_amd_matrix_destroy(X);
        slate_amd_matrix_destroy(X0);
    }
    /* ---- geqrf + unmqr (left and right): Q^H Q C = C; gels residual orthogonal to A */
    {
        const int64_t m = 256, k = 128;
        slate_amd_matrix_t A = M('G', 'd', m, k), C = M('G', 'd', m, nrhs), C0 = M('G', 'd', m, nrhs),
                           D = M('G', 'd', nrhs, m), D0 = M('G', 'd', nrhs, m);
        slate_amd_tfactors_t T = slate_amd_tfactors_create();
        slate_amd_matrix_generate(A, 0, 10);
        slate_amd_matrix_generate(C, 0, 11);
        slate_amd_copy(C, C0);
        slate_amd_geqrf(A, T);
        slate_amd_unmqr('L', 'C', A, T, C);
        slate_amd_unmqr('L', 'N', A, T, C);
        slate_amd_add(-1.0, C0, 1.0, C);
        report("unmqr_left", slate_amd_norm('M', C) / slate_amd_norm('M', C0), tol);
        slate_amd_matrix_generate(D, 0, 12);
        slate_amd_copy(D, D0);
        slate_amd_unmqr('R', 'N', A, T, D);
        slate_amd_unmqr('R', 'C', A, T, D);
        slate_amd_add(-1.0, D0, 1.0, D);
        report("unmqr_right", slate_amd_norm('M', D) / slate_amd_norm('M', D0), tol);
        slate_amd_tfactors_destroy(T);
        slate_amd_matrix_destroy(A);
        slate_amd_matrix_destroy(C);
        slate_amd_matrix_destroy(C0);
        slate_amd_matrix_destroy(D);
        slate_amd_matrix_destroy(D0);
    }
    /* ---- heev / hegv / svd_vals: eigenvalue equations through the API */
    {
        slate_amd_matrix_t A = M('L', 'd', n, n), Z = M('G', 'd', n, n), AZ = M('G', 'd', n, n);
        slate_amd_matrix_generate(A, 0, 13);
        double* w = (double*)malloc(sizeof(double) * n);
        int info = slate_amd_heev(A, w, Z);
        slate_amd_hemm('L', 1.0, A, Z, 0.0, AZ);
        /* A Z - Z diag(w): column j of Z scaled through a diagonal gemm */
        slate_amd_matrix_t W = M('G', 'd', n, n);
        slate_amd_set(0.0, 0.0, W);
        double* wl = NULL;
        int64_t mloc, nloc;
        slate_amd_matrix_local_size(W, &mloc, &nloc);
        wl = (double*)calloc((size_t)(mloc > 0 ? mloc : 1) * (size_t)(nloc > 0 ? nloc : 1), sizeof(double));
        /* local block of diag(w): global (i, i) of block-cyclic tiles */
        int pr = g_me % p, pc = g_me / p;
        for (int64_t jl = 0; jl < nloc; ++jl) {
            const int64_t jg = ((jl / nb) * q + pc) * nb + jl % nb;
            for (int64_t il = 0; il < mloc; ++il) {
                const int64_t ig = ((il / nb) * p + pr) * nb + il % nb;
                if (ig == jg) wl[il + jl * mloc] = w[ig];
            }
        }
        slate_amd_matrix_set_local(W, wl, mloc > 0 ? mloc : 1);
        slate_amd_gemm(-1.0, Z, W, 1.0, AZ);
        report(info ? "heev-FAILED" : "heev", slate_amd_norm('M', AZ) / (fabs(w[0]) + fabs(w[n - 1])), tol);
        /* hegv: values only, itype 1, against heev of the same A with B = I */
        slate_amd_matrix_t A2 = M('L', 'd', n, n), B2 = M('L', 'd', n, n);
        slate_amd_matrix_generate(A2, 0, 13);
        slate_amd_set(0.0, 1.0, B2);
        double* w2 = (double*)malloc(sizeof(double) * n);
        info = slate_amd_hegv(1, A2, B2, w2, 0);
        double dv = 0;
        for (int64_t i = 0; i < n; ++i) dv = fmax(dv, fabs(w2[i] - w[i]));
        report(info ? "hegv-FAILED" : "hegv_identity", dv / (fabs(w[0]) + fabs(w[n - 1])), tol);
        /* singular values of a Hermitian matrix = |eigenvalues| */
        slate_amd_matrix_t S = M('G', 'd', n, n);
        slate_amd_matrix_t I = M('G', 'd', n, n);
        slate_amd_set(0.0, 1.0, I);
        slate_amd_matrix_t A3 = M('L', 'd', n, n);
        slate_amd_matrix_generate(A3, 0, 13);
        slate_amd_hemm('L', 1.0, A3, I, 0.0, S);
        double* sv = (double*)malloc(sizeof(double) * n);
        info = slate_amd_svd_vals(S, sv);
        double* aw = (double*)malloc(sizeof(double) * n);
        for (int64_t i = 0; i < n; ++i) aw[i] = fabs(w[i]);
        /* sort |w| descending (insertion sort, small n) */
        for (int64_t i = 1; i < n; ++i) {
            const double x = aw[i];
            int64_t j = i - 1;
            while (j >= 0 && aw[j] < x) { aw[j + 1] = aw[j]; --j; }
            aw[j + 1] = x;
        }
        double ds = 0;
        for (int64_t i = 0; i < n; ++i) ds = fmax(ds, fabs(sv[i] - aw[i]));
        report(info ? "svd_vals-FAILED" : "svd_vals", ds / aw[0], tol);
        free(w); free(w2); free(wl); free(sv); free(aw);
        slate_amd_matrix_destroy(A);
        slate_amd_matrix_destroy(Z);
        slate_amd_matrix_destroy(AZ);
        slate_amd_matrix_destroy(W);
        slate_amd_matrix_destroy(A2);
        slate_amd_matrix_destroy(B2);
        slate_amd_matrix_destroy(S);
        slate_amd_matrix_destroy(I);
        slate_amd_matrix_destroy(A3);
    }
    /* ---- mixed precision + GMRES, RBT, nopiv, hesv (d) */
    {
        slate_amd_matrix_t A = M('G', 'd', n, n), A0 = M('G', 'd', n, n), B = M('G', 'd', n, nrhs),
                           B0 = M('G', 'd', n, nrhs), X = M('G', 'd', n, nrhs);
        slate_amd_pivots_t piv = slate_amd_pivots_create();
        slate_amd_matrix_generate(A0, 3, 14);
        slate_amd_matrix_generate(B0, 0, 15);
        const char* names[] = {"gesv_mixed", "gesv_mixed_gmres", "gesv_rbt", "gesv_nopiv"};
        for (int v = 0; v < 4; ++v) {
            slate_amd_copy(A0, A);
            slate_amd_copy(B0, B);
            int64_t iter = -99;
            int info;
            if (v == 0) info = slate_amd_gesv_mixed(A, piv, B, X, &iter);
            else if (v == 1) info = slate_amd_gesv_mixed_gmres(A, piv, B, X, &iter);
            else if (v == 2) { info = slate_amd_gesv_rbt(A, B); slate_amd_copy(B, X); }
            else { info = slate_amd_gesv_nopiv(A, B); slate_amd_copy(B, X); }
            report(info || (v < 2 && iter < 0) ? "mixed-FAILED" : names[v], solve_resid(A0, X, B0, 'd', nb, p, q), tol);
        }
        /* Hermitian indefinite: A + A^T with a zero-ish diagonal shift */
        slate_amd_matrix_t H = M('L', 'd', n, n), Hf = M('G', 'd', n, n), I = M('G', 'd', n, n);
        slate_amd_matrix_generate(H, 0, 16);
        slate_amd_set(0.0, 1.0, I);
        slate_amd_hemm('L', 1.0, H, I, 0.0, Hf);
        slate_amd_copy(B0, B);
        const int info = slate_amd_hesv(H, B);
        report(info ? "hesv-FAILED" : "hesv", solve_resid(Hf, B, B0, 'd', nb, p, q), tol);
        /* posv_mixed_gmres on an HPD matrix */
        slate_amd_matrix_t P = M('L', 'd', n, n), Pf = M('G', 'd', n, n);
        slate_amd_matrix_generate(P, 1, 17);
        slate_amd_hemm('L', 1.0, P, I, 0.0, Pf);
        int64_t iter = -99;
        const int pinfo = slate_amd_posv_mixed_gmres(P, B0, X, &iter);
        report(pinfo || iter < 0 ? "posv_mixed_gmres-FAILED" : "posv_mixed_gmres", solve_resid(Pf, X, B0, 'd', nb, p, q),
               tol);
        /* auxiliary: scale(3, 4) then scale(4, 3) is the identity */
        slate_amd_copy(B0, B);
        slate_amd_scale(3.0, 4.0, B);
        slate_amd_scale(4.0, 3.0, B);
        slate_amd_add(-1.0, B0, 1.0, B);
        report("scale", slate_amd_norm('M', B) / slate_amd_norm('M', B0), tol);
        /* a tile sub-matrix view: norm of A0[0:2, 0:2] tiles is <= norm of A0 */
        slate_amd_matrix_t S = slate_amd_matrix_sub(A0, 0, p * 2 - 1, 0, q * 2 - 1);
        int64_t sm, sn_;
        slate_amd_matrix_dims(S, &sm, &sn_);
        report("sub_dims", (sm == (p * 2 * nb < n ? p * 2 * nb : n) && sn_ == (q * 2 * nb < n ? q * 2 * nb : n)) ? 0.0
                                                                                                             : 1.0,
               0.5);
        report("sub_norm", slate_amd_norm('M', S) <= slate_amd_norm('M', A0) ? 0.0 : 1.0, 0.5);
        slate_amd_matrix_destroy(S);
        slate_amd_pivots_destroy(piv);
        slate_amd_matrix_destroy(A);
        slate_amd_matrix_destroy(A0);
        slate_amd_matrix_destroy(B);
        slate_amd_matrix_destroy(B0);
        slate_amd_matrix_destroy(X);
        slate_amd_matrix_destroy(H);
        slate_amd_matrix_destroy(Hf);
        slate_amd_matrix_destroy(I);
        slate_amd_matrix_destroy(P);
        slate_amd_matrix_destroy(Pf);
    }
    /* ---- error path: a bad handle reports, it does not abort */
    {
        const int rc = slate_amd_potrf(987654321);
        report("bad_handle", rc == SLATE_AMD_ERR_INTERNAL ? 0.0 : 1.0, 0.5);
    }
    if (g_me == 0) printf(g_fail ? "some checks FAILED\n" : "all checks passed\n");
    slate_amd_finalize();
    return g_fail;
}
