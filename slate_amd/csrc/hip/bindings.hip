#include <vector>
#include <pybind11/stl.h>
// pybind11 module exposing the gfx950 kernels to the Python runtime.
// Pointers are passed as integers (tensor.data_ptr()), streams as the raw
// hipStream_t integer (torch.cuda.current_stream().cuda_stream).
#include <pybind11/pybind11.h>
#include <pybind11/complex.h>
#include <complex>
#include "launchers.hpp"
#include "kernels.hpp"


namespace py = pybind11;
using namespace slate_hip;

void register_devpool(py::module& m);   // devpool.hip

static inline hipStream_t S(uintptr_t s) { return reinterpret_cast<hipStream_t>(s); }

static TriMask make_mask(py::object m) {
    TriMask t;
    if (m.is_none()) return t;
    py::tuple tup = m.cast<py::tuple>();
    // (mode, nb, p, pr, q, pc, row_off, col_off, diag_off)
    t.mode = tup[0].cast<int>();
    t.nb = tup[1].cast<i64>();
    t.p = tup[2].cast<int>(); t.pr = tup[3].cast<int>();
    t.q = tup[4].cast<int>(); t.pc = tup[5].cast<int>();
    t.row_off = tup[6].cast<i64>(); t.col_off = tup[7].cast<i64>();
    t.diag_off = tup[8].cast<i64>();
    return t;
}

static void py_gemm(char dtype, char ta, char tb, i64 m, i64 n, i64 k,
                    std::complex<double> alpha, uintptr_t A, i64 lda, uintptr_t B, i64 ldb,
                    std::complex<double> beta, uintptr_t C, i64 ldc,
                    i64 batch, i64 sA, i64 sB, i64 sC, py::object mask, uintptr_t stream) {
    GemmCall c;
    c.transA = ta; c.transB = tb; c.m = m; c.n = n; c.k = k;
    c.alpha_re = alpha.real(); c.alpha_im = alpha.imag();
    c.beta_re = beta.real(); c.beta_im = beta.imag();
    c.A = (const void*)A; c.lda = lda; c.strideA = sA;
    c.B = (const void*)B; c.ldb = ldb; c.strideB = sB;
    c.C = (void*)C; c.ldc = ldc; c.strideC = sC;
    c.batch = batch;
    c.mask = make_mask(mask);
    switch (dtype) {
        case 'd': gemm_real<double>(c, S(stream)); break;
        case 's': gemm_real<float>(c, S(stream)); break;
        case 'z': gemm_complex<zcplx>(c, S(stream)); break;
        case 'c': gemm_complex<ccplx>(c, S(stream)); break;
        default: throw std::invalid_argument("gemm: bad dtype");
    }
}

static void py_gemm_ptrs(char dtype, char ta, char tb, i64 m, i64 n, i64 k,
                         std::complex<double> alpha, uintptr_t Aptrs, i64 lda, uintptr_t Bptrs, i64 ldb,
                         std::complex<double> beta, uintptr_t Cptrs, i64 ldc, i64 batch,
                         bool vec_ok, uintptr_t stream) {
    GemmCall c;
    c.transA = ta; c.transB = tb; c.m = m; c.n = n; c.k = k;
    c.alpha_re = alpha.real(); c.alpha_im = alpha.imag();
    c.beta_re = beta.real(); c.beta_im = beta.imag();
    c.Aptrs = (const void* const*)Aptrs; c.lda = lda;
    c.Bptrs = (const void* const*)Bptrs; c.ldb = ldb;
    c.Cptrs = (void* const*)Cptrs; c.ldc = ldc;
    c.batch = batch; c.vec_ok = vec_ok;
    switch (dtype) {
        case 'd': gemm_real<double>(c, S(stream)); break;
        case 's': gemm_real<float>(c, S(stream)); break;
        case 'z': gemm_complex<zcplx>(c, S(stream)); break;
        case 'c': gemm_complex<ccplx>(c, S(stream)); break;
        default: throw std::invalid_argument("gemm_ptrs: bad dtype");
    }
}


template <typename F>
static void dispatch(char dt, F&& f) {
    switch (dt) {
        case 's': f(float()); break;
        case 'd': f(double()); break;
        case 'c': f(ccplx()); break;
        case 'z': f(zcplx()); break;
        default: throw std::invalid_argument("bad dtype");
    }
}
template <typename T> static T cv(std::complex<double> z) {
    if constexpr (scalar_traits<T>::is_complex) {
        using R = typename scalar_traits<T>::real;
        T r; r.re = (R)z.real(); r.im = (R)z.imag(); return r;
    } else {
        return (T)z.real();
    }
}
template <typename T> static T* P(uintptr_t p) { return reinterpret_cast<T*>(p); }

static void register_kernels(py::module& m) {
    m.def("trsm", [](char dt, char side, char uplo, char trans, char diag, i64 mm, i64 n, std::complex<double> alpha,
                     uintptr_t A, i64 lda, uintptr_t B, i64 ldb, uintptr_t st) {
        dispatch(dt, [&](auto z) { using T = decltype(z);
            trsm<T>(side, uplo, trans, diag, mm, n, cv<T>(alpha), P<T>(A), lda, P<T>(B), ldb, S(st)); });
    });
    m.def("trmm", [](char dt, char side, char uplo, char trans, char diag, i64 mm, i64 n, std::complex<double> alpha,
                     uintptr_t A, i64 lda, uintptr_t B, i64 ldb, uintptr_t st) {
        dispatch(dt, [&](auto z) { using T = decltype(z);
            trmm<T>(side, uplo, trans, diag, mm, n, cv<T>(alpha), P<T>(A), lda, P<T>(B), ldb, S(st)); });
    });
    m.def("potrf", [](char dt, char uplo, i64 n, uintptr_t A, i64 lda, uintptr_t info, uintptr_t st) {
        dispatch(dt, [&](auto z) { using T = decltype(z);
            potrf_tile<T>(uplo, (int)n, P<T>(A), lda, P<i64>(info), S(st)); });
    });
    m.def("getrf", [](char dt, i64 mm, i64 n, uintptr_t A, i64 lda, uintptr_t ipiv, uintptr_t info, double thr,
                      bool nopiv, uintptr_t work, uintptr_t st) {
        dispatch(dt, [&](auto z) { using T = decltype(z);
            getrf_panel_ws<T>(mm, n, P<T>(A), lda, P<i64>(ipiv), P<i64>(info), thr, nopiv, (void*)work, S(st)); });
    });
    m.def("tri_inv", [](char dt, char uplo, char diag, i64 n, uintptr_t A, i64 lda, uintptr_t W, i64 ldw,
                        uintptr_t st) {
        dispatch(dt, [&](auto z) { using T = decltype(z);
            tri_inv<T>(uplo, diag, n, P<const T>(A), lda, P<T>(W), ldw, S(st)); });
    });
    m.def("trtri", [](char dt, char uplo, char diag, i64 n, uintptr_t A, i64 lda, uintptr_t info, uintptr_t st) {
        dispatch(dt, [&](auto z) { using T = decltype(z);
            trtri<T>(uplo, diag, n, P<T>(A), lda, P<i64>(info), S(st)); });
    });
    m.def("stedc_secular", [](i64 n, uintptr_t d, uintptr_t z, double rho, double zz, uintptr_t org, uintptr_t mu,
                              uintptr_t zh, uintptr_t V, i64 ldv, uintptr_t st) {
        stedc_secular(n, P<double>(d), P<double>(z), rho, zz, P<i64>(org), P<double>(mu), P<double>(zh),
                      P<double>(V), ldv, S(st)); });
    m.def("steqr_leaves", [](i64 nleaf, uintptr_t lo, uintptr_t hi, uintptr_t d, uintptr_t e, uintptr_t w,
                             uintptr_t Q, i64 ldq, i64 r0, i64 r1, uintptr_t fails, uintptr_t st, int maxleaf, int maxit) {
        steqr_leaves(nleaf, P<const i64>(lo), P<const i64>(hi), P<const double>(d), P<const double>(e), P<double>(w),
                     P<double>(Q), ldq, r0, r1, P<i64>(fails), S(st), maxleaf, maxit); }, py::arg("nleaf"), py::arg("lo"),
          py::arg("hi"), py::arg("d"), py::arg("e"), py::arg("w"), py::arg("Q"), py::arg("ldq"), py::arg("r0"),
          py::arg("r1"), py::arg("fails"), py::arg("st"), py::arg("maxleaf") = 64, py::arg("maxit") = 60);
    m.def("stedc_runs", [](i64 nn, uintptr_t c, uintptr_t dd, uintptr_t z, uintptr_t ty, double tol, uintptr_t cs,
                           uintptr_t sn, uintptr_t rot, uintptr_t keep, uintptr_t st) {
        stedc_runs(nn, P<const i64>(c), P<const double>(dd), P<double>(z), P<int>(ty), tol, P<double>(cs),
                   P<double>(sn), P<int>(rot), P<int>(keep), S(st)); });
    m.def("rot_cols", [](i64 m_, uintptr_t Q, i64 ldq, i64 nrot, uintptr_t I, uintptr_t J, uintptr_t C, uintptr_t Sn,
                         uintptr_t st) {
        rot_cols(m_, P<double>(Q), ldq, nrot, P<const i64>(I), P<const i64>(J), P<const double>(C),
                 P<const double>(Sn), S(st)); });
    m.def("stedc_vectors", [](i64 n, uintptr_t d, uintptr_t zh, uintptr_t org, uintptr_t mu, i64 j0, i64 nc,
                              uintptr_t V, i64 ldv, uintptr_t st) {
        stedc_vectors(n, P<const double>(d), P<const double>(zh), P<const i64>(org), P<const double>(mu), j0, nc,
                      P<double>(V), ldv, S(st)); });
    // device-resident D&C merges of one tree level (stedc.hip)
    m.def("stedc_level_prep", [](i64 n, i64 nm, i64 maxs, uintptr_t desc, uintptr_t rho, uintptr_t W, uintptr_t Z,
                                 uintptr_t dd, uintptr_t zs, uintptr_t ty, uintptr_t order, uintptr_t c,
                                 uintptr_t keep, uintptr_t rot, uintptr_t cs, uintptr_t sn, uintptr_t meta,
                                 uintptr_t K, uintptr_t S1, uintptr_t KS1, uintptr_t S2, uintptr_t KS2, uintptr_t D,
                                 uintptr_t isK, uintptr_t rI, uintptr_t rJ, uintptr_t rC, uintptr_t rS,
                                 uintptr_t st) {
        stedc_level_prep(n, nm, maxs, P<const i64>(desc), P<const double>(rho), P<const double>(W),
                         P<const double>(Z), P<double>(dd), P<double>(zs), P<int>(ty), P<i64>(order), P<i64>(c),
                         P<int>(keep), P<int>(rot), P<double>(cs), P<double>(sn), reinterpret_cast<void*>(meta),
                         P<i64>(K), P<i64>(S1), P<i64>(KS1), P<i64>(S2), P<i64>(KS2), P<i64>(D), P<i64>(isK),
                         P<i64>(rI), P<i64>(rJ), P<double>(rC), P<double>(rS), S(st)); });
    m.def("stedc_meta_bytes", []() { return (i64)stedc_meta_bytes(); });
    m.def("stedc_lambda", [](i64 s_, uintptr_t dd, uintptr_t isK, uintptr_t dK, uintptr_t org, uintptr_t mu, int flip,
                             uintptr_t lam, uintptr_t st) {
        stedc_lambda(s_, P<const double>(dd), P<const i64>(isK), P<const double>(dK), P<const i64>(org),
                     P<const double>(mu), flip, P<double>(lam), S(st)); });
    m.def("stedc_merge2", [](uintptr_t lam, uintptr_t L1, i64 n1, uintptr_t L2, i64 n2, int rev, uintptr_t out,
                             uintptr_t st) {
        stedc_merge2(P<const double>(lam), P<const i64>(L1), n1, P<const i64>(L2), n2, rev, P<i64>(out), S(st)); });
    m.def("cols_copy", [](i64 m_, i64 nc, uintptr_t A, i64 lda, uintptr_t idx, uintptr_t B, i64 ldb, int scatter,
                          uintptr_t st) {
        cols_copy(m_, nc, P<const double>(A), lda, P<const i64>(idx), P<double>(B), ldb, scatter != 0, S(st)); });
    m.def("vec_gather", [](i64 n, uintptr_t x, uintptr_t idx, uintptr_t y, uintptr_t st) {
        vec_gather(n, P<const double>(x), P<const i64>(idx), P<double>(y), S(st)); });
    m.def("lu_persist_profile", [](int enable) {
        unsigned long long v[8];
        lu_persist_profile(enable, v);
        return std::vector<unsigned long long>(v, v + 8); });
    // tile Cholesky variants (tools / tests): 0 = one-CU potrf_lds, 1 = multi-WG potrf_mc
    m.def("potrf_tile_variant", [](int variant, i64 n, uintptr_t A, i64 lda, uintptr_t info, uintptr_t st) {
        HIP_CHECK(hipMemsetAsync(P<i64>(info), 0, sizeof(i64), S(st)));
        bool ok = variant == 1 ? potrf_mc((int)n, P<double>(A), lda, P<i64>(info), 0, S(st))
                               : potrf_lds((int)n, P<double>(A), lda, P<i64>(info), 0, S(st));
        if (!ok) throw std::invalid_argument("potrf_tile_variant: n out of range");
    });
    m.def("potrf_mc_set_prof", [](uintptr_t p) { potrf_mc_set_prof(reinterpret_cast<i64*>(p)); });
    m.def("potrf_lds_profile", [](i64 n, uintptr_t A, i64 lda, uintptr_t info, uintptr_t prof, uintptr_t st) {
        potrf_lds_profile((int)n, P<double>(A), lda, P<i64>(info), P<i64>(prof), S(st)); });
    m.def("lu_persist_fallbacks", [](int force) { return lu_persist_fallbacks(force); },
          py::arg("force") = -1);
    m.def("getrf_work_bytes", []() { return (i64)getrf_work_bytes(); });
    m.def("geqrf", [](char dt, i64 mm, i64 n, uintptr_t A, i64 lda, uintptr_t tau, uintptr_t Tm, i64 ldt,
                      uintptr_t V, i64 ldv, uintptr_t work, uintptr_t st) {
        dispatch(dt, [&](auto z) { using T = decltype(z);
            geqrf_panel_ws<T>(mm, n, P<T>(A), lda, P<T>(tau), P<T>(Tm), ldt, P<T>(V), ldv, (void*)work, S(st)); });
    });
    m.def("hb2st", [](char dt, i64 n, int b, uintptr_t A, i64 lda, uintptr_t V, uintptr_t tau, uintptr_t row,
                      uintptr_t len, uintptr_t sweep_ptr, uintptr_t ntask, uintptr_t work, i64 nsw, int nwg,
                      uintptr_t st, uintptr_t prof) {
        dispatch(dt, [&](auto z) { using T = decltype(z);
            hb2st_device<T>(n, b, P<T>(A), lda, P<T>(V), P<T>(tau), P<i64>(row), P<i64>(len), P<const i64>(sweep_ptr),
                            P<const i64>(ntask), P<int>(work), nsw, nwg, S(st), P<i64>(prof)); });
    }, py::arg("dt"), py::arg("n"), py::arg("b"), py::arg("A"), py::arg("lda"), py::arg("V"), py::arg("tau"),
       py::arg("row"), py::arg("len"), py::arg("sweep_ptr"), py::arg("ntask"), py::arg("work"), py::arg("nsw"),
       py::arg("nwg"), py::arg("st"), py::arg("prof") = 0);
    m.def("tb2bd", [](char dt, i64 n, int b, uintptr_t A, i64 lda, uintptr_t UV, uintptr_t Utau, uintptr_t Urow,
                      uintptr_t Ulen, uintptr_t VV, uintptr_t Vtau, uintptr_t Vrow, uintptr_t Vlen, uintptr_t sweep_ptr,
                      uintptr_t ntask, uintptr_t work, i64 nsw, int nwg, uintptr_t st) {
        dispatch(dt, [&](auto z) { using T = decltype(z);
            tb2bd_device<T>(n, b, P<T>(A), lda, P<T>(UV), P<T>(Utau), P<i64>(Urow), P<i64>(Ulen), P<T>(VV), P<T>(Vtau),
                            P<i64>(Vrow), P<i64>(Vlen), P<const i64>(sweep_ptr), P<const i64>(ntask), P<int>(work),
                            nsw, nwg, S(st)); });
    });
    m.def("unmtr_hb2st_blocked", [](char dt, i64 n, i64 ncols, uintptr_t Z, i64 ldz, uintptr_t V, i64 b,
                                    uintptr_t tau, uintptr_t sp, uintptr_t nt, i64 nsw, bool conj_tau, uintptr_t st) {
        bool ok = false;
        dispatch(dt, [&](auto z) { using T = decltype(z);
            ok = unmtr_hb2st_blocked<T>(n, ncols, P<T>(Z), ldz, P<const T>(V), b, P<const T>(tau), P<const i64>(sp),
                                        P<const i64>(nt), nsw, conj_tau, S(st)); });
        return ok;
    });
    m.def("unmtr_hb2st_mfma", [](i64 n, i64 ncols, uintptr_t Z, i64 ldz, uintptr_t V, i64 b, uintptr_t tau,
                                 uintptr_t sp, uintptr_t nt, uintptr_t gJ, uintptr_t gt, uintptr_t gptr, i64 ngroups,
                                 uintptr_t Tg, i64 nsw, uintptr_t st) {
        return unmtr_hb2st_mfma(n, ncols, P<double>(Z), ldz, P<const double>(V), b, P<const double>(tau),
                                P<const i64>(sp), P<const i64>(nt), P<const i64>(gJ), P<const i64>(gt),
                                P<const i64>(gptr), ngroups, P<double>(Tg), nsw, S(st));
    });
    m.def("apply_refl", [](char dt, i64 ncols, uintptr_t Z, i64 ldz, uintptr_t V, i64 b, uintptr_t tau,
                           uintptr_t row, uintptr_t len, i64 first, i64 count, bool conj_tau, uintptr_t st) {
        dispatch(dt, [&](auto z) { using T = decltype(z);
            apply_refl_batch<T>(ncols, P<T>(Z), ldz, P<const T>(V), b, P<const T>(tau), P<const i64>(row),
                                P<const i64>(len), first, count, conj_tau, S(st)); });
    });
    m.def("geqrf_work_bytes", []() { return (i64)geqrf_work_bytes(); });
    m.def("tpqrt_panel", [](char dt, i64 mm, i64 l, i64 j0, int ib, uintptr_t A, i64 lda, uintptr_t B, i64 ldb,
                            uintptr_t V, i64 ldv, uintptr_t tau, uintptr_t Tm, i64 ldt, uintptr_t st) {
        dispatch(dt, [&](auto z) { using T = decltype(z);
            tpqrt_panel<T>(mm, l, j0, ib, P<T>(A), lda, P<T>(B), ldb, P<T>(V), ldv, P<T>(tau), P<T>(Tm), ldt,
                           S(st)); });
    });
    m.def("v_explicit", [](char dt, i64 mm, i64 n, uintptr_t A, i64 lda, uintptr_t V, i64 ldv, uintptr_t st) {
        dispatch(dt, [&](auto z) { using T = decltype(z);
            v_explicit<T>(mm, n, P<T>(A), lda, P<T>(V), ldv, S(st)); });
    });
    m.def("laswp", [](char dt, i64 n, uintptr_t A, i64 lda, i64 k1, i64 k2, uintptr_t ipiv, i64 ioff, int incx,
                      uintptr_t st) {
        dispatch(dt, [&](auto z) { using T = decltype(z);
            laswp_off<T>(n, P<T>(A), lda, k1, k2, P<const i64>(ipiv), ioff, S(st), incx); });
    });
    m.def("laswp_cols", [](char dt, i64 nrows, uintptr_t A, i64 lda, i64 k1, i64 k2, uintptr_t ipiv, i64 ioff,
                           int incx, uintptr_t st) {
        dispatch(dt, [&](auto z) { using T = decltype(z);
            laswp_cols<T>(nrows, P<T>(A), lda, k1, k2, P<const i64>(ipiv), ioff, S(st), incx); });
    });
    m.def("laswp_cols_plan", [](char dt, i64 nrows, uintptr_t A, i64 lda, uintptr_t plan, uintptr_t st) {
        dispatch(dt, [&](auto z) { using T = decltype(z);
            laswp_cols_plan<T>(nrows, P<T>(A), lda, (const void*)plan, S(st)); });
    });
    m.def("lu_dist_step", [](char dt, i64 nr, uintptr_t W, i64 ldw, uintptr_t grow, int c0, int c1, int j,
                             uintptr_t recs, int p, uintptr_t Tt, i64 ldt, uintptr_t ipiv, uintptr_t info,
                             i64 info_off, double thr, uintptr_t rec, uintptr_t part, i64 diag_local, uintptr_t st) {
        dispatch(dt, [&](auto z) { using T = decltype(z);
            lu_dist_step<T>(nr, P<T>(W), ldw, P<const i64>(grow), c0, c1, j, P<const T>(recs), p, P<T>(Tt), ldt,
                            P<i64>(ipiv), P<i64>(info), info_off, thr, P<T>(rec), (void*)part, diag_local, S(st)); });
    });
    m.def("lu_dist_base", [](char dt, i64 nr, uintptr_t W, i64 ldw, uintptr_t grow, int c0, int c1, uintptr_t Tt,
                             i64 ldt, uintptr_t ipiv, uintptr_t info, i64 info_off, double thr, uintptr_t mbox, int p,
                             int me, uintptr_t part, long long seq0, int has_diag, uintptr_t err, int G, uintptr_t st) {
        LuPeer pe{P<const unsigned long long>(mbox), p, me, P<char>(part), seq0, has_diag, P<unsigned long long>(err)};
        dispatch(dt, [&](auto z) { using T = decltype(z);
            lu_dist_base<T>(nr, P<T>(W), ldw, P<const i64>(grow), c0, c1, P<T>(Tt), ldt, P<i64>(ipiv), P<i64>(info),
                            info_off, thr, pe, G, S(st)); });
    });
    m.def("lu_peer_sizes", []() {
        return py::make_tuple((i64)lu_peer_mailbox_bytes(), (i64)lu_peer_part_bytes(), lu_peer_max_b(), lu_peer_max_p());
    });
    m.def("lu_peer_alloc", [](i64 bytes) {
        char h[64];
        void* p = lu_peer_alloc((size_t)bytes, h);
        return py::make_tuple((uintptr_t)p, py::bytes(h, 64));
    });
    m.def("lu_peer_open", [](py::bytes h) {
        std::string hs = h;
        if (hs.size() != 64) throw std::invalid_argument("lu_peer_open: 64-byte handle expected");
        return (uintptr_t)lu_peer_open(hs.data());
    });
    m.def("lu_peer_close", [](uintptr_t p) { lu_peer_close((void*)p); });
    m.def("lu_peer_free", [](uintptr_t p) { lu_peer_free((void*)p); });
    m.def("spin_ns", [](double ns, uintptr_t st) { spin_ns(ns, S(st)); });
    m.def("row_gather", [](char dt, i64 mm, i64 n, uintptr_t A, i64 lda, uintptr_t B, i64 ldb, uintptr_t perm,
                           uintptr_t st) {
        dispatch(dt, [&](auto z) { using T = decltype(z);
            permute_rows_gather<T>(mm, n, P<T>(A), lda, P<T>(B), ldb, P<const i64>(perm), S(st)); });
    });
    m.def("row_scatter", [](char dt, i64 mm, i64 n, uintptr_t A, i64 lda, uintptr_t B, i64 ldb, uintptr_t perm,
                            uintptr_t st) {
        dispatch(dt, [&](auto z) { using T = decltype(z);
            permute_rows_scatter<T>(mm, n, P<T>(A), lda, P<T>(B), ldb, P<const i64>(perm), S(st)); });
    });
    m.def("swap_plan_bytes", []() { return (i64)swap_plan_bytes(); });
    m.def("swap_plan", [](i64 k1, i64 k2, uintptr_t ipiv, i64 ioff, int incx, uintptr_t plan, uintptr_t st) {
        swap_plan(k1, k2, P<const i64>(ipiv), ioff, incx, (void*)plan, S(st)); });
    m.def("xchg_gather", [](char dt, uintptr_t plan, i64 nslot, i64 n, uintptr_t A, i64 lda, uintptr_t X, i64 ldx,
                            i64 nb, int p, int pr, uintptr_t st) {
        dispatch(dt, [&](auto z) { using T = decltype(z);
            xchg_gather<T>((const void*)plan, nslot, n, P<const T>(A), lda, P<T>(X), ldx, nb, p, pr, S(st)); });
    });
    m.def("xchg_scatter", [](char dt, uintptr_t plan, i64 nslot, i64 n, uintptr_t X, i64 ldx, uintptr_t A, i64 lda,
                             i64 nb, int p, int pr, uintptr_t st) {
        dispatch(dt, [&](auto z) { using T = decltype(z);
            xchg_scatter<T>((const void*)plan, nslot, n, P<const T>(X), ldx, P<T>(A), lda, nb, p, pr, S(st)); });
    });
    m.def("sel_to_ipiv", [](uintptr_t sel, i64 kb, i64 r0, uintptr_t ipiv, uintptr_t st) {
        sel_to_ipiv(P<const i64>(sel), kb, r0, P<i64>(ipiv), S(st)); });
    m.def("geset", [](char dt, char uplo, i64 mm, i64 n, std::complex<double> off, std::complex<double> diag,
                      uintptr_t A, i64 lda, uintptr_t st) {
        dispatch(dt, [&](auto z) { using T = decltype(z);
            geset<T>(uplo, mm, n, cv<T>(off), cv<T>(diag), P<T>(A), lda, S(st)); });
    });
    m.def("gescale", [](char dt, char uplo, i64 mm, i64 n, std::complex<double> a, uintptr_t A, i64 lda, uintptr_t st) {
        dispatch(dt, [&](auto z) { using T = decltype(z); gescale<T>(uplo, mm, n, cv<T>(a), P<T>(A), lda, S(st)); });
    });
    m.def("geadd", [](char dt, char uplo, i64 mm, i64 n, std::complex<double> a, uintptr_t A, i64 lda,
                      std::complex<double> b, uintptr_t B, i64 ldb, uintptr_t st) {
        dispatch(dt, [&](auto z) { using T = decltype(z);
            geadd<T>(uplo, mm, n, cv<T>(a), P<T>(A), lda, cv<T>(b), P<T>(B), ldb, S(st)); });
    });
    m.def("gecopy_mask", [](char dt, py::object mask, i64 mm, i64 n, uintptr_t A, i64 lda, uintptr_t B, i64 ldb,
                            int real_diag, uintptr_t st) {
        const TriMask mk = make_mask(mask);
        dispatch(dt, [&](auto z) { using T = decltype(z);
            gecopy_mask<T>(mk, mm, n, P<T>(A), lda, P<T>(B), ldb, real_diag != 0, S(st)); });
    });
    m.def("gecopy", [](char ds, char dd, char uplo, char trans, i64 mm, i64 n, uintptr_t A, i64 lda, uintptr_t B,
                       i64 ldb, uintptr_t st) {
        dispatch(ds, [&](auto zs) { using Ts = decltype(zs);
            dispatch(dd, [&](auto zd) { using Td = decltype(zd);
                constexpr bool ok = !(scalar_traits<Ts>::is_complex && !scalar_traits<Td>::is_complex) ||
                                    true;
                (void)ok;
                if constexpr ((std::is_same<Ts, float>::value || std::is_same<Ts, double>::value) &&
                              (std::is_same<Td, float>::value || std::is_same<Td, double>::value))
                    gecopy<Ts, Td>(uplo, trans, mm, n, P<Ts>(A), lda, P<Td>(B), ldb, S(st));
                else if constexpr (scalar_traits<Ts>::is_complex && scalar_traits<Td>::is_complex)
                    gecopy<Ts, Td>(uplo, trans, mm, n, P<Ts>(A), lda, P<Td>(B), ldb, S(st));
                else if constexpr (std::is_same<Ts, float>::value && std::is_same<Td, ccplx>::value)
                    gecopy<Ts, Td>(uplo, trans, mm, n, P<Ts>(A), lda, P<Td>(B), ldb, S(st));
                else if constexpr (std::is_same<Ts, double>::value && std::is_same<Td, zcplx>::value)
                    gecopy<Ts, Td>(uplo, trans, mm, n, P<Ts>(A), lda, P<Td>(B), ldb, S(st));
                else if constexpr (std::is_same<Ts, zcplx>::value && std::is_same<Td, double>::value)
                    gecopy<Ts, Td>(uplo, trans, mm, n, P<Ts>(A), lda, P<Td>(B), ldb, S(st));
                else if constexpr (std::is_same<Ts, ccplx>::value && std::is_same<Td, float>::value)
                    gecopy<Ts, Td>(uplo, trans, mm, n, P<Ts>(A), lda, P<Td>(B), ldb, S(st));
                else
                    throw std::invalid_argument("gecopy: unsupported conversion");
            });
        });
    });
    m.def("gescale_row_col", [](char dt, char equed, i64 mm, i64 n, uintptr_t r, uintptr_t c, uintptr_t A, i64 lda,
                                uintptr_t st) {
        dispatch(dt, [&](auto z) { using T = decltype(z); using R = typename scalar_traits<T>::real;
            gescale_row_col<T, R>(equed, mm, n, P<R>(r), P<R>(c), P<T>(A), lda, S(st)); });
    });
    m.def("butterfly", [](char dt, bool trans, bool rows, int depth, i64 nidx, i64 nother, uintptr_t A, i64 lda,
                          uintptr_t diag, i64 ldd, uintptr_t st) {
        dispatch(dt, [&](auto z) { using T = decltype(z); using R = typename scalar_traits<T>::real;
            butterfly<T, R>(trans, rows, depth, nidx, nother, P<T>(A), lda, P<R>(diag), ldd, S(st)); });
    });
    m.def("genorm", [](char dt, char norm, char uplo, char diag, int herm, i64 mm, i64 n, uintptr_t A, i64 lda,
                       uintptr_t out, uintptr_t st) {
        dispatch(dt, [&](auto z) { using T = decltype(z); using R = typename scalar_traits<T>::real;
            genorm<T, R>(norm, uplo, diag, herm, mm, n, P<T>(A), lda, P<R>(out), S(st)); });
    });
    m.def("matgen", [](char dt, int kind, uint64_t seed, i64 mloc, i64 nloc, uintptr_t A, i64 lda, i64 gm, i64 gn,
                       i64 mb, int p, int pr, i64 nb, int q, int pc, i64 row0, i64 col0, double scale, uintptr_t st) {
        dispatch(dt, [&](auto z) { using T = decltype(z);
            matgen<T>(kind, seed, mloc, nloc, P<T>(A), lda, gm, gn, mb, p, pr, nb, q, pc, row0, col0, scale, S(st)); });
    });
}

__global__ void placement_probe_kernel(unsigned* out) {
    if (threadIdx.x == 0) {
        unsigned hw = __builtin_amdgcn_s_getreg((4) | (0 << 6) | (31 << 11));    // HW_REG_HW_ID
        unsigned xcc = __builtin_amdgcn_s_getreg((20) | (0 << 6) | (15 << 11));  // HW_REG_XCC_ID
        out[2 * blockIdx.x] = hw;
        out[2 * blockIdx.x + 1] = xcc;
        // keep the block resident briefly so blocks spread over CUs
        __builtin_amdgcn_s_sleep(127);
    }
}

PYBIND11_MODULE(_hip, m) {
    m.doc() = "slate_amd gfx950 HIP kernels";
    m.attr("arch") = "gfx950";
    m.def("gemm", &py_gemm);
    m.def("gemm_ptrs", &py_gemm_ptrs);
    register_kernels(m);
    register_devpool(m);
    // CU-masked streams: isolate latency-bound panel kernels from the bulk
    // trailing-update GEMM (hipExtStreamCreateWithCUMask).  Returns the raw
    // handle for torch.cuda.ExternalStream.
    m.def("stream_create_cu_mask", [](int device, std::vector<uint32_t> mask) {
        int old = 0;
        HIP_CHECK(hipGetDevice(&old));
        HIP_CHECK(hipSetDevice(device));
        hipStream_t st;
        HIP_CHECK(hipExtStreamCreateWithCUMask(&st, (uint32_t)mask.size(), mask.data()));
        HIP_CHECK(hipSetDevice(old));
        return (uintptr_t)st;
    });
    m.def("stream_destroy", [](uintptr_t st) { HIP_CHECK(hipStreamDestroy((hipStream_t)st)); });
    // a private non-blocking stream (not from torch's round-robin pool): a
    // captured graph owns one, so no other launcher ever shares the
    // per-stream workspaces its kernels point into (workspace.hpp)
    m.def("stream_create", [](int device) {
        int old = 0;
        HIP_CHECK(hipGetDevice(&old));
        HIP_CHECK(hipSetDevice(device));
        hipStream_t st;
        HIP_CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
        HIP_CHECK(hipSetDevice(old));
        return (uintptr_t)st;
    });
    m.def("cu_count", [](int device) {
        hipDeviceProp_t pr;
        HIP_CHECK(hipGetDeviceProperties(&pr, device));
        return pr.multiProcessorCount;
    });
    m.def("placement_probe", [](uintptr_t out, int nblocks, uintptr_t st) {
        // raw (HW_ID, XCC_ID) register values of each block: maps CU-mask
        // bits / block ids to XCDs and CUs
        hipLaunchKernelGGL(placement_probe_kernel, dim3(nblocks), dim3(64), 0, (hipStream_t)st,
                           reinterpret_cast<unsigned*>(out));
        HIP_LAUNCH_CHECK();
    });
}
