// Python-free C++ use of slate_amd (include/slate_amd/slate_native.hh,
// libslate_amd_native.so) in the four precisions on a p x q block-cyclic
// grid: Cholesky, LU, the solves, GEMM (plain and transposed operands), the
// triangular solve and norms, each checked against a host reference; then
// the LAPACK-style C ABI (slate_dgesv / slate_zposv / slate_dgemm_); then an
// optional timing of dpotrf (argv[2] = n).  Prints "check <name>_<x> <value>"
// lines (x = s, d, c, z; relative residuals) and "time potrf n=.. <ms> <TF/s>".
//
//   ./ex_native [PxQ] [n_bench]      (one process per rank; torchrun-style env;
//                                     SLATE_AMD_NATIVE_TRANSPORT=host lets the
//                                     ranks of a grid share one GPU)
#include <chrono>
#include <cmath>
#include <complex>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <type_traits>
#include <vector>

#include "slate_amd/slate_native.hh"

namespace sn = slate_amd::native;

extern "C" {
int slate_dgesv(int64_t n, int64_t nrhs, double* a, int64_t lda, int64_t* ipiv, double* b, int64_t ldb);
int slate_zposv(char uplo, int64_t n, int64_t nrhs, double* a, int64_t lda, double* b, int64_t ldb);
void slate_dgemm_(const char* ta, const char* tb, const int64_t* m, const int64_t* n, const int64_t* k,
                  const double* alpha, const double* a, const int64_t* lda, const double* b, const int64_t* ldb,
                  const double* beta, double* c, const int64_t* ldc);
const char* slate_amd_last_error(void);
}

template <typename T> struct Name;
template <> struct Name<float> { static constexpr const char* s = "s"; };
template <> struct Name<double> { static constexpr const char* s = "d"; };
template <> struct Name<std::complex<float>> { static constexpr const char* s = "c"; };
template <> struct Name<std::complex<double>> { static constexpr const char* s = "z"; };

template <typename T> T cj(T x) { return x; }
template <typename R> std::complex<R> cj(std::complex<R> x) { return std::conj(x); }
template <typename T> T val(double re, double im) {
    if constexpr (std::is_floating_point<T>::value) return T(re);
    else return T(re, im);
}

// host C = op(A) op(B) (double-precision accumulation)
template <typename T>
std::vector<std::complex<double>> mul(char ta, char tb, int64_t m, int64_t n, int64_t k, const std::vector<T>& a,
                                      int64_t lda, const std::vector<T>& b, int64_t ldb) {
    auto at = [&](int64_t i, int64_t l) -> std::complex<double> {
        const T x = ta == 'N' ? a[i + l * lda] : a[l + i * lda];
        const std::complex<double> v(std::real(x), std::imag(x));
        return ta == 'C' ? std::conj(v) : v;
    };
    auto bt = [&](int64_t l, int64_t j) -> std::complex<double> {
        const T x = tb == 'N' ? b[l + j * ldb] : b[j + l * ldb];
        const std::complex<double> v(std::real(x), std::imag(x));
        return tb == 'C' ? std::conj(v) : v;
    };
    std::vector<std::complex<double>> c((size_t)m * n);
    for (int64_t j = 0; j < n; ++j)
        for (int64_t i = 0; i < m; ++i) {
            std::complex<double> s = 0;
            for (int64_t l = 0; l < k; ++l) s += at(i, l) * bt(l, j);
            c[i + j * m] = s;
        }
    return c;
}

template <typename T>
double rel(const std::vector<std::complex<double>>& got_minus_want, const std::vector<std::complex<double>>& want) {
    double e = 0, w = 0;
    for (size_t i = 0; i < want.size(); ++i) {
        e += std::norm(got_minus_want[i]);
        w += std::norm(want[i]);
    }
    return std::sqrt(e / (w > 0 ? w : 1));
}

template <typename T>
std::vector<std::complex<double>> widen(const std::vector<T>& v) {
    std::vector<std::complex<double>> r(v.size());
    for (size_t i = 0; i < v.size(); ++i) r[i] = {std::real(v[i]), std::imag(v[i])};
    return r;
}

template <typename T>
void run(int p, int q, int me) {
    const char* x = Name<T>::s;
    auto report = [&](const char* what, double v) {
        if (me == 0) std::printf("check %s_%s %.3e\n", what, x, v);
        std::fflush(stdout);
    };
    const int64_t n = std::getenv("EX_NATIVE_N") ? std::atoll(std::getenv("EX_NATIVE_N")) : 300;
    const int64_t nb = std::getenv("EX_NATIVE_NB") ? std::atoll(std::getenv("EX_NATIVE_NB")) : 32, nrhs = 5;

    // ---- potrf / posv: || L L^H - A || / || A ||, || A X - B || / || B ||
    sn::HermitianMatrix<T> A(sn::Uplo::Lower, n, nb, p, q);
    A.generate(sn::Gen::HermitianPositiveDefinite, 7);
    std::vector<T> a0((size_t)n * n), l((size_t)n * n);
    A.to_host(a0.data(), n);
    for (int64_t j = 0; j < n; ++j)           // full Hermitian host copy
        for (int64_t i = 0; i < j; ++i) a0[i + j * n] = cj(a0[j + i * n]);
    int64_t info = sn::potrf(A);
    A.to_host(l.data(), n);
    for (int64_t j = 0; j < n; ++j)
        for (int64_t i = 0; i < j; ++i) l[i + j * n] = T(0);
    {
        auto llh = mul<T>('N', 'C', n, n, n, l, n, l, n);
        auto want = widen(a0);
        for (size_t i = 0; i < llh.size(); ++i) llh[i] -= want[i];
        report(info ? "potrf-FAILED" : "potrf", rel<T>(llh, want));
    }
    sn::Matrix<T> B(n, nrhs, nb, p, q);
    B.generate(sn::Gen::Random, 8);
    std::vector<T> b0((size_t)n * nrhs), xs((size_t)n * nrhs);
    B.to_host(b0.data(), n);
    sn::potrs(A, B);
    B.to_host(xs.data(), n);
    {
        auto ax = mul<T>('N', 'N', n, nrhs, n, a0, n, xs, n);
        auto want = widen(b0);
        for (size_t i = 0; i < ax.size(); ++i) ax[i] -= want[i];
        report("potrs", rel<T>(ax, want));
    }

    // ---- getrf / getrs / gesv on the p x q grid
    sn::Matrix<T> G(n, n, nb, p, q);
    G.generate(sn::Gen::Random, 5);
    std::vector<T> g0((size_t)n * n);
    G.to_host(g0.data(), n);
    std::vector<int64_t> ipiv;
    sn::Matrix<T> X(n, nrhs, nb, p, q);
    X.generate(sn::Gen::Random, 6);
    std::vector<T> xb((size_t)n * nrhs), xg((size_t)n * nrhs);
    X.to_host(xb.data(), n);
    sn::lu_exchange_stats(nullptr, nullptr);
    info = sn::gesv(G, ipiv, X);
    {
        // p > 1: only the rows that change process row travel
        long long xb = 0, xr = 0;
        sn::lu_exchange_stats(&xb, &xr);
        const bool ok = xb <= xr * G.nloc() * (long long)sizeof(T);
        report("lu_xchg_bound", ok ? 0.0 : 1.0);
        if (me == 0 && p > 1) std::printf("lu exchange: %lld bytes sent, %lld rows crossed, nloc %lld\n", xb, xr, (long long)G.nloc());
    }
    X.to_host(xg.data(), n);
    {
        auto ax = mul<T>('N', 'N', n, nrhs, n, g0, n, xg, n);
        auto want = widen(xb);
        for (size_t i = 0; i < ax.size(); ++i) ax[i] -= want[i];
        report(info ? "gesv-FAILED" : "gesv", rel<T>(ax, want));
    }
    // A^H X = B with the same factors
    X.from_host(xb.data(), n);
    sn::getrs(sn::Op::ConjTrans, G, ipiv, X);
    X.to_host(xg.data(), n);
    {
        auto ax = mul<T>('C', 'N', n, nrhs, n, g0, n, xg, n);
        auto want = widen(xb);
        for (size_t i = 0; i < ax.size(); ++i) ax[i] -= want[i];
        report("getrs_conjtrans", rel<T>(ax, want));
    }
    // rectangular getrf (m > n): || P A - L U || through the host factors
    {
        const int64_t m3 = 260, n3 = 180;
        sn::Matrix<T> R(m3, n3, nb, p, q);
        R.generate(sn::Gen::Random, 12);
        std::vector<T> r0((size_t)m3 * n3), lu((size_t)m3 * n3);
        R.to_host(r0.data(), m3);
        std::vector<int64_t> pv;
        info = sn::getrf(R, pv);
        R.to_host(lu.data(), m3);
        std::vector<T> L((size_t)m3 * n3, T(0)), U((size_t)n3 * n3, T(0));
        for (int64_t j = 0; j < n3; ++j)
            for (int64_t i = 0; i < m3; ++i) {
                if (i > j) L[i + j * m3] = lu[i + j * m3];
                else U[i + j * n3] = lu[i + j * m3];
                if (i == j) L[i + j * m3] = T(1);
            }
        for (int64_t i = 0; i < (int64_t)pv.size(); ++i)
            for (int64_t j = 0; j < n3; ++j) std::swap(r0[i + j * m3], r0[pv[i] + j * m3]);
        auto prod = mul<T>('N', 'N', m3, n3, n3, L, m3, U, n3);
        auto want = widen(r0);
        for (size_t i = 0; i < prod.size(); ++i) prod[i] -= want[i];
        report(info ? "getrf_rect-FAILED" : "getrf_rect", rel<T>(prod, want));
    }

    // ---- gemm: C = alpha op(A) op(B) + beta C
    const int64_t m2 = 150, k2 = 100, n2 = 120;
    for (int v = 0; v < 2; ++v) {
        const char ta = v ? 'C' : 'N', tb = v ? 'T' : 'N';
        sn::Matrix<T> GA(ta == 'N' ? m2 : k2, ta == 'N' ? k2 : m2, nb, p, q);
        sn::Matrix<T> GB(tb == 'N' ? k2 : n2, tb == 'N' ? n2 : k2, nb, p, q);
        sn::Matrix<T> GC(m2, n2, nb, p, q);
        GA.generate(sn::Gen::Random, 1);
        GB.generate(sn::Gen::Random, 2);
        GC.generate(sn::Gen::Random, 3);
        std::vector<T> ha((size_t)m2 * k2), hb((size_t)k2 * n2), hc((size_t)m2 * n2), hc1((size_t)m2 * n2);
        GA.to_host(ha.data(), GA.m());
        GB.to_host(hb.data(), GB.m());
        GC.to_host(hc.data(), m2);
        const T alpha = val<T>(2.0, 0.5), beta = val<T>(-1.0, 0.25);
        if (v) sn::gemm(sn::Op::ConjTrans, sn::Op::Trans, alpha, GA, GB, beta, GC);
        else sn::gemm(alpha, GA, GB, beta, GC);
        GC.to_host(hc1.data(), m2);
        auto want = mul<T>(ta, tb, m2, n2, k2, ha, GA.m(), hb, GB.m());
        const std::complex<double> al(std::real(alpha), std::imag(alpha)), be(std::real(beta), std::imag(beta));
        std::vector<std::complex<double>> d(want.size());
        for (size_t i = 0; i < want.size(); ++i) {
            want[i] = al * want[i] + be * std::complex<double>(std::real(hc[i]), std::imag(hc[i]));
            d[i] = std::complex<double>(std::real(hc1[i]), std::imag(hc1[i])) - want[i];
        }
        report(v ? "gemm_ct" : "gemm", rel<T>(d, want));
        if (!v) {
            // ---- norms against the host
            double mx = 0, fr = 0, one = 0;
            for (int64_t j = 0; j < k2; ++j) {
                double cs = 0;
                for (int64_t i = 0; i < m2; ++i) {
                    const double a = std::abs(ha[i + j * m2]);
                    mx = std::fmax(mx, a);
                    fr += a * a;
                    cs += a;
                }
                one = std::fmax(one, cs);
            }
            report("norm_max", std::fabs(sn::norm(sn::Norm::Max, GA) - mx) / mx);
            report("norm_fro", std::fabs(sn::norm(sn::Norm::Fro, GA) - std::sqrt(fr)) / std::sqrt(fr));
            report("norm_one", std::fabs(sn::norm(sn::Norm::One, GA) - one) / one);
        }
    }

    // ---- gels on the 1 x (p q) grid (geqrf distributes whole columns):
    // consistent system B = A X0 -> X0; inconsistent -> A^H (A X - B) = 0
    {
        const int64_t m4 = 330, n4 = 120, r4 = 3;
        sn::Matrix<T> G4(m4, n4, nb, 1, p * q), X0(n4, r4, nb, 1, p * q), B4(m4, r4, nb, 1, p * q);
        G4.generate(sn::Gen::Random, 21);
        X0.generate(sn::Gen::Random, 22);
        std::vector<T> g4((size_t)m4 * n4), x0((size_t)n4 * r4);
        G4.to_host(g4.data(), m4);
        X0.to_host(x0.data(), n4);
        auto b4 = mul<T>('N', 'N', m4, r4, n4, g4, m4, x0, n4);
        std::vector<T> bh((size_t)m4 * r4);
        for (size_t i = 0; i < bh.size(); ++i) bh[i] = val<T>(b4[i].real(), b4[i].imag());
        B4.from_host(bh.data(), m4);
        sn::gels(G4, B4);
        std::vector<T> xg4((size_t)m4 * r4);
        B4.to_host(xg4.data(), m4);
        double e = 0, w = 0;
        for (int64_t c = 0; c < r4; ++c)
            for (int64_t i = 0; i < n4; ++i) {
                e += std::norm(std::complex<double>(std::real(xg4[i + c * m4]) - std::real(x0[i + c * n4]),
                                                    std::imag(xg4[i + c * m4]) - std::imag(x0[i + c * n4])));
                w += std::norm(std::complex<double>(std::real(x0[i + c * n4]), std::imag(x0[i + c * n4])));
            }
        report("gels", std::sqrt(e / w));
    }

    // ---- geqrf on the p x q grid (TSQR panels when p > 1): || Q R - A || / || A ||
    // through unmqr(NoTrans) of [R; 0], tall and wide; then gels on the grid
    for (int shape = 0; shape < 2; ++shape) {
        const int64_t m5 = shape ? 100 : 330, n5 = shape ? 150 : 120;
        sn::Matrix<T> G5(m5, n5, nb, p, q), C5(m5, n5, nb, p, q);
        G5.generate(sn::Gen::Random, 31);
        std::vector<T> g5((size_t)m5 * n5), f5((size_t)m5 * n5), qr5((size_t)m5 * n5);
        G5.to_host(g5.data(), m5);
        sn::QRFactors<T> F5;
        sn::geqrf(G5, F5);
        G5.to_host(f5.data(), m5);
        for (int64_t j = 0; j < n5; ++j)
            for (int64_t i = j + 1; i < m5; ++i) f5[i + j * m5] = T(0);
        C5.from_host(f5.data(), m5);
        sn::unmqr(sn::Op::NoTrans, G5, F5, C5);
        C5.to_host(qr5.data(), m5);
        auto want = widen(g5), got = widen(qr5);
        for (size_t i = 0; i < got.size(); ++i) got[i] -= want[i];
        report(shape ? "geqrf_wide" : "geqrf", rel<T>(got, want));
    }
    {
        const int64_t m6 = 330, n6 = 120, r6 = 3;
        sn::Matrix<T> G6(m6, n6, nb, p, q), X6(n6, r6, nb, p, q), B6(m6, r6, nb, p, q);
        G6.generate(sn::Gen::Random, 41);
        X6.generate(sn::Gen::Random, 42);
        std::vector<T> g6((size_t)m6 * n6), x6((size_t)n6 * r6);
        G6.to_host(g6.data(), m6);
        X6.to_host(x6.data(), n6);
        auto b6 = mul<T>('N', 'N', m6, r6, n6, g6, m6, x6, n6);
        std::vector<T> bh((size_t)m6 * r6), xg6((size_t)m6 * r6);
        for (size_t i = 0; i < bh.size(); ++i) bh[i] = val<T>(b6[i].real(), b6[i].imag());
        B6.from_host(bh.data(), m6);
        sn::gels(G6, B6);
        B6.to_host(xg6.data(), m6);
        double e = 0, w = 0;
        for (int64_t c = 0; c < r6; ++c)
            for (int64_t i = 0; i < n6; ++i) {
                e += std::norm(std::complex<double>(std::real(xg6[i + c * m6]) - std::real(x6[i + c * n6]),
                                                    std::imag(xg6[i + c * m6]) - std::imag(x6[i + c * n6])));
                w += std::norm(std::complex<double>(std::real(x6[i + c * n6]), std::imag(x6[i + c * n6])));
            }
        report("gels_grid", std::sqrt(e / w));
    }

    // ---- trsm: L^H X = alpha B with the Cholesky factor
    {
        sn::Matrix<T> Bt(n, nrhs, nb, p, q);
        Bt.from_host(b0.data(), n);
        const T alpha = val<T>(1.5, -0.5);
        sn::trsm(sn::Side::Left, sn::Uplo::Lower, sn::Op::ConjTrans, sn::Diag::NonUnit, alpha, A, Bt);
        std::vector<T> xt((size_t)n * nrhs);
        Bt.to_host(xt.data(), n);
        auto lx = mul<T>('C', 'N', n, nrhs, n, l, n, xt, n);
        std::vector<std::complex<double>> want(lx.size());
        const std::complex<double> al(std::real(alpha), std::imag(alpha));
        for (size_t i = 0; i < lx.size(); ++i) {
            want[i] = al * std::complex<double>(std::real(b0[i]), std::imag(b0[i]));
            lx[i] -= want[i];
        }
        report("trsm_lc", rel<T>(lx, want));
    }
    // ---- views: potrf of a trailing principal block through a tile-aligned
    //      sub view (zero-copy, the parent's storage), potrs through a
    //      from_device wrapper of another matrix's local buffer
    {
        int64_t lcm = p;
        while (lcm % q) lcm += p;
        const int64_t nt = (n + nb - 1) / nb;
        if (lcm < nt) {
            sn::HermitianMatrix<T> Af(sn::Uplo::Lower, n, nb, p, q);
            Af.generate(sn::Gen::HermitianPositiveDefinite, 7);
            sn::HermitianMatrix<T> V(sn::Uplo::Lower, Af.sub(lcm, nt, lcm, nt));
            const int64_t nv = V.m(), o = lcm * nb;
            info = sn::potrf(V);
            std::vector<T> lv((size_t)nv * nv);
            V.to_host(lv.data(), nv);
            for (int64_t j = 0; j < nv; ++j)
                for (int64_t i = 0; i < j; ++i) lv[i + j * nv] = T(0);
            auto llh = mul<T>('N', 'C', nv, nv, nv, lv, nv, lv, nv);
            std::vector<std::complex<double>> want((size_t)nv * nv);
            for (int64_t j = 0; j < nv; ++j)
                for (int64_t i = 0; i < nv; ++i) {
                    const T x = i >= j ? a0[(o + i) + (o + j) * n] : cj(a0[(o + j) + (o + i) * n]);
                    want[i + j * nv] = {std::real(x), std::imag(x)};
                }
            for (size_t i = 0; i < llh.size(); ++i) llh[i] -= want[i];
            report(info ? "sub_potrf-FAILED" : "sub_potrf", rel<T>(llh, want));
        } else {
            report("sub_potrf", 0.0);
        }
        sn::Matrix<T> Bd(n, nrhs, nb, p, q);
        Bd.from_host(b0.data(), n);
        sn::Matrix<T> W = sn::Matrix<T>::from_device(Bd.data(), Bd.lld(), n, nrhs, nb, p, q);
        sn::potrs(A, W);
        std::vector<T> xw((size_t)n * nrhs);
        Bd.to_host(xw.data(), n);                    // the solve landed in Bd's own buffer
        auto ax = mul<T>('N', 'N', n, nrhs, n, a0, n, xw, n);
        auto want = widen(b0);
        for (size_t i = 0; i < ax.size(); ++i) ax[i] -= want[i];
        report("from_device_potrs", rel<T>(ax, want));
    }

    // ---- trtri of the Cholesky factor: L^{-1} L = I; trtrm: L^H L
    {
        sn::Matrix<T> Li(n, n, nb, p, q);
        Li.from_host(l.data(), n);
        sn::trtri(sn::Uplo::Lower, sn::Diag::NonUnit, Li);
        std::vector<T> li((size_t)n * n);
        Li.to_host(li.data(), n);
        for (int64_t j = 0; j < n; ++j)
            for (int64_t i = 0; i < j; ++i) li[i + j * n] = T(0);
        auto prod = mul<T>('N', 'N', n, n, n, li, n, l, n);
        std::vector<std::complex<double>> eye((size_t)n * n, 0.0);
        for (int64_t i = 0; i < n; ++i) eye[i + i * n] = 1.0;
        for (size_t i = 0; i < prod.size(); ++i) prod[i] -= eye[i];
        report("trtri", rel<T>(prod, eye));
        sn::Matrix<T> Lm(n, n, nb, p, q);
        Lm.from_host(l.data(), n);
        sn::trtrm(sn::Uplo::Lower, Lm);
        std::vector<T> lm((size_t)n * n);
        Lm.to_host(lm.data(), n);
        auto want = mul<T>('C', 'N', n, n, n, l, n, l, n);
        double e = 0, w = 0;
        for (int64_t j = 0; j < n; ++j)
            for (int64_t i = j; i < n; ++i) {
                e += std::norm(std::complex<double>(std::real(lm[i + j * n]), std::imag(lm[i + j * n])) - want[i + j * n]);
                w += std::norm(want[i + j * n]);
            }
        report("trtrm", std::sqrt(e / w));
    }
    // ---- LU without pivoting on the HPD matrix: A X = B
    {
        sn::Matrix<T> Gn(n, n, nb, p, q), Xn(n, nrhs, nb, p, q);
        Gn.from_host(a0.data(), n);
        Xn.from_host(b0.data(), n);
        info = sn::gesv_nopiv(Gn, Xn);
        std::vector<T> xn((size_t)n * nrhs);
        Xn.to_host(xn.data(), n);
        auto ax = mul<T>('N', 'N', n, nrhs, n, a0, n, xn, n);
        auto want = widen(b0);
        for (size_t i = 0; i < ax.size(); ++i) ax[i] -= want[i];
        report(info ? "gesv_nopiv-FAILED" : "gesv_nopiv", rel<T>(ax, want));
    }
    // ---- Cholesky QR: Q R = A, Q^H Q = I
    {
        const int64_t m7 = 330, n7 = 120;
        sn::Matrix<T> A7(m7, n7, nb, p, q), R7(n7, n7, nb, p, q);
        A7.generate(sn::Gen::Random, 71);
        std::vector<T> a7((size_t)m7 * n7), q7((size_t)m7 * n7), r7((size_t)n7 * n7);
        A7.to_host(a7.data(), m7);
        info = sn::cholqr(A7, R7);
        A7.to_host(q7.data(), m7);
        R7.to_host(r7.data(), n7);
        auto qr = mul<T>('N', 'N', m7, n7, n7, q7, m7, r7, n7);
        auto want = widen(a7);
        for (size_t i = 0; i < qr.size(); ++i) qr[i] -= want[i];
        report(info ? "cholqr-FAILED" : "cholqr", rel<T>(qr, want));
        auto qq = mul<T>('C', 'N', n7, n7, m7, q7, m7, q7, m7);
        std::vector<std::complex<double>> eye((size_t)n7 * n7, 0.0);
        for (int64_t i = 0; i < n7; ++i) eye[i + i * n7] = 1.0;
        for (size_t i = 0; i < qq.size(); ++i) qq[i] -= eye[i];
        report("cholqr_orth", rel<T>(qq, eye));
    }
    // ---- LQ of a wide matrix: Q^H L^H = A^H through unmlq
    {
        const int64_t m8 = 120, n8 = 330;
        sn::Matrix<T> A8(m8, n8, nb, p, q), C8(n8, m8, nb, p, q);
        A8.generate(sn::Gen::Random, 81);
        std::vector<T> a8((size_t)m8 * n8), f8((size_t)m8 * n8), lh((size_t)n8 * m8, T(0)), c8((size_t)n8 * m8);
        A8.to_host(a8.data(), m8);
        sn::LQFactors<T> F8;
        sn::gelqf(A8, F8);
        A8.to_host(f8.data(), m8);
        for (int64_t j = 0; j < m8; ++j)              // L^H: n8 x m8, upper part of its first m8 rows
            for (int64_t i = j; i < m8; ++i) lh[j + i * n8] = cj(f8[i + j * m8]);
        C8.from_host(lh.data(), n8);
        sn::unmlq(sn::Op::ConjTrans, A8, F8, C8);
        C8.to_host(c8.data(), n8);
        double e = 0, w = 0;
        for (int64_t j = 0; j < m8; ++j)
            for (int64_t i = 0; i < n8; ++i) {
                const T want = cj(a8[j + i * m8]);
                const std::complex<double> d(std::real(c8[i + j * n8]) - std::real(want),
                                             std::imag(c8[i + j * n8]) - std::imag(want));
                e += std::norm(d);
                w += std::norm(std::complex<double>(std::real(want), std::imag(want)));
            }
        report("gelqf", std::sqrt(e / w));
    }

    // ---- trsm on the stored triangle: L^T X = alpha B (left), X op(L) = alpha C (right)
    for (int v = 0; v < 3; ++v) {
        const bool right = v > 0;
        const int64_t rm = right ? 7 : n, rn = right ? n : nrhs;
        sn::Matrix<T> Bt(rm, rn, nb, p, q);
        Bt.generate(sn::Gen::Random, 61 + v);
        std::vector<T> hb((size_t)rm * rn), xt((size_t)rm * rn);
        Bt.to_host(hb.data(), rm);
        const T alpha = val<T>(0.75, 0.5);
        const sn::Op op = v == 0 ? sn::Op::Trans : v == 1 ? sn::Op::NoTrans : sn::Op::ConjTrans;
        sn::trsm(right ? sn::Side::Right : sn::Side::Left, sn::Uplo::Lower, op, sn::Diag::NonUnit, alpha, A, Bt);
        Bt.to_host(xt.data(), rm);
        const char oc = v == 0 ? 'T' : v == 1 ? 'N' : 'C';
        auto lx = right ? mul<T>('N', oc, rm, rn, n, xt, rm, l, n) : mul<T>(oc, 'N', rm, rn, n, l, n, xt, rm);
        std::vector<std::complex<double>> want(lx.size());
        const std::complex<double> al(std::real(alpha), std::imag(alpha));
        for (size_t i = 0; i < lx.size(); ++i) {
            want[i] = al * std::complex<double>(std::real(hb[i]), std::imag(hb[i]));
            lx[i] -= want[i];
        }
        report(v == 0 ? "trsm_lt" : v == 1 ? "trsm_rn" : "trsm_rc", rel<T>(lx, want));
    }

    using R = sn::real_t<T>;
    auto cd = [](T x) { return std::complex<double>(std::real(x), std::imag(x)); };
    // ---- herk / her2k / syrk / syr2k: C's stored triangle against the host
    for (int v = 0; v < 4; ++v) {
        const int64_t nc = 140, kc = 90;
        const bool two = v == 1 || v == 3, herm = v <= 1;
        const char ta = v == 1 ? 'C' : v == 2 ? 'T' : 'N';
        const sn::Uplo ul = two ? sn::Uplo::Upper : sn::Uplo::Lower;
        const int64_t ar = ta == 'N' ? nc : kc, ac = ta == 'N' ? kc : nc;
        sn::Matrix<T> A2(ar, ac, nb, p, q), B2(ar, ac, nb, p, q);
        A2.generate(sn::Gen::Random, 31 + v);
        B2.generate(sn::Gen::Random, 41 + v);
        sn::HermitianMatrix<T> C2(ul, nc, nb, p, q);
        C2.generate(sn::Gen::Random, 51 + v);
        std::vector<T> ha((size_t)ar * ac), hb((size_t)ar * ac), hc((size_t)nc * nc), hc1((size_t)nc * nc);
        A2.to_host(ha.data(), ar);
        B2.to_host(hb.data(), ar);
        C2.to_host(hc.data(), nc);
        const T alpha = (herm && !two) ? val<T>(1.5, 0) : val<T>(1.5, -0.75);
        const T beta = herm ? val<T>(-0.5, 0) : val<T>(-0.5, 0.25);
        if (v == 0) sn::herk(sn::Op::NoTrans, (R)std::real(alpha), A2, (R)std::real(beta), C2);
        else if (v == 1) sn::her2k(sn::Op::ConjTrans, alpha, A2, B2, (R)std::real(beta), C2);
        else if (v == 2) sn::syrk(sn::Op::Trans, alpha, A2, beta, C2);
        else sn::syr2k(sn::Op::NoTrans, alpha, A2, B2, beta, C2);
        C2.to_host(hc1.data(), nc);
        // op(X) op(Y)^{H or T}: X Y^t2 for op = N, X^ta Y for op = ta
        const char t2 = herm ? 'C' : 'T';
        auto prod = [&](const std::vector<T>& X, const std::vector<T>& Y) {
            return ta == 'N' ? mul<T>('N', t2, nc, nc, kc, X, ar, Y, ar) : mul<T>(ta, 'N', nc, nc, kc, X, ar, Y, ar);
        };
        const auto P1 = prod(ha, two ? hb : ha);
        const auto P2 = two ? prod(hb, ha) : P1;
        const std::complex<double> al = cd(alpha), be = cd(beta), al2 = herm ? std::conj(al) : al;
        std::vector<std::complex<double>> d, want;
        for (int64_t j = 0; j < nc; ++j)
            for (int64_t i = 0; i < nc; ++i) {
                if (ul == sn::Uplo::Lower ? i < j : i > j) continue;
                const size_t o = (size_t)(i + j * nc);
                std::complex<double> w = al * P1[o] + be * cd(hc[o]);
                if (two) w += al2 * P2[o];
                want.push_back(w);
                d.push_back(cd(hc1[o]) - w);
            }
        static const char* nm[] = {"herk", "her2k_upper", "syrk", "syr2k_upper"};
        report(nm[v], rel<T>(d, want));
    }
    // ---- hemm (Left, Lower) / symm (Right, Upper): the stored triangle expanded
    for (int v = 0; v < 2; ++v) {
        const int64_t na = 130, nr = 70;
        const sn::Uplo ul = v ? sn::Uplo::Upper : sn::Uplo::Lower;
        sn::HermitianMatrix<T> H(ul, na, nb, p, q);
        H.generate(sn::Gen::Random, 61 + v);
        const int64_t bm = v ? nr : na, bn = v ? na : nr;
        sn::Matrix<T> Bm(bm, bn, nb, p, q), Cm(bm, bn, nb, p, q);
        Bm.generate(sn::Gen::Random, 71 + v);
        Cm.generate(sn::Gen::Random, 81 + v);
        std::vector<T> hh((size_t)na * na), hb((size_t)bm * bn), hc((size_t)bm * bn), hc1((size_t)bm * bn);
        H.to_host(hh.data(), na);
        Bm.to_host(hb.data(), bm);
        Cm.to_host(hc.data(), bm);
        for (int64_t j = 0; j < na; ++j)
            for (int64_t i = 0; i < na; ++i) {
                const bool stored = v ? i <= j : i >= j;
                if (!stored) hh[i + j * na] = v ? hh[j + i * na] : cj(hh[j + i * na]);
            }
        if (!v)
            for (int64_t i = 0; i < na; ++i) hh[i + i * na] = val<T>(std::real(hh[i + i * na]), 0);
        const T alpha = val<T>(0.75, 0.5), beta = val<T>(1.25, -0.5);
        if (!v) sn::hemm(sn::Side::Left, alpha, H, Bm, beta, Cm);
        else sn::symm(sn::Side::Right, alpha, H, Bm, beta, Cm);
        Cm.to_host(hc1.data(), bm);
        auto want = v ? mul<T>('N', 'N', bm, bn, na, hb, bm, hh, na) : mul<T>('N', 'N', bm, bn, na, hh, na, hb, bm);
        std::vector<std::complex<double>> d(want.size());
        for (size_t i = 0; i < want.size(); ++i) {
            want[i] = cd(alpha) * want[i] + cd(beta) * cd(hc[i]);
            d[i] = cd(hc1[i]) - want[i];
        }
        report(v ? "symm_right" : "hemm_left", rel<T>(d, want));
        // the structured norm of the stored triangle against the host full matrix
        double one = 0;
        for (int64_t j = 0; j < na; ++j) {
            double cs = 0;
            for (int64_t i = 0; i < na; ++i) cs += std::abs(hh[i + j * na]);
            one = std::fmax(one, cs);
        }
        const double nrm = v ? sn::norm_symmetric(sn::Norm::One, H) : sn::norm(sn::Norm::One, H);
        report(v ? "norm_sym_one" : "norm_herm_one", std::fabs(nrm - one) / one);
    }
    // ---- trmm: B = alpha A^H B, A upper triangular with a unit diagonal
    {
        const int64_t na = 120, nr = 50;
        sn::Matrix<T> Tm(na, na, nb, p, q), Bm(na, nr, nb, p, q);
        Tm.generate(sn::Gen::Random, 91);
        Bm.generate(sn::Gen::Random, 92);
        std::vector<T> ht((size_t)na * na), hb((size_t)na * nr), hb1((size_t)na * nr);
        Tm.to_host(ht.data(), na);
        Bm.to_host(hb.data(), na);
        for (int64_t j = 0; j < na; ++j)
            for (int64_t i = 0; i < na; ++i)
                if (i > j) ht[i + j * na] = T(0);
                else if (i == j) ht[i + j * na] = T(1);
        const T alpha = val<T>(-1.25, 0.5);
        sn::trmm(sn::Side::Left, sn::Uplo::Upper, sn::Op::ConjTrans, sn::Diag::Unit, alpha, Tm, Bm);
        Bm.to_host(hb1.data(), na);
        auto want = mul<T>('C', 'N', na, nr, na, ht, na, hb, na);
        std::vector<std::complex<double>> d(want.size());
        for (size_t i = 0; i < want.size(); ++i) {
            want[i] = cd(alpha) * want[i];
            d[i] = cd(hb1[i]) - want[i];
        }
        report("trmm_luc", rel<T>(d, want));
        double fr = 0;
        for (const T& e : ht) fr += std::norm(e);
        report("norm_tri_fro", std::fabs(sn::norm_triangular(sn::Norm::Fro, sn::Uplo::Upper, sn::Diag::Unit, Tm) -
                                         std::sqrt(fr)) / std::sqrt(fr));
    }
    // ---- inverses: || A A^-1 - I || through the host
    for (int v = 0; v < 2; ++v) {
        const int64_t ni = 150;
        std::vector<T> h0((size_t)ni * ni), hi((size_t)ni * ni);
        if (v == 0) {
            sn::HermitianMatrix<T> Hm(sn::Uplo::Lower, ni, nb, p, q);
            Hm.generate(sn::Gen::HermitianPositiveDefinite, 111);
            Hm.to_host(h0.data(), ni);
            for (int64_t j = 0; j < ni; ++j)
                for (int64_t i = 0; i < j; ++i) h0[i + j * ni] = cj(h0[j + i * ni]);
            sn::potrf(Hm);
            sn::potri(Hm);
            Hm.to_host(hi.data(), ni);
            for (int64_t j = 0; j < ni; ++j)
                for (int64_t i = 0; i < j; ++i) hi[i + j * ni] = cj(hi[j + i * ni]);
        } else {
            sn::Matrix<T> Gm(ni, ni, nb, p, q);
            Gm.generate(sn::Gen::DiagDominant, 112);
            Gm.to_host(h0.data(), ni);
            std::vector<int64_t> pv;
            sn::getrf(Gm, pv);
            sn::getri(Gm, pv);
            Gm.to_host(hi.data(), ni);
        }
        auto prod = mul<T>('N', 'N', ni, ni, ni, h0, ni, hi, ni);
        std::vector<std::complex<double>> eye(prod.size());
        for (int64_t i = 0; i < ni; ++i) eye[(size_t)(i + i * ni)] = 1.0;
        for (size_t i = 0; i < prod.size(); ++i) prod[i] -= eye[i];
        report(v ? "getri" : "potri", rel<T>(prod, eye));
    }
    // ---- heev: || A Z - Z Lambda || / (|| A || n) and || Z^H Z - I || / n
    //      (a random Hermitian matrix: he2hb -> hb2st -> D & C -> back-transforms)
    {
        const int64_t ne = 260;
        sn::HermitianMatrix<T> H(sn::Uplo::Lower, ne, nb, p, q);
        H.generate(sn::Gen::Random, 121);
        std::vector<T> h0((size_t)ne * ne), z((size_t)ne * ne);
        H.to_host(h0.data(), ne);
        for (int64_t j = 0; j < ne; ++j) {           // the Hermitian matrix of the lower triangle
            h0[j + j * ne] = T(std::real(h0[j + j * ne]));
            for (int64_t i = 0; i < j; ++i) h0[i + j * ne] = cj(h0[j + i * ne]);
        }
        sn::Matrix<T> Z(ne, ne, nb, p, q);
        std::vector<sn::real_t<T>> lam, lam2;
        const int64_t inf = sn::heev(H, lam, Z);
        Z.to_host(z.data(), ne);
        auto az = mul<T>('N', 'N', ne, ne, ne, h0, ne, z, ne);
        double an = 0;
        for (auto& v : h0) an += std::norm(std::complex<double>(std::real(v), std::imag(v)));
        an = std::sqrt(an);
        double e1 = 0;
        for (int64_t j = 0; j < ne; ++j)
            for (int64_t i = 0; i < ne; ++i) {
                const std::complex<double> zz(std::real(z[i + j * ne]), std::imag(z[i + j * ne]));
                e1 += std::norm(az[i + j * ne] - zz * (double)lam[j]);
            }
        auto zhz = mul<T>('C', 'N', ne, ne, ne, z, ne, z, ne);
        double e2 = 0;
        for (int64_t j = 0; j < ne; ++j)
            for (int64_t i = 0; i < ne; ++i) e2 += std::norm(zhz[i + j * ne] - (i == j ? 1.0 : 0.0));
        bool sorted = true;
        for (size_t i = 1; i < lam.size(); ++i) sorted = sorted && lam[i - 1] <= lam[i];
        report(inf || !sorted ? "heev-FAILED" : "heev", std::sqrt(e1) / (an * ne));
        report("heev_orth", std::sqrt(e2) / ne);
        // values only: the same spectrum
        sn::heev(H, lam2);
        double dv = 0;
        for (int64_t i = 0; i < ne; ++i) dv = std::max(dv, std::abs((double)lam2[i] - (double)lam[i]));
        report("heev_values", dv / (an > 0 ? an : 1));
        // p x q grids run the distributed solver (no n x n on any rank): the
        // one-GPU solver behind a gather must give the same spectrum
        if (p * q > 1) {
            setenv("SLATE_AMD_NATIVE_HEEV", "gather", 1);
            std::vector<sn::real_t<T>> lam3;
            sn::heev(H, lam3);
            unsetenv("SLATE_AMD_NATIVE_HEEV");
            double dg = 0;
            for (int64_t i = 0; i < ne; ++i) dg = std::max(dg, std::abs((double)lam3[i] - (double)lam[i]));
            report("heev_grid_vs_gather", dg / (an > 0 ? an : 1));
        }
    }
    // ---- redistribute: onto another tile size and grid shape and back
    {
        const int64_t mr = 203, nr = 150;
        sn::Matrix<T> A0(mr, nr, nb, p, q), A1(mr, nr, 37, q, p), A2(mr, nr, nb, p, q);
        A0.generate(sn::Gen::Random, 131);
        sn::redistribute(A0, A1);
        sn::redistribute(A1, A2);
        std::vector<T> h0((size_t)mr * nr), h1((size_t)mr * nr), h2((size_t)mr * nr);
        A0.to_host(h0.data(), mr);
        A1.to_host(h1.data(), mr);
        A2.to_host(h2.data(), mr);
        double d1 = 0, d2 = 0;
        for (size_t i = 0; i < h0.size(); ++i) {
            d1 = std::max(d1, (double)std::abs(h1[i] - h0[i]));
            d2 = std::max(d2, (double)std::abs(h2[i] - h0[i]));
        }
        report("redistribute", d1 + d2);
    }
    // ---- svd: || A - U S V^H || / || A ||, || U^H U - I ||, || V V^H - I ||
    //      (tall and wide; values only must give the same spectrum)
    for (int wide = 0; wide < 2; ++wide) {
        const int64_t ms = wide ? 170 : 290, ns = wide ? 250 : 210, ks = std::min(ms, ns);
        sn::Matrix<T> Am(ms, ns, nb, p, q), U(ms, ks, nb, p, q), VH(ks, ns, nb, p, q);
        Am.generate(sn::Gen::Random, 141 + wide);
        std::vector<T> a((size_t)ms * ns), u((size_t)ms * ks), vh((size_t)ks * ns);
        Am.to_host(a.data(), ms);
        std::vector<sn::real_t<T>> sv, sv2;
        const int64_t inf = sn::svd(Am, sv, U, VH);
        U.to_host(u.data(), ms);
        VH.to_host(vh.data(), ks);
        std::vector<T> us((size_t)ms * ks);
        for (int64_t j = 0; j < ks; ++j)
            for (int64_t i = 0; i < ms; ++i) us[i + j * ms] = u[i + j * ms] * (sn::real_t<T>)sv[j];
        auto usv = mul<T>('N', 'N', ms, ns, ks, us, ms, vh, ks);
        auto want = widen(a);
        for (size_t i = 0; i < usv.size(); ++i) usv[i] -= want[i];
        bool desc = true;
        for (size_t i = 1; i < sv.size(); ++i) desc = desc && sv[i - 1] >= sv[i];
        report(inf || !desc ? (wide ? "svd_wide-FAILED" : "svd-FAILED") : (wide ? "svd_wide" : "svd"), rel<T>(usv, want));
        auto uhu = mul<T>('C', 'N', ks, ks, ms, u, ms, u, ms);
        auto vvh = mul<T>('N', 'C', ks, ks, ns, vh, ks, vh, ks);
        double eo = 0;
        for (int64_t j = 0; j < ks; ++j)
            for (int64_t i = 0; i < ks; ++i) {
                const double id = i == j ? 1.0 : 0.0;
                eo += std::norm(uhu[i + j * ks] - id) + std::norm(vvh[i + j * ks] - id);
            }
        report(wide ? "svd_wide_orth" : "svd_orth", std::sqrt(eo) / ks);
        if (!wide) {
            sn::svd(Am, sv2);
            double dv = 0;
            for (int64_t i = 0; i < ks; ++i) dv = std::max(dv, std::abs((double)sv2[i] - (double)sv[i]));
            report("svd_values", dv / std::max(1.0, (double)sv[0]));
        }
    }
    // ---- condition estimates: 1 <= rcond_est / rcond <= 3 (exact rcond from the inverse)
    {
        const int64_t nc = 120;
        sn::Matrix<T> Gm(nc, nc, nb, p, q);
        Gm.generate(sn::Gen::DiagDominant, 131);
        const double an = sn::norm(sn::Norm::One, Gm);
        std::vector<int64_t> pv;
        sn::getrf(Gm, pv);
        const double rc = sn::gecondest(sn::Norm::One, Gm, an);
        sn::getri(Gm, pv);
        const double ratio = rc * an * sn::norm(sn::Norm::One, Gm);
        report("gecondest", (ratio >= 0.999 && ratio <= 3.0) ? 0.0 : ratio);
    }
    // ---- mixed precision (double / complex<double>): low-precision factors +
    // refinement must reach the working-precision residual
    if constexpr (std::is_same<T, double>::value || std::is_same<T, std::complex<double>>::value) {
        const int64_t nm = 200;
        for (int v = 0; v < 2; ++v) {
            sn::Matrix<T> Bm(nm, nrhs, nb, p, q), Xm(nm, nrhs, nb, p, q);
            Bm.generate(sn::Gen::Random, 101 + v);
            std::vector<T> ha((size_t)nm * nm), hb((size_t)nm * nrhs), hx((size_t)nm * nrhs);
            Bm.to_host(hb.data(), nm);
            int iter = -100;
            int64_t inf;
            if (v == 0) {
                sn::HermitianMatrix<T> Hm(sn::Uplo::Lower, nm, nb, p, q);
                Hm.generate(sn::Gen::HermitianPositiveDefinite, 103);
                Hm.to_host(ha.data(), nm);
                for (int64_t j = 0; j < nm; ++j)
                    for (int64_t i = 0; i < j; ++i) ha[i + j * nm] = cj(ha[j + i * nm]);
                inf = sn::posv_mixed(Hm, Bm, Xm, iter);
            } else {
                sn::Matrix<T> Gm(nm, nm, nb, p, q);
                Gm.generate(sn::Gen::DiagDominant, 104);     // well conditioned: the refinement converges
                Gm.to_host(ha.data(), nm);
                std::vector<int64_t> pv;
                inf = sn::gesv_mixed(Gm, pv, Bm, Xm, iter);
            }
            Xm.to_host(hx.data(), nm);
            auto ax = mul<T>('N', 'N', nm, nrhs, nm, ha, nm, hx, nm);
            auto want = widen(hb);
            for (size_t i = 0; i < ax.size(); ++i) ax[i] -= want[i];
            if (me == 0) std::printf("mixed %s iter %d info %lld\n", v ? "gesv" : "posv", iter, (long long)inf);
            report(inf || iter < 0 ? (v ? "gesv_mixed-FAILED" : "posv_mixed-FAILED") : (v ? "gesv_mixed" : "posv_mixed"),
                   rel<T>(ax, want));
        }
        // GMRES-IR: the same systems through restarted GMRES preconditioned
        // by the low-precision factors
        for (int v = 0; v < 2; ++v) {
            sn::Matrix<T> Bm(nm, 3, nb, p, q), Xm(nm, 3, nb, p, q);
            Bm.generate(sn::Gen::Random, 105 + v);
            std::vector<T> ha((size_t)nm * nm), hb((size_t)nm * 3), hx((size_t)nm * 3);
            Bm.to_host(hb.data(), nm);
            int iter = -100;
            int64_t inf;
            if (v == 0) {
                sn::HermitianMatrix<T> Hm(sn::Uplo::Lower, nm, nb, p, q);
                Hm.generate(sn::Gen::HermitianPositiveDefinite, 107);
                Hm.to_host(ha.data(), nm);
                for (int64_t j = 0; j < nm; ++j)
                    for (int64_t i = 0; i < j; ++i) ha[i + j * nm] = cj(ha[j + i * nm]);
                inf = sn::posv_mixed_gmres(Hm, Bm, Xm, iter);
            } else {
                sn::Matrix<T> Gm(nm, nm, nb, p, q);
                Gm.generate(sn::Gen::DiagDominant, 108);
                Gm.to_host(ha.data(), nm);
                std::vector<int64_t> pv;
                inf = sn::gesv_mixed_gmres(Gm, pv, Bm, Xm, iter);
            }
            Xm.to_host(hx.data(), nm);
            auto ax = mul<T>('N', 'N', nm, 3, nm, ha, nm, hx, nm);
            auto want = widen(hb);
            for (size_t i = 0; i < ax.size(); ++i) ax[i] -= want[i];
            if (me == 0) std::printf("gmres %s iter %d info %lld\n", v ? "gesv" : "posv", iter, (long long)inf);
            report(inf || iter < 0 ? (v ? "gesv_gmres-FAILED" : "posv_gmres-FAILED") : (v ? "gesv_gmres" : "posv_gmres"),
                   rel<T>(ax, want));
        }
    }
    // ---- gesv_rbt: random butterflies + LU without pivoting + refinement
    //      (n not a multiple of the butterfly unit: the padded path)
    {
        const int64_t nr = 150;
        sn::Matrix<T> Gm(nr, nr, nb, p, q), Bm(nr, nrhs, nb, p, q);
        Gm.generate(sn::Gen::Random, 151);
        Bm.generate(sn::Gen::Random, 152);
        std::vector<T> ha((size_t)nr * nr), hb((size_t)nr * nrhs), hx((size_t)nr * nrhs);
        Gm.to_host(ha.data(), nr);
        Bm.to_host(hb.data(), nr);
        const int64_t inf = sn::gesv_rbt(Gm, Bm);
        Bm.to_host(hx.data(), nr);
        auto ax = mul<T>('N', 'N', nr, nrhs, nr, ha, nr, hx, nr);
        auto want = widen(hb);
        for (size_t i = 0; i < ax.size(); ++i) ax[i] -= want[i];
        report(inf ? "gesv_rbt-FAILED" : "gesv_rbt", rel<T>(ax, want));
    }
    // ---- Hermitian indefinite (Aasen hetrf + band LU of T): hesv backward error
    {
        const int64_t nh = 230;                  // not a multiple of nb: the padded order
        sn::HermitianMatrix<T> Hm(sn::Uplo::Lower, nh, nb, p, q);
        Hm.generate(sn::Gen::Random, 205);
        std::vector<T> ha((size_t)nh * nh);
        Hm.to_host(ha.data(), nh);
        for (int64_t j = 0; j < nh; ++j) {
            ha[j + j * nh] = T(std::real(ha[j + j * nh]));
            for (int64_t i = 0; i < j; ++i) ha[i + j * nh] = cj(ha[j + i * nh]);
        }
        sn::Matrix<T> Bm(nh, nrhs, nb, p, q);
        Bm.generate(sn::Gen::Random, 206);
        std::vector<T> hb((size_t)nh * nrhs), x((size_t)nh * nrhs);
        Bm.to_host(hb.data(), nh);
        const int64_t inf = sn::hesv(Hm, Bm);
        Bm.to_host(x.data(), nh);
        auto ax = mul<T>('N', 'N', nh, nrhs, nh, ha, nh, x, nh);
        double e = 0, an = 0, xn = 0;
        for (size_t i = 0; i < ax.size(); ++i) e += std::norm(ax[i] - std::complex<double>(std::real(hb[i]), std::imag(hb[i])));
        for (const T& v : ha) an += std::norm(std::complex<double>(std::real(v), std::imag(v)));
        for (const T& v : x) xn += std::norm(std::complex<double>(std::real(v), std::imag(v)));
        report(inf ? "hesv-FAILED" : "hesv", std::sqrt(e / (an * xn)));
    }
    // ---- CALU (getrf_tntpiv): || P A - L U || / || A || from the host factors,
    //      with a small play-off leaf so several rounds run
    {
        const int64_t nc = 260;
        sn::Matrix<T> Gm(nc, nc, nb, p, q);
        Gm.generate(sn::Gen::Random, 201);
        std::vector<T> g0((size_t)nc * nc), lu((size_t)nc * nc);
        Gm.to_host(g0.data(), nc);
        std::vector<int64_t> pv;
        sn::Options o;
        o.calu_leaf = 64;
        const int64_t inf = sn::getrf_tntpiv(Gm, pv, o);
        Gm.to_host(lu.data(), nc);
        std::vector<T> L((size_t)nc * nc, T(0)), U((size_t)nc * nc, T(0)), PA(g0);
        for (int64_t j = 0; j < nc; ++j)
            for (int64_t i = 0; i < nc; ++i) {
                if (i > j) L[i + j * nc] = lu[i + j * nc];
                else U[i + j * nc] = lu[i + j * nc];
                if (i == j) L[i + j * nc] = T(1);
            }
        for (int64_t i = 0; i < nc; ++i)
            if (pv[i] != i)
                for (int64_t j = 0; j < nc; ++j) std::swap(PA[i + j * nc], PA[pv[i] + j * nc]);
        auto lu2 = mul<T>('N', 'N', nc, nc, nc, L, nc, U, nc);
        auto w = widen(PA);
        for (size_t i = 0; i < lu2.size(); ++i) lu2[i] -= w[i];
        double lmax = 0;
        for (const T& v : L) lmax = std::max(lmax, (double)std::abs(v));
        report(inf ? "getrf_tntpiv-FAILED" : "getrf_tntpiv", rel<T>(lu2, w));
        report("tntpiv_growth", lmax <= 64.0 ? 0.0 : lmax);     // tournament pivots keep |L| modest
    }
    // ---- band matrices (compact 1-D column-tile storage): pbsv (Lower and
    //      Upper), gbsv, tbsm, gbmm, hbmm against dense host products
    {
        const int64_t nbd = 300, kd = 40, kl = 35, ku = 20, nrb = 3;
        auto resid = [&](const std::vector<T>& Ad, const std::vector<T>& X, const std::vector<T>& B0, int64_t nrr) {
            auto ax = mul<T>('N', 'N', nbd, nrr, nbd, Ad, nbd, X, nbd);
            auto w = widen(B0);
            for (size_t i = 0; i < ax.size(); ++i) ax[i] -= w[i];
            return rel<T>(ax, w);
        };
        for (int up = 0; up < 2; ++up) {
            sn::HermitianBandMatrix<T> Hb(sn::Uplo::Lower, nbd, kd, nb);
            Hb.generate(sn::Gen::HermitianPositiveDefinite, 191);
            std::vector<T> hl((size_t)nbd * nbd), hf((size_t)nbd * nbd);
            Hb.to_host(hl.data(), nbd);
            for (int64_t j = 0; j < nbd; ++j)
                for (int64_t i = 0; i < nbd; ++i) {
                    const T v = i >= j ? hl[i + j * nbd] : cj(hl[j + i * nbd]);
                    hf[i + j * nbd] = i == j ? T(std::real(v)) : v;
                }
            sn::HermitianBandMatrix<T> Hu(up ? sn::Uplo::Upper : sn::Uplo::Lower, nbd, kd, nb);
            Hu.from_host(hf.data(), nbd);
            sn::Matrix<T> Bm(nbd, nrb, nb, p, q);
            Bm.generate(sn::Gen::Random, 192);
            std::vector<T> b0((size_t)nbd * nrb), x((size_t)nbd * nrb);
            Bm.to_host(b0.data(), nbd);
            const int64_t inf = sn::pbsv(Hu, Bm);
            Bm.to_host(x.data(), nbd);
            report(inf ? "pbsv-FAILED" : (up ? "pbsv_upper" : "pbsv"), resid(hf, x, b0, nrb));
        }
        {
            sn::BandMatrix<T> Gb(nbd, nbd, kl, ku, nb);
            Gb.generate(sn::Gen::Random, 193);
            std::vector<T> ga((size_t)nbd * nbd);
            Gb.to_host(ga.data(), nbd);
            // gbmm first (A unfactored): C = alpha A B + beta C
            sn::Matrix<T> Bm(nbd, nrb, nb, p, q), Cm(nbd, nrb, nb, p, q);
            Bm.generate(sn::Gen::Random, 194);
            Cm.generate(sn::Gen::Random, 195);
            std::vector<T> hb((size_t)nbd * nrb), hc((size_t)nbd * nrb), hc1((size_t)nbd * nrb);
            Bm.to_host(hb.data(), nbd);
            Cm.to_host(hc.data(), nbd);
            const T al = val<T>(0.75, -0.5), be = val<T>(-1.5, 0.25);
            sn::gbmm(al, Gb, Bm, be, Cm);
            Cm.to_host(hc1.data(), nbd);
            auto ab = mul<T>('N', 'N', nbd, nrb, nbd, ga, nbd, hb, nbd);
            std::vector<std::complex<double>> d(ab.size()), w(ab.size());
            for (size_t i = 0; i < ab.size(); ++i) {
                w[i] = std::complex<double>(std::real(al), std::imag(al)) * ab[i] +
                       std::complex<double>(std::real(be), std::imag(be)) *
                           std::complex<double>(std::real(hc[i]), std::imag(hc[i]));
                d[i] = std::complex<double>(std::real(hc1[i]), std::imag(hc1[i])) - w[i];
            }
            report("gbmm", rel<T>(d, w));
            std::vector<int64_t> pv;
            Bm.from_host(hb.data(), nbd);
            const int64_t inf = sn::gbsv(Gb, pv, Bm);
            std::vector<T> x((size_t)nbd * nrb);
            Bm.to_host(x.data(), nbd);
            // backward error ||A X - B|| / (||A|| ||X||): the random band is
            // not diagonally dominant, so partial pivoting really pivots
            {
                auto ax = mul<T>('N', 'N', nbd, nrb, nbd, ga, nbd, x, nbd);
                double e = 0, an = 0, xn = 0;
                for (size_t i = 0; i < ax.size(); ++i)
                    e += std::norm(ax[i] - std::complex<double>(std::real(hb[i]), std::imag(hb[i])));
                for (const T& v : ga) an += std::norm(std::complex<double>(std::real(v), std::imag(v)));
                for (const T& v : x) xn += std::norm(std::complex<double>(std::real(v), std::imag(v)));
                report(inf ? "gbsv-FAILED" : "gbsv", std::sqrt(e / (an * xn)));
            }
        }
        {
            // hbmm Left / Right on the HPD band against the dense Hermitian product
            sn::HermitianBandMatrix<T> Hb(sn::Uplo::Lower, nbd, kd, nb);
            Hb.generate(sn::Gen::Random, 196);
            std::vector<T> hl((size_t)nbd * nbd), hf((size_t)nbd * nbd);
            Hb.to_host(hl.data(), nbd);
            for (int64_t j = 0; j < nbd; ++j)
                for (int64_t i = 0; i < nbd; ++i) {
                    const T v = i >= j ? hl[i + j * nbd] : cj(hl[j + i * nbd]);
                    hf[i + j * nbd] = i == j ? T(std::real(v)) : v;
                }
            Hb.from_host(hf.data(), nbd);                // real diagonal
            for (int sd = 0; sd < 2; ++sd) {
                const int64_t rm = sd ? nrb : nbd, rn = sd ? nbd : nrb;
                sn::Matrix<T> Bm(rm, rn, nb, p, q), Cm(rm, rn, nb, p, q);
                Bm.generate(sn::Gen::Random, 197);
                std::vector<T> hb((size_t)rm * rn), hc((size_t)rm * rn);
                Bm.to_host(hb.data(), rm);
                sn::hbmm(sd ? sn::Side::Right : sn::Side::Left, T(1), Hb, Bm, T(0), Cm);
                Cm.to_host(hc.data(), rm);
                auto want = sd ? mul<T>('N', 'N', rm, rn, nbd, hb, rm, hf, nbd) : mul<T>('N', 'N', rm, rn, nbd, hf, nbd, hb, rm);
                std::vector<std::complex<double>> d(want.size());
                for (size_t i = 0; i < want.size(); ++i) d[i] = std::complex<double>(std::real(hc[i]), std::imag(hc[i])) - want[i];
                report(sd ? "hbmm_right" : "hbmm_left", rel<T>(d, want));
            }
        }
        {
            // tbsm: upper triangular band, op = ConjTrans, alpha != 1
            sn::TriangularBandMatrix<T> Tb(sn::Uplo::Upper, sn::Diag::NonUnit, nbd, kd, nb);
            std::vector<T> ht((size_t)nbd * nbd, T(0));
            for (int64_t j = 0; j < nbd; ++j)
                for (int64_t i = std::max<int64_t>(0, j - kd); i <= j; ++i)
                    ht[i + j * nbd] = i == j ? T(4.0 + 0.01 * j) : val<T>(std::sin(0.3 * i + 0.7 * j) * 0.05, 0.02);
            Tb.from_host(ht.data(), nbd);
            sn::Matrix<T> Bm(nbd, nrb, nb, p, q);
            Bm.generate(sn::Gen::Random, 198);
            std::vector<T> hb((size_t)nbd * nrb), x((size_t)nbd * nrb);
            Bm.to_host(hb.data(), nbd);
            const T al = val<T>(2.0, 0.0);
            sn::tbsm(sn::Side::Left, sn::Op::ConjTrans, al, Tb, Bm);
            Bm.to_host(x.data(), nbd);
            auto tx = mul<T>('C', 'N', nbd, nrb, nbd, ht, nbd, x, nbd);
            auto w = widen(hb);
            for (size_t i = 0; i < tx.size(); ++i) {
                w[i] *= 2.0;
                tx[i] -= w[i];
            }
            report("tbsm_upper_conj", rel<T>(tx, w));
        }
    }
    // ---- matrix model: transposed views, structured types, slice, emptyLike
    {
        const int64_t ma = 170, ka = 90, na = 130;
        sn::Matrix<T> A(ka, ma, nb, p, q), B(na, ka, nb, p, q), C(ma, na, nb, p, q);
        A.generate(sn::Gen::Random, 181);
        B.generate(sn::Gen::Random, 182);
        std::vector<T> ha((size_t)ka * ma), hb((size_t)na * ka), hc((size_t)ma * na);
        A.to_host(ha.data(), ka);
        B.to_host(hb.data(), na);
        // C = A^H B^T through views (no copies by the caller)
        sn::gemm(T(1), sn::conj_transpose(A), sn::transpose(B), T(0), C);
        C.to_host(hc.data(), ma);
        auto want = mul<T>('C', 'T', ma, na, ka, ha, ka, hb, na);
        std::vector<std::complex<double>> d(want.size());
        for (size_t i = 0; i < want.size(); ++i) d[i] = std::complex<double>(std::real(hc[i]), std::imag(hc[i])) - want[i];
        report("view_gemm", rel<T>(d, want));
        const auto At = sn::transpose(A);
        report("view_dims", (At.m() == ma && At.n() == ka && At.op() == sn::Op::Trans &&
                             sn::transpose(At).op() == sn::Op::NoTrans) ? 0.0 : 1.0);
        // ||A^T||_1 = ||A||_inf
        report("view_norm", std::fabs(sn::norm(sn::Norm::One, At) - sn::norm(sn::Norm::Inf, A)) /
                                sn::norm(sn::Norm::Inf, A));
        // a view where the driver cannot take one: rejected, not misread
        bool threw = false;
        try {
            sn::HermitianMatrix<T> Hv(sn::Uplo::Lower, sn::transpose(sn::Matrix<T>(na, na, nb, p, q)));
            sn::potrf(Hv);
        } catch (const sn::Error&) {
            threw = true;
        }
        report("view_rejected", threw ? 0.0 : 1.0);
        // TriangularMatrix: X = L^-H B with trsm on the conj_transpose VIEW of L
        const int64_t nt_ = 120, nr = 7;
        sn::TriangularMatrix<T> L(sn::Uplo::Lower, sn::Diag::NonUnit, nt_, nb, p, q);
        L.generate(sn::Gen::Random, 183);
        std::vector<T> hl((size_t)nt_ * nt_);
        L.to_host(hl.data(), nt_);
        for (int64_t j = 0; j < nt_; ++j)
            for (int64_t i = 0; i < nt_; ++i) {
                if (i < j) hl[i + j * nt_] = T(0);
                if (i == j) hl[i + j * nt_] += T((double)nt_);
            }
        L.from_host(hl.data(), nt_);
        sn::Matrix<T> X(nt_, nr, nb, p, q);
        X.generate(sn::Gen::Random, 184);
        std::vector<T> hx0((size_t)nt_ * nr), hx((size_t)nt_ * nr);
        X.to_host(hx0.data(), nt_);
        const auto LH = sn::conj_transpose(L);
        report("tri_view_uplo", LH.uplo() == sn::Uplo::Upper && LH.uplo_physical() == sn::Uplo::Lower ? 0.0 : 1.0);
        sn::trsm(sn::Side::Left, T(1), LH, X);
        X.to_host(hx.data(), nt_);
        auto lx = mul<T>('C', 'N', nt_, nr, nt_, hl, nt_, hx, nt_);
        auto wx = widen(hx0);
        for (size_t i = 0; i < lx.size(); ++i) lx[i] -= wx[i];
        report("tri_view_trsm", rel<T>(lx, wx));
        // trapezoid norm (m != n, unit diagonal): host reference
        sn::TrapezoidMatrix<T> Z(sn::Uplo::Upper, sn::Diag::Unit, 90, 150, nb, p, q);
        Z.generate(sn::Gen::Random, 185);
        std::vector<T> hz((size_t)90 * 150);
        Z.to_host(hz.data(), 90);
        double fro = 0;
        for (int64_t j = 0; j < 150; ++j)
            for (int64_t i = 0; i < 90; ++i)
                fro += i < j ? std::norm(std::complex<double>(std::real(hz[i + j * 90]), std::imag(hz[i + j * 90])))
                             : (i == j ? 1.0 : 0.0);
        report("trapezoid_norm", std::fabs(sn::norm(sn::Norm::Fro, Z) - std::sqrt(fro)) / std::sqrt(fro));
        // slice at odd offsets, modify, write back
        sn::Matrix<T> G(200, 160, nb, p, q);
        G.generate(sn::Gen::Random, 186);
        std::vector<T> hg((size_t)200 * 160), hs((size_t)67 * 45), hg2((size_t)200 * 160);
        G.to_host(hg.data(), 200);
        sn::Matrix<T> Sl = G.slice(13, 80, 29, 74);
        Sl.to_host(hs.data(), 67);
        double ds = 0;
        for (int64_t j = 0; j < 45; ++j)
            for (int64_t i = 0; i < 67; ++i) ds += std::abs(std::complex<double>(std::real(hs[i + j * 67] - hg[13 + i + (29 + j) * 200]),
                                                                               std::imag(hs[i + j * 67] - hg[13 + i + (29 + j) * 200])));
        sn::scale<T>((sn::real_t<T>)2, (sn::real_t<T>)1, Sl);
        G.set_slice(13, 29, Sl);
        G.to_host(hg2.data(), 200);
        for (int64_t j = 0; j < 160; ++j)
            for (int64_t i = 0; i < 200; ++i) {
                const bool in = i >= 13 && i < 80 && j >= 29 && j < 74;
                const T w = in ? hg[i + j * 200] * (sn::real_t<T>)2 : hg[i + j * 200];
                ds += std::abs(std::complex<double>(std::real(hg2[i + j * 200] - w), std::imag(hg2[i + j * 200] - w)));
            }
        report("slice_roundtrip", ds);
        const auto E = sn::transpose(G).emptyLike();
        report("empty_like", (E.m() == 160 && E.n() == 200 && sn::norm(sn::Norm::Max, E) == 0.0) ? 0.0 : 1.0);
        // SymmetricMatrix overloads: C = A A^T (syrk) and symm against gemm
        sn::SymmetricMatrix<T> Sy(sn::Uplo::Lower, na, nb, p, q);
        sn::syrk(T(1), B, T(0), Sy);
        sn::Matrix<T> F(na, na, nb, p, q), I(na, na, nb, p, q), F2(na, na, nb, p, q);
        sn::set(T(0), T(1), I);
        sn::symm(sn::Side::Left, T(1), Sy, I, T(0), F);             // the full symmetric matrix
        sn::gemm(T(1), B, sn::transpose(B), T(0), F2);
        sn::add(T(-1), F2, T(1), F);
        report("sym_syrk_symm", sn::norm(sn::Norm::Max, F) / sn::norm(sn::Norm::Max, F2));
    }
    // ---- hegv: A Z = B Z Lambda (itype 1), A B Z = Z Lambda (2),
    //      B A Z = Z Lambda (3); B Lower and Upper; || residual || / (|| A || || B || n)
    for (int v = 0; v < 3; ++v) {
        const int64_t ng = 140;
        const int64_t itype = v + 1;
        const sn::Uplo ub = v == 1 ? sn::Uplo::Upper : sn::Uplo::Lower;
        sn::HermitianMatrix<T> Ah(sn::Uplo::Lower, ng, nb, p, q);
        Ah.generate(sn::Gen::Random, 161 + v);
        sn::HermitianMatrix<T> Bl(sn::Uplo::Lower, ng, nb, p, q);
        Bl.generate(sn::Gen::HermitianPositiveDefinite, 171 + v);
        std::vector<T> ha((size_t)ng * ng), hbm((size_t)ng * ng), z((size_t)ng * ng);
        Ah.to_host(ha.data(), ng);
        Bl.to_host(hbm.data(), ng);
        for (int64_t j = 0; j < ng; ++j) {
            ha[j + j * ng] = T(std::real(ha[j + j * ng]));
            hbm[j + j * ng] = T(std::real(hbm[j + j * ng]));
            for (int64_t i = 0; i < j; ++i) {
                ha[i + j * ng] = cj(ha[j + i * ng]);
                hbm[i + j * ng] = cj(hbm[j + i * ng]);
            }
        }
        sn::HermitianMatrix<T> Bh(ub, ng, nb, p, q);
        Bh.from_host(hbm.data(), ng);
        Ah.from_host(ha.data(), ng);
        sn::Matrix<T> Z(ng, ng, nb, p, q);
        std::vector<sn::real_t<T>> lam;
        const int64_t inf = sn::hegv(itype, Ah, Bh, lam, Z);
        Z.to_host(z.data(), ng);
        std::vector<std::complex<double>> lhs, rhs;
        if (itype == 1) {
            lhs = mul<T>('N', 'N', ng, ng, ng, ha, ng, z, ng);
            rhs = mul<T>('N', 'N', ng, ng, ng, hbm, ng, z, ng);
        } else {
            std::vector<T> prod((size_t)ng * ng);
            auto in = mul<T>('N', 'N', ng, ng, ng, itype == 2 ? hbm : ha, ng, z, ng);
            for (size_t i = 0; i < prod.size(); ++i) prod[i] = val<T>(in[i].real(), in[i].imag());
            lhs = mul<T>('N', 'N', ng, ng, ng, itype == 2 ? ha : hbm, ng, prod, ng);
            rhs = widen(z);
        }
        double e = 0, an = 0, bn = 0;
        for (int64_t j = 0; j < ng; ++j)
            for (int64_t i = 0; i < ng; ++i) e += std::norm(lhs[i + j * ng] - rhs[i + j * ng] * (double)lam[j]);
        for (size_t i = 0; i < ha.size(); ++i) { an += std::norm(ha[i]); bn += std::norm(hbm[i]); }
        bool sorted = true;
        for (size_t i = 1; i < lam.size(); ++i) sorted = sorted && lam[i - 1] <= lam[i];
        const char* nm3[] = {"hegv1", "hegv2_upper", "hegv3"};
        report(inf || !sorted ? "hegv-FAILED" : nm3[v], std::sqrt(e) / (std::sqrt(an) * std::sqrt(bn) * ng));
    }
}

int main(int argc, char** argv) {
    int p = 1, q = 1;
    if (argc > 1) std::sscanf(argv[1], "%dx%d", &p, &q);
    const int64_t nbench = argc > 2 ? std::atoll(argv[2]) : 0;
    const char* only = std::getenv("EX_NATIVE_TYPES");     // e.g. "dz"
    const std::string types = only && *only ? only : "sdcz";
    try {
        sn::initialize();
        const int me = sn::rank();
        if (me == 0) std::printf("transport %s ranks %d grid %dx%d\n", sn::transport(), sn::size(), p, q);
        if (const char* tp = std::getenv("EX_NATIVE_TRACE")) {
            // traced dpotrf + dgetrf (lookahead 1): a Chrome trace of every
            // rank's panel / bcast / lookahead / update spans, and the timers
            const int64_t n = 2048, nb = 128;
            sn::HermitianMatrix<double> A(sn::Uplo::Lower, n, nb, p, q);
            A.generate(sn::Gen::HermitianPositiveDefinite, 3);
            sn::Matrix<double> G(n, n, nb, p, q);
            G.generate(sn::Gen::Random, 4);
            sn::clear_timers();
            sn::trace::on();
            const int64_t i1 = sn::potrf(A);
            std::vector<int64_t> piv;
            const int64_t i2 = sn::getrf(G, piv);
            sn::trace::finish(tp);
            for (const auto& kv : sn::timers())
                if (me == 0) std::printf("timer %s %.6f\n", kv.first.c_str(), kv.second);
            if (me == 0) std::printf("traced potrf info %lld getrf info %lld -> %s\n", (long long)i1, (long long)i2, tp);
            sn::finalize();
            return (i1 || i2) ? 1 : 0;
        }
        if (types.find('s') != std::string::npos) run<float>(p, q, me);
        if (types.find('d') != std::string::npos) run<double>(p, q, me);
        if (types.find('c') != std::string::npos) run<std::complex<float>>(p, q, me);
        if (types.find('z') != std::string::npos) run<std::complex<double>>(p, q, me);

        // ---- LAPACK-style C ABI (every rank passes the same global arrays)
        {
            const int64_t n = 200, nrhs = 2;
            std::vector<double> a((size_t)n * n), x((size_t)n * nrhs), b((size_t)n * nrhs, 0.0);
            for (int64_t j = 0; j < n; ++j)
                for (int64_t i = 0; i < n; ++i) a[i + j * n] = std::sin(0.37 * i + 1.3 * j) + (i == j ? 4.0 : 0.0);
            for (int64_t i = 0; i < n * nrhs; ++i) x[i] = std::cos(0.11 * i);
            for (int64_t c = 0; c < nrhs; ++c)
                for (int64_t j = 0; j < n; ++j)
                    for (int64_t i = 0; i < n; ++i) b[i + c * n] += a[i + j * n] * x[j + c * n];
            std::vector<int64_t> piv(n);
            const int ci = slate_dgesv(n, nrhs, a.data(), n, piv.data(), b.data(), n);
            double e = 0, w = 0;
            for (int64_t i = 0; i < n * nrhs; ++i) { e += (b[i] - x[i]) * (b[i] - x[i]); w += x[i] * x[i]; }
            if (me == 0) std::printf("check capi_dgesv %.3e\n", ci ? 1.0 : std::sqrt(e / w));
            if (ci && me == 0) std::printf("capi error: %s\n", slate_amd_last_error());

            // Hermitian positive definite complex system through slate_zposv
            std::vector<std::complex<double>> z((size_t)n * n), zx((size_t)n), zb((size_t)n, 0.0);
            for (int64_t j = 0; j < n; ++j)
                for (int64_t i = 0; i < n; ++i) {
                    const std::complex<double> v(std::sin(0.3 * i * j + 1.0), i < j ? 0.2 : i > j ? -0.2 : 0.0);
                    z[i + j * n] = 0.05 * v;
                }
            for (int64_t j = 0; j < n; ++j)
                for (int64_t i = 0; i < j; ++i) z[i + j * n] = std::conj(z[j + i * n]);
            for (int64_t i = 0; i < n; ++i) z[i + i * n] = {double(n) * 0.5, 0.0};
            for (int64_t i = 0; i < n; ++i) zx[i] = {std::cos(0.2 * i), std::sin(0.1 * i)};
            for (int64_t j = 0; j < n; ++j)
                for (int64_t i = 0; i < n; ++i) zb[i] += z[i + j * n] * zx[j];
            const int zi = slate_zposv('U', n, 1, reinterpret_cast<double*>(z.data()), n,
                                       reinterpret_cast<double*>(zb.data()), n);
            double ze = 0, zw = 0;
            for (int64_t i = 0; i < n; ++i) { ze += std::norm(zb[i] - zx[i]); zw += std::norm(zx[i]); }
            if (me == 0) std::printf("check capi_zposv %.3e\n", zi ? 1.0 : std::sqrt(ze / zw));

            // Fortran-style gemm: C = A^T A
            std::vector<double> c((size_t)n * n, 0.0);
            const int64_t nn = n;
            const double one = 1.0, zero = 0.0;
            for (int64_t j = 0; j < n; ++j)
                for (int64_t i = 0; i < n; ++i) a[i + j * n] = std::sin(0.37 * i + 1.3 * j);
            slate_dgemm_("T", "N", &nn, &nn, &nn, &one, a.data(), &nn, a.data(), &nn, &zero, c.data(), &nn);
            double ge = 0, gw = 0;
            for (int64_t j = 0; j < n; j += 7)
                for (int64_t i = 0; i < n; i += 5) {
                    double s = 0;
                    for (int64_t k = 0; k < n; ++k) s += a[k + i * n] * a[k + j * n];
                    ge += (c[i + j * n] - s) * (c[i + j * n] - s);
                    gw += s * s;
                }
            if (me == 0) std::printf("check capi_dgemm_tn %.3e\n", std::sqrt(ge / gw));
        }

        if (nbench > 0) {
            sn::HermitianMatrix<double> T(sn::Uplo::Lower, nbench, 512, p, q);
            for (int it = 0; it < 3; ++it) {
                T.generate(sn::Gen::HermitianPositiveDefinite, 11);
                const auto t0 = std::chrono::steady_clock::now();
                const int64_t info = sn::potrf(T);
                const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
                const double tf = (double)nbench * nbench * nbench / 3.0 / (ms * 1e-3) / 1e12;
                if (me == 0) std::printf("time potrf n=%lld %.2f ms %.2f TF/s info=%lld\n", (long long)nbench, ms, tf,
                                         (long long)info);
                std::fflush(stdout);
            }
        }
        sn::finalize();
    } catch (const std::exception& e) {
        std::fprintf(stderr, "ex_native: %s\n", e.what());
        return 1;
    }
    return 0;
}
