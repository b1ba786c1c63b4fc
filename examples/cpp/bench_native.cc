// Headline benchmark through the Python-free library (bench.py --impl
// native runs this binary, one process per rank, and prints the JSON
// contract).  One step = restore the input (device copy, inside the timed
// region, as bench.py does) + one factorization / product; K steps timed
// between barriers, maximum over ranks.  After the timed region the
// backward error is checked on the grid with the library itself:
//   potrf / getrf: X = A \ B through the factors, ||B - A0 X|| / (||A0|| ||X|| n)
//   gemm:          ||C v - A (B v)|| / (||A|| ||B|| ||v|| n)
//
//   geqrf:         gels of a consistent system B = A0 X0,
//                  ||A0^H (A0 X - B)|| / (||A0||^2 ||X|| m)
//
//   heev:          Z V against Z (Lambda V) through A for 4 random vectors,
//                  ||A Z V - Z Lambda V|| / (||A|| ||V|| n) (no n x n host data)
//
//   bench_native routine n nb p q lookahead warmup steps check [m]
// prints "RESULT ms_per_step=<max over ranks> info=<info> resid=<r>"
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "slate_amd/slate_native.hh"

namespace sn = slate_amd::native;

int main(int argc, char** argv) {
    if (argc < 10) {
        std::fprintf(stderr, "usage: bench_native routine n nb p q lookahead warmup steps check\n");
        return 2;
    }
    const std::string routine = argv[1];
    const int64_t n = std::atoll(argv[2]), nb = std::atoll(argv[3]);
    const int p = std::atoi(argv[4]), q = std::atoi(argv[5]);
    sn::Options opts;
    opts.lookahead = std::atoi(argv[6]);
    const int warmup = std::atoi(argv[7]), steps = std::atoi(argv[8]), check = std::atoi(argv[9]);
    const int64_t mrows = argc > 10 ? std::atoll(argv[10]) : n;
    try {
        sn::initialize();
        const int me = sn::rank();
        const bool chol = routine == "potrf";
        const sn::Gen kind = chol ? sn::Gen::HermitianPositiveDefinite : sn::Gen::Random;
        const bool qr = routine == "geqrf";
        sn::Matrix<double> A0(qr ? mrows : n, n, nb, p, q);
        A0.generate(kind, 7);
        sn::Matrix<double> Aq = qr ? sn::Matrix<double>(mrows, n, nb, p, q) : sn::Matrix<double>();
        sn::QRFactors<double> F;
        sn::HermitianMatrix<double> H(sn::Uplo::Lower, n, nb, p, q);
        sn::Matrix<double> G(n, n, nb, p, q), B, C;
        if (routine == "gemm") {
            B = sn::Matrix<double>(n, n, nb, p, q);
            C = sn::Matrix<double>(n, n, nb, p, q);
            B.generate(sn::Gen::Random, 8);
        }
        std::vector<int64_t> ipiv;
        int64_t info = 0;
        const bool eig = routine == "heev";
        sn::HermitianMatrix<double> He;
        sn::Matrix<double> Ze;
        std::vector<double> lam;
        if (eig) {
            He = sn::HermitianMatrix<double>(sn::Uplo::Lower, n, nb, p, q);
            Ze = sn::Matrix<double>(n, n, nb, p, q);
        }
        auto step = [&]() {
            if (eig) {
                sn::copy(sn::Op::NoTrans, A0, He);
                info = sn::heev(He, lam, Ze, opts);
            } else if (chol) {
                sn::copy(sn::Op::NoTrans, A0, H);
                info = sn::potrf(H, opts);
            } else if (routine == "getrf") {
                sn::copy(sn::Op::NoTrans, A0, G);
                info = sn::getrf(G, ipiv, opts);
            } else if (qr) {
                sn::copy(sn::Op::NoTrans, A0, Aq);
                info = sn::geqrf(Aq, F, opts);
            } else {
                sn::gemm(1.0, A0, B, 0.0, C, opts);
            }
        };
        for (int i = 0; i < warmup; ++i) step();
        sn::barrier();
        const auto t0 = std::chrono::steady_clock::now();
        for (int i = 0; i < steps; ++i) step();
        sn::barrier();
        const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        const double ms_max = sn::allreduce_max(ms) / steps;
        double resid = -1;
        if (check) {
            const int64_t nr = 1;
            sn::Matrix<double> V(n, nr, nb, p, q), X(n, nr, nb, p, q);
            V.generate(sn::Gen::Random, 5);
            if (eig) {
                const int64_t nv = 4;
                std::vector<double> hv((size_t)n * nv), hl((size_t)n * nv);
                sn::Matrix<double> Vr(n, nv, nb, p, q), LV(n, nv, nb, p, q), ZV(n, nv, nb, p, q),
                    AZV(n, nv, nb, p, q), ZLV(n, nv, nb, p, q);
                Vr.generate(sn::Gen::Random, 6);
                Vr.to_host(hv.data(), n);
                for (int64_t j = 0; j < nv; ++j)
                    for (int64_t i = 0; i < n; ++i) hl[i + j * n] = lam[i] * hv[i + j * n];
                LV.from_host(hl.data(), n);
                sn::gemm(1.0, Ze, Vr, 0.0, ZV);
                sn::hemm(sn::Side::Left, 1.0, He, ZV, 0.0, AZV);
                sn::gemm(1.0, Ze, LV, 0.0, ZLV);
                sn::add(-1.0, ZLV, 1.0, AZV);
                resid = sn::norm(sn::Norm::Fro, AZV) /
                        (sn::norm(sn::Norm::Fro, A0) * sn::norm(sn::Norm::Fro, Vr) * (double)n);
            } else if (qr) {
                sn::Matrix<double> X0(n, nr, nb, p, q), B(mrows, nr, nb, p, q), R(mrows, nr, nb, p, q), G2(n, nr, nb, p, q);
                X0.generate(sn::Gen::Random, 5);
                sn::gemm(1.0, A0, X0, 0.0, B);
                sn::copy(sn::Op::NoTrans, B, R);
                sn::copy(sn::Op::NoTrans, A0, Aq);
                sn::gels(Aq, R);                                    // X in R(0:n)
                sn::Matrix<double> X(n, nr, nb, p, q), E(mrows, nr, nb, p, q);
                std::vector<double> hx((size_t)mrows);
                R.to_host(hx.data(), mrows);
                X.from_host(hx.data(), n);
                sn::copy(sn::Op::NoTrans, B, E);
                sn::gemm(1.0, A0, X, -1.0, E);                      // A0 X - B
                sn::gemm(sn::Op::ConjTrans, sn::Op::NoTrans, 1.0, A0, E, 0.0, G2);
                const double na = sn::norm(sn::Norm::Fro, A0);
                resid = sn::norm(sn::Norm::Fro, G2) / (na * na * sn::norm(sn::Norm::Fro, X) * (double)mrows);
            } else if (routine == "gemm") {
                sn::Matrix<double> BV(n, nr, nb, p, q), ABV(n, nr, nb, p, q);
                sn::gemm(1.0, B, V, 0.0, BV);
                sn::gemm(1.0, A0, BV, 0.0, ABV);
                // reference tester (test/test_gemm.cc:191-207): ||C x - y|| / ||y||, y = A (B x),
                // with the sqrt(k) + 2 growth factor of its reference check
                const double ny = sn::norm(sn::Norm::Fro, ABV);
                sn::gemm(1.0, C, V, -1.0, ABV);            // C v - A (B v)
                resid = sn::norm(sn::Norm::Fro, ABV) / (ny * (std::sqrt((double)n) + 2.0));
            } else {
                sn::copy(sn::Op::NoTrans, V, X);
                if (chol) sn::potrs(H, X);
                else sn::getrs(G, ipiv, X);
                sn::gemm(-1.0, A0, X, 1.0, V);             // V = B - A0 X
                const double nr_ = sn::norm(sn::Norm::Fro, V), na = sn::norm(sn::Norm::Fro, A0),
                             nx = sn::norm(sn::Norm::Fro, X);
                resid = nr_ / (na * nx * (double)n);
                if (me == 0) std::printf("norms |B-AX|=%.6e |A|=%.6e |X|=%.6e\n", nr_, na, nx);
            }
        }
        if (me == 0)
            std::printf("RESULT ms_per_step=%.4f info=%lld resid=%.3e transport=%s\n", ms_max, (long long)info,
                        resid, sn::transport());
        std::fflush(stdout);
        sn::finalize();
    } catch (const std::exception& e) {
        std::fprintf(stderr, "bench_native: %s\n", e.what());
        return 1;
    }
    return 0;
}
