// Probe of the native grid heev against the gather path: per-column
// residuals ||A z_j - lambda_j z_j|| on the host (double, small n).
//   heev_probe n nb p q
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "slate_amd/slate_native.hh"

namespace sn = slate_amd::native;

static void colres(int64_t n, const std::vector<double>& a, const std::vector<double>& z, const std::vector<double>& w,
                   const char* tag) {
    double worst = 0;
    int bad = 0;
    for (int64_t j = 0; j < n; ++j) {
        double e = 0;
        for (int64_t i = 0; i < n; ++i) {
            double acc = 0;
            for (int64_t l = 0; l < n; ++l) acc += a[i + l * n] * z[l + j * n];
            e += (acc - w[j] * z[i + j * n]) * (acc - w[j] * z[i + j * n]);
        }
        e = std::sqrt(e);
        if (e > 1e-10) {
            if (bad < 12) std::printf("  %s bad column %lld lambda %.6e res %.3e\n", tag, (long long)j, w[j], e);
            ++bad;
        }
        worst = std::max(worst, e);
    }
    std::printf("%s: worst column residual %.3e, %d bad of %lld\n", tag, worst, bad, (long long)n);
}

int main(int argc, char** argv) {
    const int64_t n = std::atoll(argv[1]), nb = std::atoll(argv[2]);
    const int p = std::atoi(argv[3]), q = std::atoi(argv[4]);
    sn::initialize();
    sn::HermitianMatrix<double> H(sn::Uplo::Lower, n, nb, p, q);
    H.generate(sn::Gen::Random, 121);
    std::vector<double> a((size_t)n * n), z((size_t)n * n), z2((size_t)n * n);
    H.to_host(a.data(), n);
    for (int64_t j = 0; j < n; ++j)
        for (int64_t i = 0; i < j; ++i) a[i + j * n] = a[j + i * n];
    sn::Matrix<double> Z(n, n, nb, p, q);
    std::vector<double> w, w2;
    const int order = argc > 5 ? std::atoi(argv[5]) : 0;
    const bool gather_first = order == 1;
    if (order == 2 || order == 3) {
        // the same path twice in one process (2: gather, 3: grid): w / z from
        // the SECOND call, w2 / z2 from the first
        if (order == 2) setenv("SLATE_AMD_NATIVE_HEEV", "gather", 1);
        sn::heev(H, w2, Z);
        Z.to_host(z2.data(), n);
        sn::heev(H, w, Z);
        Z.to_host(z.data(), n);
    } else if (gather_first) {
        setenv("SLATE_AMD_NATIVE_HEEV", "gather", 1);
        sn::heev(H, w2, Z);
        Z.to_host(z2.data(), n);
        unsetenv("SLATE_AMD_NATIVE_HEEV");
        sn::heev(H, w, Z);
        Z.to_host(z.data(), n);
    } else {
        sn::heev(H, w, Z);
        Z.to_host(z.data(), n);
        setenv("SLATE_AMD_NATIVE_HEEV", "gather", 1);
        sn::heev(H, w2, Z);
        Z.to_host(z2.data(), n);
    }
    if (sn::rank() == 0 && std::getenv("SLATE_AMD_NATIVE_HEEV_DUMP")) {
        std::FILE* f = std::fopen((std::string(std::getenv("SLATE_AMD_NATIVE_HEEV_DUMP")) + "/a.bin").c_str(), "wb");
        if (f) { std::fwrite(a.data(), sizeof(double), a.size(), f); std::fclose(f); }
    }
    if (sn::rank() == 0) {
        double dv = 0;
        for (int64_t i = 0; i < n; ++i) dv = std::max(dv, std::abs(w[i] - w2[i]));
        std::printf("n=%lld %dx%d: eigenvalue max diff %.3e\n", (long long)n, p, q, dv);
        std::vector<double> wd(w.begin(), w.end()), wd2(w2.begin(), w2.end());
        colres(n, a, z, wd, "grid");
        colres(n, a, z2, wd2, "gather");
    }
    sn::finalize();
    return 0;
}
