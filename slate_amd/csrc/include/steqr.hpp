// Implicit-shift QL / QR on a real symmetric tridiagonal (sterf / steqr;
// reference src/sterf.cc, src/steqr.cc).  Shared by the Python package's host
// module (csrc/host/eig.cpp) and the Python-free native library
// (csrc/native/native_eig.hip).  Header-only, host code.
#pragma once
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <limits>
#include <vector>

namespace slate_tridiag {

using i64 = int64_t;

inline int steqr_maxit() {
    const char* e = std::getenv("SLATE_AMD_STEQR_MAXIT");
    return e ? std::atoi(e) : 60;
}
// Implicit-shift QL/QR on the symmetric tridiagonal (d, e); optional
// eigenvector accumulation Z (nz x n, columns rotated).  Eigenvalues sorted
// ascending (with Z columns) on exit.  Returns 0 or #unconverged.
template <typename Z_t>
inline i64 steqr_impl(i64 n, double* d, double* e, Z_t* z, i64 ldz, i64 nz) {
    using R = double;
    if (n <= 1) return 0;
    const R eps = std::numeric_limits<R>::epsilon();
    std::vector<R> ew(n, 0);
    for (i64 i = 0; i < n - 1; ++i) ew[i] = e[i];
    i64 fails = 0;
    const int maxit = steqr_maxit();
    std::vector<i64> idx; std::vector<R> cs, sn;
    for (i64 l = 0; l < n; ++l) {
        i64 iter = 0;
        while (true) {
            i64 m = l;
            for (; m < n - 1; ++m) {
                R dd = std::abs(d[m]) + std::abs(d[m + 1]);
                if (std::abs(ew[m]) <= eps * dd || std::abs(ew[m]) < std::numeric_limits<R>::min()) break;
            }
            if (m == l) break;
            if (++iter > maxit) { ++fails; break; }
            // Wilkinson-type shift from the leading 2x2
            R g = (d[l + 1] - d[l]) / (2 * ew[l]);
            R r = std::hypot(g, R(1));
            g = d[m] - d[l] + ew[l] / (g + std::copysign(r, g));
            R s = 1, c = 1, p = 0;
            bool early = false;
            idx.clear(); cs.clear(); sn.clear();
            i64 i;
            for (i = m - 1; i >= l; --i) {
                R f = s * ew[i], bb = c * ew[i];
                r = std::hypot(f, g);
                ew[i + 1] = r;
                if (r == 0) { d[i + 1] -= p; ew[m] = 0; early = true; break; }
                s = f / r; c = g / r;
                g = d[i + 1] - p;
                r = (d[i] - g) * s + 2 * c * bb;
                p = s * r;
                d[i + 1] = g + p;
                g = c * r - bb;
                // rotation on columns (i, i+1):  z_{i+1} <- s z_i + c z_{i+1}; z_i <- c z_i - s z_{i+1}
                idx.push_back(i); cs.push_back(c); sn.push_back(s);
            }
            // apply in generation order: (i, i+1) with (c, s): zi' = c zi - s zj ; zj' = s zi + c zj
            if (z) {
                #pragma omp parallel for schedule(static) if (nz * (i64)idx.size() > 1 << 16)
                for (i64 rr = 0; rr < nz; ++rr) {
                    for (size_t t = 0; t < idx.size(); ++t) {
                        Z_t* zi = z + rr + idx[t] * ldz;
                        Z_t* zj = zi + ldz;
                        const Z_t a = *zi, b2 = *zj;
                        *zj = sn[t] * a + cs[t] * b2;
                        *zi = cs[t] * a - sn[t] * b2;
                    }
                }
            }
            if (early && i >= l) continue;
            d[l] -= p; ew[l] = g; ew[m] = 0;
        }
    }
    // sort ascending (selection sort on columns, O(n^2) swaps of Z columns)
    for (i64 i = 0; i < n - 1; ++i) {
        i64 k = i;
        for (i64 j = i + 1; j < n; ++j) if (d[j] < d[k]) k = j;
        if (k != i) {
            std::swap(d[i], d[k]);
            if (z) for (i64 r = 0; r < nz; ++r) std::swap(z[r + i * ldz], z[r + k * ldz]);
        }
    }
    for (i64 i = 0; i < n - 1; ++i) e[i] = 0;
    return fails;
}


}  // namespace slate_tridiag
