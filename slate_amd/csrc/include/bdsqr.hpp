// Golub-Kahan implicit-shift QR SVD of a real upper bidiagonal (bdsqr;
// reference src/bdsqr.cc) with plane-rotation accumulation into U / VT.
// Shared by the Python package's host module (csrc/host/eig.cpp) and the
// Python-free native library (csrc/native/native_eig.hip).  Header-only.
#pragma once
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <limits>
#include <vector>

namespace slate_tridiag {

using i64 = int64_t;

// ---------------------------------------------------------------- rotations
// apply a sequence of plane rotations to columns (i, i+1) of Z for all rows
// in parallel: Z(:, i), Z(:, i+1) <- c*Z_i - s*Z_{i+1}, s*Z_i + c*Z_{i+1}
template <typename Z_t, typename R>
inline void rot_seq(i64 nrow, Z_t* z, i64 ldz, const std::vector<i64>& idx, const std::vector<R>& cs,
             const std::vector<R>& sn) {
    if (!z || idx.empty()) return;
    const i64 nr = (i64)idx.size();
    #pragma omp parallel for schedule(static) if (nrow * nr > 1 << 16)
    for (i64 r = 0; r < nrow; ++r) {
        for (i64 t = 0; t < nr; ++t) {
            const i64 i = idx[t];
            Z_t* zi = z + r + i * ldz;
            Z_t* zj = z + r + (i + 1) * ldz;
            const Z_t a = *zi, b2 = *zj;
            *zi = cs[t] * a - sn[t] * b2;
            *zj = sn[t] * a + cs[t] * b2;
        }
    }
}

// ---------------------------------------------------------------- bdsqr
// SVD of the real upper bidiagonal (d, e): B = U S V^T.  U (nu x n) gets
// right-multiplied by the left rotations, VT (n x nv) left-multiplied by the
// right rotations (stored as columns of V = VT^T: we rotate rows of VT).
// Golub-Kahan implicit-shift QR with a standard deflation test; singular
// values made non-negative and sorted descending.
inline i64 bdsqr_impl(i64 n, double* d, double* e, double* u, i64 ldu, i64 nu, double* vt, i64 ldvt, i64 nv) {
    using R = double;
    if (n == 0) return 0;
    const R eps = std::numeric_limits<R>::epsilon();
    const R tiny = std::numeric_limits<R>::min();
    i64 fails = 0;
    std::vector<i64> ui, vi; std::vector<R> uc, us, vc, vs;
    auto flush = [&]() {
        if (u && !ui.empty()) {
            #pragma omp parallel for schedule(static) if (nu * (i64)ui.size() > 1 << 16)
            for (i64 r = 0; r < nu; ++r)
                for (size_t t = 0; t < ui.size(); ++t) {
                    R* a = u + r + ui[t] * ldu; R* b2 = a + ldu;
                    R x = *a, y = *b2;
                    *a = uc[t] * x + us[t] * y;
                    *b2 = -us[t] * x + uc[t] * y;
                }
        }
        if (vt && !vi.empty()) {
            #pragma omp parallel for schedule(static) if (nv * (i64)vi.size() > 1 << 16)
            for (i64 c = 0; c < nv; ++c)
                for (size_t t = 0; t < vi.size(); ++t) {
                    R* a = vt + vi[t] + c * ldvt; R* b2 = a + 1;
                    R x = *a, y = *b2;
                    *a = vc[t] * x + vs[t] * y;
                    *b2 = -vs[t] * x + vc[t] * y;
                }
        }
        ui.clear(); uc.clear(); us.clear(); vi.clear(); vc.clear(); vs.clear();
    };
    auto givens = [](R f, R g, R& c, R& s, R& r) {
        if (g == 0) { c = 1; s = 0; r = f; return; }
        if (f == 0) { c = 0; s = 1; r = g; return; }
        r = std::hypot(f, g); c = f / r; s = g / r;
    };
    i64 hi = n - 1;
    i64 iter = 0, maxit = 40 * n * n + 100;
    while (hi > 0) {
        // deflate negligible superdiagonals
        for (i64 i = 0; i < hi; ++i)
            if (std::abs(e[i]) <= eps * (std::abs(d[i]) + std::abs(d[i + 1])) || std::abs(e[i]) < tiny) e[i] = 0;
        if (e[hi - 1] == 0) { --hi; continue; }
        i64 lo = hi - 1;
        while (lo > 0 && e[lo - 1] != 0) --lo;
        if (++iter > maxit) { fails = hi; break; }
        // zero diagonal inside the block: chase the row out with rotations
        bool zd = false;
        for (i64 i = lo; i < hi; ++i) {
            if (std::abs(d[i]) <= eps * 1e-3 * (std::abs(e[i]) + (i > lo ? std::abs(e[i - 1]) : 0))) {
                d[i] = 0;
                // rotate row i against rows i+1.. to annihilate e[i]
                R f = e[i]; e[i] = 0;
                for (i64 k = i + 1; k <= hi; ++k) {
                    R c, s, r;
                    givens(d[k], f, c, s, r);
                    d[k] = r;
                    // left rotation on rows (i, k): affects U columns i, k
                    if (k < hi) { f = -s * e[k]; e[k] = c * e[k]; }
                    if (u) {
                        #pragma omp parallel for schedule(static) if (nu > 4096)
                        for (i64 rr = 0; rr < nu; ++rr) {
                            R* a = u + rr + i * ldu; R* b2 = u + rr + k * ldu;
                            R x = *a, y = *b2;
                            *a = c * x - s * y;
                            *b2 = s * x + c * y;
                        }
                    }
                }
                zd = true;
                break;
            }
        }
        if (zd) continue;
        // Wilkinson shift from the trailing 2x2 of B^T B
        R dm = d[hi - 1], dn = d[hi], em = (hi - 1 > lo) ? e[hi - 2] : 0, en = e[hi - 1];
        R t11 = dm * dm + em * em, t22 = dn * dn + en * en, t12 = dm * en;
        R dl = (t11 - t22) / 2;
        R mu = t22 - t12 * t12 / (dl + std::copysign(std::hypot(dl, t12), dl == 0 ? 1.0 : dl));
        if (!std::isfinite(mu)) mu = t22;
        R y = d[lo] * d[lo] - mu, z = d[lo] * e[lo];
        for (i64 k = lo; k < hi; ++k) {
            R c, s, r;
            givens(y, z, c, s, r);
            // right rotation on columns (k, k+1)
            if (k > lo) e[k - 1] = r;
            y = c * d[k] + s * e[k];
            e[k] = -s * d[k] + c * e[k];
            z = s * d[k + 1];
            d[k + 1] = c * d[k + 1];
            vi.push_back(k); vc.push_back(c); vs.push_back(s);
            givens(y, z, c, s, r);
            d[k] = r;
            y = c * e[k] + s * d[k + 1];
            d[k + 1] = -s * e[k] + c * d[k + 1];
            if (k < hi - 1) { z = s * e[k + 1]; e[k + 1] = c * e[k + 1]; }
            ui.push_back(k); uc.push_back(c); us.push_back(s);
        }
        e[hi - 1] = y;
        flush();
    }
    flush();
    // signs and descending order
    for (i64 i = 0; i < n; ++i)
        if (d[i] < 0) {
            d[i] = -d[i];
            if (vt) for (i64 c = 0; c < nv; ++c) vt[i + c * ldvt] = -vt[i + c * ldvt];
        }
    for (i64 i = 0; i < n - 1; ++i) {
        i64 k = i;
        for (i64 j = i + 1; j < n; ++j) if (d[j] > d[k]) k = j;
        if (k != i) {
            std::swap(d[i], d[k]);
            if (u) for (i64 r = 0; r < nu; ++r) std::swap(u[r + i * ldu], u[r + k * ldu]);
            if (vt) for (i64 c = 0; c < nv; ++c) std::swap(vt[i + c * ldvt], vt[k + c * ldvt]);
        }
    }
    return fails;
}


}  // namespace slate_tridiag
