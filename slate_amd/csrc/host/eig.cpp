// Host kernels of the eigenvalue / SVD pipelines (stage 2 + tridiagonal /
// bidiagonal solvers).  These are the parts SLATE also runs on the host:
//   hb2st  -- Hermitian band -> real symmetric tridiagonal by bulge chasing
//             (src/hb2st.cc, internal_hebr.cc: hebr1/2/3 tasks)
//   tb2bd  -- upper triangular band -> real bidiagonal (src/tb2bd.cc,
//             internal_gebr.cc: gebr1/2/3)
//   sterf / steqr -- implicit-shift QL on a symmetric tridiagonal
//             (src/sterf.cc, src/steqr.cc, steqr_impl.cc)
//   bdsqr  -- implicit-shift QR SVD of a bidiagonal (src/bdsqr.cc)
//   secular -- roots of the rank-one-update secular equation for the
//             divide & conquer merge (src/stedc_secular.cc / laed4)
// Design notes (MI355X framework): the chases keep the band in a dense
// column-major window (simple, cache friendly at the band sizes used), and
// every reflector is recorded so the back-transformations run on the GPU as
// batched kernels/GEMMs; rotation sequences of steqr/bdsqr are applied to
// the eigen/singular vector rows in parallel (OpenMP over rows).
#include <pybind11/pybind11.h>
#include <pybind11/complex.h>

#include <algorithm>
#include <cmath>
#include <complex>
#include <cstdlib>
#include <thread>
#include <atomic>
#include <cstdint>
#include <limits>
#include <stdexcept>
#include <vector>

#include "bdsqr.hpp"
#include "steqr.hpp"

namespace py = pybind11;

namespace slate_host {
namespace {

using i64 = int64_t;
template <typename T> struct rl { using type = T; };
template <typename T> struct rl<std::complex<T>> { using type = T; };
template <typename T> using R_t = typename rl<T>::type;
template <typename T> inline T cj(T x) { return x; }
template <typename T> inline std::complex<T> cj(std::complex<T> x) { return std::conj(x); }

// Householder generator: on entry x[0..k-1]; on exit v (v[0] = 1) in x,
// returns tau, beta (real) with (I - tau v v^H)^H x_in = beta e1.
template <typename T>
void hgen(i64 k, T* x, T& tau, R_t<T>& beta) {
    using R = R_t<T>;
    T alpha = x[0];
    R xn2 = 0;
    for (i64 i = 1; i < k; ++i) xn2 += std::norm(x[i]);
    R ar = std::real(alpha), ai = std::imag(alpha);
    if (xn2 == R(0) && ai == R(0)) {
        tau = T(0);
        beta = ar;
        x[0] = T(1);
        return;
    }
    beta = -std::copysign(std::sqrt(ar * ar + ai * ai + xn2), ar);
    if constexpr (std::is_same_v<T, R>) {
        tau = (beta - ar) / beta;
    } else {
        tau = T((beta - ar) / beta, -ai / beta);
    }
    T sc = T(1) / (alpha - T(beta));
    for (i64 i = 1; i < k; ++i) x[i] *= sc;
    x[0] = T(1);
}

template <typename T>
struct Dense {
    T* a; i64 ld;
    T& operator()(i64 r, i64 c) const { return a[r + c * ld]; }
};

// A[rows s..s+k-1, cols lo..hi] := H^H A[...]   (H = I - tau v v^H)
template <typename T>
void apply_left(Dense<T> A, i64 s, i64 k, const T* v, T tau, i64 lo, i64 hi) {
    if (tau == T(0)) return;
    const T ct = cj(tau);
    for (i64 c = lo; c <= hi; ++c) {
        T w = 0;
        for (i64 r = 0; r < k; ++r) w += cj(v[r]) * A(s + r, c);
        w *= ct;
        if (w == T(0)) continue;
        for (i64 r = 0; r < k; ++r) A(s + r, c) -= v[r] * w;
    }
}

// A[rows lo..hi, cols s..s+k-1] := A[...] H, column-major friendly: y = A v
// accumulated column by column (contiguous rows), then the rank-1 update
// column by column (same summation order per row as the row-wise form)
template <typename T>
void apply_right(Dense<T> A, i64 s, i64 k, const T* v, T tau, i64 lo, i64 hi) {
    if (tau == T(0) || hi < lo) return;
    const i64 nr = hi - lo + 1;
    thread_local std::vector<T> y;
    y.assign(nr, T(0));
    for (i64 c = 0; c < k; ++c) {
        const T vc = v[c];
        const T* col = &A(lo, s + c);
        for (i64 r = 0; r < nr; ++r) y[r] += col[r] * vc;
    }
    for (i64 r = 0; r < nr; ++r) y[r] *= tau;
    for (i64 c = 0; c < k; ++c) {
        const T vc = cj(v[c]);
        T* col = &A(lo, s + c);
        for (i64 r = 0; r < nr; ++r) col[r] -= y[r] * vc;
    }
}

struct Refl {            // reflector store (row-major count x b)
    void* V; void* tau; i64* row; i64* len; i64 b; i64 cap; i64 cnt = 0;
    template <typename T> void put(i64 r0, i64 k, const T* v, T t) {
        put_at(cnt, r0, k, v, t);
        ++cnt;
    }
    template <typename T> void put_at(i64 idx, i64 r0, i64 k, const T* v, T t) {
        if (idx >= cap) throw std::runtime_error("reflector store overflow");
        T* dst = static_cast<T*>(V) + idx * b;
        for (i64 i = 0; i < k; ++i) dst[i] = v[i];
        for (i64 i = k; i < b; ++i) dst[i] = T(0);
        static_cast<T*>(tau)[idx] = t;
        row[idx] = r0; len[idx] = k;
    }
};

// ---------------------------------------------------------------- hb2st
// A: dense n x n Hermitian (both triangles) of lower bandwidth b.  Reduced
// in place to Hermitian tridiagonal T = Q^H A Q, Q = prod of the recorded
// reflectors in order; sweep_ptr[j] = first reflector of sweep j.
template <typename T>
i64 hb2st(i64 n, i64 b, T* a, i64 lda, Refl& st, i64* sweep_ptr) {
    Dense<T> A{a, lda};
    std::vector<T> v(b + 1), v2(b + 1);
    for (i64 j = 0; j + 1 < n; ++j) {
        sweep_ptr[j] = st.cnt;
        i64 s = j + 1, e = std::min(j + b, n - 1), k = e - s + 1;
        if (k <= 1) continue;            // nothing below the subdiagonal
        for (i64 r = 0; r < k; ++r) v[r] = A(s + r, j);
        T tau; R_t<T> beta;
        hgen(k, v.data(), tau, beta);
        // two-sided on rows/cols s..e over the window
        i64 lo = j + 1, hi = std::min(n - 1, e + b);      // window: see hb2st_mt
        apply_left(A, s, k, v.data(), tau, lo, hi);
        apply_right(A, s, k, v.data(), tau, lo, hi);
        A(s, j) = T(beta); A(j, s) = T(beta);
        for (i64 r = 1; r < k; ++r) { A(s + r, j) = T(0); A(j, s + r) = T(0); }
        st.put(s, k, v.data(), tau);
        // chase the bulge
        while (true) {
            i64 s2 = e + 1;
            if (s2 > n - 1) break;
            i64 e2 = std::min(e + b, n - 1), k2 = e2 - s2 + 1;
            for (i64 r = 0; r < k2; ++r) v2[r] = A(s2 + r, s);
            T tau2; R_t<T> beta2;
            hgen(k2, v2.data(), tau2, beta2);
            i64 lo2 = s + 1, hi2 = std::min(n - 1, e2 + b);
            apply_left(A, s2, k2, v2.data(), tau2, lo2, hi2);
            apply_right(A, s2, k2, v2.data(), tau2, lo2, hi2);
            A(s2, s) = T(beta2); A(s, s2) = T(beta2);
            for (i64 r = 1; r < k2; ++r) { A(s2 + r, s) = T(0); A(s, s2 + r) = T(0); }
            st.put(s2, k2, v2.data(), tau2);
            s = s2; e = e2; k = k2;
        }
    }
    if (n >= 1) sweep_ptr[n - 1] = st.cnt;
    return st.cnt;
}

// Pipelined multi-threaded form (SLATE hb2st.cc runs the sweeps as OpenMP
// tasks with the same progress dependencies).  Task t of sweep j (t = 0:
// the column-j reflector, t >= 1: the t-th bulge) touches rows/columns
// [s_t - w, e_t + w], s_t = j + 1 + t b; the windows of sweep j-1's tasks
// t' > t + 1 + 2w/b lie strictly to the right.  So sweep j runs task t once
// sweep j-1 has completed min(t + D, all) tasks: the result is bitwise the
// sequential one (every pair of overlapping tasks keeps its order).  Thread
// r owns sweeps r, r + T, ...; progress counters are release/acquire
// atomics; reflectors go to fixed slots sweep_ptr[j] + t.
template <typename T>
i64 hb2st_mt(i64 n, i64 b, T* a, i64 lda, Refl& st, i64* sweep_ptr, int nthreads) {
    Dense<T> A{a, lda};
    // task window: rows/columns [col + 1, e + b] (col: the column being
    // annihilated, overwritten explicitly; e + b: band + the bulge the
    // right application creates), width <= 3b; windows of sweep j-1 lie
    // strictly right of sweep j's task t from its task t + 3 on
    const i64 D = 4;
    // task counts per sweep (same recurrence as the sequential chase)
    std::vector<i64> ntask(std::max<i64>(n, 1), 0);
    i64 total = 0;
    for (i64 j = 0; j + 1 < n; ++j) {
        sweep_ptr[j] = total;
        i64 s = j + 1, e = std::min(j + b, n - 1);
        if (e - s + 1 <= 1) continue;
        i64 t = 1;
        while (e + 1 <= n - 1) { e = std::min(e + b, n - 1); ++t; }
        ntask[j] = t;
        total += t;
    }
    if (n >= 1) sweep_ptr[n - 1] = total;
    if (total > st.cap) throw std::runtime_error("reflector store overflow");
    std::vector<std::atomic<i64>> done(std::max<i64>(n, 1));
    for (auto& d : done) d.store(0, std::memory_order_relaxed);
    const i64 nsw = std::max<i64>(n - 1, 0);
    const int T_ = (int)std::max<i64>(1, std::min<i64>(nthreads, nsw));
    auto worker = [&](int r) {
        std::vector<T> v(b + 1);
        for (i64 j = r; j < nsw; j += T_) {
            const i64 nt = ntask[j];
            i64 s = j + 1, e = std::min(j + b, n - 1), col = j;
            for (i64 t = 0; t < nt; ++t) {
                if (j > 0) {
                    const i64 need = std::min(t + D, ntask[j - 1]);
                    while (done[j - 1].load(std::memory_order_acquire) < need) std::this_thread::yield();
                }
                if (t > 0) { s = e + 1; e = std::min(e + b, n - 1); }
                const i64 k = e - s + 1;
                for (i64 q = 0; q < k; ++q) v[q] = A(s + q, col);
                T tau; R_t<T> beta;
                hgen(k, v.data(), tau, beta);
                const i64 lo = col + 1, hi = std::min(n - 1, e + b);
                apply_left(A, s, k, v.data(), tau, lo, hi);
                apply_right(A, s, k, v.data(), tau, lo, hi);
                A(s, col) = T(beta); A(col, s) = T(beta);
                for (i64 q = 1; q < k; ++q) { A(s + q, col) = T(0); A(col, s + q) = T(0); }
                st.put_at(sweep_ptr[j] + t, s, k, v.data(), tau);
                col = s;
                done[j].store(t + 1, std::memory_order_release);
            }
            if (nt == 0) done[j].store(0, std::memory_order_release);
        }
    };
    std::vector<std::thread> th;
    for (int r = 1; r < T_; ++r) th.emplace_back(worker, r);
    worker(0);
    for (auto& x : th) x.join();
    st.cnt = total;
    return total;
}

// ---------------------------------------------------------------- tb2bd
// A: dense n x n upper triangular band (bandwidth b above the diagonal),
// reduced in place to upper bidiagonal B = U^H A V.  Left reflectors go to
// `ul` (U = prod), right reflectors to `vr` (V = prod); ptrs per sweep.
template <typename T>
void tb2bd(i64 n, i64 b, T* a, i64 lda, Refl& ul, Refl& vr, i64* uptr, i64* vptr) {
    Dense<T> A{a, lda};
    std::vector<T> v(b + 1), x(b + 1);
    const i64 w = 2 * b + 1;
    for (i64 j = 0; j + 1 < n; ++j) {
        uptr[j] = ul.cnt; vptr[j] = vr.cnt;
        // right reflector on row j, columns j+1..e
        i64 cs = j + 1, ce = std::min(j + b, n - 1), k = ce - cs + 1;
        i64 row = j;
        while (true) {
            for (i64 c = 0; c < k; ++c) v[c] = cj(A(row, cs + c));
            T tau; R_t<T> beta;
            hgen(k, v.data(), tau, beta);
            i64 lo = std::max<i64>(0, cs - w), hi = std::min(n - 1, ce + w);
            apply_right(A, cs, k, v.data(), tau, lo, hi);
            A(row, cs) = T(beta);
            for (i64 c = 1; c < k; ++c) A(row, cs + c) = T(0);
            vr.put(cs, k, v.data(), tau);
            // left reflector on rows cs..ce annihilating column cs below the diagonal
            i64 rs = cs, re = std::min(cs + b - 1, n - 1);
            re = std::min(re, ce);
            i64 kr = re - rs + 1;
            for (i64 r = 0; r < kr; ++r) x[r] = A(rs + r, cs);
            T tl; R_t<T> bl;
            hgen(kr, x.data(), tl, bl);
            i64 lo2 = std::max<i64>(0, rs - w), hi2 = std::min(n - 1, re + w);
            apply_left(A, rs, kr, x.data(), tl, lo2, hi2);
            A(rs, cs) = T(bl);
            for (i64 r = 1; r < kr; ++r) A(rs + r, cs) = T(0);
            ul.put(rs, kr, x.data(), tl);
            // next: row rs has fill beyond its band -> columns ce+1 .. ce+b
            i64 ncs = ce + 1;
            if (ncs > n - 1) break;
            row = rs;
            cs = ncs; ce = std::min(ncs + b - 1, n - 1); k = ce - cs + 1;
        }
    }
    if (n >= 1) { uptr[n - 1] = ul.cnt; vptr[n - 1] = vr.cnt; }
}

// Pipelined multi-threaded tb2bd (SLATE src/tb2bd.cc:159, 280-289 runs the
// sweeps as OpenMP tasks guarded by a progress vector).  Task t of sweep j is
// one iteration of the sequential loop above (a right reflector on a row,
// then a left reflector on the columns it filled); its windows lie in
// [j + (t - 2) b, j + (t + 3) b + 1], so every task of sweep j - 1 from
// t + 8 on is strictly to the right: sweep j runs task t once sweep j - 1
// has completed min(t + 8, all) tasks, which keeps every pair of
// overlapping tasks in the sequential order (bitwise the sequential
// result).  Thread r owns sweeps r, r + T, ...; reflectors go to the fixed
// slots uptr[j] + t / vptr[j] + t, i.e. the sequential layout.
template <typename T>
void tb2bd_mt(i64 n, i64 b, T* a, i64 lda, Refl& ul, Refl& vr, i64* uptr, i64* vptr, int nthreads) {
    Dense<T> A{a, lda};
    const i64 w = 2 * b + 1, D = 8;
    const i64 nsw = std::max<i64>(n - 1, 0);
    std::vector<i64> ntask(std::max<i64>(nsw, 1), 0);
    i64 total = 0;
    for (i64 j = 0; j < nsw; ++j) {
        uptr[j] = vptr[j] = total;
        i64 ce = std::min(j + b, n - 1), t = 1;
        while (ce + 1 <= n - 1) { ce = std::min(ce + b, n - 1); ++t; }
        ntask[j] = t;
        total += t;
    }
    if (n >= 1) uptr[n - 1] = vptr[n - 1] = total;
    if (total > ul.cap || total > vr.cap) throw std::runtime_error("reflector store overflow");
    std::vector<std::atomic<i64>> done(std::max<i64>(nsw, 1));
    for (auto& d : done) d.store(0, std::memory_order_relaxed);
    const int T_ = (int)std::max<i64>(1, std::min<i64>(nthreads, nsw));
    auto worker = [&](int r) {
        std::vector<T> v(b + 1), x(b + 1);
        for (i64 j = r; j < nsw; j += T_) {
            i64 cs = j + 1, ce = std::min(j + b, n - 1), row = j;
            for (i64 t = 0; t < ntask[j]; ++t) {
                if (j > 0) {
                    const i64 need = std::min(t + D, ntask[j - 1]);
                    while (done[j - 1].load(std::memory_order_acquire) < need) std::this_thread::yield();
                }
                if (t > 0) { cs = ce + 1; ce = std::min(cs + b - 1, n - 1); }
                const i64 k = ce - cs + 1;
                for (i64 c = 0; c < k; ++c) v[c] = cj(A(row, cs + c));
                T tau; R_t<T> beta;
                hgen(k, v.data(), tau, beta);
                apply_right(A, cs, k, v.data(), tau, std::max<i64>(0, cs - w), std::min(n - 1, ce + w));
                A(row, cs) = T(beta);
                for (i64 c = 1; c < k; ++c) A(row, cs + c) = T(0);
                vr.put_at(vptr[j] + t, cs, k, v.data(), tau);
                const i64 rs = cs, re = std::min(std::min(cs + b - 1, n - 1), ce), kr = re - rs + 1;
                for (i64 q = 0; q < kr; ++q) x[q] = A(rs + q, cs);
                T tl; R_t<T> bl;
                hgen(kr, x.data(), tl, bl);
                apply_left(A, rs, kr, x.data(), tl, std::max<i64>(0, rs - w), std::min(n - 1, re + w));
                A(rs, cs) = T(bl);
                for (i64 q = 1; q < kr; ++q) A(rs + q, cs) = T(0);
                ul.put_at(uptr[j] + t, rs, kr, x.data(), tl);
                row = rs;
                done[j].store(t + 1, std::memory_order_release);
            }
        }
    };
    std::vector<std::thread> th;
    for (int r = 1; r < T_; ++r) th.emplace_back(worker, r);
    worker(0);
    for (auto& x : th) x.join();
    ul.cnt = vr.cnt = total;
}

// ---------------------------------------------------------------- steqr
// QL sweeps per eigenvalue before giving up (LAPACK: 30 n total); the
// SLATE_AMD_STEQR_MAXIT override lets tests force non-convergence
// steqr_impl: csrc/include/steqr.hpp (shared with the native library)
using slate_tridiag::steqr_impl;

// bdsqr_impl: csrc/include/bdsqr.hpp (shared with the native library)
using slate_tridiag::bdsqr_impl;

// ---------------------------------------------------------------- secular
// Roots of 1 + rho * sum_i z_i^2 / (d_i - lambda) = 0, d ascending,
// rho > 0 (caller flips signs for rho < 0), all z_i != 0 (deflated before).
// Root j lies in (d_j, d_{j+1}) (last: (d_{n-1}, d_{n-1} + rho |z|^2)).
// Returned as origin index org[j] and offset mu[j] (lambda = d[org] + mu),
// so that d_i - lambda_j = (d_i - d_org) - mu is formed without
// cancellation (needed by the Gu-Eisenstat eigenvector formula).
void secular(i64 n, const double* d, const double* z, double rho, i64* org, double* mu) {
    double zz = 0;
    for (i64 i = 0; i < n; ++i) zz += z[i] * z[i];
    #pragma omp parallel for schedule(dynamic, 16) if (n > 64)
    for (i64 j = 0; j < n; ++j) {
        const double lo_d = d[j];
        const double hi_d = (j + 1 < n) ? d[j + 1] : d[j] + rho * zz;
        // choose the origin by the sign of f at the midpoint
        const double mid = 0.5 * (hi_d - lo_d);
        auto f_at = [&](i64 o, double m) {
            double s = 1;
            for (i64 i = 0; i < n; ++i) s += rho * z[i] * z[i] / ((d[i] - d[o]) - m);
            return s;
        };
        i64 o;
        double a, b;
        if (j + 1 < n && f_at(j, mid) < 0) {   // f increasing in (d_j, d_j+1): root right of mid
            o = j + 1; a = -mid; b = 0;
        } else {
            o = j; a = 0; b = (j + 1 < n) ? mid : (hi_d - lo_d);
        }
        // bisection on mu in (a, b) -- f is increasing in lambda on the interval
        for (int it = 0; it < 200; ++it) {
            double m = 0.5 * (a + b);
            if (m == a || m == b) break;
            double fv = f_at(o, m);
            if (fv < 0) a = m; else b = m;
        }
        org[j] = o;
        mu[j] = 0.5 * (a + b);
    }
}

// Z := H_k Z for reflectors k in [first, first+count) (disjoint rows)
template <typename T>
void apply_refl_host(i64 ncols, T* Z, i64 ldz, const T* V, i64 b, const T* tau, const i64* row, const i64* len,
                     i64 first, i64 count, bool conj_tau) {
    #pragma omp parallel for schedule(static) if (ncols * count > 4096)
    for (i64 c = 0; c < ncols; ++c) {
        for (i64 k = first; k < first + count; ++k) {
            T t = conj_tau ? cj(tau[k]) : tau[k];
            if (t == T(0)) continue;
            const T* v = V + k * b;
            T* z = Z + row[k] + c * ldz;
            T w = 0;
            for (i64 i = 0; i < len[k]; ++i) w += cj(v[i]) * z[i];
            w *= t;
            for (i64 i = 0; i < len[k]; ++i) z[i] -= v[i] * w;
        }
    }
}

template <typename F>
void dispatch(char dt, F&& f) {
    switch (dt) {
        case 's': f(float()); break;
        case 'd': f(double()); break;
        case 'c': f(std::complex<float>()); break;
        case 'z': f(std::complex<double>()); break;
        default: throw std::invalid_argument("bad dtype");
    }
}
template <typename T> T* P(uintptr_t p) { return reinterpret_cast<T*>(p); }

}  // namespace

void register_eig(py::module& m) {
    m.def("hb2st", [](char dt, i64 n, i64 b, uintptr_t A, i64 lda, uintptr_t V, uintptr_t tau, uintptr_t row,
                      uintptr_t len, i64 cap, uintptr_t sweep_ptr) {
        py::gil_scoped_release nogil;
        i64 cnt = 0;
        dispatch(dt, [&](auto z) {
            using T = decltype(z);
            Refl st{(void*)V, (void*)tau, P<i64>(row), P<i64>(len), b, cap};
            int nth = 0;
            if (const char* e = std::getenv("SLATE_AMD_HB2ST_THREADS")) nth = std::atoi(e);
            if (nth <= 0) nth = (int)std::min<unsigned>(32u, std::max(1u, std::thread::hardware_concurrency()));
            cnt = nth == 1 ? hb2st<T>(n, b, P<T>(A), lda, st, P<i64>(sweep_ptr))
                           : hb2st_mt<T>(n, b, P<T>(A), lda, st, P<i64>(sweep_ptr), nth);
        });
        return cnt;
    });
    m.def("tb2bd", [](char dt, i64 n, i64 b, uintptr_t A, i64 lda, uintptr_t UV, uintptr_t Utau, uintptr_t Urow,
                      uintptr_t Ulen, uintptr_t VV, uintptr_t Vtau, uintptr_t Vrow, uintptr_t Vlen, i64 cap,
                      uintptr_t uptr, uintptr_t vptr) {
        i64 cu = 0, cv = 0;
        {
            py::gil_scoped_release nogil;
            dispatch(dt, [&](auto z) {
                using T = decltype(z);
                Refl ul{(void*)UV, (void*)Utau, P<i64>(Urow), P<i64>(Ulen), b, cap};
                Refl vr{(void*)VV, (void*)Vtau, P<i64>(Vrow), P<i64>(Vlen), b, cap};
                int nth = 0;
                if (const char* e = std::getenv("SLATE_AMD_TB2BD_THREADS")) nth = std::atoi(e);
                if (nth <= 0) nth = (int)std::min<unsigned>(32u, std::max(1u, std::thread::hardware_concurrency()));
                if (nth == 1) tb2bd<T>(n, b, P<T>(A), lda, ul, vr, P<i64>(uptr), P<i64>(vptr));
                else tb2bd_mt<T>(n, b, P<T>(A), lda, ul, vr, P<i64>(uptr), P<i64>(vptr), nth);
                cu = ul.cnt; cv = vr.cnt;
            });
        }
        return py::make_tuple(cu, cv);
    });
    m.def("apply_refl", [](char dt, i64 ncols, uintptr_t Z, i64 ldz, uintptr_t V, i64 b, uintptr_t tau,
                           uintptr_t row, uintptr_t len, i64 first, i64 count, bool conj_tau, uintptr_t /*st*/) {
        py::gil_scoped_release nogil;
        dispatch(dt, [&](auto z) {
            using T = decltype(z);
            apply_refl_host<T>(ncols, P<T>(Z), ldz, P<const T>(V), b, P<const T>(tau), P<const i64>(row),
                               P<const i64>(len), first, count, conj_tau);
        });
    });
    m.def("steqr", [](i64 n, uintptr_t d, uintptr_t e, uintptr_t z, i64 ldz, i64 nz) {
        py::gil_scoped_release nogil;
        return steqr_impl<double>(n, P<double>(d), P<double>(e), z ? P<double>(z) : nullptr, ldz, nz);
    });
    m.def("sterf", [](i64 n, uintptr_t d, uintptr_t e) {
        py::gil_scoped_release nogil;
        return steqr_impl<double>(n, P<double>(d), P<double>(e), nullptr, 1, 0);
    });
    m.def("bdsqr", [](i64 n, uintptr_t d, uintptr_t e, uintptr_t u, i64 ldu, i64 nu, uintptr_t vt, i64 ldvt,
                      i64 nv) {
        py::gil_scoped_release nogil;
        return bdsqr_impl(n, P<double>(d), P<double>(e), u ? P<double>(u) : nullptr, ldu, nu,
                          vt ? P<double>(vt) : nullptr, ldvt, nv);
    });
    m.def("secular", [](i64 n, uintptr_t d, uintptr_t z, double rho, uintptr_t org, uintptr_t mu) {
        py::gil_scoped_release nogil;
        secular(n, P<double>(d), P<double>(z), rho, P<i64>(org), P<double>(mu));
    });
}

}  // namespace slate_host
