// Host (CPU) tile kernels: the Target::Host* compute path.
//
// Same operation set and argument conventions as the gfx950 kernels in
// csrc/hip (column-major, 0-based pivots, TriMask output masks), so the
// Python dispatch layer picks _host or _hip purely by where the data lives.
// These replace the host BLAS/LAPACK the reference reaches through
// BLAS++/LAPACK++ (Tile_blas.hh, Tile_lapack.hh,
// Tile_getrf.hh, Tile_geqrf.hh, Tile_householder_reflection_generator.hh).
#include <pybind11/pybind11.h>
#include <pybind11/complex.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <cmath>
#include <complex>
#include <cstdint>
#include <limits>
#include <stdexcept>
#include <vector>
#include <map>
#include <cstring>

namespace py = pybind11;

namespace slate_host {

using i64 = int64_t;
template <typename T> struct real_of { using type = T; };
template <typename T> struct real_of<std::complex<T>> { using type = T; };
template <typename T> using real_t = typename real_of<T>::type;
template <typename T> inline T conj_(T x) { return x; }
template <typename T> inline std::complex<T> conj_(std::complex<T> x) { return std::conj(x); }
template <typename T> inline real_t<T> real_(T x) { return std::real(x); }
template <typename T> inline real_t<T> abs1_(T x) { return std::abs(std::real(x)) + std::abs(std::imag(x)); }
template <typename T> inline T from_c(std::complex<double> z) { return (T)z.real(); }
template <> inline std::complex<float> from_c(std::complex<double> z) { return {(float)z.real(), (float)z.imag()}; }
template <> inline std::complex<double> from_c(std::complex<double> z) { return z; }

struct Mask {
    int mode = 0; i64 nb = 1 << 30; int p = 1, pr = 0, q = 1, pc = 0;
    i64 row_off = 0, col_off = 0, diag_off = 0;
    static i64 l2g(i64 l, i64 nb, int p, int pr) { i64 lt = l / nb; return (lt * p + pr) * nb + (l - lt * nb); }
    bool keep(i64 r, i64 c) const {
        if (!mode) return true;
        i64 gr = l2g(r + row_off, nb, p, pr), gc = l2g(c + col_off, nb, q, pc);
        return mode == 1 ? gr + diag_off >= gc : gr <= gc + diag_off;
    }
};

static Mask make_mask(py::object m) {
    Mask t;
    if (m.is_none()) return t;
    py::tuple tup = m.cast<py::tuple>();
    t.mode = tup[0].cast<int>(); t.nb = tup[1].cast<i64>();
    t.p = tup[2].cast<int>(); t.pr = tup[3].cast<int>();
    t.q = tup[4].cast<int>(); t.pc = tup[5].cast<int>();
    t.row_off = tup[6].cast<i64>(); t.col_off = tup[7].cast<i64>(); t.diag_off = tup[8].cast<i64>();
    return t;
}

// op(X)(r, c) for a column-major X with leading dimension ld.
template <typename T>
inline T opget(const T* X, i64 ld, char op, i64 r, i64 c) {
    if (op == 'N') return X[r + c * ld];
    if (op == 'T') return X[c + r * ld];
    return conj_(X[c + r * ld]);
}

// --------------------------------------------------------------------- gemm
template <typename T>
void gemm(char ta, char tb, i64 m, i64 n, i64 k, T alpha, const T* A, i64 lda,
          const T* B, i64 ldb, T beta, T* C, i64 ldc, const Mask& mask) {
    if (m <= 0 || n <= 0) return;
    #pragma omp parallel for schedule(static) if (m * n * k > 32768)
    for (i64 j = 0; j < n; ++j) {
        std::vector<T> acc(m, T(0));
        for (i64 l = 0; l < k; ++l) {
            T b = opget(B, ldb, tb, l, j);
            if (b == T(0)) continue;
            if (ta == 'N') {
                const T* a = A + l * lda;
                for (i64 i = 0; i < m; ++i) acc[i] += a[i] * b;
            } else {
                for (i64 i = 0; i < m; ++i) acc[i] += opget(A, lda, ta, i, l) * b;
            }
        }
        T* c = C + j * ldc;
        for (i64 i = 0; i < m; ++i) {
            if (!mask.keep(i, j)) continue;
            T v = alpha * acc[i];
            if (beta != T(0)) v += beta * c[i];
            c[i] = v;
        }
    }
}

// --------------------------------------------------------------------- trsm
// op(A) X = alpha B (side L) or X op(A) = alpha B (side R); B overwritten.
template <typename T>
void trsm(char side, char uplo, char trans, char diag, i64 m, i64 n, T alpha,
          const T* A, i64 lda, T* B, i64 ldb) {
    if (m <= 0 || n <= 0) return;
    const bool unit = diag == 'U';
    // effective triangle of op(A): lower if (uplo=L, N) or (uplo=U, T/C)
    const bool lower = (uplo == 'L') == (trans == 'N');
    auto a = [&](i64 r, i64 c) { return opget(A, lda, trans, r, c); };
    if (side == 'L') {
        #pragma omp parallel for schedule(static) if (n > 4)
        for (i64 j = 0; j < n; ++j) {
            T* b = B + j * ldb;
            for (i64 i = 0; i < m; ++i) b[i] *= alpha;
            if (lower) {
                for (i64 i = 0; i < m; ++i) {
                    T s = b[i];
                    for (i64 l = 0; l < i; ++l) s -= a(i, l) * b[l];
                    b[i] = unit ? s : s / a(i, i);
                }
            } else {
                for (i64 i = m - 1; i >= 0; --i) {
                    T s = b[i];
                    for (i64 l = i + 1; l < m; ++l) s -= a(i, l) * b[l];
                    b[i] = unit ? s : s / a(i, i);
                }
            }
        }
    } else {
        // X op(A) = B  <=>  rows: x_r op(A) = b_r
        #pragma omp parallel for schedule(static) if (m > 4)
        for (i64 r = 0; r < m; ++r) {
            for (i64 j = 0; j < n; ++j) B[r + j * ldb] *= alpha;
            if (lower) {  // x_j = (b_j - sum_{l>j} x_l a(l,j)) / a(j,j)
                for (i64 j = n - 1; j >= 0; --j) {
                    T s = B[r + j * ldb];
                    for (i64 l = j + 1; l < n; ++l) s -= B[r + l * ldb] * a(l, j);
                    B[r + j * ldb] = unit ? s : s / a(j, j);
                }
            } else {
                for (i64 j = 0; j < n; ++j) {
                    T s = B[r + j * ldb];
                    for (i64 l = 0; l < j; ++l) s -= B[r + l * ldb] * a(l, j);
                    B[r + j * ldb] = unit ? s : s / a(j, j);
                }
            }
        }
    }
}

// --------------------------------------------------------------------- trmm
// B = alpha op(A) B (side L) or alpha B op(A) (side R)
template <typename T>
void trmm(char side, char uplo, char trans, char diag, i64 m, i64 n, T alpha,
          const T* A, i64 lda, T* B, i64 ldb) {
    if (m <= 0 || n <= 0) return;
    const bool unit = diag == 'U';
    const bool lower = (uplo == 'L') == (trans == 'N');
    auto a = [&](i64 r, i64 c) -> T {
        if (r == c) return unit ? T(1) : opget(A, lda, trans, r, c);
        if (lower ? r < c : r > c) return T(0);
        return opget(A, lda, trans, r, c);
    };
    if (side == 'L') {
        #pragma omp parallel for schedule(static) if (n > 4)
        for (i64 j = 0; j < n; ++j) {
            std::vector<T> x(B + j * ldb, B + j * ldb + m);
            for (i64 i = 0; i < m; ++i) {
                T s(0);
                i64 l0 = lower ? 0 : i, l1 = lower ? i + 1 : m;
                for (i64 l = l0; l < l1; ++l) s += a(i, l) * x[l];
                B[i + j * ldb] = alpha * s;
            }
        }
    } else {
        #pragma omp parallel for schedule(static) if (m > 4)
        for (i64 r = 0; r < m; ++r) {
            std::vector<T> x(n);
            for (i64 j = 0; j < n; ++j) x[j] = B[r + j * ldb];
            for (i64 j = 0; j < n; ++j) {
                T s(0);
                i64 l0 = lower ? j : 0, l1 = lower ? n : j + 1;
                for (i64 l = l0; l < l1; ++l) s += x[l] * a(l, j);
                B[r + j * ldb] = alpha * s;
            }
        }
    }
}

// -------------------------------------------------------------------- potrf
// Returns info (0 = success, k>0: leading minor k not positive definite).
template <typename T>
i64 potrf(char uplo, i64 n, T* A, i64 lda) {
    using R = real_t<T>;
    for (i64 j = 0; j < n; ++j) {
        if (uplo == 'L') {
            R d = real_(A[j + j * lda]);
            for (i64 l = 0; l < j; ++l) d -= std::norm(A[j + l * lda]);
            if (!(d > R(0)) || std::isnan(d)) { A[j + j * lda] = T(d); return j + 1; }
            d = std::sqrt(d);
            A[j + j * lda] = T(d);
            #pragma omp parallel for if (n - j > 256)
            for (i64 i = j + 1; i < n; ++i) {
                T s = A[i + j * lda];
                for (i64 l = 0; l < j; ++l) s -= A[i + l * lda] * conj_(A[j + l * lda]);
                A[i + j * lda] = s / d;
            }
        } else {
            R d = real_(A[j + j * lda]);
            for (i64 l = 0; l < j; ++l) d -= std::norm(A[l + j * lda]);
            if (!(d > R(0)) || std::isnan(d)) { A[j + j * lda] = T(d); return j + 1; }
            d = std::sqrt(d);
            A[j + j * lda] = T(d);
            #pragma omp parallel for if (n - j > 256)
            for (i64 i = j + 1; i < n; ++i) {
                T s = A[j + i * lda];
                for (i64 l = 0; l < j; ++l) s -= conj_(A[l + j * lda]) * A[l + i * lda];
                A[j + i * lda] = s / d;
            }
        }
    }
    return 0;
}

// -------------------------------------------------------------------- trtri
template <typename T>
i64 trtri(char uplo, char diag, i64 n, T* A, i64 lda) {
    const bool unit = diag == 'U';
    if (!unit)
        for (i64 j = 0; j < n; ++j)
            if (A[j + j * lda] == T(0)) return j + 1;
    if (uplo == 'L') {
        for (i64 j = n - 1; j >= 0; --j) {
            T ajj;
            if (!unit) { A[j + j * lda] = T(1) / A[j + j * lda]; ajj = -A[j + j * lda]; }
            else ajj = T(-1);
            // x = A[j+1:, j]; x = L22inv * x; x *= ajj
            i64 m = n - j - 1;
            std::vector<T> x(m);
            for (i64 i = 0; i < m; ++i) x[i] = A[j + 1 + i + j * lda];
            for (i64 i = 0; i < m; ++i) {
                T s(0);
                for (i64 l = 0; l <= i; ++l) {
                    T lv = (l == i) ? (unit ? T(1) : A[j + 1 + i + (j + 1 + l) * lda]) : A[j + 1 + i + (j + 1 + l) * lda];
                    s += lv * x[l];
                }
                A[j + 1 + i + j * lda] = s * ajj;
            }
        }
    } else {
        for (i64 j = 0; j < n; ++j) {
            T ajj;
            if (!unit) { A[j + j * lda] = T(1) / A[j + j * lda]; ajj = -A[j + j * lda]; }
            else ajj = T(-1);
            std::vector<T> x(j);
            for (i64 i = 0; i < j; ++i) x[i] = A[i + j * lda];
            for (i64 i = 0; i < j; ++i) {
                T s(0);
                for (i64 l = i; l < j; ++l) {
                    T uv = (l == i) ? (unit ? T(1) : A[i + l * lda]) : A[i + l * lda];
                    s += uv * x[l];
                }
                A[i + j * lda] = s * ajj;
            }
        }
    }
    return 0;
}

// -------------------------------------------------------------------- getrf
// Partial-pivot LU of an m x n panel.  ipiv[k] = 0-based row swapped with k.
// Returns info (first zero pivot, 1-based) or 0.
template <typename T>
i64 getrf(i64 m, i64 n, T* A, i64 lda, int64_t* ipiv, double threshold) {
    using R = real_t<T>;
    i64 info = 0;
    const i64 mn = std::min(m, n);
    for (i64 k = 0; k < mn; ++k) {
        // pivot search
        i64 p = k; R amax = -1;
        for (i64 i = k; i < m; ++i) {
            R v = abs1_(A[i + k * lda]);
            if (v > amax || std::isnan(v)) { amax = v; p = i; if (std::isnan(v)) break; }
        }
        // threshold pivoting: keep the diagonal if it is within threshold of max
        if (threshold < 0) p = k;
        else if (threshold < 1.0 && abs1_(A[k + k * lda]) >= R(threshold) * amax) p = k;
        ipiv[k] = p;
        if (A[p + k * lda] == T(0)) { if (!info) info = k + 1; continue; }
        if (p != k)
            for (i64 j = 0; j < n; ++j) std::swap(A[k + j * lda], A[p + j * lda]);
        T inv = T(1) / A[k + k * lda];
        for (i64 i = k + 1; i < m; ++i) A[i + k * lda] *= inv;
        #pragma omp parallel for if ((m - k) * (n - k) > 65536)
        for (i64 j = k + 1; j < n; ++j) {
            T u = A[k + j * lda];
            if (u == T(0)) continue;
            for (i64 i = k + 1; i < m; ++i) A[i + j * lda] -= A[i + k * lda] * u;
        }
    }
    return info;
}

// Apply row interchanges ipiv[k1..k2) (0-based, relative) to n columns.
template <typename T>
void laswp(i64 n, T* A, i64 lda, i64 k1, i64 k2, const int64_t* ipiv, int incx) {
    if (incx > 0) {
        for (i64 k = k1; k < k2; ++k) {
            i64 p = ipiv[k];
            if (p != k) for (i64 j = 0; j < n; ++j) std::swap(A[k + j * lda], A[p + j * lda]);
        }
    } else {
        for (i64 k = k2 - 1; k >= k1; --k) {
            i64 p = ipiv[k];
            if (p != k) for (i64 j = 0; j < n; ++j) std::swap(A[k + j * lda], A[p + j * lda]);
        }
    }
}

// -------------------------------------------------------------- householder
// larfg: given alpha = x[0] and x[1:], returns tau and overwrites x[1:] by v[1:],
// x[0] by beta (LAPACK convention H = I - tau v v^H, v[0] = 1).
template <typename T>
T larfg(i64 n, T* x, i64 incx) {
    using R = real_t<T>;
    if (n <= 0) return T(0);
    T alpha = x[0];
    R xnorm = 0;
    {
        R scale = 0, ssq = 1;
        for (i64 i = 1; i < n; ++i) {
            T v = x[i * incx];
            R comps[2] = {std::real(v), std::imag(v)};
            for (R c : comps) if (c != 0) {
                R a = std::abs(c);
                if (scale < a) { ssq = 1 + ssq * (scale / a) * (scale / a); scale = a; }
                else ssq += (a / scale) * (a / scale);
            }
        }
        xnorm = scale * std::sqrt(ssq);
    }
    R ar = std::real(alpha), ai = std::imag(alpha);
    if (xnorm == 0 && ai == 0) return T(0);
    R beta = -std::copysign(std::hypot(std::hypot(ar, ai), xnorm), ar);
    T tau;
    if constexpr (std::is_same<T, R>::value) tau = T((beta - ar) / beta);
    else tau = T((beta - ar) / beta, -ai / beta);
    T scal = T(1) / (alpha - T(beta));
    for (i64 i = 1; i < n; ++i) x[i * incx] *= scal;
    x[0] = T(beta);
    return tau;
}

// geqrf: Householder QR of m x n (unblocked, columnwise), tau[min(m,n)].
template <typename T>
void geqrf(i64 m, i64 n, T* A, i64 lda, T* tau) {
    const i64 k = std::min(m, n);
    for (i64 j = 0; j < k; ++j) {
        T t = larfg(m - j, A + j + j * lda, 1);
        tau[j] = t;
        if (t == T(0)) continue;
        T ajj = A[j + j * lda];
        A[j + j * lda] = T(1);
        // apply H^H = I - conj(tau) v v^H to A[j:, j+1:]
        #pragma omp parallel for if ((m - j) * (n - j) > 65536)
        for (i64 c = j + 1; c < n; ++c) {
            T s(0);
            for (i64 i = j; i < m; ++i) s += conj_(A[i + j * lda]) * A[i + c * lda];
            s *= conj_(t);
            for (i64 i = j; i < m; ++i) A[i + c * lda] -= A[i + j * lda] * s;
        }
        A[j + j * lda] = ajj;
    }
}

// tpqrt panel (host form of csrc/hip/tpqrt.hip): QR of [A; B] for the ib
// columns j0.. of an n x n upper triangle A (pointer at A(j0, j0)) over an
// m x n pentagon B (pointer at B(0, j0)); explicit V (m x ib, zeros outside
// the pentagon), tau, and the panel's ib x ib compact-WY T.
template <typename T>
void tpqrt_panel(i64 m, i64 l, i64 j0, i64 ib, T* A, i64 lda, T* B, i64 ldb, T* V, i64 ldv, T* tau, T* Tm,
                 i64 ldt) {
    using R = typename real_of<T>::type;
    auto rows = [&](i64 gc) { return std::min(m, m - l + std::min(l, gc + 1)); };
    for (i64 i = 0; i < ib; ++i) {
        const i64 pi = rows(j0 + i);
        const T x0 = A[i + i * lda];
        R xn2 = 0;
        for (i64 r = 0; r < pi; ++r) xn2 += std::norm(B[r + i * ldb]);
        const R ar = std::real(x0), ai = std::imag(x0);
        T t(0);
        R beta = ar;
        const bool trivial = (xn2 == R(0) && ai == R(0));
        if (!trivial) {
            beta = -std::copysign(std::sqrt(ar * ar + ai * ai + xn2), ar);
            if constexpr (std::is_same<T, R>::value) t = T((beta - ar) / beta);
            else t = T((beta - ar) / beta, -ai / beta);
        }
        const T den = x0 - T(beta);
        for (i64 r = 0; r < m; ++r) {
            T v(0);
            if (r < pi) {
                v = trivial ? T(0) : B[r + i * ldb] / den;
                B[r + i * ldb] = v;
            }
            V[r + i * ldv] = v;
        }
        A[i + i * lda] = T(beta);
        tau[i] = t;
        const T ct = conj_(t);
        if (ct == T(0)) continue;
        for (i64 c = i + 1; c < ib; ++c) {
            T acc(0);
            for (i64 r = 0; r < pi; ++r) acc += conj_(V[r + i * ldv]) * B[r + c * ldb];
            const T wv = ct * (A[i + c * lda] + acc);
            for (i64 r = 0; r < pi; ++r) B[r + c * ldb] -= V[r + i * ldv] * wv;
            A[i + c * lda] -= wv;
        }
    }
    const i64 pmax = ib ? rows(j0 + ib - 1) : 0;
    for (i64 i = 0; i < ib; ++i) {
        for (i64 a = 0; a < ib; ++a) if (a > i) Tm[a + i * ldt] = T(0);
        std::vector<T> g(i);
        for (i64 a = 0; a < i; ++a) {
            T acc(0);
            for (i64 r = 0; r < pmax; ++r) acc += conj_(V[r + a * ldv]) * V[r + i * ldv];
            g[a] = acc;
        }
        for (i64 a = 0; a < i; ++a) {
            T acc(0);
            for (i64 k = a; k < i; ++k) acc += Tm[a + k * ldt] * g[k];
            Tm[a + i * ldt] = -tau[i] * acc;
        }
        Tm[i + i * ldt] = tau[i];
    }
}

// gelqf: LQ via Householder on rows.
template <typename T>
void gelqf(i64 m, i64 n, T* A, i64 lda, T* tau) {
    const i64 k = std::min(m, n);
    for (i64 j = 0; j < k; ++j) {
        // row j from column j: conj then larfg
        for (i64 c = j; c < n; ++c) A[j + c * lda] = conj_(A[j + c * lda]);
        T t = larfg(n - j, A + j + j * lda, lda);
        tau[j] = t;
        T ajj = A[j + j * lda];
        A[j + j * lda] = T(1);
        if (t != T(0)) {
            #pragma omp parallel for if ((m - j) * (n - j) > 65536)
            for (i64 r = j + 1; r < m; ++r) {
                T s(0);
                for (i64 c = j; c < n; ++c) s += A[r + c * lda] * A[j + c * lda];
                s *= t;
                for (i64 c = j; c < n; ++c) A[r + c * lda] -= s * conj_(A[j + c * lda]);
            }
        }
        A[j + j * lda] = ajj;
        for (i64 c = j + 1; c < n; ++c) A[j + c * lda] = conj_(A[j + c * lda]);
    }
}

// larft (forward, columnwise): T (k x k upper) from V (m x k, unit lower) and tau.
template <typename T>
void larft(i64 m, i64 k, const T* V, i64 ldv, const T* tau, T* Tm, i64 ldt) {
    for (i64 i = 0; i < k; ++i) {
        for (i64 r = i + 1; r < k; ++r) Tm[r + i * ldt] = T(0);
        if (tau[i] == T(0)) {
            for (i64 r = 0; r <= i; ++r) Tm[r + i * ldt] = T(0);
            continue;
        }
        // T(0:i, i) = -tau_i * V(i:m, 0:i)^H V(i:m, i)
        for (i64 r = 0; r < i; ++r) {
            T s = conj_(V[i + r * ldv]);  // v_i(i) = 1
            for (i64 l = i + 1; l < m; ++l) s += conj_(V[l + r * ldv]) * V[l + i * ldv];
            Tm[r + i * ldt] = -tau[i] * s;
        }
        // T(0:i, i) = T(0:i,0:i) * T(0:i, i)
        for (i64 r = 0; r < i; ++r) {
            T s(0);
            for (i64 l = r; l < i; ++l) s += Tm[r + l * ldt] * Tm[l + i * ldt];
            Tm[r + i * ldt] = s;
        }
        Tm[i + i * ldt] = tau[i];
    }
}

// ------------------------------------------------------------------- aux ops
template <typename T>
void geset(char uplo, i64 m, i64 n, T off, T diag, T* A, i64 lda) {
    for (i64 j = 0; j < n; ++j)
        for (i64 i = 0; i < m; ++i) {
            if (uplo == 'L' && i < j) continue;
            if (uplo == 'U' && i > j) continue;
            if (uplo == 'D' && i != j) continue;
            A[i + j * lda] = (i == j) ? diag : off;
        }
}
template <typename T>
void gescale(char uplo, i64 m, i64 n, T s, T* A, i64 lda) {
    for (i64 j = 0; j < n; ++j)
        for (i64 i = 0; i < m; ++i) {
            if (uplo == 'L' && i < j) continue;
            if (uplo == 'U' && i > j) continue;
            if (uplo == 'D' && i != j) continue;
            A[i + j * lda] *= s;
        }
}
template <typename T>
void geadd(char uplo, i64 m, i64 n, T alpha, const T* A, i64 lda, T beta, T* B, i64 ldb) {
    for (i64 j = 0; j < n; ++j)
        for (i64 i = 0; i < m; ++i) {
            if (uplo == 'L' && i < j) continue;
            if (uplo == 'U' && i > j) continue;
            if (uplo == 'D' && i != j) continue;
            B[i + j * ldb] = alpha * A[i + j * lda] + (beta == T(0) ? T(0) : beta * B[i + j * ldb]);
        }
}


// --------------------------------------------------------------- copy/norms
template <typename Ts, typename Td> inline Td cvt(Ts v) {
    if constexpr (std::is_same<Td, float>::value || std::is_same<Td, double>::value) return (Td)std::real(v);
    else return Td((typename Td::value_type)std::real(v), (typename Td::value_type)std::imag(v));
}
template <typename Ts, typename Td>
void gecopy(char uplo, char trans, i64 m, i64 n, const Ts* A, i64 lda, Td* B, i64 ldb) {
    for (i64 j = 0; j < n; ++j)
        for (i64 i = 0; i < m; ++i) {
            if (uplo == 'L' && i < j) continue;
            if (uplo == 'U' && i > j) continue;
            if (uplo == 'D' && i != j) continue;
            Ts v = trans == 'N' ? A[i + j * lda] : A[j + i * lda];
            if (trans == 'C') v = conj_(v);
            B[i + j * ldb] = cvt<Ts, Td>(v);
        }
}
template <typename T>
void genorm(char norm, char uplo, char diag, int herm, i64 m, i64 n, const T* A, i64 lda, real_t<T>* out) {
    using R = real_t<T>;
    R* col = out;
    R* row = out + (norm == 'F' ? 2 * n : n);
    for (i64 j = 0; j < n; ++j) {
        R acc = 0, sc = 0, sq = 1;
        for (i64 i = 0; i < m; ++i) {
            if (uplo == 'L' && i < j) continue;
            if (uplo == 'U' && i > j) continue;
            if (uplo == 'D' && i != j) continue;
            // herm 2: Hermitian -- only the real part of the diagonal is referenced (LAPACK lanhe)
            R v = (i == j && diag == 'U') ? R(1) : (i == j && herm == 2) ? std::abs(std::real(A[i + j * lda]))
                                                                    : std::abs(A[i + j * lda]);
            int reps = (herm && i != j) ? 2 : 1;
            if (norm == 'M') { if (std::isnan(v) || v > acc || std::isnan(acc)) acc = std::isnan(acc) ? acc : v; }
            else if (norm == 'F') {
                for (int r = 0; r < reps; ++r) {
                    if (v != 0) {
                        if (sc < v) { sq = 1 + sq * (sc / v) * (sc / v); sc = v; }
                        else sq += (v / sc) * (v / sc);
                    } else if (std::isnan(v)) sc = v;
                }
            } else if (norm == 'I' && !herm) {
                row[i] += v;
            } else {
                acc += v;
                if (herm && i != j) row[i] += v;
            }
        }
        if (norm == 'F') { col[2 * j] = sc; col[2 * j + 1] = sq; }
        else if (!(norm == 'I' && !herm)) col[j] = acc;
    }
}

// ---------------------------------------------------------------- bindings
// ------------------------------------------------ distributed row interchange
// Host twins of aux.hip's swap_plan / xchg_gather / xchg_scatter / sel_to_ipiv
// (same plan layout, so the Target::HostTask + gloo path runs the same driver).
struct HostSwapPlan {
    int nt;
    int pad;
    int64_t trow[1024];
    int64_t tsrc[1024];
};

static void host_swap_plan(i64 k1, i64 k2, const int64_t* ipiv, i64 ioff, int incx, HostSwapPlan* plan) {
    // same FIXED-slot layout as aux.hip's swap_plan: window row q in slot q,
    // the row that swap q (the last swap targeting it) leaves below the
    // window in slot ns + q, -1 where none; incx < 0 = inverse permutation
    std::memset(plan, 0, sizeof(HostSwapPlan));
    const i64 ns = k2 - k1;
    if (ns <= 0) return;
    if (ns > 512) throw std::invalid_argument("swap_plan: at most 512 swaps per plan");
    std::map<i64, i64> at;                       // position -> original row
    auto get = [&](i64 r) { auto it = at.find(r); return it == at.end() ? r : it->second; };
    std::map<i64, i64> last;                     // row below the window -> last swap targeting it
    for (i64 k = k1; k < k2; ++k) {
        const i64 pv = ipiv[k] - ioff;
        const i64 a = get(k), b = get(pv);
        at[k] = b;
        at[pv] = a;
        if (pv >= k2) last[pv] = k - k1;
    }
    int64_t* dst = incx > 0 ? plan->trow : plan->tsrc;
    int64_t* src = incx > 0 ? plan->tsrc : plan->trow;
    for (i64 q = 0; q < ns; ++q) {
        dst[q] = k1 + q;
        src[q] = get(k1 + q);
        dst[ns + q] = -1;
        src[ns + q] = -1;
    }
    for (auto& kv : last) {
        dst[ns + kv.second] = kv.first;
        src[ns + kv.second] = get(kv.first);
    }
    plan->nt = (int)(2 * ns);
}

static inline i64 host_bc_local_row(i64 g, i64 nb, int p, int pr) {
    const i64 tile = g / nb;
    return (int)(tile % p) == pr ? (tile / p) * nb + g % nb : -1;
}

template <typename F>
static void dispatch(char dt, F&& f) {
    switch (dt) {
        case 's': f(float()); break;
        case 'd': f(double()); break;
        case 'c': f(std::complex<float>()); break;
        case 'z': f(std::complex<double>()); break;
        default: throw std::invalid_argument("bad dtype");
    }
}
template <typename T> static T* P(uintptr_t p) { return reinterpret_cast<T*>(p); }

// One column step of the distributed partial-pivoting LU panel (host form
// of csrc/hip/lu_dist.hip, same record layout and pivot rule): apply column
// j-1 from the p gathered records, then this rank's record of column j.
template <typename T>
static void host_lu_dist_step(i64 nr, T* W, i64 ldw, const int64_t* grow, int c0, int c1, int j, const T* recs,
                              int p, T* Tt, i64 ldt, int64_t* ipiv, int64_t* info, i64 info_off, double thr, T* rec,
                              i64 diag_local) {
    using R = real_t<T>;
    const int b = c1 - c0, recn = 3 + 2 * b;
    auto beats = [](R v, int64_t i, R w, int64_t k) { return (v != v && w == w) || v > w || (v == w && i < k); };
    if (j > c0) {
        const int jp = j - 1, jc = jp - c0;
        R bv = R(-1);
        int64_t bi = (int64_t)1 << 62;
        int win = -1, dwn = -1;
        for (int r = 0; r < p; ++r) {
            const T* rc = recs + (i64)r * recn;
            const R v = std::real(rc[0]);
            if (std::real(rc[2]) != R(0)) dwn = r;
            if (v >= R(0) || v != v) {
                const int64_t gi = (int64_t)std::real(rc[1]);
                if (win < 0 || beats(v, gi, bv, bi)) { bv = v; bi = gi; win = r; }
            }
        }
        bool use_diag = win < 0;
        if (!use_diag && thr < 1.0 && dwn >= 0) {
            const R dj = abs1_(recs[(i64)dwn * recn + 3 + b + jc]);
            if (dj == dj && (double)dj >= thr * (double)bv) use_diag = true;
        }
        const T* drow = recs + (i64)dwn * recn + 3 + b;
        const T* prow = use_diag ? drow : recs + (i64)win * recn + 3;
        const int64_t pg = use_diag ? jp : bi;
        const T u = prow[jc];
        for (i64 i = 0; i < nr; ++i) {
            const int64_t gi = grow[i];
            if (gi < jp) continue;
            T* row = W + i;
            if (gi == jp) {
                for (int c = 0; c < b; ++c) row[c * ldw] = prow[c];
                continue;
            }
            if (gi == pg)
                for (int c = 0; c < b; ++c) row[c * ldw] = drow[c];
            T l = row[jc * ldw];
            if (u != T(0)) l /= u;
            row[jc * ldw] = l;
            for (int c = jc + 1; c < b; ++c) row[c * ldw] -= l * prow[c];
        }
        for (int c = 0; c < b; ++c) Tt[jp + (i64)(c0 + c) * ldt] = prow[c];
        if (ipiv) ipiv[jp] = pg;
        if (u == T(0) && info && *info == 0) *info = jp + 1 + info_off;
    }
    if (j < c1) {
        const int jc = j - c0;
        R v = R(-1);
        i64 bi = -1;
        for (i64 i = 0; i < nr; ++i) {
            if (grow[i] < j) continue;
            const R x = abs1_(W[i + (i64)jc * ldw]);
            if (bi < 0 || beats(x, grow[i], v, grow[bi])) { v = x; bi = i; }
        }
        rec[0] = T(bi >= 0 ? v : R(-1));
        rec[1] = T(bi >= 0 ? (R)grow[bi] : R(1e30));
        rec[2] = T(diag_local >= 0 ? R(1) : R(0));
        for (int c = 0; c < b; ++c) {
            rec[3 + c] = bi >= 0 ? W[bi + (i64)c * ldw] : T(0);
            rec[3 + b + c] = diag_local >= 0 ? W[diag_local + (i64)c * ldw] : T(0);
        }
    }
}

void register_tile_kernels(py::module& m) {
    m.def("lu_dist_step", [](char dt, i64 nr, uintptr_t W, i64 ldw, uintptr_t grow, int c0, int c1, int j,
                             uintptr_t recs, int p, uintptr_t Tt, i64 ldt, uintptr_t ipiv, uintptr_t info,
                             i64 info_off, double thr, uintptr_t rec, uintptr_t /*part*/, i64 diag_local,
                             uintptr_t /*stream*/) {
        dispatch(dt, [&](auto z) {
            using T = decltype(z);
            host_lu_dist_step<T>(nr, P<T>(W), ldw, reinterpret_cast<const int64_t*>(grow), c0, c1, j, P<const T>(recs),
                                 p, P<T>(Tt), ldt, reinterpret_cast<int64_t*>(ipiv),
                                 reinterpret_cast<int64_t*>(info), info_off, thr, P<T>(rec), diag_local);
        });
    });
    m.def("gemm", [](char dt, char ta, char tb, i64 mm, i64 n, i64 k, std::complex<double> alpha,
                     uintptr_t A, i64 lda, uintptr_t B, i64 ldb, std::complex<double> beta,
                     uintptr_t C, i64 ldc, i64 batch, i64 sA, i64 sB, i64 sC, py::object mask,
                     uintptr_t /*stream*/) {
        Mask mk = make_mask(mask);
        py::gil_scoped_release nogil;
        dispatch(dt, [&](auto z) {
            using T = decltype(z);
            for (i64 b = 0; b < batch; ++b)
                gemm<T>(ta, tb, mm, n, k, from_c<T>(alpha), P<T>(A) + b * sA, lda,
                        P<T>(B) + b * sB, ldb, from_c<T>(beta), P<T>(C) + b * sC, ldc, mk);
        });
    });
    m.def("trsm", [](char dt, char side, char uplo, char trans, char diag, i64 mm, i64 n,
                     std::complex<double> alpha, uintptr_t A, i64 lda, uintptr_t B, i64 ldb, uintptr_t) {
        py::gil_scoped_release nogil;
        dispatch(dt, [&](auto z) {
            using T = decltype(z);
            trsm<T>(side, uplo, trans, diag, mm, n, from_c<T>(alpha), P<T>(A), lda, P<T>(B), ldb);
        });
    });
    m.def("trmm", [](char dt, char side, char uplo, char trans, char diag, i64 mm, i64 n,
                     std::complex<double> alpha, uintptr_t A, i64 lda, uintptr_t B, i64 ldb, uintptr_t) {
        py::gil_scoped_release nogil;
        dispatch(dt, [&](auto z) {
            using T = decltype(z);
            trmm<T>(side, uplo, trans, diag, mm, n, from_c<T>(alpha), P<T>(A), lda, P<T>(B), ldb);
        });
    });
    m.def("potrf", [](char dt, char uplo, i64 n, uintptr_t A, i64 lda, uintptr_t info, uintptr_t) {
        i64 r = 0;
        {
            py::gil_scoped_release nogil;
            dispatch(dt, [&](auto z) { using T = decltype(z); r = potrf<T>(uplo, n, P<T>(A), lda); });
        }
        if (info) *reinterpret_cast<int64_t*>(info) = r;
        return r;
    });
    m.def("trtri", [](char dt, char uplo, char diag, i64 n, uintptr_t A, i64 lda, uintptr_t info, uintptr_t) {
        i64 r = 0;
        {
            py::gil_scoped_release nogil;
            dispatch(dt, [&](auto z) { using T = decltype(z); r = trtri<T>(uplo, diag, n, P<T>(A), lda); });
        }
        if (info) *reinterpret_cast<int64_t*>(info) = r;
        return r;
    });
    m.def("getrf", [](char dt, i64 mm, i64 n, uintptr_t A, i64 lda, uintptr_t ipiv, uintptr_t info, double thr,
                      bool nopiv, uintptr_t /*work*/, uintptr_t) {
        i64 r = 0;
        {
            py::gil_scoped_release nogil;
            dispatch(dt, [&](auto z) {
                using T = decltype(z);
                std::vector<int64_t> tmp;
                int64_t* ip = reinterpret_cast<int64_t*>(ipiv);
                if (!ip) { tmp.resize(std::min(mm, n)); ip = tmp.data(); }
                r = getrf<T>(mm, n, P<T>(A), lda, ip, nopiv ? -1.0 : thr);
            });
        }
        if (info) *reinterpret_cast<int64_t*>(info) = r;
        return r;
    });
    m.def("getrf_work_bytes", []() { return (i64)0; });
    m.def("row_scatter", [](char dt, i64 mm, i64 n, uintptr_t A, i64 lda, uintptr_t B, i64 ldb, uintptr_t perm,
                            uintptr_t) {
        dispatch(dt, [&](auto z) {
            using T = decltype(z);
            const int64_t* pr = reinterpret_cast<const int64_t*>(perm);
            for (i64 j = 0; j < n; ++j)
                for (i64 i = 0; i < mm; ++i) P<T>(B)[pr[i] + j * ldb] = P<T>(A)[i + j * lda];
        });
    });
    m.def("laswp", [](char dt, i64 n, uintptr_t A, i64 lda, i64 k1, i64 k2, uintptr_t ipiv, i64 ioff, int incx,
                      uintptr_t) {
        py::gil_scoped_release nogil;
        dispatch(dt, [&](auto z) {
            using T = decltype(z);
            std::vector<int64_t> pv(reinterpret_cast<const int64_t*>(ipiv), reinterpret_cast<const int64_t*>(ipiv) + k2);
            for (auto& x : pv) x -= ioff;
            laswp<T>(n, P<T>(A), lda, k1, k2, pv.data(), incx);
        });
    });
    m.def("swap_plan_bytes", []() { return (i64)sizeof(HostSwapPlan); });
    m.def("swap_plan", [](i64 k1, i64 k2, uintptr_t ipiv, i64 ioff, int incx, uintptr_t plan, uintptr_t) {
        host_swap_plan(k1, k2, reinterpret_cast<const int64_t*>(ipiv), ioff, incx,
                       reinterpret_cast<HostSwapPlan*>(plan));
    });
    m.def("xchg_gather", [](char dt, uintptr_t plan, i64 nslot, i64 n, uintptr_t A, i64 lda, uintptr_t X, i64 ldx,
                            i64 nb, int p, int pr, uintptr_t) {
        const HostSwapPlan* pl = reinterpret_cast<const HostSwapPlan*>(plan);
        dispatch(dt, [&](auto z) {
            using T = decltype(z);
            for (i64 t = 0; t < nslot; ++t) {
                const i64 src = t < pl->nt ? pl->tsrc[t] : -1;
                const i64 lr = src >= 0 ? host_bc_local_row(src, nb, p, pr) : -1;
                for (i64 j = 0; j < n; ++j) P<T>(X)[t + j * ldx] = lr >= 0 ? P<T>(A)[lr + j * lda] : T(0);
            }
        });
    });
    m.def("xchg_scatter", [](char dt, uintptr_t plan, i64 nslot, i64 n, uintptr_t X, i64 ldx, uintptr_t A, i64 lda,
                             i64 nb, int p, int pr, uintptr_t) {
        const HostSwapPlan* pl = reinterpret_cast<const HostSwapPlan*>(plan);
        dispatch(dt, [&](auto z) {
            using T = decltype(z);
            for (i64 t = 0; t < std::min<i64>(nslot, pl->nt); ++t) {
                if (pl->trow[t] < 0) continue;
                const i64 lr = host_bc_local_row(pl->trow[t], nb, p, pr);
                if (lr < 0) continue;
                for (i64 j = 0; j < n; ++j) P<T>(A)[lr + j * lda] = P<T>(X)[t + j * ldx];
            }
        });
    });
    m.def("sel_to_ipiv", [](uintptr_t sel, i64 kb, i64 r0, uintptr_t ipiv, uintptr_t) {
        const int64_t* sl = reinterpret_cast<const int64_t*>(sel);
        int64_t* ip = reinterpret_cast<int64_t*>(ipiv);
        std::map<i64, i64> at;   // position -> original row
        std::map<i64, i64> pos;  // original row -> position
        auto where = [&](i64 r) { auto it = pos.find(r); return it == pos.end() ? r : it->second; };
        auto orig = [&](i64 x) { auto it = at.find(x); return it == at.end() ? x : it->second; };
        for (i64 i = 0; i < kb; ++i) {
            const i64 a = r0 + i, b = where(sl[i]);
            ip[i] = b - r0;
            const i64 oa = orig(a), ob = orig(b);
            at[a] = ob; at[b] = oa;
            pos[ob] = a; pos[oa] = b;
        }
    });
    m.def("row_gather", [](char dt, i64 mm, i64 n, uintptr_t A, i64 lda, uintptr_t B, i64 ldb, uintptr_t perm,
                           uintptr_t) {
        dispatch(dt, [&](auto z) {
            using T = decltype(z);
            const int64_t* pr = reinterpret_cast<const int64_t*>(perm);
            for (i64 j = 0; j < n; ++j)
                for (i64 i = 0; i < mm; ++i) P<T>(B)[i + j * ldb] = P<T>(A)[pr[i] + j * lda];
        });
    });
    m.def("geqrf", [](char dt, i64 mm, i64 n, uintptr_t A, i64 lda, uintptr_t tau) {
        py::gil_scoped_release nogil;
        dispatch(dt, [&](auto z) { using T = decltype(z); geqrf<T>(mm, n, P<T>(A), lda, P<T>(tau)); });
    });
    m.def("tpqrt_panel", [](char dt, i64 mm, i64 l, i64 j0, int ib, uintptr_t A, i64 lda, uintptr_t B, i64 ldb,
                            uintptr_t V, i64 ldv, uintptr_t tau, uintptr_t Tm, i64 ldt, uintptr_t) {
        py::gil_scoped_release nogil;
        dispatch(dt, [&](auto z) { using T = decltype(z);
            tpqrt_panel<T>(mm, l, j0, ib, P<T>(A), lda, P<T>(B), ldb, P<T>(V), ldv, P<T>(tau), P<T>(Tm), ldt); });
    });
    m.def("gelqf", [](char dt, i64 mm, i64 n, uintptr_t A, i64 lda, uintptr_t tau) {
        py::gil_scoped_release nogil;
        dispatch(dt, [&](auto z) { using T = decltype(z); gelqf<T>(mm, n, P<T>(A), lda, P<T>(tau)); });
    });
    m.def("larft", [](char dt, i64 mm, i64 k, uintptr_t V, i64 ldv, uintptr_t tau, uintptr_t Tm, i64 ldt) {
        py::gil_scoped_release nogil;
        dispatch(dt, [&](auto z) {
            using T = decltype(z);
            larft<T>(mm, k, P<T>(V), ldv, P<T>(tau), P<T>(Tm), ldt);
        });
    });
    m.def("gecopy", [](char ds, char dd, char uplo, char trans, i64 mm, i64 n, uintptr_t A, i64 lda, uintptr_t B,
                       i64 ldb, uintptr_t) {
        py::gil_scoped_release nogil;
        dispatch(ds, [&](auto zs) { using Ts = decltype(zs);
            dispatch(dd, [&](auto zd) { using Td = decltype(zd);
                gecopy<Ts, Td>(uplo, trans, mm, n, P<Ts>(A), lda, P<Td>(B), ldb); }); });
    });
    m.def("genorm", [](char dt, char norm, char uplo, char diag, int herm, i64 mm, i64 n, uintptr_t A, i64 lda,
                       uintptr_t out, uintptr_t) {
        py::gil_scoped_release nogil;
        dispatch(dt, [&](auto z) { using T = decltype(z);
            genorm<T>(norm, uplo, diag, herm, mm, n, P<T>(A), lda, P<real_t<T>>(out)); });
    });
    m.def("butterfly", [](char dt, bool trans, bool rows, int depth, i64 nidx, i64 nother, uintptr_t A, i64 lda,
                          uintptr_t diag, i64 ldd, uintptr_t) {
        dispatch(dt, [&](auto z) { using T = decltype(z); using R = real_t<T>;
            if (depth <= 0 || nidx <= 0 || nother <= 0) return;
            if (nidx % (i64(1) << depth)) throw std::invalid_argument("butterfly: n % 2^depth != 0");
            const R* dg = P<R>(diag);
            T* a = P<T>(A);
            const R sq = R(0.70710678118654752440);
            auto at = [&](i64 idx, i64 j) -> T& { return rows ? a[idx + j * lda] : a[j + idx * lda]; };
            for (int s = 0; s < depth; ++s) {
                const int l = trans ? depth - 1 - s : s;
                const i64 size = nidx >> l, h = size / 2;
                for (i64 o = 0; o < nidx; o += size)
                    for (i64 j = 0; j < nother; ++j)
                        for (i64 i = 0; i < h; ++i) {
                            const T x = at(o + i, j), y = at(o + h + i, j);
                            const R r0 = dg[l * ldd + o + i] * sq, r1 = dg[l * ldd + o + h + i] * sq;
                            if (!trans) { at(o + i, j) = r0 * x + r1 * y; at(o + h + i, j) = r0 * x - r1 * y; }
                            else { at(o + i, j) = r0 * (x + y); at(o + h + i, j) = r1 * (x - y); }
                        }
            }
        });
    });
    m.def("gescale_row_col", [](char dt, char equed, i64 mm, i64 n, uintptr_t r, uintptr_t c, uintptr_t A, i64 lda,
                                uintptr_t) {
        dispatch(dt, [&](auto z) { using T = decltype(z); using R = real_t<T>;
            const R* rr = P<R>(r); const R* cc = P<R>(c);
            for (i64 j = 0; j < n; ++j)
                for (i64 i = 0; i < mm; ++i) {
                    R sfac = 1;
                    if (equed == 'S') {
                        T& a = P<T>(A)[i + j * lda];
                        const R mg = std::abs(a);
                        a = mg > R(0) ? a / mg : T(1);
                        continue;
                    }
                    if (equed == 'R' || equed == 'B') sfac *= rr[i];
                    if (equed == 'C' || equed == 'B') sfac *= cc[j];
                    P<T>(A)[i + j * lda] *= sfac;
                }
        });
    });
    m.def("geset", [](char dt, char uplo, i64 mm, i64 n, std::complex<double> off, std::complex<double> diag,
                      uintptr_t A, i64 lda, uintptr_t) {
        dispatch(dt, [&](auto z) {
            using T = decltype(z);
            geset<T>(uplo, mm, n, from_c<T>(off), from_c<T>(diag), P<T>(A), lda);
        });
    });
    m.def("gescale", [](char dt, char uplo, i64 mm, i64 n, std::complex<double> s, uintptr_t A, i64 lda, uintptr_t) {
        dispatch(dt, [&](auto z) { using T = decltype(z); gescale<T>(uplo, mm, n, from_c<T>(s), P<T>(A), lda); });
    });
    // B = A where the block-cyclic triangle mask keeps the element, 0 else
    m.def("gecopy_mask", [](char dt, py::object mask, i64 mm, i64 n, uintptr_t A, i64 lda, uintptr_t B, i64 ldb,
                            int real_diag, uintptr_t) {
        const Mask mk = make_mask(mask);
        dispatch(dt, [&](auto z) {
            using T = decltype(z);
            const T* a = P<T>(A);
            T* b = P<T>(B);
            for (i64 j = 0; j < n; ++j)
                for (i64 i = 0; i < mm; ++i) {
                    T v = mk.keep(i, j) ? a[i + j * lda] : T(0);
                    if (real_diag && Mask::l2g(i + mk.row_off, mk.nb, mk.p, mk.pr) ==
                                         Mask::l2g(j + mk.col_off, mk.nb, mk.q, mk.pc))
                        v = T(real_(v));
                    b[i + j * ldb] = v;
                }
        });
    });
    m.def("geadd", [](char dt, char uplo, i64 mm, i64 n, std::complex<double> alpha, uintptr_t A, i64 lda,
                      std::complex<double> beta, uintptr_t B, i64 ldb, uintptr_t) {
        dispatch(dt, [&](auto z) {
            using T = decltype(z);
            geadd<T>(uplo, mm, n, from_c<T>(alpha), P<T>(A), lda, from_c<T>(beta), P<T>(B), ldb);
        });
    });
}

}  // namespace slate_host
