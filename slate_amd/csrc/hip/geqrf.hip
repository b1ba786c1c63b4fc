// Householder QR panel on gfx950 -- replaces the host/tile panel of SLATE's
// geqrf (src/geqrf.cc:96-160 -> internal::geqrf, Tile_geqrf.hh:97-330,
// a multi-threaded host kernel with a thread barrier per column).
//
// Recursive (Elmroth-Gustavson) so the bulk of the panel is MFMA GEMM/TRMM:
//   qr(A) = qr(A1); A2 -= V1 (T11^H (V1^H A2)); qr(A2'); T12 = -T11 (V1^H V2) T22
// and the compact-WY factor T of the whole panel falls out of the recursion
// (no separate larft pass).  The explicit unit-lower V of the panel is
// written to a caller buffer, ready for the trailing update GEMMs.
//
// Base case (<= 32 columns): two launches per column over many workgroups,
// ordered only by kernel boundaries (no fences/atomics):
//   A_j: reduce launch B_{j-1}'s partials -> w = conj(tau) v^H A(:, j:) and
//        the Gram column V^H v (WG 0 extends T); apply reflector j-1 to
//        columns >= j on own rows; partial ||A(j+1:, j)||^2.
//   B_j: reduce the norm partials -> larfg (beta, tau, 1/(alpha-beta)),
//        identically in every workgroup; scale own rows of v_j; publish
//        partials of v_j^H A(:, j+1:) and V(:, <j)^H v_j.
#include <type_traits>
#include "common.hpp"
#include "kernels.hpp"
#include "launchers.hpp"
#include "workspace.hpp"

namespace slate_hip {

namespace {
constexpr int QB = 32;           // base-case width
constexpr int QT = 256;          // threads per workgroup
constexpr int QMAXG = 256;       // max workgroups per base launch

template <typename T>
struct QrBuf {
    double npart[QMAXG];         // partial squared norms
    T wpart[QMAXG][QB];          // partial v^H A(:, c)
    T gpart[QMAXG][QB];          // partial V(:, l)^H v
    T beta;                      // beta of the last reflector (written to A by the next launch)
};
constexpr size_t QR_BYTES = sizeof(QrBuf<zcplx>);

template <typename T>
__device__ inline typename scalar_traits<T>::real abs2(T x) {
    if constexpr (scalar_traits<T>::is_complex) return x.re * x.re + x.im * x.im;
    else return x * x;
}

}  // namespace

template <typename T>
__global__ void __launch_bounds__(QT)
qr_step_a(i64 m, int c0, int c1, int j, T* A, i64 lda, T* tau, T* Tm, i64 ldt, void* work) {
    using R = typename scalar_traits<T>::real;
    QrBuf<T>* qb = reinterpret_cast<QrBuf<T>*>(work);
    __shared__ T wsum[QB];
    __shared__ T gsum[QB];
    __shared__ T red[QT];
    __shared__ R rr[QT];
    const int G = gridDim.x, g = blockIdx.x, tid = threadIdx.x;
    const i64 rows_per = (m + G - 1) / G;
    const i64 r0 = (i64)g * rows_per, r1 = min(m, r0 + rows_per);
    const int pc = j - 1;
    if (j > c0) {
        // ---- reduce partials of launch B_{pc}: columns (pc, c1) of w and
        //      Gram entries [c0, pc) -- 8 groups of 32 lanes over workgroups
        const int col = tid % QB, grp = tid / QB;          // 8 groups
        T sw = s_zero(T()), sg = s_zero(T());
        for (int q = grp; q < G; q += QT / QB) {
            sw = s_add(sw, qb->wpart[q][col]);
            sg = s_add(sg, qb->gpart[q][col]);
        }
        red[tid] = sw;
        __syncthreads();
        if (tid < QB) {
            T a = red[tid];
            for (int k = 1; k < QT / QB; ++k) a = s_add(a, red[tid + k * QB]);
            wsum[tid] = a;
        }
        __syncthreads();
        red[tid] = sg;
        __syncthreads();
        if (tid < QB) {
            T a = red[tid];
            for (int k = 1; k < QT / QB; ++k) a = s_add(a, red[tid + k * QB]);
            gsum[tid] = a;
        }
        __syncthreads();
        const T tp = tau[pc];
        if (pc >= r0 && pc < r1 && tid == 0) A[pc + (i64)pc * lda] = qb->beta;
        if (tid < QB) wsum[tid] = s_mul(s_conj(tp), wsum[tid]);
        __syncthreads();
        // ---- WG 0 extends T: T(c0:pc, pc) = -tau T(c0:pc, c0:pc) g
        if (g == 0 && tid < pc - c0) {
            T acc = s_zero(T());
            for (int k = tid; k < pc - c0; ++k)
                acc = s_add(acc, s_mul(Tm[(c0 + tid) + (i64)(c0 + k) * ldt], gsum[k]));
            Tm[(c0 + tid) + (i64)pc * ldt] = s_mul(s_from_real(T(), -1), s_mul(tp, acc));
        }
        if (j >= c1) return;
        // ---- apply H_pc^H to columns [j, c1) on own rows >= pc
        for (i64 i = r0 + tid; i < r1; i += QT) {
            if (i < pc) continue;
            const T v = (i == pc) ? s_from_real(T(), 1) : A[i + (i64)pc * lda];
            T a[QB];   // whole row segment in registers: loads issue together
            #pragma unroll
            for (int c = 0; c < QB; ++c)
                if (c0 + c >= j && c0 + c < c1) a[c] = A[i + (i64)(c0 + c) * lda];
            #pragma unroll
            for (int c = 0; c < QB; ++c)
                if (c0 + c >= j && c0 + c < c1) A[i + (i64)(c0 + c) * lda] = s_sub(a[c], s_mul(v, wsum[c]));
        }
    }
    // ---- partial ||A(j+1:m, j)||^2 over own rows (same thread wrote them)
    R part = R(0);
    for (i64 i = r0 + tid; i < r1; i += QT)   // same row->thread map as the update above
        if (i > j) part += abs2(A[i + (i64)j * lda]);
    rr[tid] = part;
    __syncthreads();
    for (int o = QT / 2; o > 0; o >>= 1) {
        if (tid < o) rr[tid] += rr[tid + o];
        __syncthreads();
    }
    if (tid == 0) qb->npart[g] = (double)rr[0];
}

template <typename T>
__global__ void __launch_bounds__(QT)
qr_step_b(i64 m, int c0, int c1, int j, T* A, i64 lda, T* tau, T* Tm, i64 ldt, void* work) {
    using R = typename scalar_traits<T>::real;
    QrBuf<T>* qb = reinterpret_cast<QrBuf<T>*>(work);
    __shared__ double dd[QT];
    __shared__ T red[4][QB];
    const int G = gridDim.x, g = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const i64 rows_per = (m + G - 1) / G;
    const i64 r0 = (i64)g * rows_per, r1 = min(m, r0 + rows_per);
    // ---- larfg, identically in every workgroup
    double s = 0;
    for (int q = tid; q < G; q += QT) s += qb->npart[q];
    dd[tid] = s;
    __syncthreads();
    for (int o = QT / 2; o > 0; o >>= 1) {
        if (tid < o) dd[tid] += dd[tid + o];
        __syncthreads();
    }
    const R xn2 = (R)dd[0];
    const T alpha = A[j + (i64)j * lda];
    T tj, scal;
    R beta;
    {
        R are, aim;
        if constexpr (scalar_traits<T>::is_complex) { are = alpha.re; aim = alpha.im; }
        else { are = alpha; aim = R(0); }
        if (xn2 == R(0) && aim == R(0)) {
            tj = s_zero(T()); scal = s_from_real(T(), 1); beta = are;
        } else {
            beta = -copysign(sqrt(are * are + aim * aim + xn2), are);
            if constexpr (scalar_traits<T>::is_complex) {
                tj = T{(beta - are) / beta, -aim / beta};
                scal = s_div(s_from_real(T(), 1), T{are - beta, aim});
            } else {
                tj = (beta - are) / beta;
                scal = R(1) / (are - beta);
            }
        }
    }
    // A(j, j) = beta is written by the NEXT launch: other workgroups of this
    // one may still be reading alpha from it
    if (g == 0 && tid == 0) {
        tau[j] = tj;
        Tm[j + (i64)j * ldt] = tj;
        qb->beta = s_from_real(T(), beta);
    }
    // ---- scale v on own rows, accumulate partials
    //   w_c = sum_i conj(v_i) A(i, c), c in (j, c1);  g_l = sum_i conj(V(i, l)) v_i, l in [c0, j)
    // acc[c] <-> column c0 + c:  Gram entry (c0 + c < j) or w entry (> j)
    const int w = c1 - c0, jj = j - c0;
    T acc[QB];
    #pragma unroll
    for (int c = 0; c < QB; ++c) acc[c] = s_zero(T());
    for (i64 i = r0 + tid; i < r1; i += QT) {
        if (i < j) continue;
        T v;
        if (i == j) v = s_from_real(T(), 1);
        else {
            v = s_mul(A[i + (i64)j * lda], scal);
            A[i + (i64)j * lda] = v;
        }
        const T cv = s_conj(v);
        #pragma unroll
        for (int c = 0; c < QB; ++c) {
            if (c < jj) acc[c] = s_add(acc[c], s_mul(s_conj(A[i + (i64)(c0 + c) * lda]), v));
            else if (c > jj && c < w) acc[c] = s_add(acc[c], s_mul(cv, A[i + (i64)(c0 + c) * lda]));
        }
    }
    // wave reduce then across the 4 waves
    #pragma unroll
    for (int c = 0; c < QB; ++c) {
        if (c < w && c != jj) { T t = wave_sum(acc[c]); if (lane == 0) red[wv][c] = t; }
    }
    __syncthreads();
    if (tid < w && tid != jj) {
        T a = s_add(s_add(red[0][tid], red[1][tid]), s_add(red[2][tid], red[3][tid]));
        if (tid < jj) qb->gpart[g][tid] = a;
        else qb->wpart[g][tid] = a;
    }
}

// Vout(i, c) = A(i, c) below the diagonal, 1 on it, 0 above (m x n)
template <typename T>
__global__ void v_explicit_kernel(i64 m, i64 n, const T* A, i64 lda, T* V, i64 ldv) {
    const i64 i = (i64)blockIdx.x * 256 + threadIdx.x;
    if (i >= m) return;
    for (i64 c = blockIdx.y; c < n; c += gridDim.y)
        V[i + c * ldv] = i > c ? A[i + c * lda] : (i == c ? s_from_real(T(), 1) : s_zero(T()));
}

template <typename T>
void v_explicit(i64 m, i64 n, const T* A, i64 lda, T* V, i64 ldv, hipStream_t s) {
    if (m <= 0 || n <= 0) return;
    dim3 grid((unsigned)((m + 255) / 256), (unsigned)std::min<i64>(n, 64));
    hipLaunchKernelGGL(v_explicit_kernel<T>, grid, dim3(256), 0, s, m, n, A, lda, V, ldv);
    HIP_LAUNCH_CHECK();
}

template <typename T>
static void qr_base(i64 m, int n, T* A, i64 lda, T* tau, T* Tm, i64 ldt, void* w, hipStream_t s) {
    const int G = (int)std::min<i64>(QMAXG, std::max<i64>(1, (m + QT - 1) / QT));
    for (int j = 0; j < n; ++j) {
        hipLaunchKernelGGL(qr_step_a<T>, dim3(G), dim3(QT), 0, s, m, 0, n, j, A, lda, tau, Tm, ldt, w);
        hipLaunchKernelGGL(qr_step_b<T>, dim3(G), dim3(QT), 0, s, m, 0, n, j, A, lda, tau, Tm, ldt, w);
    }
    hipLaunchKernelGGL(qr_step_a<T>, dim3(G), dim3(QT), 0, s, m, 0, n, n, A, lda, tau, Tm, ldt, w);
    HIP_LAUNCH_CHECK();
}

template <typename T>
static void gemm_T(char ta, char tb, i64 m, i64 n, i64 k, T alpha, const T* A, i64 lda,
                   const T* B, i64 ldb, T beta, T* C, i64 ldc, hipStream_t s) {
    if (m <= 0 || n <= 0) return;
    GemmCall c;
    c.transA = ta; c.transB = tb; c.m = m; c.n = n; c.k = k;
    c.A = A; c.lda = lda; c.B = B; c.ldb = ldb; c.C = C; c.ldc = ldc;
    if constexpr (scalar_traits<T>::is_complex) {
        c.alpha_re = alpha.re; c.alpha_im = alpha.im; c.beta_re = beta.re; c.beta_im = beta.im;
        gemm_complex<T>(c, s);
    } else {
        c.alpha_re = alpha; c.beta_re = beta;
        gemm_real<T>(c, s);
    }
}

// A (m x n) -> R + implicit V, tau, T (n x n upper), explicit V (m x n)
template <typename T>
static void qr_rec(i64 m, i64 n, T* A, i64 lda, T* tau, T* Tm, i64 ldt, T* V, i64 ldv, T* W,
                   void* w, hipStream_t s) {
    const char ct = scalar_traits<T>::is_complex ? 'C' : 'T';
    const T one = s_from_real(T(), 1), zero = s_zero(T()), mone = s_from_real(T(), -1);
    if (n <= QB) {
        qr_base<T>(m, (int)n, A, lda, tau, Tm, ldt, w, s);
        v_explicit<T>(m, n, A, lda, V, ldv, s);
        return;
    }
    i64 n1 = ((n / 2 + QB - 1) / QB) * QB;
    if (n1 >= n) n1 = n - QB;
    const i64 n2 = n - n1;
    qr_rec<T>(m, n1, A, lda, tau, Tm, ldt, V, ldv, W, w, s);
    T* A2 = A + n1 * lda;
    // A2 -= V1 T11^H V1^H A2      (W: n1 x n2)
    gemm_T<T>(ct, 'N', n1, n2, m, one, V, ldv, A2, lda, zero, W, n1, s);
    trmm<T>('L', 'U', ct, 'N', n1, n2, one, Tm, ldt, W, n1, s);
    gemm_T<T>('N', 'N', m, n2, n1, mone, V, ldv, W, n1, one, A2, lda, s);
    // V(:, n1:) is zero above row n1
    HIP_CHECK(hipMemset2DAsync(V + n1 * ldv, ldv * sizeof(T), 0, n1 * sizeof(T), n2, s));
    qr_rec<T>(m - n1, n2, A2 + n1, lda, tau + n1, Tm + n1 + n1 * ldt, ldt, V + n1 + n1 * ldv, ldv, W, w, s);
    // T12 = -T11 (V1^H V2) T22, V2 zero above row n1
    T* T12 = Tm + n1 * ldt;
    gemm_T<T>(ct, 'N', n1, n2, m - n1, one, V + n1, ldv, V + n1 + n1 * ldv, ldv, zero, T12, ldt, s);
    trmm<T>('L', 'U', 'N', 'N', n1, n2, mone, Tm, ldt, T12, ldt, s);
    trmm<T>('R', 'U', 'N', 'N', n1, n2, one, Tm + n1 + n1 * ldt, ldt, T12, ldt, s);
}

template <typename T>
void geqrf_panel_ws(i64 m, i64 n, T* A, i64 lda, T* tau, T* Tm, i64 ldt, T* V, i64 ldv, void* work,
                    hipStream_t s) {
    if (m <= 0 || n <= 0) return;
    const i64 k = std::min(m, n);
    if constexpr (std::is_same<T, double>::value) {
        // tall fp64 panel: shifted CholeskyQR3 + Householder reconstruction
        // (qr_fast.hip); a breakdown restores the panel and lands here
        if (m >= 8 * n && geqrf_cholqr(m, n, A, lda, tau, Tm, ldt, V, ldv, s)) return;
    }
    // T is upper triangular: zero the strict lower part once
    geset<T>('L', k, k, s_zero(T()), s_zero(T()), Tm, ldt, s);
    T* W = static_cast<T*>(workspace(s, sizeof(T) * (size_t)k * k, WS_QW));
    qr_rec<T>(m, k, A, lda, tau, Tm, ldt, V, ldv, W, work, s);
    if (n > k) {   // wide panel (m < n): apply Q^H to the remaining columns
        T* Wr = static_cast<T*>(workspace(s, sizeof(T) * (size_t)k * (n - k), WS_QW2));
        const char ct = scalar_traits<T>::is_complex ? 'C' : 'T';
        const T one = s_from_real(T(), 1), zero = s_zero(T()), mone = s_from_real(T(), -1);
        gemm_T<T>(ct, 'N', k, n - k, m, one, V, ldv, A + k * lda, lda, zero, Wr, k, s);
        trmm<T>('L', 'U', ct, 'N', k, n - k, one, Tm, ldt, Wr, k, s);
        gemm_T<T>('N', 'N', m, n - k, k, mone, V, ldv, Wr, k, one, A + k * lda, lda, s);
    }
}

size_t geqrf_work_bytes() { return QR_BYTES; }

#define INST(T)                                                                                   \
    template void geqrf_panel_ws<T>(i64, i64, T*, i64, T*, T*, i64, T*, i64, void*, hipStream_t); \
    template void v_explicit<T>(i64, i64, const T*, i64, T*, i64, hipStream_t);
INST(float) INST(double) INST(ccplx) INST(zcplx)
#undef INST

}  // namespace slate_hip
