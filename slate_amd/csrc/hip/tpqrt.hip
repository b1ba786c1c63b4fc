// Triangle-pentagonal QR panel (the tile kernel behind SLATE's TSQR tree:
// tile::tpqrt, src/internal/Tile_tpqrt.hh:142, used by internal::ttqrt and
// internal::ttmqr, src/internal/internal_ttqrt.cc:34-130).
//
// QR of the stacked [A; B]: A is n x n upper triangular, B is m x n
// pentagonal (its first m - l rows full, its last l rows upper trapezoidal).
// The reflectors have the form v = [e_i; v_B] -- the top part of every
// Householder vector is a unit vector, so the triangle A is never filled in
// and only B's pentagon carries reflector data.
//
// MI355X mapping: this kernel factors ONE ib-wide column panel (ib <= 64)
// in a single workgroup of 512 threads (8 waves): the reflector by wave 0,
// the panel's own trailing columns a wave per column (lanes over rows,
// coalesced), and at the end the panel's compact-WY factor T from
// G = V_B^H V_B (a wave per entry) with the triangular recurrence in LDS.
// Everything outside the panel -- the trailing columns of the tile (tprfb)
// and the merge of the panel T's into the full n x n T -- is MFMA GEMM /
// TRMM work issued by the caller (ops.tpqrt), like the blocked geqrf.
#include "common.hpp"
#include "kernels.hpp"

namespace slate_hip {

namespace {
constexpr int TP_THREADS = 512;
constexpr int TP_MAXIB = 64;
}

// rows of B that column c (global column index gc) of the pentagon holds
__host__ __device__ inline i64 tp_rows(i64 m, i64 l, i64 gc) {
    const i64 p = m - l + (l < gc + 1 ? l : gc + 1);
    return p < m ? p : m;
}

template <typename T>
__global__ void __launch_bounds__(TP_THREADS)
tpqrt_panel_kernel(i64 m, i64 l, i64 j0, int ib, T* __restrict__ A, i64 lda, T* __restrict__ B, i64 ldb,
                   T* __restrict__ V, i64 ldv, T* __restrict__ tau, T* __restrict__ Tm, i64 ldt) {
    using R = typename scalar_traits<T>::real;
    constexpr int NW = TP_THREADS / 64;
    __shared__ T s_tau[TP_MAXIB];
    __shared__ T s_G[TP_MAXIB * TP_MAXIB];
    __shared__ T s_T[TP_MAXIB * TP_MAXIB];
    const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
    auto Ab = [&](i64 r, i64 c) -> T& { return A[r + c * lda]; };
    auto Bb = [&](i64 r, i64 c) -> T& { return B[r + c * ldb]; };
    for (int i = 0; i < ib; ++i) {
        const i64 pi = tp_rows(m, l, j0 + i);
        // ---- reflector of column i (wave 0)
        if (w == 0) {
            const T x0 = Ab(i, i);
            R xn2 = 0;
            for (i64 r = lane; r < pi; r += 64) {
                const T x = Bb(r, i);
                xn2 += s_real(s_mul(s_conj(x), x));
            }
            xn2 = wave_sum(xn2);
            const R ar = s_real(x0);
            R ai = 0;
            if constexpr (scalar_traits<T>::is_complex) ai = x0.im;
            T t;
            R beta;
            const bool trivial = (xn2 == R(0) && ai == R(0));
            if (trivial) {
                t = s_zero(T());
                beta = ar;
            } else {
                beta = -copysign(sqrt(ar * ar + ai * ai + xn2), ar);
                if constexpr (scalar_traits<T>::is_complex) t = T{(beta - ar) / beta, -ai / beta};
                else t = (beta - ar) / beta;
            }
            T den = x0;
            if constexpr (scalar_traits<T>::is_complex) den.re -= beta;
            else den -= beta;
            for (i64 r = lane; r < m; r += 64) {
                T v = s_zero(T());
                if (r < pi) {
                    v = trivial ? s_zero(T()) : s_div(Bb(r, i), den);
                    Bb(r, i) = v;
                }
                V[r + i * ldv] = v;
            }
            if (lane == 0) {
                Ab(i, i) = s_from_real(T(), beta);
                s_tau[i] = t;
                tau[i] = t;
            }
        }
        __syncthreads();
        // ---- apply H_i^H to the panel's columns c > i: a wave per column
        const T ct = s_conj(s_tau[i]);
        if (!s_is_zero(ct)) {
            for (int c = i + 1 + w; c < ib; c += NW) {
                T acc = s_zero(T());
                for (i64 r = lane; r < pi; r += 64) acc = s_add(acc, s_mul(s_conj(V[r + i * ldv]), Bb(r, c)));
                acc = wave_sum(acc);
                const T wv = s_mul(ct, s_add(Ab(i, c), acc));
                for (i64 r = lane; r < pi; r += 64) Bb(r, c) = s_sub(Bb(r, c), s_mul(V[r + i * ldv], wv));
                if (lane == 0) Ab(i, c) = s_sub(Ab(i, c), wv);
            }
        }
        __syncthreads();
    }
    // ---- T: G = V^H V (strictly upper part), then column by column
    //      T(0:i, i) = -tau_i T(0:i, 0:i) G(0:i, i), T(i, i) = tau_i
    const i64 pmax = tp_rows(m, l, j0 + ib - 1);
    for (int e = w; e < ib * ib; e += NW) {
        const int a = e % ib, c = e / ib;
        if (a >= c) continue;
        T acc = s_zero(T());
        for (i64 r = lane; r < pmax; r += 64) acc = s_add(acc, s_mul(s_conj(V[r + a * ldv]), V[r + c * ldv]));
        acc = wave_sum(acc);
        if (lane == 0) s_G[a + c * TP_MAXIB] = acc;
    }
    __syncthreads();
    for (int i = 0; i < ib; ++i) {
        if (tid < i) {
            T acc = s_zero(T());
            for (int k = tid; k < i; ++k) acc = s_add(acc, s_mul(s_T[tid + k * TP_MAXIB], s_G[k + i * TP_MAXIB]));
            s_T[tid + i * TP_MAXIB] = s_sub(s_zero(T()), s_mul(s_tau[i], acc));
        } else if (tid == i) {
            s_T[i + i * TP_MAXIB] = s_tau[i];
        }
        __syncthreads();
    }
    for (int e = tid; e < ib * ib; e += TP_THREADS) {
        const int a = e % ib, c = e / ib;
        Tm[a + c * ldt] = a <= c ? s_T[a + c * TP_MAXIB] : s_zero(T());
    }
}

template <typename T>
void tpqrt_panel(i64 m, i64 l, i64 j0, int ib, T* A, i64 lda, T* B, i64 ldb, T* V, i64 ldv, T* tau, T* Tm,
                 i64 ldt, hipStream_t s) {
    if (ib <= 0) return;
    if (ib > TP_MAXIB) throw std::invalid_argument("tpqrt_panel: ib > 64");
    if (l < 0 || l > m) throw std::invalid_argument("tpqrt_panel: need 0 <= l <= m");
    hipLaunchKernelGGL(tpqrt_panel_kernel<T>, dim3(1), dim3(TP_THREADS), 0, s, m, l, j0, ib, A, lda, B, ldb, V,
                       ldv, tau, Tm, ldt);
    HIP_LAUNCH_CHECK();
}

#define INST(T) \
    template void tpqrt_panel<T>(i64, i64, i64, int, T*, i64, T*, i64, T*, i64, T*, T*, i64, hipStream_t);
INST(float) INST(double) INST(ccplx) INST(zcplx)
#undef INST

}  // namespace slate_hip
