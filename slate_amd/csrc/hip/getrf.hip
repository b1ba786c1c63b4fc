// LU panel factorization with partial pivoting on gfx950 -- the GPU panel
// SLATE does not have (its getrf panel always runs on the host,
// src/getrf.cc:95, src/internal/Tile_getrf.hh:160-447).
//
// Recursive (Toledo) on the panel columns so almost all flops are MFMA
// GEMMs / blocked TRSMs:
//     getrf(A) = getrf(A_left); laswp(A_right); trsm; gemm; getrf(A22); laswp(A_left)
//
// Base case (<= 32 columns): one launch per column over many workgroups
// and NO intra-kernel synchronisation (no fences, atomics or grid barriers;
// release/acquire fences cost microseconds each on gfx950):
//   launch j: every workgroup (a) reduces the per-workgroup arg-max
//   partials that launch j-1 left in a parity buffer -> pivot p of column
//   j-1 and the winning candidate row (also left there); (b) applies the
//   row interchange j-1 <-> p on the rows it owns (the old row j-1 was saved
//   by launch j-1, so no two workgroups read a row another one writes);
//   (c) eliminates column j-1 on its rows with the whole row segment held in
//   registers; (d) publishes its local arg-max of column j plus that row and
//   (owner of row j) the current row j.
// Kernel boundaries order the columns, so the panel is stream-ordered
// (graph-capturable, no host sync, no co-residency assumption).
#include "common.hpp"
#include "kernels.hpp"
#include "launchers.hpp"

namespace slate_hip {

namespace {
constexpr int NBB = 32;          // base-case width
constexpr int NTH = 256;         // threads per workgroup (one row each)
constexpr int MAXG = 512;        // max workgroups per base launch

template <typename T>
struct PanelBuf {                // one parity half of the device workspace
    double val[MAXG];
    i64 idx[MAXG];
    T cand[MAXG][NBB];
    T diag[NBB];
};
constexpr size_t PANEL_BYTES = 2 * sizeof(PanelBuf<zcplx>);
}  // namespace

template <typename T>
__global__ void __launch_bounds__(NTH)
getrf_base_step(i64 m, int c0, int c1, int j, T* A, i64 lda, i64* ipiv, i64 ioff, i64* info,
                i64 info_off, void* work, double thr, bool nopiv) {
    using R = typename scalar_traits<T>::real;
    __shared__ R sv[NTH];
    __shared__ i64 si[NTH];
    __shared__ int sg[NTH];
    __shared__ T prow[NBB];
    __shared__ T drow[NBB];
    PanelBuf<T>* pb = reinterpret_cast<PanelBuf<T>*>(work);
    const int G = gridDim.x, g = blockIdx.x, tid = threadIdx.x;
    const i64 rows_per = (m + G - 1) / G;
    const i64 r0 = (i64)g * rows_per, r1 = min(m, r0 + rows_per);
    const int w = c1 - c0;
    i64 p = -1;
    const int pc = j - 1;
    if (j > c0) {
        // ---- (a) pivot of column j-1 from launch j-1's partials
        PanelBuf<T>& in = pb[pc & 1];
        R best = R(-1); i64 bi = pc; int bg = -1;
        if (!nopiv)
            for (int q = tid; q < G; q += NTH) {
                R v = (R)in.val[q]; i64 ix = in.idx[q];
                if ((v != v && best == best) || v > best || (v == best && ix < bi)) { best = v; bi = ix; bg = q; }
            }
        sv[tid] = best; si[tid] = bi; sg[tid] = bg;
        if (tid < w) drow[tid] = in.diag[tid];
        __syncthreads();
        for (int o = NTH / 2; o > 0; o >>= 1) {
            if (tid < o) {
                R a = sv[tid], b = sv[tid + o];
                i64 ia = si[tid], ib = si[tid + o];
                bool take = (b != b && a == a) || b > a || (b == a && ib < ia);
                if (take) { sv[tid] = b; si[tid] = ib; sg[tid] = sg[tid + o]; }
            }
            __syncthreads();
        }
        p = si[0];
        int gw = sg[0];
        if (nopiv || gw < 0) { p = pc; }
        else if (thr < 1.0) {
            R dj = s_abs1(drow[pc - c0]);
            if (dj == dj && (double)dj >= thr * (double)sv[0]) p = pc;
        }
        if (tid < w) prow[tid] = (p == pc) ? drow[tid] : in.cand[gw][tid];
        __syncthreads();
        if (g == 0 && tid == 0) {
            if (ipiv) ipiv[pc] = p + ioff;
            if (s_is_zero(prow[pc - c0]) && info)
                atomicCAS(reinterpret_cast<unsigned long long*>(info), 0ull,
                          (unsigned long long)(pc + 1 + info_off));
        }
        // ---- (b) interchange: new row pc = pivot row (owner of pc writes it)
        if (pc >= r0 && pc < r1 && tid < w) A[pc + (i64)(c0 + tid) * lda] = prow[tid];
    }
    const bool last = j >= c1;
    PanelBuf<T>& out = pb[j & 1];
    R best = R(-1); i64 bi = j;
    const T u = (j > c0) ? prow[pc - c0] : s_zero(T());
    const bool uz = s_is_zero(u);
    for (i64 i = r0 + tid; i < r1; i += NTH) {
        if (j == c0) {   // first column of the block: arg-max only
            if (i >= j && !nopiv) {
                R v = s_abs1(A[i + (i64)j * lda]);
                if (v > best || (v != v && best == best)) { best = v; bi = i; }
            }
            continue;
        }
        if (i <= pc) continue;
        T a[NBB];
        const bool isp = (j > c0) && i == p && p != pc;
        if (isp) {
            #pragma unroll
            for (int c = 0; c < NBB; ++c) if (c < w) a[c] = drow[c];
        } else {
            #pragma unroll
            for (int c = 0; c < NBB; ++c) if (c < w && c0 + c >= pc) a[c] = A[i + (i64)(c0 + c) * lda];
        }
        {
            // ---- (c) eliminate column pc
            // (runtime-indexed reads of a[] would demote it to scratch: the
            // two scalars needed by position are re-read from cache/LDS)
            T l = isp ? drow[pc - c0] : A[i + (i64)pc * lda];
            if (!uz) l = s_div(l, u);
            #pragma unroll
            for (int c = 0; c < NBB; ++c) {
                if (c0 + c == pc) a[c] = l;
                if (c < w && c0 + c > pc) a[c] = s_sub(a[c], s_mul(l, prow[c]));
            }
            if (!last && !nopiv) {
                T aj = isp ? drow[j - c0] : A[i + (i64)j * lda];
                R v = s_abs1(s_sub(aj, s_mul(l, prow[j - c0])));
                if (v > best || (v != v && best == best)) { best = v; bi = i; }
            }
            if (isp) {
                #pragma unroll
                for (int c = 0; c < NBB; ++c) if (c < w) A[i + (i64)(c0 + c) * lda] = a[c];
            } else {
                #pragma unroll
                for (int c = 0; c < NBB; ++c) if (c < w && c0 + c >= pc) A[i + (i64)(c0 + c) * lda] = a[c];
            }
        }
    }
    if (last) return;
    // ---- (d) publish arg-max of column j, the candidate row, and row j
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    sv[tid] = best; si[tid] = bi;
    __syncthreads();
    for (int o = NTH / 2; o > 0; o >>= 1) {
        if (tid < o) {
            R a = sv[tid], b = sv[tid + o];
            i64 ia = si[tid], ib = si[tid + o];
            bool take = (b != b && a == a) || b > a || (b == a && ib < ia);
            if (take) { sv[tid] = b; si[tid] = ib; }
        }
        __syncthreads();
    }
    const i64 b = si[0];
    if (tid == 0) { out.val[g] = (double)sv[0]; out.idx[g] = b; }
    if (tid < w) {
        if (sv[0] >= R(0) || sv[0] != sv[0]) out.cand[g][tid] = A[b + (i64)(c0 + tid) * lda];
        if (j >= r0 && j < r1) out.diag[tid] = A[j + (i64)(c0 + tid) * lda];
    }
}

template <typename T>
static void base(i64 m, int c0, int c1, T* A, i64 lda, i64* ipiv, i64 ioff, i64* info, i64 info_off,
                 void* w, double thr, bool nopiv, hipStream_t s) {
    int G = (int)std::min<i64>(MAXG, std::max<i64>(1, (m + NTH - 1) / NTH));
    for (int j = c0; j <= c1; ++j)
        hipLaunchKernelGGL(getrf_base_step<T>, dim3(G), dim3(NTH), 0, s, m, c0, c1, j, A, lda, ipiv, ioff,
                           info, info_off, w, thr, nopiv);
    HIP_LAUNCH_CHECK();
}

template <typename T>
static void gemm_T(char ta, char tb, i64 m, i64 n, i64 k, double alpha, const T* A, i64 lda,
                   const T* B, i64 ldb, double beta, T* C, i64 ldc, hipStream_t s) {
    GemmCall c;
    c.transA = ta; c.transB = tb; c.m = m; c.n = n; c.k = k;
    c.alpha_re = alpha; c.beta_re = beta;
    c.A = A; c.lda = lda; c.B = B; c.ldb = ldb; c.C = C; c.ldc = ldc;
    if constexpr (scalar_traits<T>::is_complex) gemm_complex<T>(c, s);
    else gemm_real<T>(c, s);
}

// ipiv entries are written relative to the TOP of the outermost panel
// (ioff = row offset of this sub-panel); laswp at this level subtracts ioff.

template <typename T>
static void rec(i64 m, i64 n, T* A, i64 lda, i64* ipiv, i64 ioff, i64* info, i64 info_off, void* w,
                double thr, bool nopiv, hipStream_t s) {
    if (n <= NBB) {
        base<T>(m, 0, (int)n, A, lda, ipiv, ioff, info, info_off, w, thr, nopiv, s);
        return;
    }
    i64 n1 = ((n / 2 + NBB - 1) / NBB) * NBB;
    if (n1 >= n) n1 = n - NBB;
    rec<T>(m, n1, A, lda, ipiv, ioff, info, info_off, w, thr, nopiv, s);
    T* A12 = A + n1 * lda;
    if (!nopiv) laswp_off<T>(n - n1, A12, lda, 0, n1, ipiv, ioff, s);
    trsm<T>('L', 'L', 'N', 'U', n1, n - n1, s_from_real(T(), 1), A, lda, A12, lda, s);
    if (m > n1)
        gemm_T<T>('N', 'N', m - n1, n - n1, n1, -1.0, A + n1, lda, A12, lda, 1.0, A12 + n1, lda, s);
    if (m > n1) {
        rec<T>(m - n1, n - n1, A12 + n1, lda, ipiv ? ipiv + n1 : nullptr, ioff + n1, info, info_off + n1, w,
               thr, nopiv, s);
        if (!nopiv) laswp_off<T>(n1, A, lda, n1, std::min(m, n), ipiv, ioff, s);
    }
}

template <typename T>
void getrf_panel_ws(i64 m, i64 n, T* A, i64 lda, i64* ipiv, i64* info, double thr, bool nopiv,
                    void* work, hipStream_t s) {
    void* w = work;
    if (info) HIP_CHECK(hipMemsetAsync(info, 0, sizeof(i64), s));
    if (m <= 0 || n <= 0) return;
    const i64 k = std::min(m, n);
    rec<T>(m, k, A, lda, ipiv, 0, info, 0, w, thr, nopiv, s);
    if (n > k) {   // wide panel: U12 = L11^{-1} P A12
        if (!nopiv) laswp_off<T>(n - k, A + k * lda, lda, 0, k, ipiv, 0, s);
        trsm<T>('L', 'L', 'N', 'U', k, n - k, s_from_real(T(), 1), A, lda, A + k * lda, lda, s);
    }
}

size_t getrf_work_bytes() { return PANEL_BYTES; }

#define INST(T) \
    template void getrf_panel_ws<T>(i64, i64, T*, i64, i64*, i64*, double, bool, void*, hipStream_t);
INST(float) INST(double) INST(ccplx) INST(zcplx)
#undef INST

}  // namespace slate_hip
