// LU panel factorization with partial pivoting on gfx950 -- the GPU panel
// SLATE does not have (its getrf panel always runs on the host,
// src/getrf.cc:95, src/internal/Tile_getrf.hh:160-447).
//
// Recursive (Toledo) on the panel columns so almost all flops are MFMA
// GEMMs / blocked TRSMs:
//     getrf(A) = getrf(A_left); laswp(A_right); trsm; gemm; getrf(A22); laswp(A_left)
// Base case (<= 32 columns) is one launch per column over many workgroups:
// each workgroup eliminates the previous column on its rows (rank-1 update
// of the base block), takes a local arg-max of the new column, publishes
// it with an agent-scope release + atomic ticket; the LAST arriving
// workgroup (acquire) picks the global pivot (NaN wins, lowest index on
// ties, optional threshold pivoting), records ipiv/info and swaps the two
// rows inside the base block.  Kernel boundaries order the columns, so no
// grid barrier / co-residency assumption is needed and the whole thing is
// stream-ordered (graph-capturable, no host sync).
#include "common.hpp"
#include "kernels.hpp"
#include "launchers.hpp"

namespace slate_hip {

namespace {
constexpr int NBB = 32;          // base-case width
constexpr int WG_ROWS = 512;     // target rows per workgroup
constexpr int MAXG = 512;        // max workgroups per base launch

struct PanelWork {               // device workspace layout
    unsigned int counter;
    unsigned int pad;
    double val[MAXG];
    i64 idx[MAXG];
};
}  // namespace

template <typename T>
__global__ void __launch_bounds__(256)
getrf_base_step(i64 m, int c0, int c1, int j, T* A, i64 lda, i64* ipiv, i64 ioff, i64* info,
                i64 info_off, PanelWork* w, double thr, bool nopiv) {
    using R = typename scalar_traits<T>::real;
    __shared__ R sv[256];
    __shared__ i64 si[256];
    __shared__ T prow[NBB];
    __shared__ int s_last;
    const int G = gridDim.x;
    const i64 rows_per = (m + G - 1) / G;
    const i64 r0 = (i64)blockIdx.x * rows_per, r1 = min(m, r0 + rows_per);
    // ---- eliminate column j-1 (its pivot row j-1 already swapped in place)
    if (j > c0) {
        const int pc = j - 1;
        if (threadIdx.x < c1 - pc) prow[threadIdx.x] = A[pc + (i64)(pc + threadIdx.x) * lda];
        __syncthreads();
        const T u = prow[0];
        const bool uz = s_is_zero(u);
        for (i64 i = r0 + threadIdx.x; i < r1; i += 256) {
            if (i <= pc) continue;
            T l = A[i + (i64)pc * lda];
            if (!uz) { l = s_div(l, u); A[i + (i64)pc * lda] = l; }
            for (int c = j; c < c1; ++c) A[i + (i64)c * lda] = s_sub(A[i + (i64)c * lda], s_mul(l, prow[c - pc]));
        }
        // every wave drains its stores before the workgroup's release below,
        // and the arg-max pass (different row->thread map) sees them
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }
    if (j >= c1) return;   // final launch: elimination only
    // ---- local arg-max of column j over rows >= j
    R best = R(-1);
    i64 bi = j;
    if (!nopiv) {
        for (i64 i = max(r0, (i64)j) + threadIdx.x; i < r1; i += 256) {
            R v = s_abs1(A[i + (i64)j * lda]);
            if (v > best || (v != v && best == best)) { best = v; bi = i; }
        }
    }
    sv[threadIdx.x] = best; si[threadIdx.x] = bi;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if (threadIdx.x < o) {
            R a = sv[threadIdx.x], b = sv[threadIdx.x + o];
            i64 ia = si[threadIdx.x], ib = si[threadIdx.x + o];
            bool take = (b != b && a == a) || b > a || (b == a && ib < ia);
            if (take) { sv[threadIdx.x] = b; si[threadIdx.x] = ib; }
        }
        __syncthreads();
    }
    // (the reduction's barriers above ordered every wave's drained stores)
    if (threadIdx.x == 0) {
        w->val[blockIdx.x] = (double)sv[0];
        w->idx[blockIdx.x] = si[0];
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        unsigned old = __hip_atomic_fetch_add(&w->counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_last = (old == (unsigned)G - 1);
    }
    __syncthreads();
    if (!s_last) return;
    // ---- last arriver: global pivot, record, swap rows inside the base block
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        double bv = -1; i64 bidx = j;
        if (!nopiv) {
            for (int g = 0; g < G; ++g) {
                double v = __hip_atomic_load(&w->val[g], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                i64 ix = __hip_atomic_load(&w->idx[g], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if ((v != v && bv == bv) || v > bv || (v == bv && ix < bidx)) { bv = v; bidx = ix; }
            }
            if (thr < 1.0) {
                double dj = (double)s_abs1(A[j + (i64)j * lda]);
                if (dj >= thr * bv && dj == dj) bidx = j;
            }
        }
        si[0] = bidx;
        if (ipiv) ipiv[j] = bidx + ioff;
        T pv = A[bidx + (i64)j * lda];
        if (s_is_zero(pv) && info) {
            unsigned long long* ip = reinterpret_cast<unsigned long long*>(info);
            atomicCAS(ip, 0ull, (unsigned long long)(j + 1 + info_off));
        }
        w->counter = 0;
    }
    __syncthreads();
    const i64 p = si[0];
    if (p != j) {
        for (int c = c0 + threadIdx.x; c < c1; c += 256) {
            T a = A[j + (i64)c * lda], b = A[p + (i64)c * lda];
            A[j + (i64)c * lda] = b; A[p + (i64)c * lda] = a;
        }
    }
}

template <typename T>
__global__ void ipiv_add_kernel(i64 n, i64* ipiv, i64 d) {
    i64 i = (i64)blockIdx.x * 256 + threadIdx.x;
    if (i < n) ipiv[i] += d;
}

template <typename T>
static void base(i64 m, int c0, int c1, T* A, i64 lda, i64* ipiv, i64 ioff, i64* info, i64 info_off,
                 PanelWork* w, double thr, bool nopiv, hipStream_t s) {
    int G = (int)std::min<i64>(MAXG, std::max<i64>(1, (m + WG_ROWS - 1) / WG_ROWS));
    for (int j = c0; j <= c1; ++j)
        hipLaunchKernelGGL(getrf_base_step<T>, dim3(G), dim3(256), 0, s, m, c0, c1, j, A, lda, ipiv, ioff,
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
static void rec(i64 m, i64 n, T* A, i64 lda, i64* ipiv, i64 ioff, i64* info, i64 info_off, PanelWork* w,
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
    PanelWork* w = reinterpret_cast<PanelWork*>(work);
    HIP_CHECK(hipMemsetAsync(&w->counter, 0, sizeof(unsigned), s));
    if (info) HIP_CHECK(hipMemsetAsync(info, 0, sizeof(i64), s));
    if (m <= 0 || n <= 0) return;
    const i64 k = std::min(m, n);
    rec<T>(m, k, A, lda, ipiv, 0, info, 0, w, thr, nopiv, s);
    if (n > k) {   // wide panel: U12 = L11^{-1} P A12
        if (!nopiv) laswp_off<T>(n - k, A + k * lda, lda, 0, k, ipiv, 0, s);
        trsm<T>('L', 'L', 'N', 'U', k, n - k, s_from_real(T(), 1), A, lda, A + k * lda, lda, s);
    }
}

size_t getrf_work_bytes() { return sizeof(PanelWork); }

#define INST(T) \
    template void getrf_panel_ws<T>(i64, i64, T*, i64, i64*, i64*, double, bool, void*, hipStream_t);
INST(float) INST(double) INST(ccplx) INST(zcplx)
#undef INST

}  // namespace slate_hip
