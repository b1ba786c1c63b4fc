// Element-wise / data-movement kernels for gfx950 (SURVEY §2.5:
// device_geset/tzset, gescale/tzscale, geadd/tzadd, gecopy/tzcopy with
// precision conversion, transpose, gescale_row_col) and the row-permutation
// kernel used by LU (replacing internal_swap.cc's per-row swaps).
//
// All operate on one strided column-major block (the rank's whole local
// buffer or any sub-block of it), so a matrix-wide op is ONE launch; grids
// are (rows/256) x (columns, grid-strided) with coalesced row access.
#include "common.hpp"
#include "kernels.hpp"
#include "workspace.hpp"

namespace slate_hip {

namespace {
inline dim3 grid2(i64 m, i64 n) {
    i64 gx = (m + 255) / 256;
    i64 gy = std::min<i64>(n, 4096);
    return dim3((unsigned)std::max<i64>(gx, 1), (unsigned)std::max<i64>(gy, 1));
}
__device__ inline bool in_uplo(char uplo, i64 i, i64 j) {
    // 'L' lower, 'U' upper (both incl. the diagonal), 'D' diagonal only, else all
    return uplo == 'L' ? i >= j : (uplo == 'U' ? i <= j : (uplo == 'D' ? i == j : true));
}
}  // namespace

template <typename T>
__global__ void geset_kernel(char uplo, i64 m, i64 n, T off, T diag, T* A, i64 lda) {
    i64 i = (i64)blockIdx.x * 256 + threadIdx.x;
    if (i >= m) return;
    for (i64 j = blockIdx.y; j < n; j += gridDim.y)
        if (in_uplo(uplo, i, j)) A[i + j * lda] = (i == j) ? diag : off;
}

template <typename T>
__global__ void gescale_kernel(char uplo, i64 m, i64 n, T alpha, T* A, i64 lda) {
    i64 i = (i64)blockIdx.x * 256 + threadIdx.x;
    if (i >= m) return;
    for (i64 j = blockIdx.y; j < n; j += gridDim.y)
        if (in_uplo(uplo, i, j)) A[i + j * lda] = s_mul(alpha, A[i + j * lda]);
}

template <typename T>
__global__ void geadd_kernel(char uplo, i64 m, i64 n, T alpha, const T* A, i64 lda, T beta, T* B, i64 ldb) {
    i64 i = (i64)blockIdx.x * 256 + threadIdx.x;
    if (i >= m) return;
    const bool b0 = s_is_zero(beta);
    for (i64 j = blockIdx.y; j < n; j += gridDim.y)
        if (in_uplo(uplo, i, j)) {
            T v = s_mul(alpha, A[i + j * lda]);
            if (!b0) v = s_add(v, s_mul(beta, B[i + j * ldb]));
            B[i + j * ldb] = v;
        }
}

template <typename Ts, typename Td>
__device__ inline Td convert(Ts v) {
    if constexpr (scalar_traits<Ts>::is_complex && scalar_traits<Td>::is_complex) {
        Td r; r.re = (typename scalar_traits<Td>::real)v.re; r.im = (typename scalar_traits<Td>::real)v.im; return r;
    } else if constexpr (scalar_traits<Td>::is_complex) {
        Td r; r.re = (typename scalar_traits<Td>::real)v; r.im = 0; return r;
    } else if constexpr (scalar_traits<Ts>::is_complex) {
        return (Td)v.re;
    } else {
        return (Td)v;
    }
}

// B (m x n) = op(A) with precision conversion; uplo masks the destination.
template <typename Ts, typename Td>
__global__ void gecopy_kernel(char uplo, i64 m, i64 n, const Ts* A, i64 lda, Td* B, i64 ldb) {
    i64 i = (i64)blockIdx.x * 256 + threadIdx.x;
    if (i >= m) return;
    for (i64 j = blockIdx.y; j < n; j += gridDim.y)
        if (in_uplo(uplo, i, j)) B[i + j * ldb] = convert<Ts, Td>(A[i + j * lda]);
}

// Transposed copy through a 32x33 LDS tile: B (m x n) = op(A), A is n x m.
template <typename Ts, typename Td, bool CONJ>
__global__ void transpose_kernel(char uplo, i64 m, i64 n, const Ts* A, i64 lda, Td* B, i64 ldb) {
    __shared__ Td tile[32][33];
    const i64 bi = (i64)blockIdx.x * 32, bj = (i64)blockIdx.y * 32;   // block of B
    const int tx = threadIdx.x, ty = threadIdx.y;   // 32 x 8
    // read A block (rows bj.., cols bi..) coalesced along A's rows
    for (int r = ty; r < 32; r += 8) {
        i64 ar = bj + tx, ac = bi + r;   // A(ar, ac) -> B(ac, ar)
        if (ar < n && ac < m) {
            Td v = convert<Ts, Td>(A[ar + ac * lda]);
            if constexpr (CONJ) v = s_conj(v);
            tile[r][tx] = v;
        }
    }
    __syncthreads();
    for (int c = ty; c < 32; c += 8) {
        i64 brow = bi + tx, bcol = bj + c;
        if (brow < m && bcol < n && in_uplo(uplo, brow, bcol)) B[brow + bcol * ldb] = tile[tx][c];
    }
}

template <typename T, typename R>
__global__ void scale_row_col_kernel(char equed, i64 m, i64 n, const R* r, const R* c, T* A, i64 lda) {
    i64 i = (i64)blockIdx.x * 256 + threadIdx.x;
    if (i >= m) return;
    for (i64 j = blockIdx.y; j < n; j += gridDim.y) {
        R s = R(1);
        if (equed == 'S') {            // sign: a / |a|, 1 where a = 0 (condest's sign vector)
            const T a = A[i + j * lda];
            const R m = s_abs(a);
            A[i + j * lda] = m > R(0) ? s_mul(s_from_real(T(), R(1) / m), a) : s_from_real(T(), R(1));
            continue;
        }
        if (equed == 'R' || equed == 'B') s *= r[i];
        if (equed == 'C' || equed == 'B') s *= c[j];
        A[i + j * lda] = s_mul(s_from_real(T(), s), A[i + j * lda]);
    }
}

// ---------------------------------------------------------------------------
// Recursive random butterfly transform (RBT, src/internal/internal_gerbt.cc
// in the reference): D levels of block-diagonal butterflies
// [R0 R1; R0 -R1] / sqrt 2 applied along one dimension (rows or columns) of
// a local block.  The 2^D elements b + k nidx / 2^D (k < 2^D) are closed
// under every level, so one thread loads them once, applies all D levels
// in registers and stores once (one HBM pass instead of D).  On a process
// grid the padded size makes every butterfly partner local (see
// models/mixed.py), so the same kernel runs on each rank's local rows.
template <typename T, typename R, int D>
__global__ void __launch_bounds__(256)
butterfly_kernel(bool trans, bool rows, i64 nidx, i64 nother, T* __restrict__ A, i64 lda,
                 const R* __restrict__ diag, i64 ldd) {
    constexpr int K = 1 << D;
    const i64 quarter = nidx >> D;
    const i64 b = (i64)blockIdx.x * 256 + threadIdx.x;
    if (b >= quarter) return;
    const R sq = R(0.70710678118654752440);
    R dg[D][K];
    #pragma unroll
    for (int l = 0; l < D; ++l)
        #pragma unroll
        for (int k = 0; k < K; ++k) dg[l][k] = diag[l * ldd + b + k * quarter];
    for (i64 j = blockIdx.y; j < nother; j += gridDim.y) {
        T v[K];
        #pragma unroll
        for (int k = 0; k < K; ++k) {
            const i64 idx = b + k * quarter;
            v[k] = rows ? A[idx + j * lda] : A[j + idx * lda];
        }
        #pragma unroll
        for (int s = 0; s < D; ++s) {
            const int l = trans ? D - 1 - s : s;
            const int half = 1 << (D - 1 - l);
            #pragma unroll
            for (int k = 0; k < K; ++k) {
                if ((k & half) != 0) continue;          // k is the top of pair (k, k + half)
                const T a = v[k], c = v[k + half];
                const R ra = dg[l][k], rc = dg[l][k + half];
                if (!trans) {
                    const T x = s_mul(s_from_real(T(), ra * sq), a), y = s_mul(s_from_real(T(), rc * sq), c);
                    v[k] = s_add(x, y);
                    v[k + half] = s_sub(x, y);
                } else {
                    v[k] = s_mul(s_from_real(T(), ra * sq), s_add(a, c));
                    v[k + half] = s_mul(s_from_real(T(), rc * sq), s_sub(a, c));
                }
            }
        }
        #pragma unroll
        for (int k = 0; k < K; ++k) {
            const i64 idx = b + k * quarter;
            if (rows) A[idx + j * lda] = v[k];
            else A[j + idx * lda] = v[k];
        }
    }
}

// ---------------------------------------------------------------------------
// Row interchanges.  The LAPACK-style swap sequence ipiv[k1..k2) (0-based
// rows, ipiv[k] >= k) is first folded into a permutation of the touched rows
// (open-addressing hash map in LDS, built by one thread: O(#swaps)), then
// every workgroup moves a 32-column chunk: gather touched rows into LDS,
// barrier, scatter to their new positions.  One launch for any n.
namespace {
constexpr int HSIZE = 2048;      // hash slots (>= 2 x max swaps per call)
constexpr int MAXSW = 512;       // max swaps per call (more: split into calls)
}

__global__ void zero_words_kernel(unsigned long long* p, long long n) {
    const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
    if (i < n) p[i] = 0ull;
}

// Link-time stand-in for the loopback transport (parallel/comm.py): one
// wave holds the issuing stream for `ticks` of the constant wall clock, as
// a collective of that duration would; time-bound, so every wave exits.
__global__ void spin_ticks_kernel(unsigned long long ticks) {
    const unsigned long long t0 = wall_clock64();
    while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
}

void spin_ns(double ns, hipStream_t s) {
    static const double rate_khz = [] {
        int dev = 0, khz = 0;
        if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess ||
            khz <= 0)
            khz = 100000;
        return (double)khz;
    }();
    if (!(ns > 0)) return;
    const double capped = ns < 2e9 ? ns : 2e9;      // at most 2 s per call
    hipLaunchKernelGGL(spin_ticks_kernel, dim3(1), dim3(64), 0, s, (unsigned long long)(capped * rate_khz * 1e-6));
    HIP_LAUNCH_CHECK();
}

struct SwapPlan {                // folded permutation of one swap sequence
    int nt;
    int pad;
    i64 trow[2 * MAXSW];         // touched rows
    i64 tsrc[2 * MAXSW];         // original row now found at trow[t]
};

// Fold the swap sequence into the permutation ONCE, in parallel: swap k
// exchanges rows k and p_k >= k and no later swap touches row k, so the row
// finally at position k came from p_k "just before swap k", i.e. (walking the
// swaps backwards) from the chain k'' = last earlier swap with p_k'' == row.
// One thread per swap follows its chain over the sequence held in LDS; rows
// >= k2 are emitted by the LAST swap targeting them.  (The former
// single-thread hash-map fold cost 46-256 us per call.)
__global__ void __launch_bounds__(MAXSW)
laswp_setup_kernel(i64 k1, i64 k2, const i64* __restrict__ ipiv, i64 ioff, int incx, SwapPlan* plan,
                   bool fixed_slots) {
    __shared__ int pv[MAXSW];                // relative pivot rows (relative to k1)
    __shared__ int prv[MAXSW];               // prv[t]: last swap t' < t that targets row t (-1: none)
    __shared__ int s_cnt;
    const int ns = (int)(k2 - k1), q = threadIdx.x;
    if (q == 0) s_cnt = ns;
    if (q < ns) {
        pv[q] = (int)(ipiv[k1 + q] - ioff - k1);
        prv[q] = -1;
    }
    // incx < 0 applies the swaps in reverse order = the inverse permutation:
    // same fold, source and destination exchanged
    i64* dst = incx > 0 ? plan->trow : plan->tsrc;
    i64* srcv = incx > 0 ? plan->tsrc : plan->trow;
    __syncthreads();
    // every swap t' targets pv[t'] >= t', so the swaps targeting row t < ns all
    // come before swap t: the last of them is a max
    if (q < ns && pv[q] != q && pv[q] < ns) atomicMax(&prv[pv[q]], q);
    // swaps grouped by target row: one bitonic sort of (row, swap) keys in
    // LDS gives every swap its previous / next swap on the same row in O(1)
    // (the per-thread O(ns) backward / forward scans of the sequence cost
    // ~100 us per 512-swap plan on the LU panel critical path)
    __shared__ unsigned long long key[MAXSW];
    __shared__ int prev_same[MAXSW];
    __shared__ unsigned char is_last[MAXSW];
    key[q] = q < ns ? (((unsigned long long)(unsigned)pv[q] << 16) | (unsigned)q) : ~0ull;
    __syncthreads();
    for (int kk2 = 2; kk2 <= MAXSW; kk2 <<= 1)
        for (int jj = kk2 >> 1; jj > 0; jj >>= 1) {
            const int ixj = q ^ jj;
            if (ixj > q) {
                const bool up = (q & kk2) == 0;
                const unsigned long long a = key[q], b = key[ixj];
                if ((a > b) == up) { key[q] = b; key[ixj] = a; }
            }
            __syncthreads();
        }
    if (q < ns) {
        const unsigned long long me = key[q];
        const int x = (int)(me & 0xffff);
        const unsigned long long row = me >> 16;
        prev_same[x] = (q > 0 && (key[q - 1] >> 16) == row) ? (int)(key[q - 1] & 0xffff) : -1;
        is_last[x] = !(q + 1 < ns && (key[q + 1] >> 16) == row);
    }
    __syncthreads();
    // content of row t just before swap t: what the last earlier swap
    // targeting row t put there, i.e. row prv[t]'s content just before swap
    // prv[t] -- follow the pointers (O(1) per hop)
    auto chain = [&](int t) -> int {
        while (prv[t] >= 0) t = prv[t];
        return t;
    };
    if (q < ns) {
        // position q: content of row pv[q] just before swap q
        int r = pv[q], src;
        if (r == q) {
            src = chain(q);
        } else {
            const int kk = prev_same[q];               // last earlier swap targeting row r
            src = (kk < 0) ? r : chain(kk);
        }
        dst[q] = k1 + q;
        srcv[q] = k1 + src;
        // rows beyond the sequence: emitted by the last swap that targets them
        const bool emit = r >= ns && is_last[q];
        // fixed_slots: the emitting swap's own slot ns + q (-1 when it emits
        // nothing), so every rank that folds the same sequence numbers the
        // rows identically (the distributed exchange sums slot-wise);
        // otherwise compacted in arrival order (local laswp)
        if (emit) {
            const int slot = fixed_slots ? ns + q : atomicAdd(&s_cnt, 1);
            dst[slot] = k1 + r;
            srcv[slot] = k1 + chain(q);
        } else if (fixed_slots) {
            dst[ns + q] = -1;
            srcv[ns + q] = -1;
        }
    }
    __syncthreads();
    if (q == 0) plan->nt = fixed_slots ? 2 * ns : s_cnt;
}

template <typename T>
__global__ void __launch_bounds__(256)
laswp_apply_kernel(i64 n, T* A, i64 lda, const SwapPlan* __restrict__ plan, int CCH) {
    extern __shared__ __align__(16) unsigned char dyn[];
    T* buf = reinterpret_cast<T*>(dyn);   // [nt][CCH + 1] gathered rows
    const int nt = plan->nt;
    if (nt == 0) return;
    const i64 c0 = (i64)blockIdx.x * CCH;
    const int ncols = (int)min((i64)CCH, n - c0);
    // odd row pitch (in doubles): t-consecutive lanes then step an odd
    // number of 2-bank words, i.e. hit distinct banks.  (CCH + 1 was even
    // for the 7-column chunks of 512-swap plans: a 16-way conflict, 87 % of
    // LDS cycles in the round-2 PMC of laswp_apply_kernel.)
    const int LD = CCH | 1;
    // gather: buf[t][c] = A[tsrc[t], c0 + c]   (t fastest: the touched rows
    // of one column; the row lists are read from L2, not rebuilt)
    for (int idx = threadIdx.x; idx < nt * CCH; idx += blockDim.x) {
        int t = idx % nt, c = idx / nt;
        if (c < ncols) buf[t * LD + c] = A[plan->tsrc[t] + (c0 + c) * lda];
    }
    __syncthreads();
    for (int idx = threadIdx.x; idx < nt * CCH; idx += blockDim.x) {
        int t = idx % nt, c = idx / nt;
        if (c < ncols) A[plan->trow[t] + (c0 + c) * lda] = buf[t * LD + c];
    }
}

// The same folded plan applied to COLUMNS: the row interchanges of a matrix
// held transposed (RowMajor rows = contiguous columns here, the storage the
// LU trailing update uses -- SLATE switches its GPU tiles to RowMajor for the
// same reason, src/getrf.cc:51-55).  Every workgroup owns a 128-byte row
// segment of every touched column: gather all of them into LDS, barrier,
// write them to their new columns -- whole cache lines both ways, no strided
// 8-byte accesses.
template <typename T>
__global__ void __launch_bounds__(256)
laswp_cols_kernel(i64 nrows, T* A, i64 lda, const SwapPlan* __restrict__ plan) {
    constexpr int R = 128 / sizeof(T);                    // rows per workgroup: one cache line
    constexpr int PER = 2 * MAXSW * R / 256;              // elements per thread (128 VGPRs)
    __shared__ int src_s[2 * MAXSW], dst_s[2 * MAXSW];
    const int nt = plan->nt;
    if (nt == 0) return;
    for (int t = threadIdx.x; t < nt; t += 256) {
        src_s[t] = (int)plan->tsrc[t];
        dst_s[t] = (int)plan->trow[t];
    }
    __syncthreads();
    const i64 r0 = (i64)blockIdx.x * R;
    const int nr = (int)min((i64)R, nrows - r0), tot = nt * R;
    // every load of this workgroup in flight at once (registers, no LDS
    // round trip), then -- after ALL of them have landed -- every store
    T v[PER];
    #pragma unroll
    for (int k = 0; k < PER; ++k) {
        const int idx = threadIdx.x + k * 256, t = idx / R, r = idx % R;
        if (idx < tot && r < nr && src_s[t] >= 0) v[k] = A[r0 + r + (i64)src_s[t] * lda];
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    #pragma unroll
    for (int k = 0; k < PER; ++k) {
        const int idx = threadIdx.x + k * 256, t = idx / R, r = idx % R;
        if (idx < tot && r < nr && src_s[t] >= 0) A[r0 + r + (i64)dst_s[t] * lda] = v[k];
    }
}

template <typename T>
__global__ void row_gather_kernel(i64 m, i64 n, const T* A, i64 lda, T* B, i64 ldb, const i64* perm) {
    i64 i = (i64)blockIdx.x * 256 + threadIdx.x;
    if (i >= m) return;
    const i64 src = perm[i];
    for (i64 j = blockIdx.y; j < n; j += gridDim.y) B[i + j * ldb] = A[src + j * lda];
}

template <typename T>
__global__ void row_scatter_kernel(i64 m, i64 n, const T* A, i64 lda, T* B, i64 ldb, const i64* perm) {
    i64 i = (i64)blockIdx.x * 256 + threadIdx.x;
    if (i >= m) return;
    const i64 dst = perm[i];
    for (i64 j = blockIdx.y; j < n; j += gridDim.y) B[dst + j * ldb] = A[i + j * lda];
}

// ---------------------------------------------------------------------------
template <typename T> void geset(char uplo, i64 m, i64 n, T off, T diag, T* A, i64 lda, hipStream_t s) {
    if (m <= 0 || n <= 0) return;
    hipLaunchKernelGGL(geset_kernel<T>, grid2(m, n), dim3(256), 0, s, uplo, m, n, off, diag, A, lda);
    HIP_LAUNCH_CHECK();
}
template <typename T> void gescale(char uplo, i64 m, i64 n, T alpha, T* A, i64 lda, hipStream_t s) {
    if (m <= 0 || n <= 0) return;
    hipLaunchKernelGGL(gescale_kernel<T>, grid2(m, n), dim3(256), 0, s, uplo, m, n, alpha, A, lda);
    HIP_LAUNCH_CHECK();
}
template <typename T>
void geadd(char uplo, i64 m, i64 n, T alpha, const T* A, i64 lda, T beta, T* B, i64 ldb, hipStream_t s) {
    if (m <= 0 || n <= 0) return;
    hipLaunchKernelGGL(geadd_kernel<T>, grid2(m, n), dim3(256), 0, s, uplo, m, n, alpha, A, lda, beta, B, ldb);
    HIP_LAUNCH_CHECK();
}
template <typename Ts, typename Td>
void gecopy(char uplo, char trans, i64 m, i64 n, const Ts* A, i64 lda, Td* B, i64 ldb, hipStream_t s) {
    if (m <= 0 || n <= 0) return;
    if (trans == 'N') {
        hipLaunchKernelGGL((gecopy_kernel<Ts, Td>), grid2(m, n), dim3(256), 0, s, uplo, m, n, A, lda, B, ldb);
    } else {
        dim3 grid((unsigned)((m + 31) / 32), (unsigned)((n + 31) / 32));
        if (trans == 'C')
            hipLaunchKernelGGL((transpose_kernel<Ts, Td, true>), grid, dim3(32, 8), 0, s, uplo, m, n, A, lda, B, ldb);
        else
            hipLaunchKernelGGL((transpose_kernel<Ts, Td, false>), grid, dim3(32, 8), 0, s, uplo, m, n, A, lda, B, ldb);
    }
    HIP_LAUNCH_CHECK();
}
template <typename T, typename R>
void gescale_row_col(char equed, i64 m, i64 n, const R* r, const R* c, T* A, i64 lda, hipStream_t s) {
    if (m <= 0 || n <= 0) return;
    hipLaunchKernelGGL((scale_row_col_kernel<T, R>), grid2(m, n), dim3(256), 0, s, equed, m, n, r, c, A, lda);
    HIP_LAUNCH_CHECK();
}
template <typename T, typename R>
void butterfly(bool trans, bool rows, int depth, i64 nidx, i64 nother, T* A, i64 lda, const R* diag, i64 ldd,
               hipStream_t s) {
    if (nidx <= 0 || nother <= 0 || depth <= 0) return;
    if (depth > 4 || nidx % (1 << depth)) throw std::invalid_argument("butterfly: depth <= 4, n % 2^depth == 0");
    const i64 quarter = nidx >> depth;
    dim3 g((unsigned)((quarter + 255) / 256), (unsigned)std::min<i64>(nother, 1024));
    switch (depth) {
        case 1: hipLaunchKernelGGL((butterfly_kernel<T, R, 1>), g, dim3(256), 0, s, trans, rows, nidx, nother, A, lda, diag, ldd); break;
        case 2: hipLaunchKernelGGL((butterfly_kernel<T, R, 2>), g, dim3(256), 0, s, trans, rows, nidx, nother, A, lda, diag, ldd); break;
        case 3: hipLaunchKernelGGL((butterfly_kernel<T, R, 3>), g, dim3(256), 0, s, trans, rows, nidx, nother, A, lda, diag, ldd); break;
        default: hipLaunchKernelGGL((butterfly_kernel<T, R, 4>), g, dim3(256), 0, s, trans, rows, nidx, nother, A, lda, diag, ldd); break;
    }
    HIP_LAUNCH_CHECK();
}
template <typename T>
void laswp_off(i64 n, T* A, i64 lda, i64 k1, i64 k2, const i64* ipiv, i64 ioff, hipStream_t s, int incx) {
    if (n <= 0 || k2 <= k1) return;
    if (k2 - k1 > MAXSW) {
        if (incx > 0)
            for (i64 k = k1; k < k2; k += MAXSW) laswp_off<T>(n, A, lda, k, std::min(k2, k + MAXSW), ipiv, ioff, s, incx);
        else
            for (i64 k = k2; k > k1; k -= MAXSW) laswp_off<T>(n, A, lda, std::max(k1, k - MAXSW), k, ipiv, ioff, s, incx);
        return;
    }
    SwapPlan* plan = static_cast<SwapPlan*>(workspace(s, sizeof(SwapPlan), WS_L));
    hipLaunchKernelGGL(laswp_setup_kernel, dim3(1), dim3(MAXSW), 0, s, k1, k2, ipiv, ioff, incx, plan, false);
    const size_t per_col = (size_t)2 * (k2 - k1) * sizeof(T);
    int cch = (int)std::max<size_t>(1, std::min<size_t>(32, (64 * 1024) / per_col - 1));
    size_t shmem = per_col * (cch + 1);
    unsigned g = (unsigned)((n + cch - 1) / cch);
    hipLaunchKernelGGL(laswp_apply_kernel<T>, dim3(g), dim3(256), shmem, s, n, A, lda, plan, cch);
    HIP_LAUNCH_CHECK();
}
template <typename T>
void laswp(i64 n, T* A, i64 lda, i64 k1, i64 k2, const i64* ipiv, int incx, hipStream_t s) {
    laswp_off<T>(n, A, lda, k1, k2, ipiv, 0, s, incx);
}
// column interchanges col k <-> col ipiv[k] - ioff (k in [k1, k2)) over rows
// [0, nrows): laswp of the transposed matrix
template <typename T>
void laswp_cols(i64 nrows, T* A, i64 lda, i64 k1, i64 k2, const i64* ipiv, i64 ioff, hipStream_t s, int incx) {
    if (nrows <= 0 || k2 <= k1) return;
    if (k2 - k1 > MAXSW) {
        if (incx > 0)
            for (i64 k = k1; k < k2; k += MAXSW) laswp_cols<T>(nrows, A, lda, k, std::min(k2, k + MAXSW), ipiv, ioff, s, incx);
        else
            for (i64 k = k2; k > k1; k -= MAXSW) laswp_cols<T>(nrows, A, lda, std::max(k1, k - MAXSW), k, ipiv, ioff, s, incx);
        return;
    }
    SwapPlan* plan = static_cast<SwapPlan*>(workspace(s, sizeof(SwapPlan), WS_L));
    hipLaunchKernelGGL(laswp_setup_kernel, dim3(1), dim3(MAXSW), 0, s, k1, k2, ipiv, ioff, incx, plan, false);
    constexpr int R = 128 / sizeof(T);
    const unsigned g = (unsigned)((nrows + R - 1) / R);
    hipLaunchKernelGGL(laswp_cols_kernel<T>, dim3(g), dim3(256), 0, s, nrows, A, lda, plan);
    HIP_LAUNCH_CHECK();
}

// the same with a plan folded once per panel (swap_plan, fixed slots: -1
// entries are skipped), for several column ranges of one step
template <typename T>
void laswp_cols_plan(i64 nrows, T* A, i64 lda, const void* plan, hipStream_t s) {
    if (nrows <= 0) return;
    constexpr int R = 128 / sizeof(T);
    const unsigned g = (unsigned)((nrows + R - 1) / R);
    hipLaunchKernelGGL(laswp_cols_kernel<T>, dim3(g), dim3(256), 0, s, nrows, A, lda,
                       static_cast<const SwapPlan*>(plan));
    HIP_LAUNCH_CHECK();
}

// ---------------------------------------------------------------------------
// Distributed row interchange for LU on p > 1 process rows (no host round
// trip).  The panel's swap sequence is folded ONCE into a device-resident
// plan (SwapPlan layout with FIXED slots: window row q in slot q, the row a
// swap q moves below the window in slot ns + q, -1 when none -- identical on
// every rank, which the slot-wise all-reduce below relies on); every rank of
// a process column then
//   xchg_gather : packs the touched rows it OWNS (block-cyclic row owner)
//                 into X (S x ncols, S = 2 kb slots), zeros elsewhere,
//   <all-reduce of X over the column communicator: x + 0 is exact>,
//   xchg_scatter: writes the rows it owns at their new positions.
// The window slots [0, kb) of the reduced X are the new tile row k on every
// rank of the column (the U row the trailing update needs anyway).
void swap_plan(i64 k1, i64 k2, const i64* ipiv, i64 ioff, int incx, void* plan, hipStream_t s) {
    if (k2 - k1 > MAXSW) throw std::invalid_argument("swap_plan: at most 512 swaps per plan");
    zero_words(plan, (long long)(sizeof(SwapPlan) / 8), s);
    if (k2 <= k1) return;
    hipLaunchKernelGGL(laswp_setup_kernel, dim3(1), dim3(MAXSW), 0, s, k1, k2, ipiv, ioff, incx,
                       static_cast<SwapPlan*>(plan), true);
    HIP_LAUNCH_CHECK();
}
size_t swap_plan_bytes() { return sizeof(SwapPlan); }

__device__ inline i64 bc_local_row(i64 g, i64 nb, int p, int pr) {
    // local row of global row g on process row pr, -1 if another row owns it
    const i64 tile = g / nb;
    return (int)(tile % p) == pr ? (tile / p) * nb + g % nb : -1;
}

template <typename T>
__global__ void xchg_gather_kernel(const SwapPlan* __restrict__ plan, i64 S, i64 n, const T* A, i64 lda,
                                   T* X, i64 ldx, i64 nb, int p, int pr) {
    const i64 t = (i64)blockIdx.x * 256 + threadIdx.x;
    if (t >= S) return;
    const i64 src = t < plan->nt ? plan->tsrc[t] : -1;
    const i64 lr = src >= 0 ? bc_local_row(src, nb, p, pr) : -1;
    for (i64 j = blockIdx.y; j < n; j += gridDim.y)
        X[t + j * ldx] = lr >= 0 ? A[lr + j * lda] : s_zero(T());
}

template <typename T>
__global__ void xchg_scatter_kernel(const SwapPlan* __restrict__ plan, i64 S, i64 n, const T* X, i64 ldx,
                                    T* A, i64 lda, i64 nb, int p, int pr) {
    const i64 t = (i64)blockIdx.x * 256 + threadIdx.x;
    if (t >= S || t >= plan->nt || plan->trow[t] < 0) return;
    const i64 lr = bc_local_row(plan->trow[t], nb, p, pr);
    if (lr < 0) return;
    for (i64 j = blockIdx.y; j < n; j += gridDim.y) A[lr + j * lda] = X[t + j * ldx];
}

template <typename T>
void xchg_gather(const void* plan, i64 S, i64 n, const T* A, i64 lda, T* X, i64 ldx, i64 nb, int p, int pr,
                 hipStream_t s) {
    if (S <= 0 || n <= 0) return;
    hipLaunchKernelGGL(xchg_gather_kernel<T>, grid2(S, n), dim3(256), 0, s, static_cast<const SwapPlan*>(plan),
                       S, n, A, lda, X, ldx, nb, p, pr);
    HIP_LAUNCH_CHECK();
}
template <typename T>
void xchg_scatter(const void* plan, i64 S, i64 n, const T* X, i64 ldx, T* A, i64 lda, i64 nb, int p, int pr,
                  hipStream_t s) {
    if (S <= 0 || n <= 0) return;
    hipLaunchKernelGGL(xchg_scatter_kernel<T>, grid2(S, n), dim3(256), 0, s, static_cast<const SwapPlan*>(plan),
                       S, n, X, ldx, A, lda, nb, p, pr);
    HIP_LAUNCH_CHECK();
}

// Tournament pivoting (CALU) picks the kb pivot rows of a panel as a SET in
// order (sel[i] = global row that must end at row r0 + i).  LAPACK/SLATE
// pivots are a swap SEQUENCE; convert: swap i exchanges row r0+i with the
// current position of sel[i].  Only window rows are ever displaced (an
// unselected outside row is never touched), so the state is three kb-long
// LDS arrays and each step is O(1): one thread walks the sequence after a
// parallel set-up.
__global__ void __launch_bounds__(MAXSW)
sel_to_ipiv_kernel(const i64* __restrict__ sel, int kb, i64 r0, i64* __restrict__ ipiv) {
    __shared__ i64 at_win[MAXSW];     // original row currently at window position j
    __shared__ i64 where[MAXSW];      // current position of original row sel[i]
    __shared__ int idx_of_win[MAXSW]; // i with sel[i] == r0 + j (-1: not selected)
    const int q = threadIdx.x;
    if (q < kb) { at_win[q] = r0 + q; where[q] = sel[q]; idx_of_win[q] = -1; }
    __syncthreads();
    if (q < kb) {
        const i64 w = sel[q] - r0;
        if (w >= 0 && w < kb) idx_of_win[w] = q;
    }
    __syncthreads();
    if (q == 0) {
        for (int i = 0; i < kb; ++i) {
            const i64 pos = where[i];
            ipiv[i] = pos - r0;
            const i64 o = at_win[i];          // an original window row: moves to pos
            at_win[i] = sel[i];
            if (pos - r0 < kb) at_win[pos - r0] = o;
            const int i2 = idx_of_win[o - r0];
            if (i2 > i) where[i2] = pos;
        }
    }
}
void sel_to_ipiv(const i64* sel, i64 kb, i64 r0, i64* ipiv, hipStream_t s) {
    if (kb <= 0) return;
    if (kb > MAXSW) throw std::invalid_argument("sel_to_ipiv: kb > 512");
    hipLaunchKernelGGL(sel_to_ipiv_kernel, dim3(1), dim3(MAXSW), 0, s, sel, (int)kb, r0, ipiv);
    HIP_LAUNCH_CHECK();
}
template <typename T>
void permute_rows_gather(i64 m, i64 n, const T* A, i64 lda, T* B, i64 ldb, const i64* perm, hipStream_t s) {
    if (m <= 0 || n <= 0) return;
    hipLaunchKernelGGL(row_gather_kernel<T>, grid2(m, n), dim3(256), 0, s, m, n, A, lda, B, ldb, perm);
    HIP_LAUNCH_CHECK();
}

template <typename T>
void permute_rows_scatter(i64 m, i64 n, const T* A, i64 lda, T* B, i64 ldb, const i64* perm, hipStream_t s) {
    if (m <= 0 || n <= 0) return;
    hipLaunchKernelGGL(row_scatter_kernel<T>, grid2(m, n), dim3(256), 0, s, m, n, A, lda, B, ldb, perm);
    HIP_LAUNCH_CHECK();
}

// B = A where the block-cyclic triangle mask keeps the element, 0 elsewhere
// (the stored triangle T / strict triangle S of a distributed Hermitian
// block: the masks of hemmA, formerly torch.where over dense index grids);
// real_diag: the kept diagonal gets its imaginary part dropped (Hermitian)
template <typename T>
__global__ void gecopy_mask_kernel(TriMask mk, i64 m, i64 n, const T* __restrict__ A, i64 lda, T* __restrict__ B,
                                   i64 ldb, int real_diag) {
    const i64 i = (i64)blockIdx.x * 256 + threadIdx.x;
    if (i >= m) return;
    const i64 gr = mk.grow(i);
    // real_diag bit 0: real diagonal; bit 1: merge (B keeps its value
    // outside the mask instead of zero)
    const bool merge = (real_diag & 2) != 0;
    for (i64 j = blockIdx.y; j < n; j += gridDim.y) {
        const bool kp = mk.keep(i, j);
        if (merge && !kp) continue;
        T v = kp ? A[i + j * lda] : s_zero(T());
        if ((real_diag & 1) && gr == mk.gcol(j)) v = s_from_real(T(), s_real(v));
        B[i + j * ldb] = v;
    }
}

template <typename T>
void gecopy_mask(const TriMask& mk, i64 m, i64 n, const T* A, i64 lda, T* B, i64 ldb, bool real_diag,
                 hipStream_t s) {
    if (m <= 0 || n <= 0) return;
    hipLaunchKernelGGL(gecopy_mask_kernel<T>, grid2(m, n), dim3(256), 0, s, mk, m, n, A, lda, B, ldb,
                       real_diag ? 1 : 0);
    HIP_LAUNCH_CHECK();
}
template <typename T>
void gecopy_mask_merge(const TriMask& mk, i64 m, i64 n, const T* A, i64 lda, T* B, i64 ldb, hipStream_t s) {
    if (m <= 0 || n <= 0) return;
    hipLaunchKernelGGL(gecopy_mask_kernel<T>, grid2(m, n), dim3(256), 0, s, mk, m, n, A, lda, B, ldb, 2);
    HIP_LAUNCH_CHECK();
}

#define INST(T)                                                                                   \
    template void permute_rows_scatter<T>(i64, i64, const T*, i64, T*, i64, const i64*, hipStream_t); \
    template void gecopy_mask<T>(const TriMask&, i64, i64, const T*, i64, T*, i64, bool, hipStream_t);   \
    template void gecopy_mask_merge<T>(const TriMask&, i64, i64, const T*, i64, T*, i64, hipStream_t);   \
    template void geset<T>(char, i64, i64, T, T, T*, i64, hipStream_t);                           \
    template void gescale<T>(char, i64, i64, T, T*, i64, hipStream_t);                            \
    template void geadd<T>(char, i64, i64, T, const T*, i64, T, T*, i64, hipStream_t);            \
    template void laswp<T>(i64, T*, i64, i64, i64, const i64*, int, hipStream_t);                 \
    template void laswp_off<T>(i64, T*, i64, i64, i64, const i64*, i64, hipStream_t, int);       \
    template void laswp_cols<T>(i64, T*, i64, i64, i64, const i64*, i64, hipStream_t, int);      \
    template void laswp_cols_plan<T>(i64, T*, i64, const void*, hipStream_t);                      \
    template void permute_rows_gather<T>(i64, i64, const T*, i64, T*, i64, const i64*, hipStream_t);    \
    template void xchg_gather<T>(const void*, i64, i64, const T*, i64, T*, i64, i64, int, int, hipStream_t); \
    template void xchg_scatter<T>(const void*, i64, i64, const T*, i64, T*, i64, i64, int, int, hipStream_t);
INST(float) INST(double) INST(ccplx) INST(zcplx)
#undef INST
#define INSTC(A, B) template void gecopy<A, B>(char, char, i64, i64, const A*, i64, B*, i64, hipStream_t);
INSTC(float, float) INSTC(float, double) INSTC(double, float) INSTC(double, double)
INSTC(ccplx, ccplx) INSTC(ccplx, zcplx) INSTC(zcplx, ccplx) INSTC(zcplx, zcplx)
INSTC(float, ccplx) INSTC(double, zcplx) INSTC(zcplx, double) INSTC(ccplx, float)
#undef INSTC
template void gescale_row_col<float, float>(char, i64, i64, const float*, const float*, float*, i64, hipStream_t);
template void butterfly<float, float>(bool, bool, int, i64, i64, float*, i64, const float*, i64, hipStream_t);
template void butterfly<double, double>(bool, bool, int, i64, i64, double*, i64, const double*, i64, hipStream_t);
template void butterfly<ccplx, float>(bool, bool, int, i64, i64, ccplx*, i64, const float*, i64, hipStream_t);
template void butterfly<zcplx, double>(bool, bool, int, i64, i64, zcplx*, i64, const double*, i64, hipStream_t);
template void gescale_row_col<double, double>(char, i64, i64, const double*, const double*, double*, i64, hipStream_t);
template void gescale_row_col<ccplx, float>(char, i64, i64, const float*, const float*, ccplx*, i64, hipStream_t);
template void gescale_row_col<zcplx, double>(char, i64, i64, const double*, const double*, zcplx*, i64, hipStream_t);

}  // namespace slate_hip
