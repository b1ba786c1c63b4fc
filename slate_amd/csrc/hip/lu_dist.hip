// Distributed partial-pivoting LU panel for p > 1 process rows: the panel
// rows STAY on their owners.  Per column j of a b-wide block of the panel
// (SLATE: src/internal/Tile_getrf.hh:160-447 -- per-column MPI_Allreduce
// MAXLOC + MPI_Bcast of the pivot row, internal_getrf.cc:20-121):
//
//   lu_dist_step   (all local rows, many workgroups)
//       apply column j-1 from the p gathered records: pick the pivot
//       (NaN wins, larger |a|, lower global row; threshold pivoting), put the
//       pivot row into local row j-1 / the old row j-1 into the pivot's row,
//       multipliers and the rank-1 update of the block's columns; then each
//       workgroup's arg-max of column j over its rows with global index >= j
//   lu_dist_record (one workgroup)
//       reduce the partials; record = [|v|, global row, has-row-j, candidate
//       row (b), row j (b, its owner only)]
//   <all-gather of the p records over the column communicator>  (host)
//
// Every rank picks the same pivot from the same records (deterministic), so
// no second broadcast is needed; the b x b top rows travel inside the
// records and every rank keeps the same copy of the panel's top block T.
// Columns outside the b-wide block are brought along by the caller's
// recursion (one owner-masked row exchange per level, models/lu.py).
#include "common.hpp"
#include "kernels.hpp"

namespace slate_hip {

namespace {
constexpr int LDT = 256;          // threads per workgroup
constexpr int LU_DIST_MAXG = 1024; // max workgroups (partials workspace: 16 KB)

template <typename R>
__device__ inline bool beats_d(R v, i64 i, R w, i64 k) {
    return (v != v && w == w) || v > w || (v == w && i < k);
}
template <typename T> __device__ inline typename scalar_traits<T>::real rpart(T x) {
    if constexpr (scalar_traits<T>::is_complex) return x.re; else return x;
}
template <typename T> __device__ inline T from_r(typename scalar_traits<T>::real r) {
    return s_from_real(T(), r);
}

// pivot of column jp from the p records: winner record and its global row,
// the owner record of row jp, and whether row jp itself is the pivot row
// (no candidates left, or threshold pivoting keeps the diagonal)
template <typename T>
__device__ inline void pick_pivot(const T* recs, int p, int recn, int b, int jcol, double thr, int& win, i64& pg,
                                  int& dwn, bool& use_diag) {
    using R = typename scalar_traits<T>::real;
    R bv = R(-1);
    i64 bi = (i64)1 << 62;
    win = -1;
    dwn = -1;
    for (int r = 0; r < p; ++r) {
        const T* rc = recs + (i64)r * recn;
        const R v = rpart(rc[0]);
        if (rpart(rc[2]) != R(0)) dwn = r;
        if (v >= R(0) || v != v) {
            const i64 gi = (i64)rpart(rc[1]);
            if (win < 0 || beats_d(v, gi, bv, bi)) { bv = v; bi = gi; win = r; }
        }
    }
    pg = bi;
    use_diag = win < 0;
    if (!use_diag && thr < 1.0 && dwn >= 0) {
        const R dj = s_abs1(recs[(i64)dwn * recn + 3 + b + jcol]);
        if (dj == dj && (double)dj >= thr * (double)bv) use_diag = true;
    }
}
}  // namespace

template <typename T>
__global__ void __launch_bounds__(LDT)
lu_dist_step_kernel(i64 nr, T* W, i64 ldw, const i64* __restrict__ grow, int c0, int c1, int j,
                    const T* __restrict__ recs, int p, int recn, T* Tt, i64 ldt, i64* ipiv, i64* info,
                    i64 info_off, double thr, typename scalar_traits<T>::real* part_v, i64* part_i) {
    using R = typename scalar_traits<T>::real;
    const int b = c1 - c0;
    __shared__ R sv[LDT / 64];
    __shared__ i64 si[LDT / 64];
    const int tid = threadIdx.x;
    // ---- apply column jp = j - 1
    if (j > c0) {
        const int jp = j - 1, jc = jp - c0;
        int win, dwn;
        i64 pg;
        bool use_diag;
        pick_pivot(recs, p, recn, b, jc, thr, win, pg, dwn, use_diag);
        const T* drow = recs + (i64)dwn * recn + 3 + b;
        const T* prow = use_diag ? drow : recs + (i64)win * recn + 3;
        if (use_diag) pg = jp;
        const T u = prow[jc];
        const bool uz = s_is_zero(u);
        for (i64 i = (i64)blockIdx.x * LDT + tid; i < nr; i += (i64)gridDim.x * LDT) {
            const i64 gi = grow[i];
            if (gi < jp) continue;
            T* row = W + i;
            if (gi == jp) {
                for (int c = 0; c < b; ++c) row[c * ldw] = prow[c];
                continue;
            }
            if (gi == pg)
                for (int c = 0; c < b; ++c) row[c * ldw] = drow[c];
            T l = row[jc * ldw];
            if (!uz) l = s_div(l, u);
            row[jc * ldw] = l;
            for (int c = jc + 1; c < b; ++c) row[c * ldw] = s_sub(row[c * ldw], s_mul(l, prow[c]));
        }
        if (blockIdx.x == 0) {
            if (tid < b) Tt[jp + (i64)(c0 + tid) * ldt] = prow[tid];
            if (tid == 0) {
                if (ipiv) ipiv[jp] = pg;
                if (uz && info)
                    atomicCAS(reinterpret_cast<unsigned long long*>(info), 0ull,
                              (unsigned long long)(jp + 1 + info_off));
            }
        }
    }
    // ---- arg-max partials of column j
    if (j < c1) {
        const int jc = j - c0;
        R v = R(-1);
        i64 bi = -1;
        for (i64 i = (i64)blockIdx.x * LDT + tid; i < nr; i += (i64)gridDim.x * LDT) {
            if (grow[i] < j) continue;
            const R x = s_abs1(W[i + (i64)jc * ldw]);
            if (bi < 0 || beats_d(x, grow[i], v, grow[bi])) { v = x; bi = i; }
        }
        // wave then workgroup reduction (ties: lower global row)
        for (int o = 32; o > 0; o >>= 1) {
            const R w = __shfl_xor(v, o, 64);
            const i64 k = __shfl_xor(bi, o, 64);
            const bool take = k >= 0 && (bi < 0 || beats_d(w, grow[k], v, grow[bi]));
            if (take) { v = w; bi = k; }
        }
        if ((tid & 63) == 0) { sv[tid >> 6] = v; si[tid >> 6] = bi; }
        __syncthreads();
        if (tid == 0) {
            for (int k = 1; k < LDT / 64; ++k)
                if (si[k] >= 0 && (bi < 0 || beats_d(sv[k], grow[si[k]], v, grow[bi]))) { v = sv[k]; bi = si[k]; }
            part_v[blockIdx.x] = v;
            part_i[blockIdx.x] = bi;
        }
    }
}

template <typename T>
__global__ void __launch_bounds__(LDT)
lu_dist_record_kernel(int nparts, const T* W, i64 ldw, const i64* __restrict__ grow, int b, i64 diag_local,
                      const typename scalar_traits<T>::real* part_v, const i64* part_i, T* rec) {
    using R = typename scalar_traits<T>::real;
    __shared__ R bv_s;
    __shared__ i64 bi_s;
    const int tid = threadIdx.x;
    if (tid == 0) {
        R v = R(-1);
        i64 bi = -1;
        for (int k = 0; k < nparts; ++k) {
            const i64 i = part_i[k];
            if (i >= 0 && (bi < 0 || beats_d(part_v[k], grow[i], v, grow[bi]))) { v = part_v[k]; bi = i; }
        }
        bv_s = v;
        bi_s = bi;
        rec[0] = from_r<T>(bi >= 0 ? v : R(-1));
        rec[1] = from_r<T>(bi >= 0 ? (R)grow[bi] : R(1e30));
        rec[2] = from_r<T>(diag_local >= 0 ? R(1) : R(0));
    }
    __syncthreads();
    const i64 bi = bi_s;
    for (int c = tid; c < b; c += LDT) {
        rec[3 + c] = bi >= 0 ? W[bi + (i64)c * ldw] : s_zero(T());
        rec[3 + b + c] = diag_local >= 0 ? W[diag_local + (i64)c * ldw] : s_zero(T());
    }
}

template <typename T>
void lu_dist_step(i64 nr, T* W, i64 ldw, const i64* grow, int c0, int c1, int j, const T* recs, int p, T* Tt,
                  i64 ldt, i64* ipiv, i64* info, i64 info_off, double thr, T* rec, void* part, i64 diag_local,
                  hipStream_t s) {
    using R = typename scalar_traits<T>::real;
    const int b = c1 - c0, recn = 3 + 2 * b;
    const int G = (int)std::max<i64>(1, std::min<i64>(LU_DIST_MAXG, (nr + LDT - 1) / LDT));
    R* pv = static_cast<R*>(part);
    i64* pi = reinterpret_cast<i64*>(static_cast<char*>(part) + LU_DIST_MAXG * sizeof(double));
    hipLaunchKernelGGL(lu_dist_step_kernel<T>, dim3(G), dim3(LDT), 0, s, nr, W, ldw, grow, c0, c1, j, recs, p, recn,
                       Tt, ldt, ipiv, info, info_off, thr, pv, pi);
    if (j < c1)
        hipLaunchKernelGGL(lu_dist_record_kernel<T>, dim3(1), dim3(LDT), 0, s, G, (const T*)W, ldw, grow, b,
                           diag_local, (const R*)pv, (const i64*)pi, rec);
    HIP_LAUNCH_CHECK();
}

#define INST(T)                                                                                               \
    template void lu_dist_step<T>(i64, T*, i64, const i64*, int, int, int, const T*, int, T*, i64, i64*, i64*, \
                                  i64, double, T*, void*, i64, hipStream_t);
INST(float) INST(double) INST(ccplx) INST(zcplx)
#undef INST

}  // namespace slate_hip
