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
#include <algorithm>
#include <cstring>

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

// ---------------------------------------------------------------------------
// Device-resident base block: ONE persistent launch per b-column block, the
// p column peers exchanging their pivot records through peer-mapped
// mailboxes (hipIpcOpenMemHandle: xGMI on a node, the same HBM when ranks
// share a GPU) instead of one host-issued kernel + RCCL all-gather per column
// (SLATE: Tile_getrf.hh:160-447 does an
// MPI_Allreduce(MAXLOC) + MPI_Bcast per column from host threads).
//
// Per column j, every workgroup of every rank:
//   apply column j-1 from the p records in ITS OWN mailbox (same pivot rule
//   as lu_dist_step_kernel: every rank picks the same pivot);
//   arg-max of column j over its rows -> partial slot (tag-ordered agent-scope
//   stores: value, global row, candidate row);
// the leader workgroup (0) gathers the G partials (and the diagonal row on
// the owner rank), builds this rank's record and stores it into slot
// [parity j][me] of EVERY peer's mailbox (system-scope stores, release
// fence, then the tag).  Tags are the host's monotonic sequence numbers, two
// parities suffice (a rank posts column j+2 only after every peer posted
// j+1, i.e. after it read j).  Every wait is bounded by wall time (s_memrealtime,
// LU_PEER_TIMEOUT): a peer that never comes sets *err and the grid drains.
namespace {
constexpr int LUP_BMAX = 64, LUP_PMAX = 16, LUP_GMAX = 64;
constexpr size_t LUP_REC = 2304;     // mailbox slot: {tag, v, gi, has_diag} + cand[BMAX] + diag[BMAX] (<= 16 B each)
constexpr size_t LUP_PART = 1152;    // partial slot: {tag, gi, v, -} + cand[BMAX]
constexpr unsigned long long LU_PEER_TIMEOUT = 6000000000ull;   // 60 s of the 100 MHz real-time counter

template <int SC, typename T> __device__ inline void put_w(T* dst, T v) {
    const uint32_t* w = reinterpret_cast<const uint32_t*>(&v);
    #pragma unroll
    for (int k = 0; k < (int)(sizeof(T) / 4); ++k)
        __hip_atomic_store(reinterpret_cast<uint32_t*>(dst) + k, w[k], __ATOMIC_RELAXED, SC);
}
template <int SC, typename T> __device__ inline T get_w(const T* src) {
    T v;
    uint32_t* w = reinterpret_cast<uint32_t*>(&v);
    #pragma unroll
    for (int k = 0; k < (int)(sizeof(T) / 4); ++k)
        w[k] = __hip_atomic_load(reinterpret_cast<const uint32_t*>(src) + k, __ATOMIC_RELAXED, SC);
    return v;
}
template <int SC> __device__ inline void put_i(long long* dst, long long v) {
    __hip_atomic_store(dst, v, __ATOMIC_RELAXED, SC);
}
template <int SC> __device__ inline long long get_i(const long long* src) {
    return __hip_atomic_load(src, __ATOMIC_RELAXED, SC);
}
template <int SC> __device__ inline void put_d(double* dst, double v) { put_w<SC, double>(dst, v); }
template <int SC> __device__ inline double get_d(const double* src) { return get_w<SC, double>(src); }

// bounded poll of one tag (>= want)
template <int SC> __device__ inline bool poll_tag(const long long* t, long long want) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (get_i<SC>(t) < want) {
        __builtin_amdgcn_s_sleep(2);
        if (__builtin_amdgcn_s_memrealtime() - t0 > LU_PEER_TIMEOUT) return false;
    }
    return true;
}

// release by one wave: every lane's stores done, fence, then the tag
template <int SC> __device__ inline void wave_release() {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if constexpr (SC == __HIP_MEMORY_SCOPE_SYSTEM) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    else __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}
template <int SC> __device__ inline void wave_acquire() {
    if constexpr (SC == __HIP_MEMORY_SCOPE_SYSTEM) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    else __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

struct RecHdr { long long tag; double v; long long gi; long long has_diag; };
struct PartHdr { long long tag; long long gi; double v; long long pad; };

__device__ inline char* rec_slot(char* mbox, int par, int r) { return mbox + ((size_t)par * LUP_PMAX + r) * LUP_REC; }
__device__ inline char* part_slot(char* part, int par, int g) { return part + ((size_t)par * LUP_GMAX + g) * LUP_PART; }
__device__ inline char* diag_slot(char* part, int par) { return part + ((size_t)2 * LUP_GMAX + par) * LUP_PART; }
}  // namespace

size_t lu_peer_mailbox_bytes() { return 2 * LUP_PMAX * LUP_REC; }
size_t lu_peer_part_bytes() { return (2 * LUP_GMAX + 2) * LUP_PART; }
int lu_peer_max_b() { return LUP_BMAX; }
int lu_peer_max_p() { return LUP_PMAX; }

template <typename T>
__global__ void __launch_bounds__(LDT)
lu_dist_base_kernel(i64 nr, T* W, i64 ldw, const i64* __restrict__ grow, int c0, int c1, T* Tt, i64 ldt, i64* ipiv,
                    i64* info, i64 info_off, double thr, LuPeer pe) {
    using R = typename scalar_traits<T>::real;
    constexpr int SYS = __HIP_MEMORY_SCOPE_SYSTEM, AG = __HIP_MEMORY_SCOPE_AGENT;
    const int b = c1 - c0, G = gridDim.x, g = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int p = pe.p, me = pe.me;
    char* mine = reinterpret_cast<char*>(pe.mbox[me]);
    __shared__ T prow_s[LUP_BMAX], drow_s[LUP_BMAX];
    __shared__ R sv[LDT / 64];
    __shared__ i64 si[LDT / 64];
    __shared__ int sh_win, sh_dwn, sh_use_diag, sh_abort;
    __shared__ i64 sh_pg, sh_bi;
    __shared__ double hv_s[LUP_PMAX];
    __shared__ long long hg_s[LUP_PMAX];
    __shared__ int hd_s[LUP_PMAX];
    if (tid == 0) sh_abort = 0;
    __syncthreads();
    for (int j = c0; j <= c1; ++j) {
        // ---- apply column jp = j - 1 from the p records of my mailbox
        if (j > c0) {
            const int jp = j - 1, jc = jp - c0, par = jp & 1;
            const long long want = pe.seq0 + (jp - c0) + 1;
            if (wv == 0) {
                bool ok = true;
                if (lane < p) ok = poll_tag<SYS>(&reinterpret_cast<const RecHdr*>(rec_slot(mine, par, lane))->tag, want);
                if (__ballot(!ok) != 0ull) {
                    if (lane == 0) { sh_abort = 1; atomicOr(pe.err, 1ull); }
                } else {
                    wave_acquire<SYS>();
                    // headers of the p records -> LDS, then lane 0 picks (same rule as pick_pivot)
                    if (lane < p) {
                        const RecHdr* h = reinterpret_cast<const RecHdr*>(rec_slot(mine, par, lane));
                        hv_s[lane] = get_d<SYS>(&h->v);
                        hg_s[lane] = get_i<SYS>(&h->gi);
                        hd_s[lane] = (int)get_i<SYS>(&h->has_diag);
                    }
                    __builtin_amdgcn_wave_barrier();
                    if (lane == 0) {
                        R bv = R(-1);
                        i64 bi = (i64)1 << 62;
                        int win = -1, dwn = -1;
                        for (int r = 0; r < p; ++r) {
                            if (hd_s[r]) dwn = r;
                            const R x = (R)hv_s[r];
                            if (x >= R(0) || x != x)
                                if (win < 0 || beats_d(x, (i64)hg_s[r], bv, bi)) { bv = x; bi = hg_s[r]; win = r; }
                        }
                        bool use_diag = win < 0;
                        if (!use_diag && thr < 1.0 && dwn >= 0) {
                            const T* dr = reinterpret_cast<const T*>(rec_slot(mine, par, dwn) + sizeof(RecHdr)) + LUP_BMAX;
                            const R dj = s_abs1(get_w<SYS, T>(dr + jc));
                            if (dj == dj && (double)dj >= thr * (double)bv) use_diag = true;
                        }
                        sh_win = win; sh_dwn = dwn; sh_use_diag = use_diag; sh_pg = use_diag ? jp : bi;
                    }
                }
            }
            __syncthreads();
            if (sh_abort) break;
            const int win = sh_win, dwn = sh_dwn;
            const bool use_diag = sh_use_diag;
            const i64 pg = sh_pg;
            if (tid < b) {
                const T d = dwn >= 0 ? get_w<SYS, T>(reinterpret_cast<const T*>(rec_slot(mine, par, dwn) + sizeof(RecHdr))
                                                     + LUP_BMAX + tid)
                                     : s_zero(T());
                drow_s[tid] = d;
                prow_s[tid] = use_diag ? d
                                       : get_w<SYS, T>(reinterpret_cast<const T*>(rec_slot(mine, par, win) + sizeof(RecHdr)) + tid);
            }
            __syncthreads();
            const T u = prow_s[jc];
            const bool uz = s_is_zero(u);
            for (i64 i = (i64)g * LDT + tid; i < nr; i += (i64)G * LDT) {
                const i64 gi = grow[i];
                if (gi < jp) continue;
                T* row = W + i;
                if (gi == jp) {
                    for (int c = 0; c < b; ++c) row[c * ldw] = prow_s[c];
                    continue;
                }
                if (gi == pg)
                    for (int c = 0; c < b; ++c) row[c * ldw] = drow_s[c];
                T l = row[jc * ldw];
                if (!uz) l = s_div(l, u);
                row[jc * ldw] = l;
                for (int c = jc + 1; c < b; ++c) row[c * ldw] = s_sub(row[c * ldw], s_mul(l, prow_s[c]));
            }
            if (g == 0) {
                if (tid < b) Tt[jp + (i64)(c0 + tid) * ldt] = prow_s[tid];
                if (tid == 0) {
                    if (ipiv) ipiv[jp] = pg;
                    if (uz && info)
                        atomicCAS(reinterpret_cast<unsigned long long*>(info), 0ull,
                                  (unsigned long long)(jp + 1 + info_off));
                }
            }
            __syncthreads();
        }
        if (j >= c1) break;
        // ---- arg-max of column j over my rows -> partial slot
        const int jc = j - c0, par = j & 1;
        const long long tag = pe.seq0 + (j - c0) + 1;
        {
            R v = R(-1);
            i64 bi = -1;
            for (i64 i = (i64)g * LDT + tid; i < nr; i += (i64)G * LDT) {
                if (grow[i] < j) continue;
                const R x = s_abs1(W[i + (i64)jc * ldw]);
                if (bi < 0 || beats_d(x, grow[i], v, grow[bi])) { v = x; bi = i; }
            }
            for (int o = 32; o > 0; o >>= 1) {
                const R w = __shfl_xor(v, o, 64);
                const i64 k = __shfl_xor(bi, o, 64);
                const bool take = k >= 0 && (bi < 0 || beats_d(w, grow[k], v, grow[bi]));
                if (take) { v = w; bi = k; }
            }
            if (lane == 0) { sv[wv] = v; si[wv] = bi; }
            __syncthreads();
            if (tid == 0) {
                for (int k = 1; k < LDT / 64; ++k)
                    if (si[k] >= 0 && (bi < 0 || beats_d(sv[k], grow[si[k]], v, grow[bi]))) { v = sv[k]; bi = si[k]; }
                sv[0] = v;
                sh_bi = bi;
            }
            __syncthreads();
        }
        if (wv == 0) {
            const i64 bi = sh_bi;
            char* ps = part_slot(pe.part, par, g);
            T* cand = reinterpret_cast<T*>(ps + sizeof(PartHdr));
            for (int c = lane; c < b; c += 64) put_w<AG, T>(cand + c, bi >= 0 ? W[bi + (i64)c * ldw] : s_zero(T()));
            if (lane == 0) {
                PartHdr* h = reinterpret_cast<PartHdr*>(ps);
                put_i<AG>(&h->gi, bi >= 0 ? (long long)grow[bi] : (long long)1 << 62);
                put_d<AG>(&h->v, bi >= 0 ? (double)sv[0] : -1.0);
            }
            wave_release<AG>();
            if (lane == 0) put_i<AG>(&reinterpret_cast<PartHdr*>(ps)->tag, tag);
            // the diagonal row j (local row j on the owner rank) -> diag slot
            if (pe.has_diag && j < nr && (int)(((i64)j / LDT) % G) == g) {
                char* ds = diag_slot(pe.part, par);
                T* drow = reinterpret_cast<T*>(ds + sizeof(PartHdr));
                for (int c = lane; c < b; c += 64) put_w<AG, T>(drow + c, W[j + (i64)c * ldw]);
                wave_release<AG>();
                if (lane == 0) put_i<AG>(&reinterpret_cast<PartHdr*>(ds)->tag, tag);
            }
        }
        // ---- leader: gather the partials, post my record to every peer
        if (g == 0 && wv == 0) {
            bool ok = true;
            if (lane < G) ok = poll_tag<AG>(&reinterpret_cast<const PartHdr*>(part_slot(pe.part, par, lane))->tag, tag);
            if (ok && pe.has_diag && lane == 0)
                ok = poll_tag<AG>(&reinterpret_cast<const PartHdr*>(diag_slot(pe.part, par))->tag, tag);
            if (__ballot(!ok) != 0ull) {
                if (lane == 0) { sh_abort = 1; atomicOr(pe.err, 1ull); }
            } else {
                wave_acquire<AG>();
                double v = -1.0;
                long long gi = (long long)1 << 62;
                // the lane's own partial: `who` travels with (v, gi) so the
                // posted candidate row is the winner's, not workgroup 0's
                int who = lane < G ? lane : 0;
                if (lane < G) {
                    const PartHdr* h = reinterpret_cast<const PartHdr*>(part_slot(pe.part, par, lane));
                    v = get_d<AG>(&h->v);
                    gi = get_i<AG>(&h->gi);
                }
                for (int o = 32; o > 0; o >>= 1) {
                    const double w = __shfl_xor(v, o, 64);
                    const long long k = __shfl_xor(gi, o, 64);
                    const int ww = __shfl_xor(who, o, 64);
                    const bool wval = w >= 0.0 || w != w, mval = v >= 0.0 || v != v;
                    const bool take = wval && (!mval || beats_d((R)w, (i64)k, (R)v, (i64)gi));
                    if (take) { v = w; gi = k; who = ww; }
                }
                // lane 0's winner for every lane (NaN ties need not agree across lanes)
                v = __shfl(v, 0, 64);
                gi = __shfl(gi, 0, 64);
                who = __shfl(who, 0, 64);
                const bool none = !(v >= 0.0 || v != v);
                const T* cand = reinterpret_cast<const T*>(part_slot(pe.part, par, who) + sizeof(PartHdr));
                const T* dsrc = reinterpret_cast<const T*>(diag_slot(pe.part, par) + sizeof(PartHdr));
                for (int r = 0; r < p; ++r) {
                    char* dst = rec_slot(reinterpret_cast<char*>(pe.mbox[r]), par, me);
                    T* rc = reinterpret_cast<T*>(dst + sizeof(RecHdr));
                    for (int c = lane; c < b; c += 64) {
                        put_w<SYS, T>(rc + c, none ? s_zero(T()) : get_w<AG, T>(cand + c));
                        put_w<SYS, T>(rc + LUP_BMAX + c, pe.has_diag ? get_w<AG, T>(dsrc + c) : s_zero(T()));
                    }
                    if (lane == 0) {
                        RecHdr* h = reinterpret_cast<RecHdr*>(dst);
                        put_d<SYS>(&h->v, v);
                        put_i<SYS>(&h->gi, gi);
                        put_i<SYS>(&h->has_diag, pe.has_diag ? 1 : 0);
                    }
                }
                wave_release<SYS>();
                if (lane < p) put_i<SYS>(&reinterpret_cast<RecHdr*>(rec_slot(reinterpret_cast<char*>(pe.mbox[lane]), par, me))->tag, tag);
            }
        }
        // a leader abort stops this workgroup; the others time out on the records
        __syncthreads();
        if (sh_abort) break;
    }
}

template <typename T>
void lu_dist_base(i64 nr, T* W, i64 ldw, const i64* grow, int c0, int c1, T* Tt, i64 ldt, i64* ipiv, i64* info,
                  i64 info_off, double thr, const LuPeer& pe, int G, hipStream_t s) {
    if (c1 - c0 > LUP_BMAX) throw std::invalid_argument("lu_dist_base: base block wider than 64 columns");
    if (pe.p < 1 || pe.p > LUP_PMAX || pe.me < 0 || pe.me >= pe.p)
        throw std::invalid_argument("lu_dist_base: bad peer group");
    G = std::max(1, std::min(G, LUP_GMAX));
    hipLaunchKernelGGL(lu_dist_base_kernel<T>, dim3(G), dim3(LDT), 0, s, nr, W, ldw, grow, c0, c1, Tt, ldt, ipiv, info,
                       info_off, thr, pe);
    HIP_LAUNCH_CHECK();
}

// Peer mailboxes: uncached device memory (hipDeviceMallocUncached: every
// access goes to memory, what an in-kernel cross-device hand-off needs)
// with an IPC handle for the column peers.
void* lu_peer_alloc(size_t bytes, void* handle64) {
    void* p = nullptr;
    HIP_CHECK(hipExtMallocWithFlags(&p, bytes, hipDeviceMallocUncached));
    HIP_CHECK(hipMemset(p, 0, bytes));
    HIP_CHECK(hipDeviceSynchronize());
    hipIpcMemHandle_t h;
    HIP_CHECK(hipIpcGetMemHandle(&h, p));
    static_assert(sizeof(h) <= 64, "IPC handle larger than 64 bytes");
    std::memset(handle64, 0, 64);
    std::memcpy(handle64, &h, sizeof(h));
    return p;
}
void* lu_peer_open(const void* handle64) {
    hipIpcMemHandle_t h;
    std::memcpy(&h, handle64, sizeof(h));
    void* p = nullptr;
    HIP_CHECK(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess));
    return p;
}
void lu_peer_close(void* p) { (void)hipIpcCloseMemHandle(p); }
void lu_peer_free(void* p) { (void)hipFree(p); }

#define INST(T)                                                                                               \
    template void lu_dist_step<T>(i64, T*, i64, const i64*, int, int, int, const T*, int, T*, i64, i64*, i64*, \
                                  i64, double, T*, void*, i64, hipStream_t);
INST(float) INST(double) INST(ccplx) INST(zcplx)
#undef INST
#define INST(T)                                                                                                   \
    template void lu_dist_base<T>(i64, T*, i64, const i64*, int, int, T*, i64, i64*, i64*, i64, double, const LuPeer&, \
                                  int, hipStream_t);
INST(float) INST(double) INST(ccplx) INST(zcplx)
#undef INST

}  // namespace slate_hip
