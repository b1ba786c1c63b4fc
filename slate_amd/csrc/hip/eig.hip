// Back-transformation of the bulge-chasing reflectors on gfx950 (replaces
// SLATE's unmtr_hb2st / unmbr_tb2bd host+device mix, src/unmtr_hb2st.cc,
// internal_unmtr_hb2st.cc).
//
// The reflectors of one sweep act on disjoint row ranges, so a whole sweep
// is one launch: grid = (reflectors of the sweep) x (column chunks), one
// wave per column (lanes along the reflector's rows -> coalesced loads),
// v staged in LDS.  Sweeps are applied last-to-first (Z := H Z).
#include "common.hpp"
#include "kernels.hpp"

namespace slate_hip {

namespace {
constexpr int RW = 4;        // waves per workgroup (one column each at a time)
constexpr int RCOLS = 64;    // columns per workgroup
}

template <typename T>
__global__ void __launch_bounds__(64 * RW)
apply_refl_kernel(i64 ncols, T* Z, i64 ldz, const T* V, i64 b, const T* tau, const i64* row, const i64* len,
                  i64 first, int conj_tau) {
    extern __shared__ unsigned char smem_raw[];
    T* vs = reinterpret_cast<T*>(smem_raw);
    const i64 k = first + blockIdx.x;
    const i64 r0 = row[k], L = len[k];
    T t = tau[k];
    if (conj_tau) t = s_conj(t);
    if (s_is_zero(t)) return;
    for (i64 i = threadIdx.x; i < L; i += 64 * RW) vs[i] = V[k * b + i];
    __syncthreads();
    const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const i64 c0 = (i64)blockIdx.y * RCOLS;
    const i64 c1 = min(ncols, c0 + RCOLS);
    for (i64 c = c0 + wv; c < c1; c += RW) {
        T* z = Z + r0 + c * ldz;
        T w = s_zero(T());
        for (i64 i = lane; i < L; i += 64) w = s_add(w, s_mul(s_conj(vs[i]), z[i]));
        w = wave_sum(w);
        w = s_mul(t, w);
        for (i64 i = lane; i < L; i += 64) z[i] = s_sub(z[i], s_mul(vs[i], w));
    }
}

template <typename T>
void apply_refl_batch(i64 ncols, T* Z, i64 ldz, const T* V, i64 b, const T* tau, const i64* row, const i64* len,
                      i64 first, i64 count, bool conj_tau, hipStream_t s) {
    if (count <= 0 || ncols <= 0) return;
    dim3 grid((unsigned)count, (unsigned)((ncols + RCOLS - 1) / RCOLS));
    hipLaunchKernelGGL(apply_refl_kernel<T>, grid, dim3(64 * RW), sizeof(T) * b, s, ncols, Z, ldz, V, b, tau,
                       row, len, first, conj_tau ? 1 : 0);
    HIP_LAUNCH_CHECK();
}

#define INST(T) \
    template void apply_refl_batch<T>(i64, T*, i64, const T*, i64, const T*, const i64*, const i64*, i64, i64, \
                                      bool, hipStream_t);
INST(float) INST(double) INST(ccplx) INST(zcplx)
#undef INST


__device__ inline float shfl_xor_t(float v, int m) { return __shfl_xor(v, m, 64); }
__device__ inline double shfl_xor_t(double v, int m) { return __shfl_xor(v, m, 64); }
__device__ inline ccplx shfl_xor_t(ccplx v, int m) { return {__shfl_xor(v.re, m, 64), __shfl_xor(v.im, m, 64)}; }
__device__ inline zcplx shfl_xor_t(zcplx v, int m) { return {__shfl_xor(v.re, m, 64), __shfl_xor(v.im, m, 64)}; }

// ---------------------------------------------------------------------------
// Blocked back-transformation: Z := Q2 Z for ALL sweeps in ONE launch.
//
// Task t of sweep j acts on rows [j+1+t b, j+t b+b].  For a block J of b
// consecutive sweeps j0..j0+b-1, H(j,t) only overlaps H(j',t) and H(j',t-1)
// (j' > j); tasks of one sweep are disjoint.  So the block's product is
// G(T)...G(1)G(0) with G(t) = H(j0,t) H(j0+1,t) ... H(j0+b-1,t), and G(t)
// lives in the 2b-row window starting at j0+1+t b.  Columns of Z are
// independent, so each workgroup owns 32 columns and walks the whole
// sequence -- blocks J last-to-first, groups t = 0, 1, ... (window sliding
// down by b rows), reflectors of a group last-to-first -- with its window in
// registers (8 threads per column, b/4 rows each).  Z is read and written
// once per block instead of once per sweep; the reflectors of a group are
// staged through LDS once and read as broadcasts.
template <typename T, int B>
__global__ void __launch_bounds__(256)
unmtr_hb2st_blk_kernel(i64 n, i64 ncols, T* __restrict__ Z, i64 ldz, const T* __restrict__ V,
                       const T* __restrict__ tau, const i64* __restrict__ sp, const i64* __restrict__ nt,
                       i64 nsw, int conj_tau, i64 Jlo, i64 Jhi, i64 slot0) {
    // 8 threads per column, B/4 window rows each (2B-row window); 32 columns
    constexpr int TPC = 8, CW = 32, NT = TPC * CW, RPT = 2 * B / TPC, HALF = TPC / 2;
    __shared__ T Vs[B * B];
    __shared__ T taus[B];
    __shared__ T xfer[B * CW];
    __shared__ i64 sslot[B];
    const int tid = threadIdx.x, q = tid & (TPC - 1), c = tid / TPC;
    const i64 col = (i64)blockIdx.x * CW + c;
    const bool colok = col < ncols;
    T* zc = Z + (colok ? col : 0) * ldz;
    T z[RPT];
    // sweep blocks [Jlo, Jhi] only; V / tau hold the slots from slot0 on (a
    // chunk of the reflectors: the distributed back-transform streams them)
    for (i64 J = min(Jhi, (nsw - 1) / B); J >= Jlo; --J) {
        const i64 j0 = J * B, jn = min((i64)B, nsw - j0);
        const i64 TJ = nt[j0];                      // tasks per sweep do not grow with j
        if (TJ <= 0) continue;
        i64 w0 = j0 + 1;
        #pragma unroll
        for (int r = 0; r < RPT; ++r) {
            const i64 row = w0 + q * RPT + r;
            z[r] = (colok && row < n) ? zc[row] : s_zero(T());
        }
        for (i64 t = 0; t < TJ; ++t) {
            __syncthreads();
            if (tid < B) {
                const int jj = tid;
                i64 slot = -1;
                if (jj < jn && t < nt[j0 + jj]) slot = sp[j0 + jj] + t;
                sslot[jj] = slot;
                const T tv = slot >= 0 ? tau[slot - slot0] : s_zero(T());
                taus[jj] = conj_tau ? s_conj(tv) : tv;
            }
            __syncthreads();
            for (int idx = tid; idx < B * B; idx += NT) {
                const int jj = idx / B, vi = idx - jj * B;
                const i64 slot = sslot[jj];
                Vs[idx] = slot >= 0 ? V[(slot - slot0) * B + vi] : s_zero(T());
            }
            __syncthreads();
            for (int jj = B - 1; jj >= 0; --jj) {
                const T tj = taus[jj];
                if (s_is_zero(tj)) continue;           // uniform
                // every lane runs the same code (the shuffles below read all 8
                // lanes of a column); rows outside the reflector see v = 0
                const int v0 = q * RPT - jj;           // v index of this thread's first row
                T vr[RPT];
                T dp[4] = {s_zero(T()), s_zero(T()), s_zero(T()), s_zero(T())};
                #pragma unroll
                for (int r = 0; r < RPT; ++r) {
                    const int vi = v0 + r;
                    const bool in = vi >= 0 && vi < B;
                    const T v = Vs[jj * B + (in ? vi : 0)];
                    vr[r] = in ? v : s_zero(T());
                    dp[r & 3] = s_add(dp[r & 3], s_mul(s_conj(vr[r]), z[r]));
                }
                T dot = s_add(s_add(dp[0], dp[1]), s_add(dp[2], dp[3]));
                dot = s_add(dot, shfl_xor_t(dot, 1));
                dot = s_add(dot, shfl_xor_t(dot, 2));
                dot = s_add(dot, shfl_xor_t(dot, 4));
                const T w = s_mul(tj, dot);
                #pragma unroll
                for (int r = 0; r < RPT; ++r) z[r] = s_sub(z[r], s_mul(vr[r], w));
            }
            if (t + 1 < TJ) {
                // slide the window down by B rows: the top half is final for
                // this block, the bottom half moves up, B new rows come in
                if (q < HALF) {
                    #pragma unroll
                    for (int r = 0; r < RPT; ++r) {
                        const i64 row = w0 + q * RPT + r;
                        if (colok && row < n) zc[row] = z[r];
                    }
                } else {
                    #pragma unroll
                    for (int r = 0; r < RPT; ++r) xfer[((q - HALF) * RPT + r) * CW + c] = z[r];
                }
                __syncthreads();
                w0 += B;
                if (q < HALF) {
                    #pragma unroll
                    for (int r = 0; r < RPT; ++r) z[r] = xfer[(q * RPT + r) * CW + c];
                } else {
                    #pragma unroll
                    for (int r = 0; r < RPT; ++r) {
                        const i64 row = w0 + q * RPT + r;
                        z[r] = (colok && row < n) ? zc[row] : s_zero(T());
                    }
                }
            }
        }
        #pragma unroll
        for (int r = 0; r < RPT; ++r) {
            const i64 row = w0 + q * RPT + r;
            if (colok && row < n) zc[row] = z[r];
        }
        __syncthreads();      // this block's rows are read by other threads in the next one
    }
}

template <typename T>
bool unmtr_hb2st_blocked_range(i64 n, i64 ncols, T* Z, i64 ldz, const T* V, i64 b, const T* tau, const i64* sp,
                               const i64* nt, i64 nsw, bool conj_tau, i64 Jlo, i64 Jhi, i64 slot0, hipStream_t s) {
    if (ncols <= 0 || nsw <= 0 || Jhi < Jlo) return true;
    dim3 grid((unsigned)((ncols + 31) / 32));     // 32 columns, 256 threads per workgroup
    if (b == 64) {
        hipLaunchKernelGGL((unmtr_hb2st_blk_kernel<T, 64>), grid, dim3(256), 0, s, n, ncols, Z, ldz, V, tau, sp,
                           nt, nsw, conj_tau ? 1 : 0, Jlo, Jhi, slot0);
    } else if (b == 32) {
        hipLaunchKernelGGL((unmtr_hb2st_blk_kernel<T, 32>), grid, dim3(256), 0, s, n, ncols, Z, ldz, V, tau, sp,
                           nt, nsw, conj_tau ? 1 : 0, Jlo, Jhi, slot0);
    } else {
        return false;                               // caller falls back to one launch per sweep
    }
    HIP_LAUNCH_CHECK();
    return true;
}

template <typename T>
bool unmtr_hb2st_blocked(i64 n, i64 ncols, T* Z, i64 ldz, const T* V, i64 b, const T* tau, const i64* sp,
                         const i64* nt, i64 nsw, bool conj_tau, hipStream_t s) {
    return unmtr_hb2st_blocked_range<T>(n, ncols, Z, ldz, V, b, tau, sp, nt, nsw, conj_tau, 0, (i64)1 << 60, 0, s);
}

#define INST2(T) \
    template bool unmtr_hb2st_blocked<T>(i64, i64, T*, i64, const T*, i64, const T*, const i64*, const i64*, i64, \
                                         bool, hipStream_t); \
    template bool unmtr_hb2st_blocked_range<T>(i64, i64, T*, i64, const T*, i64, const T*, const i64*, const i64*, \
                                               i64, bool, i64, i64, i64, hipStream_t);
INST2(float) INST2(double) INST2(ccplx) INST2(zcplx)
#undef INST2


// ---------------------------------------------------------------------------
// MFMA form of the blocked back-transformation (real double, b = 64).
//
// Same grouping as above -- G(J,t) = H(j0,t) ... H(j0+b-1,t) in the 2b-row
// window at j0+1+t b -- but each group is applied as ONE block reflector
// G = I - V T V^H (forward compact WY, T upper triangular):
//   W = V^H Z_win (b x CW),  Z_win -= Y W  with Y = V T (2b x b),
// two small GEMMs on v_mfma_f64_16x16x4.  V is the parallelogram of the
// group's reflectors (reflector jj occupies window rows jj..jj+b-1); T and
// Y of every group are built once by hb2st_tfac_kernel (one workgroup per
// group), so the apply kernel has no T W product (20 % of its MFMA work)
// and no W round trip through LDS for it.
//
// MFMA f64 16x16x4 lane layout: first operand A[i = l & 15][k = l >> 4],
// second operand B[k = l >> 4][j = l & 15], accumulator register r of lane l
// holds D[(l >> 4) + 4 r][l & 15].
namespace {
constexpr int TB = 64;            // band / sweeps per block
constexpr int TCW = 64;           // Z columns per workgroup
// LDS row pitch of the raw reflectors: = 3 (mod 32) doubles.  The W = V^T Z
// A-operand read Vr[(16 wr + li) SV + w - 16 wr - li] (w = k0 + lk) of a
// half-wave then lands on double (SV - 1) li + lk = 2 li + lk (mod 32): 32
// distinct bank pairs (TB + 2 gave li + lk: 2-way, PMC 24 % conflict cycles)
constexpr int SV = TB + 3;
// LDS column pitch of the Z window (column-major): = 2 (mod 32) doubles, so
// the B-operand reads Zs[(16 j + li) SZ + row(lk)] of a half-wave (li 0..15,
// lk 0..1) land on 2 li + lk = 32 distinct bank pairs (2 TB + 4 = 4 mod 32
// put li and li + 8 on the same banks: 2-way, PMC 57.6 % conflict cycles)
constexpr int SZ = 2 * TB + 2;
constexpr int SW = TCW + 16;      // LDS row pitch of W
}

__global__ void __launch_bounds__(256)
hb2st_tfac_kernel(const double* __restrict__ V, const double* __restrict__ tau, const i64* __restrict__ sp,
                  const i64* __restrict__ nt, const i64* __restrict__ gJ, const i64* __restrict__ gt, i64 nsw,
                  double* __restrict__ Tout) {
    __shared__ double Vr[TB * SV];
    __shared__ double G[TB * (TB + 1)];
    __shared__ double Tm[TB * (TB + 1)];
    __shared__ double taus[TB];
    __shared__ i64 sslot[TB];
    const int tid = threadIdx.x;
    const i64 g = blockIdx.x;
    const i64 j0 = gJ[g] * TB, t = gt[g];
    const i64 jn = min((i64)TB, nsw - j0);
    if (tid < TB) {
        i64 slot = -1;
        if (tid < jn && t < nt[j0 + tid]) slot = sp[j0 + tid] + t;
        sslot[tid] = slot;
        taus[tid] = slot >= 0 ? tau[slot] : 0.0;
    }
    __syncthreads();
    for (int idx = tid; idx < TB * TB; idx += 256) {
        const int jj = idx / TB, vi = idx - jj * TB;
        const i64 slot = sslot[jj];
        Vr[jj * SV + vi] = slot >= 0 ? V[slot * TB + vi] : 0.0;
    }
    __syncthreads();
    // G[i][k] = v_i . v_k (i < k): v_i covers window rows i..i+b-1
    for (int idx = tid; idx < TB * TB; idx += 256) {
        const int i = idx / TB, k = idx - i * TB;
        double acc = 0.0;
        if (i < k) {
            for (int r = k; r < i + TB; ++r) acc += Vr[i * SV + (r - i)] * Vr[k * SV + (r - k)];
        }
        G[i * (TB + 1) + k] = acc;
        Tm[i * (TB + 1) + k] = 0.0;
    }
    __syncthreads();
    // forward larft: T[0:k, k] = -tau_k T[0:k, 0:k] G[0:k, k], T[k][k] = tau_k
    for (int k = 0; k < TB; ++k) {
        double acc = 0.0;
        if (tid < k) {
            for (int l = tid; l < k; ++l) acc += Tm[tid * (TB + 1) + l] * G[l * (TB + 1) + k];
        }
        __syncthreads();
        if (tid < k) Tm[tid * (TB + 1) + k] = -taus[k] * acc;
        if (tid == k) Tm[k * (TB + 1) + k] = taus[k];
        __syncthreads();
    }
    // Y = V T (2 TB x TB): the apply kernel then runs Z -= Y (V^H Z), two
    // GEMMs instead of three.  Stored in that kernel's MFMA A-operand order:
    // element (wr, ks, lane) = Y[16 wr + (lane & 15)][4 ks + (lane >> 4)],
    // wr = 2 wave + row tile, so every prefetch is one coalesced 512-B load.
    double* Yo = Tout + g * (2 * TB * TB);
    for (int f = tid; f < 2 * TB * TB; f += 256) {
        const int lf = f & 63, ks = (f >> 6) & 15, wr = f >> 10;
        const int row = 16 * wr + (lf & 15), k = 4 * ks + (lf >> 4);
        double acc = 0.0;
        for (int l = max(0, row - TB + 1); l <= min(k, row); ++l)
            acc += Vr[l * SV + (row - l)] * Tm[l * (TB + 1) + k];
        Yo[f] = acc;
    }
}

__global__ void __launch_bounds__(512)
unmtr_hb2st_mfma_kernel(i64 n, i64 ncols, double* __restrict__ Z, i64 ldz, const double* __restrict__ V,
                        const i64* __restrict__ sp, const i64* __restrict__ nt, const i64* __restrict__ gptr,
                        const double* __restrict__ Tg, i64 nsw) {
    __shared__ double Vr[TB * SV];
    __shared__ double Zs[TCW * SZ];
    __shared__ double Ws[TB * SW];
    __shared__ i64 ssp[TB], snt[TB];
    const int tid = threadIdx.x, lane = tid & 63, wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int li = lane & 15, lk = lane >> 4;
    // 8 waves, two per SIMD (MFMA latency hidden across waves): wave wv
    // owns W / Z row tiles of wr = wv & 3 and the column tiles 2 wc, 2 wc + 1
    // (wc = wv >> 2)
    const int wr = wv & 3, wc = wv >> 2;
    const i64 c0 = (i64)blockIdx.x * TCW;
    const int ncw = (int)min((i64)TCW, ncols - c0);
    // window row w of group t lives in Zs at column-major row ((w >> 6) + t) & 1) * 64 + (w & 63)
    auto zrow = [](int w, i64 t) { return (int)((((w >> 6) + t) & 1) * TB + (w & (TB - 1))); };
    // Zs element (column c, physical row r): the row's lowest bit flipped
    // for columns 8..15 of every 16, so the accumulator stores (16
    // contiguous lanes = 16 columns of one row, ds_write banks (a/4) mod 32)
    // put columns c and c + 8 on different banks; every read pattern stays
    // conflict-free (a permutation inside aligned row pairs)
    auto zi = [](int c, int r) { return c * SZ + (r ^ ((c >> 3) & 1)); };
    // register staging (software pipeline): thread (wv, lane) moves element
    // (row lane, column wv + 8 i) of a Z half and reflector element
    // (jj = wv + 8 i, vi = lane) of a group, i < 8
    constexpr int PR = TB * TB / 512;
    double pv[PR], py[32], pz[PR];
    auto fetch_v = [&](i64 t) {
        #pragma unroll
        for (int i = 0; i < PR; ++i) {
            const int jj = wv + 8 * i;
            pv[i] = (t < snt[jj]) ? V[(ssp[jj] + t) * TB + lane] : 0.0;
        }
    };
    auto fetch_z = [&](i64 row0) {
        #pragma unroll
        for (int i = 0; i < PR; ++i) {
            const int cc = wv + 8 * i;
            const i64 row = row0 + lane;
            pz[i] = (cc < ncw && row < n) ? Z[(c0 + cc) * ldz + row] : 0.0;
        }
    };
    auto put_z = [&](int phys) {
        #pragma unroll
        for (int i = 0; i < PR; ++i) Zs[zi(wv + 8 * i, phys * TB + lane)] = pz[i];
    };
    auto store_half = [&](i64 row0, int phys) {
        #pragma unroll
        for (int i = 0; i < PR; ++i) {
            const int cc = wv + 8 * i;
            const i64 row = row0 + lane;
            if (cc < ncw && row < n) Z[(c0 + cc) * ldz + row] = Zs[zi(cc, phys * TB + lane)];
        }
    };
    for (i64 J = (nsw - 1) / TB; J >= 0; --J) {
        const i64 j0 = J * TB, jn = min((i64)TB, nsw - j0);
        const i64 TJ = nt[j0];
        if (TJ <= 0) continue;
        i64 w0 = j0 + 1;
        __syncthreads();
        if (tid < TB) {
            ssp[tid] = tid < jn ? sp[j0 + tid] : 0;
            snt[tid] = tid < jn ? nt[j0 + tid] : 0;       // missing sweeps: no tasks
        }
        fetch_z(w0);
        put_z(0);
        fetch_z(w0 + TB);
        put_z(1);
        __syncthreads();
        fetch_v(0);
        for (i64 t = 0; t < TJ; ++t) {
            const double* Yg = Tg + (gptr[J] + t) * (2 * TB * TB) + (i64)(2 * wr) * 16 * 64 + lane;
            #pragma unroll
            for (int i = 0; i < 32; ++i) py[i] = Yg[i * 64];              // (row tile i / 16, k step i % 16)
            #pragma unroll
            for (int i = 0; i < PR; ++i) Vr[(wv + 8 * i) * SV + lane] = pv[i];
            __syncthreads();
            const bool more = t + 1 < TJ;
            if (more) {
                fetch_v(t + 1);                  // in flight during this group's GEMMs
                fetch_z(w0 + 2 * TB);
            }
            auto vg = [&](int w, int jj) {
                const int vi = w - jj;
                return (vi >= 0 && vi < TB) ? Vr[jj * SV + vi] : 0.0;
            };
            // (1) W = V^T Z: W rows 16 wr..16 wr+15, column tiles 2 wc, 2 wc+1
            d4 acc[2];
            #pragma unroll
            for (int j = 0; j < 2; ++j) acc[j] = d4{0.0, 0.0, 0.0, 0.0};
            // reflectors 16 wr..16 wr+15 are zero outside window rows
            // 16 wr..16 wr+78: 20 of the 32 k-steps (V is a parallelogram)
            #pragma unroll 4
            for (int k0 = 16 * wr; k0 < 16 * wr + TB + 16; k0 += 4) {
                const int w = k0 + lk;
                const double a = vg(w, 16 * wr + li);
                const int pr = zrow(w, t);
                #pragma unroll
                for (int j = 0; j < 2; ++j) {
                    const double b = Zs[zi(16 * (2 * wc + j) + li, pr)];
                    acc[j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[j], 0, 0, 0);
                }
            }
            #pragma unroll
            for (int j = 0; j < 2; ++j)
                #pragma unroll
                for (int r = 0; r < 4; ++r) Ws[(16 * wr + lk + 4 * r) * SW + 16 * (2 * wc + j) + li] = acc[j][r];
            __syncthreads();
            // (2) Z -= Y W: window rows 32 wr..32 wr+31 (2 row tiles) x
            // column tiles 2 wc, 2 wc+1; each W fragment feeds both row tiles
            {
                d4 zc[2][2];
                #pragma unroll
                for (int ri = 0; ri < 2; ++ri)
                    #pragma unroll
                    for (int j = 0; j < 2; ++j)
                        #pragma unroll
                        for (int r = 0; r < 4; ++r)
                            zc[ri][j][r] = Zs[zi(16 * (2 * wc + j) + li, zrow(32 * wr + 16 * ri + lk + 4 * r, t))];
                #pragma unroll
                for (int k0 = 0; k0 < TB; k0 += 4) {
                    const int jj = k0 + lk;
                    double bw[2];
                    #pragma unroll
                    for (int j = 0; j < 2; ++j) bw[j] = Ws[jj * SW + 16 * (2 * wc + j) + li];
                    #pragma unroll
                    for (int ri = 0; ri < 2; ++ri) {
                        const double a = -py[ri * 16 + k0 / 4];
                        #pragma unroll
                        for (int j = 0; j < 2; ++j)
                            zc[ri][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, bw[j], zc[ri][j], 0, 0, 0);
                    }
                }
                #pragma unroll
                for (int ri = 0; ri < 2; ++ri)
                    #pragma unroll
                    for (int j = 0; j < 2; ++j)
                        #pragma unroll
                        for (int r = 0; r < 4; ++r)
                            Zs[zi(16 * (2 * wc + j) + li, zrow(32 * wr + 16 * ri + lk + 4 * r, t))] = zc[ri][j][r];
            }
            __syncthreads();
            if (more) {
                // the top half (physical t & 1) is final: out, and the
                // prefetched next B rows in
                const int ph = (int)(t & 1);
                store_half(w0, ph);
                put_z(ph);
                w0 += TB;
            }
        }
        const i64 tl = TJ - 1;
        store_half(w0, (int)(tl & 1));
        store_half(w0 + TB, (int)((tl + 1) & 1));
        __syncthreads();      // next block reads rows written by other threads
    }
}

bool unmtr_hb2st_mfma(i64 n, i64 ncols, double* Z, i64 ldz, const double* V, i64 b, const double* tau,
                      const i64* sp, const i64* nt, const i64* gJ, const i64* gt, const i64* gptr, i64 ngroups,
                      double* Tg, i64 nsw, hipStream_t s, int phase) {
    // phase bit 1: build the groups' Y = V T into Tg; bit 2: apply them (the
    // native heev builds Tg on a side stream while the tridiagonal D & C runs)
    if (b != TB) return false;
    if (ncols <= 0 || nsw <= 0 || ngroups <= 0) return true;
    if (phase & 1) {
        hipLaunchKernelGGL(hb2st_tfac_kernel, dim3((unsigned)ngroups), dim3(256), 0, s, V, tau, sp, nt, gJ, gt, nsw,
                           Tg);
        HIP_LAUNCH_CHECK();
    }
    if (!(phase & 2)) return true;
    hipLaunchKernelGGL(unmtr_hb2st_mfma_kernel, dim3((unsigned)((ncols + TCW - 1) / TCW)), dim3(512), 0, s, n, ncols,
                       Z, ldz, V, sp, nt, gptr, Tg, nsw);
    HIP_LAUNCH_CHECK();
    return true;
}

}  // namespace slate_hip
