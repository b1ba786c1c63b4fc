// Divide & conquer merge kernels for the symmetric tridiagonal eigensolver
// (roles of SLATE's stedc_secular / stedc_z_vector / stedc_merge,
// src/stedc_secular.cc:132-148, src/stedc_merge.cc; LAPACK laed4/laed3).
//
// A merge of size k solves the secular equation
//     f(lambda) = 1 + rho * sum_i z_i^2 / (d_i - lambda) = 0
// for its k roots, recomputes z (Gu-Eisenstat) from the roots so the
// eigenvectors are orthogonal to working precision, and forms the k x k
// eigenvector matrix of the rank-one update that the merge GEMM applies.
// All three steps are O(k^2) and were host-bound (k = 16384 at the top of an
// n = 16384 problem: ~10^10 divisions in the bisection alone).  Here:
//
//  * secular: one thread per root, Bunch-Nielsen-Sorensen steps (bisection
//    fallback) on the offset mu from the nearer pole (lambda = d[org] + mu, so d_i - lambda = (d_i - d_org) - mu
//    has no cancellation).  d and z^2 are streamed through LDS in chunks that
//    the whole wave reads as broadcasts (no bank conflicts); one 64-thread
//    workgroup per 64 roots, so k = 16384 fills 256 CUs.
//  * zhat: one thread per pole, the product formula over all roots, same
//    LDS streaming.
//  * vectors: one workgroup per root j: v_i = zhat_i / (d_i - lambda_j),
//    column norm by a workgroup reduction, normalised column written
//    column-major (coalesced) straight into the GEMM operand.
#include <cstdlib>

#include "common.hpp"
#include "kernels.hpp"

namespace slate_hip {

namespace {
constexpr int SEC_T = 64;        // roots per workgroup (one wave)
constexpr int SEC_CH = 2048;     // poles per LDS chunk (2 x 16 KiB)
constexpr int SEC_ITMAX = 200;   // bisection cap (the host solver's)
}

__global__ void __launch_bounds__(SEC_T)
secular_kernel(i64 n, const double* __restrict__ d, const double* __restrict__ z, double rho, double zz,
               i64* __restrict__ org, double* __restrict__ mu) {
    __shared__ double sd[SEC_CH], sz2[SEC_CH];
    const i64 j = (i64)blockIdx.x * SEC_T + threadIdx.x;
    const bool live = j < n;
    const i64 jj = live ? j : n - 1;
    const bool right = jj + 1 < n;                 // a pole on the right of the interval
    // bracket: root j in (d_j, d_j+1) (last one: (d_n-1, d_n-1 + rho |z|^2))
    const double lo_d = d[jj];
    const double hi_d = right ? d[jj + 1] : d[jj] + rho * zz;
    const double mid = 0.5 * (hi_d - lo_d);
    // pass 0 decides the origin (nearer pole) from the sign of f at the
    // midpoint.  Then Bunch-Nielsen-Sorensen steps: the poles left of the
    // interval (psi) and right of it (phi) are each modelled by one pole at
    // the interval end plus a constant, matched in value and slope at the
    // current point, and the model's root is taken -- quadratic convergence
    // also for roots next to a pole, where Newton crawls.  Every evaluation
    // shrinks the bracket (a, b); a step leaving it falls back to bisection.
    i64 o = jj;
    double a = 0.0, b = mid, m = mid;
    bool done = !live;
    const double eps = 2.220446049250313e-16;
    for (int it = 0; it <= SEC_ITMAX; ++it) {
        if (__syncthreads_and(done ? 1 : 0)) break;
        const double dorg = d[o];
        double ps = 0.0, dps = 0.0, ph = 0.0, dph = 0.0;
        for (i64 c0 = 0; c0 < n; c0 += SEC_CH) {
            const int cn = (int)min((i64)SEC_CH, n - c0);
            __syncthreads();
            for (int i = threadIdx.x; i < cn; i += SEC_T) {
                sd[i] = d[c0 + i];
                const double zi = z[c0 + i];
                sz2[i] = zi * zi;
            }
            __syncthreads();
            if (!done) {
                const i64 split = jj - c0;             // local indices <= split are left poles
                #pragma unroll 4
                for (int i = 0; i < cn; ++i) {
                    const double r = 1.0 / ((sd[i] - dorg) - m);
                    const double t = sz2[i] * r;
                    const bool L = i <= split;
                    ps += L ? t : 0.0;
                    dps += L ? t * r : 0.0;
                    ph += L ? 0.0 : t;
                    dph += L ? 0.0 : t * r;
                }
            }
        }
        if (done) continue;
        const double psi = rho * ps, dpsi = rho * dps, phi = rho * ph, dphi = rho * dph;
        const double fv = 1.0 + psi + phi;
        if (it == 0) {
            if (right && fv < 0) { o = jj + 1; a = -mid; b = 0.0; }   // root right of the midpoint
            else { o = jj; a = 0.0; b = right ? mid : (hi_d - lo_d); }
            m = 0.5 * (a + b);
            continue;
        }
        // converged when f is below its own rounding error (psi / phi are
        // sums of same-sign terms: their magnitudes bound it, as laed4's erretm)
        if (fabs(fv) <= 8.0 * eps * (1.0 + fabs(psi) + fabs(phi))) { done = true; continue; }
        if (fv < 0) a = m; else b = m;
        const double Dlo = (lo_d - dorg) - m;       // < 0
        const double b1 = dpsi * Dlo * Dlo, a1 = psi - dpsi * Dlo;
        double h;
        if (!right) {
            const double c = 1.0 + a1 + phi;
            h = Dlo + b1 / c;
        } else {
            const double Dhi = (hi_d - dorg) - m;   // > 0
            const double b2 = dphi * Dhi * Dhi, a2 = phi - dphi * Dhi;
            const double c = 1.0 + a1 + a2;
            // c (Dlo - h)(Dhi - h) + b1 (Dhi - h) + b2 (Dlo - h) = 0
            const double qa = c, qb = c * (Dlo + Dhi) + b1 + b2, qc = c * Dlo * Dhi + b1 * Dhi + b2 * Dlo;
            const double disc = fmax(qb * qb - 4.0 * qa * qc, 0.0), sq = sqrt(disc);
            double h1, h2;
            if (qb >= 0) { h1 = (qb + sq) / (2.0 * qa); h2 = 2.0 * qc / (qb + sq); }
            else { h1 = 2.0 * qc / (qb - sq); h2 = (qb - sq) / (2.0 * qa); }
            const bool ok1 = h1 > Dlo && h1 < Dhi, ok2 = h2 > Dlo && h2 < Dhi;
            h = ok2 ? h2 : (ok1 ? h1 : -fv / (dpsi + dphi));
        }
        double mn = m + h;
        if (!(mn > a && mn < b)) mn = 0.5 * (a + b);
        if (mn == a || mn == b || fabs(mn - m) <= 4.0 * eps * fabs(mn)) done = true;
        m = mn;
    }
    if (live) { org[j] = o; mu[j] = m; }
}

// Wave-per-root form of secular_kernel (default): the 64 lanes of a wave
// split the pole sums of ONE root and combine them by shuffles; the bracket
// and model-step logic is wave-uniform.  k roots -> k waves (k = 16384 gives
// 64 waves per CU instead of one), each pole sum 64x shorter per lane.
__device__ inline double wave_prod(double v) {
    #pragma unroll
    for (int o = 32; o > 0; o >>= 1) v *= __shfl_xor(v, o, 64);
    return v;
}

__global__ void __launch_bounds__(256)
secular_wave_kernel(i64 n, const double* __restrict__ d, const double* __restrict__ z, double rho, double zz,
                    i64* __restrict__ org, double* __restrict__ mu) {
    const int lane = threadIdx.x & 63;
    const i64 jj = (i64)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (jj >= n) return;                           // the whole wave: no block barriers below
    const bool right = jj + 1 < n;
    const double lo_d = d[jj];
    const double hi_d = right ? d[jj + 1] : d[jj] + rho * zz;
    const double mid = 0.5 * (hi_d - lo_d);
    i64 o = jj;
    double a = 0.0, b = mid, m = mid;
    const double eps = 2.220446049250313e-16;
    for (int it = 0; it <= SEC_ITMAX; ++it) {
        const double dorg = d[o];
        double ps = 0.0, dps = 0.0, ph = 0.0, dph = 0.0;
        for (i64 i = lane; i < n; i += 64) {
            const double r = 1.0 / ((d[i] - dorg) - m);
            const double zi = z[i];
            const double t = zi * zi * r;
            if (i <= jj) { ps += t; dps += t * r; }
            else { ph += t; dph += t * r; }
        }
        ps = wave_sum(ps); dps = wave_sum(dps); ph = wave_sum(ph); dph = wave_sum(dph);
        const double psi = rho * ps, dpsi = rho * dps, phi = rho * ph, dphi = rho * dph;
        const double fv = 1.0 + psi + phi;
        if (it == 0) {
            if (right && fv < 0) { o = jj + 1; a = -mid; b = 0.0; }
            else { o = jj; a = 0.0; b = right ? mid : (hi_d - lo_d); }
            m = 0.5 * (a + b);
            continue;
        }
        if (fabs(fv) <= 8.0 * eps * (1.0 + fabs(psi) + fabs(phi))) break;
        if (fv < 0) a = m; else b = m;
        const double Dlo = (lo_d - dorg) - m;
        const double b1 = dpsi * Dlo * Dlo, a1 = psi - dpsi * Dlo;
        double h;
        if (!right) {
            const double c = 1.0 + a1 + phi;
            h = Dlo + b1 / c;
        } else {
            const double Dhi = (hi_d - dorg) - m;
            const double b2 = dphi * Dhi * Dhi, a2 = phi - dphi * Dhi;
            const double c = 1.0 + a1 + a2;
            const double qa = c, qb = c * (Dlo + Dhi) + b1 + b2, qc = c * Dlo * Dhi + b1 * Dhi + b2 * Dlo;
            const double disc = fmax(qb * qb - 4.0 * qa * qc, 0.0), sq = sqrt(disc);
            double h1, h2;
            if (qb >= 0) { h1 = (qb + sq) / (2.0 * qa); h2 = 2.0 * qc / (qb + sq); }
            else { h1 = 2.0 * qc / (qb - sq); h2 = (qb - sq) / (2.0 * qa); }
            const bool ok1 = h1 > Dlo && h1 < Dhi, ok2 = h2 > Dlo && h2 < Dhi;
            h = ok2 ? h2 : (ok1 ? h1 : -fv / (dpsi + dphi));
        }
        double mn = m + h;
        if (!(mn > a && mn < b)) mn = 0.5 * (a + b);
        const bool stop = (mn == a || mn == b || fabs(mn - m) <= 4.0 * eps * fabs(mn));
        m = mn;
        if (stop) break;
    }
    if (lane == 0) { org[jj] = o; mu[jj] = m; }
}

// wave-per-pole form of zhat_kernel
__global__ void __launch_bounds__(256)
zhat_wave_kernel(i64 n, const double* __restrict__ d, const double* __restrict__ z, double rho,
                 const i64* __restrict__ org, const double* __restrict__ mu, double* __restrict__ zh) {
    const int lane = threadIdx.x & 63;
    const i64 i = (i64)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (i >= n) return;
    const double di = d[i];
    double prod = 1.0, dii = 0.0;
    for (i64 t = lane; t < n; t += 64) {
        const double delta = (d[org[t]] - di) + mu[t];             // lambda_t - d_i
        if (t == i) { dii = delta; continue; }
        prod *= delta / (d[t] - di);
    }
    prod = wave_prod(prod);
    dii = wave_sum(dii);                                           // one lane holds it
    if (lane == 0) {
        const double v = sqrt(fabs(dii * prod / rho));
        zh[i] = z[i] < 0 ? -v : v;
    }
}

// zhat_i^2 = (lambda_i - d_i) prod_{j != i} (lambda_j - d_i) / (d_j - d_i) / rho
__global__ void __launch_bounds__(SEC_T)
zhat_kernel(i64 n, const double* __restrict__ d, const double* __restrict__ z, double rho,
            const i64* __restrict__ org, const double* __restrict__ mu, double* __restrict__ zh) {
    __shared__ double sd[SEC_CH], sl[SEC_CH], sdj[SEC_CH];
    const i64 i = (i64)blockIdx.x * SEC_T + threadIdx.x;
    const bool live = i < n;
    const double di = live ? d[i] : 0.0;
    double prod = 1.0, dii = 1.0;
    for (i64 c0 = 0; c0 < n; c0 += SEC_CH) {
        const int cn = (int)min((i64)SEC_CH, n - c0);
        __syncthreads();
        for (int t = threadIdx.x; t < cn; t += SEC_T) {
            sdj[t] = d[c0 + t];
            sd[t] = d[org[c0 + t]];
            sl[t] = mu[c0 + t];
        }
        __syncthreads();
        if (live) {
            for (int t = 0; t < cn; ++t) {
                const double delta = (sd[t] - di) + sl[t];          // lambda_j - d_i
                if (c0 + t == i) { dii = delta; continue; }
                prod *= delta / (sdj[t] - di);
            }
        }
    }
    if (live) {
        const double v = sqrt(fabs(dii * prod / rho));
        zh[i] = z[i] < 0 ? -v : v;
    }
}

// column j of the rank-one eigenvector matrix, normalised: V[i + j*ldv]
__global__ void __launch_bounds__(256)
secvec_kernel(i64 n, const double* __restrict__ d, const double* __restrict__ zh,
              const i64* __restrict__ org, const double* __restrict__ mu, double* __restrict__ V, i64 ldv) {
    __shared__ double red[4];
    const i64 j = blockIdx.x;
    const double dorg = d[org[j]], mj = mu[j];
    double* col = V + j * ldv;
    double ss = 0.0;
    for (i64 i = threadIdx.x; i < n; i += 256) {
        const double v = zh[i] / ((d[i] - dorg) - mj);            // z_i / (d_i - lambda_j)
        col[i] = v;
        ss += v * v;
    }
    ss = wave_sum(ss);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = ss;
    __syncthreads();
    const double inv = 1.0 / sqrt(red[0] + red[1] + red[2] + red[3]);
    for (i64 i = threadIdx.x; i < n; i += 256) col[i] *= inv;
}

void stedc_secular(i64 n, const double* d, const double* z, double rho, double zz, i64* org, double* mu,
                   double* zh, double* V, i64 ldv, hipStream_t s) {
    if (n <= 0) return;
    // SLATE_AMD_SECULAR_WAVE=0: one thread per root / pole (the older form)
    static const bool wave = [] { const char* e = std::getenv("SLATE_AMD_SECULAR_WAVE"); return !(e && e[0] == '0'); }();
    if (wave) {
        const unsigned g4 = (unsigned)((n + 3) / 4);
        hipLaunchKernelGGL(secular_wave_kernel, dim3(g4), dim3(256), 0, s, n, d, z, rho, zz, org, mu);
        HIP_LAUNCH_CHECK();
        hipLaunchKernelGGL(zhat_wave_kernel, dim3(g4), dim3(256), 0, s, n, d, z, rho, org, mu, zh);
        HIP_LAUNCH_CHECK();
    } else {
        const unsigned g = (unsigned)((n + SEC_T - 1) / SEC_T);
        hipLaunchKernelGGL(secular_kernel, dim3(g), dim3(SEC_T), 0, s, n, d, z, rho, zz, org, mu);
        HIP_LAUNCH_CHECK();
        hipLaunchKernelGGL(zhat_kernel, dim3(g), dim3(SEC_T), 0, s, n, d, z, rho, org, mu, zh);
        HIP_LAUNCH_CHECK();
    }
    if (V != nullptr) {
        hipLaunchKernelGGL(secvec_kernel, dim3((unsigned)n), dim3(256), 0, s, n, d, zh, org, mu, V, ldv);
        HIP_LAUNCH_CHECK();
    }
}

// ---------------------------------------------------------------------------
// Leaves of the divide & conquer tree, all in ONE launch: one wave per leaf
// (n_leaf <= 64), implicit-shift QL with Wilkinson shifts (the host steqr's
// iteration).  The scalar recurrence (d, e in LDS) is computed redundantly
// and identically by the 64 lanes; lane r owns row r of the leaf's
// eigenvector matrix (LDS, column-major, pitch 64) and applies every Givens
// rotation to it as it is generated.  Eigenvalues ascending with their
// columns.  Only the rows in [r0, r1) (this rank's rows) are written, to
// Q(row - r0, col) with ld ldq; w gets the eigenvalues at the leaf's global
// positions.  (The host solved one leaf after another: 256 leaves of 64 at
// n = 16384.)
// LEAF = 64 (one wave) or 128 (two waves; Z = 128 KB of dynamic LDS):
// larger leaves halve the number of merges of the first tree level, whose
// per-merge host work dominated small merges (n = 16384: 255 -> 127 merges).
template <int LEAF>
__global__ void __launch_bounds__(LEAF)
steqr_leaf_kernel(const i64* __restrict__ lo, const i64* __restrict__ hi, const double* __restrict__ d_in,
                  const double* __restrict__ e_in, double* __restrict__ w, double* __restrict__ Q, i64 ldq, i64 r0,
                  i64 r1, i64* fails, int maxit) {
    extern __shared__ double Z[];                  // LEAF * LEAF, column-major
    __shared__ double d[LEAF], ew[LEAF];
    const int lane = threadIdx.x;
    const i64 a = lo[blockIdx.x];
    const int n = (int)(hi[blockIdx.x] - a);
    if (lane < n) {
        d[lane] = d_in[a + lane];
        ew[lane] = lane < n - 1 ? e_in[a + lane] : 0.0;
    }
    for (int c = 0; c < n; ++c) Z[c * LEAF + lane] = (lane == c) ? 1.0 : 0.0;
    __syncthreads();
    const double eps = 2.220446049250313e-16, tiny = 2.2250738585072014e-308;
    int nfail = 0;
    for (int l = 0; l < n; ++l) {
        int iter = 0;
        while (true) {
            int m = l;
            for (; m < n - 1; ++m) {
                const double dd = fabs(d[m]) + fabs(d[m + 1]);
                if (fabs(ew[m]) <= eps * dd || fabs(ew[m]) < tiny) break;
            }
            if (m == l) break;
            if (++iter > maxit) { ++nfail; break; }
            double g = (d[l + 1] - d[l]) / (2.0 * ew[l]);
            double r = hypot(g, 1.0);
            g = d[m] - d[l] + ew[l] / (g + copysign(r, g));
            double s = 1.0, c = 1.0, p = 0.0;
            bool early = false;
            int i;
            for (i = m - 1; i >= l; --i) {
                const double f = s * ew[i], bb = c * ew[i];
                r = hypot(f, g);
                __syncthreads();                       // every lane has read ew[i] / d[]
                if (lane == 0) ew[i + 1] = r;
                if (r == 0.0) {
                    if (lane == 0) { d[i + 1] -= p; ew[m] = 0.0; }
                    __syncthreads();
                    early = true;
                    break;
                }
                s = f / r; c = g / r;
                g = d[i + 1] - p;
                r = (d[i] - g) * s + 2.0 * c * bb;
                p = s * r;
                __syncthreads();
                if (lane == 0) d[i + 1] = g + p;
                g = c * r - bb;
                // rotation on columns (i, i+1) of this lane's row
                if (lane < n) {
                    const double zi = Z[i * LEAF + lane], zj = Z[(i + 1) * LEAF + lane];
                    Z[(i + 1) * LEAF + lane] = s * zi + c * zj;
                    Z[i * LEAF + lane] = c * zi - s * zj;
                }
                __syncthreads();
            }
            if (early && i >= l) continue;
            __syncthreads();
            if (lane == 0) { d[l] -= p; ew[l] = g; ew[m] = 0.0; }
            __syncthreads();
        }
    }
    // ascending order (selection sort, columns swapped row-wise by each lane)
    for (int i = 0; i < n - 1; ++i) {
        int k = i;
        for (int j = i + 1; j < n; ++j) if (d[j] < d[k]) k = j;
        __syncthreads();
        if (k != i) {
            if (lane == 0) { const double t = d[i]; d[i] = d[k]; d[k] = t; }
            if (lane < n) {
                const double t = Z[i * LEAF + lane];
                Z[i * LEAF + lane] = Z[k * LEAF + lane];
                Z[k * LEAF + lane] = t;
            }
        }
        __syncthreads();
    }
    if (lane < n) w[a + lane] = d[lane];
    const i64 row = a + lane;
    if (lane < n && row >= r0 && row < r1)
        for (int c = 0; c < n; ++c) Q[(row - r0) + (a + c) * ldq] = Z[c * LEAF + lane];
    if (lane == 0 && nfail) atomicAdd(reinterpret_cast<unsigned long long*>(fails), (unsigned long long)nfail);
}

// Deflation of close poles (Gu-Eisenstat / LAPACK laed2), all runs at once:
// in ascending pole order, a non-deflated pole within tol of the previous
// non-deflated one is rotated into it -- its z weight moves to the later
// pole, the earlier one deflates.  A run of such poles is a sequential chain
// (each rotation uses the accumulated weight); runs are independent, so one
// thread walks each run.  start[t] marks run heads among the nn compacted
// non-deflated positions c[]; for the rotation that pairs c[t-1] with c[t]
// the kernel writes (cs[t], sn[t]) and marks rot[t] = 1; z is updated in
// place and the type bitmask of the surviving column accumulates (bit 0:
// rows of the top half, bit 1: bottom half -- a rotation mixing the halves
// makes the column dense in both, which the split merge GEMM must know).
__global__ void __launch_bounds__(256)
stedc_runs_kernel(i64 nn, const i64* __restrict__ c, const double* __restrict__ dd, double* __restrict__ z,
                  int* __restrict__ ty, double tol, double* __restrict__ cs, double* __restrict__ sn,
                  int* __restrict__ rot, int* __restrict__ keep) {
    const i64 t = (i64)blockIdx.x * 256 + threadIdx.x;
    if (t >= nn) return;
    // rot[] is zeroed by the caller: a per-thread rot[t] = 0 here could land
    // after another wave's run head has set rot[t] = 1
    const bool head = t == 0 || !(dd[c[t]] - dd[c[t - 1]] <= tol);
    if (!head) return;
    double acc = z[c[t]];
    int tacc = ty[c[t]];
    i64 u = t + 1;
    while (u < nn && dd[c[u]] - dd[c[u - 1]] <= tol) {
        const double b = z[c[u]];
        const double r = hypot(acc, b);
        const double cc = r == 0.0 ? 1.0 : b / r, ss = r == 0.0 ? 0.0 : acc / r;
        cs[u] = cc; sn[u] = ss; rot[u] = 1;
        z[c[u - 1]] = 0.0;
        z[c[u]] = r;
        tacc |= ty[c[u]];
        ty[c[u]] = tacc;
        keep[u - 1] = 0;
        acc = r;
        ++u;
    }
    keep[u - 1] = 1;
}

// Givens rotations on column pairs (I[t], J[t]) in order t = 0 .. nrot-1:
// q_I' = c q_I - s q_J, q_J' = s q_I + c q_J, one thread per row.
__global__ void __launch_bounds__(256)
rot_cols_kernel(i64 m, double* __restrict__ Q, i64 ldq, i64 nrot, const i64* __restrict__ I,
                const i64* __restrict__ J, const double* __restrict__ C, const double* __restrict__ S) {
    const i64 r = (i64)blockIdx.x * 256 + threadIdx.x;
    if (r >= m) return;
    for (i64 t = 0; t < nrot; ++t) {
        double* qi = Q + r + I[t] * ldq;
        double* qj = Q + r + J[t] * ldq;
        const double a = *qi, b = *qj, c = C[t], s = S[t];
        *qi = c * a - s * b;
        *qj = s * a + c * b;
    }
}

void steqr_leaves(i64 nleaf, const i64* lo, const i64* hi, const double* d, const double* e, double* w, double* Q,
                  i64 ldq, i64 r0, i64 r1, i64* fails, hipStream_t s, int maxleaf, int maxit) {
    if (nleaf <= 0) return;
    if (maxleaf <= 64) {
        hipLaunchKernelGGL(steqr_leaf_kernel<64>, dim3((unsigned)nleaf), dim3(64), 64 * 64 * sizeof(double), s, lo, hi,
                           d, e, w, Q, ldq, r0, r1, fails, maxit);
    } else {
        if (maxleaf > 128) throw std::invalid_argument("steqr_leaves: leaves of at most 128 rows");
        static bool attr = [] {
            HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(steqr_leaf_kernel<128>),
                                          hipFuncAttributeMaxDynamicSharedMemorySize, 128 * 128 * sizeof(double)));
            return true;
        }();
        (void)attr;
        hipLaunchKernelGGL(steqr_leaf_kernel<128>, dim3((unsigned)nleaf), dim3(128), 128 * 128 * sizeof(double), s, lo,
                           hi, d, e, w, Q, ldq, r0, r1, fails, maxit);
    }
    HIP_LAUNCH_CHECK();
}

void stedc_runs(i64 nn, const i64* c, const double* dd, double* z, int* ty, double tol, double* cs, double* sn,
                int* rot, int* keep, hipStream_t s) {
    if (nn <= 0) return;
    hipLaunchKernelGGL(stedc_runs_kernel, dim3((unsigned)((nn + 255) / 256)), dim3(256), 0, s, nn, c, dd, z, ty, tol,
                       cs, sn, rot, keep);
    HIP_LAUNCH_CHECK();
}

void rot_cols(i64 m, double* Q, i64 ldq, i64 nrot, const i64* I, const i64* J, const double* C, const double* S,
              hipStream_t s) {
    if (m <= 0 || nrot <= 0) return;
    hipLaunchKernelGGL(rot_cols_kernel, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, s, m, Q, ldq, nrot, I, J, C,
                       S);
    HIP_LAUNCH_CHECK();
}

// normalised rank-one eigenvector columns j0 .. j0+nc-1 (chunk of the merge
// GEMM's right operand): V[i + (j - j0) ldv] = zh_i / (d_i - lambda_j) / norm
void stedc_vectors(i64 n, const double* d, const double* zh, const i64* org, const double* mu, i64 j0, i64 nc,
                   double* V, i64 ldv, hipStream_t s) {
    if (n <= 0 || nc <= 0) return;
    hipLaunchKernelGGL(secvec_kernel, dim3((unsigned)nc), dim3(256), 0, s, n, d, zh, org + j0, mu + j0, V, ldv);
    HIP_LAUNCH_CHECK();
}


// ---------------------------------------------------------------------------
// Device-resident merges (one host round trip per tree LEVEL): the sort,
// deflation, Givens runs and every index set of all merges of a level are
// formed on the device; the host reads back one small meta record per merge
// (sizes) and launches the secular solver / split GEMMs with them.  Replaces
// the torch argsort / where / index ops and the two host round trips per
// merge of the former driver (stedc_solve.cc:79-238, laed2 / laed3 roles).
//
// Level arrays (length n, a merge [a, b) uses its own slice):
//   dd, zs, ty   sorted poles, permuted z, column types (1 top, 2 bottom)
//   order        local source column of sorted position
//   c, keep, rot, cs, sn   deflation (compacted non-deflated positions)
//   K, S1, KS1, S2, KS2, D, isK, rI, rJ, rC, rS   compacted index sets
// desc[mi] = (a, m, b, flip); rho[mi] = |rho|; meta[mi] = MergeMeta.
struct MergeMeta {
    i64 nn, k, nrot, n1, n2, nd, pad0, pad1;
    double tol, zzK;
};

namespace {
// v of position t of a child's ascending sequence: [lo, hi) of W, reversed
// and negated when flip
__device__ inline double child_val(const double* W, i64 lo, i64 hi, int flip, i64 t) {
    return flip ? -W[hi - 1 - t] : W[lo + t];
}
// number of elements of the child's sequence < v (strict) or <= v
__device__ inline i64 count_below(const double* W, i64 lo, i64 hi, int flip, double v, bool inclusive) {
    i64 l = 0, h = hi - lo;
    while (l < h) {
        const i64 mid = (l + h) >> 1;
        const double x = child_val(W, lo, hi, flip, mid);
        if (inclusive ? (x <= v) : (x < v)) l = mid + 1;
        else h = mid;
    }
    return l;
}

// exclusive block scan of 0/1 flags for a 1024-thread workgroup; returns the
// prefix of this thread, total in *tot (LDS)
__device__ inline int block_scan_1024(int f, int* s_w, int* tot) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int v = f;
    #pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(v, o, 64);
        if (lane >= o) v += y;
    }
    if (lane == 63) s_w[w] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        int acc = 0;
        for (int i = 0; i < 16; ++i) { const int t = s_w[i]; s_w[i] = acc; acc += t; }
        *tot = acc;
    }
    __syncthreads();
    const int r = s_w[w] + v - f;
    __syncthreads();
    return r;
}
}  // namespace

// sorted merge of the two children (each ascending; both reversed and
// negated when rho < 0): one thread per element, its position = its rank in
// its own child + its co-rank in the other (binary search)
__global__ void __launch_bounds__(256)
stedc_children_kernel(const i64* __restrict__ desc, const double* __restrict__ W, const double* __restrict__ Z,
                      double* __restrict__ dd, double* __restrict__ zs, int* __restrict__ ty, i64* __restrict__ order) {
    const i64* dm = desc + 4 * blockIdx.y;
    const i64 a = dm[0], m = dm[1], b = dm[2];
    const int flip = (int)dm[3];
    const i64 i = (i64)blockIdx.x * 256 + threadIdx.x;
    if (i >= b - a) return;
    const i64 na = m - a;
    i64 pos, orig;
    double v;
    if (i < na) {
        v = child_val(W, a, m, flip, i);
        orig = flip ? m - 1 - i : a + i;
        pos = i + count_below(W, m, b, flip, v, false);
    } else {
        const i64 u = i - na;
        v = child_val(W, m, b, flip, u);
        orig = flip ? b - 1 - u : m + u;
        pos = u + count_below(W, a, m, flip, v, true);
    }
    dd[a + pos] = v;
    zs[a + pos] = Z[orig];
    ty[a + pos] = orig < m ? 1 : 2;
    order[a + pos] = orig - a;
}

// per merge (one 1024-thread workgroup): tolerance, non-deflated positions
__global__ void __launch_bounds__(1024)
stedc_deflate_kernel(const i64* __restrict__ desc, const double* __restrict__ rho, const double* __restrict__ dd,
                     const double* __restrict__ zs, i64* __restrict__ c, MergeMeta* __restrict__ meta) {
    __shared__ double s_a[16], s_b[16];
    __shared__ int s_w[16], s_tot;
    __shared__ double s_tol, s_sq;
    const i64* dm = desc + 4 * blockIdx.x;
    const i64 a = dm[0], s = dm[2] - a;
    const double r = rho[blockIdx.x];
    double mx = 0.0, zz = 0.0;
    for (i64 i = threadIdx.x; i < s; i += 1024) {
        mx = fmax(mx, fabs(dd[a + i]));
        zz += zs[a + i] * zs[a + i];
    }
    mx = wave_max(mx);
    zz = wave_sum(zz);
    if ((threadIdx.x & 63) == 0) { s_a[threadIdx.x >> 6] = mx; s_b[threadIdx.x >> 6] = zz; }
    __syncthreads();
    if (threadIdx.x == 0) {
        double M = 0.0, S = 0.0;
        for (int i = 0; i < 16; ++i) { M = fmax(M, s_a[i]); S += s_b[i]; }
        s_tol = 8.0 * 2.220446049250313e-16 * fmax(M, r * S);
        s_sq = sqrt(S);
    }
    __syncthreads();
    const double tol = s_tol, sq = s_sq;
    i64 base = 0;
    for (i64 i0 = 0; i0 < s; i0 += 1024) {
        const i64 i = i0 + threadIdx.x;
        const int f = (i < s && !(r * fabs(zs[a + i]) * sq <= tol)) ? 1 : 0;
        const int pre = block_scan_1024(f, s_w, &s_tot);
        if (f) c[a + base + pre] = i;
        base += s_tot;
        __syncthreads();
    }
    if (threadIdx.x == 0) { meta[blockIdx.x].nn = base; meta[blockIdx.x].tol = tol; }
}

// close-pole Givens runs of every merge (stedc_runs_kernel on the merge's
// slices, sizes from meta)
__global__ void __launch_bounds__(256)
stedc_runs_level_kernel(const i64* __restrict__ desc, const MergeMeta* __restrict__ meta, const i64* __restrict__ c,
                        const double* __restrict__ dd, double* __restrict__ zs, int* __restrict__ ty,
                        double* __restrict__ cs, double* __restrict__ sn, int* __restrict__ rot,
                        int* __restrict__ keep) {
    const i64 a = desc[4 * blockIdx.y];
    const i64 nn = meta[blockIdx.y].nn;
    const double tol = meta[blockIdx.y].tol;
    const i64 t = (i64)blockIdx.x * 256 + threadIdx.x;
    if (t >= nn) return;
    const i64* cc = c + a;
    const double* d = dd + a;
    double* z = zs + a;
    int* tt = ty + a;
    const bool head = t == 0 || !(d[cc[t]] - d[cc[t - 1]] <= tol);    // rot[] zeroed by the caller
    if (!head) return;
    double acc = z[cc[t]];
    int tacc = tt[cc[t]];
    i64 u = t + 1;
    while (u < nn && d[cc[u]] - d[cc[u - 1]] <= tol) {
        const double bb = z[cc[u]];
        const double rr = hypot(acc, bb);
        cs[a + u] = rr == 0.0 ? 1.0 : bb / rr;
        sn[a + u] = rr == 0.0 ? 0.0 : acc / rr;
        rot[a + u] = 1;
        z[cc[u - 1]] = 0.0;
        z[cc[u]] = rr;
        tacc |= tt[cc[u]];
        tt[cc[u]] = tacc;
        keep[a + u - 1] = 0;
        acc = rr;
        ++u;
    }
    keep[a + u - 1] = 1;
}

// per merge (one 1024-thread workgroup): compacted index sets and sizes
__global__ void __launch_bounds__(1024)
stedc_compact_kernel(const i64* __restrict__ desc, MergeMeta* __restrict__ meta, const i64* __restrict__ c,
                     const int* __restrict__ keep, const int* __restrict__ rot, const double* __restrict__ cs,
                     const double* __restrict__ sn, const int* __restrict__ ty, const double* __restrict__ zs,
                     i64* __restrict__ K, i64* __restrict__ S1, i64* __restrict__ KS1, i64* __restrict__ S2,
                     i64* __restrict__ KS2, i64* __restrict__ D, i64* __restrict__ isK, i64* __restrict__ rI,
                     i64* __restrict__ rJ, double* __restrict__ rC, double* __restrict__ rS) {
    __shared__ int s_w[16], s_tot;
    __shared__ double s_z[16];
    const i64* dm = desc + 4 * blockIdx.x;
    const i64 a = dm[0], s = dm[2] - a;
    const i64 nn = meta[blockIdx.x].nn;
    for (i64 i = threadIdx.x; i < s; i += 1024) isK[a + i] = 0;
    __syncthreads();
    i64 kb = 0, b1 = 0, b2 = 0, br = 0;
    double zz = 0.0;
    for (i64 t0 = 0; t0 < nn; t0 += 1024) {
        const i64 t = t0 + threadIdx.x;
        const bool live = t < nn;
        const i64 col = live ? c[a + t] : 0;
        const int kf = live && keep[a + t] ? 1 : 0;
        const int tyv = kf ? ty[a + col] : 0;
        const int rf = live && rot[a + t] ? 1 : 0;
        const int pk = block_scan_1024(kf, s_w, &s_tot);
        const int nk = s_tot;
        const int f1 = (tyv & 1) ? 1 : 0, f2 = (tyv & 2) ? 1 : 0;
        const int p1 = block_scan_1024(f1, s_w, &s_tot);
        const int n1 = s_tot;
        const int p2 = block_scan_1024(f2, s_w, &s_tot);
        const int n2 = s_tot;
        const int pr = block_scan_1024(rf, s_w, &s_tot);
        const int nr = s_tot;
        if (kf) {
            const i64 j = kb + pk;
            K[a + j] = col;
            isK[a + col] = j + 1;
            zz += zs[a + col] * zs[a + col];
            if (f1) { S1[a + b1 + p1] = j; KS1[a + b1 + p1] = col; }
            if (f2) { S2[a + b2 + p2] = j; KS2[a + b2 + p2] = col; }
        }
        if (rf) {
            const i64 q = br + pr;
            rI[a + q] = c[a + t - 1];
            rJ[a + q] = col;
            rC[a + q] = cs[a + t];
            rS[a + q] = sn[a + t];
        }
        kb += nk; b1 += n1; b2 += n2; br += nr;
    }
    zz = wave_sum(zz);
    if ((threadIdx.x & 63) == 0) s_z[threadIdx.x >> 6] = zz;
    __syncthreads();
    // deflated positions (not in K), ascending
    i64 bd = 0;
    for (i64 i0 = 0; i0 < s; i0 += 1024) {
        const i64 i = i0 + threadIdx.x;
        const int f = (i < s && isK[a + i] == 0) ? 1 : 0;
        const int pre = block_scan_1024(f, s_w, &s_tot);
        if (f) D[a + bd + pre] = i;
        bd += s_tot;
    }
    if (threadIdx.x == 0) {
        double z2 = 0.0;
        for (int i = 0; i < 16; ++i) z2 += s_z[i];
        MergeMeta& M = meta[blockIdx.x];
        M.k = kb; M.n1 = b1; M.n2 = b2; M.nrot = br; M.nd = bd; M.zzK = z2;
    }
}

// lam_i = root of K position (isK - 1) or the deflated pole dd_i; negated
// when flip; the roots (K order) and the deflated poles (D order) are both
// ascending before negation: the final order is their merge
__global__ void __launch_bounds__(256)
stedc_lambda_kernel(i64 s, const double* __restrict__ dd, const i64* __restrict__ isK, const double* __restrict__ dK,
                    const i64* __restrict__ org, const double* __restrict__ mu, int flip, double* __restrict__ lam) {
    const i64 i = (i64)blockIdx.x * 256 + threadIdx.x;
    if (i >= s) return;
    const i64 j = isK[i] - 1;
    const double v = j >= 0 ? dK[org[j]] + mu[j] : dd[i];
    lam[i] = flip ? -v : v;
}

__device__ inline double list_val(const double* lam, const i64* L, i64 n, int rev, i64 t) {
    return lam[L[rev ? n - 1 - t : t]];
}
__device__ inline i64 list_count(const double* lam, const i64* L, i64 n, int rev, double v, bool inclusive) {
    i64 l = 0, h = n;
    while (l < h) {
        const i64 mid = (l + h) >> 1;
        const double x = list_val(lam, L, n, rev, mid);
        if (inclusive ? (x <= v) : (x < v)) l = mid + 1;
        else h = mid;
    }
    return l;
}

// merge of two index lists, each ascending in lam (descending when rev):
// out[pos] = index
__global__ void __launch_bounds__(256)
stedc_merge2_kernel(const double* __restrict__ lam, const i64* __restrict__ L1, i64 n1, const i64* __restrict__ L2,
                    i64 n2, int rev, i64* __restrict__ out) {
    const i64 i = (i64)blockIdx.x * 256 + threadIdx.x;
    if (i >= n1 + n2) return;
    if (i < n1) {
        const double v = list_val(lam, L1, n1, rev, i);
        out[i + list_count(lam, L2, n2, rev, v, false)] = L1[rev ? n1 - 1 - i : i];
    } else {
        const i64 u = i - n1;
        const double v = list_val(lam, L2, n2, rev, u);
        out[u + list_count(lam, L1, n1, rev, v, true)] = L2[rev ? n2 - 1 - u : u];
    }
}

// B[:, j] = A[:, idx[j]] (gather) or B[:, idx[j]] = A[:, j] (scatter)
__global__ void __launch_bounds__(256)
cols_copy_kernel(i64 m, i64 nc, const double* __restrict__ A, i64 lda, const i64* __restrict__ idx,
                 double* __restrict__ B, i64 ldb, int scatter) {
    const i64 r = (i64)blockIdx.x * 256 + threadIdx.x;
    if (r >= m) return;
    for (i64 j = blockIdx.y; j < nc; j += gridDim.y) {
        if (scatter) B[r + idx[j] * ldb] = A[r + j * lda];
        else B[r + j * ldb] = A[r + idx[j] * lda];
    }
}

// y[j] = x[idx[j]] (+ offset table for the eigenvalues)
__global__ void __launch_bounds__(256)
vec_gather_kernel(i64 n, const double* __restrict__ x, const i64* __restrict__ idx, double* __restrict__ y) {
    const i64 j = (i64)blockIdx.x * 256 + threadIdx.x;
    if (j < n) y[j] = x[idx[j]];
}

void stedc_level_prep(i64 n, i64 nm, i64 maxs, const i64* desc, const double* rho, const double* W, const double* Z,
                      double* dd, double* zs, int* ty, i64* order, i64* c, int* keep, int* rot, double* cs,
                      double* sn, void* meta, i64* K, i64* S1, i64* KS1, i64* S2, i64* KS2, i64* D, i64* isK,
                      i64* rI, i64* rJ, double* rC, double* rS, hipStream_t s) {
    if (nm <= 0 || maxs <= 0) return;
    MergeMeta* M = static_cast<MergeMeta*>(meta);
    HIP_CHECK(hipMemsetAsync(rot, 0, sizeof(int) * (size_t)n, s));
    const unsigned gx = (unsigned)((maxs + 255) / 256);
    hipLaunchKernelGGL(stedc_children_kernel, dim3(gx, (unsigned)nm), dim3(256), 0, s, desc, W, Z, dd, zs, ty, order);
    HIP_LAUNCH_CHECK();
    hipLaunchKernelGGL(stedc_deflate_kernel, dim3((unsigned)nm), dim3(1024), 0, s, desc, rho, dd, zs, c, M);
    HIP_LAUNCH_CHECK();
    hipLaunchKernelGGL(stedc_runs_level_kernel, dim3(gx, (unsigned)nm), dim3(256), 0, s, desc, M, c, dd, zs, ty, cs,
                       sn, rot, keep);
    HIP_LAUNCH_CHECK();
    hipLaunchKernelGGL(stedc_compact_kernel, dim3((unsigned)nm), dim3(1024), 0, s, desc, M, c, keep, rot, cs, sn, ty,
                       zs, K, S1, KS1, S2, KS2, D, isK, rI, rJ, rC, rS);
    HIP_LAUNCH_CHECK();
}
size_t stedc_meta_bytes() { return sizeof(MergeMeta); }

void stedc_lambda(i64 s, const double* dd, const i64* isK, const double* dK, const i64* org, const double* mu,
                  int flip, double* lam, hipStream_t st) {
    if (s <= 0) return;
    hipLaunchKernelGGL(stedc_lambda_kernel, dim3((unsigned)((s + 255) / 256)), dim3(256), 0, st, s, dd, isK, dK, org,
                       mu, flip, lam);
    HIP_LAUNCH_CHECK();
}

void stedc_merge2(const double* lam, const i64* L1, i64 n1, const i64* L2, i64 n2, int rev, i64* out,
                  hipStream_t st) {
    if (n1 + n2 <= 0) return;
    hipLaunchKernelGGL(stedc_merge2_kernel, dim3((unsigned)((n1 + n2 + 255) / 256)), dim3(256), 0, st, lam, L1, n1,
                       L2, n2, rev, out);
    HIP_LAUNCH_CHECK();
}

void cols_copy(i64 m, i64 nc, const double* A, i64 lda, const i64* idx, double* B, i64 ldb, bool scatter,
               hipStream_t st) {
    if (m <= 0 || nc <= 0) return;
    hipLaunchKernelGGL(cols_copy_kernel, dim3((unsigned)((m + 255) / 256), (unsigned)std::min<i64>(nc, 4096)),
                       dim3(256), 0, st, m, nc, A, lda, idx, B, ldb, scatter ? 1 : 0);
    HIP_LAUNCH_CHECK();
}

void vec_gather(i64 n, const double* x, const i64* idx, double* y, hipStream_t st) {
    if (n <= 0) return;
    hipLaunchKernelGGL(vec_gather_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, n, x, idx, y);
    HIP_LAUNCH_CHECK();
}

}  // namespace slate_hip
