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

}  // namespace slate_hip
