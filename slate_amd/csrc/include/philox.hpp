// Counter-based Philox4x32-10 generator shared by the host runtime and the
// gfx950 matgen kernel, so a matrix entry depends only on (seed, global i,
// global j) and never on the distribution, grid or device
// (same contract as SLATE's matgen, matgen/random.cc:36-60).
#pragma once
#include <stdint.h>
#include <math.h>

#if defined(__HIPCC__) || defined(__HIP__)
#define SLATE_HD __host__ __device__ inline
#else
#define SLATE_HD inline
#endif

namespace slate_rng {

struct u32x4 { uint32_t v[4]; };

SLATE_HD void mulhilo(uint32_t a, uint32_t b, uint32_t& hi, uint32_t& lo) {
    uint64_t p = (uint64_t)a * (uint64_t)b;
    hi = (uint32_t)(p >> 32);
    lo = (uint32_t)p;
}

SLATE_HD u32x4 philox4x32(u32x4 c, uint32_t k0, uint32_t k1) {
    const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
    const uint32_t W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
    for (int r = 0; r < 10; ++r) {
        uint32_t hi0, lo0, hi1, lo1;
        mulhilo(M0, c.v[0], hi0, lo0);
        mulhilo(M1, c.v[2], hi1, lo1);
        u32x4 n;
        n.v[0] = hi1 ^ c.v[1] ^ k0;
        n.v[1] = lo1;
        n.v[2] = hi0 ^ c.v[3] ^ k1;
        n.v[3] = lo0;
        c = n;
        k0 += W0; k1 += W1;
    }
    return c;
}

// Two uniform doubles in [0, 1) with 53 random bits each for entry (i, j).
SLATE_HD void uniform2(uint64_t seed, int64_t i, int64_t j, uint32_t stream, double& u0, double& u1) {
    u32x4 c;
    c.v[0] = (uint32_t)i; c.v[1] = (uint32_t)((uint64_t)i >> 32);
    c.v[2] = (uint32_t)j; c.v[3] = (uint32_t)((uint64_t)j >> 32) ^ (stream << 24);
    u32x4 r = philox4x32(c, (uint32_t)seed, (uint32_t)(seed >> 32));
    uint64_t a = ((uint64_t)r.v[0] << 21) ^ (uint64_t)r.v[1];
    uint64_t b = ((uint64_t)r.v[2] << 21) ^ (uint64_t)r.v[3];
    u0 = (double)(a & ((1ull << 53) - 1)) * (1.0 / 9007199254740992.0);
    u1 = (double)(b & ((1ull << 53) - 1)) * (1.0 / 9007199254740992.0);
}

// Distribution kinds (subset of SLATE's generate_matrix kinds).
enum Kind : int {
    kZeros = 0, kOnes = 1, kIdentity = 2, kIJ = 3, kJordan = 4,
    kRand = 10,    // uniform [0,1)
    kRands = 11,   // uniform [-1,1)
    kRandn = 12,   // standard normal
    kRandb = 13,   // 0/1
    kRandr = 14,   // +-1
    kRandsDominant = 20,   // rands + n*I (general, diagonally dominant)
    kPoev = 21,            // Hermitian rands + n*I (HPD)
    kHeRands = 22,         // Hermitian rands (indefinite)
    kMinij = 30, kHilb = 31, kLehmer = 32, kFrank = 33, kMoler = 34,
    // Matlab-gallery test matrices (SLATE matgen/generate_matrix_ge.cc kinds)
    kJordanT = 40, kChebspec = 41, kCircul = 42, kFiedler = 43, kGfpp = 44, kKms = 45, kOrthog = 46,
    kRiemann = 47, kRis = 48, kZielkeNS = 49, kLotkin = 50, kRedheff = 51, kTriw = 52, kPei = 53,
    kTridiag = 54, kToeppen = 55, kParter = 56, kCauchy = 57, kChow = 58, kClement = 59, kGcdmat = 60,
};

SLATE_HD int64_t gcd64(int64_t a, int64_t b) {
    while (b) { const int64_t t = a % b; a = b; b = t; }
    return a;
}

// Closed-form gallery entries (0-based i, j; N = max(m, n)); false if kind
// is not a gallery kind.
SLATE_HD bool gallery(int kind, int64_t i, int64_t j, int64_t m, int64_t n, double& re) {
    const int64_t N = m > n ? m : n;
    const int64_t d = i - j;
    const double pi = 3.141592653589793;
    switch (kind) {
        case kJordanT: re = (d == 0 || d == 1) ? 1.0 : 0.0; return true;
        case kChebspec: {
            // Chebyshev spectral differentiation on the points cos(pi (k+1) / N)
            const double xi = cos(pi * (double)(i + 1) / (double)N), xj = cos(pi * (double)(j + 1) / (double)N);
            if (i != j) {
                const double ci = (i == N - 1) ? 2.0 : 1.0, cj = (j == N - 1) ? 2.0 : 1.0;
                re = (((i + j) & 1) ? -1.0 : 1.0) * ci / (cj * (xj - xi));
            } else if (j == N - 1) {
                re = -(double)(2 * N * N + 1) / 6.0;
            } else {
                re = -0.5 * xi / (1.0 - xi * xi);
            }
            return true;
        }
        case kCircul: re = (double)(((j - i) % N + N) % N + 1); return true;
        case kFiedler: re = (double)(d < 0 ? -d : d); return true;
        case kGfpp: re = (j == n - 1) ? 1.0 : (d > 0 ? -1.0 : (d == 0 ? 0.5 : 0.0)); return true;
        case kKms: re = pow(0.5, (double)(d < 0 ? -d : d)); return true;
        case kOrthog: re = sqrt(2.0 / (double)(N + 1)) * sin((double)(i + 1) * (double)(j + 1) * pi / (double)(N + 1));
            return true;
        case kRiemann: re = ((j + 2) % (i + 2) == 0) ? (double)(j + 1) : -1.0; return true;
        case kRis: re = 0.5 / ((double)N - (double)i - (double)j - 0.5); return true;
        case kZielkeNS: re = (j < i) ? 1.0 : ((i == 0 && j == N - 1) ? -1.0 : 0.0); return true;
        case kLotkin: re = (i == 0) ? 1.0 : 1.0 / (double)(i + j + 1); return true;
        case kRedheff: re = (j == 0 || (j + 1) % (i + 1) == 0) ? 1.0 : 0.0; return true;
        case kTriw: re = (d == 0) ? 1.0 : (d > 0 ? 0.0 : -1.0); return true;
        case kPei: re = (d == 0) ? 2.0 : 1.0; return true;
        case kTridiag: re = (d == 0) ? 2.0 : ((d == 1 || d == -1) ? -1.0 : 0.0); return true;
        case kToeppen: re = (d == -1) ? 10.0 : (d == 1 ? -10.0 : ((d == 2 || d == -2) ? 1.0 : 0.0)); return true;
        case kParter: re = 1.0 / ((double)d + 0.5); return true;
        case kCauchy: re = 1.0 / (double)(i + j + 2); return true;
        case kChow: re = (d < -1) ? 0.0 : 1.0; return true;
        case kClement: re = (d == 1) ? (double)(N - j - 1) : (d == -1 ? (double)j : 0.0); return true;
        case kGcdmat: re = (double)gcd64(i + 1, j + 1); return true;
        default: return false;
    }
}

// Real and imaginary parts of entry (gi, gj) of an n x n (or m x n) matrix.
SLATE_HD void entry(int kind, uint64_t seed, int64_t gi, int64_t gj, int64_t m, int64_t n,
                    bool is_complex, double& re, double& im) {
    re = 0; im = 0;
    switch (kind) {
        case kZeros: return;
        case kOnes: re = 1; return;
        case kIdentity: re = (gi == gj) ? 1.0 : 0.0; return;
        case kIJ: {
            // i + j s with s = 10^-ceil(log10 n): the column index in the fraction
            double sc = 1.0;
            for (int64_t t = 1; t < n; t *= 10) sc *= 0.1;
            re = (double)gi + (double)gj * sc; return;
        }
        case kJordan: re = (gi == gj) ? 1.0 : (gi + 1 == gj ? 1.0 : 0.0); return;
        case kMinij: re = (double)((gi < gj ? gi : gj) + 1); return;
        case kHilb: re = 1.0 / (double)(gi + gj + 1); return;
        case kLehmer: { double a = gi + 1, b = gj + 1; re = (a < b) ? a / b : b / a; return; }
        case kFrank: { int64_t nn = n; int64_t ii = gi + 1, jj = gj + 1;
            re = (jj >= ii - 1) ? (double)(nn + 1 - (ii > jj ? ii : jj)) : 0.0; return; }
        case kMoler: { double mn = (double)((gi < gj ? gi : gj) + 1);
            re = (gi == gj) ? mn : mn - 2.0; return; }
        default:
            if (gallery(kind, gi, gj, m, n, re)) return;
            break;
    }
    bool herm = (kind == kPoev || kind == kHeRands);
    int64_t ci = gi, cj = gj;
    bool swapped = false;
    if (herm && gi < gj) { ci = gj; cj = gi; swapped = true; }
    double u0, u1;
    uniform2(seed, ci, cj, 0, u0, u1);
    switch (kind) {
        case kRand: re = u0; im = u1; break;
        case kRands: case kRandsDominant: case kPoev: case kHeRands:
            re = 2 * u0 - 1; im = 2 * u1 - 1; break;
        case kRandn: {
            double r = sqrt(-2.0 * log(u0 > 0 ? u0 : 1e-300));
            re = r * cos(6.283185307179586 * u1); im = r * sin(6.283185307179586 * u1); break;
        }
        case kRandb: re = u0 < 0.5 ? 0 : 1; im = u1 < 0.5 ? 0 : 1; break;
        case kRandr: re = u0 < 0.5 ? -1 : 1; im = u1 < 0.5 ? -1 : 1; break;
        default: break;
    }
    if (!is_complex) im = 0;
    if (herm) {
        if (gi == gj) im = 0;
        else if (swapped) im = -im;
    }
    if ((kind == kRandsDominant || kind == kPoev) && gi == gj) {
        re += (double)(m > n ? m : n);
    }
}

}  // namespace slate_rng
