// Native band matrices and drivers (include/slate_amd/slate_native.hh, "band
// matrices"): gbtrf / gbtrs / gbsv, pbtrf / pbtrs / pbsv, tbsm, gbmm, hbmm.
// Reference: src/gbtrf.cc:20-348 (panel + band-limited trailing update, the
// upper bandwidth grows to kl + ku), src/gbtrs.cc, src/pbtrf.cc,
// src/pbtrs.cc, src/tbsm.cc, src/gbmm.cc, src/hbmm.cc; the Python twin is
// slate_amd/models/band.py (same compact storage).
//
// Storage: tile columns are dealt 1-D cyclically over ALL ranks (column
// tile k on rank k % size); a local tile column is ONE contiguous device
// slab of H = (klt + kut + 1) nb rows (global rows (k - kut) nb ...
// (k + klt + 1) nb), column-major with leading dimension H, so a panel and
// every update of a step are plain strided blocks of one slab -- the
// factorizations run on the same gfx950 kernels as the dense drivers
// (potrf_fast / potrf_tile, the persistent LU panel, trsm, the MFMA GEMM).
// Per step: the panel on its owner, ONE broadcast of the panel (+ pivots)
// over the world communicator, then each rank updates its own tile columns
// inside the band window.  The dense operands of solves and products are
// replicated on every rank (device buffer, host-staged in and out), so a
// solve step is the owner's tile work plus one broadcast of the window of
// kb + bandwidth rows.
#include <algorithm>
#include <cmath>
#include <vector>

#include "../hip/kernels.hpp"
#include "native_rt.hpp"

namespace slate_amd {
namespace native {

struct BandStorage {
    i64 m = 0, n = 0, nb = 1, kl = 0, ku = 0;   // logical bandwidths
    i64 klt = 0, kut = 0;                       // tiles stored below / above the diagonal tile
    i64 mt = 0, nt = 0, H = 0;
    int rank = 0, size = 1;
    size_t esize = 8;
    i64 ncl = 0;                                // local tile columns
    void* buf = nullptr;
    ~BandStorage() {
        if (buf) (void)hipFree(buf);
    }
    int owner(i64 k) const { return (int)(k % size); }
    bool mine(i64 k) const { return owner(k) == rank; }
    i64 row0(i64 k) const { return (k - kut) * nb; }               // global row of slab row 0
    i64 rlo(i64 k) const { return std::max<i64>(0, row0(k)); }
    i64 rhi(i64 k) const { return std::min(m, (k + klt + 1) * nb); }
    i64 kb(i64 k) const { return std::min(nb, n - k * nb); }
    template <typename T> T* slab(i64 k) const { return static_cast<T*>(buf) + (k / size) * H * nb; }
    // global element (i, k nb) of column tile k
    template <typename T> T* at(i64 k, i64 i) const { return slab<T>(k) + (i - row0(k)); }
};

namespace {

template <typename KT>
__global__ void band_mask_kernel(i64 rows, i64 cols, KT* A, i64 lda, i64 gi0, i64 gj0, i64 kl, i64 ku) {
    const i64 r = (i64)blockIdx.x * 256 + threadIdx.x;
    if (r >= rows) return;
    for (i64 c = blockIdx.y; c < cols; c += gridDim.y) {
        const i64 i = gi0 + r, j = gj0 + c;
        if (i - j > kl || j - i > ku) A[r + c * lda] = slate_hip::s_from_real(KT(), 0);
    }
}

// zero the entries of a slab block outside the band (global origin gi0, gj0)
template <typename T>
void band_mask(i64 rows, i64 cols, T* A, i64 lda, i64 gi0, i64 gj0, i64 kl, i64 ku, hipStream_t s) {
    if (rows <= 0 || cols <= 0) return;
    hipLaunchKernelGGL(band_mask_kernel<K<T>>, dim3((unsigned)((rows + 255) / 256), (unsigned)std::min<i64>(cols, 1024)),
                       dim3(256), 0, s, rows, cols, kp(A), lda, gi0, gj0, kl, ku);
}

// tile Cholesky of the diagonal tile (the dense drivers' kernels)
template <typename T>
void potrf_tile(i64 n, T* A, i64 lda, i64* info, hipStream_t s) {
    if constexpr (std::is_same<T, double>::value)
        if (slate_hip::potrf_fast((int)n, A, lda, info, 0, s)) return;
    slate_hip::potrf_tile<K<T>>('L', (int)n, kp(A), lda, info, s);
}

template <typename T>
void trsm_k(char side, char uplo, char tr, char diag, i64 m, i64 n, T alpha, const T* A, i64 lda, T* B, i64 ldb,
            hipStream_t s) {
    if (m <= 0 || n <= 0) return;
    slate_hip::trsm<K<T>>(side, uplo, tr, diag, m, n, kv(alpha), kp(A), lda, kp(B), ldb, s);
}

// rows [r0, r1) of the replicated n x nrhs X (ld ldx) from `root` to every rank
template <typename T>
void bcast_rows(T* X, i64 ldx, i64 r0, i64 r1, i64 nrhs, int root, hipStream_t s) {
    Runtime& R = rt();
    if (R.size == 1 || r1 <= r0 || nrhs <= 0) return;
    const i64 h = r1 - r0;
    Scratch W(sizeof(T) * h * nrhs, s);
    if (R.rank == root) copy2d(W.as<T>(), h, X + r0, ldx, h, nrhs, s);
    world_comm()->bcast(W.p, sizeof(T) * h * nrhs, root, s);
    if (R.rank != root) copy2d(X + r0, ldx, W.as<T>(), h, h, nrhs, s);
}

// a dense native matrix <-> a replicated device copy (ld = rows)
template <typename T>
struct Replica {
    i64 rows = 0, cols = 0;
    Scratch d;
    Replica(const Matrix<T>& B, hipStream_t s)
        : rows(B.m()), cols(B.n()), d(sizeof(T) * std::max<i64>(1, B.m() * B.n()), s) {
        std::vector<T> h((size_t)std::max<i64>(1, rows * cols));
        B.to_host(h.data(), std::max<i64>(rows, 1));
        upload(d.p, h.data(), sizeof(T) * rows * cols, s);
    }
    T* p() { return d.as<T>(); }
    void to(Matrix<T>& B, hipStream_t s) {
        std::vector<T> h((size_t)std::max<i64>(1, rows * cols));
        NHIP(hipMemcpyAsync(h.data(), d.p, sizeof(T) * rows * cols, hipMemcpyDeviceToHost, s));
        NHIP(hipStreamSynchronize(s));
        B.from_host(h.data(), std::max<i64>(rows, 1));
    }
};

// first failing step over all ranks: info = k nb + tile info (LAPACK), 0 if none
int64_t band_info(const Scratch& infos, i64 nt, i64 nb, const BandStorage& S, hipStream_t s) {
    std::vector<i64> h((size_t)std::max<i64>(nt, 1));
    NHIP(hipMemcpyAsync(h.data(), infos.p, sizeof(i64) * h.size(), hipMemcpyDeviceToHost, s));
    NHIP(hipStreamSynchronize(s));
    double first = 1e300;
    for (i64 k = 0; k < nt; ++k)
        if (S.mine(k) && h[k] > 0) {
            first = (double)(k * nb + h[k]);
            break;
        }
    const double g = -allreduce_max(-first);
    return g >= 1e299 ? 0 : (int64_t)g;
}

}  // namespace

// ------------------------------------------------------------ matrices
template <typename T>
BandMatrix<T>::BandMatrix(int64_t m, int64_t n, int64_t kl, int64_t ku, int64_t nb, int64_t ku_alloc) {
    initialize();
    if (m < 0 || n < 0 || kl < 0 || ku < 0 || nb <= 0) throw Error("BandMatrix: bad dimensions");
    auto s = std::make_shared<BandStorage>();
    Runtime& R = rt();
    s->m = m; s->n = n; s->nb = nb; s->kl = kl; s->ku = ku;
    s->klt = (kl + nb - 1) / nb;
    s->kut = (std::max(ku, ku_alloc) + nb - 1) / nb;
    s->mt = (m + nb - 1) / nb;
    s->nt = (n + nb - 1) / nb;
    s->H = (s->klt + s->kut + 1) * nb;
    s->rank = R.rank;
    s->size = R.size;
    s->esize = sizeof(T);
    s->ncl = s->nt > R.rank ? (s->nt - R.rank + R.size - 1) / R.size : 0;
    const size_t bytes = sizeof(T) * (size_t)std::max<i64>(1, s->ncl) * s->H * nb;
    NHIP(hipMalloc(&s->buf, bytes));
    dzero(s->buf, bytes, R.main);
    NHIP(hipStreamSynchronize(R.main));
    s_ = s;
}
// a general band matrix has room for the gbtrf fill (upper bandwidth kl + ku)
template <typename T>
BandMatrix<T>::BandMatrix(int64_t m, int64_t n, int64_t kl, int64_t ku, int64_t nb)
    : BandMatrix(m, n, kl, ku, nb, kl + ku) {}
template <typename T> int64_t BandMatrix<T>::m() const { return s_->m; }
template <typename T> int64_t BandMatrix<T>::n() const { return s_->n; }
template <typename T> int64_t BandMatrix<T>::nb() const { return s_->nb; }
template <typename T> int64_t BandMatrix<T>::lower_bandwidth() const { return s_->kl; }
template <typename T> int64_t BandMatrix<T>::upper_bandwidth() const { return s_->ku; }

// fill my slabs from a host element function f(i, j) (band entries only)
template <typename T, typename F>
static void fill_slabs(BandStorage& S, F&& f) {
    hipStream_t s = rt().main;
    std::vector<T> h((size_t)S.H * S.nb);
    for (i64 k = S.rank; k < S.nt; k += S.size) {
        std::fill(h.begin(), h.end(), T(0));
        for (i64 c = 0; c < S.kb(k); ++c) {
            const i64 j = k * S.nb + c;
            for (i64 i = S.rlo(k); i < S.rhi(k); ++i)
                if (i - j <= S.kl && j - i <= S.ku) h[(size_t)(i - S.row0(k)) + (size_t)c * S.H] = f(i, j);
        }
        upload(S.slab<T>(k), h.data(), sizeof(T) * h.size(), s);
    }
}

// every rank's band entries into a dense host array on every rank
template <typename T, typename F>
static void gather_slabs(const BandStorage& S, T* A, int64_t lda, i64 rows, i64 cols, F&& put) {
    hipStream_t s = rt().main;
    std::vector<T> full((size_t)std::max<i64>(1, rows * cols), T(0));
    std::vector<T> h((size_t)S.H * S.nb);
    for (i64 k = S.rank; k < S.nt; k += S.size) {
        NHIP(hipMemcpyAsync(h.data(), S.slab<T>(k), sizeof(T) * h.size(), hipMemcpyDeviceToHost, s));
        NHIP(hipStreamSynchronize(s));
        for (i64 c = 0; c < S.kb(k); ++c) {
            const i64 j = k * S.nb + c;
            for (i64 i = S.rlo(k); i < S.rhi(k); ++i)
                if (i - j <= S.kl && j - i <= S.ku) put(full, i, j, h[(size_t)(i - S.row0(k)) + (size_t)c * S.H]);
        }
    }
    if (S.size > 1 && rows * cols > 0) {
        Scratch d(sizeof(T) * full.size(), s);
        upload(d.p, full.data(), sizeof(T) * full.size(), s);
        world_comm()->allreduce(d.p, full.size(), dt_of<T>::v, 's', s);
        NHIP(hipMemcpyAsync(full.data(), d.p, sizeof(T) * full.size(), hipMemcpyDeviceToHost, s));
        NHIP(hipStreamSynchronize(s));
    }
    for (i64 j = 0; j < cols; ++j)
        for (i64 i = 0; i < rows; ++i) A[i + j * lda] = full[(size_t)(i + j * rows)];
}

template <typename T>
void BandMatrix<T>::from_host(const T* A, int64_t lda) {
    fill_slabs<T>(*s_, [&](i64 i, i64 j) { return A[i + j * lda]; });
}
template <typename T>
void BandMatrix<T>::from_host_band(const T* AB, int64_t ldab, int64_t off) {
    fill_slabs<T>(*s_, [&](i64 i, i64 j) { return AB[(off + i - j) + j * ldab]; });
}
template <typename T>
void BandMatrix<T>::to_host(T* A, int64_t lda) const {
    const BandStorage& S = *s_;
    gather_slabs<T>(S, A, lda, S.m, S.n, [&](std::vector<T>& f, i64 i, i64 j, T v) { f[(size_t)(i + j * S.m)] = v; });
}
template <typename T>
void BandMatrix<T>::generate(Gen kind, uint64_t seed) {
    BandStorage& S = *s_;
    hipStream_t s = rt().main;
    const i64 big = (i64)1 << 40;
    for (i64 k = S.rank; k < S.nt; k += S.size) {
        const i64 r0 = S.rlo(k), rows = S.rhi(k) - r0, kb = S.kb(k);
        T* p = S.at<T>(k, r0);
        slate_hip::matgen<K<T>>((int)kind, seed, rows, kb, kp(p), S.H, S.m, S.n, big, 1, 0, big, 1, 0, r0, k * S.nb,
                                1.0, s);
        band_mask<T>(rows, kb, p, S.H, r0, k * S.nb, S.kl, S.ku, s);
    }
    NHIP(hipStreamSynchronize(s));
}

template <typename T>
HermitianBandMatrix<T>::HermitianBandMatrix(Uplo uplo, int64_t n, int64_t kd, int64_t nb)
    : BandMatrix<T>(n, n, kd, 0, nb, 0), uplo_(uplo) {}
// Upper: the lower band holds the conjugate transpose of the upper one
template <typename T>
void HermitianBandMatrix<T>::from_host(const T* A, int64_t lda) {
    if (uplo_ == Uplo::Lower) fill_slabs<T>(*this->s_, [&](i64 i, i64 j) { return A[i + j * lda]; });
    else fill_slabs<T>(*this->s_, [&](i64 i, i64 j) { return conj_of(A[j + i * lda]); });
}
template <typename T>
void HermitianBandMatrix<T>::to_host(T* A, int64_t lda) const {
    const BandStorage& S = *this->s_;
    const bool up = uplo_ == Uplo::Upper;
    gather_slabs<T>(S, A, lda, S.m, S.n, [&](std::vector<T>& f, i64 i, i64 j, T v) {
        if (up) f[(size_t)(j + i * S.m)] = conj_of(v);
        else f[(size_t)(i + j * S.m)] = v;
    });
}
template <typename T>
TriangularBandMatrix<T>::TriangularBandMatrix(Uplo uplo, Diag diag, int64_t n, int64_t kd, int64_t nb)
    : BandMatrix<T>(n, n, uplo == Uplo::Lower ? kd : 0, uplo == Uplo::Upper ? kd : 0, nb,
                    uplo == Uplo::Upper ? kd : 0),
      uplo_(uplo), diag_(diag) {}

// ------------------------------------------------------------ Cholesky
template <typename T>
int64_t pbtrf(HermitianBandMatrix<T>& A, const Options&) {
    NTRACE("pbtrf", nullptr);
    BandStorage& S = *A.storage();
    hipStream_t s = rt().main;
    const i64 n = S.n, nb = S.nb, nt = S.nt, H = S.H;
    const char ct = ctrans<T>();
    Scratch infos(sizeof(i64) * std::max<i64>(nt, 1), s);
    dzero(infos.p, sizeof(i64) * std::max<i64>(nt, 1), s);
    Scratch P(sizeof(T) * (S.klt + 1) * nb * nb, s);
    for (i64 k = 0; k < nt; ++k) {
        const i64 r0 = k * nb, kb = S.kb(k), r1 = std::min(n, (k + S.klt + 1) * nb), mk = r1 - r0;
        if (S.mine(k)) {
            T* d = S.at<T>(k, r0);
            potrf_tile<T>(kb, d, H, infos.as<i64>() + k, s);
            trsm_k<T>('R', 'L', ct, 'N', mk - kb, kb, T(1), d, H, d + kb, H, s);   // L21 = A21 L11^-H
            copy2d(P.as<T>(), mk, d, H, mk, kb, s);
        }
        if (S.size > 1) world_comm()->bcast(P.p, sizeof(T) * mk * kb, S.owner(k), s);
        // my tile columns inside the window: A(j:, j) -= L(j:, k) L(j, k)^H
        for (i64 j = k + 1; j <= std::min(nt - 1, k + S.klt); ++j) {
            if (!S.mine(j)) continue;
            const i64 mj = r1 - j * nb;
            if (mj <= 0) continue;
            const T* Pj = P.as<T>() + (j * nb - r0);
            gemm_k<T>('N', ct, mj, S.kb(j), kb, T(-1), Pj, mk, Pj, mk, T(1), S.at<T>(j, j * nb), H, s);
        }
    }
    return band_info(infos, nt, nb, S, s);
}

template <typename T>
int64_t pbtrs(const HermitianBandMatrix<T>& A, Matrix<T>& B, const Options&) {
    NTRACE("pbtrs", nullptr);
    const BandStorage& S = *A.storage();
    hipStream_t s = rt().main;
    if (B.m() != S.n) throw Error("native pbtrs: B must have n rows");
    const i64 n = S.n, nb = S.nb, nt = S.nt, H = S.H, nr = B.n();
    const char ct = ctrans<T>();
    Replica<T> X(B, s);
    T* x = X.p();
    for (i64 k = 0; k < nt; ++k) {                 // L y = b
        const i64 r0 = k * nb, kb = S.kb(k), r1 = std::min(n, (k + S.klt + 1) * nb), mk = r1 - r0;
        if (S.mine(k)) {
            const T* d = S.at<T>(k, r0);
            trsm_k<T>('L', 'L', 'N', 'N', kb, nr, T(1), d, H, x + r0, n, s);
            if (mk > kb) gemm_k<T>('N', 'N', mk - kb, nr, kb, T(-1), d + kb, H, x + r0, n, T(1), x + r0 + kb, n, s);
        }
        bcast_rows<T>(x, n, r0, r1, nr, S.owner(k), s);
    }
    for (i64 k = nt - 1; k >= 0; --k) {            // L^H x = y
        const i64 r0 = k * nb, kb = S.kb(k), r1 = std::min(n, (k + S.klt + 1) * nb), mk = r1 - r0;
        if (S.mine(k)) {
            const T* d = S.at<T>(k, r0);
            if (mk > kb) gemm_k<T>(ct, 'N', kb, nr, mk - kb, T(-1), d + kb, H, x + r0 + kb, n, T(1), x + r0, n, s);
            trsm_k<T>('L', 'L', ct, 'N', kb, nr, T(1), d, H, x + r0, n, s);
        }
        bcast_rows<T>(x, n, r0, r0 + kb, nr, S.owner(k), s);
    }
    X.to(B, s);
    return 0;
}

template <typename T>
int64_t pbsv(HermitianBandMatrix<T>& A, Matrix<T>& B, const Options& opts) {
    const int64_t info = pbtrf<T>(A, opts);
    if (info == 0) pbtrs<T>(A, B, opts);
    return info;
}

// ------------------------------------------------------------ LU
template <typename T>
int64_t gbtrf(BandMatrix<T>& A, std::vector<int64_t>& ipiv, const Options& opts) {
    NTRACE("gbtrf", nullptr);
    BandStorage& S = *A.storage();
    Runtime& R = rt();
    hipStream_t s = R.main;
    const i64 m = S.m, n = S.n, nb = S.nb, H = S.H;
    if ((S.kut) * nb < S.kl + S.ku)
        throw Error("native gbtrf: the band storage has no room for the kl + ku fill (construct a BandMatrix)");
    const i64 kt = std::min(S.mt, S.nt);
    const i64 PH = (S.klt + 1) * nb;
    Scratch infos(sizeof(i64) * std::max<i64>(kt, 1), s);
    dzero(infos.p, sizeof(i64) * std::max<i64>(kt, 1), s);
    Scratch pall(sizeof(i64) * std::max<i64>(kt * nb, 1), s);      // panel-relative pivots of every step
    Scratch P(sizeof(T) * PH * nb + sizeof(i64) * nb + 64, s);
    T* Pp = P.as<T>();
    i64* Ppv = reinterpret_cast<i64*>(reinterpret_cast<char*>(P.p) + sizeof(T) * PH * nb);
    // the band: entries of the fill rows above ku start as zero (constructor)
    for (i64 k = 0; k < kt; ++k) {
        const i64 r0 = k * nb, kb = std::min({nb, n - r0, m - r0}), r1 = std::min(m, (k + S.klt + 1) * nb);
        const i64 mk = r1 - r0;
        const int own = S.owner(k);
        if (S.mine(k)) {
            T* d = S.at<T>(k, r0);
            slate_hip::getrf_panel_ws<K<T>>(mk, kb, kp(d), H, Ppv, infos.as<i64>() + k, opts.pivot_threshold, false,
                                            R.lu_work, s);
            copy2d(Pp, mk, d, H, mk, kb, s);
        }
        if (S.size > 1) {
            // one message: the panel (mk x kb, ld mk) then the kb pivots
            Scratch pk(sizeof(T) * mk * kb + sizeof(i64) * kb, s);
            if (S.mine(k)) {
                dcopy(pk.p, Pp, sizeof(T) * mk * kb, s);
                dcopy(static_cast<char*>(pk.p) + sizeof(T) * mk * kb, Ppv, sizeof(i64) * kb, s);
            }
            world_comm()->bcast(pk.p, sizeof(T) * mk * kb + sizeof(i64) * kb, own, s);
            if (!S.mine(k)) {
                dcopy(Pp, pk.p, sizeof(T) * mk * kb, s);
                dcopy(Ppv, static_cast<char*>(pk.p) + sizeof(T) * mk * kb, sizeof(i64) * kb, s);
            }
        }
        dcopy(pall.as<i64>() + r0, Ppv, sizeof(i64) * kb, s);
        // my tile columns right of the panel inside the (filled) upper band
        for (i64 j = k + 1; j <= std::min(S.nt - 1, k + S.kut); ++j) {
            if (!S.mine(j)) continue;
            const i64 jb = S.kb(j);
            T* C = S.at<T>(j, r0);
            slate_hip::laswp_off<K<T>>(jb, kp(C), H, 0, kb, Ppv, 0, s);
            trsm_k<T>('L', 'L', 'N', 'U', kb, jb, T(1), Pp, mk, C, H, s);                       // U(k, j)
            if (mk > kb) gemm_k<T>('N', 'N', mk - kb, jb, kb, T(-1), Pp + kb, mk, C, H, T(1), C + kb, H, s);
        }
    }
    std::vector<i64> h((size_t)std::max<i64>(kt * nb, 1));
    NHIP(hipMemcpyAsync(h.data(), pall.p, sizeof(i64) * h.size(), hipMemcpyDeviceToHost, s));
    NHIP(hipStreamSynchronize(s));
    const i64 kmin = std::min(m, n);
    S.ku = std::min(n, S.kl + S.ku);            // the factor's upper bandwidth (SLATE gbtrf)
    ipiv.assign((size_t)kmin, 0);
    for (i64 i = 0; i < kmin; ++i) ipiv[i] = h[i] + (i / nb) * nb;
    return band_info(infos, kt, nb, S, s);
}

template <typename T>
int64_t gbtrs(const BandMatrix<T>& A, const std::vector<int64_t>& ipiv, Matrix<T>& B, const Options&) {
    NTRACE("gbtrs", nullptr);
    const BandStorage& S = *A.storage();
    hipStream_t s = rt().main;
    if (S.m != S.n || B.m() != S.n) throw Error("native gbtrs: square A, B with n rows");
    const i64 n = S.n, nb = S.nb, nt = S.nt, H = S.H, nr = B.n();
    if ((i64)ipiv.size() < n) throw Error("native gbtrs: ipiv of gbtrf expected");
    std::vector<i64> rel((size_t)n);
    for (i64 i = 0; i < n; ++i) rel[i] = ipiv[i] - (i / nb) * nb;
    Scratch pv(sizeof(i64) * std::max<i64>(n, 1), s);
    upload(pv.p, rel.data(), sizeof(i64) * n, s);
    Replica<T> X(B, s);
    T* x = X.p();
    for (i64 k = 0; k < nt; ++k) {                 // L y = P b, one step's interchanges at a time
        const i64 r0 = k * nb, kb = S.kb(k), r1 = std::min(n, (k + S.klt + 1) * nb), mk = r1 - r0;
        slate_hip::laswp_off<K<T>>(nr, kp(x + r0), n, 0, kb, pv.as<i64>() + r0, 0, s);   // every rank (replica)
        if (S.mine(k)) {
            const T* d = S.at<T>(k, r0);
            trsm_k<T>('L', 'L', 'N', 'U', kb, nr, T(1), d, H, x + r0, n, s);
            if (mk > kb) gemm_k<T>('N', 'N', mk - kb, nr, kb, T(-1), d + kb, H, x + r0, n, T(1), x + r0 + kb, n, s);
        }
        bcast_rows<T>(x, n, r0, r1, nr, S.owner(k), s);
    }
    for (i64 k = nt - 1; k >= 0; --k) {            // U x = y, column by column
        const i64 r0 = k * nb, kb = S.kb(k), ua = S.rlo(k);
        if (S.mine(k)) {
            const T* d = S.at<T>(k, r0);
            trsm_k<T>('L', 'U', 'N', 'N', kb, nr, T(1), d, H, x + r0, n, s);
            if (r0 > ua) gemm_k<T>('N', 'N', r0 - ua, nr, kb, T(-1), S.at<T>(k, ua), H, x + r0, n, T(1), x + ua, n, s);
        }
        bcast_rows<T>(x, n, ua, r0 + kb, nr, S.owner(k), s);
    }
    X.to(B, s);
    return 0;
}

template <typename T>
int64_t gbsv(BandMatrix<T>& A, std::vector<int64_t>& ipiv, Matrix<T>& B, const Options& opts) {
    const int64_t info = gbtrf<T>(A, ipiv, opts);
    if (info == 0) gbtrs<T>(A, ipiv, B, opts);
    return info;
}

// ------------------------------------------------------------ triangular band solve
template <typename T>
void tbsm(Side side, Op op, T alpha, const TriangularBandMatrix<T>& A, Matrix<T>& B, const Options&) {
    NTRACE("tbsm", nullptr);
    if (side != Side::Left) throw Error("native tbsm: Side::Left (solve the transposed system for Right)");
    const BandStorage& S = *A.storage();
    hipStream_t s = rt().main;
    if (B.m() != S.n) throw Error("native tbsm: B must have n rows");
    const i64 n = S.n, nb = S.nb, nt = S.nt, H = S.H, nr = B.n();
    const char ct = ctrans<T>(), dg = A.diag() == Diag::Unit ? 'U' : 'N';
    const bool lower = A.uplo() == Uplo::Lower, trans = op != Op::NoTrans;
    if (op == Op::Trans && is_cplx<T>()) throw Error("native tbsm: Trans of a complex matrix (use ConjTrans)");
    Replica<T> X(B, s);
    T* x = X.p();
    if (alpha != T(1) && n * nr > 0) slate_hip::gescale<K<T>>('G', n, nr, kv(alpha), kp(x), n, s);
    const bool forward = lower != trans;          // L x = b and U^H x = b go forward
    for (i64 t = 0; t < nt; ++t) {
        const i64 k = forward ? t : nt - 1 - t;
        const i64 r0 = k * nb, kb = S.kb(k);
        const T* d = S.at<T>(k, r0);
        if (lower) {
            const i64 r1 = std::min(n, (k + S.klt + 1) * nb), mk = r1 - r0;
            if (!trans) {                          // column-oriented forward
                if (S.mine(k)) {
                    trsm_k<T>('L', 'L', 'N', dg, kb, nr, T(1), d, H, x + r0, n, s);
                    if (mk > kb) gemm_k<T>('N', 'N', mk - kb, nr, kb, T(-1), d + kb, H, x + r0, n, T(1), x + r0 + kb, n, s);
                }
                bcast_rows<T>(x, n, r0, r1, nr, S.owner(k), s);
            } else {                               // L^H: row-oriented backward
                if (S.mine(k)) {
                    if (mk > kb) gemm_k<T>(ct, 'N', kb, nr, mk - kb, T(-1), d + kb, H, x + r0 + kb, n, T(1), x + r0, n, s);
                    trsm_k<T>('L', 'L', ct, dg, kb, nr, T(1), d, H, x + r0, n, s);
                }
                bcast_rows<T>(x, n, r0, r0 + kb, nr, S.owner(k), s);
            }
        } else {
            const i64 ua = S.rlo(k);
            const T* u = S.at<T>(k, ua);
            if (!trans) {                          // column-oriented backward
                if (S.mine(k)) {
                    trsm_k<T>('L', 'U', 'N', dg, kb, nr, T(1), d, H, x + r0, n, s);
                    if (r0 > ua) gemm_k<T>('N', 'N', r0 - ua, nr, kb, T(-1), u, H, x + r0, n, T(1), x + ua, n, s);
                }
                bcast_rows<T>(x, n, ua, r0 + kb, nr, S.owner(k), s);
            } else {                               // U^H: row-oriented forward
                if (S.mine(k)) {
                    if (r0 > ua) gemm_k<T>(ct, 'N', kb, nr, r0 - ua, T(-1), u, H, x + ua, n, T(1), x + r0, n, s);
                    trsm_k<T>('L', 'U', ct, dg, kb, nr, T(1), d, H, x + r0, n, s);
                }
                bcast_rows<T>(x, n, r0, r0 + kb, nr, S.owner(k), s);
            }
        }
    }
    X.to(B, s);
}

// ------------------------------------------------------------ products
// acc (replicated rows x cols, ld rows) += op(A) X for every local column
// tile of the band A (herm: A Hermitian from its lower band, the strict
// lower part also applied conjugate-transposed); then the partial products
// are summed over the ranks
template <typename T>
static void band_apply(const BandStorage& S, bool herm, const T* X, i64 ldx, i64 cols, T* acc, i64 ldc,
                       hipStream_t s) {
    const char ct = ctrans<T>();
    for (i64 k = S.rank; k < S.nt; k += S.size) {
        const i64 c0 = k * S.nb, kb = S.kb(k), r0 = S.rlo(k), r1 = S.rhi(k);
        const T* a = S.at<T>(k, r0);
        if (!herm) {
            gemm_k<T>('N', 'N', r1 - r0, cols, kb, T(1), a, S.H, X + c0, ldx, T(1), acc + r0, ldc, s);
            continue;
        }
        // Hermitian (lower band; the diagonal tile's strict upper part is
        // zero in the slab): the lower band with the diagonal, then the
        // strict lower part conjugate-transposed
        const i64 rows = r1 - c0;
        const T* lo = S.at<T>(k, c0);
        gemm_k<T>('N', 'N', rows, cols, kb, T(1), lo, S.H, X + c0, ldx, T(1), acc + c0, ldc, s);
        Scratch L(sizeof(T) * std::max<i64>(rows, 1) * kb, s);
        copy2d(L.as<T>(), rows, lo, S.H, rows, kb, s);
        slate_hip::geset<K<T>>('U', kb, kb, kv(T(0)), kv(T(0)), kp(L.as<T>()), rows, s);   // diagonal -> 0
        gemm_k<T>(ct, 'N', kb, cols, rows, T(1), L.as<T>(), rows, X + c0, ldx, T(1), acc + c0, ldc, s);
    }
    if (S.size > 1) {
        world_comm()->allreduce(acc, (size_t)ldc * cols, dt_of<T>::v, 's', s);
    }
}

// C = alpha acc + beta C through the replicas
template <typename T>
static void finish_product(T alpha, Replica<T>& acc, T beta, Matrix<T>& C, hipStream_t s) {
    Replica<T> Cr(C, s);
    if (acc.rows * acc.cols > 0)
        slate_hip::geadd<K<T>>('G', acc.rows, acc.cols, kv(alpha), kp(acc.p()), acc.rows, kv(beta), kp(Cr.p()),
                               Cr.rows, s);
    Cr.to(C, s);
}

template <typename T>
void gbmm(T alpha, const BandMatrix<T>& A, const Matrix<T>& B, T beta, Matrix<T>& C, const Options&) {
    NTRACE("gbmm", nullptr);
    const BandStorage& S = *A.storage();
    hipStream_t s = rt().main;
    if (B.m() != S.n || C.m() != S.m || C.n() != B.n()) throw Error("native gbmm: dimension mismatch");
    Replica<T> Xb(B, s);
    Matrix<T> Z(C.m(), C.n(), C.nb(), C.p(), C.q());
    Replica<T> acc(Z, s);                                  // zeros
    band_apply<T>(S, false, Xb.p(), std::max<i64>(Xb.rows, 1), B.n(), acc.p(), std::max<i64>(acc.rows, 1), s);
    finish_product<T>(alpha, acc, beta, C, s);
}

template <typename T>
void hbmm(Side side, T alpha, const HermitianBandMatrix<T>& A, const Matrix<T>& B, T beta, Matrix<T>& C,
          const Options& opts) {
    NTRACE("hbmm", nullptr);
    const BandStorage& S = *A.storage();
    hipStream_t s = rt().main;
    if (side == Side::Right) {
        // C = alpha B A + beta C  <=>  C^H = conj(alpha) A B^H + conj(beta) C^H  (A Hermitian)
        Matrix<T> Bh(B.n(), B.m(), B.nb(), B.p(), B.q()), Ch(C.n(), C.m(), C.nb(), C.p(), C.q());
        copy<T>(Op::ConjTrans, B, Bh);
        copy<T>(Op::ConjTrans, C, Ch);
        hbmm<T>(Side::Left, conj_of(alpha), A, Bh, conj_of(beta), Ch, opts);
        copy<T>(Op::ConjTrans, Ch, C);
        return;
    }
    if (B.m() != S.n || C.m() != S.n || C.n() != B.n()) throw Error("native hbmm: dimension mismatch");
    Replica<T> Xb(B, s);
    Matrix<T> Z(C.m(), C.n(), C.nb(), C.p(), C.q());
    Replica<T> acc(Z, s);
    band_apply<T>(S, true, Xb.p(), std::max<i64>(Xb.rows, 1), B.n(), acc.p(), std::max<i64>(acc.rows, 1), s);
    finish_product<T>(alpha, acc, beta, C, s);
}

// ------------------------------------------------------------ instantiation
#define SLATE_NATIVE_BAND(T)                                                                                    \
    template class BandMatrix<T>;                                                                               \
    template class HermitianBandMatrix<T>;                                                                      \
    template class TriangularBandMatrix<T>;                                                                     \
    template int64_t gbtrf<T>(BandMatrix<T>&, std::vector<int64_t>&, const Options&);                           \
    template int64_t gbtrs<T>(const BandMatrix<T>&, const std::vector<int64_t>&, Matrix<T>&, const Options&);   \
    template int64_t gbsv<T>(BandMatrix<T>&, std::vector<int64_t>&, Matrix<T>&, const Options&);                \
    template int64_t pbtrf<T>(HermitianBandMatrix<T>&, const Options&);                                         \
    template int64_t pbtrs<T>(const HermitianBandMatrix<T>&, Matrix<T>&, const Options&);                       \
    template int64_t pbsv<T>(HermitianBandMatrix<T>&, Matrix<T>&, const Options&);                              \
    template void tbsm<T>(Side, Op, T, const TriangularBandMatrix<T>&, Matrix<T>&, const Options&);             \
    template void gbmm<T>(T, const BandMatrix<T>&, const Matrix<T>&, T, Matrix<T>&, const Options&);            \
    template void hbmm<T>(Side, T, const HermitianBandMatrix<T>&, const Matrix<T>&, T, Matrix<T>&, const Options&);
SLATE_NATIVE_BAND(float)
SLATE_NATIVE_BAND(double)
SLATE_NATIVE_BAND(std::complex<float>)
SLATE_NATIVE_BAND(std::complex<double>)
#undef SLATE_NATIVE_BAND

}  // namespace native
}  // namespace slate_amd
