// Native drivers added in round 6: the generalized Hermitian-definite
// eigenproblem (hegst / hegv), GMRES-based mixed-precision refinement
// (gesv_mixed_gmres / posv_mixed_gmres) and the random butterfly transform
// solver (gesv_rbt, getrs_nopiv).  Reference: src/hegst.cc, src/hegv.cc,
// src/gesv_mixed_gmres.cc, src/posv_mixed_gmres.cc, src/gesv_rbt.cc,
// src/gerbt.cc (include/slate/slate.hh:540, 558, 688, 1082, 1138).
//
// Design (MI355X): every O(n^3) step is an existing distributed driver of
// native.hip (potrf, trsm, trmm, heev, getrf_nopiv on the MFMA kernels).
// The GMRES Krylov basis lives in ONE device buffer per rank -- the local
// rows of the restart + 1 basis vectors side by side -- so the classical
// Gram-Schmidt projections are one batched GEMV kernel and one all-reduce of
// j + 1 scalars per pass (two passes, CGS2), and only the (restart + 1) x
// restart Hessenberg least-squares problem runs on the host (Givens), as in
// the reference.  The butterflies run as the one-pass register kernel of
// csrc/hip/aux.hip on each rank's local rows: the order is padded to a
// multiple of 2^depth nb lcm(p, q), so every butterfly partner is local.
#include <algorithm>
#include <cmath>
#include <limits>
#include <numeric>
#include <random>
#include <vector>

#include "../hip/kernels.hpp"
#include "capi_util.hpp"
#include "native_rt.hpp"

namespace slate_amd {
namespace native {

namespace {

using slate_hip::s_add;
using slate_hip::s_conj;
using slate_hip::s_from_real;
using slate_hip::s_mul;
using slate_hip::s_sub;

// ------------------------------------------------------------ small vector kernels
// h[i] = sum_r conj(V[r + i ldv]) w[r], i < nv: one workgroup per basis vector
template <typename KT>
__global__ void __launch_bounds__(256) multi_dotc_kernel(i64 m, const KT* __restrict__ V, i64 ldv,
                                                         const KT* __restrict__ w, KT* __restrict__ h) {
    __shared__ KT red[256];
    const int i = blockIdx.x;
    KT acc = s_from_real(KT(), 0);
    for (i64 r = threadIdx.x; r < m; r += 256) acc = s_add(acc, s_mul(s_conj(V[r + i * ldv]), w[r]));
    red[threadIdx.x] = acc;
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
        if ((int)threadIdx.x < s) red[threadIdx.x] = s_add(red[threadIdx.x], red[threadIdx.x + s]);
        __syncthreads();
    }
    if (threadIdx.x == 0) h[i] = red[0];
}

// w[r] += alpha sum_i V[r + i ldv] h[i] (h on the device)
template <typename KT>
__global__ void __launch_bounds__(256) multi_axpy_kernel(i64 m, int nv, KT alpha, const KT* __restrict__ V, i64 ldv,
                                                         const KT* __restrict__ h, KT* __restrict__ w) {
    const i64 r = (i64)blockIdx.x * 256 + threadIdx.x;
    if (r >= m) return;
    KT acc = s_from_real(KT(), 0);
    for (int i = 0; i < nv; ++i) acc = s_add(acc, s_mul(V[r + i * ldv], h[i]));
    w[r] = s_add(w[r], s_mul(alpha, acc));
}

template <typename T>
void multi_dotc(i64 m, int nv, const T* V, i64 ldv, const T* w, T* h_d, hipStream_t s) {
    if (m > 0 && nv > 0) hipLaunchKernelGGL(multi_dotc_kernel<K<T>>, dim3(nv), dim3(256), 0, s, m, kp(V), ldv, kp(w), kp(h_d));
    else if (nv > 0) dzero(h_d, sizeof(T) * nv, s);
}

template <typename T>
void multi_axpy(i64 m, int nv, T alpha, const T* V, i64 ldv, const T* h_d, T* w, hipStream_t s) {
    if (m > 0 && nv > 0)
        hipLaunchKernelGGL(multi_axpy_kernel<K<T>>, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, s, m, nv,
                           kv(alpha), kp(V), ldv, kp(h_d), kp(w));
}

// sum over all ranks of a device array (in place), then to the host
template <typename T>
std::vector<T> allsum(T* d, int n, hipStream_t s) {
    if (Comm* w = world_comm()) w->allreduce(d, (size_t)n, dt_of<T>::v, 's', s);
    std::vector<T> h((size_t)n);
    NHIP(hipMemcpyAsync(h.data(), d, sizeof(T) * n, hipMemcpyDeviceToHost, s));
    NHIP(hipStreamSynchronize(s));
    return h;
}

// ------------------------------------------------------------ distributed n x 1 vectors
// The basis / work vectors of GMRES: n x 1 matrices on A's grid, i.e. the
// local rows live on process column 0 (other ranks hold no rows).  Column
// c of an n x k matrix B sits on process column (c / nb) % q at the SAME
// local rows, so moving it is one broadcast of mloc elements over the row
// communicator.
template <typename T>
struct VecSet {
    i64 n = 0, mloc = 0, ld = 1;
    int count = 0;
    Scratch buf;
    const Storage* shape = nullptr;
    VecSet(const Storage& S, int cnt, hipStream_t s)
        : n(S.m), mloc(S.pc == 0 ? S.mloc : 0), ld(std::max<i64>(1, (S.mloc + 15) / 16 * 16)), count(cnt),
          buf(sizeof(T) * (size_t)std::max<i64>(1, (S.pc == 0 ? ld : 1) * cnt), s), shape(&S) {
        dzero(buf.p, sizeof(T) * (size_t)std::max<i64>(1, (S.pc == 0 ? ld : 1) * cnt), s);
    }
    T* col(int i) { return buf.as<T>() + (mloc ? (i64)i * ld : 0); }
    // n x 1 Matrix over vector i (zero-copy)
    Matrix<T> mat(int i) {
        return Matrix<T>::from_device(col(i), ld, n, 1, shape->nb, shape->p, shape->q);
    }
};

// dst (mloc on process column 0) <- column c of B
template <typename T>
void get_col(const Storage& SB, i64 c, T* dst, hipStream_t s) {
    const int pcc = (int)((c / SB.nb) % SB.q);
    const i64 lc = (c / SB.nb) / SB.q * SB.nb + c % SB.nb;
    if (SB.q == 1) {
        copy2d(dst, SB.lld, static_cast<const T*>(SB.buf) + lc * SB.lld, SB.lld, SB.mloc, 1, s);
        return;
    }
    Scratch t(sizeof(T) * std::max<i64>(1, SB.mloc), s);
    if (SB.pc == pcc) copy2d(t.as<T>(), SB.mloc, static_cast<const T*>(SB.buf) + lc * SB.lld, SB.lld, SB.mloc, 1, s);
    if (SB.mloc) SB.gc->row->bcast(t.p, sizeof(T) * SB.mloc, pcc, s);
    if (SB.pc == 0) copy2d(dst, SB.mloc, t.as<T>(), SB.mloc, SB.mloc, 1, s);
    NHIP(hipStreamSynchronize(s));
}

// column c of B <- src (mloc on process column 0)
template <typename T>
void put_col(const T* src, Storage& SB, i64 c, hipStream_t s) {
    const int pcc = (int)((c / SB.nb) % SB.q);
    const i64 lc = (c / SB.nb) / SB.q * SB.nb + c % SB.nb;
    if (SB.q == 1) {
        copy2d(static_cast<T*>(SB.buf) + lc * SB.lld, SB.lld, src, SB.lld, SB.mloc, 1, s);
        return;
    }
    Scratch t(sizeof(T) * std::max<i64>(1, SB.mloc), s);
    if (SB.pc == 0) copy2d(t.as<T>(), SB.mloc, src, SB.mloc, SB.mloc, 1, s);
    if (SB.mloc) SB.gc->row->bcast(t.p, sizeof(T) * SB.mloc, 0, s);
    if (SB.pc == pcc) copy2d(static_cast<T*>(SB.buf) + lc * SB.lld, SB.lld, t.as<T>(), SB.mloc, SB.mloc, 1, s);
    NHIP(hipStreamSynchronize(s));
}

template <typename T> struct lower_of;
template <> struct lower_of<double> { using type = float; };
template <> struct lower_of<std::complex<double>> { using type = std::complex<float>; };

template <typename Hi, typename Lo>
void convert_local(const Storage& SA, Storage& SB, hipStream_t s) {
    if (SA.mloc && SA.nloc)
        slate_hip::gecopy<K<Hi>, K<Lo>>('G', 'N', SA.mloc, SA.nloc, kp(static_cast<const Hi*>(SA.buf)), SA.lld,
                                        kp(static_cast<Lo*>(SB.buf)), SB.lld, s);
}

template <typename T>
double vnorm2(VecSet<T>& W, int i, Scratch& hd, hipStream_t s) {
    multi_dotc<T>(W.mloc, 1, W.col(i), W.ld, W.col(i), hd.as<T>(), s);
    return std::sqrt(std::max(0.0, (double)std::real(allsum<T>(hd.as<T>(), 1, s)[0])));
}

template <typename T>
void vscale(VecSet<T>& W, int i, T a, hipStream_t s) {
    if (W.mloc) slate_hip::gescale<K<T>>('G', W.mloc, 1, kv(a), kp(W.col(i)), W.ld, s);
}

template <typename T>
double vmax(VecSet<T>& W, int i) {
    return norm<T>(Norm::Max, W.mat(i));
}

// complex Givens rotation zeroing b in (a, b): c real, s complex
template <typename T>
void givens(T a, T b, double& c, T& sn, T& r) {
    const double aa = std::abs(a), bb = std::abs(b);
    if (bb == 0) { c = 1; sn = T(0); r = a; return; }
    if (aa == 0) { c = 0; sn = T(1); r = b; return; }
    const double nrm = std::hypot(aa, bb);
    const T alpha = a / aa;
    c = aa / nrm;
    sn = alpha * conj_of(b) / nrm;
    r = alpha * nrm;
}

// restarted right-preconditioned GMRES on A M^-1 u = r for every column of
// X (A X = B), started from the low-precision solution already in X
template <typename T, typename Apply, typename Precond>
int gmres_ir(const Storage& SB, Matrix<T>& X, Apply&& apply_a, Precond&& precond, double anorm, const Options& opts,
             bool& converged_all) {
    hipStream_t s = rt().main;
    const i64 n = SB.m;
    const int itermax = std::max(1, opts.max_iterations);
    const int restart = std::max(1, std::min(opts.restart, itermax));
    const double eps = std::numeric_limits<real_t<T>>::epsilon();
    const double cte = anorm * eps * std::sqrt((double)n);
    Matrix<T> Bcol(n, 1, SB.nb, SB.p, SB.q);
    VecSet<T> V(*Bcol.storage(), restart + 1, s), Z(*Bcol.storage(), restart, s), Wv(*Bcol.storage(), 2, s);
    Scratch hd(sizeof(T) * (restart + 2), s);
    int total = 0;
    converged_all = true;
    Storage& SX = *X.storage();
    for (i64 col = 0; col < SB.n; ++col) {
        // Wv[1] = b, V[0] (scratch) = x
        get_col<T>(SB, col, Wv.col(1), s);
        Matrix<T> xcol(n, 1, SB.nb, SB.p, SB.q);
        get_col<T>(SX, col, xcol.data(), s);
        bool conv = false;
        int steps = 0;
        while (steps < itermax) {
            // r = b - A x
            copy2d(Wv.col(0), Wv.ld, Wv.col(1), Wv.ld, Wv.mloc, 1, s);
            Matrix<T> r = Wv.mat(0);
            apply_a(T(-1), xcol, T(1), r);
            if (vmax<T>(Wv, 0) <= norm<T>(Norm::Max, xcol) * cte) { conv = true; break; }
            const double beta = vnorm2<T>(Wv, 0, hd, s);
            if (beta == 0) { conv = true; break; }
            copy2d(V.col(0), V.ld, Wv.col(0), Wv.ld, V.mloc, 1, s);
            vscale<T>(V, 0, T(1.0 / beta), s);
            std::vector<T> H((size_t)(restart + 1) * restart, T(0)), g((size_t)restart + 1, T(0)), sn((size_t)restart);
            std::vector<double> cs((size_t)restart);
            g[0] = T(beta);
            int k = 0;
            for (int j = 0; j < restart && steps < itermax; ++j) {
                Matrix<T> vj = V.mat(j), zj = Z.mat(j), w = Wv.mat(0);
                precond(vj, zj);                                   // z_j = M^-1 v_j
                apply_a(T(1), zj, T(0), w);                        // w = A z_j
                std::vector<T> hs((size_t)j + 1, T(0));
                for (int pass = 0; pass < 2; ++pass) {             // CGS2
                    multi_dotc<T>(V.mloc, j + 1, V.col(0), V.ld, Wv.col(0), hd.as<T>(), s);
                    const std::vector<T> h = allsum<T>(hd.as<T>(), j + 1, s);
                    multi_axpy<T>(V.mloc, j + 1, T(-1), V.col(0), V.ld, hd.as<T>(), Wv.col(0), s);
                    for (int i = 0; i <= j; ++i) hs[i] += h[i];
                }
                const double hn = vnorm2<T>(Wv, 0, hd, s);
                auto Hat = [&](int r, int c) -> T& { return H[(size_t)r + (size_t)c * (restart + 1)]; };
                for (int i = 0; i <= j; ++i) Hat(i, j) = hs[i];
                Hat(j + 1, j) = T(hn);
                for (int i = 0; i < j; ++i) {                      // previous rotations
                    const T a = Hat(i, j), b = Hat(i + 1, j);
                    Hat(i, j) = cs[i] * a + sn[i] * b;
                    Hat(i + 1, j) = -conj_of(sn[i]) * a + cs[i] * b;
                }
                T r;
                givens<T>(Hat(j, j), Hat(j + 1, j), cs[j], sn[j], r);
                Hat(j, j) = r;
                Hat(j + 1, j) = T(0);
                g[j + 1] = -conj_of(sn[j]) * g[j];
                g[j] = cs[j] * g[j];
                k = j + 1;
                ++steps;
                ++total;
                if (hn == 0 || std::abs(g[j + 1]) <= 1e-14 * beta) break;
                copy2d(V.col(j + 1), V.ld, Wv.col(0), Wv.ld, V.mloc, 1, s);
                vscale<T>(V, j + 1, T(1.0 / hn), s);
            }
            // y = R^-1 g (host back substitution), x += Z y
            std::vector<T> y((size_t)k, T(0));
            for (int i = k - 1; i >= 0; --i) {
                T acc = g[i];
                for (int c = i + 1; c < k; ++c) acc -= H[(size_t)i + (size_t)c * (restart + 1)] * y[c];
                y[i] = acc / H[(size_t)i + (size_t)i * (restart + 1)];
            }
            upload(hd.p, y.data(), sizeof(T) * k, s);
            multi_axpy<T>(Z.mloc, k, T(1), Z.col(0), Z.ld, hd.as<T>(), xcol.data(), s);
            NHIP(hipStreamSynchronize(s));
        }
        if (!conv) {
            // the final check after the last correction
            copy2d(Wv.col(0), Wv.ld, Wv.col(1), Wv.ld, Wv.mloc, 1, s);
            Matrix<T> r = Wv.mat(0);
            apply_a(T(-1), xcol, T(1), r);
            conv = vmax<T>(Wv, 0) <= norm<T>(Norm::Max, xcol) * cte;
        }
        converged_all = converged_all && conv;
        put_col<T>(xcol.data(), SX, col, s);
    }
    return total;
}

// ------------------------------------------------------------ butterflies
// diagonals of W = W_depth ... W_1 of order N: exp(r / 10), r uniform in
// [-1/2, 1/2) (Baboulin et al.), identical on every rank (seeded)
std::vector<double> butterfly_diag(i64 N, int depth, uint64_t seed) {
    std::mt19937_64 g(seed);
    std::uniform_real_distribution<double> u(-0.5, 0.5);
    std::vector<double> d((size_t)N * depth);
    for (auto& x : d) x = std::exp(u(g) / 10.0);
    return d;
}

i64 rbt_size(i64 n, int depth, i64 nb, int p, int q) {
    const i64 l = (i64)p / std::gcd(p, q) * q;
    const i64 unit = ((i64)1 << depth) * nb * l;
    return std::max(unit, (n + unit - 1) / unit * unit);
}

// M := op(W) M (rows) or M op(W)^T (columns), op(W) = W^T when trans, on
// the local block: the diagonal entries of this rank's global indices
template <typename T>
void apply_w(const std::vector<double>& diag, int depth, Storage& S, bool trans, bool rows, hipStream_t s) {
    using R = real_t<T>;
    const i64 nidx = rows ? S.mloc : S.nloc, nother = rows ? S.nloc : S.mloc;
    if (!nidx || !nother) return;
    const i64 Nglob = rows ? S.m : S.n;
    std::vector<R> loc((size_t)nidx * depth);
    for (i64 i = 0; i < nidx; ++i) {
        const i64 gi = rows ? l2g(i, S.nb, S.p, S.pr) : l2g(i, S.nb, S.q, S.pc);
        for (int l = 0; l < depth; ++l) loc[(size_t)l * nidx + i] = (R)diag[(size_t)l * Nglob + gi];
    }
    Scratch dd(sizeof(R) * loc.size(), s);
    upload(dd.p, loc.data(), sizeof(R) * loc.size(), s);
    slate_hip::butterfly<K<T>, R>(trans, rows, depth, nidx, nother, kp(static_cast<T*>(S.buf)), S.lld, dd.as<R>(), nidx,
                                  s);
    NHIP(hipStreamSynchronize(s));
}

// N x k copy of M (n x k, same grid / nb): the global indices < n map to the
// same process and local position, so it is one local block copy
template <typename T>
Matrix<T> padded(const Matrix<T>& M, i64 N, i64 k, bool identity) {
    const Storage& S = *M.storage();
    Matrix<T> P(N, k, S.nb, S.p, S.q);
    if (identity) set<T>(T(0), T(1), P);
    hipStream_t s = rt().main;
    copy2d(P.data(), P.lld(), static_cast<const T*>(S.buf), S.lld, S.mloc, S.nloc, s);
    NHIP(hipStreamSynchronize(s));
    return P;
}

}  // namespace

// ------------------------------------------------------------ hegst / hegv
template <typename T>
void hegst(int64_t itype, HermitianMatrix<T>& A, const HermitianMatrix<T>& L, const Options& opts) {
    if (itype < 1 || itype > 3) throw Error("native hegst: itype must be 1, 2 or 3");
    const Storage& SA = *A.storage();
    const Storage& SL = *L.storage();
    if (SA.n != SL.n || SA.nb != SL.nb || SA.p != SL.p || SA.q != SL.q)
        throw Error("native hegst: A and B must be n x n on one grid / tile size");
    // the full Hermitian A, transformed in place, written back over A
    Matrix<T> F = expand_tri<T>(A, A.uplo(), 1);
    const bool lower = L.uplo() == Uplo::Lower;
    const Uplo u = L.uplo();
    // with B = L L^H (Lower) or U^H U (Upper, L := U^H): ops on "L" / "L^H"
    const Op opL = lower ? Op::NoTrans : Op::ConjTrans, opLH = lower ? Op::ConjTrans : Op::NoTrans;
    if (itype == 1) {
        trsm<T>(Side::Left, u, opL, Diag::NonUnit, T(1), L, F, opts);     // L^-1 A
        trsm<T>(Side::Right, u, opLH, Diag::NonUnit, T(1), L, F, opts);   // (L^-1 A) L^-H
    } else {
        trmm<T>(Side::Left, u, opLH, Diag::NonUnit, T(1), L, F, opts);    // L^H A
        trmm<T>(Side::Right, u, opL, Diag::NonUnit, T(1), L, F, opts);    // (L^H A) L
    }
    copy<T>(Op::NoTrans, F, A);
}

template <typename T>
static int64_t hegv_impl(int64_t itype, HermitianMatrix<T>& A, HermitianMatrix<T>& B, std::vector<real_t<T>>& Lambda,
                         Matrix<T>* Z, const Options& opts) {
    // the Cholesky driver factors Lower storage: an Upper B (= U^H U) is
    // factored as its conjugate transpose, L = U^H, and U written back
    const bool upper = B.uplo() == Uplo::Upper;
    HermitianMatrix<T> L = B;
    if (upper) {
        Matrix<T> Bt(B.n(), B.n(), B.nb(), B.p(), B.q());
        copy<T>(Op::ConjTrans, B, Bt);
        L = HermitianMatrix<T>(Uplo::Lower, Bt);
    }
    const int64_t info = potrf<T>(L, opts);
    if (info) return A.n() + info;
    if (upper) copy<T>(Op::ConjTrans, L, B);
    hegst<T>(itype, A, L, opts);
    const int64_t ie = Z ? heev<T>(A, Lambda, *Z, opts) : heev<T>(A, Lambda, opts);
    if (ie || !Z) return ie;
    if (itype == 3) trmm<T>(Side::Left, Uplo::Lower, Op::NoTrans, Diag::NonUnit, T(1), L, *Z, opts);   // x = L y
    else trsm<T>(Side::Left, Uplo::Lower, Op::ConjTrans, Diag::NonUnit, T(1), L, *Z, opts);            // x = L^-H y
    return 0;
}

template <typename T>
int64_t hegv(int64_t itype, HermitianMatrix<T>& A, HermitianMatrix<T>& B, std::vector<real_t<T>>& Lambda,
             Matrix<T>& Z, const Options& opts) {
    return hegv_impl<T>(itype, A, B, Lambda, &Z, opts);
}
template <typename T>
int64_t hegv(int64_t itype, HermitianMatrix<T>& A, HermitianMatrix<T>& B, std::vector<real_t<T>>& Lambda,
             const Options& opts) {
    return hegv_impl<T>(itype, A, B, Lambda, nullptr, opts);
}

// ------------------------------------------------------------ GMRES-IR
template <typename T>
int64_t gesv_mixed_gmres(Matrix<T>& A, std::vector<int64_t>& ipiv, Matrix<T>& B, Matrix<T>& X, int& iter,
                         const Options& opts) {
    using Lo = typename lower_of<T>::type;
    const Storage& SA = *A.storage();
    hipStream_t s = rt().main;
    Matrix<Lo> Al(SA.m, SA.n, SA.nb, SA.p, SA.q);
    convert_local<T, Lo>(SA, *Al.storage(), s);
    NHIP(hipStreamSynchronize(s));
    iter = 0;
    if (getrf<Lo>(Al, ipiv, opts) == 0) {
        const Storage& SB = *B.storage();
        // x0 = (LU)^-1 b in the low precision
        Matrix<Lo> Xl(SB.m, SB.n, SB.nb, SB.p, SB.q);
        convert_local<T, Lo>(SB, *Xl.storage(), s);
        NHIP(hipStreamSynchronize(s));
        getrs<Lo>(Al, ipiv, Xl, opts);
        convert_local<Lo, T>(*Xl.storage(), *X.storage(), s);
        NHIP(hipStreamSynchronize(s));
        auto apply = [&](T alpha, const Matrix<T>& x, T beta, Matrix<T>& y) { gemm<T>(alpha, A, x, beta, y, opts); };
        auto precond = [&](const Matrix<T>& v, Matrix<T>& z) {
            const Storage& SV = *v.storage();
            Matrix<Lo> t(SV.m, 1, SV.nb, SV.p, SV.q);
            convert_local<T, Lo>(SV, *t.storage(), s);
            NHIP(hipStreamSynchronize(s));
            getrs<Lo>(Al, ipiv, t, opts);
            convert_local<Lo, T>(*t.storage(), *z.storage(), s);
            NHIP(hipStreamSynchronize(s));
        };
        bool ok = false;
        const int it = gmres_ir<T>(SB, X, apply, precond, norm<T>(Norm::Max, A), opts, ok);
        if (ok) { iter = it; return 0; }
        iter = -31;
    } else {
        iter = -3;
    }
    copy<T>(Op::NoTrans, B, X);
    return gesv<T>(A, ipiv, X, opts);
}

template <typename T>
int64_t posv_mixed_gmres(HermitianMatrix<T>& A, Matrix<T>& B, Matrix<T>& X, int& iter, const Options& opts) {
    using Lo = typename lower_of<T>::type;
    const Storage& SA = *A.storage();
    hipStream_t s = rt().main;
    HermitianMatrix<Lo> Al(A.uplo(), SA.n, SA.nb, SA.p, SA.q);
    convert_local<T, Lo>(SA, *Al.storage(), s);
    NHIP(hipStreamSynchronize(s));
    iter = 0;
    if (potrf<Lo>(Al, opts) == 0) {
        const Storage& SB = *B.storage();
        Matrix<Lo> Xl(SB.m, SB.n, SB.nb, SB.p, SB.q);
        convert_local<T, Lo>(SB, *Xl.storage(), s);
        NHIP(hipStreamSynchronize(s));
        potrs<Lo>(Al, Xl, opts);
        convert_local<Lo, T>(*Xl.storage(), *X.storage(), s);
        NHIP(hipStreamSynchronize(s));
        const Matrix<T> Af = expand_tri<T>(A, A.uplo(), 1);
        auto apply = [&](T alpha, const Matrix<T>& x, T beta, Matrix<T>& y) { gemm<T>(alpha, Af, x, beta, y, opts); };
        auto precond = [&](const Matrix<T>& v, Matrix<T>& z) {
            const Storage& SV = *v.storage();
            Matrix<Lo> t(SV.m, 1, SV.nb, SV.p, SV.q);
            convert_local<T, Lo>(SV, *t.storage(), s);
            NHIP(hipStreamSynchronize(s));
            potrs<Lo>(Al, t, opts);
            convert_local<Lo, T>(*t.storage(), *z.storage(), s);
            NHIP(hipStreamSynchronize(s));
        };
        bool ok = false;
        const int it = gmres_ir<T>(SB, X, apply, precond, norm<T>(Norm::Max, Af), opts, ok);
        if (ok) { iter = it; return 0; }
        iter = -31;
    } else {
        iter = -3;
    }
    copy<T>(Op::NoTrans, B, X);
    return posv<T>(A, X, opts);
}

// ------------------------------------------------------------ RBT
template <typename T>
int64_t getrs_nopiv(const Matrix<T>& A, Matrix<T>& B, const Options& opts) {
    trsm<T>(Side::Left, Uplo::Lower, Op::NoTrans, Diag::Unit, T(1), A, B, opts);
    trsm<T>(Side::Left, Uplo::Upper, Op::NoTrans, Diag::NonUnit, T(1), A, B, opts);
    return 0;
}

template <typename T>
int64_t gesv_rbt(Matrix<T>& A, Matrix<T>& B, const Options& opts) {
    const Storage& SA = *A.storage();
    const Storage& SB = *B.storage();
    if (SA.m != SA.n || SB.m != SA.n) throw Error("native gesv_rbt: A n x n, B n x nrhs");
    if (SB.nb != SA.nb || SB.p != SA.p || SB.q != SA.q) throw Error("native gesv_rbt: A and B share grid and nb");
    hipStream_t s = rt().main;
    const int depth = std::max(1, std::min(4, opts.depth));
    const i64 n = SA.n, N = rbt_size(n, depth, SA.nb, SA.p, SA.q);
    Matrix<T> A0(n, n, SA.nb, SA.p, SA.q);
    copy<T>(Op::NoTrans, A, A0);
    Matrix<T> Ap = N == n ? A : padded<T>(A, N, N, true);
    const std::vector<double> U = butterfly_diag(N, depth, 7), V = butterfly_diag(N, depth, 8);
    apply_w<T>(U, depth, *Ap.storage(), true, true, s);      // U^T A
    apply_w<T>(V, depth, *Ap.storage(), true, false, s);     // (U^T A) V
    Options o = opts;
    const int64_t info = getrf_nopiv<T>(Ap, o);
    if (info) return info;
    // x = V (LU)^-1 U^T r on the padded order
    auto solve = [&](const Matrix<T>& R, Matrix<T>& D) {
        Matrix<T> Y = padded<T>(R, N, R.n(), false);
        apply_w<T>(U, depth, *Y.storage(), true, true, s);
        getrs_nopiv<T>(Ap, Y, o);
        apply_w<T>(V, depth, *Y.storage(), false, true, s);
        Storage& SD = *D.storage();
        copy2d(static_cast<T*>(SD.buf), SD.lld, Y.data(), Y.lld(), SD.mloc, SD.nloc, s);
        NHIP(hipStreamSynchronize(s));
    };
    Matrix<T> X(n, SB.n, SB.nb, SB.p, SB.q), R(n, SB.n, SB.nb, SB.p, SB.q), D(n, SB.n, SB.nb, SB.p, SB.q);
    solve(B, X);
    const double eps = std::numeric_limits<real_t<T>>::epsilon();
    const double cte = norm<T>(Norm::Max, A0) * eps * std::sqrt((double)n);
    const int itermax = std::min(opts.max_iterations, 10);
    for (int it = 0; it <= itermax; ++it) {
        copy<T>(Op::NoTrans, B, R);
        gemm<T>(T(-1), A0, X, T(1), R, opts);                 // R = B - A X
        if (norm<T>(Norm::Max, R) <= norm<T>(Norm::Max, X) * cte || it == itermax) break;
        solve(R, D);
        add<T>(T(1), D, T(1), X);
    }
    copy<T>(Op::NoTrans, X, B);
    return 0;
}

// ------------------------------------------------------------ hesv / scale
// ------------------------------------------------------------ Aasen (hetrf / hetrs / hesv)
// Reference: src/hetrf.cc (communication-avoiding blocked Aasen, host only
// in the reference: "GPU version not yet implemented", hetrf.cc:23), the
// band T factored by gbtrf (hetrf.cc:511), src/hetrs.cc:94-105.  Python twin:
// models/hetrf.py aasen().  Step J (block column j0:j1, H = T L^H):
//   H(0:J, J)  three strided-BATCHED MFMA GEMMs over the block tridiagonal T;
//   T(J, J)    = L(J,J)^-1 (A(J,J) - L(J,0:J) H(0:J,J) - L(J,J) T(J,J-1)
//                L(J,J-1)^H) L(J,J)^-H, symmetrised;
//   panel      = A(j1:, J) - L(j1:, 0:j1) H(0:j1, J), GPU partial-pivoting
//                LU -> L(j1:, J+1), T(J+1, J) = U L(J,J)^-H;
//   symmetric interchange of the trailing A (row swaps, conjugate
//   transpose, row swaps).
struct IndefData {
    i64 n = 0, N = 0, nb = 0;
    char dtype = 0;
    std::shared_ptr<void> L;        // Scratch: N x N unit lower (first block column [I; 0])
    std::vector<i64> perm;          // row i of P A is row perm[i] of A
    std::shared_ptr<void> Tband;    // BandMatrix<T>: gbtrf factors of T
    std::vector<int64_t> Tpiv;
    int p = 1, q = 1;
};

namespace {

template <typename T>
void gemm_batched(char ta, char tb, i64 m, i64 n, i64 k, T alpha, const T* A, i64 lda, i64 sa, const T* B, i64 ldb,
                  i64 sb, T beta, T* C, i64 ldc, i64 sc, i64 batch, hipStream_t s) {
    if (m <= 0 || n <= 0 || batch <= 0) return;
    slate_hip::GemmCall c;
    c.transA = ta; c.transB = tb; c.m = m; c.n = n; c.k = k;
    c.alpha_re = (double)std::real(alpha); c.alpha_im = (double)std::imag(alpha);
    c.beta_re = (double)std::real(beta); c.beta_im = (double)std::imag(beta);
    c.A = A; c.lda = lda; c.strideA = sa; c.B = B; c.ldb = ldb; c.strideB = sb;
    c.C = C; c.ldc = ldc; c.strideC = sc; c.batch = batch;
    if constexpr (is_cplx<T>()) slate_hip::gemm_complex<K<T>>(c, s);
    else slate_hip::gemm_real<T>(c, s);
}

template <typename T>
void aasen(i64 N, i64 nb, T* Af, T* L, T* Td, T* Tl, i64* piv_rel, i64* info, hipStream_t s) {
    const i64 NT = N / nb;
    const char ct = ctrans<T>();
    Scratch Xs(sizeof(T) * N * nb, s), Hs(sizeof(T) * N * nb, s), S(sizeof(T) * nb * nb, s),
        tmp(sizeof(T) * nb * nb, s), Wt(sizeof(T) * N * N, s);
    T* xs = Xs.as<T>();
    T* hs = Hs.as<T>();
    T* sm = S.as<T>();
    T* tp = tmp.as<T>();
    dzero(xs, sizeof(T) * N * nb, s);
    dzero(hs, sizeof(T) * N * nb, s);
    auto td = [&](i64 I) { return Td + I * nb * nb; };
    auto tl = [&](i64 I) { return Tl + I * nb * nb; };
    for (i64 J = 0; J < NT; ++J) {
        const i64 j0 = J * nb, j1 = j0 + nb;
        // X = L(J, 0:J+1)^H, then H(I, J) = Td[I] X[I] + Tl[I] X[I-1] + Tl[I+1]^H X[I+1], I < J
        slate_hip::gecopy<K<T>, K<T>>('G', 'C', j1, nb, kp(L + j0), N, kp(xs), N, s);
        if (J > 0) {
            gemm_batched<T>('N', 'N', nb, nb, nb, T(1), td(0), nb, nb * nb, xs, N, nb, T(0), hs, N, nb, J, s);
            if (J > 1)
                gemm_batched<T>('N', 'N', nb, nb, nb, T(1), tl(1), nb, nb * nb, xs, N, nb, T(1), hs + nb, N, nb, J - 1, s);
            gemm_batched<T>(ct, 'N', nb, nb, nb, T(1), tl(1), nb, nb * nb, xs + nb, N, nb, T(1), hs, N, nb, J, s);
        }
        // T(J, J)
        copy2d(sm, nb, Af + j0 + j0 * N, N, nb, nb, s);
        const T* Ljj = L + j0 + j0 * N;
        if (J > 0) {
            gemm_k<T>('N', 'N', nb, nb, j0, T(-1), L + j0, N, hs, N, T(1), sm, nb, s);
            gemm_k<T>('N', 'N', nb, nb, nb, T(1), tl(J), nb, xs + j0 - nb, N, T(0), tp, nb, s);
            gemm_k<T>('N', 'N', nb, nb, nb, T(-1), Ljj, N, tp, nb, T(1), sm, nb, s);
            slate_hip::trsm<K<T>>('L', 'L', 'N', 'U', nb, nb, kv(T(1)), kp(Ljj), N, kp(sm), nb, s);
            slate_hip::trsm<K<T>>('R', 'L', ct, 'U', nb, nb, kv(T(1)), kp(Ljj), N, kp(sm), nb, s);
        }
        slate_hip::gecopy<K<T>, K<T>>('G', 'C', nb, nb, kp(sm), nb, kp(tp), nb, s);
        slate_hip::geadd<K<T>>('G', nb, nb, kv(T(0.5)), kp(tp), nb, kv(T(0.5)), kp(sm), nb, s);
        copy2d(td(J), nb, sm, nb, nb, nb, s);
        gemm_k<T>('N', 'N', nb, nb, nb, T(1), sm, nb, xs + j0, N, T(0), hs + j0, N, s);
        if (J > 0) gemm_k<T>('N', 'N', nb, nb, nb, T(1), tl(J), nb, xs + j0 - nb, N, T(1), hs + j0, N, s);
        if (J == NT - 1) break;
        // panel: A(j1:, J) -= L(j1:, 0:j1) H(0:j1, J), LU with partial pivoting
        T* Wp = Af + j1 + j0 * N;
        const i64 mp = N - j1;
        gemm_k<T>('N', 'N', mp, nb, j1, T(-1), L + j1, N, hs, N, T(1), Wp, N, s);
        i64* piv = piv_rel + j1;
        slate_hip::getrf_panel_ws<K<T>>(mp, nb, kp(Wp), N, piv, info + J, 1.0, false, rt().lu_work, s);
        slate_hip::v_explicit<K<T>>(mp, nb, kp(Wp), N, kp(L + j1 + j1 * N), N, s);
        T* T1 = tl(J + 1);
        dzero(T1, sizeof(T) * nb * nb, s);
        slate_hip::gecopy<K<T>, K<T>>('U', 'N', nb, nb, kp(Wp), N, kp(T1), nb, s);
        slate_hip::trsm<K<T>>('R', 'L', ct, 'U', nb, nb, kv(T(1)), kp(Ljj), N, kp(T1), nb, s);
        // symmetric interchange: L's rows, then the trailing Hermitian block
        slate_hip::laswp_off<K<T>>(j1, kp(L + j1), N, 0, nb, piv, 0, s);
        T* Str = Af + j1 + j1 * N;
        slate_hip::laswp_off<K<T>>(mp, kp(Str), N, 0, nb, piv, 0, s);
        slate_hip::gecopy<K<T>, K<T>>('G', 'C', mp, mp, kp(Str), N, kp(Wt.as<T>()), N, s);
        slate_hip::laswp_off<K<T>>(mp, kp(Wt.as<T>()), N, 0, nb, piv, 0, s);
        copy2d(Str, N, Wt.as<T>(), N, mp, mp, s);
    }
}

}  // namespace

template <typename T>
int64_t hetrf(const HermitianMatrix<T>& A, IndefiniteFactors<T>& F, const Options&) {
    NTRACE("hetrf", nullptr);
    const Storage& SA = *A.storage();
    hipStream_t s = rt().main;
    const i64 n = SA.n;
    const i64 nb = std::max<i64>(8, std::min<i64>(SA.nb, 256));
    const i64 N = std::max<i64>(nb, (n + nb - 1) / nb * nb), NT = N / nb;
    // the full Hermitian matrix on every rank, padded with an identity block
    std::vector<T> h((size_t)N * N, T(0));
    {
        std::vector<T> a((size_t)std::max<i64>(n, 1) * std::max<i64>(n, 1));
        A.to_host(a.data(), std::max<i64>(n, 1));
        const bool lo = A.uplo() == Uplo::Lower;
        for (i64 j = 0; j < n; ++j)
            for (i64 i = 0; i < n; ++i) {
                const bool stored = lo ? i >= j : i <= j;
                const T v = stored ? a[i + j * n] : conj_of(a[j + i * n]);
                h[i + j * N] = i == j ? T(std::real(v)) : v;
            }
        for (i64 i = n; i < N; ++i) h[i + i * N] = T(1);
    }
    Scratch Af(sizeof(T) * N * N, s);
    upload(Af.p, h.data(), sizeof(T) * N * N, s);
    auto Ls = std::make_shared<Scratch>(sizeof(T) * N * N, s);
    dzero(Ls->p, sizeof(T) * N * N, s);
    slate_hip::geset<K<T>>('G', nb, nb, kv(T(0)), kv(T(1)), kp(Ls->as<T>()), N, s);
    Scratch Td(sizeof(T) * nb * nb * NT, s), Tl(sizeof(T) * nb * nb * (NT + 1), s);
    dzero(Td.p, sizeof(T) * nb * nb * NT, s);
    dzero(Tl.p, sizeof(T) * nb * nb * (NT + 1), s);
    Scratch piv(sizeof(i64) * N, s), inf(sizeof(i64) * NT, s);
    dzero(piv.p, sizeof(i64) * N, s);
    dzero(inf.p, sizeof(i64) * NT, s);
    aasen<T>(N, nb, Af.as<T>(), Ls->as<T>(), Td.as<T>(), Tl.as<T>(), piv.as<i64>(), inf.as<i64>(), s);
    // the permutation (block 0 keeps its rows; block J + 1's pivots are
    // relative to row (J + 1) nb)
    std::vector<i64> pr((size_t)N);
    NHIP(hipMemcpyAsync(pr.data(), piv.p, sizeof(i64) * N, hipMemcpyDeviceToHost, s));
    std::vector<T> htd((size_t)nb * nb * NT), htl((size_t)nb * nb * (NT + 1));
    NHIP(hipMemcpyAsync(htd.data(), Td.p, sizeof(T) * htd.size(), hipMemcpyDeviceToHost, s));
    NHIP(hipMemcpyAsync(htl.data(), Tl.p, sizeof(T) * htl.size(), hipMemcpyDeviceToHost, s));
    NHIP(hipStreamSynchronize(s));
    auto d = std::make_shared<IndefData>();
    d->n = n; d->N = N; d->nb = nb; d->p = SA.p; d->q = SA.q;
    d->perm.resize((size_t)N);
    for (i64 i = 0; i < N; ++i) d->perm[i] = i;
    for (i64 i = nb; i < N; ++i) {
        const i64 j = (i / nb) * nb + pr[i];
        if (j != i) std::swap(d->perm[i], d->perm[j]);
    }
    // T (kl = ku = nb) in LAPACK band layout, then its band LU
    const i64 ldab = 3 * nb + 1, off = nb;      // AB(off + i - j, j)
    std::vector<T> ab((size_t)ldab * N, T(0));
    for (i64 J = 0; J < NT; ++J)
        for (i64 c = 0; c < nb; ++c)
            for (i64 r = 0; r < nb; ++r) {
                const i64 i = J * nb + r, j = J * nb + c;
                ab[(off + i - j) + j * ldab] = htd[(size_t)J * nb * nb + r + c * nb];
                if (J + 1 < NT) {
                    const T lo = htl[(size_t)(J + 1) * nb * nb + r + c * nb];     // T(J+1, J)(r, c)
                    const i64 il = (J + 1) * nb + r;
                    if (il - j <= nb) ab[(off + il - j) + j * ldab] = lo;
                    const i64 ju = (J + 1) * nb + r, iu = J * nb + c;            // T(J, J+1) = T(J+1, J)^H
                    if (ju - iu <= nb) ab[(off + iu - ju) + ju * ldab] = conj_of(lo);
                }
            }
    auto Tb = std::make_shared<BandMatrix<T>>(N, N, nb, nb, nb);
    Tb->from_host_band(ab.data(), ldab, off);
    const int64_t info = gbtrf<T>(*Tb, d->Tpiv);
    d->L = Ls;
    d->Tband = Tb;
    F.d = d;
    return info;
}

template <typename T>
int64_t hetrs(const IndefiniteFactors<T>& F, Matrix<T>& B, const Options&) {
    NTRACE("hetrs", nullptr);
    if (!F.d) throw Error("native hetrs: factors of hetrf expected");
    const IndefData& d = *F.d;
    hipStream_t s = rt().main;
    const i64 n = d.n, N = d.N, nr = B.n();
    if (B.m() != n) throw Error("native hetrs: B must have n rows");
    const T* L = static_cast<Scratch*>(d.L.get())->template as<T>();
    std::vector<T> hb((size_t)std::max<i64>(n, 1) * std::max<i64>(nr, 1));
    B.to_host(hb.data(), std::max<i64>(n, 1));
    // P b (padded rows zero)
    std::vector<T> y((size_t)N * nr, T(0));
    for (i64 c = 0; c < nr; ++c)
        for (i64 i = 0; i < N; ++i) {
            const i64 src = d.perm[i];
            y[i + c * N] = src < n ? hb[src + c * n] : T(0);
        }
    Scratch Y(sizeof(T) * std::max<i64>(N * nr, 1), s);
    upload(Y.p, y.data(), sizeof(T) * N * nr, s);
    slate_hip::trsm<K<T>>('L', 'L', 'N', 'U', N, nr, kv(T(1)), kp(L), N, kp(Y.as<T>()), N, s);
    // T z = y with the band LU of T (any grid: B's)
    Matrix<T> Z(N, nr, B.nb(), B.p(), B.q());
    NHIP(hipMemcpyAsync(y.data(), Y.p, sizeof(T) * N * nr, hipMemcpyDeviceToHost, s));
    NHIP(hipStreamSynchronize(s));
    Z.from_host(y.data(), N);
    gbtrs<T>(*static_cast<BandMatrix<T>*>(d.Tband.get()), d.Tpiv, Z);
    Z.to_host(y.data(), N);
    upload(Y.p, y.data(), sizeof(T) * N * nr, s);
    slate_hip::trsm<K<T>>('L', 'L', ctrans<T>(), 'U', N, nr, kv(T(1)), kp(L), N, kp(Y.as<T>()), N, s);
    NHIP(hipMemcpyAsync(y.data(), Y.p, sizeof(T) * N * nr, hipMemcpyDeviceToHost, s));
    NHIP(hipStreamSynchronize(s));
    // x = P^T z
    for (i64 c = 0; c < nr; ++c)
        for (i64 i = 0; i < N; ++i)
            if (d.perm[i] < n) hb[d.perm[i] + c * n] = y[i + c * N];
    B.from_host(hb.data(), std::max<i64>(n, 1));
    return 0;
}

template <typename T>
int64_t hesv(HermitianMatrix<T>& A, Matrix<T>& B, const Options& opts) {
    IndefiniteFactors<T> F;
    const int64_t info = hetrf<T>(A, F, opts);
    if (info == 0) hetrs<T>(F, B, opts);
    return info;
}

template <typename T>
void scale(real_t<T> numer, real_t<T> denom, Matrix<T>& A) {
    using R = real_t<T>;
    if (denom == R(0)) throw Error("native scale: denom == 0");
    const Storage& S = *A.storage();
    hipStream_t s = rt().main;
    // numer / denom in up to two factors so that neither overflows
    R f1 = numer / denom, f2 = R(1);
    if (!std::isfinite((double)f1) && std::isfinite((double)numer)) {
        f1 = numer / R(2);
        f2 = R(2) / denom;
    }
    if (S.mloc && S.nloc) {
        slate_hip::gescale<K<T>>('G', S.mloc, S.nloc, kv(T(f1)), kp(static_cast<T*>(S.buf)), S.lld, s);
        if (f2 != R(1)) slate_hip::gescale<K<T>>('G', S.mloc, S.nloc, kv(T(f2)), kp(static_cast<T*>(S.buf)), S.lld, s);
    }
    NHIP(hipStreamSynchronize(s));
}

// ------------------------------------------------------------ matrix model
// Matrix::slice / set_slice: the element range at any offset moves to / from
// a new aligned matrix of the same grid and tile size with the value
// redistribution of the ScaLAPACK shims (capi_util.hpp scal_move: every
// value goes straight to its new owner, host-staged)
template <typename T>
Matrix<T> Matrix<T>::slice(int64_t i0, int64_t i1, int64_t j0, int64_t j1) const {
    const Storage& S = *storage();
    if (i0 < 0 || j0 < 0 || i1 > S.m || j1 > S.n || i0 > i1 || j0 > j1) throw Error("Matrix::slice: range outside");
    Matrix<T> R(i1 - i0, j1 - j0, S.nb, S.p, S.q);
    const Storage& SR = *R.storage();
    const i64 lda = std::max<i64>(S.mloc, 1), ldr = std::max<i64>(SR.mloc, 1);
    std::vector<T> a((size_t)lda * std::max<i64>(S.nloc, 1)), r((size_t)ldr * std::max<i64>(SR.nloc, 1));
    if (S.mloc && S.nloc) to_local_host(a.data(), lda);
    const capi::ScalLay L{S.m, S.n, S.nb, S.nb, lda, 0, 0, S.p, S.q, false};
    capi::scal_move<T>(L, i0, j0, i1 - i0, j1 - j0, a.data(), SR, r.data(), ldr, true);
    if (SR.mloc && SR.nloc) R.from_local_host(r.data(), ldr);
    return R;
}

template <typename T>
void Matrix<T>::set_slice(int64_t i0, int64_t j0, const Matrix<T>& Sv) {
    const Storage& S = *storage();
    const Matrix<T> Sm = Sv.op() == Op::NoTrans ? Sv : [&] {
        Matrix<T> M(Sv.m(), Sv.n(), Sv.nb(), Sv.p(), Sv.q());
        copy<T>(Op::NoTrans, Sv, M);
        return M;
    }();
    const Storage& SR = *Sm.storage();
    if (SR.p != S.p || SR.q != S.q || SR.nb != S.nb) throw Error("Matrix::set_slice: same grid and tile size");
    if (i0 < 0 || j0 < 0 || i0 + SR.m > S.m || j0 + SR.n > S.n) throw Error("Matrix::set_slice: range outside");
    const i64 lda = std::max<i64>(S.mloc, 1), ldr = std::max<i64>(SR.mloc, 1);
    std::vector<T> a((size_t)lda * std::max<i64>(S.nloc, 1)), r((size_t)ldr * std::max<i64>(SR.nloc, 1));
    if (S.mloc && S.nloc) to_local_host(a.data(), lda);
    if (SR.mloc && SR.nloc) Sm.to_local_host(r.data(), ldr);
    const capi::ScalLay L{S.m, S.n, S.nb, S.nb, lda, 0, 0, S.p, S.q, false};
    capi::scal_move<T>(L, i0, j0, SR.m, SR.n, a.data(), SR, r.data(), ldr, false);
    if (S.mloc && S.nloc) from_local_host(a.data(), lda);
}

template <typename T>
Matrix<T> Matrix<T>::emptyLike() const {
    return Matrix<T>(m(), n(), nb(), p(), q());
}

// structured overloads: the stored triangle and the view's op map onto the
// enum-argument drivers (trsm / trmm take op(A) of a view directly)
template <typename T>
void trsm(Side side, T alpha, const TriangularMatrix<T>& A, Matrix<T>& B, const Options& opts) {
    trsm<T>(side, A.uplo_physical(), Op::NoTrans, A.diag(), alpha, A, B, opts);
}
template <typename T>
void trmm(Side side, T alpha, const TriangularMatrix<T>& A, Matrix<T>& B, const Options& opts) {
    trmm<T>(side, A.uplo_physical(), Op::NoTrans, A.diag(), alpha, A, B, opts);
}
template <typename T>
int64_t trtri(TriangularMatrix<T>& A, const Options& opts) {
    Matrix<T>& M = A;
    return trtri<T>(A.uplo_physical(), A.diag(), M, opts);
}
// trapezoid / triangular norm: the stored trapezoid of any m x n (masked
// copy, a Unit diagonal set), then the general norm -- of op(A) for a view
template <typename T>
double norm(Norm kind, const TrapezoidMatrix<T>& A) {
    const Matrix<T> B = A.base();
    const Storage& S = *B.storage();
    if (S.m == S.n) {
        const Matrix<T> F = expand_tri<T>(B, A.uplo_physical(), 0, A.diag());
        return norm<T>(kind, A.op() == Op::NoTrans ? F : transpose(F));
    }
    Matrix<T> F(S.m, S.n, S.nb, S.p, S.q);
    Storage& SF = *F.storage();
    hipStream_t s = rt().main;
    slate_hip::TriMask mk = lower_mask(S.nb, S.p, S.pr, S.q, S.pc, 0, 0);
    if (A.uplo_physical() == Uplo::Upper) mk.mode = 2;
    const bool unit = A.diag() == Diag::Unit;
    mk.diag_off = unit ? -1 : 0;
    if (S.mloc && S.nloc)
        slate_hip::gecopy_mask<K<T>>(mk, S.mloc, S.nloc, kp(static_cast<const T*>(S.buf)), S.lld,
                                     kp(static_cast<T*>(SF.buf)), SF.lld, false, s);
    NHIP(hipStreamSynchronize(s));
    if (unit) {
        // ones on the global diagonal: F += I (the masked copy left it zero)
        Matrix<T> I(S.m, S.n, S.nb, S.p, S.q);
        set<T>(T(0), T(1), I);
        add<T>(T(1), I, T(1), F);
    }
    return norm<T>(kind, A.op() == Op::NoTrans ? F : transpose(F));
}
template <typename T>
double norm(Norm kind, const SymmetricMatrix<T>& A) {
    return norm_symmetric<T>(kind, HermitianMatrix<T>(A.uplo_physical(), A.base()));
}
template <typename T>
void symm(Side side, T alpha, const SymmetricMatrix<T>& A, const Matrix<T>& B, T beta, Matrix<T>& C,
          const Options& opts) {
    symm<T>(side, alpha, HermitianMatrix<T>(A.uplo_physical(), A.base()), B, beta, C, opts);
}
template <typename T>
void syrk(T alpha, const Matrix<T>& A, T beta, SymmetricMatrix<T>& C, const Options& opts) {
    HermitianMatrix<T> H(C.uplo_physical(), C.base());
    syrk<T>(Op::NoTrans, alpha, A, beta, H, opts);
}
template <typename T>
void herk(real_t<T> alpha, const Matrix<T>& A, real_t<T> beta, HermitianMatrix<T>& C, const Options& opts) {
    herk<T>(Op::NoTrans, alpha, A, beta, C, opts);
}
template <typename T>
void syr2k(T alpha, const Matrix<T>& A, const Matrix<T>& B, T beta, SymmetricMatrix<T>& C, const Options& opts) {
    HermitianMatrix<T> H(C.uplo_physical(), C.base());
    syr2k<T>(Op::NoTrans, alpha, A, B, beta, H, opts);
}
template <typename T>
void her2k(T alpha, const Matrix<T>& A, const Matrix<T>& B, real_t<T> beta, HermitianMatrix<T>& C,
           const Options& opts) {
    her2k<T>(Op::NoTrans, alpha, A, B, beta, C, opts);
}

// ------------------------------------------------------------ instantiation
#define SLATE_NATIVE_EXT(T)                                                                                    \
    template void hegst<T>(int64_t, HermitianMatrix<T>&, const HermitianMatrix<T>&, const Options&);            \
    template int64_t hegv<T>(int64_t, HermitianMatrix<T>&, HermitianMatrix<T>&, std::vector<real_t<T>>&,        \
                             Matrix<T>&, const Options&);                                                       \
    template int64_t hegv<T>(int64_t, HermitianMatrix<T>&, HermitianMatrix<T>&, std::vector<real_t<T>>&,        \
                             const Options&);                                                                   \
    template int64_t gesv_rbt<T>(Matrix<T>&, Matrix<T>&, const Options&);                                      \
    template int64_t getrs_nopiv<T>(const Matrix<T>&, Matrix<T>&, const Options&);                             \
    template int64_t hesv<T>(HermitianMatrix<T>&, Matrix<T>&, const Options&);                                 \
    template int64_t hetrf<T>(const HermitianMatrix<T>&, IndefiniteFactors<T>&, const Options&);               \
    template int64_t hetrs<T>(const IndefiniteFactors<T>&, Matrix<T>&, const Options&);                        \
    template void scale<T>(real_t<T>, real_t<T>, Matrix<T>&);                                                  \
    template Matrix<T> Matrix<T>::slice(int64_t, int64_t, int64_t, int64_t) const;                             \
    template void Matrix<T>::set_slice(int64_t, int64_t, const Matrix<T>&);                                    \
    template Matrix<T> Matrix<T>::emptyLike() const;                                                           \
    template void trsm<T>(Side, T, const TriangularMatrix<T>&, Matrix<T>&, const Options&);                   \
    template void trmm<T>(Side, T, const TriangularMatrix<T>&, Matrix<T>&, const Options&);                   \
    template int64_t trtri<T>(TriangularMatrix<T>&, const Options&);                                          \
    template double norm<T>(Norm, const TrapezoidMatrix<T>&);                                                 \
    template double norm<T>(Norm, const SymmetricMatrix<T>&);                                                 \
    template void symm<T>(Side, T, const SymmetricMatrix<T>&, const Matrix<T>&, T, Matrix<T>&, const Options&); \
    template void syrk<T>(T, const Matrix<T>&, T, SymmetricMatrix<T>&, const Options&);                        \
    template void herk<T>(real_t<T>, const Matrix<T>&, real_t<T>, HermitianMatrix<T>&, const Options&);        \
    template void syr2k<T>(T, const Matrix<T>&, const Matrix<T>&, T, SymmetricMatrix<T>&, const Options&);     \
    template void her2k<T>(T, const Matrix<T>&, const Matrix<T>&, real_t<T>, HermitianMatrix<T>&, const Options&);
SLATE_NATIVE_EXT(float)
SLATE_NATIVE_EXT(double)
SLATE_NATIVE_EXT(std::complex<float>)
SLATE_NATIVE_EXT(std::complex<double>)
#undef SLATE_NATIVE_EXT
#define SLATE_NATIVE_GMRES(T)                                                                                  \
    template int64_t gesv_mixed_gmres<T>(Matrix<T>&, std::vector<int64_t>&, Matrix<T>&, Matrix<T>&, int&,      \
                                         const Options&);                                                       \
    template int64_t posv_mixed_gmres<T>(HermitianMatrix<T>&, Matrix<T>&, Matrix<T>&, int&, const Options&);
SLATE_NATIVE_GMRES(double)
SLATE_NATIVE_GMRES(std::complex<double>)
#undef SLATE_NATIVE_GMRES

}  // namespace native
}  // namespace slate_amd
