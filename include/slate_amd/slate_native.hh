// slate_amd native C++ API: distributed tiled matrices and the core dense
// linear algebra routines WITHOUT the Python runtime.
//
// libslate_amd_native.so is the gfx950 HIP kernels of the package plus a
// C++ host runtime (process bootstrap, communicators, HIP stream/event
// lookahead pipelines) -- it links against libamdhip64 and librccl only.
// It mirrors the reference's public C++ interface for the routines it
// covers (include/slate/slate.hh: potrf/potrs/posv, getrf/getrs/gesv, gemm,
// trsm, norm; include/slate/Matrix.hh / HermitianMatrix.hh for the matrix
// types), in the four precisions float, double, std::complex<float>,
// std::complex<double> (src/potrf.cc:285-303 instantiates the same four).
// The LAPACK (dgetrf_, ...), ScaLAPACK (pdpotrf_, ...) and BLACS symbols of
// the library call these drivers directly (capi_native.hip).
//
// One process per GPU.  The world is taken from the torchrun-style
// environment (RANK, WORLD_SIZE, LOCAL_RANK, MASTER_ADDR; bootstrap sockets
// on SLATE_AMD_NATIVE_PORT, default MASTER_PORT + 1 -- torchrun's own store
// holds MASTER_PORT).  SLATE_AMD_NATIVE_TRANSPORT = rccl (default: RCCL over
// xGMI) or host (host-staged TCP: several ranks may share one GPU, e.g. a
// 2 x 2 grid rehearsed on one device).  A single process needs no
// environment at all and never initialises a transport.
//
//   slate_amd::native::initialize();
//   slate_amd::native::HermitianMatrix<double> A(slate_amd::native::Uplo::Lower, n, nb, p, q);
//   A.generate(slate_amd::native::Gen::HermitianPositiveDefinite, 7);
//   int64_t info = slate_amd::native::potrf(A);
//
// Matrices are 2D block-cyclic over a p x q column-major process grid
// (rank = pr + pc p), nb x nb tiles; each rank owns one column-major device
// buffer with its local rows / columns (ScaLAPACK local layout).
#ifndef SLATE_AMD_NATIVE_HH
#define SLATE_AMD_NATIVE_HH

#include <complex>
#include <cstdint>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace slate_amd {
namespace native {

class Error : public std::runtime_error {
public:
    explicit Error(const std::string& what) : std::runtime_error(what) {}
};

enum class Uplo : char { Lower = 'L', Upper = 'U' };
enum class Op : char { NoTrans = 'N', Trans = 'T', ConjTrans = 'C' };
enum class Diag : char { NonUnit = 'N', Unit = 'U' };
enum class Side : char { Left = 'L', Right = 'R' };
enum class Norm : char { One = '1', Inf = 'I', Fro = 'F', Max = 'M' };
// matgen kinds (same Philox counter-based generator as the Python package:
// an entry depends on (seed, global i, global j) only)
enum class Gen : int { Random = 11, HermitianPositiveDefinite = 21, DiagDominant = 20 };

// process runtime
void initialize();            // idempotent; called by every constructor
void finalize();              // destroys communicators and streams
int rank();
int size();
const char* version();
const char* transport();      // "none" (one rank), "rccl" or "host"
void barrier();               // all ranks, device work of this rank completed
double allreduce_max(double v);   // maximum over all ranks

// tracing (SLATE Trace, src/auxiliary/Trace.cc): host spans and per-stream
// device spans of the drivers' phases (potrf::panel / bcast / lookahead /
// update, getrf::panel / update, gemm::summa, ...); finish() gathers every
// rank's events to rank 0, which writes one Chrome trace-event JSON (pid =
// rank, tid = stream).  SLATE_AMD_NATIVE_TRACE=<path> traces from
// initialize() to finalize().
namespace trace {
void on();
void off();
bool enabled();
void finish(const std::string& path);     // collective
}  // namespace trace
// seconds per traced scope name (slate::timers): host wall time of every
// scope, and "<name>@device" device time of the spans resolved so far
std::map<std::string, double> timers();
void clear_timers();

struct Options {
    int lookahead = 1;        // SLATE Option::Lookahead
    double pivot_threshold = 1.0;
    int inner_blocking = 32;  // columns per base block of the distributed LU panel
    int depth = 2;            // SLATE Option::Depth: butterfly levels of gesv_rbt (1..4)
    int max_iterations = 30;  // SLATE Option::MaxIterations: refinement / GMRES steps
    int restart = 30;         // GMRES restart length (gesv/posv_mixed_gmres)
    int lu_method = 0;        // SLATE MethodLU: 0 partial pivoting, 1 CALU (tournament pivoting)
    int calu_leaf = 2048;     // rows per first-round CALU play-off (>= 2 nb is enforced)
};

struct Storage;               // opaque: device buffer, grid, communicators

template <typename T>
class Matrix {
public:
    Matrix() = default;
    Matrix(int64_t m, int64_t n, int64_t nb, int p = 1, int q = 1);
    // dimensions of the matrix as seen through its op (a transposed view of
    // an m x n matrix is n x m); nb / p / q / mloc / nloc / lld / data refer
    // to the storage
    int64_t m() const;
    int64_t n() const;
    int64_t nb() const;
    int p() const;
    int q() const;
    int64_t mloc() const;     // local rows / columns of this rank (storage)
    int64_t nloc() const;
    int64_t lld() const;      // leading dimension of the local buffer
    T* data();                // device pointer to the local buffer
    const T* data() const;
    void generate(Gen kind, uint64_t seed);
    // Global column-major host array, identical on every rank (LAPACK
    // layout): copy this rank's block-cyclic part to the device / gather the
    // whole matrix to every rank (one all-gather of the local blocks).
    void from_host(const T* A, int64_t lda);
    void to_host(T* A, int64_t lda) const;
    // This rank's local block in ScaLAPACK layout (host, leading dim lld).
    void from_local_host(const T* Aloc, int64_t lld);
    void to_local_host(T* Aloc, int64_t lld) const;
    // the storage of a plain (op NoTrans) matrix; a transposed view throws:
    // every driver that does not take op(A) directly rejects views instead
    // of silently reading the untransposed data (materialise with copy())
    std::shared_ptr<Storage> storage() const;
    std::shared_ptr<Storage> storage_any() const { return s_; }
    // Zero-copy wrapper of a DEVICE buffer that holds this rank's local block
    // in ScaLAPACK layout (SLATE fromScaLAPACK / fromDevices); the caller
    // keeps ownership, lld >= mloc (an even lld keeps the 16-byte MFMA loads).
    static Matrix from_device(T* d_local, int64_t lld, int64_t m, int64_t n, int64_t nb, int p = 1, int q = 1);
    // View of the tiles [i0, i1) x [j0, j1) sharing this storage (SLATE
    // Matrix::sub); i0 a multiple of p and j0 of q, so the view's tile (0, 0)
    // stays on process (0, 0) and every driver takes it as it is.
    Matrix sub(int64_t i0, int64_t i1, int64_t j0, int64_t j1) const;
    // The elements [i0, i1) x [j0, j1) at ANY offset (SLATE Matrix::slice):
    // a block-cyclic layout cannot start inside a tile, so this is a copy on
    // the same grid and tile size (each value travels to its new owner,
    // nothing else); set_slice writes such a matrix back at (i0, j0).
    Matrix slice(int64_t i0, int64_t i1, int64_t j0, int64_t j1) const;
    void set_slice(int64_t i0, int64_t j0, const Matrix& S);
    // a zeroed matrix of the same (op-applied) shape, grid and tile size
    // (SLATE emptyLike)
    Matrix emptyLike() const;
    // transposition state (SLATE BaseMatrix::op): transpose() /
    // conj_transpose() below return views sharing the storage
    Op op() const { return op_; }
    // the same storage seen untransposed
    Matrix base() const {
        Matrix b(*this);
        b.op_ = Op::NoTrans;
        return b;
    }
    // compose the view's op with o (T T = N, C C = N; a conjugation alone
    // is not a view and throws)
    void apply_op(Op o);

protected:
    std::shared_ptr<Storage> s_;
    Op op_ = Op::NoTrans;
};

// transposed / conjugate-transposed VIEWS (SLATE transpose / conj_transpose,
// BaseMatrix.hh:768-795): same storage, same class (a TriangularMatrix stays
// one, its logical uplo flips).  gemm, copy, trsm, trmm, herk / syrk,
// her2k / syr2k, norm and add take views directly; other drivers reject them.
template <typename MT>
MT transpose(const MT& A) {
    MT B(A);
    B.apply_op(Op::Trans);
    return B;
}
template <typename MT>
MT conj_transpose(const MT& A) {
    MT B(A);
    B.apply_op(Op::ConjTrans);
    return B;
}

template <typename T>
class HermitianMatrix : public Matrix<T> {
public:
    HermitianMatrix() = default;
    HermitianMatrix(Uplo uplo, int64_t n, int64_t nb, int p = 1, int q = 1)
        : Matrix<T>(n, n, nb, p, q), uplo_(uplo) {}
    // the uplo triangle of a square matrix or view, sharing its storage
    HermitianMatrix(Uplo uplo, const Matrix<T>& A) : Matrix<T>(A), uplo_(uplo) {}
    Uplo uplo() const { return uplo_; }

private:
    Uplo uplo_ = Uplo::Lower;
};

// structured matrices (SLATE TrapezoidMatrix / TriangularMatrix /
// SymmetricMatrix, include/slate/TriangularMatrix.hh:30-684): a general
// storage plus the referenced triangle; uplo() is the LOGICAL triangle of
// the (possibly transposed) view, uplo_physical() the stored one
inline Uplo flip_uplo(Uplo u) { return u == Uplo::Lower ? Uplo::Upper : Uplo::Lower; }
template <typename T>
class TrapezoidMatrix : public Matrix<T> {
public:
    TrapezoidMatrix() = default;
    TrapezoidMatrix(Uplo uplo, Diag diag, int64_t m, int64_t n, int64_t nb, int p = 1, int q = 1)
        : Matrix<T>(m, n, nb, p, q), uplo_(uplo), diag_(diag) {}
    TrapezoidMatrix(Uplo uplo, Diag diag, const Matrix<T>& A) : Matrix<T>(A), uplo_(uplo), diag_(diag) {}
    Uplo uplo() const { return this->op() == Op::NoTrans ? uplo_ : flip_uplo(uplo_); }
    Uplo uplo_physical() const { return uplo_; }
    Diag diag() const { return diag_; }

private:
    Uplo uplo_ = Uplo::Lower;
    Diag diag_ = Diag::NonUnit;
};
template <typename T>
class TriangularMatrix : public TrapezoidMatrix<T> {
public:
    TriangularMatrix() = default;
    TriangularMatrix(Uplo uplo, Diag diag, int64_t n, int64_t nb, int p = 1, int q = 1)
        : TrapezoidMatrix<T>(uplo, diag, n, n, nb, p, q) {}
    TriangularMatrix(Uplo uplo, Diag diag, const Matrix<T>& A) : TrapezoidMatrix<T>(uplo, diag, A) {}
};
template <typename T>
class SymmetricMatrix : public Matrix<T> {
public:
    SymmetricMatrix() = default;
    SymmetricMatrix(Uplo uplo, int64_t n, int64_t nb, int p = 1, int q = 1) : Matrix<T>(n, n, nb, p, q), uplo_(uplo) {}
    SymmetricMatrix(Uplo uplo, const Matrix<T>& A) : Matrix<T>(A), uplo_(uplo) {}
    Uplo uplo() const { return this->op() == Op::NoTrans ? uplo_ : flip_uplo(uplo_); }
    Uplo uplo_physical() const { return uplo_; }

private:
    Uplo uplo_ = Uplo::Lower;
};

// ---- drivers, T in {float, double, std::complex<float>, std::complex<double>}.
// Return LAPACK info (0 = success).
// Cholesky (Lower storage; Upper: factor the conjugate transpose), p x q
template <typename T> int64_t potrf(HermitianMatrix<T>& A, const Options& opts = {});
template <typename T> int64_t potrs(const HermitianMatrix<T>& A, Matrix<T>& B, const Options& opts = {});
template <typename T> int64_t posv(HermitianMatrix<T>& A, Matrix<T>& B, const Options& opts = {});
// LU with partial pivoting on p x q grids (p > 1: the panel rows stay on
// their owners, one record all-gather per column); ipiv (global, 0-based,
// LAPACK-style sequential interchanges) is returned on every rank
template <typename T> int64_t getrf(Matrix<T>& A, std::vector<int64_t>& ipiv, const Options& opts = {});
template <typename T>
int64_t getrs(const Matrix<T>& A, const std::vector<int64_t>& ipiv, Matrix<T>& B, const Options& opts = {});
// op(A) X = B with the factors of getrf; trans NoTrans or ConjTrans (real
// types: Trans == ConjTrans)
template <typename T>
int64_t getrs(Op trans, const Matrix<T>& A, const std::vector<int64_t>& ipiv, Matrix<T>& B,
              const Options& opts = {});
template <typename T> int64_t gesv(Matrix<T>& A, std::vector<int64_t>& ipiv, Matrix<T>& B, const Options& opts = {});
// C = alpha A B + beta C, SUMMA on the grid with lookahead broadcasts
template <typename T>
void gemm(T alpha, const Matrix<T>& A, const Matrix<T>& B, T beta, Matrix<T>& C, const Options& opts = {});
// C = alpha op(A) op(B) + beta C (transposed operands are redistributed
// once, tile by tile, then the SUMMA above runs)
template <typename T>
void gemm(Op opA, Op opB, T alpha, const Matrix<T>& A, const Matrix<T>& B, T beta, Matrix<T>& C,
          const Options& opts = {});
// B = op(A) (B: n x m for Trans / ConjTrans), same grid and tile size
template <typename T> void copy(Op op, const Matrix<T>& A, Matrix<T>& B);
// B = A between ANY two block-cyclic layouts of the same global shape (tile
// sizes and p x q grids may differ): one batched point-to-point exchange of
// the separable owner blocks (SLATE redistribute, slate.hh:426)
template <typename T> void redistribute(const Matrix<T>& A, Matrix<T>& B);
// B = alpha op(A)^{-1} B, A triangular (the uplo triangle of A's storage),
// Side::Left, op NoTrans or ConjTrans; distributed forward / backward
// substitution by tile steps
template <typename T>
void trsm(Side side, Uplo uplo, Op op, Diag diag, T alpha, const Matrix<T>& A, Matrix<T>& B,
          const Options& opts = {});
template <typename T> double norm(Norm kind, const Matrix<T>& A);

// B = alpha A + beta B; A = offdiag everywhere, diag on the global diagonal
template <typename T> void add(T alpha, const Matrix<T>& A, T beta, Matrix<T>& B);
template <typename T> void set(T offdiag, T diag, Matrix<T>& A);

// norms of a stored triangle: Hermitian, symmetric, triangular (square)
template <typename T> double norm(Norm kind, const HermitianMatrix<T>& A);
template <typename T> double norm_symmetric(Norm kind, const HermitianMatrix<T>& A);
template <typename T> double norm_triangular(Norm kind, Uplo uplo, Diag diag, const Matrix<T>& A);

// real type of a scalar (herk / her2k scaling factors)
template <typename T> struct real_of { using type = T; };
template <typename R> struct real_of<std::complex<R>> { using type = R; };
template <typename T> using real_t = typename real_of<T>::type;

// C = alpha op(A) op(A)^H + beta C on C's stored triangle (op: NoTrans / ConjTrans)
template <typename T>
void herk(Op op, real_t<T> alpha, const Matrix<T>& A, real_t<T> beta, HermitianMatrix<T>& C,
          const Options& opts = {});
// C = alpha op(A) op(A)^T + beta C (C symmetric, stored triangle; op: NoTrans / Trans)
template <typename T>
void syrk(Op op, T alpha, const Matrix<T>& A, T beta, HermitianMatrix<T>& C, const Options& opts = {});
// C = alpha op(A) op(B)^H + conj(alpha) op(B) op(A)^H + beta C
template <typename T>
void her2k(Op op, T alpha, const Matrix<T>& A, const Matrix<T>& B, real_t<T> beta, HermitianMatrix<T>& C,
           const Options& opts = {});
// C = alpha op(A) op(B)^T + alpha op(B) op(A)^T + beta C
template <typename T>
void syr2k(Op op, T alpha, const Matrix<T>& A, const Matrix<T>& B, T beta, HermitianMatrix<T>& C,
           const Options& opts = {});
// C = alpha A B + beta C (Left) or alpha B A + beta C (Right), A Hermitian (hemm) / symmetric (symm)
template <typename T>
void hemm(Side side, T alpha, const HermitianMatrix<T>& A, const Matrix<T>& B, T beta, Matrix<T>& C,
          const Options& opts = {});
template <typename T>
void symm(Side side, T alpha, const HermitianMatrix<T>& A, const Matrix<T>& B, T beta, Matrix<T>& C,
          const Options& opts = {});
// B = alpha op(A) B (Left) or alpha B op(A) (Right), A triangular (uplo, diag)
template <typename T>
void trmm(Side side, Uplo uplo, Op op, Diag diag, T alpha, const Matrix<T>& A, Matrix<T>& B,
          const Options& opts = {});

// Householder QR on any p x q grid: A = Q R, R in the upper triangle, the
// reflectors below it; F keeps the per-panel compact-WY factors T (device).
// With p > 1 process rows each panel is a TSQR -- every rank of the panel's
// process column factors its own rows, the stacked R factors are reduced by
// one more QR, and F also keeps that tree's reflectors.  unmqr applies
// op(Q) (NoTrans or ConjTrans; real types: Trans == ConjTrans) from the
// left; gels solves min ||A X - B|| for m >= n (X in the top n rows of BX).
// inverses from the factors: potri after potrf (stored triangle), getri after getrf
template <typename T> int64_t potri(HermitianMatrix<T>& A, const Options& opts = {});
template <typename T> int64_t getri(Matrix<T>& A, const std::vector<int64_t>& ipiv, const Options& opts = {});
// p > 1 getrf moves only the rows that change process row: bytes this rank
// sent and rows that crossed since the previous call
void lu_exchange_stats(long long* bytes, long long* rows);
// triangular inverse in place (stored triangle; Unit: the diagonal is not
// referenced) and the triangular product A <- L^H L (Lower) / U U^H (Upper)
template <typename T> int64_t trtri(Uplo uplo, Diag diag, Matrix<T>& A, const Options& opts = {});
template <typename T> void trtrm(Uplo uplo, Matrix<T>& A, const Options& opts = {});
// LU with tournament pivoting (SLATE getrf_tntpiv, MethodLU::CALU): every
// panel's pivot rows are chosen by a play-off -- partial-pivoting LU of
// row blocks, the winners of each block (on every rank of the panel's
// process column) meet in the next round, the last round runs redundantly
// on the column -- then the panel is factored without further pivoting.
template <typename T> int64_t getrf_tntpiv(Matrix<T>& A, std::vector<int64_t>& ipiv, const Options& opts = {});
// LU without pivoting (SLATE getrf_nopiv / gesv_nopiv): unit-lower L and U in A
template <typename T> int64_t getrf_nopiv(Matrix<T>& A, const Options& opts = {});
template <typename T> int64_t gesv_nopiv(Matrix<T>& A, Matrix<T>& B, const Options& opts = {});
// Cholesky QR (SLATE cholqr): A (m x n, m >= n) <- Q, R (n x n) <- the upper
// triangular factor (zero below); info > 0 when A^H A is not positive definite
template <typename T> int64_t cholqr(Matrix<T>& A, Matrix<T>& R, const Options& opts = {});

// mixed precision (double / complex<double> only): factor in float /
// complex<float>, refine in the working precision; X = A^-1 B, B unchanged;
// iter = refinement steps, < 0 when the working-precision solve ran instead
template <typename T>
int64_t posv_mixed(HermitianMatrix<T>& A, Matrix<T>& B, Matrix<T>& X, int& iter, const Options& opts = {});
template <typename T>
int64_t gesv_mixed(Matrix<T>& A, std::vector<int64_t>& ipiv, Matrix<T>& B, Matrix<T>& X, int& iter,
                   const Options& opts = {});

// reciprocal condition number estimates (Hager / Higham 1-norm estimator,
// LAPACK lacn2; reference slate.hh gecondest / pocondest / trcondest):
// gecondest from the LU factors of getrf (the interchanges do not change the
// norm), pocondest from the Cholesky factor of potrf (Lower storage), trcondest
// of a triangular matrix (the uplo triangle of A); Anorm = the norm of the
// ORIGINAL matrix in the same norm (One or Inf).  rcond = 1 / (Anorm ||A^-1||).
template <typename T> double gecondest(Norm norm, const Matrix<T>& LU, double Anorm, const Options& opts = {});
template <typename T> double pocondest(Norm norm, const HermitianMatrix<T>& L, double Anorm, const Options& opts = {});
template <typename T>
double trcondest(Norm norm, Uplo uplo, Diag diag, const Matrix<T>& A, const Options& opts = {});

// Hermitian / real symmetric eigenproblem (reference slate.hh heev:
// he2hb -> hb2st -> stedc -> back-transforms), A's stored triangle; Lambda =
// the n eigenvalues ascending (every rank), Z = the eigenvectors (same grid
// and tile size as A).  A is not modified.
template <typename T>
int64_t heev(HermitianMatrix<T>& A, std::vector<real_t<T>>& Lambda, Matrix<T>& Z, const Options& opts = {});
template <typename T>
int64_t heev(HermitianMatrix<T>& A, std::vector<real_t<T>>& Lambda, const Options& opts = {});

// singular value decomposition A = U diag(S) VH (reference slate.hh svd:
// ge2tb -> tb2bd -> bdsqr -> back-transforms): S the min(m, n) singular
// values descending (every rank), U m x min(m, n), VH min(m, n) x n on A's
// grid and tile size.  A is not modified.
template <typename T>
int64_t svd(Matrix<T>& A, std::vector<real_t<T>>& S, Matrix<T>& U, Matrix<T>& VH, const Options& opts = {});
template <typename T> int64_t svd(Matrix<T>& A, std::vector<real_t<T>>& S, const Options& opts = {});

// ---- round 6: generalized eigenproblem, GMRES-IR, random butterfly transform
// hegst (reference slate.hh:1138): reduce the generalized Hermitian-definite
// problem to standard form with the Cholesky factor of B held in L (potrf of
// B, its stored triangle): itype 1 A <- L^-1 A L^-H (Lower) / U^-H A U^-1
// (Upper); itype 2, 3 A <- L^H A L / U A U^H.  A's stored triangle is
// referenced, the full Hermitian result is written.
template <typename T>
void hegst(int64_t itype, HermitianMatrix<T>& A, const HermitianMatrix<T>& L, const Options& opts = {});
// hegv (slate.hh:1082): A x = lambda B x (itype 1), A B x = lambda x (2),
// B A x = lambda x (3); B is overwritten by its Cholesky factor, A by the
// standard-form matrix; Z (A's grid) the B-normalised eigenvectors.  info
// > 0: B not positive definite (n + the potrf info, as LAPACK)
template <typename T>
int64_t hegv(int64_t itype, HermitianMatrix<T>& A, HermitianMatrix<T>& B, std::vector<real_t<T>>& Lambda,
             Matrix<T>& Z, const Options& opts = {});
template <typename T>
int64_t hegv(int64_t itype, HermitianMatrix<T>& A, HermitianMatrix<T>& B, std::vector<real_t<T>>& Lambda,
             const Options& opts = {});
// GMRES-based iterative refinement (src/gesv_mixed_gmres.cc,
// posv_mixed_gmres.cc): the low-precision factors precondition restarted
// GMRES on the working-precision system, one right-hand side at a time.
// double / complex<double>; iter = total GMRES steps (< 0: fell back to the
// working-precision solve)
template <typename T>
int64_t gesv_mixed_gmres(Matrix<T>& A, std::vector<int64_t>& ipiv, Matrix<T>& B, Matrix<T>& X, int& iter,
                         const Options& opts = {});
template <typename T>
int64_t posv_mixed_gmres(HermitianMatrix<T>& A, Matrix<T>& B, Matrix<T>& X, int& iter, const Options& opts = {});
// random butterfly transform + LU without pivoting + refinement
// (src/gesv_rbt.cc): B <- A^-1 B; A is overwritten by the factors of the
// transformed (and, when n is not a multiple of the butterfly unit, padded)
// matrix only if n already is that multiple -- otherwise A is unchanged
template <typename T> int64_t gesv_rbt(Matrix<T>& A, Matrix<T>& B, const Options& opts = {});
// Hermitian indefinite factorization (slate.hh hetrf :804, hetrs, hesv):
// blocked left-looking Aasen, P A P^H = L T L^H with T Hermitian block
// tridiagonal (bandwidth nb), T then factored by the band LU (gbtrf).  The
// factorization runs on the device of every rank over the gathered matrix
// (the distributed Aasen is the Python package's hetrf_dist); T's band LU
// and the solves use the native band drivers.  F keeps L, P and T's LU.
struct IndefData;
template <typename T>
struct IndefiniteFactors {
    std::shared_ptr<IndefData> d;
};
template <typename T> int64_t hetrf(const HermitianMatrix<T>& A, IndefiniteFactors<T>& F, const Options& opts = {});
template <typename T> int64_t hetrs(const IndefiniteFactors<T>& F, Matrix<T>& B, const Options& opts = {});
template <typename T> int64_t hesv(HermitianMatrix<T>& A, Matrix<T>& B, const Options& opts = {});
// A <- (numer / denom) A (slate.hh scale), computed without forming the ratio
// when it would overflow
template <typename T> void scale(real_t<T> numer, real_t<T> denom, Matrix<T>& A);
// LU solve with the factors of getrf_nopiv
template <typename T> int64_t getrs_nopiv(const Matrix<T>& A, Matrix<T>& B, const Options& opts = {});

// ---- SLATE-style overloads on the structured types (slate.hh trsm / trmm /
// trtri / norm / symm / syrk / herk / syr2k / her2k taking
// TriangularMatrix / SymmetricMatrix / HermitianMatrix operands); op(A) of a
// view is honoured
template <typename T>
void trsm(Side side, T alpha, const TriangularMatrix<T>& A, Matrix<T>& B, const Options& opts = {});
template <typename T>
void trmm(Side side, T alpha, const TriangularMatrix<T>& A, Matrix<T>& B, const Options& opts = {});
template <typename T> int64_t trtri(TriangularMatrix<T>& A, const Options& opts = {});
template <typename T> double norm(Norm kind, const TrapezoidMatrix<T>& A);
template <typename T> double norm(Norm kind, const SymmetricMatrix<T>& A);
template <typename T>
void symm(Side side, T alpha, const SymmetricMatrix<T>& A, const Matrix<T>& B, T beta, Matrix<T>& C,
          const Options& opts = {});
template <typename T> void syrk(T alpha, const Matrix<T>& A, T beta, SymmetricMatrix<T>& C, const Options& opts = {});
template <typename T>
void herk(real_t<T> alpha, const Matrix<T>& A, real_t<T> beta, HermitianMatrix<T>& C, const Options& opts = {});
template <typename T>
void syr2k(T alpha, const Matrix<T>& A, const Matrix<T>& B, T beta, SymmetricMatrix<T>& C, const Options& opts = {});
template <typename T>
void her2k(T alpha, const Matrix<T>& A, const Matrix<T>& B, real_t<T> beta, HermitianMatrix<T>& C,
           const Options& opts = {});

// ---- band matrices (SLATE BandMatrix / HermitianBandMatrix /
// TriangularBandMatrix, include/slate/BandMatrix.hh; drivers slate.hh gbtrf /
// gbtrs / gbsv :568, pbtrf / pbtrs / pbsv :708, tbsm :304, gbmm :179,
// hbmm :215).  Compact storage: tile columns are dealt 1-D cyclically over
// ALL ranks (column tile k on rank k % size) and each local tile column is
// ONE contiguous device slab of its band tiles, (klt + kut + 1) nb rows --
// memory O(n (kl + ku)) per job, never the dense n x n.  A factorization
// step is one panel on its owner (GPU potrf + trsm, or the persistent LU
// panel over the kb + kl rows that can be non-zero), one broadcast of the
// panel (and pivots), then every rank updates its own tile columns inside
// the band window with one MFMA GEMM each.  Solves and products keep the
// dense operand replicated on every rank (host-staged, O(n nrhs)), which
// is what band problems with few right-hand sides need.
struct BandStorage;
template <typename T>
class BandMatrix {
public:
    BandMatrix() = default;
    // m x n, lower / upper bandwidths kl / ku, nb x nb tiles
    BandMatrix(int64_t m, int64_t n, int64_t kl, int64_t ku, int64_t nb);
    int64_t m() const;
    int64_t n() const;
    int64_t nb() const;
    int64_t lower_bandwidth() const;
    int64_t upper_bandwidth() const;
    // the band of a dense column-major host array (identical on every
    // rank); to_host writes the band (zeros elsewhere) on every rank
    void from_host(const T* A, int64_t lda);
    void to_host(T* A, int64_t lda) const;
    // Philox entries of the band (Gen kinds as Matrix::generate)
    void generate(Gen kind, uint64_t seed);
    // LAPACK band layout (gbtrf's AB): A(i, j) = AB(ldab_off + i - j, j),
    // ldab_off = ku (or any larger offset), every rank the same host array
    void from_host_band(const T* AB, int64_t ldab, int64_t ldab_off);
    std::shared_ptr<BandStorage> storage() const { return s_; }

protected:
    std::shared_ptr<BandStorage> s_;
    BandMatrix(int64_t m, int64_t n, int64_t kl, int64_t ku, int64_t nb, int64_t ku_alloc);
};
// Hermitian band: the uplo triangle of bandwidth kd (stored as the lower
// band; an Upper matrix is read / written as its conjugate transpose)
template <typename T>
class HermitianBandMatrix : public BandMatrix<T> {
public:
    HermitianBandMatrix() = default;
    HermitianBandMatrix(Uplo uplo, int64_t n, int64_t kd, int64_t nb);
    Uplo uplo() const { return uplo_; }
    int64_t kd() const { return this->lower_bandwidth(); }
    void from_host(const T* A, int64_t lda);
    void to_host(T* A, int64_t lda) const;

private:
    Uplo uplo_ = Uplo::Lower;
};
template <typename T>
class TriangularBandMatrix : public BandMatrix<T> {
public:
    TriangularBandMatrix() = default;
    TriangularBandMatrix(Uplo uplo, Diag diag, int64_t n, int64_t kd, int64_t nb);
    Uplo uplo() const { return uplo_; }
    Diag diag() const { return diag_; }

private:
    Uplo uplo_ = Uplo::Lower;
    Diag diag_ = Diag::NonUnit;
};
// band LU with partial pivoting: ipiv global 0-based (LAPACK gbtrf order);
// the upper bandwidth grows to kl + ku (allocated by the constructor)
template <typename T> int64_t gbtrf(BandMatrix<T>& A, std::vector<int64_t>& ipiv, const Options& opts = {});
template <typename T>
int64_t gbtrs(const BandMatrix<T>& A, const std::vector<int64_t>& ipiv, Matrix<T>& B, const Options& opts = {});
template <typename T>
int64_t gbsv(BandMatrix<T>& A, std::vector<int64_t>& ipiv, Matrix<T>& B, const Options& opts = {});
// band Cholesky A = L L^H (Upper: U^H U)
template <typename T> int64_t pbtrf(HermitianBandMatrix<T>& A, const Options& opts = {});
template <typename T> int64_t pbtrs(const HermitianBandMatrix<T>& A, Matrix<T>& B, const Options& opts = {});
template <typename T> int64_t pbsv(HermitianBandMatrix<T>& A, Matrix<T>& B, const Options& opts = {});
// B = alpha op(A)^-1 B (Side::Left; op NoTrans or ConjTrans)
template <typename T>
void tbsm(Side side, Op op, T alpha, const TriangularBandMatrix<T>& A, Matrix<T>& B, const Options& opts = {});
// C = alpha A B + beta C (band A); hbmm: A Hermitian band, Left or Right
template <typename T>
void gbmm(T alpha, const BandMatrix<T>& A, const Matrix<T>& B, T beta, Matrix<T>& C, const Options& opts = {});
template <typename T>
void hbmm(Side side, T alpha, const HermitianBandMatrix<T>& A, const Matrix<T>& B, T beta, Matrix<T>& C,
          const Options& opts = {});

struct QRData;
template <typename T>
struct QRFactors {
    std::shared_ptr<QRData> d;
};
template <typename T> int64_t geqrf(Matrix<T>& A, QRFactors<T>& F, const Options& opts = {});
template <typename T>
void unmqr(Op op, const Matrix<T>& A, const QRFactors<T>& F, Matrix<T>& C, const Options& opts = {});
template <typename T> int64_t gels(Matrix<T>& A, Matrix<T>& BX, const Options& opts = {});
// LQ: A = L Q (the QR of A^H, kept in F): A receives L in its lower
// trapezoid and the row reflectors above it; unmlq applies op(Q) from the
// left to C (n rows, A's grid and tile size)
template <typename T>
struct LQFactors {
    std::shared_ptr<Matrix<T>> At;     // A^H as factored by geqrf
    QRFactors<T> qr;
};
template <typename T> int64_t gelqf(Matrix<T>& A, LQFactors<T>& F, const Options& opts = {});
template <typename T>
void unmlq(Op op, const Matrix<T>& A, const LQFactors<T>& F, Matrix<T>& C, const Options& opts = {});

}  // namespace native
}  // namespace slate_amd

#endif
