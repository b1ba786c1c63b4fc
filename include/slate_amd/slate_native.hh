// slate_amd native C++ API: distributed tiled matrices and the core dense
// linear algebra routines WITHOUT the Python runtime.
//
// libslate_amd_native.so is the gfx950 HIP kernels of the package plus a
// C++ host runtime (process bootstrap, RCCL communicators, HIP stream/event
// lookahead pipelines) -- it links against libamdhip64 and librccl only.
// It mirrors the reference's public C++ interface for the routines it
// covers (include/slate/slate.hh: potrf/potrs/posv, getrf/getrs/gesv, gemm,
// norm; include/slate/Matrix.hh / HermitianMatrix.hh for the matrix types).
//
// One process per GPU.  The world is taken from the torchrun-style
// environment (RANK, WORLD_SIZE, LOCAL_RANK, MASTER_ADDR; the RCCL unique id
// travels over a TCP socket on SLATE_AMD_NATIVE_PORT, default MASTER_PORT +
// 1 -- torchrun's own store holds MASTER_PORT).  A single process needs no
// environment at all and never initialises RCCL.
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

#include <cstdint>
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
enum class Op : char { NoTrans = 'N', Trans = 'T' };
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

struct Options {
    int lookahead = 1;        // SLATE Option::Lookahead
    double pivot_threshold = 1.0;
};

struct Storage;               // opaque: device buffer, grid, communicators

template <typename T>
class Matrix {
public:
    Matrix() = default;
    Matrix(int64_t m, int64_t n, int64_t nb, int p = 1, int q = 1);
    int64_t m() const;
    int64_t n() const;
    int64_t nb() const;
    int p() const;
    int q() const;
    int64_t mloc() const;     // local rows / columns of this rank
    int64_t nloc() const;
    int64_t lld() const;      // leading dimension of the local buffer
    T* data();                // device pointer to the local buffer
    const T* data() const;
    void generate(Gen kind, uint64_t seed);
    // Global column-major host array, identical on every rank (LAPACK
    // layout): copy this rank's block-cyclic part to the device / gather the
    // whole matrix back to every rank.
    void from_host(const T* A, int64_t lda);
    void to_host(T* A, int64_t lda) const;
    std::shared_ptr<Storage> storage() const { return s_; }

protected:
    std::shared_ptr<Storage> s_;
};

template <typename T>
class HermitianMatrix : public Matrix<T> {
public:
    HermitianMatrix() = default;
    HermitianMatrix(Uplo uplo, int64_t n, int64_t nb, int p = 1, int q = 1)
        : Matrix<T>(n, n, nb, p, q), uplo_(uplo) {}
    Uplo uplo() const { return uplo_; }

private:
    Uplo uplo_ = Uplo::Lower;
};

// ---- drivers (fp64).  Return LAPACK info (0 = success).
int64_t potrf(HermitianMatrix<double>& A, const Options& opts = {});
int64_t potrs(const HermitianMatrix<double>& A, Matrix<double>& B, const Options& opts = {});
int64_t posv(HermitianMatrix<double>& A, Matrix<double>& B, const Options& opts = {});
// LU with partial pivoting on 1 x q grids; ipiv (global, 0-based,
// LAPACK-style sequential interchanges) is returned on every rank
int64_t getrf(Matrix<double>& A, std::vector<int64_t>& ipiv, const Options& opts = {});
int64_t getrs(const Matrix<double>& A, const std::vector<int64_t>& ipiv, Matrix<double>& B,
              const Options& opts = {});
int64_t gesv(Matrix<double>& A, std::vector<int64_t>& ipiv, Matrix<double>& B, const Options& opts = {});
// C = alpha op(A) op(B) + beta C, SUMMA on the grid (op = NoTrans)
void gemm(double alpha, const Matrix<double>& A, const Matrix<double>& B, double beta, Matrix<double>& C,
          const Options& opts = {});
double norm(Norm kind, const Matrix<double>& A);

}  // namespace native
}  // namespace slate_amd

#endif
