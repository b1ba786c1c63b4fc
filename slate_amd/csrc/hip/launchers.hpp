// Host-side launcher declarations shared between kernel translation units
// and the Python bindings.
#pragma once
#include "common.hpp"

namespace slate_hip {

// Generic GEMM call descriptor (type-erased; dtype chosen by the caller).
struct GemmCall {
    char transA = 'N', transB = 'N';   // 'N', 'T', 'C'
    i64 m = 0, n = 0, k = 0;
    double alpha_re = 1, alpha_im = 0, beta_re = 0, beta_im = 0;
    const void* A = nullptr; i64 lda = 1; i64 strideA = 0;
    const void* B = nullptr; i64 ldb = 1; i64 strideB = 0;
    void* C = nullptr; i64 ldc = 1; i64 strideC = 0;
    const void* const* Aptrs = nullptr;
    const void* const* Bptrs = nullptr;
    void* const* Cptrs = nullptr;
    i64 batch = 1;
    bool vec_ok = true;
    bool allow_split = true;           // split-K for small-output / long-k calls
    TriMask mask;
    // device predicate: when non-null, every launched workgroup reads *gate
    // and exits at once if it is 0 (a device-decided branch -- e.g. the
    // CholeskyQR fallback -- without a host read-back)
    const int* gate = nullptr;
};

template <typename T> void gemm_real(const GemmCall& c, hipStream_t s);
template <typename T> void gemm_complex(const GemmCall& c, hipStream_t s);

}  // namespace slate_hip
