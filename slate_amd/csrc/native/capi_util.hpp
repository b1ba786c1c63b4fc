// Shared helpers of the native C / LAPACK / ScaLAPACK ABI units
// (capi_native.hip, capi_lapack.hip, capi_handles.hip).  Not installed.
#pragma once
#include <algorithm>
#include <complex>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "native_rt.hpp"

namespace slate_amd {
namespace native {
namespace capi {

namespace sn = slate_amd::native;

constexpr int ERR_INTERNAL = -1000000;
// message of the last runtime error of this thread (slate_amd_last_error)
inline thread_local std::string g_err;

// process grid of the LAPACK-style host-array routines: 1 x WORLD_SIZE, or
// SLATE_AMD_NATIVE_GRID=PxQ
inline void grid_of(int& p, int& q) {
    const int ws = sn::size();
    p = 1;
    q = ws;
    if (const char* g = std::getenv("SLATE_AMD_NATIVE_GRID")) {
        int a = 0, b = 0;
        if (std::sscanf(g, "%dx%d", &a, &b) == 2 && a * b == ws) { p = a; q = b; }
    }
}

inline int64_t nb_of(int64_t n) {
    if (const char* e = std::getenv("SLATE_AMD_NATIVE_NB")) return std::max<int64_t>(16, std::atoll(e));
    return n >= 8192 ? 512 : (n >= 1024 ? 256 : 64);
}

template <typename F>
int64_t guarded(F&& f) {
    try {
        return (int64_t)f();
    } catch (const std::exception& e) {
        g_err = e.what();
        return ERR_INTERNAL;
    }
}

inline char up(char c) { return (c >= 'a' && c <= 'z') ? (char)(c - 32) : c; }

template <typename T> T cj(T x) { return x; }
template <typename R> std::complex<R> cj(std::complex<R> x) { return std::conj(x); }

// op(a) (rows x cols of the RESULT) into a new column-major array
template <typename T>
std::vector<T> host_op(char op, i64 rows, i64 cols, const T* a, i64 lda) {
    std::vector<T> r((size_t)rows * cols);
    for (i64 j = 0; j < cols; ++j)
        for (i64 i = 0; i < rows; ++i)
            r[i + j * rows] = op == 'N' ? a[i + j * lda] : op == 'T' ? a[j + i * lda] : cj(a[j + i * lda]);
    return r;
}

inline sn::Op op_of(char c) {
    c = up(c);
    return c == 'N' ? sn::Op::NoTrans : c == 'T' ? sn::Op::Trans : sn::Op::ConjTrans;
}
inline sn::Uplo uplo_of(char c) { return up(c) == 'U' ? sn::Uplo::Upper : sn::Uplo::Lower; }
inline sn::Diag diag_of(char c) { return up(c) == 'U' ? sn::Diag::Unit : sn::Diag::NonUnit; }
inline sn::Side side_of(char c) { return up(c) == 'R' ? sn::Side::Right : sn::Side::Left; }

}  // namespace capi
}  // namespace native
}  // namespace slate_amd
