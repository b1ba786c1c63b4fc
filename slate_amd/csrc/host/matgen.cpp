// Host matrix generator (slate_matgen equivalent, matgen/*.cc): fills the
// local part of a 2D block-cyclic matrix from global-index Philox streams.
#include <pybind11/pybind11.h>
#include <complex>
#include <cstdint>
#include "philox.hpp"

namespace py = pybind11;

namespace slate_host {

static inline int64_t l2g(int64_t l, int64_t nb, int p, int pr) {
    int64_t lt = l / nb;
    return (lt * p + pr) * nb + (l - lt * nb);
}

template <typename T>
static void gen(int kind, uint64_t seed, int64_t mloc, int64_t nloc, T* A, int64_t lda,
                int64_t m, int64_t n, int64_t mb, int p, int pr, int64_t nb, int q, int pc,
                int64_t row0, int64_t col0, double cond_scale) {
    constexpr bool cplx = sizeof(T) == 2 * sizeof(typename std::conditional<
        std::is_same<T, std::complex<float>>::value, float,
        typename std::conditional<std::is_same<T, std::complex<double>>::value, double, T>::type>::type);
    #pragma omp parallel for schedule(static)
    for (int64_t lj = 0; lj < nloc; ++lj) {
        int64_t gj = l2g(lj, nb, q, pc) + col0;
        for (int64_t li = 0; li < mloc; ++li) {
            int64_t gi = l2g(li, mb, p, pr) + row0;
            double re, im;
            slate_rng::entry(kind, seed, gi, gj, m, n, cplx, re, im);
            re *= cond_scale; im *= cond_scale;
            if constexpr (cplx) A[li + lj * lda] = T(re, im);
            else A[li + lj * lda] = T(re);
        }
    }
}

void register_matgen(py::module& m) {
    m.def("matgen", [](char dt, int kind, uint64_t seed, int64_t mloc, int64_t nloc, uintptr_t A, int64_t lda,
                       int64_t gm, int64_t gn, int64_t mb, int p, int pr, int64_t nb, int q, int pc,
                       int64_t row0, int64_t col0, double scale) {
        py::gil_scoped_release nogil;
        switch (dt) {
            case 's': gen<float>(kind, seed, mloc, nloc, (float*)A, lda, gm, gn, mb, p, pr, nb, q, pc, row0, col0, scale); break;
            case 'd': gen<double>(kind, seed, mloc, nloc, (double*)A, lda, gm, gn, mb, p, pr, nb, q, pc, row0, col0, scale); break;
            case 'c': gen<std::complex<float>>(kind, seed, mloc, nloc, (std::complex<float>*)A, lda, gm, gn, mb, p, pr, nb, q, pc, row0, col0, scale); break;
            case 'z': gen<std::complex<double>>(kind, seed, mloc, nloc, (std::complex<double>*)A, lda, gm, gn, mb, p, pr, nb, q, pc, row0, col0, scale); break;
            default: throw std::invalid_argument("matgen: bad dtype");
        }
    });
}

}  // namespace slate_host
