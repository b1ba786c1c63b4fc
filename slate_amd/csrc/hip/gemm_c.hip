#include "gemm_launch.hpp"
namespace slate_hip {
template void gemm_complex<ccplx>(const GemmCall&, hipStream_t);
}
