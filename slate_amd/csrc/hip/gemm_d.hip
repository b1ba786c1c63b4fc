#include "gemm_launch.hpp"
namespace slate_hip {
template void gemm_real<double>(const GemmCall&, hipStream_t);
}
