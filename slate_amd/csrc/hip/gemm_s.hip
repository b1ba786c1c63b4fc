#include "gemm_launch.hpp"
namespace slate_hip {
template void gemm_real<float>(const GemmCall&, hipStream_t);
}
