// Ring GEMM kernels of the epilogues <0, 0>, <1, 0>, <2, 0> (gemm_ring.h; split from gemm.hip so the
// ring instantiations compile in parallel)
#define LTX_RING_DEFINE
#include "gemm_ring.h"

namespace ltx {
template bool launch_ring<0, 0>(const GemmParams& p, int bmt, hipStream_t s);
template bool launch_ring<1, 0>(const GemmParams& p, int bmt, hipStream_t s);
template bool launch_ring<2, 0>(const GemmParams& p, int bmt, hipStream_t s);
}  // namespace ltx
