// Ring GEMM kernels of the epilogues <5, 0>, <6, 0>, <8, 0> (gemm_ring.h; split from gemm.hip so the
// ring instantiations compile in parallel)
#define LTX_RING_DEFINE
#include "gemm_ring.h"

namespace ltx {
template bool launch_ring<5, 0>(const GemmParams& p, int bmt, hipStream_t s);
template bool launch_ring<6, 0>(const GemmParams& p, int bmt, hipStream_t s);
template bool launch_ring<8, 0>(const GemmParams& p, int bmt, hipStream_t s);
}  // namespace ltx
