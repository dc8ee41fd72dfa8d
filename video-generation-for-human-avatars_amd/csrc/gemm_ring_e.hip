// Ring GEMM kernels of the epilogues <7, 8>, <7, 16>, <7, 32> (gemm_ring.h; split from gemm.hip so the
// ring instantiations compile in parallel)
#define LTX_RING_DEFINE
#include "gemm_ring.h"

namespace ltx {
template bool launch_ring<7, 8>(const GemmParams& p, int bmt, hipStream_t s);
template bool launch_ring<7, 16>(const GemmParams& p, int bmt, hipStream_t s);
template bool launch_ring<7, 32>(const GemmParams& p, int bmt, hipStream_t s);
}  // namespace ltx
