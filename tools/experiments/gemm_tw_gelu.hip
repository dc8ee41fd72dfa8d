// gemm_tw_kernel instantiations for LTX_EPI_GELU (one file per epilogue: parallel builds)
#include "gemm_tw.h"

namespace ltx {

int launch_tw_gelu(int bmt, const GemmParams& p, hipStream_t s) {
  return bmt == 224 ? launch_tw_t<LTX_EPI_GELU, 0, 224>(p, s) : launch_tw_t<LTX_EPI_GELU, 0, 256>(p, s);
}

}  // namespace ltx
