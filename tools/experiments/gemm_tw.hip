// Dispatch of the four-wave GEMM (gemm_tw.h) over the epilogues it is instantiated for.
#include "gemm_tw.h"

namespace ltx {

int launch_tw_store(int bmt, const GemmParams& p, hipStream_t s);
int launch_tw_gelu(int bmt, const GemmParams& p, hipStream_t s);
int launch_tw_gres(int bmt, const GemmParams& p, hipStream_t s);
int launch_tw_gelubwd(int bmt, const GemmParams& p, hipStream_t s);
int launch_tw_accum(int bmt, const GemmParams& p, hipStream_t s);

bool tw_supports(int epi) {
  return epi == LTX_EPI_STORE || epi == LTX_EPI_GELU || epi == LTX_EPI_GATED_RESIDUAL || epi == LTX_EPI_GELU_BWD ||
         epi == LTX_EPI_ACCUM;
}

int launch_tw(int epi, int bmt, const GemmParams& p, hipStream_t s) {
  switch (epi) {
    case LTX_EPI_STORE: return launch_tw_store(bmt, p, s);
    case LTX_EPI_GELU: return launch_tw_gelu(bmt, p, s);
    case LTX_EPI_GATED_RESIDUAL: return launch_tw_gres(bmt, p, s);
    case LTX_EPI_GELU_BWD: return launch_tw_gelubwd(bmt, p, s);
    case LTX_EPI_ACCUM: return launch_tw_accum(bmt, p, s);
    default: return fail(LTX_ERR_BAD_ARG, "gemm_tw: epilogue not instantiated");
  }
}

}  // namespace ltx
