// LoRA adapter contractions in f32 (peft 0.17.1 keeps adapters in f32 on a bf16 base:
// training.py:50-68 + autocast_adapter_dtype). Rank r <= 32 makes these skinny: the down
// projection reads x once (HBM-bound, 2 B/element for r*2 FLOP/element) and the weight grads are
// split-M reductions. The up-projection (B) and its input-gradient half are fused into the bf16
// GEMM epilogues (gemm.hip, LTX_EPI_LORA / LTX_EPI_LORA_DGRAD_ACCUM).
#include "common.h"
#include "ltx_hip.h"

namespace ltx {

// out[m,j] = alpha * sum_k x[m,k] * Wr[j*wj + k*wk]
// Block: 64 rows x all r outputs; K streamed in chunks of 64 through LDS (x as f32, W as [k][j]).
template <int R>
__global__ __launch_bounds__(256) void lora_down_kernel(const bf16_t* __restrict__ x, int64_t ldx,
                                                        const float* __restrict__ Wr, int64_t wj, int64_t wk,
                                                        float* __restrict__ out, int64_t ldo, int M, int K,
                                                        float alpha) {
  constexpr int RM = 64, KC = 64;
  constexpr int JPT = R / 4;  // outputs per thread (4 threads per row)
  __shared__ float xs[RM][KC + 1];
  __shared__ float ws[KC][R];
  const int t = threadIdx.x;
  const int m0 = blockIdx.x * RM;
  const int row = t >> 2, jq = t & 3;
  float acc[JPT];
#pragma unroll
  for (int j = 0; j < JPT; ++j) acc[j] = 0.f;
  for (int k0 = 0; k0 < K; k0 += KC) {
    {  // x chunk: 64 rows x 64 bf16 = 256 threads x 16 B
      const int r = t >> 3, c8 = (t & 7) * 8;
#pragma unroll
      for (int half = 0; half < 2; ++half) {
        const int rr = r + half * 32;
        const int gm = m0 + rr;
        float v[8];
        if (gm < M) {
          const u32x4 w = *(const u32x4*)(x + (int64_t)gm * ldx + k0 + c8);
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] = bf2f((bf16_t)(w[j >> 1] >> ((j & 1) * 16)));
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] = 0.f;
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) xs[rr][c8 + j] = v[j];
      }
    }
    for (int i = t; i < KC * R; i += 256) {  // W chunk as [k][j]
      const int kk = i / R, j = i % R;
      ws[kk][j] = Wr[(int64_t)j * wj + (int64_t)(k0 + kk) * wk];
    }
    __syncthreads();
#pragma unroll 8
    for (int kk = 0; kk < KC; ++kk) {
      const float xv = xs[row][kk];
#pragma unroll
      for (int j = 0; j < JPT; ++j) acc[j] = fmaf(xv, ws[kk][jq * JPT + j], acc[j]);
    }
    __syncthreads();
  }
  const int gm = m0 + row;
  if (gm < M) {
#pragma unroll
    for (int j = 0; j < JPT; ++j) out[(int64_t)gm * ldo + jq * JPT + j] = acc[j] * alpha;
  }
}

// dw(n,j) += alpha * sum_{m in split} y[m,n] * u[m,j]; 64 columns x r per block, f32 atomics
template <int R>
__global__ __launch_bounds__(256) void lora_wgrad_kernel(const bf16_t* __restrict__ y, int64_t ldy,
                                                         const float* __restrict__ u, int64_t ldu,
                                                         float* __restrict__ dw, int64_t on, int64_t oj, int M,
                                                         int N, int rows_per_split, float alpha) {
  constexpr int JPT = R / 4;
  const int t = threadIdx.x;
  const int n = blockIdx.x * 64 + (t & 63);
  const int jq = t >> 6;
  const int mb = blockIdx.y * rows_per_split;
  const int me = min(M, mb + rows_per_split);
  float acc[JPT];
#pragma unroll
  for (int j = 0; j < JPT; ++j) acc[j] = 0.f;
  if (n < N) {
    for (int m = mb; m < me; ++m) {
      const float yv = bf2f(y[(int64_t)m * ldy + n]);
      const float* ur = u + (int64_t)m * ldu + jq * JPT;
#pragma unroll
      for (int j = 0; j < JPT; ++j) acc[j] = fmaf(yv, ur[j], acc[j]);
    }
#pragma unroll
    for (int j = 0; j < JPT; ++j) atomicAdd(dw + (int64_t)n * on + (int64_t)(jq * JPT + j) * oj, acc[j] * alpha);
  }
}

}  // namespace ltx

using namespace ltx;

extern "C" int ltx_lora_down(const void* x, int64_t ldx, const float* Wr, int64_t wj, int64_t wk, float* out,
                             int64_t ldo, int64_t M, int64_t K, int64_t r, float alpha, void* stream) {
  LTX_CHECK_ARG(x && Wr && out && M > 0 && K > 0, "lora_down: bad args");
  LTX_CHECK_ARG(K % 64 == 0 && ldx % 8 == 0 && ((uintptr_t)x % 16) == 0, "lora_down: K %64, 16-B rows");
  const dim3 grid((unsigned)((M + 63) / 64));
  hipStream_t s = (hipStream_t)stream;
  switch (r) {
    case 8: hipLaunchKernelGGL(lora_down_kernel<8>, grid, dim3(256), 0, s, (const bf16_t*)x, ldx, Wr, wj, wk, out, ldo, (int)M, (int)K, alpha); break;
    case 16: hipLaunchKernelGGL(lora_down_kernel<16>, grid, dim3(256), 0, s, (const bf16_t*)x, ldx, Wr, wj, wk, out, ldo, (int)M, (int)K, alpha); break;
    case 32: hipLaunchKernelGGL(lora_down_kernel<32>, grid, dim3(256), 0, s, (const bf16_t*)x, ldx, Wr, wj, wk, out, ldo, (int)M, (int)K, alpha); break;
    default: return fail(LTX_ERR_BAD_ARG, "lora_down: rank must be 8, 16 or 32");
  }
  LTX_LAUNCH_CHECK();
  return LTX_OK;
}

extern "C" int ltx_lora_wgrad(const void* y, int64_t ldy, const float* u, int64_t ldu, float* dw, int64_t on,
                              int64_t oj, int64_t M, int64_t N, int64_t r, float alpha, void* stream) {
  LTX_CHECK_ARG(y && u && dw && M > 0 && N > 0, "lora_wgrad: bad args");
  LTX_CHECK_ARG((on == r && oj == 1) || (on == 1 && oj == N), "lora_wgrad: output must be a dense [N,r] or [r,N]");
  hipStream_t s = (hipStream_t)stream;
  hipError_t e = hipMemsetAsync(dw, 0, (size_t)N * r * sizeof(float), s);
  if (e != hipSuccess) return fail((int)e, hipGetErrorString(e));
  const int nb = (int)((N + 63) / 64);
  int splits = (int)((1024 + nb - 1) / nb);
  if (splits > M) splits = (int)M;
  const int rps = (int)((M + splits - 1) / splits);
  splits = (int)((M + rps - 1) / rps);
  const dim3 grid((unsigned)nb, (unsigned)splits);
  switch (r) {
    case 8: hipLaunchKernelGGL(lora_wgrad_kernel<8>, grid, dim3(256), 0, s, (const bf16_t*)y, ldy, u, ldu, dw, on, oj, (int)M, (int)N, rps, alpha); break;
    case 16: hipLaunchKernelGGL(lora_wgrad_kernel<16>, grid, dim3(256), 0, s, (const bf16_t*)y, ldy, u, ldu, dw, on, oj, (int)M, (int)N, rps, alpha); break;
    case 32: hipLaunchKernelGGL(lora_wgrad_kernel<32>, grid, dim3(256), 0, s, (const bf16_t*)y, ldy, u, ldu, dw, on, oj, (int)M, (int)N, rps, alpha); break;
    default: return fail(LTX_ERR_BAD_ARG, "lora_wgrad: rank must be 8, 16 or 32");
  }
  LTX_LAUNCH_CHECK();
  return LTX_OK;
}
