// Parameter-gradient reductions for train_mode='full' (training.py:75-91; BASELINE config Z):
// the weights that train besides LoRA are reached by column sums over token rows --
//   * biases:                    sum_rows dY                      (G = 1)
//   * AdaLN shift rows:          sum_{rows of batch b} dY         (G = B)
//   * AdaLN scale rows:          sum_rows bf16(dY * n),  n = bf16(x * rstd)          (RMSNorm)
//                                or n = bf16((x - mean) * rstd)                       (LayerNorm)
//   * AdaLN gates:               sum_rows bf16(dH * y)            (y = the pre-gate output)
//   * scale_shift_table:         sum over the batch of the per-batch rows
// with the eager bf16 semantics of autograd's broadcast reductions: each product rounded to
// bf16, the sum accumulated in f32 and rounded once per reduced tensor. Two deterministic levels:
// group_colsum_kernel writes per-(group, split) f32 partials, colsum_finish_kernel adds the splits
// (and optionally the groups) and writes / accumulates bf16 (the .grad += of the micro-steps).
// HBM-bound: every operand row is read once, 16 B per lane.
#include "common.h"
#include "ltx_hip.h"

namespace ltx {

__device__ __forceinline__ void ld8(const bf16_t* p, float* v) {
  const u32x4 w = *(const u32x4*)p;
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = bf2f((bf16_t)(w[j >> 1] >> ((j & 1) * 16)));
}

// MODE 0: a ; 1: bf16(a*b) ; 2: bf16(a * bf16(b * r[m])) ; 3: bf16(a * bf16((b - mu[m]) * r[m]))
template <int MODE>
__global__ __launch_bounds__(256) void group_colsum_kernel(const bf16_t* __restrict__ a, int64_t lda,
                                                           const bf16_t* __restrict__ b, int64_t ldb,
                                                           const float* __restrict__ r, const float* __restrict__ mu,
                                                           int64_t rpg, int D, int S, float* __restrict__ part) {
  const int split = blockIdx.x, g = blockIdx.y;
  const int64_t r0 = (int64_t)g * rpg + (int64_t)split * rpg / S;
  const int64_t r1 = (int64_t)g * rpg + (int64_t)(split + 1) * rpg / S;
  for (int c = threadIdx.x * 8; c < D; c += 256 * 8) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int64_t m = r0; m < r1; ++m) {
      float av[8];
      ld8(a + m * lda + c, av);
      if constexpr (MODE == 0) {
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += av[j];
      } else {
        float bv[8];
        ld8(b + m * ldb + c, bv);
        if constexpr (MODE == 1) {
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[j] += rbf(av[j] * bv[j]);
        } else if constexpr (MODE == 2) {
          const float rr = r[m];
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[j] += rbf(av[j] * rbf(bv[j] * rr));
        } else {
          const float rr = r[m], mm = mu[m];
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[j] += rbf(av[j] * rbf((bv[j] - mm) * rr));
        }
      }
    }
    float* o = part + ((int64_t)g * S + split) * D + c;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = acc[j];
  }
}

// out_g[d] = bf16(sum_s part[g,s,d]); sum_groups: out[d] = bf16(sum_g out_g[d]) (f32 accumulation);
// accumulate: out = bf16(out + that). A workgroup owns 16 columns: its 16 rows of 16 lanes
// (ls = tid / 16) each sum every 16th split, the 16 partial sums meet in LDS (fixed order).
constexpr int CF_COLS = 16, CF_LANES = 16;
__global__ __launch_bounds__(256) void colsum_finish_kernel(const float* __restrict__ part, int G, int S, int D,
                                                            int sum_groups, int accumulate, bf16_t* __restrict__ out,
                                                            int64_t ldo) {
  __shared__ float red[CF_LANES][CF_COLS];
  const int cl = threadIdx.x % CF_COLS, ls = threadIdx.x / CF_COLS;
  const int d = blockIdx.x * CF_COLS + cl;
  const int g0 = sum_groups ? 0 : (int)blockIdx.y;
  const int g1 = sum_groups ? G : g0 + 1;
  float tot = 0.f;
  for (int g = g0; g < g1; ++g) {
    float s = 0.f;
    if (d < D)
      for (int k = ls; k < S; k += CF_LANES) s += part[((int64_t)g * S + k) * D + d];
    red[ls][cl] = s;
    __syncthreads();
    if (ls == 0) {
      float t = 0.f;
#pragma unroll
      for (int j = 0; j < CF_LANES; ++j) t += red[j][cl];
      tot += rbf(t);
    }
    __syncthreads();
  }
  if (ls != 0 || d >= D) return;
  bf16_t* o = out + (sum_groups ? 0 : (int64_t)g0 * ldo) + d;
  const float v = rbf(tot);
  *o = f2bf(accumulate ? bf2f(*o) + v : v);
}

// torch silu_backward (bf16): dx = bf16(dy * s * (1 + x * (1 - s))), s = sigmoid(x), f32 math;
// with dres: dx = bf16(dres + that) (autograd summing a second use of the same tensor)
__global__ __launch_bounds__(256) void silu_bwd_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ dy,
                                                       const bf16_t* __restrict__ dres, bf16_t* __restrict__ dx,
                                                       int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const float xv = bf2f(x[i]), g = bf2f(dy[i]);
    const float s = 1.0f / (1.0f + expf(-xv));
    const float d = rbf(g * (s * (1.0f + xv * (1.0f - s))));
    dx[i] = f2bf(dres ? bf2f(dres[i]) + d : d);
  }
}

}  // namespace ltx

using namespace ltx;

extern "C" {

int ltx_group_colsum(const void* a, int64_t lda, const void* b, int64_t ldb, const float* r, const float* mean,
                     int mode, int64_t M, int64_t D, int64_t rows_per_group, int64_t splits, float* partials,
                     void* stream) {
  LTX_CHECK_ARG(a && partials && M > 0 && D > 0 && rows_per_group > 0 && splits > 0, "group_colsum: bad args");
  LTX_CHECK_ARG(M % rows_per_group == 0 && splits <= rows_per_group, "group_colsum: rows must split evenly");
  LTX_CHECK_ARG(D % 8 == 0 && lda % 8 == 0 && (!b || ldb % 8 == 0), "group_colsum: D and strides must be %8");
  LTX_CHECK_ARG(mode >= 0 && mode <= 3 && (mode == 0 || b) && (mode < 2 || r) && (mode < 3 || mean),
                "group_colsum: mode needs b / rstd / mean");
  const dim3 grid((unsigned)splits, (unsigned)(M / rows_per_group));
  hipStream_t s = (hipStream_t)stream;
  const bf16_t* A = (const bf16_t*)a;
  const bf16_t* Bp = (const bf16_t*)b;
  switch (mode) {
    case 0: hipLaunchKernelGGL(group_colsum_kernel<0>, grid, dim3(256), 0, s, A, lda, Bp, ldb, r, mean, rows_per_group, (int)D, (int)splits, partials); break;
    case 1: hipLaunchKernelGGL(group_colsum_kernel<1>, grid, dim3(256), 0, s, A, lda, Bp, ldb, r, mean, rows_per_group, (int)D, (int)splits, partials); break;
    case 2: hipLaunchKernelGGL(group_colsum_kernel<2>, grid, dim3(256), 0, s, A, lda, Bp, ldb, r, mean, rows_per_group, (int)D, (int)splits, partials); break;
    default: hipLaunchKernelGGL(group_colsum_kernel<3>, grid, dim3(256), 0, s, A, lda, Bp, ldb, r, mean, rows_per_group, (int)D, (int)splits, partials); break;
  }
  LTX_LAUNCH_CHECK();
  return LTX_OK;
}

int ltx_colsum_finish(const float* partials, int64_t G, int64_t S, int64_t D, int sum_groups, int accumulate,
                      void* out, int64_t ldo, void* stream) {
  LTX_CHECK_ARG(partials && out && G > 0 && S > 0 && D > 0, "colsum_finish: bad args");
  const dim3 grid((unsigned)((D + CF_COLS - 1) / CF_COLS), (unsigned)(sum_groups ? 1 : G));
  hipLaunchKernelGGL(colsum_finish_kernel, grid, dim3(256), 0, (hipStream_t)stream,
                     partials, (int)G, (int)S, (int)D, sum_groups, accumulate, (bf16_t*)out, ldo);
  LTX_LAUNCH_CHECK();
  return LTX_OK;
}

int ltx_silu_bwd_bf16(const void* x, const void* dy, const void* dres, void* dx, int64_t n, void* stream) {
  LTX_CHECK_ARG(x && dy && dx && n > 0, "silu_bwd: bad args");
  int64_t g = (n + 255) / 256;
  if (g > 4096) g = 4096;
  hipLaunchKernelGGL(silu_bwd_kernel, dim3((unsigned)g), dim3(256), 0, (hipStream_t)stream, (const bf16_t*)x,
                     (const bf16_t*)dy, (const bf16_t*)dres, (bf16_t*)dx, n);
  LTX_LAUNCH_CHECK();
  return LTX_OK;
}

}  // extern "C"
