// Flat-buffer kernels of the ZeRO-2 optimizer (ltx_amd/zero.py; BASELINE config Z:
// configs/ds_config_zero2.json -- stage 2, bf16, reduce_scatter, gradient_clipping 1.0):
// bf16 <-> f32 casts of the contiguous grad / param buffers, the shard's sum of squares for the
// global-norm clip (f64 per-block partials in the stream's workspace, added in block order), and the clip coefficient applied
// from device memory so no host sync sits between the collectives and the AdamW kernel.
#include <cmath>

#include "common.h"
#include "ltx_hip.h"

namespace ltx {

static inline unsigned grid_cap(int64_t n) {
  int64_t g = (n + 255) / 256;
  if (g > 8192) g = 8192;
  return (unsigned)(g < 1 ? 1 : g);
}

__global__ __launch_bounds__(256) void cast_bf16_f32_kernel(const bf16_t* __restrict__ src, float* __restrict__ dst,
                                                            int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    dst[i] = bf2f(src[i]);
}

__global__ __launch_bounds__(256) void cast_f32_bf16_kernel(const float* __restrict__ src, bf16_t* __restrict__ dst,
                                                            int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    dst[i] = f2bf(src[i]);
}

// part != null: block b stores its sum to part[b] and sumsq_finish_kernel adds the partials in block
// order (deterministic); part == null (no workspace): one f64 atomic per block
__global__ __launch_bounds__(256) void sumsq_kernel(const float* __restrict__ x, int64_t n, double* __restrict__ out,
                                                    double* __restrict__ part) {
  double s = 0.0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const double v = x[i];
    s += v * v;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  __shared__ double red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    const double b = red[0] + red[1] + red[2] + red[3];
    if (part != nullptr) part[blockIdx.x] = b;
    else atomicAdd(out, b);
  }
}

__global__ __launch_bounds__(256) void sumsq_finish_kernel(const double* __restrict__ part, int nparts,
                                                           double* __restrict__ out) {
  // 256 threads sum strided partials in a fixed order, then a fixed-shape tree
  double s = 0.0;
  for (int i = threadIdx.x; i < nparts; i += 256) s += part[i];
  __shared__ double red[256];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) *out += red[0];
}

// coef = inv_world * min(1, max_norm / (sqrt(sumsq) * inv_world + 1e-6)) (max_norm <= 0: no clip)
__global__ void clip_coef_kernel(const double* __restrict__ sumsq, float max_norm, float inv_world,
                                 float* __restrict__ coef) {
  float c = 1.0f;
  if (max_norm > 0.f) {
    const float norm = (float)sqrt(*sumsq) * inv_world;
    const float cc = max_norm / (norm + 1e-6f);
    if (cc < 1.0f) c = cc;
  }
  *coef = c * inv_world;
}

__global__ __launch_bounds__(256) void scale_dev_kernel(float* __restrict__ x, int64_t n,
                                                        const float* __restrict__ coef) {
  const float c = *coef;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    x[i] *= c;
}

}  // namespace ltx

using namespace ltx;

extern "C" {

int ltx_cast_bf16_f32(const void* src, float* dst, int64_t n, void* stream) {
  LTX_CHECK_ARG(src && dst && n >= 0, "cast_bf16_f32: bad args");
  if (n == 0) return LTX_OK;
  hipLaunchKernelGGL(cast_bf16_f32_kernel, dim3(grid_cap(n)), dim3(256), 0, (hipStream_t)stream, (const bf16_t*)src,
                     dst, n);
  LTX_LAUNCH_CHECK();
  return LTX_OK;
}

int ltx_cast_f32_bf16(const float* src, void* dst, int64_t n, void* stream) {
  LTX_CHECK_ARG(src && dst && n >= 0, "cast_f32_bf16: bad args");
  if (n == 0) return LTX_OK;
  hipLaunchKernelGGL(cast_f32_bf16_kernel, dim3(grid_cap(n)), dim3(256), 0, (hipStream_t)stream, src, (bf16_t*)dst,
                     n);
  LTX_LAUNCH_CHECK();
  return LTX_OK;
}

int ltx_sumsq_f32(const float* x, int64_t n, double* out, int accumulate, void* stream) {
  LTX_CHECK_ARG(x && out && n >= 0, "sumsq: bad args");
  hipStream_t s = (hipStream_t)stream;
  if (!accumulate) {
    hipError_t e = hipMemsetAsync(out, 0, sizeof(double), s);
    if (e != hipSuccess) return fail((int)e, hipGetErrorString(e));
  }
  if (n == 0) return LTX_OK;
  const unsigned g = grid_cap(n);
  size_t ws = 0;
  double* part = (double*)stream_workspace(s, &ws);
  if (part == nullptr || ws < g * sizeof(double)) part = nullptr;
  hipLaunchKernelGGL(sumsq_kernel, dim3(g), dim3(256), 0, s, x, n, out, part);
  LTX_LAUNCH_CHECK();
  if (part != nullptr) {
    hipLaunchKernelGGL(sumsq_finish_kernel, dim3(1), dim3(256), 0, s, (const double*)part, (int)g, out);
    LTX_LAUNCH_CHECK();
  }
  return LTX_OK;
}

int ltx_clip_scale_f32(float* x, int64_t n, const double* sumsq, float max_norm, float inv_world, float* coef,
                       void* stream) {
  LTX_CHECK_ARG(x && sumsq && coef && n >= 0 && inv_world > 0.f, "clip_scale: bad args");
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(clip_coef_kernel, dim3(1), dim3(1), 0, s, sumsq, max_norm, inv_world, coef);
  if (n > 0) hipLaunchKernelGGL(scale_dev_kernel, dim3(grid_cap(n)), dim3(256), 0, s, x, n, (const float*)coef);
  LTX_LAUNCH_CHECK();
  return LTX_OK;
}

}  // extern "C"
