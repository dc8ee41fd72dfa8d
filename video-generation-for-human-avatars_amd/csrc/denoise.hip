// Inference denoising-step kernels: what one iteration of the
// LTXVideoPipeline loop (pipeline_ltx_video.py:1089-1279) does around the transformer call.
//   * pixel coordinates of the latent tokens (vae_encode.py:215-226) as float32 with the time
//     axis divided by the frame rate (pipeline_ltx_video.py:1121-1122) -> RoPE indices_grid;
//   * skip-layer (STG) blends: out = a * m + c * (1 - m) per batch row, eager bf16 rounding
//     (attention.py:1071-1085 AttentionSkip / AttentionValues, :312-319 TransformerBlock);
//   * CFG / CFG* / STG / rescaling of the batched prediction (pipeline_ltx_video.py:1229-1268),
//     per-op bf16 rounding as eager torch does it, per-batch reductions in f32/f64;
//   * the rectified-flow Euler update with the scheduler's next-lower-timestep search, global or
//     per-token timesteps, and the conditioning-mask keep of denoising_step
//     (rf.py:305-374, pipeline_ltx_video.py:1346-1379).
// All HBM-bound elementwise work, 16 B per lane where rows allow.
#include <cmath>

#include "common.h"
#include "ltx_hip.h"

namespace ltx {

static inline unsigned grid_n(int64_t n, int threads = 256, int64_t cap = 8192) {
  int64_t g = (n + threads - 1) / threads;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (unsigned)g;
}

// ---- pixel coordinates -----------------------------------------------------------------------
__global__ void pixel_coords_kernel(float* __restrict__ out, int B, int F, int H, int W, int sf0, int sf1,
                                    int sf2, int causal_fix, float inv_frame_rate, int64_t* __restrict__ pix) {
  const int64_t N = (int64_t)F * H * W;
  const int64_t total = (int64_t)B * 3 * N;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t n = i % N;
    const int axis = (int)((i / N) % 3);
    const int64_t f = n / ((int64_t)H * W), h = (n / W) % H, w = n % W;
    int64_t v = axis == 0 ? f * sf0 : (axis == 1 ? h * sf1 : w * sf2);
    if (axis == 0 && causal_fix) v = v + 1 - sf0 < 0 ? 0 : v + 1 - sf0;
    if (pix) pix[i] = v;
    float fv = (float)v;  // .to(float32)
    if (axis == 0) fv = fv * inv_frame_rate;
    out[i] = fv;
  }
}

// ---- skip-layer blend --------------------------------------------------------------------------
// out[m, :] = bf16( bf16(a * mk) + bf16(c * bf16(1 - mk)) ),  mk = mask[m / rows_per_batch]
__global__ __launch_bounds__(256) void skip_blend_kernel(const bf16_t* __restrict__ a, int64_t lda,
                                                         const bf16_t* __restrict__ c, int64_t ldc,
                                                         const bf16_t* __restrict__ mask, bf16_t* __restrict__ out,
                                                         int64_t ldo, int64_t M, int D, int64_t rpb) {
  const int d8 = D / 8;
  const int64_t total = M * d8;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t m = i / d8;
    const int col = (int)(i % d8) * 8;
    const float mk = bf2f(mask[m / rpb]);
    const float om = rbf(1.0f - mk);
    const u32x4 av = *(const u32x4*)(a + m * lda + col);
    const u32x4 cv = *(const u32x4*)(c + m * ldc + col);
    u32x4 o;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float a0 = bf2f((bf16_t)av[e]), a1 = bf2f((bf16_t)(av[e] >> 16));
      const float c0 = bf2f((bf16_t)cv[e]), c1 = bf2f((bf16_t)(cv[e] >> 16));
      o[e] = pack2(rbf(a0 * mk) + rbf(c0 * om), rbf(a1 * mk) + rbf(c1 * om));
    }
    *(u32x4*)(out + m * ldo + col) = o;
  }
}

// ---- rectified-flow Euler step -------------------------------------------------------------------
// dt = t - (largest scheduled timestep < t - 1e-6, else 0); prev = sample - dt * v.
// ROUND_V (global timestep with a bf16 prediction): eager torch rounds the 0-dim dt to bf16 and
// the product to bf16 before the f32 subtraction. cond_mask: keep the input sample where
// !(t_cond - eps < 1 - cond_mask[b, n]).
template <bool SAMPLE_F32, bool V_F32, bool OUT_F32>
__global__ __launch_bounds__(256) void rf_euler_kernel(const void* __restrict__ sample, const void* __restrict__ v,
                                                       const float* __restrict__ timestep, int per_token,
                                                       const float* __restrict__ sched, int nsched,
                                                       const float* __restrict__ cond_mask, float t_cond, int round_v,
                                                       void* __restrict__ out, int64_t BN, int C) {
  const int64_t total = BN * C;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t tok = i / C;
    const float t = per_token ? timestep[tok] : timestep[0];
    float lower = 0.f;
    for (int k = 0; k < nsched; ++k) {
      const float s = sched[k];
      if (s < t - 1e-6f && s > lower) lower = s;
    }
    const float dt = t - lower;
    const float x = SAMPLE_F32 ? ((const float*)sample)[i] : bf2f(((const bf16_t*)sample)[i]);
    const float vv = V_F32 ? ((const float*)v)[i] : bf2f(((const bf16_t*)v)[i]);
    float r;
    if (round_v)
      r = x - rbf(rbf(dt) * vv);
    else
      r = x - dt * vv;
    if (cond_mask && !(t_cond - 1e-6f < 1.0f - cond_mask[tok])) r = x;
    if (OUT_F32)
      ((float*)out)[i] = r;
    else
      ((bf16_t*)out)[i] = f2bf(r);
  }
}

// ---- guidance ---------------------------------------------------------------------------------
// noise_pred [nc * B, L] bf16, chunk order (uncond, text, perturbed) restricted to the active
// conditions (pipeline_ltx_video.py:1095-1106, 1229-1233). Per-op bf16 rounding:
//   cfg*: uncond' = bf16(alpha_b * uncond), alpha_b = bf16(bf16(sum bf16(text*uncond)) /
//         bf16(bf16(sum bf16(uncond^2)) + 1e-8))
//   cfg : out = bf16(uncond' + bf16(g * bf16(text - uncond')))
//   stg : out = bf16(out + bf16(s * bf16(text - perturbed)))
//   rescale: out = bf16(out * factor_b), factor_b = bf16(bf16(r * bf16(std(text)/std(out))) + (1-r))
struct GuideParams {
  const bf16_t* pred;
  int64_t L;
  int B, i_unc, i_text, i_pert;  // chunk indices (-1: absent)
  float g, s;
  const float* alpha;   // [B] or null
  const float* factor;  // [B] or null
  bf16_t* out;
};

__device__ __forceinline__ float guide_value(const GuideParams& p, int b, int64_t j, float* text_out) {
  const float text = bf2f(p.pred[((int64_t)p.i_text * p.B + b) * p.L + j]);
  *text_out = text;
  float o = text;
  if (p.i_unc >= 0) {
    float unc = bf2f(p.pred[((int64_t)p.i_unc * p.B + b) * p.L + j]);
    if (p.alpha) unc = rbf(p.alpha[b] * unc);
    o = rbf(unc + rbf(p.g * rbf(text - unc)));
  }
  if (p.i_pert >= 0) {
    const float pert = bf2f(p.pred[((int64_t)p.i_pert * p.B + b) * p.L + j]);
    o = rbf(o + rbf(p.s * rbf(text - pert)));
  }
  return o;
}

// partial sums per (batch, block): MODE 0 -> [sum bf16(text*unc), sum bf16(unc^2)];
// MODE 1 -> [sum text, sum text^2, sum out, sum out^2] (out as guide_value computes it)
template <int MODE>
__global__ __launch_bounds__(256) void guide_partials_kernel(const GuideParams p, float* __restrict__ part) {
  const int b = blockIdx.y;
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  for (int64_t j = blockIdx.x * 256 + threadIdx.x; j < p.L; j += (int64_t)gridDim.x * 256) {
    if constexpr (MODE == 0) {
      const float text = bf2f(p.pred[((int64_t)p.i_text * p.B + b) * p.L + j]);
      const float unc = bf2f(p.pred[((int64_t)p.i_unc * p.B + b) * p.L + j]);
      acc[0] += rbf(text * unc);
      acc[1] += rbf(unc * unc);
    } else {
      float text;
      const float o = guide_value(p, b, j, &text);
      acc[0] += text;
      acc[1] += text * text;
      acc[2] += o;
      acc[3] += o * o;
    }
  }
  __shared__ float red[4][4];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const float s = wave_sum(acc[q]);
    if (lane == 0) red[w][q] = s;
  }
  __syncthreads();
  if (threadIdx.x < 4) {
    const float s = red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] + red[3][threadIdx.x];
    part[((int64_t)b * gridDim.x + blockIdx.x) * 4 + threadIdx.x] = s;
  }
}

// per batch: MODE 0 -> alpha[b]; MODE 1 -> factor[b] (rescaling r)
template <int MODE>
__global__ void guide_finalize_kernel(const float* __restrict__ part, int nblk, int64_t L, float r,
                                      float* __restrict__ res) {
  const int b = blockIdx.x;
  if (threadIdx.x != 0) return;
  double s[4] = {0, 0, 0, 0};
  for (int k = 0; k < nblk; ++k)
    for (int q = 0; q < 4; ++q) s[q] += part[((int64_t)b * nblk + k) * 4 + q];
  if constexpr (MODE == 0) {
    const float dot = rbf((float)s[0]);
    const float sq = rbf(rbf((float)s[1]) + 1e-8f);
    res[b] = rbf(dot / sq);
  } else {
    const double n = (double)L;
    const float sd_t = rbf((float)sqrt(fmax((s[1] - s[0] * s[0] / n) / (n - 1.0), 0.0)));
    const float sd_o = rbf((float)sqrt(fmax((s[3] - s[2] * s[2] / n) / (n - 1.0), 0.0)));
    const float f = rbf(sd_t / sd_o);
    res[b] = rbf(rbf(r * f) + (1.0f - r));
  }
}

__global__ __launch_bounds__(256) void guide_combine_kernel(const GuideParams p) {
  const int64_t total = (int64_t)p.B * p.L;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int b = (int)(i / p.L);
    const int64_t j = i % p.L;
    float text;
    float o = guide_value(p, b, j, &text);
    if (p.factor) o = o * p.factor[b];
    p.out[i] = f2bf(o);
  }
}

}  // namespace ltx

using namespace ltx;

extern "C" {

int ltx_pixel_coords_f32(float* out, int64_t* pixel_out, int64_t B, int64_t F, int64_t H, int64_t W, int64_t sf_t,
                         int64_t sf_h, int64_t sf_w, int causal_fix, float frame_rate, void* stream) {
  LTX_CHECK_ARG(out && B > 0 && F > 0 && H > 0 && W > 0 && frame_rate > 0.f, "pixel_coords: bad args");
  const int64_t total = B * 3 * F * H * W;
  hipLaunchKernelGGL(pixel_coords_kernel, dim3(grid_n(total)), dim3(256), 0, (hipStream_t)stream, out, (int)B,
                     (int)F, (int)H, (int)W, (int)sf_t, (int)sf_h, (int)sf_w, causal_fix, 1.0f / frame_rate,
                     pixel_out);
  LTX_LAUNCH_CHECK();
  return LTX_OK;
}

int ltx_skip_blend_bf16(const void* a, int64_t lda, const void* c, int64_t ldc, const void* mask, void* out,
                        int64_t ldo, int64_t M, int64_t D, int64_t rows_per_batch, void* stream) {
  LTX_CHECK_ARG(a && c && mask && out && M > 0 && D > 0 && rows_per_batch > 0, "skip_blend: bad args");
  LTX_CHECK_ARG(D % 8 == 0 && (lda | ldc | ldo) % 8 == 0 && (((uintptr_t)a | (uintptr_t)c | (uintptr_t)out) % 16) == 0,
                "skip_blend: rows must be 16-B aligned, D % 8 == 0");
  hipLaunchKernelGGL(skip_blend_kernel, dim3(grid_n(M * D / 8)), dim3(256), 0, (hipStream_t)stream,
                     (const bf16_t*)a, lda, (const bf16_t*)c, ldc, (const bf16_t*)mask, (bf16_t*)out, ldo, M, (int)D,
                     rows_per_batch);
  LTX_LAUNCH_CHECK();
  return LTX_OK;
}

int ltx_rf_euler_step(const void* sample, int sample_f32, const void* v, int v_f32, const float* timestep,
                      int per_token, const float* sched, int64_t nsched, const float* cond_mask, float t_cond,
                      int round_v, void* out, int out_f32, int64_t BN, int64_t C, void* stream) {
  LTX_CHECK_ARG(sample && v && timestep && sched && out && BN > 0 && C > 0 && nsched > 0, "rf_euler_step: bad args");
  const unsigned g = grid_n(BN * C);
  hipStream_t s = (hipStream_t)stream;
#define LTX_EULER(SF, VF, OF)                                                                                 \
  hipLaunchKernelGGL((rf_euler_kernel<SF, VF, OF>), dim3(g), dim3(256), 0, s, sample, v, timestep, per_token, \
                     sched, (int)nsched, cond_mask, t_cond, round_v, out, BN, (int)C)
  const int key = (sample_f32 ? 4 : 0) | (v_f32 ? 2 : 0) | (out_f32 ? 1 : 0);
  switch (key) {
    case 0: LTX_EULER(false, false, false); break;
    case 1: LTX_EULER(false, false, true); break;
    case 2: LTX_EULER(false, true, false); break;
    case 3: LTX_EULER(false, true, true); break;
    case 4: LTX_EULER(true, false, false); break;
    case 5: LTX_EULER(true, false, true); break;
    case 6: LTX_EULER(true, true, false); break;
    default: LTX_EULER(true, true, true); break;
  }
#undef LTX_EULER
  LTX_LAUNCH_CHECK();
  return LTX_OK;
}

int ltx_guidance_bf16(const void* pred, int64_t B, int64_t L, int do_cfg, int do_stg, float guidance_scale,
                      float stg_scale, float rescaling_scale, int cfg_star, float* workspace, int64_t ws_floats,
                      void* out, void* stream) {
  LTX_CHECK_ARG(pred && out && B > 0 && L > 0, "guidance: bad args");
  const int nblk = 64;
  LTX_CHECK_ARG(workspace && ws_floats >= B * (nblk * 4 + 2), "guidance: workspace needs B * 258 floats");
  hipStream_t s = (hipStream_t)stream;
  GuideParams p = {};
  p.pred = (const bf16_t*)pred;
  p.L = L;
  p.B = (int)B;
  int nc = 0;
  p.i_unc = do_cfg ? nc++ : -1;
  p.i_text = nc++;
  p.i_pert = do_stg ? nc++ : -1;
  p.g = guidance_scale;
  p.s = stg_scale;
  p.out = (bf16_t*)out;
  float* part = workspace;
  float* alpha = workspace + B * nblk * 4;
  float* factor = alpha + B;
  if (do_cfg && cfg_star) {
    hipLaunchKernelGGL(guide_partials_kernel<0>, dim3(nblk, (unsigned)B), dim3(256), 0, s, p, part);
    hipLaunchKernelGGL(guide_finalize_kernel<0>, dim3((unsigned)B), dim3(64), 0, s, part, nblk, L, 1.0f, alpha);
    p.alpha = alpha;
  }
  if (do_stg && rescaling_scale != 1.0f && stg_scale > 0.f) {
    hipLaunchKernelGGL(guide_partials_kernel<1>, dim3(nblk, (unsigned)B), dim3(256), 0, s, p, part);
    hipLaunchKernelGGL(guide_finalize_kernel<1>, dim3((unsigned)B), dim3(64), 0, s, part, nblk, L, rescaling_scale,
                       factor);
    p.factor = factor;
  }
  hipLaunchKernelGGL(guide_combine_kernel, dim3(grid_n(B * L)), dim3(256), 0, s, p);
  LTX_LAUNCH_CHECK();
  return LTX_OK;
}

}  // extern "C"
