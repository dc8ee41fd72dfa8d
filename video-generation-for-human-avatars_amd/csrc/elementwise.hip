// Byte-moving / elementwise kernels of the LTX-Video training step (HBM-bound on MI355X):
// patchifier permutation, rectified-flow noising + velocity target, the conditioning lerp,
// AdaLN modulation rows, timestep sinusoid, SiLU, transpose, column sums (bias grads),
// MSE loss + its backward seed, AdamW. All bf16 traffic is vectorised to 16 B per lane where
// the layout allows; transposes go through an LDS tile so both sides stay coalesced.
#include <cmath>
#include <cstdlib>
#include <string>

#include "common.h"
#include "ltx_hip.h"

namespace ltx {

static thread_local std::string g_last_error;
void set_error(const std::string& msg) { g_last_error = msg; }
int fail(int code, const std::string& msg) {
  g_last_error = msg;
  return code;
}

// ---------------------------------------------------------------------------------------------
// [B, R, Cn] <-> [B, Cn, R] tile transpose helper used by patchify/unpatchify/transpose.
// 64x64 tile, 256 threads; LDS row padded by 2 elements (odd dword stride) against conflicts.
// ---------------------------------------------------------------------------------------------
constexpr int TT = 64;
__global__ __launch_bounds__(256) void transpose_kernel(const bf16_t* __restrict__ in, int64_t ld_in,
                                                        int64_t bstride_in, bf16_t* __restrict__ out,
                                                        int64_t ld_out, int64_t bstride_out, int R, int C) {
  __shared__ bf16_t tile[TT][TT + 2];
  const int b = blockIdx.z;
  const int r0 = blockIdx.y * TT, c0 = blockIdx.x * TT;
  const bf16_t* src = in + (int64_t)b * bstride_in;
  bf16_t* dst = out + (int64_t)b * bstride_out;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  for (int r = ty; r < TT; r += 4) {
    const int gr = r0 + r, gc = c0 + tx;
    tile[r][tx] = (gr < R && gc < C) ? src[(int64_t)gr * ld_in + gc] : (bf16_t)0;
  }
  __syncthreads();
  for (int c = ty; c < TT; c += 4) {
    const int gc = c0 + c, gr = r0 + tx;
    if (gc < C && gr < R) dst[(int64_t)gc * ld_out + gr] = tile[tx][c];
  }
}

// 16-B vector form (R, C, strides % 8 == 0, 16-B aligned bases): a lane loads 8 consecutive
// columns of one row, and stores 8 consecutive output elements (8 tile rows of one column), so
// both HBM sides move 128-B row segments per 8 lanes. LDS rows padded to 66 elements (odd dwords).
__global__ __launch_bounds__(256) void transpose_v8_kernel(const bf16_t* __restrict__ in, int64_t ld_in,
                                                           int64_t bstride_in, bf16_t* __restrict__ out,
                                                           int64_t ld_out, int64_t bstride_out, int R, int C) {
  __shared__ bf16_t tile[TT][TT + 2];
  const int b = blockIdx.z;
  const int r0 = blockIdx.y * TT, c0 = blockIdx.x * TT;
  const bf16_t* src = in + (int64_t)b * bstride_in;
  bf16_t* dst = out + (int64_t)b * bstride_out;
  const int ch = threadIdx.x & 7, rr = threadIdx.x >> 3;  // 8-element chunk, row (0..31)
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int r = rr + 32 * h, gr = r0 + r, gc = c0 + ch * 8;
    u32x4 v = {0u, 0u, 0u, 0u};
    if (gr < R && gc < C) v = *(const u32x4*)(src + (int64_t)gr * ld_in + gc);
    uint32_t* t = (uint32_t*)&tile[r][ch * 8];  // 4-B aligned: row stride 132 B, chunk 16 B
    t[0] = v[0]; t[1] = v[1]; t[2] = v[2]; t[3] = v[3];
  }
  __syncthreads();
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int c = rr + 32 * h, gc = c0 + c, gr = r0 + ch * 8;  // output row gc, columns gr..gr+7
    if (gc >= C || gr >= R) continue;
    u32x4 o;
#pragma unroll
    for (int k = 0; k < 4; ++k)
      o[k] = (uint32_t)tile[ch * 8 + 2 * k][c] | ((uint32_t)tile[ch * 8 + 2 * k + 1][c] << 16);
    *(u32x4*)(dst + (int64_t)gc * ld_out + gr) = o;
  }
}

static int launch_transpose(const void* in, int64_t ld_in, int64_t bs_in, void* out, int64_t ld_out,
                            int64_t bs_out, int64_t R, int64_t C, int64_t B, hipStream_t s) {
  dim3 grid((unsigned)((C + TT - 1) / TT), (unsigned)((R + TT - 1) / TT), (unsigned)B);
  if (R % 8 == 0 && C % 8 == 0 && ld_in % 8 == 0 && ld_out % 8 == 0 && bs_in % 8 == 0 && bs_out % 8 == 0 &&
      ((uintptr_t)in % 16) == 0 && ((uintptr_t)out % 16) == 0) {
    hipLaunchKernelGGL(transpose_v8_kernel, grid, dim3(256), 0, s, (const bf16_t*)in, ld_in, bs_in, (bf16_t*)out,
                       ld_out, bs_out, (int)R, (int)C);
    LTX_LAUNCH_CHECK();
    return LTX_OK;
  }
  hipLaunchKernelGGL(transpose_kernel, grid, dim3(256), 0, s, (const bf16_t*)in, ld_in, bs_in,
                     (bf16_t*)out, ld_out, bs_out, (int)R, (int)C);
  LTX_LAUNCH_CHECK();
  return LTX_OK;
}

__global__ void coords_kernel(int64_t* __restrict__ coords, int B, int F, int H, int W) {
  const int64_t N = (int64_t)F * H * W;
  const int64_t total = (int64_t)B * 3 * N;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t n = i % N;
    const int a = (int)((i / N) % 3);
    const int64_t f = n / (H * W), h = (n / W) % H, w = n % W;
    coords[i] = a == 0 ? f : (a == 1 ? h : w);
  }
}

// ---------------------------------------------------------------------------------------------
// Train-step token preparation. One 64(n) x 64(c) tile per block. Latent-side tensors are
// channel-major [B,C,N] (VAE latents), token-side tensors token-major [B,N,C].
//   x_t  = bf16((1-t) x0 + t eps)               rf.py:376-386 (f32 by promotion)
//   v    = bf16((-1) x0 + (+1) eps)             rf.py:400-426
//   in   = bf16(lerp(x_t, ref, 0.85)) if frame 0 else bf16(lerp(x_t, pose, 0.5))
//                                               transformer3d.py:447-466 (ATen lerp formula)
// MODE 0: fused train-step prep (latents channel-major -> x_t, in, v)
// MODE 1: conditioning lerp only (tokens already token-major: in = lerp(tokens, ...))
// ---------------------------------------------------------------------------------------------
// ATen lerp (Lerp.h) as compiled for CPU/GPU: the weight branch of each side contracts to an FMA
__device__ __forceinline__ float torch_lerp(float self, float end, float w) {
  const float d = end - self;
  return fabsf(w) < 0.5f ? fmaf(w, d, self) : fmaf(-d, 1.0f - w, end);
}

template <int MODE>
__global__ __launch_bounds__(256) void prep_tokens_kernel(const bf16_t* __restrict__ lat,
                                                          const bf16_t* __restrict__ ref,
                                                          const bf16_t* __restrict__ pose,
                                                          const bf16_t* __restrict__ noise,
                                                          const float* __restrict__ t,
                                                          bf16_t* __restrict__ x_t,
                                                          bf16_t* __restrict__ model_in,
                                                          bf16_t* __restrict__ v_target, int C,
                                                          int F, int HW) {
  __shared__ bf16_t s_lat[TT][TT + 2];
  __shared__ bf16_t s_cond[TT][TT + 2];
  const int b = blockIdx.z;
  const int n0 = blockIdx.x * TT, c0 = blockIdx.y * TT;
  const int64_t N = (int64_t)F * HW;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  // channel-major loads: row c, column n (coalesced along n)
  for (int c = ty; c < TT; c += 4) {
    const int gc = c0 + c;
    const int64_t gn = n0 + tx;
    bf16_t lv = 0, cv = 0;
    if (gc < C && gn < N) {
      if (MODE == 0) lv = lat[((int64_t)b * C + gc) * N + gn];
      const int64_t f = gn / HW, hw = gn % HW;
      cv = (f == 0) ? ref[((int64_t)b * C + gc) * HW + hw] : pose[((int64_t)b * C + gc) * N + gn];
    }
    s_lat[c][tx] = lv;
    s_cond[c][tx] = cv;
  }
  __syncthreads();
  const float tb = (MODE == 0) ? t[b] : 0.f;
  const float alpha = 1.0f - tb;
  // token-major outputs: row n, column c (coalesced along c)
  for (int n = ty; n < TT; n += 4) {
    const int64_t gn = n0 + n;
    const int gc = c0 + tx;
    if (gn >= N || gc >= C) continue;
    const int64_t o = ((int64_t)b * N + gn) * C + gc;
    float xt;
    if (MODE == 0) {
      const float x0 = bf2f(s_lat[tx][n]);
      const float eps = bf2f(noise[o]);
      xt = rbf(alpha * x0 + tb * eps);
      if (x_t) x_t[o] = f2bf(xt);
      v_target[o] = f2bf((-1.0f) * x0 + 1.0f * eps);
    } else {
      xt = bf2f(noise[o]);  // MODE 1: `noise` carries the input tokens
    }
    const float cond = bf2f(s_cond[tx][n]);
    const bool first = (gn / HW) == 0;
    model_in[o] = f2bf(first ? torch_lerp(xt, cond, 0.85f) : torch_lerp(xt, cond, 0.5f));
  }
}

__global__ void rf_noise_velocity_kernel(const bf16_t* __restrict__ x0, const bf16_t* __restrict__ eps,
                                         const float* __restrict__ t, bf16_t* __restrict__ x_t,
                                         bf16_t* __restrict__ v, int64_t NC, int64_t total) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const float tb = t[i / NC];
    const float a = bf2f(x0[i]), e = bf2f(eps[i]);
    x_t[i] = f2bf((1.0f - tb) * a + tb * e);
    v[i] = f2bf((-1.0f) * a + 1.0f * e);
  }
}

// f32-result form of the same arithmetic: the reference's add_noise / build_velocity_target
// return f32 (f32 [B] timesteps promote the product, rf.py:376-386, 400-426). Inputs bf16 or f32.
template <typename TX, typename TE>
__global__ void rf_noise_velocity_f32_kernel(const TX* __restrict__ x0, const TE* __restrict__ eps,
                                             const float* __restrict__ t, float* __restrict__ x_t,
                                             float* __restrict__ v, int64_t NC, int64_t total) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const float tb = t[i / NC];
    const float a = to_f32(x0[i]), e = to_f32(eps[i]);
    if (x_t) x_t[i] = (1.0f - tb) * a + tb * e;
    if (v) v[i] = (-1.0f) * a + 1.0f * e;
  }
}

// ---------------------------------------------------------------------------------------------
// AdaLN modulation rows (attention.py:229-239; transformer3d.py:554-560):
//   out[b,j,d] = bf16(sst[j,d] + tmod[b, j*D + d]); onep[b,j,d] = bf16(1 + out) for scale rows
// ---------------------------------------------------------------------------------------------
__global__ void ada_kernel(const bf16_t* __restrict__ sst, const bf16_t* __restrict__ tmod, int64_t ld_tmod,
                           int64_t ld_j, bf16_t* __restrict__ out, bf16_t* __restrict__ onep, int B, int P, int D,
                           unsigned scale_mask) {
  const int64_t total = (int64_t)B * P * D;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int d = (int)(i % D);
    const int j = (int)((i / D) % P);
    const int b = (int)(i / ((int64_t)D * P));
    const float s = rbf(bf2f(sst[j * D + d]) + bf2f(tmod[(int64_t)b * ld_tmod + (int64_t)j * ld_j + d]));
    out[i] = f2bf(s);
    if (onep && ((scale_mask >> j) & 1u)) onep[i] = f2bf(1.0f + s);
  }
}

// 16-B form: a block per (b, j) row, 8 columns per lane (D, ld_tmod, ld_j % 8, 16-B aligned).
// The per-token AdaLN of the inference step makes B = batch x tokens: ~400 MB moved per block.
__global__ __launch_bounds__(256) void ada_v8_kernel(const bf16_t* __restrict__ sst, const bf16_t* __restrict__ tmod,
                                                     int64_t ld_tmod, int64_t ld_j, bf16_t* __restrict__ out,
                                                     bf16_t* __restrict__ onep, int B, int P, int D,
                                                     unsigned scale_mask) {
  const int64_t rows = (int64_t)B * P;
  const int D8 = D / 8;
  for (int64_t row = blockIdx.x; row < rows; row += gridDim.x) {
    const int j = (int)(row % P);
    const int64_t b = row / P;
    const bf16_t* tp = tmod + b * ld_tmod + (int64_t)j * ld_j;
    const bf16_t* sp = sst + (int64_t)j * D;
    bf16_t* op = out + row * D;
    const bool sc = onep && ((scale_mask >> j) & 1u);
    for (int c = threadIdx.x; c < D8; c += 256) {
      const u32x4 a = *(const u32x4*)(sp + 8 * c), t = *(const u32x4*)(tp + 8 * c);
      u32x4 o, q;
#pragma unroll
      for (int h = 0; h < 4; ++h) {
        const float s0 = rbf(bf2f((bf16_t)(a[h] & 0xffff)) + bf2f((bf16_t)(t[h] & 0xffff)));
        const float s1 = rbf(bf2f((bf16_t)(a[h] >> 16)) + bf2f((bf16_t)(t[h] >> 16)));
        o[h] = pack2(s0, s1);
        q[h] = pack2(1.0f + s0, 1.0f + s1);
      }
      *(u32x4*)(op + 8 * c) = o;
      if (sc) *(u32x4*)(onep + row * D + 8 * c) = q;
    }
  }
}

// out = bf16(R + bf16(gate[b] * y)), b = m / rows_per_batch: the GATED_RESIDUAL epilogue
// (attention.py:305-308) applied to a library GEMM's y = bf16(x.W^T + b); 8 columns per lane.
// out may alias R.
__global__ __launch_bounds__(256) void gated_residual_kernel(const bf16_t* r, int64_t ldr,
                                                             const bf16_t* __restrict__ gate, int64_t ldg,
                                                             const bf16_t* __restrict__ y, int64_t ldy, bf16_t* out,
                                                             int64_t ldo, int64_t M, int N, int rpb) {
  const int N8 = N / 8;
  const int64_t total = M * N8;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t m = i / N8;
    const int c = (int)(i - m * N8) * 8;
    const u32x4 r4 = *(const u32x4*)(r + m * ldr + c);
    const u32x4 g4 = *(const u32x4*)(gate + (m / rpb) * ldg + c);
    const u32x4 y4 = *(const u32x4*)(y + m * ldy + c);
    u32x4 o;
#pragma unroll
    for (int h = 0; h < 4; ++h) {
      float v[2];
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const float rv = bf2f((bf16_t)(r4[h] >> (16 * e))), gv = bf2f((bf16_t)(g4[h] >> (16 * e)));
        const float yv = bf2f((bf16_t)(y4[h] >> (16 * e)));
        v[e] = rv + rbf(gv * yv);
      }
      o[h] = pack2(v[0], v[1]);
    }
    *(u32x4*)(out + m * ldo + c) = o;
  }
}

// out = bf16(x + y) over rows (autograd's `.grad += new_grad` for bf16 tensors); 8 per lane,
// out may alias x
__global__ __launch_bounds__(256) void add_rows_kernel(const bf16_t* x, int64_t ldx, const bf16_t* __restrict__ y,
                                                       int64_t ldy, bf16_t* out, int64_t ldo, int64_t M, int N) {
  const int N8 = N / 8;
  const int64_t total = M * N8;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t m = i / N8;
    const int c = (int)(i - m * N8) * 8;
    const u32x4 a = *(const u32x4*)(x + m * ldx + c), b = *(const u32x4*)(y + m * ldy + c);
    u32x4 o;
#pragma unroll
    for (int h = 0; h < 4; ++h)
      o[h] = pack2(bf2f((bf16_t)(a[h] & 0xffff)) + bf2f((bf16_t)(b[h] & 0xffff)),
                   bf2f((bf16_t)(a[h] >> 16)) + bf2f((bf16_t)(b[h] >> 16)));
    *(u32x4*)(out + m * ldo + c) = o;
  }
}

// diffusers get_timestep_embedding(flip_sin_to_cos=True, downscale_freq_shift=0), f32 math
// (embeddings.py:10-50 of the reference carries the same formula), preceded by
// `timestep_scale_multiplier * timestep` (transformer3d.py:473-474), result cast to bf16.
__global__ void timestep_kernel(const float* __restrict__ t, float scale, bf16_t* __restrict__ out, int B,
                                int dim) {
  const int half = dim / 2;
  const int total = B * dim;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int b = i / dim, c = i % dim;
    const int k = c < half ? c : c - half;
    float exponent = -9.210340371976184f * (float)k;  // -math.log(10000) in f32
    exponent = exponent / (float)half;
    const float e = expf(exponent);
    const float ts = scale * t[b];
    const float arg = ts * e;
    out[i] = f2bf(c < half ? cosf(arg) : sinf(arg));
  }
}

// out = bf16(dy * gate[b]) row-wise (MulBackward of `gate * attn_output`, attention.py:265-266,
// :305-306); 8 elements per thread, D % 8 == 0
__global__ void gate_mul_kernel(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ gate, int64_t ld_gate,
                                bf16_t* __restrict__ out, int64_t M, int D, int rows_per_batch) {
  const int64_t vecs = M * (D / 8);
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < vecs; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t m = i / (D / 8);
    const int c = (int)(i % (D / 8)) * 8;
    const u32x4 a = *(const u32x4*)(dy + m * D + c);
    const u32x4 gg = *(const u32x4*)(gate + (int64_t)(m / rows_per_batch) * ld_gate + c);
    u32x4 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float lo = bf2f((bf16_t)a[j]) * bf2f((bf16_t)gg[j]);
      const float hi = bf2f((bf16_t)(a[j] >> 16)) * bf2f((bf16_t)(gg[j] >> 16));
      o[j] = pack2(lo, hi);
    }
    *(u32x4*)(out + m * D + c) = o;
  }
}

__global__ void silu_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const float v = bf2f(x[i]);
    y[i] = f2bf(v / (1.0f + expf(-v)));
  }
}

// column sums with f32 accumulation (nn.Linear bias grad = grad_out.sum(0))
// out[r, :] = bf16(sum_b x[b*rows + r, :]) with f32 accumulation, 8 columns per thread: the
// gradient of rows shared by every batch (one prompt expanded over the batch, training.py:415).
__global__ __launch_bounds__(256) void batch_sum_kernel(const bf16_t* __restrict__ x, int64_t ldx, int B,
                                                        int64_t rows, int cols, bf16_t* __restrict__ out,
                                                        int64_t ldo) {
  const int c8 = cols / 8;
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= rows * c8) return;
  const int64_t r = idx / c8;
  const int c = (int)(idx % c8) * 8;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int b = 0; b < B; ++b) {
    const u32x4 v = *(const u32x4*)(x + ((int64_t)b * rows + r) * ldx + c);
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] += bf2f((bf16_t)(v[i >> 1] >> ((i & 1) * 16)));
  }
  u32x4 o;
#pragma unroll
  for (int i = 0; i < 4; ++i) o[i] = pack2(acc[2 * i], acc[2 * i + 1]);
  *(u32x4*)(out + r * ldo + c) = o;
}

__global__ __launch_bounds__(256) void colsum_kernel(const bf16_t* __restrict__ x, int64_t ldx,
                                                     bf16_t* __restrict__ out, int M, int N) {
  __shared__ float part[4][64];
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int rg = threadIdx.x >> 6;
  float s = 0.f;
  if (c < N)
    for (int m = rg; m < M; m += 4) s += bf2f(x[(int64_t)m * ldx + c]);
  part[rg][threadIdx.x & 63] = s;
  __syncthreads();
  if (rg == 0 && c < N) out[c] = f2bf(part[0][threadIdx.x] + part[1][threadIdx.x] + part[2][threadIdx.x] + part[3][threadIdx.x]);
}

// F.mse_loss forward statistics + backward seed (training.py:159-166; ATen mse kernel rounds the
// bf16 difference and its square; mse_loss_backward = sub, * (2/n), * grad, each rounded).
constexpr int MSE_BLOCKS = 256;  // fixed grid: the partials live in stats[4 .. 4 + 3 * MSE_BLOCKS)
__global__ __launch_bounds__(256) void mse_kernel(const bf16_t* __restrict__ o, const bf16_t* __restrict__ v,
                                                  bf16_t* __restrict__ dout, float* __restrict__ stats,
                                                  int64_t n, float norm, float gscale) {
  float s0 = 0.f, s1 = 0.f, s2 = 0.f;
  const int64_t n8 = n / 8;  // 16-B vectors, then a scalar tail
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n8; i += (int64_t)gridDim.x * blockDim.x) {
    const u32x4 ow = *(const u32x4*)(o + 8 * i), vw = *(const u32x4*)(v + 8 * i);
    u32x4 dw;
#pragma unroll
    for (int h = 0; h < 4; ++h) {
      float d2[2];
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const float ov = bf2f((bf16_t)(ow[h] >> (16 * e))), vv = bf2f((bf16_t)(vw[h] >> (16 * e)));
        const float diff = rbf(ov - vv);
        s0 += rbf(diff * diff);
        s1 += vv;
        s2 += vv * vv;
        d2[e] = rbf(diff * norm) * gscale;
      }
      dw[h] = pack2(d2[0], d2[1]);
    }
    if (dout) *(u32x4*)(dout + 8 * i) = dw;
  }
  for (int64_t i = 8 * n8 + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const float ov = bf2f(o[i]), vv = bf2f(v[i]);
    const float diff = rbf(ov - vv);
    s0 += rbf(diff * diff);
    s1 += vv;
    s2 += vv * vv;
    if (dout) dout[i] = f2bf(rbf(diff * norm) * gscale);
  }
  s0 = wave_sum(s0);
  s1 = wave_sum(s1);
  s2 = wave_sum(s2);
  __shared__ float red[3][4];
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    red[0][w] = s0;
    red[1][w] = s1;
    red[2][w] = s2;
  }
  __syncthreads();
  if (threadIdx.x < 3) {
    const int c = threadIdx.x;
    stats[4 + c * MSE_BLOCKS + blockIdx.x] = red[c][0] + red[c][1] + red[c][2] + red[c][3];
  }
}

// fixed-order sum of the per-block partials (deterministic, no atomics)
__global__ __launch_bounds__(256) void mse_finish_kernel(float* __restrict__ stats) {
  const int c = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (c >= 3) return;
  float s = 0.f;
  for (int b = lane; b < MSE_BLOCKS; b += 64) s += stats[4 + c * MSE_BLOCKS + b];
  s = wave_sum(s);
  if (lane == 0) stats[c] = s;
  if (c == 0 && lane == 0) stats[3] = 0.f;
}

// torch.optim.AdamW, foreach implementation order (weight decay, lerp m, v*b2 + (1-b2) g g,
// sqrt, / sqrt(bc2), + eps, p += step_size * m / den), rounding every op for bf16 tensors.
template <bool BF16>
__device__ __forceinline__ void adamw_elem(void* __restrict__ param, const void* __restrict__ grad,
                                           void* __restrict__ m_, void* __restrict__ v_, int64_t i, float decay,
                                           float w1, float b2, float w2, float step_size, float bc2_sqrt, float eps) {
  float p, g, m, v;
  if (BF16) {
    p = bf2f(((bf16_t*)param)[i]); g = bf2f(((const bf16_t*)grad)[i]);
    m = bf2f(((bf16_t*)m_)[i]); v = bf2f(((bf16_t*)v_)[i]);
  } else {
    p = ((float*)param)[i]; g = ((const float*)grad)[i]; m = ((float*)m_)[i]; v = ((float*)v_)[i];
  }
  auto R = [](float x) { return BF16 ? rbf(x) : x; };
  p = R(p * decay);
  m = R(torch_lerp(m, g, w1));
  v = R(v * b2);
  v = R(v + w2 * g * g);
  float den = R(sqrtf(v));
  den = R(den / bc2_sqrt);
  den = R(den + eps);
  p = R(p + step_size * (m / den));
  if (BF16) {
    ((bf16_t*)param)[i] = f2bf(p); ((bf16_t*)m_)[i] = f2bf(m); ((bf16_t*)v_)[i] = f2bf(v);
  } else {
    ((float*)param)[i] = p; ((float*)m_)[i] = m; ((float*)v_)[i] = v;
  }
}

template <bool BF16>
__global__ void adamw_kernel(void* __restrict__ param, const void* __restrict__ grad, void* __restrict__ m_,
                             void* __restrict__ v_, int64_t n, float decay, float w1, float b2, float w2,
                             float step_size, float bc2_sqrt, float eps) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    adamw_elem<BF16>(param, grad, m_, v_, i, decay, w1, b2, w2, step_size, bc2_sqrt, eps);
}

// every trainable tensor of one dtype in one launch: a block per table entry
// (param, grad, exp_avg, exp_avg_sq, first element, count <= 2048), the same per-element math
template <bool BF16>
__global__ __launch_bounds__(256) void adamw_multi_kernel(const int64_t* __restrict__ table, float decay, float w1,
                                                          float b2, float w2, float step_size, float bc2_sqrt,
                                                          float eps) {
  const int64_t* e = table + (int64_t)blockIdx.x * 6;
  void* param = (void*)e[0];
  const void* grad = (const void*)e[1];
  void* m = (void*)e[2];
  void* v = (void*)e[3];
  const int64_t start = e[4], end = e[4] + e[5];
  for (int64_t i = start + threadIdx.x; i < end; i += 256)
    adamw_elem<BF16>(param, grad, m, v, i, decay, w1, b2, w2, step_size, bc2_sqrt, eps);
}

static inline unsigned grid_for(int64_t n, int threads = 256, int64_t cap = 8192) {
  int64_t g = (n + threads - 1) / threads;
  if (g > cap) g = cap;
  if (g < 1) g = 1;
  return (unsigned)g;
}

}  // namespace ltx

using namespace ltx;

extern "C" {

int ltx_abi_version(void) { return 1; }
const char* ltx_last_error(void) { return g_last_error.c_str(); }

int ltx_device_info(int* gfx_arch, int* num_cus) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return fail((int)e, hipGetErrorString(e));
  hipDeviceProp_t prop;
  e = hipGetDeviceProperties(&prop, dev);
  if (e != hipSuccess) return fail((int)e, hipGetErrorString(e));
  if (gfx_arch) {
    const std::string name(prop.gcnArchName);
    *gfx_arch = name.rfind("gfx", 0) == 0 ? (int)std::strtol(name.c_str() + 3, nullptr, 16) : 0;
  }
  if (num_cus) *num_cus = prop.multiProcessorCount;
  if (std::string(prop.gcnArchName).rfind("gfx950", 0) != 0)
    return fail(LTX_ERR_UNSUPPORTED, std::string("libltxhip is built for gfx950, device is ") + prop.gcnArchName);
  return LTX_OK;
}

int ltx_patchify_bf16(const void* latents, void* tokens, int64_t B, int64_t C, int64_t F, int64_t H,
                      int64_t W, void* stream) {
  LTX_CHECK_ARG(latents && tokens && B > 0 && C > 0 && F > 0 && H > 0 && W > 0, "patchify: bad args");
  const int64_t N = F * H * W;
  // per batch: [C, N] -> [N, C]
  return launch_transpose(latents, N, C * N, tokens, C, N * C, C, N, B, (hipStream_t)stream);
}

int ltx_unpatchify_bf16(const void* tokens, void* latents, int64_t B, int64_t C, int64_t F, int64_t H,
                        int64_t W, void* stream) {
  LTX_CHECK_ARG(latents && tokens && B > 0 && C > 0 && F > 0 && H > 0 && W > 0, "unpatchify: bad args");
  const int64_t N = F * H * W;
  return launch_transpose(tokens, C, N * C, latents, N, C * N, N, C, B, (hipStream_t)stream);
}

int ltx_latent_coords(int64_t* coords, int64_t B, int64_t F, int64_t H, int64_t W, void* stream) {
  LTX_CHECK_ARG(coords && B > 0 && F > 0 && H > 0 && W > 0, "latent_coords: bad args");
  const int64_t total = B * 3 * F * H * W;
  hipLaunchKernelGGL(coords_kernel, dim3(grid_for(total)), dim3(256), 0, (hipStream_t)stream, coords, (int)B,
                     (int)F, (int)H, (int)W);
  LTX_LAUNCH_CHECK();
  return LTX_OK;
}

int ltx_rf_noise_velocity(const void* tokens, const void* noise, const float* t, void* x_t, void* v_target,
                          int64_t B, int64_t NC, void* stream) {
  LTX_CHECK_ARG(tokens && noise && t && x_t && v_target && B > 0 && NC > 0, "rf_noise_velocity: bad args");
  const int64_t total = B * NC;
  hipLaunchKernelGGL(rf_noise_velocity_kernel, dim3(grid_for(total)), dim3(256), 0, (hipStream_t)stream,
                     (const bf16_t*)tokens, (const bf16_t*)noise, t, (bf16_t*)x_t, (bf16_t*)v_target, NC, total);
  LTX_LAUNCH_CHECK();
  return LTX_OK;
}

int ltx_rf_noise_velocity_f32(const void* tokens, int tokens_f32, const void* noise, int noise_f32,
                              const float* t, float* x_t, float* v_target, int64_t B, int64_t NC,
                              void* stream) {
  LTX_CHECK_ARG(tokens && noise && t && (x_t || v_target) && B > 0 && NC > 0, "rf_noise_velocity_f32: bad args");
  const int64_t total = B * NC;
  const dim3 g(grid_for(total)), blk(256);
  hipStream_t s = (hipStream_t)stream;
  if (tokens_f32 && noise_f32)
    hipLaunchKernelGGL((rf_noise_velocity_f32_kernel<float, float>), g, blk, 0, s, (const float*)tokens,
                       (const float*)noise, t, x_t, v_target, NC, total);
  else if (tokens_f32)
    hipLaunchKernelGGL((rf_noise_velocity_f32_kernel<float, bf16_t>), g, blk, 0, s, (const float*)tokens,
                       (const bf16_t*)noise, t, x_t, v_target, NC, total);
  else if (noise_f32)
    hipLaunchKernelGGL((rf_noise_velocity_f32_kernel<bf16_t, float>), g, blk, 0, s, (const bf16_t*)tokens,
                       (const float*)noise, t, x_t, v_target, NC, total);
  else
    hipLaunchKernelGGL((rf_noise_velocity_f32_kernel<bf16_t, bf16_t>), g, blk, 0, s, (const bf16_t*)tokens,
                       (const bf16_t*)noise, t, x_t, v_target, NC, total);
  LTX_LAUNCH_CHECK();
  return LTX_OK;
}

int ltx_condition_lerp(const void* tokens, const void* ref, const void* pose, void* out, int64_t B, int64_t C,
                       int64_t F, int64_t H, int64_t W, void* stream) {
  LTX_CHECK_ARG(tokens && ref && pose && out && B > 0 && C > 0 && F > 0 && H > 0 && W > 0,
                "condition_lerp: bad args");
  const int64_t N = F * H * W;
  dim3 grid((unsigned)((N + TT - 1) / TT), (unsigned)((C + TT - 1) / TT), (unsigned)B);
  hipLaunchKernelGGL(prep_tokens_kernel<1>, grid, dim3(256), 0, (hipStream_t)stream, nullptr, (const bf16_t*)ref,
                     (const bf16_t*)pose, (const bf16_t*)tokens, nullptr, nullptr, (bf16_t*)out, nullptr,
                     (int)C, (int)F, (int)(H * W));
  LTX_LAUNCH_CHECK();
  return LTX_OK;
}

int ltx_rf_prepare_tokens(const void* latents, const void* ref, const void* pose, const void* noise,
                          const float* t, void* x_t, void* model_in, void* v_target, int64_t B, int64_t C,
                          int64_t F, int64_t H, int64_t W, void* stream) {
  LTX_CHECK_ARG(latents && ref && pose && noise && t && model_in && v_target, "rf_prepare_tokens: null");
  LTX_CHECK_ARG(B > 0 && C > 0 && F > 0 && H > 0 && W > 0, "rf_prepare_tokens: bad shape");
  const int64_t N = F * H * W;
  dim3 grid((unsigned)((N + TT - 1) / TT), (unsigned)((C + TT - 1) / TT), (unsigned)B);
  hipLaunchKernelGGL(prep_tokens_kernel<0>, grid, dim3(256), 0, (hipStream_t)stream, (const bf16_t*)latents,
                     (const bf16_t*)ref, (const bf16_t*)pose, (const bf16_t*)noise, t, (bf16_t*)x_t,
                     (bf16_t*)model_in, (bf16_t*)v_target, (int)C, (int)F, (int)(H * W));
  LTX_LAUNCH_CHECK();
  return LTX_OK;
}

int ltx_ada_modulation(const void* sst, const void* tmod, int64_t ld_tmod, int64_t ld_j, void* out, void* onep_out,
                       int64_t B, int64_t P, int64_t D, int64_t scale_mask, void* stream) {
  LTX_CHECK_ARG(sst && tmod && out && B > 0 && P > 0 && P <= 32 && D > 0, "ada_modulation: bad args");
  const int64_t total = B * P * D;
  if (D % 8 == 0 && ld_tmod % 8 == 0 && ld_j % 8 == 0 &&
      (((uintptr_t)sst | (uintptr_t)tmod | (uintptr_t)out | (uintptr_t)onep_out) % 16) == 0) {
    const int64_t rows = B * P;
    hipLaunchKernelGGL(ada_v8_kernel, dim3((unsigned)(rows < 16384 ? rows : 16384)), dim3(256), 0,
                       (hipStream_t)stream, (const bf16_t*)sst, (const bf16_t*)tmod, ld_tmod, ld_j, (bf16_t*)out,
                       (bf16_t*)onep_out, (int)B, (int)P, (int)D, (unsigned)scale_mask);
    LTX_LAUNCH_CHECK();
    return LTX_OK;
  }
  hipLaunchKernelGGL(ada_kernel, dim3(grid_for(total)), dim3(256), 0, (hipStream_t)stream, (const bf16_t*)sst,
                     (const bf16_t*)tmod, ld_tmod, ld_j, (bf16_t*)out, (bf16_t*)onep_out, (int)B, (int)P, (int)D,
                     (unsigned)scale_mask);
  LTX_LAUNCH_CHECK();
  return LTX_OK;
}

int ltx_timestep_embedding(const float* t, float scale, void* out, int64_t B, int64_t dim, void* stream) {
  LTX_CHECK_ARG(t && out && B > 0 && dim > 0 && dim % 2 == 0, "timestep_embedding: bad args");
  hipLaunchKernelGGL(timestep_kernel, dim3(grid_for(B * dim)), dim3(256), 0, (hipStream_t)stream, t, scale,
                     (bf16_t*)out, (int)B, (int)dim);
  LTX_LAUNCH_CHECK();
  return LTX_OK;
}

int ltx_add_bf16(const void* x, int64_t ldx, const void* y, int64_t ldy, void* out, int64_t ldo, int64_t M,
                 int64_t N, void* stream) {
  LTX_CHECK_ARG(x && y && out && M > 0 && N > 0 && N % 8 == 0 && ldx % 8 == 0 && ldy % 8 == 0 && ldo % 8 == 0 &&
                    (((uintptr_t)x | (uintptr_t)y | (uintptr_t)out) % 16) == 0,
                "add_bf16: rows must be 16-B aligned, N % 8 == 0");
  hipLaunchKernelGGL(add_rows_kernel, dim3(grid_for(M * N / 8)), dim3(256), 0, (hipStream_t)stream, (const bf16_t*)x,
                     ldx, (const bf16_t*)y, ldy, (bf16_t*)out, ldo, M, (int)N);
  LTX_LAUNCH_CHECK();
  return LTX_OK;
}

int ltx_gated_residual_bf16(const void* r, int64_t ldr, const void* gate, int64_t ld_gate, const void* y,
                            int64_t ldy, void* out, int64_t ldo, int64_t M, int64_t N, int64_t rows_per_batch,
                            void* stream) {
  LTX_CHECK_ARG(r && gate && y && out && M > 0 && N > 0 && N % 8 == 0, "gated_residual: bad args");
  LTX_CHECK_ARG(ldr % 8 == 0 && ld_gate % 8 == 0 && ldy % 8 == 0 && ldo % 8 == 0 &&
                    (((uintptr_t)r | (uintptr_t)gate | (uintptr_t)y | (uintptr_t)out) % 16) == 0,
                "gated_residual: rows must be 16-B aligned");
  const int rpb = (int)(rows_per_batch > 0 ? rows_per_batch : M);
  hipLaunchKernelGGL(gated_residual_kernel, dim3(grid_for(M * N / 8)), dim3(256), 0, (hipStream_t)stream,
                     (const bf16_t*)r, ldr, (const bf16_t*)gate, ld_gate, (const bf16_t*)y, ldy, (bf16_t*)out, ldo,
                     M, (int)N, rpb);
  LTX_LAUNCH_CHECK();
  return LTX_OK;
}

int ltx_gate_mul_bf16(const void* dy, const void* gate, int64_t ld_gate, void* out, int64_t M, int64_t D,
                      int64_t rows_per_batch, void* stream) {
  LTX_CHECK_ARG(dy && gate && out && M > 0 && D > 0 && D % 8 == 0 && ld_gate % 8 == 0, "gate_mul: bad args");
  hipLaunchKernelGGL(gate_mul_kernel, dim3(grid_for(M * D / 8)), dim3(256), 0, (hipStream_t)stream,
                     (const bf16_t*)dy, (const bf16_t*)gate, ld_gate, (bf16_t*)out, M, (int)D,
                     (int)(rows_per_batch > 0 ? rows_per_batch : M));
  LTX_LAUNCH_CHECK();
  return LTX_OK;
}

int ltx_silu_bf16(const void* x, void* y, int64_t n, void* stream) {
  LTX_CHECK_ARG(x && y && n > 0, "silu: bad args");
  hipLaunchKernelGGL(silu_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, (const bf16_t*)x,
                     (bf16_t*)y, n);
  LTX_LAUNCH_CHECK();
  return LTX_OK;
}

int ltx_transpose_bf16(const void* in, int64_t ld_in, void* out, int64_t ld_out, int64_t R, int64_t C,
                       void* stream) {
  LTX_CHECK_ARG(in && out && R > 0 && C > 0 && ld_in >= C && ld_out >= R, "transpose: bad args");
  return launch_transpose(in, ld_in, 0, out, ld_out, 0, R, C, 1, (hipStream_t)stream);
}

int ltx_colsum_bf16(const void* x, int64_t ldx, void* out, int64_t M, int64_t N, void* stream) {
  LTX_CHECK_ARG(x && out && M > 0 && N > 0 && ldx >= N, "colsum: bad args");
  hipLaunchKernelGGL(colsum_kernel, dim3((unsigned)((N + 63) / 64)), dim3(256), 0, (hipStream_t)stream,
                     (const bf16_t*)x, ldx, (bf16_t*)out, (int)M, (int)N);
  LTX_LAUNCH_CHECK();
  return LTX_OK;
}

int ltx_batch_sum_bf16(const void* x, int64_t ldx, int64_t B, int64_t rows, int64_t cols, void* out, int64_t ldo,
                       void* stream) {
  LTX_CHECK_ARG(x && out && B > 0 && rows > 0 && cols > 0 && cols % 8 == 0 && ldx % 8 == 0 && ldo % 8 == 0,
                "batch_sum: bad args (cols and leading dims must be multiples of 8)");
  const int64_t n = rows * (cols / 8);
  hipLaunchKernelGGL(batch_sum_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     (const bf16_t*)x, ldx, (int)B, rows, (int)cols, (bf16_t*)out, ldo);
  LTX_LAUNCH_CHECK();
  return LTX_OK;
}

int ltx_mse_fwd_bwd(const void* out, const void* v, void* dout, float* stats, int64_t n, float grad_scale,
                    void* stream) {
  LTX_CHECK_ARG(out && v && stats && n > 0, "mse: bad args");
  LTX_CHECK_ARG(((uintptr_t)out | (uintptr_t)v | (uintptr_t)dout) % 16 == 0, "mse: operands must be 16-B aligned");
  const float norm = (float)(2.0 / (double)n);
  hipLaunchKernelGGL(mse_kernel, dim3(MSE_BLOCKS), dim3(256), 0, (hipStream_t)stream, (const bf16_t*)out,
                     (const bf16_t*)v, (bf16_t*)dout, stats, n, norm, grad_scale);
  hipLaunchKernelGGL(mse_finish_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, stats);
  LTX_LAUNCH_CHECK();
  return LTX_OK;
}

int ltx_adamw_multi(const int64_t* table, int64_t nchunks, int is_bf16, float lr, float beta1, float beta2, float eps,
                    float weight_decay, int64_t step, void* stream) {
  LTX_CHECK_ARG(table && nchunks > 0 && nchunks < (1LL << 31) && step >= 1, "adamw_multi: bad args");
  const double bc1 = 1.0 - std::pow((double)beta1, (double)step);
  const double bc2 = 1.0 - std::pow((double)beta2, (double)step);
  const float decay = (float)(1.0 - (double)lr * (double)weight_decay);
  const float step_size = (float)(-((double)lr / bc1));
  const float bc2_sqrt = (float)std::sqrt(bc2);
  const float w1 = (float)(1.0 - (double)beta1), w2 = (float)(1.0 - (double)beta2);
  if (is_bf16)
    hipLaunchKernelGGL(adamw_multi_kernel<true>, dim3((unsigned)nchunks), dim3(256), 0, (hipStream_t)stream, table,
                       decay, w1, beta2, w2, step_size, bc2_sqrt, eps);
  else
    hipLaunchKernelGGL(adamw_multi_kernel<false>, dim3((unsigned)nchunks), dim3(256), 0, (hipStream_t)stream, table,
                       decay, w1, beta2, w2, step_size, bc2_sqrt, eps);
  LTX_LAUNCH_CHECK();
  return LTX_OK;
}

int ltx_adamw_step(void* param, const void* grad, void* exp_avg, void* exp_avg_sq, int64_t n, int is_bf16,
                   float lr, float beta1, float beta2, float eps, float weight_decay, int64_t step, void* stream) {
  LTX_CHECK_ARG(param && grad && exp_avg && exp_avg_sq && n > 0 && step >= 1, "adamw: bad args");
  const double bc1 = 1.0 - std::pow((double)beta1, (double)step);
  const double bc2 = 1.0 - std::pow((double)beta2, (double)step);
  const float decay = (float)(1.0 - (double)lr * (double)weight_decay);
  const float step_size = (float)(-((double)lr / bc1));
  const float bc2_sqrt = (float)std::sqrt(bc2);
  const float w1 = (float)(1.0 - (double)beta1), w2 = (float)(1.0 - (double)beta2);
  if (is_bf16)
    hipLaunchKernelGGL(adamw_kernel<true>, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, param, grad,
                       exp_avg, exp_avg_sq, n, decay, w1, beta2, w2, step_size, bc2_sqrt, eps);
  else
    hipLaunchKernelGGL(adamw_kernel<false>, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, param, grad,
                       exp_avg, exp_avg_sq, n, decay, w1, beta2, w2, step_size, bc2_sqrt, eps);
  LTX_LAUNCH_CHECK();
  return LTX_OK;
}

}  // extern "C"
