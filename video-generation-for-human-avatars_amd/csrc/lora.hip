// LoRA adapter contractions in f32 (peft 0.17.1 keeps adapters in f32 on a bf16 base:
// training.py:50-68 + autocast_adapter_dtype). Rank r <= 32 makes these skinny, so they are
// HBM-bound (x or dY is read once: 2 B/element for 2r FLOP/element) and run on the exact-f32
// matrix core v_mfma_f32_16x16x4_f32 (an f32 fma chain, bitwise like the VALU, at 4x its rate),
// which keeps the adapters' f32 semantics while freeing the VALU for address math.
// The up-projection (B) and its input-gradient half are fused into the bf16 GEMM epilogues
// (gemm.hip: LTX_EPI_LORA / LTX_EPI_LORA_DGRAD_ACCUM).
#include "common.h"
#include "ltx_hip.h"

namespace ltx {

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// out[m,j] = alpha * sum_k x[m,k] * Wr[j*wj + k*wk]
// Block = 4 waves on the same 16 rows, K split 4 ways (grid = M/16 blocks); per 32-deep k chunk
// a lane loads 8 consecutive k of its row (one 16-B load) and of its j row, and issues 8 MFMAs
// whose k index g = lane>>4 stands for k = kb + 8g + i (the same permutation on both operands).
// The 4 partial 16 x r tiles are summed through LDS.
template <int R>
__global__ __launch_bounds__(256) void lora_down_kernel(const bf16_t* __restrict__ x, int64_t ldx,
                                                        const float* __restrict__ Wr, int64_t wj, int64_t wk,
                                                        float* __restrict__ out, int64_t ldo, int M, int K,
                                                        float alpha) {
  constexpr int JT = R / 16;  // 16-wide j tiles (R in {16, 32}); R = 8 runs as a padded tile
  constexpr int JTT = JT > 0 ? JT : 1;
  __shared__ float part[4][16][R >= 16 ? R : 16];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int m0 = blockIdx.x * 16;
  const int row = min(m0 + (lane & 15), M - 1);
  const int g = lane >> 4;
  const int kper = K / 4;
  const int kbeg = wave * kper, kend = kbeg + kper;
  f32x4 acc[JTT];
#pragma unroll
  for (int t = 0; t < JTT; ++t) acc[t] = (f32x4){0.f, 0.f, 0.f, 0.f};
  const bf16_t* xr = x + (int64_t)row * ldx;
  for (int kb = kbeg; kb < kend; kb += 32) {
    const int k = kb + 8 * g;
    const u32x4 xv = *(const u32x4*)(xr + k);
    float xf[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) xf[i] = bf2f((bf16_t)(xv[i >> 1] >> ((i & 1) * 16)));
#pragma unroll
    for (int t = 0; t < JTT; ++t) {
      const int j = t * 16 + (lane & 15);
      float wv[8];
      if (j < R) {
        const float* wp = Wr + (int64_t)j * wj + (int64_t)k * wk;
        if (wk == 1) {
          const f32x4 a = *(const f32x4*)wp, b = *(const f32x4*)(wp + 4);
#pragma unroll
          for (int i = 0; i < 4; ++i) { wv[i] = a[i]; wv[4 + i] = b[i]; }
        } else {
#pragma unroll
          for (int i = 0; i < 8; ++i) wv[i] = wp[(int64_t)i * wk];
        }
      } else {
#pragma unroll
        for (int i = 0; i < 8; ++i) wv[i] = 0.f;
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[t] = mfma4(xf[i], wv[i], acc[t]);
    }
  }
  // C layout: col j = lane & 15 (+16t), row m = (lane >> 4) * 4 + reg
#pragma unroll
  for (int t = 0; t < JTT; ++t)
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const int j = t * 16 + (lane & 15);
      if (j < (R >= 16 ? R : 16)) part[wave][(lane >> 4) * 4 + rr][j] = acc[t][rr];
    }
  __syncthreads();
  for (int e = threadIdx.x; e < 16 * R; e += 256) {
    const int rr = e / R, j = e % R;
    const int m = m0 + rr;
    if (m < M) out[(int64_t)m * ldo + j] = (part[0][rr][j] + part[1][rr][j] + part[2][rr][j] + part[3][rr][j]) * alpha;
  }
}

// dw(n,j) += alpha * sum_{m in split} y[m,n] * u[m,j]  (f32 atomics across splits)
// Block = 4 waves x 16 columns n; rows streamed in 64-row tiles through LDS (y as bf16, u as
// f32); per 4 rows one MFMA per 16-wide j tile: A = y^T [16 n x 4 m], B = u [4 m x 16 j].
template <int R>
__global__ __launch_bounds__(256) void lora_wgrad_kernel(const bf16_t* __restrict__ y, int64_t ldy,
                                                         const float* __restrict__ u, int64_t ldu,
                                                         float* __restrict__ dw, int64_t on, int64_t oj, int M,
                                                         int N, int rows_per_split, float alpha) {
  constexpr int RP = R >= 16 ? R : 16;
  constexpr int JT = RP / 16;
  __shared__ bf16_t ys[64][64 + 2];
  __shared__ float us[64][RP + 1];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int n0 = blockIdx.x * 64;
  const int mb = blockIdx.y * rows_per_split;
  const int me = min(M, mb + rows_per_split);
  f32x4 acc[JT];
#pragma unroll
  for (int t = 0; t < JT; ++t) acc[t] = (f32x4){0.f, 0.f, 0.f, 0.f};
  for (int m0 = mb; m0 < me; m0 += 64) {
    // stage y[64 rows][64 cols]: 256 threads x 16 elements (two 16-B loads)
    {
      const int r = tid >> 2, c = (tid & 3) * 16;
      const int m = m0 + r;
      u32x4 a = {0, 0, 0, 0}, b = {0, 0, 0, 0};
      if (m < me && n0 + c < N) {
        const bf16_t* p = y + (int64_t)m * ldy + n0 + c;
        a = *(const u32x4*)p;
        if (n0 + c + 8 < N) b = *(const u32x4*)(p + 8);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        ys[r][c + 2 * i] = (bf16_t)a[i];
        ys[r][c + 2 * i + 1] = (bf16_t)(a[i] >> 16);
        ys[r][c + 8 + 2 * i] = (bf16_t)b[i];
        ys[r][c + 8 + 2 * i + 1] = (bf16_t)(b[i] >> 16);
      }
    }
    for (int e = tid; e < 64 * RP; e += 256) {
      const int r = e / RP, j = e % RP;
      const int m = m0 + r;
      us[r][j] = (m < me && j < R) ? u[(int64_t)m * ldu + j] : 0.f;
    }
    __syncthreads();
#pragma unroll 4
    for (int mm = 0; mm < 64; mm += 4) {
      const float a = bf2f(ys[mm + (lane >> 4)][wave * 16 + (lane & 15)]);
#pragma unroll
      for (int t = 0; t < JT; ++t) acc[t] = mfma4(a, us[mm + (lane >> 4)][t * 16 + (lane & 15)], acc[t]);
    }
    __syncthreads();
  }
  // C: row n = wave*16 + (lane>>4)*4 + reg, col j = t*16 + (lane&15)
#pragma unroll
  for (int t = 0; t < JT; ++t)
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const int n = n0 + wave * 16 + (lane >> 4) * 4 + rr;
      const int j = t * 16 + (lane & 15);
      if (n < N && j < R) atomicAdd(dw + (int64_t)n * on + (int64_t)j * oj, acc[t][rr] * alpha);
    }
}

// 3-term bf16 split of an f32 [R, r] operand for the K-extension LoRA fusion: with
// v = hi + lo (hi = bf16(v), lo = bf16(v - hi)), the activation row is [hi | hi | lo | 0..] and
// the weight row [hi | lo | hi | 0..], so their dot product is a.hi*w.hi + a.hi*w.lo + a.lo*w.hi
// (the lo*lo term, ~2^-16 relative, is the only thing dropped).
__global__ void lora_split_kernel(const float* __restrict__ src, int64_t rs, int64_t cs, float scale, int R,
                                  int r, int role, bf16_t* __restrict__ out, int64_t ldo, int K2) {
  const int64_t total = (int64_t)R * K2;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int row = (int)(i / K2), c = (int)(i % K2);
    const int seg = c / r, j = c % r;
    float o = 0.f;
    if (seg < 3) {
      const float v = src[(int64_t)row * rs + (int64_t)j * cs] * scale;
      const float hi = rbf(v);
      const float lo = rbf(v - hi);
      // activation: hi, hi, lo ; weight: hi, lo, hi
      o = (role == 0) ? (seg < 2 ? hi : lo) : (seg == 1 ? lo : hi);
    }
    out[(int64_t)row * ldo + c] = f2bf(o);
  }
}

}  // namespace ltx

using namespace ltx;

extern "C" int ltx_lora_split_bf16(const float* src, int64_t rs, int64_t cs, float scale, int64_t R, int64_t r,
                                   int role, void* out, int64_t ldo, int64_t K2, void* stream) {
  LTX_CHECK_ARG(src && out && R > 0 && r > 0 && (role == 0 || role == 1), "lora_split: bad args");
  LTX_CHECK_ARG(K2 >= 3 * r && K2 % 64 == 0 && ldo >= K2, "lora_split: K2 must be >= 3r and a multiple of 64");
  const int64_t total = R * K2;
  int64_t g = (total + 255) / 256;
  if (g > 4096) g = 4096;
  hipLaunchKernelGGL(lora_split_kernel, dim3((unsigned)g), dim3(256), 0, (hipStream_t)stream, src, rs, cs, scale,
                     (int)R, (int)r, role, (bf16_t*)out, ldo, (int)K2);
  LTX_LAUNCH_CHECK();
  return LTX_OK;
}

extern "C" int ltx_lora_down(const void* x, int64_t ldx, const float* Wr, int64_t wj, int64_t wk, float* out,
                             int64_t ldo, int64_t M, int64_t K, int64_t r, float alpha, void* stream) {
  LTX_CHECK_ARG(x && Wr && out && M > 0 && K > 0, "lora_down: bad args");
  LTX_CHECK_ARG(K % 128 == 0 && ldx % 8 == 0 && ((uintptr_t)x % 16) == 0, "lora_down: K %128, 16-B rows");
  LTX_CHECK_ARG(wk != 1 || (wj % 4 == 0 && ((uintptr_t)Wr % 16) == 0), "lora_down: W rows must be 16-B aligned");
  const dim3 grid((unsigned)((M + 15) / 16));
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
  LTX_CHECK_ARG(N % 8 == 0 && ldy % 8 == 0 && ((uintptr_t)y % 16) == 0, "lora_wgrad: y rows must be 16-B aligned");
  hipStream_t s = (hipStream_t)stream;
  hipError_t e = hipMemsetAsync(dw, 0, (size_t)N * r * sizeof(float), s);
  if (e != hipSuccess) return fail((int)e, hipGetErrorString(e));
  const int nb = (int)((N + 63) / 64);
  int splits = (int)((1024 + nb - 1) / nb);
  const int max_splits = (int)((M + 63) / 64);
  if (splits > max_splits) splits = max_splits;
  int rps = (int)((M + splits - 1) / splits);
  rps = (rps + 63) / 64 * 64;
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
