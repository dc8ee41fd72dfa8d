// Shared helpers for the LTX-Video MI355X (gfx950 / CDNA4) kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>

namespace ltx {

typedef unsigned short bf16_t;  // raw bf16 bits in HBM
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

#define LDS_PTR(p) ((__attribute__((address_space(3))) void*)(p))

__device__ __forceinline__ float bf2f(bf16_t x) { return __uint_as_float(((unsigned)x) << 16); }

// round-to-nearest-even f32 -> bf16 (NaN kept a NaN: lowers to v_cvt_pk_bf16_f32 on gfx950)
__device__ __forceinline__ bf16_t f2bf(float f) {
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(bf16_t, b);
}
// two floats -> packed bf16 pair (one v_cvt_pk_bf16_f32; the scalar form made hipcc pair values
// from different calls and shuffle them back with and / shift / or)
typedef __bf16 bf16x2_cvt_t __attribute__((ext_vector_type(2)));
typedef float f32x2_cvt_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ unsigned pack2(float lo, float hi) {
  return __builtin_bit_cast(unsigned, __builtin_convertvector((f32x2_cvt_t){lo, hi}, bf16x2_cvt_t));
}
// value rounded through bf16 and back (mirrors an eager bf16 op boundary)
__device__ __forceinline__ float rbf(float f) { return bf2f(f2bf(f)); }
__device__ __forceinline__ float to_f32(bf16_t x) { return bf2f(x); }
__device__ __forceinline__ float to_f32(float x) { return x; }

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// tanh-approximate GELU exactly as ATen computes it in float (F.gelu(approximate="tanh"))
__device__ __forceinline__ float gelu_tanh(float x) {
  const float kBeta = 0.7978845608028654f;  // sqrt(2/pi)
  const float kKappa = 0.044715f;
  float x_cube = x * x * x;
  float inner = kBeta * (x + kKappa * x_cube);
  return 0.5f * x * (1.0f + tanhf(inner));
}
// tanh via exp: 1 - 2 / (1 + e^{2u}) (v_exp_f32 + v_rcp_f32); |error| ~1e-7 absolute, invisible
// after the bf16 rounding of the GELU output except for rare 1-ulp ties
__device__ __forceinline__ float fast_tanh(float u) {
  const float e = __expf(2.0f * u);
  return 1.0f - 2.0f / (1.0f + e);
}
__device__ __forceinline__ float gelu_tanh_fast(float x) {
  const float kBeta = 0.7978845608028654f;
  const float kKappa = 0.044715f;
  float x_cube = x * x * x;
  float inner = kBeta * (x + kKappa * x_cube);
  return 0.5f * x * (1.0f + fast_tanh(inner));
}
// GEMM-epilogue forms on float pairs (v_pk_mul/fma/add_f32: two values per VALU instruction).
// 0.5 x (1 + tanh(u)) == x * sigmoid(2u) == x / (1 + 2^w), w = -2 log2(e) u = x (A + B x^2):
// 3 packed ops + v_exp_f32 + 1 packed add + v_rcp_f32 + 1 packed mul per pair instead of ~14 ops
// per value. Differs from the tanh form by f32 rounding only (v_exp/v_rcp ~1 ulp).
typedef float f32x2 __attribute__((ext_vector_type(2)));
namespace gelu_k {
constexpr float A = -2.0f * 0.7978845608028654f * 1.4426950408889634f;  // -2 sqrt(2/pi) log2(e)
constexpr float B = A * 0.044715f;
constexpr float C0 = 2.0f * 0.7978845608028654f;                        // 2u' = C0 + C1 x^2
constexpr float C1 = 6.0f * 0.7978845608028654f * 0.044715f;
}  // namespace gelu_k
__device__ __forceinline__ f32x2 sigmoid2u_pk(f32x2 x, f32x2 x2) {
  const f32x2 w = x * __builtin_elementwise_fma(x2, (f32x2)gelu_k::B, (f32x2)gelu_k::A);
  f32x2 d;
  d[0] = __builtin_amdgcn_exp2f(w[0]);
  d[1] = __builtin_amdgcn_exp2f(w[1]);
  d = d + 1.0f;
  f32x2 s;
  s[0] = __builtin_amdgcn_rcpf(d[0]);
  s[1] = __builtin_amdgcn_rcpf(d[1]);
  return s;
}
__device__ __forceinline__ f32x2 gelu_tanh_pk(f32x2 x) { return x * sigmoid2u_pk(x, x * x); }
// d gelu / dx = s + x s (1 - s) 2u'  (s = sigmoid(2u); 0.5(1 + tanh) = s, 1 - tanh^2 = 4 s (1 - s)),
// from the forward's s: 5 packed ops per pair on top of the GELU itself
__device__ __forceinline__ f32x2 gelu_tanh_grad_s_pk(f32x2 x, f32x2 x2, f32x2 s) {
  const f32x2 du = __builtin_elementwise_fma(x2, (f32x2)gelu_k::C1, (f32x2)gelu_k::C0);
  return __builtin_elementwise_fma(s * (x * (1.0f - s)), du, s);
}
// the same from the GELU output g = x s: s + g (1 - s) 2u' (3 packed ops)
__device__ __forceinline__ f32x2 gelu_tanh_grad_g_pk(f32x2 x2, f32x2 s, f32x2 g) {
  const f32x2 du = __builtin_elementwise_fma(x2, (f32x2)gelu_k::C1, (f32x2)gelu_k::C0);
  return __builtin_elementwise_fma(__builtin_elementwise_fma(-g, s, g), du, s);
}
__device__ __forceinline__ f32x2 gelu_tanh_grad_pk(f32x2 x) {
  const f32x2 x2 = x * x;
  return gelu_tanh_grad_s_pk(x, x2, sigmoid2u_pk(x, x2));
}
// The GELU derivative the forward keeps for the backward, as 16-bit snorm of d / 2 (gelu_tanh' lies
// in (-0.17, 1.13)): q = rint(32767 clamp(d / 2, -1, 1)), one v_cvt_pknorm_i16_f32 per pair;
// absolute error <= 2^-15, against fp16's 2^-11 relative near 1. The backward's g * q is exact in f32
// (8 + 15 significant bits), so dF = bf16((g * q) * 2 / 32767) rounds twice only at the 2^-24 level.
constexpr float GELU_DQ = 2.0f / 32767.0f;
__device__ __forceinline__ uint32_t pack_gelu_q(f32x2 d) {
  const f32x2 h = d * 0.5f;
  return __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_pknorm_i16(h[0], h[1]));
}
__device__ __forceinline__ float gelu_qlo(uint32_t w) { return (float)(int16_t)(uint16_t)w; }
__device__ __forceinline__ float gelu_qhi(uint32_t w) { return (float)((int32_t)w >> 16); }

// d gelu_tanh / dx, same association as ATen's GeluBackward (approximate="tanh"); the caller
// multiplies by dy
__device__ __forceinline__ float gelu_tanh_grad(float x) {
  const float kBeta = 0.7978845608028654f;
  const float kKappa = 0.044715f;
  float x_sq = x * x;
  float x_cube = x_sq * x;
  float inner = kBeta * (x + kKappa * x_cube);
  float tanh_inner = fast_tanh(inner);
  float left = 0.5f * x;
  float right = 1.0f + tanh_inner;
  float left_derivative = 0.5f * right;
  float tanh_derivative = 1.0f - tanh_inner * tanh_inner;
  float inner_derivative = kBeta * (1.0f + 3.0f * kKappa * x_sq);
  float right_derivative = left * tanh_derivative * inner_derivative;
  return left_derivative + right_derivative;
}

}  // namespace ltx

// ---- host-side error plumbing -----------------------------------------------------------------
namespace ltx {
void set_error(const std::string& msg);
int fail(int code, const std::string& msg);
// the caller-owned f32 scratch of stream s (gemm.hip: ltx_gemm_set_workspace /
// ltx_gemm_set_stream_workspace); kernels on one stream run in order, so any launcher on that
// stream may use it between its own launches. bytes = 0 when none was set.
float* stream_workspace(hipStream_t s, size_t* bytes);
// a packed bf16 pair as the operand type of v_dot2c_f32_bf16 (__builtin_amdgcn_fdot2_f32_bf16).
// memcpy, not __builtin_bit_cast: this hipcc miscompiles a bit_cast of an ext-vector element into
// bf16x2 (in an unrolled loop over a u32x4 every use read element 0)
typedef __bf16 bf16x2_v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ bf16x2_v as_bf16x2(uint32_t w) {
  bf16x2_v r;
  __builtin_memcpy(&r, &w, 4);
  return r;
}

}  // namespace ltx

#define LTX_CHECK_ARG(cond, msg)                                   \
  do {                                                             \
    if (!(cond)) return ::ltx::fail(LTX_ERR_BAD_ARG, (msg));      \
  } while (0)

#define LTX_LAUNCH_CHECK()                                                         \
  do {                                                                             \
    hipError_t e_ = hipGetLastError();                                             \
    if (e_ != hipSuccess) return ::ltx::fail((int)e_, hipGetErrorString(e_));      \
  } while (0)
