// Row-normalisation kernels (HBM-bound): RMSNorm + AdaLN modulate, LayerNorm + modulate, and
// the attention q/k RMSNorm fused with the 3-D RoPE rotation -- forward and backward.
// One wave per row (D <= 2048): each lane keeps its 8-element slices in registers, 16-B loads
// and stores, the row reduction is a 64-lane xor-shuffle. Rounding points mirror the
// reference's eager bf16 op boundaries (see the per-kernel comments).
#include "common.h"
#include "ltx_hip.h"

namespace ltx {

constexpr int ROW_THREADS = 256;  // 4 waves -> 4 rows per block
constexpr int MAXP = 4;           // passes of 512 elements -> D <= 2048

__device__ __forceinline__ void load8(const bf16_t* p, float* v) {
  const u32x4 w = *(const u32x4*)p;
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = bf2f((bf16_t)(w[j >> 1] >> ((j & 1) * 16)));
}
__device__ __forceinline__ void load8f(const float* p, float* v) {
  const f32x4 a = *(const f32x4*)p, b = *(const f32x4*)(p + 4);
#pragma unroll
  for (int j = 0; j < 4; ++j) { v[j] = a[j]; v[4 + j] = b[j]; }
}
// the MAXP 16-B chunks of a row (chunk p at p*512 + 8*lane) issued together: addresses clamped
// into the row so no per-chunk branch separates the loads (hipcc otherwise waits vmcnt(0) on
// each chunk before issuing the next one); chunks past D are ignored by the caller
__device__ __forceinline__ void load_row_raw(const bf16_t* row, int D, int lane, u32x4 (&raw)[MAXP]) {
#pragma unroll
  for (int p = 0; p < MAXP; ++p) raw[p] = *(const u32x4*)(row + min(p * 512 + lane * 8, D - 8));
}
__device__ __forceinline__ void unpack8(const u32x4 w, float* v) {
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = bf2f((bf16_t)(w[j >> 1] >> ((j & 1) * 16)));
}
__device__ __forceinline__ void store8(bf16_t* p, const float* v) {
  u32x4 w;
#pragma unroll
  for (int j = 0; j < 4; ++j) w[j] = pack2(v[2 * j], v[2 * j + 1]);
  *(u32x4*)p = w;
}

// =============================================================================================
// RMSNorm (no affine) + modulate.  diffusers RMSNorm (attention.py:117-119, :161):
//   var = mean(x_f32^2); n = bf16(x * rsqrt(var + eps))
// then attention.py:229-239 / :289-290:  y = bf16(bf16(n * onep) + shift)
// =============================================================================================
__global__ __launch_bounds__(ROW_THREADS) void rmsnorm_mod_fwd_kernel(
    const bf16_t* __restrict__ x, const bf16_t* __restrict__ shift, const bf16_t* __restrict__ onep,
    int64_t ld_mod, bf16_t* __restrict__ y, float* __restrict__ rstd_out, int M, int D, int rows_per_batch,
    float eps) {
  const int lane = threadIdx.x & 63;
  const int m = blockIdx.x * (ROW_THREADS / 64) + (threadIdx.x >> 6);
  if (m >= M) return;
  const bf16_t* xr = x + (int64_t)m * D;
  const int b = m / rows_per_batch;
  // the row and its batch's shift / (1 + scale) chunks go out together (one memory round trip
  // per row; loaded after the reduction, each chunk's pair waited on its own)
  u32x4 raw[MAXP], sraw[MAXP], oraw[MAXP];
  load_row_raw(xr, D, lane, raw);
  load_row_raw(shift + (int64_t)b * ld_mod, D, lane, sraw);
  load_row_raw(onep + (int64_t)b * ld_mod, D, lane, oraw);
  float v[MAXP][8];
  float ss = 0.f;
#pragma unroll
  for (int p = 0; p < MAXP; ++p) {
    unpack8(raw[p], v[p]);
    if (p * 512 + lane * 8 < D) {
#pragma unroll
      for (int j = 0; j < 8; ++j) ss += v[p][j] * v[p][j];
    }
  }
  ss = wave_sum(ss);
  const float r = rsqrtf(ss / (float)D + eps);
  if (lane == 0 && rstd_out) rstd_out[m] = r;
#pragma unroll
  for (int p = 0; p < MAXP; ++p) {
    const int e = p * 512 + lane * 8;
    if (e < D) {
      float s8[8], o8[8], out[8];
      unpack8(sraw[p], s8);
      unpack8(oraw[p], o8);
#pragma unroll
      for (int j = 0; j < 8; ++j) out[j] = rbf(rbf(v[p][j] * r) * o8[j]) + s8[j];
      store8(y + (int64_t)m * D + e, out);
    }
  }
}

// Backward of the above + the residual gradient. Eager autograd roundings:
//   dn  = bf16(dy * onep)                      (MulBackward, bf16)
//   g   = f32(dn)                              (ToCopyBackward)
//   dx1 = bf16(g * r)                          (MulBackward grad for the bf16 x, cast)
//   dr  = sum(g * x); dvar = -0.5 * dr * r^3   (RsqrtBackward)
//   dx2 = bf16((dvar / D) * (2 * x))           (MeanBackward, PowBackward, ToCopyBackward)
//   dx  = bf16(dres + bf16(dx1 + dx2))
// g = bf16(dy * (1 + scale)) and x are bf16-exact, so across the row reduction they are held as
// packed bf16 pairs (32 VGPRs instead of 64: 8 waves per SIMD instead of 5), bitwise the same
__global__ __launch_bounds__(ROW_THREADS) void rmsnorm_mod_bwd_kernel(
    const bf16_t* __restrict__ dy, const bf16_t* __restrict__ x, const float* __restrict__ rstd,
    const bf16_t* __restrict__ onep, int64_t ld_mod, const bf16_t* dres, bf16_t* dx, int M, int D,
    int rows_per_batch, const bf16_t* __restrict__ gate, int64_t ld_gate, bf16_t* __restrict__ gout) {
  const int lane = threadIdx.x & 63;
  const int m = blockIdx.x * (ROW_THREADS / 64) + (threadIdx.x >> 6);
  if (m >= M) return;
  const int b = m / rows_per_batch;
  const bf16_t* op = onep + (int64_t)b * ld_mod;
  const bf16_t* gr = gate ? gate + (int64_t)b * ld_gate : nullptr;
  u32x4 gpk[MAXP], xpk[MAXP];
  float dr = 0.f;
  u32x4 dyr[MAXP], opr[MAXP], rsr[MAXP];
  load_row_raw(dy + (int64_t)m * D, D, lane, dyr);
  load_row_raw(x + (int64_t)m * D, D, lane, xpk);
  load_row_raw(op, D, lane, opr);
  // the residual gradient row and rstd go out with the other loads (after the reduction each
  // chunk had its own round trip)
  if (dres) load_row_raw(dres + (int64_t)m * D, D, lane, rsr);
  const float r = rstd[m];
#pragma unroll
  for (int p = 0; p < MAXP; ++p) {
    const int e = p * 512 + lane * 8;
    if (e < D) {
      float d8[8], o8[8], g8[8];
      unpack8(dyr[p], d8);
      unpack8(opr[p], o8);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        g8[j] = rbf(d8[j] * o8[j]);
        dr += g8[j] * bf2f((bf16_t)(xpk[p][j >> 1] >> ((j & 1) * 16)));
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) gpk[p][j] = pack2(g8[2 * j], g8[2 * j + 1]);
    }
  }
  dr = wave_sum(dr);
  const float dvar = (-0.5f * dr) * (r * r * r);
  const float dmean = dvar / (float)D;
#pragma unroll
  for (int p = 0; p < MAXP; ++p) {
    const int e = p * 512 + lane * 8;
    if (e < D) {
      float res[8], out[8];
      if (dres) unpack8(rsr[p], res);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float gj = bf2f((bf16_t)(gpk[p][j >> 1] >> ((j & 1) * 16)));
        const float xj = bf2f((bf16_t)(xpk[p][j >> 1] >> ((j & 1) * 16)));
        const float dx1 = rbf(gj * r);
        const float dx2 = rbf(dmean * (2.0f * xj));
        const float d = rbf(dx1 + dx2);
        out[j] = dres ? res[j] + d : d;
      }
      store8(dx + (int64_t)m * D + e, out);
      if (gout) {  // the previous block's bf16(dx * gate) from the stored bf16 dx (gate_mul, bitwise)
        const u32x4 gg = *(const u32x4*)(gr + e);
        float g8[8], o2[8];
        unpack8(gg, g8);
#pragma unroll
        for (int j = 0; j < 8; ++j) o2[j] = rbf(out[j]) * g8[j];
        store8(gout + (int64_t)m * D + e, o2);
      }
    }
  }
}

// =============================================================================================
// LayerNorm (no affine, eps 1e-6) + modulate: transformer3d.py:554-560.
//   xhat = bf16((x - mean) * rstd) (ATen layer_norm, f32 statistics); y = bf16(bf16(xhat*onep)+shift)
// =============================================================================================
__global__ __launch_bounds__(ROW_THREADS) void layernorm_mod_fwd_kernel(
    const bf16_t* __restrict__ x, const bf16_t* __restrict__ shift, const bf16_t* __restrict__ onep,
    int64_t ld_mod, bf16_t* __restrict__ y, float* __restrict__ mean_out, float* __restrict__ rstd_out, int M,
    int D, int rows_per_batch, float eps) {
  const int lane = threadIdx.x & 63;
  const int m = blockIdx.x * (ROW_THREADS / 64) + (threadIdx.x >> 6);
  if (m >= M) return;
  float v[MAXP][8];
  float s = 0.f;
#pragma unroll
  for (int p = 0; p < MAXP; ++p) {
    const int e = p * 512 + lane * 8;
    if (e < D) {
      load8(x + (int64_t)m * D + e, v[p]);
#pragma unroll
      for (int j = 0; j < 8; ++j) s += v[p][j];
    }
  }
  const float mean = wave_sum(s) / (float)D;
  float q = 0.f;
#pragma unroll
  for (int p = 0; p < MAXP; ++p) {
    const int e = p * 512 + lane * 8;
    if (e < D) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float d = v[p][j] - mean;
        q += d * d;
      }
    }
  }
  const float r = rsqrtf(wave_sum(q) / (float)D + eps);
  if (lane == 0) {
    mean_out[m] = mean;
    rstd_out[m] = r;
  }
  const int b = m / rows_per_batch;
#pragma unroll
  for (int p = 0; p < MAXP; ++p) {
    const int e = p * 512 + lane * 8;
    if (e < D) {
      float s8[8], o8[8], out[8];
      load8(shift + (int64_t)b * ld_mod + e, s8);
      load8(onep + (int64_t)b * ld_mod + e, o8);
#pragma unroll
      for (int j = 0; j < 8; ++j) out[j] = rbf(rbf((v[p][j] - mean) * r) * o8[j]) + s8[j];
      store8(y + (int64_t)m * D + e, out);
    }
  }
}

// dn = bf16(dy * onep); g = f32(dn); dx = bf16(r * (g - mean(g) - xhat * mean(g * xhat)))
__global__ __launch_bounds__(ROW_THREADS) void layernorm_mod_bwd_kernel(
    const bf16_t* __restrict__ dy, const bf16_t* __restrict__ x, const float* __restrict__ mean_in,
    const float* __restrict__ rstd, const bf16_t* __restrict__ onep, int64_t ld_mod, bf16_t* __restrict__ dx,
    int M, int D, int rows_per_batch) {
  const int lane = threadIdx.x & 63;
  const int m = blockIdx.x * (ROW_THREADS / 64) + (threadIdx.x >> 6);
  if (m >= M) return;
  const int b = m / rows_per_batch;
  const float mean = mean_in[m], r = rstd[m];
  float g[MAXP][8], xh[MAXP][8];
  float sg = 0.f, sgx = 0.f;
#pragma unroll
  for (int p = 0; p < MAXP; ++p) {
    const int e = p * 512 + lane * 8;
    if (e < D) {
      float d8[8], o8[8], x8[8];
      load8(dy + (int64_t)m * D + e, d8);
      load8(onep + (int64_t)b * ld_mod + e, o8);
      load8(x + (int64_t)m * D + e, x8);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        g[p][j] = rbf(d8[j] * o8[j]);
        xh[p][j] = (x8[j] - mean) * r;
        sg += g[p][j];
        sgx += g[p][j] * xh[p][j];
      }
    }
  }
  const float mg = wave_sum(sg) / (float)D;
  const float mgx = wave_sum(sgx) / (float)D;
#pragma unroll
  for (int p = 0; p < MAXP; ++p) {
    const int e = p * 512 + lane * 8;
    if (e < D) {
      float out[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) out[j] = r * (g[p][j] - mg - xh[p][j] * mgx);
      store8(dx + (int64_t)m * D + e, out);
    }
  }
}

// =============================================================================================
// q/k RMSNorm (affine, across all heads) + 3-D RoPE (attention.py:996-1012, 917-932;
// cos/sin: transformer3d.py:221-277).
// =============================================================================================
struct RopeRow {
  float fr[3];  // grid[a] / max_pos[a] * 2 - 1
};

__device__ __forceinline__ RopeRow rope_row(const void* grid, int is_float, int b, int n, int N, float mp0,
                                            float mp1, float mp2) {
  RopeRow rr;
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    const int64_t idx = ((int64_t)b * 3 + a) * N + n;
    const float gv = is_float ? ((const float*)grid)[idx] : (float)((const int64_t*)grid)[idx];
    const float mpa = a == 0 ? mp0 : (a == 1 ? mp1 : mp2);
    rr.fr[a] = (gv / mpa) * 2.0f - 1.0f;
  }
  return rr;
}

// (cos, sin) of element pair starting at even element e, rounded to bf16 like the tables
__device__ __forceinline__ void rope_cs(const RopeRow& rr, const float* __restrict__ omega, int e, int pad,
                                        float& c, float& s) {
  if (e < pad) {
    c = 1.f;
    s = 0.f;
    return;
  }
  const int q = (e - pad) >> 1;
  const int j = q / 3, a = q - 3 * j;
  const float phi = omega[j] * rr.fr[a];
  float sv, cv;
  sincosf(phi, &sv, &cv);
  c = rbf(cv);
  s = rbf(sv);
}

// cos/sin table, one packed u32 (bf16 cos | bf16 sin << 16) per element pair: rows = tokens of
// Bt batches (Bt = 1 when every batch shares its coordinates), D/2 pairs per row. Built once per
// forward and read by all 28 blocks' q/k kernels (fwd and bwd) instead of a sincosf per element.
__global__ __launch_bounds__(256) void rope_table_kernel(const void* grid, int is_float, int N, int D, int64_t total,
                                                         const float* __restrict__ omega, float mp0, float mp1,
                                                         float mp2, uint32_t* __restrict__ cs) {
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= total) return;
  const int half = D / 2;
  const int64_t row = idx / half;
  const int i = (int)(idx - row * half);
  const RopeRow rr = rope_row(grid, is_float, (int)(row / N), (int)(row % N), N, mp0, mp1, mp2);
  float c, s;
  rope_cs(rr, omega, 2 * i, D % 6, c, s);
  cs[idx] = (uint32_t)f2bf(c) | ((uint32_t)f2bf(s) << 16);
}

// the same packed table from the reference's own (cos, sin) pair (precompute_freqs_cis output,
// transformer3d.py:270-277: bf16 [rows, D], each value repeated for the element pair 2i, 2i+1), as
// the Attention.set_processor plug-in receives it
__global__ __launch_bounds__(256) void rope_pack_kernel(const bf16_t* __restrict__ cosv, const bf16_t* __restrict__ sinv,
                                                        int64_t ld, int half, int64_t total, uint32_t* __restrict__ cs) {
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= total) return;
  const int64_t row = idx / half;
  const int64_t e = row * ld + 2 * (idx - row * half);
  cs[idx] = (uint32_t)cosv[e] | ((uint32_t)sinv[e] << 16);
}

__device__ __forceinline__ void cs_unpack(const u32x4 v, float* c, float* s) {
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    c[t] = bf2f((bf16_t)(v[t] & 0xffff));
    s[t] = bf2f((bf16_t)(v[t] >> 16));
  }
}
__device__ __forceinline__ void cs4(const uint32_t* __restrict__ cs, int64_t rowbase, int e, float* c, float* s) {
  cs_unpack(*(const u32x4*)(cs + rowbase + (e >> 1)), c, s);
}
// the packed (cos, sin) words of a row's MAXP chunks (D / 2 words per row), clamped like
// load_row_raw so all chunks go out with the row loads
__device__ __forceinline__ void load_cs_raw(const uint32_t* __restrict__ csr, int D, int lane, u32x4 (&raw)[MAXP]) {
#pragma unroll
  for (int p = 0; p < MAXP; ++p) raw[p] = *(const u32x4*)(csr + (min(p * 512 + lane * 8, D - 8) >> 1));
}

// Grouped q-only launches: rows [g * rows, (g + 1) * rows) are group g, whose input / gradient /
// output rows start g * in / gin / out elements further and whose weight / rstd rows g * w / r
// (ungrouped launches: rows = M, every stride 0)
struct QkGroups {
  int rows;
  int64_t in, gin, out, w, r;
};

// one wave = one (row, q|k) item
__global__ __launch_bounds__(ROW_THREADS) void qk_norm_rope_fwd_kernel(
    const bf16_t* __restrict__ q_in, int64_t ldq_in, const bf16_t* __restrict__ k_in, int64_t ldk_in,
    bf16_t* __restrict__ q_out, int64_t ldq_out, bf16_t* __restrict__ k_out, int64_t ldk_out,
    const bf16_t* __restrict__ qw, const bf16_t* __restrict__ kw, float* __restrict__ rstd_q,
    float* __restrict__ rstd_k, const uint32_t* __restrict__ cs, int64_t cs_batch_rows, int N, int M, int D,
    int rope, int nsel, float eps, QkGroups gq) {
  const int lane = threadIdx.x & 63;
  const int item = blockIdx.x * (ROW_THREADS / 64) + (threadIdx.x >> 6);
  const int m = item / nsel;
  const int which = item - m * nsel;  // 0 = q, 1 = k
  if (m >= M) return;
  // grouped q-only launches (ltx_qk_norm_fwd_grouped): row m is row mr of group g
  const int g = m / gq.rows, mr = m - g * gq.rows;
  const bf16_t* in = which ? k_in + (int64_t)m * ldk_in : q_in + g * gq.in + (int64_t)mr * ldq_in;
  bf16_t* out = which ? k_out + (int64_t)m * ldk_out : q_out + g * gq.out + (int64_t)mr * ldq_out;
  const bf16_t* w = which ? kw : qw + g * gq.w;
  float v[MAXP][8];
  float ss = 0.f;
  // the row, the weight and the RoPE words: one round trip
  const int64_t csrow = ((int64_t)(m / N) * cs_batch_rows + (m % N)) * (D / 2);
  u32x4 wraw[MAXP], csraw[MAXP];
  {
    u32x4 raw[MAXP];
    load_row_raw(in, D, lane, raw);
    load_row_raw(w, D, lane, wraw);
    if (rope) load_cs_raw(cs + csrow, D, lane, csraw);
#pragma unroll
    for (int p = 0; p < MAXP; ++p) {
      unpack8(raw[p], v[p]);
      if (p * 512 + lane * 8 < D) {
#pragma unroll
        for (int j = 0; j < 8; ++j) ss += v[p][j] * v[p][j];
      }
    }
  }
  ss = wave_sum(ss);
  const float r = rsqrtf(ss / (float)D + eps);
  if (lane == 0) {
    if (which) rstd_k[m] = r;
    else rstd_q[g * gq.r + mr] = r;
  }
#pragma unroll
  for (int p = 0; p < MAXP; ++p) {
    const int e = p * 512 + lane * 8;
    if (e < D) {
      float w8[8], nv[8], o[8];
      unpack8(wraw[p], w8);
#pragma unroll
      for (int j = 0; j < 8; ++j) nv[j] = rbf(rbf(v[p][j] * r) * w8[j]);
      if (rope) {
        float c4[4], s4[4];
        cs_unpack(csraw[p], c4, s4);
#pragma unroll
        for (int j = 0; j < 8; j += 2) {
          const float c = c4[j >> 1], s = s4[j >> 1];
          // out = bf16(bf16(x * cos) + bf16(rot(x) * sin)), rot = (-x1, x0)
          o[j] = rbf(nv[j] * c) + rbf(-nv[j + 1] * s);
          o[j + 1] = rbf(nv[j + 1] * c) + rbf(nv[j] * s);
        }
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = nv[j];
      }
      store8(out + e, o);
    }
  }
}

// Backward. g (bf16) -> RoPE^T: dn[2i] = bf16(bf16(g0*c) + bf16(g1*s)), dn[2i+1] =
// bf16(bf16(g1*c) + (-bf16(g0*s))); weight: dxr = bf16(dn * w); then the RMSNorm backward with
// the same roundings as rmsnorm_mod_bwd_kernel.
__global__ __launch_bounds__(ROW_THREADS) void qk_norm_rope_bwd_kernel(
    const void* __restrict__ dq_in, int64_t ldq_in, int dq_f32, const void* __restrict__ dk_in, int64_t ldk_in,
    int dk_f32, const bf16_t* __restrict__ q_raw, int64_t ldq_raw, const bf16_t* __restrict__ k_raw,
    int64_t ldk_raw, const bf16_t* __restrict__ qw, const bf16_t* __restrict__ kw,
    const float* __restrict__ rstd_q, const float* __restrict__ rstd_k, bf16_t* __restrict__ dq_out,
    int64_t ldq_out, bf16_t* __restrict__ dk_out, int64_t ldk_out, const uint32_t* __restrict__ cs,
    int64_t cs_batch_rows, int N, int M, int D, int rope, int nsel, QkGroups gq) {
  const int lane = threadIdx.x & 63;
  const int item = blockIdx.x * (ROW_THREADS / 64) + (threadIdx.x >> 6);
  const int m = item / nsel;
  const int which = item - m * nsel;
  if (m >= M) return;
  // grouped q-only launches (ltx_qk_norm_bwd_grouped): row m is row mr of group g
  const int g = m / gq.rows, mr = m - g * gq.rows;
  const void* gin = which ? dk_in : (const void*)((const bf16_t*)dq_in + g * gq.gin);
  const int64_t ldg = which ? ldk_in : ldq_in;
  const int gf32 = which ? dk_f32 : dq_f32;
  const bf16_t* xin = which ? k_raw + (int64_t)m * ldk_raw : q_raw + g * gq.in + (int64_t)mr * ldq_raw;
  bf16_t* out = which ? dk_out + (int64_t)m * ldk_out : dq_out + g * gq.out + (int64_t)mr * ldq_out;
  const bf16_t* w = which ? kw : qw + g * gq.w;
  const float r = which ? rstd_k[m] : rstd_q[g * gq.r + mr];
  const int64_t csrow = ((int64_t)(m / N) * cs_batch_rows + (m % N)) * (D / 2);
  float gx[MAXP][8], xv[MAXP][8];
  float dr = 0.f;
  // the bf16 gradient row and the input row: all chunks in flight together
  u32x4 graw[MAXP], xraw[MAXP], wraw[MAXP], csraw[MAXP];
  const int mg = which ? m : mr;  // the gradient row inside its group (m when ungrouped)
  if (!gf32) load_row_raw((const bf16_t*)gin + (int64_t)mg * ldg, D, lane, graw);
  load_row_raw(xin, D, lane, xraw);
  load_row_raw(w, D, lane, wraw);
  if (rope) load_cs_raw(cs + csrow, D, lane, csraw);
#pragma unroll
  for (int p = 0; p < MAXP; ++p) {
    const int e = p * 512 + lane * 8;
    if (e < D) {
      float g8[8], w8[8], dn[8];
      if (gf32) {
        load8f((const float*)gin + (int64_t)mg * ldg + e, g8);
#pragma unroll
        for (int j = 0; j < 8; ++j) g8[j] = rbf(g8[j]);
      } else {
        unpack8(graw[p], g8);
      }
      if (rope) {
        float c4[4], s4[4];
        cs_unpack(csraw[p], c4, s4);
#pragma unroll
        for (int j = 0; j < 8; j += 2) {
          const float c = c4[j >> 1], s = s4[j >> 1];
          const float da0 = rbf(g8[j] * c), da1 = rbf(g8[j + 1] * c);
          const float dr0 = rbf(g8[j] * s), dr1 = rbf(g8[j + 1] * s);  // d(rot)
          // rot[2i] = -x[2i+1], rot[2i+1] = x[2i]
          dn[j] = rbf(da0 + dr1);
          dn[j + 1] = rbf(da1 + (-dr0));
        }
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) dn[j] = g8[j];
      }
      unpack8(wraw[p], w8);
      unpack8(xraw[p], xv[p]);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        gx[p][j] = rbf(dn[j] * w8[j]);
        dr += gx[p][j] * xv[p][j];
      }
    }
  }
  dr = wave_sum(dr);
  const float dvar = (-0.5f * dr) * (r * r * r);
  const float dmean = dvar / (float)D;
#pragma unroll
  for (int p = 0; p < MAXP; ++p) {
    const int e = p * 512 + lane * 8;
    if (e < D) {
      float o[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = rbf(gx[p][j] * r) + rbf(dmean * (2.0f * xv[p][j]));
      store8(out + e, o);
    }
  }
}

// Weight gradient of the q/k RMSNorm (train_mode='full'): y = bf16(n) * w with n = x * rstd, so
// dw = sum_rows bf16(dn * bf16(n)) where dn is the gradient at the norm output (the RoPE^T of the
// incoming gradient, same roundings as qk_norm_rope_bwd_kernel). Block (which, split) sums its
// rows for all D columns (8 per thread) into part[(which * S + split) * D + col] (f32).
__global__ __launch_bounds__(256) void qk_norm_wgrad_kernel(
    const void* __restrict__ dq_in, int64_t ldq_in, int dq_f32, const void* __restrict__ dk_in, int64_t ldk_in,
    int dk_f32, const bf16_t* __restrict__ q_raw, int64_t ldq_raw, const bf16_t* __restrict__ k_raw,
    int64_t ldk_raw, const float* __restrict__ rstd_q, const float* __restrict__ rstd_k,
    const uint32_t* __restrict__ cs, int64_t cs_batch_rows, int N, int M, int D, int rope, int S,
    float* __restrict__ part) {
  const int which = blockIdx.y;
  const int split = blockIdx.x;
  const int e = threadIdx.x * 8;
  const int m0 = (int)((int64_t)split * M / S), m1 = (int)((int64_t)(split + 1) * M / S);
  const void* gin = which ? dk_in : dq_in;
  const int64_t ldg = which ? ldk_in : ldq_in;
  const int gf32 = which ? dk_f32 : dq_f32;
  const bf16_t* xr = which ? k_raw : q_raw;
  const int64_t ldx = which ? ldk_raw : ldq_raw;
  const float* rs = which ? rstd_k : rstd_q;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (e < D) {
    for (int m = m0; m < m1; ++m) {
      float g8[8], dn[8], x8[8];
      if (gf32) {
        load8f((const float*)gin + (int64_t)m * ldg + e, g8);
#pragma unroll
        for (int j = 0; j < 8; ++j) g8[j] = rbf(g8[j]);
      } else {
        load8((const bf16_t*)gin + (int64_t)m * ldg + e, g8);
      }
      if (rope) {
        float c4[4], s4[4];
        cs4(cs, ((int64_t)(m / N) * cs_batch_rows + (m % N)) * (D / 2), e, c4, s4);
#pragma unroll
        for (int j = 0; j < 8; j += 2) {
          const float c = c4[j >> 1], s = s4[j >> 1];
          const float da0 = rbf(g8[j] * c), da1 = rbf(g8[j + 1] * c);
          const float dr0 = rbf(g8[j] * s), dr1 = rbf(g8[j + 1] * s);
          dn[j] = rbf(da0 + dr1);
          dn[j + 1] = rbf(da1 + (-dr0));
        }
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) dn[j] = g8[j];
      }
      load8(xr + (int64_t)m * ldx + e, x8);
      const float r = rs[m];
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += rbf(dn[j] * rbf(x8[j] * r));
    }
    float* o = part + ((int64_t)which * S + split) * D + e;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = acc[j];
  }
}

static inline unsigned row_blocks(int64_t items) { return (unsigned)((items + 3) / 4); }

}  // namespace ltx

using namespace ltx;

extern "C" {

int ltx_rmsnorm_modulate_fwd(const void* x, const void* shift, const void* onep, int64_t ld_mod, void* y,
                             float* rstd, int64_t M, int64_t D, int64_t rows_per_batch, float eps, void* stream) {
  LTX_CHECK_ARG(x && shift && onep && y && M > 0 && D > 0, "rmsnorm_modulate_fwd: bad args");
  LTX_CHECK_ARG(D % 8 == 0 && D <= 2048 && ld_mod % 8 == 0, "rmsnorm_modulate_fwd: D must be %8 and <= 2048");
  hipLaunchKernelGGL(rmsnorm_mod_fwd_kernel, dim3(row_blocks(M)), dim3(ROW_THREADS), 0, (hipStream_t)stream,
                     (const bf16_t*)x, (const bf16_t*)shift, (const bf16_t*)onep, ld_mod, (bf16_t*)y, rstd, (int)M,
                     (int)D, (int)(rows_per_batch > 0 ? rows_per_batch : M), eps);
  LTX_LAUNCH_CHECK();
  return LTX_OK;
}

int ltx_rmsnorm_modulate_bwd_gated(const void* dy, const void* x, const float* rstd, const void* onep,
                                   int64_t ld_mod, const void* dres, void* dx, int64_t M, int64_t D,
                                   int64_t rows_per_batch, const void* gate, int64_t ld_gate, void* gout,
                                   void* stream) {
  LTX_CHECK_ARG(dy && x && rstd && onep && dx && M > 0 && D > 0, "rmsnorm_modulate_bwd: bad args");
  LTX_CHECK_ARG(D % 8 == 0 && D <= 2048 && ld_mod % 8 == 0, "rmsnorm_modulate_bwd: D must be %8 and <= 2048");
  LTX_CHECK_ARG(!gout || (gate && ld_gate % 8 == 0 && ((uintptr_t)gate % 16) == 0),
                "rmsnorm_modulate_bwd: gated output needs 16-B aligned gate rows");
  hipLaunchKernelGGL(rmsnorm_mod_bwd_kernel, dim3(row_blocks(M)), dim3(ROW_THREADS), 0, (hipStream_t)stream,
                     (const bf16_t*)dy, (const bf16_t*)x, rstd, (const bf16_t*)onep, ld_mod, (const bf16_t*)dres,
                     (bf16_t*)dx, (int)M, (int)D, (int)(rows_per_batch > 0 ? rows_per_batch : M),
                     (const bf16_t*)gate, ld_gate, (bf16_t*)gout);
  LTX_LAUNCH_CHECK();
  return LTX_OK;
}

int ltx_rmsnorm_modulate_bwd(const void* dy, const void* x, const float* rstd, const void* onep, int64_t ld_mod,
                             const void* dres, void* dx, int64_t M, int64_t D, int64_t rows_per_batch,
                             void* stream) {
  return ltx_rmsnorm_modulate_bwd_gated(dy, x, rstd, onep, ld_mod, dres, dx, M, D, rows_per_batch, nullptr, 0,
                                        nullptr, stream);
}

int ltx_layernorm_modulate_fwd(const void* x, const void* shift, const void* onep, int64_t ld_mod, void* y,
                               float* mean, float* rstd, int64_t M, int64_t D, int64_t rows_per_batch, float eps,
                               void* stream) {
  LTX_CHECK_ARG(x && shift && onep && y && mean && rstd && M > 0, "layernorm_modulate_fwd: bad args");
  LTX_CHECK_ARG(D % 8 == 0 && D <= 2048 && ld_mod % 8 == 0, "layernorm_modulate_fwd: D must be %8 and <= 2048");
  hipLaunchKernelGGL(layernorm_mod_fwd_kernel, dim3(row_blocks(M)), dim3(ROW_THREADS), 0, (hipStream_t)stream,
                     (const bf16_t*)x, (const bf16_t*)shift, (const bf16_t*)onep, ld_mod, (bf16_t*)y, mean, rstd,
                     (int)M, (int)D, (int)(rows_per_batch > 0 ? rows_per_batch : M), eps);
  LTX_LAUNCH_CHECK();
  return LTX_OK;
}

int ltx_layernorm_modulate_bwd(const void* dy, const void* x, const float* mean, const float* rstd,
                               const void* onep, int64_t ld_mod, void* dx, int64_t M, int64_t D,
                               int64_t rows_per_batch, void* stream) {
  LTX_CHECK_ARG(dy && x && mean && rstd && onep && dx && M > 0, "layernorm_modulate_bwd: bad args");
  LTX_CHECK_ARG(D % 8 == 0 && D <= 2048 && ld_mod % 8 == 0, "layernorm_modulate_bwd: D must be %8 and <= 2048");
  hipLaunchKernelGGL(layernorm_mod_bwd_kernel, dim3(row_blocks(M)), dim3(ROW_THREADS), 0, (hipStream_t)stream,
                     (const bf16_t*)dy, (const bf16_t*)x, mean, rstd, (const bf16_t*)onep, ld_mod, (bf16_t*)dx,
                     (int)M, (int)D, (int)(rows_per_batch > 0 ? rows_per_batch : M));
  LTX_LAUNCH_CHECK();
  return LTX_OK;
}

int ltx_rope_pack_bf16(const void* cos, const void* sin, int64_t ld, int64_t rows, int64_t D, uint32_t* cs,
                       void* stream) {
  LTX_CHECK_ARG(cos && sin && cs && rows > 0 && D % 8 == 0 && D <= 2048 && ld >= D, "rope_pack: bad args");
  const int64_t total = rows * (D / 2);
  hipLaunchKernelGGL(rope_pack_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     (const bf16_t*)cos, (const bf16_t*)sin, ld, (int)(D / 2), total, cs);
  LTX_LAUNCH_CHECK();
  return LTX_OK;
}

int ltx_rope_table(const void* indices_grid, int grid_is_float, int64_t B, int64_t N, int64_t D,
                   const float* omega, float max_pos_t, float max_pos_h, float max_pos_w, uint32_t* cs,
                   void* stream) {
  LTX_CHECK_ARG(indices_grid && omega && cs && B > 0 && N > 0, "rope_table: bad args");
  LTX_CHECK_ARG(D % 8 == 0 && D <= 2048, "rope_table: D must be %8 and <= 2048");
  const int64_t total = B * N * (D / 2);
  hipLaunchKernelGGL(rope_table_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     indices_grid, grid_is_float, (int)N, (int)D, total, omega, max_pos_t, max_pos_h, max_pos_w, cs);
  LTX_LAUNCH_CHECK();
  return LTX_OK;
}

int ltx_qk_norm_rope_fwd(const void* q_in, int64_t ldq_in, const void* k_in, int64_t ldk_in, void* q_out,
                         int64_t ldq_out, void* k_out, int64_t ldk_out, const void* q_weight, const void* k_weight,
                         float* rstd_q, float* rstd_k, const uint32_t* rope_cs, int64_t cs_batch_rows, int64_t B,
                         int64_t N, int64_t D, int rope, float eps, void* stream) {
  LTX_CHECK_ARG(q_in && q_out && q_weight && rstd_q && B > 0 && N > 0, "qk_norm_rope_fwd: bad args");
  LTX_CHECK_ARG(D % 8 == 0 && D <= 2048, "qk_norm_rope_fwd: D must be %8 and <= 2048");
  LTX_CHECK_ARG(!rope || (rope_cs && ((uintptr_t)rope_cs % 16) == 0), "qk_norm_rope_fwd: rope needs a 16-B aligned table");
  const bool has_k = k_in != nullptr;
  LTX_CHECK_ARG(!has_k || (k_out && k_weight && rstd_k), "qk_norm_rope_fwd: k needs k_out, k_weight, rstd_k");
  LTX_CHECK_ARG(ldq_in % 8 == 0 && ldq_out % 8 == 0 && (!has_k || (ldk_in % 8 == 0 && ldk_out % 8 == 0)),
                "qk_norm_rope_fwd: leading dims must be %8");
  const int nsel = has_k ? 2 : 1;
  const int64_t M = B * N;
  hipLaunchKernelGGL(qk_norm_rope_fwd_kernel, dim3(row_blocks(M * nsel)), dim3(ROW_THREADS), 0,
                     (hipStream_t)stream, (const bf16_t*)q_in, ldq_in, (const bf16_t*)k_in, ldk_in, (bf16_t*)q_out,
                     ldq_out, (bf16_t*)k_out, ldk_out, (const bf16_t*)q_weight, (const bf16_t*)k_weight, rstd_q,
                     rstd_k, rope_cs, cs_batch_rows, (int)N, (int)M, (int)D, rope, nsel, eps,
                     QkGroups{(int)M, 0, 0, 0, 0, 0});
  LTX_LAUNCH_CHECK();
  return LTX_OK;
}

int ltx_qk_norm_rope_bwd(const void* dq_in, int64_t ldq_in, int dq_is_f32, const void* dk_in, int64_t ldk_in,
                         int dk_is_f32, const void* q_raw, int64_t ldq_raw, const void* k_raw, int64_t ldk_raw,
                         const void* q_weight, const void* k_weight, const float* rstd_q, const float* rstd_k,
                         void* dq_out, int64_t ldq_out, void* dk_out, int64_t ldk_out, const uint32_t* rope_cs,
                         int64_t cs_batch_rows, int64_t B, int64_t N, int64_t D, int rope, void* stream) {
  LTX_CHECK_ARG(dq_in && q_raw && q_weight && rstd_q && dq_out && B > 0 && N > 0, "qk_norm_rope_bwd: bad args");
  LTX_CHECK_ARG(D % 8 == 0 && D <= 2048, "qk_norm_rope_bwd: D must be %8 and <= 2048");
  LTX_CHECK_ARG(!rope || (rope_cs && ((uintptr_t)rope_cs % 16) == 0), "qk_norm_rope_bwd: rope needs a 16-B aligned table");
  const bool has_k = dk_in != nullptr;
  LTX_CHECK_ARG(!has_k || (k_raw && k_weight && rstd_k && dk_out), "qk_norm_rope_bwd: incomplete k operands");
  // 16-B vector loads/stores at m * ld + e: bf16 rows need ld % 8, f32 gradient rows ld % 4
  LTX_CHECK_ARG(ldq_in % (dq_is_f32 ? 4 : 8) == 0 && ldq_raw % 8 == 0 && ldq_out % 8 == 0 &&
                    (!has_k || (ldk_in % (dk_is_f32 ? 4 : 8) == 0 && ldk_raw % 8 == 0 && ldk_out % 8 == 0)),
                "qk_norm_rope_bwd: leading dims must keep 16-B rows (bf16 % 8, f32 % 4)");
  LTX_CHECK_ARG((((uintptr_t)dq_in | (uintptr_t)q_raw | (uintptr_t)dq_out | (uintptr_t)dk_in | (uintptr_t)k_raw |
                  (uintptr_t)dk_out) % 16) == 0, "qk_norm_rope_bwd: operands must be 16-B aligned");
  const int nsel = has_k ? 2 : 1;
  const int64_t M = B * N;
  hipLaunchKernelGGL(qk_norm_rope_bwd_kernel, dim3(row_blocks(M * nsel)), dim3(ROW_THREADS), 0,
                     (hipStream_t)stream, dq_in, ldq_in, dq_is_f32, dk_in, ldk_in, dk_is_f32, (const bf16_t*)q_raw,
                     ldq_raw, (const bf16_t*)k_raw, ldk_raw, (const bf16_t*)q_weight, (const bf16_t*)k_weight,
                     rstd_q, rstd_k, (bf16_t*)dq_out, ldq_out, (bf16_t*)dk_out, ldk_out, rope_cs, cs_batch_rows,
                     (int)N, (int)M, (int)D, rope, nsel, QkGroups{(int)M, 0, 0, 0, 0, 0});
  LTX_LAUNCH_CHECK();
  return LTX_OK;
}

// the text keys' RMSNorm of every block in one launch (the batched text side of LoRA training):
// group g = block g, rows = the text tokens, no RoPE, bf16 in / out
int ltx_qk_norm_fwd_grouped(const void* x, int64_t ldx, int64_t x_gs, void* y, int64_t ldy, int64_t y_gs,
                            const void* weight, int64_t w_gs, float* rstd, int64_t r_gs, int64_t rows,
                            int64_t groups, int64_t D, float eps, void* stream) {
  LTX_CHECK_ARG(x && y && weight && rstd && rows > 0 && groups > 0, "qk_norm_fwd_grouped: bad args");
  LTX_CHECK_ARG(D % 8 == 0 && D <= 2048, "qk_norm_fwd_grouped: D must be %8 and <= 2048");
  LTX_CHECK_ARG(ldx % 8 == 0 && ldy % 8 == 0 && x_gs % 8 == 0 && y_gs % 8 == 0 && w_gs % 8 == 0 &&
                    ((((uintptr_t)x | (uintptr_t)y | (uintptr_t)weight) % 16) == 0),
                "qk_norm_fwd_grouped: 16-B aligned rows and group strides");
  LTX_CHECK_ARG(rows * groups < ((int64_t)1 << 31), "qk_norm_fwd_grouped: too many rows");
  const int64_t M = rows * groups;
  hipLaunchKernelGGL(qk_norm_rope_fwd_kernel, dim3(row_blocks(M)), dim3(ROW_THREADS), 0, (hipStream_t)stream,
                     (const bf16_t*)x, ldx, (const bf16_t*)nullptr, (int64_t)0, (bf16_t*)y, ldy, (bf16_t*)nullptr,
                     (int64_t)0, (const bf16_t*)weight, (const bf16_t*)nullptr, rstd, (float*)nullptr,
                     (const uint32_t*)nullptr, (int64_t)0, (int)rows, (int)M, (int)D, 0, 1, eps,
                     QkGroups{(int)rows, x_gs, 0, y_gs, w_gs, r_gs});
  LTX_LAUNCH_CHECK();
  return LTX_OK;
}

int ltx_qk_norm_bwd_grouped(const void* dy, int64_t lddy, int64_t dy_gs, const void* x, int64_t ldx, int64_t x_gs,
                            const void* weight, int64_t w_gs, const float* rstd, int64_t r_gs, void* dx,
                            int64_t lddx, int64_t dx_gs, int64_t rows, int64_t groups, int64_t D, void* stream) {
  LTX_CHECK_ARG(dy && x && weight && rstd && dx && rows > 0 && groups > 0, "qk_norm_bwd_grouped: bad args");
  LTX_CHECK_ARG(D % 8 == 0 && D <= 2048, "qk_norm_bwd_grouped: D must be %8 and <= 2048");
  LTX_CHECK_ARG(lddy % 8 == 0 && ldx % 8 == 0 && lddx % 8 == 0 && dy_gs % 8 == 0 && x_gs % 8 == 0 &&
                    dx_gs % 8 == 0 && w_gs % 8 == 0 &&
                    ((((uintptr_t)dy | (uintptr_t)x | (uintptr_t)dx | (uintptr_t)weight) % 16) == 0),
                "qk_norm_bwd_grouped: 16-B aligned rows and group strides");
  LTX_CHECK_ARG(rows * groups < ((int64_t)1 << 31), "qk_norm_bwd_grouped: too many rows");
  const int64_t M = rows * groups;
  hipLaunchKernelGGL(qk_norm_rope_bwd_kernel, dim3(row_blocks(M)), dim3(ROW_THREADS), 0, (hipStream_t)stream, dy,
                     lddy, 0, (const void*)nullptr, (int64_t)0, 0, (const bf16_t*)x, ldx, (const bf16_t*)nullptr,
                     (int64_t)0, (const bf16_t*)weight, (const bf16_t*)nullptr, rstd, (const float*)nullptr,
                     (bf16_t*)dx, lddx, (bf16_t*)nullptr, (int64_t)0, (const uint32_t*)nullptr, (int64_t)0,
                     (int)rows, (int)M, (int)D, 0, 1, QkGroups{(int)rows, x_gs, dy_gs, dx_gs, w_gs, r_gs});
  LTX_LAUNCH_CHECK();
  return LTX_OK;
}

int ltx_qk_norm_wgrad(const void* dq_in, int64_t ldq_in, int dq_is_f32, const void* dk_in, int64_t ldk_in,
                      int dk_is_f32, const void* q_raw, int64_t ldq_raw, const void* k_raw, int64_t ldk_raw,
                      const float* rstd_q, const float* rstd_k, const uint32_t* rope_cs, int64_t cs_batch_rows,
                      int64_t B, int64_t N, int64_t D, int rope, int64_t splits, float* partials, void* stream) {
  LTX_CHECK_ARG(dq_in && q_raw && rstd_q && partials && B > 0 && N > 0 && splits > 0, "qk_norm_wgrad: bad args");
  LTX_CHECK_ARG(D % 8 == 0 && D <= 2048, "qk_norm_wgrad: D must be %8 and <= 2048");
  LTX_CHECK_ARG(!rope || (rope_cs && ((uintptr_t)rope_cs % 16) == 0), "qk_norm_wgrad: rope needs a 16-B aligned table");
  const bool has_k = dk_in != nullptr;
  LTX_CHECK_ARG(!has_k || (k_raw && rstd_k), "qk_norm_wgrad: incomplete k operands");
  LTX_CHECK_ARG(ldq_in % (dq_is_f32 ? 4 : 8) == 0 && ldq_raw % 8 == 0 &&
                    (!has_k || (ldk_in % (dk_is_f32 ? 4 : 8) == 0 && ldk_raw % 8 == 0)),
                "qk_norm_wgrad: leading dims must keep 16-B rows (bf16 % 8, f32 % 4)");
  LTX_CHECK_ARG((((uintptr_t)dq_in | (uintptr_t)q_raw | (uintptr_t)dk_in | (uintptr_t)k_raw) % 16) == 0,
                "qk_norm_wgrad: operands must be 16-B aligned");
  hipLaunchKernelGGL(qk_norm_wgrad_kernel, dim3((unsigned)splits, has_k ? 2u : 1u), dim3(256), 0, (hipStream_t)stream,
                     dq_in, ldq_in, dq_is_f32, dk_in, ldk_in, dk_is_f32, (const bf16_t*)q_raw, ldq_raw,
                     (const bf16_t*)k_raw, ldk_raw, rstd_q, rstd_k, rope_cs, cs_batch_rows, (int)N, (int)(B * N),
                     (int)D, rope, (int)splits, partials);
  LTX_LAUNCH_CHECK();
  return LTX_OK;
}

}  // extern "C"
