// Shared pieces of the bf16 GEMM kernels (gemm.hip): parameters, block order,
// fused epilogues.
#pragma once
#include "common.h"
#include "ltx_hip.h"

namespace ltx {

constexpr int BM = 128, BN = 128, BK = 64;
constexpr int GEMM_THREADS = 256;
constexpr int TILE_BYTES = BM * BK * 2;           // 16 KiB per operand tile
constexpr int STAGE_BYTES = 2 * TILE_BYTES;       // A + W
constexpr int C_STRIDE = BN * 2 + 8;              // bf16 C image row stride (bytes), 8-B aligned
constexpr int LDS_BYTES = (2 * STAGE_BYTES > BM * C_STRIDE) ? 2 * STAGE_BYTES : BM * C_STRIDE;

struct GemmParams {
  const bf16_t* A;  // [M, K] activations, row stride lda
  const bf16_t* W;  // [N, K] weights (or W^T for dgrad), row stride ldw
  bf16_t* C;        // [M, N], row stride ldc
  int64_t lda, ldw, ldc;
  int M, N, K;
  const bf16_t* bias;  // [N] or null
  // epilogue auxiliaries (meaning per epilogue, see ltx_hip.h)
  const void* aux0;
  int64_t ld0;
  const void* aux1;
  int64_t ld1;
  const void* aux2;
  int64_t ld2;
  float alpha;
  int rank;
  int rows_per_batch;
  // optional K extension (LoRA fused into the K loop): C += A2[M,K2] . W2[N,K2]^T
  const bf16_t* A2;
  const bf16_t* W2;
  int64_t lda2, ldw2;
  int K2;
  // grouped K extension (ext_gn > 0): output columns [g*ext_gn, (g+1)*ext_gn) read their A2 rows
  // at column offset g*ext_gs -- one launch for many projections that share A but each carry
  // their own LoRA operand (the text K/V projections of all blocks). ext_gn % 256 == 0, so a
  // tile never straddles two groups.
  int ext_gn;
  int64_t ext_gs;
  int dma_batch;  // large-tile kernel: issue a wave's DMA pieces in one asm block (1) or singly (0)
  int epi_batch;  // large-tile kernel: epilogue aux loads of several rows in flight (1) or one (0)
  // split-K (small grids): S partial f32 tiles [S][M][N] in a caller-provided workspace, summed by
  // splitk_epilogue_kernel which then applies bias + the epilogue
  float* ws;
  int splitk;
};

// A2 of the output tile starting at column n0 (grouped K extension, see GemmParams)
__device__ __forceinline__ const bf16_t* ext_a2(const GemmParams& p, int n0) {
  return p.ext_gn > 0 ? p.A2 + (int64_t)(n0 / p.ext_gn) * p.ext_gs : p.A2;
}

__device__ __forceinline__ void glds16(const void* gsrc, void* lds_wave_base) {
  __builtin_amdgcn_global_load_lds(gsrc, LDS_PTR(lds_wave_base), 16, 0, 0);
}

// byte offset of (row, logical 16-B chunk) inside a [128][64] bf16 swizzled tile image
__device__ __forceinline__ int swz(int row, int chunk) { return row * 128 + ((chunk ^ (row & 7)) << 4); }

__device__ __forceinline__ void block_to_tile(int bid, int ntm, int ntn, int& tm, int& tn) {
  const int nwg = ntm * ntn;
  // bijective XCD remap: blocks dealt round-robin over 8 XCDs -> give each XCD a contiguous range
  const int q = nwg / 8, r = nwg % 8, xcd = bid % 8, idx = bid / 8;
  const int wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
  // grouped raster: 8 row-tiles share each W column panel
  const int GROUP = 8;
  const int group = wg / (GROUP * ntn);
  const int first = group * GROUP;
  const int gsize = min(ntm - first, GROUP);
  tm = first + (wg % (GROUP * ntn)) % gsize;
  tn = (wg % (GROUP * ntn)) / gsize;
}

// The aux operands one epilogue row chunk reads (aux0 row m, and the gate row of m's batch for the
// gated residual), loaded ahead of the arithmetic by epi_load so a row pass keeps many loads in
// flight instead of waiting on one per row.
struct EpiAux {
  u32x4 a, g;
  int di = -1;  // STORE_ROWDOT: the delta element this lane stores (>= 0), -2 none, -1 computed per row
};
template <int EPI>
constexpr bool epi_has_aux() {
  return EPI == LTX_EPI_STORE_ROWDOT || EPI == LTX_EPI_GATED_RESIDUAL || EPI == LTX_EPI_GELU_BWD ||
         EPI == LTX_EPI_ACCUM;
}
template <int EPI>
__device__ __forceinline__ void epi_load(const GemmParams& p, int m, int n0, EpiAux& x) {
  if constexpr (epi_has_aux<EPI>()) x.a = *(const u32x4*)((const bf16_t*)p.aux0 + (int64_t)m * p.ld0 + n0);
  if constexpr (EPI == LTX_EPI_GATED_RESIDUAL)
    x.g = *(const u32x4*)((const bf16_t*)p.aux1 + (int64_t)(m / p.rows_per_batch) * p.ld1 + n0);
  if constexpr (EPI == LTX_EPI_ACCUM)
    if (p.aux1) x.g = *(const u32x4*)((const bf16_t*)p.aux1 + (int64_t)(m / p.rows_per_batch) * p.ld1 + n0);
}

// Row-dot of 8 columns (store + delta epilogue): sum of c_j * o_j over bf16 pairs in packed words,
// one v_dot2c_f32_bf16 per pair (each bf16 x bf16 product is exact in f32), the pairs in column
// order; then the head's hd / 8 lanes reduce on DPP lane moves (no LDS round trip per step, as
// __shfl_xor's ds_bpermute had): quad_perm [1,0,3,2] = xor 1, [2,3,0,1] = xor 2, row_half_mirror
// pairs quad 0 with quad 1 of each 8 lanes (= xor 4 once both quads hold their sums). Every
// epilogue site hands a row's 8-column chunks to consecutive lanes, so a head of hd = p.rank (32 /
// 64) columns is hd/8 lanes aligned at a multiple of hd/8 (N % hd == 0, checked at launch). The
// lane at the head's first chunk stores delta[b][h][row].
__device__ __forceinline__ void rowdot8(const GemmParams& p, int m, int n0, const u32x4& c4, const u32x4& o4,
                                        const EpiAux* pre) {
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < 4; ++j)
    s = __builtin_amdgcn_fdot2_f32_bf16(as_bf16x2(c4[j]), as_bf16x2(o4[j]), s, false);
  const int hd = p.rank, lanes = hd >> 3;
  s += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(s), 0xB1, 0xF, 0xF, false));
  s += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(s), 0x4E, 0xF, 0xF, false));
  if (lanes == 8) s += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(s), 0x141, 0xF, 0xF, false));
  if (pre && pre->di != -1) {  // index precomputed by the caller (no integer division per row)
    if (pre->di >= 0) ((float*)p.aux1)[pre->di] = s;
  } else if (((n0 >> 3) & (lanes - 1)) == 0) {
    const int rpb = p.rows_per_batch, H = p.N / hd;
    ((float*)p.aux1)[((int64_t)(m / rpb) * H + n0 / hd) * rpb + m % rpb] = s;
  }
}

template <int EPI, int R>
__device__ __forceinline__ void epilogue_row8(const GemmParams& p, int m, int n0, const bf16_t* cvals,
                                              float* out8, const EpiAux* pre = nullptr) {
  // cvals: 8 bf16 of bf16(acc [+ bias]) for columns n0..n0+7 of row m
  float v[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = bf2f(cvals[j]);
  if constexpr (EPI == LTX_EPI_STORE) {
#pragma unroll
    for (int j = 0; j < 8; ++j) out8[j] = v[j];
  } else if constexpr (EPI == LTX_EPI_STORE_ROWDOT) {
    const u32x4 o4 = pre ? pre->a : *(const u32x4*)((const bf16_t*)p.aux0 + (int64_t)m * p.ld0 + n0);
    u32x4 c4;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      out8[2 * j] = v[2 * j];
      out8[2 * j + 1] = v[2 * j + 1];
      c4[j] = (uint32_t)(uint16_t)cvals[2 * j] | ((uint32_t)(uint16_t)cvals[2 * j + 1] << 16);
    }
    rowdot8(p, m, n0, c4, o4, pre);
  } else if constexpr (EPI == LTX_EPI_GELU) {
    // aux0 (optional, int16 snorm of d / 2, ld0): the backward's factor d = gelu_tanh'(y) at the bf16
    // pre-activation y, from the GELU's own sigmoid (the backward then multiplies: no transcendental)
    if (p.aux0) {
      u32x4 pk;
#pragma unroll
      for (int j = 0; j < 8; j += 2) {
        const f32x2 x = {v[j], v[j + 1]}, x2 = x * x;
        const f32x2 s = sigmoid2u_pk(x, x2);
        const f32x2 g = x * s, d = gelu_tanh_grad_g_pk(x2, s, g);
        out8[j] = g[0];
        out8[j + 1] = g[1];
        pk[j >> 1] = pack_gelu_q(d);
      }
      *(u32x4*)((uint16_t*)p.aux0 + (int64_t)m * p.ld0 + n0) = pk;
    } else {
#pragma unroll
      for (int j = 0; j < 8; j += 2) {
        const f32x2 g = gelu_tanh_pk((f32x2){v[j], v[j + 1]});
        out8[j] = g[0];
        out8[j + 1] = g[1];
      }
    }
  } else if constexpr (EPI == LTX_EPI_GATED_RESIDUAL) {
    // out = R + bf16(gate[b] * y): aux0 = R [M,N] (ld0), aux1 = gate rows (batch stride ld1);
    // aux2 (optional, ld2): store of the pre-gate y (the gate's gradient in train_mode='full')
    if (p.aux2) {
      u32x4 pk;
      pk[0] = (unsigned)cvals[0] | ((unsigned)cvals[1] << 16);
      pk[1] = (unsigned)cvals[2] | ((unsigned)cvals[3] << 16);
      pk[2] = (unsigned)cvals[4] | ((unsigned)cvals[5] << 16);
      pk[3] = (unsigned)cvals[6] | ((unsigned)cvals[7] << 16);
      *(u32x4*)((bf16_t*)p.aux2 + (int64_t)m * p.ld2 + n0) = pk;
    }
    const int b = m / p.rows_per_batch;
    const u32x4 r4 = pre ? pre->a : *(const u32x4*)((const bf16_t*)p.aux0 + (int64_t)m * p.ld0 + n0);
    const u32x4 g4 = pre ? pre->g : *(const u32x4*)((const bf16_t*)p.aux1 + (int64_t)b * p.ld1 + n0);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float r = bf2f((bf16_t)(r4[j >> 1] >> ((j & 1) * 16)));
      const float g = bf2f((bf16_t)(g4[j >> 1] >> ((j & 1) * 16)));
      out8[j] = r + rbf(g * v[j]);
    }
  } else if constexpr (EPI == LTX_EPI_LORA || EPI == LTX_EPI_LORA_RESIDUAL) {
    // peft: y = bf16(bf16(base) + alpha * U[m,:] . Lb[n,:]), U = aux1 f32 [M,rank] (ld1),
    // Lb = aux2 f32 [N,rank] (ld2). LORA_RESIDUAL adds R = aux0 afterwards (bf16 add).
    const float* u = (const float*)p.aux1 + (int64_t)m * p.ld1;
    float ur[R];
#pragma unroll
    for (int r = 0; r < R; ++r) ur[r] = u[r];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float* lb = (const float*)p.aux2 + (int64_t)(n0 + j) * p.ld2;
      float s = 0.f;
#pragma unroll
      for (int r = 0; r < R; ++r) s = fmaf(ur[r], lb[r], s);
      out8[j] = v[j] + s * p.alpha;
    }
    if constexpr (EPI == LTX_EPI_LORA_RESIDUAL) {
      const u32x4 r4 = *(const u32x4*)((const bf16_t*)p.aux0 + (int64_t)m * p.ld0 + n0);
#pragma unroll
      for (int j = 0; j < 8; ++j) out8[j] = bf2f((bf16_t)(r4[j >> 1] >> ((j & 1) * 16))) + rbf(out8[j]);
    }
  } else if constexpr (EPI == LTX_EPI_GELU_BWD) {
    // dF = bf16(bf16(acc) * q * 2 / 32767), q = aux0 (int16, ld0): gelu_tanh'(F) as the LTX_EPI_GELU
    // forward kept it (acc * q is exact in f32)
    const u32x4 f4 = pre ? pre->a : *(const u32x4*)((const uint16_t*)p.aux0 + (int64_t)m * p.ld0 + n0);
#pragma unroll
    for (int j = 0; j < 8; j += 2) {
      out8[j] = (v[j] * gelu_qlo(f4[j >> 1])) * GELU_DQ;
      out8[j + 1] = (v[j + 1] * gelu_qhi(f4[j >> 1])) * GELU_DQ;
    }
  } else if constexpr (EPI == LTX_EPI_ACCUM) {
    // out = R + bf16(acc): R = aux0 (ld0); C may alias R. With aux1 (gate rows of the batch,
    // ld1) and aux2 (ld2) also aux2 = bf16(bf16(out) * gate[m / rows_per_batch]): the backward's
    // gate multiply (ltx_gate_mul_bf16, bitwise) fused into the pass that writes out
    const u32x4 r4 = pre ? pre->a : *(const u32x4*)((const bf16_t*)p.aux0 + (int64_t)m * p.ld0 + n0);
#pragma unroll
    for (int j = 0; j < 8; ++j) out8[j] = bf2f((bf16_t)(r4[j >> 1] >> ((j & 1) * 16))) + v[j];
    if (p.aux1) {
      const u32x4 g4 = pre ? pre->g
                           : *(const u32x4*)((const bf16_t*)p.aux1 + (int64_t)(m / p.rows_per_batch) * p.ld1 + n0);
      u32x4 pk;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float lo = rbf(out8[2 * j]) * bf2f((bf16_t)g4[j]);
        const float hi = rbf(out8[2 * j + 1]) * bf2f((bf16_t)(g4[j] >> 16));
        pk[j] = pack2(lo, hi);
      }
      *(u32x4*)((bf16_t*)p.aux2 + (int64_t)m * p.ld2 + n0) = pk;
    }
  } else if constexpr (EPI == LTX_EPI_LORA_DGRAD_ACCUM) {
    // out = [R +] bf16( bf16(acc) + bf16(alpha * Wd[m,:] . A[:,n]) ), Wd = aux1 f32 [M,rank]
    // (ld1), A = aux2 f32 [rank, N] (ld2 = row stride of A), R = aux0 optional (ld0)
    const float* w = (const float*)p.aux1 + (int64_t)m * p.ld1;
    float wr[R];
#pragma unroll
    for (int r = 0; r < R; ++r) wr[r] = w[r];
    float lo[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) lo[j] = 0.f;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const float* a = (const float*)p.aux2 + (int64_t)r * p.ld2 + n0;
#pragma unroll
      for (int j = 0; j < 8; ++j) lo[j] = fmaf(wr[r], a[j], lo[j]);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) out8[j] = v[j] + rbf(lo[j] * p.alpha);
    if (p.aux0) {
      const u32x4 r4 = *(const u32x4*)((const bf16_t*)p.aux0 + (int64_t)m * p.ld0 + n0);
#pragma unroll
      for (int j = 0; j < 8; ++j) out8[j] = bf2f((bf16_t)(r4[j >> 1] >> ((j & 1) * 16))) + rbf(out8[j]);
    }
  }
}

constexpr int BM2 = 256, BN2 = 256;
constexpr int C_STRIDE2 = BN2 * 2 + 8;  // bf16 C image row stride of the 256-wide tiles


}  // namespace ltx
