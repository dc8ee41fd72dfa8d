// One pass over dY for a token-sized LoRA adapter's backward (peft's f32 lora_B, training.py:50-68):
//   w  = alpha * dY . B        [M, r]  (the input-gradient term, consumed as the dgrad GEMM's
//                                       K-extension after the hi / lo split)
//   dB (+)= alpha * dY^T . u   [N, r]  (u = x . A^T, saved by the forward)
// Until now these were two kernels that each streamed dY from HBM (ltx_lora_rows and
// ltx_lora_wgrad, ~18.5 us each at M = 14336, N = 2048); here one LDS-DMA stream of dY feeds both
// products on the bf16 matrix core, and a small second kernel finishes the sums.
//
// Block = 8 waves over 512 columns x G row groups of 32 rows (grid: N / 512 column splits x
// ceil(M / 32G) row splits). Wave w owns columns c0 = 512 bx + 64 w .. +64 and streams its 32 x 64
// slot of every row group (4 KiB, the attention tiles' chunk swizzle swz<64>) through a private
// 4-slot ring, so no barrier is needed in the loop. Per slot:
//   * w:  [32 rows x 16 j] += slot . (B^T pieces)^T: 12 v_mfma_f32_16x16x32_bf16 (2 row halves x
//         2 k halves x 3 pieces), the B^T pieces (ltx_lora_pieces) in registers for the whole block;
//   * dB: [16 j x 64 cols] += (u pieces)^T . slot: 12 MFMAs (4 column blocks x 3 pieces), the
//         slot read transposed (ds_read_b64_tr_b16, the attention dQ product's k-slot order), u
//         split into exact hi / mid / lo bf16 pieces from an LDS copy of the block's u rows.
// Exact bf16 products summed in f32, as ltx_lora_rows; the sums run in a different order than
// ltx_lora_rows / ltx_lora_wgrad (f32 rounding differences only).
// Partials (deterministic, no atomics): w over the 4 column splits [CS][M][RP], dB over the row
// splits [RS][N][RP]; lora_dy_finish_kernel sums them in a fixed order, applies alpha, writes w,
// its [hi | hi | lo | 0..] split operand, and adds dB into the gradient buffer.
#include <cstdlib>

#include "attention_common.h"
#include "ltx_hip.h"

namespace ltx {

#ifndef LTX_RF_NR
#define LTX_RF_NR 5
#endif
namespace {
constexpr int DY_G = 7;      // row groups of 32 per block (14336 = 64 x 7 x 32)
constexpr int DY_NR = 4;     // ring slots per wave
constexpr int DY_COLS = 512; // columns per block
constexpr int DY_UPAD = DY_G * 32 + 4;  // u^T row length in LDS (floats; +4 spreads the banks)
constexpr int DY_MAXCS = 4;  // column splits a MODE-6 pass sums its u from (N <= 2048)
}  // namespace

// MODE: bit 0 the w product, bit 1 the dB product. MODE 2 is ltx_lora_wgrad's token-sized path
// (dw = alpha . Y^T . u on the bf16 matrix core with u's exact three-piece split, where
// lora_wgrad_kernel runs f32 MFMAs); MODE 1 is ltx_lora_rows' (u = x . A^T from A's pieces).
// Bit 2 (with bit 1, round 6): u is not read but summed from another pass's column-split w partials
// part_u[c][j][m] (c < CSu, in c order) times alpha_u -- bitwise the w lora_dy_finish_kernel writes
// from them -- so the dA pass of an adapter (dA = w^T . x) need not wait for that finish launch.
template <int R, int MODE>
__global__ __launch_bounds__(512) void lora_dy_kernel(const bf16_t* __restrict__ y, int64_t ldy,
                                                      const float* __restrict__ u, int64_t ldu,
                                                      const bf16_t* __restrict__ w3, int64_t ldw,
                                                      float* __restrict__ part_w, float* __restrict__ part_b,
                                                      int M, int N, const float* __restrict__ part_u, int CSu,
                                                      float alpha_u) {
  constexpr int RP = R >= 16 ? R : 16;
  constexpr int JT = RP / 16;
  constexpr int NF = 3 * JT;
  constexpr int RING = 8 * DY_NR * 4096;
  constexpr int UT = RP * DY_UPAD * 4;
  static_assert(R == 8 || R == 16, "rank 8 or 16 (the w partials of rank 32 would not fit the ring)");
  static_assert(8 * DY_G * 32 * (RP + 1) * 4 <= RING, "w partials fit the ring");
  // ONE shared array (the DMA target): the ring, then u^T of the block's rows
  __shared__ __attribute__((aligned(16))) char smem[RING + UT];
  float* ut = (float*)(smem + RING);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int cs = blockIdx.x, rs = blockIdx.y;
  const int c0 = cs * DY_COLS + wave * 64;
  const int mb = rs * DY_G * 32;

  // DMA: piece i of a slot = rows 8i .. 8i+7; lane -> row 8i + (lane >> 3), physical chunk lane & 7
  uint32_t yo[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = 8 * i + (lane >> 3);
    yo[i] = (uint32_t)(row * ldy + (((lane & 7) ^ swz<64>(row)) * 8)) * 2;
  }
  const uint32_t lring = lds_u32(smem + wave * (DY_NR * 4096));
  auto dma = [&](int g) {
    const char* sb = (const char*)(y + (int64_t)(mb + 32 * g) * ldy + c0);  // M % 32 == 0
    const uint32_t l = lring + (g % DY_NR) * 4096;
    unsigned keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %6\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %5\n\t"
        "s_add_u32 m0, m0, 0x400\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %2, %5\n\t"
        "s_add_u32 m0, m0, 0x400\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %3, %5\n\t"
        "s_add_u32 m0, m0, 0x400\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %4, %5\n\ts_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(yo[0]), "v"(yo[1]), "v"(yo[2]), "v"(yo[3]), "s"(sb), "s"(l)
        : "memory", "scc");
  };
  const int ng = min(DY_G, (M - mb + 31) / 32);  // row groups of this block
  // B^T pieces of this wave's 64 columns: [k half][piece x JT] (ltx_lora_rows' fragment layout).
  // Loaded first and retired, then handed to hipcc as asm outputs: its own waits for these loads
  // are counted without the asm DMA, and inside the slot loop they drained the prefetched slots
  // (vmcnt(5) .. vmcnt(0) before every slot's MFMAs)
  s16x8 bp[2][NF];
#pragma unroll
  for (int p = 0; p < 3; ++p)
#pragma unroll
    for (int t = 0; t < JT && (MODE & 1); ++t) {
      const bf16_t* src = w3 + (int64_t)(p * RP + t * 16 + (lane & 15)) * ldw + c0 + (lane >> 4) * 8;
      bp[0][p * JT + t] = *(const s16x8*)src;
      bp[1][p * JT + t] = *(const s16x8*)(src + 32);
    }
  if constexpr ((MODE & 1) != 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int f = 0; f < NF; ++f) asm volatile("" : "+v"(bp[h][f]));
  }
  // the first slots' DMA goes out ahead of the u^T staging loads, so their latencies overlap
  for (int g = 0; g < DY_NR - 1; ++g)
    if (g < ng) dma(g);

  // u^T of rows mb .. mb + 32G (zero past M): all loads in flight before the first LDS write (a
  // rolled loop waited out one load round trip per element, ~2 us per block)
  constexpr int UPT = (DY_G * 32 * RP + 511) / 512;
  float uv[UPT];
  if constexpr ((MODE & 4) != 0) {  // u from the w partials: e -> (j, row), rows fastest (coalesced)
    // every partial load in flight before the first add (CSu <= DY_MAXCS; loads past CSu or past the
    // block's rows read partial 0 / row 0 and are not added); then the sum in c order from 0
    float pv[UPT][DY_MAXCS];
#pragma unroll
    for (int i = 0; i < UPT; ++i) {
      const int e = tid + 512 * i, j = e / (DY_G * 32), rr = e % (DY_G * 32), m = mb + rr;
      const bool ok = e < DY_G * 32 * RP && m < M && j < R;
#pragma unroll
      for (int c = 0; c < DY_MAXCS; ++c)
        pv[i][c] = part_u[((int64_t)(c < CSu ? c : 0) * RP + (ok ? j : 0)) * M + (ok ? m : 0)];
    }
#pragma unroll
    for (int i = 0; i < UPT; ++i) {
      const int e = tid + 512 * i, j = e / (DY_G * 32), rr = e % (DY_G * 32), m = mb + rr;
      float acc = 0.f;
#pragma unroll
      for (int c = 0; c < DY_MAXCS; ++c)
        if (c < CSu) acc += pv[i][c];
      uv[i] = (e < DY_G * 32 * RP && m < M && j < R) ? acc * alpha_u : 0.f;
    }
#pragma unroll
    for (int i = 0; i < UPT; ++i) {
      const int e = tid + 512 * i;
      if (e < DY_G * 32 * RP) ut[(e / (DY_G * 32)) * DY_UPAD + e % (DY_G * 32)] = uv[i];
    }
  } else {
#pragma unroll
    for (int i = 0; i < UPT; ++i) {
      const int e = tid + 512 * i, rr = e / RP, j = e % RP, m = mb + rr;
      uv[i] = ((MODE & 2) && e < DY_G * 32 * RP && m < M && j < R) ? u[(int64_t)m * ldu + j] : 0.f;
    }
#pragma unroll
    for (int i = 0; i < UPT; ++i) {
      const int e = tid + 512 * i;
      if ((MODE & 2) && e < DY_G * 32 * RP) ut[(e % RP) * DY_UPAD + e / RP] = uv[i];
    }
  }
  __syncthreads();  // u^T staged; every ordinary load retired before the counted waits below

  // row reads (w product): rows 16q + (lane & 15), logical chunk 4h + (lane >> 4)
  int roff[2][2];
#pragma unroll
  for (int q = 0; q < 2; ++q)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int row = 16 * q + (lane & 15);
      roff[q][h] = row * 128 + (((4 * h + (lane >> 4)) ^ swz<64>(row)) * 16);
    }
  // transposed reads (dB product): k-slot 8g + jj = row 4g + jj (jj < 4) / 16 + 4g + jj - 4
  const int g4 = lane >> 4, qq = (lane & 15) >> 2, pp = lane & 3;
  int toffs[4];
#pragma unroll
  for (int nb = 0; nb < 4; ++nb) toffs[nb] = toff<64>(4 * g4 + qq, 2 * nb + (pp >> 1)) + 8 * (pp & 1);
  auto tr4 = [](const char* a) {
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)a);
  };

  f32x4 wacc[DY_G][2][JT];
  f32x4 bacc[JT][4];
#pragma unroll
  for (int t = 0; t < JT; ++t)
#pragma unroll
    for (int nb = 0; nb < 4; ++nb) bacc[t][nb] = (f32x4){0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int g = 0; g < DY_G; ++g) {
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
      for (int t = 0; t < JT; ++t) wacc[g][q][t] = (f32x4){0.f, 0.f, 0.f, 0.f};
    if (g >= ng) continue;
    // slot g landed: only the slots issued after it (at most DY_NR - 2) stay in flight
    const int younger = min(DY_NR - 2, ng - 1 - g);
    if (younger >= 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if (younger == 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const char* sl = smem + wave * (DY_NR * 4096) + (g % DY_NR) * 4096;
    s16x8 xf[2][2];
#pragma unroll
    for (int q = 0; q < 2 && (MODE & 1); ++q)
#pragma unroll
      for (int h = 0; h < 2; ++h) xf[q][h] = *(const s16x8*)(sl + roff[q][h]);
    s16x8 yb[4];
#pragma unroll
    for (int nb = 0; nb < 4 && (MODE & 2); ++nb) {
      const s16x4 b0 = tr4(sl + toffs[nb]), b1 = tr4(sl + toffs[nb] + 16 * 128);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        yb[nb][j] = b0[j];
        yb[nb][4 + j] = b1[j];
      }
    }
    // u pieces of this group's rows in the k-slot order: [piece][t]
    s16x8 up[3][JT];
#pragma unroll
    for (int t = 0; t < JT && (MODE & 2); ++t) {
      const float* ur = ut + (16 * t + (lane & 15)) * DY_UPAD + 32 * g + 4 * g4;
      const f32x4 lo4 = *(const f32x4*)ur, hi4 = *(const f32x4*)(ur + 16);
#pragma unroll
      for (int jj = 0; jj < 8; ++jj) {
        const float v = jj < 4 ? lo4[jj] : hi4[jj - 4];
        const bf16_t a = f2bf(v);
        const float r1 = v - bf2f(a);
        const bf16_t b = f2bf(r1);
        const bf16_t c = f2bf(r1 - bf2f(b));
        up[0][t][jj] = (short)a;
        up[1][t][jj] = (short)b;
        up[2][t][jj] = (short)c;
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // slot g read: its ring slot may be refilled
    if (g + DY_NR - 1 < ng) dma(g + DY_NR - 1);
#pragma unroll
    for (int h = 0; h < 2 && (MODE & 1); ++h)
#pragma unroll
      for (int p = 0; p < 3; ++p)
#pragma unroll
        for (int t = 0; t < JT; ++t)
#pragma unroll
          for (int q = 0; q < 2; ++q)
            wacc[g][q][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xf[q][h], bp[h][p * JT + t], wacc[g][q][t], 0, 0, 0);
#pragma unroll
    for (int p = 0; p < 3 && (MODE & 2); ++p)
#pragma unroll
      for (int t = 0; t < JT; ++t)
#pragma unroll
        for (int nb = 0; nb < 4; ++nb)
          bacc[t][nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(up[p][t], yb[nb], bacc[t][nb], 0, 0, 0);
  }
  // dB partial: C[j][n] -> part_b[rs][n][j], lane: n = c0 + 16 nb + (lane & 15), j = 16t + 4 g4 + 0..3
#pragma unroll
  for (int t = 0; t < JT && (MODE & 2); ++t)
#pragma unroll
    for (int nb = 0; nb < 4; ++nb) {
      const int n = c0 + 16 * nb + (lane & 15);
      *(f32x4*)(part_b + ((int64_t)rs * N + n) * RP + 16 * t + 4 * g4) = bacc[t][nb];
    }
  if constexpr (!(MODE & 1)) return;
  // w partial: the 8 waves' [j][32G rows] sums through LDS (the ring is free once all waves are
  // past their last slot; a C fragment's 4 values are 4 consecutive rows of one j: one 16-B write),
  // then one column-split partial part_w[cs][j][m] per row quad (16-B reads and stores)
  __syncthreads();
  constexpr int WROW = DY_G * 32 + 4;  // floats per (wave, j) row; +4 spreads the banks
  float* part = (float*)smem;
  static_assert(8 * RP * WROW * 4 <= RING, "w partials fit the ring");
#pragma unroll
  for (int g = 0; g < DY_G; ++g)
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
      for (int t = 0; t < JT; ++t)
        *(f32x4*)(part + (wave * RP + 16 * t + (lane & 15)) * WROW + 32 * g + 16 * q + 4 * g4) = wacc[g][q][t];
  __syncthreads();
  for (int e = tid; e < RP * DY_G * 8; e += 512) {  // (j, row quad)
    const int j = e / (DY_G * 8), r4 = 4 * (e % (DY_G * 8));
    if (mb + r4 >= M) continue;  // M % 32 == 0: a quad is all in or all out
    f32x4 sum = *(const f32x4*)(part + j * WROW + r4);
#pragma unroll
    for (int w = 1; w < 8; ++w) {
      const f32x4 v = *(const f32x4*)(part + (w * RP + j) * WROW + r4);
      sum[0] += v[0]; sum[1] += v[1]; sum[2] += v[2]; sum[3] += v[3];
    }
    *(f32x4*)(part_w + ((int64_t)cs * RP + j) * M + mb + r4) = sum;
  }
}

// Blocks [0, nwb): w[m,j] = alpha * sum_c part_w[c][m][j] and the [hi | hi | lo | 0..] split row,
// one thread per split element. Blocks [nwb, ..): dw[n*on + j*oj] (+)= alpha * sum_s part_b[s][n][j]
// for 64 (n, j) pairs per block, the row splits dealt to 4 thread groups (strided, independent
// loads in flight) and the 4 group sums added in a fixed order (deterministic).
// Blocks [nwb + nbb, ..) (round 6): a second row-split sum of the same kind, dwa (+)= alpha_a *
// sum_s part_a[s][n][j] over Na columns (the adapter's dA from the pass that ran after its dY pass).
template <int R>
__device__ __forceinline__ void finish_rows(const float* __restrict__ part, int RS, int N, float alpha,
                                            float* __restrict__ dw, int64_t on, int64_t oj, int accumulate, int blk,
                                            float (*red)[64]) {
  constexpr int RP = R >= 16 ? R : 16;
  const int pr = threadIdx.x & 63, grp = threadIdx.x >> 6;
  const int64_t e = (int64_t)blk * 64 + pr;  // pair (n, j), j fastest
  const bool ok = e < (int64_t)N * R;
  const int n = ok ? (int)(e / R) : 0, j = ok ? (int)(e % R) : 0;
  float sum = 0.f;
#pragma unroll 8
  for (int s = grp; s < RS; s += 4) sum += part[((int64_t)s * N + n) * RP + j];
  red[grp][pr] = sum;
  __syncthreads();
  if (grp == 0 && ok) {
    const float v = (((red[0][pr] + red[1][pr]) + red[2][pr]) + red[3][pr]) * alpha;
    float* o = dw + (int64_t)n * on + (int64_t)j * oj;
    *o = accumulate ? *o + v : v;
  }
}

template <int R>
__global__ __launch_bounds__(256) void lora_dy_finish_kernel(const float* __restrict__ part_w, int CS,
                                                             const float* __restrict__ part_b, int RS, int M, int N,
                                                             float alpha, float* __restrict__ w, int64_t ldw_out,
                                                             bf16_t* __restrict__ split, int64_t lds, int K2,
                                                             float* __restrict__ dw, int64_t on, int64_t oj,
                                                             int accumulate, int nwb, int nbb,
                                                             const float* __restrict__ part_a, int Na, float alpha_a,
                                                             float* __restrict__ dwa, int64_t ona, int64_t oja,
                                                             int acc_a) {
  constexpr int RP = R >= 16 ? R : 16;
  if ((int)blockIdx.x < nwb) {
    // thread (j quad q, row m), m fastest (the partial reads coalesce): w[m][4q..4q+3],
    // split[m][4q..] = split[m][R + 4q..] = hi, split[m][2R + 4q..] = lo, and the zero padding
    // columns 3R + 4q + kR < K2 (the R / 4 quads of a row cover 3R .. K2 between them)
    constexpr int NQ = R / 4;
    const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (e >= (int64_t)M * NQ) return;
    const int q = (int)(e / M), m = (int)(e % M);
    float v[4] = {0.f, 0.f, 0.f, 0.f};
    int c = 0;
    for (; c + 4 <= CS; c += 4) {  // 16 loads in flight, summed in split order
      float t[4][4];
#pragma unroll
      for (int cc = 0; cc < 4; ++cc)
#pragma unroll
        for (int k = 0; k < 4; ++k) t[cc][k] = part_w[((int64_t)(c + cc) * RP + 4 * q + k) * M + m];
#pragma unroll
      for (int cc = 0; cc < 4; ++cc)
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] += t[cc][k];
    }
    for (; c < CS; ++c)
#pragma unroll
      for (int k = 0; k < 4; ++k) v[k] += part_w[((int64_t)c * RP + 4 * q + k) * M + m];
    f32x4 wv;
    uint32_t hi[2], lo[2];
#pragma unroll
    for (int k = 0; k < 4; ++k) wv[k] = v[k] * alpha;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const bf16_t h0 = f2bf(wv[2 * k]), h1 = f2bf(wv[2 * k + 1]);
      hi[k] = (uint32_t)h0 | ((uint32_t)h1 << 16);
      lo[k] = (uint32_t)f2bf(wv[2 * k] - bf2f(h0)) | ((uint32_t)f2bf(wv[2 * k + 1] - bf2f(h1)) << 16);
    }
    *(f32x4*)(w + (int64_t)m * ldw_out + 4 * q) = wv;
    if (split == nullptr) return;
    bf16_t* sr = split + (int64_t)m * lds;
    *(u32x2*)(sr + 4 * q) = (u32x2){hi[0], hi[1]};
    *(u32x2*)(sr + R + 4 * q) = (u32x2){hi[0], hi[1]};
    *(u32x2*)(sr + 2 * R + 4 * q) = (u32x2){lo[0], lo[1]};
    for (int c = 3 * R + 4 * q; c < K2; c += R) *(u32x2*)(sr + c) = (u32x2){0u, 0u};
    return;
  }
  __shared__ float red[4][64];
  const int blk = (int)blockIdx.x - nwb;
  if (blk < nbb) finish_rows<R>(part_b, RS, N, alpha, dw, on, oj, accumulate, blk, red);
  else finish_rows<R>(part_a, RS, Na, alpha_a, dwa, ona, oja, acc_a, blk - nbb, red);
}

// u = alpha * x . A^T for token-sized M with the whole contraction inside one block (round 6):
// block = 8 waves on RG row groups of 32 rows, wave w owns the K / 8 = 64 CH contiguous columns
// from 64 CH w, so the block's rows are complete after its cross-wave sum and u and the split
// operand leave the kernel directly (the column-split MODE 1 pass needed lora_dy_finish_kernel
// for the 4 column partials: one more launch and 3.7 MB of partials per call). The wave's A^T
// pieces (3 x 16 j x 64 CH columns) stay in registers for its RG x CH slots, which stream through
// the same private 4-slot LDS-DMA ring as lora_dy_kernel (slot = 32 rows x 64 columns, order
// (group, chunk)). Same exact bf16 products summed in f32; the sum order is per-slot MFMA
// accumulation, then the 8 wave partials in wave order.
template <int R, int RG, int CH, int NR>
__global__ __launch_bounds__(512) void lora_rows_full_kernel(const bf16_t* __restrict__ x, int64_t ldx,
                                                             const bf16_t* __restrict__ w3, int64_t ldw,
                                                             float* __restrict__ out, int64_t ldo, int M, float alpha,
                                                             bf16_t* __restrict__ split, int64_t lds, int K2) {
  constexpr int RP = R >= 16 ? R : 16;
  constexpr int JT = RP / 16;
  constexpr int NF = 3 * JT;
  constexpr int NS = RG * CH;  // slots per wave
  constexpr int RING = 8 * NR * 4096;
  constexpr int PROW = RG * 32 + 4;  // floats per (wave, j) partial row; +4 spreads the banks
  static_assert(R == 8 || R == 16, "rank 8 or 16");
  static_assert(8 * RP * PROW * 4 <= RING, "wave partials fit the ring");
  __shared__ __attribute__((aligned(16))) char smem[RING];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int c0 = wave * 64 * CH;
  const int mb = blockIdx.x * RG * 32;
  const int ng = min(RG, (M - mb) / 32);  // M % 32 == 0
  const int ns = ng * CH;

  uint32_t yo[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = 8 * i + (lane >> 3);
    yo[i] = (uint32_t)(row * ldx + (((lane & 7) ^ swz<64>(row)) * 8)) * 2;
  }
  const uint32_t lring = lds_u32(smem + wave * (NR * 4096));
  auto dma = [&](int s) {  // slot s = (group s / CH, chunk s % CH)
    const char* sb = (const char*)(x + (int64_t)(mb + 32 * (s / CH)) * ldx + c0 + 64 * (s % CH));
    const uint32_t l = lring + (s % NR) * 4096;
    unsigned keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %6\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %5\n\t"
        "s_add_u32 m0, m0, 0x400\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %2, %5\n\t"
        "s_add_u32 m0, m0, 0x400\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %3, %5\n\t"
        "s_add_u32 m0, m0, 0x400\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %4, %5\n\ts_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(yo[0]), "v"(yo[1]), "v"(yo[2]), "v"(yo[3]), "s"(sb), "s"(l)
        : "memory", "scc");
  };
  // the ring's first slots go out first; the pieces' loads overlap them, then everything retires
  // (hipcc's own waits for the pieces are counted without the asm DMA)
  for (int s = 0; s < NR - 1; ++s)
    if (s < ns) dma(s);
  s16x8 bp[CH][2][NF];
#pragma unroll
  for (int c = 0; c < CH; ++c)
#pragma unroll
    for (int p = 0; p < 3; ++p)
#pragma unroll
      for (int t = 0; t < JT; ++t) {
        const bf16_t* src = w3 + (int64_t)(p * RP + t * 16 + (lane & 15)) * ldw + c0 + 64 * c + (lane >> 4) * 8;
        bp[c][0][p * JT + t] = *(const s16x8*)src;
        bp[c][1][p * JT + t] = *(const s16x8*)(src + 32);
      }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
  for (int c = 0; c < CH; ++c)
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int f = 0; f < NF; ++f) asm volatile("" : "+v"(bp[c][h][f]));

  int roff[2][2];
#pragma unroll
  for (int q = 0; q < 2; ++q)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int row = 16 * q + (lane & 15);
      roff[q][h] = row * 128 + (((4 * h + (lane >> 4)) ^ swz<64>(row)) * 16);
    }
  f32x4 acc[RG][2][JT];
#pragma unroll
  for (int g = 0; g < RG; ++g)
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
      for (int t = 0; t < JT; ++t) acc[g][q][t] = (f32x4){0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int s = 0; s < NS; ++s) {
    if (s >= ns) break;
    const int g = s / CH, c = s % CH;
    const int younger = min(NR - 2, ns - 1 - s);  // slots issued after s
    if (younger >= 3) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
    else if (younger == 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if (younger == 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const char* sl = smem + wave * (NR * 4096) + (s % NR) * 4096;
    s16x8 xf[2][2];
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
      for (int h = 0; h < 2; ++h) xf[q][h] = *(const s16x8*)(sl + roff[q][h]);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // slot s read: its ring slot may be refilled
    if (s + NR - 1 < ns) dma(s + NR - 1);
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int p = 0; p < 3; ++p)
#pragma unroll
        for (int t = 0; t < JT; ++t)
#pragma unroll
          for (int q = 0; q < 2; ++q)
            acc[g][q][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xf[q][h], bp[c][h][p * JT + t], acc[g][q][t], 0, 0, 0);
  }
  // the 8 wave partials [j][rows] through LDS (the ring is free once every wave is past its last
  // slot), then thread (row m, j quad q) sums them in wave order and writes u[m][4q..] and the
  // [hi | hi | lo | 0..] split row (as lora_dy_finish_kernel)
  __syncthreads();
  float* part = (float*)smem;
#pragma unroll
  for (int g = 0; g < RG; ++g)
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
      for (int t = 0; t < JT; ++t)
        *(f32x4*)(part + (wave * RP + 16 * t + (lane & 15)) * PROW + 32 * g + 16 * q + 4 * (lane >> 4)) = acc[g][q][t];
  __syncthreads();
  constexpr int NQ = R / 4;
  for (int e = tid; e < RG * 32 * NQ; e += 512) {
    const int q = e / (RG * 32), rr = e % (RG * 32), m = mb + rr;
    if (m >= M) continue;
    f32x4 wv;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float v = part[(4 * q + k) * PROW + rr];
#pragma unroll
      for (int w = 1; w < 8; ++w) v += part[(w * RP + 4 * q + k) * PROW + rr];
      wv[k] = v * alpha;
    }
    *(f32x4*)(out + (int64_t)m * ldo + 4 * q) = wv;
    if (split == nullptr) continue;
    uint32_t hi[2], lo[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const bf16_t h0 = f2bf(wv[2 * k]), h1 = f2bf(wv[2 * k + 1]);
      hi[k] = (uint32_t)h0 | ((uint32_t)h1 << 16);
      lo[k] = (uint32_t)f2bf(wv[2 * k] - bf2f(h0)) | ((uint32_t)f2bf(wv[2 * k + 1] - bf2f(h1)) << 16);
    }
    bf16_t* sr = split + (int64_t)m * lds;
    *(u32x2*)(sr + 4 * q) = (u32x2){hi[0], hi[1]};
    *(u32x2*)(sr + R + 4 * q) = (u32x2){hi[0], hi[1]};
    *(u32x2*)(sr + 2 * R + 4 * q) = (u32x2){lo[0], lo[1]};
    for (int cc = 3 * R + 4 * q; cc < K2; cc += R) *(u32x2*)(sr + cc) = (u32x2){0u, 0u};
  }
}

// ltx_lora_wgrad's token-sized path (called from lora.hip): dw (+)= alpha . Y^T . u through the
// dB product of lora_dy_kernel (bf16 matrix core, u split into exact hi / mid / lo pieces) and the
// dB half of the finish kernel. lora_wgrad_kernel spends ~9 us of f32 MFMA issue on the same
// product at M = 14336, N = 2048, r = 16. Returns false (nothing launched) where it does not apply;
// LTX_LORA_WGRAD_ROWS=0 at load keeps lora_wgrad_kernel everywhere.
bool lora_wgrad_rows(const bf16_t* y, int64_t ldy, const float* u, int64_t ldu, float* dw, int64_t on, int64_t oj,
                     int64_t M, int64_t N, int64_t r, float alpha, int accumulate, hipStream_t s) {
  static const int enabled = [] {
    const char* e = getenv("LTX_LORA_WGRAD_ROWS");
    return e ? atoi(e) : 1;
  }();
  if (!enabled || M < 2048 || M % 32 != 0 || N % DY_COLS != 0 || (r != 8 && r != 16)) return false;
  if (ldy % 8 != 0 || ((uintptr_t)y % 16) != 0 || ldy * 2 * 32 >= ((int64_t)1 << 32) || ldu < r) return false;
  const int64_t RP = r >= 16 ? r : 16;
  const int RS = (int)((M + DY_G * 32 - 1) / (DY_G * 32));
  size_t ws = 0;
  float* pb = stream_workspace(s, &ws);
  if (pb == nullptr || (size_t)RS * N * RP * sizeof(float) > ws) return false;
  const dim3 grid((unsigned)(N / DY_COLS), (unsigned)RS);
  const dim3 g2((unsigned)((N * r + 63) / 64));
#define LTX_LORA_WG(RR)                                                                                       \
  hipLaunchKernelGGL((lora_dy_kernel<RR, 2>), grid, dim3(512), 0, s, y, ldy, u, ldu, nullptr, (int64_t)0, \
                     nullptr, pb, (int)M, (int)N, (const float*)nullptr, 0, 1.f);                           \
  hipLaunchKernelGGL((lora_dy_finish_kernel<RR>), g2, dim3(256), 0, s, nullptr, 0, pb, RS, (int)M, (int)N,    \
                     alpha, nullptr, (int64_t)0, nullptr, (int64_t)0, 0, dw, on, oj, accumulate, 0, 1 << 30,   \
                     (const float*)nullptr, 0, 1.f, (float*)nullptr, (int64_t)0, (int64_t)0, 0);
  if (r == 8) {
    LTX_LORA_WG(8)
  } else {
    LTX_LORA_WG(16)
  }
#undef LTX_LORA_WG
  return true;
}

// ltx_lora_rows' token-sized path (called from lora.hip): out = alpha . x . A^T (and its split
// operand) through the w product of lora_dy_kernel (MODE 1: eight waves x 64 columns per block,
// column-split partials in the stream's workspace) and the w half of the finish kernel. Returns
// false (nothing launched) where it does not apply; LTX_LORA_ROWS_DY=0 at load keeps
// lora_rows_kernel.
bool lora_rows_dy(const bf16_t* x, int64_t ldx, const bf16_t* w3, int64_t ldw, float* out, int64_t ldo, int64_t M,
                  int64_t K, int64_t r, float alpha, bf16_t* split, int64_t ld_split, int64_t K2, hipStream_t s) {
  static const int enabled = [] {
    const char* e = getenv("LTX_LORA_ROWS_DY");
    return e ? atoi(e) : 1;
  }();
  if (!enabled || M < 2048 || M % 32 != 0 || K % DY_COLS != 0 || (r != 8 && r != 16)) return false;
  if (ldx % 8 != 0 || ((uintptr_t)x % 16) != 0 || ldx * 2 * 32 >= ((int64_t)1 << 32)) return false;
  if (ldw % 8 != 0 || ((uintptr_t)w3 % 16) != 0 || ldw < K) return false;
  if (ldo % 4 != 0 || ((uintptr_t)out % 16) != 0) return false;
  if (split && (ld_split % 4 != 0 || ((uintptr_t)split % 8) != 0 || K2 < 3 * r || (K2 - 3 * r) % 4 != 0)) return false;
  // K = 512 / 1024 / 2048: the whole contraction per block (lora_rows_full_kernel, no finish);
  // LTX_LORA_ROWS_FULL=0 at load keeps the column-split pass + finish
  static const int full = [] {
    const char* e = getenv("LTX_LORA_ROWS_FULL");
    return e ? atoi(e) : 1;
  }();
  if (full && (K == 512 || K == 1024 || K == 2048)) {
    constexpr int RG = 2, NRF = LTX_RF_NR;
    const dim3 gf((unsigned)((M + RG * 32 - 1) / (RG * 32)));
#define LTX_LORA_RF(RR, CHH)                                                                                  \
  hipLaunchKernelGGL((lora_rows_full_kernel<RR, RG, CHH, NRF>), gf, dim3(512), 0, s, x, ldx, w3, ldw, out, ldo, (int)M, \
                     alpha, split, ld_split, (int)K2)
    const int ch = (int)(K / 512);
    if (r == 8) {
      if (ch == 1) LTX_LORA_RF(8, 1); else if (ch == 2) LTX_LORA_RF(8, 2); else LTX_LORA_RF(8, 4);
    } else {
      if (ch == 1) LTX_LORA_RF(16, 1); else if (ch == 2) LTX_LORA_RF(16, 2); else LTX_LORA_RF(16, 4);
    }
#undef LTX_LORA_RF
    return true;
  }
  const int64_t RP = r >= 16 ? r : 16;
  const int CS = (int)(K / DY_COLS), RS = (int)((M + DY_G * 32 - 1) / (DY_G * 32));
  size_t ws = 0;
  float* pw = stream_workspace(s, &ws);
  if (pw == nullptr || (size_t)CS * M * RP * sizeof(float) > ws) return false;
  const dim3 grid((unsigned)CS, (unsigned)RS);
  const dim3 g2((unsigned)((M * (r / 4) + 255) / 256));
  const int nwb = (int)g2.x;
#define LTX_LORA_RW(RR)                                                                                      \
  hipLaunchKernelGGL((lora_dy_kernel<RR, 1>), grid, dim3(512), 0, s, x, ldx, nullptr, (int64_t)0, w3, ldw, pw, \
                     nullptr, (int)M, (int)K, (const float*)nullptr, 0, 1.f);                             \
  hipLaunchKernelGGL((lora_dy_finish_kernel<RR>), g2, dim3(256), 0, s, pw, CS, nullptr, 0, (int)M, (int)K,    \
                     alpha, out, ldo, split, ld_split, (int)K2, nullptr, (int64_t)0, (int64_t)0, 0, nwb, 1 << 30, \
                     (const float*)nullptr, 0, 1.f, (float*)nullptr, (int64_t)0, (int64_t)0, 0);
  if (r == 8) {
    LTX_LORA_RW(8)
  } else {
    LTX_LORA_RW(16)
  }
#undef LTX_LORA_RW
  return true;
}

extern "C" int ltx_lora_dy_workspace(int64_t M, int64_t N, int64_t r, int64_t* floats) {
  LTX_CHECK_ARG(floats && M > 0 && N > 0 && (r == 8 || r == 16), "lora_dy_workspace: bad args");
  const int64_t RP = r >= 16 ? r : 16;
  const int64_t CS = N / DY_COLS, RS = (M + DY_G * 32 - 1) / (DY_G * 32);
  *floats = CS * M * RP + RS * N * RP;
  return LTX_OK;
}

extern "C" int ltx_lora_dy(const void* y, int64_t ldy, const float* u, int64_t ldu, const void* w3, int64_t ldw3,
                           int64_t M, int64_t N, int64_t r, float alpha, float* w, int64_t ldw_out, void* split,
                           int64_t ld_split, int64_t K2, float* dw, int64_t on, int64_t oj, int accumulate,
                           float* workspace, void* stream) {
  LTX_CHECK_ARG(y && u && w3 && w && split && dw && workspace, "lora_dy: null operand");
  LTX_CHECK_ARG(M >= 32 && M % 32 == 0 && N % DY_COLS == 0 && (r == 8 || r == 16),
                "lora_dy: M % 32 == 0, N % 512 == 0, rank 8 or 16");
  LTX_CHECK_ARG(ldy % 8 == 0 && ((uintptr_t)y % 16) == 0 && ldw3 % 8 == 0 && ((uintptr_t)w3 % 16) == 0 && ldw3 >= N,
                "lora_dy: 16-B aligned rows of dY and of the pieces");
  LTX_CHECK_ARG(ldy * 2 * 32 < ((int64_t)1 << 32), "lora_dy: 32-bit DMA offsets");
  LTX_CHECK_ARG(ldw_out >= r && ldu >= r && K2 >= 3 * r && K2 % 64 == 0 && ld_split >= K2, "lora_dy: output strides");
  LTX_CHECK_ARG(ldw_out % 4 == 0 && ((uintptr_t)w % 16) == 0 && ld_split % 4 == 0 && ((uintptr_t)split % 8) == 0,
                "lora_dy: 16-B aligned w rows, 8-B aligned split rows");
  LTX_CHECK_ARG((on == r && oj == 1) || (on == 1 && oj == N), "lora_dy: dB must be a dense [N,r] or [r,N]");
  const int64_t RP = r >= 16 ? r : 16;
  const int CS = (int)(N / DY_COLS), RS = (int)((M + DY_G * 32 - 1) / (DY_G * 32));
  float* pw = workspace;
  float* pb = workspace + (int64_t)CS * M * RP;
  hipStream_t s = (hipStream_t)stream;
  const dim3 grid((unsigned)CS, (unsigned)RS);
  const int nwb = (int)((M * (r / 4) + 255) / 256);
  const dim3 g2((unsigned)(nwb + (N * r + 63) / 64));
#define LTX_LORA_DY(RR)                                                                                          \
  hipLaunchKernelGGL((lora_dy_kernel<RR, 3>), grid, dim3(512), 0, s, (const bf16_t*)y, ldy, u, ldu,                \
                     (const bf16_t*)w3, ldw3, pw, pb, (int)M, (int)N, (const float*)nullptr, 0, 1.f);          \
  LTX_LAUNCH_CHECK();                                                                                            \
  hipLaunchKernelGGL((lora_dy_finish_kernel<RR>), g2, dim3(256), 0, s, pw, CS, pb, RS, (int)M, (int)N, alpha, w, \
                     ldw_out, (bf16_t*)split, ld_split, (int)K2, dw, on, oj, accumulate, nwb, 1 << 30,           \
                     (const float*)nullptr, 0, 1.f, (float*)nullptr, (int64_t)0, (int64_t)0, 0);
  switch (r) {
    case 8: LTX_LORA_DY(8) break;
    case 16: LTX_LORA_DY(16) break;
    default: return fail(LTX_ERR_BAD_ARG, "lora_dy: rank must be 8 or 16");
  }
#undef LTX_LORA_DY
  LTX_LAUNCH_CHECK();
  return LTX_OK;
}

extern "C" int ltx_lora_dy_dA_workspace(int64_t M, int64_t N, int64_t K, int64_t r, int64_t* floats) {
  LTX_CHECK_ARG(floats && M > 0 && N > 0 && K > 0 && (r == 8 || r == 16), "lora_dy_dA_workspace: bad args");
  const int64_t RP = r >= 16 ? r : 16;
  const int64_t CS = N / DY_COLS, RS = (M + DY_G * 32 - 1) / (DY_G * 32);
  *floats = CS * M * RP + RS * N * RP + RS * K * RP;
  return LTX_OK;
}

// ltx_lora_dy + the adapter's dA = alpha_a . x^T . w ([K, r] or [r, K]) in three launches instead of
// four: the dY pass (w and dB partials), the x pass reading w from those partials (lora_dy_kernel
// MODE 6), and one finish for w / split, dB and dA. Every output is bitwise what ltx_lora_dy followed
// by ltx_lora_wgrad(x, w, alpha_a) produces (dA: where that takes lora_wgrad_rows, M >= 2048).
extern "C" int ltx_lora_dy_dA(const void* y, int64_t ldy, const float* u, int64_t ldu, const void* w3, int64_t ldw3,
                              const void* x, int64_t ldx, int64_t M, int64_t N, int64_t K, int64_t r, float alpha,
                              float* w, int64_t ldw_out, void* split, int64_t ld_split, int64_t K2, float* dw,
                              int64_t on, int64_t oj, int accumulate, float alpha_a, float* dwa, int64_t ona,
                              int64_t oja, int acc_a, float* workspace, void* stream) {
  LTX_CHECK_ARG(y && u && w3 && x && w && split && dw && dwa && workspace, "lora_dy_dA: null operand");
  LTX_CHECK_ARG(M >= 32 && M % 32 == 0 && N % DY_COLS == 0 && K % DY_COLS == 0 && (r == 8 || r == 16),
                "lora_dy_dA: M % 32 == 0, N % 512 == 0, K % 512 == 0, rank 8 or 16");
  LTX_CHECK_ARG(N <= DY_MAXCS * DY_COLS, "lora_dy_dA: N <= 2048 (the dA pass sums w from <= 4 column splits)");
  LTX_CHECK_ARG(ldy % 8 == 0 && ((uintptr_t)y % 16) == 0 && ldw3 % 8 == 0 && ((uintptr_t)w3 % 16) == 0 && ldw3 >= N,
                "lora_dy_dA: 16-B aligned rows of dY and of the pieces");
  LTX_CHECK_ARG(ldx % 8 == 0 && ((uintptr_t)x % 16) == 0 && ldx >= K, "lora_dy_dA: 16-B aligned rows of x");
  LTX_CHECK_ARG(ldy * 2 * 32 < ((int64_t)1 << 32) && ldx * 2 * 32 < ((int64_t)1 << 32),
                "lora_dy_dA: 32-bit DMA offsets");
  LTX_CHECK_ARG(ldw_out >= r && ldu >= r && K2 >= 3 * r && K2 % 64 == 0 && ld_split >= K2,
                "lora_dy_dA: output strides");
  LTX_CHECK_ARG(ldw_out % 4 == 0 && ((uintptr_t)w % 16) == 0 && ld_split % 4 == 0 && ((uintptr_t)split % 8) == 0,
                "lora_dy_dA: 16-B aligned w rows, 8-B aligned split rows");
  LTX_CHECK_ARG((on == r && oj == 1) || (on == 1 && oj == N), "lora_dy_dA: dB must be a dense [N,r] or [r,N]");
  LTX_CHECK_ARG((ona == r && oja == 1) || (ona == 1 && oja == K), "lora_dy_dA: dA must be a dense [K,r] or [r,K]");
  const int64_t RP = r >= 16 ? r : 16;
  const int CS = (int)(N / DY_COLS), CSx = (int)(K / DY_COLS), RS = (int)((M + DY_G * 32 - 1) / (DY_G * 32));
  float* pw = workspace;
  float* pb = pw + (int64_t)CS * M * RP;
  float* pa = pb + (int64_t)RS * N * RP;
  hipStream_t s = (hipStream_t)stream;
  const int nwb = (int)((M * (r / 4) + 255) / 256);
  const int nbb = (int)((N * r + 63) / 64), nba = (int)((K * r + 63) / 64);
#define LTX_LORA_DYA(RR)                                                                                           \
  hipLaunchKernelGGL((lora_dy_kernel<RR, 3>), dim3((unsigned)CS, (unsigned)RS), dim3(512), 0, s, (const bf16_t*)y, \
                     ldy, u, ldu, (const bf16_t*)w3, ldw3, pw, pb, (int)M, (int)N, (const float*)nullptr, 0, 1.f);  \
  LTX_LAUNCH_CHECK();                                                                                              \
  hipLaunchKernelGGL((lora_dy_kernel<RR, 6>), dim3((unsigned)CSx, (unsigned)RS), dim3(512), 0, s,                 \
                     (const bf16_t*)x, ldx, (const float*)nullptr, (int64_t)0, (const bf16_t*)nullptr, (int64_t)0, \
                     (float*)nullptr, pa, (int)M, (int)K, (const float*)pw, CS, alpha);                             \
  LTX_LAUNCH_CHECK();                                                                                              \
  hipLaunchKernelGGL((lora_dy_finish_kernel<RR>), dim3((unsigned)(nwb + nbb + nba)), dim3(256), 0, s, pw, CS, pb,  \
                     RS, (int)M, (int)N, alpha, w, ldw_out, (bf16_t*)split, ld_split, (int)K2, dw, on, oj,         \
                     accumulate, nwb, nbb, (const float*)pa, (int)K, alpha_a, dwa, ona, oja, acc_a);
  switch (r) {
    case 8: LTX_LORA_DYA(8) break;
    case 16: LTX_LORA_DYA(16) break;
    default: return fail(LTX_ERR_BAD_ARG, "lora_dy_dA: rank must be 8 or 16");
  }
#undef LTX_LORA_DYA
  LTX_LAUNCH_CHECK();
  return LTX_OK;
}

}  // namespace ltx
