// LoRA adapter contractions in f32 (peft 0.17.1 keeps adapters in f32 on a bf16 base:
// training.py:50-68 + autocast_adapter_dtype). Rank r <= 32 makes these skinny, so they are
// HBM-bound (x or dY is read once: 2 B/element for 2r FLOP/element) and run on the exact-f32
// matrix core v_mfma_f32_16x16x4_f32 (an f32 fma chain, bitwise like the VALU, at 4x its rate),
// which keeps the adapters' f32 semantics while freeing the VALU for address math.
// The up-projection (B) and its input-gradient half are fused into the bf16 GEMM epilogues
// (gemm.hip: LTX_EPI_LORA / LTX_EPI_LORA_DGRAD_ACCUM).
#include <cstdlib>
#include <type_traits>

#include "common.h"
#include "ltx_hip.h"

namespace ltx {

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// out[m,j] = alpha * sum_k x[m,k] * Wr[j*wj + k*wk]   (+ optional activation split, below)
// Block = 4 waves on the same 32 rows (two 16-row groups), K split 4 ways; for small M (text
// tokens) 8 waves on 16 rows, K split 8 ways, to fill the chip (K % 128 / % 256; the
// loads of 4 k steps go out together). Per 32-deep k step a
// lane loads 8 consecutive k of its row (one 16-B load per row group) and the 8 matching weights
// of its j, and issues 8 MFMAs whose k index g = lane>>4 stands for k = kb + 8g + i (the same
// permutation on both operands); one weight fetch serves both row groups. The 4 partial 32 x r
// tiles are summed through LDS. With split != null the row is also written as the K-extension
// activation operand [hi | hi | lo | 0..] (bf16, K2 columns) of the LoRA-fused GEMM.
template <int R, int RG, int KW>
__global__ __launch_bounds__(64 * KW) void lora_down_kernel(const bf16_t* __restrict__ x, int64_t ldx,
                                                        const float* __restrict__ Wr, int64_t wj, int64_t wk,
                                                        float* __restrict__ out, int64_t ldo, int M, int K,
                                                        float alpha, bf16_t* __restrict__ split, int64_t lds,
                                                        int K2, int64_t gx, int64_t gw, int64_t go, int64_t gs) {
  // group blockIdx.y: one launch for several adapters (element strides; 0 = shared operand)
  x += blockIdx.y * gx;
  Wr += blockIdx.y * gw;
  out += blockIdx.y * go;
  if (split) split += blockIdx.y * gs;
  constexpr int RP = R >= 16 ? R : 16;  // R = 8 runs as a padded 16-wide tile
  constexpr int JT = RP / 16;
  // RG = 16-row groups per block: 2 (one weight fetch serves 32 rows) when there are rows enough
  // to fill the chip, else 1
  __shared__ float part[KW][16 * RG][RP + 1];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int m0 = blockIdx.x * 16 * RG;
  const int g = lane >> 4;
  const int kper = K / KW;
  const int kbeg = wave * kper, kend = kbeg + kper;
  f32x4 acc[RG][JT];
#pragma unroll
  for (int q = 0; q < RG; ++q)
#pragma unroll
    for (int t = 0; t < JT; ++t) acc[q][t] = (f32x4){0.f, 0.f, 0.f, 0.f};
  const bf16_t* xr[RG];
#pragma unroll
  for (int q = 0; q < RG; ++q) xr[q] = x + (int64_t)min(m0 + 16 * q + (lane & 15), M - 1) * ldx;
  // NS x 32 k per call: all x and weight loads of the NS sub-steps issued before their MFMAs
  auto kstep = [&](auto ns_tag, int kb) {
    constexpr int NS = decltype(ns_tag)::value;
    u32x4 xv[NS][RG];
    float wv[NS][JT][8];
#pragma unroll
    for (int st = 0; st < NS; ++st) {
      const int k = kb + 32 * st + 8 * g;
#pragma unroll
      for (int q = 0; q < RG; ++q) xv[st][q] = *(const u32x4*)(xr[q] + k);
#pragma unroll
      for (int t = 0; t < JT; ++t) {
        const int j = t * 16 + (lane & 15);
        if (j < R) {
          const float* wp = Wr + (int64_t)j * wj + (int64_t)k * wk;
          if (wk == 1) {
            const f32x4 a = *(const f32x4*)wp, b = *(const f32x4*)(wp + 4);
#pragma unroll
            for (int i = 0; i < 4; ++i) { wv[st][t][i] = a[i]; wv[st][t][4 + i] = b[i]; }
          } else {
#pragma unroll
            for (int i = 0; i < 8; ++i) wv[st][t][i] = wp[(int64_t)i * wk];
          }
        } else {
#pragma unroll
          for (int i = 0; i < 8; ++i) wv[st][t][i] = 0.f;
        }
      }
    }
#pragma unroll
    for (int st = 0; st < NS; ++st)
#pragma unroll
      for (int q = 0; q < RG; ++q)
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const float xf = bf2f((bf16_t)(xv[st][q][i >> 1] >> ((i & 1) * 16)));
#pragma unroll
          for (int t = 0; t < JT; ++t) acc[q][t] = mfma4(xf, wv[st][t][i], acc[q][t]);
        }
  };
  int kb = kbeg;
  for (; kb + 128 <= kend; kb += 128) kstep(std::integral_constant<int, 4>{}, kb);
  for (; kb < kend; kb += 32) kstep(std::integral_constant<int, 1>{}, kb);
  // C layout: col j = lane & 15 (+16t), row m = (lane >> 4) * 4 + reg
#pragma unroll
  for (int q = 0; q < RG; ++q)
#pragma unroll
    for (int t = 0; t < JT; ++t)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) part[wave][16 * q + (lane >> 4) * 4 + rr][t * 16 + (lane & 15)] = acc[q][t][rr];
  __syncthreads();
  for (int e = threadIdx.x; e < 16 * RG * R; e += 64 * KW) {
    const int rr = e / R, j = e % R;
    const int m = m0 + rr;
    if (m >= M) continue;
    float sum = 0.f;
#pragma unroll
    for (int w = 0; w < KW; ++w) sum += part[w][rr][j];
    const float v = sum * alpha;
    out[(int64_t)m * ldo + j] = v;
    if (split) {
      const bf16_t hi = f2bf(v);
      const bf16_t lo = f2bf(v - bf2f(hi));
      bf16_t* sr = split + (int64_t)m * lds;
      sr[j] = hi;
      sr[R + j] = hi;
      sr[2 * R + j] = lo;
    }
  }
  if (split) {  // zero padding columns 3R .. K2
    const int pad = K2 - 3 * R;
    for (int e = threadIdx.x; e < 16 * RG * pad; e += 64 * KW) {
      const int rr = e / pad, c = 3 * R + e % pad;
      const int m = m0 + rr;
      if (m < M) split[(int64_t)m * lds + c] = (bf16_t)0;
    }
  }
}

// Three bf16 pieces of an f32 [R, K] operand (element (j, k) at src[j*rs + k*cs]): hi = bf16(v),
// mid = bf16(v - hi), lo = bf16(v - hi - mid) hold v to 24 significant bits, so the exact
// bf16 x bf16 products of the matrix core against an exact bf16 activation, summed in f32, stand
// in for peft's f32 contraction. Row p*RP + j of out is piece p of row j; rows j >= R (RP = 16
// for R = 8) are zero, so a 16-wide fragment never reads past the pieces.
__global__ void lora_pieces_kernel(const float* __restrict__ src, int64_t rs, int64_t cs, int R, int RP, int K,
                                   bf16_t* __restrict__ out, int64_t ldo) {
  const int64_t total = (int64_t)RP * K;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int j = (int)(i / K), k = (int)(i % K);
    const float v = j < R ? src[(int64_t)j * rs + (int64_t)k * cs] : 0.f;
    const bf16_t hi = f2bf(v);
    const float r1 = v - bf2f(hi);
    const bf16_t mid = f2bf(r1);
    const bf16_t lo = f2bf(r1 - bf2f(mid));
    out[(int64_t)j * ldo + k] = hi;
    out[(int64_t)(RP + j) * ldo + k] = mid;
    out[(int64_t)(2 * RP + j) * ldo + k] = lo;
  }
}

// The adapter row contraction for token-sized M: out[m,j] = alpha * sum_k x[m,k] * W[j,k] with W
// as its three bf16 pieces (lora_pieces_kernel), on v_mfma_f32_16x16x32_bf16. The rows stream
// through LDS by LDS-DMA (one 8-row x 128-B piece per wave-instruction, whole cache lines)
// instead of per-lane register loads of 16 rows x 64 B. Block = NW waves on 32 rows; wave w owns
// K range [w K/NW, (w+1) K/NW) and streams its own 32 x 64 slots (4 KiB) through a private
// NR-slot ring (DMA NR-1 slots ahead), with the pieces' fragments (L2-resident, shared by every
// block) loaded two slots ahead into three register sets, so no workgroup barrier is needed
// before the cross-wave sum. The loads are inline asm with counted waits: step s issues the
// fragments of slot s+2, then the DMA of slot s+NR-1; its wait leaves in flight only what was
// issued after slot s's fragments.
// LDS slot image: row r (128 B) holds k chunk c (8 bf16) at physical chunk c ^ ((r >> 1) & 7):
// conflict-free for the 16-lane groups of ds_read_b128 over rows 0-15 (two rows per 64 banks).
template <int R, int NW, int NR>
__global__ __launch_bounds__(64 * NW) void lora_rows_kernel(const bf16_t* __restrict__ x, int64_t ldx,
                                                            const bf16_t* __restrict__ w3, int64_t ldw,
                                                            float* __restrict__ out, int64_t ldo, int M, int K,
                                                            float alpha, bf16_t* __restrict__ split, int64_t lds,
                                                            int K2) {
  static_assert(NR >= 4, "ring depth (the counted waits assume D(s) precedes W(s))");
  constexpr int RP = R >= 16 ? R : 16;
  constexpr int JT = RP / 16;
  constexpr int NF = 3 * JT;  // piece fragments per 32-deep k step
  constexpr int WL = 2 * NF;  // fragment loads per slot
  __shared__ __attribute__((aligned(16))) char ring[NW][NR][4096];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // scalar DMA / load bases
  const int m0 = blockIdx.x * 32;
  const int kw = K / NW, kw0 = wave * kw, nslot = kw / 64;
  // DMA: piece i of a slot = rows 8i .. 8i+7; lane -> row 8i + (lane >> 3), physical chunk lane & 7
  uint32_t xo[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = 8 * i + (lane >> 3);
    const int lchunk = (lane & 7) ^ ((row >> 1) & 7);
    xo[i] = (uint32_t)(((int64_t)min(m0 + row, M - 1) * ldx + lchunk * 8) * 2);
  }
  const char* xbase = (const char*)(x + kw0);
  const uint32_t lbase = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) char*)&ring[wave][0][0]);
  auto dma = [&](int s) {
    const char* sb = xbase + s * 128;
    const uint32_t l = lbase + (s % NR) * 4096;
    unsigned keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %6\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %5\n\t"
        "s_add_u32 m0, m0, 0x400\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %2, %5\n\t"
        "s_add_u32 m0, m0, 0x400\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %3, %5\n\t"
        "s_add_u32 m0, m0, 0x400\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %4, %5\n\ts_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(xo[0]), "v"(xo[1]), "v"(xo[2]), "v"(xo[3]), "s"(sb), "s"(l)
        : "memory", "scc");
  };
  // piece fragments: lane -> column j = 16t + (lane & 15), k chunk lane >> 4; k half by offset
  uint32_t wo[NF];
#pragma unroll
  for (int p = 0; p < 3; ++p)
#pragma unroll
    for (int t = 0; t < JT; ++t)
      wo[p * JT + t] = (uint32_t)((((int64_t)(p * RP + t * 16 + (lane & 15))) * ldw + (lane >> 4) * 8) * 2);
  const char* wbase = (const char*)(w3 + kw0);
  s16x8 wf[3][2][NF];  // [register set][k half][fragment]
  auto wload = [&](int s, s16x8 (&dst)[2][NF]) {
    const char* sb = wbase + s * 128;
#pragma unroll
    for (int f = 0; f < NF; ++f) {
      asm volatile("global_load_dwordx4 %0, %1, %2" : "=v"(dst[0][f]) : "v"(wo[f]), "s"(sb) : "memory");
      asm volatile("global_load_dwordx4 %0, %1, %2 offset:64" : "=v"(dst[1][f]) : "v"(wo[f]), "s"(sb) : "memory");
    }
  };
  // fragment reads: rows 16q + (lane & 15), logical chunk 4h + (lane >> 4)
  int roff[2][2];
#pragma unroll
  for (int q = 0; q < 2; ++q)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int row = 16 * q + (lane & 15);
      roff[q][h] = row * 128 + (((4 * h + (lane >> 4)) ^ ((row >> 1) & 7)) * 16);
    }
  f32x4 acc[2][JT];
#pragma unroll
  for (int q = 0; q < 2; ++q)
#pragma unroll
    for (int t = 0; t < JT; ++t) acc[q][t] = (f32x4){0.f, 0.f, 0.f, 0.f};

  auto step = [&](int s, s16x8 (&cur)[2][NF], s16x8 (&nxt2)[2][NF]) {
    // issued after slot s's fragments: D(s+NR-2), W(s+1), D(s+NR-1) (those that exist)
    const int younger = 4 * (s + NR - 2 < nslot) + WL * (s + 1 < nslot) + 4 * (s + NR - 1 < nslot);
    switch (younger) {
      case 4 + WL + 4: asm volatile("s_waitcnt vmcnt(%0)" ::"n"(4 + WL + 4) : "memory"); break;
      case WL + 4: asm volatile("s_waitcnt vmcnt(%0)" ::"n"(WL + 4) : "memory"); break;
      case WL: asm volatile("s_waitcnt vmcnt(%0)" ::"n"(WL) : "memory"); break;
      case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
      default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    }
    const char* sl = &ring[wave][s % NR][0];
    s16x8 xf[2][2];
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
      for (int h = 0; h < 2; ++h) xf[q][h] = *(const s16x8*)(sl + roff[q][h]);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (s + 2 < nslot) wload(s + 2, nxt2);
    if (s + NR - 1 < nslot) dma(s + NR - 1);
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int p = 0; p < 3; ++p)
#pragma unroll
        for (int t = 0; t < JT; ++t)
#pragma unroll
          for (int q = 0; q < 2; ++q)
            acc[q][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xf[q][h], cur[h][p * JT + t], acc[q][t], 0, 0, 0);
  };
  // prologue = steps -2 and -1 of the steady pattern: D(0 .. NR-4), W(0), D(NR-3), W(1), D(NR-2)
  for (int i = 0; i + 3 < NR; ++i)
    if (i < nslot) dma(i);
  wload(0, wf[0]);
  if (NR - 3 < nslot) dma(NR - 3);
  if (nslot > 1) wload(1, wf[1]);
  if (NR - 2 < nslot) dma(NR - 2);
  for (int s = 0; s < nslot; s += 3) {
    step(s, wf[0], wf[2]);
    if (s + 1 < nslot) step(s + 1, wf[1], wf[0]);
    if (s + 2 < nslot) step(s + 2, wf[2], wf[1]);
  }
  // cross-wave sum through LDS (the ring is free once every wave is past its last reads)
  __syncthreads();
  float(*part)[32][RP + 1] = (float(*)[32][RP + 1])&ring[0][0][0];
  static_assert(NW * 32 * (RP + 1) * 4 <= NW * NR * 4096, "partials fit the ring");
  // C layout: col j = lane & 15 (+16t), row m = (lane >> 4) * 4 + reg
#pragma unroll
  for (int q = 0; q < 2; ++q)
#pragma unroll
    for (int t = 0; t < JT; ++t)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) part[wave][16 * q + (lane >> 4) * 4 + rr][t * 16 + (lane & 15)] = acc[q][t][rr];
  __syncthreads();
  for (int e = threadIdx.x; e < 32 * R; e += 64 * NW) {
    const int rr = e / R, j = e % R;
    const int m = m0 + rr;
    if (m >= M) continue;
    float sum = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) sum += part[w][rr][j];
    const float v = sum * alpha;
    out[(int64_t)m * ldo + j] = v;
    if (split) {
      const bf16_t hi = f2bf(v);
      const bf16_t lo = f2bf(v - bf2f(hi));
      bf16_t* sr = split + (int64_t)m * lds;
      sr[j] = hi;
      sr[R + j] = hi;
      sr[2 * R + j] = lo;
    }
  }
  if (split) {  // zero padding columns 3R .. K2
    const int pad = K2 - 3 * R;
    for (int e = threadIdx.x; e < 32 * pad; e += 64 * NW) {
      const int rr = e / pad, c = 3 * R + e % pad;
      const int m = m0 + rr;
      if (m < M) split[(int64_t)m * lds + c] = (bf16_t)0;
    }
  }
}

// dw(n,j) (+)= alpha * sum_m y[m,n] * u[m,j], deterministic: with one row split each block owns
// its outputs (a plain store, or load + add + store when accumulating); with S > 1 row splits each
// block stores its partial to part[g][split][r*N] and lora_wgrad_finish_kernel sums the S partials
// in split order (no atomics: the result does not depend on the order blocks finish).
// Computed as C[j][n] += U^T[j][m] . Y[m][n] on v_mfma_f32_16x16x4_f32: per 4 rows a lane loads
// u[m][j] (4 B) and 8 consecutive columns of y (one 16-B load; 16 lanes = 128 columns, 256 B
// per row), and MFMA t (t = 0..7) takes element t, so its output column c stands for
// n0 + 8c + t (a fixed permutation undone at the store). Block = 8 waves on the same 128
// columns, interleaved row quads; the wave partials are reduced through LDS in wave order.
// the token-sized paths of ltx_lora_rows and ltx_lora_wgrad (lora_dy.hip)
bool lora_rows_dy(const bf16_t* x, int64_t ldx, const bf16_t* w3, int64_t ldw, float* out, int64_t ldo, int64_t M,
                  int64_t K, int64_t r, float alpha, bf16_t* split, int64_t ld_split, int64_t K2, hipStream_t s);
bool lora_wgrad_rows(const bf16_t* y, int64_t ldy, const float* u, int64_t ldu, float* dw, int64_t on, int64_t oj,
                     int64_t M, int64_t N, int64_t r, float alpha, int accumulate, hipStream_t s);

template <int R>
__global__ __launch_bounds__(512) void lora_wgrad_kernel(const bf16_t* __restrict__ y, int64_t ldy,
                                                         const float* __restrict__ u, int64_t ldu,
                                                         float* __restrict__ dw, int64_t on, int64_t oj, int M,
                                                         int N, int rows_per_split, float alpha, int64_t gy,
                                                         int64_t gu, int64_t gd, float* __restrict__ part,
                                                         int accumulate) {
  // group blockIdx.z: one launch for several adapters (element strides; 0 = shared operand)
  y += blockIdx.z * gy;
  u += blockIdx.z * gu;
  dw += blockIdx.z * gd;
  constexpr int RP = R >= 16 ? R : 16;
  constexpr int JT = RP / 16;
  constexpr int NW = 8;  // waves per block, interleaved over row quads
  __shared__ float red[NW][RP][128 + 1];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int n0 = blockIdx.x * 128;
  const int mb = blockIdx.y * rows_per_split;
  const int me = min(M, mb + rows_per_split);
  const int c8 = n0 + 8 * (lane & 15);  // this lane's 8 columns
  const bool colok = c8 < N;            // N % 8 == 0: all 8 in or all out
  f32x4 acc[JT][8];
#pragma unroll
  for (int t = 0; t < JT; ++t)
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[t][i] = (f32x4){0.f, 0.f, 0.f, 0.f};
  // each wave takes row quads mb + 4*wave + 32*i; four quads' loads are issued before their
  // 32 MFMAs so every wave keeps 4 x 1 KiB of y in flight
  for (int m16 = mb + 4 * wave; m16 < me; m16 += 4 * 4 * NW) {
    u32x4 yv[4];
    float uv[4][JT];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int m = m16 + 4 * NW * q + (lane >> 4);
      const bool rowok = m < me;
      yv[q] = (u32x4){0, 0, 0, 0};
      if (rowok && colok) yv[q] = *(const u32x4*)(y + (int64_t)m * ldy + c8);
#pragma unroll
      for (int t = 0; t < JT; ++t) {
        const int j = t * 16 + (lane & 15);
        uv[q][t] = (rowok && j < R) ? u[(int64_t)m * ldu + j] : 0.f;
      }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float yf = bf2f((bf16_t)(yv[q][i >> 1] >> ((i & 1) * 16)));
#pragma unroll
        for (int t = 0; t < JT; ++t) acc[t][i] = mfma4(uv[q][t], yf, acc[t][i]);
      }
  }
  // C_t,i: row j = t*16 + (lane>>4)*4 + rr, col c = lane & 15 -> n = n0 + 8c + i
#pragma unroll
  for (int t = 0; t < JT; ++t)
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) red[wave][t * 16 + (lane >> 4) * 4 + rr][8 * (lane & 15) + i] = acc[t][i][rr];
  __syncthreads();
  // consecutive threads -> consecutive output addresses (j fastest when the output is [N, r])
  const bool jfast = (oj == 1);
  for (int e = tid; e < R * 128; e += 64 * NW) {
    const int j = jfast ? e % R : e / 128;
    const int c = jfast ? e / R : e % 128;
    const int n = n0 + c;
    if (n < N) {
      float sum = 0.f;
#pragma unroll
      for (int w = 0; w < NW; ++w) sum += red[w][j][c];
      const float v = sum * alpha;
      const int64_t o = (int64_t)n * on + (int64_t)j * oj;
      if (part != nullptr) {  // this split's partial, in the output's own layout
        part[((int64_t)blockIdx.z * gridDim.y + blockIdx.y) * ((int64_t)N * R) + o] = v;
      } else {
        float* d = dw + o;
        *d = accumulate ? *d + v : v;
      }
    }
  }
}

// dw[g][e] (+)= sum over the S row splits, in split order, of part[g][s][e]; 4 elements per thread
__global__ void lora_wgrad_finish_kernel(const float* __restrict__ part, float* __restrict__ dw, int64_t n_per_group,
                                         int S, int64_t gd, int accumulate) {
  const int64_t i4 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (i4 >= n_per_group) return;
  const float* p = part + (int64_t)blockIdx.y * S * n_per_group + i4;
  f32x4 acc = *(const f32x4*)p;
  for (int s = 1; s < S; ++s) {
    const f32x4 v = *(const f32x4*)(p + (int64_t)s * n_per_group);
    acc[0] += v[0]; acc[1] += v[1]; acc[2] += v[2]; acc[3] += v[3];
  }
  float* d = dw + (int64_t)blockIdx.y * gd + i4;
  if (accumulate) {
    const f32x4 o = *(const f32x4*)d;
    acc[0] = o[0] + acc[0]; acc[1] = o[1] + acc[1]; acc[2] = o[2] + acc[2]; acc[3] = o[3] + acc[3];
  }
  *(f32x4*)d = acc;
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

extern "C" int ltx_lora_down_grouped(const void* x, int64_t ldx, const float* Wr, int64_t wj, int64_t wk,
                                     float* out, int64_t ldo, int64_t M, int64_t K, int64_t r, float alpha,
                                     void* split, int64_t ld_split, int64_t K2, int64_t groups, int64_t gx,
                                     int64_t gw, int64_t go, int64_t gs, void* stream) {
  LTX_CHECK_ARG(x && Wr && out && M > 0 && K > 0, "lora_down: bad args");
  LTX_CHECK_ARG(groups >= 1 && groups <= 65535 && gx % 8 == 0 && (wk != 1 || gw % 4 == 0),
                "lora_down: groups in [1, 65535], x / W group strides keep 16-B alignment");
  LTX_CHECK_ARG(!split || (K2 >= 3 * r && K2 % 64 == 0 && ld_split >= K2), "lora_down: split needs K2 >= 3r, %64");
  LTX_CHECK_ARG(K % 128 == 0 && ldx % 8 == 0 && ((uintptr_t)x % 16) == 0, "lora_down: K %128, 16-B rows");
  LTX_CHECK_ARG(wk != 1 || (wj % 4 == 0 && ((uintptr_t)Wr % 16) == 0), "lora_down: W rows must be 16-B aligned");
  // 32-row blocks for token-sized M (16-row blocks measured 26 vs 21 us at M = 14336); K split 8
  // ways (512 threads) there: 19.7 vs 20.7 us (forward A), 18.6 vs 19.6 us (split B^T dgrad)
  const bool big = M >= 8192;
  const dim3 grid((unsigned)(big ? (M + 31) / 32 : (M + 15) / 16), (unsigned)groups);
  hipStream_t s = (hipStream_t)stream;
  bf16_t* sp = (bf16_t*)split;
#define LTX_LORA_DOWN(RR)                                                                                      \
  if (big && K % 256 == 0)                                                                                     \
    hipLaunchKernelGGL((lora_down_kernel<RR, 2, 8>), grid, dim3(512), 0, s, (const bf16_t*)x, ldx, Wr, wj, wk,  \
                       out, ldo, (int)M, (int)K, alpha, sp, ld_split, (int)K2, gx, gw, go, gs);                \
  else if (big)                                                                                                \
    hipLaunchKernelGGL((lora_down_kernel<RR, 2, 4>), grid, dim3(256), 0, s, (const bf16_t*)x, ldx, Wr, wj, wk,  \
                       out, ldo, (int)M, (int)K, alpha, sp, ld_split, (int)K2, gx, gw, go, gs);                \
  else if (K % 256 == 0)                                                                                       \
    hipLaunchKernelGGL((lora_down_kernel<RR, 1, 8>), grid, dim3(512), 0, s, (const bf16_t*)x, ldx, Wr, wj, wk,  \
                       out, ldo, (int)M, (int)K, alpha, sp, ld_split, (int)K2, gx, gw, go, gs);                \
  else                                                                                                         \
    hipLaunchKernelGGL((lora_down_kernel<RR, 1, 4>), grid, dim3(256), 0, s, (const bf16_t*)x, ldx, Wr, wj, wk,  \
                       out, ldo, (int)M, (int)K, alpha, sp, ld_split, (int)K2, gx, gw, go, gs);
  switch (r) {
    case 8: LTX_LORA_DOWN(8) break;
    case 16: LTX_LORA_DOWN(16) break;
    case 32: LTX_LORA_DOWN(32) break;
    default: return fail(LTX_ERR_BAD_ARG, "lora_down: rank must be 8, 16 or 32");
  }
#undef LTX_LORA_DOWN
  LTX_LAUNCH_CHECK();
  return LTX_OK;
}

extern "C" int ltx_lora_down(const void* x, int64_t ldx, const float* Wr, int64_t wj, int64_t wk, float* out,
                             int64_t ldo, int64_t M, int64_t K, int64_t r, float alpha, void* split,
                             int64_t ld_split, int64_t K2, void* stream) {
  return ltx_lora_down_grouped(x, ldx, Wr, wj, wk, out, ldo, M, K, r, alpha, split, ld_split, K2, 1, 0, 0, 0, 0,
                               stream);
}

extern "C" int ltx_lora_pieces(const float* src, int64_t rs, int64_t cs, int64_t r, int64_t K, void* out,
                               int64_t ldo, void* stream) {
  LTX_CHECK_ARG(src && out && K > 0 && ldo >= K && (r == 8 || r == 16 || r == 32),
                "lora_pieces: bad args (rank 8, 16 or 32)");
  const int RP = r >= 16 ? (int)r : 16;
  const int64_t total = (int64_t)RP * K;
  int64_t g = (total + 255) / 256;
  if (g > 4096) g = 4096;
  hipLaunchKernelGGL(lora_pieces_kernel, dim3((unsigned)g), dim3(256), 0, (hipStream_t)stream, src, rs, cs, (int)r, RP,
                     (int)K, (bf16_t*)out, ldo);
  LTX_LAUNCH_CHECK();
  return LTX_OK;
}

extern "C" int ltx_lora_rows(const void* x, int64_t ldx, const void* w3, int64_t ldw, float* out, int64_t ldo,
                             int64_t M, int64_t K, int64_t r, float alpha, void* split, int64_t ld_split, int64_t K2,
                             void* stream) {
  LTX_CHECK_ARG(x && w3 && out && M > 0 && K > 0 && ldo >= r, "lora_rows: bad args");
  LTX_CHECK_ARG(K % 256 == 0 && ldx % 8 == 0 && ((uintptr_t)x % 16) == 0 && ldw % 8 == 0 &&
                    ((uintptr_t)w3 % 16) == 0 && ldw >= K,
                "lora_rows: K % 256, 16-B aligned rows of x and of the pieces");
  LTX_CHECK_ARG((int64_t)ldx * 2 * (M - 1) + 2 * K < ((int64_t)1 << 32) && (int64_t)ldw * 2 * 3 * 32 < ((int64_t)1 << 32),
                "lora_rows: 32-bit DMA offsets");
  LTX_CHECK_ARG(!split || (K2 >= 3 * r && K2 % 64 == 0 && ld_split >= K2), "lora_rows: split needs K2 >= 3r, %64");
  hipStream_t s = (hipStream_t)stream;
  bf16_t* sp = (bf16_t*)split;
  if (lora_rows_dy((const bf16_t*)x, ldx, (const bf16_t*)w3, ldw, out, ldo, M, K, r, alpha, sp, ld_split, K2, s)) {
    LTX_LAUNCH_CHECK();
    return LTX_OK;
  }
  const dim3 grid((unsigned)((M + 31) / 32));
  // 4 waves x K/4 per 32-row block, 4-slot ring: 16.3 us at M = 14336, K = 2048, r = 16 against
  // 19.9 us for lora_down_kernel (8 waves x K/8 with a 3-slot ring: 17.8 us)
#define LTX_LORA_ROWS(RR)                                                                             \
  hipLaunchKernelGGL((lora_rows_kernel<RR, 4, 4>), grid, dim3(256), 0, s, (const bf16_t*)x, ldx,     \
                     (const bf16_t*)w3, ldw, out, ldo, (int)M, (int)K, alpha, sp, ld_split, (int)K2);
  switch (r) {
    case 8: LTX_LORA_ROWS(8) break;
    case 16: LTX_LORA_ROWS(16) break;
    case 32: LTX_LORA_ROWS(32) break;
    default: return fail(LTX_ERR_BAD_ARG, "lora_rows: rank must be 8, 16 or 32");
  }
#undef LTX_LORA_ROWS
  LTX_LAUNCH_CHECK();
  return LTX_OK;
}

extern "C" int ltx_lora_wgrad_grouped(const void* y, int64_t ldy, const float* u, int64_t ldu, float* dw,
                                      int64_t on, int64_t oj, int64_t M, int64_t N, int64_t r, float alpha,
                                      int accumulate, int64_t groups, int64_t gy, int64_t gu, int64_t gd,
                                      void* stream) {
  LTX_CHECK_ARG(y && u && dw && M > 0 && N > 0, "lora_wgrad: bad args");
  LTX_CHECK_ARG((on == r && oj == 1) || (on == 1 && oj == N), "lora_wgrad: output must be a dense [N,r] or [r,N]");
  LTX_CHECK_ARG(N % 8 == 0 && ldy % 8 == 0 && ((uintptr_t)y % 16) == 0, "lora_wgrad: y rows must be 16-B aligned");
  LTX_CHECK_ARG(groups >= 1 && groups <= 65535 && gy % 8 == 0 && (groups == 1 || gd >= N * r),
                "lora_wgrad: groups in [1, 65535], 16-B aligned y groups, disjoint outputs");
  hipStream_t s = (hipStream_t)stream;
  if (groups == 1 && lora_wgrad_rows((const bf16_t*)y, ldy, u, ldu, dw, on, oj, M, N, r, alpha, accumulate, s)) {
    LTX_LAUNCH_CHECK();
    return LTX_OK;
  }
  // ~512 blocks of 128 columns x >= 512 rows (8 waves x 4-quad steps): enough waves to stream y.
  // ~512 blocks (two per CU): 17.9 us vs 20.0 us with 256 at M = 14336, N = 2048, r = 16. Splits
  // of >= 256 rows in multiples of 32 (a wave's row quads stay aligned; the last 128-row step of a
  // split may be partial): M = 14336 -> 32 splits of 448 rows = exactly 512 blocks
  const int nb = (int)((N + 127) / 128);
  const int target = 512;
  int splits = (int)((target + nb * groups - 1) / (nb * groups));
  const int max_splits = (int)((M + 255) / 256);
  if (splits > max_splits) splits = max_splits;
  if (splits < 1) splits = 1;
  int rps = (int)((M + splits - 1) / splits);
  rps = (rps + 31) / 32 * 32;
  splits = (int)((M + rps - 1) / rps);
  // S > 1: per-split partials in the stream's workspace (caller-owned, stream-ordered), summed in
  // order by the finish kernel; with no room for them, one split (each block owns its outputs)
  float* part = nullptr;
  if (splits > 1) {
    size_t ws = 0;
    float* w = stream_workspace(s, &ws);
    const bool aligned = ((uintptr_t)dw % 16) == 0 && (N * r) % 4 == 0 && (groups == 1 || gd % 4 == 0);
    if (w != nullptr && aligned && (size_t)groups * splits * N * r * sizeof(float) <= ws) {
      part = w;
    } else {
      splits = 1;
      rps = (int)M;
    }
  }
  const dim3 grid((unsigned)nb, (unsigned)splits, (unsigned)groups);
  const int acc = accumulate ? 1 : 0;
  switch (r) {
    case 8: hipLaunchKernelGGL(lora_wgrad_kernel<8>, grid, dim3(512), 0, s, (const bf16_t*)y, ldy, u, ldu, dw, on, oj, (int)M, (int)N, rps, alpha, gy, gu, gd, part, acc); break;
    case 16: hipLaunchKernelGGL(lora_wgrad_kernel<16>, grid, dim3(512), 0, s, (const bf16_t*)y, ldy, u, ldu, dw, on, oj, (int)M, (int)N, rps, alpha, gy, gu, gd, part, acc); break;
    case 32: hipLaunchKernelGGL(lora_wgrad_kernel<32>, grid, dim3(512), 0, s, (const bf16_t*)y, ldy, u, ldu, dw, on, oj, (int)M, (int)N, rps, alpha, gy, gu, gd, part, acc); break;
    default: return fail(LTX_ERR_BAD_ARG, "lora_wgrad: rank must be 8, 16 or 32");
  }
  LTX_LAUNCH_CHECK();
  if (part != nullptr) {
    const int64_t npg = N * r;
    const dim3 gf((unsigned)((npg / 4 + 255) / 256), (unsigned)groups);
    hipLaunchKernelGGL(lora_wgrad_finish_kernel, gf, dim3(256), 0, s, part, dw, npg, splits, gd, acc);
    LTX_LAUNCH_CHECK();
  }
  return LTX_OK;
}

extern "C" int ltx_lora_wgrad(const void* y, int64_t ldy, const float* u, int64_t ldu, float* dw, int64_t on,
                              int64_t oj, int64_t M, int64_t N, int64_t r, float alpha, int accumulate,
                              void* stream) {
  return ltx_lora_wgrad_grouped(y, ldy, u, ldu, dw, on, oj, M, N, r, alpha, accumulate, 1, 0, 0, 0, stream);
}
