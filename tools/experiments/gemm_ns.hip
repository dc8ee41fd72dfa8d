// Eight-wave bf16 GEMM with a 4-slot LDS ring of 32-deep K-steps (C[M,N] = epi(A[M,K] . W[N,K]^T)).
#include <type_traits>

#include "gemm_common.h"

namespace ltx {

// ---------------------------------------------------------------------------------------------
// ns kernel: the 8-wave tile of gemm_nt_kernel_t (BMT x 256, BMT = 256: 4 (m) x 2 (n) waves of
// 64 x 128; BMT = 224: 2 (m) x 4 (n) waves of 112 x 64) fed through a ring of NS_SLOTS 32-deep
// K-steps (X [BMT][32] + W [256][32] bf16 per slot, 64-B rows whose 16-B chunks are XOR-swizzled by
// (-(row >> 2)) & 3: conflict-free 16x16x32 fragment reads; the swizzle is applied to the DMA
// SOURCE address, the LDS-DMA image is lane-linear).
// Per K-step t, every wave:
//   * waits for its own DMA of step t+1 (counted vmcnt: steps t+2, t+3 stay in flight) and joins
//     the workgroup barrier -> step t+1 is in LDS for everyone, and every read of step t-1's slot
//     has retired;
//   * issues its 4 DMA pieces (1 KiB each) of step t+3 into that slot, spread over the MFMAs;
//   * runs its MF x NF MFMAs on step t's fragments (registers, read during step t-1) while reading
//     step t+1's fragments into the other register set.
// So the DMA of a step has three steps of MFMAs to land, LDS reads have a whole step, and the one
// barrier per step never waits for the step being computed. Equal DMA work on all 8 waves.
// ---------------------------------------------------------------------------------------------
constexpr int NS_BKS = 32;
constexpr int NS_SLOTS = 4;
constexpr int ns_lds_bytes(int bmt) {
  return (NS_SLOTS * (bmt + 256) * NS_BKS * 2 > bmt * C_STRIDE2) ? NS_SLOTS * (bmt + 256) * NS_BKS * 2
                                                                 : bmt * C_STRIDE2;
}

template <int EPI, int R, int BMT>
__global__ __launch_bounds__(512, 1) void gemm_ns_kernel(const GemmParams p) {
  static_assert(BMT == 256 || BMT == 224, "tile height");
  constexpr int WMW = (BMT == 256) ? 4 : 2;  // waves along m
  constexpr int WNW = 8 / WMW;               // waves along n
  constexpr int WTM = BMT / WMW;             // 64 | 112
  constexpr int WTN = 256 / WNW;             // 128 | 64
  constexpr int MF = WTM / 16;               // 4 | 7
  constexpr int NF = WTN / 16;               // 8 | 4
  constexpr int XB = BMT * NS_BKS * 2;       // X bytes per slot
  constexpr int SB = XB + 256 * NS_BKS * 2;  // slot bytes
  constexpr int XP = BMT / 16;               // X pieces per slot: 16 | 14
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ntm = (p.M + BMT - 1) / BMT, ntn = (p.N + 255) / 256;
  int tm, tn;
  block_to_tile(blockIdx.x, ntm, ntn, tm, tn);
  const int m0 = tm * BMT, n0 = tn * 256;
  const int nk_main = p.K / NS_BKS;
  const int nk = nk_main + p.K2 / NS_BKS;

  // ---- LDS-DMA: wave w moves X pieces w, w+8 and W pieces w, w+8 of every step (4 per wave, so
  // every vmcnt count is a constant); lane -> (row lane >> 2 of the piece's 16, physical chunk
  // lane & 3), source chunk swizzled. 224-row tiles have 14 X pieces: the slots of pieces 14 and
  // 15 re-load piece 13 into its own place (identical bytes).
  const int prow = lane >> 2;
  const int lchunk = (lane & 3) ^ ((4 - ((lane >> 4) & 3)) & 3);
  uint32_t xo[2], wo[2], xoe[2], woe[2];
  int xdst[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int pc = min(wv + 8 * j, XP - 1);
    xdst[j] = pc * 1024;
    const int xr = min(m0 + pc * 16 + prow, p.M - 1) - m0;
    const int wr = min(n0 + (wv + 8 * j) * 16 + prow, p.N - 1) - n0;
    xo[j] = (uint32_t)(((int64_t)xr * p.lda + lchunk * 8) * 2);
    wo[j] = (uint32_t)(((int64_t)wr * p.ldw + lchunk * 8) * 2);
    xoe[j] = p.K2 ? (uint32_t)(((int64_t)xr * p.lda2 + lchunk * 8) * 2) : xo[j];
    woe[j] = p.K2 ? (uint32_t)(((int64_t)wr * p.ldw2 + lchunk * 8) * 2) : wo[j];
  }
  const char* xb = (const char*)p.A + (int64_t)m0 * p.lda * 2;
  const char* wb = (const char*)p.W + (int64_t)n0 * p.ldw * 2;
  const char* xbe = p.K2 ? (const char*)p.A2 + (int64_t)m0 * p.lda2 * 2 : xb;
  const char* wbe = p.K2 ? (const char*)p.W2 + (int64_t)n0 * p.ldw2 * 2 : wb;
  const uint32_t lds0 = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) char*)smem);
  auto glds = [&](uint32_t voff, const char* sbase, uint32_t lds) {
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(voff), "s"(sbase), "s"(lds) : "memory");
  };
  // DMA piece g (0, 1: X; 2, 3: W) of K-step kt into ring slot `slot`; the K-extension steps
  // (LoRA) come after the nk_main main steps
  auto dma = [&](int kt, int slot, int g) {
    const bool ext = kt >= nk_main;
    const int kk = ext ? kt - nk_main : kt;
    const uint32_t st = lds0 + (uint32_t)((slot % NS_SLOTS) * SB);
    if (g < 2)
      glds(ext ? xoe[g] : xo[g], (ext ? xbe : xb) + kk * (NS_BKS * 2), st + xdst[g]);
    else
      glds(ext ? woe[g - 2] : wo[g - 2], (ext ? wbe : wb) + kk * (NS_BKS * 2), st + XB + (wv + 8 * (g - 2)) * 1024);
  };

  // ---- fragment reads: lane -> row lane & 15 of a 16-row fragment, k-chunk lane >> 4
  const int wm = wv / WNW, wn = wv % WNW;
  const int fsw = (((lane >> 4) ^ ((4 - ((lane >> 2) & 3)) & 3)) * 16);
  const int xrd = (wm * WTM + (lane & 15)) * 64 + fsw;
  const int wrd = XB + (wn * WTN + (lane & 15)) * 64 + fsw;

  f32x4 acc[NF][MF];
#pragma unroll
  for (int i = 0; i < NF; ++i)
#pragma unroll
    for (int j = 0; j < MF; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  s16x8 xa[MF], wa[NF], xn[MF], wn_[NF];

  // prologue: steps 0, 1, 2 in flight; wait for step 0 (own pieces, then the barrier); read it
#pragma unroll
  for (int t = 0; t < 3; ++t)
#pragma unroll
    for (int g = 0; g < 4; ++g) dma(min(t, nk - 1), t, g);
  asm volatile("s_waitcnt vmcnt(8)\n\ts_barrier" ::: "memory");
#pragma unroll
  for (int i = 0; i < NF; ++i) wa[i] = *(const s16x8*)(smem + wrd + i * 1024);
#pragma unroll
  for (int j = 0; j < MF; ++j) xa[j] = *(const s16x8*)(smem + xrd + j * 1024);
  if (wv >= 4) __builtin_amdgcn_s_setprio(1);

  // one K-step on fragments (cx, cw) while reading step t+1's into (nx, nw). The MFMAs go in NF
  // groups of MF (one W fragment against the wave's X fragments); the 4 DMA pieces of step t+3
  // and the NF + MF fragment reads are spread over the groups. nk is even (K, K2 multiples of
  // 64): the loop runs pairs with static register sets; past the last step the DMA re-loads step
  // nk-1 into the free slot and the reads fill dead registers (constant counts, no branches on
  // data).
  auto body = [&](int t, s16x8 (&cx)[MF], s16x8 (&cw)[NF], s16x8 (&nx)[MF], s16x8 (&nw)[NF]) {
    // step t+1 landed (steps t+2, t+3 may be in flight: 8 pieces), slot of step t-1 free
    asm volatile("s_waitcnt vmcnt(4)\n\ts_barrier" ::: "memory");
    const int kd = min(t + 3, nk - 1);
    const char* nst = smem + ((t + 1) % NS_SLOTS) * SB;
#pragma unroll
    for (int i = 0; i < NF; ++i) {
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int j = 0; j < MF; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(cw[i], cx[j], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
      constexpr int DEV = NF / 4;  // a DMA piece every NF/4 groups
      if (i % DEV == 0) dma(kd, t + 3, i / DEV);
      nw[i] = *(const s16x8*)(nst + wrd + i * 1024);
#pragma unroll
      for (int j = (i * MF) / NF; j < ((i + 1) * MF) / NF; ++j) nx[j] = *(const s16x8*)(nst + xrd + j * 1024);
    }
  };
  for (int t = 0; t < nk; t += 2) {
    body(t, xa, wa, xn, wn_);
    body(t + 1, xn, wn_, xa, wa);
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");

  // ---- epilogue: bf16(acc + bias) -> LDS image [BMT m][256 n], then the fused epilogue
  // row-contiguous, 8 columns (16 B) per thread
  char* cimg = smem;
#pragma unroll
  for (int i = 0; i < NF; ++i) {
    const int nl = wn * WTN + i * 16 + (lane >> 4) * 4;
    float b4[4] = {0.f, 0.f, 0.f, 0.f};
    if (p.bias) {
      const int gn = n0 + nl;
      if (gn + 3 < p.N) {
        const u32x2 bb = *(const u32x2*)(p.bias + gn);
        b4[0] = bf2f((bf16_t)bb[0]); b4[1] = bf2f((bf16_t)(bb[0] >> 16));
        b4[2] = bf2f((bf16_t)bb[1]); b4[3] = bf2f((bf16_t)(bb[1] >> 16));
      }
    }
#pragma unroll
    for (int j = 0; j < MF; ++j) {
      const int ml = wm * WTM + j * 16 + (lane & 15);
      u32x2 pk;
      pk[0] = pack2(acc[i][j][0] + b4[0], acc[i][j][1] + b4[1]);
      pk[1] = pack2(acc[i][j][2] + b4[2], acc[i][j][3] + b4[3]);
      *(u32x2*)(cimg + ml * C_STRIDE2 + nl * 2) = pk;
    }
  }
  __syncthreads();
  const int cgrp = tid & 31;
  for (int rr = tid >> 5; rr < BMT; rr += 512 / 32) {
    const int m = m0 + rr;
    const int n = n0 + cgrp * 8;
    if (m >= p.M || n >= p.N) continue;
    const u32x2 lo = *(const u32x2*)(cimg + rr * C_STRIDE2 + cgrp * 16);
    const u32x2 hi = *(const u32x2*)(cimg + rr * C_STRIDE2 + cgrp * 16 + 8);
    bf16_t cv[8] = {(bf16_t)lo[0], (bf16_t)(lo[0] >> 16), (bf16_t)lo[1], (bf16_t)(lo[1] >> 16),
                    (bf16_t)hi[0], (bf16_t)(hi[0] >> 16), (bf16_t)hi[1], (bf16_t)(hi[1] >> 16)};
    float o[8];
    epilogue_row8<EPI, R>(p, m, n, cv, o);
    u32x4 pk;
    pk[0] = pack2(o[0], o[1]);
    pk[1] = pack2(o[2], o[3]);
    pk[2] = pack2(o[4], o[5]);
    pk[3] = pack2(o[6], o[7]);
    *(u32x4*)(p.C + (int64_t)m * p.ldc + n) = pk;
  }
}

template <int EPI, int R, int BMT>
static int launch_ns_t(const GemmParams& p, hipStream_t s) {
  static bool set = false;
  if (!set) {
    (void)hipFuncSetAttribute((const void*)gemm_ns_kernel<EPI, R, BMT>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              ns_lds_bytes(BMT));
    set = true;
  }
  const unsigned tiles = (unsigned)(((p.M + BMT - 1) / BMT) * ((p.N + 255) / 256));
  hipLaunchKernelGGL((gemm_ns_kernel<EPI, R, BMT>), dim3(tiles), dim3(512), ns_lds_bytes(BMT), s, p);
  LTX_LAUNCH_CHECK();
  return LTX_OK;
}

template <int EPI, int R>
static int launch_ns_h(int bmt, const GemmParams& p, hipStream_t s) {
  return bmt == 224 ? launch_ns_t<EPI, R, 224>(p, s) : launch_ns_t<EPI, R, 256>(p, s);
}

template <int EPI>
static int launch_ns_r(int bmt, const GemmParams& p, hipStream_t s) {
  switch (p.rank) {
    case 8: return launch_ns_h<EPI, 8>(bmt, p, s);
    case 16: return launch_ns_h<EPI, 16>(bmt, p, s);
    case 32: return launch_ns_h<EPI, 32>(bmt, p, s);
    default: return fail(LTX_ERR_BAD_ARG, "gemm lora: rank must be 8, 16 or 32");
  }
}

int launch_ns(int epi, int bmt, const GemmParams& p, hipStream_t s) {
  switch (epi) {
    case LTX_EPI_STORE: return launch_ns_h<LTX_EPI_STORE, 0>(bmt, p, s);
    case LTX_EPI_GELU: return launch_ns_h<LTX_EPI_GELU, 0>(bmt, p, s);
    case LTX_EPI_GATED_RESIDUAL: return launch_ns_h<LTX_EPI_GATED_RESIDUAL, 0>(bmt, p, s);
    case LTX_EPI_GELU_BWD: return launch_ns_h<LTX_EPI_GELU_BWD, 0>(bmt, p, s);
    case LTX_EPI_ACCUM: return launch_ns_h<LTX_EPI_ACCUM, 0>(bmt, p, s);
    case LTX_EPI_LORA: return launch_ns_r<LTX_EPI_LORA>(bmt, p, s);
    case LTX_EPI_LORA_RESIDUAL: return launch_ns_r<LTX_EPI_LORA_RESIDUAL>(bmt, p, s);
    case LTX_EPI_LORA_DGRAD_ACCUM: return launch_ns_r<LTX_EPI_LORA_DGRAD_ACCUM>(bmt, p, s);
    default: return fail(LTX_ERR_BAD_ARG, "gemm: unknown epilogue");
  }
}

}  // namespace ltx
