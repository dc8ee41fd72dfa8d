// One-wave-per-SIMD bf16 GEMM (C[M,N] = epi(A[M,K] . W[N,K]^T)) for the large training shapes.
#include <type_traits>

#include "gemm_common.h"

namespace ltx {

// ---------------------------------------------------------------------------------------------
// One-wave-per-SIMD large-tile kernel (w4): 256 threads = 4 waves as 2 (m) x 2 (n). Each wave owns
// a (BMT/2) x 128 piece of the BMT x 256 output tile as MF x 8 fragments of
// v_mfma_f32_16x16x32_bf16 (MF*32 accumulator registers: 256 at BMT = 256, which one wave per SIMD
// can hold in the unified 512-register file). One wave per SIMD reads a third fewer fragment bytes
// from LDS per MFMA than 8 waves of 64 x 128, and nothing shares its matrix pipe.
// K advances in 32-deep stages (X [BMT][32] + W [256][32] bf16, 64-B rows whose 16-B chunks are
// XOR-swizzled by (-(row >> 2)) & 3 -- conflict-free for the 16x16x32 fragment reads, applied to
// the DMA source address: the LDS-DMA image is lane-linear) through a W4_NS-deep LDS ring filled
// by LDS-DMA (global_load_lds_dwordx4, one 16-row x 64-B piece per wave-instruction) W4_NS - 2
// stages ahead of the MFMAs. Per stage: one counted vmcnt + s_barrier (stage t+1 landed for every
// wave, stage t-1 free), then 8 groups of MF MFMAs on stage t's fragments (registers), each
// followed by one DMA piece of stage t+W4_NS-1 and the ds_reads of stage t+1's fragments into the
// other register set, so LDS latency hides under a whole stage of MFMAs.
// ---------------------------------------------------------------------------------------------
constexpr int W4_BKS = 32;
constexpr int W4_NS = 4;
constexpr int w4_lds_bytes(int bmt) {
  return (W4_NS * (bmt + 256) * W4_BKS * 2 > bmt * C_STRIDE2) ? W4_NS * (bmt + 256) * W4_BKS * 2
                                                               : bmt * C_STRIDE2;
}

// epilogue of the w4 kernels: bf16(acc + bias) -> LDS image [BMT m][256 n], then the fused
// epilogue row-contiguous, 8 columns per thread, 32 threads per row
template <int EPI, int R, int BMT>
__device__ __forceinline__ void w4_epilogue(const GemmParams& p, const f32x4 (&acc)[8][BMT / 32], char* smem,
                                            int tid, int m0, int n0, int wm, int wn) {
  constexpr int NF = 8, MF = BMT / 32;
  const int lane = tid & 63;
  char* cimg = smem;
#pragma unroll
  for (int i = 0; i < NF; ++i) {
    const int nl = wn * 128 + i * 16 + (lane >> 4) * 4;
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
      const int ml = wm * (BMT / 2) + j * 16 + (lane & 15);
      u32x2 pk;
      pk[0] = pack2(acc[i][j][0] + b4[0], acc[i][j][1] + b4[1]);
      pk[1] = pack2(acc[i][j][2] + b4[2], acc[i][j][3] + b4[3]);
      *(u32x2*)(cimg + ml * C_STRIDE2 + nl * 2) = pk;
    }
  }
  __syncthreads();
  // ---- epilogue stage 2: row-contiguous, 8 columns per thread, 32 threads per row
  const int cgrp = tid & 31;
  for (int rr = tid >> 5; rr < BMT; rr += 256 / 32) {
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

template <int EPI, int R, int BMT, int VAR = 0>
__global__ __launch_bounds__(256, 1) void gemm_w4_kernel(const GemmParams p) {
  // VAR (measurement only, wrong results): bit 0 no DMA past the prologue, bit 1 no barrier in the loop
  constexpr bool NODMA = (VAR & 1) != 0, NOBAR = (VAR & 2) != 0;
  constexpr bool FULLLINE = (VAR & 4) != 0;  // DMA pieces read 8 rows x 128 B (same bytes, full lines)
  constexpr bool SAMEBYTES = (VAR & 8) != 0; // every DMA reads the same 1 KiB (issue cost only)
  static_assert(BMT == 256 || BMT == 224, "tile height");
  constexpr int MF = BMT / 32;               // m-fragments per wave: 8 | 7
  constexpr int NF = 8;                      // n-fragments per wave (128 columns)
  constexpr int XB = BMT * W4_BKS * 2;       // X bytes per stage
  constexpr int SB = XB + 256 * W4_BKS * 2;  // stage bytes
  constexpr int XP = BMT / 16;               // X pieces per stage: 16 | 14
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ntm = (p.M + BMT - 1) / BMT, ntn = (p.N + 255) / 256;
  int tm, tn;
  block_to_tile(blockIdx.x, ntm, ntn, tm, tn);
  const int m0 = tm * BMT, n0 = tn * 256;
  const int nk_main = p.K / W4_BKS;
  const int nk = nk_main + p.K2 / W4_BKS;

  // ---- LDS-DMA: wave w moves X pieces w, w+4, w+8, w+12 and W pieces w, w+4, w+8, w+12 (8 per
  // stage for every wave, so every count is a constant); lane -> (row lane >> 2 of the piece's 16,
  // physical chunk lane & 3), source chunk swizzled. With 224-row tiles (14 X pieces) the slots of
  // pieces 14 and 15 re-load piece 13 into its own place (identical bytes, +2 KiB per 30 KiB stage).
  const int prow = lane >> 2;
  const int lchunk = (lane & 3) ^ ((4 - ((lane >> 4) & 3)) & 3);
  uint32_t xo[4], wo[4], xoe[4], woe[4];
  int xdst[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int pc = min(wv + 4 * j, XP - 1);
    xdst[j] = pc * 1024;
    const int xr = min(m0 + pc * 16 + prow, p.M - 1) - m0;
    const int wr = min(n0 + (wv + 4 * j) * 16 + prow, p.N - 1) - n0;
    xo[j] = (uint32_t)(((int64_t)xr * p.lda + lchunk * 8) * 2);
    wo[j] = (uint32_t)(((int64_t)wr * p.ldw + lchunk * 8) * 2);
    if constexpr (FULLLINE) {
      xo[j] = (uint32_t)(((int64_t)(pc * 8 + (lane >> 3)) * p.lda + (lane & 7) * 8) * 2);
      wo[j] = (uint32_t)(((int64_t)((wv + 4 * j) * 8 + (lane >> 3)) * p.ldw + (lane & 7) * 8) * 2);
    }
    if constexpr (SAMEBYTES) xo[j] = wo[j] = (uint32_t)(lane * 16);
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
  // DMA slot g (0..7) of K-stage kt into ring slot `slot`: slots 0-3 the X pieces, 4-7 the W pieces;
  // the K-extension stages (LoRA) come after the nk_main main stages
  auto dma = [&](int kt, int slot, int g) {
    const bool ext = kt >= nk_main;
    const int kk = SAMEBYTES ? 0 : (FULLLINE ? (ext ? kt - nk_main : kt) / 2 : (ext ? kt - nk_main : kt));
    const uint32_t st = lds0 + (uint32_t)((slot % W4_NS) * SB);
    if (g < 4) {
      glds(ext ? xoe[g & 3] : xo[g & 3], (ext ? xbe : xb) + kk * (W4_BKS * 2), st + xdst[g & 3]);
    } else {
      glds(ext ? woe[g & 3] : wo[g & 3], (ext ? wbe : wb) + kk * (W4_BKS * 2), st + XB + (wv + 4 * (g - 4)) * 1024);
    }
  };
  // this wave's DMA of all but the `S` youngest stages done, then the workgroup barrier
  auto wait_pend = [&](auto S) {
    if constexpr (NOBAR && decltype(S)::value == W4_NS - 3) return;
    if constexpr (NODMA && decltype(S)::value == W4_NS - 3) asm volatile("s_barrier" ::: "memory");
    else if constexpr (decltype(S)::value == 0) asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
    else if constexpr (decltype(S)::value == 1) asm volatile("s_waitcnt vmcnt(8)\n\ts_barrier" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(16)\n\ts_barrier" ::: "memory");
  };

  // ---- fragment reads: lane -> row lane & 15 of a 16-row fragment, k-chunk lane >> 4
  const int wm = wv >> 1, wn = wv & 1;
  const int fsw = (((lane >> 4) ^ ((4 - ((lane >> 2) & 3)) & 3)) * 16);
  const int xrd = (wm * (BMT / 2) + (lane & 15)) * 64 + fsw;
  const int wrd = XB + (wn * 128 + (lane & 15)) * 64 + fsw;

  f32x4 acc[NF][MF];
#pragma unroll
  for (int i = 0; i < NF; ++i)
#pragma unroll
    for (int j = 0; j < MF; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  s16x8 xf[MF], wfa[NF], wfb[NF];

  // prologue: stages 0 .. NS-2 in flight, wait for stage 0, read its fragments
#pragma unroll
  for (int t = 0; t < W4_NS - 1; ++t) {
#pragma unroll
    for (int g = 0; g < 8; ++g) dma(min(t, nk - 1), t, g);
  }
  wait_pend(std::integral_constant<int, W4_NS - 2>{});
#pragma unroll
  for (int j = 0; j < MF; ++j) {  // the body's read order, so the loop header's waits stay counted
    if (j < 4) {
      wfa[2 * j] = *(const s16x8*)(smem + wrd + (2 * j) * 1024);
      wfa[2 * j + 1] = *(const s16x8*)(smem + wrd + (2 * j + 1) * 1024);
    }
    xf[j] = *(const s16x8*)(smem + xrd + j * 1024);
  }

  // one stage: MF groups of 8 MFMAs, group j = X fragment j against the 8 W fragments (cw). After
  // group j: X fragment j of stage t+1 is read in place, the next W fragments (nw) in groups 0-3,
  // and the DMA pieces of stage t+NS-1 (one per group, the rest after the last group). Every read
  // a group needs was issued a whole stage earlier. nk is even (K and K2 are multiples of 64), so
  // the loop runs whole pairs with static register sets; past the last stage the DMA re-loads
  // stage nk-1 into the free slot and the reads fill dead registers: no data-dependent branches.
  auto body = [&](int t, s16x8 (&cw)[NF], s16x8 (&nw)[NF]) {
    wait_pend(std::integral_constant<int, W4_NS - 3>{});
    const int kd = min(t + W4_NS - 1, nk - 1);
    const char* nst = smem + ((t + 1) % W4_NS) * SB;
#pragma unroll
    for (int j = 0; j < MF; ++j) {
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < NF; ++i) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(cw[i], xf[j], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (!NODMA) {
        dma(kd, t + W4_NS - 1, j);
        if (j == MF - 1)
#pragma unroll
          for (int g = MF; g < 8; ++g) dma(kd, t + W4_NS - 1, g);
      }
      if (j < 4) {
        nw[2 * j] = *(const s16x8*)(nst + wrd + (2 * j) * 1024);
        nw[2 * j + 1] = *(const s16x8*)(nst + wrd + (2 * j + 1) * 1024);
      }
      xf[j] = *(const s16x8*)(nst + xrd + j * 1024);
    }
  };
  for (int t = 0; t < nk; t += 2) {
    body(t, wfa, wfb);
    body(t + 1, wfb, wfa);
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");

  w4_epilogue<EPI, R, BMT>(p, acc, smem, tid, m0, n0, wm, wn);
}

template <int EPI, int R, int BMT, int VAR = 0>
static int launch_w4_t(const GemmParams& p, hipStream_t s) {
  static bool set = false;
  if (!set) {
    (void)hipFuncSetAttribute((const void*)gemm_w4_kernel<EPI, R, BMT, VAR>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              w4_lds_bytes(BMT));
    set = true;
  }
  const unsigned tiles = (unsigned)(((p.M + BMT - 1) / BMT) * ((p.N + 255) / 256));
  hipLaunchKernelGGL((gemm_w4_kernel<EPI, R, BMT, VAR>), dim3(tiles), dim3(256), w4_lds_bytes(BMT), s, p);
  LTX_LAUNCH_CHECK();
  return LTX_OK;
}

template <int EPI, int R>
static int launch_w4_h(int bmt, const GemmParams& p, hipStream_t s) {
  return bmt == 224 ? launch_w4_t<EPI, R, 224>(p, s) : launch_w4_t<EPI, R, 256>(p, s);
}

template <int EPI>
static int launch_w4_r(int bmt, const GemmParams& p, hipStream_t s) {
  switch (p.rank) {
    case 8: return launch_w4_h<EPI, 8>(bmt, p, s);
    case 16: return launch_w4_h<EPI, 16>(bmt, p, s);
    case 32: return launch_w4_h<EPI, 32>(bmt, p, s);
    default: return fail(LTX_ERR_BAD_ARG, "gemm lora: rank must be 8, 16 or 32");
  }
}

int launch_w4(int epi, int bmt, const GemmParams& p, hipStream_t s) {
  if (bmt < 0 && epi == LTX_EPI_STORE) {  // measurement-only variants (wrong results), 224-row tiles
    if (bmt == -1) return launch_w4_t<LTX_EPI_STORE, 0, 224, 1>(p, s);
    if (bmt == -3) return launch_w4_t<LTX_EPI_STORE, 0, 224, 4>(p, s);
    if (bmt == -4) return launch_w4_t<LTX_EPI_STORE, 0, 224, 8>(p, s);
    return launch_w4_t<LTX_EPI_STORE, 0, 224, 3>(p, s);
  }
#ifdef W4_PROBE
  return launch_w4_h<LTX_EPI_STORE, 0>(bmt, p, s);
#else
  switch (epi) {
    case LTX_EPI_STORE: return launch_w4_h<LTX_EPI_STORE, 0>(bmt, p, s);
    case LTX_EPI_GELU: return launch_w4_h<LTX_EPI_GELU, 0>(bmt, p, s);
    case LTX_EPI_GATED_RESIDUAL: return launch_w4_h<LTX_EPI_GATED_RESIDUAL, 0>(bmt, p, s);
    case LTX_EPI_GELU_BWD: return launch_w4_h<LTX_EPI_GELU_BWD, 0>(bmt, p, s);
    case LTX_EPI_ACCUM: return launch_w4_h<LTX_EPI_ACCUM, 0>(bmt, p, s);
    case LTX_EPI_LORA: return launch_w4_r<LTX_EPI_LORA>(bmt, p, s);
    case LTX_EPI_LORA_RESIDUAL: return launch_w4_r<LTX_EPI_LORA_RESIDUAL>(bmt, p, s);
    case LTX_EPI_LORA_DGRAD_ACCUM: return launch_w4_r<LTX_EPI_LORA_DGRAD_ACCUM>(bmt, p, s);
    default: return fail(LTX_ERR_BAD_ARG, "gemm: unknown epilogue");
  }
#endif
}

}  // namespace ltx
