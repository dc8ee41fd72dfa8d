// NOT BUILT (tools/experiments): measured and not adopted in round 3. Bitwise equal to
// gemm_nt_kernel_t on every training shape (7 shapes x 5 epilogues, K-extension and grouped
// K-extension), but 1-4 % slower (tools/bench_gemm.py, interleaved: e.g. FF-up 1131 vs 1167 TF,
// FF-down 1209 vs 1258 TF; hipBLASLt 1431 / 1481 TF on the same operands). Each wave's two DMA
// pieces per phase (~150 cycles of issue each among ds_reads) make the load segment longer than
// the partner group's 16-MFMA segment, so the matrix pipe idles at every barrier pair.
// Ping-pong variant of the large-tile bf16 GEMM (C = epi(A . W^T), same fused epilogues and same
// results bit for bit as gemm_nt_kernel_t: every accumulator takes its K in the same 32-deep
// steps, in the same order).
//
// Why: in gemm_nt_kernel_t all 8 waves issue their LDS-DMA pieces at the same program points, so
// both waves of a SIMD stall on DMA issue together and the matrix pipe idles (measured: the main
// loop runs 1.56-1.65 PF with the DMA removed vs 1.1-1.2 PF with it). Here the two wave groups
// (waves 0-3 and 4-7, one of each per SIMD) run one barrier apart: while one group issues its
// LDS reads and DMA pieces, the other runs its MFMAs (cdna_hip_programming.md: the 256^2 8-phase
// template, T3+T4, and MI355X_MICROARCH.md "Two waves per SIMD").
//
// Tile BMT (256 | 224) x 256, BK = 64, split into two k-halves of 32. LDS holds two K-tiles; a
// K-tile is four 'half-tiles' [X_s0 | X_s1 | W_s0 | W_s1] (rows x 32 k, 64-B rows; 1-KiB DMA
// pieces of 16 rows; 16-B chunk swizzle c ^ g((row >> 2) & 3), g = {0,2,3,1}, on the DMA source
// address and on the read: conflict-free for the 16x16x32 fragment reads).
// Wave (grp, c) owns rows grp*BMT/2 .. +BMT/2 and columns c*64 .. +64 of the tile (MF x 4
// fragments). Four phases per K-tile, phase (s, nq): [load: X frags of k-half s (nq == 0),
// 2 W frags, the next K-tile's half-tile `phase` as 2 DMA pieces] barrier [2 x MF MFMAs]
// barrier; group 1 starts one barrier late, so its loads run beside group 0's MFMAs.
// Hazards (phase k = 4t + ph; half-tile h of tile t+1 is issued in phase (t, h) and first read in
// phase (t+1, 0) or (t+1, 2), 3 or 4 phases later): each wave waits vmcnt(2) (its own pieces
// issued two or more phases ago; vmcnt(0) in the last K-tile, which issues nothing) at the start
// of every phase, and a barrier separates that wait from every read (RAW); a slot is re-issued 4
// phases after its last read (WAR).
#include "common.h"
#include "gemm_common.h"
#include "ltx_hip.h"

namespace ltx {

// chunk swizzle of a 64-B LDS row: g((row >> 2) & 3), g = {0, 2, 3, 1}
__device__ __forceinline__ int pp_swz(int row) { return (0x1320 >> (4 * ((row >> 2) & 3))) & 3; }

template <int EPI, int R, int BMT>
__global__ __launch_bounds__(512, 1) void gemm_pp_kernel(const GemmParams p) {
  static_assert(BMT == 256 || BMT == 224, "tile height");
  constexpr int MF = BMT / 32;        // m-fragments per wave (8 | 7)
  constexpr int NF = 4;               // n-fragments per wave (64 columns)
  constexpr int XH = BMT * 64;        // bytes of one X half-tile (BMT rows x 32 k)
  constexpr int WH = 256 * 64;        // bytes of one W half-tile
  constexpr int BUF = 2 * XH + 2 * WH;
  constexpr int XP = BMT / 16;        // 1-KiB pieces per X half-tile (16 | 14)
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = wave >> 2, c = wave & 3;
  const int ntm = (p.M + BMT - 1) / BMT, ntn = (p.N + 255) / 256;
  int tm, tn;
  block_to_tile(blockIdx.x, ntm, ntn, tm, tn);
  const int m0 = tm * BMT, n0 = tn * 256;
  const int nk_main = p.K / 64;
  const int nk = nk_main + p.K2 / 64;

  // ---- DMA: this wave's two pieces of every half-tile (X: clamped, the last piece repeats when
  // BMT = 224 so every wave issues exactly two per phase and the vmcnt count is uniform). Lane
  // offsets and scalar bases of the main and the K-extension operands are computed once.
  const int lr = lane >> 2, pch = lane & 3;
  int xpc[2], wpc[2];
  uint32_t xo[2][2], wo[2][2];  // [main | ext][piece]
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    xpc[i] = min(2 * wave + i, XP - 1);
    wpc[i] = 2 * wave + i;
  }
#pragma unroll
  for (int e = 0; e < 2; ++e) {
    const int64_t lx = e ? p.lda2 : p.lda, lw = e ? p.ldw2 : p.ldw;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int rx = xpc[i] * 16 + lr, rw = wpc[i] * 16 + lr;
      xo[e][i] = (uint32_t)(((int64_t)(min(m0 + rx, p.M - 1) - m0) * lx + ((pch ^ pp_swz(rx)) * 8)) * 2);
      wo[e][i] = (uint32_t)(((int64_t)(min(n0 + rw, p.N - 1) - n0) * lw + ((pch ^ pp_swz(rw)) * 8)) * 2);
    }
  }
  const char* xb0 = (const char*)p.A + (int64_t)m0 * p.lda * 2;
  const char* wb0 = (const char*)p.W + (int64_t)n0 * p.ldw * 2;
  const char* xb1 = nk > nk_main ? (const char*)ext_a2(p, n0) + (int64_t)m0 * p.lda2 * 2 : xb0;
  const char* wb1 = nk > nk_main ? (const char*)p.W2 + (int64_t)n0 * p.ldw2 * 2 : wb0;
  const uint32_t lds0 = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) char*)smem);
  auto glds2 = [&](uint32_t v0, uint32_t v1, const char* sbase, uint32_t l0, uint32_t l1) {
    unsigned keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %4\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %3\n\t"
        "s_mov_b32 m0, %5\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %2, %3\n\ts_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(v0), "v"(v1), "s"(sbase), "s"(l0), "s"(l1)
        : "memory");
  };
  // slot byte offset of half-tile h (0: X_s0, 1: W_s0, 2: X_s1, 3: W_s1) in buffer b
  auto slot = [](int b, int h) -> int {
    return b * BUF + ((h & 1) ? 2 * XH + (h >> 1) * WH : (h >> 1) * XH);
  };
  // issue half-tile h of K-tile kt (its K-extension tiles after the main ones)
  auto issue = [&](int kt, int h) {
    const bool ext = kt >= nk_main;                                           // wave-uniform
    const int kk = (ext ? kt - nk_main : kt) * 128 + (h >> 1) * 64;           // bytes along K
    const uint32_t l = lds0 + slot(kt & 1, h);
    if (h & 1)
      glds2(ext ? wo[1][0] : wo[0][0], ext ? wo[1][1] : wo[0][1], (ext ? wb1 : wb0) + kk, l + wpc[0] * 1024,
            l + wpc[1] * 1024);
    else
      glds2(ext ? xo[1][0] : xo[0][0], ext ? xo[1][1] : xo[0][1], (ext ? xb1 : xb0) + kk, l + xpc[0] * 1024,
            l + xpc[1] * 1024);
  };

  f32x4 acc[NF][MF];
#pragma unroll
  for (int i = 0; i < NF; ++i)
#pragma unroll
    for (int j = 0; j < MF; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  // fragment read: row (lane & 15) of a 16-row block, k-chunk (lane >> 4), swizzled
  const int laneoff = (lane & 15) * 64 + (((lane >> 4) ^ pp_swz(lane & 15)) << 4);
  const int xrow0 = grp * (BMT / 2), wrow0 = c * 64;

  // prologue: K-tile 0, its first k-half waited for
  issue(0, 0);
  issue(0, 1);
  issue(0, 2);
  issue(0, 3);
  asm volatile("s_waitcnt vmcnt(4)\n\ts_barrier" ::: "memory");
  if (grp == 1) asm volatile("s_barrier" ::: "memory");  // the stagger

  s16x8 xf[MF], wf[2];
  for (int kt = 0; kt < nk; ++kt) {
    const int b = kt & 1;
#pragma unroll
    for (int ph = 0; ph < 4; ++ph) {
      const int s = ph >> 1, nq = ph & 1;
      // own pieces issued two or more phases ago have landed; in the last K-tile nothing new is
      // issued, so everything is waited for; in phase 0 of K-tile 0 the prologue's second k-half
      // (needed two phases later) may stay in flight
      if (kt + 1 >= nk)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      else if (kt == 0 && ph == 0)
        asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      else
        asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
      if (nq == 0) {
        const char* xs = smem + slot(b, 2 * s) + xrow0 * 64 + laneoff;
#pragma unroll
        for (int j = 0; j < MF; ++j) xf[j] = *(const s16x8*)(xs + j * 1024);
      }
      const char* ws = smem + slot(b, 2 * s + 1) + (wrow0 + nq * 32) * 64 + laneoff;
      wf[0] = *(const s16x8*)ws;
      wf[1] = *(const s16x8*)(ws + 1024);
      if (kt + 1 < nk) issue(kt + 1, ph);
      asm volatile("s_barrier" ::: "memory");
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < MF; ++j)
          acc[nq * 2 + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[i], xf[j], acc[nq * 2 + i][j], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
      asm volatile("s_barrier" ::: "memory");
    }
  }
  if (grp == 0) asm volatile("s_barrier" ::: "memory");  // barrier counts match again
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");

  // ---- epilogue (as gemm_nt_kernel_t): bf16(acc + bias) -> LDS image [BMT m][256 n], then a
  // row-contiguous pass applying the fused epilogue with 16-B accesses
  constexpr int WTM = BMT / 2, WTN = 64, NT = 512;
  char* cimg = smem;
  u32x2 bias2[NF];
#pragma unroll
  for (int i = 0; i < NF; ++i) {
    bias2[i] = (u32x2){0u, 0u};
    const int gn = n0 + c * WTN + i * 16 + (lane >> 4) * 4;
    if (p.bias && gn + 3 < p.N) bias2[i] = *(const u32x2*)(p.bias + gn);
  }
#pragma unroll
  for (int i = 0; i < NF; ++i) {
    const int nl = c * WTN + i * 16 + (lane >> 4) * 4;
    const u32x2 bb = bias2[i];
    const float b4[4] = {bf2f((bf16_t)bb[0]), bf2f((bf16_t)(bb[0] >> 16)), bf2f((bf16_t)bb[1]),
                         bf2f((bf16_t)(bb[1] >> 16))};
#pragma unroll
    for (int j = 0; j < MF; ++j) {
      const int ml = grp * WTM + j * 16 + (lane & 15);
      u32x2 pk;
      pk[0] = pack2(acc[i][j][0] + b4[0], acc[i][j][1] + b4[1]);
      pk[1] = pack2(acc[i][j][2] + b4[2], acc[i][j][3] + b4[3]);
      *(u32x2*)(cimg + ml * C_STRIDE2 + nl * 2) = pk;
    }
  }
  const int cgrp = tid & 31;
  constexpr int RPP = NT / 32, NPASS = BMT / RPP;
  constexpr bool BATCH = epi_has_aux<EPI>();
  auto row_out = [&](int rr, const EpiAux* pre) {
    const int m = m0 + rr;
    const int n = n0 + cgrp * 8;
    if (m >= p.M || n >= p.N) return;
    const u32x2 lo = *(const u32x2*)(cimg + rr * C_STRIDE2 + cgrp * 16);
    const u32x2 hi = *(const u32x2*)(cimg + rr * C_STRIDE2 + cgrp * 16 + 8);
    bf16_t cv[8] = {(bf16_t)lo[0], (bf16_t)(lo[0] >> 16), (bf16_t)lo[1], (bf16_t)(lo[1] >> 16),
                    (bf16_t)hi[0], (bf16_t)(hi[0] >> 16), (bf16_t)hi[1], (bf16_t)(hi[1] >> 16)};
    float o[8];
    epilogue_row8<EPI, R>(p, m, n, cv, o, pre);
    u32x4 pk;
    pk[0] = pack2(o[0], o[1]);
    pk[1] = pack2(o[2], o[3]);
    pk[2] = pack2(o[4], o[5]);
    pk[3] = pack2(o[6], o[7]);
    *(u32x4*)(p.C + (int64_t)m * p.ldc + n) = pk;
  };
  if (BATCH) {
    EpiAux ax[BATCH ? NPASS : 1];
#pragma unroll
    for (int u = 0; u < NPASS; ++u)
      epi_load<EPI>(p, min(m0 + (tid >> 5) + u * RPP, p.M - 1), min(n0 + cgrp * 8, p.N - 8), ax[u]);
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
#pragma unroll
    for (int u = 0; u < NPASS; ++u) row_out((tid >> 5) + u * RPP, &ax[u]);
  } else {
    __syncthreads();
    for (int rr = tid >> 5; rr < BMT; rr += RPP) row_out(rr, nullptr);
  }
}

template <int BMT>
constexpr int pp_lds_bytes() {
  constexpr int bufs = 2 * (2 * BMT * 64 + 2 * 256 * 64);
  constexpr int img = BMT * C_STRIDE2;
  return bufs > img ? bufs : img;
}

template <int EPI, int R, int BMT>
static int launch_pp_t(const GemmParams& p, hipStream_t s) {
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)gemm_pp_kernel<EPI, R, BMT>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              pp_lds_bytes<BMT>());
    attr = true;
  }
  const int64_t tiles = (int64_t)((p.M + BMT - 1) / BMT) * ((p.N + 255) / 256);
  hipLaunchKernelGGL((gemm_pp_kernel<EPI, R, BMT>), dim3((unsigned)tiles), dim3(512), pp_lds_bytes<BMT>(), s, p);
  LTX_LAUNCH_CHECK();
  return LTX_OK;
}

template <int EPI, int R>
static int launch_pp_r(int bmt, const GemmParams& p, hipStream_t s) {
  return bmt == 224 ? launch_pp_t<EPI, R, 224>(p, s) : launch_pp_t<EPI, R, 256>(p, s);
}

template <int EPI>
static int launch_pp_lora(int R, int bmt, const GemmParams& p, hipStream_t s) {
  switch (R) {
    case 8: return launch_pp_r<EPI, 8>(bmt, p, s);
    case 16: return launch_pp_r<EPI, 16>(bmt, p, s);
    case 32: return launch_pp_r<EPI, 32>(bmt, p, s);
    default: return fail(LTX_ERR_BAD_ARG, "gemm pp: rank must be 8, 16 or 32");
  }
}

int launch_pp(int epi, int R, int bmt, const GemmParams& p, hipStream_t s) {
  switch (epi) {
    case LTX_EPI_STORE: return launch_pp_r<LTX_EPI_STORE, 0>(bmt, p, s);
    case LTX_EPI_GELU: return launch_pp_r<LTX_EPI_GELU, 0>(bmt, p, s);
    case LTX_EPI_GATED_RESIDUAL: return launch_pp_r<LTX_EPI_GATED_RESIDUAL, 0>(bmt, p, s);
    case LTX_EPI_GELU_BWD: return launch_pp_r<LTX_EPI_GELU_BWD, 0>(bmt, p, s);
    case LTX_EPI_ACCUM: return launch_pp_r<LTX_EPI_ACCUM, 0>(bmt, p, s);
    case LTX_EPI_STORE_ROWDOT: return launch_pp_r<LTX_EPI_STORE_ROWDOT, 0>(bmt, p, s);
    case LTX_EPI_LORA: return launch_pp_lora<LTX_EPI_LORA>(R, bmt, p, s);
    case LTX_EPI_LORA_RESIDUAL: return launch_pp_lora<LTX_EPI_LORA_RESIDUAL>(R, bmt, p, s);
    case LTX_EPI_LORA_DGRAD_ACCUM: return launch_pp_lora<LTX_EPI_LORA_DGRAD_ACCUM>(R, bmt, p, s);
    default: return fail(LTX_ERR_BAD_ARG, "gemm pp: unknown epilogue");
  }
}

}  // namespace ltx
