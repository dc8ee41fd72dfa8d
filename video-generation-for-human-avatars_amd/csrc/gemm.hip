// bf16 MFMA GEMM for gfx950 with fused epilogues: C[M,N] = epi(A[M,K] . W[N,K]^T).
//
// Every dense contraction on the LTX-2B training step maps onto this one "NT" form:
//   forward   X[M,K] . W[N,K]^T          (nn.Linear: weights stored [out,in], K contiguous)
//   dgrad     dY[M,N] . (W^T)[K,N]^T     (frozen weights: the W^T copy is packed once at load)
//   wgrad     dY^T[N,M] . X^T[K,M]^T     (caption_projection only; operands transposed first)
//
// Tiling: 128x128 output tile, BK = 64, 256 threads = 4 waves in 2x2, each wave 64x64 as 4x4
// v_mfma_f32_16x16x32_bf16. The MFMA "A" operand is the W tile (rows n), the "B" operand the X
// tile (rows m), so each lane's accumulator holds 4 CONSECUTIVE n of one row m: the epilogue
// packs them into one 8-byte LDS store, and the row-contiguous pass then writes 16 B per lane.
// Staging: global_load_lds_dwordx4 (1 KiB per wave-instruction) into a 2-deep LDS ring; the
// image is lane-linear in LDS, so the XOR swizzle (16-B chunk ^= row & 7, conflict-free for the
// 16x16x32 fragment reads) is applied to the per-lane SOURCE address and to the ds_read address.
// Block order: XCD-aware (blocks b, b+8 share an XCD / L2) then grouped by 8 row-tiles.
#include <cstdio>
#include <cstdlib>
#include <map>
#include <mutex>

#include "common.h"
#include "ltx_hip.h"
#include "gemm_common.h"
#include "gemm_ring.h"

namespace ltx {

constexpr int WT2 = BN2 * BK * 2;  // W tile bytes of the 256-wide kernels (32 KiB)
constexpr int LDS2 = (2 * (BM2 + BN2) * BK * 2 > BM2 * C_STRIDE2) ? 2 * (BM2 + BN2) * BK * 2 : BM2 * C_STRIDE2;

// NST = LDS stages: 2 (one K-tile in flight while the other computes) or 3 / 4 (NST - 1 in
// flight; for grids of at most one workgroup per CU, whose few K-tiles per workgroup are
// load-latency-bound)
template <int EPI, int R, int NST = 2>
__global__ __launch_bounds__(GEMM_THREADS, 2) void gemm_nt_kernel(const GemmParams p) {
  static_assert(NST >= 2 && NST <= 4, "gemm_nt_kernel: 2 to 4 stages");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int ntm = (p.M + BM - 1) / BM, ntn = (p.N + BN - 1) / BN;
  const int split = blockIdx.x / (ntm * ntn);  // split-K slice (0 unless p.splitk > 1)
  int tm, tn;
  block_to_tile(blockIdx.x % (ntm * ntn), ntm, ntn, tm, tn);
  const int m0 = tm * BM, n0 = tn * BN;

  // ---- staging addresses: wave w loads 4 x 1 KiB (8 rows each) of the X tile and of the W tile
  // lane -> (row in 8-row group = lane>>3, physical chunk = lane&7); source chunk un-swizzled
  const int lrow = lane >> 3;
  const int pchunk = lane & 7;
  const bf16_t* asrc[4];
  const bf16_t* wsrc[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = (wave * 4 + i) * 8 + lrow;             // 0..127 within the tile
    const int lchunk = pchunk ^ (row & 7);
    const int am = min(m0 + row, p.M - 1);                  // clamp: rows past M are never stored
    const int wn = min(n0 + row, p.N - 1);
    asrc[i] = p.A + (int64_t)am * p.lda + lchunk * 8;
    wsrc[i] = p.W + (int64_t)wn * p.ldw + lchunk * 8;
  }
  const int nk_main = p.K / BK;
  auto stage = [&](int buf, int kt) {
    char* base = smem + buf * STAGE_BYTES;
    if (kt < nk_main) {
      const int koff = kt * BK;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        glds16(asrc[i] + koff, base + (wave * 4 + i) * 1024);
        glds16(wsrc[i] + koff, base + TILE_BYTES + (wave * 4 + i) * 1024);
      }
    } else {  // K extension tile(s)
      const int koff = (kt - nk_main) * BK;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = (wave * 4 + i) * 8 + lrow;
        const int lchunk = pchunk ^ (row & 7);
        glds16(ext_a2(p, n0) + (int64_t)min(m0 + row, p.M - 1) * p.lda2 + koff + lchunk * 8,
               base + (wave * 4 + i) * 1024);
        glds16(p.W2 + (int64_t)min(n0 + row, p.N - 1) * p.ldw2 + koff + lchunk * 8,
               base + TILE_BYTES + (wave * 4 + i) * 1024);
      }
    }
  };

  // wave (wm, wn) owns rows m: wm*64..+63 and cols n: wn*64..+63 of the tile
  const int wm = wave >> 1, wn = wave & 1;
  f32x4 acc[4][4];  // [n-subtile i][m-subtile j]
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const int nk_all = nk_main + p.K2 / BK;
  const int S = p.splitk > 1 ? p.splitk : 1;
  const int kt0 = (int)((int64_t)split * nk_all / S), nk = (int)((int64_t)(split + 1) * nk_all / S);
  stage(0, kt0);
  if constexpr (NST > 2) {
#pragma unroll
    for (int st = 1; st < NST - 1; ++st)
      if (kt0 + st < nk) stage(st, kt0 + st);
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  const int frow = lane & 15;   // fragment row within a 16-row subtile
  const int fchunk = lane >> 4;  // fragment k-chunk (8 elements) within a 32-deep k-step
  for (int kt = kt0; kt < nk; ++kt) {
    int cur;
    if constexpr (NST > 2) {
      // stages kt .. kt+NST-2 are in flight (8 direct-to-LDS loads per thread each): wait for
      // kt's, then the barrier also retires every wave's reads of the buffer stage kt+NST-1
      // overwrites (one asm statement with a raw s_barrier: __syncthreads' fence would wait for
      // vmcnt(0))
      cur = (kt - kt0) % NST;
      const int ahead = min(NST - 2, nk - 1 - kt);  // stages issued after kt
      if (ahead >= 2)
        asm volatile("s_waitcnt vmcnt(16) lgkmcnt(0)\n\ts_barrier" ::: "memory");
      else if (ahead == 1)
        asm volatile("s_waitcnt vmcnt(8) lgkmcnt(0)\n\ts_barrier" ::: "memory");
      else
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
      if (kt + NST - 1 < nk) stage((cur + NST - 1) % NST, kt + NST - 1);
    } else {
      cur = (kt - kt0) & 1;
      if (kt + 1 < nk) stage(cur ^ 1, kt + 1);
    }
    const char* xs = smem + cur * STAGE_BYTES;
    const char* ws = xs + TILE_BYTES;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      s16x8 af[4], bfr[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = wn * 64 + i * 16 + frow;
        af[i] = *(const s16x8*)(ws + swz(row, kk * 4 + fchunk));
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int row = wm * 64 + j * 16 + frow;
        bfr[j] = *(const s16x8*)(xs + swz(row, kk * 4 + fchunk));
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if constexpr (NST == 2) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
  }
  if constexpr (NST > 2) __syncthreads();  // the epilogue's C image reuses stage 0

  if (S > 1) {  // split-K: raw f32 partial, 4 consecutive n per lane (16-B stores)
    float* part = p.ws + (int64_t)split * p.M * p.N;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int n = n0 + wn * 64 + i * 16 + (lane >> 4) * 4;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int m = m0 + wm * 64 + j * 16 + (lane & 15);
        if (m < p.M && n < p.N) *(f32x4*)(part + (int64_t)m * p.N + n) = acc[i][j];
      }
    }
    return;
  }
  // ---- epilogue stage 1: bf16(acc + bias) -> LDS image [128 m][128 n] (row stride C_STRIDE)
  // lane holds C^T[n = i*16 + (lane>>4)*4 + r][m = j*16 + (lane&15)], r = 0..3
  char* cimg = smem;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int nl = wn * 64 + i * 16 + (lane >> 4) * 4;  // local n of register 0
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
    for (int j = 0; j < 4; ++j) {
      const int ml = wm * 64 + j * 16 + (lane & 15);
      u32x2 pk;
      pk[0] = pack2(acc[i][j][0] + b4[0], acc[i][j][1] + b4[1]);
      pk[1] = pack2(acc[i][j][2] + b4[2], acc[i][j][3] + b4[3]);
      *(u32x2*)(cimg + ml * C_STRIDE + nl * 2) = pk;
    }
  }
  __syncthreads();

  // ---- epilogue stage 2: row-contiguous, 8 columns (16 B) per thread, 16 threads per row
  const int cgrp = tid & 15;
  for (int rr = tid >> 4; rr < BM; rr += GEMM_THREADS / 16) {
    const int m = m0 + rr;
    const int n = n0 + cgrp * 8;
    if (m >= p.M || n >= p.N) continue;
    const u32x2 lo = *(const u32x2*)(cimg + rr * C_STRIDE + cgrp * 16);
    const u32x2 hi = *(const u32x2*)(cimg + rr * C_STRIDE + cgrp * 16 + 8);
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

// split-K tail: sum the S partials, + bias, bf16 round (what the one-pass kernels stage in LDS),
// then the epilogue; 8 columns per thread
template <int EPI, int R>
__global__ __launch_bounds__(256) void splitk_epilogue_kernel(const GemmParams p) {
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int c8 = p.N / 8;
  if (idx >= (int64_t)p.M * c8) return;
  const int m = (int)(idx / c8);
  const int n = (int)(idx % c8) * 8;
  float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int k = 0; k < p.splitk; ++k) {
    const float* src = p.ws + ((int64_t)k * p.M + m) * p.N + n;
    const f32x4 a = *(const f32x4*)src, b = *(const f32x4*)(src + 4);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      s[i] += a[i];
      s[4 + i] += b[i];
    }
  }
  bf16_t cv[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) cv[j] = f2bf(s[j] + (p.bias ? bf2f(p.bias[n + j]) : 0.f));
  float o[8];
  epilogue_row8<EPI, R>(p, m, n, cv, o);
  u32x4 pk;
  pk[0] = pack2(o[0], o[1]);
  pk[1] = pack2(o[2], o[3]);
  pk[2] = pack2(o[4], o[5]);
  pk[3] = pack2(o[6], o[7]);
  *(u32x4*)(p.C + (int64_t)m * p.ldc + n) = pk;
}

// ---------------------------------------------------------------------------------------------
// Production large-tile kernel, templated on the tile height BMT (256 or 224) so that the tile
// count fills whole rounds of the 256 CUs: M = 14336 (= 64 x 224) gives 448 tiles of 256 x 256
// for N = 2048 (1.75 rounds -> 12.5 % of the chip idle in the tail) but 512 tiles of 224 x 256
// (exactly 2). BMT = 256: 8 waves as 4 (m) x 2 (n), each 64 x 128 (4 x 8 fragments);
// BMT = 224: 2 (m) x 4 (n), each 112 x 64 (7 x 4 fragments). Everything else is the l-kernel's
// default schedule (VAR 35): scalar-base asm LDS-DMA, tile t+2's X pieces issued after the
// mid-tile barrier and its W pieces in the next Q0, static priority for waves 4-7, quarters of
// (k-half, n-half) with the next quarter's fragments prefetched, one barrier per K-tile.
// X pieces (8 rows x 128 B) go to waves 4w..4w+3 (for BMT = 224 wave 7 moves only W pieces).
// ---------------------------------------------------------------------------------------------
template <int EPI, int R, int BMT, int DMAW, int SPLIT = 0>
__global__ __launch_bounds__(512, 1) void gemm_nt_kernel_t(const GemmParams p) {
  static_assert(BMT == 256 || BMT == 224, "tile height");
  static_assert(DMAW <= 8, "DMA waves");
  constexpr int NW = 8, NT = NW * 64;
  constexpr int WMW = (BMT == 256) ? 4 : 2;  // waves along m
  constexpr int WNW = NW / WMW;               // waves along n
  constexpr int WTM = BMT / WMW;              // 64 | 112
  constexpr int WTN = BN2 / WNW;              // 128 | 64
  constexpr int MF = WTM / 16;                // 4 | 7
  constexpr int NF = WTN / 16;                // 8 | 4
  constexpr int NFH = NF / 2;                 // n-fragments per quarter
  constexpr int XPIECES = BMT / 8;            // 32 | 28
  constexpr int XT = BMT * BK * 2;            // X tile bytes
  constexpr int ST = XT + WT2;                // stage bytes
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wv = __builtin_amdgcn_readfirstlane(wave);
  const int ntm = (p.M + BMT - 1) / BMT, ntn = (p.N + BN2 - 1) / BN2;
  int tm, tn;
  // SPLIT (split-K for grids under one round, K2 == 0): block = split * tiles + tile; the slice's
  // K-tiles [kt0, kt0 + nk) and a raw f32 partial tile into p.ws[split] (splitk_epilogue_kernel)
  int split = 0, kt0 = 0;
  if constexpr (SPLIT) {
    const int tiles = ntm * ntn;
    split = blockIdx.x / tiles;
    block_to_tile(blockIdx.x - split * tiles, ntm, ntn, tm, tn);
    kt0 = (int)((int64_t)split * (p.K / BK) / p.splitk);
  } else {
    block_to_tile(blockIdx.x, ntm, ntn, tm, tn);
  }
  const int m0 = tm * BMT, n0 = tn * BN2;
  const int nk_main = SPLIT ? (int)((int64_t)(split + 1) * (p.K / BK) / p.splitk) - kt0 : p.K / BK;
  const int nk = nk_main + (SPLIT ? 0 : p.K2 / BK);

  // ---- DMA bookkeeping (see gemm_nt_kernel_l: per-lane 32-bit offsets, scalar bases)
  // DMAW = waves that issue the LDS-DMA (8: all, 4 pieces of each operand each; 4: waves 0-3,
  // 8 pieces each, so waves 4-7 only compute)
  constexpr int PPW = 32 / DMAW;
  const int lrow = lane >> 3, pchunk = lane & 7;
  const bool dma_wave = wv < DMAW;
  const int xp = dma_wave ? min(PPW, max(0, XPIECES - PPW * wv)) : 0;  // X pieces of this wave
  const int wp = dma_wave ? PPW : 0;                                     // W pieces of this wave
  uint32_t xo[PPW], wo[PPW];
  const char* xb = nullptr;
  const char* wb = nullptr;
  auto set_x = [&](bool ext) {
    const int64_t ld = ext ? p.lda2 : p.lda;
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      const int row = min(((wave % DMAW) * PPW + i) * 8 + lrow, BMT - 1);
      xo[i] = (uint32_t)(((int64_t)(min(m0 + row, p.M - 1) - m0) * ld + ((pchunk ^ (row & 7)) * 8)) * 2);
    }
    xb = (const char*)(ext ? ext_a2(p, n0) : p.A) + (int64_t)m0 * ld * 2;
  };
  auto set_w = [&](bool ext) {
    const int64_t ld = ext ? p.ldw2 : p.ldw;
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      const int row = ((wave % DMAW) * PPW + i) * 8 + lrow;
      wo[i] = (uint32_t)(((int64_t)(min(n0 + row, p.N - 1) - n0) * ld + ((pchunk ^ (row & 7)) * 8)) * 2);
    }
    wb = (const char*)(ext ? p.W2 : p.W) + (int64_t)n0 * ld * 2;
  };
  set_x(nk_main == 0);
  set_w(nk_main == 0);
  if constexpr (SPLIT) {
    xb += (int64_t)kt0 * (BK * 2);
    wb += (int64_t)kt0 * (BK * 2);
  }
  const uint32_t lds0 = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) char*)smem);
  auto glds_s = [&](uint32_t voff, const char* sbase, uint32_t lds) {
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(voff), "s"(sbase), "s"(lds) : "memory");
  };
  // a wave's whole set of PPW pieces (consecutive 1-KiB LDS slots) in one asm block: M0 saved /
  // restored once and stepped by s_add instead of two moves per piece (g_dma_batch, A/B switch)
  auto glds_batch = [&](const uint32_t* vo, const char* sbase, uint32_t lds) {
    unsigned keep;
    if constexpr (PPW == 4) {
      asm volatile(
          "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %6\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %5\n\t"
          "s_add_u32 m0, m0, 0x400\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %2, %5\n\t"
          "s_add_u32 m0, m0, 0x400\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %3, %5\n\t"
          "s_add_u32 m0, m0, 0x400\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %4, %5\n\ts_mov_b32 m0, %0"
          : "=&s"(keep)
          : "v"(vo[0]), "v"(vo[1]), "v"(vo[2]), "v"(vo[3]), "s"(sbase), "s"(lds)
          : "memory", "scc");
    } else {
      asm volatile(
          "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %10\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %9\n\t"
          "s_add_u32 m0, m0, 0x400\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %2, %9\n\t"
          "s_add_u32 m0, m0, 0x400\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %3, %9\n\t"
          "s_add_u32 m0, m0, 0x400\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %4, %9\n\t"
          "s_add_u32 m0, m0, 0x400\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %5, %9\n\t"
          "s_add_u32 m0, m0, 0x400\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %6, %9\n\t"
          "s_add_u32 m0, m0, 0x400\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %7, %9\n\t"
          "s_add_u32 m0, m0, 0x400\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %8, %9\n\ts_mov_b32 m0, %0"
          : "=&s"(keep)
          : "v"(vo[0]), "v"(vo[1]), "v"(vo[2]), "v"(vo[3]), "v"(vo[4]), "v"(vo[5]), "v"(vo[6]), "v"(vo[7]),
            "s"(sbase), "s"(lds)
          : "memory", "scc");
    }
  };
  const bool dma_batch = p.dma_batch != 0;
  // LDS byte offsets of X / W buffer `buf`
  auto xaddr = [&](int buf) -> int { return buf * ST; };
  auto waddr = [&](int buf) -> int { return buf * ST + XT; };
  auto stage_x = [&](int st, int kt) {
    if (kt == nk_main && nk_main > 0) set_x(true);  // ext tiles come last, in issue order
    const char* sb = xb + (kt < nk_main ? kt : kt - nk_main) * (BK * 2);
    const uint32_t l = lds0 + xaddr(st) + wv * (PPW * 1024);
    if (dma_batch && xp == PPW) {
      glds_batch(xo, sb, l);
      return;
    }
#pragma unroll
    for (int i = 0; i < PPW; ++i)
      if (i < xp) glds_s(xo[i], sb, l + i * 1024);
  };
  auto stage_w = [&](int st, int kt) {
    if (kt == nk_main && nk_main > 0) set_w(true);
    const char* sb = wb + (kt < nk_main ? kt : kt - nk_main) * (BK * 2);
    const uint32_t l = lds0 + waddr(st) + wv * (PPW * 1024);
    if (dma_batch && wp == PPW) {
      glds_batch(wo, sb, l);
      return;
    }
#pragma unroll
    for (int i = 0; i < PPW; ++i)
      if (i < wp) glds_s(wo[i], sb, l + i * 1024);
  };

  const int wm = wave / WNW;
  const int wn = wave % WNW;
  f32x4 acc[NF][MF];  // [n-fragment][m-fragment]
#pragma unroll
  for (int i = 0; i < NF; ++i)
#pragma unroll
    for (int j = 0; j < MF; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const int frow = lane & 15;
  const int fchunk = lane >> 4;
  // A (W) fragment offsets per quarter q = 2h + nh, B (X) offsets per k-half h
  int aoff[4][NFH], boff[2][MF];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
#pragma unroll
    for (int j = 0; j < MF; ++j) boff[h][j] = swz(wm * WTM + j * 16 + frow, h * 4 + fchunk);
#pragma unroll
    for (int nh = 0; nh < 2; ++nh)
#pragma unroll
      for (int i = 0; i < NFH; ++i)
        aoff[2 * h + nh][i] = swz(wn * WTN + nh * (WTN / 2) + i * 16 + frow, h * 4 + fchunk);
  }
  stage_x(0, 0);
  stage_w(0, 0);
  if (nk > 1) {
    stage_x(1, 1);
    stage_w(1, 1);
    switch (xp + wp) {  // stage 0 landed: only this wave's stage-1 pieces may remain in flight
      case 16: asm volatile("s_waitcnt vmcnt(16)\n\ts_barrier" ::: "memory"); break;
      case 12: asm volatile("s_waitcnt vmcnt(12)\n\ts_barrier" ::: "memory"); break;
      case 8: asm volatile("s_waitcnt vmcnt(8)\n\ts_barrier" ::: "memory"); break;
      case 4: asm volatile("s_waitcnt vmcnt(4)\n\ts_barrier" ::: "memory"); break;
      default: asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory"); break;
    }
  } else {
    asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
  }
  s16x8 aE[NFH], aO[NFH], b0[MF], b1[MF];  // A even/odd quarter sets, B per k-half
#pragma unroll
  for (int i = 0; i < NFH; ++i) aE[i] = *(const s16x8*)(smem + waddr(0) + aoff[0][i]);
#pragma unroll
  for (int j = 0; j < MF; ++j) b0[j] = *(const s16x8*)(smem + xaddr(0) + boff[0][j]);
#define LTX_MFMA_T(AS, BS, NH)                                                                        \
  __builtin_amdgcn_sched_barrier(0);                                                                  \
  _Pragma("unroll") for (int i = 0; i < NFH; ++i)                                                     \
  _Pragma("unroll") for (int j = 0; j < MF; ++j)                                                      \
    acc[(NH) * NFH + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(AS[i], BS[j], acc[(NH) * NFH + i][j], 0, 0, 0); \
  __builtin_amdgcn_sched_barrier(0);
  if (wave >= 4) __builtin_amdgcn_s_setprio(1);

  int cur = 0;           // tile kt's stage
  bool pend_w = false;   // W half of tile kt+1's DMA still to issue in Q0
  for (int kt = 0; kt < nk; ++kt) {
    const char* xs = smem + xaddr(cur);
    const char* ws = smem + waddr(cur);
    // Q0 (h0, n0): prefetch A(Q1)
#pragma unroll
    for (int i = 0; i < NFH; ++i) aO[i] = *(const s16x8*)(ws + aoff[1][i]);
    if (pend_w) {
      stage_w(cur ^ 1, kt + 1);
      pend_w = false;
    }
    LTX_MFMA_T(aE, b0, 0)
    // Q1 (h0, n1): prefetch A(Q2), B(h1)
#pragma unroll
    for (int i = 0; i < NFH; ++i) aE[i] = *(const s16x8*)(ws + aoff[2][i]);
#pragma unroll
    for (int j = 0; j < MF; ++j) b1[j] = *(const s16x8*)(xs + boff[1][j]);
    LTX_MFMA_T(aO, b0, 1)
    // Q2 (h1, n0): prefetch A(Q3)
#pragma unroll
    for (int i = 0; i < NFH; ++i) aO[i] = *(const s16x8*)(ws + aoff[3][i]);
    LTX_MFMA_T(aE, b1, 0)
    // all reads of tile t issued: wait tile t+1, free tile t's stage, DMA tile t+2's X into it
    if (kt + 1 < nk) {
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
      if (kt + 2 < nk) {
        stage_x(cur, kt + 2);
        pend_w = true;
      }
      const char* xn = smem + xaddr(cur ^ 1);
      const char* wn_ = smem + waddr(cur ^ 1);
      // Q3 (h1, n1) of tile t: prefetch A(Q0), B(h0) of tile t+1
#pragma unroll
      for (int i = 0; i < NFH; ++i) aE[i] = *(const s16x8*)(wn_ + aoff[0][i]);
#pragma unroll
      for (int j = 0; j < MF; ++j) b0[j] = *(const s16x8*)(xn + boff[0][j]);
    }
    LTX_MFMA_T(aO, b1, 1)
    cur ^= 1;
  }
#undef LTX_MFMA_T
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
  if constexpr (SPLIT) {  // raw f32 partial: lane holds 4 consecutive n of one m (16-B stores)
    float* part = p.ws + (int64_t)split * p.M * p.N;
#pragma unroll
    for (int i = 0; i < NF; ++i) {
      const int n = n0 + wn * WTN + i * 16 + (lane >> 4) * 4;
#pragma unroll
      for (int j = 0; j < MF; ++j) {
        const int m = m0 + wm * WTM + j * 16 + (lane & 15);
        if (m < p.M && n < p.N) *(f32x4*)(part + (int64_t)m * p.N + n) = acc[i][j];
      }
    }
    return;
  }

  // epilogue stage 1: bf16(acc + bias) -> LDS image [BMT m][256 n]; the NF bias chunks are all
  // loaded before the first use (one wait, not one per fragment column)
  char* cimg = smem;
  u32x2 bias2[NF];
#pragma unroll
  for (int i = 0; i < NF; ++i) {
    bias2[i] = (u32x2){0u, 0u};
    const int gn = n0 + wn * WTN + i * 16 + (lane >> 4) * 4;
    if (p.bias && gn + 3 < p.N) bias2[i] = *(const u32x2*)(p.bias + gn);
  }
#pragma unroll
  for (int i = 0; i < NF; ++i) {
    const int nl = wn * WTN + i * 16 + (lane >> 4) * 4;
    const u32x2 bb = bias2[i];
    const float b4[4] = {bf2f((bf16_t)bb[0]), bf2f((bf16_t)(bb[0] >> 16)), bf2f((bf16_t)bb[1]),
                         bf2f((bf16_t)(bb[1] >> 16))};
#pragma unroll
    for (int j = 0; j < MF; ++j) {
      const int ml = wm * WTM + j * 16 + (lane & 15);
      u32x2 pk;
      pk[0] = pack2(acc[i][j][0] + b4[0], acc[i][j][1] + b4[1]);
      pk[1] = pack2(acc[i][j][2] + b4[2], acc[i][j][3] + b4[3]);
      *(u32x2*)(cimg + ml * C_STRIDE2 + nl * 2) = pk;
    }
  }
  const int cgrp = tid & 31;
  // row pass: this thread's rows (tid >> 5) + RPP i. Epilogues that read aux rows issue every
  // row's aux loads right after stage 1 and cross the image barrier with an LDS-only wait, so the
  // loads overlap the barrier and no row waits on its own load (hipcc had emitted one load +
  // vmcnt(0) per row; LTX_GEMM_EPI_BATCH=0 restores that one-row loop for A/B runs)
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
  if (BATCH && p.epi_batch) {
    EpiAux ax[BATCH ? NPASS : 1];
#pragma unroll
    for (int u = 0; u < NPASS; ++u)  // clamped: every load is in bounds, rows past M are not stored
      epi_load<EPI>(p, min(m0 + (tid >> 5) + u * RPP, p.M - 1), min(n0 + cgrp * 8, p.N - 8), ax[u]);
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // C image complete
#pragma unroll
    for (int u = 0; u < NPASS; ++u) row_out((tid >> 5) + u * RPP, &ax[u]);
  } else {
    __syncthreads();
    for (int rr = tid >> 5; rr < BMT; rr += RPP) row_out(rr, nullptr);
  }
}

static int g_force_small = -1;  // LTX_GEMM_SMALL=1 forces the 128x128 kernel (A/B tests)
// LDS stages of the 128x128 kernel: 0 = auto (3 when the grid is at most one round), 2..4 forced
// (LTX_GEMM_SMALL_STAGES, A/B tests)
static const int g_small_stages = [] {
  const char* e = getenv("LTX_GEMM_SMALL_STAGES");
  return e ? atoi(e) : 0;
}();
// split-K workspaces (caller-owned): a default (ltx_gemm_set_workspace) and optional per-stream
// ones (ltx_gemm_set_stream_workspace), so GEMMs running concurrently on two streams never share
// a partials buffer
struct SplitWs {
  float* ptr = nullptr;
  size_t bytes = 0;
};
static SplitWs g_ws_default;
static std::mutex g_ws_mu;
static std::map<hipStream_t, SplitWs> g_ws_stream;
static SplitWs ws_for(hipStream_t s) {
  std::lock_guard<std::mutex> lock(g_ws_mu);
  auto it = g_ws_stream.find(s);
  return it != g_ws_stream.end() ? it->second : g_ws_default;
}
float* stream_workspace(hipStream_t s, size_t* bytes) {
  const SplitWs w = ws_for(s);
  *bytes = w.bytes;
  return w.ptr;
}
// tuning knob (ltx_gemm_set_variant, or LTX_GEMM_VARIANT at load for whole-step A/B runs): 0 default
// (the ring kernel where it applies, else gemm_nt_kernel_t), 15 gemm_nt_kernel_t at the dispatcher's
// tile height, 13 / 14 gemm_nt_kernel_t forced to 256 / 224-row tiles, 20 the ring kernel. (The
// not-adopted schedules -- one wave per SIMD, 4-slot ring, three-tile X ring, persistent four-wave
// kernel -- live in tools/experiments/ and are not part of the library.)
static int g_variant = [] {
  const char* e = getenv("LTX_GEMM_VARIANT");
  return e ? atoi(e) : 0;
}();
// LTX_GEMM_RING=0 at load: variant 0 runs gemm_nt_kernel_t everywhere (the round-3 default)
static int g_ring = [] {
  const char* e = getenv("LTX_GEMM_RING");
  return e ? atoi(e) : 1;
}();
#ifdef LTX_GEMM_STAMPS
static float* g_stamps = nullptr;  // diagnostic build: 8 x u64 per workgroup of the ring kernel
extern "C" int ltx_gemm_set_stamps(void* ptr) {
  g_stamps = (float*)ptr;
  return 0;
}
#endif
// LTX_GEMM_DMA_BATCH=0: the large-tile kernel issues each LDS-DMA piece in its own asm block
// (M0 saved / set / restored per piece) instead of one block per wave's piece set
static int g_dma_batch = [] {
  const char* e = getenv("LTX_GEMM_DMA_BATCH");
  return (e && e[0] == '0') ? 0 : 1;
}();
// LTX_GEMM_EPI_BATCH: how the large-tile epilogue row pass loads its aux operands -- 2 (default)
// every row's before the ring kernel writes its C image, 1 in two batches of rows after it, 0 one
// row at a time (gemm_nt_kernel_t treats 2 as 1)
static int g_epi_batch = [] {
  const char* e = getenv("LTX_GEMM_EPI_BATCH");
  return e ? atoi(e) : 2;
}();

// The dispatcher's choice for one call, shared by launch() and ltx_gemm_describe (so bench.py can
// attribute its per-launch timings to the kernel rocprof will name).
enum GemmPath { PATH_SPLIT_T = 0, PATH_T = 1, PATH_SMALL = 3, PATH_RING = 4 };
struct GemmPlan {
  GemmPath path;
  int bmt;     // PATH_T: tile height (256 or 224)
  int splitk;  // PATH_SPLIT_T / PATH_SMALL: K slices (1 = none)
  int nst;     // PATH_SMALL: LDS stages
};

static GemmPlan plan_gemm(const GemmParams& p, int epi, int R, hipStream_t s) {
  // the grouped K extension exists in the default kernels only (gemm_nt_kernel_t, gemm_nt_kernel)
  const int g_variant = p.ext_gn > 0 ? 0 : ltx::g_variant;
  if (g_force_small < 0) {
    const char* e = getenv("LTX_GEMM_SMALL");
    g_force_small = (e && e[0] == '1') ? 1 : 0;
  }
  GemmPlan pl{PATH_SMALL, 0, 1, 2};
  // large tile once the grid still fills the chip with 256-row tiles, or fills at least 160 CUs
  // with 224-row tiles (one round at >= 62 %: the inference shapes, M = 3 x 1792 = 5376 -> 192
  // tiles, run 1.3x faster there than as 672 128x128 tiles)
  const int64_t big_tiles = (int64_t)((p.M + BM2 - 1) / BM2) * ((p.N + BN2 - 1) / BN2);
  const int64_t tiles224 = (int64_t)((p.M + 223) / 224) * ((p.N + BN2 - 1) / BN2);
  if ((epi == LTX_EPI_STORE || epi == LTX_EPI_ACCUM) && R == 0) {
    // under one round of 256x256 tiles with a long K (the full-mode weight gradients: [2048 x 2048]
    // over K = the token axis): split K over S slices of >= 16 K-tiles so the grid fills the chip
    if (!g_force_small && g_variant == 0 && p.K2 == 0 && p.M >= BM2 && p.N >= BN2 && big_tiles < 256) {
      const int nk = p.K / BK;
      int S = (int)std::min<int64_t>(8, 256 / big_tiles);
      while (S > 1 && nk / S < 16) --S;
      const SplitWs ws = ws_for(s);
      while (S > 1 && (size_t)S * p.M * p.N * sizeof(float) > ws.bytes) --S;
      if (S > 1 && big_tiles * S >= 128)  // else the 128x128 kernel's split fills the chip better
        return GemmPlan{PATH_SPLIT_T, 256, S, 2};
    }
  }
  if (!g_force_small && p.M >= BM2 &&
      (big_tiles >= 256 || ((g_variant == 0 || g_variant == 15 || g_variant == 20) && tiles224 >= 160))) {
    const int64_t ntn = (p.N + BN2 - 1) / BN2;
    const int64_t t256 = (int64_t)((p.M + 255) / 256) * ntn, t224 = (int64_t)((p.M + 223) / 224) * ntn;
    // fraction of the last round of 256 CUs that has work, per tile height
    auto fill = [](int64_t t) { return (double)t / (double)(((t + 255) / 256) * 256); };
    // the tile height that fills the last round best; variant 13 forces BMT 256, 14 forces 224
    const bool use224 = g_variant == 14 || (g_variant != 13 && fill(t224) > fill(t256) + 0.02);
    const bool ring = ((g_ring == 1 && g_variant == 0) || g_variant == 20) && ring_applies(p);
    return GemmPlan{ring ? PATH_RING : PATH_T, use224 ? 224 : 256, 1, 2};
  }
  const int ntm = (p.M + BM - 1) / BM, ntn = (p.N + BN - 1) / BN;
  const int tiles = ntm * ntn;
  const int nk = p.K / BK + p.K2 / BK;
  // split-K when the grid leaves most CUs idle and each slice keeps >= 4 K-tiles
  int S = 1;
  if (tiles < 128 && nk >= 8) {
    S = min(min(8, nk / 4), (256 + tiles - 1) / tiles);
    // (capped at the 32 MiB the small-tile split-K was tuned and validated with)
    const size_t cap = std::min<size_t>(ws_for(s).bytes, 32u << 20);
    while (S > 1 && (size_t)S * p.M * p.N * sizeof(float) > cap) --S;
  }
  // at most one workgroup per CU: three LDS stages (two K-tiles in flight)
  pl.splitk = S;
  pl.nst = g_small_stages >= 2 ? g_small_stages : ((int64_t)tiles * S <= 256 ? 3 : 2);
  return pl;
}

// rocprof's demangled name of the main kernel plan_gemm picks (the split-K tail kernel, when
// there is one, is not named)
static void describe_plan(const GemmPlan& pl, int epi, int R, int t2, char* buf, size_t len) {
  switch (pl.path) {
    case PATH_SPLIT_T:
      snprintf(buf, len, "ltx::gemm_nt_kernel_t<%d, %d, 256, 8, 1>(ltx::GemmParams)", epi, R);
      break;
    case PATH_T:
      snprintf(buf, len, "ltx::gemm_nt_kernel_t<%d, %d, %d, %d, 0>(ltx::GemmParams)", epi, R, pl.bmt,
               pl.bmt == 224 ? 4 : 8);
      break;
    case PATH_RING:
      snprintf(buf, len, "ltx::gemm_ring_kernel<%d, %d, %d, %d>(ltx::GemmParams)", epi, R, pl.bmt / 32, t2);
      break;
    default:
      snprintf(buf, len, "ltx::gemm_nt_kernel<%d, %d, %d>(ltx::GemmParams)", epi, R, pl.nst);
      break;
  }
}

template <int EPI, int R = 0>
static int launch(const GemmParams& p, hipStream_t s) {
  const GemmPlan pl = plan_gemm(p, EPI, R, s);
  if (pl.path == PATH_SPLIT_T) {
    static bool sk_set = false;
    if (!sk_set) {
      (void)hipFuncSetAttribute((const void*)gemm_nt_kernel_t<EPI, R, 256, 8, 1>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, LDS2);
      sk_set = true;
    }
    const int64_t big_tiles = (int64_t)((p.M + BM2 - 1) / BM2) * ((p.N + BN2 - 1) / BN2);
    GemmParams q = p;
    q.ws = ws_for(s).ptr;
    q.splitk = pl.splitk;
    hipLaunchKernelGGL((gemm_nt_kernel_t<EPI, R, 256, 8, 1>), dim3((unsigned)(big_tiles * pl.splitk)), dim3(512),
                       LDS2, s, q);
    LTX_LAUNCH_CHECK();
    const int64_t n8 = (int64_t)p.M * (p.N / 8);
    hipLaunchKernelGGL((splitk_epilogue_kernel<EPI, R>), dim3((unsigned)((n8 + 255) / 256)), dim3(256), 0, s, q);
    LTX_LAUNCH_CHECK();
    return LTX_OK;
  }
#ifdef LTX_GEMM_STAMPS
  GemmParams ps = p;
  ps.ws = g_stamps;
  if (pl.path == PATH_RING && launch_ring<EPI, R>(ps, pl.bmt, s)) {
#else
  if (pl.path == PATH_RING && launch_ring<EPI, R>(p, pl.bmt, s)) {
#endif
    LTX_LAUNCH_CHECK();
    return LTX_OK;
  }
  if (pl.path == PATH_T || pl.path == PATH_RING) {
    static bool t_set = false;
    if (!t_set) {
      (void)hipFuncSetAttribute((const void*)gemm_nt_kernel_t<EPI, R, 256, 8>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS2);
      (void)hipFuncSetAttribute((const void*)gemm_nt_kernel_t<EPI, R, 224, 4>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS2);
      t_set = true;
    }
    const int64_t ntn = (p.N + BN2 - 1) / BN2;
    const dim3 g224((unsigned)(((p.M + 223) / 224) * ntn)), g256((unsigned)(((p.M + 255) / 256) * ntn));
    if (pl.bmt == 224) {  // 224-row tiles: DMA by waves 0-3 measured +2-3 % (fits in 250 VGPRs)
      hipLaunchKernelGGL((gemm_nt_kernel_t<EPI, R, 224, 4>), g224, dim3(512), LDS2, s, p);
    } else {
      hipLaunchKernelGGL((gemm_nt_kernel_t<EPI, R, 256, 8>), g256, dim3(512), LDS2, s, p);
    }
    LTX_LAUNCH_CHECK();
    return LTX_OK;
  }
  const int ntm = (p.M + BM - 1) / BM, ntn = (p.N + BN - 1) / BN;
  const int tiles = ntm * ntn;
  const int S = pl.splitk, nst = pl.nst;
  const bool deep = nst > 2;
  if (deep) {
    static bool d_set = false;
    if (!d_set) {
      (void)hipFuncSetAttribute((const void*)gemm_nt_kernel<EPI, R, 3>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                3 * STAGE_BYTES);
      (void)hipFuncSetAttribute((const void*)gemm_nt_kernel<EPI, R, 4>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                4 * STAGE_BYTES);
      d_set = true;
    }
  }
  if (S > 1) {
    GemmParams q = p;
    q.ws = ws_for(s).ptr;
    q.splitk = S;
    if (nst == 4)
      hipLaunchKernelGGL((gemm_nt_kernel<EPI, R, 4>), dim3(tiles * S), dim3(GEMM_THREADS), 4 * STAGE_BYTES, s, q);
    else if (deep)
      hipLaunchKernelGGL((gemm_nt_kernel<EPI, R, 3>), dim3(tiles * S), dim3(GEMM_THREADS), 3 * STAGE_BYTES, s, q);
    else
      hipLaunchKernelGGL((gemm_nt_kernel<EPI, R>), dim3(tiles * S), dim3(GEMM_THREADS), LDS_BYTES, s, q);
    LTX_LAUNCH_CHECK();
    const int64_t n8 = (int64_t)p.M * (p.N / 8);
    hipLaunchKernelGGL((splitk_epilogue_kernel<EPI, R>), dim3((unsigned)((n8 + 255) / 256)), dim3(256), 0, s, q);
  } else if (nst == 4) {
    hipLaunchKernelGGL((gemm_nt_kernel<EPI, R, 4>), dim3(tiles), dim3(GEMM_THREADS), 4 * STAGE_BYTES, s, p);
  } else if (deep) {
    hipLaunchKernelGGL((gemm_nt_kernel<EPI, R, 3>), dim3(tiles), dim3(GEMM_THREADS), 3 * STAGE_BYTES, s, p);
  } else {
    hipLaunchKernelGGL((gemm_nt_kernel<EPI, R>), dim3(tiles), dim3(GEMM_THREADS), LDS_BYTES, s, p);
  }
  LTX_LAUNCH_CHECK();
  return LTX_OK;
}

template <int EPI>
static int launch_lora(const GemmParams& p, hipStream_t s) {
  switch (p.rank) {
    case 8: return launch<EPI, 8>(p, s);
    case 16: return launch<EPI, 16>(p, s);
    case 32: return launch<EPI, 32>(p, s);
    default: return fail(LTX_ERR_BAD_ARG, "gemm lora: rank must be 8, 16 or 32");
  }
}

}  // namespace ltx

using namespace ltx;

extern "C" int ltx_gemm_set_variant(int variant) {
  LTX_CHECK_ARG(variant == 0 || variant == 13 || variant == 14 || variant == 15 || variant == 20,
                "gemm_set_variant: 0, 13, 14, 15 or 20");
  g_variant = variant;
  return LTX_OK;
}


extern "C" int ltx_gemm_describe(int64_t M, int64_t N, int64_t K, int64_t K2, int epilogue, int64_t rank,
                                 void* stream, char* buf, int64_t len) {
  LTX_CHECK_ARG(buf && len > 0 && M > 0 && N > 0 && K > 0, "gemm_describe: bad args");
  GemmParams p{};
  p.M = (int)M; p.N = (int)N; p.K = (int)K; p.K2 = (int)K2;
  const int R = (epilogue == LTX_EPI_LORA || epilogue == LTX_EPI_LORA_RESIDUAL ||
                 epilogue == LTX_EPI_LORA_DGRAD_ACCUM) ? (int)rank : 0;
  describe_plan(plan_gemm(p, epilogue, R, (hipStream_t)stream), epilogue, R, p.K2 / 64, buf, (size_t)len);
  return LTX_OK;
}

extern "C" int ltx_gemm_set_workspace(void* ptr, int64_t bytes) {
  LTX_CHECK_ARG(bytes >= 0 && (ptr != nullptr || bytes == 0) && ((uintptr_t)ptr % 16) == 0,
                "gemm_set_workspace: bad buffer");
  std::lock_guard<std::mutex> lock(g_ws_mu);
  g_ws_default.ptr = (float*)ptr;
  g_ws_default.bytes = (size_t)bytes;
  return LTX_OK;
}

extern "C" int ltx_gemm_set_stream_workspace(void* stream, void* ptr, int64_t bytes) {
  LTX_CHECK_ARG(bytes >= 0 && (ptr != nullptr || bytes == 0) && ((uintptr_t)ptr % 16) == 0,
                "gemm_set_stream_workspace: bad buffer");
  std::lock_guard<std::mutex> lock(g_ws_mu);
  g_ws_stream[(hipStream_t)stream] = SplitWs{(float*)ptr, (size_t)bytes};
  return LTX_OK;
}

extern "C" int ltx_gemm_bf16_nt_ext(const void* A, int64_t lda, const void* W, int64_t ldw,
                                    const void* A2, int64_t lda2, const void* W2, int64_t ldw2,
                                    int64_t K2, void* C, int64_t ldc, int64_t M, int64_t N, int64_t K,
                                    int epilogue, const void* bias, const void* aux0, int64_t ld0,
                                    const void* aux1, int64_t ld1, const void* aux2, int64_t ld2,
                                    float alpha, int64_t rank, int64_t rows_per_batch, void* stream);

extern "C" int ltx_gemm_bf16_nt_gext(const void* A, int64_t lda, const void* W, int64_t ldw,
                                     const void* A2, int64_t lda2, const void* W2, int64_t ldw2,
                                     int64_t K2, int64_t ext_group_cols, int64_t ext_group_stride,
                                     void* C, int64_t ldc, int64_t M, int64_t N, int64_t K,
                                     int epilogue, const void* bias, const void* aux0, int64_t ld0,
                                     const void* aux1, int64_t ld1, const void* aux2, int64_t ld2,
                                     float alpha, int64_t rank, int64_t rows_per_batch, void* stream);

extern "C" int ltx_gemm_bf16_nt(const void* A, int64_t lda, const void* W, int64_t ldw, void* C,
                                int64_t ldc, int64_t M, int64_t N, int64_t K, int epilogue,
                                const void* bias, const void* aux0, int64_t ld0, const void* aux1,
                                int64_t ld1, const void* aux2, int64_t ld2, float alpha,
                                int64_t rank, int64_t rows_per_batch, void* stream) {
  return ltx_gemm_bf16_nt_ext(A, lda, W, ldw, nullptr, 0, nullptr, 0, 0, C, ldc, M, N, K, epilogue, bias, aux0,
                              ld0, aux1, ld1, aux2, ld2, alpha, rank, rows_per_batch, stream);
}

extern "C" int ltx_gemm_bf16_nt_ext(const void* A, int64_t lda, const void* W, int64_t ldw,
                                    const void* A2, int64_t lda2, const void* W2, int64_t ldw2,
                                    int64_t K2, void* C, int64_t ldc, int64_t M, int64_t N, int64_t K,
                                    int epilogue, const void* bias, const void* aux0, int64_t ld0,
                                    const void* aux1, int64_t ld1, const void* aux2, int64_t ld2,
                                    float alpha, int64_t rank, int64_t rows_per_batch, void* stream) {
  return ltx_gemm_bf16_nt_gext(A, lda, W, ldw, A2, lda2, W2, ldw2, K2, 0, 0, C, ldc, M, N, K, epilogue, bias,
                               aux0, ld0, aux1, ld1, aux2, ld2, alpha, rank, rows_per_batch, stream);
}

extern "C" int ltx_gemm_bf16_nt_gext(const void* A, int64_t lda, const void* W, int64_t ldw,
                                     const void* A2, int64_t lda2, const void* W2, int64_t ldw2,
                                     int64_t K2, int64_t ext_group_cols, int64_t ext_group_stride,
                                     void* C, int64_t ldc, int64_t M, int64_t N, int64_t K,
                                     int epilogue, const void* bias, const void* aux0, int64_t ld0,
                                     const void* aux1, int64_t ld1, const void* aux2, int64_t ld2,
                                     float alpha, int64_t rank, int64_t rows_per_batch, void* stream) {
  LTX_CHECK_ARG(ext_group_cols == 0 ||
                    (K2 > 0 && ext_group_cols % 256 == 0 && N % ext_group_cols == 0 && ext_group_stride >= 0 &&
                     ext_group_stride % 8 == 0 && (N / ext_group_cols - 1) * ext_group_stride + K2 <= lda2),
                "gemm: grouped K extension needs K2 > 0, groups of 256k columns dividing N, and every group's "
                "A2 columns inside the A2 row");
  LTX_CHECK_ARG(K2 == 0 || (A2 && W2 && K2 % BK == 0 && lda2 >= K2 && ldw2 >= K2 && lda2 % 8 == 0 &&
                            ldw2 % 8 == 0 && ((uintptr_t)A2 | (uintptr_t)W2) % 16 == 0),
                "gemm: K extension needs 16-B aligned A2/W2 with K2 % 64 == 0");
  LTX_CHECK_ARG(A && W && C, "gemm: null operand");
  LTX_CHECK_ARG(M > 0 && N > 0 && K > 0, "gemm: empty shape");
  LTX_CHECK_ARG(K % BK == 0, "gemm: K must be a multiple of 64");
  LTX_CHECK_ARG(N % 8 == 0, "gemm: N must be a multiple of 8");
  LTX_CHECK_ARG(lda % 8 == 0 && ldw % 8 == 0 && ldc % 8 == 0, "gemm: leading dims must be multiples of 8");
  LTX_CHECK_ARG(lda >= K && ldw >= K && ldc >= N, "gemm: leading dim smaller than the row");
  LTX_CHECK_ARG(((uintptr_t)A | (uintptr_t)W | (uintptr_t)C) % 16 == 0, "gemm: operands must be 16-B aligned");
  LTX_CHECK_ARG(M < (1LL << 31) && N < (1LL << 31), "gemm: shape too large");
  LTX_CHECK_ARG(ld0 % 8 == 0 && ((uintptr_t)aux0 % 16) == 0, "gemm: aux0 must be 16-B aligned rows");
  LTX_CHECK_ARG(bias == nullptr || ((uintptr_t)bias % 8) == 0, "gemm: bias must be 8-B aligned");
  GemmParams p;
  p.A = (const bf16_t*)A; p.W = (const bf16_t*)W; p.C = (bf16_t*)C;
  p.lda = lda; p.ldw = ldw; p.ldc = ldc;
  p.M = (int)M; p.N = (int)N; p.K = (int)K;
  p.bias = (const bf16_t*)bias;
  p.aux0 = aux0; p.ld0 = ld0; p.aux1 = aux1; p.ld1 = ld1; p.aux2 = aux2; p.ld2 = ld2;
  p.alpha = alpha; p.rank = (int)rank; p.rows_per_batch = (int)(rows_per_batch > 0 ? rows_per_batch : M);
  p.A2 = (const bf16_t*)A2; p.W2 = (const bf16_t*)W2; p.lda2 = lda2; p.ldw2 = ldw2; p.K2 = (int)K2;
  p.ext_gn = (int)ext_group_cols; p.ext_gs = ext_group_stride;
  p.dma_batch = g_dma_batch;
  p.epi_batch = g_epi_batch;
  p.ws = nullptr; p.splitk = 1;
  hipStream_t s = (hipStream_t)stream;
  switch (epilogue) {
    case LTX_EPI_STORE: return launch<LTX_EPI_STORE>(p, s);
    case LTX_EPI_GELU: return launch<LTX_EPI_GELU>(p, s);
    case LTX_EPI_GATED_RESIDUAL:
      LTX_CHECK_ARG(aux0 && aux1, "gemm gated residual: needs residual (aux0) and gate (aux1)");
      LTX_CHECK_ARG(ld1 % 8 == 0 && ((uintptr_t)aux1 % 16) == 0 && (!aux2 || (ld2 % 8 == 0 && ((uintptr_t)aux2 % 16) == 0)),
                    "gemm gated residual: gate rows (aux1) and the pre-gate store (aux2) must be 16-B aligned rows");
      return launch<LTX_EPI_GATED_RESIDUAL>(p, s);
    case LTX_EPI_LORA:
    case LTX_EPI_LORA_RESIDUAL:
      LTX_CHECK_ARG(aux1 && aux2, "gemm lora: needs U (aux1) and B (aux2)");
      LTX_CHECK_ARG(epilogue == LTX_EPI_LORA || aux0, "gemm lora residual: needs residual (aux0)");
      return epilogue == LTX_EPI_LORA ? launch_lora<LTX_EPI_LORA>(p, s)
                                      : launch_lora<LTX_EPI_LORA_RESIDUAL>(p, s);
    case LTX_EPI_GELU_BWD:
      LTX_CHECK_ARG(aux0, "gemm gelu bwd: needs the pre-activation (aux0)");
      return launch<LTX_EPI_GELU_BWD>(p, s);
    case LTX_EPI_ACCUM:
      LTX_CHECK_ARG(aux0, "gemm accum: needs the accumulator input (aux0)");
      LTX_CHECK_ARG(!aux1 == !aux2 && (!aux1 || (ld1 % 8 == 0 && ld2 % 8 == 0 && ld2 >= N && M % p.rows_per_batch == 0 &&
                                                 ((uintptr_t)aux1 | (uintptr_t)aux2) % 16 == 0)),
                    "gemm accum: the gated copy needs both the gate rows (aux1) and its output (aux2), 16-B aligned rows");
      return launch<LTX_EPI_ACCUM>(p, s);
    case LTX_EPI_LORA_DGRAD_ACCUM:
      LTX_CHECK_ARG(aux1 && aux2, "gemm lora dgrad: needs Wd (aux1) and A (aux2)");
      return launch_lora<LTX_EPI_LORA_DGRAD_ACCUM>(p, s);
    case LTX_EPI_STORE_ROWDOT:
      LTX_CHECK_ARG(aux0 && aux1 && (rank == 32 || rank == 64) && N % rank == 0 && M % p.rows_per_batch == 0,
                    "gemm store_rowdot: needs O (aux0), delta (aux1), head dim (rank) 32 or 64 dividing N, "
                    "whole batches");
      LTX_CHECK_ARG(((uintptr_t)aux1 % 4) == 0, "gemm store_rowdot: delta must be f32-aligned");
      return launch<LTX_EPI_STORE_ROWDOT>(p, s);
    default:
      return fail(LTX_ERR_BAD_ARG, "gemm: unknown epilogue");
  }
}
