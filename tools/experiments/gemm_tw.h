// Four-wave bf16 GEMM kernel template (C[M,N] = epi(A[M,K] . W[N,K]^T)) for tile-aligned training shapes:
// one wave per SIMD, each wave a (BMT/2) x 128 piece of the BMT x 256 output tile.
#include <type_traits>
#include <utility>

#pragma once
#include "gemm_common.h"

namespace ltx {

// ---------------------------------------------------------------------------------------------
// tw kernel. 256 threads = 4 waves as 2 (m) x 2 (n); wave tile (BMT/2) x 128 = MF x 8 fragments
// of v_mfma_f32_16x16x32_bf16 (256 / 224 accumulator registers at BMT = 256 / 224, which one wave
// per SIMD can hold). K-tiles of 64 in two LDS buffers ([BMT][64] X rows + [256][64] W rows, 128-B
// rows with the 16-B chunk XOR-swizzled by row & 7, applied to the DMA source), filled by LDS-DMA
// pieces of 8 rows x 128 B (full cache lines): buffer_load_dwordx4 ... offen lds with ONE per-lane
// offset register per operand, the piece's row offset in an SGPR soffset and M0 set per piece (three
// instructions per KiB: s_mov m0, s_nop, buffer_load).
// One K-tile t per iteration, per wave (QN = 2 MF x 8 MFMAs):
//   * MFMAs on tile t's k-half 0 while tile t's k-half-1 fragments are read from LDS;
//   * at MFMA QB: lgkmcnt(0) + barrier -> every wave is done with tile t's buffer; tile t+2's DMA
//     pieces (15-16 per wave) go into it, one every SP MFMAs;
//   * at MFMA QW (3/4 of the tile): a counted vmcnt (only tile t+2's pieces may be in flight) +
//     barrier -> tile t+1 is in LDS; its k-half-0 fragments are read beside the last MFMAs.
// So tile t+2 has ~1.5 K-tiles of MFMAs to land and LDS reads always have MFMAs to hide behind.
// Persistent: the K-tiles of all a workgroup's output tiles form one stream (gemm_tw_kernel below),
// and the fused epilogue runs from the accumulator registers.
// Requires M % BMT == 0, N % 256 == 0 (the dispatcher falls back to gemm_nt_kernel_t otherwise).
// ---------------------------------------------------------------------------------------------
// compile-time loop: f(std::integral_constant<int, 0>), ..., f(std::integral_constant<int, N-1>)
template <class F, int... I>
__device__ __forceinline__ void static_for_impl(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
  static_for_impl(f, std::make_integer_sequence<int, N>{});
}

// acc += a . b with the accumulator pinned to the AGPR file ("+a"): the 224-256 accumulator
// registers stay in AGPRs and the fragments in VGPRs (left to itself hipcc splits the
// accumulators over both files and copies them around every MFMA)
// Hazards the compiler does not pad around an asm MFMA are covered explicitly: the zero-fill of
// the accumulators is fenced and followed by nops (gemm_tw_kernel: zero_acc), and the epilogue
// reads them only behind the drain nops.
__device__ __forceinline__ void mfma_agpr(f32x4& acc, const s16x8& a, const s16x8& b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}
__device__ __forceinline__ void mfma_agpr0(f32x4& acc, const s16x8& a, const s16x8& b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0" : "=a"(acc) : "v"(a), "v"(b));
}

constexpr int tw_lds_bytes(int bmt) { return 2 * (bmt + 256) * 128; }

// Fused epilogue on 4 consecutive columns n..n+3 of row m, straight from the accumulator layout
// (lane: row m, 4 consecutive n). cv = bf16(acc + bias); the arithmetic and roundings are
// epilogue_row8's (gemm_common.h). The aux operands come preloaded (ax: aux0 row m, gt: aux1 gate
// row m / rows_per_batch, 4 bf16 each), so the loads of the next column group can be in flight.
template <int EPI>
__device__ __forceinline__ void tw_epi4(const GemmParams& p, int m, int n, const float (&v)[4], const u32x2 cpk,
                                        const u32x2 ax, const u32x2 gt, float (&o)[4]) {
  if constexpr (EPI == LTX_EPI_STORE) {
#pragma unroll
    for (int k = 0; k < 4; ++k) o[k] = v[k];
  } else if constexpr (EPI == LTX_EPI_GELU) {
    if (p.aux0) *(u32x2*)((bf16_t*)p.aux0 + (int64_t)m * p.ld0 + n) = cpk;
#pragma unroll
    for (int k = 0; k < 4; k += 2) {
      const f32x2 g = gelu_tanh_pk((f32x2){v[k], v[k + 1]});
      o[k] = g[0];
      o[k + 1] = g[1];
    }
  } else if constexpr (EPI == LTX_EPI_GATED_RESIDUAL) {
    if (p.aux2) *(u32x2*)((bf16_t*)p.aux2 + (int64_t)m * p.ld2 + n) = cpk;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float r = bf2f((bf16_t)(ax[k >> 1] >> ((k & 1) * 16)));
      const float g = bf2f((bf16_t)(gt[k >> 1] >> ((k & 1) * 16)));
      o[k] = r + rbf(g * v[k]);
    }
  } else if constexpr (EPI == LTX_EPI_GELU_BWD) {
#pragma unroll
    for (int k = 0; k < 4; k += 2) {
      const f32x2 f = {bf2f((bf16_t)ax[k >> 1]), bf2f((bf16_t)(ax[k >> 1] >> 16))};
      const f32x2 g = (f32x2){v[k], v[k + 1]} * gelu_tanh_grad_pk(f);
      o[k] = g[0];
      o[k + 1] = g[1];
    }
  } else if constexpr (EPI == LTX_EPI_ACCUM) {
#pragma unroll
    for (int k = 0; k < 4; ++k) o[k] = bf2f((bf16_t)(ax[k >> 1] >> ((k & 1) * 16))) + v[k];
  }
}

// ---------------------------------------------------------------------------------------------
// Persistent form: a workgroup per CU walks its output tiles (tile ids blockIdx.x + k gridDim.x:
// one XCD, so block_to_tile's L2 grouping holds) as ONE stream of K-steps. The DMA of step g+2
// goes out during step g whether or not it belongs to the next tile, so a tile's first K-steps
// are in flight while the previous tile finishes; the epilogue works from the accumulators in
// registers (no LDS image: both buffers stay with the stream) between the tile's last MFMA and
// the next tile's first (which restarts the accumulators from 0, mfma_agpr0).
// ---------------------------------------------------------------------------------------------
template <int EPI, int R, int BMT>
__global__ __launch_bounds__(256, 1) void gemm_tw_kernel(const GemmParams p) {
  static_assert(BMT == 256 || BMT == 224, "tile height");
  constexpr int WTM = BMT / 2;          // wave rows: 128 | 112
  constexpr int MF = WTM / 16;          // 8 | 7
  constexpr int NF = 8;                 // 128 columns per wave
  constexpr int XT = BMT * 128;         // X tile bytes
  constexpr int SB = XT + 256 * 128;    // buffer bytes
  constexpr int XPW = BMT / 32;         // X pieces per wave and K-step (pieces w, w+4, ...): 8 | 7
  constexpr int WPW = 8;                // W pieces per wave and K-step
  constexpr int NPW = XPW + WPW;        // 16 | 15
  constexpr int QH = MF * NF;           // MFMAs per k-half
  constexpr int QN = 2 * QH;            // MFMAs per K-step
  constexpr int QB = QN * 3 / 16;       // barrier: step g's buffer free
  constexpr int QW = QN * 3 / 4;        // counted wait + barrier: step g+1 landed
  constexpr int SP = (QW - 2 - QB) / NPW;  // MFMAs between DMA pieces
  constexpr int NR = NF + MF;           // fragment reads per k-half
  static_assert(QB + 1 + (NPW - 1) * SP < QW, "DMA pieces must all issue before the wait");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ntm = p.M / BMT, ntn = p.N / 256, tiles = ntm * ntn;
  const int G = gridDim.x;
  const int my_tiles = (tiles - (int)blockIdx.x + G - 1) / G;
  const int nk_main = p.K / BK;
  const int nk = nk_main + p.K2 / BK;
  const int total = my_tiles * nk;  // K-steps of this workgroup
  const int wm = wv >> 1, wn = wv & 1;
  auto coords = [&](int k, int& m0, int& n0) {
    int tm, tn;
    block_to_tile((int)blockIdx.x + k * G, ntm, ntn, tm, tn);
    m0 = tm * BMT;
    n0 = tn * 256;
  };

  // ---- LDS-DMA operands. Lane -> (row lane >> 3 of the 8-row piece, physical chunk lane & 7),
  // source chunk (lane & 7) ^ row (rows of a piece are 8-aligned, so row & 7 = lane >> 3).
  const int lrow = lane >> 3;
  const int lch = (lane & 7) ^ lrow;
  const uint32_t vx = (uint32_t)(((int64_t)lrow * p.lda + lch * 8) * 2);
  const uint32_t vw = (uint32_t)(((int64_t)lrow * p.ldw + lch * 8) * 2);
  const uint32_t vx2 = p.K2 ? (uint32_t)(((int64_t)lrow * p.lda2 + lch * 8) * 2) : vx;
  const uint32_t vw2 = p.K2 ? (uint32_t)(((int64_t)lrow * p.ldw2 + lch * 8) * 2) : vw;
  // byte offset of this wave's piece i (rows 8 (w + 4 i) ..) from the tile's first row
  const uint32_t sx = (uint32_t)(wv * 16 * p.lda), sxs = (uint32_t)(64 * p.lda);
  const uint32_t sw = (uint32_t)(wv * 16 * p.ldw), sws = (uint32_t)(64 * p.ldw);
  const uint32_t sx2 = (uint32_t)(wv * 16 * p.lda2), sxs2 = (uint32_t)(64 * p.lda2);
  const uint32_t sw2 = (uint32_t)(wv * 16 * p.ldw2), sws2 = (uint32_t)(64 * p.ldw2);
  const uint32_t lds0 = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) char*)smem);
  asm volatile("s_nop 4" ::: "memory");  // SGPRs derived from v_readfirstlane -> VMEM operands

  // DMA cursor: the K-step the next dma_piece calls load (tile d_tile, K-tile d_kt) as running
  // X / W K-tile pointers plus the lane / row offsets of the operand pair (main or K-extension) it
  // is in; all scalar except the two lane offsets, and touched per K-step only by a 128-B bump
  int d_tile = 0, d_kt = 0, d_m0 = 0, d_n0 = 0;
  const char* dxb;
  const char* dwb;
  uint32_t cvx = vx, cvw = vw, csx = sx, csxs = sxs, csw = sw, csws = sws;
  auto dma_tile_start = [&]() {
    dxb = (const char*)(p.A + (int64_t)d_m0 * p.lda);
    dwb = (const char*)(p.W + (int64_t)d_n0 * p.ldw);
    cvx = vx; cvw = vw; csx = sx; csxs = sxs; csw = sw; csws = sws;
  };
  coords(0, d_m0, d_n0);
  dma_tile_start();
  // past the last K-step the cursor stays on it: the DMA slots of steps total, total+1 re-load
  // that step into the buffer nothing reads any more (constant vmcnt counts, no branches)
  auto dma_advance = [&]() {
    if (d_kt + 1 < nk) {
      if (++d_kt == nk_main) {
        dxb = (const char*)(p.A2 + (int64_t)d_m0 * p.lda2);
        dwb = (const char*)(p.W2 + (int64_t)d_n0 * p.ldw2);
        cvx = vx2; cvw = vw2; csx = sx2; csxs = sxs2; csw = sw2; csws = sws2;
      } else {
        dxb += BK * 2;
        dwb += BK * 2;
      }
    } else if (d_tile + 1 < my_tiles) {
      d_kt = 0;
      coords(++d_tile, d_m0, d_n0);
      dma_tile_start();
    }
  };
  // piece pc (X: 0 .. XPW-1, W: XPW .. NPW-1) of the cursor's step into buffer `buf`
  auto dma_piece = [&](int buf, int pc) {
    const bool isx = pc < XPW;
    const int i = isx ? pc : pc - XPW;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)(isx ? dxb : dwb), 0, 0x7fffffff, 0x00020000);
    const uint32_t voff = isx ? cvx : cvw;
    const uint32_t soff = isx ? csx + i * csxs : csw + i * csws;
    const uint32_t lds = lds0 + (uint32_t)(buf * SB + (isx ? 0 : XT) + (wv + 4 * i) * 1024);
    asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, %3 offen lds"
                 :: "v"(voff), "s"(rs), "s"(lds), "s"(soff) : "memory");
  };

  // ---- fragment reads: A (W rows n) fragment i, B (X rows m) fragment j, k-half h
  const int frow = lane & 15, fch = lane >> 4;
  const int aoff0 = XT + swz(wn * 128 + frow, fch), aoff1 = XT + swz(wn * 128 + frow, 4 + fch);
  const int boff0 = swz(wm * WTM + frow, fch), boff1 = swz(wm * WTM + frow, 4 + fch);

  f32x4 acc[NF][MF];
  s16x8 a0[NF], a1[NF], b0[MF], b1[MF];

  // prologue: steps 0 and 1 in flight, wait for step 0, read its k-half-0 fragments
#pragma unroll
  for (int pc = 0; pc < NPW; ++pc) dma_piece(0, pc);
  dma_advance();
#pragma unroll
  for (int pc = 0; pc < NPW; ++pc) dma_piece(1, pc);
  dma_advance();
  if constexpr (NPW == 16)
    asm volatile("s_waitcnt vmcnt(16)\n\ts_barrier" ::: "memory");
  else
    asm volatile("s_waitcnt vmcnt(15)\n\ts_barrier" ::: "memory");
#pragma unroll
  for (int i = 0; i < NF; ++i) a0[i] = *(const s16x8*)(smem + aoff0 + i * 2048);
#pragma unroll
  for (int j = 0; j < MF; ++j) b0[j] = *(const s16x8*)(smem + boff0 + j * 2048);

  // one K-step g: its k-half-1 fragments are read beside the k-half-0 MFMAs; at QB every wave is
  // done with step g's buffer and step g+2's DMA goes into it; at QW step g+1 has landed and its
  // k-half-0 fragments are read beside the last MFMAs. The MFMA stream is
  // generated with compile-time indices, so every accumulator / fragment index is a constant.
  auto iter = [&](auto c_tag) {
    constexpr int c = decltype(c_tag)::value;  // buffer of this K-step (steps alternate)
    const char* bc = smem + c * SB;
    const char* bn = smem + (c ^ 1) * SB;
    auto step = [&](auto qc) {
      constexpr int q = decltype(qc)::value;
      constexpr int qq = q % QH, i = qq / MF, j = qq % MF;
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (q < QH)
        mfma_agpr(acc[i][j], a0[i], b0[j]);
      else
        mfma_agpr(acc[i][j], a1[i], b1[j]);
      static_for<NR>([&](auto rc) {
        constexpr int r = decltype(rc)::value;
        if constexpr (q == (r * QB) / NR) {
          if constexpr (r < NF)
            a1[r] = *(const s16x8*)(bc + aoff1 + r * 2048);
          else
            b1[r - NF] = *(const s16x8*)(bc + boff1 + (r - NF) * 2048);
        }
      });
      if constexpr (q == QB) asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      static_for<NPW>([&](auto pcc) {
        constexpr int pc = decltype(pcc)::value;
        if constexpr (q == QB + 1 + pc * SP) dma_piece(c, pc);
      });
      if constexpr (q == QW) {
        if constexpr (NPW == 16)
          asm volatile("s_waitcnt vmcnt(16)\n\ts_barrier" ::: "memory");
        else
          asm volatile("s_waitcnt vmcnt(15)\n\ts_barrier" ::: "memory");
      }
      // step g+1's k-half-0 fragments (dead reads past the last step: LDS is there, nothing in
      // flight writes it)
      static_for<NR>([&](auto rc) {
        constexpr int r = decltype(rc)::value;
        if constexpr (q == QW + 1 + (r * (QN - QW - 2)) / NR) {
          if constexpr (r < NF)
            a0[r] = *(const s16x8*)(bn + aoff0 + r * 2048);
          else
            b0[r - NF] = *(const s16x8*)(bn + boff0 + (r - NF) * 2048);
        }
      });
    };
    static_for<QN>(step);
    __builtin_amdgcn_sched_barrier(0);
  };

  // epilogue of the tile (m0, n0) from the accumulators: lane = row m, 4 consecutive columns
  // epilogue of the tile (m0, n0) from the accumulators: lane = row m, 4 consecutive columns.
  // Column group i's bias / aux loads are issued before group i-1's stores, so the compiler's
  // vmcnt waits for them count only those stores (a load behind the stores would wait for them)
  constexpr bool NEED_AX = EPI == LTX_EPI_GATED_RESIDUAL || EPI == LTX_EPI_GELU_BWD || EPI == LTX_EPI_ACCUM;
  constexpr bool NEED_GT = EPI == LTX_EPI_GATED_RESIDUAL;
  auto epilogue = [&](int m0, int n0) {
    // drain: the last MFMAs (fragment row NF-1) wrote their accumulators just now; the AGPR
    // reads below are ordered behind these statements (operands) and the nops cover the latency
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3" : "+a"(acc[NF - 1][0]));
#pragma unroll
    for (int j = 1; j < MF; ++j) asm volatile("" : "+a"(acc[NF - 1][j]));
    __builtin_amdgcn_sched_barrier(0);
    const int mrow = m0 + wm * WTM + (lane & 15);
    const int ncol = n0 + wn * 128 + (lane >> 4) * 4;
    u32x2 bb[2], ax[2][MF], gt[2][MF];
    auto load = [&](int i, int sl) {
      const int n = ncol + i * 16;
      bb[sl] = p.bias ? *(const u32x2*)(p.bias + n) : (u32x2){0u, 0u};
#pragma unroll
      for (int j = 0; j < MF; ++j) {
        const int m = mrow + j * 16;
        if constexpr (NEED_AX) ax[sl][j] = *(const u32x2*)((const bf16_t*)p.aux0 + (int64_t)m * p.ld0 + n);
        if constexpr (NEED_GT)
          gt[sl][j] = *(const u32x2*)((const bf16_t*)p.aux1 + (int64_t)(m / p.rows_per_batch) * p.ld1 + n);
      }
    };
    load(0, 0);
    static_for<NF>([&](auto ic) {
      constexpr int i = decltype(ic)::value;
      constexpr int sl = i & 1;
      if constexpr (i + 1 < NF) load(i + 1, sl ^ 1);
      __builtin_amdgcn_sched_barrier(0);
      const int n = ncol + i * 16;
      const float b4[4] = {bf2f((bf16_t)bb[sl][0]), bf2f((bf16_t)(bb[sl][0] >> 16)), bf2f((bf16_t)bb[sl][1]),
                           bf2f((bf16_t)(bb[sl][1] >> 16))};
#pragma unroll
      for (int j = 0; j < MF; ++j) {
        const int m = mrow + j * 16;
        f32x4 a = acc[i][j];
        asm volatile("" : "+v"(a));  // one accumulator at a time into VGPRs
        u32x2 cpk;  // bf16(acc + bias), what the LDS-image epilogues stage
        cpk[0] = pack2(a[0] + b4[0], a[1] + b4[1]);
        cpk[1] = pack2(a[2] + b4[2], a[3] + b4[3]);
        const float v[4] = {bf2f((bf16_t)cpk[0]), bf2f((bf16_t)(cpk[0] >> 16)), bf2f((bf16_t)cpk[1]),
                            bf2f((bf16_t)(cpk[1] >> 16))};
        float o[4];
        tw_epi4<EPI>(p, m, n, v, cpk, ax[sl][j], gt[sl][j], o);
        u32x2 pk;
        pk[0] = pack2(o[0], o[1]);
        pk[1] = pack2(o[2], o[3]);
        *(u32x2*)(p.C + (int64_t)m * p.ldc + n) = pk;
        __builtin_amdgcn_sched_barrier(0);
      }
    });
    __builtin_amdgcn_sched_barrier(0);
  };

  // accumulators restart from 0 before each tile: plain writes (VALU), then fences that order them
  // before the nops, which cover the VALU-write -> MFMA-SrcC distance the compiler does not pad for
  // asm MFMAs
  auto zero_acc = [&]() {
#pragma unroll
    for (int i = 0; i < NF; ++i)
#pragma unroll
      for (int j = 0; j < MF; ++j) {
        acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
        asm volatile("" : "+a"(acc[i][j]));
      }
    asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");
  };

  int c_kt = 0, c_tile = 0, c_m0 = 0, c_n0 = 0;
  coords(0, c_m0, c_n0);
  zero_acc();
  // two K-steps per trip (buffers 0, 1 as constants); nk is even, so tiles end on odd steps
  for (int g = 0; g < total; g += 2) {
    iter(std::integral_constant<int, 0>{});
    dma_advance();
    iter(std::integral_constant<int, 1>{});
    dma_advance();
    c_kt += 2;
    if (c_kt == nk) {
      epilogue(c_m0, c_n0);
      zero_acc();
      c_kt = 0;
      if (++c_tile < my_tiles) coords(c_tile, c_m0, c_n0);
    }
  }
  // the re-load DMA of the last two slots must land before the workgroup's LDS is released
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

template <int EPI, int R, int BMT>
static inline int launch_tw_t(const GemmParams& p, hipStream_t s) {
  static bool set = false;
  if (!set) {
    (void)hipFuncSetAttribute((const void*)gemm_tw_kernel<EPI, R, BMT>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              tw_lds_bytes(BMT));
    set = true;
  }
  // one workgroup per CU (a multiple of 8, so a workgroup's tiles stay on its XCD)
  const int tiles = (p.M / BMT) * (p.N / 256);
  const unsigned grid = (unsigned)(tiles < 256 ? tiles : 256);
  hipLaunchKernelGGL((gemm_tw_kernel<EPI, R, BMT>), dim3(grid), dim3(256), tw_lds_bytes(BMT), s, p);
  LTX_LAUNCH_CHECK();
  return LTX_OK;
}

}  // namespace ltx
