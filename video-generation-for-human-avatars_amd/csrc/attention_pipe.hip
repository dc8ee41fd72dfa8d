// dK / dV of F.scaled_dot_product_attention (attention.py:1057-1064) for head dim 64, software
// pipelined: the self-attention backward's dominant kernel at config A (N = 1792).
//
// Same algorithm and layout as attn_dkdv_kernel (attention.hip): a workgroup = 4 waves x 32 keys,
// each wave's K / V fragments in registers, dK^T and dV^T accumulated over 32-query halves:
//   A(j): S^T = K.Q^T and dP'^T = delta - V.dO^T (the accumulator starts at delta, V is negated
//         once at load), 8 MFMAs;
//   B(j): P = exp2(S.c - lse), dS = P (dP - delta) = -P dP', both to bf16 B operands (VALU);
//   C(j): dV^T += dO^T.P, dK^T += Q^T.dS, 8 MFMAs with transposed LDS reads.
// At head dim 64 a half's VALU (16 exp + 16 fma + 16 mul + 16 cvt) is as long as its 8 S/dP
// MFMAs, and in the plain kernel it sits between them and the 8 dV/dK MFMAs that need its
// results, so each wave alternates MFMA and VALU phases (MFMA-busy 0.40, r02d_pmc_sq). Here
// iteration j issues C(j-1), A(j+1) and B(j) together: the 16 MFMAs have no dependence on the
// iteration's VALU, which the scheduler spreads into their issue gaps.
//
// Q / dO / lse / delta tiles of 64 queries arrive by LDS-DMA (global_load_lds: no staging
// registers, no LDS write pass) into a 3-buffer ring: one barrier per tile. At iteration 2t+1
// tile t+1 must be resident (its DMA was issued at iteration 2t-1) and tile t-1 is no longer read,
// so its buffer takes tile t+2's DMA.
#include <cstdlib>

#include "attention_common.h"
#include "attn_bwd_body.h"
#ifdef LTX_FWD_W1  // `make fwdw1`: the one-wave forward (measured slower, not in the shipping build)
#include "attn_fwd_body.h"
#endif
#ifdef LTX_DKDV_DIAG  // `make diag`: timing-only variants of the loop (tools/gen_attn_bwd.py --diag)
#include "attn_bwd_body_diag.h"
#endif
#include "ltx_hip.h"

namespace ltx {

namespace {
constexpr int PHD = 64;                               // head dim
constexpr int PQT = 64;                               // queries per LDS tile
constexpr int P_TILE = PQT * PHD * 2;                 // one [64][64] bf16 tile: 8 KiB
constexpr int P_STAT = PQT * 4;                       // one f32 statistic per query
constexpr int P_BUF = 2 * P_TILE + 2 * P_STAT;        // Q | dO | lse | delta
constexpr int P_NBUF = 3;
constexpr int P_KEYS = 128;                           // keys per workgroup (4 waves x 32)
}  // namespace

// two f32 -> one word of two bf16 (round to nearest even): one v_cvt_pk_bf16_f32
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t cvt_pk(float lo, float hi) {
  const bf16x2_t v = {(__bf16)lo, (__bf16)hi};
  return __builtin_bit_cast(uint32_t, v);
}

// NB: LDS tile buffers (as attn_dq_pipe_kernel): 4 = each tile's DMA two tiles ahead, the tile
// barrier waiting only for the tile it opens
template <bool BIAS, int NB>
__global__ __launch_bounds__(256, 2) void attn_dkdv_pipe_kernel(const AttnParams p) {
  constexpr int HD = PHD, KS = HD / 16, DS = HD / 32;
  // ONE shared array: a second __shared__ object beside the DMA target makes hipcc wait for the
  // DMA before unrelated LDS reads
  __shared__ __attribute__((aligned(16))) char smem[NB * P_BUF];

  const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const LaneOfs<HD> lofs(lane);
  int bx, hh, b;
  xcd_block(p.xcd_order, bx, hh, b);
  const int key = bx * P_KEYS + wave * 32 + (lane & 31);
  const int kc = min(key, p.Nk - 1);
  const float c2 = p.scale * LOG2E;
  float kbias = 0.f;
  if (BIAS) {
    kbias = -INFINITY;
    if (key < p.Nk) kbias = p.key_bias ? p.key_bias[(int64_t)b * p.kvb + key] * LOG2E : 0.f;
  }

  s16x8 kf[KS], vf[KS];  // K and -V (sign flipped: exact) of the lane's key
  {
    const bf16_t* kr = p.k + ((int64_t)b * p.kvb + kc) * p.ldk + hh * HD;
    const bf16_t* vr = p.v + ((int64_t)b * p.kvb + kc) * p.ldv + hh * HD;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      kf[ks] = *(const s16x8*)(kr + ks * 16 + 8 * h);
      u32x4 w = *(const u32x4*)(vr + ks * 16 + 8 * h);
      w ^= 0x80008000u;
      vf[ks] = __builtin_bit_cast(s16x8, w);
    }
  }
  f32x16 dka[DS], dva[DS];
#pragma unroll
  for (int d = 0; d < DS; ++d)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      dka[d][r] = 0.f;
      dva[d][r] = 0.f;
    }

  const bf16_t* qbase = p.q + (int64_t)b * p.Nq * p.ldq + hh * HD;
  const bf16_t* obase = p.dout + (int64_t)b * p.Nq * p.lddo + hh * HD;
  const float* lbase = p.lse + ((int64_t)b * p.H + hh) * p.Nq;
  const float* dbase = p.delta + ((int64_t)b * p.H + hh) * p.Nq;
  const int ntiles = (p.Nq + PQT - 1) / PQT;

  // Tile t -> buffer: wave w moves Q and dO rows 16w..16w+15 (two 1-KiB pieces of 8 rows each,
  // the chunk swizzle applied on the source address), wave 0 the lse words, wave 1 the delta
  // words. Rows past Nq re-read the last row (their lse is fixed to +inf below: P = 0).
  // per-lane byte offsets inside a tile (constant but for the ragged last tile), scalar tile bases
  uint32_t qoff[2], ooff[2];
  auto set_offsets = [&](int nrows) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int row = (wave * 2 + i) * 8 + (lane >> 3);
      const int rr = min(row, nrows - 1), c = (lane & 7) ^ swz<HD>(row);
      qoff[i] = (uint32_t)(rr * p.ldq + c * 8) * 2;
      ooff[i] = (uint32_t)(rr * p.lddo + c * 8) * 2;
    }
  };
  set_offsets(PQT);
  auto dma = [&](int t, int buf) {
    char* base = smem + buf * P_BUF;
    const int q0 = t * PQT;
    if (q0 + PQT > p.Nq) set_offsets(p.Nq - q0);  // the ragged last tile (its DMA is the last)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int piece = wave * 2 + i;
      dma16s(qoff[i], qbase + (int64_t)q0 * p.ldq, lds_u32(base + piece * 1024));
      dma16s(ooff[i], obase + (int64_t)q0 * p.lddo, lds_u32(base + P_TILE + piece * 1024));
    }
    if (wave < 2) {
      const float* src = (wave == 0 ? lbase : dbase) + min(q0 + lane, p.Nq - 1);
      dma4(src, lds_u32(base + 2 * P_TILE + wave * P_STAT));
    }
  };
  // after the wait that retires tile t's DMA (wave 0 issued the lse words): rows past Nq -> +inf
  auto fix_stats = [&](int t, int buf) {
    if (wave == 0 && t * PQT + PQT > p.Nq && t * PQT + lane >= p.Nq)
      ((float*)(smem + buf * P_BUF + 2 * P_TILE))[lane] = INFINITY;
  };

  // A: S^T, dP'^T of half u of the tile in buffer `bf`
  auto stage_A = [&](int bf, int u, f32x16& s, f32x16& dp) {
    const char* qt = smem + bf * P_BUF;
    const char* ot = qt + P_TILE;
    const float* dl = (const float*)(qt + 2 * P_TILE + P_STAT);
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const f32x4 d4 = *(const f32x4*)&dl[u * 32 + 8 * g + 4 * h];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        s[4 * g + i] = 0.f;
        dp[4 * g + i] = d4[i];
      }
    }
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      s = mfma32(row_frag<HD>(qt, u * 32, ks, lofs), kf[ks], s);
      dp = mfma32(row_frag<HD>(ot, u * 32, ks, lofs), vf[ks], dp);
    }
  };
  // B: P and dS of half u -> bf16 B-operand fragments (k-steps 0, 1 of the 32 queries)
  auto stage_B = [&](int bf, int u, f32x16& s, f32x16& dp, s16x8 (&pb)[2], s16x8 (&sb)[2]) {
    const float* ls = (const float*)(smem + bf * P_BUF + 2 * P_TILE);
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const f32x4 l4 = *(const f32x4*)&ls[u * 32 + 8 * g + 4 * h];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = 4 * g + i;
        const float pr = fast_exp2(fmaf(s[r], c2, BIAS ? kbias - l4[i] : -l4[i]));
        s[r] = pr;
        dp[r] = -(pr * dp[r]);
      }
    }
#pragma unroll
    for (int ss = 0; ss < 2; ++ss) {
      pb[ss] = acc_frag(s, ss);
      sb[ss] = acc_frag(dp, ss);
    }
  };
  // C: dV^T += dO^T.P, dK^T += Q^T.dS for half u
  auto stage_C = [&](int bf, int u, const s16x8 (&pb)[2], const s16x8 (&sb)[2]) {
    const char* qt = smem + bf * P_BUF;
    const char* ot = qt + P_TILE;
#pragma unroll
    for (int ss = 0; ss < 2; ++ss)
#pragma unroll
      for (int d = 0; d < DS; ++d) {
        dva[d] = mfma32(tr_frag<HD>(ot, u * 32, ss, d, lofs), pb[ss], dva[d]);
        dka[d] = mfma32(tr_frag<HD>(qt, u * 32, ss, d, lofs), sb[ss], dka[d]);
      }
  };
  f32x16 s0, d0, s1, d1;  // S / dP' of even and odd halves
  s16x8 pb[2], sb[2];     // P, dS of the half whose C stage is next
  // One steady-state iteration j, hand-placed: C(j-1) from half uc of buffer bc (pb, sb in),
  // B(j) on (sj, dj) with the lse words of half ub of buffer bb (pb, sb out), A(j+1) into
  // (sn, dn) from half ua of buffer ba. Phase 0 issues C's transposed reads and the lse words;
  // phase 1 pairs each C MFMA with two exponentials of B and A's operand reads; phase 2 pairs
  // each A MFMA with two dS products and two bf16 packs of B. sched_barrier(0) pins each slot.
  auto iteration = [&](int bc, int uc, int bb, int ub, f32x16& sj, f32x16& dj, int ba, int ua,
                       f32x16& sn, f32x16& dn) {
    const char* cq = smem + bc * P_BUF;
    const char* co = cq + P_TILE;
    const float* ls = (const float*)(smem + bb * P_BUF + 2 * P_TILE);
    const char* aq = smem + ba * P_BUF;
    const char* ao = aq + P_TILE;
    const float* dl = (const float*)(aq + 2 * P_TILE + P_STAT);
    f32x4 l4[4];  // first: slot 0's exponentials wait for them
#pragma unroll
    for (int g = 0; g < 4; ++g) l4[g] = *(const f32x4*)&ls[ub * 32 + 8 * g + 4 * h];
    s16x8 to_[2][DS], tq[2][DS];  // in MFMA order
#pragma unroll
    for (int ss = 0; ss < 2; ++ss)
#pragma unroll
      for (int d = 0; d < DS; ++d) {
        to_[ss][d] = tr_frag<HD>(co, uc * 32, ss, d, lofs);
        tq[ss][d] = tr_frag<HD>(cq, uc * 32, ss, d, lofs);
      }
    __builtin_amdgcn_sched_barrier(0);
    s16x8 qa[KS], oa[KS];
    f32x4 d4[4];
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      const int ss = m >> 2, d = (m >> 1) & 1;
      if (m & 1) dka[d] = mfma32(tq[ss][d], sb[ss], dka[d]);
      else dva[d] = mfma32(to_[ss][d], pb[ss], dva[d]);
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int r = 2 * m + e;
        const float lv = l4[r >> 2][r & 3];
        sj[r] = fast_exp2(fmaf(sj[r], c2, BIAS ? kbias - lv : -lv));
      }
      if (m < 4) {
        qa[m] = row_frag<HD>(aq, ua * 32, m, lofs);
        oa[m] = row_frag<HD>(ao, ua * 32, m, lofs);
      } else {
        d4[m - 4] = *(const f32x4*)&dl[ua * 32 + 8 * (m - 4) + 4 * h];
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    u32x4 pw[2], sw[2];
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      const int ks = m >> 1;
      if (m & 1) {
        if (ks == 0) {
#pragma unroll
          for (int g = 0; g < 4; ++g)
#pragma unroll
            for (int i = 0; i < 4; ++i) dn[4 * g + i] = d4[g][i];
        }
        dn = mfma32(oa[ks], vf[ks], dn);
      } else {
        if (ks == 0) {
#pragma unroll
          for (int r = 0; r < 16; ++r) sn[r] = 0.f;
        }
        sn = mfma32(qa[ks], kf[ks], sn);
      }
      const int r = 2 * m;
      dj[r] = -(sj[r] * dj[r]);
      dj[r + 1] = -(sj[r + 1] * dj[r + 1]);
      uint32_t wp = cvt_pk(sj[r], sj[r + 1]), ws = cvt_pk(dj[r], dj[r + 1]);
      asm volatile("" : "+v"(wp), "+v"(ws));  // keeps the packs in this slot (not sunk to the end)
      pw[m >> 2][m & 3] = wp;
      sw[m >> 2][m & 3] = ws;
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int ss = 0; ss < 2; ++ss) {
      pb[ss] = __builtin_bit_cast(s16x8, pw[ss]);
      sb[ss] = __builtin_bit_cast(s16x8, sw[ss]);
    }
  };
  // retire this wave's DMA, fix the ragged tile's statistics, then the workgroup barrier
  auto tile_sync = [&](int t, int buf) {
    __builtin_amdgcn_s_waitcnt(0);  // vmcnt(0) expcnt(0) lgkmcnt(0): DMA landed, LDS reads back
    fix_stats(t, buf);
    __builtin_amdgcn_s_waitcnt(0);
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };

  dma(0, 0);
  if (ntiles > 1) dma(1, 1);
  if (NB == 4 && ntiles > 2) dma(2, 2);
  __builtin_amdgcn_s_waitcnt(0);
  if (ntiles > 1) fix_stats(1, 1);
  if (NB == 4 && ntiles > 2) fix_stats(2, 2);
  tile_sync(0, 0);

  stage_A(0, 0, s0, d0);                // A(0)
  stage_A(0, 1, s1, d1);                // iteration 0: A(1), B(0)
  stage_B(0, 0, s0, d0, pb, sb);
  int b0 = 0, b1 = 1;                   // buffers of tiles t, t+1
  for (int t = 0; t + 1 < ntiles; ++t) {
    // iteration 2t+1: tile t+1 resident, tile t-1's buffer free for tile t+2 (NB 3) / t+3 (NB 4)
    if constexpr (NB == 4) {
      // tile t+1 landed: tile t+2's pieces (4 per wave, + the lse / delta words of waves 0, 1)
      // may stay in flight; this wave's reads of tile t-1 done
      if (t + 2 < ntiles) {
        if (wave < 2) __builtin_amdgcn_s_waitcnt(0x0075);  // vmcnt(5) lgkmcnt(0)
        else __builtin_amdgcn_s_waitcnt(0x0074);           // vmcnt(4) lgkmcnt(0)
      } else {
        __builtin_amdgcn_s_waitcnt(0);
      }
      fix_stats(t + 1, b1);
      __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): the fix-up store
      asm volatile("" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      if (t + 3 < ntiles) dma(t + 3, (t + 3) & 3);  // into tile t-1's buffer
    } else {
      tile_sync(t + 1, b1);
      if (t + 2 < ntiles) dma(t + 2, (t + 2) % 3);
    }
    iteration(b0, 0, b0, 1, s1, d1, b1, 0, s0, d0);  // C(2t), B(2t+1), A(2t+2)
    iteration(b0, 1, b1, 0, s0, d0, b1, 1, s1, d1);  // C(2t+1), B(2t+2), A(2t+3)
    b0 = b1;
    b1 = NB == 4 ? (b1 + 1) & 3 : (b1 + 1) % 3;
  }
  // iteration J-1 (J = 2 ntiles): C(J-2), B(J-1); then C(J-1)
  stage_C(b0, 0, pb, sb);
  stage_B(b0, 1, s1, d1, pb, sb);
  stage_C(b0, 1, pb, sb);

  // dK, dV as whole rows through wave-private LDS slots (the ring is free past the last tile)
  __syncthreads();
  const int k0 = bx * P_KEYS + wave * 32, nk = min(32, p.Nk - k0);
  if (nk <= 0) return;
  store_rows_lds<HD>(smem + wave * 8192, dka, p.scale, p.dk + (int64_t)b * p.Nk * p.lddk + hh * HD, p.lddk, k0, nk,
                     lane);
  store_rows_lds<HD>(smem + wave * 8192 + 4096, dva, 1.0f, p.dv + (int64_t)b * p.Nk * p.lddv + hh * HD, p.lddv, k0,
                     nk, lane);
}

// =============================================================================================
// dK / dV at ONE wave per SIMD (self-attention shapes: no key bias, head dim 64): 4 waves x 64 keys
// (two 32-key tiles per wave) = 256 keys per workgroup, the whole loop one hand-scheduled asm
// statement (attn_bwd_body.h, generated by tools/gen_attn_bwd.py: register map, schedule and the
// out-of-range handling of ragged query tiles are described there). Same arithmetic, fragment
// layouts and MFMA accumulation order as attn_dkdv_pipe_kernel: dK / dV are bitwise equal to it.
// =============================================================================================
namespace {
constexpr int W1_KEYS = 256;  // keys per workgroup
}

__device__ __forceinline__ uint64_t srd_half(const u32x4& d, int hi) {
  return hi ? ((uint64_t)d[3] << 32 | d[2]) : ((uint64_t)d[1] << 32 | d[0]);
}

// raw buffer descriptor over [base, base + bytes): loads past `bytes` return zeros
__device__ __forceinline__ u32x4 raw_srd(const void* base, uint64_t bytes) {
  const uint64_t a = (uint64_t)base;
  u32x4 d;
  d[0] = __builtin_amdgcn_readfirstlane((unsigned)a);
  d[1] = __builtin_amdgcn_readfirstlane((unsigned)(a >> 32) & 0xffffu);  // stride 0
  d[2] = __builtin_amdgcn_readfirstlane((unsigned)(bytes > 0xffffffffull ? 0xffffffffull : bytes));
  d[3] = 0x00020000u;
  return d;
}

// diagnostic builds: shader-clock (s_memtime) and 100-MHz (s_memrealtime) stamps of a wave at kernel
// entry and exit, 4 u64 per wave after the 8 phase stamps of every wave (tools/dkdv_stamps.py)
typedef uint64_t u64x4 __attribute__((ext_vector_type(4)));
struct EdgeStamps {
  uint64_t t0 = 0, r0 = 0;
  __device__ __forceinline__ void start() {
    t0 = __builtin_amdgcn_s_memtime();
    r0 = __builtin_amdgcn_s_memrealtime();
  }
  __device__ __forceinline__ void stop(const AttnParams& p) {
    const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    const int64_t nw = (int64_t)gridDim.x * gridDim.y * gridDim.z * 4;
    const int64_t w = (blockIdx.x + (int64_t)gridDim.x * (blockIdx.y + (int64_t)gridDim.y * blockIdx.z)) * 4 +
                      (threadIdx.x >> 6);
    if ((threadIdx.x & 63) == 0) *(u64x4*)((uint64_t*)p.part + nw * 8 + w * 4) = (u64x4){t0, r0, t1, r1};
  }
};

template <int V>
__global__ __launch_bounds__(256, 1) void attn_dkdv_w1_kernel(const AttnParams p) {
  EdgeStamps es;
  if constexpr (V > 0) es.start();
  constexpr int HD = PHD;
  // the ring (3 x LTX_DKDV_W1_BUF B); after the loop the epilogue's dK / dV staging
  __shared__ __attribute__((aligned(16))) char smem[LTX_DKDV_W1_NBUF * LTX_DKDV_W1_BUF];
  const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const LaneOfs<HD> lofs(lane);
  int bx, hh, b;
  xcd_block(p.xcd_order, bx, hh, b);
  const int k0 = bx * W1_KEYS + wave * 64;
  // K / V rows of the lane's key in each 32-key tile (clamped: keys past Nk are computed, not stored)
  const bf16_t* kp[2];
  const bf16_t* vp[2];
#pragma unroll
  for (int kt = 0; kt < 2; ++kt) {
    const int kc = min(k0 + kt * 32 + (lane & 31), p.Nk - 1);
    kp[kt] = p.k + ((int64_t)b * p.kvb + kc) * p.ldk + hh * HD + 8 * h;
    vp[kt] = p.v + ((int64_t)b * p.kvb + kc) * p.ldv + hh * HD + 8 * h;
  }
  // buffer descriptors of this (batch, head)'s Q and dO columns and its lse / delta rows; each spans
  // exactly the valid rows, so a query tile's rows past Nq read as zeros
  const bf16_t* qbase = p.q + (int64_t)b * p.Nq * p.ldq + hh * HD;
  const bf16_t* obase = p.dout + (int64_t)b * p.Nq * p.lddo + hh * HD;
  const float* lbase = p.lse + ((int64_t)b * p.H + hh) * p.Nq;
  const float* dbase = p.delta + ((int64_t)b * p.H + hh) * p.Nq;
  const u32x4 srdq = raw_srd(qbase, ((uint64_t)(p.Nq - 1) * p.ldq + HD) * 2);
  const u32x4 srdo = raw_srd(obase, ((uint64_t)(p.Nq - 1) * p.lddo + HD) * 2);
  // wave 0: lse, wave 1: delta; waves 2 and 3 repeat them into a dummy slot (every wave issues the
  // same five DMA instructions per tile, so one counted wait fits all)
  const u32x4 srds = raw_srd((wave & 1) ? (const void*)dbase : (const void*)lbase, (uint64_t)p.Nq * 4);
  const uint32_t wst = __builtin_amdgcn_readfirstlane(2 * P_TILE + (wave < 2 ? wave * P_STAT : 2 * P_STAT));
  // per-lane DMA offsets inside a tile: piece 2w + i = rows 8 (2w + i) .. + 7, chunk swizzled
  uint32_t vq[2], vo[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = (wave * 2 + i) * 8 + (lane >> 3), c = (lane & 7) ^ swz<HD>(row);
    vq[i] = (uint32_t)(row * p.ldq + c * 8) * 2;
    vo[i] = (uint32_t)(row * p.lddo + c * 8) * 2;
  }
  const uint32_t vl = (uint32_t)lane * 4, vs = (uint32_t)(16 * h);
  const uint32_t lds0 = __builtin_amdgcn_readfirstlane(lds_u32(smem));
  const uint32_t wq = __builtin_amdgcn_readfirstlane(wave * 2048);
  const uint32_t qstep = __builtin_amdgcn_readfirstlane((uint32_t)(64 * p.ldq * 2));
  const uint32_t ostep = __builtin_amdgcn_readfirstlane((uint32_t)(64 * p.lddo * 2));
  const uint32_t iters = __builtin_amdgcn_readfirstlane((uint32_t)((p.Nq + 63) / 64 - 1));
  const float c2 = p.scale * LOG2E;
  // diagnostic builds only: this wave's 8 phase stamps (tools/gen_attn_bwd.py "stamps" variant)
  uint64_t* stp = (uint64_t*)p.part +
                  ((blockIdx.x + (int64_t)gridDim.x * (blockIdx.y + (int64_t)gridDim.y * blockIdx.z)) * 4 + wave) * 8;
  f32x16 dv00 = {}, dv01 = {}, dv10 = {}, dv11 = {}, dk00 = {}, dk01 = {}, dk10 = {}, dk11 = {};
#define LTX_W1_OPERANDS                                                                                      \
  : "+a"(dv00), "+a"(dv01), "+a"(dv10), "+a"(dv11), "+a"(dk00), "+a"(dk01), "+a"(dk10), "+a"(dk11) \
               : [sq0] "s"(srd_half(srdq, 0)), [sq1] "s"(srd_half(srdq, 1)), [so0] "s"(srd_half(srdo, 0)), \
                 [so1] "s"(srd_half(srdo, 1)), [ss0] "s"(srd_half(srds, 0)), [ss1] "s"(srd_half(srds, 1)), \
                 [qstep] "s"(qstep), [ostep] "s"(ostep), [lds0] "s"(lds0), [wq] "s"(wq), [wst] "s"(wst), \
                 [iters] "s"(iters), [c2] "s"(c2), [vr0] "v"(lofs.row[0]), [vr1] "v"(lofs.row[1]), \
                 [vr2] "v"(lofs.row[2]), [vr3] "v"(lofs.row[3]), [vt0] "v"(lofs.tr[0][0]), [vt1] "v"(lofs.tr[0][1]), \
                 [vt2] "v"(lofs.tr[1][0]), [vt3] "v"(lofs.tr[1][1]), [vs] "v"(vs), [vq0] "v"(vq[0]), \
                 [vq1] "v"(vq[1]), [vo0] "v"(vo[0]), [vo1] "v"(vo[1]), [vl] "v"(vl), [kp0] "v"(kp[0]), \
                 [kp1] "v"(kp[1]), [vp0] "v"(vp[0]), [vp1] "v"(vp[1]), [stp] "v"(stp) \
               : "memory", "scc", "vcc", LTX_DKDV_W1_CLOBBERS
  if constexpr (V == 0) asm volatile(LTX_DKDV_W1_BODY LTX_W1_OPERANDS);
#ifdef LTX_DKDV_DIAG  // phase stamps into p.part (tools/dkdv_stamps.py): 1 as built, 2 without VALU, 3 without LDS reads
  if constexpr (V == 1) asm volatile(LTX_DKDV_W1_BODY_V1 LTX_W1_OPERANDS);
  if constexpr (V == 2) asm volatile(LTX_DKDV_W1_BODY_V2 LTX_W1_OPERANDS);
  if constexpr (V == 3) asm volatile(LTX_DKDV_W1_BODY_V3 LTX_W1_OPERANDS);
  if constexpr (V == 4) asm volatile(LTX_DKDV_W1_BODY_V4 LTX_W1_OPERANDS);
  if constexpr (V == 5) asm volatile(LTX_DKDV_W1_BODY_V5 LTX_W1_OPERANDS);
#endif
#undef LTX_W1_OPERANDS
  // dK, dV as whole rows through wave-private LDS slots (every DMA retired inside the statement)
  __syncthreads();
  const f32x16 dk[2][2] = {{dk00, dk01}, {dk10, dk11}};
  const f32x16 dvv[2][2] = {{dv00, dv01}, {dv10, dv11}};
#pragma unroll
  for (int kt = 0; kt < 2; ++kt) {
    const int kb = k0 + kt * 32, nk = min(32, p.Nk - kb);
    if (nk > 0) {
      store_rows_lds<HD>(smem + wave * 8192, dk[kt], p.scale, p.dk + (int64_t)b * p.Nk * p.lddk + hh * HD, p.lddk,
                         kb, nk, lane);
      store_rows_lds<HD>(smem + wave * 8192 + 4096, dvv[kt], 1.0f, p.dv + (int64_t)b * p.Nk * p.lddv + hh * HD,
                         p.lddv, kb, nk, lane);
    }
  }
  if constexpr (V > 0) es.stop(p);
}

// LTX_ATTN_DKDV_W1 (attn_switches()): unset / 2 the persistent one-wave kernel (attn_dkdv_w1p_kernel), 1
// one workgroup per key block (attn_dkdv_w1_kernel), 0 attn_dkdv_pipe_kernel, 12..16 / 22 the stamped
// diagnostic variants (`make diag` builds)
static int dkdv_w1_mode() { return attn_switches().dkdv_w1; }
bool dkdv_w1_enabled() { return dkdv_w1_mode() != 0; }
// LTX_ATTN_DKDV_W1=2 (22: its stamped diagnostic variant): the persistent kernel
bool dkdv_w1p_enabled() { return dkdv_w1_mode() == 2 || dkdv_w1_mode() == 22; }

int launch_dkdv_w1(const AttnParams& p, hipStream_t s) {
  const dim3 g((unsigned)((p.Nk + W1_KEYS - 1) / W1_KEYS), (unsigned)p.H, (unsigned)p.B);
  const int mode = dkdv_w1_mode();
#ifdef LTX_DKDV_DIAG
  if (mode >= 12 && mode <= 16) {  // phase stamps into the stream's workspace (8 u64 per wave)
    AttnParams q = p;
    size_t ws = 0;
    q.part = stream_workspace(s, &ws);
    if (q.part == nullptr || ws < (size_t)g.x * g.y * g.z * 4 * 12 * 8) return fail(LTX_ERR_BAD_ARG, "stamps: workspace");
    if (mode == 12) hipLaunchKernelGGL(attn_dkdv_w1_kernel<1>, g, dim3(256), 0, s, q);
    if (mode == 13) hipLaunchKernelGGL(attn_dkdv_w1_kernel<2>, g, dim3(256), 0, s, q);
    if (mode == 14) hipLaunchKernelGGL(attn_dkdv_w1_kernel<3>, g, dim3(256), 0, s, q);
    if (mode == 15) hipLaunchKernelGGL(attn_dkdv_w1_kernel<4>, g, dim3(256), 0, s, q);
    if (mode == 16) hipLaunchKernelGGL(attn_dkdv_w1_kernel<5>, g, dim3(256), 0, s, q);
    LTX_LAUNCH_CHECK();
    return LTX_OK;
  }
#endif
  (void)mode;
  hipLaunchKernelGGL(attn_dkdv_w1_kernel<0>, g, dim3(256), 0, s, p);
  LTX_LAUNCH_CHECK();
  return LTX_OK;
}

// =============================================================================================
// dK / dV, PERSISTENT (attn_bwd_body.h LTX_DKDV_W1P_BODY, tools/gen_attn_bwd.py dkdv_p_body): one
// workgroup per CU walks the items L = blockIdx.x + i * gridDim.x (a 256-key block of one (batch,
// head), in attn_dkdv_w1_kernel's XCD-aware order), the loads of item i+1 overlapping the tail and the
// stores of item i. Per item the same loop as attn_dkdv_w1_kernel: dK / dV bitwise equal to it.
// =============================================================================================
namespace {
constexpr int W1P_MAXIT = 63;  // items per workgroup (table rows, + the null row)
constexpr int W1P_LDS = LTX_DKDV_W1P_TAB + (W1P_MAXIT + 1) * LTX_DKDV_W1P_ITEM;
}

// buffer descriptor words of [base, base + bytes) (stride 0; loads past `bytes` return zeros)
__device__ __forceinline__ void srd_words(uint32_t* w, const void* base, uint64_t bytes) {
  const uint64_t a = (uint64_t)base;
  w[0] = (uint32_t)a;
  w[1] = (uint32_t)(a >> 32) & 0xffffu;
  w[2] = (uint32_t)(bytes > 0xffffffffull ? 0xffffffffull : bytes);
  w[3] = 0x00020000u;
}
__device__ __forceinline__ void base_words(uint32_t* w, const void* base) {
  const uint64_t a = (uint64_t)base;
  w[0] = (uint32_t)a;
  w[1] = (uint32_t)(a >> 32) & 0xffffu;
}

// item L of I -> (block x, head, batch): xcd_block's bijective remap with L as the block id (the
// workgroups of XCD x run the items L = x mod 8 when the grid is a multiple of 8 or every item has
// its own workgroup), so each XCD walks a contiguous range of the (x fastest, head, batch) order
__device__ __forceinline__ void item_coords(int L, int I, int gx, int gy, int xcd_order, int& bx, int& by, int& bz) {
  int wg = L;
  if (xcd_order) {
    const int q = I / 8, r = I % 8, xcd = L % 8, idx = L / 8;
    wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
  }
  bx = wg % gx;
  by = (wg / gx) % gy;
  bz = wg / (gx * gy);
}

template <int V>
__global__ __launch_bounds__(256, 1) void attn_dkdv_w1p_kernel(const AttnParams p) {
  constexpr int HD = PHD;
  EdgeStamps es;
  if constexpr (V > 0) es.start();
  __shared__ __attribute__((aligned(16))) char smem[W1P_LDS];  // ring | staging | item table
  const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const LaneOfs<HD> lofs(lane);
  const int gx = (p.Nk + W1_KEYS - 1) / W1_KEYS, I = gx * p.H * p.B, G = gridDim.x, w = blockIdx.x;
  const int nit = (I - w + G - 1) / G;  // >= 1: the launch has G <= I
  if (tid <= nit) {  // row tid: item tid; row nit: the null row (empty K / V descriptors)
    int bx, hh, b;
    item_coords(w + min(tid, nit - 1) * G, I, gx, p.H, p.xcd_order, bx, hh, b);
    const int k0 = bx * W1_KEYS, nk = min(W1_KEYS, p.Nk - k0);
    const bool null = tid == nit;
    uint32_t* row = (uint32_t*)(smem + LTX_DKDV_W1P_TAB + tid * LTX_DKDV_W1P_ITEM);
    srd_words(row, p.k + ((int64_t)b * p.kvb + k0) * p.ldk + hh * HD, null ? 0 : ((uint64_t)(nk - 1) * p.ldk + HD) * 2);
    srd_words(row + 4, p.v + ((int64_t)b * p.kvb + k0) * p.ldv + hh * HD, null ? 0 : ((uint64_t)(nk - 1) * p.ldv + HD) * 2);
    base_words(row + 8, p.q + (int64_t)b * p.Nq * p.ldq + hh * HD);
    base_words(row + 10, p.dout + (int64_t)b * p.Nq * p.lddo + hh * HD);
    base_words(row + 12, p.lse + ((int64_t)b * p.H + hh) * p.Nq);
    base_words(row + 14, p.delta + ((int64_t)b * p.H + hh) * p.Nq);
    srd_words(row + 16, p.dk + ((int64_t)b * p.Nk + k0) * p.lddk + hh * HD, ((uint64_t)(nk - 1) * p.lddk + HD) * 2);
    srd_words(row + 20, p.dv + ((int64_t)b * p.Nk + k0) * p.lddv + hh * HD, ((uint64_t)(nk - 1) * p.lddv + HD) * 2);
  }
  __syncthreads();
  // sizes (words 2, 3) of the Q, dO and stats descriptors: the same for every item
  // (< 4 GiB: dkdv_w1p_applies)
  const uint32_t sq2 = __builtin_amdgcn_readfirstlane((uint32_t)(((p.Nq - 1) * (uint32_t)p.ldq + HD) * 2));
  const uint32_t so2 = __builtin_amdgcn_readfirstlane((uint32_t)(((p.Nq - 1) * (uint32_t)p.lddo + HD) * 2));
  const uint32_t ss2 = __builtin_amdgcn_readfirstlane((uint32_t)(p.Nq * 4));
  const uint32_t wst = __builtin_amdgcn_readfirstlane(2 * P_TILE + (wave < 2 ? wave * P_STAT : 2 * P_STAT));
  uint32_t vq[2], vo[2], vkd[2], vvd[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = (wave * 2 + i) * 8 + (lane >> 3), c = (lane & 7) ^ swz<HD>(row);
    vq[i] = (uint32_t)(row * p.ldq + c * 8) * 2;
    vo[i] = (uint32_t)(row * p.lddo + c * 8) * 2;
    // K / V region fill: even / odd 8-row pieces of the wave's 64 keys (the swizzle depends on the
    // row's bits 1-3 only: piece j's rows 8 j + (lane >> 3) swizzle as piece j & 1's), the piece's
    // 8 j rows added by its soffset
    const int kr = wave * 64 + (lane >> 3), kc = (lane & 7) ^ swz<HD>(8 * i + (lane >> 3));
    vkd[i] = (uint32_t)(kr * p.ldk + kc * 8) * 2;
    vvd[i] = (uint32_t)(kr * p.ldv + kc * 8) * 2;
  }
  const uint32_t vl = (uint32_t)lane * 4, vs = (uint32_t)(16 * h);
  const uint32_t lds0 = __builtin_amdgcn_readfirstlane(lds_u32(smem));
  const uint32_t tab = __builtin_amdgcn_readfirstlane(lds_u32(smem + LTX_DKDV_W1P_TAB));
  const uint32_t stg = __builtin_amdgcn_readfirstlane(lds_u32(smem + LTX_DKDV_W1P_STG) + wave * 8192);
  const uint32_t kvw = __builtin_amdgcn_readfirstlane(lds_u32(smem + LTX_DKDV_W1P_KV) + wave * 8192);
  const uint32_t s8k = __builtin_amdgcn_readfirstlane((uint32_t)(16 * p.ldk)), s8v = __builtin_amdgcn_readfirstlane((uint32_t)(16 * p.ldv));
  const uint32_t wq = __builtin_amdgcn_readfirstlane(wave * 2048);
  const uint32_t qstep = __builtin_amdgcn_readfirstlane((uint32_t)(64 * p.ldq * 2));
  const uint32_t ostep = __builtin_amdgcn_readfirstlane((uint32_t)(64 * p.lddo * 2));
  const uint32_t iters = __builtin_amdgcn_readfirstlane((uint32_t)((p.Nq + 63) / 64 - 1));
  const uint32_t nitems = __builtin_amdgcn_readfirstlane((uint32_t)nit);
  const uint32_t wodd = __builtin_amdgcn_readfirstlane((uint32_t)(wave & 1));
  const uint32_t s8dk = __builtin_amdgcn_readfirstlane((uint32_t)(16 * p.lddk)), s8dv = __builtin_amdgcn_readfirstlane((uint32_t)(16 * p.lddv));
  // staging: this lane's write base (row lane & 31, half h) and read base (row lane >> 3, chunk lane & 7)
  const uint32_t vwd = (uint32_t)((lane & 31) * 128 + h * 8);
  const uint32_t vrd = stg + (uint32_t)((lane >> 3) * 128 + (((lane & 7) ^ ((lane >> 3) & 7)) << 4));
  const uint32_t vdk = (uint32_t)(((wave * 64 + (lane >> 3)) * p.lddk + (lane & 7) * 8) * 2);
  const uint32_t vdv = (uint32_t)(((wave * 64 + (lane >> 3)) * p.lddv + (lane & 7) * 8) * 2);
  const float c2 = p.scale * LOG2E, scale = p.scale;
  uint64_t* stp = (uint64_t*)p.part + ((int64_t)blockIdx.x * 4 + wave) * 8;  // diagnostic builds only
#define LTX_W1P_OPERANDS                                                                                     \
  ::[sq2] "s"(sq2), [so2] "s"(so2), [ss2] "s"(ss2), [qstep] "s"(qstep), [ostep] "s"(ostep), [lds0] "s"(lds0),  \
    [wq] "s"(wq), [wst] "s"(wst), [iters] "s"(iters), [c2] "s"(c2), [tab] "s"(tab), [nitems] "s"(nitems),       \
    [wodd] "s"(wodd), [scale] "s"(scale), [s8dk] "s"(s8dk), [s8dv] "s"(s8dv), [stg] "s"(stg), [kvw] "s"(kvw),   \
    [s8k] "s"(s8k), [s8v] "s"(s8v),                                                                             \
    [vr0] "v"(lofs.row[0]), [vr1] "v"(lofs.row[1]), [vr2] "v"(lofs.row[2]), [vr3] "v"(lofs.row[3]),             \
    [vt0] "v"(lofs.tr[0][0]), [vt1] "v"(lofs.tr[0][1]), [vt2] "v"(lofs.tr[1][0]), [vt3] "v"(lofs.tr[1][1]),     \
    [vs] "v"(vs), [vq0] "v"(vq[0]), [vq1] "v"(vq[1]), [vo0] "v"(vo[0]), [vo1] "v"(vo[1]), [vl] "v"(vl),         \
    [vkd0] "v"(vkd[0]), [vkd1] "v"(vkd[1]), [vvd0] "v"(vvd[0]), [vvd1] "v"(vvd[1]), [vwd] "v"(vwd), [vrd] "v"(vrd), \
    [vdk] "v"(vdk), [vdv] "v"(vdv), [stp] "v"(stp)                                                              \
      : "memory", "scc", "vcc", LTX_DKDV_W1P_CLOBBERS
  if constexpr (V == 0) asm volatile(LTX_DKDV_W1P_BODY LTX_W1P_OPERANDS);
#ifdef LTX_DKDV_DIAG
  if constexpr (V == 1) asm volatile(LTX_DKDV_W1P_BODY_V1 LTX_W1P_OPERANDS);
#endif
#undef LTX_W1P_OPERANDS
  if constexpr (V > 0) es.stop(p);
}

static int cu_count() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
  }
  return n;
}

// the persistent kernel applies when every workgroup's items fit its table
bool dkdv_w1p_applies(const AttnParams& p) {
  const int64_t I = (int64_t)((p.Nk + W1_KEYS - 1) / W1_KEYS) * p.H * p.B;
  const uint64_t span = (uint64_t)p.Nq * (uint64_t)std::max<int64_t>(p.ldq, p.lddo) * 2;  // Q / dO descriptor sizes
  return I <= (int64_t)W1P_MAXIT * cu_count() && span < 0xffffffffull;
}

int launch_dkdv_w1p(const AttnParams& p, hipStream_t s) {
  const int I = ((p.Nk + W1_KEYS - 1) / W1_KEYS) * p.H * p.B;
  const dim3 g((unsigned)min(I, cu_count()));
#ifdef LTX_DKDV_DIAG
  if (dkdv_w1_mode() == 22) {
    AttnParams q = p;
    size_t ws = 0;
    q.part = stream_workspace(s, &ws);
    if (q.part == nullptr || ws < (size_t)g.x * 4 * 12 * 8) return fail(LTX_ERR_BAD_ARG, "stamps: workspace");
    hipLaunchKernelGGL(attn_dkdv_w1p_kernel<1>, g, dim3(256), 0, s, q);
    LTX_LAUNCH_CHECK();
    return LTX_OK;
  }
#endif
  hipLaunchKernelGGL(attn_dkdv_w1p_kernel<0>, g, dim3(256), 0, s, p);
  LTX_LAUNCH_CHECK();
  return LTX_OK;
}

// =============================================================================================
// dQ at ONE wave per SIMD (self-attention shapes: no key bias, head dim 64): 4 waves x 64 queries
// (two 32-query tiles per wave) = 256 queries per workgroup, the loop one hand-scheduled asm
// statement (attn_bwd_body.h LTX_DQ_W1_BODY, tools/gen_attn_bwd.py dq_body). Same arithmetic and
// accumulation order as attn_dq_pipe_kernel: dQ is bitwise equal to it.
// =============================================================================================
template <int V>
__global__ __launch_bounds__(256, 1) void attn_dq_w1_kernel(const AttnParams p) {
  EdgeStamps es;
  if constexpr (V > 0) es.start();
  constexpr int HD = PHD;
  __shared__ __attribute__((aligned(16))) char smem[3 * LTX_DQ_W1_BUF];
  const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const LaneOfs<HD> lofs(lane);
  int bx, hh, b;
  xcd_block(p.xcd_order, bx, hh, b);
  const int q0 = bx * 256 + wave * 64;
  // the lane's query in each 32-query tile (clamped: queries past Nq are computed, not stored)
  const bf16_t* qp[2];
  const bf16_t* op[2];
  float nl[2], nd[2];
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    const int qc = min(q0 + qt * 32 + (lane & 31), p.Nq - 1);
    qp[qt] = p.q + ((int64_t)b * p.Nq + qc) * p.ldq + hh * HD + 8 * h;
    op[qt] = p.dout + ((int64_t)b * p.Nq + qc) * p.lddo + hh * HD + 8 * h;
    const int64_t si = ((int64_t)b * p.H + hh) * p.Nq + qc;
    nl[qt] = -p.lse[si];
    nd[qt] = -p.delta[si];
  }
  // K / V columns of this (batch, head), exactly the valid key rows (keys past Nk read as zeros)
  const bf16_t* kbase = p.k + (int64_t)b * p.kvb * p.ldk + hh * HD;
  const bf16_t* vbase = p.v + (int64_t)b * p.kvb * p.ldv + hh * HD;
  const u32x4 srdk = raw_srd(kbase, ((uint64_t)(p.Nk - 1) * p.ldk + HD) * 2);
  const u32x4 srdv = raw_srd(vbase, ((uint64_t)(p.Nk - 1) * p.ldv + HD) * 2);
  uint32_t vk[2], vv[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = (wave * 2 + i) * 8 + (lane >> 3), c = (lane & 7) ^ swz<HD>(row);
    vk[i] = (uint32_t)(row * p.ldk + c * 8) * 2;
    vv[i] = (uint32_t)(row * p.ldv + c * 8) * 2;
  }
  const uint32_t lds0 = __builtin_amdgcn_readfirstlane(lds_u32(smem));
  const uint32_t wq = __builtin_amdgcn_readfirstlane(wave * 2048);
  const uint32_t kstep = __builtin_amdgcn_readfirstlane((uint32_t)(64 * p.ldk * 2));
  const uint32_t vstep = __builtin_amdgcn_readfirstlane((uint32_t)(64 * p.ldv * 2));
  const uint32_t iters = __builtin_amdgcn_readfirstlane((uint32_t)((p.Nk + 63) / 64 - 1));
  const float c2 = p.scale * LOG2E;
  uint64_t* stp = (uint64_t*)p.part +  // diagnostic builds only: this wave's 8 stamps
                  ((blockIdx.x + (int64_t)gridDim.x * (blockIdx.y + (int64_t)gridDim.y * blockIdx.z)) * 4 + wave) * 8;
  f32x16 a00 = {}, a01 = {}, a10 = {}, a11 = {};
#define LTX_DQ_OPERANDS \
               : "+a"(a00), "+a"(a01), "+a"(a10), "+a"(a11) \
               : [sk0] "s"(srd_half(srdk, 0)), [sk1] "s"(srd_half(srdk, 1)), [sv0] "s"(srd_half(srdv, 0)), \
                 [sv1] "s"(srd_half(srdv, 1)), [kstep] "s"(kstep), [vstep] "s"(vstep), [lds0] "s"(lds0), \
                 [wq] "s"(wq), [iters] "s"(iters), [c2] "s"(c2), [vr0] "v"(lofs.row[0]), [vr1] "v"(lofs.row[1]), \
                 [vr2] "v"(lofs.row[2]), [vr3] "v"(lofs.row[3]), [vt0] "v"(lofs.tr[0][0]), [vt1] "v"(lofs.tr[0][1]), \
                 [vt2] "v"(lofs.tr[1][0]), [vt3] "v"(lofs.tr[1][1]), [vk0] "v"(vk[0]), [vk1] "v"(vk[1]), \
                 [vv0] "v"(vv[0]), [vv1] "v"(vv[1]), [qp0] "v"(qp[0]), [qp1] "v"(qp[1]), [op0] "v"(op[0]), \
                 [op1] "v"(op[1]), [nl0] "v"(nl[0]), [nl1] "v"(nl[1]), [nd0] "v"(nd[0]), [nd1] "v"(nd[1]), \
                 [stp] "v"(stp) \
               : "memory", "scc", "vcc", LTX_DQ_W1_CLOBBERS
  if constexpr (V == 0) asm volatile(LTX_DQ_W1_BODY LTX_DQ_OPERANDS);
#ifdef LTX_DKDV_DIAG
  if constexpr (V == 1) asm volatile(LTX_DQ_W1_BODY_V1 LTX_DQ_OPERANDS);
  if constexpr (V == 2) asm volatile(LTX_DQ_W1_BODY_V2 LTX_DQ_OPERANDS);
#endif
#undef LTX_DQ_OPERANDS
  const f32x16 acc[2][2] = {{a00, a01}, {a10, a11}};
  if (!p.dq_f32) {  // dQ as whole rows through wave-private LDS slots
    __syncthreads();
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
      const int qb = q0 + qt * 32;
      if (qb < p.Nq)
        store_rows_lds<HD>(smem + wave * 4096, acc[qt], p.scale, (bf16_t*)p.dq + (int64_t)b * p.Nq * p.lddq + hh * HD,
                           p.lddq, qb, min(32, p.Nq - qb), lane);
    }
    if constexpr (V > 0) es.stop(p);
    return;
  }
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    const int qi = q0 + qt * 32 + (lane & 31);
    if (qi >= p.Nq) continue;
    float* qrow = (float*)p.dq + ((int64_t)b * p.Nq + qi) * p.lddq + hh * HD;
#pragma unroll
    for (int d = 0; d < 2; ++d)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        f32x4 w = {acc[qt][d][4 * g] * p.scale, acc[qt][d][4 * g + 1] * p.scale, acc[qt][d][4 * g + 2] * p.scale,
                   acc[qt][d][4 * g + 3] * p.scale};
        *(f32x4*)(qrow + d * 32 + 8 * g + 4 * h) = w;
      }
  }
}

// =============================================================================================
// dQ, PERSISTENT (attn_bwd_body.h LTX_DQ_W1P_BODY, tools/gen_attn_bwd.py dq_p_body): one workgroup per
// CU walks 256-query blocks as attn_dkdv_w1p_kernel walks key blocks; per block attn_dq_w1_kernel's
// loop (dQ bitwise equal to it). bf16 dQ only (the f32 output stays on attn_dq_w1_kernel).
// =============================================================================================
static int dq_w1_mode();
namespace {
constexpr int DQP_LDS = LTX_DQ_W1P_TAB + (W1P_MAXIT + 1) * LTX_DKDV_W1P_ITEM;
}

template <int V>
__global__ __launch_bounds__(256, 1) void attn_dq_w1p_kernel(const AttnParams p) {
  constexpr int HD = PHD;
  EdgeStamps es;
  if constexpr (V > 0) es.start();
  __shared__ __attribute__((aligned(16))) char smem[DQP_LDS];  // ring | staging | item table
  const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const LaneOfs<HD> lofs(lane);
  const int gx = (p.Nq + 255) / 256, I = gx * p.H * p.B, G = gridDim.x, w = blockIdx.x;
  const int nit = (I - w + G - 1) / G;
  if (tid <= nit) {  // row tid: block tid; row nit: the null row (empty Q / dO / stats descriptors)
    int bx, hh, b;
    item_coords(w + min(tid, nit - 1) * G, I, gx, p.H, p.xcd_order, bx, hh, b);
    const int q0 = bx * 256, nq = min(256, p.Nq - q0);
    const bool null = tid == nit;
    uint32_t* row = (uint32_t*)(smem + LTX_DQ_W1P_TAB + tid * LTX_DKDV_W1P_ITEM);
    const int64_t st = ((int64_t)b * p.H + hh) * p.Nq + q0;
    srd_words(row, p.q + ((int64_t)b * p.Nq + q0) * p.ldq + hh * HD, null ? 0 : ((uint64_t)(nq - 1) * p.ldq + HD) * 2);
    srd_words(row + 4, p.dout + ((int64_t)b * p.Nq + q0) * p.lddo + hh * HD, null ? 0 : ((uint64_t)(nq - 1) * p.lddo + HD) * 2);
    srd_words(row + 8, p.lse + st, null ? 0 : (uint64_t)nq * 4);
    srd_words(row + 12, p.delta + st, null ? 0 : (uint64_t)nq * 4);
    base_words(row + 16, p.k + (int64_t)b * p.kvb * p.ldk + hh * HD);
    base_words(row + 18, p.v + (int64_t)b * p.kvb * p.ldv + hh * HD);
    srd_words(row + 20, (bf16_t*)p.dq + ((int64_t)b * p.Nq + q0) * p.lddq + hh * HD, ((uint64_t)(nq - 1) * p.lddq + HD) * 2);
  }
  __syncthreads();
  const uint32_t sk2 = __builtin_amdgcn_readfirstlane((uint32_t)(((p.Nk - 1) * (uint32_t)p.ldk + HD) * 2));
  const uint32_t sv2 = __builtin_amdgcn_readfirstlane((uint32_t)(((p.Nk - 1) * (uint32_t)p.ldv + HD) * 2));
  uint32_t vk[2], vv[2], vqd[2], vod[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = (wave * 2 + i) * 8 + (lane >> 3), c = (lane & 7) ^ swz<HD>(row);
    vk[i] = (uint32_t)(row * p.ldk + c * 8) * 2;
    vv[i] = (uint32_t)(row * p.ldv + c * 8) * 2;
    // Q / dO region fill: even / odd 8-row pieces of the wave's 64 queries (as the persistent dK / dV
    // kernel's K / V fill), the piece's 8 j rows added by its soffset
    const int qr = wave * 64 + (lane >> 3), qc = (lane & 7) ^ swz<HD>(8 * i + (lane >> 3));
    vqd[i] = (uint32_t)(qr * p.ldq + qc * 8) * 2;
    vod[i] = (uint32_t)(qr * p.lddo + qc * 8) * 2;
  }
  const uint32_t vsd = (uint32_t)(wave * 64 + lane) * 4;  // the wave's lse / delta words
  const uint32_t lds0 = __builtin_amdgcn_readfirstlane(lds_u32(smem));
  const uint32_t tab = __builtin_amdgcn_readfirstlane(lds_u32(smem + LTX_DQ_W1P_TAB));
  const uint32_t stg = __builtin_amdgcn_readfirstlane(lds_u32(smem + LTX_DQ_W1P_STG) + wave * 4096);
  const uint32_t qow = __builtin_amdgcn_readfirstlane(lds_u32(smem + LTX_DQ_W1P_QO) + wave * 8192);
  const uint32_t stw = __builtin_amdgcn_readfirstlane(lds_u32(smem + LTX_DQ_W1P_ST) + wave * 256);
  const uint32_t vsl = stw + (uint32_t)(lane & 31) * 4;
  const uint32_t s8q = __builtin_amdgcn_readfirstlane((uint32_t)(16 * p.ldq)), s8o = __builtin_amdgcn_readfirstlane((uint32_t)(16 * p.lddo));
  const uint32_t wq = __builtin_amdgcn_readfirstlane(wave * 2048);
  const uint32_t kstep = __builtin_amdgcn_readfirstlane((uint32_t)(64 * p.ldk * 2));
  const uint32_t vstep = __builtin_amdgcn_readfirstlane((uint32_t)(64 * p.ldv * 2));
  const uint32_t iters = __builtin_amdgcn_readfirstlane((uint32_t)((p.Nk + 63) / 64 - 1));
  const uint32_t nitems = __builtin_amdgcn_readfirstlane((uint32_t)nit);
  const uint32_t s8dq = __builtin_amdgcn_readfirstlane((uint32_t)(16 * p.lddq));
  const uint32_t vwd = (uint32_t)((lane & 31) * 128 + h * 8);
  const uint32_t vrd = stg + (uint32_t)((lane >> 3) * 128 + (((lane & 7) ^ ((lane >> 3) & 7)) << 4));
  const uint32_t vdq = (uint32_t)(((wave * 64 + (lane >> 3)) * p.lddq + (lane & 7) * 8) * 2);
  const float c2 = p.scale * LOG2E, scale = p.scale;
  uint64_t* stp = (uint64_t*)p.part + ((int64_t)blockIdx.x * 4 + wave) * 8;  // diagnostic builds only
#define LTX_DQP_OPERANDS                                                                                       \
  ::[sk2] "s"(sk2), [sv2] "s"(sv2), [kstep] "s"(kstep), [vstep] "s"(vstep), [lds0] "s"(lds0), [wq] "s"(wq),    \
    [iters] "s"(iters), [c2] "s"(c2), [tab] "s"(tab), [nitems] "s"(nitems), [scale] "s"(scale), [s8dq] "s"(s8dq), \
    [stg] "s"(stg), [qow] "s"(qow), [stw] "s"(stw), [s8q] "s"(s8q), [s8o] "s"(s8o), [vr0] "v"(lofs.row[0]), [vr1] "v"(lofs.row[1]), [vr2] "v"(lofs.row[2]), [vr3] "v"(lofs.row[3]), \
    [vt0] "v"(lofs.tr[0][0]), [vt1] "v"(lofs.tr[0][1]), [vt2] "v"(lofs.tr[1][0]), [vt3] "v"(lofs.tr[1][1]),       \
    [vk0] "v"(vk[0]), [vk1] "v"(vk[1]), [vv0] "v"(vv[0]), [vv1] "v"(vv[1]), [vqd0] "v"(vqd[0]), [vqd1] "v"(vqd[1]), \
    [vod0] "v"(vod[0]), [vod1] "v"(vod[1]), [vsd] "v"(vsd), [vsl] "v"(vsl), [vwd] "v"(vwd), [vrd] "v"(vrd),        \
    [vdq] "v"(vdq), [stp] "v"(stp)                                                                                \
      : "memory", "scc", "vcc", LTX_DQ_W1P_CLOBBERS
  if constexpr (V == 0) asm volatile(LTX_DQ_W1P_BODY LTX_DQP_OPERANDS);
#ifdef LTX_DKDV_DIAG
  if constexpr (V == 1) asm volatile(LTX_DQ_W1P_BODY_V1 LTX_DQP_OPERANDS);
#endif
#undef LTX_DQP_OPERANDS
  if constexpr (V > 0) es.stop(p);
}

bool dq_w1p_applies(const AttnParams& p) {
  const int64_t I = (int64_t)((p.Nq + 255) / 256) * p.H * p.B;
  const uint64_t span = (uint64_t)p.Nk * (uint64_t)std::max<int64_t>(p.ldk, p.ldv) * 2;  // K / V descriptor sizes
  return !p.dq_f32 && I <= (int64_t)W1P_MAXIT * cu_count() && span < 0xffffffffull;
}

int launch_dq_w1p(const AttnParams& p, hipStream_t s) {
  const int I = ((p.Nq + 255) / 256) * p.H * p.B;
  const dim3 g((unsigned)min(I, cu_count()));
#ifdef LTX_DKDV_DIAG
  if (dq_w1_mode() == 22) {
    AttnParams q = p;
    size_t ws = 0;
    q.part = stream_workspace(s, &ws);
    if (q.part == nullptr || ws < (size_t)g.x * 4 * 12 * 8) return fail(LTX_ERR_BAD_ARG, "stamps: workspace");
    hipLaunchKernelGGL(attn_dq_w1p_kernel<1>, g, dim3(256), 0, s, q);
    LTX_LAUNCH_CHECK();
    return LTX_OK;
  }
#endif
  hipLaunchKernelGGL(attn_dq_w1p_kernel<0>, g, dim3(256), 0, s, p);
  LTX_LAUNCH_CHECK();
  return LTX_OK;
}

// LTX_ATTN_DQ_W1 (attn_switches()): unset / 2 the persistent one-wave kernel (bf16 dQ), 1 one workgroup per
// query block, 0 attn_dq_pipe_kernel, 12 / 13 / 22 the stamped diagnostic variants (`make diag` builds)
static int dq_w1_mode() { return attn_switches().dq_w1; }
bool dq_w1_enabled() { return dq_w1_mode() != 0; }
// LTX_ATTN_DQ_W1=2 (22: its stamped diagnostic variant): the persistent kernel
bool dq_w1p_enabled() { return dq_w1_mode() == 2 || dq_w1_mode() == 22; }

int launch_dq_w1(const AttnParams& p, hipStream_t s) {
  const dim3 g((unsigned)((p.Nq + 255) / 256), (unsigned)p.H, (unsigned)p.B);
#ifdef LTX_DKDV_DIAG
  const int mode = dq_w1_mode();
  if (mode == 12 || mode == 13) {
    AttnParams q = p;
    size_t ws = 0;
    q.part = stream_workspace(s, &ws);
    if (q.part == nullptr || ws < (size_t)g.x * g.y * g.z * 4 * 12 * 8) return fail(LTX_ERR_BAD_ARG, "stamps: workspace");
    if (mode == 12) hipLaunchKernelGGL(attn_dq_w1_kernel<1>, g, dim3(256), 0, s, q);
    else hipLaunchKernelGGL(attn_dq_w1_kernel<2>, g, dim3(256), 0, s, q);
    LTX_LAUNCH_CHECK();
    return LTX_OK;
  }
#endif
  hipLaunchKernelGGL(attn_dq_w1_kernel<0>, g, dim3(256), 0, s, p);
  LTX_LAUNCH_CHECK();
  return LTX_OK;
}

// =============================================================================================
// dQ (attn_q_kernel MODE 1 semantics) for self-attention shapes (no key bias, Nk % 64 == 0),
// software pipelined the same way. A workgroup = 4 waves x 32 queries (Q, dO fragments, -lse and
// delta of the lane's query in registers); per 32-key half j:
//   A(j): S^T = K.Q^T and dP'^T = V.dO^T - delta (the dP chain starts from a register tuple
//         holding -delta: no subtraction per element), 8 MFMAs;
//   B(j): dS = exp2(S c - lse) dP' -> bf16 (16 fma + 16 exp + 16 mul + 8 cvt);
//   C(j): dQ^T += K^T.dS^T, 4 MFMAs with transposed K reads.
// Iteration j issues C(j-1) and A(j+1) (12 MFMAs) around B(j)'s VALU; K / V tiles of 64 keys by
// LDS-DMA into a 3-buffer ring, one barrier per tile.
// =============================================================================================
namespace {
constexpr int D_KT = 64;                        // keys per LDS tile
constexpr int D_TILE = D_KT * PHD * 2;          // 8 KiB
constexpr int D_BUF = 2 * D_TILE;               // K | V
constexpr int D_QUERIES = 128;                  // queries per workgroup (4 waves x 32)
}  // namespace

// NB: LDS tile buffers. 3: a tile's DMA is issued one tile-pair ahead and the tile barrier waits for
// every outstanding piece; 4: issued two ahead, the barrier waits only for the tile it opens
// (vmcnt(4): the next tile's 4 pieces per wave stay in flight)
template <int NB>
__global__ __launch_bounds__(256, 2) void attn_dq_pipe_kernel(const AttnParams p) {
  constexpr int HD = PHD, KS = HD / 16, DS = HD / 32;
  __shared__ __attribute__((aligned(16))) char smem[NB * D_BUF];

  const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const LaneOfs<HD> lofs(lane);
  int bx, hh, b;
  xcd_block(p.xcd_order, bx, hh, b);
  const int qi = bx * D_QUERIES + wave * 32 + (lane & 31);
  const int qc = min(qi, p.Nq - 1);
  const float c2 = p.scale * LOG2E;

  s16x8 qf[KS], of[KS];
  {
    const bf16_t* qr = p.q + ((int64_t)b * p.Nq + qc) * p.ldq + hh * HD;
    const bf16_t* dr = p.dout + ((int64_t)b * p.Nq + qc) * p.lddo + hh * HD;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      qf[ks] = *(const s16x8*)(qr + ks * 16 + 8 * h);
      of[ks] = *(const s16x8*)(dr + ks * 16 + 8 * h);
    }
  }
  const int64_t si = ((int64_t)b * p.H + hh) * p.Nq + qc;
  const float nlse = -p.lse[si];
  f32x16 ndl;  // -delta in every register: the dP' chain's initial accumulator
  {
    const float v = -p.delta[si];
#pragma unroll
    for (int r = 0; r < 16; ++r) ndl[r] = v;
  }
  f32x16 acc[DS];
#pragma unroll
  for (int d = 0; d < DS; ++d)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[d][r] = 0.f;

  const bf16_t* kbase = p.k + (int64_t)b * p.kvb * p.ldk + hh * HD;
  const bf16_t* vbase = p.v + (int64_t)b * p.kvb * p.ldv + hh * HD;
  const int ntiles = p.Nk / D_KT;

  // key tile t -> buffer: wave w moves K and V rows 16w..16w+15 (two 1-KiB pieces each)
  uint32_t koff[2], voff[2];  // per-lane byte offsets inside a key tile (same for every tile)
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = (wave * 2 + i) * 8 + (lane >> 3), c = (lane & 7) ^ swz<HD>(row);
    koff[i] = (uint32_t)(row * p.ldk + c * 8) * 2;
    voff[i] = (uint32_t)(row * p.ldv + c * 8) * 2;
  }
  auto dma = [&](int t, int buf) {
    char* base = smem + buf * D_BUF;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int piece = wave * 2 + i;
      dma16s(koff[i], kbase + (int64_t)t * D_KT * p.ldk, lds_u32(base + piece * 1024));
      dma16s(voff[i], vbase + (int64_t)t * D_KT * p.ldv, lds_u32(base + D_TILE + piece * 1024));
    }
  };
  auto tile_sync = [&]() {
    __builtin_amdgcn_s_waitcnt(0);
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
  auto stage_A = [&](int bf, int u, f32x16& s, f32x16& dp) {
    const char* kt = smem + bf * D_BUF;
    const char* vt = kt + D_TILE;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      s = mfma32(row_frag<HD>(kt, u * 32, ks, lofs), qf[ks], ks == 0 ? f32x16{} : s);
      dp = mfma32(row_frag<HD>(vt, u * 32, ks, lofs), of[ks], ks == 0 ? ndl : dp);
    }
  };
  s16x8 sbf[2];  // dS of the half whose C stage is next
  auto stage_B = [&](f32x16& s, f32x16& dp) {
#pragma unroll
    for (int r = 0; r < 16; ++r) dp[r] = fast_exp2(fmaf(s[r], c2, nlse)) * dp[r];
#pragma unroll
    for (int ss = 0; ss < 2; ++ss) sbf[ss] = acc_frag(dp, ss);
  };
  auto stage_C = [&](int bf, int u) {
    const char* kt = smem + bf * D_BUF;
#pragma unroll
    for (int ss = 0; ss < 2; ++ss)
#pragma unroll
      for (int d = 0; d < DS; ++d) acc[d] = mfma32(tr_frag<HD>(kt, u * 32, ss, d, lofs), sbf[ss], acc[d]);
  };
  // steady-state iteration j, hand-placed: C(j-1) from half uc of buffer bc (its transposed K
  // fragments tk read one iteration ahead), B(j) on (sj, dj), A(j+1) into (sn, dn) from half ua of
  // buffer ba; the last four slots read the NEXT iteration's tk (half un of buffer bn) into tkn, so
  // no iteration opens on an exposed LDS latency
  auto iteration = [&](int bc, int uc, f32x16& sj, f32x16& dj, int ba, int ua, f32x16& sn, f32x16& dn,
                       s16x8 (&tk)[2][DS], int bn, int un, s16x8 (&tkn)[2][DS]) {
    (void)bc;
    (void)uc;
    const char* ak = smem + ba * D_BUF;
    const char* av = ak + D_TILE;
    const char* nk = smem + bn * D_BUF;
    s16x8 ka[KS], va[KS];
    u32x4 sw[2];
#pragma unroll
    for (int m = 0; m < 12; ++m) {
      if (m < 4) {
        acc[m & 1] = mfma32(tk[m >> 1][m & 1], sbf[m >> 1], acc[m & 1]);
        ka[m] = row_frag<HD>(ak, ua * 32, m, lofs);
        va[m] = row_frag<HD>(av, ua * 32, m, lofs);
      } else {
        const int ks = (m - 4) >> 1;
        if (m & 1) dn = mfma32(va[ks], of[ks], ks == 0 ? ndl : dn);
        else sn = mfma32(ka[ks], qf[ks], ks == 0 ? f32x16{} : sn);
        if (m >= 8) tkn[(m - 8) >> 1][(m - 8) & 1] = tr_frag<HD>(nk, un * 32, (m - 8) >> 1, (m - 8) & 1, lofs);
      }
      if (m < 8) {
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          const int r = 2 * m + e;
          sj[r] = fast_exp2(fmaf(sj[r], c2, nlse));
        }
      } else {
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          const int w = 2 * (m - 8) + e, r = 2 * w;
          dj[r] = sj[r] * dj[r];
          dj[r + 1] = sj[r + 1] * dj[r + 1];
          uint32_t ws = cvt_pk(dj[r], dj[r + 1]);
          asm volatile("" : "+v"(ws));
          sw[w >> 2][w & 3] = ws;
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int ss = 0; ss < 2; ++ss) sbf[ss] = __builtin_bit_cast(s16x8, sw[ss]);
  };

  dma(0, 0);
  if (ntiles > 1) dma(1, 1);
  if (NB == 4 && ntiles > 2) dma(2, 2);
  tile_sync();
  f32x16 s0, d0, s1, d1;
  stage_A(0, 0, s0, d0);                // A(0)
  stage_A(0, 1, s1, d1);                // iteration 0: A(1), B(0)
  stage_B(s0, d0);
  int b0 = 0, b1 = 1;
  s16x8 tka[2][DS], tkb[2][DS];         // C's transposed K fragments, current / next
#pragma unroll
  for (int ss = 0; ss < 2; ++ss)
#pragma unroll
    for (int d = 0; d < DS; ++d) tka[ss][d] = tr_frag<HD>(smem, 0, ss, d, lofs);  // C(0): buffer 0, half 0
  for (int t = 0; t + 1 < ntiles; ++t) {
    if constexpr (NB == 4) {
      // tile t+1 landed (tile t+2's pieces may stay in flight), this wave's reads of tile t-1 done
      if (t + 2 < ntiles) __builtin_amdgcn_s_waitcnt(0x0074);  // vmcnt(4) lgkmcnt(0)
      else __builtin_amdgcn_s_waitcnt(0);
      asm volatile("" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      if (t + 3 < ntiles) dma(t + 3, (t + 3) & 3);  // into tile t-1's buffer
    } else {
      tile_sync();
      if (t + 2 < ntiles) dma(t + 2, (t + 2) % 3);
    }
    iteration(b0, 0, s1, d1, b1, 0, s0, d0, tka, b0, 1, tkb);  // C(2t), B(2t+1), A(2t+2)
    iteration(b0, 1, s0, d0, b1, 1, s1, d1, tkb, b1, 0, tka);  // C(2t+1), B(2t+2), A(2t+3)
    b0 = b1;
    b1 = NB == 4 ? (b1 + 1) & 3 : (b1 + 1) % 3;
  }
  stage_C(b0, 0);                       // C(J-2)
  stage_B(s1, d1);                      // B(J-1)
  stage_C(b0, 1);                       // C(J-1)

  if (!p.dq_f32) {  // dQ as whole rows through wave-private LDS slots
    __syncthreads();
    const int q0 = bx * D_QUERIES + wave * 32;
    if (q0 < p.Nq)
      store_rows_lds<HD>(smem + wave * 4096, acc, p.scale, (bf16_t*)p.dq + (int64_t)b * p.Nq * p.lddq + hh * HD,
                         p.lddq, q0, min(32, p.Nq - q0), lane);
    return;
  }
  if (qi >= p.Nq) return;
  if (p.dq_f32) {
    float* qrow = (float*)p.dq + ((int64_t)b * p.Nq + qi) * p.lddq + hh * HD;
#pragma unroll
    for (int d = 0; d < DS; ++d)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        f32x4 w = {acc[d][4 * g] * p.scale, acc[d][4 * g + 1] * p.scale, acc[d][4 * g + 2] * p.scale,
                   acc[d][4 * g + 3] * p.scale};
        *(f32x4*)(qrow + d * 32 + 8 * g + 4 * h) = w;
      }
  } else {
    bf16_t* qrow = (bf16_t*)p.dq + ((int64_t)b * p.Nq + qi) * p.lddq + hh * HD;
#pragma unroll
    for (int d = 0; d < DS; ++d)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        u32x2 w;
        w[0] = pack2(acc[d][4 * g] * p.scale, acc[d][4 * g + 1] * p.scale);
        w[1] = pack2(acc[d][4 * g + 2] * p.scale, acc[d][4 * g + 3] * p.scale);
        *(u32x2*)(qrow + d * 32 + 8 * g + 4 * h) = w;
      }
  }
}

bool dq_pipe_enabled() { return attn_switches().dq_pipe != 0; }  // LTX_ATTN_DQ_PIPE=0: the plain dQ kernel

static int dq_nbuf() { return attn_switches().dq_nbuf; }  // LTX_ATTN_DQ_NBUF=3: the 3-buffer ring

int launch_dq_pipe(const AttnParams& p, hipStream_t s) {
  const dim3 g((unsigned)((p.Nq + D_QUERIES - 1) / D_QUERIES), (unsigned)p.H, (unsigned)p.B);
  if (dq_nbuf() == 4)
    hipLaunchKernelGGL(attn_dq_pipe_kernel<4>, g, dim3(256), 0, s, p);
  else
    hipLaunchKernelGGL(attn_dq_pipe_kernel<3>, g, dim3(256), 0, s, p);
  LTX_LAUNCH_CHECK();
  return LTX_OK;
}

// =============================================================================================
// Forward for self-attention shapes (no key bias, Nk % 64 == 0): attn_q_kernel<64, 0, false, 8>'s
// arithmetic (8 waves x 32 queries, K/V tiles of 64 keys, speculative probabilities at the running
// max, deferred rescale) with the K / V tiles brought by LDS-DMA into a 3-buffer ring: no staging
// registers, no LDS write pass, one barrier per tile instead of two (-2 % in tools/attn_bench.py).
// Measured and not kept: 32-key sub-tiles with waves 4-7 staggered half a tile behind waves 0-3
// (neutral to +3 %).
// =============================================================================================
namespace {
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
constexpr int F_KT = 64;
constexpr int F_TILE = F_KT * PHD * 2;  // 8 KiB
constexpr int F_BUF = 2 * F_TILE;       // K | V
constexpr int F_QUERIES = 256;          // 8 waves x 32
}  // namespace

// F32SUM: the row sums are f32 adds of the probabilities (4 independent chains) instead of
// v_dot2c_f32_bf16 over their bf16 packs: 32 four-cycle adds per tile against 16 dot2c that each
// cost ~10 cycles beyond their issue slot beside MFMAs (MI355X_MICROARCH.md, filler prices). The
// sum is then the f32 one (as flash attention's), not the sum of the bf16-rounded weights.
template <bool F32SUM>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4, 4))) void attn_fwd_pipe_kernel(const AttnParams p) {
  constexpr int HD = PHD, KS = HD / 16, DS = HD / 32;
  __shared__ __attribute__((aligned(16))) char smem[P_NBUF * F_BUF];

  const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const LaneOfs<HD> lofs(lane);
  int bx, hh, b;
  xcd_block(p.xcd_order, bx, hh, b);
  const int qi = bx * F_QUERIES + wave * 32 + (lane & 31);
  const int qc = min(qi, p.Nq - 1);
  const float c2 = p.scale * LOG2E;

  s16x8 qf[KS];
  {
    const bf16_t* qr = p.q + ((int64_t)b * p.Nq + qc) * p.ldq + hh * HD;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) qf[ks] = *(const s16x8*)(qr + ks * 16 + 8 * h);
  }
  f32x16 acc[DS];
#pragma unroll
  for (int d = 0; d < DS; ++d)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[d][r] = 0.f;
  float m_run = -1e30f, l_run = 0.f;

  const bf16_t* kbase = p.k + (int64_t)b * p.kvb * p.ldk + hh * HD;
  const bf16_t* vbase = p.v + (int64_t)b * p.kvb * p.ldv + hh * HD;
  const int ntiles = p.Nk / F_KT;
  // key tile t -> buffer: wave w moves K rows 8w..8w+7 and V rows 8w..8w+7 (one piece each); a
  // lane's byte offset inside a tile is the same for every tile, the tile base is scalar
  const int drow = wave * 8 + (lane >> 3), dchunk = (lane & 7) ^ swz<HD>(drow);
  const uint32_t koff = (uint32_t)(drow * p.ldk + dchunk * 8) * 2, voff = (uint32_t)(drow * p.ldv + dchunk * 8) * 2;
  auto dma = [&](int t, int buf) {
    const uint32_t base = lds_u32(smem + buf * F_BUF + wave * 1024);
    dma16s(koff, kbase + (int64_t)t * F_KT * p.ldk, base);
    dma16s(voff, vbase + (int64_t)t * F_KT * p.ldv, base + F_TILE);
  };
  auto barrier = [&]() {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
  // barrier before tile t: this wave's DMA of tile t retired (issued two tiles ago; tile t+1's, issued
  // one tile ago, stays in flight), every wave done with tile t-1, whose buffer then takes tile t+2
  auto sync = [&](int t) {
    if (t + 1 < ntiles) __builtin_amdgcn_s_waitcnt(0x0F72);  // vmcnt(2)
    else __builtin_amdgcn_s_waitcnt(0x0F70);
    barrier();
    if (t + 2 < ntiles) dma(t + 2, (t + 2) % P_NBUF);
  };
  __builtin_amdgcn_s_waitcnt(0);  // the Q fragments: no ordinary load stays pending in the loop
  dma(0, 0);
  if (ntiles > 1) dma(1, 1);
  sync(0);

  f32x16 s[2];
  s16x8 pk[2][2];  // the tile's probabilities, bf16 (the PV product's B operand)
  float ls[4];
  for (int t = 0; t < ntiles; ++t) {
    const char* kt = smem + (t % P_NBUF) * F_BUF;
    const char* vt = kt + F_TILE;
    auto scores = [&]() {
      int z = 0;  // opaque: K fragment reads stay inside the pass loop (see attn_q_kernel)
      asm volatile("" : "+s"(z));
      const char* k2 = kt + z;
#pragma unroll
      for (int u = 0; u < 2; ++u) {
#pragma unroll
        for (int r = 0; r < 16; ++r) s[u][r] = 0.f;
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) s[u] = mfma32(row_frag<HD>(k2, u * 32, ks, lofs), qf[ks], s[u]);
      }
    };
    // row sums: F32SUM = f32 adds of the probabilities; else from the bf16 probabilities the PV
    // product consumes (v_dot2c_f32_bf16 against (1, 1)), O then normalised by the sum of exactly
    // the weights it was accumulated with
    auto probs = [&]() {
      const float nm = -m_run;
#pragma unroll
      for (int i = 0; i < 4; ++i) ls[i] = 0.f;
#pragma unroll
      for (int u = 0; u < 2; ++u) {
#pragma unroll
        for (int r = 0; r < 16; ++r) s[u][r] = fast_exp2(fmaf(s[u][r], c2, nm));
#pragma unroll
        for (int ss = 0; ss < 2; ++ss) {
          if constexpr (F32SUM) {  // this k-step's 8 probabilities, then their bf16 pack
#pragma unroll
            for (int r = 0; r < 8; ++r) ls[(2 * u + ss) & 3] += s[u][8 * ss + r];
          }
          pk[u][ss] = acc_frag(s[u], ss);
          if constexpr (!F32SUM) {
#pragma unroll
            for (int j = 0; j < 4; ++j)
              ls[(2 * u + ss) & 3] = __builtin_amdgcn_fdot2_f32_bf16(
                  as_bf16x2((unsigned)(unsigned short)pk[u][ss][2 * j] |
                            ((unsigned)(unsigned short)pk[u][ss][2 * j + 1] << 16)),
                  as_bf16x2(0x3F803F80u), ls[(2 * u + ss) & 3], false);
          }
        }
      }
    };
    float alpha = 1.f;
    bool rescale = false;
#pragma unroll 1
    for (int pass = (t == 0); pass < 2; ++pass) {
      scores();
      if (pass) {
        float mr[4] = {-3.0e38f, -3.0e38f, -3.0e38f, -3.0e38f};
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
          for (int r = 0; r < 16; ++r) mr[r & 3] = fmaxf(mr[r & 3], s[u][r]);
        const float mt = xor32_max(fmaxf(fmaxf(mr[0], mr[1]), fmaxf(mr[2], mr[3])) * c2);
        const float m_new = fmaxf(m_run, mt);
        if (__any(m_new > m_run + RESCALE_TAU)) {
          alpha = fast_exp2(m_run - m_new);
          rescale = true;
          m_run = m_new;
        }
      }
      probs();
      if (pass || !__any(((ls[0] + ls[1]) + (ls[2] + ls[3])) > RESCALE_SUM)) break;
    }
    if (rescale) {
      l_run *= alpha;
#pragma unroll
      for (int d = 0; d < DS; ++d)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[d][r] *= alpha;
    }
    l_run += (ls[0] + ls[1]) + (ls[2] + ls[3]);
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int ss = 0; ss < 2; ++ss)
#pragma unroll
        for (int d = 0; d < DS; ++d) acc[d] = mfma32(tr_frag<HD>(vt, u * 32, ss, d, lofs), pk[u][ss], acc[d]);
    if (t + 1 < ntiles) sync(t + 1);
  }

  const float l_tot = xor32_sum(l_run);
  const float inv = 1.0f / l_tot;
  // O through a wave-private LDS slot (the ring is free once every wave is past its last tile)
  __syncthreads();
  const int q0 = bx * F_QUERIES + wave * 32;
  store_rows_lds<HD>(smem + wave * 4096, acc, inv, p.o_out + (int64_t)b * p.Nq * p.ldo + hh * HD, p.ldo, q0,
                     min(32, p.Nq - q0), lane);
  if (qi < p.Nq && h == 0) p.lse[((int64_t)b * p.H + hh) * p.Nq + qi] = m_run + log2f(l_tot);
}

#ifdef LTX_FWD_W1
// =============================================================================================
// Forward at ONE wave per SIMD (self-attention shapes: no key bias, head dim 64, Nk % 64 == 0, >= 4
// key tiles): 4 waves x 64 queries (two 32-query tiles per wave) = 256 queries per workgroup, the
// loop one hand-scheduled asm statement (attn_fwd_body.h, tools/gen_attn_fwd.py: the unit schedule,
// the out-of-line redo of the deferred max). Same arithmetic, decisions and accumulation order as
// attn_fwd_pipe_kernel<true>: O and lse bitwise equal to it.
// =============================================================================================
__global__ __launch_bounds__(256, 1) void attn_fwd_w1_kernel(const AttnParams p) {
  constexpr int HD = PHD;
  __shared__ __attribute__((aligned(16))) char smem[LTX_FWD_W1_NBUF * LTX_FWD_W1_BUF];
  const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const LaneOfs<HD> lofs(lane);
  int bx, hh, b;
  xcd_block(p.xcd_order, bx, hh, b);
  const int q0 = bx * 256 + wave * 64;
  const bf16_t* qp[2];
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    const int qc = min(q0 + qt * 32 + (lane & 31), p.Nq - 1);
    qp[qt] = p.q + ((int64_t)b * p.Nq + qc) * p.ldq + hh * HD + 8 * h;
  }
  const bf16_t* kbase = p.k + (int64_t)b * p.kvb * p.ldk + hh * HD;
  const bf16_t* vbase = p.v + (int64_t)b * p.kvb * p.ldv + hh * HD;
  const u32x4 srdk = raw_srd(kbase, ((uint64_t)(p.Nk - 1) * p.ldk + HD) * 2);
  const u32x4 srdv = raw_srd(vbase, ((uint64_t)(p.Nk - 1) * p.ldv + HD) * 2);
  // DMA: wave w moves K rows 16 w .. 16 w + 15 (pieces 2w, 2w+1) and the same V rows of every tile
  uint32_t vk[2], vv[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = (wave * 2 + i) * 8 + (lane >> 3), c = (lane & 7) ^ swz<HD>(row);
    vk[i] = (uint32_t)(row * p.ldk + c * 8) * 2;
    vv[i] = (uint32_t)(row * p.ldv + c * 8) * 2;
  }
  const uint32_t wq0 = __builtin_amdgcn_readfirstlane(wave * 2048), wq1 = __builtin_amdgcn_readfirstlane(wave * 2048 + 1024);
  const uint32_t wqv0 = __builtin_amdgcn_readfirstlane(8192 + wave * 2048), wqv1 = __builtin_amdgcn_readfirstlane(8192 + wave * 2048 + 1024);
  const uint32_t lds0 = __builtin_amdgcn_readfirstlane(lds_u32(smem));
  const uint32_t kstep = __builtin_amdgcn_readfirstlane((uint32_t)(64 * p.ldk * 2));
  const uint32_t vstep = __builtin_amdgcn_readfirstlane((uint32_t)(64 * p.ldv * 2));
  const int U = p.Nk / 64;
  const uint32_t iters = __builtin_amdgcn_readfirstlane((uint32_t)((U - 2) / 2));
  const uint32_t uodd = __builtin_amdgcn_readfirstlane((uint32_t)(U & 1));
  const float c2 = p.scale * LOG2E;
  f32x16 a00 = {}, a01 = {}, a10 = {}, a11 = {};
  float m0 = -1e30f, m1 = -1e30f, l0 = 0.f, l1 = 0.f;
  uint64_t* stp = (uint64_t*)p.part +  // diagnostic bodies only (tools/build_fwd_variant.sh stamps)
                  ((blockIdx.x + (int64_t)gridDim.x * (blockIdx.y + (int64_t)gridDim.y * blockIdx.z)) * 4 + wave) * 8;
  asm volatile(LTX_FWD_W1_BODY
               : "+a"(a00), "+a"(a01), "+a"(a10), "+a"(a11), "+v"(m0), "+v"(m1), "+v"(l0), "+v"(l1)
               : [sk0] "s"(srd_half(srdk, 0)), [sk1] "s"(srd_half(srdk, 1)), [sv0] "s"(srd_half(srdv, 0)),
                 [sv1] "s"(srd_half(srdv, 1)), [kstep] "s"(kstep), [vstep] "s"(vstep), [lds0] "s"(lds0),
                 [wq0] "s"(wq0), [wq1] "s"(wq1), [wqv0] "s"(wqv0), [wqv1] "s"(wqv1), [iters] "s"(iters),
                 [uodd] "s"(uodd), [c2] "s"(c2), [vr0] "v"(lofs.row[0]), [vr1] "v"(lofs.row[1]),
                 [vr2] "v"(lofs.row[2]), [vr3] "v"(lofs.row[3]), [vt0] "v"(lofs.tr[0][0]), [vt1] "v"(lofs.tr[0][1]),
                 [vt2] "v"(lofs.tr[1][0]), [vt3] "v"(lofs.tr[1][1]), [vk0] "v"(vk[0]), [vk1] "v"(vk[1]),
                 [vv0] "v"(vv[0]), [vv1] "v"(vv[1]), [qp0] "v"(qp[0]), [qp1] "v"(qp[1]), [stp] "v"(stp)
               : "memory", "scc", "vcc", LTX_FWD_W1_CLOBBERS);
  // attn_fwd_pipe_kernel's epilogue per query tile (every DMA retired inside the statement)
  const f32x16 acc[2][2] = {{a00, a01}, {a10, a11}};
  const float mr[2] = {m0, m1}, lr[2] = {l0, l1};
  __syncthreads();
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    const float l_tot = xor32_sum(lr[qt]);
    const float inv = 1.0f / l_tot;
    const int qb = q0 + qt * 32;
    if (qb < p.Nq)
      store_rows_lds<HD>(smem + wave * 8192 + qt * 4096, acc[qt], inv, p.o_out + (int64_t)b * p.Nq * p.ldo + hh * HD,
                         p.ldo, qb, min(32, p.Nq - qb), lane);
    const int qi = qb + (lane & 31);
    if (qi < p.Nq && h == 0) p.lse[((int64_t)b * p.H + hh) * p.Nq + qi] = mr[qt] + log2f(l_tot);
  }
}

// LTX_ATTN_FWD_W1 (attn_switches(), `make fwdw1` builds only): 1 the one-wave forward where it applies; unset / 0 the pipelined
// kernel (12: the diagnostic bodies of tools/build_fwd_variant.sh, stamps into the stream's workspace).
// Not the default: its loop measures 2008 cycles per 64-key unit against 1024 of MFMA (1284 without
// the softmax VALU, profiles/r05d_fwd_w1_stamps.txt) -- at two exponentials per MFMA the one-wave
// schedule adds the VALU to the MFMA time almost linearly, and the eight-wave kernel is faster
// (220 vs 236 us per layer at config A)
bool fwd_w1_enabled(const AttnParams& p) {
  const int on = attn_switches().fwd_w1;
  return on != 0 && p.Nk % 64 == 0 && p.Nk >= 256;
}

int launch_fwd_w1(const AttnParams& p, hipStream_t s) {
  const dim3 g((unsigned)((p.Nq + 255) / 256), (unsigned)p.H, (unsigned)p.B);
  if (attn_switches().fwd_w1 == 12) {
    AttnParams q = p;
    size_t ws = 0;
    q.part = stream_workspace(s, &ws);
    if (q.part == nullptr || ws < (size_t)g.x * g.y * g.z * 4 * 8 * 8) return fail(LTX_ERR_BAD_ARG, "stamps: workspace");
    hipLaunchKernelGGL(attn_fwd_w1_kernel, g, dim3(256), 0, s, q);
    LTX_LAUNCH_CHECK();
    return LTX_OK;
  }
  hipLaunchKernelGGL(attn_fwd_w1_kernel, g, dim3(256), 0, s, p);
  LTX_LAUNCH_CHECK();
  return LTX_OK;
}

#else
static bool fwd_w1_enabled(const AttnParams&) { return false; }
static int launch_fwd_w1(const AttnParams&, hipStream_t) { return LTX_OK; }
#endif  // LTX_FWD_W1

bool fwd_pipe_enabled() { return attn_switches().fwd_pipe != 0; }  // LTX_ATTN_FWD_PIPE=0: attn_q_kernel<64, 0, false, 8>

static bool fwd_f32sum() { return attn_switches().fwd_f32sum != 0; }  // LTX_ATTN_FWD_F32SUM=0: v_dot2c row sums

int launch_fwd_pipe(const AttnParams& p, hipStream_t s) {
  if (fwd_w1_enabled(p)) return launch_fwd_w1(p, s);
  const dim3 g((unsigned)((p.Nq + F_QUERIES - 1) / F_QUERIES), (unsigned)p.H, (unsigned)p.B);
  if (fwd_f32sum())
    hipLaunchKernelGGL(attn_fwd_pipe_kernel<true>, g, dim3(512), 0, s, p);
  else
    hipLaunchKernelGGL(attn_fwd_pipe_kernel<false>, g, dim3(512), 0, s, p);
  LTX_LAUNCH_CHECK();
  return LTX_OK;
}

bool dkdv_pipe_enabled() { return attn_switches().dkdv_pipe != 0; }  // LTX_ATTN_DKDV_PIPE=0: the plain dK/dV kernel

static int dkdv_nbuf() { return attn_switches().dkdv_nbuf; }  // LTX_ATTN_DKDV_NBUF=3: the 3-buffer ring

int launch_dkdv_pipe(const AttnParams& p, hipStream_t s) {
  const dim3 g((unsigned)((p.Nk + P_KEYS - 1) / P_KEYS), (unsigned)p.H, (unsigned)p.B);
  const bool bias = p.key_bias != nullptr || (p.Nk % 64) != 0;
  if (dkdv_nbuf() == 4) {
    if (bias) hipLaunchKernelGGL((attn_dkdv_pipe_kernel<true, 4>), g, dim3(256), 0, s, p);
    else hipLaunchKernelGGL((attn_dkdv_pipe_kernel<false, 4>), g, dim3(256), 0, s, p);
  } else {
    if (bias) hipLaunchKernelGGL((attn_dkdv_pipe_kernel<true, 3>), g, dim3(256), 0, s, p);
    else hipLaunchKernelGGL((attn_dkdv_pipe_kernel<false, 3>), g, dim3(256), 0, s, p);
  }
  LTX_LAUNCH_CHECK();
  return LTX_OK;
}

}  // namespace ltx
