// Flash attention for the LTX-Video blocks on gfx950 (F.scaled_dot_product_attention,
// attention.py:1057-1064): self-attention over the spatio-temporal tokens (no mask) and the
// attn2 cross-attention over the caption tokens with the key-padding bias (1-mask)*-10000
// (transformer3d.py:441-445). Head dim 64 (LTX-2B) or 32 (tiny config).
//
// All products use v_mfma_f32_32x32x16_bf16 in the "swapped" orientation: the softmax axis
// lives in the accumulator REGISTERS and the other axis on the lanes, so
//   * row statistics need no cross-lane shuffles except one xor-32 exchange,
//   * the bf16-packed accumulator is directly the B operand of the next product (sum over the
//     register axis), and the matching A operand comes from a transposed LDS read
//     (ds_read_b64_tr_b16) of a row-major tile -- no LDS round trip for P or dS.
// LDS tiles are row-major [rows][HD] bf16 with a 16-B chunk XOR swizzle (swz below):
// conflict-free for both the 16-B row reads and the transposed reads of a 32-row fragment.
//
// Forward: a workgroup = 4 waves x 32 queries; K/V tiles of 64 keys are register-prefetched
// (global -> VGPR while the current tile computes) and written to LDS after a barrier.
// Per 64-key tile a wave runs 8 MFMAs for S^T = K.Q^T and 8 for O^T += V^T.P^T.
// lse is stored in log2 units: lse2 = max2 + log2(sum 2^(s*log2e - max2)).
//
// Backward (deterministic, no atomics): dq_kernel (workgroup = 128 queries, loop over keys:
// S^T, dP^T = V.dO^T, dS^T, dQ^T += K^T.dS^T) and dkdv_kernel (workgroup = 128 keys, each wave's
// 32 keys' K/V fragments in registers, loop over 32-query tiles: S, dP, dV^T += dO^T.P,
// dK^T += Q^T.dS). Recomputing S/dP in both costs two extra products per tile but removes the
// f32 atomics a fused kernel needs for dQ (which on MI355X would be bound by the ~1.3 TB/s
// atomic rate at these sizes).
#include <cstdlib>

#include "attention_common.h"
#include "ltx_hip.h"

namespace ltx {

// NW waves (NW x 32 queries) per workgroup: 4, or 8 to halve the K/V staging per query
template <int HD, int MODE, bool BIAS, int NW = 4>
__global__ __launch_bounds__(NW * 64, MODE == 1 ? 3 : 2) void attn_q_kernel(const AttnParams p) {
  constexpr int KT = 64;                 // keys per tile
  constexpr int KS = HD / 16;            // 16-deep k-steps over the head dim
  constexpr int DS = HD / 32;            // 32-wide d subtiles
  constexpr int TILE = KT * HD * 2;
  __shared__ __attribute__((aligned(16))) char smem[2 * TILE];
  __shared__ __attribute__((aligned(16))) float kb[KT];
  char* ktile = smem;
  char* vtile = smem + TILE;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h = lane >> 5;
  const LaneOfs<HD> lofs(lane);
  int bx, hh, b;
  xcd_block(p.xcd_order, bx, hh, b);
  const int q0 = bx * (NW * 32) + wave * 32;
  const int qi = q0 + (lane & 31);
  const int qc = min(qi, p.Nq - 1);
  const float c2 = p.scale * LOG2E;

  const bf16_t* kbase = p.k + (int64_t)b * p.kvb * p.ldk + hh * HD;
  const bf16_t* vbase = p.v + (int64_t)b * p.kvb * p.ldv + hh * HD;

  s16x8 qf[KS];
  {
    const bf16_t* qr = p.q + ((int64_t)b * p.Nq + qc) * p.ldq + hh * HD;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) qf[ks] = *(const s16x8*)(qr + ks * 16 + 8 * h);
  }
  s16x8 of[KS];
  float nlse = 0.f, dlt = 0.f;  // -lse2, delta (dQ mode)
  if constexpr (MODE == 1) {
    const bf16_t* dr = p.dout + ((int64_t)b * p.Nq + qc) * p.lddo + hh * HD;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) of[ks] = *(const s16x8*)(dr + ks * 16 + 8 * h);
    const int64_t si = ((int64_t)b * p.H + hh) * p.Nq + qc;
    nlse = -p.lse[si];
    dlt = p.delta[si];
  }

  f32x16 acc[DS];
#pragma unroll
  for (int d = 0; d < DS; ++d)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[d][r] = 0.f;
  float m_run = -1e30f, l_run = 0.f;  // m_run in scaled log2 units

  TileStage<HD, KT, NW * 64> ks_, vs_;
  const int ntiles = (p.Nk + KT - 1) / KT;
  ks_.load(kbase, p.ldk, 0, p.Nk, tid);
  vs_.load(vbase, p.ldv, 0, p.Nk, tid);
  ks_.store(ktile, tid);
  vs_.store(vtile, tid);
  if (BIAS) key_bias_tile(kb, p, b, 0, KT, tid);
  __syncthreads();

  // Retire every pre-loop global load (Q/dO/K/V fragments) with a counter wait hipcc can see:
  // otherwise its loop-header merge keeps them "pending" and each in-loop use waits with a
  // vmcnt that also drains the freshly issued tile prefetch.
  __builtin_amdgcn_s_waitcnt(0);
  for (int t = 0; t < ntiles; ++t) {
    const int key0 = t * KT;
    if (t + 1 < ntiles) {  // next K/V tile -> registers, written to LDS after this tile
      ks_.load(kbase, p.ldk, key0 + KT, p.Nk, tid);
      vs_.load(vbase, p.ldv, key0 + KT, p.Nk, tid);
    }
    f32x16 s[2];
    if constexpr (MODE == 1) {
      s16x8 kf[2][KS];  // dQ: all K fragments in flight before the first MFMA
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) kf[u][ks] = row_frag<HD>(ktile, u * 32, ks, lofs);
#pragma unroll
      for (int u = 0; u < 2; ++u) {
#pragma unroll
        for (int r = 0; r < 16; ++r) s[u][r] = 0.f;
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) s[u] = mfma32(kf[u][ks], qf[ks], s[u]);
      }
    }
    if constexpr (MODE == 0) {
      // forward: stay at <= 128 VGPRs (4 waves / SIMD). S^T for the tile's 64 keys:
      auto scores = [&]() {
        // opaque zero offset: keeps the K fragment reads inside the pass loop below (hoisted out
        // of it they would hold 32 more VGPRs for the whole tile)
        int z = 0;
        asm volatile("" : "+s"(z));
        const char* kt = ktile + z;
#pragma unroll
        for (int u = 0; u < 2; ++u) {
#pragma unroll
          for (int r = 0; r < 16; ++r) s[u][r] = 0.f;
#pragma unroll
          for (int ks = 0; ks < KS; ++ks) s[u] = mfma32(row_frag<HD>(kt, u * 32, ks, lofs), qf[ks], s[u]);
        }
      };
      // probabilities at the running max, the row sum in 4 chains (not one 32-deep add chain)
      float ls[4];
      auto probs = [&]() {
        const float nm = -m_run;
#pragma unroll
        for (int i = 0; i < 4; ++i) ls[i] = 0.f;
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            f32x4 kb4;
            if constexpr (BIAS) kb4 = *(const f32x4*)&kb[u * 32 + 8 * g + 4 * h];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const int r = 4 * g + i;
              const float e = BIAS ? fast_exp2(fmaf(s[u][r], c2, kb4[i]) + nm) : fast_exp2(fmaf(s[u][r], c2, nm));
              s[u][r] = e;
              ls[r & 3] += e;
            }
          }
      };
      // Speculative fast path (every tile but the first): exponentiate at the running max straight
      // away. A lane whose 32 probabilities sum to <= 2^TAU holds no score past m_run + TAU, so if
      // no lane of the wave exceeds that the deferred-max rule below would not rescale, and these
      // ARE the tile's probabilities: the per-tile max (16 v_max3 + a lane swap) is skipped. Else
      // (the first tile, or a max that grew by more than TAU) S is recomputed and the rule runs.
      // One loop body for both passes keeps a single copy of the S and P registers.
      float alpha = 1.f;
      bool rescale = false;
#pragma unroll 1
      for (int pass = (t == 0); pass < 2; ++pass) {
        scores();
        if (pass) {
          float mt = -1e30f;
          if constexpr (BIAS) {
#pragma unroll
            for (int u = 0; u < 2; ++u)
#pragma unroll
              for (int g = 0; g < 4; ++g) {
                const f32x4 kb4 = *(const f32x4*)&kb[u * 32 + 8 * g + 4 * h];
#pragma unroll
                for (int i = 0; i < 4; ++i) mt = fmaxf(mt, fmaf(s[u][4 * g + i], c2, kb4[i]));
              }
          } else {
            float mr[4] = {-3.0e38f, -3.0e38f, -3.0e38f, -3.0e38f};  // 4 chains: ILP for v_max3
#pragma unroll
            for (int u = 0; u < 2; ++u)
#pragma unroll
              for (int r = 0; r < 16; ++r) mr[r & 3] = fmaxf(mr[r & 3], s[u][r]);
            mt = fmaxf(fmaxf(mr[0], mr[1]), fmaxf(mr[2], mr[3])) * c2;
          }
          mt = xor32_max(mt);
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
      // O and l at the old max, rescaled once outside the pass loop (inside it, the conditionally
      // written O registers cost a copy of all of them per pass)
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
        for (int ss = 0; ss < 2; ++ss) {
          const s16x8 pb = acc_frag(s[u], ss);
#pragma unroll
          for (int d = 0; d < DS; ++d) acc[d] = mfma32(tr_frag<HD>(vtile, u * 32, ss, d, lofs), pb, acc[d]);
        }
    } else {
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        f32x16 dp;
        s16x8 vfr[KS];
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) vfr[ks] = row_frag<HD>(vtile, u * 32, ks, lofs);
#pragma unroll
        for (int r = 0; r < 16; ++r) dp[r] = 0.f;
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) dp = mfma32(vfr[ks], of[ks], dp);
        if constexpr (BIAS) {
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const f32x4 kb4 = *(const f32x4*)&kb[u * 32 + 8 * g + 4 * h];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const int r = 4 * g + i;
              const float pr = fast_exp2(fmaf(s[u][r], c2, kb4[i] + nlse));
              s[u][r] = pr * (dp[r] - dlt);
            }
          }
        } else {
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const float pr = fast_exp2(fmaf(s[u][r], c2, nlse));
            s[u][r] = pr * (dp[r] - dlt);
          }
        }
#pragma unroll
        for (int ss = 0; ss < 2; ++ss) {
          const s16x8 db = acc_frag(s[u], ss);
#pragma unroll
          for (int d = 0; d < DS; ++d) acc[d] = mfma32(tr_frag<HD>(ktile, u * 32, ss, d, lofs), db, acc[d]);
        }
      }
    }
    if (t + 1 < ntiles) {
      __syncthreads();
      ks_.store(ktile, tid);
      vs_.store(vtile, tid);
      if (BIAS) key_bias_tile(kb, p, b, key0 + KT, KT, tid);
      __syncthreads();
    }
  }

  if constexpr (MODE == 0 && HD == 64) {  // O rows in 16-B pieces (store_row_swap)
    const float l_tot = xor32_sum(l_run);
    store_row_swap<HD>(acc, 1.0f / l_tot, qi < p.Nq ? p.o_out + ((int64_t)b * p.Nq + qi) * p.ldo + hh * HD : nullptr,
                       lane);
    if (qi < p.Nq && h == 0) p.lse[((int64_t)b * p.H + hh) * p.Nq + qi] = m_run + log2f(l_tot);
    return;
  }
  if constexpr (MODE == 1 && HD == 64) {
    if (!p.dq_f32) {
      store_row_swap<HD>(acc, p.scale,
                         qi < p.Nq ? (bf16_t*)p.dq + ((int64_t)b * p.Nq + qi) * p.lddq + hh * HD : nullptr, lane);
      return;
    }
  }
  if (qi >= p.Nq) return;
  if constexpr (MODE == 0) {
    const float l_tot = xor32_sum(l_run);
    const float inv = 1.0f / l_tot;
    bf16_t* orow = p.o_out + ((int64_t)b * p.Nq + qi) * p.ldo + hh * HD;
#pragma unroll
    for (int d = 0; d < DS; ++d)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        u32x2 w;
        w[0] = pack2(acc[d][4 * g] * inv, acc[d][4 * g + 1] * inv);
        w[1] = pack2(acc[d][4 * g + 2] * inv, acc[d][4 * g + 3] * inv);
        *(u32x2*)(orow + d * 32 + 8 * g + 4 * h) = w;
      }
    if (h == 0) p.lse[((int64_t)b * p.H + hh) * p.Nq + qi] = m_run + log2f(l_tot);
  } else {
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
}

// =============================================================================================
// dK / dV: keys on lanes, queries in registers; workgroup = 4 waves x 32 keys. Query tiles of 64
// (two 32-row halves) between barrier pairs, so each wave runs 32 MFMAs per LDS refill.
// =============================================================================================
// NW waves (NW x 32 keys) per workgroup: 4, or 8 to halve the Q/dO staging per key
template <int HD, bool BIAS, int NW = 4>
__global__ __launch_bounds__(NW * 64, NW == 8 ? 1 : 2) void attn_dkdv_kernel(const AttnParams p) {
  constexpr int QT = 64;
  constexpr int KS = HD / 16;
  constexpr int DS = HD / 32;
  constexpr int TILE = QT * HD * 2;
  __shared__ __attribute__((aligned(16))) char smem[2 * TILE];
  __shared__ __attribute__((aligned(16))) float st_lse[QT];
  __shared__ __attribute__((aligned(16))) float st_dl[QT];
  char* qtile = smem;
  char* otile = smem + TILE;  // dO

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h = lane >> 5;
  const LaneOfs<HD> lofs(lane);
  int bx, hh, b;
  xcd_block(p.xcd_order, bx, hh, b);
  const int key = bx * (NW * 32) + wave * 32 + (lane & 31);
  const int kc = min(key, p.Nk - 1);
  const float c2 = p.scale * LOG2E;
  float kbias = 0.f;
  if (BIAS) {
    kbias = -INFINITY;
    if (key < p.Nk) kbias = p.key_bias ? p.key_bias[(int64_t)b * p.kvb + key] * LOG2E : 0.f;
  }

  s16x8 kf[KS], vf[KS];
  {
    const bf16_t* kr = p.k + ((int64_t)b * p.kvb + kc) * p.ldk + hh * HD;
    const bf16_t* vr = p.v + ((int64_t)b * p.kvb + kc) * p.ldv + hh * HD;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      kf[ks] = *(const s16x8*)(kr + ks * 16 + 8 * h);
      vf[ks] = *(const s16x8*)(vr + ks * 16 + 8 * h);
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
  TileStage<HD, QT, NW * 64> qs_, os_;
  const int ntiles = (p.Nq + QT - 1) / QT;
  // the next tile's -lse2 / delta ride in registers with the Q/dO prefetch (wave 0's lanes): a
  // load issued after the loop body would put one L2 round trip in every barrier interval
  float nl_next = 0.f, dl_next = 0.f;
  auto load_stats = [&](int qb) {
    if (tid < QT) {
      const int qq = min(qb + tid, p.Nq - 1);
      nl_next = -lbase[qq];
      dl_next = dbase[qq];
    }
  };
  auto store_stats = [&](int qb) {
    if (tid < QT) {
      const bool in = qb + tid < p.Nq;
      st_lse[tid] = in ? nl_next : -INFINITY;  // -lse2 (rows past Nq: P = 0)
      st_dl[tid] = in ? -dl_next : 0.f;  // -delta: the dP accumulator's initial value
    }
  };
  qs_.load(qbase, p.ldq, 0, p.Nq, tid);
  os_.load(obase, p.lddo, 0, p.Nq, tid);
  load_stats(0);
  qs_.store(qtile, tid);
  os_.store(otile, tid);
  store_stats(0);
  __syncthreads();

  // Retire every pre-loop global load (Q/dO/K/V fragments) with a counter wait hipcc can see:
  // otherwise its loop-header merge keeps them "pending" and each in-loop use waits with a
  // vmcnt that also drains the freshly issued tile prefetch.
  __builtin_amdgcn_s_waitcnt(0);
  for (int t = 0; t < ntiles; ++t) {
    const int qb = t * QT;
    if (t + 1 < ntiles) {
      qs_.load(qbase, p.ldq, qb + QT, p.Nq, tid);
      os_.load(obase, p.lddo, qb + QT, p.Nq, tid);
      load_stats(qb + QT);
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      // dP^T accumulates from -delta (st_dl holds -delta): dS = P * dP' needs no subtraction
      f32x16 s, dp;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const f32x4 dl4 = *(const f32x4*)&st_dl[u * 32 + 8 * g + 4 * h];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          s[4 * g + i] = 0.f;
          dp[4 * g + i] = dl4[i];
        }
      }
      s16x8 qfr[KS], ofr[KS];
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        qfr[ks] = row_frag<HD>(qtile, u * 32, ks, lofs);
        ofr[ks] = row_frag<HD>(otile, u * 32, ks, lofs);
      }
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        s = mfma32(qfr[ks], kf[ks], s);
        dp = mfma32(ofr[ks], vf[ks], dp);
      }
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const f32x4 nl4 = *(const f32x4*)&st_lse[u * 32 + 8 * g + 4 * h];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int r = 4 * g + i;
          const float pr = fast_exp2(fmaf(s[r], c2, BIAS ? kbias + nl4[i] : nl4[i]));
          s[r] = pr;
          dp[r] = pr * dp[r];
        }
      }
#pragma unroll
      for (int ss = 0; ss < 2; ++ss) {
        const s16x8 pb = acc_frag(s, ss);
        const s16x8 sb = acc_frag(dp, ss);
#pragma unroll
        for (int d = 0; d < DS; ++d) {
          dva[d] = mfma32(tr_frag<HD>(otile, u * 32, ss, d, lofs), pb, dva[d]);
          dka[d] = mfma32(tr_frag<HD>(qtile, u * 32, ss, d, lofs), sb, dka[d]);
        }
      }
    }
    if (t + 1 < ntiles) {
      __syncthreads();
      qs_.store(qtile, tid);
      os_.store(otile, tid);
      store_stats(qb + QT);
      __syncthreads();
    }
  }
  if constexpr (HD == 64) {  // dK, dV rows in 16-B pieces (store_row_swap)
    const bool kin = key < p.Nk;
    store_row_swap<HD>(dka, p.scale, kin ? p.dk + ((int64_t)b * p.Nk + key) * p.lddk + hh * HD : nullptr, lane);
    store_row_swap<HD>(dva, 1.0f, kin ? p.dv + ((int64_t)b * p.Nk + key) * p.lddv + hh * HD : nullptr, lane);
    return;
  }
  if (key >= p.Nk) return;
  bf16_t* krow = p.dk + ((int64_t)b * p.Nk + key) * p.lddk + hh * HD;
  bf16_t* vrow = p.dv + ((int64_t)b * p.Nk + key) * p.lddv + hh * HD;
#pragma unroll
  for (int d = 0; d < DS; ++d)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      u32x2 wk, wv;
      wk[0] = pack2(dka[d][4 * g] * p.scale, dka[d][4 * g + 1] * p.scale);
      wk[1] = pack2(dka[d][4 * g + 2] * p.scale, dka[d][4 * g + 3] * p.scale);
      wv[0] = pack2(dva[d][4 * g], dva[d][4 * g + 1]);
      wv[1] = pack2(dva[d][4 * g + 2], dva[d][4 * g + 3]);
      *(u32x2*)(krow + d * 32 + 8 * g + 4 * h) = wk;
      *(u32x2*)(vrow + d * 32 + 8 * g + 4 * h) = wv;
    }
}

// key ranges of at most this many run the one-pass kernels (one 8-wave workgroup holds them all)
constexpr int BWD1_KEYS = 256;
constexpr int BWD1_THREADS = 512;
// key bias (log2 units) at or below which a key counts as padding for tile skipping: the caption
// mask's bf16(-10000) * log2(e) = -14404, and -inf past Nk. Exact as long as the scaled scores of
// a row differ by less than ~(14404 - 10000) - 150 log2 units from its unmasked maximum.
constexpr float KEY_MASKED = -10000.0f;

// =============================================================================================
// Forward for key ranges of at most 256 (the attn2 cross-attention): a workgroup = 8 waves per
// (batch, head) stages ALL K / V rows (and the key bias) into LDS once; each wave then sweeps
// query slices w, w + 8, ... (32 queries each) with no barrier, the next slice's Q fragments
// loaded while the current slice computes. The split kernel (attn_q_kernel) reloads K/V per
// 128-query workgroup in 64-key tiles behind two barriers each, which at Nk = 256 is mostly
// exposed load latency. Arithmetic per slice is attn_q_kernel's MODE 0 loop, bit for bit.
// =============================================================================================
// ROWS (round 6): O leaves as whole 128-B rows through a 1-KiB LDS slot per wave, 8 rows per pass
// and store instruction (store_rows_lds1k; the slot fits beside the K / V images at two workgroups
// per CU), instead of the 32-B pieces of 32 rows per instruction store_row_swap writes. With
// HBM-resident operands (tools/cross_bench.py, profiles/r06p_cross_stores.txt) the forward ran 41 us,
// 24.6 us with no O stores at all, and 34 us with ROWS; a 16-wave workgroup with a 4-KiB slot per
// wave (one pass) spilled 17 registers and ran 39 us. Bitwise the same O and lse.
template <int HD, bool BIAS, bool ROWS>
__global__ __launch_bounds__(BWD1_THREADS) __attribute__((amdgpu_waves_per_eu(BIAS ? 4 : 2, 4))) void attn_fwd1_kernel(const AttnParams p) {
  constexpr int KT = 64;
  constexpr int KS = HD / 16;
  constexpr int DS = HD / 32;
  constexpr int IMG = BWD1_KEYS * HD * 2;
  __shared__ __attribute__((aligned(16))) char smem[2 * IMG + (ROWS ? 1024 * (BWD1_THREADS / 64) : 0)];
  __shared__ __attribute__((aligned(16))) float kb[BWD1_KEYS];
  char* kimg = smem;
  char* vimg = smem + IMG;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h = lane >> 5;
  const LaneOfs<HD> lofs(lane);
  const int hh = blockIdx.x, b = blockIdx.y;
  const float c2 = p.scale * LOG2E;
  {
    const bf16_t* kbase = p.k + (int64_t)b * p.kvb * p.ldk + hh * HD;
    const bf16_t* vbase = p.v + (int64_t)b * p.kvb * p.ldv + hh * HD;
    TileStage<HD, BWD1_KEYS, BWD1_THREADS> ks_, vs_;
    ks_.load(kbase, p.ldk, 0, p.Nk, tid);
    vs_.load(vbase, p.ldv, 0, p.Nk, tid);
    ks_.store(kimg, tid);
    vs_.store(vimg, tid);
    if (BIAS && tid < BWD1_KEYS) {
      float v = -INFINITY;
      if (tid < p.Nk) v = p.key_bias ? p.key_bias[(int64_t)b * p.kvb + tid] * LOG2E : 0.f;
      kb[tid] = v;
    }
  }
  __syncthreads();
  const int ntiles = (p.Nk + KT - 1) / KT;
  const int nslices = (p.Nq + 31) / 32;
  // Key tiles whose every key is padding (bias <= KEY_MASKED: the caption mask's -10000) hold
  // probabilities that underflow to exactly 0 behind any unmasked key, so skipping them leaves O
  // and lse bitwise unchanged (a leading masked tile is erased by the first rescale, alpha = 0).
  // A row with no unmasked key at all keeps every tile (the reference's uniform softmax).
  unsigned act = ~0u;
  if (BIAS && p.skip_masked) {
    act = 0u;
    for (int t = 0; t < ntiles; ++t)
      if (__any(kb[min(t * KT + lane, BWD1_KEYS - 1)] > KEY_MASKED)) act |= 1u << t;
    if (act == 0u) act = ~0u;
  }
  const bf16_t* qb = p.q + (int64_t)b * p.Nq * p.ldq + hh * HD;
  s16x8 qn[KS];
  auto load_q = [&](int sl) {
    const int qc = min(sl * 32 + (lane & 31), p.Nq - 1);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) qn[ks] = *(const s16x8*)(qb + (int64_t)qc * p.ldq + ks * 16 + 8 * h);
  };
  // blockIdx.z of gridDim.z workgroups per (batch, head) takes every gridDim.z-th 8-slice group
  const int sstep = (BWD1_THREADS / 64) * gridDim.z;
  const int s0 = wave + (BWD1_THREADS / 64) * blockIdx.z;
  for (int sl = s0; sl < nslices; sl += sstep) {
    // (no cross-slice Q prefetch: at two workgroups per CU the other one covers the load, and
    // its 16 registers would push the kernel past the 128 that 4 waves per SIMD allow)
    load_q(sl);
    s16x8 qf[KS];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) qf[ks] = qn[ks];
    f32x16 acc[DS];
#pragma unroll
    for (int d = 0; d < DS; ++d)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[d][r] = 0.f;
    float m_run = -1e30f, l_run = 0.f;
    for (int t = 0; t < ntiles; ++t) {
      if (!((act >> t) & 1u)) continue;
      const int k0 = t * KT;
      f32x16 s[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
#pragma unroll
        for (int r = 0; r < 16; ++r) s[u][r] = 0.f;
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) s[u] = mfma32(row_frag<HD>(kimg, k0 + u * 32, ks, lofs), qf[ks], s[u]);
      }
      float mt = -1e30f;
      if constexpr (BIAS) {
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const f32x4 kb4 = *(const f32x4*)&kb[k0 + u * 32 + 8 * g + 4 * h];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const float x = fmaf(s[u][4 * g + i], c2, kb4[i]);
              s[u][4 * g + i] = x;
              mt = fmaxf(mt, x);
            }
          }
      } else {
        float mr[4] = {-3.0e38f, -3.0e38f, -3.0e38f, -3.0e38f};
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
          for (int r = 0; r < 16; ++r) mr[r & 3] = fmaxf(mr[r & 3], s[u][r]);
        mt = fmaxf(fmaxf(mr[0], mr[1]), fmaxf(mr[2], mr[3])) * c2;
      }
      mt = xor32_max(mt);
      const float m_new = fmaxf(m_run, mt);
      if (__any(m_new > m_run + RESCALE_TAU)) {
        const float alpha = fast_exp2(m_run - m_new);
        l_run *= alpha;
#pragma unroll
        for (int d = 0; d < DS; ++d)
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[d][r] *= alpha;
        m_run = m_new;
      }
      const float nm = -m_run;
      float ls[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float e = BIAS ? fast_exp2(s[u][r] + nm) : fast_exp2(fmaf(s[u][r], c2, nm));
          s[u][r] = e;
          ls[r & 3] += e;
        }
      l_run += (ls[0] + ls[1]) + (ls[2] + ls[3]);
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int ss = 0; ss < 2; ++ss) {
          const s16x8 pb = acc_frag(s[u], ss);
#pragma unroll
          for (int d = 0; d < DS; ++d) acc[d] = mfma32(tr_frag<HD>(vimg, k0 + u * 32, ss, d, lofs), pb, acc[d]);
        }
    }
    const int qi = sl * 32 + (lane & 31);
    const float l_tot = xor32_sum(l_run);
    const float inv = 1.0f / l_tot;
    // O rows in 16-B pieces (32 contiguous bytes per row per store instruction; the 8-B pieces of
    // the per-lane layout took half the kernel's time)
    if constexpr (ROWS)
      store_rows_lds1k<HD>(smem + 2 * IMG + wave * 1024, acc, inv, p.o_out + (int64_t)b * p.Nq * p.ldo + hh * HD,
                           p.ldo, sl * 32, min(32, p.Nq - sl * 32), lane);
    else
      store_row_swap<HD>(acc, inv, qi < p.Nq ? p.o_out + ((int64_t)b * p.Nq + qi) * p.ldo + hh * HD : nullptr, lane);
    if (qi < p.Nq && h == 0) p.lse[((int64_t)b * p.H + hh) * p.Nq + qi] = m_run + log2f(l_tot);
  }
}

// =============================================================================================
// One-pass backward for key ranges of at most 256 (the attn2 cross-attention over the caption
// tokens): a workgroup = 8 waves x 32 keys holds EVERY key of one (batch, head), so dQ needs no
// sum across workgroups and S / dP are computed once per tile instead of once in each of the
// dK/dV and dQ kernels (5 MFMA products per tile instead of 7).
// Per 64-query tile: the dK/dV kernel's S, dP, dV^T += dO^T.P, dK^T += Q^T.dS (keys on lanes);
// dS (bf16, the same rounding the dK product uses) goes to an LDS image [key][query]; after a
// barrier each wave computes dQ^T = K^T.dS^T for HD/32 16x16 output tiles over all 256 keys
// (v_mfma_f32_16x16x32_bf16, both operands by transposed reads of the [key][.] images, so the
// lane holds 4 consecutive head dims of one query: 8-byte stores).
// k-slot order inside a 32-key step: slots 8g + j (g = lane >> 4) stand for keys 4g + j (j < 4)
// and 16 + 4g + j - 4 (j >= 4), the same on both operands; each 32-lane half then reads 8
// consecutive image rows, which the row swizzle keeps conflict-free.
// =============================================================================================

// Few unmasked keys (the caption's padded prompt: 16 valid tokens of 256): when every unmasked
// key of the (batch, head) lies in ONE 32-key block kb, the 8-wave kernel below leaves 7 waves with
// only a dQ share of each tile and the whole S / dP / dV / dK chain on one wave, behind a barrier
// per 64-query tile (~2.5 us per tile at config A). Here each wave instead takes its own 32-query
// sub-tiles (w, w + 8, ...) end to end with no workgroup barrier in the loop:
//   * Q / dO rows (and the lse / delta words) of a sub-tile by LDS-DMA into a wave-private
//     2-slot ring, the next sub-tile's DMA in flight while this one computes;
//   * S, dP, P, dS, dV^T += dO^T.P and dK^T += Q^T.dS exactly as one u-half of attn_bwd1_kernel
//     (this lane's key = kb * 32 + (lane & 31) in every wave);
//   * dS (bf16) into a wave-private [32 keys][32 queries] image, dQ^T = K^T.dS^T of the sub-tile
//     (4 head-dim blocks x 2 query blocks, v_mfma_f32_16x16x32_bf16 over the block's 32 keys: the
//     same single k-step as the 8-wave kernel's, so dQ is bitwise its dQ);
//   * the 8 waves' dK / dV partials summed through LDS in wave order at the end (f32 rounding away
//     from the 8-wave kernel, whose one wave summed every tile in sequence); all other keys' dK /
//     dV rows are stored as zeros, as there.
namespace {
constexpr int FK_SLOT = 2 * 32 * 128 + 256;      // Q | dO (32 rows x 128 B each) | lse | delta
constexpr int FK_RING = 8 * 2 * FK_SLOT;          // 8 waves x 2 slots
constexpr int FK_SIMG = 32 * 64;                  // dS image [32 keys][32 queries] bf16, per wave
constexpr int FK_KIMG = 32 * 128;                 // K rows of the active block
constexpr int FK_LDS = FK_RING + 8 * FK_SIMG + FK_KIMG;
constexpr int FK_NST = 4;  // dQ store instructions per sub-tile (bf16 rows through the dS image)
static_assert(8 * 4 * 16 * 64 * 4 <= FK_RING, "the dK / dV partials fit the ring");
}  // namespace

template <int HD>
__device__ __forceinline__ void bwd1_few_keys(const AttnParams& p, char* smem, int kb, int b, int hh) {
  static_assert(HD == 64, "head dim 64");
  constexpr int KS = HD / 16, DS = HD / 32;
  const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const LaneOfs<HD> lofs(lane);
  char* ring = smem + wave * (2 * FK_SLOT);
  char* simg = smem + FK_RING + wave * FK_SIMG;
  char* kimg = smem + FK_RING + 8 * FK_SIMG;
  const int kl = kb * 32 + (lane & 31);  // this lane's key (the same in every wave)
  const int kc = min(kl, p.Nk - 1);
  const float c2 = p.scale * LOG2E;
  float kbias = -INFINITY;
  if (kl < p.Nk) kbias = p.key_bias ? p.key_bias[(int64_t)b * p.kvb + kl] * LOG2E : 0.f;
  const bf16_t* kbase = p.k + (int64_t)b * p.kvb * p.ldk + hh * HD;
  // sub-tiles of this wave: st = wave + 8 i (32 queries each)
  const int nsub = (p.Nq + 31) / 32;
  const int nmine = nsub > wave ? (nsub - wave + 7) / 8 : 0;
  const bf16_t* qbase = p.q + (int64_t)b * p.Nq * p.ldq + hh * HD;
  const bf16_t* obase = p.dout + (int64_t)b * p.Nq * p.lddo + hh * HD;
  const float* lbase = p.lse + ((int64_t)b * p.H + hh) * p.Nq;
  const float* dbase = p.delta + ((int64_t)b * p.H + hh) * p.Nq;
  // DMA piece i of a sub-tile: rows 8i + (lane >> 3), physical chunk lane & 7 (the source chunk
  // swizzled as toff expects); rows past Nq re-read the last row (their lse is set to +inf)
  auto dma = [&](int i) {
    const int q0 = (wave + 8 * i) * 32;
    char* slot = ring + (i & 1) * FK_SLOT;
#pragma unroll
    for (int pc = 0; pc < 4; ++pc) {
      const int row = 8 * pc + (lane >> 3);
      const int qr = min(q0 + row, p.Nq - 1);
      const int ch = (lane & 7) ^ swz<HD>(row);
      dma16s((uint32_t)(qr * p.ldq + ch * 8) * 2, qbase, lds_u32(slot + pc * 1024));
      dma16s((uint32_t)(qr * p.lddo + ch * 8) * 2, obase, lds_u32(slot + 4096 + pc * 1024));
    }
    const int qs = min(q0 + (lane & 31), p.Nq - 1);
    dma4((lane < 32 ? lbase : dbase) + qs, lds_u32(slot + 8192));
  };
  // the first two sub-tiles' DMA goes out ahead of this lane's K / V fragments and the K image
  // (their latencies overlap); everything retired before the counted waits below
  if (nmine > 0) dma(0);
  if (nmine > 1) dma(1);
  s16x8 kf[KS], vf[KS];
  {
    const bf16_t* kr = kbase + (int64_t)kc * p.ldk;
    const bf16_t* vr = p.v + ((int64_t)b * p.kvb + kc) * p.ldv + hh * HD;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      kf[ks] = *(const s16x8*)(kr + ks * 16 + 8 * h);
      vf[ks] = *(const s16x8*)(vr + ks * 16 + 8 * h);
    }
  }
  if (tid < 256) {  // K image of the block's 32 rows (the dQ product's A operand, swizzled)
    const int r = tid >> 3, c = tid & 7;
    const int key = min(kb * 32 + r, p.Nk - 1);
    *(u32x4*)(kimg + toff<HD>(r, c)) = *(const u32x4*)(kbase + (int64_t)key * p.ldk + c * 8);
  }
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  f32x16 dka[DS], dva[DS];
#pragma unroll
  for (int d = 0; d < DS; ++d)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      dka[d][r] = 0.f;
      dva[d][r] = 0.f;
    }
  // dQ operand offsets: K^T (head-dim block db) and dS^T (query block qb) by transposed reads
  const int g4 = lane >> 4, qq = (lane & 15) >> 2, pp = lane & 3;
  int offk[4], offs[2];
#pragma unroll
  for (int db = 0; db < 4; ++db) offk[db] = toff<HD>(4 * g4 + qq, 2 * db + (pp >> 1)) + 8 * (pp & 1);
#pragma unroll
  for (int qb = 0; qb < 2; ++qb) offs[qb] = toff<32>(4 * g4 + qq, 2 * qb + (pp >> 1)) + 8 * (pp & 1);
  auto tr4 = [](const char* a) {
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)a);
  };
  const int srow = (lane & 31) * 64 + 8 * h;  // this lane's dS image row (+ chunk ^ swizzle)
  const int sw4 = swz<32>(lane & 31);
  for (int i = 0; i < nmine; ++i) {
    // this sub-tile's 9 DMA instructions landed: younger than them are the next sub-tile's 9 (issued
    // in iteration i - 1) and iteration i - 1's dQ stores (inline asm, so exactly FK_NST; CDNA4's
    // vmcnt counts stores too)
    if (i + 1 < nmine && i >= 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(9 + FK_NST) : "memory");
    else if (i + 1 < nmine) asm volatile("s_waitcnt vmcnt(9)" ::: "memory");
    else if (i >= 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(FK_NST) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int q0 = (wave + 8 * i) * 32;
    char* slot = ring + (i & 1) * FK_SLOT;
    const char* qtile = slot;
    const char* otile = slot + 4096;
    float* sl = (float*)(slot + 8192);
    const float* sd = sl + 32;
    if (q0 + 32 > p.Nq && lane < 32 && q0 + lane >= p.Nq) sl[lane] = INFINITY;  // P = dS = 0 there
    f32x16 s, dp;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      s[r] = 0.f;
      dp[r] = 0.f;
    }
    s16x8 qfr[KS], ofr[KS];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      qfr[ks] = row_frag<HD>(qtile, 0, ks, lofs);
      ofr[ks] = row_frag<HD>(otile, 0, ks, lofs);
    }
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      s = mfma32(qfr[ks], kf[ks], s);
      dp = mfma32(ofr[ks], vf[ks], dp);
    }
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const f32x4 l4 = *(const f32x4*)&sl[8 * g + 4 * h];
      const f32x4 dl4 = *(const f32x4*)&sd[8 * g + 4 * h];
#pragma unroll
      for (int ii = 0; ii < 4; ++ii) {
        const int r = 4 * g + ii;
        const float pr = fast_exp2(fmaf(s[r], c2, kbias - l4[ii]));
        s[r] = pr;
        dp[r] = pr * (dp[r] - dl4[ii]);
      }
    }
#pragma unroll
    for (int ss = 0; ss < 2; ++ss) {
      const s16x8 pb = acc_frag(s, ss);
      const s16x8 sb = acc_frag(dp, ss);
#pragma unroll
      for (int d = 0; d < DS; ++d) {
        dva[d] = mfma32(tr_frag<HD>(otile, 0, ss, d, lofs), pb, dva[d]);
        dka[d] = mfma32(tr_frag<HD>(qtile, 0, ss, d, lofs), sb, dka[d]);
      }
      // registers 8ss + 4gg + ii are queries 16ss + 8gg + 4h + ii: chunk 2ss + gg, half h
#pragma unroll
      for (int gg = 0; gg < 2; ++gg) {
        u32x2 w;
        w[0] = (unsigned)(unsigned short)sb[4 * gg] | ((unsigned)(unsigned short)sb[4 * gg + 1] << 16);
        w[1] = (unsigned)(unsigned short)sb[4 * gg + 2] | ((unsigned)(unsigned short)sb[4 * gg + 3] << 16);
        *(u32x2*)(simg + srow + (((2 * ss + gg) ^ sw4) << 4)) = w;
      }
    }
    // every read of this slot and the dS image writes done: the slot takes sub-tile i + 2
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (i + 2 < nmine) dma(i + 2);
    // dQ^T (16 dims x 16 queries per MFMA) over the block's 32 keys
    f32x4 dqa[4][2];
    s16x8 bv[2];
#pragma unroll
    for (int qb = 0; qb < 2; ++qb) {
      const s16x4 b0 = tr4(simg + offs[qb]), b1 = tr4(simg + offs[qb] + 16 * 64);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        bv[qb][j] = b0[j];
        bv[qb][4 + j] = b1[j];
      }
    }
#pragma unroll
    for (int db = 0; db < 4; ++db) {
      const s16x4 a0 = tr4(kimg + offk[db]), a1 = tr4(kimg + offk[db] + 16 * (HD * 2));
      s16x8 av;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        av[j] = a0[j];
        av[4 + j] = a1[j];
      }
#pragma unroll
      for (int qb = 0; qb < 2; ++qb)
        dqa[db][qb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bv[qb], (f32x4){0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
    }
    // the stores: FK_NST asm instructions while another sub-tile follows (only the last sub-tile of
    // the (batch, head) can be ragged, and it is its wave's last)
    const bool last = i + 1 == nmine;
    if (!p.dq_f32) {
      // bf16 dQ as whole 128-B rows (round 6): each 16-query half through the wave's dS image (its
      // reads are done), 16-B chunks XOR row & 7, then 8 rows per store instruction. The lane's
      // pieces (4 dims of one query per head-dim block) as direct stores were 16 partial lines per
      // instruction: the kernel ran 57 us against 34 us with no dQ stores at all (HBM-resident
      // operands, tools/cross_bench.py, profiles/r06p_cross_stores.txt).
      char* dimg = simg;
#pragma unroll
      for (int qb = 0; qb < 2; ++qb) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the image's previous reads are done
        const int row = lane & 15;
#pragma unroll
        for (int db = 0; db < 4; ++db) {
          u32x2 w;
          w[0] = pack2(dqa[db][qb][0] * p.scale, dqa[db][qb][1] * p.scale);
          w[1] = pack2(dqa[db][qb][2] * p.scale, dqa[db][qb][3] * p.scale);
          const int c = 2 * db + (g4 >> 1);
          *(u32x2*)(dimg + row * 128 + ((c ^ (row & 7)) << 4) + 8 * (g4 & 1)) = w;
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        u32x4 rv[2];
#pragma unroll
        for (int h2 = 0; h2 < 2; ++h2) {
          const int rr = 8 * h2 + (lane >> 3), c = lane & 7;
          rv[h2] = *(const u32x4*)(dimg + rr * 128 + ((c ^ (rr & 7)) << 4));
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
        for (int h2 = 0; h2 < 2; ++h2) {
          const int q = q0 + 16 * qb + 8 * h2 + (lane >> 3);
          bf16_t* dst = (bf16_t*)p.dq + ((int64_t)b * p.Nq + min(q, p.Nq - 1)) * p.lddq + (int64_t)hh * HD + 8 * (lane & 7);
          if (!last) asm volatile("global_store_dwordx4 %0, %1, off" ::"v"(dst), "v"(rv[h2]) : "memory");
          else if (q < p.Nq) *(u32x4*)dst = rv[h2];
        }
      }
      continue;
    }
#pragma unroll
    for (int qb = 0; qb < 2; ++qb) {
      const int q = q0 + 16 * qb + (lane & 15);
#pragma unroll
      for (int db = 0; db < 4; ++db) {
        const int64_t off = ((int64_t)b * p.Nq + min(q, p.Nq - 1)) * p.lddq + (int64_t)hh * HD + 16 * db + 4 * g4;
        if (p.dq_f32) {
          const f32x4 w = {dqa[db][qb][0] * p.scale, dqa[db][qb][1] * p.scale, dqa[db][qb][2] * p.scale,
                           dqa[db][qb][3] * p.scale};
          float* dst = (float*)p.dq + off;
          if (!last) asm volatile("global_store_dwordx4 %0, %1, off" ::"v"(dst), "v"(w) : "memory");
          else if (q < p.Nq) *(f32x4*)dst = w;
        } else {
          u32x2 w;
          w[0] = pack2(dqa[db][qb][0] * p.scale, dqa[db][qb][1] * p.scale);
          w[1] = pack2(dqa[db][qb][2] * p.scale, dqa[db][qb][3] * p.scale);
          bf16_t* dst = (bf16_t*)p.dq + off;
          if (!last) asm volatile("global_store_dwordx2 %0, %1, off" ::"v"(dst), "v"(w) : "memory");
          else if (q < p.Nq) *(u32x2*)dst = w;
        }
      }
    }
  }
  // dK / dV partials of the 8 waves through LDS (the ring is free once every wave is done), summed
  // in wave order: wave 0 dK, wave 1 dV; waves 2-7 store the zero rows of every other key
  __syncthreads();
  float* part = (float*)smem;  // [wave][acc a][r][lane], a = 2 d + (0: dK, 1: dV)
#pragma unroll
  for (int d = 0; d < DS; ++d)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      part[((wave * 4 + 2 * d) * 16 + r) * 64 + lane] = dka[d][r];
      part[((wave * 4 + 2 * d + 1) * 16 + r) * 64 + lane] = dva[d][r];
    }
  __syncthreads();
  if (wave < 2) {
    f32x16 acc[DS];
#pragma unroll
    for (int d = 0; d < DS; ++d)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        float sum = part[((0 * 4 + 2 * d + wave) * 16 + r) * 64 + lane];
#pragma unroll
        for (int w = 1; w < 8; ++w) sum += part[((w * 4 + 2 * d + wave) * 16 + r) * 64 + lane];
        acc[d][r] = sum;
      }
    const bool kin = kl < p.Nk;
    if (wave == 0)
      store_row_swap<HD>(acc, p.scale, kin ? p.dk + ((int64_t)b * p.Nk + kl) * p.lddk + hh * HD : nullptr, lane);
    else
      store_row_swap<HD>(acc, 1.0f, kin ? p.dv + ((int64_t)b * p.Nk + kl) * p.lddv + hh * HD : nullptr, lane);
  } else {
    // zero rows: keys outside the block, 16 B per lane-store (8 per 128-B row), dK then dV
    const int nz = p.Nk - min(32, p.Nk - kb * 32);
    for (int e = (wave - 2) * 64 + lane; e < 2 * nz * 8; e += 6 * 64) {
      const int t = e / (nz * 8), rem = e % (nz * 8);
      int key = rem / 8;
      if (key >= kb * 32) key += 32;
      const int c = rem % 8;
      bf16_t* row = t == 0 ? p.dk + ((int64_t)b * p.Nk + key) * p.lddk : p.dv + ((int64_t)b * p.Nk + key) * p.lddv;
      *(u32x4*)(row + hh * HD + c * 8) = (u32x4){0u, 0u, 0u, 0u};
    }
  }
}

// QS (biased key ranges): when every unmasked key lies below 128 (the caption's padded prompt),
// waves w and w + 4 hold the same 32 keys and take the two 32-query halves of each tile (instead
// of the padding-key waves idling and the others running both halves); their dK / dV partials
// are added through LDS at the end.
template <int HD, bool BIAS, bool QS>
__global__ __launch_bounds__(BWD1_THREADS, 1) void attn_bwd1_kernel(const AttnParams p) {
  constexpr int QT = 64;
  constexpr int KS = HD / 16;
  constexpr int DS = HD / 32;
  constexpr int TILE = QT * HD * 2;
  constexpr int KIMG = BWD1_KEYS * HD * 2;  // K image [key][HD]
  constexpr int SIMG = BWD1_KEYS * QT * 2;  // dS image [key][64 queries], two of them
  constexpr int NDB = HD / 16;              // 16-wide head-dim blocks of dQ
  constexpr int QBW = HD / 32;              // 16-query blocks per wave (4 * NDB / 8 waves)
  constexpr int KSTEPS = BWD1_KEYS / 32;    // 32-key steps of the dQ product
  // Q / dO tiles and their lse / delta words arrive by LDS-DMA into a 3-slot ring (two tiles in
  // flight behind the one being computed); ONE shared array (a second __shared__ object beside the
  // DMA target makes hipcc wait for the DMA before unrelated LDS reads)
  constexpr int STAT = QT * 4;
  constexpr int SLOT = 2 * TILE + 2 * STAT;  // Q | dO | lse | delta
  constexpr int NSLOT = 3;
  constexpr int OLD_LDS = NSLOT * SLOT + KIMG + 2 * SIMG;
  __shared__ __attribute__((aligned(16))) char smem[(BIAS && !QS && HD == 64 && FK_LDS > OLD_LDS) ? FK_LDS : OLD_LDS];
  char* kimg = smem + NSLOT * SLOT;
  char* simg0 = kimg + KIMG;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h = lane >> 5;
  const LaneOfs<HD> lofs(lane);
  const int hh = blockIdx.x, b = blockIdx.y;
  // active 32-key blocks (bit kb: a key of kb*32 .. +31 above the padding bias), the same in every
  // wave. 32-key blocks whose keys are all padding have P = dS = 0 exactly behind any unmasked key:
  // their S / dP / dK / dV work and their dQ k-steps are skipped (dK = dV = 0 are still stored),
  // which leaves every output bitwise unchanged (see attn_fwd1_kernel).
  unsigned kact = 0xffu;
  if (BIAS && p.skip_masked) {
    kact = 0u;
#pragma unroll
    for (int kb = 0; kb < 8; ++kb) {
      const int key = kb * 32 + (lane & 31);
      float kbv = -INFINITY;
      if (key < p.Nk) kbv = p.key_bias ? p.key_bias[(int64_t)b * p.kvb + key] * LOG2E : 0.f;
      if (__any(kbv > KEY_MASKED)) kact |= 1u << kb;
    }
    if (kact == 0u) kact = 0xffu;  // no unmasked key at all: keep everything
  }
  if constexpr (BIAS && !QS && HD == 64) {
    // one active 32-key block: every wave takes its own query sub-tiles (bwd1_few_keys)
    if (p.few_keys && p.qsplit == 1 && __builtin_popcount(kact) == 1) {
      bwd1_few_keys<HD>(p, smem, __builtin_ctz(kact), b, hh);
      return;
    }
  }
  const bool qs = QS && (kact & 0xf0u) == 0u;  // every active key below 128: split the queries
  const int kl = (qs ? (wave & 3) : wave) * 32 + (lane & 31);  // this lane's key
  const int kc = min(kl, p.Nk - 1);
  const float c2 = p.scale * LOG2E;
  float kbias = 0.f;
  if (BIAS) {
    kbias = -INFINITY;
    if (kl < p.Nk) kbias = p.key_bias ? p.key_bias[(int64_t)b * p.kvb + kl] * LOG2E : 0.f;
  }
  const bf16_t* kbase = p.k + (int64_t)b * p.kvb * p.ldk + hh * HD;
  s16x8 kf[KS], vf[KS];
  {
    const bf16_t* kr = kbase + (int64_t)kc * p.ldk;
    const bf16_t* vr = p.v + ((int64_t)b * p.kvb + kc) * p.ldv + hh * HD;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      kf[ks] = *(const s16x8*)(kr + ks * 16 + 8 * h);
      vf[ks] = *(const s16x8*)(vr + ks * 16 + 8 * h);
    }
  }
  {  // K image of all 256 key rows (rows past Nk re-read the last: their dS is 0)
    TileStage<HD, BWD1_KEYS, BWD1_THREADS> kst;
    kst.load(kbase, p.ldk, 0, p.Nk, tid);
    kst.store(kimg, tid);
  }
  f32x16 dka[DS], dva[DS];
#pragma unroll
  for (int d = 0; d < DS; ++d)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      dka[d][r] = 0.f;
      dva[d][r] = 0.f;
    }

  // dQ: this wave's head-dim block and query blocks; per-lane transposed-read offsets (the
  // swizzle of rows 4g + q' (+16, +32 ks) depends on 4g + q' only)
  const int db = wave % NDB, qb0 = (wave / NDB) * QBW;
  const int g4 = lane >> 4, qq = (lane & 15) >> 2, pp = lane & 3;
  const int offk = toff<HD>(4 * g4 + qq, 2 * db + (pp >> 1)) + 8 * (pp & 1);
  int offs[QBW];
#pragma unroll
  for (int i = 0; i < QBW; ++i) offs[i] = toff<64>(4 * g4 + qq, 2 * (qb0 + i) + (pp >> 1)) + 8 * (pp & 1);
  const int srow = kl * (QT * 2) + 8 * h;  // this lane's dS image row (+ chunk ^ swizzle)
  const int sw4 = swz<64>(kl) << 4;
  auto tr4 = [](const char* a) {
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)a);
  };
  unsigned kmask = 0xffu;  // 32-key blocks with an unmasked key (set after the staging barrier)
  // dQ^T += K^T . dS^T over 32-key steps [k0, k1) of the dS image `sim`
  f32x4 dqa[QBW];
  auto dq_steps = [&](const char* sim, int k0, int k1) {
#pragma unroll
    for (int ks = k0; ks < k1; ++ks) {
      if (!((kmask >> ks) & 1u)) continue;
      const char* ka = kimg + ks * 32 * (HD * 2) + offk;
      const s16x4 a0 = tr4(ka), a1 = tr4(ka + 16 * (HD * 2));
      s16x8 av;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        av[j] = a0[j];
        av[4 + j] = a1[j];
      }
#pragma unroll
      for (int i = 0; i < QBW; ++i) {
        const char* sa = sim + ks * 32 * (QT * 2) + offs[i];
        const s16x4 b0 = tr4(sa), b1 = tr4(sa + 16 * (QT * 2));
        s16x8 bv;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          bv[j] = b0[j];
          bv[4 + j] = b1[j];
        }
        dqa[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bv, dqa[i], 0, 0, 0);
      }
    }
  };
  auto dq_store = [&](int q0) {
#pragma unroll
    for (int i = 0; i < QBW; ++i) {
      // lane: query 16 (qb0 + i) + (lane & 15), head dims 16 db + 4 (lane >> 4) .. +3
      const int q = q0 + 16 * (qb0 + i) + (lane & 15);
      if (q < p.Nq) {
        const int64_t col = (int64_t)hh * HD + 16 * db + 4 * g4;
        if (p.dq_f32) {
          const f32x4 w = {dqa[i][0] * p.scale, dqa[i][1] * p.scale, dqa[i][2] * p.scale, dqa[i][3] * p.scale};
          *(f32x4*)((float*)p.dq + ((int64_t)b * p.Nq + q) * p.lddq + col) = w;
        } else {
          u32x2 w;
          w[0] = pack2(dqa[i][0] * p.scale, dqa[i][1] * p.scale);
          w[1] = pack2(dqa[i][2] * p.scale, dqa[i][3] * p.scale);
          *(u32x2*)((bf16_t*)p.dq + ((int64_t)b * p.Nq + q) * p.lddq + col) = w;
        }
      }
    }
  };

  const bf16_t* qbase = p.q + (int64_t)b * p.Nq * p.ldq + hh * HD;
  const bf16_t* obase = p.dout + (int64_t)b * p.Nq * p.lddo + hh * HD;
  const float* lbase = p.lse + ((int64_t)b * p.H + hh) * p.Nq;
  const float* dbase = p.delta + ((int64_t)b * p.H + hh) * p.Nq;
  // this workgroup's query tiles [tq0, tq0 + ntiles) (all of them unless the queries are split over
  // gridDim.z = p.qsplit workgroups); t below is the tile index within the range
  const int ntot = (p.Nq + QT - 1) / QT;
  const int tq0 = (int)((int64_t)ntot * blockIdx.z / p.qsplit);
  const int ntiles = (int)((int64_t)ntot * (blockIdx.z + 1) / p.qsplit) - tq0;
  // tile t -> slot t % 3: wave w moves Q rows 8w..8w+7 and dO rows 8w..8w+7 (one 1-KiB piece each,
  // the chunk swizzle applied on the source address), wave 0 the lse words, wave 1 the delta words.
  // Rows past Nq re-read the last row; their lse is set to +inf after the DMA lands (P = dS = 0).
  const int drow = wave * 8 + (lane >> 3), dch = (lane & 7) ^ swz<HD>(drow);
  uint32_t qoff = (uint32_t)(drow * p.ldq + dch * 8) * 2, ooff = (uint32_t)(drow * p.lddo + dch * 8) * 2;
  auto dma = [&](int t) {
    char* base = smem + (t % NSLOT) * SLOT;
    const int q0 = (tq0 + t) * QT;
    if (q0 + QT > p.Nq) {  // the ragged last tile (its DMA is the last one issued)
      const int rr = min(drow, p.Nq - q0 - 1);
      qoff = (uint32_t)(rr * p.ldq + dch * 8) * 2;
      ooff = (uint32_t)(rr * p.lddo + dch * 8) * 2;
    }
    dma16s(qoff, qbase + (int64_t)q0 * p.ldq, lds_u32(base + wave * 1024));
    dma16s(ooff, obase + (int64_t)q0 * p.lddo, lds_u32(base + TILE + wave * 1024));
    if (wave < 2) dma4((wave == 0 ? lbase : dbase) + min(q0 + lane, p.Nq - 1), lds_u32(base + 2 * TILE + wave * STAT));
  };
  // this wave's DMA of tile t retired (the `later` pieces of tile t+1 may stay in flight) and the
  // LDS writes done; rows past Nq of tile t get lse = +inf; then the workgroup barrier
  auto tile_sync = [&](int t, bool later) {
    if (later) {
      if (wave < 2) __builtin_amdgcn_s_waitcnt(0x0073);  // vmcnt(3) lgkmcnt(0)
      else __builtin_amdgcn_s_waitcnt(0x0072);           // vmcnt(2) lgkmcnt(0)
    } else {
      __builtin_amdgcn_s_waitcnt(0x0070);
    }
    if (wave == 0 && (tq0 + t) * QT + QT > p.Nq && (tq0 + t) * QT + lane >= p.Nq)
      ((float*)(smem + (t % NSLOT) * SLOT + 2 * TILE))[lane] = INFINITY;
    __builtin_amdgcn_s_waitcnt(0x0070);
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
  dma(0);
  if (ntiles > 1) dma(1);
  tile_sync(0, ntiles > 1);
  kmask = kact;
  asm volatile("" : "+s"(kmask));  // opaque: the dQ k-step loop keeps its per-step test
  const bool mine = (kmask >> (kl >> 5)) & 1u;

  // Tile t's dQ product runs during tile t+1's S / dP / dK / dV (its dS image is the other
  // buffer): one barrier interval holds both, so the dQ MFMAs fill the softmax VALU gaps. Its
  // result is stored at the top of iteration t+2, before that iteration's DMA, so the counted
  // wait at the end of an iteration only has the next tile's pieces behind it.
  for (int t = 0; t < ntiles; ++t) {
    char* simg = simg0 + (t & 1) * SIMG;
    int soff = (t % NSLOT) * SLOT;
    asm volatile("" : "+s"(soff));  // opaque: no per-slot copies of the fragment addresses
    const char* qtile = smem + soff;
    const char* otile = qtile + TILE;
    const float* sl = (const float*)(qtile + 2 * TILE);
    const float* sd = sl + QT;
    const char* sprev = simg0 + ((t + 1) & 1) * SIMG;
    if (t >= 2) dq_store((tq0 + t - 2) * QT);
#pragma unroll
    for (int i = 0; i < QBW; ++i) dqa[i] = (f32x4){0.f, 0.f, 0.f, 0.f};
    if (t + 2 < ntiles) dma(t + 2);  // into tile t-1's slot (last read before the barrier)
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      if (!mine || (qs && u != (wave >> 2))) {  // padding keys / the other wave's half: dQ share only
        if (t > 0) dq_steps(sprev, u * (KSTEPS / 2), (u + 1) * (KSTEPS / 2));
        continue;
      }
      f32x16 s, dp;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        s[r] = 0.f;
        dp[r] = 0.f;
      }
      s16x8 qfr[KS], ofr[KS];
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        qfr[ks] = row_frag<HD>(qtile, u * 32, ks, lofs);
        ofr[ks] = row_frag<HD>(otile, u * 32, ks, lofs);
      }
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        s = mfma32(qfr[ks], kf[ks], s);
        dp = mfma32(ofr[ks], vf[ks], dp);
      }
      if (t > 0) dq_steps(sprev, u * (KSTEPS / 2), (u + 1) * (KSTEPS / 2));
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const f32x4 l4 = *(const f32x4*)&sl[u * 32 + 8 * g + 4 * h];
        const f32x4 dl4 = *(const f32x4*)&sd[u * 32 + 8 * g + 4 * h];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int r = 4 * g + i;
          const float pr = fast_exp2(fmaf(s[r], c2, BIAS ? kbias - l4[i] : -l4[i]));
          s[r] = pr;
          dp[r] = pr * (dp[r] - dl4[i]);
        }
      }
#pragma unroll
      for (int ss = 0; ss < 2; ++ss) {
        const s16x8 pb = acc_frag(s, ss);
        const s16x8 sb = acc_frag(dp, ss);
#pragma unroll
        for (int d = 0; d < DS; ++d) {
          dva[d] = mfma32(tr_frag<HD>(otile, u * 32, ss, d, lofs), pb, dva[d]);
          dka[d] = mfma32(tr_frag<HD>(qtile, u * 32, ss, d, lofs), sb, dka[d]);
        }
        // dS rows of this lane's key: registers 8ss + 4gg + i are queries 32u + 16ss + 8gg + 4h + i
#pragma unroll
        for (int gg = 0; gg < 2; ++gg) {
          u32x2 w;
          w[0] = (unsigned)(unsigned short)sb[4 * gg] | ((unsigned)(unsigned short)sb[4 * gg + 1] << 16);
          w[1] = (unsigned)(unsigned short)sb[4 * gg + 2] | ((unsigned)(unsigned short)sb[4 * gg + 3] << 16);
          int cx;
          asm volatile("v_xor_b32 %0, %1, %2" : "=v"(cx) : "i"((4 * u + 2 * ss + gg) << 4), "v"(sw4));
          *(u32x2*)(simg + srow + cx) = w;
        }
      }
    }
    // dS image t complete, tile t+1 resident, tile t's slot no longer read
    if (t + 1 < ntiles) tile_sync(t + 1, t + 2 < ntiles);
    else __syncthreads();
  }
  if (ntiles >= 2) dq_store((tq0 + ntiles - 2) * QT);
#pragma unroll
  for (int i = 0; i < QBW; ++i) dqa[i] = (f32x4){0.f, 0.f, 0.f, 0.f};
  dq_steps(simg0 + ((ntiles - 1) & 1) * SIMG, 0, KSTEPS);
  dq_store((tq0 + ntiles - 1) * QT);
  if (p.qsplit > 1) {  // f32 partial rows (dK unscaled): lane h holds dims 32d + 8g + 4h .. +3
    if (kl < p.Nk) {
      const int64_t plane = (int64_t)p.qsplit * p.B * p.Nk * p.H * HD;
      float* pk = p.part + (((int64_t)blockIdx.z * p.B + b) * p.Nk + kl) * (p.H * HD) + hh * HD + 4 * h;
#pragma unroll
      for (int d = 0; d < DS; ++d)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          *(f32x4*)(pk + d * 32 + 8 * g) = (f32x4){dka[d][4 * g], dka[d][4 * g + 1], dka[d][4 * g + 2], dka[d][4 * g + 3]};
          *(f32x4*)(pk + plane + d * 32 + 8 * g) =
              (f32x4){dva[d][4 * g], dva[d][4 * g + 1], dva[d][4 * g + 2], dva[d][4 * g + 3]};
        }
    }
    return;
  }
  if (qs) {  // waves 4-7's dK / dV partials into waves 0-3 (the dS images are free now)
    static_assert(4 * 2 * DS * 16 * 64 * 4 <= 2 * SIMG, "partials fit the dS images");
    float* xs = (float*)simg0 + (wave & 3) * (2 * DS * 16 * 64) + lane;
    __syncthreads();
    if (wave >= 4) {
#pragma unroll
      for (int d = 0; d < DS; ++d)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          xs[((2 * d) * 16 + r) * 64] = dka[d][r];
          xs[((2 * d + 1) * 16 + r) * 64] = dva[d][r];
        }
    }
    __syncthreads();
    if (wave >= 4) {  // keys 128 + 32 (w - 4) ..: all padding under qs, so dK = dV = 0 exactly
      const int kz = 128 + kl;
#pragma unroll
      for (int d = 0; d < DS; ++d)
#pragma unroll
        for (int r = 0; r < 16; ++r) dka[d][r] = 0.f;
      store_row_swap<HD>(dka, 1.0f, kz < p.Nk ? p.dk + ((int64_t)b * p.Nk + kz) * p.lddk + hh * HD : nullptr, lane);
      store_row_swap<HD>(dka, 1.0f, kz < p.Nk ? p.dv + ((int64_t)b * p.Nk + kz) * p.lddv + hh * HD : nullptr, lane);
      return;
    }
#pragma unroll
    for (int d = 0; d < DS; ++d)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        dka[d][r] += xs[((2 * d) * 16 + r) * 64];
        dva[d][r] += xs[((2 * d + 1) * 16 + r) * 64];
      }
  }
  // dK, dV rows in 16-B pieces (store_row_swap: both lane halves take part)
  const bool kin = kl < p.Nk;
  store_row_swap<HD>(dka, p.scale, kin ? p.dk + ((int64_t)b * p.Nk + kl) * p.lddk + hh * HD : nullptr, lane);
  store_row_swap<HD>(dva, 1.0f, kin ? p.dv + ((int64_t)b * p.Nk + kl) * p.lddv + hh * HD : nullptr, lane);
}

// sum of the query-split one-pass backward's dK / dV partials in split order (deterministic):
// dK = bf16(scale * sum), dV = bf16(sum); 8 columns per thread
template <int HD>
__global__ __launch_bounds__(256) void attn_bwd1_finish_kernel(const AttnParams p) {
  const int cols = p.H * HD;
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t rows = (int64_t)p.B * p.Nk;
  if (idx >= rows * (cols / 8)) return;
  const int64_t row = idx / (cols / 8);
  const int c = (int)(idx % (cols / 8)) * 8;
  const int64_t plane = (int64_t)p.qsplit * rows * cols;
  float k8[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, v8[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int z = 0; z < p.qsplit; ++z) {
    const float* src = p.part + ((int64_t)z * rows + row) * cols + c;
    const f32x4 a0 = *(const f32x4*)src, a1 = *(const f32x4*)(src + 4);
    const f32x4 b0 = *(const f32x4*)(src + plane), b1 = *(const f32x4*)(src + plane + 4);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      k8[i] += a0[i];
      k8[4 + i] += a1[i];
      v8[i] += b0[i];
      v8[4 + i] += b1[i];
    }
  }
  u32x4 wk, wv;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    wk[j] = pack2(k8[2 * j] * p.scale, k8[2 * j + 1] * p.scale);
    wv[j] = pack2(v8[2 * j], v8[2 * j + 1]);
  }
  *(u32x4*)(p.dk + row * p.lddk + c) = wk;
  *(u32x4*)(p.dv + row * p.lddv + c) = wv;
}

// delta[b,h,q] = sum_d dO*O (f32), one wave per (b, q) row covering all heads
template <int HD>
__global__ __launch_bounds__(256) void attn_delta_kernel(const AttnParams p, float* __restrict__ delta) {
  const int lane = threadIdx.x & 63;
  const int64_t row = blockIdx.x * 4 + (threadIdx.x >> 6);  // b*Nq + q
  if (row >= (int64_t)p.B * p.Nq) return;
  const int b = (int)(row / p.Nq), q = (int)(row % p.Nq);
  constexpr int LPH = HD / 8;  // lanes per head (8 elements each)
  const int HPP = 64 / LPH;    // heads per pass
  for (int h0 = 0; h0 < p.H; h0 += HPP) {
    const int hh = h0 + lane / LPH;
    float s = 0.f;
    if (hh < p.H) {
      const int d0 = (lane % LPH) * 8;
      const u32x4 a = *(const u32x4*)(p.dout + row * p.lddo + hh * HD + d0);
      const u32x4 o = *(const u32x4*)(p.o + row * p.ldo + hh * HD + d0);
#pragma unroll
      for (int j = 0; j < 8; ++j)
        s += bf2f((bf16_t)(a[j >> 1] >> ((j & 1) * 16))) * bf2f((bf16_t)(o[j >> 1] >> ((j & 1) * 16)));
    }
#pragma unroll
    for (int off = LPH / 2; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
    if (hh < p.H && (lane % LPH) == 0) delta[((int64_t)b * p.H + hh) * p.Nq + q] = s;
  }
}

static inline bool needs_bias(const AttnParams& p) { return p.key_bias != nullptr || (p.Nk % 64) != 0; }

#ifndef LTX_ATTN_W8_DEFAULT
#define LTX_ATTN_W8_DEFAULT 1
#endif

static AttnSwitches read_attn_switches() {
  AttnSwitches w;
  auto num = [](const char* name, int dflt) {
    const char* e = std::getenv(name);
    return (e && e[0]) ? std::atoi(e) : dflt;
  };
  auto off0 = [](const char* name) {  // "0..." switches a default-on path off
    const char* e = std::getenv(name);
    return (e && e[0] == '0') ? 0 : 1;
  };
  w.xcd = off0("LTX_ATTN_XCD");
  w.bwd1 = off0("LTX_ATTN_BWD1");
  // bit 0 = 8-wave (256-query) tiled forward, bit 1 = 8-wave (256-key) dK/dV kernel; the default
  // is the forward only (self-attention forward 297-305 vs 310-316 us, dK/dV 881-889 vs 857-862 us
  // with 8 waves, tools/attn_bench.py)
  w.w8 = num("LTX_ATTN_W8", LTX_ATTN_W8_DEFAULT);
  w.skip = off0("LTX_ATTN_SKIP");
  w.fwd1 = off0("LTX_ATTN_FWD1");
  w.fwd1_rows = off0("LTX_ATTN_FWD1_ROWS");
  {  // off by default: its step A/B was neutral, and with it dK / dV of the unmasked keys are the sum
     // of two partials (f32 rounding away from the 8 x 32-key kernel; dQ stays bitwise)
    const char* e = std::getenv("LTX_ATTN_BWD1_QS");
    w.bwd1_qs = (e && e[0] == '1') ? 1 : 0;
  }
  w.bwd1_few = off0("LTX_ATTN_BWD1_FEW");
  w.qsplit = off0("LTX_ATTN_QSPLIT");
  w.dkdv_w1 = num("LTX_ATTN_DKDV_W1", 2);
  w.dq_w1 = num("LTX_ATTN_DQ_W1", 2);
  w.dq_pipe = num("LTX_ATTN_DQ_PIPE", 1) != 0;
  {
    const char* e = std::getenv("LTX_ATTN_DQ_NBUF");
    w.dq_nbuf = (e && e[0] == '3') ? 3 : 4;
  }
  {
    const char* e = std::getenv("LTX_ATTN_FWD_W1");
    w.fwd_w1 = (e && e[0] && e[0] != '0') ? std::atoi(e) : 0;
  }
  w.fwd_pipe = num("LTX_ATTN_FWD_PIPE", 1) != 0;
  w.fwd_f32sum = off0("LTX_ATTN_FWD_F32SUM");
  w.dkdv_pipe = num("LTX_ATTN_DKDV_PIPE", 1) != 0;
  {
    const char* e = std::getenv("LTX_ATTN_DKDV_NBUF");
    w.dkdv_nbuf = (e && e[0] == '3') ? 3 : 4;
  }
  return w;
}

static AttnSwitches& switch_table() {
  static AttnSwitches w = read_attn_switches();
  return w;
}

const AttnSwitches& attn_switches() { return switch_table(); }

static int xcd_order_flag() { return attn_switches().xcd; }
static int bwd1_flag() { return attn_switches().bwd1; }
static int waves8_flag(int bit) { return (attn_switches().w8 >> bit) & 1; }
static int skip_flag() { return attn_switches().skip; }
static int fwd1_flag() { return attn_switches().fwd1; }
static int bwd1_qs_flag() { return attn_switches().bwd1_qs; }
static int bwd1_few_flag() { return attn_switches().bwd1_few; }
static int qsplit_flag() { return attn_switches().qsplit; }

template <int HD>
static int launch_fwd(AttnParams p, hipStream_t s) {
  p.xcd_order = xcd_order_flag();
  p.skip_masked = skip_flag();
  if constexpr (HD == 64) {
    if (p.Nk <= BWD1_KEYS && fwd1_flag()) {  // every key staged once per (batch, head)
      // two workgroups per (batch, head) when that still leaves >= 8 slices each: 2 per CU
      // (more when H * B leaves the chip short of 256 workgroups: inference, config X at B = 1)
      const int nsl = (p.Nq + 31) / 32;
      int z = nsl >= 16 ? 2 : 1;
      if (z == 2 && p.H * p.B < 128) z = std::max(2, std::min(nsl / 8, (256 + p.H * p.B - 1) / (p.H * p.B)));
      const dim3 g1((unsigned)p.H, (unsigned)p.B, (unsigned)z);
      const bool rows = attn_switches().fwd1_rows != 0;
      if (needs_bias(p)) {
        if (rows) hipLaunchKernelGGL((attn_fwd1_kernel<HD, true, true>), g1, dim3(BWD1_THREADS), 0, s, p);
        else hipLaunchKernelGGL((attn_fwd1_kernel<HD, true, false>), g1, dim3(BWD1_THREADS), 0, s, p);
      } else {
        if (rows) hipLaunchKernelGGL((attn_fwd1_kernel<HD, false, true>), g1, dim3(BWD1_THREADS), 0, s, p);
        else hipLaunchKernelGGL((attn_fwd1_kernel<HD, false, false>), g1, dim3(BWD1_THREADS), 0, s, p);
      }
      LTX_LAUNCH_CHECK();
      return LTX_OK;
    }
  }
  if constexpr (HD == 64) {
    if (!needs_bias(p) && fwd_pipe_enabled()) return launch_fwd_pipe(p, s);
    if (waves8_flag(0)) {
      dim3 grid((unsigned)((p.Nq + 255) / 256), (unsigned)p.H, (unsigned)p.B);
      if (needs_bias(p))
        hipLaunchKernelGGL((attn_q_kernel<HD, 0, true, 8>), grid, dim3(512), 0, s, p);
      else
        hipLaunchKernelGGL((attn_q_kernel<HD, 0, false, 8>), grid, dim3(512), 0, s, p);
      LTX_LAUNCH_CHECK();
      return LTX_OK;
    }
  }
  dim3 grid((unsigned)((p.Nq + 127) / 128), (unsigned)p.H, (unsigned)p.B);
  if (needs_bias(p))
    hipLaunchKernelGGL((attn_q_kernel<HD, 0, true>), grid, dim3(ATT_THREADS), 0, s, p);
  else
    hipLaunchKernelGGL((attn_q_kernel<HD, 0, false>), grid, dim3(ATT_THREADS), 0, s, p);
  LTX_LAUNCH_CHECK();
  return LTX_OK;
}

template <int HD>
static int launch_bwd(AttnParams p, float* delta, int delta_ready, hipStream_t s) {
  if (!delta_ready) {
    hipLaunchKernelGGL(attn_delta_kernel<HD>, dim3((unsigned)(((int64_t)p.B * p.Nq + 3) / 4)), dim3(256), 0, s,
                       p, delta);
    LTX_LAUNCH_CHECK();
  }
  p.delta = delta;
  p.xcd_order = xcd_order_flag();
  p.skip_masked = skip_flag();
  p.few_keys = p.skip_masked && bwd1_few_flag();
  if constexpr (HD == 64) {  // (head dim 32, the tiny config, keeps the split kernels)
    if (p.Nk <= BWD1_KEYS && bwd1_flag()) {  // every key in one workgroup: one-pass backward
      // under 128 (batch, head) pairs the queries are split over S workgroups each (f32 dK / dV
      // partials in the stream's workspace, summed in order by attn_bwd1_finish_kernel)
      p.qsplit = 1;
      const int ntot = (p.Nq + 63) / 64;
      if (p.H * p.B < 128 && ntot >= 4 && qsplit_flag()) {
        // S depends on the shape alone, so the dK / dV summation order does too; when its partials
        // do not fit the stream's workspace the unsplit kernel runs instead (never a smaller S)
        const int S = std::min(ntot / 2, (256 + p.H * p.B - 1) / (p.H * p.B));
        size_t ws = 0;
        float* part = stream_workspace(s, &ws);
        if (S > 1 && part != nullptr && (size_t)2 * S * p.B * p.Nk * p.H * HD * sizeof(float) <= ws) {
          p.qsplit = S;
          p.part = part;
          const dim3 gs((unsigned)p.H, (unsigned)p.B, (unsigned)S);
          if (p.key_bias != nullptr || p.Nk != BWD1_KEYS)
            hipLaunchKernelGGL((attn_bwd1_kernel<HD, true, false>), gs, dim3(BWD1_THREADS), 0, s, p);
          else
            hipLaunchKernelGGL((attn_bwd1_kernel<HD, false, false>), gs, dim3(BWD1_THREADS), 0, s, p);
          LTX_LAUNCH_CHECK();
          const int64_t n8 = (int64_t)p.B * p.Nk * p.H * HD / 8;
          hipLaunchKernelGGL((attn_bwd1_finish_kernel<HD>), dim3((unsigned)((n8 + 255) / 256)), dim3(256), 0, s, p);
          LTX_LAUNCH_CHECK();
          return LTX_OK;
        }
      }
      const dim3 g1((unsigned)p.H, (unsigned)p.B);
      if ((p.key_bias != nullptr || p.Nk != BWD1_KEYS) && bwd1_qs_flag())
        hipLaunchKernelGGL((attn_bwd1_kernel<HD, true, true>), g1, dim3(BWD1_THREADS), 0, s, p);
      else if (p.key_bias != nullptr || p.Nk != BWD1_KEYS)
        hipLaunchKernelGGL((attn_bwd1_kernel<HD, true, false>), g1, dim3(BWD1_THREADS), 0, s, p);
      else
        hipLaunchKernelGGL((attn_bwd1_kernel<HD, false, false>), g1, dim3(BWD1_THREADS), 0, s, p);
      LTX_LAUNCH_CHECK();
      return LTX_OK;
    }
  }
  dim3 gq((unsigned)((p.Nq + 127) / 128), (unsigned)p.H, (unsigned)p.B);
  bool k8 = false;
  if constexpr (HD == 64) k8 = waves8_flag(1);
  dim3 gk((unsigned)(k8 ? (p.Nk + 255) / 256 : (p.Nk + 127) / 128), (unsigned)p.H, (unsigned)p.B);
  if (HD == 64 && !k8 && dkdv_pipe_enabled()) {
    if (needs_bias(p)) {
      hipLaunchKernelGGL((attn_q_kernel<HD, 1, true>), gq, dim3(ATT_THREADS), 0, s, p);
      LTX_LAUNCH_CHECK();
    } else if (dq_w1p_enabled() && dq_w1p_applies(p)) {
      const int rc = launch_dq_w1p(p, s);
      if (rc != LTX_OK) return rc;
    } else if (dq_w1_enabled()) {
      const int rc = launch_dq_w1(p, s);
      if (rc != LTX_OK) return rc;
    } else if (dq_pipe_enabled()) {
      const int rc = launch_dq_pipe(p, s);
      if (rc != LTX_OK) return rc;
    } else {
      hipLaunchKernelGGL((attn_q_kernel<HD, 1, false>), gq, dim3(ATT_THREADS), 0, s, p);
      LTX_LAUNCH_CHECK();
    }
    if (!needs_bias(p) && dkdv_w1p_enabled() && dkdv_w1p_applies(p)) return launch_dkdv_w1p(p, s);
    if (!needs_bias(p) && dkdv_w1_enabled()) return launch_dkdv_w1(p, s);
    return launch_dkdv_pipe(p, s);
  }
  if (needs_bias(p)) {
    hipLaunchKernelGGL((attn_q_kernel<HD, 1, true>), gq, dim3(ATT_THREADS), 0, s, p);
    LTX_LAUNCH_CHECK();
    if (k8)
      hipLaunchKernelGGL((attn_dkdv_kernel<HD, true, HD == 64 ? 8 : 4>), gk, dim3(512), 0, s, p);
    else
      hipLaunchKernelGGL((attn_dkdv_kernel<HD, true>), gk, dim3(ATT_THREADS), 0, s, p);
  } else {
    hipLaunchKernelGGL((attn_q_kernel<HD, 1, false>), gq, dim3(ATT_THREADS), 0, s, p);
    LTX_LAUNCH_CHECK();
    if (k8)
      hipLaunchKernelGGL((attn_dkdv_kernel<HD, false, HD == 64 ? 8 : 4>), gk, dim3(512), 0, s, p);
    else
      hipLaunchKernelGGL((attn_dkdv_kernel<HD, false>), gk, dim3(ATT_THREADS), 0, s, p);
  }
  LTX_LAUNCH_CHECK();
  return LTX_OK;
}

static int check_common(const void* q, int64_t ldq, const void* k, int64_t ldk, const void* v, int64_t ldv,
                        int64_t B, int64_t H, int64_t Nq, int64_t Nk, int64_t d) {
  if (!(q && k && v)) return fail(LTX_ERR_BAD_ARG, "attn: null q/k/v");
  if (!(d == 32 || d == 64)) return fail(LTX_ERR_BAD_ARG, "attn: head dim must be 32 or 64");
  if (B <= 0 || H <= 0 || Nq <= 0 || Nk <= 0) return fail(LTX_ERR_BAD_ARG, "attn: empty shape");
  if (ldq < H * d || ldk < H * d || ldv < H * d) return fail(LTX_ERR_BAD_ARG, "attn: row stride < H*d");
  if ((ldq | ldk | ldv) % 8 != 0) return fail(LTX_ERR_BAD_ARG, "attn: row strides must be multiples of 8");
  if (((uintptr_t)q | (uintptr_t)k | (uintptr_t)v) % 16 != 0) return fail(LTX_ERR_BAD_ARG, "attn: 16-B alignment");
  return LTX_OK;
}

}  // namespace ltx

using namespace ltx;

extern "C" int ltx_attn_fwd(const void* q, int64_t ldq, const void* k, int64_t ldk, const void* v, int64_t ldv,
                            void* o, int64_t ldo, float* lse, const float* key_bias, int64_t B, int64_t H,
                            int64_t Nq, int64_t Nk, int64_t kv_batch_rows, int64_t d, float scale, void* stream) {
  int rc = check_common(q, ldq, k, ldk, v, ldv, B, H, Nq, Nk, d);
  if (rc) return rc;
  LTX_CHECK_ARG(kv_batch_rows == Nk || kv_batch_rows == 0, "attn_fwd: kv_batch_rows must be Nk or 0 (shared)");
  LTX_CHECK_ARG(o && lse && ldo >= H * d && ldo % 8 == 0, "attn_fwd: bad output");
  AttnParams p = {};
  p.q = (const bf16_t*)q; p.ldq = ldq; p.k = (const bf16_t*)k; p.ldk = ldk; p.v = (const bf16_t*)v; p.ldv = ldv;
  p.o_out = (bf16_t*)o; p.ldo = ldo; p.lse = lse; p.key_bias = key_bias;
  p.B = (int)B; p.H = (int)H; p.Nq = (int)Nq; p.Nk = (int)Nk; p.kvb = (int)kv_batch_rows; p.scale = scale;
  p.qsplit = 1;
  return d == 64 ? launch_fwd<64>(p, (hipStream_t)stream) : launch_fwd<32>(p, (hipStream_t)stream);
}

extern "C" int ltx_attn_bwd_ex(const void* q, int64_t ldq, const void* k, int64_t ldk, const void* v, int64_t ldv,
                               const void* o, int64_t ldo, const void* dout, int64_t lddo, const float* lse,
                               const float* key_bias, float* delta_ws, int delta_ready, void* dq, int64_t lddq,
                               int dq_is_f32, void* dk, int64_t lddk, void* dv, int64_t lddv, int64_t B, int64_t H,
                               int64_t Nq, int64_t Nk, int64_t kv_batch_rows, int64_t d, float scale,
                               void* stream) {
  int rc = check_common(q, ldq, k, ldk, v, ldv, B, H, Nq, Nk, d);
  if (rc) return rc;
  LTX_CHECK_ARG(kv_batch_rows == Nk || kv_batch_rows == 0, "attn_bwd: kv_batch_rows must be Nk or 0 (shared)");
  LTX_CHECK_ARG(dout && lse && delta_ws && dq && dk && dv && (o || delta_ready), "attn_bwd: null operand");
  LTX_CHECK_ARG((ldo | lddo | lddq | lddk | lddv) % 8 == 0, "attn_bwd: strides must be multiples of 8");
  AttnParams p = {};
  p.q = (const bf16_t*)q; p.ldq = ldq; p.k = (const bf16_t*)k; p.ldk = ldk; p.v = (const bf16_t*)v; p.ldv = ldv;
  p.o = (const bf16_t*)o; p.ldo = ldo; p.dout = (const bf16_t*)dout; p.lddo = lddo;
  p.lse = (float*)lse; p.key_bias = key_bias;
  p.dq = dq; p.lddq = lddq; p.dq_f32 = dq_is_f32;
  p.dk = (bf16_t*)dk; p.lddk = lddk; p.dv = (bf16_t*)dv; p.lddv = lddv;
  p.B = (int)B; p.H = (int)H; p.Nq = (int)Nq; p.Nk = (int)Nk; p.kvb = (int)kv_batch_rows; p.scale = scale;
  p.qsplit = 1;
  return d == 64 ? launch_bwd<64>(p, delta_ws, delta_ready, (hipStream_t)stream)
                 : launch_bwd<32>(p, delta_ws, delta_ready, (hipStream_t)stream);
}

extern "C" int ltx_attn_bwd(const void* q, int64_t ldq, const void* k, int64_t ldk, const void* v, int64_t ldv,
                            const void* o, int64_t ldo, const void* dout, int64_t lddo, const float* lse,
                            const float* key_bias, float* delta_ws, void* dq, int64_t lddq, int dq_is_f32,
                            void* dk, int64_t lddk, void* dv, int64_t lddv, int64_t B, int64_t H, int64_t Nq,
                            int64_t Nk, int64_t kv_batch_rows, int64_t d, float scale, void* stream) {
  return ltx_attn_bwd_ex(q, ldq, k, ldk, v, ldv, o, ldo, dout, lddo, lse, key_bias, delta_ws, 0, dq, lddq, dq_is_f32,
                         dk, lddk, dv, lddv, B, H, Nq, Nk, kv_batch_rows, d, scale, stream);
}

extern "C" int ltx_attn_reload_switches(void) {
  ltx::switch_table() = ltx::read_attn_switches();
  return LTX_OK;
}
