// Shared pieces of the attention kernels (attention.hip, attention_dkdv.hip): LDS tile layout and
// fragment reads for v_mfma_f32_32x32x16_bf16 in the swapped orientation, the parameter block,
// row-statistic helpers and the XCD-aware block order. See attention.hip for the design notes.
#pragma once
#include "common.h"

namespace ltx {

constexpr float LOG2E = 1.4426950408889634f;
constexpr int ATT_THREADS = 256;

// Chunk swizzle of row `row`. HD = 64 (128-B rows, 8 chunks): x = (row >> 1) & 7 bit-reversed.
//  * 16-B row reads (ds_read_b128, lane groups of 16 over rows {0-3,12-15,20-27} / {4-11,16-19,
//    28-31}): the 8 rows of one parity in a group have distinct x, so distinct chunks.
//  * transposed reads (ds_read_b64_tr_b16, 32-lane halves over rows R..R+3, R = 0 mod 4, one
//    aligned group of 4 chunks): rows R and R+2 (same bank half) differ in x's bit 0, which the
//    reversal moves to bit 2, so their chunk groups are disjoint. With the plain (row >> 1) & 7
//    they coincide: a 2-way conflict on every transposed read (SQ_LDS_BANK_CONFLICT, r02_pmc_sq).
// HD = 32 (64-B rows): four consecutive rows already cover the 64 banks.
template <int HD>
__device__ __forceinline__ int swz(int row) {
  if constexpr (HD == 64) {
    const int x = (row >> 1) & 7;
    return ((x & 1) << 2) | (x & 2) | (x >> 2);
  } else {
    return (row >> 1) & (HD / 8 - 1);
  }
}

template <int HD>
__device__ __forceinline__ int toff(int row, int chunk) {
  return row * (HD * 2) + ((chunk ^ swz<HD>(row)) << 4);
}

// Per-lane LDS byte offsets of the fragment reads, computed once per kernel. Both kinds of
// read start at a row that is a multiple of 16 (rbase = 32u, + 16s), and swz depends on
// (row >> 1) mod 8 only, so a read is this lane offset + a wave-uniform constant.
template <int HD>
struct LaneOfs {
  static constexpr int KS = HD / 16, DS = HD / 32;
  int row[KS];    // 16-B row fragment: row (lane & 31), dims ks*16 + 8*(lane >> 5) .. +7
  int tr[DS][2];  // transposed fragment: rows 4h + q (+8), columns d*32 + (lane & 31)
  __device__ __forceinline__ explicit LaneOfs(int lane) {
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) row[ks] = toff<HD>(lane & 31, ks * 2 + (lane >> 5));
    const int h = lane >> 5, g = (lane >> 4) & 1, q = (lane & 15) >> 2, p = lane & 3;
#pragma unroll
    for (int d = 0; d < DS; ++d) {
      const int col = d * 32 + 16 * g + 4 * p;
      tr[d][0] = toff<HD>(4 * h + q, col >> 3) + ((col & 7) << 1);
      tr[d][1] = toff<HD>(4 * h + q + 8, col >> 3) + ((col & 7) << 1);
    }
  }
};

// 16-B row fragment: lane reads row (base + (l&31)), dims ks*16 + 8*(l>>5) .. +7
template <int HD>
__device__ __forceinline__ s16x8 row_frag(const char* tile, int base, int ks, const LaneOfs<HD>& lo) {
  return *(const s16x8*)(tile + base * (HD * 2) + lo.row[ks]);
}

// Transposed fragment for an A operand that sums over the tile's ROW axis, matching an
// accumulator-as-B operand (k-step s of a 32-row accumulator tile): element j of lane half h
// is row 16s + 8(j>>2) + 4h + (j&3) (+ rbase), column 32d + (lane & 31).
template <int HD>
__device__ __forceinline__ s16x8 tr_frag(const char* tile, int rbase, int s, int d, const LaneOfs<HD>& lo) {
  const char* t = tile + (rbase + 16 * s) * (HD * 2);
  const s16x4 lo4 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(t + lo.tr[d][0]));
  const s16x4 hi4 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(t + lo.tr[d][1]));
  s16x8 r;
  r[0] = lo4[0]; r[1] = lo4[1]; r[2] = lo4[2]; r[3] = lo4[3];
  r[4] = hi4[0]; r[5] = hi4[1]; r[6] = hi4[2]; r[7] = hi4[3];
  return r;
}

// accumulator registers 8s..8s+7 -> bf16 B-operand fragment for k-step s
__device__ __forceinline__ s16x8 acc_frag(const f32x16& a, int s) {
  s16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = (short)f2bf(a[8 * s + j]);
  return r;
}

__device__ __forceinline__ f32x16 mfma32(const s16x8& a, const s16x8& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// row (in the register axis) of accumulator register r for lane half h
__device__ __forceinline__ int acc_row(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

// global 16-B loads of a [ROWS][HD] tile, staged in registers, written swizzled. A thread moves
// chunk c = tid % CH of rows tid / CH + i * RSTEP: its byte offsets inside a tile are constant,
// so a tile is one scalar base (row0 * ld) + a 24-bit-multiply lane offset per load (no per-tile
// 64-bit address math, no lane predicates); rows past a ragged end re-read the last row.
template <int HD, int ROWS, int NTH = ATT_THREADS>
struct TileStage {
  static constexpr int CH = HD / 8;
  static constexpr int PER = ROWS * CH / NTH;
  static constexpr int RSTEP = NTH / CH;
  static_assert(ROWS * CH % NTH == 0, "a tile must split evenly over the workgroup");
  u32x4 v[PER];
  __device__ __forceinline__ void load(const bf16_t* base, int64_t ld, int row0, int nrows, int tid) {
    const int r = tid / CH, c = tid % CH;
    const char* tb = (const char*)(base + (int64_t)row0 * ld);  // wave-uniform
    const int lim = nrows - 1 - row0;                             // rows past the end re-read the last
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const uint32_t off = __umul24((uint32_t)min(r + i * RSTEP, lim), (uint32_t)(ld * 2)) + (uint32_t)(c * 16);
      v[i] = *(const u32x4*)(tb + off);
    }
  }
  __device__ __forceinline__ void store(char* tile, int tid) const {
    const int r = tid / CH, c = tid % CH;
#pragma unroll
    for (int i = 0; i < PER; ++i) *(u32x4*)(tile + toff<HD>(r + i * RSTEP, c)) = v[i];
  }
};

// LDS-DMA pieces in inline asm: hipcc tracks its own global_load_lds builtin as an LDS write
// and waits vmcnt(0) before the next ds_read, which would drain the tile prefetch every
// iteration; hidden from it, the DMA is retired only by the kernel's tile barrier's explicit wait + barrier.
// M0 (the wave-uniform LDS destination) is written in the same statement (compiler-reserved).
__device__ __forceinline__ uint32_t lds_u32(const void* p) {
  return __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)p);
}
__device__ __forceinline__ void dma16(const void* gsrc, uint32_t lds) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(gsrc), "s"(lds) : "memory");
}
// scalar-base form: per-lane 32-bit byte offset + wave-uniform 64-bit base (no per-lane 64-bit math)
__device__ __forceinline__ void dma16s(uint32_t voff, const void* sbase, uint32_t lds) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(voff), "s"(sbase), "s"(lds) : "memory");
}
__device__ __forceinline__ void dma4(const void* gsrc, uint32_t lds) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(gsrc), "s"(lds) : "memory");
}

// The attention path's A/B switches (LTX_ATTN_*), read from the environment ONCE (first launch)
// into this table; ltx_attn_reload_switches() re-reads them (tests that compare two paths in one
// process; ops.py calls it when it sees an LTX_ATTN_* variable change). Defaults are the shipping
// configuration. Defined in attention.hip.
struct AttnSwitches {
  int xcd = 1;          // LTX_ATTN_XCD=0: hardware block order
  int bwd1 = 1;         // LTX_ATTN_BWD1=0: split dQ + dK/dV kernels for every key range
  int w8 = 1;           // LTX_ATTN_W8: bit 0 8-wave tiled forward, bit 1 8-wave dK/dV
  int skip = 1;         // LTX_ATTN_SKIP=0: one-pass kernels keep all-padding key blocks
  int fwd1 = 1;         // LTX_ATTN_FWD1=0: tiled forward for every key range
  int fwd1_rows = 1;    // LTX_ATTN_FWD1_ROWS=0: the one-pass forward stores O in 32-B pieces
  int bwd1_qs = 0;      // LTX_ATTN_BWD1_QS=1: query-split one-pass backward for biased ranges
  int bwd1_few = 1;     // LTX_ATTN_BWD1_FEW=0: keep the 8 x 32-key schedule for few unmasked keys
  int qsplit = 1;       // LTX_ATTN_QSPLIT=0: one workgroup per (batch, head) at any H * B
  int dkdv_w1 = 2;      // LTX_ATTN_DKDV_W1: 2 persistent, 1 per block, 0 pipe, 12..16 / 22 diagnostic
  int dq_w1 = 2;        // LTX_ATTN_DQ_W1: likewise for dQ
  int dq_pipe = 1;      // LTX_ATTN_DQ_PIPE=0: the plain dQ kernel
  int dq_nbuf = 4;      // LTX_ATTN_DQ_NBUF=3: 3-buffer ring
  int fwd_w1 = 0;       // LTX_ATTN_FWD_W1 (only in `make fwdw1` builds)
  int fwd_pipe = 1;     // LTX_ATTN_FWD_PIPE=0: attn_q_kernel<64, 0, false, 8>
  int fwd_f32sum = 1;   // LTX_ATTN_FWD_F32SUM=0: row sums by v_dot2c over the bf16 weights
  int dkdv_pipe = 1;    // LTX_ATTN_DKDV_PIPE=0: the plain dK/dV kernel
  int dkdv_nbuf = 4;    // LTX_ATTN_DKDV_NBUF=3: 3-buffer ring
};
const AttnSwitches& attn_switches();

struct AttnParams {
  const bf16_t* q; int64_t ldq;
  const bf16_t* k; int64_t ldk;
  const bf16_t* v; int64_t ldv;
  const bf16_t* o; int64_t ldo;      // forward output (bwd: the saved output, for delta)
  bf16_t* o_out;
  const bf16_t* dout; int64_t lddo;
  float* lse;                          // [B,H,Nq] log2 units
  const float* delta;                  // [B,H,Nq]
  const float* key_bias;               // [B,Nk] natural units, or null
  void* dq; int64_t lddq; int dq_f32;  // dQ output
  bf16_t* dk; int64_t lddk;
  bf16_t* dv; int64_t lddv;
  int B, H, Nq, Nk;
  int kvb;                             // rows between batches of K, V and key_bias (Nk, or 0: shared)
  float scale;
  int xcd_order;                       // 1: XCD-aware block order (xcd_block), 0: hardware order
  int skip_masked;                     // 1: skip all-padding key blocks (one-pass kernels), 0: keep
  // one-pass cross backward split over the queries (attn_bwd1_kernel, qsplit > 1): gridDim.z
  // workgroups per (batch, head) each take a contiguous range of query tiles and write f32 dK / dV
  // partials [2][qsplit][B][Nk][H*HD] to `part`, summed in order by attn_bwd1_finish_kernel
  int qsplit;
  float* part;
  // one-pass cross backward: a (batch, head) whose unmasked keys all lie in one 32-key block takes
  // the per-wave sub-tile schedule (attention.hip bwd1_few_keys)
  int few_keys;
};

// per-key additive term in log2 units for keys key0..key0+63 -> LDS
__device__ __forceinline__ void key_bias_tile(float* kb, const AttnParams& p, int b, int key0, int n, int tid) {
  if (tid < n) {
    const int key = key0 + tid;
    float v = -INFINITY;
    if (key < p.Nk) v = p.key_bias ? p.key_bias[(int64_t)b * p.kvb + key] * LOG2E : 0.f;
    kb[tid] = v;
  }
}

// =============================================================================================
// forward (MODE 0) and dQ (MODE 1): queries on lanes, keys in registers.
// BIAS: keys carry an additive term (encoder mask bias, or -inf past a ragged Nk); without it
// (self-attention, Nk % 64 == 0) the per-key LDS reads and adds disappear.
// VALU diet (the forward is VALU-bound at head dim 64): the running max is taken on the raw
// scores (scale > 0), each probability is one v_fma + one v_exp_f32, and the O rescale is skipped
// unless some lane's max grew by more than RESCALE_TAU (deferred max, above).
// =============================================================================================
__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

// Deferred max (forward kernels): the running max m_run (log2 units) and with it O and l are
// rescaled only when some lane's tile max exceeds it by more than RESCALE_TAU; below that the
// probabilities 2^(s - m_run) stay <= 2^TAU (exact in f32, bf16 keeps its relative precision for
// the P.V MFMA) and lse = m_run + log2(l) is unchanged in meaning. Most 64-key tiles then skip the
// O rescale pass.
#ifndef LTX_RESCALE_TAU
#define LTX_RESCALE_TAU 8.0f
#endif
constexpr float RESCALE_TAU = LTX_RESCALE_TAU;
// 2^TAU: a lane's probability sum at or under it bounds every probability of the lane by 2^TAU
constexpr float RESCALE_SUM = (float)(1u << (int)LTX_RESCALE_TAU);

// lane l and lane l ^ 32 combined without an LDS round trip (v_permlane32_swap): both halves
// get the bit-identical result (same operand order in every lane)
__device__ __forceinline__ float xor32_max(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float xor32_sum(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// XCD-aware block order: the hardware deals consecutive workgroups round-robin over the 8 XCDs,
// which would spread the blocks of one (batch, head) -- all reading the same K/V (or Q/dO) --
// over 8 L2s and fetch those operands 8 times from beyond L2 (~1 GB per launch measured at
// config A). Bijective remap: XCD x takes a contiguous range of the (x fastest, head, batch)
// block order.
__device__ __forceinline__ void xcd_block(int xcd_order, int& bx, int& by, int& bz) {
  if (!xcd_order) {
    bx = blockIdx.x;
    by = blockIdx.y;
    bz = blockIdx.z;
    return;
  }
  const int gx = gridDim.x, gy = gridDim.y;
  const int total = gx * gy * gridDim.z;
  const int L = blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z);
  const int q = total / 8, r = total % 8, xcd = L % 8, idx = L / 8;
  const int wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
  bx = wg % gx;
  by = (wg / gx) % gy;
  bz = wg / (gx * gy);
}


// Row-contiguous store of a wave's 32 x HD output block (O, dQ, dK or dV): the accumulator holds
// a row's dims in 4-wide groups at a stride of 8 (acc_row), so direct stores are 8-B pieces of 64
// different lines per instruction. Staged through a wave-private 4-KiB LDS slot (16-B chunks XOR
// row & 7: conflict-free both ways), each store instruction then writes 8 whole 128-B rows.
// `scale` multiplies before the bf16 rounding (the same values as the per-lane path).
// The same through a 1-KiB slot, 8 rows per pass (4 passes): the lanes holding a pass's rows write
// them, then every lane reads 16 B and one store instruction writes the pass's 8 whole rows.
template <int HD>
__device__ __forceinline__ void store_rows_lds1k(char* stage, const f32x16* acc, float scale, bf16_t* out,
                                                 int64_t ld, int row0, int nrows, int lane) {
  static_assert(HD == 64, "128-B rows");
  const int h = lane >> 5, r = lane & 31;
#pragma unroll
  for (int ps = 0; ps < 4; ++ps) {
    if ((r >> 3) == ps) {  // each lane's row falls in exactly one pass
      const int rl = r & 7;
#pragma unroll
      for (int d = 0; d < HD / 32; ++d)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int col = d * 32 + 8 * g + 4 * h;
          u32x2 w;
          w[0] = pack2(acc[d][4 * g] * scale, acc[d][4 * g + 1] * scale);
          w[1] = pack2(acc[d][4 * g + 2] * scale, acc[d][4 * g + 3] * scale);
          *(u32x2*)(stage + rl * 128 + ((((col >> 3) ^ rl)) << 4) + ((col >> 2) & 1) * 8) = w;
        }
    }
    const int rr = lane >> 3, c = lane & 7;
    const u32x4 v = *(const u32x4*)(stage + rr * 128 + ((c ^ rr) << 4));
    if (8 * ps + rr < nrows) *(u32x4*)(out + (int64_t)(row0 + 8 * ps + rr) * ld + c * 8) = v;
  }
}

template <int HD>
__device__ __forceinline__ void store_rows_lds(char* stage, const f32x16* acc, float scale, bf16_t* out,
                                               int64_t ld, int row0, int nrows, int lane) {
  static_assert(HD == 64, "128-B rows");
  const int h = lane >> 5, r = lane & 31;
#pragma unroll
  for (int d = 0; d < HD / 32; ++d)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int col = d * 32 + 8 * g + 4 * h;  // 4 dims: chunk col >> 3, half (col >> 2) & 1
      u32x2 w;
      w[0] = pack2(acc[d][4 * g] * scale, acc[d][4 * g + 1] * scale);
      w[1] = pack2(acc[d][4 * g + 2] * scale, acc[d][4 * g + 3] * scale);
      *(u32x2*)(stage + r * 128 + ((((col >> 3) ^ (r & 7))) << 4) + ((col >> 2) & 1) * 8) = w;
    }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int rr = i * 8 + (lane >> 3), c = lane & 7;
    const u32x4 v = *(const u32x4*)(stage + rr * 128 + ((c ^ (rr & 7)) << 4));
    if (rr < nrows) *(u32x4*)(out + (int64_t)(row0 + rr) * ld + c * 8) = v;
  }
}

// The same rows stored from registers with 16-B pieces: lanes l and l ^ 32 hold the two 4-dim
// halves of every 8-dim chunk, one v_permlane32_swap per dword hands lane l (h = 0) the even
// chunks and lane l + 32 the odd ones whole (cdna guide T21), so each store instruction writes
// 32 contiguous bytes of each of 32 rows instead of 8-B pieces. `row` is this lane's output row
// (null: not stored).
template <int HD>
__device__ __forceinline__ void store_row_swap(const f32x16* acc, float scale, bf16_t* row, int lane) {
  const int h = lane >> 5;
#pragma unroll
  for (int d = 0; d < HD / 32; ++d)
#pragma unroll
    for (int gp = 0; gp < 4; gp += 2) {
      u32x2 w[2];
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int g = gp + e;
        w[e][0] = pack2(acc[d][4 * g] * scale, acc[d][4 * g + 1] * scale);
        w[e][1] = pack2(acc[d][4 * g + 2] * scale, acc[d][4 * g + 3] * scale);
      }
      u32x4 c;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const auto r = __builtin_amdgcn_permlane32_swap(w[0][j], w[1][j], false, false);
        c[j] = r[0];      // h = 0: own dims 0-3 of chunk gp; h = 1: partner's dims 0-3 of chunk gp+1
        c[2 + j] = r[1];  // h = 0: partner's dims 4-7;        h = 1: own dims 4-7
      }
      if (row) *(u32x4*)(row + d * 32 + 8 * (gp + h)) = c;
    }
}

// the dK/dV kernel with the software-pipelined, LDS-DMA-staged loop (attention_dkdv.hip)
int launch_dkdv_pipe(const AttnParams& p, hipStream_t s);
bool dkdv_pipe_enabled();
// the dQ kernel with the same structure, for key ranges without bias (Nk % 64 == 0)
int launch_dq_pipe(const AttnParams& p, hipStream_t s);
bool dq_pipe_enabled();
// the dK/dV kernel at one wave per SIMD (hand-scheduled loop, attn_bwd_body.h): no key bias, head dim 64
int launch_dkdv_w1(const AttnParams& p, hipStream_t s);
bool dkdv_w1_enabled();
// the persistent dK/dV kernel (one workgroup per CU walking 256-key blocks; attn_bwd_body.h)
int launch_dkdv_w1p(const AttnParams& p, hipStream_t s);
bool dkdv_w1p_enabled();
bool dkdv_w1p_applies(const AttnParams& p);
// the persistent dQ kernel (one workgroup per CU walking 256-query blocks; bf16 dQ)
int launch_dq_w1p(const AttnParams& p, hipStream_t s);
bool dq_w1p_enabled();
bool dq_w1p_applies(const AttnParams& p);
// the dQ kernel at one wave per SIMD (hand-scheduled loop, attn_bwd_body.h): no key bias, head dim 64
int launch_dq_w1(const AttnParams& p, hipStream_t s);
bool dq_w1_enabled();
// the forward with K / V by LDS-DMA and one barrier per tile (no key bias, Nk % 64 == 0)
int launch_fwd_pipe(const AttnParams& p, hipStream_t s);
bool fwd_pipe_enabled();

}  // namespace ltx
