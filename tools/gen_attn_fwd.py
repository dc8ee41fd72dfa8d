"""Generates tools/experiments/attn_fwd_body.h (or the path given as the first argument; `make fwdw1` in
csrc builds the opt-in library with it -- the kernel is measured slower than the default and is not
in the shipping build): the hand-scheduled main loop of
attn_fwd_w1_kernel (attention_pipe.hip), the self-attention forward of F.scaled_dot_product_attention
(attention.py:1057-1064) for head dim 64 and no key bias, as ONE inline-asm statement.

Why: at head dim 64 a score costs one v_fma + one v_exp_f32 + one f32 add + half a
v_cvt_pk_bf16_f32 (~18 VALU cycles) against 16 MFMA cycles, and attn_fwd_pipe_kernel's eight hipcc-
scheduled waves reach MFMA-busy 0.44. Here one wave per SIMD owns 64 queries (two 32-query tiles qt,
every K / V fragment read from LDS feeds both) and every instruction is placed.

Arithmetic, accumulation order and rescale decisions are attn_fwd_pipe_kernel<true>'s, so O and lse are
bitwise equal to it (tests/test_kernels_gpu.py): S = K.Q^T by k-steps of 16 dims, the probability
exp2(S c2 - m) with the running max m, the deferred max (a tile is redone with its true max when some
lane's probability sum exceeds 2^TAU; the first tile always), four f32 sum chains per 64-key tile,
the P.V products in (32-key half, 16-key step) order per accumulator.

Schedule: units of 64 keys (one LDS tile). Unit u holds 32 MFMA slots:
  slots 4-19   C(u-1): O^T[qt][d] += V^T[kh][ss][d] . P(u-1)[qt][kh][ss]   (16 MFMAs)
  slots 20-35  A(u+1): S(u+1)[qt][kh] = K[kh].Q[qt]^T                       (16 MFMAs; 32-35 = next unit's 0-3)
  B(u): the 64 scores of the lane (2 qt x 2 kh x 16) as 32 pairs, pair p's packed-free v_fma in slot p,
        its two v_exp_f32 in p+1, its two chain adds and one v_cvt_pk in p+2 (probabilities are exponent-
        iated out of place, so S(u) survives for a redo)
  check(u-1) in slot 2: the tile's lane sums (ls0 + ls1) + (ls2 + ls3) per qt, one vote each; a vote
        branches to an out-of-line redo (recompute S(u-1), its max, the decision, its probabilities,
        the O / l rescale, and B(u)'s pairs 0-1 done so far at the new max), then back.
Tiles of 64 keys arrive by LDS-DMA into a 4-buffer ring (tiles u-1 .. u+2 live in unit u), one barrier
per unit. Keys are a multiple of 64 (the kernel's precondition); query rows past Nq are clamped loads
(computed, not stored).

Registers (hard-coded, clobbered; the O accumulators are the statement's "+a" operands %0..%3, which
hipcc places in a0..a127, and m / l are "+v" operands %4..%7):
  v[0:127]   S sets: set s, qt, kh at 64 s + 32 qt + 16 kh
  v[128:191] P packs: set p, qt, kh, ss at 128 + 32 p + 16 qt + 8 kh + 4 ss
  v[192:199] sum chains of the tile in flight: qt, chain c at 192 + 4 qt + c
  v[200:215] probability temporaries (rotating pairs)
  v[216:223] LDS addresses: RK[ks] (K rows of A's tile), TC[4] (V^T fragments of C's tile)
  v[224:231] check / redo scratch
  a[128:159] Q fragments QF[qt][ks], a[160:191] K row fragments KA[kh][ks], a[192:223] V^T fragments
             VT[kh][ss][d]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gen_attn_bwd import Emitter, I, v, a_  # noqa: E402

F_TILE = 8192            # one [64][64] bf16 tile
F_BUF = 2 * F_TILE       # K | V
NBUF = 4
TAU = 8.0
RESCALE_SUM = 256.0

SSET = lambda s, qt, kh: 64 * s + 32 * qt + 16 * kh
PK = lambda p, qt, kh, ss: 128 + 32 * p + 16 * qt + 8 * kh + 4 * ss
LSC = lambda qt, c: 192 + 4 * qt + c
PT0 = 200                # probability temporaries v[200:215]: 8 rotating pairs
RK = [216, 217, 218, 219]
TC = [220, 221, 222, 223]
VLAST = 231
QF = lambda qt, ks: 128 + 16 * qt + 4 * ks
KA = lambda kh, ks: 160 + 16 * kh + 4 * ks
VT = lambda kh, ss, d: 192 + 16 * kh + 8 * ss + 4 * d
SRDK, SRDV = 80, 84
VARIANT = set(x for x in os.environ.get("GEN_FWD_VARIANT", "").split(",") if x)  # debug: noscale, nopair


def OACC(qt, d):
    return "%" + str(2 * qt + d)


def MRUN(qt):  # the running max m of qt's queries (log2 units; the fma subtracts it)
    return "%" + str(4 + qt)


def LRUN(qt):
    return "%" + str(6 + qt)


def mfma(dst, A, B, C, needs=()):
    return I(f"v_mfma_f32_32x32x16_bf16 {dst}, {A}, {B}, {C}", needs=needs)


def a_mfmas(s):
    """A(u+1) into S set s: chains (qt, kh) interleaved k-step by k-step, each in k order"""
    out = []
    for ks in range(4):
        for qt in range(2):
            for kh in range(2):
                dst = v(SSET(s, qt, kh), 16)
                out.append(mfma(dst, a_(KA(kh, ks), 4), a_(QF(qt, ks), 4), "0" if ks == 0 else dst,
                                needs=[f"KA{kh}{ks}"]))
    return out


def c_mfmas(p):
    """C(u-1) from pack set p: for each (kh, ss) k-step, every (qt, d) accumulator (each in k order)"""
    out = []
    for kh in range(2):
        for ss in range(2):
            for qt in range(2):
                for d in range(2):
                    acc = OACC(qt, d)
                    out.append(mfma(acc, a_(VT(kh, ss, d), 4), v(PK(p, qt, kh, ss), 4), acc,
                                    needs=[f"VT{kh}{ss}{d}"]))
    return out


def pairs():
    """the 32 pairs of B in order: (qt, kh, ss, j): scores 8 ss + 2 j, +1 of S[qt][kh] (chain 2 kh + ss,
    pack word j)"""
    return [(qt, kh, ss, j) for qt in range(2) for kh in range(2) for ss in range(2) for j in range(4)]


def b_ops(s, p, pi, pair, tmp=None):
    """pair pi of B on S set s, packs p: (fma list, exp list, add+cvt list); the probabilities are
    exp2(fma(S, c2, -m)) in temporaries (S survives)"""
    qt, kh, ss, j = pair
    sr = SSET(s, qt, kh) + 8 * ss + 2 * j
    t = PT0 + 2 * (pi % 8) if tmp is None else tmp
    m = MRUN(qt)
    c = LSC(qt, 2 * kh + ss)
    fm = [I(f"v_fma_f32 {v(t)}, {v(sr)}, %[c2], -{m}"), I(f"v_fma_f32 {v(t + 1)}, {v(sr + 1)}, %[c2], -{m}")]
    ex = [I(f"v_exp_f32 {v(t)}, {v(t)}"), I(f"v_exp_f32 {v(t + 1)}, {v(t + 1)}")]
    first = j == 0
    ad = [I(f"v_add_f32 {v(c)}, 0, {v(t)}" if first else f"v_add_f32 {v(c)}, {v(c)}, {v(t)}"),
          I(f"v_add_f32 {v(c)}, {v(c)}, {v(t + 1)}"),
          I(f"v_cvt_pk_bf16_f32 {v(PK(p, qt, kh, ss) + j)}, {v(t)}, {v(t + 1)}")]
    return fm, ex, ad


def b_stream(s, p):
    """B(u) on S set s into pack set p: {slot: [I]} over slots 0 .. 33 of unit u"""
    out = {}
    for pi, pair in enumerate(pairs()):
        fm, ex, ad = b_ops(s, p, pi, pair)
        out.setdefault(pi, []).extend(fm)
        out.setdefault(pi + 1, []).extend(ex)
        out.setdefault(pi + 2, []).extend(ad)
    return out


def ka_reads(T):
    """A's K row fragments (both 32-key halves) of the tile at RK-base T"""
    out = []
    for kh in range(2):
        for ks in range(4):
            out.append(I(f"ds_read_b128 {a_(KA(kh, ks), 4)}, {v(RK[ks])} offset:{kh * 4096}", makes=f"KA{kh}{ks}"))
    return out


def vt_reads(T):
    """C's V^T fragments of the tile at address regs T (TC / TN)"""
    out = []
    for kh in range(2):
        for ss in range(2):
            for d in range(2):
                base = F_TILE + (kh * 32 + 16 * ss) * 128
                tag = f"VT{kh}{ss}{d}"
                out.append(I(f"ds_read_b64_tr_b16 {a_(VT(kh, ss, d), 2)}, {v(T[2 * d])} offset:{base}", makes=tag))
                out.append(I(f"ds_read_b64_tr_b16 {a_(VT(kh, ss, d) + 2, 2)}, {v(T[2 * d + 1])} offset:{base}",
                             makes=tag))
    return out


def dma(buf):
    """this wave's DMA of one K / V tile into the buffer at SGPR `buf`: K pieces 2w, 2w+1, V likewise"""
    out = []
    for i in range(2):
        out.append((f"s_add_u32 m0, s{buf}, %[wq{i}]", f"buffer_load_dwordx4 %[vk{i}], s[{SRDK}:{SRDK + 3}], 0 offen lds"))
        out.append((f"s_add_u32 m0, s{buf}, %[wqv{i}]", f"buffer_load_dwordx4 %[vv{i}], s[{SRDV}:{SRDV + 3}], 0 offen lds"))
    return out


def advance():
    out = []
    for srd, step in ((SRDK, "%[kstep]"), (SRDV, "%[vstep]")):
        out += [f"s_add_u32 s{srd}, s{srd}, {step}", f"s_addc_u32 s{srd + 1}, s{srd + 1}, 0",
                f"s_sub_u32 s{srd + 2}, s{srd + 2}, {step}", f"s_cselect_b32 s{srd + 2}, 0, s{srd + 2}"]
    return out


def rk_addr(buf):
    return [f"v_add_u32 {v(RK[ks])}, s{buf}, %[vr{ks}]" for ks in range(4)]


def t_addr(T, buf):
    return [f"v_add_u32 {v(T[k])}, s{buf}, %[vt{k}]" for k in range(4)]




# ---------------------------------------------------------------------------------------- the unit
LS = [224, 225]          # the checked tile's lane sums (qt 0 / 1)
T1, T2 = 226, 227
ZERO = 228               # v[228:231]: a zero tuple (the redo's accumulator copies)
REDO_T = 208             # redo temporaries v[208:215] (pairs 0, 1 of B(u) keep v[200:203])
SBUF = [88, 89, 90, 91, 92, 93]      # ring: tiles u-2+1 .. : SB[0] = u-1, SB[1] = u, .., SB[5] = u+4 (target)
STMP, SITER, SKEEP = 94, 95, 97


def rot6():
    return [f"s_mov_b32 s{STMP}, s{SBUF[0]}"] + [f"s_mov_b32 s{SBUF[i]}, s{SBUF[i + 1]}" for i in range(5)] + \
           [f"s_mov_b32 s{SBUF[5]}, s{STMP}"]


def dma6(buf):
    out = []
    for i, (m0, ld) in enumerate(dma(buf)):
        out += [m0, "s_nop 0", ld]
    return out


class Unit:
    """one 64-key unit u of the pipeline; flags say which stages exist"""
    def __init__(self, par, ctail, check, c, a, b, dma_next, ka_next, tag):
        self.par, self.ctail, self.check, self.c, self.a, self.b = par, ctail, check, c, a, b
        self.dma_next, self.ka_next, self.tag = dma_next, ka_next, tag


REDOS = []               # (label tag, par, qt) of every check emitted: their out-of-line blocks


def emit_unit(E, U, vm=4):
    a = E.raw
    par, sp = U.par, 1 - U.par
    # ---- unit start: tile u+2 landed (tile u+3 may fly), every wave done with tile u-2; the ring turns
    E.drain(f"s_waitcnt vmcnt({vm}) lgkmcnt(0)")
    a("s_barrier")
    if U.dma_next:
        for t in dma6(SBUF[5]):
            a(t)
        for t in advance():
            a(t)
    if U.c:
        for t in t_addr(TC, SBUF[0]):
            a(t)
    if U.ka_next:
        for t in rk_addr(SBUF[3]):
            a(t)
    cm_tail = c_mfmas(par)[13:] if U.ctail else []      # C(u-2): packs of tile u-2 (same parity as u)
    am = a_mfmas(sp) if U.a else []                      # A(u+1) into the other S set
    cm = c_mfmas(sp) if U.c else []                      # C(u-1): packs of tile u-1
    bcur = b_stream(par, par) if U.b else {}
    bprev = b_stream(sp, sp) if U.check else {}          # B(u-1)'s tail: slots 32, 33 -> 0, 1
    if "novalu" in VARIANT:
        bcur, bprev = {}, {}
    reads = {}
    if U.c:
        for i, x in enumerate(vt_reads(TC)):
            reads.setdefault(3 + i, []).append(x)
    if U.ka_next:
        for i, x in enumerate(ka_reads(None)):
            reads.setdefault(19 + i, []).append(x)
    for k in range(32):
        if k < 3 and cm_tail:
            E.put(cm_tail[k])
        if 3 <= k < 19 and am:
            E.put(am[k - 3])
        if k >= 19 and cm:
            E.put(cm[k - 19])
        if k == 2 and U.check and "novalu" not in VARIANT:
            emit_check(E, U)
        for ins in reads.get(k, []) + bprev.get(k + 32, []) + bcur.get(k, []):
            E.put(ins)


def emit_check(E, U):
    """check(u-1): per qt the tile's lane sums, one vote; a vote runs the redo out of line"""
    a = E.raw
    for qt in range(2):
        a(f"v_add_f32 {v(T1)}, {v(LSC(qt, 0))}, {v(LSC(qt, 1))}")
        a(f"v_add_f32 {v(T2)}, {v(LSC(qt, 2))}, {v(LSC(qt, 3))}")
        a(f"v_add_f32 {v(LS[qt])}, {v(T1)}, {v(T2)}")
        a(f"v_cmp_lt_f32 vcc, {RESCALE_SUM}, {v(LS[qt])}")
        a(f"s_cbranch_vccnz L_redo_{U.tag}_{qt}_%=")
        a(f"L_back_{U.tag}_{qt}_%=:")
        REDOS.append((U.tag, U.par, qt))
    for qt in range(2):
        a(f"v_add_f32 {LRUN(qt)}, {LRUN(qt)}, {v(LS[qt])}")


def emit_redo(E, tag, par, qt):
    """pass 1 of attn_fwd_pipe_kernel for tile u-1 (S set sp, packs sp), query tile qt: the tile's max, the
    rescale decision; on a rescale the probabilities, sums and packs at the new max, l and O scaled
    by alpha (O through MFMA copies: the accumulators are operands), and B(u)'s pairs 0-1 (done before
    the check, qt 0) redone at the new max"""
    a = E.raw
    sp = 1 - par
    a(f"L_redo_{tag}_{qt}_%=:")
    for _ in range(4):
        a("s_nop 15")
    # the tile max of the lane's 32 scores, x c2, max with the partner half (v_permlane32_swap)
    regs = [SSET(sp, qt, kh) + r for kh in range(2) for r in range(16)]
    m = REDO_T
    a(f"v_max3_f32 {v(m)}, {v(regs[0])}, {v(regs[1])}, {v(regs[2])}")
    i = 3
    while i < 32:
        if i + 1 < 32:
            a(f"v_max3_f32 {v(m)}, {v(m)}, {v(regs[i])}, {v(regs[i + 1])}")
            i += 2
        else:
            a(f"v_max_f32 {v(m)}, {v(m)}, {v(regs[i])}")
            i += 1
    a(f"v_mul_f32 {v(m)}, {v(m)}, %[c2]")
    a(f"v_mov_b32 {v(m + 1)}, {v(m)}")
    a("s_nop 1")
    a(f"v_permlane32_swap_b32 {v(m)}, {v(m + 1)}")
    a(f"v_max_f32 {v(m)}, {v(m)}, {v(m + 1)}")                 # mt
    a(f"v_max_f32 {v(m + 1)}, {MRUN(qt)}, {v(m)}")             # m_new = max(m_run, mt)
    a(f"v_add_f32 {v(m + 2)}, {TAU}, {MRUN(qt)}")              # m_run + TAU
    a(f"v_cmp_gt_f32 vcc, {v(m + 1)}, {v(m + 2)}")
    a(f"s_cbranch_vccz L_back_{tag}_{qt}_%=")                  # no rescale: the probabilities stand
    AL = m + 3
    a(f"v_sub_f32 {v(AL)}, {MRUN(qt)}, {v(m + 1)}")
    a(f"v_exp_f32 {v(AL)}, {v(AL)}")                           # alpha = exp2(m_run - m_new)
    a(f"v_mov_b32 {MRUN(qt)}, {v(m + 1)}")
    # probabilities, chains and packs of tile u-1 at the new max (temporaries v[212:215])
    for pi, pair in enumerate([p for p in pairs() if p[0] == qt]):
        fm, ex, ad = b_ops(sp, sp, pi, pair, tmp=212 + 2 * (pi % 2))
        for ins in fm + ex + ad:
            a(ins.text)
    a(f"v_add_f32 {v(T1)}, {v(LSC(qt, 0))}, {v(LSC(qt, 1))}")
    a(f"v_add_f32 {v(T2)}, {v(LSC(qt, 2))}, {v(LSC(qt, 3))}")
    a(f"v_add_f32 {v(LS[qt])}, {v(T1)}, {v(T2)}")
    a(f"v_mul_f32 {LRUN(qt)}, {LRUN(qt)}, {v(AL)}")
    # O[qt][d] *= alpha: copy the accumulator to a[192 + 16 d] (MFMA with zero operands), scale, copy back
    # (the zero tuple is set once in the prologue: a v_mov right before the MFMA reading it is a hazard)
    nd = 0 if "noscale" in VARIANT else 2
    for d in range(nd):
        a(f"v_mfma_f32_32x32x16_bf16 {a_(192 + 16 * d, 16)}, {v(ZERO, 4)}, {v(ZERO, 4)}, {OACC(qt, d)}")
    for _ in range(5):
        a("s_nop 15")
    for d in range(nd):
        for r in range(16):
            a(f"v_accvgpr_read_b32 {v(m + 4)}, {a_(192 + 16 * d + r)}")
            a(f"v_mul_f32 {v(m + 4)}, {v(m + 4)}, {v(AL)}")
            a(f"v_accvgpr_write_b32 {a_(192 + 16 * d + r)}, {v(m + 4)}")
    a("s_nop 4")
    for d in range(nd):
        a(f"v_mfma_f32_32x32x16_bf16 {OACC(qt, d)}, {v(ZERO, 4)}, {v(ZERO, 4)}, {a_(192 + 16 * d, 16)}")
    for _ in range(5):
        a("s_nop 15")
    if qt == 0 and "nopair" not in VARIANT:  # B(u)'s pairs done before the check: pair 0 (fma, exp), pair 1 (fma)
        for pi in (0, 1):
            fm, ex, ad = b_ops(par, par, pi, pairs()[pi])
            for ins in fm + (ex if pi == 0 else []):
                a(ins.text)
    a(f"s_branch L_back_{tag}_{qt}_%=")


def body():
    """the whole forward statement: prologue (Q fragments, tiles 0-3, A(0), tile 0's max), units 0 and 1,
    the two-unit loop over units 2 .. U-1 (an odd unit count adds one), the closing unit U (check and
    C of the last tile) and C's last three MFMAs"""
    E = Emitter()
    a = E.raw
    REDOS.clear()
    a(f"s_mov_b32 s{SKEEP}, m0")
    a("s_nop 4")
    for srd, nm in ((SRDK, "sk"), (SRDV, "sv")):
        a(f"s_mov_b64 s[{srd}:{srd + 1}], %[{nm}0]")
        a(f"s_mov_b64 s[{srd + 2}:{srd + 3}], %[{nm}1]")
    for qt in range(2):
        for ks in range(4):
            a(f"global_load_dwordx4 {a_(QF(qt, ks), 4)}, %[qp{qt}], off offset:{ks * 32}")
    for r in range(4):  # the redo's zero operand tuple (never written again)
        a(f"v_mov_b32 {v(ZERO + r)}, 0")
    # ring: SBUF[0] = tile -1 (buffer 5), SBUF[1..5] = tiles 0..4 (buffers 0..4)
    a(f"s_add_u32 s{SBUF[0]}, %[lds0], {5 * F_BUF}")
    for i in range(1, 6):
        a(f"s_add_u32 s{SBUF[i]}, %[lds0], {(i - 1) * F_BUF}")
    a("s_nop 2")
    for i in range(1, 5):  # tiles 0 .. 3
        for t in dma6(SBUF[i]) + advance():
            a(t)
    a("s_waitcnt vmcnt(8)")  # Q fragments, tiles 0 and 1 landed (tiles 2, 3 fly)
    a("s_barrier")
    for t in rk_addr(SBUF[1]):
        a(t)
    for ins in ka_reads(None):
        E.put(ins)
    for ins in a_mfmas(0):  # A(0): S(0) into set 0
        E.put(ins)
    for _ in range(2):
        a("s_nop 7")
    for t in rk_addr(SBUF[2]):
        a(t)
    for ins in ka_reads(None):  # tile 1's K rows for A(1) (unit 0)
        E.put(ins)
    for _ in range(2):
        a("s_nop 15")
    # tile 0 (pass 1 of the pipelined kernel): m = max over the tile x c2; l and O stay 0 (alpha = 0)
    for qt in range(2):
        regs = [SSET(0, qt, kh) + r for kh in range(2) for r in range(16)]
        m = REDO_T
        a(f"v_max3_f32 {v(m)}, {v(regs[0])}, {v(regs[1])}, {v(regs[2])}")
        i = 3
        while i < 32:
            if i + 1 < 32:
                a(f"v_max3_f32 {v(m)}, {v(m)}, {v(regs[i])}, {v(regs[i + 1])}")
                i += 2
            else:
                a(f"v_max_f32 {v(m)}, {v(m)}, {v(regs[i])}")
                i += 1
        a(f"v_mul_f32 {v(m)}, {v(m)}, %[c2]")
        a(f"v_mov_b32 {v(m + 1)}, {v(m)}")
        a("s_nop 1")
        a(f"v_permlane32_swap_b32 {v(m)}, {v(m + 1)}")
        a(f"v_max_f32 {MRUN(qt)}, {v(m)}, {v(m + 1)}")
    # unit 0: B(0), A(1); unit 1: B(1), check(0), A(2), C(0)
    emit_unit(E, Unit(0, ctail=False, check=False, c=False, a=True, b=True, dma_next=True, ka_next=True, tag="u0"), vm=4)
    for t in rot6():
        a(t)
    emit_unit(E, Unit(1, ctail=False, check=True, c=True, a=True, b=True, dma_next=True, ka_next=True, tag="u1"))
    a(f"s_mov_b32 s{SITER}, %[iters]")
    a(f"s_cmp_eq_u32 s{SITER}, 0")
    a("s_cbranch_scc1 L_loop_end_%=")
    if "stamps" in VARIANT:
        a("s_memtime s[72:73]")
    a("L_loop_%=:")
    stamp(E, 0)
    for par in (0, 1):
        for t in rot6():
            a(t)
        emit_unit(E, Unit(par, ctail=True, check=True, c=True, a=True, b=True, dma_next=True, ka_next=True,
                          tag=f"l{par}"))
        stamp(E, 1 + par)
    a(f"s_sub_u32 s{SITER}, s{SITER}, 1")
    a(f"s_cmp_eq_u32 s{SITER}, 0")
    a("s_cbranch_scc0 L_loop_%=")
    a("L_loop_end_%=:")
    if "stamps" in VARIANT:
        a("s_memtime s[74:75]")
    a("s_cmp_eq_u32 %[uodd], 0")
    a("s_cbranch_scc1 L_even_%=")
    # U odd: one more unit (u = U - 1, even), then the closing unit U (odd)
    for t in rot6():
        a(t)
    emit_unit(E, Unit(0, ctail=True, check=True, c=True, a=True, b=True, dma_next=True, ka_next=True, tag="x0"))
    close(E, 1, "c1")
    a("s_branch L_done_%=")
    a("L_even_%=:")
    close(E, 0, "c0")
    a("L_done_%=:")
    if "stamps" in VARIANT:
        for k in range(8):
            a(f"v_mov_b32 v0, s{60 + 2 * k}")
            a(f"v_mov_b32 v1, s{61 + 2 * k}")
            a(f"global_store_dwordx2 %[stp], v[0:1], off offset:{8 * k}")
            a("s_nop 1")
    a("s_waitcnt vmcnt(0)")
    a(f"s_mov_b32 m0, s{SKEEP}")
    for _ in range(3):
        a("s_nop 15")
    # out-of-line redos (reached by branches from the checks, they branch back)
    a("s_branch L_exit_%=")
    for tag, par, qt in list(REDOS):
        emit_redo(E, tag, par, qt)
    a("L_exit_%=:")
    return E.L


def stamp(E, k):
    if "stamps" not in VARIANT:
        return
    for t in (f"s_cmp_eq_u32 s{SITER}, 5", f"s_cbranch_scc0 L_st{k}_%=", f"s_memtime s[{60 + 2 * k}:{61 + 2 * k}]",
              f"L_st{k}_%=:"):
        E.raw(t)


def close(E, par, tag):
    """the closing unit U (parity par): C(U-2)'s tail, check(U-1), C(U-1); then C(U-1)'s last MFMAs"""
    a = E.raw
    for t in rot6():
        a(t)
    emit_unit(E, Unit(par, ctail=True, check=True, c=True, a=False, b=False, dma_next=False, ka_next=False,
                      tag=tag))
    for ins in c_mfmas(1 - par)[13:]:
        E.put(ins)


def clobbers():
    regs = [f'"v{r}"' for r in range(VLAST + 1)] + [f'"a{r}"' for r in range(128, 224)] + \
           [f'"s{r}"' for r in list(range(80, 88)) + SBUF + [STMP, SITER, SKEEP]]
    if "stamps" in VARIANT:
        regs += [f'"s{r}"' for r in range(60, 76)]
    return ", ".join(regs)


def main():
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    args = [x for x in sys.argv[1:] if not x.startswith("--")]
    out = args[0] if args else os.path.join(root, "tools", "experiments", "attn_fwd_body.h")

    def define(name, lines):
        return f"#define {name} \\\n" + " \\\n".join(f'  "{l}\\n\\t"' for l in lines) + "\n"
    L = body()
    txt = ["// GENERATED by tools/gen_attn_fwd.py -- do not edit by hand.",
           "// The hand-scheduled loop of attn_fwd_w1_kernel (attention_pipe.hip); see the generator's docstring.",
           "#pragma once", "", f"#define LTX_FWD_W1_BUF {F_BUF}", "#define LTX_FWD_W1_NBUF 6",
           define("LTX_FWD_W1_BODY", L), "#define LTX_FWD_W1_CLOBBERS " + clobbers() + "\n"]
    open(out, "w").write("\n".join(txt))
    print(out, len(L), "lines")


if __name__ == "__main__":
    main()
