"""Generates video-generation-for-human-avatars_amd/csrc/attn_bwd_body.h: the hand-scheduled main loop of
attn_dkdv_w1_kernel (attention_pipe.hip), the dK / dV half of F.scaled_dot_product_attention's
backward (attention.py:1057-1064) for head dim 64 and no key bias, as ONE inline-asm statement.

Why: at head dim 64 the softmax VALU of a score block costs about as
many issue cycles as its MFMAs, and at two waves per SIMD (attn_dkdv_pipe_kernel, 248 VGPRs) the two
streams' MFMAs and VALU compete for one issue port (MFMA-busy 0.53). Here one wave per SIMD owns 64
keys (two 32-key tiles, so every Q / dO fragment read from LDS feeds two MFMAs) and every
instruction is placed. Per 32-query half j the wave issues 32 MFMAs in 32 slots: C(j-1)
(dV^T += dO^T.P, dK^T += Q^T.dS) in slots 0-15 and A(j+1) (S^T = K.Q^T, dP'^T = delta - V.dO^T) in
slots 16-31. The softmax of half j, B(j), is a stream of 32 elements (the lane's 2 x 16 scores)
that runs LAG slots behind the half's start, one element per slot: element e has its exponent
argument formed in slot e + LAG - 1 (v_fma), its exponential in e + LAG, its dS product in
e + LAG + 2 (v_mul), its P / dS bf16 packs (pairs) in e + LAG + 2 / e + LAG + 3, so each MFMA gap
carries one fma, one exp, one mul, about one cvt and one LDS read -- the same filler mix in every
slot (the phase-split schedule, two exponentials per gap in one phase, measured ~50 cycles per MFMA
in that phase with in-kernel stamps). The stream ends in slot 42 = slot 10 of the next half, and
the C MFMAs run in pack order (ss, kt, d), so no pack is rewritten before the C stage of the
previous half has read it and every pack is written before the next C stage reads it.

Arithmetic and accumulation order are those of attn_dkdv_pipe_kernel (same fragment layouts, MFMA
chains in the same k order, delta as dP's initial accumulator with V negated), so dK / dV are
bitwise equal to it (tests/test_kernels_gpu.py). LDS reads carry tags; the generator inserts the
counted s_waitcnt lgkmcnt(N) in front of the first consumer of a read (LDS returns in order).

Tiles of 64 queries (Q | dO | lse | delta) arrive by LDS-DMA into a 3-buffer ring, one tile ahead,
one barrier per tile. Rows past Nq are out of range of the tile's buffer descriptor (the base
advances and num_records shrinks per tile), so they land as zeros: S = 0, lse = 0 gives P = 1, but
their dO and delta rows are 0, so they add exactly 0 to dV (dO^T.P) and dS = -P (delta - dO.V) = 0.

Registers (hard-coded, clobbered; the dV / dK accumulators are the statement's "+a" operands
%0..%7, which hipcc must place in a0..a127):
  v[0:63]    S tiles: set s (0, 1), key tile kt at 32 s + 16 kt; v[66:129] the dP' tiles likewise
             at 66 + 32 s + 16 kt (two banks away from their S)
  v[130:145] P packs  PB[kt][ss] (B operands of dV) at 130 + 8 kt + 4 ss
  v[146:161] dS packs SB[kt][ss] at 146 + 8 kt + 4 ss
  v[162:177], v[210:225]  lse tuples of even / odd halves (accumulator row order)
  v[178:193] delta tuple of the half whose A stage runs (dP chains' initial accumulator)
  v[194:206] LDS addresses: RA[ks] row fragments (A's tile), ST statistics (A's tile), TC / TN[2d+i]
             transposed fragments of the current / next tile
  a[128:159] K fragments KF[kt][ks], a[160:191] -V fragments, a[192:223] QA / OA row fragments,
  a[224:255] TO / TQ transposed fragments
  s[80:91]   buffer descriptors of Q, dO and this wave's statistic row (lse or delta)
  s[92:97]   ring buffer bases B0 / B1 / BD, scratch, loop counter, saved M0
"""
import os
import sys

P_TILE = 8192            # one [64][64] bf16 tile
P_STAT = 256             # 64 f32
W_BUF = 2 * P_TILE + 3 * P_STAT   # Q | dO | lse | delta | dummy (waves 2, 3)
NBUF = 3
LAG = 8                  # B(j)'s element e is exponentiated in slot e + LAG of half j

VARIANT = set()          # diagnostic bodies (--diag): "stamps", "novalu", "nolds", "dmalast", "expfirst"


# ---------------------------------------------------------------------------------------- registers
def SD(s, T):
    """S tiles (T even) at 32 s + 16 kt, dP' tiles (T odd) at 66 + 32 s + 16 kt: an element's S and dP'
    registers sit in different VGPR banks (index mod 4), as do S and its lse word, so no v_fma /
    v_mul reads two operands from one bank"""
    kt = T // 2
    return 32 * s + 16 * kt + (66 if T % 2 else 0)


def PB(kt, ss):
    return 130 + 8 * kt + 4 * ss


def SB(kt, ss):
    return 146 + 8 * kt + 4 * ss


LSEB = (162, 210)        # lse tuple of halves j with j % 2 == 0 / 1 (bank of row r: r + 2)
DLT = 178
RA = [194, 195, 196, 197]
ST = 198
TC = [199, 200, 201, 202]
TN = [203, 204, 205, 206]
VLAST = 225
KF = lambda kt, ks: 128 + 16 * kt + 4 * ks
VF = lambda kt, ks: 160 + 16 * kt + 4 * ks
QA = lambda ks: 192 + 4 * ks
OA = lambda ks: 208 + 4 * ks
TO = lambda ss, d: 224 + 4 * (2 * ss + d)
TQ = lambda ss, d: 240 + 4 * (2 * ss + d)
SRDQ, SRDO, SRDS = 80, 84, 88
SB0, SB1, SBD, STMP, SITER, SKEEP = 92, 93, 94, 95, 96, 97
ACC = {("dv", 0, 0): 0, ("dv", 0, 1): 1, ("dv", 1, 0): 2, ("dv", 1, 1): 3,
       ("dk", 0, 0): 4, ("dk", 0, 1): 5, ("dk", 1, 0): 6, ("dk", 1, 1): 7}


def ACC_REG(kind, kt, d):
    """the persistent kernel's accumulators: dV (kt, d) at a[16 (2 kt + d)], dK at a[64 + 16 (2 kt + d)]"""
    return (64 if kind == "dk" else 0) + 16 * (2 * kt + d)


def v(r, n=1):
    return f"v{r}" if n == 1 else f"v[{r}:{r + n - 1}]"


def a_(r, n=1):
    return f"a{r}" if n == 1 else f"a[{r}:{r + n - 1}]"


class I:
    """one instruction: text, the LDS-read tag it produces (reads) or the tags it needs (consumers)"""
    def __init__(self, text, makes=None, needs=()):
        self.text, self.makes, self.needs = text, makes, tuple(needs)


def mfma(dst, A, B, C, needs=()):
    return I(f"v_mfma_f32_32x32x16_bf16 {dst}, {A}, {B}, {C}", needs=needs)


# ---------------------------------------------------------------------------------------- stages
HARD_ACC = [False]       # persistent kernel: accumulators at fixed AGPRs (ACC_REG) instead of operands


def acc_name(kind, kt, d):
    if HARD_ACC[0]:
        return a_(ACC_REG(kind, kt, d), 16)
    return "%" + str(ACC[(kind, kt, d)])


def c_mfmas():
    """C(j-1) in pack order (ss, kt, d): dV^T[kt][d] += TO[ss][d] . PB[kt][ss], then dK^T with TQ, SB;
    each accumulator takes ss = 0 then ss = 1 (attn_dkdv_pipe_kernel's order)"""
    out = []
    for ss in range(2):
        for kt in range(2):
            for d in range(2):
                dv = acc_name("dv", kt, d)
                dk = acc_name("dk", kt, d)
                out.append(mfma(dv, a_(TO(ss, d), 4), v(PB(kt, ss), 4), dv, needs=[f"TO{ss}{d}"]))
                out.append(mfma(dk, a_(TQ(ss, d), 4), v(SB(kt, ss), 4), dk, needs=[f"TQ{ss}{d}"]))
    return out


def a_mfmas(s):
    """A(j+1) into set s: the chains S kt0, S kt1, dP' kt0, dP' kt1 interleaved k-step by k-step (each
    chain in k order; S starts from 0, dP' from the delta tuple)"""
    out = []
    for ks in range(4):
        for T in (0, 1):
            for kt in range(2):
                dst = v(SD(s, 2 * kt + T), 16)
                if T == 0:
                    out.append(mfma(dst, a_(QA(ks), 4), a_(KF(kt, ks), 4), "0" if ks == 0 else dst,
                                    needs=[f"QA{ks}"]))
                else:
                    out.append(mfma(dst, a_(OA(ks), 4), a_(VF(kt, ks), 4), v(DLT, 16) if ks == 0 else dst,
                                    needs=[f"OA{ks}", "DLT"] if ks == 0 else [f"OA{ks}"]))
    return out


def b_stream(s, lse):
    """B(j) on S/dP set s with the lse tuple at `lse`: {slot (0 .. 43, relative to half j): [I]}"""
    out = {}

    def put(k, ins):
        out.setdefault(k, []).append(ins)
    for e in range(32):  # pack order: ss-major, then kt, then the 8 rows of the pack
        ss, kt, i = e // 16, (e % 16) // 8, e % 8
        r = 8 * ss + i
        sr, dr = SD(s, 2 * kt) + r, SD(s, 2 * kt + 1) + r
        k = e + LAG
        put(k - 1, I(f"v_fma_f32 {v(sr)}, {v(sr)}, %[c2], -{v(lse + r)}", needs=[f"LSE{lse}"]))
        put(k, I(f"v_exp_f32 {v(sr)}, {v(sr)}"))
        put(k + 2, I(f"v_mul_f32 {v(dr)}, -{v(sr)}, {v(dr)}"))
        if e % 2 == 1:  # the pair (e-1, e): rows r-1, r
            put(k + 2, I(f"v_cvt_pk_bf16_f32 {v(PB(kt, ss) + i // 2)}, {v(sr - 1)}, {v(sr)}"))
            put(k + 3, I(f"v_cvt_pk_bf16_f32 {v(SB(kt, ss) + i // 2)}, {v(dr - 1)}, {v(dr)}"))
    return out


def a_reads(u):
    """A's operands for half u of the tile at RA / ST: Q rows, the delta tuple, dO rows"""
    out = [I(f"ds_read_b128 {a_(QA(ks), 4)}, {v(RA[ks])} offset:{u * 4096}", makes=f"QA{ks}") for ks in range(4)]
    out += [I(f"ds_read_b128 {v(DLT + 4 * g, 4)}, {v(ST)} offset:{2 * P_TILE + P_STAT + (u * 32 + 8 * g) * 4}",
              makes="DLT") for g in range(4)]
    out += [I(f"ds_read_b128 {a_(OA(ks), 4)}, {v(RA[ks])} offset:{P_TILE + u * 4096}", makes=f"OA{ks}")
            for ks in range(4)]
    return out


def tr_reads(T, u, ss):
    """C's transposed fragments (k-step ss) of half u of the tile at T (TC or TN)"""
    out = []
    for d in range(2):
        base = (u * 32 + 16 * ss) * 128
        for dst, region, nm in ((TO(ss, d), P_TILE, "TO"), (TQ(ss, d), 0, "TQ")):
            tag = f"{nm}{ss}{d}"
            out.append(I(f"ds_read_b64_tr_b16 {a_(dst, 2)}, {v(T[2 * d])} offset:{region + base}", makes=tag))
            out.append(I(f"ds_read_b64_tr_b16 {a_(dst + 2, 2)}, {v(T[2 * d + 1])} offset:{region + base}",
                         makes=tag))
    return out


def lse_reads(u, lse):
    return [I(f"ds_read_b128 {v(lse + 4 * g, 4)}, {v(ST)} offset:{2 * P_TILE + (u * 32 + 8 * g) * 4}",
              makes=f"LSE{lse}") for g in range(4)]


def dma_pieces(buf):
    """this wave's DMA of one tile into the buffer at SGPR `buf` (STMP = buf + this wave's piece
    offset): Q pieces 2w, 2w+1, dO pieces, its statistic row; (M0 write, load) pairs"""
    out = []
    for i in range(2):
        out.append((f"s_add_u32 m0, s{STMP}, {i * 1024}",
                    f"buffer_load_dwordx4 %[vq{i}], s[{SRDQ}:{SRDQ + 3}], 0 offen lds"))
        out.append((f"s_add_u32 m0, s{STMP}, {P_TILE + i * 1024}",
                    f"buffer_load_dwordx4 %[vo{i}], s[{SRDO}:{SRDO + 3}], 0 offen lds"))
    out.append((f"s_add_u32 m0, s{buf}, %[wst]",
                f"buffer_load_dword %[vl], s[{SRDS}:{SRDS + 3}], 0 offen lds"))
    return out


def advance_srds():
    """the three descriptors one tile on: base += step, num_records -= step (clamped at 0: rows past
    the end read as zeros)"""
    out = []
    for srd, step in ((SRDQ, "%[qstep]"), (SRDO, "%[ostep]"), (SRDS, "256")):
        out += [f"s_add_u32 s{srd}, s{srd}, {step}",
                f"s_addc_u32 s{srd + 1}, s{srd + 1}, 0",
                f"s_sub_u32 s{srd + 2}, s{srd + 2}, {step}",
                f"s_cselect_b32 s{srd + 2}, 0, s{srd + 2}"]
    return out


def addr_regs(which, sbase):
    """the LDS address registers of a buffer: RA + ST (A's tile), TC or TN (transposed reads)"""
    out = []
    if which == "A":
        for ks in range(4):
            out.append(f"v_add_u32 {v(RA[ks])}, {sbase}, %[vr{ks}]")
        out.append(f"v_add_u32 {v(ST)}, {sbase}, %[vs]")
    else:
        T = TC if which == "TC" else TN
        for k in range(4):
            out.append(f"v_add_u32 {v(T[k])}, {sbase}, %[vt{k}]")
    return out


# ---------------------------------------------------------------------------------------- emission
class Emitter:
    """instruction list + the in-order LDS reads still outstanding (tags), for counted waits"""
    def __init__(self):
        self.L = []
        self.pending = []

    def raw(self, text):
        self.L.append(text)

    def drain(self, text, keep=0):
        """a wait that leaves at most `keep` LDS reads outstanding (e.g. at a barrier)"""
        self.L.append(text)
        self.pending = self.pending[len(self.pending) - keep:] if keep else []

    def put(self, ins):
        if ins.needs and "nolds" not in VARIANT:
            last = -1
            for i, t in enumerate(self.pending):
                if t in ins.needs:
                    last = i
            if last >= 0:
                n = min(len(self.pending) - 1 - last, 15)
                self.L.append(f"s_waitcnt lgkmcnt({n})")
                self.pending = self.pending[len(self.pending) - n:] if n else []
        if ins.makes is not None:
            if "nolds" in VARIANT:
                return
            self.pending.append(ins.makes)
        self.L.append(ins.text)


STAMP_BODY = 10  # "stamps": the loop body (counted down from ntiles - 1) whose halves are stamped


def stamp(E, k):
    """s_memtime into s[60 + 2k : 61 + 2k] when the loop counter is STAMP_BODY (diagnostic only)"""
    if "stamps" not in VARIANT or "itemstamps" in VARIANT:
        return
    for t in (f"s_cmp_eq_u32 s{SITER}, {STAMP_BODY}", f"s_cbranch_scc0 L_st{k}_%=",
              f"s_memtime s[{60 + 2 * k}:{61 + 2 * k}]", f"L_st{k}_%=:"):
        E.raw(t)


def istamp(E, k):
    """"itemstamps" (diagnostic): s_memtime into s[60 + 2k : 61 + 2k] at an item-phase boundary of the
    persistent dK / dV body, every item (the last item's values are stored), retired at once so the
    generator's counted lgkmcnt waits stay exact"""
    if "itemstamps" in VARIANT:
        E.raw(f"s_memtime s[{60 + 2 * k}:{61 + 2 * k}]")
        E.raw("s_waitcnt lgkmcnt(0)")


def half(E, c, b_prev, b_cur, a_set, reads, dma=(), extra=None):
    """one 32-query half j: C(j-1) MFMAs in slots 0-15 if c, A(j+1) MFMAs (into a_set) in 16-31,
    the tail of B(j-1)'s stream (b_prev: its slots >= 32) and the head of B(j)'s (b_cur), the LDS
    reads `reads` ({slot: [I]}) and the DMA (M0, load) pairs"""
    cm = c_mfmas() if c else []
    am = a_mfmas(a_set) if a_set is not None else []
    if "novalu" in VARIANT:
        b_prev, b_cur = {}, {}
    dslot = {}
    for k, (m0, ld) in enumerate(dma):  # M0 one slot ahead of its load
        q = 2 + 6 * k
        dslot.setdefault(q - 1, []).append(m0)
        dslot.setdefault(q, []).append(ld)
    for k in range(32):
        if k < 16 and cm:
            E.put(cm[k])
        if k >= 16 and am:
            E.put(am[k - 16])
        valu = b_prev.get(k + 32, []) + b_cur.get(k, [])
        if "expfirst" in VARIANT:  # timing variant: the exponential first among the VALU fillers
            valu = [x for x in valu if "v_exp" in x.text] + [x for x in valu if "v_exp" not in x.text]
        rd = reads.get(k, [])
        dm = dslot.get(k, []) + (extra.get(k, []) if extra else [])
        # the gap opens with its LDS read (and LDS-DMA piece): placed after the VALU fillers the same
        # reads cost ~8 cycles more per gap (stamps: 1472 vs 1216 cycles per half)
        if "dmalast" in VARIANT:
            for ins in rd:
                E.put(ins)
            for ins in valu:
                E.put(ins)
            for t in dm:
                E.raw(t)
        else:
            for t in dm:
                E.raw(t)
            for ins in rd + valu:
                E.put(ins)


def read_plan(a_u, tr_T, tr_u, lse_u, lse_buf):
    """slot -> reads: A's operands (half a_u of the tile at RA / ST) in slots 0-11, C's k-step-0
    transposed fragments (half tr_u of the tile at tr_T) in 12-19, the next half's lse (lse_u) into
    lse_buf in 20-23, C's k-step-1 fragments in 24-31 (each set after the previous C stage's last
    read of those registers)"""
    plan = {}

    def lay(ins, first):
        for i, x in enumerate(ins):
            plan.setdefault(first + i, []).append(x)
    if a_u is not None:
        lay(a_reads(a_u), 0)
    if tr_T is not None:
        lay(tr_reads(tr_T, tr_u, 0), 12)
        lay(tr_reads(tr_T, tr_u, 1), 24)
    if lse_u is not None:
        lay(lse_reads(lse_u, lse_buf), 20)
    return plan


def body():
    E = Emitter()
    a = E.raw
    a("s_nop 4")  # SGPR operands fresh from v_readfirstlane -> descriptors / M0
    a(f"s_mov_b32 s{SKEEP}, m0")
    for srd, nm in ((SRDQ, "sq"), (SRDO, "so"), (SRDS, "ss")):  # descriptors as two 64-bit halves each
        a(f"s_mov_b64 s[{srd}:{srd + 1}], %[{nm}0]")
        a(f"s_mov_b64 s[{srd + 2}:{srd + 3}], %[{nm}1]")
    # ---- prologue: K, V fragments; tiles 0 and 1; A(0); half 0 (B(0) head, A(1)) ------------------
    for kt in range(2):
        for ks in range(4):
            a(f"global_load_dwordx4 {a_(KF(kt, ks), 4)}, %[kp{kt}], off offset:{ks * 32}")
    for kt in range(2):
        for ks in range(4):
            a(f"global_load_dwordx4 {v(16 * kt + 4 * ks, 4)}, %[vp{kt}], off offset:{ks * 32}")
    a(f"s_mov_b32 s{SB0}, %[lds0]")
    a(f"s_add_u32 s{SB1}, %[lds0], {W_BUF}")
    a(f"s_add_u32 s{SBD}, %[lds0], {2 * W_BUF}")
    for buf in (SB0, SB1):  # tiles 0 and 1 into buffers 0, 1
        a(f"s_add_u32 s{STMP}, s{buf}, %[wq]")
        for m0, ld in dma_pieces(buf):
            a(m0)
            a("s_nop 0")
            a(ld)
        for t in advance_srds():
            a(t)
    a("s_waitcnt vmcnt(5)")  # K, V and tile 0 landed (tile 1's five pieces may fly)
    for r in range(32):  # -V (sign flip, exact) into the accumulator file
        a(f"v_xor_b32 {v(r)}, 0x80008000, {v(r)}")
    for r in range(32):
        a(f"v_accvgpr_write_b32 {a_(160 + r)}, {v(r)}")
    a("s_barrier")
    for t in addr_regs("A", f"s{SB0}") + addr_regs("TN", f"s{SB0}"):
        a(t)
    # A(0) into set 0 (tile 0, half 0) and B(0)'s lse
    for ins in a_reads(0) + lse_reads(0, LSEB[0]):
        E.put(ins)
    a("s_nop 1")  # accvgpr writes of -V -> MFMA operand
    for ins in a_mfmas(0):
        E.put(ins)
    a("s_nop 7")
    a("s_nop 7")
    a("s_nop 3")  # the last A MFMAs' results -> B(0)'s first v_fma (no MFMA in between)
    # half 0: B(0) head (set 0, even lse), A(1) into set 1 (tile 0 half 1); reads: A(1)'s operands,
    # C(0)'s fragments (tile 0 half 0 at TN), B(1)'s lse (tile 0 half 1) into the odd tuple
    b_even, b_odd = b_stream(0, LSEB[0]), b_stream(1, LSEB[1])
    half(E, False, {}, b_even, 1, read_plan(1, TN, 0, 1, LSEB[1]))
    # ---- steady state: tile t = 0 .. ntiles - 2 ----------------------------------------------------
    # every body opens by rotating (B0, B1, BD) <- (B1, BD, B0); the prologue left B0 = buffer 0,
    # B1 = buffer 1, BD = buffer 2, so pre-rotate backwards to (buffer 2, buffer 0, buffer 1)
    a(f"s_mov_b32 s{STMP}, s{SBD}")
    a(f"s_mov_b32 s{SBD}, s{SB1}")
    a(f"s_mov_b32 s{SB1}, s{SB0}")
    a(f"s_mov_b32 s{SB0}, s{STMP}")
    a(f"s_mov_b32 s{SITER}, %[iters]")
    if "stamps" in VARIANT:
        a("s_memtime s[72:73]")
    a(f"s_cmp_eq_u32 s{SITER}, 0")
    a("s_cbranch_scc1 L_dkdv_tail_%=")
    a("L_dkdv_loop_%=:")
    stamp(E, 0)
    # tile t+1 (DMA issued one tile ago) landed in every wave and every wave's reads of tile t-1 (the
    # buffer the DMA below overwrites) are done: those ended a half ago, so only the previous half's
    # last 15 reads (all of tile t, at most 15 in flight) may stay outstanding
    E.drain("s_waitcnt vmcnt(0) lgkmcnt(15)", keep=15)
    a("s_barrier")
    stamp(E, 1)
    a(f"s_mov_b32 s{STMP}, s{SB0}")
    a(f"s_mov_b32 s{SB0}, s{SB1}")
    a(f"s_mov_b32 s{SB1}, s{SBD}")
    a(f"s_mov_b32 s{SBD}, s{STMP}")
    for t in addr_regs("A", f"s{SB1}"):  # A's reads start in slot 0; TC / TN are added in slots 1-8
        a(t)
    a(f"s_add_u32 s{STMP}, s{SBD}, %[wq]")
    later = {1 + i: [t] for i, t in enumerate(addr_regs("TC", f"s{SB0}") + addr_regs("TN", f"s{SB1}"))}
    # half 2t+1: C(2t), B(2t) tail, B(2t+1) head (set 1, odd lse), A(2t+2) into set 0 (tile t+1 half
    # 0); reads: A(2t+2)'s operands, C(2t+1)'s fragments (tile t half 1 at TC), B(2t+2)'s lse (tile
    # t+1 half 0, even tuple); the DMA of tile t+2 into BD
    half(E, True, b_even, b_odd, 0, read_plan(0, TC, 1, 0, LSEB[0]), dma_pieces(SBD), extra=later)
    stamp(E, 2)
    for t in advance_srds():
        a(t)
    # half 2t+2: C(2t+1), B(2t+1) tail, B(2t+2) head (set 0, even lse), A(2t+3) into set 1 (tile
    # t+1 half 1); reads: A(2t+3)'s operands, C(2t+2)'s fragments (tile t+1 half 0 at TN), B(2t+3)'s
    # lse (tile t+1 half 1, odd tuple)
    half(E, True, b_odd, b_even, 1, read_plan(1, TN, 0, 1, LSEB[1]))
    stamp(E, 3)
    a(f"s_sub_u32 s{SITER}, s{SITER}, 1")
    a(f"s_cmp_eq_u32 s{SITER}, 0")
    a("s_cbranch_scc0 L_dkdv_loop_%=")
    a("L_dkdv_tail_%=:")
    if "stamps" in VARIANT:
        a("s_memtime s[74:75]")
    # the reads in flight at the loop exit are those at the end of a loop body, and the prologue's
    # half 0 leaves the same kinds in the same order (an odd half's A operands, C's fragments, the
    # odd lse tuple), so the counted waits below hold on both paths
    # ---- last tile T-1: half J-1 = C(J-2), B(J-2) tail, B(J-1) head (set 1), reads C(J-1)'s
    # fragments (tile T-1 half 1 at TN); then half J: C(J-1) and B(J-1)'s tail --------------------
    half(E, True, b_even, b_odd, None, read_plan(None, TN, 1, None, None))
    half(E, True, b_odd, {}, None, {})
    if "stamps" in VARIANT:  # every lane of the wave stores the same 8 stamps to %[stp]
        E.drain("s_waitcnt lgkmcnt(0)")
        for k in range(8):
            a(f"v_mov_b32 v0, s{60 + 2 * k}")
            a(f"v_mov_b32 v1, s{61 + 2 * k}")
            a(f"global_store_dwordx2 %[stp], v[0:1], off offset:{8 * k}")
            a("s_nop 1")
    a("s_waitcnt vmcnt(0)")  # no DMA may land in the ring after the statement (epilogue staging)
    a(f"s_mov_b32 m0, s{SKEEP}")
    a("s_nop 15")
    a("s_nop 15")  # the last MFMAs' accumulators -> the compiler's reads after the statement
    return E.L


def clobbers(diag):
    regs = [f'"v{r}"' for r in range(VLAST + 1)] + [f'"a{r}"' for r in range(128, 256)] + \
           [f'"s{r}"' for r in range(80, 98)]
    if diag:
        regs += [f'"s{r}"' for r in range(60, 76)]
    return ", ".join(regs)

# =============================================================================================
# Persistent dK / dV (attn_dkdv_w1p_kernel): one workgroup per CU walks its key blocks ("items") in ONE
# asm statement. Per item: the body of attn_dkdv_w1_kernel (A(0), half 0, the tile loop, the two tail
# halves), then the dK / dV stores from the accumulators (a[0:127], fixed: ACC_REG) through a wave-
# private LDS staging area. Every load an item starts with is issued while the previous item runs:
#   * its K / V rows go by LDS-DMA into a dedicated region (each wave its own 64 keys) right after the
#     previous item has read its own fragments out of it -- a whole item (~50 us) ahead;
#   * its first two Q / dO tiles go into the two ring buffers the previous item's tail no longer
#     reads (tile T-2's and the past-the-end one) before that tail's two halves and the stores.
# The non-persistent kernel waits ~10k of its ~89k cycles per workgroup on these loads (stamps), and
# 1792 short-lived workgroups add round-to-round skew.
# Item parameters come from a table the kernel writes into LDS before the statement: one 96-B row per
# item (K / V descriptors, Q / dO / lse / delta bases, dK / dV descriptors) plus a null row (empty
# K / V descriptors: the last item's K / V prefetch writes zeros nobody reads).
# =============================================================================================
P_KV = NBUF * W_BUF                  # K / V prefetch region: [256 keys][128 B] K, then V
P_STG = P_KV + 2 * 32768             # staging: 4 waves x 8 KiB (dK | dV of one key tile)
P_TAB = P_STG + 4 * 8192             # the item table
ITEM_B = 96
SK, SV, SDK, SDV = 40, 44, 48, 52    # next item's K / V descriptors (then its Q / dO / lse / delta
#                                      bases), this item's dK / dV descriptors
SITEM = 39                           # items left
TABV = 226                           # LDS address of the current item's table row (uniform)
PRM = 66                             # v[66:89]: table reads (free at an item's start)
P_VLAST = 226


def p_kv_dma():
    """the next item's K / V rows of this wave (keys 64 w .. 64 w + 63, 8 pieces each) into the K / V
    region: piece i = rows 8 i + (lane >> 3), chunk swizzled as the ring tiles (vkd / vvd: even / odd
    pieces' lane offsets, rows stepped by soffset)"""
    out = []
    for which, srd, vo, s8, reg in (("k", SK, "%[vkd", "%[s8k]", 0), ("v", SV, "%[vvd", "%[s8v]", 32768)):
        for i in range(8):
            out += [f"s_mul_i32 s{STMP}, {s8}, {i}",
                    f"s_add_u32 m0, %[kvw], {reg + 1024 * i}",
                    "s_nop 0",
                    f"buffer_load_dwordx4 {vo}{i & 1}], s[{srd}:{srd + 3}], s{STMP} offen lds"]
    return out


def p_tile_dma(buf, tile):
    """the next item's Q / dO tile (0 or 1) into ring buffer `buf` (descriptors advanced past it)"""
    out = [f"s_add_u32 s{STMP}, s{buf}, %[wq]"]
    for m0, ld in dma_pieces(buf):
        out += [m0, "s_nop 0", ld]
    return out + advance_srds()


def p_epilogue(E):
    """dK (x scale) / dV of the item from the accumulators, one key tile per pass: bf16 rows through
    this wave's staging area (16-B chunks XOR row & 7, as store_rows_lds), then buffer stores clipped
    to the block's valid keys"""
    a = E.raw
    a("s_nop 15")
    a("s_nop 15")  # the last C MFMAs -> accvgpr reads
    # x = row & 7 (WX), this lane's write base in the wave's staging area (WB); the swizzled write
    # addresses rotate over v[198:205], the data over v[162:177]
    WX, WB = 194, 195
    a(f"v_bfe_u32 {v(WX)}, %[vwd], 7, 3")
    a(f"v_add_u32 {v(WB)}, %[stg], %[vwd]")
    for kt in range(2):
        for ti, kind in enumerate(("dk", "dv")):
            stage = ti * 4096
            for d in range(2):
                base = ACC_REG(kind, kt, d)
                for r in range(16):
                    a(f"v_accvgpr_read_b32 {v(130 + 16 * d + r)}, {a_(base + r)}")
            if kind == "dk":
                for r in range(32):
                    a(f"v_mul_f32 {v(130 + r)}, %[scale], {v(130 + r)}")
            for d in range(2):
                for g in range(4):
                    src = 130 + 16 * d + 4 * g
                    c = 4 * d + g
                    wd, wt = 162 + 2 * c, 198 + c
                    a(f"v_cvt_pk_bf16_f32 {v(wd)}, {v(src)}, {v(src + 1)}")
                    a(f"v_cvt_pk_bf16_f32 {v(wd + 1)}, {v(src + 2)}, {v(src + 3)}")
                    a(f"v_xor_b32 {v(wt)}, {c}, {v(WX)}")
                    a(f"v_lshl_add_u32 {v(wt)}, {v(wt)}, 4, {v(WB)}")
                    a(f"ds_write_b64 {v(wt)}, {v(wd, 2)} offset:{stage}")
        a("s_waitcnt lgkmcnt(0)")
        for ti in range(2):
            for i in range(4):
                a(f"ds_read_b128 {v(32 + 16 * ti + 4 * i, 4)}, %[vrd] offset:{ti * 4096 + 1024 * i}")
        a("s_waitcnt lgkmcnt(0)")
        for ti, (srd, vo, s8) in enumerate(((SDK, "%[vdk]", "%[s8dk]"), (SDV, "%[vdv]", "%[s8dv]"))):
            for i in range(4):
                a(f"s_mul_i32 s{STMP}, {s8}, {4 * kt + i}")
                a(f"buffer_store_dwordx4 {v(32 + 16 * ti + 4 * i, 4)}, {vo}, s[{srd}:{srd + 3}], s{STMP} offen")


def zero_acc_mfma(n, z=130):
    """zero n accumulator tiles a[16 i : 16 i + 15] with one 0 x 0 + 0 MFMA each (v[z : z + 3] = 0): the
    idle matrix core does what 16 n v_accvgpr_write would cost the wave's issue (+0.0, as those)"""
    out = [f"v_mov_b32 {v(z + i)}, 0" for i in range(4)] + ["s_nop 2"]
    return out + [f"v_mfma_f32_32x32x16_bf16 {a_(16 * i, 16)}, {v(z, 4)}, {v(z, 4)}, 0" for i in range(n)]


def dkdv_p_body():
    HARD_ACC[0] = True
    try:
        return _dkdv_p_body()
    finally:
        HARD_ACC[0] = False


def _dkdv_p_body():
    E = Emitter()
    a = E.raw

    def rfl(dst, src):
        a(f"v_readfirstlane_b32 s{dst}, {v(src)}")

    a("s_nop 4")
    a(f"s_mov_b32 s{SKEEP}, m0")
    a(f"v_mov_b32 {v(TABV)}, %[tab]")
    a(f"s_mov_b32 s{SITEM}, %[nitems]")
    # ---- item 0: its K / V rows, its tiles 0 and 1 -------------------------------------------------
    for i in range(4):
        a(f"ds_read_b128 {v(PRM + 4 * i, 4)}, {v(TABV)} offset:{16 * i}")
    a("s_waitcnt lgkmcnt(0)")
    for i in range(4):
        rfl(SK + i, PRM + i)
        rfl(SV + i, PRM + 4 + i)
    for srd, w in ((SRDQ, 8), (SRDO, 10)):
        rfl(srd, PRM + w)
        rfl(srd + 1, PRM + w + 1)
    rfl(SDK, PRM + 12)      # lse / delta bases (scratch: SDK is set at the item start)
    rfl(SDK + 1, PRM + 13)
    rfl(SDK + 2, PRM + 14)
    rfl(SDK + 3, PRM + 15)
    a(f"s_mov_b32 s{SRDQ + 2}, %[sq2]")
    a(f"s_mov_b32 s{SRDQ + 3}, 0x20000")
    a(f"s_mov_b32 s{SRDO + 2}, %[so2]")
    a(f"s_mov_b32 s{SRDO + 3}, 0x20000")
    a(f"s_mov_b32 s{SRDS + 2}, %[ss2]")
    a(f"s_mov_b32 s{SRDS + 3}, 0x20000")
    a("s_cmp_eq_u32 %[wodd], 0")
    a(f"s_cselect_b64 s[{SRDS}:{SRDS + 1}], s[{SDK}:{SDK + 1}], s[{SDK + 2}:{SDK + 3}]")
    a("s_nop 4")  # SGPRs fresh from v_readfirstlane -> descriptors / M0
    for t in p_kv_dma():
        a(t)
    a(f"s_mov_b32 s{SB0}, %[lds0]")
    a(f"s_add_u32 s{SB1}, %[lds0], {W_BUF}")
    a(f"s_add_u32 s{SBD}, %[lds0], {2 * W_BUF}")
    for t in p_tile_dma(SB0, 0) + p_tile_dma(SB1, 1):
        a(t)
    a("s_waitcnt vmcnt(0)")
    a("s_branch L_p_item_%=")
    a("L_p_next_%=:")
    istamp(E, 0)
    # outstanding: the previous item's dK / dV stores (16) -- its K / V region fill (issued an item
    # ago) and this item's tiles 0, 1 (issued at the previous tail) are older
    a("s_waitcnt vmcnt(16)")
    a("L_p_item_%=:")
    a("s_barrier")  # tiles 0, 1 complete in every wave
    istamp(E, 1)
    # ---- this item's K / V fragments from the region (the wave's own rows), its dK / dV
    # descriptors, the next item's K / V descriptors and Q / dO / lse / delta bases --------------------
    for ks in range(4):
        a(f"v_add_u32 {v(RA[ks])}, %[kvw], %[vr{ks}]")
    for kt in range(2):
        for ks in range(4):
            a(f"ds_read_b128 {a_(KF(kt, ks), 4)}, {v(RA[ks])} offset:{kt * 4096}")
            a(f"ds_read_b128 {v(16 * kt + 4 * ks, 4)}, {v(RA[ks])} offset:{32768 + kt * 4096}")
    for i in range(2):
        a(f"ds_read_b128 {v(PRM + 4 * i, 4)}, {v(TABV)} offset:{64 + 16 * i}")
    for i in range(4):
        a(f"ds_read_b128 {v(PRM + 8 + 4 * i, 4)}, {v(TABV)} offset:{ITEM_B + 16 * i}")
    a("s_waitcnt lgkmcnt(0)")
    for t in zero_acc_mfma(8):  # dV / dK accumulators a[0:127] (read out by the previous epilogue)
        a(t)
    a("s_nop 4")  # the previous item's stores read SDK / SDV at issue: rewrite after
    for i in range(4):
        rfl(SDK + i, PRM + i)
        rfl(SDV + i, PRM + 4 + i)
        rfl(SK + i, PRM + 8 + i)
        rfl(SV + i, PRM + 12 + i)
    a("s_nop 4")
    for t in p_kv_dma():  # the next item's K / V rows (the null row's empty descriptors: zeros)
        a(t)
    a("s_nop 4")  # the DMA's descriptor reads before SK / SV take the next item's bases
    for i in range(8):
        rfl(SK + i, PRM + 16 + i)   # SK: Q base, dO base; SV: lse base, delta base
    for r in range(32):  # -V (sign flip, exact) into the accumulator file
        a(f"v_xor_b32 {v(r)}, 0x80008000, {v(r)}")
    for r in range(32):
        a(f"v_accvgpr_write_b32 {a_(160 + r)}, {v(r)}")
    for t in addr_regs("A", f"s{SB0}") + addr_regs("TN", f"s{SB0}"):
        a(t)
    istamp(E, 2)
    for ins in a_reads(0) + lse_reads(0, LSEB[0]):
        E.put(ins)
    a("s_nop 1")
    for ins in a_mfmas(0):
        E.put(ins)
    a("s_nop 7")
    a("s_nop 7")
    a("s_nop 3")
    istamp(E, 3)
    b_even, b_odd = b_stream(0, LSEB[0]), b_stream(1, LSEB[1])
    half(E, False, {}, b_even, 1, read_plan(1, TN, 0, 1, LSEB[1]))
    a(f"s_mov_b32 s{STMP}, s{SBD}")
    a(f"s_mov_b32 s{SBD}, s{SB1}")
    a(f"s_mov_b32 s{SB1}, s{SB0}")
    a(f"s_mov_b32 s{SB0}, s{STMP}")
    a(f"s_mov_b32 s{SITER}, %[iters]")
    if "stamps" in VARIANT:
        a("s_memtime s[72:73]")
        if "itemstamps" in VARIANT:
            a("s_waitcnt lgkmcnt(0)")
    a(f"s_cmp_eq_u32 s{SITER}, 0")
    a("s_cbranch_scc1 L_p_tail_%=")
    a("L_p_loop_%=:")
    stamp(E, 0)
    E.drain("s_waitcnt vmcnt(0) lgkmcnt(15)", keep=15)
    a("s_barrier")
    stamp(E, 1)
    a(f"s_mov_b32 s{STMP}, s{SB0}")
    a(f"s_mov_b32 s{SB0}, s{SB1}")
    a(f"s_mov_b32 s{SB1}, s{SBD}")
    a(f"s_mov_b32 s{SBD}, s{STMP}")
    for t in addr_regs("A", f"s{SB1}"):
        a(t)
    a(f"s_add_u32 s{STMP}, s{SBD}, %[wq]")
    later = {1 + i: [t] for i, t in enumerate(addr_regs("TC", f"s{SB0}") + addr_regs("TN", f"s{SB1}"))}
    half(E, True, b_even, b_odd, 0, read_plan(0, TC, 1, 0, LSEB[0]), dma_pieces(SBD), extra=later)
    stamp(E, 2)
    for t in advance_srds():
        a(t)
    half(E, True, b_odd, b_even, 1, read_plan(1, TN, 0, 1, LSEB[1]))
    stamp(E, 3)
    a(f"s_sub_u32 s{SITER}, s{SITER}, 1")
    a(f"s_cmp_eq_u32 s{SITER}, 0")
    a("s_cbranch_scc0 L_p_loop_%=")
    a("L_p_tail_%=:")
    if "stamps" in VARIANT:
        a("s_memtime s[74:75]")
        if "itemstamps" in VARIANT:
            a("s_waitcnt lgkmcnt(0)")
    # ---- tail start: the next item's tiles 0, 1 into SBD (the past-the-end DMA's buffer) and SB0
    # (tile T-2: every wave past it after the barrier); the tail itself reads only SB1 -------------------
    a("s_waitcnt vmcnt(0)")  # this wave's past-the-end tile DMA into SBD landed
    E.drain("s_waitcnt lgkmcnt(15)", keep=15)
    a("s_barrier")
    a(f"s_cmp_eq_u32 s{SITEM}, 1")
    a("s_cbranch_scc1 L_p_nodma_%=")
    for srd, w in ((SRDQ, SK), (SRDO, SK + 2)):
        a(f"s_mov_b64 s[{srd}:{srd + 1}], s[{w}:{w + 1}]")
    a(f"s_mov_b32 s{SRDQ + 2}, %[sq2]")
    a(f"s_mov_b32 s{SRDO + 2}, %[so2]")
    a(f"s_mov_b32 s{SRDS + 2}, %[ss2]")
    a("s_cmp_eq_u32 %[wodd], 0")
    a(f"s_cselect_b64 s[{SRDS}:{SRDS + 1}], s[{SV}:{SV + 1}], s[{SV + 2}:{SV + 3}]")
    for t in p_tile_dma(SBD, 0) + p_tile_dma(SB0, 1):
        a(t)
    a("L_p_nodma_%=:")
    half(E, True, b_even, b_odd, None, read_plan(None, TN, 1, None, None))
    half(E, True, b_odd, {}, None, {})
    E.drain("s_waitcnt lgkmcnt(0)")
    istamp(E, 4)
    p_epilogue(E)
    istamp(E, 5)
    a(f"s_cmp_eq_u32 s{SITEM}, 1")
    a("s_cbranch_scc1 L_p_done_%=")
    # the next item's ring: tile 0 in SBD, tile 1 in SB0, SB1 (tile T-1) free
    a(f"s_mov_b32 s{STMP}, s{SB0}")
    a(f"s_mov_b32 s{SB0}, s{SBD}")
    a(f"s_mov_b32 s{SBD}, s{SB1}")
    a(f"s_mov_b32 s{SB1}, s{STMP}")
    a(f"v_add_u32 {v(TABV)}, {ITEM_B}, {v(TABV)}")
    a(f"s_sub_u32 s{SITEM}, s{SITEM}, 1")
    a("s_branch L_p_next_%=")
    a("L_p_done_%=:")
    if "stamps" in VARIANT:
        for k in range(8):
            a(f"v_mov_b32 v0, s{60 + 2 * k}")
            a(f"v_mov_b32 v1, s{61 + 2 * k}")
            a(f"global_store_dwordx2 %[stp], v[0:1], off offset:{8 * k}")
            a("s_nop 1")
    a("s_waitcnt vmcnt(0)")
    a(f"s_mov_b32 m0, s{SKEEP}")
    return E.L


def p_clobbers(diag):
    regs = [f'"v{r}"' for r in range(P_VLAST + 1)] + [f'"a{r}"' for r in range(256)] + \
           [f'"s{r}"' for r in list(range(39, 60)) + list(range(80, 98))]
    if diag:
        regs += [f'"s{r}"' for r in range(60, 76)]
    return ", ".join(regs)


# =============================================================================================
# dQ at one wave per SIMD (attn_dq_w1_kernel): 4 waves x 64 queries (two 32-query tiles qt per
# wave), keys in tiles of 64 through the same 3-buffer LDS-DMA ring (K | V), per 32-key half j:
#   A(j+1): S[qt] = K.Q^T, dP'[qt] = V.dO^T - delta (16 MFMAs; the K / V row fragments feed both qt);
#   B(j):   dS = exp2(S c2 - lse) dP' -> bf16 packs (32 elements streamed over the half's 24 slots);
#   C(j-1): dQ^T[qt][d] += K^T[ss][d] . dS[qt][ss] (8 MFMAs, the K^T fragments shared by both qt).
# A half is 24 slots: C(j-1) in slots 0-7, A(j+1) in 8-23; B(j) runs from slot 1 of its half to slot
# 4 of the next (element e in slot 3e/4 + 2). Arithmetic and accumulation order of
# attn_dq_pipe_kernel (lse, delta per lane, -delta as dP's initial accumulator): bitwise equal to it.
# Keys past Nk read as zeros (shrinking descriptors): their dS is -P delta, but their K rows are 0,
# so they add exactly 0 to dQ = dS.K.
# Registers: v[0:63] S tiles (32 s + 16 qt), v[66:129] dP' tiles, v[130:145] dS packs
# SBF[qt][ss], v[146:177] -delta tuples NDL[qt], v[178:189] LDS addresses RK[ks], TC / TN;
# a[128:159] Q fragments QF[qt][ks], a[160:191] dO fragments, a[192:223] K / V row fragments
# KA / VA[ks], a[224:239] K^T fragments KT[ss][d]; the dQ accumulators are operands %0..%3
# (acc[qt][d] at 2 qt + d, hipcc places them in a0..a127).
# =============================================================================================
D_TILE = 8192
D_BUF = 2 * D_TILE       # K | V
D_LAG = 2


def DSD(s, T):           # T: 0 S qt0, 1 dP qt0, 2 S qt1, 3 dP qt1
    qt = T // 2
    return 32 * s + 16 * qt + (66 if T % 2 else 0)


DSBF = lambda qt, ss: 130 + 8 * qt + 4 * ss
DNDL = lambda qt: 146 + 16 * qt
DRK = [178, 179, 180, 181]
DTC = [182, 183, 184, 185]
DTN = [186, 187, 188, 189]
DVLAST = 189
DQF = lambda qt, ks: 128 + 16 * qt + 4 * ks
DOF = lambda qt, ks: 160 + 16 * qt + 4 * ks
DKA = lambda ks: 192 + 4 * ks
DVA = lambda ks: 208 + 4 * ks
DKT = lambda ss, d: 224 + 4 * (2 * ss + d)
SRDK, SRDV = 80, 84


def dq_c_mfmas():
    """C(j-1) in pack order (ss, qt, d): each accumulator takes ss = 0 then ss = 1"""
    out = []
    for ss in range(2):
        for qt in range(2):
            for d in range(2):
                acc = a_(16 * (2 * qt + d), 16) if HARD_ACC[0] else "%" + str(2 * qt + d)
                out.append(mfma(acc, a_(DKT(ss, d), 4), v(DSBF(qt, ss), 4), acc, needs=[f"KT{ss}{d}"]))
    return out


def dq_a_mfmas(s):
    """A(j+1) into set s, the chains S qt0, S qt1, dP' qt0, dP' qt1 interleaved k-step by k-step"""
    out = []
    for ks in range(4):
        for T in (0, 1):
            for qt in range(2):
                dst = v(DSD(s, 2 * qt + T), 16)
                if T == 0:
                    out.append(mfma(dst, a_(DKA(ks), 4), a_(DQF(qt, ks), 4), "0" if ks == 0 else dst,
                                    needs=[f"KA{ks}"]))
                else:
                    out.append(mfma(dst, a_(DVA(ks), 4), a_(DOF(qt, ks), 4), v(DNDL(qt), 16) if ks == 0 else dst,
                                    needs=[f"VA{ks}"]))
    return out


def dq_b_stream(s):
    """B(j) on set s: {slot (relative to half j): [I]}, element e (pack order ss, qt, row) in slot
    3e/4 + D_LAG (its exponent argument one slot earlier, its product two later, pair packs three)"""
    out = {}

    def put(k, ins):
        out.setdefault(k, []).append(ins)
    for e in range(32):
        ss, qt, i = e // 16, (e % 16) // 8, e % 8
        r = 8 * ss + i
        sr, dr = DSD(s, 2 * qt) + r, DSD(s, 2 * qt + 1) + r
        k = (3 * e) // 4 + D_LAG
        nl = v(DNLR + qt) if HARD_ACC[0] else f"%[nl{qt}]"
        put(k - 1, I(f"v_fma_f32 {v(sr)}, {v(sr)}, %[c2], {nl}"))
        put(k, I(f"v_exp_f32 {v(sr)}, {v(sr)}"))
        put(k + 2, I(f"v_mul_f32 {v(dr)}, {v(sr)}, {v(dr)}"))
        if e % 2 == 1:
            put(k + 3, I(f"v_cvt_pk_bf16_f32 {v(DSBF(qt, ss) + i // 2)}, {v(dr - 1)}, {v(dr)}"))
    return out


def dq_a_reads(u):
    out = [I(f"ds_read_b128 {a_(DKA(ks), 4)}, {v(DRK[ks])} offset:{u * 4096}", makes=f"KA{ks}") for ks in range(4)]
    out += [I(f"ds_read_b128 {a_(DVA(ks), 4)}, {v(DRK[ks])} offset:{D_TILE + u * 4096}", makes=f"VA{ks}")
            for ks in range(4)]
    return out


def dq_tr_reads(T, u):
    out = []
    for ss in range(2):
        for d in range(2):
            base = (u * 32 + 16 * ss) * 128
            tag = f"KT{ss}{d}"
            out.append(I(f"ds_read_b64_tr_b16 {a_(DKT(ss, d), 2)}, {v(T[2 * d])} offset:{base}", makes=tag))
            out.append(I(f"ds_read_b64_tr_b16 {a_(DKT(ss, d) + 2, 2)}, {v(T[2 * d + 1])} offset:{base}", makes=tag))
    return out


def dq_dma(buf):
    out = []
    for i in range(2):
        out.append((f"s_add_u32 m0, s{STMP}, {i * 1024}",
                    f"buffer_load_dwordx4 %[vk{i}], s[{SRDK}:{SRDK + 3}], 0 offen lds"))
        out.append((f"s_add_u32 m0, s{STMP}, {D_TILE + i * 1024}",
                    f"buffer_load_dwordx4 %[vv{i}], s[{SRDV}:{SRDV + 3}], 0 offen lds"))
    return out


def dq_advance():
    out = []
    for srd, step in ((SRDK, "%[kstep]"), (SRDV, "%[vstep]")):
        out += [f"s_add_u32 s{srd}, s{srd}, {step}",
                f"s_addc_u32 s{srd + 1}, s{srd + 1}, 0",
                f"s_sub_u32 s{srd + 2}, s{srd + 2}, {step}",
                f"s_cselect_b32 s{srd + 2}, 0, s{srd + 2}"]
    return out


def dq_addr(which, sbase):
    T = {"A": DRK, "TC": DTC, "TN": DTN}[which]
    src = [f"%[vr{k}]" for k in range(4)] if which == "A" else [f"%[vt{k}]" for k in range(4)]
    return [f"v_add_u32 {v(T[k])}, {sbase}, {src[k]}" for k in range(4)]


def dq_half(E, c, b_prev, b_cur, a_set, a_u, tr, dma=(), extra=None, more=None):
    """one 32-key half j (24 slots): C(j-1) in slots 0-7 if c, A(j+1) (set a_set, half a_u of the
    tile at RK) in 8-23; B(j-1)'s tail and B(j)'s head; A's reads in slots 0-7, the next C's K^T
    fragments (tr = (address regs, half)) in 10-17; DMA pieces and `extra` raw lines"""
    cm = dq_c_mfmas() if c else []
    am = dq_a_mfmas(a_set) if a_set is not None else []
    if "novalu" in VARIANT:
        b_prev, b_cur = {}, {}
    reads = {}
    if a_set is not None:
        for i, x in enumerate(dq_a_reads(a_u)):
            reads.setdefault(i, []).append(x)
    if tr is not None:
        for i, x in enumerate(dq_tr_reads(*tr)):
            reads.setdefault(10 + i, []).append(x)
    for k, ins in (more or {}).items():
        reads.setdefault(k, []).extend(ins)
    dslot = {}
    for k, (m0, ld) in enumerate(dma):
        q = 2 + 5 * k
        dslot.setdefault(q - 1, []).append(m0)
        dslot.setdefault(q, []).append(ld)
    for k in range(24):
        if k < 8 and cm:
            E.put(cm[k])
        if k >= 8 and am:
            E.put(am[k - 8])
        for t in dslot.get(k, []) + (extra.get(k, []) if extra else []):
            E.raw(t)
        for ins in reads.get(k, []) + b_prev.get(k + 24, []) + b_cur.get(k, []):
            E.put(ins)


def dq_body():
    E = Emitter()
    a = E.raw
    a("s_nop 4")
    a(f"s_mov_b32 s{SKEEP}, m0")
    for srd, nm in ((SRDK, "sk"), (SRDV, "sv")):
        a(f"s_mov_b64 s[{srd}:{srd + 1}], %[{nm}0]")
        a(f"s_mov_b64 s[{srd + 2}:{srd + 3}], %[{nm}1]")
    for qt in range(2):  # the lane's Q and dO fragments (B operands of S and dP) into AGPRs
        for ks in range(4):
            a(f"global_load_dwordx4 {a_(DQF(qt, ks), 4)}, %[qp{qt}], off offset:{ks * 32}")
            a(f"global_load_dwordx4 {a_(DOF(qt, ks), 4)}, %[op{qt}], off offset:{ks * 32}")
    for qt in range(2):  # -delta in every register of the dP chains' initial accumulator
        for r in range(16):
            a(f"v_mov_b32 {v(DNDL(qt) + r)}, %[nd{qt}]")
    a(f"s_mov_b32 s{SB0}, %[lds0]")
    a(f"s_add_u32 s{SB1}, %[lds0], {D_BUF}")
    a(f"s_add_u32 s{SBD}, %[lds0], {2 * D_BUF}")
    for buf in (SB0, SB1):  # key tiles 0 and 1
        a(f"s_add_u32 s{STMP}, s{buf}, %[wq]")
        for m0, ld in dq_dma(buf):
            a(m0)
            a("s_nop 0")
            a(ld)
        for t in dq_advance():
            a(t)
    a("s_waitcnt vmcnt(4)")  # Q, dO fragments and key tile 0 landed
    a("s_barrier")
    for t in dq_addr("A", f"s{SB0}") + dq_addr("TN", f"s{SB0}"):
        a(t)
    for ins in dq_a_reads(0):
        E.put(ins)
    a("s_nop 1")
    for ins in dq_a_mfmas(0):
        E.put(ins)
    a("s_nop 7")
    a("s_nop 7")
    a("s_nop 3")
    b_even, b_odd = dq_b_stream(0), dq_b_stream(1)
    dq_half(E, False, {}, b_even, 1, 1, (DTN, 0))
    a(f"s_mov_b32 s{STMP}, s{SBD}")
    a(f"s_mov_b32 s{SBD}, s{SB1}")
    a(f"s_mov_b32 s{SB1}, s{SB0}")
    a(f"s_mov_b32 s{SB0}, s{STMP}")
    a(f"s_mov_b32 s{SITER}, %[iters]")
    if "stamps" in VARIANT:
        a("s_memtime s[72:73]")
    a(f"s_cmp_eq_u32 s{SITER}, 0")
    a("s_cbranch_scc1 L_dq_tail_%=")
    a("L_dq_loop_%=:")
    stamp(E, 0)
    E.drain("s_waitcnt vmcnt(0) lgkmcnt(15)", keep=15)
    a("s_barrier")
    stamp(E, 1)
    a(f"s_mov_b32 s{STMP}, s{SB0}")
    a(f"s_mov_b32 s{SB0}, s{SB1}")
    a(f"s_mov_b32 s{SB1}, s{SBD}")
    a(f"s_mov_b32 s{SBD}, s{STMP}")
    for t in dq_addr("A", f"s{SB1}"):
        a(t)
    a(f"s_add_u32 s{STMP}, s{SBD}, %[wq]")
    later = {1 + i: [t] for i, t in enumerate(dq_addr("TC", f"s{SB0}") + dq_addr("TN", f"s{SB1}"))}
    # half 2t+1: C(2t), B(2t) tail, B(2t+1) head (set 1), A(2t+2) into set 0 (tile t+1 half 0); the
    # K^T fragments of C(2t+1) (tile t half 1 at TC); the DMA of tile t+2
    dq_half(E, True, b_even, b_odd, 0, 0, (DTC, 1), dq_dma(SBD), extra=later)
    stamp(E, 2)
    for t in dq_advance():
        a(t)
    # half 2t+2: C(2t+1), B(2t+1) tail, B(2t+2) head (set 0), A(2t+3) into set 1 (tile t+1 half 1);
    # the K^T fragments of C(2t+2) (tile t+1 half 0 at TN)
    dq_half(E, True, b_odd, b_even, 1, 1, (DTN, 0))
    stamp(E, 3)
    a(f"s_sub_u32 s{SITER}, s{SITER}, 1")
    a(f"s_cmp_eq_u32 s{SITER}, 0")
    a("s_cbranch_scc0 L_dq_loop_%=")
    a("L_dq_tail_%=:")
    if "stamps" in VARIANT:
        a("s_memtime s[74:75]")
    dq_half(E, True, b_even, b_odd, None, None, (DTN, 1))
    dq_half(E, True, b_odd, {}, None, None, None)
    if "stamps" in VARIANT:
        E.drain("s_waitcnt lgkmcnt(0)")
        for k in range(8):
            a(f"v_mov_b32 v0, s{60 + 2 * k}")
            a(f"v_mov_b32 v1, s{61 + 2 * k}")
            a(f"global_store_dwordx2 %[stp], v[0:1], off offset:{8 * k}")
            a("s_nop 1")
    a("s_waitcnt vmcnt(0)")
    a(f"s_mov_b32 m0, s{SKEEP}")
    a("s_nop 15")
    a("s_nop 15")
    return E.L


# =============================================================================================
# Persistent dQ (attn_dq_w1p_kernel): one workgroup per CU walks its 256-query blocks in ONE asm
# statement, as the persistent dK / dV kernel walks key blocks: each block's Q / dO rows, lse and delta
# go by LDS-DMA into a dedicated region an item ahead (each wave its own 64 queries), its first two
# K / V tiles into the ring buffers the previous block's tail no longer reads. Table row (96 B): the
# Q, dO, lse, delta descriptors of the block (sizes: its valid rows), the K / V bases of the (batch,
# head), the dQ descriptor.
# =============================================================================================
DP_QO = 3 * D_BUF                     # Q / dO prefetch region: [256][128 B] Q, then dO
DP_ST = DP_QO + 2 * 32768             # lse [256] f32, then delta [256]
DP_STG = DP_ST + 2048                 # staging: 4 waves x 4 KiB (dQ of one query tile)
DP_TAB = DP_STG + 4 * 4096
DNLR = 190                            # -lse of the lane's query in qt 0 / 1 (the B stream's fma)
DP_TABV = 192
DP_VLAST = 192
DSQ, DSO, DSL, DSD_, DSDQ = 40, 44, 48, 52, 56   # next block's Q, dO, lse, delta descriptors; this block's dQ
DSITEM = 39
DKB = 80                              # (the next block's K / V bases wait in SRDK / SRDV words 0, 1)


def dqp_region_dma():
    """the next block's Q / dO rows of this wave (queries 64 w .. + 63, 8 pieces each) into the Q / dO
    region, its lse / delta words into the stats region (one dword piece each)"""
    out = []
    for srd, vo, s8, reg in ((DSQ, "%[vqd", "%[s8q]", 0), (DSO, "%[vod", "%[s8o]", 32768)):
        for i in range(8):
            out += [f"s_mul_i32 s{STMP}, {s8}, {i}",
                    f"s_add_u32 m0, %[qow], {reg + 1024 * i}",
                    "s_nop 0",
                    f"buffer_load_dwordx4 {vo}{i & 1}], s[{srd}:{srd + 3}], s{STMP} offen lds"]
    for srd, reg in ((DSL, 0), (DSD_, 1024)):
        out += [f"s_add_u32 m0, %[stw], {reg}", "s_nop 0",
                f"buffer_load_dword %[vsd], s[{srd}:{srd + 3}], 0 offen lds"]
    return out


def dqp_tile_dma(buf):
    out = [f"s_add_u32 s{STMP}, s{buf}, %[wq]"]
    for m0, ld in dq_dma(buf):
        out += [m0, "s_nop 0", ld]
    return out + dq_advance()


def dqp_epilogue(E):
    """dQ (x scale) of the block, one query tile per pass: bf16 rows through this wave's staging area,
    buffer stores clipped to the block's valid queries"""
    a = E.raw
    a("s_nop 15")
    a("s_nop 15")
    WX, WB = 178, 179
    a(f"v_bfe_u32 {v(WX)}, %[vwd], 7, 3")
    a(f"v_add_u32 {v(WB)}, %[stg], %[vwd]")
    for qt in range(2):
        for d in range(2):
            for r in range(16):
                a(f"v_accvgpr_read_b32 {v(66 + 16 * d + r)}, {a_(16 * (2 * qt + d) + r)}")
        for r in range(32):
            a(f"v_mul_f32 {v(66 + r)}, %[scale], {v(66 + r)}")
        for d in range(2):
            for g in range(4):
                src = 66 + 16 * d + 4 * g
                c = 4 * d + g
                wd, wt = 130 + 2 * c, 180 + c
                a(f"v_cvt_pk_bf16_f32 {v(wd)}, {v(src)}, {v(src + 1)}")
                a(f"v_cvt_pk_bf16_f32 {v(wd + 1)}, {v(src + 2)}, {v(src + 3)}")
                a(f"v_xor_b32 {v(wt)}, {c}, {v(WX)}")
                a(f"v_lshl_add_u32 {v(wt)}, {v(wt)}, 4, {v(WB)}")
                a(f"ds_write_b64 {v(wt)}, {v(wd, 2)}")
        a("s_waitcnt lgkmcnt(0)")
        for i in range(4):
            a(f"ds_read_b128 {v(98 + 4 * i, 4)}, %[vrd] offset:{1024 * i}")
        a("s_waitcnt lgkmcnt(0)")
        for i in range(4):
            a(f"s_mul_i32 s{STMP}, %[s8dq], {4 * qt + i}")
            a(f"buffer_store_dwordx4 {v(98 + 4 * i, 4)}, %[vdq], s[{DSDQ}:{DSDQ + 3}], s{STMP} offen")


def dq_p_body():
    HARD_ACC[0] = True
    try:
        return _dq_p_body()
    finally:
        HARD_ACC[0] = False


def _dq_p_body():
    E = Emitter()
    a = E.raw

    def rfl(dst, src):
        a(f"v_readfirstlane_b32 s{dst}, {v(src)}")

    def kv_reset():
        return [f"s_mov_b32 s{SRDK + 2}, %[sk2]", f"s_mov_b32 s{SRDK + 3}, 0x20000",
                f"s_mov_b32 s{SRDV + 2}, %[sv2]", f"s_mov_b32 s{SRDV + 3}, 0x20000"]

    a("s_nop 4")
    a(f"s_mov_b32 s{SKEEP}, m0")
    a(f"v_mov_b32 {v(DP_TABV)}, %[tab]")
    a(f"s_mov_b32 s{DSITEM}, %[nitems]")
    # ---- block 0: its region fill, its K / V tiles 0 and 1 -----------------------------------------
    for i in range(5):
        a(f"ds_read_b128 {v(66 + 4 * i, 4)}, {v(DP_TABV)} offset:{16 * i}")
    a("s_waitcnt lgkmcnt(0)")
    for j, srd in enumerate((DSQ, DSO, DSL, DSD_)):
        for i in range(4):
            rfl(srd + i, 66 + 4 * j + i)
    for i in range(2):
        rfl(SRDK + i, 82 + i)
        rfl(SRDV + i, 84 + i)
    for t in kv_reset():
        a(t)
    a("s_nop 4")
    for t in dqp_region_dma():
        a(t)
    a(f"s_mov_b32 s{SB0}, %[lds0]")
    a(f"s_add_u32 s{SB1}, %[lds0], {D_BUF}")
    a(f"s_add_u32 s{SBD}, %[lds0], {2 * D_BUF}")
    for t in dqp_tile_dma(SB0) + dqp_tile_dma(SB1):
        a(t)
    a("s_waitcnt vmcnt(0)")
    a("s_branch L_qp_item_%=")
    a("L_qp_next_%=:")
    a("s_waitcnt vmcnt(8)")  # the previous block's dQ stores (8) may fly
    a("L_qp_item_%=:")
    a("s_barrier")
    # ---- this block's fragments and stats from the region; its dQ descriptor; the next block's
    # region descriptors and K / V bases ----------------------------------------------------------------
    for ks in range(4):
        a(f"v_add_u32 {v(DRK[ks])}, %[qow], %[vr{ks}]")
    for qt in range(2):
        for ks in range(4):
            a(f"ds_read_b128 {a_(DQF(qt, ks), 4)}, {v(DRK[ks])} offset:{qt * 4096}")
            a(f"ds_read_b128 {a_(DOF(qt, ks), 4)}, {v(DRK[ks])} offset:{32768 + qt * 4096}")
    for qt in range(2):
        a(f"ds_read_b32 {v(qt)}, %[vsl] offset:{qt * 128}")
        a(f"ds_read_b32 {v(2 + qt)}, %[vsl] offset:{1024 + qt * 128}")
    a(f"ds_read_b128 {v(86, 4)}, {v(DP_TABV)} offset:80")
    for i in range(5):
        a(f"ds_read_b128 {v(66 + 4 * i, 4)}, {v(DP_TABV)} offset:{ITEM_B + 16 * i}")
    a("s_waitcnt lgkmcnt(0)")
    for t in zero_acc_mfma(4):  # dQ accumulators a[0:63]
        a(t)
    a("s_nop 4")  # the previous block's stores read DSDQ at issue: rewrite after
    for i in range(4):
        rfl(DSDQ + i, 86 + i)
    for j, srd in enumerate((DSQ, DSO, DSL, DSD_)):
        for i in range(4):
            rfl(srd + i, 66 + 4 * j + i)
    rfl(DSITEM - 1, 82)      # the next block's K / V bases: s[35:38] until its tiles are DMA'd
    rfl(DSITEM - 2, 83)
    rfl(DSITEM - 3, 84)
    rfl(DSITEM - 4, 85)
    a("s_nop 4")
    for t in dqp_region_dma():  # the next block's rows (the null row's empty descriptors: zeros)
        a(t)
    # -lse (the B stream's fma), the -delta tuples (the dP chains' initial accumulator)
    for qt in range(2):
        a(f"v_xor_b32 {v(DNLR + qt)}, 0x80000000, {v(qt)}")
        a(f"v_xor_b32 {v(2 + qt)}, 0x80000000, {v(2 + qt)}")
        for r in range(16):
            a(f"v_mov_b32 {v(DNDL(qt) + r)}, {v(2 + qt)}")
    for t in dq_addr("A", f"s{SB0}") + dq_addr("TN", f"s{SB0}"):
        a(t)
    for ins in dq_a_reads(0):
        E.put(ins)
    a("s_nop 1")
    for ins in dq_a_mfmas(0):
        E.put(ins)
    a("s_nop 7")
    a("s_nop 7")
    a("s_nop 3")
    b_even, b_odd = dq_b_stream(0), dq_b_stream(1)
    dq_half(E, False, {}, b_even, 1, 1, (DTN, 0))
    a(f"s_mov_b32 s{STMP}, s{SBD}")
    a(f"s_mov_b32 s{SBD}, s{SB1}")
    a(f"s_mov_b32 s{SB1}, s{SB0}")
    a(f"s_mov_b32 s{SB0}, s{STMP}")
    a(f"s_mov_b32 s{SITER}, %[iters]")
    if "stamps" in VARIANT:
        a("s_memtime s[72:73]")
    a(f"s_cmp_eq_u32 s{SITER}, 0")
    a("s_cbranch_scc1 L_qp_tail_%=")
    a("L_qp_loop_%=:")
    stamp(E, 0)
    E.drain("s_waitcnt vmcnt(0) lgkmcnt(15)", keep=15)
    a("s_barrier")
    stamp(E, 1)
    a(f"s_mov_b32 s{STMP}, s{SB0}")
    a(f"s_mov_b32 s{SB0}, s{SB1}")
    a(f"s_mov_b32 s{SB1}, s{SBD}")
    a(f"s_mov_b32 s{SBD}, s{STMP}")
    for t in dq_addr("A", f"s{SB1}"):
        a(t)
    a(f"s_add_u32 s{STMP}, s{SBD}, %[wq]")
    later = {1 + i: [t] for i, t in enumerate(dq_addr("TC", f"s{SB0}") + dq_addr("TN", f"s{SB1}"))}
    dq_half(E, True, b_even, b_odd, 0, 0, (DTC, 1), dq_dma(SBD), extra=later)
    stamp(E, 2)
    for t in dq_advance():
        a(t)
    dq_half(E, True, b_odd, b_even, 1, 1, (DTN, 0))
    stamp(E, 3)
    a(f"s_sub_u32 s{SITER}, s{SITER}, 1")
    a(f"s_cmp_eq_u32 s{SITER}, 0")
    a("s_cbranch_scc0 L_qp_loop_%=")
    a("L_qp_tail_%=:")
    if "stamps" in VARIANT:
        a("s_memtime s[74:75]")
    # ---- tail start: the next block's K / V tiles 0, 1 into SBD and SB0 ------------------------------
    a("s_waitcnt vmcnt(0)")
    E.drain("s_waitcnt lgkmcnt(15)", keep=15)
    a("s_barrier")
    a(f"s_cmp_eq_u32 s{DSITEM}, 1")
    a("s_cbranch_scc1 L_qp_nodma_%=")
    a(f"s_mov_b32 s{SRDK}, s{DSITEM - 1}")
    a(f"s_mov_b32 s{SRDK + 1}, s{DSITEM - 2}")
    a(f"s_mov_b32 s{SRDV}, s{DSITEM - 3}")
    a(f"s_mov_b32 s{SRDV + 1}, s{DSITEM - 4}")
    for t in kv_reset() + dqp_tile_dma(SBD) + dqp_tile_dma(SB0):
        a(t)
    a("L_qp_nodma_%=:")
    dq_half(E, True, b_even, b_odd, None, None, (DTN, 1))
    dq_half(E, True, b_odd, {}, None, None, None)
    E.drain("s_waitcnt lgkmcnt(0)")
    dqp_epilogue(E)
    a(f"s_cmp_eq_u32 s{DSITEM}, 1")
    a("s_cbranch_scc1 L_qp_done_%=")
    a(f"s_mov_b32 s{STMP}, s{SB0}")
    a(f"s_mov_b32 s{SB0}, s{SBD}")
    a(f"s_mov_b32 s{SBD}, s{SB1}")
    a(f"s_mov_b32 s{SB1}, s{STMP}")
    a(f"v_add_u32 {v(DP_TABV)}, {ITEM_B}, {v(DP_TABV)}")
    a(f"s_sub_u32 s{DSITEM}, s{DSITEM}, 1")
    a("s_branch L_qp_next_%=")
    a("L_qp_done_%=:")
    if "stamps" in VARIANT:
        for k in range(8):
            a(f"v_mov_b32 v0, s{60 + 2 * k}")
            a(f"v_mov_b32 v1, s{61 + 2 * k}")
            a(f"global_store_dwordx2 %[stp], v[0:1], off offset:{8 * k}")
            a("s_nop 1")
    a("s_waitcnt vmcnt(0)")
    a(f"s_mov_b32 m0, s{SKEEP}")
    return E.L


def dqp_clobbers(diag=False):
    regs = [f'"v{r}"' for r in range(DP_VLAST + 1)] + [f'"a{r}"' for r in range(240)] + \
           [f'"s{r}"' for r in list(range(35, 60)) + list(range(80, 88)) + list(range(92, 98))]
    if diag:
        regs += [f'"s{r}"' for r in range(60, 76)]
    return ", ".join(regs)


def dq_clobbers(diag=False):
    regs = [f'"v{r}"' for r in range(DVLAST + 1)] + [f'"a{r}"' for r in range(128, 240)] + \
           [f'"s{r}"' for r in list(range(80, 88)) + list(range(92, 98))]
    if diag:
        regs += [f'"s{r}"' for r in range(60, 76)]
    return ", ".join(regs)



def main():
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    args = [x for x in sys.argv[1:] if not x.startswith("--")]
    out = args[0] if args else os.path.join(
        root, "video-generation-for-human-avatars_amd", "csrc", "attn_bwd_body.h")
    diag = "--diag" in sys.argv

    def define(name, lines):
        return f"#define {name} \\\n" + " \\\n".join(f'  "{l}\\n\\t"' for l in lines) + "\n"
    VARIANT.clear()
    L = body()
    txt = ["// GENERATED by tools/gen_attn_bwd.py -- do not edit by hand.",
           "// The hand-scheduled loop of attn_dkdv_w1_kernel (attention_pipe.hip); see the generator's docstring.",
           "#pragma once", "",
           f"#define LTX_DKDV_W1_BUF {W_BUF}",
           f"#define LTX_DKDV_W1_NBUF {NBUF}",
           define("LTX_DKDV_W1_BODY", L)]
    if diag:  # timing-only bodies: the loop with phase stamps, without VALU, without LDS reads
        for k, var in enumerate(("stamps", "stamps+novalu", "stamps+nolds", "stamps+dmalast", "stamps+expfirst"), 1):
            VARIANT.clear()
            VARIANT.update(var.split("+"))
            txt.append(define(f"LTX_DKDV_W1_BODY_V{k}", body()))
        VARIANT.clear()
        txt.append("#undef LTX_DKDV_W1_CLOBBERS")
    txt.append("#define LTX_DKDV_W1_CLOBBERS " + clobbers(diag) + "\n")
    VARIANT.clear()
    txt += [f"#define LTX_DKDV_W1P_KV {P_KV}", f"#define LTX_DKDV_W1P_STG {P_STG}", f"#define LTX_DKDV_W1P_TAB {P_TAB}",
            f"#define LTX_DKDV_W1P_ITEM {ITEM_B}", define("LTX_DKDV_W1P_BODY", dkdv_p_body())]
    if diag:
        VARIANT.update({"stamps", "itemstamps"})  # item-phase stamps (tools/dkdv_item_stamps.py)
        txt.append(define("LTX_DKDV_W1P_BODY_V1", dkdv_p_body()))
        VARIANT.clear()
        txt.append("#undef LTX_DKDV_W1P_CLOBBERS")
    txt.append("#define LTX_DKDV_W1P_CLOBBERS " + p_clobbers(diag) + "\n")
    VARIANT.clear()
    txt += [f"#define LTX_DQ_W1_BUF {D_BUF}", define("LTX_DQ_W1_BODY", dq_body())]
    if diag:
        for k, var in enumerate(("stamps", "stamps+novalu"), 1):
            VARIANT.clear()
            VARIANT.update(var.split("+"))
            txt.append(define(f"LTX_DQ_W1_BODY_V{k}", dq_body()))
        VARIANT.clear()
        txt.append("#undef LTX_DQ_W1_CLOBBERS")
    txt.append("#define LTX_DQ_W1_CLOBBERS " + dq_clobbers(diag) + "\n")
    VARIANT.clear()
    txt += [f"#define LTX_DQ_W1P_QO {DP_QO}", f"#define LTX_DQ_W1P_ST {DP_ST}", f"#define LTX_DQ_W1P_STG {DP_STG}",
            f"#define LTX_DQ_W1P_TAB {DP_TAB}",
            define("LTX_DQ_W1P_BODY", dq_p_body())]
    if diag:
        VARIANT.update({"stamps"})
        txt.append(define("LTX_DQ_W1P_BODY_V1", dq_p_body()))
        VARIANT.clear()
        txt.append("#undef LTX_DQ_W1P_CLOBBERS")
    txt.append("#define LTX_DQ_W1P_CLOBBERS " + dqp_clobbers(diag) + "\n")
    open(out, "w").write("\n".join(txt))
    print(out, len(L), "lines")


if __name__ == "__main__":
    main()
