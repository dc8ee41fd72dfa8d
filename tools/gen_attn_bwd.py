"""Generates video-generation-for-human-avatars_amd/csrc/attn_bwd_body.h: the hand-scheduled main loop of
attn_dkdv_w1_kernel (attention_pipe.hip), the dK / dV half of F.scaled_dot_product_attention's
backward (attention.py:1057-1064) for head dim 64 and no key bias, as ONE inline-asm statement.

Why: at head dim 64 the softmax VALU of a score block costs as many
issue cycles as its MFMAs, and at two waves per SIMD (attn_dkdv_pipe_kernel, 248 VGPRs) the two
streams' MFMAs and VALU compete for one issue port (MFMA-busy 0.53). Here one wave per SIMD owns 64
keys (two 32-key tiles, so every Q / dO fragment read from LDS feeds two MFMAs) and every
instruction is placed: per 32-query half j the wave issues 32 MFMAs -- C(j-1) (dV^T += dO^T.P,
dK^T += Q^T.dS) and A(j+1) (S^T = K.Q^T, dP'^T = delta - V.dO^T) -- and each MFMA gap carries
B(j)'s softmax work (phase 1: 2 x (v_fma, v_exp); phase 2: 2 x v_mul + 2 x v_cvt_pk) plus at most
two LDS reads: 1 MFMA + <= 6 fillers per gap, at most 2 transcendental.

Arithmetic and accumulation order are those of attn_dkdv_pipe_kernel (same fragment layouts, MFMA
chains in the same k order, delta as dP's initial accumulator with V negated), so dK / dV are
bitwise equal to it (tests/test_kernels_gpu.py).

Tiles of 64 queries (Q | dO | lse | delta) arrive by LDS-DMA into a 3-buffer ring, one tile ahead,
one barrier per tile. Rows past Nq are out of range of the tile's buffer descriptor (the base
advances and num_records shrinks per tile), so they land as zeros: S = 0, lse = 0 gives P = 1, but
their dO and delta rows are 0, so they add exactly 0 to dV (dO^T.P) and dS = -P (delta - dO.V) = 0.

Registers (hard-coded, clobbered; the dV / dK accumulators are the statement's "+a" operands
%0..%7, which hipcc must place in a0..a127):
  v[0:127]   S / dP' tiles: set s (0, 1), tile T (0 S kt0, 1 dP kt0, 2 S kt1, 3 dP kt1) at 64 s + 16 T
  v[128:143] P packs  PB[kt][ss] (B operands of dV) at 128 + 8 kt + 4 ss
  v[144:159] dS packs SB[kt][ss] at 144 + 8 kt + 4 ss
  v[160:175] lse tuple of the half being exponentiated (accumulator row order)
  v[176:191] delta tuple of the half being multiplied (dP chains' initial accumulator)
  v[192:204] LDS addresses: RA[ks] row fragments (A's tile), ST statistics (A's tile), TC / TN[2d+i]
             transposed fragments of the current / next tile
  a[128:159] K fragments KF[kt][ks], a[160:191] -V fragments, a[192:223] QA / OA row fragments,
  a[224:255] TO / TQ transposed fragments
  s[80:91]   buffer descriptors of Q, dO and this wave's statistic row (lse or delta)
  s[92:98]   ring buffer bases B0 / B1 / BD, scratch, loop counter, saved M0
"""
import os
import sys

P_TILE = 8192            # one [64][64] bf16 tile
P_STAT = 256             # 64 f32
W_BUF = 2 * P_TILE + 3 * P_STAT   # Q | dO | lse | delta | dummy (waves 2, 3)
NBUF = 3

# ---------------------------------------------------------------------------------------- registers
def SD(s, T):
    return 64 * s + 16 * T


def PB(kt, ss):
    return 128 + 8 * kt + 4 * ss


def SB(kt, ss):
    return 144 + 8 * kt + 4 * ss


LSE, DLT = 160, 176
RA = [192, 193, 194, 195]
ST = 196
TC = [197, 198, 199, 200]
TN = [201, 202, 203, 204]
VLAST = 206
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


def v(r, n=1):
    return f"v{r}" if n == 1 else f"v[{r}:{r + n - 1}]"


def a_(r, n=1):
    return f"a{r}" if n == 1 else f"a[{r}:{r + n - 1}]"


def mfma(dst, A, B, C):
    return f"v_mfma_f32_32x32x16_bf16 {dst}, {A}, {B}, {C}"


# ---------------------------------------------------------------------------------------- pieces
def c_mfmas():
    """C(j-1): dV^T[kt][d] += TO[ss][d] . PB[kt][ss], dK^T[kt][d] += TQ[ss][d] . SB[kt][ss], ss-major
    (each accumulator takes ss = 0 then ss = 1, as attn_dkdv_pipe_kernel's stage C)"""
    out = []
    for ss in range(2):
        for d in range(2):
            for kt in range(2):
                dv = "%" + str(ACC[("dv", kt, d)])
                dk = "%" + str(ACC[("dk", kt, d)])
                out.append(mfma(dv, a_(TO(ss, d), 4), v(PB(kt, ss), 4), dv))
                out.append(mfma(dk, a_(TQ(ss, d), 4), v(SB(kt, ss), 4), dk))
    return out


def a_mfmas(s):
    """A(j+1) into set s, kt-major: S kt0 (ks 0..3), dP' kt0, S kt1, dP' kt1 (each chain in k order;
    S starts from 0, dP' from the delta tuple)"""
    out = []
    for kt in range(2):
        for ks in range(4):
            dst = v(SD(s, 2 * kt), 16)
            out.append(mfma(dst, a_(QA(ks), 4), a_(KF(kt, ks), 4), "0" if ks == 0 else dst))
        for ks in range(4):
            dst = v(SD(s, 2 * kt + 1), 16)
            out.append(mfma(dst, a_(OA(ks), 4), a_(VF(kt, ks), 4), v(DLT, 16) if ks == 0 else dst))
    return out


def b_phase1(s):
    """B(j) part 1 on set s: P = exp2(S c2 - lse) in place, 2 elements per slot (16 slots)"""
    slots = []
    for m in range(16):
        ins = []
        for e in (2 * m, 2 * m + 1):
            kt, r = e // 16, e % 16
            sr = SD(s, 2 * kt) + r
            ins.append(f"v_fma_f32 {v(sr)}, {v(sr)}, %[c2], -{v(LSE + r)}")
        for e in (2 * m, 2 * m + 1):
            kt, r = e // 16, e % 16
            sr = SD(s, 2 * kt) + r
            ins.append(f"v_exp_f32 {v(sr)}, {v(sr)}")
        slots.append(ins)
    return slots


def b_phase2(s):
    """B(j) part 2 on set s: dS = -(P dP') in place, then the bf16 packs of P and dS (2 per slot)"""
    slots = []
    for m in range(16):
        kt, r = (2 * m) // 16, (2 * m) % 16
        s0, d0 = SD(s, 2 * kt) + r, SD(s, 2 * kt + 1) + r
        ss, i = r // 8, (r % 8) // 2
        slots.append([f"v_mul_f32 {v(d0)}, -{v(s0)}, {v(d0)}",
                      f"v_mul_f32 {v(d0 + 1)}, -{v(s0 + 1)}, {v(d0 + 1)}",
                      f"v_cvt_pk_bf16_f32 {v(PB(kt, ss) + i)}, {v(s0)}, {v(s0 + 1)}",
                      f"v_cvt_pk_bf16_f32 {v(SB(kt, ss) + i)}, {v(d0)}, {v(d0 + 1)}"])
    return slots


def a_reads(u):
    """A's operands for half u of the tile at RA / ST: Q rows, the delta tuple, dO rows (in the order
    the kt-major A MFMAs consume them)"""
    out = [f"ds_read_b128 {a_(QA(ks), 4)}, {v(RA[ks])} offset:{u * 4096}" for ks in range(4)]
    out += [f"ds_read_b128 {v(DLT + 4 * g, 4)}, {v(ST)} offset:{2 * P_TILE + P_STAT + (u * 32 + 8 * g) * 4}"
            for g in range(4)]
    out += [f"ds_read_b128 {a_(OA(ks), 4)}, {v(RA[ks])} offset:{P_TILE + u * 4096}" for ks in range(4)]
    return out


def tr_reads(T, u):
    """C's transposed fragments of half u of the tile at T (TC or TN), in the order C consumes them"""
    out = []
    for ss in range(2):
        for d in range(2):
            base = (u * 32 + 16 * ss) * 128
            for dst, region in ((TO(ss, d), P_TILE), (TQ(ss, d), 0)):
                out.append(f"ds_read_b64_tr_b16 {a_(dst, 2)}, {v(T[2 * d])} offset:{region + base}")
                out.append(f"ds_read_b64_tr_b16 {a_(dst + 2, 2)}, {v(T[2 * d + 1])} offset:{region + base}")
    return out


def lse_reads(u):
    return [f"ds_read_b128 {v(LSE + 4 * g, 4)}, {v(ST)} offset:{2 * P_TILE + (u * 32 + 8 * g) * 4}"
            for g in range(4)]


def dma_pieces():
    """this wave's DMA of one tile into buffer BD: Q pieces 2w, 2w+1, dO pieces, its statistic row;
    (M0 write, load) pairs"""
    out = []
    for i in range(2):
        out.append((f"s_add_u32 m0, s{STMP}, {i * 1024}",
                    f"buffer_load_dwordx4 %[vq{i}], s[{SRDQ}:{SRDQ + 3}], 0 offen lds"))
        out.append((f"s_add_u32 m0, s{STMP}, {P_TILE + i * 1024}",
                    f"buffer_load_dwordx4 %[vo{i}], s[{SRDO}:{SRDO + 3}], 0 offen lds"))
    out.append((f"s_add_u32 m0, s{SBD}, %[wst]",
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


# ---------------------------------------------------------------------------------------- iteration
VARIANT = set()  # diagnostic bodies (make diag): "nowait", "novalu", "nolds", "nomfma"


def iteration(L, c, b_set, a_set, a_u, rd2, dma=()):
    """one 32-query half: C(j-1) if c, B(j) on b_set (None: no B), A(j+1) into a_set from half a_u of
    the tile at RA / ST (None: no A); rd2 = LDS reads for phase 2 (next C's fragments, next lse);
    dma = (M0, load) pairs placed in phase 2"""
    a = L.append
    if "nolds" in VARIANT:
        rd2 = []
    # phase 1: C MFMAs (or none) + B exponentials + A's operand reads
    if "nowait" not in VARIANT:
        a("s_waitcnt lgkmcnt(0)")
    cm = c_mfmas() if c and "nomfma" not in VARIANT else []
    b1 = b_phase1(b_set) if b_set is not None and "novalu" not in VARIANT else [[] for _ in range(16)]
    rd1 = a_reads(a_u) if a_set is not None and "nolds" not in VARIANT else []
    for m in range(16):
        if cm:
            a(cm[m])
        L.extend(b1[m])
        if m < len(rd1):
            a(rd1[m])
    # phase 2: A MFMAs (or none) + B products and packs + the next C's / B's operand reads + DMA
    if "nowait" not in VARIANT:
        a("s_waitcnt lgkmcnt(0)")
    am = a_mfmas(a_set) if a_set is not None and "nomfma" not in VARIANT else []
    b2 = b_phase2(b_set) if b_set is not None and "novalu" not in VARIANT else [[] for _ in range(16)]
    after = {m: [] for m in range(16)}
    for k, r in enumerate(rd2):  # reads in slots 0 .. 11 (the last ones land before phase 1)
        after[(k * 12) // max(len(rd2), 1)].append(r)
    for k, (m0, ld) in enumerate(dma):  # M0 one slot ahead of its load
        q = 2 + 3 * k
        after[q - 1].append(m0)
        after[q].append(ld)
    for m in range(16):
        if am:
            a(am[m])
        L.extend(b2[m])
        L.extend(after[m])


def c_only(L):
    """C(J-1) alone (16 MFMAs)"""
    L.append("s_waitcnt lgkmcnt(0)")
    L.extend(c_mfmas())


def body():
    L = []
    a = L.append
    a("s_nop 4")  # SGPR operands fresh from v_readfirstlane -> descriptors / M0
    a(f"s_mov_b32 s{SKEEP}, m0")
    for srd, nm in ((SRDQ, "sq"), (SRDO, "so"), (SRDS, "ss")):  # descriptors as two 64-bit halves each
        a(f"s_mov_b64 s[{srd}:{srd + 1}], %[{nm}0]")
        a(f"s_mov_b64 s[{srd + 2}:{srd + 3}], %[{nm}1]")
    # ---- prologue: K, V fragments; tiles 0 and 1; A(0); B(0) beside A(1) --------------------------
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
        for m0, ld in dma_pieces():
            a(m0.replace(f"s{SBD}", f"s{buf}"))
            a("s_nop 0")
            a(ld)
        L.extend(advance_srds())
    a("s_waitcnt vmcnt(5)")  # K, V and tile 0 landed (tile 1's five pieces may fly)
    for r in range(32):  # -V (sign flip, exact) into the accumulator file
        a(f"v_xor_b32 {v(r)}, 0x80008000, {v(r)}")
    for r in range(32):
        a(f"v_accvgpr_write_b32 {a_(160 + r)}, {v(r)}")
    a("s_barrier")
    L.extend(addr_regs("A", f"s{SB0}"))
    L.extend(addr_regs("TN", f"s{SB0}"))
    # A(0) into set 0 (tile 0, half 0), lse of B(0)
    for r in a_reads(0) + lse_reads(0):
        a(r)
    a("s_waitcnt lgkmcnt(0)")
    a("s_nop 1")  # accvgpr writes of -V -> MFMA operand
    L.extend(a_mfmas(0))
    # B(0) on set 0 beside A(1) into set 1 (tile 0, half 1); phase 2 reads C(0)'s fragments (tile 0
    # half 0) and B(1)'s lse (tile 0 half 1)
    a("s_nop 7")
    a("s_nop 7")
    a("s_nop 3")  # the last A MFMA's results -> the first exponentials (no C MFMAs in between)
    iteration(L, False, 0, 1, 1, tr_reads(TN, 0) + lse_reads(1))
    # ---- steady state: tile t = 0 .. ntiles - 2 ----------------------------------------------------
    # every body opens by rotating (B0, B1, BD) <- (B1, BD, B0); the prologue left B0 = buffer 0,
    # B1 = buffer 1, BD = buffer 2, so pre-rotate backwards to (buffer 2, buffer 0, buffer 1)
    a(f"s_mov_b32 s{STMP}, s{SBD}")
    a(f"s_mov_b32 s{SBD}, s{SB1}")
    a(f"s_mov_b32 s{SB1}, s{SB0}")
    a(f"s_mov_b32 s{SB0}, s{STMP}")
    a(f"s_mov_b32 s{SITER}, %[iters]")
    a(f"s_cmp_eq_u32 s{SITER}, 0")
    a("s_cbranch_scc1 L_dkdv_tail_%=")
    a("L_dkdv_loop_%=:")
    # tile t+1 (DMA issued one tile ago) landed in every wave, all reads of tile t-1 done
    a("s_waitcnt vmcnt(0) lgkmcnt(0)")
    a("s_barrier")
    # buffers: B0 <- t % 3, B1 <- (t+1) % 3, BD <- (t+2) % 3 (rotate the three bases)
    a(f"s_mov_b32 s{STMP}, s{SB0}")
    a(f"s_mov_b32 s{SB0}, s{SB1}")
    a(f"s_mov_b32 s{SB1}, s{SBD}")
    a(f"s_mov_b32 s{SBD}, s{STMP}")
    L.extend(addr_regs("A", f"s{SB1}"))
    L.extend(addr_regs("TC", f"s{SB0}"))
    L.extend(addr_regs("TN", f"s{SB1}"))
    a(f"s_add_u32 s{STMP}, s{SBD}, %[wq]")
    # C(2t), B(2t+1) on set 1, A(2t+2) into set 0 (tile t+1 half 0); phase 2: C(2t+1)'s fragments
    # (tile t half 1), B(2t+2)'s lse (tile t+1 half 0), the DMA of tile t+2 into BD
    iteration(L, True, 1, 0, 0, tr_reads(TC, 1) + lse_reads(0), dma_pieces())
    L.extend(advance_srds())
    # C(2t+1), B(2t+2) on set 0, A(2t+3) into set 1 (tile t+1 half 1); phase 2: C(2t+2)'s fragments
    # (tile t+1 half 0), B(2t+3)'s lse (tile t+1 half 1)
    iteration(L, True, 0, 1, 1, tr_reads(TN, 0) + lse_reads(1))
    a(f"s_sub_u32 s{SITER}, s{SITER}, 1")
    a(f"s_cmp_eq_u32 s{SITER}, 0")
    a("s_cbranch_scc0 L_dkdv_loop_%=")
    a("L_dkdv_tail_%=:")
    # ---- last tile T-1: C(J-2), B(J-1) on set 1 (phase 2 reads C(J-1)'s fragments: tile T-1 half 1,
    # at TN); then C(J-1) ------------------------------------------------------------------------
    iteration(L, True, 1, None, None, tr_reads(TN, 1))
    c_only(L)
    a("s_waitcnt vmcnt(0)")  # no DMA may land in the ring after the statement (epilogue staging)
    a(f"s_mov_b32 m0, s{SKEEP}")
    a("s_nop 15")
    a("s_nop 15")  # the last MFMAs' accumulators -> the compiler's reads after the statement
    return L


def clobbers():
    regs = [f'"v{r}"' for r in range(VLAST + 1)] + [f'"a{r}"' for r in range(128, 256)] + \
           [f'"s{r}"' for r in range(80, 98)]
    return ", ".join(regs)


def main():
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    args = [x for x in sys.argv[1:] if not x.startswith("--")]
    out = args[0] if args else os.path.join(
        root, "video-generation-for-human-avatars_amd", "csrc", "attn_bwd_body.h")
    # the tail after the loop must see TN = tile T-1's buffer: the last body computed TN from B1
    # (= (T-1) % 3), and with no body at all (T = 1) the prologue's TN (buffer 0) is tile 0's
    diag = "--diag" in sys.argv
    L = body()

    def define(name, lines):
        return f"#define {name} \\\n" + " \\\n".join(f'  "{l}\\n\\t"' for l in lines) + "\n"
    txt = ["// GENERATED by tools/gen_attn_bwd.py -- do not edit by hand.",
           "// The hand-scheduled loop of attn_dkdv_w1_kernel (attention_pipe.hip); see the generator's docstring.",
           "#pragma once", "",
           f"#define LTX_DKDV_W1_BUF {W_BUF}",
           f"#define LTX_DKDV_W1_NBUF {NBUF}",
           define("LTX_DKDV_W1_BODY", L),
           "#define LTX_DKDV_W1_CLOBBERS " + clobbers() + "\n"]
    if diag:  # timing-only bodies (wrong results): what each part of the schedule costs
        for k, var in enumerate(("nowait", "novalu", "nolds", "nomfma"), 1):
            VARIANT.clear()
            VARIANT.add(var)
            txt.append(define(f"LTX_DKDV_W1_BODY_V{k}", body()))
        VARIANT.clear()
    open(out, "w").write("\n".join(txt))
    print(out, len(L), "lines")


if __name__ == "__main__":
    main()
