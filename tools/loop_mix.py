"""Instruction mix of a kernel's innermost loop(s) in a hipcc -S (device) assembly file:
  python tools/loop_mix.py file.s kernel_substring
Counts opcodes between each 'Loop Header' label and the loop's back-branch, plus a VALU issue-cycle
estimate (MI355X_MICROARCH.md constants: transcendental 8, other VALU 4, MFMA 8 of issue; MFMA
pipe 32 cycles per 32x32x16 / 16 per 16x16x32)."""
import re
import sys
from collections import Counter

path, pat = sys.argv[1], sys.argv[2]
lines = open(path).read().split("\n")
start = None
for i, l in enumerate(lines):
    m = re.match(r"^(\S+):\s*(;.*)?$", l)
    if m and pat in m.group(1) and not m.group(1).startswith("."):
        start = i
        break
if start is None:
    sys.exit(f"no kernel matching {pat}")
end = next(i for i in range(start, len(lines)) if "s_endpgm" in lines[i])
body = lines[start:end]
# a loop = its header block + every block annotated "; in Loop: Header=<header> Depth=1"
blocks, cur = [], None
for l in body:
    m = re.match(r"^(\.LBB\S+):(.*)$", l)
    if m:
        cur = [m.group(1), m.group(2), []]
        blocks.append(cur)
    elif cur is not None:
        cur[2].append(l)
loops = []
for lab, ann, ls in blocks:
    if "Loop Header" in ann and "Depth=1" in ann:
        hdr = lab.replace(".LBB", "BB")
        members = [b for b in blocks if b[0] == lab or ("Header=" + hdr + " ") in b[1] + " "]
        loops.append((lab, [x for b in members for x in b[2]]))
TRANS = ("v_exp", "v_log", "v_rcp", "v_rsq", "v_sqrt", "v_sin", "v_cos")
for lab, ls in loops:
    c = Counter()
    for l in ls:
        t = l.strip().split()
        if not t or t[0].startswith((";", ".")):
            continue
        c[t[0]] += 1
    mf = sum(v for k, v in c.items() if k.startswith("v_mfma"))
    mf32 = sum(v for k, v in c.items() if k.startswith("v_mfma") and "32x32" in k)
    valu = {k: v for k, v in c.items() if k.startswith("v_") and not k.startswith("v_mfma")}
    cyc = sum(v * (8 if k.startswith(TRANS) else 4) for k, v in valu.items())
    print(f"loop {lab} ({len(ls)} lines): mfma {mf} (pipe {mf32 * 32 + (mf - mf32) * 16} cyc), "
          f"valu {sum(valu.values())} (~{cyc} issue cyc + {8 * mf} mfma issue)")
    print("   " + " ".join(f"{k}:{v}" for k, v in c.most_common()))
