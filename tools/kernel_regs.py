"""Per-kernel VGPR count and scratch bytes from a hipcc -S (device) assembly file:
  python tools/kernel_regs.py file.s [substring]"""
import re
import sys

cur = None
rows = []
for line in open(sys.argv[1]):
    m = re.match(r"\s*\.amdhsa_kernel\s+(\S+)", line)
    if m:
        cur = {"name": m.group(1)}
        continue
    if cur is None:
        continue
    m = re.match(r"\s*\.amdhsa_(next_free_vgpr|private_segment_fixed_size|accum_offset)\s+(\d+)", line)
    if m:
        cur[m.group(1)] = int(m.group(2))
    if line.strip().startswith(".end_amdhsa_kernel"):
        rows.append(cur)
        cur = None
pat = sys.argv[2] if len(sys.argv) > 2 else ""
for r in rows:
    if pat in r["name"]:
        print(f"vgpr {r.get('next_free_vgpr', '?'):>4} scratch {r.get('private_segment_fixed_size', '?'):>4}  {r['name']}")
