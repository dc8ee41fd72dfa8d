"""Per-kernel (name, grid) totals per training step from a rocprofv3 SQLite output (rocpd .db,
the default output format of ROCm 7 rocprofv3 --kernel-trace).
Usage: python tools/rocpd_summary.py <run_results.db> <steps_in_trace> [top]"""
import collections
import sqlite3
import sys

db, steps = sys.argv[1], float(sys.argv[2])
top = int(sys.argv[3]) if len(sys.argv) > 3 else 45
con = sqlite3.connect(db)
agg = collections.defaultdict(list)
for name, gx, gy, gz, dur in con.execute("select name, grid_x, grid_y, grid_z, duration from kernels"):
    key = (name.split("(")[0].replace("void ", "")[:58], f"{gx}x{gy}x{gz}")
    agg[key].append(dur)
tot = sum(sum(v) for v in agg.values()) / steps
print(f"total kernel time per step: {tot / 1e6:.2f} ms")
for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1]))[:top]:
    print(f"{k[0]:60s} {k[1]:>16s} {len(v) / steps:6.1f}/step {sum(v) / len(v) / 1e3:8.1f} us "
          f"{sum(v) / steps / 1e6:7.2f} ms")
