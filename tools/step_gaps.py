"""Device idle time between kernels in a rocprofv3 rocpd trace (--kernel-trace): the union of
kernel intervals vs the span, the gaps by size class, the (previous, next) kernel pairs with the
most idle time, and the largest single gaps. Host-bound stretches show up here, not in per-kernel
stats. Only the last `window_ms` of the trace (the bench's steady state) is counted.
Usage: python tools/step_gaps.py <run_results.db> [window_ms] [top] [skip_last_ms]
(skip_last_ms: leave out the end of the trace -- bench.py's per-launch timing steps there wait on
events after every launch)"""
import collections
import sqlite3
import sys

db = sys.argv[1]
window = float(sys.argv[2]) if len(sys.argv) > 2 else 1000.0
top = int(sys.argv[3]) if len(sys.argv) > 3 else 25
skip = float(sys.argv[4]) if len(sys.argv) > 4 else 0.0
con = sqlite3.connect(db)
rows = sorted(con.execute("select start, end, name from kernels"))
t_end = max(r[1] for r in rows) - skip * 1e6
rows = [r for r in rows if t_end - window * 1e6 <= r[0] and r[1] <= t_end]
span = rows[-1][1] - rows[0][0]
short = lambda n: n.replace("void ", "").split("(")[0][:44]
busy, cur_s, cur_e = 0, rows[0][0], rows[0][1]
gaps = []
prev = rows[0]
for s, e, n in rows[1:]:
    if s > cur_e:
        busy += cur_e - cur_s
        gaps.append((s - cur_e, short(prev[2]), short(n)))
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
    prev = (s, e, n)
busy += cur_e - cur_s
idle = span - busy
print(f"window {span / 1e6:.1f} ms: {len(rows)} kernels, busy {busy / 1e6:.1f} ms, idle {idle / 1e6:.2f} ms "
      f"({100 * idle / span:.1f} %), {len(gaps)} gaps")
classes = [(0, 5e3), (5e3, 2e4), (2e4, 1e5), (1e5, 1e12)]
for lo, hi in classes:
    sel = [g for g, _, _ in gaps if lo <= g < hi]
    print(f"  gaps {lo / 1e3:6.0f}-{min(hi, 1e9) / 1e3:6.0f} us: {len(sel):5d}, {sum(sel) / 1e6:6.2f} ms")
pairs = collections.defaultdict(lambda: [0, 0])
for g, a, b in gaps:
    pairs[(a, b)][0] += 1
    pairs[(a, b)][1] += g
print("by kernel pair (count, total us):")
for (a, b), (c, t) in sorted(pairs.items(), key=lambda kv: -kv[1][1])[:top]:
    print(f"  {c:5d} {t / 1e3:9.1f}  {a:44s} -> {b}")
print("largest gaps:")
for g, a, b in sorted(gaps, reverse=True)[:10]:
    print(f"  {g / 1e3:8.1f} us  {a:44s} -> {b}")
