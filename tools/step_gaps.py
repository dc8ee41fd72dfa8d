"""Device idle time between kernels in a rocprofv3 rocpd trace (--kernel-trace): the union of
kernel intervals vs the span, and the largest gaps with the kernels on either side (host-bound
stretches show up here, not in per-kernel stats). Only the last `window_ms` of the trace (the
bench's steady state) is counted.
Usage: python tools/step_gaps.py <run_results.db> [window_ms] [top]"""
import sqlite3
import sys

db = sys.argv[1]
window = float(sys.argv[2]) if len(sys.argv) > 2 else 1000.0
top = int(sys.argv[3]) if len(sys.argv) > 3 else 25
con = sqlite3.connect(db)
rows = sorted(con.execute("select start, end, name from kernels"))
t_end = max(r[1] for r in rows)
rows = [r for r in rows if r[0] >= t_end - window * 1e6]
span = rows[-1][1] - rows[0][0]
busy, cur_s, cur_e = 0, rows[0][0], rows[0][1]
gaps = []
prev = rows[0]
for s, e, n in rows[1:]:
    if s > cur_e:
        busy += cur_e - cur_s
        gaps.append((s - cur_e, prev[2], n))
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
    prev = (s, e, n)
busy += cur_e - cur_s
idle = span - busy
print(f"window {span / 1e6:.1f} ms: busy {busy / 1e6:.1f} ms, idle {idle / 1e6:.2f} ms "
      f"({100 * idle / span:.1f} %), {len(gaps)} gaps")
short = lambda n: n.replace("void ", "").split("(")[0][:48]
for g, a, b in sorted(gaps, reverse=True)[:top]:
    print(f"{g / 1e3:8.1f} us  after {short(a):48s} before {short(b)}")
