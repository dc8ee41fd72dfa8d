"""Per-kernel (name, grid) totals per training step from a rocprofv3 kernel_trace.csv.
Usage: python tools/trace_summary.py <kernel_trace.csv> <steps_in_trace> [top]"""
import collections, csv, sys

rows = list(csv.DictReader(open(sys.argv[1])))
steps = float(sys.argv[2])
top = int(sys.argv[3]) if len(sys.argv) > 3 else 40
agg = collections.defaultdict(list)
for r in rows:
    key = (r["Kernel_Name"].split("(")[0].replace("void ", "")[:52], r["Grid_Size_X"])
    agg[key].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
tot = sum(sum(v) for v in agg.values()) / steps
print(f"total kernel time per step: {tot / 1e6:.2f} ms")
for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1]))[:top]:
    print(f"{k[0]:54s} {k[1]:>8s} {len(v) / steps:6.1f}/step {sum(v) / len(v) / 1e3:8.1f} us {sum(v) / steps / 1e6:7.2f} ms")
