"""Rescale the per-step figures of a rocpd_summary.py table written with the wrong step count
(tools/final_profile.sh passed 18 = timed + warmup, but bench.py also runs one per-kernel timer
step and min(steps, 4) dominant-kernel timer steps: 23 steps in the trace).
usage: python tools/fix_trace_steps.py <trace_summary.txt> <factor>"""
import re
import sys


def main(path, factor):
    f = float(factor)
    out = []
    for line in open(path):
        m = re.match(r"total kernel time per step: ([\d.]+) ms", line)
        if m:
            line = f"total kernel time per step: {float(m.group(1)) * f:.2f} ms\n"
        else:
            m = re.match(r"(.*\s)([\d.]+)/step(\s+[\d.]+ us\s+)([\d.]+)( ms.*)", line.rstrip("\n"))
            if m:
                line = (f"{m.group(1)}{float(m.group(2)) * f:.1f}/step{m.group(3)}"
                        f"{float(m.group(4)) * f:.2f}{m.group(5)}\n")
        out.append(line)
    out.append(f"\nper-step figures rescaled by {factor} (23 bench steps in the trace, the table had been "
               "divided by 18; tools/fix_trace_steps.py).\n")
    open(path, "w").write("".join(out))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
