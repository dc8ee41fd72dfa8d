"""Per-kernel counter table from rocprofv3 --pmc CSVs (one or more counter_collection.csv files).

    python tools/pmc_table.py a.csv [b.csv ...]

Rows = (kernel, grid); values = mean per dispatch. Derived columns:
  clk_GHz     = GRBM_GUI_ACTIVE / 8 XCDs / kernel duration (MI355X_MICROARCH.md "DVFS give-back")
  mfma_busy   = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8): the fraction of SIMD
                cycles the matrix pipe was busy while the kernel ran
  wait/inst   = SQ_WAIT_ANY, SQ_WAIT_INST_ANY, SQ_ACTIVE_INST_ANY as shares of SQ_WAVE_CYCLES
"""
import csv
import sys
from collections import defaultdict


def short(name):
    name = name.replace("void ", "").replace("ltx::", "")
    if "(" in name:
        name = name[:name.index("(")]
    return name[:70]


def main(paths):
    vals = defaultdict(lambda: defaultdict(list))
    dur = defaultdict(list)
    import os
    for path in paths:
        per = defaultdict(lambda: defaultdict(float))
        meta = {}
        ktrace = {}
        kt = os.path.join(os.path.dirname(path), "run_kernel_trace.csv")
        if os.path.exists(kt):
            with open(kt, newline="") as f:
                for r in csv.DictReader(f):
                    ktrace[r["Dispatch_Id"]] = (float(r["End_Timestamp"]) - float(r["Start_Timestamp"])) / 1e3
        with open(path, newline="") as f:
            for r in csv.DictReader(f):
                d = (path, r["Dispatch_Id"])
                per[d][r["Counter_Name"]] += float(r["Counter_Value"])
                key = (short(r["Kernel_Name"]), r.get("Grid_Size", ""))
                meta[d] = key
        for d in per:
            if d[1] in ktrace:
                dur[meta[d]].append(ktrace[d[1]])
        for d, cs in per.items():
            for c, v in cs.items():
                vals[meta[d]][c].append(v)
    cols = sorted({c for k in vals for c in vals[k]})
    print("| kernel | grid | n | us | " + " | ".join(cols) + " | clk_GHz | mfma_busy | wait_any | wait_inst | active_inst |")
    print("|---|---|---|---|" + "---|" * (len(cols) + 5))
    for key in sorted(vals, key=lambda k: -sum(vals[k].get("SQ_WAVE_CYCLES", [0]))):
        cs = vals[key]
        mean = {c: sum(v) / len(v) for c, v in cs.items()}
        n = max(len(v) for v in cs.values())
        us = sorted(dur[key])[len(dur[key]) // 2] if dur[key] else float("nan")
        gui = mean.get("GRBM_GUI_ACTIVE", 0.0)
        clk = gui / 8 / (us * 1e3) if gui and us == us else float("nan")
        busy = mean.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (1024 * gui / 8) if gui else float("nan")
        wc = mean.get("SQ_WAVE_CYCLES", 0.0)
        sh = [mean.get(c, 0.0) / wc if wc else float("nan") for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY")]
        print(f"| {key[0]} | {key[1]} | {n} | {us:.1f} | " + " | ".join(f"{mean.get(c, 0):.4g}" for c in cols)
              + f" | {clk:.2f} | {busy:.3f} | {sh[0]:.3f} | {sh[1]:.3f} | {sh[2]:.3f} |")


if __name__ == "__main__":
    main(sys.argv[1:])
