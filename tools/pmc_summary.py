"""Summarise rocprofv3 outputs into the committed profiles/ files.

  python tools/pmc_summary.py stats  <kernel_stats.csv> <out.md>
      per-kernel totals of a `rocprofv3 --kernel-trace --stats` run as a markdown table.
  python tools/pmc_summary.py traffic <fetch_counter_collection.csv> <write_counter_collection.csv> <out.json>
      HBM bytes per launch of the dominant kernel (the FF-up GEMM with the GELU epilogue,
      14336x8192 output) from two separate PMC passes (FETCH_SIZE and WRITE_SIZE cannot
      share a pass on gfx950). MI355X_MICROARCH.md "HBM": FETCH_SIZE counts half the bytes of a
      16-B/lane streaming read (global_load_lds included) -> doubled; WRITE_SIZE is exact for
      16-B streaming stores. Both are reported in KB by rocprofv3 (x1024).
"""
import csv
import json
import sys
from collections import defaultdict

# the FF-up GELU GEMM (14336 x 8192 output, 256-row tiles): ceil(14336/256) * ceil(8192/256)
# workgroups of 256 threads (gemm_ring_kernel, the default) or 512 (gemm_nt_kernel_t)
DOM = (("gemm_ring_kernel<1", 56 * 32 * 256), ("gemm_nt_kernel_t<1", 56 * 32 * 512))


def _rows(path):
    with open(path, newline="") as f:
        yield from csv.DictReader(f)


def per_dispatch(path, counter):
    vals = defaultdict(float)
    names, grids = {}, {}
    for r in _rows(path):
        if r.get("Counter_Name") != counter:
            continue
        d = r["Dispatch_Id"]
        vals[d] += float(r["Counter_Value"])
        names[d] = r["Kernel_Name"]
        grids[d] = int(r.get("Grid_Size", 0) or 0)
    return vals, names, grids


def dominant(path, counter):
    vals, names, grids = per_dispatch(path, counter)
    sel = [v for d, v in vals.items() if any(m in names[d] and grids[d] == g for m, g in DOM)]
    if not sel:
        raise SystemExit(f"no dominant-kernel dispatches with {counter} in {path}")
    return sum(sel) / len(sel), len(sel)


def traffic(fetch_csv, write_csv, out):
    fetch_kb, nf = dominant(fetch_csv, "FETCH_SIZE")
    write_kb, nw = dominant(write_csv, "WRITE_SIZE")
    fetch = 2.0 * fetch_kb * 1024.0
    write = write_kb * 1024.0
    M, N, K = 14336, 8192, 2048
    algo = 2 * (M * K + N * K) + 2 * 2 * M * N  # A, W read once; activation + pre-activation stored
    res = {"kernel": "FF-up GELU GEMM (256-row tiles) [14336x2048].[8192x2048]^T (+pre-activation store)",
           "dispatches_fetch": nf, "dispatches_write": nw,
           "fetch_size_kb_raw": fetch_kb, "write_size_kb_raw": write_kb,
           "fetch_bytes_corrected": fetch, "write_bytes": write,
           "hbm_bytes_per_launch": fetch + write, "algorithmic_bytes_per_launch": algo,
           "traffic_over_algorithmic": (fetch + write) / algo,
           "correction": "FETCH_SIZE x2 (gfx950 wide streaming reads), KB x1024"}
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


def stats(path, out):
    rows = list(_rows(path))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
    lines = ["| kernel | calls | total ms | avg us | % |", "|---|---:|---:|---:|---:|"]
    for r in rows[:40]:
        name = r["Name"].replace("|", "/")
        if len(name) > 110:
            name = name[:107] + "..."
        t = float(r["TotalDurationNs"])
        lines.append(f"| `{name}` | {r['Calls']} | {t / 1e6:.2f} | {float(r['AverageNs']) / 1e3:.1f} | "
                     f"{100 * t / tot:.1f} |")
    with open(out, "w") as f:
        f.write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    if sys.argv[1] == "stats":
        stats(sys.argv[2], sys.argv[3])
    elif sys.argv[1] == "traffic":
        traffic(sys.argv[2], sys.argv[3], sys.argv[4])
    else:
        raise SystemExit(__doc__)
