"""Measured HBM bytes and GB/s per kernel (the HBM-bound kernels vs the 8 TB/s peak).

  python tools/hbm_table.py <fetch_counter_collection.csv> <write_counter_collection.csv> \
      <kernel-trace results.db> <steps_in_trace> <out.md>

Bytes from two separate PMC passes (FETCH_SIZE, WRITE_SIZE; MI355X_MICROARCH.md "HBM": FETCH_SIZE
counts half the bytes of 16-B/lane streaming reads -> x2, both in KB -> x1024), averaged per
(kernel, grid); durations from a separate, unperturbed kernel trace of the same command."""
import collections
import sqlite3
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from pmc_summary import per_dispatch  # noqa: E402

PEAK = 8000.0  # GB/s


def key(name, grid):
    return name.split("(")[0].replace("void ", "")[:60], grid


def main(fetch_csv, write_csv, db, steps, out):
    steps = float(steps)
    fv, fn, fg = per_dispatch(fetch_csv, "FETCH_SIZE")
    wv, wn, wg = per_dispatch(write_csv, "WRITE_SIZE")
    fetch, write = collections.defaultdict(list), collections.defaultdict(list)
    for d, v in fv.items():
        fetch[key(fn[d], fg[d])].append(v * 1024 * 2)
    for d, v in wv.items():
        write[key(wn[d], wg[d])].append(v * 1024)
    dur = collections.defaultdict(list)
    con = sqlite3.connect(db)
    for name, gx, gy, gz, wx, wy, wz, d in con.execute(
            "select name, grid_x, grid_y, grid_z, workgroup_x, workgroup_y, workgroup_z, duration from kernels"):
        dur[key(name, gx * gy * gz)].append(d)
    rows = []
    for k, ds in dur.items():
        if k not in fetch or k not in write:
            continue
        t = sum(ds) / len(ds) * 1e-9
        fb = sum(fetch[k]) / len(fetch[k])
        wb = sum(write[k]) / len(write[k])
        gbs = (fb + wb) / t / 1e9
        rows.append((len(ds) / steps * t * 1e3, k, len(ds) / steps, t * 1e6, fb / 1e6, wb / 1e6, gbs))
    rows.sort(reverse=True)
    with open(out, "w") as f:
        f.write("| kernel | grid (threads) | launches/step | avg us | fetch MB | write MB | GB/s | of 8 TB/s | ms/step |\n")
        f.write("|---|---:|---:|---:|---:|---:|---:|---:|---:|\n")
        for ms, (name, grid), n, us, fb, wb, gbs in rows:
            f.write(f"| `{name}` | {grid} | {n:.1f} | {us:.1f} | {fb:.1f} | {wb:.1f} | {gbs:.0f} | "
                    f"{gbs / PEAK:.0%} | {ms:.2f} |\n")
    print(open(out).read())


if __name__ == "__main__":
    main(*sys.argv[1:6])
