"""HBM bytes per launch for every kernel of a bench run, from two separate rocprofv3 PMC passes.

  python tools/kernel_traffic.py <fetch_counter_collection.csv> <write_counter_collection.csv> <out.json>

FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950 (TCC slots). MI355X_MICROARCH.md "HBM":
FETCH_SIZE counts half the bytes of a 16-B/lane streaming read (global_load_lds included) -> x2;
WRITE_SIZE is exact for 16-B streaming stores; both are in KB (x1024). The counters include
Infinity-Cache hits (memory-side L2 requests). Keys are rocprofv3 kernel names without the
argument list (what bench.py's roofline.kernel names); values are means over all dispatches of
that name in the pass."""
import json
import sys
from collections import defaultdict

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from pmc_summary import per_dispatch  # noqa: E402


def norm(name):
    return name.split("(")[0].replace("void ", "").strip()


def main(fetch_csv, write_csv, out):
    fv, fn, _ = per_dispatch(fetch_csv, "FETCH_SIZE")
    wv, wn, _ = per_dispatch(write_csv, "WRITE_SIZE")
    fetch, write = defaultdict(list), defaultdict(list)
    for d, v in fv.items():
        fetch[norm(fn[d])].append(2.0 * v * 1024.0)
    for d, v in wv.items():
        write[norm(wn[d])].append(v * 1024.0)
    res = {"correction": "FETCH_SIZE x2 (gfx950 wide streaming reads), KB x1024; means over dispatches",
           "bytes_per_launch": {}, "fetch_bytes": {}, "write_bytes": {}, "dispatches": {}}
    for k in sorted(set(fetch) & set(write)):
        f = sum(fetch[k]) / len(fetch[k])
        w = sum(write[k]) / len(write[k])
        res["fetch_bytes"][k] = f
        res["write_bytes"][k] = w
        res["bytes_per_launch"][k] = f + w
        res["dispatches"][k] = [len(fetch[k]), len(write[k])]
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    for k, v in sorted(res["bytes_per_launch"].items(), key=lambda kv: -kv[1])[:12]:
        print(f"{v / 1e6:10.1f} MB  {k}")


if __name__ == "__main__":
    main(*sys.argv[1:4])
