"""Per-kernel roofline table from one round's profile files (no GPU needed):
  * bench line `kernels` (HIP events on the launch stream around every launch of each GEMM /
    attention class in one step: ms per step and algorithmic TFLOP/s, SURVEY 8(d) FLOPs),
  * rocprofv3 --stats table (average duration per launch of the same kernels),
  * the SQ counter pass (MFMA-busy fraction per kernel).
usage: python tools/kernel_frac_table.py profiles/r02c > profiles/r02c_kernel_frac.md"""
import json
import re
import sys

PEAK = 2500.0  # TFLOP/s, dense bf16 (MI355X_MICROARCH.md)


def rows(md):
    out = []
    for line in open(md):
        if not line.startswith("| ") or line.startswith("| kernel") or line.startswith("|---"):
            continue
        out.append([c.strip().strip("`") for c in line.strip().strip("|").split("|")])
    return out


def short(name):
    return re.sub(r"\(ltx::(GemmParams|AttnParams)\)|void |ltx::", "", name).strip()


def main(prefix):
    line = open(prefix + "_bench.json").read().strip().splitlines()[-1]
    bench = json.loads(line)
    stats = rows(prefix + "_kernel_stats.md")  # kernel | calls | total ms | avg us | %
    pmc = rows(prefix + "_pmc_sq.md")          # kernel | grid | n | us | ... | mfma_busy | ...
    hdr = [h.strip() for h in open(prefix + "_pmc_sq.md").readline().strip().strip("|").split("|")]
    ib = hdr.index("mfma_busy")

    def find(tab, key, col):
        best = None
        for r in tab:
            if key in short(r[0]):
                v = float(r[col])
                best = v if best is None else max(best, v) if col == 2 else best
                if col != 2:
                    return v
        return best

    print("| kernel class (bench.py live timer) | launches / step | ms / step | TF/s (algorithmic) "
          "| frac of 2.5 PF | rocprof avg us | MFMA-busy (SQ counters) |")
    print("|---|---:|---:|---:|---:|---:|---:|")
    for k in bench["kernels"]:
        name = k["kernel"]
        # the rocprof / counter rows of the first kernel the class names
        m = re.search(r"(gemm_(?:nt_kernel_t|ring_kernel)<[^>]*>|attn_\w+_kernel<[^>]*>)", name)
        key = short(m.group(1)).replace(">", "") if m else short(name)
        key = key.split("<")[0] + "<" + key.split("<")[1] if "<" in key else key
        avg = find(stats, key, 3)
        busy = find(pmc, key, ib)
        print(f"| `{short(name)}` | {k['launches_per_step']} | {k['ms_per_step']:.2f} | {k['tflops']:.0f} "
              f"| {k['frac']:.3f} | {avg if avg is not None else '-'} | "
              f"{busy if busy is not None else '-'} |")
    r = bench["roofline"]
    print()
    print(f"Dominant class (the bench line's `roofline`): `{short(r['kernel'])}`, {r['launches']} launches "
          f"timed, {r['launch_ms'] * 1e3:.1f} us per launch, {r['achieved']:.0f} TF/s = {r['frac']:.3f} of "
          f"{PEAK:.0f}; step {bench['ms_per_step']:.1f} ms = {bench['value']:.2f} samples/s "
          f"({bench['step_mfma_frac']:.3f} of peak over the whole step).")


if __name__ == "__main__":
    main(sys.argv[1])
