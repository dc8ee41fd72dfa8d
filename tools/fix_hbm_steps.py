"""Rescale the launches/step and ms/step columns of an hbm_per_kernel table written with the
wrong step count (tools/final_profile.sh passed 4 while the traced bench ran 8 steps: warmup 1,
timed 3, one per-kernel timer step, 3 dominant-kernel timer steps).
usage: python tools/fix_hbm_steps.py <table.md> <factor>"""
import sys


def main(path, factor):
    f = float(factor)
    out = []
    for line in open(path):
        if line.startswith("| `"):
            c = line.rstrip("\n").split("|")
            # | kernel | grid | launches/step | avg us | fetch | write | GB/s | frac | ms/step |
            c[3] = f" {float(c[3]) * f:.1f} "
            c[9] = f" {float(c[9]) * f:.2f} "
            line = "|".join(c) + "\n"
        out.append(line)
    out.append(f"\nlaunches/step and ms/step rescaled by {factor} (the trace held 8 bench steps, the table "
               "had been divided by 4; tools/fix_hbm_steps.py).\n")
    open(path, "w").write("".join(out))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
