"""Steady-state launch census from tools/launch_census.sh output.

Per kernel family: launches and time per step from the difference of the
K=25 and K=5 kernel traces (2*20 steps: bench.py times every step twice),
split into the package's own HIP kernels (the __global__ names under csrc/)
and everything else (PyTorch / rocclr / hipBLASLt).  Then the launch sequence
of the last complete step of the K=25 trace, each non-HIP launch shown with
the package kernel before it, which names the call site.

usage: python tools/launch_census.py OUTDIR [STEP_MARKER]   (default marker: the first-layer forward kernel)
"""
import csv
import glob
import os
import re
import sys
from collections import Counter, defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = "adversarial_patch-based_false_positive_creation_attacks_against_aerial_imagery_object_detectors_amd"


def family(name):
    n = re.sub(r"^void\s+", "", name.strip()).replace("(anonymous namespace)::", "")
    n = re.split(r"[<(]", n)[0]
    return n.split("::")[-1].strip() or name


def own_kernels():
    names = set()
    for f in glob.glob(os.path.join(ROOT, PKG, "csrc", "*.hip")) + glob.glob(os.path.join(ROOT, PKG, "csrc", "*.h")):
        names.update(re.findall(r"__global__\s+(?:__launch_bounds__\([^)]*\)\s+)?void\s+(\w+)", open(f).read()))
    return names


def trace(d):
    out = []
    for f in sorted(glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)):
        with open(f) as fh:
            out.extend(csv.DictReader(fh))
    out.sort(key=lambda r: int(r["Start_Timestamp"]))
    return out


def main():
    outdir = sys.argv[1]
    marker = sys.argv[2] if len(sys.argv) > 2 else "first_fwd2_k"
    own = own_kernels()
    t5, t25 = trace(os.path.join(outdir, "k5")), trace(os.path.join(outdir, "k25"))
    if not t5 or not t25:
        raise SystemExit("missing k5/k25 traces under %s" % outdir)
    nsteps = 2 * 20
    cnt, ns = defaultdict(float), defaultdict(float)
    for sign, tr in ((-1, t5), (1, t25)):
        for r in tr:
            k = family(r["Kernel_Name"])
            cnt[k] += sign
            ns[k] += sign * (int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    lines = ["| kernel family | own HIP | launches/step | us/step |", "|---|---|---|---|"]
    tot = {True: [0.0, 0.0], False: [0.0, 0.0]}
    for k in sorted(cnt, key=lambda k: (k not in own, -ns[k])):
        c, u = cnt[k] / nsteps, ns[k] / nsteps / 1e3
        if abs(c) < 0.01 and abs(u) < 0.5:
            continue
        lines.append("| %s | %s | %.2f | %.1f |" % (k[:90], "yes" if k in own else "no", c, u))
        tot[k in own][0] += c
        tot[k in own][1] += u
    lines += ["", "own HIP launches/step: %.1f (%.3f ms); other launches/step: %.1f (%.3f ms)" %
              (tot[True][0], tot[True][1] / 1e3, tot[False][0], tot[False][1] / 1e3)]
    idx = [i for i, r in enumerate(t25) if family(r["Kernel_Name"]) == marker]
    if len(idx) >= 2:
        seq = t25[idx[-2]:idx[-1]]
        lines += ["", "last complete step (%d launches, from %s): non-HIP launches after the preceding own kernel" %
                  (len(seq), marker)]
        prev, runs = "(step start)", Counter()
        for r in seq:
            k = family(r["Kernel_Name"])
            if k in own:
                prev = k
            else:
                runs[(prev, k[:60])] += 1
        for (p, k), n in runs.items():
            lines.append("  after %-28s %3d x %s" % (p, n, k))
    print("\n".join(lines))


if __name__ == "__main__":
    main()
