"""Per-launch conv time (kernel trace) and HBM bytes (FETCH_SIZE/WRITE_SIZE,
MI355X_MICROARCH.md §HBM correction: bytes = (2*FETCH + WRITE) * 1024) of the
last measured steps of tools/step_breakdown.py, mapped onto its launch list.

    python tools/conv_traffic.py OUTDIR [--top N]
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

out = sys.argv[1]
top = int(sys.argv[sys.argv.index("--top") + 1]) if "--top" in sys.argv else 40
L = json.load(open(os.path.join(out, "launches.json")))
launches, steps = L["launches"], L["steps"]
n = len(launches)


def rows(sub, pattern):
    r = []
    for f in sorted(glob.glob(os.path.join(out, sub, "**", pattern), recursive=True)):
        r.extend(csv.DictReader(open(f)))
    return r


def is_main(name):
    return ("conv_k" in name or "conv_h3" in name or "conv_wino" in name) and "reduce" not in name


def conv_dispatches(rs, key):
    """[(dispatch id, kernel name)] of conv main + reduce kernels in dispatch order."""
    seen = {}
    for r in rs:
        nm = r["Kernel_Name"]
        if "conv_" in nm and ("conv_k" in nm or "conv_h3" in nm or "conv_wino" in nm or "conv_reduce_k" in nm):
            seen[int(r[key])] = nm
    return sorted(seen.items())


def group(disp):
    """Group each main conv dispatch with a following split-K reduce; keep the
    last steps * n groups."""
    groups = []
    for did, nm in disp:
        if is_main(nm):
            groups.append([did])
        elif groups:
            groups[-1].append(did)
    return groups[-steps * n:]


trace = rows("trace", "*kernel_trace.csv")
dur = {int(r["Dispatch_Id"]): int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in trace}
tg = group(conv_dispatches(trace, "Dispatch_Id"))
ctr = {}
for sub, name in (("pmc_fetch", "FETCH_SIZE"), ("pmc_write", "WRITE_SIZE")):
    rs = [r for r in rows(sub, "*counter_collection.csv") if r["Counter_Name"] == name]
    per = defaultdict(float)
    for r in rs:
        per[int(r["Dispatch_Id"])] += float(r["Counter_Value"])
    g = group(conv_dispatches(rs, "Dispatch_Id"))
    ctr[name] = [sum(per[d] for d in grp) for grp in g]
assert len(tg) == steps * n, (len(tg), steps * n)
res = []
for k, l in enumerate(launches):
    t = sum(sum(dur[d] for d in tg[s * n + k]) for s in range(steps)) / steps / 1e3      # us
    f = sum(ctr["FETCH_SIZE"][s * n + k] for s in range(steps)) / steps
    w = sum(ctr["WRITE_SIZE"][s * n + k] for s in range(steps)) / steps
    by = (2 * f + w) * 1024
    res.append((t, by, l))
tot_t = sum(r[0] for r in res)
tot_b = sum(r[1] for r in res)
print("%-5s %5s %8s %5s %5s %4s %3s %8s %8s %7s %6s" % ("kind", "blk", "M", "N", "K", "tile", "ks", "us", "MB", "GB/s", "TF"))
for t, by, l in sorted(res, key=lambda r: -r[0])[:top]:
    print("%-5s %5d %8d %5d %5d %4d %3d %8.1f %8.1f %7.0f %6.1f" % (
        l["kind"], l["block"], l["M"], l["N"], l["K"], l["tile"], l["ksplit"], t, by / 1e6, by / t / 1e3,
        2 * l["macs"] / t / 1e6))
print("conv kernels: %.3f ms/step, %.2f GB/step HBM (%.0f GB/s avg), %d launches" % (
    tot_t / 1e3, tot_b / 1e9, tot_b / tot_t / 1e3, n))
json.dump({"conv_us_per_step": tot_t, "conv_hbm_bytes_per_step": tot_b,
           "launches": [{"us": t, "hbm_bytes": by, **l} for t, by, l in res]},
          open(os.path.join(out, "conv_traffic.json"), "w"))
