"""Matrix-core busy ratio of the conv kernels from tools/pmc_mfma_bench.sh:
per kernel family, SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 1024
SIMDs) — GRBM_GUI_ACTIVE sums the 8 XCDs' busy clocks, so /8 is the
dispatch's length in (actual, DVFS-lowered) clocks — and the MFMA FLOPs the
counters imply (SQ_INSTS_MFMA x 32x32x2 x 2: every conv MFMA is
v_mfma_f32_32x32x2_f32).  The bench's frac_mfma prices the same MFMA work
against 157.3 TFLOP/s at 2.4 GHz, so the two agree when the clock holds 2.4
GHz and frac_mfma reads lower by f/2.4 GHz when it does not.
    python tools/pmc_mfma_summary.py OUTDIR"""
import csv
import glob
import sys
from collections import defaultdict

per = defaultdict(lambda: defaultdict(float))      # dispatch -> counter -> value
name = {}
for f in glob.glob(sys.argv[1] + "/pmc/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        d = r["Dispatch_Id"]
        per[d][r["Counter_Name"]] += float(r["Counter_Value"])
        name[d] = r["Kernel_Name"]


def family(k):
    for f in ("conv_wino4_k", "conv_wino3_k", "conv_wino2_k", "conv_wino_k", "conv_reduce_k", "conv_h3", "conv_k"):
        if f in k:
            return f
    return k[:40]


fam = defaultdict(lambda: defaultdict(float))
for d, c in per.items():
    f = fam[family(name[d])]
    f["n"] += 1
    for k, v in c.items():
        f[k] += v
tot = defaultdict(float)
print("%-16s %6s %14s %14s %9s %12s" % ("family", "disp", "MFMA insts", "busy cycles", "busy", "MFMA GFLOP"))
for k, f in sorted(fam.items(), key=lambda kv: -kv[1]["GRBM_GUI_ACTIVE"]):
    clocks = f["GRBM_GUI_ACTIVE"] / 8.0
    busy = f["SQ_VALU_MFMA_BUSY_CYCLES"] / (clocks * 1024.0) if clocks else 0.0
    print("%-16s %6d %14.0f %14.0f %9.3f %12.1f" % (k, f["n"], f["SQ_INSTS_MFMA"], f["SQ_VALU_MFMA_BUSY_CYCLES"],
                                                   busy, f["SQ_INSTS_MFMA"] * 4096 / 1e9))
    for key in ("SQ_INSTS_MFMA", "SQ_VALU_MFMA_BUSY_CYCLES", "GRBM_GUI_ACTIVE", "n"):
        tot[key] += f[key]
clocks = tot["GRBM_GUI_ACTIVE"] / 8.0
print("%-16s %6d %14.0f %14.0f %9.3f %12.1f" % ("all conv", tot["n"], tot["SQ_INSTS_MFMA"],
                                               tot["SQ_VALU_MFMA_BUSY_CYCLES"],
                                               tot["SQ_VALU_MFMA_BUSY_CYCLES"] / (clocks * 1024.0) if clocks else 0,
                                               tot["SQ_INSTS_MFMA"] * 4096 / 1e9))
print("busy cycles per MFMA instruction: %.1f" % (tot["SQ_VALU_MFMA_BUSY_CYCLES"] / max(tot["SQ_INSTS_MFMA"], 1)))
