"""Summarise tools/pmc_conv.sh output: per-dispatch mean of every counter.
    python tools/pmc_read.py OUTDIR"""
import csv
import glob
import sys
from collections import defaultdict

tot = defaultdict(list)
for f in sorted(glob.glob(sys.argv[1] + "/p*/**/*counter_collection.csv", recursive=True)):
    per = defaultdict(float)
    for r in csv.DictReader(open(f)):
        per[(r["Counter_Name"], r["Dispatch_Id"])] += float(r["Counter_Value"])
    for (c, _), v in per.items():
        tot[c].append(v)
for c, vs in sorted(tot.items()):
    print("%-28s %16.1f  (n=%d)" % (c, sum(vs) / len(vs), len(vs)))

# derived figures (MI355X: 1024 SIMDs; GRBM_GUI_ACTIVE sums the 8 XCDs)
m = {c: sum(vs) / len(vs) for c, vs in tot.items()}
if "SQ_VALU_MFMA_BUSY_CYCLES" in m and "GRBM_GUI_ACTIVE" in m:
    print("MFMA busy                    %16.3f" % (m["SQ_VALU_MFMA_BUSY_CYCLES"] / (m["GRBM_GUI_ACTIVE"] / 8 * 1024)))
if "SQ_INSTS_MFMA" in m and m["SQ_INSTS_MFMA"]:
    for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD"):
        if c in m:
            print("%-28s %16.2f" % (c.replace("SQ_INSTS_", "") + " per MFMA", m[c] / m["SQ_INSTS_MFMA"]))
