"""Summarise tools/pmc_conv.sh output: per-dispatch mean of every counter.
    python tools/pmc_read.py OUTDIR"""
import csv
import glob
import sys
from collections import defaultdict

import os

BY_KERNEL = os.environ.get("PMC_BY_KERNEL", "0") == "1"    # one block per kernel name (pmc_warp.sh)
tot = defaultdict(list)
for f in sorted(glob.glob(sys.argv[1] + "/p*/**/*counter_collection.csv", recursive=True)):
    per = defaultdict(float)
    for r in csv.DictReader(open(f)):
        kern = r.get("Kernel_Name", "").split("(")[0] if BY_KERNEL else ""
        per[(kern, r["Counter_Name"], r["Dispatch_Id"])] += float(r["Counter_Value"])
    for (k, c, _), v in per.items():
        tot[(k, c)].append(v)
if BY_KERNEL:
    for kern in sorted({k for k, _ in tot}):
        print("== %s" % kern)
        m = {c: sum(vs) / len(vs) for (k, c), vs in tot.items() if k == kern}
        for c in sorted(m):
            print("  %-28s %16.1f" % (c, m[c]))
        if "GRBM_GUI_ACTIVE" in m and "SQ_BUSY_CYCLES" in m:
            print("  %-28s %16.3f" % ("VALU insts per wave", m.get("SQ_INSTS_VALU", 0) / max(m.get("SQ_WAVES", 1), 1)))
        if "SQ_WAIT_INST_ANY" in m and "SQ_WAVE_CYCLES" in m:
            print("  %-28s %16.3f" % ("wait-inst / wave cycles", m["SQ_WAIT_INST_ANY"] / max(m["SQ_WAVE_CYCLES"], 1)))
        if "SQ_ACTIVE_INST_VALU" in m and "SQ_WAVE_CYCLES" in m:
            print("  %-28s %16.3f" % ("VALU-active / wave cycles", m["SQ_ACTIVE_INST_VALU"] / max(m["SQ_WAVE_CYCLES"], 1)))
    sys.exit(0)
tot = {c: vs for (_, c), vs in tot.items()}
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
