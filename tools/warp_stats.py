"""Per-kernel averages of the warp kernels in rocprofv3 --stats CSVs.
Usage: python tools/warp_stats.py DIR [DIR ...] (each holding run_kernel_stats.csv)"""
import csv
import os
import sys

for d in sys.argv[1:]:
    print(d)
    for x in csv.DictReader(open(os.path.join(d, "run_kernel_stats.csv"))):
        if any(k in x["Name"] for k in ("warp", "patch_params", "conv_first")):
            print("  %-70s %5s %9.1f us" % (x["Name"][:70], x["Calls"], float(x["AverageNs"]) / 1e3))
