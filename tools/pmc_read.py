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
