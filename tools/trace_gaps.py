"""Kernel timeline of one training step from a rocprofv3 --kernel-trace CSV:
per dispatch its duration and the idle gap before it, summed per step, so a
host-launch-bound stretch (gaps comparable to the kernels) shows up.
Usage: python tools/trace_gaps.py run_kernel_trace.csv [first-kernel-regex]
The step boundary is the first kernel matching the regex (default patch_params)."""
import csv
import re
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
pat = re.compile(sys.argv[2] if len(sys.argv) > 2 else "patch_params")
starts = [i for i, r in enumerate(rows) if pat.search(r["Kernel_Name"])]
if len(starts) < 3:
    sys.exit("fewer than 3 steps in the trace")
a, b = starts[-3], starts[-2]            # a whole step well inside the timed region
busy = gap = 0
print("%-60s %9s %9s" % ("kernel", "dur_us", "gap_us"))
prev_end = int(rows[a]["Start_Timestamp"])
for r in rows[a:b]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    g = max(0, s - prev_end)
    busy += e - s
    gap += g
    print("%-60s %9.1f %9.1f" % (r["Kernel_Name"].split("(")[0][-60:], (e - s) / 1e3, g / 1e3))
    prev_end = max(prev_end, e)
print("step: %d dispatches, busy %.3f ms, idle gaps %.3f ms, span %.3f ms" % (
    b - a, busy / 1e6, gap / 1e6, (int(rows[b]["Start_Timestamp"]) - int(rows[a]["Start_Timestamp"])) / 1e6))
