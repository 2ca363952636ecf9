"""Summarise a tools/profile_round.sh output directory into profiles/.

Inputs: rocprofv3 csv output (kernel trace + stats, and the FETCH_SIZE and
WRITE_SIZE counter passes) of `bench.py` with D = steps + warmup identical
steps and no tuning launches.  Per kernel family (template arguments
stripped) it writes calls per step, mean duration, time per step and HBM
bytes per step.

HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE are in
KiB; on gfx950 FETCH_SIZE reports half the bytes of wide (16 B/lane)
coalesced reads, which is what every hot kernel here issues, so
    hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024.

usage: python tools/pmc_summary.py OUTDIR ROUND CONFIG BATCH NSTEPS [PREC]
"""
import csv
import glob
import json
import os
import re
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def family(name):
    n = re.sub(r"^void\s+", "", name.strip()).replace("(anonymous namespace)::", "")
    n = re.split(r"[<(]", n)[0]
    return n.split("::")[-1].strip() or name


def rows(pattern, d):
    out = []
    for f in sorted(glob.glob(os.path.join(d, "**", pattern), recursive=True)):
        with open(f) as fh:
            out.extend(csv.DictReader(fh))
    return out


def main():
    outdir, rnd, cfg, batch, nsteps = sys.argv[1], sys.argv[2], sys.argv[3], int(sys.argv[4]), int(sys.argv[5])
    prec = sys.argv[6] if len(sys.argv) > 6 else "fp16x3"
    trace = rows("*kernel_trace.csv", os.path.join(outdir, "trace"))
    if not trace:
        raise SystemExit("no kernel trace under %s" % outdir)
    dur = defaultdict(list)
    for r in trace:
        dur[family(r["Kernel_Name"])].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    pmc = defaultdict(float)
    for sub, ctr in (("pmc_fetch", "FETCH_SIZE"), ("pmc_write", "WRITE_SIZE")):
        for r in rows("*counter_collection.csv", os.path.join(outdir, sub)):
            if r.get("Counter_Name") == ctr:
                pmc[(family(r["Kernel_Name"]), ctr)] += float(r["Counter_Value"])
    fams = sorted(dur, key=lambda k: -sum(dur[k]))
    table = {}
    for k in fams:
        calls = len(dur[k])
        fetch = pmc.get((k, "FETCH_SIZE"))
        write = pmc.get((k, "WRITE_SIZE"))
        hbm = None if fetch is None or write is None else (2.0 * fetch + write) * 1024.0 / nsteps
        ms = sum(dur[k]) / 1e6 / nsteps
        table[k] = {"calls_per_step": calls / nsteps, "mean_us": sum(dur[k]) / calls / 1e3, "ms_per_step": ms,
                    "hbm_bytes_per_step": hbm,
                    "fetch_size_kib_per_step": None if fetch is None else fetch / nsteps,
                    "write_size_kib_per_step": None if write is None else write / nsteps,
                    "hbm_GBps": None if hbm is None or ms == 0 else hbm / (ms * 1e-3) / 1e9}
    pdir = os.path.join(ROOT, "profiles", rnd)
    os.makedirs(pdir, exist_ok=True)
    tag = "%s_b%d_%s" % (cfg, batch, prec)
    for f in glob.glob(os.path.join(outdir, "trace", "**", "*kernel_stats.csv"), recursive=True):
        shutil.copy(f, os.path.join(pdir, "kernel_stats_%s.csv" % tag))
    lines = ["# rocprofv3 summary, %s, bench.py --config %s --batch %d (%d identical steps incl. warm-up)" %
             (rnd, cfg, batch, nsteps), "",
             "Commands: `tools/profile_round.sh %s %s %d` (kernel trace + stats; FETCH_SIZE and WRITE_SIZE passes)."
             % (rnd, cfg, batch),
             "HBM bytes = (2*FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950 FETCH_SIZE half-count correction, "
             "MI355X_MICROARCH.md §HBM).", "",
             "| kernel family | calls/step | mean us | ms/step | HBM MB/step | HBM GB/s |", "|---|---|---|---|---|---|"]
    for k in fams:
        t = table[k]
        mb = "-" if t["hbm_bytes_per_step"] is None else "%.1f" % (t["hbm_bytes_per_step"] / 1e6)
        gb = "-" if t["hbm_GBps"] is None else "%.0f" % t["hbm_GBps"]
        lines.append("| %s | %.2f | %.1f | %.3f | %s | %s |" % (k, t["calls_per_step"], t["mean_us"], t["ms_per_step"],
                                                               mb, gb))
    tot = sum(t["ms_per_step"] for t in table.values())
    lines += ["", "GPU kernel time per step: %.3f ms" % tot]
    for f in ("bench_plain.json", "bench_trace.json"):
        p = os.path.join(outdir, f)
        if os.path.exists(p):
            txt = [l for l in open(p).read().splitlines() if l.startswith("{")]
            if txt:
                lines += ["", "%s:" % f, "```", txt[-1], "```"]
    with open(os.path.join(pdir, "summary_%s.md" % tag), "w") as fh:
        fh.write("\n".join(lines) + "\n")
    conv = [table[k] for k in table if k.startswith("conv_") and k.endswith("_k")]
    hb = [t["hbm_bytes_per_step"] for t in conv]
    with open(os.path.join(ROOT, "profiles", "traffic_%s.json" % tag), "w") as fh:
        json.dump({"round": rnd, "prec": prec,
                   "kernel": "po_conv launches of one step (conv_k / conv_h3*_k tile families + split-K reduce)",
                   "conv_hbm_bytes_per_step": None if None in hb else sum(hb),
                   "conv_ms_per_step": sum(t["ms_per_step"] for t in conv),
                   "conv_calls_per_step": sum(t["calls_per_step"] for t in conv),
                   "families": table}, fh, indent=1)
    print("\n".join(lines))


if __name__ == "__main__":
    main()
