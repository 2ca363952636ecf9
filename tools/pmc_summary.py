"""Summarise a tools/profile_round.sh output directory into profiles/, in
steady state.

Inputs: rocprofv3 csv output of the same bench command at K=5 and K=25 timed
steps (kernel trace + stats, and the FETCH_SIZE and WRITE_SIZE counter
passes).  Every quantity is the K=25 run minus the K=5 run, divided by the
2*20 steps between them (bench.py runs each timed step twice: plain and
instrumented), so the one-time work of a run -- weight transforms, the
float64 Winograd weights' hipBLASLt GEMMs, plan build, warm-up -- cancels and
the per-step totals are those of the step itself.  Per kernel family
(template arguments stripped): launches per step, mean duration, time per
step and HBM bytes per step.

HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE are in
KiB; on gfx950 FETCH_SIZE reports half the bytes of wide (16 B/lane)
coalesced reads, which is what every hot kernel here issues, so
    hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024.

usage: python tools/pmc_summary.py OUTDIR ROUND CONFIG BATCH [PREC]
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
NSTEPS = 2 * (25 - 5)


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


def bench_line(path):
    if not os.path.exists(path):
        return None
    txt = [l for l in open(path).read().splitlines() if l.startswith("{")]
    return json.loads(txt[-1]) if txt else None


def main():
    outdir, rnd, cfg, batch = sys.argv[1], sys.argv[2], sys.argv[3], int(sys.argv[4])
    prec = sys.argv[5] if len(sys.argv) > 5 else "fp32"
    calls, ns = defaultdict(float), defaultdict(float)
    for sign, k in ((-1, 5), (1, 25)):
        tr = rows("*kernel_trace.csv", os.path.join(outdir, "trace_k%d" % k))
        if not tr:
            raise SystemExit("no kernel trace under %s/trace_k%d" % (outdir, k))
        for r in tr:
            f = family(r["Kernel_Name"])
            calls[f] += sign
            ns[f] += sign * (int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    pmc = defaultdict(float)
    have = {}
    for sub, ctr in (("fetch", "FETCH_SIZE"), ("write", "WRITE_SIZE")):
        for sign, k in ((-1, 5), (1, 25)):
            rr = rows("*counter_collection.csv", os.path.join(outdir, "%s_k%d" % (sub, k)))
            have[(sub, k)] = bool(rr)
            for r in rr:
                if r.get("Counter_Name") == ctr:
                    pmc[(family(r["Kernel_Name"]), ctr)] += sign * float(r["Counter_Value"])
    counters = all(have.values())
    fams = sorted((f for f in calls if calls[f] > 0.5 or ns[f] > 0), key=lambda f: -ns[f])
    table = {}
    for f in fams:
        c = calls[f] / NSTEPS
        ms = ns[f] / 1e6 / NSTEPS
        fetch, write = pmc.get((f, "FETCH_SIZE")), pmc.get((f, "WRITE_SIZE"))
        hbm = (2.0 * fetch + write) * 1024.0 / NSTEPS if counters and fetch is not None and write is not None else None
        table[f] = {"calls_per_step": c, "mean_us": (ns[f] / calls[f] / 1e3) if calls[f] > 0 else None,
                    "ms_per_step": ms, "hbm_bytes_per_step": hbm,
                    "fetch_size_kib_per_step": None if fetch is None else fetch / NSTEPS,
                    "write_size_kib_per_step": None if write is None else write / NSTEPS,
                    "hbm_GBps": None if hbm is None or ms <= 0 else hbm / (ms * 1e-3) / 1e9}
    pdir = os.path.join(ROOT, "profiles", rnd)
    os.makedirs(pdir, exist_ok=True)
    tag = "%s_b%d_%s" % (cfg, batch, prec)
    for f in glob.glob(os.path.join(outdir, "trace_k25", "**", "*kernel_stats.csv"), recursive=True):
        shutil.copy(f, os.path.join(pdir, "kernel_stats_%s_k25.csv" % tag))
    wall = bench_line(os.path.join(outdir, "bench_trace_k25.json"))
    lines = ["# rocprofv3 summary, %s, bench.py --config %s --batch %d --prec %s: steady state" % (rnd, cfg, batch, prec),
             "",
             "Commands: `tools/profile_round.sh %s %s %d %s` (kernel trace + stats, FETCH_SIZE and WRITE_SIZE passes, "
             "each at K=5 and K=25 timed steps); per step = (K=25 run - K=5 run) / %d steps, so one-time launches "
             "(weight transforms, plan build, warm-up) cancel." % (rnd, cfg, batch, prec, NSTEPS),
             "HBM bytes = (2*FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950 FETCH_SIZE half-count correction, "
             "MI355X_MICROARCH.md §HBM).", "",
             "| kernel family | launches/step | mean us | ms/step | HBM MB/step | HBM GB/s |", "|---|---|---|---|---|---|"]
    for f in fams:
        t = table[f]
        mb = "-" if t["hbm_bytes_per_step"] is None else "%.1f" % (t["hbm_bytes_per_step"] / 1e6)
        gb = "-" if t["hbm_GBps"] is None else "%.0f" % t["hbm_GBps"]
        mu = "-" if t["mean_us"] is None else "%.1f" % t["mean_us"]
        lines.append("| %s | %.2f | %s | %.3f | %s | %s |" % (f, t["calls_per_step"], mu, t["ms_per_step"], mb, gb))
    tot = sum(t["ms_per_step"] for t in table.values())
    lines += ["", "GPU kernel time per step (steady state): %.3f ms" % tot]
    if wall is not None:
        # the 2*20 differenced steps are 20 plain ones (ms_per_step) and 20 with
        # per-launch HIP events (roofline.measured_on): compare with their mean
        import re
        plain = wall["ms_per_step"]
        m = re.search(r"\(([0-9.]+) ms/step instrumented", wall.get("roofline", {}).get("measured_on", ""))
        both = (plain + float(m.group(1))) / 2 if m else plain
        lines += ["Wall time per step of the same run (bench.py `ms_per_step`, profiler attached): %.3f ms plain; "
                  "%.3f ms averaged with the instrumented pass the difference also spans" % (plain, both)]
        if tot > both * 1.005:
            lines += ["WARNING: the kernel total exceeds the wall step (the difference did not cancel the setup)."]
        lines += ["", "bench_trace_k25.json:", "```", json.dumps(wall), "```"]
    with open(os.path.join(pdir, "summary_%s.md" % tag), "w") as fh:
        fh.write("\n".join(lines) + "\n")
    conv = [table[k] for k in table if k.startswith("conv_") and k.endswith("_k")]
    hb = [t["hbm_bytes_per_step"] for t in conv]
    with open(os.path.join(ROOT, "profiles", "traffic_%s.json" % tag), "w") as fh:
        json.dump({"round": rnd, "prec": prec, "steady_state": True,
                   "kernel": "po_conv launches of one step (conv_* tile families + split-K reduce)",
                   "conv_hbm_bytes_per_step": None if (not hb or None in hb) else sum(hb),
                   "conv_ms_per_step": sum(t["ms_per_step"] for t in conv),
                   "conv_calls_per_step": sum(t["calls_per_step"] for t in conv),
                   "families": table}, fh, indent=1)
    print("\n".join(lines))


if __name__ == "__main__":
    main()
