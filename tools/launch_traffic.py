"""Per-launch HBM counters of the bench's conv launches: aligns the FETCH_SIZE
/ WRITE_SIZE passes of tools/gpu_r03g.sh (kernel filter 'conv_') with the
launch dump (ADVPATCH_LAUNCH_DUMP: one step's po_conv launches in order; a
split-K launch is followed by its conv_reduce_k) and prints, per launch, the
raw counters (KiB) and HBM MB = (2*FETCH + WRITE) KiB (the gfx950 FETCH_SIZE
half count of 16-byte lane reads, MI355X_MICROARCH.md) beside its time.
    python tools/launch_traffic.py DUMP.jsonl FETCH_DIR WRITE_DIR [top]"""
import csv
import glob
import json
import sys
from collections import defaultdict

launches = [json.loads(l) for l in open(sys.argv[1])]
seq = []
for i, d in enumerate(launches):
    seq.append((i, "main"))
    if d["ksplit"] > 1:
        seq.append((i, "reduce"))


def counter(dirname, name):
    rows = []
    for f in glob.glob(dirname + "/**/*counter_collection.csv", recursive=True):
        rows += [r for r in csv.DictReader(open(f)) if r["Counter_Name"] == name]
    per = defaultdict(float)
    kname = {}
    for r in rows:
        per[int(r["Dispatch_Id"])] += float(r["Counter_Value"])
        kname[int(r["Dispatch_Id"])] = r["Kernel_Name"]
    ids = sorted(per)
    return [(per[i], kname[i]) for i in ids]


fetch, write = counter(sys.argv[2], "FETCH_SIZE"), counter(sys.argv[3], "WRITE_SIZE")
n = len(seq)
steps = len(fetch) // n
assert steps * n == len(fetch) == len(write), (len(fetch), len(write), n)
acc = defaultdict(lambda: [0.0, 0.0])
for s in range(steps):
    for k, (i, part) in enumerate(seq):
        f, kn = fetch[s * n + k]
        w, _ = write[s * n + k]
        assert (part == "reduce") == ("conv_reduce_k" in kn), (s, k, kn)
        acc[i][0] += f / steps
        acc[i][1] += w / steps
top = int(sys.argv[4]) if len(sys.argv) > 4 else 40
order = sorted(range(len(launches)), key=lambda i: -launches[i]["us"])
tot_mb = 0.0
for i in range(len(launches)):
    tot_mb += (2 * acc[i][0] + acc[i][1]) * 1024 / 1e6
print("launch  tile  shape                         us     FETCH KiB   WRITE KiB    HBM MB   GB/s")
for i in order[:top]:
    d = launches[i]
    mb = (2 * acc[i][0] + acc[i][1]) * 1024 / 1e6
    print("%4d  t%-3d %3dx%-3d Cin%-4d N%-4d tap%d st%d %8.1f %11.0f %11.0f %9.1f %6.0f" % (
        i, d["tile"], d["Hg"], d["Wg"], d["Cin_p"], d["N"], d["ntaps"], d["in_step"], d["us"], acc[i][0], acc[i][1],
        mb, mb / d["us"] * 1e3))
print("all launches: %.1f MB HBM per step (incl. split-K reduces)" % tot_mb)
