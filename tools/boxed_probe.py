"""Time every boxed (gradient-cone gbox) po_conv launch of the bench step on
the step's own cones, for a list of (tile, ksplit) candidates.

usage: python tools/boxed_probe.py [yolov3|tiny] [iters]
Prints, per boxed launch: shape, the cached choice and its time, live
workgroups of the cached tile, and every candidate's time (us)."""
import os
import sys
import json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import __graft_entry__ as ge
import bench

cfgname = sys.argv[1] if len(sys.argv) > 1 else "yolov3"
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 10
dev = torch.device("cuda", 0)
cfg, S, P, B = bench.CONFIGS[cfgname]
os.environ["ADVPATCH_TUNE_CACHE"] = os.path.join(ge.PKG_DIR, "tiles", "conv_tiles_%s_b%d.json" % (cfgname, B))
os.environ["ADVPATCH_TUNE"] = "cache"
tp, pc, sy, W = ge._pkg("train_patch"), ge._pkg("patch_config"), ge._pkg("synthetic"), ge._pkg("weights")
nat = ge._pkg("_native")
W.ensure_synthetic(cfg, pc.synthetic_weights_path(cfg.split(":")[-1]))
tr = bench.build_trainer(tp, pc, W, cfg, B, 1, dev, "_probe")
img = sy.frames_slice(0, B, S, seed=1000).to(dev)
lab = sy.labels_slice(0, B, seed=2000).to(dev)
patch = sy.patch(P, seed=2).to(dev).requires_grad_(True)
tr.darknet_model.conv_prec = "fp32"
opt = tr.make_optimizer(patch)
for _ in range(2):
    tr.step(patch, opt, img, lab)
torch.cuda.synchronize()
plan = tr.last_plan
cones = plan.cone_boxes.cpu() if plan.cone_boxes is not None else None
lib, st = plan.lib, nat.stream()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)


def timeit(args):
    if lib.po_conv(*args, st) != 0:
        return None
    e0.record()
    for _ in range(iters):
        lib.po_conv(*args, st)
    e1.record()
    e1.synchronize()
    return 1000.0 * e0.elapsed_time(e1) / iters


rows = []
for k, (name, args, desc) in enumerate(plan.bwd_ops):
    if name != "po_conv" or not desc.gbox:
        continue
    cur = (int(desc.tile), int(desc.ksplit))
    live = plan._live_tiles(desc, cur[0], plan.WINO_TILES.get(cur[0], plan.tile_shape(cur[0]))[0], cones)
    res = {"key": json.dumps(list(plan._tune_key(args, desc))),
           "k": k, "Hg": desc.Hg, "Cin_p": desc.Cin_p, "N": desc.N, "ntaps": desc.ntaps, "cur": cur,
           "live_wg": live, "mfma_flops": plan.launch_mfma_flops(desc, cones), "t": {}}
    if cur[0] in plan.WINO_TILES:
        cands = [(t, ks) for t in (66, 67, 68, 71, 72) for ks in (1, 2, 3, 4, 6, 8) if desc.Cin_p // 16 // ks >= 2]
    else:
        cands = [(t, ks) for t in (3, 5, 7, 9, 13, 15, 17, 19) for ks in (1, 2, 4, 8, 12, 16)
                 if desc.ntaps * desc.Cin_p // plan.tile_shape(t)[2] // ks >= 2]
        if desc.ntaps == 9 and os.environ.get("PROBE_WINO_ON_DIRECT"):
            # a direct-tile 3x3 launch: the Winograd tiles too (refused ones time as None)
            cands += [(t, ks) for t in (66, 67, 68, 71, 72) for ks in (1, 2, 4, 8, 16) if desc.Cin_p // 16 // ks >= 2]
    if cur not in cands:
        cands.append(cur)
    for c in cands:
        plan._set_tile(desc, c)
        t = timeit(args)
        if t is not None:
            res["t"]["%d/%d" % c] = round(t, 1)
    plan._set_tile(desc, cur)
    best = min(res["t"].items(), key=lambda kv: kv[1])
    print("k=%3d %3d^2 Cin%4d N%4d tap%d cur %s %.1f us  live_wg %d  best %s %.1f us" % (
        k, desc.Hg, desc.Cin_p, desc.N, desc.ntaps, "%d/%d" % cur, res["t"].get("%d/%d" % cur, -1), live,
        best[0], best[1]), flush=True)
    if os.environ.get("PROBE_VERBOSE"):
        print("   ", json.dumps(res["t"]), flush=True)
    rows.append(res)
tot_cur = sum(r["t"].get("%d/%d" % r["cur"], 0) for r in rows)
tot_best = sum(min(r["t"].values()) for r in rows)
print("boxed launches: %d, cached %.1f us, per-launch best %.1f us" % (len(rows), tot_cur, tot_best))
out = os.environ.get("PROBE_OUT")
if out:
    with open(out, "w") as f:
        for r in rows:
            r["cur"] = "%d/%d" % r["cur"]
            f.write(json.dumps(r) + "\n")

wr = os.environ.get("PROBE_WRITE")
if wr:
    # per cache key (launches of one signature share a choice): the candidate
    # with the least summed time over those launches, kept where it beats the
    # cached choice by >= 3 %; the updated cache goes to PROBE_WRITE
    cache = json.load(open(os.environ["ADVPATCH_TUNE_CACHE"]))
    by = {}
    for r in rows:
        by.setdefault(r["key"], []).append(r)
    changed = 0
    for key, rs in by.items():
        curs = {r["cur"] if isinstance(r["cur"], str) else "%d/%d" % r["cur"] for r in rs}
        common = set.intersection(*(set(r["t"]) for r in rs))
        if len(curs) != 1 or not common or key not in cache:
            continue
        cur = next(iter(curs))
        tot = {c: sum(r["t"][c] for r in rs) for c in common}
        best = min(tot, key=tot.get)
        if cur in tot and tot[best] <= 0.97 * tot[cur]:
            t, ks = (int(v) for v in best.split("/"))
            print("key %s: %s %.1f us -> %s %.1f us over %d launches" % (key, cur, tot[cur], best, tot[best], len(rs)))
            cache[key] = [t, ks]
            changed += 1
    with open(wr, "w") as f:
        json.dump(cache, f)
    print("updated %d cache entries -> %s" % (changed, wr))
