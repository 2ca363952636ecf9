"""Where the non-po_* GPU time of a training step comes from: a few bench
steps (yolov3 B=16 by default) under torch.profiler with Python stacks; prints
the device kernels that are not this package's HIP kernels, grouped by the
innermost package source line that launched them.
Usage: python tools/torch_ops_profile.py [config] [batch] [steps]"""
import collections
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import __graft_entry__ as ge  # noqa: E402

cfg_name = sys.argv[1] if len(sys.argv) > 1 else "yolov3"
B = int(sys.argv[2]) if len(sys.argv) > 2 else None
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
tp, pc, sy, W = ge._pkg("train_patch"), ge._pkg("patch_config"), ge._pkg("synthetic"), ge._pkg("weights")
cfg, S, P, B0 = bench.CONFIGS[cfg_name]
B = B or B0
dev = torch.device("cuda", 0)
if cfg_name == "tiny":
    os.environ["ADVPATCH_TUNE_CACHE"] = os.path.join(ge.PKG_DIR, "tiles", "conv_tiles_tiny_b%d.json" % B)
W.ensure_synthetic(cfg, pc.synthetic_weights_path(cfg.split(":")[-1]))
tr = bench.build_trainer(tp, pc, W, cfg, B, 1, dev, "_bench" if cfg_name != "tiny" else "_bench_tiny")
img = sy.frames_slice(0, B, S, seed=1000).to(dev)
lab = sy.labels_slice(0, B, seed=2000).to(dev)
patch = sy.patch(P, seed=2).to(dev).requires_grad_(True)
opt = tr.make_optimizer(patch)
for _ in range(3):
    tr.step(patch, opt, img, lab)
torch.cuda.synchronize()
acts = [torch.profiler.ProfilerActivity.CPU, torch.profiler.ProfilerActivity.CUDA]
with torch.profiler.profile(activities=acts, with_stack=True) as prof:
    for _ in range(steps):
        tr.step(patch, opt, img, lab)
    torch.cuda.synchronize()

# CPU ops -> the device kernels they launched, located by the innermost
# package (or bench.py) frame of the op's Python stack (or of its parents')
agg = collections.defaultdict(lambda: [0, 0.0])
pkg = os.path.basename(ge.PKG_DIR)
for e in prof.events():
    ks = getattr(e, "kernels", None) or []
    if not ks:
        continue
    where, p = "?", e
    while p is not None:
        hit = [f for f in (getattr(p, "stack", None) or []) if pkg in f or "bench.py" in f]
        if hit:
            where = hit[0].split(pkg + "/")[-1]
            break
        p = getattr(p, "cpu_parent", None)
    for k in ks:
        key = (k.name[:60], e.name, where)
        agg[key][0] += 1
        agg[key][1] += k.duration
rows = sorted(agg.items(), key=lambda kv: -kv[1][1])
print("%-60s %-28s %-50s %6s %9s" % ("kernel", "op", "launched at", "n/step", "us/step"))
for (name, op, where), (n, us) in rows[:60]:
    print("%-60s %-28s %-50s %6.1f %9.1f" % (name, op[:28], where[:50], n / steps, us / steps))
