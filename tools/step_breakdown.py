"""Per-launch conv timing of the bench step (HIP events around every po_conv).

    python tools/step_breakdown.py [--config yolov3] [--batch 16] [--steps 5] [--windows 1]
"""
import argparse
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402
import __graft_entry__ as ge  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="yolov3")
ap.add_argument("--batch", type=int, default=None)
ap.add_argument("--steps", type=int, default=5)
ap.add_argument("--windows", type=int, default=1)
args = ap.parse_args()
cfg, S, P, Bdef = bench.CONFIGS[args.config]
B = args.batch or Bdef
os.environ.setdefault("ADVPATCH_TUNE_CACHE", os.path.join(ge.PKG_DIR, "tiles", "conv_tiles_%s_b%d.json" % (args.config, B)))
tp, pc, sy, W = ge._pkg("train_patch"), ge._pkg("patch_config"), ge._pkg("synthetic"), ge._pkg("weights")
dev = torch.device("cuda", 0)
wpath = pc.synthetic_weights_path(cfg.split(":")[-1])
W.ensure_synthetic(cfg, wpath)


class _Cfg(pc.ReproducePaperObj):
    def __init__(self):
        super().__init__()
        self.cfgfile, self.weightfile, self.batch_size = cfg, wpath, B


pc.patch_configs["_bd"] = _Cfg
tr = tp.PatchTrainer("_bd", device=dev, verbose=False)
tr.darknet_model.window_heads = bool(args.windows)
img, lab = sy.frames(B, S, seed=1000).to(dev), sy.labels(B, seed=2000).to(dev)
patch = sy.patch(P, seed=2).to(dev).requires_grad_(True)
opt = tr.make_optimizer(patch)
for _ in range(3):
    tr.step(patch, opt, img, lab)
torch.cuda.synchronize()
plan = tr.last_plan
plan.conv_timer = []
for _ in range(args.steps):
    tr.step(patch, opt, img, lab)
torch.cuda.synchronize()
timer = plan.conv_timer
n = len(timer) // args.steps
descs = [d for name, _, d in plan.fwd_ops + plan.bwd_ops if name == "po_conv"]
assert len(descs) == n
ms = defaultdict(float)
macs = defaultdict(float)
mfma = defaultdict(float)
for k, (e0, e1, d, c) in enumerate(timer):
    ms[k % n] += e0.elapsed_time(e1) / args.steps
    macs[k % n] += plan.launch_macs(d, c) / args.steps
    mfma[k % n] += plan.launch_mfma_flops(d, c) / args.steps
tot = sum(ms.values())
PEAK = 157.3          # dense fp32 MFMA TFLOP/s (MI355X_MICROARCH.md), v_mfma_f32_32x32x2_f32
# dense_TF: the direct convolution's FLOPs (2 x MACs of the launch's live grid) per second -- a
# Winograd launch executes 1/4 (F(4x4)) or 4/9 (F(2x2)) of them, so this is NOT a utilisation and
# may exceed the peak.  mfma_TF / frac: the FLOPs the matrix cores execute (NetPlan.launch_mfma_flops,
# the bench line's roofline) per second, and their fraction of PEAK -- the utilisation.
print("%-6s %5s %9s %5s %6s %4s %3s %9s %9s %8s %5s %6s" % ("kind", "block", "B*Hg*Wg", "N", "K", "tile", "ks", "us",
                                                           "dense_TF", "mfma_TF", "frac", "%"))
for k, d in enumerate(descs):
    K = d.ntaps * d.Cin_p
    M = d.B * d.Hg * d.Wg
    t = ms[k] * 1e-3
    print("%-6s %5d %9d %5d %6d %4d %3d %9.1f %9.1f %8.1f %5.2f %6.2f" % (
        d.kind, d.block, M, d.N, K, d.tile, d.ksplit, ms[k] * 1e3, 2 * macs[k] / t / 1e12, mfma[k] / t / 1e12,
        mfma[k] / t / 1e12 / PEAK, 100 * ms[k] / tot))
mf = sum(mfma.values())
print("total conv ms/step %.3f, launches %d, dense-equivalent TFLOP/step %.3f (not executed work), "
      "MFMA-executed TFLOP/step %.3f (= the bench line's mfma_flops_per_step), MFMA frac %.3f" % (
          tot, n, 2 * sum(macs.values()) / 1e12, mf / 1e12, mf / (tot * 1e-3) / 1e12 / PEAK))
if os.environ.get("BREAKDOWN_JSON"):
    import json
    with open(os.environ["BREAKDOWN_JSON"], "w") as f:
        json.dump({"steps": args.steps, "launches": [
            {"kind": d.kind, "block": d.block, "M": d.B * d.Hg * d.Wg, "N": d.N, "K": d.ntaps * d.Cin_p,
             "tile": d.tile, "ksplit": d.ksplit, "macs": macs[k], "mfma_flops": mfma[k], "boxed": bool(d.gbox),
             "us_events": ms[k] * 1e3}
            for k, d in enumerate(descs)]}, f)
