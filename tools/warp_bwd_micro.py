"""A/B micro-benchmark of the training warp pair at a bench workload (default
tiny: B=256, S=416, P=224): po_warp_box_fwd_fac once, then po_warp_box_bwd_fac
(factor pass + phase-B gather) timed with HIP events.  The first backward's
d_patch checksum is printed so variants (ADVPATCH_LIB=tools/var/<name>/...)
can be checked for identical bits.  Geometry: ADVPATCH_GEOMETRY (ref | f64).
Usage: python tools/warp_bwd_micro.py [B] [S] [P] [iters]"""
import hashlib
import importlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
PKG = "adversarial_patch-based_false_positive_creation_attacks_against_aerial_imagery_object_detectors_amd"
nat = importlib.import_module(PKG + "._native")
ld = importlib.import_module(PKG + ".load_data")
sy = importlib.import_module(PKG + ".synthetic")

B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
S = int(sys.argv[2]) if len(sys.argv) > 2 else 416
P = int(sys.argv[3]) if len(sys.argv) > 3 else 224
IT = int(sys.argv[4]) if len(sys.argv) > 4 else 30
dev = torch.device("cuda", 0)
nat.load()
seed, step = 0x5EED, 3
dr = sy.draws_device(seed, step, 0, B, P, dev)
lab = sy.labels(B, seed=4).to(dev)
img = sy.frames(B, S, seed=3).to(dev)
mp = sy.patch(P, seed=5).to(dev).contiguous()
_, _, _, roi, affine = ld.patch_params(lab, S, P, dr, True, with_roi=True)
out = torch.empty(B, 3, S, S, device=dev)
fac = torch.empty(B * S * S * 4, device=dev)
d_out = torch.randn(B, 3, S, S, device=dev, generator=torch.Generator(dev).manual_seed(9))
d_mp = torch.empty(3, P, P, device=dev)
st = nat.stream()
key = (seed, step, 0)


def fwd():
    nat.call("po_warp_box_fwd_fac", nat.ptr(img), nat.ptr(mp), *key, nat.ptr(dr["contrast"]), nat.ptr(dr["bright"]),
             nat.ptr(affine, torch.float64), nat.ptr(roi, torch.int32), B, S, P, 1, 0, nat.ptr(out), nat.ptr(fac), st)


def bwd():
    nat.call("po_warp_box_bwd_fac", nat.ptr(d_out), nat.ptr(mp), *key, nat.ptr(dr["contrast"]), nat.ptr(dr["bright"]),
             nat.ptr(affine, torch.float64), nat.ptr(roi, torch.int32), B, S, P, nat.ptr(fac), nat.ptr(d_mp), st)


def timed(fn, n):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) * 1000 / n


fwd()
bwd()
torch.cuda.synchronize()
h = hashlib.sha1(d_mp.cpu().numpy().tobytes()).hexdigest()[:12]
for _ in range(3):
    bwd()
tb = timed(bwd, IT)
tf = timed(fwd, IT)
print("%-10s geometry=%-3s B=%d S=%d: fwd_fac %7.1f us  bwd_fac %7.1f us  d_mp %s" % (
    os.path.basename(os.path.dirname(os.environ.get("ADVPATCH_LIB", "./default/x"))),
    os.environ.get("ADVPATCH_GEOMETRY", "ref"), B, S, tf, tb, h))
