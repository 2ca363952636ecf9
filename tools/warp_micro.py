"""Micro-benchmark of the warp + composite kernels at the bench workload
(B=16, S=608, P=224): po_warp_fwd / po_warp_bwd with the noise tensor and the
keyed variants, with the trainer's placements and with every patch moved off
the frame (the pure image-copy cost of the composite).  Prints one line per
variant: us per call and GB/s of the algorithmic bytes bench.py's
warp_roofline counts.  Usage: python tools/warp_micro.py [B] [S] [P] [iters]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import importlib  # noqa: E402

PKG = "adversarial_patch-based_false_positive_creation_attacks_against_aerial_imagery_object_detectors_amd"
nat = importlib.import_module(PKG + "._native")
ld = importlib.import_module(PKG + ".load_data")
sy = importlib.import_module(PKG + ".synthetic")

B = int(sys.argv[1]) if len(sys.argv) > 1 else 16
S = int(sys.argv[2]) if len(sys.argv) > 2 else 608
P = int(sys.argv[3]) if len(sys.argv) > 3 else 224
IT = int(sys.argv[4]) if len(sys.argv) > 4 else 50
dev = torch.device("cuda", 0)
nat.load()
seed, step = 0x5EED, 3
dr = sy.draws_device(seed, step, 0, B, P, dev)
lab = sy.labels(B, seed=4).to(dev)
img = sy.frames(B, S, seed=3).to(dev)
mp = sy.patch(P, seed=5).to(dev).contiguous()
_, _, _, roi, affine = ld.patch_params(lab, S, P, dr, True, with_roi=True)     # the trainer's (reference) geometry
_, _, _, _, off = ld.patch_params(lab, S, P, dr, True, with_roi=True, geometry="f64")   # pixel-space map rows
off[:, 2] += 4 * S                      # every sample point far right of the patch: no footprint pixel
roi_off = torch.zeros_like(roi)          # ... and an empty footprint box
out = torch.empty(B, 3, S, S, device=dev)
work = torch.empty(B * S * S * 4, device=dev)             # the box forms: [B,S,S,4] interleaved factors
d_out = torch.randn(B, 3, S, S, device=dev)
d_mp = torch.empty(3, P, P, device=dev)
fwd_bytes = B * 2 * 3 * S * S * 4 + 3 * P * P * 4
bwd_bytes = B * 3 * S * S * 4
st = nat.stream()
area = ((roi[:, 2] - roi[:, 0]).clamp(min=0) * (roi[:, 3] - roi[:, 1]).clamp(min=0)).float().mean().item()
print("B=%d S=%d P=%d: mean footprint box %.0f px (%.1f%% of the frame)" % (B, S, P, area, 100 * area / S / S))


def timed(fn):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(IT):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) * 1000 / IT


def fwd(aff, keyed):
    if keyed:
        return lambda: nat.call("po_warp_fwd_keyed", nat.ptr(img), nat.ptr(mp), seed, step, 0, nat.ptr(dr["contrast"]),
                                nat.ptr(dr["bright"]), nat.ptr(aff, torch.float64), B, S, P, 1, nat.ptr(out), st)
    return lambda: nat.call("po_warp_fwd", nat.ptr(img), nat.ptr(mp), nat.ptr(dr["noise"]), nat.ptr(dr["contrast"]),
                            nat.ptr(dr["bright"]), nat.ptr(aff, torch.float64), B, S, P, 1, nat.ptr(out), st)


def bwd(aff, keyed):
    if keyed:
        return lambda: nat.call("po_warp_bwd_keyed", nat.ptr(d_out), nat.ptr(mp), seed, step, 0,
                                nat.ptr(dr["contrast"]), nat.ptr(dr["bright"]), nat.ptr(aff, torch.float64), B, S,
                                P, 1, nat.ptr(work), nat.ptr(d_mp), st)
    return lambda: nat.call("po_warp_bwd", nat.ptr(d_out), nat.ptr(mp), nat.ptr(dr["noise"]), nat.ptr(dr["contrast"]),
                            nat.ptr(dr["bright"]), nat.ptr(aff, torch.float64), B, S, P, 1, nat.ptr(work),
                            nat.ptr(d_mp), st)


pre = torch.empty(B, 3, P, P, device=dev)


def aug():
    nat.call("po_augment_patch", nat.ptr(mp), seed, step, 0, nat.ptr(dr["contrast"]), nat.ptr(dr["bright"]), B, P,
             nat.ptr(pre), st)


def fwd_pre(aff):
    def f():
        aug()
        nat.call("po_warp_fwd_pre", nat.ptr(img), nat.ptr(pre), nat.ptr(aff, torch.float64),
                 nat.ptr(roi if aff is affine else roi_off, torch.int32), B, S, P, 1, nat.ptr(out), st)
    return f


def bwd_pre(aff):
    return lambda: nat.call("po_warp_bwd_pre", nat.ptr(d_out), nat.ptr(pre), nat.ptr(dr["contrast"]),
                            nat.ptr(aff, torch.float64), nat.ptr(roi if aff is affine else roi_off, torch.int32),
                            B, S, P, 1, nat.ptr(work), nat.ptr(d_mp), st)


copy = lambda: out.copy_(img)
t = timed(copy)
print("torch copy_ (img -> out)      %8.1f us  %7.0f GB/s" % (t, (fwd_bytes - 3 * P * P * 4) / t / 1e3))
for name, aff in (("placed", affine), ("off-frame", off)):
    for keyed in (False, True):
        t = timed(fwd(aff, keyed))
        print("fwd %-9s %-6s            %8.1f us  %7.0f GB/s" % (name, "keyed" if keyed else "tensor", t,
                                                               fwd_bytes / t / 1e3))
t = timed(aug)
print("po_augment_patch              %8.1f us" % t)
for name, aff in (("placed", affine), ("off-frame", off)):
    t = timed(fwd_pre(aff))
    print("fwd %-9s pre (+augment)   %8.1f us  %7.0f GB/s" % (name, t, fwd_bytes / t / 1e3))
    t = timed(bwd_pre(aff))
    print("bwd %-9s pre              %8.1f us  %7.0f GB/s" % (name, t, bwd_bytes / t / 1e3))
for name, aff in (("placed", affine), ("off-frame", off)):
    for keyed in (False, True):
        t = timed(bwd(aff, keyed))
        print("bwd %-9s %-6s            %8.1f us  %7.0f GB/s" % (name, "keyed" if keyed else "tensor", t,
                                                               bwd_bytes / t / 1e3))
