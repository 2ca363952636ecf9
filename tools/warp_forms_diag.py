"""Which keyed warp forms (frame / pre / box, flat or per-image box grids)
disagree, under each placement geometry: the composite, the warp-only output
and the patch gradient of every form against the tensor-noise frame form,
as max |diff| and the first differing pixel.  python tools/warp_forms_diag.py"""
import importlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
PKG = "adversarial_patch-based_false_positive_creation_attacks_against_aerial_imagery_object_detectors_amd"
ld = importlib.import_module(PKG + ".load_data")
sy = importlib.import_module(PKG + ".synthetic")
DEV = torch.device("cuda", 0)
B, S, P, b0 = 6, 608, 224, 0
seed, step = 0x5EED1234ABCD, 9
full = sy.draws_device(seed, step, b0, B, P, DEV)
keyed = {k: v for k, v in full.items() if k != "noise"}
keyed["noise_key"] = (seed, step, b0)
img = sy.frames(B, S, seed=3).to(DEV)
lab = sy.labels(B, seed=4).to(DEV)
patch = sy.patch(P, seed=5).to(DEV)
g = torch.randn(B, 3, S, S, generator=torch.Generator().manual_seed(6)).to(DEV)
for geometry in ("ref", "f64"):
    res = {}
    for dr, form in ((full, "frame"), (keyed, "frame"), (keyed, "pre"), (keyed, "box")):
        pt = ld.PatchTransformer()
        pt.warp_form, pt.geometry = form, geometry
        pg = patch.clone().requires_grad_(True)
        comp, _ = pt.forward_composite(pg, lab, img, S, draws=dr)
        comp.backward(g)
        adv, _ = pt(patch, lab, S, draws=dr)
        res[(form, "noise" in dr)] = (comp.detach(), pg.grad.clone(), adv, pt.last_roi.clone())
    base = res[("frame", True)]
    for key, val in res.items():
        for name, a, b in (("comp", base[0], val[0]), ("grad", base[1], val[1]), ("adv", base[2], val[2])):
            d = (a - b).abs()
            if bool((d != 0).any()):
                idx = (d != 0).nonzero()[0].tolist()
                print("%s %-5s tensor=%d %-4s max %.3g at %s (%d differ): %r vs %r" % (
                    geometry, key[0], key[1], name, float(d.max()), idx, int((d != 0).sum()),
                    float(a[tuple(idx)]), float(b[tuple(idx)])))
            else:
                print("%s %-5s tensor=%d %-4s equal" % (geometry, key[0], key[1], name))
    if geometry == "ref":
        print("roi", base[3].tolist())
