"""Golden fixtures (tests/golden/make_golden.py).  CPU: the oracle reproduces
them (regression pin of the restatement).  GPU: the HIP training step
reproduces them (loss terms, bit-exact cell indices, patch gradient)."""
import os

import numpy as np
import pytest
import torch

from conftest import ROOT, pkg_mod

GOLD = os.path.join(ROOT, "tests", "golden")


def _load(name):
    with np.load(os.path.join(GOLD, "golden_%s.npz" % name), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


@pytest.mark.parametrize("name", ["mini3", "yolov3_608"])
def test_oracle_reproduces_golden(name):
    import sys
    sys.path.insert(0, GOLD)
    import make_golden
    got = make_golden.compute(name)
    want = _load(name)
    np.testing.assert_array_equal(got["cells"], want["cells"])
    np.testing.assert_array_equal(got["patch_center"], want["patch_center"])
    for k in ("loss", "nps_loss", "tv_loss", "no_obj_loss", "no_cls_loss", "colorful_loss"):
        assert abs(float(got[k]) - float(want[k])) <= 1e-5 * max(1.0, abs(float(want[k]))), k
    np.testing.assert_allclose(got["obj"], want["obj"], rtol=0, atol=1e-5)
    scale = float(want["grad_absmax"])
    assert float(np.abs(got["grad_sample"] - want["grad_sample"]).max()) <= 1e-4 * scale


@pytest.mark.gpu
def test_hip_step_reproduces_golden_mini3(tmp_path):
    W, tp, pc, sy = pkg_mod("weights"), pkg_mod("train_patch"), pkg_mod("patch_config"), pkg_mod("synthetic")
    want = _load("mini3")
    path = str(tmp_path / "m.weights")
    W.write_weights(path, W.synthesize("builtin:mini3", seed=4))

    class _Cfg(pc.ReproducePaperObj):
        def __init__(self):
            super().__init__()
            self.cfgfile = "builtin:mini3"
            self.weightfile = path

    pc.patch_configs["_golden"] = _Cfg
    dev = torch.device("cuda", 0)
    tr = tp.PatchTrainer("_golden", device=dev, verbose=False)
    B, P, S = 4, 32, 64
    img, lab, patch, dr = sy.frames(B, S, seed=0), sy.labels(B, seed=1), sy.patch(P, seed=2), sy.draws(B, P, seed=3)
    pg = patch.to(dev).requires_grad_(True)
    loss, t = tr.losses(pg, img.to(dev), lab.to(dev), {k: v.to(dev) for k, v in dr.items()})
    loss.backward()
    np.testing.assert_array_equal(t["cells"].cpu().numpy(), want["cells"])
    np.testing.assert_array_equal(t["patch_center"].cpu().numpy(), want["patch_center"])
    for k in ("loss", "nps_loss", "tv_loss", "no_obj_loss", "no_cls_loss", "colorful_loss"):
        assert abs(float(t[k]) - float(want[k])) <= 2e-5 * max(1.0, abs(float(want[k]))), k
    g = pg.grad.cpu().numpy()
    rel = float(np.abs(g - want["grad"]).max() / np.abs(want["grad"]).max())
    assert rel < 1e-4, rel
