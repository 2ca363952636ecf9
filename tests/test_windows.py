"""Receptive-field windows (NetPlan._plan_windows), checked on the CPU.

The training path computes the blocks after the last full-map dependency
only on a box around the cells the loss reads (train_patch.py:449-483).  The
windows are correct when every activation the loss depends on lies inside
them: the oracle's autograd gradient of the loss w.r.t. each windowed block's
pre-activation must vanish outside the window placed the way po_cell_windows
places it (emulated here from the plan's tables)."""
import os
import tempfile

import pytest
import torch

import oracle
from conftest import pkg_mod


def _origins(plan, cells):
    """po_cell_windows on the host: cells [nheads][B] flat indices."""
    lut = plan.win_lut.cpu()
    ext = plan.win_ext.cpu()
    org = torch.zeros(plan.org.shape, dtype=torch.int32)
    for w in range(lut.size(0)):
        side, mp = int(ext[w, 0]), int(ext[w, 1])
        for b in range(plan.B):
            lo_r = lo_c = 1 << 30
            hi_r = hi_c = -(1 << 30)
            for h, hw in enumerate(plan.win_hw):
                r, c = divmod(cells[h][b], hw)
                e = lut[w, h]
                if e[r, 0] <= e[r, 1]:
                    lo_r, hi_r = min(lo_r, int(e[r, 0])), max(hi_r, int(e[r, 1]))
                if e[c, 0] <= e[c, 1]:
                    lo_c, hi_c = min(lo_c, int(e[c, 0])), max(hi_c, int(e[c, 1]))
            assert hi_r - lo_r + 1 <= side and hi_c - lo_c + 1 <= side
            org[w, b, 0] = min(max(lo_r, 0), mp - side)
            org[w, b, 1] = min(max(lo_c, 0), mp - side)
    return org


def _plan(cfg, B, S):
    W, dk = pkg_mod("weights"), pkg_mod("darknet_v3")
    net = dk.Darknet(cfg)
    with tempfile.TemporaryDirectory() as td:
        p = os.path.join(td, "w.weights")
        W.write_weights(p, W.synthesize(cfg, seed=4))
        net.load_darknet_weights(p)
    return net.plan(B, S, S, torch.device("cpu"), windowed=True), p


@pytest.mark.parametrize("cfg,S,P", [("builtin:mini3", 64, 32), ("builtin:mini3-96", 96, 32)])
def test_gradient_support_inside_windows(cfg, S, P):
    sy, W, G, ld = pkg_mod("synthetic"), pkg_mod("weights"), pkg_mod("cfg_gen"), pkg_mod("load_data")
    B = 6
    plan, _ = _plan(cfg, B, S)
    assert plan.windowed and any(plan.win[i] for i in range(plan.n))
    net = oracle.OracleDarknet(G.cfg_text(cfg), None)
    net.load_darknet_weights(W.synthesize(cfg, seed=4))
    img, lab = sy.frames(B, S, seed=80), sy.labels(B, seed=81)
    patch, dr = sy.patch(P, seed=82), sy.draws(B, P, seed=83)
    rec = {}
    ref = oracle.train_step(patch, img, lab, dr, net, ld.load_printability_colors("builtin:30values"), record=rec)
    org = _origins(plan, ref["cells"])
    checked = 0
    for j, x in rec.items():
        if plan.win[j] is None or x.grad is None:
            continue
        side = plan.win[j]
        g = x.grad.abs().sum(1)                     # [B,H,W]
        for b in range(B):
            r0, c0 = (int(v) for v in org[plan.win_idx[j], b])
            inside = torch.zeros_like(g[b], dtype=torch.bool)
            inside[r0:r0 + side, c0:c0 + side] = True
            assert float(g[b][~inside].abs().max()) == 0.0, (j, b)
            checked += 1
    assert checked > 0


def test_yolov3_window_sides():
    """Static window sides of yolov3-dota@608 (documented in DESIGN.md)."""
    dk = pkg_mod("darknet_v3")
    net = dk.Darknet("builtin:yolov3-dota")
    net._prepare = lambda d: None
    plan = dk.NetPlan.__new__(dk.NetPlan)
    # build only the shape/window analysis (no weights needed)
    net._dev = {i: {"w": torch.zeros(1), "bias": torch.zeros(1), "w27": torch.zeros(1)} for i in net._conv_meta}
    net._folded_cache = {i: torch.zeros(m["cout"], m["cin"], m["k"], m["k"], dtype=torch.float64)
                         for i, m in net._conv_meta.items()}
    plan = dk.NetPlan(net, 2, 608, 608, torch.device("cpu"), windowed=True)
    sides = {i: plan.win[i] for i in range(plan.n) if plan.win[i]}
    assert min(sides) == 75                          # everything up to the trunk end stays full-map
    assert sides[80] == sides[81] == sides[92] == sides[93] == sides[104] == sides[105] == 1
    assert sides[75] == 9 and sides[97] == 7
