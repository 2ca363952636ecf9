"""GPU parity of the test-time placements against the
oracle restatement oracle/placement_ref.py (reference load_data.py:985-1722).

PatchTransformer_test_mode: the discrete results — semi_edge, the number of
free cells, the pick and the chosen (x, y) — are compared exactly; the image
within 2e-6 of the oracle's float64-geometry evaluation.  The occupancy map
(po_place_free_map) must have exactly the zeros of the literal
inter_axis_cal.  PatchTransformer_vanishing: within 2e-6 of the float64
evaluation of the reference's ops; the fused multi-slot composite equals
PatchApplier over the [B, n, 3, S, S] output bit for bit."""
import itertools
import math

import numpy as np
import pytest
import torch

from oracle import placement_ref as pr
from conftest import pkg_mod

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _det_labels(n, seed, wmax=0.2):
    """0.01-threshold detections [1, n, 7] {x, y, w, h, obj, cls_conf, id}."""
    g = np.random.Generator(np.random.PCG64(seed))
    lab = np.zeros((1, n, 7), dtype=np.float32)
    lab[0, :, 0:2] = g.uniform(0.05, 0.95, (n, 2))
    lab[0, :, 2:4] = g.uniform(0.01, wmax, (n, 2))
    lab[0, :, 4:6] = g.uniform(0.01, 1.0, (n, 2))
    lab[0, :, 6] = g.integers(0, 15, n)
    return torch.from_numpy(lab)


def _assert_zero_sets(got, want):
    """Exact zeros (the image shows through in PatchApplier) agree, except
    where the other side holds a bilinear weight at rounding level (a float64
    fraction of ~1e-16 of an edge tap that one evaluation rounds to 0)."""
    mism = (got == 0) != (want == 0)
    if mism.any():
        assert float(got.double()[mism].abs().max()) < 1e-6 and float(want.double()[mism].abs().max()) < 1e-6


def _run_hip(patch, lab, S, angle, upick, test_mode=True):
    ld = pkg_mod("load_data")
    pt = ld.PatchTransformer_test_mode(test_mode=test_mode)
    d = {"angle": torch.tensor([angle], dtype=torch.float32, device=DEV),
         "upick": torch.tensor([upick], dtype=torch.float32, device=DEV)}
    out = pt(patch.to(DEV), lab.to(DEV), S, draws=d)
    info = dict(zip(ld.PLACE_INFO, pt.last_info[0].cpu().tolist()))
    return out.cpu(), info


TM_CASES = [
    # S, P, n, label seed, wmax, angle, upick
    (160, 48, 6, 1, 0.2, 0.3, 0.41),
    (608, 224, 20, 2, 0.15, -1.2, 0.77),
    (608, 224, 1, 3, 0.2, 0.9, 0.05),          # single detection: the 0.25 row
    (416, 96, 12, 4, 0.45, 1.45, 0.5),         # large boxes: crowded map
    (97, 32, 5, 5, 0.3, -0.7, 0.999),          # odd size: half-pixel translation
    (101, 32, 3, 6, 0.2, 0.2, 0.3),            # B*S*S and B*L not multiples of 4 (workspace sub-buffer alignment)
]


@pytest.mark.parametrize("S,P,n,seed,wmax,angle,upick", TM_CASES)
def test_test_mode_matches_oracle(S, P, n, seed, wmax, angle, upick):
    sy = pkg_mod("synthetic")
    patch = sy.patch(P, seed=30 + seed)
    lab = _det_labels(n, seed, wmax)
    angle = float(np.float32(angle))
    upick = float(np.float32(upick))
    want, winfo = pr.test_mode_place(patch, lab, S, angle, upick)
    got, info = _run_hip(patch, lab, S, angle, upick)
    assert info["flags"] == 0, info
    for k in ("semi_edge2", "n_free", "pick", "x", "y", "mask_ones"):
        assert info[k] == winfo[k], (k, info, winfo)
    diff = float((got - want).abs().max())
    assert diff < 2e-6, diff
    _assert_zero_sets(got, want)


def test_test_mode_max_area_row_and_flat_rule():
    """A detection with area > 0.99 selects the 0.25 row (load_data.py:1311-1313)."""
    sy = pkg_mod("synthetic")
    patch = sy.patch(64, seed=40)
    lab = _det_labels(4, 7)
    lab[0, 2, 2:4] = 1.0
    want, winfo = pr.test_mode_place(patch, lab, 256, 0.25, 0.3)
    got, info = _run_hip(patch, lab, 256, 0.25, 0.3)
    assert (info["x"], info["y"], info["semi_edge2"], info["n_free"]) == \
        (winfo["x"], winfo["y"], winfo["semi_edge2"], winfo["n_free"])
    assert float((got - want).abs().max()) < 2e-6


def test_test_mode_inclusive_randint_raises_like_the_reference():
    """random.randint(0, N) can return N; position_available[N] raises
    IndexError in the reference, and so does the device path."""
    sy = pkg_mod("synthetic")
    patch = sy.patch(48, seed=41)
    lab = _det_labels(5, 8)
    u = float(np.float32(1.0 - 2 ** -24))
    with pytest.raises(IndexError):
        pr.test_mode_place(patch, lab, 160, 0.1, u)
    with pytest.raises(IndexError):
        _run_hip(patch, lab, 160, 0.1, u)


FREE_CASES = list(itertools.product([1, 3, 30], [0.1, 0.6], [0.4, 3.5, 17.0]))


@pytest.mark.parametrize("n,wmax,semi", FREE_CASES)
def test_free_map_matches_inter_axis_cal(n, wmax, semi):
    ld = pkg_mod("load_data")
    pt = ld.PatchTransformer_test_mode(test_mode=True)
    S = 96
    lab = _det_labels(n, 100 + n, wmax)
    lab[0, :, 0:2] = lab[0, :, 0:2] * 1.1 - 0.05             # boxes past the edges: negative int() bounds
    st = torch.tensor(semi, dtype=torch.float32)
    want = pr.inter_axis_cal(lab, st, S) == 0
    got = pt.inter_axis_cal(lab.to(DEV), semi, S).cpu() == 0
    assert torch.equal(got, want), (int(got.sum()), int(want.sum()))


def _van_draws(BL, P, seed):
    g = torch.Generator().manual_seed(seed)
    ux, uy = torch.rand(BL, generator=g), torch.rand(BL, generator=g)
    d = {"contrast": torch.rand(BL, generator=g) * 0.4 + 0.8, "bright": torch.rand(BL, generator=g) * 0.2 - 0.1,
         "noise": torch.rand(BL, 3, P, P, generator=g) * 2 - 1,
         "angle": torch.rand(BL, generator=g) * 2 * math.pi - math.pi, "ux": ux, "uy": uy}
    # the offsets the device path derives from ux / uy (load_data.PatchTransformer_vanishing._prep)
    d["offx"] = (ux.double() * 0.4 - 0.2).float()
    d["offy"] = (uy.double() * 0.4 - 0.2).float()
    return d


def _f64(fn, *args, **kw):
    old = torch.get_default_dtype()
    torch.set_default_dtype(torch.float64)
    try:
        return fn(*args, **kw)
    finally:
        torch.set_default_dtype(old)


VAN_CASES = [
    # S, P, B, n, do_rotate, rand_loc, orient, test_real
    (160, 48, 2, 5, True, False, None, False),
    (608, 224, 1, 6, True, True, "left", False),
    (416, 64, 2, 4, False, False, "right", True),
]


@pytest.mark.parametrize("S,P,B,n,do_rotate,rand_loc,orient,test_real", VAN_CASES)
def test_vanishing_matches_oracle(S, P, B, n, do_rotate, rand_loc, orient, test_real):
    ld, sy = pkg_mod("load_data"), pkg_mod("synthetic")
    patch = sy.patch(P, seed=50 + n)
    lab = sy.labels(B, seed=51 + n)[:, :n].contiguous()
    lab[:, :, 3:5] = lab[:, :, 3:5] * 2.0               # larger boxes: patches of 10-100 px
    d = _van_draws(B * n, P, seed=52 + n)
    want = _f64(pr.vanishing_transformer, patch.double(), lab.double(), S,
                {k: v.double() for k, v in d.items()}, do_rotate=do_rotate, rand_loc=rand_loc, orient=orient,
                test_real=test_real)
    pt = ld.PatchTransformer_vanishing()
    dd = {k: v.to(DEV) for k, v in d.items()}
    got = pt(patch.to(DEV), lab.to(DEV), S, do_rotate=do_rotate, rand_loc=rand_loc, orient=orient,
             test_real=test_real, draws=dd).cpu()
    assert got.shape == (B, n, 3, S, S)
    diff = float((got.double() - want).abs().max())
    assert diff < 2e-6, diff
    _assert_zero_sets(got, want)
    # fused slot composite == PatchApplier over the slots, bit for bit
    img = sy.frames(B, S, seed=53).to(DEV)
    seq = ld.PatchApplier()(img, got.to(DEV))
    fused = pt.forward_composite(patch.to(DEV), lab.to(DEV), img, S, do_rotate=do_rotate, rand_loc=rand_loc,
                                 orient=orient, test_real=test_real, draws=dd)
    assert torch.equal(fused, seq)
