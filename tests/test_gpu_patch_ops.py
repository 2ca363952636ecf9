"""GPU parity of the patch-side HIP kernels against the oracle (PyTorch-CPU
restatement of reference load_data.py / median_pool.py).  Tolerances are
fp32-level: outputs within 1e-5 absolute, gradients within 1e-4 relative."""
import math

import pytest
import torch

import oracle
from conftest import pkg_mod

pytestmark = pytest.mark.gpu


def _dev():
    return torch.device("cuda", 0)


def test_median7_fwd_bwd_matches_oracle():
    mp = pkg_mod("median_pool")
    torch.manual_seed(0)
    x = torch.rand(1, 3, 37, 41)
    y_ref = oracle.median_pool7(x)
    xg = x.to(_dev()).requires_grad_(True)
    y = mp.MedianPool2d(7, same=True)(xg)
    assert torch.equal(y.detach().cpu(), y_ref)          # selection is exact
    g = torch.randn_like(y_ref)
    y.backward(g.to(_dev()))
    xr = x.clone().requires_grad_(True)
    oracle.median_pool7(xr).backward(g)
    torch.testing.assert_close(xg.grad.cpu(), xr.grad, rtol=0, atol=1e-6)


def test_median7_constant_patch_kat():
    # SURVEY Appendix B KAT 7: the median of a constant patch is itself and its
    # gradient passes 1:1 (ties: first window position -> one element per output)
    mp = pkg_mod("median_pool")
    x = torch.full((1, 3, 20, 20), 0.37, device=_dev(), requires_grad=True)
    y = mp.MedianPool2d(7, same=True)(x)
    assert torch.all(y == 0.37)
    y.sum().backward()
    assert abs(float(x.grad.sum()) - 3 * 400) < 1e-3


@pytest.mark.parametrize("S,P,B", [(96, 32, 5), (608, 224, 3), (97, 32, 2)])
def test_patch_transformer_matches_oracle(S, P, B):
    ld, sy = pkg_mod("load_data"), pkg_mod("synthetic")
    patch = sy.patch(P, seed=11)
    lab = sy.labels(B, seed=12)
    dr = sy.draws(B, P, seed=13)
    ref_t, ref_c = oracle.patch_transformer(patch, lab, S, dr)
    pt = ld.PatchTransformer()
    d = {k: v.to(_dev()) for k, v in dr.items()}
    out, c = pt(patch.to(_dev()), lab.to(_dev()), S, draws=d)
    torch.testing.assert_close(c.cpu(), ref_c, rtol=0, atol=0)
    diff = (out.cpu() - ref_t).abs()
    # a handful of boundary pixels may round differently; values agree to fp32
    assert float((diff > 1e-4).float().mean()) < 1e-4, float(diff.max())
    assert float(diff.mean()) < 1e-7


@pytest.mark.parametrize("S,P,B", [(96, 32, 4), (608, 224, 2)])
def test_fused_composite_fwd_bwd_matches_oracle(S, P, B):
    ld, sy = pkg_mod("load_data"), pkg_mod("synthetic")
    patch = sy.patch(P, seed=21)
    img = sy.frames(B, S, seed=22)
    lab = sy.labels(B, seed=23)
    dr = sy.draws(B, P, seed=24)
    g = torch.randn(B, 3, S, S, generator=torch.Generator().manual_seed(5))
    pr = patch.clone().requires_grad_(True)
    adv_t, c_ref = oracle.patch_transformer(pr, lab, S, dr)
    p_ref = oracle.patch_applier(img, adv_t)
    (p_ref * g).sum().backward()
    pt = ld.PatchTransformer()
    pg = patch.to(_dev()).requires_grad_(True)
    d = {k: v.to(_dev()) for k, v in dr.items()}
    p_img, c = pt.forward_composite(pg, lab.to(_dev()), img.to(_dev()), S, draws=d)
    (p_img * g.to(_dev())).sum().backward()
    diff = (p_img.detach().cpu() - p_ref.detach()).abs()
    assert float((diff > 1e-4).float().mean()) < 1e-4
    ref = pr.grad
    got = pg.grad.cpu()
    rel = float((got - ref).abs().max() / ref.abs().max())
    assert rel < 1e-4, rel


def test_patch_applier_matches_oracle():
    ld = pkg_mod("load_data")
    torch.manual_seed(3)
    img = torch.rand(2, 3, 16, 16)
    adv = torch.rand(2, 1, 3, 16, 16) * (torch.rand(2, 1, 3, 16, 16) > 0.5)
    ref = oracle.patch_applier(img, adv)
    a = adv.to(_dev()).requires_grad_(True)
    out = ld.PatchApplier()(img.to(_dev()), a)
    assert torch.equal(out.detach().cpu(), ref)
    out.sum().backward()
    assert torch.equal(a.grad.cpu(), (adv != 0).float())


@pytest.mark.parametrize("P", [224, 32])
def test_regularisers_match_oracle(P):
    ld, sy = pkg_mod("load_data"), pkg_mod("synthetic")
    patch = sy.patch(P, seed=31)
    colors = ld.load_printability_colors("builtin:30values")
    pr = patch.clone().requires_grad_(True)
    nps = oracle.nps_score(pr, colors)
    tv = oracle.total_variation(pr)
    col = oracle.colorful_loss(pr)
    loss_ref = nps * 0.01 + torch.max(tv * 2.5, torch.tensor(0.1)) + col
    loss_ref.backward()
    pg = patch.to(_dev()).requires_grad_(True)
    r = ld.regularisers(pg, colors.to(_dev()))
    loss = r[0] * 0.01 + torch.max(r[1] * 2.5, torch.tensor(0.1, device=_dev())) + r[2]
    loss.backward()
    torch.testing.assert_close(r.detach().cpu(), torch.stack([nps, tv, col]).detach(), rtol=2e-6, atol=0)
    rel = float((pg.grad.cpu() - pr.grad).abs().max() / pr.grad.abs().max())
    assert rel < 1e-4, rel


def test_nps_tv_kats_on_gpu():
    # SURVEY Appendix B KATs 2 and 3
    ld = pkg_mod("load_data")
    P = 64
    colors = ld.load_printability_colors("builtin:30values")
    k = 5
    patch = colors[k].view(3, 1, 1).expand(3, P, P).contiguous().to(_dev())
    r = ld.regularisers(patch, colors.to(_dev())).cpu()
    assert abs(float(r[0]) - math.sqrt(1e-6 + 3e-12) / 3) < 1e-9
    assert abs(float(r[1]) - 2 * (P - 1) / P * 1e-6) < 1e-10
