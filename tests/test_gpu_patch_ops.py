"""GPU parity of the patch-side HIP kernels against the oracle (PyTorch-CPU
restatement of reference load_data.py / median_pool.py).  Tolerances are
fp32-level: outputs within 1e-5 absolute, gradients within 1e-4 relative.

The trainer's placement geometry is the reference's own fp32 arithmetic
(po_patch_params geometry 1, "ref"): theta, the affine grid, the sample
points and bilinear weights are those of PyTorch-CPU's affine_grid +
grid_sample, so the warped patch equals the fp32 oracle's bit for bit.  The
opt-in float64 geometry ("f64") is compared with the float64 evaluation of
the oracle; the fp32 oracle differs from it by its own grid rounding."""
import math

import pytest
import torch

import oracle
from conftest import pkg_mod

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


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


def _f64(fn, *args):
    old = torch.get_default_dtype()
    torch.set_default_dtype(torch.float64)
    try:
        return fn(*args)
    finally:
        torch.set_default_dtype(old)


def _dbl(d):
    return {k: v.double() for k, v in d.items()}


@pytest.mark.parametrize("S,P,B", [(96, 32, 5), (608, 224, 16), (416, 224, 8), (97, 32, 2)])
def test_patch_params_reference_geometry_bit_exact(S, P, B):
    """po_patch_params geometry 1 (the trainer's default): theta and
    target_size are the fp32 values the reference computes
    (load_data.py:648-743, oracle.patch_theta on PyTorch-CPU), bit for bit,
    on the trainer's own draws (po_draws) and on seeded draws; the centres too."""
    ld, sy = pkg_mod("load_data"), pkg_mod("synthetic")
    lab = sy.labels(B, seed=31)
    for dr in (sy.draws(B, P, seed=32),
               {k: v.cpu() for k, v in sy.draws_device(3, 11, 0, B, P, _dev()).items()}):
        th_ref, c_ref, ts_ref = oracle.patch_theta(lab, S, P, dr)
        d = {k: v.to(_dev()) for k, v in dr.items()}
        th, c, ts = ld.patch_params(lab.to(_dev()), S, P, d, geometry="ref")
        assert torch.equal(th.cpu().view(B, 2, 3), th_ref)
        assert torch.equal(ts.cpu(), ts_ref)
        assert torch.equal(c.cpu(), c_ref)


@pytest.mark.parametrize("geometry", ["ref", "f64"])
@pytest.mark.parametrize("S,P,B", [(96, 32, 5), (608, 224, 3), (97, 32, 2)])
def test_patch_transformer_matches_oracle(S, P, B, geometry):
    """adv_batch_t and patch_center: centres bit-exact against the fp32
    reference (they set the loss cells).  "ref": every pixel bit-identical
    to the fp32 oracle (the reference's own affine_grid + grid_sample).
    "f64": every pixel within 2e-6 of the float64 evaluation."""
    ld, sy = pkg_mod("load_data"), pkg_mod("synthetic")
    patch = sy.patch(P, seed=11)
    lab = sy.labels(B, seed=12)
    dr = sy.draws(B, P, seed=13)
    ref32, ref_c = oracle.patch_transformer(patch, lab, S, dr)
    pt = ld.PatchTransformer()
    pt.geometry = geometry
    d = {k: v.to(_dev()) for k, v in dr.items()}
    out, c = pt(patch.to(_dev()), lab.to(_dev()), S, draws=d)
    torch.testing.assert_close(c.cpu(), ref_c, rtol=0, atol=0)
    if geometry == "ref":
        assert torch.equal(out.cpu(), ref32), float((out.cpu() - ref32).abs().max())
        return
    ref_t, _ = _f64(oracle.patch_transformer, patch.double(), lab.double(), S, _dbl(dr))
    diff = (out.cpu().double() - ref_t).abs()
    assert float(diff.max()) < 2e-6, float(diff.max())
    # exact zeros (outside the footprint) agree exactly: they decide the composite
    assert torch.equal(out.cpu() == 0, ref_t == 0)


@pytest.mark.parametrize("geometry", ["ref", "f64"])
@pytest.mark.parametrize("S,P,B", [(96, 32, 4), (608, 224, 2)])
def test_fused_composite_fwd_bwd_matches_oracle(S, P, B, geometry):
    """Fused transformer + applier.  "ref": p_img bit-identical to the fp32
    oracle's composite, and the patch gradient of a random upstream gradient
    within 1e-5 (max-abs relative) of the fp32 oracle's (the same products;
    only the order of the sums over output pixels and images differs).
    "f64": p_img within 2e-6 of float64 everywhere, the gradient within 1e-4
    of the float64 gradient; the fp32 oracle is printed beside."""
    ld, sy = pkg_mod("load_data"), pkg_mod("synthetic")
    patch = sy.patch(P, seed=21)
    img = sy.frames(B, S, seed=22)
    lab = sy.labels(B, seed=23)
    dr = sy.draws(B, P, seed=24)
    g = torch.randn(B, 3, S, S, generator=torch.Generator().manual_seed(5))

    def ref_run(dtype):
        pr = patch.to(dtype).clone().requires_grad_(True)
        adv_t, _ = oracle.patch_transformer(pr, lab.to(dtype), S, {k: v.to(dtype) for k, v in dr.items()})
        p_ref = oracle.patch_applier(img.to(dtype), adv_t)
        (p_ref * g.to(dtype)).sum().backward()
        return p_ref.detach(), pr.grad

    p32, g32 = ref_run(torch.float32)
    pt = ld.PatchTransformer()
    pt.geometry = geometry
    pg = patch.to(_dev()).requires_grad_(True)
    d = {k: v.to(_dev()) for k, v in dr.items()}
    p_img, c = pt.forward_composite(pg, lab.to(_dev()), img.to(_dev()), S, draws=d)
    (p_img * g.to(_dev())).sum().backward()
    if geometry == "ref":
        assert torch.equal(p_img.detach().cpu(), p32)
        rel = float((pg.grad.cpu().double() - g32.double()).abs().max() / g32.double().abs().max())
        print("composite patch grad vs fp32 oracle (reference geometry): %.3g" % rel)
        assert rel < 1e-5, rel
        return
    p64, g64 = _f64(ref_run, torch.float64)
    diff = (p_img.detach().cpu().double() - p64).abs()
    assert float(diff.max()) < 2e-6, float(diff.max())
    scale = g64.abs().max()
    rel = float((pg.grad.cpu().double() - g64).abs().max() / scale)
    rel32 = float((g32.double() - g64).abs().max() / scale)
    print("composite patch grad vs float64: hip %.3g, fp32 oracle %.3g" % (rel, rel32))
    assert rel < 1e-4, rel


def test_saturated_patch_ties_match_oracle(monkeypatch):
    """A patch quantised to 8 bits with saturated regions (exactly 0 and 1,
    as clamp_(0,1) leaves them after Adam steps and as a saved PNG holds
    them): 7x7 median windows full of ties (first window position)
    and exact-zero composite pixels (Q5, the image shows through).  Median
    values bit-exact; the composite bit-identical to the fp32 oracle's and the
    patch gradient within 1e-5 of it (the trainer's reference geometry), with
    the oracle's median backward on po_median7's explicit tie rule (first
    window position; torch.median's tie index is implementation-defined)."""
    ld, sy, mpm = pkg_mod("load_data"), pkg_mod("synthetic"), pkg_mod("median_pool")
    monkeypatch.setattr(oracle.reference_path, "MEDIAN_TIE_RULE", "first")
    P, S, B = 64, 160, 3
    q = (sy.patch(P, seed=91) * 255).floor() / 255
    q[:, :20, :] = 0.0                        # a black band: exact zeros survive augmentation only where
    q[:, 40:, 30:] = 1.0                      # noise/brightness push below 0 (clamp) -> exact-zero pixels
    q[0, 20:40, :10] = 0.5                    # a constant block: all-tie windows
    y_ref = oracle.median_pool7(q.unsqueeze(0))
    y = mpm.MedianPool2d(7, same=True)(q.unsqueeze(0).to(_dev()))
    assert torch.equal(y.cpu(), y_ref)
    img, lab = sy.frames(B, S, seed=92), sy.labels(B, seed=93)
    dr = sy.draws(B, P, seed=94)
    dr["bright"] = torch.tensor([-0.1, -0.05, 0.0])           # darken: more clamped-to-0 corners
    g = torch.randn(B, 3, S, S, generator=torch.Generator().manual_seed(6))

    def ref_run(dtype=torch.float64):
        pr = q.to(dtype).clone().requires_grad_(True)
        adv_t, _ = oracle.patch_transformer(pr, lab.to(dtype), S, {k: v.to(dtype) for k, v in dr.items()})
        p_ref = oracle.patch_applier(img.to(dtype), adv_t)
        (p_ref * g.to(dtype)).sum().backward()
        return adv_t.detach(), p_ref.detach(), pr.grad

    adv64, p64, g64 = _f64(ref_run)
    _, p32, g32 = ref_run(torch.float32)
    # footprint = where the warped ones-mask is nonzero (unit patch, no augmentation)
    plain = dict(_dbl(dr), contrast=torch.ones(B, dtype=torch.float64), bright=torch.zeros(B, dtype=torch.float64),
                 noise=torch.zeros(B, 3, P, P, dtype=torch.float64))
    foot, _ = _f64(oracle.patch_transformer, torch.ones(3, P, P, dtype=torch.float64), lab.double(), S, plain)
    foot = foot[:, 0, 0] != 0
    pt = ld.PatchTransformer()
    pg = q.to(_dev()).requires_grad_(True)
    d = {k: v.to(_dev()) for k, v in dr.items()}
    p_img, _ = pt.forward_composite(pg, lab.to(_dev()), img.to(_dev()), S, draws=d)
    (p_img * g.to(_dev())).sum().backward()
    zero_inside = foot & (adv64[:, 0, 0] == 0)
    assert int(zero_inside.sum()) > 100                 # exact-zero composite pixels are exercised (Q5)
    assert torch.equal(p64[:, 0][zero_inside], img.double()[:, 0][zero_inside])
    assert pt.geometry == "ref"
    assert torch.equal(p_img.detach().cpu(), p32)
    rel = float((pg.grad.cpu().double() - g32.double()).abs().max() / g32.double().abs().max())
    assert rel < 1e-5, rel


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


@pytest.mark.parametrize("k,stride,padding,same,shape", [
    (3, 1, 0, True, (2, 3, 17, 19)),
    ((3, 5), (2, 1), (1, 2, 0, 1), False, (1, 3, 20, 23)),
    (4, 2, 0, False, (1, 2, 16, 16)),              # even window: the lower median
    (5, 3, 0, True, (1, 3, 31, 29)),               # 'same' with stride 3 (uneven padding)
    (2, 1, (1, 0, 1, 0), False, (1, 1, 9, 9)),
])
def test_median_pool_general_matches_oracle(monkeypatch, k, stride, padding, same, shape):
    """MedianPool2d beyond the 7x7 training configuration (median_pool.py:8-52):
    values bit-exact; gradient on random (tie-free) data and on quantised
    data with ties (first window position, the oracle's 'first' rule)."""
    mp = pkg_mod("median_pool")
    mod = mp.MedianPool2d(k, stride, padding, same)
    for quant in (False, True):
        monkeypatch.setattr(oracle.reference_path, "MEDIAN_TIE_RULE", "first" if quant else "torch")
        g = torch.Generator().manual_seed(sum(shape) + quant)
        x = torch.rand(*shape, generator=g)
        if quant:
            x = (x * 4).floor() / 4
        pad = mod._padding(x)
        xr = x.clone().requires_grad_(True)
        ref = oracle.median_pool2d(xr, mod.k, mod.stride, pad)
        xg = x.to(_dev()).requires_grad_(True)
        y = mod(xg)
        assert y.shape == ref.shape
        assert torch.equal(y.detach().cpu(), ref.detach())
        dy = torch.randn(ref.shape, generator=g)
        ref.backward(dy)
        y.backward(dy.to(_dev()))
        torch.testing.assert_close(xg.grad.cpu(), xr.grad, rtol=0, atol=1e-6)


@pytest.mark.parametrize("geometry", ["ref", "f64"])
@pytest.mark.parametrize("S,P,B,big", [(416, 224, 6, False), (96, 32, 4, True), (97, 40, 3, False)])
def test_warp_bwd_tight_scan_matches_oracle(S, P, B, big, geometry):
    """po_warp_bwd (load_data.py:726-792 backward, gather form) with the tight
    candidate scan: the patch gradient of the composite within 1e-4 (max-abs
    relative) of the float64 oracle's ("f64" geometry), or within 1e-5 of
    the fp32 oracle's ("ref": the reference's own sample points, so only the
    summation order differs) -- down-scaled patches (an output pixel spans
    several patch pixels) and magnified ones (several output pixels per
    element); S = 97 takes the one-pixel phase A."""
    ld, sy = pkg_mod("load_data"), pkg_mod("synthetic")
    patch = sy.patch(P, seed=31)
    lab = sy.labels(B, seed=32)
    if big:
        lab[:, :, 3:5] = lab[:, :, 3:5].clamp(min=0.6)        # large boxes: the patch is magnified
    img = sy.frames(B, S, seed=33)
    dr = sy.draws(B, P, seed=34)
    g = torch.randn(B, 3, S, S, generator=torch.Generator().manual_seed(6))
    pt = ld.PatchTransformer()
    pt.geometry = geometry
    pg = patch.to(_dev()).requires_grad_(True)
    p_img, _ = pt.forward_composite(pg, lab.to(_dev()), img.to(_dev()), S,
                                    draws={k: v.to(_dev()) for k, v in dr.items()})
    (p_img * g.to(_dev())).sum().backward()
    got = pg.grad.detach().cpu().double()
    if geometry == "ref":
        pr = patch.clone().requires_grad_(True)
        adv_t, _ = oracle.patch_transformer(pr, lab, S, dr)
        (oracle.patch_applier(img, adv_t) * g).sum().backward()
        tol = 1e-5
    else:
        pr = patch.double().requires_grad_(True)
        adv_t, _ = _f64(oracle.patch_transformer, pr, lab.double(), S, _dbl(dr))
        (oracle.patch_applier(img.double(), adv_t) * g.double()).sum().backward()
        tol = 1e-4
    want = pr.grad.double()
    assert bool((got != 0).any())
    err = float((got - want).abs().max() / want.abs().max().clamp(min=1e-12))
    assert err <= tol, err


@pytest.mark.parametrize("B,S,P,b0,big", [(6, 608, 224, 0, False), (5, 416, 224, 37, False), (3, 97, 33, 2, False),
                                          (4, 96, 32, 5, True)])
def test_keyed_noise_warp_bit_identical(B, S, P, b0, big):
    """po_warp_fwd_keyed / po_warp_bwd_keyed regenerate po_draws' noise in the
    kernels, po_augment_patch + po_warp_*_pre form the augmented patches once
    from the same key, po_warp_box_*_keyed form them at the corners of the box
    pixels only (S % 4 == 0; else the frame kernels): the composite, the warp-only output and the patch
    gradient of both equal the tensor path fed po_draws' own noise tensor bit
    for bit (global image index b0 + b, odd S and P included; ``big``: magnified
    patches whose footprint boxes exceed the box kernels' one-pass grid)."""
    ld, sy = pkg_mod("load_data"), pkg_mod("synthetic")
    seed, step = 0x5EED1234ABCD, 9
    full = sy.draws_device(seed, step, b0, B, P, DEV)
    keyed = {k: v for k, v in full.items() if k != "noise"}
    keyed["noise_key"] = (seed, step, b0)
    img = sy.frames(B, S, seed=3).to(DEV)
    lab = sy.labels(B, seed=4)
    if big:
        lab[:, :, 3:5] = lab[:, :, 3:5].clamp(min=0.6)
    lab = lab.to(DEV)
    patch = sy.patch(P, seed=5).to(DEV)
    outs = []
    g = torch.randn(B, 3, S, S, generator=torch.Generator().manual_seed(6)).to(DEV)
    for dr, form in ((full, "frame"), (keyed, "frame"), (keyed, "pre"), (keyed, "box")):
        pt = ld.PatchTransformer()
        pt.warp_form = form
        pg = patch.clone().requires_grad_(True)
        comp, _ = pt.forward_composite(pg, lab, img, S, draws=dr)
        comp.backward(g)
        adv, _ = pt(patch, lab, S, draws=dr)
        outs.append((comp.detach(), pg.grad.clone(), adv))
    for other in outs[1:]:
        for a, b in zip(outs[0], other):
            assert torch.equal(a, b)
    assert (outs[0][0] != img).any()                   # the patch landed somewhere


def test_trainer_draws_are_keyed():
    """The training placement draws no noise tensor by default (keyed noise);
    ADVPATCH_NOISE_KEYED=0 restores the tensor."""
    ld = pkg_mod("load_data")
    pt = ld.PatchTransformer()
    d = pt.make_draws(4, 32, DEV)
    assert "noise" not in d and d["noise_key"] == (pt.draw_seed, 0, 0)


def _quad_box_mask(roi, B, S):
    """[B,1,S,S] bool: the quad-widened footprint boxes (po::quad_box)."""
    m = torch.zeros(B, 1, S, S, dtype=torch.bool)
    for b, (x0, y0, x1, y1) in enumerate(roi.cpu().tolist()):
        qx0, qx1 = x0 & ~3, min(S, (x1 + 3) & ~3)
        if qx1 > qx0 and y1 > y0:
            m[b, :, y0:y1, qx0:qx1] = True
    return m


@pytest.mark.parametrize("B,S,P,big", [(6, 608, 224, False), (5, 416, 224, False), (3, 96, 32, True)])
def test_sparse_composite_box_pixels_and_gradient(B, S, P, big):
    """forward_composite(sparse=True) writes only the quad-widened footprint
    boxes (po_warp_box_fwd_keyed, fill = 0): there the values equal the full
    composite's, outside them the full composite equals the frames, and the
    patch gradient is the full composite's, bit for bit."""
    ld, sy = pkg_mod("load_data"), pkg_mod("synthetic")
    seed, step, b0 = 0x1234, 4, 3
    keyed = {k: v for k, v in sy.draws_device(seed, step, b0, B, P, DEV).items() if k != "noise"}
    keyed["noise_key"] = (seed, step, b0)
    img = sy.frames(B, S, seed=13).to(DEV)
    lab = sy.labels(B, seed=14)
    if big:
        lab[:, :, 3:5] = lab[:, :, 3:5].clamp(min=0.6)
    lab = lab.to(DEV)
    patch = sy.patch(P, seed=15).to(DEV)
    g = torch.randn(B, 3, S, S, generator=torch.Generator().manual_seed(16)).to(DEV)
    outs = []
    for sparse in (False, True):
        pt = ld.PatchTransformer()
        assert pt.warp_form == "box" and pt.sparse_ok(S, keyed)
        pg = patch.clone().requires_grad_(True)
        comp, _ = pt.forward_composite(pg, lab, img, S, draws=keyed, sparse=sparse)
        comp.backward(g)
        outs.append((comp.detach(), pg.grad.clone(), pt.last_roi.clone()))
    (full, g_full, roi), (sp, g_sp, roi2) = outs
    assert torch.equal(roi, roi2)
    m = _quad_box_mask(roi, B, S).to(DEV).expand(B, 3, S, S)
    assert torch.equal(full[m], sp[m])
    assert torch.equal(full[~m], img[~m])
    assert torch.equal(g_full, g_sp)
    assert bool(m.any()) and bool((full[m] != img[m]).any())


@pytest.mark.parametrize("B,S,P,big", [(4, 416, 224, False), (3, 96, 40, True)])
def test_forward_saved_warp_factors_bit_identical(B, S, P, big, monkeypatch):
    """po_warp_box_fwd_fac / po_warp_box_bwd_fac (the forward saves the
    backward's per-pixel factors; ADVPATCH_WARP_FAC, default on) against
    po_warp_box_fwd_keyed / po_warp_box_bwd_keyed (the backward re-evaluates
    the warp): warped patches (mode 0), composites (mode 1, whole and sparse)
    and patch gradients bit for bit."""
    ld, sy = pkg_mod("load_data"), pkg_mod("synthetic")
    seed, step, b0 = 0x77, 2, 1
    keyed = {k: v for k, v in sy.draws_device(seed, step, b0, B, P, DEV).items() if k != "noise"}
    keyed["noise_key"] = (seed, step, b0)
    img = sy.frames(B, S, seed=23).to(DEV)
    lab = sy.labels(B, seed=24)
    if big:
        lab[:, :, 3:5] = lab[:, :, 3:5].clamp(min=0.6)
    lab = lab.to(DEV)
    patch = sy.patch(P, seed=25).to(DEV)
    gen = torch.Generator().manual_seed(26)
    g4 = torch.randn(B, 1, 3, S, S, generator=gen).to(DEV)
    g3 = torch.randn(B, 3, S, S, generator=gen).to(DEV)
    res = {}
    for fac in ("0", "1"):
        monkeypatch.setenv("ADVPATCH_WARP_FAC", fac)
        outs = []
        for form in ("mode0", "full", "sparse"):
            pt = ld.PatchTransformer()
            assert pt.warp_form == "box" and pt.sparse_ok(S, keyed)
            pg = patch.clone().requires_grad_(True)
            if form == "mode0":
                out, _ = pt(pg, lab, S, draws=keyed)
                out.backward(g4)
            else:
                out, _ = pt.forward_composite(pg, lab, img, S, draws=keyed, sparse=form == "sparse")
                out.backward(g3)
            out = out.detach()
            if form == "sparse":                      # only the quad-widened boxes are written
                out = out[_quad_box_mask(pt.last_roi, B, S).to(DEV).expand(B, 3, S, S)]
            outs.append((out, pg.grad.clone()))
        res[fac] = outs
    for (o0, g0), (o1, g1) in zip(res["0"], res["1"]):
        assert torch.equal(o0, o1)
        assert torch.equal(g0, g1) and bool((g0 != 0).any())


@pytest.mark.parametrize("P", [224, 37])
def test_patch_front_matches_separate_nodes(P):
    """patch_front (median pool + regularisers in one autograd node, the
    regularisers' gradient added into the median pool's by
    po_regularisers_grad) equals MedianPool2d(7, same) and regularisers() as
    two nodes whose gradients autograd sums: outputs and patch gradient bit
    for bit, also with only one of the two outputs used."""
    ld, mpm, sy = pkg_mod("load_data"), pkg_mod("median_pool"), pkg_mod("synthetic")
    patch = sy.patch(P, seed=21).to(DEV)
    colors = ld.NPSCalculator(pkg_mod("patch_config").patch_configs["paper_obj"]().printfile, P).colors.to(DEV)
    gen = torch.Generator().manual_seed(22)
    g_mp = torch.randn(3, P, P, generator=gen).to(DEV)
    g3 = torch.tensor([0.37, -1.25, 0.81]).to(DEV)
    pool = mpm.MedianPool2d(7, same=True)
    for use in ("both", "mp", "reg"):
        a = patch.clone().requires_grad_(True)
        mp_a, reg_a = ld.patch_front(a, colors)
        b = patch.clone().requires_grad_(True)
        mp_b, reg_b = pool(b.unsqueeze(0)).squeeze(0), ld.regularisers(b, colors)
        assert torch.equal(mp_a, mp_b) and torch.equal(reg_a, reg_b)
        la = (mp_a * g_mp).sum() if use != "reg" else 0
        lb = (mp_b * g_mp).sum() if use != "reg" else 0
        if use != "mp":
            la = la + (reg_a * g3).sum()
            lb = lb + (reg_b * g3).sum()
        la.backward()
        lb.backward()
        assert torch.equal(a.grad, b.grad), use


@pytest.mark.parametrize("kind", ["uniform", "ties", "zeros", "nan"])
def test_median7_network_matches_counting_kernel(kind):
    """po_median7_fwd (bitonic network + first-position scan; the counting
    rule only in windows holding a NaN) equals the general kernel
    po_median_fwd (rank by counting) with the same 7x7 reflect-3 geometry,
    values and arguments, on windows full of ties, of signed zeros and with
    NaNs."""
    nat = pkg_mod("_native")
    gen = torch.Generator().manual_seed(31)
    C, H, W = 3, 61, 45
    x = torch.rand(C, H, W, generator=gen)
    if kind == "ties":
        x = (x * 4).floor() / 4
    elif kind == "zeros":
        x = torch.where(x < 0.5, torch.zeros_like(x), -torch.zeros_like(x))
        x[0, 5, 5] = 1.0
    elif kind == "nan":
        x[x < 0.01] = float("nan")
    x = x.to(DEV)
    outs = []
    for name in ("po_median7_fwd", "po_median_fwd"):
        y = torch.full((C, H, W), 7.0, device=DEV)
        arg = torch.full((C, H, W), -1, dtype=torch.int32, device=DEV)
        if name == "po_median7_fwd":
            nat.call(name, nat.ptr(x), C, H, W, nat.ptr(y), nat.ptr(arg, torch.int32), nat.stream())
        else:
            nat.call(name, nat.ptr(x), C, H, W, 7, 7, 1, 1, 3, 3, 3, 3, nat.ptr(y), nat.ptr(arg, torch.int32),
                     nat.stream())
        torch.cuda.synchronize()
        outs.append((y, arg))
    (y7, a7), (yg, ag) = outs
    assert torch.equal(a7, ag)
    assert torch.equal(y7.nan_to_num(5.0), yg.nan_to_num(5.0))
    assert torch.equal(torch.signbit(y7), torch.signbit(yg))


def test_no_grad_forward_skips_the_factor_buffer(monkeypatch):
    """A warp forward that no backward can follow (torch.no_grad(), or a patch
    that does not require grad) runs po_warp_box_fwd_keyed and allocates no
    [B,S,S,4] factor buffer; a training forward runs po_warp_box_fwd_fac
    (needs_input_grad is True inside Function.forward even under
    no_grad, so the caller passes torch.is_grad_enabled())."""
    ld, sy, nat = pkg_mod("load_data"), pkg_mod("synthetic"), pkg_mod("_native")
    B, S, P = 3, 96, 32
    keyed = {k: v for k, v in sy.draws_device(5, 1, 0, B, P, DEV).items() if k != "noise"}
    keyed["noise_key"] = (5, 1, 0)
    img, lab = sy.frames(B, S, seed=1).to(DEV), sy.labels(B, seed=2).to(DEV)
    patch = sy.patch(P, seed=3).to(DEV).requires_grad_(True)
    seen = []
    real = nat.call
    monkeypatch.setattr(nat, "call", lambda name, *a: (seen.append(name), real(name, *a))[1])
    pt = ld.PatchTransformer()
    with torch.no_grad():
        pt.forward_composite(patch, lab, img, S, draws=keyed, sparse=True)
    pt.forward_composite(patch.detach(), lab, img, S, draws=keyed, sparse=True)
    assert "po_warp_box_fwd_fac" not in seen and seen.count("po_warp_box_fwd_keyed") == 2, seen
    seen.clear()
    out, _ = pt.forward_composite(patch, lab, img, S, draws=keyed, sparse=True)
    assert "po_warp_box_fwd_fac" in seen, seen
    out.sum().backward()
    assert "po_warp_box_bwd_fac" in seen and bool((patch.grad != 0).any())


@pytest.mark.parametrize("B", [5, 40])
def test_bwd_mixed_geometry_batch(B):
    """Phase B of the warp backward reads each image's sample-point form from
    its affine row: a batch mixing reference-form and float64-form rows gives
    the sum of the two single-form sub-batches' gradients (to fp32 summation
    order: 1e-5 relative), and repeated runs give the same bits."""
    ld, sy, nat = pkg_mod("load_data"), pkg_mod("synthetic"), pkg_mod("_native")
    S, P = 96, 32
    dr = sy.draws_device(7, 2, 0, B, P, DEV)
    lab = sy.labels(B, seed=3).to(DEV)
    mp = sy.patch(P, seed=4).to(DEV).contiguous()
    _, _, _, roi_r, aff_r = ld.patch_params(lab, S, P, dr, True, with_roi=True, geometry="ref")
    _, _, _, roi_f, aff_f = ld.patch_params(lab, S, P, dr, True, with_roi=True, geometry="f64")
    pick = (torch.arange(B, device=DEV) % 2 == 0)
    aff_m = torch.where(pick[:, None], aff_r, aff_f).contiguous()
    roi_m = torch.where(pick[:, None], roi_r, roi_f).contiguous()
    d_out = torch.randn(B, 3, S, S, device=DEV, generator=torch.Generator(DEV).manual_seed(1))
    st = nat.stream()

    def grad(aff, roi, keep):
        d = d_out * keep[:, None, None, None]
        out = torch.empty(B, 3, S, S, device=DEV)
        fac = torch.empty(B * S * S * 4, device=DEV)
        d_mp = torch.full((3, P, P), float("nan"), device=DEV)
        key = (7, 2, 0)
        nat.call("po_warp_box_fwd_fac", nat.ptr(torch.zeros(B, 3, S, S, device=DEV)), nat.ptr(mp), *key,
                 nat.ptr(dr["contrast"]), nat.ptr(dr["bright"]), nat.ptr(aff, torch.float64),
                 nat.ptr(roi, torch.int32), B, S, P, 1, 1, nat.ptr(out), nat.ptr(fac), st)
        nat.call("po_warp_box_bwd_fac", nat.ptr(d.contiguous()), nat.ptr(mp), *key, nat.ptr(dr["contrast"]),
                 nat.ptr(dr["bright"]), nat.ptr(aff, torch.float64), nat.ptr(roi, torch.int32), B, S, P,
                 nat.ptr(fac), nat.ptr(d_mp), st)
        torch.cuda.synchronize()
        return d_mp

    ones = torch.ones(B, device=DEV)
    g_mixed = grad(aff_m, roi_m, ones)
    g_ref_part = grad(aff_r, roi_r, pick.float())
    g_f64_part = grad(aff_f, roi_f, (~pick).float())
    assert torch.isfinite(g_mixed).all()
    want = g_ref_part + g_f64_part
    assert torch.allclose(g_mixed, want, rtol=1e-5, atol=1e-6 * float(want.abs().max())), \
        float((g_mixed - want).abs().max())
    # repeatable bits
    assert torch.equal(grad(aff_r, roi_r, ones), grad(aff_r, roi_r, ones))
