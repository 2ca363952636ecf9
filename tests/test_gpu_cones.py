"""Gradient cones (po_grad_boxes + po_conv gbox): the patch gradient only needs
dL/d(image) on the patch footprint, so the input-gradient convs of the early
stages compute their output only on the footprint's forward influence cone.

Checked here: the device cone evaluation against its host restatement
(NetPlan.cone_boxes_host), a boxed po_conv against the unboxed launch (inside
the box: identical values; outside: untouched), and a training step with
cones against one without (the same forward; the patch gradient agrees to
fp32 reassociation, the tiles being tuned per plan and launch kind)."""
import ctypes

import pytest
import torch

from conftest import pkg_mod

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _conv(nat, x, wt, shift, slot, bias, dst, box, prec, tile, ks, geo):
    """One po_conv launch; geo = (Hin, Hout, Hg, out_step, out_oy, out_ox)."""
    B, Hin, _, Cin = x.shape
    Cout = dst.shape[-1]
    _, Hout, Hg, step, oy, ox = geo
    d = nat.po_conv_desc()
    d.B, d.Hin, d.Win, d.Cin_p, d.Hout, d.Wout, d.Cout_p, d.Hg, d.Wg = B, Hin, Hin, Cin, Hout, Hout, Cout, Hg, Hg
    d.in_step, d.out_step, d.out_oy, d.out_ox, d.ntaps, d.N, d.act, d.tile = 1, step, oy, ox, 9, Cout, 1, tile
    for kh in range(3):
        for kw in range(3):
            d.dh[kh * 3 + kw], d.dw[kh * 3 + kw] = kh - 1, kw - 1
    ws = torch.empty(max(ks, 1) * B * Hg * Hg * Cout, device=DEV)
    d.ksplit, d.workspace = ks, ws.data_ptr()
    d.prec, d.w_shift = prec, shift
    d.in_amax = slot.data_ptr() if slot is not None else None
    d.gbox = box.data_ptr() if box is not None else None
    nat.call("po_conv", ctypes.byref(d), nat.ptr(x), nat.ptr(wt, wt.dtype), nat.ptr(bias), nat.ptr(dst), None,
             None, None, None, None, nat.stream())
    torch.cuda.synchronize()


@pytest.mark.parametrize("prec,tile", [(0, 1), (0, 3), (0, 9), (0, 11), (0, 13), (0, 17), (0, 19), (1, 34), (1, 46),
                                       (1, 29)])
@pytest.mark.parametrize("ks", [1, 3])
@pytest.mark.parametrize("geo", [(21, 21, 21, 1, 0, 0), (11, 22, 11, 2, 1, 0)])
def test_boxed_conv_matches_full_launch(prec, tile, ks, geo):
    """Boxed launches of every tile family the plans use; image 1's box is
    the whole 21x21 map, whose 441 rows end inside a 128-row tile."""
    from test_gpu_darknet import _conv_operands
    nat = pkg_mod("_native")
    B, Cin, Cout = 4, 64, 64
    Hin, Hout = geo[0], geo[1]
    gen = torch.Generator().manual_seed(5)
    x = torch.randn(B, Hin, Hin, Cin, generator=gen)
    w = torch.randn(Cout, 9, Cin, generator=gen) * (2.0 / (9 * Cin)) ** 0.5
    bias = (torch.randn(Cout, generator=gen) * 0.1).to(DEV)
    wt, shift, slot = _conv_operands(nat, w.to(DEV), x.permute(0, 3, 1, 2), prec)
    xd = x.to(DEV)
    # image 0: an inner box, 1: the whole map, 2: empty, 3: a box touching the corner
    boxes = torch.tensor([[3, 5, 12, 17], [0, 0, Hout, Hout], [7, 7, 7, 9], [Hout - 4, 0, Hout, 6]],
                         dtype=torch.int32)
    full = torch.full((B, Hout, Hout, Cout), float("nan"), device=DEV)
    boxed = torch.full_like(full, float("nan"))
    _conv(nat, xd, wt, shift, slot, bias, full, None, prec, tile, ks, geo)
    _conv(nat, xd, wt, shift, slot, bias, boxed, boxes.to(DEV), prec, tile, ks, geo)
    full, boxed = full.cpu(), boxed.cpu()
    inside = torch.zeros(B, Hout, Hout, dtype=torch.bool)
    for b, (r0, c0, r1, c1) in enumerate(boxes.tolist()):
        inside[b, r0:r1, c0:c1] = True
    written = ~torch.isnan(full[..., 0])                 # the grid's destination pixels
    assert torch.equal(boxed[inside & written], full[inside & written])
    assert torch.isnan(boxed[~(inside & written)]).all()


def test_grad_boxes_match_host_restatement(tmp_path):
    from test_gpu_darknet import _net
    net, _ = _net("builtin:yolov3-dota", tmp_path)
    B, S = 5, 608
    plan = net.plan(B, S, S, DEV)
    assert plan.cone_blocks, "the 304/152/76 stages should be boxed"
    gen = torch.Generator().manual_seed(3)
    roi = []
    for b in range(B):
        x0, y0 = int(torch.randint(0, S - 8, (1,), generator=gen)), int(torch.randint(0, S - 8, (1,), generator=gen))
        x1, y1 = x0 + int(torch.randint(1, S - x0 + 1, (1,), generator=gen)), \
            y0 + int(torch.randint(1, S - y0 + 1, (1,), generator=gen))
        roi.append([x0, y0, x1, y1])
    roi[0] = [0, 0, S, S]
    roi[1] = [300, 300, 301, 301]
    plan.set_cones(torch.tensor(roi, dtype=torch.int32, device=DEV))
    got = plan.cone_boxes.cpu()
    prog = plan._cone_prog()
    for b in range(B):
        want = plan.cone_boxes_host(prog, plan.n, roi[b])
        for j, box in want.items():
            assert tuple(got[j, b].tolist()) == box, (b, j)
    # the whole image as footprint: every cone is its full map
    plan.set_cones(None)
    for j in plan.cone_blocks:
        H, W = plan.shp[j][:2]
        assert plan.cone_boxes[j].cpu().tolist() == [[0, 0, H, W]] * B


@pytest.mark.parametrize("cfg,S,prec", [("builtin:yolov3-dota", 608, "fp32"), ("builtin:yolov3-dota", 608, "fp16x3"),
                                        ("builtin:yolov3-tiny-dota", 416, "fp32"),
                                        ("builtin:yolov3-tiny-dota", 416, "fp16x3")])
def test_cones_leave_the_patch_gradient_unchanged(tmp_path, monkeypatch, cfg, S, prec):
    """With the built-in tile choice (no autotuning) the boxed dgrads run the
    same tiles as the full ones: exact fp32 operands give the identical patch
    gradient; fp16x3 differs only through the max|x| operand scales (a boxed
    launch bounds the values it writes, a full one the whole map)."""
    from test_gpu_step import _trainer
    sy = pkg_mod("synthetic")
    B, P = 3, 224
    monkeypatch.setenv("ADVPATCH_TUNE", "0")
    out = []
    for cones in ("1", "0"):
        monkeypatch.setenv("ADVPATCH_GRAD_CONES", cones)
        tr, _ = _trainer(cfg, tmp_path, prec=prec)
        img, lab = sy.frames(B, S, seed=90).to(DEV), sy.labels(B, seed=91).to(DEV)
        dr = {k: v.to(DEV) for k, v in sy.draws(B, P, seed=93).items()}
        pg = sy.patch(P, seed=92).to(DEV).requires_grad_(True)
        loss, terms = tr.losses(pg, img, lab, dr)
        loss.backward()
        assert bool(tr.last_plan.cone_blocks) == (cones == "1")
        out.append((float(loss.detach()), terms["cells"].tolist(), pg.grad.detach().clone()))
    (l1, c1, g1), (l0, c0, g0) = out
    assert c1 == c0 and l1 == l0                  # the same forward
    if prec == "fp32":
        assert torch.equal(g1, g0)
    else:
        rel = float((g1 - g0).abs().max() / g0.abs().max())
        assert rel < 1e-5, rel


@pytest.mark.parametrize("stride,H,W", [(2, 22, 18), (1, 13, 13)])
def test_boxed_maxpool_bwd_matches_full(stride, H, W):
    """po_maxpool2_bwd_box: inside each image's box the values of the full
    po_maxpool2_bwd (accumulate + leaky mask), outside it d_src untouched;
    an empty box writes nothing, boxes == NULL is the full kernel."""
    nat = pkg_mod("_native")
    B, C, Cp = 4, 20, 32
    Ho, Wo = (H // 2, W // 2) if stride == 2 else (H, W)
    gen = torch.Generator().manual_seed(11)
    src = torch.randn(B, H, W, Cp, generator=gen).to(DEV)
    dst = torch.empty(B, Ho, Wo, Cp, device=DEV)
    am = torch.zeros(B, Ho, Wo, Cp, dtype=torch.int8, device=DEV)
    nat.call("po_maxpool2_fwd", nat.ptr(src), B, H, W, C, Cp, stride, nat.ptr(dst), nat.ptr(am, torch.int8), None,
             nat.stream())
    g = torch.randn(B, Ho, Wo, Cp, generator=gen).to(DEV)
    prev = torch.randn(B, H, W, Cp, generator=gen).to(DEV)
    mask = torch.randn(B, H, W, Cp, generator=gen).to(DEV)
    boxes = torch.tensor([[2, 3, 9, 11], [0, 0, H, W], [5, 5, 5, 8], [H - 3, W - 4, H + 2, W + 5]],
                         dtype=torch.int32, device=DEV)
    full, boxed, nobox = prev.clone(), prev.clone(), prev.clone()
    nat.call("po_maxpool2_bwd", nat.ptr(g), nat.ptr(am, torch.int8), B, H, W, C, Cp, stride, nat.ptr(full), 1,
             nat.ptr(mask), None, nat.stream())
    nat.call("po_maxpool2_bwd_box", nat.ptr(g), nat.ptr(am, torch.int8), B, H, W, C, Cp, stride, nat.ptr(boxed), 1,
             nat.ptr(mask), nat.ptr(boxes, torch.int32), None, nat.stream())
    nat.call("po_maxpool2_bwd_box", nat.ptr(g), nat.ptr(am, torch.int8), B, H, W, C, Cp, stride, nat.ptr(nobox), 1,
             nat.ptr(mask), None, None, nat.stream())
    torch.cuda.synchronize()
    assert torch.equal(nobox, full)
    inside = torch.zeros(B, H, W, dtype=torch.bool)
    for b, (r0, c0, r1, c1) in enumerate(boxes.cpu().tolist()):
        inside[b, max(r0, 0):min(r1, H), max(c0, 0):min(c1, W)] = True
    inside = inside.to(DEV)
    assert torch.equal(boxed[inside], full[inside])
    assert torch.equal(boxed[~inside], prev[~inside])


@pytest.mark.parametrize("H,W", [(22, 18), (21, 17), (416, 416)])
def test_boxed_maxpool_bwd_slope_bytes(H, W):
    """The first pool's form (argmax bytes carrying the LeakyReLU slope, no
    mask, no accumulate) on even maps (the one-thread-per-window stride-2
    kernel) and odd maps (the gathering kernel): inside the box bit-identical
    to the full po_maxpool2_bwd, the max|x| slot = max |d_src| over the box."""
    nat = pkg_mod("_native")
    B, C, Cp = 3, 13, 16
    Ho, Wo = H // 2, W // 2
    gen = torch.Generator().manual_seed(H + W)
    g = torch.randn(B, Ho, Wo, Cp, generator=gen)
    g[0, 0, 0, :4] = -0.0                                         # signed zeros go through 0 + g
    am = (torch.randint(0, 4, (B, Ho, Wo, Cp), generator=gen) | 8
          | (torch.randint(0, 2, (B, Ho, Wo, Cp), generator=gen) * 4)).to(torch.int8)
    g, am = g.to(DEV), am.to(DEV)
    prev = torch.randn(B, H, W, Cp, generator=gen).to(DEV)
    boxes = torch.tensor([[1, 3, H - 2, W - 1], [0, 0, H, W], [H // 2, W // 3, H // 2 + 3, W // 3 + 5]],
                         dtype=torch.int32, device=DEV)
    full, boxed = prev.clone(), prev.clone()
    slot = torch.zeros(64, dtype=torch.int32, device=DEV)
    nat.call("po_maxpool2_bwd", nat.ptr(g), nat.ptr(am, torch.int8), B, H, W, C, Cp, 2, nat.ptr(full), 0, None,
             None, nat.stream())
    nat.call("po_maxpool2_bwd_box", nat.ptr(g), nat.ptr(am, torch.int8), B, H, W, C, Cp, 2, nat.ptr(boxed), 0,
             None, nat.ptr(boxes, torch.int32), nat.ptr(slot, torch.int32), nat.stream())
    torch.cuda.synchronize()
    inside = torch.zeros(B, H, W, dtype=torch.bool)
    for b, (r0, c0, r1, c1) in enumerate(boxes.cpu().tolist()):
        inside[b, max(r0, 0):min(r1, H), max(c0, 0):min(c1, W)] = True
    inside = inside.to(DEV)
    assert torch.equal(boxed[inside].view(torch.int32), full[inside].view(torch.int32))
    assert torch.equal(boxed[~inside], prev[~inside])
    assert float(slot.max().reshape(1).view(torch.float32)[0]) == float(full[inside].abs().max())


def test_halo_tiles_refuse_boxes():
    """The halo kernel maps tile rows to contiguous pixels: a boxed launch
    must be refused (the autotuner then skips it), not computed wrongly."""
    from test_gpu_darknet import _conv_operands
    nat = pkg_mod("_native")
    x = torch.randn(2, 9, 9, 32, device=DEV)
    w = torch.randn(32, 9, 32, device=DEV)
    wt, shift, slot = _conv_operands(nat, w, x.permute(0, 3, 1, 2).cpu(), 1)
    box = torch.tensor([[0, 0, 4, 4]] * 2, dtype=torch.int32, device=DEV)
    y = torch.zeros(2, 9, 9, 32, device=DEV)
    with pytest.raises(RuntimeError, match="halo"):
        _conv(nat, x, wt, shift, slot, torch.zeros(32, device=DEV), y, box, 1, 53, 1, (9, 9, 9, 1, 0, 0))


@pytest.mark.parametrize("prec", ["fp32", "fp16x3"])
def test_support_box_grid_leaves_the_patch_gradient_unchanged(tmp_path, monkeypatch, prec):
    """yolov3-tiny's dgrad from the 13x13 head window into the full 13x13 map
    of block 11 runs over the window dilated by the taps only (po_conv mrows +
    per-step gbox, destination zero-filled): the same patch gradient as the
    full-map launch (ADVPATCH_SUPPORT_BOX=0) — bit for bit with exact fp32
    operands, within the operand-scale effect for fp16x3."""
    from test_gpu_step import _trainer
    sy = pkg_mod("synthetic")
    B, P, S = 5, 224, 416
    monkeypatch.setenv("ADVPATCH_TUNE", "0")
    out = []
    for sup in ("1", "0"):
        monkeypatch.setenv("ADVPATCH_SUPPORT_BOX", sup)
        tr, _ = _trainer("builtin:yolov3-tiny-dota", tmp_path, prec=prec)
        img, lab = sy.frames(B, S, seed=70).to(DEV), sy.labels(B, seed=71).to(DEV)
        dr = {k: v.to(DEV) for k, v in sy.draws(B, P, seed=73).items()}
        pg = sy.patch(P, seed=72).to(DEV).requires_grad_(True)
        loss, terms = tr.losses(pg, img, lab, dr)
        loss.backward()
        plan = tr.last_plan
        assert bool(plan.support) == (sup == "1")
        if sup == "1":
            for box, j, src, b0, nb, _, _ in plan.support:
                bx = box.cpu()
                assert bool(((bx[:, 2] - bx[:, 0]) * (bx[:, 3] - bx[:, 1]) <= 25).all())
        out.append((float(loss.detach()), pg.grad.detach().clone()))
    (l1, g1), (l0, g0) = out
    assert l1 == l0
    if prec == "fp32":
        assert torch.equal(g1, g0)
    else:
        rel = float((g1 - g0).abs().max() / g0.abs().max())
        assert rel < 1e-5, rel


@pytest.mark.parametrize("prec", ["fp32", "fp16x3"])
def test_conv_pool_fusion_leaves_the_step_unchanged(tmp_path, monkeypatch, prec):
    """yolov3-tiny's conv + 2x2/2 max pool pairs (blocks 2/3, 4/5, 6/7 with exact
    fp32 operands, 2/3 and 4/5 with fp16x3; darknet_v3.py:61-69) with the pool in the conv epilogue (po_conv_desc.pool_y,
    pool-order grid; the conv output is never stored, the argmax bytes carry
    the LeakyReLU slope): the same loss, pool outputs, window positions and
    patch gradient as the separate po_maxpool2_fwd (ADVPATCH_CONV_POOL=0) — bit
    for bit with exact fp32 operands."""
    from test_gpu_step import _trainer
    sy = pkg_mod("synthetic")
    B, P, S = 3, 224, 416
    monkeypatch.setenv("ADVPATCH_TUNE", "0")
    out = []
    for fuse in ("1", "0"):
        monkeypatch.setenv("ADVPATCH_CONV_POOL", fuse)
        tr, _ = _trainer("builtin:yolov3-tiny-dota", tmp_path, prec=prec)
        img, lab = sy.frames(B, S, seed=60).to(DEV), sy.labels(B, seed=61).to(DEV)
        dr = {k: v.to(DEV) for k, v in sy.draws(B, P, seed=63).items()}
        pg = sy.patch(P, seed=62).to(DEV).requires_grad_(True)
        loss, terms = tr.losses(pg, img, lab, dr)
        loss.backward()
        plan = tr.last_plan
        fused = ([2, 4, 6] if prec == "fp32" else [2, 4]) if fuse == "1" else []
        assert sorted(plan.conv_pool) == fused
        pools = {j: (plan.act[j].clone(), plan.argmax[j].long() & 3) for j in (3, 5, 7)}
        out.append((float(loss.detach()), pools, pg.grad.detach().clone()))
    (l1, p1, g1), (l0, p0, g0) = out
    if prec == "fp32":
        assert l1 == l0
        for j in (3, 5, 7):
            assert torch.equal(p1[j][0], p0[j][0]) and torch.equal(p1[j][1], p0[j][1])
        assert torch.equal(g1, g0)
    else:
        rel = float((g1 - g0).abs().max() / g0.abs().max())
        assert rel < 1e-5, rel


@pytest.mark.parametrize("cfg,S,B", [("builtin:yolov3-dota", 608, 5), ("builtin:yolov3-tiny-dota", 416, 7)])
def test_support_boxes_kernel_matches_torch_restatement(tmp_path, monkeypatch, cfg, S, B):
    """po_support_boxes (every compact dgrad grid's boxes in one launch) equals
    the torch-op restatement NetPlan.set_support_boxes_torch after a training
    forward + backward (windows placed, cones evaluated)."""
    from test_gpu_step import _trainer
    sy = pkg_mod("synthetic")
    P = 224
    monkeypatch.setenv("ADVPATCH_TUNE", "0")
    tr, _ = _trainer(cfg, tmp_path)
    img, lab = sy.frames(B, S, seed=40).to(DEV), sy.labels(B, seed=41).to(DEV)
    dr = {k: v.to(DEV) for k, v in sy.draws(B, P, seed=43).items()}
    pg = sy.patch(P, seed=42).to(DEV).requires_grad_(True)
    loss, _ = tr.losses(pg, img, lab, dr)
    loss.backward()
    plan = tr.last_plan
    if not plan.support:
        pytest.skip("no compact dgrad grid in this plan")
    for box, *_ in plan.support:
        box.fill_(-7)
    plan.set_support_boxes()
    got = [e[0].clone() for e in plan.support]
    for box, *_ in plan.support:
        box.fill_(-7)
    plan.set_support_boxes_torch()
    for g, (box, *_) in zip(got, plan.support):
        assert torch.equal(g, box)

