"""GPU parity of the Darknet stack (implicit-GEMM fp32 MFMA conv forward and
input-gradient, route/shortcut/upsample/maxpool) against the oracle's
PyTorch-CPU fp32 forward and autograd backward on the same synthetic weights.

Two fp32 implementations can take different LeakyReLU slopes (or maxpool
arguments) where a pre-activation is within rounding of a tie; through a deep
random network one such flip moves the input gradient by up to ~5e-2 relative
(the fp32 oracle itself differs that much from a float64 run on yolov3-dota).
So the backward is checked on aligned branches: the oracle is re-run with the
branch decisions the HIP forward took, and separately every disagreeing
branch is checked to be a rounding tie (|x| <= 1e-5 * max|x| of its layer).
"""
import pytest
import torch

import oracle
from conftest import assert_branch_ties_only, pkg_mod, plan_branches

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda", 0)


def _net(cfg, tmp_path, seed=4, prec="fp16x3"):
    dk, W, G = pkg_mod("darknet_v3"), pkg_mod("weights"), pkg_mod("cfg_gen")
    path = str(tmp_path / "w.weights")
    W.write_weights(path, W.synthesize(cfg, seed=seed))
    net = dk.Darknet(cfg)
    net.conv_prec = prec
    net.load_darknet_weights(path)
    ref = oracle.OracleDarknet(G.cfg_text(cfg), path)
    return net, ref


def _rel(a, b):
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


def _check(cfg, B, tmp_path, fwd_tol=5e-5, bwd_tol=1e-4, prec="fp16x3"):
    net, ref = _net(cfg, tmp_path, prec=prec)
    S = net.height
    x = pkg_mod("synthetic").frames(B, S, seed=7)
    xg = x.to(DEV).requires_grad_(True)
    outs = net(xg)
    plan = net.plan(B, S, S, DEV)
    br = plan_branches(plan)
    rec = {}
    with torch.no_grad():
        outs_nat = ref(x, record=rec)
    for o, r in zip(outs, outs_nat):
        assert o.shape == r.shape
        assert _rel(o.detach().cpu(), r) < fwd_tol
    assert_branch_ties_only(br, rec)
    xr = x.clone().requires_grad_(True)
    outs_ref = ref(xr, branch=br)
    gen = torch.Generator().manual_seed(9)
    grads = [torch.randn(o.shape, generator=gen) for o in outs_ref]
    sum((o * g).sum() for o, g in zip(outs_ref, grads)).backward()
    sum((o * g.to(DEV)).sum() for o, g in zip(outs, grads)).backward()
    assert _rel(xg.grad.cpu(), xr.grad) < bwd_tol
    # every max|x| slot bounds its tensor (the fp16x3 operand scales rely on
    # it; exact-fp32 plans keep no slots)
    for t in (plan.act + plan.grad if prec == "fp16x3" else []):
        if t is not None:
            bound = float(plan.amax[plan._slot_idx[t.data_ptr()]].view(torch.float32).max())
            assert float(t.abs().max()) <= bound


PRECS = ["fp16x3", "fp32"]


@pytest.mark.parametrize("prec", PRECS)
def test_mini3_fwd_bwd(tmp_path, prec):
    _check("builtin:mini3", 3, tmp_path, prec=prec)


def test_mini3_96_batch5(tmp_path):
    _check("builtin:mini3-96", 5, tmp_path)


@pytest.mark.parametrize("prec", PRECS)
def test_tiny_dota_416(tmp_path, prec):
    # maxpool s2 and the ZeroPad2d + maxpool s1 block of yolov3-tiny
    _check("builtin:yolov3-tiny-dota", 2, tmp_path, prec=prec)


@pytest.mark.parametrize("prec", PRECS)
def test_yolov3_dota_608(tmp_path, prec):
    _check("builtin:yolov3-dota", 1, tmp_path, prec=prec)


def test_conv_tile_variants(tmp_path):
    """Chains that hit every po_conv tile shape (N=32/64/128+, large/small M,
    stride-2 dgrad parity classes, odd spatial sizes, a non-fused shortcut)."""
    G = pkg_mod("cfg_gen")
    text = G._net(70) + G._conv(32, 3) + G._conv(64, 3, 2) + G._conv(48, 1) + G._conv(128, 3) + \
        G._conv(256, 3, 2) + G._conv(96, 1) + G._conv(128, 3, 2) + G._conv(96, 1) + G._conv(128, 3) + \
        G._shortcut(-3) + G._conv(60, 1, bn=False, act="linear") + G._yolo("0,1,2", G.DOTA_ANCHORS, 15, 9)
    p = tmp_path / "chain.cfg"
    p.write_text(text)
    _check(str(p), 3, tmp_path)


def test_large_m_tiles(tmp_path):
    """Big-M layers (128x128 / 128x64 tiles, XCD remap over thousands of workgroups)."""
    G = pkg_mod("cfg_gen")
    text = G._net(256) + G._conv(32, 3) + G._conv(64, 3) + G._conv(128, 3, 2) + G._conv(256, 3) + \
        G._conv(60, 1, bn=False, act="linear") + G._yolo("0,1,2", G.DOTA_ANCHORS, 15, 9)
    p = tmp_path / "big.cfg"
    p.write_text(text)
    _check(str(p), 2, tmp_path)


def test_heads_layout_matches_reference_view(tmp_path):
    # channel = anchor*20 + field, as train_patch.py:459 views it
    net, ref = _net("builtin:mini3", tmp_path)
    x = pkg_mod("synthetic").frames(2, 64, seed=8)
    heads_nhwc, plan = net.forward_nhwc(x.to(DEV))
    outs = ref(x)
    for h, r in zip(heads_nhwc, outs):
        hc = h.detach().cpu()[..., :60].permute(0, 3, 1, 2)
        assert _rel(hc, r) < 2e-5


def _conv_operands(nat, wd, x, prec):
    """(weight tensor, shift, amax slot) of a direct po_conv call: fp32 weights
    for prec 0, the split fp16 planes and max|x| slot for prec 1 (fp16x3)."""
    if prec == 0:
        return wd, 0, None
    w16, shift = pkg_mod("darknet_v3").Darknet._split16(wd)
    slot = torch.zeros(64, dtype=torch.int32)
    slot[5] = torch.tensor([float(x.abs().max())], dtype=torch.float32).view(torch.int32)   # any sub-slot
    slot = slot.to(DEV)
    return w16, shift, slot


@pytest.mark.parametrize("prec,tile", [(0, 0), (1, 0), (1, 53), (1, 54)])
@pytest.mark.parametrize("B,H,Cin,Cout,k", [(4, 5, 512, 1024, 3), (16, 1, 1024, 64, 1), (3, 7, 96, 128, 3)])
def test_split_k_matches_single_pass(B, H, Cin, Cout, k, prec, tile):
    """po_conv with the k-steps split over workgroups (partials reduced in
    split order by the epilogue kernel) against one pass and torch conv2d,
    for both operand precisions, with the default tile and with the halo
    kernel's tiles (whose split ranges start on odd channel chunks)."""
    import ctypes
    if tile and k != 3:
        pytest.skip("the halo kernel takes 3x3 convs only")
    nat = pkg_mod("_native")
    pad = (k - 1) // 2
    gen = torch.Generator().manual_seed(11)
    x = torch.randn(B, Cin, H, H, generator=gen)
    w = torch.randn(Cout, Cin, k, k, generator=gen) * (2.0 / (Cin * k * k)) ** 0.5
    bias = torch.randn(Cout, generator=gen) * 0.1
    ref = torch.nn.functional.leaky_relu(torch.nn.functional.conv2d(x.double(), w.double(), bias.double(),
                                                                    padding=pad), 0.1)
    xd = x.permute(0, 2, 3, 1).contiguous().to(DEV)
    wd = w.permute(0, 2, 3, 1).reshape(Cout, k * k, Cin).contiguous().to(DEV)
    wt, shift, slot = _conv_operands(nat, wd, x, prec)
    bd = bias.to(DEV)
    outs = {}
    for ks in (1, 2, 5, 8):
        y = torch.full((B, H, H, Cout), float("nan"), device=DEV)
        ws = torch.empty(ks * B * H * H * Cout, device=DEV)
        yslot = torch.zeros(64, dtype=torch.int32, device=DEV)
        d = nat.po_conv_desc()
        d.B, d.Hin, d.Win, d.Cin_p, d.Hout, d.Wout, d.Cout_p, d.Hg, d.Wg = B, H, H, Cin, H, H, Cout, H, H
        d.in_step, d.out_step, d.ntaps, d.N, d.act, d.tile = 1, 1, k * k, Cout, 1, tile
        for kh in range(k):
            for kw in range(k):
                d.dh[kh * k + kw], d.dw[kh * k + kw] = kh - pad, kw - pad
        d.ksplit, d.workspace = ks, ws.data_ptr()
        d.prec, d.w_shift = prec, shift
        d.in_amax = slot.data_ptr() if slot is not None else None
        d.y_amax = yslot.data_ptr()
        nat.call("po_conv", ctypes.byref(d), nat.ptr(xd), nat.ptr(wt, wt.dtype), nat.ptr(bd), nat.ptr(y), None,
                 None, None, None, None, nat.stream())
        outs[ks] = y.permute(0, 3, 1, 2).cpu()
        assert float(yslot.cpu().view(torch.float32).max()) == float(y.abs().max())      # max|y| slot
    for ks, y in outs.items():
        assert _rel(y.double(), ref) < 1e-5, (ks, _rel(y.double(), ref))
        assert _rel(y, outs[1]) < 1e-5, (ks, _rel(y, outs[1]))


@pytest.mark.parametrize("tile", list(range(1, 61)))
def test_every_conv_tile(tile):
    """Every po_conv tile (exact fp32: register-staged 1..10, LDS-DMA-staged
    11..20 and 27 — the retired 21..26 and 28 are refused; fp16x3: 29..45, LDS-DMA 46..52, halo 53..54,
    2-D halo 55..56, fragment-weight 2-D halo 57..60) on a 3x3 conv with zero
    padding, a ragged pixel count and a ragged channel count, against a
    float64 torch conv2d."""
    import ctypes
    nat = pkg_mod("_native")
    bm, bn, bk, pr = (ctypes.c_int() for _ in range(4))
    nat.call("po_conv_tile_info", tile, ctypes.byref(bm), ctypes.byref(bn), ctypes.byref(bk), ctypes.byref(pr))
    retired = pr.value < 0
    pr.value = max(pr.value, 0)
    B, H, Cin, Cout, k = 3, 7, 128 if bk.value == 64 else 96, 96, 3
    gen = torch.Generator().manual_seed(tile)
    x = torch.randn(B, Cin, H, H, generator=gen)
    w = torch.randn(Cout, Cin, k, k, generator=gen) * (2.0 / (Cin * k * k)) ** 0.5
    bias = torch.randn(Cout, generator=gen) * 0.1
    ref = torch.nn.functional.conv2d(x.double(), w.double(), bias.double(), padding=1)
    y = torch.full((B, H, H, Cout), float("nan"), device=DEV)
    d = nat.po_conv_desc()
    d.B, d.Hin, d.Win, d.Cin_p, d.Hout, d.Wout, d.Cout_p, d.Hg, d.Wg = B, H, H, Cin, H, H, Cout, H, H
    d.in_step, d.out_step, d.ntaps, d.N, d.act, d.tile = 1, 1, 9, Cout, 0, tile
    for kh in range(3):
        for kw in range(3):
            d.dh[kh * 3 + kw], d.dw[kh * 3 + kw] = kh - 1, kw - 1
    xd = x.permute(0, 2, 3, 1).contiguous().to(DEV)
    wd = w.permute(0, 2, 3, 1).reshape(Cout, 9, Cin).contiguous().to(DEV)
    wt, shift, slot = _conv_operands(nat, wd, x, pr.value)
    d.prec, d.w_shift = pr.value, shift
    d.in_amax = slot.data_ptr() if slot is not None else None
    wf = _frag(wt) if pr.value == 1 else None
    d.Wfrag = wf.data_ptr() if wf is not None else None
    args = (ctypes.byref(d), nat.ptr(xd), nat.ptr(wt, wt.dtype), nat.ptr(bias.to(DEV)), nat.ptr(y),
            None, None, None, None, None, nat.stream())
    if retired:                 # po_conv refuses a retired tile
        with pytest.raises(RuntimeError, match="retired"):
            nat.call("po_conv", *args)
        return
    nat.call("po_conv", *args)
    assert _rel(y.permute(0, 3, 1, 2).cpu().double(), ref) < 3e-6     # fp32-class error either way


def _frag(w16):
    """po_conv_desc.Wfrag layout of split weights [2][N][taps][Cin_p]."""
    two, N, T, C = w16.shape
    return w16.view(2, N // 32, 32, T, C // 16, 2, 8).permute(0, 1, 3, 4, 5, 2, 6).contiguous()


@pytest.mark.parametrize("quad,row", [(55, 29), (56, 31), (57, 29), (58, 31), (59, None), (60, None)])
@pytest.mark.parametrize("step,H,flip", [(1, 37, False), (1, 40, True), (2, 61, False), (2, 64, False)])
def test_quad_halo_tiles_match_row_tiles(quad, row, step, H, flip):
    """The 2-D tile halo kernel (tiles 55/56: 8 x 16 output pixels per tile,
    input step 1 or 2, either tap orientation) runs the same k-steps and MFMA
    sequence as the register-staged tile of the same BM x BN x BK: identical
    outputs (ragged edges at H = 37 / 61), and both within fp32 class of a
    float64 conv2d.  A boxed launch is refused."""
    import ctypes
    nat = pkg_mod("_native")
    B, Cin, Cout = 2, 48, 96
    Ho = (H - 1) // step + 1
    gen = torch.Generator().manual_seed(H + step)
    x = torch.randn(B, Cin, H, H, generator=gen)
    w = torch.randn(Cout, Cin, 3, 3, generator=gen) * (2.0 / (Cin * 9)) ** 0.5
    bias = torch.randn(Cout, generator=gen) * 0.1
    wk = w.flip(2, 3) if flip else w            # flipped tap order: dh0 = +1, sdh = -1 (dgrad orientation)
    ref = torch.nn.functional.conv2d(x.double(), w.double(), bias.double(), padding=1, stride=step)
    xd = x.permute(0, 2, 3, 1).contiguous().to(DEV)
    wd = wk.permute(0, 2, 3, 1).reshape(Cout, 9, Cin).contiguous().to(DEV)
    wt, shift, slot = _conv_operands(nat, wd, x, 1)
    wf = _frag(wt)
    if quad in (59, 60) and step == 2:
        pytest.skip("16 x 16 tiles take input step 1 only")

    def run(tile, box=None):
        y = torch.full((B, Ho, Ho, Cout), float("nan"), device=DEV)
        d = nat.po_conv_desc()
        d.B, d.Hin, d.Win, d.Cin_p, d.Hout, d.Wout, d.Cout_p, d.Hg, d.Wg = B, H, H, Cin, Ho, Ho, Cout, Ho, Ho
        d.in_step, d.out_step, d.ntaps, d.N, d.act, d.tile = step, 1, 9, Cout, 1, tile
        for kh in range(3):
            for kw in range(3):
                s_ = -1 if flip else 1
                d.dh[kh * 3 + kw], d.dw[kh * 3 + kw] = s_ * (kh - 1), s_ * (kw - 1)
        d.prec, d.w_shift, d.in_amax = 1, shift, slot.data_ptr()
        d.gbox = box.data_ptr() if box is not None else None
        d.Wfrag = wf.data_ptr()
        nat.call("po_conv", ctypes.byref(d), nat.ptr(xd), nat.ptr(wt, wt.dtype), nat.ptr(bias.to(DEV)), nat.ptr(y),
                 None, None, None, None, None, nat.stream())
        torch.cuda.synchronize()
        return y.permute(0, 3, 1, 2).cpu()

    yq = run(quad)
    assert not torch.isnan(yq).any()
    if row is not None:
        assert torch.equal(yq, run(row))
    assert _rel(yq.double(), torch.nn.functional.leaky_relu(ref, 0.1)) < 3e-6
    box = torch.tensor([[0, 0, 4, 4]] * B, dtype=torch.int32, device=DEV)
    with pytest.raises(RuntimeError, match="halo"):
        run(quad, box)


@pytest.mark.parametrize("stride,H,W,C,Cp", [(2, 13, 10, 12, 16), (1, 9, 7, 16, 16), (2, 416 // 8, 52, 30, 32), (2, 7, 7, 3, 4)])
def test_maxpool_ops_match_torch(stride, H, W, C, Cp):
    """po_maxpool2_fwd/bwd (darknet_v3.py:61-69: MaxPool2d(2,2), or
    ZeroPad2d((0,1,0,1)) + MaxPool2d(2,1)) against torch on NHWC buffers with
    padded channels; backward with accumulate and a LeakyReLU mask."""
    import torch.nn.functional as F
    nat = pkg_mod("_native")
    B = 3
    gen = torch.Generator().manual_seed(H * W + C)
    x = torch.randn(B, C, H, W, generator=gen)
    xr = x.clone().requires_grad_(True)
    xp = F.pad(xr, (0, 1, 0, 1)) if stride == 1 else xr
    ref = F.max_pool2d(xp, 2, stride)
    Ho, Wo = ref.shape[2:]
    g = torch.randn(ref.shape, generator=gen)
    ref.backward(g)
    src = torch.zeros(B, H, W, Cp)
    src[..., :C] = x.permute(0, 2, 3, 1)
    src = src.to(DEV)
    dst = torch.full((B, Ho, Wo, Cp), float("nan"), device=DEV)
    am = torch.zeros(B, Ho, Wo, Cp, dtype=torch.int8, device=DEV)
    nat.call("po_maxpool2_fwd", nat.ptr(src), B, H, W, C, Cp, stride, nat.ptr(dst), nat.ptr(am, torch.int8), None,
             nat.stream())
    assert torch.equal(dst[..., :C].permute(0, 3, 1, 2).cpu(), ref.detach())
    assert (dst[..., C:] == 0).all()
    gd = torch.zeros(B, Ho, Wo, Cp)
    gd[..., :C] = g.permute(0, 2, 3, 1)
    prev = torch.randn(B, H, W, Cp, generator=gen)
    mask = torch.randn(B, H, W, Cp, generator=gen)
    ds = prev.clone().to(DEV)
    gdd, maskd = gd.to(DEV), mask.to(DEV)        # keep the device copies alive across the launch
    nat.call("po_maxpool2_bwd", nat.ptr(gdd), nat.ptr(am, torch.int8), B, H, W, C, Cp, stride, nat.ptr(ds), 1,
             nat.ptr(maskd), None, nat.stream())
    want = (xr.grad.permute(0, 2, 3, 1) + prev[..., :C]) * torch.where(mask[..., :C] > 0, 1.0, 0.1)
    torch.testing.assert_close(ds[..., :C].cpu(), want, rtol=1e-6, atol=1e-6)
