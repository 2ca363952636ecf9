"""HBM-bound producer kernels: first conv, warp, fused conv + pool.

po_conv_first_fwd (the 3-channel first Darknet conv, darknet_v3.py:9-100
conv + BN-folded bias + LeakyReLU 0.1, cfg.py:37-56) on the GPU: the packed
two-pixel kernel (first_fwd2_k, Cout_p 16 / 32) and the one-pixel kernel
(first_fwd_k, Cout_p 64) match a PyTorch fp32 conv within fp32 rounding; ragged pixel counts (not a multiple of the 512-pixel block) and
image borders (zero padding) are covered."""
import ctypes

import pytest
import torch

from conftest import pkg_mod

pytestmark = pytest.mark.gpu


def _run(img, w, b, stride, cout_p, act):
    nat = pkg_mod("_native")
    B, _, H, W = img.shape
    Ho, Wo = (H - 1) // stride + 1, (W - 1) // stride + 1
    y = torch.full((B, Ho, Wo, cout_p), float("nan"), device=img.device)
    amax = torch.zeros(nat.PO_AMAX_SUB, dtype=torch.int32, device=img.device)
    nat.call("po_conv_first_fwd", nat.ptr(img), B, H, W, stride, nat.ptr(w), nat.ptr(b), w.size(0), cout_p,
             act, nat.ptr(y), nat.ptr(amax, torch.int32), nat.stream())
    torch.cuda.synchronize()
    amax_f = amax.view(torch.float32).max().item()
    return y, amax_f


@pytest.mark.parametrize("B,H,W,stride,cout", [(2, 37, 53, 1, 32), (3, 29, 31, 2, 32), (1, 64, 64, 1, 16),
                                              (1, 41, 23, 2, 16), (2, 19, 22, 1, 64), (1, 17, 30, 2, 40)])
def test_first_fwd_matches_torch(B, H, W, stride, cout):
    """Cout_p 16 / 32: the packed two-pixel kernel; 64: the one-pixel kernel."""
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(B * 1000 + H)
    img = torch.rand(B, 3, H, W, generator=g).to(dev)
    w = (torch.randn(cout, 3, 3, 3, generator=g) * 0.3).to(dev)
    b = (torch.randn(cout, generator=g) * 0.1).to(dev)
    w27 = w.reshape(cout, 27).contiguous()
    cp = 16 if cout <= 16 else (32 if cout <= 32 else 64)
    for act in (0, 1):
        y2, m2 = _run(img, w27, b, stride, cp, act)
        ref = torch.nn.functional.conv2d(img.cpu().double(), w.cpu().double(), b.cpu().double(), stride, 1)
        if act:
            ref = torch.nn.functional.leaky_relu(ref, 0.1)
        ref = ref.permute(0, 2, 3, 1).float()
        torch.testing.assert_close(y2[..., :cout].cpu(), ref, rtol=1e-5, atol=1e-5)
        assert abs(m2 - ref.abs().max().item()) <= 1e-5 * max(1.0, m2)


def _shifted(shape, shift, dev, fill=float("nan")):
    """A tensor of ``shape`` starting ``shift`` floats into a fresh buffer:
    shift 1 breaks the 16-byte alignment the vector kernels dispatch on."""
    n = 1
    for d in shape:
        n *= d
    return torch.full((n + 4,), fill, device=dev)[shift:shift + n].view(shape)


@pytest.mark.parametrize("mode", [0, 1])
def test_warp_quad_kernels_bit_identical(mode):
    """po_warp_fwd / po_warp_bwd (PatchTransformer affine warp + composite,
    load_data.py:726-792, 820, and its gather-form backward): the
    four-pixels-per-thread kernels (16-byte aligned buffers) write the same
    bits as the one-pixel kernels (the dispatch's fallback for unaligned
    buffers or S % 4 != 0, taken here by a buffer one float off alignment),
    patch magnified, partly outside and fully outside the frame."""
    nat = pkg_mod("_native")
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(7 + mode)
    B, S, P = 3, 64, 24
    img = torch.rand(B, 3, S, S, generator=g).to(dev)
    mp = torch.rand(3, P, P, generator=g).to(dev)
    noise = (torch.rand(B, 3, P, P, generator=g) * 2 - 1).to(dev)
    contrast = (torch.rand(B, generator=g) * 0.4 + 0.8).to(dev)
    bright = (torch.rand(B, generator=g) * 0.2 - 0.1).to(dev)
    d_out = torch.randn(B, 3, S, S, generator=g).to(dev)
    theta = torch.tensor([[1.6, 0.4, 0.1, -0.4, 1.6, -0.2],      # scaled, rotated, inside
                          [0.9, -1.1, 0.9, 1.1, 0.9, -0.8],      # large, partly outside
                          [2.0, 0.0, 3.5, 0.0, 2.0, 3.5]],       # off the frame
                         dtype=torch.float64)
    # po_warp_* take the pixel-space sampling map (po_patch_params' affine):
    # ix = a0 j + a1 i + a2, iy = a3 j + a4 i + a5 (affine_grid + unnormalize folded)
    half = 0.5 - 0.5 * S
    affine = torch.stack([theta[:, 0], theta[:, 1],
                          (theta[:, 0] + theta[:, 1]) * half + 0.5 * S * theta[:, 2] + 0.5 * (S - 1),
                          theta[:, 3], theta[:, 4],
                          (theta[:, 3] + theta[:, 4]) * half + 0.5 * S * theta[:, 5] + 0.5 * (S - 1)], 1)
    affine = affine.contiguous().to(dev)
    outs, grads = [], []
    for shift in (0, 1):
        out = _shifted((B, 3, S, S), shift, dev)
        nat.call("po_warp_fwd", nat.ptr(img) if mode == 1 else None, nat.ptr(mp), nat.ptr(noise),
                 nat.ptr(contrast), nat.ptr(bright), nat.ptr(affine, torch.float64), B, S, P, mode, nat.ptr(out),
                 nat.stream())
        dsh = _shifted((B, 3, S, S), shift, dev)
        dsh.copy_(d_out)
        work = _shifted((B, 3, S, S), shift, dev)
        dmp = torch.full((3, P, P), float("nan"), device=dev)
        nat.call("po_warp_bwd", nat.ptr(dsh), nat.ptr(mp), nat.ptr(noise), nat.ptr(contrast), nat.ptr(bright),
                 nat.ptr(affine, torch.float64), B, S, P, mode, nat.ptr(work), nat.ptr(dmp), nat.stream())
        torch.cuda.synchronize()
        outs.append(out.clone())
        grads.append(dmp)
    assert torch.equal(outs[0], outs[1])
    assert (outs[0] != (img if mode == 1 else 0)).any()      # the patch landed somewhere
    assert torch.equal(grads[0], grads[1]) and bool((grads[0] != 0).any())


@pytest.mark.parametrize("B,H,W,cout", [(2, 38, 54, 32), (3, 29, 31, 16), (1, 64, 64, 16), (2, 17, 20, 13)])
def test_first_pool_fused_matches_conv_then_pool(B, H, W, cout):
    """po_conv_first_pool_fwd (yolov3-tiny's conv 3->16 + maxpool 2/2,
    darknet_v3.py:61-69) writes the pool output po_conv_first_fwd +
    po_maxpool2_fwd write, bit for bit, and the same window positions; its
    argmax bytes carry the LeakyReLU slope, so po_maxpool2_bwd without the
    conv output gives the gradient that the unfused backward (mask = conv
    output) gives.  Odd sizes (the last row/column in no window), a ragged
    last workgroup and Cout < Cout_p are covered."""
    nat = pkg_mod("_native")
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(B * 100 + H + W)
    cp = 16 if cout <= 16 else 32
    img = torch.rand(B, 3, H, W, generator=g).to(dev)
    w27 = (torch.randn(cout, 27, generator=g) * 0.3).to(dev)
    b = (torch.randn(cout, generator=g) * 0.1).to(dev)
    Hp, Wp = H // 2, W // 2
    for act in (0, 1):
        y, _ = _run(img, w27, b, 1, cp, act)
        pooled = torch.full((B, Hp, Wp, cp), float("nan"), device=dev)
        am = torch.full((B, Hp, Wp, cp), -1, dtype=torch.int8, device=dev)
        nat.call("po_maxpool2_fwd", nat.ptr(y), B, H, W, cout, cp, 2, nat.ptr(pooled), nat.ptr(am, torch.int8), None,
                 nat.stream())
        fp = torch.full_like(pooled, float("nan"))
        fam = torch.full_like(am, -1)
        amax = torch.zeros(nat.PO_AMAX_SUB, dtype=torch.int32, device=dev)
        nat.call("po_conv_first_pool_fwd", nat.ptr(img), B, H, W, nat.ptr(w27), nat.ptr(b), cout, cp, act,
                 nat.ptr(fp), nat.ptr(fam, torch.int8), nat.ptr(amax, torch.int32), nat.stream())
        torch.cuda.synchronize()
        assert torch.equal(fp, pooled), "fused pool output differs from conv + po_maxpool2_fwd"
        assert torch.equal(fam.long()[..., :cout] & 3, am.long()[..., :cout])
        code = fam.long()[..., :cout]
        if act:
            assert bool(((code & 8) == 8).all())
            assert torch.equal((code & 4) == 4, pooled[..., :cout] <= 0)
        else:
            assert bool((code < 4).all())
        assert amax.view(torch.float32).max().item() == pooled.abs().max().item()
        # backward: leaky' from the argmax bytes == leaky' from the stored conv output
        dd = torch.randn(B, Hp, Wp, cp, generator=g).to(dev)
        d_ref = torch.full((B, H, W, cp), float("nan"), device=dev)
        d_fus = torch.full_like(d_ref, float("nan"))
        nat.call("po_maxpool2_bwd", nat.ptr(dd), nat.ptr(am, torch.int8), B, H, W, cout, cp, 2, nat.ptr(d_ref), 0,
                 nat.ptr(y) if act else None, None, nat.stream())
        nat.call("po_maxpool2_bwd", nat.ptr(dd), nat.ptr(fam, torch.int8), B, H, W, cout, cp, 2, nat.ptr(d_fus), 0,
                 None, None, nat.stream())
        torch.cuda.synchronize()
        assert torch.equal(d_fus, d_ref)


def _pool_ref64(img, w27, b, act):
    """float64 conv 3->Cout (pad 1) + LeakyReLU + 2/2 max pool on the CPU:
    (pooled [B,Hp,Wp,Cout], window position [B,Hp,Wp,Cout], second-best gap)."""
    B, _, H, W = img.shape
    cout = w27.shape[0]
    y = torch.nn.functional.conv2d(img.double().cpu(), w27.double().cpu().view(cout, 3, 3, 3),
                                   b.double().cpu(), padding=1)
    if act:
        y = torch.nn.functional.leaky_relu(y, 0.1)
    Hp, Wp = H // 2, W // 2
    win = y[:, :, :2 * Hp, :2 * Wp].reshape(B, cout, Hp, 2, Wp, 2).permute(0, 2, 4, 1, 3, 5).reshape(B, Hp, Wp, cout, 4)
    top = win.topk(2, dim=-1).values
    return win.max(-1).values, win.argmax(-1), top[..., 0] - top[..., 1]


@pytest.mark.parametrize("B,H,W,cout", [(2, 38, 54, 32), (3, 29, 31, 16), (1, 64, 64, 16), (2, 17, 20, 13),
                                        (4, 416, 416, 16)])
def test_first_pool_wino_matches_float64(B, H, W, cout):
    """po_conv_first_pool_wino_fwd (the conv as Winograd F(2x2,3x3), U from
    darknet_v3.first_wino_u) against the float64 conv + leaky + pool.
    Tolerance (stated): |pooled - ref| <= 2e-6 * (1 + |ref|) where ref is
    the conv output scale of these inputs (|y| <~ 4) -- the direct fused
    kernel's own error is of the same order; window positions equal the
    float64 argmax wherever the best two window values differ by more than
    that tolerance; argmax bits 2-3 as po_conv_first_pool_fwd."""
    nat, dv3 = pkg_mod("_native"), pkg_mod("darknet_v3")
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(B * 100 + H + W + 5)
    cp = 16 if cout <= 16 else 32
    img = torch.rand(B, 3, H, W, generator=g)
    w27 = torch.randn(cout, 27, generator=g, dtype=torch.float64) * 0.3
    b = torch.randn(cout, generator=g, dtype=torch.float64) * 0.1
    u16 = dv3.first_wino_u(w27.view(cout, 3, 3, 3)).float().contiguous().to(dev)
    w32, b32 = w27.float().to(dev), b.float().to(dev)
    imgd = img.to(dev)
    Hp, Wp = H // 2, W // 2
    for act in (0, 1):
        ref, pos, gap = _pool_ref64(img, w32, b32, act)
        outs = {}
        for name, wt in (("po_conv_first_pool_wino_fwd", u16), ("po_conv_first_pool_fwd", w32)):
            y = torch.full((B, Hp, Wp, cp), float("nan"), device=dev)
            am = torch.full((B, Hp, Wp, cp), -1, dtype=torch.int8, device=dev)
            amax = torch.zeros(nat.PO_AMAX_SUB, dtype=torch.int32, device=dev)
            nat.call(name, nat.ptr(imgd), B, H, W, nat.ptr(wt), nat.ptr(b32), cout, cp, act, nat.ptr(y),
                     nat.ptr(am, torch.int8), nat.ptr(amax, torch.int32), nat.stream())
            torch.cuda.synchronize()
            outs[name] = (y[..., :cout].double().cpu(), am.long().cpu()[..., :cout], amax)
        y, code, amax = outs["po_conv_first_pool_wino_fwd"]
        tol = 2e-6 * (1.0 + ref.abs())
        err = (y - ref).abs()
        assert bool((err <= tol).all()), "max err %.3g" % float(err.max())
        d_err = (outs["po_conv_first_pool_fwd"][0] - ref).abs().max()
        assert float(err.max()) <= 4 * float(d_err) + 1e-7      # same order as the direct form
        clear = gap > 2 * tol
        assert torch.equal((code & 3)[clear], pos[clear])
        if act:
            assert bool(((code & 8) == 8).all())
            assert torch.equal((code & 4) == 4, y <= 0)
        else:
            assert bool((code < 4).all())
        assert amax.view(torch.float32).max().item() == y.abs().max().item()


def _sparse_case(B, S, P, seed, big=False):
    """(frames, full composite, sparse composite (NaN outside the boxes), roi)."""
    ld, sy = pkg_mod("load_data"), pkg_mod("synthetic")
    dev = torch.device("cuda", 0)
    keyed = {k: v for k, v in sy.draws_device(seed, 2, 0, B, P, dev).items() if k != "noise"}
    keyed["noise_key"] = (seed, 2, 0)
    img = sy.frames(B, S, seed=seed).to(dev)
    lab = sy.labels(B, seed=seed + 1)
    if big:
        lab[:, :, 3:5] = lab[:, :, 3:5].clamp(min=0.6)
    lab = lab.to(dev)
    patch = sy.patch(P, seed=seed + 2).to(dev)
    pt = ld.PatchTransformer()
    full, _ = pt.forward_composite(patch, lab, img, S, draws=keyed)
    roi = pt.last_roi.clone()
    sp, _ = pt.forward_composite(patch, lab, img, S, draws=keyed, sparse=True)
    m = torch.zeros(B, 1, S, S, dtype=torch.bool)
    for b, (x0, y0, x1, y1) in enumerate(roi.cpu().tolist()):
        qx0, qx1 = x0 & ~3, min(S, (x1 + 3) & ~3)
        if qx1 > qx0 and y1 > y0:
            m[b, :, y0:y1, qx0:qx1] = True
    sp = torch.where(m.to(dev), sp, torch.full_like(sp, float("nan")))      # outside the boxes: never read
    return img, full.detach(), sp.detach(), roi


@pytest.mark.parametrize("B,S,stride,cout,big", [(4, 608, 1, 32, False), (3, 416, 2, 16, False),
                                                 (2, 96, 1, 32, True), (3, 64, 2, 32, True)])
def test_first_fwd_on_sparse_composite_bit_identical(B, S, stride, cout, big):
    """po_conv_first_fwd_cmp(frames, sparse composite, roi) equals
    po_conv_first_fwd on the materialised composite bit for bit (waves whose
    taps miss every box take the plain loads, the others read each tap from
    the tensor that holds it; ``big``: boxes covering most of the frame)."""
    nat = pkg_mod("_native")
    dev = torch.device("cuda", 0)
    img, full, sp, roi = _sparse_case(B, S, min(224, S // 2), seed=S + stride, big=big)
    g = torch.Generator().manual_seed(7)
    w = (torch.randn(cout, 27, generator=g) * 0.3).to(dev)
    b = (torch.randn(cout, generator=g) * 0.1).to(dev)
    cp = 16 if cout <= 16 else 32
    for act in (0, 1):
        want, m_want = _run(full, w, b, stride, cp, act)
        Ho = (S - 1) // stride + 1
        y = torch.full((B, Ho, Ho, cp), float("nan"), device=dev)
        amax = torch.zeros(nat.PO_AMAX_SUB, dtype=torch.int32, device=dev)
        nat.call("po_conv_first_fwd_cmp", nat.ptr(img), nat.ptr(sp), nat.ptr(roi, torch.int32), B, S, S, stride,
                 nat.ptr(w), nat.ptr(b), cout, cp, act, nat.ptr(y), nat.ptr(amax, torch.int32), nat.stream())
        torch.cuda.synchronize()
        assert torch.equal(y, want)
        assert amax.view(torch.float32).max().item() == m_want


@pytest.mark.parametrize("wino", [False, True])
@pytest.mark.parametrize("B,S,cout,big", [(4, 416, 16, False), (2, 96, 16, True), (2, 64, 32, True)])
def test_first_pool_on_sparse_composite_bit_identical(B, S, cout, big, wino):
    """po_conv_first_pool[_wino]_fwd_cmp on (frames, sparse composite, roi)
    equals the same kernel on the materialised composite bit for bit."""
    nat = pkg_mod("_native")
    dev = torch.device("cuda", 0)
    img, full, sp, roi = _sparse_case(B, S, min(224, S // 2), seed=S + 11, big=big)
    g = torch.Generator().manual_seed(8)
    w = (torch.randn(cout, 27, generator=g) * 0.3).to(dev)
    b = (torch.randn(cout, generator=g) * 0.1).to(dev)
    h = S // 2
    outs = []
    if wino:
        w = pkg_mod("darknet_v3").first_wino_u(w.double().view(cout, 3, 3, 3).cpu()).float().contiguous().to(dev)
    base = "po_conv_first_pool_wino_fwd" if wino else "po_conv_first_pool_fwd"
    for name, pre in ((base, ()), (base + "_cmp", None)):
        y = torch.full((B, h, h, cout), float("nan"), device=dev)
        am = torch.full((B, h, h, cout), -1, dtype=torch.int8, device=dev)
        amax = torch.zeros(nat.PO_AMAX_SUB, dtype=torch.int32, device=dev)
        head = (nat.ptr(full),) if pre == () else (nat.ptr(img), nat.ptr(sp), nat.ptr(roi, torch.int32))
        nat.call(name, *head, B, S, S, nat.ptr(w), nat.ptr(b), cout, cout, 1, nat.ptr(y), nat.ptr(am, torch.int8),
                 nat.ptr(amax, torch.int32), nat.stream())
        torch.cuda.synchronize()
        outs.append((y, am, amax))
    for u, v in zip(outs[0], outs[1]):
        assert torch.equal(u, v)


def test_cmp_entries_refuse_bad_arguments():
    nat = pkg_mod("_native")
    dev = torch.device("cuda", 0)
    img = torch.zeros(1, 3, 16, 16, device=dev)
    roi = torch.zeros(1, 4, dtype=torch.int32, device=dev)
    w = torch.zeros(64, 27, device=dev)
    y = torch.zeros(1, 16, 16, 64, device=dev)
    lib = nat.load()
    assert lib.po_conv_first_fwd_cmp(nat.ptr(img), None, nat.ptr(roi, torch.int32), 1, 16, 16, 1, nat.ptr(w), None,
                                     16, 16, 0, nat.ptr(y), None, nat.stream()) != 0
    assert lib.po_conv_first_fwd_cmp(nat.ptr(img), nat.ptr(img), nat.ptr(roi, torch.int32), 1, 16, 16, 1, nat.ptr(w),
                                     None, 64, 64, 0, nat.ptr(y), None, nat.stream()) != 0      # Cout_p 64
    assert "Cout_p <= 32" in nat.last_error()
