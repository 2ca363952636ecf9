"""po_conv tile 71 (conv_wino6_k, csrc/conv_wino6.hip): Winograd F(4x4,3x3)
as a persistent kernel, and tile 72 (the same with the input transform as a
pass of its own, bit-identical to 71).  It is a different exact-arithmetic factorisation of
the same convolution, so it is compared with float64 torch conv2d (and with
the direct fp32 kernel's own error beside it), and its epilogues with tile
70's on the same descriptor: both tap orientations, ragged 4x4 tiles on odd
and non-multiple-of-4 map sides, every epilogue-field combination the plan
launches, split-K slices (even and uneven), gradient-cone boxes, and the
launches it refuses."""
import ctypes

import pytest
import torch
import torch.nn.functional as F

from conftest import pkg_mod
from test_gpu_wino import _desc, _rel, _setup
from test_gpu_wino5 import MODES, _inputs

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)
# max-abs error relative to max|float64 output| of one F(4x4,3x3) layer (fp32
# transforms and products; a numpy model of the same arithmetic gives ~8e-6 at
# worst, ~8e-7 rms, against ~5e-7 / 1e-7 for the direct fp32 conv)
TOL71 = 2e-5


def _u6(wd, flip):
    dk = pkg_mod("darknet_v3")
    s = -1 if flip else 1
    offs = [(s * (kh - 1), s * (kw - 1)) for kh in range(3) for kw in range(3)]
    return dk.wino6_transform(wd, offs)


def _conv(nat, tile, B, H, Cin, Cout, flip, xd, wd, bias, U, U6, ksplit=1):
    y = torch.full((B, H, H, Cout), float("nan"), device=DEV)
    d = _desc(nat, B, H, Cin, Cout, tile, flip)
    d.Wwino, d.Wwino6 = U.data_ptr(), U6.data_ptr()
    ws = None
    if ksplit > 1:
        ws = torch.full((ksplit * B * H * H * Cout,), float("nan"), device=DEV)
        d.ksplit, d.workspace = ksplit, ws.data_ptr()
    nat.call("po_conv", ctypes.byref(d), nat.ptr(xd), nat.ptr(wd), nat.ptr(bias), nat.ptr(y), None, None,
             None, None, None, nat.stream())
    torch.cuda.synchronize()
    return y.permute(0, 3, 1, 2).cpu()


@pytest.mark.parametrize("B,H,Cin,Cout,flip", [(3, 7, 96, 128, False), (3, 7, 96, 128, True), (2, 38, 256, 512, False),
                                               (4, 19, 512, 256, True), (1, 76, 128, 64, False),
                                               (2, 9, 32, 64, False), (2, 10, 64, 64, True), (16, 76, 128, 256, False),
                                               (2, 13, 48, 192, False)])
def test_tile71_matches_float64_conv(B, H, Cin, Cout, flip):
    nat = pkg_mod("_native")
    x, w, bias, wd, U = _setup(B, H, Cin, Cout, flip, seed=H * Cin + flip)
    U6 = _u6(wd, flip)
    ref = F.conv2d(x.double(), w.double(), bias.double(), padding=1)
    xd = x.permute(0, 2, 3, 1).contiguous().to(DEV)
    bd = bias.to(DEV)
    outs = {t: _conv(nat, t, B, H, Cin, Cout, flip, xd, wd, bd, U, U6) for t in (71, 70, 1)}
    assert not torch.isnan(outs[71]).any()
    e = {t: _rel(o.double(), ref) for t, o in outs.items()}
    print("F(4x4) %.3g  F(2x2) %.3g  direct %.3g (max-abs relative to float64)" % (e[71], e[70], e[1]))
    assert e[71] < TOL71, e


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("B,H,Cin,Cout", [(2, 11, 64, 128), (3, 38, 256, 512), (2, 7, 32, 64), (16, 76, 128, 256)])
def test_tile71_epilogues_match_tile70(mode, B, H, Cin, Cout):
    """Each epilogue-field combination writes what tile 70 writes, up to the
    two factorisations' rounding: values within TOL71 of the layer's max,
    sign bits equal wherever the value is not within that rounding of zero,
    untouched outputs untouched."""
    from test_gpu_wino5 import _run
    nat = pkg_mod("_native")
    flip = mode.startswith("dgrad")
    xd, wd, bias, U, prev, res, mbits, m2bits = _inputs(B, H, Cin, Cout, flip, seed=H + Cin)
    U6 = _u6(wd, flip)
    runs = {}
    for t in (71, 70):
        d_runs = _run_with(nat, t, mode, B, H, Cin, Cout, flip, U, U6, xd, wd, bias, prev, res, mbits, m2bits)
        runs[t] = d_runs
    (y1, s1, z1, b1), (y0, s0, z0, b0) = runs[71], runs[70]
    for a, b in ((y1, y0), (s1, s0), (z1, z0)):
        fin = torch.isfinite(b)
        assert torch.equal(fin, torch.isfinite(a))
        if fin.any():
            scale = float(b[fin].abs().max())
            assert float((a[fin] - b[fin]).abs().max()) <= TOL71 * max(scale, 1e-30), mode
    if mode in ("fwd_bits", "fwd_shortcut"):
        # sign bits: equal except at values within rounding of zero
        ref = y0 if mode == "fwd_bits" else None
        if ref is not None:
            bits = lambda bt: ((bt.unsqueeze(-1) >> torch.arange(32, device=bt.device, dtype=torch.int32)) & 1)
            bb1, bb0 = bits(b1).reshape(ref.shape), bits(b0).reshape(ref.shape)
            tie = ref.abs() <= TOL71 * float(ref.abs().max())
            assert torch.equal(bb1[~tie], bb0[~tie])


_WINOV = []


def _winov(d):
    """Tile 72's transformed-input workspace for desc d (NaN-filled: every float
    the GEMM reads must have been written by the transform pass)."""
    n = (-(-(d.B * (-(-d.Hg // 4)) * (-(-d.Wg // 4))) // 32)) * (d.Cin_p // 16) * 18432
    v = torch.full((n,), float("nan"), device=DEV)
    _WINOV.append(v)
    d.winov, d.winov_floats = v.data_ptr(), n


def _run_with(nat, tile, mode, B, H, Cin, Cout, flip, U, U6, xd, wd, bias, prev, res, mbits, m2bits, ksplit=1,
              box=None):
    from test_gpu_wino5 import _run
    # tile 70's harness, with the F(4x4) weights (and a gradient-cone box) attached
    orig = _desc
    import test_gpu_wino5 as w5

    def desc6(nat_, B_, H_, Cin_, Cout_, tile_, flip_=False):
        d = orig(nat_, B_, H_, Cin_, Cout_, tile_, flip_)
        d.Wwino6 = U6.data_ptr()
        if box is not None:
            d.gbox = box.data_ptr()
        if tile_ == 72:
            _winov(d)
        return d
    w5._desc = desc6
    try:
        ws = torch.full((ksplit * B * H * H * Cout,), float("nan"), device=DEV) if ksplit > 1 else None
        return _run(nat, tile, mode, B, H, Cin, Cout, flip, U, xd, wd, bias, prev, res, mbits, m2bits,
                    ksplit=ksplit, ws=ws)
    finally:
        w5._desc = orig


@pytest.mark.parametrize("Cin,ks", [(512, 2), (512, 3), (512, 4), (512, 6), (256, 3)])
@pytest.mark.parametrize("mode", ["fwd_bits", "dgrad_acc_bits", "dgrad_dual"])
def test_tile71_split_k(mode, Cin, ks):
    """Split-K slices (raw partials, conv_reduce_k applies the epilogue) give
    the one-slice result up to summation order: two evaluations each within
    TOL71 of the exact value, so within 2 TOL71 of each other."""
    nat = pkg_mod("_native")
    B, H, Cout = 4, 19, 256
    flip = mode.startswith("dgrad")
    xd, wd, bias, U, prev, res, mbits, m2bits = _inputs(B, H, Cin, Cout, flip, seed=17)
    U6 = _u6(wd, flip)
    one = _run_with(nat, 71, mode, B, H, Cin, Cout, flip, U, U6, xd, wd, bias, prev, res, mbits, m2bits)
    spl = _run_with(nat, 71, mode, B, H, Cin, Cout, flip, U, U6, xd, wd, bias, prev, res, mbits, m2bits, ksplit=ks)
    for a, b in zip(spl[:3], one[:3]):
        fin = torch.isfinite(b)
        assert torch.equal(fin, torch.isfinite(a))
        if fin.any():
            assert float((a[fin] - b[fin]).abs().max()) <= 2 * TOL71 * float(b[fin].abs().max())


BOXES = {
    # per image (r0, c0, r1, c1): unaligned to the 4x4 tiles, on the ragged
    # edge, a single pixel, an empty box, the whole map
    "mixed": lambda H: [[3, 5, 14, 11], [H - 6, H - 9, H, H], [7, 7, 8, 8], [5, 5, 5, 9]],
    "full": lambda H: [[0, 0, H, H]] * 4,
    "row": lambda H: [[0, 1, 2, H], [H - 1, 0, H, H], [4, 4, 9, 6], [0, 0, H, 3]],
}


@pytest.mark.parametrize("boxes", sorted(BOXES))
@pytest.mark.parametrize("mode", ["dgrad_mask", "dgrad_acc_bits", "dgrad_dual", "dgrad_acc_dual", "fwd_plain"])
@pytest.mark.parametrize("B,H,Cin,Cout,ks", [(4, 19, 256, 128, 1), (4, 38, 128, 64, 1), (4, 17, 64, 128, 1),
                                             (4, 19, 256, 128, 3), (4, 38, 128, 64, 2)])
def test_tile71_gradient_cone_boxes(boxes, mode, B, H, Cin, Cout, ks):
    """A boxed launch (gbox, the patch-gradient cones of the dgrads) writes
    exactly each image's box, within TOL71 of tile 68 (F(2x2), boxed) there
    (2 TOL71 with split-K: partials at the box's compact rows, conv_reduce_k),
    and leaves every other pixel as it was; units with no live tile are skipped
    (the empty box), the rest see their images' boxes."""
    nat = pkg_mod("_native")
    flip = mode.startswith("dgrad")
    xd, wd, bias, U, prev, res, mbits, m2bits = _inputs(B, H, Cin, Cout, flip, seed=H + Cout + len(boxes))
    U6 = _u6(wd, flip)
    box = torch.tensor(BOXES[boxes](H), dtype=torch.int32, device=DEV)
    runs = {t: _run_with(nat, t, mode, B, H, Cin, Cout, flip, U, U6, xd, wd, bias, prev, res, mbits, m2bits, box=box,
                         ksplit=ks if t == 71 else 1)
            for t in (71, 68)}
    tol = TOL71 * (2 if ks > 1 else 1)
    inside = torch.zeros(B, H, H, 1, dtype=torch.bool, device=DEV)
    for b, (r0, c0, r1, c1) in enumerate(box.tolist()):
        inside[b, r0:r1, c0:c1] = True
    for a, b in zip(runs[71][:3], runs[68][:3]):
        assert torch.equal(a.nan_to_num(7.0), torch.where(inside, a, b).nan_to_num(7.0))   # outside: as tile 68 left it
        fin = torch.isfinite(b) & inside
        assert torch.equal(fin, torch.isfinite(a) & inside)
        if fin.any():
            scale = float(b[fin].abs().max())
            assert float((a[fin] - b[fin]).abs().max()) <= tol * max(scale, 1e-30), mode
    y0 = runs[68][0]
    assert torch.equal(torch.where(inside, prev, y0), prev)           # tile 68 itself kept the outside


def _equal(a, b):
    for u, v in zip(a, b):
        assert torch.equal(u.nan_to_num(7.0), v.nan_to_num(7.0))


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("B,H,Cin,Cout", [(2, 11, 64, 128), (3, 38, 256, 512), (2, 7, 32, 64), (16, 76, 128, 256),
                                          (1, 19, 512, 64)])
def test_tile72_bit_identical_to_71(mode, B, H, Cin, Cout):
    """Tile 72 runs tile 71's transform (as a pass of its own, wino6_pre_k),
    MFMA order and epilogues: every output bit for bit."""
    nat = pkg_mod("_native")
    flip = mode.startswith("dgrad")
    xd, wd, bias, U, prev, res, mbits, m2bits = _inputs(B, H, Cin, Cout, flip, seed=H + Cin + 5)
    U6 = _u6(wd, flip)
    runs = [_run_with(nat, t, mode, B, H, Cin, Cout, flip, U, U6, xd, wd, bias, prev, res, mbits, m2bits)
            for t in (72, 71)]
    _equal(runs[0], runs[1])


@pytest.mark.parametrize("Cin,ks", [(512, 2), (512, 3), (256, 3)])
@pytest.mark.parametrize("mode", ["fwd_bits", "dgrad_acc_bits"])
def test_tile72_split_k_bit_identical_to_71(mode, Cin, ks):
    nat = pkg_mod("_native")
    B, H, Cout = 4, 19, 256
    flip = mode.startswith("dgrad")
    xd, wd, bias, U, prev, res, mbits, m2bits = _inputs(B, H, Cin, Cout, flip, seed=23)
    U6 = _u6(wd, flip)
    runs = [_run_with(nat, t, mode, B, H, Cin, Cout, flip, U, U6, xd, wd, bias, prev, res, mbits, m2bits, ksplit=ks)
            for t in (72, 71)]
    _equal(runs[0], runs[1])


@pytest.mark.parametrize("boxes", sorted(BOXES))
@pytest.mark.parametrize("mode", ["dgrad_mask", "dgrad_dual"])
@pytest.mark.parametrize("ks", [1, 2])
def test_tile72_boxes_bit_identical_to_71(boxes, mode, ks):
    nat = pkg_mod("_native")
    B, H, Cin, Cout = 4, 38, 128, 64
    flip = True
    xd, wd, bias, U, prev, res, mbits, m2bits = _inputs(B, H, Cin, Cout, flip, seed=31)
    U6 = _u6(wd, flip)
    box = torch.tensor(BOXES[boxes](H), dtype=torch.int32, device=DEV)
    runs = [_run_with(nat, t, mode, B, H, Cin, Cout, flip, U, U6, xd, wd, bias, prev, res, mbits, m2bits, box=box,
                      ksplit=ks) for t in (72, 71)]
    _equal(runs[0], runs[1])


def test_tile72_needs_its_workspace():
    nat = pkg_mod("_native")
    B, H, Cin, Cout = 2, 16, 32, 64
    xd, wd, bias, U, prev, res, mbits, m2bits = _inputs(B, H, Cin, Cout, False, seed=9)
    U6 = _u6(wd, False)
    y = torch.zeros(B, H, H, Cout, device=DEV)
    d = _desc(nat, B, H, Cin, Cout, 72)
    d.Wwino6 = U6.data_ptr()
    call = lambda: nat.load().po_conv(ctypes.byref(d), nat.ptr(xd), nat.ptr(wd), None, nat.ptr(y), None, None, None,
                                      None, None, nat.stream())
    assert call() != 0 and "winov" in nat.last_error()
    _winov(d)
    d.winov_floats -= 1
    assert call() != 0 and "workspace" in nat.last_error()
    d.winov_floats += 1
    assert call() == 0


def test_tile71_refuses_what_it_cannot_run():
    nat = pkg_mod("_native")
    B, H, Cin, Cout = 2, 16, 32, 64
    xd, wd, bias, U, prev, res, mbits, m2bits = _inputs(B, H, Cin, Cout, False, seed=9)
    U6 = _u6(wd, False)
    y = torch.zeros(B, H, H, Cout, device=DEV)

    def call(d, mask=None):
        return nat.load().po_conv(ctypes.byref(d), nat.ptr(xd), nat.ptr(wd), None, nat.ptr(y), None, None,
                                  nat.ptr(mask), None, None, nat.stream())

    d = _desc(nat, B, H, Cin, Cout, 71)
    assert call(d) != 0 and "Wwino6" in nat.last_error()
    d.Wwino6 = U6.data_ptr()
    assert call(d) == 0
    box = torch.tensor([[0, 0, 8, 8]] * B, dtype=torch.int32, device=DEV)
    d.gbox = box.data_ptr()
    assert call(d) == 0                                              # gradient-cone boxes
    d.mrows = 8 * 8
    assert call(d) != 0                                              # ... on the full grid only
    d.gbox, d.mrows = None, 0
    slot = torch.zeros(64, dtype=torch.int32, device=DEV)
    d.y_amax = slot.data_ptr()
    assert call(d) != 0
    d.y_amax = None
    assert call(d, mask=prev) != 0
    ws = torch.empty(4 * B * H * H * Cout, device=DEV)
    d.ksplit, d.workspace = 2, ws.data_ptr()
    assert call(d) != 0 and "two k-steps" in nat.last_error()
    d.ksplit, d.workspace = 1, None
    py = torch.zeros(B, H // 2, H // 2, Cout, device=DEV)
    pam = torch.zeros(B, H // 2, H // 2, Cout, dtype=torch.int8, device=DEV)
    d.pool_y, d.pool_argmax = py.data_ptr(), pam.data_ptr()
    # the fused pool runs since round 6 (test_tile71_fused_pool), on full maps only
    assert nat.load().po_conv(ctypes.byref(d), nat.ptr(xd), nat.ptr(wd), None, None, None, None, None, None, None,
                              nat.stream()) == 0
    d.gbox = box.data_ptr()
    assert nat.load().po_conv(ctypes.byref(d), nat.ptr(xd), nat.ptr(wd), None, None, None, None, None, None, None,
                              nat.stream()) != 0
    d.gbox = None
    d = _desc(nat, 2, 16, 32, 32, 71)                      # N = 32: not a multiple of 64
    d.Wwino6 = U6.data_ptr()
    assert call(d) != 0


@pytest.mark.parametrize("tile", [71, 72])
@pytest.mark.parametrize("act", [0, 1])
@pytest.mark.parametrize("B,H,Cin,Cout,flip", [(2, 104, 32, 64, False), (2, 52, 64, 128, False), (3, 18, 32, 64, True),
                                               (2, 10, 64, 128, False)])
def test_tile71_fused_pool(tile, act, B, H, Cin, Cout, flip):
    """Tiles 71/72 with the 2x2/2 max pool in the epilogue (EF_POOL, round 6):
    pooled values, window positions and slope codes bit-identical to pooling
    tile 71's own unpooled output by po_maxpool2_fwd's rule (first position on
    ties, NaN wins); map sides that end in half a 4x4 tile (18, 10) included."""
    nat = pkg_mod("_native")
    dk = pkg_mod("darknet_v3")
    x, w, bias, wd, U = _setup(B, H, Cin, Cout, flip, seed=H + Cout + act)
    U6 = _u6(wd, flip)
    xd = x.permute(0, 2, 3, 1).contiguous().to(DEV)
    bd = bias.to(DEV)
    y = torch.full((B, H, H, Cout), float("nan"), device=DEV)
    d = _desc(nat, B, H, Cin, Cout, 71, flip)
    d.Wwino, d.Wwino6, d.act = U.data_ptr(), U6.data_ptr(), act
    nat.call("po_conv", ctypes.byref(d), nat.ptr(xd), nat.ptr(wd), nat.ptr(bd), nat.ptr(y), None, None, None, None,
             None, nat.stream())
    h = H // 2
    py = torch.full((B, h, h, Cout), float("nan"), device=DEV)
    pam = torch.full((B, h, h, Cout), -1, dtype=torch.int8, device=DEV)
    d = _desc(nat, B, H, Cin, Cout, tile, flip)
    d.Wwino, d.Wwino6, d.act = U.data_ptr(), U6.data_ptr(), act
    d.pool_y, d.pool_argmax = py.data_ptr(), pam.data_ptr()
    winov = None
    if tile == 72:
        nv = dk.NetPlan.winov_floats(d)
        winov = torch.empty(nv, device=DEV)
        d.winov, d.winov_floats = winov.data_ptr(), nv
    nat.call("po_conv", ctypes.byref(d), nat.ptr(xd), nat.ptr(wd), nat.ptr(bd), None, None, None, None, None, None,
             nat.stream())
    torch.cuda.synchronize()
    win = y.view(B, h, 2, h, 2, Cout)
    pv, arg = win[:, :, 0, :, 0], torch.zeros(B, h, h, Cout, dtype=torch.int64, device=DEV)
    for k in range(1, 4):
        v = win[:, :, k >> 1, :, k & 1]
        upd = (v > pv) | torch.isnan(v)
        pv, arg = torch.where(upd, v, pv), torch.where(upd, torch.full_like(arg, k), arg)
    if act:
        arg = arg | 8 | torch.where(pv > 0, 0, 4)
    assert torch.equal(py.view(torch.int32), pv.view(torch.int32))
    assert torch.equal(pam.long(), arg)
