"""po_conv tile 61: the exact-fp32 Winograd F(2x2,3x3) kernel (conv_wino.hip)
against float64 torch conv2d and against the direct implicit-GEMM kernel on
the same descriptor: both tap orientations (forward, and the input-gradient
launches' flipped taps), odd map sides (ragged tiles), every epilogue mode the
training plan uses (bias + LeakyReLU + sign bits, accumulate + sign-bit mask,
fused shortcut, dual output, max|x| slots), gradient-cone boxes, and the
launches it must refuse."""
import ctypes

import pytest
import torch
import torch.nn.functional as F

from conftest import pkg_mod

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)
WINO_TILES = [61, 65, 66, 67, 68]   # 64 tiles x 32 ch; 32 tiles x 64 ch (LDS-DMA input, N % 64 == 0) in 8
                                    # scheduled waves / 4 waves in 64 KB of LDS; 64 tiles x 64 ch pipelined (68: staggered)


def _rel(a, b):
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


def _desc(nat, B, H, Cin, Cout, tile, flip=False):
    d = nat.po_conv_desc()
    d.B, d.Hin, d.Win, d.Cin_p, d.Hout, d.Wout, d.Cout_p, d.Hg, d.Wg = B, H, H, Cin, H, H, Cout, H, H
    d.in_step, d.out_step, d.ntaps, d.N, d.act, d.tile = 1, 1, 9, Cout, 0, tile
    s = -1 if flip else 1
    for kh in range(3):
        for kw in range(3):
            d.dh[kh * 3 + kw], d.dw[kh * 3 + kw] = s * (kh - 1), s * (kw - 1)
    d.prec = 0
    return d


def _setup(B, H, Cin, Cout, flip, seed):
    dk = pkg_mod("darknet_v3")
    gen = torch.Generator().manual_seed(seed)
    x = torch.randn(B, Cin, H, H, generator=gen)
    w = torch.randn(Cout, Cin, 3, 3, generator=gen) * (2.0 / (Cin * 9)) ** 0.5
    bias = torch.randn(Cout, generator=gen) * 0.1
    wk = w.flip(2, 3) if flip else w           # the dgrad launches' orientation: dh0 = +1, sdh = -1
    wd = wk.permute(0, 2, 3, 1).reshape(Cout, 9, Cin).contiguous().to(DEV)
    s = -1 if flip else 1
    offs = [(s * (kh - 1), s * (kw - 1)) for kh in range(3) for kw in range(3)]
    U = dk.wino_transform(wd, offs)
    return x, w, bias, wd, U


@pytest.mark.parametrize("WINO", WINO_TILES)
@pytest.mark.parametrize("B,H,Cin,Cout,flip", [(3, 7, 96, 128, False), (3, 7, 96, 128, True), (2, 38, 256, 512, False),
                                               (4, 19, 512, 256, True), (1, 76, 128, 64, False),
                                               (2, 9, 16, 32, False)])
def test_wino_matches_float64_conv(B, H, Cin, Cout, flip, WINO):
    if WINO in (65, 66, 67, 68) and Cout % 64:
        pytest.skip("tiles 65-68 take N % 64 == 0")
    nat = pkg_mod("_native")
    x, w, bias, wd, U = _setup(B, H, Cin, Cout, flip, seed=H * Cin + flip)
    ref = F.conv2d(x.double(), w.double(), bias.double(), padding=1)
    xd = x.permute(0, 2, 3, 1).contiguous().to(DEV)
    outs = {}
    for tile in (WINO, 1):
        y = torch.full((B, H, H, Cout), float("nan"), device=DEV)
        d = _desc(nat, B, H, Cin, Cout, tile, flip)
        d.Wwino = U.data_ptr()
        nat.call("po_conv", ctypes.byref(d), nat.ptr(xd), nat.ptr(wd), nat.ptr(bias.to(DEV)), nat.ptr(y), None, None,
                 None, None, None, nat.stream())
        outs[tile] = y.permute(0, 3, 1, 2).cpu()
    assert not torch.isnan(outs[WINO]).any()
    e_w, e_d = _rel(outs[WINO].double(), ref), _rel(outs[1].double(), ref)
    print("winograd %.3g direct %.3g (max-abs relative to float64)" % (e_w, e_d))
    assert e_w < 1e-5 and e_w < 4 * e_d + 1e-7, (e_w, e_d)


@pytest.mark.parametrize("WINO", WINO_TILES)
@pytest.mark.parametrize("mode", ["fwd_bits", "fwd_shortcut", "dgrad_acc_bits", "dgrad_dual"])
def test_wino_epilogues_match_direct(mode, WINO):
    """The training plan's epilogue combinations: identical semantics to the
    direct kernel (values within fp32 class, sign bits of the written
    values, max|x| slots bounding them)."""
    nat = pkg_mod("_native")
    B, H, Cin, Cout = 2, 11, 64, 128
    flip = mode.startswith("dgrad")
    x, w, bias, wd, U = _setup(B, H, Cin, Cout, flip, seed=7)
    gen = torch.Generator().manual_seed(3)
    xd = x.permute(0, 2, 3, 1).contiguous().to(DEV)
    prev = torch.randn(B, H, H, Cout, generator=gen).to(DEV)
    res = torch.randn(B, H, H, Cout, generator=gen).to(DEV)
    mbits = torch.randint(-2 ** 31, 2 ** 31 - 1, (B, H, H, Cout // 32), generator=gen, dtype=torch.int32).to(DEV)
    m2bits = torch.randint(-2 ** 31, 2 ** 31 - 1, (B, H, H, Cout // 32), generator=gen, dtype=torch.int32).to(DEV)
    res_run = {}
    for tile in (WINO, 1):
        d = _desc(nat, B, H, Cin, Cout, tile, flip)
        d.Wwino = U.data_ptr()
        y = prev.clone()
        ssum = torch.full_like(prev, float("nan"))
        y2 = torch.full_like(prev, float("nan"))
        bits = torch.zeros(B, H, H, Cout // 32, dtype=torch.int32, device=DEV)
        slots = [torch.zeros(64, dtype=torch.int32, device=DEV) for _ in range(3)]
        args = dict(bias=None, res=None, sum=None, y2=None)
        if mode == "fwd_bits":
            d.act, d.ybits = 1, bits.data_ptr()
            args["bias"] = bias.to(DEV)
        elif mode == "fwd_shortcut":
            d.act, d.ybits = 1, bits.data_ptr()
            args.update(bias=bias.to(DEV), res=res, sum=ssum)
            d.sum_amax = slots[1].data_ptr()
        elif mode == "dgrad_acc_bits":
            d.accumulate, d.mbits = 1, mbits.data_ptr()
        else:
            d.mbits, d.m2bits = mbits.data_ptr(), m2bits.data_ptr()
            args["y2"] = y2
            d.y2_amax = slots[2].data_ptr()
        d.y_amax = slots[0].data_ptr()
        nat.call("po_conv", ctypes.byref(d), nat.ptr(xd), nat.ptr(wd), nat.ptr(args["bias"]), nat.ptr(y),
                 nat.ptr(args["res"]), nat.ptr(args["sum"]), None, nat.ptr(args["y2"]), None, nat.stream())
        torch.cuda.synchronize()
        res_run[tile] = (y.cpu(), ssum.cpu(), y2.cpu(), bits.cpu(), [s.cpu().view(torch.float32).max() for s in slots])
    (yw, sw, y2w, bw, slw), (yd, sd, y2d, bd, sld) = res_run[WINO], res_run[1]
    assert _rel(yw, yd) < 1e-5
    if mode == "fwd_shortcut":
        assert _rel(sw, sd) < 1e-5 and float(slw[1]) >= float(sw.abs().max())
    if mode == "dgrad_dual":
        assert _rel(y2w, y2d) < 1e-5 and float(slw[2]) >= float(y2w.abs().max())
    assert float(slw[0]) >= float(yw.abs().max()) * (1 - 1e-7)
    if mode.startswith("fwd"):
        # the sign bits are those of the values this launch wrote
        sh = torch.arange(32, dtype=torch.int32)
        got = ((bw.unsqueeze(-1) >> sh) & 1).reshape(B, H, H, Cout).bool()
        assert torch.equal(got, yw > 0)


@pytest.mark.parametrize("WINO", WINO_TILES)
def test_wino_gradient_cone_box(WINO):
    """A boxed launch (gbox) writes exactly the box and matches the full launch there."""
    nat = pkg_mod("_native")
    B, H, Cin, Cout = 2, 38, 64, 64
    x, w, bias, wd, U = _setup(B, H, Cin, Cout, True, seed=5)
    xd = x.permute(0, 2, 3, 1).contiguous().to(DEV)
    box = torch.tensor([[3, 5, 20, 31], [0, 0, 38, 38]], dtype=torch.int32, device=DEV)     # r0, c0, r1, c1
    out = {}
    for boxed in (False, True):
        y = torch.full((B, H, H, Cout), float("nan"), device=DEV)
        d = _desc(nat, B, H, Cin, Cout, WINO, True)
        d.Wwino = U.data_ptr()
        d.gbox = box.data_ptr() if boxed else None
        nat.call("po_conv", ctypes.byref(d), nat.ptr(xd), nat.ptr(wd), None, nat.ptr(y), None, None, None, None, None,
                 nat.stream())
        out[boxed] = y.cpu()
    full, bx = out[False], out[True]
    inside = torch.zeros(B, H, H, dtype=torch.bool)
    inside[0, 3:20, 5:31] = True
    inside[1] = True
    assert torch.equal(bx[inside], full[inside])
    assert torch.isnan(bx[~inside]).all()


@pytest.mark.parametrize("WINO", WINO_TILES)
def test_wino_refuses_what_it_cannot_run(WINO):
    import ctypes as C
    nat = pkg_mod("_native")
    B, H, Cin, Cout = 1, 8, 32, 64
    x, w, bias, wd, U = _setup(B, H, Cin, Cout, False, seed=9)
    xd = x.permute(0, 2, 3, 1).contiguous().to(DEV)
    y = torch.zeros(B, H, H, Cout, device=DEV)

    def call(d):
        return nat.load().po_conv(C.byref(d), nat.ptr(xd), nat.ptr(wd), None, nat.ptr(y), None, None, None, None,
                                  None, nat.stream())

    d = _desc(nat, B, H, Cin, Cout, WINO)
    assert call(d) != 0 and "Wwino" in nat.last_error()           # no transformed weights
    d.Wwino = U.data_ptr()
    assert call(d) == 0
    ws = torch.empty(4 * B * H * H * Cout, device=DEV)
    d.ksplit, d.workspace = 2, ws.data_ptr()
    assert (call(d) == 0) == (WINO in (66, 67, 68))                 # split-K: tiles 66, 67, 68 only
    d.ksplit = 3
    assert call(d) != 0                                             # more slices than 16-channel steps
    d = _desc(nat, B, H, Cin, Cout, WINO)
    d.Wwino = U.data_ptr()
    d.in_step = 2
    d.Hg = d.Wg = d.Hout = d.Wout = 4
    assert call(d) != 0                                             # stride 2


@pytest.mark.parametrize("tile", [66, 67, 68])
@pytest.mark.parametrize("mode", ["fwd_bits", "fwd_shortcut", "dgrad_acc_bits", "dgrad_dual"])
@pytest.mark.parametrize("B,H,Cin,Cout", [(2, 11, 64, 128), (3, 38, 256, 512), (1, 19, 512, 64), (2, 7, 16, 64)])
def test_wino_tile66_bit_identical_to_65(mode, B, H, Cin, Cout, tile):
    """Tile 66 (4-wave workgroups in 64 KB of LDS, two per CU) and tile 67
    (64 tiles x 64 channels, register-staged input, pipelined k-loop) run tile
    65's transforms, per-accumulator MFMA order and epilogue arithmetic: the
    same bits in every epilogue combination the training plan uses (sign bits
    and max|x| slots included), ragged tile counts, a single k-step."""
    nat = pkg_mod("_native")
    flip = mode.startswith("dgrad")
    x, w, bias, wd, U = _setup(B, H, Cin, Cout, flip, seed=H + Cin)
    gen = torch.Generator().manual_seed(5)
    xd = x.permute(0, 2, 3, 1).contiguous().to(DEV)
    prev = torch.randn(B, H, H, Cout, generator=gen).to(DEV)
    res = torch.randn(B, H, H, Cout, generator=gen).to(DEV)
    mbits = torch.randint(-2 ** 31, 2 ** 31 - 1, (B, H, H, Cout // 32), generator=gen, dtype=torch.int32).to(DEV)
    m2bits = torch.randint(-2 ** 31, 2 ** 31 - 1, (B, H, H, Cout // 32), generator=gen, dtype=torch.int32).to(DEV)
    runs = []
    for t_ in (tile, 65):
        d = _desc(nat, B, H, Cin, Cout, t_, flip)
        d.Wwino = U.data_ptr()
        y = prev.clone()
        ssum = torch.full_like(prev, float("nan"))
        y2 = torch.full_like(prev, float("nan"))
        bits = torch.zeros(B, H, H, Cout // 32, dtype=torch.int32, device=DEV)
        slots = [torch.zeros(64, dtype=torch.int32, device=DEV) for _ in range(3)]
        args = dict(bias=None, res=None, sum=None, y2=None)
        if mode == "fwd_bits":
            d.act, d.ybits = 1, bits.data_ptr()
            args["bias"] = bias.to(DEV)
        elif mode == "fwd_shortcut":
            d.act, d.ybits = 1, bits.data_ptr()
            args.update(bias=bias.to(DEV), res=res, sum=ssum)
            d.sum_amax = slots[1].data_ptr()
        elif mode == "dgrad_acc_bits":
            d.accumulate, d.mbits = 1, mbits.data_ptr()
        else:
            d.mbits, d.m2bits = mbits.data_ptr(), m2bits.data_ptr()
            args["y2"] = y2
            d.y2_amax = slots[2].data_ptr()
        d.y_amax = slots[0].data_ptr()
        nat.call("po_conv", ctypes.byref(d), nat.ptr(xd), nat.ptr(wd), nat.ptr(args["bias"]), nat.ptr(y),
                 nat.ptr(args["res"]), nat.ptr(args["sum"]), None, nat.ptr(args["y2"]), None, nat.stream())
        torch.cuda.synchronize()
        runs.append((y, ssum, y2, bits, [sl.max() for sl in slots]))
    for a, b in zip(runs[0][:4], runs[1][:4]):
        assert torch.equal(a.nan_to_num(7.0), b.nan_to_num(7.0))
    assert [int(v) for v in runs[0][4]] == [int(v) for v in runs[1][4]]



@pytest.mark.parametrize("tile", [61, 66, 67, 68])
@pytest.mark.parametrize("act", [0, 1])
@pytest.mark.parametrize("B,H,Cin,Cout", [(2, 12, 64, 128), (3, 26, 128, 256), (2, 104, 32, 64), (2, 52, 16, 32)])
def test_wino_fused_pool(act, B, H, Cin, Cout, tile):
    """Tiles 61 and 66 with the k=2 stride-2 max pool in the epilogue
    (po_conv_desc.pool_y): pooled values, window positions and slope codes
    bit-identical to pooling the tile's own unpooled output by
    po_maxpool2_fwd's rule (first position on ties), max|x| slot of the pooled
    map; tile 65 refuses a pooled launch."""
    if tile in (66, 67, 68) and Cout % 64:
        pytest.skip("tiles 66/67 take N % 64 == 0")
    nat = pkg_mod("_native")
    x, w, bias, wd, U = _setup(B, H, Cin, Cout, False, seed=H + Cout)
    xd = x.permute(0, 2, 3, 1).contiguous().to(DEV)
    bd = bias.to(DEV)
    y = torch.full((B, H, H, Cout), float("nan"), device=DEV)
    d = _desc(nat, B, H, Cin, Cout, tile)
    d.Wwino, d.act = U.data_ptr(), act
    nat.call("po_conv", ctypes.byref(d), nat.ptr(xd), nat.ptr(wd), nat.ptr(bd), nat.ptr(y), None, None, None, None,
             None, nat.stream())
    h = H // 2
    py = torch.full((B, h, h, Cout), float("nan"), device=DEV)
    pam = torch.full((B, h, h, Cout), -1, dtype=torch.int8, device=DEV)
    slot = torch.zeros(64, dtype=torch.int32, device=DEV)
    d = _desc(nat, B, H, Cin, Cout, tile)
    d.Wwino, d.act = U.data_ptr(), act
    d.pool_y, d.pool_argmax, d.y_amax = py.data_ptr(), pam.data_ptr(), slot.data_ptr()
    nat.call("po_conv", ctypes.byref(d), nat.ptr(xd), nat.ptr(wd), nat.ptr(bd), None, None, None, None, None,
             None, nat.stream())
    torch.cuda.synchronize()
    win = y.view(B, h, 2, h, 2, Cout)
    pv, arg = win[:, :, 0, :, 0], torch.zeros(B, h, h, Cout, dtype=torch.int64, device=DEV)
    for k in range(1, 4):
        v = win[:, :, k >> 1, :, k & 1]
        upd = (v > pv) | torch.isnan(v)
        pv, arg = torch.where(upd, v, pv), torch.where(upd, torch.full_like(arg, k), arg)
    if act:
        arg = arg | 8 | torch.where(pv > 0, 0, 4)
    assert torch.equal(py, pv)
    assert torch.equal(pam.long(), arg)
    assert int(slot.max()) == int(pv.abs().max().view(torch.int32))
    d.tile = 65
    assert nat.load().po_conv(ctypes.byref(d), nat.ptr(xd), nat.ptr(wd), nat.ptr(bd), None, None, None, None, None,
                              None, nat.stream()) != 0


@pytest.mark.parametrize("tile", [66, 67, 68])
@pytest.mark.parametrize("ks", [2, 3])
@pytest.mark.parametrize("boxed", [False, True])
@pytest.mark.parametrize("mode", ["fwd_bits", "fwd_shortcut", "dgrad_acc_bits", "dgrad_dual"])
def test_wino_tile66_split_k(mode, boxed, ks, tile):
    """Tile 66 with input-channel slices (blockIdx.y) writing raw partial
    sums at conv_reduce_k's GEMM rows (the box's compact rows with gbox), the
    reduction applying the epilogue: the unsplit launch's values within the
    fp32 summation-order class, untouched pixels outside the box, sign bits of
    the written values and max|x| slots bounding them; odd map side."""
    nat = pkg_mod("_native")
    B, H, Cin, Cout = 3, 19, 256, 128
    flip = mode.startswith("dgrad")
    x, w, bias, wd, U = _setup(B, H, Cin, Cout, flip, seed=11)
    gen = torch.Generator().manual_seed(12)
    xd = x.permute(0, 2, 3, 1).contiguous().to(DEV)
    prev = torch.randn(B, H, H, Cout, generator=gen).to(DEV)
    res = torch.randn(B, H, H, Cout, generator=gen).to(DEV)
    mbits = torch.randint(-2 ** 31, 2 ** 31 - 1, (B, H, H, Cout // 32), generator=gen, dtype=torch.int32).to(DEV)
    m2bits = torch.randint(-2 ** 31, 2 ** 31 - 1, (B, H, H, Cout // 32), generator=gen, dtype=torch.int32).to(DEV)
    box = torch.tensor([[3, 5, 14, 18], [0, 0, 19, 19], [11, 0, 12, 19]], dtype=torch.int32, device=DEV)
    ws = torch.full((ks * B * H * H * Cout,), float("nan"), device=DEV)
    runs = []
    for split in (1, ks):
        d = _desc(nat, B, H, Cin, Cout, tile, flip)
        d.Wwino = U.data_ptr()
        if split > 1:
            d.ksplit, d.workspace = split, ws.data_ptr()
        d.gbox = box.data_ptr() if boxed else None
        y = prev.clone()
        ssum = torch.full_like(prev, float("nan"))
        y2 = torch.full_like(prev, float("nan"))
        bits = torch.zeros(B, H, H, Cout // 32, dtype=torch.int32, device=DEV)
        slots = [torch.zeros(64, dtype=torch.int32, device=DEV) for _ in range(3)]
        args = dict(bias=None, res=None, sum=None, y2=None)
        if mode == "fwd_bits":
            d.act, d.ybits = 1, bits.data_ptr()
            args["bias"] = bias.to(DEV)
        elif mode == "fwd_shortcut":
            d.act, d.ybits = 1, bits.data_ptr()
            args.update(bias=bias.to(DEV), res=res, sum=ssum)
            d.sum_amax = slots[1].data_ptr()
        elif mode == "dgrad_acc_bits":
            d.accumulate, d.mbits = 1, mbits.data_ptr()
        else:
            d.mbits, d.m2bits = mbits.data_ptr(), m2bits.data_ptr()
            args["y2"] = y2
            d.y2_amax = slots[2].data_ptr()
        d.y_amax = slots[0].data_ptr()
        nat.call("po_conv", ctypes.byref(d), nat.ptr(xd), nat.ptr(wd), nat.ptr(args["bias"]), nat.ptr(y),
                 nat.ptr(args["res"]), nat.ptr(args["sum"]), None, nat.ptr(args["y2"]), None, nat.stream())
        torch.cuda.synchronize()
        runs.append((y.cpu(), ssum.cpu(), y2.cpu(), bits.cpu(), [sl.cpu().view(torch.float32).max() for sl in slots]))
    (y1, s1, z1, b1, sl1), (yk, sk, zk, bk, slk) = runs
    inside = torch.ones(B, H, H, dtype=torch.bool)
    if boxed:
        inside[:] = False
        for b, (r0, c0, r1, c1) in enumerate(box.cpu().tolist()):
            inside[b, r0:r1, c0:c1] = True
    assert torch.equal(yk[~inside], prev.cpu()[~inside])
    assert _rel(yk[inside], y1[inside]) < 1e-5
    if mode.startswith("fwd"):
        sh = torch.arange(32, dtype=torch.int32)
        got = ((bk.unsqueeze(-1) >> sh) & 1).reshape(B, H, H, Cout).bool()
        assert torch.equal(got[inside], yk[inside] > 0)
    if mode == "fwd_shortcut":
        assert _rel(sk[inside], s1[inside]) < 1e-5 and float(slk[1]) >= float(sk[inside].abs().max())
    if mode == "dgrad_dual":
        assert _rel(zk[inside], z1[inside]) < 1e-5 and float(slk[2]) >= float(zk[inside].abs().max())
    assert float(slk[0]) >= float(yk[inside].abs().max()) * (1 - 1e-7)

