"""po_conv tile 70 (conv_wino5_k, csrc/conv_wino5.hip): tile 68 as a
persistent kernel pipelined across its units.  Per unit it runs tile 68's
transforms, MFMA order, inverse transform and epilogue arithmetic, so every
output it writes must be bit-identical to tile 68's: each epilogue-field
combination the training plan launches (sign bits, fused shortcut,
accumulate, leaky masks as bits, dual output), both tap orientations (forward
and the input-gradient launches' flipped taps), ragged tile counts and odd
maps, launches with one unit per workgroup and with many, split-K slices
(conv_reduce_k) and the fused max pool; and it refuses what it cannot run."""
import ctypes

import pytest
import torch

from conftest import pkg_mod
from test_gpu_wino import _desc, _setup

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)
MODES = ["fwd_bits", "fwd_shortcut", "fwd_shortcut_nobits", "fwd_plain", "dgrad_mask", "dgrad_acc_bits",
         "dgrad_dual", "dgrad_acc_dual", "dgrad_acc"]


def _run(nat, tile, mode, B, H, Cin, Cout, flip, U, xd, wd, bias, prev, res, mbits, m2bits, ksplit=1, ws=None,
         drop_y=False):
    d = _desc(nat, B, H, Cin, Cout, tile, flip)
    d.Wwino = U.data_ptr()
    if ksplit > 1:
        d.ksplit, d.workspace = ksplit, ws.data_ptr()
    y = prev.clone()
    ssum = torch.full_like(prev, float("nan"))
    y2 = torch.full_like(prev, float("nan"))
    bits = torch.zeros(B, H, H, Cout // 32, dtype=torch.int32, device=DEV)
    args = dict(bias=None, res=None, sum=None, y2=None)
    if mode in ("fwd_bits", "fwd_shortcut", "fwd_plain"):
        d.act = 1
        args["bias"] = bias
        if mode != "fwd_plain":
            d.ybits = bits.data_ptr()
        if mode == "fwd_shortcut":
            args.update(res=res, sum=ssum)
    elif mode == "fwd_shortcut_nobits":
        d.act = 1
        args.update(bias=bias, res=res, sum=ssum)
    elif mode == "dgrad_mask":
        d.mbits = mbits.data_ptr()
    elif mode == "dgrad_acc_bits":
        d.accumulate, d.mbits = 1, mbits.data_ptr()
    elif mode == "dgrad_acc":
        d.accumulate = 1
    else:
        d.mbits, d.m2bits = mbits.data_ptr(), m2bits.data_ptr()
        d.accumulate = int(mode == "dgrad_acc_dual")
        args["y2"] = y2
    yp = None if drop_y else y
    nat.call("po_conv", ctypes.byref(d), nat.ptr(xd), nat.ptr(wd), nat.ptr(args["bias"]), nat.ptr(yp),
             nat.ptr(args["res"]), nat.ptr(args["sum"]), None, nat.ptr(args["y2"]), None, nat.stream())
    torch.cuda.synchronize()
    return y, ssum, y2, bits


def _inputs(B, H, Cin, Cout, flip, seed):
    x, w, bias, wd, U = _setup(B, H, Cin, Cout, flip, seed=seed)
    gen = torch.Generator().manual_seed(seed + 1)
    xd = x.permute(0, 2, 3, 1).contiguous().to(DEV)
    prev = torch.randn(B, H, H, Cout, generator=gen).to(DEV)
    res = torch.randn(B, H, H, Cout, generator=gen).to(DEV)
    mbits = torch.randint(-2 ** 31, 2 ** 31 - 1, (B, H, H, Cout // 32), generator=gen, dtype=torch.int32).to(DEV)
    m2bits = torch.randint(-2 ** 31, 2 ** 31 - 1, (B, H, H, Cout // 32), generator=gen, dtype=torch.int32).to(DEV)
    return xd, wd, bias.to(DEV), U, prev, res, mbits, m2bits


def _equal(a, b):
    for u, v in zip(a, b):
        assert torch.equal(u.nan_to_num(7.0), v.nan_to_num(7.0))


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("B,H,Cin,Cout", [(2, 11, 64, 128), (3, 38, 256, 512), (1, 19, 512, 64), (2, 7, 32, 64),
                                          (16, 76, 128, 256)])
def test_tile70_bit_identical_to_68(mode, B, H, Cin, Cout):
    """(16, 76, 128, 256) is a bench shape: 1,444 units over the CUs, ~6 per
    workgroup; the others hold one to a few units per workgroup, odd sides
    leave ragged 2x2 tiles, (2, 7, 32, 64) has exactly two k-steps."""
    nat = pkg_mod("_native")
    flip = mode.startswith("dgrad")
    xd, wd, bias, U, prev, res, mbits, m2bits = _inputs(B, H, Cin, Cout, flip, seed=H + Cin)
    runs = [_run(nat, t, mode, B, H, Cin, Cout, flip, U, xd, wd, bias, prev, res, mbits, m2bits) for t in (70, 68)]
    _equal(runs[0], runs[1])
    if mode == "fwd_bits":
        assert bool((runs[0][3] != 0).any())        # the sign bits were written


def test_tile70_sum_only_forward():
    """A forward conv whose activation is kept only as sign bits before a fused
    shortcut (y_out NULL, NetPlan._drop_mask_only_outputs): sum and bits as tile 68."""
    nat = pkg_mod("_native")
    B, H, Cin, Cout = 2, 38, 128, 256
    xd, wd, bias, U, prev, res, mbits, m2bits = _inputs(B, H, Cin, Cout, False, seed=3)
    runs = [_run(nat, t, "fwd_shortcut", B, H, Cin, Cout, False, U, xd, wd, bias, prev, res, mbits, m2bits,
                 drop_y=True) for t in (70, 68)]
    _equal(runs[0], runs[1])
    assert torch.equal(runs[0][0], prev)             # y untouched


@pytest.mark.parametrize("Cin,ks", [(512, 2), (512, 4), (512, 3), (512, 6), (256, 3)])
@pytest.mark.parametrize("mode", ["fwd_bits", "dgrad_acc_bits", "dgrad_dual"])
def test_tile70_split_k_bit_identical_to_68(mode, Cin, ks):
    """Even slices (32 k-steps over 2 or 4) and the uneven ones the tuner also
    offers (ks 3 and 6: slice bounds by the host's magic-number division;
    32 k-steps -> 10/11/11 and 5/5/5/5/6/6, 16 -> 5/5/6)."""
    nat = pkg_mod("_native")
    B, H, Cout = 4, 19, 256
    flip = mode.startswith("dgrad")
    xd, wd, bias, U, prev, res, mbits, m2bits = _inputs(B, H, Cin, Cout, flip, seed=17)
    runs = []
    for t in (70, 68):
        ws = torch.full((ks * B * H * H * Cout,), float("nan"), device=DEV)
        runs.append(_run(nat, t, mode, B, H, Cin, Cout, flip, U, xd, wd, bias, prev, res, mbits, m2bits, ksplit=ks,
                         ws=ws))
    _equal(runs[0], runs[1])


@pytest.mark.parametrize("act", [0, 1])
@pytest.mark.parametrize("B,H,Cin,Cout", [(2, 12, 64, 128), (8, 52, 64, 128), (2, 104, 32, 64)])
def test_tile70_fused_pool_bit_identical_to_68(act, B, H, Cin, Cout):
    nat = pkg_mod("_native")
    x, w, bias, wd, U = _setup(B, H, Cin, Cout, False, seed=H + Cout)
    xd = x.permute(0, 2, 3, 1).contiguous().to(DEV)
    bd = bias.to(DEV)
    h = H // 2
    out = []
    for tile in (70, 68):
        py = torch.full((B, h, h, Cout), float("nan"), device=DEV)
        pam = torch.full((B, h, h, Cout), -1, dtype=torch.int8, device=DEV)
        d = _desc(nat, B, H, Cin, Cout, tile)
        d.Wwino, d.act = U.data_ptr(), act
        d.pool_y, d.pool_argmax = py.data_ptr(), pam.data_ptr()
        nat.call("po_conv", ctypes.byref(d), nat.ptr(xd), nat.ptr(wd), nat.ptr(bd), None, None, None, None, None,
                 None, nat.stream())
        torch.cuda.synchronize()
        out.append((py, pam))
    assert torch.equal(out[0][0], out[1][0]) and torch.equal(out[0][1], out[1][1])


def test_tile70_refuses_what_it_cannot_run():
    nat = pkg_mod("_native")
    B, H, Cin, Cout = 2, 16, 32, 64
    xd, wd, bias, U, prev, res, mbits, m2bits = _inputs(B, H, Cin, Cout, False, seed=9)
    y = torch.zeros(B, H, H, Cout, device=DEV)

    def call(d, mask=None):
        return nat.load().po_conv(ctypes.byref(d), nat.ptr(xd), nat.ptr(wd), None, nat.ptr(y), None, None,
                                  nat.ptr(mask), None, None, nat.stream())

    d = _desc(nat, B, H, Cin, Cout, 70)
    assert call(d) != 0 and "Wwino" in nat.last_error()
    d.Wwino = U.data_ptr()
    assert call(d) == 0
    box = torch.tensor([[0, 0, 8, 8]] * B, dtype=torch.int32, device=DEV)
    d.gbox = box.data_ptr()
    assert call(d) != 0 and "boxes" in nat.last_error()              # gradient-cone boxes: tiles 66-68
    d.gbox = None
    slot = torch.zeros(64, dtype=torch.int32, device=DEV)
    d.y_amax = slot.data_ptr()
    assert call(d) != 0                                             # max|x| slots (fp16x3 plans)
    d.y_amax = None
    assert call(d, mask=prev) != 0                                  # fp32 leaky masks
    ws = torch.empty(4 * B * H * H * Cout, device=DEV)
    d.ksplit, d.workspace = 2, ws.data_ptr()
    assert call(d) != 0 and "two k-steps" in nat.last_error()       # one k-step per slice
    d = _desc(nat, 2, 16, 16, 64, 70)
    _, _, _, wd16, U16 = _setup(2, 16, 16, 64, False, seed=1)
    d.Wwino = U16.data_ptr()
    x16 = torch.zeros(2, 16, 16, 16, device=DEV)
    assert nat.load().po_conv(ctypes.byref(d), nat.ptr(x16), nat.ptr(wd16), None, nat.ptr(y), None, None, None,
                              None, None, nat.stream()) != 0       # Cin_p = 16: a single k-step
