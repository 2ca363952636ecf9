"""po_conv tile 69 (conv_halo.hip): the persistent 3x3 16 -> 32-channel conv
with its 2x2/2 max pool fused (yolov3-tiny's 208x208 conv + pool,
darknet_v3.py:37-69).  Pooled values, argmax/slope bytes and the max|x| slot
are bit-identical to the generic direct tile (9: 128 x 32 x 16, the tile the
committed tiny cache used before) on the same pooled launch, and agree with
a float64 conv + pool; ragged tile edges (maps not a multiple of 8 x 16),
both tap orientations, and the launches the tile must refuse."""
import ctypes

import pytest
import torch
import torch.nn.functional as F

from conftest import pkg_mod

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _desc(nat, B, H, W, tile, flip, act):
    d = nat.po_conv_desc()
    d.B, d.Hin, d.Win, d.Cin_p, d.Hout, d.Wout, d.Cout_p, d.Hg, d.Wg = B, H, W, 16, H, W, 32, H, W
    d.in_step, d.out_step, d.ntaps, d.N, d.act, d.tile, d.prec = 1, 1, 9, 32, act, tile, 0
    s = -1 if flip else 1
    for kh in range(3):
        for kw in range(3):
            d.dh[kh * 3 + kw], d.dw[kh * 3 + kw] = s * (kh - 1), s * (kw - 1)
    return d


def _run(nat, tile, xd, wd, bd, B, H, W, flip, act):
    py = torch.full((B, H // 2, W // 2, 32), float("nan"), device=DEV)
    pam = torch.full((B, H // 2, W // 2, 32), -1, dtype=torch.int8, device=DEV)
    slot = torch.zeros(64, dtype=torch.int32, device=DEV)
    d = _desc(nat, B, H, W, tile, flip, act)
    d.pool_y, d.pool_argmax, d.y_amax = py.data_ptr(), pam.data_ptr(), slot.data_ptr()
    nat.call("po_conv", ctypes.byref(d), nat.ptr(xd), nat.ptr(wd), nat.ptr(bd), None, None, None, None, None, None,
             nat.stream())
    torch.cuda.synchronize()
    return py, pam, slot


@pytest.mark.parametrize("B,H,W", [(3, 208, 208), (2, 26, 34), (5, 40, 18), (1, 2, 2)])
@pytest.mark.parametrize("flip", [False, True])
@pytest.mark.parametrize("act", [1, 0])
def test_halo_pool_bit_identical_to_generic_tile(B, H, W, flip, act):
    nat = pkg_mod("_native")
    gen = torch.Generator().manual_seed(H * 7 + W + flip)
    x = torch.randn(B, 16, H, W, generator=gen)
    w = torch.randn(32, 16, 3, 3, generator=gen) * (2.0 / 144) ** 0.5
    bias = torch.randn(32, generator=gen) * 0.1
    x[0, :, :2, :2] = 0.0                                    # ties: equal window values (first position wins)
    wk = w.flip(2, 3) if flip else w
    wd = wk.permute(0, 2, 3, 1).reshape(32, 9, 16).contiguous().to(DEV)
    xd, bd = x.permute(0, 2, 3, 1).contiguous().to(DEV), bias.to(DEV)
    py69, pam69, slot69 = _run(nat, 69, xd, wd, bd, B, H, W, flip, act)
    py9, pam9, slot9 = _run(nat, 9, xd, wd, bd, B, H, W, flip, act)
    assert torch.equal(py69, py9)
    assert torch.equal(pam69, pam9)
    assert torch.equal(slot69.max(), slot9.max())
    # float64 reference: conv (+ bias, leaky) then the 2x2 max
    y = F.conv2d(x.double(), w.double(), bias.double(), padding=1)
    if act:
        y = F.leaky_relu(y, 0.1)
    ref = F.max_pool2d(y, 2).permute(0, 2, 3, 1)
    assert float((py69.double().cpu() - ref).abs().max()) <= 1e-5 * max(1.0, float(ref.abs().max()))


def test_halo_refuses_what_it_cannot_run():
    nat = pkg_mod("_native")
    lib = nat.load()
    B, H = 2, 16
    xd = torch.zeros(B, H, H, 32, device=DEV)
    wd = torch.zeros(32, 9, 32, device=DEV)
    bd = torch.zeros(32, device=DEV)
    py = torch.zeros(B, H // 2, H // 2, 32, device=DEV)
    pam = torch.zeros(B, H // 2, H // 2, 32, dtype=torch.int8, device=DEV)
    y = torch.zeros(B, H, H, 32, device=DEV)

    def call(d, yout=None):
        return lib.po_conv(ctypes.byref(d), nat.ptr(xd), nat.ptr(wd), nat.ptr(bd), nat.ptr(yout), None, None, None,
                           None, None, nat.stream())

    d = _desc(nat, B, H, H, 69, False, 1)
    assert call(d, y) != 0                                   # no pool: the generic tiles' job
    d.pool_y, d.pool_argmax = py.data_ptr(), pam.data_ptr()
    d.Cin_p = 32                                             # 32 input channels
    assert call(d) != 0
    d.Cin_p = 16
    d.ksplit, d.workspace = 2, xd.data_ptr()                 # split-K
    assert call(d) != 0
    torch.cuda.synchronize()


def test_conv_refuses_destinations_past_2_31_elements():
    """The po_conv epilogues index the destination in 32 bits: a launch whose
    destination holds 2^31 or more elements is refused before anything runs."""
    nat = pkg_mod("_native")
    lib = nat.load()
    xd = torch.zeros(16, device=DEV)
    d = _desc(nat, 1 << 11, 208, 208, 9, False, 1)           # 2^11 x 208 x 208 pixels x 32 channels > 2^31
    rc = lib.po_conv(ctypes.byref(d), nat.ptr(xd), nat.ptr(xd), nat.ptr(xd), nat.ptr(xd), None, None, None, None,
                     None, nat.stream())
    assert rc != 0
    assert "2^31" in nat.last_error()
