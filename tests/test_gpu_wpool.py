"""po_conv tile 73 (conv_wpool.hip): tile 69's launch -- stride-1 3x3, 16 -> 32
channels, the 2x2/2 max pool fused -- as Winograd F(2x2,3x3) on 16x16x4 MFMAs
with the inverse transform and the pool in registers.  Its k order is tile
61's, so pooled values, window positions and slope codes must be
bit-identical to tile 61 on the same launch (both tap orientations, linear and
leaky, ragged 8 x 16-pixel tiles at the map edges, the bench layer's 208^2
map); and within the Winograd tolerance of a float64 conv + pool."""
import ctypes

import pytest
import torch
import torch.nn.functional as F

from conftest import pkg_mod
from test_gpu_wino import _desc, _setup

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _pooled(nat, d, xd, wd, bd, B, H, C):
    h = H // 2
    py = torch.full((B, h, h, C), float("nan"), device=DEV)
    pam = torch.full((B, h, h, C), -1, dtype=torch.int8, device=DEV)
    slot = torch.zeros(64, dtype=torch.int32, device=DEV)
    d.pool_y, d.pool_argmax, d.y_amax = py.data_ptr(), pam.data_ptr(), slot.data_ptr()
    nat.call("po_conv", ctypes.byref(d), nat.ptr(xd), nat.ptr(wd), nat.ptr(bd), None, None, None, None, None, None,
             nat.stream())
    torch.cuda.synchronize()
    return py, pam, slot


@pytest.mark.parametrize("act", [0, 1])
@pytest.mark.parametrize("flip", [False, True])
@pytest.mark.parametrize("B,H", [(2, 52), (3, 34), (1, 18), (2, 208)])
def test_wpool_bit_identical_to_tile61(B, H, flip, act):
    nat = pkg_mod("_native")
    Cin, Cout = 16, 32
    x, w, bias, wd, U = _setup(B, H, Cin, Cout, flip, seed=H + 3 * act + flip)
    xd = x.permute(0, 2, 3, 1).contiguous().to(DEV)
    bd = bias.to(DEV)
    out = {}
    for tile in (61, 73):
        d = _desc(nat, B, H, Cin, Cout, tile, flip)
        d.Wwino, d.act = U.data_ptr(), act
        out[tile] = _pooled(nat, d, xd, wd, bd, B, H, Cout)
    (p61, a61, s61), (p73, a73, s73) = out[61], out[73]
    assert not torch.isnan(p73).any()
    assert torch.equal(p73.view(torch.int32), p61.view(torch.int32))
    assert torch.equal(a73, a61)
    assert int(s73.max()) == int(s61.max())
    if not flip:
        # and a conv + LeakyReLU + pool in float64 of the same operands (Winograd tolerance)
        ref = F.conv2d(x.double(), w.double(), bias.double(), padding=1)
        if act:
            ref = torch.where(ref > 0, ref, 0.1 * ref)
        ref = F.max_pool2d(ref, 2).permute(0, 2, 3, 1)
        err = float((p73.cpu().double() - ref).abs().max() / ref.abs().max())
        assert err < 1e-5, err


def test_wpool_refuses_other_launches():
    """No Wwino, N != 32, no pool, split-K: refused (the tuner then skips the tile)."""
    nat = pkg_mod("_native")
    lib = nat.load()
    B, H = 1, 16
    x, w, bias, wd, U = _setup(B, H, 16, 32, False, seed=1)
    xd = x.permute(0, 2, 3, 1).contiguous().to(DEV)
    bd = bias.to(DEV)
    py = torch.zeros(B, H // 2, H // 2, 32, device=DEV)
    pam = torch.zeros(B, H // 2, H // 2, 32, dtype=torch.int8, device=DEV)
    y = torch.zeros(B, H, H, 32, device=DEV)

    def run(d, yy=None):
        return lib.po_conv(ctypes.byref(d), nat.ptr(xd), nat.ptr(wd), nat.ptr(bd), nat.ptr(yy) if yy is not None else None,
                           None, None, None, None, None, nat.stream())
    d = _desc(nat, B, H, 16, 32, 73)
    d.pool_y, d.pool_argmax = py.data_ptr(), pam.data_ptr()
    assert run(d) != 0                                   # no Wwino
    d = _desc(nat, B, H, 16, 32, 73)
    d.Wwino = U.data_ptr()
    assert run(d, y) != 0                                # not a pooled launch
    torch.cuda.synchronize()
