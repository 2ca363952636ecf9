"""po_conv's in-launch split-K reduction (ABI 28, po_conv_desc.tile_ctr): the
tile's last-arriving slice sums the partials in split order and applies the
epilogue inside the conv launch instead of in conv_reduce_k.  It runs the same
item code in the same order, so every output must be bit-identical to the
two-kernel form, for every generic exact-fp32 tile, split count and epilogue
the plans use (leaky + bias, sign bits, shortcut sum, accumulate with
sign-bit masks and a dual output, gradient-cone boxes with a compact grid);
the counters are left zero for the next launch."""
import ctypes

import pytest
import torch

from conftest import pkg_mod

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)
GENERIC_TILES = list(range(1, 21)) + [27]


def _launch(nat, ops, tile, ks, inlaunch, epi, box=None, mrows=0, ctr=None):
    x, w, bias, res, y0, mb, m2b = ops
    B, H, _, Cin = x.shape
    N = w.shape[0]
    Hg = H
    d = nat.po_conv_desc()
    d.B, d.Hin, d.Win, d.Cin_p, d.Hout, d.Wout, d.Cout_p, d.Hg, d.Wg = B, H, H, Cin, H, H, N, Hg, Hg
    d.in_step, d.out_step, d.ntaps, d.N, d.act, d.tile = 1, 1, 9, N, 1, tile
    for kh in range(3):
        for kw in range(3):
            d.dh[kh * 3 + kw], d.dw[kh * 3 + kw] = kh - 1, kw - 1
    M = B * (mrows or Hg * Hg)
    ws = torch.full((ks * M * N,), float("nan"), device=DEV)
    d.ksplit, d.workspace = ks, ws.data_ptr()
    d.mrows = mrows
    if inlaunch:
        d.tile_ctr, d.tile_ctr_n = ctr.data_ptr(), ctr.numel()
    d.gbox = box.data_ptr() if box is not None else None
    y = y0.clone() if epi == "acc" else torch.full_like(y0, float("nan"))
    s = torch.full_like(y0, float("nan")) if epi == "sum" else None
    y2 = torch.full_like(y0, float("nan")) if epi == "acc" else None
    wpp = N // 32
    ybits = torch.zeros(B * H * H * wpp, dtype=torch.int32, device=DEV) if epi in ("plain", "sum") else None
    d.ybits = ybits.data_ptr() if ybits is not None else None
    if epi == "acc":
        d.accumulate = 1
        d.mbits, d.m2bits = mb.data_ptr(), m2b.data_ptr()
    nat.call("po_conv", ctypes.byref(d), nat.ptr(x), nat.ptr(w), nat.ptr(bias), nat.ptr(y),
             nat.ptr(res) if epi == "sum" else None, nat.ptr(s) if epi == "sum" else None, None,
             nat.ptr(y2) if y2 is not None else None, None, nat.stream())
    torch.cuda.synchronize()
    return [t for t in (y, s, y2, ybits) if t is not None]


def _operands(B, H, Cin, N, seed):
    gen = torch.Generator().manual_seed(seed)
    x = torch.randn(B, H, H, Cin, generator=gen).to(DEV)
    w = (torch.randn(N, 9, Cin, generator=gen) * (2.0 / (9 * Cin)) ** 0.5).to(DEV)
    bias = (torch.randn(N, generator=gen) * 0.1).to(DEV)
    res = torch.randn(B, H, H, N, generator=gen).to(DEV)
    y0 = torch.randn(B, H, H, N, generator=gen).to(DEV)
    mb = torch.randint(-2 ** 31, 2 ** 31 - 1, (B * H * H * N // 32,), generator=gen, dtype=torch.int64)
    m2b = torch.randint(-2 ** 31, 2 ** 31 - 1, (B * H * H * N // 32,), generator=gen, dtype=torch.int64)
    return x, w, bias, res, y0, mb.to(torch.int32).to(DEV), m2b.to(torch.int32).to(DEV)


@pytest.mark.parametrize("tile", GENERIC_TILES)
@pytest.mark.parametrize("epi", ["plain", "sum", "acc"])
def test_inlaunch_reduce_bit_identical(tile, epi):
    nat = pkg_mod("_native")
    B, H, Cin, N = 3, 7, 64, 96          # 147 rows (ragged m tiles), 96 channels (ragged 64/128/256 n tiles)
    ops = _operands(B, H, Cin, N, seed=tile)
    ctr = torch.zeros(4096, dtype=torch.int32, device=DEV)
    for ks in (2, 3, 8, 16):
        want = _launch(nat, ops, tile, ks, False, epi)
        got = _launch(nat, ops, tile, ks, True, epi, ctr=ctr)
        again = _launch(nat, ops, tile, ks, True, epi, ctr=ctr)      # counters reset by the last arriver
        for a, b, c in zip(want, got, again):
            assert torch.equal(a.view(torch.int32), b.view(torch.int32)), (ks, epi)
            assert torch.equal(a.view(torch.int32), c.view(torch.int32)), (ks, epi)
        assert int(ctr.abs().sum()) == 0
        assert not torch.isnan(want[0]).any()


@pytest.mark.parametrize("tile", [3, 7, 11, 13, 17, 18])
def test_inlaunch_reduce_boxed_compact_grid(tile):
    """Gradient-cone boxes over a compact grid (mrows < Hg*Wg; dead rows and
    an empty box): inside the boxes bit-identical, outside untouched."""
    nat = pkg_mod("_native")
    B, H, Cin, N = 4, 9, 32, 64
    ops = _operands(B, H, Cin, N, seed=50 + tile)
    box = torch.tensor([[1, 2, 5, 6], [0, 0, 4, 4], [3, 3, 3, 7], [5, 4, 9, 8]], dtype=torch.int32, device=DEV)
    ctr = torch.zeros(64, dtype=torch.int32, device=DEV)
    for ks in (2, 5, 16):
        want = _launch(nat, ops, tile, ks, False, "acc", box=box, mrows=16)
        got = _launch(nat, ops, tile, ks, True, "acc", box=box, mrows=16, ctr=ctr)
        for a, b in zip(want, got):
            assert torch.equal(a.view(torch.int32), b.view(torch.int32)), ks
        assert int(ctr.abs().sum()) == 0


def test_too_few_counters_falls_back_to_the_reduce_kernel():
    """More output tiles than counters: the separate reduction runs (same bits)."""
    nat = pkg_mod("_native")
    ops = _operands(3, 7, 64, 96, seed=9)
    ctr = torch.zeros(1, dtype=torch.int32, device=DEV)
    want = _launch(nat, ops, 17, 4, False, "plain")
    got = _launch(nat, ops, 17, 4, True, "plain", ctr=ctr)
    for a, b in zip(want, got):
        assert torch.equal(a.view(torch.int32), b.view(torch.int32))
    assert int(ctr[0]) == 0
