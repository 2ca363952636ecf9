"""po_view_move (window <-> full-map moves of the receptive-field windows,
darknet_v3.py route/upsample plumbing, reference darknet_v3.py:195-220) on
the GPU: the 16-byte vector kernel is bit-identical to the scalar kernel
(the dispatch's fallback for buffers off 16-byte alignment) in all three modes (copy, nearest-x2 read, 2x2-sum
upsample gradient), with and without accumulation, LeakyReLU-gradient mask,
channel offsets and window origins (including views partly outside the
source, which read zero), and to a plain PyTorch restatement of mode 0."""
import pytest
import torch

from conftest import pkg_mod

pytestmark = pytest.mark.gpu


def _move(src, Hs, Ws, ss, so, sorg, dst, Hd, Wd, ds, doff, dorg, B, C, mode, acc, mask, ms, v1):
    nat = pkg_mod("_native")
    P = lambda t: nat.c_void_p(t.data_ptr()) if t is not None else None
    amax = torch.zeros(nat.PO_AMAX_SUB, dtype=torch.int32, device=src.device)
    if v1:
        # one float off 16-byte alignment: the dispatch falls back to the scalar kernel
        def shifted(t):
            buf = torch.empty(t.numel() + 4, device=t.device)[1:1 + t.numel()].view(t.shape)
            return buf.copy_(t)
        src_, dst_ = shifted(src), shifted(dst)
    else:
        src_, dst_ = src, dst
    nat.call("po_view_move", P(src_), Hs, Ws, ss, so, P(sorg), P(dst_), Hd, Wd, ds, doff, P(dorg), B, C, mode, acc,
             P(mask), ms, P(amax), nat.stream())
    torch.cuda.synchronize()
    if v1:
        dst.copy_(dst_)
    return amax.view(torch.float32).max().item()


@pytest.mark.parametrize("mode", [0, 1, 2])
@pytest.mark.parametrize("acc,masked", [(0, False), (1, True)])
def test_view_move_vector_bit_identical(mode, acc, masked):
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(17 * mode + acc)
    B, C, ss, so, ds, doff = 3, 48, 64, 8, 80, 16
    Hs, Ws = 11, 13
    Hd, Wd = (9, 10) if mode != 2 else (5, 6)
    src = torch.randn(B, Hs, Ws, ss, generator=g).to(dev)
    sorg = torch.tensor([[0, 0], [2, 1], [-1, 3]], dtype=torch.int32, device=dev)
    dorg = torch.tensor([[1, 2], [0, 0], [3, 1]], dtype=torch.int32, device=dev)
    mask = torch.randn(B, Hd, Wd, ds, generator=g).to(dev) if masked else None
    base = torch.randn(B, Hd, Wd, ds, generator=g).to(dev)
    outs = []
    for v1 in (False, True):
        dst = base.clone()
        m = _move(src, Hs, Ws, ss, so, sorg, dst, Hd, Wd, ds, doff, dorg, B, C, mode, acc, mask, ds if masked else 0,
                  v1)
        outs.append((dst, m))
    assert torch.equal(outs[0][0], outs[1][0])
    assert outs[0][1] == outs[1][1]
    if mode == 0 and not acc:
        ref = base.clone()
        for b in range(B):
            for y in range(Hd):
                for x in range(Wd):
                    ly, lx = y + int(dorg[b, 0]) - int(sorg[b, 0]), x + int(dorg[b, 1]) - int(sorg[b, 1])
                    ok = 0 <= ly < Hs and 0 <= lx < Ws
                    ref[b, y, x, doff:doff + C] = src[b, ly, lx, so:so + C] if ok else 0.0
        assert torch.equal(outs[0][0], ref)
