"""po_cell_loss spread over workgroups (a scratch buffer, one workgroup per 16
images) gives the same bits as the one-workgroup form: forward terms, the
objectness/class extraction, cells, flags and the head gradients, for every
objective (reference train_patch.py:428-577)."""
import pytest
import torch

from conftest import pkg_mod

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


@pytest.mark.parametrize("objective", [0, 1, 2])
@pytest.mark.parametrize("B", [1, 16, 100, 256])
def test_cell_loss_multi_workgroup_is_bit_identical(objective, B):
    nat = pkg_mod("_native")
    g = torch.Generator().manual_seed(B + objective)
    hw = [13, 26]
    Cp = 64
    heads = [torch.randn(B, h, h, Cp, generator=g).to(DEV) * 3 for h in hw]
    center = (torch.rand(B, 2, generator=g) * 416).to(DEV)
    g2 = torch.tensor([0.7, 1.3], device=DEV)
    hwa = (nat.c_int * 2)(*hw)
    res = []
    for use_scratch in (False, True):
        out2 = torch.empty(2, device=DEV)
        obj = torch.empty(B, 6, device=DEV)
        cls = torch.empty(B, 6, 15, device=DEV)
        cells = torch.empty(2, B, dtype=torch.int32, device=DEV)
        flags = torch.zeros(1, dtype=torch.int32, device=DEV)
        scratch = torch.empty(2 * B, device=DEV) if use_scratch else None
        nat.call("po_cell_loss", nat.ptr_array(heads), hwa, None, None, 2, Cp, B, 416, nat.ptr(center), 14,
                 objective, None, None, nat.ptr(out2), nat.ptr(obj), nat.ptr(cls), nat.ptr(cells, torch.int32),
                 nat.ptr(flags, torch.int32), nat.ptr(scratch), nat.stream())
        d_heads = [torch.zeros_like(h) for h in heads]
        out2b = torch.empty(2, device=DEV)
        nat.call("po_cell_loss", nat.ptr_array(heads), hwa, None, None, 2, Cp, B, 416, nat.ptr(center), 14,
                 objective, nat.ptr(g2), nat.ptr_array(d_heads), nat.ptr(out2b), None, None, None, None,
                 nat.ptr(scratch), nat.stream())
        res.append((out2, obj, cls, cells, flags, out2b, *d_heads))
    for a, b in zip(*res):
        assert torch.equal(a, b)
