"""po_loss_combine / po_loss_combine_bwd (train_patch.combine_terms_device):
the iteration's loss from the cell-loss pair and the regularisers in one
launch each way.  The terms and the gradients into (out2, reg) must equal the
PyTorch expression train_patch.combine_terms and its autograd bit for bit:
every objective, with and without data-parallel shard weights, TV above and
below the 0.1 floor, and a NaN TV (maximum propagates it)."""
import pytest
import torch

from conftest import pkg_mod

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _reference(out2, reg, objective, weights):
    tp = pkg_mod("train_patch")
    o, r = out2.clone().requires_grad_(True), reg.clone().requires_grad_(True)
    loss, terms = tp.combine_terms(o[0], o[1], r[0], r[1], r[2], objective, weights,
                                   torch.tensor(0.1, device=DEV))
    loss.backward()
    return loss.detach(), {k: v.detach() for k, v in terms.items()}, o.grad, r.grad


@pytest.mark.parametrize("objective", ["ce", "targeted", "untargeted"])
@pytest.mark.parametrize("weights", [None, (0.375, 0.375, 0.25), (0.5, 1.0, 0.5)])
@pytest.mark.parametrize("tv", [0.0123, 0.04, 0.3, float("nan")])
def test_loss_combine_matches_autograd(objective, weights, tv):
    tp = pkg_mod("train_patch")
    out2 = torch.tensor([1.734, 2.618], device=DEV)
    reg = torch.tensor([0.81, tv, 0.057], device=DEV)
    want_loss, want, want_do, want_dr = _reference(out2, reg, objective, weights)
    o, r = out2.clone().requires_grad_(True), reg.clone().requires_grad_(True)
    loss, terms = tp.combine_terms_device(o, r, objective, weights)
    loss.backward(torch.ones((), device=DEV))
    same = lambda a, b: torch.equal(a.nan_to_num(7.0), b.nan_to_num(7.0))
    assert same(loss.detach(), want_loss)
    for k in tp.LOSS_KEYS:
        assert same(terms[k].reshape(()), want[k].reshape(())), k
    assert same(o.grad, want_do) and same(r.grad, want_dr), (o.grad, want_do, r.grad, want_dr)


def test_tv_floor_tie_is_unreachable_in_fp32():
    """maximum's tie rule (half the gradient) is kept in po_loss_combine_bwd
    for fidelity, but no fp32 TV reaches it: fl(2.5 * x) never equals 0.1f
    (the candidates x around 0.1f / 2.5 round to either side)."""
    import numpy as np
    t = np.float32(0.1)
    x = np.float32(t / np.float32(2.5))
    cands = [x]
    for direction in (np.float32(0.0), np.float32(1.0)):
        y = x
        for _ in range(8):
            y = np.nextafter(y, direction)
            cands.append(y)
    assert not any(np.float32(c * np.float32(2.5)) == t for c in cands)
