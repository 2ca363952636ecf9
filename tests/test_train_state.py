"""save_train_state / load_train_state (train_patch.py): the optional fp32
training checkpoint beside the PNG.  CPU: the file loads with
torch.load(weights_only=True), and an Adam(amsgrad) + ReduceLROnPlateau pair
restored from it continues exactly as the original."""
import pytest
import torch

from conftest import pkg_mod


def _opt(p):
    o = torch.optim.Adam([p], lr=0.03, amsgrad=True)
    return o, torch.optim.lr_scheduler.ReduceLROnPlateau(o, "min", patience=1)


def _steps(p, o, s, grads, losses):
    for g, l in zip(grads, losses):
        p.grad = g.clone()
        o.step()
        o.zero_grad()
        with torch.no_grad():
            p.clamp_(0, 1)
        s.step(l)


def test_state_roundtrip_continues_identically(tmp_path):
    tp = pkg_mod("train_patch")
    gen = torch.Generator().manual_seed(3)
    grads = [torch.randn(3, 8, 8, generator=gen) for _ in range(8)]
    losses = [5.0, 4.0, 4.5, 4.6, 4.7, 3.0, 3.1, 3.2]
    p = torch.rand(3, 8, 8, generator=gen).requires_grad_(True)
    o, s = _opt(p)
    _steps(p, o, s, grads[:4], losses[:4])
    path = str(tmp_path / "4_state.pt")
    tp.save_train_state(path, p, o, s, epoch=4, step=40, ep_losses=[0.5, 0.25])
    st = torch.load(path, map_location="cpu", weights_only=True)      # no pickled objects
    assert st["epoch"] == 4 and st["step"] == 40 and st["ep_losses"] == [0.5, 0.25]
    _steps(p, o, s, grads[4:], losses[4:])

    st = tp.load_train_state(path)
    q = st["patch"].clone().requires_grad_(True)
    o2, s2 = _opt(q)
    o2.load_state_dict(st["optimizer"])
    s2.load_state_dict(st["scheduler"])
    _steps(q, o2, s2, grads[4:], losses[4:])
    assert torch.equal(p.detach(), q.detach())
    assert o.param_groups[0]["lr"] == o2.param_groups[0]["lr"] < 0.03      # the plateau cut the LR in both


def test_load_refuses_foreign_files(tmp_path):
    tp = pkg_mod("train_patch")
    path = str(tmp_path / "x.pt")
    torch.save({"patch": torch.zeros(3)}, path)
    with pytest.raises(ValueError):
        tp.load_train_state(path)
