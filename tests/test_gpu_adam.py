"""PatchAdam (po_adam_amsgrad): Adam(amsgrad) + clamp in one HIP launch
(train_patch.py:131-136, 327-330).  Checked against torch.optim.Adam(amsgrad)
on the CPU -- the reference's own optimizer, single-tensor arithmetic -- step
by step with the learning rate changed mid-run (as ReduceLROnPlateau does):
parameters and all three moment tensors within 2 fp32 ulps of the larger of
1 and the tensor's magnitude (ATen's CPU kernels contract some of the
multiply-adds differently from the written order: measured 1 ulp, printed);
the skipped update under found_inf / the flag bit; the state_dict moving both
ways."""
import pytest
import torch

from conftest import pkg_mod

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)
KEYS = ("exp_avg", "exp_avg_sq", "max_exp_avg_sq")


def _grads(n, shape, seed):
    g = torch.Generator().manual_seed(seed)
    out = []
    for k in range(n):
        x = torch.randn(shape, generator=g) * (10.0 ** (k % 3 - 2))
        x[0, 0, :3] = torch.tensor([0.0, -0.0, 1e-30])          # zero and tiny gradients
        out.append(x)
    return out


TOL = 2 * 2.0 ** -23          # 2 fp32 ulps at 1


def _rel(x, ref):
    return float((x - ref).abs().max()) / max(1.0, float(ref.abs().max()))


def _cpu_step(p, o, g):
    p.grad = g.clone()
    o.step()
    o.zero_grad()
    with torch.no_grad():
        p.clamp_(0, 1)


@pytest.mark.parametrize("shape", [(3, 224, 224), (3, 7, 5)])
def test_patch_adam_matches_torch_adam(shape):
    tp = pkg_mod("train_patch")
    gen = torch.Generator().manual_seed(1)
    p0 = torch.rand(shape, generator=gen)
    grads = _grads(8, shape, seed=2)
    pc = p0.clone().requires_grad_(True)
    oc = torch.optim.Adam([pc], lr=0.03, amsgrad=True)
    pg = p0.clone().to(DEV).requires_grad_(True)
    og = tp.PatchAdam([pg], lr=0.03)
    worst = 0.0
    for k, g in enumerate(grads):
        if k == 5:                                              # a plateau cut of the learning rate
            for o in (oc, og):
                o.param_groups[0]["lr"] = 0.003
        _cpu_step(pc, oc, g)
        pg.grad = g.to(DEV)
        og.step()
        og.zero_grad()
        assert pg.grad is None
        d = _rel(pg.detach().cpu(), pc.detach())
        for key in KEYS:
            d = max(d, _rel(og.state[pg][key].cpu(), oc.state[pc][key]))
        worst = max(worst, d)
        assert float(og.state[pg]["step"]) == float(oc.state[pc]["step"]) == k + 1
    print("PatchAdam vs torch Adam(amsgrad) over 8 steps: max |diff| / max(1, |ref|) %.3g" % worst)
    assert worst <= TOL
    assert bool(((pg.detach() >= 0) & (pg.detach() <= 1)).all())


def test_patch_adam_skips_on_found_inf_and_flag():
    tp = pkg_mod("train_patch")
    p = torch.rand(3, 16, 16, device=DEV).requires_grad_(True)
    o = tp.PatchAdam([p], lr=0.03)
    p.grad = torch.randn_like(p)
    o.step()
    before = {k: o.state[p][k].clone() for k in KEYS}
    pb = p.detach().clone()
    o.found_inf = torch.ones((), device=DEV)
    p.grad = torch.randn_like(p)
    o.step()
    assert torch.equal(p.detach(), pb) and float(o.state[p]["step"]) == 1.0
    assert all(torch.equal(o.state[p][k], before[k]) for k in KEYS)
    o.found_inf = None
    flags = torch.full((1,), tp.FLAG_NONFINITE, dtype=torch.int32, device=DEV)
    o.skip_flags = (flags, tp.FLAG_NONFINITE)
    o.step()
    assert torch.equal(p.detach(), pb) and float(o.state[p]["step"]) == 1.0
    flags.zero_()
    o.step()
    assert not torch.equal(p.detach(), pb) and float(o.state[p]["step"]) == 2.0


def test_patch_adam_state_dict_both_ways():
    tp = pkg_mod("train_patch")
    grads = _grads(6, (3, 8, 8), seed=5)
    p0 = torch.rand(3, 8, 8, generator=torch.Generator().manual_seed(6))
    # torch Adam (CPU) for three steps, its state into PatchAdam, three more on each
    pc = p0.clone().requires_grad_(True)
    oc = torch.optim.Adam([pc], lr=0.03, amsgrad=True)
    for g in grads[:3]:
        _cpu_step(pc, oc, g)
    pg = pc.detach().clone().to(DEV).requires_grad_(True)
    og = tp.PatchAdam([pg], lr=0.03)
    og.load_state_dict(oc.state_dict())
    assert og.state[pg]["step"].device == pg.device
    for g in grads[3:]:
        _cpu_step(pc, oc, g)
        pg.grad = g.to(DEV)
        og.step()
    assert _rel(pg.detach().cpu(), pc.detach()) <= TOL
    # and PatchAdam's state into a CPU torch Adam
    sd = og.state_dict()
    q = pg.detach().cpu().clone().requires_grad_(True)
    oq = torch.optim.Adam([q], lr=0.03, amsgrad=True)
    oq.load_state_dict({"state": {k: {kk: vv.cpu() for kk, vv in v.items()} for k, v in sd["state"].items()},
                        "param_groups": [dict(oc.state_dict()["param_groups"][0])]})
    _cpu_step(q, oq, grads[0])
    pg.grad = grads[0].to(DEV)
    og.step()
    assert _rel(pg.detach().cpu(), q.detach()) <= TOL
