"""MaxProbExtractor (reference load_data.py:125-311, R23) on the HIP path
(po_max_prob / po_max_prob_bwd) against the oracle restatement
(oracle.max_prob_extractor, which runs the reference's bbox_decode, transposes
and concatenation).  The maxima and their flat output_cat indices are
selections: bit-exact.  The gradient lands on the selected logit only."""
import pytest
import torch

import oracle
from conftest import pkg_mod

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)
ANCHORS = [[(181, 206), (95, 102), (78, 54)], [(42, 87), (43, 38), (40, 20)], [(28, 40), (19, 12), (15, 31)]]


def _heads(B, sides, seed, C=60):
    gen = torch.Generator().manual_seed(seed)
    return [torch.randn(B, C, s, s, generator=gen) * 3 for s in sides]


@pytest.mark.parametrize("sigmoid_mode", [False, True])
@pytest.mark.parametrize("cls_id", [0, 14])
def test_max_prob_matches_oracle(sigmoid_mode, cls_id):
    ld = pkg_mod("load_data")
    B = 3
    heads = _heads(B, (19, 38, 76), seed=cls_id + 7)
    ref_obj, ref_cls, ref_oi, ref_ci = oracle.max_prob_extractor(heads, cls_id, 15, ANCHORS, sigmoid_mode)
    ext = ld.MaxProbExtractor(cls_id, 15, None)
    hd = [h.to(DEV).requires_grad_(True) for h in heads]
    mo, mc = ext(hd, sigmoid_mode=sigmoid_mode)
    # raw logits are selected bit-exactly; sigmoid values may differ by an ulp
    # of expf between the HIP and ATen CPU implementations
    tol = dict(rtol=2e-7, atol=0) if sigmoid_mode else dict(rtol=0, atol=0)
    torch.testing.assert_close(mo.detach().cpu(), ref_obj, **tol)
    torch.testing.assert_close(mc.detach().cpu(), ref_cls, **tol)
    assert ext.last_index[0].cpu().long().tolist() == ref_oi.tolist()
    assert ext.last_index[1].cpu().long().tolist() == ref_ci.tolist()
    # gradient: exactly the oracle's autograd through the reference ops
    go, gc = torch.randn(B), torch.randn(B)
    (mo * go.to(DEV) + mc * gc.to(DEV)).sum().backward()
    hr = [h.clone().requires_grad_(True) for h in heads]
    ro, rc, _, _ = oracle.max_prob_extractor(hr, cls_id, 15, ANCHORS, sigmoid_mode)
    (ro * go + rc * gc).sum().backward()
    for a, b in zip(hd, hr):
        torch.testing.assert_close(a.grad.cpu(), b.grad, rtol=1e-6, atol=1e-7)


def test_max_prob_ties_take_the_first_index():
    """All-equal logits: torch.max's first index (head 0, anchor 0, cell 0)."""
    ld = pkg_mod("load_data")
    heads = [torch.zeros(2, 60, s, s, device=DEV) for s in (13, 26)]
    ext = ld.MaxProbExtractor(5, 15)
    mo, mc = ext(heads)
    assert mo.tolist() == [0.0, 0.0] and mc.tolist() == [0.0, 0.0]
    assert ext.last_index.cpu().tolist() == [[0, 0], [0, 0]]
    # a later equal value does not win; a larger one does
    heads[1][1, 4 + 20, 3, 5] = 1.0
    mo, _ = ext(heads)
    assert mo.tolist() == [0.0, 1.0]
    assert int(ext.last_index[0, 1]) == 3 * 13 * 13 + 1 * 26 * 26 + 3 * 26 + 5


def test_max_prob_on_nhwc_head_buffers():
    """The training plan's NHWC head buffers (channel stride Cp), viewed as
    NCHW, give the same maxima as the contiguous NCHW heads."""
    ld = pkg_mod("load_data")
    heads = _heads(2, (19, 38), seed=3)
    nhwc = []
    for h in heads:
        buf = torch.zeros(h.size(0), h.size(2), h.size(3), 64)
        buf[..., :60] = h.permute(0, 2, 3, 1)
        nhwc.append(buf.to(DEV).permute(0, 3, 1, 2))
    ext = ld.MaxProbExtractor(14, 15)
    a = ext([h.to(DEV) for h in heads], sigmoid_mode=True)
    ia = ext.last_index.clone()
    b = ext(nhwc, sigmoid_mode=True)
    assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1]) and torch.equal(ia, ext.last_index)
