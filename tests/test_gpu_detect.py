"""GPU parity of the patch-evaluation chain against the
oracle restatement oracle/detect_ref.py (reference utils.py:27-57, 93-112,
125-245, 441-519): head decode + threshold (po_region_boxes), NMS (po_nms)
and do_detect's composition with the reversed anchor groups.

Decisions are compared exactly (which candidates pass, their order, which
boxes NMS keeps); box values to fp32 ulps (the device's expf/sigmoid and the
CPU's differ in the last bit).  Inputs keep the decision margins away from
rounding ties: head logits are drawn so no confidence sits within 1e-5 of
the threshold."""
import numpy as np
import pytest
import torch

from oracle import detect_ref as ref
from conftest import pkg_mod

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _heads(B, hws, C=15, A=3, seed=0, bias=-2.0):
    g = torch.Generator().manual_seed(seed)
    return [torch.randn(B, A * (5 + C), h, h, generator=g) * 1.5 + bias for h in hws]


def _assert_boxes_equal(got, want, rtol=1e-5, sat_ties=False):
    """``sat_ties``: a class id may differ where the winning class
    probability is tied to within 1e-6 relative with the device's id (the
    oracle's 8th box element; saturated sigmoids tie exactly): the first
    index wins and the device's and CPU's last sigmoid bit decide."""
    assert len(got) == len(want), (len(got), len(want))
    for a, b in zip(got, want):
        bv = [float(v) for v in b[:7]]
        if int(a[6]) != int(bv[6]):
            assert sat_ties and int(a[6]) in b[7], (a, bv, b[7])
        np.testing.assert_allclose(np.asarray(a[:6], dtype=np.float64), np.asarray(bv[:6]), rtol=rtol, atol=1e-7)


def _away_from(x, thresh, eps=1e-5):
    return (x - thresh).abs() > eps


@pytest.mark.parametrize("h,thresh,only_obj", [(19, 0.01, 0), (38, 0.4, 0), (13, 0.2, 1)])
def test_region_boxes_match_oracle(h, thresh, only_obj):
    ut = pkg_mod("utils")
    out = _heads(2, [h], seed=h)[0]
    anchors = ut.get_anchors(None)[0]
    # keep every confidence clear of the threshold (ties could go either way)
    o = out.view(2, 3, 20, h * h)
    det = torch.sigmoid(o[:, :, 4])
    conf = det if only_obj else det * torch.sigmoid(o[:, :, 5:]).max(2).values
    o[:, :, 4] = torch.where(_away_from(conf, thresh), o[:, :, 4], o[:, :, 4] - 0.5)
    want = ref.get_region_boxes(out, thresh, 15, anchors, 3, (608, 608), only_objectness=only_obj)
    got = ut.get_region_boxes(out.to(DEV), thresh, 15, anchors, 3, (608, 608), only_objectness=only_obj)
    for b in range(2):
        assert len(want[b]) > 0
        _assert_boxes_equal(got[b], want[b])


@pytest.mark.parametrize("h,thresh", [(13, 0.05), (19, 0.02)])
def test_region_boxes_validation_matches_oracle(h, thresh):
    """get_region_boxes(validation=True) (utils.py:221-226): after the seven
    box fields, (cls_conf, c) for every other class whose det_conf * cls_conf
    clears the threshold, in class order; every product kept clear of the
    threshold so the comparison cannot flip by an ulp."""
    ut = pkg_mod("utils")
    out = _heads(2, [h], seed=100 + h)[0]
    anchors = ut.get_anchors(None)[0]
    o = out.view(2, 3, 20, h * h)
    for _ in range(4):                         # push every det * p and det * max p away from the threshold
        det = torch.sigmoid(o[:, :, 4:5])
        p = torch.sigmoid(o[:, :, 5:])
        near = (~_away_from(det * p, thresh, 1e-4)).any(2, keepdim=True)
        o[:, :, 4:5] = torch.where(near, o[:, :, 4:5] - 0.37, o[:, :, 4:5])
    want = ref.get_region_boxes(out, thresh, 15, anchors, 3, (608, 608), validation=True)
    got = ut.get_region_boxes(out.to(DEV), thresh, 15, anchors, 3, (608, 608), validation=True)
    extras = 0
    for b in range(2):
        assert len(got[b]) == len(want[b]) > 0
        _assert_boxes_equal([g[:7] for g in got[b]], [w_[:8] for w_ in want[b]])
        for g, w_ in zip(got[b], want[b]):
            ge, we = g[7:], w_[8:]
            assert len(ge) == len(we), (ge, we)
            assert [int(c) for c in ge[1::2]] == [int(c) for c in we[1::2]]
            for a_, r_ in zip(ge[0::2], we[0::2]):
                assert abs(a_ - float(r_)) <= 1e-6
            extras += len(ge) // 2
    assert extras > 0


@pytest.mark.parametrize("n,thresh", [(1, 0.4), (300, 0.4), (1000, 0.45)])
def test_nms_matches_oracle(n, thresh):
    """Random boxes in clusters (many overlaps), with duplicate confidences
    (the stable tie rule): identical kept lists, in order, and the reference's
    in-place det_conf = 0 of the suppressed boxes."""
    ut = pkg_mod("utils")
    g = torch.Generator().manual_seed(n)
    centers = torch.rand(max(1, n // 20), 2, generator=g)
    idx = torch.randint(0, centers.size(0), (n,), generator=g)
    xy = centers[idx] + torch.randn(n, 2, generator=g) * 0.02
    wh = torch.rand(n, 2, generator=g) * 0.1 + 0.02
    conf = (torch.rand(n, generator=g) * 100).floor() / 100 + 0.005           # many equal confidences
    cls = torch.randint(0, 15, (n,), generator=g)
    rows = torch.cat([xy, wh, conf[:, None], torch.rand(n, 1, generator=g), cls[:, None].float()], 1)
    boxes_ref = [[r[i].clone() for i in range(6)] + [int(r[6])] for r in rows]
    want = ref.nms(boxes_ref, thresh)
    boxes = [[float(v) for v in r[:6]] + [int(r[6])] for r in rows]
    got = ut.nms(boxes, thresh)
    pos, pos_ref = {id(b): i for i, b in enumerate(boxes)}, {id(b): i for i, b in enumerate(boxes_ref)}
    assert [pos[id(b)] for b in got] == [pos_ref[id(b)] for b in want]      # same boxes kept, same order
    _assert_boxes_equal(got, want, rtol=0)
    # side effect: suppressed boxes carry det_conf 0, as in the reference
    assert [float(b[4]) for b in boxes] == [float(b[4]) for b in boxes_ref]


def test_do_detect_composition_matches_oracle():
    """detect_batch's decode/NMS of three heads with the reversed anchor
    groups and the image-size normalisation, against do_detect's post-process
    (utils.py:495-519) on the same head tensors."""
    ut = pkg_mod("utils")
    heads = _heads(2, [19, 38, 76], seed=3, bias=-5.5)
    anchors = ut.get_anchors(None)
    assert np.array_equal(anchors[0], np.array([[15, 31], [19, 12], [28, 40]], dtype=np.float64))   # reversed groups
    det = ut.Detections(2, sum(3 * h.size(2) * h.size(3) for h in heads), DEV)
    for i, h in enumerate(heads):
        ut.region_boxes_device(h.to(DEV), 0.05, 15, anchors[i], 3, (608, 608), norm=(608, 608), det=det)
    keep, nkeep = ut.nms_device(det, 0.4)
    got = ut._box_lists(det.boxes.cpu().numpy(), det.counts.cpu().numpy(), keep.cpu().numpy(), nkeep.cpu().numpy())
    for b in range(2):
        want = ref.detect_postprocess([h[b:b + 1] for h in heads], 608, 608, anchors, 15, 0.05, 0.4)
        assert len(want) > 0
        _assert_boxes_equal(got[b], want)


def test_detect_batch_end_to_end(tmp_path):
    """The HIP Darknet forward feeding detect_batch on a synthetic frame:
    the same boxes as the oracle post-process of those HIP heads, and the
    label-file round trip the metrics read."""
    ut, us, dk, W, sy = (pkg_mod(m) for m in ("utils", "utils_self", "darknet_v3", "weights", "synthetic"))
    path = str(tmp_path / "w.weights")
    W.write_weights(path, W.synthesize("builtin:yolov3-dota", seed=4))
    net = dk.Darknet("builtin:yolov3-dota")
    net.load_darknet_weights(path)
    img = sy.frames(1, 608, seed=9).to(DEV)
    boxes = ut.detect_batch(net, img, 0.4, 0.4)[0]
    heads = [h.cpu() for h in net.forward(img)]
    want = ref.detect_postprocess(heads, 608, 608, ut.get_anchors(None), 15, 0.4, 0.4)
    assert len(boxes) == len(want)
    _assert_boxes_equal(boxes, want, sat_ties=True)
    (tmp_path / "labels").mkdir()
    us.write_labels(boxes, str(tmp_path / "labels" / "a.txt"))
    assert us.txt_len_read(str(tmp_path / "labels"))[0] == len(boxes)
