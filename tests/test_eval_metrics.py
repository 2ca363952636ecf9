"""Creation-attack metrics (utils_self drop-in; reference
test_patch_DOTA_metrics.py:301-371 over utils_self.py:166-257) against the
oracle restatement and a hand count, on label folders written the way the
evaluation writes them (utils_self.write_labels)."""
import math

from conftest import pkg_mod
from oracle import detect_ref as ref


def _folder(root, name, per_image):
    d = root / name
    d.mkdir()
    us = pkg_mod("utils_self")
    for i, boxes in enumerate(per_image):
        us.write_labels(boxes, str(d / ("img%d.txt" % i)))
    return str(d)


def test_creation_metrics_match_reference(tmp_path):
    us = pkg_mod("utils_self")
    b = lambda conf, cls: [0.5, 0.5, 0.1, 0.1, conf, 0.9, cls]
    gt001 = _folder(tmp_path, "gt001", [[b(0.5, 1), b(0.02, 3)], [b(0.7, 14)], []])
    gt04 = _folder(tmp_path, "gt04", [[b(0.5, 1)], [b(0.7, 14)], []])
    pre001 = _folder(tmp_path, "pre001", [[b(0.5, 1), b(0.02, 3), b(0.3, 14)], [b(0.7, 14), b(0.9, 14)], [b(0.05, 2)]])
    pre04 = _folder(tmp_path, "pre04", [[b(0.5, 1)], [b(0.7, 14), b(0.9, 14)], []])
    got = us.creation_metrics(pre04, gt04, pre001, gt001, 15)
    want = ref.creation_metrics(pre04, gt04, pre001, gt001, 15)
    assert got.keys() == want.keys()
    for k in got:
        assert got[k] == want[k] or (isinstance(got[k], float) and math.isclose(got[k], want[k])), k
    # by hand: 3 images; +1 instance at 0.4, +3 at 0.01
    assert got["gap_04"] == 1 and math.isclose(got["M1_04"], 1 / 3)
    assert got["gap_001"] == 3 and math.isclose(got["M1_001"], 1.0)
    assert math.isclose(got["M2_001"], (0.3 + 0.9 + 0.05) / 3)
    assert math.isclose(got["M2_04"], 0.9)
    assert got["M4"][14] == 2 and got["M4"][2] == 1 and sum(got["M4"]) == 3
    assert us.instances_per_class_cal(pre001, 15) == ref.instances_per_class_cal(pre001, 15)
    assert us.per_img_conf_sum(pre001) == ref.per_img_conf_sum(pre001)
    # the 0.4 folder as the evaluation writes it: det_conf > 0.4 only
    us.write_labels([b(0.5, 1), b(0.3, 2)], str(tmp_path / "t.txt"), thresh=0.4)
    assert open(str(tmp_path / "t.txt")).read().count("\n") == 1


def test_anchor_groups_are_reversed():
    """utils.py:441-447: head 0 gets the file's LAST group (small anchors)."""
    ut = pkg_mod("utils")
    a = ut.get_anchors(None)
    assert a.shape == (3, 3, 2)
    assert a[0].tolist() == [[15, 31], [19, 12], [28, 40]] and a[2].tolist() == [[78, 54], [95, 102], [181, 206]]
    assert ref.get_anchors_text(ut.BUILTIN_ANCHORS).tolist() == a.tolist()
    assert ut.load_class_names("builtin:dota")[14] == "helicopter"
