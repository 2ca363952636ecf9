"""Creation-attack evaluation metrics — drop-in for the helpers of reference
``utils_self.py`` that test_patch_DOTA_metrics.py uses, plus that script's
metric block as one function.

* txt_len_read            utils_self.py:166-178  lines over a label folder
* per_img_conf_sum        utils_self.py:180-196  sum of objectness (column 5)
* instances_per_class_cal utils_self.py:230-257  instances per class id (last column)
* patch_MSE_calsulator    utils_self.py:205-220  MSE of two saved patches
* load_image_file         utils_self.py:151-166  PIL open + EXIF transpose + RGB
* creation_metrics        test_patch_DOTA_metrics.py:301-371: M1 (instances
  created per image at conf 0.4 and 0.01), M2 (objectness created per new
  instance), M4 (instance gap per class)

Label files are the evaluation's ``cx cy w h det_conf cls_conf cls_id`` lines
(utils.do_detect boxes).  Host code: text parsing, no device work.
"""
import math
import os

from .eval_patch import load_image_file  # noqa: F401  (utils_self.load_image_file)
from .train_patch import patch_mse


def txt_len_read(txtfile_list):
    """(total lines, per-file line counts of non-empty files) of a label folder."""
    len_txt, counts = 0, []
    for name in os.listdir(txtfile_list):
        path = os.path.abspath(os.path.join(txtfile_list, name))
        if os.path.getsize(path):
            with open(path) as f:
                n = len(f.readlines())
            len_txt += n
            counts.append(n)
    return len_txt, counts


def per_img_conf_sum(labels):
    """Sum of the objectness column (index 4) over every label line."""
    total = 0.0
    for name in os.listdir(labels):
        if name.endswith(".txt"):
            path = os.path.abspath(os.path.join(labels, name))
            if os.path.getsize(path):
                with open(path) as f:
                    for item in f.readlines():
                        total += float(item.rsplit()[4])
    return total


def instances_per_class_cal(labels_dir, num_class):
    """Instances per class id (the last column) over a label folder."""
    ids = []
    for name in os.listdir(labels_dir):
        if name.endswith(".txt"):
            path = os.path.abspath(os.path.join(labels_dir, name))
            if os.path.getsize(path):
                with open(path) as f:
                    ids.extend(int(item.rsplit()[-1]) for item in f.readlines())
    return [ids.count(i) for i in range(num_class)]


def patch_MSE_calsulator(patchfile_0, patchfile_1):
    """MSE of two saved patches (reference name kept)."""
    return patch_mse(patchfile_0, patchfile_1)


def write_labels(boxes, path, thresh=None):
    """The evaluation's label file of one image: one ``cx cy w h det_conf
    cls_conf cls_id`` line per box (test_patch_DOTA_metrics.py:196-204);
    ``thresh``: keep only boxes with det_conf > thresh (the 0.4 folder)."""
    with open(path, "w") as f:
        for b in boxes:
            if thresh is None or b[4] > thresh:
                f.write(f"{b[0]} {b[1]} {b[2]} {b[3]} {b[4]} {b[5]} {b[6]}\n")


def creation_metrics(pre_04, gt_04, pre_001, gt_001, num_class=15):
    """test_patch_DOTA_metrics.py:301-371 over four label folders (patched
    predictions and clean ground truth, at conf 0.4 and 0.01).  M2 is NaN
    where no instance was created (the reference divides by zero there)."""
    gt_ids = instances_per_class_cal(gt_001, num_class)
    pre_ids = instances_per_class_cal(pre_001, num_class)
    n_gt = len([f for f in os.listdir(gt_04) if f.endswith(".txt")])
    gap_04 = txt_len_read(pre_04)[0] - txt_len_read(gt_04)[0]
    gap_001 = txt_len_read(pre_001)[0] - txt_len_read(gt_001)[0]
    m2_001 = (per_img_conf_sum(pre_001) - per_img_conf_sum(gt_001)) / gap_001 if gap_001 else math.nan
    m2_04 = (per_img_conf_sum(pre_04) - per_img_conf_sum(gt_04)) / gap_04 if gap_04 else math.nan
    return {"M1_04": gap_04 / n_gt, "M1_001": gap_001 / n_gt, "M2_001": m2_001, "M2_04": m2_04,
            "M4": [p - g for p, g in zip(pre_ids, gt_ids)], "gap_04": gap_04, "gap_001": gap_001}
