"""TEST INFRASTRUCTURE — CPU restatement of the reference's patch-evaluation
chain: get_anchors, get_region_boxes, bbox_iou, nms,
do_detect's post-processing (reference utils.py:27-57, 93-112, 125-245,
441-519) and the creation-attack metrics M1/M2/M4
(test_patch_DOTA_metrics.py:301-371 over utils_self.py:166-257).

Same PyTorch-CPU fp32 ops in the reference's order; the `.cuda()` calls are
dropped.  Two choices the reference leaves to the implementation are pinned:
NMS orders equal keys (1 - det_conf, fp32) by candidate index (stable sort),
and get_region_boxes enumerates candidates b -> cy -> cx -> anchor (its loop
order, utils.py:211-216).  Only tests/ import this module.
"""
import math
import os

import numpy as np
import torch


def get_anchors_text(text):
    """utils.py:441-447: the groups of the anchors file in REVERSED order
    (`[::-1]`).  With data/yolov3_anchors.txt (large, medium, small groups)
    head 0 (19x19, cfg mask 6,7,8) is decoded with the small anchors — a
    reference quirk reproduced as is."""
    anchors = [float(x) for x in text.split(",")]
    return np.array(anchors).reshape([-1, 3, 2])[::-1, :, :]


def bbox_iou(box1, box2, x1y1x2y2=True):                               # utils.py:27-57
    if x1y1x2y2:
        mx = min(box1[0], box2[0])
        Mx = max(box1[2], box2[2])
        my = min(box1[1], box2[1])
        My = max(box1[3], box2[3])
        w1 = box1[2] - box1[0]
        h1 = box1[3] - box1[1]
        w2 = box2[2] - box2[0]
        h2 = box2[3] - box2[1]
    else:
        mx = min(box1[0] - box1[2] / 2.0, box2[0] - box2[2] / 2.0)
        Mx = max(box1[0] + box1[2] / 2.0, box2[0] + box2[2] / 2.0)
        my = min(box1[1] - box1[3] / 2.0, box2[1] - box2[3] / 2.0)
        My = max(box1[1] + box1[3] / 2.0, box2[1] + box2[3] / 2.0)
        w1 = box1[2]
        h1 = box1[3]
        w2 = box2[2]
        h2 = box2[3]
    uw = Mx - mx
    uh = My - my
    cw = w1 + w2 - uw
    ch = h1 + h2 - uh
    if cw <= 0 or ch <= 0:
        return 0.0
    area1 = w1 * h1
    area2 = w2 * h2
    carea = cw * ch
    uarea = area1 + area2 - carea
    return carea / uarea


def nms(boxes, nms_thresh):                                              # utils.py:93-112
    """Greedy NMS over boxes [x,y,w,h,det_conf,...] (0-dim fp32 tensors);
    suppressed boxes get det_conf = 0 in place, as in the reference.  The
    inner loop over j (utils.py:107-110) is evaluated as one fp32 vector
    expression per kept box: the same elementwise operations in the same
    order as bbox_iou(x1y1x2y2=False) on 0-dim tensors."""
    if len(boxes) == 0:
        return boxes
    n = len(boxes)
    det_confs = torch.zeros(n)
    for i in range(n):
        det_confs[i] = 1 - boxes[i][4]
    _, sortIds = torch.sort(det_confs, stable=True)
    sb = torch.stack([torch.stack([torch.as_tensor(boxes[k][q], dtype=torch.float32) for q in range(5)])
                      for k in sortIds.tolist()])                   # [n,5] in sorted order
    alive = sb[:, 4].clone()
    out_boxes = []
    for i in range(n):
        if alive[i] > 0:
            out_boxes.append(boxes[sortIds[i]])
            b1, b2 = sb[i], sb[i + 1:]
            mx = torch.minimum(b1[0] - b1[2] / 2.0, b2[:, 0] - b2[:, 2] / 2.0)
            Mx = torch.maximum(b1[0] + b1[2] / 2.0, b2[:, 0] + b2[:, 2] / 2.0)
            my = torch.minimum(b1[1] - b1[3] / 2.0, b2[:, 1] - b2[:, 3] / 2.0)
            My = torch.maximum(b1[1] + b1[3] / 2.0, b2[:, 1] + b2[:, 3] / 2.0)
            cw = b1[2] + b2[:, 2] - (Mx - mx)
            ch = b1[3] + b2[:, 3] - (My - my)
            carea = cw * ch
            iou = carea / (b1[2] * b1[3] + b2[:, 2] * b2[:, 3] - carea)
            hit = (cw > 0) & (ch > 0) & (iou > nms_thresh)
            alive[i + 1:][hit] = 0
    for s_, k in enumerate(sortIds.tolist()):
        if alive[s_] == 0 and not (float(boxes[k][4]) == 0):
            boxes[k][4] = 0
    return out_boxes


def get_region_boxes(output, conf_thresh, num_classes, anchors, num_anchors, img_size, only_objectness=0,
                     validation=False):
    """utils.py:125-245: boxes [cx, cy, w, h, det_conf, cls_max_conf,
    cls_max_id] in input pixels, per image; validation (utils.py:221-226):
    after the test-side 8th element, (cls_conf, c) for every other class with
    det_conf * cls_conf > conf_thresh."""
    all_boxes = []
    if output.dim() == 3:
        output = output.unsqueeze(0)
    batch = output.size(0)
    assert output.size(1) == (5 + num_classes) * num_anchors
    h, w = output.size(2), output.size(3)
    stride_h = img_size[1] / h
    stride_w = img_size[0] / w
    scaled_anchors = [(aw / stride_w, ah / stride_h) for aw, ah in anchors]
    output = output.view(batch * num_anchors, 5 + num_classes, h * w)
    output = output.transpose(0, 1).contiguous()
    output = output.view(5 + num_classes, batch * num_anchors * h * w)
    grid_x = torch.linspace(0, w - 1, w).repeat(h, 1).repeat(batch * num_anchors, 1, 1).view(batch * num_anchors * h * w)
    grid_y = torch.linspace(0, h - 1, h).repeat(w, 1).t().repeat(batch * num_anchors, 1, 1).view(
        batch * num_anchors * h * w)
    xs = torch.sigmoid(output[0]) + grid_x
    ys = torch.sigmoid(output[1]) + grid_y
    anchor_w = torch.Tensor(scaled_anchors).index_select(1, torch.LongTensor([0]))
    anchor_h = torch.Tensor(scaled_anchors).index_select(1, torch.LongTensor([1]))
    anchor_w = anchor_w.repeat(batch, 1).repeat(1, 1, h * w).view(batch * num_anchors * h * w)
    anchor_h = anchor_h.repeat(batch, 1).repeat(1, 1, h * w).view(batch * num_anchors * h * w)
    ws = torch.exp(output[2]) * anchor_w
    hs = torch.exp(output[3]) * anchor_h
    xs = xs * stride_w
    ys = ys * stride_h
    ws = ws * stride_w
    hs = hs * stride_h
    det_confs = torch.sigmoid(output[4])
    cls_confs = torch.sigmoid(output[5:].transpose(0, 1))
    cls_max_confs, cls_max_ids = torch.max(cls_confs, 1)
    sz_hw = h * w
    sz_hwa = sz_hw * num_anchors
    for b in range(batch):
        boxes = []
        for cy in range(h):
            for cx in range(w):
                for i in range(num_anchors):
                    ind = b * sz_hwa + i * sz_hw + cy * w + cx
                    det_conf = det_confs[ind]
                    conf = det_confs[ind] if only_objectness else det_confs[ind] * cls_max_confs[ind]
                    if conf > conf_thresh:
                        # 8th element (test-side only): the class ids whose probability is within
                        # 1e-6 relative of the max -- the device's and the CPU's sigmoid may
                        # order such near-ties differently by an ulp
                        near = set(torch.nonzero(cls_confs[ind] >= cls_max_confs[ind] * (1 - 1e-6)).view(-1).tolist())
                        box = [xs[ind], ys[ind], ws[ind], hs[ind], det_conf, cls_max_confs[ind],
                               cls_max_ids[ind], near]
                        if (not only_objectness) and validation:                     # utils.py:221-226
                            for c in range(num_classes):
                                tmp_conf = cls_confs[ind][c]
                                if c != cls_max_ids[ind] and det_confs[ind] * tmp_conf > conf_thresh:
                                    box.append(tmp_conf)
                                    box.append(c)
                        boxes.append(box)
        all_boxes.append(boxes)
    return all_boxes


def detect_postprocess(outputs, width, height, anchors, num_classes, conf_thresh, nms_thresh):
    """do_detect after the forward (utils.py:495-519) for ONE image: decode
    every head (head i with anchors[i] of the reversed groups, num_anchors =
    len(anchors)), normalise by the image size, concatenate in head order, NMS."""
    num_anchors = len(anchors)
    boxes_list = []
    for i in range(len(anchors)):
        boxes_list.append(get_region_boxes(outputs[i], conf_thresh, num_classes, anchors[i], num_anchors,
                                           (width, height))[0])
    all_boxes = []
    for box in boxes_list:
        for i in range(len(box)):
            box[i][0] = box[i][0] / width
            box[i][2] = box[i][2] / width
            box[i][1] = box[i][1] / height
            box[i][3] = box[i][3] / height
            all_boxes.append(box[i])
    return nms(all_boxes, nms_thresh)


# ---------------------------------------------------------------------------
# creation-attack metrics (utils_self.py:166-196, 230-257;
# test_patch_DOTA_metrics.py:301-371)
# ---------------------------------------------------------------------------
def txt_len_read(txtfile_list):
    len_txt, acc = 0, []
    for name in os.listdir(txtfile_list):
        path = os.path.abspath(os.path.join(txtfile_list, name))
        if os.path.getsize(path):
            with open(path) as f:
                n = len(f.readlines())
            len_txt += n
            acc.append(n)
    return len_txt, acc


def per_img_conf_sum(labels):
    s = 0.0
    for name in os.listdir(labels):
        if name.endswith(".txt"):
            path = os.path.abspath(os.path.join(labels, name))
            if os.path.getsize(path):
                with open(path) as f:
                    for item in f.readlines():
                        s += float(item.rsplit()[4])
    return s


def instances_per_class_cal(labels_dir, num_class):
    ids = []
    for name in os.listdir(labels_dir):
        if name.endswith(".txt"):
            path = os.path.abspath(os.path.join(labels_dir, name))
            if os.path.getsize(path):
                with open(path) as f:
                    for item in f.readlines():
                        ids.append(int(item.rsplit()[-1]))
    return [ids.count(i) for i in range(num_class)]


def creation_metrics(pre_04, gt_04, pre_001, gt_001, num_class=15):
    """test_patch_DOTA_metrics.py:301-371."""
    m4 = (torch.tensor(instances_per_class_cal(pre_001, num_class))
          - torch.tensor(instances_per_class_cal(gt_001, num_class)))
    n_gt = len([f for f in os.listdir(gt_04) if f.endswith(".txt")])
    gap_04 = txt_len_read(pre_04)[0] - txt_len_read(gt_04)[0]
    gap_001 = txt_len_read(pre_001)[0] - txt_len_read(gt_001)[0]
    m2_001 = (per_img_conf_sum(pre_001) - per_img_conf_sum(gt_001)) / gap_001 if gap_001 else math.nan
    m2_04 = (per_img_conf_sum(pre_04) - per_img_conf_sum(gt_04)) / gap_04 if gap_04 else math.nan
    return {"M1_04": gap_04 / n_gt, "M1_001": gap_001 / n_gt, "M2_001": m2_001, "M2_04": m2_04,
            "M4": m4.tolist(), "gap_04": gap_04, "gap_001": gap_001}
