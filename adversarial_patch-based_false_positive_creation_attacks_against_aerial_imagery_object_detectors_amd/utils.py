"""Patch evaluation — drop-in for the detection helpers of reference
``utils.py`` used by its evaluation scripts (test_patch_DOTA*.py), with the
decode and NMS on the MI355X (csrc/detect_ops.hip):

====================  =========================  ===============================
function              reference                  here
====================  =========================  ===============================
bbox_iou              utils.py:27-57             host (scalar helper)
nms                   utils.py:93-112            po_nms (sort, IoU bit matrix, scan)
get_region_boxes      utils.py:125-245           po_region_boxes
get_anchors           utils.py:441-447           host (reversed groups, as is)
do_detect             utils.py:450-519           Darknet forward + po_region_boxes
                                                 x heads + po_nms
load_class_names      utils.py:420-427           host
====================  =========================  ===============================

``detect_batch`` is the batched form (one forward and one decode/NMS pass for
a [B,3,S,S] batch).  Boxes are lists ``[cx, cy, w, h, det_conf, cls_max_conf,
cls_max_id]`` (python floats holding the fp32 values, id an int): formatting
them with f-strings writes the label files the reference writes (its 0-dim
tensors format as their item()).

Reference quirk kept: ``get_anchors`` returns the anchor groups of the file in
reversed order and ``do_detect`` decodes head i with group i, so with
data/yolov3_anchors.txt head 0 (19x19, cfg mask 6,7,8) uses the SMALL anchors
(SURVEY.md §8f).  ``validation=True`` of get_region_boxes (extra per-class
entries) is not on the device path and raises.
"""
import os

import numpy as np
import torch

from . import _native as nat

ANCHOR_PATH = "data/yolov3_anchors.txt"        # utils.py:14
# the reference's data/yolov3_anchors.txt (large, medium, small groups)
BUILTIN_ANCHORS = "78, 54,  95, 102,  181, 206, 40, 20,  43, 38,  42, 87, 15, 31,  19, 12,  28, 40"
# the reference's data/dota.names (TARGET_ID 14 = helicopter, train_patch.py:28)
DOTA_NAMES = ["plane", "baseball-diamond", "bridge", "ground-track-field", "small-vehicle", "large-vehicle", "ship",
              "tennis-court", "basketball-court", "storage-tank", "soccer-ball-field", "roundabout", "harbor",
              "swimming-pool", "helicopter"]
BOXF = 8                                          # floats per device box record


def load_class_names(namesfile):
    """utils.py:420-427 (``builtin:dota`` or a missing data/dota.names: the 15 DOTA classes)."""
    if namesfile in (None, "builtin:dota") or not os.path.exists(namesfile):
        return list(DOTA_NAMES)
    with open(namesfile) as fp:
        return [line.rstrip() for line in fp.readlines()]


def get_anchors(anchors_path=ANCHOR_PATH):
    """utils.py:441-447: [3 groups][3][2], groups REVERSED relative to the file."""
    path = os.path.expanduser(anchors_path) if anchors_path else ""
    if path and os.path.exists(path):
        with open(path) as f:
            text = f.readline()
    else:
        text = BUILTIN_ANCHORS
    anchors = [float(x) for x in text.split(",")]
    return np.array(anchors).reshape([-1, 3, 2])[::-1, :, :]


def bbox_iou(box1, box2, x1y1x2y2=True):
    """utils.py:27-57 (host scalar helper)."""
    if x1y1x2y2:
        mx, Mx = min(box1[0], box2[0]), max(box1[2], box2[2])
        my, My = min(box1[1], box2[1]), max(box1[3], box2[3])
        w1, h1 = box1[2] - box1[0], box1[3] - box1[1]
        w2, h2 = box2[2] - box2[0], box2[3] - box2[1]
    else:
        mx = min(box1[0] - box1[2] / 2.0, box2[0] - box2[2] / 2.0)
        Mx = max(box1[0] + box1[2] / 2.0, box2[0] + box2[2] / 2.0)
        my = min(box1[1] - box1[3] / 2.0, box2[1] - box2[3] / 2.0)
        My = max(box1[1] + box1[3] / 2.0, box2[1] + box2[3] / 2.0)
        w1, h1, w2, h2 = box1[2], box1[3], box2[2], box2[3]
    uw, uh = Mx - mx, My - my
    cw, ch = w1 + w2 - uw, h1 + h2 - uh
    if cw <= 0 or ch <= 0:
        return 0.0
    carea = cw * ch
    return carea / (w1 * h1 + w2 * h2 - carea)


# ---------------------------------------------------------------------------
# device decode + NMS
# ---------------------------------------------------------------------------
class Detections:
    """Device buffers of a decode pass: boxes [B, cap, 8], counts [B]."""

    def __init__(self, B, cap, device):
        self.B, self.cap = B, cap
        self.boxes = torch.zeros(B, cap, BOXF, device=device)
        self.counts = torch.zeros(B, dtype=torch.int32, device=device)
        self.overflow = torch.zeros(1, dtype=torch.int32, device=device)


def region_boxes_device(output, conf_thresh, num_classes, anchors, num_anchors, img_size, only_objectness=0,
                        norm=None, det=None, cap=None):
    """po_region_boxes of one head [B, A*(5+C), h, w] (CUDA, fp32) appended
    to ``det`` (a Detections; new when None).  ``norm`` = (width, height):
    do_detect's division of the box by the image size."""
    nat.ensure_device(output)
    if output.dim() == 3:
        output = output.unsqueeze(0)
    output = output.contiguous().float()
    B, Cch, h, w = output.shape
    assert Cch == (5 + num_classes) * num_anchors, "head channels %d != (5+%d)*%d" % (Cch, num_classes, num_anchors)
    if det is None:
        det = Detections(B, cap or h * w * num_anchors, output.device)
    stride_h = img_size[1] / h                    # utils.py:137-141 (python float math)
    stride_w = img_size[0] / w
    scaled = [(float(aw) / stride_w, float(ah) / stride_h) for aw, ah in anchors]
    anc = (nat.c_float * (2 * len(scaled)))(*[v for pair in scaled for v in pair])
    nw, nh = (float(norm[0]), float(norm[1])) if norm is not None else (1.0, 1.0)
    nat.call("po_region_boxes", nat.ptr(output), B, num_anchors, num_classes, h, w, anc, stride_w, stride_h, nw, nh,
             float(conf_thresh), int(bool(only_objectness)), det.cap, nat.ptr(det.boxes), nat.ptr(det.counts, torch.int32),
             nat.ptr(det.overflow, torch.int32), nat.stream())
    return det


def nms_device(det, nms_thresh):
    """po_nms over every image of ``det``: -> (keep [B, cap] int32 candidate
    indices in kept order, nkeep [B])."""
    if int(det.overflow.item()):
        raise RuntimeError("po_region_boxes: more boxes than the buffer holds (cap %d)" % det.cap)
    nmax = max(1, int(det.counts.max().item()))
    kw, mw = nat.c_int64(), nat.c_int64()
    nat.call("po_nms_workspace", det.B, nmax, nat.ctypes.byref(kw), nat.ctypes.byref(mw))
    dev = det.boxes.device
    keys = torch.empty(kw.value, dtype=torch.int64, device=dev)
    mask = torch.empty(mw.value, dtype=torch.int64, device=dev)
    keep = torch.empty(det.B, det.cap, dtype=torch.int32, device=dev)
    nkeep = torch.empty(det.B, dtype=torch.int32, device=dev)
    nat.call("po_nms", nat.ptr(det.boxes), nat.ptr(det.counts, torch.int32), det.B, det.cap, nmax, float(nms_thresh),
             nat.ptr(keys, torch.int64), nat.ptr(mask, torch.int64), nat.ptr(keep, torch.int32),
             nat.ptr(nkeep, torch.int32), nat.stream())
    return keep, nkeep


def _box_lists(boxes_cpu, counts, index=None, nkeep=None):
    out = []
    for b in range(boxes_cpu.shape[0]):
        rows = boxes_cpu[b, :counts[b]] if index is None else boxes_cpu[b, index[b, :nkeep[b]]]
        out.append([[float(r[0]), float(r[1]), float(r[2]), float(r[3]), float(r[4]), float(r[5]), int(r[6])]
                    for r in rows])
    return out


def get_region_boxes(output, conf_thresh, num_classes, anchors, num_anchors, img_size, only_objectness=0,
                     validation=False):
    """utils.py:125-245 on the device: per image, the boxes [cx, cy, w, h,
    det_conf, cls_max_conf, cls_max_id] (input pixels) whose confidence
    exceeds conf_thresh, in the reference's order (cy, cx, anchor).
    validation=True (and not only_objectness, utils.py:221-226): each box also
    lists (cls_conf, c) for every other class c with det_conf * cls_conf >
    conf_thresh, in class order -- read at the record's head element
    (po_region_boxes' src field), fp32 products and comparison as torch's."""
    det = region_boxes_device(output, conf_thresh, num_classes, anchors, num_anchors, img_size, only_objectness)
    if int(det.overflow.item()):
        raise RuntimeError("po_region_boxes: buffer overflow")
    boxes_cpu, counts = det.boxes.cpu().numpy(), det.counts.cpu().numpy()
    lists = _box_lists(boxes_cpu, counts)
    if validation and not only_objectness:
        out = output.unsqueeze(0) if output.dim() == 3 else output
        B, _, h, w = out.shape
        raw = out.contiguous().float().view(B, num_anchors, 5 + num_classes, h * w)
        for b in range(B):
            n = int(counts[b])
            if n == 0:
                continue
            src = torch.from_numpy(boxes_cpu[b, :n, 7].copy()).view(torch.int32).long().to(out.device)
            a_i, cell = src // (h * w), src % (h * w)
            # det_conf and the class probabilities with torch.sigmoid on the device
            # tensor, as the reference computes both (utils.py:180-187), so the
            # product and its comparison are the reference's bit for bit
            detc = torch.sigmoid(raw[b][a_i, 4, cell]).view(n, 1)
            cc = torch.sigmoid(raw[b][a_i, 5:, cell])                    # [n, C]
            over = (detc * cc) > conf_thresh                             # utils.py:224 (fp32)
            over[torch.arange(n, device=out.device), det.boxes[b, :n, 6].long()] = False
            rc = torch.nonzero(over).cpu().tolist()                      # (box, class) in row-major order
            vals = cc[over].cpu().tolist()
            for (r, c), v in zip(rc, vals):
                lists[b][r] += [v, c]
    return lists


def nms(boxes, nms_thresh):
    """utils.py:93-112 on the device: greedy NMS of a list of boxes (by
    det_conf, ties in list order); returns the kept boxes in kept order and,
    as the reference does, sets det_conf of the suppressed ones to 0."""
    if len(boxes) == 0:
        return boxes
    dev = torch.device("cuda", torch.cuda.current_device())
    det = Detections(1, len(boxes), dev)
    rows = torch.zeros(len(boxes), BOXF)
    rows[:, :7] = torch.tensor([[float(v) for v in b[:7]] for b in boxes])
    det.boxes[0].copy_(rows)
    det.counts.fill_(len(boxes))
    keep, nkeep = nms_device(det, nms_thresh)
    kept = keep[0, :int(nkeep[0])].cpu().tolist()
    ks = set(kept)
    for i, b in enumerate(boxes):                 # utils.py:109: suppressed boxes get det_conf 0
        if i not in ks and float(b[4]) > 0:
            b[4] = 0
    return [boxes[i] for i in kept]


def detect_batch(model, imgs, conf_thresh, nms_thresh, anchors=None, num_classes=15):
    """do_detect for a [B,3,S,S] batch (CUDA, values in [0,1]): one HIP
    forward, the heads decoded with the (reversed) anchor groups, boxes
    normalised by the image size, NMS per image.  -> list of box lists."""
    nat.ensure_device(imgs)
    B, _, height, width = imgs.shape
    anchors = get_anchors(ANCHOR_PATH) if anchors is None else anchors
    num_anchors = len(anchors)                    # utils.py:496 (the number of groups, = 3)
    with torch.no_grad():
        outputs = model.forward(imgs)
    cap = sum(o.size(2) * o.size(3) for o in outputs) * num_anchors
    det = Detections(B, cap, imgs.device)
    for i in range(len(anchors)):                 # utils.py:501-506
        region_boxes_device(outputs[i], conf_thresh, num_classes, anchors[i], num_anchors, (width, height),
                            norm=(width, height), det=det)
    keep, nkeep = nms_device(det, nms_thresh)
    return _box_lists(det.boxes.cpu().numpy(), det.counts.cpu().numpy(), keep.cpu().numpy(), nkeep.cpu().numpy())


def do_detect(model, img, conf_thresh, nms_thresh, use_cuda=1):
    """utils.py:450-519: a PIL image or an HWC uint8 array -> the kept boxes."""
    from PIL import Image
    if isinstance(img, Image.Image):
        arr = np.asarray(img.convert("RGB"), dtype=np.uint8)
    elif isinstance(img, np.ndarray):
        arr = img
    else:
        raise TypeError("unknown image type")
    x = torch.from_numpy(arr.copy()).permute(2, 0, 1).float().div(255.0).unsqueeze(0)
    x = x.to(torch.device("cuda", torch.cuda.current_device()))
    return detect_batch(model, x, conf_thresh, nms_thresh)[0]
