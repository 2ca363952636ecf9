"""Folder-level patch evaluation — the reference's ``test_patch_DOTA.py``
(test_patch_DOTA.py:72-201) on the MI355X path, feeding the creation metrics
of ``test_patch_DOTA_metrics.py`` (utils_self.creation_metrics).

Per image of ``imgdir`` (``.png`` / ``.jpg``), as the reference loop does:

    load (EXIF transpose, RGB)                         utils_self.load_image_file
    grey-127 square pad at int(padding), Resize(S)     test_patch_DOTA.py:88-105
    labels: np.loadtxt of <name>.txt, ones(5) if empty test_patch_DOTA.py:135-141
    PatchTransformer(do_rotate=True, rand_loc=False)   test_patch_DOTA.py:153-154
    PatchApplier                                       test_patch_DOTA.py:158-159
    ToPILImage('RGB'): uint8 = trunc(255 x)            test_patch_DOTA.py:162
    do_detect(model, p_img_pil, 0.4, 0.4)              test_patch_DOTA.py:173
    plot_boxes -> <savedir>/pre_patched/<name>.png     test_patch_DOTA.py:190-196
    label file <savedir>/yolo-labels/<name>.txt        test_patch_DOTA.py:198-201
      one "cx cy w h det_conf cls_conf cls_id" line per box

The reference runs one image at a time on the host; here the frames are
decoded and padded on the host (PIL, as DotaDataset) and everything after —
median pool, placement, warp + composite, the uint8 quantisation, the Darknet
forward, decode and NMS — runs on the GPU in batches.  The patched frames
do not depend on the batch size: the placement draws are keyed by the image's
index in the folder (po_draws, seed ``seed``, step 0), and an image's labels
are padded to the batch's row count by repeating its own first row, which
leaves lab_transform's max-area / min-area picks (first index on ties) where
the reference's unpadded [1, n, 5] labels put them.  The detections may differ
between batch sizes at fp32 rounding (the conv tiles are tuned per batch
shape): a box whose confidence sits at the threshold can come and go.  Files are visited in sorted
order (the reference's os.listdir order is the filesystem's)."""
import math
import os
import sys

if __package__ in (None, ""):
    import importlib
    _here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, os.path.dirname(_here))
    _pkg = importlib.import_module(os.path.basename(_here))
    __package__ = _pkg.__name__

import numpy as np
import torch

from . import _native as nat
from . import utils
from .load_data import PatchApplier, PatchTransformer, u8_to_float

IMG_EXTS = (".png", ".jpg")


def load_image_file(path, mode="RGB"):
    """utils_self.load_image_file (utils_self.py:151-166): PIL open, EXIF
    transpose, convert."""
    from PIL import Image, ImageOps
    img = Image.open(path)
    img = ImageOps.exif_transpose(img)
    return img.convert(mode)


def pad_and_resize(img, img_size):
    """test_patch_DOTA.py:88-105: grey (127,127,127) square canvas, the image
    pasted at int(padding) on the short side, transforms.Resize((S, S))
    (PIL bilinear) -> PIL image."""
    from PIL import Image
    w, h = img.size
    if w == h:
        padded = img
    elif w < h:
        padded = Image.new("RGB", (h, h), color=(127, 127, 127))
        padded.paste(img, (int((h - w) / 2), 0))
    else:
        padded = Image.new("RGB", (w, w), color=(127, 127, 127))
        padded.paste(img, (0, int((w - h) / 2)))
    return padded.resize((img_size, img_size), Image.BILINEAR)


def load_eval_labels(txtpath):
    """test_patch_DOTA.py:135-141: np.loadtxt of the label file (float32 rows
    [cls, x, y, w, h]), ones(5) for an empty file -> [n, 5]."""
    if os.path.getsize(txtpath):
        lab = np.loadtxt(txtpath)
    else:
        lab = np.ones([5])
    lab = torch.from_numpy(np.asarray(lab)).float()
    if lab.dim() == 1:
        lab = lab.unsqueeze(0)
    return lab


def plot_boxes(img, boxes, savename=None, class_names=None):
    """utils.plot_boxes (utils.py:294-345): each box as a rectangle in its
    class colour (offset cls_id * 123457 % classes over the reference's six
    colour stops) with the class name above it.  The reference's font file
    (data/simhei.ttf) is not shipped: PIL's default font is used."""
    from PIL import ImageDraw
    colors = [[1, 0, 1], [0, 0, 1], [0, 1, 1], [0, 1, 0], [1, 1, 0], [1, 0, 0]]

    def get_color(c, x, max_val):
        ratio = float(x) / max_val * 5
        i, j = int(math.floor(ratio)), int(math.ceil(ratio))
        ratio -= i
        return int(((1 - ratio) * colors[i][c] + ratio * colors[j][c]) * 255)

    width, height = img.width, img.height
    draw = ImageDraw.Draw(img)
    for box in boxes:
        x1, y1 = (box[0] - box[2] / 2.0) * width, (box[1] - box[3] / 2.0) * height
        x2, y2 = (box[0] + box[2] / 2.0) * width, (box[1] + box[3] / 2.0) * height
        rgb = (255, 0, 0)
        if len(box) >= 5 and class_names:
            cls_id = int(box[6])
            classes = len(class_names)
            offset = cls_id * 123457 % classes
            rgb = (get_color(2, offset, classes), get_color(1, offset, classes), get_color(0, offset, classes))
            draw.text((x1, y1), class_names[cls_id], fill=rgb)
        draw.rectangle([x1, y1, x2, y2], outline=rgb, width=2)
    if savename:
        img.save(savename)
    return img


def quantise_u8(p_img):
    """ToPILImage('RGB') on a float image in [0, 1] (test_patch_DOTA.py:162):
    uint8 = trunc(255 x) — the same fp32 multiply and truncation on the device."""
    return p_img.mul(255).to(torch.uint8)


def evaluate_folder(darknet_model, adv_patch, imgdir, clean_labdir, savedir, conf_thresh=0.4, nms_thresh=0.4,
                    batch_size=16, seed=0, save_images=True, class_names=None, return_frames=False):
    """The reference evaluation loop over ``imgdir`` (see the module doc).
    ``adv_patch`` [3,P,P] in [0,1] (any device); ``darknet_model`` a
    darknet_v3.Darknet with weights.  Writes <savedir>/yolo-labels/<name>.txt
    (and <savedir>/pre_patched/<name>.png when ``save_images``).  Returns
    {name: boxes} (boxes [cx, cy, w, h, det_conf, cls_conf, cls_id],
    normalised), plus {name: uint8 [3,S,S] patched frame} with
    ``return_frames``."""
    dev = torch.device("cuda", torch.cuda.current_device())
    S = int(darknet_model.height)
    adv_patch = adv_patch.to(dev).float()
    names = sorted(f for f in os.listdir(imgdir) if f.endswith(IMG_EXTS))
    os.makedirs(os.path.join(savedir, "yolo-labels"), exist_ok=True)
    if save_images:
        os.makedirs(os.path.join(savedir, "pre_patched"), exist_ok=True)
    transformer, applier = PatchTransformer(), PatchApplier()
    transformer.draw_seed = seed
    results, frames_out = {}, {}
    for k0 in range(0, len(names), batch_size):
        chunk = names[k0:k0 + batch_size]
        frames, labs = [], []
        for f in chunk:
            stem = os.path.splitext(f)[0]
            img = pad_and_resize(load_image_file(os.path.join(imgdir, f)), S)
            frames.append(torch.from_numpy(np.asarray(img, dtype=np.uint8).copy()).permute(2, 0, 1))
            labs.append(load_eval_labels(os.path.join(clean_labdir, stem + ".txt")))
        L = max(l.size(0) for l in labs)
        # rows repeated from the image's first: lab_transform's first-index argmax /
        # argmin over the real rows are unchanged (the reference's labels are unpadded)
        lab = torch.stack([torch.cat([l, l[:1].expand(L - l.size(0), 5)], 0) for l in labs]).to(dev)
        img_batch = u8_to_float(torch.stack(frames).to(dev))            # ToTensor (test_patch_DOTA.py:143-144)
        transformer.draw_step, transformer.draw_b0 = 0, k0               # draws keyed by the image's index
        with torch.no_grad():
            adv_batch_t, _ = transformer(adv_patch, lab, S, do_rotate=True, rand_loc=False)
            p_img = applier(img_batch, adv_batch_t)
            q = quantise_u8(p_img)
            boxes = utils.detect_batch(darknet_model, u8_to_float(q), conf_thresh, nms_thresh)
        q_cpu = q.cpu() if (save_images or return_frames) else None
        for i, f in enumerate(chunk):
            stem = os.path.splitext(f)[0]
            results[stem] = boxes[i]
            with open(os.path.join(savedir, "yolo-labels", stem + ".txt"), "w+") as tf:
                for b in boxes[i]:
                    tf.write(f"{b[0]} {b[1]} {b[2]} {b[3]} {b[4]} {b[5]} {b[6]}\n")
            if save_images:
                from PIL import Image
                pil = Image.fromarray(q_cpu[i].permute(1, 2, 0).numpy(), "RGB")
                plot_boxes(pil, boxes[i], os.path.join(savedir, "pre_patched", stem + ".png"), class_names)
            if return_frames:
                frames_out[stem] = q_cpu[i]
    return (results, frames_out) if return_frames else results


def main(argv=None):
    """test_patch_DOTA.py as a command:
    python -m <pkg>.eval_patch --imgdir D --labdir D --patch P.png --savedir D
        [--cfg builtin:yolov3-dota] [--weights W] [--conf 0.4] [--nms 0.4]
        [--batch 16] [--seed 0] [--names data/dota.names] [--no-images]"""
    import argparse
    import time
    from PIL import Image
    from .darknet_v3 import Darknet
    from . import patch_config, weights as synth_weights
    ap = argparse.ArgumentParser(description=main.__doc__)
    ap.add_argument("--imgdir", required=True)
    ap.add_argument("--labdir", required=True)
    ap.add_argument("--patch", required=True)
    ap.add_argument("--savedir", required=True)
    ap.add_argument("--cfg", default="builtin:yolov3-dota")
    ap.add_argument("--weights", default=None)
    ap.add_argument("--conf", type=float, default=0.4)
    ap.add_argument("--nms", type=float, default=0.4)
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--names", default=None)
    ap.add_argument("--no-images", action="store_true")
    args = ap.parse_args(argv)
    nat.load()
    print("patchfile : ", args.patch)
    print("savedir : ", args.savedir)
    model = Darknet(args.cfg)
    wf = args.weights or patch_config.synthetic_weights_path(args.cfg.split(":")[-1])
    if not os.path.exists(wf):
        synth_weights.ensure_synthetic(args.cfg, wf)
    model.load_darknet_weights(wf)
    model = model.eval()
    print("input image size of yolov3: ", model.height, model.width)
    pil = load_image_file(args.patch)
    patch = torch.from_numpy(np.asarray(pil, dtype=np.uint8).copy()).permute(2, 0, 1)
    adv_patch = u8_to_float(patch.to(torch.device("cuda", torch.cuda.current_device())))
    names = utils.load_class_names(args.names) if args.names else utils.DOTA_NAMES
    t0 = time.time()
    res = evaluate_folder(model, adv_patch, args.imgdir, args.labdir, args.savedir, args.conf, args.nms,
                          args.batch, args.seed, not args.no_images, names)
    print("Processing Done!  %d images, %d boxes" % (len(res), sum(len(b) for b in res.values())))
    print("Total Running Time : ", (time.time() - t0) / 60, "minutes !")
    return res


if __name__ == "__main__":
    main()
