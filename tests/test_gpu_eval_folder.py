"""GPU test of the folder-level evaluation driver (eval_patch.evaluate_folder,
the reference's test_patch_DOTA.py:72-201) on a 4-image folder: grey pad +
resize, placement, composite, ToPILImage uint8 quantisation, detection and
label files, against the oracle restatement of each stage on the same
inputs and draws:

* frames: the host pad/resize equals the reference recipe (PIL, inline here)
  byte for byte;
* patched, quantised frames: oracle.patch_transformer (the reference's
  fp32 placement, which the HIP path reproduces bit for bit) +
  patch_applier + trunc(255 x) — byte for byte;
* boxes and label files: oracle/detect_ref.detect_postprocess of the HIP
  heads of those frames (conf 0.4, NMS 0.4), the label-file lines the
  reference writes; batching (batch 2 vs 4) changes nothing;
* creation_metrics runs on the written folder."""
import os

import numpy as np
import pytest
import torch

import oracle
from oracle import detect_ref as ref
from conftest import pkg_mod
from test_gpu_detect import _assert_boxes_equal

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _folder(tmp_path):
    from PIL import Image
    img_dir, lab_dir = tmp_path / "imgs", tmp_path / "labels"
    img_dir.mkdir()
    lab_dir.mkdir()
    rng = np.random.default_rng(5)
    sizes = [(640, 480), (300, 700), (608, 608), (200, 150)]
    for k, (w, h) in enumerate(sizes):
        arr = rng.integers(0, 256, (h, w, 3), dtype=np.uint8)
        Image.fromarray(arr, "RGB").save(str(img_dir / ("im%d.png" % k)))
        if k == 2:
            (lab_dir / ("im%d.txt" % k)).write_text("")                  # empty: ones(5)
        else:
            n = 1 + 2 * k
            rows = ["%d %.4f %.4f %.4f %.4f" % (rng.integers(0, 15), *rng.uniform(0.1, 0.9, 2), *rng.uniform(0.02, 0.3, 2))
                    for _ in range(n)]
            (lab_dir / ("im%d.txt" % k)).write_text("\n".join(rows) + "\n")
    return img_dir, lab_dir


def _reference_frame(path, S):
    """test_patch_DOTA.py:88-105 restated: grey pad at int(padding), Resize."""
    from PIL import Image, ImageOps
    img = ImageOps.exif_transpose(Image.open(path)).convert("RGB")
    w, h = img.size
    if w == h:
        padded = img
    elif w < h:
        padded = Image.new("RGB", (h, h), color=(127, 127, 127))
        padded.paste(img, (int((h - w) / 2), 0))
    else:
        padded = Image.new("RGB", (w, w), color=(127, 127, 127))
        padded.paste(img, (0, int((w - h) / 2)))
    return np.asarray(padded.resize((S, S), Image.BILINEAR), dtype=np.uint8)


def test_evaluate_folder_matches_oracle(tmp_path):
    ev, ut, us, dk, W, sy, ld = (pkg_mod(m) for m in ("eval_patch", "utils", "utils_self", "darknet_v3", "weights",
                                                     "synthetic", "load_data"))
    img_dir, lab_dir = _folder(tmp_path)
    wpath = str(tmp_path / "w.weights")
    W.write_weights(wpath, W.synthesize("builtin:yolov3-dota", seed=4))
    net = dk.Darknet("builtin:yolov3-dota")
    net.load_darknet_weights(wpath)
    S, P, seed = 608, 224, 11
    patch = sy.patch(P, seed=12)
    runs = []
    for bs in (4, 2):
        out = tmp_path / ("out%d" % bs)
        res, frames = ev.evaluate_folder(net, patch.to(DEV), str(img_dir), str(lab_dir), str(out), 0.4, 0.4,
                                         batch_size=bs, seed=seed, save_images=(bs == 4), return_frames=True)
        runs.append((res, frames, out))
    (res, frames, out), (res2, frames2, _) = runs
    assert sorted(res) == ["im0", "im1", "im2", "im3"]
    anchors = ut.get_anchors(None)
    stems = sorted(res)
    x4 = ld.u8_to_float(torch.stack([frames[st] for st in stems]).to(DEV))
    heads4 = [h.cpu() for h in net.forward(x4)]
    heads2 = [torch.cat(hs) for hs in zip(*[[h.cpu() for h in net.forward(x4[i:i + 2].contiguous())]
                                            for i in (0, 2)])]
    for k, stem in enumerate(sorted(res)):
        # the frames do not depend on the batch size (draws keyed by the image's index); the
        # detections of each run are checked against the oracle decode of that run's own heads
        assert torch.equal(frames[stem], frames2[stem])
        # oracle: pad/resize, placement (draws of image k), composite, quantisation
        base = _reference_frame(str(img_dir / (stem + ".png")), S)
        lab = ev.load_eval_labels(str(lab_dir / (stem + ".txt"))).unsqueeze(0)
        dr = {kk: v.cpu() for kk, v in sy.draws_device(seed, 0, k, 1, P, DEV).items()}
        img = torch.from_numpy(base.copy()).permute(2, 0, 1).float().div(255.0).unsqueeze(0)
        adv_t, _ = oracle.patch_transformer(patch, lab, S, dr)
        want = oracle.patch_applier(img, adv_t)[0].mul(255).to(torch.uint8)
        got = frames[stem]
        diff = (got.int() - want.int()).abs()
        assert int(diff.max()) == 0, (stem, int(diff.max()), int((diff > 0).sum()))
        # detection on the quantised frame: the HIP heads of the batch-4 forward (the
        # batch the bs=4 run detected in, so the same launches) through the oracle post-process
        want_boxes = ref.detect_postprocess([h[k:k + 1] for h in heads4], S, S, anchors, 15, 0.4, 0.4)
        _assert_boxes_equal(res[stem], want_boxes, sat_ties=True)
        want2 = ref.detect_postprocess([h[k:k + 1] for h in heads2], S, S, anchors, 15, 0.4, 0.4)
        _assert_boxes_equal(res2[stem], want2, sat_ties=True)
        lines = (out / "yolo-labels" / (stem + ".txt")).read_text().splitlines()
        assert lines == ["%s %s %s %s %s %s %s" % tuple(b) for b in res[stem]]
        assert (out / "pre_patched" / (stem + ".png")).exists()
    n = sum(len(b) for b in res.values())
    assert us.txt_len_read(str(out / "yolo-labels"))[0] == n
    # the clean frames' detections (an all-zero patch composites nothing: the reference's
    # clean-image label folders) against the patched ones
    clean = tmp_path / "clean"
    ev.evaluate_folder(net, torch.zeros_like(patch).to(DEV), str(img_dir), str(lab_dir), str(clean), 0.4, 0.4,
                       batch_size=4, seed=seed, save_images=False)
    m = us.creation_metrics(str(out / "yolo-labels"), str(clean / "yolo-labels"), str(out / "yolo-labels"),
                            str(clean / "yolo-labels"))
    assert "M1_04" in m and len(m["M4"]) == 15
