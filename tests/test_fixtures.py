"""Pins against the reference's own data files (CPU), committed as fixtures
under tests/golden/ (data, not code):

* ``30values.txt``  = reference non_printability/30values.txt, the NPS colours
  (load_data.py:369-389 parses it with np.float32 of the decimal strings);
* ``0_patch.png``   = reference training_patches_saves/trained_patches/0_patch.png,
  the saved-patch layout (train_patch.py:367-376, ToPILImage('RGB'): 224x224
  RGB 8-bit, value trunc(255*x)).

Plus the host data path (DotaDataset, load_data.py:859-978) on a tiny on-disk
set: grey-127 square padding, label re-normalisation, the empty-file ones(5)
row and pad_lab's 1e-6 rows."""
import os
import types

import numpy as np
import pytest
import torch

from conftest import ROOT, pkg_mod

GOLD = os.path.join(ROOT, "tests", "golden")
REF = "/root/reference"


def test_printability_table_equals_reference_file():
    ld, pr = pkg_mod("load_data"), pkg_mod("printability")
    path = os.path.join(GOLD, "30values.txt")
    parsed = ld.load_printability_colors(path)                     # the reference file format
    builtin = ld.load_printability_colors("builtin:30values")
    assert parsed.shape == (30, 3)
    assert torch.equal(parsed, builtin)
    # and as the reference parses it: np.float32 of each decimal string
    with open(path) as f:
        rows = [[np.float32(v) for v in line.strip().split(",")] for line in f if line.strip()]
    assert np.array_equal(np.asarray(rows, dtype=np.float32), builtin.numpy())
    assert len(pr.PRINTABLE_RGB_30) == 30


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference checkout not present")
def test_fixtures_are_the_reference_files():
    for fx, ref in (("30values.txt", "non_printability/30values.txt"),
                    ("0_patch.png", "training_patches_saves/trained_patches/0_patch.png")):
        with open(os.path.join(GOLD, fx), "rb") as a, open(os.path.join(REF, ref), "rb") as b:
            assert a.read() == b.read(), fx


def test_saved_patch_png_roundtrip_is_byte_identical(tmp_path):
    """read_image (train_patch.py:411-426: PIL RGB, Resize to patch_size,
    ToTensor) of the reference's saved patch, then save_patch_png
    (ToPILImage: trunc(255*x)), re-read: the same 224x224x3 bytes."""
    from PIL import Image
    tp = pkg_mod("train_patch")
    src = os.path.join(GOLD, "0_patch.png")
    want = np.asarray(Image.open(src).convert("RGB"))
    assert want.shape == (224, 224, 3) and want.dtype == np.uint8
    fake = types.SimpleNamespace(config=types.SimpleNamespace(patch_size=224))
    patch = tp.PatchTrainer.read_image(fake, src)
    assert patch.shape == (3, 224, 224) and patch.dtype == torch.float32
    assert torch.equal(patch, torch.from_numpy(want.copy()).permute(2, 0, 1).float() / 255.0)
    out = str(tmp_path / "0_patch.png")
    tp.save_patch_png(patch, out)
    back = Image.open(out)
    assert back.mode == "RGB" and back.size == (224, 224)
    assert np.array_equal(np.asarray(back), want)
    # the layout's quantisation: trunc, not round (ToPILImage mul(255).byte())
    p = torch.full((3, 4, 4), 0.999)
    tp.save_patch_png(p, str(tmp_path / "t.png"))
    assert int(np.asarray(Image.open(str(tmp_path / "t.png"))).max()) == 254
    assert tp.patch_mse(out, out) == 0.0


def _write(path, arr):
    from PIL import Image
    Image.fromarray(arr, "RGB").save(path)


def test_dota_dataset_padding_and_labels(tmp_path):
    """load_data.py:910-978 on three images: wider than tall, taller than
    wide (empty label file), square."""
    ld = pkg_mod("load_data")
    img_dir, lab_dir = tmp_path / "images", tmp_path / "labels"
    img_dir.mkdir()
    lab_dir.mkdir()
    rng = np.random.default_rng(0)
    _write(str(img_dir / "wide.png"), rng.integers(0, 256, (30, 40, 3), dtype=np.uint8))   # w=40, h=30
    _write(str(img_dir / "tall.png"), rng.integers(0, 256, (40, 30, 3), dtype=np.uint8))   # w=30, h=40
    _write(str(img_dir / "sq.png"), rng.integers(0, 256, (32, 32, 3), dtype=np.uint8))
    (lab_dir / "wide.txt").write_text("3 0.5 0.25 0.1 0.2\n7 0.1 0.9 0.05 0.3\n")
    (lab_dir / "tall.txt").write_text("")
    (lab_dir / "sq.txt").write_text("1 0.4 0.6 0.2 0.1\n")
    S, L = 64, 252
    ds = ld.DotaDataset(str(img_dir), str(lab_dir), L, S, shuffle=False)
    assert len(ds) == 3
    items = {os.path.splitext(n)[0]: ds[i] for i, n in enumerate(ds.img_names)}
    for name, (img, lab) in items.items():
        assert img.shape == (3, S, S) and img.dtype == torch.float32
        assert float(img.min()) >= 0 and float(img.max()) <= 1
        assert lab.shape == (L, 5)
    grey = 127 / 255.0
    # wide: padded top and bottom (5 px of 40 -> 8 px of 64); the outer rows are pure pad colour
    img, lab = items["wide"]
    assert torch.all(img[:, 0, :] == torch.tensor(grey, dtype=torch.float32))
    assert torch.all(img[:, -1, :] == torch.tensor(grey, dtype=torch.float32))
    w, h, pad = 40, 30, 5.0
    rows = torch.tensor([[3, 0.5, 0.25, 0.1, 0.2], [7, 0.1, 0.9, 0.05, 0.3]], dtype=torch.float32)
    want = rows.clone()
    want[:, 2] = (rows[:, 2] * h + pad) / w
    want[:, 4] = rows[:, 4] * h / w
    assert torch.equal(lab[:2], want)
    assert torch.all(lab[2:] == torch.tensor(1e-6, dtype=torch.float32))
    # tall, empty label file: one row of ones(5), re-normalised along x
    img, lab = items["tall"]
    assert torch.all(img[:, :, 0] == torch.tensor(grey, dtype=torch.float32))
    w, h, pad = 30, 40, 5.0
    one = torch.ones(1, 5)
    want = one.clone()
    want[:, 1] = (one[:, 1] * w + pad) / h
    want[:, 3] = one[:, 3] * w / h
    assert torch.equal(lab[:1], want)
    assert torch.all(lab[1:] == torch.tensor(1e-6, dtype=torch.float32))
    # square: labels untouched, no padding colour forced
    img, lab = items["sq"]
    assert torch.equal(lab[0], torch.tensor([1, 0.4, 0.6, 0.2, 0.1], dtype=torch.float32))
    # a DataLoader batch has the reference's collated shapes
    dl = torch.utils.data.DataLoader(ds, batch_size=3, shuffle=False)
    ib, lb = next(iter(dl))
    assert ib.shape == (3, 3, S, S) and lb.shape == (3, L, 5)


def test_dota_uint8_loader_and_prefetcher_match_float_path(tmp_path):
    """The training loader's uint8 path (DotaDataset(as_uint8=True) through a
    2-worker DataLoader with GlobalBatchSampler, then DevicePrefetcher's /255)
    yields exactly the float batches of the reference path
    (load_data.py:910-978: ToTensor on the host)."""
    ld, tp = pkg_mod("load_data"), pkg_mod("train_patch")
    img_dir, lab_dir = tmp_path / "images", tmp_path / "labels"
    img_dir.mkdir()
    lab_dir.mkdir()
    rng = np.random.default_rng(3)
    for k in range(7):
        h, w = int(rng.integers(20, 50)), int(rng.integers(20, 50))
        _write(str(img_dir / ("im%d.png" % k)), rng.integers(0, 256, (h, w, 3), dtype=np.uint8))
        (lab_dir / ("im%d.txt" % k)).write_text("%d 0.5 0.5 0.2 0.1\n" % k if k % 3 else "")
    S, L = 48, 252
    ref = ld.DotaDataset(str(img_dir), str(lab_dir), L, S, shuffle=False)
    u8 = ld.DotaDataset(str(img_dir), str(lab_dir), L, S, shuffle=False, as_uint8=True)
    smp = tp.GlobalBatchSampler(len(u8), 3, shuffle=True, seed=5)
    loader = torch.utils.data.DataLoader(u8, batch_sampler=smp, num_workers=2)
    got = list(ld.DevicePrefetcher(loader, "cpu"))
    order = [i for b in smp for i in b]
    assert len(got) == 3 and sum(g[0].size(0) for g in got) == 7
    flat_img = torch.cat([g[0] for g in got])
    flat_lab = torch.cat([g[1] for g in got])
    assert flat_img.dtype == torch.float32
    for row, i in enumerate(order):
        img, lab = ref[i]
        assert torch.equal(flat_img[row], img)
        assert torch.equal(flat_lab[row], lab)
    # the decoded-once frame cache gives the same batches, every pass
    cache = ld.FrameCache(u8, "cpu", num_workers=2, batch=4)
    for _ in range(2):
        again = list(cache.loader(smp))
        assert len(again) == len(got)
        for (a, b), (c, d) in zip(again, got):
            assert torch.equal(a, c) and torch.equal(b, d)
