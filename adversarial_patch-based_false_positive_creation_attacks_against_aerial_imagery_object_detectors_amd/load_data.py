"""Patch transform / composite / regularisers — drop-in for the training-path
classes of reference ``load_data.py`` backed by the HIP library.

=====================  ==========================================  =========================
class                  reference                                   HIP entry points
=====================  ==========================================  =========================
NPSCalculator          load_data.py:340-389                        po_regularisers
TotalVariation         load_data.py:392-411                        po_regularisers
PatchTransformer       load_data.py:414-794 (training placement)   po_median7_*, po_patch_params,
                                                                   po_warp_fwd / po_warp_bwd
PatchApplier           load_data.py:797-833                        po_apply_fwd / po_apply_bwd
PatchTransformer_      load_data.py:985-1230 (one patch per        po_vanishing_params, po_warp_fwd,
  vanishing            label, evaluation)                          po_warp_composite_multi
PatchTransformer_      load_data.py:1233-1722 (placement away      po_place_test_mode,
  test_mode            from the detections, evaluation)            po_place_free_map
HasSusRGB              load_data.py:1724-1754                      po_regularisers
DotaDataset            load_data.py:859-978 (host data loader)     (PIL / numpy, no GPU)
=====================  ==========================================  =========================

Randomness: the reference draws contrast/brightness/noise/angle from the CUDA
RNG and target_x/target_y from the CPU RNG (load_data.py:548-707).  Here all
draws are made on the device by the counter-based ``po_draws`` (keyed by seed,
step counter and GLOBAL image index, so a data-parallel rank draws exactly the
rows of its shard) unless passed in explicitly with ``draws=`` (parity tests);
a step has no host<->device sync.
"""
import fnmatch
import math
import os

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _native as nat
from .max_prob import MaxProbExtractor  # noqa: F401  (load_data.py:125-311)
from .median_pool import MedianPool2d
from .printability import PRINTABLE_RGB_30
from . import synthetic

SCALE_FACTOR = 2.          # load_data.py:32
NOISE_FACTOR = 0.10        # load_data.py:436


def read_image(path):
    """PNG/JPG -> [3,H,W] float in [0,1] (load_data.py:35-47; ToTensor)."""
    from PIL import Image
    img = Image.open(path).convert("RGB")
    return torch.from_numpy(np.asarray(img, dtype=np.uint8).copy()).permute(2, 0, 1).float().div_(255.0)


def load_printability_colors(printability_file):
    """[ncol,3] float32 colours from a reference-format file ('r,g,b' per
    line; load_data.py:369-389 converts the decimal strings with np.float32)
    or from ``builtin:30values``."""
    if printability_file in (None, "builtin:30values"):
        rows = PRINTABLE_RGB_30
    else:
        rows = []
        with open(printability_file) as f:
            for line in f:
                line = line.strip()
                if line and not line.startswith("#"):
                    rows.append(tuple(line.split(",")))
    return torch.tensor(np.asarray([[np.float32(float(v)) for v in r] for r in rows], dtype=np.float32))


# ---------------------------------------------------------------------------
# Regularisers (NPS / TV / colourfulness) as one autograd function
# ---------------------------------------------------------------------------
class _Regularisers(torch.autograd.Function):
    @staticmethod
    def forward(ctx, patch, colors):
        nat.ensure_device(patch)
        patch = patch.contiguous()
        P = patch.size(-1)
        out3 = torch.empty(3, device=patch.device)
        ws = torch.empty(16384, device=patch.device)
        nat.call("po_regularisers", nat.ptr(patch), P, nat.ptr(colors), colors.size(0), None,
                 nat.ptr(out3), None, nat.ptr(ws), nat.stream())
        ctx.save_for_backward(patch, colors)
        return out3

    @staticmethod
    def backward(ctx, g3):
        patch, colors = ctx.saved_tensors
        g3 = g3.contiguous().float()
        out3 = torch.empty(3, device=patch.device)
        ws = torch.empty(16384, device=patch.device)
        d = torch.empty_like(patch)
        nat.call("po_regularisers", nat.ptr(patch), patch.size(-1), nat.ptr(colors), colors.size(0),
                 nat.ptr(g3), nat.ptr(out3), nat.ptr(d), nat.ptr(ws), nat.stream())
        return d, None


def regularisers(patch, colors):
    """(nps, tv, colour) of the raw [3,P,P] patch as a [3] tensor."""
    return _Regularisers.apply(patch, colors)


class _PatchFront(torch.autograd.Function):
    """The two functions of the raw patch a training step takes: its 7x7
    'same' median pool (MedianPool2d(7, same=True), median_pool.py:46-52) and
    its regularisers (NPS, TV, colour).  One autograd node: the backward runs
    po_median7_bwd and adds the regularisers' gradient into the same buffer
    (po_regularisers_grad, accumulate, from the forward's statistics) -- the
    value autograd forms by summing the two contributions, bit for bit,
    without the separate sum and the regularisers' recomputed reduction."""

    @staticmethod
    def forward(ctx, patch, colors):
        nat.ensure_device(patch)
        patch = patch.contiguous()
        C, H, W = patch.shape
        mp = torch.empty_like(patch)
        arg = torch.empty(patch.shape, dtype=torch.int32, device=patch.device)
        nat.call("po_median7_fwd", nat.ptr(patch), C, H, W, nat.ptr(mp), nat.ptr(arg, torch.int32), nat.stream())
        out3 = torch.empty(3, device=patch.device)
        ws = torch.empty(16384, device=patch.device)
        nat.call("po_regularisers", nat.ptr(patch), W, nat.ptr(colors), colors.size(0), None, nat.ptr(out3), None,
                 nat.ptr(ws), nat.stream())
        ctx.save_for_backward(patch, colors, arg, ws)
        ctx.set_materialize_grads(False)
        return mp, out3

    @staticmethod
    def backward(ctx, d_mp, g3):
        patch, colors, arg, ws = ctx.saved_tensors
        if d_mp is None and g3 is None:
            return None, None
        C, H, W = patch.shape
        d = torch.empty_like(patch)
        if d_mp is not None:
            nat.call("po_median7_bwd", nat.ptr(d_mp.contiguous()), nat.ptr(arg, torch.int32), C, H, W, nat.ptr(d),
                     nat.stream())
        if g3 is not None:
            nat.call("po_regularisers_grad", nat.ptr(patch), W, nat.ptr(colors), colors.size(0),
                     nat.ptr(g3.contiguous().float()), nat.ptr(ws), int(d_mp is not None), nat.ptr(d), nat.stream())
        return d, None


def patch_front(patch, colors):
    """(median-pooled patch [3,P,P], regularisers [3]) of the raw patch
    (PatchTransformer's median pool + NPS/TV/colour) in one autograd node."""
    if patch.size(-1) != patch.size(-2):
        raise ValueError("patch_front: square patches only")
    return _PatchFront.apply(patch, colors)


class NPSCalculator(nn.Module):
    """Non-printability score (load_data.py:340-389)."""

    def __init__(self, printability_file, patch_side):
        super().__init__()
        self.patch_side = patch_side
        self.register_buffer("colors", load_printability_colors(printability_file))

    @property
    def printability_array(self):
        """The reference's [ncol,3,side,side] array (expanded view)."""
        s = self.patch_side
        return self.colors.view(-1, 3, 1, 1).expand(-1, 3, s, s)

    def get_printability_array(self, printability_file, side):
        return load_printability_colors(printability_file).view(-1, 3, 1, 1).expand(-1, 3, side, side).contiguous()

    def forward(self, adv_patch):
        return regularisers(adv_patch, self.colors.to(adv_patch.device))[0]


class TotalVariation(nn.Module):
    """Total variation of the patch (load_data.py:392-411)."""

    def __init__(self):
        super().__init__()
        self.register_buffer("colors", torch.tensor([[0.5, 0.5, 0.5]]))

    def forward(self, adv_patch):
        return regularisers(adv_patch, self.colors.to(adv_patch.device))[1]


class HasSusRGB(nn.Module):
    """Colourfulness loss sigma + 0.3*mu of (R-G, (R+G)/2-B) (load_data.py:1724-1754)."""

    def __init__(self):
        super().__init__()
        self.register_buffer("colors", torch.tensor([[0.5, 0.5, 0.5]]))

    def forward(self, RGB_img):
        return regularisers(RGB_img, self.colors.to(RGB_img.device))[2]


# ---------------------------------------------------------------------------
# Patch placement and warp
# ---------------------------------------------------------------------------
_BMM_FORM = []


def reference_bmm_form():
    """The order in which this host's PyTorch-CPU evaluates affine_grid's
    K = 3 dot product x = bx*t0 + by*t1 + t2 (load_data.py:745): MKL's sgemm
    picks its code path by CPU -- "sum" (fl(fl(bx*t0) + fl(by*t1)) + t2, the
    AMD EPYC hosts of the MI355X boxes) or "fma" (fl(fma(by, t1, fl(bx*t0)) +
    t2), Intel AVX-512).  Asked once per process with a small affine_grid:
    the "sum" form reproduces it exactly or the host uses the "fma" one
    (tests/test_geometry_ref.py pins both forms against the host's torch)."""
    if not _BMM_FORM:
        th = torch.randn(2, 2, 3, generator=torch.Generator().manual_seed(7)) * 3
        g = F.affine_grid(th, (2, 1, 64, 64), align_corners=False).numpy()
        lin = torch.linspace(-1, 1, 64).numpy()
        base = ((lin * np.float32(63)).astype(np.float32) / np.float32(64)).astype(np.float32)
        t = th.numpy()
        bx, by = base[None, None, :], base[None, :, None]
        same = True
        for r in range(2):
            t0, t1, t2 = (t[:, r, k][:, None, None] for k in range(3))
            x = (((bx * t0).astype(np.float32) + (by * t1).astype(np.float32)).astype(np.float32) + t2)
            same &= bool(np.array_equal(x.astype(np.float32), g[..., r]))
        _BMM_FORM.append("sum" if same else "fma")
    return _BMM_FORM[0]


class _Geometries(dict):
    """{"ref": 1 or 2 (po_patch_params' reference geometry for this host's
    sgemm order, reference_bmm_form()), "f64": 0}."""

    def __missing__(self, key):
        if key != "ref":
            raise KeyError(key)
        return 1 if reference_bmm_form() == "sum" else 2

    def __contains__(self, key):
        return key in ("ref", "f64")


GEOMETRIES = _Geometries(f64=0)


def default_geometry():
    """The placement geometry of the training path: "ref" (default) -- the
    reference's fp32 theta / affine_grid / grid_sample arithmetic, op by op
    (po_patch_params geometry 1); "f64" (ADVPATCH_GEOMETRY=f64) -- the same
    formulas evaluated in float64 (closer to the exact value, not to the
    reference)."""
    g = os.environ.get("ADVPATCH_GEOMETRY", "ref")
    if g not in GEOMETRIES:
        raise ValueError("ADVPATCH_GEOMETRY must be one of ('ref', 'f64')")
    return g


_SINCOS_LUT = {}


def sincos_lattice_table(device):
    """[2^24, 2] fp32 on ``device``: (sin, cos) of every angle po_draws can
    draw, angle_k = fp32(k * 2^-24 * fp32(2 pi) - pi) (csrc/draw_ops.hip),
    as the reference's torch.sin / torch.cos compute them on PyTorch-CPU
    (load_data.py:731-732).  Those run MKL VML, which is not correctly
    rounded (~5 % of values one ulp off), so no device formula reproduces
    them; po_patch_params looks each drawn angle up here.  Built once per
    process and device (the CPU's own values, 128 MiB of HBM)."""
    dev = torch.device(device)
    key = (dev.type, dev.index)
    lut = _SINCOS_LUT.get(key)
    if lut is None:
        pi = np.float32(math.pi)
        k = np.arange(1 << 24, dtype=np.int64)
        u = (k.astype(np.float32) * np.float32(2.0 ** -24)).astype(np.float64)
        ang = torch.from_numpy((u * np.float64(np.float32(2.0) * pi) + np.float64(-pi)).astype(np.float32))
        lut = torch.stack([torch.sin(ang), torch.cos(ang)], 1).contiguous().to(dev)
        _SINCOS_LUT[key] = lut
    return lut


_SQRT_LUT = {}


def sqrt_period_table(device):
    """[2^24] fp32 on ``device``: the host's torch.sqrt (load_data.py:667-668;
    MKL VML, not correctly rounded: ~17 % of values one ulp off on the AMD
    EPYC hosts of the MI355X boxes) of every float in [1, 4) -- entry i is
    sqrt of the float with bits 0x3F800000 + i.  Its values scale exactly
    with powers of 4 (tests/test_geometry_ref.py checks this on the host), so
    one period reproduces the target size's sqrt for every normal input
    (po_patch_params).  Built once per process and device (64 MiB of HBM)."""
    dev = torch.device(device)
    key = (dev.type, dev.index)
    lut = _SQRT_LUT.get(key)
    if lut is None:
        bits = np.arange(0x3F800000, 0x3F800000 + (1 << 24), dtype=np.uint32)
        lut = torch.sqrt(torch.from_numpy(bits.view(np.float32))).contiguous().to(dev)
        _SQRT_LUT[key] = lut
    return lut


def patch_params(lab_batch, img_size, P, draws, do_rotate=True, with_roi=False, geometry=None):
    """(theta [B,6], patch_center [B,2], target_size [B][, roi [B,4] int32,
    affine [B,6] float64]) on the device.  ``affine`` holds the per-image
    placement rows the warp kernels read (po_patch_params); ``geometry``:
    "ref" / "f64" (default_geometry())."""
    nat.ensure_device(lab_batch)
    geometry = default_geometry() if geometry is None else geometry
    lab = lab_batch.contiguous().float()
    B, L = lab.size(0), lab.size(1)
    dev = lab.device
    theta = torch.empty(B, 6, device=dev)
    center = torch.empty(B, 2, device=dev)
    tsize = torch.empty(B, device=dev)
    roi = torch.empty(B, 4, dtype=torch.int32, device=dev) if with_roi else None
    affine = torch.empty(B, 6, dtype=torch.float64, device=dev) if with_roi else None
    angle = draws["angle"].contiguous().float() if do_rotate else None
    lut = sincos_lattice_table(dev) if (geometry == "ref" and do_rotate) else None
    sq = sqrt_period_table(dev) if geometry == "ref" else None
    nat.call("po_patch_params", nat.ptr(lab), B, L, nat.ptr(angle), nat.ptr(draws["ux"].contiguous().float()),
             nat.ptr(draws["uy"].contiguous().float()), int(bool(do_rotate)), int(img_size), int(P),
             GEOMETRIES[geometry], nat.ptr(lut), nat.ptr(sq), nat.ptr(theta), nat.ptr(center), nat.ptr(tsize),
             nat.ptr(roi, torch.int32), nat.ptr(affine, torch.float64), nat.stream())
    if with_roi:
        return theta, center, tsize, roi, affine
    return theta, center, tsize


WARP_FORMS = ("box", "pre", "frame")


class _Warp(torch.autograd.Function):
    """Augment + warp + clamp*mask (mode 0) or + composite onto img (mode 1)."""

    @staticmethod
    def forward(ctx, mp, noise, contrast, bright, affine, img, S, mode, form="box", roi=None, sparse=False,
                grad=True):
        """``noise``: the [B,3,P,P] tensor, or a po_draws key (seed, counter,
        b0) -- the noise is then regenerated from the key and no noise tensor
        exists.  With a key and the footprint boxes ``roi``, ``form`` picks the
        kernels: "box" (default) forms mp * contrast + bright + 0.1 * noise at
        each bilinear corner of the box pixels (po_warp_box_*_keyed); "pre"
        first writes the augmented patches [B,3,P,P] (po_augment_patch, one
        Philox call per 4 elements) and gathers them (po_warp_*_pre); "frame"
        runs the per-pixel kernels over whole frames (po_warp_*_keyed).  All
        forms give the same bits.  ``sparse`` (form "box", mode 1): only the
        quad-widened boxes of ``out`` are written -- the rest of the composite
        is ``img``, and the consumer reads the two (po_conv_first_*_cmp).
        ``grad``: whether a backward can follow -- the caller's
        torch.is_grad_enabled() and mp.requires_grad (grad mode is always off
        inside forward, and needs_input_grad ignores no_grad / inference
        mode), so no-grad and eval forwards skip the factor buffer."""
        mp = mp.contiguous()
        B = affine.size(0)
        P = mp.size(-1)
        out = torch.empty(B, 3, S, S, device=mp.device)
        imgp = nat.ptr(img.contiguous() if img is not None else None)
        ctx.form = "tensor"
        keyed = isinstance(noise, tuple)
        if keyed and roi is not None and form == "box" and S % 4 == 0:
            seed, counter, b0 = noise
            head = (imgp, nat.ptr(mp), int(seed) & 0xFFFFFFFFFFFFFFFF, int(counter) & 0xFFFFFFFFFFFFFFFF, int(b0),
                    nat.ptr(contrast), nat.ptr(bright), nat.ptr(affine, torch.float64), nat.ptr(roi, torch.int32),
                    B, S, P, mode, 0 if (sparse and mode == 1) else 1, nat.ptr(out))
            # the backward's per-pixel factors, written by the forward and turned
            # into the gradient factors in place (po_warp_box_*_fac; "0": re-evaluate
            # the warp in the backward, po_warp_box_bwd_keyed -- the same bits)
            ctx.fac = None
            # only when a backward can follow (no factor buffer for no-grad / eval forwards).
            # The buffer (B*S*S*16 bytes: 0.7 GB at tiny B=256 @416, 24 MB at yolov3 B=16 @608)
            # lives from the warp forward through the detector's forward and backward.
            if grad and os.environ.get("ADVPATCH_WARP_FAC", "1") != "0":
                ctx.fac = torch.empty(B * S * S * 4, device=mp.device)
                nat.call("po_warp_box_fwd_fac", *head, nat.ptr(ctx.fac), nat.stream())
            else:
                nat.call("po_warp_box_fwd_keyed", *head, nat.stream())
            ctx.key, ctx.form = noise, "box"
            ctx.save_for_backward(mp, contrast, bright, affine, roi)
        elif sparse:
            raise ValueError("_Warp: a sparse composite needs keyed noise, footprint boxes, form 'box' and S % 4 == 0")
        elif keyed and roi is not None and form == "pre":
            seed, counter, b0 = noise
            pre = torch.empty(B, 3, P, P, device=mp.device)
            nat.call("po_augment_patch", nat.ptr(mp), int(seed) & 0xFFFFFFFFFFFFFFFF, int(counter) & 0xFFFFFFFFFFFFFFFF,
                     int(b0), nat.ptr(contrast), nat.ptr(bright), B, P, nat.ptr(pre), nat.stream())
            nat.call("po_warp_fwd_pre", imgp, nat.ptr(pre), nat.ptr(affine, torch.float64), nat.ptr(roi, torch.int32),
                     B, S, P, mode, nat.ptr(out), nat.stream())
            ctx.key, ctx.form = noise, "pre"
            ctx.save_for_backward(mp, contrast, bright, affine, pre, roi)
        elif keyed:
            seed, counter, b0 = noise
            nat.call("po_warp_fwd_keyed", imgp, nat.ptr(mp), int(seed) & 0xFFFFFFFFFFFFFFFF,
                     int(counter) & 0xFFFFFFFFFFFFFFFF, int(b0), nat.ptr(contrast), nat.ptr(bright),
                     nat.ptr(affine, torch.float64), B, S, P, mode, nat.ptr(out), nat.stream())
            ctx.key, ctx.form = noise, "frame"
            ctx.save_for_backward(mp, contrast, bright, affine)
        else:
            nat.call("po_warp_fwd", imgp, nat.ptr(mp), nat.ptr(noise), nat.ptr(contrast), nat.ptr(bright),
                     nat.ptr(affine, torch.float64), B, S, P, mode, nat.ptr(out), nat.stream())
            ctx.key = None
            ctx.save_for_backward(mp, contrast, bright, affine, noise)
        ctx.S, ctx.mode = S, mode
        return out

    @staticmethod
    def backward(ctx, d_out):
        mp, contrast, bright, affine = ctx.saved_tensors[:4]
        d_out = d_out.contiguous()
        B, P = affine.size(0), mp.size(-1)
        d_mp = torch.empty_like(mp)
        key = tuple(int(v) & 0xFFFFFFFFFFFFFFFF for v in ctx.key[:2]) + (int(ctx.key[2]),) if ctx.key else None
        if ctx.form == "box" and ctx.fac is not None:
            roi = ctx.saved_tensors[4]
            fac, ctx.fac = ctx.fac, None                 # consumed in place
            nat.call("po_warp_box_bwd_fac", nat.ptr(d_out), nat.ptr(mp), *key, nat.ptr(contrast), nat.ptr(bright),
                     nat.ptr(affine, torch.float64), nat.ptr(roi, torch.int32), B, ctx.S, P, nat.ptr(fac),
                     nat.ptr(d_mp), nat.stream())
            return d_mp, None, None, None, None, None, None, None, None, None, None, None
        # the footprint-box forms keep their per-pixel factors interleaved [B,S,S,4]
        work = (torch.empty(B * ctx.S * ctx.S * 4, device=d_out.device) if ctx.form in ("box", "pre")
                else torch.empty_like(d_out))
        if ctx.form == "box":
            roi = ctx.saved_tensors[4]
            nat.call("po_warp_box_bwd_keyed", nat.ptr(d_out), nat.ptr(mp), *key, nat.ptr(contrast), nat.ptr(bright),
                     nat.ptr(affine, torch.float64), nat.ptr(roi, torch.int32), B, ctx.S, P, ctx.mode, nat.ptr(work),
                     nat.ptr(d_mp), nat.stream())
        elif ctx.form == "pre":
            pre, roi = ctx.saved_tensors[4:6]
            nat.call("po_warp_bwd_pre", nat.ptr(d_out), nat.ptr(pre), nat.ptr(contrast), nat.ptr(affine, torch.float64),
                     nat.ptr(roi, torch.int32), B, ctx.S, P, ctx.mode, nat.ptr(work), nat.ptr(d_mp), nat.stream())
        elif ctx.form == "frame":
            nat.call("po_warp_bwd_keyed", nat.ptr(d_out), nat.ptr(mp), *key, nat.ptr(contrast), nat.ptr(bright),
                     nat.ptr(affine, torch.float64), B, ctx.S, P, ctx.mode, nat.ptr(work), nat.ptr(d_mp),
                     nat.stream())
        else:
            noise = ctx.saved_tensors[4]
            nat.call("po_warp_bwd", nat.ptr(d_out), nat.ptr(mp), nat.ptr(noise), nat.ptr(contrast),
                     nat.ptr(bright), nat.ptr(affine, torch.float64), B, ctx.S, P, ctx.mode,
                     nat.ptr(work), nat.ptr(d_mp), nat.stream())
        return d_mp, None, None, None, None, None, None, None, None, None, None, None


class PatchTransformer(nn.Module):
    """Training-time patch transformer (load_data.py:414-794): median pool,
    contrast U(0.8,1.2), brightness U(-0.1,0.1), noise 0.1*U(-1,1), clamp,
    random rotation U(-pi,pi), scale from the selected label (cols 2,3 — Q2),
    random centre (max(U,0.2), min(U,0.8) — Q4), bilinear affine warp,
    clamp * mask."""

    def __init__(self):
        super().__init__()
        self.min_contrast = 0.8
        self.max_contrast = 1.2
        self.min_brightness = -0.1
        self.max_brightness = 0.1
        self.noise_factor = NOISE_FACTOR
        self.minangle = -180 / 180 * math.pi
        self.maxangle = 180 / 180 * math.pi
        self.medianpooler = MedianPool2d(7, same=True)
        # on-device counter-based draws (po_draws): key, step counter, and the
        # global index of this process's first image (data-parallel shards)
        self.draw_seed = 3
        self.draw_step = 0
        self.draw_b0 = 0
        self.keyed_noise = os.environ.get("ADVPATCH_NOISE_KEYED", "1") != "0"
        # warp kernels for keyed noise (_Warp.forward): "box" (default), "pre", "frame"
        self.warp_form = os.environ.get("ADVPATCH_WARP", "box")
        if self.warp_form not in WARP_FORMS:
            raise ValueError("ADVPATCH_WARP must be one of %s" % (WARP_FORMS,))
        self.last_roi = None     # [B,4] int32 footprint boxes of the last placement
        # placement arithmetic: "ref" (the reference's fp32 ops) or "f64" (ADVPATCH_GEOMETRY)
        self.geometry = default_geometry()

    def lab_transform(self, lab_batch_origin):
        """[B,L,5] -> [B,1,5] (load_data.py:453-478): (max-area row + min-area row)/2,
        or 0.25 everywhere when the max area exceeds 0.99."""
        area = lab_batch_origin[:, :, 3] * lab_batch_origin[:, :, 4]
        imax = torch.argmax(area, 1)
        imin = torch.argmin(area, 1)
        ar = torch.arange(lab_batch_origin.size(0), device=lab_batch_origin.device)
        sel = (lab_batch_origin[ar, imax, :] + lab_batch_origin[ar, imin, :]) / 2.
        empty = area.max(1).values > 0.99
        sel = torch.where(empty[:, None], torch.full_like(sel, 0.25), sel)
        return sel.unsqueeze(1)

    def make_draws(self, B, P, device):
        """This step's draws for images draw_b0 .. draw_b0+B-1 of the global
        batch; advances the step counter.  With ``keyed_noise`` (default;
        ADVPATCH_NOISE_KEYED=0: off) the noise is not drawn: ``noise_key``
        (seed, step, b0) lets the warp kernels regenerate po_draws' values."""
        if self.keyed_noise:
            d = synthetic.draws_device(self.draw_seed, self.draw_step, self.draw_b0, B, P, device,
                                       keys=tuple(k for k in synthetic.DRAW_KEYS if k != "noise"))
            d["noise_key"] = (self.draw_seed, self.draw_step, self.draw_b0)
        else:
            d = synthetic.draws_device(self.draw_seed, self.draw_step, self.draw_b0, B, P, device)
        self.draw_step += 1
        return d

    @staticmethod
    def _noise(d):
        return d["noise"].contiguous() if "noise" in d else d["noise_key"]

    def _prep(self, adv_patch, lab_batch, img_size, do_rotate, draws, mp=None):
        nat.ensure_device(adv_patch)
        if mp is None:
            # load_data.py:531-532 (squeeze: a view, so its backward is no kernel)
            mp = self.medianpooler(adv_patch.unsqueeze(0)).squeeze(0)
        B, P = lab_batch.size(0), mp.size(-1)
        if draws is None:
            draws = self.make_draws(B, P, adv_patch.device)
        theta, center, _, roi, affine = patch_params(lab_batch, img_size, P, draws, do_rotate, with_roi=True,
                                                     geometry=self.geometry)
        self.last_roi = roi
        return mp, draws, affine, center

    def forward(self, adv_patch, lab_batch, img_size, do_rotate=True, rand_loc=False, draws=None):
        """-> (adv_batch_t [B,1,3,S,S], patch_center [B,2] = (x*S, y*S))."""
        mp, d, affine, center = self._prep(adv_patch, lab_batch, img_size, do_rotate, draws)
        out = _Warp.apply(mp, self._noise(d), d["contrast"].contiguous(),
                          d["bright"].contiguous(), affine, None, int(img_size), 0, self.warp_form, self.last_roi,
                          False, torch.is_grad_enabled() and mp.requires_grad)
        return out.unsqueeze(1), center

    def forward_composite(self, adv_patch, lab_batch, img_batch, img_size, do_rotate=True, draws=None,
                          sparse=False, mp=None):
        """Fused PatchTransformer + PatchApplier (the training step's path):
        -> (p_img_batch [B,3,S,S], patch_center [B,2]) without materialising
        adv_batch_t.  ``sparse`` (keyed draws, form "box", S % 4 == 0): only
        the quad-widened footprint boxes of p_img_batch (``last_roi``) are
        written; the composite equals img_batch elsewhere, and Darknet.
        forward_nhwc(p_img, roi, center, base=img_batch) reads it that way.
        ``mp``: the median-pooled patch when the caller already has it
        (patch_front)."""
        mp, d, affine, center = self._prep(adv_patch, lab_batch, img_size, do_rotate, draws, mp)
        out = _Warp.apply(mp, self._noise(d), d["contrast"].contiguous(),
                          d["bright"].contiguous(), affine, img_batch.contiguous(), int(img_size), 1, self.warp_form,
                          self.last_roi, sparse, torch.is_grad_enabled() and mp.requires_grad)
        return out, center

    def sparse_ok(self, img_size, draws=None):
        """Whether forward_composite(..., sparse=True) is available."""
        keyed = (draws is None and self.keyed_noise) or (draws is not None and "noise" not in draws)
        return keyed and self.warp_form == "box" and int(img_size) % 4 == 0


class _Apply(torch.autograd.Function):
    @staticmethod
    def forward(ctx, img, adv):
        nat.ensure_device(adv)
        img, adv = img.contiguous(), adv.contiguous()
        out = torch.empty_like(adv)
        nat.call("po_apply_fwd", nat.ptr(img), nat.ptr(adv), adv.numel(), nat.ptr(out), nat.stream())
        ctx.save_for_backward(adv)
        return out

    @staticmethod
    def backward(ctx, d_out):
        (adv,) = ctx.saved_tensors
        d_out = d_out.contiguous()
        d_img = torch.empty_like(d_out) if ctx.needs_input_grad[0] else None
        d_adv = torch.empty_like(d_out) if ctx.needs_input_grad[1] else None
        nat.call("po_apply_bwd", nat.ptr(d_out), nat.ptr(adv), adv.numel(), nat.ptr(d_img),
                 nat.ptr(d_adv), nat.stream())
        return d_img, d_adv


class PatchApplier(nn.Module):
    """img = where(adv == 0, img, adv) for every patch slot (load_data.py:808-833)."""

    def forward(self, img_batch, adv_batch):
        for adv in torch.unbind(adv_batch, 1):
            if img_batch.shape != adv.shape:
                img_batch = img_batch.expand_as(adv)
            img_batch = _Apply.apply(img_batch, adv)
        return img_batch


# ---------------------------------------------------------------------------
# Test-time placements (load_data.py:985-1722)
# ---------------------------------------------------------------------------
PLACE_FLAG_MASK, PLACE_FLAG_NOFREE, PLACE_FLAG_PICK = 1, 2, 4
PLACE_INFO = ("flags", "x", "y", "semi_edge2", "M", "n_free", "pick", "mask_ones")


def _place_workspace(B, L, S, dev):
    fw, iw = nat.c_int64(), nat.c_int64()
    nat.call("po_place_workspace", B, L, S, nat.ctypes.byref(fw), nat.ctypes.byref(iw))
    return (torch.empty(fw.value, device=dev), torch.empty(iw.value, dtype=torch.int32, device=dev))


def _label_rows(lab_batch, nlab, ncols):
    nat.ensure_device(lab_batch)
    lab = lab_batch.contiguous().float()
    if lab.dim() != 3 or lab.size(2) != ncols:
        raise ValueError("expected labels [B, L, %d], got %s" % (ncols, tuple(lab.shape)))
    B, L = lab.size(0), lab.size(1)
    if L < 1:
        raise RuntimeError("no label rows (the reference's torch.max over an empty label set fails)")
    if nlab is None:
        nlab = torch.full((B,), L, dtype=torch.int32, device=lab.device)
    else:
        nlab = torch.as_tensor(nlab, dtype=torch.int32).to(lab.device)
    return lab, nlab


def place_test_mode(mp, lab_batch, img_size, angle, upick, nlab=None, scale_factor=SCALE_FACTOR):
    """po_place_test_mode: median-pooled patch [3,P,P], labels [B,L,7] (the
    first nlab[b] rows used; all L by default), angle / upick [B] ->
    (out [B,3,S,S], info [B,8] int32 with the PLACE_INFO fields)."""
    nat.ensure_device(mp)
    lab, nlab = _label_rows(lab_batch, nlab, 7)
    B, L, S, P = lab.size(0), lab.size(1), int(img_size), mp.size(-1)
    dev = lab.device
    fw, iw = _place_workspace(B, L, S, dev)
    out = torch.empty(B, 3, S, S, device=dev)
    info = torch.empty(B, 8, dtype=torch.int32, device=dev)
    nat.call("po_place_test_mode", nat.ptr(mp.contiguous()), P, nat.ptr(lab), nat.ptr(nlab, torch.int32), B, L, S,
             float(scale_factor), nat.ptr(None if angle is None else angle.contiguous().float()),
             nat.ptr(upick.contiguous().float()), nat.ptr(fw), nat.ptr(iw, torch.int32), nat.ptr(out),
             nat.ptr(info, torch.int32), nat.stream())
    return out, info


def check_place_info(info):
    """Raise as the reference does on the conditions po_place_test_mode flags."""
    for b, row in enumerate(info.cpu().tolist()):
        f = row[0]
        if f & PLACE_FLAG_MASK:
            raise RuntimeError("image %d: fewer than two mask==1 pixels after scale/rotate (the reference fails in "
                               "torch.min / the squeeze, load_data.py:1655-1662)" % b)
        if f & PLACE_FLAG_NOFREE:
            raise IndexError("image %d: no free position (position_available is empty, load_data.py:1684)" % b)
        if f & PLACE_FLAG_PICK:
            raise IndexError("image %d: random.randint(0, %d) drew %d == len(position_available) "
                             "(load_data.py:1682-1684)" % (b, row[5], row[6]))


class PatchTransformer_test_mode(nn.Module):
    """Test-time placement that avoids the detections (load_data.py:1233-1722):
    scale from the (max-area + min-area)/2 detection, rotation (U(-pi/2, pi/2)
    with test_mode=True, else U(-pi, pi)), the inter_axis_cal occupancy map,
    a random free position, translation there.  The contrast/brightness/noise
    the reference draws are not applied (1464-1490), so they are not drawn.

    lab_batch [B, n, 7] rows {x, y, w, h, obj_conf, cls_conf, id} (the
    0.01-threshold detections, 1295-1297); the reference runs B = 1.  Every
    image uses all n rows unless ``nlab`` [B] gives per-image counts.
    Randomness: ``draws`` = {"angle": [B], "upick": [B]} or the on-device
    counter-based draws (po_draws, seed ``draw_seed``, counter ``draw_step``).
    """

    def __init__(self, test_mode=False):
        super().__init__()
        self.min_contrast = 0.8
        self.max_contrast = 1.2
        self.min_brightness = -0.1
        self.max_brightness = 0.1
        self.noise_factor = NOISE_FACTOR
        self.minangle = -180 / 180 * math.pi
        self.maxangle = 180 / 180 * math.pi
        if test_mode:                                     # load_data.py:1254-1259
            self.maxangle = 90 / 180 * math.pi
            self.minangle = -90 / 180 * math.pi
        self.test_mode = bool(test_mode)
        self.medianpooler = MedianPool2d(7, same=True)
        self.draw_seed = 5
        self.draw_step = 0
        self.last_info = None

    def lab_transform(self, lab_batch_origin):
        """[B,n,7] -> [B,1,7] (load_data.py:1262-1320): (max-area row +
        min-area row)/2 over cols 2,3; 0.25 everywhere for a single row or a
        max area above 0.99."""
        area = lab_batch_origin[:, :, 2] * lab_batch_origin[:, :, 3]
        imax, imin = torch.argmax(area, 1), torch.argmin(area, 1)
        ar = torch.arange(lab_batch_origin.size(0), device=lab_batch_origin.device)
        sel = (lab_batch_origin[ar, imax, :] + lab_batch_origin[ar, imin, :]) / 2.
        flat = (area.max(1).values > 0.99) | torch.tensor(lab_batch_origin.size(1) == 1, device=area.device)
        sel = torch.where(flat[:, None], torch.full_like(sel, 0.25), sel)
        return sel.unsqueeze(1)

    def inter_axis_cal(self, lab_batch, semi_edge, img_size, nlab=None):
        """The occupancy map of load_data.py:1322-1430 (po_place_free_map):
        [S,S] (lab_batch [1,n,7]) or [B,S,S], indexed [x][y] as the
        reference's; 0 exactly where the reference's map is 0 (its layer
        counts are not reproduced: only its zeros are read, 1678)."""
        lab, nlab = _label_rows(lab_batch if lab_batch.dim() == 3 else lab_batch.unsqueeze(0), nlab, 7)
        B, L, S = lab.size(0), lab.size(1), int(img_size)
        semi = torch.as_tensor(semi_edge, dtype=torch.float32).reshape(-1).to(lab.device)
        if semi.numel() == 1 and B > 1:
            semi = semi.expand(B).contiguous()
        fw, iw = _place_workspace(B, L, S, lab.device)
        layout = torch.empty(B, S, S, dtype=torch.int32, device=lab.device)
        nat.call("po_place_free_map", nat.ptr(lab), nat.ptr(nlab, torch.int32), B, L, S, nat.ptr(semi), nat.ptr(fw),
                 nat.ptr(iw, torch.int32), nat.ptr(layout, torch.int32), nat.stream())
        return layout[0] if lab_batch.size(0) == 1 else layout

    def make_draws(self, B, device):
        d = synthetic.draws_device(self.draw_seed, self.draw_step, 0, B, 1, device, keys=("angle", "ux"))
        self.draw_step += 1
        # po_draws' angle is U(-pi, pi); test_mode halves it (exact) to U(-pi/2, pi/2)
        angle = d["angle"] * 0.5 if self.test_mode else d["angle"]
        return {"angle": angle, "upick": d["ux"]}

    def forward(self, adv_patch, lab_batch, img_size, do_rotate=True, rand_loc=False, draws=None, nlab=None):
        """-> adv_patch_mask [B, 1, 3, S, S] (load_data.py:1432-1722).  Raises
        where the reference raises (see check_place_info); ``rand_loc`` is
        accepted and unused, as in the reference."""
        nat.ensure_device(adv_patch)
        mp = self.medianpooler(adv_patch.unsqueeze(0))[0]                 # load_data.py:1451-1452
        if draws is None:
            draws = self.make_draws(lab_batch.size(0), adv_patch.device)
        angle = draws["angle"] if do_rotate else None
        out, info = place_test_mode(mp, lab_batch, img_size, angle, draws["upick"], nlab=nlab)
        self.last_info = info
        check_place_info(info)
        return out.unsqueeze(1)


class PatchTransformer_vanishing(nn.Module):
    """One patch per label row (load_data.py:985-1230): contrast/brightness/
    noise (not with test_real), clamp, rotation U(-pi, pi), size
    sqrt((w S/8)^2 + (h S/8)^2), centre at the label (+-0.2 w/h with
    rand_loc, -+w/6 with orient "left"/"right"), single-stage theta, clamp *
    mask.  lab_batch [B, n, 5] rows {cls, x, y, w, h}.

    ``forward`` returns the reference's [B, n, 3, S, S] (po_vanishing_params
    + po_warp_fwd over the B*n patches; differentiable in adv_patch);
    ``forward_composite`` fuses the PatchApplier loop over the n slots
    (po_warp_composite_multi) without materialising them (evaluation only).
    Randomness as PatchTransformer (po_draws over the B*n patches)."""

    PRE_SCALE = 8.0                                       # load_data.py:1116

    def __init__(self):
        super().__init__()
        self.min_contrast = 0.8
        self.max_contrast = 1.2
        self.min_brightness = -0.1
        self.max_brightness = 0.1
        self.noise_factor = NOISE_FACTOR
        self.minangle = -180 / 180 * math.pi
        self.maxangle = 180 / 180 * math.pi
        self.medianpooler = MedianPool2d(7, same=True)
        self.draw_seed = 7
        self.draw_step = 0

    def make_draws(self, n, P, device):
        d = synthetic.draws_device(self.draw_seed, self.draw_step, 0, n, P, device)
        self.draw_step += 1
        return d

    def _prep(self, adv_patch, lab_batch, img_size, do_rotate, rand_loc, orient, test_real, draws):
        nat.ensure_device(adv_patch)
        lab, _ = _label_rows(lab_batch, None, 5)
        mp = self.medianpooler(adv_patch.unsqueeze(0))[0]                 # load_data.py:1041-1042
        B, L, S, P = lab.size(0), lab.size(1), int(img_size), mp.size(-1)
        if draws is None:
            draws = self.make_draws(B * L, P, adv_patch.device)
        dev = adv_patch.device
        if orient not in (None, "left", "right"):
            orient_code = 0                               # any other value: no shift (load_data.py:1158-1162)
        else:
            orient_code = {None: 0, "left": 1, "right": 2}[orient]
        angle = draws["angle"].contiguous().float() if do_rotate else None
        offx = offy = None
        if rand_loc:                                      # U(-0.2, 0.2) from the U[0,1) draws
            offx = (draws["ux"].double() * 0.4 - 0.2).float().contiguous()
            offy = (draws["uy"].double() * 0.4 - 0.2).float().contiguous()
        affine = torch.empty(B * L, 6, dtype=torch.float64, device=dev)
        roi = torch.empty(B * L, 4, dtype=torch.int32, device=dev)
        nat.call("po_vanishing_params", nat.ptr(lab), B, L, S, P, float(self.PRE_SCALE), nat.ptr(angle),
                 nat.ptr(offx), nat.ptr(offy), orient_code, nat.ptr(affine, torch.float64), nat.ptr(roi, torch.int32),
                 nat.stream())
        if test_real:                                     # load_data.py:1070-1071: no augmentation
            aug = None
        else:
            aug = (draws["noise"].contiguous().float(), draws["contrast"].contiguous().float(),
                   draws["bright"].contiguous().float())
        return mp, aug, affine, roi, (B, L, S, P)

    def forward(self, adv_patch, lab_batch, img_size, do_rotate=True, rand_loc=False, orient=None,
                test_real=False, draws=None):
        mp, aug, affine, roi, (B, L, S, P) = self._prep(adv_patch, lab_batch, img_size, do_rotate, rand_loc,
                                                        orient, test_real, draws)
        if aug is None:
            dev = mp.device
            aug = (torch.zeros(B * L, 3, P, P, device=dev), torch.ones(B * L, device=dev),
                   torch.zeros(B * L, device=dev))
        out = _Warp.apply(mp, aug[0], aug[1], aug[2], affine, None, S, 0)
        return out.view(B, L, 3, S, S)

    def forward_composite(self, adv_patch, lab_batch, img_batch, img_size, do_rotate=True, rand_loc=False,
                          orient=None, test_real=False, draws=None):
        """PatchApplier(img_batch, forward(...)) in one pass (no autograd)."""
        mp, aug, affine, roi, (B, L, S, P) = self._prep(adv_patch, lab_batch, img_size, do_rotate, rand_loc,
                                                        orient, test_real, draws)
        img = img_batch.contiguous().float()
        if tuple(img.shape) != (B, 3, S, S):
            raise ValueError("img_batch must be [%d,3,%d,%d], got %s" % (B, S, S, tuple(img.shape)))
        out = torch.empty_like(img)
        noise, contrast, bright = aug if aug is not None else (None, None, None)
        nat.call("po_warp_composite_multi", nat.ptr(img), nat.ptr(mp.detach().contiguous()), nat.ptr(noise),
                 nat.ptr(contrast), nat.ptr(bright), nat.ptr(affine, torch.float64), nat.ptr(roi, torch.int32), B, L,
                 S, P, nat.ptr(out), nat.stream())
        return out


# ---------------------------------------------------------------------------
# Host data path (load_data.py:859-978)
# ---------------------------------------------------------------------------
class DotaDataset(torch.utils.data.Dataset):
    """DOTA-style image/label folder: square grey-127 pad, bilinear resize to
    ``imgsize``, labels ``cls x y w h`` normalised and padded to ``max_lab``
    rows with 1e-6; an empty label file becomes one row of ones(5)."""

    def __init__(self, img_dir, lab_dir, max_lab, imgsize, shuffle=True, as_uint8=False):
        names = fnmatch.filter(os.listdir(img_dir), "*.png") + fnmatch.filter(os.listdir(img_dir), "*.jpg")
        n_labels = len(fnmatch.filter(os.listdir(lab_dir), "*.txt"))
        assert len(names) == n_labels, "Number of images and number of labels does't match"
        self.len = len(names)
        self.img_dir, self.lab_dir, self.imgsize = img_dir, lab_dir, imgsize
        self.img_names = names
        self.shuffle = shuffle
        self.img_paths = [os.path.join(img_dir, n) for n in names]
        self.lab_paths = [os.path.join(lab_dir, n).replace(".jpg", ".txt").replace(".png", ".txt") for n in names]
        self.max_n_labels = max_lab
        # as_uint8: images come out as uint8 [3,S,S] (a quarter of the bytes through the
        # worker queues, pinning and the PCIe copy); DevicePrefetcher / FrameCache turn
        # them into ToTensor's floats on the device (u8_to_float)
        self.as_uint8 = as_uint8

    def __len__(self):
        return self.len

    def __getitem__(self, idx):
        from PIL import Image
        assert idx <= len(self), "index range error"
        image = Image.open(self.img_paths[idx]).convert("RGB")
        lab_path = self.lab_paths[idx]
        if os.path.getsize(lab_path):
            label = np.loadtxt(lab_path)
        else:
            label = np.ones([5])
        label = torch.from_numpy(label).float()
        if label.dim() == 1:
            label = label.unsqueeze(0)
        image, label = self.pad_and_scale(image, label)
        image = torch.from_numpy(np.asarray(image, dtype=np.uint8).copy()).permute(2, 0, 1)
        if not self.as_uint8:
            image = image.float().div_(255.0)
        else:
            image = image.contiguous()
        return image, self.pad_lab(label)

    def pad_and_scale(self, img, lab):
        from PIL import Image
        w, h = img.size
        if w == h:
            padded = img
        elif w < h:
            padding = (h - w) / 2
            padded = Image.new("RGB", (h, h), color=(127, 127, 127))
            padded.paste(img, (int(padding), 0))
            lab[:, [1]] = (lab[:, [1]] * w + padding) / h
            lab[:, [3]] = (lab[:, [3]] * w / h)
        else:
            padding = (w - h) / 2
            padded = Image.new("RGB", (w, w), color=(127, 127, 127))
            padded.paste(img, (0, int(padding)))
            lab[:, [2]] = (lab[:, [2]] * h + padding) / w
            lab[:, [4]] = (lab[:, [4]] * h / w)
        padded = padded.resize((self.imgsize, self.imgsize), Image.BILINEAR)
        return padded, lab

    def pad_lab(self, lab):
        pad_size = self.max_n_labels - lab.shape[0]
        if pad_size > 0:
            return F.pad(lab, (0, 0, 0, pad_size), value=1e-6)
        return lab


_U8_LUT = {}


def u8_to_float(img):
    """uint8 -> float32 / 255 exactly as ToTensor computes it on the host.
    (On the GPU ``x.float() / 255.0`` is x * (1/255), which differs from the
    host's correctly rounded division in the last bit for some values: the
    256 host-computed quotients are gathered instead.)"""
    lut = _U8_LUT.get(img.device)
    if lut is None:
        lut = torch.arange(256, dtype=torch.uint8).float().div_(255.0).to(img.device)
        _U8_LUT[img.device] = lut
    return lut[img.long()]


class DotaCollate:
    """DataLoader collate of DotaDataset items that also forms the EMPTY batch
    of a rank whose shard of a ragged last global batch is empty
    (GlobalBatchSampler): uint8/float [0,3,S,S] frames and [0,L,5] labels."""

    def __init__(self, imgsize, max_n_labels, as_uint8=False):
        self.S, self.L, self.u8 = int(imgsize), int(max_n_labels), bool(as_uint8)

    def __call__(self, batch):
        if not batch:
            return (torch.empty(0, 3, self.S, self.S, dtype=torch.uint8 if self.u8 else torch.float32),
                    torch.empty(0, self.L, 5))
        return torch.utils.data.default_collate(batch)


class DevicePrefetcher:
    """Host->device feed of the training loop (the reference copies each batch
    with a blocking ``.cuda()``, train_patch.py:164-166).  The copy of batch
    k+1 (pinned source, non-blocking, on a side stream) is issued before batch
    k is handed out, so it overlaps batch k's step instead of sitting between
    two steps on the compute stream; the compute stream waits on an event only
    when it takes the batch.  uint8 image batches (DotaDataset(as_uint8=True))
    become float32 / 255 on the device, bit-identical to ToTensor on the host
    (u8_to_float).  Batches that are already
    on the device pass through; without a GPU it only applies the conversion."""

    def __init__(self, loader, device):
        self.loader, self.device = loader, torch.device(device)

    def __len__(self):
        return len(self.loader)

    @staticmethod
    def _to_float(img):
        return u8_to_float(img) if img.dtype == torch.uint8 else img

    def __iter__(self):
        if self.device.type != "cuda":
            for img, lab in self.loader:
                yield self._to_float(img.to(self.device)), lab.to(self.device)
            return
        side = torch.cuda.Stream(self.device)
        main = torch.cuda.current_stream(self.device)
        it = iter(self.loader)

        def issue():
            try:
                img, lab = next(it)
            except StopIteration:
                return None
            side.wait_stream(main)        # buffers freed by earlier steps are reusable on the side stream
            with torch.cuda.stream(side):
                img = self._to_float(img.to(self.device, non_blocking=True))
                lab = lab.to(self.device, non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(side)
            return img, lab, ev

        nxt = issue()
        while nxt is not None:
            img, lab, ev = nxt
            main.wait_event(ev)
            img.record_stream(main)
            lab.record_stream(main)
            nxt = issue()
            yield img, lab



def loader_context(device):
    """multiprocessing context of the DataLoader workers: "spawn" when the
    device is a GPU (the parent has initialised HIP and runs its threads: a
    forked worker can inherit a lock one of them held and hang -- seen once on
    an MI355X box with two workers), else the platform default.
    ADVPATCH_LOADER_MP=fork|spawn|forkserver overrides.  Spawned workers
    re-import the package, not the caller's code (a script's training loop
    belongs under ``if __name__ == "__main__":``, as with any spawn loader)."""
    ctx = os.environ.get("ADVPATCH_LOADER_MP")
    if ctx is None:
        ctx = "spawn" if torch.device(device).type == "cuda" else None
    return ctx


class FrameCache:
    """Decoded training frames resident in device memory.  DotaDataset's
    transform (PNG decode, grey pad, bilinear resize, label padding;
    load_data.py:910-978) is deterministic and every augmentation happens later
    on the GPU (PatchTransformer), so each frame is decoded ONCE — by a
    DataLoader over the host workers — and kept as uint8 [N,3,S,S] plus float
    labels [N,L,5] in HBM (1.1 MB per 608x608 frame: a 20k-frame set is 22 GB of
    a MI355X's 288 GB).  Every epoch after that gathers its batches on the
    device (index_select + u8_to_float, the same floats as ToTensor), so the host
    decode rate (tens of frames/s per core) no longer bounds the step rate."""

    def __init__(self, dataset, device, num_workers=8, batch=32):
        ds = dataset
        if not getattr(ds, "as_uint8", False):
            raise ValueError("FrameCache needs DotaDataset(..., as_uint8=True)")
        self.device = torch.device(device)
        n, S, L = len(ds), ds.imgsize, ds.max_n_labels
        self.frames = torch.empty(n, 3, S, S, dtype=torch.uint8, device=self.device)
        self.labels = torch.empty(n, L, 5, dtype=torch.float32, device=self.device)
        dl = torch.utils.data.DataLoader(ds, batch_size=batch, shuffle=False, num_workers=num_workers,
                                         pin_memory=self.device.type == "cuda",
                                         multiprocessing_context=loader_context(self.device) if num_workers else None)
        k = 0
        for img, lab in dl:
            m = img.size(0)
            self.frames[k:k + m].copy_(img, non_blocking=True)
            self.labels[k:k + m].copy_(lab, non_blocking=True)
            k += m
        assert k == n
        if self.device.type == "cuda":
            torch.cuda.current_stream(self.device).synchronize()

    def __len__(self):
        return self.frames.size(0)

    def batch(self, indices):
        """(img [b,3,S,S] float32 in [0,1], lab [b,L,5]) of dataset rows ``indices``, on the device."""
        idx = torch.as_tensor(indices, dtype=torch.long).to(self.device, non_blocking=True)
        return u8_to_float(self.frames.index_select(0, idx)), self.labels.index_select(0, idx)

    def loader(self, batch_sampler):
        """Iterable of device batches in ``batch_sampler``'s order (a fresh pass per iter())."""
        cache = self

        class _It:
            def __len__(self):
                return len(batch_sampler)

            def __iter__(self):
                for b in batch_sampler:
                    yield cache.batch(b)
        return _It()
