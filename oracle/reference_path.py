"""PyTorch-CPU fp32 restatement of the reference's training hot path.

TEST INFRASTRUCTURE ONLY (see ``oracle/__init__.py``): imported by ``tests/``,
``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of ``bench.py``.

Every function follows the reference op for op, in the same float32 operation
order, and cites the reference ``file:line`` it restates (paths relative to
the reference repository root).  Randomness is passed in explicitly as a
``draws`` dict so the HIP path and this oracle see identical inputs:

    contrast [B]       U(0.8, 1.2)      load_data.py:548-557
    bright   [B]       U(-0.1, 0.1)     load_data.py:560-565
    noise    [B,3,P,P] U(-1, 1)         load_data.py:566-568 (x0.1 applied here)
    angle    [B]       U(-pi, pi)       load_data.py:607-614
    ux, uy   [B]       U[0, 1)          load_data.py:693-701 (CPU torch.rand)
"""
import math

import numpy as np
import torch
import torch.nn.functional as F

__all__ = [
    "parse_model_config", "median_pool7", "median_pool2d", "lab_transform", "patch_transformer",
    "patch_applier", "load_printability", "nps_score", "total_variation",
    "colorful_loss", "OracleDarknet", "read_darknet_weights", "obj_cls_conf_find",
    "no_obj_reshape", "no_cls_reshape", "no_obj_reshape3", "no_cls_reshape3", "noCLS_Loss_CE", "noCLS_loss_targeted",
    "train_step", "train_step_f64", "adam_amsgrad_steps", "patch_theta", "cell_indices", "TV_FACTOR", "NPS_FACTOR",
    "TARGET_ID", "bbox_decode", "max_prob_extractor",
]

# train_patch.py:25-28
TV_FACTOR = 2.5
NPS_FACTOR = 0.01
TARGET_ID = 14
# load_data.py:32
SCALE_FACTOR = 2.
# load_data.py:432-440 (active PatchTransformer parameters)
NOISE_FACTOR = 0.10


# --------------------------------------------------------------------------
# cfg.py:37-56 parse_model_config
# --------------------------------------------------------------------------
def parse_model_config(text):
    """Block list from darknet cfg text (cfg.py:37-56).  'batch_normalize'
    defaults to int 0 and is otherwise the raw string value (cfg.py:49-50)."""
    lines = [x for x in text.split("\n") if x and not x.startswith("#")]
    lines = [x.strip() for x in lines]
    defs = []
    for line in lines:
        if not line:
            continue
        if line.startswith("["):
            defs.append({"type": line[1:-1].rstrip()})
            if defs[-1]["type"] == "convolutional":
                defs[-1]["batch_normalize"] = 0
        else:
            key, value = line.split("=", 1)
            defs[-1][key.rstrip()] = value.strip()
    return defs


# --------------------------------------------------------------------------
# median_pool.py:19-52 MedianPool2d(7, same=True)
# --------------------------------------------------------------------------
# Tie rule of the median's backward.  "torch": torch.median's own index
# (implementation-defined when several window values equal the median, SURVEY
# Q8) — the reference.  "first": the first window position (row-major) that
# holds the median value — the rule po_median7 documents; tests of tied
# windows select it so both sides route the gradient identically.
MEDIAN_TIE_RULE = "torch"


def median_pool7(x, k=7):
    """reflect pad per `_padding` (median_pool.py:26-44: stride 1 -> ph=pw=k-1,
    split pl=pw//2, pr=pw-pl), 7x7 unfold, median over the 49 window values
    (median_pool.py:46-52)."""
    pw = max(k - 1, 0)
    pl, pr = pw // 2, pw - pw // 2
    xp = F.pad(x, (pl, pr, pl, pr), mode="reflect")
    win = xp.unfold(2, k, 1).unfold(3, k, 1)
    win = win.contiguous().view(win.size()[:4] + (-1,))
    if MEDIAN_TIE_RULE == "first":
        med = win.detach().median(dim=-1)[0]
        first = (win.detach() == med.unsqueeze(-1)).int().argmax(dim=-1, keepdim=True)
        return torch.gather(win, -1, first).squeeze(-1)
    return win.median(dim=-1)[0]


def median_pool2d(x, k, stride, padding):
    """MedianPool2d.forward for any configuration (median_pool.py:46-52):
    reflect pad (l, r, t, b), unfold, lower median; MEDIAN_TIE_RULE as above."""
    xp = F.pad(x, padding, mode="reflect")
    win = xp.unfold(2, k[0], stride[0]).unfold(3, k[1], stride[1])
    win = win.contiguous().view(win.size()[:4] + (-1,))
    if MEDIAN_TIE_RULE == "first":
        med = win.detach().median(dim=-1)[0]
        first = (win.detach() == med.unsqueeze(-1)).int().argmax(dim=-1, keepdim=True)
        return torch.gather(win, -1, first).squeeze(-1)
    return win.median(dim=-1)[0]


# --------------------------------------------------------------------------
# load_data.py:453-478 PatchTransformer.lab_transform
# --------------------------------------------------------------------------
def lab_transform(lab_batch):
    B = lab_batch.size(0)
    sel = torch.zeros(B, 1, 5, dtype=lab_batch.dtype)
    area = lab_batch[:, :, 3] * lab_batch[:, :, 4]
    max_value, max_index = torch.max(area, 1)
    _, min_index = torch.min(area, 1)
    for i in range(B):
        if max_value[i] > 0.99:
            sel[i, :, :] = torch.tensor([0.25, 0.25, 0.25, 0.25, 0.25])
        else:
            sel[i, :, :] = (lab_batch[i, max_index[i], :] + lab_batch[i, min_index[i], :]) / 2.
    return sel


# --------------------------------------------------------------------------
# load_data.py:512-794 PatchTransformer.forward (training placement)
# --------------------------------------------------------------------------
def patch_transformer(adv_patch, lab_batch, img_size, draws, do_rotate=True, geometry="fp32"):
    """Returns (adv_batch_t [B,1,3,S,S], patch_center [B,2]).  patch_center is
    (column, row) in pixels = (target_x*S, target_y*S) (load_data.py:712-715).

    ``geometry`` (tests only): "fp32" is the reference (theta, affine_grid and
    grid_sample in the inputs' dtype: fp32 for the reference itself).  "f64"
    evaluates theta, the grid and the bilinear sampling in float64 from the
    same fp32 inputs and rounds each sampled value to fp32 once (the HIP
    path's opt-in float64 geometry, ADVPATCH_GEOMETRY=f64).  "fp32in64" (for
    float64 runs, train_step_f64): the reference's fp32 sample points --
    theta, the affine grid and grid_sample's unnormalisation exactly as the
    fp32 reference computes them (from the fp32 labels and draws) -- with the
    bilinear weights, the sampling and everything after it in the batch's
    dtype: the accuracy yardstick of an implementation that reproduces the
    reference's fp32 sample points (the HIP default, po_patch_params
    geometry 1/2)."""
    adv = median_pool7(adv_patch.unsqueeze(0))                    # 531-532
    P = adv.size(-1)
    pad = (img_size - P) / 2                                     # 534
    adv = adv.unsqueeze(0)                                       # 536
    B = lab_batch.size(0)
    adv_batch = adv.expand(B, 1, -1, -1, -1)                     # 537-538
    contrast = draws["contrast"].view(B, 1, 1, 1, 1).expand(-1, -1, 3, P, P)   # 548-557
    brightness = draws["bright"].view(B, 1, 1, 1, 1).expand(-1, -1, 3, P, P)  # 560-565
    noise = draws["noise"].view(B, 1, 3, P, P) * NOISE_FACTOR    # 566-568
    adv_batch = adv_batch * contrast + brightness + noise        # 571
    adv_batch = torch.clamp(adv_batch, 0.0, 1.)                  # 574
    msk_batch = torch.ones_like(adv_batch)                       # 598
    padl, padr = int(pad + 0.5), int(pad)
    adv_batch = F.pad(adv_batch, (padl, padr, padl, padr), value=0.)   # 601-604
    msk_batch = F.pad(msk_batch, (padl, padr, padl, padr), value=0.)   # 605
    if do_rotate:                                                # 607-614
        angle = draws["angle"].clone()
    else:
        angle = torch.zeros(B)
    sel = lab_transform(lab_batch)                               # 624
    lab_scaled = torch.zeros(B, 1, 5)
    for c in range(4):                                           # 648-655
        lab_scaled[:, :, c] = sel[:, :, c] * img_size
    target_size = torch.sqrt(((lab_scaled[:, :, 2].mul(1 / SCALE_FACTOR)) ** 2) +
                             ((lab_scaled[:, :, 3].mul(1 / SCALE_FACTOR)) ** 2))   # 662-668
    target_x = draws["ux"].clone().view(B)                        # 693-696
    target_y = draws["uy"].clone().view(B)                        # 700-702
    target_x = torch.max(target_x, torch.tensor(0.2))            # 703
    target_y = torch.min(target_y, torch.tensor(0.8))            # 706
    patch_center = torch.cat([(target_x * img_size).view(-1, 1),
                              (target_y * img_size).view(-1, 1)], 1)   # 712-715
    scale = (target_size / P).view(B)                            # 717-718
    s = adv_batch.size()
    adv_batch = adv_batch.reshape(s[0] * s[1], s[2], s[3], s[4])
    msk_batch = msk_batch.reshape(s[0] * s[1], s[2], s[3], s[4])
    if geometry == "f64":
        adv_batch, msk_batch = adv_batch.double(), msk_batch.double()
        angle, target_x, target_y, scale = angle.double(), target_x.double(), target_y.double(), scale.double()
    tx = (-target_x + 0.5) * 2                                   # 726
    ty = (-target_y + 0.5) * 2                                   # 727
    sin = torch.sin(angle)
    cos = torch.cos(angle)
    theta = torch.zeros(B, 2, 3, dtype=adv_batch.dtype)          # 733-743
    theta[:, 0, 0] = cos / scale
    theta[:, 0, 1] = sin / scale
    theta[:, 0, 2] = tx * cos / scale + ty * sin / scale
    theta[:, 1, 0] = -sin / scale
    theta[:, 1, 1] = cos / scale
    theta[:, 1, 2] = -tx * sin / scale + ty * cos / scale
    if geometry == "fp32in64":
        # the reference's own fp32 theta and grid (same ops, fp32 inputs), then the
        # fp32 sample points grid_sample takes from it (geometry_ref.unnormalize32),
        # handed to the float64 sampler as the float64 grid that lands on them
        from .geometry_ref import unnormalize32
        th32, _, _ = patch_theta(lab_batch.float(), img_size, P, {k: v.float() for k, v in draws.items()},
                                 do_rotate)
        g32 = F.affine_grid(th32, adv_batch.shape, align_corners=False).numpy()
        Hs, Ws = adv_batch.size(-2), adv_batch.size(-1)
        ix = unnormalize32(g32[..., 0], Ws).astype(np.float64)
        iy = unnormalize32(g32[..., 1], Hs).astype(np.float64)
        grid = torch.from_numpy(np.stack([(2.0 * ix + 1.0) / Ws - 1.0, (2.0 * iy + 1.0) / Hs - 1.0], -1)).to(
            adv_batch.dtype)
    else:
        grid = F.affine_grid(theta, adv_batch.shape, align_corners=False)  # 745
    adv_t = F.grid_sample(adv_batch, grid, align_corners=False)            # 748
    msk_t = F.grid_sample(msk_batch, grid, align_corners=False)            # 749
    adv_t = adv_t.view(s[0], s[1], s[2], s[3], s[4])
    msk_t = msk_t.view(s[0], s[1], s[2], s[3], s[4])
    adv_t = torch.clamp(adv_t, 0.0, 1.)                          # 791
    out = adv_t * msk_t                                          # 792-794
    if geometry == "f64":
        out = out.float()
    return out, patch_center


def patch_theta(lab_batch, img_size, P, draws, do_rotate=True):
    """The per-image affine parameters of patch_transformer (for tests)."""
    B = lab_batch.size(0)
    angle = draws["angle"].clone() if do_rotate else torch.zeros(B, dtype=lab_batch.dtype)
    sel = lab_transform(lab_batch)
    ls2 = sel[:, :, 2] * img_size
    ls3 = sel[:, :, 3] * img_size
    target_size = torch.sqrt((ls2.mul(0.5)) ** 2 + (ls3.mul(0.5)) ** 2)
    tx_ = torch.max(draws["ux"].clone().view(B), torch.tensor(0.2))
    ty_ = torch.min(draws["uy"].clone().view(B), torch.tensor(0.8))
    scale = (target_size / P).view(B)
    tx = (-tx_ + 0.5) * 2
    ty = (-ty_ + 0.5) * 2
    sin, cos = torch.sin(angle), torch.cos(angle)
    theta = torch.zeros(B, 2, 3, dtype=lab_batch.dtype)
    theta[:, 0, 0] = cos / scale
    theta[:, 0, 1] = sin / scale
    theta[:, 0, 2] = tx * cos / scale + ty * sin / scale
    theta[:, 1, 0] = -sin / scale
    theta[:, 1, 1] = cos / scale
    theta[:, 1, 2] = -tx * sin / scale + ty * cos / scale
    center = torch.stack([tx_ * img_size, ty_ * img_size], 1)
    return theta, center, target_size.view(B)


# --------------------------------------------------------------------------
# load_data.py:808-833 PatchApplier.forward
# --------------------------------------------------------------------------
def patch_applier(img_batch, adv_batch):
    for adv in torch.unbind(adv_batch, 1):
        img_batch = torch.where((adv == 0.), img_batch, adv)
    return img_batch


# --------------------------------------------------------------------------
# load_data.py:340-389 NPSCalculator
# --------------------------------------------------------------------------
def load_printability(path_or_rows):
    """Rows of (r,g,b) as float32 (load_data.py:369-389 parses 'r,g,b' lines
    and converts the decimal strings with np.float32)."""
    if isinstance(path_or_rows, str):
        rows = []
        with open(path_or_rows) as f:
            for line in f:
                line = line.strip()
                if line and not line.startswith("#"):
                    rows.append([np.float32(float(v)) for v in line.split(",")])
    else:
        rows = [[np.float32(float(v)) for v in r] for r in path_or_rows]
    return torch.from_numpy(np.asarray(rows, dtype=np.float32))


def nps_score(adv_patch, colors):
    """colors [Ncol,3]; broadcasting the [Ncol,3,P,P] printability array
    (load_data.py:357-367)."""
    P = adv_patch.size(-1)
    pa = colors.view(-1, 3, 1, 1).expand(-1, 3, P, P)
    color_dist = (adv_patch - pa + 0.000001)
    color_dist = color_dist ** 2
    color_dist = torch.sum(color_dist, 1) + 0.000001
    color_dist = torch.sqrt(color_dist)
    color_dist_prod = torch.min(color_dist, 0)[0]
    nps = torch.sum(color_dist_prod, 0)
    nps = torch.sum(nps, 0)
    return nps / torch.numel(adv_patch)


# --------------------------------------------------------------------------
# load_data.py:392-411 TotalVariation
# --------------------------------------------------------------------------
def total_variation(adv_patch):
    tv1 = torch.sum(torch.abs(adv_patch[:, :, 1:] - adv_patch[:, :, :-1] + 0.000001), 0)
    tv1 = torch.sum(torch.sum(tv1, 0), 0)
    tv2 = torch.sum(torch.abs(adv_patch[:, 1:, :] - adv_patch[:, :-1, :] + 0.000001), 0)
    tv2 = torch.sum(torch.sum(tv2, 0), 0)
    return (tv1 + tv2) / torch.numel(adv_patch)


# --------------------------------------------------------------------------
# load_data.py:1724-1754 HasSusRGB
# --------------------------------------------------------------------------
def colorful_loss(rgb):
    r, g, b = rgb[0, :, :], rgb[1, :, :], rgb[2, :, :]
    rg = r - g
    yb = 0.5 * (r + g) - b
    rg_mu, yb_mu = torch.mean(rg), torch.mean(yb)
    rg_sigma, yb_sigma = torch.var(rg), torch.var(yb)
    return torch.sqrt(rg_sigma + yb_sigma) + 0.3 * torch.sqrt(rg_mu ** 2 + yb_mu ** 2)


# --------------------------------------------------------------------------
# darknet_v3.py:9-100, 195-281 Darknet (eval mode), NCHW fp32
# --------------------------------------------------------------------------
def read_darknet_weights(path):
    """darknet_v3.py:227-232: 5 x int32 header, then a float32 stream."""
    with open(path, "rb") as f:
        header = np.fromfile(f, dtype=np.int32, count=5)
        weights = np.fromfile(f, dtype=np.float32)
    return header, weights


class OracleDarknet:
    def __init__(self, cfg_text, weights=None, requires_grad=False):
        blocks = parse_model_config(cfg_text)
        self.net = blocks.pop(0)                                   # darknet_v3.py:13
        self.width = int(self.net["width"])
        self.height = int(self.net["height"])
        self.blocks = blocks
        self.params = []
        filters = [int(self.net["channels"])]
        for i, d in enumerate(blocks):                             # darknet_v3.py:34-98
            t = d["type"]
            p = None
            if t == "convolutional":
                bn = int(d["batch_normalize"])
                f = int(d["filters"])
                k = int(d["size"])
                p = {"cin": filters[-1], "cout": f, "k": k, "stride": int(d["stride"]),
                     "pad": (k - 1) // 2, "bn": bn, "act": d["activation"],
                     "W": torch.zeros(f, filters[-1], k, k)}
                if bn:
                    p.update(bn_b=torch.zeros(f), bn_w=torch.ones(f),
                             bn_rm=torch.zeros(f), bn_rv=torch.ones(f))
                else:
                    p["b"] = torch.zeros(f)
            elif t == "route":
                f = sum(filters[1:][int(l)] for l in d["layers"].split(","))
            elif t == "shortcut":
                f = filters[1:][int(d["from"])]
            else:
                f = filters[-1]
            self.params.append(p)
            filters.append(f)
        if weights is not None:
            self.load_darknet_weights(weights)
        if requires_grad:
            for p in self.params:
                if p is not None:
                    for key in ("W", "b", "bn_b", "bn_w"):
                        if key in p:
                            p[key].requires_grad_(True)

    def load_darknet_weights(self, weights):
        """darknet_v3.py:240-281; the BN test is the truthiness of the raw cfg
        value (darknet_v3.py:245), as in the reference."""
        if isinstance(weights, str):
            _, weights = read_darknet_weights(weights)
        ptr = 0
        for d, p in zip(self.blocks, self.params):
            if d["type"] != "convolutional":
                continue
            n = p["cout"]
            if d["batch_normalize"]:
                for key in ("bn_b", "bn_w", "bn_rm", "bn_rv"):
                    p[key] = torch.from_numpy(weights[ptr:ptr + n].copy())
                    ptr += n
            else:
                p["b"] = torch.from_numpy(weights[ptr:ptr + n].copy())
                ptr += n
            nw = p["W"].numel()
            p["W"] = torch.from_numpy(weights[ptr:ptr + nw].copy()).view_as(p["W"])
            ptr += nw
        return ptr

    def forward(self, x, branch=None, record=None):                # darknet_v3.py:195-220
        """``branch`` (tests only): {block: ("leaky", bool mask NCHW)} or
        {block: ("maxpool", window-position index NCHW)} replaces the
        data-dependent branch decisions (LeakyReLU sign, maxpool argmax) with
        given ones — used to compare gradients of two fp32 implementations
        on identical branches (a pre-activation within rounding of 0 can
        take either LeakyReLU slope).  ``record``: dict filled with the
        pre-activations of leaky convs (key: block) and the windows of every
        max pool, [B,C,Ho,Wo,k*k] (key: ("maxpool", block))."""
        outs, yolo = [], []
        for i, (d, p) in enumerate(zip(self.blocks, self.params)):
            t = d["type"]
            br = branch.get(i) if branch else None
            if t == "convolutional":
                x = F.conv2d(x, p["W"], p.get("b"), stride=p["stride"], padding=p["pad"])
                if p["bn"]:
                    x = F.batch_norm(x, p["bn_rm"], p["bn_rv"], p["bn_w"], p["bn_b"],
                                     training=False, momentum=0.9, eps=1e-5)
                if record is not None:
                    if x.requires_grad:
                        x.retain_grad()
                    record[i] = x
                if p["act"] == "leaky":
                    if br is not None:
                        pos = br[1]
                        if pos.dtype != torch.bool:        # tri-state: -1 = decide here
                            pos = torch.where(pos < 0, x > 0, pos > 0)
                        x = x * torch.where(pos, torch.ones((), dtype=x.dtype), torch.full((), 0.1, dtype=x.dtype))
                    else:
                        x = F.leaky_relu(x, 0.1)
                elif p["act"] == "mish":
                    x = x * torch.tanh(F.softplus(x))
            elif t == "maxpool":                                   # darknet_v3.py:61-69
                k, s = int(d["size"]), int(d["stride"])
                if k == 2 and s == 1:
                    x = F.pad(x, (0, 1, 0, 1))
                if record is not None:                             # the pool windows (branch tie checks)
                    w_ = x.detach().unfold(2, k, s).unfold(3, k, s)
                    record[("maxpool", i)] = w_.reshape(w_.shape[:4] + (k * k,))
                if br is not None:
                    win = x.unfold(2, k, s).unfold(3, k, s)        # [B,C,Ho,Wo,k,k]
                    win = win.reshape(win.shape[:4] + (k * k,))
                    x = torch.gather(win, -1, br[1].long().unsqueeze(-1)).squeeze(-1)
                else:
                    x = F.max_pool2d(x, k, s, padding=(k - 1) // 2)
            elif t == "upsample":                                  # darknet_v3.py:103-113
                x = F.interpolate(x, scale_factor=int(d["stride"]), mode="nearest")
            elif t == "route":
                x = torch.cat([outs[int(l)] for l in d["layers"].split(",")], 1)
            elif t == "shortcut":
                x = outs[-1] + outs[int(d["from"])]
            elif t == "yolo":                                      # darknet_v3.py:144-169: identity
                yolo.append(x)
            outs.append(x)
        return yolo

    __call__ = forward

    def double(self):
        """A float64 copy (accuracy reference for fp32-vs-fp32 comparisons)."""
        import copy
        other = copy.copy(self)
        other.params = [None if p is None else
                        {k: (v.detach().double() if isinstance(v, torch.Tensor) else v) for k, v in p.items()}
                        for p in self.params]
        return other

    def parameters(self):
        for p in self.params:
            if p is not None:
                for key in ("W", "b", "bn_b", "bn_w"):
                    if key in p and p[key].requires_grad:
                        yield p[key]


# --------------------------------------------------------------------------
# train_patch.py:428-548 loss head (generalised to (nheads, 5+C))
# --------------------------------------------------------------------------
def obj_cls_conf_find(outputs, img_size, patch_center):
    """train_patch.py:428-486, including the transposed cell index
    `index = ix*w + iy` (train_patch.py:467).

    Generalised to any number of heads and C classes per
    anchor: the reference hard-codes 3 anchors x (5 + 15) = 60 channels
    (``view(batch, 3, 5 + 15, h*w)`` at 459, ``4:20`` / ``1:16`` at 470-483);
    here C = channels / 3 - 5, which is exactly that form for the reference's
    heads (C = 15) and also covers the two-head yolov3-tiny-15 (config 5)."""
    obj_all, cls_all = [], []
    for output in outputs:
        obj_inner, cls_inner = [], []
        batch, h, w = output.size(0), output.size(2), output.size(3)
        nc = output.size(1) // 3 - 5                             # 15 in the reference (459)
        feature_size = output.size(-1)
        feature_scale = img_size / feature_size
        axis = torch.div(patch_center, feature_scale, rounding_mode="floor")
        output = output.view(batch, 3, 5 + nc, h * w)
        for i in range(batch):
            index_x = int(axis[i, 0])
            index_y = int(axis[i, 1])
            index = int(index_x * feature_size + index_y)
            cells = torch.sigmoid(output[i, :, 4:5 + nc, index])
            obj_inner.append(cells[:, 0].view(-1, 3))
            cls_inner.append(cells[:, 1:1 + nc])
        obj_all.append(obj_inner)
        cls_all.append(cls_inner)
    return obj_all, cls_all


def cell_indices(heads_hw, img_size, patch_center):
    """Integer (head, image) -> flattened cell index, as obj_cls_conf_find."""
    res = []
    for hw in heads_hw:
        scale = img_size / hw
        axis = torch.div(patch_center, scale, rounding_mode="floor")
        res.append([int(int(axis[i, 0]) * hw + int(axis[i, 1])) for i in range(patch_center.size(0))])
    return res


def no_obj_reshape(index_obj_conf):
    """train_patch.py:488-503: stack the heads' [1,3] objectness rows to
    [nheads, B, 3], transpose to [B, nheads, 3] and flatten to [B, 3*nheads]
    (anchor k = head*3 + a).  The reference allocates ``zeros(3, B, 3)`` (492):
    nheads = 3; the generalised form (SURVEY.md Q10, config 5's two tiny
    heads) takes nheads = len(index_obj_conf).  ``no_obj_reshape3`` below
    keeps the literal 3-head statement the generalisation is tested against."""
    H = len(index_obj_conf)
    B = len(index_obj_conf[0])
    t = torch.zeros(H, B, 3)
    for i, obj in enumerate(index_obj_conf):
        t[i, :, :] = torch.cat(obj, 0)
    return t.transpose(0, 1).reshape(B, 3 * H)


def no_cls_reshape(index_cls_conf):
    """train_patch.py:505-524 generalised as no_obj_reshape: [nheads, B, 3, C]
    -> [B, 3*nheads, C] (the reference: ``zeros(3, B, 3, 15)``, 509-513)."""
    H = len(index_cls_conf)
    B = len(index_cls_conf[0])
    C = index_cls_conf[0][0].size(-1)
    t = torch.zeros(H, B, 3, C)
    for i, cls in enumerate(index_cls_conf):
        inner = torch.zeros(B, 3, C)
        for j, c in enumerate(cls):
            inner[j, :, :] = c
        t[i, :, :, :] = inner
    return t.transpose(0, 1).reshape(B, 3 * H, C)


def no_obj_reshape3(index_obj_conf):                               # train_patch.py:488-503, literal
    B = len(index_obj_conf[0])
    t = torch.zeros(3, B, 3)
    for i, obj in enumerate(index_obj_conf):
        t[i, :, :] = torch.cat(obj, 0)
    return t.transpose(0, 1).reshape(B, 9)


def no_cls_reshape3(index_cls_conf):                               # train_patch.py:505-524, literal
    B = len(index_cls_conf[0])
    t = torch.zeros(3, B, 3, 15)
    for i, cls in enumerate(index_cls_conf):
        inner = torch.zeros(B, 3, 15)
        for j, c in enumerate(cls):
            inner[j, :, :] = c
        t[i, :, :, :] = inner
    return t.transpose(0, 1).reshape(B, 9, 15)


def noCLS_Loss_CE(no_cls, cls_ID):                                 # train_patch.py:526-548
    B, A = no_cls.size(0), no_cls.size(1)
    ce = torch.nn.CrossEntropyLoss()
    target = torch.tensor([cls_ID]).repeat(A)
    batch_loss = torch.zeros(B)
    for i in range(B):
        batch_loss[i] = ce(no_cls[i, :, :], target)
    return torch.mean(batch_loss)


def noCLS_loss_targeted(no_cls, cls_ID):                           # train_patch.py:550-577
    B = no_cls.size(0)
    batch_loss = torch.zeros(B)
    for i in range(B):
        t = no_cls[i, :, cls_ID]
        mx, _ = torch.max(no_cls[i, :, :], dim=1)
        batch_loss[i] = torch.mean(mx - t)
    return torch.sum(batch_loss)


# --------------------------------------------------------------------------
# load_data.py:63-122 bbox_decode, 125-311 MaxProbExtractor (constructed at
# train_patch.py:74-75; its call at 255 is commented out in the reference)
# --------------------------------------------------------------------------
def bbox_decode(output, num_classes, anchors, num_anchors, img_size=(608, 608)):
    """load_data.py:63-122 (CPU: the reference's .cuda() calls dropped)."""
    batch, h, w = output.size(0), output.size(2), output.size(3)
    stride_h = img_size[1] / h
    stride_w = img_size[0] / w
    scaled = [(aw / stride_w, ah / stride_h) for aw, ah in anchors]
    output = output.view(batch * num_anchors, 5 + num_classes, h * w)
    output = output.transpose(0, 1).contiguous()
    output = output.view(5 + num_classes, batch * num_anchors * h * w)
    grid_x = torch.linspace(0, w - 1, w).repeat(h, 1).repeat(batch * num_anchors, 1, 1).view(
        batch * num_anchors * h * w)
    grid_y = torch.linspace(0, h - 1, h).repeat(w, 1).t().repeat(batch * num_anchors, 1, 1).view(
        batch * num_anchors * h * w)
    xs = torch.sigmoid(output[0]) + grid_x
    ys = torch.sigmoid(output[1]) + grid_y
    anchor_w = torch.Tensor(scaled).index_select(1, torch.LongTensor([0]))
    anchor_h = torch.Tensor(scaled).index_select(1, torch.LongTensor([1]))
    anchor_w = anchor_w.repeat(batch, 1).repeat(1, 1, h * w).view(batch * num_anchors * h * w)
    anchor_h = anchor_h.repeat(batch, 1).repeat(1, 1, h * w).view(batch * num_anchors * h * w)
    ws = torch.exp(output[2]) * anchor_w
    hs = torch.exp(output[3]) * anchor_h
    output = output.clone()          # the reference writes rows 0..3 in place of a fresh copy
    output[0] = xs / w
    output[1] = ys / h
    output[2] = ws / w
    output[3] = hs / h
    output = output.view(5 + num_classes, batch * num_anchors, h * w)
    output = output.transpose(0, 1).contiguous()
    return output.view(batch, num_anchors * (5 + num_classes), h, w)


def max_prob_extractor(outputs, cls_id, num_cls, anchors_per_head, sigmoid_mode=False):
    """MaxProbExtractor.forward (load_data.py:160-228, 311): decode every head,
    concatenate to [B, 5+C, sum 3*h*w] (index = head offset + a*h*w + cell) and
    take the per-image max of the objectness row and of row 5+cls_id, raw or
    after sigmoid.  Returns (max_obj [B], max_cls [B], obj_idx [B], cls_idx [B])."""
    singles = []
    for i, output in enumerate(outputs):
        batch, h, w = output.size(0), output.size(2), output.size(3)
        output = bbox_decode(output, num_cls, anchors_per_head[i], 3)
        output = output.view(batch, 3, 5 + num_cls, h * w)
        output = output.transpose(1, 2).contiguous()
        singles.append(output.view(batch, 5 + num_cls, 3 * h * w))
    cat = torch.cat(singles, 2)
    if sigmoid_mode:
        obj = torch.sigmoid(cat[:, 4, :])
        cls = torch.sigmoid(cat[:, 5:5 + num_cls, :])[:, cls_id, :]
    else:
        obj = cat[:, 4, :]
        cls = cat[:, 5:5 + num_cls, :][:, cls_id, :]
    max_cls, ci = torch.max(cls, dim=1)
    max_obj, oi = torch.max(obj, dim=1)
    return max_obj, max_cls, oi, ci


# --------------------------------------------------------------------------
# train_patch.py:157-330 one iteration of the batch loop
# --------------------------------------------------------------------------
def train_step(patch, img_batch, lab_batch, draws, net, colors, target_id=TARGET_ID,
               objective="ce", weight_grad=False, branch=None, record=None, combine=None, geometry="fp32"):
    """One iteration of PatchTrainer.train's batch body (train_patch.py:164-327).

    ``patch`` is the [3,P,P] leaf.  Returns a dict of loss terms (float
    tensors), the patch gradient, and the intermediates the parity tests
    check (patch_center, cell indices, obj [B,3*nheads], cls [B,3*nheads,C];
    [B,9] and [B,9,15] for the reference's three heads).
    ``objective``: "ce" (active, train_patch.py:253), "targeted"
    (noCLS_loss_targeted, train_patch.py:262) or "untargeted"
    (train_patch.py:305-307).  ``branch``, ``record``: see OracleDarknet.forward
    (recorded pre-activations keep their gradients).  ``combine`` (tests of
    the data-parallel weighting): f(no_obj_loss, no_cls_loss, nps, tv,
    colorful) -> (loss, terms) replaces the loss formula of 312-314.
    ``geometry``: see patch_transformer ("fp32" the reference; "f64" the
    placement geometry in float64; "fp32in64" the reference's fp32 sample
    points under a float64 evaluation).
    """
    leaf = patch.detach().clone().requires_grad_(True)
    img_size = net.height
    adv_batch_t, patch_center = patch_transformer(leaf, lab_batch, img_size, draws, geometry=geometry)  # 173-174
    p_img = patch_applier(img_batch, adv_batch_t)                                  # 183
    p_img = F.interpolate(p_img, (net.height, net.width))                         # 186-187
    outputs = net(p_img, branch=branch, record=record)                             # 197
    obj_l, cls_l = obj_cls_conf_find(outputs, img_size, patch_center)              # 207-208
    no_obj = no_obj_reshape(obj_l)                                                 # 213-214
    no_cls = no_cls_reshape(cls_l)                                                 # 216-217
    obj_conf_max, _ = torch.max(no_obj, 1, keepdim=True)                           # 230-231
    no_obj_loss = 4 * (1 - torch.mean(obj_conf_max))                               # 236-239
    if objective == "ce":
        no_cls_loss = noCLS_Loss_CE(no_cls, target_id)                             # 253
    elif objective == "targeted":
        no_cls_loss = noCLS_loss_targeted(no_cls, target_id)                       # 262
    else:
        no_cls_loss = torch.zeros(())
    nps = nps_score(leaf, colors)                                                  # 280
    tv = total_variation(leaf)                                                     # 281
    nps_loss = nps * NPS_FACTOR
    tv_loss = tv * TV_FACTOR
    colorful = colorful_loss(leaf)                                                 # 311
    if combine is None:
        loss = nps_loss + torch.max(tv_loss, torch.tensor(0.1)) + no_obj_loss + colorful  # 312-314
        if objective != "untargeted":
            loss = loss + no_cls_loss
    else:
        loss, t = combine(no_obj_loss, no_cls_loss, nps, tv, colorful)
        nps_loss, tv_loss, no_obj_loss, no_cls_loss, colorful = (
            t["nps_loss"], t["tv_loss"], t["no_obj_loss"], t["no_cls_loss"], t["colorful_loss"])
    loss.backward()                                                                # 327
    return {
        "loss": loss.detach(), "nps_loss": nps_loss.detach(), "tv_loss": tv_loss.detach(),
        "no_obj_loss": no_obj_loss.detach(), "no_cls_loss": no_cls_loss.detach(),
        "colorful_loss": colorful.detach(), "grad": leaf.grad.detach().clone(),
        "patch_center": patch_center.detach(), "obj": no_obj.detach(), "cls": no_cls.detach(),
        "cells": cell_indices([o.size(-1) for o in outputs], img_size, patch_center.detach()),
        "p_img": p_img.detach(), "heads": [o.detach() for o in outputs],
    }


def train_step_f64(patch, img_batch, lab_batch, draws, net, colors, **kw):
    """train_step evaluated in float64 (same ops) — the accuracy yardstick
    against which two fp32 implementations are compared."""
    old = torch.get_default_dtype()
    torch.set_default_dtype(torch.float64)
    try:
        return train_step(patch.double(), img_batch.double(), lab_batch.double(),
                          {k: v.double() for k, v in draws.items()}, net.double(), colors.double(), **kw)
    finally:
        torch.set_default_dtype(old)


def adam_amsgrad_steps(patch, grads_fn, n_steps, lr=0.03):
    """train_patch.py:131-132, 327-330: Adam(lr, amsgrad=True); step;
    zero_grad; clamp_(0,1).  ``grads_fn(patch) -> grad``."""
    leaf = patch.detach().clone().requires_grad_(True)
    opt = torch.optim.Adam([leaf], lr=lr, amsgrad=True)
    for _ in range(n_steps):
        leaf.grad = grads_fn(leaf.detach())
        opt.step()
        opt.zero_grad()
        leaf.data.clamp_(0, 1)
    return leaf.detach()
