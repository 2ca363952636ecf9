"""Darknet (YOLOv3 family) — drop-in for reference ``darknet_v3.py`` whose
forward and input-gradient run as HIP kernels on gfx950.

Surface kept from the reference: ``create_modules`` (darknet_v3.py:9-100),
``Upsample``, ``Mish``, ``YOLOLayer`` (identity on the training path,
darknet_v3.py:144-169), ``Darknet`` with ``.blocks``, ``.module_list``,
``.width``, ``.height``, ``.hyperparams``, ``.yolo_layers``,
``load_darknet_weights`` (darknet_v3.py:223-281) and ``forward(x)`` returning
the raw head tensors [B, 3*(5+C), h, w] (darknet_v3.py:195-220).

Execution (``NetPlan``): one plan per (batch, height, width, device) holds
every activation and gradient buffer in HBM (NHWC, channel stride padded to a
multiple of 16).  Forward = per block one launch: ``po_conv`` implicit-GEMM
on fp32 MFMA with BN folded into W/bias, LeakyReLU and the following
``shortcut`` add fused into its epilogue; ``route`` of one layer is an alias,
of several layers a channel-slice copy; ``upsample`` and ``maxpool`` are
data-movement kernels.  Backward computes the input gradient only (dgrad, no
weight gradients: the patch is the only trainable tensor): each conv's dgrad
is the same implicit GEMM with transposed/flipped weights (stride 2 split into
its 4 parity classes), and the LeakyReLU derivative of the producing layer is
applied in the epilogue of the last gradient contribution to it.
"""
import math
import os
from itertools import chain

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _native as nat
from .cfg import parse_model_config


# ---------------------------------------------------------------------------
# Module construction (parameter containers, as in the reference)
# ---------------------------------------------------------------------------
def create_modules(module_defs):
    """Constructs module list of layer blocks from module configuration in
    module_defs (pops the [net] block, darknet_v3.py:13-29)."""
    hyperparams = module_defs.pop(0)
    hyperparams.update({
        "batch": int(hyperparams["batch"]),
        "subdivisions": int(hyperparams["subdivisions"]),
        "width": int(hyperparams["width"]),
        "height": int(hyperparams["height"]),
        "channels": int(hyperparams["channels"]),
        "optimizer": hyperparams.get("optimizer"),
        "momentum": float(hyperparams["momentum"]),
        "decay": float(hyperparams["decay"]),
        "learning_rate": float(hyperparams["learning_rate"]),
        "burn_in": int(hyperparams["burn_in"]),
        "max_batches": int(hyperparams["max_batches"]),
        "policy": hyperparams["policy"],
        "lr_steps": list(zip(map(int, hyperparams["steps"].split(",")),
                             map(float, hyperparams["scales"].split(",")))),
    })
    assert hyperparams["height"] == hyperparams["width"], \
        "Height and width should be equal! Non square images are padded with zeros."
    output_filters = [hyperparams["channels"]]
    module_list = nn.ModuleList()
    for module_i, module_def in enumerate(module_defs):
        modules = nn.Sequential()
        t = module_def["type"]
        if t == "convolutional":
            bn = int(module_def["batch_normalize"])
            filters = int(module_def["filters"])
            k = int(module_def["size"])
            conv = torch.nn.utils.skip_init(nn.Conv2d, output_filters[-1], filters, k,
                                            stride=int(module_def["stride"]), padding=(k - 1) // 2,
                                            bias=not bn)
            with torch.no_grad():
                conv.weight.zero_()
                if conv.bias is not None:
                    conv.bias.zero_()
            modules.add_module(f"conv_{module_i}", conv)
            if bn:
                modules.add_module(f"batch_norm_{module_i}", nn.BatchNorm2d(filters, momentum=0.9, eps=1e-5))
            if module_def["activation"] == "leaky":
                modules.add_module(f"leaky_{module_i}", nn.LeakyReLU(0.1))
            if module_def["activation"] == "mish":
                modules.add_module(f"mish_{module_i}", Mish())
        elif t == "maxpool":
            k, s = int(module_def["size"]), int(module_def["stride"])
            if k == 2 and s == 1:
                modules.add_module(f"_debug_padding_{module_i}", nn.ZeroPad2d((0, 1, 0, 1)))
            modules.add_module(f"maxpool_{module_i}", nn.MaxPool2d(kernel_size=k, stride=s, padding=int((k - 1) // 2)))
            filters = output_filters[-1]
        elif t == "upsample":
            modules.add_module(f"upsample_{module_i}", Upsample(scale_factor=int(module_def["stride"]), mode="nearest"))
            filters = output_filters[-1]
        elif t == "route":
            layers = [int(x) for x in module_def["layers"].split(",")]
            filters = sum([output_filters[1:][i] for i in layers])
            modules.add_module(f"route_{module_i}", nn.Sequential())
        elif t == "shortcut":
            filters = output_filters[1:][int(module_def["from"])]
            modules.add_module(f"shortcut_{module_i}", nn.Sequential())
        elif t == "yolo":
            anchor_idxs = [int(x) for x in module_def["mask"].split(",")]
            anchors = [int(x) for x in module_def["anchors"].split(",")]
            anchors = [(anchors[i], anchors[i + 1]) for i in range(0, len(anchors), 2)]
            anchors = [anchors[i] for i in anchor_idxs]
            modules.add_module(f"yolo_{module_i}", YOLOLayer(anchors, int(module_def["classes"])))
            filters = output_filters[-1]
        else:
            raise ValueError("unsupported darknet block type %r" % t)
        module_list.append(modules)
        output_filters.append(filters)
    return hyperparams, module_list


class Upsample(nn.Module):
    """nearest upsample (darknet_v3.py:103-113)"""

    def __init__(self, scale_factor, mode="nearest"):
        super().__init__()
        self.scale_factor = scale_factor
        self.mode = mode

    def forward(self, x):
        return F.interpolate(x, scale_factor=self.scale_factor, mode=self.mode)


class Mish(nn.Module):
    """Mish activation (darknet_v3.py:116-123; unused by the yolov3 cfgs)."""

    def forward(self, x):
        return x * torch.tanh(F.softplus(x))


class YOLOLayer(nn.Module):
    """Detection layer: identity on the training path (darknet_v3.py:144-169)."""

    def __init__(self, anchors, num_classes):
        super().__init__()
        self.num_anchors = len(anchors)
        self.num_classes = num_classes
        self.no = num_classes + 5
        self.grid = torch.zeros(1)
        anchors = torch.tensor(list(chain(*anchors))).float().view(-1, 2)
        self.register_buffer("anchors", anchors)
        self.register_buffer("anchor_grid", anchors.clone().view(1, -1, 1, 1, 2))
        self.stride = None

    def forward(self, x, img_size):
        return x


def _cp(c):
    return (c + 15) // 16 * 16


# ---------------------------------------------------------------------------
# Execution plan
# ---------------------------------------------------------------------------
INPUT = -1


class NetPlan:
    """All buffers and launch lists of one (B, H, W, device) configuration."""

    def __init__(self, net, B, H, W, device, windowed=False):
        self.net, self.B, self.H, self.W, self.device = net, B, H, W, device
        self.gen = 0
        self.conv_timer = None        # list: (start, end, desc, cones) of every po_conv launch (launch_macs)
        self.first_timer = []         # (start, end, entry) of the first layer's forward while conv_timer is set
        self._cone_snap = None
        self.ws = None                # split-K workspace (shared by every launch; stream-ordered)
        blocks = net.blocks
        n = len(blocks)
        self.n = n
        self.lib = nat.load()
        # ---- shapes, roots
        shp = []                     # (H, W, C) per block
        root = list(range(n))
        srcs = [[] for _ in range(n)]
        h, w, c = H, W, net.hyperparams["channels"]
        prev = INPUT
        self.heads = []              # block indices of yolo layers
        fused = set()                # shortcut blocks fused into the previous conv
        for i, d in enumerate(blocks):
            t = d["type"]
            if t == "convolutional":
                p = net._conv_meta[i]
                h = (h + 2 * p["pad"] - p["k"]) // p["stride"] + 1
                w = (w + 2 * p["pad"] - p["k"]) // p["stride"] + 1
                c = p["cout"]
                srcs[i] = [prev]
            elif t == "maxpool":
                k, s = int(d["size"]), int(d["stride"])
                if k != 2:
                    raise NotImplementedError("maxpool size %d (only 2 on the yolov3 paths)" % k)
                if s == 2:
                    h, w = h // 2, w // 2
                srcs[i] = [prev]
            elif t == "upsample":
                if int(d["stride"]) != 2:
                    raise NotImplementedError("upsample stride %s" % d["stride"])
                h, w = 2 * h, 2 * w
                srcs[i] = [prev]
            elif t == "route":
                ls = [int(x) for x in d["layers"].split(",")]
                ls = [l if l >= 0 else i + l for l in ls]
                srcs[i] = [root[l] for l in ls]
                h, w = shp[ls[0]][0], shp[ls[0]][1]
                c = sum(shp[l][2] for l in ls)
                for l in ls:
                    assert shp[l][:2] == (h, w), "route of mismatched spatial sizes"
                if len(ls) == 1:
                    root[i] = root[ls[0]]
            elif t == "shortcut":
                f = int(d["from"])
                f = f if f >= 0 else i + f
                srcs[i] = [prev, root[f]]
                if i > 0 and blocks[i - 1]["type"] == "convolutional" and root[i - 1] == i - 1:
                    fused.add(i)
            elif t == "yolo":
                root[i] = root[i - 1]
                srcs[i] = [prev]
                self.heads.append(i)
            shp.append((h, w, c))
            prev = root[i]
        self.shp, self.root, self.srcs, self.fused = shp, root, srcs, fused
        self.cp = [_cp(s[2]) for s in shp]
        dev = device
        self.win = [None] * n          # window side of a block's buffer (None: full map)
        self.win_idx = {}              # block -> row of self.org
        self.windowed = False
        if windowed:
            self._plan_windows()
        self.dims = [(self.win[i], self.win[i]) if self.win[i] else shp[i][:2] for i in range(n)]
        for i in range(n):
            if root[i] != i:
                self.dims[i] = self.dims[root[i]]
        z = lambda i: torch.zeros(B, self.dims[i][0], self.dims[i][1], self.cp[i], device=dev)
        self.act = [z(i) if root[i] == i else None for i in range(n)]
        for i in range(n):
            if self.act[i] is None:
                self.act[i] = self.act[root[i]]
        self.argmax = {i: torch.zeros(B, self.dims[i][0], self.dims[i][1], self.cp[i], dtype=torch.int8, device=dev)
                       for i, d in enumerate(blocks) if d["type"] == "maxpool"}
        first = blocks[0]
        self.first_direct = (first["type"] == "convolutional" and net._conv_meta[0]["k"] == 3
                             and net._conv_meta[0]["cin"] == 3 and net._conv_meta[0]["cout"] <= 64)
        self.in_nhwc = None if self.first_direct else torch.zeros(B, H, W, 16, device=dev)
        # the first layer can read the training step's sparse composite (the patch
        # footprint boxes in one tensor, the frames in another: po_conv_first_*_cmp)
        self.sparse_input = self.first_direct and H == W and H % 4 == 0 and self.cp[0] <= 32
        # first conv (stride 1) whose only consumer is a k=2 stride-2 max pool
        # (yolov3-tiny): one fused launch writes the pool output and its argmax
        # (with the LeakyReLU slope encoded); the conv output is never stored
        self.first_pool = (self.first_direct and n > 1 and net._conv_meta[0]["stride"] == 1
                           and blocks[1]["type"] == "maxpool" and int(blocks[1]["stride"]) == 2
                           and self.cp[0] in (16, 32) and self.win[0] is None and self.win[1] is None
                           and [j for j in range(n) if 0 in srcs[j]] == [1]
                           and os.environ.get("ADVPATCH_FIRST_POOL", "1") != "0")
        # ... computed as Winograd F(2x2,3x3) (po_conv_first_pool_wino_fwd)
        self.first_wino = self.first_pool and os.environ.get("ADVPATCH_FIRST_WINO", "1") != "0"
        # later conv + k=2 stride-2 pool pairs (yolov3-tiny blocks 2/3, 4/5): the pool
        # runs in the conv epilogue (po_conv_desc.pool_y, pool-order grid) when the
        # conv's only consumer is the pool: with exact fp32 operands at any width
        # (the generic tiles and Winograd tile 66 carry the pool epilogue), with
        # fp16x3 operands at Cin_p <= 32 (generic tiles only, where the halo tiles
        # do not win anyway); ADVPATCH_CONV_POOL=0: off
        self.conv_pool = set()
        if os.environ.get("ADVPATCH_CONV_POOL", "1") != "0":
            for i in range(1, n - 1):
                if (blocks[i]["type"] == "convolutional" and root[i] == i and blocks[i + 1]["type"] == "maxpool"
                        and int(blocks[i + 1]["stride"]) == 2 and root[i + 1] == i + 1
                        and [j for j in range(n) if i in srcs[j]] == [i + 1]
                        and self.win[i] is None and self.win[i + 1] is None
                        and shp[i][0] % 2 == 0 and shp[i][1] % 2 == 0 and self.cp[i] % 16 == 0
                        and srcs[i][0] != INPUT and (self.cp[srcs[i][0]] <= 32 or net.conv_prec != "fp16x3")
                        and not (i - 1 == 0 and self.first_pool)):
                    self.conv_pool.add(i)
        self._build_grad_plan()
        self.prec = 1 if net.conv_prec == "fp16x3" else 0
        self._build_slots()
        self._build_bits()
        self._build_cones()
        self.support = []             # compact dgrad grids over window supports (_support_grid)
        self._build_ops()
        self._drop_mask_only_outputs()
        self._plan_tails()

    # ---------------- receptive-field windows ----------------
    def _cone(self, seed):
        """Map intervals (one axis) of every block needed for the loss to see
        the head cells in ``seed`` {block: (lo, hi)}; propagated backwards
        through the graph (conv: dilation by its window, upsample: /2,
        route/shortcut: same box)."""
        blocks, root, srcs, shp = self.net.blocks, self.root, self.srcs, self.shp
        need = dict(seed)

        def push(s, a, b):
            if s == INPUT:
                return
            a, b = max(a, 0), min(b, shp[s][0] - 1)
            if a > b:
                return
            need[s] = (min(need[s][0], a), max(need[s][1], b)) if s in need else (a, b)

        for j in range(self.n - 1, -1, -1):
            if root[j] != j or j not in need:
                continue
            lo, hi = need[j]
            t = blocks[j]["type"]
            if t == "convolutional":
                m = self.net._conv_meta[j]
                push(srcs[j][0], lo * m["stride"] - m["pad"], hi * m["stride"] - m["pad"] + m["k"] - 1)
            elif t == "maxpool":
                if int(blocks[j]["stride"]) == 2:
                    push(srcs[j][0], 2 * lo, 2 * hi + 1)
                else:
                    push(srcs[j][0], lo, hi + 1)
            elif t == "upsample":
                push(srcs[j][0], lo // 2, hi // 2)
            elif t in ("route", "shortcut"):
                for s_ in srcs[j]:
                    push(s_, lo, hi)
        return need

    def head_cells(self, v):
        """Head cells (one axis) of a patch-centre coordinate v, as po_cell_loss
        computes them (float32 floor division by S/hw, train_patch.py:446-450)."""
        out = []
        for h in self.heads:
            hw = self.shp[self.root[h]][0]
            stride = np.float32(self.H / hw)
            out.append(int(min(max(np.floor(np.float32(v) / stride), 0), hw - 1)))
        return out

    def _plan_windows(self):
        """Choose the blocks computed only on a box around the head cells.

        The loss reads every head at one cell per image (train_patch.py:449-483),
        so a block downstream of the last full-map dependency only matters on
        the union of the head cells' receptive-field cones.  A block is
        windowed when that box (its static side = the largest box over every
        patch-centre position) is smaller than its map and nothing forces it
        dense: shortcut blocks and their operands, maxpool, strided convs and
        every source of a dense block keep full maps."""
        blocks, root, srcs, shp, n = self.net.blocks, self.root, self.srcs, self.shp, self.n
        if self.H != self.W or not self.heads:
            return
        hroots = [root[h] for h in self.heads]
        hws = [shp[r][0] for r in hroots]
        maxhw = max(hws)
        nh = len(hroots)
        BIG = 1 << 30
        lo_t = np.full((n, nh, maxhw), BIG, dtype=np.int64)
        hi_t = np.full((n, nh, maxhw), -BIG, dtype=np.int64)
        for h, (r, hw) in enumerate(zip(hroots, hws)):
            for c in range(hw):
                for j, (lo, hi) in self._cone({r: (c, c)}).items():
                    lo_t[j, h, c], hi_t[j, h, c] = lo, hi
        # every combination of head cells a patch centre can produce
        combos = sorted({tuple(self.head_cells(v)) for v in np.arange(0, self.H, 1.0 / 16)})
        side = np.zeros(n, dtype=np.int64)
        for cb in combos:
            lo = np.min(np.stack([lo_t[:, h, c] for h, c in enumerate(cb)]), axis=0)
            hi = np.max(np.stack([hi_t[:, h, c] for h, c in enumerate(cb)]), axis=0)
            side = np.maximum(side, np.where(hi >= lo, hi - lo + 1, 0))
        dense = [True] * n
        for j in range(n):
            if root[j] == j and 0 < side[j] < shp[j][0] and shp[j][0] == shp[j][1]:
                dense[j] = False
        for j in range(n):
            t = blocks[j]["type"]
            if t in ("shortcut", "maxpool") or (j + 1) in self.fused:
                dense[j] = True
                if t == "shortcut":
                    for s_ in srcs[j]:
                        if s_ != INPUT:
                            dense[s_] = True
            if t == "convolutional" and (self.net._conv_meta[j]["stride"] != 1 or j == 0):
                dense[j] = True
        for j in range(n - 1, -1, -1):         # a full-map block needs full-map sources
            if root[j] == j and dense[j]:
                for s_ in srcs[j]:
                    if s_ != INPUT:
                        dense[s_] = True
        wins = [j for j in range(n) if root[j] == j and not dense[j]]
        if not wins:
            return
        for w, j in enumerate(wins):
            self.win[j] = int(side[j])
            self.win_idx[j] = w
        lut = np.zeros((len(wins), nh, maxhw, 2), dtype=np.int32)
        ext = np.zeros((len(wins), 2), dtype=np.int32)
        for w, j in enumerate(wins):
            ok = hi_t[j] >= lo_t[j]
            lut[w, :, :, 0] = np.where(ok, lo_t[j], 1)
            lut[w, :, :, 1] = np.where(ok, hi_t[j], 0)
            ext[w] = (self.win[j], shp[j][0])
        dev = self.device
        self.win_lut = torch.from_numpy(lut).to(dev)
        self.win_ext = torch.from_numpy(ext).to(dev)
        self.win_maxhw = maxhw
        self.win_hw = hws
        self.org = torch.zeros(len(wins), self.B, 2, dtype=torch.int32, device=dev)
        self.win_flags = torch.zeros(1, dtype=torch.int32, device=dev)
        self.windowed = True

    def org_of(self, i):
        """Device origin array [B,2] of block i's window (None: full map)."""
        i = self.root[i] if i != INPUT else i
        if i == INPUT or self.win[i] is None:
            return None
        return self.org[self.win_idx[i]]

    def set_windows(self, center):
        """Place every window around the head cells of ``center`` [B,2] (patch
        centres, column/row px) for the next forward (po_cell_windows)."""
        hw = (nat.c_int * len(self.win_hw))(*self.win_hw)
        nat.call("po_cell_windows", nat.ptr(center.contiguous()), self.B, self.H, len(self.win_hw), hw,
                 self.org.size(0), nat.ptr(self.win_lut, torch.int32), self.win_maxhw,
                 nat.ptr(self.win_ext, torch.int32), nat.ptr(self.org, torch.int32),
                 nat.ptr(self.win_flags, torch.int32), nat.stream())

    def head_views(self):
        """None (full-map heads) or (window sides, origin arrays) for po_cell_loss."""
        if not self.windowed:
            return None
        win = [self.dims[self.root[h]][0] for h in self.heads]
        return win, [self.org_of(h) for h in self.heads]

    # ---------------- gradient cones ----------------
    CONE_MAX_FRAC = 0.85          # a block's gradient is boxed when its typical cone is smaller

    def _cone_prog(self):
        """Rows {dst, src, kind, k, stride, pad, Hdst, Wdst} of po_grad_boxes:
        the forward influence of the input through every block, in order."""
        rows = []
        for j, d in enumerate(self.net.blocks):
            if self.root[j] != j:
                continue
            t = d["type"]
            H, W = self.shp[j][:2]
            for s in self.srcs[j]:
                src = -1 if s == INPUT else s
                if t == "convolutional":
                    m = self.net._conv_meta[j]
                    rows.append((j, src, 0, m["k"], m["stride"], m["pad"], H, W))
                elif t == "maxpool":
                    rows.append((j, src, 2 if int(d["stride"]) == 2 else 3, 2, 0, 0, H, W))
                elif t == "upsample":
                    rows.append((j, src, 4, 0, 0, 0, H, W))
                else:
                    rows.append((j, src, 1, 0, 0, 0, H, W))
        return rows

    @staticmethod
    def cone_boxes_host(prog, nbox, roi):
        """Host restatement of po_grad_boxes for one image: roi (x0, y0, x1, y1)
        -> {block: (r0, c0, r1, c1)} half-open (tests, planning)."""
        def fdiv(a, b):
            return a // b

        def cmap(kind, k, s, pad, a, b):
            if kind == 0:
                return -fdiv(-(a + pad - k + 1), s), fdiv(b + pad, s)
            if kind == 2:
                return fdiv(a, 2), fdiv(b, 2)
            if kind == 3:
                return a - 1, b
            if kind == 4:
                return 2 * a, 2 * b + 1
            return a, b

        box = {}
        for dst, src, kind, k, s, pad, H, W in prog:
            box.setdefault(dst, (0, 0, 0, 0))
        for dst, src, kind, k, s, pad, H, W in prog:
            if src < 0:
                r0, c0, r1, c1 = roi[1], roi[0], roi[3], roi[2]
            else:
                r0, c0, r1, c1 = box[src]
            if r0 >= r1 or c0 >= c1:
                continue
            a0, a1 = cmap(kind, k, s, pad, r0, r1 - 1)
            b0, b1 = cmap(kind, k, s, pad, c0, c1 - 1)
            a0, b0, a1, b1 = max(a0, 0), max(b0, 0), min(a1, H - 1), min(b1, W - 1)
            if a0 > a1 or b0 > b1:
                continue
            o = box[dst]
            if o[0] >= o[2] or o[1] >= o[3]:
                box[dst] = (a0, b0, a1 + 1, b1 + 1)
            else:
                box[dst] = (min(o[0], a0), min(o[1], b0), max(o[2], a1 + 1), max(o[3], b1 + 1))
        return box

    def _build_cones(self):
        """Blocks whose input gradient is computed on the gradient cone only.

        The patch gradient needs dL/d(image) only on the patch footprint (the
        po_patch_params roi), so block j's gradient is only needed on the
        pixels the footprint influences (po_grad_boxes).  A dgrad writing the
        gradient of such a block gets the block's per-image box (po_conv
        gbox).  Chosen when the cone of a centred S/3 footprint covers less
        than CONE_MAX_FRAC of the map: the early high-resolution stages
        (ADVPATCH_GRAD_CONES=0 disables)."""
        self.cone_blocks = set()
        self.cone_boxes = None
        if os.environ.get("ADVPATCH_GRAD_CONES", "1") == "0" or self.H != self.W:
            return
        prog = self._cone_prog()
        S = self.H
        a = S // 3
        est = self.cone_boxes_host(prog, self.n, (a, a, S - a, S - a))
        frac = float(os.environ.get("ADVPATCH_CONE_MAX_FRAC", self.CONE_MAX_FRAC))
        for j, (r0, c0, r1, c1) in est.items():
            H, W = self.shp[j][:2]
            if (self.has_grad[j] and self.win[j] is None and self.grad[j] is not None
                    and (r1 - r0) * (c1 - c0) < frac * H * W):
                self.cone_blocks.add(j)
        if not self.cone_blocks:
            return
        self.cone_prog = torch.tensor(prog, dtype=torch.int32, device=self.device).contiguous()
        self.cone_boxes = torch.zeros(self.n, self.B, 4, dtype=torch.int32, device=self.device)

    def tuning_rois(self):
        """[B,4] patch footprints (x0, y0, x1, y1) the tuner times boxed
        launches on: square footprints with sides spread over 0.10-0.30 S
        across the batch at positions spread over the frame — the range of
        the training placement (target size S/4 * sqrt(y^2 + w^2) of the
        selected label, SURVEY Q2, times the rotation's up to sqrt(2);
        ~0.16 S on the synthetic DOTA labels).  A centred S/3 footprint (the
        round-2 choice) gives boxes ~4x the typical area, and the tuner then
        leaves the real, smaller boxed launches with too few workgroups."""
        S, B = self.H, self.B
        rows = []
        for b in range(B):
            f = b / max(B - 1, 1)
            side = int(S * (0.10 + 0.20 * ((7 * b) % B) / max(B - 1, 1)))
            cx = int(S * (0.25 + 0.5 * f))
            cy = int(S * (0.25 + 0.5 * ((3 * b) % B) / max(B - 1, 1)))
            x0, y0 = max(cx - side // 2, 0), max(cy - side // 2, 0)
            rows.append([x0, y0, min(x0 + side, S), min(y0 + side, S)])
        return torch.tensor(rows, dtype=torch.int32, device=self.device)

    def set_cones(self, roi):
        """Evaluate the gradient cones of roi [B,4] (None: the whole image)."""
        if self.cone_boxes is None:
            return
        nat.call("po_grad_boxes", nat.c_void_p(roi.data_ptr()) if roi is not None else None, self.B, self.H,
                 nat.c_void_p(self.cone_prog.data_ptr()), self.cone_prog.size(0), self.n,
                 nat.c_void_p(self.cone_boxes.data_ptr()), nat.stream())

    @staticmethod
    def launch_macs(desc, cones=None):
        """MACs one po_conv launch computes: desc.macs for a full grid; for a
        boxed launch (cones = the step's po_grad_boxes output) only its
        per-image boxes' grid points, counted as the kernels enumerate them."""
        if getattr(desc, "support", None) is not None:
            bx = desc.support.tolist()
            pts = sum(max(r1 - r0, 0) * max(c1 - c0, 0) for r0, c0, r1, c1 in bx)
            return desc.macs * pts / (desc.B * desc.mrows)
        if cones is None or not desc.gbox:
            return desc.macs

        def span(lo, hi, off, step, n):
            a = 0 if lo - off <= 0 else -(-(lo - off) // step)
            b = 0 if hi - 1 - off < 0 else min(n, (hi - 1 - off) // step + 1)
            return max(b - a, 0)

        bx = cones[desc.cone_block, desc.cone_b0:desc.cone_b0 + desc.B].tolist()       # host or device tensor
        pts = sum(span(r0, r1, desc.out_oy, desc.out_step, desc.Hg) * span(c0, c1, desc.out_ox, desc.out_step, desc.Wg)
                  for r0, c0, r1, c1 in bx)
        return desc.macs * pts / (desc.B * desc.Hg * desc.Wg)

    # Winograd tiles of po_conv: (tiles = GEMM rows, output channels) per workgroup
    WINO_TILES = {61: (64, 32), 65: (32, 64), 66: (32, 64), 67: (64, 64), 68: (64, 64), 70: (64, 64),
                  71: (32, 64), 72: (32, 64)}   # 62-64 retired
    # output-tile side and transform components of each Winograd tile: F(2x2,3x3)
    # (16), except tiles 71/72, F(4x4,3x3) (36)
    WINO_SIDE = {71: 4, 72: 4}
    WINO_COMPS = {71: 36, 72: 36}
    HALO_TILE = 69               # conv_halo_pool_k (conv_halo.hip)
    WPOOL_TILE = 73              # conv_wpool_k (conv_wpool.hip): tile 69's launch as Winograd F(2x2,3x3)
    _tile_shapes = {}

    @classmethod
    def tile_shape(cls, t):
        """(BM, BN, BK) of po_conv tile t (po_conv_tile_info)."""
        if t not in cls._tile_shapes:
            bm, bn, bk, pr = nat.c_int(), nat.c_int(), nat.c_int(), nat.c_int()
            nat.call("po_conv_tile_info", t, nat.ctypes.byref(bm), nat.ctypes.byref(bn), nat.ctypes.byref(bk),
                     nat.ctypes.byref(pr))
            cls._tile_shapes[t] = (bm.value, bn.value, bk.value)
        return cls._tile_shapes[t]

    @classmethod
    def launch_mfma_flops(cls, desc, cones=None):
        """FLOPs the matrix cores EXECUTE for one exact-fp32 po_conv launch
        (v_mfma_f32_32x32x2_f32, 4096 FLOP each), as the kernels enumerate
        their work: every workgroup that holds a live row runs its whole
        BM x BN tile over every k-step (padded channels, ragged tile rows and
        the dead rows of a boxed workgroup included; a workgroup whose rows
        are all dead exits before its first MFMA).

        * direct tiles: 2 * live M-tiles * BM * ceil(N/BN)*BN * ntaps * Cin_p;
        * Winograd F(2x2,3x3) tiles (61-70): 2 * 16 * live workgroups * WT
          * Cin_p * N — 16 transform-domain GEMMs over the 2x2 output tiles,
          4/9 of the direct-conv MFMA work of the same launch; F(4x4,3x3)
          (tile 71): 2 * 36 * live units * 32 4x4-tiles * Cin_p * N, 1/4 of
          the direct work (9/16 of F(2x2)'s).
        Boxed launches (gbox) count the live rows of this step's boxes
        (conv_common.h grid_point / conv_wino.hip tile_point)."""
        if desc.prec != 0:
            return None
        t = desc.tile
        if t in cls.WINO_TILES:
            WT = cls.WINO_TILES[t][0]
            return 2.0 * cls.WINO_COMPS.get(t, 16) * cls._live_tiles(desc, t, WT, cones) * WT * desc.Cin_p * desc.N
        if t == cls.WPOOL_TILE:
            # conv_wpool_k: 8 x 16-pixel output tiles (ragged ones padded) = 32
            # 2x2 Winograd tiles, 16 transform-domain GEMMs over Cin_p x 32 channels
            return 2.0 * 16 * desc.B * (-(-desc.Hg // 8)) * (-(-desc.Wg // 16)) * 32 * desc.Cin_p * 32
        if t == cls.HALO_TILE:
            # conv_halo_pool_k: 8 x 16-pixel output tiles (ragged ones padded), 32
            # channels, K = 9 taps x 16 channels (full maps only: no boxes)
            return 2.0 * desc.B * (-(-desc.Hg // 8)) * (-(-desc.Wg // 16)) * 128 * 32 * desc.ntaps * desc.Cin_p
        BM, BN, BK = cls.tile_shape(t)
        return 2.0 * cls._live_tiles(desc, t, BM, cones) * BM * (-(-desc.N // BN) * BN) * desc.ntaps * desc.Cin_p

    @classmethod
    def _live_tiles(cls, desc, t, bm, cones=None):
        """GEMM-row workgroups of tile t (bm rows; Winograd: WT 2x2 tiles)
        that hold a live row (all of them for a full grid)."""
        boxes = None
        if getattr(desc, "support", None) is not None:
            boxes = desc.support.cpu().tolist()
        elif desc.gbox and cones is not None:
            boxes = cones[desc.cone_block, desc.cone_b0:desc.cone_b0 + desc.B].tolist()
        if t in cls.WINO_TILES:
            WT = cls.WINO_TILES[t][0]
            q = cls.WINO_SIDE.get(t, 2)
            Ht, Wt = -(-desc.Hg // q), -(-desc.Wg // q)
            per = Ht * Wt
            live = [per] * desc.B if boxes is None else [
                min(max(-(-r1 // q) - r0 // q, 0) * max(-(-c1 // q) - c0 // q, 0), per)
                for r0, c0, r1, c1 in boxes]
            return cls._live_groups(live, per, WT, desc.B)
        mrows = desc.mrows or desc.Hg * desc.Wg
        if boxes is None:
            return -(-(desc.B * mrows) // bm)

        def span(lo, hi, off, step, n):
            a = 0 if lo - off <= 0 else -(-(lo - off) // step)
            b = 0 if hi - 1 - off < 0 else min(n, (hi - 1 - off) // step + 1)
            return max(b - a, 0)
        live = [min(span(r0, r1, desc.out_oy, desc.out_step, desc.Hg) * span(c0, c1, desc.out_ox, desc.out_step, desc.Wg),
                    mrows) for r0, c0, r1, c1 in boxes]
        return cls._live_groups(live, mrows, bm, desc.B)

    @staticmethod
    def _live_groups(live, per, rows, B):
        """Workgroups of ``rows`` consecutive GEMM rows (image b owns rows
        [b*per, b*per + per), its first live[b] of them live) holding a live row."""
        if all(n == per for n in live):
            return -(-(B * per) // rows)
        ids = set()
        for b, n in enumerate(live):
            if n > 0:
                ids.update(range((b * per) // rows, (b * per + n - 1) // rows + 1))
        return len(ids)

    def _cone_ptr(self, s, b0):
        """po_conv gbox of a dgrad writing block s's gradient (images from b0)."""
        if s == INPUT or s not in self.cone_blocks:
            return None
        return self.cone_boxes[s, b0].data_ptr()

    # ---------------- gradient bookkeeping ----------------
    def _build_grad_plan(self):
        n, blocks, root = self.n, self.net.blocks, self.root
        has = [False] * n
        for j in range(n - 1, -1, -1):
            t = blocks[j]["type"]
            if t == "yolo":
                has[root[j]] = True
            elif root[j] == j and has[j]:
                for s in self.srcs[j]:
                    if s != INPUT:
                        has[s] = True
        self.has_grad = has
        ncons = [0] * n
        ext = [0] * n
        for j in range(n):
            t = blocks[j]["type"]
            if t == "yolo":
                ext[root[j]] += 1
            elif t == "route" and len(self.srcs[j]) == 1:
                continue
            elif root[j] == j and has[j]:
                for s in self.srcs[j]:
                    if s != INPUT:
                        ncons[s] += 1
        self.ncons, self.ext = ncons, ext
        # Residual stages share one gradient buffer: for a shortcut s = y_b + x_f
        # whose input f is consumed only by s and earlier blocks, dL/dx_f =
        # dL/ds + (contributions processed after s), so G_f aliases G_s and the
        # shortcut costs no pass; dL/dy_b = dL/ds * leaky'(y_b) is emitted as the
        # second epilogue output of the dgrad that completes G_s.
        consumers = [[] for _ in range(n)]
        for j in range(n):
            t = blocks[j]["type"]
            if t == "yolo" or (t == "route" and len(self.srcs[j]) == 1) or root[j] != j or not has[j]:
                continue
            for s in self.srcs[j]:
                if s != INPUT:
                    consumers[s].append(j)
        self.consumers = consumers
        self.sc_alias = {}
        for s in range(n):
            d = blocks[s]
            if d["type"] != "shortcut" or root[s] != s or not has[s]:
                continue
            b, f = self.srcs[s]
            if f == b or ext[f] or not has[f] or root[f] != f:
                continue
            if all(j <= s for j in consumers[f]) and consumers[b] == [s] and self._leaky(b):
                self.sc_alias[s] = (b, f)
        dev, B = self.device, self.B
        self.grad = [None] * n
        for i in range(n - 1, -1, -1):
            if root[i] == i and has[i] and self.grad[i] is None:
                self.grad[i] = torch.zeros(B, self.dims[i][0], self.dims[i][1], self.cp[i], device=dev)
            if i in self.sc_alias:
                self.grad[self.sc_alias[i][1]] = self.grad[i]

    def _leaky(self, r):
        return (self.net.blocks[r]["type"] == "convolutional" and self.net._conv_meta[r]["act"] == "leaky")

    # ---------------- max|x| slots (fp16x3 operand scales) ----------------
    def _build_slots(self):
        """One uint32 slot per activation/gradient tensor: every kernel writing
        the tensor atomicMax's max|value| into it, and a fp16x3 po_conv reading
        it as its A operand takes its power-of-two scale from it (zeroed at the
        start of every forward)."""
        idx = {}
        for t in self.act + self.grad + [self.in_nhwc]:
            if t is not None and t.data_ptr() not in idx:
                idx[t.data_ptr()] = len(idx)
        self._slot_idx = idx
        self.amax = torch.zeros(len(idx), nat.PO_AMAX_SUB, dtype=torch.int32, device=self.device)

    def _build_bits(self):
        """Sign bits of the leaky conv outputs that the backward uses as
        LeakyReLU masks: written by the forward conv epilogue, read by the
        dgrad epilogues instead of the fp32 activation (1/32 of the bytes).
        Only po_conv outputs with a channel stride that is a multiple of 32."""
        self.bits = {}
        if os.environ.get("ADVPATCH_MASK_BITS", "1") == "0":
            return
        for i, d in enumerate(self.net.blocks):
            if (d["type"] == "convolutional" and self.root[i] == i and self._leaky(i) and self.has_grad[i]
                    and self.cp[i] % 32 == 0 and not (i == 0 and self.first_direct) and i not in self.conv_pool):
                self.bits[self.act[i].data_ptr()] = torch.zeros(self.B, self.dims[i][0], self.dims[i][1],
                                                                self.cp[i] // 32, dtype=torch.int32,
                                                                device=self.device)

    def _img_ptr(self, t, b0):
        """Pointer to image b0 of a [B, ...] tensor (or to a bits tensor given by
        its address: the bits of the activation it belongs to)."""
        if t is None:
            return None
        if isinstance(t, int):
            bt = next(b for b in self.bits.values() if b.data_ptr() == t)
            return nat.c_void_p(t + b0 * bt[0].numel() * bt.element_size())
        return nat.c_void_p(t.data_ptr() + b0 * t[0].numel() * t.element_size())

    def _drop_mask_only_outputs(self):
        """A conv output whose fp32 values no launch reads — the activation
        before a fused shortcut, which the backward uses only as a LeakyReLU
        mask and takes from its sign bits — is not stored: the forward
        epilogue writes only its signs and the shortcut sum
        (ADVPATCH_DROP_MASK_ONLY=0 keeps every output)."""
        self.y_dropped = set()
        if os.environ.get("ADVPATCH_DROP_MASK_ONLY", "1") == "0":
            return
        used = {self.act[h].data_ptr() for h in self.heads}
        for name, args, desc in self.fwd_ops + self.bwd_ops:
            for pos, v in enumerate(args):
                if name == "po_conv" and pos == 4 and desc.kind == "fwd":
                    continue                          # a forward conv's own output
                if isinstance(v, nat.c_void_p) and v.value:
                    used.add(v.value)
        for k, (name, args, desc) in enumerate(self.fwd_ops):
            if name != "po_conv" or args[6] is None or not desc.ybits or args[4].value in used:
                continue
            self.fwd_ops[k] = (name, args[:4] + (None,) + args[5:], desc)
            desc.y_amax = None
            self.y_dropped.add(desc.block)

    def leaky_signs(self, i):
        """bool [B, h, w, C]: output of leaky conv i > 0 — from the fp32
        activation, or from its sign bits when it is not stored."""
        C = self.shp[i][2]
        if (i == 0 and self.first_pool) or i in self.conv_pool:
            return None                         # not stored (fused into the pool: its argmax bytes)
        if i in self.y_dropped:
            bits = self.bits[self.act[i].data_ptr()]
            sh = torch.arange(32, device=bits.device, dtype=torch.int32)
            b = (bits.unsqueeze(-1) >> sh) & 1
            return b.reshape(*bits.shape[:3], -1)[..., :C].bool()
        return self.act[i][..., :C] > 0

    def bits_of(self, t):
        """Device address of the sign-bit copy of activation t (None if it has none)."""
        if t is None or t.data_ptr() not in self.bits:
            return None
        return self.bits[t.data_ptr()].data_ptr()

    def slot(self, t):
        """Device address of tensor t's max|x| slot (None for None, and for
        every tensor of an exact-fp32 plan: only the fp16x3 splits read the
        bounds, and a kernel that commits one waits for its own stores)."""
        if t is None:
            return None
        if self.prec != 1:
            return nat.c_void_p(None)
        return nat.c_void_p(self.amax.data_ptr() + 4 * nat.PO_AMAX_SUB * self._slot_idx[t.data_ptr()])

    def _conv_prec(self, desc, src, wts_or_j, taps=None, cin_p=None):
        """Precision of one po_conv launch and its weight pointer: fp16x3 for
        every conv whose input is a network tensor (the NHWC copy of the image
        has no max|x| slot and keeps exact fp32)."""
        if self.prec == 1 and src != INPUT:
            if taps is None:
                w16, shift = self.net._dev16(wts_or_j)
            else:
                w16, shift = self.net._dgrad_weight16(wts_or_j, taps, cin_p, self.device)
            desc.prec, desc.w_shift = 1, shift
            desc.Wfrag = self.net._frag16(w16)
            return w16
        desc.prec, desc.w_shift = 0, 0
        if taps is None:
            return self.net._dev[wts_or_j]["w"]
        return self.net._dgrad_weight(wts_or_j, taps, cin_p, self.device)

    def _attach_wino(self, desc, w):
        """Winograd weights of an exact-fp32 launch that is a stride-1 3x3
        correlation on full maps: F(2x2,3x3) (po_conv_desc.Wwino, tiles
        61-70) and, where N % 64 == 0, F(4x4,3x3) (Wwino6, tile 71;
        ADVPATCH_WINO4X4=0: not built, so the tuner never picks tile 71)."""
        desc.Wwino = None
        desc.Wwino6 = None
        if (desc.prec != 0 or desc.ntaps != 9 or desc.in_step != 1 or desc.out_step != 1 or desc.in_org
                or desc.out_org or w.dim() != 3 or w.size(0) % 32 or w.size(2) % 16
                or os.environ.get("ADVPATCH_WINOGRAD", "1") == "0"):
            return
        offs = [(desc.dh[t], desc.dw[t]) for t in range(9)]
        if sorted(offs) != [(a, b) for a in (-1, 0, 1) for b in (-1, 0, 1)]:
            return
        desc.Wwino = self.net._wino(w, offs)
        if w.size(0) % 64 == 0 and os.environ.get("ADVPATCH_WINO4X4", "1") != "0":
            desc.Wwino6 = self.net._wino(w, offs, f4=True)

    # ---------------- launch lists ----------------
    def _build_ops(self):
        net, blocks, B = self.net, self.net.blocks, self.B
        lib = self.lib
        P = lambda t: nat.c_void_p(t.data_ptr()) if t is not None else None
        fwd, fblk = [], []

        def fa(op):
            fwd.append(op)
            fblk.append(i)

        for i, d in enumerate(blocks):
            t = d["type"]
            if t == "convolutional":
                m = net._conv_meta[i]
                wts = net._dev[i]
                src = self.srcs[i][0]
                y = self.act[i] if i not in self.fused else None
                fuse_next = (i + 1) in self.fused
                y_out = self.act[i]
                if i == 0 and self.first_pool:
                    args = (None, B, self.H, self.W, P(wts["w27"]), P(wts["bias"]), m["cout"], self.cp[i],
                            1 if m["act"] == "leaky" else 0, P(self.act[1]), P(self.argmax[1]), self.slot(self.act[1]))
                    if self.first_wino:
                        args = args[:4] + (P(wts["u16"]),) + args[5:]
                    fa(("po_conv_first_pool_wino_fwd" if self.first_wino else "po_conv_first_pool_fwd", args, "img0"))
                    assert not fuse_next
                    continue
                if i == 0 and self.first_direct:
                    args = (None, B, self.H, self.W, m["stride"], P(wts["w27"]), P(wts["bias"]), m["cout"],
                            self.cp[i], 1 if m["act"] == "leaky" else 0, P(y_out), self.slot(y_out))
                    fa(("po_conv_first_fwd", args, "img0"))
                    assert not fuse_next
                    continue
                Hin, Win = (self.H, self.W) if src == INPUT else self.dims[src]
                cin_p = 16 if src == INPUT else self.cp[src]
                desc = nat.po_conv_desc()
                desc.B, desc.Hin, desc.Win, desc.Cin_p = B, Hin, Win, cin_p
                desc.Hout, desc.Wout, desc.Cout_p = self.dims[i][0], self.dims[i][1], self.cp[i]
                desc.Hg, desc.Wg = self.dims[i][0], self.dims[i][1]
                desc.in_org, desc.out_org = self._orgp(src), self._orgp(i)
                desc.in_step, desc.out_step, desc.out_oy, desc.out_ox = m["stride"], 1, 0, 0
                k, pad = m["k"], m["pad"]
                desc.ntaps = k * k
                for kh in range(k):
                    for kw in range(k):
                        desc.dh[kh * k + kw] = kh - pad
                        desc.dw[kh * k + kw] = kw - pad
                desc.N = self.cp[i]
                desc.act = 1 if m["act"] == "leaky" else 0
                desc.accumulate = 0
                inp = self.in_nhwc if src == INPUT else self.act[src]
                res = sum_out = None
                if fuse_next:
                    sc = blocks[i + 1]
                    f = int(sc["from"])
                    f = f if f >= 0 else (i + 1) + f
                    res, sum_out = self.act[self.root[f]], self.act[i + 1]
                wptr = self._conv_prec(desc, src, i)
                self._attach_wino(desc, wptr)
                desc.in_amax = self.slot(inp).value if src != INPUT else None
                desc.y_amax = self.slot(y_out).value
                desc.sum_amax = self.slot(sum_out).value if sum_out is not None else None
                desc.ybits = self.bits_of(y_out)
                y_ptr = P(y_out)
                if i in self.conv_pool:               # the pool output instead of the conv output
                    desc.pool_y, desc.pool_argmax = self.act[i + 1].data_ptr(), self.argmax[i + 1].data_ptr()
                    desc.y_amax = self.slot(self.act[i + 1]).value
                    desc.ybits = None
                    y_ptr = None
                args = (nat.ctypes.byref(desc), P(inp), P(wptr), P(wts["bias"]), y_ptr, P(res),
                        P(sum_out), None, None, None)
                desc.macs = B * desc.Hg * desc.Wg * m["cout"] * m["cin"] * k * k      # logical channels
                desc.block, desc.kind = i, "fwd"
                fa(("po_conv", args, desc))
            elif t == "shortcut":
                if i in self.fused:
                    continue
                a, b = self.srcs[i]
                M = B * self.dims[i][0] * self.dims[i][1]
                C = self.shp[i][2]
                fa(("po_slice_accum", (P(self.act[a]), self.cp[a], 0, P(self.act[i]), self.cp[i], 0, M, C, 0,
                                               None, 0, self.slot(self.act[i])), None))
                fa(("po_slice_accum", (P(self.act[b]), self.cp[b], 0, P(self.act[i]), self.cp[i], 0, M, C, 1,
                                               None, 0, self.slot(self.act[i])), None))
            elif t == "route":
                if len(self.srcs[i]) == 1:
                    continue
                off = 0
                M = B * self.dims[i][0] * self.dims[i][1]
                for s in self.srcs[i]:
                    C = self.shp[s][2]
                    if self._same_view(s, i):
                        fa(("po_slice_accum", (P(self.act[s]), self.cp[s], 0, P(self.act[i]), self.cp[i], off,
                                                       M, C, 0, None, 0, self.slot(self.act[i])), None))
                    else:
                        fa(("po_view_move", self._move(self.act[s], s, 0, self.act[i], i, off, C, 0, 0, None),
                                    None))
                    off += C
            elif t == "upsample":
                s = self.srcs[i][0]
                hs, ws_, cs = self.shp[s]
                if self.win[i] is None and self.win[s] is None:
                    fa(("po_upsample2_fwd", (P(self.act[s]), B, hs, ws_, cs, self.cp[s], P(self.act[i]),
                                                     self.cp[i], 0, self.slot(self.act[i])), None))
                else:
                    fa(("po_view_move", self._move(self.act[s], s, 0, self.act[i], i, 0, cs, 1, 0, None),
                                None))
            elif t == "maxpool":
                if (i == 1 and self.first_pool) or (i - 1) in self.conv_pool:
                    continue                    # fused into the producing conv
                s = self.srcs[i][0]
                hs, ws_, cs = self.shp[s]
                fa(("po_maxpool2_fwd", (P(self.act[s]), B, hs, ws_, cs, self.cp[s], int(d["stride"]),
                                                P(self.act[i]), P(self.argmax[i]), self.slot(self.act[i])), None))
        self.fwd_ops, self.fwd_blk = fwd, fblk

        # backward
        bwd, bblk = [], []

        def ba(op):
            bwd.append(op)
            bblk.append(j)

        done = [0] * self.n
        root = self.root
        for r in range(self.n):
            if self.ext[r] and root[r] == r and self.has_grad[r]:
                done[r] += 1        # the head gradient is copied in first (run_backward)

        def contrib(r):
            """(accumulate?, leaky mask or None, completes G_r?) of the next
            gradient contribution to block r."""
            acc = 1 if done[r] > 0 else 0
            final = (done[r] + 1 - (1 if self.ext[r] else 0)) == self.ncons[r]
            mask = self.act[r] if (final and self._leaky(r)) else None
            done[r] += 1
            return acc, mask, final

        def dual_of(r, final):
            """second output when this contribution completes an aliased shortcut's G."""
            if final and r in self.sc_alias:
                b, _ = self.sc_alias[r]
                acc_b, mask_b, fin_b = contrib(b)
                assert acc_b == 0 and fin_b and mask_b is not None
                return self.grad[b], self.act[b]
            return None, None

        def fallback_dual(r, final):
            # the completing contribution was not a conv dgrad: extract dL/dy_b with a masked copy
            if final and r in self.sc_alias:
                b, _ = self.sc_alias[r]
                _, mask_b, _ = contrib(b)
                M = self.B * self.dims[r][0] * self.dims[r][1]
                ba(("po_slice_accum", (P(self.grad[r]), self.cp[r], 0, P(self.grad[b]), self.cp[b], 0, M,
                                               self.shp[r][2], 0, P(mask_b), self.cp[b], self.slot(self.grad[b])),
                            None))

        for j in range(self.n - 1, -1, -1):
            d = blocks[j]
            t = d["type"]
            if root[j] != j or not self.has_grad[j] or t == "yolo":
                continue
            G = self.grad[j]
            if t == "convolutional":
                m = net._conv_meta[j]
                wts = net._dev[j]
                src = self.srcs[j][0]
                if src == INPUT:
                    if self.first_direct:
                        ba(("po_conv_first_dgrad", (P(G), B, self.H, self.W, m["stride"], P(wts["w27"]),
                                                            m["cout"], self.cp[j], "roi", "dimg"), None))
                    else:
                        for desc, wd, b0 in self._dgrad_descs(j, INPUT, 0, G, self.in_nhwc):
                            ba(("po_conv", (nat.ctypes.byref(desc), self._img_ptr(G, b0), P(wd), None,
                                                    self._img_ptr(self.in_nhwc, b0), None,
                                                    None, None, None, None), desc))
                        ba(("po_nhwc_to_nchw", (P(self.in_nhwc), B, self.H, self.W, 3, 16, "dimg"), None))
                    continue
                acc, mask, final = contrib(src)
                y2, m2 = dual_of(src, final)
                for desc, wd, b0 in self._dgrad_descs(j, src, acc, G, self.grad[src], y2):
                    if desc.mrows:
                        ba(("zero", (self.grad[src],), None))
                    Pb = lambda t: self._img_ptr(t, b0)
                    if not desc.mrows:
                        desc.gbox = self._cone_ptr(src, b0)
                        desc.cone_block, desc.cone_b0 = src, b0
                    mb, m2b = self._img_ptr(self.bits_of(mask), b0), self._img_ptr(self.bits_of(m2), b0)
                    desc.mbits = mb.value if mb is not None else None
                    desc.m2bits = m2b.value if m2b is not None else None
                    ba(("po_conv", (nat.ctypes.byref(desc), Pb(G), P(wd), None, Pb(self.grad[src]), None, None,
                                            None if desc.mbits else Pb(mask), Pb(y2),
                                            None if desc.m2bits else Pb(m2)), desc))
            elif t == "shortcut":
                if j in self.sc_alias:
                    b, f = self.sc_alias[j]
                    acc, mask, final = contrib(f)      # implicit: G_f aliases G_s
                    assert acc == 0
                    if mask is not None:               # f has no later contributor: apply its mask in place
                        M = self.B * self.dims[f][0] * self.dims[f][1]
                        ba(("po_slice_accum", (P(G), self.cp[j], 0, P(self.grad[f]), self.cp[f], 0, M,
                                                       self.shp[f][2], 0, P(mask), self.cp[f], self.slot(self.grad[f])),
                                    None))
                    continue
                M = self.B * self.dims[j][0] * self.dims[j][1]
                C = self.shp[j][2]
                for s_ in self.srcs[j]:
                    acc, mask, final = contrib(s_)
                    ba(("po_slice_accum", (P(G), self.cp[j], 0, P(self.grad[s_]), self.cp[s_], 0, M, C, acc,
                                                   P(mask), self.cp[s_], self.slot(self.grad[s_])), None))
                    fallback_dual(s_, final)
            elif t == "route":
                off = 0
                M = self.B * self.dims[j][0] * self.dims[j][1]
                for s_ in self.srcs[j]:
                    C = self.shp[s_][2]
                    acc, mask, final = contrib(s_)
                    if self._same_view(s_, j):
                        ba(("po_slice_accum", (P(G), self.cp[j], off, P(self.grad[s_]), self.cp[s_], 0, M, C,
                                                       acc, P(mask), self.cp[s_], self.slot(self.grad[s_])), None))
                    else:
                        ba(("po_view_move", self._move(G, j, off, self.grad[s_], s_, 0, C, 0, acc, mask),
                                    None))
                    fallback_dual(s_, final)
                    off += C
            elif t == "upsample":
                s_ = self.srcs[j][0]
                acc, mask, final = contrib(s_)
                hs, ws_, cs = self.shp[s_]
                if self.win[j] is None and self.win[s_] is None:
                    ba(("po_upsample2_bwd", (P(G), self.cp[j], 0, B, hs, ws_, cs, P(self.grad[s_]),
                                                     self.cp[s_], acc, P(mask), self.cp[s_], self.slot(self.grad[s_])),
                                None))
                else:
                    ba(("po_view_move", self._move(G, j, 0, self.grad[s_], s_, 0, cs, 2, acc, mask), None))
                fallback_dual(s_, final)
            elif t == "maxpool":
                s_ = self.srcs[j][0]
                acc, mask, final = contrib(s_)
                if (j == 1 and self.first_pool) or s_ in self.conv_pool:
                    # the LeakyReLU slopes come from the argmax bytes (the conv output is not stored)
                    assert acc == 0 and final
                    mask = None
                hs, ws_, cs = self.shp[s_]
                # on a gradient-cone source only its per-image boxes are written
                cone = self._cone_ptr(s_, 0)
                ba(("po_maxpool2_bwd_box", (P(G), P(self.argmax[j]), B, hs, ws_, cs, self.cp[s_],
                                                    int(d["stride"]), P(self.grad[s_]), acc, P(mask),
                                                    nat.c_void_p(cone) if cone else None,
                                                    self.slot(self.grad[s_])), None))
                fallback_dual(s_, final)
        self.bwd_ops, self.bwd_blk = bwd, bblk

    # ---------------- head tails on a second stream ----------------
    def _plan_tails(self):
        """Head tails: the chain of convs that feeds a YOLO head and nothing
        else (yolov3: blocks 80-81 and 92-93; yolov3-tiny: 14-15), after the
        branch point b whose other consumer carries on to the next head.
        Their launches (receptive-field windows: small, latency-bound) run on
        a second stream concurrently with the main chain: in the forward from
        the end of block b on, joined before the heads are returned; in the
        backward from the head-gradient copy on, except the group that
        accumulates into grad[b], which runs in its place of the original
        order (the accumulation order, hence the bits, are unchanged) with the
        main stream waiting on it.  The last head's tail has nothing after it
        to overlap and stays on the main stream.  Opt-in (ADVPATCH_STREAMS=1):
        measured not to pay on the bench plans (interleaved A/B, yolov3 B=16:
        887/889 img/s with the second stream against 903/889 without;
        profiles/r04/streams_ab.txt), the tails' windows being too small to
        fill what the main chain leaves idle."""
        self.tails = []
        self.side = None
        self.ws_side = None
        if os.environ.get("ADVPATCH_STREAMS", "0") != "1" or torch.device(self.device).type != "cuda":
            return
        for chain, src in self.tail_chains():
            tail = set(chain)
            f_ops = [k for k, b in enumerate(self.fwd_blk) if b in tail]
            trigger = max(k for k, b in enumerate(self.fwd_blk) if b <= src)
            b_early = [k for k, b in enumerate(self.bwd_blk) if b in tail and b != chain[0]]
            b_final = [k for k, b in enumerate(self.bwd_blk) if b == chain[0]]
            if not f_ops or not b_final or trigger >= f_ops[0]:
                continue
            self.tails.append({"blocks": chain, "branch": src, "fwd": f_ops, "trigger": trigger,
                               "bwd_early": b_early, "bwd_final": b_final})
        if self.tails:
            self.side = torch.cuda.Stream(device=self.device)
            self._side_f = {k for t in self.tails for k in t["fwd"]}
            self._trig_f = {}
            for t in self.tails:
                self._trig_f.setdefault(t["trigger"], []).append(t)
            self._side_b = {k for t in self.tails for k in t["bwd_early"] + t["bwd_final"]}
            self._final_b = {t["bwd_final"][0]: t for t in self.tails}
            self.bind_side_workspace()

    def tail_chains(self):
        """[(tail blocks in forward order, branch point b)] of every head but
        the last: the convs from b's consumer up to the YOLO layer, each the
        only consumer of the one before."""
        blocks, n = self.net.blocks, self.n
        cons = [set() for _ in range(n)]
        for i in range(n):
            for src in self.srcs[i]:
                if src != INPUT:
                    cons[src].add(i)
        out = []
        for y in self.heads:
            chain, nxt, src = [], y, self.srcs[y][0]
            while (src != INPUT and blocks[src]["type"] == "convolutional" and self.root[src] == src
                   and cons[src] == {nxt} and src not in self.fused and (src + 1) not in self.fused
                   and src not in self.conv_pool):
                chain.append(src)
                nxt, src = src, self.srcs[src][0]
            if not chain or src == INPUT or src in self.sc_alias or any(src in v for v in self.sc_alias.values()):
                continue
            chain.reverse()                       # forward order: chain[0] reads act[b]
            if not any(i > chain[-1] and blocks[i]["type"] != "yolo" and i not in chain for i in range(n)):
                continue                          # the last head: nothing after it to overlap
            out.append((chain, src))
        return out

    def _side_descs(self):
        for t in self.tails:
            for k in t["fwd"]:
                if self.fwd_ops[k][0] == "po_conv":
                    yield self.fwd_ops[k][2]
            for k in t["bwd_early"] + t["bwd_final"]:
                if self.bwd_ops[k][0] == "po_conv":
                    yield self.bwd_ops[k][2]

    def bind_side_workspace(self):
        """Split-K launches on the second stream get their own workspace (the
        main one is stream-ordered on the main stream only)."""
        if not self.tails:
            return
        need = max([d.ksplit * d.B * d.Hg * d.Wg * d.N for d in self._side_descs() if d.ksplit > 1] + [0])
        if need and (self.ws_side is None or self.ws_side.numel() < need):
            self.ws_side = torch.empty(need, device=self.device)
        for d in self._side_descs():
            if d.ksplit > 1:
                d.workspace = self.ws_side.data_ptr()
                if d.tile_ctr:
                    d.tile_ctr = self._tile_ctr(side=True).data_ptr()
        need = max([self.winov_floats(d) for d in self._side_descs() if d.tile == self.WINOV_TILE] + [0])
        if need:
            if getattr(self, "winov_side", None) is None or self.winov_side.numel() < need:
                self.winov_side = torch.empty(need, device=self.device)
            for d in self._side_descs():
                if d.tile == self.WINOV_TILE:
                    d.winov, d.winov_floats = self.winov_side.data_ptr(), self.winov_floats(d)

    def _orgp(self, i):
        o = self.org_of(i)
        return o.data_ptr() if o is not None else None

    def _same_view(self, a, b):
        """Blocks a and b have buffers of the same spatial layout (both full
        maps, or the same window)."""
        ra, rb = self.root[a], self.root[b]
        if self.win[ra] is None and self.win[rb] is None:
            return True
        return self.win[ra] is not None and self.win_idx.get(ra) == self.win_idx.get(rb)

    def _move(self, src, si, soff, dst, di, doff, C, mode, acc, mask):
        """po_view_move arguments: dst block di (=|+=) src block si (spatial views)."""
        P = lambda t: nat.c_void_p(t.data_ptr()) if t is not None else None
        Hs, Ws = self.dims[si]
        Hd, Wd = self.dims[di]
        o = lambda i: nat.c_void_p(self._orgp(i)) if self._orgp(i) is not None else None
        return (P(src), Hs, Ws, self.cp[si], soff, o(si), P(dst), Hd, Wd, self.cp[di], doff, o(di), self.B, C,
                mode, acc, P(mask), self.cp[di], self.slot(dst))

    def _dgrad_descs(self, j, src, acc, G, dst, dst2=None):
        """po_conv launches computing d(input of conv j) (one per stride parity
        class): G = dL/d(output of j), dst (and dst2, the dual output) receive
        the input gradient."""
        m = self.net._conv_meta[j]
        s, k, pad = m["stride"], m["k"], m["pad"]
        if self.win[j] is not None or (src != INPUT and self.win[src] is not None):
            assert s == 1, "windowed dgrad needs a stride-1 conv"
            Hin, Win = self.dims[src]
        else:
            Hin, Win = (self.H, self.W) if src == INPUT else self.shp[src][:2]
        cin_p = 16 if src == INPUT else self.cp[src]
        out = []
        # one launch per parity class over the whole batch (image-range groups,
        # ``groups``, measured no faster: the G re-reads hit the Infinity Cache)
        groups = [(0, self.B)]
        for (b0, nb), py, px in [(g, py, px) for g in groups for py in range(s) for px in range(s)]:
            Hg = (Hin - py + s - 1) // s
            Wg = (Win - px + s - 1) // s
            if Hg <= 0 or Wg <= 0:
                continue
            taps = [(kh, kw) for kh in range(k) for kw in range(k)
                    if (py + pad - kh) % s == 0 and (px + pad - kw) % s == 0]
            desc = nat.po_conv_desc()
            wd = self._conv_prec(desc, src, j, taps, cin_p)
            desc.in_amax = self.slot(G).value
            desc.y_amax = self.slot(dst).value
            desc.y2_amax = self.slot(dst2).value if dst2 is not None else None
            desc.B, desc.Hin, desc.Win, desc.Cin_p = nb, self.dims[j][0], self.dims[j][1], self.cp[j]
            desc.Hout, desc.Wout, desc.Cout_p = Hin, Win, cin_p
            desc.in_org, desc.out_org = self._orgp(j), (self._orgp(src) if src != INPUT else None)
            desc.Hg, desc.Wg = Hg, Wg
            desc.in_step, desc.out_step, desc.out_oy, desc.out_ox = 1, s, py, px
            desc.ntaps = len(taps)
            for ti, (kh, kw) in enumerate(taps):
                desc.dh[ti] = (py + pad - kh) // s
                desc.dw[ti] = (px + pad - kw) // s
            desc.N = cin_p
            self._attach_wino(desc, wd)
            desc.act = 0
            desc.accumulate = acc
            desc.macs = nb * Hg * Wg * m["cin"] * len(taps) * m["cout"]
            desc.block, desc.kind = j, "dgrad"
            self._support_grid(desc, j, src, acc, dst, dst2, b0)
            out.append((desc, wd, b0))
        return out

    def _support_grid(self, desc, j, src, acc, dst, dst2, b0):
        """A dgrad from a receptive-field window (G_j lives on a window of side
        w) into a full map is nonzero only on the window dilated by the taps:
        rows [org - max(dh), org + w - min(dh)), columns likewise.  Such a
        launch runs over that box only — a compact grid of mrows points per
        image with per-step boxes (po_conv gbox, ∩ the gradient cone), the
        destination zero-filled first (its consumers read the whole map).
        Only first contributions (acc = 0) without a dual output.  Off with
        ADVPATCH_SUPPORT_BOX=0."""
        if (os.environ.get("ADVPATCH_SUPPORT_BOX", "1") == "0" or src == INPUT or self.win[j] is None
                or self.win[src] is not None or acc or dst2 is not None or desc.in_step != 1
                or desc.out_step != 1 or desc.Wwino):
            return
        if sum(1 for g in self.grad if g is not None and g.data_ptr() == dst.data_ptr()) > 1:
            return                              # a shared (residual) gradient buffer: no zero fill
        dh = [desc.dh[t] for t in range(desc.ntaps)]
        dw = [desc.dw[t] for t in range(desc.ntaps)]
        w = self.win[j]
        hr, wc = min(w + max(dh) - min(dh), desc.Hg), min(w + max(dw) - min(dw), desc.Wg)
        if hr * wc >= desc.Hg * desc.Wg:
            return
        box = torch.zeros(desc.B, 4, dtype=torch.int32, device=self.device)
        self.support.append((box, j, src, b0, desc.B, (max(dh), min(dh), max(dw), min(dw)), dst))
        desc.gbox = box.data_ptr()
        desc.mrows = hr * wc
        desc.macs = desc.macs * desc.mrows // (desc.Hg * desc.Wg)
        desc.cone_block = None                  # launch_macs: counted over the support boxes
        desc.support = box

    def set_support_boxes(self):
        """Per-step support boxes of the compact dgrad grids (after set_cones):
        the window dilated by the taps, clipped to the map, ∩ the cone box --
        every entry in one po_support_boxes launch."""
        if not self.support:
            return
        key = tuple(e[0].data_ptr() for e in self.support) + (self.cone_boxes is not None,)
        if getattr(self, "_support_key", None) != key:          # (re)built with the op list
            rows, ptrs = [], []
            for box, j, src, b0, nb, (dh1, dh0, dw1, dw0), _ in self.support:
                H, W = self.shp[src][:2]
                cone = src if (self.cone_boxes is not None and src in self.cone_blocks) else -1
                rows.append([self.win_idx[self.root[j]], b0, nb, dh1, dh0, dw1, dw0, H, W, self.win[j], cone, 0])
                ptrs.append(box.data_ptr())
            self._support_prog = torch.tensor(rows, dtype=torch.int32, device=self.device)
            self._support_dst = torch.tensor(ptrs, dtype=torch.int64, device=self.device)
            self._support_key = key
        nat.call("po_support_boxes", nat.ptr(self.org, torch.int32), nat.ptr(self.cone_boxes, torch.int32),
                 nat.ptr(self._support_prog, torch.int32), nat.ptr(self._support_dst, torch.int64),
                 len(self.support), self.B, nat.stream())

    def set_support_boxes_torch(self):
        """The torch-op restatement of set_support_boxes (tests)."""
        for box, j, src, b0, nb, (dh1, dh0, dw1, dw0), _ in self.support:
            org = self.org_of(j)[b0:b0 + nb]
            H, W = self.shp[src][:2]
            w = self.win[j]
            r0 = (org[:, 0] - dh1).clamp(0, H)
            c0 = (org[:, 1] - dw1).clamp(0, W)
            r1 = (org[:, 0] + w - dh0).clamp(0, H)
            c1 = (org[:, 1] + w - dw0).clamp(0, W)
            bx = torch.stack([r0, c0, r1, c1], 1)
            if self.cone_boxes is not None and src in self.cone_blocks:
                cb = self.cone_boxes[src, b0:b0 + nb]
                bx = torch.cat([torch.maximum(bx[:, :2], cb[:, :2]), torch.minimum(bx[:, 2:], cb[:, 2:])], 1)
            box.copy_(bx)

    def conv_macs(self):
        """MACs (logical channels) of the po_conv launches of one forward +
        backward of this plan — the work the MFMA kernel does per step."""
        return sum(d.macs for name, _, d in self.fwd_ops + self.bwd_ops if name == "po_conv")

    # ---------------- autotuning ----------------
    SPLITS = (2, 4, 8, 16, 32)
    WS_FLOATS = 64 << 20          # split-K workspace cap (256 MB)
    WINO_SPLIT_TILES = (66, 67, 68, 70, 71, 72)   # Winograd tiles with split-K (conv_wino3_k .. conv_wino6_k)
    WINOV_TILE = 72               # F(4x4,3x3) on an input transformed beforehand (po_conv_desc.winov)

    def _ensure_ws(self, floats):
        if self.ws is None or self.ws.numel() < floats:
            self.ws = torch.empty(floats, device=self.device)
        return self.ws

    def tune(self, cache, iters=4, time_missing=True):
        """Time every candidate (tile, split-K) of po_conv for each distinct
        launch shape of this plan on the current GPU and keep the fastest
        (wave quantisation over the 256 CUs, the k-step size and, for launches
        with few tiles — the receptive-field windows — splitting K over more
        workgroups decide it per shape).  ``cache`` maps a launch signature
        to (tile, ksplit) and is shared between plans.  ``time_missing``
        False (ADVPATCH_TUNE=cache): shapes not in the cache keep the
        built-in heuristic instead of being timed, so a run is bit-for-bit
        reproducible from the committed cache alone."""
        lib = self.lib
        st = nat.stream()
        convs = [(args, desc) for name, args, desc in self.fwd_ops + self.bwd_ops if name == "po_conv"]
        if not time_missing:
            for args, desc in convs:
                key = self._tune_key(args, desc)
                if key in cache and self._cached_ok(desc, cache[key]):
                    self._set_tile(desc, cache[key])
            for args, desc in convs:                 # the workspaces may have grown
                if desc.ksplit > 1:
                    desc.workspace = self.ws.data_ptr()
                if desc.tile == self.WINOV_TILE:
                    desc.winov = self.winov.data_ptr()
            self.bind_side_workspace()
            return
        if all(self._tune_key(args, desc) in cache and self._cached_ok(desc, cache[self._tune_key(args, desc)])
               for args, desc in convs):
            for args, desc in convs:                 # every shape already tuned: no launches
                self._set_tile(desc, cache[self._tune_key(args, desc)])
            for args, desc in convs:
                if desc.ksplit > 1:
                    desc.workspace = self.ws.data_ptr()
                if desc.tile == self.WINOV_TILE:
                    desc.winov = self.winov.data_ptr()
            self.bind_side_workspace()
            return
        bufs = {id(t): t for t in self.act + self.grad if t is not None}
        if self.in_nhwc is not None:
            bufs[id(self.in_nhwc)] = self.in_nhwc
        with torch.no_grad():
            for t in bufs.values():
                t.uniform_(-1.0, 1.0)           # time on random data, not zeros (clock)
        self.amax.fill_(0x3F800000)             # max|x| = 1.0 for the U(-1,1) buffers
        self.join_cone_stream()                 # no early cone evaluation still writing cone_boxes
        if self.cone_boxes is not None:         # boxed dgrads: time them on training-like footprints
            self.set_cones(self.tuning_rois())
        self.set_support_boxes()                # compact dgrad grids: boxes at the current window origins
        tiles = []
        for t in range(1, nat.PO_CONV_NTILES + 1):
            bm, bn, bk, pr = nat.c_int(), nat.c_int(), nat.c_int(), nat.c_int()
            nat.call("po_conv_tile_info", t, nat.ctypes.byref(bm), nat.ctypes.byref(bn), nat.ctypes.byref(bk),
                     nat.ctypes.byref(pr))
            tiles.append((t, bm.value, bn.value, bk.value, pr.value))
        cones_host = self.cone_boxes.cpu() if self.cone_boxes is not None else None
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for name, args, desc in self.fwd_ops + self.bwd_ops:
            if name != "po_conv":
                continue
            key = self._tune_key(args, desc)
            if key in cache and self._cached_ok(desc, cache[key]):
                self._set_tile(desc, cache[key])
                continue
            M = desc.B * (desc.mrows or desc.Hg * desc.Wg)
            best = None
            timed = []
            for t, bm, bn, bk, pr in tiles:
                if pr != desc.prec or desc.Cin_p % bk:
                    continue
                if bn > max(32, desc.N):
                    continue
                # workgroups that hold live rows (a boxed launch: those of the tuning boxes)
                live = self._live_tiles(desc, t, bm, cones_host)
                ntiles = live * -(-desc.N // bn)
                nks = desc.ntaps * desc.Cin_p // bk
                cands = [1]
                if t in self.WINO_TILES:
                    if t in self.WINO_SPLIT_TILES and not desc.pool_y:
                        # input-channel slices re-quantise a Winograd launch whose
                        # workgroup count fills the 512 slots badly (19x19 maps: 800)
                        # or that has few live workgroups (small gradient-cone boxes)
                        ks_ok = (2, 3, 4, 6, 8) if ntiles < 512 else (2, 3)
                        cands += [k for k in ks_ok if desc.Cin_p // bk // k >= 4 and k * M * desc.N <= self.WS_FLOATS]
                elif ntiles < 256:
                    cands += [k for k in self.SPLITS if k * ntiles <= 2048 and nks // k >= 4
                              and k * M * desc.N <= self.WS_FLOATS]
                for ks in cands:
                    self._set_tile(desc, (t, ks))
                    if lib.po_conv(*args, st) != 0:      # tile not applicable to this launch
                        continue
                    for _ in range(1):
                        lib.po_conv(*args, st)
                    e0.record()
                    for _ in range(iters):
                        lib.po_conv(*args, st)
                    e1.record()
                    e1.synchronize()
                    ms = e0.elapsed_time(e1)
                    timed.append((ms, (t, ks)))
                    if best is None or ms < best[0]:
                        best = (ms, (t, ks))
            if best is None:
                raise RuntimeError("po_conv: no tile applies to launch %s (%s)" % (key, nat.last_error()))
            # refinement: the three fastest candidates again, in interleaved
            # rounds of longer runs, keeping each one's best round (a single
            # short timing per candidate picks noisily between close tiles)
            finalists = [c for _, c in sorted(timed)[:3]]
            if len(finalists) > 1:
                score = {c: float("inf") for c in finalists}
                for _ in range(3):
                    for c in finalists:
                        self._set_tile(desc, c)
                        lib.po_conv(*args, st)
                        e0.record()
                        for _ in range(2 * iters):
                            lib.po_conv(*args, st)
                        e1.record()
                        e1.synchronize()
                        score[c] = min(score[c], e0.elapsed_time(e1))
                best = min((v, c) for c, v in score.items())
            self._set_tile(desc, best[1])
            cache[key] = list(best[1])
        for name, _, desc in self.fwd_ops + self.bwd_ops:     # the workspaces may have grown
            if name == "po_conv" and desc.ksplit > 1:
                desc.workspace = self.ws.data_ptr()
            if name == "po_conv" and desc.tile == self.WINOV_TILE:
                desc.winov = self.winov.data_ptr()
        self.bind_side_workspace()
        with torch.no_grad():
            for t in bufs.values():
                t.zero_()
        self.amax.zero_()
        torch.cuda.synchronize()

    def _cached_ok(self, desc, choice):
        """Whether a cached (tile, ksplit) can run this launch as built: a
        Winograd tile needs its transformed weights, which ADVPATCH_WINOGRAD=0
        / ADVPATCH_WINO4X4=0 leave unbuilt (po_conv would refuse the launch).
        A choice that cannot run is treated as missing from the cache."""
        t = choice if isinstance(choice, int) else choice[0]
        if t in (71, self.WINOV_TILE):
            return getattr(desc, "Wwino6", None) is not None
        if t in self.WINO_TILES or t == self.WPOOL_TILE:
            return getattr(desc, "Wwino", None) is not None
        return True

    @staticmethod
    def _tune_key(args, desc):
        key = (desc.B, desc.Hin, desc.Win, desc.Cin_p, desc.Hg, desc.Wg, desc.in_step, desc.ntaps, desc.N,
               desc.accumulate, args[6] is not None, args[7] is not None or bool(desc.mbits),
               args[8] is not None, desc.prec, bool(desc.ybits), bool(desc.gbox))
        if desc.pool_y:
            key = key + ("pool", 1)
        return key + ("mrows", desc.mrows) if desc.mrows else key

    _tile_map = None

    @classmethod
    def tile_map(cls):
        """ADVPATCH_TILE_MAP ("68:70,66:70"), parsed once per value: a diagnostic
        A/B remap of cached / tuned tiles (kept only where the target tile takes the launch)."""
        remap = os.environ.get("ADVPATCH_TILE_MAP", "")
        if cls._tile_map is None or cls._tile_map[0] != remap:
            m = dict(tuple(int(v) for v in kv.split(":")) for kv in remap.split(",") if kv.strip())
            cls._tile_map = (remap, m)
        return cls._tile_map[1]

    def _set_tile(self, desc, choice):
        t, ks = (choice, 1) if isinstance(choice, int) else choice
        desc.tile, desc.ksplit = t, ks
        self._apply_ws(desc)
        remap = self.tile_map()
        if remap and t in remap:
            # only where the target tile takes the launch: po_conv is called under
            # a stream capture that is discarded (its argument checks run, its
            # kernels never do); a refused remap keeps the chosen tile
            desc.tile = remap[t]
            self._apply_ws(desc)
            if not self._probe_conv(desc):
                desc.tile = t
                self._apply_ws(desc)

    def _probe_conv(self, desc):
        args = next((a for n, a, d in self.fwd_ops + self.bwd_ops if d is desc), None)
        if args is None or any(isinstance(a, str) for a in args):
            return False
        side = torch.cuda.Stream(device=self.device)
        graph = torch.cuda.CUDAGraph()
        ok = False
        try:
            with torch.cuda.graph(graph, stream=side, capture_error_mode="relaxed"):
                ok = self.lib.po_conv(*args, nat.stream()) == 0
        except RuntimeError:
            ok = False
        del graph
        return ok

    @staticmethod
    def winov_floats(desc):
        """Floats of tile 72's transformed-input workspace for launch desc
        (include/advpatch.h po_conv_desc.winov)."""
        tiles = desc.B * (-(-desc.Hg // 4)) * (-(-desc.Wg // 4))
        return -(-tiles // 32) * (desc.Cin_p // 16) * 18432

    def _ensure_winov(self, floats):
        if getattr(self, "winov", None) is None or self.winov.numel() < floats:
            self.winov = torch.empty(floats, device=self.device)
        return self.winov

    TILE_CTRS = 4096              # in-launch split-K arrival counters per stream (po_conv_desc.tile_ctr)

    def _tile_ctr(self, side=False):
        """The zeroed int32 arrival counters of po_conv's in-launch split-K
        reduction (ABI 28): one array for the main stream, one for the head-tail
        stream (launches that may overlap need separate counters).  Every launch
        leaves them zero."""
        name = "_ctr_side" if side else "_ctr_main"
        t = getattr(self, name, None)
        if t is None:
            t = torch.zeros(self.TILE_CTRS, dtype=torch.int32, device=self.device)
            setattr(self, name, t)
        return t

    @staticmethod
    def inlaunch_reduce():
        """ADVPATCH_INLAUNCH_REDUCE=1 (opt-in): split-K launches on the generic
        tiles reduce their slices inside the launch (the tile's last arriving
        slice) instead of in conv_reduce_k; bit-identical.  Off by default:
        measured slower on both bench plans (yolov3 B=16: 1000-1005 img/s
        against 1029 with the separate reduction, tiny B=256: 41.0-41.2k
        against 42.2-42.5k; profiles/r06/inlaunch_reduce_not_kept_ab.txt) --
        every slice's agent-scope release writes back its XCD's L2, and one
        workgroup reading all of a tile's slices is slower than a reduction
        spread over the whole chip."""
        return os.environ.get("ADVPATCH_INLAUNCH_REDUCE", "0") == "1"

    def _apply_ws(self, desc):
        ks = desc.ksplit
        if ks > 1:
            desc.workspace = self._ensure_ws(ks * desc.B * desc.Hg * desc.Wg * desc.N).data_ptr()
        else:
            desc.workspace = None
        if ks > 1 and self.inlaunch_reduce():
            desc.tile_ctr, desc.tile_ctr_n = self._tile_ctr().data_ptr(), self.TILE_CTRS
        else:
            desc.tile_ctr, desc.tile_ctr_n = None, 0
        if desc.tile == self.WINOV_TILE:
            n = self.winov_floats(desc)
            desc.winov, desc.winov_floats = self._ensure_winov(n).data_ptr(), n
        else:
            desc.winov, desc.winov_floats = None, 0

    # ---------------- execution ----------------
    def run_forward(self, x, base=None, roi=None):
        """x: [B,3,H,W] contiguous CUDA float32 (NCHW).  Returns NHWC head buffers.
        ``base`` (with ``roi`` [B,4] int32): x is the sparse patch composite --
        valid only inside each image's quad-widened footprint box of roi
        (po_warp_box_fwd_keyed, fill = 0) -- and the input equals ``base``
        elsewhere; the first layer reads the two (po_conv_first_*_cmp)."""
        self.gen += 1
        st = nat.stream()
        lib = self.lib
        if self.prec == 1:
            self.amax.zero_()                 # the fp16x3 max|x| slots (exact fp32 plans have none)
        xp = nat.c_void_p(x.data_ptr())
        if base is not None:
            if not self.sparse_input or roi is None:
                raise ValueError("NetPlan.run_forward: this plan's first layer cannot read a sparse composite")
            cmp = (nat.c_void_p(base.data_ptr()), xp, nat.c_void_p(roi.data_ptr()))
        self.join_cone_stream()               # a previous forward's cone write is ordered before this one
        self._cones_for = None
        self.last_first_op = None
        if roi is not None and self.cone_boxes is not None and os.environ.get("ADVPATCH_EARLY_CONES", "1") != "0":
            # the gradient cones depend on the footprint boxes only: evaluate them
            # (a serial walk of the block graph, one small workgroup per image)
            # beside the forward instead of at the head of the backward
            if getattr(self, "_cone_stream", None) is None:
                self._cone_stream = torch.cuda.Stream(device=self.device)
            self._cone_stream.wait_stream(torch.cuda.current_stream())
            roi.record_stream(self._cone_stream)          # read there: not reused before that read ends
            with torch.cuda.stream(self._cone_stream):
                self.set_cones(roi)
            self._cones_for = roi
        if not self.first_direct:
            nat.call("po_nchw_to_nhwc", xp, self.B, self.H, self.W, 3, 16, nat.c_void_p(self.in_nhwc.data_ptr()), st)
        side = self.side if self.tails else None
        for k, (name, args, desc) in enumerate(self.fwd_ops):
            if side is not None and k in self._side_f:
                continue                                  # a head tail: launched on the side stream
            if name in ("po_conv_first_fwd", "po_conv_first_pool_fwd", "po_conv_first_pool_wino_fwd"):
                if base is not None:
                    name, args = name + "_cmp", cmp + args[1:]
                else:
                    args = (xp,) + args[1:]
                self.last_first_op = name
            self._launch(lib, name, args, desc, st)
            if side is not None and k in self._trig_f:
                # block b is done: its tail runs beside the rest of the network
                side.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(side):
                    sst = nat.stream()
                    for t in self._trig_f[k]:
                        for kk in t["fwd"]:
                            n_, a_, d_ = self.fwd_ops[kk]
                            self._launch(lib, n_, a_, d_, sst)
        if side is not None:
            torch.cuda.current_stream().wait_stream(side)
        return [self.act[h] for h in self.heads]

    def join_cone_stream(self):
        """Order the current stream after any cone evaluation still pending on
        the side stream (run_forward with roi evaluates the cones there; a
        forward whose backward never runs would otherwise leave that write
        unordered with the next set_cones or a host read of cone_boxes)."""
        cs = getattr(self, "_cone_stream", None)
        if cs is not None:
            torch.cuda.current_stream().wait_stream(cs)

    def _launch(self, lib, name, args, desc, st):
        timer = self.conv_timer
        if timer is not None and name == "po_conv":
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            rc = lib.po_conv(*args, st)
            e1.record()
            timer.append((e0, e1, desc, self._cone_snap if desc.gbox else None))
        elif timer is not None and name.startswith("po_conv_first_") and "dgrad" not in name:
            # the first layer's forward (bench.py's HBM roofline of the frame read)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            rc = getattr(lib, name)(*args, st)
            e1.record()
            self.first_timer.append((e0, e1, name))
        else:
            rc = getattr(lib, name)(*args, st)
        if rc:
            raise RuntimeError("%s failed: %s" % (name, nat.last_error()))

    def run_backward(self, d_heads, d_x, roi=None):
        """d_heads: NHWC gradient tensors of the head buffers (list, in head order);
        d_x: [B,3,H,W] output buffer for the input gradient; roi: optional [B,4]
        int32 boxes — d_x is then only computed inside them."""
        st = nat.stream()
        lib = self.lib
        for hi, h in enumerate(self.heads):
            r = self.root[h]
            g = d_heads[hi].contiguous()
            M = self.B * self.dims[r][0] * self.dims[r][1]
            mask = self.act[r] if (self.ncons[r] == 0 and self._leaky(r)) else None
            nat.call("po_slice_accum", nat.c_void_p(g.data_ptr()), self.cp[r], 0,
                     nat.c_void_p(self.grad[r].data_ptr()), self.cp[r], 0, M, self.cp[r], 0,
                     nat.c_void_p(mask.data_ptr()) if mask is not None else None, self.cp[r],
                     self.slot(self.grad[r]), st)
        dxp = nat.c_void_p(d_x.data_ptr())
        roip = nat.c_void_p(roi.data_ptr()) if roi is not None else None
        if roi is not None and getattr(self, "_cones_for", None) is roi:
            torch.cuda.current_stream().wait_stream(self._cone_stream)     # evaluated beside the forward
        else:
            self.join_cone_stream()           # an unconsumed early evaluation must land before this one
            self.set_cones(roi)
        self._cones_for = None
        self.set_support_boxes()
        if self.conv_timer is not None and self.cone_boxes is not None:
            self._cone_snap = self.cone_boxes.clone()        # this step's cones, for launch_macs
        side = self.side if self.tails else None

        def run(k, sst):
            name, args, desc = self.bwd_ops[k]
            if name == "zero":
                args[0].zero_()
                return
            if args and args[-1] == "dimg":
                if name == "po_conv_first_dgrad":
                    args = args[:-2] + (roip, dxp)
                else:
                    args = args[:-1] + (dxp,)
            self._launch(lib, name, args, desc, sst)

        if side is not None:
            # the head gradients, cones and support boxes are in place: the tails'
            # inner dgrads start beside the main chain
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                sst = nat.stream()
                for t in self.tails:
                    for k in t["bwd_early"]:
                        run(k, sst)
        for k in range(len(self.bwd_ops)):
            if side is not None and k in self._side_b:
                if k in self._final_b:
                    # the group accumulating into grad[b], in its place of the order
                    side.wait_stream(torch.cuda.current_stream())
                    with torch.cuda.stream(side):
                        sst = nat.stream()
                        for kk in self._final_b[k]["bwd_final"]:
                            run(kk, sst)
                    torch.cuda.current_stream().wait_stream(side)
                continue
            run(k, st)



# Winograd F(2x2,3x3): U = G g G^T with G = [[1,0,0],[.5,.5,.5],[.5,-.5,.5],[0,0,1]]
_WINO_G = ((1.0, 0.0, 0.0), (0.5, 0.5, 0.5), (0.5, -0.5, 0.5), (0.0, 0.0, 1.0))


def first_wino_u(w):
    """First-layer weights [Cout,3,3,3] (float64) -> the F(2x2,3x3) kernel
    transforms U[co][c] = G g G^T, [Cout,3,16] row-major over the 4x4 (the
    operand of po_conv_first_pool_wino_fwd), computed in float64."""
    G = torch.tensor([[1.0, 0.0, 0.0], [0.5, 0.5, 0.5], [0.5, -0.5, 0.5], [0.0, 0.0, 1.0]], dtype=torch.float64)
    w = w.double()
    return torch.einsum("ik,ockl,jl->ocij", G, w, G).reshape(w.shape[0], 3, 16)


def wino_transform(w, offs):
    """po_conv_desc.Wwino of launch weights w [N][9][Cin_p] (fp32) whose tap t
    reads source offset offs[t] = (dh, dw) in {-1,0,1}^2: U = G g G^T in
    float64, rounded once to fp32, in MFMA fragment order
    [N/32][Cin_p/16][16][2][64 lanes][4]: element (lane l, s) of block
    (nb, kc, xi) = U[xi][16 kc + 8 (l >> 5) + s][32 nb + (l & 31)] sits at
    [nb][kc][xi][s >> 2][l][s & 3] (a wave reads each half as 1 KB)."""
    N, T, C = w.shape
    assert T == 9 and N % 32 == 0 and C % 16 == 0
    g = torch.zeros(N, C, 3, 3, dtype=torch.float64, device=w.device)
    for t, (dh, dw) in enumerate(offs):
        g[:, :, dh + 1, dw + 1] = w[:, t, :].double()
    G = torch.tensor(_WINO_G, dtype=torch.float64, device=w.device)
    U = torch.einsum("xa,ncab,yb->xycn", G, g, G).reshape(16, C, N).float()        # [xi][c][n]
    return U.view(16, C // 16, 2, 2, 4, N // 32, 32).permute(5, 1, 0, 3, 2, 6, 4).contiguous()


# Winograd F(4x4,3x3) (Lavin; points 0, +-1, +-2, inf): U = G g G^T with this G,
# the input transform B^T and inverse A^T as csrc/conv_wino6.hip's bt6 / at6
_WINO6_G = ((1 / 4, 0.0, 0.0), (-1 / 6, -1 / 6, -1 / 6), (-1 / 6, 1 / 6, -1 / 6), (1 / 24, 1 / 12, 1 / 6),
            (1 / 24, -1 / 12, 1 / 6), (0.0, 0.0, 1.0))
WINO6_BT = ((4, 0, -5, 0, 1, 0), (0, -4, -4, 1, 1, 0), (0, 4, -4, -1, 1, 0), (0, -2, -1, 2, 1, 0),
            (0, 2, -1, -2, 1, 0), (0, 4, 0, -5, 0, 1))
WINO6_AT = ((1, 1, 1, 1, 1, 0), (0, 1, -1, 2, -2, 0), (0, 1, 1, 4, 4, 0), (0, 1, -1, 8, -8, 1))


def wino6_transform(w, offs):
    """po_conv_desc.Wwino6 of launch weights w [N][9][Cin_p] (fp32) whose tap
    t reads source offset offs[t]: U = G g G^T (F(4x4,3x3), component xi =
    6 i + j) in float64, rounded once to fp32, in MFMA fragment order
    [N/32][Cin_p/16][36][2][64 lanes][4] (wino_transform's order with 36
    components)."""
    N, T, C = w.shape
    assert T == 9 and N % 32 == 0 and C % 16 == 0
    g = torch.zeros(N, C, 3, 3, dtype=torch.float64, device=w.device)
    for t, (dh, dw) in enumerate(offs):
        g[:, :, dh + 1, dw + 1] = w[:, t, :].double()
    G = torch.tensor(_WINO6_G, dtype=torch.float64, device=w.device)
    U = torch.einsum("xa,ncab,yb->xycn", G, g, G).reshape(36, C, N).float()        # [xi][c][n]
    return U.view(36, C // 16, 2, 2, 4, N // 32, 32).permute(5, 1, 0, 3, 2, 6, 4).contiguous()


class _DarknetFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, plan, nchw, roi=None, base=None):
        heads = plan.run_forward(x.contiguous(), base, roi)
        ctx.plan, ctx.gen, ctx.nchw, ctx.roi = plan, plan.gen, nchw, roi
        if not nchw:
            return tuple(h.clone() if plan.net.clone_heads else h.detach() for h in heads)
        outs = []
        for hb, h in zip(heads, plan.heads):
            hh, ww, c = plan.shp[h]
            o = torch.empty(plan.B, c, hh, ww, device=x.device)
            nat.call("po_nhwc_to_nchw", nat.c_void_p(hb.data_ptr()), plan.B, hh, ww, c, plan.cp[h],
                     nat.c_void_p(o.data_ptr()), nat.stream())
            outs.append(o)
        return tuple(outs)

    @staticmethod
    def backward(ctx, *grads):
        plan = ctx.plan
        if plan.gen != ctx.gen:
            raise RuntimeError("Darknet activations were overwritten by a later forward of the same "
                               "plan before backward (one forward per backward per batch shape)")
        d_heads = []
        for g, h in zip(grads, plan.heads):
            hh, ww, c = plan.shp[h]
            if g is None:
                g = torch.zeros(plan.B, hh, ww, plan.cp[h], device=plan.device)
            elif ctx.nchw:
                gn = torch.empty(plan.B, hh, ww, plan.cp[h], device=plan.device)
                nat.call("po_nchw_to_nhwc", nat.c_void_p(g.contiguous().data_ptr()), plan.B, hh, ww, c, plan.cp[h],
                         nat.c_void_p(gn.data_ptr()), nat.stream())
                g = gn
            d_heads.append(g.contiguous())
        d_x = torch.empty(plan.B, 3, plan.H, plan.W, device=plan.device)
        plan.run_backward(d_heads, d_x, ctx.roi)
        return d_x, None, None, None, None


class Darknet(nn.Module):
    """YOLOv3 object detection model (darknet_v3.py:179-309), HIP execution."""

    def __init__(self, config_path):
        super().__init__()
        self.blocks = parse_model_config(config_path)
        self.width = int(self.blocks[0]["width"])
        self.height = int(self.blocks[0]["height"])
        self.hyperparams, self.module_list = create_modules(self.blocks)
        self.yolo_layers = [layer[0] for layer in self.module_list if isinstance(layer[0], YOLOLayer)]
        self.seen = 0
        self.header_info = np.array([0, 0, 0, self.seen, 0], dtype=np.int32)
        self.clone_heads = False
        # receptive-field windows on the training path (ADVPATCH_WINDOWS=0: full maps)
        self.window_heads = os.environ.get("ADVPATCH_WINDOWS", "1") != "0"
        # conv operand precision: "fp32" (exact fp32 MFMA, the reference's
        # arithmetic; default) or "fp16x3" (operands split into two fp16
        # pieces, ~22 significant bits, three fp16 MFMA products; opt-in)
        self.conv_prec = os.environ.get("ADVPATCH_CONV_PREC", "fp32")
        if self.conv_prec not in ("fp16x3", "fp32"):
            raise ValueError("ADVPATCH_CONV_PREC must be fp16x3 or fp32, got %r" % self.conv_prec)
        self._conv_meta = {}
        cin = [int(self.hyperparams["channels"])]
        for i, (d, mod) in enumerate(zip(self.blocks, self.module_list)):
            if d["type"] == "convolutional":
                conv = mod[0]
                self._conv_meta[i] = {"cin": conv.in_channels, "cout": conv.out_channels,
                                      "k": conv.kernel_size[0], "stride": conv.stride[0],
                                      "pad": conv.padding[0], "bn": int(d["batch_normalize"]),
                                      "act": d["activation"]}
                if d["activation"] not in ("leaky", "linear"):
                    self._conv_meta[i]["unsupported"] = d["activation"]
        self._dev = None
        self._dev_device = None
        self._dgrad_cache = {}
        self._frag = {}
        self._plans = {}
        self._tile_cache = {}

    # ---------------- weights ----------------
    def load_darknet_weights(self, weights_path):
        """Parses and loads the weights stored in 'weights_path' (darknet_v3.py:223-281)."""
        with open(weights_path, "rb") as f:
            header = np.fromfile(f, dtype=np.int32, count=5)
            self.header_info = header
            self.seen = header[3]
            weights = np.fromfile(f, dtype=np.float32)
        cutoff = 75 if "darknet53.conv.74" in weights_path else None
        ptr = 0
        for i, (module_def, module) in enumerate(zip(self.blocks, self.module_list)):
            if i == cutoff:
                break
            if module_def["type"] != "convolutional":
                continue
            conv_layer = module[0]
            with torch.no_grad():
                if module_def["batch_normalize"]:
                    bn = module[1]
                    nb = bn.bias.numel()
                    for t in (bn.bias, bn.weight, bn.running_mean, bn.running_var):
                        t.copy_(torch.from_numpy(weights[ptr:ptr + nb]).view_as(t))
                        ptr += nb
                else:
                    nb = conv_layer.bias.numel()
                    conv_layer.bias.copy_(torch.from_numpy(weights[ptr:ptr + nb]).view_as(conv_layer.bias))
                    ptr += nb
                nw = conv_layer.weight.numel()
                conv_layer.weight.copy_(torch.from_numpy(weights[ptr:ptr + nw]).view_as(conv_layer.weight))
                ptr += nw
        self.invalidate()
        return ptr

    def save_darknet_weights(self, path, cutoff=-1):
        """Write the darknet .weights layout (the reference's version refers to an
        undefined attribute, darknet_v3.py:293; this one works)."""
        with open(path, "wb") as fp:
            self.header_info[3] = self.seen
            np.asarray(self.header_info, dtype=np.int32).tofile(fp)
            pairs = list(zip(self.blocks, self.module_list))
            if cutoff != -1:
                pairs = pairs[:cutoff]
            for module_def, module in pairs:
                if module_def["type"] != "convolutional":
                    continue
                conv_layer = module[0]
                if module_def["batch_normalize"]:
                    bn = module[1]
                    for t in (bn.bias, bn.weight, bn.running_mean, bn.running_var):
                        t.detach().cpu().numpy().astype(np.float32).tofile(fp)
                else:
                    conv_layer.bias.detach().cpu().numpy().astype(np.float32).tofile(fp)
                conv_layer.weight.detach().cpu().numpy().astype(np.float32).tofile(fp)

    def invalidate(self):
        """Drop device-side folded weights and plans (after a weight change)."""
        self._dev = None
        self._dgrad_cache = {}
        self._frag = {}
        self._plans = {}

    def _folded(self, i):
        """(W [Cout,Cin,k,k], bias [Cout]) with eval BN folded (float64 fold)."""
        mod = self.module_list[i]
        conv = mod[0]
        W = conv.weight.detach().double().cpu()
        if self._conv_meta[i]["bn"]:
            bn = mod[1]
            scale = bn.weight.detach().double().cpu() / torch.sqrt(bn.running_var.detach().double().cpu() + bn.eps)
            bias = bn.bias.detach().double().cpu() - bn.running_mean.detach().double().cpu() * scale
            W = W * scale.view(-1, 1, 1, 1)
        else:
            bias = conv.bias.detach().double().cpu()
        return W, bias

    def _prepare(self, device):
        if self._dev is not None and self._dev_device == device:
            return
        for i, m in self._conv_meta.items():
            if "unsupported" in m:
                raise NotImplementedError("activation %r (block %d) is not on the HIP path" % (m["unsupported"], i))
        self._dev, self._dgrad_cache, self._plans = {}, {}, {}
        self._frag = {}
        self._folded_cache = {}
        for i, m in self._conv_meta.items():
            W, bias = self._folded(i)
            self._folded_cache[i] = W
            cout, cin, k = m["cout"], m["cin"], m["k"]
            cop, cip = _cp(cout), _cp(cin)
            Wn = torch.zeros(cop, k * k, cip, dtype=torch.float64)
            Wn[:cout, :, :cin] = W.permute(0, 2, 3, 1).reshape(cout, k * k, cin)
            b = torch.zeros(cop, dtype=torch.float64)
            b[:cout] = bias
            ent = {"w": Wn.float().contiguous().to(device), "bias": b.float().to(device)}
            if i == 0 and cin == 3 and k == 3:
                ent["w27"] = W.reshape(cout, 27).float().contiguous().to(device)
                ent["u16"] = first_wino_u(W).float().contiguous().to(device)
            self._dev[i] = ent
        self._dev_device = device

    @staticmethod
    def _split16(w):
        """fp32 weights -> (fp16 [2, *w.shape] = hi, lo pieces of w * 2^shift,
        shift), with max|w * 2^shift| in [2^13, 2^14) (po_conv prec 1)."""
        m = float(w.abs().max())
        shift = 14 - math.frexp(m)[1] if m > 0 else 0
        ws = w * (2.0 ** shift)                       # exact: power of two, no overflow
        hi = ws.half()
        lo = (ws - hi.float()).half()
        return torch.stack([hi, lo]).contiguous(), shift

    def _frag16(self, w16):
        """Device address of w16 ([2][N][taps][Cin_p] fp16) in MFMA B-fragment
        order [2][N/32][taps][Cin_p/16][64][8] (po_conv_desc.Wfrag), built once
        per weight tensor; None when N is not a multiple of 32."""
        if w16.dim() != 4:
            return None
        two, N, T, C = w16.shape
        if N % 32 or C % 16:
            return None
        key = w16.data_ptr()
        if key not in self._frag:
            f = w16.view(2, N // 32, 32, T, C // 16, 2, 8).permute(0, 1, 3, 4, 5, 2, 6).contiguous()
            self._frag[key] = (w16, f)          # keep w16 alive with its key
        return nat.c_void_p(self._frag[key][1].data_ptr())

    def _wino(self, w, offs, f4=False):
        """Device address of the Winograd weights of launch weights w with tap
        offsets offs (wino_transform; f4: F(4x4,3x3), wino6_transform), built
        once per (weights, tap order, form)."""
        key = (w.data_ptr(), tuple(offs), bool(f4))
        if key not in self._frag:
            self._frag[key] = (w, (wino6_transform if f4 else wino_transform)(w, offs))   # keep w alive with its key
        return nat.c_void_p(self._frag[key][1].data_ptr())

    def _dev16(self, i):
        """Split-fp16 forward weights of conv i (built on first use)."""
        ent = self._dev[i]
        if "w16" not in ent:
            ent["w16"], ent["w16_shift"] = self._split16(ent["w"])
        return ent["w16"], ent["w16_shift"]

    def _dgrad_weight16(self, j, taps, cin_p, device):
        key = (j, tuple(taps), cin_p, "f16")
        if key not in self._dgrad_cache:
            self._dgrad_cache[key] = self._split16(self._dgrad_weight(j, taps, cin_p, device))
        return self._dgrad_cache[key]

    def _dgrad_weight(self, j, taps, cin_p, device):
        """[Cin_p][len(taps)][Cout_p] weights of one dgrad launch of conv j."""
        key = (j, tuple(taps), cin_p)
        if key not in self._dgrad_cache:
            W = self._folded_cache[j]
            m = self._conv_meta[j]
            cout, cin = m["cout"], m["cin"]
            Wd = torch.zeros(cin_p, len(taps), _cp(cout), dtype=torch.float64)
            for ti, (kh, kw) in enumerate(taps):
                Wd[:cin, ti, :cout] = W[:, :, kh, kw].t()
            self._dgrad_cache[key] = Wd.float().contiguous().to(device)
        return self._dgrad_cache[key]

    def plan(self, B, H, W, device, windowed=False):
        """The execution plan for a batch shape (built, and its conv tiles
        autotuned on the device, on first use; ADVPATCH_TUNE=0 keeps the
        built-in tile heuristic, ADVPATCH_TUNE=cache takes the tiles of
        ADVPATCH_TUNE_CACHE and times nothing).  ``windowed``: blocks past the last
        full-map dependency run on receptive-field windows around the loss
        cells (NetPlan._plan_windows); only the training path uses it."""
        self._prepare(device)
        key = (B, H, W, str(device), bool(windowed), self.conv_prec)
        if key not in self._plans:
            p = NetPlan(self, B, H, W, device, windowed=windowed)
            if torch.device(device).type == "cuda" and os.environ.get("ADVPATCH_TUNE", "1") != "0":
                path = os.environ.get("ADVPATCH_TUNE_CACHE")
                if path and os.path.exists(path) and not self._tile_cache:
                    import json
                    with open(path) as f:
                        self._tile_cache.update({tuple(json.loads(k)): v for k, v in json.load(f).items()})
                n0 = len(self._tile_cache)
                p.tune(self._tile_cache, time_missing=os.environ.get("ADVPATCH_TUNE", "1") != "cache")
                if path and len(self._tile_cache) != n0:
                    import json
                    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
                    tmp = "%s.%d.tmp" % (path, os.getpid())
                    with open(tmp, "w") as f:
                        json.dump({json.dumps(list(k)): v for k, v in self._tile_cache.items()}, f)
                    os.replace(tmp, path)
            self._plans[key] = p
        return self._plans[key]

    # ---------------- forward ----------------
    def forward(self, x):
        """x [B,3,H,W] -> list of raw head tensors [B, 3*(5+C), h, w] (NCHW)."""
        nat.ensure_device(x)
        p = self.plan(x.size(0), x.size(2), x.size(3), x.device)
        return list(_DarknetFn.apply(x, p, True))

    def forward_nhwc(self, x, input_roi=None, center=None, base=None):
        """Training-path forward: returns (head buffers, plan).  Head buffers
        are NHWC [B, h, w, Cp] (Cp = padded channel stride, channel =
        anchor*(5+C) + field).
        ``input_roi`` [B,4] int32: the input gradient is only needed (and only
        computed) inside these per-image boxes (the patch footprint).
        ``center`` [B,2] (patch centres, px): the loss reads the heads only
        at the cells of these centres (train_patch.py:449-483); the plan then
        computes the blocks after the last full-map dependency on windows
        around them, and the heads come back as windows
        (``plan.head_views()``).
        ``base``: x is the sparse composite of PatchTransformer.
        forward_composite(sparse=True) -- valid inside the quad-widened boxes
        of input_roi only, ``base`` (the frames) elsewhere (NetPlan.run_forward)."""
        nat.ensure_device(x)
        windowed = center is not None and self.window_heads
        p = self.plan(x.size(0), x.size(2), x.size(3), x.device, windowed=windowed)
        if p.windowed:
            p.set_windows(center)
        return list(_DarknetFn.apply(x, p, False, input_roi, base)), p

    def sparse_input_ok(self, B, H, W, device, center=None):
        """Whether forward_nhwc(x, roi, center, base=frames) can run (the plan's
        first layer reads a sparse composite: po_conv_first_*_cmp)."""
        windowed = center is not None and self.window_heads
        return self.plan(B, H, W, device, windowed=windowed).sparse_input
