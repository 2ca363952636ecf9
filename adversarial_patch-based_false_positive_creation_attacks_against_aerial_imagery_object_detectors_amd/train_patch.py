"""Adversarial-patch training loop — drop-in for reference ``train_patch.py``.

``PatchTrainer(mode)`` / ``.train()`` keep the reference's entry points
(train_patch.py:48-606) and its loss:

    loss = 0.01*NPS + max(2.5*TV, 0.1) + 4*(1 - mean_b max_9 obj) + COLOUR + CE(cls -> 14)

with every op of one iteration on the MI355X HIP path:

    median pool -> placement params -> fused augment/warp/composite   (load_data)
    -> Darknet forward (implicit-GEMM fp32 MFMA)                      (darknet_v3)
    -> cell loss (objectness / CE at the patch cell)                  (po_cell_loss)
    -> NPS/TV/colour                                                  (po_regularisers)
    -> backward: cell-loss grad -> Darknet dgrad -> warp bwd -> median bwd
    -> [multi-GPU: one all-reduce of the patch gradient]
    -> Adam(amsgrad) + clamp_(0,1) in PyTorch-ROCm.

No host synchronisation happens inside a step (the reference does 2*3*B
``int()`` syncs in ``obj_cls_conf_find`` plus 5 ``.cpu()`` per iteration);
error flags (cell out of range, window misplaced, non-finite gradient) are
OR-ed into a device word and checked once per epoch (``check_flags``).
Multi-GPU: one process per GPU (torchrun); each rank runs a contiguous shard
of every global batch (``GlobalBatchSampler``; draws keyed by the global image
index), weights its loss terms by its share (``shard_weights``) and ONE
all-reduce(SUM) of [patch grad | loss scalars] yields exactly the global-batch
gradient, whatever the number of ranks — replacing the reference's
``nn.DataParallel`` (train_patch.py:63-71), which scatters one global batch.
"""
import fnmatch
import os
import sys
import time

if __package__ in (None, ""):
    # executed as a script: bootstrap the package (its directory name is not an identifier)
    import importlib
    _here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, os.path.dirname(_here))
    _pkg = importlib.import_module(os.path.basename(_here))
    __package__ = _pkg.__name__

import numpy as np
import torch
import torch.nn.functional as F
from torch import optim

from . import _native as nat
from . import patch_config
from . import synthetic
from . import weights as synth_weights
from .darknet_v3 import Darknet
from .load_data import (DevicePrefetcher, DotaCollate, DotaDataset, FrameCache, HasSusRGB, NPSCalculator, PatchApplier,
                        PatchTransformer, TotalVariation, loader_context, patch_front, read_image as _read_image,
                        regularisers)

TV_FACTOR = 2.5      # train_patch.py:25
NPS_FACTOR = 0.01    # train_patch.py:26
TARGET_ID = 14       # train_patch.py:28 (helicopter)
OBJECTIVES = {"ce": 0, "targeted": 1, "untargeted": 2}
# classes per anchor that po_cell_loss reads: 5 + 15 channels per anchor, the
# layout the reference's loss head hard-codes (train_patch.py:459; NCLS in
# csrc/loss_ops.hip).  PatchTrainer refuses a network with another count.
CELL_CLASSES = 15


def _head_args(hw, views):
    """ctypes arrays (hw, win, org) of po_cell_loss; views = None (full maps)
    or (window sides, origin tensors [B,2] int32 or None per head)."""
    n = len(hw)
    hwa = (nat.c_int * n)(*hw)
    if views is None:
        return hwa, None, None
    win, orgs = views
    return hwa, (nat.c_int * n)(*win), nat.ptr_array(orgs)


class _CellLoss(torch.autograd.Function):
    """(no_obj, no_cls) at the patch cells of the NHWC head buffers (po_cell_loss)."""

    @staticmethod
    def forward(ctx, center, S, target, objective, hw, Cp, views, flags, *heads):
        B = center.size(0)
        dev = center.device
        A = 3 * len(heads)
        out2 = torch.empty(2, device=dev)
        obj = torch.empty(B, A, device=dev)
        cls = torch.empty(B, A, CELL_CLASSES, device=dev)
        cells = torch.empty(len(heads), B, dtype=torch.int32, device=dev)
        if flags is None:
            flags = torch.zeros(1, dtype=torch.int32, device=dev)
        hwa, wina, orga = _head_args(hw, views)
        scratch = torch.empty(2 * B, device=dev)
        nat.call("po_cell_loss", nat.ptr_array(heads), hwa, wina, orga, len(heads), Cp, B, S,
                 nat.ptr(center.contiguous()), target, objective, None, None, nat.ptr(out2), nat.ptr(obj),
                 nat.ptr(cls), nat.ptr(cells, torch.int32), nat.ptr(flags, torch.int32), nat.ptr(scratch),
                 nat.stream())
        ctx.save_for_backward(center, *heads)
        ctx.meta = (S, target, objective, tuple(hw), Cp, views)
        ctx.mark_non_differentiable(obj, cls, cells, flags)
        ctx.set_materialize_grads(False)          # no zero tensors for the non-differentiable outputs
        return out2, obj, cls, cells, flags

    @staticmethod
    def backward(ctx, g2, *unused):
        center, *heads = ctx.saved_tensors
        S, target, objective, hw, Cp, views = ctx.meta
        arena = torch.zeros(sum(h.numel() for h in heads), device=center.device)     # one fill for all heads
        d_heads, o = [], 0
        for h in heads:
            d_heads.append(arena[o:o + h.numel()].view_as(h))
            o += h.numel()
        out2 = torch.empty(2, device=center.device)
        hwa, wina, orga = _head_args(hw, views)
        scratch = torch.empty(2 * center.size(0), device=center.device)
        nat.call("po_cell_loss", nat.ptr_array(heads), hwa, wina, orga, len(heads), Cp, center.size(0), S,
                 nat.ptr(center.contiguous()), target, objective, nat.ptr(g2.contiguous().float()),
                 nat.ptr_array(d_heads), nat.ptr(out2), None, None, None, None, nat.ptr(scratch), nat.stream())
        return (None, None, None, None, None, None, None, None) + tuple(d_heads)


def cell_loss(heads, plan, img_size, patch_center, target=TARGET_ID, objective="ce", flags=None):
    """-> (out2 [2] = {no_obj_loss, no_cls_loss}, obj [B,9], cls [B,9,15], cells, flags).
    ``heads`` are the plan's head buffers (full maps, or receptive-field
    windows when the plan was run with the patch centres); ``flags``: an
    int32 [1] device accumulator the kernel ORs its error bits into (a fresh
    zero word when None)."""
    hw = [plan.shp[h][0] for h in plan.heads]
    Cp = plan.cp[plan.heads[0]]
    for h in plan.heads:
        assert plan.cp[h] == Cp and plan.shp[h][0] == plan.shp[h][1]
    return _CellLoss.apply(patch_center, int(img_size), int(target), OBJECTIVES[objective], hw, Cp,
                           plan.head_views(), flags, *heads)


LOSS_KEYS = ("loss", "nps_loss", "tv_loss", "no_obj_loss", "no_cls_loss", "colorful_loss")

# error bits of the trainer's device flag word (check_flags)
FLAG_BITS = {1: "patch-centre cell outside its head map (clamped)",
             2: "loss cell outside its receptive-field window (planning error)",
             4: "receptive-field window too small for the needed box (planning error)",
             8: "non-finite patch gradient (NaN/Inf; the reference ran under detect_anomaly)"}
FLAG_NONFINITE = 8


def shard_weights(n_local, n_global, world, objective="ce"):
    """(w_img, w_cls, w_patch): multipliers that make the per-rank losses add
    up to the global-batch loss under an all-reduce SUM.

    * image terms that are batch MEANS (objectness, CE) count with this
      rank's share of the global batch, n_local / n_global;
    * the targeted class term is a batch SUM (noCLS_loss_targeted,
      train_patch.py:575) and counts with weight 1;
    * the patch terms (NPS, TV, colour) are identical on every rank and
      count 1/world each.
    Unequal (ragged last) shards come out right too."""
    w_img = float(n_local) / float(n_global)
    w_cls = 1.0 if objective == "targeted" else w_img
    return w_img, w_cls, 1.0 / float(world)


def combine_terms(no_obj_loss, no_cls_loss, nps, tv, colorful, objective="ce", weights=None, tv_floor=None):
    """The reference's loss (train_patch.py:230-314):

        loss = 0.01*NPS + max(2.5*TV, 0.1) + 4*(1 - mean max obj) + COLOUR [+ CLS]

    ``weights`` = shard_weights(...) for a data-parallel rank (None: one
    process, no scaling).  Returns (loss, terms dict) with every term already
    weighted, so the SUM over ranks of each is its global value."""
    nps_loss = nps * NPS_FACTOR
    tv_loss = tv * TV_FACTOR
    if tv_floor is None:
        tv_floor = torch.tensor(0.1, device=tv.device, dtype=tv.dtype)
    tv_term = torch.max(tv_loss, tv_floor)
    if weights is not None:
        w_img, w_cls, w_patch = weights
        no_obj_loss, no_cls_loss = no_obj_loss * w_img, no_cls_loss * w_cls
        nps_loss, tv_loss, tv_term, colorful = nps_loss * w_patch, tv_loss * w_patch, tv_term * w_patch, colorful * w_patch
    loss = nps_loss + tv_term + no_obj_loss + colorful
    if objective != "untargeted":
        loss = loss + no_cls_loss
    return loss, {"loss": loss, "nps_loss": nps_loss, "tv_loss": tv_loss, "no_obj_loss": no_obj_loss,
                  "no_cls_loss": no_cls_loss, "colorful_loss": colorful}


class _LossCombine(torch.autograd.Function):
    """combine_terms on the device in one launch each way (po_loss_combine /
    po_loss_combine_bwd): the same fp32 values as the PyTorch expression and
    its autograd, without its ~25 elementwise, select and fill kernels.
    out2 = {no_obj, no_cls} (po_cell_loss), reg = {nps, tv, colour}
    (po_regularisers).  Returns (loss, terms [6]) with terms = LOSS_KEYS'
    values; only the loss is differentiable."""

    @staticmethod
    def forward(ctx, out2, reg, weights, with_cls):
        dev = out2.device
        w = weights if weights is not None else (1.0, 1.0, 1.0)
        loss = torch.empty((), device=dev)
        terms = torch.empty(6, device=dev)
        nat.call("po_loss_combine", nat.ptr(out2), nat.ptr(reg), float(w[0]), float(w[1]), float(w[2]),
                 int(weights is not None), int(with_cls), nat.ptr(terms), nat.ptr(loss), nat.stream())
        ctx.save_for_backward(reg)
        ctx.meta = (w, weights is not None, with_cls)
        ctx.mark_non_differentiable(terms)
        ctx.set_materialize_grads(False)
        return loss, terms

    @staticmethod
    def backward(ctx, g_loss, _):
        reg, = ctx.saved_tensors
        w, weighted, with_cls = ctx.meta
        d_out2 = torch.empty(2, device=reg.device)
        d_reg = torch.empty(3, device=reg.device)
        nat.call("po_loss_combine_bwd", nat.ptr(reg), nat.ptr(g_loss.contiguous().float()), float(w[0]), float(w[1]),
                 float(w[2]), int(weighted), int(with_cls), nat.ptr(d_out2), nat.ptr(d_reg), nat.stream())
        return d_out2, d_reg, None, None


def combine_terms_device(out2, reg, objective="ce", weights=None):
    """combine_terms(out2[0], out2[1], reg[0], reg[1], reg[2], objective,
    weights) as one device launch (and one for its gradient)."""
    loss, t = _LossCombine.apply(out2, reg, weights, objective != "untargeted")
    return loss, {"loss": loss, "nps_loss": t[1], "tv_loss": t[2], "no_obj_loss": t[3], "no_cls_loss": t[4],
                  "colorful_loss": t[5]}


def allreduce_patch_grad(grad, terms, group=None):
    """Data-parallel reduction of one step: every rank holds
    the gradient of its WEIGHTED loss (combine_terms with shard_weights), so
    ONE all-reduce(SUM) of the fused buffer [patch grad | 6 loss scalars]
    gives the global-batch gradient and loss terms on every rank (RCCL over
    xGMI with backend "nccl"; gloo on CPU).  ``grad`` is updated in place,
    ``terms``' loss scalars are replaced by their global values."""
    import torch.distributed as dist
    flat = torch.cat([grad.reshape(-1)] + [terms[k].detach().reshape(1).to(grad.dtype) for k in LOSS_KEYS])
    dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=group)
    n = grad.numel()
    grad.copy_(flat[:n].view_as(grad))
    for i, k in enumerate(LOSS_KEYS):
        terms[k] = flat[n + i]
    return grad


class GlobalBatchSampler(torch.utils.data.Sampler):
    """Distributed batch sampler with the reference's DataParallel semantics
    (train_patch.py:63-71, 123-127: ONE shuffled loader of ``global_batch``
    images per step, scattered over the GPUs).

    Every rank draws the same permutation (seed + epoch, ``set_epoch``) and
    yields its CONTIGUOUS slice [lo, hi) of each global batch, so the images of
    global step k are the same for any number of ranks and so are their
    transformer draws (keyed by the global index lo + i).  A ragged last batch
    is split as evenly as possible (the loss weights account for it); when it
    holds fewer images than there are ranks, the surplus ranks get EMPTY
    shards and contribute only their share of the patch terms (PatchTrainer.
    losses on an empty batch), so the epoch trains on the same images in the
    same steps as one process whatever the world size."""

    def __init__(self, n_items, global_batch, rank=0, world=1, shuffle=True, seed=0):
        self.n, self.G, self.rank, self.world = int(n_items), int(global_batch), int(rank), int(world)
        self.shuffle, self.seed, self.epoch = shuffle, int(seed), 0

    def set_epoch(self, epoch):
        self.epoch = int(epoch)

    def __len__(self):
        return -(-self.n // self.G)

    def shard_of(self, k):
        """(lo, hi, n_global) of this rank's slice of global batch k."""
        ng = min(self.G, self.n - k * self.G)
        return self.rank * ng // self.world, (self.rank + 1) * ng // self.world, ng

    def __iter__(self):
        if self.shuffle:
            g = torch.Generator()
            g.manual_seed(self.seed + self.epoch)
            perm = torch.randperm(self.n, generator=g).tolist()
        else:
            perm = list(range(self.n))
        for k in range(len(self)):
            lo, hi, _ = self.shard_of(k)
            yield perm[k * self.G + lo:k * self.G + hi]


class PatchAdam(optim.Optimizer):
    """Adam(amsgrad) + the patch clamp as one HIP launch per step
    (po_adam_amsgrad; train_patch.py:131-136 builds the reference's
    torch.optim.Adam(amsgrad=True), :327-330 clamps after each step).  The
    update is torch's single-tensor Adam arithmetic (include/advpatch.h);
    PyTorch's fused Adam instead costs three multi-tensor launches plus the
    clamp, ~75 us per step on these 150k-element patches, for a 5 MB update.
    The state is torch's (``step``, ``exp_avg``, ``exp_avg_sq``,
    ``max_exp_avg_sq``; ``step`` a 0-dim float32 on the device, as under
    fused=True), so state_dicts move between the two and ReduceLROnPlateau
    drives ``lr`` as for torch's Adam.  ``found_inf`` (a device float) or
    ``skip_flags`` ((flag tensor, bit)) skips the update on the device, with
    the count unchanged.  CUDA float32 contiguous parameters only: there is no
    CPU path (use torch.optim.Adam there)."""

    clamps = True     # the trainer skips its own clamp_

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, clamp=(0.0, 1.0)):
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=0, amsgrad=True, maximize=False, foreach=None,
                        capturable=False, differentiable=False, fused=True)
        super().__init__(params, defaults)
        self.clamp = clamp
        self.found_inf = None
        self.skip_flags = None
        self._spare = {}

    def load_state_dict(self, state_dict):
        """torch's, then every ``step`` count onto its parameter's device as a
        0-dim float32 (a CPU Adam's state keeps it on the host)."""
        super().load_state_dict(state_dict)
        for p, st in self.state.items():
            if "step" in st:
                st["step"] = torch.as_tensor(st["step"]).to(device=p.device, dtype=torch.float32).reshape(())
            self._spare.pop(p, None)

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for group in self.param_groups:
            beta1, beta2 = group["betas"]
            for p in group["params"]:
                if p.grad is None:
                    continue
                if not (p.is_cuda and p.dtype == torch.float32 and p.is_contiguous() and p.grad.is_contiguous()):
                    raise RuntimeError("PatchAdam: CUDA float32 contiguous parameters and gradients only")
                st = self.state[p]
                if len(st) == 0:
                    st["step"] = torch.zeros((), dtype=torch.float32, device=p.device)
                    for k in ("exp_avg", "exp_avg_sq", "max_exp_avg_sq"):
                        st[k] = torch.zeros_like(p, memory_format=torch.contiguous_format)
                spare = self._spare.get(p)
                if spare is None or spare.device != p.device or spare is st["step"]:
                    spare = torch.empty((), dtype=torch.float32, device=p.device)
                flags, bit = self.skip_flags if self.skip_flags is not None else (None, 0)
                lo, hi = self.clamp if self.clamp is not None else (0.0, 0.0)
                nat.call("po_adam_amsgrad", nat.ptr(p), nat.ptr(p.grad), nat.ptr(st["exp_avg"]),
                         nat.ptr(st["exp_avg_sq"]), nat.ptr(st["max_exp_avg_sq"]), p.numel(), nat.ptr(st["step"]),
                         nat.ptr(spare), float(group["lr"]), float(beta1), float(beta2), float(group["eps"]),
                         nat.ptr(self.found_inf) if self.found_inf is not None else None,
                         nat.ptr(flags, torch.int32) if flags is not None else None, int(bit),
                         int(self.clamp is not None), float(lo), float(hi), nat.stream())
                self._spare[p] = st["step"]
                st["step"] = spare
        return loss


class PatchTrainer(object):
    """train_patch.py:48-577"""

    def __init__(self, mode, device=None, objective="ce", distributed=None, verbose=True):
        self.config = patch_config.patch_configs[mode]()
        self.verbose = verbose
        if verbose:
            print("training mode : ", mode)
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.objective = objective
        self.last_plan = None      # NetPlan of the latest forward (tests, bench)
        self.darknet_model = Darknet(self.config.cfgfile)
        wf = self.config.weightfile
        if not os.path.exists(wf) and wf == patch_config.synthetic_weights_path("yolov3-dota"):
            synth_weights.ensure_synthetic(self.config.cfgfile, wf)
        self.darknet_model.load_darknet_weights(wf)
        self.darknet_model = self.darknet_model.eval()
        self.darknet_model_1 = self.darknet_model
        # classes per anchor of the YOLO heads; po_cell_loss reads 5 + 15 channels per
        # anchor, as the reference's loss head does (train_patch.py:459)
        self.num_classes = int(next(b["classes"] for b in self.darknet_model.blocks if b["type"] == "yolo"))
        if self.num_classes != CELL_CLASSES:
            raise ValueError("%s: YOLO heads with %d classes; the loss head (po_cell_loss, train_patch.py:459) "
                             "reads 5 + %d channels per anchor" % (self.config.cfgfile, self.num_classes, CELL_CLASSES))
        self.patch_applier = PatchApplier()
        self.patch_transformer = PatchTransformer()
        self.nps_calculator = NPSCalculator(self.config.printfile, self.config.patch_size).to(self.device)
        self.total_variation = TotalVariation().to(self.device)
        self.colorful_loss = HasSusRGB().to(self.device)
        self.dist = distributed if distributed is not None else (
            torch.distributed.is_available() and torch.distributed.is_initialized())
        self.rank = torch.distributed.get_rank() if self.dist else 0
        self.world = torch.distributed.get_world_size() if self.dist else 1
        self._tv_floor = None
        # device word of error bits (FLAG_BITS), OR-ed by the kernels, read by check_flags()
        self.flags = torch.zeros(1, dtype=torch.int32, device=self.device)
        # NaN/Inf guard on the patch gradient (replaces detect_anomaly, train_patch.py:158)
        self.check_finite = os.environ.get("ADVPATCH_CHECK_FINITE", "1") != "0"
        self._found_inf = None
        self._seed = None

    # ------------------------------------------------------------------
    def generate_patch(self, type):
        """'gray' or 'random' [3,P,P] patch (train_patch.py:391-409)."""
        if type == "gray":
            return torch.full((3, self.config.patch_size, self.config.patch_size), 0.5)
        elif type == "random":
            return torch.rand((3, self.config.patch_size, self.config.patch_size))
        raise ValueError(type)

    def read_image(self, path):
        """Load a trained patch and resize to patch_size (train_patch.py:411-426)."""
        from PIL import Image
        img = Image.open(path).convert("RGB").resize((self.config.patch_size, self.config.patch_size),
                                                     Image.BILINEAR)
        return torch.from_numpy(np.asarray(img, dtype=np.uint8).copy()).permute(2, 0, 1).float().div_(255.0)

    # ------------------------------------------------------------------
    def losses(self, adv_patch, img_batch, lab_batch, draws=None, objective=None, weights=None):
        """Forward of one iteration (train_patch.py:164-314) on the HIP path.
        ``weights``: shard_weights(...) of a data-parallel rank (None: the
        whole batch is here).  Returns (loss, terms dict); ``loss.backward()``
        yields adv_patch.grad."""
        objective = objective or self.objective
        img_size = self.darknet_model.height
        if img_batch.size(0) == 0:
            return self._patch_terms_only(adv_patch, objective, weights)
        net = self.darknet_model
        B, S = img_batch.size(0), img_batch.size(-1)
        # the composite is written only inside the patch footprints when the first
        # layer can read it beside the frames (po_conv_first_*_cmp): no B*3*S*S copy
        sparse = (img_batch.size(-2) == S == net.height == net.width and self.patch_transformer.sparse_ok(S, draws)
                  and net.sparse_input_ok(B, S, S, img_batch.device, center=True)
                  and os.environ.get("ADVPATCH_SPARSE_COMPOSITE", "1") != "0")
        self.last_sparse = sparse
        # the median pool and the regularisers of the patch: one autograd node
        mp, reg = patch_front(adv_patch, self.nps_calculator.colors)
        p_img, center = self.patch_transformer.forward_composite(adv_patch, lab_batch, img_batch, img_size,
                                                                 do_rotate=True, draws=draws, sparse=sparse, mp=mp)
        roi = self.patch_transformer.last_roi
        if p_img.size(-1) != net.width or p_img.size(-2) != net.height:
            p_img = F.interpolate(p_img, (net.height, net.width))
            roi = None
        # the warp backward reads dL/dp_img only inside the patch footprint:
        # the first conv's input gradient is computed there only
        heads, plan = net.forward_nhwc(p_img, input_roi=roi, center=center,
                                       base=img_batch.contiguous() if sparse else None)
        self.last_plan = plan
        out2, obj, cls, cells, flags = cell_loss(heads, plan, img_size, center, TARGET_ID, objective,
                                                 flags=self.flags)
        loss, terms = combine_terms_device(out2, reg, objective, weights)
        terms.update({"patch_center": center, "obj": obj, "cls": cls, "cells": cells, "flags": flags})
        return loss, terms

    def _patch_terms_only(self, adv_patch, objective, weights):
        """The loss of a rank whose shard of a global batch is empty (a ragged
        last batch with fewer images than ranks, GlobalBatchSampler): no image
        terms, its 1/world share of NPS/TV/colour, so the SUM all-reduce still
        yields the global-batch loss and gradient."""
        dev = adv_patch.device
        reg = regularisers(adv_patch, self.nps_calculator.colors)
        if self._tv_floor is None or self._tv_floor.device != dev:
            self._tv_floor = torch.tensor(0.1, device=dev)
        z = torch.zeros((), device=dev)
        loss, terms = combine_terms(z, z, reg[0], reg[1], reg[2], objective, weights, self._tv_floor)
        terms.update({"patch_center": torch.empty(0, 2, device=dev), "obj": torch.empty(0, 0, device=dev),
                      "cls": torch.empty(0, 0, self.num_classes, device=dev), "cells": torch.empty(0, 0, dtype=torch.int32,
                                                                                   device=dev),
                      "flags": self.flags})
        return loss, terms

    def allreduce_grad(self, adv_patch, terms):
        """One all-reduce(SUM) of [patch grad | weighted loss scalars] over all ranks.
        With ``self.ar_timer`` a list (bench.py's instrumented pass), a pair of
        device events brackets the reduction on the current stream."""
        if self.dist:
            timer = getattr(self, "ar_timer", None)
            if timer is not None and adv_patch.grad.is_cuda:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                allreduce_patch_grad(adv_patch.grad, terms)
                e1.record()
                timer.append((e0, e1))
            else:
                allreduce_patch_grad(adv_patch.grad, terms)

    def step(self, adv_patch, optimizer, img_batch, lab_batch, draws=None, weights=None):
        """One full iteration: forward, backward, [all-reduce], Adam, clamp (train_patch.py:164-330)."""
        loss, terms = self.losses(adv_patch, img_batch, lab_batch, draws, weights=weights)
        if self._seed is None or self._seed.device != loss.device:
            self._seed = torch.ones((), device=loss.device)                 # dL/dL, allocated once
        loss.backward(self._seed)
        self.allreduce_grad(adv_patch, terms)
        if self.check_finite and isinstance(optimizer, PatchAdam):
            # after the all-reduce (every rank sees the same gradient, raises the same
            # bit and skips the same update); PatchAdam reads the flag word itself
            g = adv_patch.grad
            nat.call("po_check_finite", nat.ptr(g), g.numel(), FLAG_NONFINITE, nat.ptr(self.flags, torch.int32),
                     nat.stream())
            optimizer.skip_flags = (self.flags, FLAG_NONFINITE)
        elif self.check_finite:
            # after the all-reduce: a NaN/Inf on any rank reaches every rank's reduced
            # gradient, so all ranks raise the same bit and skip the same updates
            g = adv_patch.grad
            fused = bool(optimizer.defaults.get("fused"))
            if fused and (self._found_inf is None or self._found_inf.device != g.device):
                # po_check_finite_inf writes it from the flag word after the check
                self._found_inf = torch.zeros((), device=g.device)         # 0-dim, as Adam's step counters
            nat.call("po_check_finite_inf", nat.ptr(g), g.numel(), FLAG_NONFINITE, nat.ptr(self.flags, torch.int32),
                     nat.ptr(self._found_inf) if fused else None, nat.stream())
            if fused:
                # once the bit is up the fused Adam skips its update (found_inf, as under
                # GradScaler): the patch stays at its last finite value until check_flags
                # raises at the end of the epoch, instead of being corrupted by the NaN
                optimizer.found_inf = self._found_inf
        optimizer.step()
        optimizer.zero_grad()
        if not getattr(optimizer, "clamps", False):
            adv_patch.data.clamp_(0, 1)
        return terms

    def check_flags(self):
        """Raise if any kernel raised an error bit since the trainer was built
        (one device->host read; call it per epoch, not per step)."""
        f = int(self.flags.item())
        plan = self.last_plan
        if plan is not None and getattr(plan, "windowed", False):
            f |= int(plan.win_flags.item())
        if f:
            raise RuntimeError("advpatch step error flags 0x%x: %s" % (
                f, "; ".join(v for k, v in FLAG_BITS.items() if f & k)))

    def make_optimizer(self, adv_patch):
        """Adam(amsgrad) as the reference (train_patch.py:131-136); on the GPU
        PyTorch's fused single-kernel implementation (same update rule) instead
        of the multi-launch foreach one.  north_star keeps the outer Adam step
        in PyTorch-ROCm, so that is the default; ADVPATCH_HIP_ADAM=1 selects
        PatchAdam (one po_adam_amsgrad launch, the clamp fused; measured +1 %
        on config 5, neutral on the headline, profiles/r06/patch_adam_ab.txt)."""
        if adv_patch.is_cuda and os.environ.get("ADVPATCH_HIP_ADAM") == "1":
            return PatchAdam([adv_patch], lr=self.config.start_learning_rate)
        return optim.Adam([adv_patch], lr=self.config.start_learning_rate, amsgrad=True,
                          fused=bool(adv_patch.is_cuda) or None)

    # ------------------------------------------------------------------
    def train(self, max_n_epochs=401, save_dir="training_patches_saves/trained_patches", num_workers=10,
              data=None, seed=0, cache_frames=None, save_state=False, resume=None):
        """Optimise a patch on the configured dataset (train_patch.py:85-389).
        ``config.batch_size`` is the GLOBAL batch, as in the reference; under
        torchrun every rank loads its contiguous shard of each global batch
        (GlobalBatchSampler).  ``data``: optional iterable of (img_batch,
        lab_batch) replacing the DataLoader (under torchrun: this rank's
        equal shards).  ``cache_frames``: decode the dataset once into device
        memory (FrameCache) instead of every epoch; None = when the uint8
        frames take at most a quarter of the free device memory.
        ``save_state``: beside every saved PNG also write ``<epoch>_state.pt``
        (fp32 patch, Adam(amsgrad) moments, LR-scheduler state, epoch and step
        counters; save_train_state).  ``resume``: such a file; training
        continues at the epoch after it with the same patch, optimizer and
        scheduler state, and since the loader order (seed + epoch) and the
        transformer draws (global step) are keyed, not streamed, the resumed
        run ends where the uninterrupted one does.  The reference resumes
        only from a PNG (read_image, train_patch.py:119-121)."""
        img_size = self.darknet_model.height
        batch_size = self.config.batch_size
        max_lab = 252
        rank0 = self.rank == 0
        torch.manual_seed(seed)
        adv_patch = self.generate_patch("random").to(self.device).requires_grad_(True)
        state = load_train_state(resume) if resume else None
        sampler = None
        if data is None:
            n_images = len(fnmatch.filter(os.listdir(self.config.img_dir), "*.png")) + \
                len(fnmatch.filter(os.listdir(self.config.img_dir), "*.jpg"))
            if self.verbose and rank0:
                print("Total images in TrainSet : ", n_images)
            ds = DotaDataset(self.config.img_dir, self.config.lab_dir, max_lab, img_size, shuffle=True, as_uint8=True)
            collate = DotaCollate(img_size, max_lab, as_uint8=True)
            sampler = GlobalBatchSampler(len(ds), batch_size, self.rank, self.world, shuffle=True, seed=seed)
            if cache_frames is None:
                need = len(ds) * (3 * img_size * img_size + max_lab * 5 * 4)
                cache_frames = self.device.type == "cuda" and need <= torch.cuda.mem_get_info(self.device)[0] // 4
            if cache_frames:
                loader = FrameCache(ds, self.device, num_workers=num_workers).loader(sampler)
            else:
                loader = DevicePrefetcher(torch.utils.data.DataLoader(
                    ds, batch_sampler=sampler, num_workers=num_workers, pin_memory=True,
                    persistent_workers=num_workers > 0, collate_fn=collate,
                    multiprocessing_context=loader_context(self.device) if num_workers else None), self.device)
        else:
            loader = DevicePrefetcher(data, self.device)
        optimizer = self.make_optimizer(adv_patch)
        scheduler = self.config.scheduler_factory(optimizer)
        ep_loss_list = []
        keys = LOSS_KEYS
        step = 0
        first_epoch = 0
        if state is not None:
            with torch.no_grad():
                adv_patch.copy_(state["patch"])
            optimizer.load_state_dict(state["optimizer"])
            scheduler.load_state_dict(state["scheduler"])
            first_epoch, step = int(state["epoch"]) + 1, int(state["step"])
            ep_loss_list = [float(v) for v in state["ep_losses"]]
        self.patch_transformer.draw_seed = seed + 3
        for epoch in range(first_epoch, max_n_epochs):
            if sampler is not None:
                sampler.set_epoch(epoch)
            sums = {k: torch.zeros((), device=self.device) for k in keys}
            nb = 0
            et0 = time.time()
            for k, (img_batch, lab_batch) in enumerate(loader):
                weights = None
                if sampler is not None:
                    lo, hi, ng = sampler.shard_of(k)
                    b0 = lo
                    if self.dist:
                        weights = shard_weights(hi - lo, ng, self.world, self.objective)
                else:
                    n = img_batch.size(0)
                    b0 = self.rank * n
                    if self.dist:
                        weights = shard_weights(n, n * self.world, self.world, self.objective)
                # draws of global step `step`, rows of this rank's images
                self.patch_transformer.draw_step, self.patch_transformer.draw_b0 = step, b0
                terms = self.step(adv_patch, optimizer, img_batch, lab_batch, weights=weights)
                for key in keys:
                    sums[key] += terms[key].detach()
                nb += 1
                step += 1
            self.check_flags()
            ep = {key: (v / max(nb, 1)).item() for key, v in sums.items()}
            scheduler.step(ep["loss"] * max(nb, 1))        # the reference steps on the epoch SUM (332)
            ep_loss_list.append(ep["no_obj_loss"] / 4)
            if self.verbose and rank0:
                print("  EPOCH NR: ", epoch)
                print("EPOCH LOSS: ", ep["loss"])
                print("  NPS LOSS: ", ep["nps_loss"])
                print("   TV LOSS: ", ep["tv_loss"])
                print("  NO_OBJ LOSS: ", ep["no_obj_loss"])
                print("  NO_CLS LOSS: ", ep["no_cls_loss"])
                print("  COLORFUL LOSS: ", ep["colorful_loss"])
                print("EPOCH TIME: ", time.time() - et0)
            if epoch % 20 == 0 and save_dir and rank0:
                path = os.path.join(save_dir, "%d_patch.png" % epoch)
                save_patch_png(adv_patch.detach(), path)
                if save_state:
                    save_train_state(os.path.join(save_dir, "%d_state.pt" % epoch), adv_patch, optimizer, scheduler,
                                     epoch, step, ep_loss_list)
                if self.verbose:
                    print("saved patch dir : ", save_dir)
                if epoch > 0 and self.verbose:
                    prev = os.path.join(save_dir, "%d_patch.png" % (epoch - 20))
                    print("MSE-loss between adjacent patch : ", patch_mse(prev, path))
        return adv_patch.detach(), ep_loss_list

    # ------------------------------------------------------------------
    # Reference loss-head methods (train_patch.py:428-577), vectorised on the
    # device for drop-in use on NCHW head tensors; the training step uses the
    # fused po_cell_loss kernel instead.
    def obj_cls_conf_find(self, outputs, img_size, patch_center):
        obj_all, cls_all = [], []
        for output in outputs:
            batch, h, w = output.size(0), output.size(2), output.size(3)
            feature_size = output.size(-1)
            axis = torch.div(patch_center, img_size / feature_size, rounding_mode="floor").long()
            index = axis[:, 0] * feature_size + axis[:, 1]
            o = output.view(batch, 3, 20, h * w)
            cells = torch.sigmoid(o[torch.arange(batch, device=o.device), :, 4:20, index])   # [B,3,16]
            obj_all.append([cells[i, :, 0].view(-1, 3) for i in range(batch)])
            cls_all.append([cells[i, :, 1:16] for i in range(batch)])
        return obj_all, cls_all

    def no_obj_reshape(self, index_obj_conf):
        B = len(index_obj_conf[0])
        t = torch.stack([torch.cat(o, 0) for o in index_obj_conf], 0)     # [3,B,3]
        return t.transpose(0, 1).reshape(B, 9)

    def no_cls_reshape(self, index_cls_conf):
        B = len(index_cls_conf[0])
        t = torch.stack([torch.stack(c, 0) for c in index_cls_conf], 0)   # [3,B,3,15]
        return t.transpose(0, 1).reshape(B, 9, 15)

    def noCLS_Loss_CE(self, no_cls_reshape, cls_ID):
        B, A = no_cls_reshape.size(0), no_cls_reshape.size(1)
        target = torch.full((B * A,), cls_ID, dtype=torch.long, device=no_cls_reshape.device)
        per = F.cross_entropy(no_cls_reshape.reshape(B * A, -1), target, reduction="none").view(B, A)
        return per.mean(1).mean()

    def noCLS_loss_targeted(self, no_cls_reshape, cls_ID):
        t = no_cls_reshape[:, :, cls_ID]
        mx, _ = torch.max(no_cls_reshape, dim=2)
        return (mx - t).mean(1).sum()


def _to_cpu(obj):
    if torch.is_tensor(obj):
        return obj.detach().cpu()
    if isinstance(obj, dict):
        return {k: _to_cpu(v) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return type(obj)(_to_cpu(v) for v in obj)
    return obj


def save_train_state(path, adv_patch, optimizer, scheduler, epoch, step, ep_losses):
    """Training state after ``epoch`` (SURVEY §5's optional fp32 checkpoint
    beside the PNG): the exact fp32 patch (the PNG holds trunc(255*x)), Adam's
    state_dict (step counters, exp_avg, exp_avg_sq, max_exp_avg_sq), the
    scheduler's and the counters.  Tensors only, no pickled objects, so
    load_train_state reads it with torch.load(weights_only=True)."""
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    torch.save({"format": "advpatch-train-state-1", "patch": adv_patch.detach().float().cpu(),
                "optimizer": _to_cpu(optimizer.state_dict()), "scheduler": _to_cpu(scheduler.state_dict()),
                "epoch": int(epoch), "step": int(step), "ep_losses": [float(v) for v in ep_losses]}, path)


def load_train_state(path):
    st = torch.load(path, map_location="cpu", weights_only=True)
    if not isinstance(st, dict) or st.get("format") != "advpatch-train-state-1":
        raise ValueError("%s is not an advpatch training state (save_train_state)" % path)
    return st


def save_patch_png(patch, path):
    """``ToPILImage('RGB')`` layout: uint8 = trunc(255*x) (train_patch.py:369-376)."""
    from PIL import Image
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    arr = patch.detach().float().cpu().mul(255).byte().permute(1, 2, 0).numpy()
    Image.fromarray(arr, "RGB").save(path)


def patch_mse(path0, path1):
    """MSE between two saved patches read back as ToTensor floats
    (utils_self.patch_MSE_calsulator, utils_self.py:205-220)."""
    a, b = _read_image(path0), _read_image(path1)
    return float(((a - b) ** 2).mean())


def main():
    """train_patch.py:580-606; the mode is a real CLI argument (default paper_obj)."""
    mode = sys.argv[1] if len(sys.argv) > 1 else "paper_obj"
    trainer = PatchTrainer(mode)
    return trainer.train()


if __name__ == "__main__":
    t0 = time.time()
    print("TV FACTOR : ", TV_FACTOR)
    print("NPS FACTOR : ", NPS_FACTOR)
    print("TARGET ID : ", TARGET_ID)
    main()
    print("Total training time: {:.4f} minutes".format((time.time() - t0) / 60))
