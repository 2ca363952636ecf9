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
``int()`` syncs in ``obj_cls_conf_find`` plus 5 ``.cpu()`` per iteration).
Multi-GPU: one process per GPU (torchrun); each rank runs its shard of the
global batch and the patch gradient (with the loss scalars) is averaged with a
single all-reduce — replacing the reference's ``nn.DataParallel``
(train_patch.py:63-71).
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
from .load_data import (DotaDataset, HasSusRGB, NPSCalculator, PatchApplier, PatchTransformer,
                        TotalVariation, read_image as _read_image, regularisers)

TV_FACTOR = 2.5      # train_patch.py:25
NPS_FACTOR = 0.01    # train_patch.py:26
TARGET_ID = 14       # train_patch.py:28 (helicopter)
OBJECTIVES = {"ce": 0, "targeted": 1, "untargeted": 2}


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
    def forward(ctx, center, S, target, objective, hw, Cp, views, *heads):
        B = center.size(0)
        dev = center.device
        A = 3 * len(heads)
        out2 = torch.empty(2, device=dev)
        obj = torch.empty(B, A, device=dev)
        cls = torch.empty(B, A, 15, device=dev)
        cells = torch.empty(len(heads), B, dtype=torch.int32, device=dev)
        flags = torch.zeros(1, dtype=torch.int32, device=dev)
        hwa, wina, orga = _head_args(hw, views)
        nat.call("po_cell_loss", nat.ptr_array(heads), hwa, wina, orga, len(heads), Cp, B, S,
                 nat.ptr(center.contiguous()), target, objective, None, None, nat.ptr(out2), nat.ptr(obj),
                 nat.ptr(cls), nat.ptr(cells, torch.int32), nat.ptr(flags, torch.int32), nat.stream())
        ctx.save_for_backward(center, *heads)
        ctx.meta = (S, target, objective, tuple(hw), Cp, views)
        ctx.mark_non_differentiable(obj, cls, cells, flags)
        return out2, obj, cls, cells, flags

    @staticmethod
    def backward(ctx, g2, *unused):
        center, *heads = ctx.saved_tensors
        S, target, objective, hw, Cp, views = ctx.meta
        d_heads = [torch.zeros_like(h) for h in heads]
        out2 = torch.empty(2, device=center.device)
        hwa, wina, orga = _head_args(hw, views)
        nat.call("po_cell_loss", nat.ptr_array(heads), hwa, wina, orga, len(heads), Cp, center.size(0), S,
                 nat.ptr(center.contiguous()), target, objective, nat.ptr(g2.contiguous().float()),
                 nat.ptr_array(d_heads), nat.ptr(out2), None, None, None, None, nat.stream())
        return (None, None, None, None, None, None, None) + tuple(d_heads)


def cell_loss(heads, plan, img_size, patch_center, target=TARGET_ID, objective="ce"):
    """-> (out2 [2] = {no_obj_loss, no_cls_loss}, obj [B,9], cls [B,9,15], cells, flags).
    ``heads`` are the plan's head buffers (full maps, or receptive-field
    windows when the plan was run with the patch centres)."""
    hw = [plan.shp[h][0] for h in plan.heads]
    Cp = plan.cp[plan.heads[0]]
    for h in plan.heads:
        assert plan.cp[h] == Cp and plan.shp[h][0] == plan.shp[h][1]
    return _CellLoss.apply(patch_center, int(img_size), int(target), OBJECTIVES[objective], hw, Cp,
                           plan.head_views(), *heads)


LOSS_KEYS = ("loss", "nps_loss", "tv_loss", "no_obj_loss", "no_cls_loss", "colorful_loss")


def allreduce_patch_grad(grad, terms, group=None):
    """Data-parallel reduction of one step: every rank holds
    the gradient of its local-mean loss; ONE all-reduce of the fused buffer
    [patch grad | 6 loss scalars] averages them, which equals the
    global-batch gradient for equal shards (the NPS/TV/colour terms are
    identical on every rank).  RCCL (backend "nccl") reduces with AVG; gloo
    with SUM then a division.  ``grad`` is updated in place, ``terms``' loss
    scalars are replaced by their averages."""
    import torch.distributed as dist
    world = dist.get_world_size(group)
    flat = torch.cat([grad.reshape(-1)] + [terms[k].detach().reshape(1).to(grad.dtype) for k in LOSS_KEYS])
    if dist.get_backend(group) == "nccl":
        dist.all_reduce(flat, op=dist.ReduceOp.AVG, group=group)
    else:
        dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=group)
        flat.div_(world)
    n = grad.numel()
    grad.copy_(flat[:n].view_as(grad))
    for i, k in enumerate(LOSS_KEYS):
        terms[k] = flat[n + i]
    return grad


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
        self.patch_applier = PatchApplier()
        self.patch_transformer = PatchTransformer()
        self.nps_calculator = NPSCalculator(self.config.printfile, self.config.patch_size).to(self.device)
        self.total_variation = TotalVariation().to(self.device)
        self.colorful_loss = HasSusRGB().to(self.device)
        self.dist = distributed if distributed is not None else (
            torch.distributed.is_available() and torch.distributed.is_initialized())
        self._tv_floor = None

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
    def losses(self, adv_patch, img_batch, lab_batch, draws=None, objective=None):
        """Forward of one iteration (train_patch.py:164-314) on the HIP path.
        Returns (loss, terms dict); ``loss.backward()`` yields adv_patch.grad."""
        objective = objective or self.objective
        img_size = self.darknet_model.height
        p_img, center = self.patch_transformer.forward_composite(adv_patch, lab_batch, img_batch, img_size,
                                                                 do_rotate=True, draws=draws)
        roi = self.patch_transformer.last_roi
        if p_img.size(-1) != self.darknet_model.width or p_img.size(-2) != self.darknet_model.height:
            p_img = F.interpolate(p_img, (self.darknet_model.height, self.darknet_model.width))
            roi = None
        # the warp backward reads dL/dp_img only inside the patch footprint:
        # the first conv's input gradient is computed there only
        heads, plan = self.darknet_model.forward_nhwc(p_img, input_roi=roi, center=center)
        self.last_plan = plan
        out2, obj, cls, cells, flags = cell_loss(heads, plan, img_size, center, TARGET_ID, objective)
        no_obj_loss, no_cls_loss = out2[0], out2[1]
        reg = regularisers(adv_patch, self.nps_calculator.colors)
        nps_loss = reg[0] * NPS_FACTOR
        tv_loss = reg[1] * TV_FACTOR
        colorful = reg[2]
        if self._tv_floor is None or self._tv_floor.device != adv_patch.device:
            self._tv_floor = torch.tensor(0.1, device=adv_patch.device)
        loss = nps_loss + torch.max(tv_loss, self._tv_floor) + no_obj_loss + colorful
        if objective != "untargeted":
            loss = loss + no_cls_loss
        terms = {"loss": loss, "nps_loss": nps_loss, "tv_loss": tv_loss, "no_obj_loss": no_obj_loss,
                 "no_cls_loss": no_cls_loss, "colorful_loss": colorful, "patch_center": center,
                 "obj": obj, "cls": cls, "cells": cells, "flags": flags}
        return loss, terms

    def allreduce_grad(self, adv_patch, terms):
        """One all-reduce(avg) of [patch grad | loss scalars] over all ranks."""
        if self.dist:
            allreduce_patch_grad(adv_patch.grad, terms)

    def step(self, adv_patch, optimizer, img_batch, lab_batch, draws=None):
        """One full iteration: forward, backward, [all-reduce], Adam, clamp (train_patch.py:164-330)."""
        loss, terms = self.losses(adv_patch, img_batch, lab_batch, draws)
        loss.backward()
        self.allreduce_grad(adv_patch, terms)
        optimizer.step()
        optimizer.zero_grad()
        adv_patch.data.clamp_(0, 1)
        return terms

    def make_optimizer(self, adv_patch):
        """Adam(amsgrad) as the reference (train_patch.py:131-136); on the GPU
        PyTorch's fused single-kernel implementation (same update rule) instead
        of the multi-launch foreach one."""
        return optim.Adam([adv_patch], lr=self.config.start_learning_rate, amsgrad=True,
                          fused=bool(adv_patch.is_cuda) or None)

    # ------------------------------------------------------------------
    def train(self, max_n_epochs=401, save_dir="training_patches_saves/trained_patches", num_workers=10,
              data=None):
        """Optimise a patch on the configured dataset (train_patch.py:85-389).
        ``data``: optional iterable of (img_batch, lab_batch) replacing the DataLoader."""
        img_size = self.darknet_model.height
        batch_size = self.config.batch_size
        max_lab = 252
        adv_patch = self.generate_patch("random").to(self.device).requires_grad_(True)
        if data is None:
            n_images = len(fnmatch.filter(os.listdir(self.config.img_dir), "*.png")) + \
                len(fnmatch.filter(os.listdir(self.config.img_dir), "*.jpg"))
            if self.verbose:
                print("Total images in TrainSet : ", n_images)
            loader = torch.utils.data.DataLoader(
                DotaDataset(self.config.img_dir, self.config.lab_dir, max_lab, img_size, shuffle=True),
                batch_size=batch_size, shuffle=True, num_workers=num_workers, pin_memory=True)
        else:
            loader = data
        optimizer = self.make_optimizer(adv_patch)
        scheduler = self.config.scheduler_factory(optimizer)
        ep_loss_list = []
        keys = ("loss", "nps_loss", "tv_loss", "no_obj_loss", "no_cls_loss", "colorful_loss")
        for epoch in range(max_n_epochs):
            sums = {k: torch.zeros((), device=self.device) for k in keys}
            nb = 0
            et0 = time.time()
            for img_batch, lab_batch in loader:
                img_batch = img_batch.to(self.device, non_blocking=True)
                lab_batch = lab_batch.to(self.device, non_blocking=True)
                terms = self.step(adv_patch, optimizer, img_batch, lab_batch)
                for k in keys:
                    sums[k] += terms[k].detach()
                nb += 1
            ep = {k: (v / max(nb, 1)).item() for k, v in sums.items()}
            scheduler.step(ep["loss"] * max(nb, 1))
            ep_loss_list.append(ep["no_obj_loss"] / 4)
            if self.verbose:
                print("  EPOCH NR: ", epoch)
                print("EPOCH LOSS: ", ep["loss"])
                print("  NPS LOSS: ", ep["nps_loss"])
                print("   TV LOSS: ", ep["tv_loss"])
                print("  NO_OBJ LOSS: ", ep["no_obj_loss"])
                print("  NO_CLS LOSS: ", ep["no_cls_loss"])
                print("  COLORFUL LOSS: ", ep["colorful_loss"])
                print("EPOCH TIME: ", time.time() - et0)
            if epoch % 20 == 0 and save_dir:
                save_patch_png(adv_patch.detach(), os.path.join(save_dir, "%d_patch.png" % epoch))
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


def save_patch_png(patch, path):
    """``ToPILImage('RGB')`` layout: uint8 = trunc(255*x) (train_patch.py:369-376)."""
    from PIL import Image
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    arr = patch.detach().float().cpu().mul(255).byte().permute(1, 2, 0).numpy()
    Image.fromarray(arr, "RGB").save(path)


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
