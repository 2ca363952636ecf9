"""MaxProbExtractor (reference load_data.py:125-311) on the HIP path.

Re-exported by ``load_data`` under the reference's name.  The reference
constructs it (train_patch.py:74-75) but its call is commented out (255); it is
the full-map variant of the objectness objective.
"""
import torch
import torch.nn as nn

from . import _native as nat


def _head_strides(heads):
    """(h [n], w [n], strides [3n] = image, channel, pixel element strides).  A
    head is [B, 3*(5+C), h, w] with any strides whose pixel index r*w + c maps
    to one pixel stride (NCHW contiguous, or an NHWC buffer viewed as NCHW)."""
    n = len(heads)
    hs, ws, st = (nat.c_int * n)(), (nat.c_int * n)(), (nat.c_int64 * (3 * n))()
    for k, t in enumerate(heads):
        sb, sc, sr, sq = t.stride()
        if sr != t.size(3) * sq:
            raise ValueError("MaxProbExtractor: head %d rows and columns do not share one pixel stride" % k)
        hs[k], ws[k] = t.size(2), t.size(3)
        st[3 * k], st[3 * k + 1], st[3 * k + 2] = sb, sc, sq
    return hs, ws, st


class _MaxProb(torch.autograd.Function):
    @staticmethod
    def forward(ctx, cls_id, num_cls, sigmoid_mode, *heads):
        nat.ensure_device(heads[0])
        B = heads[0].size(0)
        for t in heads:
            if t.dtype != torch.float32 or t.dim() != 4 or t.size(0) != B or t.size(1) < 3 * (5 + num_cls):
                raise ValueError("MaxProbExtractor: heads must be float32 [B, >=3*(5+%d), h, w]" % num_cls)
        hs, ws, st = _head_strides(heads)
        out = torch.empty(2, B, device=heads[0].device)
        idx = torch.empty(2, B, dtype=torch.int32, device=heads[0].device)
        nat.call("po_max_prob", nat.ptr_array(heads), hs, ws, st, len(heads), B, int(num_cls), int(cls_id),
                 int(bool(sigmoid_mode)), nat.ptr(out), nat.ptr(idx, torch.int32), nat.stream())
        ctx.save_for_backward(idx, *heads)
        ctx.meta = (int(cls_id), int(num_cls), int(bool(sigmoid_mode)))
        ctx.mark_non_differentiable(idx)
        return out[0], out[1], idx

    @staticmethod
    def backward(ctx, g_obj, g_cls, _):
        idx, *heads = ctx.saved_tensors
        cls_id, num_cls, sigmoid_mode = ctx.meta
        B = heads[0].size(0)
        g = torch.zeros(2, B, device=heads[0].device)
        if g_obj is not None:
            g[0] = g_obj
        if g_cls is not None:
            g[1] = g_cls
        d_heads = [torch.zeros_like(t) for t in heads]
        for t, d in zip(heads, d_heads):
            if d.stride() != t.stride():
                raise RuntimeError("MaxProbExtractor: gradient buffer strides differ from the head's")
        hs, ws, st = _head_strides(heads)
        nat.call("po_max_prob_bwd", nat.ptr_array(heads), hs, ws, st, len(heads), B, num_cls, cls_id, sigmoid_mode,
                 nat.ptr(idx, torch.int32), nat.ptr(g), nat.ptr_array(d_heads), nat.stream())
        return (None, None, None) + tuple(d_heads)


class MaxProbExtractor(nn.Module):
    """Per-image max objectness and max class-``cls_id`` confidence over every
    anchor of every head (load_data.py:125-311).  ``forward(YOLOoutputs,
    sigmoid_mode=False)`` takes the raw head tensors [B, 3*(5+C), h, w] of
    ``Darknet.forward`` and returns (max_obj_conf [B], max_cls_conf [B]).
    bbox_decode (load_data.py:63-122) only rewrites the box fields, so no
    decode pass runs; one workgroup per image and quantity reduces with wave
    shuffles (po_max_prob), and the gradient goes to the selected element
    (torch.max's first index on ties)."""

    def __init__(self, cls_id, num_cls, config=None):
        super().__init__()
        self.cls_id = cls_id
        self.num_cls = num_cls
        self.config = config
        self.last_index = None      # [2,B] int32 flat output_cat indices of the maxima

    def forward(self, YOLOoutputs, sigmoid_mode=False):
        max_obj, max_cls, idx = _MaxProb.apply(self.cls_id, self.num_cls, sigmoid_mode, *YOLOoutputs)
        self.last_index = idx
        return max_obj, max_cls
