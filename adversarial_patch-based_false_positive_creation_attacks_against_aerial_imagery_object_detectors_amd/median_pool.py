"""MedianPool2d — drop-in for reference ``median_pool.py:8-52`` on the HIP path.

The training path uses ``MedianPool2d(7, same=True)`` on the [1,3,P,P] patch
(load_data.py:439, 531).  That configuration (k=7, stride 1, 'same' reflect
padding) runs as ``po_median7_fwd``/``po_median7_bwd`` (49 values in
registers); every other kernel size / stride / padding runs as the general
``po_median_fwd``/``po_median_bwd`` (the reference module's full surface).

Tie rule (the reference's is implementation-defined): the
gradient goes to the first window position, row-major, holding the median.
"""
import torch
import torch.nn as nn
from torch.nn.modules.utils import _pair, _quadruple

from . import _native as nat


class _Median7(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        nat.ensure_device(x)
        x = x.contiguous()
        N, C, H, W = x.shape
        y = torch.empty_like(x)
        arg = torch.empty(x.shape, dtype=torch.int32, device=x.device)
        nat.call("po_median7_fwd", nat.ptr(x), N * C, H, W, nat.ptr(y), nat.ptr(arg, torch.int32),
                 nat.stream())
        ctx.save_for_backward(arg)
        ctx.shape = (N * C, H, W)
        return y

    @staticmethod
    def backward(ctx, dy):
        (arg,) = ctx.saved_tensors
        dy = dy.contiguous()
        dx = torch.empty_like(dy)
        C, H, W = ctx.shape
        nat.call("po_median7_bwd", nat.ptr(dy), nat.ptr(arg, torch.int32), C, H, W, nat.ptr(dx),
                 nat.stream())
        return dx


class _MedianGeneral(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k, stride, pad):
        nat.ensure_device(x)
        x = x.contiguous()
        N, C, H, W = x.shape
        (kh, kw), (sh, sw), (pl, pr, pt, pb) = k, stride, pad
        Ho, Wo = (H + pt + pb - kh) // sh + 1, (W + pl + pr - kw) // sw + 1
        y = torch.empty(N, C, Ho, Wo, device=x.device)
        arg = torch.empty(N, C, Ho, Wo, dtype=torch.int32, device=x.device)
        nat.call("po_median_fwd", nat.ptr(x), N * C, H, W, kh, kw, sh, sw, pl, pr, pt, pb, nat.ptr(y),
                 nat.ptr(arg, torch.int32), nat.stream())
        ctx.save_for_backward(arg)
        ctx.meta = (x.shape, k, stride, pad)
        return y

    @staticmethod
    def backward(ctx, dy):
        (arg,) = ctx.saved_tensors
        shape, (kh, kw), (sh, sw), (pl, pr, pt, pb) = ctx.meta
        N, C, H, W = shape
        dx = torch.empty(shape, device=dy.device)
        nat.call("po_median_bwd", nat.ptr(dy.contiguous()), nat.ptr(arg, torch.int32), N * C, H, W, kh, kw, sh, sw,
                 pl, pr, pt, pb, nat.ptr(dx), nat.stream())
        return dx, None, None, None


def median_pool7(x):
    """[N,C,H,W] -> [N,C,H,W], 7x7 median with reflect 'same' padding."""
    return _Median7.apply(x)


class MedianPool2d(nn.Module):
    """Median pool (usable as median filter when stride=1) module.

    Args (as the reference):
         kernel_size: size of pooling kernel, int or 2-tuple
         stride: pool stride, int or 2-tuple
         padding: pool padding, int or 4-tuple (l, r, t, b) as in pytorch F.pad
         same: override padding and enforce same padding, boolean
    """

    def __init__(self, kernel_size=3, stride=1, padding=0, same=False):
        super().__init__()
        self.k = _pair(kernel_size)
        self.stride = _pair(stride)
        self.padding = _quadruple(padding)
        self.same = same

    def _padding(self, x):
        """(l, r, t, b) exactly as reference median_pool.py:26-44."""
        if self.same:
            ih, iw = x.size()[2:]
            ph = max(self.k[0] - (self.stride[0] if ih % self.stride[0] == 0 else ih % self.stride[0]), 0)
            pw = max(self.k[1] - (self.stride[1] if iw % self.stride[1] == 0 else iw % self.stride[1]), 0)
            return (pw // 2, pw - pw // 2, ph // 2, ph - ph // 2)
        return self.padding

    def forward(self, x):
        """reflect pad, kh x kw windows at the stride, lower median
        (median_pool.py:46-52); the 7x7 'same' case takes the fast kernels."""
        pad = tuple(int(v) for v in self._padding(x))
        if self.k == (7, 7) and self.stride == (1, 1) and pad == (3, 3, 3, 3):
            return median_pool7(x)
        return _MedianGeneral.apply(x, tuple(self.k), tuple(self.stride), pad)
