"""ctypes binding of libadvpatch_hip.so (C ABI declared in include/advpatch.h).

The library is the product path: there is no CPU or PyTorch fallback.  If the
shared object is missing, or the device is not gfx950, every op raises.
"""
import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
# ADVPATCH_LIB: an ablation build (tools/build_variant.sh) for A/B measurements only
LIB_PATH = os.environ.get("ADVPATCH_LIB") or os.path.join(_HERE, "libadvpatch_hip.so")

c_int, c_float, c_int64, c_void_p = ctypes.c_int, ctypes.c_float, ctypes.c_int64, ctypes.c_void_p
c_double = ctypes.c_double

PO_ABI_VERSION = 30   # include/advpatch.h
PO_CONV_NTILES = 73   # include/advpatch.h
PO_AMAX_SUB = 64      # sub-slots per max|x| slot


class po_conv_desc(ctypes.Structure):
    _fields_ = [(n, c_int) for n in (
        "B", "Hin", "Win", "Cin_p", "Hout", "Wout", "Cout_p", "Hg", "Wg",
        "in_step", "out_step", "out_oy", "out_ox", "ntaps")] + [
        ("dh", c_int * 9), ("dw", c_int * 9),
        ("N", c_int), ("act", c_int), ("accumulate", c_int), ("tile", c_int),
        ("in_org", c_void_p), ("out_org", c_void_p), ("ksplit", c_int), ("workspace", c_void_p),
        ("prec", c_int), ("w_shift", c_int), ("in_amax", c_void_p), ("y_amax", c_void_p),
        ("sum_amax", c_void_p), ("y2_amax", c_void_p), ("ybits", c_void_p), ("mbits", c_void_p),
        ("m2bits", c_void_p), ("gbox", c_void_p), ("Wfrag", c_void_p), ("Wwino", c_void_p), ("mrows", c_int),
        ("pool_y", c_void_p), ("pool_argmax", c_void_p),
        ("Wwino6", c_void_p), ("winov", c_void_p), ("winov_floats", c_int64),
        ("tile_ctr", c_void_p), ("tile_ctr_n", c_int)]


_SIGS = {
    "po_abi_version": [],
    "po_device_check": [c_int],
    "po_median7_fwd": [c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p],
    "po_median7_bwd": [c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p],
    "po_median_fwd": [c_void_p] + [c_int] * 11 + [c_void_p, c_void_p, c_void_p],
    "po_median_bwd": [c_void_p, c_void_p] + [c_int] * 11 + [c_void_p, c_void_p],
    "po_patch_params": [c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int,
                        c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p],
    "po_draws": [ctypes.c_uint64, ctypes.c_uint64, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                 c_void_p, c_void_p, c_void_p],
    "po_check_finite": [c_void_p, c_int64, c_int, c_void_p, c_void_p],
    "po_check_finite_inf": [c_void_p, c_int64, c_int, c_void_p, c_void_p, c_void_p],
    "po_adam_amsgrad": [c_void_p] * 5 + [c_int64, c_void_p, c_void_p] + [c_double] * 4 +
                       [c_void_p, c_void_p, c_int, c_int, c_float, c_float, c_void_p],
    "po_loss_combine": [c_void_p, c_void_p, c_float, c_float, c_float, c_int, c_int, c_void_p, c_void_p, c_void_p],
    "po_loss_combine_bwd": [c_void_p, c_void_p, c_float, c_float, c_float, c_int, c_int, c_void_p, c_void_p,
                            c_void_p],
    "po_region_boxes": [c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p, c_float, c_float, c_float, c_float,
                        c_float, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p],
    "po_nms": [c_void_p, c_void_p, c_int, c_int, c_int, c_float, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p],
    "po_nms_workspace": [c_int, c_int, ctypes.POINTER(c_int64), ctypes.POINTER(c_int64)],
    "po_place_test_mode": [c_void_p, c_int, c_void_p, c_void_p, c_int, c_int, c_int, c_float, c_void_p, c_void_p,
                           c_void_p, c_void_p, c_void_p, c_void_p, c_void_p],
    "po_place_workspace": [c_int, c_int, c_int, ctypes.POINTER(c_int64), ctypes.POINTER(c_int64)],
    "po_place_free_map": [c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p],
    "po_vanishing_params": [c_void_p, c_int, c_int, c_int, c_int, c_float, c_void_p, c_void_p, c_void_p, c_int,
                            c_void_p, c_void_p, c_void_p],
    "po_warp_composite_multi": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int,
                                c_int, c_int, c_void_p, c_void_p],
    "po_warp_fwd": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int,
                    c_int, c_void_p, c_void_p],
    "po_warp_bwd": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int,
                    c_int, c_void_p, c_void_p, c_void_p],
    "po_warp_fwd_keyed": [c_void_p, c_void_p, ctypes.c_uint64, ctypes.c_uint64, c_int, c_void_p, c_void_p, c_void_p,
                          c_int, c_int, c_int, c_int, c_void_p, c_void_p],
    "po_augment_patch": [c_void_p, ctypes.c_uint64, ctypes.c_uint64, c_int, c_void_p, c_void_p, c_int, c_int, c_void_p,
                         c_void_p],
    "po_warp_fwd_pre": [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p],
    "po_warp_bwd_pre": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p,
                        c_void_p, c_void_p],
    "po_warp_box_fwd_keyed": [c_void_p, c_void_p, ctypes.c_uint64, ctypes.c_uint64, c_int, c_void_p, c_void_p,
                              c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p],
    "po_warp_box_bwd_keyed": [c_void_p, c_void_p, ctypes.c_uint64, ctypes.c_uint64, c_int, c_void_p, c_void_p,
                              c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p],
    "po_warp_box_fwd_fac": [c_void_p, c_void_p, ctypes.c_uint64, ctypes.c_uint64, c_int, c_void_p, c_void_p,
                            c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p],
    "po_warp_box_bwd_fac": [c_void_p, c_void_p, ctypes.c_uint64, ctypes.c_uint64, c_int, c_void_p, c_void_p,
                            c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p],
    "po_warp_bwd_keyed": [c_void_p, c_void_p, ctypes.c_uint64, ctypes.c_uint64, c_int, c_void_p, c_void_p, c_void_p,
                          c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p],
    "po_apply_fwd": [c_void_p, c_void_p, c_int64, c_void_p, c_void_p],
    "po_apply_bwd": [c_void_p, c_void_p, c_int64, c_void_p, c_void_p, c_void_p],
    "po_regularisers": [c_void_p, c_int, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                        c_void_p],
    "po_regularisers_grad": [c_void_p, c_int, c_void_p, c_int, c_void_p, c_void_p, c_int, c_void_p, c_void_p],
    "po_cell_loss": [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_int,
                     c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                     c_void_p],
    "po_cell_windows": [c_void_p, c_int, c_int, c_int, c_void_p, c_int, c_void_p, c_int, c_void_p, c_void_p,
                        c_void_p, c_void_p],
    "po_support_boxes": [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p],
    "po_grad_boxes": [c_void_p, c_int, c_int, c_void_p, c_int, c_int, c_void_p, c_void_p],
    "po_max_prob": [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p,
                    c_void_p],
    "po_max_prob_bwd": [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p,
                        c_void_p, c_void_p, c_void_p],
    "po_conv": [ctypes.POINTER(po_conv_desc), c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                c_void_p, c_void_p, c_void_p, c_void_p, c_void_p],
    "po_conv_tile_info": [c_int, ctypes.POINTER(c_int), ctypes.POINTER(c_int), ctypes.POINTER(c_int),
                          ctypes.POINTER(c_int)],
    "po_conv_first_fwd": [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_int, c_int,
                          c_int, c_void_p, c_void_p, c_void_p],
    "po_conv_first_pool_fwd": [c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p,
                               c_void_p, c_void_p, c_void_p],
    "po_conv_first_fwd_cmp": [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_int,
                              c_int, c_int, c_void_p, c_void_p, c_void_p],
    "po_conv_first_pool_fwd_cmp": [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_int, c_int,
                                   c_int, c_void_p, c_void_p, c_void_p, c_void_p],
    "po_conv_first_pool_wino_fwd": [c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_int, c_int, c_int,
                                    c_void_p, c_void_p, c_void_p, c_void_p],
    "po_conv_first_pool_wino_fwd_cmp": [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_int,
                                        c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p],
    "po_conv_first_dgrad": [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_int, c_int, c_void_p,
                            c_void_p, c_void_p],
    "po_slice_accum": [c_void_p, c_int, c_int, c_void_p, c_int, c_int, c_int64, c_int, c_int,
                       c_void_p, c_int, c_void_p, c_void_p],
    "po_view_move": [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_int, c_int, c_int, c_int,
                     c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_int, c_void_p, c_void_p],
    "po_upsample2_fwd": [c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p, c_int, c_int, c_void_p,
                         c_void_p],
    "po_upsample2_bwd": [c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p, c_int, c_int,
                         c_void_p, c_int, c_void_p, c_void_p],
    "po_maxpool2_fwd": [c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p,
                        c_void_p, c_void_p],
    "po_maxpool2_bwd": [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p, c_int,
                        c_void_p, c_void_p, c_void_p],
    "po_maxpool2_bwd_box": [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p, c_int,
                            c_void_p, c_void_p, c_void_p, c_void_p],
    "po_nhwc_to_nchw": [c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p],
    "po_nchw_to_nhwc": [c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p],
}

_lib = None
_checked_devices = set()


def load():
    """Load the shared object and declare every entry point of advpatch.h."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError("libadvpatch_hip.so is not built (%s); run `python -c 'import "
                          "__graft_entry__ as g; g.build()'` or `make -C csrc`" % LIB_PATH)
    lib = ctypes.CDLL(LIB_PATH)
    lib.po_abi_version.argtypes = []
    lib.po_abi_version.restype = c_int
    got = lib.po_abi_version()
    if got != PO_ABI_VERSION:
        raise ImportError("libadvpatch_hip.so has ABI %d, this package needs %d: rebuild it "
                          "(make -C csrc, or __graft_entry__.build())" % (got, PO_ABI_VERSION))
    for name, argtypes in _SIGS.items():
        fn = getattr(lib, name)
        fn.argtypes = argtypes
        fn.restype = c_int
    lib.po_last_error.argtypes = []
    lib.po_last_error.restype = ctypes.c_char_p
    _lib = lib
    return lib


def symbols():
    return sorted(list(_SIGS) + ["po_last_error"])


def last_error():
    return load().po_last_error().decode(errors="replace")


# Per-entry HIP-event timing for bench.py's roofline pass: {entry name: [(e0, e1), ...]}
# (events recorded on the current torch stream, the stream every entry is launched on), or None.
TIMERS = None


def call(name, *args):
    timers = TIMERS
    if timers is not None and name in timers:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        rc = getattr(load(), name)(*args)
        e1.record()
        timers[name].append((e0, e1))
    else:
        rc = getattr(load(), name)(*args)
    if rc != 0:
        raise RuntimeError("%s failed (%d): %s" % (name, rc, last_error()))


def stream():
    return c_void_p(torch.cuda.current_stream().cuda_stream)


def ensure_device(t):
    """The HIP path runs on gfx950 CUDA tensors only (fails loudly otherwise)."""
    if not (isinstance(t, torch.Tensor) and t.is_cuda):
        raise RuntimeError("advpatch HIP ops need CUDA (ROCm) tensors; got %s" %
                           (t.device if isinstance(t, torch.Tensor) else type(t)))
    dev = t.device.index if t.device.index is not None else torch.cuda.current_device()
    if dev not in _checked_devices:
        call("po_device_check", dev)
        _checked_devices.add(dev)


def ptr(t, dtype=torch.float32):
    """Device pointer of a contiguous tensor of ``dtype`` (None -> NULL)."""
    if t is None:
        return None
    if t.dtype != dtype:
        raise TypeError("expected %s tensor, got %s" % (dtype, t.dtype))
    if not t.is_contiguous():
        raise ValueError("expected a contiguous tensor")
    return c_void_p(t.data_ptr())


def ptr_array(ts):
    arr = (c_void_p * len(ts))(*[t.data_ptr() if t is not None else None for t in ts])
    return arr
