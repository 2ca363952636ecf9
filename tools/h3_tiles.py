"""Time every po_conv tile of one precision on a set of conv shapes (one process).

    python tools/h3_tiles.py [prec=1] [shape-set=main]
Prints TFLOP/s (fp32-equivalent: 2*M*N*K per launch) per tile index.
"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import __graft_entry__ as ge  # noqa: E402

nat = ge._pkg("_native")
Darknet = ge._pkg("darknet_v3").Darknet
dev = torch.device("cuda", 0)
prec = int(sys.argv[1]) if len(sys.argv) > 1 else 1
SHAPES = [(16, 76, 128, 256, 3, 1), (16, 38, 256, 512, 3, 1), (16, 19, 512, 1024, 3, 1), (16, 152, 64, 128, 3, 1),
          (16, 304, 32, 64, 3, 1), (16, 76, 256, 128, 1, 1), (16, 38, 512, 256, 1, 1), (16, 19, 1024, 512, 1, 1),
          (16, 304, 64, 32, 1, 1), (16, 152, 64, 128, 3, 2)]
tiles = []
for t in range(1, nat.PO_CONV_NTILES + 1):
    v = [ctypes.c_int() for _ in range(4)]
    nat.call("po_conv_tile_info", t, *[ctypes.byref(x) for x in v])
    if v[3].value == prec:
        tiles.append((t, v[0].value, v[1].value, v[2].value))
st = nat.stream()
for (B, H, Cin, Cout, k, s) in SHAPES:
    pad = (k - 1) // 2
    Ho = (H + 2 * pad - k) // s + 1
    x = torch.randn(B, H, H, Cin, device=dev)
    w = torch.randn(Cout, k * k, Cin, device=dev) * 0.05
    b = torch.zeros(Cout, device=dev)
    y = torch.empty(B, Ho, Ho, Cout, device=dev)
    slot = torch.zeros(64, dtype=torch.int32, device=dev)
    slot[0] = torch.tensor([float(x.abs().max())]).view(torch.int32)[0]
    d = nat.po_conv_desc()
    d.B, d.Hin, d.Win, d.Cin_p, d.Hout, d.Wout, d.Cout_p, d.Hg, d.Wg = B, H, H, Cin, Ho, Ho, Cout, Ho, Ho
    d.in_step, d.out_step, d.out_oy, d.out_ox, d.ntaps = s, 1, 0, 0, k * k
    for kh in range(k):
        for kw in range(k):
            d.dh[kh * k + kw] = kh - pad
            d.dw[kh * k + kw] = kw - pad
    d.N, d.act, d.accumulate = Cout, 1, 0
    if prec == 1:
        wt, d.w_shift = Darknet._split16(w)
        d.prec, d.in_amax = 1, slot.data_ptr()
    else:
        wt = w
    args = (ctypes.byref(d), nat.ptr(x), nat.ptr(wt, wt.dtype), nat.ptr(b), nat.ptr(y), None, None, None, None, None)
    fl = 2.0 * B * Ho * Ho * Cout * Cin * k * k
    res = []
    ref = None
    for t, bm, bn, bk in tiles:
        if bn > Cout or Cin % bk:
            continue
        d.tile = t
        if nat.load().po_conv(*args, st) != 0:       # tile not applicable (e.g. halo on a 1x1 / strided conv)
            continue
        for _ in range(2):
            nat.call("po_conv", *args, st)
        torch.cuda.synchronize()
        if ref is None:
            ref = y.clone()
        else:
            err = float((y - ref).abs().max() / ref.abs().max())
            assert err < 1e-5, (t, err)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        it = 20
        e0.record()
        for _ in range(it):
            nat.call("po_conv", *args, st)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / it
        res.append("%d(%dx%dx%d):%.0f" % (t, bm, bn, bk, fl / ms / 1e9))
    print("B%d H%d %d->%d k%d s%d  " % (B, H, Cin, Cout, k, s) + " ".join(res), flush=True)
