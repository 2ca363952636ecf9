"""Time every po_conv tile config on a set of conv shapes (one process)."""
import sys, os, ctypes
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import __graft_entry__ as ge
nat = ge._pkg("_native")
dev = torch.device("cuda", 0)
SHAPES = [(16, 76, 128, 256, 3, 1), (16, 38, 256, 512, 3, 1), (16, 19, 512, 1024, 3, 1), (16, 152, 64, 128, 3, 1),
          (16, 304, 32, 64, 3, 1), (16, 76, 256, 128, 1, 1), (16, 38, 512, 256, 1, 1), (16, 19, 1024, 512, 1, 1),
          (16, 304, 64, 32, 1, 1), (16, 152, 64, 128, 3, 2)]
TILES = ["128x128x16", "128x128x32", "64x128x16", "64x128x32", "128x64x16", "128x64x32", "64x64x16", "64x64x32",
         "128x128x16g", "128x128x32g", "64x128x16g", "64x128x32g", "64x64x16g", "64x64x32g",
         "128x32x16", "128x32x32", "256x128x16", "256x128x16g", "128x256x16", "128x256x16g", "default"]
st = nat.stream()
for (B, H, Cin, Cout, k, s) in SHAPES:
    pad = (k - 1) // 2
    Ho = (H + 2 * pad - k) // s + 1
    x = torch.randn(B, H, H, Cin, device=dev)
    w = torch.randn(Cout, k * k, Cin, device=dev) * 0.05
    b = torch.zeros(Cout, device=dev)
    y = torch.empty(B, Ho, Ho, Cout, device=dev)
    d = nat.po_conv_desc()
    d.B, d.Hin, d.Win, d.Cin_p, d.Hout, d.Wout, d.Cout_p, d.Hg, d.Wg = B, H, H, Cin, Ho, Ho, Cout, Ho, Ho
    d.in_step, d.out_step, d.out_oy, d.out_ox, d.ntaps = s, 1, 0, 0, k * k
    for kh in range(k):
        for kw in range(k):
            d.dh[kh * k + kw] = kh - pad
            d.dw[kh * k + kw] = kw - pad
    d.N, d.act, d.accumulate = Cout, 1, 0
    args = (ctypes.byref(d), nat.ptr(x), nat.ptr(w), nat.ptr(b), nat.ptr(y), None, None, None, None, None)
    fl = 2.0 * B * Ho * Ho * Cout * Cin * k * k
    res = []
    ref = None
    for t in TILES:
        if t == "default":
            os.environ.pop("ADVPATCH_CONV_TILE", None)
        else:
            os.environ["ADVPATCH_CONV_TILE"] = t
        if Cout < int(t.split("x")[1]) if t != "default" else False:
            continue
        for _ in range(2):
            nat.call("po_conv", *args, st)
        torch.cuda.synchronize()
        if ref is None:
            ref = y.clone()
        else:
            err = float((y - ref).abs().max())
            assert err < 1e-3, (t, err)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        it = 20
        e0.record()
        for _ in range(it):
            nat.call("po_conv", *args, st)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / it
        res.append("%s:%.0f" % (t, fl / ms / 1e9))
    print("B%d H%d %d->%d k%d s%d  " % (B, H, Cin, Cout, k, s) + " ".join(res), flush=True)
