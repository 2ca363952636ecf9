"""Per-layer error of the exact-fp32 conv tiles against float64 on the
yolov3-dota layer shapes tile 71 takes (stride-1 3x3 on full maps, forward
and input-gradient orientation, B=2 maps of the 608 network): tile 71
(Winograd F(4x4,3x3)), tile 70 (F(2x2,3x3)) and the direct tile 1, each
against torch float64 conv2d of the same operands (U(-1,1)-scaled He-init
weights, N(0,1) inputs): max-abs error / max|output|.  Markdown to stdout
(DESIGN.md §4).
    python tools/w6_layer_errors.py > profiles/r05/wino_layer_errors.md"""
import ctypes
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import torch
import torch.nn.functional as F
import __graft_entry__ as ge
from test_gpu_wino import _desc, _setup

nat = ge._pkg("_native")
dk = ge._pkg("darknet_v3")
dev = torch.device("cuda", 0)
B = 2
shapes = [(304, 32, 64), (152, 64, 128), (76, 128, 256), (38, 256, 512), (19, 512, 1024)]
print("| layer (B=%d) | orientation | F(4x4) tile 71 | F(2x2) tile 70 | direct tile 1 | 71 / direct |" % B)
print("|---|---|---|---|---|---|")
for H, c1, c2 in shapes:
    for flip in (False, True):
        Cin, Cout = (c2, c1) if flip else (c1, c2)
        x, w, bias, wd, U = _setup(B, H, Cin, Cout, flip, seed=H + Cin)
        s = -1 if flip else 1
        offs = [(s * (kh - 1), s * (kw - 1)) for kh in range(3) for kw in range(3)]
        U6 = dk.wino6_transform(wd, offs)
        ref = F.conv2d(x.double(), w.double(), bias.double(), padding=1)
        xd = x.permute(0, 2, 3, 1).contiguous().to(dev)
        bd = bias.to(dev)
        err = {}
        for tile in (71, 70, 1):
            y = torch.full((B, H, H, Cout), float("nan"), device=dev)
            d = _desc(nat, B, H, Cin, Cout, tile, flip)
            d.Wwino, d.Wwino6 = U.data_ptr(), U6.data_ptr()
            if nat.load().po_conv(ctypes.byref(d), nat.ptr(xd), nat.ptr(wd), nat.ptr(bd), nat.ptr(y), None, None,
                                  None, None, None, nat.stream()) != 0:
                err[tile] = None                  # the tile does not take this launch (N % 64)
                continue
            out = y.permute(0, 3, 1, 2).cpu().double()
            err[tile] = float((out - ref).abs().max() / ref.abs().max())
        f = lambda e: "n/a (N % 64)" if e is None else "%.2e" % e
        print("| %d^2 %d->%d | %s | %s | %s | %s | %s |" % (H, Cin, Cout, "dgrad (flipped taps)" if flip else "forward",
              f(err[71]), f(err[70]), f(err[1]), "-" if err[71] is None else "%.1f" % (err[71] / err[1])), flush=True)
