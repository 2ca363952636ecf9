"""Diagnostic: tile 71 (F(4x4,3x3)) against float64 on small shapes; prints
where the error sits (per output row / column / channel group)."""
import ctypes, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import torch
import torch.nn.functional as F
import __graft_entry__ as ge
nat = ge._pkg("_native")
dk = ge._pkg("darknet_v3")
from test_gpu_wino import _desc, _setup
DEV = torch.device("cuda", 0)
for (B, H, Cin, Cout, flip) in [(1, 8, 32, 64, False), (2, 7, 32, 64, False), (3, 7, 96, 128, False)]:
    x, w, bias, wd, U = _setup(B, H, Cin, Cout, flip, seed=1)
    s = -1 if flip else 1
    offs = [(s * (kh - 1), s * (kw - 1)) for kh in range(3) for kw in range(3)]
    U6 = dk.wino6_transform(wd, offs)
    ref = F.conv2d(x.double(), w.double(), bias.double(), padding=1)
    xd = x.permute(0, 2, 3, 1).contiguous().to(DEV)
    y = torch.full((B, H, H, Cout), float("nan"), device=DEV)
    d = _desc(nat, B, H, Cin, Cout, 71, flip)
    d.Wwino, d.Wwino6 = U.data_ptr(), U6.data_ptr()
    nat.call("po_conv", ctypes.byref(d), nat.ptr(xd), nat.ptr(wd), nat.ptr(bias.to(DEV)), nat.ptr(y), None, None,
             None, None, None, nat.stream())
    torch.cuda.synchronize()
    out = y.permute(0, 3, 1, 2).cpu().double()
    err = (out - ref).abs() / ref.abs().max()
    print("B=%d H=%d Cin=%d Cout=%d: max rel %.3g, nan %d" % (B, H, Cin, Cout, float(err.nan_to_num(9).max()),
                                                           int(torch.isnan(out).sum())))
    print("  per image", [round(float(err[b].nan_to_num(9).max()), 4) for b in range(B)])
    print("  per row  ", [round(float(err[:, :, i].nan_to_num(9).max()), 4) for i in range(H)])
    print("  per col  ", [round(float(err[:, :, :, j].nan_to_num(9).max()), 4) for j in range(H)])
    print("  per 16 ch", [round(float(err[:, c:c + 16].nan_to_num(9).max()), 4) for c in range(0, Cout, 16)])
    print("  ref[0,0,:4,:4]", ref[0, 0, :4, :4].numpy().round(3).tolist())
    print("  out[0,0,:4,:4]", out[0, 0, :4, :4].numpy().round(3).tolist())
