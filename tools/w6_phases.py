"""Phase timing of tile 71 / 72 (W6_TILE; conv_wino6_k) from a diagnostic build with
per-workgroup s_memtime sums (-DPO_W6_STAMP):
    OUT=tools/abl_push bash tools/build_ablate.sh w6stamp -DPO_W6_STAMP
    MICRO_LIB=tools/abl_push/libadvpatch_w6stamp.so python tools/w6_phases.py B H Cin Cout [ksplit]
Prints, per unit, the mean shader cycles of the k-loop (unit top through all
but the last k-step), the peeled last step and the epilogue, and the launch span."""
import ctypes
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
import __graft_entry__ as ge

nat = ge._pkg("_native")
nat.LIB_PATH = os.environ["MICRO_LIB"]
dk = ge._pkg("darknet_v3")
B, H, Cin, Cout = (int(x) for x in sys.argv[1:5])
ks = int(sys.argv[5]) if len(sys.argv) > 5 else 1
dev = torch.device("cuda", 0)
x = torch.randn(B, H, H, Cin, device=dev)
w = torch.randn(Cout, 9, Cin, device=dev) * 0.05
b = torch.zeros(Cout, device=dev)
y = torch.empty(B, H, H, Cout, device=dev)
res = torch.randn(B, H, H, Cout, device=dev)
sm = torch.empty_like(res)
bits = torch.empty(B * H * H * (Cout // 32), dtype=torch.int32, device=dev)
d = nat.po_conv_desc()
d.B, d.Hin, d.Win, d.Cin_p, d.Hout, d.Wout, d.Cout_p, d.Hg, d.Wg = B, H, H, Cin, H, H, Cout, H, H
d.in_step, d.out_step, d.out_oy, d.out_ox, d.ntaps = 1, 1, 0, 0, 9
for t in range(9):
    d.dh[t], d.dw[t] = t // 3 - 1, t % 3 - 1
d.N, d.act, d.accumulate, d.tile = Cout, 1, 0, int(os.environ.get("W6_TILE", "71"))
offs = [(d.dh[t], d.dw[t]) for t in range(9)]
U6 = dk.wino6_transform(w, offs)
d.Wwino6 = U6.data_ptr()
if d.tile == 72:                                 # the pre-transformed input's workspace
    nv = dk.NetPlan.winov_floats(d)
    winov = torch.empty(nv, device=dev)
    d.winov, d.winov_floats = winov.data_ptr(), nv
mode = os.environ.get("W6_MODE", "resy")       # resy: y + sum + bits; res: sum + bits (the plan's); y: y only
if mode != "y":
    d.ybits = bits.data_ptr()
ws = None
if ks > 1:
    ws = torch.empty(ks * B * H * H * Cout, device=dev)
    d.ksplit, d.workspace = ks, ws.data_ptr()
args = (ctypes.byref(d), nat.ptr(x), nat.ptr(w), nat.ptr(b), None if mode == "res" else nat.ptr(y),
        None if mode == "y" else nat.ptr(res), None if mode == "y" else nat.ptr(sm), None, None, None)
st = nat.stream()
for _ in range(5):
    nat.call("po_conv", *args, st)
torch.cuda.synchronize()
n = 256
buf = np.zeros((n, 8), dtype=np.uint64)
lib = ctypes.CDLL(nat.LIB_PATH)
assert lib.po_debug_w6_stamps(buf.ctypes.data_as(ctypes.c_void_p), n) == 0
live = buf[:, 3] > 0
u = buf[live, 3].astype(np.float64)
ph = buf[live, :3].astype(np.float64)
span = (buf[live, 5].max() - buf[live, 4].min()) / 100.0
tot = ph.sum(1)
print("[%s] B=%d H=%d %d->%d ks=%d: %d workgroups, %.2f units each, span %.1f us (%.0f cycles/us by memtime/realtime)" % (
    mode, B, H, Cin, Cout, ks, int(live.sum()), u.mean(), span, tot.mean() / span))
for i, name in enumerate(("k-loop (unit top .. step K-2)", "last k-step", "epilogue (4 passes)")):
    print("  %-32s %8.0f cycles/unit  (%.1f %%)" % (name, (ph[:, i] / u).mean(), 100 * ph[:, i].sum() / ph.sum()))
kst = Cin // 16 // ks
mfma = 72 * kst
print("  per k-step (k-loop / (K-1)): %.0f cycles; MFMA floor per wave pair %d cycles" % (
    (ph[:, 0] / u).mean() / max(kst - 1, 1), 2 * 72 * 64))
