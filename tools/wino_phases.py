"""Phase timing of the Winograd tile-67/68 kernel (conv_wino4_k) from a
diagnostic build with per-workgroup s_memrealtime stamps (-DPO_WINO_STAMP):
    bash tools/build_ablate.sh stamp -DPO_WINO_STAMP
    MICRO_LIB=tools/abl/libadvpatch_stamp.so python tools/wino_phases.py B H Cin Cout [tile]
Prints the mean workgroup prologue (start -> k-loop entry), k-loop and
epilogue durations, the launch span and how many workgroups ran at once."""
import ctypes
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
import __graft_entry__ as ge

nat = ge._pkg("_native")
nat.LIB_PATH = os.environ["MICRO_LIB"]
B, H, Cin, Cout = (int(x) for x in sys.argv[1:5])
tile = int(sys.argv[5]) if len(sys.argv) > 5 else 68
dev = torch.device("cuda", 0)
x = torch.randn(B, H, H, Cin, device=dev)
w = torch.randn(Cout, 9, Cin, device=dev) * 0.05
b = torch.zeros(Cout, device=dev)
y = torch.empty(B, H, H, Cout, device=dev)
d = nat.po_conv_desc()
d.B, d.Hin, d.Win, d.Cin_p, d.Hout, d.Wout, d.Cout_p, d.Hg, d.Wg = B, H, H, Cin, H, H, Cout, H, H
d.in_step, d.out_step, d.out_oy, d.out_ox, d.ntaps = 1, 1, 0, 0, 9
for t in range(9):
    d.dh[t], d.dw[t] = t // 3 - 1, t % 3 - 1
d.N, d.act, d.accumulate, d.tile = Cout, 1, 0, tile
U = ge._pkg("darknet_v3").wino_transform(w, [(d.dh[t], d.dw[t]) for t in range(9)])
d.Wwino = U.data_ptr()
args = (ctypes.byref(d), nat.ptr(x), nat.ptr(w), nat.ptr(b), nat.ptr(y), None, None, None, None, None)
st = nat.stream()
for _ in range(5):
    nat.call("po_conv", *args, st)
torch.cuda.synchronize()
Ht = (H + 1) // 2
nwg = -(-(B * Ht * Ht) // 64) * (Cout // 64)
buf = np.zeros((nwg, 16), dtype=np.uint64)
lib = ctypes.CDLL(nat.LIB_PATH)
assert lib.po_debug_wino_stamps(buf.ctypes.data_as(ctypes.c_void_p), nwg) == 0
cyc = buf[:, 10:12].astype(np.float64)
sub = (buf[:, :10].astype(np.float64) - buf[:, :1].astype(np.float64)) / 100.0
buf = buf[:, [0, 1, 2, 9]]
t = (buf.astype(np.float64) - float(buf[:, 0].min())) / 100.0      # 100 MHz -> us
pro, kl, epi = t[:, 1] - t[:, 0], t[:, 2] - t[:, 1], t[:, 3] - t[:, 2]
span = t[:, 3].max()
grid = np.linspace(0, span, 200)
conc = [int(((t[:, 0] <= g) & (t[:, 3] > g)).sum()) for g in grid]
print("B=%d H=%d %d->%d tile %d: %d workgroups, %d k-steps, span %.1f us" % (B, H, Cin, Cout, tile, nwg, Cin // 16, span))
print("  per workgroup: prologue %.2f us, k-loop %.2f us (%.3f us/k-step), epilogue %.2f us, total %.2f us" % (
    pro.mean(), kl.mean(), kl.mean() / (Cin // 16), epi.mean(), (t[:, 3] - t[:, 0]).mean()))
print("  p10/p90 total %.2f / %.2f us; concurrent workgroups mean %.0f max %d; last start %.1f us" % (
    np.percentile(t[:, 3] - t[:, 0], 10), np.percentile(t[:, 3] - t[:, 0], 90), np.mean(conc), max(conc),
    t[:, 0].max()))
ghz = (cyc[:, 1] - cyc[:, 0]) / (t[:, 2] - t[:, 1]) / 1e3
print("  shader clock in the k-loop %.2f GHz (p10 %.2f, p90 %.2f): %.0f cycles per k-step per SIMD (MFMA floor 8192)" % (
    np.median(ghz), np.percentile(ghz, 10), np.percentile(ghz, 90), np.median(ghz) * 1e3 * kl.mean() / (Cin // 16)))
names = ["loop exit", "p0 loads+sync", "p0 LDS dump+sync", "p0 inverse", "p1 sync", "p1 LDS dump+sync", "p1 inverse",
         "stores+end"]
d = np.diff(sub[:, 2:10], axis=1).mean(axis=0)
print("  epilogue steps (us): " + ", ".join("%s %.2f" % (n, v) for n, v in zip(names[1:], d)))
