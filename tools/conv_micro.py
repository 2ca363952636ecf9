"""Microbenchmark of one po_conv launch shape (fwd of a k x k conv).
usage: python tools/conv_micro.py B H Cin Cout k stride [iters]"""
import sys, os, ctypes, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import __graft_entry__ as ge
nat = ge._pkg("_native")
if os.environ.get("MICRO_LIB"):             # ablation builds (tools/bin)
    nat.LIB_PATH = os.environ["MICRO_LIB"]
B, H, Cin, Cout, k, s = (int(x) for x in sys.argv[1:7])
iters = int(sys.argv[7]) if len(sys.argv) > 7 else 50
dev = torch.device("cuda", 0)
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
if os.environ.get("MICRO_PREC", "0") == "1":          # fp16x3 operands
    slot = torch.zeros(64, dtype=torch.int32, device=dev)
    slot[0] = torch.tensor([float(x.abs().max())]).view(torch.int32)[0]
    w, d.w_shift = ge._pkg("darknet_v3").Darknet._split16(w)
    d.prec, d.in_amax = 1, slot.data_ptr()
    wf = ge._pkg("darknet_v3").Darknet.__new__(ge._pkg("darknet_v3").Darknet)
    wf._frag = {}
    d.Wfrag = wf._frag16(w)                             # fragment-ordered copy (tiles 57..60)
d.tile = int(os.environ.get("MICRO_TILE", "0"))
if d.tile in (61, 62, 63, 64, 65, 66, 67, 68, 70, 71, 72):                             # Winograd: transformed weights
    offs = [(d.dh[t], d.dw[t]) for t in range(9)]
    U = ge._pkg("darknet_v3").wino_transform(w, offs)
    d.Wwino = U.data_ptr()
    if d.tile in (71, 72):                                                               # F(4x4,3x3)
        U6 = ge._pkg("darknet_v3").wino6_transform(w, offs)
        d.Wwino6 = U6.data_ptr()
    if d.tile == 72:                                                                     # its transformed input
        nv = ge._pkg("darknet_v3").NetPlan.winov_floats(d)
        winov = torch.empty(nv, device=dev)
        d.winov, d.winov_floats = winov.data_ptr(), nv
ws = None
if int(os.environ.get("MICRO_KSPLIT", "1")) > 1:        # split-K slices + conv_reduce_k
    d.ksplit = int(os.environ["MICRO_KSPLIT"])
    ws = torch.empty(d.ksplit * B * Ho * Ho * Cout, device=dev)
    d.workspace = ws.data_ptr()
res = sm = None
if os.environ.get("MICRO_RES") == "1":                 # fused shortcut epilogue (res + sum_out) and sign bits
    res = torch.randn(B, Ho, Ho, Cout, device=dev)
    sm = torch.empty_like(res)
    bits = torch.empty(B * Ho * Ho * (Cout // 32), dtype=torch.int32, device=dev)
    d.ybits = bits.data_ptr()
yp = y
if os.environ.get("MICRO_POOL") == "1":                # fused 2x2/2 max pool: only the pooled outputs
    pool = torch.empty(B, Ho // 2, Ho // 2, Cout, device=dev)
    pam = torch.empty(B, Ho // 2, Ho // 2, Cout, dtype=torch.int8, device=dev)
    d.pool_y, d.pool_argmax, yp = pool.data_ptr(), pam.data_ptr(), None
box = None
if os.environ.get("MICRO_BOX"):                       # gradient-cone boxes: a centred square of side frac * Ho per image
    f = float(os.environ["MICRO_BOX"])
    a0 = int(Ho * (1 - f) / 2)
    a1 = a0 + int(Ho * f)
    box = torch.tensor([[a0, a0, a1, a1]] * B, dtype=torch.int32, device=dev)
    d.gbox = box.data_ptr()
args = (ctypes.byref(d), nat.ptr(x), nat.ptr(w, w.dtype), nat.ptr(b), nat.ptr(yp), nat.ptr(res), nat.ptr(sm), None,
        None, None)
st = nat.stream()
for _ in range(3):
    nat.call("po_conv", *args, st)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(iters):
    nat.call("po_conv", *args, st)
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / iters
fl = 2.0 * B * Ho * Ho * Cout * Cin * k * k
print("B=%d H=%d Cin=%d Cout=%d k=%d s=%d: %.1f us  %.1f TFLOP/s" % (B, H, Cin, Cout, k, s, ms * 1e3, fl / ms / 1e9))
