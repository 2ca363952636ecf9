"""Time the first layer (po_conv_first_fwd / po_conv_first_pool_fwd / _wino_fwd) on the
bench shapes: yolov3 B=16 @608 3->32 and yolov3-tiny B=256 @416 3->16 + pool.
usage: [MICRO_LIB=...] [FIRST_ONLY=False|True|wino] python tools/first_micro.py [iters]
Seeded inputs; each line ends with a hash of the outputs (pooled values and argmax bytes), so
two libraries' lines compare bit for bit."""
import hashlib
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import __graft_entry__ as ge
nat = ge._pkg("_native")
if os.environ.get("MICRO_LIB"):
    nat.LIB_PATH = os.environ["MICRO_LIB"]
iters = int(sys.argv[1]) if len(sys.argv) > 1 else 20
dev = torch.device("cuda", 0)
torch.manual_seed(0)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
first_wino_u = ge._pkg("darknet_v3").first_wino_u
for B, S, co, pool in ((16, 608, 32, False), (256, 416, 16, True), (256, 416, 16, "wino")):
    img = torch.rand(B, 3, S, S, device=dev)
    w = torch.randn(co, 27, device=dev) * 0.2
    b = torch.randn(co, device=dev) * 0.1
    if os.environ.get("FIRST_ONLY") and os.environ["FIRST_ONLY"] != str(pool):
        continue
    if pool:
        y = torch.empty(B, S // 2, S // 2, co, device=dev)
        am = torch.empty(B, S // 2, S // 2, co, dtype=torch.int8, device=dev)
        name, wt = "po_conv_first_pool_fwd", w
        if pool == "wino":
            name, wt = "po_conv_first_pool_wino_fwd", first_wino_u(w.double().cpu().view(co, 3, 3, 3)).float().to(dev)
        call = lambda: nat.call(name, nat.ptr(img), B, S, S, nat.ptr(wt), nat.ptr(b), co, co, 1,
                                nat.ptr(y), nat.c_void_p(am.data_ptr()), None, nat.stream())
        byts = img.numel() * 4 + y.numel() * 5
    else:
        y = torch.empty(B, S, S, co, device=dev)
        call = lambda: nat.call("po_conv_first_fwd", nat.ptr(img), B, S, S, 1, nat.ptr(w), nat.ptr(b), co, co, 1,
                                nat.ptr(y), None, nat.stream())
        byts = img.numel() * 4 + y.numel() * 4
    for _ in range(3):
        call()
    torch.cuda.synchronize()
    e0.record()
    for _ in range(iters):
        call()
    e1.record()
    torch.cuda.synchronize()
    us = 1000.0 * e0.elapsed_time(e1) / iters
    h = hashlib.sha1(y.cpu().numpy().tobytes())
    if pool:
        h.update(am.cpu().numpy().tobytes())
    print("B=%d S=%d 3->%d%s: %.1f us  %.2f TB/s  out %s" % (B, S, co, {False: "", True: " + pool"}.get(pool, " + pool (F(2x2))"),
                                                      us, byts / us / 1e6, h.hexdigest()[:12]))
