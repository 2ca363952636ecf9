"""Micro-benchmark of yolov3-tiny's conv 16 -> 32 + 2x2 max pool launch (B=256,
208^2, leaky) on po_conv tiles 69 (direct halo), 61 (generic F(2x2)) and 73
(conv_wpool_k), HIP events over repeated launches; checksum of the pooled map.
Usage: python tools/wpool_micro.py [B] [H] [iters]"""
import ctypes
import hashlib
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from test_gpu_wino import _desc, _setup   # noqa: E402
from conftest import pkg_mod              # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
H = int(sys.argv[2]) if len(sys.argv) > 2 else 208
IT = int(sys.argv[3]) if len(sys.argv) > 3 else 20
DEV = torch.device("cuda", 0)
nat = pkg_mod("_native")
x, w, bias, wd, U = _setup(B, H, 16, 32, False, seed=5)
xd = x.permute(0, 2, 3, 1).contiguous().to(DEV)
bd = bias.to(DEV)
h = H // 2
py = torch.empty(B, h, h, 32, device=DEV)
pam = torch.empty(B, h, h, 32, dtype=torch.int8, device=DEV)
for tile in (69, 61, 73, 69, 73):
    d = _desc(nat, B, H, 16, 32, tile)
    d.Wwino, d.act = U.data_ptr(), 1
    d.pool_y, d.pool_argmax = py.data_ptr(), pam.data_ptr()
    args = (ctypes.byref(d), nat.ptr(xd), nat.ptr(wd), nat.ptr(bd), None, None, None, None, None, None, nat.stream())
    nat.call("po_conv", *args)
    torch.cuda.synchronize()
    hsh = hashlib.sha1(py.cpu().numpy().tobytes()).hexdigest()[:12]
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(IT):
        nat.call("po_conv", *args)
    e1.record()
    e1.synchronize()
    us = e0.elapsed_time(e1) * 1000 / IT
    print("tile %d B=%d H=%d: %8.1f us  %6.1f TFLOP/s direct-equivalent  pooled %s" % (
        tile, B, H, us, 2 * B * H * H * 32 * 144 / us / 1e6, hsh))
