"""Which fp32 operation sequence does this host's F.affine_grid (ATen base grid
@ theta^T through MKL sgemm, K = 3) follow?  Prints, for every evaluation order
of x = bx*t0 + by*t1 + 1*t2 with and without fused multiply-adds, the number of
grid values that differ from torch's (0 = the restatement to use; DESIGN.md §4,
oracle/geometry_ref.py).  CPU only:  python tools/affine_grid_probe.py"""
import itertools
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import geometry_ref as G  # noqa: E402

f32 = np.float32
print("cpu capability", torch.backends.cpu.get_cpu_capability(), "threads", torch.get_num_threads())
try:
    print(open("/proc/cpuinfo").read().split("model name")[1].split("\n")[0])
except Exception:
    pass


def variants(b, t):
    """b = (bx, by, 1) broadcast arrays, t = (t0, t1, t2): every pairing / fma choice."""
    out = {}
    prod = lambda k: (b[k] * t[k]).astype(f32)
    for (i, j, k) in ((0, 1, 2), (0, 2, 1), (1, 2, 0)):
        inners = {
            "fl(p%d)+fl(p%d)" % (i, j): (prod(i) + prod(j)).astype(f32),
            "fma(p%d,fl(p%d))" % (i, j): G.fma32(b[i], t[i], prod(j)),
            "fma(p%d,fl(p%d))" % (j, i): G.fma32(b[j], t[j], prod(i)),
        }
        for name, inner in inners.items():
            out["(%s)+fl(p%d)" % (name, k)] = (inner + prod(k)).astype(f32)
            out["fma(p%d,%s)" % (k, name)] = G.fma32(b[k], t[k], inner)
    return out


torch.manual_seed(0)
tot = {}
for S, B in ((608, 4), (416, 4), (96, 3), (608, 16), (13, 2)):
    th = torch.randn(B, 2, 3) * 3
    g = F.affine_grid(th, (B, 3, S, S), align_corners=False).numpy()
    base = G.base32(S)
    bx = np.broadcast_to(base[None, None, :], (B, S, S)).astype(f32)
    by = np.broadcast_to(base[None, :, None], (B, S, S)).astype(f32)
    one = np.ones((B, S, S), f32)
    for r in range(2):
        t = [np.broadcast_to(th[:, r, k].numpy()[:, None, None], (B, S, S)).astype(f32) for k in range(3)]
        for name, v in variants((bx, by, one), t).items():
            tot[name] = tot.get(name, 0) + int(np.count_nonzero(v != g[..., r]))
for name, n in sorted(tot.items(), key=lambda kv: kv[1]):
    print("%8d  %s" % (n, name))
