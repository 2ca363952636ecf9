"""Data for reproducing this host's torch.sqrt (MKL VML vsSqrt) on fp32:
every float in [1, 4) through torch.sqrt, stored as the signed ulp offset
from the correctly rounded value (int8), plus the host CPU's hardware
rsqrt / rcp approximations over the same inputs (tools/probe/approx).
    python tools/sqrt_probe.py OUTDIR"""
import os
import subprocess
import sys

import numpy as np
import torch

out = sys.argv[1]
os.makedirs(out, exist_ok=True)
bits = np.arange(0x3F800000, 0x3F800000 + (1 << 24), dtype=np.uint32)
x = bits.view(np.float32)
t = torch.sqrt(torch.from_numpy(x)).numpy()
cr = np.sqrt(x.astype(np.float64)).astype(np.float32)
d = (t.view(np.int32).astype(np.int64) - cr.view(np.int32).astype(np.int64))
print("sqrt mismatch %.3f %%, offsets %s" % (100.0 * np.mean(d != 0), np.unique(d, return_counts=True)))
np.savez_compressed(os.path.join(out, "sqrt_offsets.npz"), d=d.astype(np.int8))
# the same for torch.sin / cos over their lattice subsample (context) and scale invariance checks
for sc in (0.25, 4.0, 1024.0, 1.0 / 1024):
    xs = (x[::97] * np.float32(sc)).astype(np.float32)
    ts = torch.sqrt(torch.from_numpy(xs)).numpy()
    ref = (t[::97] * np.float32(np.sqrt(sc))).astype(np.float32)
    print("scale %g: sqrt(x*s) == sqrt(x)*sqrt(s) for %.4f %%" % (sc, 100.0 * np.mean(ts == ref)))
exe = os.path.join(os.path.dirname(os.path.abspath(__file__)), "probe", "approx")
subprocess.check_call([exe, out])
for name in ("rsqrt14", "rsqrt", "rcp14", "rcp"):
    a = np.fromfile(os.path.join(out, name + ".u32"), dtype=np.uint32)
    np.savez_compressed(os.path.join(out, name + ".npz"), a=a)
    os.remove(os.path.join(out, name + ".u32"))
print(sorted(os.listdir(out)))
