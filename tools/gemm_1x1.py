"""1x1-conv GEMM shapes of the yolov3 B=16 step: library fp32 GEMM
(torch.matmul -> hipBLASLt) beside po_conv's direct tiles (k=1 launches).
usage: python tools/gemm_1x1.py"""
import os
import sys
import subprocess
import torch
torch.backends.cuda.matmul.allow_tf32 = False
dev = torch.device("cuda", 0)
SHAPES = [(16, 304, 64, 32), (16, 152, 128, 64), (16, 152, 64, 128), (16, 76, 256, 128), (16, 76, 128, 256),
          (16, 38, 512, 256), (16, 38, 256, 512), (16, 19, 1024, 512), (16, 19, 512, 1024)]
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for B, H, K, N in SHAPES:
    M = B * H * H
    a = torch.randn(M, K, device=dev)
    w = torch.randn(N, K, device=dev)
    for _ in range(3):
        c = a @ w.t()
    torch.cuda.synchronize()
    e0.record()
    for _ in range(20):
        c = a @ w.t()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 20
    print("hipblaslt %3d^2 %4d->%4d  M=%d: %.1f us  %.1f TFLOP/s" % (H, K, N, M, ms * 1e3, 2.0 * M * N * K / ms / 1e9),
          flush=True)
    for t in os.environ.get("TILES", "3 5 9 13 14 17 18").split():
        out = subprocess.run([sys.executable, "tools/conv_micro.py", str(B), str(H), str(K), str(N), "1", "1", "20"],
                             env=dict(os.environ, MICRO_TILE=t), capture_output=True, text=True, timeout=60)
        line = [l for l in out.stdout.splitlines() if "TFLOP" in l]
        print("   tile %2s %s" % (t, line[-1].split(":")[-1] if line else out.stderr.strip()[-80:]), flush=True)
