"""Calibration: library fp32 GEMM throughput (torch.matmul -> hipBLASLt/rocBLAS)
on square and conv-shaped problems, next to the po_conv roofline."""
import torch
torch.backends.cuda.matmul.allow_tf32 = False
dev = torch.device("cuda", 0)
for (M, N, K) in [(8192, 8192, 8192), (92416, 256, 1152), (23104, 512, 2304), (5776, 1024, 4608), (369664, 128, 576)]:
    a = torch.randn(M, K, device=dev)
    b = torch.randn(K, N, device=dev)
    for _ in range(3):
        c = a @ b
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n = 10
    e0.record()
    for _ in range(n):
        c = a @ b
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / n
    print("matmul fp32 M=%d N=%d K=%d: %.1f us  %.1f TFLOP/s" % (M, N, K, ms * 1e3, 2.0 * M * N * K / ms / 1e9))
