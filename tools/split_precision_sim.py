"""CPU estimate of the patch-gradient error of split-bf16 MFMA convolutions.

Runs the oracle's yolov3 step with every conv (forward and dgrad) replaced by
a sum of bf16-piece products, each product evaluated exactly and summed in
fp32 (what a v_mfma_f32_32x32x16_bf16 accumulation does), and reports
max|g - g64| / max|g64| against the float64 step on the same LeakyReLU
branches, next to the plain fp32 oracle's error.

    python tools/split_precision_sim.py [S] [B]
"""
import sys
import types

import torch
import torch.nn.functional as F

sys.path.insert(0, ".")
import oracle  # noqa: E402
from oracle import reference_path as rp  # noqa: E402
import __graft_entry__ as ge  # noqa: E402


def split(x, n, half=False):
    """n bf16 pieces; half=True: n fp16 pieces of x scaled by a power of two
    that puts max|x| just under 2^15 (pieces returned unscaled)."""
    r = x.float()
    sc = 1.0
    if half:
        m = float(r.abs().max())
        sc = 2.0 ** (14 - int(torch.tensor(m).log2().ceil())) if m > 0 else 1.0
        r = r * sc
    parts = []
    for _ in range(n):
        h = (r.half() if half else r.bfloat16()).float()
        parts.append(h / sc)
        r = r - h
    return parts


def pairs(scheme):
    if scheme == "bf16x3":
        return 2, [(0, 0), (0, 1), (1, 0)]
    if scheme == "bf16x4":
        return 2, [(0, 0), (0, 1), (1, 0), (1, 1)]
    if scheme == "fp16x3":
        return 2, [(0, 0), (0, 1), (1, 0)]
    if scheme == "bf16x6":
        return 3, [(i, j) for i in range(3) for j in range(3) if i + j <= 2]
    raise ValueError(scheme)


def make_conv(scheme):
    npart, prs = pairs(scheme)
    half = scheme.startswith("fp16")

    class SplitConv(torch.autograd.Function):
        @staticmethod
        def forward(ctx, x, W, stride, padding):
            ctx.save_for_backward(W)
            ctx.cfg = (stride, padding, x.shape)
            xs, ws = split(x, npart, half), split(W, npart, half)
            y = None
            for i, j in prs:
                t = F.conv2d(xs[i], ws[j], None, stride=stride, padding=padding)
                y = t if y is None else y + t
            return y.to(x.dtype)

        @staticmethod
        def backward(ctx, g):
            (W,) = ctx.saved_tensors
            stride, padding, xshape = ctx.cfg
            gs, ws = split(g, npart, half), split(W, npart, half)
            dx = None
            for i, j in prs:
                t = torch.nn.grad.conv2d_input(xshape, ws[j], gs[i], stride=stride, padding=padding)
                dx = t if dx is None else dx + t
            return dx.to(g.dtype), None, None, None

    def conv2d(x, W, b=None, stride=1, padding=0):
        y = SplitConv.apply(x, W.detach(), stride, padding)
        if b is not None:
            y = y + b.view(1, -1, 1, 1)
        return y

    return conv2d


def main():
    S = int(sys.argv[1]) if len(sys.argv) > 1 else 416
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    torch.set_num_threads(8)
    sy, W, G, ld = ge._pkg("synthetic"), ge._pkg("weights"), ge._pkg("cfg_gen"), ge._pkg("load_data")
    cfg = "builtin:yolov3-dota"
    text = G.cfg_text(cfg).replace("width=608", "width=%d" % S).replace("height=608", "height=%d" % S)
    net = oracle.OracleDarknet(text, W.synthesize(cfg, seed=4))
    colors = ld.load_printability_colors("builtin:30values")
    img, lab = sy.frames(B, S, seed=40), sy.labels(B, seed=41)
    patch, dr = sy.patch(224, seed=42), sy.draws(B, 224, seed=43)
    rec = {}
    r32 = oracle.train_step(patch, img, lab, dr, net, colors, record=rec)
    br = {i: ("leaky", (x.detach() > 0)) for i, x in rec.items()}
    r64 = oracle.train_step_f64(patch, img, lab, dr, net, colors, branch=br)
    r32 = oracle.train_step(patch, img, lab, dr, net, colors, branch=br)
    g64 = r64["grad"]
    scale = g64.abs().max()
    err = lambda g: float((g.double() - g64).abs().max() / scale)
    print("S=%d B=%d fp32 oracle: grad err %.3g, loss %.8f (f64 %.8f)" % (S, B, err(r32["grad"]), float(r32["loss"]),
                                                                      float(r64["loss"])))
    real_F = rp.F
    for scheme in ("bf16x3", "fp16x3", "bf16x6"):
        shim = types.SimpleNamespace(**{k: getattr(real_F, k) for k in dir(real_F) if not k.startswith("__")})
        shim.conv2d = make_conv(scheme)
        rp.F = shim
        try:
            r = oracle.train_step(patch, img, lab, dr, net, colors, branch=br)
        finally:
            rp.F = real_F
        d32 = float((r["grad"] - r32["grad"]).abs().max() / r32["grad"].abs().max())
        print("%s: grad err %.3g (vs fp32 oracle %.3g), loss %.8f, obj max err %.3g, head max err %.3g" % (
            scheme, err(r["grad"]), d32, float(r["loss"]), float((r["obj"].double() - r64["obj"]).abs().max()),
            max(float((h.double() - h64).abs().max() / h64.abs().max()) for h, h64 in zip(r["heads"], r64["heads"]))))


if __name__ == "__main__":
    main()
