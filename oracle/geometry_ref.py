"""TEST INFRASTRUCTURE — the reference's fp32 placement arithmetic written out
as explicit IEEE-754 binary32 operations (numpy).

The reference builds the placement of its patch with PyTorch-CPU ops in fp32
(load_data.py:726-749: theta from sin/cos/scale, ``F.affine_grid`` and
``F.grid_sample``, both with align_corners=False).  Those ops live in the
third-party dependency PyTorch (here 2.10.0+rocm7.0, CPU capability AVX512,
BLAS = MKL 2024.2), not in the reference, so this module restates what they
compute, one rounding at a time, and ``tests/test_geometry_ref.py`` pins the
restatement against the installed torch bit for bit.  The HIP kernels'
reference-geometry form (csrc/warp_geom.h ``ref_*``) is this sequence:

  linspace(-1, 1, S)  ATen RangeFactoriesKernel linspace_kernel: step =
                      2 / (S-1); i < S/2: start + step*i, else end -
                      step*(S-1-i), each contracted to one FMA (GCC -O2 with
                      FMA codegen; measured: no other form matches).
  affine_grid base    AffineGridGenerator.cpp linspace_from_neg_one:
                      range * (S-1) / S (two roundings).
  affine_grid bmm     base_grid [N,H*W,3] @ theta^T through MKL sgemm with
                      K = 3, whose code path MKL picks by CPU: on the MI355X
                      boxes' AMD EPYC 9575F x = fl(fl(fl(bx*t0) + fl(by*t1)) +
                      t2) ("sum", HIP geometry 1); on this build container's
                      Intel AVX-512 Xeon x = fl(fma(by, t1, fl(bx*t0)) + t2)
                      ("fma", geometry 2); tools/affine_grid_probe.py measures
                      every evaluation order on a host.
  grid_sample         GridSamplerKernel.cpp (vectorised CPU kernel),
                      bilinear, zeros padding: ix = fma(g + 1, S/2, -0.5);
                      w = ix - floor(ix), e = 1 - w (same for rows: n, s);
                      weights nw = s*e, ne = s*w, sw = n*e, se = n*w; value =
                      fma(v_se, se, fma(v_sw, sw, fma(v_ne, ne, v_nw*nw))),
                      out-of-image corners reading 0.
  sin, cos, sqrt      torch.sin/cos/sqrt on CPU fp32 tensors run MKL VML
                      (vsSin/vsCos/vsSqrt, HA mode): not correctly rounded
                      (measured: ~5 % of sin/cos values and ~0.5 % of sqrt
                      values differ by one ulp from the rounded exact value).
                      No restatement is possible; see ``sincos_lattice``.

Only tests/ import this module.
"""
import math

import numpy as np

f32 = np.float32
f64 = np.float64


def fma32(a, b, c):
    """Correctly rounded fp32 a*b + c, elementwise (broadcasting): the product
    of two binary32 values is exact in binary64; the binary64 sum is made
    round-to-odd with TwoSum, so the final rounding to binary32 is correct
    (53 >= 24 + 2 bits)."""
    a, b, c = (np.asarray(x, dtype=f32) for x in (a, b, c))
    p = a.astype(f64) * b.astype(f64)
    cc = c.astype(f64)
    s = np.asarray(p + cc, dtype=f64)
    bb = s - p
    err = (p - (s - bb)) + (cc - bb)
    even = (s.view(np.int64) & 1) == 0
    fix = (err != 0) & even & np.isfinite(s)
    if np.any(fix):
        s = np.where(fix, np.nextafter(s, np.where(err > 0, np.inf, -np.inf)), s)
    return s.astype(f32)


def linspace32(S):
    """torch.linspace(-1, 1, S) in fp32 (ATen linspace_kernel, FMA-contracted)."""
    if S == 1:
        return np.array([-1.0], dtype=f32)
    step = f32(f32(2.0) / f32(S - 1))
    i = np.arange(S)
    lo = fma32(step, i.astype(f32), f32(-1.0))
    hi = fma32(-step, (S - 1 - i).astype(f32), f32(1.0))
    return np.where(i < S // 2, lo, hi).astype(f32)


def base32(S):
    """affine_grid's base coordinates, align_corners=False: range*(S-1)/S."""
    if S <= 1:
        return np.zeros(max(S, 1), dtype=f32)
    return ((linspace32(S) * f32(S - 1)).astype(f32) / f32(S)).astype(f32)


def base32_markstein(S):
    """base32 as the HIP kernels form it (warp_geom.h ref_base): the division
    by S replaced by the correctly rounded reciprocal rcp = fl(1/S) and one
    Markstein step, q = fl(x rcp), fl(fma(fma(-q, S, x), rcp, q)).  Equal to
    base32 bit for bit for every S <= 32768 (tests/test_geometry_ref.py)."""
    if S <= 1:
        return np.zeros(max(S, 1), dtype=f32)
    x = (linspace32(S) * f32(S - 1)).astype(f32)
    rcp = f32(f32(1.0) / f32(S))
    q = (x * rcp).astype(f32)
    return fma32(fma32(-q, f32(S), x), rcp, q)


BMM_FORMS = ("sum", "fma")          # HIP geometry 1, 2


def affine_grid32(theta, H, W, form):
    """F.affine_grid(theta [N,2,3] fp32, (N,C,H,W), align_corners=False) ->
    [N,H,W,2] fp32, with the host sgemm's K = 3 order ``form`` ("sum" / "fma")."""
    th = np.asarray(theta, dtype=f32)
    bx = base32(W)[None, None, :]
    by = base32(H)[None, :, None]
    out = []
    for r in range(2):
        t0, t1, t2 = (th[:, r, k][:, None, None] for k in range(3))
        if form == "fma":
            acc = fma32(by, t1, (bx * t0).astype(f32))
        else:
            acc = ((bx * t0).astype(f32) + (by * t1).astype(f32)).astype(f32)
        out.append((acc + t2).astype(f32))
    return np.stack(out, -1)


def host_bmm_form():
    """The form this host's torch follows (None: neither)."""
    import torch
    import torch.nn.functional as F
    th = torch.randn(2, 2, 3, generator=torch.Generator().manual_seed(7)) * 3
    g = F.affine_grid(th, (2, 1, 64, 64), align_corners=False).numpy()
    for form in BMM_FORMS:
        if np.array_equal(affine_grid32(th.numpy(), 64, 64, form), g):
            return form
    return None


def unnormalize32(g, size):
    return fma32((g + f32(1.0)).astype(f32), f32(size) / f32(2.0), f32(-0.5))


def grid_sample32(img, grid):
    """F.grid_sample(img [N,C,H,W], grid [N,Ho,Wo,2], bilinear, zeros,
    align_corners=False) in fp32."""
    img = np.asarray(img, dtype=f32)
    N, C, H, W = img.shape
    ix = unnormalize32(grid[..., 0], W)
    iy = unnormalize32(grid[..., 1], H)
    x0 = np.floor(ix)
    y0 = np.floor(iy)
    w = (ix - x0).astype(f32)
    e = (f32(1.0) - w).astype(f32)
    n = (iy - y0).astype(f32)
    s = (f32(1.0) - n).astype(f32)
    wts = [(s * e).astype(f32), (s * w).astype(f32), (n * e).astype(f32), (n * w).astype(f32)]
    x0 = x0.astype(np.int64)
    y0 = y0.astype(np.int64)
    bi = np.arange(N)[:, None, None]

    def corner(yy, xx):
        ok = (xx >= 0) & (xx < W) & (yy >= 0) & (yy < H)
        v = img[bi, :, np.clip(yy, 0, H - 1), np.clip(xx, 0, W - 1)]      # [N,Ho,Wo,C]
        return np.where(ok[..., None], v, f32(0.0)).astype(f32)

    vals = [corner(y0, x0), corner(y0, x0 + 1), corner(y0 + 1, x0), corner(y0 + 1, x0 + 1)]
    acc = (vals[0] * wts[0][..., None]).astype(f32)
    for k in (1, 2, 3):
        acc = fma32(vals[k], wts[k][..., None], acc)
    return np.moveaxis(acc, -1, 1)


def theta32(sin, cos, scale, tx, ty):
    """load_data.py:738-743, each tensor op one rounding: [B,2,3] fp32."""
    sn, cs, sc, tx, ty = (np.asarray(v, dtype=f32) for v in (sin, cos, scale, tx, ty))
    th = np.zeros(sn.shape + (2, 3), dtype=f32)
    th[..., 0, 0] = cs / sc
    th[..., 0, 1] = sn / sc
    th[..., 0, 2] = ((tx * cs).astype(f32) / sc).astype(f32) + ((ty * sn).astype(f32) / sc).astype(f32)
    th[..., 1, 0] = (-sn) / sc
    th[..., 1, 1] = cs / sc
    th[..., 1, 2] = (((-tx) * sn).astype(f32) / sc).astype(f32) + ((ty * cs).astype(f32) / sc).astype(f32)
    return th


# po_draws' angle lattice (csrc/draw_ops.hip, oracle/draws_ref.py): angle_k =
# fp32(k * 2^-24 * fp32(2*pi_f) + (-pi_f)) for k in [0, 2^24)
LATTICE_N = 1 << 24


def lattice_angles(k=None):
    pi = f32(math.pi)
    span, frm = f64(f32(2.0) * pi), f64(-pi)
    k = np.arange(LATTICE_N, dtype=np.int64) if k is None else np.asarray(k, dtype=np.int64)
    u = (k.astype(f32) * f32(2.0 ** -24)).astype(f64)
    return (u * span + frm).astype(f32)
