"""TEST INFRASTRUCTURE — numpy restatement of po_draws (csrc/draw_ops.hip).

The reference draws its augmentation randomness from unseeded CUDA/CPU RNGs
(load_data.py:548-574 contrast/brightness/noise, 607-614 angle, 693-707
target_x/y), so there is no reference stream to reproduce; the build replaces
it with a counter-based generator whose variates depend only on (seed, step,
global image index, element).  This module restates that generator on the CPU
so tests can check the HIP kernel bit-exactly, and can check the property the
data-parallel trainer relies on: the draws of images [b0, b0+B) do not depend
on how the global batch is split over ranks.

Philox4x32-10 (Salmon, Moraes, Dror, Shaw: "Parallel random numbers: as easy as
1, 2, 3", SC'11; constants and round function as published with Random123).
Only tests/ and __graft_entry__.smoke() import this.
"""
import math

import numpy as np

M0, M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
W0, W1 = 0x9E3779B9, 0xBB67AE85
MASK = np.uint64(0xFFFFFFFF)


def philox4x32_10(c0, c1, c2, c3, k0, k1):
    """Vectorised Philox4x32-10: counters c0..c3 (uint32 arrays or scalars),
    key (k0, k1) -> four uint32 arrays."""
    c = [np.asarray(x, dtype=np.uint64) & MASK for x in (c0, c1, c2, c3)]
    k0, k1 = int(k0) & 0xFFFFFFFF, int(k1) & 0xFFFFFFFF
    for _ in range(10):
        p0 = M0 * c[0]
        p1 = M1 * c[2]
        hi0, lo0 = p0 >> np.uint64(32), p0 & MASK
        hi1, lo1 = p1 >> np.uint64(32), p1 & MASK
        c = [hi1 ^ c[1] ^ np.uint64(k0), lo1, hi0 ^ c[3] ^ np.uint64(k1), lo0]
        k0 = (k0 + W0) & 0xFFFFFFFF
        k1 = (k1 + W1) & 0xFFFFFFFF
    return [x.astype(np.uint32) for x in c]


def _unif(x):
    return (x >> np.uint32(8)).astype(np.float32) * np.float32(2.0 ** -24)


def _affine(u, span, frm):
    # po_draws: float64(u) * float64(fp32 span) is exact; + float64(fp32 from)
    # rounds once in float64, then to fp32
    return (u.astype(np.float64) * np.float64(np.float32(span)) + np.float64(np.float32(frm))).astype(np.float32)


def draws(seed, counter, b0, B, P):
    """The po_draws outputs (numpy float32) for images b0 .. b0+B-1."""
    k0, k1 = seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF
    c2, c3 = counter & 0xFFFFFFFF, (counter >> 32) & 0xFFFFFFFF
    n = 3 * P * P
    ng = (n + 3) // 4
    gb = np.arange(b0, b0 + B, dtype=np.uint64)
    g = np.arange(ng, dtype=np.uint64)
    G, GB = np.meshgrid(g, gb)                                # [B, ng]
    r = philox4x32_10(G, GB, c2, c3, k0, k1)
    noise = np.stack([_affine(_unif(x), 2.0, -1.0) for x in r], axis=-1).reshape(B, 4 * ng)[:, :n]
    s = philox4x32_10(np.uint64(0xFFFFFFFF), gb, c2, c3, k0, k1)
    t = philox4x32_10(np.uint64(0xFFFFFFFE), gb, c2, c3, k0, k1)
    pi = np.float32(math.pi)
    return {
        "contrast": _affine(_unif(s[0]), 0.4, 0.8),
        "bright": _affine(_unif(s[1]), 0.2, -0.1),
        "noise": noise.reshape(B, 3, P, P).astype(np.float32),
        "angle": _affine(_unif(s[2]), np.float32(2.0) * pi, -pi),
        "ux": _unif(s[3]),
        "uy": _unif(t[0]),
    }
