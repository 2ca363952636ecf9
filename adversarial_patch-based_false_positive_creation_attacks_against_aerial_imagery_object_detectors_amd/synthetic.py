"""Seeded synthetic inputs of the reference's training shapes.

There is no dataset and no pretrained checkpoint in this environment, so
benches and parity tests run on synthetic data of the DOTA loader's shapes:

* frames  [B,3,S,S] float32 = uint8 U{0..255}/255 (PNG quantisation)   seed 0
* labels  [B,L,5]   rows [cls,x,y,w,h] normalised, padded to L=252 with 1e-6
  (reference load_data.py:968-978); every 8th frame is an empty-label file,
  i.e. one row of ones(5) (load_data.py:918-923)                      seed 1
* patch   [3,P,P]   U[0,1) (train_patch.py:404-406)                    seed 2
* draws   the PatchTransformer random draws (load_data.py:548-707)      seed 3
          (angles on po_draws' lattice, as the trainer draws them)

All generators use numpy's PCG64 so the oracle and the HIP path see the
same bytes.  ``draws_device`` is the on-device generator the training loop
uses (po_draws: counter-based Philox keyed by the global image index).
"""
import math

import numpy as np
import torch

MAX_LAB = 252  # train_patch.py:116


def _rng(seed):
    return np.random.Generator(np.random.PCG64(seed))


def frames(B, S, seed=0):
    g = _rng(seed)
    u8 = g.integers(0, 256, size=(B, 3, S, S), dtype=np.uint8)
    return torch.from_numpy(u8.astype(np.float32) / np.float32(255.0))


def labels(B, L=MAX_LAB, seed=1, n_classes=15):
    g = _rng(seed)
    out = np.full((B, L, 5), 1e-6, dtype=np.float32)
    for b in range(B):
        if b % 8 == 7:
            out[b, 0, :] = 1.0          # empty label file -> np.ones([5])
            continue
        n = int(min(max(g.poisson(9.0), 1), 50))
        out[b, :n, 0] = g.integers(0, n_classes, size=n)
        out[b, :n, 1] = g.uniform(0.05, 0.95, size=n)
        out[b, :n, 2] = g.uniform(0.05, 0.95, size=n)
        out[b, :n, 3] = g.uniform(0.01, 0.20, size=n)
        out[b, :n, 4] = g.uniform(0.01, 0.20, size=n)
    return torch.from_numpy(out)


def patch(P, seed=2):
    return torch.from_numpy(_rng(seed).random((3, P, P), dtype=np.float32))


def draws(B, P, seed=3):
    g = _rng(seed)
    f32 = np.float32
    return {
        "contrast": torch.from_numpy(g.uniform(0.8, 1.2, B).astype(f32)),
        "bright": torch.from_numpy(g.uniform(-0.1, 0.1, B).astype(f32)),
        "noise": torch.from_numpy(g.uniform(-1.0, 1.0, (B, 3, P, P)).astype(f32)),
        "angle": torch.from_numpy(lattice_angle(np.floor(g.random(B) * 2.0 ** 24))),
        "ux": torch.from_numpy(g.random(B, dtype=f32)),
        "uy": torch.from_numpy(g.random(B, dtype=f32)),
    }


def lattice_angle(k):
    """U(-pi, pi) on po_draws' lattice (csrc/draw_ops.hip): fp32(k 2^-24 *
    fp32(2 pi) - pi) for integer k in [0, 2^24) -- the only angles the
    trainer draws (load_data.sincos_lattice_table tabulates their sin/cos)."""
    pi = np.float32(math.pi)
    u = (np.asarray(k, dtype=np.float64).astype(np.float32) * np.float32(2.0 ** -24)).astype(np.float64)
    return (u * np.float64(np.float32(2.0) * pi) + np.float64(-pi)).astype(np.float32)


DRAW_KEYS = ("contrast", "bright", "noise", "angle", "ux", "uy")


def draws_device(seed, counter, b0, B, P, device, keys=DRAW_KEYS):
    """On-device counter-based draws (po_draws, csrc/draw_ops.hip) for images
    b0 .. b0+B-1 of a global batch at step ``counter``: the rows do not depend
    on how the global batch is split over ranks.  ``keys``: the outputs to
    make (the others are not drawn)."""
    from . import _native as nat
    dev = torch.device(device)
    f = lambda *shape: torch.empty(*shape, device=dev)
    shapes = {"noise": (B, 3, P, P)}
    d = {k: f(*shapes.get(k, (B,))) for k in keys}
    nat.call("po_draws", int(seed) & 0xFFFFFFFFFFFFFFFF, int(counter) & 0xFFFFFFFFFFFFFFFF, int(b0), int(B), int(P),
             *(nat.ptr(d.get(k)) for k in DRAW_KEYS), nat.stream())
    return d


def frames_slice(b0, B, S, seed=0):
    """Images b0 .. b0+B-1 of a seeded global batch of frames, one PCG64
    stream per image (a rank generates only its shard)."""
    out = np.empty((B, 3, S, S), dtype=np.float32)
    for i in range(B):
        g = np.random.Generator(np.random.PCG64([seed, b0 + i]))
        out[i] = g.integers(0, 256, size=(3, S, S), dtype=np.uint8).astype(np.float32) / np.float32(255.0)
    return torch.from_numpy(out)


def labels_slice(b0, B, L=MAX_LAB, seed=1, n_classes=15):
    """Label rows of images b0 .. b0+B-1 of a seeded global batch (one stream
    per image; the empty-label rule keys on the global index)."""
    out = np.full((B, L, 5), 1e-6, dtype=np.float32)
    for i in range(B):
        gi = b0 + i
        if gi % 8 == 7:
            out[i, 0, :] = 1.0
            continue
        g = np.random.Generator(np.random.PCG64([seed, gi]))
        n = int(min(max(g.poisson(9.0), 1), 50))
        out[i, :n, 0] = g.integers(0, n_classes, size=n)
        out[i, :n, 1] = g.uniform(0.05, 0.95, size=n)
        out[i, :n, 2] = g.uniform(0.05, 0.95, size=n)
        out[i, :n, 3] = g.uniform(0.01, 0.20, size=n)
        out[i, :n, 4] = g.uniform(0.01, 0.20, size=n)
    return torch.from_numpy(out)


def shard(t, rank, world):
    """Contiguous equal shard of the global batch."""
    n = t.size(0)
    assert n % world == 0, "global batch %d not divisible by world size %d" % (n, world)
    per = n // world
    return t[rank * per:(rank + 1) * per]


def shard_draws(d, rank, world):
    return {k: shard(v, rank, world) for k, v in d.items()}
