"""Synthetic darknet ``.weights`` files (the pretrained file is absent).

Layout written = layout read by reference ``darknet_v3.py:223-281``:
a header of 5 x int32, then per convolutional block in cfg order
``[bn_bias, bn_weight, bn_mean, bn_var, W]`` (BN) or ``[bias, W]`` with
``W`` in PyTorch ``[Cout, Cin, k, k]`` order, all float32.

Initialisation (seeded PCG64), built so that 75 layers of random weights
neither saturate the sigmoid heads nor zero the patch gradient (SURVEY.md §7
hard part 4):

* convs: W ~ N(0, 2/fan_in); BN gamma ~ U(0.8,1.2), beta ~ U(-0.05,0.05);
* BN running mean/var are *calibrated*: one forward pass over a seeded
  synthetic frame at ``calib_size`` sets each BN's (mean, var) to the batch
  statistics of its conv output, so every BN output is ~N(beta, gamma^2);
* the conv feeding each residual shortcut has gamma x ``residual_gain``;
* linear head convs: W ~ N(0, 1/fan_in) * ``head_gain``, bias 0.

The calibration pass is data generation (torch CPU ops, run once per weights
file, never on the training step).
"""
import os

import numpy as np
import torch
import torch.nn.functional as F

from .cfg import parse_model_config_text
from .cfg_gen import cfg_text

HEADER = np.array([0, 2, 0, 0, 0], dtype=np.int32)


def conv_layout(blocks):
    """[(block_index, cin, cout, k, bn_for_loading)] in cfg order, with the
    channel bookkeeping of darknet_v3.create_modules (darknet_v3.py:32-98).
    ``blocks`` includes the leading [net] block."""
    net = blocks[0]
    filters = [int(net["channels"])]
    out = []
    for i, d in enumerate(blocks[1:]):
        t = d["type"]
        if t == "convolutional":
            f = int(d["filters"])
            out.append((i, filters[-1], f, int(d["size"]), bool(d["batch_normalize"])))
        elif t == "route":
            f = sum(filters[1:][int(l)] for l in d["layers"].split(","))
        elif t == "shortcut":
            f = filters[1:][int(d["from"])]
        else:
            f = filters[-1]
        filters.append(f)
    return out


def synthesize(cfg, seed=4, residual_gain=0.35, head_gain=0.5, calib_size=256):
    """Return the float32 weight stream for ``cfg`` (path or builtin:<name>)."""
    blocks = parse_model_config_text(cfg_text(cfg))
    g = np.random.Generator(np.random.PCG64(seed))
    defs = blocks[1:]
    feeds_shortcut = {i - 1 for i, d in enumerate(defs) if d["type"] == "shortcut"}
    layout = {i: (cin, cout, k, bn) for (i, cin, cout, k, bn) in conv_layout(blocks)}
    params = {}
    for i in sorted(layout):
        cin, cout, k, bn = layout[i]
        fan_in = cin * k * k
        if bn:
            gamma = g.uniform(0.8, 1.2, cout) * (residual_gain if i in feeds_shortcut else 1.0)
            beta = g.uniform(-0.05, 0.05, cout)
            w = g.standard_normal((cout, cin, k, k)) * np.sqrt(2.0 / fan_in)
            params[i] = {"beta": beta, "gamma": gamma, "W": w}
        else:
            w = g.standard_normal((cout, cin, k, k)) * (np.sqrt(1.0 / fan_in) * head_gain)
            params[i] = {"b": np.zeros(cout), "W": w}
    # calibration forward (float64 for stable statistics)
    gi = np.random.Generator(np.random.PCG64(seed + 1))
    x = torch.from_numpy(gi.integers(0, 256, (1, 3, calib_size, calib_size)).astype(np.float64) / 255.0)
    outs = []
    with torch.no_grad():
        for i, d in enumerate(defs):
            t = d["type"]
            if t == "convolutional":
                cin, cout, k, bn = layout[i]
                p = params[i]
                x = F.conv2d(x, torch.from_numpy(p["W"]), None if bn else torch.from_numpy(p["b"]),
                             stride=int(d["stride"]), padding=(k - 1) // 2)
                if bn:
                    mean = x.mean(dim=(0, 2, 3))
                    var = x.var(dim=(0, 2, 3), unbiased=False) + 1e-3
                    p["mean"], p["var"] = mean.numpy(), var.numpy()
                    x = F.batch_norm(x, mean, var, torch.from_numpy(p["gamma"]),
                                     torch.from_numpy(p["beta"]), training=False, eps=1e-5)
                if d["activation"] == "leaky":
                    x = F.leaky_relu(x, 0.1)
            elif t == "maxpool":
                ks, st = int(d["size"]), int(d["stride"])
                if ks == 2 and st == 1:
                    x = F.pad(x, (0, 1, 0, 1))
                x = F.max_pool2d(x, ks, st, padding=(ks - 1) // 2)
            elif t == "upsample":
                x = F.interpolate(x, scale_factor=int(d["stride"]), mode="nearest")
            elif t == "route":
                x = torch.cat([outs[int(l)] for l in d["layers"].split(",")], 1)
            elif t == "shortcut":
                x = outs[-1] + outs[int(d["from"])]
            outs.append(x)
    chunks = []
    for i in sorted(layout):
        p = params[i]
        if layout[i][3]:
            chunks += [p["beta"], p["gamma"], p["mean"], p["var"]]
        else:
            chunks.append(p["b"])
        chunks.append(p["W"].reshape(-1))
    return np.concatenate(chunks).astype(np.float32)


def write_weights(path, stream):
    with open(path, "wb") as f:
        HEADER.tofile(f)
        np.asarray(stream, dtype=np.float32).tofile(f)


def read_weights(path):
    with open(path, "rb") as f:
        header = np.fromfile(f, dtype=np.int32, count=5)
        stream = np.fromfile(f, dtype=np.float32)
    return header, stream


def ensure_synthetic(cfg, path, seed=4):
    """Write the synthetic weights for ``cfg`` to ``path`` unless present."""
    if not os.path.exists(path):
        d = os.path.dirname(os.path.abspath(path))
        os.makedirs(d, exist_ok=True)
        tmp = path + ".tmp%d" % os.getpid()
        write_weights(tmp, synthesize(cfg, seed))
        os.replace(tmp, path)
    return path
