"""Patch-optimisation images/s on synthetic DOTA-shaped batches (BASELINE.json metric).

One step = one iteration of the reference's batch loop (train_patch.py:164-330):
on-device draws -> median pool -> placement -> fused augment/warp/composite ->
YOLOv3-DOTA forward -> cell loss + NPS/TV/colour -> backward (dgrad) ->
[all-reduce of the patch gradient over RCCL when N > 1] -> Adam(amsgrad) + clamp.
Inputs (frames, labels, patch) are resident in HBM before the timed region.

    python bench.py [--gpus N --steps K --warmup W --batch B --config yolov3|tiny --prec fp32|both|fp16x3]

``value`` is measured with exact fp32 convolutions (v_mfma_f32_32x32x2_f32,
the reference's arithmetic); ``--prec both`` also times the opt-in fp16x3
split-precision path and reports it beside (``value_fp16x3``).
N > 1: one process per GPU (RCCL over xGMI).  ``bench.py --gpus N`` started
without a torchrun environment launches the N ranks itself (torch.distributed.run
as a child process, before anything touches the GPU) — the replacement for the
reference's in-process ``nn.DataParallel`` (train_patch.py:63-71); under
torchrun (WORLD_SIZE set) it is one rank.  The global batch is N*B (weak
scaling), each rank runs its contiguous shard of one seeded global batch with
draws keyed by global image index, and one all-reduce(SUM) of the weighted
patch gradient per step.  ``--dry-run`` exercises only the
launch, the sharding and the fused all-reduce (no GPU, no HIP step; CPU tests).
"""
import argparse
import json
import os
import platform
import socket
import subprocess
import sys
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402

PEAK_FP32_MFMA_TFLOPS = 157.3   # MI355X dense fp32 matrix peak (MI355X_MICROARCH.md)
PEAK_FP16_MFMA_TFLOPS = 2500.0  # MI355X dense fp16/bf16 matrix peak (no sparsity)
PEAK_HBM_GBS = 8000.0
# fp32-equivalent peak of each conv operand precision: exact fp32 MFMA, or
# fp16x3 (three fp16 MFMA products per fp32 product)
PEAK_CONV = {"fp32": PEAK_FP32_MFMA_TFLOPS, "fp16x3": PEAK_FP16_MFMA_TFLOPS / 3.0}

# kernel of each specialised po_conv tile (others: the generic conv_k<BM,BN,WM,BK>)
TILE_KERNELS = {61: "conv_wino_k", 65: "conv_wino2_k", 66: "conv_wino3_k", 67: "conv_wino4_k",
                68: "conv_wino4_k<stagger>", 69: "conv_halo_pool_k",
                70: "conv_wino5_k (persistent)", 71: "conv_wino6_k (F(4x4), persistent)",
                72: "wino6_pre_k + conv_wino6_k<PT> (F(4x4), pre-transformed input)",
                73: "conv_wpool_k (F(2x2) + pool, persistent)"}

CONFIGS = {
    # name: (cfg, S, P, default per-GPU batch)
    "yolov3": ("builtin:yolov3-dota", 608, 224, 16),
    "tiny": ("builtin:yolov3-tiny-dota", 416, 224, 256),
}


def conv_macs(net):
    """Algorithmic MACs per image of the forward convolutions (logical channels)."""
    plan_shapes = {}
    h = w = net.height
    total = 0
    shp = []
    for i, d in enumerate(net.blocks):
        t = d["type"]
        if t == "convolutional":
            m = net._conv_meta[i]
            h = (h + 2 * m["pad"] - m["k"]) // m["stride"] + 1
            w = (w + 2 * m["pad"] - m["k"]) // m["stride"] + 1
            total += h * w * m["cout"] * m["cin"] * m["k"] * m["k"]
        elif t == "maxpool" and int(d["stride"]) == 2:
            h, w = h // 2, w // 2
        elif t == "upsample":
            h, w = 2 * h, 2 * w
        elif t == "route":
            ls = [int(x) for x in d["layers"].split(",")]
            l0 = ls[0] if ls[0] >= 0 else i + ls[0]
            h, w = shp[l0]
        shp.append((h, w))
    return total


def _usable_cpus():
    """CPUs this process may actually use: the cgroup CPU quota (cpu.max) and
    the affinity mask bound it; os.cpu_count() reports the whole machine."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(int(quota) // int(period))))
    except (OSError, ValueError):
        pass
    return n


def _cpu_model():
    cpu = platform.processor() or platform.machine()
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return cpu


def cpu_baseline(cfg, S, P, B=16, warmup=1, iters=3):
    """the oracle (PyTorch-CPU fp32 restatement of the
    reference step, weight gradients ON as in the reference, no
    detect_anomaly) on the host cores, batch B, 1 warm-up + ``iters`` timed
    steps (3 for yolov3 @608, ~30 s; 10 for tiny @416, a few seconds).
    Threads: every CPU the process may use (the cgroup quota; on the GPU
    box os.cpu_count() shows the whole 256-CPU machine while the job's quota
    is 16, and oversubscribing a quota only slows torch down)."""
    import oracle
    sy, W, G, ld = ge._pkg("synthetic"), ge._pkg("weights"), ge._pkg("cfg_gen"), ge._pkg("load_data")
    cores = _usable_cpus()
    torch.set_num_threads(cores)
    stream = W.synthesize(cfg, seed=4)
    net = oracle.OracleDarknet(G.cfg_text(cfg), None, requires_grad=True)
    net.load_darknet_weights(stream)
    for p in net.params:
        if p is not None:
            for k in ("W", "b", "bn_b", "bn_w"):
                if k in p:
                    p[k].requires_grad_(True)
    colors = ld.load_printability_colors("builtin:30values")
    img, lab, patch, dr = sy.frames(B, S, seed=100), sy.labels(B, seed=101), sy.patch(P, seed=102), sy.draws(B, P, seed=103)
    for _ in range(warmup):
        oracle.train_step(patch, img, lab, dr, net, colors)
    t0 = time.time()
    for _ in range(iters):
        oracle.train_step(patch, img, lab, dr, net, colors)
    el = time.time() - t0
    return {"value": iters * B / el, "unit": "images/s", "cores": cores, "kind": "port",
            "sample": "oracle train_step (PyTorch-CPU fp32, weight grads on, no detect_anomaly), %s batch %d @%d, "
                      "%d timed steps after %d warm-up, %.1fs, %d threads (cgroup quota; os.cpu_count()=%d) of %s"
                      % (cfg, B, S, iters, warmup, el, cores, os.cpu_count() or 0, _cpu_model())}


WARP_ENTRIES = ("po_warp_fwd", "po_warp_bwd", "po_warp_fwd_keyed", "po_warp_bwd_keyed", "po_augment_patch",
                "po_warp_fwd_pre", "po_warp_bwd_pre", "po_warp_box_fwd_keyed", "po_warp_box_bwd_keyed",
                "po_warp_box_fwd_fac", "po_warp_box_bwd_fac")


def measure(tr, prec, patch, img, lab, B, world, rank, steps, warmup, weights):
    """Warm-up, K timed steps (barrier + synchronize on both sides, max over
    ranks), then K instrumented steps with HIP events around every po_conv
    launch and every warp entry (the roofline pass; kept out of the timed
    region because each event pair adds a ~10 us dispatch gap, profiles/r01)."""
    nat = ge._pkg("_native")
    net = tr.darknet_model
    net.conv_prec = prec
    opt = tr.make_optimizer(patch)
    pt = tr.patch_transformer
    pt.draw_b0 = rank * B                 # draws keyed by global image index (po_draws)

    def step():
        return tr.step(patch, opt, img, lab, weights=weights)

    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    if getattr(tr, "last_plan", None) is None or tr.last_plan.prec != (1 if prec == "fp16x3" else 0):
        tr.losses(patch, img, lab, weights=weights)      # --warmup 0: build the plan outside the timed region
        torch.cuda.synchronize()
    plan = tr.last_plan
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        terms = step()
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=img.device)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        elapsed = float(t)
    plan.conv_timer, plan.first_timer = [], []
    nat.TIMERS = {k: [] for k in WARP_ENTRIES}
    tr.ar_timer = [] if world > 1 else None
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    instrumented_ms = (time.perf_counter() - t1) * 1000.0 / steps
    timer, plan.conv_timer = plan.conv_timer, None
    # each step's cone snapshot to the host once (launch_macs reads per-image boxes)
    snaps = {}
    timer = [(e0, e1, d, None if c is None else snaps.setdefault(id(c), c.cpu())) for e0, e1, d, c in timer]
    warp, nat.TIMERS = nat.TIMERS, None
    ar, tr.ar_timer = tr.ar_timer, None
    # the fused [patch grad | 6 loss scalars] all-reduce, per step (this rank's view;
    # it includes the wait for the slowest rank to arrive)
    allreduce_ms = sum(e0.elapsed_time(e1) for e0, e1 in ar) / steps if ar else None
    conv_ms = sum(e0.elapsed_time(e1) for e0, e1, _, _ in timer) / steps
    # MACs actually computed: a boxed dgrad (gradient cones) counts its boxes only
    conv_flops = 2.0 * sum(plan.launch_macs(d, c) for _, _, d, c in timer) / steps
    # per tile family: time, dense-equivalent FLOPs and the FLOPs the matrix cores execute
    fam = {}
    for e0, e1, d, c in timer:
        key = ("winograd" if d.tile in plan.WINO_TILES or d.tile == plan.WPOOL_TILE
               else ("halo" if d.tile == plan.HALO_TILE else "direct"))
        f = fam.setdefault(key, {"ms": 0.0, "flops": 0.0, "mfma_flops": 0.0, "launches": 0, "tiles": {}})
        ms = e0.elapsed_time(e1)
        mf = plan.launch_mfma_flops(d, c)
        f["ms"] += ms
        f["flops"] += 2.0 * plan.launch_macs(d, c)
        f["mfma_flops"] += mf or 0.0
        f["launches"] += 1
        tt = f["tiles"].setdefault(int(d.tile), {"ms": 0.0, "mfma_flops": 0.0, "launches": 0})
        tt["ms"] += ms
        tt["mfma_flops"] += mf or 0.0
        tt["launches"] += 1
    for f in fam.values():
        for key in ("ms", "flops", "mfma_flops", "launches"):
            f[key] /= steps
        for tt in f["tiles"].values():
            for key in ("ms", "mfma_flops", "launches"):
                tt[key] /= steps
    warp_ms = {k: sum(e0.elapsed_time(e1) for e0, e1 in v) / steps for k, v in warp.items()}
    first = {}
    for e0, e1, name in plan.first_timer:
        first[name] = first.get(name, 0.0) + e0.elapsed_time(e1) / steps
    plan.first_timer = []
    # pixels of the quad-widened footprint boxes (the sparse composite's written
    # region, po::quad_box) of the last step: the box warp kernels' unit count
    roi = pt.last_roi.cpu().tolist() if pt.last_roi is not None else []
    box_px = sum(max(0, y1 - y0) * max(0, min(img.size(-1), (x1 + 3) & ~3) - (x0 & ~3)) for x0, y0, x1, y1 in roi
                 if min(img.size(-1), (x1 + 3) & ~3) > (x0 & ~3) and y1 > y0)
    dump = os.environ.get("ADVPATCH_LAUNCH_DUMP")
    if dump:
        # per-launch table (launch order of one step, averaged over the K steps)
        n = len(timer) // steps
        with open(dump, "w") as f:
            for k in range(n):
                _, _, d, c = timer[k]
                us = 1000.0 * sum(timer[s * n + k][0].elapsed_time(timer[s * n + k][1]) for s in range(steps)) / steps
                mf = plan.launch_mfma_flops(d, c) or 0.0
                f.write(json.dumps({"k": k, "tile": int(d.tile), "ksplit": int(d.ksplit), "B": d.B, "Hg": d.Hg,
                                    "Wg": d.Wg, "Hin": d.Hin, "Cin_p": d.Cin_p, "N": d.N, "ntaps": d.ntaps,
                                    "in_step": d.in_step, "mrows": d.mrows, "boxed": bool(d.gbox),
                                    "pool": bool(d.pool_y), "us": us, "mfma_tflops": mf / us / 1e6,
                                    "frac_mfma": mf / us / 1e6 / PEAK_CONV[prec]}) + "\n")
    tr.check_flags()
    return {"elapsed": elapsed, "ms_per_step": elapsed * 1000.0 / steps, "value": world * B * steps / elapsed,
            "conv_ms": conv_ms, "conv_flops": conv_flops, "launches": len(timer) // steps, "families": fam,
            "warp_ms": warp_ms, "first_ms": first, "box_px": box_px, "instrumented_ms": instrumented_ms,
            "loss": float(terms["loss"].detach()),
            "allreduce_ms": allreduce_ms, "plan": plan}


def roofline(cfg_name, B, prec, m, ref_flops_step):
    traffic = None
    tfile = os.path.join(ROOT, "profiles", "traffic_%s_b%d_%s.json" % (cfg_name, B, prec))
    if os.path.exists(tfile):
        with open(tfile) as f:
            traffic = json.load(f).get("conv_hbm_bytes_per_step")
    dense = m["conv_flops"] / (m["conv_ms"] * 1e-3) / 1e12
    peak = PEAK_CONV[prec]
    r = {"bound": "mfma",
         "kernel": "po_conv implicit GEMM (%s): every Darknet fwd + dgrad launch of a step" % (
             "conv_h3*_k, fp16x3 split operands" if prec == "fp16x3" else
             "conv_k + Winograd conv_wino*_k, exact fp32 v_mfma_f32_32x32x2_f32"),
         # fp32: replaced below by the FLOPs the matrix cores execute (a utilisation)
         "achieved": dense, "peak": peak, "unit": "TFLOP/s", "frac": dense / peak, "traffic": traffic,
         "achieved_dense_equiv": dense, "frac_dense_equiv": dense / peak,
         "dense_equiv_is": "2 x the direct-conv MACs of every launch (Winograd launches counted at their direct-conv "
                           "FLOPs) / conv time: NOT a utilisation (Winograd executes 4/9 of it)",
         "traffic_per": "step: HBM bytes of all conv launches + split-K reduces (rocprofv3 FETCH_SIZE/WRITE_SIZE "
                        "passes, profiles/traffic_*.json)",
         "peak_note": "fp32-equivalent: fp16 dense 2500 / 3 products" if prec == "fp16x3" else "fp32 dense MFMA",
         "flops_per_step": m["conv_flops"], "conv_ms_per_step": m["conv_ms"],
         "conv_launches_per_step": m["launches"],
         "measured_on": "a second pass of K steps with per-launch HIP events (%.3f ms/step instrumented vs %.3f "
                        "plain)" % (m["instrumented_ms"], m["ms_per_step"]),
         "reference_dense_flops_per_step": ref_flops_step,
         # SURVEY §8d's algorithmic rate: the reference's dense fwd + dgrad FLOPs of the
         # images processed, over the whole step's wall time (windows, cones and Winograd
         # skip part of that work, so this can exceed the MFMA peak)
         "achieved_algorithmic": ref_flops_step / (m["ms_per_step"] * 1e-3) / 1e12,
         "frac_algorithmic": ref_flops_step / (m["ms_per_step"] * 1e-3) / 1e12 / peak,
         "frac_algorithmic_is": "the reference's dense fwd+dgrad FLOPs over the step's wall time: includes the work "
                                "removed by receptive-field windows, gradient cones and Winograd (not a utilisation)",
         "receptive_field_windows": bool(m["plan"].windowed)}
    if prec == "fp32":
        fam = m["families"]
        mf = sum(f["mfma_flops"] for f in fam.values())
        r["mfma_flops_per_step"] = mf
        r["achieved_mfma"] = mf / (m["conv_ms"] * 1e-3) / 1e12
        r["frac_mfma"] = r["achieved_mfma"] / peak
        r["achieved"], r["frac"] = r["achieved_mfma"], r["frac_mfma"]
        r["achieved_is"] = r["frac_mfma_is"] = (
            "FLOPs the matrix cores execute (v_mfma_f32_32x32x2_f32: padded tiles, Winograd F(2x2) at 16 GEMMs "
            "per 2x2 tile = 4/9 of the direct work, F(4x4) at 36 per 4x4 tile = 1/4; NetPlan.launch_mfma_flops) "
            "/ conv time / the 157.3 TFLOP/s peak at 2.4 GHz: the MFMA utilisation of the conv launches")
        r["families"] = {k: {"ms_per_step": f["ms"], "launches_per_step": f["launches"],
                             "mfma_tflops": f["mfma_flops"] / (f["ms"] * 1e-3) / 1e12 if f["ms"] else None,
                             "frac_mfma": f["mfma_flops"] / (f["ms"] * 1e-3) / 1e12 / peak if f["ms"] else None,
                             "dense_equiv_tflops": f["flops"] / (f["ms"] * 1e-3) / 1e12 if f["ms"] else None}
                         for k, f in fam.items()}
        # the dominant kernel: the tile with the most time per step
        best = max(((t, tt, k) for k, f in fam.items() for t, tt in f["tiles"].items()), key=lambda x: x[1]["ms"])
        t, tt, k = best
        name = TILE_KERNELS.get(t, "conv_k")
        r["dominant_kernel"] = {"kernel": "%s (po_conv tile %d, %s)" % (name, t, k), "ms_per_step": tt["ms"],
                                "launches_per_step": tt["launches"],
                                "avg_launch_us": 1000.0 * tt["ms"] / max(tt["launches"], 1e-9),
                                "mfma_tflops": tt["mfma_flops"] / (tt["ms"] * 1e-3) / 1e12,
                                "frac_mfma": tt["mfma_flops"] / (tt["ms"] * 1e-3) / 1e12 / peak}
    return r


def warp_roofline(m, B, S, P, cp0=None):
    """HBM fractions of the fused augment/warp/composite kernels, per call,
    HIP events on the launch stream.  Algorithmic bytes: the
    whole-frame forms (po_warp_*_pre, _keyed) read the frame and write the
    composite, 2*3*S^2*4 B per image, plus the 3*P^2*4 B patch; their
    backward reads dL/dp_img, 3*S^2*4 B per image.  The training step's box
    form (po_warp_box_*_keyed on the sparse composite) touches only the
    quad-widened footprint boxes: forward 3*4 B read (frame) + 3*4 B written
    per box pixel plus the patch, backward 3*4 B of dL/dp_img read + 3*4 B of
    gfac written and read again per box pixel plus the 3*P^2*4 B patch
    gradient written; the frame itself is then read by the first layer
    (po_conv_first_*_cmp: 3*S^2*4 B per image in, its NHWC output out),
    reported as ``first_layer``.  With the forward-saved factors
    (po_warp_box_*_fac, the default) the forward also writes 16 B of factors
    per box pixel and the backward reads them (16 B) instead of re-evaluating
    the warp: 40 B and 60 B per box pixel."""
    out = {}
    wm = m["warp_ms"]
    box_px = m.get("box_px") or 0
    if wm.get("po_warp_box_fwd_fac"):
        forms = (("po_warp_fwd", "po_warp_box_fwd_fac", box_px * 40 + 3 * P * P * 4),
                 ("po_warp_bwd", "po_warp_box_bwd_fac", box_px * 60 + 3 * P * P * 4))
    elif wm.get("po_warp_box_fwd_keyed"):
        forms = (("po_warp_fwd", "po_warp_box_fwd_keyed", box_px * 24 + 3 * P * P * 4),
                 ("po_warp_bwd", "po_warp_box_bwd_keyed", box_px * 36 + 3 * P * P * 4))
    else:
        forms = []
        for base, per_img, extra in (("po_warp_fwd", 2 * 3 * S * S * 4, 3 * P * P * 4),
                                     ("po_warp_bwd", 3 * S * S * 4, 0)):
            if wm.get(base + "_pre"):
                forms.append((base, base + "_pre", B * per_img + extra))
            else:
                forms.append((base, base + "_keyed" if wm.get(base + "_keyed") else base, B * per_img + extra))
    for base, name, byts in forms:
        ms = wm.get(name)
        if name == "po_warp_fwd_pre" and ms:
            ms += wm.get("po_augment_patch", 0.0)
            name += " + po_augment_patch"
        if not ms:
            continue
        gbs = byts / (ms * 1e-3) / 1e9
        r = {"entries": name, "bound": "hbm", "algorithmic_bytes": byts, "us_per_call": ms * 1000.0,
             "achieved": gbs, "peak": PEAK_HBM_GBS, "unit": "GB/s", "frac": gbs / PEAK_HBM_GBS}
        if "box" in name:
            r["box_pixels"] = box_px
            r["note"] = ("sparse composite: only the footprint boxes (%.2f%% of the frames) are warped and written; "
                         "the %d-byte frame copy of the whole-frame forms no longer exists (first_layer reads the "
                         "frames)" % (100.0 * box_px / (B * S * S), 2 * 3 * S * S * 4 * B))
        out[base] = r
    first = m.get("first_ms") or {}
    if first and cp0:
        name, ms = max(first.items(), key=lambda kv: kv[1])
        ho = S // 2 if "pool" in name else S        # the configs' first layers: stride 1 (+ fused 2x2 pool)
        byts = B * 3 * S * S * 4 + B * ho * ho * cp0 * (5 if "pool" in name else 4)
        gbs = byts / (ms * 1e-3) / 1e9
        out["first_layer"] = {"entries": name, "bound": "hbm", "algorithmic_bytes": byts, "us_per_call": ms * 1000.0,
                              "achieved": gbs, "peak": PEAK_HBM_GBS, "unit": "GB/s", "frac": gbs / PEAK_HBM_GBS,
                              "bytes_are": "frames in (3*S^2*4 B per image) + NHWC output out (pool: floats + "
                                           "argmax bytes)"}
    return out


def build_trainer(tp, pc, W, cfg, B, world, dev, name):
    wpath = pc.synthetic_weights_path(cfg.split(":")[-1])

    class _Cfg(pc.ReproducePaperObj):
        def __init__(self):
            super().__init__()
            self.cfgfile = cfg
            self.weightfile = wpath
            self.batch_size = B * world

    pc.patch_configs[name] = _Cfg
    return tp.PatchTrainer(name, device=dev, verbose=False, distributed=world > 1)


def measure_tiny(args, dev):
    """Config 5 (yolov3-tiny-15 @416, B=256, 1 GPU) in the same run: exact
    fp32 value, conv roofline with frac_mfma, and the warp kernels' HBM
    fractions (the bandwidth-bound stress this config exists for)."""
    tp, pc, sy, W = ge._pkg("train_patch"), ge._pkg("patch_config"), ge._pkg("synthetic"), ge._pkg("weights")
    cfg, S, P, B = CONFIGS["tiny"]
    old = os.environ.get("ADVPATCH_TUNE_CACHE")
    os.environ["ADVPATCH_TUNE_CACHE"] = os.path.join(ge.PKG_DIR, "tiles", "conv_tiles_tiny_b%d.json" % B)
    try:
        W.ensure_synthetic(cfg, pc.synthetic_weights_path(cfg.split(":")[-1]))
        tr = build_trainer(tp, pc, W, cfg, B, 1, dev, "_bench_tiny")
        img = sy.frames_slice(0, B, S, seed=1000).to(dev)
        lab = sy.labels_slice(0, B, seed=2000).to(dev)
        patch = sy.patch(P, seed=2).to(dev).requires_grad_(True)
        m = measure(tr, "fp32", patch, img, lab, B, 1, 0, args.steps, args.warmup, None)
    finally:
        if old is None:
            os.environ.pop("ADVPATCH_TUNE_CACHE", None)
        else:
            os.environ["ADVPATCH_TUNE_CACHE"] = old
    ref = 4.0 * conv_macs(tr.darknet_model) * B
    return {"value_tiny": m["value"], "ms_per_step_tiny": m["ms_per_step"],
            "config_tiny": {"workload": "%s S=%d P=%d batch=%d (BASELINE config 5)" % (cfg, S, P, B),
                            "global_batch": B, "image_size": S, "patch_size": P, "parallelism": "dp1",
                            "conv_precision": "fp32"},
            "roofline_tiny": roofline("tiny", B, "fp32", m, ref), "warp_roofline_tiny": warp_roofline(m, B, S, P, m["plan"].cp[0]),
            "loss_tiny": m["loss"]}


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def visible_gpu_count():
    """GPUs this process could use, counted without any HIP call (the parent
    of the ranks must leave the devices untouched): the KFD topology's GPU
    nodes (simd_count > 0), narrowed by the visible-device variables the ROCm
    runtime honours.  None when neither source is readable (the ranks then
    find out themselves)."""
    n = None
    try:
        root = "/sys/class/kfd/kfd/topology/nodes"
        n = 0
        for d in os.listdir(root):
            try:
                with open(os.path.join(root, d, "properties")) as f:
                    props = dict(line.split()[:2] for line in f if len(line.split()) >= 2)
            except OSError:
                continue
            if int(props.get("simd_count", "0")) > 0:
                n += 1
    except (OSError, ValueError):
        n = None
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            k = len([x for x in v.split(",") if x.strip() != ""])
            n = k if n is None else min(n, k)
    return n


def launch_ranks(args):
    """``bench.py --gpus N`` outside torchrun: start the N ranks as children
    (python -m torch.distributed.run, one process per GPU, rendezvous on
    127.0.0.1) and exit with their status.  Nothing here touches the GPU
    (visible_gpu_count reads the KFD topology and the environment), so the
    children own the devices.  Every rank inherits stdout; only rank 0 prints the JSON line."""
    n = args.gpus
    if args.dist_backend == "nccl" and not args.dry_run:
        ndev = visible_gpu_count()
        if ndev is not None and n > ndev:
            raise SystemExit("bench.py --gpus %d: only %d GPU(s) visible; RCCL needs one GPU per rank "
                             "(use --dist-backend gloo to rehearse ranks sharing a GPU)" % (n, ndev))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("OMP_NUM_THREADS", "1")
    return subprocess.call(cmd, env=env)


def dry_run(args, world, rank):
    """--dry-run: the multi-rank plumbing without a GPU — the process group,
    this rank's shard of the global batch (GlobalBatchSampler.shard_of, as
    train() and the synthetic bench slice it), and the fused all-reduce of
    [patch grad | 6 loss scalars] (train_patch.allreduce_patch_grad), checked
    against its known sum.  Prints a line with value null: nothing is measured."""
    tp = ge._pkg("train_patch")
    cfg, S, P, Bdef = CONFIGS[args.config]
    B = args.batch or Bdef
    G = B * world
    lo, hi, ng = tp.GlobalBatchSampler(G, G, rank, world, shuffle=False).shard_of(0)
    grad = torch.full((3, P, P), float(rank + 1))
    t0 = time.perf_counter()
    for _ in range(args.steps):
        g = grad.clone()
        terms = {k: torch.tensor(float(hi - lo)) for k in tp.LOSS_KEYS}
        if world > 1:
            tp.allreduce_patch_grad(g, terms)
    el = time.perf_counter() - t0
    want = world * (world + 1) / 2.0
    assert float(g.min()) == float(g.max()) == want, (float(g.min()), want)
    assert all(float(terms[k]) == G for k in tp.LOSS_KEYS)
    shards = [(lo, hi)] * world
    if world > 1:
        torch.distributed.all_gather_object(shards, (lo, hi))
    if rank == 0:
        print(json.dumps({"metric": "patch-opt images/sec (dry run: launch, sharding and all-reduce only)",
                          "value": None, "unit": "images/s", "n_gpus": world, "steps": args.steps,
                          "warmup": args.warmup, "dry_run": True,
                          "dist_backend": torch.distributed.get_backend() if world > 1 else None,
                          "config": {"workload": "%s S=%d P=%d batch=%d per GPU, global %d" % (cfg, S, P, B, G),
                                     "global_batch": G, "per_gpu_batch": B, "parallelism": "dp%d" % world},
                          "shards": shards, "allreduce_ms_per_step": el * 1000.0 / args.steps,
                          "allreduce_bytes": 4 * (3 * P * P + len(tp.LOSS_KEYS))}))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1, help="ranks, one per GPU (launched here unless under torchrun)")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=None, help="per-GPU batch")
    ap.add_argument("--config", default="yolov3", choices=sorted(CONFIGS))
    ap.add_argument("--prec", default="fp32", choices=("fp32", "both", "fp16x3"),
                    help="conv operand precision(s) timed: value is exact fp32; 'both' adds the opt-in fp16x3 "
                         "split-precision path beside it")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-tiny", action="store_true", help="skip config 5 (timed beside the yolov3 line at N=1)")
    ap.add_argument("--dist-backend", default="nccl", help="nccl (= RCCL); gloo only to rehearse ranks on one GPU")
    ap.add_argument("--tile-cache", default=None, help="conv tile cache (default: the committed tiles/ file)")
    ap.add_argument("--dry-run", action="store_true", help="launch + sharding + all-reduce only (no GPU)")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and rank == 0:
        print("bench.py: --gpus %d but WORLD_SIZE=%d; measuring %d ranks" % (args.gpus, world, world),
              file=sys.stderr)
    if args.dry_run:
        if world > 1:
            torch.distributed.init_process_group("gloo" if args.dist_backend == "nccl" else args.dist_backend)
        dry_run(args, world, rank)
        if world > 1:
            torch.distributed.destroy_process_group()
        return
    ndev = torch.cuda.device_count()
    if world > 1:
        torch.cuda.set_device(local % ndev)
        if args.dist_backend == "nccl":
            torch.distributed.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            torch.distributed.init_process_group(args.dist_backend)
    dev = torch.device("cuda", local % ndev)
    cfg, S, P, Bdef = CONFIGS[args.config]
    B = args.batch or Bdef
    # conv tile choices: the committed per-(config, batch) cache keeps runs
    # reproducible (same tiles -> same summation order); shapes it lacks are
    # autotuned on first use
    os.environ["ADVPATCH_TUNE_CACHE"] = args.tile_cache or os.path.join(
        ge.PKG_DIR, "tiles", "conv_tiles_%s_b%d.json" % (args.config, B))

    tp, pc, sy, W = ge._pkg("train_patch"), ge._pkg("patch_config"), ge._pkg("synthetic"), ge._pkg("weights")
    wpath = pc.synthetic_weights_path(cfg.split(":")[-1])
    if rank == 0:
        W.ensure_synthetic(cfg, wpath)
    if world > 1:
        torch.distributed.barrier()
    tr = build_trainer(tp, pc, W, cfg, B, world, dev, "_bench")

    # this rank's contiguous shard of one seeded global batch
    img = sy.frames_slice(rank * B, B, S, seed=1000).to(dev)
    lab = sy.labels_slice(rank * B, B, seed=2000).to(dev)
    patch = sy.patch(P, seed=2).to(dev).requires_grad_(True)
    weights = tp.shard_weights(B, B * world, world, tr.objective) if world > 1 else None
    ref_flops_step = 4.0 * conv_macs(tr.darknet_model) * B      # reference algorithm: dense fwd + dgrad (§8d)

    precs = ["fp32", "fp16x3"] if args.prec == "both" else [args.prec]
    res = {p: measure(tr, p, patch, img, lab, B, world, rank, args.steps, args.warmup, weights) for p in precs}

    if rank == 0:
        head = precs[0]
        m = res[head]
        line = {
            "metric": "patch-opt images/sec (608x608, YOLOv3-DOTA) at 1/2/4/8 MI355X" if args.config == "yolov3"
            else "patch-opt images/sec (416x416, YOLOv3-tiny-15)",
            "value": m["value"], "unit": "images/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": m["ms_per_step"], "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "fp32" if head == "fp32" else "fp32 (fp16x3 split MFMA, fp32 accumulate)",
            "data": "synthetic (seeded DOTA-shaped frames/labels, synthetic calibrated weights)",
            "config": {"workload": "%s S=%d P=%d batch=%d per GPU, global %d" % (cfg, S, P, B, B * world),
                       "global_batch": B * world, "per_gpu_batch": B, "image_size": S, "patch_size": P,
                       "parallelism": "dp%d" % world, "conv_precision": head},
            "roofline": roofline(args.config, B, head, m, ref_flops_step),
            "warp_roofline": warp_roofline(m, B, S, P, m["plan"].cp[0]),
            "loss": m["loss"],
        }
        if world > 1:
            line["dist_backend"] = args.dist_backend
            line["allreduce_ms_per_step"] = m["allreduce_ms"]
            line["allreduce_bytes"] = 4 * (3 * P * P + len(tp.LOSS_KEYS))
        if "fp16x3" in res and head != "fp16x3":
            f = res["fp16x3"]
            line["value_fp16x3"] = f["value"]
            line["ms_per_step_fp16x3"] = f["ms_per_step"]
            line["dtype_fp16x3"] = ("fp32 operands held as two fp16 pieces (~22 significant bits) under a "
                                    "power-of-two scale, three fp16 MFMA products, fp32 accumulate")
            line["roofline_fp16x3"] = roofline(args.config, B, "fp16x3", f, ref_flops_step)
            line["loss_fp16x3"] = f["loss"]
        if world == 1 and args.config == "yolov3" and not args.no_tiny:
            line.update(measure_tiny(args, dev))
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(cfg, S, P, B=16)
            if "value_tiny" in line:
                # BASELINE.md's CPU sample for config 5: the oracle tiny-15 step, B=16 @416
                tcfg, tS, tP, _ = CONFIGS["tiny"]
                line["cpu_baseline_tiny"] = cpu_baseline(tcfg, tS, tP, B=16, iters=10)
        print(json.dumps(line))
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
