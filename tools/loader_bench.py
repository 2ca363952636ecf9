"""Host data-path throughput: DotaDataset decode + pad + resize
through a DataLoader (GlobalBatchSampler, pinned batches), and the
DevicePrefetcher feed, on synthetic DOTA-like PNGs written to a temp dir.

    python tools/loader_bench.py [--n 128] [--side 1024] [--size 608] [--batch 16] [--workers 1,4,8,16]

Prints one JSON line per configuration: images/s of the loader alone, and of
loader + prefetcher (uint8 H2D copy + /255 on the device) when a GPU is present."""
import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as ge  # noqa: E402


def make_set(d, n, side, seed=0):
    from PIL import Image
    rng = np.random.default_rng(seed)
    os.makedirs(os.path.join(d, "images"))
    os.makedirs(os.path.join(d, "labels"))
    yy, xx = np.mgrid[0:side, 0:side].astype(np.float32) / side
    for k in range(n):
        h = side if k % 3 else side * 3 // 4                      # some non-square frames (padding path)
        base = 128 + 60 * np.sin(6.3 * (xx[:h] * (1 + k % 5) + yy[:h] * 2))[..., None] * np.array([1.0, 0.8, 0.6])
        img = np.clip(base + rng.normal(0, 12, (h, side, 3)), 0, 255).astype(np.uint8)
        Image.fromarray(img, "RGB").save(os.path.join(d, "images", "%05d.png" % k))
        rows = rng.uniform(0.05, 0.95, (int(rng.integers(1, 40)), 5))
        rows[:, 0] = rng.integers(0, 15, len(rows))
        np.savetxt(os.path.join(d, "labels", "%05d.txt" % k), rows, fmt="%.6f")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=128)
    ap.add_argument("--side", type=int, default=1024)
    ap.add_argument("--size", type=int, default=608)
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--workers", default="1,4,8,16")
    args = ap.parse_args()
    ld, tp = ge._pkg("load_data"), ge._pkg("train_patch")
    gpu = torch.cuda.is_available()
    with tempfile.TemporaryDirectory() as d:
        t0 = time.time()
        make_set(d, args.n, args.side)
        png_mb = sum(os.path.getsize(os.path.join(d, "images", f)) for f in os.listdir(os.path.join(d, "images"))) / 1e6
        for w in [int(x) for x in args.workers.split(",")]:
            ds = ld.DotaDataset(os.path.join(d, "images"), os.path.join(d, "labels"), 252, args.size, as_uint8=True)
            smp = tp.GlobalBatchSampler(len(ds), args.batch, shuffle=True, seed=0)
            dl = torch.utils.data.DataLoader(ds, batch_sampler=smp, num_workers=w, pin_memory=gpu,
                                             persistent_workers=w > 0, prefetch_factor=4 if w else None)
            for _ in dl:                          # warm-up epoch: workers up, page cache hot
                pass
            t = time.perf_counter()
            n = sum(img.size(0) for img, _ in dl)
            host = n / (time.perf_counter() - t)
            line = {"workers": w, "images": n, "loader_img_s": host, "frame": "%dx%d PNG (%.2f MB avg)" % (
                args.side, args.side, png_mb / args.n), "out": "%dx%d uint8" % (args.size, args.size),
                "host_cpus": len(os.sched_getaffinity(0))}
            if gpu:
                dev = torch.device("cuda", 0)
                pf = ld.DevicePrefetcher(dl, dev)
                torch.cuda.synchronize()
                t = time.perf_counter()
                n = 0
                for img, lab in pf:
                    n += img.size(0)
                torch.cuda.synchronize()
                line["loader_prefetch_img_s"] = n / (time.perf_counter() - t)
            print(json.dumps(line), flush=True)
            del dl
        if gpu:
            # device frame cache: one decode pass, then batches gathered in HBM
            dev = torch.device("cuda", 0)
            w = max(int(x) for x in args.workers.split(","))
            ds = ld.DotaDataset(os.path.join(d, "images"), os.path.join(d, "labels"), 252, args.size, as_uint8=True)
            t = time.perf_counter()
            cache = ld.FrameCache(ds, dev, num_workers=w)
            fill = time.perf_counter() - t
            smp = tp.GlobalBatchSampler(len(ds), args.batch, shuffle=True, seed=0)
            it = cache.loader(smp)
            for _ in it:
                pass
            torch.cuda.synchronize()
            t = time.perf_counter()
            n = 0
            for _ in range(5):
                for img, lab in it:
                    n += img.size(0)
            torch.cuda.synchronize()
            print(json.dumps({"frame_cache_fill_img_s": len(ds) / fill, "workers": w,
                              "cached_batches_img_s": n / (time.perf_counter() - t),
                              "hbm_bytes_per_frame": 3 * args.size * args.size + 252 * 5 * 4}), flush=True)
            # the copy alone: a pinned uint8 batch vs a pinned float32 batch, host -> device
            dev = torch.device("cuda", 0)
            for dt in (torch.uint8, torch.float32):
                x = torch.zeros(args.batch, 3, args.size, args.size, dtype=dt).pin_memory()
                y = torch.empty_like(x, device=dev)
                for _ in range(3):
                    y.copy_(x, non_blocking=True)
                torch.cuda.synchronize()
                t = time.perf_counter()
                for _ in range(20):
                    y.copy_(x, non_blocking=True)
                torch.cuda.synchronize()
                el = (time.perf_counter() - t) / 20
                print(json.dumps({"h2d_batch": str(dt), "ms": el * 1e3, "GB_s": x.numel() * x.element_size() / el / 1e9,
                                  "img_s": args.batch / el}), flush=True)
        print(json.dumps({"setup_s": time.time() - t0}), flush=True)


if __name__ == "__main__":
    main()
