"""Throughput of the frames-from-files stage: tmrnet_amd.frames.load_frames =
the reference's pil_loader (train_only_non-local_pretrained.py:96-99) in a host thread pool ->
pinned batch -> HBM -> tmr_resize_u8 (Resize((250, 250)), :336), next to the train step's
consumption rate.

Threads (decode_frames) and worker processes (DecodePool).  Synthetic JPEGs (smooth colour field + noise, quality 95, written to a temp dir) at Cholec80's
native 854x480 and at a pre-resized 250x250.  Prints one JSON line per (size, workers)."""
import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np
from PIL import Image

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def write_jpegs(d, n, w, h, seed=0):
    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:h, 0:w]
    paths = []
    for i in range(n):
        base = np.stack([(xx * (1 + i % 5) + yy) % 256, (yy * 2 + i * 7) % 256,
                         (xx + yy * 3 + i * 13) % 256], -1).astype(np.float32)
        img = np.clip(base + rng.normal(0, 12, base.shape), 0, 255).astype(np.uint8)
        p = os.path.join(d, "%05d.jpg" % i)
        Image.fromarray(img).save(p, quality=95)
        paths.append(p)
    return paths


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=640, help="one C2 step's frames per batch")
    ap.add_argument("--batches", type=int, default=3)
    ap.add_argument("--workers", default="8,16")
    ap.add_argument("--sizes", default="854x480,250x250")
    ap.add_argument("--modes", default="threads,processes",
                    help="threads = decode_frames' thread pool; processes = DecodePool workers")
    args = ap.parse_args()
    import torch
    from tmrnet_amd import frames
    dev = torch.device("cuda:0") if torch.cuda.is_available() else None
    for size in args.sizes.split(","):
        w, h = (int(v) for v in size.split("x"))
        with tempfile.TemporaryDirectory() as d:
            paths = write_jpegs(d, args.frames, w, h)
            mb = sum(os.path.getsize(p) for p in paths) / 1e6
            for mode in args.modes.split(","):
                for nw in (int(v) for v in args.workers.split(",")):
                    pool = frames.DecodePool(workers=nw) if mode == "processes" else None
                    dec = ((lambda ps: pool.decode(ps)) if pool is not None else
                           (lambda ps: frames.decode_frames(ps, workers=nw)))
                    dec(paths[:64])   # warm the page cache / the pool's workers
                    t0 = time.perf_counter()
                    for _ in range(args.batches):
                        host = dec(paths)
                    t_dec = (time.perf_counter() - t0) / args.batches
                    rec = {"stage": "frames-from-files", "mode": mode, "size": size, "workers": nw,
                           "frames": args.frames, "jpeg_mb": round(mb, 1),
                           "decode_frames_per_s": round(args.frames / t_dec, 1)}
                    if dev is not None:
                        frames.load_frames(paths[:64], device=dev, workers=nw, pool=pool)
                        torch.cuda.synchronize()
                        t0 = time.perf_counter()
                        for _ in range(args.batches):
                            out = frames.load_frames(paths, device=dev, workers=nw, pool=pool)
                        torch.cuda.synchronize()
                        t_all = (time.perf_counter() - t0) / args.batches
                        assert tuple(out.shape) == (args.frames, 250, 250, 3)
                        rec["load_frames_per_s"] = round(args.frames / t_all, 1)
                    if pool is not None:
                        pool.close()
                    rec["host_cpus"] = len(os.sched_getaffinity(0))
                    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
