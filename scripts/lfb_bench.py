"""LFB construction throughput on one MI355X.

Workload: `--videos` synthetic videos of `--frames` uint8 250x250x3 frames resident in HBM, a
random-init ``resnet_lstm_LFB`` (T = --seq), fp32.  Two device paths over the same clips:

* ``builder``   -- tmrnet_amd.lfb_build (each frame encoded once, gate table, batched recurrence);
* ``per_clip``  -- the reference's loop structure (train_only_non-local_pretrained.py:570-581) on
                   the same kernels: every clip's T frames through the model, 64 clips a batch
                   (timed on a bounded sample of `--per-clip-batches` batches, then scaled).

Both report clips/s (bank rows per second); frames/s for the builder counts encoded frames.
The rows of the two paths are compared (max |diff|).  Prints one JSON line.
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--videos", type=int, default=4)
    ap.add_argument("--frames", type=int, default=1500)
    ap.add_argument("--seq", type=int, default=10)
    ap.add_argument("--per-clip-batches", type=int, default=4)
    args = ap.parse_args()
    import tmrnet_amd
    from tmrnet_amd import lfb_build, ops

    dev = torch.device("cuda:0")
    T = args.seq
    torch.manual_seed(0)
    m = tmrnet_amd.resnet_lstm_LFB(seq_len=T).to(dev).eval()
    lengths = [args.frames] * args.videos
    g = torch.Generator().manual_seed(1)
    frames = torch.randint(0, 256, (sum(lengths), 250, 250, 3), generator=g,
                           dtype=torch.uint8).to(dev)
    b = lfb_build.LFBBuilder(m)
    b.build(frames[:T * 4], [T * 4])            # warm-up (kernels, allocator)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    bank, valid = b.build(frames, lengths)
    torch.cuda.synchronize()
    tb = time.perf_counter() - t0

    # reference loop structure on the same kernels, bounded sample
    B = 64
    off = torch.full((B, 2), lfb_build.center_offset(250), dtype=torch.int32, device=dev)
    nb = min(args.per_clip_batches, len(valid) // B)
    rows = []

    def batch(i):
        starts = valid[i * B:(i + 1) * B]
        idx = torch.tensor([s + j for s in starts for j in range(T)], device=dev)
        x4 = ops.crop_normalize(frames.index_select(0, idx), off, T)
        with torch.no_grad():
            return m(x4)

    batch(0)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(nb):
        rows.append(batch(i))
    torch.cuda.synchronize()
    tp = time.perf_counter() - t0
    diff = (torch.cat(rows) - bank[:nb * B]).abs().max().item()
    line = {"metric": "LFB construction clips/s (resnet_lstm_LFB, seq=%d)" % T,
            "value": round(len(valid) / tb, 1), "unit": "clips/s", "n_gpus": 1,
            "higher_is_better": True, "dtype": "fp32",
            "data": "synthetic (%d videos x %d uint8 250x250x3 frames in HBM, random-init weights)"
                    % (args.videos, args.frames),
            "builder": {"clips": len(valid), "frames_encoded": sum(lengths), "seconds": round(tb, 3),
                        "clips_per_s": round(len(valid) / tb, 1),
                        "frames_per_s": round(sum(lengths) / tb, 1)},
            "per_clip_reference_structure": {"clips": nb * B, "seconds": round(tp, 3),
                                             "clips_per_s": round(nb * B / tp, 1),
                                             "frames_per_s": round(nb * B * T / tp, 1)},
            "speedup": round((len(valid) / tb) / (nb * B / tp), 2),
            "max_abs_row_diff": diff}
    print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
