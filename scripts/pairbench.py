"""FWD vs DGRAD on identical GEMM dimensions (M = F*H*W, N, K) -- isolates view-specific costs.

usage: python scripts/pairbench.py [--frames 640] [--reps 5]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tmrnet_amd import ops  # noqa: E402

# (h, small, big): FWD small->big and DGRAD of big->small have the same GEMM (M, N=big, K=small)
PAIRS = [(56, 64, 256), (28, 128, 512), (14, 256, 1024), (7, 512, 2048)]


def timeit(fn, reps):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=640)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    for h, s, b in PAIRS:
        n = a.frames
        xs = torch.randn(n, h, h, s, device=dev)          # FWD input (K = s)
        wf = torch.randn(b, 1, 1, s, device=dev)          # FWD weight (N = b)
        yb = torch.empty(n, h, h, b, device=dev)
        wd = torch.randn(s, 1, 1, b, device=dev)          # conv b->s; dgrad N = b, K = s
        dys = torch.randn(n, h, h, s, device=dev)
        dxb = torch.empty(n, h, h, b, device=dev)
        tf = timeit(lambda: ops.conv_fwd(xs, wf, 1, 0, out=yb), a.reps)
        td = timeit(lambda: ops.conv_dgrad(dys, wd, (h, h), 1, 0, out=dxb), a.reps)
        gb = (n * h * h * (s + b) * 4) / 1e9
        print("M=%d N=%d K=%d  fwd %.3f ms (%.2f TB/s)  dgrad %.3f ms (%.2f TB/s)  ratio %.2f"
              % (n * h * h, b, s, tf, gb / tf, td, gb / td, td / tf), flush=True)


if __name__ == "__main__":
    main()
