"""Microbenchmark of the fused BN-backward 1x1 dgrads of the train step, in the step's own forms:
the Bottleneck conv1 dgrads adding into the residual-stream gradient (beta 1; bf16 step: y, z, old
gradient bf16, g stored bf16 -- EpiForm 1; fp32 step: y, old gradient fp32, ReLU-mask bits --
EpiForm 2) and the conv3 dgrads (mask from y, beta 0).  Per shape: ms per launch and the
algorithmic HBM rate (every operand byte once: dy, y, z / bits, old g, new g).

usage: python scripts/resdgrad_bench.py [--frames 640] [--reps 10] [--prec bf16,fp32]
                                        [--kinds res,c3] [--json out.json]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tmrnet_amd import ops  # noqa: E402

# (h, dx channels N, dy channels K): the residual conv1 dgrads (N = 4 planes, K = planes) and the
# conv3 dgrads (N = planes, K = 4 planes) of ResNet-50's stride-1 blocks
RES = [(56, 256, 64), (28, 512, 128), (14, 1024, 256), (7, 2048, 512)]
C3 = [(56, 64, 256), (28, 128, 512), (14, 256, 1024), (7, 512, 2048)]
# the 1x1 stride-1 forwards with the fused BN statistics: (h, output channels N, input channels K)
FWD = [(56, 256, 64), (28, 512, 128), (14, 1024, 256), (56, 128, 256), (7, 2048, 512)]


def pack_bits(keep):
    """bool -> int32 ReLU-mask words, element e = bit e % 32 of word e // 32 (bn_apply_bits)."""
    m = keep.reshape(-1).to(torch.int64)
    m = torch.cat([m, m.new_zeros((-m.numel()) % 32)]).view(-1, 32)
    w = (m << torch.arange(32, dtype=torch.int64, device=m.device)).sum(1)
    return torch.where(w >= 2 ** 31, w - 2 ** 32, w).to(torch.int32)


def run(kind, prec, F, h, n, k, reps, dev):
    g = torch.Generator(device="cpu").manual_seed(1)
    bf = prec == "bf16"
    dt = torch.bfloat16 if bf else torch.float32
    dy = torch.randn(F, h, h, k, generator=g).to(dev).to(dt)
    w = (torch.randn(k, n, 1, 1, generator=g) / k ** 0.5).to(dev)
    wct = ops.weight_to_crsk(w, bf16=bf)
    y = torch.randn(F, h, h, n, generator=g).to(dev).to(dt)
    mean = torch.zeros(n, device=dev)
    zf = torch.relu(y.float() + 0.3)
    if kind == "fwd":
        x = torch.randn(F, h, h, k, generator=g).to(dev).to(dt)
        wk = ops.weight_to_krsc((torch.randn(n, k, 1, 1, generator=g) / k ** 0.5).to(dev), bf16=bf)
        fn = lambda: ops.conv_fwd_bnstats(x, wk, 1, 0, math=prec, y16=bf)
        per = 2 if bf else 4   # y
        dy = x                 # (the operand read: x)
    elif kind == "res":
        old = torch.randn(F, h, h, n, generator=g).to(dev).to(dt)
        if bf:
            z = zf.to(dt)
            fn = lambda: ops.conv_dgrad_bnbwd(dy, wct, (h, h), 1, 0, y, mean, 1, z=z, out=old,
                                              beta=1.0, math=prec, wt=True, g16=True)
            per = 2 * 4          # y, z, old, new (bf16)
        else:
            bits = pack_bits(zf > 0)
            fn = lambda: ops.conv_dgrad_bnbwd(dy, wct, (h, h), 1, 0, y, mean, 3, z=bits, out=old,
                                              beta=1.0, math=prec, wt=True)
            per = 4 * 3 + 1 / 8  # y, old, new (fp32), bits
    else:
        sc = torch.rand(n, device=dev) + 0.5
        sh = torch.randn(n, device=dev) * 0.1
        fn = lambda: ops.conv_dgrad_bnbwd(dy, wct, (h, h), 1, 0, y, mean, 2, scale=sc, shift=sh,
                                          math=prec, wt=True, g16=bf)
        per = 2 * 2 if bf else 4 * 2   # y, new
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    m = F * h * h
    byt = m * n * per + m * k * dy.element_size() + wct.numel() * wct.element_size()
    return {"kind": kind, "prec": prec, "tiles": bool(ops._TILES[0]), "frames": F, "h": h, "N": n, "K": k, "ms": round(ms, 4),
            "GBps": round(byt / (ms * 1e-3) / 1e9, 1), "TF": round(2.0 * m * n * k / (ms * 1e-3) / 1e12, 1)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=640)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--prec", default="bf16,fp32")
    ap.add_argument("--kinds", default="res,c3,fwd")
    ap.add_argument("--json", default=None)
    ap.add_argument("--tiles", action="store_true",
                    help="one tile per workgroup (TMR_IO_TILES): the launch the wave-specialised "
                         "dgrad replaces")
    args = ap.parse_args()
    if args.tiles:
        ops._TILES[0] = True
    dev = torch.device("cuda:0")
    rows = []
    for prec in args.prec.split(","):
        for kind in args.kinds.split(","):
            for h, n, k in {"res": RES, "c3": C3, "fwd": FWD}[kind]:
                r = run(kind, prec, args.frames, h, n, k, args.reps, dev)
                rows.append(r)
                print(json.dumps(r), flush=True)
                torch.cuda.empty_cache()
    if args.json:
        with open(args.json, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
