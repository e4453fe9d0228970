"""Microbenchmark of the implicit-GEMM conv kernels on every distinct ResNet-50 conv shape
(F frames), weighted by how often each shape occurs in one train step.

usage: python scripts/convbench.py [--frames 640] [--reps 5] [--kinds fwd,dgrad,wgrad]
Env TMR_GEMM_CFG=<i> forces a tile config (experiments; see gemm_conv.hip kCfgs).
"""
import argparse
import json
import os
import sys
from collections import Counter

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tmrnet_amd import ops  # noqa: E402


def resnet50_convs(F):
    """(n, h, w, cin, cout, r, stride, pad) of every conv in the trunk, in order."""
    out = [(F, 224, 224, 3, 64, 7, 2, 3)]
    h, cin = 56, 64
    for planes, blocks, stride in ((64, 3, 1), (128, 4, 2), (256, 6, 2), (512, 3, 2)):
        for b in range(blocks):
            s = stride if b == 0 else 1
            out.append((F, h, h, cin, planes, 1, 1, 0))
            out.append((F, h, h, planes, planes, 3, s, 1))
            ho = h // s
            out.append((F, ho, ho, planes, planes * 4, 1, 1, 0))
            if b == 0:
                out.append((F, h, h, cin, planes * 4, 1, s, 0))
            cin, h = planes * 4, ho
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=640)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--kinds", default="fwd,dgrad,wgrad")
    ap.add_argument("--json", default=None)
    ap.add_argument("--stats", action="store_true",
                    help="forward with the fused BatchNorm-statistics epilogue (as the train step)")
    ap.add_argument("--pro", action="store_true",
                    help="operand prologues as the folded train step uses them: BN+ReLU on the X "
                         "operand (fwd, wgrad) and the BN backward on dY (dgrad, wgrad), every "
                         "conv but the stem")
    ap.add_argument("--math", choices=["fp32", "bf16"], default="fp32",
                    help="conv operand precision (bf16 = the C4/C5 configs)")
    ap.add_argument("--io16", action="store_true",
                    help="bf16 math with every operand stored bf16 (x, KRSC w, dy; dgrad reads the "
                         "transposed CRSK copy): the LDS-DMA engine, as the bf16 train step")
    ap.add_argument("--bnbwd", action="store_true",
                    help="dgrad with the fused BN-backward epilogue (ReLU mask from z, per-tile "
                         "partials), as the train step runs every dgrad but the stem's")
    ap.add_argument("--wt32", action="store_true",
                    help="fp32 dgrad on the LDS-DMA engine (transposed fp32 weights, "
                         "TMR_IO_WT_F32), as the fp32 train step")
    ap.add_argument("--y16", action="store_true",
                    help="forward with the fused statistics writing y as bf16 (the bf16-activation "
                         "step, GemmArgs::c16)")
    ap.add_argument("--only", default=None,
                    help="comma list of cin:cout:r:h filters, e.g. 64:256:1:56")
    ap.add_argument("--dgrad-beta", type=float, default=0.0,
                    help="accumulate dgrad into its output (the train step does for conv1/ds)")
    ap.add_argument("--classes", action="store_true",
                    help="strided dgrads as one launch per stride-parity class (TMR_IO_CLASSES, "
                         "the A/B of the one-launch form)")
    args = ap.parse_args()
    if args.classes:
        ops._CLASSES[0] = True
    dev = torch.device("cuda:0")
    shapes = Counter(resnet50_convs(args.frames))
    kinds = args.kinds.split(",")
    res = []
    tot = {k: [0.0, 0.0] for k in kinds}
    only = None
    if args.only:
        only = [tuple(int(v) for v in f.split(":")) for f in args.only.split(",")]
    for shp, cnt in shapes.items():
        n, h, w, cin, cout, r, st, pad = shp
        if only is not None and (cin, cout, r, h) not in only:
            continue
        cs = 4 if cin == 3 else cin
        x = torch.randn(n, h, w, cs, device=dev)
        wk = torch.randn(cout, r, r, cs, device=dev)
        y = ops.conv_fwd(x, wk, st, pad)
        dy = torch.randn_like(y)
        wdg, wt = wk, False
        if args.io16:
            args.math = "bf16"
            wo = torch.randn(cout, cs, r, r, device=dev)
            wk = ops.weight_to_krsc(wo, bf16=True)
            dy = dy.to(torch.bfloat16)
            if cin != 3:   # the stem's 4-channel input stays fp32 (register-staged gather)
                x = x.to(torch.bfloat16)
                wdg, wt = ops.weight_to_crsk(wo), True
            else:
                wdg = wk
        elif args.wt32 and cin != 3:
            wdg, wt = ops.weight_to_crsk(torch.randn(cout, cs, r, r, device=dev), bf16=False), True
        xpro = dpro = None
        if args.pro and cin != 3:
            xpro = (torch.rand(cs, device=dev) + 0.5, torch.randn(cs, device=dev) * 0.1)
            dpro = (torch.randn_like(y), torch.randn(3, cout, device=dev))
        dx = torch.empty(n, h, w, cs, device=dev)
        if args.bnbwd and cin != 3:
            yb, zb = torch.randn_like(dx), torch.rand_like(dx) - 0.3
            meanb = torch.randn(cs, device=dev)
        for kind in kinds:
            if kind == "dgrad" and cin == 3:
                continue
            mt = args.math
            fn = {"fwd": (lambda: ops.conv_fwd_bnstats(x, wk, st, pad, c_real=cin, xpro=xpro,
                                                       math=mt, y16=args.y16))
                  if (args.stats or xpro is not None or args.y16)
                  else (lambda: ops.conv_fwd(x, wk, st, pad, out=y, math=mt)),
                  "dgrad": (lambda: ops.conv_dgrad_bnbwd(dy, wdg, (h, w), st, pad, yb, meanb, 1,
                                                         z=zb, out=dx, beta=args.dgrad_beta,
                                                         math=mt, wt=wt))
                  if args.bnbwd else
                  (lambda: ops.conv_dgrad(dy, wdg, (h, w), st, pad, out=dx,
                                          beta=args.dgrad_beta, dpro=dpro, math=mt, wt=wt)),
                  "wgrad": lambda: ops.conv_wgrad(x, dy, r, r, st, pad, c_real=cin, xpro=xpro,
                                                  dpro=dpro, math=mt)}[kind]
            fn()
            torch.cuda.synchronize()
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.reps):
                fn()
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / args.reps
            flops = 2.0 * n * y.shape[1] * y.shape[2] * cout * r * r * cin
            tf = flops / (ms * 1e-3) / 1e12
            res.append({"kind": kind, "shape": shp, "count": cnt, "ms": ms, "tflops": tf})
            tot[kind][0] += ms * cnt
            tot[kind][1] += flops * cnt
            print("%-6s %-34s x%d %8.3f ms %7.1f TF" % (kind, shp, cnt, ms, tf), flush=True)
    allms = sum(v[0] for v in tot.values())
    allf = sum(v[1] for v in tot.values())
    summ = {k: {"ms": round(v[0], 2), "tflops": round(v[1] / (v[0] * 1e-3) / 1e12, 1)}
            for k, v in tot.items()}
    print("TOTAL per step: %.2f ms, %.1f TF  %s  cfg=%s" % (allms, allf / (allms * 1e-3) / 1e12,
                                                            json.dumps(summ),
                                                            os.environ.get("TMR_GEMM_CFG", "auto")))
    if args.json:
        json.dump({"rows": res, "summary": summ, "total_ms": allms}, open(args.json, "w"))


if __name__ == "__main__":
    main()
