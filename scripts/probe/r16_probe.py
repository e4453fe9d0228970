"""Timing of the bf16 residual-gradient dgrads (R16: mask 1 from z, bf16 old dx accumulated in
place, bf16 masked output, BN partials of the rounded values) at the ResNet-50 conv1 shapes, as
the C5 step runs them.  Tile config / epilogue depth experiments: TMR_GEMM16_CFG, TMR_LIB_PATH.

usage: python scripts/probe/r16_probe.py [frames]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from tmrnet_amd import ops  # noqa: E402


def main():
    F = int(sys.argv[1]) if len(sys.argv) > 1 else 1920
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    tot = 0.0
    for (h, cin, cout, cnt) in ((56, 256, 64, 2), (56, 256, 128, 1), (28, 512, 128, 3),
                                (14, 1024, 256, 5), (7, 2048, 512, 2)):
        bf = torch.bfloat16
        dy = torch.randn(F, h, h, cout, device=dev, generator=g).to(bf)
        wt = ops.weight_to_crsk(torch.randn(cout, cin, 1, 1, device=dev, generator=g) / cin ** 0.5)
        y = torch.randn(F, h, h, cin, device=dev, generator=g).to(bf)
        z = (torch.rand(F, h, h, cin, device=dev, generator=g) - 0.3).to(bf)
        dx = torch.randn(F, h, h, cin, device=dev, generator=g).to(bf)
        mean = torch.randn(cin, device=dev, generator=g)
        run = lambda: ops.conv_dgrad_bnbwd(dy, wt, (h, h), 1, 0, y, mean, 1, z=z, out=dx, beta=1.0,
                                           math="bf16", wt=True, g16=True)
        run()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            run()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 10
        gb = F * h * h * (2 * cout + 8 * cin) / 1e9
        tot += ms * cnt
        print("dgrad_r16 %3d %4d<-%4d x%d %7.3f ms %6.0f GB/s" % (h, cin, cout, cnt, ms, gb / ms * 1e3),
              flush=True)
    print("TOTAL %.2f ms  cfg=%s lib=%s" % (tot, os.environ.get("TMR_GEMM16_CFG", "auto"),
                                            os.environ.get("TMR_LIB_PATH", "default")))


if __name__ == "__main__":
    main()
