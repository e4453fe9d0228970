"""Run one bf16 LDS-DMA conv launch shape repeatedly (PMC / trace target).
usage: python scripts/one_conv.py KIND N H W CIN COUT R STRIDE PAD [reps]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tmrnet_amd import ops  # noqa: E402


def main():
    kind = sys.argv[1]
    n, h, w, cin, cout, r, st, pad = [int(v) for v in sys.argv[2:10]]
    reps = int(sys.argv[10]) if len(sys.argv) > 10 else 20
    dev = torch.device("cuda:0")
    x = (torch.rand(n, h, w, cin, device=dev) * 2 - 1).to(torch.bfloat16)
    wo = torch.randn(cout, cin, r, r, device=dev) * 0.05
    wk, wt = ops.weight_to_krsc(wo, bf16=True), ops.weight_to_crsk(wo)
    y = ops.conv_fwd(x, wk, st, pad, math="bf16")
    dy = (torch.rand_like(y) * 2 - 1).to(torch.bfloat16)
    for _ in range(reps):
        if kind == "fwd":
            ops.conv_fwd(x, wk, st, pad, out=y, math="bf16")
        elif kind == "dgrad":
            ops.conv_dgrad(dy, wt, (h, w), st, pad, math="bf16", wt=True)
        else:
            ops.conv_wgrad(x, dy, r, r, st, pad, math="bf16")
    torch.cuda.synchronize()
    print("done", kind, n, h, w, cin, cout, r, st, pad)


if __name__ == "__main__":
    main()
