"""Runs the direct 3x3 kernels at C5's layer1 geometry (1920 frames, 56x56, 64 -> 64) and the deep
stem's 112x112 32 -> 64 conv a few times each, for rocprofv3 kernel-trace / PMC passes."""
import sys
import torch
import os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from tmrnet_amd import ops

dev = torch.device("cuda:0")
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
for (n, hw, c, k) in ((1920, 56, 64, 64), (640, 112, 32, 64)):
    x = torch.randn(n, hw, hw, c, device=dev).to(torch.bfloat16)
    w = torch.randn(k, c, 3, 3, device=dev) / 24
    wk = ops.weight_to_krsc(w, bf16=True)
    wt = ops.weight_to_crsk(w)
    dy = torch.randn(n, hw, hw, k, device=dev).to(torch.bfloat16)
    y = torch.randn(n, hw, hw, c, device=dev).to(torch.bfloat16)
    sc, sh, mu = (torch.rand(c, device=dev) + 0.5, torch.randn(c, device=dev), torch.zeros(c, device=dev))
    for _ in range(reps):
        ops.conv_fwd_bnstats(x, wk, 1, 1, math="bf16", y16=True)
        ops.conv_dgrad_bnbwd(dy, wt, (hw, hw), 1, 1, y, mu, 2, scale=sc, shift=sh, math="bf16",
                             wt=True, g16=(hw == 56))
        ops.conv_wgrad(x, dy, 3, 3, 1, 1, math="bf16")
    torch.cuda.synchronize()
    del x, dy, y
print("ok")
