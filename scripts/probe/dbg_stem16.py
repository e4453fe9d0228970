import sys, os, torch, numpy as np
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import torch.nn.functional as F
from tmrnet_amd import ops
dev = torch.device("cuda:0")
n = 2
g = torch.Generator().manual_seed(14)
x = torch.relu(torch.randn(n, 3, 224, 224, generator=g)) + 0.5
wt = torch.randn(64, 3, 7, 7, generator=g) / np.sqrt(147)
x4 = ops.nchw_to_nhwc(x.to(dev), cpad=4)
wk4 = ops.weight_to_krsc(wt.to(dev).contiguous(), cpad=4, bf16=True)
y, stats, nparts = ops.conv_fwd_bnstats(x4, wk4, 2, 3, c_real=3, math="bf16", y16=True)
torch.cuda.synchronize()
ref = F.conv2d(x.to(torch.bfloat16).double(), wt.to(torch.bfloat16).double(), stride=2, padding=3).permute(0, 2, 3, 1)
yf = y.double().cpu()
ulp = 2.0 ** (torch.floor(torch.log2(ref.abs().clamp_min(1e-30))) - 7)
bad = (yf - ref).abs() > ulp * 1.0001
print("bad count", int(bad.sum()), "of", bad.numel())
idx = bad.nonzero()
print(idx[:20])
for t in idx[:10].tolist():
    print(t, float(yf[tuple(t)]), float(ref[tuple(t)]), float(ulp[tuple(t)]))
# distribution over pixel columns / channels / rows
if len(idx):
    print("ow hist", torch.bincount(idx[:, 2], minlength=112).nonzero().flatten().tolist()[:40])
    print("oh hist", torch.bincount(idx[:, 1], minlength=112).nonzero().flatten().tolist()[:40])
    print("co hist", torch.bincount(idx[:, 3], minlength=64).nonzero().flatten().tolist())
