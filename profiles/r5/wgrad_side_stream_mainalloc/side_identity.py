"""One small train step with trunk.WGRAD_SIDE on and off: logits, every gradient and the running
statistics must be bit-identical (the side stream only reorders independent launches)."""
import sys
import torch
sys.path.insert(0, ".")
import tmrnet_amd
from tmrnet_amd import ops, trunk

dev = torch.device("cuda:0")
B, T, L = 2, 5, 7
g = torch.Generator().manual_seed(5)
frames = torch.randint(0, 256, (B * T, 250, 250, 3), generator=g, dtype=torch.uint8).to(dev)
off = torch.randint(0, 27, (B, 2), generator=g, dtype=torch.int32).to(dev)
lt = (torch.rand(B, L, 512, generator=g) * 2 - 1).to(dev)
labels = torch.randint(0, 7, (B,), generator=g).to(dev)
for prec in ("fp32", "bf16"):
    res = {}
    for side in (True, False):
        trunk.WGRAD_SIDE = side
        torch.manual_seed(0)
        m = tmrnet_amd.resnet_lstm(seq_len=T, precision=prec).to(dev).train()
        m.nl_block.forced_mask = torch.ones(B, 512, device=dev)
        m.forced_head_mask = torch.ones(B, 512, device=dev)
        out = m(ops.crop_normalize(frames, off, T), lt)
        tmrnet_amd.CrossEntropyLoss(size_average=False)(out, labels).backward()
        torch.cuda.synchronize()
        res[side] = (out.detach().clone(), {n: p.grad.clone() for n, p in m.named_parameters()})
    assert torch.equal(res[True][0], res[False][0])
    bad = [n for n in res[True][1] if not torch.equal(res[True][1][n], res[False][1][n])]
    assert not bad, bad
    print(prec, "side-stream wgrads bit-identical over", len(res[True][1]), "gradients")
