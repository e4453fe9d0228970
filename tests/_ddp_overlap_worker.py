"""Rank body for test_ddp_gpu.test_overlap_matches_post_backward (launched by torch.distributed.run).

One TMRNet train step per rank (different frames per rank), gradients summed twice: once with the
trunk's per-block early launch (GradAllReduce.grads_ready from TrunkFn.backward) and once with all
buckets after the backward.  Rank 0 prints the largest relative difference."""
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    rank = int(os.environ["RANK"])
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    backend = os.environ.get("TMR_TEST_BACKEND", "gloo")
    if backend == "nccl":
        dist.init_process_group("nccl", device_id=dev)
    else:
        dist.init_process_group(backend)
    import tmrnet_amd
    from tmrnet_amd import ops
    from tmrnet_amd.ddp import GradAllReduce
    from tmrnet_amd.trunk import set_grad_ready

    B, T, L = 2, 3, 5
    torch.manual_seed(0)
    m = tmrnet_amd.resnet_lstm(seq_len=T).to(dev).train()
    # a one-rank RCCL run forces the collectives (world size 1 would skip them)
    red = GradAllReduce(m, dist, overlap=False, force=dist.get_world_size() == 1)
    g = torch.Generator().manual_seed(10 + rank)
    frames = torch.randint(0, 256, (B * T, 250, 250, 3), generator=g, dtype=torch.uint8).to(dev)
    off = torch.randint(0, 27, (B, 2), generator=g, dtype=torch.int32).to(dev)
    lt = (torch.rand(B, L, 512, generator=g) * 2 - 1).to(dev)
    labels = torch.randint(0, 7, (B,), generator=g).to(dev)
    m.nl_block.forced_mask = torch.ones(B, 512, device=dev)
    m.forced_head_mask = torch.ones(B, 512, device=dev)
    crit = tmrnet_amd.CrossEntropyLoss(size_average=False)

    launched = []

    def grads(overlap):
        set_grad_ready(m.share, red.grads_ready if overlap else None)
        for p in m.parameters():
            p.grad = None
        loss = crit(m(ops.crop_normalize(frames, off, T), lt), labels)
        loss.backward()
        launched.append(len(red.early))   # per-block launches made inside the backward
        red.all_reduce_sum()
        torch.cuda.synchronize()
        return [p.grad.detach().clone() for p in m.parameters()]

    ref = grads(False)
    ovl = grads(True)
    worst = 0.0
    for a, b in zip(ref, ovl):
        worst = max(worst, ((a - b).abs().max() / a.abs().max().clamp_min(1e-30)).item())
    if rank == 0:
        print("OVERLAP_REL_DIFF %.3g %d %d %d" % (worst, len(ref), launched[0], launched[1]),
              flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
