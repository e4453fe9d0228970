"""Data-parallel gradient exchange: one process per GPU, RCCL all-reduce SUM over xGMI.

Replaces torch.nn.DataParallel (train_only_non-local_pretrained.py:628): DP sums
every clip's gradient onto cuda:0 because the loss is CrossEntropyLoss(reduction='sum') over the
global batch, so the exchange here is a SUM (DDP's default would average).  BN statistics stay
per rank, as DP's per-replica BN does.  Gradients are packed into ~25 MB buckets (few, large
collectives suit the per-link-bound xGMI ring) and reduced with the "nccl" (= RCCL) backend.
The trunk's gradients are launched block by block from inside its backward (grads_ready), so
their exchange overlaps the remaining backward; the rest go in buckets after the backward.
"""
import torch


class GradAllReduce:
    def __init__(self, model, dist, bucket_bytes=25 * 1024 * 1024, broadcast_init=True):
        self.dist = dist
        self.params = [p for p in model.parameters() if p.requires_grad]
        self.buckets = []
        cur, size = [], 0
        for p in reversed(self.params):         # backward produces grads roughly in this order
            cur.append(p)
            size += p.numel() * p.element_size()
            if size >= bucket_bytes:
                self.buckets.append(cur)
                cur, size = [], 0
        if cur:
            self.buckets.append(cur)
        if broadcast_init and dist is not None:
            with torch.no_grad():
                for p in self.params:
                    dist.broadcast(p, 0)
                for b in model.buffers():
                    dist.broadcast(b, 0)

        self.early = []         # (params, grads, flat, handle) launched during the backward
        self.early_ids = set()

    def grads_ready(self, pairs):
        """Launch the SUM of some final gradients while the backward is still running.

        `pairs` = [(param, grad)] whose grads no later backward work touches (the trunk calls this
        once per bottleneck block, deepest first, TrunkFn.backward).  The grads are packed into a
        fresh buffer on the compute stream, so autograd may still steal or clone them into
        `p.grad`; all_reduce_sum() waits and copies the reduced values into `p.grad`."""
        if self.dist is None or self.dist.get_world_size() == 1 or not pairs:
            return
        params = [p for p, _ in pairs]
        grads = [g for _, g in pairs]
        flat = torch._utils._flatten_dense_tensors(grads)
        self.early.append((params, grads, flat, self.dist.all_reduce(flat, async_op=True)))
        self.early_ids.update(id(p) for p in params)

    def all_reduce_sum(self):
        if self.dist is None or self.dist.get_world_size() == 1:
            return
        handles, early, done = [], self.early, self.early_ids
        self.early, self.early_ids = [], set()
        for bucket in self.buckets:
            bucket = [p for p in bucket if id(p) not in done]
            if not bucket:
                continue
            grads = [p.grad if p.grad is not None else torch.zeros_like(p) for p in bucket]
            flat = torch._utils._flatten_dense_tensors(grads)
            handles.append((bucket, grads, flat, self.dist.all_reduce(flat, async_op=True)))
        for bucket, grads, flat, h in early + handles:
            h.wait()
            for p, g in zip(bucket, torch._utils._unflatten_dense_tensors(flat, grads)):
                if p.grad is None:
                    p.grad = g
                else:
                    p.grad.copy_(g)
