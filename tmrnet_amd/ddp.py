"""Data-parallel gradient exchange: one process per GPU, RCCL all-reduce SUM over xGMI.

Replaces torch.nn.DataParallel (train_only_non-local_pretrained.py:628): DP sums
every clip's gradient onto cuda:0 because the loss is CrossEntropyLoss(reduction='sum') over the
global batch, so the exchange here is a SUM (DDP's default would average).  BN statistics stay
per rank, as DP's per-replica BN does.  Gradients are packed into ~25 MB buckets (few, large
collectives suit the per-link-bound xGMI ring) and reduced with the "nccl" (= RCCL) backend.

Overlap: with ``overlap=True`` the reducer registers itself with the model's trunk
(``trunk.set_grad_ready``), which hands over each bottleneck block's final gradients from inside
its backward, deepest block first; their all-reduce then runs while the rest of the backward
does.  The hook is kept in a weak side table, not on the module, so ``copy.deepcopy(model)`` and
``torch.save(model)`` are unaffected.

Semantics kept from torch.optim + DataParallel:
* gradient accumulation (several backwards before ``all_reduce_sum``): an early launch is used
  only when it is exact -- the parameter had no gradient before this backward and no second
  backward touched it since; otherwise the accumulated ``p.grad`` goes through the buckets;
* ``p.grad is None`` stays None when it is None on every rank (torch.optim.SGD then skips the
  parameter); a presence flag per parameter rides in the same bucket, so no extra collective.

Diagnostics (``counts``, ``timing``): launches and bytes per exchange, and with ``timing=True``
the time the compute stream spends from the end of the backward to the reduced gradients being
installed (``exposed_ms()``: the exchange's cost the overlap did not hide; events on the compute
stream, no host synchronisation inside the step).
"""
import warnings

import torch

_flatten = torch._utils._flatten_dense_tensors
_unflatten = torch._utils._unflatten_dense_tensors


class GradAllReduce:
    def __init__(self, model, dist, bucket_bytes=25 * 1024 * 1024, broadcast_init=True,
                 overlap=True, force=False):
        """force: run the collectives even at world size 1 (a one-rank RCCL communicator: lets a
        one-GPU box exercise the exchange path -- streams, early launches, waits -- on RCCL)."""
        self.dist = dist
        self.force = bool(force)
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
        self.early = []         # (params, flat, handle) launched during the backward
        self.early_ids = set()  # params whose reduced gradient an early launch will deliver
        self.stale_ids = set()  # early-launched params touched again by a later backward
        self.overlap = bool(overlap) and self._multi()
        self._warned_accum = False
        self.counts = {"reduces": 0, "early_launches": 0, "bucket_launches": 0, "bytes": 0}
        self.timing = False
        self._events = []       # (start, end) CUDA events around each exchange's waits
        share = getattr(model, "share", None)
        if self.overlap and share is not None:
            from .trunk import set_grad_ready
            set_grad_ready(share, self.grads_ready)

    def _multi(self):
        return self.dist is not None and (self.force or self.dist.get_world_size() > 1)

    def grads_ready(self, pairs):
        """Launch the SUM of some final gradients while the backward is still running.

        `pairs` = [(param, grad)]: this backward's gradient of each param, final for this
        backward (the trunk calls this once per bottleneck block, TrunkFn.backward).  The grads
        are packed into a fresh buffer on the compute stream, so autograd may still steal them
        into `p.grad`; all_reduce_sum() waits and installs the reduced values.  Every rank runs
        the same sequence of backwards, so the launch decisions below agree across ranks."""
        if not self._multi() or not pairs:
            return
        params = [p for p, _ in pairs]
        ids = [id(p) for p in params]
        # a second backward before all_reduce_sum: the earlier launch holds one micro-batch only
        if any(i in self.early_ids for i in ids):
            self.stale_ids.update(i for i in ids if i in self.early_ids)
            return
        # accumulating into an existing gradient: the launch would miss the earlier part
        if any(p.grad is not None for p in params):
            if not self._warned_accum:
                self._warned_accum = True
                warnings.warn("GradAllReduce: trunk gradients already exist at backward time "
                              "(zero_grad(set_to_none=False) or gradient accumulation), so the "
                              "backward/all-reduce overlap is off for them; use "
                              "optimizer.zero_grad(set_to_none=True) to keep it", RuntimeWarning)
            return
        flat = _flatten([g for _, g in pairs])
        self.early.append((params, flat, self.dist.all_reduce(flat, async_op=True)))
        self.early_ids.update(ids)
        self.counts["early_launches"] += 1
        self.counts["bytes"] += flat.numel() * flat.element_size()

    def reset(self):
        """Drop (after waiting for) early launches of a backward that is not being reduced."""
        for _, _, h in self.early:
            h.wait()
        self.early, self.early_ids, self.stale_ids = [], set(), set()

    def all_reduce_sum(self):
        if not self._multi():
            return
        early, stale = self.early, self.stale_ids
        done = self.early_ids - stale
        self.early, self.early_ids, self.stale_ids = [], set(), set()
        handles = []
        for bucket in self.buckets:
            bucket = [p for p in bucket if id(p) not in done]
            if not bucket:
                continue
            grads = [p.grad if p.grad is not None else torch.zeros_like(p) for p in bucket]
            local = [p.grad is not None for p in bucket]
            if all(local):   # the common case: no host round trip
                present = torch.ones(len(bucket), dtype=grads[0].dtype, device=grads[0].device)
            else:
                present = torch.tensor([float(v) for v in local],
                                       dtype=grads[0].dtype).to(grads[0].device)
            flat = _flatten(grads + [present])
            handles.append((bucket, grads + [present], flat, all(local),
                            self.dist.all_reduce(flat, async_op=True)))
            self.counts["bucket_launches"] += 1
            self.counts["bytes"] += flat.numel() * flat.element_size()
        self.counts["reduces"] += 1
        ev = None
        if self.timing and torch.cuda.is_available() and self.params and self.params[0].is_cuda:
            ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            ev[0].record()
        for params, flat, h in early:
            h.wait()
            for p, g in zip(params, _unflatten(flat, params)):
                if id(p) not in stale:          # stale ones were reduced again from p.grad
                    p.grad = g
        for bucket, like, flat, all_local, h in handles:
            h.wait()
            outs = _unflatten(flat, like)
            # every local grad present -> every sum >= 1; read the flags only otherwise
            present = [1.0] * len(bucket) if all_local else outs[-1].tolist()
            for p, g, n in zip(bucket, outs[:-1], present):
                if n == 0:
                    p.grad = None                   # no rank produced a gradient
                elif p.grad is None:
                    p.grad = g
                else:
                    p.grad.copy_(g)
        if ev is not None:
            ev[1].record()
            self._events.append(ev)

    def exposed_ms(self, clear=True):
        """Per exchange since the last call (timing=True): milliseconds of the compute stream from
        the end of the backward to the reduced gradients being installed.  Synchronises."""
        if not self._events:
            return []
        self._events[-1][1].synchronize()
        out = [a.elapsed_time(b) for a, b in self._events]
        if clear:
            self._events = []
        return out
