"""Multi-process (world_size 2, gloo, CPU) check of the data-parallel gradient exchange:
tmrnet_amd.ddp.GradAllReduce must SUM gradients across ranks (the reference's DataParallel
reduce-adds onto cuda:0 under CrossEntropyLoss(reduction='sum')) and
broadcast rank 0's initial weights."""
import os
import socket

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q, early=False):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from tmrnet_amd.ddp import GradAllReduce
    torch.manual_seed(100 + rank)           # different init per rank -> broadcast must fix it
    m = torch.nn.Sequential(torch.nn.Linear(300, 200), torch.nn.Linear(200, 7))
    red = GradAllReduce(m, dist, bucket_bytes=4 * 1024)
    ps = list(m.parameters())
    grads = [torch.full_like(p, float(rank + 1) * (i + 1)) for i, p in enumerate(ps)]
    if early:   # the trunk's per-block launch during the backward (TrunkFn.backward), made
        # before autograd stores the gradients into p.grad (else the launch is skipped)
        red.grads_ready([(p, g.clone()) for p, g in zip(ps[2:], grads[2:])])
    for p, g in zip(ps, grads):
        p.grad = g
    red.all_reduce_sum()
    # numpy copies: torch tensors would travel as shared-memory fds that vanish with the child
    out = [p.grad.numpy().copy() for p in m.parameters()]
    w = [p.detach().numpy().copy() for p in m.parameters()]
    q.put((rank, out, w, len(red.buckets), dict(red.counts)))
    dist.destroy_process_group()


import pytest


@pytest.mark.parametrize("world", [2, 4])
@pytest.mark.parametrize("early", [False, True])
def test_grad_all_reduce_sum_world2(early, world):
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, early)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        rank, grads, weights, nb, counts = q.get(timeout=120)
        res[rank] = (grads, weights, nb, counts)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[0][2] > 1                       # several buckets exercised
    ranks_sum = sum(r + 1 for r in range(world))
    for i, g in enumerate(res[0][0]):
        expect = ranks_sum * (i + 1)           # sum over ranks, not mean
        assert (g == expect).all()
        for r in range(1, world):
            assert (g == res[r][0][i]).all()
    for r in range(1, world):
        for w0, w1 in zip(res[0][1], res[r][1]):
            assert (w0 == w1).all()
    # the exchange's diagnostics (bench.rank_diagnostics): one exchange, the early launch counted,
    # every gradient element (+ one presence flag per bucketed parameter) sent exactly once
    n_el = sum(g.size for g in res[0][0])
    for r in range(world):
        c = res[r][3]
        assert c["reduces"] == 1 and c["early_launches"] == (1 if early else 0), c
        assert c["bucket_launches"] >= 1
        n_flags = 2 if early else 4            # presence flags of the bucketed parameters
        assert c["bytes"] == 4 * (n_el + n_flags), (c, n_el)


def _accum_worker(rank, world, port, q):
    """Two backwards before all_reduce_sum; the early per-block launch of the first must not
    replace the accumulated gradient (ddp.py overwrote it with micro-batch 2 only)."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from tmrnet_amd.ddp import GradAllReduce
    torch.manual_seed(0)
    m = torch.nn.Sequential(torch.nn.Linear(30, 20), torch.nn.Linear(20, 7),
                            torch.nn.Linear(7, 3))
    unused = m[2]
    red = GradAllReduce(m, dist, bucket_bytes=1024, overlap=False)
    ps = list(m.parameters())[:4]
    for mb in range(2):          # micro-batches: what TrunkFn.backward + autograd would do
        local = [torch.full_like(p, float((rank + 1) * (mb + 1) * (i + 1)))
                 for i, p in enumerate(ps)]
        red.grads_ready([(p, g) for p, g in zip(ps[2:], local[2:])])
        for p, g in zip(ps, local):
            p.grad = g.clone() if p.grad is None else p.grad + g
    # unused[2]: grad None on both ranks (stays None); weight of layer 3 present on rank 1 only
    if rank == 1:
        unused.weight.grad = torch.full_like(unused.weight, 5.0)
    red.all_reduce_sum()
    out = [None if p.grad is None else p.grad.numpy().copy() for p in m.parameters()]
    # grads not cleared before the next backward (zero_grad(set_to_none=False)): the early launch
    # is skipped -- with a one-time warning, and no collective is started
    import warnings
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        red.overlap = True
        red.grads_ready([(p, p.grad.clone()) for p in ps[2:]])
        red.grads_ready([(p, p.grad.clone()) for p in ps[2:]])
    warned = [x for x in w if issubclass(x.category, RuntimeWarning)]
    q.put((rank, (out, len(warned), len(red.early))))
    dist.destroy_process_group()


def test_grad_accumulation_and_none_grads_world2():
    world = 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_accum_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        g, nwarn, nearly = res[r]
        assert nwarn == 1 and nearly == 0, (nwarn, nearly)
        for i in range(4):
            # sum over ranks (1, 2) of micro-batches (1, 2): (1+2) * (1+2) * (i+1)
            assert (g[i] == 9.0 * (i + 1)).all(), (r, i, g[i].ravel()[:3])
        assert (g[4] == 5.0).all()          # present on one rank: the sum, not None
        assert g[5] is None                 # None everywhere stays None (SGD skips it)
