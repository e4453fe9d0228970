"""The data-parallel train step end to end on the GPU: bench.py at world size 2, both ranks on
cuda:0 with the gloo backend (RCCL needs one GPU per rank; the 8-GPU RCCL run is the driver's).
Exercises rank-0 weight broadcast, the bucketed gradient SUM (tmrnet_amd.ddp.GradAllReduce), the
barrier/max-over-ranks timing and the rank-0 JSON line (train_only_non-local_pretrained.py:628,
DataParallel -> one process per GPU)."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_bench_two_ranks_one_gpu():
    # plain `bench.py --gpus 2`: bench.py launches its own two ranks (the driver's 1->8 run may
    # call it without a launcher); rehearsal knobs put both ranks on cuda:0 over gloo
    env = dict(os.environ, TMR_BENCH_DEVICE="0", TMR_BENCH_DIST_BACKEND="gloo",
               HSA_ENABLE_IPC_MODE_LEGACY="0")
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, "bench.py", "--gpus", "2",
           "--steps", "2", "--warmup", "1", "--clips", "2", "--no-cpu-baseline", "--no-roofline"]
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]      # rank 0 prints exactly one line
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["global_batch"] == 4
    assert d["config"]["parallelism"] == "dp2" and d["value"] > 0
    # what the communicator saw: two ranks, an all-reduce of ones = 2 (bench.check_ranks)
    assert d["config"]["ranks_seen"] == {"world_size": 2, "backend": "gloo", "allreduce_ones": 2}
    assert d["loss_last"] == d["loss_last"]       # finite
    # the per-rank diagnostics an 8-GPU line is read by (bench.rank_diagnostics)
    r = d["ranks"]
    for k in ("wall_ms_per_step", "step_ms_min", "step_ms_mean", "step_ms_max",
              "allreduce_wait_ms", "allreduce_wait_ms_max"):
        assert len(r[k]) == 2 and all(v >= 0 for v in r[k]), (k, r[k])
    assert all(a <= b <= c for a, b, c in zip(r["step_ms_min"], r["step_ms_mean"],
                                              r["step_ms_max"]))
    assert r["early_launches_per_step"] == 16             # one per bottleneck block
    assert r["bucket_launches_per_step"] >= 1
    # every parameter's gradient travels once per step (+ the bucket presence flags)
    assert 115 <= r["allreduce_mb_per_step"] <= 117, r["allreduce_mb_per_step"]


def test_overlap_matches_post_backward():
    """Trunk grads launched per block during the backward sum to the same values as the
    all-after-backward buckets (a block handed over too early, or skipped, would differ ~2x)."""
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           "tests/_ddp_overlap_worker.py"]
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    line = [l for l in p.stdout.splitlines() if l.startswith("OVERLAP_REL_DIFF")]
    assert len(line) == 1, p.stdout[-2000:]
    f = line[0].split()
    worst, n, early_off, early_on = float(f[1]), int(f[2]), int(f[3]), int(f[4])
    assert early_off == 0 and early_on == 16, line[0]    # one launch per bottleneck block
    assert n > 100 and worst < 1e-5, line[0]


def test_overlap_on_rccl_one_rank():
    """The overlapped exchange on the production backend: one rank over RCCL ("nccl"), the
    collectives forced at world size 1 (GradAllReduce(force=True)) -- all-reduces issued from the
    autograd thread during TrunkFn.backward, waited on the main thread.  A one-rank sum is the
    identity, so both schedules must return the local gradients bit-exactly."""
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", TMR_TEST_BACKEND="nccl")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           "tests/_ddp_overlap_worker.py"]
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    line = [l for l in p.stdout.splitlines() if l.startswith("OVERLAP_REL_DIFF")]
    assert len(line) == 1, p.stdout[-2000:]
    f = line[0].split()
    worst, early_off, early_on = float(f[1]), int(f[3]), int(f[4])
    assert worst == 0.0 and early_off == 0 and early_on == 16, line[0]
