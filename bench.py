"""Benchmark: TMRNet train step (ResNet50 + LSTM + NLBlock, seq_len=10, LFB=40) on MI355X.

One step = the reference's default training transform (use_flip=1: per-clip RandomCrop, ColorJitter,
flip, RandomRotation, ToTensor, Normalize -- bit-exact to PIL, on the device; --augment crop keeps
only crop+normalize) of B clips x T synthetic 250x250x3 uint8 frames resident in HBM ->
LFB row table (reference rule, on device) -> TMRNet forward (rows read from the resident bank)
-> CE(sum) -> backward -> [RCCL all-reduce SUM of grads when N>1] -> fused SGD step.
This is the per-step work of train_only_non-local_pretrained.py:698-725 (BASELINE.json configs[1],
configs[2] at N=8).  Synthetic data/weights per SURVEY.md §8d (seeds 1-5, torch.manual_seed(0)).

Prints ONE JSON line (rank 0).  Multi-GPU: launched by torch.distributed.run, one rank per GPU,
each rank trains its own B clips (weak scaling), gradients summed across ranks.
"""
import argparse
import json
import os
import platform
import socket
import subprocess
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

MFMA_F32_PEAK_TF = 157.3     # MI355X dense f32 MFMA (guides: 256 CU x 2.4 GHz x 256 FLOP/clk)
MFMA_BF16_PEAK_TF = 2516.6
HBM_PEAK_GBS = 8000.0
# algorithmic train-step GFLOP per frame: 3 x 2 x trunk GMAC (fwd, dgrad, wgrad; no stem dgrad)
# + LSTM/NL/TimeConv/head (oracle.tmrnet_ref.trunk_gmacs_per_frame)
GFLOP_PER_FRAME = {"resnet50": 24.33, "resnest50": 32.3}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--clips", type=int, default=64, help="clips per rank (reference batch)")
    ap.add_argument("--seq", type=int, default=10)
    ap.add_argument("--lfb", type=int, default=40)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--conv-table", action="store_true", help="per-launch conv table on stderr")
    ap.add_argument("--cpu-clips", type=int, default=4)
    ap.add_argument("--cpu-steps", type=int, default=5)
    ap.add_argument("--cpu-warmup", type=int, default=2)
    ap.add_argument("--augment", choices=["reference", "crop"], default="reference",
                    help="reference = the scripts' default train transform (use_flip=1, "
                         "train_only_non-local_pretrained.py:342-350) on the device; crop = "
                         "RandomCrop + Normalize only")
    ap.add_argument("--model", choices=["resnet50", "resnest50"], default="resnet50",
                    help="resnest50 = C4 model (ResNeSt50 + TimeConv head, fp32 here); the "
                         "metric line is defined on resnet50")
    ap.add_argument("--precision", choices=["fp32", "bf16"], default="fp32",
                    help="trunk conv operand precision (bf16 = configs C4/C5; the metric "
                         "line's config C2 is fp32)")
    return ap.parse_args()


def launch_ranks(args):
    """`bench.py --gpus N` without a launcher: start N ranks with torch.distributed.run as a
    child process (this process has not touched the GPU) and exit with its status."""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           "--nproc-per-node", str(args.gpus), "--master-addr", "127.0.0.1",
           "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    return subprocess.call(cmd, env=env)


def synth_inputs(args, rank, world, dev, nvar=2):
    B, T, L = args.clips, args.seq, args.lfb
    # LFB geometry of SURVEY.md §8d: 40 videos x 2500 frames
    lengths = [2500] * 40
    from tmrnet_amd.lfb import valid_starts
    from tmrnet_amd.sampler import ClipSampler
    vs = valid_starts(T, lengths)
    g1 = torch.Generator().manual_seed(1)
    frames = [torch.randint(0, 256, (B * T, 250, 250, 3), generator=g1, dtype=torch.uint8).to(dev)
              for _ in range(nvar)]
    g3 = torch.Generator().manual_seed(3)
    bank = (torch.rand(len(vs), 512, generator=g3) * 2 - 1).to(dev)
    vs_d = torch.tensor(vs, dtype=torch.int64, device=dev)
    steps = args.warmup + args.steps + 2
    g2 = torch.Generator().manual_seed(2 + 1000 * rank)
    offs = torch.randint(0, 27, (steps, B, 2), generator=g2, dtype=torch.int32).to(dev)
    # rank-disjoint clips: one shuffled start list shared by all ranks (seed 4), global batch i
    # split into per-rank chunks as DataParallel scatters it (tmrnet_amd.sampler.ClipSampler)
    sampler = ClipSampler(vs, B, rank, world, seed=4)
    if steps > sampler.steps_per_epoch():
        raise SystemExit("bench: %d steps exceed one epoch of %d global batches"
                         % (steps, sampler.steps_per_epoch()))
    perm = sampler.permutation(0)
    starts = torch.from_numpy(np.stack([sampler.batch(i, perm=perm) for i in range(steps)]))
    starts = starts.to(torch.int64).to(dev)
    g5 = torch.Generator().manual_seed(5 + 1000 * rank)
    labels = torch.randint(0, 7, (steps, B), generator=g5).to(dev)
    return frames, bank, vs_d, offs, starts, labels


def _dump_maps_at_exit(path):
    """Diagnostics: write /proc/self/maps at interpreter exit (TMR_EXIT_MAPS=path), so a fault
    in a native exit handler can be attributed to a library from its PC."""
    import atexit

    def dump():
        with open("/proc/self/maps") as f, open(path, "w") as g:
            g.write(f.read())
    atexit.register(dump)


def main():
    args = parse()
    if os.environ.get("TMR_EXIT_MAPS"):
        _dump_maps_at_exit(os.environ["TMR_EXIT_MAPS"])
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world:
        print("bench: --gpus %d but WORLD_SIZE %d (launch with --nproc-per-node equal to --gpus)"
              % (args.gpus, world), file=sys.stderr)
        sys.exit(2)
    # rehearsal knobs (a multi-rank run on a one-GPU box): TMR_BENCH_DEVICE pins every rank to
    # one device, TMR_BENCH_DIST_BACKEND=gloo replaces RCCL (which needs one GPU per rank)
    dev = torch.device("cuda", int(os.environ.get("TMR_BENCH_DEVICE", local)))
    torch.cuda.set_device(dev)
    dist = None
    if world > 1:
        import torch.distributed as dist
        backend = os.environ.get("TMR_BENCH_DIST_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
    ranks_seen = check_ranks(dist, world, dev)

    import tmrnet_amd
    from tmrnet_amd import ops, LFBRows
    from tmrnet_amd.ddp import GradAllReduce
    from tmrnet_amd.optim import sgd_param_groups

    torch.manual_seed(0)
    if args.model == "resnet50":
        model = tmrnet_amd.resnet_lstm(seq_len=args.seq, precision=args.precision).to(dev).train()
    else:
        model = tmrnet_amd.resnet_lstm(seq_len=args.seq, time_conv=True, backbone="resnest50",
                                       precision=args.precision).to(dev).train()
    lr = 5e-7  # reference default (-l 5e-7), groups at lr/10 and lr (:646-655)
    opt = tmrnet_amd.SGD(sgd_param_groups(model, lr), lr=lr / 10, momentum=0.9,
                         weight_decay=5e-4)
    crit = tmrnet_amd.CrossEntropyLoss(size_average=False)
    # trunk grads are exchanged block by block during the backward unless TMR_DDP_OVERLAP=0
    reducer = (GradAllReduce(model, dist, overlap=os.environ.get("TMR_DDP_OVERLAP", "1") != "0")
               if dist is not None else None)
    frames, bank, vs_d, offs, starts, labels = synth_inputs(args, rank, world, dev)
    B, T, L = args.clips, args.seq, args.lfb
    from tmrnet_amd.augment import ClipAugment
    aug = ClipAugment(seq_len=T, use_flip=1) if args.augment == "reference" else None

    def step(i):
        opt.zero_grad(set_to_none=True)
        if aug is not None:
            x4 = aug(frames[i % len(frames)])
        else:
            x4 = ops.crop_normalize(frames[i % len(frames)], offs[i], T)
        rows = ops.lfb_index(vs_d, starts[i], L)
        out = model(x4, LFBRows(bank, rows))
        loss = crit(out, labels[i])
        loss.backward()
        if reducer is not None:
            reducer.all_reduce_sum()
        opt.step()
        return loss

    for i in range(args.warmup):
        step(i)
    torch.cuda.synchronize()
    if reducer is not None:
        reducer.timing = True
        c0 = dict(reducer.counts)
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    # per-step events on the compute stream (no host sync inside the timed region): the per-rank
    # step-time spread of the diagnostics below
    marks = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
    t0 = time.perf_counter()
    marks[0].record()
    for i in range(args.warmup, args.warmup + args.steps):
        loss = step(i)
        marks[i - args.warmup + 1].record()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    diag = rank_diagnostics(dist, world, dev, elapsed, marks, reducer,
                            c0 if reducer is not None else None, args.steps)
    if dist is not None:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
    frames_total = B * T * world * args.steps
    fps = frames_total / elapsed
    ms = elapsed / args.steps * 1e3
    loss_v = float(loss.item())

    # ---- live roofline of the dominant kernel family (implicit-GEMM conv) ----
    roof = None
    # the committed PMC passes profile the default geometry (64 clips x 10 frames, L=40)
    traffic = (load_traffic(args.model, args.precision, args.seq, args.lfb)
               if args.clips == 64 else None)
    stale = bool(traffic and traffic.get("stale"))
    if stale:
        traffic_src = traffic
        traffic = None
    if not args.no_roofline:
        ops.PROF = []
        torch.cuda.synchronize()
        i = args.warmup + args.steps
        step(i)
        torch.cuda.synchronize()
        recs, ops.PROF = ops.PROF, None
        tot_ms = sum(r[2].elapsed_time(r[3]) for r in recs)
        tot_flops = sum(r[1] for r in recs)
        tot_bytes = sum(r[5] for r in recs)
        if args.conv_table and rank == 0:
            for kind, f, e0, e1, shp, nb in recs:
                t = e0.elapsed_time(e1)
                print("%-10s %-34s %8.3f ms %7.1f TF %7.0f GB/s" % (kind, shp, t, f / (t * 1e-3) / 1e12,
                                                                    nb / (t * 1e-3) / 1e9),
                      file=sys.stderr)
        achieved = tot_flops / (tot_ms * 1e-3) / 1e12
        per_kind = {}
        for kind, f, e0, e1, _, _ in recs:
            a = per_kind.setdefault(kind, [0, 0.0, 0.0])
            a[0] += 1; a[1] += f; a[2] += e0.elapsed_time(e1)
        peak = MFMA_F32_PEAK_TF if args.precision == "fp32" else MFMA_BF16_PEAK_TF
        roof = {"bound": "mfma",
                "kernel": ("gemm16_kernel (LDS-DMA implicit-GEMM conv fwd/dgrad/wgrad, %s MFMA; "
                           "gemm16_par_kernel: strided dgrads; dgrad_ws_kernel: the 1x1 residual "
                           "dgrads)%s"
                           % ("f32" if args.precision == "fp32" else "bf16 operands, f32 acc",
                              " + stem_fwd_k / stem_wgrad_k (direct fp32 7x7 stem)"
                              if args.precision == "fp32" else "")),
                "achieved": round(achieved, 2), "peak": peak, "unit": "TFLOP/s",
                "frac": round(achieved / peak, 4),
                # HBM bytes per conv call (PMC, per step / calls per step), same unit as achieved
                "traffic": int(traffic["hbm_bytes_per_step"] / len(recs)) if traffic else None,
                "traffic_source": (traffic or (traffic_src if stale else {})).get("source"),
                # the committed PMC record was collected on a different build of libtmr.so
                "traffic_stale": stale,
                "build_sha": lib_sha(),
                # SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs) over the conv
                # launches of the same committed PMC record
                "mfma_busy_frac": traffic.get("mfma_busy_frac") if traffic else None,
                "alg_bytes_per_launch": int(tot_bytes / max(1, len(recs))),
                "flops_per_launch": int(tot_flops / max(1, len(recs))),
                "launches": len(recs), "avg_launch_ms": round(tot_ms / max(1, len(recs)), 4),
                "conv_ms_per_step": round(tot_ms, 2),
                "per_kind": {k: {"launches": v[0], "tflops": round(v[1] / (v[2] * 1e-3) / 1e12, 2),
                                 "ms": round(v[2], 2)} for k, v in per_kind.items()},
                "step_mfma_frac": round(fps / world * GFLOP_PER_FRAME.get(args.model, 0.0) * 1e9 /
                                        (peak * 1e12), 4)}
        # per-launch roofline: each launch bound by max(FLOPs / MFMA peak, algorithmic bytes /
        # HBM peak) -- the short-reduction convs and the fused BN-backward dgrads are HBM-bound, so
        # `frac` (all FLOPs against the MFMA peak) understates how close the family is to its roof
        att_ms = sum(max(r[1] / (peak * 1e12), r[5] / (HBM_PEAK_GBS * 1e9)) for r in recs) * 1e3
        roof["attainable_ms"] = round(att_ms, 2)
        roof["attainable_frac"] = round(att_ms / tot_ms, 4) if tot_ms > 0 else None
        roof["hbm_bound_launches"] = sum(
            1 for r in recs if r[5] / (HBM_PEAK_GBS * 1e9) > r[1] / (peak * 1e12))

    # whole-step HBM fraction: SURVEY.md §8d's activation-traffic model
    # (4 touches x 32.0 M activation elements per frame x dtype bytes) and the measured PMC bytes
    # of every kernel of a step (committed profile of this workload), both over the step time
    act_bytes = 4 * 32.0e6 * (4 if args.precision == "fp32" else 2)
    hbm = {"model_bytes_per_frame": act_bytes,
           "model_frac": round(fps / world * act_bytes / (HBM_PEAK_GBS * 1e9), 4),
           "pmc_bytes_per_step": traffic["all_kernels_bytes_per_step"] if traffic else None,
           "pmc_stale": stale,
           "pmc_frac": (round(traffic["all_kernels_bytes_per_step"] / (ms * 1e-3)
                              / (HBM_PEAK_GBS * 1e9), 4) if traffic else None),
           "peak_gbs": HBM_PEAK_GBS}

    # the CPU baseline runs on rank 0 after the GPU ranks are done (at N > 1 too: north_star asks
    # for the CPU path next to every GPU count), so it never competes with a timed GPU step
    if dist is not None:
        dist.destroy_process_group()
        dist = None
    cpu = None
    if rank == 0 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args)

    if rank == 0:
        print("sgd table uploads: %d over %d steps" % (opt.table_uploads, args.warmup + args.steps),
              file=sys.stderr)
        line = {
            "metric": ("train frames/sec, TMRNet ResNet50 seq=%d LFB=%d" % (T, L)
                       if args.model == "resnet50" else
                       "train frames/sec, TMRNet ResNeSt50+TimeConv seq=%d LFB=%d" % (T, L)),
            "value": round(fps, 2), "unit": "frames/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms, 2), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": args.precision,
            "data": "synthetic (uint8 250x250x3 frames, U(-1,1) LFB bank 99640x512, random-init weights)",
            "config": {"workload": workload_name(args),
                       "model": ("resnet_lstm (train_only_non-local_pretrained)"
                                 if args.model == "resnet50" else
                                 "resnet_lstm (train_non-local_mutiConv_resnest)"),
                       "global_batch": B * world, "clips_per_gpu": B, "seq_len": T, "lfb_len": L,
                       "frames_per_step": B * T * world, "parallelism": "dp%d" % world,
                       "ranks_seen": ranks_seen,
                       "input_transform": ("reference train transform (use_flip=1) on device"
                                           if aug is not None else "crop+normalize")},
            "loss_last": loss_v,
            "ranks": diag,
            "roofline": roof,
            "hbm": hbm,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)


def rank_diagnostics(dist, world, dev, elapsed, marks, reducer, c0, steps):
    """What limits a multi-GPU line, from every rank: its wall time over the
    timed steps, its per-step GPU times (min / mean / max from the stream events), the time its
    compute stream waited on the gradient exchange per step (GradAllReduce.exposed_ms: the part
    of the all-reduce the backward overlap did not hide) and the exchange's launches per step
    (early = the trunk's per-block launches during the backward, 16 expected; buckets = the
    post-backward buckets of the LSTM / NLBlock / head gradients) -> a dict for the JSON line:
    stragglers show as a spread of `step_ms_mean`, RCCL as `allreduce_wait_ms`, input feeding as
    `wall_ms_per_step` above the GPU step time."""
    st = [a.elapsed_time(b) for a, b in zip(marks[:-1], marks[1:])]
    row = [elapsed * 1e3 / steps, min(st), sum(st) / len(st), max(st)]
    if reducer is not None:
        waits = reducer.exposed_ms()
        c = {k: reducer.counts[k] - c0[k] for k in reducer.counts}
        n = max(1, c["reduces"])
        row += [sum(waits) / max(1, len(waits)), max(waits) if waits else 0.0,
                c["early_launches"] / n, c["bucket_launches"] / n, c["bytes"] / n]
        reducer.timing = False
    else:
        row += [0.0, 0.0, 0.0, 0.0, 0.0]
    t = torch.tensor(row, dtype=torch.float64, device=dev)
    if dist is not None:
        if dist.get_backend() != "nccl":
            t = t.cpu()
        allr = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(allr, t)
        rows = [r.tolist() for r in allr]
    else:
        rows = [t.tolist()]
    means = [r[2] for r in rows]
    return {"wall_ms_per_step": [round(r[0], 3) for r in rows],
            "step_ms_min": [round(r[1], 3) for r in rows],
            "step_ms_mean": [round(r[2], 3) for r in rows],
            "step_ms_max": [round(r[3], 3) for r in rows],
            "step_ms_spread": round(max(means) - min(means), 3),
            "allreduce_wait_ms": [round(r[4], 3) for r in rows],
            "allreduce_wait_ms_max": [round(r[5], 3) for r in rows],
            "early_launches_per_step": rows[0][6], "bucket_launches_per_step": rows[0][7],
            "allreduce_mb_per_step": round(rows[0][8] / 2 ** 20, 2),
            "exchange": ("none (one rank)" if reducer is None else
                         "%s all-reduce SUM, %d trunk blocks launched during the backward"
                         % ("RCCL" if dist.get_backend() == "nccl" else dist.get_backend(),
                            rows[0][6]))}


def workload_name(args):
    if args.model == "resnest50":
        return ("C4: TMRNet ResNeSt50+LSTM+NLBlock+TimeConv train step, %s convs"
                % args.precision)
    if args.precision == "bf16" or args.seq != 10 or args.lfb != 40:
        return ("C5-style: TMRNet ResNet50+LSTM+NLBlock train step, seq %d, LFB %d, %s convs"
                % (args.seq, args.lfb, args.precision))
    return "C2/C3: TMRNet ResNet50+LSTM+NLBlock train step"


def check_ranks(dist, world, dev):
    """What the communicator actually saw (train_only_non-local_pretrained.py:628 replaces
    DataParallel): world size, backend and one all-reduce SUM of ones, which must equal N.
    A bench line is never printed for fewer ranks than --gpus."""
    if dist is None:
        return {"world_size": 1, "backend": None, "allreduce_ones": 1}
    backend = dist.get_backend()
    t = torch.ones(1, device=dev if backend == "nccl" else "cpu")
    dist.all_reduce(t)
    seen = {"world_size": dist.get_world_size(), "backend": backend,
            "allreduce_ones": int(round(t.item()))}
    if seen["world_size"] != world or seen["allreduce_ones"] != world:
        raise SystemExit("bench: communicator saw %s, expected %d ranks" % (seen, world))
    return seen


def lib_sha():
    """Build stamp of the library this run loaded (scripts/pmc_summary.lib_sha)."""
    import hashlib
    with open(os.path.join(ROOT, "tmrnet_amd", "libtmr.so"), "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()[:16]


def load_traffic(model, precision, seq, lfb):
    """HBM bytes (and MFMA-busy cycles) of the conv kernels per step from the committed rocprofv3
    PMC passes of THIS workload (scripts/pmc.sh -> scripts/pmc_summary.py ->
    profiles/<round>/pmc_traffic_<model>_<precision>_s<seq>_l<lfb>.json: FETCH_SIZE x2 (gfx950
    wide-read correction) + WRITE_SIZE of the conv engines and the split-K reductions, per train
    step; SQ_VALU_MFMA_BUSY_CYCLES / GRBM_GUI_ACTIVE).  Round-2 records (pmc_traffic_<model>[_bf16]
    .json) cover the default geometry only.  None when no PMC pass has been committed."""
    import glob
    names = ["pmc_traffic_%s_%s_s%d_l%d.json" % (model, precision, seq, lfb)]
    if (seq, lfb) == (10, 40):
        names.append("pmc_traffic_%s%s.json" % (model, "" if precision == "fp32" else "_bf16"))
    files = []
    for n in names:
        files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", n)))
        if files:
            break
    if not files:
        return None
    with open(files[-1]) as f:
        d = json.load(f)
    fams = d.get("families", {})
    # the conv family: gemm_kernel / tmrg::gemm_kernel (register-staged), tmrg::gemm16_kernel
    # (LDS-DMA engine) with its one-launch strided dgrads (gemm16_par_kernel, round 5) and the
    # wave-specialised 1x1 dgrads (dgrad_ws_kernel, round 6), the direct stems (stem_fwd_k / stem_wgrad_k, round 3; stem16_*, round 4),
    # the direct 3x3 kernels (d3_k, d3w_k, d3s_k, d3sw_k, round 4) and the split-K weight-gradient
    # reductions
    conv = [k for k in fams
            if any(t in k for t in ("gemm_kernel", "gemm16_kernel", "gemm16_par_kernel",
                                    "dgrad_ws_kernel", "wgrad_reduce", "stem_fwd_k",
                                    "stem_wgrad_k", "stem16_fwd_k", "stem16_wgrad_k", "d3_k",
                                    "d3w_k", "d3s_k", "d3sw_k"))]
    if not conv:
        return None
    if d.get("build_sha") != lib_sha():
        # collected on another build: the bytes and MFMA-busy cycles describe other kernels
        return {"stale": True, "source": os.path.relpath(files[-1], ROOT),
                "record_build_sha": d.get("build_sha")}
    per_step = sum(fams[k]["hbm_bytes_per_step"] for k in conv)
    busy = sum(fams[k].get("mfma_busy_cycles", 0.0) for k in conv)
    gui = sum(fams[k].get("gui_active_cycles", 0.0) for k in conv)
    return {"hbm_bytes_per_step": per_step,
            "all_kernels_bytes_per_step": sum(f["hbm_bytes_per_step"] for f in fams.values()),
            "mfma_busy_frac": round(busy / (gui / 8.0 * 1024.0), 4) if gui > 0 else None,
            "source": os.path.relpath(files[-1], ROOT)}


def cpu_threads():
    """Host threads for the CPU baseline.  BASELINE.md §4 asks for os.cpu_count(); on the GPU box
    that reports the whole host (many times the job's CPU share), so the share is taken from
    OMP_NUM_THREADS (set to it there) or the affinity mask; os.cpu_count() is reported beside."""
    env = os.environ.get("OMP_NUM_THREADS", "")
    if env.isdigit() and int(env) > 0:
        return int(env)
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:
        return os.cpu_count() or 1


def cpu_baseline(args):
    """The CPU oracle (pure-torch restatement of the reference step) on the host cores:
    BASELINE.md §4 -- C1 (memory-bank model, 4 clips x 10) and the C2 model at 4 clips x 10,
    L=40, fp32, 2 warm-up + 5 timed steps each."""
    from oracle import tmrnet_ref as ref
    from tmrnet_amd.optim import sgd_param_groups
    threads = cpu_threads()
    torch.set_num_threads(threads)
    B, T, L = args.cpu_clips, args.seq, args.lfb
    g = torch.Generator().manual_seed(1)
    frames = torch.randint(0, 256, (B * T, 250, 250, 3), generator=g, dtype=torch.uint8)
    off = torch.randint(0, 27, (B, 2), generator=g, dtype=torch.int32)
    lt = torch.rand(B, L, 512, generator=g) * 2 - 1
    labels = torch.randint(0, 7, (B,), generator=g)
    labels_f = torch.randint(0, 7, (B * T,), generator=g)

    def inputs():
        if args.augment == "reference":
            return ref.augment_ref(frames.numpy(), range(B * T), T).view(B, T, 3, 224, 224)
        return ref.crop_normalize_ref(frames, off, T).view(B, T, 3, 224, 224)

    def run(model, one):
        opt = torch.optim.SGD(sgd_param_groups(model, 5e-7), lr=5e-8, momentum=0.9,
                              weight_decay=5e-4)
        for _ in range(args.cpu_warmup):
            one(model, opt)
        t0 = time.perf_counter()
        for _ in range(args.cpu_steps):
            one(model, opt)
        return B * T * args.cpu_steps / (time.perf_counter() - t0)

    def step_c2(m, opt):   # train_only_non-local_pretrained.py:698-725
        ref.train_step_ref(m, opt, inputs(), lt, labels)

    def step_c1(m, opt):   # train_singlenet_phase_1fc.py:545-566: CE on outputs[T-1::T]
        opt.zero_grad()
        out = m(inputs())[T - 1::T]
        loss = ref.ce_sum_ref(out, labels_f[T - 1::T])
        loss.backward()
        opt.step()

    torch.manual_seed(0)
    c2 = run(ref.TMRNetRef(seq_len=T, time_conv=(args.model == "resnest50"),
                           backbone=args.model).train(), step_c2)
    c1 = None
    if args.model == "resnet50":
        torch.manual_seed(0)
        c1 = run(ref.MemoryBankRef(seq_len=T).train(), step_c1)
    model_name = platform.processor() or "unknown"
    try:
        for l in subprocess.check_output(["lscpu"], text=True).splitlines():
            if l.startswith("Model name"):
                model_name = l.split(":", 1)[1].strip()
    except Exception:
        pass
    return {"value": round(c2, 3), "unit": "frames/s", "cores": threads,
            "os_cpu_count": os.cpu_count(), "kind": "port", "cpu": model_name,
            "threads_rule": ("OMP_NUM_THREADS" if os.environ.get("OMP_NUM_THREADS", "").isdigit()
                             else "sched_getaffinity") + " (the job's host share; BASELINE.md "
                            "section 4 names os.cpu_count(), which reports the whole host)",
            "c1_memory_bank_frames_per_s": round(c1, 3) if c1 is not None else None,
            "sample": "oracle fp32 train steps on the host (%s, fwd, CE-sum, bwd, SGD): value = C2 "
                      "model (TMRNetRef) at %d clips x %d frames, L=%d; c1 = memory-bank model "
                      "(MemoryBankRef) at %d x %d; %d timed steps after %d warm-up each"
                      % ("PIL train transform" if args.augment == "reference" else "crop+norm",
                         B, T, L, B, T, args.cpu_steps, args.cpu_warmup)}


if __name__ == "__main__":
    main()
