"""Measure the bf16 train step's gradients against the fp32 step at the benchmarked size (VERDICT r4
item 1): per parameter group cosine / relative L2 of the weight gradients for every storage
contract variant (tests/_bf16_grads.VARIANTS), plus SGD loss trajectories.

  python scripts/bf16_grad_study.py --geo c5 --frames noise --variants fp32,fp32p,bf16 \
      --lrs 1e-4 --steps 20 --out gpurun_out/bf16_grads
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests import _bf16_grads as bg  # noqa: E402

GEOS = {"c5": ("resnet50", False, 30, 300), "c4": ("resnest50", True, 10, 40),
        "c2": ("resnet50", False, 10, 40)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--geo", default="c5")
    ap.add_argument("--frames", default="noise")
    ap.add_argument("--B", type=int, default=64)
    ap.add_argument("--variants", default="fp32,fp32p,bf16,bf16_g16off,bf16_r16off,bf16_actoff")
    ap.add_argument("--lrs", default="")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--traj-variants", default="fp32,bf16")
    ap.add_argument("--out", default="gpurun_out/bf16_grads")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    backbone, tc, T, L = GEOS[a.geo]
    os.makedirs(a.out, exist_ok=True)
    tag = "%s_%s_B%d" % (a.geo, a.frames, a.B)
    x4, lfb, labels = bg.full_inputs(dev, a.B, T, L, a.frames)
    mk = bg.masks(a.B, 6)
    sd = None
    res = {"geo": a.geo, "frames": a.frames, "B": a.B, "T": T, "L": L, "variants": {}}
    g_ref = None
    for v in a.variants.split(","):
        t0 = time.time()
        with bg.variant(v) as prec:
            m = bg.make_model(dev, T, backbone, tc, prec, sd)
            if sd is None:
                sd = {k: t.detach().clone() for k, t in m.state_dict().items()}
            xin = bg.perturb_ulp(x4) if v == "fp32p" else x4
            loss, out, g = bg.grads_of(m, xin, lfb, labels, mk)
        del m
        torch.cuda.empty_cache()
        if g_ref is None:
            g_ref, out_ref, loss_ref = g, out, loss
            print("%s %s: loss %.4f (%.1f s)" % (tag, v, loss, time.time() - t0), flush=True)
            continue
        groups, per = bg.compare(g, g_ref)
        worst = sorted(per.items(), key=lambda kv: kv[1]["cos"])[:8]
        res["variants"][v] = {"loss": loss, "loss_ref": loss_ref,
                              "logit_rel": ((out - out_ref).abs().max() /
                                            out_ref.abs().max()).item(),
                              "groups": groups, "worst_params": worst, "per_param": per}
        print("%s %s: loss %.4f vs %.4f (%.1f s)" % (tag, v, loss, loss_ref, time.time() - t0))
        for k, s in groups.items():
            print("   %-10s cos %.4f  rel_l2 %.4f" % (k, s["cos"], s["rel_l2"]))
        sys.stdout.flush()
    with open(os.path.join(a.out, "grads_%s.json" % tag), "w") as f:
        json.dump(res, f, indent=1)
    if a.lrs:
        traj = {}
        batches = [(x4, lfb, labels)]
        for lr in [float(s) for s in a.lrs.split(",")]:
            for v in a.traj_variants.split(","):
                t0 = time.time()
                with bg.variant(v) as prec:
                    m = bg.make_model(dev, T, backbone, tc, prec, sd)
                    losses = bg.trajectory(m, batches, mk, lr, a.steps)
                del m
                torch.cuda.empty_cache()
                traj["%s_lr%g" % (v, lr)] = losses
                print("traj %s lr %g (%.1f s): %s" % (v, lr, time.time() - t0,
                                                       " ".join("%.3f" % x for x in losses)),
                      flush=True)
        with open(os.path.join(a.out, "traj_%s.json" % tag), "w") as f:
            json.dump(traj, f, indent=1)


if __name__ == "__main__":
    main()
