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
    ap.add_argument("--ensemble", type=int, default=0,
                    help="K: gradient ensembles over perturbed inputs (bf16: 1-ulp, fp32n: 2^-9)")
    ap.add_argument("--ens-variants", default="bf16n,fp32n")
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
            loss, out, g = bg.grads_of(m, bg.inputs_for(v, x4), lfb, labels, mk)
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
    if a.ensemble:
        ens = {}
        for v in a.ens_variants.split(","):
            # <variant>n: the variant on input frames with +-2^-9 relative noise (one bf16 rounding:
            # a perturbation the bf16 step's own input rounding cannot absorb); else 1 fp32 ulp
            noisy = v.endswith("n") and v[:-1] in bg.VARIANTS
            base = v[:-1] if noisy else v
            gs = []
            t0 = time.time()
            for k in range(2 * a.ensemble):
                with bg.variant(base) as prec:
                    m = bg.make_model(dev, T, backbone, tc, prec, sd)
                    xin = (bg.perturb_rel(x4, 2.0 ** -9, 100 + k) if noisy
                           else bg.perturb_ulp(x4, 100 + k))
                    _, _, g = bg.grads_of(m, xin, lfb, labels, mk)
                del m
                gs.append({n: t.float() for n, t in g.items()})
            ens[v] = gs
            print("ensemble %s: %d samples (%.1f s)" % (v, len(gs), time.time() - t0), flush=True)
        K = a.ensemble
        rec = {}
        names = list(ens)
        for v in names:
            A, B = ens[v][:K], ens[v][K:]
            rec[v + "_self"] = bg.ensemble_stats(A + B, A + B, same=True)   # |g*|^2
            rec[v + "_AB"] = bg.ensemble_stats(A, B)
        for i, v in enumerate(names):
            for w in names[i + 1:]:
                rec[v + "_x_" + w] = bg.ensemble_stats(ens[v], ens[w])
        gref = {n: t.float() for n, t in g_ref.items()}
        for v in names:
            rec[v + "_x_fp32"] = bg.ensemble_stats(ens[v], [gref])
        rec["fp32_norm2"] = bg.ensemble_stats([gref], [gref])
        # smooth-gradient cosine between two variants: <g*_v, g*_w> / sqrt(|g*_v|^2 |g*_w|^2)
        print("group      " + "  ".join("%-22s" % k for k in ("c*(%s,%s)" % (names[0], names[-1]),
                                                                "c1(%s,fp32)" % names[0],
                                                                "c1(%s,fp32)" % names[-1])))
        summ = {}
        for grp in rec["fp32_norm2"]:
            s0, s1 = rec[names[0] + "_self"].get(grp), rec[names[-1] + "_self"].get(grp)
            x = rec[names[0] + "_x_" + names[-1]].get(grp) if len(names) > 1 else None
            c_star = x / (max(s0, 1e-300) * max(s1, 1e-300)) ** 0.5 if (x is not None and s0 > 0
                                                                           and s1 > 0) else None
            summ[grp] = {"c_star": c_star, "self": {v: rec[v + "_self"][grp] for v in names},
                         "x_fp32": {v: rec[v + "_x_fp32"][grp] for v in names},
                         "fp32_norm2": rec["fp32_norm2"][grp]}
            print("%-10s %s" % (grp, c_star))
        with open(os.path.join(a.out, "ensemble_%s_K%d.json" % (tag, K)), "w") as f:
            json.dump({"K": K, "stats": rec, "summary": summ}, f, indent=1)
    if a.lrs:
        traj = {}
        for lr in [float(s) for s in a.lrs.split(",")]:
            for v in a.traj_variants.split(","):
                t0 = time.time()
                with bg.variant(v) as prec:
                    m = bg.make_model(dev, T, backbone, tc, prec, sd)
                    losses = bg.trajectory(m, [(bg.inputs_for(v, x4), lfb, labels)], mk, lr,
                                           a.steps)
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
