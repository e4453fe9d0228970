"""Generate tests/golden/bf16_ensemble_<geo>.npz / .json: the CPU side of the bf16 gradient
contract check (DESIGN.md §2 "bf16 gradients", §16).

For one train step at a host-runnable geometry (tests/_bf16_ensemble.GEOS: ResNet-50 B=4 x T=10,
L=40; ResNeSt-50 + TimeConv B=2 x T=10, L=40), the fp32 oracle (oracle.TMRNetRef, the reference's
arithmetic) and its float emulation of the bf16 contract (oracle.emulate_bf16_convs(activations=
True, grads=True): what libtmr.so's bf16 step is specified to compute) each run an ensemble of N
samples over +-2^-9 relative input noise (the same signs the GPU test draws).  Every sample's
weight gradients are reduced to per-group Gram matrices over all samples of all variants; the
fixture holds those matrices (float64) and the statistics derived from them.

Attribution variants (ResNet-50 only; which rounding of the contract shrinks the expected
gradient): operand rounding without the storage roundings, forward operands only, backward
operands only, the output gradient dy only, and the fp32 step at larger input noise (2^-7, 2^-5:
is the bf16 step's expected gradient the fp32 step's smoothed over a larger perturbation?).

Run: python -m tests.golden.make_bf16_ensemble [geo ...]   (about 12 min for r50 on 8 threads)
"""
import json
import os
import sys
import time

import numpy as np
import torch

from oracle import tmrnet_ref as ref
from tests import _bf16_ensemble as E

HERE = os.path.dirname(os.path.abspath(__file__))
N = 8
# variant -> (precision, bf16_act, emulate ops or None, input noise eps)
VARIANTS = {
    "fp32": ("fp32", None, None, E.EPS),
    "bf16": ("bf16", True, None, E.EPS),
    "bf16_ops": ("bf16", False, None, E.EPS),
    "fwd_ops": ("bf16", False, ("fx", "fw"), E.EPS),
    "bwd_ops": ("bf16", False, ("dy", "bx", "bw"), E.EPS),
    "dy_only": ("bf16", False, ("dy",), E.EPS),
    "fp32_e7": ("fp32", None, None, 2.0 ** -7),
    "fp32_e5": ("fp32", None, None, 2.0 ** -5),
}
PER_GEO = {"r50": list(VARIANTS), "rst": ["fp32", "bf16", "fp32_e7"]}


def model(geo, v, sd):
    backbone, tc, B, T, L, _, _ = E.GEOS[geo]
    prec, act, ops, _ = VARIANTS[v]
    r = ref.TMRNetRef(seq_len=T, backbone=backbone, time_conv=tc)
    r.load_state_dict(sd)
    if prec == "bf16":
        ref.emulate_bf16_convs(r.share, activations=act, ops=ops or ref.ROUND_ALL)
    return r.train()


def sample(r, geo, x, lt, labels, masks, k, eps):
    backbone, tc, B, T, L, _, _ = E.GEOS[geo]
    g = torch.Generator().manual_seed(1000 + k)
    s = torch.randint(0, 2, x.shape, generator=g).to(x.dtype) * 2 - 1
    xk = x * (1 + eps * s)
    if eps == E.EPS:
        assert torch.equal(xk, E.noisy(x, k))
    r.zero_grad(set_to_none=True)
    out = r(xk.view(B, T, 3, 224, 224), lt, masks=masks)
    loss = ref.ce_sum_ref(out, labels)
    loss.backward()
    vec = {k_: t.float() for k_, t in E.group_vectors({n: p.grad for n, p in r.named_parameters()
                                                        if p.grad is not None}).items()}
    return float(loss.detach()), vec


def run(geo):
    torch.set_num_threads(int(os.environ.get("OMP_NUM_THREADS", "8")))
    sd = E.weights(geo)
    x, lt, labels, masks = E.inputs(geo)
    samples, index, losses = [], [], {}
    for v in PER_GEO[geo]:
        r = model(geo, v, sd)
        losses[v] = []
        for k in range(N):
            t0 = time.time()
            loss, vec = sample(r, geo, x, lt, labels, masks, k, VARIANTS[v][3])
            samples.append(vec)
            index.append(v)
            losses[v].append(loss)
            print("%s %s k=%d loss %.6f (%.1fs)" % (geo, v, k, loss, time.time() - t0), flush=True)
        del r
    groups = list(samples[0])
    grams = {}
    for gname in groups:
        m = torch.stack([s[gname] for s in samples]).double()
        grams[gname] = (m @ m.T).numpy()
    meta = {"geo": geo, "geometry": dict(zip(("backbone", "time_conv", "B", "T", "L",
                                               "weight_seed", "input_seed"), E.GEOS[geo])),
            "n": N, "eps": E.EPS, "index": index, "groups": groups, "losses": losses,
            "x_digest": E.digest(x), "lt_digest": E.digest(lt),
            "weights_digest": E.digest(torch.cat([t.float().reshape(-1) for t in sd.values()
                                                  if t.is_floating_point()])),
            "torch": torch.__version__,
            "variants": {v: {"precision": VARIANTS[v][0], "bf16_act": VARIANTS[v][1],
                             "ops": VARIANTS[v][2], "eps": VARIANTS[v][3]}
                         for v in PER_GEO[geo]}}
    np.savez_compressed(os.path.join(HERE, "bf16_ensemble_%s.npz" % geo),
                        **{"gram_" + gname: grams[gname] for gname in groups})
    restat(geo, meta)


def restat(geo, meta=None):
    """(Re)derive the fixture's statistics from its Gram matrices."""
    path = os.path.join(HERE, "bf16_ensemble_%s.json" % geo)
    if meta is None:
        with open(path) as f:
            meta = json.load(f)
    z = np.load(os.path.join(HERE, "bf16_ensemble_%s.npz" % geo))
    index, n = meta["index"], meta["n"]
    base = [i for i, v in enumerate(index) if v == "fp32"]
    stats = {}
    for v in meta["variants"]:
        if v == "fp32":
            continue
        sub = [i for i, w in enumerate(index) if w == v] + base
        stats[v] = {g: E.stats(z["gram_" + g][np.ix_(sub, sub)], n) for g in meta["groups"]}
    meta["stats_vs_fp32"] = stats
    with open(path, "w") as f:
        json.dump(meta, f, indent=1)
    for v, st in stats.items():
        print(v, " ".join("%s r%.2f p%.2f c%.2f" % (g, s["ratio"], s["proj"], s["cstar"])
                          for g, s in st.items()))


if __name__ == "__main__":
    args = sys.argv[1:]
    if args and args[0] == "--restat":
        for geo in (args[1:] or ["r50", "rst"]):
            restat(geo)
    else:
        for geo in (args or ["r50", "rst"]):
            run(geo)
