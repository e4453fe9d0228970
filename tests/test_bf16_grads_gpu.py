"""Gradient-level acceptance of the bf16 train step (configs C4, C5) against the fp32 step the
reference runs (`loss.backward(); optimizer.step()`, code/Training TMRNet/
train_non-local_mutiConv_resnest.py:751-752, train_only_non-local_pretrained.py:724-725), at the
benchmarked size: 64 clips, C5 T=30 / L=300 (1920 frames, ResNet-50), C4 T=10 / L=40 (640 frames,
ResNeSt-50 + TimeConv), the benchmark's i.i.d.-noise frames (and structured frames), the same
weights, LFB rows, labels and dropout masks on both sides.  The fp32 HIP step stands in for the
reference's arithmetic: it is pinned to the CPU oracle (tests/test_geometry_gpu.py, full-size C2
logits within 2.1e-5).  Bounds and their reasons: DESIGN.md §2 "bf16 gradients".

What the train step's gradients can and cannot be held to.  At this random init the trunk
gradients of the fp32 step itself are chaotic: one fp32 ulp of input noise moves them 1-2% (rel
L2), one bf16 rounding of the input frames (2^-9) moves them by 60-100% (single-sample cosine 0.4-
0.75 with the unperturbed fp32 gradient; tests/_bf16_grads.py variants fp32p, fp32xb, fp32n).  A
bf16 step rounds ~50 conv operands per frame, so no bf16 implementation's single trunk gradient
can be close to the fp32 one; what can be asserted is
  1. the clip branch (LSTM, NLBlock, TimeConv, head) per group: cos >= CLIP_COS, rel L2 <=
     CLIP_REL (measured >= 0.963 / <= 0.285);
  2. the two gradient-storage narrowings (trunk.G16: bn1/bn2 output gradients bf16; trunk.R16: the
     residual stream's gradient bf16) earn their place: turning both off moves no group's cosine
     with fp32 by more than NARROW_DCOS (measured <= 0.003);
  3. in expectation over bf16-sized input noise (ensembles of 2K samples each, the noise-free
     inner products <g*_a, g*_b> estimated from pairs of independent samples,
     _bf16_grads.ensemble_stats), the bf16 step's gradient points the fp32 step's way in every
     group: c* = <g*16, g*32> / (|g*16| |g*32|) >= TRUNK_CSTAR (trunk; measured C5 0.67-0.87, C4
     0.78-0.95) and >= CLIP_CSTAR (clip branch; >= 0.989);
     The same ensembles bound the magnitude (round 6): the projection of E g16 on the fp32
     direction, <g*16, g*32> / |g*32|^2, >= TRUNK_PROJ per trunk group (C5 0.39-0.47 on
     stem..layer3 in round 5) and >= CLIP_PROJ per clip-branch group.  That the shrinkage is the
     contract's and not the kernels' is asserted at a host-runnable geometry against the CPU
     emulation (tests/test_bf16_ensemble_gpu.py: HIP within 0.08 of the emulation per group);
  4. SGD with the reference's groups (momentum 0.9, wd 5e-4, trunk / LSTM at lr / 10) for 20 steps
     on the batch: the bf16 loss curve within TRAJ_BAND x the initial loss of the fp32 curve at
     every step, and its final loss within TRAJ_FINAL x fp32's, at lr 1e-4 and 3e-5 (the loss
     falls from ~150 to ~1 / ~12-34); at lr 1e-5, where the shrinkage shows (C5 loss 50.3 vs 36.7
     after 20 steps in round 5), the bf16 curve must fall monotonically to <= SLOW_DROP x its
     initial loss and end within SLOW_FINAL x fp32's.
The records (gpurun_out/bf16_grads_*.json) keep every group's numbers; profiles/r5/bf16_grads/
holds the study runs (scripts/bf16_grad_study.py) with the attribution over G16 / R16 / ACT16 and
the lr = 1e-5 trajectories, where the bf16 step trains visibly slower (C5: loss 50.3 vs 36.7 after
20 steps; the same with only operand rounding, ACT16 off: 48.4; storage narrowings off: 50.6).
"""
import json
import os

import pytest
import torch

from tests import _bf16_grads as bg

pytestmark = pytest.mark.gpu
OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out")

CLIP = ("lstm", "time_conv", "nl_block", "head")
TRUNK = ("stem", "layer1", "layer2", "layer3", "layer4")
CLIP_COS, CLIP_REL = 0.95, 0.35
NARROW_DCOS = 0.02
TRUNK_CSTAR, CLIP_CSTAR = 0.6, 0.95
TRUNK_PROJ, CLIP_PROJ = 0.3, 0.9
ENS_K = 4
TRAJ_BAND, TRAJ_FINAL = 0.05, 1.25
TRAJ_LRS = (1e-4, 3e-5)
SLOW_LR, SLOW_DROP, SLOW_FINAL = 1e-5, 0.6, 1.6

GEOS = {"c5": ("resnet50", False, 30, 300), "c4": ("resnest50", True, 10, 40)}


def _record(name, data):
    os.makedirs(OUT, exist_ok=True)
    with open(os.path.join(OUT, "bf16_grads_%s.json" % name), "w") as f:
        json.dump(data, f, indent=1)


class _Step:
    """Shared inputs / initial weights of one geometry; grads(variant, x) runs one step."""

    def __init__(self, dev, geo, frames):
        self.dev = dev
        self.backbone, self.tc, self.T, self.L = GEOS[geo]
        self.x4, self.lfb, self.labels = bg.full_inputs(dev, 64, self.T, self.L, frames)
        self.mk = bg.masks(64, 6)
        m = bg.make_model(dev, self.T, self.backbone, self.tc, "fp32")
        self.sd = {k: t.detach().clone() for k, t in m.state_dict().items()}
        del m

    def model(self, prec):
        return bg.make_model(self.dev, self.T, self.backbone, self.tc, prec, self.sd)

    def grads(self, v, x=None):
        with bg.variant(v) as prec:
            m = self.model(prec)
            _, _, g = bg.grads_of(m, self.x4 if x is None else x, self.lfb, self.labels, self.mk)
        del m
        return g


@pytest.mark.parametrize("frames", ["noise", "struct"])
@pytest.mark.parametrize("geo", ["c5", "c4"])
def test_bf16_grads_single_step(dev, geo, frames):
    """Bounds 1 and 2 of the module doc on one full-size step."""
    st = _Step(dev, geo, frames)
    g32 = st.grads("fp32")
    g16 = st.grads("bf16")
    g16o = st.grads("bf16_gradsoff")
    grp16, _ = bg.compare(g16, g32)
    grpo, _ = bg.compare(g16o, g32)
    _record("%s_%s_single" % (geo, frames), {"bf16": grp16, "bf16_gradsoff": grpo})
    for k in CLIP:
        if k in grp16:
            assert grp16[k]["cos"] >= CLIP_COS and grp16[k]["rel_l2"] <= CLIP_REL, (k, grp16[k])
    for k in grp16:
        assert abs(grp16[k]["cos"] - grpo[k]["cos"]) <= NARROW_DCOS, (k, grp16[k], grpo[k])


@pytest.mark.parametrize("geo", ["c5", "c4"])
def test_bf16_grads_expectation(dev, geo):
    """Bound 3: bf16 and fp32 gradient ensembles over +-2^-9 input noise (2K samples each)."""
    st = _Step(dev, geo, "noise")
    ens = {}
    for prec in ("bf16", "fp32"):
        ens[prec] = []
        for k in range(2 * ENS_K):
            x = bg.perturb_rel(st.x4, 2.0 ** -9, 100 + k)
            ens[prec].append({n: t.float() for n, t in st.grads(prec, x).items()})
    s16 = bg.ensemble_stats(ens["bf16"], ens["bf16"], same=True)
    s32 = bg.ensemble_stats(ens["fp32"], ens["fp32"], same=True)
    x = bg.ensemble_stats(ens["bf16"], ens["fp32"])
    rec = {k: {"c_star": x[k] / (max(s16[k], 1e-300) * max(s32[k], 1e-300)) ** 0.5,
               "ratio": (max(s16[k], 0.0) / max(s32[k], 1e-300)) ** 0.5,
               "proj": x[k] / max(s32[k], 1e-300),
               "s16": s16[k], "s32": s32[k], "x": x[k]} for k in x}
    _record("%s_expectation_K%d" % (geo, ENS_K), rec)
    for k, r in rec.items():
        assert s16[k] > 0 and s32[k] > 0, (k, r)
        bound = TRUNK_CSTAR if k in TRUNK else CLIP_CSTAR
        assert r["c_star"] >= bound, (k, r)
        assert r["proj"] >= (TRUNK_PROJ if k in TRUNK else CLIP_PROJ), (k, r)


@pytest.mark.parametrize("geo", ["c5", "c4"])
def test_bf16_sgd_trajectory(dev, geo):
    """Bound 4: 20 SGD steps on the batch, bf16 vs fp32 loss curves."""
    st = _Step(dev, geo, "noise")
    rec = {}
    for lr in TRAJ_LRS + (SLOW_LR,):
        curves = {}
        for prec in ("fp32", "bf16"):
            m = st.model(prec)
            curves[prec] = bg.trajectory(m, [(st.x4, st.lfb, st.labels)], st.mk, lr, 20)
            del m
            torch.cuda.empty_cache()
        rec["lr%g" % lr] = curves
    _record("%s_trajectory" % geo, rec)
    for lr in TRAJ_LRS:
        l32, l16 = rec["lr%g" % lr]["fp32"], rec["lr%g" % lr]["bf16"]
        assert l32[-1] < 0.5 * l32[0], ("the lr must move the loss", l32)
        band = TRAJ_BAND * l32[0]
        assert max(abs(a - b) for a, b in zip(l16, l32)) <= band, (lr, l16, l32)
        assert l16[-1] <= TRAJ_FINAL * l32[-1], (lr, l16[-1], l32[-1])
    l32, l16 = rec["lr%g" % SLOW_LR]["fp32"], rec["lr%g" % SLOW_LR]["bf16"]
    assert all(b < a for a, b in zip(l16, l16[1:])), ("bf16 loss must fall every step", l16)
    assert l16[-1] <= SLOW_DROP * l16[0], (l16[0], l16[-1])
    assert l16[-1] <= SLOW_FINAL * l32[-1], (l16[-1], l32[-1])
