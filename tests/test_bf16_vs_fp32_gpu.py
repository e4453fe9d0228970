"""SURVEY.md §8c acceptance check of the bf16 configs (C4, C5) against the reference's fp32
arithmetic.

The reference is fp32 only (train_non-local_mutiConv_resnest.py:210-249,
NLBlock_MutiConv6_3.py:10-79); the bf16 builds have no reference implementation.  The other bf16
tests (test_bf16_gpu.py, test_geometry_gpu.py) hold the HIP bf16 path to the float64 emulation of
its OWN contract (oracle.emulate_bf16_convs); this file bounds the contract's cumulative drift
from the fp32 model the reference runs:

* small geometry, against the fp32 CPU oracle (TMRNetRef(precision="fp32")) on the same weights,
  inputs, LFB rows and dropout masks, train mode (batch-stat BN) and eval mode (running stats):
    - |logit_bf16 - logit_fp32| <= bound * max|logit_fp32|, bound = max(LOGIT_TOL, EMU_RATIO *
      e_emu, e_64 + SENS_RATIO * e_sens): LOGIT_TOL = 2e-2 (§8c line 451); e_emu = the same
      distance for the CPU float emulation of the bf16 contract (oracle.emulate_bf16_convs),
      EMU_RATIO = 1.25 -- the kernels add no drift beyond the contract's own; e_64 = the
      emulation with exact (float64) accumulation vs fp32, e_sens = the fp32 emulation vs the
      float64 one (how far fp32 summation order alone moves the contract: which way its bf16
      roundings break), SENS_RATIO = 2 -- the HIP kernels, another fp32 summation order, at most
      twice as far from the exact contract as the CPU emulation is
    - identical argmax on every clip whose fp32 top-2 margin exceeds 2 * bound * max|logit|
  C5: ResNet-50 + LSTM + NLBlock, T=30, L=300, LFB rows from a resident bank;
  C4: ResNeSt-50 + LSTM + TimeConv + NLBlock, T=10, L=40.
* full size (C4: 64 clips x 10 frames; C5: 64 clips x 30 frames = 1920 frames), HIP bf16 against
  HIP fp32 (the fp32 HIP path is itself pinned to the oracle at 1e-4, test_geometry_gpu.py):
  eval mode within LOGIT_TOL, train mode within FULL_TRAIN_TOL = 6e-2 on structured frames and
  within max(FULL_TRAIN_TOL, XB_RATIO x e_xb) on noise frames, e_xb = how far the fp32 step moves
  when only its input frames are rounded to bf16 (XB_RATIO = 4: the bf16 step rounds ~50 operands
  per frame; measured 2.3-3.2x), the argmax rule, agreement rates recorded in gpurun_out/.

Frames.  Structured synthetic frames (a random 6x6 colour field, bilinearly upsampled, plus pixel
noise of sigma 20) differ in their global statistics, as video frames do.  On frames of i.i.d.
uniform pixel noise (the benchmark's data) every frame has the same global statistics to ~1%, so a
batch-statistic BatchNorm over per-frame pooled features (ResNeSt's split attention: GAP -> fc1 ->
BN over the frames; the head's BN-free layers then carry it) normalises differences of that size
and amplifies any rounding of its inputs ~100x.  There the train-mode drift is a property of the
bf16 contract itself, not of the kernels: the CPU float emulation of the contract is 5e-2 from the
fp32 oracle at C4's geometry on noise frames, and the HIP bf16 path 1e-1 (two independent roundings
of a chaotic map), which the e_sens term bounds.  Every case is asserted.
The gradients: tests/test_bf16_grads_gpu.py.

Why train mode drifts at all.  A randomly initialised deep network with batch-statistic BatchNorm
is chaotic in its forward map (each BN re-normalises the perturbation along with the signal):
measured on the CPU oracle at C5's geometry, bf16 operand rounding of ~1e-3 per conv grows to
1.5e-2 relative at layer1's output, 5e-2 at layer2's and 1.8e-1 at layer3's (train mode), while
in eval mode (running statistics, an affine BN) it stays at 6e-3 - 1.1e-2.  The fp32 paths are in
the same regime with 2^-24 rounding (HIP fp32 vs the CPU oracle: 1e-4 on the logits,
test_geometry_gpu.py).  Measured here (gpurun records; HIP / emulation): C5 train 2.4e-2 /
2.5e-2, eval 2.8e-2 / 3.0e-2; C4 train 3.2e-2 / 3.3e-2, eval 7e-4 / 7e-4.
"""
import json
import os

import pytest
import torch

import tmrnet_amd
from tmrnet_amd import ops, LFBRows
from oracle import tmrnet_ref as ref
from tests.test_model_parity_gpu import _inputs, l2_err
from tests.test_geometry_gpu import _bank_rows, _masks

pytestmark = pytest.mark.gpu
OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out")

LOGIT_TOL = 2e-2      # relative to max|logit| of the fp32 result
EMU_RATIO = 1.25      # small geometry: bound = max(LOGIT_TOL, EMU_RATIO x the contract's own drift,
SENS_RATIO = 2.0      #   |emu64 - fp32| + SENS_RATIO x |emu32 - emu64|)
XB_RATIO = 4.0        # full size, noise frames, train: within XB_RATIO x the fp32 step's own drift
                      # when only its input frames are rounded to bf16
FULL_TRAIN_TOL = 6e-2  # full-size train mode (batch statistics), structured frames


def _record(name, data):
    os.makedirs(OUT, exist_ok=True)
    with open(os.path.join(OUT, "bf16_vs_fp32_%s.json" % name), "w") as f:
        json.dump(data, f, indent=1)


def _agreement(out16, out32, bound=LOGIT_TOL):
    """-> (max |diff| / max|logit|, sure mask, argmax agreement per clip); a clip is "sure" when
    its fp32 top-2 margin exceeds twice the logit bound"""
    o16 = out16.detach().double().cpu()
    o32 = out32.detach().double().cpu()
    scale = o32.abs().max().item()
    rel = (o16 - o32).abs().max().item() / scale
    top2 = o32.topk(2, dim=1).values
    sure = (top2[:, 0] - top2[:, 1]) > 2 * bound * scale
    same = o16.argmax(1) == o32.argmax(1)
    return rel, sure, same


def structured_frames(n, seed):
    """(n, 250, 250, 3) uint8: a random 6x6 RGB field upsampled bilinearly + N(0, 20) noise."""
    g = torch.Generator().manual_seed(seed)
    lo = torch.rand(n, 3, 6, 6, generator=g) * 255
    img = torch.nn.functional.interpolate(lo, size=(250, 250), mode="bilinear", align_corners=False)
    img = img + torch.randn(n, 3, 250, 250, generator=g) * 20
    return img.clamp(0, 255).round().to(torch.uint8).permute(0, 2, 3, 1).contiguous()


def _check(name, out16, out32, bound, extra=None):
    rel, sure, same = _agreement(out16, out32, bound)
    rec = {"rel_max_diff": rel, "bound": bound, "clips": int(same.numel()),
           "sure_clips": int(sure.sum()), "argmax_agree_sure": int(same[sure].sum()),
           "argmax_agree_all": int(same.sum()),
           "max_abs_logit": out32.detach().abs().max().item()}
    rec.update(extra or {})
    _record(name, rec)
    assert rel <= bound, rec
    assert bool(same[sure].all()), rec
    return rec


GEOMETRIES = {
    # name: (backbone, time_conv, B, T, L, seed, nvid, vlen)
    "c5": ("resnet50", False, 2, 30, 300, 41, 2, 600),
    "c4": ("resnest50", True, 2, 10, 40, 51, 3, None),
}


@pytest.mark.parametrize("frames_kind", ["struct", "noise"])
@pytest.mark.parametrize("train", [True, False], ids=["train", "eval"])
@pytest.mark.parametrize("geo", sorted(GEOMETRIES))
def test_bf16_vs_fp32_oracle(dev, geo, train, frames_kind):
    """HIP bf16 model vs the fp32 CPU oracle at the C4 / C5 geometry (§8c)."""
    backbone, tc, B, T, L, seed, nvid, vlen = GEOMETRIES[geo]
    torch.manual_seed(seed)
    m = tmrnet_amd.resnet_lstm(seq_len=T, precision="bf16", backbone=backbone,
                               time_conv=tc).to(dev).train(train)
    r = ref.TMRNetRef(seq_len=T, precision="fp32", backbone=backbone, time_conv=tc).train(train)
    r.load_state_dict({k: v.detach().cpu() for k, v in m.state_dict().items()})
    frames, off, _, labels = _inputs(B, T, L, seed=seed + 1)
    if frames_kind == "struct":
        frames = structured_frames(B * T, seed + 4)
    bank, vs, starts, rows = _bank_rows(B, L, T, seed + 2, nvid=nvid, vlen=vlen)
    lt = bank[rows.view(-1)].view(B, L, 512)
    masks = None
    if train:
        masks = _masks(B, seed + 3)
        m.nl_block.forced_mask = masks["nl"].to(dev)
        m.forced_head_mask = masks["head"].to(dev)
    x4 = ops.crop_normalize(frames.to(dev), off.to(dev), T)
    x_ref = ref.crop_normalize_ref(frames, off, T).view(B, T, 3, 224, 224)
    out = m(x4, LFBRows(bank.to(dev), rows.to(torch.int32).to(dev)))
    out_r = r(x_ref, lt, masks=masks)
    # the contract's own drift: its CPU float emulation (oracle.emulate_bf16_convs) vs fp32
    r16 = ref.TMRNetRef(seq_len=T, precision="bf16", backbone=backbone, time_conv=tc).train(train)
    r16.load_state_dict({k: v.detach().cpu() for k, v in m.state_dict().items()})
    with torch.no_grad():
        out_e = r16(x_ref, lt, masks=masks)
    e_emu, _, same_e = _agreement(out_e, out_r)
    # ... and how far the contract's own rounding ties move it: the emulation with exact (float64)
    # accumulation against the fp32 emulation.  The HIP kernels accumulate in fp32 in another
    # order, so they may sit up to SENS_RATIO x that far from the exact contract:
    # |hip - fp32| <= |emu64 - fp32| + SENS_RATIO * |emu32 - emu64|
    import copy
    r64 = copy.deepcopy(r16).double()
    with torch.no_grad():
        out_e64 = r64(x_ref.double(), lt.double(),
                      masks={k: v.double() for k, v in masks.items()} if masks else None)
    e_sens, _, _ = _agreement(out_e, out_e64)
    e64, _, _ = _agreement(out_e64, out_r)
    extra = {"emu_rel_max_diff": e_emu, "emu_argmax_agree_all": int(same_e.sum()),
             "emu64_rel_max_diff": e64, "emu32_vs_emu64": e_sens}
    bound = max(LOGIT_TOL, EMU_RATIO * e_emu, e64 + SENS_RATIO * e_sens)
    if train:
        # the bf16 step's gradients against the fp32 reference's, recorded (informative: at
        # random init with 20-60 frames per BN batch the trunk gradients are ill-conditioned,
        # tests/test_model_parity_gpu._assert_vs_fp64)
        tmrnet_amd.CrossEntropyLoss(size_average=False)(out, labels.to(dev)).backward()
        ref.ce_sum_ref(out_r, labels).backward()
        gr = dict(r.named_parameters())
        rows_ = [(n, l2_err(p.grad, gr[n].grad)) for n, p in m.named_parameters()
                 if gr[n].grad is not None and gr[n].grad.norm() > 0]
        extra["grad_rel_l2"] = {n: e for n, e in rows_}
        head = [e for n, e in rows_ if not n.startswith("share")]
        extra["grad_rel_l2_head_max"] = max(head)
    _check("%s_%s_%s" % (geo, "train" if train else "eval", frames_kind), out, out_r, bound, extra)


def _full_inputs(dev, B, T, L, frames_kind):
    from tmrnet_amd.augment import ClipAugment
    from tmrnet_amd.lfb import valid_starts
    from tmrnet_amd.sampler import ClipSampler
    vs = valid_starts(T, [2500] * 40)
    g = torch.Generator().manual_seed(3)
    bank = (torch.rand(len(vs), 512, generator=g) * 2 - 1).to(dev)
    starts = torch.from_numpy(ClipSampler(vs, B, seed=4).batch(0)).to(dev)
    rows = ops.lfb_index(torch.tensor(vs, dtype=torch.int64, device=dev), starts, L)
    if frames_kind == "struct":
        frames = structured_frames(B * T, 7).to(dev)
    else:
        g1 = torch.Generator().manual_seed(1)
        frames = torch.randint(0, 256, (B * T, 250, 250, 3), generator=g1, dtype=torch.uint8).to(dev)
    x4 = ClipAugment(seq_len=T, use_flip=1)(frames)
    return x4, LFBRows(bank, rows)


@pytest.mark.parametrize("frames_kind", ["struct", "noise"])
@pytest.mark.parametrize("geo", sorted(GEOMETRIES))
def test_bf16_vs_fp32_full_size(dev, geo, frames_kind):
    """The benchmarked C4 (640 frames) / C5 (1920 frames) forward, HIP bf16 vs HIP fp32, train
    mode (batch statistics over the whole step, dropout masks injected) and eval mode."""
    backbone, tc, _, T, L, _, _, _ = GEOMETRIES[geo]
    B = 64
    x4, lfb = _full_inputs(dev, B, T, L, frames_kind)
    masks = _masks(B, 6)
    outs = {}
    torch.manual_seed(0)
    sd = None
    for prec in ("fp32", "bf16", "fp32xb"):
        m = tmrnet_amd.resnet_lstm(seq_len=T, precision=prec[:4], backbone=backbone, time_conv=tc)
        m = m.to(dev)
        xin = x4.to(torch.bfloat16).float() if prec == "fp32xb" else x4
        if sd is None:
            sd = {k: v.detach().clone() for k, v in m.state_dict().items()}
        else:
            m.load_state_dict(sd)
        m.nl_block.forced_mask = masks["nl"].to(dev)
        m.forced_head_mask = masks["head"].to(dev)
        with torch.no_grad():
            outs[prec, "train"] = m.train()(xin, lfb).cpu()
            outs[prec, "eval"] = m.eval()(xin, lfb).cpu()
        del m
        torch.cuda.empty_cache()
    for mode in ("train", "eval"):
        e_xb, _, _ = _agreement(outs["fp32xb", mode], outs["fp32", mode])
        bound = LOGIT_TOL if mode == "eval" else FULL_TRAIN_TOL
        if mode == "train" and frames_kind == "noise":
            # i.i.d.-noise frames: batch-statistic BN over near-identical frames amplifies any
            # rounding (module doc); the bound scales with what rounding the fp32 step's input
            # frames to bf16 alone does to it
            bound = max(bound, XB_RATIO * e_xb)
        _check("%s_full_%s_%s" % (geo, mode, frames_kind), outs["bf16", mode], outs["fp32", mode],
               bound, {"fp32_bf16_input_rel_max_diff": e_xb})
