"""Helpers for the bf16-vs-fp32 gradient acceptance (tests/test_bf16_grads_gpu.py,
scripts/bf16_grad_study.py): the benchmarked C4 / C5 train step run at several precisions /
storage contracts on identical weights, inputs, LFB rows, dropout masks and labels, and the
weight gradients compared per parameter group.

Reference step: `loss.backward(); optimizer.step()` in fp32
(code/Training TMRNet/train_non-local_mutiConv_resnest.py:751-752,
train_only_non-local_pretrained.py:724-725).  The fp32 HIP step is itself pinned to the CPU oracle
(tests/test_geometry_gpu.py), so it stands in for the reference's fp32 arithmetic at full size.
"""
import contextlib
import math

import torch

import tmrnet_amd
from tmrnet_amd import ops, trunk, LFBRows

# variant -> (precision, trunk-module overrides).  "fp32p": the fp32 step on input frames perturbed
# by one fp32 ulp (random sign per element; see perturb_ulp): the fp32 noise floor of the
# comparison -- how far the step's own rounding level moves its gradients.
VARIANTS = {
    "fp32": ("fp32", {}),
    "fp32p": ("fp32", {}),
    "fp32xb": ("fp32", {}),     # the fp32 step on the input frames rounded to bf16 (see inputs_for)
    "fp32n": ("fp32", {}),      # ... on the input frames with +-2^-9 relative noise (inputs_for)
    "bf16n": ("bf16", {}),      # the bf16 step on those frames
    "bf16": ("bf16", {}),
    "bf16_g16off": ("bf16", {"G16": False}),
    "bf16_r16off": ("bf16", {"R16": False}),
    "bf16_gradsoff": ("bf16", {"G16": False, "R16": False}),
    "bf16_actoff": ("bf16", {"ACT16": False}),
}

GROUPS = ("stem", "layer1", "layer2", "layer3", "layer4", "lstm", "time_conv", "nl_block", "head")


def group_of(name):
    if name.startswith("share."):
        part = name.split(".")[1]
        return part if part.startswith("layer") else "stem"
    if name.startswith(("fc_h_c.", "fc_c.")):
        return "head"
    return name.split(".")[0]


@contextlib.contextmanager
def variant(name):
    prec, over = VARIANTS[name]
    old = {k: getattr(trunk, k) for k in over}
    for k, v in over.items():
        setattr(trunk, k, v)
    try:
        yield prec
    finally:
        for k, v in old.items():
            setattr(trunk, k, v)


def structured_frames(n, seed):
    """(n, 250, 250, 3) uint8: a random 6x6 RGB field upsampled bilinearly + N(0, 20) noise."""
    g = torch.Generator().manual_seed(seed)
    lo = torch.rand(n, 3, 6, 6, generator=g) * 255
    img = torch.nn.functional.interpolate(lo, size=(250, 250), mode="bilinear", align_corners=False)
    img = img + torch.randn(n, 3, 250, 250, generator=g) * 20
    return img.clamp(0, 255).round().to(torch.uint8).permute(0, 2, 3, 1).contiguous()


def perturb_ulp(x4, seed=9):
    """x4 with every element moved by one fp32 ulp up or down (random sign, seeded): a
    perturbation of the size of one fp32 rounding."""
    g = torch.Generator(device=x4.device).manual_seed(seed)
    sgn = torch.randint(0, 2, x4.shape, generator=g, device=x4.device, dtype=torch.int32) * 2 - 1
    bits = x4.contiguous().view(torch.int32)
    out = (bits + sgn * (x4 != 0).to(torch.int32)).view(torch.float32)
    return out


def perturb_rel(x4, eps, seed):
    """x4 * (1 + eps * s), s = +-1 at random per element (seeded): input noise of a chosen
    relative size (eps = 2^-9: one bf16 rounding)."""
    g = torch.Generator(device=x4.device).manual_seed(seed)
    sgn = torch.randint(0, 2, x4.shape, generator=g, device=x4.device).to(x4.dtype) * 2 - 1
    return x4 * (1 + eps * sgn)


def ensemble_stats(gs_a, gs_b, same=False):
    """Per group: the mean pairwise inner product of two gradient ensembles, <g_i, g_j> over
    i in a, j in b, leaving out i == j: within one ensemble (`same`) a sample with itself, across
    two a pair run on the same input-noise sample (both ensembles draw noise sample k for their
    k-th member, so that pair shares its noise term).  For samples g = g* + n with independent
    zero-mean noise this estimates <g*_a, g*_b> without the noise terms."""
    out = {}
    names = [n for n in gs_a[0] if not (n == "nl_block.linear2.bias" or n.endswith("fc1.bias"))]
    for n in names:
        grp = group_of(n)
        tot, cnt = 0.0, 0
        for i, ga in enumerate(gs_a):
            for j, gb_ in enumerate(gs_b):
                if (same and j <= i) or i == j:
                    continue
                tot += float((ga[n].double() * gb_[n].double()).sum())
                cnt += 1
        out[grp] = out.get(grp, 0.0) + tot / max(cnt, 1)
    return out


def inputs_for(v, x4):
    """The frames a variant runs on: fp32p one fp32 ulp off (perturb_ulp), fp32xb rounded to bf16
    (one bf16 rounding of the input alone: the size of the operand rounding the bf16 step applies
    at every conv), every other variant x4 itself."""
    if v == "fp32p":
        return perturb_ulp(x4)
    if v == "fp32xb":
        return x4.to(torch.bfloat16).to(torch.float32)
    if v in ("fp32n", "bf16n"):
        return perturb_rel(x4, 2.0 ** -9, 9)
    return x4


def masks(B, seed):
    g = torch.Generator().manual_seed(seed)
    return {"nl": (torch.rand(B, 512, generator=g) >= 0.2).float() / 0.8,
            "head": (torch.rand(B, 512, generator=g) >= 0.5).float() / 0.5}


def full_inputs(dev, B, T, L, frames_kind, seed=0):
    """The bench's inputs: a 40 x 2500-frame bank, sampled starts, the reference
    train transform on the device; frames i.i.d. uniform ("noise", the benchmark's data) or
    structured -> (x4 NHWC4, LFBRows, labels)."""
    from tmrnet_amd.augment import ClipAugment
    from tmrnet_amd.lfb import valid_starts
    from tmrnet_amd.sampler import ClipSampler
    vs = valid_starts(T, [2500] * 40)
    g = torch.Generator().manual_seed(3)
    bank = (torch.rand(len(vs), 512, generator=g) * 2 - 1).to(dev)
    starts = torch.from_numpy(ClipSampler(vs, B, seed=4 + seed).batch(0)).to(dev)
    rows = ops.lfb_index(torch.tensor(vs, dtype=torch.int64, device=dev), starts, L)
    if frames_kind == "struct":
        frames = structured_frames(B * T, 7 + seed).to(dev)
    else:
        g1 = torch.Generator().manual_seed(1 + seed)
        frames = torch.randint(0, 256, (B * T, 250, 250, 3), generator=g1, dtype=torch.uint8).to(dev)
    x4 = ClipAugment(seq_len=T, use_flip=1)(frames)
    labels = torch.randint(0, 7, (B,), generator=torch.Generator().manual_seed(5 + seed)).to(dev)
    return x4, LFBRows(bank, rows), labels


def make_model(dev, T, backbone, time_conv, prec, sd=None):
    torch.manual_seed(0)
    m = tmrnet_amd.resnet_lstm(seq_len=T, precision=prec, backbone=backbone,
                               time_conv=time_conv).to(dev)
    if sd is not None:
        m.load_state_dict(sd)
    return m


def grads_of(m, x4, lfb, labels, mk):
    """One train-mode forward + CE-sum backward -> (loss, {name: grad on the host})."""
    m.train()
    m.nl_block.forced_mask = mk["nl"].to(x4.device)
    m.forced_head_mask = mk["head"].to(x4.device)
    m.zero_grad(set_to_none=True)
    out = m(x4, lfb)
    loss = tmrnet_amd.CrossEntropyLoss(size_average=False)(out, labels)
    loss.backward()
    g = {n: p.grad.detach().double().cpu() for n, p in m.named_parameters() if p.grad is not None}
    return loss.item(), out.detach().double().cpu(), g


def compare(g, g_ref, exact_zero=("nl_block.linear2.bias",)):
    """Per group and per parameter: cosine similarity and relative L2 of g against g_ref.  Skips
    parameters whose exact gradient is 0 (nl_block.linear2.bias: the q.b2 score term is constant
    over the LFB rows and cancels in the softmax; ResNeSt's fc1 biases before a batch-stat BN)."""
    per_param, acc = {}, {k: [0.0, 0.0, 0.0, 0.0] for k in GROUPS}
    for n, r in g_ref.items():
        if n in exact_zero or n.endswith("fc1.bias") or n not in g:
            continue
        a = g[n]
        dot, na, nr, nd = (a * r).sum().item(), a.norm().item() ** 2, r.norm().item() ** 2, \
            (a - r).norm().item() ** 2
        per_param[n] = {"cos": dot / math.sqrt(max(na * nr, 1e-300)),
                        "rel_l2": math.sqrt(nd / max(nr, 1e-300))}
        s = acc[group_of(n)]
        s[0] += dot; s[1] += na; s[2] += nr; s[3] += nd
    groups = {k: {"cos": s[0] / math.sqrt(max(s[1] * s[2], 1e-300)),
                  "rel_l2": math.sqrt(s[3] / max(s[2], 1e-300))}
              for k, s in acc.items() if s[2] > 0}
    return groups, per_param


def sgd(m, lr):
    """The reference's optimizer (train_only_non-local_pretrained.py:646-655): SGD momentum 0.9,
    wd 5e-4, share / lstm at lr/10, the rest at lr."""
    slow = [p for n, p in m.named_parameters() if n.startswith(("share.", "lstm."))]
    fast = [p for n, p in m.named_parameters() if not n.startswith(("share.", "lstm."))]
    return tmrnet_amd.SGD([{"params": slow}, {"params": fast, "lr": lr}], lr=lr / 10,
                          momentum=0.9, weight_decay=5e-4)


def trajectory(m, batches, mk, lr, steps):
    """`steps` SGD steps cycling over `batches` [(x4, lfb, labels)] -> the loss of every step."""
    opt = sgd(m, lr)
    m.train()
    m.nl_block.forced_mask = mk["nl"].to(batches[0][0].device)
    m.forced_head_mask = mk["head"].to(batches[0][0].device)
    crit = tmrnet_amd.CrossEntropyLoss(size_average=False)
    losses = []
    for i in range(steps):
        x4, lfb, labels = batches[i % len(batches)]
        opt.zero_grad()
        loss = crit(m(x4, lfb), labels)
        loss.backward()
        opt.step()
        losses.append(loss.item())
    return losses
