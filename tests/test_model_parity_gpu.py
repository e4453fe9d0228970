"""End-to-end parity of the HIP path against the CPU oracle (oracle/tmrnet_ref.py) and the
reference-generated golden fixtures (tests/golden/).

Contract (BASELINE.json north_star / SURVEY.md §8c): fp32 logits within 1e-4 absolute and
bit-identical argmax phase ids on identical inputs and weights, in train mode (batch-stat BN,
dropout masks injected so both sides use the same mask) and in eval mode.  Gradients are
compared per parameter with a relative tolerance (fp32, different summation order).
"""
import os

import numpy as np
import pytest
import torch

import tmrnet_amd
from tmrnet_amd import ops
from oracle import tmrnet_ref as ref
from tests.golden.golden_inputs import (nlblock_params, nlblock_inputs, projection_probes,
                                        project, timeconv_params, timeconv_inputs, NL_CASES)

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


def rel_err(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return ((a - b).abs().max() / (b.abs().max() + 1e-30)).item()


@pytest.mark.parametrize("case", NL_CASES, ids=lambda c: "L%d" % c["L"])
@pytest.mark.parametrize("lfb_rows", [False, True])
def test_nlblock_golden(dev, case, lfb_rows):
    """HIP NLBlock vs outputs/grads of the reference module (NLBlock_MutiConv6_3.py:10-40)."""
    B, L, seed = case["B"], case["L"], case["seed"]
    z = np.load(os.path.join(GOLD, "nlblock_L%d.npz" % L))
    m = tmrnet_amd.NLBlock().to(dev).eval()
    m.load_state_dict({k: torch.from_numpy(v) for k, v in nlblock_params(seed).items()})
    St_np, Lt_np, g_np = nlblock_inputs(seed, B, L)
    St = torch.from_numpy(St_np).to(dev).requires_grad_(True)
    if lfb_rows:
        # the same Lt served as rows of a resident bank (rows permuted + duplicated bank)
        bank = torch.from_numpy(Lt_np.reshape(B * L, 512)).to(dev)
        perm = torch.randperm(B * L)
        bank2 = torch.empty_like(bank)
        bank2[perm.to(dev)] = bank
        rows = perm.view(B, L).to(torch.int32).to(dev)
        Lt = tmrnet_amd.LFBRows(bank2, rows)
    else:
        Lt = torch.from_numpy(Lt_np).to(dev).requires_grad_(True)
    out = m(St, Lt)
    out.backward(torch.from_numpy(g_np).to(dev))
    assert np.abs(out.detach().cpu().numpy() - z["out"]).max() < 1e-5
    assert rel_err(St.grad, torch.from_numpy(z["dSt"])) < 1e-5
    if not lfb_rows:
        assert rel_err(Lt.grad, torch.from_numpy(z["dLt"])) < 1e-5
    probes = projection_probes(seed, (512, 512), 16)
    for name, p in m.named_parameters():
        key = "d_" + name.replace(".", "_")
        g = p.grad.detach().cpu().numpy()
        if g.shape == (512, 512):
            pr = project(g, probes)
            ex = z[key + "_proj"]
            assert np.abs(pr - ex).max() <= 1e-5 * np.abs(ex).max() + 1e-6, name
            assert np.abs(g[0] - z[key + "_row0"]).max() <= 1e-5 * np.abs(z[key + "_row0"]).max() + 1e-7
        else:
            ex = z[key]
            assert np.abs(g.reshape(ex.shape) - ex).max() <= 1e-5 * np.abs(ex).max() + 1e-6, name


def _make_pair(dev, seq_len, seed=0):
    torch.manual_seed(seed)
    m = tmrnet_amd.resnet_lstm(seq_len=seq_len).to(dev)
    r = ref.TMRNetRef(seq_len=seq_len)
    r.load_state_dict({k: v.detach().cpu() for k, v in m.state_dict().items()})
    return m, r


def _double_copy(r, masks, B, T, L):
    import copy
    m64 = copy.deepcopy(r).double()
    m64.load_state_dict({k: v.double() if v.is_floating_point() else v
                         for k, v in r.state_dict().items()})
    # running stats were already updated by r's forward: restore the pre-forward values
    for (n, b) in m64.named_buffers():
        if n.endswith("running_mean"):
            b.zero_()
        elif n.endswith("running_var"):
            b.fill_(1.0)
        elif n.endswith("num_batches_tracked"):
            b.zero_()
    for p in m64.parameters():
        p.grad = None
    return m64


def _inputs(B, T, L, seed=1):
    g = torch.Generator().manual_seed(seed)
    frames = torch.randint(0, 256, (B * T, 250, 250, 3), generator=g, dtype=torch.uint8)
    off = torch.randint(0, 27, (B, 2), generator=g, dtype=torch.int32)
    lt = torch.rand(B, L, 512, generator=g) * 2 - 1
    labels = torch.randint(0, 7, (B,), generator=g)
    return frames, off, lt, labels


@pytest.mark.parametrize("train", [True, False])
def test_tmrnet_step_parity(dev, train):
    B, T, L = 2, 3, 5
    m, r = _make_pair(dev, T)
    frames, off, lt, labels = _inputs(B, T, L)
    x_ref = ref.crop_normalize_ref(frames, off, T)
    x4 = ops.crop_normalize(frames.to(dev), off.to(dev), T)
    assert torch.equal(x4[..., :3].permute(0, 3, 1, 2).cpu(), x_ref)
    g = torch.Generator().manual_seed(7)
    masks = {"nl": (torch.rand(B, 512, generator=g) >= 0.2).float() / 0.8,
             "head": (torch.rand(B, 512, generator=g) >= 0.5).float() / 0.5}
    m.train(train); r.train(train)
    if train:
        m.nl_block.forced_mask = masks["nl"].to(dev)
        m.forced_head_mask = masks["head"].to(dev)
    out = m(x4, lt.to(dev))
    out_r = r(x_ref.view(B, T, 3, 224, 224), lt, masks=masks if train else None)
    err = (out.detach().cpu() - out_r.detach()).abs().max().item()
    assert err < 1e-4, err
    assert torch.equal(out.detach().cpu().argmax(1), out_r.detach().argmax(1))
    if not train:
        return
    crit = tmrnet_amd.CrossEntropyLoss(size_average=False)
    loss = crit(out, labels.to(dev))
    loss_r = ref.ce_sum_ref(out_r, labels)
    assert abs(loss.item() - loss_r.item()) <= 1e-4 * max(1.0, abs(loss_r.item()))
    loss.backward()
    loss_r.backward()
    # float64 oracle: the fp32 CPU oracle's own rounding error sets the scale for the HIP path's
    m64 = _double_copy(r, masks, B, T, L)
    out64 = m64(x_ref.double().view(B, T, 3, 224, 224), lt.double(),
                masks={k: v.double() for k, v in masks.items()})
    ref.ce_sum_ref(out64, labels).backward()
    g = lambda mod: {n: p.grad for n, p in mod.named_parameters()}
    _assert_vs_fp64(g(m), g(r), g(m64), "grad")
    # running statistics after one train-mode forward
    rb = dict(r.named_buffers())
    for name, b in m.named_buffers():
        if b.dtype.is_floating_point:
            assert rel_err(b, rb[name]) < 1e-4, name
        else:
            assert torch.equal(b.cpu(), rb[name]), name


def l2_err(a, b, scale=None):
    """relative L2 error; `scale` replaces |b| for quantities that are exactly zero in exact
    arithmetic (e.g. the bias of a Linear followed by batch-stat BatchNorm)."""
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return ((a - b).norm() / ((b.norm() if scale is None else scale) + 1e-30)).item()


GRAD_RATIO = 4.0      # per parameter: e_hip <= GRAD_RATIO * e_cpu + 1e-5 (+ slack)
AGG_RATIO = 1.5       # all parameters: sqrt(sum e_hip^2 / sum e_cpu^2) <= AGG_RATIO


def _assert_vs_fp64(ours, ref32, ref64, what, scales=None, slack=0.0, record=None):
    """HIP result vs the float64 oracle, scaled by the fp32 CPU oracle's own distance from it.

    At random init the trunk gradients are ill-conditioned in fp32 whatever the BN batch: each
    Bottleneck's BatchNorm backward (a projection with cancellation) multiplies the relative
    error, so the fp32 CPU oracle is ~1e-5 from float64 at the head but 1-2e-2 at the stem
    (measured at B=2, T=3 and at the benchmarked B=2, T=10, tests/test_geometry_gpu.py).  A
    fixed tolerance would test fp32 rounding noise at the stem or be loose at the head, so the
    bound is scale-free and has no absolute floor: taken together the HIP gradients may be no
    further from float64 than AGG_RATIO x the fp32 oracle (measured 1.16-1.21), and no single
    parameter further than GRAD_RATIO x (+1e-5 relative; a per-parameter ratio is a ratio of two
    noisy errors, and the CPU oracle accumulates BN reductions in double where the kernels use
    fp32 tiles: measured worst 1.3-3.6).  `slack` adds an explicit allowance (bf16 head ReLU
    flips, tests/test_geometry_gpu.py)."""
    import inspect
    import json
    scales = scales or {}
    rows, bad = [], []
    for name, t in ours.items():
        e_hip = l2_err(t, ref64[name], scales.get(name))
        e_cpu = l2_err(ref32[name], ref64[name], scales.get(name))
        rows.append((name, e_hip, e_cpu))
        if not e_hip <= GRAD_RATIO * e_cpu + 1e-5 + slack:
            bad.append((name, e_hip, e_cpu))
    # a parameter whose exact gradient is 0 (nl_block.linear2.bias: the q.b2 score term is
    # constant over the LFB rows and cancels in the softmax) has no relative error
    agg_rows = [r for r in rows if not r[0].endswith("linear2.bias") or r[0] in scales]
    agg = (sum(h * h for _, h, _ in agg_rows) / max(sum(c * c for _, _, c in agg_rows), 1e-300)) ** 0.5
    rec = {"test": record or inspect.stack()[1].function, "what": what, "slack": slack,
           "max_ratio": max(h / max(c, 1e-12) for _, h, c in agg_rows), "agg_ratio": agg}
    out = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out")
    os.makedirs(out, exist_ok=True)     # scratch record of the measured ratios
    with open(os.path.join(out, "grad_ratios.jsonl"), "a") as f:
        f.write(json.dumps(rec) + "\n")
    assert not bad, (what, bad[:5])
    assert agg <= AGG_RATIO, (what, agg)


def test_sgd_step_after_backward_parity(dev):
    """Two full steps (forward, CE-sum, backward, SGD with the reference's param groups)."""
    B, T, L = 2, 3, 5
    m, r = _make_pair(dev, T, seed=3)
    frames, off, lt, labels = _inputs(B, T, L, seed=4)
    m.train(); r.train()
    masks = {"nl": torch.ones(B, 512), "head": torch.ones(B, 512)}
    m.nl_block.forced_mask = masks["nl"].to(dev)
    m.forced_head_mask = masks["head"].to(dev)
    r64 = _double_copy(r, masks, B, T, L)
    lr = 1e-3
    opt = tmrnet_amd.SGD(ref.sgd_param_groups(m, lr), lr=lr / 10, momentum=0.9,
                         weight_decay=5e-4)
    opt_r = torch.optim.SGD(ref.sgd_param_groups(r, lr), lr=lr / 10, momentum=0.9,
                            weight_decay=5e-4)
    opt_64 = torch.optim.SGD(ref.sgd_param_groups(r64, lr), lr=lr / 10, momentum=0.9,
                             weight_decay=5e-4)
    x4 = ops.crop_normalize(frames.to(dev), off.to(dev), T)
    x_ref = ref.crop_normalize_ref(frames, off, T).view(B, T, 3, 224, 224)
    crit = tmrnet_amd.CrossEntropyLoss(size_average=False)
    m64 = {k: v.double() for k, v in masks.items()}
    p0 = {n: p.detach().cpu().double().clone() for n, p in r.named_parameters()}
    for _ in range(2):
        opt.zero_grad()
        loss = crit(m(x4, lt.to(dev)), labels.to(dev))
        loss.backward()
        opt.step()
        ref.train_step_ref(r, opt_r, x_ref, lt, labels, masks=masks)
        ref.train_step_ref(r64, opt_64, x_ref.double(), lt.double(), labels, masks=m64)
    # compare the parameter UPDATES (p - p0) against the float64 trajectory
    upd = lambda named: {n: p.detach().cpu().double() - p0[n] for n, p in named}
    _assert_vs_fp64(upd(m.named_parameters()), upd(r.named_parameters()),
                    upd(r64.named_parameters()), "update")


def test_memory_bank_model_parity(dev):
    """Config 1 model (train_singlenet_phase_1fc.py:201-232) on the HIP path vs the oracle."""
    B, T = 2, 3
    torch.manual_seed(5)
    m = tmrnet_amd.MemoryBankModel(seq_len=T).to(dev)
    r = ref.MemoryBankRef(seq_len=T)
    r.load_state_dict({k: v.detach().cpu() for k, v in m.state_dict().items()})
    r64 = _double_copy(r, None, B, T, 1)
    frames, off, _, labels = _inputs(B, T, 1, seed=6)
    mask = (torch.rand(B * T, 512) >= 0.2).float() / 0.8
    m.forced_mask = mask.to(dev)
    x4 = ops.crop_normalize(frames.to(dev), off.to(dev), T)
    x_ref = ref.crop_normalize_ref(frames, off, T)
    out = m(x4)
    out_r = r(x_ref, mask=mask)
    assert (out.detach().cpu() - out_r.detach()).abs().max().item() < 1e-4
    assert torch.equal(out.detach().cpu().argmax(1), out_r.detach().argmax(1))
    sel = out[T - 1::T]
    loss = tmrnet_amd.CrossEntropyLoss(size_average=False)(sel, labels.to(dev))
    loss.backward()
    ref.ce_sum_ref(out_r[T - 1::T], labels).backward()
    out64 = r64(x_ref.double(), mask=mask.double())
    ref.ce_sum_ref(out64[T - 1::T], labels).backward()
    g = lambda mod: {n: p.grad for n, p in mod.named_parameters()}
    _assert_vs_fp64(g(m), g(r), g(r64), "grad")


def test_timeconv_golden(dev):
    """HIP TimeConv vs the reference module's outputs/grads at L=30 (NLBlock_MutiConv6_3.py:43-79)."""
    from tmrnet_amd.timeconv import TimeConv
    from tests.golden.golden_inputs import TC_CASES
    case = TC_CASES[0]
    B, L, seed = case["B"], case["L"], case["seed"]
    z = np.load(os.path.join(GOLD, "timeconv_L%d.npz" % L))
    m = TimeConv().to(dev)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in timeconv_params(seed).items()})
    x_np, g_np = timeconv_inputs(seed, B, L)
    x = torch.from_numpy(x_np).to(dev).requires_grad_(True)
    y = m(x)
    y.backward(torch.from_numpy(g_np).to(dev))
    assert np.abs(y.detach().cpu().numpy() - z["out"]).max() < 1e-5
    assert rel_err(x.grad, torch.from_numpy(z["dx"])) < 1e-5
    for name, p in m.named_parameters():
        key = "d_" + name.replace(".", "_")
        g = p.grad.detach().cpu().numpy()
        if g.ndim == 3:
            probes = projection_probes(seed + 7, g.shape, 16)
            ex = z[key + "_proj"]
            assert np.abs(project(g, probes) - ex).max() <= 1e-5 * np.abs(ex).max(), name
        else:
            assert np.abs(g - z[key]).max() <= 1e-5 * np.abs(z[key]).max(), name


@pytest.mark.parametrize("L", [1, 7, 40])
def test_timeconv_generalised_L(dev, L):
    from tmrnet_amd.timeconv import TimeConv
    torch.manual_seed(L)
    m = TimeConv().to(dev)
    r = ref.TimeConvRef()
    r.load_state_dict({k: v.cpu() for k, v in m.state_dict().items()})
    x = torch.rand(3, L, 512) * 2 - 1
    y = m(x.to(dev))
    assert (y.cpu() - r(x)).abs().max().item() < 1e-5


def test_tmrnet_muticonv_parity(dev):
    """resnet_lstm with TimeConv (train_non-local_mutiConv_resnet.py:208-253), L=40."""
    B, T, L = 2, 3, 40
    torch.manual_seed(2)
    m = tmrnet_amd.resnet_lstm(seq_len=T, num_classes=6, time_conv=True).to(dev).eval()
    r = ref.TMRNetRef(seq_len=T, num_classes=6, time_conv=True).eval()
    r.load_state_dict({k: v.detach().cpu() for k, v in m.state_dict().items()})
    frames, off, lt, labels = _inputs(B, T, L, seed=8)
    x4 = ops.crop_normalize(frames.to(dev), off.to(dev), T)
    out = m(x4, lt.to(dev))
    out_r = r(ref.crop_normalize_ref(frames, off, T).view(B, T, 3, 224, 224), lt)
    assert (out.detach().cpu() - out_r.detach()).abs().max().item() < 1e-4
    assert torch.equal(out.detach().cpu().argmax(1), out_r.argmax(1))

