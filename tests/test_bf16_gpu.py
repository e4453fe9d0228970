"""bf16 operand math (TMR_MATH_BF16) for the bf16 configs C4/C5 (BASELINE.json configs[3],[4]).

The reference is fp32-only, so the bf16 contract is defined by the build and restated in the
oracle (oracle/tmrnet_ref.py emulate_bf16_convs): every trunk convolution rounds its operands to
bf16 (RNE) -- fwd (x, w), dgrad (dy, w), wgrad (x, dy) -- multiplies exactly and accumulates in
fp32; activations, BatchNorm, LSTM, NLBlock, TimeConv and the head stay fp32.

Kernel level: the HIP bf16 conv against float64 convs of the same rounded operands (only the
fp32 accumulation order differs: 5e-6 relative).  Model level: the bf16 TMRNet against the
bf16-emulating oracle.  The two differ by fp32 summation order; a 1-ulp fp32 difference flips
the bf16 rounding of an activation now and then, and with batch-statistic BatchNorm over 6
frames those flips reach the logits at ~1e-2 (the fp32 CPU oracle is that far from its own
float64 run).  So logits and gradients are both judged against the float64 oracle with the
criterion of tests/test_model_parity_gpu.py: no further from it than 3x the fp32 CPU oracle
(floor 2e-3); argmax must agree wherever the float64 top-2 margin exceeds that error.
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

import tmrnet_amd
from tmrnet_amd import ops
from oracle import tmrnet_ref as ref
from tests.test_kernels_gpu import CONV_CASES, rel_err
from tests.test_model_parity_gpu import _assert_vs_fp64, _double_copy, _inputs

pytestmark = pytest.mark.gpu


def _r(t):
    return ref.bf16_round(t)


@pytest.mark.parametrize("case", CONV_CASES)
def test_conv_bf16(dev, case):
    n, h, w, cin, cout, r, st, pad = case
    g = torch.Generator().manual_seed(hash(case) % 1000 + 1)
    x = torch.randn(n, cin, h, w, generator=g, dtype=torch.float64)
    wt = torch.randn(cout, cin, r, r, generator=g, dtype=torch.float64) / np.sqrt(cin * r * r)
    x32, w32 = x.float(), wt.float()
    y_ref = F.conv2d(_r(x32).double(), _r(w32).double(), stride=st, padding=pad)
    dy = torch.randn(y_ref.shape, generator=g, dtype=torch.float64)
    dyb = _r(dy.float()).double()
    dx_ref = torch.nn.grad.conv2d_input(x.shape, _r(w32).double(), dyb, st, pad)
    dw_ref = torch.nn.grad.conv2d_weight(_r(x32).double(), wt.shape, dyb, st, pad)
    cs = 4 if cin == 3 else cin
    x4 = ops.nchw_to_nhwc(x32.to(dev), cpad=cs)
    wk = ops.weight_to_krsc(w32.to(dev).contiguous(), cpad=cs)
    y = ops.conv_fwd(x4, wk, st, pad, math="bf16")
    assert rel_err(y.permute(0, 3, 1, 2), y_ref) < 5e-6
    dyd = dy.float().permute(0, 2, 3, 1).contiguous().to(dev)
    if cin != 3:
        dx = ops.conv_dgrad(dyd, wk, (h, w), st, pad, math="bf16")
        assert rel_err(dx.permute(0, 3, 1, 2), dx_ref) < 5e-6
    dw = ops.conv_wgrad(x4, dyd, r, r, st, pad, c_real=cin, math="bf16")
    assert rel_err(dw, dw_ref) < 5e-6
    # the bf16 path really rounds: differs from the fp32 path by ~bf16 precision
    y32 = ops.conv_fwd(x4, wk, st, pad)
    d = rel_err(y, y32)
    assert 1e-5 < d < 3e-2, d


def _step_pair(dev, backbone, time_conv, seed):
    B, T, L = 2, 3, 7
    torch.manual_seed(seed)
    m = tmrnet_amd.resnet_lstm(seq_len=T, time_conv=time_conv, backbone=backbone,
                               precision="bf16").to(dev).train()
    r = ref.TMRNetRef(seq_len=T, time_conv=time_conv, backbone=backbone,
                      precision="bf16").train()
    r.load_state_dict({k: v.detach().cpu() for k, v in m.state_dict().items()})
    frames, off, lt, labels = _inputs(B, T, L, seed=seed + 1)
    gm = torch.Generator().manual_seed(seed + 2)
    masks = {"nl": (torch.rand(B, 512, generator=gm) >= 0.2).float() / 0.8,
             "head": (torch.rand(B, 512, generator=gm) >= 0.5).float() / 0.5}
    m.nl_block.forced_mask = masks["nl"].to(dev)
    m.forced_head_mask = masks["head"].to(dev)
    x4 = ops.crop_normalize(frames.to(dev), off.to(dev), T)
    x_ref = ref.crop_normalize_ref(frames, off, T).view(B, T, 3, 224, 224)
    m64 = _double_copy(r, masks, B, T, L)      # before r's forward touches running stats
    out = m(x4, lt.to(dev))
    out_r = r(x_ref, lt, masks=masks)
    out64 = m64(x_ref.double(), lt.double(), masks={k: v.double() for k, v in masks.items()})
    # bf16 rounding flips make even the fp32 CPU oracle differ from float64 by ~1e-2 here
    e_hip = (out.detach().cpu().double() - out64.detach()).abs().max().item()
    e_cpu = (out_r.detach().double() - out64.detach()).abs().max().item()
    assert e_hip < max(2e-3, 3 * e_cpu), (e_hip, e_cpu)
    top2 = out64.detach().topk(2, dim=1).values
    sure = (top2[:, 0] - top2[:, 1]) > 2 * max(e_hip, e_cpu)
    assert torch.equal(out.detach().cpu().argmax(1)[sure], out64.detach().argmax(1)[sure])
    tmrnet_amd.CrossEntropyLoss(size_average=False)(out, labels.to(dev)).backward()
    ref.ce_sum_ref(out_r, labels).backward()
    ref.ce_sum_ref(out64, labels).backward()
    grads = lambda mod: {n: p.grad for n, p in mod.named_parameters()}
    return grads(m), grads(r), grads(m64)


def test_tmrnet_resnet50_bf16_step(dev):
    """C5's model path at bf16 (ResNet50 + LSTM + NLBlock), one train step."""
    ours, r32, r64 = _step_pair(dev, "resnet50", False, 21)
    _assert_vs_fp64(ours, r32, r64, "grad")


def test_tmrnet_resnest50_bf16_step(dev):
    """C4's model (ResNeSt50 + LSTM + NLBlock + TimeConv) at bf16, one train step."""
    from tests.test_resnest_gpu import _zero_grad_scales
    ours, r32, r64 = _step_pair(dev, "resnest50", True, 31)
    _assert_vs_fp64(ours, r32, r64, "grad", scales=_zero_grad_scales(r64))


@pytest.mark.parametrize("backbone,time_conv", [("resnet50", False), ("resnest50", True)])
def test_tmrnet_bf16_eval_logits(dev, backbone, time_conv):
    """Eval mode (running-stat BN: no batch-statistic amplification).  The bf16 HIP model is no
    further from the float64 bf16-emulating oracle than 5e-4 (or 3x the fp32 oracle's own
    distance: the random-init ResNet-50 grows activations to O(100) in eval mode, where a
    flipped bf16 rounding is worth ~3e-3 on the logits even between fp32 and float64)."""
    import copy
    B, T, L = 2, 3, 7
    torch.manual_seed(41)
    m = tmrnet_amd.resnet_lstm(seq_len=T, time_conv=time_conv, backbone=backbone,
                               precision="bf16").to(dev)
    g = torch.Generator().manual_seed(43)
    for mod in m.modules():     # non-trivial running statistics
        if isinstance(mod, torch.nn.BatchNorm2d):
            c = mod.running_mean.numel()
            mod.running_mean.copy_(torch.rand(c, generator=g) * 0.2 - 0.1)
            mod.running_var.copy_(torch.rand(c, generator=g) * 1.5 + 0.5)
    m.eval()
    r = ref.TMRNetRef(seq_len=T, time_conv=time_conv, backbone=backbone, precision="bf16").eval()
    r.load_state_dict({k: v.detach().cpu() for k, v in m.state_dict().items()})
    frames, off, lt, _ = _inputs(B, T, L, seed=42)
    x_ref = ref.crop_normalize_ref(frames, off, T).view(B, T, 3, 224, 224)
    r64 = copy.deepcopy(r).double()
    x4 = ops.crop_normalize(frames.to(dev), off.to(dev), T)
    with torch.no_grad():
        out = m(x4, lt.to(dev)).cpu().double()
        out_r = r(x_ref, lt).double()
        out64 = r64(x_ref.double(), lt.double())
    e_hip = (out - out64).abs().max().item()
    e_cpu = (out_r - out64).abs().max().item()
    assert e_hip < max(5e-4 * max(1.0, out64.abs().max().item()), 3 * e_cpu), (e_hip, e_cpu)
    assert torch.equal(out.argmax(1), out64.argmax(1))


def test_conv_bf16_all_resnet50_shapes(dev):
    """Every distinct ResNet-50 conv shape at 4 frames (large-M tile configs, strided 1x1/3x3,
    the 7x7 stem): fwd, dgrad and wgrad in bf16 math against float64 convs of the rounded
    operands, and each against the fp32 path run on the same bf16-representable operands
    (then bf16 and fp32 math must agree to fp32 accumulation error)."""
    from scripts.convbench import resnet50_convs
    g = torch.Generator().manual_seed(5)
    for shp in sorted(set(resnet50_convs(4))):
        n, h, w, cin, cout, r, st, pad = shp
        cs = 4 if cin == 3 else cin
        x = _r(torch.randn(n, h, w, cs, generator=g))
        if cin == 3:
            x[..., 3] = 0
        wk = _r(torch.randn(cout, r, r, cs, generator=g) / (cin * r * r) ** 0.5)
        if cin == 3:
            wk[..., 3] = 0
        xd, wd = x.to(dev), wk.to(dev)
        y16 = ops.conv_fwd(xd, wd, st, pad, math="bf16")
        y32 = ops.conv_fwd(xd, wd, st, pad)
        assert rel_err(y16, y32) < 5e-6, ("fwd", shp)
        dy = _r(torch.randn(y16.shape, generator=g)).to(dev)
        if cin != 3:
            d16 = ops.conv_dgrad(dy, wd, (h, w), st, pad, math="bf16")
            d32 = ops.conv_dgrad(dy, wd, (h, w), st, pad)
            assert rel_err(d16, d32) < 5e-6, ("dgrad", shp)
        w16 = ops.conv_wgrad(xd, dy, r, r, st, pad, c_real=cin, math="bf16")
        w32 = ops.conv_wgrad(xd, dy, r, r, st, pad, c_real=cin)
        assert rel_err(w16, w32) < 5e-6, ("wgrad", shp)


@pytest.mark.parametrize("backbone,time_conv", [("resnet50", False)])
def test_bf16_storage_bit_identical(dev, backbone, time_conv):
    """bf16 storage of the conv-operand-only tensors (KRSC weights, non-residual BN+ReLU outputs,
    BatchNorm-backward outputs; tmr_conv_desc.io) against fp32 storage of the same bf16-math
    step: the convs round those operands to bf16 (RNE) either way, so the logits, every
    gradient and the running statistics are bit-identical."""
    from tmrnet_amd import trunk
    B, T, L = 2, 5, 7
    frames, off, lt, labels = _inputs(B, T, L, seed=51)
    res = {}
    saved = trunk.BF16_STORE
    try:
        for store in (True, False):
            trunk.BF16_STORE = store
            torch.manual_seed(52)
            m = tmrnet_amd.resnet_lstm(seq_len=T, time_conv=time_conv, backbone=backbone,
                                       precision="bf16").to(dev).train()
            m.nl_block.forced_mask = torch.ones(B, 512, device=dev)
            m.forced_head_mask = torch.ones(B, 512, device=dev)
            x4 = ops.crop_normalize(frames.to(dev), off.to(dev), T)
            out = m(x4, lt.to(dev))
            tmrnet_amd.CrossEntropyLoss(size_average=False)(out, labels.to(dev)).backward()
            torch.cuda.synchronize()
            res[store] = (out.detach().clone(),
                          {n: p.grad.clone() for n, p in m.named_parameters()},
                          {n: b.clone() for n, b in m.named_buffers()})
            if store:   # eval mode (fused conv epilogue) with bf16 weights
                m.eval()
                with torch.no_grad():
                    res["eval16"] = m(x4, lt.to(dev)).clone()
            else:
                m.eval()
                with torch.no_grad():
                    res["eval32"] = m(x4, lt.to(dev)).clone()
    finally:
        trunk.BF16_STORE = saved
    assert torch.equal(res[True][0], res[False][0])
    for n in res[True][1]:
        assert torch.equal(res[True][1][n], res[False][1][n]), n
    for n in res[True][2]:
        assert torch.equal(res[True][2][n], res[False][2][n]), n
    assert torch.equal(res["eval16"], res["eval32"])


def test_bf16_storage_conv_kernels(dev):
    """Each bf16-stored operand combination (tmr_conv_desc.io) against the same conv with the
    operands stored fp32 (already bf16-representable): bit-identical (same rounding, same
    arithmetic), on every distinct ResNet-50 shape at 2 frames, incl. the stem and strided 1x1 /
    3x3 convs (dgrad parity classes) and frame-chunked launches."""
    from scripts.convbench import resnet50_convs
    g = torch.Generator().manual_seed(61)
    saved = ops.MAX_FRAMES
    try:
        for mf in (0, 1):
            ops.MAX_FRAMES = mf
            for shp in sorted(set(resnet50_convs(2))):
                n, h, w, cin, cout, r, st, pad = shp
                cs = 4 if cin == 3 else cin
                x = _r(torch.randn(n, h, w, cs, generator=g))
                if cin == 3:
                    x[..., 3] = 0
                wt = torch.randn(cout, cin, r, r, generator=g) / (cin * r * r) ** 0.5
                xd, wd = x.to(dev), wt.to(dev)
                w32 = ops.weight_to_krsc(wd, cpad=cs)
                w16 = ops.weight_to_krsc(wd, cpad=cs, bf16=True)
                assert torch.equal(w16.float(), _r(w32.cpu()).to(dev)), shp
                x16 = xd.to(torch.bfloat16)
                xin = xd if cin == 3 else x16     # the stem input stays fp32 (VAR 1 gather)
                y32, _, _ = ops.conv_fwd_bnstats(xd, w32, st, pad, c_real=cin, math="bf16")
                y16, _, _ = ops.conv_fwd_bnstats(xin, w16, st, pad, c_real=cin, math="bf16")
                assert torch.equal(y16, y32), ("fwd", shp, mf)
                dy = _r(torch.randn(y32.shape, generator=g)).to(dev)
                dy16 = dy.to(torch.bfloat16)
                if cin != 3:
                    d32 = ops.conv_dgrad(dy, w32, (h, w), st, pad, math="bf16")
                    d16 = ops.conv_dgrad(dy16, w16, (h, w), st, pad, math="bf16")
                    assert torch.equal(d16, d32), ("dgrad", shp, mf)
                for xa in ((xd, x16) if cin != 3 else (xd,)):
                    g32 = ops.conv_wgrad(xd, dy, r, r, st, pad, c_real=cin, math="bf16")
                    g16 = ops.conv_wgrad(xa, dy16, r, r, st, pad, c_real=cin, math="bf16")
                    assert torch.equal(g16, g32), ("wgrad", shp, mf, xa.dtype)
    finally:
        ops.MAX_FRAMES = saved
