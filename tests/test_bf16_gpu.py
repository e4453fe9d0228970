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
def test_bf16_storage_bit_identical(dev, monkeypatch, backbone, time_conv, engine):
    """bf16 storage of the conv-operand-only tensors (KRSC weights, non-residual BN+ReLU outputs,
    BatchNorm-backward outputs; tmr_conv_desc.io) against fp32 storage of the same bf16-math
    step: the convs round those operands to bf16 (RNE) either way, so the logits, every
    gradient and the running statistics are bit-identical.  On the implicit-GEMM engine: the
    direct 3x3 kernels (direct3.hip) take only all-bf16 operands, a different summation order
    (tested against float64 and the engine in tests/test_direct3_gpu.py), so ops.engine_only here."""
    from tmrnet_amd import trunk
    engine.use(True)
    B, T, L = 2, 5, 7
    frames, off, lt, labels = _inputs(B, T, L, seed=51)
    res = {}
    saved = trunk.BF16_STORE, trunk.FULL16, trunk.G16
    trunk.FULL16 = False   # the all-bf16 LDS-DMA path: test_bf16_full16_step
    trunk.G16 = False      # (bf16 gradients need that path: fp32 storage keeps fp32 gradients)
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
        trunk.BF16_STORE, trunk.FULL16, trunk.G16 = saved
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
                    # the LDS-DMA engine (transposed bf16 weights): same k order -> same bits
                    dt = ops.conv_dgrad(dy16, ops.weight_to_crsk(wd), (h, w), st, pad,
                                        math="bf16", wt=True)
                    assert torch.equal(dt, d32), ("dgrad wt", shp, mf)
                g32 = ops.conv_wgrad(xd, dy, r, r, st, pad, c_real=cin, math="bf16")
                g16 = ops.conv_wgrad(xd, dy16, r, r, st, pad, c_real=cin, math="bf16")
                assert torch.equal(g16, g32), ("wgrad", shp, mf)
                if cin != 3:
                    # all-bf16 operands: the LDS-DMA engine, whose split-K plan (tile count) may
                    # differ -> the same products summed in another order
                    g16 = ops.conv_wgrad(x16, dy16, r, r, st, pad, c_real=cin, math="bf16")
                    err = (g16 - g32).abs().max().item() / g32.abs().max().item()
                    assert err < 2e-6, ("wgrad all-bf16", shp, mf, err)
    finally:
        ops.MAX_FRAMES = saved


def _conv_ref16(x, wt, stride, pad):
    """float64 conv of bf16-rounded operands (NHWC x, OIHW w) -> NHWC."""
    xn = x.double().permute(0, 3, 1, 2)
    y = torch.nn.functional.conv2d(xn, wt.double(), stride=stride, padding=pad)
    return y.permute(0, 2, 3, 1)


@pytest.mark.parametrize("case", [
    # n, h, w, cin, cout, r, stride, pad, x channel offset in a wider tensor (0 = dense)
    (2, 9, 11, 32, 64, 3, 1, 1, 0),      # 32 channels per tap: a k-tile spans two taps (TAPV)
    (3, 10, 10, 16, 32, 3, 2, 1, 0),     # 16 per tap, stride 2, odd output width
    (2, 7, 7, 8, 16, 3, 1, 1, 0),        # 8 per tap (one piece per tap)
    (2, 13, 9, 64, 128, 1, 1, 0, 0),     # 1x1, M not a tile multiple
    (1, 20, 20, 128, 64, 3, 2, 1, 0),    # strided 3x3 (dgrad parity classes), N = 64
    (2, 8, 8, 64, 64, 3, 1, 1, 64),      # channel-slice operand (grouped conv), x_ld = 128
    (5, 14, 14, 256, 256, 3, 1, 1, 0),   # 256x256 tiles
    (2, 6, 6, 512, 1024, 1, 2, 0, 0),    # strided 1x1 with empty parity classes in dgrad
])
def test_gemm16_views(dev, case, monkeypatch):
    """The bf16 LDS-DMA engine (every operand bf16 in HBM) on its three views against float64
    convolutions of the same bf16 operands: FWD / DGRAD / WGRAD, TAPV (k-tiles spanning taps),
    partial tiles, strided parity classes and channel-slice operands.  FWD and DGRAD also
    bit-identical to the register-staged bf16 engine (same k order)."""
    n, h, w, cin, cout, r, st, pad, xoff = case
    g = torch.Generator().manual_seed(71 + cin + cout)
    wt = _r(torch.randn(cout, cin, r, r, generator=g) / (cin * r * r) ** 0.5)
    xs = _r(torch.randn(n, h, w, cin + xoff, generator=g))
    x16 = xs.to(dev).to(torch.bfloat16)[..., xoff:]
    xd = xs.to(dev)[..., xoff:]
    wd = wt.to(dev)
    w16, w32 = ops.weight_to_krsc(wd, bf16=True), ops.weight_to_krsc(wd)
    if xoff:   # channel-slice operand (the forward with BN statistics takes dense x only)
        y16 = ops.conv_fwd(x16, w16, st, pad, math="bf16")
    else:
        y16, _, _ = ops.conv_fwd_bnstats(x16, w16, st, pad, math="bf16")
    ref = _conv_ref16(xs[..., xoff:], wt, st, pad)
    err = (y16.double().cpu() - ref).abs().max().item() / ref.abs().max().item()
    assert err < 1e-5, ("fwd", err)
    y32 = ops.conv_fwd(xd.contiguous(), w32, st, pad, math="bf16")
    assert torch.equal(y16, y32)
    if not xoff:   # bf16 output (TMR_IO_Y_BF16): the rounded accumulators, BN partials of those
        yb, stb, npb = ops.conv_fwd_bnstats(x16, w16, st, pad, math="bf16", y16=True)
        assert yb.dtype == torch.bfloat16 and torch.equal(yb, y32.to(torch.bfloat16))
        c = yb.shape[-1]
        mean, inv, _, _ = ops.bn_finalize(stb, npb, torch.ones(c, device=dev),
                                          torch.zeros(c, device=dev), torch.zeros(c, device=dev),
                                          torch.ones(c, device=dev), 0.1, 1e-5)
        ye = yb.double().reshape(-1, c)
        assert torch.allclose(mean.double(), ye.mean(0), rtol=1e-5, atol=1e-6)
        var_ref = ye.var(0, unbiased=False)
        assert torch.allclose((1.0 / inv.double() ** 2 - 1e-5), var_ref, rtol=1e-4, atol=1e-6)
    dy = _r(torch.randn(y16.shape, generator=g))
    dy16 = dy.to(dev).to(torch.bfloat16)
    dx = ops.conv_dgrad(dy16, ops.weight_to_crsk(wd), (h, w), st, pad, math="bf16", wt=True)
    xr = xs[..., xoff:].double().permute(0, 3, 1, 2).requires_grad_(True)
    wr = wt.double().requires_grad_(True)
    yr = torch.nn.functional.conv2d(xr, wr, stride=st, padding=pad)
    yr.backward(dy.double().permute(0, 3, 1, 2))
    dx_ref = xr.grad.permute(0, 2, 3, 1)
    err = (dx.double().cpu() - dx_ref).abs().max().item() / dx_ref.abs().max().item()
    assert err < 1e-5, ("dgrad", err)
    if cout >= 32:   # the register-staged engine needs one tap per 32-deep k-tile
        assert torch.equal(dx, ops.conv_dgrad(dy16, w16, (h, w), st, pad, math="bf16"))
    dw = ops.conv_wgrad(x16, dy16, r, r, st, pad, math="bf16")
    err = (dw.double().cpu() - wr.grad).abs().max().item() / wr.grad.abs().max().item()
    assert err < 1e-5, ("wgrad", err)


@pytest.mark.parametrize("case", [
    # n, h, w, cin, cout, stride: 1x1 forwards over the tile configs (256x256, 128x128, 256x64)
    (5, 14, 14, 64, 256, 1), (2, 13, 9, 64, 128, 1), (3, 9, 9, 128, 64, 1), (3, 9, 9, 64, 64, 1),
    (2, 9, 9, 64, 200, 1),     # N not a multiple of 64: a 32-column block with 8 valid columns
    (3, 7, 7, 32, 96, 1),      # N = 96: a partial 64-column wave block
    (2, 12, 12, 64, 512, 2),   # strided
])
def test_gemm16_y16_store_forms(dev, case):
    """bf16 y (TMR_IO_Y_BF16): the whole-line store form of epilogue_batched (the pair form on
    tiles with an odd number of 32-column blocks) writes the same bytes as the fp32 output rounded
    to bf16, including ragged M and N and the one-stage (gemm16_kernel NST = 1) one-k-tile
    forwards; its BN statistics are those of the stored values (float64)."""
    n, h, w, cin, cout, st = case
    g = torch.Generator().manual_seed(5 + cin + cout)
    wt = _r(torch.randn(cout, cin, 1, 1, generator=g) / cin ** 0.5)
    x16 = _r(torch.randn(n, h, w, cin, generator=g)).to(dev).to(torch.bfloat16)
    w16 = ops.weight_to_krsc(wt.to(dev), bf16=True)
    y32, st32, _ = ops.conv_fwd_bnstats(x16, w16, st, 0, math="bf16")
    yb, stb, npb = ops.conv_fwd_bnstats(x16, w16, st, 0, math="bf16", y16=True)
    assert torch.equal(yb.view(torch.int16), y32.to(torch.bfloat16).view(torch.int16))
    c = yb.shape[-1]
    one, zero = torch.ones(c, device=dev), torch.zeros(c, device=dev)
    mean, inv, _, _ = ops.bn_finalize(stb, npb, one, zero, zero.clone(), one.clone(), 0.1, 1e-5)
    ye = yb.double().reshape(-1, c)
    assert torch.allclose(mean.double(), ye.mean(0), rtol=1e-5, atol=1e-6)
    assert torch.allclose(1.0 / inv.double() ** 2 - 1e-5, ye.var(0, unbiased=False), rtol=1e-4,
                          atol=1e-6)


def test_bf16_full16_step(dev):
    """The all-bf16-operand train step (trunk.FULL16: bf16 block-output copies, bf16 maxpool
    output, transposed bf16 dgrad weights, every conv but the stem on the LDS-DMA engine) against
    the register-staged bf16 step: the same operands rounded the same way; only the BN-statistic
    tile partials and the wgrad split-K plans differ (summation order), so logits agree to fp32
    rounding and gradients to the ill-conditioning of a 10-frame BN batch."""
    from tmrnet_amd import trunk
    B, T, L = 2, 5, 7
    frames, off, lt, labels = _inputs(B, T, L, seed=53)
    res = {}
    saved = trunk.FULL16, trunk.ACT16
    trunk.ACT16 = False   # the engine A/B; the bf16-activation contract: the fp64 tests above
    try:
        for full in (True, False):
            trunk.FULL16 = full
            torch.manual_seed(54)
            m = tmrnet_amd.resnet_lstm(seq_len=T, precision="bf16").to(dev).train()
            m.nl_block.forced_mask = torch.ones(B, 512, device=dev)
            m.forced_head_mask = torch.ones(B, 512, device=dev)
            x4 = ops.crop_normalize(frames.to(dev), off.to(dev), T)
            out = m(x4, lt.to(dev))
            tmrnet_amd.CrossEntropyLoss(size_average=False)(out, labels.to(dev)).backward()
            torch.cuda.synchronize()
            res[full] = (out.detach().clone(), {n: p.grad.clone() for n, p in m.named_parameters()})
    finally:
        trunk.FULL16, trunk.ACT16 = saved
    assert (res[True][0] - res[False][0]).abs().max().item() < 1e-4
    assert torch.equal(res[True][0].argmax(1), res[False][0].argmax(1))
    # two fp32 summation orders of the same step: at 10 frames per BN batch the trunk gradients
    # are ill-conditioned (the fp32 CPU oracle itself is ~2% (L2) from float64), so
    # this is a gross-error check; each path's gradients are held to the float64 criterion by
    # test_tmrnet_resnet50_bf16_step (default path) and the register-staged tests
    num = sum(((res[True][1][k] - res[False][1][k]).double() ** 2).sum() for k in res[True][1])
    den = sum((res[False][1][k].double() ** 2).sum() for k in res[True][1])
    assert (num / den).sqrt().item() < 5e-2
    for k in res[True][1]:
        assert torch.isfinite(res[True][1][k]).all(), k


@pytest.mark.parametrize("case", [
    # n, h, w, cin(dx channels), cout(dy channels), r, stride, pad, mask, beta, bf16 y/z
    (3, 14, 14, 64, 256, 1, 1, 0, 2, 0.0, True),     # conv3 dgrad -> conv2's BN (mask from y)
    (2, 14, 14, 128, 128, 3, 2, 1, 2, 0.0, True),    # strided 3x3: four parity-class launches
    (3, 12, 12, 256, 64, 1, 1, 0, 1, 1.0, True),     # conv1 dgrad += identity grad (mask from z)
    (2, 14, 14, 256, 512, 1, 2, 0, 1, 1.0, True),    # strided 1x1 downsample: tap-less classes
    (2, 9, 9, 64, 64, 3, 1, 1, 0, 0.0, True),        # no ReLU
    (3, 12, 12, 256, 64, 1, 1, 0, 1, 1.0, False),    # fp32 y / z (bf16 operands only)
    (2, 20, 20, 512, 64, 1, 1, 0, 2, 0.0, True),     # 256x64 tiles (N = 512... rows of 800)
])
def test_gemm16_dgrad_fused_bn_backward(dev, case):
    """The LDS-DMA engine's dgrad with the fused BatchNorm-backward epilogue (LDS-staged, 8
    columns per thread) against its plain dgrad followed by the separate BN backward: the masked
    dx bit-exactly, dy / dgamma / dbeta to fp32 summation-order tolerance; y / z bf16 (the bf16
    step's activations) or fp32."""
    n, h, w, cin, cout, r, st, pad, mask, beta, y16 = case
    g = torch.Generator().manual_seed(13)
    ho = (h + 2 * pad - r) // st + 1
    wo = (w + 2 * pad - r) // st + 1
    dy = _r(torch.randn(n, ho, wo, cout, generator=g)).to(dev).to(torch.bfloat16)
    wt = (torch.randn(cout, cin, r, r, generator=g) / np.sqrt(cout * r * r)).to(dev)
    wct = ops.weight_to_crsk(wt)
    yf = torch.randn(n, h, w, cin, generator=g).to(dev)
    y = yf.to(torch.bfloat16) if y16 else yf
    ye = y.float()
    mean = ye.view(-1, cin).mean(0)
    inv = 1.0 / (ye.view(-1, cin).var(0, unbiased=False) + 1e-5).sqrt()
    gamma = (torch.rand(cin, generator=g) + 0.5).to(dev)
    scale = gamma * inv
    shift = (torch.randn(cin, generator=g) * 0.1).to(dev) - mean * scale
    res = torch.randn(n, h, w, cin, generator=g).to(dev)
    z = torch.relu(ye * scale + shift + res) if mask == 1 else None
    if z is not None and y16:
        z = z.to(torch.bfloat16)
    old = torch.randn(n, h, w, cin, generator=g).to(dev)
    dz = ops.conv_dgrad(dy, wct, (h, w), st, pad, out=old.clone(), beta=beta, math="bf16", wt=True)
    ze = z.float() if z is not None else None
    if mask:
        keep = (ze > 0) if mask == 1 else (ye * scale + shift > 0)
        dres_ref = torch.where(keep, dz, torch.zeros_like(dz))
    else:
        dres_ref = dz
    dzf, parts, npart = ops.conv_dgrad_bnbwd(dy, wct, (h, w), st, pad, y, mean, mask, z=z,
                                              scale=scale, shift=shift, out=old.clone(), beta=beta,
                                              math="bf16", wt=True)
    dyf, dgf, dbf = ops.bn_bwd_parts(dzf, ye, parts, npart, mean, inv, gamma)
    dy_ref, _, dg_ref, db_ref = ops.bn_bwd(dres_ref, ye, None, mean, inv, gamma, False)
    torch.cuda.synchronize()
    assert torch.equal(dzf, dres_ref)
    assert rel_err(dyf, dy_ref) < 1e-5
    assert rel_err(dgf, dg_ref) < 1e-5 and rel_err(dbf, db_ref) < 1e-5


@pytest.mark.parametrize("case", [
    # n, h, w, cin(dx channels), cout(dy channels), r, stride, pad
    (3, 14, 14, 64, 256, 1, 1, 0),     # conv3 dgrad -> bn2's gradient (256x64 tiles)
    (2, 14, 14, 128, 128, 3, 2, 1),    # strided 3x3 conv2 dgrad -> bn1's gradient: parity classes
    (2, 20, 20, 256, 128, 3, 1, 1),    # 128x128 tiles
])
def test_gemm16_dgrad_g16(dev, case):
    """TMR_IO_G16: the fused BN-backward dgrad storing the masked gradient g as bf16 (the
    non-residual units of the bf16 step) writes exactly the RNE rounding of the fp32 path's g; its
    BN partials are those of the rounded values (vs float64 sums); and the BN-backward apply
    reading bf16 g (tmr_bn_bwd_parts_g16) is bit-identical to the fp32-g apply on the same
    values and partials."""
    n, h, w, cin, cout, r, st, pad = case
    g = torch.Generator().manual_seed(17)
    ho = (h + 2 * pad - r) // st + 1
    wo = (w + 2 * pad - r) // st + 1
    dy = _r(torch.randn(n, ho, wo, cout, generator=g)).to(dev).to(torch.bfloat16)
    wt = (torch.randn(cout, cin, r, r, generator=g) / np.sqrt(cout * r * r)).to(dev)
    wct = ops.weight_to_crsk(wt)
    y = torch.randn(n, h, w, cin, generator=g).to(dev).to(torch.bfloat16)
    ye = y.float()
    mean = ye.view(-1, cin).mean(0)
    inv = 1.0 / (ye.view(-1, cin).var(0, unbiased=False) + 1e-5).sqrt()
    gamma = (torch.rand(cin, generator=g) + 0.5).to(dev)
    scale = gamma * inv
    shift = (torch.randn(cin, generator=g) * 0.1).to(dev) - mean * scale
    kw = dict(scale=scale, shift=shift, math="bf16", wt=True)
    d32, p32, n32 = ops.conv_dgrad_bnbwd(dy, wct, (h, w), st, pad, y, mean, 2, **kw)
    d16, p16, n16 = ops.conv_dgrad_bnbwd(dy, wct, (h, w), st, pad, y, mean, 2, g16=True, **kw)
    torch.cuda.synchronize()
    assert d16.dtype == torch.bfloat16 and n16 == n32
    assert torch.equal(d16, d32.to(torch.bfloat16))
    gd = d16.double().view(-1, cin)
    want = torch.stack([gd.sum(0), (gd * (ye.double().view(-1, cin) - mean.double())).sum(0)], -1)
    got = p16[:n16].double().sum(0)
    assert (got - want).abs().max().item() <= 1e-5 * want.abs().max().item() + 1e-6
    a = ops.bn_bwd_parts(d16, y, p16, n16, mean, inv, gamma)
    b = ops.bn_bwd_parts(d16.float(), y, p16, n16, mean, inv, gamma)
    torch.cuda.synchronize()
    assert a[0].dtype == torch.bfloat16
    for u, v in zip(a, b):
        assert torch.equal(u, v)


@pytest.mark.parametrize("case", [
    # n, h, w, cin(dx channels), cout(dy channels), old dtype
    (3, 14, 14, 256, 64, "bf16"),      # a Bottleneck conv1 dgrad adding into the bf16 stream
    (2, 12, 12, 512, 128, "fp32"),     # ... reading the fp32 stream (downsample dgrad / last block)
])
@pytest.mark.parametrize("mask", [1, 3])
def test_gemm16_dgrad_residual_g16(dev, case, mask):
    """The bf16 residual-stream gradient (trunk.R16, tmr_conv2d_dgrad_bnbwd_acc / TMR_IO_G16 with
    beta): the conv1 dgrad adds into the old gradient (bf16 in place, or fp32 from another tensor),
    masks by the previous block's ReLU (z, or its bits) and stores bf16 -- exactly the RNE rounding
    of the fp32 path's result on the same old values; partials those of the rounded values."""
    n, h, w, cin, cout, odt = case
    g = torch.Generator().manual_seed(23)
    dy = _r(torch.randn(n, h, w, cout, generator=g)).to(dev).to(torch.bfloat16)
    wt = (torch.randn(cout, cin, 1, 1, generator=g) / np.sqrt(cout)).to(dev)
    wct = ops.weight_to_crsk(wt)
    y = torch.randn(n, h, w, cin, generator=g).to(dev).to(torch.bfloat16)
    ye = y.float()
    mean = ye.view(-1, cin).mean(0)
    zf = torch.relu(ye + torch.randn(n, h, w, cin, generator=g).to(dev) * 0.5)
    z = zf.to(torch.bfloat16)
    zm = z
    if mask == 3:
        from tests.test_kernels_gpu import _pack_bits
        zm = _pack_bits((z.float() > 0).cpu()).to(dev)
    old = torch.randn(n, h, w, cin, generator=g).to(dev)
    if odt == "bf16":
        old = old.to(torch.bfloat16)
    old32 = old.float().clone()
    kw = dict(z=zm, math="bf16", wt=True, beta=1.0)
    d32, p32, n32 = ops.conv_dgrad_bnbwd(dy, wct, (h, w), 1, 0, y, mean, mask, out=old32, **kw)
    if odt == "bf16":
        o16 = old.clone()
        d16, p16, n16 = ops.conv_dgrad_bnbwd(dy, wct, (h, w), 1, 0, y, mean, mask, out=o16,
                                             g16=True, **kw)
        assert d16.data_ptr() == o16.data_ptr()
    else:
        d16, p16, n16 = ops.conv_dgrad_bnbwd(dy, wct, (h, w), 1, 0, y, mean, mask, g16=True,
                                             old=old, **kw)
    torch.cuda.synchronize()
    assert d16.dtype == torch.bfloat16 and n16 == n32
    assert torch.equal(d16, d32.to(torch.bfloat16))
    gd = d16.double().view(-1, cin)
    want = torch.stack([gd.sum(0), (gd * (ye.double().view(-1, cin) - mean.double())).sum(0)], -1)
    got = p16[:n16].double().sum(0)
    assert (got - want).abs().max().item() <= 1e-5 * want.abs().max().item() + 1e-6


def test_bn_bwd_bf16_dz(dev):
    """The downsample branch's BN backward with the bf16 residual-stream gradient as dz
    (tmr_bn_bwd_g16): bit-identical to the fp32-dz path on the same values."""
    g = torch.Generator().manual_seed(29)
    rows, c = 3 * 14 * 14, 256
    y = torch.randn(3, 14, 14, c, generator=g).to(dev).to(torch.bfloat16)
    dz = torch.randn(3, 14, 14, c, generator=g).to(dev).to(torch.bfloat16)
    ye = y.float().view(rows, c)
    mean = ye.mean(0)
    inv = 1.0 / (ye.var(0, unbiased=False) + 1e-5).sqrt()
    gamma = (torch.rand(c, generator=g) + 0.5).to(dev)
    a = ops.bn_bwd(dz, y, None, mean, inv, gamma, False)
    b = ops.bn_bwd(dz.float(), y, None, mean, inv, gamma, False)
    torch.cuda.synchronize()
    assert a[0].dtype == torch.bfloat16 and a[1] is None
    assert torch.equal(a[0], b[0]) and torch.equal(a[2], b[2]) and torch.equal(a[3], b[3])


def test_stem_nhwc8_bf16_input(dev):
    """The bf16 step's stem input (tmr_nhwc4_to_bf16x8): bit-exact bf16 (RNE) of the NHWC4 fp32
    pixels with channels 3-7 zero; the 7x7/2 stem on it (bf16 LDS-DMA engine, forward and
    wgrad) against float64 convs of the rounded operands (summation order only, 5e-6)."""
    g = torch.Generator().manual_seed(21)
    n, h, w = 3, 40, 36
    x = torch.randn(n, 3, h, w, generator=g)
    x4 = ops.nchw_to_nhwc(x.to(dev), cpad=4)
    x8 = ops.nhwc4_to_bf16x8(x4)
    want = torch.zeros(n, h, w, 8, dtype=torch.bfloat16)
    want[..., :3] = x.permute(0, 2, 3, 1).to(torch.bfloat16)
    torch.cuda.synchronize()
    assert x8.dtype == torch.bfloat16 and torch.equal(x8.cpu(), want)
    wt = torch.randn(64, 3, 7, 7, generator=g) / np.sqrt(147)
    wk = ops.weight_to_krsc(wt.to(dev), cpad=8, bf16=True)
    y = ops.conv_fwd(x8, wk, 2, 3, math="bf16")
    xr = x.to(torch.bfloat16).double()
    wr = wt.to(torch.bfloat16).double()
    y_ref = F.conv2d(xr, wr, stride=2, padding=3)
    assert rel_err(y.permute(0, 3, 1, 2), y_ref) < 5e-6
    dy = torch.randn(y_ref.shape, generator=g).to(torch.bfloat16)
    dyd = dy.permute(0, 2, 3, 1).contiguous().to(dev)
    dw = ops.conv_wgrad(x8, dyd, 7, 7, 2, 3, c_real=3, math="bf16")
    xg = xr.clone().requires_grad_(False)
    wg = wr.clone().requires_grad_(True)
    F.conv2d(xg, wg, stride=2, padding=3).backward(dy.double())
    assert rel_err(dw, wg.grad) < 5e-6
    with pytest.raises(RuntimeError):
        ops.nhwc4_to_bf16x8(torch.randn(1, 4, 4, 3, device=dev))
