"""ResNeSt-50 backbone (train_non-local_mutiConv_resnest.py:204-249) on the HIP path.

Kernel level: split attention and the general average pools against float64 torch CPU
computations of the reference's ops.  Model level: the ResNeSt trunk and the ResNeSt TMRNet
(TimeConv head) against oracle/tmrnet_ref.py (resnest50_share / TMRNetRef(backbone=...)) --
logits within 1e-4 and identical argmax; gradients against the float64 oracle with the same
criterion as tests/test_model_parity_gpu.py.  The resnest package is absent from the
reference and from this image, so the ResNeSt restatement itself is "parity unpinned"
(pinned only by its parameter count and GMAC, tests/test_oracle_cpu.py)."""
import copy

import pytest
import torch
import torch.nn.functional as F

import tmrnet_amd
from tmrnet_amd import ops
from tmrnet_amd.resnest import AvgPoolFn, SplAtFn, ResNeSt50Share
from oracle import tmrnet_ref as ref
from tests.test_model_parity_gpu import (_assert_vs_fp64, _double_copy, _inputs, l2_err,
                                         rel_err)

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("case", [(2, 56, 56, 64, 3, 2, 1, True, False),
                                  (2, 56, 56, 256, 2, 2, 0, False, True),
                                  (3, 7, 7, 32, 3, 1, 1, True, False),
                                  (2, 15, 13, 8, 2, 2, 0, False, True),    # ragged + ceil
                                  (2, 15, 13, 8, 3, 2, 1, True, False)])
def test_avgpool2d(dev, case):
    n, h, w, c, k, s, p, incl, ceil = case
    g = torch.Generator().manual_seed(sum(case[:4]))
    x = torch.randn(n, c, h, w, generator=g, dtype=torch.float64)
    xr = x.clone().requires_grad_(True)
    yr = F.avg_pool2d(xr, k, s, p, ceil_mode=ceil, count_include_pad=incl)
    gy = torch.randn(yr.shape, generator=g, dtype=torch.float64)
    yr.backward(gy)
    xd = x.float().permute(0, 2, 3, 1).contiguous().to(dev).requires_grad_(True)
    y = AvgPoolFn.apply(xd, k, s, p, incl, ceil)
    assert y.shape[1:3] == yr.shape[2:]
    y.backward(gy.float().permute(0, 2, 3, 1).contiguous().to(dev))
    assert rel_err(y.permute(0, 3, 1, 2), yr) < 1e-6
    assert rel_err(xd.grad.permute(0, 3, 1, 2), xr.grad) < 1e-6


@pytest.mark.parametrize("case", [(2, 56, 56, 64, 3, 2, 1, True, False),
                                  (2, 56, 56, 256, 2, 2, 0, False, True),
                                  (3, 7, 7, 32, 3, 1, 1, True, False),
                                  (2, 15, 13, 8, 2, 2, 0, False, True),
                                  (2, 15, 13, 8, 3, 2, 1, True, False),
                                  (2, 14, 14, 512, 3, 2, 1, True, False)])
def test_avgpool2d_a16_exact(dev, case):
    """The bf16 AvgPool2d forward (ResNeSt's avd / avg_down under bf16 activations; the 3x3/2 and
    2x2/2 windows take the compile-time-window kernel, the rest the generic one) against the
    kernels' arithmetic restated in fp32 torch ops: taps summed in window order (dy, then dx) from
    0, scaled by 1/count, rounded to bf16 -- equal values."""
    n, h, w, c, k, s, p, incl, ceil = case
    g = torch.Generator().manual_seed(7 + sum(case[:4]))
    x = torch.randn(n, h, w, c, generator=g).to(torch.bfloat16)
    y = ops.avgpool2d_fwd(x.to(dev), k, s, p, incl, ceil).cpu()
    ho, wo = ops.pool_out(h, k, s, p, ceil), ops.pool_out(w, k, s, p, ceil)
    xf = x.float()
    acc = torch.zeros(n, ho, wo, c)
    cnt = torch.zeros(1, ho, wo, 1)
    oy = torch.arange(ho).view(ho, 1) * s - p
    ox = torch.arange(wo).view(1, wo) * s - p
    for dy in range(k):
        for dx in range(k):
            iy, ix = oy + dy, ox + dx
            ok = (iy >= 0) & (iy < h) & (ix >= 0) & (ix < w)
            v = xf[:, iy.clamp(0, h - 1), ix.clamp(0, w - 1), :]
            acc = acc + torch.where(ok.view(1, ho, wo, 1), v, torch.zeros_like(v))
            cnt = cnt + ok.view(1, ho, wo, 1).float()
    inv = (1.0 / torch.full_like(cnt, float(k * k))) if incl else 1.0 / cnt.clamp(min=1)
    ref = (acc * inv).to(torch.bfloat16)
    assert y.shape == ref.shape
    assert torch.equal(y.float(), ref.float())


def _zero_grad_scales(g64):
    """fc1.bias feeds batch-stat BatchNorm: its exact gradient is 0; judge it on the scale of
    the fc1.weight gradient instead of its own (rounding-noise) magnitude."""
    return {n: g64[n[:-4] + "weight"].double().norm().item()
            for n in g64 if n.endswith("fc1.bias")}


def _splat_ref(m, x2, C, gy):
    """The reference SplAtConv2d tail (after conv+bn0+relu), in m's dtype."""
    xr = x2.clone().requires_grad_(True)
    b = x2.shape[0]
    splits = torch.split(xr, C, dim=1)
    gap = F.adaptive_avg_pool2d(sum(splits), 1)
    gap = F.relu(m.bn1(m.fc1(gap)))
    att = m.fc2(gap).view(b, 1, 2, -1).transpose(1, 2)
    att = F.softmax(att, dim=1).reshape(b, -1, 1, 1)
    atts = torch.split(att, C, dim=1)
    yr = sum(a * s_ for a, s_ in zip(atts, splits))
    yr.backward(gy)
    return yr, xr.grad, {n: p.grad for n, p in m.named_parameters() if p.grad is not None}


@pytest.mark.parametrize("n,h,w,C", [(4, 56, 56, 64), (6, 7, 7, 512), (3, 5, 3, 32)])
def test_split_attention(dev, n, h, w, C):
    """SplAtFn vs the reference SplAtConv2d tail in float64; the fp32 CPU run of the same
    module sets the error scale (BN over n rows amplifies rounding when n is tiny)."""
    torch.manual_seed(C + h)
    m32 = ref.SplAtConv2d(C, C).train()
    m64 = copy.deepcopy(m32).double()
    x2 = torch.rand(n, 2 * C, h, w, dtype=torch.float64)
    gy = torch.randn(n, C, h, w, dtype=torch.float64)
    y64, dx64, g64 = _splat_ref(m64, x2, C, gy)
    y32, dx32, g32 = _splat_ref(m32, x2.float(), C, gy.float())
    from tmrnet_amd.resnest import SplAtConv2d
    md = SplAtConv2d(C, C).to(dev).train()
    md.load_state_dict(m32.state_dict())
    md.bn1.running_mean.zero_(); md.bn1.running_var.fill_(1.0)
    xd = x2.float().permute(0, 2, 3, 1).contiguous().to(dev).requires_grad_(True)
    y = SplAtFn.apply(xd, md.fc1.weight, md.fc1.bias, md.bn1.weight, md.bn1.bias, md.fc2.weight,
                      md.fc2.bias, md.bn1)
    y.backward(gy.float().permute(0, 2, 3, 1).contiguous().to(dev))
    ok = lambda ours, r32, r64, floor, sc=None: (l2_err(ours, r64, sc)
                                                 <= max(floor, 3 * l2_err(r32, r64, sc)))
    assert ok(y.permute(0, 3, 1, 2), y32, y64, 1e-6)
    assert ok(xd.grad.permute(0, 3, 1, 2), dx32, dx64, 1e-5)
    sc = _zero_grad_scales(g64)
    for name, p in md.named_parameters():
        if name in g64:
            assert ok(p.grad, g32[name], g64[name], 1e-5, sc.get(name)), name


def test_resnest_trunk_parity(dev):
    """share = resnest50 children (train_non-local_mutiConv_resnest.py:210-220), train mode."""
    torch.manual_seed(11)
    m = ResNeSt50Share().to(dev).train()
    r = ref.resnest50_share().train()
    r.load_state_dict({k: v.detach().cpu() for k, v in m.state_dict().items()})
    r64 = _double_copy(r, None, 0, 0, 0)
    g = torch.Generator().manual_seed(12)
    x = torch.rand(4, 3, 224, 224, generator=g) * 4 - 2
    feat = m(x.to(dev))
    feat_r = r(x)
    feat64 = r64(x.double())
    assert feat.shape == (4, 2048)
    # train-mode BN over 4 frames: judge the fp32 error against the float64 oracle, scaled by
    # the fp32 CPU oracle's own error (same criterion as the gradients below)
    e_hip = l2_err(feat, feat64)
    e_cpu = l2_err(feat_r, feat64)
    assert e_hip < max(1e-5, 3 * e_cpu), (e_hip, e_cpu)
    gy = torch.randn(4, 2048, generator=g)
    feat.backward(gy.to(dev))
    feat_r.backward(gy)
    feat64.backward(gy.double())
    grads = lambda mod: {n: p.grad for n, p in mod.named_parameters()}
    _assert_vs_fp64(grads(m), grads(r), grads(r64), "grad", scales=_zero_grad_scales(grads(r64)))
    rb = dict(r.named_buffers())
    for name, b in m.named_buffers():
        if b.dtype.is_floating_point:
            assert rel_err(b, rb[name]) < 1e-4, name
        else:
            assert torch.equal(b.cpu(), rb[name]), name


def test_resnest_trunk_eval(dev):
    torch.manual_seed(13)
    m = ResNeSt50Share().to(dev)
    for mod in m.modules():     # non-trivial running statistics
        if isinstance(mod, torch.nn.BatchNorm2d):
            mod.running_mean.uniform_(-0.1, 0.1)
            mod.running_var.uniform_(0.5, 2.0)
    m.eval()
    r = ref.resnest50_share().eval()
    r.load_state_dict({k: v.detach().cpu() for k, v in m.state_dict().items()})
    x = torch.rand(3, 3, 224, 224) * 4 - 2
    with torch.no_grad():
        f = m(x.to(dev)).cpu()
        fr = r(x)
    assert (f - fr).abs().max().item() < 1e-4 * max(1.0, fr.abs().max().item())


def test_tmrnet_resnest_parity(dev):
    """resnet_lstm of train_non-local_mutiConv_resnest.py (ResNeSt + LSTM + NLBlock + TimeConv),
    one train-mode step: logits, CE-sum and gradients vs the oracle."""
    B, T, L = 2, 3, 7
    torch.manual_seed(14)
    m = tmrnet_amd.resnet_lstm(seq_len=T, num_classes=7, time_conv=True,
                               backbone="resnest50").to(dev).train()
    r = ref.TMRNetRef(seq_len=T, num_classes=7, time_conv=True, backbone="resnest50").train()
    r.load_state_dict({k: v.detach().cpu() for k, v in m.state_dict().items()})
    frames, off, lt, _ = _inputs(B, T, L, seed=15)
    labels = torch.tensor([1, 5])
    g = torch.Generator().manual_seed(16)
    masks = {"nl": (torch.rand(B, 512, generator=g) >= 0.2).float() / 0.8,
             "head": (torch.rand(B, 512, generator=g) >= 0.5).float() / 0.5}
    m.nl_block.forced_mask = masks["nl"].to(dev)
    m.forced_head_mask = masks["head"].to(dev)
    x4 = ops.crop_normalize(frames.to(dev), off.to(dev), T)
    x_ref = ref.crop_normalize_ref(frames, off, T)
    out = m(x4, lt.to(dev))
    out_r = r(x_ref.view(B, T, 3, 224, 224), lt, masks=masks)
    assert (out.detach().cpu() - out_r.detach()).abs().max().item() < 1e-4
    assert torch.equal(out.detach().cpu().argmax(1), out_r.detach().argmax(1))
    loss = tmrnet_amd.CrossEntropyLoss(size_average=False)(out, labels.to(dev))
    loss.backward()
    ref.ce_sum_ref(out_r, labels).backward()
    m64 = _double_copy(r, masks, B, T, L)
    out64 = m64(x_ref.double().view(B, T, 3, 224, 224), lt.double(),
                masks={k: v.double() for k, v in masks.items()})
    ref.ce_sum_ref(out64, labels).backward()
    grads = lambda mod: {n: p.grad for n, p in mod.named_parameters()}
    _assert_vs_fp64(grads(m), grads(r), grads(m64), "grad", scales=_zero_grad_scales(grads(m64)))
