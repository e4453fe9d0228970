"""The whole-trunk ResNeSt-50 train node (tmrnet_amd/resnest.py ResNeStTrunkFn) and the kernels it
adds: grouped convolutions on the conv engine (tmr_conv_desc.groups -- SplAtConv2d's radix-2 3x3,
train_non-local_mutiConv_resnest.py:210-220) and the split attention with bn0 + ReLU applied on
load (tmr_splat_*_bn).  Each against float64 torch computations of the reference's ops; the
model-level checks of the node live in tests/test_resnest_gpu.py (fp32) and
tests/test_bf16_gpu.py / tests/test_geometry_gpu.py (bf16)."""
import copy

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from tmrnet_amd import ops
from oracle import tmrnet_ref as ref
from tests.test_kernels_gpu import rel_err
from tests.test_model_parity_gpu import l2_err

pytestmark = pytest.mark.gpu

GROUPED = [  # n, h, w, cin, cout, stride  (cin / cout totals over the 2 groups)
    (2, 56, 56, 64, 128, 1),     # layer1 (avd: the conv runs at stride 1)
    (3, 14, 14, 256, 512, 1),    # layer3
    (2, 9, 7, 128, 256, 2),      # ragged, strided
]


def _nhwc(t):
    return t.permute(0, 2, 3, 1).contiguous()


def _nchw(t):
    return t.permute(0, 3, 1, 2)


@pytest.mark.parametrize("bf16", [False, True])
@pytest.mark.parametrize("case", GROUPED)
def test_grouped_conv_views(dev, case, bf16):
    """Forward (+ BN-statistics epilogue, bf16 output under bf16 activations), dgrad (plain and
    with the fused BN backward of the producer, mask 2) and wgrad of a groups=2 conv."""
    n, h, w, cin, cout, st = case
    G = 2
    g = torch.Generator().manual_seed(cin + h)
    x = torch.randn(n, cin, h, w, generator=g, dtype=torch.float64)
    wt = torch.randn(cout, cin // G, 3, 3, generator=g, dtype=torch.float64) / np.sqrt(9 * cin / G)
    rnd = (lambda t: ref.bf16_round(t.float()).double()) if bf16 else (lambda t: t)
    math = "bf16" if bf16 else "fp32"
    sdt = torch.bfloat16 if bf16 else torch.float32
    xb, wb = rnd(x), rnd(wt)
    y64 = F.conv2d(xb, wb, stride=st, padding=1, groups=G)
    xd = _nhwc(x.float()).to(dev).to(sdt)
    wk = ops.weight_to_krsc(wt.float().to(dev).contiguous(), cpad=cin // G, bf16=bf16)
    y, stats, nparts = ops.conv_fwd_bnstats(xd, wk, st, 1, math=math, y16=bf16, groups=G)
    yf = _nchw(y.float()).cpu().double()
    assert rel_err(yf, y64) < (4e-3 if bf16 else 2e-6)
    # the BN statistics describe the stored values
    c1 = torch.ones(cout, device=dev)
    mean, inv, _, _ = ops.bn_finalize(stats, nparts, c1, torch.zeros_like(c1),
                                      torch.zeros_like(c1), torch.ones_like(c1), 0.1, 1e-5)
    ym = yf.permute(1, 0, 2, 3).reshape(cout, -1)
    assert rel_err(mean.cpu(), ym.mean(1)) < 1e-5
    assert rel_err(inv.cpu(), 1 / torch.sqrt(ym.var(1, unbiased=False) + 1e-5)) < 1e-5
    # dgrad on the per-group transposed weights
    dy = torch.randn(y64.shape, generator=g, dtype=torch.float64)
    dyb = rnd(dy)
    dyd = _nhwc(dy.float()).to(dev).to(sdt)
    wtr = ops.weight_to_crsk_grouped(wt.float().to(dev).contiguous(), G, bf16=bf16)
    dx64 = torch.nn.grad.conv2d_input(x.shape, wb, dyb, st, 1, groups=G)
    dx = ops.conv_dgrad(dyd, wtr, (h, w), st, 1, math=math, wt=True, groups=G)
    assert rel_err(_nchw(dx).cpu(), dx64) < 2e-6 * (50 if bf16 else 1)
    # fused backward of the BN + ReLU that produced x: mask y*scale+shift > 0, column sums
    yp = torch.randn(n, h, w, cin, generator=g)
    sc = torch.rand(cin, generator=g) + 0.5
    sh = torch.randn(cin, generator=g) * 0.5
    mu = torch.randn(cin, generator=g) * 0.1
    ypd = yp.to(dev).to(sdt)
    ypv = ypd.float().cpu().double()
    dxm, parts, np_ = ops.conv_dgrad_bnbwd(dyd, wtr, (h, w), st, 1, ypd, mu.to(dev), 2,
                                           scale=sc.to(dev), shift=sh.to(dev), math=math, wt=True,
                                           groups=G)
    keep = (ypv.float() * sc + sh > 0).double()
    gm = _nhwc(dx64) * keep
    assert rel_err(dxm.cpu(), gm) < 2e-6 * (50 if bf16 else 1)
    ps = parts[:np_].double().sum(0).cpu()
    assert rel_err(ps[:, 0], gm.reshape(-1, cin).sum(0)) < 1e-4
    assert rel_err(ps[:, 1], (gm * (ypv - mu.double())).reshape(-1, cin).sum(0)) < 1e-4
    # wgrad: (K, C/G, 3, 3)
    dw64 = torch.nn.grad.conv2d_weight(xb, wt.shape, dyb, st, 1, groups=G)
    dw = ops.conv_wgrad(xd, dyd, 3, 3, st, 1, math=math, groups=G)
    assert dw.shape == wt.shape
    assert rel_err(dw.cpu(), dw64) < (5e-6 if bf16 else 2e-6)


def _splat_tail_ref(m, y, C, gy, rnd):
    """bn0 (batch stats) -> relu -> [bf16 storage] -> SplAtConv2d's attention tail -> [bf16]
    in m's dtype; -> (out, dy, param grads)."""
    yr = y.clone().requires_grad_(True)
    x = F.relu(m.bn0(yr))
    if rnd:
        x = ref._RoundFn.apply(x)
    b = y.shape[0]
    splits = torch.split(x, C, dim=1)
    gap = F.adaptive_avg_pool2d(sum(splits), 1)
    gap = F.relu(m.bn1(m.fc1(gap)))
    att = m.fc2(gap).view(b, 1, 2, -1).transpose(1, 2)
    att = F.softmax(att, dim=1).reshape(b, -1, 1, 1)
    atts = torch.split(att, C, dim=1)
    out = sum(a * s_ for a, s_ in zip(atts, splits))
    if rnd:
        out = ref._RoundFn.apply(out)
    out.backward(gy)
    return out, yr.grad, {n: p.grad for n, p in m.named_parameters() if p.grad is not None}


@pytest.mark.parametrize("bf16", [False, True])
@pytest.mark.parametrize("n,h,w,C", [(6, 56, 56, 64), (8, 7, 7, 512), (5, 5, 3, 32)])
def test_split_attention_bn_on_load(dev, n, h, w, C, bf16):
    """tmr_splat_{gap,combine,bwd_reduce,bn0_coefs,bwd_apply}_bn (through resnest._splat_fwd /
    _splat_bwd) vs the reference's bn0 -> ReLU -> split attention in float64; the fp32 CPU run of
    the same module sets the error scale (batch-statistic BN over few frames)."""
    from tmrnet_amd.resnest import SplAtConv2d, _splat_fwd, _splat_bwd
    torch.manual_seed(C + h + int(bf16))
    m32 = ref.SplAtConv2d(C, C).train()
    with torch.no_grad():
        m32.bn0.weight.uniform_(0.5, 1.5)
        m32.bn0.bias.uniform_(-0.3, 0.3)
    m64 = copy.deepcopy(m32).double()
    y = torch.randn(n, 2 * C, h, w, dtype=torch.float64) + 0.2
    if bf16:
        y = ref.bf16_round(y.float()).double()   # a stored bf16 conv output
    gy = torch.randn(n, C, h, w, dtype=torch.float64)
    o64, dy64, g64 = _splat_tail_ref(m64, y, C, gy, bf16)
    o32, dy32, g32 = _splat_tail_ref(m32, y.float(), C, gy.float(), bf16)
    md = SplAtConv2d(C, C).to(dev).train()
    md.load_state_dict(m32.state_dict())
    sdt = torch.bfloat16 if bf16 else torch.float32
    yd = _nhwc(y.float()).to(dev).to(sdt)
    bn0 = md.bn0
    mean, inv, sc, sh = ops.bn_fwd_train(_nhwc(y.float()).to(dev).view(-1, 2 * C),
                                         bn0.weight.detach(), bn0.bias.detach(), bn0.running_mean,
                                         bn0.running_var, bn0.momentum, bn0.eps)
    out, spl = _splat_fwd(md, yd, sc, sh, [])
    assert out.dtype == sdt
    r2 = {"y": yd, "scale": sc, "shift": sh, "mean": mean, "inv": inv}
    grads = {}
    dy = _splat_bwd(md, spl, r2, _nhwc(gy.float()).to(dev), grads)
    assert dy.dtype == sdt
    floor = 4e-3 if bf16 else 1e-5
    ok = lambda ours, r32, r64, sc_=None: l2_err(ours, r64, sc_) <= max(floor, 3 * l2_err(r32, r64, sc_))
    assert ok(_nchw(out.float()), o32, o64), (l2_err(_nchw(out.float()), o64), l2_err(o32, o64))
    assert ok(_nchw(dy.float()), dy32, dy64), (l2_err(_nchw(dy.float()), dy64), l2_err(dy32, dy64))
    names = dict(md.named_parameters())
    for name, g_ in g64.items():
        if name.startswith("conv."):
            continue
        sc_ = g64["fc1.weight"].double().norm().item() if name == "fc1.bias" else None
        assert ok(grads[names[name]], g32[name], g_, sc_), name


@pytest.mark.parametrize("n,h,w,C", [(6, 56, 56, 64), (8, 7, 7, 512), (5, 5, 3, 32)])
def test_split_attention_8wide_bit_identical(dev, n, h, w, C):
    """The 8-channel bf16 combine and backward apply (splat_combine_bn8_k, splat_bwd_apply_bn8_k:
    both radix halves per thread, coefficients in registers) against the 4-wide forms (the same
    y handed over 8 bytes off a 16-B boundary, which the 8-wide kernels do not take): the same
    arithmetic per element, so out and dy bit-identical."""
    from tests.test_stem_pool8_gpu import _off8
    from tmrnet_amd.resnest import SplAtConv2d, _splat_fwd, _splat_bwd
    torch.manual_seed(3 * C + h)
    md = SplAtConv2d(C, C).to(dev).train()
    y = (torch.randn(n, h, w, 2 * C) + 0.2).to(dev).to(torch.bfloat16)
    gy = torch.randn(n, h, w, C).to(dev)
    bn0 = md.bn0
    mean, inv, sc, sh = ops.bn_fwd_train(y.float().view(-1, 2 * C), bn0.weight.detach(),
                                         bn0.bias.detach(), bn0.running_mean, bn0.running_var,
                                         bn0.momentum, bn0.eps)
    r2 = {"y": y, "scale": sc, "shift": sh, "mean": mean, "inv": inv}
    outs, dys = [], []
    for yy in (y, _off8(y)):
        r2["y"] = yy
        out, spl = _splat_fwd(md, yy, sc, sh, [])
        outs.append(out)
        dys.append(_splat_bwd(md, spl, r2, gy, {}))
    torch.cuda.synchronize()
    assert outs[0].dtype == torch.bfloat16 and torch.equal(outs[0], outs[1])
    assert dys[0].dtype == torch.bfloat16 and torch.equal(dys[0], dys[1])
