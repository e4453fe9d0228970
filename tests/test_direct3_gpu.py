"""The direct 3x3 stride-1 kernels of the bf16 step's narrow 112x112 convs (direct3.hip: ResNeSt-50's
deep-stem 32 -> 32 and 32 -> 64 convs, third-party resnest50() at
train_non-local_mutiConv_resnest.py:210) against float64 of the same bf16 operands and against the
implicit-GEMM engine (ops.engine_only, TMR_IO_ENGINE).

Sixteen frames = 1792 output rows over 512-768 persistent workgroups: each takes a contiguous range
of 2-4 rows, so the input-row ring is reused within a range, ranges cross frame boundaries (the
zero rows above / below a frame) and the statistics / partial sums are merged over a range."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from tmrnet_amd import ops

pytestmark = pytest.mark.gpu
N = 16


@pytest.fixture(scope="module")
def dev():
    return torch.device("cuda:0")


def rel_err(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return ((a - b).norm() / (b.norm() + 1e-30)).item()


def _bf(t):
    return t.to(torch.bfloat16)


def _ulp_bound(y, ref, k=1.0):
    ulp = 2.0 ** (torch.floor(torch.log2(ref.abs().clamp_min(1e-30))) - 7)
    floor = 1e-6 * ref.abs().max().item()
    return ((y - ref).abs() <= k * ulp * 1.0001 + k * floor).all().item()


@pytest.mark.parametrize("cout", [32, 64])
def test_direct3_fwd_bnstats(dev, monkeypatch, cout, engine):
    """y = conv(x) stored bf16: within one bf16 ulp of float64 of the bf16 operands (plus the fp32
    accumulation floor), within two of the engine; BatchNorm statistics of the stored values."""
    g = torch.Generator().manual_seed(40 + cout)
    x = _bf(torch.relu(torch.randn(N, 112, 112, 32, generator=g)))
    w = _bf(torch.randn(cout, 32, 3, 3, generator=g) / np.sqrt(288))
    xd = x.to(dev)
    wk = ops.weight_to_krsc(w.float().to(dev).contiguous(), bf16=True)
    engine.use(False)
    y, stats, nparts = ops.conv_fwd_bnstats(xd, wk, 1, 1, math="bf16", y16=True)
    engine.use(True)
    y0, st0, np0 = ops.conv_fwd_bnstats(xd, wk, 1, 1, math="bf16", y16=True)
    torch.cuda.synchronize()
    assert y.dtype == torch.bfloat16 and tuple(y.shape) == (N, 112, 112, cout)
    assert nparts == (512 * 2 if cout == 64 else 768 * 4) and np0 != nparts   # workgroups x WM
    ref = F.conv2d(x.permute(0, 3, 1, 2).double(), w.double(), padding=1).permute(0, 2, 3, 1)
    yf = y.double().cpu()
    assert _ulp_bound(yf, ref)
    assert _ulp_bound(yf, y0.double().cpu(), 2.0)
    yd = yf.reshape(-1, cout)
    ones, zeros = torch.ones(cout, device=dev), torch.zeros(cout, device=dev)
    mean, inv, _, _ = ops.bn_finalize(stats, nparts, ones, zeros, zeros.clone(), ones.clone(), 0.1, 1e-5)
    assert rel_err(mean, yd.mean(0)) < 1e-6
    assert rel_err(inv, 1 / torch.sqrt(yd.var(0, unbiased=False) + 1e-5)) < 1e-5


@pytest.mark.parametrize("cout", [32, 64])
@pytest.mark.parametrize("mask,beta", [(2, 0.0), (1, 0.0), (0, 1.0)])
def test_direct3_dgrad_bnbwd(dev, monkeypatch, cout, mask, beta, engine):
    """dx = conv_transpose(dy) on the transposed bf16 weights, masked by the previous unit's ReLU
    (mask 1: z > 0, 2: y * scale + shift > 0; 0: none, with beta * old dx), and the partial sums
    sum(g), sum(g * (y - mean)) per channel: against float64 and against the engine."""
    g = torch.Generator().manual_seed(50 + cout + 7 * mask)
    dy = _bf(torch.randn(N, 112, 112, cout, generator=g))
    w = _bf(torch.randn(cout, 32, 3, 3, generator=g) / np.sqrt(9 * cout))
    y = _bf(torch.randn(N, 112, 112, 32, generator=g))
    z = _bf(torch.relu(torch.randn(N, 112, 112, 32, generator=g)))
    scale = torch.rand(32, generator=g) + 0.5
    shift = torch.randn(32, generator=g) * 0.3
    mean = torch.randn(32, generator=g) * 0.1
    old = torch.randn(N, 112, 112, 32, generator=g)
    wt = ops.weight_to_crsk(w.float().to(dev).contiguous())
    args = dict(z=z.to(dev) if mask == 1 else None, scale=scale.to(dev), shift=shift.to(dev),
                beta=beta, math="bf16", wt=True)
    outs = []
    for direct in ("1", "0"):
        engine.use(direct == "0")
        dx, parts, nparts = ops.conv_dgrad_bnbwd(dy.to(dev), wt, (112, 112), 1, 1, y.to(dev),
                                                 mean.to(dev), mask, out=old.to(dev).clone(), **args)
        outs.append((dx, parts[:nparts].double().sum(0).cpu(), nparts))
    torch.cuda.synchronize()
    ref = F.conv_transpose2d(dy.permute(0, 3, 1, 2).double(), w.double(), padding=1)
    ref = ref.permute(0, 2, 3, 1) + beta * old.double()
    yd = y.double()
    keep = {0: torch.ones_like(yd, dtype=torch.bool), 1: z.double() > 0,
            2: yd * scale.double() + shift.double() > 0}[mask]
    ref = torch.where(keep, ref, torch.zeros_like(ref))
    (dx, ps, npd), (dx0, ps0, _) = outs
    assert npd == (512 if cout == 64 else 512)
    assert rel_err(dx, ref) < 2e-6 and rel_err(dx0, ref) < 2e-6
    gd = dx.double().cpu().reshape(-1, 32)
    s_ref = gd.sum(0)
    q_ref = (gd * (yd.reshape(-1, 32) - mean.double())).sum(0)
    assert rel_err(ps[:, 0], s_ref) < 1e-5 and rel_err(ps[:, 1], q_ref) < 1e-5
    assert rel_err(ps, ps0) < 1e-5


@pytest.mark.parametrize("cout", [32, 64])
def test_direct3_wgrad(dev, monkeypatch, cout, engine):
    """dW = sum over pixels of dy^T x per tap (ds_read_b64_tr_b16 fragments of both [pixel][channel]
    rows, slabs reduced in a fixed order): against float64 of the bf16 operands, with beta
    accumulation, and against the engine."""
    g = torch.Generator().manual_seed(60 + cout)
    x = _bf(torch.relu(torch.randn(N, 112, 112, 32, generator=g)))
    dy = _bf(torch.randn(N, 112, 112, cout, generator=g))
    ref = torch.nn.grad.conv2d_weight(x.permute(0, 3, 1, 2).double(), (cout, 32, 3, 3),
                                      dy.permute(0, 3, 1, 2).double(), padding=1)
    xd, dyd = x.to(dev), dy.to(dev)
    engine.use(False)
    dw = ops.conv_wgrad(xd, dyd, 3, 3, 1, 1, math="bf16")
    prev = torch.randn(cout, 32, 3, 3, generator=g).to(dev)
    acc = ops.conv_wgrad(xd, dyd, 3, 3, 1, 1, math="bf16", out=prev.clone(), beta=0.5)
    engine.use(True)
    dw0 = ops.conv_wgrad(xd, dyd, 3, 3, 1, 1, math="bf16")
    torch.cuda.synchronize()
    assert rel_err(dw, ref) < 2e-6 and rel_err(dw0, ref) < 2e-6
    assert rel_err(acc, 0.5 * prev.double().cpu() + ref) < 2e-6


def test_direct3_small_frames(dev, monkeypatch, engine):
    """Fewer rows than workgroups (one 112-row frame: every workgroup one row, no reuse) and a
    short frame height (h = 5: every row range touches a frame edge)."""
    g = torch.Generator().manual_seed(70)
    for n, hh in ((1, 112), (7, 5)):
        x = _bf(torch.randn(n, hh, 112, 32, generator=g))
        w = _bf(torch.randn(64, 32, 3, 3, generator=g) / np.sqrt(288))
        wk = ops.weight_to_krsc(w.float().to(dev).contiguous(), bf16=True)
        engine.use(False)
        y, stats, nparts = ops.conv_fwd_bnstats(x.to(dev), wk, 1, 1, math="bf16", y16=True)
        dy = _bf(torch.randn(n, hh, 112, 64, generator=g))
        dw = ops.conv_wgrad(x.to(dev), dy.to(dev), 3, 3, 1, 1, math="bf16")
        torch.cuda.synchronize()
        ref = F.conv2d(x.permute(0, 3, 1, 2).double(), w.double(), padding=1).permute(0, 2, 3, 1)
        assert _ulp_bound(y.double().cpu(), ref)
        assert nparts == min(n * hh, 512) * 2
        rw = torch.nn.grad.conv2d_weight(x.permute(0, 3, 1, 2).double(), (64, 32, 3, 3),
                                         dy.permute(0, 3, 1, 2).double(), padding=1)
        assert rel_err(dw, rw) < 2e-6


def test_direct3_stem_fwd_bnstats(dev, monkeypatch, engine):
    """The deep stem's first conv (3x3/2, 3 -> 32) from the NHWC4 fp32 frames, 3 channels packed
    per column: within one bf16 ulp of float64 of the bf16-rounded operands, within two of the
    LDS-DMA engine on the NHWC8 copy; BatchNorm statistics of the stored values."""
    g = torch.Generator().manual_seed(80)
    x = torch.relu(torch.randn(N, 3, 224, 224, generator=g)) + 0.25
    w = torch.randn(32, 3, 3, 3, generator=g) / np.sqrt(27)
    x4 = ops.nchw_to_nhwc(x.to(dev), cpad=4)
    wk4 = ops.weight_to_krsc(w.to(dev).contiguous(), cpad=4, bf16=True)
    engine.use(False)
    y, stats, nparts = ops.conv_fwd_bnstats(x4, wk4, 2, 1, c_real=3, math="bf16", y16=True)
    engine.use(True)
    x8 = ops.nhwc4_to_bf16x8(x4)
    wk8 = ops.weight_to_krsc(w.to(dev).contiguous(), cpad=8, bf16=True)
    y0, _, _ = ops.conv_fwd_bnstats(x8, wk8, 2, 1, c_real=3, math="bf16", y16=True)
    torch.cuda.synchronize()
    assert y.dtype == torch.bfloat16 and tuple(y.shape) == (N, 112, 112, 32)
    assert nparts == 4 * 768
    ref = F.conv2d(_bf(x).double(), _bf(w).double(), stride=2, padding=1).permute(0, 2, 3, 1)
    yf = y.double().cpu()
    assert _ulp_bound(yf, ref)
    assert _ulp_bound(yf, y0.double().cpu(), 2.0)
    yd = yf.reshape(-1, 32)
    ones, zeros = torch.ones(32, device=dev), torch.zeros(32, device=dev)
    mean, inv, _, _ = ops.bn_finalize(stats, nparts, ones, zeros, zeros.clone(), ones.clone(), 0.1, 1e-5)
    assert rel_err(mean, yd.mean(0)) < 1e-6
    assert rel_err(inv, 1 / torch.sqrt(yd.var(0, unbiased=False) + 1e-5)) < 1e-5


def test_direct3_stem_wgrad(dev, monkeypatch, engine):
    """Its weight gradient (per input row im2col columns transposed in LDS, dy by transposed reads):
    against float64 of the bf16 operands, with beta accumulation, and against the engine."""
    g = torch.Generator().manual_seed(81)
    x = torch.relu(torch.randn(N, 3, 224, 224, generator=g)) + 0.25
    dy = _bf(torch.randn(N, 112, 112, 32, generator=g))
    x4 = ops.nchw_to_nhwc(x.to(dev), cpad=4)
    ref = torch.nn.grad.conv2d_weight(_bf(x).double(), (32, 3, 3, 3),
                                      dy.permute(0, 3, 1, 2).double(), stride=2, padding=1)
    engine.use(False)
    dw = ops.conv_wgrad(x4, dy.to(dev), 3, 3, 2, 1, c_real=3, math="bf16")
    prev = torch.randn(32, 3, 3, 3, generator=g).to(dev)
    acc = ops.conv_wgrad(x4, dy.to(dev), 3, 3, 2, 1, c_real=3, math="bf16", out=prev.clone(),
                         beta=0.5)
    engine.use(True)
    dw0 = ops.conv_wgrad(x4, dy.to(dev), 3, 3, 2, 1, c_real=3, math="bf16")
    torch.cuda.synchronize()
    assert rel_err(dw, ref) < 2e-6 and rel_err(dw0, ref) < 2e-6
    assert rel_err(acc, 0.5 * prev.double().cpu() + ref) < 2e-6


W56 = 8   # frames of the 56x56 cases: 448 rows over 384-512 workgroups (ranges of 1-2 rows)


def test_direct3_w56_fwd_bnstats(dev, monkeypatch, engine):
    """ResNet-50 layer1's 3x3 64 -> 64 conv at 56x56 (C5, bf16): 3.5 m-tiles of 16 pixels per row
    (the last half empty: zeros, not counted in the statistics)."""
    g = torch.Generator().manual_seed(90)
    x = _bf(torch.relu(torch.randn(W56, 56, 56, 64, generator=g)))
    w = _bf(torch.randn(64, 64, 3, 3, generator=g) / np.sqrt(576))
    wk = ops.weight_to_krsc(w.float().to(dev).contiguous(), bf16=True)
    engine.use(False)
    y, stats, nparts = ops.conv_fwd_bnstats(x.to(dev), wk, 1, 1, math="bf16", y16=True)
    engine.use(True)
    y0, _, np0 = ops.conv_fwd_bnstats(x.to(dev), wk, 1, 1, math="bf16", y16=True)
    torch.cuda.synchronize()
    assert nparts == min(W56 * 56, 768) and np0 != nparts
    ref = F.conv2d(x.permute(0, 3, 1, 2).double(), w.double(), padding=1).permute(0, 2, 3, 1)
    yf = y.double().cpu()
    assert _ulp_bound(yf, ref) and _ulp_bound(yf, y0.double().cpu(), 2.0)
    yd = yf.reshape(-1, 64)
    ones, zeros = torch.ones(64, device=dev), torch.zeros(64, device=dev)
    mean, inv, _, _ = ops.bn_finalize(stats, nparts, ones, zeros, zeros.clone(), ones.clone(), 0.1, 1e-5)
    assert rel_err(mean, yd.mean(0)) < 1e-6
    assert rel_err(inv, 1 / torch.sqrt(yd.var(0, unbiased=False) + 1e-5)) < 1e-5


@pytest.mark.parametrize("g16,mask,beta", [(True, 2, 0.0), (False, 2, 0.0), (False, 1, 0.0),
                                           (False, 0, 1.0)])
def test_direct3_w56_dgrad_bnbwd(dev, monkeypatch, g16, mask, beta, engine):
    """Its dgrad with the fused BatchNorm backward of bn1; g16: the masked gradient stored bf16
    (TMR_IO_G16, the C5 step's contract) with the partial sums of the stored values."""
    g = torch.Generator().manual_seed(91 + mask)
    dy = _bf(torch.randn(W56, 56, 56, 64, generator=g))
    w = _bf(torch.randn(64, 64, 3, 3, generator=g) / np.sqrt(576))
    y = _bf(torch.randn(W56, 56, 56, 64, generator=g))
    z = _bf(torch.relu(torch.randn(W56, 56, 56, 64, generator=g)))
    scale = torch.rand(64, generator=g) + 0.5
    shift = torch.randn(64, generator=g) * 0.3
    mean = torch.randn(64, generator=g) * 0.1
    old = torch.randn(W56, 56, 56, 64, generator=g)
    wt = ops.weight_to_crsk(w.float().to(dev).contiguous())
    outs = []
    for direct in ("1", "0"):
        engine.use(direct == "0")
        dx, parts, nparts = ops.conv_dgrad_bnbwd(
            dy.to(dev), wt, (56, 56), 1, 1, y.to(dev), mean.to(dev), mask,
            z=z.to(dev) if mask == 1 else None, scale=scale.to(dev), shift=shift.to(dev),
            out=None if g16 else old.to(dev).clone(), beta=beta, math="bf16", wt=True, g16=g16)
        outs.append((dx, parts[:nparts].double().sum(0).cpu(), nparts))
    torch.cuda.synchronize()
    ref = F.conv_transpose2d(dy.permute(0, 3, 1, 2).double(), w.double(), padding=1)
    ref = ref.permute(0, 2, 3, 1) + beta * old.double()
    yd = y.double()
    keep = {0: torch.ones_like(yd, dtype=torch.bool), 1: z.double() > 0,
            2: yd * scale.double() + shift.double() > 0}[mask]
    ref = torch.where(keep, ref, torch.zeros_like(ref))
    (dx, ps, npd), (dx0, ps0, _) = outs
    assert npd == min(W56 * 56, 512)
    if g16:
        assert dx.dtype == torch.bfloat16
        assert _ulp_bound(dx.double().cpu(), ref) and _ulp_bound(dx.double().cpu(), dx0.double().cpu(), 2.0)
    else:
        assert rel_err(dx, ref) < 2e-6 and rel_err(dx0, ref) < 2e-6
    gd = dx.double().cpu().reshape(-1, 64)
    assert rel_err(ps[:, 0], gd.sum(0)) < 1e-5
    assert rel_err(ps[:, 1], (gd * (yd.reshape(-1, 64) - mean.double())).sum(0)) < 1e-5
    assert rel_err(ps, ps0) < (2e-3 if g16 else 1e-5)


def test_direct3_w56_wgrad(dev, monkeypatch, engine):
    """Its weight gradient: K = 56 pixels per row padded to 64, 36 accumulator tiles per wave."""
    g = torch.Generator().manual_seed(93)
    x = _bf(torch.relu(torch.randn(W56, 56, 56, 64, generator=g)))
    dy = _bf(torch.randn(W56, 56, 56, 64, generator=g))
    ref = torch.nn.grad.conv2d_weight(x.permute(0, 3, 1, 2).double(), (64, 64, 3, 3),
                                      dy.permute(0, 3, 1, 2).double(), padding=1)
    engine.use(False)
    dw = ops.conv_wgrad(x.to(dev), dy.to(dev), 3, 3, 1, 1, math="bf16")
    prev = torch.randn(64, 64, 3, 3, generator=g).to(dev)
    acc = ops.conv_wgrad(x.to(dev), dy.to(dev), 3, 3, 1, 1, math="bf16", out=prev.clone(), beta=0.5)
    engine.use(True)
    dw0 = ops.conv_wgrad(x.to(dev), dy.to(dev), 3, 3, 1, 1, math="bf16")
    torch.cuda.synchronize()
    assert rel_err(dw, ref) < 2e-6 and rel_err(dw0, ref) < 2e-6
    assert rel_err(acc, 0.5 * prev.double().cpu() + ref) < 2e-6
