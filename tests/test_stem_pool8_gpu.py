"""The 8-channel forms of the bf16 stem's maxpool forward (maxpool_fwd_bn8_a16, TMR_MAXPOOL8) and
of its BatchNorm/maxpool backward apply (stem_bwd_apply8, TMR_STEM_BWD8) against the 4-channel
forms they replace: bit-identical outputs, argmax and gradients, including ties (quantised
inputs: the first maximum in scan order must win), odd spatial sizes (partial windows at the
right / bottom edges) and a channel count that takes the 4-wide fallback.  The 4-wide forms are
checked against the float64 oracle of the stem in tests/test_kernels_gpu.py / test_bf16_gpu.py."""
import pytest
import torch

from tmrnet_amd import ops

pytestmark = pytest.mark.gpu


def _stem_case(dev, n, h, w, c, seed):
    g = torch.Generator().manual_seed(seed)
    # quantised to a few levels: many equal values inside a window (ties)
    y = (torch.randint(-6, 7, (n, h, w, c), generator=g).float() / 4).to(torch.bfloat16).to(dev)
    scale = (torch.rand(c, generator=g) + 0.5).to(dev)
    shift = (torch.randn(c, generator=g) * 0.2).to(dev)
    return y, scale, shift


@pytest.mark.parametrize("shape", [(3, 112, 112, 64), (2, 13, 11, 16), (2, 9, 10, 24)])
def test_maxpool_fwd_bn8_bit_identical(dev, shape, monkeypatch):
    y, scale, shift = _stem_case(dev, *shape, seed=sum(shape))
    p8, a8 = ops.maxpool_fwd_bn(y, scale, shift)
    monkeypatch.setenv("TMR_MAXPOOL8", "0")
    p4, a4 = ops.maxpool_fwd_bn(y, scale, shift)
    monkeypatch.delenv("TMR_MAXPOOL8")
    assert torch.equal(p8.view(torch.int16), p4.view(torch.int16))
    assert torch.equal(a8, a4)
    # and the values are relu(bn(y)) maxima of the windows, argmax inside the window
    z = torch.relu(y.float() * scale + shift)
    ref = torch.nn.functional.max_pool2d(z.permute(0, 3, 1, 2), 3, 2, 1).permute(0, 2, 3, 1)
    assert torch.equal(p8.float(), ref.to(torch.bfloat16).float())
    assert int(a8.max()) <= 8


@pytest.mark.parametrize("shape", [(3, 112, 112, 64), (2, 13, 11, 16), (2, 12, 9, 8), (2, 9, 10, 24)])
def test_stem_bwd_apply8_bit_identical(dev, shape, monkeypatch):
    n, h, w, c = shape
    y, scale, shift = _stem_case(dev, *shape, seed=7 + sum(shape))
    _, am = ops.maxpool_fwd_bn(y, scale, shift)
    ho, wo = am.shape[1], am.shape[2]
    g = torch.Generator().manual_seed(11)
    dyp = torch.randn(n, ho, wo, c, generator=g).to(dev)
    mean = y.float().mean((0, 1, 2))
    inv = 1.0 / (y.float().var((0, 1, 2), unbiased=False) + 1e-5).sqrt()
    gamma = (torch.rand(c, generator=g) + 0.5).to(dev)
    d8, g8, b8 = ops.bn_bwd_maxpool(dyp, am, y, scale, shift, mean, inv, gamma)
    # the per-pixel 8-channel form (TMR_STEM_QUAD=0) against the default 2x2-quad form
    monkeypatch.setenv("TMR_STEM_QUAD", "0")
    dp_, gp_, bp_ = ops.bn_bwd_maxpool(dyp, am, y, scale, shift, mean, inv, gamma)
    monkeypatch.delenv("TMR_STEM_QUAD")
    assert torch.equal(dp_.view(torch.int16), d8.view(torch.int16))
    assert torch.equal(gp_, g8) and torch.equal(bp_, b8)
    monkeypatch.setenv("TMR_STEM_BWD8", "0")
    d4, g4, b4 = ops.bn_bwd_maxpool(dyp, am, y, scale, shift, mean, inv, gamma)
    monkeypatch.delenv("TMR_STEM_BWD8")
    assert torch.equal(d8.view(torch.int16), d4.view(torch.int16))
    assert torch.equal(g8, g4) and torch.equal(b8, b4)
    # the maxpool gradient routed through argmax, masked by the stem ReLU, then the BN backward
    ids = am.long()
    dz = torch.zeros(n, h + 2, w + 2, c, dtype=torch.float64, device=dev)
    oy = torch.arange(ho, device=dev).view(1, ho, 1, 1) * 2
    ox = torch.arange(wo, device=dev).view(1, 1, wo, 1) * 2
    iy, ix = oy + ids // 3, ox + ids % 3            # padded coordinates
    nn_ = torch.arange(n, device=dev).view(n, 1, 1, 1).expand_as(ids)
    cc = torch.arange(c, device=dev).view(1, 1, 1, c).expand_as(ids)
    dz.index_put_((nn_, iy, ix, cc), dyp.double(), accumulate=True)
    dz = dz[:, 1:h + 1, 1:w + 1]
    yd = y.double()
    dz = torch.where(yd * scale.double() + shift.double() > 0, dz, torch.zeros_like(dz))
    xh = (yd - mean.double()) * inv.double()
    m = n * h * w
    sdz, sdx = dz.sum((0, 1, 2)), (dz * xh).sum((0, 1, 2))
    ref = gamma.double() * inv.double() * (dz - sdz / m - xh * sdx / m)
    err = (d8.double() - ref).abs().max().item() / ref.abs().max().item()
    assert err < 1e-2, err    # bf16 output


@pytest.mark.parametrize("rows,c", [(3 * 56 * 56, 256), (1001, 64), (37, 24)])
def test_bn_apply8_a16_bit_identical(dev, rows, c, monkeypatch):
    """bf16 BN applies (relu(bn(y)), relu(bn(y) + residual), relu(bn(y) + bn_ds(y_ds))) 8 per
    thread (bn_apply8_a16_k) vs the 4-wide forms (TMR_BN_APPLY8=0): identical bytes; c = 24 takes
    the 4-wide form in both runs."""
    g = torch.Generator().manual_seed(rows + c)
    mk = lambda: (torch.randn(rows, c, generator=g) * 2).to(torch.bfloat16).to(dev)
    y, r, yr = mk(), mk(), mk()
    sc, sf, rs, rf = [(torch.rand(c, generator=g) + 0.5).to(dev) for _ in range(4)]
    outs = {}
    for v in ("1", "0"):
        monkeypatch.setenv("TMR_BN_APPLY8", v)
        outs[v] = [ops.bn_apply(y, sc, sf), ops.bn_apply(y, sc, sf, residual=r),
                   ops.bn_apply(y, sc, sf, residual=r, relu=False),
                   ops.bn_apply2(y, sc, sf, yr, rs, rf), ops.bn_apply2(y, sc, sf, yr, rs, rf, relu=False)]
    monkeypatch.delenv("TMR_BN_APPLY8")
    for a, b in zip(outs["1"], outs["0"]):
        assert torch.equal(a.view(torch.int16), b.view(torch.int16))
    ref = torch.relu(y.double() * sc.double() + sf.double() + r.double())
    assert torch.allclose(outs["1"][1].double(), ref, rtol=1e-2, atol=1e-2)   # one bf16 rounding
