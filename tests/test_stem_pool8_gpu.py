"""The 8-channel forms of the stem's maxpool forward (maxpool_fwd_bn8; bf16 and, since round 5, fp32 y), of its
BatchNorm/maxpool backward apply (stem_bwd_apply8q, per 2x2 input quad; fp32 y too) and of the bf16 BN applies
(bn_apply8_a16_k) against the 4-channel forms the library falls back to: the 8-wide kernels need
16-B aligned tensors, so the same values handed over 8 bytes off a 16-B boundary take the 4-wide
form (no environment switch).  Bit-identical outputs, argmax and gradients, including ties
(quantised inputs: the first maximum in scan order must win), odd spatial sizes (partial windows
at the right / bottom edges) and a channel count that takes the 4-wide form either way; plus
float64 checks of the values."""
import pytest
import torch

from tmrnet_amd import ops

pytestmark = pytest.mark.gpu


def _off8(t):
    """A copy of t whose data starts 8 bytes past a 16-B boundary (contiguous, same values)."""
    n = t.numel()
    per = 8 // t.element_size()
    buf = torch.empty(n + 2 * per, dtype=t.dtype, device=t.device)
    base = (buf.data_ptr() // t.element_size()) % (16 // t.element_size())
    start = (per - base) % (16 // t.element_size())
    v = buf[start:start + n].view(t.shape)
    v.copy_(t)
    assert v.data_ptr() % 16 == 8 and v.is_contiguous()
    return v


def _stem_case(dev, n, h, w, c, seed, dtype=torch.bfloat16):
    g = torch.Generator().manual_seed(seed)
    # quantised to a few levels: many equal values inside a window (ties)
    y = (torch.randint(-6, 7, (n, h, w, c), generator=g).float() / 4).to(dtype).to(dev)
    scale = (torch.rand(c, generator=g) + 0.5).to(dev)
    shift = (torch.randn(c, generator=g) * 0.2).to(dev)
    return y, scale, shift


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("shape", [(3, 112, 112, 64), (2, 13, 11, 16), (2, 9, 10, 24)])
def test_maxpool_fwd_bn8_bit_identical(dev, shape, dtype):
    """(fp32 y in and out: the fp32 step's stem takes the 8-channel form since round 5.)"""
    y, scale, shift = _stem_case(dev, *shape, seed=sum(shape), dtype=dtype)
    p8, a8 = ops.maxpool_fwd_bn(y, scale, shift)
    p4, a4 = ops.maxpool_fwd_bn(_off8(y), scale, shift)    # the 4-wide form
    assert p8.dtype == dtype
    assert torch.equal(p8.view(torch.int16), p4.view(torch.int16))
    assert torch.equal(a8, a4)
    # the values are relu(bn(y)) maxima of the windows, argmax inside the window at a maximum
    # (float64 products: the kernels' single-rounding fmaf)
    z = torch.relu((y.double() * scale.double() + shift.double()).float())
    ref = torch.nn.functional.max_pool2d(z.permute(0, 3, 1, 2), 3, 2, 1).permute(0, 2, 3, 1)
    if dtype == torch.bfloat16:
        assert torch.equal(p8.float(), ref.to(torch.bfloat16).float())
    else:
        assert torch.allclose(p8, ref, rtol=1e-6, atol=1e-7)
    assert int(a8.max()) <= 8
    n, h, w, c = shape
    ho, wo = a8.shape[1], a8.shape[2]
    zp = torch.nn.functional.pad(z.permute(0, 3, 1, 2), (1, 1, 1, 1), value=-1.0)
    ids = a8.long().permute(0, 3, 1, 2)
    oy = torch.arange(ho, device=dev).view(1, 1, ho, 1) * 2
    ox = torch.arange(wo, device=dev).view(1, 1, 1, wo) * 2
    nn_ = torch.arange(n, device=dev).view(n, 1, 1, 1).expand_as(ids)
    cc = torch.arange(c, device=dev).view(1, c, 1, 1).expand_as(ids)
    picked = zp[nn_, cc, oy + ids // 3, ox + ids % 3]
    assert torch.allclose(picked.to(dtype).float(), ref.permute(0, 3, 1, 2).to(dtype).float(),
                          rtol=1e-6, atol=1e-7)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("shape", [(3, 112, 112, 64), (2, 13, 11, 16), (2, 12, 9, 8), (2, 9, 10, 24)])
def test_stem_bwd_apply8_bit_identical(dev, shape, dtype):
    """(fp32 y: the fp32 step's stem takes the same quad form since round 5.)"""
    n, h, w, c = shape
    y, scale, shift = _stem_case(dev, *shape, seed=7 + sum(shape), dtype=dtype)
    _, am = ops.maxpool_fwd_bn(y, scale, shift)
    ho, wo = am.shape[1], am.shape[2]
    g = torch.Generator().manual_seed(11)
    dyp = torch.randn(n, ho, wo, c, generator=g).to(dev)
    mean = y.float().mean((0, 1, 2))
    inv = 1.0 / (y.float().var((0, 1, 2), unbiased=False) + 1e-5).sqrt()
    gamma = (torch.rand(c, generator=g) + 0.5).to(dev)
    d8, g8, b8 = ops.bn_bwd_maxpool(dyp, am, y, scale, shift, mean, inv, gamma)
    # the 4-wide, one-pixel-per-thread form against the default 8-channel 2x2-quad form
    d4, g4, b4 = ops.bn_bwd_maxpool(dyp, am, _off8(y), scale, shift, mean, inv, gamma)
    assert torch.equal(d8.view(torch.int16), d4.view(torch.int16))   # (fp32: both halves)
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
    assert torch.allclose(b8.double(), sdz, rtol=1e-4, atol=1e-3)
    assert torch.allclose(g8.double(), sdx, rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("rows,c", [(3 * 56 * 56, 256), (1001, 64), (37, 24)])
def test_bn_apply8_a16_bit_identical(dev, rows, c):
    """bf16 BN applies (relu(bn(y)), relu(bn(y) + residual), relu(bn(y) + bn_ds(y_ds))) 8 per
    thread (bn_apply8_a16_k) vs the 4-wide forms (misaligned operands): identical bytes; c = 24
    takes the 4-wide form in both runs.  Values against float64 within one bf16 rounding."""
    g = torch.Generator().manual_seed(rows + c)
    mk = lambda: (torch.randn(rows, c, generator=g) * 2).to(torch.bfloat16).to(dev)
    y, r, yr = mk(), mk(), mk()
    sc, sf, rs, rf = [(torch.rand(c, generator=g) + 0.5).to(dev) for _ in range(4)]
    outs = {}
    for form, (yy, rr, yyr) in (("8", (y, r, yr)), ("4", (_off8(y), _off8(r), _off8(yr)))):
        outs[form] = [ops.bn_apply(yy, sc, sf), ops.bn_apply(yy, sc, sf, residual=rr),
                      ops.bn_apply(yy, sc, sf, residual=rr, relu=False),
                      ops.bn_apply2(yy, sc, sf, yyr, rs, rf),
                      ops.bn_apply2(yy, sc, sf, yyr, rs, rf, relu=False)]
    for a, b in zip(outs["8"], outs["4"]):
        assert torch.equal(a.view(torch.int16), b.view(torch.int16))
    yd, rd, yrd = y.double(), r.double(), yr.double()
    bn = yd * sc.double() + sf.double()
    bnr = yrd * rs.double() + rf.double()
    refs = [torch.relu(bn), torch.relu(bn + rd), bn + rd, torch.relu(bn + bnr), bn + bnr]
    for got, ref in zip(outs["8"], refs):
        assert torch.allclose(got.double(), ref, rtol=1e-2, atol=1e-2)   # one bf16 rounding
