"""The wave-specialised persistent fused BN-backward dgrad (gemm16_ws.h, round 6) against the
one-tile-per-workgroup engine launch it replaces (TMR_IO_TILES, ops.dgrad_tile_launches()).

The 1x1 stride-1 dgrads of the train step in their own forms: the Bottleneck conv1 dgrads adding
into the residual-stream gradient (bf16: y, z, the old gradient in place and g bf16; fp32: ReLU
bits, the fp32 old gradient), K <= 256 (bf16) / 128 (fp32).  Both launches
run the same MFMA sequence per output element, so dx must match bit for bit; the partials too where
the engine would use the 4-wave 128x128 tile (the same thread -> row map and summation order), and
to summation-order tolerance where it would use the 8-wave one (fp32, N >= 512), both against
float64 sums of the returned gradient.  Each case is sized past the kernel's 512-tile threshold
with a partial last m-tile, and checks (tmr_dgrad_ws_launches) that the new kernel really ran.
Reference: the backward of torchvision Bottleneck.conv1 + the previous block's bn3 + relu that
code/Training TMRNet/train_only_non-local_pretrained.py:724-725 (loss.backward) runs.
"""
import os

import numpy as np
import pytest
import torch

from tmrnet_amd import ops
from tmrnet_amd._lib import lib

pytestmark = pytest.mark.gpu


def _pack_bits(m):
    m = m.reshape(-1).to(torch.int64)
    m = torch.cat([m, m.new_zeros((-m.numel()) % 32)]).view(-1, 32)
    w = (m << torch.arange(32, dtype=torch.int64, device=m.device)).sum(1)
    return torch.where(w >= 2 ** 31, w - 2 ** 32, w).to(torch.int32)


def _launches():
    return int(lib().tmr_dgrad_ws_launches())


# (prec, kind, frames, h, dx channels N, dy channels K); M = frames * h * h is not a multiple of 128
CASES = [
    ("bf16", "res", 11, 56, 256, 64),     # layer1 conv1 dgrad: one k-tile
    ("bf16", "res", 21, 28, 512, 128),    # layer2: two k-tiles
    ("bf16", "res", 43, 14, 1024, 256),   # layer3: four k-tiles
    ("fp32", "res", 11, 56, 256, 64),     # fp32 (32-float k-tiles): two
    ("fp32", "res", 21, 28, 512, 128),    # four; the engine's 8-wave tile (partials reordered)
]


@pytest.mark.parametrize("case", CASES, ids=lambda c: "%s-%s-%dx%d-%d<-%d" % (c[0], c[1], c[3], c[3], c[4], c[5]))
def test_dgrad_ws_vs_tiles(dev, case):
    prec, kind, F, h, n, k = case
    bf = prec == "bf16"
    dt = torch.bfloat16 if bf else torch.float32
    g = torch.Generator().manual_seed(31)
    dy = (torch.randn(F, h, h, k, generator=g) * 0.5).to(dev).to(dt)
    w = (torch.randn(k, n, 1, 1, generator=g) / np.sqrt(k)).to(dev)
    wct = ops.weight_to_crsk(w, bf16=bf)
    y = torch.randn(F, h, h, n, generator=g).to(dev).to(dt)
    ye = y.float()
    mean = ye.view(-1, n).mean(0)
    kw = dict(math=prec, wt=True, beta=1.0)
    z = torch.relu(ye + torch.randn(F, h, h, n, generator=g).to(dev) * 0.5)
    old = torch.randn(F, h, h, n, generator=g).to(dev).to(dt)
    if bf:
        zm, mask = z.to(dt), 1
        kw.update(g16=True)
    else:
        zm, mask = _pack_bits(z > 0), 3
    kw.update(z=zm)

    def run(tiles):
        o = old.clone()
        if tiles:
            with ops.dgrad_tile_launches():
                return ops.conv_dgrad_bnbwd(dy, wct, (h, h), 1, 0, y, mean, mask, out=o, **kw)
        return ops.conv_dgrad_bnbwd(dy, wct, (h, h), 1, 0, y, mean, mask, out=o, **kw)

    n0 = _launches()
    ref, pref, npref = run(True)
    torch.cuda.synchronize()
    assert _launches() == n0, "TMR_IO_TILES must keep the one-tile-per-workgroup launch"
    got, pgot, npgot = run(False)
    torch.cuda.synchronize()
    assert _launches() == n0 + 1, "the wave-specialised dgrad did not serve this shape"
    assert npgot == npref
    assert torch.equal(got, ref)
    a, b = pgot[:npgot], pref[:npref]
    eight_wave = (not bf) and n >= 512
    if not eight_wave:
        assert torch.equal(a, b)
    else:
        scale = b.abs().amax(0, keepdim=True) + 1e-6
        assert ((a - b).abs() / scale).max().item() < 1e-5
    gd = got.double().view(-1, n)
    want = torch.stack([gd.sum(0), (gd * (ye.double().view(-1, n) - mean.double())).sum(0)], -1)
    tot = a.double().sum(0)
    assert (tot - want).abs().max().item() <= 1e-5 * want.abs().max().item() + 1e-6


def test_dgrad_ws_small_launch_stays_tiled(dev):
    """Below the 512-tile threshold the engine's own launch runs (as for the shapes the kernel
    does not take: 3x3, strided, the MFMA-bound fp32 K >= 256 -- below)."""
    g = torch.Generator().manual_seed(5)
    F, h, n, k = 2, 14, 256, 64
    dy = torch.randn(F, h, h, k, generator=g).to(dev).to(torch.bfloat16)
    wct = ops.weight_to_crsk((torch.randn(k, n, 1, 1, generator=g) / 8).to(dev))
    y = torch.randn(F, h, h, n, generator=g).to(dev).to(torch.bfloat16)
    z = torch.relu(y.float()).to(torch.bfloat16)
    old = torch.randn(F, h, h, n, generator=g).to(dev).to(torch.bfloat16)
    n0 = _launches()
    ops.conv_dgrad_bnbwd(dy, wct, (h, h), 1, 0, y, y.float().view(-1, n).mean(0), 1, z=z,
                         out=old, beta=1.0, math="bf16", wt=True, g16=True)
    torch.cuda.synchronize()
    assert _launches() == n0


@pytest.mark.skipif(os.environ.get("TMR_DGRAD_WS_MFMA", "0") != "0",
                    reason="TMR_DGRAD_WS_MFMA widens the kernel's scope to these shapes")
def test_dgrad_ws_mfma_bound_stays_tiled(dev):
    """fp32 K = 256 (14x14 1024<-256, 8 k-tiles): MFMA-bound, left to the engine's tiles."""
    g = torch.Generator().manual_seed(6)
    F, h, n, k = 43, 14, 1024, 256
    dy = torch.randn(F, h, h, k, generator=g).to(dev)
    wct = ops.weight_to_crsk((torch.randn(k, n, 1, 1, generator=g) / 16).to(dev), bf16=False)
    y = torch.randn(F, h, h, n, generator=g).to(dev)
    bits = _pack_bits(y > 0)
    old = torch.randn(F, h, h, n, generator=g).to(dev)
    n0 = _launches()
    ops.conv_dgrad_bnbwd(dy, wct, (h, h), 1, 0, y, y.view(-1, n).mean(0), 3, z=bits, out=old,
                         beta=1.0, math="fp32", wt=True)
    torch.cuda.synchronize()
    assert _launches() == n0


WIDE = [
    ("fp32", "res", 43, 14, 1024, 256),   # eight k-tiles
    ("fp32", "res", 85, 7, 2048, 512),    # sixteen, 16 n-tiles
]


@pytest.mark.skipif(os.environ.get("TMR_DGRAD_WS_MFMA", "0") == "0",
                    reason="the MFMA-bound fp32 shapes run on the engine's tiles by default")
@pytest.mark.parametrize("case", WIDE, ids=lambda c: "%s-%dx%d-%d<-%d" % (c[0], c[3], c[3], c[4], c[5]))
def test_dgrad_ws_wide_scope(dev, case):
    """TMR_DGRAD_WS_MFMA=1 (A/B of the wider scope): the fp32 K >= 256 residual dgrads on the
    wave-specialised kernel, against the one-tile launch."""
    test_dgrad_ws_vs_tiles(dev, case)
