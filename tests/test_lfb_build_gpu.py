"""LFB construction (tmrnet_amd/lfb_build.py) against the oracle's restatement of the
reference loop (oracle.build_lfb_ref = train_only_non-local_pretrained.py:534-607):
same seeded weights (random BN running statistics so eval-mode BN is not the identity), same
uint8 frames; bank rows are LSTM hidden states in (-1, 1), compared to 1e-4 absolute (the
north-star fp32 tolerance) with the row order = valid-start order checked exactly."""
import numpy as np
import pytest
import torch

import tmrnet_amd
from tmrnet_amd import lfb_build
from oracle import tmrnet_ref as ref

pytestmark = pytest.mark.gpu


def _randomize_bn(model, seed):
    g = torch.Generator().manual_seed(seed)
    for m in model.modules():
        if isinstance(m, torch.nn.BatchNorm2d):
            c = m.num_features
            m.running_mean.copy_(torch.randn(c, generator=g) * 0.1)
            m.running_var.copy_(torch.rand(c, generator=g) + 0.5)
            with torch.no_grad():
                m.weight.copy_(torch.rand(c, generator=g) * 0.5 + 0.25)
                m.bias.copy_(torch.randn(c, generator=g) * 0.1)


@pytest.fixture(scope="module")
def lfb_case():
    T = 3
    torch.manual_seed(0)
    r = ref.LFBModelRef(seq_len=T)
    _randomize_bn(r, 1)
    lengths = [6, 2, 5]                      # the 2-frame video has no valid start
    g = torch.Generator().manual_seed(2)
    frames = torch.randint(0, 256, (sum(lengths), 250, 250, 3), generator=g, dtype=torch.uint8)
    bank_ref, valid_ref = ref.build_lfb_ref(r, frames, lengths, batch_clips=4)
    return T, r, lengths, frames, bank_ref, valid_ref


@pytest.mark.parametrize("fpl,cpl,loader", [(640, 8192, False), (4, 3, True)])
def test_lfb_build_matches_reference_loop(dev, lfb_case, fpl, cpl, loader):
    T, r, lengths, frames, bank_ref, valid_ref = lfb_case
    m = tmrnet_amd.resnet_lstm_LFB(seq_len=T).to(dev)
    m.load_state_dict({k: v for k, v in r.state_dict().items()})
    m.train()                                   # build() must switch to eval and back
    src = (lambda f0, n: frames[f0:f0 + n]) if loader else frames.to(dev)
    bank, valid = lfb_build.build_lfb(m, src, lengths, frames_per_launch=fpl,
                                      clips_per_launch=cpl)
    torch.cuda.synchronize()
    assert m.training
    assert list(valid) == list(valid_ref)
    assert bank.shape == (len(valid_ref), 512)
    err = np.abs(bank.cpu().double().numpy() - bank_ref).max()
    assert err < 1e-4, err


def test_lfb_build_sharded_rows_match(dev, lfb_case):
    """Each rank's share (world=3, gathered by hand here) equals the corresponding rows."""
    T, r, lengths, frames, bank_ref, valid_ref = lfb_case
    m = tmrnet_amd.resnet_lstm_LFB(seq_len=T).to(dev)
    m.load_state_dict(r.state_dict())
    b = lfb_build.LFBBuilder(m)
    full, _ = b.build(frames.to(dev), lengths)
    m.eval()                                    # encode()/recur() are build()'s eval-mode stages
    valid, used, grow = lfb_build.clip_plan(T, lengths)
    for rank in range(3):
        lo, hi = lfb_build.shard_range(len(valid), rank, 3)
        g_lo, g_hi = int(grow[lo]), int(grow[hi - 1]) + T
        gates = torch.empty((g_hi - g_lo, 2048), device=dev)
        b.encode(frames.to(dev), used[g_lo:g_hi], gates)
        part = torch.empty((hi - lo, 512), device=dev)
        b.recur(gates, grow[lo:hi] - g_lo, part)
        assert (part - full[lo:hi]).abs().max().item() < 1e-5


def test_lfb_build_eval_trunk_matches_oracle(dev, lfb_case):
    """The eval-mode trunk (fused conv+BN+residual+ReLU launches) vs the oracle's eval share."""
    T, r, lengths, frames, _, _ = lfb_case
    m = tmrnet_amd.resnet_lstm_LFB(seq_len=T).to(dev).eval()
    m.load_state_dict(r.state_dict())
    x = ref.crop_normalize_ref(frames[:4], [(13, 13)], 4)
    with torch.no_grad():
        f_ref = r.eval().share(x).view(4, 2048)
        f = m.share(x.to(dev)).view(4, 2048)
    err = ((f.cpu() - f_ref).abs().max() / f_ref.abs().max()).item()
    assert err < 1e-5, err
