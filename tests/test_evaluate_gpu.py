"""Eval loop (tmrnet_amd/evaluate.PhaseEvaluator) vs the oracle restatement of
eval/python/test_singlenet_phase_non-local_pretrained_2fc_copy_mutiConv6_3.py:449-492:
eval-mode logits -> nn.Softmax -> torch.max -> weighted CE-sum on the probabilities."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

import tmrnet_amd
from tmrnet_amd import ops, evaluate
from tmrnet_amd.lfb import LongFeatureBank
from oracle import tmrnet_ref as ref

pytestmark = pytest.mark.gpu


def test_softmax_max_kernel(dev):
    g = torch.Generator().manual_seed(0)
    x = torch.randn(1000, 7, generator=g) * 5
    x[3] = 1.0                                   # ties: first index wins, like ce_sum / torch.max
    probs, pmax, preds = ops.softmax_max(x.to(dev))
    p_ref = torch.softmax(x.double(), 1)
    assert (probs.cpu().double() - p_ref).abs().max().item() < 1e-6
    assert (pmax.cpu().double() - p_ref.max(1).values).abs().max().item() < 1e-6
    assert torch.equal(preds.cpu(), x.argmax(1))
    assert preds[3].item() == 0


def test_phase_evaluator_matches_reference_loop(dev):
    T, L, B = 3, 5, 4
    torch.manual_seed(0)
    m = tmrnet_amd.resnet_lstm(seq_len=T).to(dev).eval()
    r = ref.TMRNetRef(seq_len=T).eval()
    r.load_state_dict({k: v.detach().cpu() for k, v in m.state_dict().items()})
    g = torch.Generator().manual_seed(1)
    lengths = [20, 15]
    valid = ref.get_useful_start_idx(T, lengths)
    bank_np = (torch.rand(len(valid), 512, generator=g) * 2 - 1)
    bank = LongFeatureBank(bank_np, valid, L, dev)
    weight = torch.tensor([0.5, 1.0, 2.0, 1.5, 0.7, 1.2, 0.9])
    evl = evaluate.PhaseEvaluator(m, bank, weight=weight.to(dev))
    rng = np.random.default_rng(3)
    loss_ref, preds_ref, scores_ref, labels_all = 0.0, [], [], []
    for it in range(3):
        starts = rng.choice(valid, size=B, replace=False)
        frames = torch.randint(0, 256, (B * T, 250, 250, 3), generator=g, dtype=torch.uint8)
        off = torch.full((B, 2), 13, dtype=torch.int32)
        labels = torch.randint(0, 7, (B * T,), generator=g)
        x4 = ops.crop_normalize(frames.to(dev), off.to(dev), T)
        evl.step(x4, labels.to(dev), clip_starts=starts)
        # oracle: the reference loop body
        lt = bank_np[torch.tensor(ref.lfb_index_table(starts, valid, L))]
        with torch.no_grad():
            out = r(ref.crop_normalize_ref(frames, off, T).view(B, T, 3, 224, 224), lt)
        probs = torch.softmax(out, 1)
        poss, pr = torch.max(probs, 1)
        lab = labels[T - 1::T]
        loss_ref += F.cross_entropy(probs, lab, weight=weight, reduction="sum").item()
        preds_ref += pr.tolist(); scores_ref += poss.tolist(); labels_all += lab.tolist()
    res = evl.result()
    assert list(res["preds"]) == preds_ref
    assert np.abs(res["scores"] - np.array(scores_ref)).max() < 1e-5
    assert res["loss_sum"] == pytest.approx(loss_ref, rel=1e-5)
    acc_ref = np.mean(np.array(preds_ref) == np.array(labels_all))
    assert res["accuracy"] == pytest.approx(acc_ref)
    assert res["average_loss"] == pytest.approx(loss_ref / len(preds_ref), rel=1e-5)
