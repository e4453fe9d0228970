"""CPU tests: the oracle (oracle/tmrnet_ref.py) pinned against the reference-generated golden
fixtures, plus host-side logic.  No GPU and no reference checkout needed."""
import os

import numpy as np
import pytest
import torch

from oracle import tmrnet_ref as ref
from tests.golden.golden_inputs import (NL_CASES, TC_CASES, nlblock_inputs, nlblock_params,
                                        project, projection_probes, timeconv_inputs,
                                        timeconv_params)

GOLD = os.path.join(os.path.dirname(__file__), "golden")


@pytest.mark.parametrize("case", NL_CASES, ids=lambda c: "L%d" % c["L"])
def test_oracle_nlblock_matches_reference_fixture(case):
    B, L, seed = case["B"], case["L"], case["seed"]
    z = np.load(os.path.join(GOLD, "nlblock_L%d.npz" % L))
    m = ref.NLBlockRef().eval()
    m.load_state_dict({k: torch.from_numpy(v) for k, v in nlblock_params(seed).items()})
    St_np, Lt_np, g_np = nlblock_inputs(seed, B, L)
    St = torch.from_numpy(St_np).requires_grad_(True)
    Lt = torch.from_numpy(Lt_np).requires_grad_(True)
    out = m(St, Lt)
    out.backward(torch.from_numpy(g_np))
    # the restatement is op-for-op the reference: identical results on CPU
    assert np.array_equal(out.detach().numpy(), z["out"])
    assert np.array_equal(St.grad.numpy(), z["dSt"])
    assert np.array_equal(Lt.grad.numpy(), z["dLt"])
    probes = projection_probes(seed, (512, 512), 16)
    for name, p in m.named_parameters():
        key = "d_" + name.replace(".", "_")
        g = p.grad.numpy()
        if g.shape == (512, 512):
            assert np.allclose(project(g, probes), z[key + "_proj"], rtol=0, atol=1e-9)
            assert np.array_equal(g[0], z[key + "_row0"])
        else:
            assert np.array_equal(g.reshape(z[key].shape), z[key])


def test_nlblock_gemv_form_matches_reference_form():
    """The re-associated GEMV form used by the HIP kernels (include/tmr.h tmr_nl_attn_fwd)
    restated in float64 equals the reference formulation."""
    case = NL_CASES[1]
    B, L, seed = case["B"], case["L"], case["seed"]
    p = {k: torch.from_numpy(v).double() for k, v in nlblock_params(seed).items()}
    St_np, Lt_np, _ = nlblock_inputs(seed, B, L)
    St, Lt = torch.from_numpy(St_np).double(), torch.from_numpy(Lt_np).double()
    q = St @ p["linear1.weight"].t() + p["linear1.bias"]
    u = q @ p["linear2.weight"]
    s = torch.einsum("bld,bd->bl", Lt, u) * (1 / 512) ** 0.5
    pr = torch.softmax(s, dim=1)
    ctx = torch.einsum("bl,bld->bd", pr, Lt)
    sll = ctx @ p["linear3.weight"].t() + p["linear3.bias"]
    m = ref.NLBlockRef().double().eval()
    m.load_state_dict(p)
    with torch.no_grad():
        St1 = m.linear1(St.view(-1, 1, 512))
        SL = torch.softmax(torch.matmul(St1, m.linear2(Lt).transpose(1, 2)) * (1 / 512) ** 0.5, 2)
        sll_ref = torch.matmul(SL, m.linear3(Lt)).view(B, 512)
    assert (sll - sll_ref).abs().max().item() < 1e-12


def test_oracle_timeconv_matches_reference_fixture():
    case = TC_CASES[0]
    B, L, seed = case["B"], case["L"], case["seed"]
    z = np.load(os.path.join(GOLD, "timeconv_L%d.npz" % L))
    m = ref.TimeConvRef()
    m.load_state_dict({k: torch.from_numpy(v) for k, v in timeconv_params(seed).items()},
                      strict=False)
    x_np, g_np = timeconv_inputs(seed, B, L)
    x = torch.from_numpy(x_np).requires_grad_(True)
    y = m(x)
    y.backward(torch.from_numpy(g_np))
    assert np.abs(y.detach().numpy() - z["out"]).max() == 0.0
    assert np.abs(x.grad.numpy() - z["dx"]).max() < 1e-6
    for name, p in m.named_parameters():
        key = "d_" + name.replace(".", "_")
        g = p.grad.numpy()
        if g.ndim == 3:
            probes = projection_probes(seed + 7, g.shape, 16)
            ex = z[key + "_proj"]
            assert np.abs(project(g, probes) - ex).max() <= 1e-6 * np.abs(ex).max()
        else:
            assert np.abs(g - z[key]).max() <= 1e-6 * np.abs(z[key]).max()


@pytest.mark.parametrize("name", ["tiny", "ragged", "empty", "c2", "c5"])
def test_lfb_index_rule_matches_reference(name):
    z = np.load(os.path.join(GOLD, "lfb_index_%s.npz" % name))
    lengths, T, L = list(z["lengths"]), int(z["T"]), int(z["L"])
    starts = ref.get_useful_start_idx(T, lengths)
    assert np.array_equal(np.array(starts, dtype=np.int64).reshape(-1), z["starts"])
    if len(starts) == 0:
        return
    table = ref.lfb_index_table(z["query"], starts, L)
    assert np.array_equal(np.array(table), z["table"])
    # closed form used on the device: first valid start >= max(s-k-1, 0)
    q = z["query"][:, None] - np.arange(L)[None, :] - 1
    dev_rule = np.searchsorted(z["starts"], np.maximum(q, 0), side="left")
    assert np.array_equal(dev_rule, z["table"])


def test_lfb_survey_example():
    starts = ref.get_useful_start_idx(3, [6, 5])
    assert starts == [0, 1, 2, 3, 6, 7, 8]
    assert ref.lfb_index_table([6], starts, 5) == [[4, 4, 3, 2, 1]]


def test_oracle_model_shapes_and_counts():
    assert abs(ref.trunk_gmacs_per_frame() - 4.0871) < 1e-3
    m = ref.TMRNetRef(seq_len=2)
    assert sum(p.numel() for p in m.parameters()) == 30335047
    m.eval()
    with torch.no_grad():
        out = m(torch.randn(2, 2, 3, 224, 224), torch.randn(2, 5, 512))
    assert out.shape == (2, 7)


def test_resnest_oracle_counts_and_keys():
    """ResNeSt restatement (parity unpinned: the resnest package is not in the reference):
    25,434,240 trunk parameters, 5.369 conv GMAC/frame, TMRNet-ResNeSt+TimeConv 36,194,951
    (SURVEY.md §8a-5); the HIP module tree carries exactly the same state_dict keys/shapes."""
    share = ref.resnest50_share().eval()
    assert sum(p.numel() for p in share.parameters()) == 25434240
    macs = []
    hook = lambda mod, inp, out: macs.append(out.numel() * mod.weight[0].numel())
    for mod in share.modules():
        if isinstance(mod, torch.nn.Conv2d):
            mod.register_forward_hook(hook)
    with torch.no_grad():
        assert share(torch.randn(1, 3, 224, 224)).shape == (1, 2048)
    assert abs(sum(macs) / 1e9 - 5.369) < 1e-3
    m = ref.TMRNetRef(seq_len=2, num_classes=7, time_conv=True, backbone="resnest50")
    assert sum(p.numel() for p in m.parameters()) == 36194951
    from tmrnet_amd.resnest import ResNeSt50Share
    ours = {k: v.shape for k, v in ResNeSt50Share().state_dict().items()}
    theirs = {k: v.shape for k, v in share.state_dict().items()}
    assert ours == theirs


def test_timeconv_generalised_L():
    m = ref.TimeConvRef()
    for L in (1, 7, 40):
        assert m(torch.randn(2, L, 512)).shape == (2, L, 512)


def test_bf16_conv_emulation():
    """emulate_bf16_convs: forward = conv of bf16-rounded operands; backward rounds dy and
    uses the rounded saved operands (the TMR_MATH_BF16 contract of include/tmr.h)."""
    torch.manual_seed(0)
    conv = torch.nn.Conv2d(8, 16, 3, 2, 1, bias=False)
    emu = ref.emulate_bf16_convs(torch.nn.Sequential(conv))
    x = torch.randn(2, 8, 9, 7, requires_grad=True)
    y = emu(x)
    r = ref.bf16_round
    assert torch.equal(y, torch.nn.functional.conv2d(r(x), r(conv.weight), None, 2, 1))
    gy = torch.randn_like(y)
    y.backward(gy)
    dx = torch.nn.grad.conv2d_input(x.shape, r(conv.weight), r(gy), 2, 1)
    dw = torch.nn.grad.conv2d_weight(r(x), conv.weight.shape, r(gy), 2, 1)
    assert torch.equal(x.grad, dx) and torch.equal(conv.weight.grad, dw)
    assert not torch.equal(r(x), x)
