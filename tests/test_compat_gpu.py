"""The `code/models.py` drop-in (tmrnet_amd/compat/models.py) run on the GPU the way
`code/train_memorybank.py:222-272` drives it: resnet_lstm(args, num_class), a 5-D
(B,T,3,224,224) NCHW input (:258), outputs[T-1::T] (:262), CrossEntropyLoss(reduction='sum',
weight=class weights) (:221), loss.backward(), get_optimizers().step() (:228, :272) for opt 0
(SGD) and opt 1 (Adam) (models.py:50-69).

Oracle: MemoryBankRef (train_singlenet_phase_1fc.py:201-232, the working form of models.py:38-48)
with the indexed `res.{0,1,4,5,6,7}.*` keys mapped onto `share.*`.  Logits within 1e-4 and the
same argmax; gradients (and the SGD update) by the float64 criterion of
tests/test_model_parity_gpu._assert_vs_fp64; the Adam update against torch.optim.Adam applied to
the same gradients.
"""
import sys
from types import SimpleNamespace as NS

import pytest
import torch

import tmrnet_amd
import tmrnet_amd.compat as compat
from oracle import tmrnet_ref as ref
from tests.test_model_parity_gpu import _assert_vs_fp64, _double_copy, _inputs

pytestmark = pytest.mark.gpu

RES = {"0": "conv1", "1": "bn1", "4": "layer1", "5": "layer2", "6": "layer3", "7": "layer4"}


def _to_share(key):
    if key.startswith("res."):
        head, rest = key[4:].split(".", 1)
        return "share.%s.%s" % (RES[head], rest)
    return key


def _models_module():
    sys.path.insert(0, compat.PATH)
    try:
        import models
    finally:
        sys.path.remove(compat.PATH)
    return models


@pytest.mark.parametrize("opt", [0, 1], ids=["sgd", "adam"])
def test_models_resnet_lstm_step(dev, opt):
    B, T, K = 2, 3, 7
    models = _models_module()
    args = NS(num_frames=T, opt=opt, lr=5e-4, momentum=0.9, dampening=0, weightdecay=5e-4,
              nesterov=False)
    torch.manual_seed(21)
    m = models.resnet_lstm(args, K).to(dev).train()
    r = ref.MemoryBankRef(seq_len=T, num_classes=K).train()
    r.load_state_dict({_to_share(k): v.detach().cpu() for k, v in m.state_dict().items()})
    r64 = _double_copy(r, None, B, T, 1)
    frames, off, _, labels = _inputs(B, T, 1, seed=22)
    labels_f = labels.repeat_interleave(T)            # per-frame labels, kept at [T-1::T]
    weight = torch.tensor([0.5, 1.0, 1.5, 2.0, 0.75, 1.25, 3.0])
    mask = (torch.rand(B * T, 512, generator=torch.Generator().manual_seed(23)) >= 0.2).float() / 0.8
    m.forced_mask = mask.to(dev)
    x = ref.crop_normalize_ref(frames, off, T).view(B, T, 3, 224, 224)
    p0 = {_to_share(n): p.detach().cpu().double().clone() for n, p in m.named_parameters()}
    optimizer = m.get_optimizers()
    optimizer.zero_grad()
    out = m.forward(x.to(dev))
    assert tuple(out.shape) == (B * T, K)
    sel = out[T - 1::T]
    crit = tmrnet_amd.CrossEntropyLoss(weight=weight.to(dev), reduction="sum")
    loss = crit(sel, labels_f.to(dev)[T - 1::T])
    out_r = r(x, mask=mask)
    assert (out.detach().cpu() - out_r.detach()).abs().max().item() < 1e-4
    assert torch.equal(out.detach().cpu().argmax(1), out_r.detach().argmax(1))
    loss_r = ref.ce_sum_ref(out_r[T - 1::T], labels, weight)
    assert abs(loss.item() - loss_r.item()) <= 1e-4 * max(1.0, abs(loss_r.item()))
    loss.backward()
    loss_r.backward()
    ref.ce_sum_ref(r64(x.double(), mask=mask.double())[T - 1::T], labels, weight.double()).backward()
    grads = {_to_share(n): p.grad for n, p in m.named_parameters()}
    g = lambda mod: {n: p.grad for n, p in mod.named_parameters()}
    _assert_vs_fp64(grads, g(r), g(r64), "models_grad")
    grads_cpu = {n: t.detach().cpu().clone() for n, t in grads.items()}
    optimizer.step()
    upd = {_to_share(n): p.detach().cpu().double() - p0[_to_share(n)]
           for n, p in m.named_parameters()}
    groups = lambda mod: [{"params": list(mod.share.parameters())},
                          {"params": list(mod.lstm.parameters()), "lr": args.lr},
                          {"params": list(mod.fc.parameters()), "lr": args.lr}]
    if opt == 0:
        kw = dict(lr=args.lr / 10, momentum=args.momentum, dampening=args.dampening,
                  weight_decay=args.weightdecay, nesterov=args.nesterov)
        torch.optim.SGD(groups(r), **kw).step()
        torch.optim.SGD(groups(r64), **kw).step()
        d = lambda mod: {n: p.detach().double() - p0[n] for n, p in mod.named_parameters()}
        _assert_vs_fp64(upd, d(r), d(r64), "models_sgd_update")
    else:
        # the Adam step itself, on the HIP gradients: torch.optim.Adam (models.py:63-68)
        rc = ref.MemoryBankRef(seq_len=T, num_classes=K)
        rc.load_state_dict({n: p0[n].float() if n in p0 else v
                            for n, v in r.state_dict().items()})
        for n, p in rc.named_parameters():
            p.grad = grads_cpu[n]
        torch.optim.Adam(groups(rc), lr=args.lr / 10).step()
        # elementwise: 1e-5 of the update plus two fp32 ulps of the parameter (the new value is
        # rounded to fp32 on both sides)
        for n, p in rc.named_parameters():
            exp = p.detach().double() - p0[n]
            bound = 1e-5 * exp.abs() + 2.0 ** -22 * p0[n].abs() + 1e-12
            assert ((upd[n] - exp).abs() <= bound).all(), (n, (upd[n] - exp).abs().max().item())



def test_models_resnet_lstm_threads(dev):
    """One models.resnet_lstm instance driven from two threads at once with different clip
    lengths (DataParallel calls its replicas from Python threads, SURVEY.md §8b Threading;
    code/models.py:38-48): T comes from each call's 5-D input and is never written into the module,
    so each thread's logits equal a single-threaded call's."""
    import threading
    models = _models_module()
    args = NS(num_frames=10, opt=0, lr=5e-4, momentum=0.9, dampening=0, weightdecay=5e-4,
              nesterov=False)
    torch.manual_seed(31)
    m = models.resnet_lstm(args, 7).to(dev).eval()
    xs = {}
    for B, T in ((2, 3), (1, 5)):
        frames, off, _, _ = _inputs(B, T, 1, seed=32 + T)
        xs[T] = ref.crop_normalize_ref(frames, off, T).view(B, T, 3, 224, 224).to(dev)
    with torch.no_grad():
        solo = {T: m(x).cpu() for T, x in xs.items()}
    got, errs = {}, []
    barrier = threading.Barrier(len(xs))

    def run(T):
        try:
            barrier.wait()
            with torch.no_grad():
                for _ in range(3):
                    o = m(xs[T])
                    torch.cuda.current_stream().synchronize()
                    got.setdefault(T, []).append(o.cpu())
        except Exception as e:   # noqa: BLE001 -- reported below
            errs.append(e)
    th = [threading.Thread(target=run, args=(T,)) for T in xs]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
    assert not errs, errs
    assert m.seq_len == 10
    for T, outs in got.items():
        assert len(outs) == 3
        for o in outs:
            assert o.shape == solo[T].shape and torch.equal(o, solo[T]), T
