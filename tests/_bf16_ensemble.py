"""The bf16 gradient contract at a host-runnable geometry: gradient ensembles
of one train step over +-2^-9 relative input noise, for the bf16 contract and for the fp32 step,
reduced to per-group Gram matrices from which every ensemble statistic is derived.

Used by tests/golden/make_bf16_ensemble.py (CPU: the fp32 oracle and its float emulation of the
bf16 contract, `oracle.emulate_bf16_convs(activations=True, grads=True)`; the fixture
tests/golden/bf16_ensemble_*.json) and tests/test_bf16_ensemble_gpu.py (the HIP fp32 and bf16
steps on the same weights, inputs, bank rows, masks and noise signs).  Reference step:
`loss.backward(); optimizer.step()` in fp32 (code/Training TMRNet/train_only_non-local_pretrained.py
:724-725, train_non-local_mutiConv_resnest.py:751-752).

Statistics (g = g* + n, n independent zero-mean noise between samples of one ensemble; sample k
of every ensemble runs on input-noise sample k, so cross pairs with equal k are left out):
  s_a   = mean_{i<j in a} <g_i, g_j>      estimates |g*_a|^2 without the noise term
  x     = mean_{i in 16, j in 32, i != j} <g_i, g_j>  estimates <g*_16, g*_32>
  ratio = sqrt(s_16 / s_32)               |E g16| / |E g32|
  proj  = x / s_32                        the fp32-direction component of E g16, in units of E g32
  cstar = x / sqrt(s_16 s_32)             the cosine of the two expected gradients
Jackknife (leave noise sample k out of both ensembles) gives each statistic's standard error.
"""
import hashlib
import math

import numpy as np
import torch

from tests._bf16_grads import group_of

TRUNK = ("stem", "layer1", "layer2", "layer3", "layer4")
CLIP = ("lstm", "time_conv", "nl_block", "head")
EPS = 2.0 ** -9
# (backbone, time_conv, B, T, L, weight seed, input seed)
GEOS = {"r50": ("resnet50", False, 4, 10, 40, 61, 62),
        "rst": ("resnest50", True, 2, 10, 40, 71, 72)}
SKIP = ("nl_block.linear2.bias",)   # exact gradient 0 (the q.b2 score term cancels in the softmax)


def weights(geo):
    """The state_dict both sides load: the oracle's own init under a fixed seed."""
    from oracle import tmrnet_ref as ref
    backbone, tc, B, T, L, ws, _ = GEOS[geo]
    torch.manual_seed(ws)
    r = ref.TMRNetRef(seq_len=T, backbone=backbone, time_conv=tc)
    return {k: v.detach().clone() for k, v in r.state_dict().items()}


def inputs(geo):
    """-> x (B*T, 3, 224, 224) fp32 (crop + Normalize of uint8 noise frames, the benchmark's data),
    lt (B, L, 512) bank rows by the reference's row rule, labels (B,), dropout masks."""
    from oracle import tmrnet_ref as ref
    backbone, tc, B, T, L, _, s = GEOS[geo]
    g = torch.Generator().manual_seed(s)
    frames = torch.randint(0, 256, (B * T, 250, 250, 3), generator=g, dtype=torch.uint8)
    off = torch.randint(0, 27, (B, 2), generator=g, dtype=torch.int32)
    labels = torch.randint(0, 7, (B,), generator=g)
    vs = ref.get_useful_start_idx(T, [L + 2 * T] * 3)
    bank = torch.rand(len(vs), 512, generator=g) * 2 - 1
    pick = torch.randint(0, len(vs), (B,), generator=g)
    starts = np.asarray([vs[i] for i in pick.tolist()], dtype=np.int64)
    rows = torch.from_numpy(np.asarray(ref.lfb_index_table(starts, vs, L), dtype=np.int64))
    lt = bank[rows.view(-1)].view(B, L, 512)
    masks = {"nl": (torch.rand(B, 512, generator=g) >= 0.2).float() / 0.8,
             "head": (torch.rand(B, 512, generator=g) >= 0.5).float() / 0.5}
    x = ref.crop_normalize_ref(frames, off, T)
    return x, lt, labels, masks


def noisy(x, k):
    """Sample k of the input ensemble: x * (1 + EPS * s), s = +-1 per element (CPU generator,
    so the host and the GPU box draw the same signs)."""
    g = torch.Generator().manual_seed(1000 + k)
    s = torch.randint(0, 2, x.shape, generator=g).to(x.dtype) * 2 - 1
    return x * (1 + EPS * s)


def to_nhwc4(x):
    """(F,3,H,W) -> the HIP step's (F,H,W,4) NHWC4 input (channel 3 zero)."""
    f, _, h, w = x.shape
    out = torch.zeros(f, h, w, 4, dtype=x.dtype)
    out[..., :3] = x.permute(0, 2, 3, 1)
    return out


def digest(t):
    return hashlib.sha256(t.detach().cpu().contiguous().numpy().tobytes()).hexdigest()[:16]


def group_vectors(grads):
    """{name: grad} -> {group: flat float64 vector} (SKIP and ResNeSt's fc1 biases, whose exact
    gradient is 0 before a batch-statistic BN, left out)."""
    per = {}
    for n in sorted(grads):
        if n in SKIP or n.endswith("fc1.bias"):
            continue
        per.setdefault(group_of(n), []).append(grads[n].detach().double().cpu().reshape(-1))
    return {k: torch.cat(v) for k, v in per.items()}


def gram(samples):
    """[{group: vector}] -> {group: n x n Gram matrix (nested lists)}."""
    out = {}
    for k in samples[0]:
        m = torch.stack([s[k] for s in samples])
        out[k] = (m @ m.T).tolist()
    return out


def _stats(G, ia, ib):
    """ia[k] and ib[k] ran on the same noise sample k (paired ensembles): their shared noise term
    would bias the cross product, so pairs with equal k are left out of x as same-ensemble pairs
    are left out of s16 / s32."""
    G = np.asarray(G, dtype=np.float64)
    a, b = list(ia), list(ib)
    s16 = np.mean([G[i, j] for n, i in enumerate(a) for j in a[n + 1:]])
    s32 = np.mean([G[i, j] for n, i in enumerate(b) for j in b[n + 1:]])
    x = np.mean([G[i, j] for n, i in enumerate(a) for m, j in enumerate(b) if n != m])
    r = {"s16": s16, "s32": s32, "x": x,
         "ratio": math.sqrt(max(s16, 0.0) / s32) if s32 > 0 else float("nan"),
         "proj": x / s32 if s32 > 0 else float("nan"),
         "cstar": x / math.sqrt(s16 * s32) if s16 > 0 and s32 > 0 else float("nan")}
    return r


def stats(G, n):
    """Statistics of one group's Gram matrix over [n samples of the variant, n fp32 samples],
    sample k of both on noise sample k, with delete-one jackknife standard errors (sample k of
    both ensembles left out together)."""
    ia, ib = list(range(n)), list(range(n, 2 * n))
    full = _stats(G, ia, ib)
    loo = [_stats(G, [i for i in ia if i != d], [j for j in ib if j != n + d]) for d in range(n)]
    for key in ("ratio", "proj", "cstar"):
        v = np.asarray([p[key] for p in loo])
        full[key + "_se"] = math.sqrt((n - 1) / n * float(((v - v.mean()) ** 2).sum()))
    return full
