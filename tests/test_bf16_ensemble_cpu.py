"""The CPU side of the bf16 gradient-contract fixture (tests/golden/bf16_ensemble_*.json / .npz,
made by tests/golden/make_bf16_ensemble.py): its inputs and weights regenerate from their seeds
(the digests the GPU test also checks), its statistics re-derive from its Gram matrices, and the
attribution it records holds -- the emulated contract's expected trunk gradient is shortened by the
forward operand rounding and the activation storage, not by the backward roundings, and the fp32
step at 4x the input noise is shortened further."""
import json
import os

import numpy as np
import pytest
import torch

from tests import _bf16_ensemble as E

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _load(geo):
    with open(os.path.join(GOLD, "bf16_ensemble_%s.json" % geo)) as f:
        meta = json.load(f)
    return meta, np.load(os.path.join(GOLD, "bf16_ensemble_%s.npz" % geo))


@pytest.mark.parametrize("geo", ["r50", "rst"])
def test_fixture_regenerates(geo):
    meta, z = _load(geo)
    x, lt, _, _ = E.inputs(geo)
    assert E.digest(x) == meta["x_digest"] and E.digest(lt) == meta["lt_digest"]
    sd = E.weights(geo)
    assert E.digest(torch.cat([t.float().reshape(-1) for t in sd.values()
                               if t.is_floating_point()])) == meta["weights_digest"]
    index, n = meta["index"], meta["n"]
    base = [i for i, v in enumerate(index) if v == "fp32"]
    for v, st in meta["stats_vs_fp32"].items():
        sub = [i for i, w in enumerate(index) if w == v] + base
        for g, s in st.items():
            G = z["gram_" + g]
            assert np.allclose(G, G.T) and (np.diag(G) > 0).all()
            r = E.stats(G[np.ix_(sub, sub)], n)
            for key in ("ratio", "proj", "cstar"):
                assert abs(r[key] - s[key]) < 1e-12, (v, g, key)


def test_attribution_r50():
    meta, _ = _load("r50")
    st = meta["stats_vs_fp32"]
    for g in E.TRUNK:
        # the backward operand roundings (dy, and x / w as the dgrad / wgrad read them) change
        # nothing measurable in expectation
        for v in ("bwd_ops", "dy_only"):
            assert abs(st[v][g]["ratio"] - 1) < 0.05 and abs(st[v][g]["proj"] - 1) < 0.05, (v, g)
        # the forward operand rounding alone shortens it, the activation storage further, and the
        # fp32 step under 4x the input noise further still
        assert st["fwd_ops"][g]["proj"] < 0.8, g
        assert abs(st["fwd_ops"][g]["proj"] - st["bf16_ops"][g]["proj"]) < 0.05, g
        assert st["bf16"][g]["proj"] < st["fwd_ops"][g]["proj"], g
        assert st["fp32_e7"][g]["proj"] < st["bf16"][g]["proj"], g
        assert st["fp32_e5"][g]["proj"] < st["fp32_e7"][g]["proj"], g
    for g in E.CLIP:
        if g in st["bf16"]:
            assert st["bf16"][g]["proj"] > 0.95, g
