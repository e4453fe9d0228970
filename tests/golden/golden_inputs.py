"""Seeded, version-stable generators for the golden-fixture inputs.

Shared by ``make_golden.py`` (which feeds them to the reference) and by the
tests (which feed them to the oracle and to the HIP path).  numpy's PCG64
stream is stable across numpy releases, so regenerating from a seed is
bit-identical everywhere; only expected outputs are stored in the fixtures.
"""
import numpy as np

NL_CASES = [
    {"B": 4, "L": 30, "seed": 101},
    {"B": 4, "L": 40, "seed": 102},
    {"B": 2, "L": 300, "seed": 103},
]
TC_CASES = [
    {"B": 2, "L": 30, "seed": 201},
]
LFB_CASES = [
    # the survey's worked example
    {"name": "tiny", "lengths": [6, 5], "T": 3, "L": 5, "seed": 1, "max_query": 10**9},
    # ragged videos, some shorter than the clip length (no valid start)
    {"name": "ragged", "lengths": [12, 3, 1, 25, 10, 2, 17], "T": 4, "L": 7,
     "seed": 2, "max_query": 10**9},
    # no video long enough: zero valid starts
    {"name": "empty", "lengths": [2, 1], "T": 3, "L": 4, "seed": 3, "max_query": 10**9},
    # benchmark bank geometry: 40 videos x 2500 frames
    {"name": "c2", "lengths": [2500] * 40, "T": 10, "L": 40, "seed": 4, "max_query": 512},
    {"name": "c5", "lengths": [2500] * 40, "T": 30, "L": 300, "seed": 5, "max_query": 128},
]


def _u(rng, shape, a):
    return rng.uniform(-a, a, size=shape).astype(np.float32)


def nlblock_params(seed):
    rng = np.random.default_rng(seed)
    p = {}
    xav = (6.0 / 1024.0) ** 0.5
    for i in range(1, 5):
        p["linear%d.weight" % i] = _u(rng, (512, 512), xav)
        p["linear%d.bias" % i] = _u(rng, (512,), 512 ** -0.5)
    p["layer_norm.weight"] = (1.0 + 0.2 * rng.standard_normal((1, 512))).astype(np.float32)
    p["layer_norm.bias"] = (0.1 * rng.standard_normal((1, 512))).astype(np.float32)
    return p


def nlblock_inputs(seed, B, L):
    rng = np.random.default_rng(seed + 1000)
    St = _u(rng, (B, 512), 1.0)
    Lt = _u(rng, (B, L, 512), 1.0)
    gout = rng.standard_normal((B, 512)).astype(np.float32)
    return St, Lt, gout


def timeconv_params(seed):
    rng = np.random.default_rng(seed)
    p = {}
    for i, k in ((1, 3), (2, 5), (3, 7)):
        b = (512.0 * k) ** -0.5
        p["timeconv%d.weight" % i] = _u(rng, (512, 512, k), b)
        p["timeconv%d.bias" % i] = _u(rng, (512,), b)
    return p


def timeconv_inputs(seed, B, L):
    rng = np.random.default_rng(seed + 1000)
    x = _u(rng, (B, L, 512), 1.0)
    gout = rng.standard_normal((B, L, 512)).astype(np.float32)
    return x, gout


def projection_probes(seed, shape, n):
    rng = np.random.default_rng(seed + 5000)
    return [rng.standard_normal(shape) for _ in range(n)]


def project(grad, probes):
    g = np.asarray(grad, dtype=np.float64).reshape(grad.shape[0], -1)
    return np.array([(g * p.reshape(g.shape)).sum() for p in probes])
