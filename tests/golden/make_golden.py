"""Generate the golden fixtures that pin the CPU oracle to the reference.

Runs ONLY in the build container, where the read-only reference checkout is
mounted at /root/reference.  The reference's Python never travels to the GPU
box: this script imports it here, runs it on seeded inputs, and commits the
resulting *data* (inputs are regenerated from the seeds recorded below; the
expected outputs are stored) as small .npz files next to this script.

What is pinned, and against which reference code:

* ``nlblock_L{30,40,300}.npz`` -- ``NLBlock.forward`` / autograd backward,
  reference ``code/Training TMRNet/NLBlock_MutiConv6_3.py:10-40`` imported by
  path (eval mode, i.e. dropout off; train-mode dropout is random and is
  covered by the mask-injection parity tests instead).
* ``timeconv_L30.npz`` -- ``TimeConv.forward`` and weight gradients,
  ``NLBlock_MutiConv6_3.py:43-79`` (the reference only runs at L=30).
* ``lfb_index_*.npz`` -- the long-term-feature-bank row table produced by the
  reference's own ``get_useful_start_idx`` + ``get_long_feature``
  (``code/Training TMRNet/train_only_non-local_pretrained.py:273-311``,
  dict built as at ``:507-511``), AST-extracted from the script (the script
  itself cannot be imported: argparse runs at import time) and executed with
  ``LFB_length`` injected and ``lfb = arange(N)`` so the gathered "features"
  are row ids.

Weights and inputs are drawn with numpy's PCG64 (``np.random.default_rng``),
whose stream is stable across numpy versions, so the tests regenerate them
bit-identically from the recorded seeds instead of storing them.  Parameter
gradients of the 512x512 linears are stored as 16 fixed random projections
plus their first row and column (full tensors would be several MB each).

Usage:  python tests/golden/make_golden.py
"""
import ast
import importlib.util
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from tests.golden.golden_inputs import (  # noqa: E402
    nlblock_params, nlblock_inputs, timeconv_params, timeconv_inputs,
    projection_probes, NL_CASES, TC_CASES, LFB_CASES)

REF = "/root/reference/code/Training TMRNet"


def load_reference_nlblock_module():
    spec = importlib.util.spec_from_file_location(
        "ref_NLBlock_MutiConv6_3", os.path.join(REF, "NLBlock_MutiConv6_3.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def extract_index_functions(lfb_length):
    """AST-extract get_useful_start_idx / get_long_feature from the script."""
    path = os.path.join(REF, "train_only_non-local_pretrained.py")
    with open(path) as f:
        tree = ast.parse(f.read())
    keep = [n for n in tree.body if isinstance(n, ast.FunctionDef)
            and n.name in ("get_useful_start_idx", "get_long_feature")]
    assert len(keep) == 2
    mod = ast.Module(body=keep, type_ignores=[])
    ns = {"LFB_length": lfb_length}
    exec(compile(mod, path, "exec"), ns)
    return ns["get_useful_start_idx"], ns["get_long_feature"]


def proj(grad, probes):
    g = grad.reshape(grad.shape[0], -1).astype(np.float64)
    return np.array([(g * p.reshape(g.shape)).sum() for p in probes])


def gen_nlblock(ref):
    for case in NL_CASES:
        B, L, seed = case["B"], case["L"], case["seed"]
        m = ref.NLBlock()
        sd = {k: torch.from_numpy(v) for k, v in nlblock_params(seed).items()}
        m.load_state_dict(sd)
        m.eval()
        St_np, Lt_np, gout_np = nlblock_inputs(seed, B, L)
        St = torch.from_numpy(St_np).requires_grad_(True)
        Lt = torch.from_numpy(Lt_np).requires_grad_(True)
        out = m(St, Lt)
        out.backward(torch.from_numpy(gout_np))
        probes = projection_probes(seed, (512, 512), 16)
        rec = {"out": out.detach().numpy(), "dSt": St.grad.numpy(),
               "dLt": Lt.grad.numpy()}
        for name, p in m.named_parameters():
            g = p.grad.numpy()
            key = "d_" + name.replace(".", "_")
            if g.ndim == 2 and g.shape == (512, 512):
                rec[key + "_proj"] = proj(g, probes)
                rec[key + "_row0"] = g[0].copy()
                rec[key + "_col0"] = g[:, 0].copy()
            else:
                rec[key] = g.copy()
        fn = os.path.join(HERE, "nlblock_L%d.npz" % L)
        np.savez_compressed(fn, **rec)
        print("wrote", fn)


def gen_timeconv(ref):
    for case in TC_CASES:
        B, L, seed = case["B"], case["L"], case["seed"]
        m = ref.TimeConv()
        sd = {k: torch.from_numpy(v) for k, v in timeconv_params(seed).items()}
        m.load_state_dict(sd)
        x_np, gout_np = timeconv_inputs(seed, B, L)
        x = torch.from_numpy(x_np).requires_grad_(True)
        y = m(x)
        y.backward(torch.from_numpy(gout_np))
        rec = {"out": y.detach().numpy(), "dx": x.grad.numpy()}
        for name, p in m.named_parameters():
            g = p.grad.numpy()
            key = "d_" + name.replace(".", "_")
            if g.ndim == 3:
                probes = projection_probes(seed + 7, g.shape, 16)
                rec[key + "_proj"] = proj(g, probes)
                rec[key + "_row0"] = g[0].copy()
            else:
                rec[key] = g.copy()
        fn = os.path.join(HERE, "timeconv_L%d.npz" % L)
        np.savez_compressed(fn, **rec)
        print("wrote", fn)


def gen_lfb_index():
    for case in LFB_CASES:
        name, lengths, T, L = case["name"], case["lengths"], case["T"], case["L"]
        get_useful_start_idx, get_long_feature = extract_index_functions(L)
        starts = get_useful_start_idx(T, lengths)
        if len(starts) == 0:
            np.savez_compressed(os.path.join(HERE, "lfb_index_%s.npz" % name),
                                lengths=np.array(lengths, np.int64), T=T, L=L,
                                starts=np.zeros(0, np.int64),
                                query=np.zeros(0, np.int64),
                                table=np.zeros((0, L), np.int64))
            continue
        # dict start-frame -> bank row, exactly as :507-511
        dict_index, dict_value = zip(*list(enumerate(starts)))
        d = dict(zip(dict_value, dict_index))
        lfb = np.arange(len(starts), dtype=np.int64)  # feature == row id
        rng = np.random.default_rng(case["seed"])
        if len(starts) <= case["max_query"]:
            query = np.array(starts, np.int64)
        else:
            # every start of the first two videos (boundary behaviour) plus a
            # random sample of the rest
            first = [s for s in starts if s < lengths[0] + lengths[1]]
            rest = rng.choice(np.array(starts), case["max_query"], replace=False)
            query = np.unique(np.concatenate([np.array(first), rest]))
        table = np.array(get_long_feature(list(query), d, lfb), dtype=np.int64)
        fn = os.path.join(HERE, "lfb_index_%s.npz" % name)
        np.savez_compressed(fn, lengths=np.array(lengths, np.int64), T=T, L=L,
                            starts=np.array(starts, np.int64), query=query,
                            table=table.reshape(len(query), L))
        print("wrote", fn, table.shape)


if __name__ == "__main__":
    torch.set_num_threads(8)
    ref = load_reference_nlblock_module()
    gen_nlblock(ref)
    gen_timeconv(ref)
    gen_lfb_index()
