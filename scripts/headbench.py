"""Clip-branch microbenchmark: tmr_lstm_fwd/bwd (persistent one-launch recurrence vs the per-step
path) and the NLBlock attention core (tmr_nl_attn_fwd/bwd, Lt rows from the resident bank) at the
C2 (B=64, T=10, L=40) and C5 (B=64, T=30, L=300) shapes.  HIP events on the launching stream;
prints one JSON object.  NL GB/s = algorithmic bytes (every Lt row read once per pass + the
(B,L) score/probability traffic) / kernel time."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tmrnet_amd import ops  # noqa: E402


def timed(fn, reps=20, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def lstm_case(B, T, I=2048, H=512):
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    x = torch.randn(B, T, I, device=dev)
    w_ih = torch.randn(4 * H, I, device=dev) * 0.02
    w_hh = torch.randn(4 * H, H, device=dev) * 0.04
    b_ih = torch.zeros(4 * H, device=dev)
    b_hh = torch.zeros(4 * H, device=dev)
    out = {}
    for mode in ("1", "0"):
        os.environ["TMR_LSTM_PERSIST"] = mode
        st = {}
        st["fwd"] = ops.lstm_fwd(x, w_ih, w_hh, b_ih, b_hh)
        y, saved = st["fwd"][0], st["fwd"][3]
        dy = torch.randn_like(y)
        f = timed(lambda: ops.lstm_fwd(x, w_ih, w_hh, b_ih, b_hh))
        b = timed(lambda: ops.lstm_bwd(dy, x, w_ih, w_hh, y, saved))
        out["persistent" if mode == "1" else "per_step"] = {"fwd_ms": round(f, 4),
                                                             "bwd_ms": round(b, 4)}
    os.environ.pop("TMR_LSTM_PERSIST", None)
    return out


def nl_case(B, L, N=99640, D=512):
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(1)
    bank = torch.rand(N, D, device=dev, generator=g) * 2 - 1
    rows = torch.randint(0, N, (B, L), device=dev, generator=g).to(torch.int32)
    u = torch.randn(B, D, device=dev, generator=g)
    dctx = torch.randn(B, D, device=dev, generator=g)
    scale = (1.0 / D) ** 0.5
    p, _ = ops.nl_attn_fwd(bank, rows, u, B, L, scale)
    f = timed(lambda: ops.nl_attn_fwd(bank, rows, u, B, L, scale))
    b = timed(lambda: ops.nl_attn_bwd(bank, rows, u, p, dctx, B, L, scale, False))
    lt = B * L * D * 4
    small = B * L * 4 * 3 + B * L * 4   # scores/p, row table
    return {"fwd_ms": round(f, 4), "bwd_ms": round(b, 4),
            "fwd_GBps": round((lt + small) / (f * 1e-3) / 1e9, 1),
            "bwd_GBps": round((2 * lt + 2 * small) / (b * 1e-3) / 1e9, 1),
            "lt_bytes": lt}


if __name__ == "__main__":
    res = {"lstm_c2_B64_T10": lstm_case(64, 10), "lstm_c5_B64_T30": lstm_case(64, 30),
           "nl_c2_B64_L40": nl_case(64, 40), "nl_c5_B64_L300": nl_case(64, 300)}
    print(json.dumps(res))
