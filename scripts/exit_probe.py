"""Diagnostics for the exit-time SIGSEGV under rocprofv3: run one ingredient of
the train step and exit normally, so a profiled run can tell which one leaves the HIP runtime's
exit handler calling into a torn-down HSA runtime.

usage: rocprofv3 --kernel-trace -d DIR -- python3 scripts/exit_probe.py MODE
MODE: plain | pinned | lib | conv | lstm | lstm_reset | step
(lstm_reset: hipDeviceReset from an interpreter atexit hook, i.e. before the C-level exit handlers)"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(mode):
    dev = torch.device("cuda:0")
    x = torch.ones(1024, device=dev)
    if mode in ("pinned", "step"):
        h = torch.empty(1 << 20, dtype=torch.uint8).pin_memory()
        x2 = h.to(dev, non_blocking=True)
        torch.cuda.synchronize()
        del x2
    if mode in ("lib", "conv", "lstm", "step"):
        from tmrnet_amd import _lib
        _lib.lib()
    if mode in ("conv", "step"):
        from tmrnet_amd import ops
        a = torch.randn(2, 16, 16, 64, device=dev)
        w = torch.randn(64, 1, 1, 64, device=dev)
        ops.conv_fwd(a, w, 1, 0)
    if mode == "lstm_reset":
        import atexit
        import ctypes
        hip = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))
        atexit.register(lambda: hip.hipDeviceReset())
    if mode in ("lstm", "lstm_reset", "step"):
        from tmrnet_amd import ops
        xs = torch.randn(64, 10, 2048, device=dev)
        wi = torch.randn(2048, 2048, device=dev) * 0.01
        wh = torch.randn(2048, 512, device=dev) * 0.01
        b = torch.zeros(2048, device=dev)
        ops.lstm_fwd(xs, wi, wh, b, b)
    torch.cuda.synchronize()
    print("probe %s ok: %g" % (mode, float(x.sum())), flush=True)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "plain")
