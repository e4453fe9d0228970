"""SGD with the semantics of torch.optim.SGD (momentum, dampening, weight_decay, nesterov, per-group
lr).  Mirrors the reference's optimizer wiring (train_only_non-local_pretrained.py:636-667:
momentum 0.9, wd 5e-4, groups share/lstm at lr/10 and nl_block/fc at lr).  Being a
torch.optim.Optimizer, the reference's lr schedulers (StepLR, ReduceLROnPlateau) attach unchanged.

One step is ONE kernel launch over every parameter of every group (tmr_sgd_step_multi): the
per-tensor table (pointers, sizes, group hyper-parameters) is built on the host and uploaded only
when it changes (gradient addresses move between steps), through pinned memory and an async
copy on the step's stream, so a step never blocks the host.
"""
import numpy as np
import torch

from ._lib import call, query, stream_ptr
from . import health

_ENTRY = np.dtype([("p", "<u8"), ("g", "<u8"), ("buf", "<u8"), ("n", "<i8"),
                   ("block_begin", "<i8"), ("lr", "<f4"), ("momentum", "<f4"),
                   ("dampening", "<f4"), ("weight_decay", "<f4"), ("nesterov", "<i4"),
                   ("first_step", "<i4")])
assert _ENTRY.itemsize == 64   # sizeof(tmr_sgd_tensor), include/tmr.h


class SGD(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, momentum=0.0, dampening=0.0, weight_decay=0.0,
                 nesterov=False):
        if nesterov and (momentum <= 0 or dampening != 0):
            raise ValueError("Nesterov momentum requires a momentum and zero dampening")
        defaults = dict(lr=lr, momentum=momentum, dampening=dampening,
                        weight_decay=weight_decay, nesterov=nesterov)
        super().__init__(params, defaults)
        self._table_key = None
        self._table_dev = None
        self._keep = None
        self.table_uploads = 0

    @torch.no_grad()
    def step(self, closure=None):
        health.check()   # device-side failures of earlier steps (no sync; health.py)
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        entries, keep, dev = [], [], None
        chunk = None
        for group in self.param_groups:
            mom = group["momentum"]
            for p in group["params"]:
                if p.grad is None:
                    continue
                if p.dtype != torch.float32 or not p.is_cuda or not p.is_contiguous():
                    raise RuntimeError("SGD: parameters must be contiguous fp32 GPU tensors")
                if dev is None:
                    dev = p.device
                    chunk = int(query("tmr_sgd_chunk"))
                elif p.device != dev:
                    raise RuntimeError("SGD: all parameters must be on one device")
                g = p.grad
                if not g.is_contiguous():
                    g = g.contiguous()
                keep.append(g)
                state = self.state[p]
                first = 0
                buf = None
                if mom != 0:
                    buf = state.get("momentum_buffer")
                    if buf is None:
                        buf = torch.empty_like(p)
                        state["momentum_buffer"] = buf
                        first = 1
                entries.append((p.data_ptr(), g.data_ptr(), buf.data_ptr() if buf is not None else 0,
                                p.numel(), 0, group["lr"], mom, group["dampening"],
                                group["weight_decay"], int(group["nesterov"]), first))
        entries = [e for e in entries if e[3] > 0]
        if not entries:
            return loss
        tab = np.array(entries, dtype=_ENTRY)
        nblk = (tab["n"] + chunk - 1) // chunk
        tab["block_begin"] = np.concatenate([[0], np.cumsum(nblk)[:-1]])
        key = tab.tobytes()
        if key != self._table_key or self._table_dev is None or self._table_dev.device != dev:
            # pinned staging from torch's host caching allocator + async copy on this stream:
            # no host sync, and the block is not reused before the copy has run
            host = torch.frombuffer(bytearray(key), dtype=torch.uint8).pin_memory()
            self._table_dev = host.to(dev, non_blocking=True)
            self._table_key = key
            self.table_uploads += 1
        self._keep = keep        # contiguous grad copies stay alive until the next step
        # the kernel reads the device health word and skips the update when this step failed
        call("tmr_sgd_step_multi", self._table_dev, len(entries), int(nblk.sum()),
             health.status_word(dev), stream_ptr(dev))
        return loss


_ADAM_ENTRY = np.dtype([("p", "<u8"), ("g", "<u8"), ("m", "<u8"), ("v", "<u8"), ("n", "<i8"),
                        ("block_begin", "<i8"), ("beta1", "<f4"), ("beta2", "<f4"), ("eps", "<f4"),
                        ("weight_decay", "<f4"), ("step_size", "<f4"), ("bc2_sqrt", "<f4"),
                        ("maximize", "<i4"), ("reserved", "<i4")])
assert _ADAM_ENTRY.itemsize == 80   # sizeof(tmr_adam_tensor), include/tmr.h


class Adam(torch.optim.Optimizer):
    """torch.optim.Adam (amsgrad off) on one multi-tensor launch per step (tmr_adam_step_multi):
    the reference's -o 1 optimizer (train_only_non-local_pretrained.py:644-645, code/models.py:63-68:
    default betas / eps, per-group lr).  State keys as torch's ('step', 'exp_avg', 'exp_avg_sq'),
    so state_dict()s interchange; 'step' is a CPU float tensor as in torch."""

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0,
                 amsgrad=False, maximize=False):
        if amsgrad:
            raise NotImplementedError("Adam(amsgrad=True) is not used by the reference")
        if not 0.0 <= betas[0] < 1.0 or not 0.0 <= betas[1] < 1.0:
            raise ValueError("Invalid beta parameters: %s" % (betas,))
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, amsgrad=False,
                        maximize=maximize)
        super().__init__(params, defaults)

    @torch.no_grad()
    def step(self, closure=None):
        health.check()   # device-side failures of earlier steps (no sync; health.py)
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        entries, keep, dev, chunk = [], [], None, None
        for group in self.param_groups:
            b1, b2 = group["betas"]
            for p in group["params"]:
                if p.grad is None:
                    continue
                if p.dtype != torch.float32 or not p.is_cuda or not p.is_contiguous():
                    raise RuntimeError("Adam: parameters must be contiguous fp32 GPU tensors")
                if dev is None:
                    dev = p.device
                    chunk = int(query("tmr_sgd_chunk"))
                elif p.device != dev:
                    raise RuntimeError("Adam: all parameters must be on one device")
                g = p.grad if p.grad.is_contiguous() else p.grad.contiguous()
                keep.append(g)
                st = self.state[p]
                if len(st) == 0:
                    st["step"] = torch.tensor(0.0, dtype=torch.float32)
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                st["step"] += 1
                step = float(st["step"].item())
                bc1 = 1.0 - b1 ** step
                bc2 = 1.0 - b2 ** step
                entries.append((p.data_ptr(), g.data_ptr(), st["exp_avg"].data_ptr(),
                                st["exp_avg_sq"].data_ptr(), p.numel(), 0, b1, b2, group["eps"],
                                group["weight_decay"], group["lr"] / bc1, bc2 ** 0.5,
                                int(group["maximize"]), 0))
        entries = [e for e in entries if e[4] > 0]
        if not entries:
            return loss
        tab = np.array(entries, dtype=_ADAM_ENTRY)
        nblk = (tab["n"] + chunk - 1) // chunk
        tab["block_begin"] = np.concatenate([[0], np.cumsum(nblk)[:-1]])
        # the step sizes change every step: upload the table each time (pinned, async)
        host = torch.frombuffer(bytearray(tab.tobytes()), dtype=torch.uint8).pin_memory()
        self._table_dev = host.to(dev, non_blocking=True)
        self._keep = keep
        call("tmr_adam_step_multi", self._table_dev, len(entries), int(nblk.sum()),
             health.status_word(dev), stream_ptr(dev))
        return loss


def sgd_param_groups(model, lr):
    """Parameter groups of the reference's multi_optim=1 optimizer: `share` and `lstm` at the
    optimizer's default lr (the scripts pass lr/10), every later module at `lr`.

    train_only_non-local_pretrained.py:646-655 (share, lstm, nl_block, fc_h_c, fc_c);
    train_non-local_mutiConv_resnet.py:797-804 and the resnest twin add `time_conv` at `lr`
    between lstm and nl_block.  The memory-bank model (`fc` head,
    Training memory bank model/train_singlenet_phase_1fc.py:498-501) puts lstm and fc at `lr`.
    Use as ``SGD(sgd_param_groups(model, lr), lr=lr / 10, ...)``.
    """
    if hasattr(model, "fc") and not hasattr(model, "nl_block"):
        # memory-bank model, train_singlenet_phase_1fc.py:498-501: only `share` at lr/10
        return [{"params": list(model.share.parameters())},
                {"params": list(model.lstm.parameters()), "lr": lr},
                {"params": list(model.fc.parameters()), "lr": lr}]
    groups = [{"params": list(model.share.parameters())},
              {"params": list(model.lstm.parameters())}]
    if getattr(model, "time_conv", None) is not None:
        groups.append({"params": list(model.time_conv.parameters()), "lr": lr})
    for name in ("nl_block", "fc_h_c", "fc_c"):
        groups.append({"params": list(getattr(model, name).parameters()), "lr": lr})
    return groups
