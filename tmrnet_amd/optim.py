"""SGD with the semantics of torch.optim.SGD (momentum, dampening, weight_decay, nesterov, per-group
lr), stepping each parameter with the fused tmr_sgd_step kernel.  Mirrors the reference's
optimizer wiring (train_only_non-local_pretrained.py:636-667: momentum 0.9, wd 5e-4, groups
share/lstm at lr/10 and nl_block/fc at lr).  Being a torch.optim.Optimizer, the reference's
lr schedulers (StepLR, ReduceLROnPlateau) attach unchanged."""
import torch

from . import ops


class SGD(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, momentum=0.0, dampening=0.0, weight_decay=0.0,
                 nesterov=False):
        if nesterov and (momentum <= 0 or dampening != 0):
            raise ValueError("Nesterov momentum requires a momentum and zero dampening")
        defaults = dict(lr=lr, momentum=momentum, dampening=dampening,
                        weight_decay=weight_decay, nesterov=nesterov)
        super().__init__(params, defaults)

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for group in self.param_groups:
            mom = group["momentum"]
            for p in group["params"]:
                if p.grad is None:
                    continue
                g = p.grad
                if not g.is_contiguous():
                    g = g.contiguous()
                state = self.state[p]
                first = False
                buf = None
                if mom != 0:
                    buf = state.get("momentum_buffer")
                    if buf is None:
                        buf = torch.empty_like(p)
                        state["momentum_buffer"] = buf
                        first = True
                ops.sgd_step(p, g, buf, group["lr"], mom, group["dampening"],
                             group["weight_decay"], group["nesterov"], first)
        return loss
