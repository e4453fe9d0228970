"""CrossEntropyLoss(reduction='sum') on libtmr (train_only_non-local_pretrained.py:631 uses
``nn.CrossEntropyLoss(size_average=False)``; train_non-local_mutiConv_resnet.py:780 adds balanced
class weights).  Forward computes loss, dlogits and argmax preds in one kernel; backward scales
the saved dlogits by the incoming scalar gradient on the device (no host sync)."""
import torch
import torch.nn as nn

from . import ops


class CESumFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, labels, weight):
        loss, dl, preds = ops.ce_sum(logits.contiguous(), labels.contiguous(), weight)
        ctx.save_for_backward(dl)
        ctx.preds = preds
        ctx.mark_non_differentiable(preds)
        ctx.set_materialize_grads(False)   # no zero-filled gradient for preds
        return loss.view(()), preds

    @staticmethod
    def backward(ctx, dloss, dpreds):
        (dl,) = ctx.saved_tensors
        return ops.mul(dl, None, dloss.reshape(1).contiguous()), None, None


class CrossEntropyLoss(nn.Module):
    """nn.CrossEntropyLoss drop-in for reduction='sum' (the reference's only training reduction)."""

    def __init__(self, weight=None, size_average=None, reduction="sum"):
        super().__init__()
        if size_average is not None and size_average:
            reduction = "mean"
        if reduction != "sum":
            raise NotImplementedError("only reduction='sum' (size_average=False) is implemented")
        self.register_buffer("weight", weight)
        self.last_preds = None

    def forward(self, logits, labels):
        w = self.weight.contiguous() if self.weight is not None else None
        loss, preds = CESumFn.apply(logits, labels, w)
        self.last_preds = preds   # == torch.max(outputs, 1)[1]
        return loss
