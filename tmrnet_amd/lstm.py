"""Single-layer batch-first LSTM on libtmr kernels (drop-in for nn.LSTM(2048, 512,
batch_first=True) at code/Training TMRNet/train_only_non-local_pretrained.py:215).

Parameter names/shapes match nn.LSTM (weight_ih_l0 (4H,I), weight_hh_l0 (4H,H),
bias_ih_l0, bias_hh_l0; gate order i,f,g,o), so `lstm.*` state_dict keys load
unchanged, and `all_weights` is provided for the reference's
``init.xavier_normal_(self.lstm.all_weights[0][0])`` (:221-222).

Forward (tmr_lstm_fwd): one MFMA GEMM for the input projection of all B*T frames
(x W_ih^T + b_ih + b_hh), then the whole T-step recurrence -- gate GEMM h_{t-1} W_hh^T,
sigma/tanh, cell update -- in one persistent launch (csrc/lstm.hip).  Backward
(tmr_lstm_bwd): BPTT in one persistent launch, then one GEMM each for dW_ih, dW_hh and dX
over all steps.
"""
import math

import torch
import torch.nn as nn

from . import health, ops


class LSTMFn(torch.autograd.Function):
    """tmr_lstm_fwd / tmr_lstm_bwd: one C call each way (the recurrence is one persistent launch,
    include/tmr.h)."""

    @staticmethod
    def forward(ctx, x, w_ih, w_hh, b_ih, b_hh):
        x = x.contiguous()
        wi, wh = w_ih.detach().contiguous(), w_hh.detach().contiguous()
        train = torch.is_grad_enabled() or any(ctx.needs_input_grad)
        y, hn, cn, saved, _ = ops.lstm_fwd(x, wi, wh, b_ih.detach().contiguous(),
                                           b_hh.detach().contiguous(), train=train)
        if saved is not None:
            ctx.save_for_backward(x, wi, wh, y, saved)
        hn, cn = hn.unsqueeze(0), cn.unsqueeze(0)
        ctx.mark_non_differentiable(hn, cn)
        ctx.set_materialize_grads(False)   # no zero-filled gradients for h_n / c_n
        return y, hn, cn

    @staticmethod
    def backward(ctx, dy, dhn, dcn):
        x, wi, wh, y, saved = ctx.saved_tensors
        dy = dy.contiguous() if dy is not None else ops.zeros(y.shape, y)
        dx, dw_ih, dw_hh, db_ih, db_hh, _ = ops.lstm_bwd(dy, x, wi, wh, y, saved,
                                                         want_dx=ctx.needs_input_grad[0])
        return dx, dw_ih, dw_hh, db_ih, db_hh


class LSTM(nn.Module):
    """nn.LSTM(input_size, hidden_size, batch_first=True), one layer, unidirectional."""

    def __init__(self, input_size, hidden_size, batch_first=True):
        super().__init__()
        if not batch_first:
            raise NotImplementedError("only batch_first=True (as the reference uses) is supported")
        self.input_size = input_size
        self.hidden_size = hidden_size
        self.batch_first = True
        H = hidden_size
        self.weight_ih_l0 = nn.Parameter(torch.empty(4 * H, input_size))
        self.weight_hh_l0 = nn.Parameter(torch.empty(4 * H, H))
        self.bias_ih_l0 = nn.Parameter(torch.empty(4 * H))
        self.bias_hh_l0 = nn.Parameter(torch.empty(4 * H))
        self.reset_parameters()

    def reset_parameters(self):
        stdv = 1.0 / math.sqrt(self.hidden_size)
        for w in self.parameters():
            nn.init.uniform_(w, -stdv, stdv)

    @property
    def all_weights(self):
        return [[self.weight_ih_l0, self.weight_hh_l0, self.bias_ih_l0, self.bias_hh_l0]]

    def flatten_parameters(self):
        pass

    def forward(self, x, hx=None):
        if hx is not None:
            raise NotImplementedError("initial state hx is not supported (reference passes none)")
        y, hn, cn = LSTMFn.apply(x, self.weight_ih_l0, self.weight_hh_l0, self.bias_ih_l0,
                                 self.bias_hh_l0)
        if not torch.is_grad_enabled():
            # inference (eval loops run under no_grad): no optimizer step will read the health
            # word, so wait for the recurrence and raise now rather than return invalid outputs
            health.check(sync=True, device=x.device)
        return y, (hn, cn)
