"""Single-layer batch-first LSTM on libtmr kernels (drop-in for nn.LSTM(2048, 512,
batch_first=True) at code/Training TMRNet/train_only_non-local_pretrained.py:215).

Parameter names/shapes match nn.LSTM (weight_ih_l0 (4H,I), weight_hh_l0 (4H,H),
bias_ih_l0, bias_hh_l0; gate order i,f,g,o), so `lstm.*` state_dict keys load
unchanged, and `all_weights` is provided for the reference's
``init.xavier_normal_(self.lstm.all_weights[0][0])`` (:221-222).

Forward: one MFMA GEMM for the input projection of all B*T frames
(x W_ih^T + b_ih + b_hh), then per step a GEMM h_{t-1} W_hh^T and a fused
gate/cell kernel.  Backward: per-step fused gate backward + the recurrent dgrad
GEMM, then one GEMM each for dW_ih, dW_hh and dX over all steps.
"""
import math

import torch
import torch.nn as nn

from . import ops


class LSTMFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w_ih, w_hh, b_ih, b_hh):
        B, T, I = x.shape
        H = w_hh.shape[1]
        x2 = x.contiguous().view(B * T, I)
        bias = ops.residual_mask(b_ih.detach().contiguous(), b_hh.detach().contiguous(), None)
        gx = ops.gemm_nt(x2, w_ih.detach(), bias=bias).view(B, T, 4 * H)   # x W_ih^T + b
        y = torch.empty((B, T, H), dtype=x.dtype, device=x.device)
        cs = torch.empty((T, B, H), dtype=x.dtype, device=x.device)
        acts = torch.empty((T, B, 4 * H), dtype=x.dtype, device=x.device)
        ghh = torch.empty((B, 4 * H), dtype=x.dtype, device=x.device)
        whh = w_hh.detach()
        for t in range(T):
            if t > 0:
                ops.gemm_nt(y[:, t - 1, :], whh, out=ghh)                  # h_{t-1} W_hh^T
            ops.lstm_cell_fwd(gx[:, t, :], ghh if t > 0 else None,
                              cs[t - 1] if t > 0 else None, y[:, t, :], cs[t], acts[t])
        ctx.save_for_backward(x2, w_ih, w_hh, y, cs, acts)
        ctx.dims = (B, T, I, H)
        hn = y[:, T - 1, :].unsqueeze(0).contiguous()
        cn = cs[T - 1].unsqueeze(0).contiguous()
        ctx.mark_non_differentiable(hn, cn)
        return y, hn, cn

    @staticmethod
    def backward(ctx, dy, dhn, dcn):
        x2, w_ih, w_hh, y, cs, acts = ctx.saved_tensors
        B, T, I, H = ctx.dims
        dy = dy.contiguous() if dy is not None else torch.zeros_like(y)
        dg = torch.empty((B, T, 4 * H), dtype=y.dtype, device=y.device)
        whh = w_hh.detach()
        dcp = [torch.empty((B, H), dtype=y.dtype, device=y.device) for _ in range(2)]
        dh_buf = torch.empty((B, H), dtype=y.dtype, device=y.device)
        dh_rec = None
        dc_next = None
        for t in range(T - 1, -1, -1):
            ops.lstm_cell_bwd(dy[:, t, :], dh_rec, dc_next, acts[t], cs[t],
                              cs[t - 1] if t > 0 else None, dg[:, t, :], dcp[t & 1])
            dc_next = dcp[t & 1]
            if t > 0:
                ops.gemm_nn(dg[:, t, :], whh, out=dh_buf)                 # dgates_t W_hh
                dh_rec = dh_buf
        # h_{t-1} for every (b,t), zero at t=0
        hprev = torch.zeros((B, T, H), dtype=y.dtype, device=y.device)
        if T > 1:
            hprev[:, 1:, :].copy_(y[:, :-1, :])
        dg2 = dg.view(B * T, 4 * H)
        dw_ih = ops.gemm_tn(dg2, x2)                                      # (4H, I)
        dw_hh = ops.gemm_tn(dg2, hprev.view(B * T, H))                    # (4H, H)
        db = ops.col_sum(dg2, B * T, 4 * H, 4 * H)
        dx = None
        if ctx.needs_input_grad[0]:
            dx = ops.gemm_nn(dg2, w_ih.detach()).view(B, T, I)
        return dx, dw_ih, dw_hh, db, ops.mul(db)


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
        return y, (hn, cn)
