"""NLBlock (the temporal-variation layer) on libtmr kernels.

Drop-in for ``NLBlock`` of code/Training TMRNet/NLBlock_MutiConv6_3.py:10-40
(identical class in code/eval/python/NLBlock.py:10-40): same constructor,
parameter names (linear1..4, layer_norm with weight/bias of shape (1,512)),
xavier_uniform init, Dropout(0.2) in train mode, ``forward(St, Lt)``.

The single-query attention runs in re-associated GEMV form (see
include/tmr.h, tmr_nl_attn_fwd): u = W2^T (W1 St + b1) once per clip, then one
pass over the L long-term rows for the scores and one for the context, so the
L x 512 x 512 projections of the reference (linear2/linear3 applied to every
LFB row) are never materialised.  ``Lt`` can be a dense (B,L,512) tensor or an
``LFBRows`` view (resident bank + device row table), in which case the rows are
read straight from the bank in HBM.
"""
import math

import torch
import torch.nn as nn
import torch.nn.init as init

from . import ops


class LFBRows:
    """Lt given as rows of the resident long-term feature bank: bank (N,D) fp32 on the
    device, rows (B,L) int32 (tmr_lfb_index output)."""

    def __init__(self, bank, rows):
        self.bank = bank
        self.rows = rows

    @property
    def shape(self):
        return (self.rows.shape[0], self.rows.shape[1], self.bank.shape[1])

    def dense(self):
        return ops.lfb_gather(self.bank, self.rows)


class _DropoutRNG:
    """Counter-based dropout masks (tmr_dropout_mask): seed from torch's generator, a new
    offset per call."""

    def __init__(self):
        self.seed = None
        self.offset = 0

    def mask(self, n, p, like):
        if self.seed is None:
            self.seed = int(torch.initial_seed()) & 0xFFFFFFFFFFFF
        m = ops.dropout_mask(n, p, self.seed, self.offset, like)
        self.offset += n
        return m


class NLBlockFn(torch.autograd.Function):
    """One autograd node over tmr_nlblock_fwd / tmr_nlblock_bwd (the whole block is one C call
    each way; include/tmr.h)."""

    @staticmethod
    def forward(ctx, St, lt, rows, mask, L, w1, b1, w2, b2, w3, b3, g, bt, w4, b4):
        St = St.contiguous()
        weights = [t.detach().contiguous().reshape(-1) if t.dim() == 2 and t.shape[0] == 1
                   else t.detach().contiguous() for t in (w1, b1, w2, b2, w3, b3, g, bt, w4, b4)]
        out, saved = ops.nlblock_fwd(St, lt, rows, L, mask, weights)
        ctx.save_for_backward(St, lt, rows, mask, saved, *weights)
        ctx.L = L
        ctx.lt_grad = ctx.needs_input_grad[1] and rows is None
        ctx.g_shape = g.shape
        return out

    @staticmethod
    def backward(ctx, dout):
        St, lt, rows, mask, saved, *weights = ctx.saved_tensors
        dSt, dlt, gr = ops.nlblock_bwd(dout.contiguous(), St, lt, rows, ctx.L, mask, saved,
                                       weights, ctx.lt_grad)
        dw1, db1, dw2, db2, dw3, db3, dg, dbt, dw4, db4 = gr
        return (dSt, dlt, None, None, None, dw1, db1, dw2, db2, dw3, db3,
                dg.view(ctx.g_shape), dbt.view(ctx.g_shape), dw4, db4)


class NLBlock(nn.Module):
    def __init__(self, feature_num=512):
        super().__init__()
        if feature_num != 512:
            raise ValueError("NLBlock is fixed at 512 features (LayerNorm([1,512]) in the reference)")
        self.linear1 = nn.Linear(feature_num, feature_num)
        self.linear2 = nn.Linear(feature_num, feature_num)
        self.linear3 = nn.Linear(feature_num, feature_num)
        self.linear4 = nn.Linear(feature_num, feature_num)
        self.layer_norm = nn.LayerNorm([1, 512])
        self.dropout = nn.Dropout(0.2)
        init.xavier_uniform_(self.linear1.weight)
        init.xavier_uniform_(self.linear2.weight)
        init.xavier_uniform_(self.linear3.weight)
        init.xavier_uniform_(self.linear4.weight)
        self._rng = _DropoutRNG()
        self.forced_mask = None  # parity tests: externally supplied scaled mask (B,512)

    def drop_mask(self, B, like):
        """The Dropout(0.2) mask of this forward (scaled by 1/0.8), or None in eval mode."""
        if not (self.training and self.dropout.p > 0):
            return None
        if self.forced_mask is not None:
            return self.forced_mask
        return self._rng.mask(B * 512, self.dropout.p, like).view(B, 512)

    def forward(self, St, Lt):
        B = St.shape[0]
        if isinstance(Lt, LFBRows):
            lt, rows, L = Lt.bank, Lt.rows, Lt.rows.shape[1]
        else:
            lt, rows, L = Lt.contiguous(), None, Lt.shape[1]
        mask = self.drop_mask(B, St)
        return NLBlockFn.apply(St, lt, rows, mask, L,
                               self.linear1.weight, self.linear1.bias,
                               self.linear2.weight, self.linear2.bias,
                               self.linear3.weight, self.linear3.bias,
                               self.layer_norm.weight, self.layer_norm.bias,
                               self.linear4.weight, self.linear4.bias)
