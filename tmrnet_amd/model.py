"""TMRNet models with the reference's nn.Module surface, running on libtmr kernels.

* ``resnet_lstm``      -- inline TMRNet of code/Training TMRNet/train_only_non-local_pretrained.py:201-240
                           (``time_conv=True``: train_non-local_mutiConv_resnet.py:208-253;
                           ``backbone='resnest50'``: train_non-local_mutiConv_resnest.py:204-249)
* ``resnet_lstm_LFB``  -- frozen LFB extractor, train_only_non-local_pretrained.py:243-270
* ``MemoryBankModel``  -- memory-bank model, Training memory bank model/train_singlenet_phase_1fc.py:201-232

State-dict keys are the reference's (share.*, lstm.*, nl_block.*, time_conv.*,
fc_h_c.*, fc_c.*, fc.*).  The reference reads the clip length from a module
global (``sequence_length`` / ``SEQ_LENGTH``, :229); here it is the
``seq_len`` constructor argument (default 10 as in the reference's CLI).
"""
import torch
import torch.nn as nn
import torch.nn.init as init

from . import ops
from ._lib import call, stream_ptr
from .lstm import LSTM
from .nlblock import NLBlock, LFBRows, _DropoutRNG
from .trunk import ResNet50Share


class ClipHeadFn(torch.autograd.Function):
    """The clip branch after the LSTM as ONE autograd node (train_only_non-local_pretrained.py:
    232-239): the last step of each clip y = lstm_out[:, T-1] (tmr_seq_last), the NLBlock on
    (y, Lt) (tmr_nlblock_fwd/bwd, NLBlock_MutiConv6_3.py:10-40) and the head on cat(y, y_1).
    y feeds both the NLBlock query and the head; the backward writes d(lstm_out) in one pass --
    the two gradients of y summed at step T-1, zeros elsewhere (tmr_seq_last_bwd) -- so no zero
    fill, scatter or add runs outside libtmr."""

    @staticmethod
    def forward(ctx, y_seq, lt, rows, nl_mask, L, head_mask, w1, b1, w2, b2, w3, b3, g, bt, w4, b4,
                wh, bh, wc, bc):
        y_seq = y_seq.contiguous()
        B, T, H = y_seq.shape
        y = torch.empty((B, H), dtype=y_seq.dtype, device=y_seq.device)
        call("tmr_seq_last", y_seq, y, B, T, H, stream_ptr())
        nlw = [t.detach().contiguous().reshape(-1) if t.dim() == 2 and t.shape[0] == 1
               else t.detach().contiguous() for t in (w1, b1, w2, b2, w3, b3, g, bt, w4, b4)]
        y1, saved = ops.nlblock_fwd(y, lt, rows, L, nl_mask, nlw)
        whd = wh.detach()
        h = ops.gemm_nt(y, whd, bias=bh.detach(), K=H, ldb=2 * H)
        ops.gemm_nt(y1, whd[:, H:], out=h, beta=1.0, K=H, ldb=2 * H)
        a = ops.mask_relu_fwd(h, head_mask)
        logits = ops.gemm_nt(a, wc.detach(), bias=bc.detach())
        ctx.save_for_backward(y, y1, lt, rows, nl_mask, saved, head_mask, a, wh, wc, *nlw)
        ctx.cfg = (B, T, H, L, ctx.needs_input_grad[1] and rows is None, g.shape)
        return logits

    @staticmethod
    def backward(ctx, dl):
        y, y1, lt, rows, nl_mask, saved, head_mask, a, wh, wc, *nlw = ctx.saved_tensors
        B, T, H, L, lt_grad, g_shape = ctx.cfg
        dl = dl.contiguous()
        K = dl.shape[1]
        dwc = ops.gemm_tn(dl, a)
        dbc = ops.col_sum(dl, B, K, K)
        da = ops.gemm_nn(dl, wc.detach())
        dh = ops.mask_relu_bwd(da, a, head_mask)
        whd = wh.detach()
        dy = ops.gemm_nn(dh, whd, N=H, ldb=2 * H)
        dy1 = ops.gemm_nn(dh, whd[:, H:], N=H, ldb=2 * H)
        dwh = torch.empty_like(whd)
        ops.gemm_tn(dh, y, out=dwh, N=H, ldc=2 * H)
        ops.gemm_tn(dh, y1, out=dwh[:, H:], N=H, ldc=2 * H)
        dbh = ops.col_sum(dh, B, dh.shape[1], dh.shape[1])
        dst, dlt, gr = ops.nlblock_bwd(dy1, y, lt, rows, L, nl_mask, saved, nlw, lt_grad)
        dw1, db1, dw2, db2, dw3, db3, dg, dbt, dw4, db4 = gr
        dy_seq = torch.empty((B, T, H), dtype=dl.dtype, device=dl.device)
        call("tmr_seq_last_bwd", dy, dst, dy_seq, B, T, H, stream_ptr())
        return (dy_seq, dlt, None, None, None, None, dw1, db1, dw2, db2, dw3, db3,
                dg.view(g_shape), dbt.view(g_shape), dw4, db4, dwh, dbh, dwc, dbc)


class LinearMaskFn(torch.autograd.Function):
    """out = (x * mask) W^T + b  (dropout then Linear; train_singlenet_phase_1fc.py:230-231)."""

    @staticmethod
    def forward(ctx, x, mask, w, b):
        x = x.contiguous()
        xm = ops.mul(x, mask) if mask is not None else x
        out = ops.gemm_nt(xm, w.detach(), bias=b.detach())
        ctx.save_for_backward(xm, mask, w)
        return out

    @staticmethod
    def backward(ctx, dout):
        xm, mask, w = ctx.saved_tensors
        dout = dout.contiguous()
        B, K = dout.shape
        dw = ops.gemm_tn(dout, xm)
        db = ops.col_sum(dout, B, K, K)
        dxm = ops.gemm_nn(dout, w.detach())
        dx = ops.mul(dxm, mask) if mask is not None else dxm
        return dx, None, dw, db


def _frames_to_features(share, x):
    """x: (B,T,3,224,224)/(F,3,224,224) NCHW fp32, or an NHWC4 (F,224,224,4) tensor."""
    if x.dim() == 4 and x.shape[-1] == 4 and x.shape[1] != 3:
        return share.features_nhwc4(x.contiguous())
    return share(x).view(-1, 2048)


def _make_trunk(backbone, precision):
    if precision not in ("fp32", "bf16"):
        raise ValueError("precision must be 'fp32' or 'bf16', got %r" % precision)
    if backbone == "resnet50":
        return ResNet50Share(precision=precision)
    if backbone == "resnest50":
        from .resnest import ResNeSt50Share
        return ResNeSt50Share(precision=precision)
    raise ValueError("unknown backbone %r" % backbone)


class resnet_lstm(nn.Module):  # noqa: N801  (reference class name)
    """precision='bf16' runs the trunk convolutions (fwd, dgrad, wgrad) with bf16 operands on
    the bf16 matrix cores, fp32 accumulation, fp32 activations/BN/master weights (the bf16
    configs C4/C5); everything else stays fp32."""

    def __init__(self, seq_len=10, num_classes=7, time_conv=False, backbone="resnet50",
                 precision="fp32"):
        super().__init__()
        self.seq_len = seq_len
        self.share = _make_trunk(backbone, precision)
        self.lstm = LSTM(2048, 512, batch_first=True)
        self.fc_c = nn.Linear(512, num_classes)
        self.fc_h_c = nn.Linear(1024, 512)
        self.nl_block = NLBlock()
        self.dropout = nn.Dropout(p=0.5)
        if time_conv:
            from .timeconv import TimeConv
            self.time_conv = TimeConv()
        init.xavier_normal_(self.lstm.all_weights[0][0])
        init.xavier_normal_(self.lstm.all_weights[0][1])
        init.xavier_uniform_(self.fc_c.weight)
        init.xavier_uniform_(self.fc_h_c.weight)
        self._rng = _DropoutRNG()
        self.forced_head_mask = None  # parity tests: scaled (B,512) mask

    def forward(self, x, long_feature=None):
        T = self.seq_len
        feat = _frames_to_features(self.share, x)
        self.lstm.flatten_parameters()
        y_seq, _ = self.lstm(feat.view(-1, T, 2048))   # y.view(-1,512)[T-1::T] inside ClipHeadFn
        Lt = long_feature
        if hasattr(self, "time_conv"):
            if isinstance(Lt, LFBRows):
                Lt = Lt.dense()
            Lt = self.time_conv(Lt)
        nl = self.nl_block
        if isinstance(Lt, LFBRows):
            lt, rows, L = Lt.bank, Lt.rows, Lt.rows.shape[1]
        else:
            lt, rows, L = Lt.contiguous(), None, Lt.shape[1]
        B = y_seq.shape[0]
        nl_mask = nl.drop_mask(B, y_seq)
        mask = None
        if self.training and self.dropout.p > 0:
            mask = (self.forced_head_mask if self.forced_head_mask is not None
                    else self._rng.mask(B * 512, self.dropout.p, y_seq).view(B, 512))
        return ClipHeadFn.apply(y_seq, lt, rows, nl_mask, L, mask,
                                nl.linear1.weight, nl.linear1.bias, nl.linear2.weight,
                                nl.linear2.bias, nl.linear3.weight, nl.linear3.bias,
                                nl.layer_norm.weight, nl.layer_norm.bias, nl.linear4.weight,
                                nl.linear4.bias, self.fc_h_c.weight, self.fc_h_c.bias,
                                self.fc_c.weight, self.fc_c.bias)


class resnet_lstm_LFB(nn.Module):  # noqa: N801
    def __init__(self, seq_len=10, backbone="resnet50", precision="fp32"):
        super().__init__()
        self.seq_len = seq_len
        self.share = _make_trunk(backbone, precision)
        self.lstm = LSTM(2048, 512, batch_first=True)
        init.xavier_normal_(self.lstm.all_weights[0][0])
        init.xavier_normal_(self.lstm.all_weights[0][1])

    def forward(self, x):
        T = self.seq_len
        feat = _frames_to_features(self.share, x)
        y, _ = self.lstm(feat.view(-1, T, 2048))
        return y[:, T - 1, :]


class MemoryBankModel(nn.Module):
    """ResNet50 -> LSTM -> dropout(0.2) -> fc on every frame (returns (F, K) logits; the
    caller keeps outputs[T-1::T], train_singlenet_phase_1fc.py:555)."""

    def __init__(self, seq_len=10, num_classes=7, indexed_trunk=False):
        super().__init__()
        self.seq_len = seq_len
        trunk = ResNet50Share(indexed=indexed_trunk)
        if indexed_trunk:
            self.res = trunk
        else:
            self.share = trunk
        self.lstm = LSTM(2048, 512, batch_first=True)
        self.fc = nn.Linear(512, num_classes)
        self.dropout = nn.Dropout(p=0.2)
        init.xavier_normal_(self.lstm.all_weights[0][0])
        init.xavier_normal_(self.lstm.all_weights[0][1])
        init.xavier_uniform_(self.fc.weight)
        self._rng = _DropoutRNG()
        self.forced_mask = None

    def trunk(self):
        return self.res if hasattr(self, "res") else self.share

    def forward(self, x, seq_len=None):
        """seq_len overrides the constructor's T for this call only (no module state is written,
        so one instance can be driven from several threads, as DataParallel replicas are)."""
        T = self.seq_len if seq_len is None else int(seq_len)
        feat = _frames_to_features(self.trunk(), x)
        y, _ = self.lstm(feat.view(-1, T, 2048))
        y = y.reshape(-1, 512)
        mask = None
        if self.training and self.dropout.p > 0:
            mask = (self.forced_mask if self.forced_mask is not None
                    else self._rng.mask(y.numel(), self.dropout.p, y).view_as(y))
        return LinearMaskFn.apply(y, mask, self.fc.weight, self.fc.bias)
