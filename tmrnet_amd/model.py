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
from .lstm import LSTM
from .nlblock import NLBlock, LFBRows, _DropoutRNG
from .trunk import ResNet50Share


class HeadFn(torch.autograd.Function):
    """cat([y, y1]) -> fc_h_c -> dropout(mask) -> ReLU -> fc_c (train_only_non-local_pretrained.py:236-239).
    The concat is folded into two GEMMs on the column halves of fc_h_c.weight."""

    @staticmethod
    def forward(ctx, y, y1, mask, wh, bh, wc, bc):
        y = y.contiguous(); y1 = y1.contiguous()
        B, D = y.shape
        whd = wh.detach()
        h = ops.gemm_nt(y, whd, bias=bh.detach(), K=D, ldb=2 * D)
        ops.gemm_nt(y1, whd[:, D:], out=h, beta=1.0, K=D, ldb=2 * D)
        a = ops.mask_relu_fwd(h, mask)
        logits = ops.gemm_nt(a, wc.detach(), bias=bc.detach())
        ctx.save_for_backward(y, y1, mask, a, wh, wc)
        return logits

    @staticmethod
    def backward(ctx, dl):
        y, y1, mask, a, wh, wc = ctx.saved_tensors
        dl = dl.contiguous()
        B, K = dl.shape
        D = y.shape[1]
        dwc = ops.gemm_tn(dl, a)
        dbc = ops.col_sum(dl, B, K, K)
        da = ops.gemm_nn(dl, wc.detach())
        dh = ops.mask_relu_bwd(da, a, mask)
        whd = wh.detach()
        dy = ops.gemm_nn(dh, whd, N=D, ldb=2 * D)
        dy1 = ops.gemm_nn(dh, whd[:, D:], N=D, ldb=2 * D)
        dwh = torch.empty_like(whd)
        ops.gemm_tn(dh, y, out=dwh, N=D, ldc=2 * D)
        ops.gemm_tn(dh, y1, out=dwh[:, D:], N=D, ldc=2 * D)
        dbh = ops.col_sum(dh, B, dh.shape[1], dh.shape[1])
        return dy, dy1, None, dwh, dbh, dwc, dbc


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
        y, _ = self.lstm(feat.view(-1, T, 2048))
        y = y[:, T - 1, :]                      # == y.view(-1,512)[T-1::T]
        Lt = long_feature
        if hasattr(self, "time_conv"):
            if isinstance(Lt, LFBRows):
                Lt = Lt.dense()
            Lt = self.time_conv(Lt)
        y_1 = self.nl_block(y, Lt)
        mask = None
        if self.training and self.dropout.p > 0:
            B = y.shape[0]
            mask = (self.forced_head_mask if self.forced_head_mask is not None
                    else self._rng.mask(B * 512, self.dropout.p, y).view(B, 512))
        return HeadFn.apply(y, y_1, mask, self.fc_h_c.weight, self.fc_h_c.bias,
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

    def forward(self, x):
        T = self.seq_len
        feat = _frames_to_features(self.trunk(), x)
        y, _ = self.lstm(feat.view(-1, T, 2048))
        y = y.reshape(-1, 512)
        mask = None
        if self.training and self.dropout.p > 0:
            mask = (self.forced_mask if self.forced_mask is not None
                    else self._rng.mask(y.numel(), self.dropout.p, y).view_as(y))
        return LinearMaskFn.apply(y, mask, self.fc.weight, self.fc.bias)
