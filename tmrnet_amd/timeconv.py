"""TimeConv (multi-scale temporal convolution over the LFB) on libtmr kernels.

Drop-in for ``TimeConv`` of code/Training TMRNet/NLBlock_MutiConv6_3.py:43-79 (used at
train_non-local_mutiConv_resnet.py:246): parameters timeconv{1,2,3} = Conv1d(512,512,k,pad=(k-1)/2)
with k = 3, 5, 7 (same names, shapes, torch default init), output
max(x, conv3(x), conv5(x), conv7(x), maxpool2(pad_left0(x))) elementwise.

The reference hard-codes L=30 (``view(-1,30,512,1)``, :57-77) and raises for any other L;
this module accepts any L (identical results at L=30, pinned by tests/golden/timeconv_L30.npz).
Forward and backward are one C call each (tmr_timeconv_fwd / tmr_timeconv_wgrad, csrc/nlblock.hip):
each Conv1d runs as an implicit-GEMM conv on the (B, L, 1, 512) NHWC view (L as H, kernel k x 1,
padding (k-1)/2 along L only); the max-of-5 and its gradient routing are one kernel each.
"""
import torch
import torch.nn as nn

from . import ops


class TimeConvFn(torch.autograd.Function):
    """tmr_timeconv_fwd / tmr_timeconv_wgrad (include/tmr.h): one C call each way."""

    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2, w3, b3):
        x = x.contiguous()
        ws = [t.detach().contiguous() for t in (w1, b1, w2, b2, w3, b3)]
        out, saved = ops.timeconv_fwd(x, *ws)
        ctx.save_for_backward(x, saved, ws[0], ws[2], ws[4])
        return out

    @staticmethod
    def backward(ctx, dy):
        x, saved, w1, w2, w3 = ctx.saved_tensors
        dx, dw1, db1, dw2, db2, dw3, db3 = ops.timeconv_wgrad(dy.contiguous(), x, saved, w1, w2,
                                                              w3, ctx.needs_input_grad[0])
        return dx, dw1, db1, dw2, db2, dw3, db3


class TimeConv(nn.Module):
    def __init__(self):
        super().__init__()
        self.timeconv1 = nn.Conv1d(512, 512, kernel_size=3, padding=1)
        self.timeconv2 = nn.Conv1d(512, 512, kernel_size=5, padding=2)
        self.timeconv3 = nn.Conv1d(512, 512, kernel_size=7, padding=3)
        self.maxpool_m = nn.MaxPool1d(2, stride=1)
        self.maxpool = nn.AdaptiveMaxPool2d((512, 1))

    def forward(self, x):
        return TimeConvFn.apply(x, self.timeconv1.weight, self.timeconv1.bias,
                                self.timeconv2.weight, self.timeconv2.bias,
                                self.timeconv3.weight, self.timeconv3.bias)
