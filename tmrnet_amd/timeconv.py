"""TimeConv (multi-scale temporal convolution over the LFB) on libtmr kernels.

Drop-in for ``TimeConv`` of code/Training TMRNet/NLBlock_MutiConv6_3.py:43-79 (used at
train_non-local_mutiConv_resnet.py:246): parameters timeconv{1,2,3} = Conv1d(512,512,k,pad=(k-1)/2)
with k = 3, 5, 7 (same names, shapes, torch default init), output
max(x, conv3(x), conv5(x), conv7(x), maxpool2(pad_left0(x))) elementwise.

The reference hard-codes L=30 (``view(-1,30,512,1)``, :57-77) and raises for any other L;
this module accepts any L (identical results at L=30, pinned by tests/golden/timeconv_L30.npz).
Each Conv1d runs as an implicit-GEMM conv on the (B, L, 1, 512) NHWC view (L as H, kernel k x 1,
padding (k-1)/2 along L only); the max-of-5 and its gradient routing are one kernel each.
"""
import torch
import torch.nn as nn

from . import ops
from ._lib import call, stream_ptr


class TimeConvFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2, w3, b3):
        x = x.contiguous()
        B, L, C = x.shape
        x4 = x.view(B, L, 1, C)
        ys, wks = [], []
        for w, b in ((w1, b1), (w2, b2), (w3, b3)):
            k = w.shape[2]
            wk = w.detach().permute(0, 2, 1).contiguous().view(w.shape[0], k, 1, C)  # KRSC
            ys.append(ops.conv_fwd(x4, wk, 1, (k - 1) // 2, bias=b.detach(), pad_w=0))
            wks.append(wk)
        out = torch.empty_like(x)
        code = torch.empty((B, L, C), dtype=torch.uint8, device=x.device)
        call("tmr_timeconv_max5_fwd", x, ys[0], ys[1], ys[2], out, code, B, L, C, stream_ptr())
        ctx.save_for_backward(x, code, *wks)
        return out

    @staticmethod
    def backward(ctx, dy):
        x, code, wk1, wk2, wk3 = ctx.saved_tensors
        B, L, C = x.shape
        dy = dy.contiguous()
        d = [torch.empty_like(dy) for _ in range(3)]
        want_dx = ctx.needs_input_grad[0]
        dx = torch.empty_like(dy) if want_dx else None
        call("tmr_timeconv_max5_bwd", dy, code, d[0], d[1], d[2], dx, B, L, C, stream_ptr())
        x4 = x.view(B, L, 1, C)
        grads = []
        for di, wk in zip(d, (wk1, wk2, wk3)):
            k = wk.shape[1]
            d4 = di.view(B, L, 1, C)
            dw_oihw = ops.conv_wgrad(x4, d4, k, 1, 1, (k - 1) // 2, pad_w=0)   # (C, C, k, 1)
            grads.append(dw_oihw.view(C, C, k))
            grads.append(ops.col_sum(di, B * L, C, C))
            if want_dx:
                ops.conv_dgrad(d4, wk, (L, 1), 1, (k - 1) // 2, out=dx.view(B, L, 1, C), beta=1.0,
                               pad_w=0)
        return (dx,) + tuple(grads)


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
