"""CPU oracle: a plain-PyTorch (fp32, CPU) restatement of TMRNet's train-step hot path.

TEST INFRASTRUCTURE ONLY.  Nothing in ``tmrnet_amd/`` imports this module; only
``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg
use it, and only as the checker / the timed CPU baseline.  The product path
runs the HIP kernels of ``libtmr.so`` and fails loudly without them.

Every function cites the reference code it restates (paths relative to the
reference checkout, ``code/``):

* ``NLBlockRef``      -- ``Training TMRNet/NLBlock_MutiConv6_3.py:10-40``
                         (pinned by ``tests/golden/nlblock_L*.npz``)
* ``TimeConvRef``     -- ``Training TMRNet/NLBlock_MutiConv6_3.py:43-79``,
                         generalised from the hard-coded L=30 (``:57-77``) to any L;
                         identical at L=30 (pinned by ``tests/golden/timeconv_L30.npz``)
* ``ResNet50Ref``     -- torchvision ``resnet50`` as used by
                         ``Training TMRNet/train_only_non-local_pretrained.py:204-214``.
                         torchvision is not vendored in the reference nor installed here:
                         restated from its published v1.5 definition (stride on the 3x3,
                         kaiming_normal fan_out convs, BN gamma=1 beta=0).  PARITY UNPINNED
                         for the trunk beyond torch's own Conv2d/BatchNorm2d semantics.
* ``TMRNetRef``       -- inline ``resnet_lstm`` (``train_only_non-local_pretrained.py:201-240``;
                         with ``time_conv``: ``train_non-local_mutiConv_resnet.py:208-253``)
* ``MemoryBankRef``   -- ``Training memory bank model/train_singlenet_phase_1fc.py:201-232``
* ``get_useful_start_idx`` / ``lfb_index_table`` --
                         ``train_only_non-local_pretrained.py:273-311`` (+ dict :507-511)
                         (pinned by ``tests/golden/lfb_index_*.npz``)
* ``crop_normalize_ref`` -- crop at a per-clip offset + ToTensor + Normalize
                         (``train_only_non-local_pretrained.py:101-126``, ``:335-341``)
* ``train_step_ref``  -- the step at ``train_only_non-local_pretrained.py:698-725``
* ``augment_ref``     -- the training transform classes RandomCrop / ColorJitter /
                         RandomHorizontalFlip / RandomRotation (train_only_non-local_pretrained.py
                         :101-177, composed :334-350) on PIL, with torchvision's thin F_pil
                         wrappers (adjust_brightness/contrast/saturation = ImageEnhance, adjust_hue
                         = HSV round trip, rotate = Image.rotate NEAREST fill 0) restated inline
                         (torchvision is not installed; PIL is)
* ``LFBModelRef`` / ``build_lfb_ref`` -- ``resnet_lstm_LFB`` (:243-270) and the LFB
                         construction loop (:534-607): eval mode, centre crop (:360-366),
                         clips in valid-start order, last hidden state per clip, float64 bank
* ``emulate_bf16_convs`` -- the bf16 configs (BASELINE.json configs[3], [4]) have no reference
                         implementation (the reference is fp32 only): this restates the
                         build's TMR_MATH_BF16 contract on torch ops -- every trunk conv with
                         operands rounded to bf16 (RNE), exact products, accumulation in the
                         tensor dtype; fwd rounds (x, w), dgrad (dy, w), wgrad (x, dy).
                         With activations=True (the train step's bf16-activation contract,
                         tmrnet_amd/trunk.py ACT16, both backbones) every conv output and every
                         Bottleneck output -- for ResNeSt-50 also relu(bn0) and the output of
                         the split attention and the avd pool output -- is stored rounded to
                         bf16 in train mode (straight-through: the rounding is storage,
                         gradients pass unchanged).
"""
import math

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F
import torch.nn.init as init

MEAN = (0.41757566, 0.26098573, 0.25888634)
STD = (0.21938758, 0.1983, 0.19342837)


# --------------------------------------------------------------------------
# NLBlock / TimeConv
# --------------------------------------------------------------------------
class NLBlockRef(nn.Module):
    """NLBlock_MutiConv6_3.py:10-40, op for op."""

    def __init__(self, feature_num=512):
        super().__init__()
        self.linear1 = nn.Linear(feature_num, feature_num)
        self.linear2 = nn.Linear(feature_num, feature_num)
        self.linear3 = nn.Linear(feature_num, feature_num)
        self.linear4 = nn.Linear(feature_num, feature_num)
        self.layer_norm = nn.LayerNorm([1, 512])
        self.dropout = nn.Dropout(0.2)
        for lin in (self.linear1, self.linear2, self.linear3, self.linear4):
            init.xavier_uniform_(lin.weight)

    def forward(self, St, Lt, drop_mask=None):
        St_1 = self.linear1(St.view(-1, 1, 512))
        Lt_1 = self.linear2(Lt).transpose(1, 2)
        SL = torch.matmul(St_1, Lt_1) * ((1 / 512) ** 0.5)
        SL = F.softmax(SL, dim=2)
        SLL = torch.matmul(SL, self.linear3(Lt))
        SLL = F.relu(self.layer_norm(SLL))
        SLL = self.linear4(SLL)
        if drop_mask is not None:          # externally supplied dropout mask (already scaled)
            SLL = SLL * drop_mask.view(-1, 1, 512)
        else:
            SLL = self.dropout(SLL)
        return St + SLL.view(-1, 512)


class TimeConvRef(nn.Module):
    """NLBlock_MutiConv6_3.py:43-79 generalised to any L.

    y = max(x, conv3(x), conv5(x), conv7(x), maxpool2(pad_left0(x))) elementwise;
    the reference's AdaptiveMaxPool2d((512,1)) over the 5 stacked branches (:75-76)
    is exactly that max (verified against the golden fixture at L=30).
    """

    def __init__(self):
        super().__init__()
        self.timeconv1 = nn.Conv1d(512, 512, kernel_size=3, padding=1)
        self.timeconv2 = nn.Conv1d(512, 512, kernel_size=5, padding=2)
        self.timeconv3 = nn.Conv1d(512, 512, kernel_size=7, padding=3)
        self.maxpool_m = nn.MaxPool1d(2, stride=1)

    def forward(self, x):
        xt = x.transpose(1, 2)                       # (B,512,L)
        y1 = self.timeconv1(xt)
        y2 = self.timeconv2(xt)
        y3 = self.timeconv3(xt)
        y4 = self.maxpool_m(F.pad(xt, (1, 0), mode="constant", value=0))
        y = torch.stack((xt, y1, y2, y3, y4), dim=3).amax(dim=3)
        return y.transpose(1, 2).contiguous()


# --------------------------------------------------------------------------
# ResNet-50 v1.5 (torchvision definition, torchvision state_dict keys)
# --------------------------------------------------------------------------
class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        self.conv1 = nn.Conv2d(inplanes, planes, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.conv2 = nn.Conv2d(planes, planes, 3, stride=stride, padding=1, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        self.conv3 = nn.Conv2d(planes, planes * 4, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(planes * 4)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample
        self.stride = stride

    def forward(self, x):
        identity = x
        rg = getattr(self, "round_grad", False) and self.training   # emulate_bf16_convs(grads)
        out = self.relu(self.bn1(self.conv1(x)))
        if rg:
            out = _GradRoundFn.apply(out)
        out = self.relu(self.bn2(self.conv2(out)))
        if rg:
            out = _GradRoundFn.apply(out)
        out = self.bn3(self.conv3(out))
        if self.downsample is not None:
            identity = self.downsample(x)
        out = _act(self, out + identity)
        if getattr(self, "round_out", False) and self.training:   # emulate_bf16_convs(activations)
            out = _RoundFn.apply(out)
        if getattr(self, "round_res_grad", False) and self.training:
            # trunk.R16: the gradient of this block output (the residual stream's), masked by the
            # ReLU, is stored bf16 -- mask * round(g) == round(mask * g)
            out = _GradRoundFn.apply(out)
        return out


def _act(blk, v):
    """The block output ReLU; with `blk.forced_act` set (a 0/1 tensor of v's shape, test
    instrumentation) the given active set instead -- v * act, the ReLU's value and gradient on
    that set.  The geometry tests force the HIP step's own last-block active set on both oracles,
    as they do for the head ReLU (tests/test_geometry_gpu.py)."""
    act = getattr(blk, "forced_act", None)
    if act is None:
        return blk.relu(v)
    blk.pre_act = v.detach()   # (the tests count the elements the forced set moves)
    return v * act.to(v.dtype)


def make_layer(inplanes, planes, blocks, stride):
    downsample = None
    if stride != 1 or inplanes != planes * 4:
        downsample = nn.Sequential(nn.Conv2d(inplanes, planes * 4, 1, stride=stride, bias=False),
                                   nn.BatchNorm2d(planes * 4))
    layers = [Bottleneck(inplanes, planes, stride, downsample)]
    for _ in range(1, blocks):
        layers.append(Bottleneck(planes * 4, planes))
    return nn.Sequential(*layers)


def resnet50_share():
    """nn.Sequential with the reference's `share.*` module names (:204-214)."""
    share = nn.Sequential()
    share.add_module("conv1", nn.Conv2d(3, 64, 7, stride=2, padding=3, bias=False))
    share.add_module("bn1", nn.BatchNorm2d(64))
    share.add_module("relu", nn.ReLU(inplace=True))
    share.add_module("maxpool", nn.MaxPool2d(3, stride=2, padding=1))
    share.add_module("layer1", make_layer(64, 64, 3, 1))
    share.add_module("layer2", make_layer(256, 128, 4, 2))
    share.add_module("layer3", make_layer(512, 256, 6, 2))
    share.add_module("layer4", make_layer(1024, 512, 3, 2))
    share.add_module("avgpool", nn.AdaptiveAvgPool2d((1, 1)))
    for m in share.modules():
        if isinstance(m, nn.Conv2d):
            nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
        elif isinstance(m, nn.BatchNorm2d):
            nn.init.constant_(m.weight, 1)
            nn.init.constant_(m.bias, 0)
    return share


# --------------------------------------------------------------------------
# ResNeSt-50 (radix 2, cardinality 1, deep stem 32, avg_down, avd) -- the
# third-party `resnest` package's resnest50() used at
# Training TMRNet/train_non-local_mutiConv_resnest.py:210-220.  The package is
# neither vendored in the reference nor installed here: restated from its
# published definition.  PARITY UNPINNED (checked by parameter count
# 25,434,240 and 5.369 GMAC/frame).
# --------------------------------------------------------------------------
class SplAtConv2d(nn.Module):
    def __init__(self, in_channels, channels, stride=1, radix=2, reduction_factor=4):
        super().__init__()
        inter = max(in_channels * radix // reduction_factor, 32)
        self.radix = radix
        self.channels = channels
        self.conv = nn.Conv2d(in_channels, channels * radix, 3, stride, 1, groups=radix, bias=False)
        self.bn0 = nn.BatchNorm2d(channels * radix)
        self.relu = nn.ReLU(inplace=True)
        self.fc1 = nn.Conv2d(channels, inter, 1, groups=1)
        self.bn1 = nn.BatchNorm2d(inter)
        self.fc2 = nn.Conv2d(inter, channels * radix, 1, groups=1)

    def forward(self, x):
        x = self.relu(self.bn0(self.conv(x)))
        rnd = getattr(self, "round_out", False) and self.training   # emulate_bf16_convs(activations)
        if rnd:   # relu(bn0) as a stored bf16 activation (the HIP path recomputes it rounded)
            x = _RoundFn.apply(x)
        b = x.shape[0]
        splits = torch.split(x, self.channels, dim=1)
        gap = F.adaptive_avg_pool2d(sum(splits), 1)
        gap = self.relu(self.bn1(self.fc1(gap)))
        att = self.fc2(gap).view(b, 1, self.radix, -1).transpose(1, 2)
        att = F.softmax(att, dim=1).reshape(b, -1, 1, 1)
        atts = torch.split(att, self.channels, dim=1)
        out = sum(a * s_ for a, s_ in zip(atts, splits))
        return _RoundFn.apply(out) if rnd else out


class BottleneckS(nn.Module):
    expansion = 4

    def __init__(self, inplanes, planes, stride=1, downsample=None, is_first=False):
        super().__init__()
        gw = planes
        self.conv1 = nn.Conv2d(inplanes, gw, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(gw)
        self.avd = stride > 1 or is_first
        if self.avd:
            self.avd_layer = nn.AvgPool2d(3, stride, padding=1)
            stride = 1
        self.conv2 = SplAtConv2d(gw, gw, stride=stride)
        self.conv3 = nn.Conv2d(gw, planes * 4, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(planes * 4)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample

    def forward(self, x):
        rnd = getattr(self, "round_out", False) and self.training   # emulate_bf16_convs(activations)
        out = self.relu(self.bn1(self.conv1(x)))
        if getattr(self, "round_grad", False) and self.training:
            # resnest.py: the grouped conv's fused dgrad stores relu(bn1)'s gradient bf16 (G16)
            out = _GradRoundFn.apply(out)
        out = self.conv2(out)
        if self.avd:
            out = self.avd_layer(out)
            if rnd:
                out = _RoundFn.apply(out)
        out = self.bn3(self.conv3(out))
        res = self.downsample(x) if self.downsample is not None else x
        out = _act(self, out + res)
        out = _RoundFn.apply(out) if rnd else out
        if getattr(self, "round_res_grad", False) and self.training:   # trunk.R16, as Bottleneck
            out = _GradRoundFn.apply(out)
        return out


def _make_layer_s(inplanes, planes, blocks, stride):
    downsample = None
    if stride != 1 or inplanes != planes * 4:
        pool = (nn.AvgPool2d(stride, stride, ceil_mode=True, count_include_pad=False) if stride != 1
                else nn.AvgPool2d(1, 1, ceil_mode=True, count_include_pad=False))
        downsample = nn.Sequential(pool, nn.Conv2d(inplanes, planes * 4, 1, bias=False),
                                   nn.BatchNorm2d(planes * 4))
    layers = [BottleneckS(inplanes, planes, stride, downsample)]
    for _ in range(1, blocks):
        layers.append(BottleneckS(planes * 4, planes))
    return nn.Sequential(*layers)


class GlobalAvgPool2d(nn.Module):
    def forward(self, x):
        return F.adaptive_avg_pool2d(x, 1).view(x.size(0), -1)


def resnest50_share():
    share = nn.Sequential()
    share.add_module("conv1", nn.Sequential(
        nn.Conv2d(3, 32, 3, 2, 1, bias=False), nn.BatchNorm2d(32), nn.ReLU(inplace=True),
        nn.Conv2d(32, 32, 3, 1, 1, bias=False), nn.BatchNorm2d(32), nn.ReLU(inplace=True),
        nn.Conv2d(32, 64, 3, 1, 1, bias=False)))
    share.add_module("bn1", nn.BatchNorm2d(64))
    share.add_module("relu", nn.ReLU(inplace=True))
    share.add_module("maxpool", nn.MaxPool2d(3, 2, 1))
    share.add_module("layer1", _make_layer_s(64, 64, 3, 1))
    share.add_module("layer2", _make_layer_s(256, 128, 4, 2))
    share.add_module("layer3", _make_layer_s(512, 256, 6, 2))
    share.add_module("layer4", _make_layer_s(1024, 512, 3, 2))
    share.add_module("avgpool", GlobalAvgPool2d())
    for m in share.modules():   # resnest ResNet.__init__ init
        if isinstance(m, nn.Conv2d):
            n = m.kernel_size[0] * m.kernel_size[1] * m.out_channels
            m.weight.data.normal_(0, math.sqrt(2.0 / n))
        elif isinstance(m, nn.BatchNorm2d):
            m.weight.data.fill_(1)
            m.bias.data.zero_()
    return share


# --------------------------------------------------------------------------
# TMRNet / memory-bank model
# --------------------------------------------------------------------------
def bf16_round(t):
    """Round to the nearest bf16 (ties to even), returned in t's dtype."""
    return t.to(torch.bfloat16).to(t.dtype)


ROUND_ALL = ("fx", "fw", "dy", "bx", "bw")


class _RoundFn(torch.autograd.Function):
    """Storage rounding to bf16 (RNE) with a straight-through gradient."""

    @staticmethod
    def forward(ctx, x):
        return bf16_round(x)

    @staticmethod
    def backward(ctx, g):
        return g


class _GradRoundFn(torch.autograd.Function):
    """Identity whose gradient is stored rounded to bf16 (RNE): the bf16 train step keeps the
    BN-output gradient of the non-residual units (relu(bn1), relu(bn2) of a Bottleneck) as bf16
    (tmrnet_amd/trunk.py G16, TMR_IO_G16)."""

    @staticmethod
    def forward(ctx, x):
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        return bf16_round(g)


class _Bf16ConvFn(torch.autograd.Function):
    """Conv with bf16-rounded operands.  `ops` names the roundings applied (all five by default,
    the contract; subsets are the attribution study of tests/golden/make_bf16_ensemble.py):
    fx / fw the forward's x and w, dy the output gradient, bx / bw the x and w the backward
    views read."""

    @staticmethod
    def forward(ctx, x, w, stride, padding, groups, ops=ROUND_ALL):
        xf = bf16_round(x) if "fx" in ops else x
        wf = bf16_round(w) if "fw" in ops else w
        ctx.save_for_backward(x, w)
        ctx.cfg = (stride, padding, groups, ops)
        return F.conv2d(xf, wf, None, stride, padding, 1, groups)

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        stride, padding, groups, ops = ctx.cfg
        xb = bf16_round(x) if "bx" in ops else x
        wb = bf16_round(w) if "bw" in ops else w
        gyb = bf16_round(gy) if "dy" in ops else gy
        dx = None
        if ctx.needs_input_grad[0]:
            dx = torch.nn.grad.conv2d_input(xb.shape, wb, gyb, stride, padding, 1, groups)
        dw = torch.nn.grad.conv2d_weight(xb, wb.shape, gyb, stride, padding, 1, groups)
        return dx, dw, None, None, None, None


class Bf16Conv2d(nn.Conv2d):
    """nn.Conv2d (no bias) whose operands are rounded to bf16 (see emulate_bf16_convs)."""

    def forward(self, x):
        assert self.bias is None
        y = _Bf16ConvFn.apply(x, self.weight, self.stride, self.padding, self.groups,
                              getattr(self, "round_ops", ROUND_ALL))
        if getattr(self, "round_out", False) and self.training:   # bf16-stored conv output
            y = _RoundFn.apply(y)
        return y


def emulate_bf16_convs(module, skip=("fc1", "fc2"), activations=False, grads=None, res_grads=None,
                       ops=ROUND_ALL):
    """Switch every trunk Conv2d of `module` to bf16-operand math (class swap, so deepcopy
    and .double() keep it); the split-attention fc1/fc2 (GEMMs in fp32 on the device) stay.
    activations=True: in train mode the conv outputs and the Bottleneck outputs are rounded to
    bf16 as well (the bf16-activation contract of the train step; ResNeSt-50 also stores the
    split attention's relu(bn0) input and output and the avd pool output as bf16).
    grads (default: activations): the ResNet-50 Bottleneck's relu(bn1) / relu(bn2) gradients (the
    ResNeSt BottleneckS's relu(bn1), round 4) are rounded to bf16 in the backward (trunk.G16: the
    fused dgrad stores them bf16), and so is the
    gradient of every Bottleneck (ResNeSt: BottleneckS) output but the last (trunk.R16: the
    residual stream's gradient, written by the next block's conv1 dgrad; the last block's comes
    from the avgpool in fp32).
    res_grads (default: grads) switches the second part alone.  ops: the operand roundings of
    every conv (_Bf16ConvFn; the contract rounds all five)."""
    grads = activations if grads is None else grads
    res_grads = grads if res_grads is None else res_grads
    blocks = [m for m in module.modules() if isinstance(m, (Bottleneck, BottleneckS))]
    for name, m in module.named_modules():
        if type(m) is nn.Conv2d and name.split(".")[-1] not in skip:
            m.__class__ = Bf16Conv2d
            m.round_out = activations
            m.round_ops = tuple(ops)
        elif isinstance(m, (Bottleneck, BottleneckS, SplAtConv2d)):
            m.round_out = activations
            if isinstance(m, (Bottleneck, BottleneckS)):
                m.round_grad = grads
            if isinstance(m, (Bottleneck, BottleneckS)):
                m.round_res_grad = res_grads and m is not blocks[-1]
    return module


class TMRNetRef(nn.Module):
    """Inline `resnet_lstm` (train_only_non-local_pretrained.py:201-240); with
    time_conv=True the mutiConv variant (train_non-local_mutiConv_resnet.py:208-253).
    precision='bf16': trunk convs with bf16 operands (emulate_bf16_convs); bf16_act (default on)
    adds the bf16 storage of the train step's activations (conv and block outputs, ResNeSt's split
    attention) in train mode."""

    def __init__(self, seq_len=10, num_classes=7, time_conv=False, backbone="resnet50",
                 precision="fp32", bf16_act=None):
        super().__init__()
        self.seq_len = seq_len
        self.share = resnet50_share() if backbone == "resnet50" else resnest50_share()
        if precision == "bf16":
            emulate_bf16_convs(self.share, activations=True if bf16_act is None else bf16_act)
        self.lstm = nn.LSTM(2048, 512, batch_first=True)
        self.fc_c = nn.Linear(512, num_classes)
        self.fc_h_c = nn.Linear(1024, 512)
        self.nl_block = NLBlockRef()
        self.dropout = nn.Dropout(p=0.5)
        if time_conv:
            self.time_conv = TimeConvRef()
        init.xavier_normal_(self.lstm.all_weights[0][0])
        init.xavier_normal_(self.lstm.all_weights[0][1])
        init.xavier_uniform_(self.fc_c.weight)
        init.xavier_uniform_(self.fc_h_c.weight)

    def forward(self, x, long_feature, masks=None):
        T = self.seq_len
        x = self.share(x.reshape(-1, 3, 224, 224)).reshape(-1, T, 2048)
        y, _ = self.lstm(x)
        y = y.contiguous().view(-1, 512)[T - 1::T]
        Lt = self.time_conv(long_feature) if hasattr(self, "time_conv") else long_feature
        if masks is None:
            y_1 = self.nl_block(y, Lt)
            h = self.dropout(self.fc_h_c(torch.cat([y, y_1], dim=1)))
        else:
            y_1 = self.nl_block(y, Lt, drop_mask=masks["nl"])
            h = self.fc_h_c(torch.cat([y, y_1], dim=1)) * masks["head"]
            if "head_act" in masks:
                # test hook: the head ReLU's active set taken from another run (the HIP step), so
                # a pre-ReLU unit within rounding distance of 0 cannot take the other branch here
                return self.fc_c(h * masks["head_act"])
        return self.fc_c(F.relu(h))


class MemoryBankRef(nn.Module):
    """train_singlenet_phase_1fc.py:201-232: trunk -> LSTM -> dropout(0.2) -> fc on all frames."""

    def __init__(self, seq_len=10, num_classes=7):
        super().__init__()
        self.seq_len = seq_len
        self.share = resnet50_share()
        self.lstm = nn.LSTM(2048, 512, batch_first=True)
        self.fc = nn.Linear(512, num_classes)
        self.dropout = nn.Dropout(p=0.2)
        init.xavier_normal_(self.lstm.all_weights[0][0])
        init.xavier_normal_(self.lstm.all_weights[0][1])
        init.xavier_uniform_(self.fc.weight)

    def forward(self, x, mask=None):
        x = self.share(x.reshape(-1, 3, 224, 224)).reshape(-1, self.seq_len, 2048)
        y, _ = self.lstm(x)
        y = y.contiguous().view(-1, 512)
        y = y * mask if mask is not None else self.dropout(y)
        return self.fc(y)


class LFBModelRef(nn.Module):
    """resnet_lstm_LFB (train_only_non-local_pretrained.py:243-270)."""

    def __init__(self, seq_len=10):
        super().__init__()
        self.seq_len = seq_len
        self.share = resnet50_share()
        self.lstm = nn.LSTM(2048, 512, batch_first=True)
        init.xavier_normal_(self.lstm.all_weights[0][0])
        init.xavier_normal_(self.lstm.all_weights[0][1])

    def forward(self, x):
        T = self.seq_len
        x = self.share(x.reshape(-1, 3, 224, 224)).reshape(-1, T, 2048)
        y, _ = self.lstm(x)
        return y.contiguous().view(-1, 512)[T - 1::T]


def build_lfb_ref(model, frames_u8, lengths, batch_clips=4):
    """The LFB construction loop of train_only_non-local_pretrained.py:547-607: SeqSampler over
    train_idx_LFB (each valid start + its T-1 successors, :491-494), test transform = centre crop
    (crop_type 1, :360-366), model in eval mode under no_grad, outputs appended row by row with
    np.concatenate onto a float64 (0, 512) array (:574-581).  frames_u8: (N,250,250,3) uint8."""
    T = model.seq_len
    model.eval()
    valid = get_useful_start_idx(T, lengths)
    off = int(round((frames_u8.shape[1] - 224) / 2.0))
    bank = np.zeros(shape=(0, 512))
    with torch.no_grad():
        for b0 in range(0, len(valid), batch_clips):
            starts = valid[b0:b0 + batch_clips]
            idx = [s + j for s in starts for j in range(T)]
            x = crop_normalize_ref(frames_u8[idx], [(off, off)] * len(starts), T)
            out = model(x.view(-1, T, 3, 224, 224))
            for j in range(len(out)):
                bank = np.concatenate((bank, out.data.cpu()[j].numpy().reshape(1, 512)), axis=0)
    return bank, valid


# --------------------------------------------------------------------------
# LFB index rule, input transform, loss, step
# --------------------------------------------------------------------------
def get_useful_start_idx(seq_len, lengths):
    """train_only_non-local_pretrained.py:273-280."""
    idx, count = [], 0
    for n in lengths:
        idx.extend(range(count, count + (n + 1 - seq_len)))
        count += n
    return idx


def lfb_index_table(starts_query, valid_starts, L):
    """Row table of get_long_feature (train_only_non-local_pretrained.py:293-311)
    with the start->row dict of :507-511: out[j][k] is the bank row for the
    k-th most recent earlier start of clip j, falling back to the last row that
    existed (own row at k=0), crossing video boundaries as the reference does."""
    row_of = {s: r for r, s in enumerate(valid_starts)}
    out = []
    for s in starts_query:
        s = int(s)
        last = row_of[s]
        rows = []
        for k in range(L):
            p = s - k - 1
            if p in row_of:
                last = row_of[p]
            rows.append(last)
        out.append(rows)
    return out


def crop_normalize_ref(frames_u8, offsets, seq_len):
    """frames (F,250,250,3) uint8 HWC, offsets (B,2) int (x1,y1) per clip ->
    (F,3,224,224) fp32: PIL crop((x1,y1,x1+224,y1+224)) then ToTensor+Normalize."""
    Fn = frames_u8.shape[0]
    out = torch.empty(Fn, 3, 224, 224, dtype=torch.float32)
    mean = torch.tensor(MEAN).view(3, 1, 1)
    std = torch.tensor(STD).view(3, 1, 1)
    for f in range(Fn):
        x1, y1 = (int(v) for v in offsets[f // seq_len])
        crop = frames_u8[f, y1:y1 + 224, x1:x1 + 224, :].permute(2, 0, 1).float() / 255.0
        out[f] = (crop - mean) / std
    return out


def _adjust_hue_pil(img, hue_factor):
    """torchvision (0.15) functional_pil.adjust_hue."""
    from PIL import Image
    h, s, v = img.convert("HSV").split()
    np_h = np.array(h, dtype=np.uint8)
    np_h = (np_h.astype(np.int64) + (int(math.trunc(hue_factor * 255)) & 255)) & 255  # uint8 wrap
    h = Image.fromarray(np_h.astype(np.uint8), "L")
    return Image.merge("HSV", (h, s, v)).convert("RGB")


def augment_ref(frames_u8, counts, seq_len, use_flip=1, crop=224):
    """Reference training transform per frame (PIL), then ToTensor + Normalize -> (F,3,crop,crop).
    frames_u8: numpy/torch uint8 (F, H, W, 3); counts: the transforms' call counter per frame."""
    import random
    from PIL import Image, ImageEnhance
    frames_u8 = np.asarray(frames_u8)
    mean = torch.tensor(MEAN).view(3, 1, 1)
    std = torch.tensor(STD).view(3, 1, 1)
    out = torch.empty(len(frames_u8), 3, crop, crop)
    rnd = random.Random()
    for i, (fr, count) in enumerate(zip(frames_u8, counts)):
        img = Image.fromarray(fr)
        seed = int(count) // seq_len
        w, h = img.size
        if not (w == crop and h == crop):                                   # RandomCrop :110-126
            rnd.seed(seed)
            x1 = rnd.randint(0, w - crop)
            y1 = rnd.randint(0, h - crop)
            img = img.crop((x1, y1, x1 + crop, y1 + crop))
        if use_flip == 1:                                                   # ColorJitter :162-177
            rnd.seed(seed)
            bf = rnd.uniform(1 - 0.1, 1 + 0.1)
            cf = rnd.uniform(1 - 0.1, 1 + 0.1)
            sf = rnd.uniform(1 - 0.1, 1 + 0.1)
            hf = rnd.uniform(-0.05, 0.05)
            img = ImageEnhance.Brightness(img).enhance(bf)
            img = ImageEnhance.Contrast(img).enhance(cf)
            img = ImageEnhance.Color(img).enhance(sf)
            img = _adjust_hue_pil(img, hf)
        rnd.seed(seed)                                                      # flip :133-141
        if rnd.random() < 0.5:
            img = img.transpose(Image.FLIP_LEFT_RIGHT)
        if use_flip == 1:                                                   # rotation :147-153
            rnd.seed(seed)
            angle = rnd.randint(-5, 5)
            img = img.rotate(angle, Image.NEAREST, expand=False, center=None, fillcolor=(0, 0, 0))
        t = torch.from_numpy(np.array(img, copy=True)).permute(2, 0, 1).float().div(255)
        out[i] = (t - mean) / std
    return out


def ce_sum_ref(logits, labels, weight=None):
    """nn.CrossEntropyLoss(size_average=False) / reduction='sum' (:631, mutiConv :780)."""
    return F.cross_entropy(logits, labels, weight=weight, reduction="sum")


def sgd_param_groups(model, lr):
    """Param groups of train_only_non-local_pretrained.py:646-655 (multi_optim=1)."""
    groups = [{"params": list(model.share.parameters())},
              {"params": list(model.lstm.parameters())}]
    if hasattr(model, "time_conv"):
        groups.append({"params": list(model.time_conv.parameters()), "lr": lr})
    for name in ("nl_block", "fc_h_c", "fc_c"):
        groups.append({"params": list(getattr(model, name).parameters()), "lr": lr})
    return groups


def train_step_ref(model, opt, frames, long_feature, labels, masks=None, weight=None):
    opt.zero_grad()
    out = model(frames, long_feature, masks=masks)
    loss = ce_sum_ref(out, labels, weight)
    loss.backward()
    opt.step()
    return out.detach(), loss.detach()


def trunk_gmacs_per_frame():
    """Algorithmic MACs of the ResNet-50 trunk at 224x224 (fwd), for the roofline."""
    total = 0
    h = 112
    total += h * h * 64 * 3 * 49
    h = 56
    cin = 64
    for planes, blocks, stride in ((64, 3, 1), (128, 4, 2), (256, 6, 2), (512, 3, 2)):
        for b in range(blocks):
            s = stride if b == 0 else 1
            ho = h // s
            total += h * h * cin * planes            # 1x1 (at input res)
            total += ho * ho * planes * planes * 9   # 3x3 (stride here)
            total += ho * ho * planes * planes * 4   # 1x1 expand
            if b == 0:
                total += ho * ho * cin * planes * 4  # downsample
            cin = planes * 4
            h = ho
    return total / 1e9
