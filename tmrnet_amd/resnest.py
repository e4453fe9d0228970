"""ResNeSt-50 frame encoder (`share` of the ResNeSt TMRNet) on libtmr kernels.

Drop-in for the `share` Sequential of code/Training TMRNet/train_non-local_mutiConv_resnest.py:210-220
built from the third-party ``resnest50()`` (radix 2, cardinality 1, deep stem of width 32,
avg_down shortcut, avd pooling on strided blocks): same child names and state_dict keys
(``share.conv1.0.weight``, ``share.layer1.0.conv2.conv.weight``, ``...conv2.fc1.bias``, ...),
25,434,240 parameters.

Train mode (fp32 math, or bf16 math under the bf16-activation contract): the whole trunk is ONE
autograd node, `ResNeStTrunkFn`, built on trunk.py's conv-unit engine (the ResNet-50 TrunkFn's):
  * every conv runs on the LDS-DMA implicit-GEMM engine with its BatchNorm statistics from the
    epilogue -- the radix-2 grouped 3x3 included (tmr_conv_desc.groups: one launch per group on
    channel slices, one BN-partial row over all channels);
  * bf16 math stores every activation as bf16 (the C5 contract of trunk.py ACT16: conv outputs
    rounded by their epilogue, BN(+residual)(+ReLU) outputs computed in fp32 and rounded);
  * bn0 + ReLU of SplAtConv2d are applied on load by the split-attention kernels
    (tmr_splat_*_bn): the post-BN tensor is never written, and its backward -- weighted-sum
    gradient, ReLU mask and the bn0 BatchNorm backward -- is one reduction pass and one apply pass
    that writes the grouped conv's dy;
  * residual / branch gradients accumulate in the dgrad epilogues (beta = 1), each dgrad fused with
    the backward of the BatchNorm that produced its input (conv2's with bn1, conv1's with the
    previous block's bn3), so no PyTorch kernel sums gradients.
Eval mode (and inference without grad) keeps the per-stage nodes below.

Per-stage nodes (eval / legacy path), activations NHWC:
  * ConvBNActFn   -- (grouped) implicit-GEMM conv + BatchNorm (batch stats) + residual + ReLU
  * SplAtFn       -- split attention: radix-summed GAP, fc1 -> BN -> ReLU -> fc2 GEMMs,
                     r-softmax and weighted sum (and their backward)
  * AvgPoolFn / MaxPoolFn / GlobalPoolFn
Grouped convolutions run one GEMM launch per group on channel slices (pixel strides in
tmr_conv_desc), so no channel shuffles are materialised.

bf16 math in train mode (config C4): every conv but the 4-channel stem reads bf16 operands from
HBM -- a bf16 copy of its input (written by the producing BN pass next to the fp32 tensor the
residual / split attention / pools use, or cast once for split-attention and pool outputs), KRSC
and transposed CRSK bf16 weights, bf16 dy -- and therefore runs on the LDS-DMA engine
(gemm16_kernel.h).  The contract is unchanged (the bf16 convs round exactly those operands).
"""
import math

import torch
import torch.nn as nn

from . import ops
from ._lib import call, stream_ptr


def _bn_train_or_eval(y, bn, training):
    k = y.shape[-1]
    if training:
        mean, inv, scale, shift = ops.bn_fwd_train(y.view(-1, k), bn.weight.detach(), bn.bias.detach(),
                                                   bn.running_mean, bn.running_var, bn.momentum, bn.eps)
        bn.num_batches_tracked.add_(1)
        return mean, inv, scale, shift
    scale, shift = ops.bn_eval_params(bn.weight.detach(), bn.bias.detach(), bn.running_mean,
                                      bn.running_var, bn.eps)
    return None, None, scale, shift




class ConvBNActFn(torch.autograd.Function):
    """x (fp32, autograd) and x16 (its bf16 copy or None, not differentiable) -> (z, z16): z16 is
    the bf16 copy of z written by the same BN pass when the bf16 operand path is on (else None)."""

    @staticmethod
    def forward(ctx, x, x16, w, gamma, beta, residual, bn, stride, pad, groups, relu, c_real, math):
        x = x.contiguous()
        n, h, wd, _ = x.shape
        cs = (x16 if x16 is not None else x).shape[-1]   # stored channels of the conv operand
        k, cg, r, s = w.shape
        kg = k // groups
        cgs = cs // groups                       # stored channels per group
        training = bn.training
        f16 = x16 is not None
        wks = [ops.weight_to_krsc(w.detach()[g * kg:(g + 1) * kg].contiguous(), cpad=cgs, bf16=f16)
               for g in range(groups)]
        xc = x16 if f16 else x                   # the conv operand
        if groups == 1 and training:
            y, stats, nparts = ops.conv_fwd_bnstats(xc, wks[0], stride, pad, c_real=c_real,
                                                    math=math)
            mean, inv, scale, shift = ops.bn_finalize(stats, nparts, gamma.detach(), beta.detach(),
                                                      bn.running_mean, bn.running_var, bn.momentum,
                                                      bn.eps)
            bn.num_batches_tracked.add_(1)
        else:
            ho = (h + 2 * pad - r) // stride + 1
            wo = (wd + 2 * pad - s) // stride + 1
            y = torch.empty((n, ho, wo, k), dtype=x.dtype, device=x.device)
            for g in range(groups):
                ops.conv_fwd(xc[..., g * cgs:(g + 1) * cgs], wks[g], stride, pad,
                             out=y[..., g * kg:(g + 1) * kg], c_real=min(cg, c_real), math=math)
            mean, inv, scale, shift = _bn_train_or_eval(y, bn, training)
        res = residual.contiguous() if residual is not None else None
        z16 = None
        if f16 and training:   # z in fp32 (residual, split attention, pools) + its bf16 copy
            z, z16 = ops.bn_apply_dual(y, scale, shift, res, relu)
            ctx.mark_non_differentiable(z16)
        else:
            z = ops.bn_apply(y, scale, shift, res, relu)
        # the dgrad view of the bf16 operand path reads transposed bf16 weights
        wts = ([ops.weight_to_crsk(w.detach()[g * kg:(g + 1) * kg].contiguous())
                for g in range(groups)] if f16 and training and cgs == cg else [])
        # without a residual the backward recomputes the ReLU mask from y and scale/shift
        ctx.save_for_backward(xc, y, z if residual is not None else None, scale, shift, mean, inv,
                              gamma, *wks, *wts)
        ctx.cfg = (stride, pad, groups, relu, c_real, residual is not None, r, s, math, f16,
                   len(wts))
        return z, z16

    @staticmethod
    def backward(ctx, dz, _dz16=None):
        x, y, z, scale, shift, mean, inv, gamma, *ws = ctx.saved_tensors
        stride, pad, groups, relu, c_real, has_res, r, s, math, f16, nwt = ctx.cfg
        wks, wts = ws[:groups], ws[groups:]
        if mean is None:
            raise RuntimeError("backward through eval-mode BatchNorm is not supported")
        dz = dz.contiguous()
        # dy only feeds this conv's dgrad / wgrad: bf16 on the bf16 operand path
        dy, dres, dg, db = ops.bn_bwd(dz, y, z, mean, inv, gamma.detach(), relu, want_dres=has_res,
                                      scale=scale, shift=shift, bf16=f16)
        n, h, wd, cs = x.shape
        k = y.shape[-1]
        kg, cgs = k // groups, cs // groups
        creal_g = min(c_real, cgs)
        dw = torch.empty((k, creal_g, r, s), dtype=torch.float32, device=x.device)
        dx = torch.empty(x.shape, dtype=torch.float32, device=x.device) \
            if ctx.needs_input_grad[0] else None
        for g in range(groups):
            dyg = dy[..., g * kg:(g + 1) * kg]
            ops.conv_wgrad(x[..., g * cgs:(g + 1) * cgs], dyg, r, s, stride, pad, c_real=creal_g,
                           out=dw[g * kg:(g + 1) * kg], math=math)
            if dx is not None:
                if nwt:
                    ops.conv_dgrad(dyg, wts[g], (h, wd), stride, pad,
                                   out=dx[..., g * cgs:(g + 1) * cgs], math=math, wt=True)
                else:
                    ops.conv_dgrad(dyg, wks[g], (h, wd), stride, pad,
                                   out=dx[..., g * cgs:(g + 1) * cgs], math=math)
        return dx, None, dw, dg, db, dres, None, None, None, None, None, None, None


class SplAtFn(torch.autograd.Function):
    """Split attention after the grouped conv + bn0 + ReLU: x2 (N,H,W,2C) -> (N,H,W,C).

    Train mode runs fc1 on GAP rows centered over the batch (tmr_center_cols): BatchNorm
    removes any per-channel constant exactly, so BN(W1 gap + b1) = BN(W1 (gap - c)), while the
    fp32 error then scales with the batch spread of the GAP rows (~1% of their magnitude)
    instead of the magnitude.  The running mean gets the removed W1 c + b1 back (tmr_axpy).
    The same identity makes d b1 exactly zero (sum_n dh1 = 0 under batch-stat BN)."""

    @staticmethod
    def forward(ctx, x2, w1, b1, g1, bt1, w2, b2, bn1):
        x2 = x2.contiguous()
        n, h, w, c2 = x2.shape
        C = c2 // 2
        hw = h * w
        gap = torch.empty((n, C), dtype=x2.dtype, device=x2.device)
        call("tmr_splat_gap", x2, gap, n, hw, C, stream_ptr())
        inter = w1.shape[0]
        w1d = w1.detach().reshape(inter, C)
        w2d = w2.detach().reshape(c2, inter)
        training = bn1.training
        if training:
            center = torch.empty((1, C), dtype=x2.dtype, device=x2.device)
            gap_c = torch.empty_like(gap)
            call("tmr_center_cols", gap, n, C, center, gap_c, stream_ptr())
            h1 = ops.gemm_nt(gap_c, w1d)
            mean, inv, scale, shift = _bn_train_or_eval(h1, bn1, True)
            shift_back = ops.gemm_nt(center, w1d, bias=b1.detach())      # W1 c + b1
            call("tmr_axpy", inter, float(bn1.momentum), shift_back, bn1.running_mean,
                 stream_ptr())
            gap = gap_c
        else:
            h1 = ops.gemm_nt(gap, w1d, bias=b1.detach())
            mean, inv, scale, shift = _bn_train_or_eval(h1, bn1, False)
        a1 = ops.bn_apply(h1, scale, shift, None, True)
        zl = ops.gemm_nt(a1, w2d, bias=b2.detach())
        att = torch.empty((n, c2), dtype=x2.dtype, device=x2.device)
        out = torch.empty((n, h, w, C), dtype=x2.dtype, device=x2.device)
        call("tmr_splat_combine", x2, zl, att, out, n, hw, C, stream_ptr())
        ctx.save_for_backward(x2, gap, h1, a1, att, mean, inv, w1, w2, g1)
        return out

    @staticmethod
    def backward(ctx, dout):
        x2, gap, h1, a1, att, mean, inv, w1, w2, g1 = ctx.saved_tensors
        if mean is None:
            raise RuntimeError("backward through eval-mode BatchNorm is not supported")
        dout = dout.contiguous()
        n, h, w, c2 = x2.shape
        C = c2 // 2
        hw = h * w
        inter = w1.shape[0]
        dzl = torch.empty((n, c2), dtype=x2.dtype, device=x2.device)
        call("tmr_splat_bwd", dout, x2, att, dzl, n, hw, C, stream_ptr())
        dw2 = ops.gemm_tn(dzl, a1).view_as(w2)
        db2 = ops.col_sum(dzl, n, c2, c2)
        da1 = ops.gemm_nn(dzl, w2.detach().reshape(c2, inter))
        dh1, _, dg1, dbt1 = ops.bn_bwd(da1, h1, a1, mean, inv, g1.detach(), True)
        dw1 = ops.gemm_tn(dh1, gap).view_as(w1)          # gap is centered (see class doc)
        db1 = torch.zeros((inter,), dtype=x2.dtype, device=x2.device)
        dgap = ops.gemm_nn(dh1, w1.detach().reshape(inter, C))
        dx2 = torch.empty_like(x2)
        call("tmr_splat_bwd_apply", dout, att, dgap, dx2, n, hw, C, stream_ptr())
        return dx2, dw1, db1, dg1, dbt1, dw2, db2, None


def _pool_out(h, k, s, p, ceil):
    if not ceil:
        return (h + 2 * p - k) // s + 1
    o = -(-(h + 2 * p - k) // s) + 1
    if (o - 1) * s >= h + p:   # last window must start inside the input (PyTorch rule)
        o -= 1
    return o


class AvgPoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k, s, p, incl, ceil):
        x = x.contiguous()
        n, h, w, c = x.shape
        ho, wo = _pool_out(h, k, s, p, ceil), _pool_out(w, k, s, p, ceil)
        y = torch.empty((n, ho, wo, c), dtype=x.dtype, device=x.device)
        call("tmr_avgpool2d_fwd", x, y, n, h, w, c, ho, wo, k, s, p, int(incl), stream_ptr())
        ctx.cfg = (n, h, w, c, ho, wo, k, s, p, incl)
        return y

    @staticmethod
    def backward(ctx, dy):
        n, h, w, c, ho, wo, k, s, p, incl = ctx.cfg
        dx = torch.empty((n, h, w, c), dtype=dy.dtype, device=dy.device)
        call("tmr_avgpool2d_bwd", dy.contiguous(), dx, n, h, w, c, ho, wo, k, s, p, int(incl),
             stream_ptr())
        return dx, None, None, None, None, None


class MaxPoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        y, am = ops.maxpool_fwd(x.contiguous())
        ctx.save_for_backward(am)
        ctx.hw = (x.shape[1], x.shape[2])
        return y

    @staticmethod
    def backward(ctx, dy):
        (am,) = ctx.saved_tensors
        return ops.maxpool_bwd(dy.contiguous(), am, ctx.hw)


class GlobalPoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        ctx.hw = (x.shape[1], x.shape[2])
        return ops.avgpool_fwd(x.contiguous())

    @staticmethod
    def backward(ctx, dy):
        return ops.avgpool_bwd(dy.contiguous(), ctx.hw)


class ResNeStTrunkFn(torch.autograd.Function):
    """Whole ResNeSt-50 trunk, train mode, as one autograd node: x NHWC4 (F,224,224,4) -> (F,2048).

    Forward per BottleneckS (train_non-local_mutiConv_resnest.py:210-220 -> resnest50()):
    conv1+bn1+relu -> grouped conv + bn0 (deferred) -> split attention (fc1 -> bn1 -> relu -> fc2
    -> r-softmax -> weighted sum) -> [avd AvgPool2d(3, s, 1)] -> conv3 + bn3 + [avg_down pool ->
    conv -> bn] + relu.  The backward mirrors trunk.TrunkFn's."""

    @staticmethod
    def forward(ctx, x4, share, keep, *params):
        # every conv weight layout of the step in one launch (ops.layout_session)
        with ops.layout_session(share, ("resnest50", share.training, bool(keep),
                                 share.precision)):
            return ResNeStTrunkFn._forward(ctx, x4, share, keep, params)

    @staticmethod
    def _forward(ctx, x4, share, keep, params):
        from .trunk import _conv_bn, _act16
        mt = share.precision
        a16 = _act16(mt)
        nbt = []
        stem = []
        c = share.conv1
        # the stem input: under bf16 activations the NHWC4 fp32 frames themselves for the direct
        # 3x3/2 stem conv (direct3.hip: rounded to bf16 as it is staged), or an NHWC8 bf16 copy
        # for the LDS-DMA engine (ops.engine_only, tests: its 8-channel pieces)
        xs = ops.nhwc4_to_bf16x8(x4) if (a16 and ops.engine_forced()) else x4
        z = _conv_bn(xs, c[0], c[1], 2, 1, True, True, recs=stem, math=mt, nbt=nbt)
        z = _conv_bn(z, c[3], c[4], 1, 1, True, True, recs=stem, math=mt, nbt=nbt)
        # share.bn1 + relu applied inside the maxpool (its backward recomputes the mask from y)
        y0, sc0, sh0 = _conv_bn(z, c[6], share.bn1, 1, 1, True, True, recs=stem, math=mt,
                                defer=True, nbt=nbt)
        h, am = ops.maxpool_fwd_bn(y0, sc0, sh0)
        stem_hw = (y0.shape[1], y0.shape[2])
        blocks = []
        for layer in (share.layer1, share.layer2, share.layer3, share.layer4):
            for blk in layer:
                rec = {"blk": blk, "in_hw": (h.shape[1], h.shape[2])}
                r1, r2, r3, rd = [], [], [], []
                z1 = _conv_bn(h, blk.conv1, blk.bn1, 1, 0, True, True, recs=r1, math=mt, nbt=nbt)
                sp = blk.conv2
                y2, sc2, sh2 = _conv_bn(z1, sp.conv, sp.bn0, sp.stride, 1, True, True, recs=r2,
                                        math=mt, defer=True, nbt=nbt, groups=sp.radix)
                out, spl = _splat_fwd(sp, y2, sc2, sh2, nbt)
                if blk.avd:
                    rec["avd_hw"] = (out.shape[1], out.shape[2])
                    out = ops.avgpool2d_fwd(out, 3, blk.avd_stride, 1, True, False)
                if blk.downsample is not None:
                    pool, dconv, dbn = blk.downsample[0], blk.downsample[1], blk.downsample[2]
                    xr = h
                    if pool.kernel_size != 1:
                        rec["pool"] = (pool.kernel_size, pool.stride)
                        xr = ops.avgpool2d_fwd(h, pool.kernel_size, pool.stride, 0, False, True)
                    idn = _conv_bn(xr, dconv, dbn, 1, 0, False, True, recs=rd, math=mt, defer=True,
                                   nbt=nbt)
                    h = _conv_bn(out, blk.conv3, blk.bn3, 1, 0, True, True, branch=idn, recs=r3,
                                 math=mt, nbt=nbt)
                else:
                    h = _conv_bn(out, blk.conv3, blk.bn3, 1, 0, True, True, residual=h, recs=r3,
                                 math=mt, nbt=nbt)
                rec.update(r1=r1[0], r2=r2[0], r3=r3[0], rd=rd[0] if rd else None, spl=spl)
                blocks.append(rec)
        feat = ops.avgpool_fwd(h)
        ops.counters_add_one(nbt)
        ctx.keep = keep
        if keep:
            ctx.share, ctx.params = share, params
            ctx.stem, ctx.pool, ctx.blocks = stem, (am, stem_hw), blocks
            ctx.last_hw = (h.shape[1], h.shape[2])
        return feat

    @staticmethod
    def backward(ctx, dfeat):
        from . import trunk
        from .trunk import _conv_bn_bwd, get_grad_ready
        if not ctx.keep:
            raise RuntimeError("trunk backward needs train mode and a forward with grad enabled")
        grads = {}
        g = ops.avgpool_bwd(dfeat.contiguous(), ctx.last_hw)   # grad at the last block output
        blocks = ctx.blocks
        pending = None     # BN-backward partials of g from the fused dgrad that produced it
        ready = get_grad_ready(ctx.share)
        while blocks:
            rec = blocks.pop()
            blk = rec["blk"]
            prev3 = blocks[-1]["r3"] if blocks else None
            # bn3 (+ReLU) backward; g (owned) becomes the masked gradient = the residual branch's
            r3, rd, dyd = rec["r3"], rec["rd"], None
            if rd is not None and pending is not None and trunk._ds_dual(g, r3, rd):
                # bn3 and the downsample BN share g: one apply pass (trunk.DS_DUAL)
                dy3, dg3, db3, dyd, dgd, dbd = ops.bn_bwd_parts_ds(
                    g, r3["y"], pending[0], pending[1], r3["mean"], r3["inv"],
                    r3["bn"].weight.detach(), rd["y"], rd["mean"], rd["inv"],
                    rd["bn"].weight.detach())
                grads[r3["bn"].weight], grads[r3["bn"].bias] = dg3, db3
                grads[rd["bn"].weight], grads[rd["bn"].bias] = dgd, dbd
                dout, _, _ = _conv_bn_bwd(r3, None, grads, dy=dy3)
                dres = g
                del dy3
            else:
                dout, dres, _ = _conv_bn_bwd(r3, g, grads, want_dres=True, dres_inplace=True,
                                             parts=pending)
            if blk.avd:
                dout = ops.avgpool2d_bwd(dout, rec["avd_hw"], 3, blk.avd_stride, 1, True)
            # split attention + bn0 backward -> dy of the grouped conv
            r2 = rec["r2"]
            dy2 = _splat_bwd(blk.conv2, rec["spl"], r2, dout, grads)
            del dout
            # (relu(bn1)'s gradient stored bf16 by the grouped dgrad: trunk.G16, round 4)
            dz1, _, fz1 = _conv_bn_bwd(r2, None, grads, dy=dy2, fuse_prev=rec["r1"], g16=True)
            del dy2
            if rd is not None:
                if dyd is not None:
                    dxr, _, _ = _conv_bn_bwd(rd, None, grads, dy=dyd)
                    del dyd
                else:
                    dxr, _, _ = _conv_bn_bwd(rd, dres, grads)
                if "pool" in rec:
                    k, st = rec["pool"]
                    dxr = ops.avgpool2d_bwd(dxr, rec["in_hw"], k, st, 0, False)
                # (trunk.R16: the sum is returned as a new bf16 tensor when dxr is fp32)
                dx, _, pending = _conv_bn_bwd(rec["r1"], dz1, grads, parts=fz1, dx_out=dxr,
                                              dx_beta=1.0, fuse_prev=prev3, r16=True)
            else:
                dx, _, pending = _conv_bn_bwd(rec["r1"], dz1, grads, parts=fz1, dx_out=dres,
                                              dx_beta=1.0, fuse_prev=prev3, r16=True)
            del dz1, dres, rec
            g = dx
            if ready is not None:   # this block's parameter grads are final: start their exchange
                ready([(p, grads[p]) for p in blk.parameters() if p in grads])
        am, stem_hw = ctx.pool
        st = ctx.stem
        d2, _, f2 = _conv_bn_bwd(st[2], None, grads, pool=(g, am), fuse_prev=st[1])
        d1, _, f1 = _conv_bn_bwd(st[1], d2, grads, parts=f2, fuse_prev=st[0])
        _conv_bn_bwd(st[0], d1, grads, parts=f1, need_dx=False)
        out = [grads.get(p) for p in ctx.params]
        ctx.blocks = ctx.stem = None
        return (None, None, None) + tuple(out)


def _splat_fwd(sp, y2, sc, sh, nbt):
    """Split attention of SplAtConv2d on the grouped conv's pre-BN output y2 (bn0 + ReLU applied
    on load); fc1 -> BatchNorm runs on batch-centered GAP rows (see SplAtFn).  -> (out, saved)."""
    n = y2.shape[0]
    C = y2.shape[-1] // 2
    inter = sp.fc1.weight.shape[0]
    w1 = sp.fc1.weight.detach().reshape(inter, C)
    w2 = sp.fc2.weight.detach().reshape(2 * C, inter)
    gap = ops.splat_gap_bn(y2, sc, sh)
    center = torch.empty((1, C), dtype=gap.dtype, device=gap.device)
    gap_c = torch.empty_like(gap)
    call("tmr_center_cols", gap, n, C, center, gap_c, stream_ptr())
    h1 = ops.gemm_nt(gap_c, w1)
    bn1 = sp.bn1
    mean, inv, scale, shift = ops.bn_fwd_train(h1, bn1.weight.detach(), bn1.bias.detach(),
                                               bn1.running_mean, bn1.running_var, bn1.momentum,
                                               bn1.eps)
    nbt.append(bn1.num_batches_tracked)
    shift_back = ops.gemm_nt(center, w1, bias=sp.fc1.bias.detach())      # W1 c + b1
    call("tmr_axpy", inter, float(bn1.momentum), shift_back, bn1.running_mean, stream_ptr())
    a1 = ops.bn_apply(h1, scale, shift, None, True)
    zl = ops.gemm_nt(a1, w2, bias=sp.fc2.bias.detach())
    att = ops.splat_att(zl)
    out = ops.splat_combine_bn(y2, sc, sh, att)
    return out, {"gap": gap_c, "h1": h1, "a1": a1, "att": att, "mean": mean, "inv": inv}


def _splat_bwd(sp, spl, r2, dout, grads):
    """Backward of the split attention and of bn0 + ReLU -> dy2 (the grouped conv's output
    gradient, dtype of y2); writes the fc1 / bn1 / fc2 / bn0 parameter gradients."""
    y2 = r2["y"]
    n, hh, ww, c2 = y2.shape
    C = c2 // 2
    inter = sp.fc1.weight.shape[0]
    att = spl["att"]
    dout = dout.contiguous()
    dzl, sums = ops.splat_bwd_reduce_bn(dout, y2, r2["scale"], r2["shift"], r2["mean"], att)
    grads[sp.fc2.weight] = ops.gemm_tn(dzl, spl["a1"]).view_as(sp.fc2.weight)
    grads[sp.fc2.bias] = ops.col_sum(dzl, n, c2, c2)
    da1 = ops.gemm_nn(dzl, sp.fc2.weight.detach().reshape(c2, inter))
    dh1, _, dg1, dbt1 = ops.bn_bwd(da1, spl["h1"], spl["a1"], spl["mean"], spl["inv"],
                                   sp.bn1.weight.detach(), True)
    grads[sp.bn1.weight], grads[sp.bn1.bias] = dg1, dbt1
    grads[sp.fc1.weight] = ops.gemm_tn(dh1, spl["gap"]).view_as(sp.fc1.weight)   # centered gap
    grads[sp.fc1.bias] = ops.zeros((inter,), dh1)   # exactly 0 under batch-stat BN (SplAtFn)
    dgap = ops.gemm_nn(dh1, sp.fc1.weight.detach().reshape(inter, C))
    coef, dg0, db0 = ops.splat_bn0_coefs(att, dgap, sums, r2["mean"], r2["inv"],
                                         sp.bn0.weight.detach(), hh * ww)
    grads[sp.bn0.weight], grads[sp.bn0.bias] = dg0, db0
    return ops.splat_bwd_apply_bn(dout, y2, r2["scale"], r2["shift"], r2["mean"], att, dgap, coef)


def _trunk_node_ok(share):
    """The whole-trunk node covers fp32 math and bf16 math under the bf16-activation contract."""
    from .trunk import _act16, FOLD_BN
    return not FOLD_BN and (share.precision == "fp32" or _act16(share.precision))


def conv_bn_act(x, conv, bn, stride, pad, relu, groups=1, residual=None, c_real=None,
                math="fp32"):
    """conv -> BN -> (+residual) -> (ReLU).  On the bf16 operand path (bf16 math, train mode) the
    conv reads x's bf16 copy: the one its producer attached (`_tmr_bf16`), else a cast; the
    4-channel stem input as an NHWC8 bf16 copy (tmr_nhwc4_to_bf16x8)."""
    x16 = None
    if math == "bf16" and bn.training and x.shape[-1] % 8 == 0:
        x16 = getattr(x, "_tmr_bf16", None)
        if x16 is None:
            x16 = ops.to_bf16(x.contiguous())
    elif math == "bf16" and bn.training and x.shape[-1] == 4 and groups == 1:
        x16 = ops.nhwc4_to_bf16x8(x.contiguous())
    z, z16 = ConvBNActFn.apply(x, x16, conv.weight, bn.weight, bn.bias, residual, bn, stride, pad,
                               groups, relu,
                               c_real if c_real is not None else conv.weight.shape[1] * groups, math)
    if z16 is not None:
        z._tmr_bf16 = z16
    return z


# ------------------------------------------------------------------ modules
class SplAtConv2d(nn.Module):
    """resnest SplAtConv2d(radix=2, groups=1, reduction_factor=4): parameter container."""

    def __init__(self, in_channels, channels, stride=1, radix=2):
        super().__init__()
        inter = max(in_channels * radix // 4, 32)
        self.radix, self.channels, self.stride = radix, channels, stride
        self.math = "fp32"   # set by ResNeSt50Share(precision=...)
        self.conv = nn.Conv2d(in_channels, channels * radix, 3, stride, 1, groups=radix, bias=False)
        self.bn0 = nn.BatchNorm2d(channels * radix)
        self.relu = nn.ReLU(inplace=True)
        self.fc1 = nn.Conv2d(channels, inter, 1, groups=1)
        self.bn1 = nn.BatchNorm2d(inter)
        self.fc2 = nn.Conv2d(inter, channels * radix, 1, groups=1)

    def forward(self, x):
        x2 = conv_bn_act(x, self.conv, self.bn0, self.stride, 1, True, groups=self.radix,
                         math=self.math)
        return SplAtFn.apply(x2, self.fc1.weight, self.fc1.bias, self.bn1.weight, self.bn1.bias,
                             self.fc2.weight, self.fc2.bias, self.bn1)


class BottleneckS(nn.Module):
    expansion = 4

    def __init__(self, inplanes, planes, stride=1, downsample=None, is_first=False):
        super().__init__()
        self.conv1 = nn.Conv2d(inplanes, planes, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.avd = stride > 1 or is_first
        self.avd_stride = stride
        if self.avd:
            self.avd_layer = nn.AvgPool2d(3, stride, padding=1)
            stride = 1
        self.conv2 = SplAtConv2d(planes, planes, stride=stride)
        self.conv3 = nn.Conv2d(planes, planes * 4, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(planes * 4)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample
        self.math = "fp32"

    def forward(self, x):
        mt = self.math
        out = conv_bn_act(x, self.conv1, self.bn1, 1, 0, True, math=mt)
        out = self.conv2(out)
        if self.avd:
            out = AvgPoolFn.apply(out, 3, self.avd_stride, 1, True, False)
        res = x
        if self.downsample is not None:
            pool, conv, bn = self.downsample[0], self.downsample[1], self.downsample[2]
            if pool.kernel_size != 1:
                res = AvgPoolFn.apply(x, pool.kernel_size, pool.stride, 0, False, True)
            res = conv_bn_act(res, conv, bn, 1, 0, False, math=mt)
        return conv_bn_act(out, self.conv3, self.bn3, 1, 0, True, residual=res, math=mt)


def _make_layer(inplanes, planes, blocks, stride):
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
    def forward(self, x):  # unused (the engine pools NHWC); kept for the module tree
        raise RuntimeError("use ResNeSt50Share.forward")


class ResNeSt50Share(nn.Sequential):
    def __init__(self, precision="fp32"):
        super().__init__()
        self.precision = precision
        self.add_module("conv1", nn.Sequential(
            nn.Conv2d(3, 32, 3, 2, 1, bias=False), nn.BatchNorm2d(32), nn.ReLU(inplace=True),
            nn.Conv2d(32, 32, 3, 1, 1, bias=False), nn.BatchNorm2d(32), nn.ReLU(inplace=True),
            nn.Conv2d(32, 64, 3, 1, 1, bias=False)))
        self.add_module("bn1", nn.BatchNorm2d(64))
        self.add_module("relu", nn.ReLU(inplace=True))
        self.add_module("maxpool", nn.MaxPool2d(3, 2, 1))
        self.add_module("layer1", _make_layer(64, 64, 3, 1))
        self.add_module("layer2", _make_layer(256, 128, 4, 2))
        self.add_module("layer3", _make_layer(512, 256, 6, 2))
        self.add_module("layer4", _make_layer(1024, 512, 3, 2))
        self.add_module("avgpool", GlobalAvgPool2d())
        for m in self.modules():   # resnest ResNet.__init__ init
            if isinstance(m, nn.Conv2d):
                nk = m.kernel_size[0] * m.kernel_size[1] * m.out_channels
                m.weight.data.normal_(0, math.sqrt(2.0 / nk))
            elif isinstance(m, nn.BatchNorm2d):
                m.weight.data.fill_(1)
                m.bias.data.zero_()
        for m in self.modules():
            if isinstance(m, (BottleneckS, SplAtConv2d)):
                m.math = precision

    def features_nhwc4(self, x4):
        if self.training and _trunk_node_ok(self):
            params = list(self.parameters())
            # grad mode is off inside autograd.Function.forward: decide here whether to save
            keep = torch.is_grad_enabled() and any(p.requires_grad for p in params)
            return ResNeStTrunkFn.apply(x4, self, keep, *params)
        c, mt = self.conv1, self.precision
        h = conv_bn_act(x4, c[0], c[1], 2, 1, True, c_real=3, math=mt)
        h = conv_bn_act(h, c[3], c[4], 1, 1, True, math=mt)
        h = conv_bn_act(h, c[6], self.bn1, 1, 1, True, math=mt)
        h = MaxPoolFn.apply(h)
        for layer in (self.layer1, self.layer2, self.layer3, self.layer4):
            for blk in layer:
                h = blk(h)
        return GlobalPoolFn.apply(h)

    def forward(self, x):
        x = x.reshape(-1, 3, x.shape[-2], x.shape[-1]).contiguous()
        return self.features_nhwc4(ops.nchw_to_nhwc(x, cpad=4))
