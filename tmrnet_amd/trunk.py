"""ResNet-50 frame encoder (`share`) on libtmr's NHWC implicit-GEMM kernels.

Drop-in for the `share` nn.Sequential of the reference's inline TMRNet model
(code/Training TMRNet/train_only_non-local_pretrained.py:204-214, built from
torchvision resnet50): same child names (conv1, bn1, relu, maxpool,
layer1..4, avgpool), same Bottleneck sub-module names and therefore identical
``state_dict`` keys ("share.layer1.0.conv1.weight", "share.bn1.running_mean",
...).  nn.Conv2d / nn.BatchNorm2d modules are kept as parameter/buffer
containers only (their torch forward is never called); the whole trunk runs
as ONE autograd node (`TrunkFn`) that keeps activations NHWC in HBM and drives
conv -> BN(batch stats) -> ReLU(+residual) on the HIP kernels, with the
backward pass (BN backward, dgrad, wgrad) in reverse layer order.

BN semantics follow nn.BatchNorm2d in train mode: batch mean / biased variance
for normalisation, running stats updated with momentum and the unbiased
variance, num_batches_tracked += 1; eval mode uses running stats.
"""
import os
import weakref

import torch
import torch.nn as nn

from . import ops


class Bottleneck(nn.Module):
    """torchvision v1.5 Bottleneck (stride on the 3x3) as a parameter container."""
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


def _make_layer(inplanes, planes, blocks, stride):
    downsample = None
    if stride != 1 or inplanes != planes * 4:
        downsample = nn.Sequential(nn.Conv2d(inplanes, planes * 4, 1, stride=stride, bias=False),
                                   nn.BatchNorm2d(planes * 4))
    layers = [Bottleneck(inplanes, planes, stride, downsample)]
    for _ in range(1, blocks):
        layers.append(Bottleneck(planes * 4, planes))
    return nn.Sequential(*layers)


# --------------------------------------------------------------------- engine
# share module -> callable(pairs) told each block's final gradients during the backward
# (ddp.GradAllReduce registers itself here).  A weak side table rather than a module attribute,
# so deepcopy / torch.save of the model never see the reducer or its process group.
_GRAD_READY = weakref.WeakKeyDictionary()


def set_grad_ready(share, fn):
    """Register (fn) or clear (None) the per-block gradient hook of a trunk module."""
    if fn is None:
        _GRAD_READY.pop(share, None)
    else:
        _GRAD_READY[share] = fn


def get_grad_ready(share):
    return _GRAD_READY.get(share, getattr(share, "grad_ready", None))

def _bn_momentum(bn):
    if bn.momentum is None:
        raise NotImplementedError("BatchNorm2d(momentum=None) (cumulative average) is not supported")
    return bn.momentum


# Train-mode BatchNorm folding (TMR_FOLD_BN=1; off by default): the BN+ReLU outputs of each
# Bottleneck's first two units are never written -- the next conv reads the pre-BN y through an
# X-operand prologue (tmr_conv_prologue) in its forward and wgrad loaders -- and no BatchNorm
# backward writes dy: the conv's dgrad and wgrad read the masked gradient g and y through a
# dY-operand prologue with per-channel coefficients.  Bit-identical to the explicit passes
# (tests/test_kernels_gpu.py::test_bn_fold_bit_identical), but measured slower on MI355X: the
# prologue costs the MFMA-bound fp32 GEMMs more than the HBM-bound passes it removes (~17 ms).
# Register-staged engine (round 2): wgrad +21 ms, dgrad +12 ms, fwd +6 ms per step, C2 210 vs 181
# ms/step (profiles/r2/convbench_fold/).  LDS-DMA engine (round 4, gemm16_kernel PRO: each lane
# transforms its landed pieces in LDS before the barrier that publishes the k-tile): fwd +3.0,
# wgrad +12.7, dgrad +21.0 ms per step, C2 193.3 vs 173.9 ms/step, 3312 vs 3680 frames/s, same
# box (profiles/r4/fold_ab/): the transform sits between the LDS-DMA landing and the barrier with
# every MFMA idle, and on the narrow tiles (256x64: 8 pieces per lane per k-tile) it triples the
# LDS traffic; the dgrads also read y next to g (twice the A-operand bytes).  Retired to an A/B
# build: the prologue entry points (include/tmr_prologue.h) exist only in `make PROLOGUES=1`'s
# tmrnet_amd/libtmr_pro.so (run with TMR_LIB_PATH pointing at it); the default library rejects
# TMR_FOLD_BN=1 at the first conv.
FOLD_BN = os.environ.get("TMR_FOLD_BN", "0") == "1"
# The bf16 form (round 5, same A/B build, TMR_FOLD16=1): under the bf16-activation step the relu(bn)
# outputs of each Bottleneck's bn1 / bn2 are never written -- conv2 / conv3 read the bf16 pre-BN y
# through the bf16 X-operand prologue of the LDS-DMA engine (relu(fmaf(y, scale, shift)) rounded
# RNE: bn_apply8_a16_k's arithmetic, so bit-identical), forward and wgrad views.  Not for an input
# the direct 3x3 kernels read (direct3.hip: ResNet-50 layer1's 56x56 64 -> 64 conv2).
FOLD16 = os.environ.get("TMR_FOLD16", "0") == "1"
# ... and its dY half (round 5, same A/B build, TMR_FOLD16_DY=1): no BatchNorm backward writes dy --
# the conv's dgrad and wgrad read the bf16 masked gradient g and the bf16 y through the bf16
# dY-operand prologue (fmaf(A, g, fmaf(B, y, C)) rounded RNE: bn_bwd_apply8_a16's arithmetic, so
# bit-identical), for every unit whose g is stored bf16 (bn1 / bn2 under G16, bn3 / downsample
# under R16: all but the last block's bn3) and whose conv is not a direct 3x3 (direct3.hip).
FOLD16DY = os.environ.get("TMR_FOLD16_DY", "0") == "1"


def _direct3_conv(rec):
    """This unit's conv runs on the direct 3x3 kernels (direct3.hip d3_shape: 56x56 64 -> 64,
    ResNeSt's deep-stem 112x112 32 -> 32 / 64), which take no operand prologue."""
    k, c, r, s = rec["conv"].weight.shape
    w = rec["x"].shape[2]
    return (r == 3 and s == 3 and rec["stride"] == 1 and rec.get("groups", 1) == 1
            and ((w == 56 and c == 64 and k == 64) or (w == 112 and c == 32 and k in (32, 64))))


def _direct3_input(blk, h):
    """The direct 3x3 kernel (direct3.hip d3_shape) serves conv2 of this block at input width h."""
    return tuple(blk.conv2.weight.shape) == (64, 64, 3, 3) and blk.stride == 1 and h == 56

# bf16 math (configs C4/C5): the tensors consumed only as conv operands -- the KRSC weights, the
# BN+ReLU outputs of each Bottleneck's first two units, every BatchNorm-backward output dy -- are
# stored as bf16 (tmr_conv_desc.io).  Exact: the bf16 convs round those operands to bf16 (RNE)
# when staging them anyway, so results are bit-identical to fp32 storage; the convs read half the
# bytes with no conversion.  TMR_BF16_STORE=0 keeps them fp32 (A/B measurements).
BF16_STORE = os.environ.get("TMR_BF16_STORE", "1") != "0"


def _store16(math):
    return math == "bf16" and BF16_STORE


# bf16 math with EVERY conv operand bf16 in HBM (train mode): the block outputs are written fp32
# (identity residual, ReLU mask) and as a bf16 copy in the same pass (bn_apply_dual / bn_apply2
# dual), the stem maxpool output as bf16 only (layer1.0 has a downsample, so it is never a
# residual), and each conv's dgrad reads a transposed bf16 weight copy (weight_to_crsk).  Every conv
# but the 4-channel stem then runs on the LDS-DMA engine (gemm16_kernel.h).  Same rounding of the
# same operands as the register-staged bf16 path, tests/test_bf16_gpu.py.  (A module attribute, no
# environment switch: tests/test_bf16_gpu.py turns it off to reach the fp32-storage forms.)
FULL16 = True

# bf16 activations (train mode, on top of FULL16; TMR_BF16_ACT=0 turns it off): every conv output
# y is stored rounded to bf16 by its epilogue (the BN statistics are those of the rounded values)
# and every BatchNorm(+residual)(+ReLU) output z is computed in fp32 and stored rounded to bf16 --
# block outputs included, so the identity residual is the bf16 block output.  Gradients stay fp32
# (dy, a conv operand, bf16).  This changes the numerics contract of the bf16 step (the oracle's
# emulate_bf16_convs(activations=True) restates it); the HBM traffic of every BatchNorm pass and of
# the conv epilogues halves.
ACT16 = os.environ.get("TMR_BF16_ACT", "1") != "0"


# fp32 math: the dgrad view runs on the fp32 form of the LDS-DMA engine, reading a transposed fp32
# weight copy (TMR_IO_WT_F32; the forward view takes that engine by itself).  (A module attribute
# for the prologue A/B test of the retired fold build, tests/test_kernels_gpu.py.)
DMA32 = True

# bf16-activation step: the masked BN-output gradient of the non-residual units (bn1, bn2 of every
# Bottleneck) stored bf16 by the fused dgrad (TMR_IO_G16; the residual stream's gradient stays
# fp32) -- halves the bytes of the dgrad store and of the BN-backward apply's read of g.  The
# contract (oracle.emulate_bf16_convs(grads=True)) rounds the gradient at those two points.
G16 = os.environ.get("TMR_G16", "1") != "0"

# bf16-activation step (ResNet-50 and ResNeSt-50 trunks): the residual stream's gradient -- the
# masked gradient of every Bottleneck's sum bn3(y3) + identity but the last block's -- is stored
# bf16 too
# (TMR_BF16_RESGRAD=0: fp32).  Each block's conv1 dgrad adds its part to the identity branch's
# gradient (read bf16, or fp32 from the downsample dgrad / the last block), masks it by the previous
# block's ReLU and rounds once (tmr_conv2d_dgrad_bnbwd_acc); the BN backward of bn3 and of the
# downsample BN read it bf16 (tmr_bn_bwd_parts_g16, tmr_bn_bwd_g16).  12-14 -> 6-7 B per element on
# the residual dgrads' epilogue.  The contract (oracle.emulate_bf16_convs(grads=True)) rounds the
# gradient of every block output but the last.
R16 = os.environ.get("TMR_BF16_RESGRAD", "1") != "0"

# downsample blocks: the BatchNorm backward of bn3 and of the downsample BN -- both take the
# block's masked pre-ReLU gradient g -- in one call whose apply pass reads g once for both dy's
# (tmr_bn_bwd_parts_ds: the values of the two separate passes; C2 174.2 -> 173.6 ms/step, C5
# 161.8 -> 161.5, profiles/r5/ds_dual/.  A module attribute for the bit-identity test.)
DS_DUAL = True


def _ds_dual(g, r3, rd):
    """DS_DUAL applies: g, y3 and y_ds of one dtype, which is also the dy dtype the separate passes
    would write (fp32 y under bf16 storage writes bf16 dy: not this path), 8-channel multiples;
    not under the dY-prologue A/B (FOLD16DY), which writes no dy at all."""
    y = r3["y"]
    return (DS_DUAL and not FOLD16DY and g.is_contiguous() and g.dtype == y.dtype == rd["y"].dtype
            and y.shape == rd["y"].shape and y.shape[-1] % 8 == 0
            and not (_store16(r3["math"]) and y.dtype == torch.float32))

# the fp32 block outputs' ReLU masks as bits for the mask-3 dgrads (round 2: 3622 -> 3634 frames/s,
# profiles/r2/bench_r3a/).  The bf16-activation step re-reads its 2-byte z instead: bits measured no
# faster there (profiles/r3/bench_r4i/, round-4 A/B under R16: the step unchanged) and were retired.


def _dma32(math):
    # (FOLD_BN too: the fp32 LDS-DMA engine applies the operand prologues in LDS, gemm16_kernel PRO)
    return math == "fp32" and DMA32


# bf16 activations: the direct bf16 stem takes the NHWC4 fp32 input itself (stem16.hip, round 4:
# 147 of 176 multiplies useful instead of 147 of 392); on the implicit-GEMM engine
# (ops.engine_only, tests) the stem reads an NHWC8 bf16 copy of it (LDS-DMA engine pieces)


def _full16(math):
    return _store16(math) and FULL16 and not FOLD_BN


def _act16(math):
    return _full16(math) and ACT16


def _conv_bn(x, conv, bn, stride, pad, relu, training, residual=None, recs=None, math="fp32",
             defer=False, branch=None, nbt=None, dual=False, groups=1):
    """conv (NHWC implicit GEMM) -> BN -> (+residual) -> (ReLU); returns z.

    Train mode only: ``defer`` returns (y, scale, shift) instead of applying the BN -- the
    consumer applies it on load (the downsample branch inside its block's BN3 pass, the stem
    inside the maxpool, with FOLD_BN the next conv's loaders); ``branch`` = such a deferred
    (y, scale, shift) used as the residual; ``x`` may itself be a deferred (y, scale, shift) of a
    ReLU unit, read through the conv's X-operand prologue.  ``dual`` (block outputs under
    _full16): returns (z fp32, z bf16 copy).  ``groups``: a grouped conv
    (train mode; ResNeSt's radix-2 3x3, tmr_conv_desc.groups)."""
    xpro = None
    if isinstance(x, tuple):
        x, xpro = x[0], (x[1], x[2])
    w = conv.weight
    k, c, r, s = w.shape
    cs = x.shape[3]
    s16 = _store16(math)
    if r == 1 and s == 1 and c == cs and not s16:
        wk = w.detach().contiguous().view(k, 1, 1, c)   # OIHW == KRSC for 1x1
    else:   # (grouped: torch's (K, C/G, R, S) -> stacked per-group KRSC blocks (K, R, S, C/G))
        wk = ops.weight_to_krsc(w.detach().contiguous(), cpad=cs // groups, bf16=s16)
    if groups > 1 and not training:
        raise RuntimeError("grouped convs run in the train-mode trunk only")
    if training:
        # batch statistics come out of the conv epilogue (no separate pass over y)
        y, stats, nparts = ops.conv_fwd_bnstats(x, wk, stride, pad, c_real=c * groups, math=math,
                                                xpro=xpro, y16=_act16(math), groups=groups)
        mean, inv, scale, shift = ops.bn_finalize(
            stats, nparts, bn.weight.detach(), bn.bias.detach(), bn.running_mean,
            bn.running_var, _bn_momentum(bn), bn.eps)
        # num_batches_tracked += 1; the trunk batches these into one launch (nbt list)
        if nbt is None:
            bn.num_batches_tracked.add_(1)
        else:
            nbt.append(bn.num_batches_tracked)
    else:
        if xpro is not None:
            raise RuntimeError("deferred BatchNorm inputs exist in train mode only")
        # eval: running-stat BN, residual and ReLU in the conv epilogue (one launch, no y pass;
        # same arithmetic as conv_fwd + bn_apply)
        scale, shift = ops.bn_eval_params(bn.weight.detach(), bn.bias.detach(), bn.running_mean,
                                          bn.running_var, bn.eps)
        return ops.conv_fwd_fused(x, wk, stride, pad, scale, shift, residual, relu, c_real=c,
                                  math=math)
    # fp32 block outputs on the LDS-DMA path also record their ReLU mask as bits: the dgrad that
    # produces their gradient reads 1 bit instead of z's 4 bytes (mask 3)
    zbits = None
    # (bf16 activations too: the bits of the rounded z, tmr_bn_apply_bits_a16)
    bits = (recs is not None and relu and not dual and _dma32(math) and y.dtype == torch.float32
            and (residual is not None or branch is not None))
    if defer:
        z = None
    elif branch is not None and bits:
        z, zbits = ops.bn_apply2_bits(y, scale, shift, branch[0], branch[1], branch[2])
    elif bits:
        z, zbits = ops.bn_apply_bits(y, scale, shift, residual)
    elif branch is not None:
        z = ops.bn_apply2(y, scale, shift, branch[0], branch[1], branch[2], relu, dual=dual)
    elif dual:
        z = ops.bn_apply_dual(y, scale, shift, residual, relu)
    else:
        # a non-residual unit's output is only ever a conv operand (next conv's forward and
        # wgrad; the backward recomputes its ReLU mask from y): bf16 under bf16 math (with bf16
        # activations every z is bf16: the dtype of y decides)
        z = ops.bn_apply(y, scale, shift, residual, relu, bf16=s16 and residual is None)
    if recs is not None:
        # without a residual the backward recomputes the ReLU mask from y (scale/shift)
        has_res = residual is not None or branch is not None
        # the dgrad view of a bf16-operand conv reads the transposed weights (LDS-DMA engine)
        if groups > 1 and ((_full16(math) and x.dtype == torch.bfloat16) or _dma32(math)):
            wt = ops.weight_to_crsk_grouped(w.detach().contiguous(), groups,
                                            bf16=x.dtype == torch.bfloat16)
        elif _full16(math) and x.dtype == torch.bfloat16:
            wt = ops.weight_to_crsk(w.detach().contiguous())
        elif _dma32(math) and c % 8 == 0 and x.dtype == torch.float32:
            wt = ops.weight_to_crsk(w.detach().contiguous(), bf16=False)
        else:   # (the stem's 3 input channels: no dgrad)
            wt = None
        recs.append({"x": x, "xpro": xpro, "wk": wk, "wt": wt, "y": y,
                     "z": (z[0] if dual else z) if has_res else None, "zbits": zbits,
                     "scale": scale, "shift": shift, "mean": mean, "inv": inv,
                     "stride": stride, "pad": pad, "relu": relu, "conv": conv, "bn": bn,
                     "c_real": c, "math": math, "groups": groups})
    return (y, scale, shift) if defer else z


def _conv_bn_bwd(rec, dz, grads, want_dres=False, dx_out=None, dx_beta=0.0, need_dx=True,
                 dres_inplace=False, parts=None, fuse_prev=None, pool=None, dy=None, g16=False,
                 r16=False):
    """BN backward, wgrad, dgrad (optionally accumulated into dx_out) of one conv+BN unit.

    parts: dz was produced by a fused dgrad (conv_dgrad_bnbwd): it is already ReLU-masked and
    `parts` holds its BN-backward partial sums.  Otherwise the ReLU mask comes from the saved z,
    or is recomputed from y when there was no residual.  dres_inplace: the pre-activation
    gradient (the identity branch's) overwrites dz and is returned as dres.
    fuse_prev: the unit whose BN output gradient this unit's dgrad produces -- its mask and
    partial sums are then computed in the dgrad epilogue; returned as the third value.
    pool: (pooled gradient, argmax) of the maxpool that consumed this unit's output (the stem);
    dz is then gathered from it inside the BN backward.
    dy: the conv's output gradient computed by the caller (ResNeSt's split-attention backward
    writes the grouped conv's dy with bn0's backward folded in): only wgrad and dgrad run here.
    g16: the fused dgrad may store fuse_prev's masked gradient as bf16 (TMR_IO_G16) when that unit
    has no residual and the dgrad runs on the bf16 LDS-DMA engine (the bf16-activation step).
    r16: the same for fuse_prev a block output (R16): the dgrad adds into dx_out (bf16 in place,
    or fp32 read and a new bf16 tensor returned)."""
    conv, bn = rec["conv"], rec["bn"]
    dpro = None    # (y, coef): dy = A*g + B*y + C evaluated by the consumer convs' loaders
    s16 = _store16(rec["math"])   # dy feeds only this conv's dgrad / wgrad
    dy_given = dy is not None
    if dy_given:
        dres = None
    elif pool is not None:
        # the stem: maxpool backward + ReLU mask + BN backward without writing dz
        dy, dg, db = ops.bn_bwd_maxpool(pool[0], pool[1], rec["y"], rec["scale"], rec["shift"],
                                        rec["mean"], rec["inv"], bn.weight.detach(), bf16=s16)
        dres = None
    elif FOLD_BN:
        rows = rec["y"].numel() // rec["y"].shape[-1]
        if parts is not None:   # dz already masked by the producing dgrad's epilogue
            coef, dg, db = ops.bn_bwd_coefs(parts[0], parts[1], rec["mean"], rec["inv"],
                                            bn.weight.detach(), rows)
        else:                   # one reduction pass; the ReLU mask is applied to dz in place
            if want_dres and not dres_inplace:
                raise RuntimeError("folded BN backward: the identity gradient is dz itself")
            coef, dg, db = ops.bn_bwd_coefs_dense(dz, rec["y"], rec["z"], rec["scale"],
                                                  rec["shift"], rec["mean"], rec["inv"],
                                                  bn.weight.detach(), rec["relu"])
        dy, dpro = dz, (rec["y"], coef)
        dres = dz if want_dres else None
    elif (FOLD16DY and dz.dtype == torch.bfloat16 and rec["y"].dtype == torch.bfloat16
          and (parts is not None or not rec["relu"]) and rec.get("groups", 1) == 1
          and not _direct3_conv(rec)):
        # the bf16 dY prologue: coefficients only, the consumers read g and y
        if parts is not None:
            coef, dg, db = ops.bn_bwd_coefs(parts[0], parts[1], rec["mean"], rec["inv"],
                                            bn.weight.detach(), rec["y"].numel() // rec["y"].shape[-1])
        else:   # the downsample BN (no ReLU): one reduction pass over g and y
            coef, dg, db = ops.bn_bwd_coefs_g16(dz, rec["y"], rec["mean"], rec["inv"],
                                                bn.weight.detach())
        dy, dpro = dz, (rec["y"], coef)
        dres = dz if want_dres else None
    elif parts is not None:
        dy, dg, db = ops.bn_bwd_parts(dz, rec["y"], parts[0], parts[1], rec["mean"], rec["inv"],
                                      bn.weight.detach(), bf16=s16)
        dres = dz if want_dres else None
    else:
        dy, dres, dg, db = ops.bn_bwd(dz, rec["y"], rec["z"], rec["mean"], rec["inv"],
                                      bn.weight.detach(), rec["relu"], want_dres=want_dres,
                                      dres_out=dz if dres_inplace else None,
                                      scale=rec["scale"], shift=rec["shift"], bf16=s16)
    if not dy_given:
        grads[bn.weight] = dg
        grads[bn.bias] = db
    x = rec["x"]
    k, c, r, s = conv.weight.shape
    grp = rec.get("groups", 1)
    grads[conv.weight] = ops.conv_wgrad(x, dy, r, s, rec["stride"], rec["pad"],
                                        c_real=rec["c_real"], math=rec["math"],
                                        xpro=rec.get("xpro"), dpro=dpro, groups=grp)
    dx, fused = None, None
    if need_dx:
        hw = (x.shape[1], x.shape[2])
        wt = rec.get("wt") is not None
        wdg = rec["wt"] if wt else rec["wk"]
        if fuse_prev is not None:
            p = fuse_prev
            mask = (1 if p["z"] is not None else 2) if p["relu"] else 0
            zm = p["z"]
            if mask == 1 and wt and p.get("zbits") is not None:
                mask, zm = 3, p["zbits"]   # the ReLU mask as bits (fp32 LDS-DMA dgrad)
            bf8 = (wt and (dpro is None or dpro[0].dtype == torch.bfloat16) and
                   p["y"].dtype == torch.bfloat16 and
                   (p["y"].shape[-1] // grp) % 8 == 0)
            # (a grouped dgrad -- ResNeSt's radix-2 conv -- stores its per-group channel slices bf16
            # too; the residual accumulation stays ungrouped)
            gb = (g16 and G16 and mask == 2 and dx_out is None and dx_beta == 0.0 and bf8)
            rb = (r16 and R16 and mask in (1, 3) and dx_out is not None and dx_beta == 1.0 and bf8
                  and grp == 1)
            old = None
            if rb and dx_out.dtype != torch.bfloat16:   # fp32 old dx -> a new bf16 dx
                old, dx_out = dx_out, None
            dx, pp, npp = ops.conv_dgrad_bnbwd(dy, wdg, hw, rec["stride"], rec["pad"],
                                               p["y"], p["mean"], mask, z=zm,
                                               scale=p["scale"], shift=p["shift"], out=dx_out,
                                               beta=dx_beta, math=rec["math"], dpro=dpro,
                                               wt=wt, groups=grp, g16=gb or rb, old=old)
            fused = (pp, npp)
        else:
            dx = ops.conv_dgrad(dy, wdg, hw, rec["stride"], rec["pad"], out=dx_out,
                                beta=dx_beta, math=rec["math"], dpro=dpro, wt=wt, groups=grp)
    return dx, dres, fused


class TrunkFn(torch.autograd.Function):
    """Whole ResNet-50 trunk as one autograd node: x NHWC4 (F,224,224,4) -> (F,2048)."""

    @staticmethod
    def forward(ctx, x4, share, keep, *params):
        # every conv weight layout of the step in one launch (ops.layout_session)
        with ops.layout_session(share, ("resnet50", share.training, bool(keep),
                                 share.precision)):
            return TrunkFn._forward(ctx, x4, share, keep, params)

    @staticmethod
    def _forward(ctx, x4, share, keep, params):
        training = share.training
        keep = keep and training
        recs = [] if keep else None
        nbt = []   # BatchNorm num_batches_tracked counters, incremented together at the end
        conv1, bn1, layers = share.trunk_parts()
        mt = share.precision
        a16 = training and _act16(mt)            # every activation bf16: no fp32 copies
        f16 = training and _full16(mt) and not a16
        if training:
            # bf16 activations: the stem reads an NHWC8 bf16 copy of its input (8-channel
            # pieces: the LDS-DMA engine; exact, the bf16 math rounds x anyway)
            xs = ops.nhwc4_to_bf16x8(x4) if (a16 and ops.engine_forced()) else x4
            # share.bn1 + relu applied inside the maxpool (the backward recomputes the ReLU
            # mask from y, so the stem's BN output is never needed)
            y0, sc0, sh0 = _conv_bn(xs, conv1, bn1, 2, 3, True, training, recs=recs, math=mt,
                                    defer=True, nbt=nbt)
            p, am = ops.maxpool_fwd_bn(y0, sc0, sh0, bf16=f16)
            stem_hw = (y0.shape[1], y0.shape[2])
        else:
            z = _conv_bn(x4, conv1, bn1, 2, 3, True, training, recs=recs, math=mt, nbt=nbt)
            p, am = ops.maxpool_fwd(z)
            stem_hw = (z.shape[1], z.shape[2])
        # h: the block input as the identity residual (fp32), hx: as the conv operand (the bf16
        # copy under f16; the maxpool output is only ever a conv operand)
        h, hx = (None, p) if f16 else (p, p)
        blocks = []
        for layer in layers:
            for blk in layer:
                brec = [] if keep else None
                fold = training and FOLD_BN
                fd16 = a16 and FOLD16
                z1 = _conv_bn(hx, blk.conv1, blk.bn1, 1, 0, True, training, recs=brec, math=mt,
                              nbt=nbt,
                              defer=fold or (fd16 and not _direct3_input(blk, hx.shape[2])))
                z2 = _conv_bn(z1, blk.conv2, blk.bn2, blk.stride, 1, True, training, recs=brec,
                              math=mt, nbt=nbt, defer=fold or fd16)
                if blk.downsample is not None:
                    # train: the branch's BN is applied inside the BN3 pass (bn_apply2)
                    idn = _conv_bn(hx, blk.downsample[0], blk.downsample[1], blk.stride, 0, False,
                                   training, recs=brec, math=mt, defer=training, nbt=nbt)
                else:
                    if h is None:
                        raise RuntimeError("identity residual of the stem output (no downsample)")
                    idn = h
                if isinstance(idn, tuple):
                    h = _conv_bn(z2, blk.conv3, blk.bn3, 1, 0, True, training, branch=idn,
                                 recs=brec, math=mt, nbt=nbt, dual=f16)
                else:
                    h = _conv_bn(z2, blk.conv3, blk.bn3, 1, 0, True, training, residual=idn,
                                 recs=brec, math=mt, nbt=nbt, dual=f16)
                h, hx = h if f16 else (h, h)
                blocks.append((blk, brec))
        feat = ops.avgpool_fwd(h)
        ops.counters_add_one(nbt)
        ctx.keep = keep
        if keep:
            ctx.share = share
            ctx.params = params
            ctx.stem = recs
            ctx.pool = (am, stem_hw)
            ctx.blocks = blocks
            ctx.last_hw = (h.shape[1], h.shape[2])
        return feat

    @staticmethod
    def backward(ctx, dfeat):
        if not ctx.keep:
            raise RuntimeError("trunk backward needs train mode and a forward with grad enabled")
        grads = {}
        g = ops.avgpool_bwd(dfeat.contiguous(), ctx.last_hw)   # grad at the last block output
        blocks = ctx.blocks
        pending = None     # BN-backward partials of g when the dgrad that produced it was fused
        ready = get_grad_ready(ctx.share)   # ddp.GradAllReduce.grads_ready, or None
        while blocks:
            blk, brec = blocks.pop()
            has_ds = blk.downsample is not None
            r1, r2 = brec[0], brec[1]
            rd = brec[2] if has_ds else None
            r3 = brec[-1]
            # the previous block's last unit: its BN output gradient is this block's dx
            prev3 = blocks[-1][1][-1] if blocks else None
            # g (owned here) becomes the masked pre-ReLU gradient = the identity-branch grad
            dyd = None
            if (has_ds and _ds_dual(g, r3, rd) and pending is not None):
                # (g came masked from the next block's fused dgrad)
                dy3, dg3, db3, dyd, dgd, dbd = ops.bn_bwd_parts_ds(
                    g, r3["y"], pending[0], pending[1], r3["mean"], r3["inv"],
                    r3["bn"].weight.detach(), rd["y"], rd["mean"], rd["inv"],
                    rd["bn"].weight.detach())
                grads[r3["bn"].weight], grads[r3["bn"].bias] = dg3, db3
                grads[rd["bn"].weight], grads[rd["bn"].bias] = dgd, dbd
                dz2, _, fz2 = _conv_bn_bwd(r3, None, grads, fuse_prev=r2, g16=True, dy=dy3)
                dres = g
                del dy3
            else:
                dz2, dres, fz2 = _conv_bn_bwd(r3, g, grads, want_dres=True, dres_inplace=True,
                                              parts=pending, fuse_prev=r2, g16=True)
            dz1, _, fz1 = _conv_bn_bwd(r2, dz2, grads, parts=fz2, fuse_prev=r1, g16=True)
            del dz2
            if has_ds:
                # the strided downsample dgrad writes dx (its tap-less parity classes as zeros),
                # the stride-1 conv1 dgrad accumulates into it with the fused BN backward
                # (measured 51.1 vs 51.6 ms of dgrads per C2 step against the other order,
                # profiles/r3/bench_r4f/)
                if dyd is not None:
                    dx, _, _ = _conv_bn_bwd(rd, None, grads, dy=dyd)
                    del dyd
                else:
                    dx, _, _ = _conv_bn_bwd(rd, dres, grads)
                dx, _, pending = _conv_bn_bwd(r1, dz1, grads, parts=fz1, dx_out=dx, dx_beta=1.0,
                                              fuse_prev=prev3, r16=True)
            else:
                dx, _, pending = _conv_bn_bwd(r1, dz1, grads, parts=fz1, dx_out=dres, dx_beta=1.0,
                                              fuse_prev=prev3, r16=True)
            del dz1, brec, dres
            g = dx
            if ready is not None:   # this block's parameter grads are final: start their exchange
                ready([(p, grads[p]) for p in blk.parameters() if p in grads])
        dh = g
        am, stem_hw = ctx.pool
        _conv_bn_bwd(ctx.stem[0], None, grads, need_dx=False, pool=(dh, am))
        out = [grads.get(p) for p in ctx.params]
        ctx.blocks = ctx.stem = None
        return (None, None, None) + tuple(out)


_CHILD_NAMES = ("conv1", "bn1", "relu", "maxpool", "layer1", "layer2", "layer3", "layer4",
                "avgpool")


class ResNet50Share(nn.Sequential):
    """The reference's `share` Sequential (keys identical to torchvision's resnet50 children).

    ``indexed=True`` names the children "0".."8" instead, which is the
    ``Sequential(*list(resnet50().children())[:-1])`` layout of code/models.py:26-28
    (keys ``res.0.weight``, ``res.4.0.conv1.weight``, ...).
    """

    def __init__(self, indexed=False, precision="fp32"):
        super().__init__()
        self.precision = precision   # conv operand precision: "fp32" | "bf16" (ops.MATH)
        mods = (nn.Conv2d(3, 64, 7, stride=2, padding=3, bias=False), nn.BatchNorm2d(64),
                nn.ReLU(inplace=True), nn.MaxPool2d(3, stride=2, padding=1),
                _make_layer(64, 64, 3, 1), _make_layer(256, 128, 4, 2),
                _make_layer(512, 256, 6, 2), _make_layer(1024, 512, 3, 2),
                nn.AdaptiveAvgPool2d((1, 1)))
        for i, (name, m) in enumerate(zip(_CHILD_NAMES, mods)):
            self.add_module(str(i) if indexed else name, m)
        # torchvision init: kaiming_normal fan_out for convs, BN gamma=1 beta=0
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.constant_(m.weight, 1)
                nn.init.constant_(m.bias, 0)

    def trunk_parts(self):
        ch = list(self.children())
        return ch[0], ch[1], ch[4:8]

    def features_nhwc4(self, x4):
        """x4: (F,224,224,4) fp32 NHWC, 4th channel zero -> (F,2048)."""
        params = list(self.parameters())
        # grad mode is off inside autograd.Function.forward: decide here whether to save
        keep = torch.is_grad_enabled() and any(p.requires_grad for p in params)
        return TrunkFn.apply(x4, self, keep, *params)

    def forward(self, x):
        """x: (F,3,224,224) fp32 NCHW (reference layout) -> (F,2048,1,1)."""
        x = x.reshape(-1, 3, x.shape[-2], x.shape[-1]).contiguous()
        x4 = ops.nchw_to_nhwc(x, cpad=4)
        feat = self.features_nhwc4(x4)
        return feat.view(feat.shape[0], feat.shape[1], 1, 1)


def resnet50_share():
    return ResNet50Share()
