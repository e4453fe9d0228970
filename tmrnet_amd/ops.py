"""Tensor-level wrappers over the libtmr C ABI.

Every function takes CUDA(HIP) tensors, allocates outputs with torch's caching
allocator (the library never allocates), passes raw pointers plus the current
stream, and raises RuntimeError on a failed call.  No function here computes
anything itself: all arithmetic runs in the HIP kernels of libtmr.so.
"""
import contextlib
import threading
import weakref

import numpy as np
import torch

from ._lib import call, query, stream_ptr, has_prologues, ConvDesc, ConvPrologue
from . import health
import ctypes

f32 = torch.float32

# Optional live instrumentation (bench.py): when a list, every conv launch appends
# (kind, algorithmic_flops, start_event, end_event, shape, algorithmic_bytes) recorded on the
# launching stream.  Algorithmic bytes = each operand read once + the output written once
# (+ read once more when accumulating with beta != 0).
PROF = None


class _prof:
    def __init__(self, kind, flops, shape=None, nbytes=0):
        self.kind, self.flops, self.shape, self.nbytes = kind, flops, shape, nbytes

    def __enter__(self):
        if PROF is not None:
            self.e0 = torch.cuda.Event(enable_timing=True)
            self.e1 = torch.cuda.Event(enable_timing=True)
            self.e0.record()
        return self

    def __exit__(self, *a):
        if PROF is not None:
            self.e1.record()
            PROF.append((self.kind, self.flops, self.e0, self.e1, self.shape, self.nbytes))
        return False


def _req(t, name, dtype=f32):
    if not t.is_cuda:
        raise RuntimeError("%s must be a GPU tensor (libtmr has no CPU path)" % name)
    if t.dtype != dtype:
        raise RuntimeError("%s must be %s, got %s" % (name, dtype, t.dtype))
    if not t.is_contiguous():
        raise RuntimeError("%s must be contiguous" % name)
    return t


def _nhwc_ld(t, name):
    """Pixel stride of an NHWC tensor or channel-slice view of one (0 when dense)."""
    if t.is_contiguous():
        return 0
    n, h, w, c = t.shape
    ld = t.stride(2)
    if t.stride(3) != 1 or t.stride(1) != w * ld or t.stride(0) != h * w * ld:
        raise RuntimeError("%s must be NHWC or a channel slice of an NHWC tensor" % name)
    return ld


def _empty(shape, like, dtype=f32):
    return torch.empty(shape, dtype=dtype, device=like.device)


# ----------------------------------------------------------------- conv / gemm
MATH = {"fp32": 0, "bf16": 1}   # tmr_conv_desc.math (TMR_MATH_F32 / TMR_MATH_BF16)
_SUFFIX = {"fp32": "", "bf16": "_bf16"}
# frames per conv launch (tmr_conv_desc.max_frames): 0 = automatic (operands < 2 GiB); tests set
# a small cap to exercise the frame-chunked launches at small sizes
MAX_FRAMES = 0


IO_X, IO_W, IO_DY, IO_WT = 1, 2, 4, 8   # tmr_conv_desc.io: bf16-stored x / KRSC w / dy / CRSK w
IO_Y, IO_BN = 16, 32    # bf16 conv output y (forward) / bf16 y, z of the fused BN backward (dgrad)
IO_WT32 = 64            # dgrad, fp32 math: w is the transposed fp32 copy (fp32 LDS-DMA engine)
IO_G16 = 128            # fused BN-backward dgrad: g (dx) written bf16 (non-residual bf16 units)
IO_ENGINE = 256         # the implicit-GEMM engine even where a direct kernel serves the geometry
IO_CLASSES = 512        # strided dgrad: one launch per stride-parity class (tests' comparison form)
IO_TILES = 1024         # fused dgrad: one tile per workgroup, not the wave-specialised kernel (tests)

# test instrumentation (process-wide: autograd runs the backward of a CUDA graph on its own
# device thread, which must see the same routing as the forward)
_ENGINE = [False]


@contextlib.contextmanager
def engine_only():
    """Within the block every conv runs on the implicit-GEMM engine, also where a direct kernel
    serves the geometry (the 7x7 stems, the narrow 3x3 convs of direct3.hip): TMR_IO_ENGINE, the
    independent second implementation tests compare those kernels with.  Tests only."""
    prev = _ENGINE[0]
    _ENGINE[0] = True
    try:
        yield
    finally:
        _ENGINE[0] = prev


def engine_forced():
    return _ENGINE[0]


_CLASSES = [False]


@contextlib.contextmanager
def dgrad_class_launches():
    """Within the block a strided dgrad runs as one launch per stride-parity class
    (TMR_IO_CLASSES) instead of one launch over every class's tiles.  Tests only."""
    prev = _CLASSES[0]
    _CLASSES[0] = True
    try:
        yield
    finally:
        _CLASSES[0] = prev

_TILES = [False]


@contextlib.contextmanager
def dgrad_tile_launches():
    """Within the block a fused BN-backward dgrad runs one output tile per workgroup
    (TMR_IO_TILES) also where the wave-specialised persistent kernel serves its shape (the 1x1
    stride-1 dgrads, round 6).  Tests only."""
    prev = _TILES[0]
    _TILES[0] = True
    try:
        yield
    finally:
        _TILES[0] = prev


BF16 = torch.bfloat16


def _io(x=None, w=None, dy=None, wt=False):
    """tmr_conv_desc.io from the operands' dtypes (bf16 storage of conv-operand-only tensors);
    wt: w is the transposed [Cin][R][S][Cout] copy (dgrad view, weight_to_crsk): bf16 with bf16
    math (TMR_IO_WT_BF16), fp32 with fp32 operands (TMR_IO_WT_F32)."""
    if wt and w.dtype == f32:
        if (dy is not None and dy.dtype != f32) or (x is not None and x.dtype != f32):
            raise RuntimeError("fp32 transposed (CRSK) weights need fp32 operands")
        return IO_WT32
    io = 0
    for t, bit in ((x, IO_X), (w, IO_WT if wt else IO_W), (dy, IO_DY)):
        if t is not None and t.dtype == torch.bfloat16:
            io |= bit
    if wt and not io & IO_WT:
        raise RuntimeError("transposed (CRSK) weights must be bf16 or fp32")
    return io


def _dgrad_w(w, wt, groups=1):
    """(k, r, s, c) totals of a dgrad weight operand: KRSC (k, r, s, c/groups), or with wt the
    transposed copy (c, r, s, k) -- per group (groups, c/groups, r, s, k/groups)."""
    if wt and groups > 1:
        g, cg, r, s, kg = w.shape
        return kg * g, r, s, cg * g
    if wt:
        c, r, s, k = w.shape
    else:
        k, r, s, c = w.shape
        c *= groups
    return k, r, s, c


def _esz(t):
    return t.element_size() if t is not None else 4


def conv_desc(n, h, w, c, k, r, s, stride, pad, pad_w=None, x_ld=0, y_ld=0, math="fp32", io=0,
              groups=1):
    pad_w = pad if pad_w is None else pad_w
    ho = (h + 2 * pad - r) // stride + 1
    wo = (w + 2 * pad_w - s) // stride + 1
    if io and io != IO_WT32 and math != "bf16":
        raise RuntimeError("bf16-stored conv operands need math='bf16'")
    if io & IO_WT32 and math != "fp32":
        raise RuntimeError("fp32 transposed weights (TMR_IO_WT_F32) need math='fp32'")
    if engine_forced():
        io |= IO_ENGINE
    if _CLASSES[0] and stride == 2:
        io |= IO_CLASSES
    if _TILES[0] and r == 1 and s == 1 and stride == 1:
        io |= IO_TILES
    return ConvDesc(n, h, w, c, k, r, s, stride, pad, ho, wo, pad_w, x_ld, y_ld, MATH[math],
                    MAX_FRAMES, io, groups if groups > 1 else 0)


def _req_op(t, name):
    """A conv operand: fp32, or bf16 (stored rounded; bf16 math only)."""
    return _req(t, name, torch.bfloat16 if t.dtype == torch.bfloat16 else f32)


def conv_fwd(x, w_krsc, stride, pad, bias=None, out=None, beta=0.0, c_real=None, pad_w=None,
             math="fp32"):
    """x (N,H,W,C) NHWC (or channel-slice view), w_krsc (K,R,S,C) -> y (N,Ho,Wo,K);
    `out` may be a channel-slice view of a wider NHWC tensor (grouped convolution)."""
    _req_op(w_krsc, "w")
    n, h, w, c = x.shape
    k, r, s, c2 = w_krsc.shape
    assert c == c2, (x.shape, w_krsc.shape)
    d = conv_desc(n, h, w, c, k, r, s, stride, pad, pad_w, math=math, io=_io(x, w_krsc))
    if out is None:
        out = _empty((n, d.ho, d.wo, k), x)
    d.x_ld = _nhwc_ld(x, "x")
    d.y_ld = _nhwc_ld(out, "out")
    ysz = n * d.ho * d.wo * k
    with _prof("conv_fwd" + _SUFFIX[math], 2.0 * n * d.ho * d.wo * k * r * s * (c_real or c),
               (n, h, w, c, k, r, stride),
               4 * (n * h * w * c + k * r * s * c + ysz * (2 if beta else 1))):
        call("tmr_conv2d_fwd", ctypes.byref(d), x, w_krsc, bias if bias is not None else None,
             out, float(beta), stream_ptr())
    return out


def conv_fwd_fused(x, w_krsc, stride, pad, scale, shift, residual=None, relu=True, c_real=None,
                   pad_w=None, math="fp32"):
    """Inference conv + BN(running stats) [+ residual] [+ ReLU] in one launch:
    [relu](conv(x, w_krsc) * scale + shift + residual) -> (N,Ho,Wo,K)."""
    _req_op(x, "x"); _req_op(w_krsc, "w"); _req(scale, "scale"); _req(shift, "shift")
    n, h, w, c = x.shape
    k, r, s, c2 = w_krsc.shape
    assert c == c2, (x.shape, w_krsc.shape)
    d = conv_desc(n, h, w, c, k, r, s, stride, pad, pad_w, math=math, io=_io(x, w_krsc))
    out = _empty((n, d.ho, d.wo, k), x)
    if residual is not None:
        _req(residual, "residual")
        if residual.shape != out.shape:
            raise RuntimeError("conv_fwd_fused: residual %s != output %s"
                               % (tuple(residual.shape), tuple(out.shape)))
    ysz = n * d.ho * d.wo * k
    with _prof("conv_fwd" + _SUFFIX[math], 2.0 * ysz * r * s * (c_real or c),
               (n, h, w, c, k, r, stride),
               4 * (n * h * w * c + k * r * s * c + ysz * (2 if residual is not None else 1))):
        call("tmr_conv2d_fwd_fused", ctypes.byref(d), x, w_krsc, scale, shift, residual, out,
             int(relu), stream_ptr())
    return out


def _need_prologues():
    if not has_prologues():
        raise RuntimeError("operand prologues (TMR_FOLD_BN=1) are a retired A/B experiment: build "
                           "`make PROLOGUES=1` and set TMR_LIB_PATH=tmrnet_amd/libtmr_pro.so")


def _prologue(xpro=None, dpro=None):
    """tmr_conv_prologue from (scale, shift) of the X operand's producer BN+ReLU and/or (y, coef)
    of this conv's BN backward; None when neither is given."""
    if xpro is None and dpro is None:
        return None
    _need_prologues()
    p = ConvPrologue()
    if xpro is not None:
        p.x_scale, p.x_shift = _req(xpro[0], "x_scale").data_ptr(), _req(xpro[1], "x_shift").data_ptr()
    if dpro is not None:
        # (y fp32, or bf16 with the bf16 engine's dY prologue: g's element type)
        p.dy_y, p.dy_coef = _req_op(dpro[0], "dy_y").data_ptr(), _req(dpro[1], "dy_coef").data_ptr()
    return p


def conv_fwd_bnstats(x, w_krsc, stride, pad, c_real=None, pad_w=None, math="fp32", xpro=None,
                     y16=False, groups=1):
    """conv_fwd whose epilogue also emits BatchNorm partials; returns (y, stats, nparts).
    xpro = (scale, shift): x is a pre-BN tensor read as relu(x*scale + shift) (0 at padding).
    y16: y stored rounded to bf16, the partials describing the rounded values (TMR_IO_Y_BF16).
    groups: a grouped conv (w_krsc (K, R, S, C/groups), torch's grouped layout); c_real is the
    total real input channels."""
    _req_op(x, "x"); _req_op(w_krsc, "w")
    n, h, w, c = x.shape
    k, r, s, c2 = w_krsc.shape
    assert c == c2 * groups, (x.shape, w_krsc.shape, groups)
    d = conv_desc(n, h, w, c, k, r, s, stride, pad, pad_w, math=math,
                  io=_io(x, w_krsc) | (IO_Y if y16 else 0), groups=groups)
    out = _empty((n, d.ho, d.wo, k), x, dtype=BF16 if y16 else f32)
    nparts = query("tmr_conv2d_fwd_stats_parts", ctypes.byref(d))
    stats = torch.empty((nparts, k, 4), dtype=f32, device=x.device)
    with _prof("conv_fwd" + _SUFFIX[math], 2.0 * n * d.ho * d.wo * k * r * s * (c_real or c) / groups,
               (n, h, w, c, k, r, stride),
               _esz(x) * n * h * w * c + _esz(w_krsc) * k * r * s * c2
               + out.element_size() * n * d.ho * d.wo * k + stats.numel() * 4):
        pro = _prologue(xpro)
        if pro is None:
            call("tmr_conv2d_fwd_bnstats", ctypes.byref(d), x, w_krsc, out, stats,
                 ctypes.c_size_t(stats.numel() * 4), stream_ptr())
        else:
            call("tmr_conv2d_fwd_bnstats_pro", ctypes.byref(d), x, w_krsc, out, stats,
                 ctypes.c_size_t(stats.numel() * 4), ctypes.byref(pro), stream_ptr())
    return out, stats, nparts


def bn_finalize(stats, nparts, gamma, beta, running_mean, running_var, momentum, eps):
    c = stats.shape[1]
    mean = _empty((c,), stats); inv = _empty((c,), stats)
    scale = _empty((c,), stats); shift = _empty((c,), stats)
    nb = query("tmr_bn_parts_ws_bytes", int(nparts), c)
    ws = torch.empty(((nb + 7) // 8,), dtype=torch.float64, device=stats.device)
    call("tmr_bn_finalize_ws", stats, nparts, c, gamma, beta, running_mean, running_var,
         float(momentum), float(eps), mean, inv, scale, shift, ws, ctypes.c_size_t(ws.numel() * 8),
         stream_ptr())
    return mean, inv, scale, shift


def conv_dgrad(dy, w_krsc, in_hw, stride, pad, out=None, beta=0.0, pad_w=None, math="fp32",
               dpro=None, wt=False, groups=1):
    """dy (N,Ho,Wo,K), w_krsc (K,R,S,C) -> dx (N,H,W,C) (dy/out may be channel slices).
    dpro = (y, coef): dy is the masked BN-output gradient g, read as the BN backward
    A*g + B*y + C (tmr_bn_bwd_coefs).  wt: w_krsc is the transposed copy (C,R,S,K)
    (weight_to_crsk; the LDS-DMA engine: bf16 with bf16 dy, or fp32 with fp32 math)."""
    _req_op(w_krsc, "w")
    n, ho, wo, k = dy.shape
    k2, r, s, c = _dgrad_w(w_krsc, wt, groups)
    h, w = in_hw
    d = conv_desc(n, h, w, c, k, r, s, stride, pad, pad_w, math=math, io=_io(None, w_krsc, dy, wt),
                  groups=groups)
    assert (d.ho, d.wo) == (ho, wo), ((d.ho, d.wo), (ho, wo))
    if out is None:
        out = _empty((n, h, w, c), dy)
    d.x_ld = _nhwc_ld(out, "dx")
    d.y_ld = _nhwc_ld(dy, "dy")
    with _prof("conv_dgrad" + _SUFFIX[math], 2.0 * n * ho * wo * k * r * s * c / groups, (n, h, w, c, k, r, stride),
               _esz(dy) * n * ho * wo * k * (2 if dpro is not None else 1) + _esz(w_krsc) * w_krsc.numel()
               + 4 * n * h * w * c * (2 if beta else 1)):
        pro = _prologue(None, dpro)
        if pro is None:
            call("tmr_conv2d_dgrad", ctypes.byref(d), dy, w_krsc, out, float(beta), stream_ptr())
        else:
            call("tmr_conv2d_dgrad_pro", ctypes.byref(d), dy, w_krsc, out, float(beta),
                 ctypes.byref(pro), stream_ptr())
    return out


def conv_dgrad_bnbwd(dy, w_krsc, in_hw, stride, pad, y, mean, mask, z=None, scale=None,
                     shift=None, out=None, beta=0.0, math="fp32", dpro=None, wt=False, groups=1,
                     g16=False, old=None):
    """conv_dgrad whose epilogue masks dx by the previous unit's ReLU (mask 1: z > 0, 2:
    y*scale+shift > 0) and emits that unit's BN-backward partials -> (dx_masked, parts, nparts).
    wt: as conv_dgrad.  y / z may be bf16 (the bf16-activation step, TMR_IO_BN_BF16).
    g16: dx_masked stored bf16, the partials those of the rounded values (TMR_IO_G16); with beta
    the old dx is `out` itself (bf16, in place) or `old` (fp32 or bf16; tmr_conv2d_dgrad_bnbwd_acc,
    a new bf16 dx is returned)."""
    if old is not None:
        if not (g16 and beta != 0.0 and out is None and groups == 1):
            raise RuntimeError("conv_dgrad_bnbwd: a separate old dx needs g16, beta, no out / "
                               "groups")
        if old.dtype not in (f32, BF16) or not old.is_contiguous():
            raise RuntimeError("conv_dgrad_bnbwd: old dx must be a contiguous fp32 / bf16 tensor")
    if g16 and groups > 1 and beta != 0.0:
        raise RuntimeError("conv_dgrad_bnbwd: a grouped dgrad accumulates (beta != 0) into an fp32 "
                           "dx only")
    _req_op(w_krsc, "w"); _req_op(y, "y"); _req(mean, "mean")
    if mask == 3:   # z = ReLU-mask bits of dx's shape (bn_apply_bits)
        if z is None or z.dtype != torch.int32 or z.numel() * 32 < y.numel():
            raise RuntimeError("conv_dgrad_bnbwd: mask 3 takes the int32 ReLU-mask bits of y's shape")
    elif z is not None and z.dtype != y.dtype:
        raise RuntimeError("conv_dgrad_bnbwd: y and z must have one dtype")
    n, ho, wo, k = dy.shape
    k2, r, s, c = _dgrad_w(w_krsc, wt, groups)
    h, w = in_hw
    d = conv_desc(n, h, w, c, k, r, s, stride, pad, math=math,
                  io=_io(None, w_krsc, dy, wt) | (IO_BN if y.dtype == BF16 else 0)
                  | (IO_G16 if g16 else 0), groups=groups)
    assert (d.ho, d.wo) == (ho, wo), ((d.ho, d.wo), (ho, wo))
    if out is None:
        out = _empty((n, h, w, c), dy, dtype=BF16 if g16 else f32)
    elif out.dtype != (BF16 if g16 else f32):
        raise RuntimeError("conv_dgrad_bnbwd: dx must be %s" % ("bf16 (g16)" if g16 else "fp32"))
    if tuple(y.shape) != tuple(out.shape) or (z is not None and mask != 3
                                              and tuple(z.shape) != tuple(out.shape)):
        raise RuntimeError("conv_dgrad_bnbwd: y/z must have dx's shape %s" % (tuple(out.shape),))
    if old is not None and tuple(old.shape) != tuple(out.shape):
        raise RuntimeError("conv_dgrad_bnbwd: old dx must have dx's shape %s" % (tuple(out.shape),))
    d.x_ld = _nhwc_ld(out, "dx")
    d.y_ld = _nhwc_ld(dy, "dy")
    nparts = query("tmr_conv2d_dgrad_bnbwd_parts", ctypes.byref(d))
    if nparts < 0:
        raise RuntimeError("tmr_conv2d_dgrad_bnbwd_parts failed")
    parts = torch.empty((max(nparts, 1), c, 2), dtype=f32, device=dy.device)
    with _prof("conv_dgrad" + _SUFFIX[math], 2.0 * n * ho * wo * k * r * s * c / groups, (n, h, w, c, k, r, stride),
               _esz(dy) * n * ho * wo * k * (2 if dpro is not None else 1) + _esz(w_krsc) * w_krsc.numel()
               + (2 if g16 else 4) * n * h * w * c
               + ((old.element_size() if old is not None else (2 if g16 else 4)) * n * h * w * c
                  if beta else 0)
               + y.element_size() * n * h * w * c * (2 if z is not None and mask != 3 else 1)
               + (n * h * w * c // 8 if mask == 3 else 0)):
        pro = _prologue(None, dpro)
        if old is not None and pro is None:
            call("tmr_conv2d_dgrad_bnbwd_acc", ctypes.byref(d), dy, w_krsc, out, float(beta), old,
                 int(old.dtype == BF16), y, z, scale, shift, mean, int(mask), parts,
                 ctypes.c_size_t(parts.numel() * 4), stream_ptr())
        elif old is not None:
            call("tmr_conv2d_dgrad_bnbwd_acc_pro", ctypes.byref(d), dy, w_krsc, out, float(beta),
                 old, int(old.dtype == BF16), y, z, scale, shift, mean, int(mask), parts,
                 ctypes.c_size_t(parts.numel() * 4), ctypes.byref(pro), stream_ptr())
        elif pro is None:
            call("tmr_conv2d_dgrad_bnbwd", ctypes.byref(d), dy, w_krsc, out, float(beta), y, z,
                 scale, shift, mean, int(mask), parts, ctypes.c_size_t(parts.numel() * 4),
                 stream_ptr())
        else:
            call("tmr_conv2d_dgrad_bnbwd_pro", ctypes.byref(d), dy, w_krsc, out, float(beta), y,
                 z, scale, shift, mean, int(mask), parts, ctypes.c_size_t(parts.numel() * 4),
                 ctypes.byref(pro), stream_ptr())
    return out, parts, nparts


def bn_bwd_maxpool(dyp, am, y, scale, shift, mean, inv, gamma, bf16=False):
    """Stem backward: maxpool(3,2,1) backward + ReLU mask (from y) + BN backward in two passes
    over y; the maxpool's input gradient is never written.  -> (dy, dgamma, dbeta)."""
    n, h, w, c = y.shape
    _, ho, wo, _ = dyp.shape
    ws, nb = _bn_ws(n * h * w, c, y.device)
    if y.dtype == BF16:   # bf16 activations: dy is bf16 too
        dy = torch.empty_like(y)
        dgamma = _empty((c,), dyp); dbeta = _empty((c,), dyp)
        call("tmr_bn_bwd_maxpool_a16", dyp, am, n, h, w, ho, wo, y, scale, shift, mean, inv, gamma,
             dy, dgamma, dbeta, c, ws, ctypes.c_size_t(nb), stream_ptr())
        return dy, dgamma, dbeta
    dy = torch.empty_like(y, dtype=torch.bfloat16 if bf16 else y.dtype)
    dgamma = _empty((c,), y); dbeta = _empty((c,), y)
    call("tmr_bn_bwd_maxpool_x", dyp, am, n, h, w, ho, wo, y, scale, shift, mean, inv, gamma, dy,
         dgamma, dbeta, c, ws, ctypes.c_size_t(nb), int(bf16), stream_ptr())
    return dy, dgamma, dbeta


def bn_bwd_coefs(parts, nparts, mean, inv, gamma, rows):
    """BN backward coefficients from conv_dgrad_bnbwd partials -> (coef [3][c], dgamma, dbeta);
    the consumers apply dy = A*g + B*y + C on load (dpro=(y, coef))."""
    _need_prologues()
    c = mean.shape[0]
    coef = _empty((3, c), mean)
    dgamma = _empty((c,), mean); dbeta = _empty((c,), mean)
    nb = query("tmr_bn_parts_ws_bytes", int(nparts), c)
    ws = torch.empty(((nb + 7) // 8,), dtype=torch.float64, device=mean.device)
    call("tmr_bn_bwd_coefs", parts, int(nparts), mean, inv, gamma, coef, dgamma, dbeta, int(rows),
         c, ws, ctypes.c_size_t(ws.numel() * 8), stream_ptr())
    return coef, dgamma, dbeta


def bn_bwd_coefs_dense(g, y, z, scale, shift, mean, inv, gamma, relu):
    """BN backward coefficients from the output gradient g itself (one reduction pass over g and
    y); with relu, g is masked IN PLACE (z > 0, or y*scale+shift > 0 when z is None).
    -> (coef [3][c], dgamma, dbeta)."""
    _need_prologues()
    c = y.shape[-1]
    rows = y.numel() // c
    _req(g, "g"); _req(y, "y")
    coef = _empty((3, c), y)
    dgamma = _empty((c,), y); dbeta = _empty((c,), y)
    ws, nb = _bn_ws(rows, c, y.device)
    call("tmr_bn_bwd_coefs_dense", g, y, z, scale, shift, mean, inv, gamma, coef, dgamma, dbeta,
         rows, c, int(relu), ws, ctypes.c_size_t(nb), stream_ptr())
    return coef, dgamma, dbeta


def bn_bwd_coefs_g16(g, y, mean, inv, gamma):
    """BN backward coefficients of a unit without ReLU from its bf16 output gradient g and bf16 y
    (the downsample BN of the bf16-activation step) -> (coef [3][c], dgamma, dbeta)."""
    _need_prologues()
    c = y.shape[-1]
    rows = y.numel() // c
    if g.dtype != BF16 or y.dtype != BF16 or g.shape != y.shape:
        raise RuntimeError("bn_bwd_coefs_g16: g and y must be bf16 tensors of one shape")
    _req_op(g, "g"); _req_op(y, "y")
    coef = _empty((3, c), mean)
    dgamma = _empty((c,), mean); dbeta = _empty((c,), mean)
    ws, nb = _bn_ws(rows, c, y.device)
    call("tmr_bn_bwd_coefs_g16", g, y, mean, inv, gamma, coef, dgamma, dbeta, rows, c, ws,
         ctypes.c_size_t(nb), stream_ptr())
    return coef, dgamma, dbeta


def bn_bwd_parts_ds(g, y, parts, nparts, mean, inv, gamma, yd, mean_d, inv_d, gamma_d):
    """BN backward of a downsample block's bn3 (from the fused dgrad's partials, g already
    masked) and of its downsample BN (a reduction pass over g and y_ds), with one apply pass that
    reads g once -> (dy, dgamma, dbeta, dy_ds, dgamma_ds, dbeta_ds); the values of bn_bwd_parts +
    bn_bwd.  g, y, y_ds all fp32 or all bf16 (the dy's take their dtype)."""
    c = y.shape[-1]
    rows = y.numel() // c
    t = y.dtype
    if not (g.dtype == t and yd.dtype == t and t in (f32, BF16) and g.shape == y.shape == yd.shape
            and g.is_contiguous() and y.is_contiguous() and yd.is_contiguous()):
        raise RuntimeError("bn_bwd_parts_ds: g, y and y_ds must be contiguous tensors of one shape "
                           "and one dtype (fp32 or bf16)")
    nb = query("tmr_bn_bwd_parts_ds_ws_bytes", int(nparts), rows, c)
    ws = torch.empty(((nb + 7) // 8,), dtype=torch.float64, device=y.device)
    dy, dyd = torch.empty_like(y), torch.empty_like(yd)
    dg, db = _empty((c,), mean), _empty((c,), mean)
    dgd, dbd = _empty((c,), mean), _empty((c,), mean)
    call("tmr_bn_bwd_parts_ds", g, y, parts, int(nparts), mean, inv, gamma, dy, dg, db, yd, mean_d,
         inv_d, gamma_d, dyd, dgd, dbd, rows, c, int(t == BF16), ws, ctypes.c_size_t(ws.numel() * 8),
         stream_ptr())
    return dy, dg, db, dyd, dgd, dbd


def bn_bwd_parts(g, y, parts, nparts, mean, inv, gamma, bf16=False):
    """BN backward from conv_dgrad_bnbwd partials: g already masked -> (dy, dgamma, dbeta);
    bf16=True stores dy rounded (consumed only by the bf16-math dgrad / wgrad)."""
    c = y.shape[-1]
    rows = y.numel() // c
    nb = query("tmr_bn_parts_ws_bytes", int(nparts), c)
    ws = torch.empty(((nb + 7) // 8,), dtype=torch.float64, device=y.device)
    if y.dtype == BF16:   # bf16 activations: dy is bf16 too (g bf16 from a g16 dgrad, or fp32)
        dy = torch.empty_like(y)
        dgamma = _empty((c,), mean); dbeta = _empty((c,), mean)
        call("tmr_bn_bwd_parts_g16" if g.dtype == BF16 else "tmr_bn_bwd_parts_a16", g, y, parts,
             int(nparts), mean, inv, gamma, dy, dgamma, dbeta, rows, c, ws,
             ctypes.c_size_t(ws.numel() * 8), stream_ptr())
        return dy, dgamma, dbeta
    dy = torch.empty_like(y, dtype=torch.bfloat16 if bf16 else y.dtype)
    dgamma = _empty((c,), y); dbeta = _empty((c,), y)
    call("tmr_bn_bwd_parts_x", g, y, parts, int(nparts), mean, inv, gamma, dy, dgamma, dbeta, rows,
         c, ws, ctypes.c_size_t(ws.numel() * 8), int(bf16), stream_ptr())
    return dy, dgamma, dbeta


def conv_wgrad(x, dy, r, s, stride, pad, c_real=None, out=None, beta=0.0, pad_w=None,
               math="fp32", xpro=None, dpro=None, groups=1):
    """x (N,H,W,C), dy (N,Ho,Wo,K) -> dW (K, c_real, R, S) in OIHW (x/dy may be channel slices).
    xpro = (scale, shift): x read as relu(x*scale + shift); dpro = (y, coef): dy read as the BN
    backward A*dy + B*y + C.  groups: c_real = real input channels per group."""
    n, h, w, c = x.shape
    k = dy.shape[3]
    c_real = c // groups if c_real is None else c_real
    d = conv_desc(n, h, w, c, k, r, s, stride, pad, pad_w, math=math, io=_io(x, None, dy),
                  groups=groups)
    d.x_ld = _nhwc_ld(x, "x")
    d.y_ld = _nhwc_ld(dy, "dy")
    assert (d.ho, d.wo) == tuple(dy.shape[1:3])
    if out is None:
        out = _empty((k, c_real, r, s), x)
    ws_bytes = query("tmr_conv2d_wgrad_ws_bytes", ctypes.byref(d))
    ws = torch.empty(max(1, (ws_bytes + 3) // 4), dtype=f32, device=x.device)
    with _prof("conv_wgrad" + _SUFFIX[math], 2.0 * n * d.ho * d.wo * k * r * s * c_real,
               (n, h, w, c, k, r, stride),
               _esz(x) * n * h * w * c + _esz(dy) * n * d.ho * d.wo * k * (2 if dpro is not None else 1)
               + 4 * k * r * s * c_real):
        pro = _prologue(xpro, dpro)
        if pro is None:
            call("tmr_conv2d_wgrad", ctypes.byref(d), x, dy, out, int(c_real), float(beta), ws,
                 ctypes.c_size_t(ws.numel() * 4), stream_ptr())
        else:
            call("tmr_conv2d_wgrad_pro", ctypes.byref(d), x, dy, out, int(c_real), float(beta),
                 ws, ctypes.c_size_t(ws.numel() * 4), ctypes.byref(pro), stream_ptr())
    return out


def gemm_nt(a, b, bias=None, out=None, beta=0.0, M=None, N=None, K=None, lda=None, ldb=None,
            ldc=None):
    """out[M][N] = beta*out + a[M][K] @ b[N][K]^T (+bias)."""
    M = a.shape[0] if M is None else M
    K = a.shape[1] if K is None else K
    N = b.shape[0] if N is None else N
    lda = a.stride(0) if lda is None else lda
    ldb = b.stride(0) if ldb is None else ldb
    if out is None:
        out = _empty((M, N), a)
    ldc = out.stride(0) if ldc is None else ldc
    call("tmr_gemm_nt", M, N, K, a, lda, b, ldb, bias, out, ldc, float(beta), stream_ptr())
    return out


def gemm_nn(a, b, out=None, beta=0.0, M=None, N=None, K=None, lda=None, ldb=None, ldc=None):
    """out[M][N] = beta*out + a[M][K] @ b[K][N]."""
    M = a.shape[0] if M is None else M
    K = a.shape[1] if K is None else K
    N = b.shape[1] if N is None else N
    lda = a.stride(0) if lda is None else lda
    ldb = b.stride(0) if ldb is None else ldb
    if out is None:
        out = _empty((M, N), a)
    ldc = out.stride(0) if ldc is None else ldc
    call("tmr_gemm_nn", M, N, K, a, lda, b, ldb, out, ldc, float(beta), stream_ptr())
    return out


def gemm_tn(a, b, out=None, beta=0.0, M=None, N=None, K=None, lda=None, ldb=None, ldc=None):
    """out[M][N] = beta*out + a[K][M]^T @ b[K][N]."""
    K = a.shape[0] if K is None else K
    M = a.shape[1] if M is None else M
    N = b.shape[1] if N is None else N
    lda = a.stride(0) if lda is None else lda
    ldb = b.stride(0) if ldb is None else ldb
    if out is None:
        out = _empty((M, N), a)
    ldc = out.stride(0) if ldc is None else ldc
    call("tmr_gemm_tn", M, N, K, a, lda, b, ldb, out, ldc, float(beta), stream_ptr())
    return out


def col_sum(x, rows, cols, ld, out=None, beta=0.0):
    if out is None:
        out = _empty((cols,), x)
    call("tmr_col_sum", x, rows, cols, ld, out, float(beta), stream_ptr())
    return out


# --------------------------------------------------------------------- layout
# ---- weight layouts of a train step in one launch (round 5) ---------------------------------
# A trunk forward converts every conv weight (OIHW fp32) to its KRSC forward / CRSK dgrad operand,
# ~70 small launches a step.  Inside `layout_session(key)`, the first forward records the
# conversions it asks for (normal launches, outputs kept); every later forward with the same key
# refreshes all of them with one tmr_weight_layouts_multi launch at the session's start, and the
# weight_to_* calls return the refreshed tensors -- the same values (copies and RNE roundings).
# A request the record lacks (other weights, shapes, flags) is converted directly and the record
# is rebuilt on the next forward.
# Lifetime: records hang off their owner module (the trunk) in a weak table, so a
# model's converted copies are freed with it, and a new model can never reuse a dead one's record
# (its id() may be reused, its table would hold freed weight addresses).  Before every refresh the
# record checks that each parameter it was recorded from is alive at the same address; if not it
# re-records instead of reading stale pointers.  clear_layout_sessions() drops every record.
class _LayoutRecord:
    def __init__(self, owner):
        self.lookup = {}     # request key -> returned tensor
        self.rows = []       # table rows (w ptr, out tensor, k, c, rs, cpad, kind, bf16)
        self.table = None    # device table (uint8 bytes of _WL_DTYPE rows)
        self.blocks = 0
        self.valid = True
        # the owner's parameters at recording time: (weakref, data_ptr)
        self.sources = [(weakref.ref(p), p.data_ptr()) for p in owner.parameters()]

    def live(self):
        """Every source parameter alive at its recorded address (the table's pointers hold)."""
        for ref, ptr in self.sources:
            p = ref()
            if p is None or p.data_ptr() != ptr:
                return False
        return True


# owner module -> {(session key, thread): _LayoutRecord}: each thread refreshes its own copies;
# an exited thread's records go with `clear_layout_sessions` or the owner
_LAYOUTS = weakref.WeakKeyDictionary()
_TLS = threading.local()   # .session = [active record, recording?]


# include/tmr.h tmr_wlayout (56 bytes, no padding)
_WL_DTYPE = np.dtype([("w", "<u8"), ("out", "<u8"), ("n", "<i8"), ("block0", "<i8"),
                      ("k", "<i4"), ("c", "<i4"), ("rs", "<i4"), ("cpad", "<i4"),
                      ("kind", "<i4"), ("bf16", "<i4")])


def _session():
    st = getattr(_TLS, "session", None)
    if st is None:
        st = _TLS.session = [None, False]
    return st


LAYOUT_SESSIONS = True   # (the equality test turns it off for its reference run)


def clear_layout_sessions(owner=None):
    """Drop the recorded weight layouts (of `owner`, or of every module) and the converted
    copies they hold; the next forward records again."""
    if owner is None:
        _LAYOUTS.clear()
    else:
        _LAYOUTS.pop(owner, None)


def layout_session_count():
    """Records held (tests)."""
    return sum(len(v) for v in _LAYOUTS.values())


@contextlib.contextmanager
def layout_session(owner, key):
    """See above.  owner: the module whose parameters are converted (the trunk); key: one per
    mode and precision (the set of conversions it asks for)."""
    if not LAYOUT_SESSIONS:
        yield
        return
    recs = _LAYOUTS.get(owner)
    if recs is None:
        recs = _LAYOUTS[owner] = {}
    key = (key, threading.get_ident())
    rec = recs.get(key)
    recording = rec is None or not rec.valid or rec.table is None or not rec.live()
    if recording:
        rec = recs[key] = _LayoutRecord(owner)
    else:
        call("tmr_weight_layouts_multi", rec.table, len(rec.rows), rec.blocks, stream_ptr())
    st = _session()
    prev = list(st)
    st[0], st[1] = rec, recording
    try:
        yield
    finally:
        st[0], st[1] = prev
        if recording and rec.rows and rec.valid:
            epb = int(query("tmr_weight_layouts_epb"))
            tab = np.zeros(len(rec.rows), dtype=_WL_DTYPE)
            b0 = 0
            for j, (wp, out, k, c, rs, cpad, kind, b16) in enumerate(rec.rows):
                n = out.numel()
                tab[j] = (wp, out.data_ptr(), n, b0, k, c, rs, cpad, kind, b16)
                b0 += (n + epb - 1) // epb
            rec.table = torch.from_numpy(tab.view(np.uint8).copy()).to(rec.rows[0][1].device)
            rec.blocks = b0


def _layout(key, convert, rows):
    """The tensor for request `key`: from the active session's record when it holds it, else
    convert() (recorded with its table rows -- rows(out) -- when the session is recording)."""
    rec, recording = _session()
    if rec is None:
        return convert()
    out = rec.lookup.get(key)
    if out is not None and not recording:
        return out
    out = convert()
    if recording:
        rec.lookup[key] = out
        rec.rows.extend(rows(out))
    else:
        rec.valid = False   # a conversion the record lacks: re-record on the next forward
    return out


def weight_to_krsc(w, cpad=None, bf16=False):
    """OIHW fp32 -> KRSC (channels zero-padded to cpad); bf16=True stores it rounded (RNE), for
    the bf16-math convs (tmr_conv_desc.io TMR_IO_W_BF16)."""
    k, c, r, s = w.shape
    cpad = c if cpad is None else cpad
    _req(w, "w")

    def convert():
        out = _empty((k, r, s, cpad), w, dtype=torch.bfloat16 if bf16 else f32)
        call("tmr_weight_oihw_to_krsc_x", w, out, k, c, r, s, cpad, int(bf16), stream_ptr())
        return out
    return _layout((w.data_ptr(), "krsc", k, c, r * s, cpad, int(bf16)), convert,
                   lambda out: [(w.data_ptr(), out, k, c, r * s, cpad, 0, int(bf16))])


def weight_to_crsk(w, bf16=True):
    """OIHW fp32 -> the transposed dgrad operand (Cin, R, S, Cout): the weights of the LDS-DMA
    engine's dgrad view, bf16 (RNE; TMR_IO_WT_BF16) or fp32 (bf16=False; TMR_IO_WT_F32)."""
    k, c, r, s = w.shape
    _req(w, "w")

    def convert():
        out = _empty((c, r, s, k), w, dtype=torch.bfloat16 if bf16 else f32)
        call("tmr_weight_oihw_to_crsk_x", w, out, k, c, r, s, int(bf16), stream_ptr())
        return out
    return _layout((w.data_ptr(), "crsk", k, c, r * s, c, int(bf16)), convert,
                   lambda out: [(w.data_ptr(), out, k, c, r * s, c, 1, int(bf16))])


def weight_to_crsk_grouped(w, groups, bf16=True):
    """Grouped OIHW (K, C/G, R, S) -> the per-group transposed dgrad operand (G, C/G, R, S, K/G)."""
    k, cg, r, s = w.shape
    kg = k // groups
    _req(w, "w")

    def convert():
        out = _empty((groups, cg, r, s, kg), w, dtype=torch.bfloat16 if bf16 else f32)
        for g in range(groups):
            call("tmr_weight_oihw_to_crsk_x", w[g * kg:(g + 1) * kg], out[g], kg, cg, r, s,
                 int(bf16), stream_ptr())
        return out

    def rows(out):
        return [(w[g * kg:(g + 1) * kg].data_ptr(), out[g], kg, cg, r * s, cg, 1, int(bf16))
                for g in range(groups)]
    return _layout((w.data_ptr(), "crsk_g", k, cg, r * s, groups, int(bf16)), convert, rows)


def nhwc4_to_bf16x8(x4):
    """(F,H,W,4) fp32 NHWC4 stem input -> (F,H,W,8) bf16 (tmr_nhwc4_to_bf16x8): the bf16 step's
    stem operand (8-channel pieces for the LDS-DMA engine)."""
    _req(x4, "x4")
    if x4.dim() != 4 or x4.shape[3] != 4:
        raise RuntimeError("nhwc4_to_bf16x8: expects (F,H,W,4), got %s" % (tuple(x4.shape),))
    out = torch.empty(x4.shape[:3] + (8,), dtype=BF16, device=x4.device)
    call("tmr_nhwc4_to_bf16x8", x4, out, x4.numel() // 4, stream_ptr())
    return out


def to_bf16(x):
    """fp32 -> bf16 (RNE) copy (tmr_cast_f32_bf16): the bf16 conv operand of an fp32 tensor."""
    _req(x, "x")
    out = torch.empty_like(x, dtype=BF16)
    call("tmr_cast_f32_bf16", x, out, ctypes.c_long(x.numel()), stream_ptr())
    return out


def nchw_to_nhwc(x, cpad=None):
    n, c, h, w = x.shape
    cpad = c if cpad is None else cpad
    out = _empty((n, h, w, cpad), x)
    call("tmr_nchw_to_nhwc", _req(x, "x"), out, n, c, h, w, cpad, stream_ptr())
    return out


def nhwc_to_nchw(x, c=None):
    n, h, w, cs = x.shape
    c = cs if c is None else c
    out = _empty((n, c, h, w), x)
    call("tmr_nhwc_to_nchw", _req(x, "x"), out, n, c, cs, h, w, stream_ptr())
    return out


MEAN = (0.41757566, 0.26098573, 0.25888634)
STD = (0.21938758, 0.1983, 0.19342837)


def crop_normalize(frames_u8, offsets_i32, seq_len, crop=224, mean=MEAN, std=STD, out=None):
    """frames (F,Hin,Win,3) uint8, offsets (F/seq,2) int32 (x1,y1) -> (F,crop,crop,4) fp32 NHWC4."""
    _req(frames_u8, "frames", torch.uint8)
    _req(offsets_i32, "offsets", torch.int32)
    f, hin, win, _ = frames_u8.shape
    if out is None:
        out = _empty((f, crop, crop, 4), frames_u8)
    call("tmr_crop_normalize", frames_u8, offsets_i32, out, f, hin, win, seq_len, crop,
         *[float(v) for v in mean], *[float(v) for v in std], stream_ptr())
    return out


# ---------------------------------------------------------------- batch norm
def _bn_ws(rows, c, device):
    nb = query("tmr_bn_ws_bytes", rows, c)
    return torch.empty((nb + 7) // 8, dtype=torch.float64, device=device), nb


def bn_fwd_train(y2d, gamma, beta, running_mean, running_var, momentum, eps):
    rows, c = y2d.shape
    ws, nb = _bn_ws(rows, c, y2d.device)
    mean = _empty((c,), y2d); inv = _empty((c,), y2d)
    scale = _empty((c,), y2d); shift = _empty((c,), y2d)
    call("tmr_bn_fwd_stats", y2d, rows, c, gamma, beta, running_mean, running_var,
         float(momentum), float(eps), mean, inv, scale, shift, ws, ctypes.c_size_t(nb),
         stream_ptr())
    return mean, inv, scale, shift


def bn_eval_params(gamma, beta, running_mean, running_var, eps):
    c = running_mean.numel()
    scale = _empty((c,), running_mean); shift = _empty((c,), running_mean)
    call("tmr_bn_eval_params", gamma, beta, running_mean, running_var, float(eps), c, scale, shift,
         stream_ptr())
    return scale, shift


def bn_apply(y, scale, shift, residual=None, relu=True, out=None, bf16=False):
    """z = act(y*scale + shift (+ residual)); bf16=True stores z rounded (a tensor consumed only
    as a bf16-math conv operand)."""
    c = y.shape[-1]
    rows = y.numel() // c
    if y.dtype == BF16:   # bf16 activations: y, residual and z bf16
        if residual is not None and residual.dtype != BF16:
            raise RuntimeError("bn_apply: a bf16 y takes a bf16 residual")
        out = torch.empty_like(y) if out is None else out
        call("tmr_bn_apply_a16", y, scale, shift, residual, out, rows, c, int(relu), stream_ptr())
        return out
    if out is None:
        out = torch.empty_like(y, dtype=torch.bfloat16 if bf16 else y.dtype)
    call("tmr_bn_apply_x", y, scale, shift, residual, out, rows, c, int(relu),
         int(out.dtype == torch.bfloat16), stream_ptr())
    return out


def relu_bits_empty(like):
    """The ReLU-mask bit buffer of a tensor (tmr_bn_apply_bits): ceil(numel / 32) int32 words."""
    return torch.empty(((like.numel() + 31) // 32,), dtype=torch.int32, device=like.device)


def bn_apply_bits(y, scale, shift, residual=None):
    """Block output with ReLU: z = relu(y*scale + shift (+ residual)) and its ReLU mask as bits
    (tmr_bn_apply_bits, or _bits_a16 for bf16 activations: y, residual and z bf16) -> (z, bits),
    for the mask-3 residual-gradient dgrads."""
    _req(y, "y", y.dtype)
    c = y.shape[-1]
    z = torch.empty_like(y)
    bits = relu_bits_empty(y)
    if y.dtype == BF16:
        if residual is not None and residual.dtype != BF16:
            raise RuntimeError("bn_apply_bits: a bf16 y takes a bf16 residual")
        call("tmr_bn_apply_bits_a16", y, scale, shift, residual, z, bits, y.numel() // c, c,
             stream_ptr())
    else:
        call("tmr_bn_apply_bits", y, scale, shift, residual, z, bits, y.numel() // c, c,
             stream_ptr())
    return z, bits


def bn_apply2_bits(y, scale, shift, yr, rscale, rshift):
    """bn_apply2 with ReLU plus the ReLU mask as bits -> (z, bits); fp32, or bf16 y / yr / z."""
    _req(y, "y", y.dtype); _req(yr, "yr", y.dtype)
    if yr.shape != y.shape:
        raise RuntimeError("bn_apply2_bits: branch shape %s != %s" % (tuple(yr.shape), tuple(y.shape)))
    c = y.shape[-1]
    z = torch.empty_like(y)
    bits = relu_bits_empty(y)
    name = "tmr_bn_apply2_bits_a16" if y.dtype == BF16 else "tmr_bn_apply2_bits"
    call(name, y, scale, shift, yr, rscale, rshift, z, bits, y.numel() // c, c, stream_ptr())
    return z, bits


def bn_apply_dual(y, scale, shift, residual=None, relu=True):
    """bn_apply writing z in fp32 and a bf16 (RNE) copy in one pass -> (z, z16): a block output
    is the next block's identity residual (fp32) and its bf16-math convs' operand (bf16)."""
    c = y.shape[-1]
    rows = y.numel() // c
    z = torch.empty_like(y)
    z16 = torch.empty_like(y, dtype=torch.bfloat16)
    call("tmr_bn_apply_dual", y, scale, shift, residual, z, z16, rows, c, int(relu), stream_ptr())
    return z, z16


def bn_apply2(y, scale, shift, yr, rscale, rshift, relu=True, out=None, dual=False):
    """act(y*scale + shift + (yr*rscale + rshift)): BN3 + the downsample branch's BN + ReLU.
    dual=True -> (z, z16) with a bf16 copy (bn_apply_dual)."""
    c = y.shape[-1]
    rows = y.numel() // c
    if yr.shape != y.shape:
        raise RuntimeError("bn_apply2: branch shape %s != %s" % (tuple(yr.shape), tuple(y.shape)))
    if y.dtype == BF16:   # bf16 activations: y, yr and z bf16
        if yr.dtype != BF16 or dual:
            raise RuntimeError("bn_apply2: bf16 y takes a bf16 branch and writes one bf16 z")
        out = torch.empty_like(y) if out is None else out
        call("tmr_bn_apply2_a16", y, scale, shift, yr, rscale, rshift, out, rows, c, int(relu),
             stream_ptr())
        return out
    if out is None:
        out = torch.empty_like(y)
    z16 = torch.empty_like(y, dtype=torch.bfloat16) if dual else None
    call("tmr_bn_apply2_x", y, scale, shift, yr, rscale, rshift, out, z16, rows, c, int(relu),
         stream_ptr())
    return (out, z16) if dual else out


def bn_bwd(dz, y, z, mean, inv, gamma, relu, want_dres=False, dres_out=None, scale=None,
           shift=None, bf16=False):
    """ReLU mask from the saved output z, or (z=None) recomputed from y with the forward's
    scale/shift -- only valid when the forward had no residual.  bf16=True: dy stored rounded."""
    c = y.shape[-1]
    rows = y.numel() // c
    ws, nb = _bn_ws(rows, c, y.device)
    if y.dtype == BF16 and dz.dtype == BF16:
        # the bf16 residual-stream gradient into a BN without ReLU (the downsample branch)
        if relu or want_dres:
            raise RuntimeError("bn_bwd: a bf16 dz takes no ReLU mask / identity gradient")
        dy = torch.empty_like(y)
        dgamma = _empty((c,), mean); dbeta = _empty((c,), mean)
        call("tmr_bn_bwd_g16", dz, y, mean, inv, gamma, dy, dgamma, dbeta, rows, c, ws,
             ctypes.c_size_t(nb), stream_ptr())
        return dy, None, dgamma, dbeta
    if y.dtype == BF16:   # bf16 activations: y, z bf16; dz, dres fp32; dy bf16
        dy = torch.empty_like(y)
        dres = None
        if want_dres:
            dres = torch.empty_like(dz) if dres_out is None else dres_out
        dgamma = _empty((c,), dz); dbeta = _empty((c,), dz)
        call("tmr_bn_bwd_a16", dz, y, z if relu else None, scale, shift, mean, inv, gamma, dy, dres,
             dgamma, dbeta, rows, c, int(relu), ws, ctypes.c_size_t(nb), stream_ptr())
        return dy, dres, dgamma, dbeta
    dy = torch.empty_like(y, dtype=torch.bfloat16 if bf16 else y.dtype)
    dres = None
    if want_dres:
        dres = torch.empty_like(y) if dres_out is None else dres_out
    dgamma = _empty((c,), y); dbeta = _empty((c,), y)
    call("tmr_bn_bwd_x", dz, y, z if relu else None, scale, shift, mean, inv, gamma, dy, dres,
         dgamma, dbeta, rows, c, int(relu), ws, ctypes.c_size_t(nb), int(bf16), stream_ptr())
    return dy, dres, dgamma, dbeta


# ------------------------------------------------------------------- pooling
def maxpool_fwd(x):
    n, h, w, c = x.shape
    ho = (h + 2 - 3) // 2 + 1
    wo = (w + 2 - 3) // 2 + 1
    y = _empty((n, ho, wo, c), x)
    am = torch.empty((n, ho, wo, c), dtype=torch.uint8, device=x.device)
    call("tmr_maxpool2d_fwd", x, y, am, n, h, w, c, ho, wo, stream_ptr())
    return y, am


def maxpool_fwd_bn(x, scale, shift, bf16=False):
    """MaxPool2d(3,2,1)(relu(x*scale + shift)) with the BN+ReLU applied on load; bf16=True stores
    the output rounded (it is only a bf16-math conv operand)."""
    n, h, w, c = x.shape
    ho = (h + 2 - 3) // 2 + 1
    wo = (w + 2 - 3) // 2 + 1
    am = torch.empty((n, ho, wo, c), dtype=torch.uint8, device=x.device)
    if x.dtype == BF16:   # bf16 activations: the stem's bf16 y in, bf16 out
        y = _empty((n, ho, wo, c), x, dtype=BF16)
        call("tmr_maxpool2d_fwd_bn_a16", x, scale, shift, y, am, n, h, w, c, ho, wo, stream_ptr())
        return y, am
    y = _empty((n, ho, wo, c), x, dtype=torch.bfloat16 if bf16 else f32)
    call("tmr_maxpool2d_fwd_bn_x", x, scale, shift, y, am, n, h, w, c, ho, wo, int(bf16),
         stream_ptr())
    return y, am


def maxpool_bwd(dy, am, in_hw):
    n, ho, wo, c = dy.shape
    h, w = in_hw
    dx = _empty((n, h, w, c), dy)
    call("tmr_maxpool2d_bwd", dy, am, dx, n, h, w, c, ho, wo, stream_ptr())
    return dx


def avgpool_fwd(x):
    n, h, w, c = x.shape
    y = _empty((n, c), x)
    call("tmr_avgpool_fwd_a16" if x.dtype == BF16 else "tmr_avgpool_fwd", x, y, n, h * w, c,
         stream_ptr())
    return y


def avgpool_bwd(dy, hw):
    n, c = dy.shape
    h, w = hw
    dx = _empty((n, h, w, c), dy)
    call("tmr_avgpool_bwd", dy, dx, n, h * w, c, stream_ptr())
    return dx


# ----------------------------------------------------------------- head ops
def dropout_mask(n, p, seed, offset, like):
    m = _empty((n,), like)
    call("tmr_dropout_mask", m, n, float(p), ctypes.c_uint64(seed), ctypes.c_uint64(offset),
         stream_ptr())
    return m


def ce_sum(logits, labels, weight=None, gscale=1.0, want_grad=True):
    b, k = logits.shape
    loss = _empty((1,), logits)
    dl = _empty((b, k), logits) if want_grad else None
    preds = torch.empty((b,), dtype=torch.int64, device=logits.device)
    call("tmr_ce_sum", _req(logits, "logits"), _req(labels, "labels", torch.int64), weight, b, k,
         float(gscale), loss, dl, preds, stream_ptr())
    return loss, dl, preds


def softmax_max(logits):
    """(probs, max prob, argmax) of nn.Softmax(dim=1) + torch.max(., 1) over (B, K) logits."""
    _req(logits, "logits")
    b, k = logits.shape
    probs = _empty((b, k), logits)
    pmax = _empty((b,), logits)
    preds = torch.empty((b,), dtype=torch.int64, device=logits.device)
    call("tmr_softmax_max", logits, b, k, probs, pmax, preds, stream_ptr())
    return probs, pmax, preds


def sgd_step(p, g, buf, lr, momentum, dampening, weight_decay, nesterov, first_step):
    call("tmr_sgd_step", p, g, buf, p.numel(), float(lr), float(momentum), float(dampening),
         float(weight_decay), int(nesterov), int(first_step), stream_ptr())


def lfb_index(valid_starts_i64, clip_starts_i64, L):
    b = clip_starts_i64.numel()
    rows = torch.empty((b, L), dtype=torch.int32, device=clip_starts_i64.device)
    call("tmr_lfb_index", _req(valid_starts_i64, "valid_starts", torch.int64),
         valid_starts_i64.numel(), _req(clip_starts_i64, "clip_starts", torch.int64), b, L, rows,
         stream_ptr())
    return rows


def lfb_gather(bank, rows):
    d = bank.shape[1]
    out = _empty(tuple(rows.shape) + (d,), bank)
    call("tmr_lfb_gather", _req(bank, "bank"), _req(rows, "rows", torch.int32), out, rows.numel(),
         d, stream_ptr())
    return out


def layernorm_relu_fwd(x, gamma, beta, eps):
    rows, d = x.shape
    y = torch.empty_like(x)
    mean = _empty((rows,), x); rstd = _empty((rows,), x)
    call("tmr_layernorm_relu_fwd", x, gamma, beta, y, mean, rstd, rows, d, float(eps),
         stream_ptr())
    return y, mean, rstd


def layernorm_relu_bwd(dy, x, y, gamma, mean, rstd):
    rows, d = x.shape
    dx = torch.empty_like(x)
    dg = _empty((d,), x); db = _empty((d,), x)
    call("tmr_layernorm_relu_bwd", dy, x, y, gamma, mean, rstd, dx, dg, db, rows, d,
         stream_ptr())
    return dx, dg, db


def residual_mask(base, z, mask):
    out = torch.empty_like(base)
    call("tmr_residual_mask", base, z, mask, out, base.numel(), stream_ptr())
    return out


def mask_relu_fwd(h, mask):
    a = torch.empty_like(h)
    call("tmr_mask_relu_fwd", h, mask, a, h.numel(), stream_ptr())
    return a


def mask_relu_bwd(da, a, mask):
    dh = torch.empty_like(da)
    call("tmr_mask_relu_bwd", da, a, mask, dh, da.numel(), stream_ptr())
    return dh


def mul(a, b=None, scalar=None, out=None):
    out = torch.empty_like(a) if out is None else out
    call("tmr_mul", a, b, scalar, out, a.numel(), stream_ptr())
    return out


def _ws(nbytes, like):
    """Scratch / saved buffer for the module-level entry points (torch's caching allocator)."""
    return torch.empty(max(int(nbytes), 1), dtype=torch.uint8, device=like.device)


def nl_attn_fwd(lt, rows, u, B, L, scale):
    d = u.shape[1]
    p = _empty((B, L), u)
    ctx = _empty((B, d), u)
    ws = _ws(query("tmr_nl_attn_ws_bytes", B, L, d), u)
    call("tmr_nl_attn_fwd", lt, rows, u, p, ctx, B, L, d, float(scale), ws, ws.numel(),
         stream_ptr())
    return p, ctx


def nl_attn_bwd(lt, rows, u, p, dctx, B, L, scale, want_dlt):
    d = u.shape[1]
    ut = _empty((B, d), u)
    dlt = _empty((B, L, d), u) if want_dlt else None
    ws = _ws(query("tmr_nl_attn_ws_bytes", B, L, d), u)
    call("tmr_nl_attn_bwd", lt, rows, u, p, dctx, ut, dlt, B, L, d, float(scale), ws, ws.numel(),
         stream_ptr())
    return ut, dlt


# ------------------------------------------------------- module-level entry points
def _nl_ptrs(ts):
    from ._lib import NLBlockPtrs
    for t in ts:
        _req(t, "NLBlock parameter")
    return NLBlockPtrs(*[t.data_ptr() for t in ts])


def nlblock_fwd(st, lt, rows, L, mask, weights):
    """tmr_nlblock_fwd: weights = (w1, b1, w2, b2, w3, b3, ln_w, ln_b, w4, b4) (detached,
    contiguous).  Returns (out, saved)."""
    B = st.shape[0]
    _req(st, "St")
    _req(lt, "Lt")
    if rows is not None:
        _req(rows, "rows", torch.int32)
    out = _empty((B, 512), st)
    saved = _ws(query("tmr_nlblock_saved_bytes", B, L), st)
    ws = _ws(query("tmr_nlblock_ws_bytes", B, L), st)
    w = _nl_ptrs(weights)
    call("tmr_nlblock_fwd", ctypes.byref(w), st, lt, rows, B, L, mask, out, saved, saved.numel(),
         ws, ws.numel(), stream_ptr())
    return out, saved


def nlblock_bwd(dout, st, lt, rows, L, mask, saved, weights, want_dlt):
    """tmr_nlblock_bwd -> (dSt, dLt or None, [grads in weight order])."""
    B = st.shape[0]
    _req(dout, "dout")
    dst = _empty((B, 512), st)
    dlt = _empty((B, L, 512), st) if want_dlt else None
    grads = [torch.empty_like(t) for t in weights]
    ws = _ws(query("tmr_nlblock_ws_bytes", B, L), st)
    w = _nl_ptrs(weights)
    g = _nl_ptrs(grads)
    call("tmr_nlblock_bwd", ctypes.byref(w), dout, st, lt, rows, B, L, mask, saved, saved.numel(),
         dst, dlt, ctypes.byref(g), ws, ws.numel(), stream_ptr())
    return dst, dlt, grads


def timeconv_fwd(x, w3, b3, w5, b5, w7, b7):
    """tmr_timeconv_fwd: x (B,L,512) -> (out, saved max-branch codes)."""
    _req(x, "x")
    B, L, _ = x.shape
    out = torch.empty_like(x)
    saved = _ws(query("tmr_timeconv_saved_bytes", B, L), x)
    ws = _ws(query("tmr_timeconv_ws_bytes", B, L), x)
    for t in (w3, b3, w5, b5, w7, b7):
        _req(t, "TimeConv parameter")
    call("tmr_timeconv_fwd", x, B, L, w3, b3, w5, b5, w7, b7, out, saved, saved.numel(), ws,
         ws.numel(), stream_ptr())
    return out, saved


def timeconv_wgrad(dy, x, saved, w3, w5, w7, want_dx):
    """tmr_timeconv_wgrad -> (dx or None, dw3, db3, dw5, db5, dw7, db7)."""
    _req(dy, "dy")
    B, L, C = x.shape
    dx = torch.empty_like(x) if want_dx else None
    g = [torch.empty_like(w) for w in (w3, w5, w7)]
    bg = [_empty((C,), x) for _ in range(3)]
    ws = _ws(query("tmr_timeconv_ws_bytes", B, L), x)
    call("tmr_timeconv_wgrad", dy, x, B, L, w3, w5, w7, saved, saved.numel(), dx, g[0], bg[0],
         g[1], bg[1], g[2], bg[2], ws, ws.numel(), stream_ptr())
    return dx, g[0], bg[0], g[1], bg[1], g[2], bg[2]


def lstm_fwd(x, w_ih, w_hh, b_ih, b_hh, train=True):
    """tmr_lstm_fwd: x (B,T,I) -> (y (B,T,H), h_n (B,H), c_n (B,H), saved or None, ws)."""
    _req(x, "x")
    for t in (w_ih, w_hh, b_ih, b_hh):
        _req(t, "LSTM parameter")
    B, T, I = x.shape
    H = w_hh.shape[1]
    y = _empty((B, T, H), x)
    hn = _empty((B, H), x)
    cn = _empty((B, H), x)
    saved = _ws(query("tmr_lstm_saved_bytes", B, T, H), x) if train else None
    ws = _ws(query("tmr_lstm_ws_bytes", B, T, I, H), x)
    call("tmr_lstm_fwd", x, B, T, I, H, w_ih, w_hh, b_ih, b_hh, y, hn, cn, saved,
         saved.numel() if saved is not None else 0, ws, ws.numel(), stream_ptr())
    health.note_lstm(ws)   # a grid-barrier give-up is raised at the next optimizer step
    return y, hn, cn, saved, ws


def lstm_bwd(dy, x, w_ih, w_hh, y, saved, want_dx=True):
    """tmr_lstm_bwd -> (dx or None, dw_ih, dw_hh, db_ih, db_hh, ws)."""
    _req(dy, "dy")
    B, T, I = x.shape
    H = w_hh.shape[1]
    dx = torch.empty_like(x) if want_dx else None
    dw_ih, dw_hh = torch.empty_like(w_ih), torch.empty_like(w_hh)
    db_ih, db_hh = _empty((4 * H,), x), _empty((4 * H,), x)
    ws = _ws(query("tmr_lstm_ws_bytes", B, T, I, H), x)
    call("tmr_lstm_bwd", dy, x, B, T, I, H, w_ih, w_hh, y, saved, saved.numel(), dx, dw_ih, dw_hh,
         db_ih, db_hh, ws, ws.numel(), stream_ptr())
    health.note_lstm(ws)
    return dx, dw_ih, dw_hh, db_ih, db_hh, ws


def lstm_sync_status(ws):
    """Timeout word of the last persistent LSTM launch on `ws` (0 = all grid barriers done)."""
    v = ctypes.c_uint(0)
    call("tmr_lstm_sync_status", ws, ctypes.byref(v), stream_ptr())
    return v.value


def linear_fwd(x, w, b=None):
    _req(x, "x"); _req(w, "w")
    rows, i = x.shape
    o = w.shape[0]
    y = _empty((rows, o), x)
    call("tmr_linear_fwd", x, rows, i, o, w, b, y, stream_ptr())
    return y


def linear_bwd(dy, x, w, want_dx=True, want_db=True):
    _req(dy, "dy")
    rows, i = x.shape
    o = w.shape[0]
    dx = _empty((rows, i), x) if want_dx else None
    dw = torch.empty_like(w)
    db = _empty((o,), x) if want_db else None
    call("tmr_linear_bwd", dy, x, rows, i, o, w, dx, dw, db, 0.0, stream_ptr())
    return dx, dw, db


def lstm_cell_fwd(gx_t, ghh, c_prev, h_t, c_t, act_t=None):
    """gx_t (B,4H) row-strided view, h_t (B,H) row-strided view of y[:, t]; act_t None =
    inference (activations not saved)."""
    B, H = c_t.shape
    call("tmr_lstm_cell_fwd", gx_t, gx_t.stride(0), ghh, c_prev, h_t, h_t.stride(0), c_t, act_t,
         B, H, stream_ptr())


def lstm_cell_bwd(dh_out_t, dh_rec, dc_next, act_t, c_t, c_prev, dg_t, dc_prev):
    B, H = c_t.shape
    call("tmr_lstm_cell_bwd", dh_out_t, dh_out_t.stride(0), dh_rec, dc_next, act_t, c_t, c_prev,
         dg_t, dg_t.stride(0), dc_prev, B, H, stream_ptr())


# ------------------------------------------- ResNeSt split attention, bn0 applied on load
def _act16(y):
    if y.dtype not in (f32, BF16):
        raise RuntimeError("split attention: y must be fp32 or bf16, got %s" % y.dtype)
    return int(y.dtype == BF16)


def splat_gap_bn(y2, scale, shift):
    """gap[n][c] = mean_hw(x_0 + x_1), x_r = relu(bn0(y2_r)) recomputed (tmr_splat_gap_bn)."""
    _req(y2, "y2", y2.dtype)
    n, h, w, c2 = y2.shape
    gap = _empty((n, c2 // 2), y2)
    call("tmr_splat_gap_bn", y2, scale, shift, gap, n, h * w, c2 // 2, _act16(y2), stream_ptr())
    return gap


def splat_att(zl):
    """r-softmax over the radix pair of the fc2 logits zl (n, 2C) -> att (n, 2C)."""
    n, c2 = zl.shape
    att = torch.empty_like(zl)
    call("tmr_splat_att", _req(zl, "zl"), att, n, c2 // 2, stream_ptr())
    return att


def splat_combine_bn(y2, scale, shift, att):
    """out = att_0*x_0 + att_1*x_1 (dtype of y2) -> (n, h, w, C)."""
    _req(y2, "y2", y2.dtype)
    n, h, w, c2 = y2.shape
    out = torch.empty((n, h, w, c2 // 2), dtype=y2.dtype, device=y2.device)
    call("tmr_splat_combine_bn", y2, scale, shift, att, out, n, h * w, c2 // 2, _act16(y2),
         stream_ptr())
    return out


def splat_bwd_reduce_bn(dout, y2, scale, shift, mean, att):
    """-> (dzl (n, 2C), sums (4, n, 2C)) of tmr_splat_bwd_reduce_bn."""
    _req(dout, "dout"); _req(y2, "y2", y2.dtype)
    n, h, w, c2 = y2.shape
    if tuple(dout.shape) != (n, h, w, c2 // 2):
        raise RuntimeError("splat_bwd_reduce_bn: dout %s vs y2 %s" % (tuple(dout.shape), tuple(y2.shape)))
    dzl = _empty((n, c2), dout)
    sums = _empty((4, n, c2), dout)
    call("tmr_splat_bwd_reduce_bn", dout, y2, scale, shift, mean, att, dzl, sums, n, h * w, c2 // 2,
         _act16(y2), stream_ptr())
    return dzl, sums


def splat_bn0_coefs(att, dgap, sums, mean, inv, gamma, hw):
    """bn0 backward from the reduction sums -> (coef (3, 2C), dgamma, dbeta)."""
    n, c2 = att.shape
    coef = _empty((3, c2), att)
    dgamma = _empty((c2,), att); dbeta = _empty((c2,), att)
    call("tmr_splat_bn0_coefs", att, _req(dgap, "dgap"), sums, mean, inv, gamma, coef, dgamma, dbeta,
         n, hw, c2 // 2, stream_ptr())
    return coef, dgamma, dbeta


def splat_bwd_apply_bn(dout, y2, scale, shift, mean, att, dgap, coef):
    """dy2 (dtype of y2: the grouped conv's dgrad / wgrad operand) of tmr_splat_bwd_apply_bn."""
    n, h, w, c2 = y2.shape
    dy = torch.empty_like(y2)
    call("tmr_splat_bwd_apply_bn", dout, y2, scale, shift, mean, att, dgap, coef, dy, n, h * w,
         c2 // 2, _act16(y2), stream_ptr())
    return dy


def avgpool2d_fwd(x, k, s, p, count_include_pad, ceil_mode):
    """nn.AvgPool2d on NHWC fp32 or bf16 (bf16: fp32 sums, rounded output) -> (y, geometry)."""
    n, h, w, c = x.shape
    ho, wo = pool_out(h, k, s, p, ceil_mode), pool_out(w, k, s, p, ceil_mode)
    y = torch.empty((n, ho, wo, c), dtype=x.dtype, device=x.device)
    name = "tmr_avgpool2d_fwd_a16" if x.dtype == BF16 else "tmr_avgpool2d_fwd"
    call(name, _req(x, "x", x.dtype), y, n, h, w, c, ho, wo, k, s, p, int(count_include_pad),
         stream_ptr())
    return y


def avgpool2d_bwd(dy, in_hw, k, s, p, count_include_pad):
    """Gradient of avgpool2d_fwd (fp32) -> dx (n, h, w, c)."""
    n, ho, wo, c = dy.shape
    h, w = in_hw
    dx = _empty((n, h, w, c), dy)
    call("tmr_avgpool2d_bwd", _req(dy, "dy"), dx, n, h, w, c, ho, wo, k, s, p,
         int(count_include_pad), stream_ptr())
    return dx


def pool_out(h, k, s, p, ceil):
    """Output size of a pooling window (PyTorch's rule, incl. ceil_mode)."""
    if not ceil:
        return (h + 2 * p - k) // s + 1
    o = -(-(h + 2 * p - k) // s) + 1
    if (o - 1) * s >= h + p:   # last window must start inside the input
        o -= 1
    return o


# ------------------------------------------------------------------- bookkeeping
def zeros(shape, like):
    """fp32 zeros on like's device from libtmr's fill kernel."""
    out = torch.empty(shape, dtype=f32, device=like.device)
    call("tmr_fill_f32", out, ctypes.c_long(out.numel()), 0.0, stream_ptr())
    return out


# device pointer tables of counter sets, keyed by their addresses; the entry holds the counters
# themselves so their memory cannot be reused while the table points at it
_COUNTER_TABLES = {}


def counters_add_one(counters):
    """counters[i] += 1 for every int64 counter (BatchNorm num_batches_tracked) in one launch."""
    if not counters:
        return
    key = tuple(t.data_ptr() for t in counters)
    ent = _COUNTER_TABLES.get(key)
    if ent is None:
        for t in counters:
            _req(t, "counter", torch.int64)
        tab = torch.tensor(key, dtype=torch.int64).to(counters[0].device)
        ent = _COUNTER_TABLES[key] = (tab, list(counters))
    call("tmr_counters_add", ent[0], len(counters), 1, stream_ptr())
