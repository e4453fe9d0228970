"""ctypes binding of libtmr.so, the C-ABI kernel library (include/tmr.h).

The product path has no fallback: if the library is missing or a call fails,
this raises.  ``call(name, *args)`` converts torch tensors to device pointers,
checks the returned status and raises ``RuntimeError(tmr_last_error())``.
"""
import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("TMR_LIB_PATH") or os.path.join(_HERE, "libtmr.so")  # override: experiments

P = ctypes.c_void_p
I = ctypes.c_int
L = ctypes.c_long
F = ctypes.c_float
U64 = ctypes.c_uint64
SZ = ctypes.c_size_t


class ConvDesc(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int) for n in
                ("n", "h", "w", "c", "k", "r", "s", "stride", "pad", "ho", "wo", "pad_w",
                 "x_ld", "y_ld", "math", "max_frames", "io", "groups")]


DP = ctypes.POINTER(ConvDesc)


class ConvPrologue(ctypes.Structure):
    """tmr_conv_prologue: BN(+ReLU) of the X operand / BN backward of the dY operand on load."""
    _fields_ = [(n, ctypes.c_void_p) for n in ("x_scale", "x_shift", "dy_y", "dy_coef")]


PP = ctypes.POINTER(ConvPrologue)

_NL_FIELDS = ("w1", "b1", "w2", "b2", "w3", "b3", "ln_w", "ln_b", "w4", "b4")


class NLBlockPtrs(ctypes.Structure):
    """tmr_nlblock_weights / tmr_nlblock_grads: ten device pointers in NLBlock parameter order."""
    _fields_ = [(n, ctypes.c_void_p) for n in _NL_FIELDS]

# name -> argtypes (restype is int unless listed in _RESTYPES)
SIGNATURES = {
    "tmr_abi_version": [],
    "tmr_last_error": [],
    "tmr_clear_error": [],
    "tmr_conv2d_fwd": [DP, P, P, P, P, F, P],
    "tmr_conv2d_fwd_fused": [DP, P, P, P, P, P, P, I, P],
    "tmr_conv2d_fwd_stats_parts": [DP],
    "tmr_conv2d_fwd_bnstats": [DP, P, P, P, P, SZ, P],
    "tmr_conv2d_dgrad": [DP, P, P, P, F, P],
    "tmr_conv2d_dgrad_bnbwd_parts": [DP],
    "tmr_conv2d_dgrad_bnbwd": [DP, P, P, P, F, P, P, P, P, P, I, P, SZ, P],
    "tmr_conv2d_wgrad_ws_bytes": [DP],
    "tmr_conv2d_wgrad": [DP, P, P, P, I, F, P, SZ, P],
    "tmr_conv2d_dgrad_bnbwd_acc": [DP, P, P, P, F, P, I, P, P, P, P, P, I, P, SZ, P],
    "tmr_bn_apply_x": [P, P, P, P, P, I, I, I, I, P],
    "tmr_bn_bwd_parts_x": [P, P, P, I, P, P, P, P, P, P, I, I, P, SZ, I, P],
    "tmr_bn_bwd_x": [P, P, P, P, P, P, P, P, P, P, P, P, I, I, I, P, SZ, I, P],
    "tmr_bn_bwd_maxpool_x": [P, P, I, I, I, I, I, P, P, P, P, P, P, P, P, P, I, P, SZ, I, P],
    "tmr_weight_oihw_to_krsc_x": [P, P, I, I, I, I, I, I, P],
    "tmr_weight_oihw_to_crsk_x": [P, P, I, I, I, I, I, P],
    "tmr_bn_apply_dual": [P, P, P, P, P, P, I, I, I, P],
    "tmr_bn_apply2_x": [P, P, P, P, P, P, P, P, I, I, I, P],
    "tmr_bn_apply_bits": [P, P, P, P, P, P, I, I, P],
    "tmr_bn_apply2_bits": [P, P, P, P, P, P, P, P, I, I, P],
    "tmr_maxpool2d_fwd_bn_x": [P, P, P, P, P, I, I, I, I, I, I, I, P],
    "tmr_bn_apply_a16": [P, P, P, P, P, I, I, I, P],
    "tmr_bn_apply2_a16": [P, P, P, P, P, P, P, I, I, I, P],
    "tmr_bn_apply_bits_a16": [P, P, P, P, P, P, I, I, P],
    "tmr_bn_apply2_bits_a16": [P, P, P, P, P, P, P, P, I, I, P],
    "tmr_bn_bwd_a16": [P, P, P, P, P, P, P, P, P, P, P, P, I, I, I, P, SZ, P],
    "tmr_bn_bwd_parts_a16": [P, P, P, I, P, P, P, P, P, P, I, I, P, SZ, P],
    "tmr_bn_bwd_parts_g16": [P, P, P, I, P, P, P, P, P, P, I, I, P, SZ, P],
    "tmr_bn_bwd_g16": [P, P, P, P, P, P, P, P, I, I, P, SZ, P],
    "tmr_weight_layouts_epb": [],
    "tmr_weight_layouts_multi": [P, I, I, P],
    "tmr_bn_bwd_parts_ds_ws_bytes": [I, I, I],
    "tmr_bn_bwd_parts_ds": [P, P, P, I, P, P, P, P, P, P, P, P, P, P, P, P, P, I, I, I, P, SZ, P],
    "tmr_bn_bwd_maxpool_a16": [P, P, I, I, I, I, I, P, P, P, P, P, P, P, P, P, I, P, SZ, P],
    "tmr_maxpool2d_fwd_bn_a16": [P, P, P, P, P, I, I, I, I, I, I, P],
    "tmr_avgpool_fwd_a16": [P, P, I, I, I, P],
    "tmr_cast_f32_bf16": [P, P, ctypes.c_long, P],
    "tmr_nhwc4_to_bf16x8": [P, P, ctypes.c_long, P],
    "tmr_adam_step_multi": [P, I, ctypes.c_int64, P, P],
    "tmr_resize_ksize": [I, I],
    "tmr_resize_coeffs": [I, I, P, P, I],
    "tmr_resize_tmp_bytes": [I, I, I, I, I],
    "tmr_resize_u8": [P, I, I, I, P, SZ, P, I, I, P, P, I, P, P, I, I, I, P],
    "tmr_gemm_nt": [I, I, I, P, I, P, I, P, P, I, F, P],
    "tmr_gemm_nn": [I, I, I, P, I, P, I, P, I, F, P],
    "tmr_gemm_tn": [I, I, I, P, I, P, I, P, I, F, P],
    "tmr_weight_oihw_to_krsc": [P, P, I, I, I, I, I, P],
    "tmr_nchw_to_nhwc": [P, P, I, I, I, I, I, P],
    "tmr_nhwc_to_nchw": [P, P, I, I, I, I, I, P],
    "tmr_clip_augment": [P, P, P, P, I, I, I, I, F, F, F, F, F, F, P],
    "tmr_crop_normalize": [P, P, P, I, I, I, I, I, F, F, F, F, F, F, P],
    "tmr_bn_ws_bytes": [I, I],
    "tmr_bn_fwd_stats": [P, I, I, P, P, P, P, F, F, P, P, P, P, P, SZ, P],
    "tmr_bn_finalize": [P, I, I, P, P, P, P, F, F, P, P, P, P, P],
    "tmr_bn_finalize_ws": [P, I, I, P, P, P, P, F, F, P, P, P, P, P, SZ, P],
    "tmr_bn_parts_ws_bytes": [I, I],
    "tmr_bn_eval_params": [P, P, P, P, F, I, P, P, P],
    "tmr_bn_apply": [P, P, P, P, P, I, I, I, P],
    "tmr_bn_apply2": [P, P, P, P, P, P, P, I, I, I, P],
    "tmr_bn_bwd_parts": [P, P, P, I, P, P, P, P, P, P, I, I, P, SZ, P],
    "tmr_bn_bwd_maxpool": [P, P, I, I, I, I, I, P, P, P, P, P, P, P, P, P, I, P, SZ, P],
    "tmr_bn_bwd": [P, P, P, P, P, P, P, P, P, P, P, P, I, I, I, P, SZ, P],
    "tmr_maxpool2d_fwd": [P, P, P, I, I, I, I, I, I, P],
    "tmr_maxpool2d_fwd_bn": [P, P, P, P, P, I, I, I, I, I, I, P],
    "tmr_maxpool2d_bwd": [P, P, P, I, I, I, I, I, I, P],
    "tmr_avgpool_fwd": [P, P, I, I, I, P],
    "tmr_avgpool_bwd": [P, P, I, I, I, P],
    "tmr_splat_gap": [P, P, I, I, I, P],
    "tmr_splat_combine": [P, P, P, P, I, I, I, P],
    "tmr_splat_bwd": [P, P, P, P, I, I, I, P],
    "tmr_splat_bwd_apply": [P, P, P, P, I, I, I, P],
    "tmr_splat_gap_bn": [P, P, P, P, I, I, I, I, P],
    "tmr_splat_att": [P, P, I, I, P],
    "tmr_splat_combine_bn": [P, P, P, P, P, I, I, I, I, P],
    "tmr_splat_bwd_reduce_bn": [P, P, P, P, P, P, P, P, I, I, I, I, P],
    "tmr_splat_bn0_coefs": [P, P, P, P, P, P, P, P, P, I, I, I, P],
    "tmr_splat_bwd_apply_bn": [P, P, P, P, P, P, P, P, P, I, I, I, I, P],
    "tmr_avgpool2d_fwd_a16": [P, P, I, I, I, I, I, I, I, I, I, I, P],
    "tmr_fill_f32": [P, L, F, P],
    "tmr_seq_last": [P, P, I, I, I, P],
    "tmr_seq_last_bwd": [P, P, P, I, I, I, P],
    "tmr_counters_add": [P, I, ctypes.c_int64, P],
    "tmr_center_cols": [P, I, I, P, P, P],
    "tmr_axpy": [I, F, P, P, P],
    "tmr_avgpool2d_fwd": [P, P, I, I, I, I, I, I, I, I, I, I, P],
    "tmr_avgpool2d_bwd": [P, P, I, I, I, I, I, I, I, I, I, I, P],
    "tmr_col_sum": [P, I, I, I, P, F, P],
    "tmr_dropout_mask": [P, L, F, U64, U64, P],
    "tmr_softmax_max": [P, I, I, P, P, P, P],
    "tmr_ce_sum": [P, P, P, I, I, F, P, P, P, P],
    "tmr_sgd_chunk": [],
    "tmr_sgd_step_multi": [P, I, ctypes.c_int64, P, P],
    "tmr_sgd_step": [P, P, P, L, F, F, F, F, I, I, P],
    "tmr_lfb_index": [P, I, P, I, I, P, P],
    "tmr_lfb_gather": [P, P, P, L, I, P],
    "tmr_layernorm_relu_fwd": [P, P, P, P, P, P, I, I, F, P],
    "tmr_layernorm_relu_bwd": [P, P, P, P, P, P, P, P, P, I, I, P],
    "tmr_residual_mask": [P, P, P, P, L, P],
    "tmr_mask_relu_fwd": [P, P, P, L, P],
    "tmr_mask_relu_bwd": [P, P, P, P, L, P],
    "tmr_mul": [P, P, P, P, L, P],
    "tmr_nl_attn_ws_bytes": [I, I, I],
    "tmr_nl_attn_fwd": [P, P, P, P, P, I, I, I, F, P, SZ, P],
    "tmr_nl_attn_bwd": [P, P, P, P, P, P, P, I, I, I, F, P, SZ, P],
    "tmr_linear_fwd": [P, I, I, I, P, P, P, P],
    "tmr_linear_bwd": [P, P, I, I, I, P, P, P, P, F, P],
    "tmr_nlblock_saved_bytes": [I, I],
    "tmr_nlblock_ws_bytes": [I, I],
    "tmr_nlblock_fwd": [P, P, P, P, I, I, P, P, P, SZ, P, SZ, P],
    "tmr_nlblock_bwd": [P, P, P, P, P, I, I, P, P, SZ, P, P, P, P, SZ, P],
    "tmr_timeconv_saved_bytes": [I, I],
    "tmr_timeconv_ws_bytes": [I, I],
    "tmr_timeconv_fwd": [P, I, I, P, P, P, P, P, P, P, P, SZ, P, SZ, P],
    "tmr_timeconv_wgrad": [P, P, I, I, P, P, P, P, SZ, P, P, P, P, P, P, P, P, SZ, P],
    "tmr_lstm_saved_bytes": [I, I, I],
    "tmr_lstm_ws_bytes": [I, I, I, I],
    "tmr_lstm_fwd": [P, I, I, I, I, P, P, P, P, P, P, P, P, SZ, P, SZ, P],
    "tmr_lstm_bwd": [P, P, I, I, I, I, P, P, P, P, SZ, P, P, P, P, P, P, SZ, P],
    "tmr_lstm_sync_status": [P, ctypes.POINTER(ctypes.c_uint), P],
    "tmr_lstm_status_or": [P, P, P],
    "tmr_test_hold_cus": [I, F, P],
    "tmr_dgrad_ws_launches": [],
    "tmr_timeconv_max5_fwd": [P, P, P, P, P, P, I, I, I, P],
    "tmr_timeconv_max5_bwd": [P, P, P, P, P, P, I, I, I, P],
    "tmr_lstm_cell_fwd": [P, I, P, P, P, I, P, P, I, I, P],
    "tmr_lstm_cell_bwd": [P, I, P, P, P, P, P, P, I, P, I, I, P],
}
# include/tmr_prologue.h: the retired operand-prologue experiment, bound only when the loaded
# library is the A/B build (`make PROLOGUES=1` -> libtmr_pro.so)
PROLOGUE_SIGNATURES = {
    "tmr_conv2d_fwd_bnstats_pro": [DP, P, P, P, P, SZ, PP, P],
    "tmr_conv2d_dgrad_pro": [DP, P, P, P, F, PP, P],
    "tmr_conv2d_dgrad_bnbwd_pro": [DP, P, P, P, F, P, P, P, P, P, I, P, SZ, PP, P],
    "tmr_conv2d_wgrad_pro": [DP, P, P, P, I, F, P, SZ, PP, P],
    "tmr_bn_bwd_coefs": [P, I, P, P, P, P, P, P, I, I, P, SZ, P],
    "tmr_bn_bwd_coefs_dense": [P, P, P, P, P, P, P, P, P, P, P, I, I, I, P, SZ, P],
    "tmr_conv2d_dgrad_bnbwd_acc_pro": [DP, P, P, P, F, P, I, P, P, P, P, P, I, P, SZ, PP, P],
    "tmr_bn_bwd_coefs_g16": [P, P, P, P, P, P, P, P, I, I, P, SZ, P],
}
_RESTYPES = {
    "tmr_last_error": ctypes.c_char_p,
    "tmr_clear_error": None,
    "tmr_conv2d_wgrad_ws_bytes": SZ,
    "tmr_dgrad_ws_launches": L,
    "tmr_resize_tmp_bytes": SZ,
    "tmr_bn_ws_bytes": SZ,
    "tmr_bn_parts_ws_bytes": SZ,
    "tmr_bn_bwd_parts_ds_ws_bytes": SZ,
    "tmr_sgd_chunk": ctypes.c_int64,
    "tmr_nl_attn_ws_bytes": SZ,
    "tmr_nlblock_saved_bytes": SZ,
    "tmr_nlblock_ws_bytes": SZ,
    "tmr_timeconv_saved_bytes": SZ,
    "tmr_timeconv_ws_bytes": SZ,
    "tmr_lstm_saved_bytes": SZ,
    "tmr_lstm_ws_bytes": SZ,
}

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                "libtmr.so not found at %s: build it with `make` or "
                "`python -c 'import __graft_entry__ as g; g.build()'` (no CPU fallback exists)"
                % LIB_PATH)
        h = ctypes.CDLL(LIB_PATH)
        for name, args in SIGNATURES.items():
            fn = getattr(h, name)
            fn.argtypes = args
            fn.restype = _RESTYPES.get(name, ctypes.c_int)
        for name, args in PROLOGUE_SIGNATURES.items():
            if hasattr(h, name):
                fn = getattr(h, name)
                fn.argtypes = args
                fn.restype = ctypes.c_int
        _lib = h
    return _lib


def has_prologues():
    """True when the loaded library is the operand-prologue A/B build (include/tmr_prologue.h)."""
    return all(hasattr(lib(), n) for n in PROLOGUE_SIGNATURES)


def exported_symbols():
    return list(SIGNATURES)


def _conv(a):
    if isinstance(a, torch.Tensor):
        return ctypes.c_void_p(a.data_ptr())
    return a


def stream_ptr(device=None):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def call(name, *args):
    fn = getattr(lib(), name)
    rc = fn(*[_conv(a) for a in args])
    if rc != 0:
        raise RuntimeError("%s failed (%d): %s" % (name, rc, lib().tmr_last_error().decode()))
    return rc


def query(name, *args):
    """Size / count queries (workspace bytes, partial-row counts).  Integer queries report a
    bad argument as a negative value; size queries as 0 with tmr_last_error set -- both raise."""
    h = lib()
    h.tmr_clear_error()
    fn = getattr(h, name)
    v = fn(*[_conv(a) for a in args])
    err = h.tmr_last_error()
    if (_RESTYPES.get(name, ctypes.c_int) is ctypes.c_int and v < 0) or err:
        raise RuntimeError("%s failed (%d): %s" % (name, v, (err or b"").decode()))
    return v
