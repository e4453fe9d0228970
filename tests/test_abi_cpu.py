"""The C-ABI library builds for gfx950, loads on a CPU-only host and exports every symbol that
include/tmr.h declares (no compute calls: those need a GPU)."""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "tmrnet_amd", "libtmr.so")


def header_symbols(name="tmr.h"):
    src = open(os.path.join(ROOT, "include", name)).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(tmr_[a-z0-9_]+)\s*\(", src)))


@pytest.fixture(scope="module")
def built():
    if not os.path.exists(LIB):
        subprocess.check_call(["make", "-j8"], cwd=ROOT)
    return LIB


def test_library_exports_every_declared_symbol(built):
    out = subprocess.check_output(["nm", "-D", "--defined-only", built]).decode()
    exported = set(l.split()[-1] for l in out.splitlines() if " T " in l)
    missing = [s for s in header_symbols() if s not in exported]
    assert not missing, missing


def test_python_binding_covers_header(built):
    from tmrnet_amd import _lib
    assert sorted(_lib.SIGNATURES) == header_symbols()
    assert sorted(_lib.PROLOGUE_SIGNATURES) == header_symbols("tmr_prologue.h")


def test_retired_prologues_absent_from_default_library(built):
    """The operand prologues (include/tmr_prologue.h, measured slower) are an A/B build only:
    the product library exports none of their entry points and the binding reports them absent."""
    from tmrnet_amd import _lib
    out = subprocess.check_output(["nm", "-D", "--defined-only", built]).decode()
    exported = set(l.split()[-1] for l in out.splitlines() if " T " in l)
    assert not set(header_symbols("tmr_prologue.h")) & exported
    if os.path.abspath(_lib.LIB_PATH) == os.path.abspath(built):
        assert not _lib.has_prologues()


def test_library_loads_and_reports_version(built):
    from tmrnet_amd import _lib
    h = _lib.lib()
    assert h.tmr_abi_version() == 8
    assert isinstance(h.tmr_last_error(), bytes)


def test_code_object_targets_gfx950(built):
    blob = open(built, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob
    for other in (b"--gfx942", b"--gfx90a", b"--gfx1100"):
        assert other not in blob


def test_argument_errors_raise_with_message(built):
    """Bad arguments come back as a non-zero status + tmr_last_error() text, raised by the
    binding as RuntimeError (include/tmr.h contract; checked before any device work)."""
    import ctypes
    from tmrnet_amd import _lib
    with pytest.raises(RuntimeError, match="null descriptor"):
        _lib.call("tmr_conv2d_fwd", None, None, None, None, None, 0.0, None)
    d = _lib.ConvDesc(2, 8, 8, 3, 16, 3, 3, 1, 1, 8, 8, 1, 0, 0, 0, 0)   # c=3: not a power of 2
    with pytest.raises(RuntimeError, match="power of two"):
        _lib.call("tmr_conv2d_fwd", ctypes.byref(d), None, None, None, None, 0.0, None)
    d.c, d.math = 4, 7
    with pytest.raises(RuntimeError, match="bad math mode"):
        _lib.call("tmr_conv2d_fwd", ctypes.byref(d), None, None, None, None, 0.0, None)
    with pytest.raises(RuntimeError, match="tmr_bn_ws_bytes"):
        _lib.query("tmr_bn_ws_bytes", 0, 64)
    with pytest.raises(RuntimeError, match="tmr_bn_parts_ws_bytes"):
        _lib.query("tmr_bn_parts_ws_bytes", -1, 64)
    with pytest.raises(RuntimeError, match="stats_parts"):
        _lib.query("tmr_conv2d_fwd_stats_parts", None)
    with pytest.raises(RuntimeError, match="wgrad_ws_bytes"):
        _lib.query("tmr_conv2d_wgrad_ws_bytes", None)
    # module-level entry points: size queries and null operands fail before any device work
    for q, args in (("tmr_lstm_ws_bytes", (4, 10, 2048, 0)), ("tmr_lstm_saved_bytes", (-1, 10, 512)),
                    ("tmr_nlblock_ws_bytes", (4, 0)), ("tmr_nlblock_saved_bytes", (-2, 40)),
                    ("tmr_timeconv_ws_bytes", (4, 0)), ("tmr_nl_attn_ws_bytes", (4, 40, 300))):
        with pytest.raises(RuntimeError, match=q):
            _lib.query(q, *args)
    with pytest.raises(RuntimeError, match="tmr_lstm_fwd: bad sizes"):
        _lib.call("tmr_lstm_fwd", None, 2, 3, 0, 512, *([None] * 7), None, 0, None, 0, None)
    with pytest.raises(RuntimeError, match="tmr_lstm_fwd: null operand"):
        _lib.call("tmr_lstm_fwd", None, 2, 3, 64, 512, *([None] * 7), None, 0, None, 0, None)
    with pytest.raises(RuntimeError, match="tmr_nlblock_fwd: null operand"):
        _lib.call("tmr_nlblock_fwd", None, None, None, None, 2, 40, None, None, None, 0, None, 0,
                  None)
    with pytest.raises(RuntimeError, match="tmr_timeconv_wgrad: null operand"):
        _lib.call("tmr_timeconv_wgrad", *([None] * 2), 2, 30, *([None] * 4), 0, *([None] * 8), 0,
                  None)
    with pytest.raises(RuntimeError, match="tmr_linear_fwd: bad sizes"):
        _lib.call("tmr_linear_fwd", None, 4, 0, 8, None, None, None, None)
    with pytest.raises(RuntimeError, match="feature dim"):
        _lib.call("tmr_nl_attn_fwd", None, None, None, None, None, 2, 40, 300, 1.0, None, 0, None)
    # a good query after a failure is not poisoned by the old message
    assert _lib.query("tmr_bn_ws_bytes", 1024, 64) > 0
    assert _lib.query("tmr_lstm_ws_bytes", 64, 10, 2048, 512) > 0


def test_stem_entry_points_host_checks(built):
    """The direct stem's host-side contract (no GPU work): the wgrad workspace query covers the
    direct kernel's 512 partial slabs at the stem geometry (direct or on the engine), and
    the fused stem entries refuse other geometries / null operands before any launch."""
    import ctypes
    from tmrnet_amd import _lib, ops
    d = ops.conv_desc(640, 224, 224, 4, 64, 7, 7, 2, 3)
    assert _lib.query("tmr_conv2d_wgrad_ws_bytes", ctypes.byref(d)) >= 512 * 64 * 49 * 4 * 4
    # the bf16 stem's (stem16.hip) slabs: 768 persistent workgroups
    d16 = ops.conv_desc(640, 224, 224, 4, 64, 7, 7, 2, 3, math="bf16", io=ops.IO_DY)
    assert _lib.query("tmr_conv2d_wgrad_ws_bytes", ctypes.byref(d16)) >= 768 * 64 * 49 * 4 * 4


def test_grouped_bf16_accumulating_dgrad_rejected():
    """A grouped fused dgrad cannot accumulate (beta != 0) into a bf16 gradient: the
    wrapper raises before any library call (the C entry point rejects it too, gemm_conv.hip)."""
    import torch
    from tmrnet_amd import ops
    dy = torch.zeros(1, 4, 4, 16, dtype=torch.bfloat16)
    y = torch.zeros(1, 4, 4, 16, dtype=torch.bfloat16)
    with pytest.raises(RuntimeError, match="grouped dgrad accumulates"):
        ops.conv_dgrad_bnbwd(dy, torch.zeros(16, 3, 3, 8), (4, 4), 1, 1, y, torch.zeros(16), 2,
                             scale=torch.ones(16), shift=torch.zeros(16), out=y, beta=1.0,
                             math="bf16", wt=True, groups=2, g16=True)
