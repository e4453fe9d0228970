"""The C-ABI library builds for gfx950, loads on a CPU-only host and exports every symbol that
include/tmr.h declares (no compute calls: those need a GPU)."""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "tmrnet_amd", "libtmr.so")


def header_symbols():
    src = open(os.path.join(ROOT, "include", "tmr.h")).read()
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


def test_library_loads_and_reports_version(built):
    from tmrnet_amd import _lib
    h = _lib.lib()
    assert h.tmr_abi_version() == 1
    assert isinstance(h.tmr_last_error(), bytes)


def test_code_object_targets_gfx950(built):
    blob = open(built, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob
    for other in (b"--gfx942", b"--gfx90a", b"--gfx1100"):
        assert other not in blob
