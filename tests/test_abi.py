"""CPU: the C-ABI library builds, loads and exports every symbol the headers
declare; without a GPU it fails loudly (there is no CPU path)."""
import ctypes
import os
import re

import pytest
from conftest import ROOT

import sstcodec
from sstcodec import _lib


def declared_functions(header):
    src = open(header).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    src = re.sub(r"//[^\n]*", "", src)
    names = re.findall(r"^[A-Za-z_][\w \*]*?\b(\w+)\s*\(", src, flags=re.M)
    return sorted({n for n in names if not n.startswith("SSTC_") and n not in ("if", "defined")})


def test_library_built():
    assert os.path.exists(_lib.LIB_PATH), "run lsm-kv-storage_amd/build.py"


def test_exports_every_declared_symbol():
    lib = ctypes.CDLL(_lib.LIB_PATH)
    names = declared_functions(os.path.join(ROOT, "include", "sstcodec.h"))
    assert "sstc_roundtrip_blocks" in names and len(names) >= 13
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing


def test_host_table_symbols():
    hdr = os.path.join(ROOT, "include", "sstc_table.h")
    if not os.path.exists(hdr):
        pytest.skip("no host table header")
    lib = ctypes.CDLL(_lib.LIB_PATH)
    names = [n for n in declared_functions(hdr) if n.startswith("sstc_")]
    missing = [n for n in names if not hasattr(lib, n)]
    assert names and not missing, missing


def test_version():
    assert _lib.load().sstc_version() == 1


def test_no_gpu_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    h = ctypes.c_void_p()
    rc = _lib.load().sstc_ctx_create(0, None, ctypes.byref(h))
    assert rc == -4  # SSTC_E_NO_DEVICE
    assert b"no HIP device" in _lib.load().sstc_last_error_string()
    with pytest.raises(Exception):
        sstcodec.Codec(0)
