"""CPU tests of the drop-in boundary: libulg.so loads, exports every symbol
include/ulg.h declares, and refuses cleanly where there is no GPU."""
import ctypes
import os

import pytest

import ulg


def test_library_exports_every_header_symbol():
    L = ulg.lib()
    syms = ulg.header_symbols()
    assert len(syms) >= 10
    missing = [s for s in syms if not hasattr(L, s)]
    assert missing == []


def test_library_is_gfx950_code_object():
    # the fat binary must carry a gfx950 code object (no other targets)
    data = open(ulg.LIB_PATH, "rb").read()
    assert b"gfx950" in data


def test_version_string():
    assert b"gfx950" in ulg.lib().ulg_version()


def test_create_fails_loudly_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(ulg.ULGError):
        ulg.Context(0)


def test_bad_arguments_rejected_without_device():
    L = ulg.lib()
    h = ctypes.c_void_p()
    # ndev != 1 is an argument error, checked before touching HIP
    assert L.ulg_create((ctypes.c_int * 2)(0, 1), 2, ctypes.byref(h)) == 1
    assert L.ulg_create(None, 1, ctypes.byref(h)) == 1
