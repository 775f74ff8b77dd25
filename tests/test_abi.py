"""CPU-side checks of the C-ABI boundary: the library loads, exports every
symbol include/ewvit.h declares, reports its ABI version, and rejects bad
arguments with an error message — no GPU compute is issued here."""
import ctypes
import os
import re

import pytest

from conftest import PKG, REPO

HEADER = os.path.join(REPO, 'include', 'ewvit.h')
LIB = os.path.join(PKG, 'ewvit', 'libewvit.so')


def declared_symbols():
    text = open(HEADER).read()
    return sorted(set(re.findall(r'\b(ewvit_[a-z0-9_]+)\s*\(', text)))


@pytest.fixture(scope='module')
def lib():
    if not os.path.exists(LIB):
        pytest.fail(f'{LIB} not built (run __graft_entry__.build())')
    return ctypes.CDLL(LIB)


def test_every_declared_symbol_is_exported(lib):
    syms = declared_symbols()
    assert len(syms) >= 12
    for s in syms:
        assert hasattr(lib, s), f'{s} declared in include/ewvit.h but not exported'


def test_python_binding_covers_the_header():
    from ewvit import _lib
    syms = set(declared_symbols()) - {'ewvit_abi_version', 'ewvit_last_error'}
    bound = set(_lib.SIGNATURES) | set(_lib.QUERIES)
    assert syms == bound, syms ^ bound


def test_abi_version(lib):
    lib.ewvit_abi_version.restype = ctypes.c_int
    from ewvit import _lib
    assert lib.ewvit_abi_version() == _lib.ABI_VERSION


def test_argument_errors_are_reported_without_gpu():
    from ewvit import _lib
    lib = _lib.load()
    # null operands -> EINVAL (1000) and a message; no HIP call is reached
    rc = lib.ewvit_dwt_haar_fwd(None, None, None, 1, 1, 8, 8, 1, 0, 0, None)
    assert rc == 1000
    assert b'null' in lib.ewvit_last_error()
    rc = lib.ewvit_dwt_haar_fwd(ctypes.c_void_p(16), ctypes.c_void_p(16), ctypes.c_void_p(16), 1, 1, 8, 8, 9, 0, 0, None)
    assert rc == 1000 and b'levels' in lib.ewvit_last_error()
    with pytest.raises(RuntimeError, match='unit stride'):
        _lib.call('ewvit_gemm', ctypes.c_void_p(16), 1, 7, 7, ctypes.c_void_p(16), 1, 1, 4,
                  ctypes.c_void_p(16), 0, 4, 4, 4, 4, 1.0, 0.0, None, 0, None, 0.0, 0, None, None, 0, 0, 1, None,
                  None)
    with pytest.raises(RuntimeError, match='nq=9'):
        _lib.call('ewvit_attn_fwd', ctypes.c_void_p(16), 0, 0, ctypes.c_void_p(16), 0, 0, ctypes.c_void_p(16),
                  0, 0, ctypes.c_void_p(16), 0, 0, None, 1, 1, 9, 2, 64, 1.0, None)


def test_ops_refuse_cpu_tensors():
    import torch
    import ewvit
    x = torch.randn(1, 3, 8, 8)
    with pytest.raises(RuntimeError, match='MI355X only'):
        ewvit.dwt_haar(x, 1)
    with pytest.raises(RuntimeError, match='MI355X only'):
        ewvit.linear(torch.randn(2, 4), torch.randn(3, 4))
