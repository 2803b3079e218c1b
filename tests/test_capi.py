"""The C ABI library: it loads without a GPU, exports every function include/nldpc.h declares,
and validates arguments on the host (no device compute here)."""
import ctypes
import os
import re

import pytest

from conftest import ROOT


def _declared():
    src = open(os.path.join(ROOT, "include", "nldpc.h")).read()
    return sorted(set(re.findall(r"^\s*(?:int|const char\*)\s+(nldpc_\w+)\s*\(", src, re.M)))


def test_header_lists_boundary():
    names = _declared()
    for n in ("nldpc_graph_create", "nldpc_forward", "nldpc_backward", "nldpc_ber_count", "nldpc_awgn_llr"):
        assert n in names


def test_library_exports_every_declared_symbol():
    from nldpc import _lib
    lib = _lib.lib()
    for name in _declared():
        assert hasattr(lib, name), name
    assert set(_lib.EXPORTED) == set(_declared())
    assert lib.nldpc_abi_version() == _lib.ABI_VERSION


def test_host_side_validation():
    from nldpc import _lib
    lib = _lib.lib()
    out = ctypes.c_void_p()
    tbl = (ctypes.c_int32 * 4)(0, -1, 1, 2)
    assert lib.nldpc_graph_create(0, 2, 4, tbl, 0, ctypes.byref(out)) == _lib.NLDPC_EINVAL
    assert b"positive" in lib.nldpc_last_error()
    bad = (ctypes.c_int32 * 4)(0, -2, 1, 2)
    assert lib.nldpc_graph_create(2, 2, 4, bad, 0, ctypes.byref(out)) == _lib.NLDPC_EINVAL
    with pytest.raises(ValueError):
        _lib.check(_lib.NLDPC_EINVAL, "x")
    assert lib.nldpc_forward(None, None, 1, 1, None, None, None, None, None, None, None, None, None, None,
                             None) == _lib.NLDPC_EINVAL
    counts = (ctypes.c_int64 * 2)()
    assert lib.nldpc_ber_count(None, None, 1, 1, 0, counts, None) == _lib.NLDPC_EINVAL
    assert lib.nldpc_awgn_llr(None, 1, 1, 1.0, 0, 0, 0, None) == _lib.NLDPC_EINVAL


def test_cfg_struct_layout_matches_header():
    from nldpc import _lib
    src = open(os.path.join(ROOT, "include", "nldpc.h")).read()
    body = re.search(r"typedef struct nldpc_cfg \{(.*?)\} nldpc_cfg;", src, re.S).group(1)
    fields = re.findall(r"^\s*(?:int32_t|float)\s+(\w+);", body, re.M)
    assert fields == [f for f, _ in _lib.NldpcCfg._fields_]
    assert ctypes.sizeof(_lib.NldpcCfg) == 4 * len(fields)
