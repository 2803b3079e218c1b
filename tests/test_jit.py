"""Run-time kernels for lifting sizes the library was not built for (nldpc.jit, csrc/gen_fused.py
jit_source), on the CPU: every 5G NR base-graph-2 lifting size has a register-resident
geometry and generates, and one kernel compiles into a gfx950 code object with the entry point the
library attaches (the GPU tests run them: tests/test_gpu_forward.py)."""
import os

import numpy as np
import pytest

from conftest import ROOT

BG2 = np.loadtxt(os.path.join(ROOT, "resources", "basegraph2_set0.txt"), int, delimiter="\t")
# TS 38.212 Table 5.3.2-1: the lifting sizes (every a x 2^j up to 384)
NR_Z = sorted({a * 2 ** j for a in (2, 3, 5, 7, 9, 11, 13, 15) for j in range(8) if a * 2 ** j <= 384})


def _gen():
    from nldpc import jit
    return jit._generator()


def test_every_nr_lifting_size_has_a_geometry():
    gen = _gen()
    assert len(NR_Z) == 51
    for Z in NR_Z:
        G, P, Q = gen.auto_geometry(BG2, Z)
        S = gen.Spec("t", BG2, Z, G, P, Q, sched="pipe2")
        assert S.threads <= 1024 and S.lanes_pad % 64 == 0 and (S.lanes_pad - S.lanes) * 4 <= S.lanes_pad, Z
        assert max(len(s) for s in S.slots) * Q <= gen.MAX_STATE_REGS, Z


@pytest.mark.parametrize("Z", [2, 13, 52, 104, 208, 320])
def test_jit_source_generates(Z):
    gen = _gen()
    for mode in (0, 4):
        src, geo = gen.jit_source(BG2, Z, 3, mode)
        entry = "nldpc_fxb" if mode == 4 else "nldpc_fx"
        assert f'extern "C" __global__' in src and f"void {entry}(" in src
        assert geo["threads"] <= 1024 and geo["threads"] % 64 == 0


def test_jit_compiles_a_code_object(tmp_path, monkeypatch):
    """hipcc --genco of one run-time kernel (BG2 z=52, Neural decode): the cached code object exists and
    holds the unmangled entry point nldpc_graph_attach_kernel looks up."""
    import shutil
    if not os.path.exists("/opt/rocm/bin/hipcc"):
        pytest.skip("hipcc not installed")
    from nldpc import jit
    monkeypatch.setenv("NLDPC_JIT_CACHE", str(tmp_path))
    path, geo = jit.code_object(BG2, 52, 3, 0)
    assert os.path.dirname(path) == str(tmp_path) and os.path.getsize(path) > 1000
    assert geo["G"] == 2 and geo["padded"]
    assert b"nldpc_fx" in open(path, "rb").read()
    again, _ = jit.code_object(BG2, 52, 3, 0)  # a cache hit: same file, no recompile
    assert again == path
    # the argument-layout signature is read from the host bytes (no device copy in attach)
    import ctypes
    from nldpc import _lib
    L = _lib.lib()
    data = open(path, "rb").read()
    sig, exp = ctypes.c_uint32(), ctypes.c_uint32()
    assert L.nldpc_code_object_sig(data, len(data), 0, ctypes.byref(sig), ctypes.byref(exp)) == _lib.NLDPC_OK
    assert sig.value == exp.value != 0
    assert L.nldpc_code_object_sig(data, len(data), 4, ctypes.byref(sig), ctypes.byref(exp)) == _lib.NLDPC_OK
    assert sig.value != exp.value  # a forward kernel is not a backward one
    assert L.nldpc_code_object_sig(data[:200], 200, 0, ctypes.byref(sig), ctypes.byref(exp)) == _lib.NLDPC_EINVAL
    shutil.rmtree(tmp_path, ignore_errors=True)


def test_code_object_sig_reads_a_tampered_layout(tmp_path):
    """A code object generated with another nldpc_sig value reads back that value (what
    nldpc_graph_attach_kernel compares before loading the module)."""
    import ctypes
    import subprocess
    if not os.path.exists("/opt/rocm/bin/hipcc"):
        pytest.skip("hipcc not installed")
    from nldpc import _lib, jit
    src, _ = _gen().jit_source(BG2, 16, 3, 0)
    bad = src.replace("nldpc_sig = nldpc::kFusedArgsSig", "nldpc_sig = 0x12345678u")
    assert bad != src
    s, co = str(tmp_path / "k.hip"), str(tmp_path / "k.co")
    open(s, "w").write(bad)
    subprocess.run([jit.HIPCC, *jit.FLAGS, "-O1", s, "-o", co], check=True, capture_output=True)
    data = open(co, "rb").read()
    sig, exp = ctypes.c_uint32(), ctypes.c_uint32()
    assert _lib.lib().nldpc_code_object_sig(data, len(data), 0, ctypes.byref(sig), ctypes.byref(exp)) == _lib.NLDPC_OK
    assert sig.value == 0x12345678 and exp.value != sig.value


def test_missing_hipcc_falls_back_to_streaming(monkeypatch):
    """a host without the ROCm SDK (no hipcc) must not make decode() raise -- ensure() warns,
    remembers the failure and returns False, so the decode streams.  code_object raises NldpcError
    before touching the compiler; ensure() is driven here with a stand-in handle (no GPU on this host)."""
    from nldpc import _lib, jit
    from nldpc.graph import LiftedGraph
    monkeypatch.setattr(jit, "HIPCC", "/nonexistent/hipcc")
    monkeypatch.setenv("NLDPC_JIT_CACHE", "/tmp/nldpc-jit-test-nohipcc")
    with pytest.raises(_lib.NldpcError, match="no hipcc"):
        jit.code_object(BG2, 44, 3, 0)
    g = LiftedGraph(BG2, 44)
    monkeypatch.setattr(g, "handle", lambda dev: 1)
    monkeypatch.setattr(jit, "kernel_mask", lambda h: 0)
    jit._failed.clear()
    with pytest.warns(UserWarning, match="streaming"):
        assert jit.ensure(g, "cuda", 3, 0) is False
    assert jit.ensure(g, "cuda", 3, 0) is False  # remembered: no second attempt, no second warning


def test_unreadable_generator_sources_fall_back(monkeypatch, tmp_path):
    """An installed package without csrc/ (OSError opening the generator or the headers) streams too."""
    from nldpc import jit
    from nldpc.graph import LiftedGraph
    monkeypatch.setattr(jit, "CSRC", str(tmp_path / "missing"))
    monkeypatch.setattr(jit, "_gen", None)
    g = LiftedGraph(BG2, 36)
    monkeypatch.setattr(g, "handle", lambda dev: 1)
    monkeypatch.setattr(jit, "kernel_mask", lambda h: 0)
    jit._failed.clear()
    with pytest.warns(UserWarning, match="streaming"):
        assert jit.ensure(g, "cuda", 3, 0) is False


def test_wanted_skips_kernels_the_fused_path_never_takes(monkeypatch):
    """decode() asks for a run-time compile only when the fused path could take the call."""
    from nldpc import jit
    from nldpc.decode import KIND_NEURAL, KIND_QMS, DecodeCfg
    monkeypatch.delenv("NLDPC_DISABLE_FUSED", raising=False)
    assert jit.wanted(DecodeCfg(kind=KIND_NEURAL))
    assert jit.wanted(DecodeCfg(kind=KIND_QMS, qbit=5))
    assert not jit.wanted(DecodeCfg(kind=KIND_QMS, qbit=7))  # identity quantiser: streaming kernels only
    monkeypatch.setenv("NLDPC_DISABLE_FUSED", "1")
    assert not jit.wanted(DecodeCfg(kind=KIND_NEURAL))
