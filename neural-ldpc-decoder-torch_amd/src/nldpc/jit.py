"""Register-resident kernels compiled at run time for lifted graphs the library was not built for
(SURVEY.md §8 F4).

The reference builds its decoder for any lifting size at run time (ConnectingMatrix(Z, basegraph),
boosted.../ConnectingMatrix.py:5-53).  libnldpc.so carries generated fused kernels for a fixed set of
(base graph, Z); every other lifted graph would decode on the streaming kernels, about ten times
slower.  Here the first decode of such a graph with a given decoder kind and mode generates that one
kernel (csrc/gen_fused.py jit_source: auto_geometry, the same emitted code as the built-in kernels),
compiles it for gfx950 with hipcc into a code object, caches it on disk, and attaches it to the graph
handle (nldpc_graph_attach_kernel).  Later decodes, in this process or another, load it from the cache.

Modes: 0 decode, 1 decode + save for backward, 2 / 3 count-only, 4 backward (include/nldpc.h).
Environment: NLDPC_JIT=0 disables compiling (graphs without a built-in kernel stream);
NLDPC_JIT_CACHE=<dir> moves the cache (default: lib/jit next to libnldpc.so, else ~/.cache/nldpc-jit);
NLDPC_JIT_LOG=<file> appends one line per compile (also logged on the "nldpc.jit" logger and kept in
`compile_log`).  Any failure to build (no geometry, no hipcc, no generator sources, an unwritable cache,
a compiler error) warns once and leaves that kernel to the streaming path.
"""
from __future__ import annotations

import ctypes
import hashlib
import importlib.util
import logging
import os
import shutil
import subprocess
import tempfile
import threading
import time
import warnings

from . import _lib

_PKG = os.path.normpath(os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
CSRC = os.path.join(_PKG, "csrc")
INCLUDE = os.path.normpath(os.path.join(_PKG, "..", "include"))
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["--genco", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-fno-fast-math",
         "-fno-slp-vectorize", "-Wno-unused-function", "-I" + INCLUDE, "-I" + CSRC]
_HEADERS = ("nldpc_fused.h", "nldpc_node.h", "nldpc_math.h", "nldpc_internal.h", "nldpc_sleef.h")

_lock = threading.Lock()
_gen = None
_failed = set()  # (graph key, kind, mode) that could not be built: not retried in this process
_log = logging.getLogger("nldpc.jit")
# one dict per compile in this process: Z, kind, mode, geometry, seconds (profiles/ records them)
compile_log: list = []


def enabled() -> bool:
    return os.environ.get("NLDPC_JIT", "1") != "0"


def _generator():
    global _gen
    if _gen is None:
        spec = importlib.util.spec_from_file_location("nldpc_gen_fused", os.path.join(CSRC, "gen_fused.py"))
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
        _gen = mod
    return _gen


def cache_dir() -> str:
    d = os.environ.get("NLDPC_JIT_CACHE") or os.path.join(os.path.dirname(_lib.LIB_PATH), "jit")
    try:
        os.makedirs(d, exist_ok=True)
        if os.access(d, os.W_OK):
            return d
    except OSError:
        pass
    d = os.path.join(os.path.expanduser("~"), ".cache", "nldpc-jit")
    os.makedirs(d, exist_ok=True)
    return d


def _key(source: str) -> str:
    h = hashlib.sha256(source.encode())
    for name in _HEADERS:
        with open(os.path.join(CSRC, name), "rb") as f:
            h.update(f.read())
    with open(os.path.join(INCLUDE, "nldpc.h"), "rb") as f:
        h.update(f.read())
    h.update(" ".join(FLAGS[:-2]).encode())  # (not the include paths: the same text anywhere)
    return h.hexdigest()[:32]


def kernel_mask(handle) -> int:
    m = ctypes.c_uint32(0)
    _lib.check(_lib.lib().nldpc_graph_kernels(handle, ctypes.byref(m)), "nldpc_graph_kernels")
    return int(m.value)


def code_object(basegraph, Z: int, kind: int, mode: int):
    """(path of the cached code object, geometry) for one kernel, compiling it on a cache miss."""
    gen = _generator()
    src, geo = gen.jit_source(basegraph, int(Z), int(kind), int(mode))
    path = os.path.join(cache_dir(), f"fx_{_key(src)}.co")
    if not os.path.exists(path):
        exe = HIPCC if os.path.isabs(HIPCC) else shutil.which(HIPCC)
        if not exe or not os.path.exists(exe):
            raise _lib.NldpcError(f"no hipcc at {HIPCC} to compile the run-time kernel (Z={Z})")
        t0 = time.perf_counter()
        with tempfile.TemporaryDirectory() as tmp:
            s = os.path.join(tmp, "k.hip")
            with open(s, "w") as f:
                f.write(src)
            out = os.path.join(tmp, "k.co")
            r = subprocess.run([exe, *FLAGS, s, "-o", out], capture_output=True, text=True)
            if r.returncode != 0 or not os.path.exists(out):
                raise _lib.NldpcError(f"hipcc failed on the run-time kernel (Z={Z}, kind {kind}, mode {mode}):\n"
                                      f"{r.stderr[-3000:]}")
            part = path + f".{os.getpid()}.tmp"
            os.replace(out, part)
            os.replace(part, path)  # atomic: a concurrent process sees the whole file or none
        rec = {"Z": int(Z), "kind": int(kind), "mode": int(mode), "G": geo["G"], "P": geo["P"], "Q": geo["Q"],
               "threads": geo["threads"], "padded": bool(geo["padded"]),
               "seconds": round(time.perf_counter() - t0, 3)}
        compile_log.append(rec)
        line = (f"nldpc.jit: compiled Z={rec['Z']} kind={rec['kind']} mode={rec['mode']} (G={rec['G']} P={rec['P']} "
                f"Q={rec['Q']} threads={rec['threads']}{' padded' if rec['padded'] else ''}) in {rec['seconds']:.2f} s")
        _log.info(line)
        if os.environ.get("NLDPC_JIT_LOG"):
            with open(os.environ["NLDPC_JIT_LOG"], "a") as f:
                f.write(line + "\n")
    return path, geo


def wanted(cfg) -> bool:
    """Whether the fused path could take a decode at all (so a run-time compile can pay off): not when
    NLDPC_DISABLE_FUSED is set, and not for QMS with a quantiser the fused QMS kernels do not carry (an
    inactive qbit decodes on the streaming kernels)."""
    if os.environ.get("NLDPC_DISABLE_FUSED") is not None:
        return False
    return not (cfg.kind == _lib.NLDPC_QMS and cfg.qbit not in (6, 5, -5, 4, 3))


def ensure(graph, device, kind: int, mode: int) -> bool:
    """Make the fused kernel of (graph, kind, mode) available on `device`'s graph handle: built in,
    already attached, loaded from the cache, or compiled now.  False when the graph cannot have one
    (no register-resident geometry), compiling is disabled, or the compile failed (with a warning):
    the decode then runs on the streaming kernels."""
    h = graph.handle(device)
    bit = 1 << (int(mode) * 4 + int(kind))
    if kernel_mask(h) & bit:
        return True
    key = (graph.basegraph.tobytes(), graph.basegraph.shape, graph.Z, int(kind), int(mode))
    if not enabled() or key in _failed:
        return False
    with _lock:
        if kernel_mask(h) & bit:
            return True
        try:
            path, geo = code_object(graph.basegraph, graph.Z, kind, mode)
        except SystemExit as e:  # auto_geometry: no register-resident geometry for this graph
            _failed.add(key)
            warnings.warn(f"nldpc: no fused kernel for Z={graph.Z} ({e}); decoding on the streaming kernels")
            return False
        except (_lib.NldpcError, OSError, subprocess.SubprocessError) as e:
            # no hipcc / no generator sources (an installed package without csrc/) / an unwritable cache /
            # a compiler error: this kernel streams for the rest of the process
            _failed.add(key)
            warnings.warn(f"nldpc: no run-time kernel for Z={graph.Z} kind {kind} mode {mode} ({e}); "
                          "decoding on the streaming kernels")
            return False
        with open(path, "rb") as f:
            data = f.read()
        buf = ctypes.create_string_buffer(data, len(data))
        _lib.check(_lib.lib().nldpc_graph_attach_kernel(h, int(mode), int(kind), buf, len(data), geo["G"],
                                                        geo["threads"], geo["waves_per_part"]),
                   "nldpc_graph_attach_kernel")
    return True
