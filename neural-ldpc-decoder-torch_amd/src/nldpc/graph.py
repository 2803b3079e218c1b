"""Lifted QC-LDPC Tanner graph as an edge list (host tables + lazily created device handles).

Replaces the dense routing of the reference's ConnectingMatrix (boosted.../ConnectingMatrix.py:82-163,
neural.../ConnectingMatrix.py:68-140).  Edge e is the e-th non-(-1) entry of the base graph in
row-major ("C-order") order, with check chk[e], variable var[e] and cyclic shift s[e] = Hb mod Z:
row (i, h) of the lifted H has its 1 at column (j, (h + s) mod Z).  The dense matrices the reference
exposes are derivable from these tables (see dense_* below) but never needed by the decoder.
"""
from __future__ import annotations

import ctypes
import threading

import numpy as np
import torch

from . import _lib


class LiftedGraph:
    def __init__(self, basegraph, Z: int):
        hb = np.asarray(basegraph)
        if hb.ndim != 2:
            raise ValueError("basegraph must be a 2-D shift table")
        self.basegraph = hb.astype(np.int64).copy()
        self.M, self.N = self.basegraph.shape
        self.Z = int(Z)
        if self.Z <= 0:
            raise ValueError("Z must be positive")
        rows, cols = np.nonzero(self.basegraph != -1)
        self.E = int(len(rows))
        self.chk = rows.astype(np.int64)
        self.var = cols.astype(np.int64)
        self.shift = (self.basegraph[rows, cols] % self.Z).astype(np.int64)
        self.deg_c = np.bincount(self.chk, minlength=self.M).astype(np.int64)
        self.deg_v = np.bincount(self.var, minlength=self.N).astype(np.int64)
        # V-order (column-major) position of every C-order edge (lifting_matrix_1 / W_odd2even columns)
        self.v_order = np.lexsort((self.chk, self.var))  # v_order[k] = C-order edge at V-position k
        self._handles = {}
        self._idx = {}
        self._lock = threading.Lock()

    # ------------------------------------------------------------------ device side
    def handle(self, device: torch.device) -> int:
        """nldpc_graph* for a ROCm device (created on first use)."""
        device = torch.device(device)
        if device.type != "cuda":
            raise RuntimeError(
                f"the MI355X decoder runs on a ROCm GPU device ('cuda' in PyTorch); got '{device}'. "
                "There is no CPU path.")
        idx = device.index if device.index is not None else torch.cuda.current_device()
        with self._lock:
            h = self._handles.get(idx)
            if h is None:
                L = _lib.lib()
                tbl = np.ascontiguousarray(self.basegraph, dtype=np.int32)
                out = ctypes.c_void_p()
                _lib.check(L.nldpc_graph_create(self.M, self.N, self.Z,
                                                tbl.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), idx,
                                                ctypes.byref(out)), "nldpc_graph_create")
                h = out.value
                self._handles[idx] = h
        return h

    def index_tensor(self, name: str, device) -> torch.Tensor:
        """int64 index tables on a device (chk / var) for differentiable weight expansion."""
        key = (name, str(device))
        t = self._idx.get(key)
        if t is None:
            t = torch.as_tensor(getattr(self, name), dtype=torch.long, device=device)
            self._idx[key] = t
        return t

    def __del__(self):
        try:
            if self._handles and _lib._lib is not None:
                for h in self._handles.values():
                    _lib._lib.nldpc_graph_destroy(h)
        except Exception:
            pass

    # ------------------------------------------------------------------ dense views (reference API)
    def _cpos(self):
        return np.arange(self.E)

    def dense_W_skipconn2even(self, dtype=np.float32):
        """[N, E]: 1 at (var(e), V-position of e)  (ConnectingMatrix.py:149-155)."""
        W = np.zeros((self.N, self.E), dtype=dtype)
        W[self.var[self.v_order], np.arange(self.E)] = 1
        return W

    def dense_W_odd2even(self, dtype=np.float32):
        """[E(C-order), E(V-order)]: 1 if same column, different row (ConnectingMatrix.py:101-120)."""
        W = np.zeros((self.E, self.E), dtype=dtype)
        for k, e in enumerate(self.v_order):
            others = np.nonzero((self.var == self.var[e]) & (np.arange(self.E) != e))[0]
            W[others, k] = 1
        return W

    def dense_W_even2odd(self, dtype=np.float32, with_self=False):
        """[E(V-order), E(C-order)]: 1 if same row (and different edge unless with_self) (:122-135)."""
        W = np.zeros((self.E, self.E), dtype=dtype)
        for k, e in enumerate(self.v_order):
            same = np.nonzero(self.chk == self.chk[e])[0]
            W[k, same] = 1
            if not with_self:
                W[k, e] = 0
        return W

    def dense_W_output(self, dtype=np.float32):
        """[E(C-order), N]: 1 at (e, var(e))  (ConnectingMatrix.py:137-147)."""
        W = np.zeros((self.E, self.N), dtype=dtype)
        W[np.arange(self.E), self.var] = 1
        return W

    def dense_W_skipconn2odd(self, dtype=np.float32):
        """[M, E(C-order)]: 1 at (chk(e), e)  (ConnectingMatrix.py:157-163)."""
        W = np.zeros((self.M, self.E), dtype=dtype)
        W[self.chk, np.arange(self.E)] = 1
        return W

    def dense_lifting(self, which: int, dtype=np.float32):
        """(E*Z)^2 permutation: which=1 V-order blocks (:84-91), which=2 C-order blocks (:92-99)."""
        EZ = self.E * self.Z
        L = np.zeros((EZ, EZ), dtype=dtype)
        order = self.v_order if which == 1 else np.arange(self.E)
        h = np.arange(self.Z)
        for k, e in enumerate(order):
            L[k * self.Z + h, k * self.Z + (h + self.shift[e]) % self.Z] = 1
        return L
