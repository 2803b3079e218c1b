"""Shared implementation of the reference's ConnectingMatrix / ConnectingMatrixTorch API.

Reference: src/{neural_ldpc_decoder,boosted_neural_ldpc_decoder}/ConnectingMatrix.py and
ConnectingMatrixTorch.py.  The attribute surface is kept (M, N, Z, basegraph, basegraph_binary,
sum_edge_c, sum_edge_v, sum_edge, neurons_per_*_layer, dtype_*, W_*, lifting_matrix_{1,2}), but the
dense routing matrices are computed only when somebody reads them: the decoder itself runs on the
edge list (nldpc.graph.LiftedGraph), so BG2 z=384 never allocates the reference's 2 x 22.9 GB
lifting matrices.
"""
from __future__ import annotations

import numpy as np
import torch

from .graph import LiftedGraph

_HOST_MATS = {
    "W_odd2even": lambda g, dt: g.dense_W_odd2even(dt),
    "W_skipconn2even": lambda g, dt: g.dense_W_skipconn2even(dt),
    "W_even2odd": lambda g, dt: g.dense_W_even2odd(dt),
    "W_even2odd_with_self": lambda g, dt: g.dense_W_even2odd(dt, with_self=True),
    "W_output": lambda g, dt: g.dense_W_output(dt),
    "W_skipconn2odd": lambda g, dt: g.dense_W_skipconn2odd(dt),
    "lifting_matrix_1": lambda g, dt: g.dense_lifting(1, dt),
    "lifting_matrix_2": lambda g, dt: g.dense_lifting(2, dt),
}

_DTYPE_ATTR = {
    "W_odd2even": "dtype_w_odd2even",
    "W_skipconn2even": "dtype_w_skipconn2even",
    "W_even2odd": "dtype_w_even2odd",
    "W_even2odd_with_self": "dtype_w_even2odd_with_self",
    "W_output": "dtype_w_output",
    "W_skipconn2odd": "dtype_w_skipconn2odd",
    "lifting_matrix_1": "dtype_lifting_matrix",
    "lifting_matrix_2": "dtype_lifting_matrix",
}


class ConnectingMatrixBase:
    """ConnectingMatrix(Z, basegraph, dtype_...) — host graph description."""

    _matrices = ("W_odd2even", "W_skipconn2even", "W_even2odd", "W_output", "lifting_matrix_1", "lifting_matrix_2")

    def __init__(self, Z: int, basegraph: np.ndarray, **dtypes):
        self.basegraph = np.asarray(basegraph).copy()
        self.M, self.N = self.basegraph.shape
        self.Z = Z
        self.basegraph_binary = (self.basegraph != -1).astype(self.basegraph.dtype)
        self.sum_edge_c = np.sum(self.basegraph_binary, axis=1)
        self.sum_edge_v = np.sum(self.basegraph_binary, axis=0)
        self.sum_edge = np.sum(self.sum_edge_v)
        for name in set(_DTYPE_ATTR.values()):
            setattr(self, name, dtypes.get(name, np.float32))
        self.neurons_per_even_layer = np.copy(self.sum_edge)
        self.neurons_per_odd_layer = np.copy(self.sum_edge)
        self.graph = LiftedGraph(self.basegraph, Z)
        self._dense = {}

    def __getattr__(self, name):
        if name in type(self)._matrices:
            d = self.__dict__.setdefault("_dense", {})
            if name not in d:
                d[name] = _HOST_MATS[name](self.graph, getattr(self, _DTYPE_ATTR[name]))
            return d[name]
        raise AttributeError(name)


class ConnectingMatrixTorchBase:
    """ConnectingMatrixTorch(connecting_matrix, device, dtype_...) — the graph bound to a device."""

    _matrices = ConnectingMatrixBase._matrices

    def __init__(self, connecting_matrix: ConnectingMatrixBase, device: torch.device = torch.device("cpu"),
                 **dtypes):
        self.device = device
        cm = connecting_matrix
        self.N, self.M, self.Z = cm.N, cm.M, cm.Z
        self.basegraph = cm.basegraph.copy()
        self.sum_edge_c = cm.sum_edge_c.copy()
        self.sum_edge_v = cm.sum_edge_v.copy()
        self.sum_edge = cm.sum_edge.copy()
        for name in set(_DTYPE_ATTR.values()):
            setattr(self, name, dtypes.get(name, torch.float32))
        self.neurons_per_even_layer = np.copy(self.sum_edge)
        self.neurons_per_odd_layer = np.copy(self.sum_edge)
        self.connecting_matrix = cm
        self.graph: LiftedGraph = cm.graph

    def __getattr__(self, name):
        if name in type(self)._matrices:
            d = self.__dict__.setdefault("_dense", {})
            if name not in d:
                host = getattr(self.__dict__["connecting_matrix"], name)
                d[name] = torch.tensor(host, dtype=getattr(self, _DTYPE_ATTR[name]), device=self.device)
            return d[name]
        raise AttributeError(name)
