"""ConnectingMatrix of the boosted decoder (reference: src/boosted_neural_ldpc_decoder/ConnectingMatrix.py:4-163).

Adds W_even2odd_with_self and W_skipconn2odd to the neural variant.  All dense matrices are lazy;
the decoder runs on the edge list in `self.graph`.
"""
import numpy as np

from nldpc.connecting import ConnectingMatrixBase

_ALL = ("W_odd2even", "W_skipconn2even", "W_even2odd", "W_even2odd_with_self", "W_output", "W_skipconn2odd",
        "lifting_matrix_1", "lifting_matrix_2")


class ConnectingMatrix(ConnectingMatrixBase):
    _matrices = _ALL

    def __init__(self, Z: int, basegraph: np.ndarray, dtype_w_odd2even=np.float32, dtype_w_skipconn2even=np.float32,
                 dtype_w_even2odd=np.float32, dtype_w_even2odd_with_self=np.float32, dtype_w_output=np.float32,
                 dtype_w_skipconn2odd=np.float32, dtype_lifting_matrix=np.float32):
        super().__init__(Z, basegraph, dtype_w_odd2even=dtype_w_odd2even, dtype_w_skipconn2even=dtype_w_skipconn2even,
                         dtype_w_even2odd=dtype_w_even2odd, dtype_w_even2odd_with_self=dtype_w_even2odd_with_self,
                         dtype_w_output=dtype_w_output, dtype_w_skipconn2odd=dtype_w_skipconn2odd,
                         dtype_lifting_matrix=dtype_lifting_matrix)
        self.neurons_per_even_layer = self.sum_edge
        self.neurons_per_odd_layer = self.sum_edge
