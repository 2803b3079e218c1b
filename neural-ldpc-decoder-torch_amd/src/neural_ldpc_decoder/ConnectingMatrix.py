"""ConnectingMatrix of the Dai et al. decoder (reference: src/neural_ldpc_decoder/ConnectingMatrix.py:3-66).

Dense W_* / lifting matrices are computed on first access only; the decoder uses the edge list.
"""
import numpy as np

from nldpc.connecting import ConnectingMatrixBase


class ConnectingMatrix(ConnectingMatrixBase):
    def __init__(self, Z: int, basegraph: np.ndarray, dtype_w_odd2even=np.float32, dtype_w_skipconn2even=np.float32,
                 dtype_w_even2odd=np.float32, dtype_w_output=np.float32, dtype_lifting_matrix=np.float32):
        super().__init__(Z, basegraph, dtype_w_odd2even=dtype_w_odd2even, dtype_w_skipconn2even=dtype_w_skipconn2even,
                         dtype_w_even2odd=dtype_w_even2odd, dtype_w_output=dtype_w_output,
                         dtype_lifting_matrix=dtype_lifting_matrix)
