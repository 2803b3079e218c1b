"""ConnectingMatrixTorch of the Dai et al. decoder (reference: src/neural_ldpc_decoder/ConnectingMatrixTorch.py:6-46).

Holds the graph for a device; dense tensors are materialised only if read.
"""
import torch

from nldpc.connecting import ConnectingMatrixTorchBase

from .ConnectingMatrix import ConnectingMatrix


class ConnectingMatrixTorch(ConnectingMatrixTorchBase):
    def __init__(self, connecting_matrix: ConnectingMatrix, device: torch.device = torch.device("cpu"),
                 dtype_w_odd2even: torch.dtype = torch.float32, dtype_w_skipconn2even: torch.dtype = torch.float32,
                 dtype_w_even2odd: torch.dtype = torch.float32, dtype_w_output: torch.dtype = torch.float32,
                 dtype_lifting_matrix: torch.dtype = torch.float32):
        super().__init__(connecting_matrix, device, dtype_w_odd2even=dtype_w_odd2even,
                         dtype_w_skipconn2even=dtype_w_skipconn2even, dtype_w_even2odd=dtype_w_even2odd,
                         dtype_w_output=dtype_w_output, dtype_lifting_matrix=dtype_lifting_matrix)
