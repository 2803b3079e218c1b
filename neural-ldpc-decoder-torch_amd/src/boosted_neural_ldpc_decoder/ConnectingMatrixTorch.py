"""ConnectingMatrixTorch of the boosted decoder (reference: src/boosted_neural_ldpc_decoder/ConnectingMatrixTorch.py:6-54)."""
import torch

from nldpc.connecting import ConnectingMatrixTorchBase

from boosted_neural_ldpc_decoder.ConnectingMatrix import _ALL, ConnectingMatrix


class ConnectingMatrixTorch(ConnectingMatrixTorchBase):
    _matrices = _ALL

    def __init__(self, connecting_matrix: ConnectingMatrix, device: torch.device = torch.device("cpu"),
                 dtype_w_odd2even: torch.dtype = torch.float32, dtype_w_skipconn2even: torch.dtype = torch.float32,
                 dtype_w_even2odd: torch.dtype = torch.float32, dtype_w_even2odd_with_self: torch.dtype = torch.float32,
                 dtype_w_output: torch.dtype = torch.float32, dtype_w_skipconn2odd: torch.dtype = torch.float32,
                 dtype_lifting_matrix: torch.dtype = torch.float32):
        super().__init__(connecting_matrix, device, dtype_w_odd2even=dtype_w_odd2even,
                         dtype_w_skipconn2even=dtype_w_skipconn2even, dtype_w_even2odd=dtype_w_even2odd,
                         dtype_w_even2odd_with_self=dtype_w_even2odd_with_self, dtype_w_output=dtype_w_output,
                         dtype_w_skipconn2odd=dtype_w_skipconn2odd, dtype_lifting_matrix=dtype_lifting_matrix)
        self.neurons_per_even_layer = connecting_matrix.neurons_per_even_layer
        self.neurons_per_odd_layer = connecting_matrix.neurons_per_odd_layer
