"""Drop-in for the reference package `neural_ldpc_decoder` (src/neural_ldpc_decoder/__init__.py:1-4).

As in the reference, the package attributes are rebound from submodules to classes, so
`import neural_ldpc_decoder.NeuralLDPCDecoder as NeuralLDPCDecoder` yields the class.
"""
from .AWGNPassedDatagen import AWGNPassedDatagen
from .ConnectingMatrix import ConnectingMatrix
from .ConnectingMatrixTorch import ConnectingMatrixTorch
from .NeuralLDPCDecoder import NeuralLDPCDecoder

__all__ = ["AWGNPassedDatagen", "ConnectingMatrix", "ConnectingMatrixTorch", "NeuralLDPCDecoder"]
