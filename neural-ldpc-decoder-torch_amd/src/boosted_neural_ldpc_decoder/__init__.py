"""Drop-in for the reference package `boosted_neural_ldpc_decoder`
(src/boosted_neural_ldpc_decoder/__init__.py:1-4): Kwak et al. 2023 boosted SP/MS/QMS decoder."""
from boosted_neural_ldpc_decoder.AWGNPassedDatagen import AWGNPassedDatagen
from boosted_neural_ldpc_decoder.ConnectingMatrix import ConnectingMatrix
from boosted_neural_ldpc_decoder.ConnectingMatrixTorch import ConnectingMatrixTorch
from boosted_neural_ldpc_decoder.Functions import Functions

__all__ = ["AWGNPassedDatagen", "ConnectingMatrix", "ConnectingMatrixTorch", "Functions"]
