"""Punctured bit range, 1-based inclusive (reference struct/Puncture.py:1-14)."""
from boosted_neural_ldpc_decoder.struct._Range import InclusiveRange


class Puncture(InclusiveRange):
    _what = "puncture"
