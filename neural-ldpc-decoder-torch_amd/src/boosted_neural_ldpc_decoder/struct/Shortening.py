"""Shortened bit range, 1-based inclusive (reference struct/Shortening.py:1-14)."""
from boosted_neural_ldpc_decoder.struct._Range import InclusiveRange


class Shortening(InclusiveRange):
    _what = "shortening"
