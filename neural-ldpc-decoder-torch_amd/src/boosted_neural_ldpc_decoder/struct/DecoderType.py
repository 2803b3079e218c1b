"""Check-node rule selector (reference struct/DecoderType.py:4-7); values are part of the API."""
from enum import Enum


class DecoderType(Enum):
    SP = 0   # sum-product (tanh / atanh)
    MS = 1   # min-sum, messages clipped to allowed_llr_range
    QMS = 2  # quantised min-sum (decoder_qms_qbit)
