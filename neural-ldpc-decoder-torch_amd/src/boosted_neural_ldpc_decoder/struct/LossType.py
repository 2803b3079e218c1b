"""Loss selector of LDPCDecoderLoss (reference struct/LossType.py:4-7)."""
from enum import Enum


class LossType(Enum):
    BCE = "BCE"
    SoftBEROnAllZero = "SoftBEROnAllZero"
    FEROnAllZero = "FEROnAllZero"
