"""Parameter kind used in parameter names `{kind}_{node}_{iter}` (reference struct/ParamType.py:4-6)."""
from enum import Enum


class ParamType(Enum):
    Weight = "weight"
    Bias = "bias"
