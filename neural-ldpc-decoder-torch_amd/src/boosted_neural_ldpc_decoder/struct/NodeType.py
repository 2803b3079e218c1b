"""Node families that may carry learned weights (reference struct/NodeType.py:3-6)."""
from enum import Enum


class NodeType(Enum):
    CN = "CN"    # check node
    UCN = "UCN"  # unsatisfied check node
    VN = "VN"    # variable node (channel input)
