"""Weight-sharing codes per node family (reference struct/NodeWeightSharingConfig.py:4-40).

  0 none · 1 per edge and iteration · 2 per node and iteration · 3 per iteration
  4 per edge, temporal (fixed_iterative_nodes) · 5 per node, temporal
Iteration yields (NodeType, code) for CN, UCN, VN in that order."""
from boosted_neural_ldpc_decoder.struct.NodeType import NodeType


class NodeWeightSharingConfig:
    def __init__(self, cn_weight_sharing: int, ucn_weight_sharing: int, vn_weight_sharing: int):
        self.cn_weight_sharing = cn_weight_sharing
        self.ucn_weight_sharing = ucn_weight_sharing
        self.vn_weight_sharing = vn_weight_sharing

    def _codes(self):
        return {NodeType.CN: self.cn_weight_sharing, NodeType.UCN: self.ucn_weight_sharing,
                NodeType.VN: self.vn_weight_sharing}

    def __iter__(self):
        return iter(self._codes().items())

    def get(self, node_type: NodeType):
        return self._codes().get(node_type)
