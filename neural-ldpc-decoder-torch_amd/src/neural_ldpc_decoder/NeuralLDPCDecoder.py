"""NeuralLDPCDecoder (Dai et al. 2021 neural min-sum) on MI355X.

Reference: src/neural_ldpc_decoder/NeuralLDPCDecoder.py:6-100.  Same constructor, parameters
(`weights_var.{t}` init 0.5, `biases_var.{t}` init 0, one [E] vector each per iteration, C-order
edges) and forward contract: forward(xa [B, N, Z]) -> list of T posteriors [B, N*Z].  The iteration
loop runs as HIP kernels through libnldpc.so (nldpc.decode); gradients flow to the weights and
biases through nldpc_backward.  The reference's dense routing buffers (W_*, Lift_Matrix*) are not
registered (22.9 GB each at z=384); their keys in an old state_dict are accepted and ignored.
"""
import torch
import torch.nn as nn

from nldpc.decode import KIND_NEURAL, DecodeCfg, decode_autograd, decode_count

from .ConnectingMatrixTorch import ConnectingMatrixTorch

_DENSE_BUFFERS = ("W_odd2even", "W_skipconn2even", "W_even2odd", "W_output", "Lift_Matrix1", "Lift_Matrix2")


class NeuralLDPCDecoder(nn.Module):
    def __init__(self, iter_node_counts, batch_size, connecting_matrix: ConnectingMatrixTorch):
        super().__init__()
        self.iter_node_counts = iter_node_counts
        self.batch_size = batch_size
        self.conn_mat = connecting_matrix
        self.N = self.conn_mat.N
        self.M = self.conn_mat.M
        self.Z = self.conn_mat.Z
        self.sum_edge = self.conn_mat.sum_edge
        self.neurons_per_odd_layer = self.conn_mat.neurons_per_odd_layer
        self.neurons_per_even_layer = self.conn_mat.neurons_per_even_layer
        E = int(self.sum_edge)
        self.weights_var = nn.ParameterList(
            [nn.Parameter(torch.full((E,), 0.5, dtype=torch.float32)) for _ in range(iter_node_counts)])
        self.biases_var = nn.ParameterList(
            [nn.Parameter(torch.zeros(E, dtype=torch.float32)) for _ in range(iter_node_counts)])
        self._cfg = DecodeCfg(kind=KIND_NEURAL, keep_state=False)  # forward() never resumes from a state

    def _load_from_state_dict(self, state_dict, prefix, local_metadata, strict, missing_keys, unexpected_keys,
                              error_msgs):
        for k in _DENSE_BUFFERS:  # reference checkpoints carry the dense routing buffers
            state_dict.pop(prefix + k, None)
        super()._load_from_state_dict(state_dict, prefix, local_metadata, strict, missing_keys, unexpected_keys,
                                      error_msgs)

    def _weights(self):
        """The per-iteration weights and biases as [T, E] tensors, stacked on every call.  (A cache keyed
        on the parameters' storage and in-place version missed updates made through `p.data`, which
        do not bump the version -- the reference itself clamps parameters that way, Boosted…py:177 --
        so a serving loop could have decoded with stale weights; the two stack launches cost ~10 us.)"""
        return torch.stack(list(self.weights_var)), torch.stack(list(self.biases_var))

    def forward(self, xa):
        T = self.iter_node_counts
        w, b = self._weights()
        outs, _ = decode_autograd(self.conn_mat.graph, self._cfg, xa, T, w_cn=w, bias=b)
        return outs

    @torch.no_grad()
    def count_errors(self, xa, y=None, convention=0):
        """Count-only decode (extension): int64 [T, 2] device tensor of (bit errors, frame
        errors) per iteration, equal to nldpc.channel.ber_counts(self.forward(xa), y, convention=...)
        without materialising the T posteriors.  y: [B, N*Z] codeword bits or None (all-zero)."""
        T = self.iter_node_counts
        w, b = self._weights()
        return decode_count(self.conn_mat.graph, self._cfg, xa, T, w_cn=w, bias=b, y=y, convention=convention)
