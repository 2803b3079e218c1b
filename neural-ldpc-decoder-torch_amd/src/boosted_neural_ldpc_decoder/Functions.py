"""Helper functions of the boosted decoder (reference: src/boosted_neural_ldpc_decoder/Functions.py:4-102).

The straight-through helpers and the quantiser are elementwise torch expressions (API helpers; the
decoder itself quantises inside the HIP kernels).  evaluate_ber_fer keeps the reference's literal
rule bit = (LLR < 0) and return types, but counts every iteration with the fused device counter
(nldpc_ber_count) and a single host synchronisation instead of 2T `.item()` calls.
"""
import numpy as np
import torch

# (clip bound, quantisation step) per supported bit width; q=6 keeps the reference's +-15.5 clip
_QMS = {6: (15.5, 1.0), 5: (7.5, 0.5), -5: (15.0, 1.0), 4: (7.0, 1.0), 3: (6.0, 2.0)}


def _grid(x, step):
    if step == 1.0:
        return torch.round(x)
    if step == 0.5:
        return torch.round(x * 2.0) / 2.0
    return torch.round(x / 2) * 2


class Functions:
    @staticmethod
    def hard_sigmoid_torch(x: torch.Tensor) -> torch.Tensor:
        return torch.clamp(x, 0.0, 1.0)

    @staticmethod
    def proxy_sign_torch(x: torch.Tensor) -> torch.Tensor:
        return torch.clamp(x, -1.0, 1.0)

    @staticmethod
    def inv_exp_torch(x: torch.Tensor) -> torch.Tensor:
        return 2.0 / (1.0 + torch.exp(-x)) - 1.0

    @staticmethod
    def round_through_torch(x: torch.Tensor) -> torch.Tensor:
        soft = Functions.hard_sigmoid_torch(x)
        return soft + (torch.round(x) - soft).detach()

    @staticmethod
    def sign_through_torch(x: torch.Tensor) -> torch.Tensor:
        approx = Functions.inv_exp_torch(x)
        return approx + (torch.sign(x) - approx).detach()

    @staticmethod
    def qms_clipping_torch(x: torch.Tensor, q_bit: int) -> torch.Tensor:
        if q_bit not in _QMS:
            return x
        bound = _QMS[q_bit][0]
        return torch.clamp(x, -bound, bound)

    @staticmethod
    def cal_msa_q_torch(x: torch.Tensor, q_bit: int) -> torch.Tensor:
        """QMS quantiser, forward = quantised value, backward = clip-range straight-through."""
        if q_bit not in _QMS:
            return x
        bound, step = _QMS[q_bit]
        q_value = torch.clamp(_grid(x, step), -bound, bound)
        clip_value = torch.clamp(x, -bound, bound)
        return clip_value + (q_value - clip_value).detach()

    @staticmethod
    def Cal_MSA_Q(x, q_bit):
        """numpy quantiser used by the datagen (round half to even, then clip)."""
        if q_bit not in _QMS:
            return x
        bound, step = _QMS[q_bit]
        if step == 1.0:
            g = np.round(x)
        elif step == 0.5:
            g = np.round(x * 2) / 2
        else:
            g = np.round(x / 2) * 2
        return np.clip(g, -bound, bound)

    @staticmethod
    def evaluate_ber_fer(expected: torch.Tensor, actual: list):
        """((bit errors per iteration, bits), (frame errors per iteration, frames)) with the
        reference helper's literal decision rule bit = (LLR < 0) (with the
        decoder's own convention this reports ~1 - BER; nldpc.channel.ber_counts(convention=0) gives
        the decoder-convention counts)."""
        from nldpc.channel import ber_counts
        counts = ber_counts(actual, expected, convention=1).cpu().tolist()
        bit_errors = [float(c[0]) for c in counts]
        frame_errors = [float(c[1]) for c in counts]
        return (bit_errors, expected.numel()), (frame_errors, expected.shape[0])
