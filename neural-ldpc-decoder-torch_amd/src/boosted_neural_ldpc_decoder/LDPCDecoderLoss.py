"""Multi-iteration decoder loss (reference: src/boosted_neural_ldpc_decoder/LDPCDecoderLoss.py:7-108).

loss = sum_k etha^c_k * L(outputs[k], expected[k]) / sum_k etha^c_k, then the batch mean, with
L = BCE-with-logits (LossType.BCE), sigmoid(LLR) (SoftBEROnAllZero) or a straight-through frame-error
indicator (FEROnAllZero).  Terms are accumulated from the last output to the first, as in the
reference.  This is the backward seed of config 5; its gradient w.r.t. each output is what
nldpc_backward consumes.  On ROCm tensors the BCE over a list of outputs with one label tensor (the
training script's call) runs as one fused HIP pass per direction (nldpc.loss.bce_multi).
"""
from typing import Optional

import torch
import torch.nn as nn

from boosted_neural_ldpc_decoder.Functions import Functions
from boosted_neural_ldpc_decoder.struct.LossType import LossType
from nldpc.loss import bce_multi


class LDPCDecoderLoss(nn.Module):
    def __init__(self, loss_type: LossType = LossType.BCE, etha: float = 1.0):
        super().__init__()
        self.loss_type = loss_type
        self.etha = etha

    def _term(self, actual, expect):
        if self.loss_type == LossType.BCE:
            return nn.functional.binary_cross_entropy_with_logits(actual, expect)
        if self.loss_type == LossType.SoftBEROnAllZero:
            return torch.sigmoid(actual)
        if self.loss_type == LossType.FEROnAllZero:
            return 0.5 * (1 - Functions.sign_through_torch(torch.min(-actual, dim=1)[0]))
        return 0

    def forward(self, outputs: Optional[list], expected: Optional[list], coeff_param=1) -> torch.Tensor:
        single = isinstance(outputs, torch.Tensor) and isinstance(expected, torch.Tensor)
        listed = isinstance(outputs, list) and isinstance(expected, torch.Tensor)
        paired = isinstance(outputs, list) and isinstance(expected, list) and len(outputs) == len(expected)
        if not (single or listed or paired):
            raise ValueError(
                "Invalid types for outputs and expected in LDPCDecoderLoss. Outputs must be either a torch.Tensor "
                "or a list of torch.Tensor. expected must be either a torch.Tensor or a list of torch.Tensor with "
                "matching length to outputs.")
        if single and not isinstance(coeff_param, int):
            raise ValueError("Invalid coeff_param provided to LDPCDecoderLoss. Must be an integer when outputs is a "
                             "single torch.Tensor.")
        n = 1 if single else len(outputs)
        if (self.loss_type == LossType.BCE and listed and expected.is_cuda and all(
                isinstance(o, torch.Tensor) and o.is_cuda and o.shape == expected.shape for o in outputs)):
            # device path: every term in one HIP pass (nldpc.loss); same sum, fixed-order fp64 reduction
            ws = []
            for k in range(n):
                c = 1
                if coeff_param is not None:
                    c = coeff_param[k] if isinstance(coeff_param, list) else coeff_param
                ws.append(pow(self.etha, c))
            norm = sum(ws)
            coef = [w / norm for w in ws] if norm > 0 else ws
            return 1.0 * bce_multi(outputs, expected, coef)
        total, norm = 0, 0
        for k in reversed(range(n)):
            actual = outputs if single else outputs[k]
            expect = expected[k] if paired else expected
            c = 1
            if coeff_param is not None:
                c = coeff_param[k] if isinstance(coeff_param, list) else coeff_param
            w = pow(self.etha, c)
            total = total + w * self._term(actual, expect)
            norm = norm + w
        if norm > 0:
            total = total / norm
        return 1.0 * total.mean()
