"""On-device channel model and error accounting (the steps either side of the decode path).

awgn_llr       codeword (all-zero or given y) over BPSK/AWGN, LLR = 2*((-1)^(1-y) + sigma*n)/sigma^2, with the
               reference's QMS quantiser, puncturing and shortening; n from Philox-4x32-10 at
               counter (b_offset + b)*L + k: a batch sharded over ranks draws exactly the noise of the
               unsharded batch (replaces the numpy per-codeword loop of AWGNPassedDatagen.py:75-193).
sigma_for      the reference's Eb/N0 -> sigma mapping with its code-rate formula (AWGNPassedDatagen.py:47-49).
ber_counts     fused bit/frame error counters for a list of posteriors (Functions.evaluate_ber_fer,
               Functions.py:85-102) without 2T host synchronisations.
"""
from __future__ import annotations

import math

import torch

from . import _lib


def sigma_for(ebn0_db: float, code_rate: float) -> float:
    return math.sqrt(1.0 / (2.0 * code_rate * 10.0 ** (ebn0_db / 10.0)))


def boosted_code_rate(N: int, M: int, n_punct: int = 1, n_short: int = 1) -> float:
    """K / (N - len(puncture) - len(shortening)); the reference's defaults have length 1 each (Q4)."""
    return (N - M) / (N - n_punct - n_short)


def awgn_llr(B: int, N: int, Z: int, sigma: float, *, seed: int = 2042, b_offset: int = 0, qbit: int = 0,
             device=None, out: torch.Tensor | None = None, y: torch.Tensor | None = None, puncturing=None,
             shortening=None, puncture_value: float = 0.0, shortening_value: float = -20.0) -> torch.Tensor:
    """[B, N, Z] fp32 channel LLRs on the device.  y: [B, N*Z] codeword bits (None = all-zero);
    puncturing / shortening: (start, end) 1-based inclusive bit ranges of every codeword, or objects
    with .start / .end (the reference's Puncture / Shortening; start 0 = none), set after the QMS
    quantiser to puncture_value (reference: 0, 0.001 for SP) / shortening_value (-|llr_hi|)."""
    device = torch.device(device if device is not None else "cuda")
    if out is None:
        out = torch.empty((B, N, Z), dtype=torch.float32, device=device)
    L = N * Z
    rng = lambda r: (0, 0) if r is None else ((r.start, r.end) if hasattr(r, "start") else tuple(r))  # noqa: E731
    (p0, p1), (s0, s1) = rng(puncturing), rng(shortening)
    yb = None
    if y is not None:
        if y.device != out.device or y.numel() != B * L:
            raise ValueError(f"y must be a [B, N*Z] = [{B}, {L}] tensor on {out.device}")
        yb = (y != 0).to(torch.uint8).reshape(B, L).contiguous()
    _lib.check(_lib.lib().nldpc_channel_llr(out.data_ptr(), B, L, float(sigma), int(seed) & (2 ** 64 - 1),
                                            int(b_offset), int(qbit), _lib.ptr(yb), int(p0), int(p1),
                                            float(puncture_value), int(s0), int(s1), float(shortening_value),
                                            _lib.stream_of(out.device)), "nldpc_channel_llr")
    return out


def ber_counts(outputs, y: torch.Tensor | None = None, *, convention: int = 0) -> torch.Tensor:
    """int64 [T, 2] device tensor of (bit errors, frame errors) per output in `outputs`.

    convention 0: bit = (LLR > 0), the decoder's sign convention; 1: bit = (LLR < 0), the literal rule
    of the reference helper.  y: [B, L] bits (any dtype) or None for the all-zero codeword."""
    outputs = list(outputs)
    dev = outputs[0].device
    if dev.type != "cuda":
        raise RuntimeError("ber_counts runs on the ROCm device (no CPU path)")
    counts = torch.zeros((len(outputs), 2), dtype=torch.int64, device=dev)
    yb = None
    if y is not None:
        yb = (y != 0).to(torch.uint8).contiguous()
    L = _lib.lib()
    s = _lib.stream_of(dev)
    for t, o in enumerate(outputs):
        o2 = o.reshape(o.shape[0], -1).to(torch.float32).contiguous()
        _lib.check(L.nldpc_ber_count(o2.data_ptr(), None if yb is None else yb.data_ptr(), o2.shape[0], o2.shape[1],
                                     int(convention), counts[t].data_ptr(), s), "nldpc_ber_count")
    return counts
