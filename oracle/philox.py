"""CPU restatement of the device channel generator (nldpc_aux.hip awgn_kernel / nldpc_channel_llr).

TEST INFRASTRUCTURE ONLY (see oracle/ldpc_oracle.py's header for the import rule).

The device draws the synthetic AWGN channel of SURVEY.md §8(d) D2 with Philox-4x32-10 (Salmon et al.,
SC'11; the Random123 constants) keyed by the 64-bit seed, at counter = the global group index
g = (b_offset * L + i) // 4 of each 4 consecutive LLRs, so a rank that starts at codeword b_offset
draws exactly the noise a single device would at those codewords.  Box-Muller in
fp64 turns each counter's 4 words into 4 normals; the LLR is 2 * (-1 + sigma * n) / sigma^2 rounded
to fp32 (the all-zero codeword's BPSK, boosted.../AWGNPassedDatagen.py:97-103).
"""
from __future__ import annotations

import numpy as np

M0, M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
W0, W1 = 0x9E3779B9, 0xBB67AE85
MASK = np.uint64(0xFFFFFFFF)


def philox4x32_10(ctr: np.ndarray, key: tuple[int, int]) -> np.ndarray:
    """ctr: uint32 [n, 4]; key (k0, k1) -> uint32 [n, 4] (Random123 philox4x32, 10 rounds)."""
    c = ctr.astype(np.uint64)
    k0, k1 = int(key[0]) & 0xFFFFFFFF, int(key[1]) & 0xFFFFFFFF
    x, y, z, w = c[:, 0], c[:, 1], c[:, 2], c[:, 3]
    for _ in range(10):
        p0 = M0 * x
        p1 = M1 * z
        hi0, lo0 = p0 >> np.uint64(32), p0 & MASK
        hi1, lo1 = p1 >> np.uint64(32), p1 & MASK
        x, y, z, w = hi1 ^ y ^ np.uint64(k0), lo1, hi0 ^ w ^ np.uint64(k1), lo0
        k0 = (k0 + W0) & 0xFFFFFFFF
        k1 = (k1 + W1) & 0xFFFFFFFF
    return np.stack([x, y, z, w], axis=1).astype(np.uint32)


def awgn_llr(B: int, L: int, sigma: float, seed: int, b_offset: int = 0) -> np.ndarray:
    """fp32 [B, L] LLRs of the all-zero codeword, as nldpc_awgn_llr(xa, B, L, sigma, seed, b_offset, 0)."""
    first = b_offset * L
    idx = np.arange(first, first + B * L, dtype=np.int64)
    groups = np.unique(idx >> 2)
    ctr = np.zeros((len(groups), 4), dtype=np.uint32)
    ctr[:, 0] = (groups & 0xFFFFFFFF).astype(np.uint32)
    ctr[:, 1] = (groups >> 32).astype(np.uint32)
    r = philox4x32_10(ctr, (seed & 0xFFFFFFFF, seed >> 32)).astype(np.float64)
    u = (r + 1.0) * (1.0 / 4294967296.0)
    rad0, th0 = np.sqrt(-2.0 * np.log(u[:, 0])), 6.283185307179586 * u[:, 1]
    rad1, th1 = np.sqrt(-2.0 * np.log(u[:, 2])), 6.283185307179586 * u[:, 3]
    n = np.stack([rad0 * np.cos(th0), rad0 * np.sin(th0), rad1 * np.cos(th1), rad1 * np.sin(th1)], axis=1)
    noise = n.reshape(-1)[idx - groups[0] * 4]
    sg = float(np.float32(sigma))  # the ABI takes sigma as fp32, the kernel computes in fp64
    llr = (2.0 * (-1.0 + sg * noise) / (sg * sg)).astype(np.float32)
    return llr.reshape(B, L)
