"""AWGN-channel training data for the Dai et al. decoder (host, numpy).

Reference: src/neural_ldpc_decoder/AWGNPassedDatagen.py:5-98.  Same constructor, call signature,
RNG streams (numpy RandomState seeded with awgn_noise_seed / wordgen_random_seed, consumed in the
same order) and output: lists (one entry per SNR) of x [B, N*Z] float32 LLRs and y [B, N*Z] bits.
Kept quirks: code rate (N-M)/(N-2); every bit is mapped to -1 (the reference's `-1 ** (1 - y)`).
For large synthetic batches use nldpc.channel.awgn_llr (generated on the GPU) instead.
"""
import numpy as np
from numpy.random import RandomState


class AWGNPassedDatagen:
    def __init__(self, N: int, M: int, snr_db: np.ndarray, awgn_noise_seed: int = 2042,
                 wordgen_random_seed: int = 1074, x_dtype=np.float32, y_dtype=np.int64, gen_matrix: np.ndarray = None):
        self.N = N
        self.M = M
        self.K = N - M
        self.snr_db = snr_db
        self.code_rate = 1.0 * (N - M) / (N - 2)
        self.snr_lin = 10.0 ** (self.snr_db / 10.0)
        self.snr_sigma = np.sqrt(1.0 / (2.0 * self.snr_lin * self.code_rate))
        self._awgn_noise_random = RandomState(awgn_noise_seed)
        self._wordgen_random = RandomState(wordgen_random_seed)
        self.x_dtype = x_dtype
        self.y_dtype = y_dtype
        self.gen_matrix = gen_matrix

    def __call__(self, *args, **kwargs):
        return self._gendata(*args, **kwargs)

    def _gendata(self, word_length: int, Z: int, is_y_all_zero: bool = True):
        if word_length <= 0:
            raise ValueError("word_length must be positive integer")
        xs, ys = [], []
        for sigma in self.snr_sigma:
            if is_y_all_zero:
                y = np.dot(np.zeros((word_length, self.K * Z), dtype=self.y_dtype), self.gen_matrix) % 2
            else:
                if self.gen_matrix is None:
                    raise ValueError("self.gen_matrix must be provided when is_y_all_zero is False")
                info = self._wordgen_random.randint(0, 2, size=(word_length, self.K * Z)).astype(self.y_dtype)
                y = np.dot(info, self.gen_matrix) % 2
            noise = self._awgn_noise_random.normal(0.0, 1.0, size=(word_length, self.gen_matrix.shape[1]))
            noise = noise.astype(self.x_dtype)
            # reference quirk: `-1 ** (1 - y)` parses as -(1 ** (1 - y)) == -1 for every bit
            tx = -np.ones_like(y)
            x = (2 * (noise * sigma + tx) / (sigma ** 2)).astype(self.x_dtype)
            xs.append(x)
            ys.append(y)
        return xs, ys
