"""AWGN-channel data for the boosted decoder (host, numpy).

Reference: src/boosted_neural_ldpc_decoder/AWGNPassedDatagen.py:14-203.  Same constructor, call
signature (`gentype` "per_snr" / "mix_snr"), RNG streams and values: codeword c is drawn with the
noise RandomState(awgn_noise_seed) and codeword RandomState(wordgen_random_seed) in the reference's
order, BPSK maps bit 0 -> -1, LLR = 2 y / sigma^2 in float64, QMS inputs quantised, punctured bits
set to 0 (0.001 for SP).  Outputs X [B, N, Z] float64 and Y [B, N*Z] int64, like the reference.
The reference's per-codeword np.vstack loop (O(B^2) copying) is replaced by one vectorised draw;
numpy's legacy generators produce the same stream either way (pinned by tests/golden/datagen_*).
Kept quirks: "per_snr" uses only the first SNR; the code rate counts
len(Puncture(0, 0)) == 1 (Q4).  Divergence: shortening writes -allowed_llr_range.end where the
reference raises AttributeError (Clipping has no `.abs`).
"""
import numpy as np
from numpy.random import RandomState

from boosted_neural_ldpc_decoder.Functions import Functions
from boosted_neural_ldpc_decoder.struct.Clipping import Clipping
from boosted_neural_ldpc_decoder.struct.DecoderType import DecoderType
from boosted_neural_ldpc_decoder.struct.Puncture import Puncture
from boosted_neural_ldpc_decoder.struct.Shortening import Shortening


class AWGNPassedDatagen:
    def __init__(self, N: int, M: int, snr_db: np.ndarray, awgn_noise_seed: int = 2042,
                 wordgen_random_seed: int = 1074, x_dtype=np.float32, y_dtype=np.int64, gen_matrix: np.ndarray = None,
                 puncturing: Puncture = Puncture(0, 0), shortening: Shortening = Shortening(0, 0),
                 allowed_llr_range: Clipping = Clipping(abs=20.0)):
        self.N = N
        self.M = M
        self.K = N - M
        self.snr_db = snr_db
        self.code_rate = 1.0 * self.K / (N - len(puncturing) - len(shortening))
        self.snr_lin = 10.0 ** (self.snr_db / 10.0)
        self.snr_sigma = np.sqrt(1.0 / (2.0 * self.snr_lin * self.code_rate))
        self._awgn_noise_random = RandomState(awgn_noise_seed)
        self._wordgen_random = RandomState(wordgen_random_seed)
        self.x_dtype = x_dtype
        self.y_dtype = y_dtype
        self.gen_matrix = gen_matrix
        self.puncturing = puncturing
        self.shortening = shortening
        self.allowed_llr_range = allowed_llr_range

    def __call__(self, gentype: str = "per_snr", *args, **kwargs):
        if gentype == "per_snr":
            return self._gendata_per_snr(*args, **kwargs)
        if gentype == "mix_snr":
            return self._gendata_mixed(*args, **kwargs)
        raise AttributeError('attribute `gentype` must be "per_snr" or "mix_snr".')

    def _gendata_per_snr(self, word_length: int, Z: int, is_y_all_zero: bool = True,
                         decoding_type: DecoderType = DecoderType.MS, decoder_qms_qbit: int = 5):
        if word_length <= 0:
            raise ValueError("word_length must be positive integer")
        sigmas = np.full(word_length, np.asarray(self.snr_sigma).reshape(-1)[0])
        return self._generate(sigmas, Z, is_y_all_zero, decoding_type, decoder_qms_qbit)

    def _gendata_mixed(self, word_length: int, Z: int, is_y_all_zero: bool = True,
                       decoding_type: DecoderType = DecoderType.MS, decoder_qms_qbit: int = 5):
        if word_length <= 0:
            raise ValueError("word_length must be positive integer")
        s = np.asarray(self.snr_sigma).reshape(-1)
        return self._generate(s[np.arange(word_length) % len(s)], Z, is_y_all_zero, decoding_type, decoder_qms_qbit)

    def _generate(self, sigmas, Z, is_y_all_zero, decoding_type, q):
        B = len(sigmas)
        Y = self._gen_y(B, Z, is_y_all_zero)
        noise = self._awgn_noise_random.normal(0.0, 1.0, Y.shape)
        sf = sigmas[:, None]
        X = 2 * (noise * sf + (-1) ** (1 - Y)) / (sf ** 2)
        if decoding_type == DecoderType.QMS:
            X = Functions.Cal_MSA_Q(X, q)
        if self.puncturing.start > 0:
            X[:, self.puncturing.start - 1:self.puncturing.end] = 0.001 if decoding_type == DecoderType.SP else 0
        if self.shortening.start > 0:
            X[:, self.shortening.start - 1:self.shortening.end] = -abs(self.allowed_llr_range.end)
        X = X.astype(np.result_type(self.x_dtype, np.float64), copy=False)
        Y = Y.astype(np.result_type(self.y_dtype, Y.dtype), copy=False)
        return np.reshape(X, [B, self.N, Z]), Y

    def _gen_y(self, word_length: int, Z: int, is_y_all_zero: bool) -> np.ndarray:
        if is_y_all_zero:
            return np.zeros([word_length, self.N * Z], dtype=self.y_dtype)
        if self.gen_matrix is None:
            raise ValueError("gen_matrix must be provided when is_y_all_zero is False")
        info = self._wordgen_random.randint(0, 2, size=(word_length, self.K * Z))
        return np.dot(info, self.gen_matrix) % 2
