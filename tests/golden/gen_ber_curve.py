"""Golden BER curve from the REFERENCE decoder (run in the survey/build container only).

Writes tests/golden/ber_curve_neural_bg2_z16.npz: per-iteration bit/frame error counts of the
reference NeuralLDPCDecoder (default parameters w=0.5, b=0), BG2 z=16, T=20, all-zero codewords,
inputs from the reference neural AWGNPassedDatagen (default seeds 2042/1074), Eb/N0 = 1.0..4.0 dB in
0.5 dB steps, 250 codewords per point -- SURVEY.md §8(d) D2/D7 and BASELINE.md §2's table.
Hard decision: bit = (LLR > 0) (the decoder convention).  Also stores a checksum of each
point's input so a mismatch in the build's datagen restatement is told apart from a decoder mismatch.

    python tests/golden/gen_ber_curve.py [--ref /root/reference]
"""
import argparse
import hashlib
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
SNRS = np.arange(1.0, 4.01, 0.5)
WORDS, T, Z = 250, 20, 16


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    args = ap.parse_args()
    sys.path.insert(0, os.path.join(args.ref, "src"))
    import neural_ldpc_decoder as nref

    res = os.path.join(args.ref, "resources")
    bg2 = np.loadtxt(os.path.join(res, "basegraph2_set0.txt"), int, delimiter="\t")
    gen16 = np.loadtxt(os.path.join(res, "gen_matrix_bg2_z16.txt"), int, delimiter=",")
    M, N = bg2.shape
    dg = nref.AWGNPassedDatagen(N=N, M=M, snr_db=SNRS.copy(), gen_matrix=gen16)
    xs, ys = dg(word_length=WORDS, Z=Z, is_y_all_zero=True)
    conn = nref.ConnectingMatrixTorch(nref.ConnectingMatrix(Z, bg2.copy()), device=torch.device("cpu"))
    model = nref.NeuralLDPCDecoder(T, WORDS, conn)
    bit_err = np.zeros((len(SNRS), T), np.int64)
    frame_err = np.zeros((len(SNRS), T), np.int64)
    x_sha = []
    for k in range(len(SNRS)):
        x = np.reshape(xs[k], [WORDS, N, Z]).astype(np.float32)
        y = np.asarray(ys[k]).reshape(WORDS, N * Z)
        x_sha.append(hashlib.sha256(x.tobytes()).hexdigest())
        with torch.no_grad():
            outs = model(torch.from_numpy(x))
        for t, o in enumerate(outs):
            wrong = (o.numpy() > 0).astype(np.int64) != y
            bit_err[k, t] = wrong.sum()
            frame_err[k, t] = wrong.any(axis=1).sum()
        print(f"Eb/N0 {SNRS[k]:.1f} dB: BER {bit_err[k, -1] / (WORDS * N * Z):.3e} FER {frame_err[k, -1] / WORDS:.3f}",
              flush=True)
    np.savez_compressed(os.path.join(HERE, "ber_curve_neural_bg2_z16.npz"), ebn0_db=SNRS, words=np.int64(WORDS),
                        T=np.int64(T), Z=np.int64(Z), bit_errors=bit_err, frame_errors=frame_err,
                        x_sha256=np.array(x_sha))


if __name__ == "__main__":
    main()
