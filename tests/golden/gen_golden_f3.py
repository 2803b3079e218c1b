"""Golden fixtures for the stateful parts of BoostedNeuralLDPCDecoder.forward, made by
running the REFERENCE in the development container (like gen_golden.py; the GPU box never sees it).

Each fixture is a sequence of forward calls on one module, the last one with gradients:
  stateful_*_listxa      list-valued xa (one channel tensor per iteration, fixed_iter=[]): the state
                         flows from iteration to iteration inside one call, gradients through it
                         (BoostedNeuralLDPCDecoder.py:300-323, 376-377, 512)
  stateful_*_resume      call 1 (no_grad) decodes iterations 0..3, call 2 (grad) decodes 4..7 from
                         the stored self.llr[4] (:343, :377) -- the train loop's fixed_iter > 0 case
  stateful_*_fullresume  call 1 (no_grad) decodes all T, call 2 (grad) target_iter=[3, 4, 5] resumes
                         from the state after iteration 2 of call 1
  stateful_*_split       one call, target_iter=[0, 1, 2, 5, 6]: iteration 5 resumes from the initial
                         zero state, with the cumulative VN weights of 0..2 applied (:325-337)
Stored: inputs, parameters, each call's iteration list, the last call's outputs, LDPCDecoderLoss BCE
value and parameter gradients.

Run (from the repo root):  PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_golden_f3.py
"""
import argparse
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    args = ap.parse_args()
    sys.path.insert(0, os.path.join(args.ref, "src"))
    res = os.path.join(args.ref, "resources")
    import boosted_neural_ldpc_decoder as bref
    from boosted_neural_ldpc_decoder.BoostedNeuralLDPCDecoder import BoostedNeuralLDPCDecoder
    from boosted_neural_ldpc_decoder.LDPCDecoderLoss import LDPCDecoderLoss
    from boosted_neural_ldpc_decoder.struct.DecoderType import DecoderType
    from boosted_neural_ldpc_decoder.struct.LossType import LossType
    from boosted_neural_ldpc_decoder.struct.NodeWeightSharingConfig import NodeWeightSharingConfig as NW

    torch.manual_seed(0)
    bg2 = np.loadtxt(os.path.join(res, "basegraph2_set0.txt"), int, delimiter="\t")
    gen16 = np.loadtxt(os.path.join(res, "gen_matrix_bg2_z16.txt"), int, delimiter=",")
    N, M, Z, B = bg2.shape[1], bg2.shape[0], 16, 4

    def channel(dtype, q, seed):
        dg = bref.AWGNPassedDatagen(N=N, M=M, snr_db=np.array([1.5, 2.0]), awgn_noise_seed=seed,
                                    wordgen_random_seed=seed + 1, gen_matrix=gen16)
        X, Y = dg(gentype="mix_snr", word_length=B, Z=Z, is_y_all_zero=False, decoding_type=dtype, decoder_qms_qbit=q)
        return np.reshape(X, [B, N, Z]).astype(np.float32), np.asarray(Y)

    def case(name, dtype, q, nw, T, calls, seed):
        """calls: list of (iterations, channel index or list of indices, grad)."""
        conn = bref.ConnectingMatrixTorch(bref.ConnectingMatrix(Z, bg2.copy()), device=torch.device("cpu"))
        model = BoostedNeuralLDPCDecoder(iter_node_counts=T, batch_size=B, connecting_matrix=conn,
                                         node_weight_sharing_config=NW(*nw), decoding_type=dtype, decoder_qms_qbit=q)
        r = np.random.default_rng(seed)
        params = {}
        with torch.no_grad():
            for pname, p in model.named_parameters():
                v = r.uniform(0.6, 1.4, tuple(p.shape)).astype(np.float32)
                p.copy_(torch.from_numpy(v))
                params["param__" + pname] = v
        xs, ys = zip(*[channel(dtype, q, seed + 10 * k) for k in range(T + 2)])
        store = {f"x{k}": x for k, x in enumerate(xs)}
        store["y"] = ys[0].astype(np.int8)
        for c, (iters, xsel, grad) in enumerate(calls):
            store[f"call{c}_iters"] = np.array(iters, np.int32)
            store[f"call{c}_x"] = np.array(xsel if isinstance(xsel, list) else [xsel], np.int32)
            store[f"call{c}_listed"] = np.int32(isinstance(xsel, list))
            xin = [torch.from_numpy(xs[k]) for k in xsel] if isinstance(xsel, list) else torch.from_numpy(xs[xsel])
            kw = {"fixed_iter": []} if isinstance(xsel, list) else {}
            if grad:
                outs = model(xin, target_iter=list(iters), **kw)
                yt = torch.from_numpy(ys[0].astype(np.float32))
                loss = LDPCDecoderLoss(loss_type=LossType.BCE, etha=1.0)(outs, yt, coeff_param=list(range(len(outs))))
                loss.backward()
                store["outputs"] = np.stack([o.detach().numpy() for o in outs]).astype(np.float32)
                store["loss"] = np.float32(loss.item())
                for n, p in model.named_parameters():
                    if p.grad is not None:
                        store["grad__" + n] = p.grad.numpy().astype(np.float32)
            else:
                with torch.no_grad():
                    model(xin, target_iter=list(iters), **kw)
        store.update(T=np.int32(T), Z=np.int32(Z), q=np.int32(q), dtype=np.int32(dtype.value), nw=np.array(nw, np.int32),
                     ncalls=np.int32(len(calls)))
        path = os.path.join(HERE, name + ".npz")
        np.savez_compressed(path, **store, **params)
        print(f"wrote {name}.npz ({os.path.getsize(path) / 1024:.1f} KiB)")

    QMS, MS = DecoderType.QMS, DecoderType.MS
    case("stateful_bg2_z16_qms5_nw303_listxa", QMS, 5, (3, 0, 3), 6, [(list(range(6)), list(range(6)), True)], 600)
    case("stateful_bg2_z16_ms_nw112_listxa", MS, 5, (1, 1, 2), 5, [(list(range(5)), list(range(5)), True)], 610)
    case("stateful_bg2_z16_qms5_nw303_resume", QMS, 5, (3, 0, 3), 8,
         [(list(range(0, 4)), 0, False), (list(range(4, 8)), 1, True)], 620)
    case("stateful_bg2_z16_ms_nw223_fullresume", MS, 5, (2, 2, 3), 8,
         [(list(range(8)), 0, False), ([3, 4, 5], 1, True)], 630)
    case("stateful_bg2_z16_qms5_nw213_split", QMS, 5, (2, 1, 3), 8, [([0, 1, 2, 5, 6], 0, True)], 640)


if __name__ == "__main__":
    main()
