"""Generate the golden fixtures under tests/golden/ by running the REFERENCE implementation.

This script is the only place that imports the reference (ShapeLayer/neural-ldpc-decoder-torch,
read-only at /root/reference).  It runs in the development container only; the GPU box never sees
the reference.  What it writes is data: inputs, parameters and the reference's outputs / losses /
gradients, as small compressed .npz files.  Nothing of the reference's source is stored.

Run (from the repo root):
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_golden.py [--ref /root/reference]

Fixture inventory:
  graph_*.npz          dense routing matrices of the reference ConnectingMatrix as coordinate lists
                       (boosted.../ConnectingMatrix.py:82-163) at BG2 z=16 and WiMAX z=24
  neural_*.npz         NeuralLDPCDecoder.forward outputs (NeuralLDPCDecoder.py:44-100), + grads
  boosted_*.npz        BoostedNeuralLDPCDecoder.forward outputs (BoostedNeuralLDPCDecoder.py:260-538)
  train_*.npz          config-5 step: outputs, LDPCDecoderLoss value and parameter grads
  datagen_*.npz        AWGNPassedDatagen outputs for fixed seeds (both packages)
  loss_*.npz           LDPCDecoderLoss values for the three LossTypes
  ber_*.npz            Functions.evaluate_ber_fer literal outputs
"""
import argparse
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))


def _save(name, **arrs):
    path = os.path.join(HERE, name + ".npz")
    np.savez_compressed(path, **arrs)
    print(f"wrote {name}.npz  ({os.path.getsize(path) / 1024:.1f} KiB)")


def _coords(m):
    r, c = np.nonzero(np.asarray(m))
    return np.stack([r, c], 1).astype(np.int32)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    args = ap.parse_args()
    sys.path.insert(0, os.path.join(args.ref, "src"))
    res = os.path.join(args.ref, "resources")

    import neural_ldpc_decoder as nref
    import boosted_neural_ldpc_decoder as bref
    from boosted_neural_ldpc_decoder.BoostedNeuralLDPCDecoder import BoostedNeuralLDPCDecoder
    from boosted_neural_ldpc_decoder.LDPCDecoderLoss import LDPCDecoderLoss
    from boosted_neural_ldpc_decoder.struct.DecoderType import DecoderType
    from boosted_neural_ldpc_decoder.struct.LossType import LossType
    from boosted_neural_ldpc_decoder.struct.NodeWeightSharingConfig import NodeWeightSharingConfig as NW
    from boosted_neural_ldpc_decoder.struct.Puncture import Puncture
    from boosted_neural_ldpc_decoder.struct.Shortening import Shortening
    from boosted_neural_ldpc_decoder.Functions import Functions

    torch.manual_seed(0)
    bg2 = np.loadtxt(os.path.join(res, "basegraph2_set0.txt"), int, delimiter="\t")
    wimax = np.loadtxt(os.path.join(res, "wman_N0576_R34_z24.txt"), int, delimiter="\t")
    gen16 = np.loadtxt(os.path.join(res, "gen_matrix_bg2_z16.txt"), int, delimiter=",")

    # ---------------------------------------------------------------- graphs (C3-1)
    for tag, bg, Z in (("bg2_z16", bg2, 16), ("wimax_z24", wimax, 24)):
        cm = bref.ConnectingMatrix(Z, bg.copy())
        _save(
            "graph_" + tag,
            basegraph=bg.astype(np.int32), Z=np.int32(Z),
            W_odd2even=_coords(cm.W_odd2even), W_skipconn2even=_coords(cm.W_skipconn2even),
            W_even2odd=_coords(cm.W_even2odd), W_even2odd_with_self=_coords(cm.W_even2odd_with_self),
            W_output=_coords(cm.W_output), W_skipconn2odd=_coords(cm.W_skipconn2odd),
            lift1=np.argmax(cm.lifting_matrix_1, axis=1).astype(np.int32),
            lift2=np.argmax(cm.lifting_matrix_2, axis=1).astype(np.int32),
            sum_edge_c=cm.sum_edge_c.astype(np.int32), sum_edge_v=cm.sum_edge_v.astype(np.int32),
        )

    def awgn_llr(rng, B, N, Z, ebn0_db, rate, y=None):
        sigma = np.sqrt(1.0 / (2.0 * rate * 10.0 ** (ebn0_db / 10.0)))
        bits = np.zeros((B, N * Z), np.int64) if y is None else y
        x = (-1.0) ** (1 - bits) + sigma * rng.standard_normal((B, N * Z))
        return (2.0 * x / sigma ** 2).astype(np.float32).reshape(B, N, Z), bits

    # ---------------------------------------------------------------- neural (C3-2, C3-3)
    def neural_case(name, bg, Z, T, x, y, weights=None, biases=None, grads=False):
        conn = nref.ConnectingMatrixTorch(nref.ConnectingMatrix(Z, bg.copy()), device=torch.device("cpu"))
        model = nref.NeuralLDPCDecoder(T, x.shape[0], conn)
        E = int(conn.sum_edge)
        if weights is not None:
            with torch.no_grad():
                for t in range(T):
                    model.weights_var[t].copy_(torch.from_numpy(weights[t]))
                    model.biases_var[t].copy_(torch.from_numpy(biases[t]))
        w = np.stack([p.detach().numpy() for p in model.weights_var]).astype(np.float32)
        b = np.stack([p.detach().numpy() for p in model.biases_var]).astype(np.float32)
        xt = torch.from_numpy(x)
        outs = model(xt)
        extra = {}
        if grads:
            yt = torch.from_numpy(y.astype(np.float32))
            loss = sum(torch.nn.functional.binary_cross_entropy_with_logits(o, yt) for o in outs) / T
            loss.backward()
            extra = dict(
                loss=np.float32(loss.item()),
                grad_w=np.stack([p.grad.numpy() for p in model.weights_var]).astype(np.float32),
                grad_b=np.stack([p.grad.numpy() for p in model.biases_var]).astype(np.float32),
            )
        _save(name, x=x, y=y.astype(np.int8), weights=w, biases=b, T=np.int32(T), Z=np.int32(Z), E=np.int32(E),
              outputs=np.stack([o.detach().numpy() for o in outs]).astype(np.float32), **extra)

    # cfg1: BG2 z=16, batch=1, 5 iters, reference datagen (seeds 2042/1074), Eb/N0 1..4 dB
    N, M = bg2.shape[1], bg2.shape[0]
    dg = nref.AWGNPassedDatagen(N=N, M=M, snr_db=np.array([1.0, 2.0, 3.0, 4.0]), gen_matrix=gen16)
    xs, ys = dg(word_length=1, Z=16, is_y_all_zero=True)
    for k, snr in enumerate((1, 2, 3, 4)):
        x = np.reshape(xs[k], [1, N, 16]).astype(np.float32)
        neural_case(f"neural_cfg1_snr{snr}_default", bg2, 16, 5, x, ys[k])
    rng = np.random.default_rng(11)
    T = 5
    E = 197
    wr = rng.uniform(0.0, 1.5, (T, E)).astype(np.float32)
    br = rng.normal(0.0, 0.1, (T, E)).astype(np.float32)
    neural_case("neural_cfg1_snr2_random", bg2, 16, T, np.reshape(xs[1], [1, N, 16]).astype(np.float32), ys[1],
                wr, br)
    # B=16 random codewords via G, random params, grads through all outputs
    dg2 = nref.AWGNPassedDatagen(N=N, M=M, snr_db=np.array([1.5]), gen_matrix=gen16, awgn_noise_seed=7,
                                 wordgen_random_seed=8)
    xs2, ys2 = dg2(word_length=16, Z=16, is_y_all_zero=False)
    x16 = np.reshape(xs2[0], [16, N, 16]).astype(np.float32)
    # neural datagen maps every bit to -1 (reference quirk Q2): keep its y for the loss anyway
    neural_case("neural_bg2_z16_b16_t5_random", bg2, 16, T, x16, ys2[0], wr, br, grads=True)
    # WiMAX z=24, B=16, T=20, all-zero, random params
    Nw, Mw = wimax.shape[1], wimax.shape[0]
    Ew = int((wimax != -1).sum())
    rw = np.random.default_rng(12)
    xw, yw = awgn_llr(rw, 16, Nw, 24, 2.0, (Nw - Mw) / (Nw - 2))
    ww = rw.uniform(0.2, 1.2, (20, Ew)).astype(np.float32)
    bw = rw.normal(0.0, 0.1, (20, Ew)).astype(np.float32)
    neural_case("neural_wimax_z24_b16_t20_random", wimax, 24, 20, xw, yw, ww, bw, grads=True)

    # ---------------------------------------------------------------- boosted (C3-4, C3-5)
    def boosted_case(name, bg, Z, T, B, dtype, q, nw, x, y, seed, fixed_nodes=(), target_iter=None,
                     loss_step=False, store_outputs=True, init_range=(0.5, 1.5)):
        conn = bref.ConnectingMatrixTorch(bref.ConnectingMatrix(Z, bg.copy()), device=torch.device("cpu"))
        model = BoostedNeuralLDPCDecoder(
            iter_node_counts=T, batch_size=B, connecting_matrix=conn,
            node_weight_sharing_config=NW(*nw), decoding_type=dtype, decoder_qms_qbit=q,
            fixed_iterative_nodes=list(fixed_nodes),
        )
        r = np.random.default_rng(seed)
        params = {}
        with torch.no_grad():
            for pname, p in model.named_parameters():
                v = r.uniform(init_range[0], init_range[1], tuple(p.shape)).astype(np.float32)
                p.copy_(torch.from_numpy(v))
                params["param__" + pname] = v
        xt = torch.from_numpy(x)
        if loss_step:
            yt = torch.from_numpy(y.astype(np.float32))
            outs = model(xt, target_iter=list(range(0, T)))
            crit = LDPCDecoderLoss(loss_type=LossType.BCE, etha=1.0)
            loss = crit(outs, yt, coeff_param=list(range(len(outs))))
            loss.backward()
            grads = {"grad__" + n: p.grad.numpy().astype(np.float32) for n, p in model.named_parameters()
                     if p.grad is not None}
            sel = [0, 1, T // 2, T - 1]
            _save(name, x=x, y=y.astype(np.int8), T=np.int32(T), Z=np.int32(Z), q=np.int32(q),
                  dtype=np.int32(dtype.value), nw=np.array(nw, np.int32), loss=np.float32(loss.item()),
                  out_iters=np.array(sel, np.int32),
                  outputs=np.stack([outs[i].detach().numpy() for i in sel]).astype(np.float32), **params, **grads)
            return
        with torch.no_grad():
            outs = model(xt) if target_iter is None else model(xt, target_iter=target_iter)
        if isinstance(outs, torch.Tensor):
            outs = [outs]
        _save(name, x=x, y=y.astype(np.int8), T=np.int32(T), Z=np.int32(Z), q=np.int32(q),
              dtype=np.int32(dtype.value), nw=np.array(nw, np.int32), fixed_nodes=np.array(fixed_nodes, np.int32),
              outputs=np.stack([o.numpy() for o in outs]).astype(np.float32), **params)

    def boosted_input(dtype, q, B, seed, snr=(1.5, 2.0, 2.5), Z=16, bg=bg2, gen=gen16):
        Nn, Mm = bg.shape[1], bg.shape[0]
        dgb = bref.AWGNPassedDatagen(N=Nn, M=Mm, snr_db=np.array(snr), awgn_noise_seed=seed,
                                     wordgen_random_seed=seed + 1, gen_matrix=gen)
        X, Y = dgb(gentype="mix_snr", word_length=B, Z=Z, is_y_all_zero=gen is None, decoding_type=dtype,
                   decoder_qms_qbit=q)
        return np.reshape(X, [B, Nn, Z]).astype(np.float32), Y

    QMS, MS, SP = DecoderType.QMS, DecoderType.MS, DecoderType.SP
    combos = [
        ("qms5_nw303", QMS, 5, (3, 0, 3)),
        ("qms5_nw333", QMS, 5, (3, 3, 3)),
        ("qms5_nw112", QMS, 5, (1, 1, 2)),
        ("qms5_nw220", QMS, 5, (2, 2, 0)),
        ("qms5_nw100", QMS, 5, (1, 0, 0)),
        ("qms5_nw000", QMS, 5, (0, 0, 0)),
        ("qms5_nw213", QMS, 5, (2, 1, 3)),
        ("qms6_nw303", QMS, 6, (3, 0, 3)),
        ("qms4_nw303", QMS, 4, (3, 0, 3)),
        ("qms3_nw303", QMS, 3, (3, 0, 3)),
        ("qmsm5_nw303", QMS, -5, (3, 0, 3)),
        ("ms_nw303", MS, 5, (3, 0, 3)),
        ("ms_nw112", MS, 5, (1, 1, 2)),
        ("ms_nw223", MS, 5, (2, 2, 3)),
        ("ms_nw330", MS, 5, (3, 3, 0)),
        ("sp_nw303", SP, 5, (3, 0, 3)),
        ("sp_nw112", SP, 5, (1, 1, 2)),
        ("sp_nw220", SP, 5, (2, 2, 0)),
    ]
    for k, (tag, dt, q, nw) in enumerate(combos):
        x, y = boosted_input(dt, q, 4, 100 + k)
        boosted_case(f"boosted_bg2_z16_{tag}", bg2, 16, 10, 4, dt, q, nw, x, y, seed=200 + k)
    # temporal (code 4) sharing with fixed iterative nodes
    x, y = boosted_input(QMS, 5, 4, 150)
    boosted_case("boosted_bg2_z16_qms5_nw400_fixed", bg2, 16, 10, 4, QMS, 5, (4, 0, 0), x, y, seed=250,
                 fixed_nodes=(0, 5))
    # target_iter as a prefix list
    boosted_case("boosted_bg2_z16_qms5_nw303_target6", bg2, 16, 10, 4, QMS, 5, (3, 0, 3), x, y, seed=251,
                 target_iter=list(range(0, 6)))
    # WiMAX, all-zero codewords
    for k, (tag, dt, q, nw) in enumerate([("qms5_nw112", QMS, 5, (1, 1, 2)), ("ms_nw333", MS, 5, (3, 3, 3)),
                                          ("sp_nw303", SP, 5, (3, 0, 3))]):
        x, y = boosted_input(dt, q, 4, 300 + k, Z=24, bg=wimax, gen=None)
        boosted_case(f"boosted_wimax_z24_{tag}", wimax, 24, 10, 4, dt, q, nw, x, y, seed=310 + k)

    # config-5 training step (train/train_BoostedNeuralLDPCDecoder.py:274-294), one step from fixed weights
    x, y = boosted_input(QMS, 5, 20, 2042, snr=(2, 2.5, 3.0, 3.5, 4.0))
    boosted_case("train_bg2_z16_qms5_nw303_t20", bg2, 16, 20, 20, QMS, 5, (3, 0, 3), x, y, seed=400,
                 loss_step=True, init_range=(0.8, 1.2))
    boosted_case("train_bg2_z16_qms5_nw303_t50", bg2, 16, 50, 20, QMS, 5, (3, 0, 3), x, y, seed=401,
                 loss_step=True, init_range=(0.8, 1.2))
    x4, y4 = boosted_input(MS, 5, 4, 2050)
    boosted_case("train_bg2_z16_ms_nw112_t10", bg2, 16, 10, 4, MS, 5, (1, 1, 2), x4, y4, seed=402,
                 loss_step=True)
    boosted_case("train_bg2_z16_ms_nw220_t10", bg2, 16, 10, 4, MS, 5, (2, 2, 0), x4, y4, seed=403,
                 loss_step=True)
    x5, y5 = boosted_input(QMS, 5, 4, 2051)
    boosted_case("train_bg2_z16_qms5_nw333_t10", bg2, 16, 10, 4, QMS, 5, (3, 3, 3), x5, y5, seed=404,
                 loss_step=True)
    x6, y6 = boosted_input(SP, 5, 4, 2052)
    boosted_case("train_bg2_z16_sp_nw303_t10", bg2, 16, 10, 4, SP, 5, (3, 0, 3), x6, y6, seed=405,
                 loss_step=True)

    # ---------------------------------------------------------------- datagen (C3-7)
    Nb, Mb = bg2.shape[1], bg2.shape[0]
    for gt in ("per_snr", "mix_snr"):
        for dt, q in ((QMS, 5), (MS, 5), (SP, 5)):
            dgb = bref.AWGNPassedDatagen(N=Nb, M=Mb, snr_db=np.array([2.0, 2.5, 3.0]), gen_matrix=gen16)
            X, Y = dgb(gentype=gt, word_length=6, Z=16, is_y_all_zero=False, decoding_type=dt, decoder_qms_qbit=q)
            X2, Y2 = dgb(gentype=gt, word_length=5, Z=16, is_y_all_zero=True, decoding_type=dt, decoder_qms_qbit=q)
            _save(f"datagen_boosted_{gt}_{dt.name}", X=np.asarray(X), Y=np.asarray(Y).astype(np.int8),
                  X2=np.asarray(X2), Y2=np.asarray(Y2).astype(np.int8))
    # shortening with start>0 raises AttributeError in the reference (Clipping has no `.abs`,
    # AWGNPassedDatagen.py:118,177): only puncturing is pinned here.
    dgp = bref.AWGNPassedDatagen(N=Nb, M=Mb, snr_db=np.array([2.0]), gen_matrix=gen16,
                                 puncturing=Puncture(1, 16), shortening=Shortening(0, 0))
    Xp, Yp = dgp(gentype="per_snr", word_length=3, Z=16, is_y_all_zero=False, decoding_type=MS)
    Xs, Ys = dgp(gentype="mix_snr", word_length=3, Z=16, is_y_all_zero=False, decoding_type=SP)
    _save("datagen_boosted_puncture", X=np.asarray(Xp), Y=np.asarray(Yp).astype(np.int8), Xs=np.asarray(Xs),
          Ys=np.asarray(Ys).astype(np.int8), code_rate=np.float64(dgp.code_rate))
    dgn = nref.AWGNPassedDatagen(N=Nb, M=Mb, snr_db=np.array([1.0, 3.0]), gen_matrix=gen16)
    xa, ya = dgn(word_length=3, Z=16, is_y_all_zero=False)
    xb, yb = dgn(word_length=2, Z=16, is_y_all_zero=True)
    _save("datagen_neural", xa=np.stack(xa), ya=np.stack(ya).astype(np.int8), xb=np.stack(xb),
          yb=np.stack(yb).astype(np.int8), code_rate=np.float64(dgn.code_rate))

    # ---------------------------------------------------------------- loss + BER (C3-6)
    r = np.random.default_rng(5)
    outs = [torch.from_numpy(r.normal(0, 3, (3, 40)).astype(np.float32)) for _ in range(4)]
    yy = torch.from_numpy((r.uniform(size=(3, 40)) < 0.3).astype(np.float32))
    res_l = {}
    for lt in (LossType.BCE, LossType.SoftBEROnAllZero, LossType.FEROnAllZero):
        for etha in (1.0, 0.5):
            crit = LDPCDecoderLoss(loss_type=lt, etha=etha)
            res_l[f"{lt.value}_{etha}_list"] = np.float32(crit(outs, yy, coeff_param=list(range(4))).item())
            res_l[f"{lt.value}_{etha}_single"] = np.float32(crit(outs[0], yy, coeff_param=1).item())
    _save("loss_values", outs=np.stack([o.numpy() for o in outs]), y=yy.numpy(), **res_l)
    (be, bits), (fe, frames) = Functions.evaluate_ber_fer(yy, outs)
    _save("ber_values", outs=np.stack([o.numpy() for o in outs]), y=yy.numpy(), bit_errors=np.array(be),
          bits=np.int64(bits), frame_errors=np.array(fe), frames=np.int64(frames))
    q_in = r.normal(0, 6, 2000).astype(np.float32)
    q_in[:16] = [0.25, 0.75, 1.25, -0.25, -0.75, 2.5, 7.5, 7.75, -7.75, 15.5, 16.0, -15.25, 0.0, 1.0, 3.0, 5.0]
    qres = {f"q{abs(qb)}{'m' if qb < 0 else ''}": Functions.cal_msa_q_torch(torch.from_numpy(q_in), qb).numpy()
            for qb in (6, 5, -5, 4, 3, 7)}
    _save("quantize_values", x=q_in, **qres)


if __name__ == "__main__":
    main()
