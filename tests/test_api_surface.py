"""CPU tests of the drop-in boundary (no GPU): import surface, constructors, parameter registry,
dense routing matrices, datagen, loss and quantiser parity with the reference's golden fixtures."""
import os

import numpy as np
import pytest
import torch

from conftest import ROOT

BG2 = np.loadtxt(os.path.join(ROOT, "resources", "basegraph2_set0.txt"), int, delimiter="\t")
WIMAX = np.loadtxt(os.path.join(ROOT, "resources", "wman_N0576_R34_z24.txt"), int, delimiter="\t")
GEN16 = np.loadtxt(os.path.join(ROOT, "resources", "gen_matrix_bg2_z16.txt"), int, delimiter=",")


def test_import_surface_like_reference_tests():
    # test/test_neural_ldpc_decoder/test_NeuralLDPCDecoder.py:8-11 imports submodules and calls them
    import neural_ldpc_decoder.AWGNPassedDatagen as AWGNPassedDatagen
    import neural_ldpc_decoder.ConnectingMatrix as ConnectingMatrix
    import neural_ldpc_decoder.ConnectingMatrixTorch as ConnectingMatrixTorch
    import neural_ldpc_decoder.NeuralLDPCDecoder as NeuralLDPCDecoder
    for c in (AWGNPassedDatagen, ConnectingMatrix, ConnectingMatrixTorch, NeuralLDPCDecoder):
        assert isinstance(c, type)
    # train/train_BoostedNeuralLDPCDecoder.py:8-19
    from boosted_neural_ldpc_decoder import ConnectingMatrixTorch, ConnectingMatrix, AWGNPassedDatagen, Functions  # noqa
    from boosted_neural_ldpc_decoder.BoostedNeuralLDPCDecoder import BoostedNeuralLDPCDecoder  # noqa
    from boosted_neural_ldpc_decoder.struct.Clipping import Clipping  # noqa
    from boosted_neural_ldpc_decoder.struct.DecoderType import DecoderType  # noqa
    from boosted_neural_ldpc_decoder.LDPCDecoderLoss import LDPCDecoderLoss  # noqa
    from boosted_neural_ldpc_decoder.struct.LearningRate import LearningRate  # noqa
    from boosted_neural_ldpc_decoder.struct.LossType import LossType  # noqa
    from boosted_neural_ldpc_decoder.struct.NodeWeightSharingConfig import NodeWeightSharingConfig  # noqa
    from boosted_neural_ldpc_decoder.struct.Puncture import Puncture  # noqa
    from boosted_neural_ldpc_decoder.struct.Shortening import Shortening  # noqa
    from boosted_neural_ldpc_decoder.struct.NodeType import NodeType  # noqa
    from boosted_neural_ldpc_decoder.struct.ParamType import ParamType  # noqa
    from checkpoint_utils import CheckPointUtil, MetricsLogger  # noqa
    import boosted_neural_ldpc_decoder.Debug  # noqa


def test_struct_semantics():
    from boosted_neural_ldpc_decoder.struct.Clipping import Clipping
    from boosted_neural_ldpc_decoder.struct.DecoderType import DecoderType
    from boosted_neural_ldpc_decoder.struct.LearningRate import LearningRate
    from boosted_neural_ldpc_decoder.struct.NodeType import NodeType
    from boosted_neural_ldpc_decoder.struct.NodeWeightSharingConfig import NodeWeightSharingConfig as NW
    from boosted_neural_ldpc_decoder.struct.Puncture import Puncture
    from boosted_neural_ldpc_decoder.struct.Shortening import Shortening
    assert (DecoderType.SP.value, DecoderType.MS.value, DecoderType.QMS.value) == (0, 1, 2)
    c = Clipping(abs=-3.0)
    assert (c.start, c.end) == (-3.0, 3.0)
    c = Clipping(start=0, end=2)
    assert (c.start, c.end) == (0, 2)
    with pytest.raises(ValueError):
        Clipping(start=1)
    assert len(Puncture(0, 0)) == 1 and len(Shortening(3, 7)) == 5
    with pytest.raises(ValueError):
        Puncture(3, 1)
    with pytest.raises(ValueError):
        Shortening(-1, 2)
    nw = NW(3, 0, 2)
    assert list(nw) == [(NodeType.CN, 3), (NodeType.UCN, 0), (NodeType.VN, 2)]
    assert nw.get(NodeType.VN) == 2
    lr = LearningRate(1.0, 0.5, 2)
    assert [lr() for _ in range(5)] == [1.0, 1.0, 0.5, 0.5, 0.25]
    assert LearningRate(0.1, 0, 5)() == 0.1


def _boosted(nw, T=4, B=3, fixed=(), **kw):
    import boosted_neural_ldpc_decoder as bd
    from boosted_neural_ldpc_decoder.BoostedNeuralLDPCDecoder import BoostedNeuralLDPCDecoder
    from boosted_neural_ldpc_decoder.struct.NodeWeightSharingConfig import NodeWeightSharingConfig as NW
    conn = bd.ConnectingMatrixTorch(bd.ConnectingMatrix(16, BG2))
    return BoostedNeuralLDPCDecoder(T, B, conn, node_weight_sharing_config=NW(*nw), fixed_iterative_nodes=list(fixed),
                                    **kw)


def test_boosted_parameter_registry_matches_reference(golden):
    # names and shapes of the reference model of the config-5 fixture (48 state_dict keys there,
    # 8 of them dense buffers this build does not register)
    d = golden("train_bg2_z16_qms5_nw303_t20")
    m = _boosted((3, 0, 3), T=20, B=20)
    ref = {k[7:]: v.shape for k, v in d.items() if k.startswith("param__")}
    got = {k: tuple(v.shape) for k, v in m.named_parameters()}
    assert got == ref
    d = golden("boosted_bg2_z16_qms5_nw112")
    m = _boosted((1, 1, 2), T=10, B=4)
    assert {k: tuple(v.shape) for k, v in m.named_parameters()} == {k[7:]: v.shape for k, v in d.items()
                                                                     if k.startswith("param__")}
    assert len(m.get_trainable_parameters()) == 30


def test_boosted_fetch_param_temporal_and_constraints():
    from boosted_neural_ldpc_decoder.struct.NodeType import NodeType
    from boosted_neural_ldpc_decoder.struct.ParamType import ParamType
    m = _boosted((4, 0, 0), T=10, fixed=(0, 5))
    names = sorted(n for n, _ in m.named_parameters())
    assert names == ["weight_CN_0", "weight_CN_5"]
    assert m.fetch_param(ParamType.Weight, NodeType.CN, 3) is m.weight_CN_0
    assert m.fetch_param(ParamType.Weight, NodeType.CN, 7) is m.weight_CN_5
    assert m.fetch_param(ParamType.Weight, NodeType.VN, 7) is None
    with torch.no_grad():
        m.weight_CN_5.fill_(3.0)
        m.weight_CN_0.fill_(-1.0)
    m._apply_constraints()
    assert float(m.weight_CN_5.max()) == 2.0 and float(m.weight_CN_0.min()) == 0.0
    with pytest.raises(ValueError):
        _boosted((6, 0, 0))
    m = _boosted((3, 0, 3), T=6, fixed_iterative_nodes_init_weight=2)
    assert len(m.get_trainable_parameters()) == 8  # iterations < 2 are frozen


def test_boosted_tied_rows_and_multi_tensor_clamps():
    """Sharing code 3: the rows the forward stacks as one expand of the stacked scalars (_tied_rows) equal
    the per-iteration expands (_iteration_weights), and their gradient reaches every parameter; the
    multi-tensor _apply_constraints equals clamp_(lo, hi) per parameter, values outside on both sides."""
    from boosted_neural_ldpc_decoder.struct.NodeType import NodeType
    m = _boosted((3, 3, 3), T=5)
    g = torch.Generator().manual_seed(3)
    with torch.no_grad():
        for p_ in m.parameters():
            p_.copy_(torch.randn(p_.shape, generator=g) * 3)
    run = [0, 1, 2, 3, 4]
    for nt, width in ((NodeType.CN, int(m.sum_edge)), (NodeType.UCN, int(m.sum_edge)), (NodeType.VN, m.N)):
        rows = m._tied_rows(nt, run, width)
        k = {NodeType.CN: 0, NodeType.UCN: 1, NodeType.VN: 2}[nt]
        ref = torch.stack([m._iteration_weights(t, [], None, 0, torch.device("cpu"))[k] for t in run])
        assert torch.equal(rows, ref)
    rows = m._tied_rows(NodeType.CN, run, int(m.sum_edge))
    rows.sum().backward()
    for t in run:
        assert float(m.weight_CN_3.grad if t == 3 else getattr(m, f"weight_CN_{t}").grad) == float(m.sum_edge)
    want = {n: p_.detach().clone().clamp_(m.allowed_weight_range.start, m.allowed_weight_range.end)
            for n, p_ in m.named_parameters()}
    m._apply_constraints()
    for n, p_ in m.named_parameters():
        assert torch.equal(p_.detach(), want[n]), n


def test_neural_parameters_and_state_dict_compat():
    import neural_ldpc_decoder as nd
    conn = nd.ConnectingMatrixTorch(nd.ConnectingMatrix(16, BG2))
    m = nd.NeuralLDPCDecoder(5, 1, conn)
    keys = list(m.state_dict().keys())
    assert keys == [f"weights_var.{i}" for i in range(5)] + [f"biases_var.{i}" for i in range(5)]
    assert all(float(p.mean()) == 0.5 for p in m.weights_var) and all(float(p.abs().sum()) == 0 for p in m.biases_var)
    # a reference checkpoint also carries the dense routing buffers: accepted and ignored
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    sd["W_odd2even"] = torch.zeros(3, 3)
    sd["Lift_Matrix1"] = torch.zeros(3, 3)
    sd["weights_var.2"] = torch.full((197,), 0.25)
    m.load_state_dict(sd)
    assert float(m.weights_var[2].mean()) == 0.25


@pytest.mark.parametrize("tag,bg", [("bg2_z16", BG2), ("wimax_z24", WIMAX)])
def test_dense_matrices_match_reference(golden, tag, bg):
    import boosted_neural_ldpc_decoder as bd
    d = golden("graph_" + tag)
    Z = int(d["Z"])
    cm = bd.ConnectingMatrix(Z, bg)
    ct = bd.ConnectingMatrixTorch(cm)
    assert (cm.M, cm.N, cm.Z, int(cm.sum_edge)) == (bg.shape[0], bg.shape[1], Z, int((bg != -1).sum()))
    assert np.array_equal(cm.sum_edge_c, d["sum_edge_c"]) and np.array_equal(cm.sum_edge_v, d["sum_edge_v"])
    for name in ("W_odd2even", "W_skipconn2even", "W_even2odd", "W_even2odd_with_self", "W_output", "W_skipconn2odd"):
        got = np.stack(np.nonzero(getattr(cm, name)), 1)
        assert np.array_equal(got, d[name]), name
        assert torch.equal(getattr(ct, name), torch.from_numpy(getattr(cm, name)))
    assert np.array_equal(np.argmax(cm.lifting_matrix_1, 1), d["lift1"])
    assert np.array_equal(np.argmax(cm.lifting_matrix_2, 1), d["lift2"])


def test_graph_tables():
    from nldpc.graph import LiftedGraph
    g = LiftedGraph(BG2, 384)
    assert (g.M, g.N, g.E) == (42, 52, 197)
    assert g.deg_v.max() == 23 and g.deg_c.max() == 10 and int((g.deg_v == 1).sum()) == 38
    assert np.all(g.shift == BG2[g.chk, g.var] % 384)
    assert np.all(np.diff(g.chk) >= 0)  # C-order
    with pytest.raises(RuntimeError):
        g.handle(torch.device("cpu"))  # there is no CPU decode path


@pytest.mark.parametrize("gentype", ["per_snr", "mix_snr"])
@pytest.mark.parametrize("dt", ["QMS", "MS", "SP"])
def test_boosted_datagen_matches_reference(golden, gentype, dt):
    import boosted_neural_ldpc_decoder as bd
    from boosted_neural_ldpc_decoder.struct.DecoderType import DecoderType
    d = golden(f"datagen_boosted_{gentype}_{dt}")
    g = bd.AWGNPassedDatagen(N=52, M=42, snr_db=np.array([2.0, 2.5, 3.0]), gen_matrix=GEN16)
    X, Y = g(gentype=gentype, word_length=6, Z=16, is_y_all_zero=False, decoding_type=DecoderType[dt],
             decoder_qms_qbit=5)
    X2, Y2 = g(gentype=gentype, word_length=5, Z=16, is_y_all_zero=True, decoding_type=DecoderType[dt],
               decoder_qms_qbit=5)
    assert X.dtype == d["X"].dtype and Y.dtype == np.int64
    assert np.array_equal(X, d["X"]) and np.array_equal(Y, d["Y"])
    assert np.array_equal(X2, d["X2"]) and np.array_equal(Y2, d["Y2"])


def test_datagen_puncture_and_neural(golden):
    import boosted_neural_ldpc_decoder as bd
    import neural_ldpc_decoder as nd
    from boosted_neural_ldpc_decoder.struct.DecoderType import DecoderType
    from boosted_neural_ldpc_decoder.struct.Puncture import Puncture
    d = golden("datagen_boosted_puncture")
    g = bd.AWGNPassedDatagen(N=52, M=42, snr_db=np.array([2.0]), gen_matrix=GEN16, puncturing=Puncture(1, 16))
    assert g.code_rate == float(d["code_rate"])
    X, _ = g(gentype="per_snr", word_length=3, Z=16, is_y_all_zero=False, decoding_type=DecoderType.MS)
    Xs, _ = g(gentype="mix_snr", word_length=3, Z=16, is_y_all_zero=False, decoding_type=DecoderType.SP)
    assert np.array_equal(X, d["X"]) and np.array_equal(Xs, d["Xs"])
    d = golden("datagen_neural")
    g = nd.AWGNPassedDatagen(N=52, M=42, snr_db=np.array([1.0, 3.0]), gen_matrix=GEN16)
    xa, ya = g(word_length=3, Z=16, is_y_all_zero=False)
    xb, yb = g(word_length=2, Z=16, is_y_all_zero=True)
    assert np.array_equal(np.stack(xa), d["xa"]) and np.array_equal(np.stack(ya), d["ya"])
    assert np.array_equal(np.stack(xb), d["xb"]) and np.array_equal(np.stack(yb), d["yb"])
    with pytest.raises(ValueError):
        g(word_length=0, Z=16)
    with pytest.raises(AttributeError):
        bd.AWGNPassedDatagen(N=52, M=42, snr_db=np.array([2.0]))("bogus", 3, 16)


def test_loss_values_match_reference(golden):
    from boosted_neural_ldpc_decoder.LDPCDecoderLoss import LDPCDecoderLoss
    from boosted_neural_ldpc_decoder.struct.LossType import LossType
    d = golden("loss_values")
    outs = [torch.from_numpy(o) for o in d["outs"]]
    y = torch.from_numpy(d["y"])
    for lt in (LossType.BCE, LossType.SoftBEROnAllZero, LossType.FEROnAllZero):
        for etha in (1.0, 0.5):
            crit = LDPCDecoderLoss(loss_type=lt, etha=etha)
            np.testing.assert_allclose(crit(outs, y, coeff_param=list(range(4))).item(),
                                       float(d[f"{lt.value}_{etha}_list"]), rtol=1e-6)
            np.testing.assert_allclose(crit(outs[0], y, coeff_param=1).item(), float(d[f"{lt.value}_{etha}_single"]),
                                       rtol=1e-6)
    with pytest.raises(ValueError):
        LDPCDecoderLoss()(outs[0], y, coeff_param=[1])
    with pytest.raises(ValueError):
        LDPCDecoderLoss()("x", y)


def test_quantizers_match_reference(golden):
    from boosted_neural_ldpc_decoder import Functions
    d = golden("quantize_values")
    x = torch.from_numpy(d["x"])
    for qb, key in ((6, "q6"), (5, "q5"), (-5, "q5m"), (4, "q4"), (3, "q3"), (7, "q7")):
        assert np.array_equal(Functions.cal_msa_q_torch(x, qb).numpy(), d[key]), key
        np.testing.assert_array_equal(Functions.Cal_MSA_Q(d["x"].astype(np.float64), qb).astype(np.float32), d[key])
    # straight-through gradient: 1 inside the closed clip range
    xr = torch.tensor([-8.0, -7.5, 0.3, 7.5, 9.0], requires_grad=True)
    Functions.cal_msa_q_torch(xr, 5).sum().backward()
    assert xr.grad.tolist() == [0.0, 1.0, 1.0, 1.0, 0.0]


def test_checkpoint_roundtrip(tmp_path):
    import neural_ldpc_decoder as nd
    from checkpoint_utils import CheckPointUtil, MetricsLogger
    conn = nd.ConnectingMatrixTorch(nd.ConnectingMatrix(16, BG2))
    m = nd.NeuralLDPCDecoder(2, 1, conn)
    opt = torch.optim.Adam(m.parameters(), lr=1e-3)
    cu = CheckPointUtil(str(tmp_path / "ck"))
    cu.save("a.pth", m, opt, epoch=3, metrics={"loss": 0.5}, config={"batch_size": 1})
    cu.save_weights("w", m, as_txt=True)
    assert os.path.exists(tmp_path / "ck" / "w_weights_txt" / "index.txt")
    m2 = nd.NeuralLDPCDecoder(2, 1, conn)
    with torch.no_grad():
        m.weights_var[0].fill_(0.9)
    cu.save("b.pth", m)
    ck = cu.load("b.pth", m2)
    assert float(m2.weights_var[0].mean()) == pytest.approx(0.9)
    assert "model_state_dict" in ck
    ml = MetricsLogger(str(tmp_path / "ck"))
    ml.log(0, {"loss": 1.0, "ber_last_iter": 1e-3}, "a.pth", config={"lr": 1})
    ml.log(5, {"loss": 0.5, "ber_last_iter": 1e-4}, "NA")
    lines = open(tmp_path / "ck" / "training_metrics.txt").read().splitlines()
    assert lines[0].startswith("# Training started") and lines[-1].endswith("NA") and "1.000000e-04" in lines[-1]
    assert ml.is_best(0.1) and not ml.is_best(0.2)
