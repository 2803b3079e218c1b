"""Pin the CPU oracle (oracle/ldpc_oracle.py) against the reference's own outputs.

The fixtures under tests/golden/ were produced by tests/golden/gen_golden.py, which runs the
reference (ShapeLayer/neural-ldpc-decoder-torch) in the development container.  Soft outputs of
every kind (Neural / MS / QMS / SP) must match bit for bit -- SP through the oracle's restatement of
ATen's CPU torch.prod order (oracle/ldpc_oracle.py _prod_aten); gradients within
rtol 1e-4 (batch-sum order).
"""
import glob
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN, ROOT
from oracle.ldpc_oracle import OracleGraph, boosted_forward, neural_forward, quantize

BG2 = np.loadtxt(os.path.join(ROOT, "resources", "basegraph2_set0.txt"), int, delimiter="\t")
WIMAX = np.loadtxt(os.path.join(ROOT, "resources", "wman_N0576_R34_z24.txt"), int, delimiter="\t")

NEURAL = ["neural_cfg1_snr1_default", "neural_cfg1_snr2_default", "neural_cfg1_snr3_default",
          "neural_cfg1_snr4_default", "neural_cfg1_snr2_random", "neural_bg2_z16_b16_t5_random",
          "neural_wimax_z24_b16_t20_random"]
BOOSTED = sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN, "boosted_*.npz")))
TRAIN = sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN, "train_*.npz")))


def _bg(name):
    return WIMAX if "wimax" in name else BG2


def _fetch(d, node, code, fixed, params=None):
    def f(t):
        if code in (1, 2, 3):
            k = t
        elif fixed:
            v = [i for i in fixed if i <= t]
            k = max(v) if v else fixed[0]
        else:
            k = 0
        key = f"weight_{node}_{k}"
        return params[key] if params is not None else torch.from_numpy(d["param__" + key])
    return f


def test_graph_edge_orders_match_reference(golden):
    for tag, bg in (("bg2_z16", BG2), ("wimax_z24", WIMAX)):
        d = golden("graph_" + tag)
        Z = int(d["Z"])
        g = OracleGraph(bg, Z)
        # lifting_matrix_2 (C-order): row e*Z+h has its 1 at e*Z + (h+s_e) mod Z
        exp2 = np.array([e * Z + (h + g.shift[e]) % Z for e in range(g.E) for h in range(Z)])
        assert np.array_equal(d["lift2"], exp2)
        # W_output rows are C-order edges, columns their variable
        wo = d["W_output"]
        assert np.array_equal(g.var[wo[:, 0]], wo[:, 1]) and len(wo) == g.E
        # W_skipconn2odd: [M, E_c] check of each C-order edge
        so = d["W_skipconn2odd"]
        assert np.array_equal(g.chk[so[:, 1]], so[:, 0]) and len(so) == g.E


@pytest.mark.parametrize("name", NEURAL)
def test_oracle_neural_bit_exact(golden, name):
    d = golden(name)
    g = OracleGraph(_bg(name), int(d["Z"]))
    outs = neural_forward(g, torch.from_numpy(d["x"]), [torch.from_numpy(w) for w in d["weights"]],
                          [torch.from_numpy(b) for b in d["biases"]])
    o = torch.stack(outs).numpy()
    assert np.array_equal(o, d["outputs"]), f"{(o != d['outputs']).sum()} soft values differ"


@pytest.mark.parametrize("name", BOOSTED)
def test_oracle_boosted(golden, name):
    d = golden(name)
    g = OracleGraph(_bg(name), int(d["Z"]))
    T = int(d["T"])
    nw = tuple(int(v) for v in d["nw"])
    fixed = [int(v) for v in d.get("fixed_nodes", [])]
    iters = list(range(6)) if "target6" in name else list(range(T))
    outs = boosted_forward(g, torch.from_numpy(d["x"]), dtype=int(d["dtype"]), q=int(d["q"]), nw=nw, iters=iters,
                           w_cn=_fetch(d, "CN", nw[0], fixed), w_ucn=_fetch(d, "UCN", nw[1], fixed),
                           w_vn=_fetch(d, "VN", nw[2], fixed))
    o = torch.stack([outs[i] for i in iters]).numpy()
    ref = d["outputs"]
    assert np.array_equal(o, ref), f"{(o != ref).sum()} soft values differ"


@pytest.mark.parametrize("name", ["neural_bg2_z16_b16_t5_random", "neural_wimax_z24_b16_t20_random"])
def test_oracle_neural_grads(golden, name):
    d = golden(name)
    g = OracleGraph(_bg(name), int(d["Z"]))
    W = [torch.tensor(w, requires_grad=True) for w in d["weights"]]
    Bs = [torch.tensor(b, requires_grad=True) for b in d["biases"]]
    outs = neural_forward(g, torch.from_numpy(d["x"]), W, Bs)
    y = torch.from_numpy(d["y"].astype(np.float32))
    loss = sum(torch.nn.functional.binary_cross_entropy_with_logits(o, y) for o in outs) / len(outs)
    loss.backward()
    np.testing.assert_allclose(loss.item(), float(d["loss"]), rtol=1e-6)
    np.testing.assert_allclose(torch.stack([w.grad for w in W]).numpy(), d["grad_w"], rtol=1e-4,
                               atol=1e-4 * np.abs(d["grad_w"]).max())
    np.testing.assert_allclose(torch.stack([b.grad for b in Bs]).numpy(), d["grad_b"], rtol=1e-4,
                               atol=1e-4 * np.abs(d["grad_b"]).max())


@pytest.mark.parametrize("name", [n for n in TRAIN if "t50" not in n])
def test_oracle_boosted_grads(golden, name):
    d = golden(name)
    g = OracleGraph(BG2, int(d["Z"]))
    T = int(d["T"])
    nw = tuple(int(v) for v in d["nw"])
    P = {k[7:]: torch.tensor(v, requires_grad=True) for k, v in d.items() if k.startswith("param__")}
    outs = boosted_forward(g, torch.from_numpy(d["x"]), dtype=int(d["dtype"]), q=int(d["q"]), nw=nw,
                           iters=list(range(T)), w_cn=_fetch(d, "CN", nw[0], [], P),
                           w_ucn=_fetch(d, "UCN", nw[1], [], P), w_vn=_fetch(d, "VN", nw[2], [], P))
    y = torch.from_numpy(d["y"].astype(np.float32))
    loss = sum(torch.nn.functional.binary_cross_entropy_with_logits(outs[t], y) for t in range(T)) / T
    loss.backward()
    tol = 1e-4
    for k, p in P.items():
        if "grad__" + k in d:
            r = d["grad__" + k]
            np.testing.assert_allclose(p.grad.numpy(), r, rtol=tol, atol=tol * max(np.abs(r).max(), 1e-12))


def test_oracle_quantizer(golden):
    d = golden("quantize_values")
    x = torch.from_numpy(d["x"])
    for qb, key in ((6, "q6"), (5, "q5"), (-5, "q5m"), (4, "q4"), (3, "q3"), (7, "q7")):
        assert np.array_equal(quantize(x, qb).numpy(), d[key]), key


def test_oracle_reproduces_reference_ber_curve(golden):
    """The oracle's per-iteration error counts equal the reference decoder's over the whole z=16 BER
    curve (tests/golden/gen_ber_curve.py: 250 codewords per Eb/N0 point, 1.0..4.0 dB, T=20)."""
    import hashlib
    import sys
    sys.path.insert(0, os.path.join(ROOT, "neural-ldpc-decoder-torch_amd", "src"))
    import neural_ldpc_decoder as nd
    d = golden("ber_curve_neural_bg2_z16")
    bg = np.loadtxt(os.path.join(ROOT, "resources", "basegraph2_set0.txt"), int, delimiter="\t")
    gen16 = np.loadtxt(os.path.join(ROOT, "resources", "gen_matrix_bg2_z16.txt"), int, delimiter=",")
    M, N = bg.shape
    W, T, Z = int(d["words"]), int(d["T"]), int(d["Z"])
    xs, ys = nd.AWGNPassedDatagen(N=N, M=M, snr_db=d["ebn0_db"].copy(), gen_matrix=gen16)(
        word_length=W, Z=Z, is_y_all_zero=True)
    g = OracleGraph(bg, Z)
    w = [torch.full((g.E,), 0.5) for _ in range(T)]
    b = [torch.zeros(g.E) for _ in range(T)]
    for k in range(len(d["ebn0_db"])):
        x = np.reshape(xs[k], [W, N, Z]).astype(np.float32)
        assert hashlib.sha256(x.tobytes()).hexdigest() == str(d["x_sha256"][k])
        y = np.asarray(ys[k]).reshape(W, N * Z)
        outs = neural_forward(g, torch.from_numpy(x), w, b)
        wrong = [(o.numpy() > 0) != y for o in outs]
        assert [int(m.sum()) for m in wrong] == d["bit_errors"][k].tolist()
        assert [int(m.any(axis=1).sum()) for m in wrong] == d["frame_errors"][k].tolist()


@pytest.mark.parametrize("E", [7, 32, 197, 316])
def test_prod_order_model_matches_torch_prod(E):
    """_prod_aten's model of ATen's CPU reduction order reproduces torch.prod bit for bit on the CPU
    the fixtures were made on (it is the order the SP fixtures above pin)."""
    from oracle.ldpc_oracle import _prod_aten
    gen = torch.Generator().manual_seed(E)
    t = (torch.rand(4, 1, 64, E, generator=gen) * 1.6 - 0.8)
    t = torch.where(torch.rand(t.shape, generator=gen) < 0.3, torch.ones_like(t), t)
    ref = torch.prod(t, dim=3)
    got = _prod_aten(t, list(range(E)), E)
    assert torch.equal(got, ref), f"{(got != ref).sum().item()} of {ref.numel()} products differ"


def test_tanh_table_reproduces_torch_tanh():
    """The recorded torch.tanh values (gen_tanh_table.py, used by the device SP check node and by the
    oracle) equal this host's torch.tanh -- the function the reference's SP calls -- on random inputs
    of the check node's domain |x| <= 10 and on the table's own correction points."""
    from oracle import ldpc_oracle as lo
    tab = lo._tanh_table()
    if tab is None:
        pytest.skip("lib/nldpc_tanh_ref.bin not built")
    gen = torch.Generator().manual_seed(11)
    x = torch.cat([(torch.rand(1 << 20, generator=gen) * 20 - 10),
                   torch.from_numpy(tab[0][::97].astype(np.int32)).view(torch.float32)])
    x = torch.cat([x, -x])
    got = lo._tanh(x)
    assert torch.equal(got, torch.tanh(x)), f"{(got != torch.tanh(x)).sum().item()} values differ"
