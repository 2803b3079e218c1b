"""BoostedNeuralLDPCDecoder at the headline graph (BG2 z=384) against the CPU oracle.

The reference cannot run z=384 (its dense lifting matrices are 22.9 GB each), so
parity there is transitive: the oracle (oracle/ldpc_oracle.py) is pinned bit-exactly to the
reference's fixtures at z=16/z=24 (tests/test_oracle_golden.py), and here the drop-in module --
driven exactly as train/train_BoostedNeuralLDPCDecoder.py:274-291 drives it -- is compared with the
oracle on the same inputs and weights:
  * cfg5: QMS q=5, NW(3,0,3), T=50, forward + LDPCDecoderLoss BCE + backward.  Outputs bit-exact;
    loss against an fp64 sum of torch's fp32 terms within the bound derived in tests/bce_bounds.py;
    weight gradients rtol 1e-4 (the batch / edge sum order of the gradient reductions differs from
    autograd's);
  * MS / QMS forward with per-edge / per-check weights, UCN, cumulative VN weights: bit-exact;
  * SP forward: hard decisions exact, soft values within the SP tolerance of test_gpu_forward.py.
Reference: src/boosted_neural_ldpc_decoder/BoostedNeuralLDPCDecoder.py:260-538,
LDPCDecoderLoss.py:38-108.
"""
import os

import numpy as np
import pytest
import torch

from bce_bounds import assert_loss, bce_reference
from conftest import ROOT

pytestmark = pytest.mark.gpu

BG2 = np.loadtxt(os.path.join(ROOT, "resources", "basegraph2_set0.txt"), int, delimiter="\t")
DEV = torch.device("cuda")
Z = 384


def _model(T, B, nw, dtype, q=5):
    import boosted_neural_ldpc_decoder as bd
    from boosted_neural_ldpc_decoder.BoostedNeuralLDPCDecoder import BoostedNeuralLDPCDecoder
    from boosted_neural_ldpc_decoder.struct.DecoderType import DecoderType
    from boosted_neural_ldpc_decoder.struct.NodeWeightSharingConfig import NodeWeightSharingConfig as NW
    conn = bd.ConnectingMatrixTorch(bd.ConnectingMatrix(Z, BG2), device=DEV)
    return BoostedNeuralLDPCDecoder(T, B, conn, node_weight_sharing_config=NW(*nw), decoding_type=DecoderType(dtype),
                                    decoder_qms_qbit=q).to(DEV)


def _channel(B, seed, qbit, ebn0=2.0):
    """Reference datagen arithmetic (AWGNPassedDatagen.py:97-107): all-zero codeword, BPSK bit 0 -> -1,
    LLR = 2y/sigma^2 in f64, then the QMS quantiser when the decoder is QMS."""
    from boosted_neural_ldpc_decoder.Functions import Functions
    sigma = (1.0 / (2 * 0.2 * 10 ** (ebn0 / 10))) ** 0.5
    gen = torch.Generator().manual_seed(seed)
    x = (2 * (-1 + sigma * torch.randn(B, 52, Z, generator=gen, dtype=torch.float64)) / sigma ** 2).numpy()
    if qbit:
        x = Functions.Cal_MSA_Q(x, qbit)
    return torch.from_numpy(np.asarray(x, dtype=np.float32))


def _randomise(model, seed, lo=0.5, hi=1.5):
    gen = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for _, p in model.named_parameters():
            p.copy_(lo + (hi - lo) * torch.rand(p.shape, generator=gen))


def _oracle(model, x, nw, dtype, q, T, requires_grad=False):
    from oracle.ldpc_oracle import OracleGraph, boosted_forward
    P = {n: p.detach().cpu().clone().requires_grad_(requires_grad) for n, p in model.named_parameters()}

    def fetch(node, code):
        return lambda t: P.get(f"weight_{node}_{t}") if code else None

    outs = boosted_forward(OracleGraph(BG2, Z), x, dtype=dtype, q=q, nw=nw, iters=list(range(T)),
                           w_cn=fetch("CN", nw[0]), w_ucn=fetch("UCN", nw[1]), w_vn=fetch("VN", nw[2]))
    return [outs[t] for t in range(T)], P


def _ref_loss(outs, y):
    """LDPCDecoderLoss BCE, etha = 1, coeff_param = range(T) (LDPCDecoderLoss.py:73-108): the terms
    summed from the last iteration down, divided by the coefficient sum."""
    tot = 0
    for k in range(len(outs) - 1, -1, -1):
        tot = tot + torch.nn.functional.binary_cross_entropy_with_logits(outs[k], y)
    return 1.0 * (tot / float(len(outs))).mean()


def test_cfg5_train_step_matches_oracle():
    """cfg5 at its own graph and depth: QMS q=5 NW(3,0,3) T=50 (reference init weights 1.0), one
    forward + BCE + backward as train_BoostedNeuralLDPCDecoder.py:274-291."""
    from boosted_neural_ldpc_decoder.LDPCDecoderLoss import LDPCDecoderLoss
    from boosted_neural_ldpc_decoder.struct.LossType import LossType
    T, B, nw, dtype, q = 50, 2, (3, 0, 3), 2, 5
    model = _model(T, B, nw, dtype, q)
    x = _channel(B, 2042, q)
    y = torch.zeros(B, 52 * Z)
    model.train()
    outs = model(x.to(DEV), target_iter=list(range(T)))
    loss = LDPCDecoderLoss(loss_type=LossType.BCE, etha=1.0)(outs, y.to(DEV), coeff_param=list(range(T)))
    loss.backward()
    ref_outs, P = _oracle(model, x, nw, dtype, q, T, requires_grad=True)
    ref_loss = _ref_loss(ref_outs, y)
    ref_loss.backward()
    for t in range(T):
        o, r = outs[t].detach().cpu(), ref_outs[t].detach()
        assert torch.equal(o, r), f"iteration {t}: {(o != r).sum().item()} of {r.numel()} soft values differ"
    ref64, bound, _ = bce_reference(ref_outs, y)
    assert_loss(loss.item(), ref64, bound)
    n = 0
    for name, p in model.named_parameters():
        r = P[name].grad
        if r is None:
            assert p.grad is None or not p.grad.any(), name
            continue
        np.testing.assert_allclose(p.grad.cpu().numpy(), r.numpy(), rtol=1e-4,
                                   atol=1e-4 * max(float(r.abs().max()), 1e-12), err_msg=name)
        n += 1
    assert n == 2 * T  # weight_CN_t and weight_VN_t of every iteration


@pytest.mark.parametrize("dtype,nw", [(2, (1, 0, 2)), (1, (2, 0, 3)), (2, (3, 3, 0)), (1, (1, 1, 2)), (2, (1, 1, 2))])
def test_boosted_forward_matches_oracle(dtype, nw):
    """MS / QMS forward at z=384 with random weights: per-edge (code 1), per-check / per-column
    (code 2) and per-iteration (code 3) sharing, UCN weighting (codes 3/3 and 1/1), cumulative VN
    weights.  Bit-exact."""
    T, B, q = 12, 3, 5
    model = _model(T, B, nw, dtype, q)
    _randomise(model, 17 * dtype + nw[0])
    x = _channel(B, 7 + nw[0], q if dtype == 2 else 0, ebn0=1.5)
    with torch.no_grad():
        outs = model(x.to(DEV))
    ref, _ = _oracle(model, x, nw, dtype, q, T)
    for t in range(T):
        o = outs[t].cpu()
        assert torch.equal(o, ref[t]), f"iteration {t}: {(o != ref[t]).sum().item()} of {o.numel()} values differ"


def test_boosted_ms_grads_match_oracle():
    """MS training step at z=384 with per-edge CN weights and per-column VN weights (codes 1 / 2)."""
    from boosted_neural_ldpc_decoder.LDPCDecoderLoss import LDPCDecoderLoss
    from boosted_neural_ldpc_decoder.struct.LossType import LossType
    T, B, nw, dtype = 8, 2, (1, 0, 2), 1
    model = _model(T, B, nw, dtype)
    _randomise(model, 3, 0.7, 1.3)
    x = _channel(B, 99, 0, ebn0=1.0)
    y = torch.zeros(B, 52 * Z)
    model.train()
    outs = model(x.to(DEV), target_iter=list(range(T)))
    loss = LDPCDecoderLoss(loss_type=LossType.BCE, etha=1.0)(outs, y.to(DEV), coeff_param=list(range(T)))
    loss.backward()
    ref_outs, P = _oracle(model, x, nw, dtype, 5, T, requires_grad=True)
    ref_loss = _ref_loss(ref_outs, y)
    ref_loss.backward()
    for t in range(T):
        assert torch.equal(outs[t].detach().cpu(), ref_outs[t].detach()), t
    ref64, bound, _ = bce_reference(ref_outs, y)
    assert_loss(loss.item(), ref64, bound)
    for name, p in model.named_parameters():
        r = P[name].grad
        if r is not None:
            np.testing.assert_allclose(p.grad.cpu().numpy(), r.numpy(), rtol=1e-4,
                                       atol=1e-4 * max(float(r.abs().max()), 1e-12), err_msg=name)


def test_boosted_sp_forward_matches_oracle():
    """SP forward at z=384 (T=20): hard decisions exact, soft values as the SP fixtures."""
    T, B, nw = 20, 2, (3, 0, 3)
    model = _model(T, B, nw, 0)
    _randomise(model, 5, 0.8, 1.2)
    x = _channel(B, 11, 0)
    with torch.no_grad():
        outs = model(x.to(DEV))
    ref, _ = _oracle(model, x, nw, 0, 5, T)
    from test_gpu_forward import sp_check
    sp_check(torch.stack([o.cpu() for o in outs]).numpy(), torch.stack(ref).numpy())
