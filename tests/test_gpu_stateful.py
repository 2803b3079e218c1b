"""The stateful forward contracts of BoostedNeuralLDPCDecoder on the GPU against the
reference's own results (tests/golden/gen_golden_f3.py): list-valued xa, a call that resumes from the
state another call stored (self.llr, BoostedNeuralLDPCDecoder.py:343, 377, 512) -- also from the
middle of that call's iterations --, and a split iteration list.  The last call of each sequence runs
with gradients: outputs bit-exact, LDPCDecoderLoss BCE value within the bound derived in tests/bce_bounds.py, parameter gradients rtol 1e-4
(batch-sum order)."""
import glob
import os

import numpy as np
import pytest
import torch

from bce_bounds import assert_loss, bce_reference
from conftest import GOLDEN, ROOT

pytestmark = pytest.mark.gpu

BG2 = np.loadtxt(os.path.join(ROOT, "resources", "basegraph2_set0.txt"), int, delimiter="\t")
DEV = torch.device("cuda")
CASES = sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN, "stateful_*.npz")))


@pytest.mark.parametrize("name", CASES)
def test_stateful_sequence_matches_reference(golden, name):
    import boosted_neural_ldpc_decoder as bd
    from boosted_neural_ldpc_decoder.BoostedNeuralLDPCDecoder import BoostedNeuralLDPCDecoder
    from boosted_neural_ldpc_decoder.LDPCDecoderLoss import LDPCDecoderLoss
    from boosted_neural_ldpc_decoder.struct.DecoderType import DecoderType
    from boosted_neural_ldpc_decoder.struct.LossType import LossType
    from boosted_neural_ldpc_decoder.struct.NodeWeightSharingConfig import NodeWeightSharingConfig as NW
    d = golden(name)
    T, Z = int(d["T"]), int(d["Z"])
    B = d["x0"].shape[0]
    conn = bd.ConnectingMatrixTorch(bd.ConnectingMatrix(Z, BG2), device=DEV)
    model = BoostedNeuralLDPCDecoder(T, B, conn, node_weight_sharing_config=NW(*[int(v) for v in d["nw"]]),
                                     decoding_type=DecoderType(int(d["dtype"])), decoder_qms_qbit=int(d["q"])).to(DEV)
    with torch.no_grad():
        for n, p in model.named_parameters():
            p.copy_(torch.from_numpy(d["param__" + n]))
    ncalls = int(d["ncalls"])
    for c in range(ncalls):
        iters = [int(v) for v in d[f"call{c}_iters"]]
        sel = [int(v) for v in d[f"call{c}_x"]]
        listed = bool(int(d[f"call{c}_listed"]))
        xin = [torch.from_numpy(d[f"x{k}"]).to(DEV) for k in sel] if listed else torch.from_numpy(d[f"x{sel[0]}"]).to(DEV)
        kw = {"fixed_iter": []} if listed else {}
        if c < ncalls - 1:
            with torch.no_grad():
                model(xin, target_iter=list(iters), **kw)
            continue
        outs = model(xin, target_iter=list(iters), **kw)
        y = torch.from_numpy(d["y"].astype(np.float32)).to(DEV)
        loss = LDPCDecoderLoss(loss_type=LossType.BCE, etha=1.0)(outs, y, coeff_param=list(range(len(outs))))
        loss.backward()
    got = np.stack([o.detach().cpu().numpy() for o in outs])
    assert np.array_equal(got, d["outputs"]), f"{(got != d['outputs']).sum()} of {got.size} soft values differ"
    ref64, bound, stored = bce_reference(outs, y)  # fp64 sum of torch's fp32 terms (bce_bounds.py)
    assert_loss(loss.item(), ref64, bound)
    assert abs(float(d["loss"]) - ref64) <= stored, (float(d["loss"]), ref64, stored)
    n = 0
    for pname, p in model.named_parameters():
        key = "grad__" + pname
        if key in d:
            r = d[key]
            assert p.grad is not None, pname
            np.testing.assert_allclose(p.grad.cpu().numpy(), r, rtol=1e-4, atol=1e-4 * max(np.abs(r).max(), 1e-12),
                                       err_msg=pname)
            n += 1
        elif p.grad is not None:
            assert not p.grad.any(), pname
    assert n > 0


@pytest.mark.parametrize("dtype,nw", [(2, (3, 0, 3)), (1, (1, 1, 2))])
def test_resume_after_caller_refills_input(dtype, nw):
    """forward(x); x.copy_(next batch) in place; forward(x2, target_iter=[k..T-1]) resumes from the state
    the first call reached at k -- computed from the ORIGINAL x, as the reference stores it
    (BoostedNeuralLDPCDecoder.py:512) -- not from the refilled buffer."""
    import boosted_neural_ldpc_decoder as bd
    from boosted_neural_ldpc_decoder.BoostedNeuralLDPCDecoder import BoostedNeuralLDPCDecoder
    from boosted_neural_ldpc_decoder.struct.DecoderType import DecoderType
    from boosted_neural_ldpc_decoder.struct.NodeWeightSharingConfig import NodeWeightSharingConfig as NW
    T, B, Z, k = 8, 3, 16, 5
    conn = bd.ConnectingMatrixTorch(bd.ConnectingMatrix(Z, BG2), device=DEV)

    def model():
        m = BoostedNeuralLDPCDecoder(T, B, conn, node_weight_sharing_config=NW(*nw), decoding_type=DecoderType(dtype),
                                     decoder_qms_qbit=5).to(DEV)
        g = torch.Generator().manual_seed(7)
        with torch.no_grad():
            for _, p in m.named_parameters():
                p.copy_(0.6 + 0.8 * torch.rand(p.shape, generator=g))
        return m

    g = torch.Generator().manual_seed(3)
    x = (torch.randn(B, 52, Z, generator=g) * 4 + 1).to(DEV)
    x2 = (torch.randn(B, 52, Z, generator=g) * 4 + 1).to(DEV)
    ref_model, dut = model(), model()
    with torch.no_grad():
        ref_model(x.clone())
        ref = [o.clone() for o in ref_model(x2, target_iter=list(range(k, T)))]
        buf = x.clone()
        dut(buf)
        buf.copy_(x2)  # the caller refills its input buffer in place
        got = dut(x2, target_iter=list(range(k, T)))
    for t, (a, b) in enumerate(zip(got, ref)):
        assert torch.equal(a, b), f"iteration {k + t}: {(a != b).sum().item()} values differ"


@pytest.mark.parametrize("dtype,ucn", [("MS", True), ("QMS", False)])
def test_dropped_final_state_recomputes_bit_identical(dtype, ucn):
    """a call that runs up to the last iteration does not write self.llr[T] (keep_state=False, the
    fused kernel skips 19.8 GB at cfg3); reading it afterwards recomputes it from the call's record.  That
    state must equal, bit for bit, the state of the same decode run with keep_state=True -- and it is a
    constant (no graph), unlike the reference's attached tensor (the module docstring says so)."""
    import dataclasses
    import boosted_neural_ldpc_decoder as bd
    from boosted_neural_ldpc_decoder.BoostedNeuralLDPCDecoder import BoostedNeuralLDPCDecoder
    from boosted_neural_ldpc_decoder.struct.DecoderType import DecoderType
    from boosted_neural_ldpc_decoder.struct.NodeWeightSharingConfig import NodeWeightSharingConfig as NW
    from nldpc.decode import decode_autograd
    T, Z, B = 6, 384, 3
    conn = bd.ConnectingMatrixTorch(bd.ConnectingMatrix(Z, BG2), device=DEV)
    model = BoostedNeuralLDPCDecoder(T, B, conn, node_weight_sharing_config=NW(1, 1 if ucn else 0, 2),
                                     decoding_type=getattr(DecoderType, dtype), decoder_qms_qbit=5).to(DEV)
    gen = torch.Generator().manual_seed(77)
    with torch.no_grad():
        for p in model.parameters():
            p.copy_(0.6 + 0.8 * torch.rand(p.shape, generator=gen))
    x = (2 * (-1 + 0.8 * torch.randn(B, 52, Z, generator=gen)) / 0.64).float()
    if dtype == "QMS":
        x = torch.clamp(torch.round(2 * x) / 2, -7.5, 7.5)
    x = x.to(DEV)
    with torch.no_grad():
        model(x)
    assert isinstance(model.llr[T], BoostedNeuralLDPCDecoder._Pending)  # not written by the fused kernel
    rec = model.llr[T].rec
    got = model._state(T)
    assert got is not None and got.shape == (B, int(model.sum_edge), Z) and not got.requires_grad
    cfg = dataclasses.replace(rec["cfg"], keep_state=True)
    with torch.no_grad():
        _, ref = decode_autograd(conn.graph, cfg, x, T, w_cn=rec["w_cn"], w_ucn=rec["w_ucn"], w_vn=rec["w_vn"],
                                 c2v=None, app_prev=None)
    assert torch.equal(got.view(torch.int32), ref.view(torch.int32))
