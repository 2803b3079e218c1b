"""Drop-in module parity on the GPU: the reference's own API (NeuralLDPCDecoder,
BoostedNeuralLDPCDecoder, LDPCDecoderLoss, Functions.evaluate_ber_fer) driven exactly as
test/ and train/ drive it, compared with the reference's golden outputs, losses and gradients."""
import glob
import os

import numpy as np
import pytest
import torch

from bce_bounds import assert_loss, bce_reference
from conftest import GOLDEN, ROOT

pytestmark = pytest.mark.gpu

BG2 = np.loadtxt(os.path.join(ROOT, "resources", "basegraph2_set0.txt"), int, delimiter="\t")
WIMAX = np.loadtxt(os.path.join(ROOT, "resources", "wman_N0576_R34_z24.txt"), int, delimiter="\t")
DEV = torch.device("cuda")


def _bg(name):
    return WIMAX if "wimax" in name else BG2


def _neural_model(d, name):
    import neural_ldpc_decoder as nd
    conn = nd.ConnectingMatrixTorch(nd.ConnectingMatrix(int(d["Z"]), _bg(name)), device=DEV)
    model = nd.NeuralLDPCDecoder(int(d["T"]), d["x"].shape[0], conn).to(DEV)
    with torch.no_grad():
        for t in range(int(d["T"])):
            model.weights_var[t].copy_(torch.from_numpy(d["weights"][t]))
            model.biases_var[t].copy_(torch.from_numpy(d["biases"][t]))
    return model


def _boosted_model(d, name, B=None):
    import boosted_neural_ldpc_decoder as bd
    from boosted_neural_ldpc_decoder.BoostedNeuralLDPCDecoder import BoostedNeuralLDPCDecoder
    from boosted_neural_ldpc_decoder.struct.DecoderType import DecoderType
    from boosted_neural_ldpc_decoder.struct.NodeWeightSharingConfig import NodeWeightSharingConfig as NW
    conn = bd.ConnectingMatrixTorch(bd.ConnectingMatrix(int(d["Z"]), _bg(name)), device=DEV)
    model = BoostedNeuralLDPCDecoder(int(d["T"]), B or d["x"].shape[0], conn,
                                     node_weight_sharing_config=NW(*[int(v) for v in d["nw"]]),
                                     decoding_type=DecoderType(int(d["dtype"])), decoder_qms_qbit=int(d["q"]),
                                     fixed_iterative_nodes=[int(v) for v in d.get("fixed_nodes", [])]).to(DEV)
    with torch.no_grad():
        for n, p in model.named_parameters():
            p.copy_(torch.from_numpy(d["param__" + n]))
    return model


def _assert_out(o, ref, sp):
    o = o.detach().cpu().numpy()
    assert np.array_equal(o > 0, ref > 0)
    if sp:
        from test_gpu_forward import sp_check
        sp_check(o, ref)
    else:
        assert np.array_equal(o, ref), f"{(o != ref).sum()} of {o.size} soft values differ"


@pytest.mark.parametrize("name", ["neural_cfg1_snr2_default", "neural_cfg1_snr2_random", "neural_bg2_z16_b16_t5_random",
                                  "neural_wimax_z24_b16_t20_random"])
def test_neural_module_forward(golden, name):
    d = golden(name)
    model = _neural_model(d, name)
    with torch.no_grad():
        outs = model(torch.from_numpy(d["x"]).to(DEV))
    assert isinstance(outs, list) and len(outs) == int(d["T"])
    for t, o in enumerate(outs):
        _assert_out(o, d["outputs"][t], False)


@pytest.mark.parametrize("name", ["neural_bg2_z16_b16_t5_random", "neural_wimax_z24_b16_t20_random"])
def test_neural_module_grads(golden, name):
    d = golden(name)
    model = _neural_model(d, name)
    y = torch.from_numpy(d["y"].astype(np.float32)).to(DEV)
    outs = model(torch.from_numpy(d["x"]).to(DEV))
    loss = sum(torch.nn.functional.binary_cross_entropy_with_logits(o, y) for o in outs) / len(outs)
    loss.backward()
    # torch's own fp32 reductions on both sides: each within its derived error of the fp64 sum
    ref64, _, stored = bce_reference(outs, y)
    assert abs(loss.item() - ref64) <= stored and abs(float(d["loss"]) - ref64) <= stored
    gw = torch.stack([p.grad for p in model.weights_var]).cpu().numpy()
    gb = torch.stack([p.grad for p in model.biases_var]).cpu().numpy()
    np.testing.assert_allclose(gw, d["grad_w"], rtol=1e-4, atol=1e-4 * np.abs(d["grad_w"]).max())
    np.testing.assert_allclose(gb, d["grad_b"], rtol=1e-4, atol=1e-4 * np.abs(d["grad_b"]).max())


BOOSTED = sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN, "boosted_*.npz")))


@pytest.mark.parametrize("name", BOOSTED)
def test_boosted_module_forward(golden, name):
    d = golden(name)
    model = _boosted_model(d, name)
    x = torch.from_numpy(d["x"]).to(DEV)
    with torch.no_grad():
        if "target6" in name:
            outs = model(x, target_iter=list(range(0, 6)))
        else:
            outs = model(x)
            assert outs is model.outputs  # module-owned list, as in the reference
    for t, o in enumerate(outs):
        _assert_out(o, d["outputs"][t], int(d["dtype"]) == 0)
    if "target6" not in name and not d.get("fixed_nodes", np.zeros(0)).size:
        # count-only decode (§8 F2): the counts of the outputs just checked, without writing them
        from nldpc.channel import ber_counts
        assert torch.equal(model.count_errors(x, convention=1), ber_counts(outs, convention=1))


TRAIN = sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN, "train_*.npz")))


@pytest.mark.parametrize("name", TRAIN)
def test_boosted_train_step_grads(golden, name):
    """One config-5 step as train/train_BoostedNeuralLDPCDecoder.py:274-291 runs it."""
    from boosted_neural_ldpc_decoder.LDPCDecoderLoss import LDPCDecoderLoss
    from boosted_neural_ldpc_decoder.struct.LossType import LossType
    d = golden(name)
    T = int(d["T"])
    model = _boosted_model(d, name)
    x = torch.from_numpy(d["x"]).to(DEV)
    y = torch.from_numpy(d["y"].astype(np.float32)).to(DEV)
    model.train()
    outs = model(x, target_iter=list(range(0, T)))
    loss = LDPCDecoderLoss(loss_type=LossType.BCE, etha=1.0)(outs, y, coeff_param=list(range(len(outs))))
    loss.backward()
    sp = int(d["dtype"]) == 0
    for k, t in enumerate(d["out_iters"]):
        _assert_out(outs[int(t)], d["outputs"][k], sp)
    # the device loss against an fp64 sum of torch's fp32 terms of the same outputs, and the
    # reference's stored fp32 loss against that sum within torch's own reduction error (bce_bounds.py)
    ref64, bound, stored = bce_reference(outs, y)
    assert_loss(loss.item(), ref64, bound)
    assert abs(float(d["loss"]) - ref64) <= stored, (float(d["loss"]), ref64, stored)
    tol = 2e-3 if sp else 1e-4
    n = 0
    for pname, p in model.named_parameters():
        if "grad__" + pname in d:
            r = d["grad__" + pname]
            np.testing.assert_allclose(p.grad.cpu().numpy(), r, rtol=tol, atol=tol * max(np.abs(r).max(), 1e-12),
                                       err_msg=pname)
            n += 1
    assert n > 0


def test_neural_no_grad_forward_sees_data_mutations():
    """parameters changed through `p.data` (the reference clamps its weights that way,
    Boosted…py:177) between two torch.no_grad() forwards are the ones the second decode uses -- no
    stacked-weight cache can go stale."""
    import neural_ldpc_decoder as nd
    conn = nd.ConnectingMatrixTorch(nd.ConnectingMatrix(16, BG2), device=DEV)
    gen = torch.Generator().manual_seed(3)
    x = (2.0 * torch.randn(4, 52, 16, generator=gen) + 1.0).to(DEV)
    model = nd.NeuralLDPCDecoder(5, 4, conn).to(DEV)
    ref = nd.NeuralLDPCDecoder(5, 4, conn).to(DEV)
    with torch.no_grad():
        for t in range(5):
            ref.weights_var[t].fill_(0.25)
            ref.biases_var[t].fill_(-0.125)
        a = model(x)[-1].clone()
        for t in range(5):
            model.weights_var[t].data.clamp_(0.0, 0.25)   # 0.5 -> 0.25, no _version bump
            model.biases_var[t].data.sub_(0.125)
        b = model(x)[-1].clone()
        c = ref(x)[-1].clone()
    assert not torch.equal(a, b)
    assert torch.equal(b.view(torch.int32), c.view(torch.int32))


def test_evaluate_ber_fer_literal(golden):
    from boosted_neural_ldpc_decoder import Functions
    d = golden("ber_values")
    outs = [torch.from_numpy(o).to(DEV) for o in d["outs"]]
    (be, bits), (fe, frames) = Functions.evaluate_ber_fer(torch.from_numpy(d["y"]).to(DEV), outs)
    assert be == [float(v) for v in d["bit_errors"]] and bits == int(d["bits"])
    assert fe == [float(v) for v in d["frame_errors"]] and frames == int(d["frames"])


def test_ber_counts_decoder_convention():
    from nldpc.channel import ber_counts
    g = torch.Generator().manual_seed(3)
    outs = [torch.randn(37, 1000, generator=g) for _ in range(3)]
    y = (torch.rand(37, 1000, generator=g) < 0.5).to(torch.int64)
    c = ber_counts([o.to(DEV) for o in outs], y.to(DEV)).cpu().numpy()
    for t, o in enumerate(outs):
        err = (o > 0) != y.bool()
        assert c[t, 0] == int(err.sum()) and c[t, 1] == int(err.any(1).sum())
    c0 = ber_counts([o.to(DEV) for o in outs]).cpu().numpy()  # all-zero codeword
    assert c0[0, 0] == int((outs[0] > 0).sum())


def test_awgn_llr_statistics_and_sharding():
    from nldpc.channel import awgn_llr
    B, N, Z, sigma = 64, 52, 384, 0.8
    full = awgn_llr(B, N, Z, sigma, seed=11, device=DEV)
    half = awgn_llr(B // 2, N, Z, sigma, seed=11, b_offset=B // 2, device=DEV)
    assert torch.equal(full[B // 2:], half)  # a rank-offset shard draws the same noise
    noise = (full * sigma ** 2 / 2 + 1) / sigma  # back to N(0, 1)
    assert abs(noise.mean().item()) < 0.01 and abs(noise.std().item() - 1) < 0.01
    other = awgn_llr(B, N, Z, sigma, seed=12, device=DEV)
    assert not torch.equal(full, other)
    # the device generator against its CPU restatement (oracle/philox.py, Random123-pinned Philox): the
    # same counters and Box-Muller; fp64 log / cos / sin of the device and of glibc may differ in the
    # last bit, which the rounding to fp32 almost always absorbs
    from oracle.philox import awgn_llr as awgn_host
    host = awgn_host(B // 2, N * Z, sigma, seed=11, b_offset=B // 2)
    dev = half.reshape(B // 2, N * Z).cpu().numpy()
    assert (dev != host).mean() < 1e-4
    np.testing.assert_allclose(dev, host, rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("qbit", [0, 5])
def test_channel_codeword_puncture_shorten(qbit):
    """§8 F1 on the device: given codeword bits (BPSK (-1)^(1-y)), the QMS quantiser, then puncturing /
    shortening of 1-based inclusive bit ranges -- the steps of AWGNPassedDatagen._generate
    (AWGNPassedDatagen.py:75-134), here over the device's Philox noise (the reference's numpy stream is
    pinned by the host restatement, tests/test_api_surface.py)."""
    from boosted_neural_ldpc_decoder.Functions import Functions
    from boosted_neural_ldpc_decoder.struct.Puncture import Puncture
    from nldpc.channel import awgn_llr
    B, N, Z, sigma = 24, 52, 16, 0.7
    L = N * Z
    gen = torch.Generator().manual_seed(qbit)
    y = torch.randint(0, 2, (B, L), generator=gen).to(DEV)
    plain = awgn_llr(B, N, Z, sigma, seed=5, b_offset=3, device=DEV)  # all-zero codeword, no quantiser
    noise = (plain.double().reshape(B, L) * sigma ** 2 / 2 + 1) / sigma
    want = 2 * ((2 * y.double() - 1) + sigma * noise) / sigma ** 2
    if qbit:
        want = torch.as_tensor(Functions.Cal_MSA_Q(want.float().cpu().numpy(), qbit), device=DEV).double()
    want[:, 0:2 * Z] = 0.001          # Puncture(1, 2Z): columns 0 and 1
    want[:, 100:130] = -20.0          # Shortening(101, 130)
    got = awgn_llr(B, N, Z, sigma, seed=5, b_offset=3, qbit=qbit, device=DEV, y=y, puncturing=Puncture(1, 2 * Z),
                   shortening=(101, 130), puncture_value=0.001, shortening_value=-20.0).reshape(B, L)
    if qbit:  # on the quantiser's grid: equal except where the rounding of the recovered noise flips a step
        assert (got != want.float()).float().mean().item() < 1e-3
    else:
        torch.testing.assert_close(got.double(), want, rtol=1e-5, atol=1e-5)
    assert torch.all(got[:, 0:2 * Z] == 0.001) and torch.all(got[:, 100:130] == -20.0)
    ref0 = awgn_llr(B, N, Z, sigma, seed=5, b_offset=3, qbit=qbit, device=DEV)
    same = awgn_llr(B, N, Z, sigma, seed=5, b_offset=3, qbit=qbit, device=DEV, y=torch.zeros_like(y))
    assert torch.equal(ref0, same)  # y = 0 is the all-zero channel, bit for bit


@pytest.mark.parametrize("K,etha", [(3, 1.0), (7, 0.8), (70, 1.1)])
def test_bce_multi_matches_torch(K, etha):
    """The fused device BCE (LDPCDecoderLoss's list branch) equals the reference's per-term torch
    formula: loss and the gradient of every output (K=70 exercises the >64-term grouping)."""
    from boosted_neural_ldpc_decoder.LDPCDecoderLoss import LDPCDecoderLoss
    from boosted_neural_ldpc_decoder.struct.LossType import LossType
    g = torch.Generator().manual_seed(K)
    n0, n1 = 37, 513
    outs = [(torch.randn(n0, n1, generator=g) * 6).to(DEV).requires_grad_() for _ in range(K)]
    y = (torch.rand(n0, n1, generator=g) < 0.3).float().to(DEV)
    crit = LDPCDecoderLoss(loss_type=LossType.BCE, etha=etha)
    loss = crit(outs, y, coeff_param=list(range(K)))
    loss.backward()
    ref_outs = [o.detach().clone().requires_grad_() for o in outs]
    tot, norm = 0, 0
    for k in reversed(range(K)):
        tot = tot + etha ** k * torch.nn.functional.binary_cross_entropy_with_logits(ref_outs[k], y)
        norm = norm + etha ** k
    ref = 1.0 * (tot / norm).mean()
    ref.backward()
    ref64, bound, _ = bce_reference(outs, y, etha)  # fp64 sum of torch's fp32 terms, derived bound
    assert_loss(loss.item(), ref64, bound)
    for o, r in zip(outs, ref_outs):
        np.testing.assert_allclose(o.grad.cpu().numpy(), r.grad.cpu().numpy(), rtol=1e-5,
                                   atol=1e-6 * r.grad.abs().max().item())


@pytest.mark.gpu
@pytest.mark.parametrize("seed_scale", [1.0, 3.0])
def test_bce_loss_grad_one_pass_equals_two_passes(seed_scale):
    """The training path's single pass (nldpc_bce_loss_grad: loss + unit-seed gradients) and the backward's
    nldpc_bce_grad_unless_unit give the gradients of the two-pass form (nldpc_bce_loss, then
    nldpc_bce_grad with the seed that arrives) bit for bit -- with loss.backward()'s unit seed and with a
    scaled one, which the second call recomputes on the device; grid logits (the table) and off-grid ones,
    an odd length (the scalar tail)."""
    from nldpc import _lib
    from nldpc.loss import bce_multi
    import ctypes
    g = torch.Generator().manual_seed(11)
    K, n = 5, 4 * 3001 + 3
    xs = [(torch.randint(-40, 41, (n,), generator=g).float() * 0.5) for _ in range(K)]
    xs[1][::7] += 0.37
    y = (torch.rand(n, generator=g) < 0.4).float().to(DEV)
    coef = [0.1, 0.2, 0.3, 0.15, 0.25]
    outs = [x.to(DEV).requires_grad_() for x in xs]
    loss = bce_multi(outs, y, coef)
    (seed_scale * loss).backward()
    # the two-pass form through the C ABI
    L = _lib.lib()
    dx = [x.to(DEV) for x in xs]
    c = (ctypes.c_float * K)(*coef)
    nb = ctypes.c_size_t(0)
    _lib.check(L.nldpc_bce_workspace(n, K, ctypes.byref(nb)))
    work = torch.empty((int(nb.value),), dtype=torch.uint8, device=DEV)
    ref_loss = torch.empty((), dtype=torch.float32, device=DEV)
    px, k1 = _lib.ptr_array(dx)
    _lib.check(L.nldpc_bce_loss(px, K, c, _lib.ptr(y), n, _lib.ptr(ref_loss), _lib.ptr(work), int(work.numel()),
                                _lib.stream_of(DEV)))
    grads = [torch.empty_like(x) for x in dx]
    gs = torch.tensor(seed_scale, dtype=torch.float32, device=DEV)
    pg, k2 = _lib.ptr_array(grads)
    _lib.check(L.nldpc_bce_grad(px, K, c, _lib.ptr(y), n, _lib.ptr(gs), pg, _lib.stream_of(DEV)))
    torch.cuda.synchronize()
    assert loss.item() == ref_loss.item()
    for o, r in zip(outs, grads):
        assert torch.equal(o.grad.view(torch.int32), r.view(torch.int32))
    # the two-pass opt-out (fuse_grad=False) gives the same loss and gradients
    outs2 = [x.to(DEV).requires_grad_() for x in xs]
    loss2 = bce_multi(outs2, y, coef, fuse_grad=False)
    (seed_scale * loss2).backward()
    assert loss2.item() == ref_loss.item()
    for o, r in zip(outs2, grads):
        assert torch.equal(o.grad.view(torch.int32), r.view(torch.int32))


@pytest.mark.gpu
def test_bce_loss_grid_table_path():
    """The loss pass takes half-integer logits with 0/1 labels (every QMS decoder output) from a table of
    the same term function (nldpc_aux.hip bce_term_tab): grid logits, off-grid logits, logits past the
    table's range and a non-binary label, one call, against the fp64 reference and its derived bound;
    and a grid-only call must equal the direct formula's fp64 sum of torch's terms within the bound."""
    from boosted_neural_ldpc_decoder.LDPCDecoderLoss import LDPCDecoderLoss
    from boosted_neural_ldpc_decoder.struct.LossType import LossType
    g = torch.Generator().manual_seed(5)
    n0, n1, K = 64, 1999, 9
    grid = [torch.randint(-80, 81, (n0, n1), generator=g).float() * 0.5 for _ in range(K)]  # |k| up to 80 > 64
    mixed = [x.clone() for x in grid]
    for x in mixed[::2]:
        x[::3] += 0.123  # off the grid
    for y in ((torch.rand(n0, n1, generator=g) < 0.5).float(),
              torch.where(torch.rand(n0, n1, generator=g) < 0.1, torch.tensor(0.3), torch.tensor(1.0))):
        for outs in (grid, mixed):
            dev_outs = [o.to(DEV) for o in outs]
            loss = LDPCDecoderLoss(loss_type=LossType.BCE, etha=1.0)(dev_outs, y.to(DEV), coeff_param=list(range(K)))
            ref64, bound, _ = bce_reference(outs, y)
            assert_loss(loss.item(), ref64, bound)
