"""CPU oracle: an edge-list restatement of the reference decoders' arithmetic.

TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's `cpu_baseline` leg
may import this module, and only as the checker (or as the timed CPU baseline).  The product path
(neural-ldpc-decoder-torch_amd/) never imports it and fails loudly without its HIP library.

What it restates (reference = ShapeLayer/neural-ldpc-decoder-torch):
  * graph / edge orders ........ src/boosted_neural_ldpc_decoder/ConnectingMatrix.py:82-163
                                 (identical in src/neural_ldpc_decoder/ConnectingMatrix.py:68-140)
  * Neural forward ............. src/neural_ldpc_decoder/NeuralLDPCDecoder.py:44-100
  * Boosted forward ............ src/boosted_neural_ldpc_decoder/BoostedNeuralLDPCDecoder.py:260-538
  * QMS quantiser + STE ........ BoostedNeuralLDPCDecoder.py:187-214, Functions.py:43-67
Instead of the reference's dense (E*Z)^2 lifting matrices and [B,Z,E,E] tiles, messages live per
edge as [B, Z] tensors; the cyclic lift is a torch.roll, and the check-node tile is built per check
row ([B, Z, d_c, d_c]) so min / prod / tie-break semantics are the reference's.  Every fp32 sum the
reference evaluates through MKL sgemm over 0/1 matrices is evaluated here left-to-right in ascending
C-order edge index starting from +0 (the order SURVEY.md §0.3 verified), so Neural / MS / QMS outputs
are bit-identical to the reference; the SP product follows ATen's CPU reduction order (_prod_aten).

Parity pinning: tests/test_oracle_golden.py checks this module against the golden fixtures under
tests/golden/ that tests/golden/gen_golden.py produced by running the reference itself.
The oracle is differentiable (plain torch autograd), which makes it the gradient checker too.
"""
from __future__ import annotations

import os

import numpy as np
import torch

SP, MS, QMS = 0, 1, 2  # reference DecoderType values (struct/DecoderType.py:4-7)

_TANH_BIN = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "neural-ldpc-decoder-torch_amd",
                         "lib", "nldpc_tanh_ref.bin")
_tanh_tab = None


def _tanh_table():
    """torch.tanh's fp32 values on the machine the fixtures were made on, as gen_tanh_table.py recorded
    them at build time (corrections to the correctly rounded tanh), or None when not built."""
    global _tanh_tab
    if _tanh_tab is None:
        if not os.path.exists(_TANH_BIN):
            _tanh_tab = False
        else:
            raw = np.fromfile(_TANH_BIN, dtype=np.uint32)
            _, ver, sh, kmax, n, nov = (int(v) for v in raw[:6])
            h = 6 + (16 if ver >= 2 else 0)  # version 2: 64 bytes of build-host provenance
            nidx = (kmax >> sh) + 2
            ent = raw[h + nidx:h + nidx + n]
            ov = raw[h + nidx + n:h + nidx + n + 2 * nov].reshape(-1, 2)
            _tanh_tab = ((ent & 0x7FFFFFFF).astype(np.int64), (ent >> 31).astype(np.int64), ov.astype(np.int64), kmax)
    return _tanh_tab or None


def tanh_table_provenance():
    """'torch version|CPU capability|CPU model' of the host that built lib/nldpc_tanh_ref.bin (version 2
    tables), '' for a version 1 table, None when there is no table."""
    if not os.path.exists(_TANH_BIN):
        return None
    raw = np.fromfile(_TANH_BIN, dtype=np.uint32, count=22)
    return raw[6:22].tobytes().split(b"\0")[0].decode() if int(raw[1]) >= 2 else ""


def _tanh(x: torch.Tensor) -> torch.Tensor:
    """torch.tanh (BoostedNeuralLDPCDecoder.py:402) with the values of the fixture machine's CPU
    torch.tanh (MKL vector math, not correctly rounded; another host's vector math may differ in the
    last bit, which atanh near saturation amplifies): the rounded double tanh plus the recorded
    corrections.  Without the table, this host's torch.tanh.  The gradient is torch.tanh's."""
    t = torch.tanh(x)
    tab = _tanh_table()
    if tab is None:
        return t
    keys, dirs, ov, kmax = tab
    xd = x.detach()
    key = (xd.abs().contiguous().view(torch.int32).numpy().astype(np.int64))
    r = torch.tanh(xd.abs().double()).float().contiguous().view(torch.int32).numpy().astype(np.int64)
    pos = np.clip(np.searchsorted(keys, key), 0, len(keys) - 1)
    hit = (keys[pos] == key) & (key <= kmax)
    r = r + np.where(hit, 2 * dirs[pos] - 1, 0)
    for k, v in ov:
        r = np.where(key == k, v, r)
    ref = torch.from_numpy(r.astype(np.int32)).view(torch.float32).reshape(x.shape)
    ref = torch.copysign(ref, xd)
    return t + (ref - t).detach()


class OracleGraph:
    """Edge tables of the lifted Tanner graph.  C-order edge index e (row-major over the base graph,
    ConnectingMatrix.py:92-99, 137-147) is the one used for messages and learned weights."""

    def __init__(self, basegraph, Z):
        hb = np.asarray(basegraph, dtype=np.int64)
        self.M, self.N = hb.shape
        self.Z = int(Z)
        rows, cols = np.nonzero(hb != -1)  # row-major == C-order
        self.E = len(rows)
        self.chk = rows.astype(np.int64)
        self.var = cols.astype(np.int64)
        self.shift = (hb[rows, cols] % self.Z).astype(np.int64)
        self.row_edges = [np.nonzero(self.chk == i)[0].tolist() for i in range(self.M)]
        # V-order (column-major, ConnectingMatrix.py:84-91) index of every C-order edge: the position of
        # an edge on the last axis of the reference's [B, Z, E, E] check-node tile
        order = np.lexsort((self.chk, self.var))
        self.vidx = np.empty(self.E, dtype=np.int64)
        self.vidx[order] = np.arange(self.E)
        # column edge lists ascend in check row == ascending C-order index
        self.col_edges = [np.nonzero(self.var == j)[0].tolist() for j in range(self.N)]


def quantize(x: torch.Tensor, q: int) -> torch.Tensor:
    """QMS quantiser with the straight-through estimator (BoostedNeuralLDPCDecoder.py:187-214)."""
    if q == 6:
        lo, hi, qv = -15.5, 15.5, torch.clamp(torch.round(x), -15.5, 15.5)
    elif q == 5:
        lo, hi, qv = -7.5, 7.5, torch.clamp(torch.round(x * 2) / 2, -7.5, 7.5)
    elif q == -5:
        lo, hi, qv = -15, 15, torch.clamp(torch.round(x), -15, 15)
    elif q == 4:
        lo, hi, qv = -7, 7, torch.clamp(torch.round(x), -7, 7)
    elif q == 3:
        lo, hi, qv = -6, 6, torch.clamp(torch.round(x / 2) * 2, -6, 6)
    else:
        return x
    xc = torch.clamp(x, lo, hi)
    return xc + (qv - xc).detach()


def _lift(x: torch.Tensor, s: int) -> torch.Tensor:
    """[B, Z] variable-copy domain -> check-copy domain: out[h] = x[(h + s) mod Z]  (lifting_matrix_1)."""
    return torch.roll(x, -s, dims=1) if s else x


def _unlift(x: torch.Tensor, s: int) -> torch.Tensor:
    """check-copy domain -> variable-copy domain: out[v] = x[(v - s) mod Z]  (lifting_matrix_2)."""
    return torch.roll(x, s, dims=1) if s else x


def _seq_sum(terms, like):
    """(((+0 + t0) + t1) + ...) in fp32, the MKL sgemm order over a 0/1 column."""
    acc = torch.zeros_like(like)
    for t in terms:
        acc = acc + t
    return acc


def _vn(g: OracleGraph, ch: torch.Tensor, c2v):
    """Variable-node extrinsic sums: v2c[e] = (0 + ch[var(e)]) + sum_{e' in col, e' != e} c2v[e']."""
    v2c = [None] * g.E
    zero = torch.zeros_like(ch[:, 0, :])
    for j in range(g.N):
        es = g.col_edges[j]
        x0 = zero + ch[:, j, :]
        for e in es:
            v2c[e] = x0 + _seq_sum([c2v[e2] for e2 in es if e2 != e], zero)
    return v2c


def _prod_aten(t: torch.Tensor, pos, E: int) -> torch.Tensor:
    """torch.prod(tile, dim=3) of the reference's [B, Z, E, E] SP tile, restricted to one check row:
    t [B, Z, d_out, d_in] holds the row's factors (every other tile entry is exactly 1.0), pos[l] is
    in-edge l's position on the reduced axis (its V-order index).  Reproduces the multiplication order
    of ATen's CPU vectorised reduction (aten/src/ATen/native/cpu/Reduce.h, reduction128 +
    vectorized_reduction) as dispatched on the fixture machine: 4 accumulators of 8-float vectors over
    the first E // 32 * 32 positions (accumulator j = pos // 8 % 4, lane pos % 8, chunks in order),
    lanes combined as (a0 * a1) * (a2 * a3), then the 8 lanes left to right, then the tail positions
    one by one.  Factors of exactly 1.0 are skipped (multiplying by 1 is exact), so only the row's
    edges enter.  Checked against torch.prod on random rows (0 mismatches in 1500) and against the
    reference's SP fixtures (tests/test_oracle_golden.py)."""
    d = t.shape[3]
    full = (E // 32) * 32
    slots = {}
    tail = []
    for l in sorted(range(d), key=lambda l: pos[l]):
        if pos[l] < full:
            slots.setdefault((pos[l] // 8 % 4, pos[l] % 8), []).append(l)
        else:
            tail.append(l)
    lanes = []
    for lane in range(8):
        acc = []
        for j in range(4):
            members = slots.get((j, lane), [])
            a = None
            for l in members:
                a = t[..., l] if a is None else a * t[..., l]
            acc.append(a)
        ab = acc[0] if acc[1] is None else (acc[1] if acc[0] is None else acc[0] * acc[1])
        cd = acc[2] if acc[3] is None else (acc[3] if acc[2] is None else acc[2] * acc[3])
        x = ab if cd is None else (cd if ab is None else ab * cd)
        if x is not None:
            lanes.append(x)
    out = None
    for x in lanes + [t[..., l] for l in tail]:
        out = x if out is None else out * x
    return out if out is not None else torch.ones_like(t[..., 0])


def _cn_row_tile(g: OracleGraph, i: int, m_list):
    """Stack a check row's lifted inputs into the reference's masked tile [B, Z, d, d] (self masked)."""
    m = torch.stack(m_list, dim=2)  # [B, Z, d]
    d = m.shape[2]
    w = 1.0 - torch.eye(d, dtype=m.dtype)
    return m.unsqueeze(2) * w  # [B, Z, k(out), l(in)] == x_tile * W_even2odd^T restricted to the row


def neural_forward(g: OracleGraph, xa: torch.Tensor, weights, biases):
    """NeuralLDPCDecoder.forward (NeuralLDPCDecoder.py:44-100).  xa [B, N, Z] fp32; weights/biases:
    sequences of T tensors [E].  Returns the list of T outputs [B, N*Z]."""
    B = xa.shape[0]
    Z = g.Z
    zero = torch.zeros((B, Z), dtype=torch.float32)
    c2v = [zero] * g.E
    outs = []
    for t in range(len(weights)):
        v2c = _vn(g, xa, c2v)
        cn = [None] * g.E
        for i in range(g.M):
            es = g.row_edges[i]
            tile = _cn_row_tile(g, i, [_lift(v2c[e], int(g.shift[e])) for e in es])
            a = torch.abs(tile)
            x3 = torch.min(a + 10000 * (1 - (a > 0).float()), dim=3)[0]  # :74-75
            x4 = torch.ones_like(tile) - 2 * ((-tile) < 0).float()  # :77-78
            x_out0 = x3 * torch.sign(-torch.prod(x4, dim=3))  # :79-80
            for k, e in enumerate(es):
                cn[e] = _unlift(x_out0[:, :, k], int(g.shift[e]))
        new = []
        for e in range(g.E):
            a = torch.abs(cn[e]) * weights[t][e] + biases[t][e]  # :89 (two roundings)
            a = a * (a > 0).float()
            new.append(a * torch.sign(cn[e]))
        c2v = new
        y = torch.stack([xa[:, j, :] + _seq_sum([c2v[e] for e in g.col_edges[j]], zero) for j in range(g.N)], 1)
        outs.append(y.reshape(B, g.N * Z))
    return outs


def boosted_forward(g: OracleGraph, xa: torch.Tensor, *, dtype: int, q: int, nw, iters, w_cn, w_ucn, w_vn,
                    llr_lo=-20.0, llr_hi=20.0, fixed_iteration=(), fixed_iter_weight=None):
    """BoostedNeuralLDPCDecoder.forward (BoostedNeuralLDPCDecoder.py:260-538) for a tensor input and an
    iteration list that starts from the zero message state.

    w_cn / w_ucn / w_vn: callables it -> weight tensor (the value `fetch_param` returns) or None.
    Returns the dict {iteration: output [B, N*Z]}."""
    cn_s, ucn_s, vn_s = nw
    B = xa.shape[0]
    Z = g.Z
    zero = torch.zeros((B, Z), dtype=torch.float32)
    c2v = [zero] * g.E
    xa_input = xa  # [B, N, Z] (the reference keeps [B, Z, N]; weights broadcast over N either way)
    xa_origin = xa.clone()
    outputs = {}
    fixed_idx = 0
    chk = torch.from_numpy(g.chk)
    for t in iters:
        wv = w_vn(t) if vn_s else None
        if vn_s in (2, 3):
            xa_input = xa_input * (wv.view(1, -1, 1) if vn_s == 2 else wv)
        elif vn_s == 4:
            wsel = wv if t not in fixed_iteration else fixed_iter_weight[fixed_idx]
            xa_input = xa_input * wsel
        if dtype == QMS:
            xa_input = quantize(xa_input, q)
        ucn_flag = None
        if ucn_s > 0:
            app = xa_input if t == 0 else outputs[t - 1].reshape(B, g.N, Z)
            vapp = -app
            f = (vapp > 0).float() - (vapp <= 0).float()  # :347
            ucn_flag = []
            for i in range(g.M):
                es = g.row_edges[i]
                p = torch.prod(torch.stack([_lift(f[:, int(g.var[e]), :], int(g.shift[e])) for e in es], 2), 2)
                ucn_flag.append((p < 0).float())  # [B, Z(h)]
        v2c = _vn(g, xa_input, c2v)
        cn = [None] * g.E
        for i in range(g.M):
            es = g.row_edges[i]
            ms = []
            for e in es:
                x2 = _lift(v2c[e], int(g.shift[e]))
                x2 = quantize(x2, q) if dtype == QMS else torch.clamp(x2, llr_lo, llr_hi)  # :386-389
                if dtype in (MS, QMS):
                    x2 = x2 + 0.0001 * (1 - (torch.abs(x2) > 0).float())  # :391-393
                ms.append(x2)
            tile = _cn_row_tile(g, i, ms)
            if dtype == SP:
                th = _tanh(torch.mul(-0.5, tile))  # :402
                x3 = _prod_aten(torch.add(th, 1 - (torch.abs(th) > 0).float()),  # :403-404
                                [int(g.vidx[e]) for e in es], g.E)
                x3 = torch.clamp(x3, -1 + 1e-7, 1 - 1e-7)  # :406-407
                x_out0 = torch.mul(-2.0, torch.atanh(x3))  # :408
            else:
                a = torch.add(torch.abs(tile), torch.mul(10000.0, 1.0 - (torch.abs(tile) > 0).float()))
                x3 = torch.min(a, dim=3)[0]  # :415
                x3 = torch.add(x3, torch.mul(-0.0001, torch.add(-(x3 > 0.0001).float(), 1.0)))  # :416
                x4 = torch.add(torch.zeros_like(tile), 1 - 2 * (torch.mul(-1.0, tile) < 0).float())
                x_out0 = torch.mul(x3, torch.sign(torch.mul(-1.0, torch.prod(x4, dim=3))))  # :422-423
            for k, e in enumerate(es):
                cn[e] = _unlift(x_out0[:, :, k], int(g.shift[e]))
        # learned weights by sharing code (:431-503), per edge
        wc = w_cn(t) if cn_s else None
        wu = w_ucn(t) if (ucn_s and ucn_s == cn_s and cn_s in (1, 2, 3)) else None
        if cn_s == 4 and t in fixed_iteration:
            wc = fixed_iter_weight[fixed_idx]

        def per_edge(w, e):
            if cn_s in (1, 4):
                return w[e]
            if cn_s == 2:
                return w[chk[e]]
            return w[0] if w.numel() == 1 else w

        new = []
        for e in range(g.E):
            x0 = cn[e]
            if cn_s == 0:
                x1 = torch.abs(x0)
            elif wu is not None:
                u = _unlift(ucn_flag[int(g.chk[e])], int(g.shift[e]))
                x11 = torch.abs(x0) * per_edge(wc, e)
                x12 = torch.abs(x0) * per_edge(wu, e)
                x1 = x11 * (-u + 1.0) + x12 * u
            elif cn_s in (1, 2, 3, 4):
                x1 = torch.abs(x0) * per_edge(wc, e)
            else:
                raise UnboundLocalError("CN sharing code 5 is not handled by the reference forward (:505)")
            x2 = x1 * (x1 > 0).float()
            x2 = quantize(x2, q) if dtype == QMS else torch.clamp(x2, llr_lo, llr_hi)
            new.append(x2 * torch.sign(x0))
        c2v = new
        if dtype == QMS:
            xa_origin = quantize(xa_origin, q)
        y = torch.stack([xa_origin[:, j, :] + _seq_sum([c2v[e] for e in g.col_edges[j]], zero)
                         for j in range(g.N)], 1)
        y = torch.clamp(y, llr_lo, llr_hi)
        outputs[t] = y.reshape(B, g.N * Z)
        if t in fixed_iteration:
            fixed_idx += 1
    return outputs


def ber_counts(outputs, y):
    """Per-iteration (bit errors, frame errors) with the decoder's own convention bit = (LLR > 0)
    (SURVEY §0.4); frame = any of the N*Z bits wrong (Functions.py:93-99)."""
    res = []
    yb = y.to(torch.bool)
    for o in outputs:
        err = (o > 0) != yb
        res.append((int(err.sum()), int(err.any(dim=1).sum())))
    return res
