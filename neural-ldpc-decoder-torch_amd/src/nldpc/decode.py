"""Host side of the decode path: buffers, C-ABI calls and the autograd Functions.

`decode(...)` runs T flooding iterations of a decoder on the device through nldpc_forward
(include/nldpc.h).  `NeuralDecodeFn` / `BoostedDecodeFn` wrap it in torch.autograd so that
NeuralLDPCDecoder / BoostedNeuralLDPCDecoder keep the reference's training semantics
(gradients of the learned weights through every iteration) via nldpc_backward.
"""
from __future__ import annotations

import ctypes
import dataclasses
from dataclasses import dataclass

import torch

from . import _lib, jit
from .graph import LiftedGraph

KIND_SP, KIND_MS, KIND_QMS, KIND_NEURAL = _lib.NLDPC_SP, _lib.NLDPC_MS, _lib.NLDPC_QMS, _lib.NLDPC_NEURAL


@dataclass
class DecodeCfg:
    kind: int
    qbit: int = 5
    ucn: bool = False
    vn_cumulative: bool = False
    llr_lo: float = -20.0
    llr_hi: float = 20.0
    first_iter: int = 0
    vn_prefix: int = 0
    path: str = "auto"        # "auto" | "stream" | "fused" (register-resident kernel)
    keep_state: bool = True   # False: the final c2v state is not needed (lets the fused path skip it)
    # every row of w_cn repeats one weight (sharing code 3): the backward may put each iteration's gradient
    # total into a few entries of the row (only row sums are meaningful, which is what the expand() that
    # built the row passes on) -- NLDPC_FLAG_CN_TIED
    cn_tied: bool = False

    def flags(self) -> int:
        f = {"auto": 0, "stream": _lib.FLAG_STREAM, "fused": _lib.FLAG_FUSED}[self.path]
        f |= _lib.FLAG_CN_TIED if self.cn_tied else 0
        return f | (0 if self.keep_state else _lib.FLAG_NO_STATE)

    def c_struct(self, c2v_in: bool) -> _lib.NldpcCfg:
        return _lib.NldpcCfg(self.kind, int(self.qbit), int(bool(self.ucn)), int(bool(self.vn_cumulative)),
                             float(self.llr_lo), float(self.llr_hi), int(self.first_iter), int(bool(c2v_in)),
                             int(self.vn_prefix), self.flags())


def _require_device_tensor(x: torch.Tensor, name: str):
    if not isinstance(x, torch.Tensor):
        raise TypeError(f"{name} must be a torch.Tensor")
    if x.device.type != "cuda":
        raise RuntimeError(f"{name} is on '{x.device}': the MI355X decoder needs ROCm device tensors (no CPU path)")


def _f32c(t):
    return None if t is None else t.detach().to(torch.float32).contiguous()


def decode(graph: LiftedGraph, cfg: DecodeCfg, xa: torch.Tensor, T: int, *, w_cn=None, w_ucn=None, bias=None,
           w_vn=None, c2v=None, app_prev=None, save=False, out_mask=None):
    """Run T iterations.  xa [B, N, Z] fp32 device tensor.  Weights: [T, E] / [T, N] tensors or None.

    Returns (outputs [T, B, N*Z], c2v state [B, E, Z], saved byte buffer for the backward or None).
    c2v: optional incoming state [B, E, Z] (None = all-zero messages)."""
    _require_device_tensor(xa, "xa")
    cfg = _honour_tied(cfg, w_cn)  # (r6: the tied flag also selects the tied saving forward)
    if xa.dim() != 3 or xa.shape[1] != graph.N or xa.shape[2] != graph.Z:
        raise ValueError(f"xa must be [B, {graph.N}, {graph.Z}], got {tuple(xa.shape)}")
    dev = xa.device
    B = int(xa.shape[0])
    xa_c = _f32c(xa)
    E, N, Z = graph.E, graph.N, graph.Z
    outs = torch.empty((T, B, N * Z), dtype=torch.float32, device=dev)
    c2v_in = c2v is not None
    c = cfg.c_struct(c2v_in)
    L = _lib.lib()
    h = graph.handle(dev)
    if cfg.path != "stream" and not c2v_in and T <= 64 and jit.wanted(cfg):  # no built-in kernel: compile one
        jit.ensure(graph, dev, cfg.kind, 1 if save else 0)
    fast = ctypes.c_int32(0)
    _lib.check(L.nldpc_fast_path(h, ctypes.byref(c), B, T, int(bool(save)), ctypes.byref(fast)), "nldpc_fast_path")
    if c2v_in:
        state = c2v.detach().to(torch.float32).contiguous().clone()
    elif fast.value and not cfg.keep_state:
        state = None
    else:
        state = torch.empty((B, E, Z), dtype=torch.float32, device=dev)
    saved = None
    if save:
        nbytes = ctypes.c_size_t(0)
        _lib.check(L.nldpc_saved_bytes(h, ctypes.byref(c), B, T, ctypes.byref(nbytes)), "nldpc_saved_bytes")
        saved = torch.empty((int(nbytes.value),), dtype=torch.uint8, device=dev)
    # the streaming path works on a v2c scratch (training too: QMS saves int8 codes, not the messages)
    scratch = None if fast.value else torch.empty((B, E, Z), dtype=torch.float32, device=dev)
    tensors = [None if (out_mask is not None and not out_mask[t]) else outs[t] for t in range(T)]
    pp, keep = _lib.ptr_array(tensors)
    w_cn, w_ucn, bias, w_vn = _f32c(w_cn), _f32c(w_ucn), _f32c(bias), _f32c(w_vn)
    app = _f32c(app_prev)
    st = L.nldpc_forward(h, ctypes.byref(c), B, T, _lib.ptr(xa_c), _lib.ptr(w_cn), _lib.ptr(w_ucn),
                         _lib.ptr(bias), _lib.ptr(w_vn), pp, _lib.ptr(app), _lib.ptr(state), _lib.ptr(scratch),
                         _lib.ptr(saved), _lib.stream_of(dev))
    del keep
    _lib.check(st, "nldpc_forward")
    return outs, state, saved


def decode_count(graph: LiftedGraph, cfg: DecodeCfg, xa: torch.Tensor, T: int, *, w_cn=None, w_ucn=None, bias=None,
                 w_vn=None, y=None, convention: int = 0, app_prev=None) -> torch.Tensor:
    """Count-only decode: int64 [T, 2] device tensor of (bit errors, frame errors) of
    every iteration's posterior -- what decode(...) followed by channel.ber_counts(outputs, y,
    convention=...) returns, counted inside the fused kernel (nldpc_forward_count) so the T posteriors
    are never written.  Configurations the fused path does not cover (UCN, a resumed state, a graph
    without a compiled kernel, UCN resumed at first_iter > 0) run decode + the device counter instead
    (both on the device); app_prev: the posterior of iteration first_iter - 1 for those UCN calls."""
    _require_device_tensor(xa, "xa")
    cfg = _honour_tied(cfg, w_cn)  # (r6: the tied flag also selects the tied saving forward)
    if xa.dim() != 3 or xa.shape[1] != graph.N or xa.shape[2] != graph.Z:
        raise ValueError(f"xa must be [B, {graph.N}, {graph.Z}], got {tuple(xa.shape)}")
    dev = xa.device
    B = int(xa.shape[0])
    c = cfg.c_struct(False)
    c.flags |= _lib.FLAG_NO_STATE
    L = _lib.lib()
    h = graph.handle(dev)
    yb = None if y is None else (y != 0).to(torch.uint8).reshape(B, graph.N * graph.Z).contiguous()
    mode = 3 if (yb is not None or convention) else 2  # the count-only kernel variant
    if cfg.path != "stream" and T <= 64 and not (cfg.ucn and cfg.first_iter > 0) and jit.wanted(cfg):
        jit.ensure(graph, dev, cfg.kind, mode)
    fast = ctypes.c_int32(0)
    _lib.check(L.nldpc_fast_path(h, ctypes.byref(c), B, T, mode, ctypes.byref(fast)), "nldpc_fast_path")
    if not fast.value or (cfg.ucn and cfg.first_iter > 0):  # (nldpc_forward_count has no app_prev)
        from .channel import ber_counts
        outs, _, _ = decode(graph, cfg, xa, T, w_cn=w_cn, w_ucn=w_ucn, bias=bias, w_vn=w_vn, app_prev=app_prev)
        return ber_counts(list(outs), yb, convention=convention)
    counts = torch.zeros((T, 2), dtype=torch.int64, device=dev)
    xa_c = _f32c(xa)
    w_cn, w_ucn, bias, w_vn = _f32c(w_cn), _f32c(w_ucn), _f32c(bias), _f32c(w_vn)
    _lib.check(L.nldpc_forward_count(h, ctypes.byref(c), B, T, _lib.ptr(xa_c), _lib.ptr(w_cn), _lib.ptr(w_ucn),
                                     _lib.ptr(bias), _lib.ptr(w_vn), _lib.ptr(yb), int(convention),
                                     counts.data_ptr(), _lib.stream_of(dev)), "nldpc_forward_count")
    return counts


def _honour_tied(cfg: DecodeCfg, w_cn) -> DecodeCfg:
    """cfg.cn_tied holds only for a w_cn whose rows are one repeated value by construction (an expand(): stride 0
    along the edges, as the drop-in module passes sharing code 3); any other w_cn gets the per-edge gradient
    (the tied kernel computes a row's masks from its first weight, so per-edge weights under the
    flag would give wrong row sums)."""
    if cfg.cn_tied and (w_cn is None or w_cn.dim() != 2 or w_cn.stride(1) != 0):
        return dataclasses.replace(cfg, cn_tied=False)
    return cfg


def decode_backward(graph: LiftedGraph, cfg: DecodeCfg, xa, T, grad_outs, outs, saved, *, w_cn=None, w_ucn=None,
                    bias=None, w_vn=None, app_prev=None, need=(True, True, True, True), c2v_in=False,
                    grad_state=None, want_state_grad=False):
    """Gradients of the per-edge / per-column weights and, with want_state_grad, of the incoming message
    state (c2v_in: the forward resumed from a state).  grad_state: gradient arriving at the final state
    [B, E, Z] (None = zero).  Returns (g_w_cn, g_w_ucn, g_bias, g_w_vn, g_c2v_in)."""
    dev = xa.device
    B = int(xa.shape[0])
    cfg = _honour_tied(cfg, w_cn)

    def z(ref, on):
        return torch.zeros(tuple(ref.shape), dtype=torch.float32, device=dev) if (ref is not None and on) else None

    g_cn = z(w_cn, need[0])
    g_ucn = z(w_ucn, need[1])
    g_b = z(bias, need[2])
    g_vn = z(w_vn, need[3])
    g_state = torch.zeros((B, graph.E, graph.Z), dtype=torch.float32, device=dev) if want_state_grad else None
    gs_in = None if grad_state is None else grad_state.to(torch.float32).contiguous()
    c = cfg.c_struct(c2v_in)
    L = _lib.lib()
    h = graph.handle(dev)
    if (cfg.path != "stream" and not cfg.ucn and cfg.vn_prefix == 0 and T <= 64 and jit.wanted(cfg)
            and grad_state is None and not want_state_grad and not c2v_in):  # the fused backward's conditions
        jit.ensure(graph, dev, cfg.kind, 4)
    nbytes = ctypes.c_size_t(0)
    _lib.check(L.nldpc_backward_workspace(h, ctypes.byref(c), B, T, ctypes.byref(nbytes)), "nldpc_backward_workspace")
    work = torch.empty((max(int(nbytes.value), 1),), dtype=torch.uint8, device=dev)
    go = [None if g is None else g.to(torch.float32).contiguous() for g in grad_outs]
    ob = [o for o in outs]
    pg, keep1 = _lib.ptr_array(go)
    po, keep2 = _lib.ptr_array(ob)
    xa_c = _f32c(xa)
    w_cn, w_ucn, bias, w_vn = _f32c(w_cn), _f32c(w_ucn), _f32c(bias), _f32c(w_vn)
    st = L.nldpc_backward(h, ctypes.byref(c), B, T, _lib.ptr(xa_c), _lib.ptr(w_cn), _lib.ptr(w_ucn), _lib.ptr(bias),
                          _lib.ptr(w_vn), po, pg, _lib.ptr(_f32c(app_prev)), _lib.ptr(saved), _lib.ptr(gs_in),
                          _lib.ptr(g_state), _lib.ptr(g_cn), _lib.ptr(g_ucn), _lib.ptr(g_b), _lib.ptr(g_vn),
                          _lib.ptr(work), int(work.numel()), _lib.stream_of(dev))
    del keep1, keep2
    _lib.check(st, "nldpc_backward")
    return g_cn, g_ucn, g_b, g_vn, g_state


class DecodeFn(torch.autograd.Function):
    """outputs, state = decoder(xa, c2v_in; w_cn, w_ucn, bias, w_vn) with gradients for the four weight
    tensors and for the incoming message state, and the final state differentiable too -- so that
    segments of one forward chained through the state (list-valued xa, split iteration runs;
    BoostedNeuralLDPCDecoder.py:320-512 keeps self.llr[t+1] in the autograd graph) backpropagate
    across segment boundaries.

    forward returns the T outputs as separate tensors (views of one [T, B, N*Z] buffer) plus the
    final message state [B, E, Z] (an empty tensor when the fused path did not keep it)."""

    @staticmethod
    def forward(ctx, graph, cfg, T, app_prev, xa, c2v_in, w_cn, w_ucn, bias, w_vn):
        need_grad = any(t is not None and t.requires_grad for t in (c2v_in, w_cn, w_ucn, bias, w_vn))
        outs, state, saved = decode(graph, cfg, xa, T, w_cn=w_cn, w_ucn=w_ucn, bias=bias, w_vn=w_vn, c2v=c2v_in,
                                    app_prev=app_prev, save=need_grad)
        ctx.graph, ctx.cfg, ctx.T = graph, cfg, T
        ctx.has_state_in = c2v_in is not None
        ctx.set_materialize_grads(False)
        if need_grad:
            ctx.save_for_backward(xa, w_cn, w_ucn, bias, w_vn, app_prev, outs, saved)
        if state is None:
            state = outs.new_empty((0,))
            ctx.mark_non_differentiable(state)
        return (*outs.unbind(0), state)

    @staticmethod
    def backward(ctx, *grads):
        xa, w_cn, w_ucn, bias, w_vn, app_prev, outs, saved = ctx.saved_tensors
        grad_outs = list(grads[:ctx.T])
        g_state_out = grads[ctx.T]
        if g_state_out is not None and g_state_out.numel() == 0:
            g_state_out = None
        want_state = ctx.has_state_in and ctx.needs_input_grad[5]
        need = (ctx.needs_input_grad[6], ctx.needs_input_grad[7], ctx.needs_input_grad[8], ctx.needs_input_grad[9])
        g_cn, g_ucn, g_b, g_vn, g_c2v = decode_backward(
            ctx.graph, ctx.cfg, xa, ctx.T, grad_outs, outs.unbind(0), saved, w_cn=w_cn, w_ucn=w_ucn, bias=bias,
            w_vn=w_vn, app_prev=app_prev, need=need, c2v_in=ctx.has_state_in, grad_state=g_state_out,
            want_state_grad=want_state)
        return (None, None, None, None, None, g_c2v if want_state else None, g_cn if need[0] else None,
                g_ucn if need[1] else None, g_b if need[2] else None, g_vn if need[3] else None)


def decode_autograd(graph, cfg, xa, T, *, w_cn=None, w_ucn=None, bias=None, w_vn=None, c2v=None, app_prev=None):
    """Differentiable decode.  Returns (list of T outputs [B, N*Z], final state [B, E, Z]).  c2v: the
    incoming message state (None = all-zero); gradients flow into it when it requires grad.
    cfg.cn_tied is honoured only for a stride-0 w_cn (_honour_tied)."""
    cfg = _honour_tied(cfg, w_cn)
    res = DecodeFn.apply(graph, cfg, T, app_prev, xa, c2v, w_cn, w_ucn, bias, w_vn)
    return list(res[:T]), res[T]
