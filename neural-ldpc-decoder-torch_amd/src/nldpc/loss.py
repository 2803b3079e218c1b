"""Multi-iteration BCE training loss on the device (config 5): the LossType.BCE branch of
LDPCDecoderLoss.forward over a list of decoder outputs and one label tensor
(src/boosted_neural_ldpc_decoder/LDPCDecoderLoss.py:70-108) as two HIP passes (nldpc_bce_loss /
nldpc_bce_grad) instead of a chain of per-term elementwise ops and reductions."""
from __future__ import annotations

import ctypes

import torch

from . import _lib


class BCEMultiFn(torch.autograd.Function):
    """loss = sum_k coef[k] * mean(bce_with_logits(outputs[k], target)); coef already normalised.

    When an output needs a gradient, the forward pass also writes every output's gradient for a unit seed
    (nldpc_bce_loss_grad: the logits are read once for both directions), and backward returns those,
    recomputed on the device only if the seed that arrives is not 1 (nldpc_bce_grad_unless_unit) -- the
    same values as the separate gradient pass for any seed.  Those K gradient tensors (the size of the outputs:
    8.2 GB at cfg5) are held on ctx from the forward until backward runs or the graph is freed; a loss computed
    with grad enabled but never backpropagated (logging, validation outside torch.no_grad) pays that write and
    memory for nothing -- pass fuse_grad=False to bce_multi to keep the two-pass form there."""

    @staticmethod
    def forward(ctx, target, coef, fuse_grad, *outputs):
        L = _lib.lib()
        dev = outputs[0].device
        n = outputs[0].numel()
        xs = [o.detach().to(torch.float32).contiguous() for o in outputs]
        t = target.detach().to(torch.float32).contiguous()
        K = len(xs)
        c = (ctypes.c_float * K)(*[float(v) for v in coef])
        nb = ctypes.c_size_t(0)
        _lib.check(L.nldpc_bce_workspace(n, K, ctypes.byref(nb)), "nldpc_bce_workspace")
        work = torch.empty((int(nb.value),), dtype=torch.uint8, device=dev)
        loss = torch.empty((), dtype=torch.float32, device=dev)
        px, keep = _lib.ptr_array(xs)
        ctx.grads = None
        if fuse_grad and any(ctx.needs_input_grad[3:]) and hasattr(L, "nldpc_bce_loss_grad"):
            grads = [torch.empty_like(x) for x in xs]
            pg, keep_g = _lib.ptr_array(grads)
            st = L.nldpc_bce_loss_grad(px, K, c, _lib.ptr(t), n, _lib.ptr(loss), pg, _lib.ptr(work),
                                       int(work.numel()), _lib.stream_of(dev))
            del keep_g
            _lib.check(st, "nldpc_bce_loss_grad")
            ctx.grads = grads
        else:
            st = L.nldpc_bce_loss(px, K, c, _lib.ptr(t), n, _lib.ptr(loss), _lib.ptr(work), int(work.numel()),
                                  _lib.stream_of(dev))
            _lib.check(st, "nldpc_bce_loss")
        del keep
        ctx.coef = [float(v) for v in coef]
        ctx.save_for_backward(t, *xs)
        return loss

    @staticmethod
    def backward(ctx, g):
        t, *xs = ctx.saved_tensors
        L = _lib.lib()
        dev = xs[0].device
        K, n = len(xs), xs[0].numel()
        grads, ctx.grads = ctx.grads, None  # (a second backward through a retained graph recomputes them)
        entry = L.nldpc_bce_grad_unless_unit if grads is not None else L.nldpc_bce_grad
        if grads is None:
            grads = [torch.empty_like(x) for x in xs]
        c = (ctypes.c_float * K)(*ctx.coef)
        gs = g.detach().to(torch.float32).reshape(()).contiguous()
        px, k1 = _lib.ptr_array(xs)
        pg, k2 = _lib.ptr_array(grads)
        st = entry(px, K, c, _lib.ptr(t), n, _lib.ptr(gs), pg, _lib.stream_of(dev))
        del k1, k2
        _lib.check(st, "nldpc_bce_grad")
        return (None, None, None, *grads)


def bce_multi(outputs, target, coef, fuse_grad: bool = True):
    """Differentiable multi-term BCE-with-logits on ROCm tensors (see BCEMultiFn).  fuse_grad=False: the loss
    pass writes no gradients ahead of a backward (for a loss that is only logged)."""
    return BCEMultiFn.apply(target, list(coef), bool(fuse_grad), *outputs)
