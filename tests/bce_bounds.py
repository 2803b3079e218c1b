"""Reference value and error bounds for the multi-iteration BCE loss (LDPCDecoderLoss.py:73-108,
LossType.BCE): loss = sum_k c_k * mean_i term(x_ki, y_i), c_k = etha^k / sum etha^k, where torch's
fp32 term is bce_with_logits = (1 - y) x - log_sigmoid(x), log_sigmoid(x) = min(x, 0) - log1p(exp(-|x|)).

The reference value is computed in fp64 from torch's own fp32 terms (reduction='none') of the given
outputs, so it carries no reduction-order noise.  Two bounds are derived from how each side computes:

* the device (nldpc_bce_loss, nldpc_aux.hip): the same fp32 term formula, fp32 terms summed in fp64 in
  a fixed order, one rounding to fp32 at the end.  Its terms can differ from torch's only through the
  libm: exp and log1p are each within 2 ulp on either side, so |L_dev - L_torch| <= 8 eps L
  (L = log1p(exp(-|x|)), eps = 2^-24), and the two roundings that follow (min(x,0) - L, then
  (1-y) x - that) can each land one fp32 ulp apart.  An element whose L is below half an ulp of |x|
  (|x| >~ 15: both roundings return x exactly, whatever L is) contributes nothing.  Per element
  delta_i = 8 eps L_i + ulp(|x_i| + L_i) + ulp(term_i); bound = sum_k c_k mean_i delta_ki + ulp(ref) / 2.
* the reference's stored fp32 loss (torch's fp32 mean of n terms, then T fp32 additions): cascade
  summation error <= (ceil(log2 n) + 1) eps per mean, plus one eps per term added, relative to the
  sum of magnitudes.
"""
import math

import numpy as np
import torch

EPS = 2.0 ** -24


def _ulp(v):
    v = np.abs(np.asarray(v, dtype=np.float32))
    return np.spacing(v).astype(np.float64)


def bce_reference(outs, y, etha=1.0):
    """(fp64 reference loss, device bound, stored-fp32 bound) for outputs `outs` (list of tensors, any
    device) and labels y."""
    K = len(outs)
    coef = np.array([etha ** k for k in range(K)], dtype=np.float64)
    coef = coef / coef.sum()
    yy = y.detach().float().cpu()
    ref = dev_bound = mag = 0.0
    n = None
    for k, o in enumerate(outs):
        x = o.detach().float().cpu()
        n = x.numel()
        term = torch.nn.functional.binary_cross_entropy_with_logits(x, yy, reduction="none").numpy().astype(np.float32)
        xa = np.abs(x.numpy().astype(np.float64))
        L = np.log1p(np.exp(-xa))
        live = L * (1 + 8 * EPS) >= 0.5 * _ulp(xa)  # elements whose rounding can see the libm's L
        delta = np.where(live, 8 * EPS * L + _ulp(xa + L) + _ulp(term), 0.0)
        ref += coef[k] * term.astype(np.float64).sum() / n
        dev_bound += coef[k] * delta.sum() / n
        mag += coef[k] * np.abs(term.astype(np.float64)).sum() / n
    dev_bound += 0.5 * float(_ulp(ref))
    stored_bound = (math.ceil(math.log2(max(n, 2))) + 1 + K + 1) * EPS * mag
    return ref, dev_bound, stored_bound


def assert_loss(dev_loss, ref, bound, what="loss"):
    d = abs(float(dev_loss) - ref)
    assert d <= bound, f"{what}: |device - fp64 reference| = {d:.3e} > derived bound {bound:.3e} (ref {ref:.9g})"
