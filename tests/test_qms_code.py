"""The QMS saved-state code (nldpc_math.h qms_code): the nine-operation form the kernels use equals the
definition code = rint(2 m'), m' = Q(m) inside the quantiser's clip range and sign(m) (hi + 1) outside
(Q: BoostedNeuralLDPCDecoder.py:187-214 forward value), for every active q, in fp32 (numpy float32
arithmetic is IEEE round-to-nearest-even like the device's)."""
import numpy as np
import pytest

f = np.float32
HI = {6: 15.5, 5: 7.5, -5: 15.0, 4: 7.0, 3: 6.0}
S = {5: 2.0, 3: 0.5}


def quantize(x, q):  # the reference's STE forward value, op by op
    s, inv, hi = f(S.get(q, 1.0)), f(1.0 / S.get(q, 1.0)), f(HI[q])
    with np.errstate(over="ignore", invalid="ignore"):
        qv = np.clip((np.rint(x * s) * inv).astype(f), -hi, hi)
        xc = np.clip(x, -hi, hi)
        return (xc + (qv - xc).astype(f)).astype(f)


def code_definition(m, q):
    hi = f(HI[q])
    with np.errstate(invalid="ignore"):
        inr = (m >= -hi) & (m <= hi)
        mp = np.where(inr, quantize(m, q), np.where(m > 0, hi + f(1), -(hi + f(1)))).astype(f)
        return np.rint((f(2) * mp).astype(f))


def code_kernel(m, q):  # nldpc_math.h qms_code, active q
    hi, s = f(HI[q]), f(S.get(q, 1.0))
    k2, hs, c_out = f(2.0 / S.get(q, 1.0)), f(HI[q] * S.get(q, 1.0)), f(2 * HI[q] + 2)
    with np.errstate(over="ignore", invalid="ignore"):
        t = (np.clip(np.rint((m * s).astype(f)), -hs, hs) * k2).astype(f)
        return np.where(np.abs(m) <= hi, t, np.where(m > 0, c_out, -c_out))


@pytest.mark.parametrize("q", sorted(HI))
def test_qms_code_identity(q):
    rng = np.random.default_rng(q + 10)
    xs = np.concatenate([np.arange(-40, 40, 1 / 512, dtype=f), rng.normal(0, 12, 200_000).astype(f),
                         np.array([0.0, -0.0, np.inf, -np.inf, np.nan, 1e-30, -1e-30, 3e38, -3e38], f)])
    xs = np.concatenate([xs, np.nextafter(xs, f(np.inf)), np.nextafter(xs, f(-np.inf))]).astype(f)
    a, b = code_definition(xs, q), code_kernel(xs, q)
    assert np.array_equal(a, b)
    assert np.abs(a).max() <= 2 * HI[q] + 2
