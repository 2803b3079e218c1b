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


def med3(x, lo, hi):  # v_med3_f32 with constant bounds lo <= hi: a NaN x gives min(lo, hi) = lo (gfx9 ISA)
    with np.errstate(invalid="ignore"):
        return np.where(np.isnan(x), lo, np.minimum(np.maximum(x, lo), hi)).astype(f)


def code_kernel_fast(m, q):  # nldpc_math.h qms_code_p, NLDPC_QFAST: no compare or select
    s = f(S.get(q, 1.0))
    hs, k2 = f(HI[q] * S.get(q, 1.0)), f(2.0 / S.get(q, 1.0))
    with np.errstate(over="ignore", invalid="ignore"):
        u = (m * s).astype(f)
        cl = med3(u, -hs, hs)
        w = (u - cl).astype(f)
        # fma(w, 2^30, rint(cl)): w * 2^30 is exact (power of two), so fma rounds once like the add below
        c = (w * f(2 ** 30)).astype(f) + med3(np.rint(u), -hs, hs)
        co = f(hs + s)
        return (med3(c.astype(f), -co, co) * k2).astype(f)


def quantize_fast(x, q):  # nldpc_fused.h qms_q, NLDPC_QFAST: fma(med3(rint(x s), +-hi s), inv, +0)
    s, inv = f(S.get(q, 1.0)), f(1.0 / S.get(q, 1.0))
    hs = f(HI[q] * S.get(q, 1.0))
    with np.errstate(over="ignore", invalid="ignore"):
        return ((med3(np.rint((x * s).astype(f)), -hs, hs) * inv).astype(f) + f(0)).astype(f)


def inputs(q):
    rng = np.random.default_rng(q + 10)
    xs = np.concatenate([np.arange(-40, 40, 1 / 512, dtype=f), rng.normal(0, 12, 200_000).astype(f),
                         np.array([0.0, -0.0, np.inf, -np.inf, np.nan, 1e-30, -1e-30, 3e38, -3e38], f)])
    return np.concatenate([xs, np.nextafter(xs, f(np.inf)), np.nextafter(xs, f(-np.inf))]).astype(f)


@pytest.mark.parametrize("q", sorted(HI))
def test_qms_code_fast_form(q):
    """The compare-free code (r6) equals the definition on every input, NaN and infinities included."""
    xs = inputs(q)
    code = code_kernel_fast(xs, q)
    assert np.array_equal(code_definition(xs, q), code)
    # the kernel's conversion: fma(code, 1, 1.5 * 2^23) keeps the code in the low mantissa bits; the byte store keeps
    # the low byte, the code's two's complement
    byte = ((code + f(12582912.0)).astype(f).view(np.uint32) & 0xFF).astype(np.uint8).view(np.int8)
    assert np.array_equal(byte.astype(f), code)


@pytest.mark.parametrize("q", sorted(HI))
def test_fast_quantiser_equals_quantize(q):
    """qms_q in the fused kernels (r6): the compare-free form equals the reference's STE forward value bit for bit
    (signed zeros included) for every non-NaN input, so the posteriors, the VN-weight chain and the saved xin are
    unchanged (NaN: -hi instead of NaN)."""
    xs = inputs(q)
    ok = ~np.isnan(xs)
    a, b = quantize(xs[ok], q), quantize_fast(xs[ok], q)
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))


@pytest.mark.parametrize("q", sorted(HI))
def test_qms_code_identity(q):
    rng = np.random.default_rng(q + 10)
    xs = np.concatenate([np.arange(-40, 40, 1 / 512, dtype=f), rng.normal(0, 12, 200_000).astype(f),
                         np.array([0.0, -0.0, np.inf, -np.inf, np.nan, 1e-30, -1e-30, 3e38, -3e38], f)])
    xs = np.concatenate([xs, np.nextafter(xs, f(np.inf)), np.nextafter(xs, f(-np.inf))]).astype(f)
    a, b = code_definition(xs, q), code_kernel(xs, q)
    assert np.array_equal(a, b)
    assert np.abs(a).max() <= 2 * HI[q] + 2
