// Device-side scalar arithmetic shared by the forward and backward kernels.
//
// Every helper reproduces one fp32 operation sequence of the reference exactly:
// one IEEE rounding per reference op, no contraction (the library is built with
// -ffp-contract=off and the products/sums below use explicit _rn intrinsics), round-half-even
// quantisation, and the reference's masking constants.
#pragma once

#include <hip/hip_runtime.h>

namespace nldpc {

__device__ __forceinline__ float fadd(float a, float b) { return __fadd_rn(a, b); }
__device__ __forceinline__ float fmul(float a, float b) { return __fmul_rn(a, b); }

// torch.clamp(x, lo, hi): NaN passes through
__device__ __forceinline__ float clampf(float x, float lo, float hi) {
    float y = x < lo ? lo : x;
    return y > hi ? hi : y;
}

// torch.sign
__device__ __forceinline__ float signf_t(float x) { return (float)(x > 0.f) - (float)(x < 0.f); }

// x * (x > 0).float()  (the reference's ReLU-by-mask, NeuralLDPCDecoder.py:90, Boosted…py:505) as one
// v_max_f32: the same value for every non-NaN x (x <= 0 gives +0 where the reference's product gives
// -0 for negative x; a zero c2v of either sign only ever meets the +0-started sums of the VN, so no
// output or later message differs)
__device__ __forceinline__ float relu_mask(float x) { return __builtin_fmaxf(x, 0.f); }

// QMS quantiser (BoostedNeuralLDPCDecoder.py:187-214): forward value of the straight-through
// estimator, x_clipped + (q_value - x_clipped), evaluated in fp32 like the reference.
struct QRange {
    float lo, hi;
    bool active;
};

__device__ __forceinline__ QRange q_range(int q) {
    switch (q) {
        case 6: return {-15.5f, 15.5f, true};
        case 5: return {-7.5f, 7.5f, true};
        case -5: return {-15.f, 15.f, true};
        case 4: return {-7.f, 7.f, true};
        case 3: return {-6.f, 6.f, true};
        default: return {0.f, 0.f, false};
    }
}

__device__ __forceinline__ float quantize(float x, int q) {
    // Branch-free over the (wave-uniform) q: every active q is clamp(rint(x*s)/s) with s in {2, 1, 1/2},
    // where the scalings are exact, so this equals the per-q formulas of the reference bit for bit:
    // q=5 rint(2x)/2 in +-7.5, q=6 rint(x) in +-15.5, q=-5 rint(x) in +-15, q=4 rint(x) in +-7,
    // q=3 rint(x/2)*2 in +-6.  The parameter selects are scalar and hoisted out of loops.
    const float s = q == 5 ? 2.f : (q == 3 ? 0.5f : 1.f);
    const float inv = q == 5 ? 0.5f : (q == 3 ? 2.f : 1.f);
    const float hi = q == 6 ? 15.5f : (q == 5 ? 7.5f : (q == -5 ? 15.f : (q == 4 ? 7.f : 6.f)));
    const bool active = q == 6 || q == 5 || q == -5 || q == 4 || q == 3;
    const float qv = clampf(fmul(rintf(fmul(x, s)), inv), -hi, hi);
    const float xc = clampf(x, -hi, hi);
    const float r = fadd(xc, __fsub_rn(qv, xc));
    return active ? r : x;
}

// The same quantiser in four operations when q is active: clamp(rint(x*s), +-hi*s) * inv.  Equal to
// quantize() for every non-NaN x: the STE form xc + (qv - xc) is exactly qv (|qv - xc| is below the
// grid step, so the difference is exact and so is the sum), and clamping commutes with the exact
// power-of-two scalings (checked exhaustively over random and boundary inputs for every q).
__device__ __forceinline__ float quantize_active(float x, int q) {
    const float s = q == 5 ? 2.f : (q == 3 ? 0.5f : 1.f);
    const float inv = q == 5 ? 0.5f : (q == 3 ? 2.f : 1.f);
    const float hs = q == 6 ? 15.5f : (q == 5 ? 15.f : (q == -5 ? 15.f : (q == 4 ? 7.f : 3.f)));  // hi * s
    return fmul(__builtin_amdgcn_fmed3f(rintf(fmul(x, s)), -hs, hs), inv);
}
__device__ __forceinline__ bool qms_active_q(int q) { return q == 6 || q == 5 || q == -5 || q == 4 || q == 3; }

// An active quantiser's constants, computed once on the host (FusedArgs::qp) so the fused kernels read
// four kernel-argument floats instead of re-deriving them from q with scalar compare/select chains at
// every use: scale s, 1/s, clip hi and hi*s (s in {2, 1, 1/2}: every scaling is exact).
struct QParams {
    float s, inv, hi, hs;
};
__host__ __device__ inline QParams q_params(int q) {
    const float s = q == 5 ? 2.f : (q == 3 ? 0.5f : 1.f);
    const float hi = q == 6 ? 15.5f : (q == 5 ? 7.5f : (q == -5 ? 15.f : (q == 4 ? 7.f : 6.f)));
    return QParams{s, q == 5 ? 0.5f : (q == 3 ? 2.f : 1.f), hi, hi * s};
}
// quantize() for an active q (the reference's STE form, same operations in the same order)
__device__ __forceinline__ float quantize_p(float x, const QParams& p) {
    const float qv = clampf(fmul(rintf(fmul(x, p.s)), p.inv), -p.hi, p.hi);
    const float xc = clampf(x, -p.hi, p.hi);
    return fadd(xc, __fsub_rn(qv, xc));
}
// quantize_active() with the constants given
__device__ __forceinline__ float quantize_active_p(float x, const QParams& p) {
    return fmul(__builtin_amdgcn_fmed3f(rintf(fmul(x, p.s)), -p.hs, p.hs), p.inv);
}

// QMS training state.  The backward reads a saved v2c message m only through Q(m) and the STE mask of
// Q's clip on m, so QMS saves one signed byte 2*m' per message: m' = Q(m) inside the clip range and
// sign(m) * (hi + 1) outside it, which gives Q(m') == Q(m) and the same mask (Q's values are
// multiples of 1/2 with |2 m'| <= 33).  A quarter of the fp32 traffic, both directions.
// For an active q in nine operations (the saved-state writes are a QMS training forward's hottest VALU
// work): inside the clip range 2 Q(m) = med3(rint(m s), +-hi s) * 2/s exactly (quantize_active); outside
// it sign(m) (2 hi + 2); NaN gives -(2 hi + 2) as the definition does (tests/test_qms_code.py checks the
// identity over every grid boundary and random inputs for every q).
__device__ __forceinline__ int qms_code(float m, int q) {
    const QRange r = q_range(q);
    if (!r.active) {  // (not used: QMS saves codes only with an active quantiser)
        const float mp = (m >= r.lo && m <= r.hi) ? quantize(m, q) : (m > 0.f ? r.hi + 1.f : -(r.hi + 1.f));
        return (int)rintf(2.f * mp);
    }
    const float s = q == 5 ? 2.f : (q == 3 ? 0.5f : 1.f);
    const float k2 = q == 5 ? 1.f : (q == 3 ? 4.f : 2.f);  // 2 / s
    const float hs = q == 6 ? 15.5f : (q == 5 ? 15.f : (q == -5 ? 15.f : (q == 4 ? 7.f : 3.f)));  // hi * s
    const float c_out = 2.f * r.hi + 2.f;
    const float t = fmul(__builtin_amdgcn_fmed3f(rintf(fmul(m, s)), -hs, hs), k2);
    const float c = fabsf(m) <= r.hi ? t : (m > 0.f ? c_out : -c_out);
    return (int)c;
}
// qms_code() for an active q with the constants given (2 / s = 2 inv); NLDPC_QFAST: the code modulo 256 (byte stores)
// NLDPC_QFAST (default; r6): no compare or select.  With u = m s (exact), cl = med3(u, +-hi s) and w = u - cl (0
// inside the clip range, of the sign of m and at least one ulp of hi s outside it): w * 2^30 + med3(rint(u), +-hi s)
// is the in-range value inside the range and beyond (hi + 1) s outside it, so one more med3 at +-(hi + 1) s gives
// the code / (2/s) in both cases.  (rint before the clip, as quantize_active: q = 6's hi s = 15.5 is not an integer.)  NaN: v_med3_f32 with a NaN operand returns the minimum of the other two (the gfx9 ISA definition,
// also LLVM's constant folding of llvm.amdgcn.fmed3), so cl = -hi s, c = NaN and the code -(2 hi + 2), as defined.
// (tests/test_qms_code.py models both forms.)
#ifndef NLDPC_QFAST
#define NLDPC_QFAST 1
#endif
__device__ __forceinline__ int qms_code_p(float m, const QParams& p) {
#if NLDPC_QFAST
    const float u = fmul(m, p.s);
    const float cl = __builtin_amdgcn_fmed3f(u, -p.hs, p.hs);
    const float r = __builtin_amdgcn_fmed3f(rintf(u), -p.hs, p.hs);
    const float c = __builtin_fmaf(__fsub_rn(u, cl), 1073741824.f, r);
    const float co = p.hs + p.s;  // (hi + 1) s
    // the conversion to an integer as an add of 1.5 * 2^23 folded into the scaling: the code k (|k| <= 33) is exact in
    // the low mantissa bits of 1.5 * 2^23 + k, whose low byte is k's two's complement -- all the byte store keeps
    // (no v_cvt_i32_f32; the returned int is the code only modulo 256)
    return __builtin_bit_cast(int, __builtin_fmaf(__builtin_amdgcn_fmed3f(c, -co, co), 2.f * p.inv, 12582912.f));
#else
    const float c_out = 2.f * p.hi + 2.f;
    const float t = fmul(__builtin_amdgcn_fmed3f(rintf(fmul(m, p.s)), -p.hs, p.hs), 2.f * p.inv);
    const float c = fabsf(m) <= p.hi ? t : (m > 0.f ? c_out : -c_out);
    return (int)c;
#endif
}
__device__ __forceinline__ float qms_decode(int c) { return 0.5f * (float)c; }

// STE / clamp gradient mask: 1 on the closed interval (torch.clamp backward), else 0
__device__ __forceinline__ float in_range(float x, float lo, float hi) { return (x >= lo && x <= hi) ? 1.f : 0.f; }

// Check-node magnitude cap for entries masked out of the tile (NeuralLDPCDecoder.py:74,
// Boosted…py:411-414): the masked value 10000 takes part in the min.
constexpr float kMaskMag = 10000.f;
constexpr float kZeroFix = 1e-4f;  // 0.0001 as fp32 (Boosted…py:393, :416)
// 1 - 1e-7 rounded to fp32 (Boosted…py:406-407)
constexpr float kSpClip = 0.99999988079071044921875f;

}  // namespace nldpc
