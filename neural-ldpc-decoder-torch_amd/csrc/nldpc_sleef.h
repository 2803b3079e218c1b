// tanhf / atanhf with the exact results of the CPU libm the reference's SP check node runs on.
//
// The reference's sum-product check node (src/boosted_neural_ldpc_decoder/BoostedNeuralLDPCDecoder.py:
// 400-408) evaluates torch.tanh and torch.atanh on CPU tensors.  ATen vectorises both through SLEEF's
// 1.0-ulp single-precision functions (Sleef_tanhf16_u10 / Sleef_atanhf16_u10 with AVX-512 FMA, the
// same arithmetic as the AVX2 FMA variants), whose results are not correctly rounded; a device tanhf
// that is a closer approximation still differs from the reference in the last bit of some values,
// and atanh's 1 / (1 - P^2) near saturation amplifies that to beyond the 1e-4 relative parity bar.
// These are restatements of SLEEF's published double-float algorithms (SLEEF 3.x, sleefsimdsp.c:
// xtanhf_u1 over expk2f, xatanhf over logk2f; df.h double-float primitives in their FMA form) in
// plain fp32 operations, so the device reproduces ATen's values bit for bit.  Checked exhaustively
// against ATen's own Sleef_*f16_u10 on every fp32 input of the decoder's domain
// (tools/dev/sleef_probe.c; tanh: |x| <= 10 after the +-20 LLR clamp, atanh: |x| < 1).
//
// Host and device: plain C arithmetic with explicit fmaf; compile without FP contraction
// (-ffp-contract=off) so no other multiply-add is fused.
#pragma once

#include <stdint.h>

#ifdef __HIPCC__
#define NLDPC_SLEEF_FN __host__ __device__ static inline
#else
#include <math.h>
#define NLDPC_SLEEF_FN static inline
#endif

namespace nldpc_sleef {

struct df2 {
    float x, y;
};

NLDPC_SLEEF_FN float bits2f(uint32_t u) {
    float f;
    __builtin_memcpy(&f, &u, 4);
    return f;
}
NLDPC_SLEEF_FN uint32_t f2bits(float f) {
    uint32_t u;
    __builtin_memcpy(&u, &f, 4);
    return u;
}
NLDPC_SLEEF_FN float fmaf_(float a, float b, float c) { return __builtin_fmaf(a, b, c); }
NLDPC_SLEEF_FN float pow2i(int q) { return bits2f((uint32_t)(q + 0x7f) << 23); }
NLDPC_SLEEF_FN float ldexp2(float d, int e) { return d * pow2i(e >> 1) * pow2i(e - (e >> 1)); }
NLDPC_SLEEF_FN int rint_i(float x) {  // round half to even (cvtps2dq)
    return (int)__builtin_rintf(x);
}

// ---- double-float primitives (df.h, FMA variants)
NLDPC_SLEEF_FN df2 dfadd_f_df(float x, df2 y) {  // |x| >= |y|
    const float s = x + y.x;
    return {s, ((x - s) + y.x) + y.y};
}
NLDPC_SLEEF_FN df2 dfadd_df_df(df2 x, df2 y) {  // |x| >= |y|
    const float s = x.x + y.x;
    return {s, (((x.x - s) + y.x) + x.y) + y.y};
}
NLDPC_SLEEF_FN df2 dfadd2_df_f(df2 x, float y) {
    const float s = x.x + y;
    const float v = s - x.x;
    const float w = (x.x - (s - v)) + (y - v);
    return {s, w + x.y};
}
NLDPC_SLEEF_FN df2 dfadd2_f_f(float x, float y) {
    const float s = x + y;
    const float v = s - x;
    return {s, (x - (s - v)) + (y - v)};
}
NLDPC_SLEEF_FN df2 dfadd2_df_df(df2 x, df2 y) {
    const float s = x.x + y.x;
    const float v = s - x.x;
    const float t = (x.x - (s - v)) + (y.x - v);
    return {s, t + (x.y + y.y)};
}
NLDPC_SLEEF_FN df2 dfneg(df2 x) { return {-x.x, -x.y}; }
NLDPC_SLEEF_FN df2 dfscale(df2 d, float s) { return {d.x * s, d.y * s}; }
NLDPC_SLEEF_FN df2 dfmul_df_f(df2 x, float y) {
    const float s = x.x * y;
    return {s, fmaf_(x.y, y, fmaf_(x.x, y, -s))};
}
NLDPC_SLEEF_FN df2 dfmul_df_df(df2 x, df2 y) {
    const float s = x.x * y.x;
    return {s, fmaf_(x.x, y.y, fmaf_(x.y, y.x, fmaf_(x.x, y.x, -s)))};
}
NLDPC_SLEEF_FN df2 dfsqu(df2 x) {
    const float s = x.x * x.x;
    return {s, fmaf_(x.x + x.x, x.y, fmaf_(x.x, x.x, -s))};
}
NLDPC_SLEEF_FN df2 dfrec_df(df2 d) {
    const float s = 1.0f / d.x;
    return {s, s * fmaf_(-d.y, s, fmaf_(-d.x, s, 1.0f))};
}
NLDPC_SLEEF_FN df2 dfdiv(df2 n, df2 d) {
    const float t = 1.0f / d.x;
    const float s = n.x * t;
    const float u = fmaf_(t, n.x, -s);
    const float v = fmaf_(-d.y, t, fmaf_(-d.x, t, 1.0f));
    return {s, fmaf_(s, v, fmaf_(n.y, t, u))};
}

// ---- exp(d) as a double-float (sleefsimdsp.c expk2f)
NLDPC_SLEEF_FN df2 expk2f(df2 d) {
    const float R_LN2f = 1.442695040888963407359924681001892137426645954152985934135449406931f;
    const float L2Uf = 0.693145751953125f, L2Lf = 1.428606765330187045e-06f;
    const float uq = (d.x + d.y) * R_LN2f;
    const int q = rint_i(uq);
    df2 s = dfadd2_df_f(d, (float)q * -L2Uf);
    s = dfadd2_df_f(s, (float)q * -L2Lf);
    float u = 0.1980960224e-3f;
    u = fmaf_(u, s.x, 0.1394256484e-2f);
    u = fmaf_(u, s.x, 0.8333456703e-2f);
    u = fmaf_(u, s.x, 0.4166637361e-1f);
    df2 t = dfadd2_df_f(dfmul_df_f(s, u), 0.166666659414234244790680580464e+0f);
    t = dfadd2_df_f(dfmul_df_df(s, t), 0.5f);
    t = dfadd2_df_df(s, dfmul_df_df(dfsqu(s), t));
    t = dfadd_f_df(1.0f, t);
    t.x = ldexp2(t.x, q);
    t.y = ldexp2(t.y, q);
    if (d.x < -104.0f) t = {0.0f, 0.0f};
    return t;
}

// ---- log(d) as a double-float (sleefsimdsp.c logk2f), d > 0 normal
NLDPC_SLEEF_FN df2 logk2f(df2 d) {
    const float a = d.x * (1.0f / 0.75f);
    const int e = (int)((f2bits(a) >> 23) & 0xff) - 127;  // ilogb / getexp of a normal number
    const df2 m = dfscale(d, pow2i(-e));
    const df2 x = dfdiv(dfadd2_df_f(m, -1.0f), dfadd2_df_f(m, 1.0f));
    const df2 x2 = dfsqu(x);
    float t = 0.2392828464508056640625f;
    t = fmaf_(t, x2.x, 0.28518211841583251953125f);
    t = fmaf_(t, x2.x, 0.400005877017974853515625f);
    t = fmaf_(t, x2.x, 0.666666686534881591796875f);
    df2 s = dfmul_df_f(df2{0.69314718246459960938f, -1.904654323148236017e-09f}, (float)e);
    s = dfadd_df_df(s, dfscale(x, 2.0f));
    s = dfadd_df_df(s, dfmul_df_f(dfmul_df_df(x2, x), t));
    return s;
}

NLDPC_SLEEF_FN float copysign_(float y, float x) {
    return bits2f((f2bits(y) & 0x7fffffffu) | (f2bits(x) & 0x80000000u));
}

// Sleef_tanhf*_u10 (xtanhf_u1)
NLDPC_SLEEF_FN float tanhf_u10(float x) {
    const float ax = bits2f(f2bits(x) & 0x7fffffffu);
    df2 d = expk2f(df2{ax, 0.0f});
    const df2 e = dfrec_df(d);
    d = dfdiv(dfadd_df_df(d, dfneg(e)), dfadd_df_df(d, e));
    float y = d.x + d.y;
    if (ax > 8.664339742f || y != y) y = 1.0f;
    y = copysign_(y, x);
    if (x != x) y = x;
    return y;
}

// Sleef_atanhf*_u10 (xatanhf)
NLDPC_SLEEF_FN float atanhf_u10(float x) {
    const float ax = bits2f(f2bits(x) & 0x7fffffffu);
    const df2 d = logk2f(dfdiv(dfadd2_f_f(1.0f, ax), dfadd2_f_f(1.0f, -ax)));
    float y;
    if (ax > 1.0f) y = bits2f(0x7fc00000u);
    else if (ax == 1.0f) y = __builtin_inff();
    else y = (d.x + d.y) * 0.5f;
    y = copysign_(y, x);
    if (x != x) y = x;
    return y;
}

}  // namespace nldpc_sleef
