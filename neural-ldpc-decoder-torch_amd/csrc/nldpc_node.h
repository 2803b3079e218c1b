// Per-node arithmetic of the decoders, shared by the forward and backward kernels.
//
// check-node core (cn_core): the min-sum / quantised min-sum / Neural / sum-product update of one
// check copy over its d gathered inputs, reproducing NeuralLDPCDecoder.py:65-80 and
// BoostedNeuralLDPCDecoder.py:386-423 operation for operation;
// check-node epilogue (cn_epilogue): learned weighting + ReLU-mask + clip/quantise + sign
// (NeuralLDPCDecoder.py:89-91, Boosted…py:431-512);
// variable-node channel (vn_channel): cumulative VN weighting + quantisation (Boosted…py:325-337).
#pragma once

#include "nldpc_internal.h"
#include "nldpc_math.h"
#include "nldpc_sleef.h"

// gen_fused.py defines NLDPC_CNB_SPARSE 1 in the generated backward units (the tied check node of cn_bwd_ms, r6)
#ifndef NLDPC_CNB_SPARSE
#define NLDPC_CNB_SPARSE 0
#endif
#ifndef NLDPC_CNB_P2  // (r6) the tied QMS check node's folded pass 2 (cn_bwd_ms)
#define NLDPC_CNB_P2 1
#endif

namespace nldpc {

// ---- sum-product check node arithmetic, value for value the reference's CPU tensors
// (BoostedNeuralLDPCDecoder.py:400-408):
//   tanh   torch.tanh of a CPU fp32 tensor: the correctly rounded value of a double tanh, corrected
//          where torch's vector math differs by one ulp (table from gen_tanh_table.py, TanhRef)
//   prod   torch.prod(dim=3) in ATen's reduction order (sp_prod_others, the per-row plan of
//          nldpc_graph.cpp sp_plans)
//   atanh  ATen's vectorised atanh, SLEEF's Sleef_atanhf16_u10 (nldpc_sleef.h)
__device__ __noinline__ float tanh_ref(float x, TanhRef t) {
    const uint32_t key = __float_as_uint(x) & 0x7fffffffu;
    uint32_t r = __float_as_uint((float)tanh((double)__uint_as_float(key)));
    if (t.idx && key <= t.kmax) {  // no table (lib/nldpc_tanh_ref.bin missing): the rounded double tanh
        const uint32_t b = key >> t.sh;
        uint32_t lo = t.idx[b], hi = t.idx[b + 1];
        const uint32_t end = hi;
        while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            if ((t.ent[mid] & 0x7fffffffu) < key) lo = mid + 1;
            else hi = mid;
        }
        if (lo < end && (t.ent[lo] & 0x7fffffffu) == key) r = (t.ent[lo] >> 31) ? r + 1u : r - 1u;
        for (int i = 0; i < t.novr; ++i)
            if (t.ovr[2 * i] == key) r = t.ovr[2 * i + 1];
    }
    return __uint_as_float(r | (__float_as_uint(x) & 0x80000000u));
}

__device__ __noinline__ float atanh_ref(float x) { return nldpc_sleef::atanhf_u10(x); }

// Product of a row's SP factors except the sorted position sk, in ATen's order: ts holds the row's
// factors sorted by (lane, accumulator, position) (plan ord), code[s] = accumulator (bits 0-1) | a new
// lane starts at s (bit 2) | tail position (bit 3).  Every product the reference forms with a factor
// of exactly 1.0 (the other rows' entries, the masked self entry) is exact, so it is skipped.
template <int DC>
__device__ __forceinline__ void sp_step(float v, int c, float& P, float& a0, float& a1, float& a2, float& a3, bool& open) {
    // branch-free (selects): the code bytes are runtime values, and a branchy step unrolled DC^2 times
    // per check copy multiplied the kernels' control flow
    const bool tail = (c & 8) != 0;
    const int j = c & 3;
    const bool flush = open && (tail || (c & 4) != 0);
    P = flush ? fmul(P, fmul(fmul(a0, a1), fmul(a2, a3))) : P;
    a0 = flush ? 1.f : a0;
    a1 = flush ? 1.f : a1;
    a2 = flush ? 1.f : a2;
    a3 = flush ? 1.f : a3;
    const float tgt = tail ? P : (j == 0 ? a0 : (j == 1 ? a1 : (j == 2 ? a2 : a3)));
    const float pr = fmul(tgt, v);
    P = tail ? pr : P;
    a0 = (!tail && j == 0) ? pr : a0;
    a1 = (!tail && j == 1) ? pr : a1;
    a2 = (!tail && j == 2) ? pr : a2;
    a3 = (!tail && j == 3) ? pr : a3;
    open = !tail;
}

// (Check degrees above 16 -- the 24 / 32 buckets of the streaming kernels -- run the loop rolled: SP
// there is rare, and unrolling DC^2 work per check copy for them dominated the library's build.)
template <int DC>
__device__ __forceinline__ float sp_prod_others(const float (&ts)[DC], int d, int sk, const uint8_t* code) {
    float P = 1.f, a0 = 1.f, a1 = 1.f, a2 = 1.f, a3 = 1.f;
    bool open = false;
    if constexpr (DC > 16) {
#pragma unroll 1
        for (int s = 0; s < d; ++s) sp_step<DC>(s == sk ? 1.f : ts[s], code[s], P, a0, a1, a2, a3, open);
    } else {
#pragma unroll
        for (int s = 0; s < DC; ++s)
            if (s < d) sp_step<DC>(s == sk ? 1.f : ts[s], code[s], P, a0, a1, a2, a3, open);
    }
    if (open) P = fmul(P, fmul(fmul(a0, a1), fmul(a2, a3)));
    return P;
}

// what the SP check node of one row needs: the row's plan (kSpPlanBytes: ord | inv | code) and the
// tanh table
struct SpRow {
    const uint8_t* plan;
    TanhRef tanh;
};

// Launch geometry shared by all node kernels: blockDim = (Vt copies, Bt codewords); grid =
// (ceil(B/Bt), nodes, ceil(Z/Vt)).  The node index (column j / check row i) is blockIdx.y, so a
// workgroup works on one node and every graph-table load is wave-uniform (scalar); lanes run along
// consecutive lifted copies, so each wave touches 64 consecutive floats of a message row.
struct Geo {
    int v;      // lifted copy
    int node;   // column j (VN) or check row i (CN)
    int64_t b;  // codeword
    bool ok;
};

__device__ __forceinline__ Geo geo(int64_t B, int Z) {
    Geo g;
    g.v = blockIdx.z * blockDim.x + threadIdx.x;
    g.node = blockIdx.y;
    g.b = (int64_t)blockIdx.x * blockDim.y + threadIdx.y;
    g.ok = g.v < Z && g.b < B;
    return g;
}

// Workgroups are always whole waves (a multiple of 64 threads) so wave-level shuffles in the
// reductions see 64 live lanes: Bt codewords are stacked until Vt*Bt is a multiple of 64, and a
// copy count that cannot get there within 512 threads is padded to a multiple of 64 lanes.
inline void node_geometry(int64_t B, int Z, int nodes, dim3& grid, dim3& block) {
    int vt, bt;
    if (Z > 512) {
        vt = 256;
        bt = 1;
    } else {
        int g = 64;
        while (Z % g) g >>= 1;  // gcd(Z, 64)
        const int base = 64 / g;
        if (Z * base <= 512) {
            vt = Z;
            bt = base * ((256 / (Z * base)) > 1 ? (256 / (Z * base)) : 1);
        } else {
            vt = (Z + 63) & ~63;
            bt = vt >= 256 ? 1 : 256 / vt;
        }
    }
    block = dim3(vt, bt, 1);
    grid = dim3((unsigned)((B + bt - 1) / bt), (unsigned)nodes, (unsigned)((Z + vt - 1) / vt));
}

// A node's degree is uniform over its workgroup (node-uniform grid), so the kernels switch on it once
// and run a body templated on the exact degree: fully unrolled edge loops without per-edge
// predicates, register arrays sized to the degree.  f(D, d): D = the compile-time array bound, d =
// the degree as a value (a constant for the exact cases; the bucketed tail passes the runtime degree).
template <int D>
struct Deg {
    static constexpr int value = D;
};
template <int MAXD, typename F>
__device__ __forceinline__ void deg_switch(int d, F&& f) {
    // only the cases up to MAXD (the launch's bucket of the graph's maximum degree) are instantiated,
    // so the register allocation is that of the largest degree that can occur
#define NLDPC_DEG_CASE(n) \
    case n:                \
        if constexpr (n <= MAXD) f(Deg<n>{}, n); \
        break;
    switch (d) {
        NLDPC_DEG_CASE(1) NLDPC_DEG_CASE(2) NLDPC_DEG_CASE(3) NLDPC_DEG_CASE(4) NLDPC_DEG_CASE(5)
        NLDPC_DEG_CASE(6) NLDPC_DEG_CASE(7) NLDPC_DEG_CASE(8) NLDPC_DEG_CASE(9) NLDPC_DEG_CASE(10)
        NLDPC_DEG_CASE(11) NLDPC_DEG_CASE(12)
        default:
            if constexpr (MAXD > 12) {
                if (d <= 16) {
                    if constexpr (MAXD >= 16) f(Deg<16>{}, d);
                } else if (d <= 24) {
                    if constexpr (MAXD >= 24) f(Deg<24>{}, d);
                } else if (d <= 32) {
                    if constexpr (MAXD >= 32) f(Deg<32>{}, d);
                } else {
                    if constexpr (MAXD >= 64) f(Deg<64>{}, d);
                }
            }
    }
#undef NLDPC_DEG_CASE
}

// Bucket of a graph's maximum degree (the MAXD of deg_switch): 12, 16, 24, 32 or 64.
inline int deg_max_bucket(int d) { return d <= 12 ? 12 : d <= 16 ? 16 : d <= 24 ? 24 : d <= 32 ? 32 : 64; }

// xin of absolute VN step `steps-1`: Q(...Q(Q(xa*w0)*w1)...) (Boosted…py:325-337).
template <int KIND>
__device__ __forceinline__ float vn_channel(float xa, const float* w_vn, int N, int j, int steps, int qbit) {
    if (KIND == NLDPC_NEURAL) return xa;
    float x = xa;
    if (w_vn) {
        for (int s = 0; s < steps; ++s) {
            x = fmul(x, w_vn[(int64_t)s * N + j]);
            if (KIND == NLDPC_QMS) x = quantize(x, qbit);
        }
    } else if (KIND == NLDPC_QMS) {
        x = quantize(x, qbit);  // idempotent: Q applied every iteration equals Q applied once
    }
    return x;
}

// Output of the check-node core for one check copy.
template <int DC>
struct CnCore {
    float out0[DC];  // x_output_0 per edge (before weighting)
    float mq[DC];    // MS/QMS/Neural: conditioned input (after Q/clip and the 1e-4 zero fix); SP: t' = tanh or 1
    float sg[DC];    // MS/QMS/Neural: sign factor (+-1) the magnitude is multiplied with
    float min1, min2;
    int idx1, idx2;  // first-index argmins (torch.min tie-break); -1 = none below the mask value
};

// the row's SP factors sorted by the plan (ts[s] = mq[ord[s]])
template <int DC>
__device__ __forceinline__ void sp_sorted(const float (&mq)[DC], int d, const uint8_t* plan, float (&ts)[DC]) {
    if constexpr (DC > 16) {
        for (int s = 0; s < DC; ++s) ts[s] = s < d ? mq[plan[s]] : 1.f;
    } else {
#pragma unroll
        for (int s = 0; s < DC; ++s) {
            float v = 1.f;
            if (s < d) {
                const int o = plan[s];
#pragma unroll
                for (int l = 0; l < DC; ++l) v = (l == o) ? mq[l] : v;
            }
            ts[s] = v;
        }
    }
}

template <int DC, int KIND>
__device__ __forceinline__ void cn_core(const float (&m)[DC], int d, int qbit, float lo, float hi, CnCore<DC>& c,
                                        const SpRow& sp) {
    if constexpr (KIND == NLDPC_SP && DC > 32) {
        return;  // validate_cfg rejects check degrees above 32 (the 64 bucket is never launched)
    } else if (KIND == NLDPC_SP) {
#pragma unroll
        for (int k = 0; k < DC; ++k) {
            if (k < d) {
                const float x = clampf(m[k], lo, hi);
                const float t = tanh_ref(fmul(-0.5f, x), sp.tanh);
                c.mq[k] = fadd(t, (fabsf(t) > 0.f) ? 0.f : 1.f);
            } else {
                c.mq[k] = 1.f;
            }
        }
        float ts[DC];
        sp_sorted<DC>(c.mq, d, sp.plan, ts);
#pragma unroll
        for (int k = 0; k < DC; ++k) {
            if (k < d) {
                float P = sp_prod_others<DC>(ts, d, sp.plan[32 + k], sp.plan + 64);
                P = clampf(P, -kSpClip, kSpClip);
                c.out0[k] = fmul(-2.f, atanh_ref(P));
            } else {
                c.out0[k] = 0.f;
            }
        }
        c.min1 = c.min2 = 0.f;
        c.idx1 = c.idx2 = -1;
        return;
    }
    float min1 = kMaskMag, min2 = kMaskMag;
    int idx1 = -1, idx2 = -1;
    unsigned npos = 0, posm = 0;
#pragma unroll
    for (int k = 0; k < DC; ++k) {
        if (k < d) {
            float x = m[k];
            if (KIND == NLDPC_QMS) x = quantize(x, qbit);
            if (KIND == NLDPC_MS) x = clampf(x, lo, hi);
            if (KIND != NLDPC_NEURAL) x = fadd(x, fmul(kZeroFix, (fabsf(x) > 0.f) ? 0.f : 1.f));
            c.mq[k] = x;
            const float ax = fabsf(x);
            const unsigned pos = x > 0.f;
            npos ^= pos;
            posm |= pos << k;
            if (ax > 0.f) {  // exact zeros are masked out of the min (Neural only; Boosted has none)
                if (ax < min1) {
                    min2 = min1;
                    idx2 = idx1;
                    min1 = ax;
                    idx1 = k;
                } else if (ax < min2) {
                    min2 = ax;
                    idx2 = k;
                }
            }
        } else {
            c.mq[k] = 0.f;
        }
    }
#pragma unroll
    for (int k = 0; k < DC; ++k) {
        if (k < d) {
            float mag = (k == idx1) ? min2 : min1;
            if (KIND != NLDPC_NEURAL) mag = (mag > kZeroFix) ? mag : fadd(mag, -kZeroFix);
            const float sgn = ((npos ^ (posm >> k)) & 1u) ? 1.f : -1.f;
            c.sg[k] = sgn;
            c.out0[k] = fmul(mag, sgn);
        } else {
            c.sg[k] = 0.f;
            c.out0[k] = 0.f;
        }
    }
    c.min1 = min1;
    c.min2 = min2;
    c.idx1 = idx1;
    c.idx2 = idx2;
}

// Intermediate values of the epilogue of one edge (kept for the backward).
struct CnEpi {
    float c;    // resulting c2v message
    float x1;   // pre-ReLU weighted magnitude (Neural: |x|*w + b)
    float x2;   // post-ReLU (pre Q/clip) value (Boosted)
};

template <int KIND, bool UCN>
__device__ __forceinline__ CnEpi cn_epilogue(float x, float wc, float wu, float bias, float u, bool has_w, bool has_u,
                                             int qbit, float lo, float hi) {
    CnEpi r;
    const float ax = fabsf(x);
    if (KIND == NLDPC_NEURAL) {
        const float t = fadd(fmul(ax, wc), bias);  // two roundings (NeuralLDPCDecoder.py:89)
        r.x1 = t;
        r.x2 = relu_mask(t);
        r.c = fmul(r.x2, signf_t(x));
        return r;
    }
    float x1;
    if (!has_w) {
        x1 = ax;
    } else if (UCN && has_u) {
        const float x11 = fmul(ax, wc);
        const float x12 = fmul(ax, wu);
        x1 = fadd(fmul(x11, fadd(-u, 1.f)), fmul(x12, u));
    } else {
        x1 = fmul(ax, wc);
    }
    const float x2 = relu_mask(x1);
    const float x3 = (KIND == NLDPC_QMS) ? quantize(x2, qbit) : clampf(x2, lo, hi);
    r.x1 = x1;
    r.x2 = x2;
    r.c = fmul(x3, signf_t(x));
    return r;
}

// Hard-decision parity of a check copy for the UCN flag: odd number of row variables with
// APP >= 0 (Boosted…py:346-359).  app == nullptr: APP = xin_0 recomputed from xa and w_vn row 0.
template <int DC, int KIND>
__device__ __forceinline__ float ucn_flag(const DevGraph& g, int beg, int d, const int (&vv)[DC], int64_t b,
                                          const float* app, const float* xa, const float* w_vn0, int qbit) {
    int par = 0;
#pragma unroll
    for (int k = 0; k < DC; ++k) {
        if (k < d) {
            const int j = g.e_var[beg + k];
            const int64_t off = (b * g.N + j) * g.Z + vv[k];
            float v;
            if (app) {
                v = app[off];
            } else {
                v = xa[off];
                if (w_vn0) v = fmul(v, w_vn0[j]);
                if (KIND == NLDPC_QMS) v = quantize(v, qbit);
            }
            par ^= (-v <= 0.f) ? 1 : 0;
        }
    }
    return par ? 1.f : 0.f;
}

// Backward of one check copy of a degree-DC row (shared by the streaming cnb_kernel and the fused
// backward kernels): from the gathered v2c inputs m and the incoming dL/dc2v gc, recompute the
// forward (cn_core + cn_epilogue) and push the gradient back through sign, clip/quantise
// (straight-through, closed interval), ReLU mask, learned weights, |.|, and the min (to the
// first-index argmin of the others, as torch.min's backward) or the sum-product chain.
// Out: gm = dL/dm per edge, gw/gu/gb = this copy's contributions to dL/dw_cn, dL/dw_ucn, dL/dbias.
template <int DC, int KIND, bool UCN>
__device__ __forceinline__ void cn_backward(const float (&m)[DC], const float (&gc)[DC], int d, float u,
                                            const float (&wc)[DC], const float (&wu)[DC], const float (&bb)[DC],
                                            bool has_w, bool has_u, int qbit, float lo, float hi, float (&gm)[DC],
                                            float (&gw)[DC], float (&gu)[DC], float (&gb)[DC], const SpRow& sp) {
    CnCore<DC> core;
    cn_core<DC, KIND>(m, d, qbit, lo, hi, core, sp);

    const QRange qr = q_range(qbit);
    float gout[DC];  // dL/dx_output_0 per edge
#pragma unroll
    for (int k = 0; k < DC; ++k) {
        gw[k] = gu[k] = gb[k] = 0.f;
        gout[k] = 0.f;
        if (k < d) {
            const float x = core.out0[k];
            const CnEpi r = cn_epilogue<KIND, UCN>(x, wc[k], wu[k], bb[k], u, has_w, has_u, qbit, lo, hi);
            const float s = signf_t(x), ax = fabsf(x);
            float gabs;
            if (KIND == NLDPC_NEURAL) {
                const float ga = (gc[k] * s) * (r.x1 > 0.f ? 1.f : 0.f);
                gw[k] = ga * ax;
                gb[k] = ga;
                gabs = ga * wc[k];
            } else {
                float g2 = gc[k] * s;
                if (KIND == NLDPC_QMS) {
                    if (qr.active) g2 *= in_range(r.x2, qr.lo, qr.hi);
                } else {
                    g2 *= in_range(r.x2, lo, hi);
                }
                const float g1 = g2 * (r.x1 > 0.f ? 1.f : 0.f);
                if (!has_w) {
                    gabs = g1;
                } else if (UCN && has_u) {
                    const float g11 = g1 * (1.f - u), g12 = g1 * u;
                    gw[k] = g11 * ax;
                    gu[k] = g12 * ax;
                    gabs = g11 * wc[k] + g12 * wu[k];
                } else {
                    gw[k] = g1 * ax;
                    gabs = g1 * wc[k];
                }
            }
            gout[k] = gabs * s;
        }
    }

    if (KIND == NLDPC_SP) {
        float graw[DC], ts[DC];
#pragma unroll
        for (int l = 0; l < DC; ++l) graw[l] = 0.f;
        sp_sorted<DC>(core.mq, d, sp.plan, ts);
#pragma unroll
        for (int k = 0; k < DC; ++k) {
            if (k < d) {
                const float P = sp_prod_others<DC>(ts, d, sp.plan[32 + k], sp.plan + 64);
                const float Pc = clampf(P, -kSpClip, kSpClip);
                // d(-2 atanh(P))/dP = -2 / (1 - P^2); clamp passes on the closed interval
                const float gP = gout[k] * (-2.f / (1.f - Pc * Pc)) * in_range(P, -kSpClip, kSpClip);
#pragma unroll
                for (int l = 0; l < DC; ++l)
                    if (l < d && l != k) graw[l] += gP * (P / core.mq[l]);  // torch.prod backward form
            }
        }
#pragma unroll
        for (int l = 0; l < DC; ++l) {
            if (l < d) {
                const float xc = clampf(m[l], lo, hi);
                const float t = tanh_ref(fmul(-0.5f, xc), sp.tanh);
                gm[l] = graw[l] * (1.f - t * t) * -0.5f * in_range(m[l], lo, hi);
            } else {
                gm[l] = 0.f;
            }
        }
    } else {
        // torch.min backward: edge k's magnitude came from the first-index argmin of the OTHER
        // edges, i.e. idx2 for k == idx1 and idx1 otherwise, so only two inputs receive gradient
        float g_at1 = 0.f, g_at2 = 0.f;
#pragma unroll
        for (int k = 0; k < DC; ++k) {
            if (k < d) {
                const float gmag = gout[k] * core.sg[k];
                if (k == core.idx1) g_at2 += gmag;
                else g_at1 += gmag;
            }
        }
#pragma unroll
        for (int l = 0; l < DC; ++l) {
            float msk = 1.f;
            if (KIND == NLDPC_QMS && qr.active) msk = in_range(m[l], qr.lo, qr.hi);
            if (KIND == NLDPC_MS) msk = in_range(m[l], lo, hi);
            const float gl = l == core.idx1 ? g_at1 : (l == core.idx2 ? g_at2 : 0.f);
            gm[l] = (gl * signf_t(core.mq[l])) * msk;
        }
    }
}

// Register-light min-sum backward of one check copy (MS / QMS / Neural) for the fused backward
// kernels: cn_backward's arithmetic (same operations, same order, same results) restructured into
// three passes over the edges so that only the two minima and per-edge bit masks stay live between
// them.  load_m(k) gives edge k's v2c input (QMS: the decoded int8 code of the saved state, with an
// active quantiser); lds[k * stride] holds dL/dc2v on entry and receives
// dL/dv2c.  gwa / gba accumulate this copy's dL/dw_cn and dL/dbias contributions.
// SAMEW (the tied-weight kernel: one CN weight for the whole row): every edge but the first-index argmin
// has the same magnitude, so the epilogue's masks take two values per row, computed once (the same
// operations on the same values as per edge: the results are bit-identical), and the weight gradient is one
// running sum in gwa[0] (r5: cfg5 backward 27.3 -> 26.5 ms, profiles/r5o_ab_tied_bwd_masks.txt).
template <int DC, int KIND, bool SAMEW = false, typename LoadM>
__device__ __forceinline__ void cn_bwd_ms(LoadM&& load_m, float* lds, int stride, const float (&wc)[DC],
                                          const float (&bb)[DC], bool has_w, int qbit, float lo, float hi,
                                          float (&gwa)[DC], float (&gba)[DC]) {
    const QRange qr = q_range(qbit);
    float min1 = kMaskMag, min2 = kMaskMag;
    int idx1 = -1, idx2 = -1;
    uint32_t npos = 0, posm = 0, negm = 0, mskm = 0;
    // r6 (gen_fused.py NLDPC_GEN_CNBSPARSE): the tied kernel's check node with fewer VALU (below); the untied kernel
    // keeps the r5 form (the same edits there spilled 204 VGPRs)
    constexpr bool kSparse = NLDPC_CNB_SPARSE && SAMEW;
    constexpr bool kKeys = kSparse && KIND == NLDPC_QMS && DC >= 2 && DC <= 16;
    // (r6, NLDPC_CNB_P2) key bits below the index: the sign and the STE mask of the edge, so that pass 3 reads the two
    // argmins' own from their keys; every code value's float has its low 17 mantissa bits clear
    constexpr bool kP2 = kKeys && NLDPC_CNB_P2;
    uint32_t ka = 0, kb = 0;
    if constexpr (kP2) {
        // pass 1: key = max(bits(|xc|), bits(1e-4) & ~63) | k << 2 | neg << 1 | ok -- the zero fix as the max (every
        // nonzero |xc| >= 0.5), the sign from xd's sign bit (a decoded code is never -0, and the clamp and the zero fix
        // keep it), the mask as clamp(x) == x; the ordering by (|x|, k) is the r6 key's
        constexpr uint32_t kZk = 0x38D1B717u & ~63u;
        static_assert(__builtin_bit_cast(uint32_t, kZeroFix) == 0x38D1B717u, "zero-fix constant");
#pragma unroll
        for (int k = 0; k < DC; ++k) {
            const float xd = load_m(k);
            const float xc = __builtin_amdgcn_fmed3f(xd, qr.lo, qr.hi);
            const uint32_t ok = xc == xd;
            const uint32_t neg = __builtin_bit_cast(uint32_t, xd) >> 31;
            negm |= neg << k;
            const uint32_t key = max(__builtin_bit_cast(uint32_t, xc) & 0x7FFFFFFFu, kZk) | ((uint32_t)k << 2) | (neg << 1) | ok;
            if (k == 0) {
                ka = key;
            } else if (k == 1) {
                kb = max(ka, key);
                ka = min(ka, key);
            } else {
                asm("v_med3_u32 %0, %1, %2, %3" : "=v"(kb) : "v"(ka), "v"(kb), "v"(key));
                ka = min(ka, key);
            }
        }
        posm = ~negm & ((1u << DC) - 1u);
        npos = (uint32_t)__builtin_popcount(posm) & 1u;
        idx1 = (int)((ka >> 2) & 15u);
        idx2 = (int)((kb >> 2) & 15u);
        min1 = (ka & ~63u) == kZk ? kZeroFix : __builtin_bit_cast(float, ka & ~63u);
        min2 = (kb & ~63u) == kZk ? kZeroFix : __builtin_bit_cast(float, kb & ~63u);
    } else if constexpr (kKeys) {
        // (r6) QMS pass 1 on ordering keys: every conditioned input is a decoded int8 code (a multiple of 0.5 below 17,
        // a few mantissa bits) or the zero fix 1e-4, so (bits(|x|) & ~15) | k orders the edges by |x| with the first
        // index winning ties -- torch.min's argmin -- and the two smallest keys (v_min_u32 / v_med3_u32, two ops per
        // edge) give both minima and both indices: no compare-and-select chain per edge.  The STE mask as one compare
        // (clamp(x) == x), x never 0 after the zero fix so x < 0 is !(x > 0).  Bit-identical inputs to passes 2 and 3.
#pragma unroll
        for (int k = 0; k < DC; ++k) {
            const float xd = load_m(k);
            const float xc = __builtin_amdgcn_fmed3f(xd, qr.lo, qr.hi);
            const uint32_t msk = xc == xd;
            const float x = xc == 0.f ? kZeroFix : xc;
            const uint32_t pos = x > 0.f;
            npos ^= pos;
            posm |= pos << k;
            mskm |= msk << k;
            const uint32_t key = (__builtin_bit_cast(uint32_t, fabsf(x)) & ~15u) | (uint32_t)k;
            if (k == 0) {
                ka = key;
            } else if (k == 1) {
                kb = max(ka, key);
                ka = min(ka, key);
            } else {
                asm("v_med3_u32 %0, %1, %2, %3" : "=v"(kb) : "v"(ka), "v"(kb), "v"(key));
                ka = min(ka, key);
            }
        }
        negm = ~posm & ((1u << DC) - 1u);
        idx1 = (int)(ka & 15u);
        idx2 = (int)(kb & 15u);
        constexpr uint32_t kZf = 0x38D1B717u;  // bits of kZeroFix (1e-4f): the one conditioned value with low bits set
        static_assert(__builtin_bit_cast(uint32_t, kZeroFix) == kZf, "zero-fix constant");
        min1 = (ka & ~15u) == (kZf & ~15u) ? kZeroFix : __builtin_bit_cast(float, ka & ~15u);
        min2 = (kb & ~15u) == (kZf & ~15u) ? kZeroFix : __builtin_bit_cast(float, kb & ~15u);
    } else {
#pragma unroll
    for (int k = 0; k < DC; ++k) {  // pass 1: conditioned inputs, minima, signs, STE masks
        float x = load_m(k);
        bool msk = true;
        if (KIND == NLDPC_QMS) msk = x >= qr.lo && x <= qr.hi;
        if (KIND == NLDPC_MS) msk = x >= lo && x <= hi;
        // QMS inputs are decoded int8 codes (qms_code): on the quantiser's grid inside the clip range,
        // +-(hi + 1) outside it, so Q(m) is a clamp
        if (KIND == NLDPC_QMS) x = __builtin_amdgcn_fmed3f(x, qr.lo, qr.hi);
        if (KIND == NLDPC_MS) x = __builtin_amdgcn_fmed3f(x, lo, hi);
        if (KIND != NLDPC_NEURAL) x = x == 0.f ? kZeroFix : x;
        const float ax = fabsf(x);
        const uint32_t pos = x > 0.f;
        npos ^= pos;
        posm |= pos << k;
        negm |= (uint32_t)(x < 0.f) << k;
        mskm |= (uint32_t)msk << k;
        if constexpr (kSparse) {
        // (r6) branch-free: the nested ifs compiled to exec-mask branches with v_mov copies of the four trackers at
        // every edge (60 VALU per edge copy in the tied QMS kernel).  MS / QMS inputs are never 0 after the zero fix,
        // so only Neural needs the ax > 0 test (a NaN fails every compare either way).  lt1 implies lt2 (min1 <= min2).
            const bool ok = KIND == NLDPC_NEURAL ? ax > 0.f : true;
            const bool lt1 = ok && ax < min1, lt2 = ok && ax < min2;
            const float t2 = lt2 ? ax : min2;
            const int i2 = lt2 ? k : idx2;
            min2 = lt1 ? min1 : t2;
            idx2 = lt1 ? idx1 : i2;
            min1 = lt1 ? ax : min1;
            idx1 = lt1 ? k : idx1;
        } else {
        if (ax > 0.f) {
            if (ax < min1) {
                min2 = min1;
                idx2 = idx1;
                min1 = ax;
                idx1 = k;
            } else if (ax < min2) {
                min2 = ax;
                idx2 = k;
            }
        }
        }
    }
    }
    float g_at1 = 0.f, g_at2 = 0.f;
    if constexpr (kP2) {
        // (r6) the tied QMS check node's pass 2 with the per-row constants folded: the masks mA / mB are 0 or 1, so
        // ((gc s) m) |mag| == (gc s)(m |mag|) and ((gc s) m) w == (gc s)(m w) up to the sign of a zero (every sum here
        // starts from +0); s = +-1 is a sign flip of gc (bit k of R: s_k = -1), no compare or multiply; the first-index
        // argmin's own term (g_at2) once per row from its LDS slot instead of a select per edge, and its g_at1 term a
        // +0.  The same sums in the same order, bit for bit, for finite gradients (profiles/r6_ab_cnb_p2.txt).
        const float magA = (min1 > kZeroFix) ? min1 : fadd(min1, -kZeroFix);
        const float magB = (min2 > kZeroFix) ? min2 : fadd(min2, -kZeroFix);
        const float x1A = has_w ? fmul(fabsf(magA), wc[0]) : fabsf(magA);
        const float x1B = has_w ? fmul(fabsf(magB), wc[0]) : fabsf(magB);
        // (x1 > 0 ? in_range(relu(x1), lo, hi) : 0) with lo < 0: x1 in (0, hi] (NaN: 0, as before)
        const float mA = (x1A > 0.f && (!qr.active || x1A <= qr.hi)) ? 1.f : 0.f;
        const float mB = (x1B > 0.f && (!qr.active || x1B <= qr.hi)) ? 1.f : 0.f;
        const float PA = fmul(mA, fabsf(magA)), PB = fmul(mB, fabsf(magB));
        const float QA = has_w ? fmul(mA, wc[0]) : mA, QB = has_w ? fmul(mB, wc[0]) : mB;
        const uint32_t R = ~(posm ^ (0u - (npos & 1u)));
#pragma unroll
        for (int k = 0; k < DC; ++k) {
            const bool sel = k == idx1;
            const float gcs = __builtin_bit_cast(float, __builtin_bit_cast(uint32_t, lds[k * stride]) ^
                                                            ((R << (31 - k)) & 0x80000000u));
            if (has_w) gwa[0] += gcs * (sel ? PB : PA);
            g_at1 += gcs * (sel ? 0.f : QA);
        }
        const float gc1 = lds[idx1 * stride];
        const float gcs1 = __builtin_bit_cast(float, __builtin_bit_cast(uint32_t, gc1) ^ (((R >> idx1) & 1u) << 31));
        g_at2 = fadd(0.f, gcs1 * QB);
    } else if constexpr (SAMEW && KIND != NLDPC_NEURAL) {
        // A: every edge but idx1 (magnitude min1), B: edge idx1 (min2); the zero-fix correction, x1 = |x| w
        // (|x| = |mag|: x = mag * (+-1)), the clip / quantiser mask of relu(x1) and the relu mask, per row
        const float magA = (min1 > kZeroFix) ? min1 : fadd(min1, -kZeroFix);
        const float magB = (min2 > kZeroFix) ? min2 : fadd(min2, -kZeroFix);
        const float x1A = has_w ? fmul(fabsf(magA), wc[0]) : fabsf(magA);
        const float x1B = has_w ? fmul(fabsf(magB), wc[0]) : fabsf(magB);
        // (g2 * mq) * mp == g2 * (mq * mp) bit for bit when both masks are 0 or 1: one mask per case
        const bool qmask = KIND == NLDPC_MS || qr.active;
        const float mqA = !qmask ? 1.f : KIND == NLDPC_QMS ? in_range(relu_mask(x1A), qr.lo, qr.hi) : in_range(relu_mask(x1A), lo, hi);
        const float mqB = !qmask ? 1.f : KIND == NLDPC_QMS ? in_range(relu_mask(x1B), qr.lo, qr.hi) : in_range(relu_mask(x1B), lo, hi);
        const float mA = (x1A > 0.f) ? mqA : 0.f, mB = (x1B > 0.f) ? mqB : 0.f;
#pragma unroll
        for (int k = 0; k < DC; ++k) {
            const bool sel = k == idx1;
            const float mag = sel ? magB : magA;
            const float sgn = ((npos ^ (posm >> k)) & 1u) ? 1.f : -1.f;
            const float x = fmul(mag, sgn);
            // (r6 sparse) QMS: mag >= 0 (the minima are >= the zero fix 1e-4), so sign(x) is sgn, or 0 with mag == 0,
            // where x1 = 0 and the relu mask makes g1 a zero either way (its sign is lost in the +0-started sums)
            const float s = (kSparse && KIND == NLDPC_QMS) ? sgn : signf_t(x);
            const float ax = kSparse ? fabsf(mag) : fabsf(x);  // (|mag * (+-1)| == |mag|: no multiply for it)
            const float gc = lds[k * stride];
            const float g1 = (gc * s) * (sel ? mB : mA);
            float gabs;
            if (!has_w) {
                gabs = g1;
            } else {
                // one running sum in gwa[0] instead of one per edge: the tied kernel adds gwa[0..DC-1] in edge
                // order from 0 (cnb_row), and 0 + ... + g1_k ax_k in edge order is that sum bit for bit (a
                // partial sum from +0 is never -0, so adding +-0 terms directly or as 0 + term is the same)
                gwa[0] += g1 * ax;
                gabs = g1 * wc[kSparse ? 0 : k];  // (r6 sparse: the tied contract -- the row is wc[0] -- one scalar)
            }
            // (r6 sparse) s = sgn, or s = 0 with a zero magnitude, where g1 and gabs are +-0: (gabs * s) * sgn == gabs up
            // to the sign of a zero, which the +0-started sums g_at1 / g_at2 never keep
            const float gmag = kSparse ? gabs : (gabs * s) * sgn;
            if (sel) g_at2 += gmag;
            else g_at1 += gmag;
        }
    } else {
#pragma unroll
    for (int k = 0; k < DC; ++k) {  // pass 2: epilogue backward per edge (cn_backward's formulas)
        float mag = (k == idx1) ? min2 : min1;
        if (KIND != NLDPC_NEURAL) mag = (mag > kZeroFix) ? mag : fadd(mag, -kZeroFix);
        const float sgn = ((npos ^ (posm >> k)) & 1u) ? 1.f : -1.f;
        const float x = fmul(mag, sgn);
        const CnEpi r = cn_epilogue<KIND, false>(x, wc[k], 0.f, bb[k], 0.f, has_w, false, qbit, lo, hi);
        const float s = signf_t(x), ax = fabsf(x);
        const float gc = lds[k * stride];
        float gabs;
        if (KIND == NLDPC_NEURAL) {
            const float ga = (gc * s) * (r.x1 > 0.f ? 1.f : 0.f);
            gwa[k] += ga * ax;
            gba[k] += ga;
            gabs = ga * wc[k];
        } else {
            float g2 = gc * s;
            if (KIND == NLDPC_QMS) {
                if (qr.active) g2 *= in_range(r.x2, qr.lo, qr.hi);
            } else {
                g2 *= in_range(r.x2, lo, hi);
            }
            const float g1 = g2 * (r.x1 > 0.f ? 1.f : 0.f);
            if (!has_w) {
                gabs = g1;
            } else {
                gwa[k] += g1 * ax;
                gabs = g1 * wc[k];
            }
        }
        const float gmag = (gabs * s) * sgn;
        if (k == idx1) g_at2 += gmag;
        else g_at1 += gmag;
    }
    }
    if constexpr (kSparse) {
    // (r6) pass 3 sparse: every edge gets 0, then the two argmins their value at a per-lane LDS address -- (gl * smq) *
    // msk of the dense form for those two, +0 instead of a -0 for the others (every consumer adds them to a sum
    // started from +0: the owners' VN backward and the degree-1 chains)
#pragma unroll
    for (int l = 0; l < DC; ++l) lds[l * stride] = 0.f;
    if constexpr (kP2) {
        // (r6) the argmins' sign and mask from their keys: (gl * (+-1)) * msk as a sign flip and a select (a zero of
        // either sign for a masked edge, as the dense form's product -- every consumer's sum starts from +0)
        auto putk = [&](uint32_t key, float gl) {
            const float v = __builtin_bit_cast(float, __builtin_bit_cast(uint32_t, gl) ^ ((key & 2u) << 30));
            lds[((key >> 2) & 15u) * stride] = (key & 1u) ? v : 0.f;
        };
        putk(ka, g_at1);
        putk(kb, g_at2);
        return;
    }
    auto put = [&](int l, float gl) {
        const float smq = ((posm >> l) & 1u) ? 1.f : (((negm >> l) & 1u) ? -1.f : 0.f);
        lds[l * stride] = (gl * smq) * (((mskm >> l) & 1u) ? 1.f : 0.f);
    };
    if (idx1 >= 0) put(idx1, g_at1);
    if (idx2 >= 0) put(idx2, g_at2);
    } else {
#pragma unroll
    for (int l = 0; l < DC; ++l) {  // pass 3: the two argmins receive the gradient
        const float gl = l == idx1 ? g_at1 : (l == idx2 ? g_at2 : 0.f);
        const float smq = ((posm >> l) & 1u) ? 1.f : (((negm >> l) & 1u) ? -1.f : 0.f);
        lds[l * stride] = (gl * smq) * (((mskm >> l) & 1u) ? 1.f : 0.f);
    }
    }
}

}  // namespace nldpc
