// Backward through the unrolled decoder (config 5: training the learned weights; the reference
// gets these gradients from autograd over BoostedNeuralLDPCDecoder.py:320-526 and
// NeuralLDPCDecoder.py:54-98).
//
// Per iteration k, from the last to the first:
//   CNB(k)  one thread per check copy: recompute the check node from the saved v2c_k (gathered at
//           the cyclic shift), take dL/dc2v_{k+1} at the same addresses, and push it back through
//           sign, clip/quantise (straight-through, closed interval), ReLU mask, learned weights
//           (per-edge weight gradients: block reduction + one atomic per edge and block), |.|, and
//           the min (routed to the first-index argmin of the others, as torch.min's backward) or
//           the sum-product chain (tanh / product / atanh); writes dL/dv2c_k in place of v2c_k's
//           addresses.
//   VNB(k)  one thread per variable copy: dL/dc2v_k[e] = dL/dy_{k-1} (output clamp mask) +
//           sum of dL/dv2c_k over the column's other edges; and the cumulative VN-weight chain
//           xin_k = Q(xin_{k-1} * w_k) (straight-through masks, per-column weight gradients).
// Gradient sums over the batch use fp32 atomics, so the last bits may vary from run to run
// (tests use rtol 1e-4).
#include <hip/hip_runtime.h>

#include "nldpc_node.h"

namespace nldpc {

struct VNBArgs {
    DevGraph g;
    int64_t B;
    const float* gv2c;     // [B][E][Z] dL/dv2c_k, or nullptr (k == T)
    const float* gy;       // [B][N][Z] dL/dy_{k-1}, or nullptr
    const uint8_t* ymask;  // [B][N][Z] clamp mask of y_{k-1}, or nullptr (Neural: no clamp)
    float* gc2v;           // [B][E][Z] dL/dc2v_k out, or nullptr (k == 0)
    // cumulative VN weights (nullptr = no VN-weight gradient)
    const float* xa;
    const float* w_vn;     // [steps][N]
    float* g_w_vn;         // [steps][N]
    float* carry;          // [B][N][Z] dL/du_{p+1} * w_{p+1}
    int32_t step;          // absolute VN step p of this iteration
    int32_t qbit;
};

struct CNBArgs {
    DevGraph g;
    int64_t B;
    const float* v2c;     // saved v2c_k
    const float* gc2v;    // dL/dc2v_{k+1}
    float* gv2c;          // dL/dv2c_k out
    const float* w_cn;    // [E] or nullptr
    const float* w_ucn;   // [E] or nullptr
    const float* bias;    // [E] or nullptr
    float* g_w_cn;        // [E] or nullptr
    float* g_w_ucn;       // [E] or nullptr
    float* g_bias;        // [E] or nullptr
    const float* app;     // UCN hard-decision source (see CNArgs)
    const float* xa;
    const float* w_vn0;
    int32_t qbit;
    float lo, hi;
};

// Sum of one value over the workgroup, added once to *dst (lane 0 of wave 0).  Every thread of
// the block must call it (uniform control flow).
__device__ __forceinline__ void block_atomic_add(float v, float* dst, float* lds) {
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    const int tid = threadIdx.y * blockDim.x + threadIdx.x;
    const int nw = (blockDim.x * blockDim.y + 63) >> 6;
    if ((tid & 63) == 0) lds[tid >> 6] = v;
    __syncthreads();
    if (tid == 0) {
        float s = 0.f;
        for (int w = 0; w < nw; ++w) s += lds[w];
        if (s != 0.f) atomicAdd(dst, s);
    }
    __syncthreads();
}

template <int DV, int KIND>
__global__ __launch_bounds__(512) void vnb_kernel(VNBArgs a) {
    __shared__ float red[8];
    const int Z = a.g.Z, N = a.g.N, E = a.g.E;
    const Geo q = geo(a.B, Z);
    const int v = q.ok ? q.v : 0, j = q.node;
    const int64_t b = q.ok ? q.b : 0;
    const int64_t idx = (b * N + j) * Z + v;
    const int beg = a.g.col_ptr[j];
    const int d = a.g.col_ptr[j + 1] - beg;
    const int64_t base = b * E;

    float gsum = 0.f;  // sum over the column of dL/dv2c_k = dL/dxin_k (direct part)
    if (q.ok) {
        float g[DV];
        int eidx[DV];
#pragma unroll
        for (int k = 0; k < DV; ++k) {
            eidx[k] = k < d ? a.g.col_edge[beg + k] : 0;
            g[k] = (k < d && a.gv2c) ? a.gv2c[(base + eidx[k]) * Z + v] : 0.f;
        }
        if (a.gc2v) {
            float gyv = 0.f;
            if (a.gy) {
                gyv = a.gy[idx];
                if (a.ymask) gyv = a.ymask[idx] ? gyv : 0.f;
            }
            // others-sum via prefix / suffix
            float suf[DV + 1];
            suf[DV] = 0.f;
#pragma unroll
            for (int k = DV - 1; k >= 0; --k) suf[k] = (k < d) ? suf[k + 1] + g[k] : 0.f;
            float pre = 0.f;
#pragma unroll
            for (int k = 0; k < DV; ++k) {
                if (k < d) {
                    a.gc2v[(base + eidx[k]) * Z + v] = gyv + (pre + suf[k + 1]);
                    pre += g[k];
                }
            }
        }
#pragma unroll
        for (int k = 0; k < DV; ++k)
            if (k < d) gsum += g[k];
    }

    if (a.g_w_vn) {  // block-uniform branch
        float contrib = 0.f;
        if (q.ok) {
            // recompute xin_{p-1} and u_p = xin_{p-1} * w_p
            const float xav = a.xa[idx];
            float xprev = xav;
            for (int s = 0; s < a.step; ++s) {
                xprev = fmul(xprev, a.w_vn[(int64_t)s * N + j]);
                if (KIND == NLDPC_QMS) xprev = quantize(xprev, a.qbit);
            }
            const float wp = a.w_vn[(int64_t)a.step * N + j];
            const float u = fmul(xprev, wp);
            float mask = 1.f;
            if (KIND == NLDPC_QMS) {
                const QRange r = q_range(a.qbit);
                if (r.active) mask = in_range(u, r.lo, r.hi);
            }
            const float dxin = gsum + a.carry[idx];
            const float du = dxin * mask;
            contrib = du * xprev;
            a.carry[idx] = du * wp;
        }
        block_atomic_add(contrib, a.g_w_vn + (int64_t)a.step * N + j, red);
    }
}

template <int DC, int KIND, bool UCN>
__global__ __launch_bounds__(512) void cnb_kernel(CNBArgs a) {
    __shared__ float red[8];
    const int Z = a.g.Z, E = a.g.E;
    const Geo q = geo(a.B, Z);
    const int h = q.ok ? q.v : 0, i = q.node;
    const int64_t b = q.ok ? q.b : 0;
    const int beg = a.g.row_ptr[i];
    const int d = a.g.row_ptr[i + 1] - beg;
    const int64_t base = b * E;

    int vv[DC];
    float m[DC], gc[DC];
#pragma unroll
    for (int k = 0; k < DC; ++k) {
        if (k < d && q.ok) {
            const int t = h + a.g.e_shift[beg + k];
            vv[k] = t >= Z ? t - Z : t;
            const int64_t off = (base + beg + k) * Z + vv[k];
            m[k] = a.v2c[off];
            gc[k] = a.gc2v[off];
        } else {
            vv[k] = 0;
            m[k] = 0.f;
            gc[k] = 0.f;
        }
    }
    const float u = (UCN && q.ok) ? ucn_flag<DC, KIND>(a.g, beg, d, vv, b, a.app, a.xa, a.w_vn0, a.qbit) : 0.f;
    CnCore<DC> core;
    cn_core<DC, KIND>(m, d, a.qbit, a.lo, a.hi, core);

    const QRange qr = q_range(a.qbit);
    float gout[DC];  // dL/dx_output_0 per edge
    float gw[DC], gu[DC], gb[DC];
#pragma unroll
    for (int k = 0; k < DC; ++k) {
        gw[k] = gu[k] = gb[k] = 0.f;
        gout[k] = 0.f;
        if (k < d) {
            const int e = beg + k;
            const float x = core.out0[k];
            const float wc = a.w_cn ? a.w_cn[e] : 1.f;
            const float wu = a.w_ucn ? a.w_ucn[e] : 0.f;
            const CnEpi r = cn_epilogue<KIND, UCN>(x, wc, wu, a.bias ? a.bias[e] : 0.f, u, a.w_cn != nullptr,
                                                   a.w_ucn != nullptr, a.qbit, a.lo, a.hi);
            const float s = signf_t(x), ax = fabsf(x);
            float gabs;
            if (KIND == NLDPC_NEURAL) {
                const float ga = (gc[k] * s) * (r.x1 > 0.f ? 1.f : 0.f);
                gw[k] = ga * ax;
                gb[k] = ga;
                gabs = ga * wc;
            } else {
                float g2 = gc[k] * s;
                if (KIND == NLDPC_QMS) {
                    if (qr.active) g2 *= in_range(r.x2, qr.lo, qr.hi);
                } else {
                    g2 *= in_range(r.x2, a.lo, a.hi);
                }
                const float g1 = g2 * (r.x1 > 0.f ? 1.f : 0.f);
                if (!a.w_cn) {
                    gabs = g1;
                } else if (UCN && a.w_ucn) {
                    const float g11 = g1 * (1.f - u), g12 = g1 * u;
                    gw[k] = g11 * ax;
                    gu[k] = g12 * ax;
                    gabs = g11 * wc + g12 * wu;
                } else {
                    gw[k] = g1 * ax;
                    gabs = g1 * wc;
                }
            }
            gout[k] = gabs * s;
        }
    }

    float gm[DC];
    if (KIND == NLDPC_SP) {
        float graw[DC];
#pragma unroll
        for (int l = 0; l < DC; ++l) graw[l] = 0.f;
#pragma unroll
        for (int k = 0; k < DC; ++k) {
            if (k < d) {
                float P = 1.f;
#pragma unroll
                for (int l = 0; l < DC; ++l)
                    if (l < d && l != k) P = fmul(P, core.mq[l]);
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
                const float xc = clampf(m[l], a.lo, a.hi);
                const float t = tanhf(fmul(-0.5f, xc));
                gm[l] = graw[l] * (1.f - t * t) * -0.5f * in_range(m[l], a.lo, a.hi);
            } else {
                gm[l] = 0.f;
            }
        }
    } else {
        float gq[DC];
#pragma unroll
        for (int l = 0; l < DC; ++l) gq[l] = 0.f;
#pragma unroll
        for (int k = 0; k < DC; ++k) {
            if (k < d) {
                const int tgt = (k == core.idx1) ? core.idx2 : core.idx1;
                const float gmag = gout[k] * core.sg[k];
#pragma unroll
                for (int l = 0; l < DC; ++l)
                    if (l == tgt) gq[l] += gmag * signf_t(core.mq[l]);
            }
        }
#pragma unroll
        for (int l = 0; l < DC; ++l) {
            float msk = 1.f;
            if (KIND == NLDPC_QMS && qr.active) msk = in_range(m[l], qr.lo, qr.hi);
            if (KIND == NLDPC_MS) msk = in_range(m[l], a.lo, a.hi);
            gm[l] = gq[l] * msk;
        }
    }
    if (q.ok) {
#pragma unroll
        for (int k = 0; k < DC; ++k)
            if (k < d) a.gv2c[(base + beg + k) * Z + vv[k]] = gm[k];
    }
    // per-edge weight gradients: one block reduction per edge of the row
#pragma unroll
    for (int k = 0; k < DC; ++k) {
        if (k < d) {
            if (a.g_w_cn) block_atomic_add(gw[k], a.g_w_cn + beg + k, red);
            if (UCN && a.g_w_ucn) block_atomic_add(gu[k], a.g_w_ucn + beg + k, red);
            if (KIND == NLDPC_NEURAL && a.g_bias) block_atomic_add(gb[k], a.g_bias + beg + k, red);
        }
    }
}

template <int DV, int KIND>
static hipError_t launch_vnb(const VNBArgs& a, hipStream_t s) {
    dim3 grid, block;
    node_geometry(a.B, a.g.Z, a.g.N, grid, block);
    prof_start(PROF_VNB, s);
    hipLaunchKernelGGL((vnb_kernel<DV, KIND>), grid, block, 0, s, a);
    prof_stop(s);
    return hipGetLastError();
}

template <int KIND>
static hipError_t vnb_dispatch(const VNBArgs& a, hipStream_t s) {
    switch (deg_bucket(a.g.max_dv)) {
        case 8: return launch_vnb<8, KIND>(a, s);
        case 16: return launch_vnb<16, KIND>(a, s);
        case 32: return launch_vnb<32, KIND>(a, s);
        default: return launch_vnb<64, KIND>(a, s);
    }
}

static hipError_t vnb_launch(int kind, const VNBArgs& a, hipStream_t s) {
    switch (kind) {
        case NLDPC_NEURAL: return vnb_dispatch<NLDPC_NEURAL>(a, s);
        case NLDPC_SP: return vnb_dispatch<NLDPC_SP>(a, s);
        case NLDPC_MS: return vnb_dispatch<NLDPC_MS>(a, s);
        default: return vnb_dispatch<NLDPC_QMS>(a, s);
    }
}

template <int DC, int KIND, bool UCN>
static hipError_t launch_cnb(const CNBArgs& a, hipStream_t s) {
    dim3 grid, block;
    node_geometry(a.B, a.g.Z, a.g.M, grid, block);
    prof_start(PROF_CNB, s);
    hipLaunchKernelGGL((cnb_kernel<DC, KIND, UCN>), grid, block, 0, s, a);
    prof_stop(s);
    return hipGetLastError();
}

template <int KIND, bool UCN>
static hipError_t cnb_dispatch2(const CNBArgs& a, hipStream_t s) {
    switch (deg_bucket(a.g.max_dc)) {
        case 8: return launch_cnb<8, KIND, UCN>(a, s);
        case 16: return launch_cnb<16, KIND, UCN>(a, s);
        case 32: return launch_cnb<32, KIND, UCN>(a, s);
        default: return hipErrorInvalidValue;
    }
}

static hipError_t cnb_launch(int kind, bool ucn, const CNBArgs& a, hipStream_t s) {
    switch (kind) {
        case NLDPC_NEURAL: return cnb_dispatch2<NLDPC_NEURAL, false>(a, s);
        case NLDPC_SP: return ucn ? cnb_dispatch2<NLDPC_SP, true>(a, s) : cnb_dispatch2<NLDPC_SP, false>(a, s);
        case NLDPC_MS: return ucn ? cnb_dispatch2<NLDPC_MS, true>(a, s) : cnb_dispatch2<NLDPC_MS, false>(a, s);
        default: return ucn ? cnb_dispatch2<NLDPC_QMS, true>(a, s) : cnb_dispatch2<NLDPC_QMS, false>(a, s);
    }
}

struct WorkLayout {
    size_t gc_off, gv_off, carry_off, total;
};

static WorkLayout work_layout(const nldpc_graph* g, const nldpc_cfg* cfg, int64_t B) {
    WorkLayout w;
    const size_t ez = (size_t)B * g->dev.E * g->dev.Z * sizeof(float);
    const size_t nz = (size_t)B * g->dev.N * g->dev.Z * sizeof(float);
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    w.gc_off = 0;
    w.gv_off = al(ez);
    w.carry_off = w.gv_off + al(ez);
    w.total = w.carry_off + (cfg->vn_cumulative ? al(nz) : 0);
    return w;
}

}  // namespace nldpc

using namespace nldpc;

extern "C" int nldpc_backward_workspace(const nldpc_graph* g, const nldpc_cfg* cfg, int64_t B, int32_t T,
                                        size_t* bytes) {
    int st = validate_cfg(g, cfg, B, T);
    if (st) return st;
    if (!bytes) return fail(NLDPC_EINVAL, "nldpc_backward_workspace: null output");
    *bytes = work_layout(g, cfg, B).total;
    return NLDPC_OK;
}

extern "C" int nldpc_backward(const nldpc_graph* g, const nldpc_cfg* cfg, int64_t B, int32_t T, const float* xa,
                              const float* w_cn, const float* w_ucn, const float* bias, const float* w_vn,
                              const float* const* outs, const float* const* grad_outs, const float* app_prev,
                              const void* saved, float* g_w_cn, float* g_w_ucn, float* g_bias, float* g_w_vn,
                              void* work, size_t work_bytes, void* stream) {
    int st = validate_cfg(g, cfg, B, T);
    if (st) return st;
    if (!xa || !outs || !grad_outs || !saved || !work) return fail(NLDPC_EINVAL, "nldpc_backward: null argument");
    const WorkLayout WL = work_layout(g, cfg, B);
    if (work_bytes < WL.total) return fail(NLDPC_EINVAL, "nldpc_backward: workspace too small");
    if (cfg->ucn && cfg->first_iter > 0 && !app_prev) return fail(NLDPC_EINVAL, "nldpc_backward: UCN needs app_prev");
    if (cfg->ucn)
        for (int k = 0; k + 1 < T; ++k)
            if (!outs[k]) return fail(NLDPC_EINVAL, "nldpc_backward: UCN needs the forward outputs");
    if (g_w_vn && (!cfg->vn_cumulative || !w_vn)) return fail(NLDPC_EINVAL, "nldpc_backward: g_w_vn needs w_vn");
    DeviceGuard guard(g->device);
    hipStream_t s = static_cast<hipStream_t>(stream);
    const DevGraph& G = g->dev;
    const SavedLayout SL = saved_layout(g, cfg, B, T);
    const float* sv2c = reinterpret_cast<const float*>(static_cast<const char*>(saved) + SL.v2c_off);
    const uint8_t* smask = SL.has_ymask ? static_cast<const uint8_t*>(saved) + SL.ymask_off : nullptr;
    char* wb = static_cast<char*>(work);
    float* gc = reinterpret_cast<float*>(wb + WL.gc_off);
    float* gv = reinterpret_cast<float*>(wb + WL.gv_off);
    float* carry = cfg->vn_cumulative ? reinterpret_cast<float*>(wb + WL.carry_off) : nullptr;
    const bool vn_grad = g_w_vn != nullptr;
    if (vn_grad) NLDPC_HIP_CHECK(hipMemsetAsync(carry, 0, (size_t)B * G.N * G.Z * sizeof(float), s));
    const int P0 = cfg->vn_prefix;

    // dL/dc2v_T from the last output only
    {
        VNBArgs va{G, B, nullptr, grad_outs[T - 1],
                   smask ? smask + (int64_t)(T - 1) * SL.ymask_stride : nullptr, gc, xa, w_vn, nullptr, carry, 0,
                   cfg->qbit};
        hipError_t e = vnb_launch(cfg->kind, va, s);
        if (e != hipSuccess) return hip_fail(e, "vnb_kernel launch");
    }
    for (int k = T - 1; k >= 0; --k) {
        const float* app = nullptr;
        if (cfg->ucn) app = k >= 1 ? outs[k - 1] : (cfg->first_iter > 0 ? app_prev : nullptr);
        CNBArgs ca{G,
                   B,
                   sv2c + (int64_t)k * SL.v2c_stride,
                   gc,
                   gv,
                   w_cn ? w_cn + (int64_t)k * G.E : nullptr,
                   (cfg->ucn && w_ucn) ? w_ucn + (int64_t)k * G.E : nullptr,
                   bias ? bias + (int64_t)k * G.E : nullptr,
                   (g_w_cn && w_cn) ? g_w_cn + (int64_t)k * G.E : nullptr,
                   (g_w_ucn && cfg->ucn && w_ucn) ? g_w_ucn + (int64_t)k * G.E : nullptr,
                   (g_bias && bias) ? g_bias + (int64_t)k * G.E : nullptr,
                   app,
                   xa,
                   cfg->vn_cumulative ? w_vn : nullptr,
                   cfg->qbit,
                   cfg->llr_lo,
                   cfg->llr_hi};
        hipError_t e = cnb_launch(cfg->kind, cfg->ucn != 0, ca, s);
        if (e != hipSuccess) return hip_fail(e, "cnb_kernel launch");
        if (k == 0 && !vn_grad) break;
        VNBArgs va{G,
                   B,
                   gv,
                   k >= 1 ? grad_outs[k - 1] : nullptr,
                   (k >= 1 && smask) ? smask + (int64_t)(k - 1) * SL.ymask_stride : nullptr,
                   k >= 1 ? gc : nullptr,
                   xa,
                   w_vn,
                   vn_grad ? g_w_vn : nullptr,
                   carry,
                   P0 + k,
                   cfg->qbit};
        e = vnb_launch(cfg->kind, va, s);
        if (e != hipSuccess) return hip_fail(e, "vnb_kernel launch");
    }
    // VN-weight chain through the steps applied before this call's first iteration
    for (int p = P0 - 1; vn_grad && p >= 0; --p) {
        VNBArgs va{G, B, nullptr, nullptr, nullptr, nullptr, xa, w_vn, g_w_vn, carry, p, cfg->qbit};
        hipError_t e = vnb_launch(cfg->kind, va, s);
        if (e != hipSuccess) return hip_fail(e, "vnb_kernel launch");
    }
    return NLDPC_OK;
}
