// Backward through the unrolled decoder (config 5: training the learned weights; the reference
// gets these gradients from autograd over BoostedNeuralLDPCDecoder.py:320-526 and
// NeuralLDPCDecoder.py:54-98).
//
// Per iteration k, from the last to the first:
//   CNB(k)  one thread per check copy: recompute the check node from the saved v2c_k (gathered at
//           the cyclic shift), take dL/dc2v_{k+1} at the same addresses, and push it back through
//           sign, clip/quantise (straight-through, closed interval), ReLU mask, learned weights
//           (per-edge weight gradients: per-workgroup partial sums, reduced at the end), |.|, and
//           the min (routed to the first-index argmin of the others, as torch.min's backward) or
//           the sum-product chain (tanh / product / atanh); writes dL/dv2c_k in place of v2c_k's
//           addresses.
//   VNB(k)  one thread per variable copy: dL/dc2v_k[e] = dL/dy_{k-1} (output clamp mask) +
//           sum of dL/dv2c_k over the column's other edges; and the cumulative VN-weight chain
//           xin_k = Q(xin_{k-1} * w_k) (straight-through masks, per-column weight gradients).
// Weight gradients are summed over the batch without atomics: every workgroup writes its partial sum
// per edge (column) and iteration into the workspace, and one reduction kernel at the end adds them
// up in a fixed order (deterministic; thousands of same-address float atomics on a handful of cache
// lines serialised in L2 and bounded both backward kernels before).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "nldpc_fused.h"

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
    float* p_vn;           // [nb][N] per-workgroup partials of dL/dw_vn[step], or nullptr
    float* carry;          // [B][N][Z] dL/du_{p+1} * w_{p+1}
    const float* xin_prev; // [B][N][Z] saved xin_{p-1} (the forward's value), or nullptr: recompute
    int32_t step;          // absolute VN step p of this iteration
    int32_t qbit;
};

struct CNBArgs {
    DevGraph g;
    int64_t B;
    const float* v2c;     // saved v2c_k (fp32), or nullptr when v2c_code is given
    const int8_t* v2c_code;  // saved v2c_k as QMS int8 codes (qms_code), or nullptr
    const float* gc2v;    // dL/dc2v_{k+1}
    float* gv2c;          // dL/dv2c_k out
    const float* w_cn;    // [E] or nullptr
    const float* w_ucn;   // [E] or nullptr
    const float* bias;    // [E] or nullptr
    float* p_cn;          // [nb][E] per-workgroup partials of dL/dw_cn (this iteration), or nullptr
    float* p_ucn;         // [nb][E] dL/dw_ucn partials, or nullptr
    float* p_bias;        // [nb][E] dL/dbias partials, or nullptr
    const float* app;     // UCN hard-decision source (see CNArgs)
    const float* xa;
    const float* w_vn0;
    int32_t qbit;
    float lo, hi;
};

__device__ __forceinline__ int block_slot() { return blockIdx.x * gridDim.z + blockIdx.z; }

// Sum of one value over the workgroup, stored by thread 0 into dst[block_slot() * width].  Every
// thread of the block calls it (uniform control flow).
__device__ __forceinline__ void block_partial(float v, float* dst, int width, float* lds) {
    v = wave_sum(v);  // DPP reduction (nldpc_fused.h)
    const int tid = threadIdx.y * blockDim.x + threadIdx.x;
    const int nw = (blockDim.x * blockDim.y + 63) >> 6;
    if ((tid & 63) == 0) lds[tid >> 6] = v;
    __syncthreads();
    if (tid == 0) {
        float s = 0.f;
        for (int w = 0; w < nw; ++w) s += lds[w];
        dst[(int64_t)block_slot() * width] = s;
    }
}

// Per-edge sums of up to NA gradient arrays over the workgroup: a wave reduction per edge, the
// wave partials in LDS, ONE barrier, then one store per (array, edge) into dst[a][block_slot()][e].
// Every thread of the block calls it (uniform control flow); d is block-uniform.
constexpr int kMaxWaves = 8;
template <int DC, int NA>
__device__ __forceinline__ void block_edge_partials(float (&v)[NA][DC], int d, float* const (&dst)[NA], int E,
                                                    float* lds /* [kMaxWaves][NA][DC] */) {
    const int tid = threadIdx.y * blockDim.x + threadIdx.x;
    const int wv = tid >> 6, nw = (blockDim.x * blockDim.y + 63) >> 6;
#pragma unroll
    for (int a = 0; a < NA; ++a) {
        if (!dst[a]) continue;
#pragma unroll
        for (int k = 0; k < DC; ++k) {
            if (k < d) {
                const float x = wave_sum(v[a][k]);
                if ((tid & 63) == 0) lds[(wv * NA + a) * DC + k] = x;
            }
        }
    }
    __syncthreads();
    if (tid < NA * DC) {
        const int a = tid / DC, k = tid - a * DC;
        if (k < d && dst[a]) {
            float s = 0.f;
            for (int w = 0; w < nw; ++w) s += lds[(w * NA + a) * DC + k];
            dst[a][(int64_t)block_slot() * E + k] = s;
        }
    }
}

// y += x (n floats)
__global__ void add_kernel(float* __restrict__ y, const float* __restrict__ x, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        y[i] += x[i];
}
static hipError_t add_launch(float* y, const float* x, int64_t n, hipStream_t s) {
    const int64_t b = (n + 255) / 256;
    hipLaunchKernelGGL(add_kernel, dim3((unsigned)(b < 16384 ? b : 16384)), dim3(256), 0, s, y, x, n);
    return hipGetLastError();
}

// The weight gradients from their partials, in a fixed order (deterministic), two levels so that
// thousands of partials per weight are summed by many workgroups:
// level 1: part[r][k*CH][c] = sum over b in [k*CH, k*CH + CH) of part[r][b][c], ascending b (in place:
//          each chunk's sum replaces its own first row, which only that thread reads)
// level 2: out[r][c] += sum over k of part[r][k*CH][c], ascending k
constexpr int kReduceChunk = 64;
__global__ void reduce_chunks(float* __restrict__ part, int64_t nb, int64_t width) {
    const int64_t r = blockIdx.y, k = blockIdx.x;
    float* p = part + (r * nb + k * kReduceChunk) * width;
    const int64_t nrow = nb - k * kReduceChunk < kReduceChunk ? nb - k * kReduceChunk : kReduceChunk;
    for (int64_t c = threadIdx.x; c < width; c += blockDim.x) {
        float s = 0.f;
        for (int64_t b = 0; b < nrow; ++b) s += p[b * width + c];
        p[c] = s;
    }
}
__global__ void reduce_partials(const float* __restrict__ part, int64_t rows, int64_t nb, int64_t width,
                                float* __restrict__ out) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= rows * width) return;
    const int64_t r = t / width, c = t - r * width;
    const float* p = part + r * nb * width + c;
    float s = 0.f;
    for (int64_t b = 0; b < nb; b += kReduceChunk) s += p[b * width];
    out[t] += s;
}

template <int DV, int KIND>
__device__ __forceinline__ void vnb_body(const VNBArgs& a, const Geo& q, const int beg, const int d, float* red) {
    const int Z = a.g.Z, N = a.g.N, E = a.g.E;
    const int v = q.ok ? q.v : 0, j = q.node;
    const int64_t b = q.ok ? q.b : 0;
    const int64_t idx = (b * N + j) * Z + v;
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

    if (a.p_vn) {  // block-uniform branch
        float contrib = 0.f;
        if (q.ok) {
            // recompute xin_{p-1} and u_p = xin_{p-1} * w_p
            float xprev;
            if (a.xin_prev) {
                xprev = a.xin_prev[idx];
            } else {
                xprev = a.xa[idx];
                for (int s = 0; s < a.step; ++s) {
                    xprev = fmul(xprev, a.w_vn[(int64_t)s * N + j]);
                    if (KIND == NLDPC_QMS) xprev = quantize(xprev, a.qbit);
                }
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
        block_partial(contrib, a.p_vn + j, N, red);
    }
}

template <int DC, int KIND, bool UCN>
__device__ __forceinline__ void cnb_body(const CNBArgs& a, const Geo& q, const int beg, const int d, float* red) {
    const int Z = a.g.Z, E = a.g.E;
    const int h = q.ok ? q.v : 0;
    const int64_t b = q.ok ? q.b : 0;
    const int64_t base = b * E;

    int vv[DC];
    float m[DC], gc[DC];
#pragma unroll
    for (int k = 0; k < DC; ++k) {
        if (k < d && q.ok) {
            const int t = h + a.g.e_shift[beg + k];
            vv[k] = t >= Z ? t - Z : t;
            const int64_t off = (base + beg + k) * Z + vv[k];
            const int64_t offh = (base + beg + k) * Z + h;  // saved v2c: check order
            m[k] = a.v2c_code ? qms_decode(a.v2c_code[offh]) : a.v2c[offh];
            gc[k] = a.gc2v[off];
        } else {
            vv[k] = 0;
            m[k] = 0.f;
            gc[k] = 0.f;
        }
    }
    const float u = (UCN && q.ok) ? ucn_flag<DC, KIND>(a.g, beg, d, vv, b, a.app, a.xa, a.w_vn0, a.qbit) : 0.f;
    float wc[DC], wu[DC], bb[DC], gm[DC], gw[DC], gu[DC], gb[DC];
#pragma unroll
    for (int k = 0; k < DC; ++k) {
        wc[k] = (k < d && a.w_cn) ? a.w_cn[beg + k] : 1.f;
        wu[k] = (k < d && a.w_ucn) ? a.w_ucn[beg + k] : 0.f;
        bb[k] = (k < d && a.bias) ? a.bias[beg + k] : 0.f;
    }
    cn_backward<DC, KIND, UCN>(m, gc, d, u, wc, wu, bb, a.w_cn != nullptr, a.w_ucn != nullptr, a.qbit, a.lo, a.hi, gm,
                               gw, gu, gb, SpRow{a.g.sp_plan + q.node * kSpPlanBytes, a.g.tanh});
    if (q.ok) {
#pragma unroll
        for (int k = 0; k < DC; ++k)
            if (k < d) a.gv2c[(base + beg + k) * Z + vv[k]] = gm[k];
    }
    // per-edge weight gradients: wave reductions, one barrier, one partial per edge and block
    float gacc[3][DC];
#pragma unroll
    for (int k = 0; k < DC; ++k) {
        gacc[0][k] = gw[k];
        gacc[1][k] = gu[k];
        gacc[2][k] = gb[k];
    }
    float* const dst[3] = {a.p_cn ? a.p_cn + beg : nullptr, (UCN && a.p_ucn) ? a.p_ucn + beg : nullptr,
                           (KIND == NLDPC_NEURAL && a.p_bias) ? a.p_bias + beg : nullptr};
    block_edge_partials<DC, 3>(gacc, d, dst, E, red);
}

// Kernels: one switch on the workgroup-uniform degree, then a body with a compile-time degree
// (deg_switch, nldpc_node.h).  The bodies hold barriers: every thread of a block takes the same case.
template <int KIND, int MAXD>
__global__ __launch_bounds__(512) void vnb_kernel(VNBArgs a) {
    __shared__ float red[kMaxWaves];
    const Geo q = geo(a.B, a.g.Z);
    const int beg = a.g.col_ptr[q.node];
    deg_switch<MAXD>(a.g.col_ptr[q.node + 1] - beg,
                     [&](auto D, int d) { vnb_body<decltype(D)::value, KIND>(a, q, beg, d, red); });
}

template <int KIND, bool UCN, int MAXD>
__global__ __launch_bounds__(512) void cnb_kernel(CNBArgs a) {
    __shared__ float red[kMaxWaves * 3 * MAXD];
    const Geo q = geo(a.B, a.g.Z);
    const int beg = a.g.row_ptr[q.node];
    deg_switch<MAXD>(a.g.row_ptr[q.node + 1] - beg,
                     [&](auto D, int d) { cnb_body<decltype(D)::value, KIND, UCN>(a, q, beg, d, red); });
}

template <int KIND>
static hipError_t launch_vnb(const VNBArgs& a, hipStream_t s) {
    dim3 grid, block;
    node_geometry(a.B, a.g.Z, a.g.N, grid, block);
    prof_start(PROF_VNB, s);
    switch (deg_max_bucket(a.g.max_dv)) {
        case 12: hipLaunchKernelGGL((vnb_kernel<KIND, 12>), grid, block, 0, s, a); break;
        case 16: hipLaunchKernelGGL((vnb_kernel<KIND, 16>), grid, block, 0, s, a); break;
        case 24: hipLaunchKernelGGL((vnb_kernel<KIND, 24>), grid, block, 0, s, a); break;
        case 32: hipLaunchKernelGGL((vnb_kernel<KIND, 32>), grid, block, 0, s, a); break;
        default: hipLaunchKernelGGL((vnb_kernel<KIND, 64>), grid, block, 0, s, a); break;
    }
    prof_stop(s);
    return hipGetLastError();
}

static hipError_t vnb_launch(int kind, const VNBArgs& a, hipStream_t s) {
    switch (kind) {
        case NLDPC_NEURAL: return launch_vnb<NLDPC_NEURAL>(a, s);
        case NLDPC_SP: return launch_vnb<NLDPC_SP>(a, s);
        case NLDPC_MS: return launch_vnb<NLDPC_MS>(a, s);
        default: return launch_vnb<NLDPC_QMS>(a, s);
    }
}

template <int KIND, bool UCN>
static hipError_t launch_cnb(const CNBArgs& a, hipStream_t s) {
    dim3 grid, block;
    node_geometry(a.B, a.g.Z, a.g.M, grid, block);
    prof_start(PROF_CNB, s);
    // SP's check node (DC^2 ordered products per copy) is instantiated for two degree buckets only
    const int bucket = deg_max_bucket(a.g.max_dc);
    if constexpr (KIND == NLDPC_SP) {
        if (bucket <= 16) hipLaunchKernelGGL((cnb_kernel<KIND, UCN, 16>), grid, block, 0, s, a);
        else hipLaunchKernelGGL((cnb_kernel<KIND, UCN, 32>), grid, block, 0, s, a);
    } else {
        switch (bucket) {
            case 12: hipLaunchKernelGGL((cnb_kernel<KIND, UCN, 12>), grid, block, 0, s, a); break;
            case 16: hipLaunchKernelGGL((cnb_kernel<KIND, UCN, 16>), grid, block, 0, s, a); break;
            case 24: hipLaunchKernelGGL((cnb_kernel<KIND, UCN, 24>), grid, block, 0, s, a); break;
            default: hipLaunchKernelGGL((cnb_kernel<KIND, UCN, 32>), grid, block, 0, s, a); break;
        }
    }
    prof_stop(s);
    return hipGetLastError();
}

static hipError_t cnb_launch(int kind, bool ucn, const CNBArgs& a, hipStream_t s) {
    switch (kind) {
        case NLDPC_NEURAL: return launch_cnb<NLDPC_NEURAL, false>(a, s);
        case NLDPC_SP: return ucn ? launch_cnb<NLDPC_SP, true>(a, s) : launch_cnb<NLDPC_SP, false>(a, s);
        case NLDPC_MS: return ucn ? launch_cnb<NLDPC_MS, true>(a, s) : launch_cnb<NLDPC_MS, false>(a, s);
        default: return ucn ? launch_cnb<NLDPC_QMS, true>(a, s) : launch_cnb<NLDPC_QMS, false>(a, s);
    }
}

struct WorkLayout {
    size_t gc_off, gv_off, carry_off, pcn_off, pvn_off, total;
    int64_t nb;  // workgroup slots along the batch (block_slot() range) of the node kernels
};

// pcn: [3][T][nb][E] per-workgroup partials of dL/d(w_cn, w_ucn, bias); pvn: [vn_prefix+T][nb][N]
static WorkLayout work_layout(const nldpc_graph* g, const nldpc_cfg* cfg, int64_t B, int32_t T) {
    WorkLayout w;
    const size_t ez = (size_t)B * g->dev.E * g->dev.Z * sizeof(float);
    const size_t nz = (size_t)B * g->dev.N * g->dev.Z * sizeof(float);
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    dim3 grid, block;
    node_geometry(B, g->dev.Z, 1, grid, block);
    w.nb = (int64_t)grid.x * grid.z;
    w.gc_off = 0;
    w.gv_off = al(ez);
    w.carry_off = w.gv_off + al(ez);
    w.pcn_off = w.carry_off + (cfg->vn_cumulative ? al(nz) : 0);
    w.pvn_off = w.pcn_off + al((size_t)3 * T * w.nb * g->dev.E * sizeof(float));
    w.total = w.pvn_off + (cfg->vn_cumulative ? al((size_t)(cfg->vn_prefix + T) * w.nb * g->dev.N * sizeof(float)) : 0);
    return w;
}

static hipError_t reduce_launch(float* part, int64_t rows, int64_t nb, int64_t width, float* out, hipStream_t s) {
    const int64_t n = rows * width;
    if (n == 0) return hipSuccess;
    const int64_t nk = (nb + kReduceChunk - 1) / kReduceChunk;
    hipLaunchKernelGGL(reduce_chunks, dim3((unsigned)nk, (unsigned)rows), dim3(256), 0, s, part, nb, width);
    hipLaunchKernelGGL(reduce_partials, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, part, rows, nb, width, out);
    return hipGetLastError();
}

// ---- fused backward (register-resident kernels generated by gen_fused.py emit_bwd) ---------------
static bool fused_bwd_eligible(const nldpc_graph* g, const nldpc_cfg* cfg, int32_t T, bool state_grads) {
    static const bool disabled = std::getenv("NLDPC_DISABLE_FUSED") != nullptr;
    if (disabled || state_grads || (cfg->flags & NLDPC_FLAG_STREAM) || !fused_launch(g, 4, cfg->kind)) return false;
    if (cfg->kind == NLDPC_QMS && !qms_active(cfg->qbit)) return false;  // QMS saved state = int8 codes
    return !cfg->ucn && cfg->vn_prefix == 0 && T <= kFusedMaxT;
}

struct FusedWork {
    size_t carry_off, pcn_off, pbias_off, pvn_off, total;
    int64_t nslots;  // partial-sum slots per iteration: workgroups x waves per part
};

static FusedWork fused_work_layout(const nldpc_graph* g, const nldpc_cfg* cfg, int64_t B, int32_t T) {
    const FusedLaunch f = fused_launch(g, 4, cfg->kind);
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    FusedWork w;
    w.nslots = (B + f.G - 1) / f.G * f.waves_per_part;
    const size_t pe = (size_t)T * w.nslots * g->dev.E * sizeof(float);
    w.carry_off = 0;
    w.pcn_off = al(cfg->vn_cumulative ? (size_t)B * g->dev.N * g->dev.Z * sizeof(float) : 0);
    w.pbias_off = w.pcn_off + al(pe);
    w.pvn_off = w.pbias_off + (cfg->kind == NLDPC_NEURAL ? al(pe) : 0);
    w.total = w.pvn_off + (cfg->vn_cumulative ? al((size_t)T * w.nslots * g->dev.N * sizeof(float)) : 0);
    return w;
}

static int fused_backward(const nldpc_graph* g, const nldpc_cfg* cfg, int64_t B, int32_t T, const float* xa,
                          const float* w_cn, const float* bias, const float* w_vn, const float* const* grad_outs,
                          const void* saved, float* g_w_cn, float* g_bias, float* g_w_vn, void* work,
                          hipStream_t s) {
    // a tied CN weight (NLDPC_FLAG_CN_TIED) whose gradient is wanted: the kernel that reduces each row copy's
    // contributions once (MODE 5); its partials put each iteration's totals into a few entries per row.  (A tied
    // VN weight needs no other kernel: its partials are one wave reduction per column either way.)
    const bool tied = cfg->kind != NLDPC_NEURAL && g_w_cn && w_cn && (cfg->flags & NLDPC_FLAG_CN_TIED);
    const FusedLaunch ft = tied ? fused_launch(g, 5, cfg->kind) : FusedLaunch{};
    const FusedLaunch f = ft ? ft : fused_launch(g, 4, cfg->kind);
    const FusedWork W = fused_work_layout(g, cfg, B, T);
    const SavedLayout SL = saved_layout(g, cfg, B, T);
    const DevGraph& G = g->dev;
    const char* sb = static_cast<const char*>(saved);
    char* wb = static_cast<char*>(work);
    FusedBwdArgs a{};
    a.sig = kFusedBwdArgsSig;
    a.B = B;
    a.T = T;
    a.qbit = cfg->qbit;
    a.lo = cfg->llr_lo;
    a.hi = cfg->llr_hi;
    a.xa = xa;
    a.w_cn = w_cn;
    a.bias = bias;
    a.w_vn = (g_w_vn && cfg->vn_cumulative) ? w_vn : nullptr;  // the chain only feeds dL/dw_vn
    a.sp_plan = g->dev.sp_plan;
    a.tanh = g->dev.tanh;
    a.sv2c = sb + SL.v2c_off;
    a.symask = SL.has_ymask ? reinterpret_cast<const uint8_t*>(sb + SL.ymask_off) : nullptr;
    a.sxin = SL.has_xin ? reinterpret_cast<const float*>(sb + SL.xin_off) : nullptr;
    a.sv2c_stride = SL.v2c_stride;
    a.symask_stride = SL.ymask_stride;
    a.sxin_stride = SL.xin_stride;
    a.p_cn = (g_w_cn && w_cn) ? reinterpret_cast<float*>(wb + W.pcn_off) : nullptr;
    a.p_bias = (g_bias && bias && cfg->kind == NLDPC_NEURAL) ? reinterpret_cast<float*>(wb + W.pbias_off) : nullptr;
    a.p_vn = a.w_vn ? reinterpret_cast<float*>(wb + W.pvn_off) : nullptr;
    a.carry = a.w_vn ? reinterpret_cast<float*>(wb + W.carry_off) : nullptr;
    a.nslots = W.nslots;
    a.cn_tied = ft ? 1 : 0;
    a.vn_tied = 0;
    // the tied kernel writes one entry per part and wave slot: the rest of its partials must read 0
    if (ft && a.p_cn) NLDPC_HIP_CHECK(hipMemsetAsync(a.p_cn, 0, (size_t)T * W.nslots * G.E * sizeof(float), s));
    for (int k = 0; k < kFusedMaxT; ++k) a.gy.p[k] = k < T ? const_cast<float*>(grad_outs[k]) : nullptr;
    // diagnostic stamp build (lib_stamps/): NLDPC_STAMPS_BWD=<file> collects the phase stamps of each call
    static const char* stamp_file = std::getenv("NLDPC_STAMPS_BWD");
    const size_t stamp_n = (size_t)256 * (f.threads / 64) * T * 16;
    if (stamp_file) NLDPC_HIP_CHECK(hipMalloc(&a.stamps, stamp_n * sizeof(uint64_t)));
    if (stamp_file) NLDPC_HIP_CHECK(hipMemsetAsync(a.stamps, 0, stamp_n * sizeof(uint64_t), s));
    void* args[] = {&a};
    const int64_t blocks = (B + f.G - 1) / f.G;
    prof_start(PROF_FUSED_BWD, s);
    hipError_t e = f.launch(blocks, args, s);
    prof_stop(s);
    if (e == hipSuccess) e = hipGetLastError();
    if (e != hipSuccess) return hip_fail(e, "fused backward launch");
    if (stamp_file) {
        std::vector<uint64_t> h(stamp_n);
        NLDPC_HIP_CHECK(hipStreamSynchronize(s));
        NLDPC_HIP_CHECK(hipMemcpy(h.data(), a.stamps, stamp_n * sizeof(uint64_t), hipMemcpyDeviceToHost));
        if (FILE* fp = std::fopen(stamp_file, "wb")) {
            const int32_t hdr[4] = {256, f.threads / 64, T, 16};
            std::fwrite(hdr, sizeof(hdr), 1, fp);
            std::fwrite(h.data(), sizeof(uint64_t), stamp_n, fp);
            std::fclose(fp);
        }
        (void)hipFree(a.stamps);
    }
    if (a.p_cn) e = reduce_launch(a.p_cn, T, W.nslots, G.E, g_w_cn, s);
    if (e == hipSuccess && a.p_bias) e = reduce_launch(a.p_bias, T, W.nslots, G.E, g_bias, s);
    if (e == hipSuccess && a.p_vn) e = reduce_launch(a.p_vn, T, W.nslots, G.N, g_w_vn, s);
    if (e != hipSuccess) return hip_fail(e, "reduce_partials launch");
    return NLDPC_OK;
}

}  // namespace nldpc

using namespace nldpc;

extern "C" int nldpc_backward_workspace(const nldpc_graph* g, const nldpc_cfg* cfg, int64_t B, int32_t T,
                                        size_t* bytes) {
    int st = validate_cfg(g, cfg, B, T);
    if (st) return st;
    if (!bytes) return fail(NLDPC_EINVAL, "nldpc_backward_workspace: null output");
    // enough for either path (a call with message-state gradients always streams)
    const size_t streaming = work_layout(g, cfg, B, T).total;
    const size_t fused = fused_bwd_eligible(g, cfg, T, false) ? fused_work_layout(g, cfg, B, T).total : 0;
    *bytes = fused > streaming ? fused : streaming;
    return NLDPC_OK;
}

extern "C" int nldpc_backward(const nldpc_graph* g, const nldpc_cfg* cfg, int64_t B, int32_t T, const float* xa,
                              const float* w_cn, const float* w_ucn, const float* bias, const float* w_vn,
                              const float* const* outs, const float* const* grad_outs, const float* app_prev,
                              const void* saved, const float* grad_c2v_out, float* grad_c2v_in, float* g_w_cn,
                              float* g_w_ucn, float* g_bias, float* g_w_vn, void* work, size_t work_bytes,
                              void* stream) {
    int st = validate_cfg(g, cfg, B, T);
    if (st) return st;
    if (!xa || !outs || !grad_outs || !saved || !work) return fail(NLDPC_EINVAL, "nldpc_backward: null argument");
    // (the fused kernels stage the saved messages by 16-byte LDS-DMA: a 16-byte aligned buffer)
    const bool fusedb = fused_bwd_eligible(g, cfg, T, grad_c2v_out || grad_c2v_in) &&
                        (reinterpret_cast<uintptr_t>(saved) & 15) == 0;
    const WorkLayout WL = work_layout(g, cfg, B, T);
    if (work_bytes < (fusedb ? fused_work_layout(g, cfg, B, T).total : WL.total))
        return fail(NLDPC_EINVAL, "nldpc_backward: workspace too small");
    if (cfg->ucn && cfg->first_iter > 0 && !app_prev) return fail(NLDPC_EINVAL, "nldpc_backward: UCN needs app_prev");
    if (cfg->ucn)
        for (int k = 0; k + 1 < T; ++k)
            if (!outs[k]) return fail(NLDPC_EINVAL, "nldpc_backward: UCN needs the forward outputs");
    if (g_w_vn && (!cfg->vn_cumulative || !w_vn)) return fail(NLDPC_EINVAL, "nldpc_backward: g_w_vn needs w_vn");
    DeviceGuard guard(g->device);
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (fusedb) return fused_backward(g, cfg, B, T, xa, w_cn, bias, w_vn, grad_outs, saved, g_w_cn, g_bias, g_w_vn, work, s);
    const DevGraph& G = g->dev;
    const SavedLayout SL = saved_layout(g, cfg, B, T);
    const char* sv2c = static_cast<const char*>(saved) + SL.v2c_off;  // fp32, or QMS int8 codes
    const uint8_t* smask = SL.has_ymask ? static_cast<const uint8_t*>(saved) + SL.ymask_off : nullptr;
    const float* sxin = SL.has_xin ? reinterpret_cast<const float*>(static_cast<const char*>(saved) + SL.xin_off) : nullptr;
    char* wb = static_cast<char*>(work);
    float* gc = reinterpret_cast<float*>(wb + WL.gc_off);
    float* gv = reinterpret_cast<float*>(wb + WL.gv_off);
    float* carry = cfg->vn_cumulative ? reinterpret_cast<float*>(wb + WL.carry_off) : nullptr;
    const int64_t nbE = WL.nb * G.E, nbN = WL.nb * G.N;
    float* pcn = reinterpret_cast<float*>(wb + WL.pcn_off);  // [3][T][nb][E]
    float* p_cn = (g_w_cn && w_cn) ? pcn : nullptr;
    float* p_ucn = (g_w_ucn && cfg->ucn && w_ucn) ? pcn + (int64_t)T * nbE : nullptr;
    float* p_bias = (g_bias && bias) ? pcn + 2 * (int64_t)T * nbE : nullptr;
    float* p_vn = cfg->vn_cumulative ? reinterpret_cast<float*>(wb + WL.pvn_off) : nullptr;  // [P0+T][nb][N]
    const bool vn_grad = g_w_vn != nullptr;
    if (vn_grad) NLDPC_HIP_CHECK(hipMemsetAsync(carry, 0, (size_t)B * G.N * G.Z * sizeof(float), s));
    const int P0 = cfg->vn_prefix;

    // dL/dc2v_T from the last output only
    {
        VNBArgs va{G, B, nullptr, grad_outs[T - 1],
                   smask ? smask + (int64_t)(T - 1) * SL.ymask_stride : nullptr, gc, xa, w_vn, nullptr, carry, nullptr, 0,
                   cfg->qbit};
        hipError_t e = vnb_launch(cfg->kind, va, s);
        if (e != hipSuccess) return hip_fail(e, "vnb_kernel launch");
        if (grad_c2v_out) {  // + the gradient arriving at the final message state (a later segment's input)
            e = add_launch(gc, grad_c2v_out, B * G.E * G.Z, s);
            if (e != hipSuccess) return hip_fail(e, "add_kernel launch");
        }
    }
    for (int k = T - 1; k >= 0; --k) {
        const float* app = nullptr;
        if (cfg->ucn) app = k >= 1 ? outs[k - 1] : (cfg->first_iter > 0 ? app_prev : nullptr);
        CNBArgs ca{G,
                   B,
                   SL.v2c_code ? nullptr : reinterpret_cast<const float*>(sv2c) + (int64_t)k * SL.v2c_stride,
                   SL.v2c_code ? reinterpret_cast<const int8_t*>(sv2c) + (int64_t)k * SL.v2c_stride : nullptr,
                   gc,
                   gv,
                   w_cn ? w_cn + (int64_t)k * G.E : nullptr,
                   (cfg->ucn && w_ucn) ? w_ucn + (int64_t)k * G.E : nullptr,
                   bias ? bias + (int64_t)k * G.E : nullptr,
                   p_cn ? p_cn + (int64_t)k * nbE : nullptr,
                   p_ucn ? p_ucn + (int64_t)k * nbE : nullptr,
                   p_bias ? p_bias + (int64_t)k * nbE : nullptr,
                   app,
                   xa,
                   cfg->vn_cumulative ? w_vn : nullptr,
                   cfg->qbit,
                   cfg->llr_lo,
                   cfg->llr_hi};
        hipError_t e = cnb_launch(cfg->kind, cfg->ucn != 0, ca, s);
        if (e != hipSuccess) return hip_fail(e, "cnb_kernel launch");
        if (k == 0 && !vn_grad && !grad_c2v_in) break;
        VNBArgs va{G,
                   B,
                   gv,
                   k >= 1 ? grad_outs[k - 1] : nullptr,
                   (k >= 1 && smask) ? smask + (int64_t)(k - 1) * SL.ymask_stride : nullptr,
                   k >= 1 ? gc : grad_c2v_in,  // k = 0: dL/d(the incoming message state)
                   xa,
                   w_vn,
                   vn_grad ? p_vn + (int64_t)(P0 + k) * nbN : nullptr,
                   carry,
                   (sxin && k >= 1) ? sxin + (int64_t)(k - 1) * SL.xin_stride : nullptr,
                   P0 + k,
                   cfg->qbit};
        e = vnb_launch(cfg->kind, va, s);
        if (e != hipSuccess) return hip_fail(e, "vnb_kernel launch");
    }
    // VN-weight chain through the steps applied before this call's first iteration
    for (int p = P0 - 1; vn_grad && p >= 0; --p) {
        VNBArgs va{G, B, nullptr, nullptr, nullptr, nullptr, xa, w_vn, p_vn + (int64_t)p * nbN, carry, nullptr, p,
                   cfg->qbit};
        hipError_t e = vnb_launch(cfg->kind, va, s);
        if (e != hipSuccess) return hip_fail(e, "vnb_kernel launch");
    }
    // the weight gradients: one fixed-order sum over the per-workgroup partials
    hipError_t e = hipSuccess;
    if (p_cn) e = reduce_launch(p_cn, T, WL.nb, G.E, g_w_cn, s);
    if (e == hipSuccess && p_ucn) e = reduce_launch(p_ucn, T, WL.nb, G.E, g_w_ucn, s);
    if (e == hipSuccess && p_bias) e = reduce_launch(p_bias, T, WL.nb, G.E, g_bias, s);
    if (e == hipSuccess && vn_grad) e = reduce_launch(p_vn, P0 + T, WL.nb, G.N, g_w_vn, s);
    if (e != hipSuccess) return hip_fail(e, "reduce_partials launch");
    return NLDPC_OK;
}
