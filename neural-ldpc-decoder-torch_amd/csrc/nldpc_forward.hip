// Forward decode: the flooding belief-propagation iteration of the reference decoders as two
// gather kernels per iteration over the lifted Tanner graph's edge list.
//
//   VN kernel  one thread per variable copy (b, j, v), lanes = consecutive v (coalesced):
//              reads the column's c2v messages, writes every v2c message of the column
//              (sum of the others, sequential fp32 in ascending check row) and, fused, the
//              posterior output of the previous iteration (= the reference's W_output matmul +
//              channel add of that iteration, NeuralLDPCDecoder.py:93-98 / Boosted…py:513-526).
//   CN kernel  one thread per check copy (b, i, h), lanes = consecutive h: gathers the row's v2c
//              at the cyclic shift (h + s_e) mod Z (the reference's lifting_matrix_1 GEMM), does
//              the min-sum / sum-product update + learned weighting (NeuralLDPCDecoder.py:65-91,
//              Boosted…py:386-512) and scatters c2v back to the same addresses (lifting_matrix_2).
// Message state is [B][E][Z] fp32 in HBM with E in C-order; see DESIGN.md for the roofline.
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "nldpc_fused.h"

namespace nldpc {

struct VNArgs {
    DevGraph g;
    int64_t B;
    const float* xa;     // [B][N][Z]
    const float* c2v;    // [B][E][Z] or nullptr (all-zero state)
    float* v2c;          // [B][E][Z] or nullptr (posterior only)
    float* post;         // [B][N][Z] or nullptr
    uint8_t* ymask;      // [B][N][Z] clamp mask of the posterior (training) or nullptr
    const float* w_vn;   // [steps][N] cumulative VN weights (boosted) or nullptr
    int32_t n_vn_steps;  // number of cumulative weighting/quantisation steps for xin
    int32_t qbit;
    float lo, hi;
};

struct CNArgs {
    DevGraph g;
    int64_t B;
    const float* v2c;    // [B][E][Z]
    float* c2v;          // [B][E][Z]
    const float* w_cn;   // [E] (this iteration) or nullptr
    const float* w_ucn;  // [E] or nullptr
    const float* bias;   // [E] or nullptr (Neural)
    // UCN: hard-decision source.  app != nullptr: posterior [B][N][Z] of the previous iteration;
    // else xin_0 recomputed from xa and w_vn0 (absolute iteration 0, Boosted…py:340-341).
    const float* app;
    const float* xa;
    const float* w_vn0;  // [N] or nullptr
    int32_t qbit;
    float lo, hi;
};

template <int DV, int KIND>
__global__ __launch_bounds__(512) void vn_kernel(VNArgs a) {
    const int Z = a.g.Z, N = a.g.N, E = a.g.E;
    const Geo q = geo(a.B, Z);
    if (!q.ok) return;
    const int v = q.v, j = q.node;
    const int64_t b = q.b;
    const int64_t idx = (b * N + j) * Z + v;
    const int beg = a.g.col_ptr[j];
    const int d = a.g.col_ptr[j + 1] - beg;
    const float xav = a.xa[idx];
    const int64_t base = b * E;

    int eidx[DV];
    float c[DV];
#pragma unroll
    for (int k = 0; k < DV; ++k) {
        eidx[k] = k < d ? a.g.col_edge[beg + k] : 0;
        c[k] = (k < d && a.c2v) ? a.c2v[(base + eidx[k]) * Z + v] : 0.f;
    }

    if (a.post) {
        // y = ch_o + ((0 + c0) + c1 + ...)  (W_output sgemm order), Boosted: ch_o = Q(xa), clamp
        float P = 0.f;
#pragma unroll
        for (int k = 0; k < DV; ++k)
            if (k < d) P = fadd(P, c[k]);
        float y;
        if (KIND == NLDPC_NEURAL) {
            y = fadd(xav, P);
        } else {
            const float xo = (KIND == NLDPC_QMS) ? quantize(xav, a.qbit) : xav;
            const float yp = fadd(xo, P);
            y = clampf(yp, a.lo, a.hi);
            if (a.ymask) a.ymask[idx] = (uint8_t)in_range(yp, a.lo, a.hi);
        }
        a.post[idx] = y;
    }

    if (a.v2c) {
        const float ch = vn_channel<KIND>(xav, a.w_vn, N, j, a.n_vn_steps, a.qbit);
        const float x0 = fadd(0.f, ch);  // xa_input @ W_skipconn2even
        float P = 0.f;                   // prefix ((0 + c0) + ... + c_{k-1})
#pragma unroll
        for (int k = 0; k < DV; ++k) {
            if (k < d) {
                float S = P;  // sum of the others, left to right, skipping k
#pragma unroll
                for (int m = k + 1; m < DV; ++m)
                    if (m < d) S = fadd(S, c[m]);
                a.v2c[(base + eidx[k]) * Z + v] = fadd(x0, S);
                P = fadd(P, c[k]);
            }
        }
    }
}

template <int DC, int KIND, bool UCN>
__global__ __launch_bounds__(512) void cn_kernel(CNArgs a) {
    const int Z = a.g.Z, E = a.g.E;
    const Geo q = geo(a.B, Z);
    if (!q.ok) return;
    const int h = q.v, i = q.node;
    const int64_t b = q.b;
    const int beg = a.g.row_ptr[i];
    const int d = a.g.row_ptr[i + 1] - beg;
    const int64_t base = b * E;

    int vv[DC];
    float m[DC];
#pragma unroll
    for (int k = 0; k < DC; ++k) {
        if (k < d) {
            const int t = h + a.g.e_shift[beg + k];
            vv[k] = t >= Z ? t - Z : t;
            m[k] = a.v2c[(base + beg + k) * Z + vv[k]];
        } else {
            vv[k] = 0;
            m[k] = 0.f;
        }
    }
    const float u = UCN ? ucn_flag<DC, KIND>(a.g, beg, d, vv, b, a.app, a.xa, a.w_vn0, a.qbit) : 0.f;
    CnCore<DC> core;
    cn_core<DC, KIND>(m, d, a.qbit, a.lo, a.hi, core);
#pragma unroll
    for (int k = 0; k < DC; ++k) {
        if (k < d) {
            const int e = beg + k;
            const CnEpi r = cn_epilogue<KIND, UCN>(core.out0[k], a.w_cn ? a.w_cn[e] : 1.f,
                                                   a.w_ucn ? a.w_ucn[e] : 0.f, a.bias ? a.bias[e] : 0.f, u,
                                                   a.w_cn != nullptr, a.w_ucn != nullptr, a.qbit, a.lo, a.hi);
            a.c2v[(base + e) * Z + vv[k]] = r.c;
        }
    }
}

template <int DV, int KIND>
static hipError_t launch_vn(const VNArgs& a, hipStream_t s) {
    dim3 grid, block;
    node_geometry(a.B, a.g.Z, a.g.N, grid, block);
    hipLaunchKernelGGL((vn_kernel<DV, KIND>), grid, block, 0, s, a);
    return hipGetLastError();
}

template <int DC, int KIND, bool UCN>
static hipError_t launch_cn(const CNArgs& a, hipStream_t s) {
    dim3 grid, block;
    node_geometry(a.B, a.g.Z, a.g.M, grid, block);
    hipLaunchKernelGGL((cn_kernel<DC, KIND, UCN>), grid, block, 0, s, a);
    return hipGetLastError();
}

template <int KIND>
static hipError_t dispatch_vn(int dv, const VNArgs& a, hipStream_t s) {
    switch (deg_bucket(dv)) {
        case 8: return launch_vn<8, KIND>(a, s);
        case 16: return launch_vn<16, KIND>(a, s);
        case 32: return launch_vn<32, KIND>(a, s);
        default: return launch_vn<64, KIND>(a, s);
    }
}

static hipError_t vn_launch(int kind, const VNArgs& a, hipStream_t s) {
    switch (kind) {
        case NLDPC_NEURAL: return dispatch_vn<NLDPC_NEURAL>(a.g.max_dv, a, s);
        case NLDPC_SP: return dispatch_vn<NLDPC_SP>(a.g.max_dv, a, s);
        case NLDPC_MS: return dispatch_vn<NLDPC_MS>(a.g.max_dv, a, s);
        default: return dispatch_vn<NLDPC_QMS>(a.g.max_dv, a, s);
    }
}

template <int KIND, bool UCN>
static hipError_t dispatch_cn2(const CNArgs& a, hipStream_t s) {
    switch (deg_bucket(a.g.max_dc)) {
        case 8: return launch_cn<8, KIND, UCN>(a, s);
        case 16: return launch_cn<16, KIND, UCN>(a, s);
        case 32: return launch_cn<32, KIND, UCN>(a, s);
        default: return hipErrorInvalidValue;  // d_c > 32 needs a wider sign mask
    }
}

template <int KIND>
static hipError_t dispatch_cn(bool ucn, const CNArgs& a, hipStream_t s) {
    return ucn ? dispatch_cn2<KIND, true>(a, s) : dispatch_cn2<KIND, false>(a, s);
}

static hipError_t cn_launch(int kind, bool ucn, const CNArgs& a, hipStream_t s) {
    switch (kind) {
        case NLDPC_NEURAL: return dispatch_cn2<NLDPC_NEURAL, false>(a, s);
        case NLDPC_SP: return dispatch_cn<NLDPC_SP>(ucn, a, s);
        case NLDPC_MS: return dispatch_cn<NLDPC_MS>(ucn, a, s);
        default: return dispatch_cn<NLDPC_QMS>(ucn, a, s);
    }
}

int validate_cfg(const nldpc_graph* g, const nldpc_cfg* cfg, int64_t B, int32_t T) {
    if (!g || !cfg) return fail(NLDPC_EINVAL, "null graph or cfg");
    if (B <= 0 || T <= 0) return fail(NLDPC_EINVAL, "B and T must be positive");
    if (cfg->kind < NLDPC_SP || cfg->kind > NLDPC_NEURAL) return fail(NLDPC_EINVAL, "unknown decoder kind");
    if (g->dev.max_dc > 32) return fail(NLDPC_EUNSUPPORTED, "check degree above 32 is not supported");
    if (cfg->kind == NLDPC_NEURAL && (cfg->ucn || cfg->vn_cumulative))
        return fail(NLDPC_EINVAL, "the Neural decoder has no UCN / VN weighting");
    if (B > 0x7FFFFFFFLL) return fail(NLDPC_EUNSUPPORTED, "batch too large for one launch (split the batch)");
    if (cfg->vn_prefix < 0 || (cfg->vn_prefix > 0 && !cfg->vn_cumulative))
        return fail(NLDPC_EINVAL, "vn_prefix needs vn_cumulative");
    return NLDPC_OK;
}

SavedLayout saved_layout(const nldpc_graph* g, const nldpc_cfg* cfg, int64_t B, int32_t T) {
    SavedLayout L;
    const int64_t EZ = (int64_t)g->dev.E * g->dev.Z, NZ = (int64_t)g->dev.N * g->dev.Z;
    L.v2c_off = 0;
    L.v2c_stride = B * EZ;  // floats per iteration
    const size_t v2c_bytes = (size_t)T * B * EZ * sizeof(float);
    L.ymask_off = (v2c_bytes + 255) & ~(size_t)255;
    L.ymask_stride = B * NZ;  // bytes per iteration
    L.has_ymask = cfg->kind != NLDPC_NEURAL;
    L.total = L.has_ymask ? L.ymask_off + (size_t)T * B * NZ : v2c_bytes;
    return L;
}

static bool fused_eligible(const nldpc_graph* g, const nldpc_cfg* cfg, int32_t T, bool saving) {
    static const bool disabled = std::getenv("NLDPC_DISABLE_FUSED") != nullptr;
    if (disabled || (cfg->flags & NLDPC_FLAG_STREAM)) return false;
    return g->fused >= 0 && !saving && !cfg->ucn && !cfg->c2v_in && T <= kFusedMaxT;
}

static int fused_forward(const nldpc_graph* g, const nldpc_cfg* cfg, int64_t B, int32_t T, const float* xa,
                         const float* w_cn, const float* bias, const float* w_vn, float* const* outs, float* c2v,
                         hipStream_t s) {
    int n = 0;
    const FusedSpec& f = fused_specs(&n)[g->fused];
    FusedArgs fa{};
    fa.B = B;
    fa.T = T;
    fa.qbit = cfg->qbit;
    fa.xa = xa;
    fa.w_cn = w_cn;
    fa.bias = bias;
    fa.w_vn = cfg->vn_cumulative ? w_vn : nullptr;
    fa.vn_prefix = cfg->vn_prefix;
    fa.lo = cfg->llr_lo;
    fa.hi = cfg->llr_hi;
    fa.c2v_out = (cfg->flags & NLDPC_FLAG_NO_STATE) ? nullptr : c2v;
    for (int k = 0; k < kFusedMaxT; ++k) fa.outs.p[k] = k < T ? outs[k] : nullptr;
    void* args[] = {&fa};
    const int64_t blocks = (B + f.G - 1) / f.G;
    prof_start(PROF_FUSED, s);
    hipError_t e = hipLaunchKernel(f.kernels[cfg->kind], dim3((unsigned)blocks), dim3(f.threads), args, 0, s);
    prof_stop(s);
    if (e == hipSuccess) e = hipGetLastError();
    return e == hipSuccess ? NLDPC_OK : hip_fail(e, "fused kernel launch");
}

}  // namespace nldpc

using namespace nldpc;

extern "C" int nldpc_fast_path(const nldpc_graph* g, const nldpc_cfg* cfg, int64_t B, int32_t T, int32_t saving,
                               int32_t* eligible) {
    int st = validate_cfg(g, cfg, B, T);
    if (st) return st;
    if (!eligible) return fail(NLDPC_EINVAL, "nldpc_fast_path: null output");
    *eligible = fused_eligible(g, cfg, T, saving != 0) ? 1 : 0;
    return NLDPC_OK;
}

extern "C" int nldpc_saved_bytes(const nldpc_graph* g, const nldpc_cfg* cfg, int64_t B, int32_t T, size_t* bytes) {
    int st = validate_cfg(g, cfg, B, T);
    if (st) return st;
    if (!bytes) return fail(NLDPC_EINVAL, "nldpc_saved_bytes: null output");
    *bytes = saved_layout(g, cfg, B, T).total;
    return NLDPC_OK;
}

extern "C" int nldpc_forward(const nldpc_graph* g, const nldpc_cfg* cfg, int64_t B, int32_t T, const float* xa,
                             const float* w_cn, const float* w_ucn, const float* bias, const float* w_vn,
                             float* const* outs, const float* app_prev, float* c2v, float* v2c, void* saved,
                             void* stream) {
    int st = validate_cfg(g, cfg, B, T);
    if (st) return st;
    if (!xa || !outs) return fail(NLDPC_EINVAL, "nldpc_forward: xa and outs are required");
    if (cfg->kind == NLDPC_NEURAL && (!w_cn || !bias))
        return fail(NLDPC_EINVAL, "nldpc_forward: the Neural decoder needs w_cn and bias");
    if (cfg->ucn) {
        for (int k = 0; k + 1 < T; ++k)
            if (!outs[k]) return fail(NLDPC_EINVAL, "nldpc_forward: UCN needs every intermediate output");
        if (cfg->first_iter > 0 && !app_prev)
            return fail(NLDPC_EINVAL, "nldpc_forward: UCN after iteration 0 needs app_prev");
    }
    if (cfg->vn_cumulative && !w_vn) return fail(NLDPC_EINVAL, "nldpc_forward: vn_cumulative needs w_vn");
    if (saved) {
        for (int k = 0; k < T; ++k)
            if (!outs[k]) return fail(NLDPC_EINVAL, "nldpc_forward: saving for backward needs every output");
    }
    DeviceGuard guard(g->device);
    hipStream_t s = static_cast<hipStream_t>(stream);
    const bool fused = fused_eligible(g, cfg, T, saved != nullptr);
    if ((cfg->flags & NLDPC_FLAG_FUSED) && !fused)
        return fail(NLDPC_EUNSUPPORTED, "nldpc_forward: the fused path is not available for this call");
    if (fused) {
        if (!c2v && !(cfg->flags & NLDPC_FLAG_NO_STATE))
            return fail(NLDPC_EINVAL, "nldpc_forward: c2v is required unless NLDPC_FLAG_NO_STATE");
        return fused_forward(g, cfg, B, T, xa, w_cn, bias, w_vn, outs, c2v, s);
    }
    if (!c2v) return fail(NLDPC_EINVAL, "nldpc_forward: c2v is required by the streaming path");
    if (!v2c && !saved) return fail(NLDPC_EINVAL, "nldpc_forward: need v2c scratch or saved buffer");
    const DevGraph& G = g->dev;
    const SavedLayout SL = saved_layout(g, cfg, B, T);
    float* saved_v2c = saved ? reinterpret_cast<float*>(static_cast<char*>(saved) + SL.v2c_off) : nullptr;
    uint8_t* saved_mask = (saved && SL.has_ymask) ? static_cast<uint8_t*>(saved) + SL.ymask_off : nullptr;
    bool state_valid = cfg->c2v_in != 0;
    for (int k = 0; k < T; ++k) {
        float* v2c_k = saved_v2c ? saved_v2c + (int64_t)k * SL.v2c_stride : v2c;
        VNArgs va{G,
                  B,
                  xa,
                  state_valid ? c2v : nullptr,
                  v2c_k,
                  k >= 1 ? outs[k - 1] : nullptr,
                  (k >= 1 && saved_mask) ? saved_mask + (int64_t)(k - 1) * SL.ymask_stride : nullptr,
                  cfg->vn_cumulative ? w_vn : nullptr,
                  cfg->vn_prefix + k + 1,
                  cfg->qbit,
                  cfg->llr_lo,
                  cfg->llr_hi};
        prof_start(PROF_VN, s);
        hipError_t e = vn_launch(cfg->kind, va, s);
        prof_stop(s);
        if (e != hipSuccess) return hip_fail(e, "vn_kernel launch");
        const float* app = nullptr;
        if (cfg->ucn) app = k >= 1 ? outs[k - 1] : (cfg->first_iter > 0 ? app_prev : nullptr);
        CNArgs ca{G,
                  B,
                  v2c_k,
                  c2v,
                  w_cn ? w_cn + (int64_t)k * G.E : nullptr,
                  (cfg->ucn && w_ucn) ? w_ucn + (int64_t)k * G.E : nullptr,
                  bias ? bias + (int64_t)k * G.E : nullptr,
                  app,
                  xa,
                  cfg->vn_cumulative ? w_vn : nullptr,
                  cfg->qbit,
                  cfg->llr_lo,
                  cfg->llr_hi};
        prof_start(PROF_CN, s);
        e = cn_launch(cfg->kind, cfg->ucn != 0, ca, s);
        prof_stop(s);
        if (e != hipSuccess) return hip_fail(e, "cn_kernel launch");
        state_valid = true;
    }
    if (outs[T - 1]) {
        VNArgs va{G, B, xa, c2v, nullptr, outs[T - 1],
                  saved_mask ? saved_mask + (int64_t)(T - 1) * SL.ymask_stride : nullptr, nullptr, 0, cfg->qbit,
                  cfg->llr_lo, cfg->llr_hi};
        prof_start(PROF_POST, s);
        hipError_t e = vn_launch(cfg->kind, va, s);
        prof_stop(s);
        if (e != hipSuccess) return hip_fail(e, "posterior launch");
    }
    return NLDPC_OK;
}
