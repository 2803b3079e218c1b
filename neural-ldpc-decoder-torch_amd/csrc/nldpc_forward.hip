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
// Message state is [B][E][Z] fp32 in HBM with E in C-order; see DESIGN.md for the roofline.  The c2v
// state is indexed by variable copy v; the v2c messages (scratch, and the copies saved for the backward)
// by check copy h = (v - s_e) mod Z, so the check node reads them unrotated and the fused kernels save
// and stage them as contiguous blocks of their check-ordered LDS images.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "nldpc_fused.h"

namespace nldpc {

struct VNArgs {
    DevGraph g;
    int64_t B;
    const float* xa;     // [B][N][Z]
    const float* c2v;    // [B][E][Z] or nullptr (all-zero state)
    float* v2c;          // [B][E][Z] or nullptr (posterior only)
    int8_t* v2c_code;    // [B][E][Z] QMS int8 codes of v2c (saved for the backward), or nullptr
    float* post;         // [B][N][Z] or nullptr
    uint8_t* ymask;      // [B][N][Z] clamp mask of the posterior (training) or nullptr
    const float* w_vn;   // [steps][N] cumulative VN weights (boosted) or nullptr
    int32_t n_vn_steps;  // number of cumulative weighting/quantisation steps for xin
    const float* xin_prev;  // [B][N][Z] xin after n_vn_steps-1 steps (saved), or nullptr: from xa
    float* xin_out;         // [B][N][Z] xin of this iteration (saved for the backward), or nullptr
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
__device__ __forceinline__ void vn_body(const VNArgs& a, const Geo& q, const int beg, const int d) {
    const int Z = a.g.Z, N = a.g.N, E = a.g.E;
    const int v = q.v, j = q.node;
    const int64_t b = q.b;
    const int64_t idx = (b * N + j) * Z + v;
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
        float ch;
        if (KIND != NLDPC_NEURAL && a.xin_prev) {  // one more step of the chain (same ops, same result)
            ch = fmul(a.xin_prev[idx], a.w_vn[(int64_t)(a.n_vn_steps - 1) * N + j]);
            if (KIND == NLDPC_QMS) ch = quantize(ch, a.qbit);
        } else {
            ch = vn_channel<KIND>(xav, a.w_vn, N, j, a.n_vn_steps, a.qbit);
        }
        if (KIND != NLDPC_NEURAL && a.xin_out) a.xin_out[idx] = ch;
        const float x0 = fadd(0.f, ch);  // xa_input @ W_skipconn2even
        float P = 0.f;                   // prefix ((0 + c0) + ... + c_{k-1})
#pragma unroll
        for (int k = 0; k < DV; ++k) {
            if (k < d) {
                float S = P;  // sum of the others, left to right, skipping k
#pragma unroll
                for (int m = k + 1; m < DV; ++m)
                    if (m < d) S = fadd(S, c[m]);
                const float m = fadd(x0, S);
                // v2c is kept in CHECK order: slot h = (v - s_e) mod Z is read by check copy h
                int hh = v - a.g.e_shift[eidx[k]];
                hh += hh < 0 ? Z : 0;
                a.v2c[(base + eidx[k]) * Z + hh] = m;
                if (KIND == NLDPC_QMS && a.v2c_code) a.v2c_code[(base + eidx[k]) * Z + hh] = (int8_t)qms_code(m, a.qbit);
                P = fadd(P, c[k]);
            }
        }
    }
}

template <int DC, int KIND, bool UCN>
__device__ __forceinline__ void cn_body(const CNArgs& a, const Geo& q, const int beg, const int d) {
    const int Z = a.g.Z, E = a.g.E;
    const int h = q.v;
    const int64_t b = q.b;
    const int64_t base = b * E;

    int vv[DC];
    float m[DC];
#pragma unroll
    for (int k = 0; k < DC; ++k) {
        if (k < d) {
            const int t = h + a.g.e_shift[beg + k];
            vv[k] = t >= Z ? t - Z : t;
            m[k] = a.v2c[(base + beg + k) * Z + h];  // (check order: the VN kernel rotated it)
        } else {
            vv[k] = 0;
            m[k] = 0.f;
        }
    }
    const float u = UCN ? ucn_flag<DC, KIND>(a.g, beg, d, vv, b, a.app, a.xa, a.w_vn0, a.qbit) : 0.f;
    CnCore<DC> core;
    cn_core<DC, KIND>(m, d, a.qbit, a.lo, a.hi, core, SpRow{a.g.sp_plan + q.node * kSpPlanBytes, a.g.tanh});
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

template <int KIND, int MAXD>
__global__ __launch_bounds__(512) void vn_kernel(VNArgs a) {
    const Geo q = geo(a.B, a.g.Z);
    if (!q.ok) return;
    const int beg = a.g.col_ptr[q.node];
    deg_switch<MAXD>(a.g.col_ptr[q.node + 1] - beg,
                     [&](auto D, int d) { vn_body<decltype(D)::value, KIND>(a, q, beg, d); });
}

template <int KIND, bool UCN, int MAXD>
__global__ __launch_bounds__(512) void cn_kernel(CNArgs a) {
    const Geo q = geo(a.B, a.g.Z);
    if (!q.ok) return;
    const int beg = a.g.row_ptr[q.node];
    deg_switch<MAXD>(a.g.row_ptr[q.node + 1] - beg,
                     [&](auto D, int d) { cn_body<decltype(D)::value, KIND, UCN>(a, q, beg, d); });
}

template <int KIND, int MAXD>
static hipError_t vn_launch_k(const VNArgs& a, hipStream_t s) {
    dim3 grid, block;
    node_geometry(a.B, a.g.Z, a.g.N, grid, block);
    hipLaunchKernelGGL((vn_kernel<KIND, MAXD>), grid, block, 0, s, a);
    return hipGetLastError();
}

template <int KIND>
static hipError_t vn_launch_m(const VNArgs& a, hipStream_t s) {
    switch (deg_max_bucket(a.g.max_dv)) {
        case 12: return vn_launch_k<KIND, 12>(a, s);
        case 16: return vn_launch_k<KIND, 16>(a, s);
        case 24: return vn_launch_k<KIND, 24>(a, s);
        case 32: return vn_launch_k<KIND, 32>(a, s);
        default: return vn_launch_k<KIND, 64>(a, s);
    }
}

template <int KIND, bool UCN>
static hipError_t cn_launch_k(const CNArgs& a, hipStream_t s) {
    dim3 grid, block;
    node_geometry(a.B, a.g.Z, a.g.M, grid, block);
    // SP's check node (DC^2 ordered products per copy) is instantiated for two degree buckets only
    const int bucket = deg_max_bucket(a.g.max_dc);
    if constexpr (KIND == NLDPC_SP) {
        if (bucket <= 16) hipLaunchKernelGGL((cn_kernel<KIND, UCN, 16>), grid, block, 0, s, a);
        else hipLaunchKernelGGL((cn_kernel<KIND, UCN, 32>), grid, block, 0, s, a);
    } else {
        switch (bucket) {
            case 12: hipLaunchKernelGGL((cn_kernel<KIND, UCN, 12>), grid, block, 0, s, a); break;
            case 16: hipLaunchKernelGGL((cn_kernel<KIND, UCN, 16>), grid, block, 0, s, a); break;
            case 24: hipLaunchKernelGGL((cn_kernel<KIND, UCN, 24>), grid, block, 0, s, a); break;
            default: hipLaunchKernelGGL((cn_kernel<KIND, UCN, 32>), grid, block, 0, s, a); break;
        }
    }
    return hipGetLastError();
}

static hipError_t vn_launch(int kind, const VNArgs& a, hipStream_t s) {
    switch (kind) {
        case NLDPC_NEURAL: return vn_launch_m<NLDPC_NEURAL>(a, s);
        case NLDPC_SP: return vn_launch_m<NLDPC_SP>(a, s);
        case NLDPC_MS: return vn_launch_m<NLDPC_MS>(a, s);
        default: return vn_launch_m<NLDPC_QMS>(a, s);
    }
}

static hipError_t cn_launch(int kind, bool ucn, const CNArgs& a, hipStream_t s) {
    switch (kind) {
        case NLDPC_NEURAL: return cn_launch_k<NLDPC_NEURAL, false>(a, s);
        case NLDPC_SP: return ucn ? cn_launch_k<NLDPC_SP, true>(a, s) : cn_launch_k<NLDPC_SP, false>(a, s);
        case NLDPC_MS: return ucn ? cn_launch_k<NLDPC_MS, true>(a, s) : cn_launch_k<NLDPC_MS, false>(a, s);
        default: return ucn ? cn_launch_k<NLDPC_QMS, true>(a, s) : cn_launch_k<NLDPC_QMS, false>(a, s);
    }
}

int validate_cfg(const nldpc_graph* g, const nldpc_cfg* cfg, int64_t B, int32_t T) {
    if (!g || !cfg) return fail(NLDPC_EINVAL, "null graph or cfg");
    if (B <= 0 || T <= 0) return fail(NLDPC_EINVAL, "B and T must be positive");
    if (cfg->kind < NLDPC_SP || cfg->kind > NLDPC_NEURAL) return fail(NLDPC_EINVAL, "unknown decoder kind");
    if (g->dev.max_dc > 32) return fail(NLDPC_EUNSUPPORTED, "check degree above 32 is not supported");
    if (g->dev.max_dv > 64) return fail(NLDPC_EUNSUPPORTED, "variable degree above 64 is not supported");
    if (cfg->kind == NLDPC_NEURAL && (cfg->ucn || cfg->vn_cumulative))
        return fail(NLDPC_EINVAL, "the Neural decoder has no UCN / VN weighting");
    if (B > 0x7FFFFFFFLL) return fail(NLDPC_EUNSUPPORTED, "batch too large for one launch (split the batch)");
    if (cfg->vn_prefix < 0 || (cfg->vn_prefix > 0 && !cfg->vn_cumulative))
        return fail(NLDPC_EINVAL, "vn_prefix needs vn_cumulative");
    if (cfg->kind == NLDPC_SP && !g->dev.tanh.idx) {
        // without the table the device tanh is the rounded double tanh: within one ulp of torch.tanh
        // (gen_tanh_table.py), so SP stays within the SP tolerance but is no longer value for value
        static bool warned = false;
        if (!warned) {
            warned = true;
            std::fprintf(stderr, "nldpc: lib/nldpc_tanh_ref.bin not found next to libnldpc.so (or $NLDPC_TANH_TABLE): "
                                 "the SP check node uses the correctly rounded tanh, within one ulp of torch.tanh\n");
        }
    }
    return NLDPC_OK;
}

SavedLayout saved_layout(const nldpc_graph* g, const nldpc_cfg* cfg, int64_t B, int32_t T) {
    SavedLayout L;
    const int64_t EZ = (int64_t)g->dev.E * g->dev.Z, NZ = (int64_t)g->dev.N * g->dev.Z;
    L.v2c_off = 0;
    L.v2c_stride = B * EZ;  // messages per iteration
    L.v2c_code = cfg->kind == NLDPC_QMS && qms_active(cfg->qbit);
    const size_t v2c_bytes = (size_t)T * B * EZ * (L.v2c_code ? 1 : sizeof(float));
    L.ymask_off = (v2c_bytes + 255) & ~(size_t)255;
    L.ymask_stride = B * NZ;  // bytes per iteration
    L.has_ymask = cfg->kind != NLDPC_NEURAL;
    const size_t end = L.has_ymask ? L.ymask_off + (size_t)T * B * NZ : v2c_bytes;
    L.has_xin = cfg->vn_cumulative != 0;
    L.xin_off = (end + 255) & ~(size_t)255;
    L.xin_stride = B * NZ;  // floats per iteration
    L.total = L.has_xin ? L.xin_off + (size_t)T * B * NZ * sizeof(float) : end;
    return L;
}

// mode: 0 decode, 1 decode + save for backward, 2 / 3 count-only (the fused kernel variants)
static bool fused_eligible(const nldpc_graph* g, const nldpc_cfg* cfg, int32_t T, int mode) {
    const bool saving = mode == 1;
    static const bool disabled = std::getenv("NLDPC_DISABLE_FUSED") != nullptr;
    if (disabled || (cfg->flags & NLDPC_FLAG_STREAM)) return false;
    // QMS: the fused kernels' check node is the active quantiser's (boosted_row), and the SAVE kernels'
    // int8 codes need one too; an inactive qbit decodes on the streaming kernels
    (void)saving;
    if (cfg->kind == NLDPC_QMS && !qms_active(cfg->qbit)) return false;
    return fused_launch(g, mode, cfg->kind) && !cfg->c2v_in && T <= kFusedMaxT;
}

static int fused_forward(const nldpc_graph* g, const nldpc_cfg* cfg, int64_t B, int32_t T, const float* xa,
                         const float* w_cn, const float* w_ucn, const float* bias, const float* w_vn,
                         float* const* outs, const float* app_prev, float* c2v, void* saved, hipStream_t s,
                         const uint8_t* cnt_y = nullptr, int32_t cnt_conv = 0, int64_t* counts = nullptr) {
    const int mode = saved ? 1 : (counts ? ((cnt_y || cnt_conv) ? 3 : 2) : 0);
    // (r6) a saving forward with one CN weight per iteration (NLDPC_FLAG_CN_TIED: sharing code 3, cfg5's NW(3,0,3)) and no
    // UCN runs the kernel specialised for it when the library has one: one scalar weight per iteration instead of a
    // per-edge row in SGPRs (the per-edge kernel spilled ~1 450 SGPRs), the UCN code not compiled
    const bool tied = saved && (cfg->flags & NLDPC_FLAG_CN_TIED) && w_cn && !cfg->ucn &&
                      (cfg->kind == NLDPC_MS || cfg->kind == NLDPC_QMS);
    // (r6) a plain decode with UCN and CN / UCN / cumulative VN weights all given (the Boosted NW(1,1,2) decode) runs the
    // kernel with those flags compiled in when the library has one (MODE 7; fewer uniform branches and SGPR spills)
    const bool ucnw = mode == 0 && cfg->ucn && w_cn && w_ucn && cfg->vn_cumulative && w_vn &&
                      (cfg->kind == NLDPC_MS || cfg->kind == NLDPC_QMS);
    const FusedLaunch ft = tied ? fused_launch(g, 6, cfg->kind) : ucnw ? fused_launch(g, 7, cfg->kind) : FusedLaunch{};
    const FusedLaunch f = ft ? ft : fused_launch(g, mode, cfg->kind);
    if (!f) return fail(NLDPC_EUNSUPPORTED, "no register-resident kernel for this graph / mode / kind");
    FusedArgs fa{};
    fa.sig = kFusedArgsSig;
    fa.B = B;
    fa.T = T;
    fa.qbit = cfg->qbit;
    fa.qp = q_params(cfg->qbit);
    fa.xa = xa;
    fa.w_cn = w_cn;
    fa.bias = bias;
    fa.ucn = cfg->ucn ? 1 : 0;
    fa.w_ucn = cfg->ucn ? w_ucn : nullptr;
    fa.first_iter = cfg->first_iter;
    fa.app_prev = (cfg->ucn && cfg->first_iter > 0) ? app_prev : nullptr;
    fa.w_vn = cfg->vn_cumulative ? w_vn : nullptr;
    fa.vn_prefix = cfg->vn_prefix;
    fa.sp_plan = g->dev.sp_plan;
    fa.tanh = g->dev.tanh;
    fa.lo = cfg->llr_lo;
    fa.hi = cfg->llr_hi;
    fa.c2v_out = (cfg->flags & NLDPC_FLAG_NO_STATE) ? nullptr : c2v;
    for (int k = 0; k < kFusedMaxT; ++k) fa.outs.p[k] = (outs && k < T) ? outs[k] : nullptr;
    fa.cnt_y = cnt_y;
    fa.cnt_conv = cnt_conv;
    fa.cnt = reinterpret_cast<unsigned long long*>(counts);
    if (saved) {
        const SavedLayout SL = saved_layout(g, cfg, B, T);
        char* sb = static_cast<char*>(saved);
        fa.sv2c = sb + SL.v2c_off;  // QMS: int8 codes (the kernel knows from its kind)
        fa.sv2c_stride = SL.v2c_stride;
        fa.symask = SL.has_ymask ? reinterpret_cast<uint8_t*>(sb + SL.ymask_off) : nullptr;
        fa.symask_stride = SL.ymask_stride;
        fa.sxin = SL.has_xin ? reinterpret_cast<float*>(sb + SL.xin_off) : nullptr;
        fa.sxin_stride = SL.xin_stride;
    }
    // diagnostic stamp build (lib_stamps/): NLDPC_STAMPS=<file> collects the phase stamps of each call
    static const char* stamp_file = std::getenv("NLDPC_STAMPS");
    const size_t stamp_n = (size_t)256 * (f.threads / 64) * T * 16;
    if (stamp_file) NLDPC_HIP_CHECK(hipMalloc(&fa.stamps, stamp_n * sizeof(uint64_t)));
    if (stamp_file) NLDPC_HIP_CHECK(hipMemsetAsync(fa.stamps, 0, stamp_n * sizeof(uint64_t), s));
    void* args[] = {&fa};
    const int64_t blocks = (B + f.G - 1) / f.G;
    prof_start(PROF_FUSED, s);
    hipError_t e = f.launch(blocks, args, s);
    prof_stop(s);
    if (e == hipSuccess) e = hipGetLastError();
    if (stamp_file && e == hipSuccess) {
        std::vector<uint64_t> h(stamp_n);
        NLDPC_HIP_CHECK(hipStreamSynchronize(s));
        NLDPC_HIP_CHECK(hipMemcpy(h.data(), fa.stamps, stamp_n * sizeof(uint64_t), hipMemcpyDeviceToHost));
        if (FILE* fp = std::fopen(stamp_file, "wb")) {
            const int32_t hdr[4] = {256, f.threads / 64, T, 16};
            std::fwrite(hdr, sizeof(hdr), 1, fp);
            std::fwrite(h.data(), sizeof(uint64_t), stamp_n, fp);
            std::fclose(fp);
        }
        (void)hipFree(fa.stamps);
    }
    return e == hipSuccess ? NLDPC_OK : hip_fail(e, "fused kernel launch");
}

}  // namespace nldpc

using namespace nldpc;

extern "C" int nldpc_fast_path(const nldpc_graph* g, const nldpc_cfg* cfg, int64_t B, int32_t T, int32_t saving,
                               int32_t* eligible) {
    int st = validate_cfg(g, cfg, B, T);
    if (st) return st;
    if (!eligible) return fail(NLDPC_EINVAL, "nldpc_fast_path: null output");
    if (saving < 0 || saving > 3) return fail(NLDPC_EINVAL, "nldpc_fast_path: saving is 0, 1 (or 2 / 3: count-only)");
    *eligible = fused_eligible(g, cfg, T, saving) ? 1 : 0;
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
    const bool fused = fused_eligible(g, cfg, T, saved != nullptr ? 1 : 0);
    if ((cfg->flags & NLDPC_FLAG_FUSED) && !fused)
        return fail(NLDPC_EUNSUPPORTED, "nldpc_forward: the fused path is not available for this call");
    if (fused) {
        if (!c2v && !(cfg->flags & NLDPC_FLAG_NO_STATE))
            return fail(NLDPC_EINVAL, "nldpc_forward: c2v is required unless NLDPC_FLAG_NO_STATE");
        return fused_forward(g, cfg, B, T, xa, w_cn, w_ucn, bias, w_vn, outs, app_prev, c2v, saved, s);
    }
    if (!c2v) return fail(NLDPC_EINVAL, "nldpc_forward: c2v is required by the streaming path");
    if (!v2c && !saved) return fail(NLDPC_EINVAL, "nldpc_forward: need v2c scratch or saved buffer");
    const DevGraph& G = g->dev;
    const SavedLayout SL = saved_layout(g, cfg, B, T);
    float* saved_v2c = (saved && !SL.v2c_code) ? reinterpret_cast<float*>(static_cast<char*>(saved) + SL.v2c_off) : nullptr;
    int8_t* saved_code = (saved && SL.v2c_code) ? reinterpret_cast<int8_t*>(static_cast<char*>(saved) + SL.v2c_off) : nullptr;
    if (saved_code && !v2c) return fail(NLDPC_EINVAL, "nldpc_forward: QMS training needs the v2c scratch");
    uint8_t* saved_mask = (saved && SL.has_ymask) ? static_cast<uint8_t*>(saved) + SL.ymask_off : nullptr;
    float* saved_xin = (saved && SL.has_xin) ? reinterpret_cast<float*>(static_cast<char*>(saved) + SL.xin_off) : nullptr;
    bool state_valid = cfg->c2v_in != 0;
    for (int k = 0; k < T; ++k) {
        float* v2c_k = saved_v2c ? saved_v2c + (int64_t)k * SL.v2c_stride : v2c;
        VNArgs va{G,
                  B,
                  xa,
                  state_valid ? c2v : nullptr,
                  v2c_k,
                  saved_code ? saved_code + (int64_t)k * SL.v2c_stride : nullptr,
                  k >= 1 ? outs[k - 1] : nullptr,
                  (k >= 1 && saved_mask) ? saved_mask + (int64_t)(k - 1) * SL.ymask_stride : nullptr,
                  cfg->vn_cumulative ? w_vn : nullptr,
                  cfg->vn_prefix + k + 1,
                  (saved_xin && k >= 1) ? saved_xin + (int64_t)(k - 1) * SL.xin_stride : nullptr,
                  saved_xin ? saved_xin + (int64_t)k * SL.xin_stride : nullptr,
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
        VNArgs va{G, B, xa, c2v, nullptr, nullptr, outs[T - 1],
                  saved_mask ? saved_mask + (int64_t)(T - 1) * SL.ymask_stride : nullptr, nullptr, 0, nullptr,
                  nullptr, cfg->qbit,
                  cfg->llr_lo, cfg->llr_hi};
        prof_start(PROF_POST, s);
        hipError_t e = vn_launch(cfg->kind, va, s);
        prof_stop(s);
        if (e != hipSuccess) return hip_fail(e, "posterior launch");
    }
    return NLDPC_OK;
}

extern "C" int nldpc_forward_count(const nldpc_graph* g, const nldpc_cfg* cfg, int64_t B, int32_t T, const float* xa,
                                   const float* w_cn, const float* w_ucn, const float* bias, const float* w_vn,
                                   const uint8_t* y, int32_t convention, int64_t* counts, void* stream) {
    int st = validate_cfg(g, cfg, B, T);
    if (st) return st;
    if (!xa || !counts) return fail(NLDPC_EINVAL, "nldpc_forward_count: xa and counts are required");
    if (convention != 0 && convention != 1) return fail(NLDPC_EINVAL, "nldpc_forward_count: convention is 0 or 1");
    if (cfg->kind == NLDPC_NEURAL && (!w_cn || !bias))
        return fail(NLDPC_EINVAL, "nldpc_forward_count: the Neural decoder needs w_cn and bias");
    if (cfg->vn_cumulative && !w_vn) return fail(NLDPC_EINVAL, "nldpc_forward_count: vn_cumulative needs w_vn");
    if (!fused_eligible(g, cfg, T, (y || convention) ? 3 : 2) || (cfg->ucn && cfg->first_iter > 0))
        return fail(NLDPC_EUNSUPPORTED, "nldpc_forward_count: needs the fused path (a compiled base graph, no UCN, "
                                        "fresh state, T <= 64); use nldpc_forward + nldpc_ber_count instead");
    DeviceGuard guard(g->device);
    nldpc_cfg c = *cfg;
    c.flags |= NLDPC_FLAG_NO_STATE;
    return fused_forward(g, &c, B, T, xa, w_cn, w_ucn, bias, w_vn, nullptr, nullptr, nullptr, nullptr,
                         static_cast<hipStream_t>(stream), y, convention, counts);
}
