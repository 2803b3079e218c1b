// Register-resident fused decoder: shared declarations for the generated kernels
// (gen_fused.py -> nldpc_fused_gen.hip) and their dispatcher in nldpc_forward.hip.
#pragma once

#include "nldpc_node.h"

namespace nldpc {

constexpr int kFusedMaxT = 64;

struct OutPtrs {
    float* p[kFusedMaxT];
};

struct FusedArgs {
    int64_t B;
    int32_t T;
    int32_t qbit;
    const float* xa;     // [B][N][Z]
    const float* w_cn;   // [T][E] or nullptr
    const float* bias;   // [T][E] or nullptr
    const float* w_vn;   // [vn_prefix + T][N] or nullptr
    int32_t vn_prefix;
    float lo, hi;
    float* c2v_out;      // [B][E][Z] final message state, or nullptr
    OutPtrs outs;        // T posteriors [B][N][Z] (nullptr entries are skipped)
};

// posterior of one variable copy: Neural xa + P; Boosted clamp(Q(xa) + P) (Boosted…py:513-521)
template <int KIND>
__device__ __forceinline__ float posterior(float xav, float P, const FusedArgs& a) {
    if (KIND == NLDPC_NEURAL) return fadd(xav, P);
    const float xo = (KIND == NLDPC_QMS) ? quantize(xav, a.qbit) : xav;
    return clampf(fadd(xo, P), a.lo, a.hi);
}

struct FusedSpec {
    const char* tag;
    int32_t M, N, Z, E, G, threads;
    const int32_t* basegraph;  // [M*N]
    void* kernels[4];          // indexed by nldpc_kind
};

const FusedSpec* fused_specs(int* n);

}  // namespace nldpc
