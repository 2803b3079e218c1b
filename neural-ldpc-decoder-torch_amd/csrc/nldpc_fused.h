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

// Global memory of the fused kernels goes through buffer descriptors built from wave-uniform values:
// one 32-bit VGPR byte offset per lane serves every access (the per-column constant rides in the
// SGPR/immediate offset), instead of a 64-bit VGPR address pair per access.  The descriptor's size
// covers only the block's live codewords: loads beyond it return 0, stores are dropped, so the lanes
// of a partial last workgroup need no predication.
using rsrc_t = __amdgpu_buffer_rsrc_t;

__device__ __forceinline__ rsrc_t make_rsrc(const float* p, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ float bload(rsrc_t r, uint32_t vo, int so) {
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, vo, so, 0));
}
__device__ __forceinline__ void bstore(rsrc_t r, uint32_t vo, int so, float v) {
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), r, vo, so, 0);
}

// posterior of one variable copy: Neural xa + P; Boosted clamp(Q(xa) + P) (Boosted…py:513-521)
template <int KIND>
__device__ __forceinline__ float posterior(float xav, float P, const FusedArgs& a) {
    if (KIND == NLDPC_NEURAL) return fadd(xav, P);
    const float xo = (KIND == NLDPC_QMS) ? quantize(xav, a.qbit) : xav;
    return clampf(fadd(xo, P), a.lo, a.hi);
}

// Weights are wave-uniform per edge: read through the constant address space so they arrive by
// scalar loads (a row's edges are consecutive in C order: one s_load_dwordx8/x16 per row).
typedef const float __attribute__((address_space(4)))* cfloat_p;

// Neural check node of one check copy of a degree-DC row, in place: m[k] (gathered v2c) -> c2v, with
// the reference's arithmetic (NeuralLDPCDecoder.py:74-91) specialised to what the Neural rule can
// produce.  The magnitude is min(10000, min over the OTHER edges' nonzero |m|); with the ordering key
// bits(|x|) - 1 (unsigned: exact zeros become the largest key, positive floats keep their order) the
// two smallest keys are tracked branch-free, and an edge whose key equals the minimum gets the second
// minimum (ties give min1 == min2, as the first-index argmin of cn_core does).  sign: +1 iff the
// number of strictly positive OTHER inputs is odd (x_output_0's sign product).  The epilogue is
// relu(|x|*w + b) * sign with the same two roundings.  Bit-identical to cn_core + cn_epilogue
// (tests compare the fused and streaming paths).
template <int DC>
__device__ __forceinline__ void neural_row(float (&m)[DC], const float (&w)[DC], const float (&b)[DC]) {
    constexpr uint32_t kInit = 0x461C3FFFu;  // bits(10000.f) - 1
    uint32_t min1 = kInit, min2 = kInit;
    uint32_t key[DC];
    bool pos[DC];
    bool par = false;
#pragma unroll
    for (int k = 0; k < DC; ++k) {
        key[k] = (__builtin_bit_cast(uint32_t, m[k]) & 0x7fffffffu) - 1u;
        pos[k] = m[k] > 0.f;
        par ^= pos[k];
        min2 = min(min2, max(min1, key[k]));
        min1 = min(min1, key[k]);
    }
    const float f1 = __builtin_bit_cast(float, min1 + 1u);
    const float f2 = __builtin_bit_cast(float, min2 + 1u);
#pragma unroll
    for (int k = 0; k < DC; ++k) {
        const float mag = key[k] == min1 ? f2 : f1;
        const float r = relu_mask(fadd(fmul(mag, w[k]), b[k]));
        m[k] = (par != pos[k]) ? r : -r;  // x * (+-1): an exact sign flip
    }
}

struct FusedSpec {
    const char* tag;
    int32_t M, N, Z, E, G, threads;
    const int32_t* basegraph;  // [M*N]
    void* kernels[4];          // indexed by nldpc_kind
};

const FusedSpec* fused_specs(int* n);

}  // namespace nldpc
