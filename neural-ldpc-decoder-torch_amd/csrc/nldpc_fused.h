// Register-resident fused decoder: shared declarations for the generated kernels
// (gen_fused.py -> lib/gen/fused_*.hip) and their dispatcher in nldpc_forward.hip.
#pragma once

#include <type_traits>

#include "nldpc_node.h"

namespace nldpc {

constexpr int kFusedMaxT = 64;

struct OutPtrs {
    float* p[kFusedMaxT];
};

// Launcher / kernel agreement on the argument structs: the host writes kFused*Sig into `sig` (the first
// field, so any layout reads it), and a generated kernel whose compiled layout differs returns at once
// instead of reading every later field at the wrong offset (r3: an experiment library whose kernels were
// built against a newer FusedArgs than its launcher ran a loop bounded by a pointer's low word).  Bump
// kFusedArgsVersion with every layout change that keeps the size.
constexpr uint32_t kFusedArgsVersion = 5;

struct FusedArgs {
    uint32_t sig;        // kFusedArgsSig
    int64_t B;
    int32_t T;
    int32_t qbit;
    QParams qp;          // QMS: the active quantiser's constants (q_params(qbit)); QMS needs an active q here
    const float* xa;     // [B][N][Z]
    const float* w_cn;   // [T][E] or nullptr
    const float* bias;   // [T][E] or nullptr
    const float* w_ucn;  // [T][E] UCN weights (ucn), or nullptr
    const float* app_prev;  // [B][N][Z] posterior of iteration first_iter-1 (UCN, first_iter > 0), or nullptr
    int32_t ucn, first_iter;
    const float* w_vn;   // [vn_prefix + T][N] or nullptr
    int32_t vn_prefix;
    float lo, hi;
    const uint8_t* sp_plan;  // [M][kSpPlanBytes] SP product order (DevGraph::sp_plan)
    TanhRef tanh;            // torch.tanh table (SP)
    float* c2v_out;      // [B][E][Z] final message state, or nullptr
    // what the backward needs (SAVE kernels only; SavedLayout in nldpc_internal.h)
    char* sv2c;          // [T][B][E][Z] v2c of every iteration by check copy (fp32; QMS: int8 codes, qms_code)
    uint8_t* symask;     // [T][B][N][Z] posterior clamp masks (Boosted), or nullptr
    float* sxin;         // [T][B][N][Z] channel value xin of every iteration (cumulative VN weights), or nullptr
    int64_t sv2c_stride, symask_stride, sxin_stride;  // elements per iteration
    OutPtrs outs;        // T posteriors [B][N][Z] (nullptr entries are skipped)
    // count-only decode (MODE 2 kernels): nldpc_forward_count
    const uint8_t* cnt_y;  // [B][N][Z] codeword bits (MODE 3), or nullptr (all-zero codeword, MODE 2)
    int32_t cnt_conv;      // 0: bit = LLR > 0; 1: bit = LLR < 0
    unsigned long long* cnt;  // [T][2] (+=) bit errors, frame errors
    uint64_t* stamps;    // diagnostic stamp build only (make STAMPS=1): [256][waves][T][16] s_memtime
};

constexpr uint32_t kFusedArgsSig = 0x4e4c0000u ^ ((uint32_t)sizeof(FusedArgs) << 4) ^ kFusedArgsVersion;

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
// Stores are non-temporal (cache-policy nt): the T posteriors stream out once and are never re-read by
// the kernel, so they should not evict what is re-read from L2 -- the channel values of the Boosted
// posterior with cumulative VN weights, and the descriptors' other lines.  Measured on MI355X: cfg3
// Neural kernel 54.9 -> 51.7 ms, cfg3 Boosted MS NW(1,1,2) 116.4 -> 106.8 ms (profiles/r2_ab_boosted.txt).
#ifndef NLDPC_STORE_AUX
#define NLDPC_STORE_AUX 2
#endif
__device__ __forceinline__ void bstore(rsrc_t r, uint32_t vo, int so, float v) {
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), r, vo, so, NLDPC_STORE_AUX);
}
__device__ __forceinline__ void bstore8(rsrc_t r, uint32_t vo, int so, bool v) {
    __builtin_amdgcn_raw_buffer_store_b8((uint8_t)v, r, vo, so, 0);
}
__device__ __forceinline__ void bstore_i8(rsrc_t r, uint32_t vo, int so, int v) {
    __builtin_amdgcn_raw_buffer_store_b8((uint8_t)(v & 0xff), r, vo, so, 0);
}
// (r6, gen_fused.py NLDPC_GEN_FWDNT8, default on: the training forward's byte stores -- clamp masks, QMS saved codes --
// non-temporal like its fp32 stores, so they do not evict the channel values the posteriors re-read)
__device__ __forceinline__ void bstore8_nt(rsrc_t r, uint32_t vo, int so, bool v) {
    __builtin_amdgcn_raw_buffer_store_b8((uint8_t)v, r, vo, so, NLDPC_STORE_AUX);
}
__device__ __forceinline__ void bstore_i8_nt(rsrc_t r, uint32_t vo, int so, int v) {
    __builtin_amdgcn_raw_buffer_store_b8((uint8_t)(v & 0xff), r, vo, so, NLDPC_STORE_AUX);
}
// bytes per saved v2c message of a kernel kind (QMS saves int8 codes)
template <int KIND>
constexpr int saved_msg_bytes() { return KIND == NLDPC_QMS ? 1 : 4; }

// Channel value the VN adds.  With cumulative VN weights (Boosted, w_vn set) the registers hold xin
// itself, advanced one step per iteration by chan_step (Boosted…py:325-337: xin <- Q(xin * w_t)),
// so the chain is never re-run from xa; otherwise they hold xa and QMS quantises it (idempotent).
// QMS quantiser of the channel values and posteriors in the fused kernels
// (the generic quantize(): the four-operation quantize_active behind a select measured 15 % slower in the
// fused QMS kernels, cfg3 NW(1,1,2) 187.6 -> 217 ms -- register allocation, not operation count)
// r6 (NLDPC_QFAST, default): quantize_active_p's four operations with the last multiply as fma(., inv, +0) -- the
// reference's STE form never returns -0 (xc + (qv - xc) rounds an exact cancellation to +0), and the +0 addend
// makes the zeros agree too: equal to quantize_p bit for bit for every non-NaN x (tests/test_qms_code.py), where
// quantize_p spends two compare-and-select clamps (four v_cmp, 5.2 cycles each) on NaN propagation.  A NaN channel
// value gives -hi here instead of NaN.
__device__ __forceinline__ float qms_q(float x, const QParams& p) {
#if NLDPC_QFAST
    return __builtin_fmaf(__builtin_amdgcn_fmed3f(rintf(fmul(x, p.s)), -p.hs, p.hs), p.inv, 0.f);
#else
    return quantize_p(x, p);
#endif
}

template <int KIND>
__device__ __forceinline__ float chan(float x, const FusedArgs& a) {
    if (KIND == NLDPC_NEURAL || a.w_vn) return x;
    return KIND == NLDPC_QMS ? qms_q(x, a.qp) : x;
}
template <int KIND>
__device__ __forceinline__ float chan_step(float x, const FusedArgs& a, float w) {
    x = fmul(x, w);
    return KIND == NLDPC_QMS ? qms_q(x, a.qp) : x;
}

// posterior of one variable copy: Neural xa + P; Boosted clamp(Q(xa) + P) (Boosted…py:513-521), the
// clamp as one med3 (the same value for every non-NaN sum; lo <= hi)
template <int KIND>
__device__ __forceinline__ float posterior(float xav, float P, const FusedArgs& a) {
    if (KIND == NLDPC_NEURAL) return fadd(xav, P);
    const float xo = (KIND == NLDPC_QMS) ? qms_q(xav, a.qp) : xav;
    return __builtin_amdgcn_fmed3f(fadd(xo, P), a.lo, a.hi);
}

// Boosted posterior and its clamp mask (saved for the backward): in_range of the pre-clamp value
template <int KIND>
__device__ __forceinline__ float posterior_m(float xav, float P, const FusedArgs& a, bool& m) {
    const float xo = (KIND == NLDPC_QMS) ? qms_q(xav, a.qp) : xav;
    const float yp = fadd(xo, P);
#if NLDPC_QFAST
    // (r6) the clamp as one med3 and the mask as "the clamp changed nothing": one v_cmp instead of four and two
    // selects; the same for every non-NaN sum (lo <= hi); NaN: mask 0 as before, the value lo instead of NaN
    const float y = __builtin_amdgcn_fmed3f(yp, a.lo, a.hi);
    m = y == yp;
    return y;
#else
    m = yp >= a.lo && yp <= a.hi;
    return clampf(yp, a.lo, a.hi);
#endif
}

// v2c of a degree-1 edge from the channel value its check-node thread holds (degree-1 bypass): Neural
// holds 0 + xa already; Boosted forms (0 + chan(xin)) + 0 as the owner's VN sum would (ZADD: the
// reference's sums start from 0; a lone message adds nothing else)
template <int KIND, int ZADD>
__device__ __forceinline__ float d1_v2c(float cd, const FusedArgs& a) {
    if constexpr (KIND == NLDPC_NEURAL) return cd;
    const float x = chan<KIND>(cd, a);
    return ZADD ? fadd(fadd(0.f, x), 0.f) : x;
}

// UCN hard-decision exchange (Boosted…py:339-374): the owner of variable copy v of column j ORs the bit
// APP[j][v] >= 0 into the codeword's LDS bit array (word base + v / 32); the check node of copy h reads
// the bits of its row's variables at (h + s_e) mod Z and takes their parity (odd = unsatisfied).
__device__ __forceinline__ void app_or(uint32_t* appw, int base, int v, bool bit) {
    if (bit) atomicOr(appw + base + (v >> 5), 1u << (v & 31));
}
// this lane's index in its wave (v_mbcnt: no register kept live for it)
__device__ __forceinline__ int lane_id() { return (int)__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }

// Diagnostic stamp builds only (gen_fused.py NLDPC_GEN_STAMPS): s_memtime of wave w of workgroup b at phase ph of
// iteration it into stamps[256][waves][T][16].  Branch-free across the lanes, with a wave-uniform (scalar) offset: every
// lane stores the same value to the same address (vector stores).  r6: r5's lane-0 branch with per-lane address math
// pushed the training forward's stamp build from 9 to 5 632 spilled VGPRs, so its stamps timed a kernel ten times slower
// than the real one (profiles/r6_stamps_fwd.txt).
__device__ __forceinline__ void stamp_store(uint64_t* stamps, int waves, int T, int it, int ph) {
    if (!stamps || blockIdx.x >= 256) return;
    const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t off = ((((uint32_t)blockIdx.x * waves + wv) * T + it) * 16 + ph) * 8;
    const uint64_t t = __builtin_amdgcn_s_memtime();
    const rsrc_t r = make_rsrc((const float*)stamps, 256u * waves * T * 16 * 8);
    __builtin_amdgcn_raw_buffer_store_b32((uint32_t)t, r, 0, off, 0);
    __builtin_amdgcn_raw_buffer_store_b32((uint32_t)(t >> 32), r, 0, off + 4, 0);
}


// Weights are wave-uniform per edge: read through the constant address space so they arrive by
// scalar loads (a row's edges are consecutive in C order: one s_load_dwordx8/x16 per row).
typedef const float __attribute__((address_space(4)))* cfloat_p;
typedef float __attribute__((address_space(3)))* lds_fp;  // LDS pointer (32-bit)

// Neural check node of one check copy of a degree-DC row, in place: m[k] (gathered v2c) -> c2v, with
// the reference's arithmetic (NeuralLDPCDecoder.py:74-91) specialised to what the Neural rule can
// produce.  The magnitude is min(10000, min over the OTHER edges' nonzero |m|); with the ordering key
// (bits(x) << 1) - 2 = 2*bits(|x|) - 2 (unsigned: exact zeros of either sign wrap to the largest keys,
// nonzero magnitudes keep their order, NaNs sort above 10000 and never win, as in cn_core) the
// two smallest keys are tracked branch-free, and an edge whose key equals the minimum gets the second
// minimum (ties give min1 == min2, as the first-index argmin of cn_core does).  sign: +1 iff the
// number of strictly positive OTHER inputs is odd (x_output_0's sign product).  The epilogue is
// relu(|x|*w + b) * sign with the same two roundings.  Bit-identical to cn_core + cn_epilogue
// (tests compare the fused and streaming paths).
// The two smallest of DC keys (as a multiset: equal keys give min1 == min2), streaming: with a <= b the
// running pair, b' = med3(a, b, x), a' = min(a, x) -- two VALU per key (v_med3_u32, v_min_u32).  Measured
// on gfx950 against a log-depth tournament (pairs, then merges of 3-4 ops): 6 % fewer SIMD cycles per
// row copy at 4 waves per SIMD (tools/dev/cn_micro.hip) -- the other waves cover the serial chain.
__device__ __forceinline__ uint32_t med3_u32(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t d;
    asm("v_med3_u32 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c));
    return d;
}

template <int DC>
__device__ __forceinline__ void two_smallest(const uint32_t (&key)[DC], uint32_t& min1, uint32_t& min2) {
    if constexpr (DC == 1) {
        min1 = key[0];
        min2 = 0xFFFFFFFFu;
    } else {
        uint32_t a = min(key[0], key[1]), b = max(key[0], key[1]);
#pragma unroll
        for (int k = 2; k < DC; ++k) {
            b = med3_u32(a, b, key[k]);
            a = min(a, key[k]);
        }
        min1 = a;
        min2 = b;
    }
}

// The two smallest of |m_k| (as a multiset) in the float domain, |m_k| as a source modifier.  Inline
// asm: written as fminf/fmaxf the compiler materialises every fabsf (v_and_b32) and, in IEEE mode,
// canonicalises each operand (v_max_f32 x, x) -- three extra VALU per edge.  Plain VALU, no hazards.
__device__ __forceinline__ float min_aa(float x, float y) {
    float d;
    asm("v_min_f32_e64 %0, |%1|, |%2|" : "=v"(d) : "v"(x), "v"(y));
    return d;
}
__device__ __forceinline__ float max_aa(float x, float y) {
    float d;
    asm("v_max_f32_e64 %0, |%1|, |%2|" : "=v"(d) : "v"(x), "v"(y));
    return d;
}
__device__ __forceinline__ float min_a(float a, float x) {  // min(a, |x|), a >= 0
    float d;
    asm("v_min_f32_e64 %0, %1, |%2|" : "=v"(d) : "v"(a), "v"(x));
    return d;
}
__device__ __forceinline__ float med3_a(float a, float b, float x) {  // med3(a, b, |x|)
    float d;
    asm("v_med3_f32 %0, %1, %2, |%3|" : "=v"(d) : "v"(a), "v"(b), "v"(x));
    return d;
}

template <int DC>
__device__ __forceinline__ void two_smallest_abs(const float (&m)[DC], float& min1, float& min2) {
    if constexpr (DC == 1) {
        min1 = fabsf(m[0]);
        min2 = __builtin_inff();
    } else {
        float a = min_aa(m[0], m[1]), b = max_aa(m[0], m[1]);
#pragma unroll
        for (int k = 2; k < DC; ++k) {
            b = med3_a(a, b, m[k]);
            a = min_a(a, m[k]);
        }
        min1 = a;
        min2 = b;
    }
}

// The two smallest of |m_k| (as a multiset) with three-input min / median: the first three by one
// v_min3 + one v_med3, then two more at a time by three ops -- with a <= b the running pair,
// a' = min3(a, |x|, |y|), b' = min(b, med3(a, |x|, |y|)) -- and a last single one by med3 + min:
// 1.5 ops per element instead of 2 (on gfx950 min / max / med3 all issue at half the v_add_f32 rate,
// profiles/r3_valu_rate2*.txt).  CAP: the reference's masked tile entries (10000) take part as one
// more element, so the minima come out capped (for an even DC that costs one op instead of two clamps).
__device__ __forceinline__ float min3_aaa(float x, float y, float z) {
    float d;
    asm("v_min3_f32 %0, |%1|, |%2|, |%3|" : "=v"(d) : "v"(x), "v"(y), "v"(z));
    return d;
}
__device__ __forceinline__ float med3_aaa(float x, float y, float z) {
    float d;
    asm("v_med3_f32 %0, |%1|, |%2|, |%3|" : "=v"(d) : "v"(x), "v"(y), "v"(z));
    return d;
}
__device__ __forceinline__ float min3_ra(float a, float x, float y) {  // min3(a, |x|, |y|)
    float d;
    asm("v_min3_f32 %0, %1, |%2|, |%3|" : "=v"(d) : "v"(a), "v"(x), "v"(y));
    return d;
}
__device__ __forceinline__ float med3_ra(float a, float x, float y) {  // med3(a, |x|, |y|)
    float d;
    asm("v_med3_f32 %0, %1, |%2|, |%3|" : "=v"(d) : "v"(a), "v"(x), "v"(y));
    return d;
}
__device__ __forceinline__ float min_rr(float a, float b) {  // v_min_f32 without fminf's canonicalising v_max
    float d;
    asm("v_min_f32_e32 %0, %1, %2" : "=v"(d) : "v"(a), "v"(b));
    return d;
}
template <int DC, bool CAP>
__device__ __forceinline__ void two_smallest_abs3(const float (&m)[DC], float& min1, float& min2) {
    constexpr int n = DC + (CAP ? 1 : 0);
    static_assert(n >= 3, "two_smallest_abs3 needs three elements");
    const float cap = 10000.f;
    auto el = [&](int k) { return k < DC ? m[k] : cap; };  // the cap (positive) is its own |x|
    float a = min3_aaa(el(0), el(1), el(2)), b = med3_aaa(el(0), el(1), el(2));
    int k = 3;
#pragma unroll
    for (; k + 1 < n; k += 2) {
        const float md = med3_ra(a, el(k), el(k + 1));
        a = min3_ra(a, el(k), el(k + 1));
        b = min_rr(b, md);
    }
    if (k < n) {
        b = med3_a(a, b, el(k));
        a = min_a(a, el(k));
    }
    min1 = a;
    min2 = b;
}

// Float-domain form: per edge two min-tracking ops, the argmin compare with |m_k| as a modifier, the
// epilogue and the sign -- no per-edge key and no per-row key decode.  Exact zeros (the reference's
// "masked" entries: 0 counts as 10000 in the minimum, and is not positive) are rare after iteration 0; a
// row copy in which any lane of the wave sees one (min1 == 0) takes a wave-uniform branch that maps each
// 0 to -20000 (magnitude above the 10000 clamp, not positive) and tracks the minimum again.  Bit-identical
// to cn_core (tests compare the fused and streaming paths).  Measured r3/r4 alternatives, all bit-exact and
// slower on the cfg3 kernel (profiles/r3b_ab.txt, r4_ab.txt): an integer key per edge (4 %), the magnitude
// select as sat(a + b - |m|) + v_med3_u32 (48.9 -> 51.4 ms) or as min(|m|, mg2) + v_sub_u32 (51.5 ms; r6: 49.7 ms, and
// 48.5-48.8 ms -- a tie -- with each row copy's interleave pinned by sched_group_barrier, profiles/r6_ab_cfg3_cn.txt),
// signs by bit arithmetic (noise), two row copies with a packed epilogue.
template <int DC>
__device__ __forceinline__ void neural_row(float (&m)[DC], const float (&w)[DC], const float (&b)[DC]) {
    float min1, min2, mg1, mg2;
    if constexpr (DC >= 3) {
        // the minima capped at 10000 inside the tracking (even DC) or by one min each (odd DC)
        constexpr bool cap = DC % 2 == 0;
        two_smallest_abs3<DC, cap>(m, min1, min2);
        if (__builtin_expect(__builtin_amdgcn_ballot_w64(min1 == 0.f) != 0, 0)) {
#pragma unroll
            for (int k = 0; k < DC; ++k) m[k] = m[k] == 0.f ? -20000.f : m[k];
            two_smallest_abs3<DC, cap>(m, min1, min2);
        }
        mg1 = cap ? min1 : min_rr(min1, 10000.f);
        mg2 = cap ? min2 : min_rr(min2, 10000.f);
    } else {
        two_smallest_abs<DC>(m, min1, min2);
        if (__builtin_expect(__builtin_amdgcn_ballot_w64(min1 == 0.f) != 0, 0)) {
#pragma unroll
            for (int k = 0; k < DC; ++k) m[k] = m[k] == 0.f ? -20000.f : m[k];
            two_smallest_abs<DC>(m, min1, min2);
        }
        mg1 = __builtin_amdgcn_fmed3f(min1, 0.f, 10000.f);  // the masked tile entries (10000) take part
        mg2 = __builtin_amdgcn_fmed3f(min2, 0.f, 10000.f);  // in the min (min1, min2 >= 0: a clamp)
    }
    bool pos[DC];
    bool par = false;
#pragma unroll
    for (int k = 0; k < DC; ++k) {
        pos[k] = m[k] > 0.f;
        par ^= pos[k];
    }
    asm volatile("" : "+v"(mg1), "+v"(mg2));
#pragma unroll
    for (int k = 0; k < DC; ++k) {
        const float mag = fabsf(m[k]) == min1 ? mg2 : mg1;
        const float r = relu_mask(fadd(fmul(mag, w[k]), b[k]));
        m[k] = (par != pos[k]) ? r : -r;  // x * (+-1): an exact sign flip
    }
}

// Backward of the fused decoder (training): one workgroup per G codewords walks the iterations in
// reverse with dL/dc2v in registers (same ownership as the forward's c2v), reading only the saved
// v2c / clamp masks / xin and the incoming output gradients.  Weight gradients go to per-wave
// partial sums [T][nslots][E|N] reduced afterwards (nldpc_backward.hip).  vn_prefix must be 0.
struct FusedBwdArgs {
    uint32_t sig;          // kFusedBwdArgsSig (see kFusedArgsSig)
    int64_t B;
    int32_t T, qbit;
    float lo, hi;
    const float* xa;       // [B][N][Z]
    const float* w_cn;     // [T][E] or nullptr
    const float* bias;     // [T][E] (Neural) or nullptr
    const float* w_vn;     // [T][N] or nullptr
    const uint8_t* sp_plan;  // SP product order (DevGraph::sp_plan)
    TanhRef tanh;            // torch.tanh table (SP)
    const char* sv2c;      // saved [T][B][E][Z] by check copy (fp32; QMS: int8 codes); 16-byte aligned
    const uint8_t* symask; // saved [T][B][N][Z] or nullptr (Neural)
    const float* sxin;     // saved [T][B][N][Z] or nullptr
    int64_t sv2c_stride, symask_stride, sxin_stride;
    float* p_cn;           // [T][nslots][E] or nullptr
    float* p_bias;         // [T][nslots][E] or nullptr
    float* p_vn;           // [T][nslots][N] or nullptr
    float* carry;          // [B][N][Z] VN-chain carry (workspace; written before it is read)
    int64_t nslots;
    int32_t cn_tied, vn_tied;  // the MODE-5 (tied CN weight) kernel runs; vn_tied: reserved (0)
    OutPtrs gy;            // T output gradients [B][N][Z] (nullptr = zero)
    uint64_t* stamps;      // diagnostic stamp build only (make STAMPS=1): [256][waves][T][16] s_memtime
};

constexpr uint32_t kFusedBwdArgsSig = 0x4e420000u ^ ((uint32_t)sizeof(FusedBwdArgs) << 4) ^ kFusedArgsVersion;

// LDS-DMA operands (__builtin_amdgcn_global_load_lds: global source per lane, wave-uniform LDS base)
typedef __attribute__((address_space(1))) void* gptr_t;
typedef __attribute__((address_space(3))) void* lptr_t;
__device__ __forceinline__ uint32_t bload8(rsrc_t r, uint32_t vo, int so) {
    return __builtin_amdgcn_raw_buffer_load_b8(r, vo, so, 0);
}
// Where a posterior goes.  Decode kernels store it; count-only kernels (CNT) compare its hard decision
// with the codeword bit and count the difference (Functions.py:85-102 evaluate_ber_fer on every
// iteration's output, without writing the T posteriors).
struct PostSink {
    rsrc_t yr;  // codeword bits [N][Z] per codeword (empty descriptor: all-zero codeword)
    int ec;     // this thread's bit errors of the iteration being completed
    int conv;
    // the errors of iteration `it` into this codeword's LDS counters (two iterations per word)
    __device__ __forceinline__ void flush(int* cntl, int it) {
        if (ec) atomicAdd(cntl + (it >> 1), ec << ((it & 1) * 16));
        ec = 0;
    }
    // same, when the whole wave belongs to one codeword: one LDS atomic per wave
    __device__ __forceinline__ void flush_wave(int* cntl, int it);
};
// CM 0: store; 1: count against the all-zero codeword in the decoder convention (bit = LLR > 0: one
// compare and one add-with-carry per posterior, the BER-sweep case); 2: any convention, against y
// when given (its loads cost registers the decoder state needs, hence a kernel variant of its own)
template <int CM>
__device__ __forceinline__ void put_post(rsrc_t pr, uint32_t vo, int so, float v, PostSink& ps) {
    if constexpr (CM == 0) {
        bstore(pr, vo, so, v);
    } else if constexpr (CM == 1) {
        ps.ec += v > 0.f ? 1 : 0;
    } else {
        const uint32_t bit = ps.conv ? (v < 0.f) : (v > 0.f);
        uint32_t y = 0u;
        // byte offset of the bit = float offset / 4; the sum first: a rotated copy's lane offset can
        // wrap below zero (vo + (-4Z)), which only the 32-bit total undoes
        if constexpr (CM == 2) y = __builtin_amdgcn_raw_buffer_load_b8(ps.yr, (vo + (uint32_t)so) >> 2, 0, 0) & 1u;
        ps.ec += (int)(bit ^ y);
    }
}
// end of a count-only decode: iteration it of the workgroup's nlive codewords -> the global counters
// (summed over the workgroup first: two global atomics per iteration and workgroup)
__device__ __forceinline__ void count_iteration(const FusedArgs& a, const int* cnt_all, int nlive, int it) {
    unsigned long long bits = 0, frames = 0;
    for (int g = 0; g < nlive; ++g) {
        const unsigned v = ((unsigned)cnt_all[g * 32 + (it >> 1)] >> ((it & 1) * 16)) & 0xFFFFu;
        bits += v;
        frames += v != 0;
    }
    if (bits) {
        atomicAdd(a.cnt + 2 * it, bits);
        atomicAdd(a.cnt + 2 * it + 1, frames);
    }
}
// dL/dy of one variable copy through the Boosted output clamp (mask saved by the forward)
template <int KIND>
__device__ __forceinline__ float gy_masked(rsrc_t gr, rsrc_t mr, uint32_t vo, uint32_t vm, int so) {
    const float g = bload(gr, vo, so);
    if (KIND == NLDPC_NEURAL) return g;
    return bload8(mr, vm, so >> 2) ? g : 0.f;
}
// r6 backward cache policy (gen_fused.py NLDPC_GEN_BWDCACHE, default on): streams read once per iteration loaded
// non-temporal, so that they do not evict the VN-weight carry the next iteration reads back; the carry stored temporal
__device__ __forceinline__ float bload_nt(rsrc_t r, uint32_t vo, int so) {
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, vo, so, 2));
}
template <int KIND>
__device__ __forceinline__ float gy_masked_nt(rsrc_t gr, rsrc_t mr, uint32_t vo, uint32_t vm, int so) {
    const float g = bload_nt(gr, vo, so);
    if (KIND == NLDPC_NEURAL) return g;
    return __builtin_amdgcn_raw_buffer_load_b8(mr, vm, so >> 2, 2) ? g : 0.f;
}
__device__ __forceinline__ void bstore_keep(rsrc_t r, uint32_t vo, int so, float v) {
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), r, vo, so, 0);
}
// Sum over the 64 lanes of a wave (wave-uniform result): DPP within rows of 16 (quad permutes, then the
// half-row and row mirrors), then the gfx9 row broadcasts 15 / 31 carry the row sums up to lane 63,
// read back with v_readlane -- all VALU, no LDS traffic (__shfl_xor issues a ds_bpermute per step).
template <int CTRL, int ROW_MASK = 0xf>
__device__ __forceinline__ float dpp_mov(float x) {
    return __builtin_bit_cast(float,
                              __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), CTRL, ROW_MASK, 0xf, false));
}
__device__ __forceinline__ float wave_sum(float x) {
    x += dpp_mov<0xB1>(x);        // quad_perm [1,0,3,2]
    x += dpp_mov<0x4E>(x);        // quad_perm [2,3,0,1]: quad sums
    x += dpp_mov<0x141>(x);       // row_half_mirror: 8-lane sums
    x += dpp_mov<0x140>(x);       // row_mirror: every lane holds its row's (16-lane) sum
    x += dpp_mov<0x142, 0xa>(x);  // row_bcast:15 into rows 1, 3: rows 0+1 | 2+3
    x += dpp_mov<0x143, 0xc>(x);  // row_bcast:31 into rows 2, 3: lane 63 = the wave's sum
    return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, x), 63));
}
__device__ __forceinline__ void PostSink::flush_wave(int* cntl, int it) {
    const int s = (int)wave_sum((float)ec);  // exact: counts below 2^24
    if ((threadIdx.x & 63) == 0 && s) atomicAdd(cntl + (it >> 1), s << ((it & 1) * 16));
    ec = 0;
}

// Boosted MS / QMS (active quantiser) check node of one check copy in place, specialised like
// neural_row: cn_core + cn_epilogue's values (Boosted…py:386-423, 431-512) with the conditioning as
// one med3 (MS clamp) or quantize_active (QMS), the zero fix as a select (x + 1e-4*(x==0)), the two
// smallest magnitudes on the integer key bits(x) << 1 (every conditioned input is nonzero), the
// 1e-4 correction of a tiny minimum applied once per row, and sign(x_output_0) * clip/Q(relu(|x|*w))
// as one sign select.  Results equal cn_core + cn_epilogue (a zero c2v may differ in its sign bit
// only, which no sum of the decoder can observe).  ~19 VALU per edge copy instead of ~45.
template <int DC, int KIND>
__device__ __forceinline__ void boosted_row_keys(float (&m)[DC], const float (&w)[DC], bool has_w, const QParams& qp, float lo,
                                                 float hi, bool ucn, float uf, const float (&wu)[DC]) {
    constexpr uint32_t kInit = 0x461C4000u << 1;  // key of 10000.f
    uint32_t key[DC];
    bool pos[DC];
    bool par = false;
#pragma unroll
    for (int k = 0; k < DC; ++k) {
        float x = KIND == NLDPC_QMS ? quantize_active_p(m[k], qp) : __builtin_amdgcn_fmed3f(m[k], lo, hi);
        x = x == 0.f ? kZeroFix : x;
        key[k] = __builtin_bit_cast(uint32_t, x) << 1;
        pos[k] = x > 0.f;
        par ^= pos[k];
    }
    uint32_t min1, min2;
    two_smallest<DC>(key, min1, min2);
    min1 = min(min1, kInit);
    min2 = min(min2, kInit);
    float mg1 = __builtin_bit_cast(float, min1 >> 1);
    float mg2 = __builtin_bit_cast(float, min2 >> 1);
    mg1 = mg1 > kZeroFix ? mg1 : fadd(mg1, -kZeroFix);
    mg2 = mg2 > kZeroFix ? mg2 : fadd(mg2, -kZeroFix);
    // MS: a minimum below 1e-4 turns negative here (x_output_0 = mag * sign flips its sign); QMS
    // magnitudes are 1e-4 or multiples of the grid step, so they stay >= 0
    bool n1 = false, n2 = false;
    if (KIND == NLDPC_MS) {
        n1 = mg1 < 0.f;
        n2 = mg2 < 0.f;
        mg1 = fabsf(mg1);
        mg2 = fabsf(mg2);
    }
    asm volatile("" : "+v"(mg1), "+v"(mg2));  // once per row, not after every per-edge select
#pragma unroll
    for (int k = 0; k < DC; ++k) {
        const bool sel = key[k] == min1;
        const float mag = sel ? mg2 : mg1;
        // with UCN: (|x| w_cn)(1 - u) + (|x| w_ucn) u, the reference's arithmetic (Boosted…py:436-488)
        const float x1 = !has_w ? mag
                         : (ucn ? fadd(fmul(fmul(mag, w[k]), fadd(-uf, 1.f)), fmul(fmul(mag, wu[k]), uf))
                                : fmul(mag, w[k]));
        const float x2 = relu_mask(x1);
        const float x3 = KIND == NLDPC_QMS ? quantize_active_p(x2, qp) : __builtin_amdgcn_fmed3f(x2, lo, hi);
        const bool neg = KIND == NLDPC_MS && (sel ? n2 : n1);
        m[k] = ((par != pos[k]) != neg) ? x3 : -x3;
    }
}

// Float-domain form of boosted_row (r2), the two smallest of |m| tracked with |m| as a source modifier
// as in neural_row (2 VALU per edge), no per-edge conditioning, zero fix or key.  What makes the raw
// magnitudes enough: each edge's c2v magnitude is "min over the OTHER edges" of the conditioned values,
// and min over others commutes with any non-decreasing map of |m|:
//  * MS with a symmetric clip (lo == -hi): |clamp(m)| = min(|m|, hi).  The zero fix (0 -> 1e-4) is not
//    monotone, and a minimum <= 1e-4 changes sign in the magnitude correction, so a row copy in which
//    any lane of the wave has min1 <= 1e-4 (exact zeros: punctured columns in the first iteration) takes
//    the key form above (wave-uniform branch).
//  * active QMS: Q is odd and non-decreasing, |Q(m)| = Q(|m|); the zero fix maps Q's 0 to 1e-4 and the
//    magnitude correction maps 1e-4 back to 0 (every nonzero Q value is >= the 0.5 grid step), so the
//    magnitude is Q(min over others |m|) in every case.  pos_k = Q(m_k) >= 0 (zeros are fixed to +1e-4)
//    = m_k >= -0.5 / s (the scaling by s is exact).
// The epilogue clip/Q(relu(.)) is one med3 (relu folds into the lower bound); UCN flags are 0/1, so
// the reference's (|x| w)(1 - u) + (|x| w_u) u is exactly |x| w or |x| w_u (a select).  DC == 1 rows
// (the masked 10000 would be the magnitude) keep the key form.  Equal to boosted_row_keys up to the
// sign bit of a zero c2v, which no sum of the decoder observes.
// TIED (the tied saving forward, MODE 5: one CN weight per row, w[k] == w[0], 1.f without weights, no UCN): every edge's
// epilogue is one of two values -- the magnitudes mg1 / mg2 times the one weight, clipped or quantised -- computed once
// per row copy from the same operands (bit-identical), so an edge costs the two selects only (r6).
#ifndef NLDPC_TIEDROW
#define NLDPC_TIEDROW 1
#endif
template <int DC, int KIND, bool TIED = false>
__device__ __forceinline__ void boosted_row(float (&m)[DC], const float (&w)[DC], bool has_w, const QParams& qp, float lo,
                                            float hi, bool ucn, float uf, const float (&wu)[DC], bool ufb) {
    if constexpr (DC >= 2) {
        float min1, min2;
        if constexpr (DC >= 3) two_smallest_abs3<DC, false>(m, min1, min2);
        else two_smallest_abs<DC>(m, min1, min2);
        bool fast = true;
        if constexpr (KIND == NLDPC_MS)
            fast = lo == -hi && hi > kZeroFix && __builtin_amdgcn_ballot_w64(min1 <= kZeroFix) == 0;
        if (__builtin_expect(fast, 1)) {
            float mg1, mg2, thr, top, inv;
            if constexpr (KIND == NLDPC_MS) {
                mg1 = fminf(min1, hi);
                mg2 = fminf(min2, hi);
                thr = 0.f;
                top = hi;
                inv = 1.f;
            } else {
                const float s = qp.s;
                inv = qp.inv;
                top = qp.hs;  // hi * s
                // s * Q(min) = min(rint(min s), hi s): the magnitude pre-scaled by s, so the per-edge
                // product (s mag) w = s (mag w) exactly and Q's own scaling needs no multiply
                mg1 = fminf(rintf(fmul(min1, s)), top);
                mg2 = fminf(rintf(fmul(min2, s)), top);
                thr = fmul(-0.5f, inv);
            }
            asm volatile("" : "+v"(mg1), "+v"(mg2));
            const float lo0 = KIND == NLDPC_MS ? fmaxf(lo, 0.f) : 0.f;
            bool pos[DC];
            bool par = false;
#pragma unroll
            for (int k = 0; k < DC; ++k) {
                pos[k] = KIND == NLDPC_MS ? m[k] > 0.f : m[k] >= thr;
                par ^= pos[k];
            }
            if constexpr (TIED && NLDPC_TIEDROW) {
                // (w[0] is 1.f without weights: mag * 1 == mag, the !has_w value)
                auto epi = [&](float mag) {
                    const float x1 = fmul(mag, w[0]);
                    return KIND == NLDPC_MS ? __builtin_amdgcn_fmed3f(x1, lo0, top)
                                            : fmul(__builtin_amdgcn_fmed3f(rintf(x1), 0.f, top), inv);
                };
                const float x3a = epi(mg1), x3b = epi(mg2);
#pragma unroll
                for (int k = 0; k < DC; ++k) {
                    const float x3 = fabsf(m[k]) == min1 ? x3b : x3a;
                    m[k] = (par != pos[k]) ? x3 : -x3;
                }
                return;
            }
            // (r6) the weights are 1.f without a CN weight (the kernels' preload), and mag * 1 == mag: no per-edge select of
            // the unweighted value; the UCN weight only with CN weights (the reference's CN sharing 0 ignores UCN)
            const bool uw = ucn && has_w && ufb;  // (ufb == (uf != 0): the flag as the lane mask it was computed as)
#pragma unroll
            for (int k = 0; k < DC; ++k) {
                const float mag = fabsf(m[k]) == min1 ? mg2 : mg1;
                // (a wave-uniform branch to the plain weights when no copy is unsatisfied, i.e. two versions
                // of this loop, measured 15 % slower: code size)
                float x1;
                if constexpr (NLDPC_TIEDROW) {
                    // (r6) both products, then the select: a multiply takes its SGPR weight directly, where a select of
                    // the two SGPR weights first moved both into VGPRs (two v_mov per edge copy); the fence keeps the
                    // compiler from folding the select back into the multiply
                    float xw = fmul(mag, w[k]);
                    const float xu = fmul(mag, wu[k]);
                    asm volatile("" : "+v"(xw));
                    x1 = uw ? xu : xw;
                } else {
                    x1 = !has_w ? mag : fmul(mag, (ucn && uf != 0.f) ? wu[k] : w[k]);
                }
                float x3;
                if constexpr (KIND == NLDPC_MS) x3 = __builtin_amdgcn_fmed3f(x1, lo0, top);
                else x3 = fmul(__builtin_amdgcn_fmed3f(rintf(x1), 0.f, top), inv);
                m[k] = (par != pos[k]) ? x3 : -x3;
            }
            return;
        }
    }
    boosted_row_keys<DC, KIND>(m, w, has_w, qp, lo, hi, ucn, uf, wu);
}

// check node of one check copy in place (m: gathered v2c -> c2v), every kind: Neural through the
// specialised neural_row, MS / QMS through boosted_row, SP through the shared cn_core + cn_epilogue
// bv: Neural biases, or (Boosted with UCN) the UCN weights; uf: the copy's UCN flag
// NOUCN: the kernel variant without UCN and with one CN weight per row (the tied saving forward, MODE 5): the UCN
// branch is not compiled and the row's epilogue is computed once (boosted_row TIED)
// ucn_on: the kernel's UCN flag (a.ucn, or a constant in the specialised kernels); ufb: uf != 0 (uf is 0 or 1)
template <int KIND, int DC, bool NOUCN = false>
__device__ __forceinline__ void cn_copy(float (&m)[DC], const float (&wv)[DC], const float (&bv)[DC],
                                        const FusedArgs& a, bool has_w, int row, float uf, bool ucn_on, bool ufb) {
    if constexpr (KIND == NLDPC_NEURAL) {
        neural_row<DC>(m, wv, bv);
    } else if constexpr (KIND == NLDPC_MS || KIND == NLDPC_QMS) {
        // QMS reaches the fused kernels only with an active quantiser (fused_eligible): the generic
        // cn_core is not compiled into them (it had made the QMS kernels 6x the code of the MS ones)
        boosted_row<DC, KIND, NOUCN>(m, wv, has_w, a.qp, a.lo, a.hi, !NOUCN && ucn_on, uf, bv, ufb);
    } else {
        CnCore<DC> core;
        cn_core<DC, KIND>(m, DC, a.qbit, a.lo, a.hi, core, SpRow{a.sp_plan + row * kSpPlanBytes, a.tanh});
        if (ucn_on) {
#pragma unroll
            for (int k = 0; k < DC; ++k)
                m[k] = cn_epilogue<KIND, true>(core.out0[k], wv[k], bv[k], 0.f, uf, has_w, true, a.qbit, a.lo, a.hi).c;
        } else {
#pragma unroll
            for (int k = 0; k < DC; ++k)
                m[k] = cn_epilogue<KIND, false>(core.out0[k], wv[k], 0.f, 0.f, 0.f, has_w, false, a.qbit, a.lo, a.hi).c;
        }
    }
}

struct FusedSpec {
    const char* tag;
    int32_t M, N, Z, E, G, threads;
    const int32_t* basegraph;  // [M*N]
    void* kernels[4][4];       // [MODE: decode / save / count / count against y][nldpc_kind]
    void* bwd[4];              // backward kernels [nldpc_kind]
    int32_t waves_per_part;    // partial-sum slots per workgroup
    void* bwd_tied[4];         // backward kernels for tied CN / VN weights (MODE 5 in fused_launch), or nullptr
    uint32_t sig[6];           // the argument layout each MODE's unit was built for (kFusedArgsSig / kFusedBwdArgsSig):
                               // fused_launch refuses a kernel whose layout differs from the launcher's
    void* save_tied[4];        // (r6) saving forward for one CN weight per iteration and no UCN (MODE 6 in fused_launch;
                               // the generated kernel<KIND, 5>), or nullptr; built in the saving unit (sig[1])
    void* decode_ucnw[4];      // (r6) decode with UCN and CN / UCN / cumulative VN weights all given (MODE 7 in
                               // fused_launch; the generated kernel<KIND, 6>), or nullptr; built in the decode unit (sig[0])
};

const FusedSpec* fused_specs(int* n);

// How to launch the register-resident kernel of (graph, MODE, kind) (MODE 4: the backward; MODE 5: the
// backward for tied weights; MODE 6: the saving forward for tied CN weights without UCN; MODE 7: the decode with UCN
// and CN / UCN / cumulative VN weights -- MODES 5 to 7 library kernels only, a run-time compiled graph uses MODE 4 / 1): one compiled
// into the library (fused_specs table, hipLaunchKernel) or one compiled at run time for this graph and
// attached (nldpc_graph_attach_kernel, hipModuleLaunchKernel); empty when neither exists.
struct FusedLaunch {
    const void* host = nullptr;
    hipFunction_t fn = nullptr;
    int32_t G = 0, threads = 0, waves_per_part = 0;
    explicit operator bool() const { return host != nullptr || fn != nullptr; }
    hipError_t launch(int64_t blocks, void** args, hipStream_t s) const {
        if (fn) return hipModuleLaunchKernel(fn, (unsigned)blocks, 1, 1, (unsigned)threads, 1, 1, 0, s, args, nullptr);
        return hipLaunchKernel(host, dim3((unsigned)blocks), dim3((unsigned)threads), args, 0, s);
    }
};
FusedLaunch fused_launch(const nldpc_graph* g, int mode, int kind);

}  // namespace nldpc
