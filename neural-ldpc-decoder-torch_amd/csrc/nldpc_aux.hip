// The steps either side of the decode path:
//   nldpc_awgn_llr   synthetic BPSK/AWGN channel LLRs generated in HBM (Philox-4x32-10 + Box-Muller)
//   nldpc_ber_count  fused bit/frame error counting of a posterior (Functions.evaluate_ber_fer)
//   nldpc_bce_loss / nldpc_bce_grad  the multi-iteration BCE training loss and its gradient
//                    (LDPCDecoderLoss.py:70-108), one pass over all T outputs each
//   nldpc_hbm_probe  the measured HBM ceilings the bench's roofline quotes beside the 8 TB/s spec
#include <hip/hip_runtime.h>

#include "nldpc_internal.h"
#include "nldpc_math.h"

namespace nldpc {

// ---------------------------------------------------------------- Philox-4x32-10 (Salmon et al. 2011)
struct U4 {
    uint32_t x, y, z, w;
};

__device__ __forceinline__ U4 philox4x32_10(U4 c, uint32_t k0, uint32_t k1) {
    constexpr uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u, W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint32_t hi0 = __umulhi(M0, c.x), lo0 = M0 * c.x;
        const uint32_t hi1 = __umulhi(M1, c.z), lo1 = M1 * c.z;
        c = U4{hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
        k0 += W0;
        k1 += W1;
    }
    return c;
}

__device__ __forceinline__ double u01(uint32_t r) { return ((double)r + 1.0) * (1.0 / 4294967296.0); }

// one thread = 4 consecutive elements of the global (b_offset + b) * L + n stream
// Channel options beyond the all-zero codeword (F1; AWGNPassedDatagen.py:75-134): the codeword bits y
// (BPSK (-1)^(1-y)), and the punctured / shortened bit ranges [start-1, end) of every codeword set to a
// constant after the quantiser (the reference's order).  start = 0: no range.
struct ChannelOpts {
    const uint8_t* y;  // [B][L] or nullptr
    int64_t L, p0, p1, s0, s1;
    float pval, sval;
};

__global__ __launch_bounds__(256) void awgn_kernel(float* xa, int64_t total, int64_t first, double sigma,
                                                   uint64_t seed, int qbit, ChannelOpts o) {
    const int64_t g4 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;  // local group of 4
    const int64_t g0 = (first >> 2) + g4;                                 // global group index
    const int64_t e0 = g0 * 4;
    if (e0 >= first + total) return;
    U4 r = philox4x32_10(U4{(uint32_t)g0, (uint32_t)(g0 >> 32), 0u, 0u}, (uint32_t)seed, (uint32_t)(seed >> 32));
    const double rad0 = sqrt(-2.0 * log(u01(r.x))), th0 = 6.283185307179586 * u01(r.y);
    const double rad1 = sqrt(-2.0 * log(u01(r.z))), th1 = 6.283185307179586 * u01(r.w);
    const double n[4] = {rad0 * cos(th0), rad0 * sin(th0), rad1 * cos(th1), rad1 * sin(th1)};
    const double s2 = sigma * sigma;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int64_t e = e0 + q;
        if (e < first || e >= first + total) continue;
        // BPSK bit 0 -> -1, 1 -> +1 (AWGNPassedDatagen.py:97-103), LLR = 2 y / sigma^2
        const int64_t i = e - first;
        const double bpsk = (o.y && o.y[i]) ? 1.0 : -1.0;
        float llr = (float)(2.0 * (bpsk + sigma * n[q]) / s2);
        if (qbit) llr = quantize(llr, qbit);
        const int64_t k = i % o.L;  // bit index within the codeword
        if (k >= o.p0 && k < o.p1) llr = o.pval;
        if (k >= o.s0 && k < o.s1) llr = o.sval;
        xa[i] = llr;
    }
}

__global__ __launch_bounds__(256) void ber_kernel(const float* llr, const uint8_t* y, int64_t B, int64_t L,
                                                  int convention, unsigned long long* counts) {
    __shared__ unsigned long long s_bits[4];
    __shared__ int s_frame[4];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    unsigned long long bits_acc = 0;
    unsigned long long frames_acc = 0;
    for (int64_t b = blockIdx.x; b < B; b += gridDim.x) {
        unsigned long long cnt = 0;
        const float* row = llr + b * L;
        const uint8_t* yr = y ? y + b * L : nullptr;
        for (int64_t n = threadIdx.x; n < L; n += blockDim.x) {
            const float x = row[n];
            const int bit = convention == 0 ? (x > 0.f) : (x < 0.f);
            const int ref = yr ? (yr[n] != 0) : 0;
            cnt += (bit != ref);
        }
        // wave reduce (64 lanes)
        for (int off = 32; off > 0; off >>= 1) cnt += __shfl_down(cnt, off, 64);
        if (lane == 0) s_bits[wid] = cnt;
        __syncthreads();
        if (threadIdx.x == 0) {
            unsigned long long t = 0;
            for (int w = 0; w < (int)(blockDim.x >> 6); ++w) t += s_bits[w];
            bits_acc += t;
            frames_acc += (t > 0);
        }
        __syncthreads();
    }
    (void)s_frame;
    if (threadIdx.x == 0) {
        atomicAdd(&counts[0], bits_acc);
        atomicAdd(&counts[1], frames_acc);
    }
}

// ---------------------------------------------------------------- multi-iteration BCE loss
constexpr int kBceMaxK = 64;
constexpr int kBceBlocks = 16384;  // element blocks (workgroups) of the loss pass
struct BceArgs {
    const float* x[kBceMaxK];
    float coef[kBceMaxK];
    int32_t K;
};

// torch.nn.functional.binary_cross_entropy_with_logits term: (1 - t) * x - log_sigmoid(x)
__device__ __forceinline__ float bce_term(float x, float t) {
    const float ls = fminf(x, 0.f) - log1pf(expf(-fabsf(x)));
    return (1.f - t) * x - ls;
}

// One workgroup per element block, every term: each thread reads its labels once and the K logits at
// the same positions (16 B loads), and sums coef_k * term in fp64 (fp32 terms, as torch's); the finish
// kernel adds the per-block partial sums in a fixed order (deterministic) and divides by n.  (r2 read
// the labels once per term, twice the bytes at cfg5: 6.7 ms for 8.2 GB of logits.)  r3: the pass is
// bound by the latency of its dependent chains (exp -> log1p -> fp64 sum), not by HBM: 8x the
// element blocks (about two float4 of every term per thread) and two fp64 accumulators (even / odd
// terms): 7.4 -> 7.0 ms at cfg5; then the grid table above.
// Logits on the half-integer grid (every QMS decoder output is one: Q(xa) plus quantised check messages,
// clamped to the QMS range) with a 0/1 label take their term from a per-block table of bce_term at
// those grid points -- the same function at the same argument, so the same fp32 value -- instead of
// exp + log1p per element (the pass was bound by that arithmetic: cfg5 7.0 ms for 8.2 GB).  Any other
// logit or label computes the term.
constexpr int kBceGrid = 64;  // table covers x = k/2, |k| <= kBceGrid
__device__ __forceinline__ float bce_term_tab(float x, float t, const float (*tab)[2 * kBceGrid + 1]) {
    const float k2 = x * 2.f;  // exact
    if (k2 == rintf(k2) && fabsf(k2) <= (float)kBceGrid && (t == 0.f || t == 1.f))
        return tab[t == 1.f][(int)k2 + kBceGrid];
    return bce_term(x, t);
}

// GRAD: the same pass also writes every term's gradient for a unit seed (dL/dloss = 1, what
// loss.backward() sends), grads[k][i] = (coef[k] / n) * (sigmoid(x) - t) -- bce_grad_kernel's expression
// with *gseed = 1, so the same bits -- reading the logits once for both directions instead of twice
// (cfg5: the separate gradient pass re-read 8.2 GB of logits and took 3.7 ms).  The sigmoid of a grid logit
// comes from a table of the same expression, as the term does.
__device__ __forceinline__ float bce_sig(float x) { return 1.f / (1.f + expf(-x)); }
__device__ __forceinline__ float bce_sig_tab(float x, const float* tab) {
    const float k2 = x * 2.f;
    if (k2 == rintf(k2) && fabsf(k2) <= (float)kBceGrid) return tab[(int)k2 + kBceGrid];
    return bce_sig(x);
}

template <bool GRAD>
__global__ __launch_bounds__(256) void bce_loss_kernel(BceArgs a, const float* __restrict__ target, int64_t n,
                                                       double* __restrict__ part, BceArgs g) {
    __shared__ double red[4];
    __shared__ float tab[2][2 * kBceGrid + 1];
    __shared__ float stab[GRAD ? 2 * kBceGrid + 1 : 1];
    for (int i = threadIdx.x; i < 2 * (2 * kBceGrid + 1); i += blockDim.x) {
        const int lab = i / (2 * kBceGrid + 1), k = i % (2 * kBceGrid + 1) - kBceGrid;
        tab[lab][k + kBceGrid] = bce_term(0.5f * (float)k, (float)lab);
        if (GRAD && lab == 0) stab[k + kBceGrid] = bce_sig(0.5f * (float)k);
    }
    __syncthreads();
    const float scale = 1.f / (float)n;  // bce_grad_kernel's *gseed / (float)n at *gseed = 1
#define bce_term(x, t) bce_term_tab((x), (t), tab)
    // one term's gradient for four elements
    auto grad4 = [&](int k, const float4& v, const float4& t, int64_t i) {
        if constexpr (GRAD) {
            const float c = scale * a.coef[k];
            float4 r;
            r.x = c * (bce_sig_tab(v.x, stab) - t.x);
            r.y = c * (bce_sig_tab(v.y, stab) - t.y);
            r.z = c * (bce_sig_tab(v.z, stab) - t.z);
            r.w = c * (bce_sig_tab(v.w, stab) - t.w);
            reinterpret_cast<float4*>(const_cast<float*>(g.x[k]))[i] = r;
        }
    };
    double acc0 = 0.0, acc1 = 0.0;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    const int64_t i0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    bool vec = (reinterpret_cast<uintptr_t>(target) & 15) == 0;
    for (int k = 0; k < a.K; ++k) {
        vec = vec && (reinterpret_cast<uintptr_t>(a.x[k]) & 15) == 0;
        if (GRAD) vec = vec && (reinterpret_cast<uintptr_t>(g.x[k]) & 15) == 0;
    }
    const int64_t n4 = vec ? n / 4 : 0;
    for (int64_t i = i0; i < n4; i += stride) {
        const float4 t = target ? reinterpret_cast<const float4*>(target)[i] : make_float4(0.f, 0.f, 0.f, 0.f);
        int k = 0;
        for (; k + 1 < a.K; k += 2) {
            const float4 v = reinterpret_cast<const float4*>(a.x[k])[i];
            const float4 u = reinterpret_cast<const float4*>(a.x[k + 1])[i];
            acc0 += (double)a.coef[k] * (((double)bce_term(v.x, t.x) + (double)bce_term(v.y, t.y)) +
                                         ((double)bce_term(v.z, t.z) + (double)bce_term(v.w, t.w)));
            acc1 += (double)a.coef[k + 1] * (((double)bce_term(u.x, t.x) + (double)bce_term(u.y, t.y)) +
                                             ((double)bce_term(u.z, t.z) + (double)bce_term(u.w, t.w)));
            grad4(k, v, t, i);
            grad4(k + 1, u, t, i);
        }
        if (k < a.K) {
            const float4 v = reinterpret_cast<const float4*>(a.x[k])[i];
            acc0 += (double)a.coef[k] * (((double)bce_term(v.x, t.x) + (double)bce_term(v.y, t.y)) +
                                         ((double)bce_term(v.z, t.z) + (double)bce_term(v.w, t.w)));
            grad4(k, v, t, i);
        }
    }
    for (int64_t i = 4 * n4 + i0; i < n; i += stride) {
        const float t = target ? target[i] : 0.f;
        for (int k = 0; k < a.K; ++k) {
            const float x = a.x[k][i];
            acc0 += (double)a.coef[k] * (double)bce_term(x, t);
            if (GRAD) const_cast<float*>(g.x[k])[i] = (scale * a.coef[k]) * (bce_sig_tab(x, stab) - t);
        }
    }
#undef bce_term
    double acc = acc0 + acc1;
    for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) part[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

// fixed-order sum of the block partials: 64 lanes each add a contiguous slice, lane 0 adds the slices
__global__ __launch_bounds__(64) void bce_finish_kernel(const double* __restrict__ part, int nb, int64_t n,
                                                        float* __restrict__ loss, int accumulate) {
    __shared__ double sl[64];
    const int per = (nb + 63) / 64;
    double s = 0.0;
    for (int b = threadIdx.x * per; b < nb && b < (int)(threadIdx.x + 1) * per; ++b) s += part[b];
    sl[threadIdx.x] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        double t = 0.0;
        for (int l = 0; l < 64; ++l) t += sl[l];
        const float v = (float)(t / (double)n);
        *loss = accumulate ? *loss + v : v;
    }
}

// UNLESS_UNIT: the gradients of a unit seed are already in g (bce_loss_kernel<true>); recompute only when
// the seed that arrived is not 1 (read on the device: no host synchronisation)
template <bool UNLESS_UNIT>
__global__ __launch_bounds__(256) void bce_grad_kernel(BceArgs a, const float* __restrict__ target, int64_t n,
                                                       const float* __restrict__ gseed, BceArgs g) {
    if (UNLESS_UNIT && *gseed == 1.f) return;
    const float scale = *gseed / (float)n;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const float t = target ? target[i] : 0.f;
        for (int k = 0; k < a.K; ++k) {
            const float sg = 1.f / (1.f + expf(-a.x[k][i]));
            const_cast<float*>(g.x[k])[i] = (scale * a.coef[k]) * (sg - t);
        }
    }
}

// ---------------------------------------------------------------- HBM ceiling probes (bench.py roofline)
// kind 0: stream copy (read + write), 1: write-only fill (the decoder's traffic is ~95 % posterior writes), 2: read
// only (one partial sum per workgroup is written so the loads are live): 16 B per lane, each workgroup moving tiles of
// 256 lanes x kUnroll float4 (every load of a tile issued before its first use, 8 loads in flight per lane;
// non-temporal, as the decoder's posterior stores), grid-stride over the tiles.  VERDICT r5: the r5 probe (one float4
// per lane and trip) measured copy 4.8 TB/s against the guide's 6.29 TB/s float4 copy; r6 sweep (28 configurations,
// tools/dev/hbm_probe_sweep.hip): copy tops out at 5.2-5.5 TB/s on this box in every form.  kind 3: read only with 4 B
// per lane, the decoder's own load width (calibrates the FETCH_SIZE counter for those loads; kept as it was).
constexpr int kProbeUnroll = 8;
typedef float probe_v4 __attribute__((ext_vector_type(4)));  // (the nontemporal builtins take native vectors)
__global__ __launch_bounds__(256) void hbm_probe_kernel(int kind, float4* __restrict__ dst4,
                                                        const float4* __restrict__ src4, int64_t n4) {
    constexpr int64_t TILE = 256 * kProbeUnroll;
    probe_v4* dst = reinterpret_cast<probe_v4*>(dst4);
    const probe_v4* src = reinterpret_cast<const probe_v4*>(src4);
    const int64_t ntiles = n4 / TILE;
    float acc = 0.f;
    if (kind <= 2) {
        for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
            const int64_t base = t * TILE + threadIdx.x;
            if (kind == 1) {  // (plain stores: 5.82 TB/s against 5.67 non-temporal, profiles/r6_hbm_probe_sweep.txt)
                const probe_v4 v = {1.f, 2.f, 3.f, 4.f};
#pragma unroll
                for (int k = 0; k < kProbeUnroll; ++k) dst[base + k * 256] = v;
                continue;
            }
            probe_v4 v[kProbeUnroll];
#pragma unroll
            for (int k = 0; k < kProbeUnroll; ++k) v[k] = __builtin_nontemporal_load(src + base + k * 256);
            if (kind == 0) {
#pragma unroll
                for (int k = 0; k < kProbeUnroll; ++k) __builtin_nontemporal_store(v[k], dst + base + k * 256);
            } else {
#pragma unroll
                for (int k = 0; k < kProbeUnroll; ++k) acc += (v[k].x + v[k].y) + (v[k].z + v[k].w);
            }
        }
        // the tail past the last whole tile (n4 % TILE float4), one float4 per lane
        for (int64_t i = ntiles * TILE + (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
            if (kind == 0) dst[i] = src[i];
            else if (kind == 1) dst[i] = probe_v4{1.f, 2.f, 3.f, 4.f};
            else acc += (src[i].x + src[i].y) + (src[i].z + src[i].w);
        }
        if (kind != 2) return;
    } else {
        const int64_t stride = (int64_t)gridDim.x * blockDim.x;
        const float* s1 = reinterpret_cast<const float*>(src4);
        for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < 4 * n4; i += stride) acc += s1[i];
    }
    __shared__ float red[256];
    red[threadIdx.x] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        float s = 0.f;
        for (int k = 0; k < 256; ++k) s += red[k];
        dst4[blockIdx.x] = make_float4(s, 0.f, 0.f, 0.f);
    }
}

}  // namespace nldpc

using namespace nldpc;

extern "C" int nldpc_hbm_probe(int32_t kind, float* dst, const float* src, int64_t n, void* stream) {
    if (kind < 0 || kind > 3 || !dst || (kind != 1 && !src) || n <= 0 || (n & 3))
        return fail(NLDPC_EINVAL, "nldpc_hbm_probe: bad argument");
    const int64_t n4 = n >> 2;
    // kinds 0-2: workgroups of 256 looping over 32 KB tiles, 16 per CU for copy / write, 2 for read (the best of the
    // r6 sweep, profiles/r6_hbm_probe_sweep.txt); kind 3: 32 per CU (the r2 calibration)
    const int blocks = kind == 3 ? 256 * 32 : kind == 2 ? 256 * 2 : 256 * 16;
    hipLaunchKernelGGL(hbm_probe_kernel, dim3(blocks), dim3(256), 0, static_cast<hipStream_t>(stream), kind,
                       reinterpret_cast<float4*>(dst), reinterpret_cast<const float4*>(src), n4);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? NLDPC_OK : hip_fail(e, "hbm_probe_kernel launch");
}

extern "C" int nldpc_bce_workspace(int64_t n, int32_t K, size_t* bytes) {
    if (!bytes || n <= 0 || K <= 0) return fail(NLDPC_EINVAL, "nldpc_bce_workspace: bad argument");
    *bytes = (size_t)kBceBlocks * sizeof(double);
    return NLDPC_OK;
}

static int bce_blocks(int64_t n) {  // ~2 float4 of every term per thread, at most kBceBlocks element blocks
    const int64_t b = (n + 256 * 8 - 1) / (256 * 8);
    return (int)(b < 1 ? 1 : (b < kBceBlocks ? b : kBceBlocks));
}

extern "C" int nldpc_bce_loss(const float* const* logits, int32_t K, const float* coef, const float* target, int64_t n,
                              float* loss, void* work, size_t work_bytes, void* stream) {
    if (!logits || !coef || !loss || !work || n <= 0 || K <= 0) return fail(NLDPC_EINVAL, "nldpc_bce_loss: bad argument");
    if (work_bytes < (size_t)kBceBlocks * sizeof(double))
        return fail(NLDPC_EINVAL, "nldpc_bce_loss: workspace too small");
    hipStream_t s = static_cast<hipStream_t>(stream);
    const int nb = bce_blocks(n);
    for (int k0 = 0; k0 < K; k0 += kBceMaxK) {  // groups of up to 64 terms, accumulated into *loss
        BceArgs a{};
        a.K = K - k0 < kBceMaxK ? K - k0 : kBceMaxK;
        for (int k = 0; k < a.K; ++k) {
            if (!logits[k0 + k]) return fail(NLDPC_EINVAL, "nldpc_bce_loss: null logits");
            a.x[k] = logits[k0 + k];
            a.coef[k] = coef[k0 + k];
        }
        double* part = static_cast<double*>(work);
        hipLaunchKernelGGL(bce_loss_kernel<false>, dim3(nb), dim3(256), 0, s, a, target, n, part, BceArgs{});
        hipLaunchKernelGGL(bce_finish_kernel, dim3(1), dim3(64), 0, s, part, nb, n, loss, k0 > 0 ? 1 : 0);
    }
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? NLDPC_OK : hip_fail(e, "bce_loss_kernel launch");
}

static int bce_grad(const float* const* logits, int32_t K, const float* coef, const float* target, int64_t n,
                    const float* gseed, float* const* grads, void* stream, bool unless_unit) {
    if (!logits || !coef || !gseed || !grads || n <= 0 || K <= 0) return fail(NLDPC_EINVAL, "nldpc_bce_grad: bad argument");
    hipStream_t s = static_cast<hipStream_t>(stream);
    for (int k0 = 0; k0 < K; k0 += kBceMaxK) {
        BceArgs a{}, g{};
        a.K = g.K = K - k0 < kBceMaxK ? K - k0 : kBceMaxK;
        for (int k = 0; k < a.K; ++k) {
            if (!logits[k0 + k] || !grads[k0 + k]) return fail(NLDPC_EINVAL, "nldpc_bce_grad: null pointer");
            a.x[k] = logits[k0 + k];
            a.coef[k] = coef[k0 + k];
            g.x[k] = grads[k0 + k];
        }
        if (unless_unit)
            hipLaunchKernelGGL(bce_grad_kernel<true>, dim3(4096), dim3(256), 0, s, a, target, n, gseed, g);
        else
            hipLaunchKernelGGL(bce_grad_kernel<false>, dim3(4096), dim3(256), 0, s, a, target, n, gseed, g);
    }
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? NLDPC_OK : hip_fail(e, "bce_grad_kernel launch");
}

extern "C" int nldpc_bce_grad(const float* const* logits, int32_t K, const float* coef, const float* target, int64_t n,
                              const float* gseed, float* const* grads, void* stream) {
    return bce_grad(logits, K, coef, target, n, gseed, grads, stream, false);
}

extern "C" int nldpc_bce_grad_unless_unit(const float* const* logits, int32_t K, const float* coef, const float* target,
                                          int64_t n, const float* gseed, float* const* grads, void* stream) {
    return bce_grad(logits, K, coef, target, n, gseed, grads, stream, true);
}

extern "C" int nldpc_bce_loss_grad(const float* const* logits, int32_t K, const float* coef, const float* target,
                                   int64_t n, float* loss, float* const* grads, void* work, size_t work_bytes,
                                   void* stream) {
    if (!logits || !coef || !loss || !grads || !work || n <= 0 || K <= 0)
        return fail(NLDPC_EINVAL, "nldpc_bce_loss_grad: bad argument");
    if (work_bytes < (size_t)kBceBlocks * sizeof(double))
        return fail(NLDPC_EINVAL, "nldpc_bce_loss_grad: workspace too small");
    hipStream_t s = static_cast<hipStream_t>(stream);
    const int nb = bce_blocks(n);
    for (int k0 = 0; k0 < K; k0 += kBceMaxK) {
        BceArgs a{}, g{};
        a.K = g.K = K - k0 < kBceMaxK ? K - k0 : kBceMaxK;
        for (int k = 0; k < a.K; ++k) {
            if (!logits[k0 + k] || !grads[k0 + k]) return fail(NLDPC_EINVAL, "nldpc_bce_loss_grad: null pointer");
            a.x[k] = logits[k0 + k];
            a.coef[k] = coef[k0 + k];
            g.x[k] = grads[k0 + k];
        }
        double* part = static_cast<double*>(work);
        hipLaunchKernelGGL(bce_loss_kernel<true>, dim3(nb), dim3(256), 0, s, a, target, n, part, g);
        hipLaunchKernelGGL(bce_finish_kernel, dim3(1), dim3(64), 0, s, part, nb, n, loss, k0 > 0 ? 1 : 0);
    }
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? NLDPC_OK : hip_fail(e, "bce_loss_kernel launch");
}

extern "C" int nldpc_awgn_llr(float* xa, int64_t B, int64_t L, float sigma, uint64_t seed, int64_t b_offset,
                              int32_t qbit, void* stream) {
    return nldpc_channel_llr(xa, B, L, sigma, seed, b_offset, qbit, nullptr, 0, 0, 0.f, 0, 0, 0.f, stream);
}

extern "C" int nldpc_channel_llr(float* xa, int64_t B, int64_t L, float sigma, uint64_t seed, int64_t b_offset,
                                 int32_t qbit, const uint8_t* y, int64_t puncture_start, int64_t puncture_end,
                                 float puncture_value, int64_t shorten_start, int64_t shorten_end, float shorten_value,
                                 void* stream) {
    if (!xa || B <= 0 || L <= 0 || !(sigma > 0.f)) return fail(NLDPC_EINVAL, "nldpc_channel_llr: bad argument");
    if (puncture_start < 0 || shorten_start < 0 || puncture_end > L || shorten_end > L)
        return fail(NLDPC_EINVAL, "nldpc_channel_llr: puncture / shortening range outside the codeword");
    ChannelOpts o{y, L, 0, 0, 0, 0, puncture_value, shorten_value};
    if (puncture_start > 0) { o.p0 = puncture_start - 1; o.p1 = puncture_end; }
    if (shorten_start > 0) { o.s0 = shorten_start - 1; o.s1 = shorten_end; }
    const int64_t total = B * L;
    const int64_t first = b_offset * L;
    const int64_t groups = ((first + total + 3) >> 2) - (first >> 2);
    const int64_t blocks = (groups + 255) / 256;
    if (blocks > 0x7FFFFFFF) return fail(NLDPC_EUNSUPPORTED, "nldpc_awgn_llr: too large");
    hipLaunchKernelGGL(awgn_kernel, dim3((unsigned)blocks), dim3(256), 0, static_cast<hipStream_t>(stream), xa, total,
                       first, (double)sigma, seed, qbit, o);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? NLDPC_OK : hip_fail(e, "awgn_kernel launch");
}

extern "C" int nldpc_ber_count(const float* llr, const uint8_t* y, int64_t B, int64_t L, int32_t convention,
                               int64_t* counts, void* stream) {
    if (!llr || !counts || B <= 0 || L <= 0) return fail(NLDPC_EINVAL, "nldpc_ber_count: bad argument");
    const int64_t blocks = B < 4096 ? B : 4096;
    hipLaunchKernelGGL(ber_kernel, dim3((unsigned)blocks), dim3(256), 0, static_cast<hipStream_t>(stream), llr, y, B, L,
                       convention, reinterpret_cast<unsigned long long*>(counts));
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? NLDPC_OK : hip_fail(e, "ber_kernel launch");
}
