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

namespace nldpc {

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

template <int DC, int KIND>
__device__ __forceinline__ void cn_core(const float (&m)[DC], int d, int qbit, float lo, float hi, CnCore<DC>& c) {
    if (KIND == NLDPC_SP) {
#pragma unroll
        for (int k = 0; k < DC; ++k) {
            if (k < d) {
                const float x = clampf(m[k], lo, hi);
                const float t = tanhf(fmul(-0.5f, x));
                c.mq[k] = fadd(t, (fabsf(t) > 0.f) ? 0.f : 1.f);
            } else {
                c.mq[k] = 1.f;
            }
        }
#pragma unroll
        for (int k = 0; k < DC; ++k) {
            if (k < d) {
                float P = 1.f;
#pragma unroll
                for (int l = 0; l < DC; ++l)
                    if (l < d && l != k) P = fmul(P, c.mq[l]);
                P = clampf(P, -kSpClip, kSpClip);
                c.out0[k] = fmul(-2.f, atanhf(P));
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

}  // namespace nldpc
