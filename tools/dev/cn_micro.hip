// Microbenchmark (development only): cost of the Neural check-node row arithmetic variants on gfx950,
// register-only (no LDS), 1024-thread workgroups (4 waves per SIMD, like the fused kernel), one
// workgroup per CU.  Each thread runs R rounds of 3 row copies of degree DC; the outputs feed the
// next round.  Prints ns and SIMD-cycles per wave-level row copy for each variant.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I../../include -I../../neural-ldpc-decoder-torch_amd/csrc cn_micro.hip -o /tmp/cn_micro
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#include "nldpc_fused.h"

using namespace nldpc;

__device__ __forceinline__ uint32_t med3u(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t d;
    asm volatile("v_med3_u32 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c));
    return d;
}

template <int DC>
__device__ __forceinline__ void two_smallest_med3(const uint32_t (&key)[DC], uint32_t& min1, uint32_t& min2) {
    uint32_t a = min(key[0], key[1]), b = max(key[0], key[1]);
#pragma unroll
    for (int k = 2; k < DC; ++k) {
        b = med3u(a, b, key[k]);
        a = min(a, key[k]);
    }
    min1 = a;
    min2 = b;
}

// VAR 0: neural_row as shipped; 1: mag select by med3 arithmetic (no compare mask); 2: no sign (bound);
// 3: streaming med3 two-smallest; 4: 1 + 3
template <int VAR, int DC>
__device__ __forceinline__ void row(float (&m)[DC], const float (&w)[DC], const float (&b)[DC]) {
    if constexpr (VAR == 0) {
        neural_row<DC>(m, w, b);
        return;
    }
    constexpr uint32_t kInit = (0x461C4000u << 1) - 2u;
    uint32_t key[DC];
    bool pos[DC];
    bool par = false;
#pragma unroll
    for (int k = 0; k < DC; ++k) {
        key[k] = (__builtin_bit_cast(uint32_t, m[k]) << 1) - 2u;
        pos[k] = m[k] > 0.f;
        par ^= pos[k];
    }
    uint32_t min1, min2;
    if constexpr (VAR == 3 || VAR == 4)
        two_smallest_med3<DC>(key, min1, min2);
    else
        two_smallest<DC>(key, min1, min2);
    min1 = min(min1, kInit);
    min2 = min(min2, kInit);
    float mg1 = __builtin_bit_cast(float, (min1 + 2u) >> 1);
    float mg2 = __builtin_bit_cast(float, (min2 + 2u) >> 1);
    const uint32_t S = min1 + min2 + 2u;
    asm volatile("" : "+v"(mg1), "+v"(mg2));
#pragma unroll
    for (int k = 0; k < DC; ++k) {
        float mag;
        if constexpr (VAR == 1 || VAR == 4)
            mag = __builtin_bit_cast(float, (S - med3u(key[k], min1, min2)) >> 1);
        else
            mag = key[k] == min1 ? mg2 : mg1;
        const float r = relu_mask(fadd(fmul(mag, w[k]), b[k]));
        if constexpr (VAR == 2)
            m[k] = r;
        else
            m[k] = (par != pos[k]) ? r : -r;
    }
}

template <int VAR, int DC>
__global__ __launch_bounds__(1024) void kern(const float* in, float* out, const float* wb, int R) {
    const int t = blockIdx.x * 1024 + threadIdx.x;
    float m[3][DC];
#pragma unroll
    for (int c = 0; c < 3; ++c)
#pragma unroll
        for (int k = 0; k < DC; ++k) m[c][k] = in[(t * 3 + c) * DC + k];
    const cfloat_p cw = (cfloat_p)wb;
    float w[DC], b[DC];
#pragma unroll
    for (int k = 0; k < DC; ++k) {
        w[k] = cw[k];
        b[k] = cw[DC + k];
    }
    for (int r = 0; r < R; ++r) {
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            row<VAR, DC>(m[c], w, b);
            // the fused kernel handles one row copy at a time (register budget)
            __builtin_amdgcn_sched_barrier(0);
        }
    }
#pragma unroll
    for (int c = 0; c < 3; ++c)
#pragma unroll
        for (int k = 0; k < DC; ++k) out[(t * 3 + c) * DC + k] = m[c][k];
}

template <int VAR, int DC>
void run(const char* name, float* din, float* dout, float* dwb, int blocks, int R) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    kern<VAR, DC><<<blocks, 1024>>>(din, dout, dwb, R);
    hipEventRecord(e0);
    const int reps = 5;
    for (int i = 0; i < reps; ++i) kern<VAR, DC><<<blocks, 1024>>>(din, dout, dwb, R);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    ms /= reps;
    // wave-level row copies per SIMD: (16 waves / 4 SIMDs) x R x 3, blocks = CUs
    const double per_simd = 4.0 * R * 3 * (blocks / 256.0);
    std::vector<float> h(3 * DC);
    hipMemcpy(h.data(), dout, sizeof(float) * 3 * DC, hipMemcpyDeviceToHost);
    printf("DC=%2d var %d %-22s %8.3f ms  %7.1f SIMD-cycles per row copy (%.2f per edge)  [%g]\n", DC, VAR, name, ms,
           ms * 1e-3 * 2.4e9 / per_simd, ms * 1e-3 * 2.4e9 / per_simd / DC, (double)h[0]);
}

template <int DC>
void all(float* din, float* dout, float* dwb, int blocks, int R) {
    run<0, DC>("shipped", din, dout, dwb, blocks, R);
    run<1, DC>("med3 mag select", din, dout, dwb, blocks, R);
    run<2, DC>("no sign (bound)", din, dout, dwb, blocks, R);
    run<3, DC>("streaming med3 min", din, dout, dwb, blocks, R);
    run<4, DC>("med3 select+stream", din, dout, dwb, blocks, R);
}

int main() {
    const int blocks = 256, R = 2000, DCMAX = 10;
    const size_t n = (size_t)blocks * 1024 * 3 * DCMAX;
    std::vector<float> h(n);
    uint32_t s = 12345;
    for (auto& x : h) {
        s = s * 1664525u + 1013904223u;
        x = ((s >> 8) * (1.0f / 16777216.0f) - 0.5f) * 8.f;
    }
    std::vector<float> hw(2 * DCMAX);
    for (int k = 0; k < DCMAX; ++k) {
        hw[k] = 0.9f + 0.01f * k;
        hw[DCMAX + k] = -0.05f;
    }
    float *din, *dout, *dwb;
    hipMalloc(&din, n * 4);
    hipMalloc(&dout, n * 4);
    hipMalloc(&dwb, 2 * DCMAX * 4);
    hipMemcpy(din, h.data(), n * 4, hipMemcpyHostToDevice);
    hipMemcpy(dwb, hw.data(), 2 * DCMAX * 4, hipMemcpyHostToDevice);
    all<10>(din, dout, dwb, blocks, R);
    all<4>(din, dout, dwb, blocks, R);
    return 0;
}
