// Microbenchmark (development only, r3): can v_mfma_f32_4x4x1_16b_f32 (the per-lane 4-output fma form:
// B = the lane's own value, A = a per-lane 0/1 pattern) run beside VALU adds without taking their
// issue slots?  Times per trip of: MFMA only, VALU only, both interleaved (same counts), 4 waves/SIMD.
// Also checks the numerics claim: 4x4x1 accumulation == fmaf chain, bit for bit.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off mfma_mix.hip -o mfma_mix
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
typedef float f4 __attribute__((ext_vector_type(4)));

template <int NM, int NV>
__global__ __launch_bounds__(1024) void kern(float* out, unsigned long long* cyc, int R, float seed) {
    const int l = threadIdx.x & 63;
    const float a = (l & 3) == 1 ? 0.f : 1.f;  // the "skip own edge" pattern
    f4 c[8];
    float v[16];
#pragma unroll
    for (int i = 0; i < 8; ++i) c[i] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < 16; ++i) v[i] = seed + threadIdx.x * 1e-3f + i;
    const float bb = seed * 1e-7f;
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < R; ++r) {
#pragma unroll
        for (int g = 0; g < 8; ++g) {
#pragma unroll
            for (int i = 0; i < NM; ++i)
                c[(g * NM + i) & 7] = __builtin_amdgcn_mfma_f32_4x4x1f32(a, v[(g + i) & 15], c[(g * NM + i) & 7], 0, 0, 0);
#pragma unroll
            for (int i = 0; i < NV; ++i) v[(g * NV + i) & 15] = v[(g * NV + i) & 15] + bb;
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 16 + threadIdx.x / 64] = t1 - t0;
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) s += c[i].x + c[i].y + c[i].z + c[i].w;
#pragma unroll
    for (int i = 0; i < 16; ++i) s += v[i];
    out[blockIdx.x * 1024 + threadIdx.x] = s;
}

template <int NM, int NV>
void run(float* d, unsigned long long* dc) {
    const int R = 4000;
    for (int i = 0; i < 2; ++i) kern<NM, NV><<<256, 1024>>>(d, dc, R, 1.f);
    kern<NM, NV><<<256, 1024>>>(d, dc, R, 1.f);
    static unsigned long long h[256 * 16];
    (void)hipMemcpy(h, dc, sizeof(h), hipMemcpyDeviceToHost);
    double mx = 0;
    for (int i = 0; i < 256 * 16; ++i) mx = h[i] > mx ? h[i] : mx;
    // per SIMD: 4 waves x R trips x 8 groups
    const double per = 4.0 * R * 8;
    printf("MFMA %d + v_add %d per group: %7.2f SIMD-cycles per group (MFMA-only bound %d, VALU-only bound %.1f)\n", NM, NV,
           mx / per, NM * 8, NV * 2.0);
}

__global__ void numerics(float* out) {  // lane l: chain over 8 inputs with a 0/1 pattern vs fmaf chain
    const int l = threadIdx.x;
    f4 c = {0.f, 0.f, 0.f, 0.f};
    float ref[4] = {0.f, 0.f, 0.f, 0.f};
    for (int k = 0; k < 8; ++k) {
        const float b = __sinf(0.37f * (l + 1) * (k + 1)) * (k & 1 ? 1e3f : 1e-3f);
        const float a = ((l + k) % 3 == 0) ? 0.f : 1.f;
        c = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c, 0, 0, 0);
        // lane l's output r: A[block][r] * B[block][l & 3], A from lane 4*block + r
        for (int r = 0; r < 4; ++r) {
            const int al = (l & ~3) + r;
            const float ar = ((al + k) % 3 == 0) ? 0.f : 1.f;
            ref[r] = __builtin_fmaf(ar, b, ref[r]);
        }
    }
    int bad = 0;
    for (int r = 0; r < 4; ++r) bad += __float_as_uint(c[r]) != __float_as_uint(ref[r]);
    out[l] = (float)bad;
}

int main() {
    float* d;
    unsigned long long* dc;
    (void)hipMalloc(&d, 256 * 1024 * 4);
    (void)hipMalloc(&dc, 256 * 16 * 8);
    numerics<<<1, 64>>>(d);
    float h[64];
    (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    int bad = 0;
    for (float x : h) bad += (int)x;
    printf("4x4x1 f32 MFMA vs fmaf chain (0/1 A, 8 steps, 64 lanes x 4 outputs): %d mismatches\n", bad);
    run<1, 0>(d, dc);
    run<2, 0>(d, dc);
    run<0, 4>(d, dc);
    run<0, 8>(d, dc);
    run<1, 4>(d, dc);
    run<1, 8>(d, dc);
    run<2, 8>(d, dc);
    run<1, 2>(d, dc);
    return 0;
}
