// Standalone check of the DPP/permlane wave_sum (nldpc_fused.h) against a shfl_xor reduction.
#include <hip/hip_runtime.h>
#include <cstdio>
#include "nldpc_fused.h"
using namespace nldpc;
__global__ void k(const float* x, float* a, float* b) {
    const float v = x[blockIdx.x * 64 + threadIdx.x];
    float r = v;
    for (int off = 32; off > 0; off >>= 1) r += __shfl_xor(r, off, 64);
    a[blockIdx.x * 64 + threadIdx.x] = r;
    b[blockIdx.x * 64 + threadIdx.x] = wave_sum(v);
    // stage probes: after DPP only
    float y = v;
    y += dpp_mov<0xB1>(y);
    if (blockIdx.x == 0) b[64 * 8 + threadIdx.x] = y;
}
int main() {
    const int nb = 8, n = nb * 64 + 64;
    float hx[n], ha[n], hb[n];
    for (int i = 0; i < n; ++i) hx[i] = (i % 64 == 0) ? 1.f : 0.f;
    for (int i = 64; i < nb * 64; ++i) hx[i] = (float)((i * 37) % 11) - 5.f;
    float *x, *a, *b;
    hipMalloc(&x, n * 4); hipMalloc(&a, n * 4); hipMalloc(&b, n * 4);
    hipMemcpy(x, hx, n * 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(nb), dim3(64), 0, 0, x, a, b);
    hipMemcpy(ha, a, n * 4, hipMemcpyDeviceToHost);
    hipMemcpy(hb, b, n * 4, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < nb * 64; ++i) if (ha[i] != hb[i]) { if (bad < 8) printf("lane %d: shfl %g dpp %g\n", i, ha[i], hb[i]); ++bad; }
    printf("mismatches %d of %d\n", bad, nb * 64);
    printf("quad_perm probe lanes 0..7:"); for (int i = 0; i < 8; ++i) printf(" %g", hb[64 * 8 + i]); printf("\n");
    return bad != 0;
}
