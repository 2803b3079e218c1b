// HBM ceiling probe sweep: copy / write / read kernels over 4 GiB with U float4 in flight per lane,
// plain or non-temporal loads and stores, W workgroups of 256 per CU; best of 5 launches (HIP events), GB/s of bytes
// moved.  Picks the configuration nldpc_hbm_probe (csrc/nldpc_aux.hip) should use.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/dev/hbm_probe_sweep tools/dev/hbm_probe_sweep.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef float v4 __attribute__((ext_vector_type(4)));

template <int U, bool NTL, bool NTS, int KIND>
__global__ __launch_bounds__(256) void probe(v4* __restrict__ dst, const v4* __restrict__ src, long n4) {
    constexpr long TILE = 256L * U;
    const long ntiles = n4 / TILE;
    float acc = 0.f;
    for (long t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const long base = t * TILE + threadIdx.x;
        if (KIND == 1) {
            const v4 v = {1.f, 2.f, 3.f, 4.f};
#pragma unroll
            for (int k = 0; k < U; ++k) {
                if (NTS) __builtin_nontemporal_store(v, dst + base + k * 256);
                else dst[base + k * 256] = v;
            }
            continue;
        }
        v4 v[U];
#pragma unroll
        for (int k = 0; k < U; ++k) v[k] = NTL ? __builtin_nontemporal_load(src + base + k * 256) : src[base + k * 256];
        if (KIND == 0) {
#pragma unroll
            for (int k = 0; k < U; ++k) {
                if (NTS) __builtin_nontemporal_store(v[k], dst + base + k * 256);
                else dst[base + k * 256] = v[k];
            }
        } else {
#pragma unroll
            for (int k = 0; k < U; ++k) acc += (v[k].x + v[k].y) + (v[k].z + v[k].w);
        }
    }
    if (KIND == 2 && acc == 1234.5f) dst[blockIdx.x] = v4{acc, 0.f, 0.f, 0.f};
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

template <int U, bool NTL, bool NTS, int KIND>
void run(v4* d, const v4* s, long n4, int wpc, int cus) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    float best = 1e30f;
    for (int r = 0; r < 6; ++r) {
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL((probe<U, NTL, NTS, KIND>), dim3(cus * wpc), dim3(256), 0, 0, d, s, n4);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (r > 0 && ms < best) best = ms;
    }
    const double bytes = (KIND == 0 ? 32.0 : 16.0) * n4;
    printf("%-5s U=%2d ntload=%d ntstore=%d wg/CU=%2d : %8.1f GB/s\n", KIND == 0 ? "copy" : KIND == 1 ? "write" : "read",
           U, NTL, NTS, wpc, bytes / (best * 1e-3) / 1e9);
}

int main() {
    const long n4 = (4L << 30) / 16;
    v4 *a, *b;
    CK(hipMalloc(&a, n4 * 16));
    CK(hipMalloc(&b, n4 * 16));
    CK(hipMemset(a, 0, n4 * 16));
    hipDeviceProp_t p;
    CK(hipGetDeviceProperties(&p, 0));
    const int cus = p.multiProcessorCount;
    printf("%s, %d CUs\n", p.name, cus);
    for (int wpc : {2, 4, 8, 16}) {
        run<1, false, false, 0>(b, a, n4, wpc, cus);
        run<4, false, false, 0>(b, a, n4, wpc, cus);
        run<8, false, false, 0>(b, a, n4, wpc, cus);
        run<8, true, true, 0>(b, a, n4, wpc, cus);
        run<8, false, true, 0>(b, a, n4, wpc, cus);
        run<16, false, false, 0>(b, a, n4, wpc, cus);
        run<16, false, true, 0>(b, a, n4, wpc, cus);
        run<8, false, false, 1>(b, a, n4, wpc, cus);
        run<8, false, true, 1>(b, a, n4, wpc, cus);
        run<8, false, false, 2>(b, a, n4, wpc, cus);
        run<8, true, false, 2>(b, a, n4, wpc, cus);
    }
    CK(hipFree(a));
    CK(hipFree(b));
    return 0;
}
