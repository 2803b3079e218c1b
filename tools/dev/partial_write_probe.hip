// Does a byte-per-lane store that covers half a 128-byte line make the L2 fetch the line from HBM?
// (r5: the cfg5 saving forward fetches ~8.4 GB per launch that no load of its own explains; its
// posterior clamp masks are such stores.)  Run under rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE:
//   kind 0: 4 B per lane, a wave writes 256 contiguous bytes (two full lines)          1 GiB written
//   kind 1: 1 B per lane, a wave writes 64 contiguous bytes, the next wave the other half of the line
//   kind 2: 1 B per lane, only the first 64 bytes of every 128-byte line written
//   kind 3: like kind 1, but each lane stores 4 masks of 4 columns as one 32-bit word (a lane's 4 bytes)
//   kind 4: kind 1 with non-temporal stores (__builtin_nontemporal_store)
//   kind 5: kind 2 with non-temporal stores
// Build: hipcc --offload-arch=gfx950 -O3 tools/dev/partial_write_probe.hip -o /tmp/pwp
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ __launch_bounds__(256) void probe(int kind, uint8_t* dst, int64_t nbytes) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t nthreads = (int64_t)gridDim.x * 256;
    if (kind == 0) {
        float* d = reinterpret_cast<float*>(dst);
        for (int64_t i = t; i < nbytes / 4; i += nthreads) d[i] = (float)(i & 7);
    } else if (kind == 1) {
        for (int64_t i = t; i < nbytes; i += nthreads) dst[i] = (uint8_t)(i & 1);
    } else if (kind == 2) {
        // lane l of wave w writes byte 128 * w' + l: only the first half of each line
        const int64_t lane = threadIdx.x & 63, wave = t >> 6, nwaves = nthreads >> 6;
        for (int64_t w = wave; w < nbytes / 128; w += nwaves) dst[w * 128 + lane] = (uint8_t)(lane & 1);
    } else if (kind == 3) {
        uint32_t* d = reinterpret_cast<uint32_t*>(dst);
        for (int64_t i = t; i < nbytes / 4; i += nthreads) d[i] = 0x01000100u;
    } else if (kind == 4) {
        for (int64_t i = t; i < nbytes; i += nthreads) __builtin_nontemporal_store((uint8_t)(i & 1), dst + i);
    } else {
        const int64_t lane = threadIdx.x & 63, wave = t >> 6, nwaves = nthreads >> 6;
        for (int64_t w = wave; w < nbytes / 128; w += nwaves) __builtin_nontemporal_store((uint8_t)(lane & 1), dst + w * 128 + lane);
    }
}

int main() {
    const int64_t n = 1ll << 30;
    uint8_t* p = nullptr;
    if (hipMalloc(&p, n) != hipSuccess) return 1;
    hipMemset(p, 0, n);
    for (int kind = 0; kind < 6; ++kind) {
        hipLaunchKernelGGL(probe, dim3(4096), dim3(256), 0, 0, kind, p, n);
        if (hipDeviceSynchronize() != hipSuccess) return 2;
    }
    hipFree(p);
    printf("probe kinds 0..5 done, 1 GiB each\n");
    return 0;
}
