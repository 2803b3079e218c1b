// Microbenchmark / probe (development only, r4): ds_write_addtid_b32 / ds_read_addtid_b32 on gfx950.
// 1. Address range: which LDS dword does lane l write for M0 = m (address = M0[?:0] + offset + 4*l)?
//    m above 64 KiB tells whether M0 bits past 15 take part (the guide says M0[15:0]).
// 2. Issue rate: wave-instructions per CU-cycle of ds_write_addtid_b32 vs ds_write_b32 (own address VGPR)
//    vs ds_read_addtid_b32 vs ds_read_b32, 16 waves per CU (4 per SIMD), no waits inside the loop.
//   hipcc --offload-arch=gfx950 -O3 addtid_probe.hip -o addtid_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ void where(uint32_t* out, uint32_t m) {
    extern __shared__ uint32_t s[];  // 160 KiB
    for (int i = threadIdx.x; i < 40960; i += blockDim.x) s[i] = 0xFFFFFFFFu;
    __syncthreads();
    if (threadIdx.x < 64) {
        const uint32_t v = threadIdx.x;
        asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tds_write_addtid_b32 %1\n\ts_waitcnt lgkmcnt(0)" :: "s"(m), "v"(v) : "memory");
    }
    __syncthreads();
    for (int i = threadIdx.x; i < 40960; i += blockDim.x) out[i] = s[i];
}

// 3. Under a partial EXEC: lanes 40..63 only.  Does lane l write M0 + 4*l (thread id) or M0 + 4*(l - 40) (index
//    among the active lanes)?
__global__ void partial(uint32_t* out) {
    extern __shared__ uint32_t s[];
    for (int i = threadIdx.x; i < 256; i += blockDim.x) s[i] = 0xFFFFFFFFu;
    __syncthreads();
    if (threadIdx.x < 64) {
        const uint32_t v = threadIdx.x;
        uint64_t sv;
        asm volatile("s_mov_b64 %0, exec\n\ts_and_b64 exec, %0, %1\n\ts_mov_b32 m0, 0\n\ts_nop 0\n\t"
                     "ds_write_addtid_b32 %2\n\ts_mov_b64 exec, %0\n\ts_nop 0\n\ts_waitcnt lgkmcnt(0)"
                     : "=&s"(sv) : "s"(~0ull << 40), "v"(v) : "memory");
    }
    __syncthreads();
    for (int i = threadIdx.x; i < 256; i += blockDim.x) out[i] = s[i];
}

// 4. The owner-write pattern of gen_fused.py OWNTID: 128 threads (two waves, u = 0..127), edge region of Z=384
//    slots at byte `base0` of LDS, copy offset cq: lane copy u writes slot cq + u, wrapped to cq + u - 384 for
//    u >= 384 - cq, once through ds_write_b32 (VGPR address) into region A and once by ds_write_addtid_b32
//    with the wrapped lanes under their own EXEC into region B.  Counts mismatching slots.
__device__ __forceinline__ uint64_t wrap_mask_p(int T, int u0) {
    const int sh = T - u0;
    return sh <= 0 ? ~0ull : (sh >= 64 ? 0ull : (~0ull << sh));
}
__global__ void ownpat(uint32_t* out, int cq, int baseA, int baseB) {
    extern __shared__ uint32_t s[];
    for (int i = threadIdx.x; i < 2048; i += blockDim.x) s[i] = 0xFFFFFFFFu;
    __syncthreads();
    const int u = threadIdx.x;
    const uint32_t v = 1000u + u;
    const int T = 384 - cq;
    const int ia = cq + u - (u >= T ? 384 : 0);
    s[baseA / 4 + ia] = v;
    const int su0 = __builtin_amdgcn_readfirstlane(u);
    const uint32_t slu = __builtin_amdgcn_readfirstlane((uint32_t)baseB + 4u * (uint32_t)u);
    if (cq + 128 <= 384) {
        asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tds_write_addtid_b32 %1" :: "s"(slu + 4u * cq), "v"(v) : "memory", "m0");
    } else {
        const uint64_t wm = wrap_mask_p(T, su0);
        uint64_t sv;
        asm volatile("s_mov_b64 %0, exec\n\ts_andn2_b64 exec, %0, %1\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
                     "ds_write_addtid_b32 %4\n\ts_and_b64 exec, %0, %1\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
                     "ds_write_addtid_b32 %4\n\ts_mov_b64 exec, %0\n\ts_nop 0"
                     : "=&s"(sv) : "s"(wm), "s"(slu + 4u * cq), "s"(slu + 4u * (uint32_t)(cq - 384)), "v"(v) : "memory", "m0");
    }
    __syncthreads();
    int bad = 0;
    for (int i = threadIdx.x; i < 384; i += blockDim.x) bad += s[baseA / 4 + i] != s[baseB / 4 + i];
    atomicAdd(out, bad);
}

template <int OP>
__global__ void rate(uint32_t* out, unsigned long long* cyc, int R) {
    extern __shared__ uint32_t s[];
    const int w = threadIdx.x >> 6;
    const uint32_t base = __builtin_amdgcn_readfirstlane((uint32_t)w * 1024u);  // bytes: each wave its own 1 KiB slice
    uint32_t v = threadIdx.x, acc = 0;
    const uint32_t a = base + 4u * (threadIdx.x & 63);
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < R; ++r) {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            if constexpr (OP == 0) asm volatile("s_mov_b32 m0, %0\n\tds_write_addtid_b32 %1" :: "s"(base), "v"(v) : "memory");
            if constexpr (OP == 1) asm volatile("ds_write_b32 %0, %1" :: "v"(a), "v"(v) : "memory");
            if constexpr (OP == 2) { uint32_t t; asm volatile("s_mov_b32 m0, %1\n\tds_read_addtid_b32 %0" : "=v"(t) : "s"(base) : "memory"); acc += t; }
            if constexpr (OP == 3) { uint32_t t; asm volatile("ds_read_b32 %0, %1" : "=v"(t) : "v"(a) : "memory"); acc += t; }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 16 + w] = t1 - t0;
    out[blockIdx.x * 1024 + threadIdx.x] = acc;
}

int main() {
    uint32_t* d;
    unsigned long long* dc;
    (void)hipMalloc(&d, 256 * 1024 * 4 + 40960 * 4);
    (void)hipMalloc(&dc, 256 * 16 * 8);
    hipFuncSetAttribute((const void*)where, hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
    static uint32_t h[40960];
    for (uint32_t m : {0x0u, 0x100u, 0xFF00u, 0x10000u, 0x10100u, 0x20000u}) {
        where<<<1, 256, 163840>>>(d, m);
        (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
        int first = -1, n = 0;
        for (int i = 0; i < 40960; ++i)
            if (h[i] != 0xFFFFFFFFu) { if (first < 0) first = i; ++n; }
        printf("M0 = 0x%05x: %d dwords written, first at byte 0x%05x (lane 0 value %u)\n", m, n, first * 4,
               first >= 0 ? h[first] : 0);
    }
    partial<<<1, 256, 1024>>>(d);
    (void)hipMemcpy(h, d, 256 * 4, hipMemcpyDeviceToHost);
    {
        int first = -1, n = 0;
        for (int i = 0; i < 256; ++i)
            if (h[i] != 0xFFFFFFFFu) { if (first < 0) first = i; ++n; }
        printf("EXEC = lanes 40..63: %d dwords written, first at dword %d holding lane %u's value "
               "(40: address by thread id; 0: by active-lane index)\n", n, first, first >= 0 ? h[first] : 0);
    }
    for (int bB : {0, 4096}) {
        int tot = 0;
        for (int cq = 0; cq < 384; cq += 7) {
            (void)hipMemset(d, 0, 4);
            ownpat<<<1, 128, 8192>>>(d, cq, bB == 0 ? 4096 : 0, bB);
            uint32_t b = 0;
            (void)hipMemcpy(&b, d, 4, hipMemcpyDeviceToHost);
            if (b && tot < 3) printf("  owner pattern cq=%d region B at byte %d: %u slots differ\n", cq, bB, b);
            tot += b != 0;
        }
        printf("owner addtid pattern, region B at LDS byte %d: %d of 55 copy offsets wrong\n", bB, tot);
    }
    const int R = 20000;
    const char* names[4] = {"ds_write_addtid_b32", "ds_write_b32 (address VGPR)", "ds_read_addtid_b32", "ds_read_b32"};
    void (*ks[4])(uint32_t*, unsigned long long*, int) = {rate<0>, rate<1>, rate<2>, rate<3>};
    for (int k = 0; k < 4; ++k) {
        hipFuncSetAttribute((const void*)ks[k], hipFuncAttributeMaxDynamicSharedMemorySize, 65536);
        ks[k]<<<256, 1024, 65536>>>(d, dc, 100);
        ks[k]<<<256, 1024, 65536>>>(d, dc, R);
        (void)hipDeviceSynchronize();
        static unsigned long long hc[256 * 16];
        (void)hipMemcpy(hc, dc, sizeof(hc), hipMemcpyDeviceToHost);
        double mx = 0;
        for (auto x : hc) mx = x > mx ? x : mx;
        // 16 waves x R x 16 instructions per CU; s_memtime counts at 100 MHz on gfx9? report raw and per-instr
        printf("%-28s %.3f memtime ticks per CU-wave-instruction (16 waves/CU)\n", names[k], mx / (16.0 * R * 16));
    }
    return 0;
}
