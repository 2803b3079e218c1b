// Microbenchmark (development only, r3): VALU issue rate of the SIMD on gfx950, written to settle
// whether a wave64 fp32 VALU instruction costs 2 or 4 SIMD cycles when several waves share a SIMD.
//  * plain C arithmetic (no inline asm, so no compiler-inserted hazard NOPs around asm blocks),
//  * 16 independent accumulators per lane, each touched once per group of 16 (no dependent issue),
//  * 256 instructions per loop trip (the loop's 3 SALU are < 1.2 % of the issue),
//  * 1, 2, 4 and 8 waves per SIMD (8 = two 1024-thread workgroups per CU).
// Cycles come from s_memtime (shader clock) of the slowest wave over the loop; the event time over the
// whole launch gives an independent check (assumed clock printed).
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off valu_rate2.hip -o /tmp/valu_rate2
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f2 __attribute__((ext_vector_type(2)));

#define R16(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15)

template <int OP>
__device__ __forceinline__ void body(float (&a)[16], f2 (&p)[16], float b0, float b1, f2 q0, f2 q1) {
    // 16 groups x 16 independent instructions = 256 per trip
#pragma unroll
    for (int g = 0; g < 16; ++g) {
        const float bb = (g & 1) ? b1 : b0;
        const f2 qq = (g & 1) ? q1 : q0;
#define ADD(i) a[i] = a[i] + bb;
#define FMA(i) a[i] = __builtin_fmaf(a[i], bb, b1);
#define MIN(i) a[i] = __builtin_fminf(a[i], bb);
#define PKADD(i) p[i] = p[i] + qq;
#define PKMUL(i) p[i] = p[i] * qq;
#define PKFMA(i) p[i] = __builtin_elementwise_fma(p[i], qq, q1);
#define CHAIN(i) a[0] = a[0] + a[i];
#define PKCHAIN(i) p[0] = p[0] + p[i];
        if constexpr (OP == 0) { R16(ADD) }
        if constexpr (OP == 1) { R16(FMA) }
        if constexpr (OP == 2) { R16(PKADD) }
        if constexpr (OP == 3) { R16(PKMUL) }
        if constexpr (OP == 4) { R16(PKFMA) }
        if constexpr (OP == 5) { R16(CHAIN) }    // one dependent chain (latency-bound per wave)
        if constexpr (OP == 6) { R16(PKCHAIN) }  // one dependent packed chain
        if constexpr (OP == 7) { R16(MIN) }
        if constexpr (OP == 8) {  // half scalar adds, half packed adds
#define MIX(i) if ((i) & 1) { p[i] = p[i] + qq; } else { a[i] = a[i] + bb; }
            R16(MIX)
        }
        if constexpr (OP == 9) {  // 2 dependent chains per 16-instruction group, 8 deep, interleaved
#define TWO(i) if ((i) & 1) { a[1] = a[1] + a[(i) | 8]; } else { a[0] = a[0] + a[(i) | 8]; }
            R16(TWO)
        }
        if constexpr (OP == 10) {  // 4 interleaved dependent packed chains
#define PK4(i) p[(i) & 3] = p[(i) & 3] + p[((i) & 7) | 8];
            R16(PK4)
        }
        asm volatile("" : "+v"(a[0]), "+v"(p[0]));  // keep the groups from folding across trips
    }
}

template <int OP, int TPB>
__global__ __launch_bounds__(TPB) void kern(float* out, unsigned long long* cyc, int R, float seed) {
    float a[16];
    f2 p[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        a[i] = seed + threadIdx.x * 0.001f + i;
        p[i] = f2{a[i], a[i] * 0.5f};
    }
    const float b0 = seed * 1e-7f, b1 = seed * 2e-7f;
    const f2 q0 = {b0, b1}, q1 = {b1, b0};
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < R; ++r) body<OP>(a, p, b0, b1, q0, q1);
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * (TPB / 64) + threadIdx.x / 64] = t1 - t0;
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) s += a[i] + p[i].x + p[i].y;
    out[blockIdx.x * TPB + threadIdx.x] = s;
}

template <int OP, int TPB, int BPC = 1>
void run(const char* name, float* d, unsigned long long* dc) {
    const int R = 2000, blocks = 256 * BPC;
    const double wps = TPB / 256.0 * BPC;  // waves per SIMD
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int i = 0; i < 2; ++i) kern<OP, TPB><<<blocks, TPB>>>(d, dc, R, 1.f);
    (void)hipEventRecord(e0);
    kern<OP, TPB><<<blocks, TPB>>>(d, dc, R, 1.f);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const int nw = blocks * (TPB / 64);
    static unsigned long long h[512 * 16];
    (void)hipMemcpy(h, dc, nw * 8, hipMemcpyDeviceToHost);
    double mx = 0;
    for (int i = 0; i < nw; ++i) mx = h[i] > mx ? h[i] : mx;
    const double per_simd = wps * R * 256.0;  // wave-instructions issued per SIMD
    printf("%d waves/SIMD  %-34s %8.3f ms  %5.2f cyc/wave-instr (s_memtime)  %5.2f (event, 2.4 GHz)\n", (int)wps, name,
           ms, mx / per_simd, ms * 1e-3 * 2.4e9 / per_simd);
}

template <int OP>
void sweep(const char* name, float* d, unsigned long long* dc) {
    run<OP, 256>(name, d, dc);
    run<OP, 512>(name, d, dc);
    run<OP, 1024>(name, d, dc);
    run<OP, 1024, 2>(name, d, dc);
}

int main() {
    float* d;
    unsigned long long* dc;
    (void)hipMalloc(&d, 512 * 1024 * 4);
    (void)hipMalloc(&dc, 512 * 16 * 8);
    sweep<0>("v_add_f32 (16 indep)", d, dc);
    sweep<1>("v_fma_f32 (16 indep)", d, dc);
    sweep<7>("v_min_f32 (16 indep)", d, dc);
    sweep<2>("v_pk_add_f32 (16 indep)", d, dc);
    sweep<3>("v_pk_mul_f32 (16 indep)", d, dc);
    sweep<4>("v_pk_fma_f32 (16 indep)", d, dc);
    sweep<8>("v_add_f32 / v_pk_add_f32 mix", d, dc);
    sweep<5>("v_add_f32 (1 dependent chain)", d, dc);
    sweep<9>("v_add_f32 (2 interleaved chains)", d, dc);
    sweep<6>("v_pk_add_f32 (1 dependent chain)", d, dc);
    sweep<10>("v_pk_add_f32 (4 interleaved chains)", d, dc);
    return 0;
}
