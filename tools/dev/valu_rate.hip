// Microbenchmark (development only): SIMD-level issue cost of VALU instruction classes on gfx950 with
// 1024-thread workgroups (4 waves per SIMD), one workgroup per CU: 8 independent chains per lane,
// each loop iteration issues 8 instructions of one class.  Prints SIMD-cycles per wave-instruction
// at 2.4 GHz (s_memtime-free: hipEvent time over a fixed instruction count).
//   hipcc --offload-arch=gfx950 -O3 valu_rate.hip -o /tmp/valu_rate
#include <hip/hip_runtime.h>
#include <cstdio>

#define OP8(I)                                                                                            \
    I(a0, b0) I(a1, b1) I(a2, b2) I(a3, b3) I(a4, b0) I(a5, b1) I(a6, b2) I(a7, b3)

#define ADDF(x, y) asm volatile("v_add_f32 %0, %0, %1" : "+v"(x) : "v"(y));
#define MINU(x, y) asm volatile("v_min_u32 %0, %0, %1" : "+v"(x) : "v"(y));
#define MED3(x, y) asm volatile("v_med3_u32 %0, %0, %1, %2" : "+v"(x) : "v"(y), "v"(b1));
#define LSHLADD(x, y) asm volatile("v_lshl_add_u32 %0, %0, 1, %1" : "+v"(x) : "v"(y));
#define MULS(x, y) asm volatile("v_mul_f32 %0, %1, %0" : "+v"(x) : "s"(sw));
#define CMPSEL(x, y) asm volatile("v_cmp_lt_f32 %1, 0, %0\n\tv_cndmask_b32 %0, %0, %2, %1" : "+v"(x), "=s"(mk) : "v"(y));
#define CMPVCC(x, y) asm volatile("v_cmp_lt_f32 vcc, 0, %0\n\tv_cndmask_b32 %0, %0, %1, vcc" : "+v"(x) : "v"(y) : "vcc");
#define CNDM(x, y) asm volatile("v_cndmask_b32 %0, %0, %1, %2" : "+v"(x) : "v"(y), "s"(mk0));
#define PKADD(x, y) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(p##x) : "v"(q##y));
#define PKMUL(x, y) asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(p##x) : "v"(q##y));
#define PKFMA(x, y) asm volatile("v_pk_fma_f32 %0, %0, %1, %1" : "+v"(p##x) : "v"(q##y));
#define SXOR(x, y) asm volatile("s_xor_b64 %0, %0, %1" : "+s"(sa) : "s"(sb));

template <int OP, int TPB>
__global__ __launch_bounds__(TPB) void kern(float* out, unsigned long long* cyc, int R, float seed, float sw) {
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    float a0 = seed + threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6,
          a7 = a0 + 7;
    float b0 = 0.5f, b1 = 0.25f, b2 = 0.125f, b3 = 1.f;
    uint64_t mk = 0, mk0 = 0x5555555555555555ull, sa = 1, sb = 3;
    typedef float f2 __attribute__((ext_vector_type(2)));
    f2 pa0 = {a0, a1}, pa1 = {a1, a2}, pa2 = {a2, a3}, pa3 = {a3, a4}, pa4 = {a4, a5}, pa5 = {a5, a6}, pa6 = {a6, a7},
       pa7 = {a7, a0};
    f2 qb0 = {b0, b1}, qb1 = {b1, b2}, qb2 = {b2, b3}, qb3 = {b3, b0};
    for (int r = 0; r < R; ++r) {
        if constexpr (OP == 0) { OP8(ADDF) }
        if constexpr (OP == 1) { OP8(MINU) }
        if constexpr (OP == 2) { OP8(MED3) }
        if constexpr (OP == 3) { OP8(LSHLADD) }
        if constexpr (OP == 4) { OP8(MULS) }
        if constexpr (OP == 5) { OP8(CMPSEL) }  // 2 instructions each
        if constexpr (OP == 6) { OP8(CMPVCC) }  // 2 instructions each
        if constexpr (OP == 7) { OP8(CNDM) }
        if constexpr (OP == 8) { OP8(PKADD) }
        if constexpr (OP == 9) { OP8(SXOR) OP8(ADDF) }  // 8 SALU + 8 VALU
        if constexpr (OP == 10) { OP8(PKMUL) }
        if constexpr (OP == 11) { OP8(PKFMA) }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * (TPB / 64) + threadIdx.x / 64] = t1 - t0;
    const f2 ps = pa0 + pa1 + pa2 + pa3 + pa4 + pa5 + pa6 + pa7;
    out[blockIdx.x * 1024 + threadIdx.x] = ps.x + ps.y + a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + (float)(mk & 1) + (float)(sa & 1);
}

template <int OP, int TPB = 1024>
void run(const char* name, int ninst, float* d) {
    const int R = 20000, blocks = 256;
    constexpr double wps = TPB / 256.0;  // waves per SIMD
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    unsigned long long* dc;
    (void)hipMalloc(&dc, blocks * 16 * 8);
    for (int i = 0; i < 3; ++i) kern<OP, TPB><<<blocks, TPB>>>(d, dc, R, 1.f, 1.0001f);
    (void)hipEventRecord(e0);
    kern<OP, TPB><<<blocks, TPB>>>(d, dc, R, 1.f, 1.0001f);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const double per_simd = wps * R * ninst;  // wave-instructions per SIMD
    unsigned long long h[256 * 16];
    const int nw = blocks * (TPB / 64);
    (void)hipMemcpy(h, dc, nw * 8, hipMemcpyDeviceToHost);
    double mx = 0;
    for (int i = 0; i < nw; ++i) mx = h[i] > mx ? h[i] : mx;
    (void)hipFree(dc);
    // s_memtime counts shader-clock cycles: the slowest wave's loop = the SIMD's time for all its waves
    printf("%d waves/SIMD %-28s %8.3f ms  %5.2f cycles/wave-instr (s_memtime)  clock %.2f GHz\n", (int)wps, name, ms,
           mx / per_simd, mx / (ms * 1e-3) / 1e9);
}

int main() {
    float* d;
    (void)hipMalloc(&d, 256 * 1024 * 4);
    run<0>("v_add_f32", 8, d);
    run<1>("v_min_u32", 8, d);
    run<2>("v_med3_u32", 8, d);
    run<3>("v_lshl_add_u32", 8, d);
    run<4>("v_mul_f32 (sgpr operand)", 8, d);
    run<5>("v_cmp->sgpr + v_cndmask", 16, d);
    run<6>("v_cmp->vcc + v_cndmask", 16, d);
    run<7>("v_cndmask (sgpr mask)", 8, d);
    run<8>("v_pk_add_f32", 8, d);
    run<10>("v_pk_mul_f32", 8, d);
    run<11>("v_pk_fma_f32", 8, d);
    run<0, 256>("v_add_f32", 8, d);
    run<0, 512>("v_add_f32", 8, d);
    run<8, 256>("v_pk_add_f32", 8, d);
    run<1, 256>("v_min_u32", 8, d);
    return 0;
}
