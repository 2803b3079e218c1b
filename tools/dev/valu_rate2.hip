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
__device__ __forceinline__ void body(float (&a)[16], f2 (&p)[16], uint32_t (&u)[16], float b0, float b1, f2 q0, f2 q1) {
    uint64_t ms[8];
    uint64_t mk;
    asm volatile("s_mov_b64 %0, 0x55" : "=s"(mk));
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
        if constexpr (OP == 11) {  // v_med3_f32 with three VGPR sources
#define MED3V(i) a[i] = __builtin_amdgcn_fmed3f(a[i], a[((i) + 5) & 15], a[((i) + 9) & 15]);
            R16(MED3V)
        }
        if constexpr (OP == 12) {  // v_fma_f32 with three VGPR sources
#define FMAV(i) a[i] = __builtin_fmaf(a[i], a[((i) + 5) & 15], a[((i) + 9) & 15]);
            R16(FMAV)
        }
        if constexpr (OP == 13) {  // v_mul_f32 VGPR x SGPR (the check node's weight product)
#define MULS(i) a[i] = a[i] * bb;
            R16(MULS)
        }
        if constexpr (OP == 14) {  // v_cmp (VGPR vs VGPR -> SGPR pair) + v_cndmask: 8 pairs
#define CSEL(i) if ((i) & 1) { a[i] = (a[(i) ^ 1] < a[((i) + 6) & 15]) ? a[i] : a[((i) + 3) & 15]; }
            R16(CSEL)
        }
        if constexpr (OP == 15) {  // v_max_f32 with |x| modifiers on two VGPR sources
#define MAXA(i) a[i] = __builtin_fmaxf(__builtin_fabsf(a[i]), __builtin_fabsf(a[((i) + 7) & 15]));
            R16(MAXA)
        }
        if constexpr (OP == 16) {  // v_min_f32_e64 |x|, |y| (inline asm, VOP3 with abs modifiers)
#define MINAA(i) asm("v_min_f32_e64 %0, |%0|, |%1|" : "+v"(a[i]) : "v"(a[((i) + 7) & 15]));
            R16(MINAA)
        }
        if constexpr (OP == 17) {  // v_cndmask_b32_e64 with a fixed SGPR-pair mask
#define CNDS(i) asm("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(a[i]) : "v"(a[((i) + 7) & 15]), "s"(mk));
            R16(CNDS)
        }
        if constexpr (OP == 18) {  // v_cmp_lt_f32_e64 into 8 rotating SGPR pairs (results xor-ed once per group)
#define CMPS(i) asm volatile("v_cmp_lt_f32_e64 %0, %1, %2" : "=s"(ms[(i) & 7]) : "v"(a[i]), "v"(a[((i) + 7) & 15]));
            R16(CMPS)
            a[0] = (ms[0] ^ ms[3] ^ ms[5]) & 1 ? a[0] : a[1];
        }
        if constexpr (OP == 19) {  // v_max_f32_e32 0, x (the ReLU)
#define MAX0(i) asm("v_max_f32_e32 %0, 0, %0" : "+v"(a[i]));
            R16(MAX0)
        }
        if constexpr (OP == 20) {  // v_min3_f32 with three VGPR sources
#define MIN3V(i) asm("v_min3_f32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(a[((i) + 5) & 15]), "v"(a[((i) + 9) & 15]));
            R16(MIN3V)
        }
        if constexpr (OP == 21) {  // v_med3_f32 with an |x| modifier and two VGPR sources + constant
#define MED3K(i) asm("v_med3_f32 %0, %0, 0, |%1|" : "+v"(a[i]) : "v"(a[((i) + 5) & 15]));
            R16(MED3K)
        }
        if constexpr (OP == 22) {  // v_cmp_eq_f32_e64 |x|, y into 8 rotating SGPR pairs
#define CMPE(i) asm volatile("v_cmp_eq_f32_e64 %0, |%1|, %2" : "=s"(ms[(i) & 7]) : "v"(a[i]), "v"(a[((i) + 7) & 15]));
            R16(CMPE)
            a[0] = (ms[0] ^ ms[3] ^ ms[5]) & 1 ? a[0] : a[1];
        }
        if constexpr (OP == 23) {  // v_add_f32_e32, two VGPR sources, asm (compare with the C form)
#define ADDV(i) asm("v_add_f32_e32 %0, %0, %1" : "+v"(a[i]) : "v"(a[((i) + 7) & 15]));
            R16(ADDV)
        }
        if constexpr (OP == 24) {
#define X24(i) asm("v_add_u32_e32 %0, %0, %1" : "+v"(u[i]) : "v"(u[((i) + 7) & 15]));
            R16(X24)
        }
        if constexpr (OP == 25) {
#define X25(i) asm("v_xor_b32_e32 %0, %0, %1" : "+v"(u[i]) : "v"(u[((i) + 7) & 15]));
            R16(X25)
        }
        if constexpr (OP == 26) {
#define X26(i) asm("v_and_b32_e32 %0, %0, %1" : "+v"(u[i]) : "v"(u[((i) + 7) & 15]));
            R16(X26)
        }
        if constexpr (OP == 27) {
#define X27(i) asm("v_bfi_b32 %0, %1, %0, %2" : "+v"(u[i]) : "v"(u[((i) + 3) & 15]), "v"(u[((i) + 7) & 15]));
            R16(X27)
        }
        if constexpr (OP == 28) {
#define X28(i) asm("v_lshlrev_b32_e32 %0, 1, %0" : "+v"(u[i]));
            R16(X28)
        }
        if constexpr (OP == 29) {
#define X29(i) asm("v_med3_u32 %0, %0, %1, %2" : "+v"(u[i]) : "v"(u[((i) + 3) & 15]), "v"(u[((i) + 7) & 15]));
            R16(X29)
        }
        if constexpr (OP == 30) {
#define X30(i) asm("v_min_u32_e32 %0, %0, %1" : "+v"(u[i]) : "v"(u[((i) + 7) & 15]));
            R16(X30)
        }
        if constexpr (OP == 31) {
#define X31(i) asm("v_mov_b32_e32 %0, %1" : "=v"(u[i]) : "v"(u[((i) + 7) & 15]));
            R16(X31)
        }
        if constexpr (OP == 32) {
#define X32(i) asm("v_sub_u32_e32 %0, %0, %1" : "+v"(u[i]) : "v"(u[((i) + 7) & 15]));
            R16(X32)
        }
        if constexpr (OP == 33) {
#define X33(i) asm("v_add_f32_e64 %0, %0, |%1|" : "+v"(a[i]) : "v"(a[((i) + 7) & 15]));
            R16(X33)
        }
        if constexpr (OP == 34) {
#define X34(i) asm("v_fmac_f32_e32 %0, %1, %2" : "+v"(a[i]) : "v"(a[((i) + 7) & 15]), "v"(a[((i) + 3) & 15]));
            R16(X34)
        }
        if constexpr (OP == 35) {
#define X35(i) asm("v_add3_u32 %0, %0, %1, %2" : "+v"(u[i]) : "v"(u[((i) + 3) & 15]), "v"(u[((i) + 7) & 15]));
            R16(X35)
        }
        if constexpr (OP == 36) {
#define X36(i) asm("v_and_or_b32 %0, %0, %1, %2" : "+v"(u[i]) : "v"(u[((i) + 3) & 15]), "v"(u[((i) + 7) & 15]));
            R16(X36)
        }
        if constexpr (OP == 37) {
#define X37(i) asm("v_lshl_add_u32 %0, %0, 1, %1" : "+v"(u[i]) : "v"(u[((i) + 7) & 15]));
            R16(X37)
        }
        if constexpr (OP == 38) {
#define X38(i) asm("v_cvt_f32_u32_e32 %0, %1" : "=v"(a[i]) : "v"(u[((i) + 7) & 15]));
            R16(X38)
        }
        if constexpr (OP == 39) {
#define X39(i) asm("v_mul_f32_e64 %0, %0, -%1" : "+v"(a[i]) : "v"(a[((i) + 7) & 15]));
            R16(X39)
        }
        if constexpr (OP == 40) {
#define X40(i) asm("v_sub_f32_e32 %0, %0, %1" : "+v"(a[i]) : "v"(a[((i) + 7) & 15]));
            R16(X40)
        }
        if constexpr (OP == 41) {
#define X41(i) asm("v_ldexp_f32 %0, %0, %1" : "+v"(a[i]) : "v"(u[((i) + 7) & 15]));
            R16(X41)
        }
        if constexpr (OP == 42) {
#define X42(i) asm("v_mul_u32_u24_e32 %0, %0, %1" : "+v"(u[i]) : "v"(u[((i) + 7) & 15]));
            R16(X42)
        }
        if constexpr (OP == 43) {
#define X43(i) asm("v_perm_b32 %0, %0, %1, %2" : "+v"(u[i]) : "v"(u[((i) + 3) & 15]), "v"(u[((i) + 7) & 15]));
            R16(X43)
        }
        asm volatile("" : "+v"(a[0]), "+v"(p[0]), "+v"(u[0]));  // keep the groups from folding across trips
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
    uint32_t u[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) u[i] = __float_as_uint(a[i]) * 2654435761u;
    for (int r = 0; r < R; ++r) body<OP>(a, p, u, b0, b1, q0, q1);
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * (TPB / 64) + threadIdx.x / 64] = t1 - t0;
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) s += a[i] + p[i].x + p[i].y + (float)(u[i] & 1023);
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
    run<OP, 1024>(name, d, dc);
    run<OP, 1024, 2>(name, d, dc);
}

int main(int argc, char**) {
    float* d;
    unsigned long long* dc;
    (void)hipMalloc(&d, 512 * 1024 * 4);
    (void)hipMalloc(&dc, 512 * 16 * 8);
    if (argc < 2) {  // (r3 first pass; "valu_rate2 2" runs the second set only)
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
    sweep<11>("v_med3_f32 (3 VGPR sources)", d, dc);
    sweep<12>("v_fma_f32 (3 VGPR sources)", d, dc);
    sweep<13>("v_mul_f32 (VGPR x SGPR)", d, dc);
    sweep<14>("v_cmp + v_cndmask (per pair: 2 instr)", d, dc);
    }
    if (argc == 3) {
    sweep<24>("v_add_u32_e32", d, dc);
    sweep<25>("v_xor_b32_e32", d, dc);
    sweep<26>("v_and_b32_e32", d, dc);
    sweep<27>("v_bfi_b32", d, dc);
    sweep<28>("v_lshlrev_b32_e32", d, dc);
    sweep<29>("v_med3_u32", d, dc);
    sweep<30>("v_min_u32_e32", d, dc);
    sweep<31>("v_mov_b32_e32", d, dc);
    sweep<32>("v_sub_u32_e32", d, dc);
    sweep<33>("v_add_f32_e64 |x|", d, dc);
    sweep<34>("v_fmac_f32_e32", d, dc);
    sweep<35>("v_add3_u32", d, dc);
    sweep<36>("v_and_or_b32", d, dc);
    sweep<37>("v_lshl_add_u32", d, dc);
    sweep<38>("v_cvt_f32_u32", d, dc);
    sweep<39>("v_mul_f32_e64 -x", d, dc);
    sweep<40>("v_sub_f32_e32", d, dc);
    sweep<41>("v_ldexp_f32", d, dc);
    sweep<42>("v_mul_u32_u24", d, dc);
    sweep<43>("v_perm_b32", d, dc);
    return 0;
    }
    sweep<16>("v_min_f32_e64 |x|,|y| (asm)", d, dc);
    sweep<17>("v_cndmask_b32_e64 (SGPR mask)", d, dc);
    sweep<18>("v_cmp_lt_f32_e64 -> SGPR", d, dc);
    sweep<19>("v_max_f32_e32 0, x", d, dc);
    sweep<20>("v_min3_f32 (3 VGPR)", d, dc);
    sweep<21>("v_med3_f32 x, 0, |y|", d, dc);
    sweep<22>("v_cmp_eq_f32_e64 |x|, y -> SGPR", d, dc);
    sweep<23>("v_add_f32_e32 (asm, 2 VGPR)", d, dc);
    return 0;
}
