// Exhaustive check of csrc/nldpc_sleef.h against ATen's own SLEEF (libtorch_cpu.so exports
// Sleef_tanhf16_u10 / Sleef_atanhf16_u10): every fp32 input with |x| <= 10 (tanh) / |x| < 1 (atanh).
// Build: tools/dev/sleef_probe.sh.  Development tool: needs the CPU torch library, no GPU.
#include <immintrin.h>
#include <stdio.h>
#include <stdint.h>
#include <string.h>
#include "nldpc_sleef.h"

extern "C" __m512 Sleef_tanhf16_u10(__m512);
extern "C" __m512 Sleef_atanhf16_u10(__m512);

template <class REF, class MINE>
static long check(const char* name, uint32_t lo, uint32_t hi, REF ref, MINE mine) {
    long bad = 0, shown = 0;
    alignas(64) float in[16], out[16];
    for (uint64_t u = lo; u <= hi; u += 16) {
        for (int k = 0; k < 16; ++k) {
            uint32_t b = (uint32_t)(u + k > hi ? hi : u + k);
            memcpy(&in[k], &b, 4);
        }
        _mm512_store_ps(out, ref(_mm512_load_ps(in)));
        for (int k = 0; k < 16; ++k) {
            const float m = mine(in[k]);
            uint32_t a, c;
            memcpy(&a, &out[k], 4);
            memcpy(&c, &m, 4);
            if (a != c) {
                ++bad;
                if (shown++ < 8) printf("  %s(%a = %.9g): sleef %a, mine %a\n", name, in[k], in[k], out[k], m);
            }
        }
    }
    printf("%s: %ld mismatches over [%08x, %08x]\n", name, bad, lo, hi);
    return bad;
}

int main() {
    float ten = 10.0f, one_m = 0.99999994f;
    uint32_t t10, a1;
    memcpy(&t10, &ten, 4);
    memcpy(&a1, &one_m, 4);
    long bad = 0;
    bad += check("tanh+", 0u, t10, Sleef_tanhf16_u10, nldpc_sleef::tanhf_u10);
    bad += check("tanh-", 0x80000000u, 0x80000000u | t10, Sleef_tanhf16_u10, nldpc_sleef::tanhf_u10);
    bad += check("atanh+", 0u, a1, Sleef_atanhf16_u10, nldpc_sleef::atanhf_u10);
    bad += check("atanh-", 0x80000000u, 0x80000000u | a1, Sleef_atanhf16_u10, nldpc_sleef::atanhf_u10);
    return bad ? 1 : 0;
}
