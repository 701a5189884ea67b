// AVX-512 inner loops of the host-side helpers (host.hip), compiled by g++ with per-function
// target attributes and chosen at run time (sglm_host_simd_level): the GPU box's EPYC and the
// build container both have AVX-512; a CPU without it takes host.hip's scalar loops.
#include <immintrin.h>
#include <stdint.h>

extern "C" int sglm_host_simd_level(void) {
    __builtin_cpu_init();
    return (__builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512bw")) ? 1 : 0;
}

// One row range [r0, r1) (r0 % 32 == 0) of a row-major float64 block (column c at base + c, row
// stride S): bit r of bits[c * nwords + r / 32] = (value == 1.0); bad[c] |= a value other than
// 0.0 / 1.0 (NaN included); cnt[c] += the 1.0 count.  16 columns per vector: two 8-double
// compares per row make one 16-bit mask, OR-ed into the 16 column words at bit k.
extern "C" __attribute__((target("avx512f,avx512bw"))) void sglm_host_pack_block_avx512(
    const double* base, int64_t S, int32_t ncols, int64_t r0, int64_t r1, int64_t nwords,
    uint32_t* bits, uint8_t* bad, int64_t* cnt) {
    const int ng = (ncols + 15) / 16;
    const __m512d one = _mm512_set1_pd(1.0), zero = _mm512_setzero_pd();
    __m512i wd[16];                                   // ncols <= 256 per call
    __mmask16 badm[16];
    alignas(64) uint32_t tmp[16];
    for (int g = 0; g < ng; ++g) badm[g] = 0;
    for (int64_t w0 = r0; w0 < r1; w0 += 32) {
        for (int g = 0; g < ng; ++g) wd[g] = _mm512_setzero_si512();
        const int64_t e = (r1 - w0) < 32 ? (r1 - w0) : 32;
        for (int64_t k = 0; k < e; ++k) {
            const double* row = base + (w0 + k) * S;
            const __m512i bit = _mm512_set1_epi32((int)(1u << k));
            for (int g = 0; g < ng; ++g) {
                const int c0 = 16 * g;
                const int rem = ncols - c0;
                const __mmask8 lo = rem >= 8 ? (__mmask8)0xff : (__mmask8)((1u << rem) - 1u);
                const __mmask8 hi = rem >= 16 ? (__mmask8)0xff
                                  : rem > 8 ? (__mmask8)((1u << (rem - 8)) - 1u) : (__mmask8)0;
                const __m512d a = _mm512_maskz_loadu_pd(lo, row + c0);
                const __m512d b = _mm512_maskz_loadu_pd(hi, row + c0 + 8);
                const __mmask8 a1 = _mm512_cmp_pd_mask(a, one, _CMP_EQ_OQ);
                const __mmask8 b1 = _mm512_cmp_pd_mask(b, one, _CMP_EQ_OQ);
                const __mmask8 a0 = _mm512_cmp_pd_mask(a, zero, _CMP_EQ_OQ);
                const __mmask8 b0 = _mm512_cmp_pd_mask(b, zero, _CMP_EQ_OQ);
                const __mmask16 m1 = (__mmask16)(a1 | ((unsigned)b1 << 8));
                const __mmask16 ok = (__mmask16)((a0 | a1) | ((unsigned)(b0 | b1) << 8));
                const __mmask16 valid = (__mmask16)(lo | ((unsigned)hi << 8));
                badm[g] |= (__mmask16)(valid & ~ok);
                wd[g] = _mm512_mask_or_epi32(wd[g], m1, wd[g], bit);
            }
        }
        for (int g = 0; g < ng; ++g) {
            _mm512_store_si512((__m512i*)tmp, wd[g]);
            const int nc = ncols - 16 * g < 16 ? ncols - 16 * g : 16;
            for (int j = 0; j < nc; ++j) {
                bits[(int64_t)(16 * g + j) * nwords + w0 / 32] = tmp[j];
                cnt[16 * g + j] += __builtin_popcount(tmp[j]);
            }
        }
    }
    for (int g = 0; g < ng; ++g) {
        const int nc = ncols - 16 * g < 16 ? ncols - 16 * g : 16;
        for (int j = 0; j < nc; ++j) bad[16 * g + j] |= (uint8_t)((badm[g] >> j) & 1u);
    }
}
