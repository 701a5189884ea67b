// Shared helpers for the libsglm_hip kernels (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>
#include <stdio.h>
#include "../../include/sglm_hip.h"

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

namespace sglm {

void set_error(const char* fmt, ...);

inline hipStream_t as_stream(sglm_stream_t s) { return reinterpret_cast<hipStream_t>(s); }

// Check the launch of the kernel just issued.
int check_launch(const char* what);

constexpr int kWave = 64;

__device__ __forceinline__ float bf16_bits_to_f32(uint16_t b) {
    return __uint_as_float(static_cast<uint32_t>(b) << 16);
}

// Per-sample half-Tweedie loss pieces (sklearn/_loss/loss.py), single precision.
// family 0: 0.5 (eta - y)^2 (identity); family 1: HalfTweedieLoss(power), log link.
struct LossOut { float loss, g, h; };

__device__ __forceinline__ LossOut half_loss(int family, float power, float y, float eta) {
    LossOut o;
    if (family == SGLM_FAM_SQUARED) {
        float r = eta - y;
        o.loss = 0.5f * r * r; o.g = r; o.h = 1.0f;
    } else if (power == 1.0f) {
        float mu = __expf(eta);
        o.loss = mu - y * eta; o.g = mu - y; o.h = mu;
    } else if (power == 2.0f) {
        float e = __expf(-eta);
        o.loss = eta + y * e; o.g = 1.0f - y * e; o.h = y * e;
    } else {
        float a = __expf((2.0f - power) * eta);
        float b = __expf((1.0f - power) * eta);
        o.loss = a / (2.0f - power) - y * b / (1.0f - power);
        o.g = a - y * b;
        o.h = (2.0f - power) * a - (1.0f - power) * y * b;
    }
    return o;
}

// double-precision loss for reductions that decide line searches / scores
__device__ __forceinline__ double half_loss_d(int family, double power, double y, double eta) {
    if (family == SGLM_FAM_SQUARED) { double r = eta - y; return 0.5 * r * r; }
    if (power == 1.0) return exp(eta) - y * eta;
    if (power == 2.0) return eta + y * exp(-eta);
    return exp((2.0 - power) * eta) / (2.0 - power) - y * exp((1.0 - power) * eta) / (1.0 - power);
}

__device__ __forceinline__ double inv_link_d(int family, double eta) {
    return family == SGLM_FAM_SQUARED ? eta : exp(eta);
}

__device__ __forceinline__ double wave_sum_d(double v) {
    #pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// ---- bit-plane designs (Gram v6, eta/xtr on MFMA) -----------------------------------
// Inside a 32-bit word, element rho (row or predictor) sits at bit
// 4*(rho/8) + (rho%8)/2 + 16*(rho%2): the dword of MFMA fragment elements (2j, 2j+1) of 8-element
// chunk g has its two bits at p = 4g + j and p + 16, so
//   rotr(word, p - 14) & 0x40004000  = two bf16 values 2.0 / 0.0   (2 VALU)
//   pk_ashr_i16(rotr(word, p - 15), 15) = two 16-bit masks          (2 VALU)
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const u32x2 g_uint2;
typedef __attribute__((address_space(1))) const u32x4 g_uint4;
typedef short s16x2 __attribute__((ext_vector_type(2)));

// generic -> global address-space pointer (lets the compiler emit global_load)
template <typename G>
__device__ __forceinline__ G* as_global(const void* p) {
    return reinterpret_cast<G*>(reinterpret_cast<uintptr_t>(p));
}

__device__ __forceinline__ uint32_t rotr32(uint32_t x, uint32_t s) {
    return __builtin_amdgcn_alignbit(x, x, s);
}

// source element of target bit t (0..31) of a fragment-ordered word
__device__ __forceinline__ int frag_bit_source(int t) {
    const int tt = t & 15;
    return 8 * (tt >> 2) + 2 * (tt & 3) + (t >> 4);
}

// logical block id whose consecutive values share an XCD (blocks b and b + 8 do)
__device__ __forceinline__ int xcd_logical(int w, int nwg) {
    const int q = nwg / 8, r = nwg % 8, x = w % 8, l = w / 8;
    return x < r ? x * (q + 1) + l : r * (q + 1) + (x - r) * q + l;
}

// bf16 2.0/0 fragment (8 elements of chunk q = 2*ks + h) from a 64-element word pair
__device__ __forceinline__ bf16x8 frag_two(u32x2 w, int ks, int h) {
    const uint32_t word = ks < 2 ? w.x : w.y;
    const uint32_t p0 = 8 * (ks & 1) + 4 * h;
    uint32_t d[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) d[j] = rotr32(word, (p0 + j + 18) & 31) & 0x40004000u;
    return __builtin_bit_cast(bf16x8, make_uint4(d[0], d[1], d[2], d[3]));
}

// Loads in inline asm so LLVM cannot sink a prefetch to its use (it does for plain loads);
// the consumer must first run an asm "s_waitcnt vmcnt(0)" that ties the loaded registers.
__device__ __forceinline__ u32x2 gld2(g_uint2* p) {
    u32x2 v;
    asm volatile("global_load_dwordx2 %0, %1, off" : "=v"(v) : "v"(p) : "memory");
    return v;
}
// wave-uniform 64-bit base in an SGPR pair + per-lane 32-bit byte offset + immediate: no VALU
// address arithmetic (the per-step advance is scalar)
template <int IMM>
__device__ __forceinline__ u32x2 gld2s(uint64_t sbase, uint32_t voff) {
    u32x2 v;
    asm volatile("global_load_dwordx2 %0, %1, %2 offset:%3"
                 : "=v"(v)
                 : "v"(voff), "s"(sbase), "i"(IMM)
                 : "memory");
    return v;
}
template <int IMM>
__device__ __forceinline__ u32x4 gld4s(uint64_t sbase, uint32_t voff) {
    u32x4 v;
    asm volatile("global_load_dwordx4 %0, %1, %2 offset:%3"
                 : "=v"(v)
                 : "v"(voff), "s"(sbase), "i"(IMM)
                 : "memory");
    return v;
}
__device__ __forceinline__ u32x4 gld4(g_uint4* p) {
    u32x4 v;
    asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(v) : "v"(p) : "memory");
    return v;
}

// three bf16 pieces hi + mid + lo == x exactly (f32 has 24 significand bits)
__device__ __forceinline__ void split3(float x, __bf16& hi, __bf16& mid, __bf16& lo) {
    hi = (__bf16)x;
    const float r1 = x - (float)hi;
    mid = (__bf16)r1;
    lo = (__bf16)(r1 - (float)mid);
}

}  // namespace sglm
