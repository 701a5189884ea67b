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

}  // namespace sglm
