// Trailing-update tile of the blocked Cholesky through LDS (chol.hip chol_update_lds_kernel
// and the fused update + diagonal step of chol_diag4.hip share it).
#pragma once
#include "common.h"

namespace sglm {

constexpr int kLU = 68;             // strip row stride (floats)
constexpr int kLUFloats = 2 * 2 * 32 * kLU;   // the two strips, double-buffered

// H[i][j] -= sum_r U[k0+r][i] U[k0+r][j] over r < kc for the 64 x 64 tile t (tiles of the
// trailing upper triangle from block (s0, s0), row by row) of one fit's H: both 64-column
// strips of the panel rows staged through LDS (lds: kLUFloats floats), K in blocks of 32 rows,
// two LDS buffers with the next block's loads in registers during this block's 16 MFMAs per
// wave, one barrier per block.
__device__ __forceinline__ void update_lds_tile(float* __restrict__ H, int32_t P, int32_t k0,
                                                int32_t kc, int32_t s0, int t,
                                                float* __restrict__ lds) {
    float* sa[2] = {lds, lds + 32 * kLU};
    float* sb[2] = {lds + 2 * 32 * kLU, lds + 3 * 32 * kLU};
    const int T = P / 64 - s0;
    int bi = 0, bj;
    {
        int rowlen = T;
        while (t >= rowlen) { t -= rowlen; ++bi; --rowlen; }
        bj = bi + t;
    }
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int r32 = lane & 31, kh = lane >> 5;
    const int wr = wave >> 1, wc = wave & 1;
    const int ca = (s0 + bi) * 64, cb = (s0 + bj) * 64;       // strip columns
    const int lr = tid >> 3, lcol = 8 * (tid & 7);             // this thread's block share
    const float* ga = H + (int64_t)(k0 + lr) * P + ca + lcol;
    const float* gb = H + (int64_t)(k0 + lr) * P + cb + lcol;
    f32x4 ra0, ra1, rb0, rb1;
    auto gload = [&](int r) {
        ra0 = *reinterpret_cast<const f32x4*>(ga + (int64_t)r * P);
        ra1 = *reinterpret_cast<const f32x4*>(ga + (int64_t)r * P + 4);
        rb0 = *reinterpret_cast<const f32x4*>(gb + (int64_t)r * P);
        rb1 = *reinterpret_cast<const f32x4*>(gb + (int64_t)r * P + 4);
    };
    auto sstore = [&](int buf) {
        *reinterpret_cast<f32x4*>(&sa[buf][lr * kLU + lcol]) = ra0;
        *reinterpret_cast<f32x4*>(&sa[buf][lr * kLU + lcol + 4]) = ra1;
        *reinterpret_cast<f32x4*>(&sb[buf][lr * kLU + lcol]) = rb0;
        *reinterpret_cast<f32x4*>(&sb[buf][lr * kLU + lcol + 4]) = rb1;
    };
    f32x16 acc = {};
    gload(0);
    sstore(0);
    __syncthreads();
    int cur = 0;
    for (int r = 0; r < kc; r += 32) {
        const bool more = r + 32 < kc;
        if (more) gload(r + 32);
        const float* A = &sa[cur][kh * kLU + wr * 32 + r32];
        const float* Bq = &sb[cur][kh * kLU + wc * 32 + r32];
#pragma unroll
        for (int u = 0; u < 16; ++u)
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(A[2 * u * kLU], Bq[2 * u * kLU], acc, 0, 0,
                                                       0);
        if (more) sstore(cur ^ 1);
        __syncthreads();
        cur ^= 1;
    }
    const int ci = ca + wr * 32, cj = cb + wc * 32;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
        float* h = &H[(int64_t)(ci + (q & 3) + 8 * (q >> 2) + 4 * kh) * P + cj + r32];
        *h -= acc[q];
    }
}

}  // namespace sglm
