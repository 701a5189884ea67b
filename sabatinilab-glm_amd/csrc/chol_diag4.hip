// Diagonal-block step of the blocked Cholesky for the factor + explicit-inverse chain
// (sglm_chol_solve_inv): four waves per fit instead of one.
//
// Wave w holds rows r = 4j + w (j = 0..15) of every column of the 64 x 64 block (lane c =
// column c), together with the same rows of V = (U_kk^T)^-1 (eliminated alongside, the panel
// step's operator).  Step Q: the owner wave (Q mod 4) forms the pivot and row Q of U and of V
// and publishes them in LDS; after one barrier every wave applies the rank-1 update to its 16
// rows (rows <= Q see a zero multiplier: U[Q][i] = 0 there).  Per step a wave issues 32 FMAs
// and four broadcast ds_read_b128 instead of the single-wave kernel's ~190 VALU (64 readlane
// broadcasts), and at ~70 VGPRs it co-resides with the gradient kernel that runs beside the
// chain (the single-wave kernel needs 330 and waits for a whole SIMD).  Rows of U and V are
// double-buffered, so one barrier per step suffices.  Pivot rules as chol_diag_kernel: a pivot
// not above 1e-6 of the original diagonal (or a frozen coordinate) is dropped -- U row zero,
// diagonal 1, V row zero -- and counted in info.  The rhs forward solve of chol_diag_kernel is
// not done: the inverse chain solves on the explicit inverse later.
#include "common.h"

namespace sglm {

__device__ __forceinline__ float lane4f(float v, int l) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}

static __global__ void __launch_bounds__(256) chol_diag4_kernel(
    float* __restrict__ Hall, int32_t P, int32_t k0, const int32_t* __restrict__ fits,
    uint8_t* __restrict__ frozen_all, const float* __restrict__ diag_all,
    int32_t* __restrict__ info, float* __restrict__ minv_all, float* __restrict__ Mall) {
    __shared__ __attribute__((aligned(16))) float su[2][64];   // row Q of U, position (i&3)*16 + (i>>2)
    __shared__ float sx[2][64];                                // row Q of V, by column
    __shared__ float sv[64][65];                               // V transposed (Mall row stores)
    const int fit = fits[blockIdx.x];
    float* H = Hall + (int64_t)fit * P * P;
    uint8_t* frz = frozen_all + (int64_t)fit * P + k0;
    const int c = threadIdx.x & 63, w = threadIdx.x >> 6;
    float a[16], v[16];
    {
        int cl = c;                                  // opaque lane index: the selects below are
        asm volatile("" : "+v"(cl));                 // not CSE'd into the steps
        const float* col = H + (int64_t)(k0 + w) * P + k0 + c;
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const float x = col[(int64_t)(4 * j) * P];
            a[j] = 4 * j + w <= cl ? x : 0.0f;
            v[j] = 4 * j + w == cl ? 1.0f : 0.0f;
        }
    }
    int myfrz = frz[c];
    const float thr = 1e-6f * diag_all[(int64_t)fit * P + k0 + c];
    int dropped = 0;
    const int upos = (c & 3) * 16 + (c >> 2);
#pragma unroll
    for (int Q = 0; Q < 64; ++Q) {
        const int buf = Q & 1;
        if (w == (Q & 3)) {                          // wave-uniform: the owner of row Q
            const int jq = Q >> 2;
            const int verdict = (myfrz ? 2 : 0) | (a[jq] > thr ? 0 : 1);
            const int vq = __builtin_amdgcn_readlane(verdict, Q);
            const bool was = (vq & 2) != 0;
            const bool drop = vq != 0;
            const float piv = lane4f(a[jq], Q);
            const float r = drop ? 0.0f : __builtin_amdgcn_rsqf(piv);
            const float d = drop ? 1.0f : piv * r;
            const float u = c > Q ? a[jq] * r : 0.0f;            // U[Q][c]
            a[jq] = c == Q ? d : (c > Q ? u : a[jq]);
            const float xq = v[jq] * r;                          // V[Q][c]
            v[jq] = xq;
            const bool newly = drop && !was && c == Q;
            myfrz = newly ? 1 : myfrz;
            dropped = newly ? 1 : dropped;
            su[buf][upos] = u;
            sx[buf][c] = xq;
        }
        __syncthreads();
        const float uc = su[buf][upos];
        const float xc = sx[buf][c];
        const f32x4* ur = reinterpret_cast<const f32x4*>(&su[buf][w * 16]);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const f32x4 ui = ur[q];                              // U[Q][4j + w], j = 4q..4q+3
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                a[4 * q + e] = fmaf(-ui[e], uc, a[4 * q + e]);
                v[4 * q + e] = fmaf(-ui[e], xc, v[4 * q + e]);
            }
        }
    }
    // whole block (the strictly-lower part is never read); M_kk row-major for the panel step
    float* col = H + (int64_t)(k0 + w) * P + k0 + c;
    float* mo = minv_all + (int64_t)blockIdx.x * 64 * 64 + (int64_t)w * 64 + c;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        col[(int64_t)(4 * j) * P] = a[j];
        mo[j * 4 * 64] = v[j];
        sv[c][4 * j + w] = v[j];
    }
    if ((c & 3) == w) {                              // the owner of step c
        frz[c] = (uint8_t)myfrz;
        if (dropped) atomicAdd(&info[fit], 1);
    }
    if (!Mall) return;
    __syncthreads();
    // explicit inverse's diagonal block: row cc of U_kk^-1 = column cc of V, 16 entries per thread
    const int cc = threadIdx.x >> 2, part = (threadIdx.x & 3) * 16;
    float* mr = Mall + (int64_t)fit * P * P + (int64_t)(k0 + cc) * P + k0 + part;
#pragma unroll
    for (int e = 0; e < 16; e += 4)
        *reinterpret_cast<f32x4*>(mr + e) = f32x4{sv[cc][part + e], sv[cc][part + e + 1],
                                                  sv[cc][part + e + 2], sv[cc][part + e + 3]};
}

void launch_chol_diag4(int nact, hipStream_t s, float* Hall, int32_t P, int32_t k0,
                       const int32_t* fits, uint8_t* frozen_all, const float* diag_all,
                       int32_t* info, float* minv_all, float* Mall) {
    chol_diag4_kernel<<<nact, 256, 0, s>>>(Hall, P, k0, fits, frozen_all, diag_all, info,
                                           minv_all, Mall);
}

}  // namespace sglm
