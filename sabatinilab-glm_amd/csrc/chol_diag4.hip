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
    // per buffer and step h of the pair: the row multipliers U[Q+h][i] at position rpos(i)
    // (row Q+1 zeroed in step 0's: the owner applied that term itself), the column multipliers
    // U[Q+h][c] and V[Q+h][c] by column
    __shared__ __attribute__((aligned(16))) float srow[2][2][64];
    __shared__ float scol[2][2][64];
    __shared__ float sx[2][2][64];
    __shared__ float sv[64][65];                               // V transposed (Mall row stores)
    const int fit = fits[blockIdx.x];
    float* H = Hall + (int64_t)fit * P * P;
    uint8_t* frz = frozen_all + (int64_t)fit * P + k0;
    const int c = threadIdx.x & 63, w = threadIdx.x >> 6;
    // register k of wave w holds row 8 (k >> 1) + 2 w + (k & 1)
    float a[16], v[16];
    {
        int cl = c;                                  // opaque lane index: the selects below are
        asm volatile("" : "+v"(cl));                 // not CSE'd into the steps
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const int r = 8 * (k >> 1) + 2 * w + (k & 1);
            const float x = H[(int64_t)(k0 + r) * P + k0 + c];
            a[k] = r <= cl ? x : 0.0f;
            v[k] = r == cl ? 1.0f : 0.0f;
        }
    }
    int myfrz = frz[c];
    const float thr = 1e-6f * diag_all[(int64_t)fit * P + k0 + c];
    int dropped = 0;
    const int rpos = ((c >> 1) & 3) * 16 + 2 * (c >> 3) + (c & 1);
#pragma unroll
    for (int Q = 0; Q < 64; Q += 2) {
        const int buf = (Q >> 1) & 1;
        if (w == ((Q >> 1) & 3)) {                   // wave-uniform: the owner of rows Q, Q+1
            const int k = 2 * (Q >> 3);              // row Q in a[k], row Q+1 in a[k + 1]
            // step Q
            int verdict = (myfrz ? 2 : 0) | (a[k] > thr ? 0 : 1);
            int vq = __builtin_amdgcn_readlane(verdict, Q);
            bool drop = vq != 0;
            bool newly = drop && (vq & 2) == 0 && c == Q;
            float piv = lane4f(a[k], Q);
            float r = drop ? 0.0f : __builtin_amdgcn_rsqf(piv);
            float d = drop ? 1.0f : piv * r;
            const float u0 = c > Q ? a[k] * r : 0.0f;            // U[Q][c]
            a[k] = c == Q ? d : (c > Q ? u0 : a[k]);
            const float x0 = v[k] * r;                           // V[Q][c]
            v[k] = x0;
            myfrz = newly ? 1 : myfrz;
            dropped = newly ? 1 : dropped;
            // its term on row Q+1 (this wave's own row)
            const float t = lane4f(u0, Q + 1);                  // U[Q][Q+1]
            a[k + 1] = fmaf(-t, u0, a[k + 1]);
            v[k + 1] = fmaf(-t, x0, v[k + 1]);
            // step Q+1
            verdict = (myfrz ? 2 : 0) | (a[k + 1] > thr ? 0 : 1);
            vq = __builtin_amdgcn_readlane(verdict, Q + 1);
            drop = vq != 0;
            newly = drop && (vq & 2) == 0 && c == Q + 1;
            piv = lane4f(a[k + 1], Q + 1);
            r = drop ? 0.0f : __builtin_amdgcn_rsqf(piv);
            d = drop ? 1.0f : piv * r;
            const float u1 = c > Q + 1 ? a[k + 1] * r : 0.0f;    // U[Q+1][c]
            a[k + 1] = c == Q + 1 ? d : (c > Q + 1 ? u1 : a[k + 1]);
            const float x1 = v[k + 1] * r;                       // V[Q+1][c]
            v[k + 1] = x1;
            myfrz = newly ? 1 : myfrz;
            dropped = newly ? 1 : dropped;
            srow[buf][0][rpos] = c == Q + 1 ? 0.0f : u0;
            srow[buf][1][rpos] = u1;
            scol[buf][0][c] = u0;
            scol[buf][1][c] = u1;
            sx[buf][0][c] = x0;
            sx[buf][1][c] = x1;
        }
        __syncthreads();
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const float uc = scol[buf][h][c];
            const float xc = sx[buf][h][c];
            const f32x4* ur = reinterpret_cast<const f32x4*>(&srow[buf][h][w * 16]);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const f32x4 ui = ur[q];                          // U[Q+h][row of a[4q + e]]
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    a[4 * q + e] = fmaf(-ui[e], uc, a[4 * q + e]);
                    v[4 * q + e] = fmaf(-ui[e], xc, v[4 * q + e]);
                }
            }
        }
    }
    // whole block (the strictly-lower part is never read); M_kk row-major for the panel step
    float* mo = minv_all + (int64_t)blockIdx.x * 64 * 64 + c;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const int r = 8 * (k >> 1) + 2 * w + (k & 1);
        H[(int64_t)(k0 + r) * P + k0 + c] = a[k];
        mo[r * 64] = v[k];
        sv[c][r] = v[k];
    }
    if (((c >> 1) & 3) == w) {                       // the owner of step c
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

// The same step with FOUR pivots per barrier (chol_diag4q_kernel): wave w holds rows
// 16 j + 4 w + e (register 4 j + e), so the four rows Q .. Q+3 of a step are one wave's; the
// owner forms the four pivots in order, applying each one's term to its own later rows of the
// quad (readlane of U[Q+h][Q+g]), and publishes the four rows of U and V; after ONE barrier
// every wave applies the four rank-1 terms in pivot order.  Per element the same FMAs in the
// same order as chol_diag4_kernel (bitwise equal factor and inverse), 16 barriers instead of 32.
static __global__ void __launch_bounds__(256) chol_diag4q_kernel(
    float* __restrict__ Hall, int32_t P, int32_t k0, const int32_t* __restrict__ fits,
    uint8_t* __restrict__ frozen_all, const float* __restrict__ diag_all,
    int32_t* __restrict__ info, float* __restrict__ minv_all, float* __restrict__ Mall) {
    // per buffer and pivot h of the quad: the row multipliers U[Q+h][i] at position rpos(i)
    // (rows of the quad after h zeroed: the owner applied those terms itself), the column
    // multipliers U[Q+h][c] and V[Q+h][c] by column
    __shared__ __attribute__((aligned(16))) float srow[2][4][64];
    __shared__ float scol[2][4][64];
    __shared__ float sx[2][4][64];
    __shared__ float sv[64][65];
    const int fit = fits[blockIdx.x];
    float* H = Hall + (int64_t)fit * P * P;
    uint8_t* frz = frozen_all + (int64_t)fit * P + k0;
    const int c = threadIdx.x & 63, w = threadIdx.x >> 6;
    // register k of wave w holds row 16 (k >> 2) + 4 w + (k & 3)
    float a[16], v[16];
    {
        int cl = c;
        asm volatile("" : "+v"(cl));
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const int r = 16 * (k >> 2) + 4 * w + (k & 3);
            const float x = H[(int64_t)(k0 + r) * P + k0 + c];
            a[k] = r <= cl ? x : 0.0f;
            v[k] = r == cl ? 1.0f : 0.0f;
        }
    }
    int myfrz = frz[c];
    const float thr = 1e-6f * diag_all[(int64_t)fit * P + k0 + c];
    int dropped = 0;
    const int rpos = ((c >> 2) & 3) * 16 + 4 * (c >> 4) + (c & 3);
#pragma unroll
    for (int Q = 0; Q < 64; Q += 4) {
        const int buf = (Q >> 2) & 1;
        if (w == ((Q >> 2) & 3)) {                   // wave-uniform: the owner of rows Q..Q+3
            const int k = 4 * (Q >> 4);              // row Q + h in a[k + h]
            float u[4], x[4];
#pragma unroll
            for (int h = 0; h < 4; ++h) {
                const int q = Q + h;
                const int verdict = (myfrz ? 2 : 0) | (a[k + h] > thr ? 0 : 1);
                const int vq = __builtin_amdgcn_readlane(verdict, q);
                const bool drop = vq != 0;
                const bool newly = drop && (vq & 2) == 0 && c == q;
                const float piv = lane4f(a[k + h], q);
                const float rr = drop ? 0.0f : __builtin_amdgcn_rsqf(piv);
                const float d = drop ? 1.0f : piv * rr;
                u[h] = c > q ? a[k + h] * rr : 0.0f;                   // U[q][c]
                a[k + h] = c == q ? d : (c > q ? u[h] : a[k + h]);
                x[h] = v[k + h] * rr;                                  // V[q][c]
                v[k + h] = x[h];
                myfrz = newly ? 1 : myfrz;
                dropped = newly ? 1 : dropped;
                // its terms on the quad's later rows (this wave's own)
#pragma unroll
                for (int g = h + 1; g < 4; ++g) {
                    const float t = lane4f(u[h], Q + g);              // U[q][Q+g]
                    a[k + g] = fmaf(-t, u[h], a[k + g]);
                    v[k + g] = fmaf(-t, x[h], v[k + g]);
                }
            }
#pragma unroll
            for (int h = 0; h < 4; ++h) {
                // the quad's rows after h already carry pivot h's term
                const bool own_later = c > Q + h && c <= Q + 3;
                srow[buf][h][rpos] = own_later ? 0.0f : u[h];
                scol[buf][h][c] = u[h];
                sx[buf][h][c] = x[h];
            }
        }
        __syncthreads();
#pragma unroll
        for (int h = 0; h < 4; ++h) {
            const float uc = scol[buf][h][c];
            const float xc = sx[buf][h][c];
            const f32x4* ur = reinterpret_cast<const f32x4*>(&srow[buf][h][w * 16]);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const f32x4 ui = ur[q];                          // U[Q+h][row of a[4q + e]]
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    a[4 * q + e] = fmaf(-ui[e], uc, a[4 * q + e]);
                    v[4 * q + e] = fmaf(-ui[e], xc, v[4 * q + e]);
                }
            }
        }
    }
    float* mo = minv_all + (int64_t)blockIdx.x * 64 * 64 + c;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const int r = 16 * (k >> 2) + 4 * w + (k & 3);
        H[(int64_t)(k0 + r) * P + k0 + c] = a[k];
        mo[r * 64] = v[k];
        sv[c][r] = v[k];
    }
    if (((c >> 2) & 3) == w) {                       // the owner of step c
        frz[c] = (uint8_t)myfrz;
        if (dropped) atomicAdd(&info[fit], 1);
    }
    if (!Mall) return;
    __syncthreads();
    const int cc = threadIdx.x >> 2, part = (threadIdx.x & 3) * 16;
    float* mr = Mall + (int64_t)fit * P * P + (int64_t)(k0 + cc) * P + k0 + part;
#pragma unroll
    for (int e = 0; e < 16; e += 4)
        *reinterpret_cast<f32x4*>(mr + e) = f32x4{sv[cc][part + e], sv[cc][part + e + 1],
                                                  sv[cc][part + e + 2], sv[cc][part + e + 3]};
}

void launch_chol_diag4q(int nact, hipStream_t s, float* Hall, int32_t P, int32_t k0,
                        const int32_t* fits, uint8_t* frozen_all, const float* diag_all,
                        int32_t* info, float* minv_all, float* Mall) {
    chol_diag4q_kernel<<<nact, 256, 0, s>>>(Hall, P, k0, fits, frozen_all, diag_all, info,
                                            minv_all, Mall);
}

void launch_chol_diag4(int nact, hipStream_t s, float* Hall, int32_t P, int32_t k0,
                       const int32_t* fits, uint8_t* frozen_all, const float* diag_all,
                       int32_t* info, float* minv_all, float* Mall) {
    chol_diag4_kernel<<<nact, 256, 0, s>>>(Hall, P, k0, fits, frozen_all, diag_all, info,
                                           minv_all, Mall);
}

}  // namespace sglm
