// Batched penalised Newton solve:  (H_k + diag(dshift_k)) delta_k = -g_k.
//
// Replaces the per-iteration linear solve of sklearn's Newton / Ridge paths
// (_newton_solver.py NewtonCholeskySolver.inner_solve -> scipy cho_solve; Ridge
// _solve_cholesky -> linalg.solve(assume_a='pos'), _ridge.py:201-213).
//
// One 256-thread workgroup per fit.  H_k is row-major P x P; only a <= b is read (the
// upper triangle that sglm_syrk writes).  Right-looking blocked Cholesky H = U^T U with
// NB = 64:
//   1. diagonal block factored in LDS by one wave (lane = column, no block barriers);
//   2. row panel U_kj = U_kk^{-T} A_kj, one thread per column j (64-entry register vector);
//      the forward substitution of the right-hand side is fused into this step;
//   3. trailing update A_ij -= U_ki^T U_kj over 64x64 tiles, 4x4 register micro-tiles.
// Then blocked back substitution.  Frozen coordinates (dshift < 0, zero diagonal, or a
// pivot that collapses below 1e-6 of its original diagonal) get delta = 0.
// `refactor` = 0 reuses the factor left in H by a previous call with the same fits
// (constant-Hessian families: Gaussian refinement iterations).
#include "common.h"

namespace sglm {

constexpr int kNB = 64;
constexpr int kCT = 256;
constexpr int kMaxP = 8192;

__global__ void __launch_bounds__(kCT) chol_solve_kernel(
    float* __restrict__ Hall, int32_t P, const int32_t* __restrict__ fits,
    const double* __restrict__ gall, const float* __restrict__ dshift_all,
    float* __restrict__ delta_all, int32_t* __restrict__ info, uint8_t* __restrict__ frozen_all,
    int32_t refactor) {
    __shared__ float sD[kNB][kNB + 1];
    __shared__ __attribute__((aligned(16))) float sPi[kNB][kNB];
    __shared__ __attribute__((aligned(16))) float sPj[kNB][kNB];
    __shared__ float rhs[kMaxP];          // running right-hand side, then x
    __shared__ uint8_t frz[kMaxP];
    __shared__ int ndrop;

    const int fit = fits[blockIdx.x];
    float* H = Hall + (int64_t)fit * P * P;
    const double* g = gall + (int64_t)fit * P;
    const float* dsh = dshift_all + (int64_t)fit * P;
    float* delta = delta_all + (int64_t)fit * P;
    uint8_t* frozen = frozen_all + (int64_t)fit * P;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int nb = P / kNB;

    if (tid == 0) ndrop = 0;
    if (refactor) {
        // ---- pre-pass: penalty shift, frozen coordinates
        for (int j = tid; j < P; j += kCT) {
            const float d = H[(int64_t)j * P + j] + dsh[j];
            const bool f = dsh[j] < 0.0f || !(d > 0.0f);
            frz[j] = f;
            if (!f) H[(int64_t)j * P + j] = d;
        }
        __syncthreads();
        for (int j = 0; j < P; ++j) {
            if (!frz[j]) continue;                       // uniform (LDS flag)
            for (int e = tid; e < P; e += kCT) {
                if (e > j) H[(int64_t)j * P + e] = 0.0f;     // row j, right of diagonal
                if (e < j) H[(int64_t)e * P + j] = 0.0f;     // column j, above diagonal
            }
            if (tid == 0) H[(int64_t)j * P + j] = 1.0f;
        }
    } else {
        for (int j = tid; j < P; j += kCT) frz[j] = frozen[j];
    }
    for (int j = tid; j < P; j += kCT) rhs[j] = frz[j] ? 0.0f : (float)g[j];
    __syncthreads();

    for (int kb = 0; kb < nb; ++kb) {
        const int k0 = kb * kNB;
        // ---- 1. diagonal block
        for (int e = tid; e < kNB * kNB; e += kCT) {
            const int r = e / kNB, c = e % kNB;
            sD[r][c] = (r <= c) ? H[(int64_t)(k0 + r) * P + k0 + c] : 0.0f;
        }
        __syncthreads();
        if (refactor && wave == 0) {
            // lane = column c of the block; rows are walked sequentially
            const int c = lane;
            const float orig = sD[c][c];
            for (int q = 0; q < kNB; ++q) {
                float piv = __shfl(sD[q][c], q, 64);     // sD[q][q]
                const float origq = __shfl(orig, q, 64);
                bool drop = frz[k0 + q] || !(piv > 1e-6f * origq);
                float d = drop ? 1.0f : sqrtf(piv);
                // row q of U: U[q][c] = A[q][c] / d for c > q
                float u = sD[q][c];
                if (c == q) u = d;
                else if (c > q) u = drop ? 0.0f : u / d;
                sD[q][c] = u;
                if (drop && c == q && !frz[k0 + q]) { frz[k0 + q] = 1; atomicAdd(&ndrop, 1); }
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                // trailing: for rows i in (q, c]: A[i][c] -= U[q][i] U[q][c]
                if (c > q) {
                    for (int i = q + 1; i <= c; ++i) sD[i][c] -= sD[q][i] * u;
                }
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            }
        }
        __syncthreads();
        if (refactor) {
            for (int e = tid; e < kNB * kNB; e += kCT) {
                const int r = e / kNB, c = e % kNB;
                if (r <= c) H[(int64_t)(k0 + r) * P + k0 + c] = sD[r][c];
            }
        }
        // forward substitution of the rhs block: U_kk^T z = rhs_k (one wave, lane = row)
        if (wave == 0) {
            float zc = rhs[k0 + lane];
            for (int q = 0; q < kNB; ++q) {
                const float zq = __shfl(zc, q, 64) / sD[q][q];
                const float zz = frz[k0 + q] ? 0.0f : zq;
                if (lane == q) zc = zz;
                else if (lane > q) zc -= sD[q][lane] * zz;
            }
            rhs[k0 + lane] = zc;
        }
        __syncthreads();
        // ---- 2. row panel + rhs update
        for (int j = k0 + kNB + tid; j < P; j += kCT) {
            float x[kNB];
#pragma unroll
            for (int r = 0; r < kNB; ++r) x[r] = H[(int64_t)(k0 + r) * P + j];
            if (refactor) {
#pragma unroll
                for (int c = 0; c < kNB; ++c) {
                    float v = x[c];
#pragma unroll
                    for (int r = 0; r < c; ++r) v -= sD[r][c] * x[r];
                    x[c] = frz[k0 + c] ? 0.0f : v / sD[c][c];
                }
#pragma unroll
                for (int r = 0; r < kNB; ++r) H[(int64_t)(k0 + r) * P + j] = x[r];
            }
            float s = 0.0f;
#pragma unroll
            for (int r = 0; r < kNB; ++r) s += x[r] * rhs[k0 + r];
            rhs[j] -= s;
        }
        __syncthreads();
        if (!refactor) continue;
        // ---- 3. trailing update of the remaining upper triangle
        const int ty = tid >> 4, tx = tid & 15;
        for (int bi = kb + 1; bi < nb; ++bi) {
            for (int e = tid; e < kNB * kNB; e += kCT) {
                const int r = e / kNB, c = e % kNB;
                sPi[r][c] = H[(int64_t)(k0 + r) * P + bi * kNB + c];
            }
            for (int bj = bi; bj < nb; ++bj) {
                for (int e = tid; e < kNB * kNB / 4; e += kCT) {
                    const int r = e / (kNB / 4), c4 = e % (kNB / 4);
                    *reinterpret_cast<f32x4*>(&sPj[r][c4 * 4]) =
                        *reinterpret_cast<const f32x4*>(&H[(int64_t)(k0 + r) * P + bj * kNB + c4 * 4]);
                }
                __syncthreads();
                float acc[4][4] = {};
#pragma unroll 8
                for (int r = 0; r < kNB; ++r) {
                    const f32x4 a = *reinterpret_cast<const f32x4*>(&sPi[r][ty * 4]);
                    const f32x4 b = *reinterpret_cast<const f32x4*>(&sPj[r][tx * 4]);
#pragma unroll
                    for (int u = 0; u < 4; ++u)
#pragma unroll
                        for (int v = 0; v < 4; ++v) acc[u][v] += a[u] * b[v];
                }
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    float* row = &H[(int64_t)(bi * kNB + ty * 4 + u) * P + bj * kNB + tx * 4];
                    f32x4 cur = *reinterpret_cast<f32x4*>(row);
                    cur[0] -= acc[u][0]; cur[1] -= acc[u][1];
                    cur[2] -= acc[u][2]; cur[3] -= acc[u][3];
                    *reinterpret_cast<f32x4*>(row) = cur;
                }
                __syncthreads();
            }
        }
        __syncthreads();
    }

    // ---- back substitution U x = z (rhs holds z), blocks from the bottom
    __shared__ float part[kNB];
    for (int kb = nb - 1; kb >= 0; --kb) {
        const int k0 = kb * kNB;
        // s_r = z_r - sum_{j >= k0+NB} U[k0+r][j] x_j : each wave takes 16 rows
        for (int rr = 0; rr < kNB / 4; ++rr) {
            const int r = wave * (kNB / 4) + rr;
            float s = 0.0f;
            for (int j = k0 + kNB + lane; j < P; j += 64) s += H[(int64_t)(k0 + r) * P + j] * rhs[j];
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
            if (lane == 0) part[r] = s;
        }
        for (int e = tid; e < kNB * kNB; e += kCT) {
            const int r = e / kNB, c = e % kNB;
            sD[r][c] = (r <= c) ? H[(int64_t)(k0 + r) * P + k0 + c] : 0.0f;
        }
        __syncthreads();
        if (wave == 0) {
            float v = rhs[k0 + lane] - part[lane];
            for (int q = kNB - 1; q >= 0; --q) {
                const float xq = frz[k0 + q] ? 0.0f : __shfl(v, q, 64) / sD[q][q];
                if (lane == q) v = xq;
                else if (lane < q) v -= sD[lane][q] * xq;
            }
            rhs[k0 + lane] = v;
        }
        __syncthreads();
    }
    for (int j = tid; j < P; j += kCT) {
        delta[j] = frz[j] ? 0.0f : -rhs[j];
        if (refactor) frozen[j] = frz[j];
    }
    if (tid == 0 && refactor) info[fit] = ndrop;
}

}  // namespace sglm

using namespace sglm;

extern "C" int sglm_chol_solve_ex(float* H, int32_t P, const int32_t* fits, int32_t nact,
                                  const double* g, const float* dshift, float* delta,
                                  int32_t* info, uint8_t* frozen, int32_t refactor,
                                  sglm_stream_t stream) {
    if (nact <= 0) return SGLM_OK;
    if (!H || !fits || !g || !dshift || !delta || !info || !frozen || P % kNB || P > kMaxP) {
        set_error("sglm_chol_solve: bad args (P=%d, max %d)", P, kMaxP);
        return SGLM_EINVAL;
    }
    chol_solve_kernel<<<nact, kCT, 0, as_stream(stream)>>>(H, P, fits, g, dshift, delta, info,
                                                           frozen, refactor);
    return check_launch("chol_solve_kernel");
}
