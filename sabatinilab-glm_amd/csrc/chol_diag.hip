// Diagonal-block step of the blocked Cholesky (chol.hip): one wave per fit factors the 64 x 64
// diagonal block in registers, forms its inverse and forward-solves the block's right-hand
// side.  Its own translation unit: the fully unrolled 64-step register elimination takes the
// device compiler minutes, so edits to the rest of chol.hip do not recompile it.
#include "common.h"

namespace sglm {

constexpr int kNB = 64;

__device__ __forceinline__ float lanef(float v, int l) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}

// rank-1 update of this lane's column by row q of U: a[i] -= U[q][i] * u for i > q, where
// U[q][i] = lane i's u; the same broadcasts carry the elimination into v (lane i's column of
// the block inverse, see chol_diag_kernel): v[i] -= U[q][i] * x_q.  Chunks of 8 readlane + FMA
// pairs behind scheduling fences, so that the scalar broadcasts are consumed as they are
// produced instead of all being hoisted (SGPR spills).
template <int Q>
__device__ __forceinline__ void diag_rank1(float (&a)[kNB], float (&v)[kNB], float u, float xq) {
#pragma unroll
    for (int i0 = Q + 1; i0 < kNB; i0 += 8) {
        float sc[8];                                 // broadcasts first: the readlane ->
#pragma unroll                                       // VALU hazard is covered by distance
        for (int i = i0; i < i0 + 8 && i < kNB; ++i) sc[i - i0] = lanef(u, i);
#pragma unroll
        for (int i = i0; i < i0 + 8 && i < kNB; ++i) {
            a[i] = fmaf(-sc[i - i0], u, a[i]);
            v[i] = fmaf(-sc[i - i0], xq, v[i]);
        }
        __builtin_amdgcn_sched_barrier(0);
    }
}

template <int Q>
__device__ __forceinline__ void diag_steps(float (&a)[kNB], float (&v)[kNB], float& rinv, int c,
                                           float thr, int& myfrz, int& dropped) {
    if constexpr (Q < kNB) {
        // the pivot test runs lane-locally (lane Q's a[Q] against its own threshold) and only
        // its verdict is broadcast: a broadcast of the loop-invariant threshold would be
        // hoisted for all 64 steps and spilled
        const int verdict = (myfrz ? 2 : 0) | (a[Q] > thr ? 0 : 1);
        const int vq = __builtin_amdgcn_readlane(verdict, Q);
        const bool was = (vq & 2) != 0;
        const bool drop = vq != 0;
        // uniform pivot arithmetic: d = sqrt(piv) and its reciprocal from one v_rsq
        const float piv = lanef(a[Q], Q);
        const float r = drop ? 0.0f : __builtin_amdgcn_rsqf(piv);
        const float d = drop ? 1.0f : piv * r;
        const float u = c > Q ? a[Q] * r : 0.0f;     // row Q of U (0 for a dropped pivot)
        a[Q] = c == Q ? d : (c > Q ? u : a[Q]);
        rinv = c == Q ? r : rinv;                    // lane Q keeps 1 / U[Q][Q] (0 if dropped)
        const float xq = v[Q] * r;                   // x_Q of lane c's unit right-hand side
        v[Q] = xq;
        // row Q is final from here on: materialise it now, or its selects sink to the store
        // at the end and keep every step's masks and pivots live (SGPR spills)
        asm volatile("" : "+v"(a[Q]), "+v"(rinv), "+v"(v[Q]));
        const bool newly = drop && !was && c == Q;
        myfrz = newly ? 1 : myfrz;
        dropped = newly ? 1 : dropped;
        diag_rank1<Q>(a, v, u, xq);
        diag_steps<Q + 1>(a, v, rinv, c, thr, myfrz, dropped);
    }
}

// One wave per fit: factor the diagonal block (refactor) and forward-solve the rhs block.
// Lane c holds column c of the block in registers (a[r] = A[k0+r][k0+c]); step q reads the
// pivot and row q of U with v_readlane (scalar broadcasts), so the whole 64-step
// factorisation is register FMAs (entries below the diagonal are updated too and ignored),
// branch-free: lane-dependent choices are selects, pivot decisions are wave-uniform.
static __global__ void __launch_bounds__(64) chol_diag_kernel(
    float* __restrict__ Hall, int32_t P, int32_t k0, const int32_t* __restrict__ fits,
    uint8_t* __restrict__ frozen_all, float* __restrict__ rhs_all,
    const float* __restrict__ diag_all, int32_t* __restrict__ info, int32_t nrefac,
    float* __restrict__ minv_all, float* __restrict__ Mall) {
    const int fit = fits[blockIdx.x];
    const bool refactor = (int)blockIdx.x < nrefac;
    float* H = Hall + (int64_t)fit * P * P;
    uint8_t* frz = frozen_all + (int64_t)fit * P + k0;
    float* rhs = rhs_all + (int64_t)fit * P + k0;
    const int c = threadIdx.x;
    float a[kNB];
    {
        int cl = c;                                  // opaque copies of the lane index keep the
        asm volatile("" : "+v"(cl));                 // load / store masks out of the steps' CSE
#pragma unroll
        for (int r = 0; r < kNB; ++r) {              // whole block (no branches), lower -> 0
            const float v = H[(int64_t)(k0 + r) * P + k0 + c];
            a[r] = r <= cl ? v : 0.0f;
        }
    }
    int myfrz = frz[c];
    // lane q: 1 / U[q][q] (0 for a frozen pivot) -- one VGPR, not 64 uniform SGPRs
    float rinv = 0.0f;
    if (refactor) {
        const float thr = 1e-6f * diag_all[(int64_t)fit * P + k0 + c];
        int dropped = 0;
        // v: lane c's column of M = (U_kk^T)^-1 (rows of frozen coordinates zero), built by
        // eliminating e_c alongside the factorisation -- the panel step's operator
        float v[kNB];
        {
            int ci = c;
            asm volatile("" : "+v"(ci));
#pragma unroll
            for (int r = 0; r < kNB; ++r) v[r] = r == ci ? 1.0f : 0.0f;
        }
        diag_steps<0>(a, v, rinv, c, thr, myfrz, dropped);
        if (dropped) atomicAdd(&info[fit], 1);
        frz[c] = (uint8_t)myfrz;
        // whole block: the strictly-lower part is never read (consumers use row <= column)
#pragma unroll
        for (int r = 0; r < kNB; ++r) H[(int64_t)(k0 + r) * P + k0 + c] = a[r];
        // row-major M[r][i] (lane i writes column i: coalesced rows)
        float* mo = minv_all + (int64_t)blockIdx.x * kNB * kNB + c;
#pragma unroll
        for (int r = 0; r < kNB; ++r) mo[r * kNB] = v[r];
        if (Mall) {
            // the explicit inverse's diagonal block: M_kk = U_kk^-1, row c = this lane's v
            // (v[r] = (U_kk^-T)[r][c]; zero below the diagonal and in frozen columns)
            float* mr = Mall + (int64_t)fit * P * P + (int64_t)(k0 + c) * P + k0;
#pragma unroll
            for (int r = 0; r < kNB; r += 4)
                *reinterpret_cast<f32x4*>(mr + r) = f32x4{v[r], v[r + 1], v[r + 2], v[r + 3]};
        }
    } else {
        float ucc = 1.0f;                            // U[c][c] (selects: no dynamic index)
#pragma unroll
        for (int r = 0; r < kNB; ++r) ucc = r == c ? a[r] : ucc;
        rinv = myfrz ? 0.0f : 1.0f / ucc;
    }
    // forward solve U_kk^T z = rhs_k, lane = row: step q needs 1/U[q][q] and U[q][c] (this
    // lane's a[q]); z_q = 0 for a frozen coordinate (rinv 0)
    float zc = rhs[c];
    int cf = c;
    asm volatile("" : "+v"(cf));                     // opaque copy: the factorisation's lane
                                                     // masks are not CSE'd into 64 live pairs
#pragma unroll
    for (int q = 0; q < kNB; ++q) {
        const float zq = lanef(zc, q) * lanef(rinv, q);
        const float m = cf > q ? a[q] : 0.0f;
        zc = fmaf(-m, zq, zc);
        zc = cf == q ? zq : zc;
    }
    rhs[c] = zc;
}


void launch_chol_diag(int nact, hipStream_t s, float* Hall, int32_t P, int32_t k0,
                      const int32_t* fits, uint8_t* frozen_all, float* rhs_all,
                      const float* diag_all, int32_t* info, int32_t nrefac, float* minv_all,
                      float* Mall) {
    chol_diag_kernel<<<nact, 64, 0, s>>>(Hall, P, k0, fits, frozen_all, rhs_all, diag_all, info,
                                         nrefac, minv_all, Mall);
}

}  // namespace sglm
