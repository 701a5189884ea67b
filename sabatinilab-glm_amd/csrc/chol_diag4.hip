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
#include "chol_tile.h"

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

// Four pivots per barrier with look-ahead and packed FMAs (chol_diag4l_kernel, bitwise the
// same factor and inverse as chol_diag4q_kernel).  In diag4q the quad's owner forms its four
// pivots while the other three waves wait at the barrier, and then every wave applies the
// quad's terms: per quad the serial pivot chain and the 128-FMA update run one after the
// other.  Here the owner of the NEXT quad first applies quad Q's terms to its four rows of
// quad Q + 4, forms quad Q + 4's pivots and publishes them (the other buffer), and only then
// applies quad Q's terms to its other rows -- while the other waves apply theirs: the pivot
// chain overlaps the update.  Rows of A and of V are held as pairs (a, v) so that both
// rank-1 terms of an element are one v_pk_fma_f32.  Per element the same FMAs in the same
// order as before, except that a register group whose rows all precede quad Q (16 g + 15 < Q)
// is not sent quad Q's terms: their multipliers U[Q+h][row] are exact zeros there (a no-op up
// to the sign of a zero).  Timestamps inside the kernel (s_memtime, one fit, a probe build):
// per quad ~1,700 clocks, of them ~250 the owner's apply to its next rows, ~820 its four
// pivots, the rest its other rows' applies and the barrier; skipping the dead groups took the
// 1-fit chain 1.00 -> 0.97 ms, 20 fits 2.90 -> 2.86 ms.
typedef float f32x2v __attribute__((ext_vector_type(2)));

// the owner's four pivots of quad Q (rows Q + h in registers 4 (Q >> 4) + h), published into
// one buffer: row multipliers by row position, U and V multipliers by column
__device__ __forceinline__ void diag4l_quad(const int Q, f32x2v (&av)[16], const int c,
                                            const float thr, int& myfrz, int& dropped,
                                            const int rpos, float* srow_b, float* scol_b,
                                            float* sx_b) {
    const int k = 4 * (Q >> 4);
    float u[4], x[4];
#pragma unroll
    for (int h = 0; h < 4; ++h) {
        const int q = Q + h;
        const int verdict = (myfrz ? 2 : 0) | (av[k + h].x > thr ? 0 : 1);
        const int vq = __builtin_amdgcn_readlane(verdict, q);
        const bool drop = vq != 0;
        const bool newly = drop && (vq & 2) == 0 && c == q;
        const float piv = lane4f(av[k + h].x, q);
        const float rr = drop ? 0.0f : __builtin_amdgcn_rsqf(piv);
        const float d = drop ? 1.0f : piv * rr;
        u[h] = c > q ? av[k + h].x * rr : 0.0f;                       // U[q][c]
        av[k + h].x = c == q ? d : (c > q ? u[h] : av[k + h].x);
        x[h] = av[k + h].y * rr;                                      // V[q][c]
        av[k + h].y = x[h];
        myfrz = newly ? 1 : myfrz;
        dropped = newly ? 1 : dropped;
#pragma unroll
        for (int g = h + 1; g < 4; ++g) {
            const float t = lane4f(u[h], Q + g);                      // U[q][Q+g]
            av[k + g].x = fmaf(-t, u[h], av[k + g].x);
            av[k + g].y = fmaf(-t, x[h], av[k + g].y);
        }
    }
#pragma unroll
    for (int h = 0; h < 4; ++h) {
        const bool own_later = c > Q + h && c <= Q + 3;   // already applied by the owner
        srow_b[h * 64 + rpos] = own_later ? 0.0f : u[h];
        scol_b[h * 64 + c] = u[h];
        sx_b[h * 64 + c] = x[h];
    }
}

// quad Q's four terms (buffer b) on register group g (rows of av[4g .. 4g+3])
__device__ __forceinline__ void diag4l_apply(f32x2v (&av)[16], const int g, const float* srow_b,
                                             const float* scol_b, const float* sx_b,
                                             const int w, const int c) {
#pragma unroll
    for (int h = 0; h < 4; ++h) {
        const f32x2v m = {scol_b[h * 64 + c], sx_b[h * 64 + c]};
        const f32x4 ui = reinterpret_cast<const f32x4*>(&srow_b[h * 64 + w * 16])[g];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const f32x2v nu = {-ui[e], -ui[e]};
            av[4 * g + e] = __builtin_elementwise_fma(nu, m, av[4 * g + e]);
        }
    }
}

struct Diag4lSmem {
    __attribute__((aligned(16))) float srow[2][4][64];
    float scol[2][4][64];
    float sx[2][4][64];
    float sv[64][65];
};

// the diagonal step of block k0 for fit `fit` (launch slot `slot`: its block inverse goes to
// minv_all + slot * 64 * 64) by one 256-thread workgroup
__device__ __forceinline__ void diag4l_block(float* __restrict__ Hall, int32_t P, int32_t k0,
                                             int fit, int slot, uint8_t* __restrict__ frozen_all,
                                             const float* __restrict__ diag_all,
                                             int32_t* __restrict__ info,
                                             float* __restrict__ minv_all,
                                             float* __restrict__ Mall, Diag4lSmem& sm) {
    float* H = Hall + (int64_t)fit * P * P;
    uint8_t* frz = frozen_all + (int64_t)fit * P + k0;
    const int c = threadIdx.x & 63, w = threadIdx.x >> 6;
    // register k of wave w holds row 16 (k >> 2) + 4 w + (k & 3)
    f32x2v av[16];
    {
        int cl = c;
        asm volatile("" : "+v"(cl));
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const int r = 16 * (k >> 2) + 4 * w + (k & 3);
            const float x = H[(int64_t)(k0 + r) * P + k0 + c];
            av[k].x = r <= cl ? x : 0.0f;
            av[k].y = r == cl ? 1.0f : 0.0f;
        }
    }
    int myfrz = frz[c];
    const float thr = 1e-6f * diag_all[(int64_t)fit * P + k0 + c];
    int dropped = 0;
    const int rpos = ((c >> 2) & 3) * 16 + 4 * (c >> 4) + (c & 3);
    if (w == 0)
        diag4l_quad(0, av, c, thr, myfrz, dropped, rpos, &sm.srow[0][0][0], &sm.scol[0][0][0],
                    &sm.sx[0][0][0]);
    __syncthreads();
#pragma unroll
    for (int Q = 0; Q < 64; Q += 4) {
        const int buf = (Q >> 2) & 1;
        const float* rb = &sm.srow[buf][0][0];
        const float* cb = &sm.scol[buf][0][0];
        const float* xb = &sm.sx[buf][0][0];
        const int Qn = Q + 4;
        if (Qn < 64 && w == ((Qn >> 2) & 3)) {       // wave-uniform: the next quad's owner
            const int gn = Qn >> 4;
            diag4l_apply(av, gn, rb, cb, xb, w, c);
            diag4l_quad(Qn, av, c, thr, myfrz, dropped, rpos, &sm.srow[buf ^ 1][0][0],
                        &sm.scol[buf ^ 1][0][0], &sm.sx[buf ^ 1][0][0]);
#pragma unroll
            for (int g = 0; g < 4; ++g)
                if (g != gn && 16 * g + 15 >= Q) diag4l_apply(av, g, rb, cb, xb, w, c);
        } else {
#pragma unroll
            for (int g = 0; g < 4; ++g)
                if (16 * g + 15 >= Q) diag4l_apply(av, g, rb, cb, xb, w, c);
        }
        __syncthreads();
    }
    float* mo = minv_all + (int64_t)slot * 64 * 64 + c;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const int r = 16 * (k >> 2) + 4 * w + (k & 3);
        H[(int64_t)(k0 + r) * P + k0 + c] = av[k].x;
        mo[r * 64] = av[k].y;
        sm.sv[c][r] = av[k].y;
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
        *reinterpret_cast<f32x4*>(mr + e) = f32x4{sm.sv[cc][part + e], sm.sv[cc][part + e + 1],
                                                  sm.sv[cc][part + e + 2],
                                                  sm.sv[cc][part + e + 3]};
}

static __global__ void __launch_bounds__(256) chol_diag4l_kernel(
    float* __restrict__ Hall, int32_t P, int32_t k0, const int32_t* __restrict__ fits,
    uint8_t* __restrict__ frozen_all, const float* __restrict__ diag_all,
    int32_t* __restrict__ info, float* __restrict__ minv_all, float* __restrict__ Mall) {
    __shared__ Diag4lSmem sm;
    diag4l_block(Hall, P, k0, fits[blockIdx.x], blockIdx.x, frozen_all, diag_all, info, minv_all,
                 Mall, sm);
}

// The trailing update (chol_tile.h) fused with the NEXT diagonal step: the workgroup of tile
// (s0, s0) -- the first tile of the launch, and the last piece of the next diagonal block --
// factors that block right after updating it, while the other tiles' workgroups run on: one
// launch (and one dependency) fewer per block step, the diagonal step's latency overlapped
// with the rest of the update.  The panel step of block s0 follows the launch.
union UpdDiagSmem {
    float upd[kLUFloats];
    Diag4lSmem diag;
};

static __global__ void __launch_bounds__(256) chol_update_diag4l_kernel(
    float* __restrict__ Hall, int32_t P, int32_t k0, int32_t kc, int32_t s0,
    const int32_t* __restrict__ fits, uint8_t* __restrict__ frozen_all,
    const float* __restrict__ diag_all, int32_t* __restrict__ info, float* __restrict__ minv_all,
    float* __restrict__ Mall) {
    __shared__ UpdDiagSmem sm;
    const int fit = fits[blockIdx.y];
    update_lds_tile(Hall + (int64_t)fit * P * P, P, k0, kc, s0, blockIdx.x, sm.upd);
    if (blockIdx.x != 0) return;
    __syncthreads();                    // the tile's update is visible to the whole workgroup
    diag4l_block(Hall, P, s0 * 64, fit, blockIdx.y, frozen_all, diag_all, info, minv_all, Mall,
                 sm.diag);
}

void launch_chol_update_diag4l(dim3 grid, hipStream_t s, float* Hall, int32_t P, int32_t k0,
                               int32_t kc, int32_t s0, const int32_t* fits, uint8_t* frozen_all,
                               const float* diag_all, int32_t* info, float* minv_all,
                               float* Mall) {
    chol_update_diag4l_kernel<<<grid, 256, 0, s>>>(Hall, P, k0, kc, s0, fits, frozen_all,
                                                   diag_all, info, minv_all, Mall);
}

void launch_chol_diag4l(int nact, hipStream_t s, float* Hall, int32_t P, int32_t k0,
                        const int32_t* fits, uint8_t* frozen_all, const float* diag_all,
                        int32_t* info, float* minv_all, float* Mall) {
    chol_diag4l_kernel<<<nact, 256, 0, s>>>(Hall, P, k0, fits, frozen_all, diag_all, info,
                                            minv_all, Mall);
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
