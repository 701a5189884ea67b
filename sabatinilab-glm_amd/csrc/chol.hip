// Batched penalised Newton solve:  (H_k + diag(dshift_k)) delta_k = -g_k.
//
// Replaces the per-iteration linear solve of sklearn's Newton / Ridge paths
// (_newton_solver.py NewtonCholeskySolver.inner_solve -> scipy cho_solve; Ridge
// _solve_cholesky -> linalg.solve(assume_a='pos'), _ridge.py:201-213).
//
// H_k is row-major P x P; only a <= b is read (the upper triangle sglm_syrk writes).
// Right-looking blocked Cholesky H = U^T U, NB = 64, spread over many workgroups so that a
// handful of fits still fills the chip (8-GPU runs hold ~15 fits per rank):
//   prep    (1 WG / fit)            penalty shift, frozen coordinates, rhs = g
//   per block column kb:
//     diag  (1 wave / fit)          U_kk in LDS (lane = column), forward solve z_k
//     panel (fits x column chunks)  U_kj = U_kk^-T A_kj (thread = column), rhs_j -= U_kj.z_k
//     update(fits x 64x64 tiles)    A_ij -= U_ki^T U_kj, 4x4 register micro-tiles
//   back    (1 WG of 1024 / fit)    right-looking blocked back substitution, delta = -x
// Frozen coordinates (dshift < 0, zero diagonal, or a pivot collapsing below 1e-6 of its
// original diagonal) get delta = 0.  refactor = 0 reuses the factor and frozen set left in
// H by a previous call (kept Hessians, constant-Hessian Gaussian refinement): only the two
// triangular solves run (chol_fwd2 / chol_back2).
#include <cstdlib>
#include <cstring>
#include <functional>
#include <map>
#include <mutex>
#include <vector>

#include "common.h"
#include "chol_tile.h"

namespace sglm {

constexpr int kNB = 64;
constexpr int kCT = 256;
constexpr int kMaxP = 8192;

// chol_diag.hip
void launch_chol_diag(int nact, hipStream_t s, float* Hall, int32_t P, int32_t k0,
                      const int32_t* fits, uint8_t* frozen_all, float* rhs_all,
                      const float* diag_all, int32_t* info, int32_t nrefac, float* minv_all,
                      float* Mall);
void launch_chol_diag4(int nact, hipStream_t s, float* Hall, int32_t P, int32_t k0,
                       const int32_t* fits, uint8_t* frozen_all, const float* diag_all,
                       int32_t* info, float* minv_all, float* Mall);

void launch_chol_diag4q(int nact, hipStream_t s, float* Hall, int32_t P, int32_t k0,
                        const int32_t* fits, uint8_t* frozen_all, const float* diag_all,
                        int32_t* info, float* minv_all, float* Mall);
void launch_chol_diag4l(int nact, hipStream_t s, float* Hall, int32_t P, int32_t k0,
                        const int32_t* fits, uint8_t* frozen_all, const float* diag_all,
                        int32_t* info, float* minv_all, float* Mall);
void launch_chol_update_diag4l(dim3 grid, hipStream_t s, float* Hall, int32_t P, int32_t k0,
                               int32_t kc, int32_t s0, const int32_t* fits, uint8_t* frozen_all,
                               const float* diag_all, int32_t* info, float* minv_all,
                               float* Mall);

// Four pivots per barrier in the four-wave diagonal step (chol_diag4q_kernel, bitwise the same
// factor; the default: chain of 1 / 20 representatives 1.10 -> 1.07 / 2.53 -> 2.50 ms, C4 grid
// 47.95 -> 47.67 ms in an A/B on one box); SGLM_DIAG4Q=0 for two (read per chain capture; part
// of the chain-graph key).
static bool diag4q() {
    const char* e = getenv("SGLM_DIAG4Q");
    return !(e && e[0] == '0');
}

// The four-pivot step with look-ahead and packed FMAs (chol_diag4l_kernel, bitwise the same
// factor); SGLM_DIAG4L=0 for chol_diag4q_kernel (read per chain capture; part of the key).
static bool diag4l() {
    const char* e = getenv("SGLM_DIAG4L");
    return !(e && e[0] == '0');
}

// The trailing update fused with the next diagonal step (chol_update_diag4l_kernel; with
// chol_diag4l_kernel, bitwise the same factor); SGLM_UPD_DIAG=0 launches them separately
// (read per chain capture; part of the key).
static bool upd_diag() {
    const char* e = getenv("SGLM_UPD_DIAG");
    return !(e && e[0] == '0');
}

// Four-wave diagonal step (chol_diag4.hip) in the factor + inverse chain; SGLM_DIAG4=0 keeps
// the single-wave kernel (comparison runs).
static bool diag4() {
    static const bool v = [] {
        const char* e = getenv("SGLM_DIAG4");
        return !(e && e[0] == '0');
    }();
    return v;
}

// rhs/z/x scratch per fit lives in `work` (float, [B][P]); the original diagonal in
// `work + B*P` (float, [B][P]); the dropped-pivot counter is info[].

__global__ void __launch_bounds__(kCT) chol_prep_kernel(
    float* __restrict__ Hall, int32_t P, const int32_t* __restrict__ fits,
    const double* __restrict__ gall, const float* __restrict__ dshift_all,
    uint8_t* __restrict__ frozen_all, float* __restrict__ rhs_all, float* __restrict__ diag_all,
    int32_t* __restrict__ info, int32_t nrefac) {
    const int fit = fits[blockIdx.x];
    const bool refactor = (int)blockIdx.x < nrefac;
    float* H = Hall + (int64_t)fit * P * P;
    const float* dsh = dshift_all + (int64_t)fit * P;
    uint8_t* frz = frozen_all + (int64_t)fit * P;
    float* rhs = rhs_all + (int64_t)fit * P;
    float* dg = diag_all + (int64_t)fit * P;
    const int tid = threadIdx.x;
    if (refactor) {
        if (tid == 0) info[fit] = 0;
        for (int j = tid; j < P; j += kCT) {
            const float d = H[(int64_t)j * P + j] + dsh[j];
            const bool f = dsh[j] < 0.0f || !(d > 0.0f);
            frz[j] = f;
            dg[j] = f ? 1.0f : d;
            H[(int64_t)j * P + j] = f ? 1.0f : d;
        }
    }
    if (!gall) return;                      // solves on the explicit inverse read g themselves
    const double* g = gall + (int64_t)fit * P;
    __syncthreads();
    for (int j = tid; j < P; j += kCT) rhs[j] = frz[j] ? 0.0f : (float)g[j];
}

// Frozen rows / columns of the refactored fits' upper triangles set to the identity's: one
// 64 x 64 tile per workgroup (tiles of the upper triangle, row by row), nothing written where
// neither the tile's rows nor its columns hold a frozen coordinate.
__global__ void __launch_bounds__(kCT) chol_freeze_kernel(float* __restrict__ Hall, int32_t P,
                                                          const int32_t* __restrict__ fits,
                                                          const uint8_t* __restrict__ frozen_all) {
    const int fit = fits[blockIdx.y];
    float* H = Hall + (int64_t)fit * P * P;
    const uint8_t* frz = frozen_all + (int64_t)fit * P;
    int t = blockIdx.x, bi = 0;
    {
        int rowlen = P / kNB;
        while (t >= rowlen) { t -= rowlen; ++bi; --rowlen; }
    }
    const int bj = bi + t;
    __shared__ uint8_t fr[kNB], fc[kNB];
    __shared__ int any;
    const int tid = threadIdx.x;
    if (tid == 0) any = 0;
    __syncthreads();
    if (tid < kNB) {
        fr[tid] = frz[bi * kNB + tid];
        if (fr[tid]) any = 1;
    } else if (tid < 2 * kNB) {
        fc[tid - kNB] = frz[bj * kNB + tid - kNB];
        if (fc[tid - kNB]) any = 1;
    }
    __syncthreads();
    if (!any) return;
    const int c = tid & 63;
    for (int r = tid >> 6; r < kNB; r += kCT / 64) {
        const int i = bi * kNB + r, j = bj * kNB + c;
        if (i > j || !(fr[r] | fc[c])) continue;
        H[(int64_t)i * P + j] = i == j ? 1.0f : 0.0f;
    }
}

// Right-hand sides of fits solved on ANOTHER slot's factor (engine.irls cross-mask Hessian
// sharing): rhs[fit] = g[fit] * rscale, zero on the factor's frozen coordinates.
__global__ void __launch_bounds__(kCT) chol_alias_prep_kernel(
    int32_t P, const int32_t* __restrict__ fits, const int32_t* __restrict__ fsrc,
    const double* __restrict__ gall, const float* __restrict__ rscale,
    const uint8_t* __restrict__ frozen_all, float* __restrict__ rhs_all) {
    const int fit = fits[blockIdx.x];
    const uint8_t* frz = frozen_all + (int64_t)fsrc[blockIdx.x] * P;
    const double* g = gall + (int64_t)fit * P;
    float* rhs = rhs_all + (int64_t)fit * P;
    const double sc = (double)rscale[blockIdx.x];
    for (int j = threadIdx.x; j < P; j += kCT) rhs[j] = frz[j] ? 0.0f : (float)(g[j] * sc);
}

__device__ __forceinline__ float lanef(float v, int l) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}

// Panel: block row k0 of U for columns j >= k0+NB, X = M B (M from the diagonal step, B the
// block row as the trailing updates left it) as a 64 x 64-tile GEMM on v_mfma_f32_32x32x2f32
// (exact f32 products): one 64-column tile per workgroup, one 32 x 32 quadrant per wave, the
// whole K = 64 operand set loaded up front (lower-triangular M: the upper row half stops at
// K = 32).  The same pass applies the block to the right-hand side, rhs[j] -= sum_r X[r][j] z[r]
// (z = the block's forward-solved rhs); kept-factor slots only do that with their stored rows.
__global__ void __launch_bounds__(kCT) chol_panel_kernel(
    float* __restrict__ Hall, int32_t P, int32_t k0, const int32_t* __restrict__ fits,
    const float* __restrict__ minv_all, float* __restrict__ rhs_all, int32_t nrefac) {
    __shared__ float zs[kNB];
    __shared__ float sred[2][kNB];
    const int slot = blockIdx.x;
    const int fit = fits[slot];
    const bool refactor = slot < nrefac;
    float* H = Hall + (int64_t)fit * P * P;
    float* rhs = rhs_all + (int64_t)fit * P;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int r32 = lane & 31, kh = lane >> 5;
    const int rh = wave >> 1, ch = wave & 1;
    const int j0 = k0 + kNB + blockIdx.y * kNB;        // P and k0 are multiples of 64
    const int j = j0 + ch * 32 + r32;
    if (tid < kNB) zs[tid] = rhs[k0 + tid];
    float b[32];
    const float* pb = H + (int64_t)(k0 + kh) * P + j;
#pragma unroll
    for (int u = 0; u < 32; ++u) b[u] = pb[(int64_t)(2 * u) * P];
    __syncthreads();
    float s = 0.0f;
    if (refactor) {
        const float* pm = minv_all + (int64_t)slot * kNB * kNB + (rh * 32 + r32) * kNB + kh;
        float m[32];
#pragma unroll
        for (int u = 0; u < 32; ++u) m[u] = (rh || u < 16) ? pm[2 * u] : 0.0f;
        f32x16 acc = {};
#pragma unroll
        for (int u = 0; u < 16; ++u)
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(m[u], b[u], acc, 0, 0, 0);
        if (rh) {
#pragma unroll
            for (int u = 16; u < 32; ++u)
                acc = __builtin_amdgcn_mfma_f32_32x32x2f32(m[u], b[u], acc, 0, 0, 0);
        }
        __syncthreads();                             // every wave has consumed its B rows
        // X[row i][col j]: reg q -> i = (q&3) + 8(q>>2) + 4*kh within the quadrant
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            const int i = rh * 32 + (q & 3) + 8 * (q >> 2) + 4 * kh;
            H[(int64_t)(k0 + i) * P + j] = acc[q];
            s = fmaf(acc[q], zs[i], s);
        }
    } else if (rh == 0) {
#pragma unroll
        for (int u = 0; u < 32; ++u) s = fmaf(b[u], zs[2 * u + kh], s);
    }
    s += __shfl_xor(s, 32, 64);
    if (kh == 0) sred[rh][ch * 32 + r32] = s;
    __syncthreads();
    if (tid < kNB) rhs[j0 + tid] -= sred[0][tid] + sred[1][tid];
}

// Trailing update of the upper triangle with `kc` rows of U (64 for a look-ahead band, up to
// kLA*64 when a group of block steps is folded into one pass over the trailing matrix), blocks
// counted from s0.  One 64x64 tile per workgroup,
// one 32x32 quadrant per wave on v_mfma_f32_32x32x2f32 (exact f32 products, f32 accumulate),
// operands loaded straight from the panel rows (L2-resident: grid x = tile, so one fit's
// tiles run together), no LDS.  D[i][j] = sum_r U[k0+r][i] U[k0+r][j]; H[i][j] -= D.
template <bool PIPE>
__global__ void __launch_bounds__(kCT) chol_update_kernel(float* __restrict__ Hall, int32_t P,
                                                          int32_t k0, int32_t kc, int32_t s0,
                                                          const int32_t* __restrict__ fits) {
    const int fit = fits[blockIdx.y];
    float* H = Hall + (int64_t)fit * P * P;
    const int T = P / kNB - s0;
    // tiles row by row from block (s0, s0): the grid size alone selects the whole trailing
    // triangle or only its first few block rows (the look-ahead band)
    int t = blockIdx.x, bi = 0, bj;
    {
        int rowlen = T;
        while (t >= rowlen) { t -= rowlen; ++bi; --rowlen; }
        bj = bi + t;
    }
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int r32 = lane & 31, kh = lane >> 5;
    const int ci = (s0 + bi) * kNB + (wave >> 1) * 32;
    const int cj = (s0 + bj) * kNB + (wave & 1) * 32;
    const float* pa = H + (int64_t)(k0 + kh) * P + ci + r32;
    const float* pb = H + (int64_t)(k0 + kh) * P + cj + r32;
    f32x16 acc = {};
    if (!PIPE) {
        for (int r = 0; r < kc; r += 16) {
            float av[8], bv[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                av[u] = pa[(int64_t)(r + 2 * u) * P];
                bv[u] = pb[(int64_t)(r + 2 * u) * P];
            }
#pragma unroll
            for (int u = 0; u < 8; ++u)
                acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av[u], bv[u], acc, 0, 0, 0);
        }
    } else {
        // two register stages of 16 rows (kc is a multiple of 64): the next stage's 16 loads
        // are in flight while this stage's 8 MFMAs run
        float a0[8], b0[8], a1[8], b1[8];
#define SGLM_UPD_LOAD(A, B, R)                                                             \
    _Pragma("unroll") for (int u = 0; u < 8; ++u) {                                        \
        A[u] = pa[(int64_t)((R) + 2 * u) * P];                                             \
        B[u] = pb[(int64_t)((R) + 2 * u) * P];                                             \
    }
#define SGLM_UPD_MMA(A, B)                                                                 \
    _Pragma("unroll") for (int u = 0; u < 8; ++u)                                          \
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(A[u], B[u], acc, 0, 0, 0);
        SGLM_UPD_LOAD(a0, b0, 0)
        for (int r = 0; r < kc; r += 32) {
            SGLM_UPD_LOAD(a1, b1, r + 16)
            SGLM_UPD_MMA(a0, b0)
            if (r + 32 < kc) {
                SGLM_UPD_LOAD(a0, b0, r + 32)
            }
            SGLM_UPD_MMA(a1, b1)
        }
#undef SGLM_UPD_LOAD
#undef SGLM_UPD_MMA
    }
    // D[row i][col j]: reg q -> i = (q&3) + 8(q>>2) + 4*kh, j = r32
#pragma unroll
    for (int q = 0; q < 16; ++q) {
        float* h = &H[(int64_t)(ci + (q & 3) + 8 * (q >> 2) + 4 * kh) * P + cj + r32];
        *h -= acc[q];
    }
}

// The trailing update with both 64-column strips of the panel rows staged through LDS
// (the default): K in blocks of 32 rows, each strip loaded once per workgroup with float4
// row loads (the register variant has every wave fetch its own 32 columns of both strips, so
// each crosses L2 twice, as scalar loads), two LDS buffers with the next block's loads in
// registers during this block's 16 MFMAs per wave, one barrier per block (chol_tile.h).
__global__ void __launch_bounds__(kCT) chol_update_lds_kernel(float* __restrict__ Hall,
                                                              int32_t P, int32_t k0, int32_t kc,
                                                              int32_t s0,
                                                              const int32_t* __restrict__ fits) {
    __shared__ __attribute__((aligned(16))) float lds[kLUFloats];
    const int fit = fits[blockIdx.y];
    update_lds_tile(Hall + (int64_t)fit * P * P, P, k0, kc, s0, blockIdx.x, lds);
}

// Triangular solves on a stored factor, right-looking, one 1024-thread workgroup per fit: per
// 64-block, wave 0 solves the 64 x 64 diagonal triangle (readlane broadcasts, branch-free),
// then all 16 waves fold the solved block into the rest of the right-hand side, which stays in
// LDS.  The factor is streamed once with many loads in flight: forward, each thread takes 4
// consecutive columns of the block's 64-row panel (float4 per row, coalesced per row);
// backward, 16 lanes share one row of the block's 64-column slab (float4 each, a 16-lane
// shuffle reduction), 64 rows per pass.
constexpr int kST = 1024;

__device__ __forceinline__ void tri_lower_solve64(const float* __restrict__ H, int32_t P,
                                                  int k0, const uint8_t* __restrict__ frz,
                                                  float* z, int lane) {
    // U_kk^T z_k = r_k (lane = column c of U_kk; a[q] = U[k0+q][k0+c] for q < c, else 0)
    const float* blk = H + (int64_t)k0 * P + k0 + lane;
    const float ucc = blk[(int64_t)lane * P];
    float a[kNB];
    int cl = lane;
    asm volatile("" : "+v"(cl));
#pragma unroll
    for (int q = 0; q < kNB; ++q) {
        const float hv = blk[(int64_t)q * P];
        a[q] = q < cl ? hv : 0.0f;
    }
    const float rinv = frz[k0 + lane] ? 0.0f : 1.0f / ucc;
    float v = z[k0 + lane];
    int cf = lane;
    asm volatile("" : "+v"(cf));
#pragma unroll
    for (int q = 0; q < kNB; ++q) {
        const float zq = lanef(v * rinv, q);
        v = fmaf(-a[q], zq, v);
        v = cf == q ? zq : v;
    }
    z[k0 + lane] = v;
}

__device__ __forceinline__ void tri_upper_solve64(const float* __restrict__ H, int32_t P,
                                                  int k0, const uint8_t* __restrict__ frz,
                                                  float* x, int lane) {
    // U_kk x_k = r_k (lane = row r of U_kk; row[q] = U[k0+r][k0+q] for q > r, else 0)
    const float* blk = H + (int64_t)(k0 + lane) * P + k0;
    const float urr = blk[lane];
    float row[kNB];
    int cl = lane;
    asm volatile("" : "+v"(cl));
#pragma unroll
    for (int q = 0; q < kNB; ++q) {
        const float hv = blk[q];
        row[q] = q > cl ? hv : 0.0f;
    }
    const float rd = frz[k0 + lane] ? 0.0f : 1.0f / urr;
    float v = x[k0 + lane];
    int l = lane;
    asm volatile("" : "+v"(l));
#pragma unroll
    for (int q = kNB - 1; q >= 0; --q) {
        const float xq = lanef(v * rd, q);
        v = fmaf(-row[q], xq, v);
        v = l == q ? xq : v;
    }
    x[k0 + lane] = v;
}

__global__ void __launch_bounds__(kST) chol_fwd2_kernel(
    const float* __restrict__ Hall, int32_t P, const int32_t* __restrict__ fits,
    const int32_t* __restrict__ fsrc, const uint8_t* __restrict__ frozen_all,
    float* __restrict__ rhs_all) {
    __shared__ float z[kMaxP];
    const int fit = fits[blockIdx.x];
    const int src = fsrc ? fsrc[blockIdx.x] : fit;    // slot holding the factor
    const float* H = Hall + (int64_t)src * P * P;
    const uint8_t* frz = frozen_all + (int64_t)src * P;
    float* rhs = rhs_all + (int64_t)fit * P;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    for (int j = tid; j < P; j += kST) z[j] = rhs[j];
    const int nb = P / kNB;
    for (int kb = 0; kb < nb; ++kb) {
        const int k0 = kb * kNB;
        __syncthreads();
        if (wave == 0) tri_lower_solve64(H, P, k0, frz, z, lane);
        __syncthreads();
        const int c0 = k0 + kNB;
        const float* pan = H + (int64_t)k0 * P;
        for (int j = c0 + 4 * tid; j < P; j += 4 * kST) {
            f32x4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll 16
            for (int q = 0; q < kNB; ++q) {
                const f32x4 u = *reinterpret_cast<const f32x4*>(pan + (int64_t)q * P + j);
                const float zq = z[k0 + q];
                acc += u * zq;
            }
            z[j] -= acc[0];
            z[j + 1] -= acc[1];
            z[j + 2] -= acc[2];
            z[j + 3] -= acc[3];
        }
    }
    __syncthreads();
    for (int j = tid; j < P; j += kST) rhs[j] = z[j];
}

__global__ void __launch_bounds__(kST) chol_back2_kernel(
    const float* __restrict__ Hall, int32_t P, const int32_t* __restrict__ fits,
    const int32_t* __restrict__ fsrc, const uint8_t* __restrict__ frozen_all,
    const float* __restrict__ rhs_all, float* __restrict__ delta_all) {
    __shared__ float x[kMaxP];
    const int fit = fits[blockIdx.x];
    const int src = fsrc ? fsrc[blockIdx.x] : fit;
    const float* H = Hall + (int64_t)src * P * P;
    const uint8_t* frz = frozen_all + (int64_t)src * P;
    const float* z = rhs_all + (int64_t)fit * P;
    float* delta = delta_all + (int64_t)fit * P;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int sub = tid & 15;                         // float4 slot of a 64-column row slab
    for (int j = tid; j < P; j += kST) x[j] = z[j];
    const int nb = P / kNB;
    for (int kb = nb - 1; kb >= 0; --kb) {
        const int k0 = kb * kNB;
        __syncthreads();
        if (wave == 0) tri_upper_solve64(H, P, k0, frz, x, lane);
        __syncthreads();
        const f32x4 xk = *reinterpret_cast<const f32x4*>(&x[k0 + 4 * sub]);
        for (int r0 = 0; r0 < k0; r0 += kST / 16) {
            const int r = r0 + (tid >> 4);
            f32x4 u = {0.0f, 0.0f, 0.0f, 0.0f};
            if (r < k0) u = *reinterpret_cast<const f32x4*>(H + (int64_t)r * P + k0 + 4 * sub);
            float d = u[0] * xk[0] + u[1] * xk[1] + u[2] * xk[2] + u[3] * xk[3];
#pragma unroll
            for (int o = 8; o > 0; o >>= 1) d += __shfl_xor(d, o, 16);
            if (r < k0 && sub == 0) x[r] -= d;
        }
    }
    __syncthreads();
    for (int j = tid; j < P; j += kST) delta[j] = frz[j] ? 0.0f : -x[j];
}


// ---- explicit inverse of the factor and the solves on it -----------------------------------
// M = U^-1 (upper triangular, frozen / dropped-pivot columns zero), stored row-major per slot
// in Mall.  The diagonal blocks come from chol_diag_kernel; the rest by recursive doubling over
// aligned super-blocks [[A, B], [0, C]] of size 2s (s = 64, 128, ...):
//     (U^-1)_AC = -M_A (B M_C),
// two 64 x 64-tile GEMM launches per level (T = B M_C, then X = -M_A T), log2(P/64) levels.
// A solve is then two GEMMs over the right-hand sides sharing a factor, Y = G M and
// delta = -Y M^T -- full-chip launches instead of a 32-step substitution chain per solve.
//
// Wave tile: 32 x 32 on v_mfma_f32_32x32x2f32 (exact f32 products, f32 accumulation).  K is
// consumed in chunks of 8 with the lane -> k assignment k = kc + 4 kh + u (u = 0..3) for both
// operands, so a lane's A operands are 4 consecutive k of one row (one 16-byte load) and its
// B operands 4 rows of one column (coalesced 128-byte rows across the 32 lanes).

// one level of the recursive doubling; STEP 0: T = B M_C (scratch), STEP 1: X = -M_A T (into M);
// one 64 x 64 tile per workgroup, one 32 x 32 quadrant per wave over the whole K range (an
// unrolled and a split-K variant both measured slower on the C4 chains)
template <int STEP, bool PIPE>
__global__ void __launch_bounds__(kCT) chol_inv_level_kernel(const float* __restrict__ Hall,
                                                             float* __restrict__ Mall,
                                                             float* __restrict__ Tall,
                                                             int32_t P, int32_t s,
                                                             const int32_t* __restrict__ fits,
                                                             int64_t tcap) {
    const int fit = fits[blockIdx.y];
    const float* H = Hall + (int64_t)fit * P * P;
    float* M = Mall + (int64_t)fit * P * P;
    const int sb = s / kNB;
    int t = blockIdx.x;
    const int pair = t / (sb * sb);
    t -= pair * sb * sb;
    const int ti = t / sb, tj = t - ti * sb;
    const int a0 = 2 * s * pair, c0 = a0 + s;
    const int cs = min(s, P - c0);
    if (cs <= 0 || tj * kNB >= cs) return;
    float* T = Tall + (int64_t)blockIdx.y * tcap + (int64_t)pair * s * s;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int r32 = lane & 31, kh = lane >> 5;
    const int i0 = ti * kNB + (wave >> 1) * 32;        // quadrant rows / cols (local)
    const int j0 = tj * kNB + (wave & 1) * 32;
    const float* pa;
    const float* pb;
    int64_t ldb;
    int klo, khi;
    if (STEP == 0) {                                   // A = U[a0 + i][c0 + k], B = M[c0 + k][c0 + j]
        pa = H + (int64_t)(a0 + i0 + r32) * P + c0;
        pb = M + (int64_t)c0 * P + c0 + j0 + r32;
        ldb = P;
        klo = 0;
        khi = (tj + 1) * kNB;                          // M_C upper triangular
    } else {                                           // A = M[a0 + i][a0 + k], B = T[k][j]
        pa = M + (int64_t)(a0 + i0 + r32) * P + a0;
        pb = T + j0 + r32;
        ldb = s;
        klo = ti * kNB;                                // M_A upper triangular
        khi = s;
    }
    f32x16 acc = {};
    if (!PIPE) {
        for (int kc = klo; kc < khi; kc += 8) {
            const f32x4 a = *reinterpret_cast<const f32x4*>(pa + kc + 4 * kh);
            float b[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) b[u] = pb[(int64_t)(kc + 4 * kh + u) * ldb];
#pragma unroll
            for (int u = 0; u < 4; ++u)
                acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[u], b[u], acc, 0, 0, 0);
        }
    } else {
        // K in blocks of 32 through two register stages (klo and khi are multiples of 64):
        // block b+1's 20 loads are in flight while block b's 16 MFMAs run, instead of every
        // 4-MFMA chunk waiting out a full load latency
        f32x4 a0[4], a1[4];
        float b0[4][4], b1[4][4];
#define SGLM_INV_LOAD(A, B, KC)                                                            \
    _Pragma("unroll") for (int v = 0; v < 4; ++v) {                                        \
        const int k = (KC) + 8 * v + 4 * kh;                                               \
        A[v] = *reinterpret_cast<const f32x4*>(pa + k);                                    \
        _Pragma("unroll") for (int u = 0; u < 4; ++u) B[v][u] = pb[(int64_t)(k + u) * ldb]; \
    }
#define SGLM_INV_MMA(A, B)                                                                 \
    _Pragma("unroll") for (int v = 0; v < 4; ++v)                                          \
        _Pragma("unroll") for (int u = 0; u < 4; ++u)                                      \
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(A[v][u], B[v][u], acc, 0, 0, 0);
        SGLM_INV_LOAD(a0, b0, klo)
        for (int kc = klo; kc < khi; kc += 64) {
            SGLM_INV_LOAD(a1, b1, kc + 32)
            SGLM_INV_MMA(a0, b0)
            if (kc + 64 < khi) {
                SGLM_INV_LOAD(a0, b0, kc + 64)
            }
            SGLM_INV_MMA(a1, b1)
        }
#undef SGLM_INV_LOAD
#undef SGLM_INV_MMA
    }
#pragma unroll
    for (int q = 0; q < 16; ++q) {
        const int i = i0 + (q & 3) + 8 * (q >> 2) + 4 * kh, j = j0 + r32;
        if (STEP == 0)
            T[(int64_t)i * s + j] = acc[q];
        else
            M[(int64_t)(a0 + i) * P + c0 + j] = -acc[q];
    }
}

// The same level with the 64 x 64 tile's operands staged through LDS (the default): K in
// blocks of 32, A [64][32] and B [32][64] loaded once per workgroup (the register variant has
// every wave fetch its own 32 rows and 32 columns, so each operand crosses L2 twice), two LDS
// buffers with the next block's global loads in registers while this block's 16 MFMAs per wave
// run, one barrier per block.
constexpr int kLA = 36;             // A row stride (floats): 16-byte aligned rows
constexpr int kLB = 72;             // B row stride: the two k-halves of a wave on disjoint banks
template <int STEP>
__global__ void __launch_bounds__(kCT) chol_inv_level_lds_kernel(const float* __restrict__ Hall,
                                                                 float* __restrict__ Mall,
                                                                 float* __restrict__ Tall,
                                                                 int32_t P, int32_t s,
                                                                 const int32_t* __restrict__ fits,
                                                                 int64_t tcap) {
    __shared__ __attribute__((aligned(16))) float sa[2][64 * kLA];
    __shared__ __attribute__((aligned(16))) float sb[2][32 * kLB];
    const int fit = fits[blockIdx.y];
    const float* H = Hall + (int64_t)fit * P * P;
    float* M = Mall + (int64_t)fit * P * P;
    const int nsb = s / kNB;
    int t = blockIdx.x;
    const int pair = t / (nsb * nsb);
    t -= pair * nsb * nsb;
    const int ti = t / nsb, tj = t - ti * nsb;
    const int a0 = 2 * s * pair, c0 = a0 + s;
    const int cs = min(s, P - c0);
    if (cs <= 0 || tj * kNB >= cs) return;
    float* T = Tall + (int64_t)blockIdx.y * tcap + (int64_t)pair * s * s;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int r32 = lane & 31, kh = lane >> 5;
    const int wr = wave >> 1, wc = wave & 1;
    // global operand bases: A rows (64 of them, stride P), B rows k (stride ldb), 64 columns
    const float* ga;
    const float* gb;
    int64_t ldb;
    int klo, khi;
    if (STEP == 0) {                                   // A = U[a0 + i][c0 + k], B = M[c0 + k][c0 + j]
        ga = H + (int64_t)(a0 + ti * kNB) * P + c0;
        gb = M + (int64_t)c0 * P + c0 + tj * kNB;
        ldb = P;
        klo = 0;
        khi = (tj + 1) * kNB;
    } else {                                           // A = M[a0 + i][a0 + k], B = T[k][j]
        ga = M + (int64_t)(a0 + ti * kNB) * P + a0;
        gb = T + tj * kNB;
        ldb = s;
        klo = ti * kNB;
        khi = s;
    }
    // this thread's share of a block: A row tid>>2, k 8*(tid&3) .. +7; B row k = tid>>3,
    // columns 8*(tid&7) .. +7
    const int ar = tid >> 2, ak = 8 * (tid & 3);
    const int bk = tid >> 3, bj = 8 * (tid & 7);
    f32x4 ra0, ra1, rb0, rb1;
    auto gload = [&](int kb) {
        const float* pa = ga + (int64_t)ar * P + kb + ak;
        ra0 = *reinterpret_cast<const f32x4*>(pa);
        ra1 = *reinterpret_cast<const f32x4*>(pa + 4);
        const float* pb = gb + (int64_t)(kb + bk) * ldb + bj;
        rb0 = *reinterpret_cast<const f32x4*>(pb);
        rb1 = *reinterpret_cast<const f32x4*>(pb + 4);
    };
    auto sstore = [&](int buf) {
        *reinterpret_cast<f32x4*>(&sa[buf][ar * kLA + ak]) = ra0;
        *reinterpret_cast<f32x4*>(&sa[buf][ar * kLA + ak + 4]) = ra1;
        *reinterpret_cast<f32x4*>(&sb[buf][bk * kLB + bj]) = rb0;
        *reinterpret_cast<f32x4*>(&sb[buf][bk * kLB + bj + 4]) = rb1;
    };
    f32x16 acc = {};
    gload(klo);
    sstore(0);
    __syncthreads();
    int cur = 0;
    for (int kb = klo; kb < khi; kb += 32) {
        const bool more = kb + 32 < khi;
        if (more) gload(kb + 32);
        const float* A = &sa[cur][(wr * 32 + r32) * kLA + 4 * kh];
        const float* Bq = &sb[cur][(4 * kh) * kLB + wc * 32 + r32];
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
            const f32x4 a = *reinterpret_cast<const f32x4*>(A + 8 * kk);
#pragma unroll
            for (int u = 0; u < 4; ++u)
                acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[u], Bq[(8 * kk + u) * kLB], acc, 0,
                                                           0, 0);
        }
        if (more) sstore(cur ^ 1);
        __syncthreads();
        cur ^= 1;
    }
    const int i0 = ti * kNB + wr * 32, j0 = tj * kNB + wc * 32;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
        const int i = i0 + (q & 3) + 8 * (q >> 2) + 4 * kh, j = j0 + r32;
        if (STEP == 0)
            T[(int64_t)i * s + j] = acc[q];
        else
            M[(int64_t)(a0 + i) * P + c0 + j] = -acc[q];
    }
}

// The same level with split-precision products (round 6, the default; SGLM_INV_X3=0 for the
// f32 kernel above): the staging
// of chol_inv_level_lds_kernel, but each 16-deep K-step as three v_mfma_f32_32x32x16_bf16 on
// the operands split x = hi + lo (hi = bf16(x), lo = bf16(x - hi)): hi hi + hi lo + lo hi, ~2^-17
// relative per product (f32 accumulation) -- M is a preconditioner (delta = -M M^T g, the
// direction rounded to bf16 before use; the fixed point is the exact gradient's), so its f32
// rounding is not needed; 16 bf16 products per MFMA against 2 f32 ones.
__device__ __forceinline__ void split8(const float (&x)[8], bf16x8& hi, bf16x8& lo) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const __bf16 h = (__bf16)x[j];
        hi[j] = h;
        lo[j] = (__bf16)(x[j] - (float)h);
    }
}

template <int STEP>
__global__ void __launch_bounds__(kCT) chol_inv_level_x3_kernel(const float* __restrict__ Hall,
                                                                float* __restrict__ Mall,
                                                                float* __restrict__ Tall,
                                                                int32_t P, int32_t s,
                                                                const int32_t* __restrict__ fits,
                                                                int64_t tcap) {
    __shared__ __attribute__((aligned(16))) float sa[2][64 * kLA];
    __shared__ __attribute__((aligned(16))) float sb[2][32 * kLB];
    const int fit = fits[blockIdx.y];
    const float* H = Hall + (int64_t)fit * P * P;
    float* M = Mall + (int64_t)fit * P * P;
    const int nsb = s / kNB;
    int t = blockIdx.x;
    const int pair = t / (nsb * nsb);
    t -= pair * nsb * nsb;
    const int ti = t / nsb, tj = t - ti * nsb;
    const int a0 = 2 * s * pair, c0 = a0 + s;
    const int cs = min(s, P - c0);
    if (cs <= 0 || tj * kNB >= cs) return;
    float* T = Tall + (int64_t)blockIdx.y * tcap + (int64_t)pair * s * s;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int r32 = lane & 31, h = lane >> 5;
    const int wr = wave >> 1, wc = wave & 1;
    const float* ga;
    const float* gb;
    int64_t ldb;
    int klo, khi;
    if (STEP == 0) {
        ga = H + (int64_t)(a0 + ti * kNB) * P + c0;
        gb = M + (int64_t)c0 * P + c0 + tj * kNB;
        ldb = P;
        klo = 0;
        khi = (tj + 1) * kNB;
    } else {
        ga = M + (int64_t)(a0 + ti * kNB) * P + a0;
        gb = T + tj * kNB;
        ldb = s;
        klo = ti * kNB;
        khi = s;
    }
    const int ar = tid >> 2, ak = 8 * (tid & 3);
    const int bk = tid >> 3, bj = 8 * (tid & 7);
    f32x4 ra0, ra1, rb0, rb1;
    auto gload = [&](int kb) {
        const float* pa = ga + (int64_t)ar * P + kb + ak;
        ra0 = *reinterpret_cast<const f32x4*>(pa);
        ra1 = *reinterpret_cast<const f32x4*>(pa + 4);
        const float* pb = gb + (int64_t)(kb + bk) * ldb + bj;
        rb0 = *reinterpret_cast<const f32x4*>(pb);
        rb1 = *reinterpret_cast<const f32x4*>(pb + 4);
    };
    auto sstore = [&](int buf) {
        *reinterpret_cast<f32x4*>(&sa[buf][ar * kLA + ak]) = ra0;
        *reinterpret_cast<f32x4*>(&sa[buf][ar * kLA + ak + 4]) = ra1;
        *reinterpret_cast<f32x4*>(&sb[buf][bk * kLB + bj]) = rb0;
        *reinterpret_cast<f32x4*>(&sb[buf][bk * kLB + bj + 4]) = rb1;
    };
    f32x16 acc = {};
    gload(klo);
    sstore(0);
    __syncthreads();
    int cur = 0;
    for (int kb = klo; kb < khi; kb += 32) {
        const bool more = kb + 32 < khi;
        if (more) gload(kb + 32);
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            // A[row wr 32 + r32][k = 16 ks + 8 h + j], B[k = 16 ks + 8 h + j][col wc 32 + r32]
            const float* A = &sa[cur][(wr * 32 + r32) * kLA + 16 * ks + 8 * h];
            const float* Bq = &sb[cur][(16 * ks + 8 * h) * kLB + wc * 32 + r32];
            const f32x4 a0v = *reinterpret_cast<const f32x4*>(A);
            const f32x4 a1v = *reinterpret_cast<const f32x4*>(A + 4);
            float xa[8] = {a0v[0], a0v[1], a0v[2], a0v[3], a1v[0], a1v[1], a1v[2], a1v[3]};
            float xb[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) xb[j] = Bq[j * kLB];
            bf16x8 ah, al, bh, bl;
            split8(xa, ah, al);
            split8(xb, bh, bl);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bl, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bh, acc, 0, 0, 0);
        }
        if (more) sstore(cur ^ 1);
        __syncthreads();
        cur ^= 1;
    }
    const int i0 = ti * kNB + wr * 32, j0 = tj * kNB + wc * 32;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
        const int i = i0 + (q & 3) + 8 * (q >> 2) + 4 * h, j = j0 + r32;
        if (STEP == 0)
            T[(int64_t)i * s + j] = acc[q];
        else
            M[(int64_t)(a0 + i) * P + c0 + j] = -acc[q];
    }
}

// Block column J of M = U^-1, left-looking (round 6):
//     M[I][J] = -(sum_{k=I}^{J-1} M[I][k] U[k][J]) M[J][J]      for the row blocks I < J,
// one 64 x 64 tile per workgroup (blockIdx.x = I), the product staged exactly as in
// chol_inv_level_lds_kernel, then the tile times the diagonal block's inverse M[J][J] (written
// by the diagonal step; exact zeros below its diagonal and in the columns of dropped pivots, so
// frozen columns of M stay zero).  Everything it reads is final once block J is factored: U's
// block rows k < J after their panel steps, M's columns < J from the launches for J' < J.  So
// the chain launches it on a branch of its own right after the launch that factored block J,
// beside the rest of the factorisation, and only the last column follows the chain (the
// recursive-doubling levels all ran after it: 0.12 ms at one fit, 0.88 ms at 20).
__global__ void __launch_bounds__(kCT) chol_inv_col_kernel(const float* __restrict__ Hall,
                                                           float* __restrict__ Mall, int32_t P,
                                                           int32_t J,
                                                           const int32_t* __restrict__ fits) {
    __shared__ __attribute__((aligned(16))) float sa[2][64 * kLA];
    __shared__ __attribute__((aligned(16))) float sb[2][32 * kLB];
    const int fit = fits[blockIdx.y];
    const float* H = Hall + (int64_t)fit * P * P;
    float* M = Mall + (int64_t)fit * P * P;
    const int ti = blockIdx.x;
    if (ti >= J) return;
    const int c0 = J * kNB;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int r32 = lane & 31, kh = lane >> 5;
    const int wr = wave >> 1, wc = wave & 1;
    // A = M[ti rows][k], B = U[k][c0 + j] (H's upper triangle), k in [64 ti, 64 J)
    const float* ga = M + (int64_t)(ti * kNB) * P;
    const float* gb = H + c0;
    const int klo = ti * kNB, khi = c0;
    const int ar = tid >> 2, ak = 8 * (tid & 3);
    const int bk = tid >> 3, bj = 8 * (tid & 7);
    f32x4 ra0, ra1, rb0, rb1;
    auto gload = [&](int kb) {
        const float* pa = ga + (int64_t)ar * P + kb + ak;
        ra0 = *reinterpret_cast<const f32x4*>(pa);
        ra1 = *reinterpret_cast<const f32x4*>(pa + 4);
        const float* pb = gb + (int64_t)(kb + bk) * P + bj;
        rb0 = *reinterpret_cast<const f32x4*>(pb);
        rb1 = *reinterpret_cast<const f32x4*>(pb + 4);
    };
    auto sstore = [&](int buf) {
        *reinterpret_cast<f32x4*>(&sa[buf][ar * kLA + ak]) = ra0;
        *reinterpret_cast<f32x4*>(&sa[buf][ar * kLA + ak + 4]) = ra1;
        *reinterpret_cast<f32x4*>(&sb[buf][bk * kLB + bj]) = rb0;
        *reinterpret_cast<f32x4*>(&sb[buf][bk * kLB + bj + 4]) = rb1;
    };
    f32x16 acc = {};
    gload(klo);
    sstore(0);
    __syncthreads();
    int cur = 0;
    for (int kb = klo; kb < khi; kb += 32) {
        const bool more = kb + 32 < khi;
        if (more) gload(kb + 32);
        const float* A = &sa[cur][(wr * 32 + r32) * kLA + 4 * kh];
        const float* Bq = &sb[cur][(4 * kh) * kLB + wc * 32 + r32];
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
            const f32x4 a = *reinterpret_cast<const f32x4*>(A + 8 * kk);
#pragma unroll
            for (int u = 0; u < 4; ++u)
                acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[u], Bq[(8 * kk + u) * kLB], acc, 0,
                                                           0, 0);
        }
        if (more) sstore(cur ^ 1);
        __syncthreads();
        cur ^= 1;
    }
    // the tile Y (rows wr 32 .., columns wc 32 .. per wave) into LDS as the A operand of the
    // second product, M[J][J] as its B operand (64 rows over the two B buffers)
    constexpr int kLY = 68;
    float* sy = &sa[0][0];
#pragma unroll
    for (int q = 0; q < 16; ++q)
        sy[(wr * 32 + (q & 3) + 8 * (q >> 2) + 4 * kh) * kLY + wc * 32 + r32] = acc[q];
    {
        const int k = tid >> 2, cq = 16 * (tid & 3);
        const float* pm = M + (int64_t)(c0 + k) * P + c0 + cq;
        float* dst = &sb[0][0] + k * kLB + cq;
#pragma unroll
        for (int e = 0; e < 16; e += 4)
            *reinterpret_cast<f32x4*>(dst + e) = *reinterpret_cast<const f32x4*>(pm + e);
    }
    __syncthreads();
    f32x16 z = {};
    const float* A = sy + (wr * 32 + r32) * kLY + 4 * kh;
    const float* Bq = &sb[0][0] + (4 * kh) * kLB + wc * 32 + r32;
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) {
        const f32x4 a = *reinterpret_cast<const f32x4*>(A + 8 * kk);
#pragma unroll
        for (int u = 0; u < 4; ++u)
            z = __builtin_amdgcn_mfma_f32_32x32x2f32(a[u], Bq[(8 * kk + u) * kLB], z, 0, 0, 0);
    }
    const int i0 = ti * kNB + wr * 32, j0 = c0 + wc * 32;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
        const int i = i0 + (q & 3) + 8 * (q >> 2) + 4 * kh;
        M[(int64_t)i * P + j0 + r32] = -z[q];
    }
}

// The same level on 128 x 128 output tiles (levels with s >= 128 when enough fits fill the
// chip): four waves of 64 x 64 (2 x 2 quadrants of v_mfma_f32_32x32x2f32), K in blocks of
// 16 staged through double-buffered LDS (37 KB: static LDS stays under 64 KB) -- half the
// operand traffic per flop of the 64 x 64 tile.  The triangles are bounded at 64-block granularity as in the 64 x 64 kernel: operand
// elements of M in a strictly lower 64-block (never written) are zeroed while staging.
constexpr int kT2 = 128;
constexpr int kKB2 = 16;            // K block
constexpr int kLA2 = 20;            // A [128][16] row stride (floats): 8 lanes of a b128 read
                                    // on disjoint banks
constexpr int kLB2 = 136;           // B [16][128] row stride: the k-halves on disjoint banks
template <int STEP>
__global__ void __launch_bounds__(kCT) chol_inv_level128_kernel(const float* __restrict__ Hall,
                                                                float* __restrict__ Mall,
                                                                float* __restrict__ Tall,
                                                                int32_t P, int32_t s,
                                                                const int32_t* __restrict__ fits,
                                                                int64_t tcap) {
    __shared__ __attribute__((aligned(16))) float sa[2][kT2 * kLA2];
    __shared__ __attribute__((aligned(16))) float sb[2][kKB2 * kLB2];
    const int fit = fits[blockIdx.y];
    const float* H = Hall + (int64_t)fit * P * P;
    float* M = Mall + (int64_t)fit * P * P;
    const int nsb = s / kT2;
    int t = blockIdx.x;
    const int pair = t / (nsb * nsb);
    t -= pair * nsb * nsb;
    const int ti = t / nsb, tj = t - ti * nsb;
    const int a0 = 2 * s * pair, c0 = a0 + s;
    const int cs = min(s, P - c0);
    if (cs <= 0 || tj * kT2 >= cs) return;
    float* T = Tall + (int64_t)blockIdx.y * tcap + (int64_t)pair * s * s;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int r32 = lane & 31, kh = lane >> 5;
    const int wr = wave >> 1, wc = wave & 1;
    const float* ga;
    const float* gb;
    int64_t ldb;
    int klo, khi;
    if (STEP == 0) {                                   // A = U[a0 + i][c0 + k], B = M[c0 + k][c0 + j]
        ga = H + (int64_t)(a0 + ti * kT2) * P + c0;
        gb = M + (int64_t)c0 * P + c0 + tj * kT2;
        ldb = P;
        klo = 0;
        khi = (tj + 1) * kT2;
    } else {                                           // A = M[a0 + i][a0 + k], B = T[k][j]
        ga = M + (int64_t)(a0 + ti * kT2) * P + a0;
        gb = T + tj * kT2;
        ldb = s;
        klo = ti * kT2;
        khi = s;
    }
    // staging shares: A row tid >> 1, k 8 (tid & 1) .. +7; B row k = tid >> 4, columns
    // 8 (tid & 15) .. +7
    const int ar = tid >> 1, ak = 8 * (tid & 1);
    const int bk = tid >> 4, bj = 8 * (tid & 15);
    f32x4 ra[2], rb[2];
    auto gload = [&](int kb) {
        const float* pa = ga + (int64_t)ar * P + kb + ak;
        const float* pb = gb + (int64_t)(kb + bk) * ldb + bj;
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            ra[u] = *reinterpret_cast<const f32x4*>(pa + 4 * u);
            rb[u] = *reinterpret_cast<const f32x4*>(pb + 4 * u);
        }
        if (STEP == 1) {
            // A = M_A row ti*128 + ar, columns kb + ak + ..: zero where the column's 64-block
            // lies left of the row's (a strictly lower 64-block of M)
            const int rowb = (ti * kT2 + ar) >> 6;
#pragma unroll
            for (int u = 0; u < 2; ++u)
                if (((kb + ak + 4 * u) >> 6) < rowb) ra[u] = (f32x4){0.f, 0.f, 0.f, 0.f};
        } else {
            // B = M_C row kb + bk, columns tj*128 + bj + ..: zero below the 64-block diagonal
            const int rowb = (kb + bk) >> 6;
#pragma unroll
            for (int u = 0; u < 2; ++u)
                if (((tj * kT2 + bj + 4 * u) >> 6) < rowb) rb[u] = (f32x4){0.f, 0.f, 0.f, 0.f};
        }
    };
    auto sstore = [&](int buf) {
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            *reinterpret_cast<f32x4*>(&sa[buf][ar * kLA2 + ak + 4 * u]) = ra[u];
            *reinterpret_cast<f32x4*>(&sb[buf][bk * kLB2 + bj + 4 * u]) = rb[u];
        }
    };
    f32x16 acc[2][2];
#pragma unroll
    for (int qi = 0; qi < 2; ++qi)
#pragma unroll
        for (int qj = 0; qj < 2; ++qj) acc[qi][qj] = (f32x16){};
    gload(klo);
    sstore(0);
    __syncthreads();
    int cur = 0;
    for (int kb = klo; kb < khi; kb += kKB2) {
        const bool more = kb + kKB2 < khi;
        if (more) gload(kb + kKB2);
#pragma unroll
        for (int kk = 0; kk < kKB2 / 8; ++kk) {
            f32x4 a[2];
#pragma unroll
            for (int qi = 0; qi < 2; ++qi)
                a[qi] = *reinterpret_cast<const f32x4*>(
                    &sa[cur][(wr * 64 + qi * 32 + r32) * kLA2 + 4 * kh + 8 * kk]);
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                float b[2];
#pragma unroll
                for (int qj = 0; qj < 2; ++qj)
                    b[qj] = sb[cur][(4 * kh + 8 * kk + u) * kLB2 + wc * 64 + qj * 32 + r32];
#pragma unroll
                for (int qi = 0; qi < 2; ++qi)
#pragma unroll
                    for (int qj = 0; qj < 2; ++qj)
                        acc[qi][qj] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[qi][u], b[qj],
                                                                           acc[qi][qj], 0, 0, 0);
            }
        }
        if (more) sstore(cur ^ 1);
        __syncthreads();
        cur ^= 1;
    }
#pragma unroll
    for (int qi = 0; qi < 2; ++qi)
#pragma unroll
        for (int qj = 0; qj < 2; ++qj) {
            const int i0 = ti * kT2 + wr * 64 + qi * 32, j0 = tj * kT2 + wc * 64 + qj * 32;
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                const int i = i0 + (q & 3) + 8 * (q >> 2) + 4 * kh, j = j0 + r32;
                if (STEP == 0)
                    T[(int64_t)i * s + j] = acc[qi][qj][q];
                else
                    M[(int64_t)(a0 + i) * P + c0 + j] = -acc[qi][qj][q];
            }
        }
}

// Solves on explicit inverses.  Tile t = rows [start, start + cnt) of the fit list (cnt <= 32,
// one factor: slot fsrc[start]); blockIdx.x = a 32-wide output column block; the 4 waves split
// K and reduce through LDS.  SECOND = false: Y[q][j] = sum_k G[q][k] M[k][j] with G = rscale *
// g (float64 -> f32) zeroed on the factor's frozen coordinates.  SECOND = true:
// delta[fit][i] = -sum_j Y[q][j] M[i][j], zero on frozen coordinates.
// STAGE (first pass only, the default): each wave copies its 64 x 32 block of M into
// LDS with eight float4 row loads per lane and reads the B operands from there, instead of 32
// scalar column loads per lane from L2.
template <bool SECOND, bool STAGE = false>
__global__ void __launch_bounds__(kCT) chol_inv_apply_kernel(
    const float* __restrict__ Mall, int32_t P, const int32_t* __restrict__ fits,
    const int32_t* __restrict__ fsrc, const float* __restrict__ rscale,
    const int32_t* __restrict__ tiles, const double* __restrict__ gall,
    const uint8_t* __restrict__ frozen_all, float* __restrict__ Y, float* __restrict__ delta_all) {
    __shared__ float red[4][16 * 64];
    __shared__ __attribute__((aligned(16))) float sm[STAGE ? 4 : 1][STAGE ? 64 * 32 : 4];
    const int start = tiles[2 * blockIdx.y], cnt = tiles[2 * blockIdx.y + 1];
    const int src = fsrc[start];
    const float* M = Mall + (int64_t)src * P * P;
    const uint8_t* frz = frozen_all + (int64_t)src * P;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int r32 = lane & 31, kh = lane >> 5;
    const int c0 = blockIdx.x * 32;
    const bool valid = r32 < cnt;
    const int q = start + (valid ? r32 : 0);
    f32x16 acc = {};
    if (!SECOND) {
        const double* g = gall + (int64_t)fits[q] * P;
        const double sc = (double)rscale[q];
        const float* pb = M + c0 + r32;
        const int khi = (c0 / kNB + 1) * kNB;           // M upper triangular
        // wave w takes the 64-k blocks w, w + 4, ...; a block's 8 chunks load together
        for (int kb = kNB * wave; kb < khi; kb += 4 * kNB) {
            float a[8][4], b[8][4];
            const float* pbk = pb + (int64_t)(kb + 4 * kh) * P;
            if (STAGE) {
                const float* src = M + (int64_t)kb * P + c0 + 4 * (lane & 7);
                f32x4 tv[8];
#pragma unroll
                for (int i = 0; i < 8; ++i)
                    tv[i] = *reinterpret_cast<const f32x4*>(src + (int64_t)((lane >> 3) + 8 * i) * P);
#pragma unroll
                for (int i = 0; i < 8; ++i)
                    *reinterpret_cast<f32x4*>(&sm[wave][((lane >> 3) + 8 * i) * 32 + 4 * (lane & 7)]) =
                        tv[i];
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                __builtin_amdgcn_wave_barrier();
            }
#pragma unroll
            for (int v = 0; v < 8; ++v) {
                const int k = kb + 8 * v + 4 * kh;
                const uint32_t fz = *reinterpret_cast<const uint32_t*>(frz + k);
                const double2 g01 = *reinterpret_cast<const double2*>(g + k);
                const double2 g23 = *reinterpret_cast<const double2*>(g + k + 2);
                a[v][0] = (float)(g01.x * sc);
                a[v][1] = (float)(g01.y * sc);
                a[v][2] = (float)(g23.x * sc);
                a[v][3] = (float)(g23.y * sc);
                const uint32_t keep = valid ? ~fz : 0u;        // a byte != 0: frozen
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    if (((keep >> (8 * u)) & 0xff) != 0xff) a[v][u] = 0.0f;
                    b[v][u] = STAGE ? sm[wave][(8 * v + 4 * kh + u) * 32 + r32]
                                    : pbk[(8 * v + u) * P];
                }
            }
#pragma unroll
            for (int v = 0; v < 8; ++v)
#pragma unroll
                for (int u = 0; u < 4; ++u)
                    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[v][u], b[v][u], acc, 0, 0, 0);
            if (STAGE) {                             // this block's reads done before the next
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");     // block's writes
                __builtin_amdgcn_wave_barrier();
            }
        }
    } else {
        const float* py = Y + (int64_t)q * P;
        const float* pm = M + (int64_t)(c0 + r32) * P;
        const int klo = (c0 / kNB) * kNB;               // M[i][j] = 0 for j < i
        for (int kb = klo + kNB * wave; kb < P; kb += 4 * kNB) {
            f32x4 a[8], b[8];
#pragma unroll
            for (int v = 0; v < 8; ++v) {
                const int k = kb + 8 * v + 4 * kh;
                a[v] = *reinterpret_cast<const f32x4*>(py + k);
                if (!valid) a[v] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
                b[v] = *reinterpret_cast<const f32x4*>(pm + k);
            }
#pragma unroll
            for (int v = 0; v < 8; ++v)
#pragma unroll
                for (int u = 0; u < 4; ++u)
                    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[v][u], b[v][u], acc, 0, 0, 0);
        }
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) red[wave][r * 64 + lane] = acc[r];
    __syncthreads();
#pragma unroll
    for (int m = 0; m < 4; ++m) {
        const int o = threadIdx.x + kCT * m;            // (register r, lane l) of the quadrant
        const float v = red[0][o] + red[1][o] + red[2][o] + red[3][o];
        const int r = o >> 6, l = o & 63;
        const int row = (r & 3) + 8 * (r >> 2) + 4 * (l >> 5), col = c0 + (l & 31);
        if (row >= cnt) continue;
        if (!SECOND)
            Y[(int64_t)(start + row) * P + col] = v;
        else
            delta_all[(int64_t)fits[start + row] * P + col] = frz[col] ? 0.0f : -v;
    }
}

}  // namespace sglm

using namespace sglm;

// recursive-doubling scratch per factored fit: the largest level's T blocks
static int64_t inv_tcap(int32_t P) {
    int64_t cap = 0;
    for (int s = kNB; s < P; s *= 2) {
        const int64_t pairs = (P - s + 2 * s - 1) / (2 * s);
        const int64_t v = pairs * s * s;
        cap = v > cap ? v : cap;
    }
    return cap;
}

extern "C" size_t sglm_chol_work_bytes(int32_t P, int32_t B) {
    // rhs, original diagonal, diagonal-block inverses; for sglm_chol_solve_inv also Y (B x P)
    // and the inversion scratch
    return ((size_t)3 * (size_t)B * (size_t)P + (size_t)B * kNB * kNB +
            (size_t)B * (size_t)inv_tcap(P)) * sizeof(float);
}

// Look-ahead depth of the blocked factorisation (block steps per trailing sweep); the
// SGLM_CHOL_LOOKAHEAD environment variable (1..8) overrides the default 4 for experiments.
static int chol_lookahead() {
    const char* e = getenv("SGLM_CHOL_LOOKAHEAD");           // read per chain (graph key)
    const int v = e ? atoi(e) : 4;
    return v >= 1 && v <= 8 ? v : 4;
}

// Inversion levels with the two-stage register pipeline (default; 1.52 -> 1.42 ms per 1-fit
// chain) or the one-chunk loop (SGLM_CHOL_PIPE=0, comparison runs).
static bool inv_pipe() {
    static const bool v = [] {
        const char* e = getenv("SGLM_CHOL_PIPE");
        return !(e && e[0] == '0');
    }();
    return v;
}

// Inversion levels through LDS (chol_inv_level_lds_kernel; default: 1-fit chain 1.22 -> 1.16 ms,
// 3 fits 1.47 -> 1.33 ms, C4 grid 60-62 -> 58-59 ms on one box), SGLM_INV_LDS=0 for the
// register variants.
// Split-precision inversion levels (chol_inv_level_x3_kernel, the default: chain of 1 / 6 / 11
// / 20 representatives 0.97 / 1.39 / 1.92 / 2.86 -> 0.95 / 1.28 / 1.74 / 2.53 ms, C4 grid
// 28.82 -> 28.41 ms in a 10-round A/B, profiles/r06b_inv_x3_ab.json); SGLM_INV_X3=0 for the f32
// MFMA levels (read per chain capture; part of the chain-graph key).
static bool inv_x3() {
    const char* e = getenv("SGLM_INV_X3");
    return !(e && e[0] == '0');
}

static bool inv_lds() {
    static const bool v = [] {
        const char* e = getenv("SGLM_INV_LDS");
        return !(e && e[0] == '0');
    }();
    return v;
}

// 128 x 128 inversion tiles on a level whose 128-tile grid has at least SGLM_INV128_WG
// workgroups (read per chain capture).  Off by default: measured slower than the 64 x 64
// LDS kernel at every fit count (C4 chain at 20 fits: 2.55 -> 2.64..2.69 ms).
static bool inv128(int64_t wgs) {
    const char* e = getenv("SGLM_INV128_WG");
    const int64_t mn = e ? atoll(e) : 0;
    return mn > 0 && wgs >= mn;
}

// The two-stage update measured slower on the box (16.5 vs 13.3 us per launch at 3 fits), so
// it is opt-in (SGLM_UPD_PIPE=1).
static bool upd_pipe() {
    static const bool v = [] {
        const char* e = getenv("SGLM_UPD_PIPE");
        return e && e[0] == '1';
    }();
    return v;
}

// First inverse-solve pass with LDS-staged M blocks (chol_inv_apply_kernel<false, true>;
// default: the same operands and MFMA order, C4 grid 59.6 / 57.2 -> 57.4 / 56.9 ms and the
// 8-rank share 22.8 -> 21.9 ms in an alternating A/B), SGLM_APPLY_STAGE=0 for column loads.
static bool apply_stage() {
    static const bool v = [] {
        const char* e = getenv("SGLM_APPLY_STAGE");
        return !(e && e[0] == '0');
    }();
    return v;
}

// Trailing updates through LDS (chol_update_lds_kernel; default: the same MFMA sequence as
// the register kernel, so bitwise the same factor; 1-fit chain 1.19 -> 1.09 ms, C4 grid
// 58.8-59.2 -> 58.0-58.2 ms in an alternating A/B), SGLM_UPD_LDS=0 for the register kernel.
static bool upd_lds() {
    static const bool v = [] {
        const char* e = getenv("SGLM_UPD_LDS");
        return !(e && e[0] == '0');
    }();
    return v;
}

static void launch_update(dim3 grid, hipStream_t s, float* H, int32_t P, int32_t k0, int32_t kc,
                          int32_t s0, const int32_t* fits) {
    if (upd_lds())
        chol_update_lds_kernel<<<grid, kCT, 0, s>>>(H, P, k0, kc, s0, fits);
    else if (upd_pipe())
        chol_update_kernel<true><<<grid, kCT, 0, s>>>(H, P, k0, kc, s0, fits);
    else
        chol_update_kernel<false><<<grid, kCT, 0, s>>>(H, P, k0, kc, s0, fits);
}

// fits[0 .. nrefac) are factored, fits[nrefac .. nact) reuse the factor and frozen set a
// previous call left in H (engine.irls' kept Hessians): one launch chain for both, the
// trailing updates over the refactored fits only.
static int chol_solve_mixed(float* H, int32_t P, const int32_t* fits, int32_t nact,
                            int32_t nrefac, const double* g, const float* dshift, float* delta,
                            int32_t* info, uint8_t* frozen, int32_t B, void* work,
                            hipStream_t s, float* Mall = nullptr,
                            const std::function<void(int)>* on_diag = nullptr) {
    if (nact <= 0) return SGLM_OK;
    if (!H || !fits || (!g && !Mall) || !dshift || !delta || !info || !frozen || !work ||
        P % kNB || P > kMaxP || B < nact || nrefac < 0 || nrefac > nact) {
        set_error("sglm_chol_solve: bad args (P=%d, max %d)", P, kMaxP);
        return SGLM_EINVAL;
    }
    float* rhs = (float*)work;
    float* dg = rhs + (size_t)B * P;
    float* minv = dg + (size_t)B * P;
    chol_prep_kernel<<<nact, kCT, 0, s>>>(H, P, fits, g, dshift, frozen, rhs, dg, info, nrefac);
    int st = check_launch("chol_prep_kernel");
    if (st) return st;
    if (nrefac > 0) {
        const int nb = P / kNB;
        chol_freeze_kernel<<<dim3((unsigned)(nb * (nb + 1) / 2), (unsigned)nrefac), kCT, 0, s>>>(
            H, P, fits, frozen);
        if ((st = check_launch("chol_freeze_kernel"))) return st;
    }
    if (nrefac == 0 && Mall) return SGLM_OK;
    if (nrefac == 0) {                       // stored factors only: two triangular solves
        chol_fwd2_kernel<<<nact, kST, 0, s>>>(H, P, fits, nullptr, frozen, rhs);
        st = check_launch("chol_fwd2_kernel");
        if (st) return st;
        chol_back2_kernel<<<nact, kST, 0, s>>>(H, P, fits, nullptr, frozen, rhs, delta);
        return check_launch("chol_back2_kernel");
    }
    const int nb = P / kNB;
    // look-ahead depth kLA: block steps in groups of kLA; after step b only the band of block
    // rows b+1 .. (end of the group) is updated with panel b (K = 64), and once per group ONE
    // rank-(kLA*64) update of the rest of the trailing matrix -- the trailing matrix (the HBM
    // read-modify-write that bounds the chain at large batches) is swept P/(kLA*64) times
    const bool fuse = Mall && nrefac == nact && diag4() && diag4q() && diag4l() && upd_lds() &&
                      upd_diag();
    bool have_diag = false;                  // the next diagonal step ran inside an update
    auto factor_step = [&](int kb) {
        const int k0 = kb * kNB;
        if (have_diag)
            ;
        else if (Mall && nrefac == nact && diag4() && diag4q() && diag4l())
            launch_chol_diag4l(nact, s, H, P, k0, fits, frozen, dg, info, minv, Mall);
        else if (Mall && nrefac == nact && diag4() && diag4q())
            launch_chol_diag4q(nact, s, H, P, k0, fits, frozen, dg, info, minv, Mall);
        else if (Mall && nrefac == nact && diag4())
            launch_chol_diag4(nact, s, H, P, k0, fits, frozen, dg, info, minv, Mall);
        else
            launch_chol_diag(nact, s, H, P, k0, fits, frozen, rhs, dg, info, nrefac, minv, Mall);
        if (!have_diag && on_diag) (*on_diag)(kb);        // block kb factored by this launch
        const int rem = P - k0 - kNB;
        if (rem > 0)
            chol_panel_kernel<<<dim3(nact, rem / kNB), kCT, 0, s>>>(H, P, k0, fits, minv, rhs,
                                                                    nrefac);
    };
    const int la = chol_lookahead();
    for (int kb = 0; kb < nb; kb += la) {
        const int ke = kb + la < nb ? kb + la : nb;            // group [kb, ke)
        for (int b = kb; b < ke; ++b) {
            factor_step(b);
            have_diag = false;
            const int nr = ke - 1 - b;                         // band rows b+1 .. ke-1
            const int T = nb - b - 1;
            if (nrefac > 0 && nr > 0) {
                const dim3 g(nr * T - nr * (nr - 1) / 2, nrefac);
                if (fuse) {
                    // tile (b+1, b+1) is complete after this band update: factor it there
                    launch_chol_update_diag4l(g, s, H, P, b * kNB, kNB, b + 1, fits, frozen, dg,
                                              info, minv, Mall);
                    have_diag = true;
                    if (on_diag) (*on_diag)(b + 1);
                } else {
                    launch_update(g, s, H, P, b * kNB, kNB, b + 1, fits);
                }
            }
        }
        const int T = nb - ke;
        if (nrefac > 0 && T > 0) {
            const dim3 g(T * (T + 1) / 2, nrefac);
            if (fuse) {
                launch_chol_update_diag4l(g, s, H, P, kb * kNB, (ke - kb) * kNB, ke, fits, frozen,
                                          dg, info, minv, Mall);
                have_diag = true;
                if (on_diag) (*on_diag)(ke);
            } else {
                launch_update(g, s, H, P, kb * kNB, (ke - kb) * kNB, ke, fits);
            }
        }
    }
    st = check_launch("chol block kernels");
    if (st) return st;
    if (Mall) return SGLM_OK;                // the caller solves on the explicit inverses
    chol_back2_kernel<<<nact, kST, 0, s>>>(H, P, fits, nullptr, frozen, rhs, delta);
    return check_launch("chol_back2_kernel");
}

extern "C" int sglm_chol_solve_ex(float* H, int32_t P, const int32_t* fits, int32_t nact,
                                  const double* g, const float* dshift, float* delta,
                                  int32_t* info, uint8_t* frozen, int32_t refactor,
                                  int32_t B, void* work, sglm_stream_t stream) {
    return chol_solve_mixed(H, P, fits, nact, refactor ? nact : 0, g, dshift, delta, info,
                            frozen, B, work, as_stream(stream));
}

// Solves on stored factors of other slots: for i < nact, fit = fits[i] solves
// (H_src / rscale[i]) delta = -g, i.e. delta[fit] = -rscale[i] * F_src^-1 F_src^-T g[fit],
// src = fsrc[i] (frozen set of src).  The factors must be complete (a previous call).
extern "C" int sglm_chol_solve_alias(const float* H, int32_t P, const int32_t* fits,
                                     const int32_t* fsrc, int32_t nact, const double* g,
                                     const float* rscale, float* delta, const uint8_t* frozen,
                                     int32_t B, void* work, sglm_stream_t stream) {
    if (nact <= 0) return SGLM_OK;
    if (!H || !fits || !fsrc || !g || !rscale || !delta || !frozen || !work || P % kNB ||
        P > kMaxP || B < nact) {
        set_error("sglm_chol_solve_alias: bad args (P=%d)", P);
        return SGLM_EINVAL;
    }
    hipStream_t s = as_stream(stream);
    float* rhs = (float*)work;
    chol_alias_prep_kernel<<<nact, kCT, 0, s>>>(P, fits, fsrc, g, rscale, frozen, rhs);
    int st = check_launch("chol_alias_prep_kernel");
    if (st) return st;
    chol_fwd2_kernel<<<nact, kST, 0, s>>>(H, P, fits, fsrc, frozen, rhs);
    st = check_launch("chol_fwd2_kernel");
    if (st) return st;
    chol_back2_kernel<<<nact, kST, 0, s>>>(H, P, fits, fsrc, frozen, rhs, delta);
    return check_launch("chol_back2_kernel");
}

extern "C" int sglm_chol_solve_mixed(float* H, int32_t P, const int32_t* fits, int32_t nact,
                                     int32_t nrefac, const double* g, const float* dshift,
                                     float* delta, int32_t* info, uint8_t* frozen, int32_t B,
                                     void* work, sglm_stream_t stream) {
    return chol_solve_mixed(H, P, fits, nact, nrefac, g, dshift, delta, info, frozen, B, work,
                            as_stream(stream));
}


// The inverse by left-looking block columns beside the factorisation (chol_inv_col_kernel);
// opt-in, SGLM_INV_COL=1 (read per chain capture; part of the chain-graph key).  Measured
// slower than the recursive-doubling levels after the chain (tools/chol_bench.py, one box,
// profiles/r06_inv_col_ab.json): chain of 1 / 3 / 11 / 20 representatives 0.95 / 1.13 / 1.92 /
// 2.83 -> 1.18 / 1.31 / 2.01 / 2.80 ms, C4 grid 34.2 -> 37.3 ms.  A column's longest tile runs
// K = 64 J serially (~40 us at J = 31), longer than a block step of the chain, so the branch
// falls behind and its last columns trail the chain by ~3 columns; at 20 fits the columns'
// work competes with the chain's group-end updates instead of filling idle CUs.
static bool inv_col() {
    const char* e = getenv("SGLM_INV_COL");
    return e && e[0] == '1';
}

// The branch the inverse columns run on: one stream and a set of events per host thread and
// device, created before any capture begins (a chain captured on stream s forks onto it at
// each factored block and joins back at its end, so the graph holds both branches).
struct InvColCtx {
    hipStream_t s2 = nullptr;
    std::vector<hipEvent_t> ev;
};

static InvColCtx* inv_col_ctx(int nev) {
    thread_local std::map<int, InvColCtx> ctxs;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return nullptr;
    InvColCtx& c = ctxs[dev];
    if (!c.s2 && hipStreamCreateWithFlags(&c.s2, hipStreamNonBlocking) != hipSuccess) {
        c.s2 = nullptr;
        return nullptr;
    }
    while ((int)c.ev.size() < nev) {
        hipEvent_t e = nullptr;
        if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return nullptr;
        c.ev.push_back(e);
    }
    return &c;
}

// The factorisation + inversion chain (~110 launches) of fits[0 .. n).  ctx: the inverse
// columns' branch (inv_col), or null for the recursive-doubling levels after the chain.
static int inv_levels(const float* H, float* Minv, int32_t P, const int32_t* fits, int32_t n,
                      int32_t B, void* work, hipStream_t s);

static int factor_inv_launch(float* H, float* Minv, int32_t P, const int32_t* fits, int32_t n,
                             const float* dshift, float* delta, int32_t* info, uint8_t* frozen,
                             int32_t B, void* work, hipStream_t s, InvColCtx* ctx = nullptr,
                             bool levels = true) {
    int st;
    if (ctx && levels) {
        int nev = 0, st2 = SGLM_OK;
        const std::function<void(int)> hook = [&](int J) {
            if (J <= 0 || st2 != SGLM_OK) return;
            const hipEvent_t e = ctx->ev[nev++];
            if (hipEventRecord(e, s) != hipSuccess || hipStreamWaitEvent(ctx->s2, e, 0) != hipSuccess) {
                set_error("chol inverse columns: fork failed");
                st2 = SGLM_EHIP;
                return;
            }
            chol_inv_col_kernel<<<dim3((unsigned)J, (unsigned)n), kCT, 0, ctx->s2>>>(H, Minv, P, J,
                                                                                  fits);
        };
        st = chol_solve_mixed(H, P, fits, n, n, nullptr, dshift, delta, info, frozen, B, work, s,
                              Minv, &hook);
        if (nev > 0) {                       // join the branch back (also after an error)
            const hipEvent_t e = ctx->ev[nev];
            if ((hipEventRecord(e, ctx->s2) != hipSuccess || hipStreamWaitEvent(s, e, 0) != hipSuccess)
                && !st && !st2) {
                set_error("chol inverse columns: join failed");
                st2 = SGLM_EHIP;
            }
        }
        if (st) return st;
        if (st2) return st2;
        return check_launch("chol_inv_col_kernel");
    }
    if ((st = chol_solve_mixed(H, P, fits, n, n, nullptr, dshift, delta, info, frozen, B, work, s,
                               Minv)))
        return st;
    return levels ? inv_levels(H, Minv, P, fits, n, B, work, s) : SGLM_OK;
}

// The explicit inverses M = U^-1 of fits[0 .. n) whose factors (and the diagonal blocks of M)
// a factorisation chain left in H / Minv: recursive doubling over aligned super-blocks,
// (U^-1)_AC = -M_A (B M_C), two launches per level, log2(P / 64) levels.
static int inv_levels(const float* H, float* Minv, int32_t P, const int32_t* fits, int32_t n,
                      int32_t B, void* work, hipStream_t s) {
    // work: rhs, original diagonal (B x P each), diagonal-block inverses (B x 64 x 64),
    // Y (B x P), T (B x tcap)
    float* T = (float*)work + (size_t)3 * B * P + (size_t)B * kNB * kNB;
    const int64_t tcap = inv_tcap(P);
    const bool pipe = inv_pipe();
    for (int sz = kNB; sz < P; sz *= 2) {
        const int pairs = (P - sz + 2 * sz - 1) / (2 * sz);
        const int sb = sz / kNB;
        const dim3 grid((unsigned)(pairs * sb * sb), (unsigned)n);
        const int sb2 = sz / kT2;
        if (sz >= kT2 && sz % kT2 == 0 && P % kT2 == 0 && inv128((int64_t)pairs * sb2 * sb2 * n)) {
            const dim3 grid2((unsigned)(pairs * sb2 * sb2), (unsigned)n);
            chol_inv_level128_kernel<0><<<grid2, kCT, 0, s>>>(H, Minv, T, P, sz, fits, tcap);
            chol_inv_level128_kernel<1><<<grid2, kCT, 0, s>>>(H, Minv, T, P, sz, fits, tcap);
        } else if (inv_x3()) {
            chol_inv_level_x3_kernel<0><<<grid, kCT, 0, s>>>(H, Minv, T, P, sz, fits, tcap);
            chol_inv_level_x3_kernel<1><<<grid, kCT, 0, s>>>(H, Minv, T, P, sz, fits, tcap);
        } else if (inv_lds()) {
            chol_inv_level_lds_kernel<0><<<grid, kCT, 0, s>>>(H, Minv, T, P, sz, fits, tcap);
            chol_inv_level_lds_kernel<1><<<grid, kCT, 0, s>>>(H, Minv, T, P, sz, fits, tcap);
        } else if (pipe) {
            chol_inv_level_kernel<0, true><<<grid, kCT, 0, s>>>(H, Minv, T, P, sz, fits, tcap);
            chol_inv_level_kernel<1, true><<<grid, kCT, 0, s>>>(H, Minv, T, P, sz, fits, tcap);
        } else {
            chol_inv_level_kernel<0, false><<<grid, kCT, 0, s>>>(H, Minv, T, P, sz, fits, tcap);
            chol_inv_level_kernel<1, false><<<grid, kCT, 0, s>>>(H, Minv, T, P, sz, fits, tcap);
        }
    }
    return check_launch("chol_inv_level_kernel");
}

// The chain is launch-bound on the host (~110 dependent launches, ~1.4 ms of enqueue against
// ~1 ms of GPU time), so it is captured once per argument set into a HIP graph and replayed
// (one launch).  Graphs are keyed by every pointer and size the chain bakes in; the caller
// keeps `fits` in a stable buffer.  SGLM_CHOL_GRAPH=0 launches the chain directly.
struct ChainKey {
    const void *H, *Minv, *fits, *dshift, *delta, *info, *frozen, *work;
    int32_t P, n, B, la, q;
    bool operator<(const ChainKey& o) const {
        return std::memcmp(this, &o, sizeof(ChainKey)) < 0;
    }
};

static bool chol_graphs_enabled() {
    static const bool on = [] {
        const char* e = getenv("SGLM_CHOL_GRAPH");
        return !(e && e[0] == '0');
    }();
    return on;
}

// Bounded LRU of instantiated chains.  Each entry keeps an event recorded after its latest
// launch; an evicted (or cleared) executable is destroyed only after that event completed, so
// a replay still in flight on any stream is never freed under it.  The reference's drivers
// loop files x responses x runs (er_refactored_from_scratch_cleanup.py:261,388,393), and
// every worker thread / reallocated buffer set is a new key: without a bound the cache would
// grow by one ~110-node executable per key for the life of the process.
namespace {
struct ChainEntry {
    hipGraphExec_t exec = nullptr;
    hipEvent_t done = nullptr;
    uint64_t used = 0;
};
std::mutex g_chain_mu;
std::map<ChainKey, ChainEntry> g_chain_cache;
std::vector<ChainEntry> g_chain_pending;   // evicted, destroyed once their last replay is done
uint64_t g_chain_tick = 0;

int chain_cache_cap() {
    static const int cap = [] {
        const char* e = getenv("SGLM_CHOL_GRAPH_CAP");
        const int v = e ? atoi(e) : 32;
        return v > 0 ? v : 1;
    }();
    return cap;
}

void chain_entry_destroy(ChainEntry& e) {
    if (e.done) {
        (void)hipEventSynchronize(e.done);
        (void)hipEventDestroy(e.done);
    }
    if (e.exec) (void)hipGraphExecDestroy(e.exec);
    e.exec = nullptr;
    e.done = nullptr;
}

// call with g_chain_mu held: evicted entries go to the pending list (no synchronisation
// under the lock -- a chain's stream may sit behind an all-reduce of a row-sharded solve)
void chain_cache_evict_to(size_t keep) {
    while (g_chain_cache.size() > keep) {
        auto lru = g_chain_cache.begin();
        for (auto it = g_chain_cache.begin(); it != g_chain_cache.end(); ++it)
            if (it->second.used < lru->second.used) lru = it;
        g_chain_pending.push_back(lru->second);
        g_chain_cache.erase(lru);
    }
}

// call WITHOUT g_chain_mu: destroy the pending entries whose last replay has completed (all of
// them, waiting for each, when `wait`)
void chain_pending_reap(bool wait) {
    std::vector<ChainEntry> done;
    {
        std::lock_guard<std::mutex> lock(g_chain_mu);
        for (size_t i = 0; i < g_chain_pending.size();) {
            ChainEntry& e = g_chain_pending[i];
            if (wait || !e.done || hipEventQuery(e.done) == hipSuccess) {
                done.push_back(e);
                e = g_chain_pending.back();
                g_chain_pending.pop_back();
            } else {
                ++i;
            }
        }
    }
    for (auto& e : done) chain_entry_destroy(e);
}
}  // namespace

extern "C" int32_t sglm_chol_graph_cache_size(void) {
    std::lock_guard<std::mutex> lock(g_chain_mu);
    return (int32_t)g_chain_cache.size();
}

extern "C" int sglm_chol_graph_cache_clear(void) {
    {
        std::lock_guard<std::mutex> lock(g_chain_mu);
        chain_cache_evict_to(0);
    }
    chain_pending_reap(true);
    return SGLM_OK;
}

static int factor_inv_cached(float* H, float* Minv, int32_t P, const int32_t* fits, int32_t n,
                             const float* dshift, float* delta, int32_t* info, uint8_t* frozen,
                             int32_t B, void* work, hipStream_t s, InvColCtx* ctx, bool levels);

static int factor_inv(float* H, float* Minv, int32_t P, const int32_t* fits, int32_t n,
                      const float* dshift, float* delta, int32_t* info, uint8_t* frozen,
                      int32_t B, void* work, hipStream_t s, bool levels = true) {
    // (every diagonal-step variant writes its block of M, which the columns read)
    InvColCtx* ctx = (levels && inv_col()) ? inv_col_ctx(P / kNB + 1) : nullptr;
    if (!chol_graphs_enabled() || s == nullptr)      // the null stream cannot be captured
        return factor_inv_launch(H, Minv, P, fits, n, dshift, delta, info, frozen, B, work, s,
                                 ctx, levels);
    const int st = factor_inv_cached(H, Minv, P, fits, n, dshift, delta, info, frozen, B, work, s,
                                     ctx, levels);
    chain_pending_reap(false);                        // evicted chains that finished, unlocked
    return st;
}

static int factor_inv_cached(float* H, float* Minv, int32_t P, const int32_t* fits, int32_t n,
                             const float* dshift, float* delta, int32_t* info, uint8_t* frozen,
                             int32_t B, void* work, hipStream_t s, InvColCtx* ctx, bool levels) {
    ChainKey key;
    std::memset(&key, 0, sizeof(key));
    key.H = H; key.Minv = Minv; key.fits = fits; key.dshift = dshift; key.delta = delta;
    key.info = info; key.frozen = frozen; key.work = work;
    key.P = P; key.n = n; key.B = B; key.la = chol_lookahead(); key.q = (diag4q() ? (diag4l() ? (upd_diag() ? 3 : 2) : 1) : 0) | (ctx ? 4 : 0) | (levels ? 0 : 8) | (inv_x3() ? 16 : 0);
    // the lock is held across capture and launch: a concurrent eviction must not destroy the
    // entry between lookup and launch (captures are thread-local, so nothing else is stalled
    // but other chains' host enqueue, which is short next to the chain itself)
    std::lock_guard<std::mutex> lock(g_chain_mu);
    auto it = g_chain_cache.find(key);
    if (it == g_chain_cache.end()) {
        hipGraph_t graph = nullptr;
        if (hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal) != hipSuccess) {
            set_error("chol graph: hipStreamBeginCapture failed");
            return SGLM_EHIP;
        }
        const int st = factor_inv_launch(H, Minv, P, fits, n, dshift, delta, info, frozen, B,
                                         work, s, ctx, levels);
        const hipError_t ec = hipStreamEndCapture(s, &graph);
        if (st) {
            if (graph) (void)hipGraphDestroy(graph);
            return st;
        }
        if (ec != hipSuccess || !graph) {
            set_error("chol graph: hipStreamEndCapture failed");
            return SGLM_EHIP;
        }
        ChainEntry e;
        const hipError_t ei = hipGraphInstantiate(&e.exec, graph, nullptr, nullptr, 0);
        (void)hipGraphDestroy(graph);
        if (ei != hipSuccess) {
            set_error("chol graph: hipGraphInstantiate failed");
            return SGLM_EHIP;
        }
        if (hipEventCreateWithFlags(&e.done, hipEventDisableTiming) != hipSuccess) {
            (void)hipGraphExecDestroy(e.exec);
            set_error("chol graph: hipEventCreate failed");
            return SGLM_EHIP;
        }
        chain_cache_evict_to((size_t)chain_cache_cap() - 1);
        it = g_chain_cache.emplace(key, e).first;
    }
    it->second.used = ++g_chain_tick;
    if (hipGraphLaunch(it->second.exec, s) != hipSuccess) {
        set_error("chol graph: hipGraphLaunch failed");
        return SGLM_EHIP;
    }
    if (hipEventRecord(it->second.done, s) != hipSuccess) {
        set_error("chol graph: hipEventRecord failed");
        return SGLM_EHIP;
    }
    return SGLM_OK;
}

// Factor fits[0 .. nrefac) (penalty shift, frozen set, blocked Cholesky) and form their
// explicit inverses M = U^-1 in Minv; then every fit of the list solves on a stored inverse:
// delta[fits[q]] = -rscale[q] * M_f M_f^T g[fits[q]], f = fsrc[q] (fsrc[q] = fits[q] for a fit
// on its own factor, the representative's slot for a cross-mask alias).  tiles: ntiles x
// (start, count <= 32) runs of the list sharing one factor.
extern "C" int sglm_chol_solve_inv(float* H, float* Minv, int32_t P, const int32_t* fits,
                                   const int32_t* fsrc, const float* rscale, int32_t nact,
                                   int32_t nrefac, const int32_t* tiles, int32_t ntiles,
                                   const double* g, const float* dshift, float* delta,
                                   int32_t* info, uint8_t* frozen, int32_t B, void* work,
                                   sglm_stream_t stream) {
    if (nact <= 0) return SGLM_OK;
    if (!H || !Minv || !fits || (ntiles > 0 && (!fsrc || !rscale || !tiles || !g)) || !delta ||
        !frozen || !work || P % kNB || P > kMaxP || B < nact || nrefac < 0 || nrefac > nact ||
        (nrefac > 0 && (!dshift || !info))) {
        set_error("sglm_chol_solve_inv: bad args (P=%d, max %d)", P, kMaxP);
        return SGLM_EINVAL;
    }
    hipStream_t s = as_stream(stream);
    int st;
    if (nrefac > 0 && (st = factor_inv(H, Minv, P, fits, nrefac, dshift, delta, info, frozen, B,
                                       work, s)))
        return st;
    if (ntiles <= 0) return SGLM_OK;         // factor + invert only (the solve comes later)
    float* Y = (float*)work + (size_t)2 * B * P + (size_t)B * kNB * kNB;
    const dim3 grid((unsigned)(P / 32), (unsigned)ntiles);
    if (apply_stage())
        chol_inv_apply_kernel<false, true><<<grid, kCT, 0, s>>>(Minv, P, fits, fsrc, rscale, tiles,
                                                               g, frozen, Y, delta);
    else
        chol_inv_apply_kernel<false><<<grid, kCT, 0, s>>>(Minv, P, fits, fsrc, rscale, tiles, g,
                                                           frozen, Y, delta);
    chol_inv_apply_kernel<true><<<grid, kCT, 0, s>>>(Minv, P, fits, fsrc, rscale, tiles, g,
                                                      frozen, Y, delta);
    return check_launch("chol_inv_apply_kernel");
}

// The two halves of sglm_chol_solve_inv's factorisation (round 6): sglm_chol_factor runs the
// chain (penalty shift, frozen set, blocked Cholesky; the diagonal blocks of M written) and
// sglm_chol_invert the inversion levels after it -- bitwise the factor and inverse of
// sglm_chol_solve_inv.  The engine solves the iteration on the fresh factors by substitution
// (sglm_chol_solve_alias) and leaves the inversion to run beside its next main-stream work.
extern "C" int sglm_chol_factor(float* H, float* Minv, int32_t P, const int32_t* fits,
                                int32_t n, const float* dshift, int32_t* info, uint8_t* frozen,
                                int32_t B, void* work, sglm_stream_t stream) {
    if (n <= 0) return SGLM_OK;
    if (!H || !Minv || !fits || !dshift || !info || !frozen || !work || P % kNB || P > kMaxP ||
        B < n) {
        set_error("sglm_chol_factor: bad args (P=%d, max %d)", P, kMaxP);
        return SGLM_EINVAL;
    }
    float* scratch = (float*)work + (size_t)2 * B * P + (size_t)B * kNB * kNB;   // unused delta
    return factor_inv(H, Minv, P, fits, n, dshift, scratch, info, frozen, B, work,
                      as_stream(stream), false);
}

extern "C" int sglm_chol_invert(const float* H, float* Minv, int32_t P, const int32_t* fits,
                                int32_t n, int32_t B, void* work, sglm_stream_t stream) {
    if (n <= 0) return SGLM_OK;
    if (!H || !Minv || !fits || !work || P % kNB || P > kMaxP || B < n) {
        set_error("sglm_chol_invert: bad args (P=%d, max %d)", P, kMaxP);
        return SGLM_EINVAL;
    }
    return inv_levels(H, Minv, P, fits, n, B, work, as_stream(stream));
}
