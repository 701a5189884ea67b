// Batched weighted Gram  H_k = X^T diag(w_k) X  — the dominant IRLS kernel.
//
// Replaces the Hessian work of every solver iteration inside self.model.fit
// (backend/sglm.py:241): sklearn's X^T diag(h) X for newton-cholesky / the X^T X of Ridge's
// cholesky (_ridge.py:201-213) and, for lbfgs, the 2 GEMVs per evaluation it stands in for.
//
// Three forms, all v_mfma on gfx950, upper triangle by 256- (v2) or 128-blocks (v6, f32):
//   * v6 (sglm_syrk_cbits): 0/1 event designs, per-mask row-compacted bit-planes expanded to
//     bf16 in registers, one wave per 128x128 block, no LDS -- the C4 production path;
//   * v2 (sglm_syrk / sglm_syrk_masked): any bf16 design, 256x256 tiles of 8 waves staged
//     through LDS by LDS-DMA, optional 8-row-group lists that skip rows outside a mask;
//   * f32 (sglm_syrk_f32): exact f32 products for designs that are not bf16-representable,
//     where the Gram itself must be exact (coordinate descent, Gaussian closed forms).
// Optional split-K over rows into fixed-order f32 slabs (deterministic).
#include "common.h"


namespace sglm {

constexpr int kBM = 256;       // v2 output tile edge (slab reduction granularity)

__device__ __forceinline__ void tile_coords(int t, int nt, int& ti, int& tj) {
    // enumerate upper-triangular tiles row by row: (0,0),(0,1)..(0,nt-1),(1,1)...
    ti = 0;
    int rowlen = nt;
    while (t >= rowlen) { t -= rowlen; ++ti; --rowlen; }
    tj = ti + t;
}

// Sum the split slabs (fixed order) into H for the upper-triangular tiles only.
__global__ void __launch_bounds__(256) syrk_reduce(const float* __restrict__ slab, int32_t P,
                                                   int32_t nact, int32_t splits,
                                                   const int32_t* __restrict__ fits,
                                                   float* __restrict__ H) {
    const int slot = blockIdx.y;
    const int64_t PP = (int64_t)P * P;
    for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < PP;
         e += (int64_t)gridDim.x * 256) {
        const int64_t a = e / P, b = e % P;
        if (a / kBM > b / kBM) continue;
        float s = 0.0f;
        for (int z = 0; z < splits; ++z) s += slab[((int64_t)z * nact + slot) * PP + e];
        H[(int64_t)fits[slot] * PP + e] = s;
    }
}

}  // namespace sglm

using namespace sglm;

extern "C" {

size_t sglm_syrk_work_bytes(int32_t P, int32_t nact, int32_t splits) {
    if (splits <= 1) return 0;
    return (size_t)splits * (size_t)nact * (size_t)P * (size_t)P * sizeof(float);
}

}  // extern "C"

// ---------------------------------------------------------------------------------------
// Exact-f32 variant for designs that are not bf16-representable (real-valued predictors):
// v_mfma_f32_32x32x2_f32 (exact f32 products, f32 accumulate).  Used where the Gram itself
// must be accurate (coordinate descent, Gaussian closed forms); IRLS on such designs keeps
// the bf16 Gram because the exact gradient corrects the Newton step.
// 128x128 tile, 256 threads = 4 waves (2x2), each wave 64x64 = 2x2 tiles of 32x32;
// K-step 16 rows; LDS panels [128 predictors][16 rows + 1 pad] f32.
namespace sglm {
constexpr int kFBM = 128, kFBK = 16, kFRow = kFBK + 1;

__global__ void __launch_bounds__(256) syrk_f32_kernel(
    const float* __restrict__ Xf, int64_t ld, int32_t P, int64_t nsteps_total,
    int64_t steps_per_split, const float* __restrict__ W, const int32_t* __restrict__ fits,
    int32_t ntiles, float* __restrict__ H, float* __restrict__ slab, int32_t nact) {
    __shared__ float sA[kFBM][kFRow];
    __shared__ float sB[kFBM][kFRow];
    const int nt = P / kFBM;
    const int tile = blockIdx.x % ntiles;
    const int slot = blockIdx.x / ntiles;
    const int split = blockIdx.y;
    int ti, tj;
    tile_coords(tile, nt, ti, tj);
    const int fit = fits[slot];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wr = wave >> 1, wc = wave & 1;
    const int r = lane & 31, h = lane >> 5;
    const int64_t s0 = (int64_t)split * steps_per_split;
    const int64_t s1 = min(s0 + steps_per_split, nsteps_total);
    const float* XA = Xf + (int64_t)ti * kFBM * ld;
    const float* XB = Xf + (int64_t)tj * kFBM * ld;
    const float* w = W + (int64_t)fit * ld;
    f32x16 acc[2][2];
    for (int m = 0; m < 2; ++m)
        for (int q = 0; q < 2; ++q) acc[m][q] = (f32x16){};
    // staging: 128 predictors x 16 rows = 2048 floats per panel, 8 per thread (2 x f32x4)
    const int col = tid >> 1, part = (tid & 1) * 8;
    for (int64_t s = s0; s < s1; ++s) {
        const int64_t i = s * kFBK + part;
        const f32x4 a0 = *reinterpret_cast<const f32x4*>(XA + (int64_t)col * ld + i);
        const f32x4 a1 = *reinterpret_cast<const f32x4*>(XA + (int64_t)col * ld + i + 4);
        const f32x4 b0 = *reinterpret_cast<const f32x4*>(XB + (int64_t)col * ld + i);
        const f32x4 b1 = *reinterpret_cast<const f32x4*>(XB + (int64_t)col * ld + i + 4);
        const f32x4 w0 = *reinterpret_cast<const f32x4*>(w + i);
        const f32x4 w1 = *reinterpret_cast<const f32x4*>(w + i + 4);
        __syncthreads();
        for (int e = 0; e < 4; ++e) {
            sA[col][part + e] = a0[e];
            sA[col][part + 4 + e] = a1[e];
            sB[col][part + e] = b0[e] * w0[e];
            sB[col][part + 4 + e] = b1[e] * w1[e];
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < kFBK; k += 2) {
            float av[2], bv[2];
            for (int m = 0; m < 2; ++m) av[m] = sA[wr * 64 + m * 32 + r][k + h];
            for (int q = 0; q < 2; ++q) bv[q] = sB[wc * 64 + q * 32 + r][k + h];
            for (int m = 0; m < 2; ++m)
                for (int q = 0; q < 2; ++q)
                    acc[m][q] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[m], bv[q], acc[m][q], 0, 0, 0);
        }
    }
    float* out = slab ? slab + ((int64_t)split * nact + slot) * (int64_t)P * P
                      : H + (int64_t)fit * P * P;
    const int64_t rb = (int64_t)ti * kFBM + wr * 64, cb = (int64_t)tj * kFBM + wc * 64;
    for (int m = 0; m < 2; ++m)
        for (int q = 0; q < 2; ++q)
            for (int j = 0; j < 16; ++j)
                out[(rb + m * 32 + (j & 3) + 8 * (j >> 2) + 4 * h) * P + cb + q * 32 + r] = acc[m][q][j];
}

__global__ void __launch_bounds__(256) syrk_reduce_t(const float* __restrict__ slab, int32_t P,
                                                     int32_t nact, int32_t splits, int32_t tbm,
                                                     const int32_t* __restrict__ fits,
                                                     float* __restrict__ H) {
    const int slot = blockIdx.y;
    const int64_t PP = (int64_t)P * P;
    for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < PP;
         e += (int64_t)gridDim.x * 256) {
        const int64_t a = e / P, b = e % P;
        if (a / tbm > b / tbm) continue;
        float s = 0.0f;
        for (int z = 0; z < splits; ++z) s += slab[((int64_t)z * nact + slot) * PP + e];
        H[(int64_t)fits[slot] * PP + e] = s;
    }
}
}  // namespace sglm

extern "C" int sglm_syrk_f32(const float* Xf, int64_t ld, int32_t P, int64_t n, const float* W,
                             const int32_t* fits, int32_t nact, int32_t splits, float* H,
                             void* work, sglm_stream_t stream) {
    if (nact <= 0) return SGLM_OK;
    if (!Xf || !W || !fits || !H || P % kFBM || ld % kFBK || n > ld || splits < 1 ||
        (splits > 1 && !work)) {
        set_error("sglm_syrk_f32: bad args");
        return SGLM_EINVAL;
    }
    const int nt = P / kFBM;
    const int ntiles = nt * (nt + 1) / 2;
    const int64_t nst = (n + kFBK - 1) / kFBK;
    const int64_t sps = (nst + splits - 1) / splits;
    hipStream_t s = as_stream(stream);
    float* slab = splits > 1 ? (float*)work : nullptr;
    syrk_f32_kernel<<<dim3((unsigned)(ntiles * nact), (unsigned)splits), 256, 0, s>>>(
        Xf, ld, P, nst, sps, W, fits, ntiles, H, slab, nact);
    int st = check_launch("syrk_f32_kernel");
    if (st || splits == 1) return st;
    const int64_t PP = (int64_t)P * P;
    unsigned gx = (unsigned)((PP + 255) / 256 < 4096 ? (PP + 255) / 256 : 4096);
    syrk_reduce_t<<<dim3(gx, (unsigned)nact), 256, 0, s>>>(slab, P, nact, splits, kFBM, fits, H);
    return check_launch("syrk_reduce_t");
}

// ---------------------------------------------------------------------------------------
// v2: LDS-DMA staging.  Both X panels go global -> LDS with global_load_lds_dwordx4 (no
// VGPR staging, no ds_write); the weights are applied in registers to the B fragments
// after ds_read (8 v_mul + 4 v_cvt_pk per fragment, hidden between MFMAs).
//   * BK = 64 rows per K-step; a predictor's K-slice is one 128-B LDS row; a panel is
//     256 rows x 128 B = 32 KB = 32 wave-instructions of 1 KB (8 predictors each).
//   * 16-B chunk q of predictor c is stored at position q ^ ((c >> 1) & 7): the 16-lane
//     groups of ds_read_b128 (distinct r mod 16) then hit 16 distinct (bank-row half,
//     chunk) pairs -> conflict-free.  The permutation is applied to the per-lane GLOBAL
//     source address (the LDS destination of an LDS-DMA is lane-linear).
//   * diagonal tiles (ti == tj) stage one panel and read both operands from it.
//   * 2 stages x (A 32 KB + B 32 KB + w 256 B) = 128.5 KB LDS, one workgroup per CU.
namespace sglm {
typedef __attribute__((address_space(3))) void lds_void_t;
constexpr int k2BK = 64;
constexpr int k2Panel = 256 * 128;                 // bytes
constexpr int k2Stage = 2 * k2Panel + 256;         // A, B, w[64]

__device__ __forceinline__ void glds16(const void* g, char* l) {
    __builtin_amdgcn_global_load_lds(g, (lds_void_t*)l, 16, 0, 0);
}
__device__ __forceinline__ void glds4(const void* g, char* l) {
    __builtin_amdgcn_global_load_lds(g, (lds_void_t*)l, 4, 0, 0);
}

__global__ void __launch_bounds__(512) syrk2_kernel(
    const uint16_t* __restrict__ Xb, int64_t ld, int32_t P, int64_t nsteps_total,
    int32_t splits, const float* __restrict__ W, const int32_t* __restrict__ fits,
    int32_t ntiles, float* __restrict__ H, float* __restrict__ slab, int32_t nact,
    const int32_t* __restrict__ grp, const int64_t* __restrict__ grp_off,
    const int32_t* __restrict__ grp_cnt) {
    extern __shared__ __attribute__((aligned(16))) char sm2[];
    const int nt = P / 256;
    const int tile = blockIdx.x % ntiles;
    const int slot = blockIdx.x / ntiles;
    const int split = blockIdx.y;
    int ti, tj;
    tile_coords(tile, nt, ti, tj);
    const bool diag = ti == tj;
    const int fit = fits[slot];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wr = wave >> 2, wc = wave & 3;
    const int r = lane & 31, h = lane >> 5;
    // row-group gather: K-step s covers the 8-row groups grp[8s .. 8s+7] of this fit's list
    // (groups holding no training row are skipped); identity when grp == nullptr.
    const int32_t* gl = grp ? grp + grp_off[fit] : nullptr;
    const int64_t ngrp = grp ? (int64_t)grp_cnt[fit] : nsteps_total * 8;
    const int64_t nst_fit = (ngrp + 7) / 8;
    const int64_t sps = (nst_fit + splits - 1) / splits;
    const int64_t step0 = (int64_t)split * sps;
    const int64_t step1 = min(step0 + sps, nst_fit);
    const int64_t nsteps = step1 - step0;
    const uint16_t* XA = Xb + (int64_t)(ti * 256) * ld;
    const uint16_t* XB = Xb + (int64_t)(tj * 256) * ld;
    const float* w = W + (int64_t)fit * ld;

    // LDS-DMA lane mapping: wave handles column blocks cb = 4*wave + u (8 predictors each)
    const int lc = lane >> 3, lpos = lane & 7;
    // column c = (4*wave + u)*8 + lc is the same lc for every u, so the swizzled chunk
    // q(u) = lpos ^ ((c >> 1) & 7) only depends on u through (c >> 1) & 7 = (4u' + lc) >> 1 ...
    int64_t coff[4];
    int qsel[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int c = (4 * wave + u) * 8 + lc;
        coff[u] = (int64_t)c * ld;
        qsel[u] = lpos ^ ((c >> 1) & 7);
    }
    const int64_t glast = ngrp - 1;
    // Group indices of K-step t (8 ints) ride the same LDS-DMA path as the data: wave 0
    // loads those of step t+2 into ring slot (t+2) % 3 while step t+1's panels are issued,
    // so no VGPR-destination global load ever sits in the loop (hipcc would drain the
    // in-flight DMA at its first use).  Identity mapping when there is no list.
    int32_t* iring = reinterpret_cast<int32_t*>(sm2 + 2 * k2Stage);   // 3 x 64 ints
    auto idx_glds = [&](int t) {              // relative step t -> slot t % 3 (wave 0 only)
        if (gl && wave == 0) {
            const int64_t gi = (step0 + t) * 8 + (lane & 7);
            glds4(gl + (gi < ngrp ? gi : glast), reinterpret_cast<char*>(iring + (t % 3) * 64));
        }
    };
    auto group_of = [&](int t, int k) -> int64_t {       // group index of chunk k of step t
        if (!gl) return (step0 + t) * 8 + k;
        return iring[(t % 3) * 64 + k];
    };
    auto stage = [&](int buf, int t) {
        char* base = sm2 + buf * k2Stage;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int64_t row = group_of(t, qsel[u]) * 8;
            glds16(XA + coff[u] + row, base + (4 * wave + u) * 1024);
            if (!diag) glds16(XB + coff[u] + row, base + k2Panel + (4 * wave + u) * 1024);
        }
        if (wave == 0) {
            const int gsel = lane >> 3;
            const int64_t wrow = ((step0 + t) * 8 + gsel < ngrp)
                                     ? group_of(t, gsel) * 8 + (lane & 7)
                                     : (int64_t)ld - 1;      // padding row: w == 0
            glds4(w + wrow, base + 2 * k2Panel);
        }
    };

    f32x16 acc[4][2];
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int n = 0; n < 2; ++n) acc[m][n] = (f32x16){};

    if (nsteps > 0) {
        idx_glds(0);
        if (nsteps > 1) idx_glds(1);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        stage(0, 0);
        if (nsteps > 2) idx_glds(2);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        for (int s = 0; s < (int)nsteps; ++s) {
            const int cur = s & 1;
            if (s + 1 < nsteps) {
                stage(cur ^ 1, s + 1);
                if (s + 3 < nsteps) idx_glds(s + 3);
            }
            const char* A = sm2 + cur * k2Stage;
            const char* Bp = diag ? A : A + k2Panel;
            const float* wv = reinterpret_cast<const float*>(A + 2 * k2Panel);
#pragma unroll
            for (int ks = 0; ks < k2BK / 16; ++ks) {
                const int q = 2 * ks + h;
                bf16x8 af[4], bfr[2];
#pragma unroll
                for (int m = 0; m < 4; ++m) {
                    const int c = wr * 128 + m * 32 + r;
                    af[m] = *reinterpret_cast<const bf16x8*>(A + c * 128 + 16 * (q ^ ((c >> 1) & 7)));
                }
                const f32x4 w0 = *reinterpret_cast<const f32x4*>(wv + 16 * ks + 8 * h);
                const f32x4 w1 = *reinterpret_cast<const f32x4*>(wv + 16 * ks + 8 * h + 4);
#pragma unroll
                for (int n = 0; n < 2; ++n) {
                    const int c = wc * 64 + n * 32 + r;
                    const bf16x8 raw = *reinterpret_cast<const bf16x8*>(Bp + c * 128 + 16 * (q ^ ((c >> 1) & 7)));
                    bf16x8 sc;
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        sc[j] = (__bf16)((float)raw[j] * w0[j]);
                        sc[4 + j] = (__bf16)((float)raw[4 + j] * w1[j]);
                    }
                    bfr[n] = sc;
                }
#pragma unroll
                for (int m = 0; m < 4; ++m)
#pragma unroll
                    for (int n = 0; n < 2; ++n)
                        acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[m], bfr[n],
                                                                            acc[m][n], 0, 0, 0);
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
        }
    }
    float* out = slab ? slab + ((int64_t)split * nact + slot) * (int64_t)P * P
                      : H + (int64_t)fit * P * P;
    const int64_t rbase = (int64_t)ti * 256 + wr * 128;
    const int64_t cbase = (int64_t)tj * 256 + wc * 64;
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int n = 0; n < 2; ++n)
#pragma unroll
            for (int j = 0; j < 16; ++j)
                out[(rbase + m * 32 + (j & 3) + 8 * (j >> 2) + 4 * h) * P + cbase + n * 32 + r] =
                    acc[m][n][j];
}
}  // namespace sglm

static int syrk2_launch(const uint16_t* Xb, int64_t ld, int32_t P, int64_t n, const float* W,
                        const int32_t* fits, int32_t nact, int32_t splits, float* H, void* work,
                        const int32_t* grp, const int64_t* grp_off, const int32_t* grp_cnt,
                        sglm_stream_t stream);

// All rows (w carries the mask): the v2 LDS-DMA kernel without row-group lists.
extern "C" int sglm_syrk(const uint16_t* Xb, int64_t ld, int32_t P, int64_t n, const float* W,
                         const int32_t* fits, int32_t nact, int32_t splits, float* H, void* work,
                         sglm_stream_t stream) {
    return syrk2_launch(Xb, ld, P, n, W, fits, nact, splits, H, work, nullptr, nullptr, nullptr,
                        stream);
}

extern "C" int sglm_syrk_masked(const uint16_t* Xb, int64_t ld, int32_t P, int64_t n,
                                const float* W, const int32_t* fits, int32_t nact,
                                int32_t splits, float* H, void* work, const int32_t* row_groups,
                                const int64_t* group_offset, const int32_t* group_count,
                                sglm_stream_t stream) {
    if (!row_groups || !group_offset || !group_count) {
        set_error("sglm_syrk_masked: null group list");
        return SGLM_EINVAL;
    }
    return syrk2_launch(Xb, ld, P, n, W, fits, nact, splits, H, work, row_groups, group_offset,
                        group_count, stream);
}

static int syrk2_launch(const uint16_t* Xb, int64_t ld, int32_t P, int64_t n, const float* W,
                        const int32_t* fits, int32_t nact, int32_t splits, float* H, void* work,
                        const int32_t* grp, const int64_t* grp_off, const int32_t* grp_cnt,
                        sglm_stream_t stream) {
    if (nact <= 0) return SGLM_OK;
    if (!Xb || !W || !fits || !H || P % 256 || ld % 256 || n > ld || splits < 1 ||
        (splits > 1 && !work)) {
        set_error("sglm_syrk: bad args");
        return SGLM_EINVAL;
    }
    const int nt = P / 256;
    const int ntiles = nt * (nt + 1) / 2;
    const int64_t nst = (n + k2BK - 1) / k2BK;
    const size_t lds = (size_t)2 * k2Stage + 3 * 64 * sizeof(int32_t);
    hipStream_t s = as_stream(stream);
    static bool attr2 = false;
    if (!attr2) {
        (void)hipFuncSetAttribute((const void*)syrk2_kernel,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        attr2 = true;
    }
    float* slab = splits > 1 ? (float*)work : nullptr;
    syrk2_kernel<<<dim3((unsigned)(ntiles * nact), (unsigned)splits), 512, lds, s>>>(
        Xb, ld, P, nst, splits, W, fits, ntiles, H, slab, nact, grp, grp_off, grp_cnt);
    int st = check_launch("syrk2_kernel");
    if (st || splits == 1) return st;
    const int64_t PP = (int64_t)P * P;
    unsigned gx = (unsigned)((PP + 255) / 256 < 4096 ? (PP + 255) / 256 : 4096);
    syrk_reduce<<<dim3(gx, (unsigned)nact), 256, 0, s>>>(slab, P, nact, splits, fits, H);
    return check_launch("syrk_reduce");
}

namespace sglm {
// Bit-plane packing of a feature-major bf16 design: bit b of word q of predictor a is
// (X[a][32q + b] != 0).  One wave per 64 rows: __ballot gives two words at once.  Sets
// *nonbinary if any value is not exactly 0 or 1.
__global__ void __launch_bounds__(256) pack_bits_kernel(const uint16_t* __restrict__ Xb,
                                                        int64_t ld, int32_t P,
                                                        uint32_t* __restrict__ bits,
                                                        int32_t* nonbinary) {
    const int lane = threadIdx.x & 63;
    const int64_t wid = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 6;   // global wave id
    const int64_t per_col = ld / 64;
    const int64_t total = per_col * P;
    for (int64_t g = wid; g < total; g += ((int64_t)gridDim.x * 256) >> 6) {
        const int64_t a = g / per_col, blk = g % per_col;
        const uint16_t v = Xb[a * ld + blk * 64 + lane];
        const bool one = v == 0x3F80u;
        const bool bad = !(one || v == 0 || v == 0x8000u);
        const unsigned long long m = __ballot(one);
        if (__any(bad) && lane == 0) atomicOr(nonbinary, 1);
        if (lane == 0) {
            bits[a * (ld / 32) + blk * 2] = (uint32_t)m;
            bits[a * (ld / 32) + blk * 2 + 1] = (uint32_t)(m >> 32);
        }
    }
}
}  // namespace sglm

extern "C" int sglm_pack_bits(const uint16_t* Xb, int64_t ld, int32_t P, uint32_t* bits,
                              int32_t* nonbinary, sglm_stream_t stream) {
    if (!Xb || !bits || !nonbinary || ld % 64) {
        set_error("sglm_pack_bits: bad args");
        return SGLM_EINVAL;
    }
    pack_bits_kernel<<<2048, 256, 0, as_stream(stream)>>>(Xb, ld, P, bits, nonbinary);
    return check_launch("pack_bits_kernel");
}

// ---------------------------------------------------------------------------------------
// v6: row-compacted bit-plane designs, register-only (no LDS, no barriers).
//   * Every distinct row mask gets its own bit-plane copy holding only its rows
//     (sglm_pack_bits_rows), so the K loop runs over exactly the fit's rows.  The weights are
//     gathered to the same compact order and rounded to bf16 once (sglm_gather_w).
//   * Layout K-step-major: bits[step][predictor] = uint2 (64 rows), so the 128 predictors of
//     a 128-column block are 1 KB contiguous per K-step.  Inside a 32-row word, row rho sits
//     at bit 4*(rho/8) + (rho%8)/2 + 16*(rho%2): the dword of MFMA fragment rows (2j, 2j+1)
//     of 8-row chunk g has its two bits 16 apart at p = 4g + j and p + 16.
//   * A operand (unscaled): rotr(word, p - 14) & 0x40004000 = two bf16 values 2.0 / 0
//     (2 VALU per dword; the factor 2 is removed exactly when storing).  B operand (weighted):
//     pk_ashr_i16(rotr(word, p - 15), 15) -> 16-bit masks, AND bf16 weight pair (3 VALU).
//   * One wave per workgroup computes a 128 x 128 block (4 x 4 tiles of
//     v_mfma_f32_32x32x16_bf16, 256 AGPRs) of the upper triangle (block row <= block col);
//     each lane loads the 8-byte words of its columns straight into registers, two K-steps
//     ahead.  ~80 VALU per 16 MFMA, nothing else in the loop.
//   * per-slot descriptor (4 x int64): bit-plane base, rows, bf16 compact weights, row list
//     (0 = identity; used by the weight gather only).
namespace sglm {

struct Step6 {
    u32x2 a[4], b[4];
    u32x4 w[4];
};

// operand addresses of one wave: scalar bases at K-step 0 and per-step strides (bytes) plus
// the lane's byte offsets (column r of the A / B blocks; row group h of the weights)
struct Addr6 {
    uint64_t a, b, w, stride_ab;
    uint32_t voff_ab, voff_w;
};

__device__ __forceinline__ void load6(Step6& t, const Addr6& ad, int64_t s) {
    const uint64_t sa = ad.a + (uint64_t)s * ad.stride_ab;
    const uint64_t sb = ad.b + (uint64_t)s * ad.stride_ab;
    const uint64_t sw = ad.w + (uint64_t)s * 128;
    t.a[0] = gld2s<0>(sa, ad.voff_ab);
    t.a[1] = gld2s<256>(sa, ad.voff_ab);
    t.a[2] = gld2s<512>(sa, ad.voff_ab);
    t.a[3] = gld2s<768>(sa, ad.voff_ab);
    t.b[0] = gld2s<0>(sb, ad.voff_ab);
    t.b[1] = gld2s<256>(sb, ad.voff_ab);
    t.b[2] = gld2s<512>(sb, ad.voff_ab);
    t.b[3] = gld2s<768>(sb, ad.voff_ab);
    t.w[0] = gld4s<0>(sw, ad.voff_w);
    t.w[1] = gld4s<32>(sw, ad.voff_w);
    t.w[2] = gld4s<64>(sw, ad.voff_w);
    t.w[3] = gld4s<96>(sw, ad.voff_w);
}

__device__ __forceinline__ void wait6(Step6& t) {
    asm volatile("s_waitcnt vmcnt(0)"
                 : "+v"(t.a[0]), "+v"(t.a[1]), "+v"(t.a[2]), "+v"(t.a[3]), "+v"(t.b[0]),
                   "+v"(t.b[1]), "+v"(t.b[2]), "+v"(t.b[3]), "+v"(t.w[0]), "+v"(t.w[1]),
                   "+v"(t.w[2]), "+v"(t.w[3])
                 :
                 : "memory");
}

struct Frag6 {
    bf16x8 a[4], b[4];
};

// fragments of sub-step ks (16 rows) of a K-step: A = 2.0/0 values, B = bf16 weights/0
__device__ __forceinline__ void frags6(const Step6& t, int ks, int h, Frag6& f) {
    const uint32_t p0 = 8 * (ks & 1) + 4 * h;            // bit of row pair j = 0
    const uint32_t wp[4] = {t.w[ks].x, t.w[ks].y, t.w[ks].z, t.w[ks].w};
#pragma unroll
    for (int m = 0; m < 4; ++m) f.a[m] = frag_two(t.a[m], ks, h);
#pragma unroll
    for (int n = 0; n < 4; ++n) {
        const uint32_t word = ks < 2 ? t.b[n].x : t.b[n].y;
        uint32_t d[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const s16x2 v = __builtin_bit_cast(s16x2, rotr32(word, (p0 + j + 17) & 31));
            d[j] = __builtin_bit_cast(uint32_t, (s16x2)(v >> (s16x2){15, 15})) & wp[j];
        }
        f.b[n] = __builtin_bit_cast(bf16x8, make_uint4(d[0], d[1], d[2], d[3]));
    }
}

// 16 MFMAs of one sub-step; a diagonal block (DIAG) skips its 6 strictly-lower 32 x 32
// tiles (never read: consumers use block row <= block col, element row <= col)
template <bool DIAG>
__device__ __forceinline__ void mfma16(const Frag6& f, f32x16 (&acc)[4][4]) {
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int n = 0; n < 4; ++n)
            if (!DIAG || m <= n)
                acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f.a[m], f.b[n], acc[m][n],
                                                                    0, 0, 0);
}

// one scheduling region: the sub-step's MFMAs, each followed by its share of the 80 VALU
// that build the next sub-step's fragments (16 x 5, or 10 x 8 for a diagonal block)
template <bool DIAG>
__device__ __forceinline__ void interleave16() {
#pragma unroll
    for (int i = 0; i < (DIAG ? 10 : 16); ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);     // MFMA
        __builtin_amdgcn_sched_group_barrier(0x002, DIAG ? 8 : 5, 0);     // VALU
    }
    __builtin_amdgcn_sched_barrier(0);
}

// K-step held in `cur` (its sub-step 0 fragments already in F); loads step `snext` into
// `nxt` first and leaves F = sub-step 0 fragments of `nxt`.
template <bool DIAG>
__device__ __forceinline__ void half6(const Step6& cur, Step6& nxt, Frag6& F, int h,
                                      f32x16 (&acc)[4][4], const Addr6& ad, int64_t snext) {
    load6(nxt, ad, snext);
    __builtin_amdgcn_sched_barrier(0);
    Frag6 G;
    frags6(cur, 1, h, G);
    mfma16<DIAG>(F, acc);
    interleave16<DIAG>();
    frags6(cur, 2, h, F);
    mfma16<DIAG>(G, acc);
    interleave16<DIAG>();
    frags6(cur, 3, h, G);
    mfma16<DIAG>(F, acc);
    interleave16<DIAG>();
    wait6(nxt);
    frags6(nxt, 0, h, F);
    mfma16<DIAG>(G, acc);
    interleave16<DIAG>();
}

template <bool DIAG>
__device__ __forceinline__ void gram6_loop(f32x16 (&acc)[4][4], const Addr6& ad, int nsteps,
                                           int h) {
    Step6 A, B;                                      // two register sets, one step in flight
    Frag6 F;
    load6(A, ad, 0);
    wait6(A);
    frags6(A, 0, h, F);
    int s = 0;
    for (; s + 1 < nsteps; s += 2) {
        half6<DIAG>(A, B, F, h, acc, ad, s + 1);
        half6<DIAG>(B, A, F, h, acc, ad, s + 2 < nsteps ? s + 2 : nsteps - 1);
    }
    if (s < nsteps) {                                // odd step count: last step from A
        Frag6 G;
        frags6(A, 1, h, G);
        mfma16<DIAG>(F, acc);
        frags6(A, 2, h, F);
        mfma16<DIAG>(G, acc);
        frags6(A, 3, h, G);
        mfma16<DIAG>(F, acc);
        mfma16<DIAG>(G, acc);
    }
}

// XCD-banded placement of the Gram's 128-blocks (SGLM_SYRK_XCD): the nb block rows are cut
// into four bands of bs = nb / 4 and the ten band pairs (I <= J) dealt to the eight XCDs --
// six off-diagonal pairs one each, the four diagonal pairs two by two -- so an XCD's blocks
// read the bit-plane strips of two bands (8 of the 16 at P = 2048) instead of nearly all of
// them, and its L2 serves each strip to every block that reads it.  Blocks are dealt
// round-robin to the XCDs (b % 8; placement only, not correctness); block b = 8 k + x is item
// k of XCD x's list [(slot, split) major][unit]; past the list's end it returns at once.
__device__ __forceinline__ int xcd_band_units(int x, int bs) {
    return x < 6 ? bs * bs : bs * (bs + 1);
}
__device__ __forceinline__ bool xcd_band_unit(int b, int nb, int nact, int splits, int& slot,
                                              int& split, int& bi, int& bj) {
    const int x = b & 7, k = b >> 3, bs = nb / 4;
    const int u = xcd_band_units(x, bs);
    if (k >= u * nact * splits) return false;
    const int pair = k / u, ui = k % u;
    slot = pair / splits;
    split = pair % splits;
    if (x < 6) {
        const int I = x < 3 ? 0 : (x < 5 ? 1 : 2);
        const int J = x < 3 ? x + 1 : (x < 5 ? x - 1 : 3);
        bi = I * bs + ui / bs;
        bj = J * bs + ui % bs;
    } else {
        const int tri = bs * (bs + 1) / 2;
        const int D = (x - 6) * 2 + (ui >= tri ? 1 : 0);
        int ti, tj;
        tile_coords(ui >= tri ? ui - tri : ui, bs, ti, tj);
        bi = D * bs + ti;
        bj = D * bs + tj;
    }
    return true;
}

__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(1, 1)))
syrk6_kernel(const int64_t* __restrict__ desc, int32_t P, int32_t splits,
             const int32_t* __restrict__ fits, int32_t nunits, float* __restrict__ H,
             float* __restrict__ slab, int32_t nact, int32_t xmap) {
    int slot, split, bi, bj;
    if (xmap) {
        if (!xcd_band_unit(blockIdx.x, P / 128, nact, splits, slot, split, bi, bj)) return;
    } else {
        const int unit = blockIdx.x % nunits;
        slot = blockIdx.x / nunits;
        split = blockIdx.y;
        tile_coords(unit, P / 128, bi, bj);
    }
    const int fit = fits[slot];
    const int64_t* dsc = desc + 4 * slot;
    g_uint2* bits = reinterpret_cast<g_uint2*>(dsc[0]);
    const int64_t nrows = dsc[1];
    const int64_t wbf = dsc[2];                                 // bf16 weights (address)
    const int64_t nblk = (nrows + 63) / 64;
    const int64_t sps = (nblk + splits - 1) / splits;
    const int64_t blk0 = (int64_t)split * sps;
    const int64_t blk1 = min(blk0 + sps, nblk);
    const int nsteps = blk1 > blk0 ? (int)(blk1 - blk0) : 0;
    const int lane = threadIdx.x, r = lane & 31, h = lane >> 5;
    Addr6 ad;
    ad.a = reinterpret_cast<uint64_t>(bits + blk0 * P + bi * 128);
    ad.b = reinterpret_cast<uint64_t>(bits + blk0 * P + bj * 128);
    ad.w = (uint64_t)(wbf + 2 * blk0 * 64);
    ad.stride_ab = (uint64_t)P * 8;
    ad.voff_ab = 8u * r;
    ad.voff_w = 16u * h;

    f32x16 acc[4][4];
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int n = 0; n < 4; ++n) acc[m][n] = (f32x16){};

    if (nsteps > 0) {
        if (bi == bj)
            gram6_loop<true>(acc, ad, nsteps, h);
        else
            gram6_loop<false>(acc, ad, nsteps, h);
    }
    float* out = slab ? slab + ((int64_t)split * nact + slot) * (int64_t)P * P
                      : H + (int64_t)fit * P * P;
    const int64_t rbase = (int64_t)bi * 128;
    const int64_t cbase = (int64_t)bj * 128;
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int n = 0; n < 4; ++n)
#pragma unroll
            for (int j = 0; j < 16; ++j)
                out[(rbase + m * 32 + (j & 3) + 8 * (j >> 2) + 4 * h) * P + cbase + n * 32 + r] =
                    0.5f * acc[m][n][j];
}

// split-K reduction over the 128-blocks v6 writes (block row <= block col)
__global__ void __launch_bounds__(256) syrk6_reduce(const float* __restrict__ slab, int32_t P,
                                                    int32_t nact, int32_t splits,
                                                    const int32_t* __restrict__ fits,
                                                    float* __restrict__ H) {
    const int slot = blockIdx.y;
    const int64_t PP = (int64_t)P * P;
    for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < PP;
         e += (int64_t)gridDim.x * 256) {
        const int64_t a = e / P, b = e % P;
        if (a / 128 > b / 128) continue;
        float s = 0.0f;
        for (int z = 0; z < splits; ++z) s += slab[((int64_t)z * nact + slot) * PP + e];
        H[(int64_t)fits[slot] * PP + e] = s;
    }
}

// Compact bit-plane packing (layout above): output row k = X[.][rows[k]] (rows == nullptr:
// row k) for k < nrows, zero to the next multiple of 64.  One wave per (64-row block,
// predictor), consecutive waves -> consecutive predictors (contiguous 8-B stores); each
// lane's bit is shuffled to its target lane, then one __ballot gives both words.
__global__ void __launch_bounds__(256) pack_bits_rows_kernel(
    const uint16_t* __restrict__ Xb, int64_t ld, int32_t P, const int32_t* __restrict__ rows,
    int64_t nrows, uint2* __restrict__ out, int32_t* nonbinary) {
    const int lane = threadIdx.x & 63;
    const int64_t wid = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
    const int64_t nblk = (nrows + 63) / 64;
    const int64_t total = nblk * P;
    const int src = (lane & 32) | frag_bit_source(lane & 31);
    for (int64_t g = wid; g < total; g += ((int64_t)gridDim.x * 256) >> 6) {
        const int64_t blk = g / P, a = g % P;
        const int64_t k = blk * 64 + lane;
        uint16_t v = 0;
        if (k < nrows) v = Xb[a * ld + (rows ? (int64_t)rows[k] : k)];
        const bool one = v == 0x3F80u;
        const bool bad = !(one || v == 0 || v == 0x8000u);
        const int mine = __shfl((int)one, src, 64);
        const unsigned long long m = __ballot(mine);
        if (__any(bad) && lane == 0) atomicOr(nonbinary, 1);
        if (lane == 0) out[g] = make_uint2((uint32_t)m, (uint32_t)(m >> 32));
    }
}

// Same output as pack_bits_rows_kernel, gathered from the column-packed bit-planes of
// sglm_pack_bits (bit b of word q of predictor a = row 32q + b): 256 MB of source instead of
// the 4 GB bf16 design, so building a fold's compacted design is L2/Infinity-Cache bound.
__global__ void __launch_bounds__(256) compact_bits_kernel(
    const uint32_t* __restrict__ xbits, int64_t ld, int32_t P, const int32_t* __restrict__ rows,
    int64_t nrows, uint2* __restrict__ out) {
    // one wave per (64-row output block, 32 predictors): the row index is loaded once and the
    // 32 predictor words are gathered with 8 loads in flight per lane
    const int lane = threadIdx.x & 63;
    const int64_t wid = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
    const int64_t nblk = (nrows + 63) / 64;
    const int64_t pg = P / 32;
    const int64_t total = nblk * pg;
    const int64_t wpc = ld / 32;
    const int src = (lane & 32) | frag_bit_source(lane & 31);
    for (int64_t g = wid; g < total; g += ((int64_t)gridDim.x * 256) >> 6) {
        const int64_t blk = g / pg, a0 = (g % pg) * 32;
        const int64_t k = blk * 64 + lane;
        const bool valid = k < nrows;
        const int64_t row = valid ? (rows ? (int64_t)rows[k] : k) : 0;
        const uint32_t* base = xbits + a0 * wpc + (row >> 5);
        const int sh = (int)(row & 31);
        for (int a8 = 0; a8 < 32; a8 += 8) {
            uint32_t w[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) w[u] = base[(int64_t)(a8 + u) * wpc];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int one = valid ? (int)((w[u] >> sh) & 1u) : 0;
                const int mine = __shfl(one, src, 64);
                const unsigned long long m = __ballot(mine);
                if (lane == 0)
                    out[blk * P + a0 + a8 + u] = make_uint2((uint32_t)m, (uint32_t)(m >> 32));
            }
        }
    }
}

// Same output again, from the ROW-major planes (rbits[t][i] = the 64 predictor bits of row i,
// predictors 64t..64t+63, fragment order): one wave per (64-row output block, 64-predictor
// group).  Lane l loads the word pair of mask row k = 64 blk + src(l) (so that the ballots come
// out in fragment order), then 64 ballots transpose the 64 x 64 bit tile: ballot j is
// predictor j's 64-row word, kept by lane j, and the wave stores 64 consecutive predictors
// (512 B).  One 8-byte load per row and 64 register ballots, instead of a gather of one bit
// per (row, predictor) from the column-packed planes.
__global__ void __launch_bounds__(256) compact_rbits_kernel(
    const u32x2* __restrict__ rbits, int64_t ld, int32_t P, const int32_t* __restrict__ rows,
    int64_t nrows, uint2* __restrict__ out) {
    const int lane = threadIdx.x & 63;
    const int64_t wid = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
    const int64_t nblk = (nrows + 63) / 64;
    const int32_t ng = P / 64;
    const int64_t total = nblk * ng;
    const int src = (lane & 32) | frag_bit_source(lane & 31);
    for (int64_t g = wid; g < total; g += ((int64_t)gridDim.x * 256) >> 6) {
        const int64_t blk = g / ng;
        const int t = (int)(g % ng);
        const int64_t k = blk * 64 + src;
        u32x2 w = {0u, 0u};
        if (k < nrows) w = rbits[(int64_t)t * ld + (rows ? (int64_t)rows[k] : k)];
        uint32_t lo = 0u, hi = 0u;
#pragma unroll
        for (int j = 0; j < 64; ++j) {
            const int rho = j & 31;
            const int pos = 4 * (rho >> 3) + ((rho & 7) >> 1) + 16 * (rho & 1);
            const uint32_t word = j < 32 ? w.x : w.y;
            const unsigned long long m = __ballot((word >> pos) & 1u);
            lo = lane == j ? (uint32_t)m : lo;
            hi = lane == j ? (uint32_t)(m >> 32) : hi;
        }
        out[blk * P + (int64_t)t * 64 + lane] = make_uint2(lo, hi);
    }
}

// compact bf16 weights: wbf(slot)[k] = bf16(W[fits[slot]][row(k)]) for k < rows, 0 to pad 64
__global__ void __launch_bounds__(256) gather_w_kernel(const float* __restrict__ W, int64_t ld,
                                                       const int32_t* __restrict__ fits,
                                                       const int64_t* __restrict__ desc) {
    const int slot = blockIdx.y;
    const int64_t* dsc = desc + 4 * slot;
    const int64_t nrows = dsc[1];
    __bf16* wc = reinterpret_cast<__bf16*>(dsc[2]);
    const int32_t* rows = reinterpret_cast<const int32_t*>(dsc[3]);
    const float* w = W + (int64_t)fits[slot] * ld;
    const int64_t npad = (nrows + 63) / 64 * 64;
    for (int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x; k < npad;
         k += (int64_t)gridDim.x * 256)
        wc[k] = (__bf16)(k < nrows ? w[rows ? (int64_t)rows[k] : k] : 0.0f);
}
}  // namespace sglm

extern "C" int sglm_pack_bits_rows(const uint16_t* Xb, int64_t ld, int32_t P, const int32_t* rows,
                                   int64_t nrows, uint32_t* out, int32_t* nonbinary,
                                   sglm_stream_t stream) {
    if (!Xb || !out || !nonbinary || nrows < 0 || (!rows && nrows > ld)) {
        set_error("sglm_pack_bits_rows: bad args");
        return SGLM_EINVAL;
    }
    if (nrows == 0) return SGLM_OK;
    pack_bits_rows_kernel<<<4096, 256, 0, as_stream(stream)>>>(
        Xb, ld, P, rows, nrows, reinterpret_cast<uint2*>(out), nonbinary);
    return check_launch("pack_bits_rows_kernel");
}

extern "C" int sglm_compact_bits(const uint32_t* xbits, int64_t ld, int32_t P,
                                 const int32_t* rows, int64_t nrows, uint32_t* out,
                                 sglm_stream_t stream) {
    if (!xbits || !out || nrows < 0 || ld % 64 || (!rows && nrows > ld)) {
        set_error("sglm_compact_bits: bad args");
        return SGLM_EINVAL;
    }
    if (nrows == 0) return SGLM_OK;
    if (P % 32) {
        set_error("sglm_compact_bits: P must be a multiple of 32");
        return SGLM_EINVAL;
    }
    compact_bits_kernel<<<4096, 256, 0, as_stream(stream)>>>(xbits, ld, P, rows, nrows,
                                                              reinterpret_cast<uint2*>(out));
    return check_launch("compact_bits_kernel");
}

extern "C" int sglm_compact_rbits(const uint32_t* rbits, int64_t ld, int32_t P,
                                  const int32_t* rows, int64_t nrows, uint32_t* out,
                                  sglm_stream_t stream) {
    if (!rbits || !out || nrows < 0 || ld % 64 || P % 64 || (!rows && nrows > ld)) {
        set_error("sglm_compact_rbits: bad args");
        return SGLM_EINVAL;
    }
    if (nrows == 0) return SGLM_OK;
    const int64_t waves = (nrows + 63) / 64 * (P / 64);
    const int64_t blocks = (waves + 3) / 4;
    compact_rbits_kernel<<<(unsigned)(blocks < 16384 ? blocks : 16384), 256, 0,
                           as_stream(stream)>>>(reinterpret_cast<const u32x2*>(rbits), ld, P,
                                                rows, nrows, reinterpret_cast<uint2*>(out));
    return check_launch("compact_rbits_kernel");
}

extern "C" int sglm_gather_w(const float* W, int64_t ld, const int32_t* fits, int32_t nact,
                             const int64_t* desc, int64_t max_rows, sglm_stream_t stream) {
    if (nact <= 0) return SGLM_OK;
    if (!W || !fits || !desc || max_rows < 0) {
        set_error("sglm_gather_w: bad args");
        return SGLM_EINVAL;
    }
    const int64_t npad = (max_rows + 63) / 64 * 64;
    unsigned gx = (unsigned)((npad + 2047) / 2048);
    if (gx < 1) gx = 1;
    gather_w_kernel<<<dim3(gx, (unsigned)nact), 256, 0, as_stream(stream)>>>(W, ld, fits, desc);
    return check_launch("gather_w_kernel");
}

extern "C" int sglm_syrk_cbits(const int64_t* desc, int32_t P, const int32_t* fits, int32_t nact,
                               int32_t splits, float* H, void* work, sglm_stream_t stream) {
    if (nact <= 0) return SGLM_OK;
    if (!desc || !fits || !H || P % 256 || splits < 1 || (splits > 1 && !work)) {
        set_error("sglm_syrk_cbits: bad args");
        return SGLM_EINVAL;
    }
    const int nb = P / 128;
    const int nunits = nb * (nb + 1) / 2;
    hipStream_t s = as_stream(stream);
    float* slab = splits > 1 ? (float*)work : nullptr;
    const char* ex = getenv("SGLM_SYRK_XCD");         // read per call (A/B in one process)
    if (ex && ex[0] == '1' && nb % 4 == 0 && nb >= 4) {
        const int bs = nb / 4;
        const unsigned grid = 8u * (unsigned)(bs * (bs + 1) * nact * splits);
        syrk6_kernel<<<grid, 64, 0, s>>>(desc, P, splits, fits, nunits, H, slab, nact, 1);
    } else {
        syrk6_kernel<<<dim3((unsigned)(nunits * nact), (unsigned)splits), 64, 0, s>>>(
            desc, P, splits, fits, nunits, H, slab, nact, 0);
    }
    int st = check_launch("syrk6_kernel");
    if (st || splits == 1) return st;
    const int64_t PP = (int64_t)P * P;
    unsigned gx = (unsigned)((PP + 255) / 256 < 4096 ? (PP + 255) / 256 : 4096);
    syrk6_reduce<<<dim3(gx, (unsigned)nact), 256, 0, s>>>(slab, P, nact, splits, fits, H);
    return check_launch("syrk6_reduce");
}
