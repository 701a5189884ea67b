// eta = X beta on the MFMA path for 0/1 designs (gfx950).
//
// The reference evaluates X @ coef for every loss/gradient evaluation and predict
// (backend/sglm.py:347 -> sklearn glm.py:350).  Here, for a 0/1 design:
//   * X is held a second time as ROW-major bit-planes, K-step-major: rbits[t][i] = uint2 with
//     the 64 bits of predictors 64t..64t+63 of row i, fragment order (common.h), 256 MB at
//     1M x 2048 — built once per design (sglm_pack_bits_t);
//   * beta (f32) is split into three bf16 pieces hi + mid + lo == beta exactly, so the MFMA
//     products (2.0 or 0) x piece are exact and the f32 accumulation is the only rounding —
//     the same accuracy class as an f32 FMA GEMV;
//   * one wave computes 32 fits x 128 rows: A = the 3 x 32 piece rows (loaded directly),
//     B = row bits expanded in registers (2 VALU per dword), acc[3][4] of
//     v_mfma_f32_32x32x16_bf16; the three pieces of a fit land in the same lane, so the
//     result is summed in registers and written coalesced (eta is [fit][row]).
#include "common.h"

namespace sglm {

// rbits[t * ld + i]: bits of X[64t + alpha][i], alpha = 0..63, fragment order.  One thread
// per (row, 64-predictor step); consecutive threads -> consecutive rows (coalesced).
__global__ void __launch_bounds__(256) pack_bits_t_kernel(const uint16_t* __restrict__ Xb,
                                                          int64_t ld, int32_t P,
                                                          u32x2* __restrict__ out,
                                                          int32_t* nonbinary) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int t = blockIdx.y;
    if (i >= ld) return;
    uint32_t w[2] = {0u, 0u};
    bool bad = false;
#pragma unroll 8
    for (int al = 0; al < 64; ++al) {
        const uint16_t v = Xb[(int64_t)(64 * t + al) * ld + i];
        bad |= !(v == 0x3F80u || v == 0 || v == 0x8000u);
        const int rho = al & 31;
        const int pos = 4 * (rho >> 3) + ((rho & 7) >> 1) + 16 * (rho & 1);
        w[al >> 5] |= (uint32_t)(v == 0x3F80u) << pos;
    }
    out[(int64_t)t * ld + i] = (u32x2){w[0], w[1]};
    if (bad) atomicOr(nonbinary, 1);
}

// out[p][f][e] (p = 0,1,2: hi, mid, lo) for f < Bp, e < len; rows f >= B are zero; row f
// holds source row rows[f] (f when rows is null)
__global__ void __launch_bounds__(256) split3_kernel(const float* __restrict__ src, int64_t len,
                                                     int32_t B, int32_t Bp,
                                                     const int32_t* __restrict__ rows,
                                                     __bf16* __restrict__ out) {
    const int64_t total = (int64_t)Bp * len;
    for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total;
         e += (int64_t)gridDim.x * 256) {
        const int64_t f = e / len;
        const float x = f < B ? src[(rows ? (int64_t)rows[f] : f) * len + (e - f * len)] : 0.0f;
        __bf16 hi, mid, lo;
        split3(x, hi, mid, lo);
        out[e] = hi;
        out[total + e] = mid;
        out[2 * total + e] = lo;
    }
}

// One-piece form of the operand for Newton directions: out[f][e] = bf16(src[rows[f]][e]) and
// the source row is overwritten with that bf16 value, so the caller updates its coefficients
// with exactly the direction whose X d the kernel computes (the predictor stays X beta).
__global__ void __launch_bounds__(256) round1_kernel(float* __restrict__ src, int64_t len,
                                                     int32_t B, int32_t Bp,
                                                     const int32_t* __restrict__ rows,
                                                     __bf16* __restrict__ out) {
    const int64_t total = (int64_t)Bp * len;
    for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total;
         e += (int64_t)gridDim.x * 256) {
        const int64_t f = e / len;
        __bf16 v = (__bf16)0.0f;
        if (f < B) {
            float* q = src + (rows ? (int64_t)rows[f] : f) * len + (e - f * len);
            v = (__bf16)*q;
            *q = (float)v;
        }
        out[e] = v;
    }
}

template <int NP, int NT>
struct StepE {
    u32x2 b[NT];         // row bits of the NT row tiles
    u32x4 a[NP][4];      // piece x sub-step: 8 bf16 of this lane's fit
};

template <int NP, int NT>
__device__ __forceinline__ void loadE(StepE<NP, NT>& t, g_uint2* pb, g_uint4* pa, int64_t ld,
                                      int64_t pstride, int s) {
#pragma unroll
    for (int n = 0; n < NT; ++n) t.b[n] = gld2(pb + (int64_t)s * ld + 32 * n);
#pragma unroll
    for (int pc = 0; pc < NP; ++pc)
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) t.a[pc][ks] = gld4(pa + pc * pstride + s * 8 + 2 * ks);
}

// wait until only the two later steps' loads (2 (NT + 4 NP)) are in flight, then tie the step's
// registers
template <int NP, int NT>
__device__ __forceinline__ void waitE(StepE<NP, NT>& t, bool all) {
    constexpr int kLater = 2 * (NT + 4 * NP);
    if (all)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else if constexpr (kLater == 32)
        asm volatile("s_waitcnt vmcnt(32)" ::: "memory");
    else if constexpr (kLater == 24)
        asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
    else if constexpr (kLater == 16)
        asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    else
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
    for (int n = 0; n < NT; ++n) asm volatile("" : "+v"(t.b[n]));
#pragma unroll
    for (int pc = 0; pc < NP; ++pc)
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) asm volatile("" : "+v"(t.a[pc][ks]));
}

template <int NP, int NT>
__device__ __forceinline__ void mmaE(const StepE<NP, NT>& t, int h, f32x16 (&acc)[NP][NT]) {
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
        bf16x8 bx[NT];
#pragma unroll
        for (int n = 0; n < NT; ++n) bx[n] = frag_two(t.b[n], ks, h);
#pragma unroll
        for (int pc = 0; pc < NP; ++pc) {
            const bf16x8 a = __builtin_bit_cast(bf16x8, t.a[pc][ks]);
#pragma unroll
            for (int n = 0; n < NT; ++n)
                acc[pc][n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, bx[n], acc[pc][n], 0, 0, 0);
        }
    }
}

// NP = 3: beta as three bf16 pieces (exact); NP = 1: one bf16 piece (a rounded direction).
// One wave: 32 fits x 32 NT rows (NT = 8 for one piece: the direction pieces are re-read from
// L2 by every wave, so a wave covering more rows halves that traffic; NT = 4 for three pieces,
// whose 3 x 8 accumulator tiles fill the register file).
template <int NP, int NT>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(1, 1)))
eta_bits_kernel(const u32x2* __restrict__ rbits, int64_t ld, int32_t P,
                const __bf16* __restrict__ Dp, int32_t Bp, int32_t B,
                const int32_t* __restrict__ slots, float* __restrict__ eta) {
    const int lane = threadIdx.x, r = lane & 31, h = lane >> 5;
    const int64_t row0 = (int64_t)blockIdx.x * 32 * NT;
    const int g = blockIdx.y;
    g_uint2* pb = as_global<g_uint2>(rbits + row0 + r);
    g_uint4* pa = as_global<g_uint4>(Dp + (int64_t)(g * 32 + r) * P + 8 * h);
    const int64_t pstride = (int64_t)Bp * P / 8;           // one piece plane, in uint4
    const int nsteps = P / 64;

    f32x16 acc[NP][NT];
#pragma unroll
    for (int pc = 0; pc < NP; ++pc)
#pragma unroll
        for (int n = 0; n < NT; ++n) acc[pc][n] = (f32x16){};

    // 3-stage register ring: the loads of step s+2 are issued before step s's MFMAs, so two
    // steps' L2 round trips overlap the MFMA work (clamped duplicate loads at the tail)
    StepE<NP, NT> A, Bs, C;
    const int last = nsteps - 1;
    loadE(A, pb, pa, ld, pstride, 0);
    loadE(Bs, pb, pa, ld, pstride, 1 < last ? 1 : last);
    for (int s = 0; s < nsteps; s += 3) {
        loadE(C, pb, pa, ld, pstride, s + 2 < last ? s + 2 : last);
        waitE(A, false);
        __builtin_amdgcn_sched_barrier(0);
        mmaE(A, h, acc);
        __builtin_amdgcn_sched_barrier(0);
        loadE(A, pb, pa, ld, pstride, s + 3 < last ? s + 3 : last);
        waitE(Bs, false);
        __builtin_amdgcn_sched_barrier(0);
        if (s + 1 < nsteps) mmaE(Bs, h, acc);
        __builtin_amdgcn_sched_barrier(0);
        loadE(Bs, pb, pa, ld, pstride, s + 4 < last ? s + 4 : last);
        waitE(C, false);
        __builtin_amdgcn_sched_barrier(0);
        if (s + 2 < nsteps) mmaE(C, h, acc);
        __builtin_amdgcn_sched_barrier(0);
    }
    waitE(A, true);
    waitE(Bs, true);

#pragma unroll
    for (int n = 0; n < NT; ++n)
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const int f = g * 32 + (j & 3) + 8 * (j >> 2) + 4 * h;
            if (f < B) {
                float v = acc[0][n][j];
                if constexpr (NP == 3) v = (v + acc[1][n][j]) + acc[2][n][j];
                eta[(int64_t)(slots ? slots[f] : f) * ld + row0 + n * 32 + r] = 0.5f * v;
            }
        }
}

// eta on the MFMA with the coefficient tile staged in LDS: a workgroup of four waves covers
// 256 rows (two 32-row tiles per wave) x NG 32-fit groups, so each expanded bit fragment feeds
// NP x NG MFMAs instead of NP (eta_bits_kernel<1, 8>: eight VALU per MFMA for the bit
// expansion, the limiter) and the coefficients cross L2 once per 256 rows for all four waves.
// NP = 1: Newton directions rounded to one bf16 piece, 4 groups (the same products and f32
// accumulation order per (fit, row) as eta_bits_kernel<1, NT>: bitwise equal results).
// NP = 3: exact coefficients as three bf16 pieces, 2 groups, a hi accumulator and a mid + lo
// accumulator per tile (as the gradient kernel).
constexpr int kENT = 2;             // 32-row tiles per wave
constexpr int kEDS = 144;           // LDS bytes per fit segment (64 k x 2 B + pad)

template <int NP, int NG>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2)))
eta_dir_kernel(const u32x2* __restrict__ rbits, int64_t ld, int32_t P,
               const __bf16* __restrict__ Dp, int32_t Bp, int32_t B,
               const int32_t* __restrict__ slots, float* __restrict__ eta) {
    constexpr int kF = NG * 32;                  // fits per workgroup
    constexpr int kJ = NP * NG;                  // staging chunks per thread
    constexpr int kA = NP == 1 ? 1 : 2;          // accumulator sets
    __shared__ __attribute__((aligned(16))) char lds[2][NP * kF * kEDS];
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, r = lane & 31, h = lane >> 5;
    const int64_t row0 = (int64_t)blockIdx.x * (4 * kENT * 32) + wave * (kENT * 32);
    const int gb = blockIdx.y * NG;
    const int ng = min(NG, Bp / 32 - gb);              // fit groups present (uniform)
    const int nsteps = P / 64;
    g_uint2* pb = as_global<g_uint2>(rbits + row0 + r);
    // staging: chunk j of this thread = piece j / NG, fit (tid >> 3) + 32 (j % NG), 16-B
    // piece tid & 7 of that fit's 64-k segment
    const char* dbase = reinterpret_cast<const char*>(Dp) +
                        ((int64_t)(gb * 32 + (tid >> 3)) * P) * 2 + (tid & 7) * 16;
    const int64_t pstride = (int64_t)Bp * P * 2;
    const int lbase = (tid >> 3) * kEDS + (tid & 7) * 16;
    auto goff = [&](int j) { return (j / NG) * pstride + (int64_t)(32 * (j % NG)) * P * 2; };
    auto loff = [&](int j) { return lbase + ((j / NG) * kF + 32 * (j % NG)) * kEDS; };
    auto gl = [&](int j) { return (j % NG) < ng; };
    f32x16 acc[kA][NG][kENT];
#pragma unroll
    for (int a = 0; a < kA; ++a)
#pragma unroll
        for (int gi = 0; gi < NG; ++gi)
#pragma unroll
            for (int n = 0; n < kENT; ++n) acc[a][gi][n] = (f32x16){};
    u32x2 b0[kENT], b1[kENT];
    u32x4 dv[kJ];
    auto gload = [&](u32x2 (&b)[kENT], int s) {
#pragma unroll
        for (int n = 0; n < kENT; ++n) b[n] = gld2(pb + (int64_t)s * ld + 32 * n);
#pragma unroll
        for (int j = 0; j < kJ; ++j)
            if (gl(j)) dv[j] = *reinterpret_cast<const u32x4*>(dbase + goff(j) + (int64_t)s * 128);
    };
    auto sstore = [&](int buf) {
#pragma unroll
        for (int j = 0; j < kJ; ++j)
            if (gl(j)) *reinterpret_cast<u32x4*>(&lds[buf][loff(j)]) = dv[j];
    };
    gload(b0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
    for (int n = 0; n < kENT; ++n) asm volatile("" : "+v"(b0[n]));
    sstore(0);
    __syncthreads();
    // unrolled by two so the bit registers never trade places through copies
    auto step = [&](u32x2 (&bc)[kENT], u32x2 (&bn)[kENT], int s, int cur) {
        const bool more = s + 1 < nsteps;
        if (more) gload(bn, s + 1);
        const char* lb = &lds[cur][r * kEDS + h * 16];
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
            bf16x8 bx[kENT];
#pragma unroll
            for (int n = 0; n < kENT; ++n) bx[n] = frag_two(bc[n], ks, h);
#pragma unroll
            for (int pc = 0; pc < NP; ++pc)
#pragma unroll
                for (int gi = 0; gi < NG; ++gi) {
                    if (gi < ng) {
                        const bf16x8 a = __builtin_bit_cast(bf16x8,
                            *reinterpret_cast<const u32x4*>(lb + (pc * kF + gi * 32) * kEDS +
                                                            32 * ks));
                        const int as = pc == 0 ? 0 : 1;
#pragma unroll
                        for (int n = 0; n < kENT; ++n) {
                            if (NP == 1 || as == 0)
                                acc[0][gi][n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
                                    a, bx[n], acc[0][gi][n], 0, 0, 0);
                            else
                                acc[kA - 1][gi][n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
                                    a, bx[n], acc[kA - 1][gi][n], 0, 0, 0);
                        }
                    }
                }
        }
        if (more) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
            for (int n = 0; n < kENT; ++n) asm volatile("" : "+v"(bn[n]));
            sstore(cur ^ 1);
        }
        __syncthreads();
    };
    int s = 0;
    for (; s + 1 < nsteps; s += 2) {
        step(b0, b1, s, 0);
        step(b1, b0, s + 1, 1);
    }
    if (s < nsteps) step(b0, b1, s, 0);
#pragma unroll
    for (int gi = 0; gi < NG; ++gi) {
        if (gi >= ng) break;
#pragma unroll
        for (int n = 0; n < kENT; ++n)
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                const int f = (gb + gi) * 32 + (j & 3) + 8 * (j >> 2) + 4 * h;
                if (f < B) {
                    const float v = NP == 1 ? acc[0][gi][n][j]
                                            : acc[0][gi][n][j] + acc[kA - 1][gi][n][j];
                    eta[(int64_t)(slots ? slots[f] : f) * ld + row0 + n * 32 + r] = 0.5f * v;
                }
            }
    }
}

// eta_dir_kernel deepened (eta_pipe_kernel<NP, NG, NT, WPE>): each wave covers NT 32-row tiles
// (a staged coefficient fragment feeds NT MFMAs; the coefficient tile crosses L2 once per
// 4 x NT x 32 rows) at WPE waves per SIMD; the bit words are loaded two K-steps ahead through a
// three-set register ring and the next step's coefficient tile one step ahead (all loads in asm
// with static vmcnt counts -- loads for absent fit groups and past the last step re-read valid
// addresses), one barrier per K-step.  The defaults (NT = 2, two waves per SIMD) measured
// fastest: with NT = 4 at one wave per SIMD the per-step barrier bubble is left uncovered.
// NP = 1 (rounded directions): the products and f32 accumulation order per (fit, row) of
// eta_bits_kernel<1, .> -- bitwise equal; NP = 3 (exact coefficients): those of
// eta_dir_kernel<3, .>, a hi accumulator and a mid + lo one -- bitwise equal to it.
template <int NT>
struct EtaRing {
    u32x2 b[NT];
};

template <int NT>
__device__ __forceinline__ void eta_ring_load(EtaRing<NT>& t, g_uint2* pb, int64_t ld, int s) {
#pragma unroll
    for (int n = 0; n < NT; ++n) t.b[n] = gld2(pb + (int64_t)s * ld + 32 * n);
}

template <int NT>
__device__ __forceinline__ void eta_ring_tie(EtaRing<NT>& t) {
#pragma unroll
    for (int n = 0; n < NT; ++n) asm volatile("" : "+v"(t.b[n]));
}

template <int NP, int NG, int NT, int WPE = 1>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE, WPE)))
eta_pipe_kernel(const u32x2* __restrict__ rbits, int64_t ld, int32_t P,
                const __bf16* __restrict__ Dp, int32_t Bp, int32_t B,
                const int32_t* __restrict__ slots, float* __restrict__ eta) {
    constexpr int kF = NG * 32;
    constexpr int kJ = NP * NG;                  // staging chunks per thread
    constexpr int kA = NP == 1 ? 1 : 2;          // accumulator sets
    __shared__ __attribute__((aligned(16))) char lds[2][NP * kF * kEDS];
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, r = lane & 31, h = lane >> 5;
    const int64_t row0 = (int64_t)blockIdx.x * (4 * NT * 32) + wave * (NT * 32);
    const bool live = row0 < ld;                        // wave-uniform (ld % 128 == 0)
    const int gb = blockIdx.y * NG;
    const int ng = min(NG, Bp / 32 - gb);
    const int nsteps = P / 64, last = nsteps - 1;
    g_uint2* pb = as_global<g_uint2>(rbits + (live ? row0 : 0) + r);
    // staging chunk j of this thread: piece j / NG, fit (tid >> 3) + 32 (j % NG) (group 0's
    // row for an absent group), 16-B part tid & 7 of the fit's 64-k segment of the step
    const char* dbase = reinterpret_cast<const char*>(Dp) + (tid & 7) * 16;
    const int64_t pstride = (int64_t)Bp * P * 2;
    int64_t doff[kJ];
#pragma unroll
    for (int j = 0; j < kJ; ++j) {
        const int gi = j % NG;
        doff[j] = (j / NG) * pstride +
                  (int64_t)((gb + (gi < ng ? gi : 0)) * 32 + (tid >> 3)) * P * 2;
    }
    const int lbase = (tid >> 3) * kEDS + (tid & 7) * 16;
    u32x4 dv[kJ];
    auto dload = [&](int st) {
#pragma unroll
        for (int j = 0; j < kJ; ++j)
            dv[j] = gld4(as_global<g_uint4>(dbase + doff[j] + (int64_t)st * 128));
    };
    auto dstore = [&](int buf) {
#pragma unroll
        for (int j = 0; j < kJ; ++j) {
            asm volatile("" : "+v"(dv[j]));
            *reinterpret_cast<u32x4*>(
                &lds[buf][lbase + ((j / NG) * kF + 32 * (j % NG)) * kEDS]) = dv[j];
        }
    };
    f32x16 acc[kA][NG][NT];
#pragma unroll
    for (int a = 0; a < kA; ++a)
#pragma unroll
        for (int gi = 0; gi < NG; ++gi)
#pragma unroll
            for (int n = 0; n < NT; ++n) acc[a][gi][n] = (f32x16){};

    auto compute = [&](const EtaRing<NT>& t, int buf) {
        const char* lb = &lds[buf][r * kEDS + h * 16];
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
            bf16x8 bx[NT];
#pragma unroll
            for (int n = 0; n < NT; ++n) bx[n] = frag_two(t.b[n], ks, h);
#pragma unroll
            for (int pc = 0; pc < NP; ++pc)
#pragma unroll
                for (int gi = 0; gi < NG; ++gi) {
                    if (gi < ng) {
                        const bf16x8 a = __builtin_bit_cast(
                            bf16x8, *reinterpret_cast<const u32x4*>(
                                        lb + (pc * kF + gi * 32) * kEDS + 32 * ks));
                #pragma unroll
                        for (int n = 0; n < NT; ++n) {
                            if (pc == 0)
                                acc[0][gi][n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
                                    a, bx[n], acc[0][gi][n], 0, 0, 0);
                            else
                                acc[kA - 1][gi][n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
                                    a, bx[n], acc[kA - 1][gi][n], 0, 0, 0);
                        }
                    }
                }
        }
    };
    // step st on ring set `cur` (its bits landed) and LDS buffer st & 1: issue the coefficient
    // tile of st + 1 and the bits of st + 2 into `nn`, compute, then wait for everything but
    // the NT bit loads just issued, stage the tile, barrier
    auto step = [&](EtaRing<NT>& cur, EtaRing<NT>& nxt, EtaRing<NT>& nn, int st) {
        dload(st + 1 < last ? st + 1 : last);
        eta_ring_load(nn, pb, ld, st + 2 < last ? st + 2 : last);
        __builtin_amdgcn_sched_barrier(0);
        compute(cur, st & 1);
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (NT == 2)
            asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
        else if constexpr (NT == 4)
            asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        else if constexpr (NT == 8)
            asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        else
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        eta_ring_tie(nxt);
        dstore((st + 1) & 1);
        __syncthreads();
    };

    EtaRing<NT> R0, R1, R2;
    dload(0);
    eta_ring_load(R0, pb, ld, 0);
    eta_ring_load(R1, pb, ld, 1 < last ? 1 : last);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    eta_ring_tie(R0);
    eta_ring_tie(R1);
    dstore(0);
    __syncthreads();
    for (int st = 0; st < nsteps; st += 3) {
        step(R0, R1, R2, st);
        if (st + 1 >= nsteps) break;
        step(R1, R2, R0, st + 1);
        if (st + 2 >= nsteps) break;
        step(R2, R0, R1, st + 2);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (!live) return;
#pragma unroll
    for (int gi = 0; gi < NG; ++gi) {
        if (gi >= ng) break;
#pragma unroll
        for (int n = 0; n < NT; ++n)
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                const int f = (gb + gi) * 32 + (j & 3) + 8 * (j >> 2) + 4 * h;
                if (f < B) {
                    const float v = NP == 1 ? acc[0][gi][n][j]
                                            : acc[0][gi][n][j] + acc[kA - 1][gi][n][j];
                    eta[(int64_t)(slots ? slots[f] : f) * ld + row0 + n * 32 + r] = 0.5f * v;
                }
            }
    }
}

// eta_pipe_kernel (default, both kinds; SGLM_ETA_PIPE=0 for the two-wave eta_dir_kernel /
// one-wave eta_bits_kernel choices below; read per launch)
// Direction products (one piece) by fit-group count, measured in-process (tools/ab_micro.py
// etap, C4 design): two or more groups take eta_pipe_kernel<1, 4, 2> at two waves per SIMD
// (120 fits 0.58 ms against 0.66 for eta_dir_kernel and 0.77 for the one-wave <1, 4, 4>; 96
// fits 0.50 vs 0.57; 64 fits 0.40 vs 0.46), one group eta_bits_kernel<1, 8>.
// SGLM_ETA_PIPE_CFG forces a variant for comparisons: 1 <1, 2, 8>, 2 <1, 4, 2> at two waves per
// SIMD, 3 <1, 4, 4>, 4 <1, 1, 8>.  Exact coefficients take <3, 2, 2> at two waves per SIMD
// (120 fits 1.23 ms against 1.57 for the one-wave <3, 2, 4> and 1.77 for eta_dir_kernel<3, 2>;
// SGLM_ETA3_CFG=0 forces <3, 2, 4>) (read per launch).
static int eta_pipe_cfg() {
    const char* e = getenv("SGLM_ETA_PIPE_CFG");
    return e ? atoi(e) : 0;
}

static bool eta_pipe_on() {
    const char* e = getenv("SGLM_ETA_PIPE");
    return !(e && e[0] == '0');
}

// the staged-direction kernel from four fit groups on (in one process on the C4 design:
// 120 fits 0.80 vs 0.91 ms, 96 fits 0.65 vs 0.68, 70 fits 0.61 vs 0.59, 16 fits 0.32 vs
// 0.16); SGLM_ETA_DIR=0 / 1 force it off / on (read per launch)
static bool eta_dir_on(int32_t Bp) {
    const char* e = getenv("SGLM_ETA_DIR");
    if (e && e[0] == '0') return false;
    if (e && e[0] == '1') return true;
    return Bp / 32 >= 4;
}

// the staged kernel for exact coefficients (three pieces) at every fit count -- one kernel, so
// a fit's eta is bitwise the same whatever else is in the call -- unless
// SGLM_ETA_EXACT_STAGED=0 (read per launch)
static bool eta_exact_staged(int32_t) {
    const char* e = getenv("SGLM_ETA_EXACT_STAGED");
    return !(e && e[0] == '0');
}

// ---------------------------------------------------------------------------------------
// g = X^T R (the gradient, sklearn _linear_loss.py:266-330) on the MFMA for 0/1 designs.
// A = the design's compacted bit-planes with identity rows ([ld/64][P] uint2, the Gram v6
// layout, K = rows), B = R split into three bf16 pieces (exact products); one wave computes
// kXT x 32 predictors x 32 fits over one split-K slab of rows; slabs are reduced in float64 in
// a fixed order.  Two f32 accumulators per tile: the hi piece alone and mid + lo together
// (the small pieces round at their own magnitude, so the sum keeps the accuracy of three
// separate accumulators with two thirds of the registers; 8 tiles per wave still spill).
// Workgroups are numbered so that the predictor panels of one (fit group, row slab) are
// consecutive on one XCD (blocks are dealt round-robin over the 8 XCDs): the slab of R they
// all read comes from that XCD's L2 instead of once per XCD from the fabric.
constexpr int kXT = 4;              // 32-predictor tiles per wave

struct StepX {
    u32x2 a[kXT];        // predictor bits of the tiles, one 64-row block
    u32x4 b[3][4];       // piece x sub-step: 8 bf16 of this lane's fit
};

// Loads from a wave-uniform SGPR base + one per-lane offset + immediates (no per-lane address
// registers): A tile m at +256 m bytes, R piece sub-step ks at +32 ks bytes.
template <int M>
__device__ __forceinline__ void loadA(u32x2 (&a)[kXT], uint64_t sb, uint32_t vo) {
    a[M] = gld2s<M * 256>(sb, vo);
    if constexpr (M + 1 < kXT) loadA<M + 1>(a, sb, vo);
}
template <int KS>
__device__ __forceinline__ void loadB(u32x4 (&b)[4], uint64_t sb, uint32_t vo) {
    b[KS] = gld4s<KS * 32>(sb, vo);
    if constexpr (KS + 1 < 4) loadB<KS + 1>(b, sb, vo);
}

// step s: A bytes at abase + s * P * 8, piece pc of R at bbase + pc * plane + s * 128
__device__ __forceinline__ void loadX(StepX& t, uint64_t abase, uint32_t avo, uint64_t bbase,
                                      uint32_t bvo, uint64_t plane, int32_t P, int64_t s) {
    loadA<0>(t.a, abase + (uint64_t)s * P * 8, avo);
#pragma unroll
    for (int pc = 0; pc < 3; ++pc) loadB<0>(t.b[pc], bbase + pc * plane + (uint64_t)s * 128, bvo);
}

// wait for every load in flight, then tie the step's registers (one empty asm per register,
// after the wait, so no use of them can be scheduled before it)
__device__ __forceinline__ void waitX(StepX& t) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
    for (int m = 0; m < kXT; ++m) asm volatile("" : "+v"(t.a[m]));
#pragma unroll
    for (int pc = 0; pc < 3; ++pc)
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) asm volatile("" : "+v"(t.b[pc][ks]));
}

__device__ __forceinline__ void mmaX(const StepX& t, int h, f32x16 (&ah)[kXT],
                                     f32x16 (&al)[kXT]) {
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
        const bf16x8 b0 = __builtin_bit_cast(bf16x8, t.b[0][ks]);
        const bf16x8 b1 = __builtin_bit_cast(bf16x8, t.b[1][ks]);
        const bf16x8 b2 = __builtin_bit_cast(bf16x8, t.b[2][ks]);
#pragma unroll
        for (int m = 0; m < kXT; ++m) {
            // expand one tile's bits right before its three MFMAs (a fence per tile keeps the
            // compiler from hoisting all expansions: registers, not latency, are the limit)
            const bf16x8 ax = frag_two(t.a[m], ks, h);
            ah[m] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ax, b0, ah[m], 0, 0, 0);
            al[m] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ax, b1, al[m], 0, 0, 0);
            al[m] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ax, b2, al[m], 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
        }
    }
}


__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(1, 1)))
xtr_bits_kernel(const u32x2* __restrict__ cbits, int64_t ld, int32_t P, int64_t nblk,
                const __bf16* __restrict__ Rp, int32_t Bp, int32_t Bps, int32_t B,
                int32_t splits, float* __restrict__ part) {
    const int lane = threadIdx.x, r = lane & 31, h = lane >> 5;
    const int npan = P / (32 * kXT), ngrp = Bp / 32;
    const int L = xcd_logical(blockIdx.x, npan * ngrp * splits);
    const int pn = L % npan, g = (L / npan) % ngrp, z = L / (npan * ngrp);
    const int64_t sps = (nblk + splits - 1) / splits;
    const int64_t blk0 = (int64_t)z * sps;
    const int64_t blk1 = min(blk0 + sps, nblk);
    const int nsteps = blk1 > blk0 ? (int)(blk1 - blk0) : 0;
    const uint64_t abase = (uint64_t)(cbits + blk0 * P);
    const uint32_t avo = (uint32_t)((pn * (32 * kXT) + r) * 8);
    const uint64_t bbase = (uint64_t)(Rp + blk0 * 64);
    const uint32_t bvo = (uint32_t)(((int64_t)(g * 32 + r) * ld + 8 * h) * 2);
    const uint64_t plane = (uint64_t)Bps * ld * 2;     // rows per R piece plane

    f32x16 ah[kXT], al[kXT];
#pragma unroll
    for (int m = 0; m < kXT; ++m) {
        ah[m] = (f32x16){};
        al[m] = (f32x16){};
    }
    if (nsteps > 0) {
        StepX A, Bs;
        loadX(A, abase, avo, bbase, bvo, plane, P, 0);
        waitX(A);
        int s = 0;
        for (; s + 1 < nsteps; s += 2) {
            loadX(Bs, abase, avo, bbase, bvo, plane, P, s + 1);
            __builtin_amdgcn_sched_barrier(0);
            mmaX(A, h, ah, al);
            __builtin_amdgcn_sched_barrier(0);
            waitX(Bs);
            loadX(A, abase, avo, bbase, bvo, plane, P, s + 2 < nsteps ? s + 2 : nsteps - 1);
            __builtin_amdgcn_sched_barrier(0);
            mmaX(Bs, h, ah, al);
            __builtin_amdgcn_sched_barrier(0);
            waitX(A);
        }
        if (s < nsteps) mmaX(A, h, ah, al);
    }
    // D[row = predictor][col = fit]: lane r = fit, reg j -> predictor (j&3)+8(j>>2)+4h
    const int f = g * 32 + r;
    if (f < B) {
        float* out = part + ((int64_t)z * B + f) * P + pn * (32 * kXT);
#pragma unroll
        for (int m = 0; m < kXT; ++m)
#pragma unroll
            for (int j = 0; j < 16; ++j)
                out[m * 32 + (j & 3) + 8 * (j >> 2) + 4 * h] = 0.5f * (ah[m][j] + al[m][j]);
    }
}

// Four panels per workgroup (256 predictors... 512 with kXT = 4: one panel per wave), the
// three R pieces of the 32 fits staged through LDS once per 64-row step for all four waves:
// R crosses L2 once per 512 predictors instead of once per 128 (xtr_bits_kernel), the A
// operand (bit-planes) is per wave as before.  Same MFMA sequence per wave, so the same
// partial sums bit for bit.  LDS: 2 buffers x 3 pieces x 32 fits x 144 B (a fit's 64-row
// segment is 128 B; the 16-B pad spreads the 8 lanes of each ds_read_b128 pass over all banks).
constexpr int kXW = 4;              // waves (panels) per workgroup
constexpr int kRS = 144;            // LDS bytes per fit segment (128 + pad)

// NGW = 32-fit groups per workgroup: with two, every expanded bit fragment feeds six MFMAs
// (three pieces x two groups) instead of three -- the bit expansion is VALU work that the
// single MFMA stream of a one-wave-per-SIMD kernel cannot hide.
// WPE = waves per SIMD: 2 (one fit group, <= 256 registers per lane) doubles the loads in
// flight of the latency-bound small batches, at the price of the SIMD room a concurrent
// factorisation chain needs.
template <int NGW, int WPE = 1>
__global__ void __launch_bounds__(64 * kXW) __attribute__((amdgpu_waves_per_eu(WPE, WPE)))
xtr_bits4_kernel(const u32x2* __restrict__ cbits, int64_t ld, int32_t P, int64_t nblk,
                 const __bf16* __restrict__ Rp, int32_t Bp, int32_t Bps, int32_t B,
                 int32_t splits, float* __restrict__ part) {
    constexpr int kF = NGW * 32;                 // fits per workgroup
    constexpr int kJ = 3 * NGW;                  // staging chunks per thread
    __shared__ __attribute__((aligned(16))) char lds[2][3 * kF * kRS];
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, r = lane & 31, h = lane >> 5;
    const int npan4 = P / (32 * kXT * kXW), ngrp = Bp / 32, ngrp2 = (ngrp + NGW - 1) / NGW;
    const int L = xcd_logical(blockIdx.x, npan4 * ngrp2 * splits);
    const int pq = L % npan4, g2 = (L / npan4) % ngrp2, z = L / (npan4 * ngrp2);
    const int g0 = g2 * NGW, ngv = min(NGW, ngrp - g0);       // groups present (uniform)
    const int pn = pq * kXW + wave;
    const int64_t sps = (nblk + splits - 1) / splits;
    const int64_t blk0 = (int64_t)z * sps;
    const int64_t blk1 = min(blk0 + sps, nblk);
    const int nsteps = blk1 > blk0 ? (int)(blk1 - blk0) : 0;
    const uint64_t abase = (uint64_t)(cbits + blk0 * P);
    const uint32_t avo = (uint32_t)((pn * (32 * kXT) + r) * 8);
    // R staging: thread tid moves 16-B chunks c = tid + 256 j of the step's tile: piece
    // c / (256 NGW), fit (c >> 3) % kF, chunk c & 7 of that fit's 128-B row segment
    const char* rb = reinterpret_cast<const char*>(Rp) + blk0 * 128;
    const int64_t plane = (int64_t)Bps * ld * 2;       // rows per R piece plane
    // chunk j: piece j / NGW, fit (tid >> 3) + 32 (j % NGW) -- a per-thread base plus
    // wave-uniform strides (kept in scalar registers)
    const int64_t gbase = (int64_t)(g0 * 32 + (tid >> 3)) * ld * 2 + (tid & 7) * 16;
    const int64_t gstep = (int64_t)32 * ld * 2;
    const int lbase = (tid >> 3) * kRS + (tid & 7) * 16;
    auto goff = [&](int j) { return gbase + (j / NGW) * plane + (j % NGW) * gstep; };
    auto loff = [&](int j) { return lbase + ((j / NGW) * kF + 32 * (j % NGW)) * kRS; };
    auto gl = [&](int j) { return (j % NGW) < ngv; };
    f32x16 ah[NGW][kXT], al[NGW][kXT];
#pragma unroll
    for (int gi = 0; gi < NGW; ++gi)
#pragma unroll
        for (int m = 0; m < kXT; ++m) {
            ah[gi][m] = (f32x16){};
            al[gi][m] = (f32x16){};
        }
    if (nsteps > 0) {
        u32x2 a0[kXT], a1[kXT];
        u32x4 rv[kJ];
        loadA<0>(a0, abase, avo);
#pragma unroll
        for (int j = 0; j < kJ; ++j)
            if (gl(j)) rv[j] = *reinterpret_cast<const u32x4*>(rb + goff(j));
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
        for (int j = 0; j < kJ; ++j)
            if (gl(j)) *reinterpret_cast<u32x4*>(&lds[0][loff(j)]) = rv[j];
        __syncthreads();
        // one step on A registers ac with the next step's loads into an: the loop is unrolled
        // by two so the buffers never trade places through copies (an asm-loaded register
        // copied before its s_waitcnt would copy stale data)
        auto step = [&](u32x2 (&ac)[kXT], u32x2 (&an)[kXT], int s, int cur) {
            const bool more = s + 1 < nsteps;
            if (more) {
                loadA<0>(an, abase + (uint64_t)(s + 1) * P * 8, avo);
#pragma unroll
                for (int j = 0; j < kJ; ++j)
                    if (gl(j))
                        rv[j] = *reinterpret_cast<const u32x4*>(rb + (int64_t)(s + 1) * 128 +
                                                                goff(j));
            }
#pragma unroll
            for (int m = 0; m < kXT; ++m) asm volatile("" : "+v"(ac[m]));
            // per K-slice: the four tiles' expansions, then the MFMAs ordered by piece so that
            // the two accumulations into al are 4 NGW MFMAs apart (each accumulator still sums
            // b1 then b2 per slice: the same results bit for bit)
            const char* lb = &lds[cur][r * kRS + h * 16];
#pragma unroll
            for (int ks = 0; ks < 4; ++ks) {
                bf16x8 ax[kXT];
#pragma unroll
                for (int m = 0; m < kXT; ++m) ax[m] = frag_two(ac[m], ks, h);
#pragma unroll
                for (int pc = 0; pc < 3; ++pc)
#pragma unroll
                    for (int gi = 0; gi < NGW; ++gi) {
                        if (gi < ngv) {
                            const bf16x8 b = __builtin_bit_cast(bf16x8,
                                *reinterpret_cast<const u32x4*>(
                                    lb + (pc * kF + gi * 32) * kRS + 32 * ks));
#pragma unroll
                            for (int m = 0; m < kXT; ++m) {
                                if (pc == 0)
                                    ah[gi][m] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
                                        ax[m], b, ah[gi][m], 0, 0, 0);
                                else
                                    al[gi][m] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
                                        ax[m], b, al[gi][m], 0, 0, 0);
                            }
                        }
                    }
            }
            if (more) {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
                for (int m = 0; m < kXT; ++m) asm volatile("" : "+v"(an[m]));
#pragma unroll
                for (int j = 0; j < kJ; ++j)
                    if (gl(j)) *reinterpret_cast<u32x4*>(&lds[cur ^ 1][loff(j)]) = rv[j];
            }
            __syncthreads();
        };
        int s = 0;
        for (; s + 1 < nsteps; s += 2) {
            step(a0, a1, s, 0);
            step(a1, a0, s + 1, 1);
        }
        if (s < nsteps) step(a0, a1, s, 0);
    }
#pragma unroll
    for (int gi = 0; gi < NGW; ++gi) {
        const int f = (g0 + gi) * 32 + r;
        if (gi < ngv && f < B) {
            float* out = part + ((int64_t)z * B + f) * P + pn * (32 * kXT);
#pragma unroll
            for (int m = 0; m < kXT; ++m)
#pragma unroll
                for (int j = 0; j < 16; ++j)
                    out[m * 32 + (j & 3) + 8 * (j >> 2) + 4 * h] =
                        0.5f * (ah[gi][m][j] + al[gi][m][j]);
        }
    }
}

// ---- software-pipelined four-panel gradient (xtr_bits5_kernel) ----------------------------
// The same workgroup tiling, LDS staging and MFMA sequence as xtr_bits4_kernel (so the same
// partial sums bit for bit), scheduled the way the Gram mainloop is (syrk.hip half6): the
// fragments of sub-step ks + 1 -- the bit expansions (32 VALU) and the R reads from LDS
// (3 NGW ds_read_b128) -- are built while the MFMAs of sub-step ks run, one or two per MFMA gap,
// instead of in a block between MFMA groups that a one-wave-per-SIMD kernel cannot hide.  The
// step's single barrier sits between sub-steps 2 and 3, after the staging write of the next
// step; the loads of step s + 2 are issued right after it (into the A registers step s no
// longer needs), so a load has four sub-steps (~3,000 cycles at NGW = 2) to land.  R is loaded
// in inline asm from a scalar base and one per-lane 32-bit offset (a plain load may be sunk to
// its use by the compiler, which would expose its whole latency at the staging write).
template <int NGW, int NPC>
struct XFrag {
    bf16x8 a[kXT];          // expanded bit fragments of the wave's tiles
    bf16x8 b[NPC][NGW];     // R piece x fit group, from LDS
};

template <int NGW, int NPC>
__device__ __forceinline__ void xfrags(const u32x2 (&ac)[kXT], const char* lb, int ks, int h,
                                       XFrag<NGW, NPC>& f) {
    constexpr int kF = NGW * 32;
#pragma unroll
    for (int m = 0; m < kXT; ++m) f.a[m] = frag_two(ac[m], ks, h);
#pragma unroll
    for (int pc = 0; pc < NPC; ++pc)
#pragma unroll
        for (int gi = 0; gi < NGW; ++gi)
            f.b[pc][gi] = __builtin_bit_cast(
                bf16x8, *reinterpret_cast<const u32x4*>(lb + (pc * kF + gi * 32) * kRS + 32 * ks));
}

// one sub-step's MFMAs in xtr_bits4_kernel's order (piece, group, tile)
template <int NGW, int NPC>
__device__ __forceinline__ void xmfma(const XFrag<NGW, NPC>& f, f32x16 (&ah)[NGW][kXT],
                                      f32x16 (&al)[NGW][kXT]) {
#pragma unroll
    for (int pc = 0; pc < NPC; ++pc)
#pragma unroll
        for (int gi = 0; gi < NGW; ++gi)
#pragma unroll
            for (int m = 0; m < kXT; ++m) {
                if (pc == 0)
                    ah[gi][m] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f.a[m], f.b[pc][gi],
                                                                        ah[gi][m], 0, 0, 0);
                else
                    al[gi][m] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f.a[m], f.b[pc][gi],
                                                                        al[gi][m], 0, 0, 0);
            }
}

// the sub-step's MFMAs, each followed by its share of the next fragments' LDS reads and VALU
template <int NGW, int NPC>
__device__ __forceinline__ void xinterleave() {
#ifdef XTR_NO_INTERLEAVE
    return;
#endif
    constexpr int NM = NPC * NGW * kXT;           // MFMAs
    constexpr int ND = NPC * NGW;                 // ds_read_b128
    constexpr int NV = (8 * kXT + NM - 1) / NM;   // VALU per gap (32 expansion VALU in all)
#pragma unroll
    for (int i = 0; i < NM; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);          // MFMA
        if (i < ND) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);   // DS read
        __builtin_amdgcn_sched_group_barrier(0x002, NV, 0);         // VALU
    }
    __builtin_amdgcn_sched_barrier(0);
}

template <int NGW, int WPE = 1, int NPC = 3>
__global__ void __launch_bounds__(64 * kXW) __attribute__((amdgpu_waves_per_eu(WPE, WPE)))
xtr_bits5_kernel(const u32x2* __restrict__ cbits, int64_t ld, int32_t P, int64_t nblk,
                 const __bf16* __restrict__ Rp, int32_t Bp, int32_t Bps, int32_t B,
                 int32_t splits, float* __restrict__ part) {
    constexpr int kF = NGW * 32;                 // fits per workgroup
    constexpr int kJ = NPC * NGW;                // staging chunks per thread
    __shared__ __attribute__((aligned(16))) char lds[2][NPC * kF * kRS];
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, r = lane & 31, h = lane >> 5;
    const int npan4 = P / (32 * kXT * kXW), ngrp = Bp / 32, ngrp2 = (ngrp + NGW - 1) / NGW;
    const int L = xcd_logical(blockIdx.x, npan4 * ngrp2 * splits);
    const int pq = L % npan4, g2 = (L / npan4) % ngrp2, z = L / (npan4 * ngrp2);
    const int g0 = g2 * NGW, ngv = min(NGW, ngrp - g0);       // groups present (uniform)
    const int pn = pq * kXW + wave;
    const int64_t sps = (nblk + splits - 1) / splits;
    const int64_t blk0 = (int64_t)z * sps;
    const int64_t blk1 = min(blk0 + sps, nblk);
    const int nsteps = blk1 > blk0 ? (int)(blk1 - blk0) : 0;
    const uint64_t abase = (uint64_t)(cbits + blk0 * P);
    const uint32_t avo = (uint32_t)((pn * (32 * kXT) + r) * 8);
    // staging chunk j (16 B): piece j / NGW, fit (tid >> 3) + 32 (j % NGW), byte 16 (tid & 7)
    // of the fit's 128-B row segment; an absent group (ngv < NGW) re-reads group 0 (never used)
    const uint64_t rbase = (uint64_t)(reinterpret_cast<const char*>(Rp) + blk0 * 128 +
                                      (int64_t)g0 * 32 * ld * 2);
    const uint32_t rvo = (uint32_t)((tid >> 3) * ld * 2 + (tid & 7) * 16);
    const uint64_t plane = (uint64_t)Bps * ld * 2;     // rows per R piece plane
    const uint64_t gstep = (uint64_t)32 * ld * 2;
    auto joff = [&](int j) {
        const int gi = j % NGW;
        return (uint64_t)(j / NGW) * plane + (gi < ngv ? (uint64_t)gi * gstep : 0);
    };
    const int lbase = (tid >> 3) * kRS + (tid & 7) * 16;
    auto loff = [&](int j) { return lbase + ((j / NGW) * kF + 32 * (j % NGW)) * kRS; };
    if (nsteps <= 0) {                          // an empty slab: zero partials, no loop
#pragma unroll
        for (int gi = 0; gi < NGW; ++gi) {
            const int f = (g0 + gi) * 32 + r;
            if (gi < ngv && f < B) {
                float* out = part + ((int64_t)z * B + f) * P + pn * (32 * kXT);
                for (int m = 0; m < kXT; ++m)
                    for (int j = 0; j < 16; ++j) out[m * 32 + (j & 3) + 8 * (j >> 2) + 4 * h] = 0.0f;
            }
        }
        return;
    }
    f32x16 ah[NGW][kXT], al[NGW][kXT];
#pragma unroll
    for (int gi = 0; gi < NGW; ++gi)
#pragma unroll
        for (int m = 0; m < kXT; ++m) {
            ah[gi][m] = (f32x16){};
            al[gi][m] = (f32x16){};
        }
    {
        u32x2 a0[kXT] = {}, a1[kXT] = {};
        u32x4 rv[kJ];
        auto issue = [&](u32x2 (&an)[kXT], int s) {
            loadA<0>(an, abase + (uint64_t)s * P * 8, avo);
#pragma unroll
            for (int j = 0; j < kJ; ++j) rv[j] = gld4s<0>(rbase + (uint64_t)s * 128 + joff(j), rvo);
        };
        auto land = [&](u32x2 (&an)[kXT], int buf) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
            for (int m = 0; m < kXT; ++m) asm volatile("" : "+v"(an[m]));
#pragma unroll
            for (int j = 0; j < kJ; ++j) asm volatile("" : "+v"(rv[j]));
#pragma unroll
            for (int j = 0; j < kJ; ++j) *reinterpret_cast<u32x4*>(&lds[buf][loff(j)]) = rv[j];
        };
        const int lofs = r * kRS + h * 16;
        XFrag<NGW, NPC> F, G;
        issue(a0, 0);
        land(a0, 0);
        __syncthreads();
        if (nsteps > 1) issue(a1, 1);
        xfrags<NGW, NPC>(a0, &lds[0][lofs], 0, h, F);
        // step s from A registers ac and LDS buffer c (F = its sub-step 0 fragments; the loads
        // of step s + 1 in flight into an and rv); leaves F = sub-step 0 of step s + 1
        auto step = [&](u32x2 (&ac)[kXT], u32x2 (&an)[kXT], int s, int c) {
            const char* lb = &lds[c][lofs];
            __builtin_amdgcn_sched_barrier(0);
            xfrags<NGW, NPC>(ac, lb, 1, h, G);
            xmfma<NGW, NPC>(F, ah, al);
            xinterleave<NGW, NPC>();
            xfrags<NGW, NPC>(ac, lb, 2, h, F);
            xmfma<NGW, NPC>(G, ah, al);
            xinterleave<NGW, NPC>();
            xfrags<NGW, NPC>(ac, lb, 3, h, G);
            xmfma<NGW, NPC>(F, ah, al);
            xinterleave<NGW, NPC>();
            const bool more = s + 1 < nsteps;
            if (more) land(an, c ^ 1);
            __syncthreads();
            if (s + 2 < nsteps) issue(ac, s + 2);
            __builtin_amdgcn_sched_barrier(0);
            // unconditional (one scheduling region with the MFMAs): past the last step it
            // expands stale registers and LDS that nothing uses
            xfrags<NGW, NPC>(an, &lds[c ^ 1][lofs], 0, h, F);
            xmfma<NGW, NPC>(G, ah, al);
            xinterleave<NGW, NPC>();
        };
        int s = 0;
        for (; s + 1 < nsteps; s += 2) {
            step(a0, a1, s, 0);
            step(a1, a0, s + 1, 1);
        }
        if (s < nsteps) step(a0, a1, s, 0);
    }
#pragma unroll
    for (int gi = 0; gi < NGW; ++gi) {
        const int f = (g0 + gi) * 32 + r;
        if (gi < ngv && f < B) {
            float* out = part + ((int64_t)z * B + f) * P + pn * (32 * kXT);
#pragma unroll
            for (int m = 0; m < kXT; ++m)
#pragma unroll
                for (int j = 0; j < 16; ++j)
                    out[m * 32 + (j & 3) + 8 * (j >> 2) + 4 * h] =
                        NPC == 1 ? 0.5f * ah[gi][m][j] : 0.5f * (ah[gi][m][j] + al[gi][m][j]);
        }
    }
}

// Gradient kernel per call (read per launch: tests switch it inside one process):
//   2 = four-panel, two fit groups per workgroup -- an even group count (P % 512 == 0);
//   0 = one-panel -- otherwise (an odd count leaves half-empty two-group workgroups, and the
//       one-group four-panel kernel measured no faster than the one-panel kernel once the
//       row slabs fill whole rounds: C4, 120 fits 1.20 / 1.46 / 1.43 ms, 70 fits
//       1.19 / 1.13 / 1.08 ms for variants 2 / 1 / 0 in one process);
//   1 = four-panel, one group -- only on request.
// SGLM_XTR4=0 forces 0, SGLM_XTR_NGW=1 / 2 / 3 force 1 / 2 / 3 where P allows.
// sglm_xtr_prefer(1) (per thread) asks for the one-group four-panel kernel: 262 registers
// per lane leave room on every SIMD for the factorisation chain's waves (the two-group kernel
// holds all 512), so a chain running beside the gradient progresses instead of waiting for it.
static thread_local int t_xtr_prefer = -1;
// SGLM_XTR_PIPE (read per launch; default 1): the software-pipelined kernel (xtr_bits5_kernel)
// for the four-panel variants.  Measured on the C4 design, 120 / 70 fits: 1.30 / 1.19 ms
// (two groups) -> 1.03 / 0.95 pipelined; the two-wave one-group form pipelined 0.99 / 0.72,
// the fastest of all -- the pipelined default.
static bool xtr_pipe() {
    const char* ep = getenv("SGLM_XTR_PIPE");
    return !(ep && ep[0] == '0');
}
static int xtr_variant(int32_t P, int32_t B) {
    const int ngrp = (B + 31) / 32;
    if (P % (32 * kXT * kXW) != 0) return 0;
    if (t_xtr_prefer == 1) return 1;
    const char* e3 = getenv("SGLM_XTR_WPE2");
    const bool wpe2 = !(e3 && e3[0] == '0');
    const char* e4 = getenv("SGLM_XTR4");
    if (e4 && e4[0] == '0') return 0;
    const char* e = getenv("SGLM_XTR_NGW");
    if (e && e[0] == '1') return 1;
    if (e && e[0] == '2') return ngrp >= 2 ? 2 : 1;
    if (e && e[0] == '3') return 3;
    if (xtr_pipe()) return wpe2 ? 3 : 1;
    if (ngrp >= 2 && ngrp % 2 == 0) return 2;
    return wpe2 ? 3 : 0;
}

static void launch_xtr_bits(const u32x2* cbits, int64_t ld, int32_t P, int64_t nblk,
                            const __bf16* Rp, int32_t Bp, int32_t Bps, int32_t B, int32_t splits,
                            float* part, hipStream_t s) {
    const int v = xtr_variant(P, B);
    const unsigned tiles = (unsigned)((P / (32 * kXT)) * (Bp / 32) * splits);
    const int ngw = v == 2 ? 2 : 1;
    const unsigned wgs4 = (unsigned)((P / (32 * kXT * kXW)) * ((Bp / 32 + ngw - 1) / ngw) *
                                     splits);
    // the pipelined kernel (SGLM_XTR_PIPE, read per launch) takes R's per-lane offsets in 32 bits
    const bool pipe = v != 0 && xtr_pipe() && (int64_t)32 * ld * 2 < ((int64_t)1 << 32);
    if (pipe) {
        if (v == 3)
            xtr_bits5_kernel<1, 2><<<wgs4, 64 * kXW, 0, s>>>(cbits, ld, P, nblk, Rp, Bp, Bps, B,
                                                             splits, part);
        else if (v == 2)
            xtr_bits5_kernel<2><<<wgs4, 64 * kXW, 0, s>>>(cbits, ld, P, nblk, Rp, Bp, Bps, B, splits,
                                                          part);
        else
            xtr_bits5_kernel<1><<<wgs4, 64 * kXW, 0, s>>>(cbits, ld, P, nblk, Rp, Bp, Bps, B, splits,
                                                          part);
        return;
    }
    if (v == 3)
        xtr_bits4_kernel<1, 2><<<wgs4, 64 * kXW, 0, s>>>(cbits, ld, P, nblk, Rp, Bp, Bps, B, splits,
                                                         part);
    else if (v == 2)
        xtr_bits4_kernel<2><<<wgs4, 64 * kXW, 0, s>>>(cbits, ld, P, nblk, Rp, Bp, Bps, B, splits, part);
    else if (v == 1)
        xtr_bits4_kernel<1><<<wgs4, 64 * kXW, 0, s>>>(cbits, ld, P, nblk, Rp, Bp, Bps, B, splits, part);
    else
        xtr_bits_kernel<<<tiles, 64, 0, s>>>(cbits, ld, P, nblk, Rp, Bp, Bps, B, splits, part);
}

// out[slots[f]][a] = sum over slabs z of part[z][f][a] (f = e / P), fixed order
__global__ void __launch_bounds__(256) reduce_slabs_f64(const float* __restrict__ part,
                                                        int64_t len, int32_t nz, int32_t P,
                                                        const int32_t* __restrict__ slots,
                                                        double* __restrict__ out) {
    for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < len;
         e += (int64_t)gridDim.x * 256) {
        double s = 0.0;
        for (int z = 0; z < nz; ++z) s += (double)part[(int64_t)z * len + e];
        const int64_t f = e / P;
        out[(slots ? (int64_t)slots[f] : f) * P + (e - f * P)] = s;
    }
}

// Row slabs of the gradient: the workgroup count is a multiple of the row-slab count, and
// both kernels hold one wave per SIMD (256 four-wave workgroups, or 1024 one-wave workgroups,
// resident at once), so the slab count minimises rounds x (K-steps per slab + a fixed cost
// of ~8 steps per workgroup) -- a grid just over a multiple of the resident count would run a
// nearly empty extra round.  four = the four-panel kernel.
static int xtr_splits_for(int32_t P, int32_t B, int64_t nblk, int variant) {
    const int64_t ngrp = (B + 31) / 32;
    const int ngw = variant == 2 ? 2 : 1;
    const int64_t wps = variant ? (P / (32 * kXT * kXW)) * ((ngrp + ngw - 1) / ngw)
                                : (P / (32 * kXT)) * ngrp;
    const int64_t resident = variant == 3 ? 512 : variant ? 256 : 1024;
    const int64_t cap = nblk / 32 > 1 ? nblk / 32 : 1;      // >= 32 K-steps per slab
    int best = 1;
    double bestc = 1e300;
    for (int64_t s = 1; s <= cap && s <= 4096; ++s) {
        const double c = (double)((wps * s + resident - 1) / resident) *
                         ((double)((nblk + s - 1) / s) + 8.0);
        if (c < bestc) {
            bestc = c;
            best = (int)s;
        }
    }
    return best;
}
static int xtr_bits_splits(int32_t P, int32_t B, int64_t nblk) {
    return xtr_splits_for(P, B, nblk, xtr_variant(P, B));
}
// sglm_xtr_bits keeps every row slab at <= 1024 K-steps (65,536 rows): integer-valued R pieces
// with |piece| <= 128 (the digit planes of enet.xty) then sum EXACTLY in the f32 accumulators
// (|2 x 128 x 65536| = 2^24 with the 2.0 operand encoding), and the float64 slab reduction is
// exact too
constexpr int64_t kExactSlabSteps = 1024;
static int xtr_bits_splits_capped(int32_t P, int32_t B, int64_t nblk) {
    const int s = xtr_bits_splits(P, B, nblk);
    const int64_t lo = (nblk + kExactSlabSteps - 1) / kExactSlabSteps;
    return (int64_t)s < lo ? (int)lo : s;
}
// workspace bound over every variant (the switches may change between the query and a launch)
static size_t xtr_part_bytes(int32_t P, int32_t B, int64_t nblk) {
    const int s = std::max(std::max(xtr_splits_for(P, B, nblk, 0), xtr_splits_for(P, B, nblk, 3)),
                           std::max(xtr_splits_for(P, B, nblk, 1), xtr_splits_for(P, B, nblk, 2)));
    return (size_t)s * B * P * sizeof(float);
}

// Balanced base-256 digit planes of fixed-point m*y (the exact X^T(m y) of 0/1 designs):
// pair i = (response pr[i], mask pm[i]); v = rint(m[row] * y[row] * scale[i]) (|v| < 2^38 by the
// caller's scale), digit q = ((v + 128) mod 256) - 128, v <- (v - digit) / 256, written as bf16
// (exact) to D[q * c + i][row].  Rows >= n are not written (the caller keeps them zero).
__global__ void __launch_bounds__(256) digit_planes_kernel(
    const uint8_t* __restrict__ M, int64_t ldm, const double* __restrict__ Y, int64_t ldy,
    int64_t n, const int32_t* __restrict__ pr, const int32_t* __restrict__ pm,
    const double* __restrict__ scale, int32_t c, int32_t nd, __bf16* __restrict__ D,
    int64_t ld) {
    const int i = blockIdx.y;
    const uint8_t* m = M + (int64_t)pm[i] * ldm;
    const double* y = Y + (int64_t)pr[i] * ldy;
    const double sc = scale[i];
    for (int64_t row = (int64_t)blockIdx.x * 256 + threadIdx.x; row < n;
         row += (int64_t)gridDim.x * 256) {
        const double mv = (double)m[row];
        int64_t v = mv == 0.0 ? 0 : (int64_t)rint(mv * y[row] * sc);
        for (int q = 0; q < nd; ++q) {
            const int64_t dq = ((v + 128) & 255) - 128;       // floor mod for two's complement
            D[((int64_t)q * c + i) * ld + row] = (__bf16)(float)dq;
            v = (v - dq) >> 8;                                // exact: v - dq is a multiple of 256
        }
    }
}

}  // namespace sglm

using namespace sglm;

extern "C" {

int sglm_xtr_prefer(int32_t variant) {
    t_xtr_prefer = variant == 1 ? 1 : -1;
    return SGLM_OK;
}

int sglm_pack_bits_t(const uint16_t* Xb, int64_t ld, int32_t P, uint32_t* out,
                     int32_t* nonbinary, sglm_stream_t stream) {
    if (!Xb || !out || !nonbinary || ld % 256 || P % 64) {
        set_error("sglm_pack_bits_t: bad args");
        return SGLM_EINVAL;
    }
    pack_bits_t_kernel<<<dim3((unsigned)(ld / 256), (unsigned)(P / 64)), 256, 0,
                         as_stream(stream)>>>(Xb, ld, P, reinterpret_cast<u32x2*>(out),
                                              nonbinary);
    return check_launch("pack_bits_t_kernel");
}

size_t sglm_eta_bits_work_bytes(int32_t P, int32_t B) {
    const int64_t Bp = ((int64_t)B + 31) / 32 * 32;
    return (size_t)3 * (size_t)Bp * (size_t)P * 2;
}

int sglm_gemv_eta_bits(const uint32_t* rbits, int64_t ld, int32_t P, float* beta,
                       int32_t B, const int32_t* slots, int32_t exact, float* eta, void* work,
                       sglm_stream_t stream) {
    if (B <= 0) return SGLM_OK;
    if (!rbits || !beta || !eta || !work || ld % 256 || P % 256) {
        set_error("sglm_gemv_eta_bits: bad args");
        return SGLM_EINVAL;
    }
    const int32_t Bp = (B + 31) / 32 * 32;
    hipStream_t s = as_stream(stream);
    __bf16* Dp = reinterpret_cast<__bf16*>(work);
    const int64_t total = (int64_t)Bp * P;
    const unsigned gs = (unsigned)((total + 255) / 256 < 2048 ? (total + 255) / 256 : 2048);
    int st;
    if (exact) {
        split3_kernel<<<gs, 256, 0, s>>>(beta, P, B, Bp, slots, Dp);
        st = check_launch("split3_kernel");
        if (st) return st;
        const char* e3 = getenv("SGLM_ETA3_CFG");
        if (eta_pipe_on() && !(e3 && e3[0] == '0'))
            eta_pipe_kernel<3, 2, 2, 2><<<dim3((unsigned)(ld / 256), (unsigned)((Bp / 32 + 1) / 2)),
                                          256, 0, s>>>(reinterpret_cast<const u32x2*>(rbits), ld,
                                                       P, Dp, Bp, B, slots, eta);
        else if (eta_pipe_on())
            eta_pipe_kernel<3, 2, 4><<<dim3((unsigned)((ld + 511) / 512), (unsigned)((Bp / 32 + 1) / 2)),
                                       256, 0, s>>>(reinterpret_cast<const u32x2*>(rbits), ld, P,
                                                    Dp, Bp, B, slots, eta);
        else if (eta_exact_staged(Bp))
            eta_dir_kernel<3, 2><<<dim3((unsigned)(ld / 256), (unsigned)((Bp / 32 + 1) / 2)),
                                   256, 0, s>>>(reinterpret_cast<const u32x2*>(rbits), ld, P,
                                                Dp, Bp, B, slots, eta);
        else
            eta_bits_kernel<3, 4><<<dim3((unsigned)(ld / 128), (unsigned)(Bp / 32)), 64, 0, s>>>(
                reinterpret_cast<const u32x2*>(rbits), ld, P, Dp, Bp, B, slots, eta);
    } else {
        round1_kernel<<<gs, 256, 0, s>>>(beta, P, B, Bp, slots, Dp);
        st = check_launch("round1_kernel");
        if (st) return st;
        const int ngr = Bp / 32;
        const u32x2* rb = reinterpret_cast<const u32x2*>(rbits);
        const int cfg = eta_pipe_on() ? eta_pipe_cfg() : -1;
        if (cfg == 2 || (cfg == 0 && ngr >= 2))
            eta_pipe_kernel<1, 4, 2, 2><<<dim3((unsigned)((ld + 255) / 256), (unsigned)((ngr + 3) / 4)),
                                          256, 0, s>>>(rb, ld, P, Dp, Bp, B, slots, eta);
        else if (cfg == 1)
            eta_pipe_kernel<1, 2, 8><<<dim3((unsigned)((ld + 1023) / 1024), (unsigned)((ngr + 1) / 2)),
                                       256, 0, s>>>(rb, ld, P, Dp, Bp, B, slots, eta);
        else if (cfg == 3)
            eta_pipe_kernel<1, 4, 4><<<dim3((unsigned)((ld + 511) / 512), (unsigned)((ngr + 3) / 4)),
                                    256, 0, s>>>(rb, ld, P, Dp, Bp, B, slots, eta);
        else if (cfg == 4)
            eta_pipe_kernel<1, 1, 8><<<dim3((unsigned)((ld + 1023) / 1024), (unsigned)ngr), 256, 0,
                                       s>>>(rb, ld, P, Dp, Bp, B, slots, eta);
        else if (eta_dir_on(Bp))
            eta_dir_kernel<1, 4><<<dim3((unsigned)(ld / 256), (unsigned)((Bp / 32 + 3) / 4)),
                                   256, 0, s>>>(reinterpret_cast<const u32x2*>(rbits), ld, P,
                                                Dp, Bp, B, slots, eta);
        else
            eta_bits_kernel<1, 8><<<dim3((unsigned)(ld / 256), (unsigned)(Bp / 32)), 64, 0, s>>>(
                reinterpret_cast<const u32x2*>(rbits), ld, P, Dp, Bp, B, slots, eta);
    }
    return check_launch("eta_bits_kernel");
}

size_t sglm_xtr_bits_work_bytes(int32_t P, int32_t B, int64_t ld) {
    const int64_t Bp = ((int64_t)B + 31) / 32 * 32;
    const int64_t nblk = ld / 64;
    const int64_t lo = (nblk + kExactSlabSteps - 1) / kExactSlabSteps;
    const size_t floor_bytes = (size_t)lo * B * P * sizeof(float);
    const size_t part = xtr_part_bytes(P, B, nblk);
    return (size_t)3 * Bp * ld * 2 + (part > floor_bytes ? part : floor_bytes);
}

int sglm_xtr_bits(const uint32_t* cbits, int64_t ld, int32_t P, int64_t n, const float* R,
                  int32_t B, double* G, void* work, sglm_stream_t stream) {
    if (B <= 0) return SGLM_OK;
    if (!cbits || !R || !G || !work || ld % 256 || P % 256 || n > ld) {
        set_error("sglm_xtr_bits: bad args");
        return SGLM_EINVAL;
    }
    const int32_t Bp = (B + 31) / 32 * 32;
    const int64_t nblk = (n + 63) / 64;
    const int splits = xtr_bits_splits_capped(P, B, ld / 64);
    hipStream_t s = as_stream(stream);
    __bf16* Rp = reinterpret_cast<__bf16*>(work);
    float* part = reinterpret_cast<float*>(reinterpret_cast<char*>(work) + (size_t)3 * Bp * ld * 2);
    const int64_t total = (int64_t)Bp * ld;
    split3_kernel<<<(unsigned)((total + 255) / 256 < 8192 ? (total + 255) / 256 : 8192), 256, 0,
                    s>>>(R, ld, B, Bp, nullptr, Rp);
    int st = check_launch("split3_kernel");
    if (st) return st;
    launch_xtr_bits(reinterpret_cast<const u32x2*>(cbits), ld, P, nblk, Rp, Bp, Bp, B, splits,
                    part, s);
    st = check_launch("xtr_bits_kernel");
    if (st) return st;
    const int64_t len = (int64_t)B * P;
    reduce_slabs_f64<<<(unsigned)((len + 255) / 256 < 4096 ? (len + 255) / 256 : 4096), 256, 0,
                       s>>>(part, len, splits, P, nullptr, G);
    return check_launch("reduce_slabs_f64");
}

// X^T R with R already in the packed three-piece operand layout ([3][Bp][ld] bf16, as
// sglm_link_update writes it): G[slots[f]] (float64) for f < B.  `work`: the slab partials,
// sglm_xtr_bits_packed_work_bytes(P, B, ld): enough for any call with at most B fits (fewer
// fits take more row slabs, so the bound is the maximum over b <= B).
size_t sglm_xtr_bits_packed_work_bytes(int32_t P, int32_t B, int64_t ld) {
    size_t mx = 0;
    for (int32_t b = 1; b <= B; ++b) {
        const size_t w = xtr_part_bytes(P, b, ld / 64);
        mx = w > mx ? w : mx;
    }
    return mx;
}

int sglm_digit_planes(const uint8_t* M, int64_t ldm, const double* Y, int64_t ldy, int64_t n,
                      const int32_t* pr, const int32_t* pm, const double* scale, int32_t c,
                      int32_t nd, void* D, int64_t ld, sglm_stream_t stream) {
    if (c <= 0 || n <= 0) return SGLM_OK;
    if (!M || !Y || !pr || !pm || !scale || !D || nd < 1 || nd > 8 || n > ld || n > ldm ||
        n > ldy || c > 65535) {
        set_error("sglm_digit_planes: bad args");
        return SGLM_EINVAL;
    }
    const int64_t gx = (n + 255) / 256 < 1024 ? (n + 255) / 256 : 1024;
    digit_planes_kernel<<<dim3((unsigned)gx, (unsigned)c), 256, 0, as_stream(stream)>>>(
        M, ldm, Y, ldy, n, pr, pm, scale, c, nd, reinterpret_cast<__bf16*>(D), ld);
    return check_launch("digit_planes_kernel");
}

// X^T D for integer-valued columns D (|d| <= 256, exact in bf16: one piece instead of three),
// D given as bf16 [Bp][ld] (rows B..Bp-1 readable, their results unused).  The pipelined
// kernel with one piece: four 32-column groups per workgroup (the accumulators the two low
// pieces used), row slabs of <= 1024 K-steps so the f32 sums of integers stay exact (|2 d| x
// 65,536 <= 2^25: the operand 2.0 doubles the products; sums up to 2^24 x 2 are exact in f32
// for even integers).  P % 512 == 0.
static int xtr_int_ngw(int32_t B) {
    const int ngrp = (B + 31) / 32;
    return ngrp >= 4 ? 4 : ngrp >= 2 ? 2 : 1;
}
static int xtr_int_splits(int32_t P, int32_t B, int64_t nblk) {
    const int64_t ngw = xtr_int_ngw(B), ngrp = (B + 31) / 32;
    const int64_t wps = (P / (32 * kXT * kXW)) * ((ngrp + ngw - 1) / ngw);
    const int64_t cap = nblk / 32 > 1 ? nblk / 32 : 1;
    int best = 1;
    double bestc = 1e300;
    for (int64_t s = 1; s <= cap && s <= 4096; ++s) {
        const double c = (double)((wps * s + 255) / 256) * ((double)((nblk + s - 1) / s) + 8.0);
        if (c < bestc) {
            bestc = c;
            best = (int)s;
        }
    }
    const int64_t lo = (nblk + kExactSlabSteps - 1) / kExactSlabSteps;
    return (int64_t)best < lo ? (int)lo : best;
}

size_t sglm_xtr_bits_int_work_bytes(int32_t P, int32_t B, int64_t ld) {
    return (size_t)xtr_int_splits(P, B, ld / 64) * B * P * sizeof(float);
}

int sglm_xtr_bits_int(const uint32_t* cbits, int64_t ld, int32_t P, int64_t n, const void* D,
                      int32_t B, double* G, void* work, sglm_stream_t stream) {
    if (B <= 0) return SGLM_OK;
    if (!cbits || !D || !G || !work || ld % 256 || P % 512 || n > ld ||
        (int64_t)32 * ld * 2 >= ((int64_t)1 << 32)) {
        set_error("sglm_xtr_bits_int: bad args (P %% 512, ld < 2^26)");
        return SGLM_EINVAL;
    }
    const int32_t Bp = (B + 31) / 32 * 32;
    const int64_t nblk = (n + 63) / 64;
    const int splits = xtr_int_splits(P, B, ld / 64);
    const int ngw = xtr_int_ngw(B);
    const unsigned wgs = (unsigned)((P / (32 * kXT * kXW)) * ((Bp / 32 + ngw - 1) / ngw) * splits);
    hipStream_t s = as_stream(stream);
    float* part = reinterpret_cast<float*>(work);
    const u32x2* cb = reinterpret_cast<const u32x2*>(cbits);
    const __bf16* Db = reinterpret_cast<const __bf16*>(D);
    if (ngw == 4)
        xtr_bits5_kernel<4, 1, 1><<<wgs, 64 * kXW, 0, s>>>(cb, ld, P, nblk, Db, Bp, Bp, B, splits, part);
    else if (ngw == 2)
        xtr_bits5_kernel<2, 1, 1><<<wgs, 64 * kXW, 0, s>>>(cb, ld, P, nblk, Db, Bp, Bp, B, splits, part);
    else
        xtr_bits5_kernel<1, 1, 1><<<wgs, 64 * kXW, 0, s>>>(cb, ld, P, nblk, Db, Bp, Bp, B, splits, part);
    int st = check_launch("xtr_bits5_kernel<1 piece>");
    if (st) return st;
    const int64_t len = (int64_t)B * P;
    reduce_slabs_f64<<<(unsigned)((len + 255) / 256 < 4096 ? (len + 255) / 256 : 4096), 256, 0,
                       s>>>(part, len, splits, P, nullptr, G);
    return check_launch("reduce_slabs_f64");
}

int sglm_xtr_bits_packed(const uint32_t* cbits, int64_t ld, int32_t P, int64_t n,
                         const void* Rp, int32_t B, const int32_t* slots, double* G, void* work,
                         sglm_stream_t stream) {
    return sglm_xtr_bits_packed_bp(cbits, ld, P, n, Rp, B, (B + 31) / 32 * 32, slots, G, work,
                                   stream);
}

int sglm_xtr_bits_packed_bp(const uint32_t* cbits, int64_t ld, int32_t P, int64_t n,
                            const void* Rp, int32_t B, int32_t Bp, const int32_t* slots,
                            double* G, void* work, sglm_stream_t stream) {
    if (B <= 0) return SGLM_OK;
    if (!cbits || !Rp || !G || !work || ld % 256 || P % 256 || n > ld || Bp % 32 ||
        Bp < (B + 31) / 32 * 32) {
        set_error("sglm_xtr_bits_packed: bad args");
        return SGLM_EINVAL;
    }
    const int64_t nblk = (n + 63) / 64;
    const int splits = xtr_bits_splits(P, B, ld / 64);
    hipStream_t s = as_stream(stream);
    float* part = reinterpret_cast<float*>(work);
    // Bp: the planes' row stride (>= the fit groups' padded count, which the kernels use)
    launch_xtr_bits(reinterpret_cast<const u32x2*>(cbits), ld, P, nblk,
                    reinterpret_cast<const __bf16*>(Rp), (B + 31) / 32 * 32, Bp, B, splits, part,
                    s);
    int st = check_launch("xtr_bits_kernel");
    if (st) return st;
    const int64_t len = (int64_t)B * P;
    reduce_slabs_f64<<<(unsigned)((len + 255) / 256 < 4096 ? (len + 255) / 256 : 4096), 256, 0,
                       s>>>(part, len, splits, P, slots, G);
    return check_launch("reduce_slabs_f64");
}

}  // extern "C"
