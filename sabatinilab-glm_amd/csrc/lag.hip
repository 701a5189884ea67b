// Gradient of a time-shifted event design, from the events themselves.
//
// The design of the north-star configuration is a timeshift expansion (backend/sglm_pp.py:
// 23-103, sglm_ez.timeshift_cols): column (b, a) of X is event column a of the base matrix E
// shifted by s_b rows, X[t, (b, a)] = E[t + row0 - s_b, a].  For a 0/1 event matrix
//     g[(b, a)] = sum_t R[t] X[t, (b, a)] = sum over occurrences u of event a of R[u - row0 + s_b],
// so X^T R needs every R value once per occurrence window (K lags), not once per predictor:
// ~ nnz(E) * K adds per fit instead of n * p.  (The dense bit-plane MFMA path, xtr_bits, reads
// each R row for every 128-predictor panel and needs three bf16 pieces of R to be exact.)
//
// Work split: a workgroup owns a fit group (FG fits, lanes = (fit, lag) pairs) and a range of
// row tiles (kLagU design rows each).  Per tile it stages R[f][t0 .. t0 + kLagU) in LDS, then
// walks every event's occurrences whose window reaches the tile (offsets precomputed per tile)
// and adds R[u - row0 + s_b] for its lag when that row lies in the tile: consecutive lanes read
// consecutive LDS words (conflict-free), all lanes walk the same occurrence list (uniform
// control flow).  One float64 accumulator per event stays in registers across the tiles of the
// range; the range's partial sums go to `work` and a fixed-order pass sums the ranges (the
// result does not depend on scheduling).  The intercept column p is the plain sum of R.
#include "common.h"

namespace sglm {
namespace {

constexpr int kLagT = 256;        // threads per workgroup: (fit, lag) pairs
constexpr int kLagU = 4096;       // design rows per tile
constexpr int kLagFG = 6;         // fits per workgroup at most (LDS: kLagFG x kLagU floats)
constexpr int kLagC = 8192;       // occurrences staged in LDS per chunk
constexpr int kLagMaxM = 64;      // events (register accumulators per lane)

struct LagArgs {
    const int32_t* occ;           // occurrence rows u of every event, event-major, ascending
    const int32_t* tbeg;          // [m][ntiles]: first occurrence index of event a whose
    const int32_t* tend;          //   window reaches tile i / one past the last
    const int32_t* shifts;        // [K]
    int32_t m, K, layout, P;      // layout 0: column b*m + a (shift-major), 1: a*K + b
    int64_t row0, n, ntiles;
};

// LDS: R tile [kLagFG][kLagU] f32 | occurrences [kLagC] i32 | per-event chunk ranges
struct LagLds {
    float r[kLagFG * kLagU];
    int32_t occ[kLagC];
    int32_t beg[kLagMaxM], len[kLagMaxM];          // this tile's segment of each event
    int32_t lo[kLagMaxM], hi[kLagMaxM];            // its part in the current chunk
    int32_t src[kLagMaxM];                         // occ index of lo
    int32_t done;                                  // all segments staged
};

template <int MAXM>
__global__ void __launch_bounds__(kLagT) lag_xtr_kernel(LagArgs a, const float* __restrict__ R,
                                                        int64_t ld,
                                                        const int32_t* __restrict__ slots,
                                                        int32_t nact, int32_t FG,
                                                        int32_t tiles_per,
                                                        double* __restrict__ part) {
    extern __shared__ __attribute__((aligned(16))) char lds_raw[];
    LagLds& L = *reinterpret_cast<LagLds*>(lds_raw);
    const int tid = threadIdx.x;
    const int f = tid / a.K, b = tid - f * a.K;
    const int q = blockIdx.y * FG + f;             // index in the active list
    const bool on = f < FG && q < nact;
    const int64_t range = blockIdx.x;
    const int64_t tile0 = range * tiles_per;
    const int64_t tile1 = tile0 + tiles_per < a.ntiles ? tile0 + tiles_per : a.ntiles;
    const int s = on ? a.shifts[b] : 0;
    const int nf = (nact - (int)blockIdx.y * FG) < FG ? (nact - (int)blockIdx.y * FG) : FG;
    double acc[MAXM];
#pragma unroll
    for (int e = 0; e < MAXM; ++e) acc[e] = 0.0;
    // intercept column: the plain sum of R, accumulated by the staging threads (thread tid,
    // fit ff: rows tid, tid + 256, ... of every tile), reduced in a fixed order at the end
    double accI[kLagFG];
#pragma unroll
    for (int ff = 0; ff < kLagFG; ++ff) accI[ff] = 0.0;
    for (int64_t tile = tile0; tile < tile1; ++tile) {
        const int64_t t0 = tile * kLagU;
        __syncthreads();                           // the previous tile's reads are done
        // R rows of the tile, float4 loads (kLagU and t0 are multiples of 4; ld >= n, and
        // rows past n are masked to 0)
#pragma unroll
        for (int ff = 0; ff < kLagFG; ++ff) {
            if (ff < nf) {
                const float* r = R + (int64_t)slots[blockIdx.y * FG + ff] * ld;
                f32x4 v[kLagU / 4 / kLagT];
#pragma unroll
                for (int j = 0; j < kLagU / 4 / kLagT; ++j) {
                    const int64_t t = t0 + 4 * (tid + j * kLagT);
                    v[j] = t + 4 <= a.n ? *reinterpret_cast<const f32x4*>(r + t)
                                        : f32x4{t < a.n ? r[t] : 0.0f,
                                                t + 1 < a.n ? r[t + 1] : 0.0f,
                                                t + 2 < a.n ? r[t + 2] : 0.0f, 0.0f};
                }
#pragma unroll
                for (int j = 0; j < kLagU / 4 / kLagT; ++j) {
                    *reinterpret_cast<f32x4*>(&L.r[ff * kLagU + 4 * (tid + j * kLagT)]) = v[j];
                    accI[ff] += ((double)v[j][0] + (double)v[j][1]) +
                                ((double)v[j][2] + (double)v[j][3]);
                }
            }
        }
        if (tid < a.m) {
            const int32_t i0 = a.tbeg[(int64_t)tid * a.ntiles + tile];
            L.beg[tid] = i0;
            L.len[tid] = a.tend[(int64_t)tid * a.ntiles + tile] - i0;
        }
        if (tid == 0) L.done = 0;
        const int64_t off = s - a.row0 - t0;       // tile row of occurrence u: u + off
        int e_cur = 0, i_cur = 0;                  // next segment position (uniform)
        while (true) {
            __syncthreads();
            if (L.done) break;
            // chunk layout (thread 0, which alone carries the resume point): whole or partial
            // event segments from (e_cur, i_cur), at most kLagC occurrences
            if (tid == 0) {
                int fill = 0, e = e_cur, i = i_cur;
                for (int x = 0; x < a.m; ++x) { L.lo[x] = 0; L.hi[x] = 0; }
                while (e < a.m && fill < kLagC) {
                    const int take = min(L.len[e] - i, kLagC - fill);
                    L.lo[e] = fill; L.hi[e] = fill + take; L.src[e] = L.beg[e] + i;
                    fill += take;
                    i += take;
                    if (i == L.len[e]) { ++e; i = 0; }
                }
                L.done = e >= a.m ? 2 : 0;                        // 2: the last chunk
                e_cur = e;
                i_cur = i;
            }
            __syncthreads();
            // stage the chunk's occurrences: flattened position j -> (event, index); each
            // thread walks j = tid, tid + 256, ... with a monotone event cursor, 4 loads in
            // flight at a time
            {
                int fill = 0;
                for (int x = 0; x < a.m; ++x) fill = L.hi[x] > fill ? L.hi[x] : fill;
                int e = 0;
                for (int j0 = tid; j0 < fill; j0 += 4 * kLagT) {
                    int32_t v[4];
                    int jj[4];
#pragma unroll
                    for (int z = 0; z < 4; ++z) {
                        const int j = j0 + z * kLagT;
                        jj[z] = j;
                        v[z] = 0;
                        if (j < fill) {
                            while (L.hi[e] <= j) ++e;
                            int ez = e;
                            while (L.lo[ez] > j) --ez;
                            v[z] = a.occ[L.src[ez] + (j - L.lo[ez])];
                        }
                    }
#pragma unroll
                    for (int z = 0; z < 4; ++z)
                        if (jj[z] < fill) L.occ[jj[z]] = v[z];
                }
            }
            __syncthreads();
            const float* rf = L.r + f * kLagU;
#pragma unroll
            for (int e = 0; e < MAXM; ++e) {
                if (e < a.m) {
                    const int i0 = L.lo[e], i1 = L.hi[e];
                    // 8 occurrences per step: their LDS reads are independent, the f64 sum is
                    // a fixed pairwise tree (deterministic)
                    double se = 0.0;
                    int i = i0;
                    for (; i + 8 <= i1; i += 8) {
                        float v[8];
#pragma unroll
                        for (int z = 0; z < 8; ++z) {
                            const int64_t tr = (int64_t)L.occ[i + z] + off;
                            v[z] = (on && tr >= 0 && tr < kLagU) ? rf[tr] : 0.0f;
                        }
                        se += (((double)v[0] + (double)v[1]) + ((double)v[2] + (double)v[3])) +
                              (((double)v[4] + (double)v[5]) + ((double)v[6] + (double)v[7]));
                    }
                    for (; i < i1; ++i) {
                        const int64_t tr = (int64_t)L.occ[i] + off;
                        if (on && tr >= 0 && tr < kLagU) se += (double)rf[tr];
                    }
                    acc[e] += se;
                }
            }
            __syncthreads();
            if (tid == 0) L.done = L.done == 2 ? 1 : 0;
        }
    }
    __syncthreads();                               // LDS reused for the intercept sums
    double* red = reinterpret_cast<double*>(lds_raw);  // [nf][kLagT]
#pragma unroll
    for (int ff = 0; ff < kLagFG; ++ff)
        if (ff < nf) red[ff * kLagT + tid] = accI[ff];
    __syncthreads();
    double I = 0.0;
    if (on && b == 0)
        for (int i = 0; i < kLagT; ++i) I += red[f * kLagT + i];
    if (!on) return;
    double* out = part + (range * nact + q) * (int64_t)a.P;
#pragma unroll
    for (int e = 0; e < MAXM; ++e) {
        if (e < a.m) {
            const int col = a.layout ? e * a.K + b : b * a.m + e;
            out[col] = acc[e];
        }
    }
    if (b == 0) out[(int64_t)a.m * a.K] = I;
}

// g[slots[q]][c] = sum over ranges of part[range][q][c] (fixed order); padding columns 0
__global__ void __launch_bounds__(256) lag_reduce_kernel(const double* __restrict__ part,
                                                         int64_t nranges, int32_t nact,
                                                         int32_t P, int32_t ncols,
                                                         const int32_t* __restrict__ slots,
                                                         double* __restrict__ g) {
    const int64_t len = (int64_t)nact * P;
    for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < len;
         e += (int64_t)gridDim.x * 256) {
        const int64_t q = e / P, c = e - q * P;
        double v = 0.0;
        if (c < ncols)
            for (int64_t r = 0; r < nranges; ++r) v += part[(r * nact) * (int64_t)P + e];
        g[(int64_t)slots[q] * P + c] = v;
    }
}

struct LagPlan {
    int FG, groups, tiles_per;
    int64_t ntiles, nranges;
};

LagPlan lag_plan(int32_t K, int32_t nact, int64_t n) {
    LagPlan p;
    p.FG = kLagT / K;
    if (p.FG > kLagFG) p.FG = kLagFG;              // LDS: FG x kLagU floats
    p.groups = (nact + p.FG - 1) / p.FG;
    p.ntiles = (n + kLagU - 1) / kLagU;
    // ~3 workgroups per CU over the fit groups x row ranges
    int64_t nr = (768 + p.groups - 1) / p.groups;
    if (nr > p.ntiles) nr = p.ntiles;
    if (nr < 1) nr = 1;
    p.tiles_per = (int)((p.ntiles + nr - 1) / nr);
    p.nranges = (p.ntiles + p.tiles_per - 1) / p.tiles_per;
    return p;
}

}  // namespace
}  // namespace sglm

using namespace sglm;

extern "C" int32_t sglm_lag_tile_rows(void) { return kLagU; }

extern "C" size_t sglm_lag_xtr_work_bytes(int32_t P, int32_t K, int32_t B, int64_t n) {
    if (K <= 0 || K > kLagT) return 0;
    size_t mx = 0;
    for (int32_t b = 1; b <= B; ++b) {
        const LagPlan p = lag_plan(K, b, n);
        const size_t w = (size_t)p.nranges * b * P * sizeof(double);
        if (w > mx) mx = w;
    }
    return mx;
}

extern "C" int sglm_lag_xtr(const int32_t* occ, const int32_t* tbeg, const int32_t* tend,
                            const int32_t* shifts, int32_t m, int32_t K, int32_t layout,
                            int64_t row0, int64_t n, int32_t P, const float* R, int64_t ld,
                            const int32_t* slots, int32_t nact, double* g, void* work,
                            sglm_stream_t stream) {
    if (nact <= 0) return SGLM_OK;
    if (!occ || !tbeg || !tend || !shifts || !R || !slots || !g || !work || m < 1 ||
        m > kLagMaxM || K < 1 || K > kLagT || (int64_t)m * K + 1 > P || n > ld || n <= 0) {
        set_error("sglm_lag_xtr: bad args (m=%d <= %d, K=%d, P=%d)", m, kLagMaxM, K, P);
        return SGLM_EINVAL;
    }
    const LagPlan pl = lag_plan(K, nact, n);
    LagArgs a;
    a.occ = occ; a.tbeg = tbeg; a.tend = tend; a.shifts = shifts;
    a.m = m; a.K = K; a.layout = layout; a.P = P; a.row0 = row0; a.n = n; a.ntiles = pl.ntiles;
    hipStream_t s = as_stream(stream);
    const size_t lds = sizeof(LagLds);
    double* part = (double*)work;
    dim3 grid((unsigned)pl.nranges, (unsigned)pl.groups);
    static bool attr = false;                      // > 64 KB of dynamic LDS (gfx950: 160 KB)
    if (!attr) {
        if (hipFuncSetAttribute(reinterpret_cast<const void*>(&lag_xtr_kernel<16>),
                                hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)sizeof(LagLds)) != hipSuccess ||
            hipFuncSetAttribute(reinterpret_cast<const void*>(&lag_xtr_kernel<kLagMaxM>),
                                hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)sizeof(LagLds)) != hipSuccess) {
            set_error("lag_xtr_kernel: %d bytes of LDS refused", (int)sizeof(LagLds));
            return SGLM_EHIP;
        }
        attr = true;
    }
    if (m <= 16)
        lag_xtr_kernel<16><<<grid, kLagT, lds, s>>>(a, R, ld, slots, nact, pl.FG, pl.tiles_per,
                                                    part);
    else
        lag_xtr_kernel<kLagMaxM><<<grid, kLagT, lds, s>>>(a, R, ld, slots, nact, pl.FG,
                                                          pl.tiles_per, part);
    int st = check_launch("lag_xtr_kernel");
    if (st) return st;
    const int64_t len = (int64_t)nact * P;
    lag_reduce_kernel<<<(unsigned)((len + 255) / 256 < 4096 ? (len + 255) / 256 : 4096), 256, 0,
                        s>>>(part, pl.nranges, nact, P, m * K + 1, slots, g);
    return check_launch("lag_reduce_kernel");
}
