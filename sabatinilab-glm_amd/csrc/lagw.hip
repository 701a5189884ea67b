// Weighted Gram of a time-shifted 0/1 event design from its events (sglm_lag_gram_w).
//
// The design's column (b, a) is event a shifted by s_b: X[t][(b, a)] = e_a(t + row0 - s_b), plus
// the ones column p.  For one fit with row weights w (the IRLS weights, mask multiplicities
// folded in) the Gram entry of columns (b1, a1), (b2, a2) is, with v = t + row0 - s_b1 an
// occurrence of a1 and d = s_b1 - s_b2,
//     H[(b1,a1)][(b2,a2)] = sum over v in occ(a1) of e_a2(v + d) * w(v - row0 + s_b1)
// -- for each event a1 ONE matrix product over a1's occurrences:
//     G_a1[(d, a2)][(s, f)] = sum_v A[v][(d, a2)] B[v][(s, f)],
//     A[v][(d, a2)] = e_a2(v + d)            (bit a2 of the row word R[v + d])
//     B[v][(s, f)] = bf16(w_f(v - row0 + s))
// and every G entry whose second shift s - d is a column is one H entry.  The dense Gram sums n
// rows of p^2 products; this sums nnz(E) occurrences of about (m + 1) L^2 products per fit,
// rho of the dense work at event density rho (C4: 0.02).  The products are the dense kernel's
// (bf16 w times exact 0/1, f32 accumulation), in another order.
//
// Layout: R[u] (u64 per raw row u): bit a = e_a(u), bit m = 1 (the ones column: d = 0).
// Rows: every a2 but only d >= 0 -- the entry of d < 0 is the transpose of event a2's entry at
// -d > 0 (and at d = 0, a2 < a1 is left to a2's piece): each H entry formed once.
// Workgroup ("piece"): one event a1, a group of d rows (both 32-event halves) and a block of
// (shift, fit) columns, over ALL of a1's occurrences (no split: every H entry is written once, by
// one lane, no reduction).  8 waves (two per SIMD), each 2 M tiles x 4 N tiles of
// v_mfma_f32_32x32x16_bf16.  Per stage of 128 occurrences:
// * weights: 16 lanes stage one occurrence's columns (a contiguous run of the (row, fit) weights,
//   one aligned copy of the 8) with 16-byte loads and ds_write_b128 into an [occurrence][column]
//   image whose 16-byte chunks are XOR-swizzled by row; the B operand comes back with two
//   ds_read_b64_tr_b16 (the hardware transpose), conflict-free on that image;
// * row words: lanes over the d rows of one occurrence pair (consecutive words), stored
//   pair-interleaved (the two words' low / high halves in one dword: the A fragment is one
//   rotate and one mask per dword), rows padded so that stores and b128 reads are conflict-free;
// * the staging of stage s + 1 (stores) and s + 2 (loads) rides inside the K-steps of stage s,
//   every load unconditional (clamped addresses, validity applied at the store) so the
//   compiler's wait counts stay exact;
// * each wave's live N tiles (those whose columns meet one of its d rows with a second shift
//   that is a column) are a range fixed for the launch: the stage loop is instantiated per range,
//   so the MFMA stream has no branch;
// * pieces run longest first (the last round of workgroups holds the lightest);
// * result: every H entry is written at the row of the column (s_b1, a1) that formed it
//   (H[(b1, a1)][(b2, a2)]: a2 contiguous in a shift-major design) and lag_gram_w_sym builds the
//   upper triangle from whichever of (i, j) / (j, i) holds an entry (round 5's kernel wrote every
//   d > 0 entry down a column of the upper triangle: 4-byte scatter, 9x write amplification).
#include <algorithm>
#include <cstring>
#include <functional>
#include <map>
#include <mutex>
#include <queue>
#include <type_traits>
#include <vector>

#include "common.h"

namespace sglm {
namespace {

__device__ __forceinline__ int lag_col2(int layout, int m, int K, int b, int ev) {
    return layout ? ev * K + b : b * m + ev;
}

// H_f[p][p] = sum_t bf16(w_f(t)): kLwRed partial sums per fit (fixed row chunks, fixed tree
// order), then summed in order by lag_gram_w_aux; the padding columns / rows of the upper
// triangle zeroed there (the dense kernel's zero bits)
constexpr int kLwRed = 128;

__global__ void __launch_bounds__(256) lag_gram_w_part(const float* __restrict__ W, int64_t ld,
                                                       int32_t n, const int32_t* __restrict__ fits,
                                                       float* __restrict__ part) {
    const float* w = W + (int64_t)fits[blockIdx.y] * ld;
    const int64_t chunk = ((int64_t)n + kLwRed - 1) / kLwRed;
    const int64_t t0 = (int64_t)blockIdx.x * chunk, t1 = min((int64_t)n, t0 + chunk);
    float s = 0.0f;
    for (int64_t t = t0 + threadIdx.x; t < t1; t += 256) s += (float)(__bf16)w[t];
    __shared__ float red[256];
    red[threadIdx.x] = s;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
        __syncthreads();
    }
    if (threadIdx.x == 0) part[blockIdx.y * kLwRed + blockIdx.x] = red[0];
}

__global__ void __launch_bounds__(256) lag_gram_w_aux(const float* __restrict__ part,
                                                      const int32_t* __restrict__ fits,
                                                      float* __restrict__ H, int32_t P,
                                                      int32_t p) {
    float* Hf = H + (int64_t)fits[blockIdx.y] * P * P;
    if (blockIdx.x == 0) {
        if (threadIdx.x == 0) {
            float t = 0.0f;
            for (int b = 0; b < kLwRed; ++b) t += part[blockIdx.y * kLwRed + b];
            Hf[(int64_t)p * P + p] = t;
        }
        return;
    }
    const int w = P - p - 1;                             // padding columns p + 1 .. P - 1
    const int64_t tot = (int64_t)P * w;
    for (int64_t e = (int64_t)(blockIdx.x - 1) * 256 + threadIdx.x; e < tot;
         e += (int64_t)(gridDim.x - 1) * 256) {
        const int64_t i = e / w, j = p + 1 + e % w;
        if (i <= j) Hf[i * P + j] = 0.0f;
    }
}

// Wt copy c, element j = bf16(W[fits[f]][u - row0 + smin]) at i = j + c = u nf + f: the weights of
// raw rows u - smin .. in (row, fit) order, shifted by c; 0 off the design's rows and for raw rows
// u >= zrow (the padding columns of the last column block read there)
__global__ void __launch_bounds__(256) lag_gram_w_prep(const float* __restrict__ W, int64_t ld,
                                                       int32_t n, const int32_t* __restrict__ fits,
                                                       int32_t nf, int32_t row0, int32_t smin,
                                                       int64_t wlen, int64_t zrow,
                                                       uint16_t* __restrict__ Wt) {
    const int c = blockIdx.y;
    for (int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x; j < wlen;
         j += (int64_t)gridDim.x * 256) {
        const int64_t i = j + c;
        const int64_t u = i / nf;
        const int f = (int)(i % nf);
        const int64_t t = u - row0 + smin;
        const float x = (t >= 0 && t < n && u < zrow) ? W[(int64_t)fits[f] * ld + t] : 0.0f;
        Wt[c * wlen + j] = __builtin_bit_cast(uint16_t, (__bf16)x);
    }
}

constexpr int kKS2 = 128;                 // occurrences per stage
constexpr int kKP2 = kKS2 / 2;            // occurrence pairs per stage
constexpr int kRX2 = kKP2 + 4;            // dwords per (half, X / Y) row of a d row's words
constexpr int kRS2 = 4 * kRX2 + 4;        // dwords per d row of the staged row words
constexpr int kSentR = -(1 << 28);        // row index of a past-the-end occurrence: its R reads
                                          // (x 8 bytes, unsigned) fall past the buffer -> zeros
constexpr uint32_t kSentW = 0xfffff000u;  // weight byte offset of a past-the-end occurrence

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

struct LagW2Args {
    const uint16_t* Wt;             // 8 shifted copies of the bf16 weights by (raw row, fit)
    int64_t wlen;                   // elements per copy (a multiple of 8)
    const uint64_t* R;
    const int32_t* occ;
    const int32_t* ev_off;
    const int32_t* bidx;            // [K]: b of shift smin + i
    const int32_t* fits;
    float* H;
    float* Hb;                      // [nf][P][P]: the second halves of split pieces
    int32_t nf, P, p, m, K, smin, smax, layout, nraw, D, Gm, Gy;
    // job list (longest first): block b runs job jobs[b / m] on event b % m.  A job is a piece
    // type t = g + Gm y (bits 0-13) and the stages it covers (bits 14-15: 0 all, 1 the first
    // half -> H, 2 the second half -> Hb; lag_gram_w_sym adds the two, first + second, so the
    // result is deterministic).  njobs == 0: block b runs piece type b / m whole.
    int32_t njobs;
    int32_t ms;                     // blocks per job (= m)
    int32_t wsh;                    // 1: a piece's column window starts at its first d row
    uint16_t jobs[256];
#ifdef SGLM_LAGW_TRACE
    uint64_t* trace;                // probe build: per block start / end clock, hardware slot, job
#endif
};

template <int NCH>
__device__ __forceinline__ int lagw_swz(int row) {       // chunk XOR of the weight image's row
    return NCH == 16 ? ((row & 3) << 2) : (((row >> 1) & 1) << 2);
}

template <int MT, int NT, int WM, int WN, int NH>
struct LagW2Smem {
    static constexpr int MB = WM * MT, NN = WN * NT * 32, ND = MB / NH;
    uint32_t rw[2][ND * kRS2];                                  // [buf][d row][pl][xy][pair]
    __attribute__((aligned(16))) uint16_t ws[2][kKS2 * NN];     // [buf][occurrence][column]
    int32_t vo[4][kKS2];            // per occurrence of a stage: its raw row (kSentR past the end)
    uint32_t wo[4][kKS2];           // the byte offset of its weight columns (kSentW past the end)
};

// Staging of one stage (128 occurrences) per workgroup: every load is an unconditional
// buffer load whose range check supplies the zeros (raw rows past the end, occurrences past the
// event's end), so no address is selected and the compiler's wait counts stay exact; the
// per-occurrence address arithmetic is done once, by the thread that loads the occurrence.
template <int MT, int NT, int WM, int WN, int NH>
__global__ void __launch_bounds__(64 * WM * WN) __attribute__((amdgpu_waves_per_eu(2, 2)))
lag_gram_w2_kernel(LagW2Args a) {
    using SM = LagW2Smem<MT, NT, WM, WN, NH>;
    constexpr int NTH = 64 * WM * WN, MB = SM::MB, NN = SM::NN, ND = SM::ND, NCH = NN / 8;
    static_assert(MB % NH == 0, "d rows per piece");
    static_assert((kKS2 * NCH) % NTH == 0, "weight tasks per thread");
    constexpr int kWT = kKS2 * NCH / NTH;
    static_assert((kKP2 * ND) % NTH == 0, "row-word tasks per thread");
    constexpr int kRT = kKP2 * ND / NTH;
    static_assert(kWT <= 4, "staging pieces per K-step");
    __shared__ SM sm;
#ifdef SGLM_LAGW_TRACE
    const uint64_t t_beg = __builtin_amdgcn_s_memrealtime();
#endif
    const int blk = blockIdx.x;
    const int a1 = blk % a.ms;
    if (a1 >= a.m) return;
    int type, half = 0;
    if (a.njobs > 0) {
        if (blk >= a.njobs * a.ms) return;
        const int jb = a.jobs[blk / a.ms];
        type = jb & 0x3fff;
        half = jb >> 14;
    } else {
        type = blk / a.ms;
        if (type >= a.Gm * a.Gy) return;
    }
    const int g = type % a.Gm, y = type / a.Gm;
    const int Tm = a.D * NH;
    const int t0 = g * MB;
    if (t0 >= Tm) return;
    const int di0 = t0 / NH;
    // the piece's column window starts at its first d row's first live column (shift smin + di0,
    // fit 0): the columns below hold no H entry for any of its rows (round 6: 1-fit launches
    // issue a third fewer MFMAs, 5-fit ones 8 %)
    const int n0 = y * NN + a.wsh * di0 * a.nf;
    // a G entry of row d and a column of shift smin + sb is an H entry only when sb >= d (its
    // second shift smin + sb - d is then a column): a piece whose columns all precede its d rows
    // has nothing to store
    if (n0 / a.nf >= a.K || min(a.K - 1, (n0 + NN - 1) / a.nf) < di0) return;
    int o_beg = a.ev_off[a1], o_end = a.ev_off[a1 + 1];
    if (half) {
        const int hs = ((o_end - o_beg + kKS2 - 1) / kKS2 + 1) / 2;   // stages of the first half
        if (half == 1) o_end = min(o_end, o_beg + hs * kKS2);
        else o_beg += hs * kKS2;
    }
    const int nst = max(0, (o_end - o_beg + kKS2 - 1) / kKS2);
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h = lane >> 5, r = lane & 31;
    const int wm = wave % WM, wn = wave / WM;

    const __amdgpu_buffer_rsrc_t rsR =
        __builtin_amdgcn_make_buffer_rsrc((void*)a.R, 0, a.nraw * 8, 0x00020000);
    const __amdgpu_buffer_rsrc_t rsW =
        __builtin_amdgcn_make_buffer_rsrc((void*)a.Wt, 0, (int)(uint32_t)(a.wlen * 16), 0x00020000);
    const __amdgpu_buffer_rsrc_t rsO =
        __builtin_amdgcn_make_buffer_rsrc((void*)a.occ, 0, a.ev_off[a.m] * 4, 0x00020000);

    // the fixed tasks of this thread: weight chunks i (occurrence k, 16-byte chunk ch: its LDS
    // slot), row-word tasks i (pair kp, d row dl: its LDS slot and row offset)
    int wk[kWT], wsl[kWT];
#pragma unroll
    for (int i = 0; i < kWT; ++i) {
        const int t = tid + NTH * i;
        wk[i] = t / NCH;
        const int ch = t % NCH;
        wsl[i] = wk[i] * NN + 8 * (ch ^ lagw_swz<NCH>(wk[i]));
        wk[i] = wk[i] | (ch << 16);
    }
    int rkp[kRT], rdl[kRT];
#pragma unroll
    for (int i = 0; i < kRT; ++i) {
        const int t = tid + NTH * i;
        rkp[i] = t / ND;
        rdl[i] = t % ND;
    }

    // one register set: a stage is stored to LDS during the next stage's first K-steps, then
    // the registers receive the stage after next (clang vectors: arrays of HIP's uint4 struct
    // stay allocas)
    u32x4 wA[kWT];
    u32x2 rA[kRT][2];
    int32_t oreg = 0;
    bool ovalid = false;

    auto occ_load = [&](int s) __attribute__((always_inline)) {
        const int o = o_beg + s * kKS2 + (tid & (kKS2 - 1));
        ovalid = o < o_end;
        oreg = __builtin_amdgcn_raw_buffer_load_b32(rsO, o * 4, 0, 0);
    };
    auto occ_store = [&](int s) __attribute__((always_inline)) {
        if (tid < kKS2) {                                        // wave-uniform
            const int v = ovalid ? oreg : kSentR;
            const int64_t x = (int64_t)(ovalid ? oreg : 0) * a.nf + n0;
            const int c = (int)(x & 7);
            sm.vo[s & 3][tid] = v;
            sm.wo[s & 3][tid] = ovalid ? (uint32_t)(2 * (c * a.wlen + x - c)) : kSentW;
        }
    };
    auto load_w = [&](int s, int i) __attribute__((always_inline)) {
        const uint32_t off = sm.wo[s & 3][wk[i] & 0xffff];
        wA[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                              rsW, off + 16 * (wk[i] >> 16), 0, 0));
    };
    auto load_r = [&](int s) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < kRT; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int u = sm.vo[s & 3][2 * rkp[i] + j] + di0 + rdl[i];
                rA[i][j] = __builtin_bit_cast(
                    u32x2, __builtin_amdgcn_raw_buffer_load_b64(rsR, (uint32_t)u << 3, 0, 0));
            }
    };
    auto store_w = [&](int buf, int i) __attribute__((always_inline)) {
        *reinterpret_cast<u32x4*>(&sm.ws[buf][wsl[i]]) = wA[i];
    };
    auto store_r = [&](int buf) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < kRT; ++i) {
            uint32_t* dst = &sm.rw[buf][rdl[i] * kRS2 + rkp[i]];
#pragma unroll
            for (int pl = 0; pl < NH; ++pl) {
                const uint32_t w0 = rA[i][0][pl], w1 = rA[i][1][pl];
                dst[(2 * pl) * kRX2] = __builtin_amdgcn_perm(w1, w0, 0x05040100u);
                dst[(2 * pl + 1) * kRX2] = __builtin_amdgcn_perm(w1, w0, 0x07060302u);
            }
        }
    };
    auto data_load = [&](int s) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < kWT; ++i) load_w(s, i);
        load_r(s);
    };
    auto data_store = [&](int buf) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < kWT; ++i) store_w(buf, i);
        store_r(buf);
    };

    f32x16 acc[MT][NT];
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j) acc[i][j] = (f32x16){};

    // A: tile i = (d row, event half) -> its staged words.  Live N tiles: tile j's columns meet a
    // d of this wave's tiles with a second shift that is a column (sb_hi(j) >= d) and are not
    // all padding (sb_lo(j) < K) -- a range [j0, j1] of the wave's tiles, wave-uniform and fixed
    // for the whole launch: the stage loop is instantiated per range (below), so the MFMA stream
    // has no branch and the fragment reads can be scheduled ahead of it
    int aoff[MT];
    int dmin_w = 1 << 30;
#pragma unroll
    for (int i = 0; i < MT; ++i) {
        const int tau = min(t0 + wm * MT + i, Tm - 1);
        const int dl = tau / NH - di0, hf = tau % NH;
        aoff[i] = dl * kRS2 + (2 * hf + (r >> 4)) * kRX2 + 4 * h;
        if (t0 + wm * MT + i < Tm) dmin_w = min(dmin_w, di0 + dl);
    }
    int j0 = NT, j1 = -1;
#pragma unroll
    for (int j = 0; j < NT; ++j) {
        const int c0 = n0 + (wn * NT + j) * 32;
        const int sb_lo = c0 / a.nf, sb_hi = min(a.K - 1, (c0 + 31) / a.nf);
        if (sb_lo < a.K && sb_hi >= dmin_w) {
            j0 = min(j0, j);
            j1 = max(j1, j);
        }
    }
    const int jcode = __builtin_amdgcn_readfirstlane(j0 > j1 ? -1 : j0 * NT + j1);
    // B: lane 4q + pp of 16-lane group g4 supplies row 8 (g4 >> 1) + q (+ 4), columns
    // 16 (g4 & 1) + 4 pp .. + 3 of N tile j; it receives column r of rows 8 h .. 8 h + 7
    int boff[NT];
    {
        const int g4 = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
        const int row = 8 * (g4 >> 1) + q;
#pragma unroll
        for (int j = 0; j < NT; ++j) {
            const int col = (wn * NT + j) * 32 + 16 * (g4 & 1) + 4 * pp;
            boff[j] = row * NN * 2 + 16 * ((col >> 3) ^ lagw_swz<NCH>(row)) + 8 * (pp & 1);
        }
    }
    const uint32_t rsh = (uint32_t)(r - 14 - 16 * (r >> 4)) & 31u;   // bit r (mod 16) -> 14

    // the multiplication of stage s (buffer s & 1) over the live N tiles J0 .. J1, with the
    // staging of the next stages inside its K-steps: stage s + 1 is stored to the other buffer
    // over the first K-steps (one piece behind each K-step's MFMAs) and stage s + 2 is loaded
    // into the freed registers over the last ones, so the LDS writes and the address work of the
    // staging overlap the MFMAs instead of following the barrier in lockstep on both waves of a
    // SIMD
    auto compute = [&](int s, auto J0c, auto J1c) __attribute__((always_inline)) {
        constexpr int J0 = decltype(J0c)::value, J1 = decltype(J1c)::value;
        const int buf = s & 1;
        const uint32_t* rwb = &sm.rw[buf][0];
        const char* wsb = reinterpret_cast<const char*>(&sm.ws[buf][0]);
        // the fragments of K-step ks: A as the staged row words (expanded below), B as read
        auto fetch = [&](int ks, u32x4 (&wq)[MT], s16x4 (&t1)[NT], s16x4 (&t2)[NT])
                         __attribute__((always_inline)) {
#pragma unroll
            for (int j = J0; j <= J1; ++j) {
                const char* pb = wsb + boff[j] + ks * 16 * NN * 2;
                t1[j] = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                    (lds_s16x4*)(__attribute__((address_space(3))) char*)pb);
                t2[j] = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                    (lds_s16x4*)(__attribute__((address_space(3))) char*)(pb + 4 * NN * 2));
            }
#pragma unroll
            for (int i = 0; i < MT; ++i)
                wq[i] = *reinterpret_cast<const u32x4*>(rwb + aoff[i] + 8 * ks);
        };
        auto mult = [&](const u32x4 (&wq)[MT], const s16x4 (&t1)[NT], const s16x4 (&t2)[NT])
                        __attribute__((always_inline)) {
            bf16x8 bq[NT];
#pragma unroll
            for (int j = J0; j <= J1; ++j) {
                const uint2 u1 = __builtin_bit_cast(uint2, t1[j]);
                const uint2 u2 = __builtin_bit_cast(uint2, t2[j]);
                bq[j] = __builtin_bit_cast(bf16x8, make_uint4(u1.x, u1.y, u2.x, u2.y));
            }
            bf16x8 aq[MT];
#pragma unroll
            for (int i = 0; i < MT; ++i) {
                uint32_t dq[4];
#pragma unroll
                for (int q = 0; q < 4; ++q) dq[q] = rotr32(wq[i][q], rsh) & 0x40004000u;
                aq[i] = __builtin_bit_cast(bf16x8, make_uint4(dq[0], dq[1], dq[2], dq[3]));
            }
#pragma unroll
            for (int i = 0; i < MT; ++i)
#pragma unroll
                for (int j = J0; j <= J1; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(aq[i], bq[j], acc[i][j],
                                                                        0, 0, 0);
        };
        auto staging = [&](int ks) __attribute__((always_inline)) {
            if (ks < kWT) store_w(buf ^ 1, ks);
            if (ks == kWT) store_r(buf ^ 1);
            if (ks == 4) occ_load(s + 4);
            if (ks >= 4 && ks - 4 < kWT) load_w(s + 2, ks - 4);
            if (ks == 7) load_r(s + 2);
        };
        // the fragments of K-step ks + 1 are read while the MFMAs of ks run (hipcc sinks the
        // reads to their MFMAs unless the scheduling barriers hold them ahead).  (Three buffers
        // with the barrier after the stores and the next stage's first fragments read during
        // K-step 7 -- no stage starting on an LDS round trip -- spilled 150+ VGPRs; not kept.)
        u32x4 wq[2][MT];
        s16x4 t1[2][NT], t2[2][NT];
        fetch(0, wq[0], t1[0], t2[0]);
#pragma unroll
        for (int ks = 0; ks < kKS2 / 16; ++ks) {
            staging(ks);
            if (ks + 1 < kKS2 / 16)
                fetch(ks + 1, wq[(ks + 1) & 1], t1[(ks + 1) & 1], t2[(ks + 1) & 1]);
            __builtin_amdgcn_sched_barrier(0);
            mult(wq[ks & 1], t1[ks & 1], t2[ks & 1]);
            __builtin_amdgcn_sched_barrier(0);
        }
    };
    // stage s: the occurrences of stage s + 3 are stored, stage s is multiplied (stage s + 1 is
    // stored, the occurrences of stage s + 4 and the data of stage s + 2 are loaded inside)
    auto main_loop = [&](auto J0c, auto J1c) __attribute__((always_inline)) {
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            occ_load(j);
            occ_store(j);
        }
        __syncthreads();
        data_load(0);
        data_store(0);
        occ_load(3);
        data_load(1);
        for (int s = 0; s < nst; ++s) {
            occ_store(s + 3);
            __syncthreads();
            compute(s, J0c, J1c);
        }
    };
    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;
    using I2 = std::integral_constant<int, 2>;
    using I3 = std::integral_constant<int, 3>;
    using IN = std::integral_constant<int, -1>;
    if (nst > 0) {
        // an event that never occurs leaves acc = 0 (its H entries are written as zeros)
        if constexpr (NT == 4) {
            switch (jcode) {
                case 0: main_loop(I0{}, I0{}); break;
                case 1: main_loop(I0{}, I1{}); break;
                case 2: main_loop(I0{}, I2{}); break;
                case 3: main_loop(I0{}, I3{}); break;
                case 5: main_loop(I1{}, I1{}); break;
                case 6: main_loop(I1{}, I2{}); break;
                case 7: main_loop(I1{}, I3{}); break;
                case 10: main_loop(I2{}, I2{}); break;
                case 11: main_loop(I2{}, I3{}); break;
                case 15: main_loop(I3{}, I3{}); break;
                default: main_loop(I0{}, IN{}); break;      // no live tile: staging only
            }
        } else {
            static_assert(NT == 2, "N tiles per wave");
            switch (jcode) {
                case 0: main_loop(I0{}, I0{}); break;
                case 1: main_loop(I0{}, I1{}); break;
                case 3: main_loop(I1{}, I1{}); break;
                default: main_loop(I0{}, IN{}); break;
            }
        }
    }

    // epilogue: G entry (d, a2) x (f, b1) -> H_f[(b1, a1)][(b2, a2)] at the row of (b1, a1)
#pragma unroll
    for (int j = 0; j < NT; ++j) {
        const int nn = n0 + (wn * NT + j) * 32 + r;
        const int sb = nn / a.nf, f = nn % a.nf;           // column: shift smin + sb, fit f
        if (sb >= a.K) continue;
        const int b1 = a.bidx[sb];
        if (b1 < 0) continue;
        float* Hrow = (half == 2 ? a.Hb + (int64_t)f * a.P * a.P
                                 : a.H + (int64_t)a.fits[f] * a.P * a.P) +
                      (int64_t)lag_col2(a.layout, a.m, a.K, b1, a1) * a.P;
#pragma unroll
        for (int i = 0; i < MT; ++i) {
            const int tau = t0 + wm * MT + i;
            if (tau >= Tm) continue;
            const int dd = tau / NH;
            const int hf = tau % NH;
            if (sb < dd) continue;                           // second shift below smin
            const int b2 = a.bidx[sb - dd];
            if (b2 < 0) continue;
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                const int a2 = 32 * hf + (q & 3) + 8 * (q >> 2) + 4 * h;
                const float val = 0.5f * acc[i][j][q];
                if (a2 < a.m) {
                    if (dd == 0 && a2 < a1) continue;        // formed by event a2's piece
                    Hrow[lag_col2(a.layout, a.m, a.K, b2, a2)] = val;
                } else if (a2 == a.m && dd == 0) {
                    Hrow[a.p] = val;
                }
            }
        }
    }
#ifdef SGLM_LAGW_TRACE
    __syncthreads();
    if (tid == 0) {
        const uint64_t t_end = __builtin_amdgcn_s_memrealtime();
        const uint32_t hw = __builtin_amdgcn_s_getreg(4 | (31 << 11));    // HW_ID
        const uint32_t xcc = __builtin_amdgcn_s_getreg(20 | (31 << 11));  // XCC_ID
        a.trace[4 * blk + 0] = t_beg;
        a.trace[4 * blk + 1] = t_end;
        a.trace[4 * blk + 2] = (uint64_t)hw | ((uint64_t)xcc << 32);
        a.trace[4 * blk + 3] = (uint64_t)type | ((uint64_t)a1 << 16) | ((uint64_t)nst << 32);
    }
#endif
}

// The pieces a launch split in two (their second halves in Hb): the piece type of an entry is
// found from its holder row's column (b1, a1) and its column (b2, a2) -- d = s1 - s2, the event
// half of a2, the (shift, fit) column of (s1, f).
struct LagwSplit {
    const float* Hb;                // null: nothing split
    int32_t smin, nh, MB, NN, Gm, nf, wsh;
    uint32_t mask[8];               // bit t: piece type t split
};

// Upper triangle of H_f from the entries lag_gram_w2_kernel wrote: entry {i, j} (i < j) sits at
// row i when column i has the larger shift, or the same shift and the smaller event (the ones
// column p: at row i); continuous columns of a mixed design and the padding columns are zeroed
// (the continuous rows / columns are written after this by _mix_hess).  One 256-thread workgroup
// per 64 x 64 upper tile (I, J) of one fit: the transposed tile (J, I) staged through LDS.  A
// split piece's entries are its first half (H) + its second half (Hb), in that order.
__global__ void __launch_bounds__(256) lag_gram_w_sym(float* __restrict__ H,
                                                      const int32_t* __restrict__ fits, int32_t P,
                                                      int32_t p, int32_t m, int32_t K,
                                                      int32_t layout,
                                                      const int32_t* __restrict__ shifts,
                                                      LagwSplit sp) {
    __shared__ float tl[64][65], tb[64][65];     // H and Hb rows J*64.., columns I*64..
    __shared__ int ks_i[64], ks_j[64];           // (shift, event) keys of the tile's columns
    const int T = P / 64;
    int I = 0, rem = blockIdx.x;
    while (rem >= T - I) { rem -= T - I; ++I; }  // tile (I, J), I <= J, row-major over the upper
    const int J = I + rem;
    float* Hf = H + (int64_t)fits[blockIdx.y] * P * P;
    const float* Hbf = sp.Hb ? sp.Hb + (int64_t)blockIdx.y * P * P : nullptr;
    const int tid = threadIdx.x;
    const int plag = m * K;
    if (tid < 128) {
        const int c = (tid < 64 ? I : J) * 64 + (tid & 63);
        int key = -1;                            // -1: no lag column
        if (c < plag) {
            const int b = layout ? c % K : c / m, e = layout ? c / K : c % m;
            key = (shifts[b] + 65536) * 64 + (63 - e);    // larger key = the row that holds it
        }
        (tid < 64 ? ks_i : ks_j)[tid & 63] = key;
    }
    // split piece of the entry held at row (key kr) and column (key kc; event a2 = m: ones)
    auto split = [&](int kr, int kc, int a2) -> bool {
        if (!Hbf) return false;
        const int s1 = kr / 64 - 65536, s2 = kc / 64 - 65536;
        const int tau = (s1 - s2) * sp.nh + a2 / 32;
        const int g = tau / sp.MB;                       // its piece: d group, column block
        const int y = ((s1 - sp.smin - sp.wsh * (g * sp.MB / sp.nh)) * sp.nf + (int)blockIdx.y) /
                      sp.NN;
        const int t = g + sp.Gm * y;
        return (sp.mask[t >> 5] >> (t & 31)) & 1u;
    };
    // stage H rows J*64.., columns I*64.. (the lower counterpart), and Hb's when split
    for (int e = tid; e < 64 * 64; e += 256) {
        const int rr = e >> 6, cc = e & 63;
        tl[rr][cc] = Hf[(int64_t)(J * 64 + rr) * P + I * 64 + cc];
        if (Hbf) tb[rr][cc] = Hbf[(int64_t)(J * 64 + rr) * P + I * 64 + cc];
    }
    __syncthreads();
    for (int e = tid; e < 64 * 64; e += 256) {
        const int il = e >> 6, jl = e & 63;
        const int i = I * 64 + il, j = J * 64 + jl;
        if (i > j) continue;
        float* dst = Hf + (int64_t)i * P + j;
        if (j > p) {                             // padding (and its diagonal)
            *dst = 0.0f;
            continue;
        }
        const int ki = ks_i[il], kj = ks_j[jl];
        if (i == j) {                            // diagonal: in place (H[p][p] by aux)
            if (ki >= 0 && split(ki, ki, 63 - ki % 64)) *dst += Hbf[(int64_t)i * P + j];
            continue;
        }
        if (j == p) {
            if (i >= plag) *dst = 0.0f;          // a continuous column's ones entry
            else if (split(ki, ki, m)) *dst += Hbf[(int64_t)i * P + j];   // a lag column's: row i
            continue;
        }
        if (ki < 0 || kj < 0) *dst = 0.0f;       // a continuous column
        else if (kj > ki)                        // held at row j
            *dst = split(kj, ki, 63 - ki % 64) ? tl[jl][il] + tb[jl][il] : tl[jl][il];
        else if (split(ki, kj, 63 - kj % 64))    // held at row i
            *dst += Hbf[(int64_t)i * P + j];
    }
}

// The launch's job list.  Piece order: longest first (measured 0.634 -> 0.600 ms per C4
// launch against XCD-local ranges: the last round of workgroups holds the lightest pieces).  Work
// of a piece type per stage, in units of one live MFMA per K-step: the live MFMAs of the busier
// SIMD (waves w and w + 4 share one) + 7 for the staging every piece does (fitted to per-piece
// timelines of the C4 launches, tools/lagw_trace.py).  With one workgroup per CU and ~2 pieces per
// CU, LPT still left the CUs 20 % idle over a 5-fit launch (the heaviest pieces + a light one set
// the end), so the heaviest types may run as two half-occurrence jobs: the split set is chosen
// by simulating the greedy dispatch (each free CU takes the next job) over the CU count, a half
// priced at half its piece + 2 % of the heaviest.  (Adding the halves into zeroed H entries with
// float atomics cost more than the tail: 0.881 -> 1.085 ms per 5-fit call; the second halves
// now go to a scratch image that the symmetrize pass adds.)  Cached per launch shape.
struct LagwPlan {
    int njobs = 0;                                     // -1: no live piece
    bool split = false;
    uint16_t jobs[256];
    uint32_t mask[8] = {0, 0, 0, 0, 0, 0, 0, 0};
};

static int lagw_cus() {
    static const int n = [] {
        int dev = 0, v = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
            v <= 0)
            v = 256;
        return v;
    }();
    return n;
}

static LagwPlan lagw_plan(int m, int K, int nf, int NH, int MT, int NT, int WM, int Gm, int Gy,
                          bool can_split, int wsh) {
    static std::mutex mu;
    static std::map<std::vector<int>, LagwPlan> cache;
    const char* e = getenv("SGLM_LAGW_SPLIT");          // read per launch (A/B, tests)
    const bool sp_ok = can_split && !(e && e[0] == '0');
    const std::vector<int> key{m, K, nf, NH, MT, NT, WM, Gm, Gy, sp_ok, wsh};
    std::lock_guard<std::mutex> lk(mu);
    auto it = cache.find(key);
    if (it != cache.end()) return it->second;
    LagwPlan pl;
    const int per = Gm * Gy, MB = WM * MT, NN = NT * 32, Tm = K * NH;
    if (per > 128) return cache[key] = pl;              // natural order (njobs = 0)
    std::vector<std::pair<double, int>> types;          // (cost, type), live types only
    for (int t = 0; t < per; ++t) {
        const int g = t % Gm, y = t / Gm;
        const int t0 = g * MB, di0 = t0 / NH, n0 = y * NN + wsh * di0 * nf;   // the kernel's
        if (t0 >= Tm || n0 / nf >= K || std::min(K - 1, (n0 + NN - 1) / nf) < di0) continue;
        int simd[4] = {0, 0, 0, 0};
        for (int wm = 0; wm < WM; ++wm) {
            int dmin = 1 << 30;
            for (int i = 0; i < MT; ++i)
                if (t0 + wm * MT + i < Tm) dmin = std::min(dmin, (t0 + wm * MT + i) / NH);
            int j0 = NT, j1 = -1;
            for (int j = 0; j < NT; ++j) {
                const int c0 = n0 + 32 * j;
                if (c0 / nf < K && std::min(K - 1, (c0 + 31) / nf) >= dmin) {
                    j0 = std::min(j0, j);
                    j1 = std::max(j1, j);
                }
            }
            simd[wm % 4] += j1 >= j0 ? MT * (j1 - j0 + 1) : 0;
        }
        const int mx = std::max(std::max(simd[0], simd[1]), std::max(simd[2], simd[3]));
        types.push_back({mx + 7.0, t});
    }
    std::stable_sort(types.begin(), types.end(),
                     [](const std::pair<double, int>& x, const std::pair<double, int>& y) {
                         return x.first > y.first;
                     });
    const int nt = (int)types.size();
    if (nt == 0) {
        pl.njobs = -1;
        return cache[key] = pl;
    }
    // split the ns heaviest types, ns = 0 .. nt: the best simulated makespan (ties: fewer)
    const int ncu = lagw_cus();
    const double fix = 0.02 * types[0].first;
    int best_ns = 0;
    double best = 0.0;
    for (int ns = 0; ns <= (sp_ok ? nt : 0); ++ns) {
        if (nt + ns > 256) break;
        std::vector<double> jc;
        for (int i = 0; i < nt; ++i) {
            const double c = types[i].first;
            if (i < ns) jc.insert(jc.end(), 2 * (size_t)m, 0.5 * c + fix);
            else jc.insert(jc.end(), (size_t)m, c);
        }
        std::stable_sort(jc.begin(), jc.end(), std::greater<double>());
        std::priority_queue<double, std::vector<double>, std::greater<double>> q;
        for (int c = 0; c < ncu; ++c) q.push(0.0);
        double mk = 0.0;
        for (double c : jc) {
            const double t = q.top() + c;
            q.pop();
            q.push(t);
            mk = std::max(mk, t);
        }
        if (ns == 0 || mk < best * 0.98) {
            best = mk;
            best_ns = ns;
        }
    }
    std::vector<std::pair<double, int>> jl;
    for (int i = 0; i < nt; ++i) {
        const double c = types[i].first;
        const int t = types[i].second;
        if (i < best_ns) {
            jl.push_back({0.5 * c + fix, t | (1 << 14)});
            jl.push_back({0.5 * c + fix, t | (2 << 14)});
            pl.mask[t >> 5] |= 1u << (t & 31);
        } else {
            jl.push_back({c, t});
        }
    }
    std::stable_sort(jl.begin(), jl.end(),
                     [](const std::pair<double, int>& x, const std::pair<double, int>& y) {
                         return x.first > y.first;
                     });
    pl.njobs = (int)jl.size();
    pl.split = best_ns > 0;
    for (int i = 0; i < pl.njobs; ++i) pl.jobs[i] = (uint16_t)jl[i].second;
    return cache[key] = pl;
}

// Kernel-only timing (sglm_lag_gram_w_timing): while on, every lag_gram_w2_kernel launch is
// bracketed by two HIP events on its stream -- the bench's roofline divides by exactly the
// kernel's time, the figure rocprofv3 reports for it (the call also holds the weight copies, the
// ones sum and the symmetrize pass).  Events come from a pool; nothing is timed while off.
std::mutex g_tmu;
bool g_ton = false;
std::vector<hipEvent_t> g_tpool;
std::vector<std::pair<hipEvent_t, hipEvent_t>> g_trec;

hipEvent_t lagw_event() {
    if (!g_tpool.empty()) {
        hipEvent_t e = g_tpool.back();
        g_tpool.pop_back();
        return e;
    }
    hipEvent_t e = nullptr;
    return hipEventCreate(&e) == hipSuccess ? e : nullptr;
}

template <int MT, int NT, int WM, int WN, int NH>
int launch_lagw2(const LagW2Args& a0, hipStream_t s, LagwSplit& sp) {
    LagW2Args a = a0;
    constexpr int MB = WM * MT, NN = WN * NT * 32;
    static_assert(WN == 1, "one wave column");
    a.Gm = (a.D * NH + MB - 1) / MB;
    a.Gy = (a.nf * a.K + NN - 1) / NN;
    // (SGLM_LAGW_WSHIFT=0: every piece's window at column 0 of its block, the round-6 v3 tiling;
    // read per launch, A/B)
    const char* ew = getenv("SGLM_LAGW_WSHIFT");
    a.wsh = (ew && ew[0] == '0') ? 0 : 1;
    const LagwPlan pl = lagw_plan(a.m, a.K, a.nf, NH, MT, NT, WM, a.Gm, a.Gy, a.Hb != nullptr,
                                  a.wsh);
    if (pl.njobs < 0) return SGLM_OK;
    sp.Hb = pl.split ? a.Hb : nullptr;
    sp.smin = a.smin;
    sp.nh = NH;
    sp.MB = MB;
    sp.NN = NN;
    sp.Gm = a.Gm;
    sp.nf = a.nf;
    sp.wsh = a.wsh;
    std::memcpy(sp.mask, pl.mask, sizeof(sp.mask));
    // (Rounding the blocks per job up to a multiple of 8, so that every piece of an event -- its
    // d groups, column blocks and halves, which stream the same weight rows -- lands on one
    // XCD's L2 (block b -> XCD b mod 8): HBM reads 1294 -> 1133 MB per launch, but the XCDs'
    // fixed event sets unbalance the launch: 5-fit call 0.854 -> 0.930 ms, 1-fit 0.312 -> 0.407
    // ms.  Dropped.)
    a.ms = a.m;
    unsigned nblk;
    if (pl.njobs > 0) {
        a.njobs = pl.njobs;
        std::memcpy(a.jobs, pl.jobs, sizeof(a.jobs));
        nblk = (unsigned)(pl.njobs * a.ms);
    } else {
        a.njobs = 0;
        nblk = (unsigned)(a.Gm * a.Gy * a.ms);
    }
#ifdef SGLM_LAGW_TRACE
    hipMalloc(&a.trace, (size_t)nblk * 32);
    hipMemsetAsync(a.trace, 0, (size_t)nblk * 32, s);
#endif
    // (MFMA bursts at raised wave priority, s_setprio 1: no gain, 0.848 / 0.890 vs 0.893 / 0.886
    // ms per 5-fit call on one box)
    hipEvent_t t0 = nullptr, t1 = nullptr;
    {
        std::lock_guard<std::mutex> lk(g_tmu);
        if (g_ton) {
            t0 = lagw_event();
            t1 = lagw_event();
        }
    }
    if (t0 && t1) (void)hipEventRecord(t0, s);
    lag_gram_w2_kernel<MT, NT, WM, WN, NH><<<dim3(nblk), 64 * WM * WN, 0, s>>>(a);
    if (t0 && t1) {
        (void)hipEventRecord(t1, s);
        std::lock_guard<std::mutex> lk(g_tmu);
        g_trec.push_back({t0, t1});
    }
#ifdef SGLM_LAGW_TRACE
    {
        static int seq = 0;
        std::vector<uint64_t> tr((size_t)nblk * 4);
        hipStreamSynchronize(s);
        hipMemcpy(tr.data(), a.trace, tr.size() * 8, hipMemcpyDeviceToHost);
        hipFree(a.trace);
        const char* out = getenv("SGLM_LAGW_TRACE_OUT");
        if (out) {
            char path[512];
            snprintf(path, sizeof(path), "%s_%d_nf%d.bin", out, seq++, a.nf);
            if (FILE* f = fopen(path, "wb")) {
                fwrite(tr.data(), 8, tr.size(), f);
                fclose(f);
            }
        }
    }
#endif
    return check_launch("lag_gram_w2_kernel");
}

}  // namespace
}  // namespace sglm

using namespace sglm;

// the zero raw row (weights 0) and the elements of one weight copy (sglm_lag_gram_w's work: 8
// copies of 2-byte elements): every read of a workgroup -- a valid occurrence's columns, the last
// column block's padding columns, the zero row's -- lies below wlen
static int64_t lagw_zrow(int32_t nraw, int32_t K) { return (int64_t)nraw + K + 8; }
static int64_t lagw_wlen(int32_t nraw, int32_t K, int32_t nf) {
    return ((lagw_zrow(nraw, K) + K + 8) * nf + 512 + 7) / 8 * 8;
}

// work: the weight copies, the ones-diagonal partial sums, the split pieces' second halves
static size_t lagw_hb_off(int32_t nraw, int32_t K, int32_t nf) {
    return ((size_t)(8 * lagw_wlen(nraw, K, nf) * 2) + (size_t)nf * kLwRed * 4 + 255) / 256 * 256;
}

extern "C" size_t sglm_lag_gram_w_work_bytes(int32_t nraw, int32_t K, int32_t nf, int32_t P) {
    return lagw_hb_off(nraw, K, nf) + (size_t)nf * P * P * 4;
}

extern "C" int sglm_lag_gram_w(const uint64_t* R, const int32_t* occ, const int32_t* ev_off,
                               int32_t m, int32_t nraw, const int32_t* shifts,
                               const int32_t* bidx, int32_t K, int32_t smin, int32_t smax,
                               int32_t layout, int32_t row0, int32_t n, const float* W,
                               int64_t ld, const int32_t* fits, int32_t nf, float* H, int32_t P,
                               int32_t pones, void* work, sglm_stream_t stream) {
    if (nf <= 0) return SGLM_OK;
    const int p = pones;                       // the ones column (K m, or after continuous ones)
    if (!R || !occ || !ev_off || !shifts || !bidx || !W || !fits || !H || !work || m < 1 ||
        m > 63 || K < 1 || smax - smin + 1 != K || p < K * m || p + 1 > P || n < 0 || ld < n) {
        set_error("sglm_lag_gram_w: bad args (m=%d K=%d P=%d)", m, K, P);
        return SGLM_EINVAL;
    }
    const int64_t wlen = lagw_wlen(nraw, K, nf);
    if (nraw >= (1 << 28) || wlen >= ((int64_t)1 << 27)) {
        // the launch addresses R and the weight image through 32-bit buffer offsets
        set_error("sglm_lag_gram_w: %d raw rows x %d fits exceed one launch (split the fits)",
                  nraw, nf);
        return SGLM_EINVAL;
    }
    hipStream_t s = as_stream(stream);
    LagW2Args b{};
    b.wlen = wlen;
    b.Wt = (const uint16_t*)work;
    lag_gram_w_prep<<<dim3(1024, 8), 256, 0, s>>>(W, ld, n, fits, nf, row0, smin, b.wlen,
                                                  lagw_zrow(nraw, K), (uint16_t*)work);
    {
        const int st0 = check_launch("lag_gram_w_prep");
        if (st0) return st0;
    }
    b.R = R; b.occ = occ; b.ev_off = ev_off; b.bidx = bidx;
    b.fits = fits; b.H = H; b.nf = nf; b.P = P; b.p = p; b.m = m; b.K = K;
    b.smin = smin; b.smax = smax; b.layout = layout; b.nraw = nraw;
    b.D = K;                                             // d = s_b1 - s_b2 >= 0 only
    float* part = (float*)((uint16_t*)work + 8 * b.wlen);
    lag_gram_w_part<<<dim3(kLwRed, (unsigned)nf), 256, 0, s>>>(W, ld, n, fits, part);
    b.Hb = (float*)((char*)work + lagw_hb_off(nraw, K, nf));
    const bool two = m + 1 > 32;                         // two 32-event halves per d row
    LagwSplit sp{};
    const int st = (nf * K <= 64) ? (two ? launch_lagw2<2, 2, 8, 1, 2>(b, s, sp)
                                         : launch_lagw2<2, 2, 8, 1, 1>(b, s, sp))
                                  : (two ? launch_lagw2<2, 4, 8, 1, 2>(b, s, sp)
                                         : launch_lagw2<2, 4, 8, 1, 1>(b, s, sp));
    if (st) return st;
    const int T = P / 64;
    lag_gram_w_sym<<<dim3((unsigned)(T * (T + 1) / 2), (unsigned)nf), 256, 0, s>>>(
        H, fits, P, p, m, K, layout, shifts, sp);
    lag_gram_w_aux<<<dim3(1, (unsigned)nf), 256, 0, s>>>(part, fits, H, P, p);
    return check_launch("lag_gram_w_aux");
}

extern "C" int sglm_lag_gram_w_timing(int32_t mode, double* ms, int32_t* n) {
    std::lock_guard<std::mutex> lk(g_tmu);
    if (mode == 0) {
        g_ton = false;
        return SGLM_OK;
    }
    double tot = 0.0;
    int cnt = 0;
    for (auto& pr : g_trec) {
        if (mode == 2) {
            float x = 0.0f;
            if (hipEventSynchronize(pr.second) == hipSuccess &&
                hipEventElapsedTime(&x, pr.first, pr.second) == hipSuccess) {
                tot += x;
                ++cnt;
            }
        }
        g_tpool.push_back(pr.first);
        g_tpool.push_back(pr.second);
    }
    g_trec.clear();
    if (mode == 1) g_ton = true;
    if (ms) *ms = tot;
    if (n) *n = cnt;
    return SGLM_OK;
}

// R[u] = sum_a bit(e_a(u)) << a | 1 << m from the occurrence bitmaps ebits[m][nwords]
__global__ void __launch_bounds__(256) lag_rowwords_kernel(const int32_t* __restrict__ ebits,
                                                           int32_t m, int32_t nwords,
                                                           int32_t nraw, uint64_t* __restrict__ R) {
    const int u = blockIdx.x * 256 + threadIdx.x;
    if (u >= nraw) return;
    uint64_t x = (uint64_t)1 << m;
    for (int e = 0; e < m; ++e)
        x |= (uint64_t)(((uint32_t)ebits[(int64_t)e * nwords + (u >> 5)] >> (u & 31)) & 1u) << e;
    R[u] = x;
}

extern "C" int sglm_lag_rowwords(const int32_t* ebits, int32_t m, int32_t nwords, int32_t nraw,
                                 uint64_t* R, sglm_stream_t stream) {
    if (!ebits || !R || m < 1 || m > 63 || nraw < 0 || nwords * 32 < nraw) {
        set_error("sglm_lag_rowwords: bad args");
        return SGLM_EINVAL;
    }
    if (nraw == 0) return SGLM_OK;
    lag_rowwords_kernel<<<(nraw + 255) / 256, 256, 0, as_stream(stream)>>>(ebits, m, nwords, nraw,
                                                                           R);
    return check_launch("lag_rowwords_kernel");
}
