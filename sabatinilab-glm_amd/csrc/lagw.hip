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
#include <type_traits>

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
// raw rows u - smin .. in (row, fit) order, shifted by c; 0 off the
// design's rows and for raw rows u >= zrow (the zero row a workgroup reads past its event's end)
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
    int32_t nf, P, p, m, K, smin, smax, layout, nraw, nh, D, Gm, Gy, Q, npieces, zrow;
    // piece order: ntypes > 0 -> block b runs piece type types[b / m] (types in decreasing
    // order of work) of event b % m (longest pieces first: the last round holds the lightest);
    // ntypes == 0 -> XCD x = b mod 8 takes the pieces [x Q, x Q + Q), event-major
    int32_t ntypes;
    uint8_t types[128];             // type = g + Gm y
};

template <int NCH>
__device__ __forceinline__ int lagw_swz(int row) {       // chunk XOR of the weight image's row
    return NCH == 16 ? ((row & 3) << 2) : (((row >> 1) & 1) << 2);
}

template <int MT, int NT, int WM, int WN>
struct LagW2Smem {
    static constexpr int MB = WM * MT, NN = WN * NT * 32;
    uint32_t rw[2][MB * kRS2];                                  // [buf][d row][pl][xy][pair]
    __attribute__((aligned(16))) uint16_t ws[2][kKS2 * NN];     // [buf][occurrence][column]
    int32_t occ[4][64 * WM * WN];          // every thread stores (rows kKS2 .. : unread)
};

template <int MT, int NT, int WM, int WN, int WPS>
__global__ void __launch_bounds__(64 * WM * WN) __attribute__((amdgpu_waves_per_eu(WPS, WPS)))
lag_gram_w2_kernel(LagW2Args a) {
    using SM = LagW2Smem<MT, NT, WM, WN>;
    constexpr int NTH = 64 * WM * WN, MB = SM::MB, NN = SM::NN, NCH = NN / 8;
    static_assert((kKS2 * NCH) % NTH == 0, "weight tasks per thread");
    constexpr int kWT = kKS2 * NCH / NTH;
    constexpr int kRT = (kKP2 * MB + NTH - 1) / NTH;
    __shared__ SM sm;
    // piece of this workgroup: XCD x = b mod 8 takes pieces [x Q, x Q + Q), event-major, the
    // d groups of one column block adjacent (they stream the same weights)
    int a1, rem;
    if (a.ntypes > 0) {
        const int b = blockIdx.x;
        if (b >= a.ntypes * a.m) return;
        a1 = b % a.m;
        rem = a.types[b / a.m];
    } else {
        const int pc = (int)(blockIdx.x & 7) * a.Q + (int)(blockIdx.x >> 3);
        if (pc >= a.npieces) return;
        const int per = a.Gm * a.Gy;
        a1 = pc / per;
        rem = pc % per;
    }
    const int g = rem % a.Gm, y = rem / a.Gm;
    const int nh = a.nh, Tm = a.D * nh;
    const int t0 = g * MB;
    if (t0 >= Tm) return;
    const int di0 = t0 / nh;
    const int di1 = min(Tm - 1, t0 + MB - 1) / nh;
    const int nd = di1 - di0 + 1;
    const int n0 = y * NN;
    // a G entry of row d and a column of shift smin + sb is an H entry only when sb >= d (its
    // second shift smin + sb - d is then a column): a piece whose columns all precede its d rows
    // has nothing to store
    if (n0 / a.nf >= a.K || min(a.K - 1, (n0 + NN - 1) / a.nf) < di0) return;
    const int o_beg = a.ev_off[a1], o_end = a.ev_off[a1 + 1];
    // every load of the pipeline is unconditional (a stage past the event's end reads the zero
    // row), so the compiler's wait counts stay exact
    const int nst = (o_end - o_beg + kKS2 - 1) / kKS2;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h = lane >> 5, r = lane & 31;
    const int wm = wave % WM, wn = wave / WM;

    // the row-word tasks of this thread (the same every stage): pair kp, d row dl
    const int ntr = kKP2 * nd;
    int rkp[kRT], rdl[kRT];
#pragma unroll
    for (int i = 0; i < kRT; ++i) {
        const int t = tid + NTH * i;
        rkp[i] = t < ntr ? t / nd : -1;
        rdl[i] = t < ntr ? t % nd : 0;
    }

    // Every load below is unconditional, from a clamped address, and what is invalid is masked
    // when the registers are stored (a load whose result is selected against a constant makes
    // hipcc wait for it right away, which would serialise the staging pipeline)
    // one register set: a stage is stored to LDS right after the barrier, then the registers
    // receive the stage after next (clang vectors: arrays of HIP's uint4 struct stay allocas)
    u32x4 wA[kWT];
    uint64_t rA[kRT][2];
    uint32_t vA = 0;                          // validity of the row-word loads, bit 2 i + j
    int32_t oreg = 0;
    bool ovalid = false;

    auto occ_load = [&](int s) __attribute__((always_inline)) {
        const int o = o_beg + s * kKS2 + tid;
        ovalid = tid < kKS2 && o < o_end;
        oreg = a.occ[ovalid ? o : o_beg];
    };
    auto occ_store = [&](int s) __attribute__((always_inline)) { sm.occ[s & 3][tid] = ovalid ? oreg : -1; };
    // staging pieces: weight chunk task i, and all row-word tasks (loads of stage s into the
    // registers; stores of the registers to buffer buf)
    auto load_w = [&](int s, int i) __attribute__((always_inline)) {
        const int* ov = sm.occ[s & 3];
        const int t = tid + NTH * i;
        const int k = t / NCH, ch = t % NCH;
        const int v = ov[k];
        const int64_t u = v >= 0 ? v : a.zrow;              // past the event's end: zero weights
        const int64_t x = u * a.nf + n0 + 8 * ch;
        const int c = (int)(x & 7);
        wA[i] = *reinterpret_cast<const u32x4*>(a.Wt + c * a.wlen + (x - c));
    };
    auto load_r = [&](int s) __attribute__((always_inline)) {
        const int* ov = sm.occ[s & 3];
        uint32_t vb = 0;
#pragma unroll
        for (int i = 0; i < kRT; ++i) {
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int v = ov[2 * max(rkp[i], 0) + j];
                const int u = v + di0 + rdl[i];
                const bool ok = rkp[i] >= 0 && v >= 0 && u < a.nraw;
                vb |= (uint32_t)ok << (2 * i + j);
                rA[i][j] = a.R[ok ? u : 0];
            }
        }
        vA = vb;
    };
    auto store_w = [&](int buf, int i) __attribute__((always_inline)) {
        const int t = tid + NTH * i;
        const int k = t / NCH, ch = t % NCH;
        *reinterpret_cast<u32x4*>(&sm.ws[buf][k * NN + 8 * (ch ^ lagw_swz<NCH>(k))]) = wA[i];
    };
    auto store_r = [&](int buf) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < kRT; ++i) {
            // a thread without a task writes a pad dword (kp 64 of d row 0: never read)
            uint32_t* dst = &sm.rw[buf][rkp[i] >= 0 ? rdl[i] * kRS2 + rkp[i] : kKP2];
            const uint64_t r0 = ((vA >> (2 * i)) & 1u) ? rA[i][0] : 0ull;
            const uint64_t r1 = ((vA >> (2 * i + 1)) & 1u) ? rA[i][1] : 0ull;
#pragma unroll
            for (int pl = 0; pl < 2; ++pl) {
                const uint32_t w0 = (uint32_t)(r0 >> (32 * pl));
                const uint32_t w1 = (uint32_t)(r1 >> (32 * pl));
                dst[(2 * pl) * kRX2] = (w0 & 0xffffu) | (w1 << 16);
                dst[(2 * pl + 1) * kRX2] = (w0 >> 16) | (w1 & 0xffff0000u);
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
        const int dl = tau / nh - di0, hf = tau % nh;
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

    // the multiplication of stage s (buffer s & 1) over the live N tiles J0 .. J1; with two
    // waves per SIMD the staging of the next stages rides inside its K-steps: stage s + 1 is
    // stored to the other buffer over the first K-steps (one piece behind each K-step's
    // MFMAs) and stage s + 2 is loaded into the freed registers over the last ones, so the
    // LDS writes and the address work of the staging overlap the MFMAs instead of following
    // the barrier in lockstep on both waves of a SIMD
    auto compute = [&](int s, auto J0c, auto J1c) __attribute__((always_inline)) {
        constexpr int J0 = decltype(J0c)::value, J1 = decltype(J1c)::value;
        const int buf = s & 1;
        const uint32_t* rwb = &sm.rw[buf][0];
        const char* wsb = reinterpret_cast<const char*>(&sm.ws[buf][0]);
        if constexpr (WPS == 1) {
            // one wave per SIMD: nothing else hides the LDS latency, so the fragments of K-step
            // ks + 1 are read (two register sets) while the MFMAs of ks run
            u32x4 wq[2][MT];
            s16x4 t1[2][NT], t2[2][NT];
            auto fetch = [&](int ks, int st) __attribute__((always_inline)) {
#pragma unroll
                for (int j = J0; j <= J1; ++j) {
                    const char* pb = wsb + boff[j] + ks * 16 * NN * 2;
                    t1[st][j] = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                        (lds_s16x4*)(__attribute__((address_space(3))) char*)pb);
                    t2[st][j] = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                        (lds_s16x4*)(__attribute__((address_space(3))) char*)(pb + 4 * NN * 2));
                }
#pragma unroll
                for (int i = 0; i < MT; ++i)
                    wq[st][i] = *reinterpret_cast<const u32x4*>(rwb + aoff[i] + 8 * ks);
            };
            fetch(0, 0);
#pragma unroll
            for (int ks = 0; ks < kKS2 / 16; ++ks) {
                const int st = ks & 1;
                if (ks + 1 < kKS2 / 16) fetch(ks + 1, st ^ 1);
                bf16x8 bq[NT];
#pragma unroll
                for (int j = J0; j <= J1; ++j) {
                    const uint2 u1 = __builtin_bit_cast(uint2, t1[st][j]);
                    const uint2 u2 = __builtin_bit_cast(uint2, t2[st][j]);
                    bq[j] = __builtin_bit_cast(bf16x8, make_uint4(u1.x, u1.y, u2.x, u2.y));
                }
#pragma unroll
                for (int i = 0; i < MT; ++i) {
                    uint32_t dq[4];
#pragma unroll
                    for (int q = 0; q < 4; ++q) dq[q] = rotr32(wq[st][i][q], rsh) & 0x40004000u;
                    const bf16x8 aq =
                        __builtin_bit_cast(bf16x8, make_uint4(dq[0], dq[1], dq[2], dq[3]));
#pragma unroll
                    for (int j = J0; j <= J1; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(aq, bq[j], acc[i][j],
                                                                            0, 0, 0);
                }
            }
            return;
        }
        static_assert(WPS == 1 || kWT <= 4, "staging pieces per K-step");
#pragma unroll
        for (int ks = 0; ks < kKS2 / 16; ++ks) {
            if (ks < kWT) store_w(buf ^ 1, ks);
            if (ks == kWT) store_r(buf ^ 1);
            if (ks == 4) occ_load(s + 4);
            if (ks >= 4 && ks - 4 < kWT) load_w(s + 2, ks - 4);
            if (ks == 7) load_r(s + 2);
            bf16x8 bq[NT];
#pragma unroll
            for (int j = J0; j <= J1; ++j) {
                const char* pb = wsb + boff[j] + ks * 16 * NN * 2;
                const s16x4 t1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                    (lds_s16x4*)(__attribute__((address_space(3))) char*)pb);
                const s16x4 t2 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                    (lds_s16x4*)(__attribute__((address_space(3))) char*)(pb + 4 * NN * 2));
                const uint2 u1 = __builtin_bit_cast(uint2, t1), u2 = __builtin_bit_cast(uint2, t2);
                bq[j] = __builtin_bit_cast(bf16x8, make_uint4(u1.x, u1.y, u2.x, u2.y));
            }
            bf16x8 aq[MT];
#pragma unroll
            for (int i = 0; i < MT; ++i) {
                const uint4 wq = *reinterpret_cast<const uint4*>(rwb + aoff[i] + 8 * ks);
                const uint32_t wv[4] = {wq.x, wq.y, wq.z, wq.w};
                uint32_t dq[4];
#pragma unroll
                for (int q = 0; q < 4; ++q) dq[q] = rotr32(wv[q], rsh) & 0x40004000u;
                aq[i] = __builtin_bit_cast(bf16x8, make_uint4(dq[0], dq[1], dq[2], dq[3]));
            }
#pragma unroll
            for (int i = 0; i < MT; ++i)
#pragma unroll
                for (int j = J0; j <= J1; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(aq[i], bq[j], acc[i][j],
                                                                        0, 0, 0);
        }
    };
    // stage s: stage s + 1 (loaded during stage s - 1) is stored to the other buffer, the
    // occurrence rows of stage s + 4 and the data of stage s + 2 are loaded, stage s is
    // multiplied (its loads overlap it)
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
            if constexpr (WPS == 1) {
                data_store((s + 1) & 1);     // past the end: zero rows, never read
                occ_load(s + 4);
                data_load(s + 2);
            }
            compute(s, J0c, J1c);            // WPS 2: stores s + 1, loads s + 2 inside
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
        float* Hrow = a.H + (int64_t)a.fits[f] * a.P * a.P + (int64_t)lag_col2(a.layout, a.m, a.K,
                                                                             b1, a1) * a.P;
#pragma unroll
        for (int i = 0; i < MT; ++i) {
            const int tau = t0 + wm * MT + i;
            if (tau >= Tm) continue;
            const int dd = tau / nh;
            const int hf = tau % nh;
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
}

// Upper triangle of H_f from the entries lag_gram_w2_kernel wrote: entry {i, j} (i < j) sits at
// row i when column i has the larger shift, or the same shift and the smaller event (the ones
// column p: at row i); continuous columns of a mixed design and the padding columns are zeroed
// (the continuous rows / columns are written after this by _mix_hess).  One 256-thread workgroup
// per 64 x 64 upper tile (I, J) of one fit: the transposed tile (J, I) staged through LDS.
__global__ void __launch_bounds__(256) lag_gram_w_sym(float* __restrict__ H,
                                                      const int32_t* __restrict__ fits, int32_t P,
                                                      int32_t p, int32_t m, int32_t K,
                                                      int32_t layout,
                                                      const int32_t* __restrict__ shifts) {
    __shared__ float tl[64][65];
    __shared__ int ks_i[64], ks_j[64];           // (shift, event) keys of the tile's columns
    const int T = P / 64;
    int I = 0, rem = blockIdx.x;
    while (rem >= T - I) { rem -= T - I; ++I; }  // tile (I, J), I <= J, row-major over the upper
    const int J = I + rem;
    float* Hf = H + (int64_t)fits[blockIdx.y] * P * P;
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
    // stage H rows J*64.., columns I*64.. (the lower counterpart)
    for (int e = tid; e < 64 * 64; e += 256) {
        const int rr = e >> 6, cc = e & 63;
        tl[rr][cc] = Hf[(int64_t)(J * 64 + rr) * P + I * 64 + cc];
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
        if (i == j) continue;                    // diagonal: written in place (H[p][p] by aux)
        if (j == p) {
            if (i >= plag) *dst = 0.0f;          // a continuous column's ones entry
            continue;                            // a lag column's: at row i
        }
        const int ki = ks_i[il], kj = ks_j[jl];
        if (ki < 0 || kj < 0) *dst = 0.0f;       // a continuous column
        else if (kj > ki) *dst = tl[jl][il];     // held at row j
    }
}

template <int MT, int NT, int WM, int WN, int WPS>
int launch_lagw2(const LagW2Args& a0, hipStream_t s) {
    LagW2Args a = a0;
    constexpr int MB = WM * MT, NN = WN * NT * 32;
    a.Gm = (a.D * a.nh + MB - 1) / MB;
    a.Gy = (a.nf * a.K + NN - 1) / NN;
    a.npieces = a.m * a.Gm * a.Gy;
    a.Q = (a.npieces + 7) / 8;
    a.ntypes = 0;
    // longest pieces first (default; measured 0.634 -> 0.600 ms per launch on the C4 grid
    // against the XCD-local ranges: the last round of workgroups then holds the lightest pieces,
    // which outweighs the L2 sharing of one event's pieces); SGLM_LAGW_ORDER=0: XCD ranges
    static const int lpt = [] {
        const char* e = getenv("SGLM_LAGW_ORDER");
        return e ? atoi(e) : 1;
    }();
    const int per = a.Gm * a.Gy;
    if (lpt && per <= 128) {
        // work of a piece type: its live (M tile, N tile) MFMA pairs per K-step plus the
        // staging every piece does (about a quarter of a full piece's MFMA time)
        int cost[128];
        for (int t = 0; t < per; ++t) {
            const int g = t % a.Gm, y = t / a.Gm;
            const int t0 = g * MB, Tm = a.D * a.nh;
            int live = 0;
            for (int tau = t0; tau < t0 + MB && tau < Tm; ++tau) {
                const int d = tau / a.nh;
                for (int j = 0; j < NN / 32; ++j) {
                    const int c0 = y * NN + 32 * j;
                    const int sb_lo = c0 / a.nf, sb_hi = std::min(a.K - 1, (c0 + 31) / a.nf);
                    if (sb_lo < a.K && sb_hi >= d) ++live;
                }
            }
            const int n0 = y * NN, di0 = t0 / a.nh;
            const bool dead = t0 >= Tm || n0 / a.nf >= a.K ||
                              std::min(a.K - 1, (n0 + NN - 1) / a.nf) < di0;
            cost[t] = dead ? -1 : live + MB * (NN / 32) / 4;
        }
        int nt = 0;
        for (int t = 0; t < per; ++t)
            if (cost[t] >= 0) a.types[nt++] = (uint8_t)t;
        std::stable_sort(a.types, a.types + nt,
                         [&](uint8_t x, uint8_t y) { return cost[x] > cost[y]; });
        a.ntypes = nt;
        if (nt == 0) return SGLM_OK;
        lag_gram_w2_kernel<MT, NT, WM, WN, WPS><<<dim3((unsigned)(nt * a.m)), 64 * WM * WN, 0,
                                                  s>>>(a);
        return check_launch("lag_gram_w2_kernel");
    }
    lag_gram_w2_kernel<MT, NT, WM, WN, WPS><<<dim3((unsigned)(8 * a.Q)), 64 * WM * WN, 0, s>>>(a);
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

extern "C" size_t sglm_lag_gram_w_work_bytes(int32_t nraw, int32_t K, int32_t nf) {
    return (size_t)(8 * lagw_wlen(nraw, K, nf) * 2) + (size_t)nf * kLwRed * 4;
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
    hipStream_t s = as_stream(stream);
    LagW2Args b{};
    b.wlen = lagw_wlen(nraw, K, nf);
    b.Wt = (const uint16_t*)work;
    b.zrow = (int32_t)lagw_zrow(nraw, K);
    lag_gram_w_prep<<<dim3(1024, 8), 256, 0, s>>>(W, ld, n, fits, nf, row0, smin, b.wlen, b.zrow,
                                                  (uint16_t*)work);
    {
        const int st0 = check_launch("lag_gram_w_prep");
        if (st0) return st0;
    }
    b.R = R; b.occ = occ; b.ev_off = ev_off; b.bidx = bidx;
    b.fits = fits; b.H = H; b.nf = nf; b.P = P; b.p = p; b.m = m; b.K = K;
    b.smin = smin; b.smax = smax; b.layout = layout; b.nraw = nraw;
    b.nh = (m + 1 + 31) / 32;
    b.D = K;                                             // d = s_b1 - s_b2 >= 0 only
    float* part = (float*)((uint16_t*)work + 8 * b.wlen);
    lag_gram_w_part<<<dim3(kLwRed, (unsigned)nf), 256, 0, s>>>(W, ld, n, fits, part);
    static const int wps1 = [] {
        const char* e = getenv("SGLM_LAGW_WPS1");
        return e ? atoi(e) : 0;
    }();
    const int st = wps1 ? ((nf * K <= 64) ? launch_lagw2<4, 2, 4, 1, 1>(b, s)
                                          : launch_lagw2<4, 4, 4, 1, 1>(b, s))
                        : ((nf * K <= 64) ? launch_lagw2<2, 2, 8, 1, 2>(b, s)
                                          : launch_lagw2<2, 4, 8, 1, 2>(b, s));
    if (st) return st;
    const int T = P / 64;
    lag_gram_w_sym<<<dim3((unsigned)(T * (T + 1) / 2), (unsigned)nf), 256, 0, s>>>(
        H, fits, P, p, m, K, layout, shifts);
    lag_gram_w_aux<<<dim3(1, (unsigned)nf), 256, 0, s>>>(part, fits, H, P, p);
    return check_launch("lag_gram_w_aux");
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
