// Event design matrix of a behaviour session (pp_design_mat.make_design_mat and its helpers,
// /root/reference/pp_design_mat.py:6-205) on the GPU.
//
// The reference is pandas: per-row column products, and groupby('nTrial') cumcount / nth /
// first / sum plus Series.map lookups into the trial table.  Here a groupby is a GROUPING of
// the rows -- a permutation that makes every key's rows contiguous, in row order within the
// key (pandas' group order and within-group order), rows with a NaN key left out (groupby
// drops them) -- and every per-group operation is one wave walking its group's rows in 64-row
// slabs (ballot / popcount prefix counts, first-match search, fixed-order sums).  Session
// columns are float64 struct-of-arrays (a pandas float block), so row kernels stream whole
// columns.  The grouping is a stable partition of the valid rows when the key is already
// ordered (the session's nTrial is a running trial count), a stable radix sort otherwise.
#include "common.h"

#include <hipcub/hipcub.hpp>
#include <math.h>

namespace sglm {
namespace {

constexpr int kDmT = 256;                 // threads per workgroup (4 waves)
constexpr int kOrdRows = 16;              // rows per thread in the ordering check

// order-preserving image of a double (total order of the non-NaN values, -0 == +0); NaN maps
// to all ones and sorts last
__device__ __forceinline__ uint64_t key_bits(double v) {
    if (isnan(v)) return ~0ull;
    if (v == 0.0) v = 0.0;
    const uint64_t b = (uint64_t)__double_as_longlong(v);
    return (b >> 63) ? ~b : (b | (1ull << 63));
}

__device__ __forceinline__ uint64_t lanemask_lt(int lane) {
    return lane == 0 ? 0ull : (~0ull >> (64 - lane));
}

// ---- grouping -------------------------------------------------------------------------
struct Ord {          // ordering summary of a row range (valid rows only)
    uint64_t f1, f2, l1, l2;
    long long cnt;
    long long heads;  // key changes within the range, its first valid row counted as one
    int ok;
};

__device__ __forceinline__ bool lex_le(uint64_t a1, uint64_t a2, uint64_t b1, uint64_t b2) {
    return a1 < b1 || (a1 == b1 && a2 <= b2);
}

__device__ __forceinline__ Ord ord_comb(const Ord& a, const Ord& b) {
    if (a.cnt == 0) return b;
    if (b.cnt == 0) return a;
    Ord r;
    r.f1 = a.f1; r.f2 = a.f2; r.l1 = b.l1; r.l2 = b.l2;
    r.cnt = a.cnt + b.cnt;
    r.heads = a.heads + b.heads - ((a.l1 == b.f1 && a.l2 == b.f2) ? 1 : 0);
    r.ok = a.ok && b.ok && lex_le(a.l1, a.l2, b.f1, b.f2);
    return r;
}

// Per workgroup: is the valid-row key sequence of its range non-decreasing (lexicographic in
// (key, key2)), how many valid rows; also the valid flags.
__global__ void __launch_bounds__(kDmT) group_order_kernel(const double* __restrict__ key,
                                                           const double* __restrict__ key2,
                                                           int64_t n, uint8_t* __restrict__ valid,
                                                           Ord* __restrict__ part) {
    __shared__ Ord sh[kDmT];
    const int64_t r0 = ((int64_t)blockIdx.x * kDmT + threadIdx.x) * kOrdRows;
    Ord o = {0, 0, 0, 0, 0, 0, 1};
    for (int j = 0; j < kOrdRows; ++j) {
        const int64_t i = r0 + j;
        if (i >= n) break;
        const double a = key[i], b = key2 ? key2[i] : 0.0;
        const bool v = !isnan(a) && !isnan(b);
        valid[i] = v;
        if (!v) continue;
        Ord e = {key_bits(a), key_bits(b), key_bits(a), key_bits(b), 1, 1, 1};
        o = ord_comb(o, e);
    }
    sh[threadIdx.x] = o;
    __syncthreads();
    if (threadIdx.x == 0) {
        Ord r = sh[0];
        for (int t = 1; t < kDmT; ++t) r = ord_comb(r, sh[t]);
        part[blockIdx.x] = r;
    }
}

// Over the workgroup summaries in order: the verdict (ordered?, valid rows, groups) and per
// block the exclusive offsets of its valid rows and group heads in the compacted order and
// the last valid key before it (for the head test of its first valid row).
struct BlockOff { long long v, h; uint64_t p1, p2; int has; };

__global__ void __launch_bounds__(kDmT) group_order_final_kernel(const Ord* __restrict__ part,
                                                                 int64_t nb,
                                                                 long long* __restrict__ res,
                                                                 BlockOff* __restrict__ off) {
    __shared__ Ord sh[kDmT];
    const int64_t per = (nb + kDmT - 1) / kDmT;
    const int64_t b0 = (int64_t)threadIdx.x * per;
    const int64_t b1 = b0 + per < nb ? b0 + per : nb;
    Ord o = {0, 0, 0, 0, 0, 0, 1};
    for (int64_t b = b0; b < b1; ++b) o = ord_comb(o, part[b]);
    sh[threadIdx.x] = o;
    __syncthreads();
    if (threadIdx.x == 0) {
        Ord r = sh[0];
        for (int t = 1; t < kDmT; ++t) r = ord_comb(r, sh[t]);
        res[0] = r.ok;
        res[1] = r.cnt;
        res[2] = r.heads;
    }
    // exclusive prefix of the runs before this thread's, then walk the run
    Ord pre = {0, 0, 0, 0, 0, 0, 1};
    for (int t = 0; t < (int)threadIdx.x; ++t) pre = ord_comb(pre, sh[t]);
    for (int64_t b = b0; b < b1; ++b) {
        const Ord& cur = part[b];
        BlockOff bo;
        bo.v = pre.cnt;
        bo.h = pre.heads;
        bo.has = pre.cnt > 0;
        bo.p1 = pre.l1;
        bo.p2 = pre.l2;
        off[b] = bo;
        pre = ord_comb(pre, cur);
    }
}

// Stable compaction of an ORDERED key sequence: perm = the valid rows in row order, seg = the
// positions in perm where the key changes (group starts); thread = 16 consecutive rows,
// in-block prefix counts and "last valid key before me" by Hillis-Steele passes in LDS.
__global__ void __launch_bounds__(kDmT) group_compact_kernel(const double* __restrict__ key,
                                                             const double* __restrict__ key2,
                                                             int64_t n,
                                                             const BlockOff* __restrict__ off,
                                                             int64_t* __restrict__ perm,
                                                             int64_t* __restrict__ seg) {
    __shared__ int cv[kDmT], ch[kDmT], hv[kDmT];
    __shared__ uint64_t k1s[kDmT], k2s[kDmT];
    const int tid = threadIdx.x;
    const BlockOff bo = off[blockIdx.x];
    const int64_t r0 = ((int64_t)blockIdx.x * kDmT + tid) * kOrdRows;
    uint64_t a1[kOrdRows], a2[kOrdRows];
    uint32_t vm = 0;
    int nv = 0;
    uint64_t l1 = 0, l2 = 0;
#pragma unroll
    for (int j = 0; j < kOrdRows; ++j) {
        const int64_t i = r0 + j;
        a1[j] = a2[j] = 0;
        if (i < n) {
            const double x = key[i], y = key2 ? key2[i] : 0.0;
            if (!isnan(x) && !isnan(y)) {
                vm |= 1u << j;
                a1[j] = key_bits(x);
                a2[j] = key_bits(y);
                l1 = a1[j];
                l2 = a2[j];
                ++nv;
            }
        }
    }
    // nearest valid key before this thread's run: inclusive scan of (has, last key), shifted
    hv[tid] = nv > 0;
    k1s[tid] = l1;
    k2s[tid] = l2;
    cv[tid] = nv;
    __syncthreads();
    for (int o = 1; o < kDmT; o <<= 1) {
        int h = 0, c = 0;
        uint64_t x1 = 0, x2 = 0;
        const bool take = tid >= o;
        if (take) { h = hv[tid - o]; x1 = k1s[tid - o]; x2 = k2s[tid - o]; c = cv[tid - o]; }
        __syncthreads();
        if (take) {
            if (!hv[tid] && h) { hv[tid] = 1; k1s[tid] = x1; k2s[tid] = x2; }
            cv[tid] += c;
        }
        __syncthreads();
    }
    // exclusive: the values of thread tid - 1 (block prefix for thread 0)
    int has_prev = tid > 0 ? hv[tid - 1] : 0;
    uint64_t p1 = tid > 0 ? k1s[tid - 1] : 0, p2 = tid > 0 ? k2s[tid - 1] : 0;
    if (!has_prev && bo.has) { has_prev = 1; p1 = bo.p1; p2 = bo.p2; }
    const int vpre = tid > 0 ? cv[tid - 1] : 0;
    // heads of this thread's run
    int nh = 0;
    {
        int hp = has_prev;
        uint64_t q1 = p1, q2 = p2;
#pragma unroll
        for (int j = 0; j < kOrdRows; ++j) {
            if (vm >> j & 1u) {
                if (!hp || a1[j] != q1 || a2[j] != q2) ++nh;
                hp = 1; q1 = a1[j]; q2 = a2[j];
            }
        }
    }
    __syncthreads();
    ch[tid] = nh;
    __syncthreads();
    for (int o = 1; o < kDmT; o <<= 1) {
        const int c = tid >= o ? ch[tid - o] : 0;
        __syncthreads();
        ch[tid] += c;
        __syncthreads();
    }
    const int hpre = tid > 0 ? ch[tid - 1] : 0;
    int64_t pv = bo.v + vpre, ph = bo.h + hpre;
    int hp = has_prev;
    uint64_t q1 = p1, q2 = p2;
#pragma unroll
    for (int j = 0; j < kOrdRows; ++j) {
        if (vm >> j & 1u) {
            if (!hp || a1[j] != q1 || a2[j] != q2) seg[ph++] = pv;
            perm[pv++] = r0 + j;
            hp = 1; q1 = a1[j]; q2 = a2[j];
        }
    }
}

__global__ void group_finish2_kernel(int64_t* __restrict__ seg, const long long* __restrict__ res,
                                     int64_t* __restrict__ counts) {
    const long long m = res[1], g = res[2];
    seg[g] = m;
    counts[0] = m;
    counts[1] = g;
}

// radix keys: the key's image, all ones when either key is NaN (those rows sort last)
__global__ void group_keys_kernel(const double* __restrict__ key, const double* __restrict__ key2,
                                  const int64_t* __restrict__ order, int64_t n, int use2,
                                  uint64_t* __restrict__ out, int64_t* __restrict__ iota) {
    const int64_t q = (int64_t)blockIdx.x * kDmT + threadIdx.x;
    if (q >= n) return;
    const int64_t i = order ? order[q] : q;
    const double a = key[i], b = key2 ? key2[i] : 0.0;
    const bool v = !isnan(a) && !isnan(b);
    out[q] = v ? key_bits(use2 ? b : a) : ~0ull;
    if (iota) iota[q] = q;
}

__global__ void group_heads_kernel(const double* __restrict__ key, const double* __restrict__ key2,
                                   const int64_t* __restrict__ perm, int64_t m,
                                   uint8_t* __restrict__ head) {
    const int64_t q = (int64_t)blockIdx.x * kDmT + threadIdx.x;
    if (q >= m) return;
    bool h = q == 0;
    if (!h) {
        const int64_t i = perm[q], j = perm[q - 1];
        h = key_bits(key[i]) != key_bits(key[j]) ||
            (key2 && key_bits(key2[i]) != key_bits(key2[j]));
    }
    head[q] = h;
}

__global__ void group_finish_kernel(int64_t* __restrict__ seg, const int* __restrict__ nseg,
                                    int64_t m, int64_t* __restrict__ counts) {
    const int g = *nseg;
    seg[g] = m;
    counts[0] = m;
    counts[1] = g;
}

// ---- per-group walks --------------------------------------------------------------------
// wave w of the grid handles groups w, w + W, ... (W waves in the grid)
#define DM_FOR_GROUPS(counts)                                                                   \
    const int lane = threadIdx.x & 63;                                                          \
    const int64_t nseg_ = (counts)[1];                                                          \
    for (int64_t s = (int64_t)blockIdx.x * (kDmT / 64) + (threadIdx.x >> 6); s < nseg_;         \
         s += (int64_t)gridDim.x * (kDmT / 64))

__device__ __forceinline__ double wave_sum_d(double v) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

struct HmArgs {
    const double *clock, *cue, *cons, *scons;
    const int32_t* tidx;
    const double* tsel;
    double *off_sel, *from_cue, *from_cons, *sel_cons, *off_cons;
    int64_t n;
};

// add_heatmap_columns (pp_design_mat.py:108-126), rows outside every group (NaN nTrial): the
// maps give NaN
__global__ void __launch_bounds__(kDmT) hm_rows_kernel(HmArgs a) {
    const int64_t i = (int64_t)blockIdx.x * kDmT + threadIdx.x;
    if (i >= a.n) return;
    a.off_sel[i] = NAN; a.from_cue[i] = NAN; a.from_cons[i] = NAN;
    a.sel_cons[i] = NAN; a.off_cons[i] = NAN;
}

// per group: the first non-null trial_clock of its Cue == 1 rows and of its Consumption == 1
// rows (groupby first, :114, 117), the sums of Consumption and stateConsumption (agg sum,
// skipna, :120), then every row of the group (:112-124)
__global__ void __launch_bounds__(kDmT) hm_groups_kernel(HmArgs a,
                                                         const int64_t* __restrict__ perm,
                                                         const int64_t* __restrict__ seg,
                                                         const int64_t* __restrict__ counts) {
    DM_FOR_GROUPS(counts) {
        const int64_t q0 = seg[s], q1 = seg[s + 1];
        double fcue = NAN, fcons = NAN, sc = 0.0, ssc = 0.0;
        bool got_cue = false, got_cons = false;
        for (int64_t b = q0; b < q1; b += 64) {
            const int64_t q = b + lane;
            const bool v = q < q1;
            const int64_t i = v ? perm[q] : 0;
            const double ck = v ? a.clock[i] : NAN;
            const double cu = v ? a.cue[i] : 0.0, co = v ? a.cons[i] : 0.0;
            const double scv = v ? a.scons[i] : 0.0;
            const uint64_t mc = __ballot(cu == 1.0 && !isnan(ck));
            if (!got_cue && mc) { fcue = __shfl(ck, __ffsll((long long)mc) - 1, 64); got_cue = true; }
            const uint64_t mo = __ballot(co == 1.0 && !isnan(ck));
            if (!got_cons && mo) { fcons = __shfl(ck, __ffsll((long long)mo) - 1, 64); got_cons = true; }
            sc += isnan(co) ? 0.0 : co;
            ssc += isnan(scv) ? 0.0 : scv;
        }
        const double stc = (wave_sum_d(ssc) - wave_sum_d(sc)) * (1000.0 / 50.0);
        for (int64_t b = q0; b < q1; b += 64) {
            const int64_t q = b + lane;
            if (q >= q1) break;
            const int64_t i = perm[q];
            const double ck = a.clock[i];
            const int32_t t = a.tidx ? a.tidx[i] : -1;
            const double off = t >= 0 ? a.tsel[t] : NAN;
            a.from_cue[i] = ck - fcue;
            a.from_cons[i] = ck - fcons;
            a.sel_cons[i] = stc;
            a.off_sel[i] = off;
            a.off_cons[i] = stc + off;
        }
    }
}

constexpr int kMaxCols = 32;

struct LickArgs {
    const double* lick_src;            // iSpout (from_spout) or the Lick column
    int from_spout;
    const double* states[kMaxCols];
    double* out[kMaxCols];
    int ns;
    double* lick_out;                  // optional: the Lick column (int 0/1 as float64)
    int64_t n;
};

// Lick = ~isnan(iSpout) (:160); classify_lick_state: '<sta>_lick' = state * Lick (:20-21)
__global__ void __launch_bounds__(kDmT) licks_kernel(LickArgs a) {
    const int64_t i = (int64_t)blockIdx.x * kDmT + threadIdx.x;
    if (i >= a.n) return;
    const double src = a.lick_src[i];
    const double L = a.from_spout ? (isnan(src) ? 0.0 : 1.0) : src;
    if (a.lick_out) a.lick_out[i] = L;
    for (int c = 0; c < a.ns; ++c) a.out[c][i] = a.states[c][i] * L;
}

struct CntArgs {
    const double *enl, *cue, *senlp;
    double *tenl, *tenlp, *cue_on;
    int64_t n;
};

// rows outside the groups: the counter of a row that meets the condition is NaN (cumcount of
// a NaN-key row), 0 otherwise; no cue onset
__global__ void __launch_bounds__(kDmT) counters_rows_kernel(CntArgs a) {
    const int64_t i = (int64_t)blockIdx.x * kDmT + threadIdx.x;
    if (i >= a.n) return;
    const bool pe = a.enl[i] == 1.0 || a.cue[i] == 1.0;
    a.tenl[i] = pe ? NAN : 0.0;
    a.tenlp[i] = a.senlp[i] == 1.0 ? NAN : 0.0;
    if (a.cue_on) a.cue_on[i] = 0.0;
}

// time_from_enl_onset = cumcount**2 / (50*100) over the (ENL == 1 | Cue == 1) rows of each
// nTrial group (:171); the cue column: 1 on the first Cue == 1 row of each group (:175, 183)
__global__ void __launch_bounds__(kDmT) counters_enl_kernel(CntArgs a,
                                                            const int64_t* __restrict__ perm,
                                                            const int64_t* __restrict__ seg,
                                                            const int64_t* __restrict__ counts) {
    DM_FOR_GROUPS(counts) {
        const int64_t q0 = seg[s], q1 = seg[s + 1];
        long long c = 0;
        bool onset = false;
        for (int64_t b = q0; b < q1; b += 64) {
            const int64_t q = b + lane;
            const bool v = q < q1;
            const int64_t i = v ? perm[q] : 0;
            const bool cu = v && a.cue[i] == 1.0;
            const bool pe = v && (cu || a.enl[i] == 1.0);
            const uint64_t m = __ballot(pe);
            if (pe) {
                const long long k = c + __popcll(m & lanemask_lt(lane));
                a.tenl[i] = (double)(k * k) / 5000.0;
            }
            c += __popcll(m);
            const uint64_t mc = __ballot(cu);
            if (!onset && mc) {
                if (a.cue_on && lane == __ffsll((long long)mc) - 1) a.cue_on[i] = 1.0;
                onset = true;
            }
        }
    }
}

// time_from_enlp_onset = cumcount**2 / (50*100) over the state_ENLP == 1 rows of each
// (nTrial, nENL) group (:172)
__global__ void __launch_bounds__(kDmT) counters_enlp_kernel(CntArgs a,
                                                             const int64_t* __restrict__ perm,
                                                             const int64_t* __restrict__ seg,
                                                             const int64_t* __restrict__ counts) {
    DM_FOR_GROUPS(counts) {
        const int64_t q0 = seg[s], q1 = seg[s + 1];
        long long c = 0;
        for (int64_t b = q0; b < q1; b += 64) {
            const int64_t q = b + lane;
            const bool v = q < q1;
            const int64_t i = v ? perm[q] : 0;
            const bool p = v && a.senlp[i] == 1.0;
            const uint64_t m = __ballot(p);
            if (p) {
                const long long k = c + __popcll(m & lanemask_lt(lane));
                a.tenlp[i] = (double)(k * k) / 5000.0;
            }
            c += __popcll(m);
        }
    }
}

constexpr int kMaxPull = 16;

struct PullArgs {
    double* bout;
    double* col[kMaxPull];
    int nth[kMaxPull];
    int np;
    int64_t n;
};

__global__ void __launch_bounds__(kDmT) pull_zero_kernel(PullArgs a) {
    const int64_t i = (int64_t)blockIdx.x * kDmT + threadIdx.x;
    if (i >= a.n) return;
    for (int j = 0; j < a.np; ++j) a.col[j][i] = 0.0;
}

// pull_lick_from_bout (:44-53): for each position in processing order, the nth (nth - 1 >= 0
// from the start, < 0 from the end) bout == 1 row of each group moves to its column (the
// column is reset first, as `t_[new_col] = 0` does), and the bout row is zeroed
__global__ void __launch_bounds__(kDmT) pull_groups_kernel(PullArgs a,
                                                           const int64_t* __restrict__ perm,
                                                           const int64_t* __restrict__ seg,
                                                           const int64_t* __restrict__ counts) {
    DM_FOR_GROUPS(counts) {
        const int64_t q0 = seg[s], q1 = seg[s + 1];
        for (int j = 0; j < a.np; ++j) {
            const long long k = a.nth[j] - 1;
            double* col = a.col[j];
            long long total = 0;
            if (k < 0) {
                for (int64_t b = q0; b < q1; b += 64) {
                    const int64_t q = b + lane;
                    total += __popcll(__ballot(q < q1 && a.bout[perm[q]] == 1.0));
                }
            }
            const long long target = k >= 0 ? k : total + k;
            long long c = 0;
            for (int64_t b = q0; b < q1; b += 64) {
                const int64_t q = b + lane;
                const bool v = q < q1;
                const int64_t i = v ? perm[q] : 0;
                if (v) col[i] = 0.0;
                const bool l = v && a.bout[i] == 1.0;
                const uint64_t m = __ballot(l);
                if (l && c + __popcll(m & lanemask_lt(lane)) == target) {
                    col[i] = 1.0;
                    a.bout[i] = 0.0;
                }
                c += __popcll(m);
            }
        }
    }
}

// Series.map(trial table) (:93, 112, 192): per row the trial-table row of its nTrial value
// (binary search over the sorted trial ids), -1 when the key is NaN or absent
__global__ void __launch_bounds__(kDmT) trial_lookup_kernel(const double* __restrict__ key,
                                                            int64_t n,
                                                            const double* __restrict__ tkeys,
                                                            int64_t nt,
                                                            int32_t* __restrict__ tidx) {
    const int64_t i = (int64_t)blockIdx.x * kDmT + threadIdx.x;
    if (i >= n) return;
    const double k = key[i];
    int32_t r = -1;
    if (!isnan(k) && nt > 0) {
        int64_t lo = 0, hi = nt;
        while (lo < hi) {
            const int64_t mid = (lo + hi) >> 1;
            if (tkeys[mid] < k) lo = mid + 1; else hi = mid;
        }
        if (lo < nt && tkeys[lo] == k) r = (int32_t)lo;
    }
    tidx[i] = r;
}

// out[dst_cols[c]][i] = (src_cols[c] < 0 ? 1 : src[src_cols[c]][i]) * vals[val_cols[c]][t(i)],
// NaN where the row maps to no trial: event_interactions_dummies' products of the lick
// columns with the mapped dummies (:93-99), the flag's mapped isna (:192)
__global__ void __launch_bounds__(kDmT) trial_map_kernel(int64_t n,
                                                         const int32_t* __restrict__ tidx,
                                                         const double* __restrict__ src,
                                                         int64_t ld_src,
                                                         const int32_t* __restrict__ src_cols,
                                                         const double* __restrict__ vals,
                                                         int64_t nt,
                                                         const int32_t* __restrict__ val_cols,
                                                         double* __restrict__ dst, int64_t ld_dst,
                                                         const int32_t* __restrict__ dst_cols) {
    const int64_t i = (int64_t)blockIdx.x * kDmT + threadIdx.x;
    const int c = blockIdx.y;
    if (i >= n) return;
    const int32_t t = tidx[i];
    const int32_t sc = src_cols[c];
    const double x = sc < 0 ? 1.0 : src[(int64_t)sc * ld_src + i];
    const double v = t >= 0 ? vals[(int64_t)val_cols[c] * nt + t] : NAN;
    dst[(int64_t)dst_cols[c] * ld_dst + i] = x * v;
}

// trials whose rows sum to 0 over the listed columns (groupby sum, skipna, then the row sum,
// :198-203): flag = 1 on all their rows
__global__ void __launch_bounds__(kDmT) zero_groups_flag_kernel(const int64_t* __restrict__ perm,
                                                                const int64_t* __restrict__ seg,
                                                                const int64_t* __restrict__ counts,
                                                                const double* __restrict__ src,
                                                                int64_t ld,
                                                                const int32_t* __restrict__ cols,
                                                                int32_t ncols,
                                                                double* __restrict__ flag,
                                                                uint8_t* __restrict__ gz) {
    DM_FOR_GROUPS(counts) {
        const int64_t q0 = seg[s], q1 = seg[s + 1];
        double tot = 0.0;
        for (int c = 0; c < ncols; ++c) {
            const double* x = src + (int64_t)cols[c] * ld;
            double acc = 0.0;
            for (int64_t b = q0; b < q1; b += 64) {
                const int64_t q = b + lane;
                const double v = q < q1 ? x[perm[q]] : 0.0;
                acc += isnan(v) ? 0.0 : v;
            }
            tot += wave_sum_d(acc);
        }
        if (gz && lane == 0) gz[s] = tot == 0.0;
        if (tot == 0.0)
            for (int64_t b = q0; b < q1; b += 64) {
                const int64_t q = b + lane;
                if (q < q1) flag[perm[q]] = 1.0;
            }
    }
}

inline unsigned rows_grid(int64_t n) { return (unsigned)((n + kDmT - 1) / kDmT); }

// groups are walked by a fixed grid of waves (the group count lives on the device)
inline unsigned groups_grid(int64_t n) {
    int64_t g = (n + 64 * kDmT - 1) / (64 * kDmT);
    if (g < 64) g = 64;
    if (g > 2048) g = 2048;
    return (unsigned)g;
}

struct GroupWork {
    uint8_t* valid;
    Ord* part;
    BlockOff* off;
    long long* res;
    int* nsel;
    uint64_t *ka, *kb;
    int64_t *va, *vb;
    void* temp;
    size_t temp_bytes;
};

size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

size_t cub_temp_bytes(int64_t n) {
    size_t a = 0, b = 0, c = 0;
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, a, (const uint64_t*)nullptr,
                                             (uint64_t*)nullptr, (const int64_t*)nullptr,
                                             (int64_t*)nullptr, (int)(n > 0 ? n : 1));
    (void)hipcub::DeviceSelect::Flagged(nullptr, b, hipcub::CountingInputIterator<int64_t>(0),
                                        (const uint8_t*)nullptr, (int64_t*)nullptr,
                                        (int*)nullptr, (int)(n > 0 ? n : 1));
    c = a > b ? a : b;
    return c;
}

GroupWork carve(void* work, int64_t n) {
    GroupWork w;
    const int64_t nb = (n + (int64_t)kDmT * kOrdRows - 1) / ((int64_t)kDmT * kOrdRows);
    char* p = (char*)work;
    w.valid = (uint8_t*)p; p += align256((size_t)n);
    w.part = (Ord*)p; p += align256((size_t)(nb > 0 ? nb : 1) * sizeof(Ord));
    w.off = (BlockOff*)p; p += align256((size_t)(nb > 0 ? nb : 1) * sizeof(BlockOff));
    w.res = (long long*)p; p += 256;
    w.nsel = (int*)p; p += 256;
    w.ka = (uint64_t*)p; p += align256((size_t)n * 8);
    w.kb = (uint64_t*)p; p += align256((size_t)n * 8);
    w.va = (int64_t*)p; p += align256((size_t)n * 8);
    w.vb = (int64_t*)p; p += align256((size_t)n * 8);
    w.temp = p;
    w.temp_bytes = cub_temp_bytes(n);
    return w;
}

}  // namespace
}  // namespace sglm

using namespace sglm;

extern "C" size_t sglm_group_rows_work_bytes(int64_t n) {
    if (n < 0) n = 0;
    const int64_t nb = (n + (int64_t)kDmT * kOrdRows - 1) / ((int64_t)kDmT * kOrdRows);
    return align256((size_t)n) + align256((size_t)(nb > 0 ? nb : 1) * sizeof(Ord)) +
           align256((size_t)(nb > 0 ? nb : 1) * sizeof(BlockOff)) + 512 +
           4 * align256((size_t)n * 8) + cub_temp_bytes(n) + 256;
}

extern "C" int sglm_group_rows(const double* key, const double* key2, int64_t n, int64_t* perm,
                               int64_t* seg, int64_t* counts, int32_t* sorted_out, void* work,
                               sglm_stream_t stream) {
    if (n < 0 || !key || !perm || !seg || !counts || !work || n > (int64_t)0x7fffffff) {
        set_error("sglm_group_rows: bad args (n=%lld)", (long long)n);
        return SGLM_EINVAL;
    }
    hipStream_t s = as_stream(stream);
    if (n == 0) {
        if (hipMemsetAsync(counts, 0, 2 * sizeof(int64_t), s) != hipSuccess ||
            hipMemsetAsync(seg, 0, sizeof(int64_t), s) != hipSuccess) {
            set_error("sglm_group_rows: hipMemsetAsync failed");
            return SGLM_EHIP;
        }
        if (sorted_out) *sorted_out = 1;
        return SGLM_OK;
    }
    GroupWork w = carve(work, n);
    const int64_t nb = (n + (int64_t)kDmT * kOrdRows - 1) / ((int64_t)kDmT * kOrdRows);
    group_order_kernel<<<(unsigned)nb, kDmT, 0, s>>>(key, key2, n, w.valid, w.part);
    group_order_final_kernel<<<1, kDmT, 0, s>>>(w.part, nb, w.res, w.off);
    int st = check_launch("group_order_kernel");
    if (st) return st;
    long long res[3];
    if (hipMemcpyAsync(res, w.res, sizeof(res), hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess) {
        set_error("sglm_group_rows: readback failed");
        return SGLM_EHIP;
    }
    const int64_t m = res[1];
    if (sorted_out) *sorted_out = (int32_t)res[0];
    size_t tb = w.temp_bytes;
    if (res[0]) {
        // already grouped: the valid rows in row order and the group starts, one pass
        group_compact_kernel<<<(unsigned)nb, kDmT, 0, s>>>(key, key2, n, w.off, perm, seg);
        group_finish2_kernel<<<1, 1, 0, s>>>(seg, w.res, counts);
        return check_launch("group_compact_kernel");
    } else {
        // stable LSD radix sort: by key2 first (if any), then by key; NaN rows last
        const unsigned g = rows_grid(n);
        const int64_t* order = nullptr;
        int64_t* cur = w.vb;
        if (key2) {
            group_keys_kernel<<<g, kDmT, 0, s>>>(key, key2, nullptr, n, 1, w.ka, w.va);
            if (hipcub::DeviceRadixSort::SortPairs(w.temp, tb, w.ka, w.kb, w.va, w.vb, (int)n, 0,
                                                   64, s) != hipSuccess) {
                set_error("sglm_group_rows: SortPairs failed");
                return SGLM_EHIP;
            }
            order = w.vb;
            group_keys_kernel<<<g, kDmT, 0, s>>>(key, key2, order, n, 0, w.ka, nullptr);
            // values: the row ids in the key2 order
            if (hipMemcpyAsync(w.va, w.vb, (size_t)n * 8, hipMemcpyDeviceToDevice, s) !=
                hipSuccess) {
                set_error("sglm_group_rows: hipMemcpyAsync failed");
                return SGLM_EHIP;
            }
        } else {
            group_keys_kernel<<<g, kDmT, 0, s>>>(key, nullptr, nullptr, n, 0, w.ka, w.va);
        }
        tb = w.temp_bytes;
        if (hipcub::DeviceRadixSort::SortPairs(w.temp, tb, w.ka, w.kb, w.va, cur, (int)n, 0, 64,
                                               s) != hipSuccess) {
            set_error("sglm_group_rows: SortPairs failed");
            return SGLM_EHIP;
        }
        if (hipMemcpyAsync(perm, cur, (size_t)n * 8, hipMemcpyDeviceToDevice, s) != hipSuccess) {
            set_error("sglm_group_rows: hipMemcpyAsync failed");
            return SGLM_EHIP;
        }
    }
    if (m > 0) {
        group_heads_kernel<<<rows_grid(m), kDmT, 0, s>>>(key, key2, perm, m, w.valid);
        tb = w.temp_bytes;
        if (hipcub::DeviceSelect::Flagged(w.temp, tb, hipcub::CountingInputIterator<int64_t>(0),
                                          w.valid, seg, w.nsel, (int)m, s) != hipSuccess) {
            set_error("sglm_group_rows: DeviceSelect::Flagged failed");
            return SGLM_EHIP;
        }
    } else if (hipMemsetAsync(w.nsel, 0, sizeof(int), s) != hipSuccess) {
        set_error("sglm_group_rows: hipMemsetAsync failed");
        return SGLM_EHIP;
    }
    group_finish_kernel<<<1, 1, 0, s>>>(seg, w.nsel, m, counts);
    return check_launch("group_finish_kernel");
}

extern "C" int sglm_trial_lookup(const double* key, int64_t n, const double* tkeys, int64_t nt,
                                 int32_t* tidx, sglm_stream_t stream) {
    if (n <= 0) return SGLM_OK;
    if (!key || !tidx || (nt > 0 && !tkeys) || nt < 0) {
        set_error("sglm_trial_lookup: bad args");
        return SGLM_EINVAL;
    }
    trial_lookup_kernel<<<rows_grid(n), kDmT, 0, as_stream(stream)>>>(key, n, tkeys, nt, tidx);
    return check_launch("trial_lookup_kernel");
}

extern "C" int sglm_dm_heatmap(const double* clock, const double* cue, const double* cons,
                               const double* scons, int64_t n, const int64_t* perm,
                               const int64_t* seg, const int64_t* counts, const int32_t* tidx,
                               const double* tsel, double* out, int64_t ld_out,
                               sglm_stream_t stream) {
    if (n <= 0) return SGLM_OK;
    if (!clock || !cue || !cons || !scons || !perm || !seg || !counts || !out || ld_out < n ||
        (tidx && !tsel)) {
        set_error("sglm_dm_heatmap: bad args");
        return SGLM_EINVAL;
    }
    hipStream_t s = as_stream(stream);
    HmArgs a;
    a.clock = clock; a.cue = cue; a.cons = cons; a.scons = scons; a.tidx = tidx; a.tsel = tsel;
    a.off_sel = out; a.from_cue = out + ld_out; a.from_cons = out + 2 * ld_out;
    a.sel_cons = out + 3 * ld_out; a.off_cons = out + 4 * ld_out; a.n = n;
    hm_rows_kernel<<<rows_grid(n), kDmT, 0, s>>>(a);
    hm_groups_kernel<<<groups_grid(n), kDmT, 0, s>>>(a, perm, seg, counts);
    return check_launch("hm_groups_kernel");
}

extern "C" int sglm_dm_licks(const double* lick_src, int32_t from_spout,
                             const double* const* states, int32_t nstates, int64_t n,
                             double* const* out, double* lick_out, sglm_stream_t stream) {
    if (n <= 0) return SGLM_OK;
    if (!lick_src || nstates < 0 || nstates > kMaxCols || (nstates > 0 && (!states || !out))) {
        set_error("sglm_dm_licks: bad args (nstates=%d, max %d)", nstates, kMaxCols);
        return SGLM_EINVAL;
    }
    LickArgs a = {};
    a.lick_src = lick_src; a.from_spout = from_spout; a.ns = nstates; a.lick_out = lick_out;
    a.n = n;
    for (int c = 0; c < nstates; ++c) {
        if (!states[c] || !out[c]) {
            set_error("sglm_dm_licks: null column %d", c);
            return SGLM_EINVAL;
        }
        a.states[c] = states[c];
        a.out[c] = out[c];
    }
    licks_kernel<<<rows_grid(n), kDmT, 0, as_stream(stream)>>>(a);
    return check_launch("licks_kernel");
}

extern "C" int sglm_dm_counters(const double* enl, const double* cue, const double* senlp,
                                int64_t n, const int64_t* perm, const int64_t* seg,
                                const int64_t* counts, const int64_t* perm2,
                                const int64_t* seg2, const int64_t* counts2, double* tenl,
                                double* tenlp, double* cue_on, sglm_stream_t stream) {
    if (n <= 0) return SGLM_OK;
    if (!enl || !cue || !senlp || !perm || !seg || !counts || !perm2 || !seg2 || !counts2 ||
        !tenl || !tenlp) {
        set_error("sglm_dm_counters: bad args");
        return SGLM_EINVAL;
    }
    hipStream_t s = as_stream(stream);
    CntArgs a;
    a.enl = enl; a.cue = cue; a.senlp = senlp; a.tenl = tenl; a.tenlp = tenlp; a.cue_on = cue_on;
    a.n = n;
    counters_rows_kernel<<<rows_grid(n), kDmT, 0, s>>>(a);
    counters_enl_kernel<<<groups_grid(n), kDmT, 0, s>>>(a, perm, seg, counts);
    counters_enlp_kernel<<<groups_grid(n), kDmT, 0, s>>>(a, perm2, seg2, counts2);
    return check_launch("counters_enlp_kernel");
}

extern "C" int sglm_dm_pull(double* bout, int64_t n, const int64_t* perm, const int64_t* seg,
                            const int64_t* counts, const int32_t* nth, int32_t npull,
                            double* const* cols, sglm_stream_t stream) {
    if (n <= 0 || npull == 0) return SGLM_OK;
    if (!bout || !perm || !seg || !counts || !nth || !cols || npull < 0 || npull > kMaxPull) {
        set_error("sglm_dm_pull: bad args (npull=%d, max %d)", npull, kMaxPull);
        return SGLM_EINVAL;
    }
    PullArgs a = {};
    a.bout = bout; a.np = npull; a.n = n;
    for (int j = 0; j < npull; ++j) {
        if (!cols[j]) {
            set_error("sglm_dm_pull: null column %d", j);
            return SGLM_EINVAL;
        }
        a.col[j] = cols[j];
        a.nth[j] = nth[j];
    }
    hipStream_t s = as_stream(stream);
    pull_zero_kernel<<<rows_grid(n), kDmT, 0, s>>>(a);
    pull_groups_kernel<<<groups_grid(n), kDmT, 0, s>>>(a, perm, seg, counts);
    return check_launch("pull_groups_kernel");
}

extern "C" int sglm_trial_map(int64_t n, const int32_t* tidx, const double* src, int64_t ld_src,
                              const int32_t* src_cols, const double* vals, int64_t nt,
                              const int32_t* val_cols, int32_t ncols, double* dst,
                              int64_t ld_dst, const int32_t* dst_cols, sglm_stream_t stream) {
    if (n <= 0 || ncols <= 0) return SGLM_OK;
    if (!tidx || !src_cols || !val_cols || !dst || !dst_cols || ld_dst < n || nt < 0 ||
        (nt > 0 && !vals) || ncols > 65535) {
        set_error("sglm_trial_map: bad args");
        return SGLM_EINVAL;
    }
    trial_map_kernel<<<dim3(rows_grid(n), (unsigned)ncols), kDmT, 0, as_stream(stream)>>>(
        n, tidx, src, ld_src, src_cols, vals, nt, val_cols, dst, ld_dst, dst_cols);
    return check_launch("trial_map_kernel");
}

extern "C" int sglm_zero_groups_flag(int64_t n, const int64_t* perm, const int64_t* seg,
                                     const int64_t* counts, const double* src, int64_t ld,
                                     const int32_t* cols, int32_t ncols, double* flag,
                                     uint8_t* group_zero, sglm_stream_t stream) {
    if (n <= 0) return SGLM_OK;
    if (!perm || !seg || !counts || !flag || ncols < 0 || (ncols > 0 && (!src || !cols))) {
        set_error("sglm_zero_groups_flag: bad args");
        return SGLM_EINVAL;
    }
    zero_groups_flag_kernel<<<groups_grid(n), kDmT, 0, as_stream(stream)>>>(
        perm, seg, counts, src, ld, cols, ncols, flag, group_zero);
    return check_launch("zero_groups_flag_kernel");
}
