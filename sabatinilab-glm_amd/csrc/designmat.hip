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

// A tile of kOrdTile consecutive rows per workgroup, staged through LDS as key images with
// coalesced loads (all ones = a NaN key, never the image of a number); thread t then owns
// the 16 consecutive rows t*16 .. t*16+15 of the tile (padded LDS index: one slot per 16, so
// the 16-row strides of the 64 lanes spread over the banks).
constexpr int kOrdTile = kDmT * kOrdRows;
__device__ __forceinline__ int pad16(int p) { return p + (p >> 4); }

template <bool TWO>
struct TileKeys {
    uint64_t k1[kOrdTile + kOrdTile / 16];
    uint64_t k2[TWO ? kOrdTile + kOrdTile / 16 : 1];
    __device__ __forceinline__ uint64_t b(int p) const { return TWO ? k2[p] : 0ull; }
};

template <bool TWO>
__device__ __forceinline__ void load_tile(const double* __restrict__ key,
                                          const double* __restrict__ key2, int64_t n,
                                          int64_t t0, TileKeys<TWO>& sk) {
#pragma unroll 4
    for (int r = 0; r < kOrdRows; ++r) {
        const int p = r * kDmT + threadIdx.x;
        const int64_t i = t0 + p;
        uint64_t a = ~0ull, b = 0ull;
        if (i < n) {
            const double x = key[i];
            const double y = TWO ? key2[i] : 0.0;
            if (!isnan(x) && !isnan(y)) { a = key_bits(x); b = key_bits(y); }
        }
        sk.k1[pad16(p)] = a;
        if (TWO) sk.k2[pad16(p)] = b;
    }
    __syncthreads();
}

__device__ __forceinline__ Ord ord_shfl(const Ord& o, int src) {
    Ord r;
    r.f1 = __shfl(o.f1, src, 64); r.f2 = __shfl(o.f2, src, 64);
    r.l1 = __shfl(o.l1, src, 64); r.l2 = __shfl(o.l2, src, 64);
    r.cnt = __shfl(o.cnt, src, 64); r.heads = __shfl(o.heads, src, 64);
    r.ok = __shfl(o.ok, src, 64);
    return r;
}

// Per tile: is the valid-row key sequence non-decreasing (lexicographic in (key, key2)), how
// many valid rows, how many key changes.
template <bool TWO>
__global__ void __launch_bounds__(kDmT) group_order_kernel(const double* __restrict__ key,
                                                           const double* __restrict__ key2,
                                                           int64_t n, Ord* __restrict__ part) {
    __shared__ TileKeys<TWO> sk;
    __shared__ Ord sw[kDmT / 64];
    load_tile(key, key2, n, (int64_t)blockIdx.x * kOrdTile, sk);
    Ord o = {0, 0, 0, 0, 0, 0, 1};
    const int base = threadIdx.x * kOrdRows;
#pragma unroll
    for (int j = 0; j < kOrdRows; ++j) {
        const uint64_t a = sk.k1[pad16(base + j)], b = sk.b(pad16(base + j));
        if (a == ~0ull) continue;
        const Ord e = {a, b, a, b, 1, 1, 1};
        o = ord_comb(o, e);
    }
    // ordered combine over the wave (lane order), then the four waves
    const int lane = threadIdx.x & 63;
    for (int d = 1; d < 64; d <<= 1) {
        const Ord nb = ord_shfl(o, lane + d < 64 ? lane + d : lane);
        if ((lane & (2 * d - 1)) == 0 && lane + d < 64) o = ord_comb(o, nb);
    }
    if (lane == 0) sw[threadIdx.x >> 6] = o;
    __syncthreads();
    if (threadIdx.x == 0) {
        Ord r = sw[0];
        for (int w = 1; w < kDmT / 64; ++w) r = ord_comb(r, sw[w]);
        part[blockIdx.x] = r;
    }
}

// Over the tile summaries in order (one workgroup): the verdict (ordered?, valid rows,
// groups) and per tile the exclusive offsets of its valid rows and group heads in the
// compacted order and the last valid key before it (for the head test of its first valid
// row).  Each thread combines a run of consecutive tiles; an exclusive Hillis-Steele scan
// of the run summaries over the threads.
struct BlockOff { long long v, h; uint64_t p1, p2; int has; };

// state of the unordered-key path (rx_* kernels below), reset by group_order_final_kernel
constexpr int kRxTickets = 2 * 8 + 1;     // one per digit pass (two keys x 8), one for heads
struct RxState {
    unsigned long long or_[2], and_[2];   // [0]: key images, [1]: key2 images (every row)
    unsigned int nsel;                    // group heads found after the sort
    unsigned int ticket[kRxTickets];      // workgroups done with a pass's counts
};

constexpr int kFinT = 1024;
__global__ void __launch_bounds__(kFinT) group_order_final_kernel(const Ord* __restrict__ part,
                                                                  int64_t nb,
                                                                  long long* __restrict__ res,
                                                                  BlockOff* __restrict__ off,
                                                                  RxState* __restrict__ st) {
    __shared__ Ord sh[2][kFinT];
    const int tid = threadIdx.x;
    const int64_t per = (nb + kFinT - 1) / kFinT;
    const int64_t b0 = (int64_t)tid * per < nb ? (int64_t)tid * per : nb;
    const int64_t b1 = b0 + per < nb ? b0 + per : nb;
    Ord o = {0, 0, 0, 0, 0, 0, 1};
    for (int64_t b = b0; b < b1; ++b) o = ord_comb(o, part[b]);
    int cur = 0;
    sh[0][tid] = o;
    __syncthreads();
    for (int d = 1; d < kFinT; d <<= 1) {               // inclusive scan, double-buffered
        const Ord& mine = sh[cur][tid];
        sh[cur ^ 1][tid] = tid >= d ? ord_comb(sh[cur][tid - d], mine) : mine;
        cur ^= 1;
        __syncthreads();
    }
    if (tid == kFinT - 1) {
        const Ord& r = sh[cur][tid];
        res[0] = r.ok;
        res[1] = r.cnt;
        res[2] = r.heads;
        st->or_[0] = st->or_[1] = 0ull;
        st->and_[0] = st->and_[1] = ~0ull;
        st->nsel = 0;
        for (int q = 0; q < kRxTickets; ++q) st->ticket[q] = 0u;
    }
    Ord pre = {0, 0, 0, 0, 0, 0, 1};
    if (tid > 0) pre = sh[cur][tid - 1];
    for (int64_t b = b0; b < b1; ++b) {
        const Ord cb = part[b];
        BlockOff bo;
        bo.v = pre.cnt;
        bo.h = pre.heads;
        bo.has = pre.cnt > 0;
        bo.p1 = pre.l1;
        bo.p2 = pre.l2;
        off[b] = bo;
        pre = ord_comb(pre, cb);
    }
}

// Stable compaction of an ORDERED key sequence: perm = the valid rows in row order, seg = the
// positions in perm where the key changes (group starts).  Thread = 16 consecutive rows of
// the LDS tile, in-tile prefix counts and "last valid key before me" by Hillis-Steele passes;
// the tile's perm entries are assembled in LDS and written out coalesced.
template <bool TWO>
__global__ void __launch_bounds__(kDmT) group_compact_kernel(const double* __restrict__ key,
                                                             const double* __restrict__ key2,
                                                             int64_t n,
                                                             const long long* __restrict__ res,
                                                             const BlockOff* __restrict__ off,
                                                             int64_t* __restrict__ perm,
                                                             int64_t* __restrict__ seg) {
    if (!res[0]) return;                    // unordered keys: the radix path
    __shared__ TileKeys<TWO> sk;
    __shared__ int cv[kDmT], ch[kDmT], hv[kDmT];
    __shared__ uint64_t k1s[kDmT], k2s[kDmT];
    __shared__ uint16_t rowof[kOrdTile];
    const int tid = threadIdx.x;
    const int64_t t0 = (int64_t)blockIdx.x * kOrdTile;
    load_tile(key, key2, n, t0, sk);
    const BlockOff bo = off[blockIdx.x];
    const int base = tid * kOrdRows;
    uint32_t vm = 0;
    int nv = 0;
    uint64_t l1 = 0, l2 = 0;
#pragma unroll
    for (int j = 0; j < kOrdRows; ++j) {
        const uint64_t a = sk.k1[pad16(base + j)];
        if (a != ~0ull) {
            vm |= 1u << j;
            l1 = a;
            l2 = sk.b(pad16(base + j));
            ++nv;
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
    // exclusive: the values of thread tid - 1 (tile prefix for thread 0)
    int has_prev = tid > 0 ? hv[tid - 1] : 0;
    uint64_t p1 = tid > 0 ? k1s[tid - 1] : 0, p2 = tid > 0 ? k2s[tid - 1] : 0;
    if (!has_prev && bo.has) { has_prev = 1; p1 = bo.p1; p2 = bo.p2; }
    const int vpre = tid > 0 ? cv[tid - 1] : 0;
    const int tile_valid = cv[kDmT - 1];
    // heads of this thread's run
    int nh = 0;
    {
        int hp = has_prev;
        uint64_t q1 = p1, q2 = p2;
#pragma unroll
        for (int j = 0; j < kOrdRows; ++j) {
            if (vm >> j & 1u) {
                const uint64_t a = sk.k1[pad16(base + j)], b = sk.b(pad16(base + j));
                if (!hp || a != q1 || b != q2) ++nh;
                hp = 1; q1 = a; q2 = b;
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
    int lv = vpre;
    int64_t ph = bo.h + hpre;
    int hp = has_prev;
    uint64_t q1 = p1, q2 = p2;
#pragma unroll
    for (int j = 0; j < kOrdRows; ++j) {
        if (vm >> j & 1u) {
            const uint64_t a = sk.k1[pad16(base + j)], b = sk.b(pad16(base + j));
            if (!hp || a != q1 || b != q2) seg[ph++] = bo.v + lv;
            rowof[lv++] = (uint16_t)(base + j);
            hp = 1; q1 = a; q2 = b;
        }
    }
    __syncthreads();
    for (int q = tid; q < tile_valid; q += kDmT) perm[bo.v + q] = t0 + rowof[q];
}


// ---- unordered keys: a stable LSD radix sort on the device -------------------------------
// Every kernel of both paths is enqueued unconditionally; each reads the ordering verdict
// (res[0], written by group_order_final_kernel) and returns at once when its path is not the
// one taken, so the grouping never waits on the host.  Keys are order-preserving 64-bit images
// (all ones for a row with a NaN key, which sorts last); the sort visits only the 8-bit digits
// of the span of bits that vary over the rows (a device-side OR / AND of the images decides;
// the passes of a trial-id key are ~3 of 8, the rest return at once).  Two keys: the key2
// images first, then the key images regenerated in that order (stable, so lexicographic).
constexpr int kRxT = 256;             // threads per workgroup
constexpr int kRxR = 32;              // rows per thread
constexpr int kRxTile = kRxT * kRxR;  // rows per workgroup tile
constexpr int kRxPasses = 8;          // digit passes per 64-bit image (the maximum)

// passes of phase ph and the lowest varying bit; 0 passes when every image is the same
__device__ __forceinline__ int rx_npass(const RxState* st, int ph, int* lo) {
    const unsigned long long v = st->or_[ph] ^ st->and_[ph];
    if (!v) { *lo = 0; return 0; }
    *lo = __builtin_ctzll(v);
    const int hi = 63 - __builtin_clzll(v);
    return (hi - *lo) / 8 + 1;
}

// pass j of phase ph (1: key2 images, 0: key images): its global index g (the input buffer
// is g & 1) and digit shift; false when the pass has nothing to do
__device__ __forceinline__ bool rx_pass(const long long* res, const RxState* st, int two,
                                        int ph, int j, int* g, int* shift) {
    if (res[0]) return false;                        // ordered keys: the partition path
    int lo2 = 0, lo1 = 0;
    const int ja = two ? rx_npass(st, 1, &lo2) : 0;
    const int jb = rx_npass(st, 0, &lo1);
    if (ph == 1) {
        if (j >= ja) return false;
        *g = j;
        *shift = lo2 + 8 * j;
    } else {
        if (j >= jb) return false;
        *g = ja + j;
        *shift = lo1 + 8 * j;
    }
    return true;
}

__device__ __forceinline__ unsigned long long wave_or64(unsigned long long v) {
    for (int o = 32; o > 0; o >>= 1) v |= __shfl_xor(v, o, 64);
    return v;
}

__device__ __forceinline__ unsigned long long wave_and64(unsigned long long v) {
    for (int o = 32; o > 0; o >>= 1) v &= __shfl_xor(v, o, 64);
    return v;
}

// images of the first phase's key (key2 if two, else key) and row ids, plus the OR / AND of
// both images over all rows
__global__ void __launch_bounds__(kRxT) rx_prep_kernel(const double* __restrict__ key,
                                                       const double* __restrict__ key2,
                                                       int64_t n, const long long* __restrict__ res,
                                                       RxState* __restrict__ st,
                                                       unsigned long long* __restrict__ kout,
                                                       uint32_t* __restrict__ vout) {
    if (res[0]) return;
    __shared__ unsigned long long sh[4][kRxT / 64];
    unsigned long long o1 = 0, a1 = ~0ull, o2 = 0, a2 = ~0ull;
    const int64_t t0 = (int64_t)blockIdx.x * kRxTile;
    for (int r = 0; r < kRxR; ++r) {
        const int64_t q = t0 + (int64_t)r * kRxT + threadIdx.x;
        if (q >= n) break;
        const double a = key[q], b = key2 ? key2[q] : 0.0;
        const bool v = !isnan(a) && !isnan(b);
        const unsigned long long i1 = v ? key_bits(a) : ~0ull;
        const unsigned long long i2 = v ? key_bits(b) : ~0ull;
        o1 |= i1; a1 &= i1; o2 |= i2; a2 &= i2;
        kout[q] = key2 ? i2 : i1;
        vout[q] = (uint32_t)q;
    }
    o1 = wave_or64(o1); a1 = wave_and64(a1); o2 = wave_or64(o2); a2 = wave_and64(a2);
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) { sh[0][w] = o1; sh[1][w] = a1; sh[2][w] = o2; sh[3][w] = a2; }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int k = 1; k < kRxT / 64; ++k) {
            sh[0][0] |= sh[0][k]; sh[1][0] &= sh[1][k]; sh[2][0] |= sh[2][k]; sh[3][0] &= sh[3][k];
        }
        atomicOr(&st->or_[0], sh[0][0]);
        atomicAnd(&st->and_[0], sh[1][0]);
        atomicOr(&st->or_[1], sh[2][0]);
        atomicAnd(&st->and_[1], sh[3][0]);
    }
}

// Exclusive prefix of h[0 .. total) in place by one workgroup of kRxT threads (each thread a
// run of consecutive entries, a Hillis-Steele scan of the run sums); returns the total.
__device__ uint32_t block_exclusive_scan(uint32_t* __restrict__ h, int64_t total,
                                         uint32_t* __restrict__ sh) {
    const int tid = threadIdx.x;
    const int64_t per = (total + kRxT - 1) / kRxT;
    const int64_t b0 = (int64_t)tid * per < total ? (int64_t)tid * per : total;
    const int64_t b1 = b0 + per < total ? b0 + per : total;
    uint32_t s = 0;
    for (int64_t i = b0; i < b1; ++i) s += h[i];
    sh[tid] = s;
    __syncthreads();
    for (int o = 1; o < kRxT; o <<= 1) {
        const uint32_t v = tid >= o ? sh[tid - o] : 0u;
        __syncthreads();
        sh[tid] += v;
        __syncthreads();
    }
    const uint32_t all = sh[kRxT - 1];
    uint32_t run = tid ? sh[tid - 1] : 0u;
    for (int64_t i = b0; i < b1; ++i) {
        const uint32_t c = h[i];
        h[i] = run;
        run += c;
    }
    return all;
}

// The last workgroup to finish a counting pass (a ticket per pass) scans the counts for the
// next kernel, so a pass needs no separate scan launch.  Every workgroup publishes its counts
// before taking its ticket (release); the last one fences before reading them (acquire).
__device__ __forceinline__ bool last_block(unsigned int* ticket) {
    __shared__ int last;
    __threadfence();
    __syncthreads();
    if (threadIdx.x == 0) last = atomicAdd(ticket, 1u) == gridDim.x - 1;
    __syncthreads();
    if (last) __threadfence();
    return last;
}

// per tile: the count of each digit value, digit-major (hist[d * nblk + tile]); the last tile
// turns them into the first output position of each (digit, tile)
__global__ void __launch_bounds__(kRxT) rx_hist_kernel(const long long* __restrict__ res,
                                                       RxState* __restrict__ st, int two,
                                                       int ph, int j,
                                                       const unsigned long long* __restrict__ k0,
                                                       const unsigned long long* __restrict__ k1,
                                                       int64_t n, uint32_t* __restrict__ hist,
                                                       int64_t nblk) {
    int g, shift;
    if (!rx_pass(res, st, two, ph, j, &g, &shift)) return;
    __shared__ uint32_t cnt[256];
    const unsigned long long* keys = (g & 1) ? k1 : k0;
    cnt[threadIdx.x] = 0;
    __syncthreads();
    const int64_t t0 = (int64_t)blockIdx.x * kRxTile;
    for (int r = 0; r < kRxR; ++r) {
        const int64_t q = t0 + (int64_t)r * kRxT + threadIdx.x;
        if (q >= n) break;
        atomicAdd(&cnt[(unsigned)(keys[q] >> shift) & 255u], 1u);
    }
    __syncthreads();
    hist[(int64_t)threadIdx.x * nblk + blockIdx.x] = cnt[threadIdx.x];
    if (last_block(&st->ticket[g])) block_exclusive_scan(hist, 256 * nblk, cnt);
}

__device__ __forceinline__ uint64_t lanemask_lt64(int lane) {
    return lane == 0 ? 0ull : (~0ull >> (64 - lane));
}

// stable scatter of one digit pass: rounds of 256 consecutive rows in order; a row's rank
// among the earlier rows of its digit = the running count of the tile's earlier rounds + the
// counts of the earlier waves of this round + its rank among the matching lanes of its wave
// (eight ballots on the digit bits)
__global__ void __launch_bounds__(kRxT) rx_scatter_kernel(
    const long long* __restrict__ res, const RxState* __restrict__ st, int two, int ph, int j,
    unsigned long long* __restrict__ k0, unsigned long long* __restrict__ k1,
    uint32_t* __restrict__ v0, uint32_t* __restrict__ v1, int64_t n,
    const uint32_t* __restrict__ hist, int64_t nblk) {
    int g, shift;
    if (!rx_pass(res, st, two, ph, j, &g, &shift)) return;
    __shared__ uint32_t base[256];
    __shared__ uint32_t wc[kRxT / 64][256];
    const unsigned long long* kin = (g & 1) ? k1 : k0;
    unsigned long long* kout = (g & 1) ? k0 : k1;
    const uint32_t* vin = (g & 1) ? v1 : v0;
    uint32_t* vout = (g & 1) ? v0 : v1;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    base[tid] = hist[(int64_t)tid * nblk + blockIdx.x];
#pragma unroll
    for (int k = 0; k < kRxT / 64; ++k) wc[k][tid] = 0;
    __syncthreads();
    const int64_t t0 = (int64_t)blockIdx.x * kRxTile;
    for (int r = 0; r < kRxR; ++r) {
        if (t0 + (int64_t)r * kRxT >= n) break;                  // uniform over the block
        const int64_t q = t0 + (int64_t)r * kRxT + tid;
        const bool valid = q < n;
        const unsigned long long key = valid ? kin[q] : 0ull;
        const uint32_t val = valid ? vin[q] : 0u;
        const unsigned d = (unsigned)(key >> shift) & 255u;
        uint64_t peers = __ballot(valid);
#pragma unroll
        for (int b = 0; b < 8; ++b) {
            const uint64_t m = __ballot((d >> b) & 1u);
            peers &= ((d >> b) & 1u) ? m : ~m;
        }
        const int rank = __popcll(peers & lanemask_lt64(lane));
        if (valid && rank == 0) wc[w][d] = (uint32_t)__popcll(peers);
        __syncthreads();
        if (valid) {
            uint32_t pos = base[d] + (uint32_t)rank;
            for (int k = 0; k < w; ++k) pos += wc[k][d];
            kout[pos] = key;
            vout[pos] = val;
        }
        __syncthreads();
        uint32_t add = 0;
#pragma unroll
        for (int k = 0; k < kRxT / 64; ++k) {
            add += wc[k][tid];
            wc[k][tid] = 0;
        }
        base[tid] += add;
        __syncthreads();
    }
}

// two keys: after the key2 passes, the key images in the sorted order (in place)
__global__ void __launch_bounds__(kRxT) rx_regen_kernel(const double* __restrict__ key,
                                                        const double* __restrict__ key2,
                                                        int64_t n, const long long* __restrict__ res,
                                                        const RxState* __restrict__ st,
                                                        unsigned long long* __restrict__ k0,
                                                        unsigned long long* __restrict__ k1,
                                                        const uint32_t* __restrict__ v0,
                                                        const uint32_t* __restrict__ v1) {
    if (res[0]) return;
    int lo;
    const int cur = rx_npass(st, 1, &lo) & 1;
    unsigned long long* kc = cur ? k1 : k0;
    const uint32_t* vc = cur ? v1 : v0;
    const int64_t q = (int64_t)blockIdx.x * kRxT + threadIdx.x;
    if (q >= n) return;
    const uint32_t i = vc[q];
    const double a = key[i], b = key2[i];
    kc[q] = (!isnan(a) && !isnan(b)) ? key_bits(a) : ~0ull;
}

__device__ __forceinline__ const uint32_t* rx_final_vals(const RxState* st, int two,
                                                         const uint32_t* v0, const uint32_t* v1) {
    int lo;
    const int jt = (two ? rx_npass(st, 1, &lo) : 0) + rx_npass(st, 0, &lo);
    return (jt & 1) ? v1 : v0;
}

__device__ __forceinline__ bool same_key(const double* key, const double* key2, int64_t i,
                                         int64_t j) {
    return key_bits(key[i]) == key_bits(key[j]) &&
           (!key2 || key_bits(key2[i]) == key_bits(key2[j]));
}

// the sorted row ids into perm (int64), group heads flagged (thread = 32 consecutive
// positions) and counted per tile
__global__ void __launch_bounds__(kRxT) rx_heads_count_kernel(
    const double* __restrict__ key, const double* __restrict__ key2, int64_t n,
    const long long* __restrict__ res, RxState* __restrict__ st,
    const uint32_t* __restrict__ v0, const uint32_t* __restrict__ v1,
    int64_t* __restrict__ perm, uint8_t* __restrict__ head, uint32_t* __restrict__ hc) {
    if (res[0]) return;
    __shared__ uint32_t sh[kRxT / 64];
    const uint32_t* vals = rx_final_vals(st, key2 != nullptr, v0, v1);
    const int64_t m = res[1];
    // row ids: coalesced copy of the tile
    const int64_t t0 = (int64_t)blockIdx.x * kRxTile;
    for (int r = 0; r < kRxR; ++r) {
        const int64_t q = t0 + (int64_t)r * kRxT + threadIdx.x;
        if (q < n) perm[q] = vals[q];
    }
    uint32_t c = 0;
    const int64_t q0 = t0 + (int64_t)threadIdx.x * kRxR;
    for (int e = 0; e < kRxR; ++e) {
        const int64_t q = q0 + e;
        if (q >= m) break;
        const bool h = q == 0 || !same_key(key, key2, vals[q], vals[q - 1]);
        head[q] = h;
        c += h;
    }
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t = 0;
        for (int k = 0; k < kRxT / 64; ++k) t += sh[k];
        hc[blockIdx.x] = t;
    }
    __shared__ uint32_t scr[kRxT];
    if (last_block(&st->ticket[kRxTickets - 1])) {
        const uint32_t all = block_exclusive_scan(hc, gridDim.x, scr);
        if (threadIdx.x == 0) st->nsel = all;
    }
}

// segment starts: the flagged positions in order (tile offsets from rx_scan over hc)
__global__ void __launch_bounds__(kRxT) rx_heads_write_kernel(int64_t n,
                                                              const long long* __restrict__ res,
                                                              const uint8_t* __restrict__ head,
                                                              const uint32_t* __restrict__ hc,
                                                              int64_t* __restrict__ seg) {
    if (res[0]) return;
    __shared__ uint32_t sc[kRxT];
    const int64_t m = res[1];
    const int tid = threadIdx.x;
    const int64_t q0 = (int64_t)blockIdx.x * kRxTile + (int64_t)tid * kRxR;
    uint32_t c = 0;
    for (int e = 0; e < kRxR; ++e) {
        const int64_t q = q0 + e;
        if (q >= m) break;
        c += head[q];
    }
    sc[tid] = c;
    __syncthreads();
    for (int o = 1; o < kRxT; o <<= 1) {
        const uint32_t v = tid >= o ? sc[tid - o] : 0u;
        __syncthreads();
        sc[tid] += v;
        __syncthreads();
    }
    int64_t pos = (int64_t)hc[blockIdx.x] + (tid ? sc[tid - 1] : 0u);
    for (int e = 0; e < kRxR; ++e) {
        const int64_t q = q0 + e;
        if (q >= m) break;
        if (head[q]) seg[pos++] = q;
    }
}

// counts = {m, nseg, ordered} and the closing segment bound, for whichever path ran
__global__ void group_finish_kernel(int64_t* __restrict__ seg, const long long* __restrict__ res,
                                    const RxState* __restrict__ st,
                                    int64_t* __restrict__ counts) {
    const long long m = res[1];
    const long long g = res[0] ? res[2] : (long long)st->nsel;
    seg[g] = m;
    counts[0] = m;
    counts[1] = g;
    counts[2] = res[0] ? 1 : 0;
}

__global__ void group_empty_kernel(int64_t* __restrict__ seg, int64_t* __restrict__ counts) {
    seg[0] = 0;
    counts[0] = 0;
    counts[1] = 0;
    counts[2] = 1;
}

// ---- per-group walks --------------------------------------------------------------------
// wave w of the grid handles groups w, w + W, ... (W waves in the grid)
#define DM_FOR_GROUPS(counts)                                                                   \
    const int lane = threadIdx.x & 63;                                                          \
    const int64_t nseg_ = (counts)[1];                                                          \
    const bool ident_ = perm_ident(counts, n_);                                                 \
    for (int64_t s = (int64_t)blockIdx.x * (kDmT / 64) + (threadIdx.x >> 6); s < nseg_;         \
         s += (int64_t)gridDim.x * (kDmT / 64))

__device__ __forceinline__ double wave_sum_d(double v) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// The perm range of one group.  A group whose rows are consecutive in the session (the usual
// case: an ordered trial count without NaN keys inside a trial) is read without the perm
// indirection, which takes a dependent load off every slab.
struct GSpan { int64_t q0, q1, base; bool contig; };

// ident: every row is grouped and the keys were ordered (counts = {n, *, 1}), so perm is the
// identity and no perm entry is read at all
__device__ __forceinline__ bool perm_ident(const int64_t* __restrict__ counts, int64_t n) {
    return counts[2] != 0 && counts[0] == n;
}

__device__ __forceinline__ GSpan gspan(const int64_t* __restrict__ perm,
                                       const int64_t* __restrict__ seg, int64_t s,
                                       bool ident) {
    GSpan g;
    g.q0 = seg[s];
    g.q1 = seg[s + 1];
    if (ident) {
        g.base = g.q0;
        g.contig = true;
        return g;
    }
    const int64_t a = perm[g.q0], b = perm[g.q1 - 1];
    g.base = a;
    g.contig = (b - a) == (g.q1 - 1 - g.q0);        // strictly increasing rows: contiguous
    return g;
}

__device__ __forceinline__ int64_t grow(const GSpan& g, const int64_t* __restrict__ perm,
                                        int64_t q) {
    return g.contig ? g.base + (q - g.q0) : perm[q];
}

constexpr int kSlabs = 2;                   // 64-row slabs whose loads are issued together

struct HmArgs {
    const double *clock, *cue, *cons, *scons;
    const int32_t* tidx;
    const double* tsel;
    double *off_sel, *from_cue, *from_cons, *sel_cons, *off_cons;
    const double* key;                      // when given, the rows kernel writes NaN-key rows only
    int64_t n;
};

// add_heatmap_columns (pp_design_mat.py:108-126), rows outside every group (NaN nTrial): the
// maps give NaN
__global__ void __launch_bounds__(kDmT) hm_rows_kernel(HmArgs a) {
    const int64_t i = (int64_t)blockIdx.x * kDmT + threadIdx.x;
    if (i >= a.n) return;
    if (a.key && !isnan(a.key[i])) return;          // a group row: the group walk writes it
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
    const int64_t n_ = a.n;
    DM_FOR_GROUPS(counts) {
        const GSpan g = gspan(perm, seg, s, ident_);
        // a group of at most 64 * kSlabs rows (the usual trial) is held in registers from the
        // first pass: the second pass reloads nothing but the mapped selection time
        const bool small = g.q1 - g.q0 <= 64 * kSlabs;
        double fcue = NAN, fcons = NAN, sc = 0.0, ssc = 0.0;
        bool got_cue = false, got_cons = false;
        double ck0[kSlabs];
        int64_t ii0[kSlabs];
        int32_t tv0[kSlabs];
        for (int64_t b = g.q0; b < g.q1; b += 64 * kSlabs) {
            double ck[kSlabs], cu[kSlabs], co[kSlabs], scv[kSlabs];
#pragma unroll
            for (int h = 0; h < kSlabs; ++h) {
                const int64_t q = b + 64 * h + lane;
                const bool v = q < g.q1;
                const int64_t i = v ? grow(g, perm, q) : -1;
                ck[h] = v ? a.clock[i] : NAN;
                cu[h] = v ? a.cue[i] : 0.0;
                co[h] = v ? a.cons[i] : 0.0;
                scv[h] = v ? a.scons[i] : 0.0;
                ck0[h] = ck[h];
                ii0[h] = i;
                tv0[h] = (small && v && a.tidx) ? a.tidx[i] : -1;
            }
#pragma unroll
            for (int h = 0; h < kSlabs; ++h) {
                const uint64_t mc = __ballot(cu[h] == 1.0 && !isnan(ck[h]));
                if (!got_cue && mc) {
                    fcue = __shfl(ck[h], __ffsll((long long)mc) - 1, 64);
                    got_cue = true;
                }
                const uint64_t mo = __ballot(co[h] == 1.0 && !isnan(ck[h]));
                if (!got_cons && mo) {
                    fcons = __shfl(ck[h], __ffsll((long long)mo) - 1, 64);
                    got_cons = true;
                }
                sc += isnan(co[h]) ? 0.0 : co[h];
                ssc += isnan(scv[h]) ? 0.0 : scv[h];
            }
        }
        const double stc = (wave_sum_d(ssc) - wave_sum_d(sc)) * (1000.0 / 50.0);
        if (small) {
#pragma unroll
            for (int h = 0; h < kSlabs; ++h) {
                const int64_t i = ii0[h];
                if (i < 0) continue;
                const double off = tv0[h] >= 0 ? a.tsel[tv0[h]] : NAN;
                a.from_cue[i] = ck0[h] - fcue;
                a.from_cons[i] = ck0[h] - fcons;
                a.sel_cons[i] = stc;
                a.off_sel[i] = off;
                a.off_cons[i] = stc + off;
            }
            continue;
        }
        for (int64_t b = g.q0; b < g.q1; b += 64 * kSlabs) {
#pragma unroll
            for (int h = 0; h < kSlabs; ++h) {
                const int64_t q = b + 64 * h + lane;
                if (q >= g.q1) break;
                const int64_t i = grow(g, perm, q);
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
    const double *key, *key2;          // when given, the rows kernel writes NaN-key rows only
    int64_t n;
};

// rows outside the groups: the counter of a row that meets the condition is NaN (cumcount of
// a NaN-key row), 0 otherwise; no cue onset.  Rows inside a group are written by the walks.
__global__ void __launch_bounds__(kDmT) counters_rows_kernel(CntArgs a) {
    const int64_t i = (int64_t)blockIdx.x * kDmT + threadIdx.x;
    if (i >= a.n) return;
    const bool out1 = !a.key || isnan(a.key[i]);                   // outside the nTrial groups
    const bool out2 = out1 || !a.key2 || isnan(a.key2[i]);         // outside (nTrial, nENL)
    if (out1) {
        const bool pe = a.enl[i] == 1.0 || a.cue[i] == 1.0;
        a.tenl[i] = pe ? NAN : 0.0;
        if (a.cue_on) a.cue_on[i] = 0.0;
    }
    if (out2) a.tenlp[i] = a.senlp[i] == 1.0 ? NAN : 0.0;
}

// time_from_enl_onset = cumcount**2 / (50*100) over the (ENL == 1 | Cue == 1) rows of each
// nTrial group (:171), 0 on the group's other rows; the cue column: 1 on the first Cue == 1
// row of each group (:175, 183), 0 on the others
__global__ void __launch_bounds__(kDmT) counters_enl_kernel(CntArgs a,
                                                            const int64_t* __restrict__ perm,
                                                            const int64_t* __restrict__ seg,
                                                            const int64_t* __restrict__ counts) {
    const int64_t n_ = a.n;
    DM_FOR_GROUPS(counts) {
        const GSpan g = gspan(perm, seg, s, ident_);
        long long c = 0;
        bool onset = false;
        for (int64_t b = g.q0; b < g.q1; b += 64 * kSlabs) {
            int64_t ii[kSlabs];
            double cu[kSlabs], en[kSlabs];
#pragma unroll
            for (int h = 0; h < kSlabs; ++h) {
                const int64_t q = b + 64 * h + lane;
                const bool v = q < g.q1;
                ii[h] = v ? grow(g, perm, q) : -1;
                cu[h] = v ? a.cue[ii[h]] : 0.0;
                en[h] = v ? a.enl[ii[h]] : 0.0;
            }
#pragma unroll
            for (int h = 0; h < kSlabs; ++h) {
                const bool v = ii[h] >= 0;
                const bool cuh = v && cu[h] == 1.0;
                const bool pe = v && (cuh || en[h] == 1.0);
                const uint64_t m = __ballot(pe);
                const long long k = c + __popcll(m & lanemask_lt(lane));
                if (v) a.tenl[ii[h]] = pe ? (double)(k * k) / 5000.0 : 0.0;
                c += __popcll(m);
                const uint64_t mc = __ballot(cuh);
                if (a.cue_on && v)
                    a.cue_on[ii[h]] = (!onset && mc && lane == __ffsll((long long)mc) - 1) ? 1.0
                                                                                           : 0.0;
                if (mc) onset = true;
            }
        }
    }
}

// time_from_enlp_onset = cumcount**2 / (50*100) over the state_ENLP == 1 rows of each
// (nTrial, nENL) group (:172), 0 on the group's other rows
__global__ void __launch_bounds__(kDmT) counters_enlp_kernel(CntArgs a,
                                                             const int64_t* __restrict__ perm,
                                                             const int64_t* __restrict__ seg,
                                                             const int64_t* __restrict__ counts) {
    const int64_t n_ = a.n;
    DM_FOR_GROUPS(counts) {
        const GSpan g = gspan(perm, seg, s, ident_);
        long long c = 0;
        for (int64_t b = g.q0; b < g.q1; b += 64 * kSlabs) {
            int64_t ii[kSlabs];
            double se[kSlabs];
#pragma unroll
            for (int h = 0; h < kSlabs; ++h) {
                const int64_t q = b + 64 * h + lane;
                const bool v = q < g.q1;
                ii[h] = v ? grow(g, perm, q) : -1;
                se[h] = v ? a.senlp[ii[h]] : 0.0;
            }
#pragma unroll
            for (int h = 0; h < kSlabs; ++h) {
                const bool v = ii[h] >= 0;
                const bool p = v && se[h] == 1.0;
                const uint64_t m = __ballot(p);
                const long long k = c + __popcll(m & lanemask_lt(lane));
                if (v) a.tenlp[ii[h]] = p ? (double)(k * k) / 5000.0 : 0.0;
                c += __popcll(m);
            }
        }
    }
}

constexpr int kMaxPull = 16;

struct PullArgs {
    double* bout;
    double* col[kMaxPull];
    int nth[kMaxPull];
    int np;
    const double* key;                 // when given, the zero kernel writes NaN-key rows only
    int64_t n;
};

__global__ void __launch_bounds__(kDmT) pull_zero_kernel(PullArgs a) {
    const int64_t i = (int64_t)blockIdx.x * kDmT + threadIdx.x;
    if (i >= a.n) return;
    if (a.key && !isnan(a.key[i])) return;          // a group row: the group walk writes it
    for (int j = 0; j < a.np; ++j) a.col[j][i] = 0.0;
}

// pull_lick_from_bout (:44-53): for each position in processing order, the nth (nth - 1 >= 0
// from the start, < 0 from the end) bout == 1 row of each group moves to its column (the
// column is reset first, as `t_[new_col] = 0` does), and the bout row is zeroed
__global__ void __launch_bounds__(kDmT) pull_groups_kernel(PullArgs a,
                                                           const int64_t* __restrict__ perm,
                                                           const int64_t* __restrict__ seg,
                                                           const int64_t* __restrict__ counts) {
    const int64_t n_ = a.n;
    DM_FOR_GROUPS(counts) {
        const GSpan g = gspan(perm, seg, s, ident_);
        for (int j = 0; j < a.np; ++j) {
            const long long k = a.nth[j] - 1;
            double* col = a.col[j];
            long long total = 0;
            if (k < 0) {
                for (int64_t b = g.q0; b < g.q1; b += 64) {
                    const int64_t q = b + lane;
                    total += __popcll(__ballot(q < g.q1 && a.bout[grow(g, perm, q)] == 1.0));
                }
            }
            const long long target = k >= 0 ? k : total + k;
            long long c = 0;
            for (int64_t b = g.q0; b < g.q1; b += 64 * kSlabs) {
                int64_t ii[kSlabs];
                double bv[kSlabs];
#pragma unroll
                for (int h = 0; h < kSlabs; ++h) {
                    const int64_t q = b + 64 * h + lane;
                    const bool v = q < g.q1;
                    ii[h] = v ? grow(g, perm, q) : -1;
                    bv[h] = v ? a.bout[ii[h]] : 0.0;
                }
#pragma unroll
                for (int h = 0; h < kSlabs; ++h) {
                    const bool v = ii[h] >= 0;
                    const bool l = v && bv[h] == 1.0;
                    const uint64_t m = __ballot(l);
                    const bool pick = l && c + __popcll(m & lanemask_lt(lane)) == target;
                    if (v) col[ii[h]] = pick ? 1.0 : 0.0;
                    if (pick) a.bout[ii[h]] = 0.0;
                    c += __popcll(m);
                }
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
        // consecutive trial ids (a running trial count): the position is the offset
        const double off = k - tkeys[0];
        if (off >= 0.0 && off < (double)nt && off == floor(off) && tkeys[(int64_t)off] == k) {
            tidx[i] = (int32_t)off;
            return;
        }
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
constexpr int kMapCols = 8;                 // destination columns per thread (tidx read once)
template <typename TV>
__global__ void __launch_bounds__(kDmT) trial_map_kernel(int64_t n,
                                                         const int32_t* __restrict__ tidx,
                                                         const double* __restrict__ src,
                                                         int64_t ld_src,
                                                         const int32_t* __restrict__ src_cols,
                                                         const TV* __restrict__ vals,
                                                         int64_t nt,
                                                         const int32_t* __restrict__ val_cols,
                                                         int32_t ncols,
                                                         double* __restrict__ dst, int64_t ld_dst,
                                                         const int32_t* __restrict__ dst_cols) {
    const int64_t i = (int64_t)blockIdx.x * kDmT + threadIdx.x;
    if (i >= n) return;
    const int c0 = blockIdx.y * kMapCols;
    const int c1 = c0 + kMapCols < ncols ? c0 + kMapCols : ncols;
    const int32_t t = tidx[i];
    for (int c = c0; c < c1; ++c) {
        const int32_t sc = src_cols[c];
        const double x = sc < 0 ? 1.0 : src[(int64_t)sc * ld_src + i];
        const double v = t >= 0 ? (double)vals[(int64_t)val_cols[c] * nt + t] : NAN;
        dst[(int64_t)dst_cols[c] * ld_dst + i] = x * v;
    }
}

// trials whose rows sum to 0 over the listed columns (groupby sum, skipna, then the row sum,
// :198-203): flag = 1 on all their rows
constexpr int kZeroCols = 8;                // columns summed in registers per slab
__global__ void __launch_bounds__(kDmT) zero_groups_flag_kernel(int64_t n_,
                                                                const int64_t* __restrict__ perm,
                                                                const int64_t* __restrict__ seg,
                                                                const int64_t* __restrict__ counts,
                                                                const double* __restrict__ src,
                                                                int64_t ld,
                                                                const int32_t* __restrict__ cols,
                                                                int32_t ncols,
                                                                double* __restrict__ flag,
                                                                uint8_t* __restrict__ gz) {
    DM_FOR_GROUPS(counts) {
        const GSpan g = gspan(perm, seg, s, ident_);
        double tot = 0.0;
        for (int c0 = 0; c0 < ncols; c0 += kZeroCols) {
            // every listed column of a slab loaded together; per column the lane sums run
            // over the slabs in order, then the wave sum, columns added in order
            double acc[kZeroCols];
#pragma unroll
            for (int c = 0; c < kZeroCols; ++c) acc[c] = 0.0;
            for (int64_t b = g.q0; b < g.q1; b += 64 * kSlabs) {
#pragma unroll
                for (int h = 0; h < kSlabs; ++h) {
                    const int64_t q = b + 64 * h + lane;
                    const bool v = q < g.q1;
                    const int64_t i = v ? grow(g, perm, q) : 0;
#pragma unroll
                    for (int c = 0; c < kZeroCols; ++c) {
                        if (c0 + c < ncols) {
                            const double x = v ? src[(int64_t)cols[c0 + c] * ld + i] : 0.0;
                            acc[c] += isnan(x) ? 0.0 : x;
                        }
                    }
                }
            }
#pragma unroll
            for (int c = 0; c < kZeroCols; ++c)
                if (c0 + c < ncols) tot += wave_sum_d(acc[c]);
        }
        if (gz && lane == 0) gz[s] = tot == 0.0;
        if (tot == 0.0)
            for (int64_t b = g.q0; b < g.q1; b += 64) {
                const int64_t q = b + lane;
                if (q < g.q1) flag[grow(g, perm, q)] = 1.0;
            }
    }
}

inline unsigned rows_grid(int64_t n) { return (unsigned)((n + kDmT - 1) / kDmT); }

// groups are walked by a fixed grid of waves (the group count lives on the device)
// (a group walk is latency-bound: enough waves that each walks only a few groups)
inline unsigned groups_grid(int64_t n) {
    int64_t g = (n + 8 * kDmT - 1) / (8 * kDmT);
    if (g < 64) g = 64;
    if (g > 4096) g = 4096;
    return (unsigned)g;
}

struct GroupWork {
    Ord* part;
    BlockOff* off;
    long long* res;
    RxState* st;
    uint8_t* head;
    unsigned long long* k[2];
    uint32_t* v[2];
    uint32_t* hist;
    uint32_t* hc;
};

size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

int64_t order_blocks(int64_t n) {
    const int64_t nb = (n + (int64_t)kDmT * kOrdRows - 1) / ((int64_t)kDmT * kOrdRows);
    return nb > 0 ? nb : 1;
}

int64_t rx_blocks(int64_t n) {
    const int64_t nb = (n + kRxTile - 1) / kRxTile;
    return nb > 0 ? nb : 1;
}

// carve the scratch (or, with work == nullptr, return its size through *bytes)
GroupWork carve(void* work, int64_t n, size_t* bytes) {
    GroupWork w = {};
    const int64_t nb = order_blocks(n), nr = rx_blocks(n);
    const size_t nn = (size_t)(n > 0 ? n : 1);
    char* p = (char*)work;
    size_t o = 0;
    auto take = [&](size_t sz) { char* q = p ? p + o : nullptr; o += align256(sz); return q; };
    w.part = (Ord*)take((size_t)nb * sizeof(Ord));
    w.off = (BlockOff*)take((size_t)nb * sizeof(BlockOff));
    w.res = (long long*)take(8 * sizeof(long long));
    w.st = (RxState*)take(sizeof(RxState));
    w.head = (uint8_t*)take(nn);
    w.k[0] = (unsigned long long*)take(nn * 8);
    w.k[1] = (unsigned long long*)take(nn * 8);
    w.v[0] = (uint32_t*)take(nn * 4);
    w.v[1] = (uint32_t*)take(nn * 4);
    w.hist = (uint32_t*)take((size_t)256 * nr * 4);
    w.hc = (uint32_t*)take((size_t)nr * 4);
    if (bytes) *bytes = o;
    return w;
}

}  // namespace
}  // namespace sglm

using namespace sglm;

extern "C" size_t sglm_group_rows_work_bytes(int64_t n) {
    size_t b = 0;
    carve(nullptr, n < 0 ? 0 : n, &b);
    return b;
}

// Ordered keys (the session's running trial count): one ordering pass, its verdict and block
// offsets, and a stable compaction.  Unordered keys: the rx_* radix passes.  Both paths are
// enqueued and the device takes one (no host round trip); *sorted_out, when asked for, costs
// a stream synchronisation.
extern "C" int sglm_group_rows(const double* key, const double* key2, int64_t n, int64_t* perm,
                               int64_t* seg, int64_t* counts, int32_t* sorted_out, void* work,
                               sglm_stream_t stream) {
    if (n < 0 || !key || !perm || !seg || !counts || !work || n > (int64_t)0x7fffffff) {
        set_error("sglm_group_rows: bad args (n=%lld)", (long long)n);
        return SGLM_EINVAL;
    }
    hipStream_t s = as_stream(stream);
    if (n == 0) {
        group_empty_kernel<<<1, 1, 0, s>>>(seg, counts);
        if (sorted_out) *sorted_out = 1;
        return check_launch("group_empty_kernel");
    }
    GroupWork w = carve(work, n, nullptr);
    const int64_t nb = order_blocks(n), nr = rx_blocks(n);
    const int two = key2 != nullptr;
    if (two) {
        group_order_kernel<true><<<(unsigned)nb, kDmT, 0, s>>>(key, key2, n, w.part);
    } else {
        group_order_kernel<false><<<(unsigned)nb, kDmT, 0, s>>>(key, key2, n, w.part);
    }
    group_order_final_kernel<<<1, kFinT, 0, s>>>(w.part, nb, w.res, w.off, w.st);
    if (two) {
        group_compact_kernel<true><<<(unsigned)nb, kDmT, 0, s>>>(key, key2, n, w.res, w.off,
                                                                 perm, seg);
    } else {
        group_compact_kernel<false><<<(unsigned)nb, kDmT, 0, s>>>(key, key2, n, w.res, w.off,
                                                                  perm, seg);
    }
    // the radix path: key2 images first (two keys), then the key images
    rx_prep_kernel<<<(unsigned)nr, kRxT, 0, s>>>(key, key2, n, w.res, w.st, w.k[0], w.v[0]);
    for (int ph = two; ph >= 0; --ph) {
        if (ph == 0 && two)
            rx_regen_kernel<<<rows_grid(n), kRxT, 0, s>>>(key, key2, n, w.res, w.st, w.k[0],
                                                          w.k[1], w.v[0], w.v[1]);
        for (int j = 0; j < kRxPasses; ++j) {
            rx_hist_kernel<<<(unsigned)nr, kRxT, 0, s>>>(w.res, w.st, two, ph, j, w.k[0], w.k[1],
                                                         n, w.hist, nr);
            rx_scatter_kernel<<<(unsigned)nr, kRxT, 0, s>>>(w.res, w.st, two, ph, j, w.k[0],
                                                            w.k[1], w.v[0], w.v[1], n, w.hist,
                                                            nr);
        }
    }
    rx_heads_count_kernel<<<(unsigned)nr, kRxT, 0, s>>>(key, key2, n, w.res, w.st, w.v[0],
                                                        w.v[1], perm, w.head, w.hc);
    rx_heads_write_kernel<<<(unsigned)nr, kRxT, 0, s>>>(n, w.res, w.head, w.hc, seg);
    group_finish_kernel<<<1, 1, 0, s>>>(seg, w.res, w.st, counts);
    int st = check_launch("group_finish_kernel");
    if (st) return st;
    if (sorted_out) {
        long long ok = 0;
        if (hipMemcpyAsync(&ok, w.res, sizeof(ok), hipMemcpyDeviceToHost, s) != hipSuccess ||
            hipStreamSynchronize(s) != hipSuccess) {
            set_error("sglm_group_rows: readback failed");
            return SGLM_EHIP;
        }
        *sorted_out = (int32_t)ok;
    }
    return SGLM_OK;
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
    return sglm_dm_heatmap_k(clock, cue, cons, scons, nullptr, n, perm, seg, counts, tidx, tsel,
                             out, ld_out, stream);
}

extern "C" int sglm_dm_heatmap_k(const double* clock, const double* cue, const double* cons,
                                 const double* scons, const double* key, int64_t n,
                                 const int64_t* perm, const int64_t* seg, const int64_t* counts,
                                 const int32_t* tidx, const double* tsel, double* out,
                                 int64_t ld_out, sglm_stream_t stream) {
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
    a.sel_cons = out + 3 * ld_out; a.off_cons = out + 4 * ld_out; a.key = key; a.n = n;
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
    return sglm_dm_counters_k(enl, cue, senlp, nullptr, nullptr, n, perm, seg, counts, perm2,
                              seg2, counts2, tenl, tenlp, cue_on, stream);
}

extern "C" int sglm_dm_counters_k(const double* enl, const double* cue, const double* senlp,
                                  const double* key, const double* key2, int64_t n,
                                  const int64_t* perm, const int64_t* seg, const int64_t* counts,
                                  const int64_t* perm2, const int64_t* seg2,
                                  const int64_t* counts2, double* tenl, double* tenlp,
                                  double* cue_on, sglm_stream_t stream) {
    if (n <= 0) return SGLM_OK;
    if (!enl || !cue || !senlp || !perm || !seg || !counts || !perm2 || !seg2 || !counts2 ||
        !tenl || !tenlp) {
        set_error("sglm_dm_counters: bad args");
        return SGLM_EINVAL;
    }
    hipStream_t s = as_stream(stream);
    CntArgs a;
    a.enl = enl; a.cue = cue; a.senlp = senlp; a.tenl = tenl; a.tenlp = tenlp; a.cue_on = cue_on;
    a.key = key; a.key2 = key ? key2 : nullptr; a.n = n;
    counters_rows_kernel<<<rows_grid(n), kDmT, 0, s>>>(a);
    counters_enl_kernel<<<groups_grid(n), kDmT, 0, s>>>(a, perm, seg, counts);
    counters_enlp_kernel<<<groups_grid(n), kDmT, 0, s>>>(a, perm2, seg2, counts2);
    return check_launch("counters_enlp_kernel");
}

extern "C" int sglm_dm_pull(double* bout, int64_t n, const int64_t* perm, const int64_t* seg,
                            const int64_t* counts, const int32_t* nth, int32_t npull,
                            double* const* cols, sglm_stream_t stream) {
    return sglm_dm_pull_k(bout, nullptr, n, perm, seg, counts, nth, npull, cols, stream);
}

extern "C" int sglm_dm_pull_k(double* bout, const double* key, int64_t n, const int64_t* perm,
                              const int64_t* seg, const int64_t* counts, const int32_t* nth,
                              int32_t npull, double* const* cols, sglm_stream_t stream) {
    if (n <= 0 || npull == 0) return SGLM_OK;
    if (!bout || !perm || !seg || !counts || !nth || !cols || npull < 0 || npull > kMaxPull) {
        set_error("sglm_dm_pull: bad args (npull=%d, max %d)", npull, kMaxPull);
        return SGLM_EINVAL;
    }
    PullArgs a = {};
    a.bout = bout; a.np = npull; a.key = key; a.n = n;
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

template <typename TV>
static int trial_map_launch(int64_t n, const int32_t* tidx, const double* src, int64_t ld_src,
                            const int32_t* src_cols, const TV* vals, int64_t nt,
                            const int32_t* val_cols, int32_t ncols, double* dst, int64_t ld_dst,
                            const int32_t* dst_cols, sglm_stream_t stream) {
    if (n <= 0 || ncols <= 0) return SGLM_OK;
    if (!tidx || !src_cols || !val_cols || !dst || !dst_cols || ld_dst < n || nt < 0 ||
        (nt > 0 && !vals) || ncols > 65535 * kMapCols) {
        set_error("sglm_trial_map: bad args");
        return SGLM_EINVAL;
    }
    trial_map_kernel<TV><<<dim3(rows_grid(n), (unsigned)((ncols + kMapCols - 1) / kMapCols)),
                           kDmT, 0, as_stream(stream)>>>(n, tidx, src, ld_src, src_cols, vals,
                                                         nt, val_cols, ncols, dst, ld_dst,
                                                         dst_cols);
    return check_launch("trial_map_kernel");
}

extern "C" int sglm_trial_map(int64_t n, const int32_t* tidx, const double* src, int64_t ld_src,
                              const int32_t* src_cols, const double* vals, int64_t nt,
                              const int32_t* val_cols, int32_t ncols, double* dst,
                              int64_t ld_dst, const int32_t* dst_cols, sglm_stream_t stream) {
    return trial_map_launch(n, tidx, src, ld_src, src_cols, vals, nt, val_cols, ncols, dst,
                            ld_dst, dst_cols, stream);
}

extern "C" int sglm_trial_map_u8(int64_t n, const int32_t* tidx, const double* src,
                                 int64_t ld_src, const int32_t* src_cols, const uint8_t* vals,
                                 int64_t nt, const int32_t* val_cols, int32_t ncols, double* dst,
                                 int64_t ld_dst, const int32_t* dst_cols, sglm_stream_t stream) {
    return trial_map_launch(n, tidx, src, ld_src, src_cols, vals, nt, val_cols, ncols, dst,
                            ld_dst, dst_cols, stream);
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
        n, perm, seg, counts, src, ld, cols, ncols, flag, group_zero);
    return check_launch("zero_groups_flag_kernel");
}
