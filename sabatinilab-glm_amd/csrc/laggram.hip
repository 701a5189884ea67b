// Gram of a time-shifted 0/1 event design at a constant weight, from the event occurrences.
//
// Column (b, a) of the design is event a of the base matrix E shifted by s_b rows,
// X[t, (b, a)] = E[t + row0 - s_b, a] for design rows t < n (sglm_ez.timeshift_cols,
// backend/sglm_ez.py:102-123).  At a fit's intercept-only start every row of an all-rows mask
// has the same weight w (eta is constant there), so its Hessian is w X^T X, and
//     (X^T X)[(b1, a1), (b2, a2)] = #{u in occ(a1) : u in window(s1), u + s1 - s2 in occ(a2)}
// with window(s) = [row0 - s, row0 - s + n).  An occurrence u of the interior range
// [row0 - smin, row0 + n - smax) lies in every shift's window, so over the interior the count
// depends on the lag difference d = s1 - s2 only: one cross-correlation histogram per event
// pair (a1, a2) over d in [smin - smax, smax - smin] (lag_corr_kernel, ~nnz(E) * span bit
// tests per event pair instead of n * p^2 MFMA work); the few occurrences near the two ends
// of the design are added per (s1, s2) when the Gram is written (lag_gram_fill_kernel).  The
// intercept column counts each column's occurrences in its window; padding columns are 0.
// Counts are exact integers; H = bf16(w) * count in f32 (the MFMA Gram uses the same
// bf16-rounded weight and sums the same products in f32).
#include "common.h"

namespace sglm {
namespace {

constexpr int kLgT = 256;
constexpr int kLgMaxBins = 4097;           // lag span <= 2048

struct LagGramArgs {
    const int32_t* occ;        // occurrence rows of every event, event-major, ascending
    const int32_t* ev_off;     // [m + 1] segment offsets into occ
    const uint32_t* ebits;     // [m][nwords] occurrence bitmap, bit v & 31 of word v >> 5
    const int32_t* shifts;     // [K]
    int64_t nwords, row0, n, n_raw;
    int32_t m, K, layout, P, smin, smax;
    int32_t pc;                // intercept column (m * K, or later when continuous columns
                               // sit between the lag columns and it: they are written as 0)
};

__device__ __forceinline__ int lower_bound_i32(const int32_t* a, int lo, int hi, int64_t x) {
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if ((int64_t)a[mid] < x) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

__device__ __forceinline__ bool ebit(const LagGramArgs& A, int a, int64_t v) {
    if (v < 0 || v >= A.n_raw) return false;
    return (A.ebits[(int64_t)a * A.nwords + (v >> 5)] >> (v & 31)) & 1u;
}

// hist[a1][a2][d - dmin] over the interior occurrences u of a1: #{u : u + d in occ(a2)}
__global__ void __launch_bounds__(kLgT) lag_corr_kernel(LagGramArgs A, int32_t* __restrict__ hist,
                                                        int32_t* __restrict__ bnd) {
    extern __shared__ int32_t h[];
    const int a1 = blockIdx.x, a2 = blockIdx.y, tid = threadIdx.x;
    const int dmin = A.smin - A.smax, nb = 2 * (A.smax - A.smin) + 1;
    for (int j = tid; j < nb; j += kLgT) h[j] = 0;
    const int64_t ulo = A.row0 - A.smin;
    const int64_t uhi = A.row0 + A.n - A.smax > ulo ? A.row0 + A.n - A.smax : ulo;
    const int s0 = A.ev_off[a1], s1 = A.ev_off[a1 + 1];
    __shared__ int rng[2];
    if (tid == 0) {
        rng[0] = lower_bound_i32(A.occ, s0, s1, ulo);
        rng[1] = lower_bound_i32(A.occ, s0, s1, uhi);
        if (a2 == 0) {
            // boundary occurrences of a1: [row0 - smax, ulo) and [uhi, row0 + n - smin)
            int32_t* bq = bnd + 4 * a1;
            bq[0] = lower_bound_i32(A.occ, s0, s1, A.row0 - A.smax);
            bq[1] = rng[0];
            bq[2] = rng[1];
            bq[3] = lower_bound_i32(A.occ, s0, s1, A.row0 + A.n - A.smin);
        }
    }
    __syncthreads();
    const uint32_t* eb = A.ebits + (int64_t)a2 * A.nwords;
    for (int i = rng[0] + tid; i < rng[1]; i += kLgT) {
        const int64_t u = A.occ[i];
        int64_t lo = u + dmin, hi = u - dmin;              // inclusive lag window of a2 rows
        if (lo < 0) lo = 0;
        if (hi > A.n_raw - 1) hi = A.n_raw - 1;
        for (int64_t w = lo >> 5; w <= (hi >> 5); ++w) {
            uint32_t word = eb[w];
            const int64_t wb = w << 5;
            if (wb < lo) word &= ~0u << (lo - wb);
            if (wb + 31 > hi) word &= ~0u >> (wb + 31 - hi);
            while (word) {
                const int b = __builtin_ctz(word);
                word &= word - 1;
                atomicAdd(&h[(int)(wb + b - u) - dmin], 1);
            }
        }
    }
    __syncthreads();
    int32_t* out = hist + ((int64_t)a1 * A.m + a2) * nb;
    for (int j = tid; j < nb; j += kLgT) out[j] = h[j];
}

__device__ __forceinline__ void col_of(const LagGramArgs& A, int c, int& b, int& a) {
    if (A.layout == 0) { b = c / A.m; a = c - b * A.m; }
    else { a = c / A.K; b = c - a * A.K; }
}

// the (b1, a1) x (b2, a2) entry's count: interior histogram + boundary occurrences of a1
__device__ int pair_count(const LagGramArgs& A, const int32_t* hist, const int32_t* bnd, int b1,
                          int a1, int b2, int a2) {
    const int sa = A.shifts[b1], sb = A.shifts[b2];
    const int d = sa - sb, dmin = A.smin - A.smax, nb = 2 * (A.smax - A.smin) + 1;
    int cnt = hist[((int64_t)a1 * A.m + a2) * nb + (d - dmin)];
    const int64_t wlo = A.row0 - sa, whi = A.row0 - sa + A.n;     // window(s1)
    const int32_t* bq = bnd + 4 * a1;
#pragma unroll
    for (int r = 0; r < 2; ++r)
        for (int i = bq[2 * r]; i < bq[2 * r + 1]; ++i) {
            const int64_t u = A.occ[i];
            if (u >= wlo && u < whi && ebit(A, a2, u + d)) ++cnt;
        }
    return cnt;
}

// eight rows of one 128 x 128 block (I <= J) of the upper triangle per workgroup (blockIdx.y =
// the row chunk: ~2k workgroups, so the dependent lookups of many entries overlap), for every
// fit of the list
__global__ void __launch_bounds__(kLgT) lag_gram_fill_kernel(LagGramArgs A,
                                                             const int32_t* __restrict__ hist,
                                                             const int32_t* __restrict__ bnd,
                                                             const float* __restrict__ W,
                                                             int64_t ldw,
                                                             const int32_t* __restrict__ fits,
                                                             int32_t nfits, float* __restrict__ H) {
    int t = blockIdx.x, I = 0;
    {
        int rowlen = A.P / 128;
        while (t >= rowlen) { t -= rowlen; ++I; --rowlen; }
    }
    const int J = I + t;
    const int p = A.pc, pl = A.m * A.K;     // intercept column; lag columns 0 .. pl
    const int tid = threadIdx.x;
    const int jc = J * 128 + (tid & 127);
    int bj = 0, aj = 0;
    if (jc < pl) col_of(A, jc, bj, aj);
    // the intercept column's count for row ic: occurrences of ic's event in its window
    for (int r = 8 * blockIdx.y + (tid >> 7); r < 8 * blockIdx.y + 8; r += kLgT / 128) {
        const int ic = I * 128 + r;
        float cnt;
        if (ic > p || jc > p || (ic >= pl && ic < p) || (jc >= pl && jc < p)) {
            cnt = 0.0f;
        } else if (ic == p && jc == p) {
            cnt = (float)A.n;
        } else if (jc == p || ic == p) {
            int b, a;
            col_of(A, jc == p ? ic : jc, b, a);
            const int64_t wlo = A.row0 - A.shifts[b];
            const int s0 = A.ev_off[a], s1 = A.ev_off[a + 1];
            cnt = (float)(lower_bound_i32(A.occ, s0, s1, wlo + A.n) -
                          lower_bound_i32(A.occ, s0, s1, wlo));
        } else {
            int bi, ai;
            col_of(A, ic, bi, ai);
            cnt = (float)pair_count(A, hist, bnd, bi, ai, bj, aj);
        }
        for (int q = 0; q < nfits; ++q) {
            const int f = fits[q];
            const float w = (float)(__bf16)W[(int64_t)f * ldw];
            H[((int64_t)f * A.P + ic) * A.P + jc] = w * cnt;
        }
    }
}

}  // namespace
}  // namespace sglm

using namespace sglm;

extern "C" {

size_t sglm_lag_gram_work_bytes(int32_t m, int32_t smin, int32_t smax) {
    const int64_t nb = 2 * ((int64_t)smax - smin) + 1;
    return (size_t)((int64_t)m * m * nb + 4 * (int64_t)m) * sizeof(int32_t);
}

int sglm_lag_gram(const int32_t* occ, const int32_t* ev_off, const uint32_t* ebits,
                  int64_t nwords, const int32_t* shifts, int32_t m, int32_t K, int32_t layout,
                  int32_t smin, int32_t smax, int64_t row0, int64_t n, int64_t n_raw, int32_t P,
                  const float* W, int64_t ldw, const int32_t* fits, int32_t nfits, float* H,
                  void* work, sglm_stream_t stream) {
    return sglm_lag_gram_pc(occ, ev_off, ebits, nwords, shifts, m, K, layout, smin, smax, row0, n,
                            n_raw, P, m * K, W, ldw, fits, nfits, H, work, stream);
}

int sglm_lag_gram_pc(const int32_t* occ, const int32_t* ev_off, const uint32_t* ebits,
                     int64_t nwords, const int32_t* shifts, int32_t m, int32_t K, int32_t layout,
                     int32_t smin, int32_t smax, int64_t row0, int64_t n, int64_t n_raw,
                     int32_t P, int32_t pc, const float* W, int64_t ldw, const int32_t* fits,
                     int32_t nfits, float* H, void* work, sglm_stream_t stream) {
    if (nfits <= 0) return SGLM_OK;
    const int64_t nb = 2 * ((int64_t)smax - smin) + 1;
    if (!occ || !ev_off || !ebits || !shifts || !W || !fits || !H || !work || m <= 0 || K <= 0 ||
        smax < smin || nb > kLgMaxBins || P % 128 || pc < m * K || pc + 1 > P || n <= 0 ||
        n_raw <= 0 || nwords * 32 < n_raw || (layout != 0 && layout != 1)) {
        set_error("sglm_lag_gram: bad args (m=%d K=%d P=%d span=%d)", m, K, P, smax - smin);
        return SGLM_EINVAL;
    }
    hipStream_t s = as_stream(stream);
    LagGramArgs A{occ, ev_off, ebits, shifts, nwords, row0, n, n_raw, m, K, layout, P, smin, smax,
                  pc};
    int32_t* hist = reinterpret_cast<int32_t*>(work);
    int32_t* bnd = hist + (int64_t)m * m * nb;
    lag_corr_kernel<<<dim3((unsigned)m, (unsigned)m), kLgT, (size_t)nb * sizeof(int32_t), s>>>(
        A, hist, bnd);
    int st = check_launch("lag_corr_kernel");
    if (st) return st;
    const int nb128 = P / 128;
    lag_gram_fill_kernel<<<dim3((unsigned)(nb128 * (nb128 + 1) / 2), 16), kLgT, 0, s>>>(
        A, hist, bnd, W, ldw, fits, nfits, H);
    return check_launch("lag_gram_fill_kernel");
}

}  // extern "C"
