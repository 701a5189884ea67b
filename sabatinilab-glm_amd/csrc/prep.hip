// Session preprocessing (lynne_pp.preprocess_lynne, lynne_pp.py:217-249) on the GPU: the trial
// segmentation, reward flags, port-event indicators and first-time events of a behaviour
// session, as row-parallel kernels plus chunked scans (cumulative sums, segmented per-trial
// sums, forward/backward fills).  All columns are float64 struct-of-arrays (one contiguous
// column per variable, the layout of a pandas float block), so every kernel streams whole
// columns with coalesced loads.
#include "common.h"
#include <math.h>

namespace sglm {
namespace {

constexpr int kPT = 256;          // threads per scan workgroup (4 waves)
constexpr int kPJ = 32;           // 64-row slabs per wave
constexpr int kPW = 64 * kPJ;     // consecutive rows per wave (the scan unit)
constexpr int kCT1 = 1024;        // carry-scan workgroup

enum { OP_ADD = 0, OP_MAX = 1 };

// Scan element over NC columns at once: values plus a "segment starts here" bit (shared by
// the columns: they are segmented by the same key).  ADD with heads is the segmented sum (a
// head resets the running values), MAX ignores heads.  The operator is associative but not
// commutative, so every combination below keeps row order.
template <int NC> struct Agg { double v[NC]; int h; };

template <int OP, int NC> __device__ __forceinline__ Agg<NC> ident() {
    Agg<NC> a;
#pragma unroll
    for (int c = 0; c < NC; ++c) a.v[c] = OP == OP_MAX ? -INFINITY : 0.0;
    a.h = 0;
    return a;
}
template <int OP, int NC> __device__ __forceinline__ Agg<NC> comb(const Agg<NC>& a,
                                                                  const Agg<NC>& b) {
    Agg<NC> r;
#pragma unroll
    for (int c = 0; c < NC; ++c)
        r.v[c] = OP == OP_MAX ? fmax(a.v[c], b.v[c]) : (b.h ? b.v[c] : a.v[c] + b.v[c]);
    r.h = OP == OP_MAX ? 0 : (a.h | b.h);
    return r;
}
template <int NC> __device__ __forceinline__ Agg<NC> shfl_up(const Agg<NC>& a, int o) {
    Agg<NC> r;
#pragma unroll
    for (int c = 0; c < NC; ++c) r.v[c] = __shfl_up(a.v[c], o, 64);
    r.h = __shfl_up(a.h, o, 64);
    return r;
}
template <int NC> __device__ __forceinline__ Agg<NC> shfl(const Agg<NC>& a, int l) {
    Agg<NC> r;
#pragma unroll
    for (int c = 0; c < NC; ++c) r.v[c] = __shfl(a.v[c], l, 64);
    r.h = __shfl(a.h, l, 64);
    return r;
}
template <int OP, int NC> __device__ __forceinline__ Agg<NC> wave_incl(Agg<NC> a) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const Agg<NC> t = shfl_up(a, o);
        if (lane >= o) a = comb<OP, NC>(t, a);
    }
    return a;
}

struct ScanCols {
    const double* x[3];    // inputs (NC used)
    double* y[3];          // outputs (may alias x)
    const double* key;     // segment key or nullptr
    int64_t n;
    int rev;
    int keep;              // NC == 1: rows with a NaN VALUE get the running total (rows with a
                           // NaN key stay NaN) -- the per-trial totals need it
};

// Logical row i is physical row rev ? n-1-i : i.  NaN values contribute the identity and stay
// NaN in the output (pandas' skipna cumsum); with a key, rows whose key is NaN are NaN (the
// groupby drops them) and a row is a segment head when its key differs from the previous
// logical row's.
template <int OP, int NC>
__device__ __forceinline__ Agg<NC> load_elem(const ScanCols& a, int64_t i, bool& nan_out) {
    const int64_t p = a.rev ? a.n - 1 - i : i;
    Agg<NC> e;
    e.h = 0;
    bool kn = false;
    if (a.key) {
        const double kp = a.key[p];
        kn = isnan(kp);
        e.h = (i == 0) || (kp != a.key[a.rev ? p + 1 : p - 1]);
    }
    nan_out = kn;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        const double v = a.x[c][p];
        const bool nn = kn || isnan(v);
        e.v[c] = nn ? (OP == OP_MAX ? -INFINITY : 0.0) : v;
        nan_out = nan_out || (NC == 1 && nn);
    }
    return e;
}

// The scan unit is one wave: wave g owns rows [g*kPW, (g+1)*kPW) as kPJ slabs of 64
// consecutive rows (lane = row within the slab: every load is coalesced), slabs chained in
// order.  Pass 1 writes each wave's aggregate, one workgroup turns them into exclusive carries,
// pass 2 rescans with the carry and writes -- no LDS, no barriers, few registers.
template <int OP, int NC>
__global__ void __launch_bounds__(kPT) scan_reduce_kernel(ScanCols a, Agg<NC>* agg) {
    const int lane = threadIdx.x & 63;
    const int64_t g = (int64_t)blockIdx.x * (kPT / 64) + (threadIdx.x >> 6);
    const int64_t base = g * kPW + lane;
    if (g * kPW >= a.n) return;
    Agg<NC> run = ident<OP, NC>();
#pragma unroll 8
    for (int j = 0; j < kPJ; ++j) {
        const int64_t i = base + j * 64;
        bool nanr;
        const Agg<NC> e = i < a.n ? load_elem<OP, NC>(a, i, nanr) : ident<OP, NC>();
        run = comb<OP, NC>(run, shfl(wave_incl<OP, NC>(e), 63));
    }
    if (lane == 0) agg[g] = run;
}

// One workgroup turns the wave aggregates into exclusive carries, in place: thread t owns a
// contiguous run of entries, the runs are chained in order across the workgroup.
template <int OP, int NC>
__global__ void __launch_bounds__(kCT1) scan_carry_kernel(Agg<NC>* agg, int64_t nchunks) {
    __shared__ Agg<NC> lds[kCT1 / 64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t per = (nchunks + kCT1 - 1) / kCT1;
    const int64_t c0 = (int64_t)threadIdx.x * per;
    const int64_t c1 = c0 + per < nchunks ? c0 + per : nchunks;
    // loads in groups of 8 issued together (independent), combined in order afterwards
    constexpr int G = 8;
    Agg<NC> a = ident<OP, NC>();
    for (int64_t c = c0; c < c1; c += G) {
        Agg<NC> v[G];
#pragma unroll
        for (int q = 0; q < G; ++q) v[q] = c + q < c1 ? agg[c + q] : ident<OP, NC>();
#pragma unroll
        for (int q = 0; q < G; ++q) a = comb<OP, NC>(a, v[q]);
    }
    const Agg<NC> inc = wave_incl<OP, NC>(a);
    Agg<NC> exc = shfl_up(inc, 1);
    if (lane == 0) exc = ident<OP, NC>();
    if (lane == 63) lds[w] = inc;
    __syncthreads();
    Agg<NC> wp = ident<OP, NC>();
    for (int v = 0; v < w; ++v) wp = comb<OP, NC>(wp, lds[v]);
    Agg<NC> run = comb<OP, NC>(wp, exc);
    for (int64_t c = c0; c < c1; c += G) {
        Agg<NC> v[G];
#pragma unroll
        for (int q = 0; q < G; ++q) v[q] = c + q < c1 ? agg[c + q] : ident<OP, NC>();
#pragma unroll
        for (int q = 0; q < G; ++q) {
            if (c + q < c1) agg[c + q] = run;
            run = comb<OP, NC>(run, v[q]);
        }
    }
}

template <int OP, int NC>
__global__ void __launch_bounds__(kPT) scan_apply_kernel(ScanCols a,
                                                         const Agg<NC>* __restrict__ carry) {
    const int lane = threadIdx.x & 63;
    const int64_t g = (int64_t)blockIdx.x * (kPT / 64) + (threadIdx.x >> 6);
    const int64_t base = g * kPW + lane;
    if (g * kPW >= a.n) return;
    Agg<NC> run = carry[g];
#pragma unroll 8
    for (int j = 0; j < kPJ; ++j) {
        const int64_t i = base + j * 64;
        bool nanr = true;
        const Agg<NC> e = i < a.n ? load_elem<OP, NC>(a, i, nanr) : ident<OP, NC>();
        const Agg<NC> inc = wave_incl<OP, NC>(e);
        if (i < a.n) {
            const Agg<NC> r = comb<OP, NC>(run, inc);
            const int64_t p = a.rev ? a.n - 1 - i : i;
            const bool kn = a.key && isnan(a.key[p]);
#pragma unroll
            for (int c = 0; c < NC; ++c) {
                const double v = NC == 1 ? ((nanr && !(a.keep && !kn)) ? NAN : r.v[c])
                                         : ((kn || isnan(a.x[c][p])) ? NAN : r.v[c]);
                a.y[c][p] = v;
            }
        }
        run = comb<OP, NC>(run, shfl(inc, 63));
    }
}

inline int64_t nwaves_of(int64_t n) { return (n + kPW - 1) / kPW; }

// Inclusive scans of NC columns (in place allowed): ADD (pandas cumsum, skipna; segmented by
// `key` when given) or MAX, forward or backward.
template <int OP, int NC>
int scan(const ScanCols& a, void* agg, hipStream_t s) {
    const int64_t nw = nwaves_of(a.n);
    const int64_t nb = (nw + kPT / 64 - 1) / (kPT / 64);
    scan_reduce_kernel<OP, NC><<<nb, kPT, 0, s>>>(a, (Agg<NC>*)agg);
    scan_carry_kernel<OP, NC><<<1, kCT1, 0, s>>>((Agg<NC>*)agg, nw);
    scan_apply_kernel<OP, NC><<<nb, kPT, 0, s>>>(a, (const Agg<NC>*)agg);
    return check_launch("prep scan");
}

ScanCols cols1(const double* x, double* y, const double* key, int64_t n, int rev,
               int keep = 0) {
    ScanCols a = {};
    a.x[0] = x; a.y[0] = y; a.key = key; a.n = n; a.rev = rev; a.keep = keep;
    return a;
}

// ---- row kernels (one thread per row) ---------------------------------------------------
struct In {   // input columns (SGLM_PREP_IN_* order)
    const double *cpn, *lpx, *rpx, *lpn, *rpn, *r, *nr, *rl, *ll;
};

__device__ __forceinline__ bool present(double v) { return v != 0.0 && !isnan(v); }

// x.replace(0, nan) * f  (lynne_pp.py:29-31)
__device__ __forceinline__ double code(double v, double f) { return present(v) ? v * f : NAN; }

// event_col before its backward fill: cpn*1 combine_first lpx*2 combine_first rpx*2
// (lynne_pp.py:29-33); T1 = -row where present (a backward MAX scan then gives -(next row)).
__global__ void prep_codes_kernel(In in, int64_t n, double* __restrict__ ev_raw,
                                  double* __restrict__ nxt) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    double e = code(in.cpn[t], 1.0);
    if (isnan(e)) e = code(in.lpx[t], 2.0);
    if (isnan(e)) e = code(in.rpx[t], 2.0);
    ev_raw[t] = e;
    nxt[t] = isnan(e) ? -INFINITY : -(double)t;
}

__device__ __forceinline__ double ev_at(const double* ev_raw, const double* nxt, int64_t t) {
    const double j = nxt[t];
    return j == -INFINITY ? NAN : ev_raw[(int64_t)(-j)];
}

// event_col = bfill; trial start = (ev == 1) & (ev.shift(-1) != 1), shifted by -k rows
// (lynne_pp.py:34-35).  Rows whose shifted source falls outside the session are NaN.
__global__ void prep_start_kernel(const double* __restrict__ ev_raw,
                                  const double* __restrict__ nxt, int64_t n, int32_t k,
                                  double* __restrict__ event_col, double* __restrict__ flag) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    event_col[t] = ev_at(ev_raw, nxt, t);
    const int64_t u = t + k;
    double f = NAN;
    if (u >= 0 && u < n) {
        const bool c = ev_at(ev_raw, nxt, u) == 1.0 &&
                       !(u + 1 < n && ev_at(ev_raw, nxt, u + 1) == 1.0);
        f = c ? 1.0 : 0.0;
    }
    flag[t] = f;
}

// event_col_end before its forward fill: lpx*2 combine_first rpx*2 combine_first
// trial_start_flag.replace(0, nan) (lynne_pp.py:39); T1 = row where present.
__global__ void prep_end_codes_kernel(In in, const double* __restrict__ flag, int64_t n,
                                      double* __restrict__ ece_raw, double* __restrict__ prv) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    double e = code(in.lpx[t], 2.0);
    if (isnan(e)) e = code(in.rpx[t], 2.0);
    if (isnan(e)) e = code(flag[t], 1.0);
    ece_raw[t] = e;
    prv[t] = isnan(e) ? -INFINITY : (double)t;
}

__device__ __forceinline__ double ece_at(const double* ece_raw, const double* prv, int64_t t) {
    const double j = prv[t];
    return j == -INFINITY ? NAN : ece_raw[(int64_t)j];
}

// event_col_end = ffill; trial end = (ece == 2) & (ece.shift(1) != 2) & (nTrial > 0), shifted
// by +k rows (lynne_pp.py:40-41).
__global__ void prep_end_kernel(const double* __restrict__ ece_raw,
                                const double* __restrict__ prv,
                                const double* __restrict__ ntrial, int64_t n, int32_t k,
                                double* __restrict__ event_col_end,
                                double* __restrict__ end_flag) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    event_col_end[t] = ece_at(ece_raw, prv, t);
    const int64_t u = t - k;
    double f = NAN;
    if (u >= 0 && u < n) {
        const bool c = ece_at(ece_raw, prv, u) == 2.0 &&
                       !(u >= 1 && ece_at(ece_raw, prv, u - 1) == 2.0) && ntrial[u] > 0.0;
        f = c ? 1.0 : 0.0;
    }
    end_flag[t] = f;
}

struct Out {  // output columns (SGLM_PREP_OUT_* order)
    double* c[SGLM_PREP_NOUT];
};

// Reward flags (per-trial sum of r = forward + backward segmented sums - r, NaN r counted as 0
// as groupby().transform(sum) skips it; the scans carry their running totals through NaN-r
// rows), port indicators,
// side-agnostic sums, nn / xx (lynne_pp.py:121-123, 142-151, 170-178, 193-194).
__global__ void prep_rows_kernel(In in, const double* __restrict__ ntrial, int64_t n, Out o,
                                 const double* __restrict__ s0, const double* __restrict__ s1) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    const double r = in.r[t], nr = in.nr[t];
    const double rpx = in.rpx[t], lpx = in.lpx[t], rpn = in.rpn[t], lpn = in.lpn[t];
    const bool has = !isnan(ntrial[t]);
    // s0 = forward, s1 = backward segmented sums (NaN r rows hold the running totals)
    const double tot = s0[t] + s1[t] - (isnan(r) ? 0.0 : r);
    o.c[SGLM_PREP_OUT_R_TRIAL][t] = (has && tot > 0.0) ? 1.0 : 0.0;
    o.c[SGLM_PREP_OUT_NR_TRIAL][t] = (has && tot <= 0.0) ? 1.0 : 0.0;
    const double rpxr = r * rpx, rpxnr = nr * rpx, lpxr = r * lpx, lpxnr = nr * lpx;
    const double rpnr = r * rpn, rpnnr = nr * rpn, lpnr = r * lpn, lpnnr = nr * lpn;
    o.c[SGLM_PREP_OUT_RPXR][t] = rpxr;
    o.c[SGLM_PREP_OUT_RPXNR][t] = rpxnr;
    o.c[SGLM_PREP_OUT_LPXR][t] = lpxr;
    o.c[SGLM_PREP_OUT_LPXNR][t] = lpxnr;
    o.c[SGLM_PREP_OUT_RPNR][t] = rpnr;
    o.c[SGLM_PREP_OUT_RPNNR][t] = rpnnr;
    o.c[SGLM_PREP_OUT_LPNR][t] = lpnr;
    o.c[SGLM_PREP_OUT_LPNNR][t] = lpnnr;
    o.c[SGLM_PREP_OUT_SPN][t] = rpn + lpn;
    o.c[SGLM_PREP_OUT_SPX][t] = rpx + lpx;
    o.c[SGLM_PREP_OUT_SPNR][t] = rpnr + lpnr;
    o.c[SGLM_PREP_OUT_SPNNR][t] = rpnnr + lpnnr;
    o.c[SGLM_PREP_OUT_SPXR][t] = rpxr + lpxr;
    o.c[SGLM_PREP_OUT_SPXNR][t] = rpxnr + lpxnr;
    o.c[SGLM_PREP_OUT_SL][t] = in.rl[t] + in.ll[t];
    // DataFrame.sum(axis=1): NaN skipped, all-NaN rows sum to 0
    const double nn = (isnan(lpn) ? 0.0 : lpn) + (isnan(rpn) ? 0.0 : rpn);
    const double xx = (isnan(lpx) ? 0.0 : lpx) + (isnan(rpx) ? 0.0 : rpx);
    o.c[SGLM_PREP_OUT_NN][t] = nn;
    o.c[SGLM_PREP_OUT_XX][t] = xx;
}

// ((cumsum == 1) * 1).diff(), negatives zeroed by multiplication (so -1 becomes -0.0, row 0
// stays NaN) (lynne_pp.py:196-198).
__device__ __forceinline__ double first_step(const double* cs, int64_t t) {
    if (t == 0) return NAN;
    const double d = (cs[t] == 1.0 ? 1.0 : 0.0) - (cs[t - 1] == 1.0 ? 1.0 : 0.0);
    return d * (d >= 0.0 ? 1.0 : 0.0);
}

// First-time events (lynne_pp.py:196-213).
__global__ void prep_first_kernel(In in, const double* __restrict__ cs_nn,
                                  const double* __restrict__ cs_xx,
                                  const double* __restrict__ cs_cpn, int64_t n, Out o) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    // nn, xx, spn, spx recomputed from the inputs (cheaper than re-reading the outputs)
    const double lpn = in.lpn[t], rpn = in.rpn[t], lpx = in.lpx[t], rpx = in.rpx[t];
    const double nn = (isnan(lpn) ? 0.0 : lpn) + (isnan(rpn) ? 0.0 : rpn);
    const double xx = (isnan(lpx) ? 0.0 : lpx) + (isnan(rpx) ? 0.0 : rpx);
    const double spn = rpn + lpn, spx = rpx + lpx;
    const double r = in.r[t], nr = in.nr[t];
    o.c[SGLM_PREP_OUT_FT_NN][t] = first_step(cs_nn, t);
    o.c[SGLM_PREP_OUT_FT_XX][t] = first_step(cs_xx, t);
    o.c[SGLM_PREP_OUT_FT_CPN][t] = first_step(cs_cpn, t);
    const double ft_lpn = nn * lpn, ft_rpn = nn * rpn, ft_spn = nn * spn;
    o.c[SGLM_PREP_OUT_FT_LPN][t] = ft_lpn;
    o.c[SGLM_PREP_OUT_FT_RPN][t] = ft_rpn;
    o.c[SGLM_PREP_OUT_FT_SPN][t] = ft_spn;
    o.c[SGLM_PREP_OUT_FT_LPX][t] = xx * lpx;
    o.c[SGLM_PREP_OUT_FT_RPX][t] = xx * rpx;
    o.c[SGLM_PREP_OUT_FT_SPX][t] = xx * spx;
    o.c[SGLM_PREP_OUT_FT_R_RPN][t] = ft_rpn * r;
    o.c[SGLM_PREP_OUT_FT_R_LPN][t] = ft_lpn * r;
    o.c[SGLM_PREP_OUT_FT_R_SPN][t] = ft_spn * r;
    o.c[SGLM_PREP_OUT_FT_NR_RPN][t] = ft_rpn * nr;
    o.c[SGLM_PREP_OUT_FT_NR_LPN][t] = ft_lpn * nr;
    o.c[SGLM_PREP_OUT_FT_NR_SPN][t] = ft_spn * nr;
}

// ---- gen_signal_df.generate_signal_df (sglm/sglm/features/gen_signal_df.py:327-470) ------
// Trial-table values aligned onto the signal rows (pandas index alignment of
// df_t_tmp.set_index(col)[...], :416-427): NaN everywhere, then out[c][rows[t]] = vals[c][t].
__global__ void __launch_bounds__(256) fill_nan_kernel(double* __restrict__ out, int64_t ld,
                                                       int32_t nc, int64_t n) {
    const int c = blockIdx.y;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * 256)
        out[(int64_t)c * ld + i] = NAN;
}

__global__ void __launch_bounds__(256) scatter_rows_kernel(const int64_t* __restrict__ rows,
                                                           int64_t nr,
                                                           const double* __restrict__ vals,
                                                           int32_t nc, double* __restrict__ out,
                                                           int64_t ld, int64_t n) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= nr) return;
    const int64_t r = rows[t];
    if (r < 0 || r >= n) return;                     // labels absent from the signal index
    for (int c = 0; c < nc; ++c) out[(int64_t)c * ld + r] = vals[(int64_t)c * nr + t];
}

// trial start / end flags: ((~isna) & (x == 1)) * 1 (get_trial_start / get_trial_end, :251-281)
__global__ void __launch_bounds__(256) sig_flags_kernel(const double* __restrict__ cin,
                                                        const double* __restrict__ sout,
                                                        int64_t n, double* __restrict__ fs,
                                                        double* __restrict__ fe) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    fs[i] = cin[i] == 1.0 ? 1.0 : 0.0;
    fe[i] = sout[i] == 1.0 ? 1.0 : 0.0;
}

__device__ __forceinline__ double shifted(const double* x, int64_t i, int64_t k, int64_t n) {
    const int64_t j = i - k;                         // Series.shift(k): out[i] = in[i - k]
    return j >= 0 && j < n ? x[j] : NAN;
}

// nTrial = cumsum(start).shift(kb), nEndTrial = cumsum(end).shift(ka), diffTrialNums, the
// duplication flag F = diffTrialNums > 1 (:430-441) and each row's run-head index (nTrial
// runs are contiguous: a cumulative count shifted)
__global__ void __launch_bounds__(256) sig_shift_kernel(const double* __restrict__ cs,
                                                        const double* __restrict__ ce,
                                                        int64_t n, int64_t kb, int64_t ka,
                                                        double* __restrict__ ntrial,
                                                        double* __restrict__ nend,
                                                        double* __restrict__ diff,
                                                        double* __restrict__ F,
                                                        double* __restrict__ head) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const double a = shifted(cs, i, kb, n), b = shifted(ce, i, ka, n);
    const double prev = i > 0 ? shifted(cs, i - 1, kb, n) : NAN;
    ntrial[i] = a;
    nend[i] = b;
    const double d = a - b;
    diff[i] = d;
    F[i] = d > 1.0 ? 1.0 : 0.0;
    head[i] = (i == 0 || !(a == prev)) ? (double)i : -INFINITY;
}

// Output row map of the duplication loop (:437-458): per nTrial run (value v, in order), the
// rows with F = 1 as copies (nTrial v - 1, dupe True), then the run itself; rows whose nTrial
// is NaN are dropped.  G: inclusive cumsum of F; Fs / Fb: forward / backward cumsums of F within
// the run; S: the run's first row.
__global__ void __launch_bounds__(256) sig_map_kernel(const double* __restrict__ ntrial,
                                                      const double* __restrict__ F,
                                                      const double* __restrict__ G,
                                                      const double* __restrict__ Fs,
                                                      const double* __restrict__ Fb,
                                                      const double* __restrict__ S, int64_t n,
                                                      int64_t nan_lead,
                                                      int64_t* __restrict__ src,
                                                      uint8_t* __restrict__ dup) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n || isnan(ntrial[i])) return;
    const int64_t f = (int64_t)F[i], fs = (int64_t)Fs[i];
    const int64_t total = fs + (int64_t)Fb[i] - f;         // copies made in this run
    const int64_t before = (int64_t)G[i] - fs;              // copies made in earlier runs
    const int64_t pos = (i - nan_lead) + before + total;
    src[pos] = i;
    dup[pos] = 0;
    if (f) {
        const int64_t pd = ((int64_t)S[i] - nan_lead) + before + fs - 1;
        src[pd] = i;
        dup[pd] = 1;
    }
}

}  // namespace
}  // namespace sglm

using namespace sglm;

extern "C" int sglm_scatter_rows(int64_t n, const int64_t* rows, int64_t nrows,
                                 const double* vals, int32_t ncols, double* out, int64_t ld_out,
                                 sglm_stream_t stream) {
    if (n <= 0 || ncols <= 0) return SGLM_OK;
    if (!out || ld_out < n || (nrows > 0 && (!rows || !vals))) {
        set_error("sglm_scatter_rows: bad args");
        return SGLM_EINVAL;
    }
    hipStream_t s = as_stream(stream);
    const int64_t g = (n + 255) / 256;
    fill_nan_kernel<<<dim3((unsigned)(g < 4096 ? g : 4096), (unsigned)ncols), 256, 0, s>>>(
        out, ld_out, ncols, n);
    int st = check_launch("fill_nan_kernel");
    if (st || nrows <= 0) return st;
    scatter_rows_kernel<<<(unsigned)((nrows + 255) / 256), 256, 0, s>>>(rows, nrows, vals, ncols,
                                                                       out, ld_out, n);
    return check_launch("scatter_rows_kernel");
}

extern "C" size_t sglm_signal_trials_work_bytes(int64_t n) {
    if (n < 0) n = 0;
    return (size_t)7 * (size_t)n * sizeof(double) + (size_t)nwaves_of(n) * sizeof(Agg<1>) + 256;
}

extern "C" int sglm_signal_trials(const double* center_in, const double* side_out, int64_t n,
                                  int64_t k_before, int64_t k_after, double* ntrial,
                                  double* nend, double* diff, int64_t* src, uint8_t* dup,
                                  double* ncopies, void* work, sglm_stream_t stream) {
    if (n <= 0) return SGLM_OK;
    if (!center_in || !side_out || !ntrial || !nend || !diff || !src || !dup || !ncopies ||
        !work) {
        set_error("sglm_signal_trials: null pointer");
        return SGLM_EINVAL;
    }
    hipStream_t s = as_stream(stream);
    double* T0 = (double*)work;                     // start flags -> cumsum
    double* T1 = T0 + n;                            // end flags -> cumsum
    double* F = T1 + n;
    double* H = F + n;                              // head index -> run start (max scan)
    double* G = H + n;
    double* Fs = G + n;
    double* Fb = Fs + n;
    void* agg = (void*)(((uintptr_t)(Fb + n) + 63) & ~(uintptr_t)63);
    const int64_t g = (n + 255) / 256;
    int st;
    sig_flags_kernel<<<g, 256, 0, s>>>(center_in, side_out, n, T0, T1);
    if ((st = scan<OP_ADD, 1>(cols1(T0, T0, nullptr, n, 0), agg, s))) return st;
    if ((st = scan<OP_ADD, 1>(cols1(T1, T1, nullptr, n, 0), agg, s))) return st;
    sig_shift_kernel<<<g, 256, 0, s>>>(T0, T1, n, k_before, k_after, ntrial, nend, diff, F, H);
    if ((st = scan<OP_ADD, 1>(cols1(F, G, nullptr, n, 0), agg, s))) return st;
    if ((st = scan<OP_ADD, 1>(cols1(F, Fs, ntrial, n, 0), agg, s))) return st;
    if ((st = scan<OP_ADD, 1>(cols1(F, Fb, ntrial, n, 1), agg, s))) return st;
    if ((st = scan<OP_MAX, 1>(cols1(H, H, nullptr, n, 0), agg, s))) return st;
    const int64_t lead = k_before > 0 ? (k_before < n ? k_before : n) : 0;
    sig_map_kernel<<<g, 256, 0, s>>>(ntrial, F, G, Fs, Fb, H, n, lead, src, dup);
    if ((st = check_launch("sig_map_kernel"))) return st;
    // total copies = G[n-1]
    if (hipMemcpyAsync(ncopies, G + (n - 1), sizeof(double), hipMemcpyDeviceToDevice, s) !=
        hipSuccess) {
        set_error("sglm_signal_trials: hipMemcpyAsync failed");
        return SGLM_EHIP;
    }
    return SGLM_OK;
}

extern "C" size_t sglm_prep_work_bytes(int64_t n) {
    if (n < 0) n = 0;
    return (size_t)3 * (size_t)n * sizeof(double) + (size_t)nwaves_of(n) * sizeof(Agg<3>) + 256;
}

extern "C" int sglm_prep_session(const double* in, int64_t ld_in, int64_t n, int32_t k,
                                 double* out, int64_t ld_out, void* work, sglm_stream_t stream) {
    if (n == 0) return SGLM_OK;
    if (!in || !out || !work || n < 0 || ld_in < n || ld_out < n) {
        set_error("sglm_prep_session: bad args (n=%lld, ld_in=%lld, ld_out=%lld)",
                  (long long)n, (long long)ld_in, (long long)ld_out);
        return SGLM_EINVAL;
    }
    hipStream_t s = as_stream(stream);
    In x;
    const double** xc[SGLM_PREP_NIN] = {&x.cpn, &x.lpx, &x.rpx, &x.lpn, &x.rpn,
                                        &x.r,   &x.nr,  &x.rl,  &x.ll};
    for (int c = 0; c < SGLM_PREP_NIN; ++c) *xc[c] = in + (int64_t)c * ld_in;
    Out o;
    for (int c = 0; c < SGLM_PREP_NOUT; ++c) o.c[c] = out + (int64_t)c * ld_out;
    double* T0 = (double*)work;
    double* T1 = T0 + n;
    double* T2 = T1 + n;
    void* agg = (void*)(((uintptr_t)(T2 + n) + 63) & ~(uintptr_t)63);
    const int bs = 256;
    const int64_t g = (n + bs - 1) / bs;
    double* ntrial = o.c[SGLM_PREP_OUT_NTRIAL];
    double* flag = o.c[SGLM_PREP_OUT_TRIAL_START_FLAG];
    double* eflag = o.c[SGLM_PREP_OUT_TRIAL_END_FLAG];
    int st;
    // trial starts: codes -> backward fill -> start flag -> cumulative sum (nTrial)
    prep_codes_kernel<<<g, bs, 0, s>>>(x, n, T0, T1);
    if ((st = scan<OP_MAX, 1>(cols1(T1, T1, nullptr, n, 1), agg, s))) return st;
    prep_start_kernel<<<g, bs, 0, s>>>(T0, T1, n, k, o.c[SGLM_PREP_OUT_EVENT_COL], flag);
    if ((st = scan<OP_ADD, 1>(cols1(flag, ntrial, nullptr, n, 0), agg, s))) return st;
    // trial ends: codes -> forward fill -> end flag -> cumulative sum (nEndTrial)
    prep_end_codes_kernel<<<g, bs, 0, s>>>(x, flag, n, T0, T1);
    if ((st = scan<OP_MAX, 1>(cols1(T1, T1, nullptr, n, 0), agg, s))) return st;
    prep_end_kernel<<<g, bs, 0, s>>>(T0, T1, ntrial, n, k, o.c[SGLM_PREP_OUT_EVENT_COL_END],
                                     eflag);
    if ((st = scan<OP_ADD, 1>(cols1(eflag, o.c[SGLM_PREP_OUT_NENDTRIAL], nullptr, n, 0), agg,
                              s)))
        return st;
    // per-trial reward totals (forward + backward segmented sums), indicators
    if ((st = scan<OP_ADD, 1>(cols1(x.r, T0, ntrial, n, 0, 1), agg, s))) return st;
    if ((st = scan<OP_ADD, 1>(cols1(x.r, T1, ntrial, n, 1, 1), agg, s))) return st;
    prep_rows_kernel<<<g, bs, 0, s>>>(x, ntrial, n, o, T0, T1);
    // per-trial cumulative sums of nn, xx, cpn in one 3-column scan, then first-time events
    ScanCols c3 = {};
    c3.x[0] = o.c[SGLM_PREP_OUT_NN]; c3.x[1] = o.c[SGLM_PREP_OUT_XX]; c3.x[2] = x.cpn;
    c3.y[0] = T0; c3.y[1] = T1; c3.y[2] = T2;
    c3.key = ntrial; c3.n = n; c3.rev = 0;
    if ((st = scan<OP_ADD, 3>(c3, agg, s))) return st;
    prep_first_kernel<<<g, bs, 0, s>>>(x, T0, T1, T2, n, o);
    return check_launch("prep_first_kernel");
}
