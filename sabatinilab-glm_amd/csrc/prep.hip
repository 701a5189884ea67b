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

constexpr int kPT = 256;          // threads per scan workgroup
constexpr int kPR = 8;            // consecutive rows per thread
constexpr int kPC = kPT * kPR;    // rows per scan chunk
constexpr int kCT1 = 1024;        // carry-scan workgroup

enum { OP_ADD = 0, OP_MAX = 1 };

// Scan element: value plus a "segment starts here" bit.  ADD with heads is the segmented sum
// (a head resets the running value), MAX ignores heads.  The operator is associative but not
// commutative, so every reduction below keeps row order.
struct Agg { double v; int h; };

template <int OP> __device__ __forceinline__ Agg ident() {
    return {OP == OP_MAX ? -INFINITY : 0.0, 0};
}
template <int OP> __device__ __forceinline__ Agg comb(Agg a, Agg b) {
    if (OP == OP_MAX) return {fmax(a.v, b.v), 0};
    return {b.h ? b.v : a.v + b.v, a.h | b.h};
}

// Ordered exclusive scan over the NW waves of a workgroup; `total` = the workgroup aggregate.
template <int OP, int NW>
__device__ __forceinline__ Agg block_excl(Agg a, Agg* lds, Agg& total) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    Agg inc = a;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        Agg t;
        t.v = __shfl_up(inc.v, o, 64);
        t.h = __shfl_up(inc.h, o, 64);
        if (lane >= o) inc = comb<OP>(t, inc);
    }
    if (lane == 63) lds[w] = inc;
    Agg up;
    up.v = __shfl_up(inc.v, 1, 64);
    up.h = __shfl_up(inc.h, 1, 64);
    __syncthreads();
    Agg wp = ident<OP>(), tot = ident<OP>();
#pragma unroll
    for (int i = 0; i < NW; ++i) {
        if (i < w) wp = comb<OP>(wp, lds[i]);
        tot = comb<OP>(tot, lds[i]);
    }
    total = tot;
    return comb<OP>(wp, lane == 0 ? ident<OP>() : up);
}

// Logical row i of a scan in direction `rev` is physical row rev ? n-1-i : i.  A row's value
// is x (NaN rows contribute the identity: pandas' skipna cumsum); with a key column a row is a
// segment head when its key differs from the previous logical row's (NaN keys never match).
template <int OP>
__device__ __forceinline__ Agg load_elem(const double* __restrict__ x,
                                         const double* __restrict__ key, int64_t n, int rev,
                                         int64_t i, double& raw) {
    const int64_t p = rev ? n - 1 - i : i;
    raw = x[p];
    Agg e = {isnan(raw) ? ident<OP>().v : raw, 0};
    if (key) {
        const int64_t q = rev ? p + 1 : p - 1;
        e.h = (i == 0) || (key[p] != key[q]);
    }
    return e;
}

template <int OP>
__global__ void __launch_bounds__(kPT) scan_reduce_kernel(const double* __restrict__ x,
                                                          const double* __restrict__ key,
                                                          int64_t n, int rev, Agg* agg) {
    __shared__ Agg lds[kPT / 64];
    const int64_t base = (int64_t)blockIdx.x * kPC + (int64_t)threadIdx.x * kPR;
    Agg a = ident<OP>();
    for (int j = 0; j < kPR; ++j) {
        const int64_t i = base + j;
        if (i < n) {
            double raw;
            a = comb<OP>(a, load_elem<OP>(x, key, n, rev, i, raw));
        }
    }
    Agg total;
    block_excl<OP, kPT / 64>(a, lds, total);
    if (threadIdx.x == 0) agg[blockIdx.x] = total;
}

// One workgroup turns the chunk aggregates into exclusive carries, in place: thread t owns a
// contiguous run of chunks, the runs are scanned in order across the workgroup.
template <int OP>
__global__ void __launch_bounds__(kCT1) scan_carry_kernel(Agg* agg, int64_t nchunks) {
    __shared__ Agg lds[kCT1 / 64];
    const int64_t per = (nchunks + kCT1 - 1) / kCT1;
    const int64_t c0 = (int64_t)threadIdx.x * per;
    const int64_t c1 = c0 + per < nchunks ? c0 + per : nchunks;
    Agg a = ident<OP>();
    for (int64_t c = c0; c < c1; ++c) a = comb<OP>(a, agg[c]);
    Agg total;
    Agg run = block_excl<OP, kCT1 / 64>(a, lds, total);
    for (int64_t c = c0; c < c1; ++c) {
        const Agg v = agg[c];
        agg[c] = run;
        run = comb<OP>(run, v);
    }
}

template <int OP>
__global__ void __launch_bounds__(kPT) scan_apply_kernel(const double* __restrict__ x,
                                                         const double* __restrict__ key,
                                                         int64_t n, int rev,
                                                         const Agg* __restrict__ carry,
                                                         double* __restrict__ y) {
    __shared__ Agg lds[kPT / 64];
    const int64_t base = (int64_t)blockIdx.x * kPC + (int64_t)threadIdx.x * kPR;
    Agg e[kPR];
    double raw[kPR];
    Agg a = ident<OP>();
#pragma unroll
    for (int j = 0; j < kPR; ++j) {
        const int64_t i = base + j;
        if (i < n) {
            e[j] = load_elem<OP>(x, key, n, rev, i, raw[j]);
            a = comb<OP>(a, e[j]);
        }
    }
    Agg total;
    Agg run = comb<OP>(carry[blockIdx.x], block_excl<OP, kPT / 64>(a, lds, total));
#pragma unroll
    for (int j = 0; j < kPR; ++j) {
        const int64_t i = base + j;
        if (i < n) {
            run = comb<OP>(run, e[j]);
            y[rev ? n - 1 - i : i] = isnan(raw[j]) ? raw[j] : run.v;
        }
    }
}

inline int64_t nchunks_of(int64_t n) { return (n + kPC - 1) / kPC; }

// y = inclusive scan of x (in place allowed): ADD (pandas cumsum, skipna) or MAX, forward or
// backward, segmented by `key` when given (ADD only).
int scan(int op, const double* x, const double* key, int64_t n, int rev, double* y, Agg* agg,
         hipStream_t s) {
    const int64_t nc = nchunks_of(n);
    if (op == OP_ADD) {
        scan_reduce_kernel<OP_ADD><<<nc, kPT, 0, s>>>(x, key, n, rev, agg);
        scan_carry_kernel<OP_ADD><<<1, kCT1, 0, s>>>(agg, nc);
        scan_apply_kernel<OP_ADD><<<nc, kPT, 0, s>>>(x, key, n, rev, agg, y);
    } else {
        scan_reduce_kernel<OP_MAX><<<nc, kPT, 0, s>>>(x, key, n, rev, agg);
        scan_carry_kernel<OP_MAX><<<1, kCT1, 0, s>>>(agg, nc);
        scan_apply_kernel<OP_MAX><<<nc, kPT, 0, s>>>(x, key, n, rev, agg, y);
    }
    return check_launch("prep scan");
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

// r restricted to rows with a trial number (groupby drops NaN keys, lynne_pp.py:121).
__global__ void prep_mask_r_kernel(const double* __restrict__ r,
                                   const double* __restrict__ ntrial, int64_t n,
                                   double* __restrict__ rm) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    rm[t] = isnan(ntrial[t]) ? NAN : r[t];
}

struct Out {  // output columns (SGLM_PREP_OUT_* order)
    double* c[SGLM_PREP_NOUT];
};

// Reward flags (per-trial sum of r = forward + backward segmented sums - r), port indicators,
// side-agnostic sums, nn / xx (lynne_pp.py:121-123, 142-151, 170-178, 193-194); the per-trial
// cumulative-sum inputs of nn, xx, cpn (NaN outside trials) go to s0..s2.
__global__ void prep_rows_kernel(In in, const double* __restrict__ ntrial, int64_t n, Out o,
                                 double* __restrict__ s0, double* __restrict__ s1,
                                 double* __restrict__ s2) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    const double r = in.r[t], nr = in.nr[t];
    const double rpx = in.rpx[t], lpx = in.lpx[t], rpn = in.rpn[t], lpn = in.lpn[t];
    const bool has = !isnan(ntrial[t]);
    const double tot = s0[t] + s1[t] - r;      // s0 = forward, s1 = backward segmented sums
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
    s0[t] = has ? nn : NAN;
    s1[t] = has ? xx : NAN;
    s2[t] = has ? in.cpn[t] : NAN;
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
    const double nn = o.c[SGLM_PREP_OUT_NN][t], xx = o.c[SGLM_PREP_OUT_XX][t];
    const double spn = o.c[SGLM_PREP_OUT_SPN][t], spx = o.c[SGLM_PREP_OUT_SPX][t];
    const double r = in.r[t], nr = in.nr[t];
    o.c[SGLM_PREP_OUT_FT_NN][t] = first_step(cs_nn, t);
    o.c[SGLM_PREP_OUT_FT_XX][t] = first_step(cs_xx, t);
    o.c[SGLM_PREP_OUT_FT_CPN][t] = first_step(cs_cpn, t);
    const double ft_lpn = nn * in.lpn[t], ft_rpn = nn * in.rpn[t], ft_spn = nn * spn;
    o.c[SGLM_PREP_OUT_FT_LPN][t] = ft_lpn;
    o.c[SGLM_PREP_OUT_FT_RPN][t] = ft_rpn;
    o.c[SGLM_PREP_OUT_FT_SPN][t] = ft_spn;
    o.c[SGLM_PREP_OUT_FT_LPX][t] = xx * in.lpx[t];
    o.c[SGLM_PREP_OUT_FT_RPX][t] = xx * in.rpx[t];
    o.c[SGLM_PREP_OUT_FT_SPX][t] = xx * spx;
    o.c[SGLM_PREP_OUT_FT_R_RPN][t] = ft_rpn * r;
    o.c[SGLM_PREP_OUT_FT_R_LPN][t] = ft_lpn * r;
    o.c[SGLM_PREP_OUT_FT_R_SPN][t] = ft_spn * r;
    o.c[SGLM_PREP_OUT_FT_NR_RPN][t] = ft_rpn * nr;
    o.c[SGLM_PREP_OUT_FT_NR_LPN][t] = ft_lpn * nr;
    o.c[SGLM_PREP_OUT_FT_NR_SPN][t] = ft_spn * nr;
}

}  // namespace
}  // namespace sglm

using namespace sglm;

extern "C" size_t sglm_prep_work_bytes(int64_t n) {
    if (n < 0) n = 0;
    return (size_t)3 * (size_t)n * sizeof(double) + (size_t)nchunks_of(n) * sizeof(Agg) + 256;
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
    Agg* agg = (Agg*)(((uintptr_t)(T2 + n) + 63) & ~(uintptr_t)63);
    const int bs = 256;
    const int64_t g = (n + bs - 1) / bs;
    double* ntrial = o.c[SGLM_PREP_OUT_NTRIAL];
    double* flag = o.c[SGLM_PREP_OUT_TRIAL_START_FLAG];
    double* eflag = o.c[SGLM_PREP_OUT_TRIAL_END_FLAG];
    int st;
    // trial starts: codes -> backward fill -> start flag -> cumulative sum (nTrial)
    prep_codes_kernel<<<g, bs, 0, s>>>(x, n, T0, T1);
    if ((st = scan(OP_MAX, T1, nullptr, n, 1, T1, agg, s))) return st;
    prep_start_kernel<<<g, bs, 0, s>>>(T0, T1, n, k, o.c[SGLM_PREP_OUT_EVENT_COL], flag);
    if ((st = scan(OP_ADD, flag, nullptr, n, 0, ntrial, agg, s))) return st;
    // trial ends: codes -> forward fill -> end flag -> cumulative sum (nEndTrial)
    prep_end_codes_kernel<<<g, bs, 0, s>>>(x, flag, n, T0, T1);
    if ((st = scan(OP_MAX, T1, nullptr, n, 0, T1, agg, s))) return st;
    prep_end_kernel<<<g, bs, 0, s>>>(T0, T1, ntrial, n, k, o.c[SGLM_PREP_OUT_EVENT_COL_END],
                                     eflag);
    if ((st = scan(OP_ADD, eflag, nullptr, n, 0, o.c[SGLM_PREP_OUT_NENDTRIAL], agg, s)))
        return st;
    // per-trial reward totals, indicators, per-trial cumulative sums, first-time events
    prep_mask_r_kernel<<<g, bs, 0, s>>>(x.r, ntrial, n, T2);
    if ((st = scan(OP_ADD, T2, ntrial, n, 0, T0, agg, s))) return st;
    if ((st = scan(OP_ADD, T2, ntrial, n, 1, T1, agg, s))) return st;
    prep_rows_kernel<<<g, bs, 0, s>>>(x, ntrial, n, o, T0, T1, T2);
    for (double* T : {T0, T1, T2})
        if ((st = scan(OP_ADD, T, ntrial, n, 0, T, agg, s))) return st;
    prep_first_kernel<<<g, bs, 0, s>>>(x, T0, T1, T2, n, o);
    return check_launch("prep_first_kernel");
}
