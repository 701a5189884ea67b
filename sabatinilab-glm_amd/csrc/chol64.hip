// Float64 factorisation with exact rank decisions, float64 Newton solves, and the
// minimum-norm projection of unpenalised rank-deficient fits.
//
// The reference's OLS is LinearRegression -> scipy.linalg.lstsq (backend/sglm.py:96-101 ->
// sklearn linear_model/_base.py:701): on a rank-deficient design it returns the MINIMUM-NORM
// coefficients (two identical columns share the weight equally), and its unpenalised Poisson
// (TweedieRegressor alpha = 0, lbfgs from w = 0, backend/sglm.py:112-115) stays in the row space
// of X and reaches the same minimum-norm minimiser.  A float32 factor cannot tell an exactly
// dependent column (pivot ~ eps32 of its diagonal) from an ill-conditioned but independent one
// (pivot ~ 1/cond), so the rank decision is taken here, in float64, on the exact mask Gram:
//
//   sglm_chol64_factor   U^T U = G[hsrc[f]] + shift (upper triangle, right-looking blocked,
//                        64-column blocks: diagonal block in LDS, panel strips, 64 x 64
//                        trailing tiles).  A pivot whose Schur complement falls to
//                        <= tol * its original diagonal is DEPENDENT: its row of U is zeroed
//                        (U_dd = 1) and its column above the diagonal, U[K][d] = U_KK^-T G_Kd,
//                        is kept -- the representation of column d in the kept columns.
//   sglm_chol64_solve    delta = -U^-1 U^-T g on the kept coordinates (the Gaussian Newton /
//                        closed-form step, float64 throughout), 0 elsewhere.
//   sglm_chol64_minnorm  null vectors N_d = e_d - U_KK^-1 U[K][d] for every dependent d,
//                        orthonormalised in the coefficient part (classical Gram-Schmidt, two
//                        passes), then w <- w - N (N_w^T N_w)^-1 N_w^T w for every listed fit:
//                        the minimum-|w| point of the fit's solution set.  X~ N = 0 on the
//                        mask rows, so the fitted values are unchanged.
//
// Coordinate states (state[f][j]): 0 kept, 1 dependent (a null direction), 2 excluded
// (dshift < 0: an unfitted intercept, padding), 3 zero column (zero diagonal without a ridge
// term; its coefficient is 0 and it is already orthogonal to every null vector).
#include <math.h>

#include "common.h"

namespace sglm {
namespace {

constexpr int kB = 64;
constexpr int kMaxP64 = 8192;
enum : uint8_t { ST_KEPT = 0, ST_DEP = 1, ST_EXCL = 2, ST_ZERO = 3 };

// U[f] (upper triangle, rows i <= j; the strict lower part of diagonal tiles zeroed) from the f32
// Gram H[hsrc[f]] (i <= j read) plus the penalty row lamp[dsrc[f]] (float64) on the diagonal;
// a mixed design's continuous coordinates (cmap[j] = c >= 0) read their rows and columns from the
// float64 block S[f][c][0 .. P) instead (sglm_mixed_gram, exact to float64 rounding);
// excluded (dshift < 0) and zero-diagonal coordinates become identity rows / columns.  One
// 64 x 64 tile of the upper triangle per workgroup; diagonal tiles also write state and d0.
__global__ void __launch_bounds__(256) c64_init_kernel(
    const float* __restrict__ H, int32_t P, const int32_t* __restrict__ hsrc,
    const float* __restrict__ dshift, const double* __restrict__ lamp,
    const int32_t* __restrict__ dsrc, const double* __restrict__ S, int32_t k,
    const int32_t* __restrict__ cmap, double* __restrict__ U, uint8_t* __restrict__ state,
    double* __restrict__ d0) {
    const int f = blockIdx.y;
    int t = blockIdx.x, bi = 0;
    {
        int rowlen = P / kB;
        while (t >= rowlen) { t -= rowlen; ++bi; --rowlen; }
    }
    const int bj = bi + t;
    const float* Hs = H + (int64_t)hsrc[f] * P * P;
    const float* dsh = dshift + (int64_t)dsrc[f] * P;
    const double* lp = lamp ? lamp + (int64_t)dsrc[f] * P : nullptr;
    double* Uf = U + (int64_t)f * P * P;
    const double* Sf = S ? S + (int64_t)f * k * P : nullptr;
    auto gram = [&](int i, int j) -> double {
        if (Sf) {
            const int ci = cmap[i];
            if (ci >= 0) return Sf[(int64_t)ci * P + j];
            const int cj = cmap[j];
            if (cj >= 0) return Sf[(int64_t)cj * P + i];
        }
        return (double)Hs[(int64_t)i * P + j];
    };
    __shared__ uint8_t sr[kB], sc[kB];
    const int tid = threadIdx.x;
    if (tid < 2 * kB) {
        const bool row = tid < kB;
        const int j = (row ? bi : bj) * kB + (tid & 63);
        uint8_t s = ST_EXCL;
        double d = 0.0;
        if (!(dsh[j] < 0.0f)) {
            d = gram(j, j) + (lp ? lp[j] : (double)dsh[j]);
            s = d > 0.0 ? ST_KEPT : ST_ZERO;
        }
        if (row) sr[tid] = s; else sc[tid - kB] = s;
        if (row && bi == bj) {
            state[(int64_t)f * P + j] = s;
            d0[(int64_t)f * P + j] = d;
        }
    }
    __syncthreads();
    const int c = tid & 63;
    for (int r = tid >> 6; r < kB; r += 4) {
        const int i = bi * kB + r, j = bj * kB + c;
        double v;
        if (i > j) v = 0.0;
        else if (sr[r] != ST_KEPT || sc[c] != ST_KEPT) v = i == j ? 1.0 : 0.0;
        else {
            v = gram(i, j);
            if (i == j) v += lp ? lp[j] : (double)dsh[j];
        }
        Uf[(int64_t)i * P + j] = v;
    }
}

// Diagonal block kb of every factor: one wave per factor, the 64 x 64 block in LDS, lane c owns
// column c.  Dependent pivots (Schur complement <= tol * d0) are marked and their row zeroed.
__global__ void __launch_bounds__(64) c64_diag_kernel(double* __restrict__ U, int32_t P,
                                                      int32_t kb, uint8_t* __restrict__ state,
                                                      const double* __restrict__ d0, double tol) {
    const int f = blockIdx.x;
    double* Uf = U + (int64_t)f * P * P;
    __shared__ double A[kB][kB + 1];
    __shared__ double dd[kB];
    __shared__ uint8_t st[kB];
    const int c = threadIdx.x;
    const int k0 = kb * kB;
    for (int r = 0; r < kB; ++r) A[r][c] = r <= c ? Uf[(int64_t)(k0 + r) * P + k0 + c] : 0.0;
    st[c] = state[(int64_t)f * P + k0 + c];
    dd[c] = d0[(int64_t)f * P + k0 + c];
    __syncthreads();
    for (int j = 0; j < kB; ++j) {
        const uint8_t s = st[j];
        const double piv = A[j][j];
        const bool keep = s == ST_KEPT && piv > tol * dd[j];
        __syncthreads();
        if (!keep) {
            if (c == j) {
                A[j][j] = 1.0;
                if (s == ST_KEPT) st[j] = ST_DEP;
            } else if (c > j) {
                A[j][c] = 0.0;
            }
            __syncthreads();
            continue;
        }
        const double r = sqrt(piv);
        if (c == j) A[j][j] = r;
        else if (c > j) A[j][c] /= r;
        __syncthreads();
        if (c > j) {
            const double ujc = A[j][c];
            for (int i = j + 1; i <= c; ++i) A[i][c] -= A[j][i] * ujc;
        }
    }
    __syncthreads();
    for (int r = 0; r <= c; ++r) Uf[(int64_t)(k0 + r) * P + k0 + c] = A[r][c];
    state[(int64_t)f * P + k0 + c] = st[c];
}

// Panel of block row kb: U[kb rows][c] = U_kk^-T A[kb rows][c] for the columns right of the
// diagonal block (one 64-column chunk per workgroup, lane = column); rows of non-kept
// pivots are zero.
__global__ void __launch_bounds__(64) c64_panel_kernel(double* __restrict__ U, int32_t P,
                                                       int32_t kb,
                                                       const uint8_t* __restrict__ state) {
    const int f = blockIdx.y;
    const int k0 = kb * kB;
    const int t = threadIdx.x;
    const int c = (kb + 1 + (int)blockIdx.x) * kB + t;
    double* Uf = U + (int64_t)f * P * P;
    __shared__ double D[kB][kB + 1];
    __shared__ double X[kB][kB + 1];
    __shared__ uint8_t st[kB];
    for (int r = 0; r < kB; ++r) {
        D[r][t] = r <= t ? Uf[(int64_t)(k0 + r) * P + k0 + t] : 0.0;
        X[r][t] = Uf[(int64_t)(k0 + r) * P + c];
    }
    st[t] = state[(int64_t)f * P + k0 + t];
    __syncthreads();
    for (int j = 0; j < kB; ++j) {
        const double xj = st[j] == ST_KEPT ? X[j][t] / D[j][j] : 0.0;
        X[j][t] = xj;
        for (int i = j + 1; i < kB; ++i) X[i][t] -= D[j][i] * xj;
    }
    for (int r = 0; r < kB; ++r) Uf[(int64_t)(k0 + r) * P + c] = X[r][t];
}

// Trailing update after block kb: A_ij -= sum_k U[k][i] U[k][j] over the kb block's rows, for
// the 64 x 64 tiles (BI <= BJ) right of it; 4 x 4 float64 register tiles per thread.
__global__ void __launch_bounds__(256) c64_update_kernel(double* __restrict__ U, int32_t P,
                                                         int32_t kb) {
    const int f = blockIdx.y;
    int t = blockIdx.x, bi = 0;
    {
        int rowlen = P / kB - kb - 1;
        while (t >= rowlen) { t -= rowlen; ++bi; --rowlen; }
    }
    const int BI = kb + 1 + bi, BJ = BI + t;
    const int k0 = kb * kB;
    double* Uf = U + (int64_t)f * P * P;
    __shared__ double Si[kB][kB + 2];
    __shared__ double Sj[kB][kB + 2];
    const int tid = threadIdx.x;
    for (int e = tid; e < kB * kB; e += 256) {
        const int k = e >> 6, x = e & 63;
        Si[k][x] = Uf[(int64_t)(k0 + k) * P + BI * kB + x];
        Sj[k][x] = Uf[(int64_t)(k0 + k) * P + BJ * kB + x];
    }
    __syncthreads();
    const int tr = tid >> 4, tc = tid & 15;
    double acc[4][4] = {};
    for (int k = 0; k < kB; ++k) {
        double a[4], b[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            a[q] = Si[k][tr * 4 + q];
            b[q] = Sj[k][tc * 4 + q];
        }
#pragma unroll
        for (int x = 0; x < 4; ++x)
#pragma unroll
            for (int y = 0; y < 4; ++y) acc[x][y] = fma(a[x], b[y], acc[x][y]);
    }
#pragma unroll
    for (int x = 0; x < 4; ++x) {
        const int i = BI * kB + tr * 4 + x;
#pragma unroll
        for (int y = 0; y < 4; ++y) {
            const int j = BJ * kB + tc * 4 + y;
            if (i <= j) Uf[(int64_t)i * P + j] -= acc[x][y];
        }
    }
}

// Dependent pivots of each factor in ascending order (nulls[f][0 .. nd)), counts[f] = {nd,
// nd + zero columns}: one wave per factor.
__global__ void __launch_bounds__(64) c64_list_kernel(const uint8_t* __restrict__ state,
                                                      int32_t P, int32_t* __restrict__ nulls,
                                                      int32_t* __restrict__ counts) {
    const int f = blockIdx.x;
    const int l = threadIdx.x;
    int nd = 0, nz = 0;
    for (int base = 0; base < P; base += kB) {
        const uint8_t s = state[(int64_t)f * P + base + l];
        const uint64_t m = __ballot(s == ST_DEP);
        if (s == ST_DEP) nulls[(int64_t)f * P + nd + __popcll(m & ((1ull << l) - 1ull))] = base + l;
        nd += __popcll(m);
        nz += __popcll(__ballot(s == ST_ZERO));
    }
    if (l == 0) {
        counts[2 * f] = nd;
        counts[2 * f + 1] = nd + nz;
    }
}

// Triangular solves on a float64 factor, one workgroup (4 waves) per right-hand side, the
// solution vector in LDS.  NULLV = false: delta[fits[q]] = -U^-1 U^-T g[fits[q]] on the kept
// coordinates of factor fsrc[q] (float32 out, 0 elsewhere).  NULLV = true: right-hand side q of
// factor blockIdx.y is dependent pivot d = nulls[f][q]; N[f][q] = e_d - U_KK^-1 U[K][d].
template <bool NULLV, bool OUT64 = false>
__global__ void __launch_bounds__(256) c64_solve_kernel(
    const double* __restrict__ U, int32_t P, const uint8_t* __restrict__ state,
    const int32_t* __restrict__ fits, const int32_t* __restrict__ fsrc,
    const double* __restrict__ g, float* __restrict__ delta, const int32_t* __restrict__ nulls,
    const int32_t* __restrict__ counts, double* __restrict__ N, double* __restrict__ x64 = nullptr,
    const int32_t* __restrict__ gsrc = nullptr) {
    extern __shared__ double z[];
    __shared__ double part[4][kB];
    __shared__ double tail[kB];
    const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
    int f, fit = 0, d = 0;
    if (NULLV) {
        f = blockIdx.y;
        if ((int)blockIdx.x >= counts[2 * f]) return;
        d = nulls[(int64_t)f * P + blockIdx.x];
    } else {
        fit = fits[blockIdx.x];
        f = fsrc[blockIdx.x];
    }
    const double* Uf = U + (int64_t)f * P * P;
    const uint8_t* sf = state + (int64_t)f * P;
    const int nb = P / kB;
    int bhi = nb - 1, cend = P;
    if (NULLV) {
        for (int i = tid; i < P; i += 256)
            z[i] = (i < d && sf[i] == ST_KEPT) ? Uf[(int64_t)i * P + d] : 0.0;
        bhi = d / kB;
        cend = (bhi + 1) * kB;
        __syncthreads();
    } else {
        const double* gf = g + (int64_t)(gsrc ? gsrc[blockIdx.x] : fit) * P;
        // forward: U^T z = g, block by block
        for (int b = 0; b < nb; ++b) {
            const int c = b * kB + l;
            double acc = 0.0;
            for (int i = w; i < b * kB; i += 4) acc = fma(Uf[(int64_t)i * P + c], z[i], acc);
            part[w][l] = acc;
            __syncthreads();
            if (w == 0) {
                double tv = gf[c] - (part[0][l] + part[1][l] + part[2][l] + part[3][l]);
                for (int j = 0; j < kB; ++j) {
                    const int cj = b * kB + j;
                    double zj = 0.0;
                    if (l == j && sf[cj] == ST_KEPT) zj = tv / Uf[(int64_t)cj * P + cj];
                    zj = __shfl(zj, j, 64);
                    if (l > j) tv = fma(-Uf[(int64_t)cj * P + c], zj, tv);
                    if (l == j) z[cj] = zj;
                }
            }
            __syncthreads();
        }
    }
    // back: U x = z in place, block by block from the last
    for (int b = bhi; b >= 0; --b) {
        for (int rr = w; rr < kB; rr += 4) {
            const int r = b * kB + rr;
            double acc = 0.0;
            for (int c = (b + 1) * kB + l; c < cend; c += kB)
                acc = fma(Uf[(int64_t)r * P + c], z[c], acc);
            acc = wave_sum_d(acc);
            if (l == 0) tail[rr] = acc;
        }
        __syncthreads();
        if (w == 0) {
            const int r = b * kB + l;
            double tv = z[r] - tail[l];
            for (int j = kB - 1; j >= 0; --j) {
                const int rj = b * kB + j;
                double xj = 0.0;
                if (l == j && sf[rj] == ST_KEPT) xj = tv / Uf[(int64_t)rj * P + rj];
                xj = __shfl(xj, j, 64);
                if (l < j) tv = fma(-Uf[(int64_t)r * P + rj], xj, tv);
                if (l == j) z[rj] = xj;
            }
        }
        __syncthreads();
    }
    if (NULLV) {
        double* Nq = N + ((int64_t)f * P + blockIdx.x) * P;
        for (int i = tid; i < P; i += 256) Nq[i] = i == d ? 1.0 : (i < d ? -z[i] : 0.0);
    } else if (OUT64) {
        double* xf = x64 + (int64_t)fit * P;
        for (int i = tid; i < P; i += 256) xf[i] += z[i];
    } else {
        float* df = delta + (int64_t)fit * P;
        for (int i = tid; i < P; i += 256) df[i] = (float)(-z[i]);
    }
}

// r[fit] = c[csrc[q]] - (G[f] + diag(lamp[fit])) x[fit] for fit = fits[q], f = fsrc[q]: the
// float64 Gram-space residual of a squared-loss fit.  G[f] is read from the f32 upper triangle
// H[hsrc[f]] (exact integer counts of a 0/1 mask Gram), a mixed design's continuous rows and
// columns (cmap[j] = c >= 0) from the float64 rows S[f][c][0 .. P).  Coordinates excluded
// (dshift < 0) contribute nothing.  One workgroup per fit: pass A, a wave per row j, the
// upper part sum_{i >= j} G[j][i] x[i] (coalesced row reads, wave reduction); pass B, a lane per
// column i, the lower part sum_{j < i} G[j][i] x[j] (coalesced per j).  Deterministic.
__device__ __forceinline__ double g_upper(const float* __restrict__ Hs, const double* __restrict__ Sf,
                                          const int32_t* __restrict__ cm, int32_t P, int j, int i) {
    if (Sf) {
        const int cj = cm[j];
        if (cj >= 0) return Sf[(int64_t)cj * P + i];
        const int ci = cm[i];
        if (ci >= 0) return Sf[(int64_t)ci * P + j];
    }
    return (double)Hs[(int64_t)j * P + i];
}

__global__ void __launch_bounds__(256) c64_resid_kernel(
    const float* __restrict__ H, int32_t P, const int32_t* __restrict__ hsrc,
    const double* __restrict__ S, int32_t k, const int32_t* __restrict__ cmap,
    const int32_t* __restrict__ fits, const int32_t* __restrict__ fsrc,
    const int32_t* __restrict__ csrc, const double* __restrict__ c,
    const double* __restrict__ lamp, const float* __restrict__ dshift,
    const double* __restrict__ x, double* __restrict__ r) {
    extern __shared__ double sh[];
    double* xs = sh;                 // [P] x with excluded coordinates zeroed
    double* up = sh + P;             // [P] pass-A sums
    int32_t* cm = reinterpret_cast<int32_t*>(sh + 2 * P);
    const int q = blockIdx.x, fit = fits[q], f = fsrc[q];
    const float* Hs = H + (int64_t)hsrc[f] * P * P;
    const double* Sf = S ? S + (int64_t)f * k * P : nullptr;
    const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
    const float* dsh = dshift + (int64_t)fit * P;
    for (int i = tid; i < P; i += 256) {
        xs[i] = dsh[i] < 0.0f ? 0.0 : x[(int64_t)fit * P + i];
        cm[i] = S ? cmap[i] : -1;
    }
    __syncthreads();
    for (int j = w; j < P; j += 4) {
        double acc = 0.0;
        for (int i = j + l; i < P; i += 64) acc = fma(g_upper(Hs, Sf, cm, P, j, i), xs[i], acc);
        acc = wave_sum_d(acc);
        if (l == 0) up[j] = acc;
    }
    __syncthreads();
    const double* lp = lamp + (int64_t)fit * P;
    const double* cf = c + (int64_t)csrc[q] * P;
    for (int i = tid; i < P; i += 256) {
        double acc = up[i];
        for (int j = 0; j < i; ++j) acc = fma(g_upper(Hs, Sf, cm, P, j, i), xs[j], acc);
        acc = fma(lp[i], xs[i], acc);
        r[(int64_t)fit * P + i] = dsh[i] < 0.0f ? 0.0 : cf[i] - acc;
    }
}

__device__ __forceinline__ double block_sum(double v, double* red) {
    v = wave_sum_d(v);
    const int tid = threadIdx.x;
    __syncthreads();
    if ((tid & 63) == 0) red[tid >> 6] = v;
    __syncthreads();
    return red[0] + red[1] + red[2] + red[3];
}

// Orthonormalise factor f's null vectors (N[f][0 .. nd)) in their coefficient part (coordinates
// < pw) by classical Gram-Schmidt with reorthogonalisation; the full vectors (intercept entry
// included) follow the same combinations.  One workgroup per factor.
__global__ void __launch_bounds__(256) c64_orth_kernel(double* __restrict__ N, int32_t P,
                                                       int32_t pw,
                                                       const int32_t* __restrict__ counts) {
    extern __shared__ double h[];
    __shared__ double red[4];
    const int f = blockIdx.x;
    const int nd = counts[2 * f];
    const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
    double* Nf = N + (int64_t)f * P * P;
    for (int q = 0; q < nd; ++q) {
        double* v = Nf + (int64_t)q * P;
        for (int pass = 0; pass < 2 && q > 0; ++pass) {
            for (int r = w; r < q; r += 4) {
                const double* Qr = Nf + (int64_t)r * P;
                double acc = 0.0;
                for (int i = l; i < pw; i += kB) acc = fma(Qr[i], v[i], acc);
                acc = wave_sum_d(acc);
                if (l == 0) h[r] = acc;
            }
            __syncthreads();
            for (int i = tid; i < P; i += 256) {
                double acc = v[i];
                for (int r = 0; r < q; ++r) acc = fma(-h[r], Nf[(int64_t)r * P + i], acc);
                v[i] = acc;
            }
            __syncthreads();
        }
        double s = 0.0;
        for (int i = tid; i < pw; i += 256) s = fma(v[i], v[i], s);
        s = block_sum(s, red);
        const double inv = s > 0.0 ? 1.0 / sqrt(s) : 0.0;
        for (int i = tid; i < P; i += 256) v[i] *= inv;
        __syncthreads();
    }
}

// w <- w - sum_q Q_q (Q_q,w . w) for fit fits[k] on factor fsrc[k] (its orthonormalised null
// vectors Q = N[fsrc[k]]): the minimum-norm point of the fit's solution set.
__global__ void __launch_bounds__(256) c64_project_kernel(
    const double* __restrict__ N, int32_t P, int32_t pw, const int32_t* __restrict__ counts,
    const int32_t* __restrict__ fits, const int32_t* __restrict__ fsrc, double* __restrict__ beta) {
    extern __shared__ double a[];
    const int f = fsrc[blockIdx.x];
    const int nd = counts[2 * f];
    if (nd == 0) return;
    const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
    const double* Nf = N + (int64_t)f * P * P;
    double* wv = beta + (int64_t)fits[blockIdx.x] * P;
    for (int q = w; q < nd; q += 4) {
        const double* Qq = Nf + (int64_t)q * P;
        double acc = 0.0;
        for (int i = l; i < pw; i += kB) acc = fma(Qq[i], wv[i], acc);
        acc = wave_sum_d(acc);
        if (l == 0) a[q] = acc;
    }
    __syncthreads();
    for (int i = tid; i < P; i += 256) {
        double acc = wv[i];
        for (int q = 0; q < nd; ++q) acc = fma(-a[q], Nf[(int64_t)q * P + i], acc);
        wv[i] = acc;
    }
}

// dynamic LDS above the default 64 KiB per workgroup (P > 8000 vectors) must be opted into
template <typename K>
int allow_lds(K kernel, size_t bytes) {
    if (bytes <= 65536) return SGLM_OK;
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(kernel),
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes) != hipSuccess) {
        set_error("chol64: cannot reserve %zu bytes of LDS", bytes);
        return SGLM_EHIP;
    }
    return SGLM_OK;
}

}  // namespace
}  // namespace sglm

using namespace sglm;

extern "C" size_t sglm_chol64_work_bytes(int32_t P, int32_t nf) {
    return (size_t)(nf > 0 ? nf : 0) * (size_t)(P > 0 ? P : 0) * sizeof(double);
}

extern "C" int sglm_chol64_factor(const float* H, int32_t P, const int32_t* hsrc,
                                  const float* dshift, const double* lamp, const int32_t* dsrc,
                                  int32_t nf, double tol, double* U, uint8_t* state,
                                  int32_t* nulls, int32_t* counts, void* work,
                                  sglm_stream_t stream) {
    return sglm_chol64_factor_mixed(H, P, hsrc, dshift, lamp, dsrc, nf, tol, nullptr, 0, nullptr,
                                    U, state, nulls, counts, work, stream);
}

extern "C" int sglm_chol64_factor_mixed(const float* H, int32_t P, const int32_t* hsrc,
                                        const float* dshift, const double* lamp,
                                        const int32_t* dsrc, int32_t nf, double tol,
                                        const double* S, int32_t k, const int32_t* cmap,
                                        double* U, uint8_t* state, int32_t* nulls,
                                        int32_t* counts, void* work, sglm_stream_t stream) {
    if (nf <= 0) return SGLM_OK;
    if (!H || !hsrc || !dshift || !dsrc || !U || !state || !nulls || !counts || !work ||
        P <= 0 || P % kB || P > kMaxP64 || !(tol >= 0.0) || (S && (k <= 0 || !cmap))) {
        set_error("sglm_chol64_factor: bad args (P=%d must be a multiple of %d, <= %d)", P, kB,
                  kMaxP64);
        return SGLM_EINVAL;
    }
    hipStream_t s = as_stream(stream);
    const int nb = P / kB;
    double* d0 = (double*)work;
    c64_init_kernel<<<dim3((unsigned)(nb * (nb + 1) / 2), (unsigned)nf), 256, 0, s>>>(
        H, P, hsrc, dshift, lamp, dsrc, S, k, cmap, U, state, d0);
    for (int kb = 0; kb < nb; ++kb) {
        c64_diag_kernel<<<nf, kB, 0, s>>>(U, P, kb, state, d0, tol);
        const int m = nb - kb - 1;
        if (m == 0) break;
        c64_panel_kernel<<<dim3((unsigned)m, (unsigned)nf), kB, 0, s>>>(U, P, kb, state);
        c64_update_kernel<<<dim3((unsigned)(m * (m + 1) / 2), (unsigned)nf), 256, 0, s>>>(U, P,
                                                                                            kb);
    }
    c64_list_kernel<<<nf, kB, 0, s>>>(state, P, nulls, counts);
    return check_launch("sglm_chol64_factor");
}

extern "C" int sglm_chol64_solve(const double* U, int32_t P, const uint8_t* state,
                                 const int32_t* fits, const int32_t* fsrc, int32_t nq,
                                 const double* g, float* delta, sglm_stream_t stream) {
    if (nq <= 0) return SGLM_OK;
    if (!U || !state || !fits || !fsrc || !g || !delta || P <= 0 || P % kB || P > kMaxP64) {
        set_error("sglm_chol64_solve: bad args (P=%d)", P);
        return SGLM_EINVAL;
    }
    const size_t lds = (size_t)P * sizeof(double);
    if (int st = allow_lds(c64_solve_kernel<false>, lds)) return st;
    c64_solve_kernel<false><<<nq, 256, lds, as_stream(stream)>>>(
        U, P, state, fits, fsrc, g, delta, nullptr, nullptr, nullptr);
    return check_launch("sglm_chol64_solve");
}

extern "C" int sglm_chol64_solve_add(const double* U, int32_t P, const uint8_t* state,
                                     const int32_t* fits, const int32_t* fsrc,
                                     const int32_t* gsrc, int32_t nq, const double* g,
                                     double* x, sglm_stream_t stream) {
    if (nq <= 0) return SGLM_OK;
    if (!U || !state || !fits || !fsrc || !g || !x || P <= 0 || P % kB || P > kMaxP64) {
        set_error("sglm_chol64_solve_add: bad args (P=%d)", P);
        return SGLM_EINVAL;
    }
    const size_t lds = (size_t)P * sizeof(double);
    if (int st = allow_lds(c64_solve_kernel<false, true>, lds)) return st;
    c64_solve_kernel<false, true><<<nq, 256, lds, as_stream(stream)>>>(
        U, P, state, fits, fsrc, g, nullptr, nullptr, nullptr, nullptr, x, gsrc);
    return check_launch("sglm_chol64_solve_add");
}

extern "C" int sglm_chol64_resid(const float* H, int32_t P, const int32_t* hsrc, const double* S,
                                 int32_t k, const int32_t* cmap, const int32_t* fits,
                                 const int32_t* fsrc, const int32_t* csrc, int32_t nq,
                                 const double* c, const double* lamp, const float* dshift,
                                 const double* x, double* r, sglm_stream_t stream) {
    if (nq <= 0) return SGLM_OK;
    if (!H || !hsrc || !fits || !fsrc || !csrc || !c || !lamp || !dshift || !x || !r ||
        P <= 0 || P % kB || P > kMaxP64 || (S && (k <= 0 || !cmap))) {
        set_error("sglm_chol64_resid: bad args (P=%d)", P);
        return SGLM_EINVAL;
    }
    const size_t lds = (size_t)P * (2 * sizeof(double) + sizeof(int32_t));
    if (int st = allow_lds(c64_resid_kernel, lds)) return st;
    c64_resid_kernel<<<nq, 256, lds, as_stream(stream)>>>(H, P, hsrc, S, k, cmap, fits, fsrc, csrc,
                                                         c, lamp, dshift, x, r);
    return check_launch("sglm_chol64_resid");
}

extern "C" size_t sglm_chol64_minnorm_work_bytes(int32_t P, int32_t nf) {
    return (size_t)(nf > 0 ? nf : 0) * (size_t)(P > 0 ? P : 0) * (size_t)(P > 0 ? P : 0) *
           sizeof(double);
}

extern "C" int sglm_chol64_minnorm(const double* U, int32_t P, int32_t pw, const uint8_t* state,
                                   const int32_t* nulls, const int32_t* counts, int32_t nf,
                                   const int32_t* fits, const int32_t* fsrc, int32_t nfit,
                                   double* beta, void* work, sglm_stream_t stream) {
    if (nf <= 0 || nfit <= 0) return SGLM_OK;
    if (!U || !state || !nulls || !counts || !fits || !fsrc || !beta || !work || P <= 0 ||
        P % kB || P > kMaxP64 || pw < 0 || pw > P) {
        set_error("sglm_chol64_minnorm: bad args (P=%d, pw=%d)", P, pw);
        return SGLM_EINVAL;
    }
    hipStream_t s = as_stream(stream);
    double* N = (double*)work;
    const size_t lds = (size_t)P * sizeof(double);
    int st;
    if ((st = allow_lds(c64_solve_kernel<true>, lds)) || (st = allow_lds(c64_orth_kernel, lds)) ||
        (st = allow_lds(c64_project_kernel, lds)))
        return st;
    c64_solve_kernel<true><<<dim3((unsigned)P, (unsigned)nf), 256, lds, s>>>(
        U, P, state, nullptr, nullptr, nullptr, nullptr, nulls, counts, N);
    c64_orth_kernel<<<nf, 256, lds, s>>>(N, P, pw, counts);
    c64_project_kernel<<<nfit, 256, lds, s>>>(N, P, pw, counts, fits, fsrc, beta);
    return check_launch("sglm_chol64_minnorm");
}
