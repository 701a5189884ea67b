// Gram-space cyclic coordinate descent for Lasso / ElasticNet.
//
// Replaces sklearn's cd_fast.enet_coordinate_descent reached through
// backend/sglm.py:106-110 (Lasso / ElasticNet), objective
//   1/(2n) ||y - Xw - b||^2 + alpha rho |w|_1 + alpha (1 - rho)/2 ||w||^2
// (sklearn/linear_model/_coordinate_descent.py:420-422), on centred data.  Multiplied by n:
//   1/2 w^T Q w - q^T w + l1 |w|_1 + l2/2 |w|^2,  l1 = alpha rho n, l2 = alpha (1-rho) n,
// with Q = X_c^T X_c and q = X_c^T y_c taken from the augmented Gram that sglm_syrk forms
// with W = mask (ones column at index p):
//   Q_jk = G_jk - G_jp G_kp / G_pp,   q_j = c_j - G_jp * c_p / G_pp,   c = X^T (m y).
// Q is formed once per mask (center_gram) and shared by every fit of that mask; the CD kernels
// run several fits of one Q per workgroup, float64 throughout.
#include "common.h"

namespace sglm {

constexpr int kCDT = 256;
constexpr int kCDMaxP = 4096;

__device__ __forceinline__ float gram_at(const float* G, int P, int a, int b) {
    return a <= b ? G[(int64_t)a * P + b] : G[(int64_t)b * P + a];
}

// ---------------------------------------------------------------------------------------
// Shared-Gram form for many fits per mask (multi-response lambda paths):
//   center_gram: Q_m = G_xx - g g^T / n (fit_intercept) or G_xx, float64, once per mask;
//   enet_cd_shared: one workgroup per fit, Q_m addressed by qidx[fit], q (the centred
//   X^T y of the fit) given; no per-fit copy of the p x p matrix.
__global__ void __launch_bounds__(256) center_gram_kernel(const float* __restrict__ Hall,
                                                          int32_t P, int32_t p,
                                                          const int32_t* __restrict__ gram_of,
                                                          int32_t center,
                                                          double* __restrict__ Qall) {
    const int m = blockIdx.y;
    const float* G = Hall + (int64_t)gram_of[m] * P * P;
    double* Q = Qall + (int64_t)m * p * p;
    const double n = (double)G[(int64_t)p * P + p];
    for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < (int64_t)p * p;
         e += (int64_t)gridDim.x * 256) {
        const int a = (int)(e / p), b = (int)(e % p);
        double q = (double)gram_at(G, P, a, b);
        if (center && n > 0) q -= (double)G[(int64_t)a * P + p] * (double)G[(int64_t)b * P + p] / n;
        Q[e] = q;
    }
}

__global__ void __launch_bounds__(kCDT) enet_cd_shared_kernel(
    const double* __restrict__ Qall, int32_t p, const int32_t* __restrict__ qidx,
    const double* __restrict__ qv, const double* __restrict__ l1v,
    const double* __restrict__ l2v, int32_t max_sweeps, double tol, double* __restrict__ wout,
    int32_t* __restrict__ sweeps_out) {
    __shared__ double w[kCDMaxP];
    __shared__ double hv[kCDMaxP];
    __shared__ double s_delta[2], s_maxdw, s_maxw;
    const int f = blockIdx.x;
    const double* Q = Qall + (int64_t)qidx[f] * p * p;
    const double* q = qv + (int64_t)f * p;
    const double l1 = l1v[f], l2 = l2v[f];
    const int tid = threadIdx.x;
    for (int j = tid; j < p; j += kCDT) {
        hv[j] = -q[j];
        w[j] = 0.0;
    }
    __syncthreads();
    int sweep = 0;
    for (; sweep < max_sweeps; ++sweep) {
        if (tid == 0) { s_maxdw = 0.0; s_maxw = 0.0; }
        for (int j = 0; j < p; ++j) {
            if (tid == 0) {
                double d = 0.0;
                const double qjj = Q[(int64_t)j * p + j];
                if (qjj > 0.0) {
                    const double wj = w[j];
                    const double rho = -(hv[j] - qjj * wj);
                    const double mag = fabs(rho) - l1;
                    const double nw = mag > 0.0 ? copysign(mag, rho) / (qjj + l2) : 0.0;
                    d = nw - wj;
                    w[j] = nw;
                    s_maxdw = fmax(s_maxdw, fabs(d));
                    s_maxw = fmax(s_maxw, fabs(nw));
                }
                s_delta[j & 1] = d;
            }
            __syncthreads();
            const double d = s_delta[j & 1];
            if (d != 0.0) {
                const double* Qj = Q + (int64_t)j * p;
                for (int k = tid; k < p; k += kCDT) hv[k] += Qj[k] * d;
                __syncthreads();
            }
        }
        __syncthreads();
        const double mdw = s_maxdw, mw = s_maxw;
        __syncthreads();
        if (mw == 0.0 || mdw <= tol * mw) { ++sweep; break; }
    }
    for (int j = tid; j < p; j += kCDT) wout[(int64_t)f * p + j] = w[j];
    if (tid == 0) sweeps_out[f] = sweep;
}

// Several fits of one shared Q per workgroup (C5: 1280 fits per mask).  The coordinate step
// reads row j of Q once for all FPW fits (the row stream, not the arithmetic, bounds the dense
// fits of a lambda path), each fit's decision runs on its own thread, and the fits' running
// gradients hv and coefficients w live in dynamic LDS (2 x FPW x p doubles, plus Q's diagonal).  A fit that has
// converged stops moving; the workgroup ends when all its fits have.
template <int FPW>
__global__ void __launch_bounds__(kCDT) enet_cd_multi_kernel(
    const double* __restrict__ Qall, int32_t p, const int32_t* __restrict__ wg_fits,
    const int32_t* __restrict__ wg_q, const double* __restrict__ qv,
    const double* __restrict__ l1v, const double* __restrict__ l2v, int32_t max_sweeps,
    double tol, double* __restrict__ wout, int32_t* __restrict__ sweeps_out) {
    extern __shared__ double lds[];
    double* hv = lds;                               // [FPW][p]
    double* w = lds + (size_t)FPW * p;              // [FPW][p]
    double* qd = lds + (size_t)2 * FPW * p;         // [p] diagonal of Q
    __shared__ double s_d[2][FPW], s_maxdw[FPW], s_maxw[FPW];
    __shared__ int s_act[FPW], s_nact;
    const int tid = threadIdx.x;
    const double* Q = Qall + (int64_t)wg_q[blockIdx.x] * p * p;
    int f_me = -1;                                  // thread i < FPW owns fit slot i
    double l1 = 0.0, l2 = 0.0;
    if (tid < FPW) {
        f_me = wg_fits[blockIdx.x * FPW + tid];
        s_act[tid] = f_me >= 0;
        if (f_me >= 0) { l1 = l1v[f_me]; l2 = l2v[f_me]; }
    }
    for (int i = 0; i < FPW; ++i) {
        const int f = wg_fits[blockIdx.x * FPW + i];
        for (int j = tid; j < p; j += kCDT) {
            hv[i * p + j] = f >= 0 ? -qv[(int64_t)f * p + j] : 0.0;
            w[i * p + j] = 0.0;
        }
    }
    for (int j = tid; j < p; j += kCDT) qd[j] = Q[(int64_t)j * p + j];
    if (tid == 0) {
        int a = 0;
        for (int i = 0; i < FPW; ++i) a += wg_fits[blockIdx.x * FPW + i] >= 0;
        s_nact = a;
    }
    __syncthreads();
    // row j+1 of Q is loaded into registers while coordinate j is decided and applied, so the
    // global-load latency of the next row overlaps the barriers instead of following them
    constexpr int kRowRegs = (kCDMaxP + kCDT - 1) / kCDT;
    const int nr = (p + kCDT - 1) / kCDT;
    double qn[kRowRegs];
    int sweep = 0;
    for (; sweep < max_sweeps && s_nact > 0; ++sweep) {
        if (tid < FPW) { s_maxdw[tid] = 0.0; s_maxw[tid] = 0.0; }
#pragma unroll
        for (int r = 0; r < kRowRegs; ++r) {
            const int k = tid + r * kCDT;
            qn[r] = (r < nr && k < p) ? Q[k] : 0.0;
        }
        for (int j = 0; j < p; ++j) {
            double qc[kRowRegs];
#pragma unroll
            for (int r = 0; r < kRowRegs; ++r) qc[r] = qn[r];
            if (j + 1 < p) {
                const double* Qn = Q + (int64_t)(j + 1) * p;
#pragma unroll
                for (int r = 0; r < kRowRegs; ++r) {
                    const int k = tid + r * kCDT;
                    if (r < nr && k < p) qn[r] = Qn[k];
                }
            }
            if (tid < FPW) {
                const double qjj = qd[j];
                double d = 0.0;
                if (s_act[tid] && qjj > 0.0) {
                    double* wi = w + tid * p;
                    const double wj = wi[j];
                    const double rho = -(hv[tid * p + j] - qjj * wj);
                    const double mag = fabs(rho) - l1;
                    const double nw = mag > 0.0 ? copysign(mag, rho) / (qjj + l2) : 0.0;
                    d = nw - wj;
                    wi[j] = nw;
                    s_maxdw[tid] = fmax(s_maxdw[tid], fabs(d));
                    s_maxw[tid] = fmax(s_maxw[tid], fabs(nw));
                }
                s_d[j & 1][tid] = d;
            }
            __syncthreads();
            double dv[FPW];
            bool any = false;
#pragma unroll
            for (int i = 0; i < FPW; ++i) {
                dv[i] = s_d[j & 1][i];
                any |= dv[i] != 0.0;
            }
            if (any) {
#pragma unroll
                for (int r = 0; r < kRowRegs; ++r) {
                    const int k = tid + r * kCDT;
                    if (r < nr && k < p) {
#pragma unroll
                        for (int i = 0; i < FPW; ++i) hv[i * p + k] += qc[r] * dv[i];
                    }
                }
                __syncthreads();
            }
        }
        __syncthreads();
        if (tid < FPW && s_act[tid]) {
            const double mdw = s_maxdw[tid], mw = s_maxw[tid];
            if (mw == 0.0 || mdw <= tol * mw) {
                s_act[tid] = 0;
                sweeps_out[f_me] = sweep + 1;
            }
        }
        __syncthreads();
        if (tid == 0) {
            int a = 0;
            for (int i = 0; i < FPW; ++i) a += s_act[i];
            s_nact = a;
        }
        __syncthreads();
    }
    if (tid < FPW && f_me >= 0 && s_act[tid]) sweeps_out[f_me] = sweep;
    for (int i = 0; i < FPW; ++i) {
        const int f = wg_fits[blockIdx.x * FPW + i];
        if (f < 0) continue;
        for (int j = tid; j < p; j += kCDT) wout[(int64_t)f * p + j] = w[i * p + j];
    }
}

// Register-resident form (p <= kCDT * kRegRows): thread t owns coordinates k = t + kCDT r; it
// holds those coordinates' running gradients hv, coefficients w and Q diagonal for all FPW
// fits in registers.  Coordinate j's owner decides the FPW fits' moves on its own and
// publishes them (double-buffered by j parity); after ONE barrier every thread folds row j of
// Q (prefetched into registers one coordinate ahead) into its hv.  No LDS traffic on the
// gradient, one barrier per coordinate.
constexpr int kRegRows = 8;

template <int FPW>
__global__ void __launch_bounds__(kCDT) enet_cd_reg_kernel(
    const double* __restrict__ Qall, int32_t p, const int32_t* __restrict__ wg_fits,
    const int32_t* __restrict__ wg_q, const double* __restrict__ qv,
    const double* __restrict__ l1v, const double* __restrict__ l2v, int32_t max_sweeps,
    double tol, double* __restrict__ wout, int32_t* __restrict__ sweeps_out) {
    __shared__ double s_d[2][FPW];
    __shared__ double s_red[2][FPW][kCDT / 64];
    __shared__ int s_act[FPW];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const double* Q = Qall + (int64_t)wg_q[blockIdx.x] * p * p;
    int fit[FPW];
    double l1[FPW], l2[FPW];
#pragma unroll
    for (int i = 0; i < FPW; ++i) {
        fit[i] = wg_fits[blockIdx.x * FPW + i];
        l1[i] = fit[i] >= 0 ? l1v[fit[i]] : 0.0;
        l2[i] = fit[i] >= 0 ? l2v[fit[i]] : 0.0;
    }
    double hv[FPW][kRegRows], w[FPW][kRegRows], qdg[kRegRows], qn[kRegRows];
#pragma unroll
    for (int r = 0; r < kRegRows; ++r) {
        const int k = tid + r * kCDT;
        const bool ok = k < p;
        qdg[r] = ok ? Q[(int64_t)k * p + k] : 0.0;
#pragma unroll
        for (int i = 0; i < FPW; ++i) {
            hv[i][r] = (ok && fit[i] >= 0) ? -qv[(int64_t)fit[i] * p + k] : 0.0;
            w[i][r] = 0.0;
        }
    }
    bool act[FPW];
#pragma unroll
    for (int i = 0; i < FPW; ++i) act[i] = fit[i] >= 0;
    int sweep = 0;
    int sw_done[FPW];
#pragma unroll
    for (int i = 0; i < FPW; ++i) sw_done[i] = max_sweeps;
    for (; sweep < max_sweeps; ++sweep) {
        bool anyact = false;
#pragma unroll
        for (int i = 0; i < FPW; ++i) anyact |= act[i];
        if (!anyact) break;
        double mdw[FPW], mw[FPW];
#pragma unroll
        for (int i = 0; i < FPW; ++i) { mdw[i] = 0.0; mw[i] = 0.0; }
#pragma unroll
        for (int r = 0; r < kRegRows; ++r) {
            const int k = tid + r * kCDT;
            qn[r] = k < p ? Q[k] : 0.0;                       // row 0
        }
#pragma unroll
        for (int rr = 0; rr < kRegRows; ++rr) {               // owner register of coordinate j
            for (int t = 0; t < kCDT; ++t) {
                const int j = t + rr * kCDT;
                if (j >= p) break;                            // uniform
                double qc[kRegRows];
#pragma unroll
                for (int r = 0; r < kRegRows; ++r) qc[r] = qn[r];
                if (j + 1 < p) {
                    const double* Qn = Q + (int64_t)(j + 1) * p;
#pragma unroll
                    for (int r = 0; r < kRegRows; ++r) {
                        const int k = tid + r * kCDT;
                        if (k < p) qn[r] = Qn[k];
                    }
                }
                if (tid == t) {                               // the owner decides
                    const double qjj = qdg[rr];
#pragma unroll
                    for (int i = 0; i < FPW; ++i) {
                        double d = 0.0;
                        if (act[i] && qjj > 0.0) {
                            const double wj = w[i][rr];
                            const double rho = -(hv[i][rr] - qjj * wj);
                            const double mag = fabs(rho) - l1[i];
                            const double nw = mag > 0.0 ? copysign(mag, rho) / (qjj + l2[i]) : 0.0;
                            d = nw - wj;
                            w[i][rr] = nw;
                            mdw[i] = fmax(mdw[i], fabs(d));
                            mw[i] = fmax(mw[i], fabs(nw));
                        }
                        s_d[j & 1][i] = d;
                    }
                }
                __syncthreads();
                double dv[FPW];
                bool any = false;
#pragma unroll
                for (int i = 0; i < FPW; ++i) {
                    dv[i] = s_d[j & 1][i];
                    any |= dv[i] != 0.0;
                }
                if (any) {
#pragma unroll
                    for (int r = 0; r < kRegRows; ++r)
#pragma unroll
                        for (int i = 0; i < FPW; ++i) hv[i][r] = fma(qc[r], dv[i], hv[i][r]);
                }
            }
        }
        // per-fit convergence: block max of the sweep's max |dw| and max |w|
#pragma unroll
        for (int i = 0; i < FPW; ++i) {
            double a = mdw[i], b = mw[i];
            for (int o = 32; o > 0; o >>= 1) {
                a = fmax(a, __shfl_xor(a, o, 64));
                b = fmax(b, __shfl_xor(b, o, 64));
            }
            if (lane == 0) { s_red[0][i][wave] = a; s_red[1][i][wave] = b; }
        }
        __syncthreads();
        if (tid < FPW && act[tid > FPW ? 0 : tid]) {
            double a = 0.0, b = 0.0;
            for (int v = 0; v < kCDT / 64; ++v) {
                a = fmax(a, s_red[0][tid][v]);
                b = fmax(b, s_red[1][tid][v]);
            }
            s_act[tid] = !(b == 0.0 || a <= tol * b);
        }
        __syncthreads();
#pragma unroll
        for (int i = 0; i < FPW; ++i) {
            if (act[i] && !s_act[i]) sw_done[i] = sweep + 1;
            act[i] = act[i] && s_act[i];
        }
        __syncthreads();
    }
#pragma unroll
    for (int i = 0; i < FPW; ++i) {
        if (fit[i] < 0) continue;
        if (tid == 0) sweeps_out[fit[i]] = sw_done[i];
#pragma unroll
        for (int r = 0; r < kRegRows; ++r) {
            const int k = tid + r * kCDT;
            if (k < p) wout[(int64_t)fit[i] * p + k] = w[i][r];
        }
    }
}

// Lane-parallel decisions (enet_cd_lane_kernel): thread t owns coordinates k = t + NT r
// (r < RR) and holds their running gradients hv for all FPW fits of the workgroup; the FPW
// decisions of coordinate j run on FPW lanes of the owner's wave at once (lane i = fit i,
// the owner's hv[i] brought over by v_readlane) instead of one after another on the owner
// thread, the divisions overlapping.  The coefficients w live in dynamic LDS ([FPW][p], only
// the deciding lane touches them), Q rows are prefetched D coordinates ahead in a register
// ring, and consecutive workgroups (fits of one Q and one alpha: equal sweep counts, equal
// pace) are placed on one XCD, so a Q row fetched for one of them is an L2 hit for the others.
// Per coordinate the arithmetic and the fold order are enet_cd_reg_kernel's: the coefficients
// are the same bit for bit.
__device__ __forceinline__ double readlane_d(double v, int l) {
    const uint64_t u = __builtin_bit_cast(uint64_t, v);
    const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)u, l);
    const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(u >> 32), l);
    return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}

template <int FPW, int NT, int RR, int D>
__global__ void __launch_bounds__(NT) enet_cd_lane_kernel(
    const double* __restrict__ Qall, int32_t p, const int32_t* __restrict__ wg_fits,
    const int32_t* __restrict__ wg_q, const double* __restrict__ qv,
    const double* __restrict__ l1v, const double* __restrict__ l2v, int32_t max_sweeps,
    double tol, double* __restrict__ wout, int32_t* __restrict__ sweeps_out, int32_t nwg) {
    static_assert(NT % D == 0 && FPW <= 64, "ring tiles the owner loop; one wave of deciders");
    extern __shared__ double s_w[];                   // [FPW][p] coefficients
    __shared__ double s_d[2][FPW];
    __shared__ double s_red[2][FPW][NT / 64];
    __shared__ int s_act[FPW];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int L = xcd_logical(blockIdx.x, nwg);
    const double* Q = Qall + (int64_t)wg_q[L] * p * p;
    const int* fits = wg_fits + (int64_t)L * FPW;
    // decision lane constants (lane i < FPW of every wave decides fit i)
    const bool dl = lane < FPW;
    const int fl = fits[dl ? lane : 0];
    const double l1 = (dl && fl >= 0) ? l1v[fl] : 0.0;
    const double l2 = (dl && fl >= 0) ? l2v[fl] : 0.0;
    bool act = dl && fl >= 0;
    int sw_done = max_sweeps;
    double hv[FPW][RR], qdg[RR], qb[D][RR];
#pragma unroll
    for (int r = 0; r < RR; ++r) {
        const int k = tid + r * NT;
        const bool ok = k < p;
        qdg[r] = ok ? Q[(int64_t)k * p + k] : 0.0;
#pragma unroll
        for (int i = 0; i < FPW; ++i) {
            const int f = fits[i];
            hv[i][r] = (ok && f >= 0) ? -qv[(int64_t)f * p + k] : 0.0;
            if (ok) s_w[i * p + k] = 0.0;
        }
    }
    __syncthreads();
    for (int sweep = 0; sweep < max_sweeps; ++sweep) {
        if (!__syncthreads_or(act ? 1 : 0)) break;
        double mdw = 0.0, mw = 0.0;
#pragma unroll
        for (int u = 0; u < D; ++u)                           // rows 0 .. D-1
#pragma unroll
            for (int r = 0; r < RR; ++r) {
                const int k = tid + r * NT;
                qb[u][r] = (u < p && k < p) ? Q[(int64_t)u * p + k] : 0.0;
            }
#pragma unroll
        for (int rr = 0; rr < RR; ++rr) {                     // owner register of coordinate j
            if (rr * NT >= p) break;                          // uniform
            for (int t0 = 0; t0 < NT; t0 += D) {
                if (t0 + rr * NT >= p) break;                 // uniform
#pragma unroll
                for (int u = 0; u < D; ++u) {
                    const int t = t0 + u;
                    const int j = t + rr * NT;
                    if (j >= p) break;                        // uniform
                    double qc[RR];
#pragma unroll
                    for (int r = 0; r < RR; ++r) qc[r] = qb[u][r];
                    if (j + D < p) {                          // row j + D into the freed slot
                        const double* Qn = Q + (int64_t)(j + D) * p;
#pragma unroll
                        for (int r = 0; r < RR; ++r) {
                            const int k = tid + r * NT;
                            if (k < p) qb[u][r] = Qn[k];
                        }
                    }
                    if (wave == (t >> 6)) {                   // the owner's wave decides
                        const int ol = t & 63;
                        double h = 0.0;
#pragma unroll
                        for (int i = 0; i < FPW; ++i) {
                            const double x = readlane_d(hv[i][rr], ol);
                            h = lane == i ? x : h;
                        }
                        const double qjj = readlane_d(qdg[rr], ol);
                        if (dl) {
                            double d = 0.0;
                            if (act && qjj > 0.0) {
                                const double wj = s_w[lane * p + j];
                                const double rho = -(h - qjj * wj);
                                const double mag = fabs(rho) - l1;
                                const double nw = mag > 0.0 ? copysign(mag, rho) / (qjj + l2) : 0.0;
                                d = nw - wj;
                                s_w[lane * p + j] = nw;
                                mdw = fmax(mdw, fabs(d));
                                mw = fmax(mw, fabs(nw));
                            }
                            s_d[j & 1][lane] = d;
                        }
                    }
                    __syncthreads();
                    double dv[FPW];
                    bool any = false;
#pragma unroll
                    for (int i = 0; i < FPW; ++i) {
                        dv[i] = s_d[j & 1][i];
                        any |= dv[i] != 0.0;
                    }
                    if (any) {
#pragma unroll
                        for (int r = 0; r < RR; ++r)
#pragma unroll
                            for (int i = 0; i < FPW; ++i) hv[i][r] = fma(qc[r], dv[i], hv[i][r]);
                    }
                }
            }
        }
        // per-fit convergence: the max over the waves' deciding lanes
        if (dl) {
            s_red[0][lane][wave] = mdw;
            s_red[1][lane][wave] = mw;
        }
        __syncthreads();
        if (tid < FPW) {
            double a = 0.0, b = 0.0;
            for (int v = 0; v < NT / 64; ++v) {
                a = fmax(a, s_red[0][tid][v]);
                b = fmax(b, s_red[1][tid][v]);
            }
            s_act[tid] = !(b == 0.0 || a <= tol * b);
        }
        __syncthreads();
        if (dl) {
            if (act && !s_act[lane]) sw_done = sweep + 1;
            act = act && s_act[lane];
        }
    }
    __syncthreads();
    if (tid < FPW && fl >= 0) sweeps_out[fl] = sw_done;
#pragma unroll
    for (int i = 0; i < FPW; ++i) {
        const int f = fits[i];
        if (f < 0) continue;
        for (int k = tid; k < p; k += NT) wout[(int64_t)f * p + k] = s_w[i * p + k];
    }
}

template <int FPW>
static int launch_cd_multi(const double* Q, int32_t p, const int32_t* wg_fits, int32_t nwg,
                           const int32_t* wg_q, const double* q, const double* l1,
                           const double* l2, int32_t max_sweeps, double tol, double* w,
                           int32_t* sweeps, hipStream_t s) {
    const size_t lds = (size_t)(2 * FPW + 1) * p * sizeof(double);
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(&enet_cd_multi_kernel<FPW>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess) {
        set_error("enet_cd_multi_kernel: %zu bytes of LDS refused", lds);
        return SGLM_EHIP;
    }
    enet_cd_multi_kernel<FPW><<<nwg, kCDT, lds, s>>>(Q, p, wg_fits, wg_q, q, l1, l2, max_sweeps,
                                                   tol, w, sweeps);
    return check_launch("enet_cd_multi_kernel");
}

}  // namespace sglm

using namespace sglm;

// fits per workgroup that the LDS holds ((2 fpw + 1) x p doubles within 160 KiB; 1 if none)
// SGLM_CD_FPW (read per call): 8 (default) = enet_cd_lane_kernel (eight fits per 512-thread
// workgroup), 4 = enet_cd_reg_kernel (four fits, 256 threads)
static int cd_reg_fpw() {
    const char* e = getenv("SGLM_CD_FPW");
    return (e && e[0] == '4') ? 4 : 8;
}

extern "C" int32_t sglm_enet_cd_fits_per_wg(int32_t p) {
    if (p <= kCDT * kRegRows) return cd_reg_fpw();   // register-resident forms
    const int64_t row = (int64_t)p * sizeof(double);
    for (int f : {8, 4, 2})
        if ((2 * f + 1) * row <= 160 * 1024 - 1024) return f;
    return 1;
}

extern "C" int sglm_enet_cd_grouped(const double* Q, int32_t p, const int32_t* wg_fits,
                                    int32_t nwg, int32_t fpw, const int32_t* wg_q,
                                    const double* q, const double* l1, const double* l2,
                                    int32_t max_sweeps, double tol, double* w, int32_t* sweeps,
                                    sglm_stream_t stream) {
    if (nwg <= 0) return SGLM_OK;
    if (!Q || !wg_fits || !wg_q || !q || !l1 || !l2 || !w || !sweeps || p <= 0 ||
        fpw != sglm_enet_cd_fits_per_wg(p) || fpw < 2) {
        set_error("sglm_enet_cd_grouped: bad args (p=%d fpw=%d)", p, fpw);
        return SGLM_EINVAL;
    }
    hipStream_t s = as_stream(stream);
    if (p <= kCDT * kRegRows && fpw == 8) {          // register-resident, lane decisions
        const size_t lds = (size_t)8 * p * sizeof(double);
        if (hipFuncSetAttribute(reinterpret_cast<const void*>(&enet_cd_lane_kernel<8, 512, 4, 2>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) !=
            hipSuccess) {
            set_error("enet_cd_lane_kernel: %zu bytes of LDS refused", lds);
            return SGLM_EHIP;
        }
        enet_cd_lane_kernel<8, 512, 4, 2><<<nwg, 512, lds, s>>>(Q, p, wg_fits, wg_q, q, l1, l2,
                                                                max_sweeps, tol, w, sweeps, nwg);
        return check_launch("enet_cd_lane_kernel");
    }
    if (p <= kCDT * kRegRows && fpw >= 4) {          // register-resident form
        enet_cd_reg_kernel<4><<<nwg, kCDT, 0, s>>>(Q, p, wg_fits, wg_q, q, l1, l2, max_sweeps,
                                                   tol, w, sweeps);
        return check_launch("enet_cd_reg_kernel");
    }
    switch (fpw) {
        case 8: return launch_cd_multi<8>(Q, p, wg_fits, nwg, wg_q, q, l1, l2, max_sweeps, tol, w, sweeps, s);
        case 4: return launch_cd_multi<4>(Q, p, wg_fits, nwg, wg_q, q, l1, l2, max_sweeps, tol, w, sweeps, s);
        default: return launch_cd_multi<2>(Q, p, wg_fits, nwg, wg_q, q, l1, l2, max_sweeps, tol, w, sweeps, s);
    }
}

extern "C" int sglm_center_gram(const float* H, int32_t P, int32_t p, const int32_t* gram_of,
                                int32_t nmask, int32_t center, double* Q, sglm_stream_t stream) {
    if (nmask <= 0) return SGLM_OK;
    if (!H || !gram_of || !Q || p >= P) {
        set_error("sglm_center_gram: bad args");
        return SGLM_EINVAL;
    }
    const int64_t pp = (int64_t)p * p;
    unsigned gx = (unsigned)((pp + 255) / 256 < 2048 ? (pp + 255) / 256 : 2048);
    center_gram_kernel<<<dim3(gx, (unsigned)nmask), 256, 0, as_stream(stream)>>>(H, P, p, gram_of,
                                                                               center, Q);
    return check_launch("center_gram_kernel");
}

extern "C" int sglm_enet_cd_shared(const double* Q, int32_t p, const int32_t* qidx, int32_t nfit,
                                   const double* q, const double* l1, const double* l2,
                                   int32_t max_sweeps, double tol, double* w, int32_t* sweeps,
                                   sglm_stream_t stream) {
    if (nfit <= 0) return SGLM_OK;
    if (!Q || !qidx || !q || !l1 || !l2 || !w || !sweeps || p > kCDMaxP) {
        set_error("sglm_enet_cd_shared: bad args (p=%d, max %d)", p, kCDMaxP);
        return SGLM_EINVAL;
    }
    enet_cd_shared_kernel<<<nfit, kCDT, 0, as_stream(stream)>>>(Q, p, qidx, q, l1, l2, max_sweeps,
                                                                tol, w, sweeps);
    return check_launch("enet_cd_shared_kernel");
}

// ---- fold scores of shared-Gram fits by Gram algebra --------------------------------------
// ss[f] = sum over the rows of a mask of (y - x~ beta_f)^2 = yy[f] - 2 beta_f.c[cidx[f]]
//         + beta_f^T G beta_f, with G the mask's augmented Gram (f32 upper triangle, exact
// integer counts for 0/1 designs), beta_f float64 over the pa = p + 1 active coordinates.
// Quadratic part: workgroup = (row block of 32 rows of G, chunk of 256 fits of one Gram),
// thread = fit; the block's G rows and the fits' beta columns are staged through LDS 32
// columns at a time (beta rows loaded coalesced, read transposed), 32 float64 row
// accumulators per thread; partials per row block, summed in a fixed order with the linear
// term by one wave per fit.
namespace sglm {
namespace {
constexpr int kQR = 32;           // G rows per workgroup
constexpr int kQF = 256;          // fits per workgroup (one per thread)
constexpr int kQC = 32;           // columns per staging step

__global__ void __launch_bounds__(kQF) gram_quad_kernel(const float* __restrict__ H, int32_t P,
                                                        int32_t pa,
                                                        const int32_t* __restrict__ grp_slot,
                                                        const int32_t* __restrict__ grp_off,
                                                        const int32_t* __restrict__ fits,
                                                        const double* __restrict__ beta,
                                                        double* __restrict__ part,
                                                        int32_t nfit) {
    __shared__ float g[kQR][kQC + 1];
    __shared__ double bt[kQF][kQC + 1];
    __shared__ double brow[kQF][kQR + 1];
    const int tid = threadIdx.x;
    const int grp = blockIdx.z;
    const int f0 = grp_off[grp] + blockIdx.y * kQF;
    const int f1 = grp_off[grp + 1];
    if (f0 >= f1) return;
    const int nf = min(kQF, f1 - f0);
    const int a0 = blockIdx.x * kQR;
    if (a0 >= pa) return;
    const float* G = H + (int64_t)grp_slot[grp] * P * P;
    const bool on = tid < nf;
    const int fit = on ? fits[f0 + tid] : 0;
    // this block's beta rows (coordinates a0 .. a0 + 31 of every fit), read transposed
    for (int e = tid; e < nf * kQR; e += kQF) {
        const int ff = e / kQR, j = e - ff * kQR;
        const int a = a0 + j;
        brow[ff][j] = a < pa ? beta[(int64_t)fits[f0 + ff] * P + a] : 0.0;
    }
    double acc[kQR];
#pragma unroll
    for (int j = 0; j < kQR; ++j) acc[j] = 0.0;
    for (int c0 = a0; c0 < pa; c0 += kQC) {
        __syncthreads();
        for (int e = tid; e < kQR * kQC; e += kQF) {
            const int r = e / kQC, c = e - r * kQC;
            const int a = a0 + r, b = c0 + c;
            // strictly upper part only (b > a); the diagonal is added separately
            g[r][c] = (a < pa && b < pa && b > a) ? G[(int64_t)a * P + b] : 0.0f;
        }
        for (int e = tid; e < nf * kQC; e += kQF) {
            const int ff = e / kQC, c = e - ff * kQC;
            const int b = c0 + c;
            bt[ff][c] = b < pa ? beta[(int64_t)fits[f0 + ff] * P + b] : 0.0;
        }
        __syncthreads();
        if (on) {
#pragma unroll 4
            for (int c = 0; c < kQC; ++c) {
                const double bv = bt[tid][c];
#pragma unroll
                for (int j = 0; j < kQR; ++j) acc[j] = fma((double)g[j][c], bv, acc[j]);
            }
        }
    }
    if (!on) return;
    double q = 0.0;
#pragma unroll
    for (int j = 0; j < kQR; ++j) {
        const int a = a0 + j;
        const double ba = brow[tid][j];
        const double gaa = a < pa ? (double)G[(int64_t)a * P + a] : 0.0;
        q += ba * (gaa * ba + 2.0 * acc[j]);
    }
    part[(int64_t)blockIdx.x * nfit + (f0 + tid)] = q;
    (void)fit;
}

// one wave per fit: ss = max(yy - 2 beta.c + sum over row blocks of the quadratic part, 0)
__global__ void __launch_bounds__(256) gram_quad_finish(const double* __restrict__ part,
                                                        int32_t nblk, int32_t nfit,
                                                        const int32_t* __restrict__ fits,
                                                        const double* __restrict__ beta,
                                                        const double* __restrict__ c,
                                                        const int32_t* __restrict__ cidx,
                                                        const double* __restrict__ yy,
                                                        int32_t P, int32_t pa,
                                                        double* __restrict__ ss) {
    const int w = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (w >= nfit) return;
    const double* bf = beta + (int64_t)fits[w] * P;
    const double* cf = c + (int64_t)cidx[w] * P;
    double lin = 0.0;
    for (int a = lane; a < pa; a += 64) lin = fma(bf[a], cf[a], lin);
    for (int o = 32; o > 0; o >>= 1) lin += __shfl_xor(lin, o, 64);
    if (lane == 0) {
        double q = 0.0;
        for (int k = 0; k < nblk; ++k) q += part[(int64_t)k * nfit + w];
        const double v = yy[w] - 2.0 * lin + q;
        ss[w] = v > 0.0 ? v : 0.0;
    }
}
}  // namespace
}  // namespace sglm

extern "C" size_t sglm_gram_ss_work_bytes(int32_t pa, int32_t nfit) {
    return (size_t)((pa + kQR - 1) / kQR) * (size_t)nfit * sizeof(double);
}

extern "C" int sglm_gram_ss(const float* H, int32_t P, int32_t pa, const int32_t* grp_slot,
                            const int32_t* grp_off, int32_t ngrp, int32_t max_per_grp,
                            const int32_t* fits, int32_t nfit, const double* beta,
                            const double* c, const int32_t* cidx, const double* yy, double* ss,
                            void* work, sglm_stream_t stream) {
    if (nfit <= 0) return SGLM_OK;
    if (!H || !grp_slot || !grp_off || !fits || !beta || !c || !cidx || !yy || !ss || !work ||
        pa < 1 || pa > P || ngrp < 1 || ngrp > 65535 || max_per_grp < 1) {
        set_error("sglm_gram_ss: bad args");
        return SGLM_EINVAL;
    }
    hipStream_t s = as_stream(stream);
    const int nblk = (pa + kQR - 1) / kQR;
    dim3 grid((unsigned)nblk, (unsigned)((max_per_grp + kQF - 1) / kQF), (unsigned)ngrp);
    gram_quad_kernel<<<grid, kQF, 0, s>>>(H, P, pa, grp_slot, grp_off, fits, beta,
                                          (double*)work, nfit);
    int st = check_launch("gram_quad_kernel");
    if (st) return st;
    gram_quad_finish<<<(unsigned)((nfit + 3) / 4), 256, 0, s>>>((const double*)work, nblk, nfit,
                                                                fits, beta, c, cidx, yy, P, pa,
                                                                ss);
    return check_launch("gram_quad_finish");
}
