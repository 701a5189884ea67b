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
// One workgroup per fit, float64 throughout; the running gradient Qw lives in LDS and only
// changes when a coordinate moves (sparse updates on Lasso paths).
#include "common.h"

namespace sglm {

constexpr int kCDT = 256;
constexpr int kCDMaxP = 4096;

__device__ __forceinline__ float gram_at(const float* G, int P, int a, int b) {
    return a <= b ? G[(int64_t)a * P + b] : G[(int64_t)b * P + a];
}

__global__ void __launch_bounds__(kCDT) enet_cd_kernel(
    const float* __restrict__ Hall, int32_t P, int32_t p, const int32_t* __restrict__ fits,
    const double* __restrict__ call, const double* __restrict__ l1v,
    const double* __restrict__ l2v, const int32_t* __restrict__ fitint, int32_t max_sweeps,
    double tol, double* __restrict__ Qall, double* __restrict__ coef_all,
    int32_t* __restrict__ sweeps_out) {
    __shared__ double w[kCDMaxP];
    __shared__ double hv[kCDMaxP];
    __shared__ double dg[kCDMaxP];
    __shared__ double s_delta[2], s_maxdw, s_maxw;   // s_delta double-buffered by j parity

    const int slot = blockIdx.x;
    const int fit = fits[slot];
    const float* G = Hall + (int64_t)fit * P * P;
    const double* c = call + (int64_t)fit * P;
    double* Q = Qall + (int64_t)slot * p * p;
    const bool fi = fitint[fit] != 0;
    const double l1 = l1v[fit], l2 = l2v[fit];
    const double n = (double)G[(int64_t)p * P + p];
    const double cp = c[p];
    const int tid = threadIdx.x;

    // centred Gram (full symmetric, float64) and centred X^T y
    for (int64_t e = tid; e < (int64_t)p * p; e += kCDT) {
        const int a = (int)(e / p), b = (int)(e % p);
        double q = (double)gram_at(G, P, a, b);
        if (fi && n > 0) q -= (double)G[(int64_t)a * P + p] * (double)G[(int64_t)b * P + p] / n;
        Q[e] = q;
    }
    __syncthreads();
    for (int j = tid; j < p; j += kCDT) {
        double qj = c[j];
        if (fi && n > 0) qj -= (double)G[(int64_t)j * P + p] * cp / n;
        hv[j] = -qj;                 // hv = Q w - q with w = 0
        w[j] = 0.0;
        dg[j] = Q[(int64_t)j * p + j];
    }
    __syncthreads();

    int sweep = 0;
    for (; sweep < max_sweeps; ++sweep) {
        if (tid == 0) { s_maxdw = 0.0; s_maxw = 0.0; }
        for (int j = 0; j < p; ++j) {
            if (tid == 0) {
                double d = 0.0;
                const double qjj = dg[j];
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
    double* out = coef_all + (int64_t)fit * P;
    for (int j = tid; j < P; j += kCDT) out[j] = j < p ? w[j] : 0.0;
    __syncthreads();
    if (tid == 0) {
        double b = 0.0;
        if (fi && n > 0) {
            b = cp / n;
            for (int j = 0; j < p; ++j) b -= (double)G[(int64_t)j * P + p] / n * w[j];
        }
        out[p] = b;
        sweeps_out[fit] = sweep;
    }
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

}  // namespace sglm

using namespace sglm;

extern "C" size_t sglm_enet_work_bytes(int32_t p, int32_t nact) {
    return (size_t)nact * (size_t)p * (size_t)p * sizeof(double);
}

extern "C" int sglm_enet_cd(const float* H, int32_t P, int32_t p, const int32_t* fits,
                            int32_t nact, const double* c, const double* l1, const double* l2,
                            const int32_t* fit_intercept, int32_t max_sweeps, double tol,
                            double* coef, int32_t* sweeps, void* work, sglm_stream_t stream) {
    if (nact <= 0) return SGLM_OK;
    if (!H || !fits || !c || !l1 || !l2 || !fit_intercept || !coef || !sweeps || !work ||
        p >= P || p > kCDMaxP) {
        set_error("sglm_enet_cd: bad args (p=%d P=%d, max p %d)", p, P, kCDMaxP);
        return SGLM_EINVAL;
    }
    enet_cd_kernel<<<nact, kCDT, 0, as_stream(stream)>>>(H, P, p, fits, c, l1, l2, fit_intercept,
                                                         max_sweeps, tol, (double*)work, coef,
                                                         sweeps);
    return check_launch("enet_cd_kernel");
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
