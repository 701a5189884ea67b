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
