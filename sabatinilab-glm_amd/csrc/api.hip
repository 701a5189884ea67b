// libsglm_hip: design construction, GEMV-class and elementwise kernels of the IRLS step.
// (The bf16-MFMA Gram lives in syrk.hip, the batched Cholesky in chol.hip.)
#include "common.h"

#include <stdarg.h>
#include <string.h>

namespace sglm {

static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

int check_launch(const char* what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_error("%s: %s", what, hipGetErrorString(e));
        return SGLM_EHIP;
    }
    return SGLM_OK;
}

// ------------------------------------------------------------------------------ timeshift
// One output column per blockIdx.y (grid-strided), rows grid-strided over x.  For the
// feature-major engine layout (rs = 1) both the read of the source column segment and the
// write of the output column are contiguous: the lag expansion is a shifted memcpy.
// rows (nullable): output row t reads source row rows[t] - shift instead of t + row0 - shift
// (a row selection of the lagged frame, sglm_timeshift_gather).
template <typename T>
__global__ void __launch_bounds__(256) timeshift_kernel(
    const T* __restrict__ src, int64_t n_src, int64_t rs_src, int64_t cs_src,
    const int32_t* __restrict__ src_col, const int32_t* __restrict__ shift, int32_t ncols,
    T* __restrict__ out, int64_t n_out, int64_t rs_out, int64_t cs_out, int64_t row0, T fill,
    const int64_t* __restrict__ rows) {
    for (int j = blockIdx.y; j < ncols; j += gridDim.y) {
        const int64_t c = src_col[j];
        const int64_t s = shift[j];
        for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n_out;
             t += (int64_t)gridDim.x * blockDim.x) {
            const int64_t r = (rows ? rows[t] : t + row0) - s;
            out[t * rs_out + j * cs_out] =
                (r >= 0 && r < n_src) ? src[r * rs_src + c * cs_src] : fill;
        }
    }
}

// ------------------------------------------------------------------------------ pack
// 64x64 LDS transpose: row-major f32/f64 source -> feature-major bf16 (+ f32).
// dst0: first destination row (a 64-aligned chunk of a chunked upload); src row i goes to
// destination row dst0 + i, and only the tiles covering the chunk are written.
template <typename TS>
__global__ void __launch_bounds__(256) pack_kernel(
    const TS* __restrict__ src, int64_t n, int32_t p, int64_t rs, int64_t cs, int32_t add_ones,
    uint16_t* __restrict__ Xb, float* __restrict__ Xf, int64_t ld, int32_t* inexact,
    int64_t dst0 = 0, int32_t* __restrict__ colflag = nullptr) {
    __shared__ float tile[64][65];
    __shared__ int nonbin[64];
    const int64_t i0 = (int64_t)blockIdx.x * 64;
    const int32_t a0 = blockIdx.y * 64;
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;   // 64 x 4
    int bad = 0, nb = 0;
    if (threadIdx.x < 64) nonbin[threadIdx.x] = 0;
    for (int r = ty; r < 64; r += 4) {           // r: row i offset, tx: column a offset
        const int64_t i = i0 + r;
        const int32_t a = a0 + tx;
        float v = 0.0f;
        if (i < n) {
            if (a < p) {
                const TS sv = src[i * rs + (int64_t)a * cs];
                v = (float)sv;
                nb |= !(sv == (TS)0 || sv == (TS)1);    // NaN included
            } else if (a == p && add_ones) {
                v = 1.0f;
            }
        }
        tile[r][tx] = v;
    }
    __syncthreads();
    // per-column "holds a value other than 0 / 1" flags (mixed designs), judged on the source
    // values before any rounding
    if (colflag && nb) atomicOr(&nonbin[tx], 1);
    __syncthreads();
    if (colflag && threadIdx.x < 64 && nonbin[threadIdx.x] && a0 + (int)threadIdx.x < p &&
        !colflag[a0 + threadIdx.x])
        atomicOr(&colflag[a0 + threadIdx.x], 1);
    for (int c = ty; c < 64; c += 4) {           // c: column a offset, tx: row i offset
        const float v = tile[tx][c];
        const __bf16 hb = (__bf16)v;
        bad |= ((float)hb != v);
        const int64_t off = (int64_t)(a0 + c) * ld + dst0 + i0 + tx;
        Xb[off] = __builtin_bit_cast(uint16_t, hb);
        if (Xf) Xf[off] = v;
    }
    if (__any(bad) && (threadIdx.x & 63) == 0) atomicOr(inexact, 1);
}

// ------------------------------------------------------------------------------ eta
// eta[k][i] = sum_a X[a][i] beta[k][a] — VALU, 256 rows x 32 fits per block, the beta tile
// staged transposed in LDS and read as wave-uniform broadcasts.  (f32 VALU FMA and f32
// MFMA have the same peak on gfx950; this op is ~1 % of an IRLS step.)
constexpr int kEtaFits = 32;
constexpr int kEtaChunk = 128;
template <typename TX>
__global__ void __launch_bounds__(256) eta_kernel(const TX* __restrict__ X, int64_t ld, int32_t P,
                                                  const float* __restrict__ beta, int32_t B,
                                                  float* __restrict__ eta) {
    __shared__ float bt[kEtaChunk][kEtaFits];
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int k0 = blockIdx.y * kEtaFits;
    float acc[kEtaFits];
#pragma unroll
    for (int k = 0; k < kEtaFits; ++k) acc[k] = 0.0f;
    for (int a0 = 0; a0 < P; a0 += kEtaChunk) {
        __syncthreads();
        for (int e = threadIdx.x; e < kEtaChunk * kEtaFits; e += 256) {
            const int kk = e / kEtaChunk, aa = e % kEtaChunk;
            const int k = k0 + kk, a = a0 + aa;
            bt[aa][kk] = (k < B && a < P) ? beta[(int64_t)k * P + a] : 0.0f;
        }
        __syncthreads();
        const int na = min(kEtaChunk, P - a0);
        for (int aa = 0; aa < na; ++aa) {
            const float x = (float)X[(int64_t)(a0 + aa) * ld + i];
            const f32x4* bv = reinterpret_cast<const f32x4*>(&bt[aa][0]);
#pragma unroll
            for (int q = 0; q < kEtaFits / 4; ++q) {
                const f32x4 b4 = bv[q];
                acc[4 * q + 0] += x * b4[0];
                acc[4 * q + 1] += x * b4[1];
                acc[4 * q + 2] += x * b4[2];
                acc[4 * q + 3] += x * b4[3];
            }
        }
    }
#pragma unroll
    for (int k = 0; k < kEtaFits; ++k)
        if (k0 + k < B) eta[(int64_t)(k0 + k) * ld + i] = acc[k];
}

// ------------------------------------------------------------------------------ link
// Row y of the launch is fit slot k = slots[y] (all slots when slots is null).  W and the
// optional f32 R are written per slot; Rp (optional) receives R as three bf16 pieces
// hi + mid + lo == R in the packed operand layout of the gradient kernel, row y of each piece
// plane (Bp rows per plane): the split is fused here instead of a separate pass over R.
__global__ void __launch_bounds__(256) link_kernel(int32_t family, float power, int64_t n,
                                                   int64_t ld, const int32_t* __restrict__ slots,
                                                   float* __restrict__ eta,
                                                   const float* __restrict__ Y,
                                                   const uint8_t* __restrict__ M,
                                                   const int32_t* __restrict__ fit_resp,
                                                   const int32_t* __restrict__ fit_mask,
                                                   float* __restrict__ W, float* __restrict__ R,
                                                   __bf16* __restrict__ Rp, int32_t Bp,
                                                   const float* __restrict__ step,
                                                   const float* __restrict__ deta,
                                                   const int32_t* __restrict__ rpos) {
    const int y = blockIdx.y;
    const int k = slots ? slots[y] : y;
    const int ry = rpos ? rpos[y] : y;          // packed-R row of this fit (< 0: none)
    float* e = eta + (int64_t)k * ld;
    // fused predictor update of the previous Newton step: eta += step[y] * deta (then the link)
    const float t = deta ? step[y] : 0.0f;
    const float* dv = deta ? deta + (int64_t)k * ld : nullptr;
    const float* yv = Y + (int64_t)fit_resp[k] * ld;
    const uint8_t* m = M + (int64_t)fit_mask[k] * ld;
    float* w = W + (int64_t)k * ld;
    float* r = R ? R + (int64_t)k * ld : nullptr;
    const int64_t plane = (int64_t)Bp * ld;
    __bf16* rp = (Rp && ry >= 0) ? Rp + (int64_t)ry * ld : nullptr;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < ld;
         i += (int64_t)gridDim.x * 256) {
        float wi = 0.0f, ri = 0.0f;
        if (i < n) {
            float ei = e[i];
            if (dv && t != 0.0f) {
                ei += t * dv[i];
                e[i] = ei;
            }
            const float mi = (float)m[i];
            if (mi != 0.0f) {
                const LossOut o = half_loss(family, power, yv[i], ei);
                wi = mi * o.h;
                ri = mi * o.g;
            }
        }
        w[i] = wi;
        if (r) r[i] = ri;
        if (rp) {
            __bf16 hi, mid, lo;
            split3(ri, hi, mid, lo);
            rp[i] = hi;
            rp[plane + i] = mid;
            rp[2 * plane + i] = lo;
        }
    }
}

// ------------------------------------------------------------------------------ X^T R
// G[k][a] = sum_i X[a][i] R[k][i] with v_mfma_f32_32x32x2_f32 (exact f32 products).
// Block: 4 waves, 128 predictors x 32 fits, one row chunk.  Lane (r, h) streams 8
// consecutive rows of predictor a0+r and of fit k0+r; MFMA step j consumes row 8h+j of the
// 16-row group on both operands, so A and B agree on the K index by construction.
struct XtrPlan { int32_t nz; int64_t ch; };
static XtrPlan xtr_plan(int32_t P, int32_t B, int64_t n) {
    const int64_t tiles = (int64_t)((P + 127) / 128) * ((B + 31) / 32);
    int64_t nz = (2048 + tiles - 1) / tiles;
    const int64_t maxz = (n + 1023) / 1024;
    if (nz > maxz) nz = maxz;
    if (nz < 1) nz = 1;
    int64_t ch = (n + nz - 1) / nz;
    ch = (ch + 15) / 16 * 16;
    nz = (n + ch - 1) / ch;
    if (nz < 1) nz = 1;
    return {(int32_t)nz, ch};
}

template <typename TX>
__device__ __forceinline__ void load8(const TX* p, float (&v)[8]);
template <>
__device__ __forceinline__ void load8<__bf16>(const __bf16* p, float (&v)[8]) {
    const bf16x8 x = *reinterpret_cast<const bf16x8*>(p);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (float)x[j];
}
template <>
__device__ __forceinline__ void load8<float>(const float* p, float (&v)[8]) {
    const f32x4 a = *reinterpret_cast<const f32x4*>(p);
    const f32x4 b = *reinterpret_cast<const f32x4*>(p + 4);
    v[0] = a[0]; v[1] = a[1]; v[2] = a[2]; v[3] = a[3];
    v[4] = b[0]; v[5] = b[1]; v[6] = b[2]; v[7] = b[3];
}

template <typename TX>
__global__ void __launch_bounds__(256) xtr_kernel(const TX* __restrict__ X, int64_t ld, int32_t P,
                                                  int64_t n, int64_t ch,
                                                  const float* __restrict__ R, int32_t B,
                                                  float* __restrict__ part) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int r = lane & 31, h = lane >> 5;
    const int a = blockIdx.x * 128 + wave * 32 + r;        // P is a multiple of 256
    const int k0 = blockIdx.y * 32;
    const int k = k0 + r;
    const bool kval = k < B;
    const int64_t ib = (int64_t)blockIdx.z * ch;
    const int64_t ie = min(ib + ch, ((n + 15) / 16) * 16);   // X/R rows padded with zeros
    const TX* xp = X + (int64_t)a * ld;
    const float* rp = R + (int64_t)(kval ? k : 0) * ld;
    f32x16 acc = {};
    for (int64_t i = ib + 8 * h; i < ie; i += 16) {
        float xv[8], rv[8];
        load8<TX>(xp + i, xv);
        load8<float>(rp + i, rv);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const float rr = kval ? rv[j] : 0.0f;
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(xv[j], rr, acc, 0, 0, 0);
        }
    }
    // D[row = a][col = k]: reg j -> row (j&3) + 8(j>>2) + 4h, col r
    if (kval) {
        float* out = part + ((int64_t)blockIdx.z * B + k) * P + blockIdx.x * 128 + wave * 32;
#pragma unroll
        for (int j = 0; j < 16; ++j) out[(j & 3) + 8 * (j >> 2) + 4 * h] = acc[j];
    }
}

__global__ void __launch_bounds__(256) reduce_f32_to_f64(const float* __restrict__ part,
                                                         int64_t len, int32_t nz,
                                                         double* __restrict__ out) {
    for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < len;
         e += (int64_t)gridDim.x * 256) {
        double s = 0.0;
        for (int z = 0; z < nz; ++z) s += (double)part[(int64_t)z * len + e];
        out[e] = s;
    }
}

// ------------------------------------------------------------------------------ row sums
// Deterministic two-level float64 reductions over rows: block partials, then a fixed-order
// sum over chunks.
constexpr int64_t kRowChunk = 8192;
static int32_t row_chunks(int64_t n) { return (int32_t)((n + kRowChunk - 1) / kRowChunk); }

__device__ __forceinline__ double block_sum_d(double v, double* sh) {
    v = wave_sum_d(v);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    __syncthreads();
    if (lane == 0) sh[wave] = v;
    __syncthreads();
    double s = 0.0;
    if (threadIdx.x == 0)
        for (int w = 0; w < (int)(blockDim.x >> 6); ++w) s += sh[w];
    return s;
}

constexpr int kMaxTrials = 8;
__global__ void __launch_bounds__(256) loss_trials_kernel(
    int32_t family, float power, int64_t n, int64_t ld, const float* __restrict__ eta,
    const float* __restrict__ deta, const float* __restrict__ Y, const uint8_t* __restrict__ M,
    const int32_t* __restrict__ fit_resp, const int32_t* __restrict__ fit_mask,
    const float* __restrict__ tv, int32_t T, double* __restrict__ part,
    float* __restrict__ dmax, const int32_t* __restrict__ slots) {
    __shared__ double sh[4];
    __shared__ float shm[4];
    const int q = blockIdx.y;                       // output row
    const int k = slots ? slots[q] : q;             // fit slot
    const int32_t nchunks = gridDim.x;
    const float* e = eta + (int64_t)k * ld;
    const float* d = deta + (int64_t)k * ld;
    const float* y = Y + (int64_t)fit_resp[k] * ld;
    const uint8_t* m = M + (int64_t)fit_mask[k] * ld;
    double acc[kMaxTrials];
    for (int j = 0; j < kMaxTrials; ++j) acc[j] = 0.0;
    float mx = 0.0f;
    const int64_t i0 = (int64_t)blockIdx.x * kRowChunk;
    const int64_t i1 = min(i0 + kRowChunk, n);
    // Poisson with the first-round step lengths {0, 1, 1/2, 1/4, 1/8}: exp(eta + t d) =
    // exp(eta) exp(d/8)^(8t) -- two exps and three squarings per row instead of five exps
    const bool halving = family == SGLM_FAM_TWEEDIE_LOG && power == 1.0f && T == 5 &&
                         tv[0] == 0.0f && tv[1] == 1.0f && tv[2] == 0.5f && tv[3] == 0.25f &&
                         tv[4] == 0.125f;
    if (halving) {
        auto row = [&](double mi, double yi, double ei, double di) {
            mx = fmaxf(mx, fabsf((float)di));
            const double mu = exp(ei), e8 = exp(0.125 * di);
            const double e4 = e8 * e8, e2 = e4 * e4, e1 = e2 * e2;
            acc[0] += mi * (mu - yi * ei);
            acc[1] += mi * (mu * e1 - yi * (ei + di));
            acc[2] += mi * (mu * e2 - yi * (ei + 0.5 * di));
            acc[3] += mi * (mu * e4 - yi * (ei + 0.25 * di));
            acc[4] += mi * (mu * e8 - yi * (ei + 0.125 * di));
        };
        // four consecutive rows per thread from 4-byte / 16-byte loads (rows are 16-byte
        // aligned: ld and the chunk starts are multiples of 256): four times the bytes in
        // flight per load instruction of the one-row loop
        for (int64_t i = i0 + 4 * threadIdx.x; i < i1; i += 1024) {
            if (i + 4 <= i1) {
                const uint32_t m4 = *reinterpret_cast<const uint32_t*>(m + i);
                if (m4 == 0u) continue;
                const f32x4 y4 = *reinterpret_cast<const f32x4*>(y + i);
                const f32x4 e4 = *reinterpret_cast<const f32x4*>(e + i);
                const f32x4 d4 = *reinterpret_cast<const f32x4*>(d + i);
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const double mi = (double)((m4 >> (8 * j)) & 0xffu);
                    if (mi != 0.0) row(mi, y4[j], e4[j], d4[j]);
                }
            } else {
                for (int64_t q = i; q < i1; ++q) {
                    const double mi = (double)m[q];
                    if (mi != 0.0) row(mi, y[q], e[q], d[q]);
                }
            }
        }
    } else {
        for (int64_t i = i0 + threadIdx.x; i < i1; i += 256) {
            const double mi = (double)m[i];
            if (mi == 0.0) continue;
            const double yi = y[i], ei = e[i], di = d[i];
            mx = fmaxf(mx, fabsf((float)di));
            for (int j = 0; j < T; ++j)
                acc[j] += mi * half_loss_d(family, (double)power, yi, ei + (double)tv[j] * di);
        }
    }
    for (int j = 0; j < T; ++j) {
        const double s = block_sum_d(acc[j], sh);
        if (threadIdx.x == 0) part[((int64_t)q * T + j) * nchunks + blockIdx.x] = s;
    }
    if (dmax) {                 // max |d_eta| over the fit's rows (Hessian drift bound)
        for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
        if ((threadIdx.x & 63) == 0) shm[threadIdx.x >> 6] = mx;
        __syncthreads();
        if (threadIdx.x == 0)
            atomicMax(reinterpret_cast<unsigned int*>(dmax + q),
                      __float_as_uint(fmaxf(fmaxf(shm[0], shm[1]), fmaxf(shm[2], shm[3]))));
    }
}

__global__ void __launch_bounds__(256) score_kernel(
    int32_t family, float power, int64_t n, int64_t ld, const float* __restrict__ eta,
    const float* __restrict__ Y, const uint8_t* __restrict__ M,
    const int32_t* __restrict__ fit_resp, const int32_t* __restrict__ sets,
    double* __restrict__ part) {
    __shared__ double sh[4];
    const int k = blockIdx.y;
    const int32_t nchunks = gridDim.x;
    const float* e = eta + (int64_t)k * ld;
    const float* y = Y + (int64_t)fit_resp[k] * ld;
    const int s0 = sets[2 * k], s1 = sets[2 * k + 1];
    const uint8_t* m0 = s0 >= 0 ? M + (int64_t)s0 * ld : nullptr;
    const uint8_t* m1 = s1 >= 0 ? M + (int64_t)s1 * ld : nullptr;
    double acc[4] = {0.0, 0.0, 0.0, 0.0};
    const int64_t i0 = (int64_t)blockIdx.x * kRowChunk;
    const int64_t i1 = min(i0 + kRowChunk, n);
    for (int64_t i = i0 + threadIdx.x; i < i1; i += 256) {
        const double w0 = m0 ? (double)m0[i] : 0.0;
        const double w1 = m1 ? (double)m1[i] : 0.0;
        if (w0 == 0.0 && w1 == 0.0) continue;
        const double yi = y[i], ei = e[i];
        const double mu = inv_link_d(family, ei);
        const double r2 = (yi - mu) * (yi - mu);
        const double l = half_loss_d(family, (double)power, yi, ei);
        acc[0] += w0 * r2; acc[1] += w0 * l;
        acc[2] += w1 * r2; acc[3] += w1 * l;
    }
    for (int q = 0; q < 4; ++q) {
        const double s = block_sum_d(acc[q], sh);
        if (threadIdx.x == 0) part[((int64_t)k * 4 + q) * nchunks + blockIdx.x] = s;
    }
}

__global__ void __launch_bounds__(256) reduce_chunks_d(const double* __restrict__ part,
                                                       int64_t rows, int32_t nchunks,
                                                       double* __restrict__ out) {
    const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (e >= rows) return;
    double s = 0.0;
    for (int c = 0; c < nchunks; ++c) s += part[e * nchunks + c];
    out[e] = s;
}

__global__ void __launch_bounds__(256) eta_axpy_kernel(int64_t n, int64_t ld,
                                                       const int32_t* __restrict__ slots,
                                                       const float* __restrict__ step,
                                                       const float* __restrict__ deta,
                                                       float* __restrict__ eta) {
    const int k = slots ? slots[blockIdx.y] : blockIdx.y;
    const float t = step[blockIdx.y];
    if (t == 0.0f) return;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * 256)
        eta[(int64_t)k * ld + i] += t * deta[(int64_t)k * ld + i];
}

// eta += t * deta, and dmax[k] = max_i |t * deta[k][i]| over the fit's mask rows (the
// drift bound that decides whether fit k may keep its Hessian factor).  dmax must be zeroed;
// non-negative floats order like their bit patterns, so an unsigned atomicMax reduces them.
__global__ void __launch_bounds__(256) eta_axpy_max_kernel(int64_t n, int64_t ld,
                                                           const float* __restrict__ step,
                                                           const float* __restrict__ deta,
                                                           const uint8_t* __restrict__ M,
                                                           const int32_t* __restrict__ fit_mask,
                                                           float* __restrict__ eta,
                                                           float* __restrict__ dmax) {
    const int k = blockIdx.y;
    const float t = step[k];
    if (t == 0.0f) return;
    const uint8_t* m = M + (int64_t)fit_mask[k] * ld;
    float mx = 0.0f;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * 256) {
        const float dv = t * deta[(int64_t)k * ld + i];
        eta[(int64_t)k * ld + i] += dv;
        if (m[i]) mx = fmaxf(mx, fabsf(dv));
    }
    for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
    __shared__ float sh[4];
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = mx;
    __syncthreads();
    if (threadIdx.x == 0) {
        mx = fmaxf(fmaxf(sh[0], sh[1]), fmaxf(sh[2], sh[3]));
        atomicMax(reinterpret_cast<unsigned int*>(dmax + k), __float_as_uint(mx));
    }
}

// out[q] = max over the rows of mask fit_mask[a] of |eta[a][i] - eta[b][i]|, (a, b) =
// pairs[2q], pairs[2q+1] (same mask): how far apart the IRLS weights of two fits are, which
// decides whether b may be factored from a's Gram.  out must be zeroed.
__global__ void __launch_bounds__(256) eta_pair_absmax_kernel(
    int64_t n, int64_t ld, const int32_t* __restrict__ pairs, const uint8_t* __restrict__ M,
    const int32_t* __restrict__ fit_mask, const float* __restrict__ eta, float* __restrict__ out) {
    const int q = blockIdx.y;
    const int a = pairs[2 * q], b = pairs[2 * q + 1];
    const float* ea = eta + (int64_t)a * ld;
    const float* eb = eta + (int64_t)b * ld;
    const uint8_t* m = M + (int64_t)fit_mask[a] * ld;
    float mx = 0.0f;
    // four consecutive rows per thread (4-byte mask / 16-byte eta loads; rows 16-byte aligned)
    for (int64_t i = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4; i < n;
         i += (int64_t)gridDim.x * 1024) {
        if (i + 4 <= n) {
            const uint32_t m4 = *reinterpret_cast<const uint32_t*>(m + i);
            if (m4 == 0u) continue;
            const f32x4 a4 = *reinterpret_cast<const f32x4*>(ea + i);
            const f32x4 b4 = *reinterpret_cast<const f32x4*>(eb + i);
#pragma unroll
            for (int j = 0; j < 4; ++j)
                if ((m4 >> (8 * j)) & 0xffu) mx = fmaxf(mx, fabsf(a4[j] - b4[j]));
        } else {
            for (int64_t q2 = i; q2 < n; ++q2)
                if (m[q2]) mx = fmaxf(mx, fabsf(ea[q2] - eb[q2]));
        }
    }
    for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
    __shared__ float sh[4];
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = mx;
    __syncthreads();
    if (threadIdx.x == 0) {
        mx = fmaxf(fmaxf(sh[0], sh[1]), fmaxf(sh[2], sh[3]));
        atomicMax(reinterpret_cast<unsigned int*>(out + q), __float_as_uint(mx));
    }
}

// Statistics of every (mask f, response r) pair in one pass (float64, deterministic two-level
// reduction): count = sum m, sum m (y - K_r), sum m (y - K_r)^2, min over m > 0 of y and, when
// power >= 0, sum m c_power(y) with c the half-Tweedie loss constant (sklearn
// constant_to_optimal_zero).  K_r is a per-response shift that keeps the centred sums exact.
constexpr int kStat = 5;
__device__ __forceinline__ double tweedie_const(double power, double y) {
    if (power == 0.0) return -0.5 * y * y;
    if (power == 1.0) return (y > 0.0 ? y * log(y) : 0.0) - y;
    if (power == 2.0) return -log(y) - 1.0;
    return pow(fmax(y, 0.0), 2.0 - power) / (1.0 - power) / (2.0 - power);
}

__global__ void __launch_bounds__(256) mask_stats_kernel(const uint8_t* __restrict__ M,
                                                         const double* __restrict__ Y,
                                                         const double* __restrict__ K,
                                                         int64_t n, int64_t ldm, int32_t F,
                                                         double power,
                                                         double* __restrict__ part) {
    __shared__ double sh[4];
    const int f = blockIdx.y, r = blockIdx.z;
    const uint8_t* m = M + (int64_t)f * ldm;
    const double* y = Y + (int64_t)r * n;
    const double kr = K[r];
    double a[kStat - 1] = {0.0, 0.0, 0.0, 0.0};
    double mn = INFINITY;
    const int64_t i0 = (int64_t)blockIdx.x * kRowChunk;
    const int64_t i1 = min(i0 + kRowChunk, n);
    for (int64_t i = i0 + threadIdx.x; i < i1; i += 256) {
        const double w = (double)m[i];
        if (w == 0.0) continue;
        const double yi = y[i], d = yi - kr;
        a[0] += w;
        a[1] += w * d;
        a[2] += w * d * d;
        if (power >= 0.0) a[3] += w * tweedie_const(power, yi);
        mn = fmin(mn, yi);
    }
    const int64_t nch = gridDim.x;
    double* out = part + (((int64_t)r * F + f) * kStat) * nch + blockIdx.x;
    for (int q = 0; q < kStat - 1; ++q) {
        const double v = block_sum_d(a[q], sh);
        if (threadIdx.x == 0) out[q * nch] = v;
    }
    for (int o = 32; o > 0; o >>= 1) mn = fmin(mn, __shfl_xor(mn, o, 64));
    __syncthreads();
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = mn;
    __syncthreads();
    if (threadIdx.x == 0) out[(kStat - 1) * nch] = fmin(fmin(sh[0], sh[1]), fmin(sh[2], sh[3]));
}

__global__ void __launch_bounds__(256) mask_stats_reduce(const double* __restrict__ part,
                                                         int64_t rows, int32_t nch,
                                                         double* __restrict__ out) {
    const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (e >= rows) return;
    const bool is_min = e % kStat == kStat - 1;
    double s = is_min ? INFINITY : 0.0;
    for (int c = 0; c < nch; ++c) {
        const double v = part[e * nch + c];
        s = is_min ? fmin(s, v) : s + v;
    }
    out[e] = s;
}

// Per-fit scalars of a Newton step, one workgroup per active fit k = slots[q] (float64): the
// directional derivative g.d, the penalty terms sum lam w^2, sum lam w d, sum lam d^2 (lam =
// the fit's penalty row), max |d| and, for every trial step t[j], max |w + t[j] d| (the scale
// of the stopping rule after that step).  out[q][0..5+T).
constexpr int kMaxStepT = 16;
__global__ void __launch_bounds__(256) step_scalars_kernel(
    int32_t P, int32_t ncoef, const int32_t* __restrict__ slots, const double* __restrict__ g,
    const double* __restrict__ beta, const float* __restrict__ delta,
    const double* __restrict__ lamp, const double* __restrict__ t, int32_t T,
    double* __restrict__ out) {
    __shared__ double sh[4];
    const int q = blockIdx.x, k = slots[q];
    const double* gk = g + (int64_t)k * P;
    const double* bk = beta + (int64_t)k * P;
    const float* dk = delta + (int64_t)k * P;
    const double* lk = lamp + (int64_t)k * P;
    double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0, md = 0.0, mi = 0.0;
    double mb[kMaxStepT];
    double tv[kMaxStepT];
    for (int j = 0; j < T; ++j) { mb[j] = 0.0; tv[j] = t[j]; }
    for (int a = threadIdx.x; a < P; a += 256) {
        const double d = (double)dk[a], b = bk[a], l = lk[a];
        s0 += gk[a] * d;
        s1 += l * b * b;
        s2 += l * b * d;
        s3 += l * d * d;
        if (a < ncoef) md = fmax(md, fabs(d)); else mi = fmax(mi, fabs(d));
        if (a < ncoef)
            for (int j = 0; j < T; ++j) mb[j] = fmax(mb[j], fabs(b + tv[j] * d));
    }
    double* o = out + (int64_t)q * (6 + T);
    double v;
    v = block_sum_d(s0, sh); if (threadIdx.x == 0) o[0] = v;
    v = block_sum_d(s1, sh); if (threadIdx.x == 0) o[1] = v;
    v = block_sum_d(s2, sh); if (threadIdx.x == 0) o[2] = v;
    v = block_sum_d(s3, sh); if (threadIdx.x == 0) o[3] = v;
    for (int j = -1; j <= T; ++j) {
        double m = j < 0 ? md : (j < T ? mb[j] : mi);
        for (int off = 32; off > 0; off >>= 1) m = fmax(m, __shfl_xor(m, off, 64));
        __syncthreads();
        if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = m;
        __syncthreads();
        if (threadIdx.x == 0) o[5 + j] = fmax(fmax(sh[0], sh[1]), fmax(sh[2], sh[3]));
    }
}

// The Anderson (secant) correction of the Newton directions (engine.irls, ANDERSON), one
// workgroup per active fit k = slots[q]: f = delta[k] (this iteration's raw direction); where
// sel[q] (the same factor as the previous step, which was taken with t = tprev[q]):
//   df = f - raw_prev, db = used_prev * t, gamma = df.f / max(df.df, 1e-30),
//   d = f - gamma (db + df), kept when df.df > 1e-12 f.f, gamma in [-2, 0.5] and g.d < 0;
// rm[k] = (max_{j < p} |f_j|, |f_p|) for those (0 elsewhere), raw_prev[k] = f for every fit.
// float32 as the torch expressions it replaces; sums in a fixed order.
__global__ void __launch_bounds__(256) aa_step_kernel(int32_t P, int32_t p,
                                                      const int32_t* __restrict__ slots,
                                                      const uint8_t* __restrict__ sel,
                                                      const float* __restrict__ tprev,
                                                      float* __restrict__ delta,
                                                      float* __restrict__ raw_prev,
                                                      const float* __restrict__ used_prev,
                                                      const double* __restrict__ gtot,
                                                      float* __restrict__ rm) {
    __shared__ float sh[4][8];
    const int q = blockIdx.x, k = slots[q];
    float* d = delta + (int64_t)k * P;
    float* rp = raw_prev + (int64_t)k * P;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    if (!sel[q]) {
        for (int a = tid; a < P; a += 256) rp[a] = d[a];
        if (tid == 0) { rm[2 * k] = 0.0f; rm[2 * k + 1] = 0.0f; }
        return;
    }
    const float t = tprev[q];
    const float* up_ = used_prev + (int64_t)k * P;
    const double* g = gtot + (int64_t)k * P;
    float den = 0.0f, num = 0.0f, ff = 0.0f, mx = 0.0f, fp = 0.0f;
    for (int a = tid; a < P; a += 256) {
        const float f = d[a];
        const float df = f - rp[a];
        den = fmaf(df, df, den);
        num = fmaf(df, f, num);
        ff = fmaf(f, f, ff);
        if (a < p) mx = fmaxf(mx, fabsf(f));
        if (a == p) fp = fabsf(f);
    }
    auto wsum = [&](float v) { for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64); return v; };
    den = wsum(den); num = wsum(num); ff = wsum(ff);
    for (int o = 32; o > 0; o >>= 1) {
        mx = fmaxf(mx, __shfl_xor(mx, o, 64));
        fp = fmaxf(fp, __shfl_xor(fp, o, 64));
    }
    if (lane == 0) {
        sh[w][0] = den; sh[w][1] = num; sh[w][2] = ff; sh[w][3] = mx; sh[w][5] = fp;
    }
    __syncthreads();
    den = sh[0][0] + sh[1][0] + sh[2][0] + sh[3][0];
    num = sh[0][1] + sh[1][1] + sh[2][1] + sh[3][1];
    ff = sh[0][2] + sh[1][2] + sh[2][2] + sh[3][2];
    mx = fmaxf(fmaxf(sh[0][3], sh[1][3]), fmaxf(sh[2][3], sh[3][3]));
    fp = fmaxf(fmaxf(sh[0][5], sh[1][5]), fmaxf(sh[2][5], sh[3][5]));
    const float gam = num / fmaxf(den, 1e-30f);
    // g.d of the corrected direction
    float gdn = 0.0f;
    for (int a = tid; a < P; a += 256) {
        const float f = d[a];
        const float df = f - rp[a];
        const float db = up_[a] * t;
        const float dn = f - gam * (db + df);
        gdn = fmaf((float)g[a], dn, gdn);
    }
    gdn = wsum(gdn);
    __syncthreads();
    if (lane == 0) sh[w][4] = gdn;
    __syncthreads();
    gdn = sh[0][4] + sh[1][4] + sh[2][4] + sh[3][4];
    const bool good = den > 1e-12f * ff && gam >= -2.0f && gam <= 0.5f && gdn < 0.0f;
    for (int a = tid; a < P; a += 256) {
        const float f = d[a];
        const float df = f - rp[a];
        const float db = up_[a] * t;
        if (good) d[a] = f - gam * (db + df);
        rp[a] = f;
    }
    if (tid == 0) { rm[2 * k] = mx; rm[2 * k + 1] = fp; }
}

// beta[k] += step[q] * delta[k] for k = slots[q] (float64 coefficients, f32 direction)
__global__ void __launch_bounds__(256) step_update_kernel(int32_t P,
                                                          const int32_t* __restrict__ slots,
                                                          const double* __restrict__ step,
                                                          const float* __restrict__ delta,
                                                          double* __restrict__ beta) {
    const int q = blockIdx.x, k = slots[q];
    const double t = step[q];
    if (t == 0.0) return;
    for (int a = threadIdx.x; a < P; a += 256)
        beta[(int64_t)k * P + a] += t * (double)delta[(int64_t)k * P + a];
}

// The Newton iteration's decisions on the device (engine.irls restated; the host reads the
// verdicts back with the trial losses instead of recomputing them, so the step and the next
// link are enqueued before the host has seen anything): per active fit q (slot act[q]),
//   stage-1 Armijo over t in ts[1..4] of obj(t) = L(t) + (A + 2 t B + t^2 C) / 2: the first t
//   with obj(t) - obj(0) <= sigma t g.d, or |obj(t) - obj(0)| <= 1e-13 |obj(0)|;
//   scale = max(max|w + t d|, floor) (legacy: 1 + max|w + t d|), prop = max(max|d| / scale,
//   |d_intercept|) (legacy: max|d| / scale), relv = t prop (with the secant's raw-step floor);
//   stop on tol, stagnation (fresh Hessian, relv < 1e-4, no better than half the previous) or a
//   failed search on a fresh Hessian; out of iterations; continue otherwise.
// A fit whose stage-1 search fails goes to the host's stage 2: it keeps t = 0 here and a packed
// R row (rpos) reserved.  Fits that continue (or await stage 2) get consecutive rows in act
// order: rpos[q] (-1: none), nxt[0 .. *cnt) their slots.  f64 operations are written out
// (_rn intrinsics, no contraction) in the order of the host's numpy expressions.
enum DecideFlags {
    kDecHit = 1, kDecStop = 2, kDecConv = 4, kDecOoi = 8, kDecTol = 16, kDecStag = 32,
    kDecFail = 64, kDecLsFail = 128, kDecMore = 256, kDecRow = 512
};
constexpr int kDecT = 1024;
__global__ void __launch_bounds__(kDecT) step_decide_kernel(
    int32_t na, const int32_t* __restrict__ act, const double* __restrict__ L,
    const double* __restrict__ sc, int32_t nts, const double* __restrict__ ts, double sigma,
    double tol, double sfloor, int32_t legacy, const float* __restrict__ aa_rm,
    const double* __restrict__ prev_rel, const uint8_t* __restrict__ fresh,
    const int32_t* __restrict__ n_iter, const int32_t* __restrict__ max_iter,
    double* __restrict__ step64, float* __restrict__ step32, double* __restrict__ relv_o,
    double* __restrict__ prop_o, int32_t* __restrict__ flags, int32_t* __restrict__ tix_o,
    int32_t* __restrict__ rpos, int32_t* __restrict__ nxt, int32_t* __restrict__ cnt) {
    __shared__ int32_t sh[kDecT];
    __shared__ int32_t base;
    if (threadIdx.x == 0) base = 0;
    __syncthreads();
    const int W = 6 + nts;
    for (int q0 = 0; q0 < na; q0 += kDecT) {
        const int q = q0 + threadIdx.x;
        int row = 0;
        if (q < na) {
            const double* Lq = L + (int64_t)q * 5;
            const double* s = sc + (int64_t)q * W;
            const double gdir = s[0], A = s[1], B = s[2], C = s[3], maxd = s[4];
            const double maxdi = s[5 + nts];
            double obj[5];
#pragma unroll
            for (int j = 0; j < 5; ++j) {
                const double t = ts[j];
                const double lin = __dadd_rn(A, __dmul_rn(__dmul_rn(2.0, t), B));
                const double quad = __dadd_rn(lin, __dmul_rn(__dmul_rn(t, t), C));
                obj[j] = __dadd_rn(Lq[j], __dmul_rn(0.5, quad));
            }
            int tix = 0;
            for (int j = 1; j < 5; ++j) {
                const double dlt = __dsub_rn(obj[j], obj[0]);
                const bool ok = dlt <= __dmul_rn(__dmul_rn(sigma, ts[j]), gdir) ||
                                fabs(dlt) <= __dmul_rn(1e-13, fabs(obj[0]));
                if (ok) { tix = j; break; }
            }
            const bool hit = tix > 0;
            const double step = hit ? ts[tix] : 0.0;
            int f = hit ? kDecHit : kDecMore;
            double relv = 0.0, prop = 0.0;
            if (hit) {
                const double mb = s[5 + tix];
                double scale, pr;
                if (legacy) {
                    scale = __dadd_rn(1.0, mb);
                    pr = __ddiv_rn(maxd, scale);
                } else {
                    scale = fmax(mb, sfloor);
                    pr = fmax(__ddiv_rn(maxd, scale), maxdi);
                }
                prop = pr;
                relv = __dmul_rn(step, pr);
                if (aa_rm) {
                    const int k = act[q];
                    const double rm0 = (double)aa_rm[2 * k], rm1 = (double)aa_rm[2 * k + 1];
                    relv = fmax(relv, fmax(__ddiv_rn(rm0, scale), rm1));
                }
                const bool fr = fresh[q] != 0;
                const bool stop_tol = relv <= tol;
                const bool stop_stag = !stop_tol && fr && relv < 1e-4 &&
                                       relv >= __dmul_rn(0.5, prev_rel[q]);
                const bool stop = stop_tol || stop_stag;
                const bool ooi = !stop && (n_iter[q] + 1 >= max_iter[q]);
                if (stop_tol) f |= kDecTol | kDecConv;
                if (stop_stag) f |= kDecStag;
                if (stop) f |= kDecStop;
                if (ooi) f |= kDecOoi;
                row = !stop && !ooi;
            } else {
                row = 1;                                   // stage 2 decides; a row reserved
            }
            if (row) f |= kDecRow;
            step64[q] = step;
            step32[q] = (float)step;
            relv_o[q] = relv;
            prop_o[q] = prop;
            flags[q] = f;
            tix_o[q] = tix;
        }
        // rows in act order: inclusive scan of the row flags of this chunk
        sh[threadIdx.x] = row;
        __syncthreads();
        for (int o = 1; o < kDecT; o <<= 1) {
            const int v = threadIdx.x >= o ? sh[threadIdx.x - o] : 0;
            __syncthreads();
            sh[threadIdx.x] += v;
            __syncthreads();
        }
        if (q < na) {
            const int pos = base + sh[threadIdx.x] - row;
            rpos[q] = row ? pos : -1;
            if (row) nxt[pos] = act[q];
        }
        __syncthreads();
        if (threadIdx.x == kDecT - 1) base += sh[kDecT - 1];
        __syncthreads();
    }
    if (threadIdx.x == 0) *cnt = base;
}

static unsigned grid1(int64_t work, int64_t per_block, unsigned cap = 8192) {
    int64_t g = (work + per_block - 1) / per_block;
    if (g < 1) g = 1;
    if (g > cap) g = cap;
    return (unsigned)g;
}

}  // namespace sglm

using namespace sglm;

extern "C" {

const char* sglm_last_error(void) { return g_err; }
int sglm_version(void) { return 1; }

static int timeshift_launch(const void* src, int64_t n_src, int64_t rs_src, int64_t cs_src,
                            const int32_t* src_col, const int32_t* shift, int32_t ncols_out,
                            void* out, int64_t n_out, int64_t rs_out, int64_t cs_out,
                            int64_t row0, int32_t elem_size, uint64_t fill_bits,
                            const int64_t* rows, sglm_stream_t stream);

int sglm_timeshift_expand(const void* src, int64_t n_src, int64_t rs_src, int64_t cs_src,
                          const int32_t* src_col, const int32_t* shift, int32_t ncols_out,
                          void* out, int64_t n_out, int64_t rs_out, int64_t cs_out,
                          int64_t row0, int32_t elem_size, uint64_t fill_bits,
                          sglm_stream_t stream) {
    return timeshift_launch(src, n_src, rs_src, cs_src, src_col, shift, ncols_out, out, n_out,
                            rs_out, cs_out, row0, elem_size, fill_bits, nullptr, stream);
}

int sglm_timeshift_gather(const void* src, int64_t n_src, int64_t rs_src, int64_t cs_src,
                          const int32_t* src_col, const int32_t* shift, int32_t ncols_out,
                          void* out, int64_t n_out, int64_t rs_out, int64_t cs_out,
                          const int64_t* rows, int32_t elem_size, uint64_t fill_bits,
                          sglm_stream_t stream) {
    if (n_out > 0 && ncols_out > 0 && !rows) {
        set_error("sglm_timeshift_gather: null row list");
        return SGLM_EINVAL;
    }
    return timeshift_launch(src, n_src, rs_src, cs_src, src_col, shift, ncols_out, out, n_out,
                            rs_out, cs_out, 0, elem_size, fill_bits, rows, stream);
}

static int timeshift_launch(const void* src, int64_t n_src, int64_t rs_src, int64_t cs_src,
                            const int32_t* src_col, const int32_t* shift, int32_t ncols_out,
                            void* out, int64_t n_out, int64_t rs_out, int64_t cs_out,
                            int64_t row0, int32_t elem_size, uint64_t fill_bits,
                            const int64_t* rows, sglm_stream_t stream) {
    if (ncols_out <= 0 || n_out <= 0) return SGLM_OK;
    if (!src || !out || !src_col || !shift || n_src < 0) {
        set_error("sglm_timeshift_expand: null pointer or negative size");
        return SGLM_EINVAL;
    }
    dim3 grid(grid1(n_out, 256, 1024), (unsigned)(ncols_out < 32768 ? ncols_out : 32768));
    hipStream_t s = as_stream(stream);
    switch (elem_size) {
        case 1: timeshift_kernel<uint8_t><<<grid, 256, 0, s>>>((const uint8_t*)src, n_src, rs_src, cs_src, src_col, shift, ncols_out, (uint8_t*)out, n_out, rs_out, cs_out, row0, (uint8_t)fill_bits, rows); break;
        case 2: timeshift_kernel<uint16_t><<<grid, 256, 0, s>>>((const uint16_t*)src, n_src, rs_src, cs_src, src_col, shift, ncols_out, (uint16_t*)out, n_out, rs_out, cs_out, row0, (uint16_t)fill_bits, rows); break;
        case 4: timeshift_kernel<uint32_t><<<grid, 256, 0, s>>>((const uint32_t*)src, n_src, rs_src, cs_src, src_col, shift, ncols_out, (uint32_t*)out, n_out, rs_out, cs_out, row0, (uint32_t)fill_bits, rows); break;
        case 8: timeshift_kernel<uint64_t><<<grid, 256, 0, s>>>((const uint64_t*)src, n_src, rs_src, cs_src, src_col, shift, ncols_out, (uint64_t*)out, n_out, rs_out, cs_out, row0, (uint64_t)fill_bits, rows); break;
        default: set_error("sglm_timeshift_expand: elem_size %d not in {1,2,4,8}", elem_size); return SGLM_EINVAL;
    }
    return check_launch("timeshift_kernel");
}

int sglm_pack_design_rows(const void* src, int32_t src_is_f64, int64_t n, int32_t p, int64_t rs,
                          int64_t cs, int32_t add_ones, uint16_t* Xb, float* Xf, int64_t ld,
                          int32_t P, int64_t dst0, int32_t* inexact, sglm_stream_t stream) {
    return sglm_pack_design_rows_cf(src, src_is_f64, n, p, rs, cs, add_ones, Xb, Xf, ld, P, dst0,
                                    inexact, nullptr, stream);
}

int sglm_pack_design_rows_cf(const void* src, int32_t src_is_f64, int64_t n, int32_t p,
                             int64_t rs, int64_t cs, int32_t add_ones, uint16_t* Xb, float* Xf,
                             int64_t ld, int32_t P, int64_t dst0, int32_t* inexact,
                             int32_t* colflag, sglm_stream_t stream) {
    if (n <= 0) return SGLM_OK;
    if (!Xb || !inexact || (p > 0 && !src)) { set_error("sglm_pack_design_rows: null pointer"); return SGLM_EINVAL; }
    if (ld % 64 || P % 64 || dst0 % 64 || dst0 < 0 || dst0 + n > ld || P < p + (add_ones ? 1 : 0)) {
        set_error("sglm_pack_design_rows: bad rows dst0=%lld n=%lld ld=%lld", (long long)dst0,
                  (long long)n, (long long)ld);
        return SGLM_EINVAL;
    }
    dim3 grid((unsigned)((n + 63) / 64), (unsigned)(P / 64));
    hipStream_t s = as_stream(stream);
    if (src_is_f64)
        pack_kernel<double><<<grid, 256, 0, s>>>((const double*)src, n, p, rs, cs, add_ones, Xb, Xf, ld, inexact, dst0, colflag);
    else
        pack_kernel<float><<<grid, 256, 0, s>>>((const float*)src, n, p, rs, cs, add_ones, Xb, Xf, ld, inexact, dst0, colflag);
    return check_launch("pack_kernel");
}

int sglm_pack_design(const void* src, int32_t src_is_f64, int64_t n, int32_t p, int64_t rs,
                     int64_t cs, int32_t add_ones, uint16_t* Xb, float* Xf, int64_t ld,
                     int32_t P, int32_t* inexact, sglm_stream_t stream) {
    if (!Xb || !inexact || (n > 0 && p > 0 && !src)) { set_error("sglm_pack_design: null pointer"); return SGLM_EINVAL; }
    if (ld % 64 || P % 64 || ld < n || P < p + (add_ones ? 1 : 0)) {
        set_error("sglm_pack_design: bad padding ld=%lld P=%d n=%lld p=%d", (long long)ld, P, (long long)n, p);
        return SGLM_EINVAL;
    }
    dim3 grid((unsigned)(ld / 64), (unsigned)(P / 64));
    hipStream_t s = as_stream(stream);
    if (src_is_f64)
        pack_kernel<double><<<grid, 256, 0, s>>>((const double*)src, n, p, rs, cs, add_ones, Xb, Xf, ld, inexact);
    else
        pack_kernel<float><<<grid, 256, 0, s>>>((const float*)src, n, p, rs, cs, add_ones, Xb, Xf, ld, inexact);
    return check_launch("pack_kernel");
}

int sglm_gemv_eta(const void* X, int32_t xtype, int64_t ld, int32_t P, int64_t n,
                  const float* beta, int32_t B, float* eta, sglm_stream_t stream) {
    if (B <= 0) return SGLM_OK;
    if (!X || !beta || !eta || ld % 256 || P % 256) { set_error("sglm_gemv_eta: bad args"); return SGLM_EINVAL; }
    (void)n;
    dim3 grid((unsigned)(ld / 256), (unsigned)((B + kEtaFits - 1) / kEtaFits));
    hipStream_t s = as_stream(stream);
    if (xtype == SGLM_X_BF16)
        eta_kernel<__bf16><<<grid, 256, 0, s>>>((const __bf16*)X, ld, P, beta, B, eta);
    else
        eta_kernel<float><<<grid, 256, 0, s>>>((const float*)X, ld, P, beta, B, eta);
    return check_launch("eta_kernel");
}

int sglm_link_update(int32_t family, float power, int64_t n, int64_t ld, int32_t B,
                     const int32_t* slots, float* eta, const float* Y, const uint8_t* M,
                     const int32_t* fit_resp, const int32_t* fit_mask, float* W, float* R,
                     void* Rp, const float* step, const float* deta, sglm_stream_t stream) {
    if (B <= 0) return SGLM_OK;
    if (!eta || !Y || !M || !fit_resp || !fit_mask || !W || (!R && !Rp)) { set_error("sglm_link_update: null pointer"); return SGLM_EINVAL; }
    dim3 grid(grid1(ld, 256, 1024), (unsigned)B);
    link_kernel<<<grid, 256, 0, as_stream(stream)>>>(family, power, n, ld, slots, eta, Y, M,
                                                     fit_resp, fit_mask, W, R, (__bf16*)Rp,
                                                     (B + 31) / 32 * 32, step, deta, nullptr);
    return check_launch("link_kernel");
}

int sglm_link_update_rp(int32_t family, float power, int64_t n, int64_t ld, int32_t B,
                        const int32_t* slots, float* eta, const float* Y, const uint8_t* M,
                        const int32_t* fit_resp, const int32_t* fit_mask, float* W, float* R,
                        void* Rp, int32_t Bp, const int32_t* rpos, const float* step,
                        const float* deta, sglm_stream_t stream) {
    if (B <= 0) return SGLM_OK;
    if (!eta || !Y || !M || !fit_resp || !fit_mask || !W || (!R && !Rp) || !slots ||
        (Rp && (!rpos || Bp < B || Bp % 32)) || (deta && !step)) {
        set_error("sglm_link_update_rp: bad args");
        return SGLM_EINVAL;
    }
    dim3 grid(grid1(ld, 256, 1024), (unsigned)B);
    link_kernel<<<grid, 256, 0, as_stream(stream)>>>(family, power, n, ld, slots, eta, Y, M,
                                                     fit_resp, fit_mask, W, R, (__bf16*)Rp, Bp,
                                                     step, deta, rpos);
    return check_launch("link_kernel");
}

size_t sglm_xtr_work_bytes(int32_t P, int32_t B, int64_t n) {
    const XtrPlan pl = xtr_plan(P, B, n);
    return (size_t)pl.nz * (size_t)B * (size_t)P * sizeof(float);
}

int sglm_xtr(const void* X, int32_t xtype, int64_t ld, int32_t P, int64_t n, const float* R,
             int32_t B, double* G, void* work, sglm_stream_t stream) {
    if (B <= 0) return SGLM_OK;
    if (!X || !R || !G || !work || P % 256 || ld % 256 || n > ld) { set_error("sglm_xtr: bad args"); return SGLM_EINVAL; }
    const XtrPlan pl = xtr_plan(P, B, n);
    dim3 grid((unsigned)(P / 128), (unsigned)((B + 31) / 32), (unsigned)pl.nz);
    hipStream_t s = as_stream(stream);
    float* part = (float*)work;
    if (xtype == SGLM_X_BF16)
        xtr_kernel<__bf16><<<grid, 256, 0, s>>>((const __bf16*)X, ld, P, n, pl.ch, R, B, part);
    else
        xtr_kernel<float><<<grid, 256, 0, s>>>((const float*)X, ld, P, n, pl.ch, R, B, part);
    int st = check_launch("xtr_kernel");
    if (st) return st;
    const int64_t len = (int64_t)B * P;
    reduce_f32_to_f64<<<grid1(len, 256, 4096), 256, 0, s>>>(part, len, pl.nz, G);
    return check_launch("reduce_f32_to_f64");
}

size_t sglm_rowsum_work_bytes(int32_t B, int32_t T, int64_t n) {
    return (size_t)B * (size_t)T * (size_t)row_chunks(n) * sizeof(double);
}

int sglm_loss_trials(int32_t family, float power, int64_t n, int64_t ld, int32_t B,
                     const int32_t* slots, const float* eta, const float* deta, const float* Y, const uint8_t* M,
                     const int32_t* fit_resp, const int32_t* fit_mask, const float* t,
                     int32_t T, double* out, void* work, sglm_stream_t stream) {
    if (B <= 0) return SGLM_OK;
    if (T < 1 || T > kMaxTrials || !eta || !deta || !Y || !M || !t || !out || !work) {
        set_error("sglm_loss_trials: bad args (T=%d)", T);
        return SGLM_EINVAL;
    }
    (void)ld;
    const int32_t nc = row_chunks(n);
    hipStream_t s = as_stream(stream);
    loss_trials_kernel<<<dim3((unsigned)nc, (unsigned)B), 256, 0, s>>>(family, power, n, ld, eta, deta, Y, M, fit_resp, fit_mask, t, T, (double*)work, nullptr, slots);
    int st = check_launch("loss_trials_kernel");
    if (st) return st;
    const int64_t rows = (int64_t)B * T;
    reduce_chunks_d<<<grid1(rows, 256), 256, 0, s>>>((const double*)work, rows, nc, out);
    return check_launch("reduce_chunks_d");
}

int sglm_loss_trials_max(int32_t family, float power, int64_t n, int64_t ld, int32_t B,
                         const int32_t* slots, const float* eta, const float* deta, const float* Y, const uint8_t* M,
                         const int32_t* fit_resp, const int32_t* fit_mask, const float* t,
                         int32_t T, double* out, float* dmax, void* work, sglm_stream_t stream) {
    if (B <= 0) return SGLM_OK;
    if (T < 1 || T > kMaxTrials || !eta || !deta || !Y || !M || !t || !out || !dmax || !work) {
        set_error("sglm_loss_trials_max: bad args (T=%d)", T);
        return SGLM_EINVAL;
    }
    const int32_t nc = row_chunks(n);
    hipStream_t s = as_stream(stream);
    if (hipMemsetAsync(dmax, 0, sizeof(float) * (size_t)B, s) != hipSuccess) {
        set_error("sglm_loss_trials_max: hipMemsetAsync failed");
        return SGLM_EHIP;
    }
    loss_trials_kernel<<<dim3((unsigned)nc, (unsigned)B), 256, 0, s>>>(family, power, n, ld, eta, deta, Y, M, fit_resp, fit_mask, t, T, (double*)work, dmax, slots);
    int st = check_launch("loss_trials_kernel");
    if (st) return st;
    const int64_t rows = (int64_t)B * T;
    reduce_chunks_d<<<grid1(rows, 256), 256, 0, s>>>((const double*)work, rows, nc, out);
    return check_launch("reduce_chunks_d");
}

int sglm_eta_axpy(int64_t n, int64_t ld, int32_t B, const int32_t* slots, const float* step,
                  const float* deta, float* eta, sglm_stream_t stream) {
    if (B <= 0) return SGLM_OK;
    if (!step || !deta || !eta) { set_error("sglm_eta_axpy: null pointer"); return SGLM_EINVAL; }
    dim3 grid(grid1(n, 256, 1024), (unsigned)B);
    eta_axpy_kernel<<<grid, 256, 0, as_stream(stream)>>>(n, ld, slots, step, deta, eta);
    return check_launch("eta_axpy_kernel");
}

int sglm_eta_axpy_max(int64_t n, int64_t ld, int32_t B, const float* step, const float* deta,
                      const uint8_t* M, const int32_t* fit_mask, float* eta, float* dmax,
                      sglm_stream_t stream) {
    if (B <= 0) return SGLM_OK;
    if (!step || !deta || !M || !fit_mask || !eta || !dmax) {
        set_error("sglm_eta_axpy_max: null pointer");
        return SGLM_EINVAL;
    }
    hipStream_t s = as_stream(stream);
    if (hipMemsetAsync(dmax, 0, sizeof(float) * (size_t)B, s) != hipSuccess) {
        set_error("sglm_eta_axpy_max: hipMemsetAsync failed");
        return SGLM_EHIP;
    }
    dim3 grid(grid1(n, 256, 1024), (unsigned)B);
    eta_axpy_max_kernel<<<grid, 256, 0, s>>>(n, ld, step, deta, M, fit_mask, eta, dmax);
    return check_launch("eta_axpy_max_kernel");
}

int sglm_eta_pair_absmax(int64_t n, int64_t ld, int32_t npairs, const int32_t* pairs,
                         const uint8_t* M, const int32_t* fit_mask, const float* eta,
                         float* out, sglm_stream_t stream) {
    if (npairs <= 0) return SGLM_OK;
    if (!pairs || !M || !fit_mask || !eta || !out) {
        set_error("sglm_eta_pair_absmax: null pointer");
        return SGLM_EINVAL;
    }
    hipStream_t s = as_stream(stream);
    if (hipMemsetAsync(out, 0, sizeof(float) * (size_t)npairs, s) != hipSuccess) {
        set_error("sglm_eta_pair_absmax: hipMemsetAsync failed");
        return SGLM_EHIP;
    }
    dim3 grid(grid1(n, 256, 256), (unsigned)npairs);
    eta_pair_absmax_kernel<<<grid, 256, 0, s>>>(n, ld, pairs, M, fit_mask, eta, out);
    return check_launch("eta_pair_absmax_kernel");
}

int sglm_step_scalars(int32_t P, int32_t ncoef, int32_t B, const int32_t* slots, const double* g,
                      const double* beta, const float* delta, const double* lamp,
                      const double* t, int32_t T, double* out, sglm_stream_t stream) {
    if (B <= 0) return SGLM_OK;
    if (!slots || !g || !beta || !delta || !lamp || !t || !out || T < 0 || T > kMaxStepT) {
        set_error("sglm_step_scalars: bad args (T=%d, max %d)", T, kMaxStepT);
        return SGLM_EINVAL;
    }
    step_scalars_kernel<<<(unsigned)B, 256, 0, as_stream(stream)>>>(P, ncoef, slots, g, beta,
                                                                    delta, lamp, t, T, out);
    return check_launch("step_scalars_kernel");
}

int sglm_step_decide(int32_t na, const int32_t* act, const double* L, const double* sc,
                     int32_t nts, const double* ts, double sigma, double tol, double sfloor,
                     int32_t legacy, const float* aa_rm, const double* prev_rel,
                     const uint8_t* fresh, const int32_t* n_iter, const int32_t* max_iter,
                     double* step64, float* step32, double* relv, double* prop, int32_t* flags,
                     int32_t* tix, int32_t* rpos, int32_t* nxt, int32_t* cnt,
                     sglm_stream_t stream) {
    if (na <= 0) return SGLM_OK;
    if (!act || !L || !sc || !ts || nts < 5 || nts > kMaxStepT || !prev_rel || !fresh ||
        !n_iter || !max_iter || !step64 || !step32 || !relv || !prop || !flags || !tix ||
        !rpos || !nxt || !cnt) {
        set_error("sglm_step_decide: bad args");
        return SGLM_EINVAL;
    }
    step_decide_kernel<<<1, kDecT, 0, as_stream(stream)>>>(
        na, act, L, sc, nts, ts, sigma, tol, sfloor, legacy, aa_rm, prev_rel, fresh, n_iter,
        max_iter, step64, step32, relv, prop, flags, tix, rpos, nxt, cnt);
    return check_launch("step_decide_kernel");
}

int sglm_aa_step(int32_t P, int32_t p, int32_t na, const int32_t* slots, const uint8_t* sel,
                 const float* tprev, float* delta, float* raw_prev, const float* used_prev,
                 const double* gtot, float* rm, sglm_stream_t stream) {
    if (na <= 0) return SGLM_OK;
    if (!slots || !sel || !tprev || !delta || !raw_prev || !used_prev || !gtot || !rm ||
        p < 0 || p >= P) {
        set_error("sglm_aa_step: bad args");
        return SGLM_EINVAL;
    }
    aa_step_kernel<<<(unsigned)na, 256, 0, as_stream(stream)>>>(P, p, slots, sel, tprev, delta,
                                                                raw_prev, used_prev, gtot, rm);
    return check_launch("aa_step_kernel");
}

int sglm_step_update(int32_t P, int32_t B, const int32_t* slots, const double* step,
                     const float* delta, double* beta, sglm_stream_t stream) {
    if (B <= 0) return SGLM_OK;
    if (!slots || !step || !delta || !beta) {
        set_error("sglm_step_update: null pointer");
        return SGLM_EINVAL;
    }
    step_update_kernel<<<(unsigned)B, 256, 0, as_stream(stream)>>>(P, slots, step, delta, beta);
    return check_launch("step_update_kernel");
}

size_t sglm_mask_stats_work_bytes(int32_t F, int32_t R, int64_t n) {
    return (size_t)F * R * kStat * row_chunks(n) * sizeof(double);
}

int sglm_mask_stats(const uint8_t* M, int64_t ldm, int32_t F, const double* Y, int32_t R,
                    int64_t n, const double* K, double power, double* out, void* work,
                    sglm_stream_t stream) {
    if (F <= 0 || R <= 0) return SGLM_OK;
    if (!M || !Y || !K || !out || !work || ldm < n) {
        set_error("sglm_mask_stats: bad args");
        return SGLM_EINVAL;
    }
    hipStream_t s = as_stream(stream);
    const int32_t nc = row_chunks(n);
    mask_stats_kernel<<<dim3((unsigned)nc, (unsigned)F, (unsigned)R), 256, 0, s>>>(
        M, Y, K, n, ldm, F, power, (double*)work);
    int st = check_launch("mask_stats_kernel");
    if (st) return st;
    const int64_t rows = (int64_t)R * F * kStat;
    mask_stats_reduce<<<grid1(rows, 256), 256, 0, s>>>((const double*)work, rows, nc, out);
    return check_launch("mask_stats_reduce");
}

int sglm_score_sums(int32_t family, float power, int64_t n, int64_t ld, int32_t B,
                    const float* eta, const float* Y, const uint8_t* M,
                    const int32_t* fit_resp, const int32_t* sets, double* out, void* work,
                    sglm_stream_t stream) {
    if (B <= 0) return SGLM_OK;
    if (!eta || !Y || !M || !fit_resp || !sets || !out || !work) { set_error("sglm_score_sums: null pointer"); return SGLM_EINVAL; }
    const int32_t nc = row_chunks(n);
    hipStream_t s = as_stream(stream);
    score_kernel<<<dim3((unsigned)nc, (unsigned)B), 256, 0, s>>>(family, power, n, ld, eta, Y, M, fit_resp, sets, (double*)work);
    int st = check_launch("score_kernel");
    if (st) return st;
    const int64_t rows = (int64_t)B * 4;
    reduce_chunks_d<<<grid1(rows, 256), 256, 0, s>>>((const double*)work, rows, nc, out);
    return check_launch("reduce_chunks_d");
}

}  // extern "C"
