// Mixed 0/1 + continuous designs: the k non-binary columns are held as a dense float64 block
// C [k][ldc] beside the bit-planes of the 0/1 columns (their bit columns are zero), at design
// positions cpos[c].  Every product the bit-plane kernels form over a zero column is completed
// here, so the 0/1 columns keep the bf16-MFMA Gram / gradient / predictor kernels and the
// continuous columns enter the fit in float64 (the reference fits float64 X:
// sglm_cb_concat_make_design_mat.py:224-244 adds cumcount^2/5000 counters beside the 0/1
// events, pp_design_mat.py:167-172, and fits OLS through simple_cv_fit, :356-363).
//
//   sglm_mixed_wc      R[s*k + c] = W[slot_s] * C[c]  (f32 rows: the operand of the bit-plane
//                      X^T R kernel for the Gram rows X^T W C of a weighted IRLS Hessian)
//   sglm_mixed_gram    S[s][c][cpos[c']] = sum_r wt_s(r) C[c][r] C[c'][r]  (float64, both
//                      orders), wt = f32 IRLS weights or uint8 mask multiplicities
//   sglm_mixed_xtr     g[gslot_q][cpos[c]] = sum_r C[c][r] R_q(r)  (float64: the gradient's
//                      continuous coordinates; R as f32 rows, the link kernel's packed three
//                      bf16 pieces, or one bf16 integer digit plane)
//   sglm_mixed_eta     eta[slot][r] += sum_c C[c][r] beta[slot][cpos[c]]  (float64 sum)
//   sglm_mixed_to_h    H[slot][i][cpos[c]] = H[slot][cpos[c]][i] = S[s][c][i]  (f32 Hessian)
//
// Reductions over rows are chunked (kMxRows rows per workgroup) and the chunk partials summed
// in a fixed order by a second kernel: results are deterministic run to run.
#include "common.h"

namespace sglm {
namespace {

constexpr int kMxT = 256;           // threads per workgroup
constexpr int kMxRows = 8192;       // rows of one reduction chunk (32 per thread)
constexpr int kMxTile = 8;          // outputs (column pairs) per workgroup
constexpr int kMxMaxK = 1024;       // continuous columns (LDS of the predictor kernel)

enum : int { WT_F32 = 0, WT_U8 = 1, R_PIECES = 2, R_BF16 = 3 };

template <int MODE>
__device__ __forceinline__ double weight_at(const void* __restrict__ src, int64_t ld, int64_t row,
                                            int64_t Bp, int64_t r) {
    if (MODE == WT_F32) return (double)reinterpret_cast<const float*>(src)[row * ld + r];
    if (MODE == WT_U8) return (double)reinterpret_cast<const uint8_t*>(src)[row * ld + r];
    const uint16_t* b = reinterpret_cast<const uint16_t*>(src);
    if (MODE == R_BF16) return (double)bf16_bits_to_f32(b[row * ld + r]);
    // R_PIECES: [3][Bp][ld], hi + mid + lo == R exactly
    const int64_t o = row * ld + r, ps = Bp * ld;
    return ((double)bf16_bits_to_f32(b[o]) + (double)bf16_bits_to_f32(b[o + ps])) +
           (double)bf16_bits_to_f32(b[o + 2 * ps]);
}

// part[((s * nchunk) + chunk) * npairs + q] = sum over the chunk's rows of
// wt(s, r) * C[pa[q]][r] * (pb[q] < k ? C[pb[q]][r] : 1); blockIdx = (chunk, s, pair tile)
template <int MODE>
__global__ void __launch_bounds__(kMxT) mixed_dot_kernel(
    const void* __restrict__ wsrc, int64_t ldw, int64_t Bp, const int32_t* __restrict__ wsel,
    const double* __restrict__ C, int64_t ldc, int32_t k, const int32_t* __restrict__ pa,
    const int32_t* __restrict__ pb, int32_t npairs, int64_t n, int32_t nchunk,
    double* __restrict__ part) {
    const int chunk = blockIdx.x, s = blockIdx.y, q0 = blockIdx.z * kMxTile;
    const int nq = min(kMxTile, npairs - q0);
    const int64_t row = wsel ? wsel[s] : s;
    int ia[kMxTile], ib[kMxTile];
#pragma unroll
    for (int q = 0; q < kMxTile; ++q) {
        ia[q] = q < nq ? pa[q0 + q] : 0;
        ib[q] = q < nq ? pb[q0 + q] : k;
    }
    double acc[kMxTile];
#pragma unroll
    for (int q = 0; q < kMxTile; ++q) acc[q] = 0.0;
    const int64_t r0 = (int64_t)chunk * kMxRows;
    const int64_t r1 = min<int64_t>(r0 + kMxRows, n);
    for (int64_t r = r0 + threadIdx.x; r < r1; r += kMxT) {
        const double w = weight_at<MODE>(wsrc, ldw, row, Bp, r);
#pragma unroll
        for (int q = 0; q < kMxTile; ++q) {
            if (q < nq) {
                const double a = C[(int64_t)ia[q] * ldc + r];
                const double b = ib[q] < k ? C[(int64_t)ib[q] * ldc + r] : 1.0;
                acc[q] = fma(w * a, b, acc[q]);
            }
        }
    }
    __shared__ double red[kMxT / kWave][kMxTile];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
    for (int q = 0; q < kMxTile; ++q) {
        const double v = wave_sum_d(acc[q]);
        if (lane == 0) red[wv][q] = v;
    }
    __syncthreads();
    if (threadIdx.x < nq) {
        const int q = threadIdx.x;
        double v = red[0][q];
        for (int w = 1; w < kMxT / kWave; ++w) v += red[w][q];
        part[((int64_t)s * nchunk + chunk) * npairs + q0 + q] = v;
    }
}

// Fixed-order sum of the chunk partials of output (s, q), written to its destination:
// GRAD = 0 (Gram block): S[s][a][cpos[b]] and S[s][b][cpos[a]]; GRAD = 1: g[gsl[s]][cpos[a]].
template <int GRAD>
__global__ void __launch_bounds__(kMxT) mixed_finish_kernel(
    const double* __restrict__ part, int32_t ns, int32_t nchunk, int32_t npairs,
    const int32_t* __restrict__ pa, const int32_t* __restrict__ pb, int32_t k,
    const int32_t* __restrict__ cpos, int32_t P, const int32_t* __restrict__ gsl,
    double* __restrict__ dst) {
    const int64_t t = (int64_t)blockIdx.x * kMxT + threadIdx.x;
    if (t >= (int64_t)ns * npairs) return;
    const int s = (int)(t / npairs), q = (int)(t % npairs);
    const double* pp = part + (int64_t)s * nchunk * npairs + q;
    double v = 0.0;
    for (int c = 0; c < nchunk; ++c) v += pp[(int64_t)c * npairs];
    const int a = pa[q], b = pb[q];
    if (GRAD) {
        const int64_t row = gsl ? gsl[s] : s;
        dst[row * P + cpos[a]] = v;
    } else {
        dst[((int64_t)s * k + a) * P + cpos[b]] = v;
        dst[((int64_t)s * k + b) * P + cpos[a]] = v;
    }
}

// Gradient rows: part[((q * nchunk) + chunk) * k + c] = sum over the chunk's rows of
// C[c][r] R_q(r) for the fits q of one group of kMxG (blockIdx.y) and the columns c of one tile
// of kMxKT (blockIdx.z).  Each lane takes 4 consecutive rows per step (one 32-B load of C per
// column, one 8-B load of each R piece per fit): C is read once per group of fits, not once per
// fit, and the fits' R pieces once per column tile.
constexpr int kMxG = 8;             // fits per workgroup (gradient / predictor kernels)
constexpr int kMxKT = 4;            // continuous columns per workgroup
constexpr int kMxGRows = 32768;     // rows of one gradient chunk (32 steps of 4 rows per lane)

template <int MODE>
__device__ __forceinline__ void r4_at(const void* __restrict__ src, int64_t ld, int64_t row,
                                      int64_t Bp, int64_t r, double out[4]) {
    if (MODE == WT_F32) {
        const float4 v = *reinterpret_cast<const float4*>(
            reinterpret_cast<const float*>(src) + row * ld + r);
        out[0] = v.x; out[1] = v.y; out[2] = v.z; out[3] = v.w;
        return;
    }
    const uint16_t* b = reinterpret_cast<const uint16_t*>(src);
    const int64_t o = row * ld + r;
    const uint2 h = *reinterpret_cast<const uint2*>(b + o);
    double t[4] = {(double)__uint_as_float(h.x << 16), (double)__uint_as_float(h.x & 0xffff0000u),
                   (double)__uint_as_float(h.y << 16), (double)__uint_as_float(h.y & 0xffff0000u)};
    if (MODE == R_PIECES) {
        const int64_t ps = Bp * ld;
        const uint2 m = *reinterpret_cast<const uint2*>(b + o + ps);
        const uint2 l = *reinterpret_cast<const uint2*>(b + o + 2 * ps);
        t[0] = (t[0] + (double)__uint_as_float(m.x << 16)) + (double)__uint_as_float(l.x << 16);
        t[1] = (t[1] + (double)__uint_as_float(m.x & 0xffff0000u)) +
               (double)__uint_as_float(l.x & 0xffff0000u);
        t[2] = (t[2] + (double)__uint_as_float(m.y << 16)) + (double)__uint_as_float(l.y << 16);
        t[3] = (t[3] + (double)__uint_as_float(m.y & 0xffff0000u)) +
               (double)__uint_as_float(l.y & 0xffff0000u);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) out[j] = t[j];
}

template <int MODE>
__global__ void __launch_bounds__(kMxT) mixed_grad_kernel(
    const void* __restrict__ R, int64_t ldr, int64_t Bp, const int32_t* __restrict__ rsel,
    int32_t nq, const double* __restrict__ C, int64_t ldc, int32_t k, int64_t n,
    int32_t nchunk, double* __restrict__ part) {
    const int chunk = blockIdx.x, q0 = blockIdx.y * kMxG, c0 = blockIdx.z * kMxKT;
    const int nf = min(kMxG, nq - q0), nc = min(kMxKT, k - c0);
    int64_t row[kMxG];
#pragma unroll
    for (int f = 0; f < kMxG; ++f) row[f] = f < nf ? (rsel ? rsel[q0 + f] : q0 + f) : 0;
    double acc[kMxG][kMxKT];
#pragma unroll
    for (int f = 0; f < kMxG; ++f)
#pragma unroll
        for (int c = 0; c < kMxKT; ++c) acc[f][c] = 0.0;
    const int64_t r0 = (int64_t)chunk * kMxGRows;
    const int64_t r1 = min<int64_t>(r0 + kMxGRows, n);
    for (int64_t r = r0 + 4 * (int64_t)threadIdx.x; r < r1; r += 4 * kMxT) {
        double cv[kMxKT][4];
#pragma unroll
        for (int c = 0; c < kMxKT; ++c) {
            if (c < nc && r + 3 < r1) {
                const double4 v = *reinterpret_cast<const double4*>(C + (int64_t)(c0 + c) * ldc + r);
                cv[c][0] = v.x; cv[c][1] = v.y; cv[c][2] = v.z; cv[c][3] = v.w;
            } else {
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    cv[c][j] = (c < nc && r + j < r1) ? C[(int64_t)(c0 + c) * ldc + r + j] : 0.0;
            }
        }
#pragma unroll
        for (int f = 0; f < kMxG; ++f) {
            if (f < nf) {
                double rv[4];
                r4_at<MODE>(R, ldr, row[f], Bp, r, rv);     // rows < ld: in bounds (ld % 4 == 0)
#pragma unroll
                for (int c = 0; c < kMxKT; ++c)
#pragma unroll
                    for (int j = 0; j < 4; ++j) acc[f][c] = fma(cv[c][j], rv[j], acc[f][c]);
            }
        }
    }
    __shared__ double red[kMxT / kWave][kMxG * kMxKT];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
    for (int f = 0; f < kMxG; ++f)
#pragma unroll
        for (int c = 0; c < kMxKT; ++c) {
            const double v = wave_sum_d(acc[f][c]);
            if (lane == 0) red[wv][f * kMxKT + c] = v;
        }
    __syncthreads();
    if (threadIdx.x < kMxG * kMxKT) {
        const int f = threadIdx.x / kMxKT, c = threadIdx.x % kMxKT;
        if (f < nf && c < nc) {
            double v = red[0][threadIdx.x];
            for (int w = 1; w < kMxT / kWave; ++w) v += red[w][threadIdx.x];
            part[((int64_t)(q0 + f) * nchunk + chunk) * k + c0 + c] = v;
        }
    }
}

// eta[slot][r] += sum_c C[c][r] * beta[slot][cpos[c]] for r < n (float64 sum, one rounding) for
// the fits of one group of kMxG (blockIdx.y): lanes take 4 consecutive rows, C read once per
// group (columns in tiles of kMxKT)
constexpr int kMxEtaK = 64;         // continuous columns of the grouped predictor kernel

__global__ void __launch_bounds__(kMxT) mixed_eta4_kernel(
    const double* __restrict__ C, int64_t ldc, int32_t k, int64_t n,
    const int32_t* __restrict__ cpos, const float* __restrict__ beta, int32_t P,
    const int32_t* __restrict__ slots, int32_t nb, float* __restrict__ eta, int64_t ld) {
    __shared__ double b[kMxG][kMxEtaK];
    const int q0 = blockIdx.y * kMxG;
    const int nf = min(kMxG, nb - q0);
    int64_t slot[kMxG];
#pragma unroll
    for (int f = 0; f < kMxG; ++f) slot[f] = f < nf ? (slots ? slots[q0 + f] : q0 + f) : 0;
    for (int t = threadIdx.x; t < kMxG * k; t += kMxT) {
        const int f = t / k, c = t % k;
        b[f][c] = f < nf ? (double)beta[slot[f] * P + cpos[c]] : 0.0;
    }
    __syncthreads();
    for (int64_t r = 4 * ((int64_t)blockIdx.x * kMxT + threadIdx.x); r < n;
         r += 4 * (int64_t)gridDim.x * kMxT) {
        double acc[kMxG][4];
#pragma unroll
        for (int f = 0; f < kMxG; ++f)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[f][j] = 0.0;
        for (int c = 0; c < k; ++c) {
            double cv[4];
            if (r + 3 < n) {
                const double4 v = *reinterpret_cast<const double4*>(C + (int64_t)c * ldc + r);
                cv[0] = v.x; cv[1] = v.y; cv[2] = v.z; cv[3] = v.w;
            } else {
#pragma unroll
                for (int j = 0; j < 4; ++j) cv[j] = r + j < n ? C[(int64_t)c * ldc + r + j] : 0.0;
            }
#pragma unroll
            for (int f = 0; f < kMxG; ++f)
#pragma unroll
                for (int j = 0; j < 4; ++j) acc[f][j] = fma(cv[j], b[f][c], acc[f][j]);
        }
#pragma unroll
        for (int f = 0; f < kMxG; ++f) {
            if (f < nf) {
                float* e = eta + slot[f] * ld + r;
                if (r + 3 < n) {
                    float4 v = *reinterpret_cast<float4*>(e);
                    v.x = (float)((double)v.x + acc[f][0]);
                    v.y = (float)((double)v.y + acc[f][1]);
                    v.z = (float)((double)v.z + acc[f][2]);
                    v.w = (float)((double)v.w + acc[f][3]);
                    *reinterpret_cast<float4*>(e) = v;
                } else {
                    for (int j = 0; j < 4 && r + j < n; ++j)
                        e[j] = (float)((double)e[j] + acc[f][j]);
                }
            }
        }
    }
}

// eta[slot][r] += sum_c C[c][r] * beta[slot][cpos[c]] for r < n (float64 sum, one rounding)
__global__ void __launch_bounds__(kMxT) mixed_eta_kernel(
    const double* __restrict__ C, int64_t ldc, int32_t k, int64_t n,
    const int32_t* __restrict__ cpos, const float* __restrict__ beta, int32_t P,
    const int32_t* __restrict__ slots, float* __restrict__ eta, int64_t ld) {
    __shared__ double b[kMxMaxK];
    const int64_t slot = slots ? slots[blockIdx.y] : blockIdx.y;
    for (int c = threadIdx.x; c < k; c += kMxT) b[c] = (double)beta[slot * P + cpos[c]];
    __syncthreads();
    float* e = eta + slot * ld;
    for (int64_t r = (int64_t)blockIdx.x * kMxT + threadIdx.x; r < n;
         r += (int64_t)gridDim.x * kMxT) {
        double acc = (double)e[r];
        for (int c = 0; c < k; ++c) acc = fma(C[(int64_t)c * ldc + r], b[c], acc);
        e[r] = (float)acc;
    }
}

// R[q][r] = W[slots[q / k]][r] * f32(C[q % k][r]) for r < n, 0 for n <= r < ld
__global__ void __launch_bounds__(kMxT) mixed_wc_kernel(
    const float* __restrict__ W, int64_t ldw, const int32_t* __restrict__ slots, int32_t k,
    const double* __restrict__ C, int64_t ldc, int64_t n, int64_t ld, float* __restrict__ R) {
    const int q = blockIdx.y;
    const int64_t slot = slots ? slots[q / k] : q / k;
    const int c = q % k;
    const float* w = W + slot * ldw;
    const double* cc = C + (int64_t)c * ldc;
    float* out = R + (int64_t)q * ld;
    for (int64_t r = (int64_t)blockIdx.x * kMxT + threadIdx.x; r < ld;
         r += (int64_t)gridDim.x * kMxT)
        out[r] = r < n ? w[r] * (float)cc[r] : 0.0f;
}

// H[slot][i][cpos[c]] = H[slot][cpos[c]][i] = f32(S[s][c][i]), i < P
__global__ void __launch_bounds__(kMxT) mixed_to_h_kernel(
    const double* __restrict__ S, int32_t k, int32_t P, const int32_t* __restrict__ cpos,
    const int32_t* __restrict__ slots, float* __restrict__ H) {
    const int s = blockIdx.y, c = blockIdx.z;
    const int i = blockIdx.x * kMxT + threadIdx.x;
    if (i >= P) return;
    const int64_t slot = slots ? slots[s] : s;
    const float v = (float)S[((int64_t)s * k + c) * P + i];
    const int64_t j = cpos[c];
    float* Hs = H + slot * (int64_t)P * P;
    Hs[(int64_t)i * P + j] = v;
    Hs[j * P + i] = v;
}

int nchunks(int64_t n) { return (int)((n + kMxRows - 1) / kMxRows); }

template <int MODE>
void launch_dot(const void* w, int64_t ldw, int64_t Bp, const int32_t* wsel, int32_t ns,
                const double* C, int64_t ldc, int32_t k, const int32_t* pa, const int32_t* pb,
                int32_t npairs, int64_t n, double* part, hipStream_t s) {
    const int nc = nchunks(n);
    dim3 grid((unsigned)nc, (unsigned)ns, (unsigned)((npairs + kMxTile - 1) / kMxTile));
    mixed_dot_kernel<MODE><<<grid, kMxT, 0, s>>>(w, ldw, Bp, wsel, C, ldc, k, pa, pb, npairs, n,
                                                 nc, part);
}

}  // namespace
}  // namespace sglm

using namespace sglm;

extern "C" {

size_t sglm_mixed_work_bytes(int32_t ns, int32_t k, int64_t n) {
    if (ns <= 0 || k <= 0 || n <= 0) return 16;
    const int64_t npairs = (int64_t)k * (k + 1) / 2 > k ? (int64_t)k * (k + 1) / 2 : k;
    return (size_t)((int64_t)ns * nchunks(n) * npairs * sizeof(double));   // >= the gradient's
}

int sglm_mixed_wc(const float* W, int64_t ldw, const int32_t* slots, int32_t ns,
                  const double* C, int64_t ldc, int32_t k, int64_t n, int64_t ld, float* R,
                  sglm_stream_t stream) {
    if (ns <= 0 || k <= 0) return SGLM_OK;
    if (!W || !C || !R || n < 0 || ld < n || ldw < n || ldc < n || (int64_t)ns * k > 65535) {
        set_error("sglm_mixed_wc: bad args (ns=%d k=%d n=%lld)", ns, k, (long long)n);
        return SGLM_EINVAL;
    }
    const int64_t blocks = (ld + kMxT * 4 - 1) / (kMxT * 4);
    dim3 grid((unsigned)(blocks < 1 ? 1 : blocks), (unsigned)(ns * k));
    mixed_wc_kernel<<<grid, kMxT, 0, as_stream(stream)>>>(W, ldw, slots, k, C, ldc, n, ld, R);
    return check_launch("sglm_mixed_wc");
}

int sglm_mixed_gram(int32_t wmode, const void* wsrc, int64_t ldw, const int32_t* wsel, int32_t ns,
                    const double* C, int64_t ldc, int32_t k, int64_t n, const int32_t* cpos,
                    int32_t P, const int32_t* pairs, double* S, void* work, sglm_stream_t stream) {
    if (ns <= 0 || k <= 0) return SGLM_OK;
    if (!wsrc || !C || !cpos || !S || !work || !pairs || n <= 0 || ldc < n || ldw < n ||
        (wmode != WT_F32 && wmode != WT_U8) || ns > 65535) {
        set_error("sglm_mixed_gram: bad args (mode=%d ns=%d k=%d)", wmode, ns, k);
        return SGLM_EINVAL;
    }
    hipStream_t s = as_stream(stream);
    const int npairs = k * (k + 1) / 2;
    double* part = (double*)work;
    const int32_t* pa = pairs;
    const int32_t* pb = pairs + npairs;
    if (wmode == WT_F32)
        launch_dot<WT_F32>(wsrc, ldw, 0, wsel, ns, C, ldc, k, pa, pb, npairs, n, part, s);
    else
        launch_dot<WT_U8>(wsrc, ldw, 0, wsel, ns, C, ldc, k, pa, pb, npairs, n, part, s);
    int st = check_launch("mixed_dot_kernel");
    if (st) return st;
    const int64_t tot = (int64_t)ns * npairs;
    mixed_finish_kernel<0><<<(unsigned)((tot + kMxT - 1) / kMxT), kMxT, 0, s>>>(
        part, ns, nchunks(n), npairs, pa, pb, k, cpos, P, nullptr, S);
    return check_launch("sglm_mixed_gram");
}

int sglm_mixed_xtr(int32_t rmode, const void* R, int64_t ldr, int64_t Bp, const int32_t* rsel,
                   const int32_t* gslots, int32_t nq, const double* C, int64_t ldc, int32_t k,
                   int64_t n, const int32_t* cpos, int32_t P, const int32_t* pairs, double* g,
                   void* work, sglm_stream_t stream) {
    if (nq <= 0 || k <= 0) return SGLM_OK;
    if (!R || !C || !cpos || !g || !work || !pairs || n <= 0 || ldc < n || ldr < n ||
        (rmode != WT_F32 && rmode != R_PIECES && rmode != R_BF16) || nq > 65535 ||
        (rmode == R_PIECES && Bp < nq)) {
        set_error("sglm_mixed_xtr: bad args (mode=%d nq=%d k=%d)", rmode, nq, k);
        return SGLM_EINVAL;
    }
    if (ldr % 4 || ldc % 4) {
        set_error("sglm_mixed_xtr: row strides must be multiples of 4 (ldr=%lld ldc=%lld)",
                  (long long)ldr, (long long)ldc);
        return SGLM_EINVAL;
    }
    hipStream_t s = as_stream(stream);
    double* part = (double*)work;
    const int32_t* pa = pairs;        // 0 .. k-1
    const int32_t* pb = pairs + k;    // k (the ones factor)
    const int nc = (int)((n + kMxGRows - 1) / kMxGRows);
    dim3 grid((unsigned)nc, (unsigned)((nq + kMxG - 1) / kMxG), (unsigned)((k + kMxKT - 1) / kMxKT));
    if (rmode == WT_F32)
        mixed_grad_kernel<WT_F32><<<grid, kMxT, 0, s>>>(R, ldr, Bp, rsel, nq, C, ldc, k, n, nc, part);
    else if (rmode == R_PIECES)
        mixed_grad_kernel<R_PIECES><<<grid, kMxT, 0, s>>>(R, ldr, Bp, rsel, nq, C, ldc, k, n, nc, part);
    else
        mixed_grad_kernel<R_BF16><<<grid, kMxT, 0, s>>>(R, ldr, Bp, rsel, nq, C, ldc, k, n, nc, part);
    int st = check_launch("mixed_grad_kernel");
    if (st) return st;
    const int64_t tot = (int64_t)nq * k;
    mixed_finish_kernel<1><<<(unsigned)((tot + kMxT - 1) / kMxT), kMxT, 0, s>>>(
        part, nq, nc, k, pa, pb, k, cpos, P, gslots, g);
    return check_launch("sglm_mixed_xtr");
}

int sglm_mixed_eta(const double* C, int64_t ldc, int32_t k, int64_t n, const int32_t* cpos,
                   const float* beta, int32_t P, const int32_t* slots, int32_t nb, float* eta,
                   int64_t ld, sglm_stream_t stream) {
    if (nb <= 0 || k <= 0 || n <= 0) return SGLM_OK;
    if (!C || !cpos || !beta || !eta || k > kMxMaxK || ldc < n || ld < n || nb > 65535) {
        set_error("sglm_mixed_eta: bad args (k=%d nb=%d)", k, nb);
        return SGLM_EINVAL;
    }
    if (ld % 4 == 0 && ldc % 4 == 0 && k <= kMxEtaK) {
        // rows in steps of 4 per lane, fits in groups of kMxG; ~2 K workgroups in total
        const int ng = (nb + kMxG - 1) / kMxG;
        int64_t blocks = (n + 4 * kMxT - 1) / (4 * kMxT);
        const int64_t want = (2048 + ng - 1) / ng;
        if (blocks > want) blocks = want;
        mixed_eta4_kernel<<<dim3((unsigned)blocks, (unsigned)ng), kMxT, 0, as_stream(stream)>>>(
            C, ldc, k, n, cpos, beta, P, slots, nb, eta, ld);
        return check_launch("sglm_mixed_eta");
    }
    int64_t blocks = (n + kMxT * 8 - 1) / (kMxT * 8);
    if (blocks > 4096) blocks = 4096;
    mixed_eta_kernel<<<dim3((unsigned)blocks, (unsigned)nb), kMxT, 0, as_stream(stream)>>>(
        C, ldc, k, n, cpos, beta, P, slots, eta, ld);
    return check_launch("sglm_mixed_eta");
}

int sglm_mixed_to_h(const double* S, int32_t ns, int32_t k, int32_t P, const int32_t* cpos,
                    const int32_t* slots, float* H, sglm_stream_t stream) {
    if (ns <= 0 || k <= 0) return SGLM_OK;
    if (!S || !cpos || !H || P <= 0 || ns > 65535 || k > 65535) {
        set_error("sglm_mixed_to_h: bad args (ns=%d k=%d P=%d)", ns, k, P);
        return SGLM_EINVAL;
    }
    dim3 grid((unsigned)((P + kMxT - 1) / kMxT), (unsigned)ns, (unsigned)k);
    mixed_to_h_kernel<<<grid, kMxT, 0, as_stream(stream)>>>(S, k, P, cpos, slots, H);
    return check_launch("sglm_mixed_to_h");
}

}  // extern "C"
