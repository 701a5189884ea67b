// Bit-planes of a time-shifted 0/1 event design straight from the events.
//
// Column (b, a) of the design is event a shifted by s_b rows, X[t, (b, a)] = E[t + row0 - s_b, a]
// (sglm_ez.timeshift_cols, backend/sglm_ez.py:102-123), plus the ones column at p.  The Gram and
// the gradient read the column planes (xbits: bit i of word w of column j = X[32 w + i, j]) and
// the predictor products the row-major planes (rbits: per 64-column group g and row t, the
// group's 64 bits in the MFMA fragment order).  Both used to be packed from the dense bf16
// design (P x ld, 4 GB at C4: written by the timeshift kernel, read by two pack kernels); here
// a column word is a 32-bit window of its event's occurrence bitmap, cut at the shifted row:
//   event_bits: E (bf16, event-major) -> one bitmap per event, one wave ballot per 64 rows;
//   lag_xbits:  xbits[j][w] = bits [32 w + row0 - s_j, +32) of bitmap cols[j] (zero outside
//               the raw rows, masked to the design's n rows), the ones column, zero padding;
//   lag_rbits:  a 64 x 64 bit transpose per (64 rows, 64 columns) with 64 wave ballots.
#include "common.h"

namespace sglm {
namespace {

// ebits[a][w] bit i = (E[32 w + i][a] != 0); Eb is bf16 [m][lde] (event-major)
__global__ void __launch_bounds__(256) event_bits_kernel(const uint16_t* __restrict__ Eb,
                                                         int64_t lde, int32_t m, int64_t n_raw,
                                                         int64_t nwords,
                                                         uint32_t* __restrict__ ebits) {
    const int lane = threadIdx.x & 63;
    const int64_t nch = (n_raw + 63) / 64;
    const int64_t total = nch * m;
    for (int64_t g = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 6; g < total;
         g += ((int64_t)gridDim.x * 256) >> 6) {
        const int64_t a = g / nch, c = g % nch;
        const int64_t u = c * 64 + lane;
        const uint16_t v = u < n_raw ? Eb[a * lde + u] : (uint16_t)0;
        const unsigned long long b = __ballot((v & 0x7FFFu) != 0);
        if (lane == 0) {
            ebits[a * nwords + 2 * c] = (uint32_t)b;
            if (2 * c + 1 < nwords) ebits[a * nwords + 2 * c + 1] = (uint32_t)(b >> 32);
        }
    }
}

__device__ __forceinline__ uint32_t bit_window(const uint32_t* __restrict__ words, int64_t nwords,
                                               int64_t o) {
    if (o >= 32 * nwords || o <= -32) return 0u;
    const int64_t q = o >> 5;                     // floor(o / 32)
    const int sh = (int)(o & 31);
    const uint32_t w0 = (q >= 0 && q < nwords) ? words[q] : 0u;
    if (sh == 0) return w0;
    const uint32_t w1 = (q + 1 >= 0 && q + 1 < nwords) ? words[q + 1] : 0u;
    return (w0 >> sh) | (w1 << (32 - sh));
}

__global__ void __launch_bounds__(256) lag_xbits_kernel(
    const uint32_t* __restrict__ ebits, int64_t nwords, const int32_t* __restrict__ cols,
    const int32_t* __restrict__ shifts, int32_t p, int64_t row0, int64_t n, int64_t ld,
    int32_t P, uint32_t* __restrict__ xbits) {
    const int64_t wpc = ld / 32;                  // words per column
    const int64_t total = (int64_t)P * wpc;
    for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total;
         e += (int64_t)gridDim.x * 256) {
        const int64_t j = e / wpc, w = e % wpc;
        const int64_t t0 = 32 * w;
        uint32_t v = 0u;
        if (t0 < n && j <= p) {
            v = j < p ? bit_window(ebits + (int64_t)cols[j] * nwords, nwords,
                                   t0 + row0 - shifts[j])
                      : 0xFFFFFFFFu;
            if (t0 + 32 > n) v &= (1u << (int)(n - t0)) - 1u;
        }
        xbits[e] = v;
    }
}

// one wave per (64-row block, 64-column group): lane l loads column 64 g + l's 64 bits of the
// block, 64 ballots give the rows, lane i keeps row i and writes it in the fragment order
// (column al at bit 4 (al' >> 3) + ((al' & 7) >> 1) + 16 (al' & 1) of word al >> 5, al' = al & 31)
__global__ void __launch_bounds__(256) lag_rbits_kernel(const uint32_t* __restrict__ xbits,
                                                        int64_t ld, int32_t P,
                                                        u32x2* __restrict__ rbits) {
    const int lane = threadIdx.x & 63;
    const int64_t nrb = ld / 64, ngr = P / 64;
    const int64_t total = nrb * ngr;
    for (int64_t g = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 6; g < total;
         g += ((int64_t)gridDim.x * 256) >> 6) {
        const int64_t grp = g / nrb, rb = g % nrb;
        const uint32_t* col = xbits + (64 * grp + lane) * (ld / 32) + 2 * rb;
        const uint64_t cb = (uint64_t)col[0] | ((uint64_t)col[1] << 32);
        uint64_t mine = 0;
#pragma unroll 8
        for (int i = 0; i < 64; ++i) {
            const unsigned long long r = __ballot((cb >> i) & 1ull);
            mine = lane == i ? (uint64_t)r : mine;
        }
        uint32_t w[2] = {0u, 0u};
#pragma unroll
        for (int al = 0; al < 64; ++al) {
            const int rho = al & 31;
            const int pos = 4 * (rho >> 3) + ((rho & 7) >> 1) + 16 * (rho & 1);
            w[al >> 5] |= (uint32_t)((mine >> al) & 1ull) << pos;
        }
        rbits[grp * ld + rb * 64 + lane] = (u32x2){w[0], w[1]};
    }
}

}  // namespace
}  // namespace sglm

using namespace sglm;

extern "C" int sglm_event_bits(const uint16_t* Eb, int64_t lde, int32_t m, int64_t n_raw,
                               uint32_t* ebits, int64_t nwords, sglm_stream_t stream) {
    if (m <= 0 || n_raw <= 0) return SGLM_OK;
    if (!Eb || !ebits || lde < n_raw || nwords != (n_raw + 31) / 32) {
        set_error("sglm_event_bits: bad args");
        return SGLM_EINVAL;
    }
    const int64_t waves = (n_raw + 63) / 64 * m;
    const int64_t blocks = (waves + 3) / 4;
    event_bits_kernel<<<(unsigned)(blocks < 16384 ? blocks : 16384), 256, 0,
                        as_stream(stream)>>>(Eb, lde, m, n_raw, nwords, ebits);
    return check_launch("event_bits_kernel");
}

extern "C" int sglm_lag_bits(const uint32_t* ebits, int64_t nwords, const int32_t* cols,
                             const int32_t* shifts, int32_t p, int64_t row0, int64_t n,
                             int64_t ld, int32_t P, uint32_t* xbits, void* rbits,
                             sglm_stream_t stream) {
    if (!ebits || !xbits || !rbits || (p > 0 && (!cols || !shifts)) || ld % 64 || P % 64 ||
        p >= P || n > ld || n < 0) {
        set_error("sglm_lag_bits: bad args");
        return SGLM_EINVAL;
    }
    hipStream_t s = as_stream(stream);
    const int64_t total = (int64_t)P * (ld / 32);
    lag_xbits_kernel<<<(unsigned)((total + 255) / 256 < 32768 ? (total + 255) / 256 : 32768), 256,
                       0, s>>>(ebits, nwords, cols, shifts, p, row0, n, ld, P, xbits);
    int st = check_launch("lag_xbits_kernel");
    if (st) return st;
    const int64_t waves = (ld / 64) * (P / 64);
    const int64_t blocks = (waves + 3) / 4;
    lag_rbits_kernel<<<(unsigned)(blocks < 32768 ? blocks : 32768), 256, 0, s>>>(
        xbits, ld, P, reinterpret_cast<u32x2*>(rbits));
    return check_launch("lag_rbits_kernel");
}
