// Host-side (CPU) helpers of the grid setup, multithreaded.
//
// sglm_host_masks: the per-fold row masks of a CV grid from their index lists, written
// straight into the (pinned) upload buffer.  Replaces the per-fold `X[idx_train, :]` /
// `y[idx_train]` selections of the reference's fold loop (backend/sglm_cv.py:107-110) as
// one uint8 mask row per fold: 0/1 for a strictly increasing list (GroupShuffleSplit folds),
// the multiplicity for a list with repeats (holdout resampling), 1 on every listed row for a
// row list, all ones for "every row".  One thread per mask (a mask is ~1 MB of stores).
#include <algorithm>
#include <cstring>
#include <thread>
#include <vector>

#include "common.h"

extern "C" int sglm_host_simd_level(void);                      // host_simd.cpp
extern "C" void sglm_host_pack_block_avx512(const double* base, int64_t S, int32_t ncols,
                                            int64_t r0, int64_t r1, int64_t nwords,
                                            uint32_t* bits, uint8_t* bad, int64_t* cnt);

namespace {

struct MaskJob {
    const int64_t* idx;
    int64_t len;
    int32_t kind;
    uint8_t* out;
    int64_t n, ld;
    int64_t nnz = 0;
    double sum = 0.0;
    int err = 0;            // 1: index out of range, 2: a row repeats > 255 times
};

void build_mask(MaskJob& j) {
    uint8_t* m = j.out;
    const int64_t n = j.n;
    std::memset(m + n, 0, (size_t)(j.ld - n));
    if (j.kind == SGLM_MASK_ALL) {
        std::memset(m, 1, (size_t)n);
        j.nnz = n;
        j.sum = (double)n;
        return;
    }
    std::memset(m, 0, (size_t)n);
    const int64_t* idx = j.idx;
    const int64_t L = j.len;
    // numpy fancy-indexing semantics (X[idx_train], backend/sglm_cv.py:107-110): an index in
    // [-n, 0) names row idx + n
    auto row = [n](int64_t v) { return v < 0 ? v + n : v; };
    // one pass: every index in range, and whether the list is strictly increasing
    bool bad = false, increasing = true;
    int64_t prev = -1;
    for (int64_t t = 0; t < L; ++t) {
        const int64_t v = row(idx[t]);
        bad |= (uint64_t)v >= (uint64_t)n;
        increasing &= v > prev;
        prev = v;
    }
    if (bad) { j.err = 1; return; }
    if (j.kind == SGLM_MASK_ROWS || increasing) {
        for (int64_t t = 0; t < L; ++t) m[row(idx[t])] = 1;
        if (increasing) {
            j.nnz = L;
            j.sum = (double)L;
            return;
        }
        int64_t c = 0;
        for (int64_t i = 0; i < n; ++i) c += m[i];
        j.nnz = c;
        j.sum = (double)c;
        return;
    }
    // multiplicities (repeats)
    for (int64_t t = 0; t < L; ++t) {
        const int64_t r = row(idx[t]);
        if (m[r] == 255) { j.err = 2; return; }
        ++m[r];
    }
    int64_t c = 0;
    for (int64_t i = 0; i < n; ++i) c += m[i] != 0;
    j.nnz = c;
    j.sum = (double)L;
}

}  // namespace

using sglm::set_error;

extern "C" int sglm_host_masks(int32_t nm, const int64_t* const* idx, const int64_t* len,
                               const int32_t* kind, int64_t n, int64_t ld, uint8_t* out,
                               int64_t* nnz, double* sum, int32_t nthreads) {
    if (nm <= 0) return SGLM_OK;
    if (!idx || !len || !kind || !out || n < 0 || ld < n) {
        set_error("sglm_host_masks: bad args");
        return SGLM_EINVAL;
    }
    std::vector<MaskJob> jobs((size_t)nm);
    for (int32_t f = 0; f < nm; ++f) {
        if (kind[f] != SGLM_MASK_ALL && kind[f] != SGLM_MASK_FOLD && kind[f] != SGLM_MASK_ROWS) {
            set_error("sglm_host_masks: mask %d has unknown kind %d", f, kind[f]);
            return SGLM_EINVAL;
        }
        if (kind[f] != SGLM_MASK_ALL && len[f] > 0 && !idx[f]) {
            set_error("sglm_host_masks: mask %d has no index list", f);
            return SGLM_EINVAL;
        }
        MaskJob& j = jobs[(size_t)f];
        j.idx = idx[f];
        j.len = kind[f] == SGLM_MASK_ALL ? 0 : len[f];
        j.kind = kind[f];
        j.out = out + (int64_t)f * ld;
        j.n = n;
        j.ld = ld;
    }
    int nt = nthreads > 0 ? nthreads : 1;
    if (nt > nm) nt = nm;
    std::vector<std::thread> pool;
    pool.reserve((size_t)nt);
    for (int w = 0; w < nt; ++w)
        pool.emplace_back([&jobs, w, nt] {
            for (size_t f = (size_t)w; f < jobs.size(); f += (size_t)nt) build_mask(jobs[f]);
        });
    for (auto& t : pool) t.join();
    for (int32_t f = 0; f < nm; ++f) {
        const MaskJob& j = jobs[(size_t)f];
        if (j.err == 1) {
            set_error("sglm_host_masks: mask %d lists a row outside [-%lld, %lld)", f,
                      (long long)n, (long long)n);
            return SGLM_EINVAL;
        }
        if (j.err == 2) {
            set_error("an index repeats more than 255 times in one split");
            return SGLM_EINVAL;
        }
        if (nnz) nnz[f] = j.nnz;
        if (sum) sum[f] = j.sum;
    }
    return SGLM_OK;
}

// Threaded host copies for the chunked uploads (engine.Design.from_host, the lagged frames of
// sglm_pp.timeshift_multiple): a pageable numpy buffer is copied into a pinned staging buffer
// by `nthreads` threads so that the DMA engine reads page-locked memory at full PCIe rate
// (torch's pageable .to(device) is one staged, single-threaded copy).
// sglm_host_copy: dst[0 .. nbytes) = src[0 .. nbytes).
// sglm_host_gather_cols: dst[c * nrows * elem .. ) = column c (src[c], nrows elements of elem
//   bytes, stride[c] elements apart; stride NULL: contiguous) for c < ncols -- the event
//   columns of a DataFrame (a row-major block's columns are strided), column-major.
extern "C" int sglm_host_copy(void* dst, const void* src, int64_t nbytes, int32_t nthreads) {
    if (nbytes <= 0) return SGLM_OK;
    if (!dst || !src) { sglm::set_error("sglm_host_copy: null pointer"); return SGLM_EINVAL; }
    const int nt = nthreads > 1 ? (int)std::min<int64_t>(nthreads, (nbytes >> 22) + 1) : 1;
    const int64_t per = (nbytes + nt - 1) / nt;
    std::vector<std::thread> th;
    for (int t = 0; t < nt; ++t) {
        const int64_t a = (int64_t)t * per, b = std::min<int64_t>(nbytes, a + per);
        if (a >= b) break;
        th.emplace_back([=] {
            std::memcpy((char*)dst + a, (const char*)src + a, (size_t)(b - a));
        });
    }
    for (auto& x : th) x.join();
    return SGLM_OK;
}

extern "C" int sglm_host_gather_cols(const void* const* src, const int64_t* stride,
                                     int32_t ncols, int64_t nrows, int32_t elem, void* dst,
                                     int32_t nthreads) {
    if (ncols <= 0 || nrows <= 0) return SGLM_OK;
    if (!src || !dst || elem <= 0) { sglm::set_error("sglm_host_gather_cols: bad args"); return SGLM_EINVAL; }
    for (int c = 0; c < ncols; ++c)
        if (!src[c]) { sglm::set_error("sglm_host_gather_cols: null column %d", c); return SGLM_EINVAL; }
    // threads own row ranges; inside a range of 2048 rows every column is copied in turn, so
    // the columns of one row-major block (stride > 1) read the same cache lines back to back
    const int64_t chunk = 2048;
    const int64_t nchunks = (nrows + chunk - 1) / chunk;
    const int nt = (int)std::max<int64_t>(1, std::min<int64_t>(nthreads, nchunks));
    std::vector<std::thread> th;
    for (int t = 0; t < nt; ++t)
        th.emplace_back([=] {
            for (int64_t q = t; q < nchunks; q += nt) {
                const int64_t r0 = q * chunk, r1 = std::min(nrows, r0 + chunk);
                for (int c = 0; c < ncols; ++c) {
                    const int64_t st = stride ? stride[c] : 1;
                    char* out = (char*)dst + ((size_t)c * nrows + r0) * elem;
                    const char* in = (const char*)src[c] + (size_t)r0 * st * elem;
                    if (st == 1) {
                        std::memcpy(out, in, (size_t)(r1 - r0) * elem);
                    } else if (elem == 8) {
                        const uint64_t* a = (const uint64_t*)in;
                        uint64_t* b = (uint64_t*)out;
                        for (int64_t r = 0; r < r1 - r0; ++r) b[r] = a[r * st];
                    } else {
                        for (int64_t r = 0; r < r1 - r0; ++r)
                            std::memcpy(out + r * elem, in + r * st * elem, (size_t)elem);
                    }
                }
            }
        });
    for (auto& x : th) x.join();
    return SGLM_OK;
}

// sglm_host_pack_bits_cols: for each column (float64, src[c] with element stride stride[c]),
// bit r of bits[c * nwords + r / 32] = (value == 1.0), and binary[c] = 1 when every value is
// 0.0 or 1.0 (a NaN, -0.0 is 0.0, or any other value clears it) -- a 0/1 event column crosses
// PCIe as 1 bit per row instead of 8 bytes; ones[c] (when not NULL) = the column's count of
// 1.0 cells.  Threads own 2048-row ranges; nwords = ceil(nrows
// / 32).
extern "C" int sglm_host_pack_bits_cols(const void* const* src, const int64_t* stride,
                                        int32_t ncols, int64_t nrows, uint32_t* bits,
                                        uint8_t* binary, int64_t* ones, int32_t nthreads) {
    if (ncols <= 0 || nrows <= 0) return SGLM_OK;
    if (!src || !bits || !binary) { sglm::set_error("sglm_host_pack_bits_cols: bad args"); return SGLM_EINVAL; }
    const int64_t nwords = (nrows + 31) / 32;
    const int64_t chunk = 2048;
    const int64_t nchunks = (nrows + chunk - 1) / chunk;
    const int nt = (int)std::max<int64_t>(1, std::min<int64_t>(nthreads, nchunks));
    std::vector<std::vector<uint8_t>> bad(nt, std::vector<uint8_t>(ncols, 0));
    std::vector<std::vector<int64_t>> cnt(nt, std::vector<int64_t>(ncols, 0));
    std::vector<std::thread> th;
    // the columns of ONE row-major block (a DataFrame built from a C-order array: column c at
    // base + c, row stride S >= ncols) are read row by row, each row's run of ncols values
    // once and in address order, instead of one strided pass per column
    const int64_t S = stride ? stride[0] : 1;
    bool block = ncols > 1 && S >= ncols;
    for (int c = 1; block && c < ncols; ++c)
        block = stride[c] == S && (const double*)src[c] == (const double*)src[0] + c;
    if (block && ncols <= 256 && sglm_host_simd_level() > 0) {
        // AVX-512: 16 columns per vector op (host_simd.cpp)
        const double* base = (const double*)src[0];
        for (int t = 0; t < nt; ++t)
            th.emplace_back([=, &bad, &cnt] {
                for (int64_t q = t; q < nchunks; q += nt) {
                    const int64_t r0 = q * chunk, r1 = std::min(nrows, r0 + chunk);
                    sglm_host_pack_block_avx512(base, S, ncols, r0, r1, nwords, bits,
                                                bad[t].data(), cnt[t].data());
                }
            });
        for (auto& x : th) x.join();
        for (int c = 0; c < ncols; ++c) {
            uint8_t x = 0;
            int64_t o = 0;
            for (int t = 0; t < nt; ++t) {
                x |= bad[t][c];
                o += cnt[t][c];
            }
            binary[c] = !x;
            if (ones) ones[c] = o;
        }
        return SGLM_OK;
    }
    if (block) {
        const double* base = (const double*)src[0];
        for (int t = 0; t < nt; ++t)
            th.emplace_back([=, &bad, &cnt] {
                std::vector<uint32_t> word(ncols);
                std::vector<uint8_t> b(ncols, 0);
                uint8_t* bl = b.data();
                uint32_t* wd = word.data();
                for (int64_t q = t; q < nchunks; q += nt) {
                    const int64_t r0 = q * chunk, r1 = std::min(nrows, r0 + chunk);
                    for (int64_t w0 = r0; w0 < r1; w0 += 32) {
                        std::fill(word.begin(), word.end(), 0u);
                        const int64_t e = std::min<int64_t>(32, r1 - w0);
                        for (int64_t k = 0; k < e; ++k) {
                            const double* row = base + (w0 + k) * S;
                            for (int c = 0; c < ncols; ++c) {
                                const double v = row[c];
                                wd[c] |= (uint32_t)(v == 1.0) << k;
                                bl[c] |= (uint8_t)!(v == 0.0 || v == 1.0);
                            }
                        }
                        for (int c = 0; c < ncols; ++c) {
                            bits[(size_t)c * nwords + w0 / 32] = wd[c];
                            cnt[t][c] += __builtin_popcount(wd[c]);
                        }
                    }
                }
                for (int c = 0; c < ncols; ++c) bad[t][c] = bl[c];
            });
        for (auto& x : th) x.join();
        for (int c = 0; c < ncols; ++c) {
            uint8_t x = 0;
            int64_t o = 0;
            for (int t = 0; t < nt; ++t) {
                x |= bad[t][c];
                o += cnt[t][c];
            }
            binary[c] = !x;
            if (ones) ones[c] = o;
        }
        return SGLM_OK;
    }
    for (int t = 0; t < nt; ++t)
        th.emplace_back([=, &bad, &cnt] {
            for (int64_t q = t; q < nchunks; q += nt) {
                const int64_t r0 = q * chunk, r1 = std::min(nrows, r0 + chunk);
                for (int c = 0; c < ncols; ++c) {
                    const int64_t st = stride ? stride[c] : 1;
                    const double* in = (const double*)src[c];
                    uint32_t* out = bits + (size_t)c * nwords;
                    uint8_t b = 0;
                    for (int64_t w0 = r0; w0 < r1; w0 += 32) {
                        uint32_t word = 0;
                        const int64_t e = std::min<int64_t>(32, r1 - w0);
                        for (int64_t k = 0; k < e; ++k) {
                            const double v = in[(w0 + k) * st];
                            word |= (uint32_t)(v == 1.0) << k;
                            b |= (uint8_t)!(v == 0.0 || v == 1.0);
                        }
                        out[w0 / 32] = word;
                        cnt[t][c] += __builtin_popcount(word);
                    }
                    bad[t][c] |= b;
                }
            }
        });
    for (auto& x : th) x.join();
    for (int c = 0; c < ncols; ++c) {
        uint8_t b = 0;
        int64_t o = 0;
        for (int t = 0; t < nt; ++t) {
            b |= bad[t][c];
            o += cnt[t][c];
        }
        binary[c] = !b;
        if (ones) ones[c] = o;
    }
    return SGLM_OK;
}

extern "C" int sglm_host_group_rows(const int64_t* gidx, int64_t n, const uint8_t* side,
                                    int32_t nsplits, int64_t G, int64_t* const* out,
                                    const int64_t* len, int32_t nthreads) {
    if (nsplits <= 0 || n <= 0) return SGLM_OK;
    if (!gidx || !side || !out || !len || G <= 0) {
        sglm::set_error("sglm_host_group_rows: bad args");
        return SGLM_EINVAL;
    }
    // threads own row ranges: pass 1 counts each range's rows per list (and checks the group
    // index), the offsets are a prefix over the ranges, pass 2 writes every list's rows of the
    // range in ascending order
    const int nj = 2 * nsplits;
    const int nt = (int)std::max<int64_t>(1, std::min<int64_t>(nthreads, (n + 65535) / 65536));
    std::vector<int64_t> cnt((size_t)nt * nj, 0);
    std::vector<int> bad(nt, 0);
    auto range = [n, nt](int t, int64_t& a, int64_t& b) {
        a = n * t / nt;
        b = n * (t + 1) / nt;
    };
    std::vector<std::thread> th;
    for (int t = 0; t < nt; ++t)
        th.emplace_back([=, &cnt, &bad] {
            int64_t a, b;
            range(t, a, b);
            int64_t* c = cnt.data() + (size_t)t * nj;
            for (int64_t i = a; i < b; ++i)
                if ((uint64_t)gidx[i] >= (uint64_t)G) { bad[t] = 1; return; }
            for (int k = 0; k < nsplits; ++k) {
                const uint8_t* sd = side + (int64_t)k * G;
                int64_t c1 = 0, c2 = 0;
                for (int64_t i = a; i < b; ++i) {
                    const uint8_t v = sd[gidx[i]];
                    c1 += v == 1;
                    c2 += v == 2;
                }
                c[2 * k] = c1;
                c[2 * k + 1] = c2;
            }
        });
    for (auto& x : th) x.join();
    th.clear();
    for (int t = 0; t < nt; ++t)
        if (bad[t]) {
            sglm::set_error("sglm_host_group_rows: group index outside [0, %lld)", (long long)G);
            return SGLM_EINVAL;
        }
    std::vector<int64_t> off((size_t)nt * nj);
    for (int j = 0; j < nj; ++j) {
        int64_t o = 0;
        for (int t = 0; t < nt; ++t) {
            off[(size_t)t * nj + j] = o;
            o += cnt[(size_t)t * nj + j];
        }
        if (o != len[j]) {
            sglm::set_error("sglm_host_group_rows: list %d has %lld rows, len %lld", j,
                            (long long)o, (long long)len[j]);
            return SGLM_EINVAL;
        }
        if (o && !out[j]) { sglm::set_error("sglm_host_group_rows: null list %d", j); return SGLM_EINVAL; }
    }
    for (int t = 0; t < nt; ++t)
        th.emplace_back([=, &off] {
            int64_t a, b;
            range(t, a, b);
            for (int k = 0; k < nsplits; ++k) {
                const uint8_t* sd = side + (int64_t)k * G;
                int64_t* o1 = out[2 * k] + off[(size_t)t * nj + 2 * k];
                int64_t* o2 = out[2 * k + 1] + off[(size_t)t * nj + 2 * k + 1];
                for (int64_t i = a; i < b; ++i) {
                    const uint8_t v = sd[gidx[i]];
                    if (v == 1) *o1++ = i;
                    else if (v == 2) *o2++ = i;
                }
            }
        });
    for (auto& x : th) x.join();
    return SGLM_OK;
}

// sglm_host_group_runs: sglm_host_group_rows for groups laid out as runs of consecutive rows
// (a non-decreasing trial id): run r covers rows start[r] .. start[r] + rlen[r] - 1 and belongs to
// group grp[r]; list 2k (2k + 1) = the rows of the runs whose group has side[k][g] == 1 (2), in
// ascending order.  One thread per list; no per-row group index is read or built.
extern "C" int sglm_host_group_runs(const int64_t* start, const int64_t* rlen, const int64_t* grp,
                                    int64_t nruns, const uint8_t* side, int32_t nsplits,
                                    int64_t G, int64_t* const* out, const int64_t* len,
                                    int32_t nthreads) {
    if (nsplits <= 0 || nruns <= 0) return SGLM_OK;
    if (!start || !rlen || !grp || !side || !out || !len || G <= 0) {
        sglm::set_error("sglm_host_group_runs: bad args");
        return SGLM_EINVAL;
    }
    for (int64_t r = 0; r < nruns; ++r)
        if ((uint64_t)grp[r] >= (uint64_t)G || rlen[r] < 0 ||
            (r > 0 && start[r] < start[r - 1] + rlen[r - 1])) {
            sglm::set_error("sglm_host_group_runs: run %lld invalid (group %lld of %lld)",
                            (long long)r, (long long)grp[r], (long long)G);
            return SGLM_EINVAL;
        }
    const int nj = 2 * nsplits;
    std::vector<int> bad(nj, 0);
    std::vector<std::thread> th;
    const int nt = std::max(1, std::min<int>(nthreads, nj));
    for (int t = 0; t < nt; ++t)
        th.emplace_back([=, &bad] {
            for (int j = t; j < nj; j += nt) {
                const uint8_t* sd = side + (int64_t)(j / 2) * G;
                const uint8_t want = (uint8_t)(1 + (j & 1));
                int64_t* o = out[j];
                int64_t w = 0;
                for (int64_t r = 0; r < nruns; ++r) {
                    if (sd[grp[r]] != want) continue;
                    if (w + rlen[r] > len[j]) { bad[j] = 1; break; }
                    for (int64_t i = 0; i < rlen[r]; ++i) o[w + i] = start[r] + i;
                    w += rlen[r];
                }
                if (w != len[j]) bad[j] = 1;
            }
        });
    for (auto& x : th) x.join();
    for (int j = 0; j < nj; ++j)
        if (bad[j]) {
            sglm::set_error("sglm_host_group_runs: list %d length mismatch", j);
            return SGLM_EINVAL;
        }
    return SGLM_OK;
}
