/*
 * sglm_hip.h — C ABI of libsglm_hip.so, the MI355X (gfx950) engine behind the sglm hot path.
 *
 * The reference (kimerein/sabatinilab-glm) is pure Python: its "FFI" for this path is the
 * scikit-learn estimator protocol that GLM.__init__ instantiates (backend/sglm.py:128-130)
 * and calls (fit backend/sglm.py:241, predict :347, score :184), plus numpy for the
 * timeshift (backend/sglm_pp.py:298-357) and the CV fold copies (backend/sglm_cv.py:106-110).
 * Each entry point below names the reference interface whose arithmetic it replaces.
 * The Python host layer (sabatinilab-glm_amd/sglm_hip/_lib.py) binds these with ctypes.
 *
 * Conventions
 *  - Every pointer is a DEVICE pointer owned by the caller (PyTorch-ROCm tensors), except
 *    where a parameter says "host".
 *  - Every call is asynchronous on `stream` (a hipStream_t; 0 = legacy default stream) and
 *    performs no allocation and no host synchronisation; scratch is the caller's `work`
 *    buffer, sized by the matching *_work_bytes() query.
 *  - Return value: SGLM_OK (0) or an error code; sglm_last_error() gives a thread-local
 *    message.  Launch-time HIP errors are reported as SGLM_EHIP.
 *
 * Data layout in HBM
 *  - Design X: FEATURE-MAJOR ("column-major") X[a * ld + i], a in [0, P), i in [0, ld):
 *    one contiguous row stream per predictor, the ones column (intercept) at a = p, zero
 *    columns up to P (multiple of 256), zero rows up to ld (multiple of 256).
 *    Stored bf16 (exact for 0/1 event designs) and, when X is not bf16-exact, also f32.
 *  - Per-fit vectors are fit-major: eta/W/R[k * ld + i]; coefficients beta[k * P + a].
 *  - Responses Y[r * ld + i] (f32); row masks M[f * ld + i] (uint8 multiplicities).
 */
#ifndef SGLM_HIP_H
#define SGLM_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void* sglm_stream_t; /* hipStream_t */

enum sglm_status { SGLM_OK = 0, SGLM_EINVAL = 1, SGLM_EHIP = 2, SGLM_ENOTPD = 3 };

/* Loss family codes: half-Tweedie losses of sklearn/_loss/loss.py.
 *  SGLM_FAM_SQUARED   : 0.5 (eta - y)^2, identity link (LinearRegression / Ridge /
 *                       TweedieRegressor(power=0) objectives; backend/sglm.py:96-105,116).
 *  SGLM_FAM_TWEEDIE_LOG: HalfTweedieLoss(power) with log link, power in [1, 2] covers
 *                       Poisson (1) and Gamma (2) (backend/sglm.py:112-115). */
enum sglm_family { SGLM_FAM_SQUARED = 0, SGLM_FAM_TWEEDIE_LOG = 1 };

enum sglm_xtype { SGLM_X_BF16 = 0, SGLM_X_F32 = 1 };

const char* sglm_last_error(void);
int sglm_version(void);

/* --- design-matrix construction --------------------------------------------------------
 * Generic strided timeshift/gather: out(t, j) = src(t + row0 - shift[j], src_col[j]) when
 * that source row lies in [0, n_src), else the bit pattern `fill_bits`.  Element (r, c) of
 * src is at src + (r * rs_src + c * cs_src) * elem_size; likewise for out.  elem_size in
 * {1, 2, 4, 8} (int8 .. float64; NaN fill = its bit pattern).  src_col/shift are device
 * int32 arrays of length ncols_out.
 * Replaces: sglm_pp.shift / timeshift / timeshift_multiple (backend/sglm_pp.py:23-103,
 * 298-486), sglm_ez.timeshift_cols (backend/sglm_ez.py:102-123) and
 * setup_model_fit.timeshift_vals_by_dict (sglm/sglm/features/setup_model_fit.py:43-96). */
int sglm_timeshift_expand(const void* src, int64_t n_src, int64_t rs_src, int64_t cs_src,
                          const int32_t* src_col, const int32_t* shift, int32_t ncols_out,
                          void* out, int64_t n_out, int64_t rs_out, int64_t cs_out,
                          int64_t row0, int32_t elem_size, uint64_t fill_bits,
                          sglm_stream_t stream);

/* sglm_timeshift_expand with a row list: out(t, j) = src(rows[t] - shift[j], src_col[j]) when
 * that source row lies in [0, n_src), else fill_bits (rows: device int64 [n_out]) -- the rows
 * a lagged DataFrame keeps after its NaN / holdout filters (sglm_hip.lagframe), expanded
 * without the intermediate frame the reference materialises (backend/sglm_pp.py:58-103). */
int sglm_timeshift_gather(const void* src, int64_t n_src, int64_t rs_src, int64_t cs_src,
                          const int32_t* src_col, const int32_t* shift, int32_t ncols_out,
                          void* out, int64_t n_out, int64_t rs_out, int64_t cs_out,
                          const int64_t* rows, int32_t elem_size, uint64_t fill_bits,
                          sglm_stream_t stream);

/* Pack a row-major (n x p) f32/f64 design (strides in elements) into the feature-major
 * layout: Xb (bf16, required), Xf (f32, optional/nullable), ones column at a = p when
 * add_ones, zero padding to (P, ld).  *inexact (device int32, caller-zeroed) is set to 1
 * if any value is not exactly representable in bf16.
 * Replaces: the float64 validation copy sklearn makes inside every fit (glm.py:191-198,
 * X[idx_train,:] copies at backend/sglm_cv.py:107-110). */
int sglm_pack_design(const void* src, int32_t src_is_f64, int64_t n, int32_t p,
                     int64_t rs, int64_t cs, int32_t add_ones, uint16_t* Xb, float* Xf,
                     int64_t ld, int32_t P, int32_t* inexact, sglm_stream_t stream);

/* sglm_pack_design for one chunk of a chunked upload: source rows 0 .. n go to design rows
 * dst0 .. dst0 + n (dst0 a multiple of 64); only the 64-row tiles of the chunk are written
 * (rows past the chunk inside its last tile as zero: chunks go in ascending order). */
int sglm_pack_design_rows(const void* src, int32_t src_is_f64, int64_t n, int32_t p, int64_t rs,
                          int64_t cs, int32_t add_ones, uint16_t* Xb, float* Xf, int64_t ld,
                          int32_t P, int64_t dst0, int32_t* inexact, sglm_stream_t stream);

/* --- IRLS inner step (one batched Newton iteration over B fits) -------------------------
 * Replaces the per-fit solver iterations inside self.model.fit (backend/sglm.py:241):
 * TweedieRegressor lbfgs/newton (sklearn glm.py:266-306), Ridge cholesky (_ridge.py:201),
 * LinearRegression lstsq (_base.py:701). */

/* eta[k][i] = sum_a X[a][i] * beta[k][a]  for k < B, i < n (f32; also used for d_eta). */
/* sglm_pack_design_rows that also sets colflag[a] = 1 (device int32 [p], accumulated over
 * calls) for every source column a holding a value other than 0 or 1 (NaN included), judged on
 * the source values before rounding: the split of a mixed 0/1 + continuous design. */
int sglm_pack_design_rows_cf(const void* src, int32_t src_is_f64, int64_t n, int32_t p,
                             int64_t rs, int64_t cs, int32_t add_ones, uint16_t* Xb, float* Xf,
                             int64_t ld, int32_t P, int64_t dst0, int32_t* inexact,
                             int32_t* colflag, sglm_stream_t stream);

int sglm_gemv_eta(const void* X, int32_t xtype, int64_t ld, int32_t P, int64_t n,
                  const float* beta, int32_t B, float* eta, sglm_stream_t stream);

/* Link/variance update over B fits: launch row q is fit slot k = slots[q] (q when slots is
 * NULL).  With response r = fit_resp[k], mask m = fit_mask[k]:
 *   W[k][i] = M[m][i] * d2loss/deta2,   R[k][i] = M[m][i] * dloss/deta,   rows i < n.
 * Rows n <= i < ld are written as 0.  R (f32 per slot) and Rp may each be NULL (not both):
 * Rp receives R as three bf16 pieces hi + mid + lo == R, bf16 [3][Bp][ld] with
 * Bp = ceil(B/32)*32, row q = launch row -- the operand of sglm_xtr_bits_packed.
 * deta (optional, with step[q]): first eta[k] += step[q] * deta[k] (the previous Newton
 * step's predictor update, fused), then the link on the updated eta. */
int sglm_link_update(int32_t family, float power, int64_t n, int64_t ld, int32_t B,
                     const int32_t* slots, float* eta, const float* Y, const uint8_t* M,
                     const int32_t* fit_resp, const int32_t* fit_mask, float* W, float* R,
                     void* Rp, const float* step, const float* deta, sglm_stream_t stream);
/* sglm_link_update_rp: sglm_link_update (slots required) writing launch row y's packed R into
 * row rpos[y] of planes of Bp rows (rpos[y] < 0: no packed row; W, R and the fused predictor
 * update as usual) -- the rows of the fits that continue, compacted by sglm_step_decide. */
int sglm_link_update_rp(int32_t family, float power, int64_t n, int64_t ld, int32_t B,
                        const int32_t* slots, float* eta, const float* Y, const uint8_t* M,
                        const int32_t* fit_resp, const int32_t* fit_mask, float* W, float* R,
                        void* Rp, int32_t Bp, const int32_t* rpos, const float* step,
                        const float* deta, sglm_stream_t stream);

/* G[k][a] = sum_i X[a][i] * R[k][i] (float64 out; f32 MFMA partial sums, fixed-order
 * float64 reduction over row chunks).  `work`: sglm_xtr_work_bytes(P, B, n). */
size_t sglm_xtr_work_bytes(int32_t P, int32_t B, int64_t n);
int sglm_xtr(const void* X, int32_t xtype, int64_t ld, int32_t P, int64_t n,
             const float* R, int32_t B, double* G, void* work, sglm_stream_t stream);

/* Batched weighted Gram, the X^T W X contraction, bf16 MFMA (v_mfma_f32_32x32x16_bf16),
 * f32 accumulate:  H[k][a][b] = sum_i X[a][i] W[k][i] X[b][i] for every fit k in
 * fits[0..nact) and every (a, b) whose 256-tiles satisfy tile(a) <= tile(b) (upper
 * triangle incl. diagonal tiles).  `splits` > 1 splits the rows over workgroups and
 * reduces slabs in `work` (sglm_syrk_work_bytes) in fixed order. */
size_t sglm_syrk_work_bytes(int32_t P, int32_t nact, int32_t splits);
int sglm_syrk(const uint16_t* Xb, int64_t ld, int32_t P, int64_t n, const float* W,
              const int32_t* fits, int32_t nact, int32_t splits, float* H, void* work,
              sglm_stream_t stream);

/* As sglm_syrk, but fit k only visits the 8-row groups row_groups[group_offset[k] ..
 * + group_count[k]) (ascending group indices, group g = rows 8g..8g+7): groups holding no
 * row of the fit's mask are skipped.  Indexed by fit id (like W).  Requires ld > n (a zero
 * padding row).  This is the fold-copy-free replacement of X[idx_train, :]. */
int sglm_syrk_masked(const uint16_t* Xb, int64_t ld, int32_t P, int64_t n, const float* W,
                     const int32_t* fits, int32_t nact, int32_t splits, float* H, void* work,
                     const int32_t* row_groups, const int64_t* group_offset,
                     const int32_t* group_count, sglm_stream_t stream);

/* Bit-plane form of a 0/1 design: bits[a * (ld/32) + q] bit b = (X[a][32q + b] != 0).
 * *nonbinary (device int32, caller-zeroed) is set if any value is not exactly 0 or 1. */
int sglm_pack_bits(const uint16_t* Xb, int64_t ld, int32_t P, uint32_t* bits,
                   int32_t* nonbinary, sglm_stream_t stream);

/* Row-compacted bit-plane design (Gram v6).  Output row k is X[.][rows[k]] (rows == NULL:
 * row k) for k < nrows, zero up to the next multiple of 64.  Layout K-step-major:
 * out[(blk * P + a) * 2 + {0,1}] = the two 32-row words of 64-row block blk of predictor a;
 * inside a word, row rho is bit 4*(rho/8) + (rho%8)/2 + 16*(rho%2) (MFMA fragment order).
 * Size: ceil(nrows/64) * P * 8 bytes.  *nonbinary as for sglm_pack_bits.
 * Replaces the X[idx_train, :] copies of backend/sglm_cv.py:107-110 for 0/1 designs. */
int sglm_pack_bits_rows(const uint16_t* Xb, int64_t ld, int32_t P, const int32_t* rows,
                        int64_t nrows, uint32_t* out, int32_t* nonbinary, sglm_stream_t stream);

/* sglm_pack_bits_rows from the column-packed planes of sglm_pack_bits (same output; reads
 * 1 bit per element instead of the bf16 design). */
int sglm_compact_bits(const uint32_t* xbits, int64_t ld, int32_t P, const int32_t* rows,
                      int64_t nrows, uint32_t* out, sglm_stream_t stream);
/* sglm_compact_bits from the row-major planes of sglm_pack_bits_t (rbits, [P/64][ld] x 8 B):
 * identical output, one 64 x 64 bit-tile transpose (64 wave ballots) per wave. */
int sglm_compact_rbits(const uint32_t* rbits, int64_t ld, int32_t P, const int32_t* rows,
                       int64_t nrows, uint32_t* out, sglm_stream_t stream);

/* Per-slot descriptor for Gram v6, 4 x int64 per slot: [0] device address of the slot's
 * compacted bit-plane design, [1] its row count, [2] device address of the slot's compact
 * bf16 weights (>= ceil(rows/64)*64 entries), [3] device address of its int32 row list
 * (0 = identity).  sglm_gather_w fills [2]: bf16(W[fits[s]][row(k)]), zero padded. */
int sglm_gather_w(const float* W, int64_t ld, const int32_t* fits, int32_t nact,
                  const int64_t* desc, int64_t max_rows, sglm_stream_t stream);

/* Gram v6: H[fits[s]] = X_s^T diag(w_s) X_s over each slot's compacted rows, bf16 MFMA from
 * bit-planes expanded in registers; writes the 128-blocks with block row <= block col.
 * work: sglm_syrk_work_bytes(P, nact, splits) when splits > 1. */
int sglm_syrk_cbits(const int64_t* desc, int32_t P, const int32_t* fits, int32_t nact,
                    int32_t splits, float* H, void* work, sglm_stream_t stream);

/* Weighted Gram of a time-shifted 0/1 event design from its events (lagw.hip): for each
 * fits[f], H[fits[f]] = X^T diag(bf16(W[fits[f]])) X with X[t][col(b, a)] =
 * e_a(t + row0 - shifts[b]) and the ones column pones (K m, or past a mixed design's continuous
 * columns K m .. pones - 1, whose rows / columns are zeroed here and left to sglm_mixed_to_h),
 * written on the upper triangle (row <= col; the padding columns > pones zeroed; the lower
 * triangle is scratch: the kernel writes each entry at the row of its column with the larger
 * shift and a symmetrize pass builds the upper triangle).  col(b, a) = layout ? a K + b : b m + a.
 * R: sglm_lag_rowwords of the events; occ / ev_off: every event's occurrence rows, event-major,
 * ascending, and the event segments (m + 1); shifts[b] = the shift of block b, which must be
 * exactly the values smin .. smax (K = smax - smin + 1 distinct shifts, in any order), and
 * bidx[s - smin] = b of shift s -- its inverse permutation (the caller builds both; an entry
 * < 0 of bidx is skipped, never written through).
 * Replaces the dense Gram's n p^2 products by about nnz(E) (m + 1) K^2 per fit (each event's
 * occurrences x every event at the shift differences d >= 0 x the shifts). */
int sglm_lag_gram_w(const uint64_t* R, const int32_t* occ, const int32_t* ev_off, int32_t m,
                    int32_t nraw, const int32_t* shifts, const int32_t* bidx, int32_t K,
                    int32_t smin, int32_t smax, int32_t layout, int32_t row0, int32_t n,
                    const float* W, int64_t ld, const int32_t* fits, int32_t nf, float* H,
                    int32_t P, int32_t pones, void* work, sglm_stream_t stream);
/* work bytes of sglm_lag_gram_w: 8 shifted bf16 copies of the launch's weights over every raw
 * row (~16 B per raw row per fit -- the engine splits large launches to bound it) and a P x P
 * f32 image per fit for the second halves of the pieces a launch splits (load balance) */
size_t sglm_lag_gram_w_work_bytes(int32_t nraw, int32_t K, int32_t nf, int32_t P);
/* Measurement hook (no reference counterpart): mode 1 clears and starts bracketing every
 * structured-Gram kernel launch with HIP events on its stream, mode 2 waits for the recorded
 * launches and returns their summed kernel time (ms) and count, then clears, mode 0 stops. */
int sglm_lag_gram_w_timing(int32_t mode, double* ms, int32_t* n);

/* Row words of m <= 63 events: R[u] bit a = e_a(u) (ebits[m][nwords], bit u & 31 of word
 * u >> 5), bit m = 1, for u < nraw. */
int sglm_lag_rowwords(const int32_t* ebits, int32_t m, int32_t nwords, int32_t nraw,
                      uint64_t* R, sglm_stream_t stream);

/* Row-major bit-planes of a 0/1 design for the MFMA GEMVs: out[(t * ld + i) * 2 + {0,1}] =
 * the bits of X[64t + alpha][i], alpha = 0..63, fragment order (see sglm_pack_bits_rows).
 * Size (P/64) * ld * 8 bytes.  *nonbinary as for sglm_pack_bits. */
int sglm_pack_bits_t(const uint16_t* Xb, int64_t ld, int32_t P, uint32_t* out,
                     int32_t* nonbinary, sglm_stream_t stream);

/* eta[k] = X beta[k] (as sglm_gemv_eta) for a 0/1 design given as sglm_pack_bits_t planes,
 * bf16 MFMA with f32 accumulation, for the B slots k = slots[q] (q < B; all k < B when slots
 * is NULL).  exact = 1: beta split into three bf16 pieces (exact products).  exact = 0 (a
 * Newton direction): beta[k] is rounded to bf16 IN PLACE and X times the rounded vector is
 * computed (one piece, a third of the MFMA work) -- the caller steps with the rounded
 * direction, so the predictor stays X beta.  Writes all ld rows of eta (padding rows: 0).
 * work: sglm_eta_bits_work_bytes(P, B) bytes.
 * Replaces X @ coef (backend/sglm.py:347 -> sklearn glm.py:350). */
size_t sglm_eta_bits_work_bytes(int32_t P, int32_t B);
int sglm_gemv_eta_bits(const uint32_t* rbits, int64_t ld, int32_t P, float* beta, int32_t B,
                       const int32_t* slots, int32_t exact, float* eta, void* work,
                       sglm_stream_t stream);

/* g[k] = X^T R[k] (as sglm_xtr, float64 out) for a 0/1 design given as its identity-row
 * compacted planes (sglm_compact_bits with rows = NULL, nrows = n): R split into three bf16
 * pieces (exact products), bf16 MFMA, f32 slabs reduced in float64 in a fixed order.
 * work: sglm_xtr_bits_work_bytes(P, B, ld). */
size_t sglm_xtr_bits_work_bytes(int32_t P, int32_t B, int64_t ld);
int sglm_xtr_bits(const uint32_t* cbits, int64_t ld, int32_t P, int64_t n, const float* R,
                  int32_t B, double* G, void* work, sglm_stream_t stream);

/* sglm_xtr_bits with R already split into the packed bf16 pieces that sglm_link_update writes
 * (Rp: [3][Bp][ld]): G[slots[q]] = X^T R_q for q < B (G[q] when slots is NULL).
 * work: sglm_xtr_bits_packed_work_bytes(P, Bmax, ld), valid for every call with B <= Bmax. */
size_t sglm_xtr_bits_packed_work_bytes(int32_t P, int32_t B, int64_t ld);
int sglm_xtr_bits_packed(const uint32_t* cbits, int64_t ld, int32_t P, int64_t n,
                         const void* Rp, int32_t B, const int32_t* slots, double* G,
                         void* work, sglm_stream_t stream);
/* sglm_xtr_bits_packed_bp: the same with the packed planes' row stride Bp given (>= the padded
 * fit count): the R rows sglm_link_update_rp wrote at compacted positions of a longer launch. */
int sglm_xtr_bits_packed_bp(const uint32_t* cbits, int64_t ld, int32_t P, int64_t n,
                            const void* Rp, int32_t B, int32_t Bp, const int32_t* slots,
                            double* G, void* work, sglm_stream_t stream);

/* G[q] = X^T D_q (float64) for integer-valued columns, |D| <= 256 (the base-256 digit planes
 * of an exact X^T y): D as bf16 [Bp][ld] (Bp = ceil(B/32)*32 rows allocated), one bf16 piece,
 * row slabs of <= 65,536 rows -- the sums are exact.  P % 512 == 0, ld < 2^26.
 * work: sglm_xtr_bits_int_work_bytes(P, B, ld). */
/* The operand of sglm_xtr_bits_int for an exact X^T (m y): pair i = (response pr[i] of Y
 * [R][ldy] float64, mask pm[i] of M [F][ldm] uint8); v = rint(m y scale[i]) split into nd
 * balanced base-256 digits, digit q of pair i -> D[q c + i][row] (bf16), rows < n only. */
int sglm_digit_planes(const uint8_t* M, int64_t ldm, const double* Y, int64_t ldy, int64_t n,
                      const int32_t* pr, const int32_t* pm, const double* scale, int32_t c,
                      int32_t nd, void* D, int64_t ld, sglm_stream_t stream);
size_t sglm_xtr_bits_int_work_bytes(int32_t P, int32_t B, int64_t ld);
int sglm_xtr_bits_int(const uint32_t* cbits, int64_t ld, int32_t P, int64_t n, const void* D,
                      int32_t B, double* G, void* work, sglm_stream_t stream);

/* Bit-planes of a time-shifted 0/1 event design straight from its events (no dense bf16 design):
 * sglm_event_bits: ebits[a][w] bit i = (E[32 w + i][a] != 0), E as bf16 [m][lde] event-major,
 * nwords = ceil(n_raw / 32).  sglm_lag_bits: the design's column planes xbits [P][ld/32]
 * (column j < p = event cols[j] shifted by shifts[j]: X[t, j] = E[t + row0 - shifts[j]][cols[j]],
 * zero outside the raw rows; column p = ones on rows < n; padding zero) and the row-major MFMA
 * planes rbits [P/64][ld] x uint2 -- what sglm_pack_bits / sglm_pack_bits_t produce from the dense
 * design.  Replaces the expansion + packing of sglm_ez.timeshift_cols' design
 * (backend/sglm_ez.py:102-123) for 0/1 events. */
int sglm_event_bits(const uint16_t* Eb, int64_t lde, int32_t m, int64_t n_raw, uint32_t* ebits,
                    int64_t nwords, sglm_stream_t stream);
int sglm_lag_bits(const uint32_t* ebits, int64_t nwords, const int32_t* cols, const int32_t* shifts,
                  int32_t p, int64_t row0, int64_t n, int64_t ld, int32_t P, uint32_t* xbits,
                  void* rbits, sglm_stream_t stream);

/* Shared-Gram elastic net for many fits per mask (multi-response lambda paths):
 * sglm_center_gram: Q[m] (float64 p x p) = G_xx - g g^T / n (center) or G_xx from the
 *   augmented Gram H[gram_of[m]] (ones column at index p, as sglm_syrk forms it with W = mask);
 * sglm_enet_cd_shared: per fit f, minimise 1/2 w^T Q w - q^T w + l1|w|_1 + l2/2|w|^2 with
 *   Q = Q[qidx[f]], q = q[f] (float64, p), cyclic CD to max|dw| <= tol max|w| -> w[f].
 * Replaces sklearn ElasticNet/Lasso (cd_fast) per response and lambda, backend/sglm.py:106-110. */
int sglm_center_gram(const float* H, int32_t P, int32_t p, const int32_t* gram_of, int32_t nmask,
                     int32_t center, double* Q, sglm_stream_t stream);
int sglm_enet_cd_shared(const double* Q, int32_t p, const int32_t* qidx, int32_t nfit,
                        const double* q, const double* l1, const double* l2, int32_t max_sweeps,
                        double tol, double* w, int32_t* sweeps, sglm_stream_t stream);

/* sglm_enet_cd_shared with several fits of one Q per workgroup: workgroup g solves fits
 * wg_fits[g*fpw .. g*fpw+fpw) (-1 = empty slot), all on Q[wg_q[g]]; row j of Q is read once
 * per coordinate step for all of them.  fpw must equal sglm_enet_cd_fits_per_wg(p) (>= 2;
 * (2 fpw + 1) x p doubles of LDS).  Same outputs as sglm_enet_cd_shared (w [fit][p], sweeps). */
int32_t sglm_enet_cd_fits_per_wg(int32_t p);
int sglm_enet_cd_grouped(const double* Q, int32_t p, const int32_t* wg_fits, int32_t nwg,
                         int32_t fpw, const int32_t* wg_q, const double* q, const double* l1,
                         const double* l2, int32_t max_sweeps, double tol, double* w,
                         int32_t* sweeps, sglm_stream_t stream);

/* sglm_gram_ss: residual sums of squares of shared-Gram fits by Gram algebra (the C5 fold
 * scores, backend/sglm.py:150-184 neg_mse / R^2 over a mask, without forming X beta):
 * ss[q] = max(yy[q] - 2 beta_f . c[cidx[q]] + beta_f^T G beta_f, 0) for f = fits[q], with
 * beta [*][P] float64 (augmented: intercept at p, pa = p + 1 coordinates used), G the f32 upper
 * triangle H[grp_slot[g]] (P x P) of the group g holding q (fits sorted by group: group g is
 * q in [grp_off[g], grp_off[g+1]), at most max_per_grp), c [*][P] float64 = X~^T (m y), yy =
 * sum m y^2.  Float64 arithmetic; work: sglm_gram_ss_work_bytes(pa, nfit). */
size_t sglm_gram_ss_work_bytes(int32_t pa, int32_t nfit);
int sglm_gram_ss(const float* H, int32_t P, int32_t pa, const int32_t* grp_slot,
                 const int32_t* grp_off, int32_t ngrp, int32_t max_per_grp, const int32_t* fits,
                 int32_t nfit, const double* beta, const double* c, const int32_t* cidx,
                 const double* yy, double* ss, void* work, sglm_stream_t stream);

/* Same contraction from the f32 design (v_mfma_f32_32x32x2_f32, exact f32 products) for
 * designs that are not bf16-exact, where the Gram itself must be accurate (coordinate
 * descent, Gaussian closed forms).  128-tiles; work sized by sglm_syrk_work_bytes. */
int sglm_syrk_f32(const float* Xf, int64_t ld, int32_t P, int64_t n, const float* W,
                  const int32_t* fits, int32_t nact, int32_t splits, float* H, void* work,
                  sglm_stream_t stream);

/* Penalised Newton solve per fit k in fits[]:  (H_k + diag(dshift_k)) delta_k = -g_k.
 * H_k upper triangle (as written by sglm_syrk) is overwritten by its Cholesky factor.
 * dshift[k][a] >= 0 adds to the diagonal (ridge penalty; 0 for the intercept); a negative
 * entry freezes coordinate a (delta = 0: padding, fit_intercept=False).  Coordinates with
 * a zero diagonal or a pivot collapsing below 1e-6 of its diagonal are frozen too and
 * counted in info[k]; frozen[k][a] records the frozen set.  refactor = 0 skips the
 * factorisation and reuses the factor (and frozen set) a previous call left in H — the
 * constant-Hessian (Gaussian) refinement path.  P must be a multiple of 64, <= 8192.
 * B = rows of g/dshift/delta/frozen; `work`: sglm_chol_work_bytes(P, B).  Multi-workgroup
 * blocked factorisation (diag / panel / trailing-update launches per 64-column block). */
size_t sglm_chol_work_bytes(int32_t P, int32_t B);
int sglm_chol_solve_ex(float* H, int32_t P, const int32_t* fits, int32_t nact,
                       const double* g, const float* dshift, float* delta, int32_t* info,
                       uint8_t* frozen, int32_t refactor, int32_t B, void* work,
                       sglm_stream_t stream);

/* sglm_chol_solve_ex over a mixed set: fits[0 .. nrefac) are factored, fits[nrefac .. nact)
 * reuse the factor a previous call left in H (engine.irls: fits whose Hessian is kept), in one
 * launch chain (trailing updates over the refactored fits only). */
int sglm_chol_solve_mixed(float* H, int32_t P, const int32_t* fits, int32_t nact,
                          int32_t nrefac, const double* g, const float* dshift, float* delta,
                          int32_t* info, uint8_t* frozen, int32_t B, void* work,
                          sglm_stream_t stream);
/* sglm_chol_solve_inv: factor fits[0 .. nrefac) as sglm_chol_solve_mixed does and form their
 * explicit inverses M = U^-1 (Minv: B x P x P, upper triangle; frozen columns zero) by
 * recursive doubling; then every fit q of the list solves on a stored inverse,
 * delta[fits[q]] = -rscale[q] * M_f M_f^T g[fits[q]] with f = fsrc[q] (= fits[q] on its own
 * factor, a representative's slot for a cross-mask alias), zero on f's frozen coordinates.
 * tiles: ntiles x (start, count <= 32) runs of the list that share one f.  ntiles = 0 only
 * factors and inverts (g unused), nrefac = 0 only solves: the factorisation can run on
 * another stream than the gradient and the solve.  work: sglm_chol_work_bytes(P, B).  Replaces the per-iteration triangular solves (scipy
 * cho_solve inside _newton_solver.py NewtonCholeskySolver.inner_solve). */
int sglm_chol_solve_inv(float* H, float* Minv, int32_t P, const int32_t* fits,
                        const int32_t* fsrc, const float* rscale, int32_t nact, int32_t nrefac,
                        const int32_t* tiles, int32_t ntiles, const double* g,
                        const float* dshift, float* delta, int32_t* info, uint8_t* frozen,
                        int32_t B, void* work, sglm_stream_t stream);

/* The two halves of sglm_chol_solve_inv's factorisation (round 6).  sglm_chol_factor: the chain
 * alone for fits[0 .. n) -- penalty shift, frozen set, blocked Cholesky, the diagonal blocks of
 * M = U^-1 written to Minv -- after which sglm_chol_solve_alias solves on the factors;
 * sglm_chol_invert: the recursive-doubling levels that complete M, on any later stream point
 * before a sglm_chol_solve_inv solve (nrefac = 0) reads it.  Factor and inverse are bitwise those
 * of sglm_chol_solve_inv.  work: sglm_chol_work_bytes(P, B), a buffer of its own per stream. */
int sglm_chol_factor(float* H, float* Minv, int32_t P, const int32_t* fits, int32_t n,
                     const float* dshift, int32_t* info, uint8_t* frozen, int32_t B, void* work,
                     sglm_stream_t stream);
int sglm_chol_invert(const float* H, float* Minv, int32_t P, const int32_t* fits, int32_t n,
                     int32_t B, void* work, sglm_stream_t stream);

/* The factor + inverse chain of sglm_chol_solve_inv is captured per argument set (device
 * pointers, P, n, B) into a HIP graph and replayed.  The cache is a bounded LRU
 * (SGLM_CHOL_GRAPH_CAP entries, default 32); an evicted executable is destroyed after its last
 * replay completed.  _size reports the live entries; _clear destroys them all (call it before
 * freeing buffers whose addresses a cached chain holds, if they may be reused later). */
int32_t sglm_chol_graph_cache_size(void);
int sglm_chol_graph_cache_clear(void);

/* Solves on the stored factor of ANOTHER slot (engine.irls cross-mask Hessian sharing: a CV
 * split fit preconditioned by the full-data fit's Hessian at the same penalty, scaled by the
 * row-count ratio).  For i < nact: delta[fits[i]] = -rscale[i] * F^-1 F^-T g[fits[i]] with F the
 * factor a previous sglm_chol_solve_* call left in H[fsrc[i]] (its frozen set applies).
 * Replaces nothing in the reference (sklearn re-factors per fold copy, _newton_solver.py). */
int sglm_chol_solve_alias(const float* H, int32_t P, const int32_t* fits, const int32_t* fsrc,
                          int32_t nact, const double* g, const float* rscale, float* delta,
                          const uint8_t* frozen, int32_t B, void* work, sglm_stream_t stream);

/* --- float64 factorisation, exact rank decisions, minimum-norm projection --------------
 * The reference's OLS is LinearRegression -> scipy.linalg.lstsq (backend/sglm.py:96-101 ->
 * sklearn linear_model/_base.py:701), float64, minimum-norm on a rank-deficient design; its
 * unpenalised Poisson (TweedieRegressor alpha = 0, lbfgs from 0, backend/sglm.py:112-115) stays
 * in the row space of X.  These three calls replace that arithmetic:
 * sglm_chol64_factor: U[f] (float64 [nf][P][P], upper) = Cholesky of the f32 upper triangle
 *   H[hsrc[f]] plus the float64 penalty row lamp[dsrc[f]] on the diagonal (lamp NULL: dshift);
 *   coordinates with dshift[dsrc[f]][j] < 0 are excluded (state 2), zero diagonals are zero
 *   columns (state 3), a pivot whose Schur complement is <= tol * its diagonal is DEPENDENT
 *   (state 1: its row of U zeroed, U_jj = 1, its column above the diagonal kept); state 0 =
 *   kept.  nulls[f][0 .. counts[2f]) = the dependent coordinates (ascending), counts[2f + 1] =
 *   dependent + zero columns.  work: sglm_chol64_work_bytes(P, nf).  P % 64 == 0, P <= 8192.
 * sglm_chol64_solve: delta[fits[q]] = -U_f^-1 U_f^-T g[fits[q]] (f32 out) on the kept
 *   coordinates of f = fsrc[q], 0 elsewhere (g float64 [*][P]).
 * sglm_chol64_minnorm: for each fit k = fits[q] on factor f = fsrc[q]: beta[k] (float64 [*][P])
 *   -= N (N_w^T N_w)^-1 N_w^T beta[k], N = the null vectors e_d - U_KK^-1 U[K][d] of f's
 *   dependent coordinates, N_w their first pw coordinates (the coefficients, without the
 *   intercept): the minimum-norm point of the fit's solution set, fitted values unchanged on
 *   the factor's rows.  work: sglm_chol64_minnorm_work_bytes(P, nf). */
size_t sglm_chol64_work_bytes(int32_t P, int32_t nf);
int sglm_chol64_factor(const float* H, int32_t P, const int32_t* hsrc, const float* dshift,
                       const double* lamp, const int32_t* dsrc, int32_t nf, double tol,
                       double* U, uint8_t* state, int32_t* nulls, int32_t* counts, void* work,
                       sglm_stream_t stream);
/* sglm_chol64_factor_mixed: sglm_chol64_factor for a mixed 0/1 + continuous design: the rows
 *   and columns of the continuous coordinates j (cmap[j] = c >= 0, cmap[j] = -1 elsewhere) are
 *   read from the float64 Gram block S[f][c][0 .. P) (sglm_mixed_gram, exact to rounding)
 *   instead of the f32 H, so that the rank decision of a continuous column is taken on its
 *   float64 Gram row (lstsq's float64 X, sklearn _base.py:701). */
int sglm_chol64_factor_mixed(const float* H, int32_t P, const int32_t* hsrc, const float* dshift,
                             const double* lamp, const int32_t* dsrc, int32_t nf, double tol,
                             const double* S, int32_t k, const int32_t* cmap, double* U,
                             uint8_t* state, int32_t* nulls, int32_t* counts, void* work,
                             sglm_stream_t stream);
int sglm_chol64_solve(const double* U, int32_t P, const uint8_t* state, const int32_t* fits,
                      const int32_t* fsrc, int32_t nq, const double* g, float* delta,
                      sglm_stream_t stream);
/* sglm_chol64_solve_add: x[fits[q]] += U_f^-1 U_f^-T g[gsrc[q]] (float64 out; gsrc NULL: the
 *   fit's own row) on the kept coordinates of f = fsrc[q].
 * sglm_chol64_resid: r[fits[q]] = c[csrc[q]] - (G_f + diag(lamp[fits[q]])) x[fits[q]] (float64)
 *   with G_f the symmetric Gram of factor f = fsrc[q] read from the f32 upper triangle
 *   H[hsrc[f]] (exact 0/1 mask counts) and, for a mixed design, the float64 rows S[f][c] of its
 *   continuous coordinates (cmap[j] = c >= 0); 0 on excluded coordinates (dshift < 0).
 *   Together: the squared-loss fit in Gram space, x = (G + lam I')^-1 X^T (m y) with one float64
 *   refinement -- the normal equations of sklearn Ridge(solver='cholesky') (_ridge.py:201-213)
 *   and the lstsq answer of LinearRegression (_base.py:701) to float64 rounding. */
int sglm_chol64_solve_add(const double* U, int32_t P, const uint8_t* state, const int32_t* fits,
                          const int32_t* fsrc, const int32_t* gsrc, int32_t nq, const double* g,
                          double* x, sglm_stream_t stream);
int sglm_chol64_resid(const float* H, int32_t P, const int32_t* hsrc, const double* S, int32_t k,
                      const int32_t* cmap, const int32_t* fits, const int32_t* fsrc,
                      const int32_t* csrc, int32_t nq, const double* c, const double* lamp,
                      const float* dshift, const double* x, double* r, sglm_stream_t stream);
size_t sglm_chol64_minnorm_work_bytes(int32_t P, int32_t nf);
int sglm_chol64_minnorm(const double* U, int32_t P, int32_t pw, const uint8_t* state,
                        const int32_t* nulls, const int32_t* counts, int32_t nf,
                        const int32_t* fits, const int32_t* fsrc, int32_t nfit, double* beta,
                        void* work, sglm_stream_t stream);

/* Per-fit scalars of a Newton step for the B fits k = slots[q], float64 (one workgroup per
 * fit): out[q][0..6+T) = { g.d, sum lam w^2, sum lam w d, sum lam d^2, max|d_a|,
 * max|w_a + t[j] d_a| for j < T, max|d_b| } over the P coordinates of g[k] (float64), beta[k]
 * (float64), delta[k] (f32), lamp[k] (float64 penalty row); a runs over the first `ncoef`
 * coordinates (the coefficients), b over the rest (the intercept; padding is 0) -- the two
 * scales of the stopping rule (ncoef = P: every coordinate in the a terms, max|d_b| = 0).  The Armijo test and the stopping rule of sklearn's Newton
 * solver (_newton_solver.py:201-260) need only these.  T <= 16. */
int sglm_step_scalars(int32_t P, int32_t ncoef, int32_t B, const int32_t* slots, const double* g,
                      const double* beta, const float* delta, const double* lamp,
                      const double* t, int32_t T, double* out, sglm_stream_t stream);
/* beta[k] += step[q] * delta[k] for k = slots[q], q < B (float64 coefficients). */
/* sglm_step_decide: the Newton iteration's decisions for na active fits (slots act) on the
 * device -- engine.irls' stage-1 Armijo search over ts[1..4] from the trial losses L [na][5]
 * and the step scalars sc [na][6 + nts] (sglm_loss_trials_max / sglm_step_scalars), the stopping
 * rule (tol, stagnation on a fresh Hessian, failed search, iteration cap; sfloor / legacy as
 * STOP_SCALE_FLOOR / STOP_LEGACY; aa_rm [slot][2] the secant's raw steps or NULL) with the
 * per-fit prev_rel, fresh, n_iter, max_iter.  Out per fit: step64 / step32 (0 when stage 1
 * fails: flag 256, the host's stage 2 decides), relv, prop, flags (1 hit, 2 stop, 4 converged,
 * 8 out of iterations, 16 stop_tol, 32 stagnation, 64 failed, 256 stage 2, 512 a packed-R row),
 * tix (index into ts); rpos[q] = the fit's row among those that continue or await stage 2
 * (act order, -1 none), nxt[0 .. *cnt) their slots.  One workgroup. */
int sglm_step_decide(int32_t na, const int32_t* act, const double* L, const double* sc,
                     int32_t nts, const double* ts, double sigma, double tol, double sfloor,
                     int32_t legacy, const float* aa_rm, const double* prev_rel,
                     const uint8_t* fresh, const int32_t* n_iter, const int32_t* max_iter,
                     double* step64, float* step32, double* relv, double* prop, int32_t* flags,
                     int32_t* tix, int32_t* rpos, int32_t* nxt, int32_t* cnt,
                     sglm_stream_t stream);
/* sglm_aa_step: the Anderson (secant) correction of the Newton directions of the na active
 * fits (slots; engine.irls ANDERSON) in one launch: where sel[q], delta[k] becomes f - gamma (db
 * + df) (f = delta[k], df = f - raw_prev[k], db = used_prev[k] * tprev[q], gamma = df.f / df.df)
 * when that is a descent direction with gamma in [-2, 0.5]; rm[k] = (max_{j<p} |f_j|, |f_p|)
 * there, (0, 0) elsewhere; raw_prev[k] = f for every fit.  float32, fixed-order sums. */
int sglm_aa_step(int32_t P, int32_t p, int32_t na, const int32_t* slots, const uint8_t* sel,
                 const float* tprev, float* delta, float* raw_prev, const float* used_prev,
                 const double* gtot, float* rm, sglm_stream_t stream);
int sglm_step_update(int32_t P, int32_t B, const int32_t* slots, const double* step,
                     const float* delta, double* beta, sglm_stream_t stream);

/* Statistics of every (row mask, response) pair, one float64 pass: out[r][f][0..4] =
 * { sum m, sum m (y - K[r]), sum m (y - K[r])^2, sum m c(y), min over m > 0 of y } with M
 * [F][ldm] uint8 multiplicities, Y [R][n] float64, K a per-response shift (e.g. the mean of y),
 * c the half-Tweedie loss constant of `power` (sklearn constant_to_optimal_zero; power < 0:
 * not computed, 0).  The CV scores (R^2 / D^2 / mse, backend/sglm.py:150-184) and sklearn's
 * y-range check need only these.  work: sglm_mask_stats_work_bytes(F, R, n). */
size_t sglm_mask_stats_work_bytes(int32_t F, int32_t R, int64_t n);
int sglm_mask_stats(const uint8_t* M, int64_t ldm, int32_t F, const double* Y, int32_t R,
                    int64_t n, const double* K, double power, double* out, void* work,
                    sglm_stream_t stream);

/* Line search: out[q][j] = sum_i M[m][i] * loss(y_i, eta_i + t[j] * deta_i) (float64),
 * for j < T, over fit slot k = slots[q] (q when slots is NULL), q < B.
 * `work`: sglm_rowsum_work_bytes(B, T, n). */
size_t sglm_rowsum_work_bytes(int32_t B, int32_t T, int64_t n);
int sglm_loss_trials(int32_t family, float power, int64_t n, int64_t ld, int32_t B,
                     const int32_t* slots, const float* eta, const float* deta, const float* Y, const uint8_t* M,
                     const int32_t* fit_resp, const int32_t* fit_mask, const float* t,
                     int32_t T, double* out, void* work, sglm_stream_t stream);

/* sglm_loss_trials plus dmax[q] = max over the rows of mask fit_mask[k] of |deta[k][i]| (B
 * floats, zeroed by the call): the step's predictor drift per unit step length, returned with
 * the trial losses so that the host needs one round trip per Newton iteration. */
int sglm_loss_trials_max(int32_t family, float power, int64_t n, int64_t ld, int32_t B,
                         const int32_t* slots, const float* eta, const float* deta, const float* Y, const uint8_t* M,
                         const int32_t* fit_resp, const int32_t* fit_mask, const float* t,
                         int32_t T, double* out, float* dmax, void* work, sglm_stream_t stream);

/* eta[k][i] += step[q] * deta[k][i], k = slots[q] (q when slots is NULL), q < B
 * (host-chosen step per fit, device array). */
int sglm_eta_axpy(int64_t n, int64_t ld, int32_t B, const int32_t* slots, const float* step,
                  const float* deta, float* eta, sglm_stream_t stream);

/* sglm_eta_axpy plus dmax[k] = max over the rows of mask fit_mask[k] of |step[k] d_eta[k][i]|
 * (B floats, zeroed by the call): the per-step drift of the linear predictor that bounds the
 * relative change of the IRLS weights since a fit's Hessian was formed (engine.irls reuses a
 * factor while the accumulated drift stays below SGLM Hessian-reuse tolerance). */
int sglm_eta_axpy_max(int64_t n, int64_t ld, int32_t B, const float* step, const float* deta,
                      const uint8_t* M, const int32_t* fit_mask, float* eta, float* dmax,
                      sglm_stream_t stream);

/* out[q] = max over the rows of mask fit_mask[a] of |eta[a][i] - eta[b][i]| for the fit pairs
 * (a, b) = (pairs[2q], pairs[2q+1]) of one mask (npairs floats, zeroed by the call).  engine.irls
 * lets fit b take its Hessian from fit a's Gram when this distance is within tolerance. */
int sglm_eta_pair_absmax(int64_t n, int64_t ld, int32_t npairs, const int32_t* pairs,
                         const uint8_t* M, const int32_t* fit_mask, const float* eta,
                         float* out, sglm_stream_t stream);

/* Scores (GLM.score / get_residuals, backend/sglm.py:150-184, 314-331): for fit k and each
 * set s in {0, 1} with mask sets[2k + s] (-1 = empty):
 *   out[k][s][0] = sum_i M * (y_i - mu_i)^2,  out[k][s][1] = sum_i M * loss(y_i, eta_i),
 * mu = inverse link(eta).  `work`: sglm_rowsum_work_bytes(B, 4, n). */
int sglm_score_sums(int32_t family, float power, int64_t n, int64_t ld, int32_t B,
                    const float* eta, const float* Y, const uint8_t* M,
                    const int32_t* fit_resp, const int32_t* sets, double* out, void* work,
                    sglm_stream_t stream);

/* gen_signal_df.generate_signal_df (sglm/sglm/features/gen_signal_df.py:327-470).
 * sglm_scatter_rows: out[c][i] = NaN for i < n, then out[c][rows[t]] = vals[c][t] for
 * t < nrows with 0 <= rows[t] < n -- a trial-table column aligned onto the signal rows by index
 * label (`signal_df[col] = df_t_tmp.set_index(col)[...]`, :416-427); rows must be distinct.
 * sglm_signal_trials: nTrial = cumsum(center_in == 1).shift(k_before), nEndTrial =
 * cumsum(side_out == 1).shift(k_after), diffTrialNums, and the output row map of the per-trial
 * duplication loop (:437-458): src[q] = signal row of output row q, dup[q] = 1 for the copies
 * (rows with diffTrialNums > 1 repeated ahead of their nTrial run with nTrial - 1); rows with
 * a NaN nTrial are dropped.  Output rows = n - |k_before| (clamped) + *ncopies (device
 * double).  src/dup need 2n entries; work: sglm_signal_trials_work_bytes(n). */
int sglm_scatter_rows(int64_t n, const int64_t* rows, int64_t nrows, const double* vals,
                      int32_t ncols, double* out, int64_t ld_out, sglm_stream_t stream);
size_t sglm_signal_trials_work_bytes(int64_t n);
int sglm_signal_trials(const double* center_in, const double* side_out, int64_t n,
                       int64_t k_before, int64_t k_after, double* ntrial, double* nend,
                       double* diff, int64_t* src, uint8_t* dup, double* ncopies, void* work,
                       sglm_stream_t stream);

/* --- session preprocessing (lynne_pp.preprocess_lynne, lynne_pp.py:217-249) -------------
 * Input: SGLM_PREP_NIN float64 columns of n rows, column c at in + c * ld_in, in the order of
 * enum sglm_prep_in (the renamed session columns of lynne_pp.rename_columns, :95-111).
 * Output: SGLM_PREP_NOUT float64 columns, column c at out + c * ld_out, in the order of enum
 * sglm_prep_out, which is the order in which the reference appends them:
 *   define_trial_starts_ends (:20-44): event_col (cpn*1 | lpx*2 | rpx*2, zeros as NaN,
 *     backward fill), trial_start_flag ((ev == 1) & (ev.shift(-1) != 1), shifted by -k),
 *     nTrial (its NaN-skipping cumulative sum), event_col_end (lpx*2 | rpx*2 | start flag,
 *     forward fill), trial_end_flag ((ece == 2) & (ece.shift(1) != 2) & (nTrial > 0), shifted
 *     by +k), nEndTrial;  set_reward_flags (:113-125): r_trial / nr_trial from the per-trial
 *     sum of r;  set_port_entry_exit_... (:127-158): r / nr products;  define_side_agnostic_
 *     events (:160-180): left + right sums;  get_first_time_events (:182-215): nn, xx, the
 *     first-transition indicators of the per-trial cumulative sums of nn, xx, cpn and the
 *     nn / xx / r / nr products.
 * k = trial_shift_bounds (any sign).  Rows whose shifted source lies outside [0, n) are NaN in
 * the flag columns and the cumulative sums skip them (pandas skipna).  Exact for integer-
 * valued event columns (indicator counts); per-trial sums of non-integer r are summed in
 * chunk order.  `work`: sglm_prep_work_bytes(n) bytes.  n == 0 is a no-op. */
enum sglm_prep_in {
    SGLM_PREP_IN_CPN = 0, SGLM_PREP_IN_LPX, SGLM_PREP_IN_RPX, SGLM_PREP_IN_LPN, SGLM_PREP_IN_RPN,
    SGLM_PREP_IN_R, SGLM_PREP_IN_NR, SGLM_PREP_IN_RL, SGLM_PREP_IN_LL, SGLM_PREP_NIN
};
enum sglm_prep_out {
    SGLM_PREP_OUT_EVENT_COL = 0, SGLM_PREP_OUT_TRIAL_START_FLAG, SGLM_PREP_OUT_NTRIAL,
    SGLM_PREP_OUT_EVENT_COL_END, SGLM_PREP_OUT_TRIAL_END_FLAG, SGLM_PREP_OUT_NENDTRIAL,
    SGLM_PREP_OUT_R_TRIAL, SGLM_PREP_OUT_NR_TRIAL,
    SGLM_PREP_OUT_RPXR, SGLM_PREP_OUT_RPXNR, SGLM_PREP_OUT_LPXR, SGLM_PREP_OUT_LPXNR,
    SGLM_PREP_OUT_RPNR, SGLM_PREP_OUT_RPNNR, SGLM_PREP_OUT_LPNR, SGLM_PREP_OUT_LPNNR,
    SGLM_PREP_OUT_SPN, SGLM_PREP_OUT_SPX, SGLM_PREP_OUT_SPNR, SGLM_PREP_OUT_SPNNR,
    SGLM_PREP_OUT_SPXR, SGLM_PREP_OUT_SPXNR, SGLM_PREP_OUT_SL,
    SGLM_PREP_OUT_NN, SGLM_PREP_OUT_XX,
    SGLM_PREP_OUT_FT_NN, SGLM_PREP_OUT_FT_XX, SGLM_PREP_OUT_FT_LPN, SGLM_PREP_OUT_FT_RPN,
    SGLM_PREP_OUT_FT_SPN, SGLM_PREP_OUT_FT_LPX, SGLM_PREP_OUT_FT_RPX, SGLM_PREP_OUT_FT_SPX,
    SGLM_PREP_OUT_FT_CPN,
    SGLM_PREP_OUT_FT_R_RPN, SGLM_PREP_OUT_FT_R_LPN, SGLM_PREP_OUT_FT_R_SPN,
    SGLM_PREP_OUT_FT_NR_RPN, SGLM_PREP_OUT_FT_NR_LPN, SGLM_PREP_OUT_FT_NR_SPN,
    SGLM_PREP_NOUT
};
size_t sglm_prep_work_bytes(int64_t n);
int sglm_prep_session(const double* in, int64_t ld_in, int64_t n, int32_t k, double* out,
                      int64_t ld_out, void* work, sglm_stream_t stream);

/* --- gradient of a time-shifted event design ---------------------------------------------
 * X[t, col(b, a)] = E[t + row0 - shifts[b], a] for a 0/1 event matrix E (m events, K lags;
 * col = b*m + a for layout 0 (shift-major, sglm_ez.timeshift_cols), a*K + b for layout 1
 * (event-major, setup_model_fit.timeshift_vals_by_dict)), the ones column at m*K:
 * g[slots[q]][c] = sum_{t < n} X[t, c] R[slots[q]][t] (float64, c < P; columns past m*K zero)
 * from the event occurrences: occ = every event's occurrence rows u of E, event-major and
 * ascending; tbeg / tend [m][ntiles] = the occurrence index range of event a whose window
 * [u - row0 + min(shifts), u - row0 + max(shifts)] meets design-row tile i (tiles of
 * sglm_lag_tile_rows() rows, ntiles = ceil(n / that)).  m <= 64, K <= 256.  Replaces the
 * X^T (y - mu) products of sklearn's gradient (_linear_loss.py:37-54) on the expanded design.
 * work: sglm_lag_xtr_work_bytes(P, K, B, n) for up to B active fits. */
int32_t sglm_lag_tile_rows(void);
size_t sglm_lag_xtr_work_bytes(int32_t P, int32_t K, int32_t B, int64_t n);
int sglm_lag_xtr(const int32_t* occ, const int32_t* tbeg, const int32_t* tend,
                 const int32_t* shifts, int32_t m, int32_t K, int32_t layout, int64_t row0,
                 int64_t n, int32_t P, const float* R, int64_t ld, const int32_t* slots,
                 int32_t nact, double* g, void* work, sglm_stream_t stream);

/* sglm_xtr_prefer(1): this thread's following sglm_xtr_bits / _packed calls use the
 * one-fit-group four-panel gradient kernel (fewer registers per lane, so work on another
 * stream -- the factorisation chain -- can share the SIMDs); -1 restores the automatic choice. */
int sglm_xtr_prefer(int32_t variant);

/* --- Gram of a time-shifted event design at a constant weight ---------------------------
 * H[fits[q]] = bf16(W[fits[q] * ldw]) * X^T X (f32, the 128-blocks I <= J of the P x P upper
 * triangle; other entries untouched) over design rows t < n of the design above (layout 0 / 1,
 * the ones column at m*K, zero padding to P), from the occurrences: occ / ev_off (event-major
 * ascending rows, segment offsets [m + 1]), ebits = [m][nwords] occurrence bitmap of E (bit
 * v & 31 of word v >> 5, n_raw rows), smin / smax = min / max of shifts (span <= 2048).  The
 * Hessian of every all-rows fit at its intercept-only start (constant weight on every row):
 * the first Newton iteration's Gram of engine.irls, which replaces the first cho_solve
 * Hessian of sklearn's NewtonCholeskySolver on the expanded design (_newton_solver.py,
 * backend/sglm.py:112-115).  work: sglm_lag_gram_work_bytes(m, smin, smax). */
size_t sglm_lag_gram_work_bytes(int32_t m, int32_t smin, int32_t smax);
int sglm_lag_gram(const int32_t* occ, const int32_t* ev_off, const uint32_t* ebits,
                  int64_t nwords, const int32_t* shifts, int32_t m, int32_t K, int32_t layout,
                  int32_t smin, int32_t smax, int64_t row0, int64_t n, int64_t n_raw, int32_t P,
                  const float* W, int64_t ldw, const int32_t* fits, int32_t nfits, float* H,
                  void* work, sglm_stream_t stream);

/* sglm_lag_gram with the intercept column at pc >= m*K: columns m*K .. pc-1 (a mixed
 * design's continuous columns, completed by sglm_mixed_gram / sglm_mixed_to_h) are written 0. */
int sglm_lag_gram_pc(const int32_t* occ, const int32_t* ev_off, const uint32_t* ebits,
                     int64_t nwords, const int32_t* shifts, int32_t m, int32_t K, int32_t layout,
                     int32_t smin, int32_t smax, int64_t row0, int64_t n, int64_t n_raw, int32_t P,
                     int32_t pc, const float* W, int64_t ldw, const int32_t* fits, int32_t nfits,
                     float* H, void* work, sglm_stream_t stream);

/* --- mixed 0/1 + continuous designs ------------------------------------------------------
 * The production design of the reference (sglm_cb_concat_make_design_mat.py:224-244, 310) puts
 * continuous counters (cumcount^2 / 5000, pp_design_mat.py:167-172) beside 0/1 event lags and
 * fits it in float64 through simple_cv_fit (:356-363 -> backend/sglm_cv.py:106-131 -> sklearn).
 * Here the k continuous columns are a float64 block C [k][ldc] at design positions cpos[c]
 * (their bit-plane columns are zero); these calls complete the bit-plane kernels' products.
 * Row sums are chunked and summed in a fixed order (deterministic).
 * sglm_mixed_wc: R[q][r] = W[slots[q / k]][r] * f32(C[q % k][r]) (r < n; 0 up to ld), the f32
 *   operand of sglm_xtr_bits for the Gram rows X^T W C of an IRLS Hessian.
 * sglm_mixed_gram: S[s][c][cpos[c']] = S[s][c'][cpos[c]] = sum_r wt_s(r) C[c][r] C[c'][r]
 *   (float64) for c <= c' (pairs: device int32 [2][k(k+1)/2], the (c, c') lists); wt_s =
 *   f32 W[wsel[s]] (wmode 0) or uint8 mask M[wsel[s]] (wmode 1), rows of ldw elements.
 * sglm_mixed_xtr: g[gslots[q]][cpos[c]] = sum_r C[c][r] R_q(r) (float64) for q < nq, R_q = row
 *   rsel[q] (q when NULL) of: f32 [*][ldr] (rmode 0); the packed three-piece bf16 buffer of
 *   sglm_link_update, [3][Bp][ldr] (rmode 2); one bf16 plane [*][ldr] (rmode 3).  pairs: device
 *   int32 [2][k] = {0 .. k-1, k .. k}.  Replaces the continuous coordinates of X^T (mu - y).
 * sglm_mixed_eta: eta[slot][r] += sum_c C[c][r] beta[slot][cpos[c]] (float64 sum, r < n) for
 *   slot = slots[q] (q when NULL), q < nb; k <= 1024.
 * sglm_mixed_to_h: H[slot][i][cpos[c]] = H[slot][cpos[c]][i] = f32(S[s][c][i]) for i < P,
 *   slot = slots[s] (s when NULL).
 * work (gram, xtr): sglm_mixed_work_bytes(ns or nq, k, n). */
size_t sglm_mixed_work_bytes(int32_t ns, int32_t k, int64_t n);
int sglm_mixed_wc(const float* W, int64_t ldw, const int32_t* slots, int32_t ns, const double* C,
                  int64_t ldc, int32_t k, int64_t n, int64_t ld, float* R, sglm_stream_t stream);
int sglm_mixed_gram(int32_t wmode, const void* wsrc, int64_t ldw, const int32_t* wsel, int32_t ns,
                    const double* C, int64_t ldc, int32_t k, int64_t n, const int32_t* cpos,
                    int32_t P, const int32_t* pairs, double* S, void* work, sglm_stream_t stream);
int sglm_mixed_xtr(int32_t rmode, const void* R, int64_t ldr, int64_t Bp, const int32_t* rsel,
                   const int32_t* gslots, int32_t nq, const double* C, int64_t ldc, int32_t k,
                   int64_t n, const int32_t* cpos, int32_t P, const int32_t* pairs, double* g,
                   void* work, sglm_stream_t stream);
int sglm_mixed_eta(const double* C, int64_t ldc, int32_t k, int64_t n, const int32_t* cpos,
                   const float* beta, int32_t P, const int32_t* slots, int32_t nb, float* eta,
                   int64_t ld, sglm_stream_t stream);
int sglm_mixed_to_h(const double* S, int32_t ns, int32_t k, int32_t P, const int32_t* cpos,
                    const int32_t* slots, float* H, sglm_stream_t stream);

/* --- event design matrix (pp_design_mat.make_design_mat, pp_design_mat.py:6-205) --------
 * Float64 session columns (a pandas float block) on the device.  A pandas groupby over a float
 * key is a GROUPING here:
 * sglm_group_rows: perm[0 .. m) = the rows whose key (and key2, when not NULL) is not NaN,
 *   grouped by key value (lexicographic (key, key2)), row order kept within a group (pandas'
 *   group and within-group order; NaN-key rows are dropped as groupby drops them);
 *   seg[0 .. nseg] = group starts in perm plus m; counts = {m, nseg, ordered} (device int64,
 *   3 entries).  Ordered keys (non-decreasing over the valid rows) take a stable compaction,
 *   others a stable LSD radix sort; both paths are enqueued and the device picks one, so the
 *   call never waits on the host -- unless sorted_out (host, may be NULL) asks for the verdict,
 *   which costs one stream synchronisation.  work: sglm_group_rows_work_bytes(n).  n < 2^31.
 *   Replaces groupby('nTrial') / groupby(['nTrial', 'nENL']) (:52, 114-120, 171-175, 200).
 * sglm_trial_lookup: tidx[i] = position of key[i] in the ascending, unique trial ids tkeys,
 *   -1 when NaN or absent -- Series.map(trials[...]) (:93, 112, 123, 192).
 * sglm_dm_heatmap: add_heatmap_columns (:108-126) into out (5 x ld_out): hm_t_cue_offset_to_sel
 *   = tsel[tidx] (tidx NULL: NaN), hm_t_from_cue_onset, hm_t_from_cons_onset (trial_clock minus
 *   the group's first non-null clock of its Cue == 1 / Consumption == 1 rows),
 *   hm_t_sel_to_cons = (sum stateConsumption - sum Consumption) * 20, hm_t_cue_offset_to_cons.
 *   Group sums run in a fixed order: exact for integer-valued state columns.
 * sglm_dm_licks: Lick = ~isnan(iSpout) (from_spout) or the given Lick column; out[c] =
 *   states[c] * Lick (classify_lick_state, :6-23); lick_out (may be NULL) gets Lick.  Host
 *   arrays of device pointers, nstates <= 32.
 * sglm_dm_counters: time_from_enl_onset = cumcount^2 / 5000 over the (ENL == 1 | Cue == 1)
 *   rows of each nTrial group, time_from_enlp_onset over the state_ENLP == 1 rows of each
 *   (nTrial, nENL) group (NaN on such rows with a NaN key, 0 elsewhere) (:167-172); cue_on (may
 *   be NULL): 1 on each group's first Cue == 1 row (:175, 182-183).
 * sglm_dm_pull: pull_lick_from_bout (:26-58) for positions nth[0 .. npull) in processing order:
 *   cols[j] = 1 on the (nth - 1)-th (negative: from the end) bout == 1 row of each group, that
 *   bout row set to 0.  npull <= 16; nth and cols are host arrays.
 * sglm_dm_heatmap_k / sglm_dm_counters_k / sglm_dm_pull_k: the same with the grouping keys
 *   (key = nTrial, key2 = nENL of the second grouping): the per-row default pass then writes only
 *   the rows outside the groups (the group walks write every row of a group), a second write
 *   of the whole column saved.  NULL keys: the entries above.
 * sglm_trial_map: dst[dst_cols[c]][i] = (src_cols[c] < 0 ? 1 : src[src_cols[c]][i]) *
 *   vals[val_cols[c]][tidx[i]] (NaN when tidx[i] < 0): event_interactions_dummies (:87-99)
 *   and the flag's mapped isna (:192).  Index arrays on the device.  sglm_trial_map_u8: the same
 *   with a uint8 value table (0/1 dummy products and isna flags: exact, 1/8 of the upload).
 * sglm_zero_groups_flag: flag = 1 on every row of the groups whose listed columns sum to 0
 *   (skipna) -- the trials without a cue dummy (:198-203); group_zero (may be NULL, >= nseg
 *   bytes) gets 1 for those groups (the printed trials_without_dummies, :201-202). */
size_t sglm_group_rows_work_bytes(int64_t n);
int sglm_group_rows(const double* key, const double* key2, int64_t n, int64_t* perm,
                    int64_t* seg, int64_t* counts, int32_t* sorted_out, void* work,
                    sglm_stream_t stream);
int sglm_trial_lookup(const double* key, int64_t n, const double* tkeys, int64_t nt,
                      int32_t* tidx, sglm_stream_t stream);
int sglm_dm_heatmap(const double* clock, const double* cue, const double* cons,
                    const double* scons, int64_t n, const int64_t* perm, const int64_t* seg,
                    const int64_t* counts, const int32_t* tidx, const double* tsel, double* out,
                    int64_t ld_out, sglm_stream_t stream);
int sglm_dm_licks(const double* lick_src, int32_t from_spout, const double* const* states,
                  int32_t nstates, int64_t n, double* const* out, double* lick_out,
                  sglm_stream_t stream);
int sglm_dm_counters(const double* enl, const double* cue, const double* senlp, int64_t n,
                     const int64_t* perm, const int64_t* seg, const int64_t* counts,
                     const int64_t* perm2, const int64_t* seg2, const int64_t* counts2,
                     double* tenl, double* tenlp, double* cue_on, sglm_stream_t stream);
int sglm_dm_pull(double* bout, int64_t n, const int64_t* perm, const int64_t* seg,
                 const int64_t* counts, const int32_t* nth, int32_t npull, double* const* cols,
                 sglm_stream_t stream);
int sglm_dm_heatmap_k(const double* clock, const double* cue, const double* cons,
                      const double* scons, const double* key, int64_t n, const int64_t* perm,
                      const int64_t* seg, const int64_t* counts, const int32_t* tidx,
                      const double* tsel, double* out, int64_t ld_out, sglm_stream_t stream);
int sglm_dm_counters_k(const double* enl, const double* cue, const double* senlp,
                       const double* key, const double* key2, int64_t n, const int64_t* perm,
                       const int64_t* seg, const int64_t* counts, const int64_t* perm2,
                       const int64_t* seg2, const int64_t* counts2, double* tenl, double* tenlp,
                       double* cue_on, sglm_stream_t stream);
int sglm_dm_pull_k(double* bout, const double* key, int64_t n, const int64_t* perm,
                   const int64_t* seg, const int64_t* counts, const int32_t* nth, int32_t npull,
                   double* const* cols, sglm_stream_t stream);
int sglm_trial_map(int64_t n, const int32_t* tidx, const double* src, int64_t ld_src,
                   const int32_t* src_cols, const double* vals, int64_t nt,
                   const int32_t* val_cols, int32_t ncols, double* dst, int64_t ld_dst,
                   const int32_t* dst_cols, sglm_stream_t stream);
int sglm_trial_map_u8(int64_t n, const int32_t* tidx, const double* src, int64_t ld_src,
                      const int32_t* src_cols, const uint8_t* vals, int64_t nt,
                      const int32_t* val_cols, int32_t ncols, double* dst, int64_t ld_dst,
                      const int32_t* dst_cols, sglm_stream_t stream);
int sglm_zero_groups_flag(int64_t n, const int64_t* perm, const int64_t* seg,
                          const int64_t* counts, const double* src, int64_t ld,
                          const int32_t* cols, int32_t ncols, double* flag,
                          uint8_t* group_zero, sglm_stream_t stream);

/* --- grid setup on the host (CPU, multithreaded; no device pointers) -------------------
 * sglm_host_masks: row mask f (uint8, out + f * ld, zero past n) of a CV grid from its index
 * list -- the fold selections of the reference's loop (backend/sglm_cv.py:107-110):
 * SGLM_MASK_ALL every row (idx unused), SGLM_MASK_FOLD a fold list (0/1 when strictly
 * increasing, else the multiplicity of each row; > 255 repeats is an error), SGLM_MASK_ROWS a
 * row list (1 on every listed row).  nnz[f] = rows with a nonzero mask, sum[f] = the summed
 * multiplicity (either may be NULL).  An index in [-n, 0) names row idx + n (numpy fancy
 * indexing, as X[idx_train] treats it); indices outside [-n, n) are an error. */
enum { SGLM_MASK_ALL = 0, SGLM_MASK_FOLD = 1, SGLM_MASK_ROWS = 2 };
int sglm_host_masks(int32_t nm, const int64_t* const* idx, const int64_t* len,
                    const int32_t* kind, int64_t n, int64_t ld, uint8_t* out, int64_t* nnz,
                    double* sum, int32_t nthreads);

/* Threaded host copies into pinned staging buffers (chunked uploads): sglm_host_copy copies
 * nbytes; sglm_host_gather_cols copies ncols columns of nrows elements of elem bytes (host
 * pointers src[c], element strides stride[c], NULL = contiguous) to dst column-major.  Host only, no device pointers. */
int sglm_host_copy(void* dst, const void* src, int64_t nbytes, int32_t nthreads);
int sglm_host_gather_cols(const void* const* src, const int64_t* stride, int32_t ncols,
                          int64_t nrows, int32_t elem, void* dst, int32_t nthreads);
/* sglm_host_pack_bits_cols: float64 columns (src[c], element stride stride[c]) as bit-planes,
 * bit r of bits[c * ceil(nrows / 32) + r / 32] = (value == 1.0); binary[c] = 1 when every
 * value is 0.0 or 1.0; ones[c] (may be NULL) = the count of 1.0 values.  The 0/1 event
 * columns of a lagged frame cross PCIe as bits. */
int sglm_host_pack_bits_cols(const void* const* src, const int64_t* stride, int32_t ncols,
                             int64_t nrows, uint32_t* bits, uint8_t* binary, int64_t* ones,
                             int32_t nthreads);
/* sglm_host_group_rows: the row lists of GroupShuffleSplit folds from per-group sides --
 * out[j] (caller-allocated, len[j] entries) = the ascending rows i < n with
 * side[(j / 2) * G + gidx[i]] == 1 + (j % 2) (1 train, 2 test), j < 2 * nsplits:
 * np.flatnonzero(is_train[gidx]) / (is_test[gidx]) per split (sklearn _split.py:2181-2187,
 * as backend/sglm_pp.py:236-264 draws them).  len[j] must equal the row count it selects. */
int sglm_host_group_rows(const int64_t* gidx, int64_t n, const uint8_t* side, int32_t nsplits,
                         int64_t G, int64_t* const* out, const int64_t* len, int32_t nthreads);
/* sglm_host_group_runs: the same lists for groups laid out as runs of consecutive rows (a
 * non-decreasing trial id column): run r = rows start[r] .. start[r] + rlen[r] - 1 of group
 * grp[r] (runs ascending, disjoint); list 2k / 2k + 1 = the rows of the runs whose group has
 * side[k][g] == 1 / 2.  No per-row group index (cv_idx_by_trial_id on a sorted trial column). */
int sglm_host_group_runs(const int64_t* start, const int64_t* rlen, const int64_t* grp,
                         int64_t nruns, const uint8_t* side, int32_t nsplits, int64_t G,
                         int64_t* const* out, const int64_t* len, int32_t nthreads);

#ifdef __cplusplus
}
#endif
#endif /* SGLM_HIP_H */
