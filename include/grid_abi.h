/*
 * grid_abi.h -- C ABI of libgridhip.so, the MI355X (gfx950) implementation of
 * GRiD pipeline steps 4-7 (depth normalisation -> nearest neighbours ->
 * diploid CN -> haploid inference).
 *
 * The reference (caterer-z-t/GRiD) is pure Python; its "FFI" for this path is
 * the set of step functions the orchestrator calls
 * (grid/pipeline.py:66-103).  Our Python step modules (grid_amd/utils/ step modules)
 * keep those signatures and bind THIS header through ctypes
 * (grid_amd/_abi.py).  Each entry point below cites the reference code it
 * replaces.  Plain C: pointers + sizes, no torch types.
 *
 * Conventions
 *  - Every function returns int: GRID_OK (0) or an error code; the message is
 *    in grid_last_error() (thread-local).  No C++ exception crosses the ABI.
 *  - "d_" pointers are DEVICE pointers (from grid_dev_alloc, or any HIP
 *    allocation of the same runtime, e.g. a torch tensor's data_ptr()).
 *    "h_" pointers are host pointers.  Caller owns every buffer.
 *  - Work is enqueued on the context's stream; results are ready after
 *    grid_sync(ctx) (or a later blocking grid_d2h).
 *  - Depth matrices hold mosdepth depths as int32 HUNDREDTHS (the reference
 *    parses "%.2f" text with float(); q/100.0 in IEEE fp64 is that same
 *    double).  GRID_MISSING marks a NaN cell.
 *  - All fp64 statistics reproduce the reference's NumPy operation order
 *    bit for bit (kernels are built with -ffp-contract=off).
 */
#ifndef GRID_ABI_H
#define GRID_ABI_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GRID_OK 0
#define GRID_EINVAL 1
#define GRID_EHIP 2
#define GRID_EZERODIV 3
#define GRID_EUNSUPPORTED 4
#define GRID_ERANGE 5

#define GRID_MISSING ((int32_t)0x80000000)   /* NaN depth cell            */
#define GRID_ZQ_NAN ((int32_t)0x80000000)    /* z printed as "NA"         */
#define GRID_ZQ_NEG0 ((int32_t)0x80000001)   /* z printed as "-0.00"      */
#define GRID_BLOCK 8192                      /* NumPy reduction buffer    */
/* Compact depth matrix codes (uint16 hundredths; see grid_depth16). */
#define GRID_Q16_MAXV 0xFFFD                 /* largest value stored inline */
#define GRID_Q16_ESC 0xFFFE                  /* value in the escape table   */
#define GRID_Q16_MISS 0xFFFF                 /* NaN depth cell              */

typedef struct grid_ctx grid_ctx;

/* ---------------------------------------------------------------- runtime */
const char *grid_last_error(void);
/* Provenance of this build (no reference counterpart): a JSON object with the
 * sha256 of the native sources it was compiled from (grid_amd/csrc/Makefile
 * HASHED), the compiler, the target arch and the UTC build time, written into
 * out (NUL-terminated, truncated to cap - 1); returns the full length.
 * grid_amd/_abi.py refuses a library whose hash is not the tree's. */
int grid_build_info(char *out, int64_t cap);
int grid_abi_version(void);
int grid_device_count(int *n);
int grid_ctx_create(int device, grid_ctx **out);
int grid_ctx_destroy(grid_ctx *ctx);
/* Enqueue on an external hipStream_t (e.g. torch.cuda.current_stream()
 * .cuda_stream); NULL selects the default (null) stream.
 * grid_ctx_own_stream restores the context's private non-blocking stream. */
int grid_ctx_set_stream(grid_ctx *ctx, void *hip_stream);
int grid_ctx_own_stream(grid_ctx *ctx);
/* Compute units of the context's device (persistent grids, batch sizing). */
int grid_ctx_cu_count(grid_ctx *ctx, int32_t *n);
/* The context's own stream re-created with a CU mask (hipExtStreamCreateWithCUMask;
 * bit c of mask[c / 32] = CU c): the device chain gives its one-workgroup
 * phasing lane one CU and its one-round column-statistics passes the others,
 * so the two never share a CU.  grid_ctx_stream: the stream the context
 * enqueues on (for a caller's events). */
int grid_ctx_own_stream_cumask(grid_ctx *ctx, const uint32_t *mask, int32_t nwords);
int grid_ctx_stream(grid_ctx *ctx, void **out);
/* hipMemGetInfo of the context's device: free and total HBM bytes (buffer
 * lifetime checks: the step-4 ingest releases its device buffers). */
int grid_mem_info(grid_ctx *ctx, size_t *free_bytes, size_t *total_bytes);
int grid_sync(grid_ctx *ctx);
int grid_dev_alloc(grid_ctx *ctx, size_t bytes, void **d_ptr);
int grid_dev_free(grid_ctx *ctx, void *d_ptr);
/* Page-locked host memory (copies at PCIe speed; the device ingest stages). */
int grid_host_alloc(size_t bytes, void **h_ptr);
int grid_host_free(void *h_ptr);
int grid_h2d(grid_ctx *ctx, void *d_dst, const void *h_src, size_t bytes);
int grid_d2h(grid_ctx *ctx, void *h_dst, const void *d_src, size_t bytes);
int grid_d2d(grid_ctx *ctx, void *d_dst, const void *d_src, size_t bytes);
/* Asynchronous copies on the context stream (page-locked host memory; the
 * caller keeps the host buffer unchanged until an event after the copy). */
int grid_h2d_async(grid_ctx *ctx, void *d_dst, const void *h_src, size_t bytes);
int grid_d2h_async(grid_ctx *ctx, void *h_dst, const void *d_src, size_t bytes);
/* Named events for stream-to-stream and stream-to-host ordering (the device
 * ingest's pipeline: copy stream -> inflate/parse stream -> host reuse of the
 * staging buffers).  put = record on ctx's stream; wait = ctx's stream waits;
 * host_wait = the calling thread blocks until the event completes. */
int grid_event_new(void **ev);
int grid_event_free(void *ev);
int grid_event_put(grid_ctx *ctx, void *ev);
int grid_event_wait(grid_ctx *ctx, void *ev);
int grid_event_host_wait(void *ev);
int grid_memset(grid_ctx *ctx, void *d_dst, int value, size_t bytes);
/* Event timing on the context stream (for bench.py): returns ms between two
 * recorded markers. */
int grid_event_record(grid_ctx *ctx, int slot);
int grid_event_elapsed(grid_ctx *ctx, int slot_a, int slot_b, float *ms);
/* Order ctx's stream after everything enqueued so far on src's stream (an
 * event recorded on src, waited on by ctx): the runtime's own cross-stream
 * dependency, so work on ctx sees memory src's copies wrote (the device
 * ingest's CPU-inflated text, copied on its own stream). */
int grid_stream_after(grid_ctx *ctx, grid_ctx *src);

/* --------------------------------------------------------- step 4: normalize
 * Replaces grid/utils/normalize_mosdepth.py normalize_matrix :419-476 and
 * individual_raw_means :120 (np.nanmean(axis=1) -> 8192-block pairwise sums;
 * np.nanmean/np.nansum(axis=0) -> sequential over rows).
 *
 * d_q: [n][ld] int32 hundredths, columns [0, m) are this shard, whose first
 * column sits at a GLOBAL offset that is a multiple of GRID_BLOCK. */

/* Compact depth matrix: the same hundredths as uint16 q[i*ld + j] (half the
 * HBM bytes of every pass), values > GRID_Q16_MAXV exactly in a row-sorted
 * escape table (eoff: [n+1] offsets, ecol / eval: column and value).  All
 * pointers are device pointers; the struct itself is passed from the host. */
typedef struct grid_depth16 {
  const uint16_t *q;
  const int64_t *eoff;
  const int32_t *ecol;
  const int32_t *eval;
} grid_depth16;
/* int32 hundredths -> compact form.  Escape table capacity exc_cap entries;
 * *h_nexc receives the number needed (GRID_ERANGE if > exc_cap). */
int grid_q16_encode(grid_ctx *ctx, const int32_t *d_q, int64_t n, int64_t m, int64_t ld,
                    uint16_t *d_q16, int64_t ld16, int64_t *d_eoff, int32_t *d_ecol,
                    int32_t *d_eval, int64_t exc_cap, int64_t *h_nexc);
/* The q16 forms of the four step-4 passes below (same outputs bit for bit). */
int grid_norm_row_blocks_q16(grid_ctx *ctx, const grid_depth16 *q, int64_t n, int64_t m,
                             int64_t ld, double *d_blocksum, int32_t *d_blockcnt);
int grid_norm_col_means_q16(grid_ctx *ctx, const grid_depth16 *q, int64_t n, int64_t m,
                            int64_t ld, const double *d_rowmean, double *d_mu);
int grid_norm_col_vars_q16(grid_ctx *ctx, const grid_depth16 *q, int64_t n, int64_t m,
                           int64_t ld, const double *d_rowmean, const double *d_mu,
                           double *d_var, double *d_ratio);

/* Per-row, per-8192-block pairwise sums of q/100 (NaN->0) and counts.
 * d_blocksum/d_blockcnt: [n][ceil(m/8192)]. */
int grid_norm_row_blocks(grid_ctx *ctx, const int32_t *d_q, int64_t n, int64_t m, int64_t ld,
                         double *d_blocksum, int32_t *d_blockcnt);
/* rowmean[i] = (((0 + b0) + b1) + ...) / count  (np.nanmean axis=1). */
int grid_norm_row_means(grid_ctx *ctx, const double *d_blocksum, const int32_t *d_blockcnt,
                        int64_t n, int64_t nblk, double *d_rowmean);
/* mu[j] = nanmean_i(q_ij/100/rm_i); cnt; (normalize_mosdepth.py:442-445) */
int grid_norm_col_means(grid_ctx *ctx, const int32_t *d_q, int64_t n, int64_t m, int64_t ld,
                        const double *d_rowmean, double *d_mu);
/* var[j] = nansum_i((y_ij-mu_j)^2)/(n-1); ratio = mu>0 ? 100*var/mu : NaN  (:446-451) */
int grid_norm_col_vars(grid_ctx *ctx, const int32_t *d_q, int64_t n, int64_t m, int64_t ld,
                       const double *d_rowmean, const double *d_mu, double *d_var,
                       double *d_ratio);
/* Ascending sort of the non-NaN values of d_v; *h_nvalid receives the count.
 * d_sorted must hold n doubles.  (np.median :462 / sorted() :495) */
int grid_sort_valid(grid_ctx *ctx, const double *d_v, int64_t n, double *d_sorted,
                    int64_t *h_nvalid);
/* fp64 depths (the route for depth text that is not exact hundredths; the
 * reference reads any decimal with float(), :272,334): d_x [n][ld] doubles,
 * NaN = missing.  The same results as the int32 hundredths entry points
 * (NumPy pairwise row sums, sequential column sums, exact %.2f codes), without
 * their fast paths. */
int grid_norm_row_blocks_f64(grid_ctx *ctx, const double *d_x, int64_t n, int64_t m, int64_t ld,
                             double *d_bsum, int32_t *d_bcnt);
/* mu, var, ratio of every column (grid_norm_col_means + grid_norm_col_vars) */
int grid_norm_col_stats_f64(grid_ctx *ctx, const double *d_x, int64_t n, int64_t m, int64_t ld,
                            const double *d_rowmean, double *d_mu, double *d_var, double *d_ratio);
/* int32 z hundredths of the selected columns (grid_norm_zquant's codes) */
int grid_norm_zquant_f64(grid_ctx *ctx, const double *d_x, int64_t n, int64_t ld, const int32_t *d_sel,
                         int64_t r, const double *d_rm, const double *d_mu, double scale, int32_t *d_zq,
                         int64_t ld_zq, int32_t *h_overflow);
/* Count of the non-NaN values of d_v (the length grid_sort_valid would report). */
int grid_count_valid(grid_ctx *ctx, const double *d_v, int64_t n, int64_t *h_nvalid);
/* h_vals[j] = the h_ks[j]-th smallest (0-based) non-NaN value of d_v, for
 * 1 <= nk <= 4 ranks 0 <= k < count: the sorted()[k] / np.median reads of
 * :462 / :495 without sorting (radix select, 8 passes over d_v).  Ranks -0.0
 * before +0.0 where grid_sort_valid (like sorted()) keeps equal zeros in input
 * order, so a zero may differ in sign only; every use compares values. */
int grid_select_kth(grid_ctx *ctx, const double *d_v, int64_t n, const int64_t *h_ks, int32_t nk,
                    double *h_vals);
/* Stable compaction of indices j with v[j] > thr (NaN never kept). (:499) */
int grid_select_gt(grid_ctx *ctx, const double *d_v, int64_t n, double thr, int32_t *d_idx,
                   int64_t *h_count);
/* out[i] = float("%.{decimals}f" % v[i]) (exact decimal rounding, half-even on
 * the binary value; NaN/inf pass through). */
int grid_round_decimals(grid_ctx *ctx, const double *d_v, int64_t n, int decimals,
                        double *d_out);
/* Gather: out[i] = v[idx[i]] (NaN where idx[i] < 0). */
int grid_gather_f64(grid_ctx *ctx, const double *d_v, const int32_t *d_idx, int64_t n,
                    double *d_out);
/* find_neighbors.py:171 keep-mask -> column map: colmap[s] = rank among kept
 * (or -1); *h_ruse = number kept.  keep = finite(r) && r>=smin && r<=smax. */
int grid_colmap_range(grid_ctx *ctx, const double *d_r, int64_t n, double smin, double smax,
                      int32_t *d_colmap, int64_t *h_ruse);
/* Region selection on the device (the chain's pass C without host round
 * trips).  State d_st: GRID_SEL_STATE int64 slots (doubles stored as bits).
 * Stage 1: nvalid = count of non-NaN d_rall[:rlen]; v0, v1 = the median pair's
 * order statistics and v2 = thr = sorted(...)[int(top_frac * nvalid)]
 * (normalize_mosdepth.py:462,495; err = 1 for Python's IndexError);
 * d_sel = {j < ml : d_ratio[j] > thr} (r_loc of them, :499); d_r3[i] =
 * float("%.3f" % d_ratio[d_sel[i]]) for i < r_loc and NaN up to len_pad;
 * r_tot = r_loc (the caller sums it over ranks before stage 2).
 * Stage 2: nv = count of non-NaN d_r3all[:r3len]; smin = sorted(r3all)
 * [min(int(r_tot * (1 - frac_r)), nv - 1)], smax = sigma2_max (both +-inf when
 * nv == 0; find_neighbors.py:166-171); d_colmap as grid_colmap_range over
 * d_r3[:r_loc] (entries up to ml: -1), ruse = kept count.
 * grid_sel_read: copy the slots to h_st (synchronises the stream). */
#define GRID_SEL_STATE 16
#define GRID_SEL_NVALID 0
#define GRID_SEL_RLOC 1
#define GRID_SEL_RTOT 2
#define GRID_SEL_NV 3
#define GRID_SEL_RUSE 4
#define GRID_SEL_ERR 5
#define GRID_SEL_THR 8
#define GRID_SEL_V0 9
#define GRID_SEL_SMIN 12
#define GRID_SEL_SMAX 13
int grid_sel_stage1(grid_ctx *ctx, const double *d_rall, int64_t rlen, const double *d_ratio, int64_t ml,
                    int64_t len_pad, double top_frac, int32_t *d_sel, double *d_r3, int64_t *d_st);
int grid_sel_stage2(grid_ctx *ctx, const double *d_r3all, int64_t r3len, const double *d_r3, int64_t ml,
                    double frac_r, double sigma2_max, int32_t *d_colmap, int64_t *d_st);
int grid_sel_read(grid_ctx *ctx, const int64_t *d_st, int64_t *h_st);
/* Deferred status: called with h_overflow = h_nesc = NULL (grid_norm_zquant_kb16*)
 * or h_zerodiv = NULL (grid_dipcn), those calls do not synchronise; this copies
 * the 16-byte status block the call just left (int32 flags at byte 0, uint64
 * escape count at byte 8) to d_dst on the stream, to be read later.  Call it
 * before any other entry point runs on the context. */
int grid_status_copy(grid_ctx *ctx, void *d_dst);
/* z_{i,s} = ((q/100/rm_i - mu_j)/sqrt(mu_j))*scale for j = sel[s]
 * (normalize_mosdepth.py:458,470), quantised exactly as "%.2f" into
 * d_zq[i*ld_zq + s] (GRID_ZQ_NAN / GRID_ZQ_NEG0 sentinels; may be NULL), and,
 * for colmap[s] >= 0, clip(., -qmax, qmax) hundredths stored as bf16 into
 * d_zb[i*ld_zb + colmap[s]] (find_neighbors.py:57-58,65; may be NULL).
 * *h_overflow (may be NULL) reports |z*100| >= 2^31. */
int grid_norm_zquant(grid_ctx *ctx, const int32_t *d_q, int64_t n, int64_t ld,
                     const int32_t *d_sel, int64_t r, const double *d_rowmean,
                     const double *d_mu, double scale, int32_t *d_zq, int64_t ld_zq,
                     const int32_t *d_colmap, int32_t qmax, uint16_t *d_zb, int64_t ld_zb,
                     int32_t *h_overflow);
/* The same with the bf16 panel K-blocked, as grid_knn_gram_kb reads it:
 * element (i, c) at d_zb[(c/64)*np_zb*64 + i*64 + c%64]; np_zb >= n, % 64 == 0. */
int grid_norm_zquant_kb(grid_ctx *ctx, const int32_t *d_q, int64_t n, int64_t ld,
                        const int32_t *d_sel, int64_t r, const double *d_rowmean,
                        const double *d_mu, double scale, int32_t *d_zq, int64_t ld_zq,
                        const int32_t *d_colmap, int32_t qmax, uint16_t *d_zb, int64_t np_zb,
                        int32_t *h_overflow);

/* The same with the step-4 output compacted to int16 (half the HBM writes):
 * d_zq16[i*ld_zq + s] = the hundredths v when GRID_ZQ16_MIN <= v <=
 * GRID_ZQ16_MAX, GRID_ZQ16_NAN / GRID_ZQ16_NEG0 for the sentinels, and
 * GRID_ZQ16_ESC for any other v, which is recorded exactly in the escape list
 * (d_esc_idx[e] = i*ld_zq + s, d_esc_val[e] = v; *h_nesc = entries, in no
 * particular order).  Bit 0 of *h_overflow as above; bit 1 = more than
 * esc_cap escapes (the list holds the first esc_cap; the caller reruns
 * grid_norm_zquant_kb with int32 output).  Needs ld % 4 == 0. */
#define GRID_ZQ16_NAN (-32768)
#define GRID_ZQ16_NEG0 (-32767)
#define GRID_ZQ16_ESC (-32766)
#define GRID_ZQ16_MIN (-32765)
#define GRID_ZQ16_MAX 32767
int grid_norm_zquant_kb16(grid_ctx *ctx, const int32_t *d_q, int64_t n, int64_t ld,
                          const int32_t *d_sel, int64_t r, const double *d_rowmean,
                          const double *d_mu, double scale, int16_t *d_zq16, int64_t ld_zq,
                          const int32_t *d_colmap, int32_t qmax, uint16_t *d_zb, int64_t np_zb,
                          int64_t *d_esc_idx, int32_t *d_esc_val, int64_t esc_cap, int64_t *h_nesc,
                          int32_t *h_overflow);

int grid_norm_zquant_kb_q16(grid_ctx *ctx, const grid_depth16 *q, int64_t n, int64_t ld,
                            const int32_t *d_sel, int64_t r, const double *d_rowmean,
                            const double *d_mu, double scale, int32_t *d_zq, int64_t ld_zq,
                            const int32_t *d_colmap, int32_t qmax, uint16_t *d_zb, int64_t np_zb,
                            int32_t *h_overflow);
/* grid_norm_zquant_kb16 on the compact depth matrix (ld % 8 == 0): the same
 * int16 codes, escape list and panel as on the int32 matrix it encodes. */
int grid_norm_zquant_kb16_q16(grid_ctx *ctx, const grid_depth16 *q, int64_t n, int64_t ld,
                              const int32_t *d_sel, int64_t r, const double *d_rowmean,
                              const double *d_mu, double scale, int16_t *d_zq16, int64_t ld_zq,
                              const int32_t *d_colmap, int32_t qmax, uint16_t *d_zb, int64_t np_zb,
                              int64_t *d_esc_idx, int32_t *d_esc_val, int64_t esc_cap, int64_t *h_nesc,
                              int32_t *h_overflow);

/* Verification (tests): recompute every selected cell with plain IEEE fp64
 * in the reference's order and the "%.2f" rule, compare with the int16 codes
 * (d_zq16[i*ld_zq + s]) and, if d_zb, the K-blocked bf16 panel at colmap[s].
 * h_counts[3]: z mismatches, panel mismatches, skipped (missing) cells. */
int grid_verify_zquant(grid_ctx *ctx, const int32_t *d_q, int64_t n, int64_t ld, const int32_t *d_sel,
                       int64_t r, const double *d_rm, const double *d_mu, double scale,
                       const int16_t *d_zq16, int64_t ld_zq, const int32_t *d_colmap, int32_t qmax,
                       const uint16_t *d_zb, int64_t np_zb, int64_t *h_counts);

/* The full fp64 matrix normalize_matrix returns (:458, :470): z[i*m+j] =
 * ((y-mu)/sqrt(mu))*scale where mu > 0, y*scale elsewhere, NaN if missing. */
int grid_norm_zfull(grid_ctx *ctx, const int32_t *d_q, int64_t n, int64_t m, int64_t ld,
                    const double *d_rowmean, const double *d_mu, double scale, double *d_z);

/* ---------------------------------------------------- step 5: neighbours
 * Replaces grid/utils/find_neighbors.py find_neighbors_sklearn :179-227
 * (sklearn NearestNeighbors brute Euclidean ArgKmin).
 *
 * d_zb: [np][kpad] bf16 integer hundredths (|v| <= qmax <= 256), rows >= n
 * and columns >= R_use zero.  np % 128 == 0, kpad % 64 == 0.
 * Gram G = Zb Zb^T exactly: bf16 MFMA with fp32 partial sums flushed to
 * integers every <= 2^24/qmax^2 products, int64 atomics across K-slices.
 * d_gram: [np][np] int64, must be zeroed; only tiles (ti <= tj) are written. */
int grid_knn_gram(grid_ctx *ctx, const uint16_t *d_zb, int64_t np_, int64_t kpad, int64_t ld,
                  int32_t qmax, int64_t *d_gram);
/* The same on a K-blocked panel [kpad/32][np][32] (grid_norm_zquant_kb's
 * layout: one K-step of a row panel is contiguous); np % 256 == 0. */
int grid_knn_gram_kb(grid_ctx *ctx, const uint16_t *d_zb, int64_t np_, int64_t kpad, int32_t qmax,
                     int64_t *d_gram);
/* Cohort split of step 5 (the reference's all-pairs search,
 * find_neighbors.py:204-213, with the Gram's ROWS sharded over ranks): rows
 * [row0, row0 + nrows) x columns [row0, np) of G = Zb Zb^T on the K-blocked
 * panel of grid_knn_gram_kb -- the upper-triangle 256x128 tiles whose rows lie
 * in the range (row0, nrows multiples of 256) -- ADDED as int64 into
 * d_out[(i - row0) * ld + (j - row0)], ld >= np - row0.  Called once per
 * panel piece (the pieces' K ranges are disjoint; integer sums, so any order
 * is exact).  Entries below the diagonal outside the 256-row diagonal tiles
 * are not written (grid_knn_mirror_ld completes them). */
int grid_knn_gram_kb_rows(grid_ctx *ctx, const uint16_t *d_zb, int64_t np_, int64_t kpad, int32_t qmax,
                          int64_t row0, int64_t nrows, int64_t *d_out, int64_t ld);
/* Lower triangle from the upper: every 64x64 block (a, b), a > b, of the
 * [np][np] Gram becomes the transpose of block (b, a), so row i is contiguous
 * (np % 64 == 0).  Idempotent. */
int grid_knn_mirror(grid_ctx *ctx, int64_t *d_gram, int64_t np_);
/* The same on the leading n x n block of a row-major buffer of stride ld
 * (n % 64 == 0, ld >= n): the diagonal block of a cohort-split segment. */
int grid_knn_mirror_ld(grid_ctx *ctx, int64_t *d, int64_t n, int64_t ld);
/* d_norms[j] = G_jj (= ||z_j||^2) for j < n. */
int grid_knn_diag(grid_ctx *ctx, const int64_t *d_gram, int64_t np_, int64_t n, int64_t *d_norms);
/* Row top-k on complete Gram rows: d_rows[r*ld + j] = G(row0 + r, j) for
 * j < n (a mirrored Gram, or one rank's row block after the multi-GPU
 * reduce-scatter), d_norms[j] = G_jj.  Per row i = row0 + r: the min(k+1, n)
 * smallest (d2, j) with d2 = G_ii + G_jj - 2 G_ij, self dropped, first k kept
 * (find_neighbors.py:205-225).  d_idx/d_d2: [nrows][k]; d_cnt[r] = entries
 * written; unused slots hold idx -1, d2 0.  n is the total sample count. */
int grid_knn_topk_rows(grid_ctx *ctx, const int64_t *d_rows, int64_t ld, const int64_t *d_norms,
                       int64_t n, int64_t k, int64_t row0, int64_t nrows, int32_t *d_idx,
                       int64_t *d_d2, int32_t *d_cnt);
/* General values (not bf16-exact: |hundredths| > 256, or not hundredths at
 * all, e.g. zmax = 2.005 clips): direct-difference distances
 * d2[i][j] = sum_k (z_ik - z_jk)^2, sequential over k, for all pairs (the
 * lower triangle mirrored), into d_d2 [np][np] fp64:
 *   grid_knn_dist_i32: z integer hundredths, exact int64 sums (the caller
 *     keeps 4 max|z|^2 r < 2^53 so the fp64 store is exact; |z| < 2^30);
 *   grid_knn_dist_f64: z fp64 values, fixed-order fp64 sums (no FMA).
 * d_z: [n][ld] row-major; np % 64 == 0. */
int grid_knn_dist_i32(grid_ctx *ctx, const int32_t *d_z, int64_t n, int64_t r, int64_t ld, double *d_d2,
                      int64_t np_);
int grid_knn_dist_f64(grid_ctx *ctx, const double *d_z, int64_t n, int64_t r, int64_t ld, double *d_d2,
                      int64_t np_);
/* Row top-k on d2 rows (d_d2rows[r*ld + j] = d2(row0 + r, j)), ordered by
 * (floor(d2 * key_scale), j) with floor(d2 * key_scale) < 2^44: key_scale =
 * 1 keeps exact integer distances exact; d_d2 receives the d2 values. */
int grid_knn_topk_d2(grid_ctx *ctx, const double *d_d2rows, int64_t ld, double key_scale, int64_t n,
                     int64_t k, int64_t row0, int64_t nrows, int32_t *d_idx, double *d_d2,
                     int32_t *d_cnt);
/* Step-5 inputs from the step-4 hundredths (find_neighbors.py:57-58,171):
 * columns d_cols[0..r) of d_zq [n][ld], clipped to +-qmax (+-zmax) with
 * GRID_MISSING -> 0, as the K-blocked bf16 panel of grid_knn_gram_kb
 * ([kpad/32][np][32], zero padded; qmax <= 256), as dense int32 [n][r], or
 * as fp64 values clip(q/100, +-zmax) [n][r]. */
int grid_knn_panel_i32(grid_ctx *ctx, const int32_t *d_zq, int64_t n, int64_t ld, const int32_t *d_cols,
                       int64_t r, int32_t qmax, uint16_t *d_zb, int64_t np_, int64_t kpad);
int grid_knn_gather_i32(grid_ctx *ctx, const int32_t *d_zq, int64_t n, int64_t ld, const int32_t *d_cols,
                        int64_t r, int32_t qmax, int32_t *d_out);
int grid_knn_gather_f64(grid_ctx *ctx, const int32_t *d_zq, int64_t n, int64_t ld, const int32_t *d_cols,
                        int64_t r, double zmax, double *d_out);
/* grid_knn_mirror + grid_knn_diag + grid_knn_topk_rows on rows [row0,
 * row0 + nrows) of a Gram whose upper tiles are written (the lower triangle
 * is filled in place). */
int grid_knn_topk(grid_ctx *ctx, int64_t *d_gram, int64_t n, int64_t np_, int64_t k,
                  int64_t row0, int64_t nrows, int32_t *d_idx, int64_t *d_d2, int32_t *d_cnt);
/* Multi-GPU (the sharded chain's step 5; find_neighbors.py:207-225 on a Gram
 * summed over bin shards): ranks reduce only upper-triangle SEGMENTS of the
 * Gram -- block b = rows [r0, r0 + nrows) x columns [c0, c0 + ncols), r0 = c0
 * = b*B -- and take the neighbours from candidates.  grid_knn_seg_topk on one
 * segment (d_seg[u*ld + t] = G(r0 + u, c0 + t), norms as grid_knn_topk_rows):
 *   d_rowc [nrows][GRID_SEG_K1]: per segment row i < n, the k+1 smallest
 *     packed keys (d2 << 20 | j) over its columns j in [c0, n), ascending;
 *   d_colc [ncols][GRID_SEG_K1]: per column j < n, the k+1 smallest keys
 *     (d2 << 20 | i) over the segment's rows i < n;
 * unused entries ~0.  grid_knn_seg_merge: rows' candidates d_rowc [n'][K1]
 * in global row order and every block's column lists d_colc [2W][ldc][K1]
 * (block b's column t = sample b*B + t) -> the neighbour lists of all n rows,
 * as grid_knn_topk_rows would give them on complete rows (exact: every pair
 * is in the segment of the lower block index, as row or as column). */
#define GRID_SEG_K1 16
int grid_knn_seg_topk(grid_ctx *ctx, const int64_t *d_seg, int64_t ld, int64_t nrows, int64_t ncols,
                      const int64_t *d_norms, int64_t n, int64_t k, int64_t r0, int64_t c0,
                      unsigned long long *d_rowc, unsigned long long *d_colc);
/* The bin split's reduce-scatter send buffer from the whole (upper-triangle)
 * Gram [np_][np_] int64: for every rank q, its blocks b = q and 2W-1-q, each
 * [B][(2W - b) B] (rows b B.., columns b B..; cells beyond np_ zero), at
 * d_send + q * seg_len (seg_len = B (2W+1) B). */
int grid_knn_seg_pack(grid_ctx *ctx, const int64_t *d_gram, int64_t np_, int64_t W, int64_t B, int64_t *d_send);
int grid_knn_seg_merge(grid_ctx *ctx, const unsigned long long *d_rowc, const unsigned long long *d_colc,
                       int64_t ldc, int64_t B, int64_t n, int64_t k, int32_t *d_idx, int64_t *d_d2,
                       int32_t *d_cnt);

/* ---------------------------------------------------- step 6: diploid CN
 * Replaces grid/utils/compute_dipcn.py :62-88.
 * For each sample i: if has_reads[i] and scale[i] known: over nbr list
 * d_nbr[i*ld + t] (t < nbr_cnt[i]; -1 = neighbour absent from the counts)
 * take the first n_nbr present, total += reads[j]/nbr_scale[i*ld+t];
 * out[i] = (reads[i]/scale[i])/(total/count); valid[i] = 1 if written.
 * *h_zerodiv = 1 if the reference would raise ZeroDivisionError. */
int grid_dipcn(grid_ctx *ctx, int64_t n, const double *d_reads, const uint8_t *d_has_reads,
               const double *d_scale, const int32_t *d_nbr, const double *d_nbr_scale,
               const int32_t *d_nbr_cnt, int64_t ld, int64_t n_nbr, double *d_out,
               uint8_t *d_valid, int32_t *h_zerodiv);

/* ---------------------------------------------------- step 7: haploid
 * Replaces grid/utils/hi_inference.py _run_phasing :175-226 and _compute_imp
 * :229-250.  Hap-neighbour lists in CSR over 2n haplotypes (d_off[2n+1],
 * d_nbr hap indices, d_w weights).  The in-place Gauss-Seidel sweep is run
 * as a level schedule (grid_hi_levels) that is bit-identical to the
 * sequential order.  Outputs hap[2n] (NaN = unphased), imp[2n], *h_mean.
 * grid_hi_phase flags: GRID_HI_UNIT_WEIGHTS when every weight is 1.0;
 * max_list = longest list (selects the register capacity of the kernel).
 * Default kernel: one workgroup, one haplotype per lane, with hap in LDS while
 * 3n doubles fit (about 4,700 samples; 256 lanes, k_phase4) and in d_hap
 * otherwise (512 lanes).
 * Every flag selects a kernel with the same results. */
int grid_hi_levels(int64_t n, const int64_t *h_off, const int32_t *h_nbr, int32_t *h_order,
                   int32_t *h_level_off, int32_t *h_nlevels);
/* Host: schedule-ordered packed neighbour lists for the kernel (cap = 16 per
 * haplotype; longer lists are flagged -1 in pk_cnt and read from the CSR).
 * pk_nbr [n][2][cap], pk_w [n][2][cap], pk_cnt [n][2].  pk_w may be NULL when
 * every weight is 1.0 (GRID_HI_UNIT_WEIGHTS kernels do not read it). */
int grid_hi_pack(int64_t n, const int64_t *h_off, const int32_t *h_nbr, const double *h_w,
                 const int32_t *h_order, int32_t cap, int32_t *h_pk_nbr, double *h_pk_w,
                 int32_t *h_pk_cnt);
int grid_hi_phase(grid_ctx *ctx, int64_t n, const double *d_irr, const int64_t *d_off,
                  const int32_t *d_nbr, const double *d_w, int64_t min_nbr, int64_t n_iters,
                  const int32_t *d_order, const int32_t *d_level_off, int32_t nlevels,
                  const int32_t *d_pk_nbr, const double *d_pk_w, const int32_t *d_pk_cnt,
                  double *d_hap, double *d_imp, double *d_mean, int32_t flags, int32_t max_list);
#define GRID_HI_UNIT_WEIGHTS 1   /* every weight is 1.0 (IBS lists): weights are not read */
#define GRID_HI_LEGACY 2         /* A/B: the previous (per-neighbour LDS round trip) kernel */
#define GRID_HI_PAIRED 4         /* A/B: register-pipelined kernel with both haplotypes per lane */
#define GRID_HI_PH2 8            /* A/B: round 5's split-lane kernel (512 lanes) instead of k_phase4 */

/* Haplotype-neighbour files -> CSR (host C++; Python text semantics for ASCII
 * input).  ids_nl: the dipCN file's sample IDs joined by '\n' (index = line
 * order).  GRID_EUNSUPPORTED for inputs whose Python behaviour the parser does
 * not restate (non-ASCII text, NaN segment lengths, duplicate IDs); callers
 * then run the Python loaders.  Fetch: off [2n+1], nbr / w [nnz]. */
int grid_load_ibs(const char *path, const char *ids_nl, int64_t n_ids, int64_t max_nbr,
                  void **h_out, int64_t *nnz);                          /* hi_inference.py:34-74 */
int grid_load_ibd(const char *path, const char *ids_nl, int64_t n_ids, int64_t max_nbr,
                  int32_t weighted, int64_t region_start, int64_t region_end, double min_length,
                  double min_match, double weight_scale, void **h_out, int64_t *nnz); /* :86-172 */
int grid_hapnbr_fetch(const void *h, int64_t *off, int32_t *nbr, double *w);
int grid_hapnbr_free(void *h);

/* Batched loci (BASELINE config 5: one _run_phasing + _compute_imp per VNTR
 * region, hi_inference.py:175-250, all in one launch, one workgroup per
 * locus).  Every pointer is a device pointer with grid_hi_phase's meaning for
 * that locus; the array of descriptors itself is in device memory. */
typedef struct grid_hi_locus {
  int64_t n;                       /* samples of this locus */
  const double *irr;               /* [n] */
  const int64_t *off;              /* [2n+1] CSR offsets into nbr / w */
  const int32_t *nbr;
  const double *w;
  const int32_t *order;            /* [n] level schedule (grid_hi_levels) */
  const int32_t *loff;             /* [nlev+1] */
  int32_t nlev;
  int32_t reserved;
  const int32_t *pk_nbr;           /* grid_hi_pack output, schedule order */
  const double *pk_w;              /* NULL allowed when every weight of the locus is 1.0 */
  const int32_t *pk_cnt;
  double *hap;                     /* [2n] out */
  double *imp;                     /* [2n] out */
  double *mean;                    /* [1] out */
} grid_hi_locus;
/* grid_hi_pack of every locus on the device: fills each descriptor's pk_nbr
 * [n][2][16], pk_cnt [n][2] and (when non-NULL) pk_w from its off / nbr / w /
 * order -- the same arrays as the host grid_hi_pack, without their host build
 * and upload (config 5: 6.8 MB per 50k-sample locus).  max_n: the largest n. */
int grid_hi_pack_batch(grid_ctx *ctx, int64_t n_loci, const grid_hi_locus *d_loci, int64_t max_n);
/* max_n / max_nlev: the largest n / nlev in the batch (LDS sizing); flags and
 * max_list as grid_hi_phase, over the whole batch. */
int grid_hi_phase_batch(grid_ctx *ctx, int64_t n_loci, const grid_hi_locus *d_loci, int64_t max_n,
                        int32_t max_nlev, int64_t min_nbr, int64_t n_iters, int32_t flags,
                        int32_t max_list);

/* ---------------------------------------------------- synthetic input
 * Counter-based synthetic cohort (bench/smoke input, not a product path):
 * d_q[i*ld + j] = hundredths depth of sample i at GLOBAL bin col0 + j. */
int grid_synth_depth(grid_ctx *ctx, uint64_t seed, int64_t n, int64_t m, int64_t ld, int64_t col0,
                     int32_t nclusters, int32_t *d_q);
/* The same cohort in the compact form (grid_depth16), escapes included. */
int grid_synth_depth_q16(grid_ctx *ctx, uint64_t seed, int64_t n, int64_t m, int64_t ld16, int64_t col0,
                         int32_t nclusters, uint16_t *d_q16, int64_t *d_eoff, int32_t *d_ecol,
                         int32_t *d_eval, int64_t exc_cap, int64_t *h_nexc);

/* ---------------------------------------------------- host formatting
 * Exact "%.2f" text for integer hundredths (GRID_ZQ_* sentinels -> "NA",
 * "-0.00"), tab-joined.  Returns bytes written in *h_len (no terminator). */
/* ---------------------------------------------------- normalised-matrix text
 * The step 4 -> 5 file (normalize_mosdepth.py:502-554 writes it,
 * find_neighbors.py:81-124 reads it), host C++, threaded.
 * Writer: rows formatted exactly ("%.2f" from integer hundredths, "%.3f"
 * header values, "NA") and deflated as independent gzip members in parallel,
 * written in order (multi-member gzip: the decompressed text is the
 * reference's byte for byte).  ids_nl: IDs joined by '\n'. */
int grid_write_normalized_gz(const char *path, int64_t n, int64_t r, const char *ids_nl,
                             const double *raw, const double *sel_means, const double *sel_ratios,
                             const int32_t *zq, int64_t ld_zq, int32_t level, int32_t threads);
/* The same file from step 4's int32 hundredths still in HBM (d_zq [n][ld_zq],
 * GRID_ZQ_* sentinels): the row members are formatted, CRC'd, LZ77-parsed
 * (per 4 KiB segment against 2 KiB of the member before it) and Huffman-coded
 * on the device (one dynamic-Huffman deflate block per member, one pair of
 * canonical codes per file from the first batch's token histogram), the
 * header member (level) on the host; only compressed bytes cross PCIe.
 * batch_bytes: text formatted per device batch (<= 0: 2 GiB).  Same member
 * layout and 'GR' index as grid_write_normalized_gz; the decompressed text is
 * identical.  Its device and page-locked buffers stay on ctx between calls
 * (freed by grid_ctx_destroy), so the writer is not re-entrant per context:
 * one call at a time on a given ctx (contexts are per thread anyway). */
int grid_write_normalized_gz_dev(grid_ctx *ctx, const char *path, int64_t n, int64_t r, const char *ids_nl,
                                 const double *raw, const double *sel_means, const double *sel_ratios,
                                 const int32_t *d_zq, int64_t ld_zq, int32_t level, int32_t threads,
                                 int64_t batch_bytes);
/* Host form of that member coding (tests, small inputs): text[0, n) as one
 * plain gzip member, the device parse's LZ77 tokens (restated on the host) in
 * one dynamic-Huffman block whose codes come from text's own token
 * histogram.  *out_len = bytes needed (GRID_EINVAL when above cap). */
int grid_gz_huffman_member(const uint8_t *text, int64_t n, uint8_t *out, int64_t cap, int64_t *out_len);
/* The same file written by W ranks of a distributed `grid wgs` (each rank
 * holds the z rows [row0, row0 + n) of the cohort): the rank codes its row
 * members into host memory (a parts handle: _rows_dev from int32 hundredths
 * in HBM, as grid_write_normalized_gz_dev codes them; _rows from host memory,
 * as grid_write_normalized_gz does), rank 0 also member 0 (_header, N =
 * n_total); the ranks exchange their byte counts (_size) and each writes its
 * bytes at the exclusive prefix sum of the counts before it (_write: the file
 * exists, created by rank 0).  Every member keeps the 'GR' {size, first row}
 * index with GLOBAL row numbers, so the reader sees one indexed file and the
 * text after gunzip is the reference's.  Replaces the single writer of
 * grid/utils/normalize_mosdepth.py:502-554 under torch.distributed. */
typedef struct grid_gz_parts grid_gz_parts;
int grid_gz_parts_new(grid_gz_parts **out);
int grid_gz_parts_header(grid_gz_parts *h, int64_t n_total, int64_t r, const double *sel_means,
                         const double *sel_ratios, int32_t level, int32_t threads);
int grid_gz_parts_rows(grid_gz_parts *h, int64_t n, int64_t row0, int64_t r, const char *ids_nl, const double *raw,
                       const int32_t *zq, int64_t ld_zq, int32_t level, int32_t threads);
int grid_gz_parts_rows_dev(grid_ctx *ctx, grid_gz_parts *h, int64_t n, int64_t row0, int64_t r, const char *ids_nl,
                           const double *raw, const int32_t *d_zq, int64_t ld_zq, int32_t threads,
                           int64_t batch_bytes);
int grid_gz_parts_size(const grid_gz_parts *h, int64_t *bytes);
int grid_gz_parts_write(const grid_gz_parts *h, const char *path, int64_t offset, int32_t threads);
int grid_gz_parts_free(grid_gz_parts *h);
/* Reader: parse into a handle (*n_out rows, *r_out columns); z values as
 * integer hundredths (GRID_MISSING for "NA").  GRID_EUNSUPPORTED if the text
 * leaves the grammar (e.g. more than 2 decimals): callers fall back to the
 * general parser.  Fetch with grid_ntext_fetch, release with grid_ntext_free. */
int grid_read_normalized_gz(const char *path, int32_t threads, void **h_out, int64_t *n_out,
                            int64_t *r_out);
int grid_ntext_ids_len(const void *h, int64_t *len);
int grid_ntext_fetch(const void *h, char *ids_nl, int64_t ids_cap, double *scales, double *means,
                     double *ratios, int32_t *zq);
int grid_ntext_free(void *h);

int grid_format_hundredths(const int32_t *h_v, int64_t n, char *h_out, int64_t cap,
                           int64_t *h_len);

/* ---------------------------------------------------- host ingest (R1-R4)
 * mosdepth *.regions.bed.gz files -> int32-hundredths matrix, replacing the
 * reference's two Python passes: compute_population_mean_depths
 * (normalize_mosdepth.py:218-301), process_one_individual (:304-357) and
 * build_matrix_from_regions (:379-416).  One multithreaded inflate+parse per
 * file (a second and third only when the parsed records exceed cache_bytes);
 * population means accumulated in h_paths order (the reference's threads=1
 * order), valid = min_depth <= mean <= max_depth.
 *  h_paths[i]    file of sample i (NULL or "" = missing, contributes nothing)
 *  chrom_prefix  raw-line startswith filter (norm_chrom'd), NULL = none
 *  has_window    1 = keep end >= start && start <= end (start_bp, end_bp)
 *  mask          n_mask chromosomes (norm_chrom'd names), kb values of chrom c
 *                in mask_kb[mask_off[c] .. mask_off[c+1])
 * Returns GRID_EUNSUPPORTED if a file leaves the strict mosdepth grammar
 * (the caller then uses its line-by-line restatement).  Per-file status:
 * 0 ok, 1 failed (the reference drops the sample), 3 missing. */
typedef struct grid_ingest grid_ingest;
int grid_ingest_mosdepth(const char *const *h_paths, int64_t n_files, const char *chrom_prefix,
                         int has_window, int64_t start, int64_t end, int64_t n_mask,
                         const char *const *mask_chroms, const int64_t *mask_off,
                         const int64_t *mask_kb, double min_depth, double max_depth, int threads,
                         int64_t cache_bytes, grid_ingest **out);
/* columns (valid regions), per-file status and valid-record counts */
int grid_ingest_summary(const grid_ingest *h, int64_t *n_cols, int32_t *h_file_status,
                        int64_t *h_nvalid);
/* sorted (start, end) of the n_cols columns */
int grid_ingest_columns(const grid_ingest *h, int64_t *h_starts, int64_t *h_ends);
/* every (start, end) seen and its population mean (size query if cap < n) */
int grid_ingest_population_means(const grid_ingest *h, int64_t *h_starts, int64_t *h_ends,
                                 double *h_means, int64_t cap, int64_t *n_keys);
/* fill rows: h_q[row_of_file[i]*ld + col] (GRID_MISSING elsewhere); -1 = skip */
int grid_ingest_fill(grid_ingest *h, const int32_t *h_row_of_file, int32_t *h_q, int64_t n_rows,
                     int64_t ld);
int grid_ingest_free(grid_ingest *h);

/* ---- gzip on the device (step-4 ingest: normalize_mosdepth.py:96-112 reads
 * every regions.bed.gz with gzip.open; grid_amd/csrc/inflate.hip) ---- */
/* one gzip member of an inflated file: output bytes [start, end), trailer */
typedef struct grid_gz_member {
  int64_t start, end;
  uint32_t crc, isize;
} grid_gz_member;
#define GRID_GZ_EDATA 1     /* invalid deflate / gzip data */
#define GRID_GZ_ETRUNC 2    /* input ended inside a member */
#define GRID_GZ_ESPACE 3    /* output or member capacity exceeded */
#define GRID_GZ_EHEADER 4   /* not a gzip file (or empty) */
#define GRID_GZ_ECRC 5      /* a member's CRC-32 does not match its bytes */
/* ---- mosdepth text -> depth matrix on the device (grid_amd/csrc/mosdepth_dev.hip;
 * normalize_mosdepth.py:218-416 as ingest.cpp restates it).  Driven per batch of
 * inflated files by grid_amd/utils/ingest_device.py; every file is cut in
 * 64 KiB chunks (chunk c: file d_cfile[c], byte offset d_cstart[c]; a file's
 * chunks are d_cfirst[f] .. d_cfirst[f+1]-1). ---- */
typedef struct grid_md_opts {
  const char *d_prefix;            /* chromosome prefix (raw startswith), npre bytes */
  int32_t npre;
  int32_t has_window;
  int64_t start, end;              /* window: keep e >= start && s <= end */
  int32_t nmask;                   /* repeat mask: normalised chromosome names ... */
  int32_t reserved;
  const char *d_mask_names;
  const int32_t *d_mask_name_off;  /* [nmask + 1] */
  const int64_t *d_mask_kb_off;    /* [nmask + 1] */
  const int64_t *d_mask_kb;        /* ... and their sorted 1 kb keys */
} grid_md_opts;
#define GRID_MD_EXOTIC 1   /* a line outside the canonical grammar, or a byte >= 0x80 */
#define GRID_MD_NOTINK 2   /* a kept (start, end) outside the reference key list */
/* newlines per chunk and their per-file prefix; flags |= GRID_MD_EXOTIC for bytes >= 0x80 */
int grid_md_count(grid_ctx *ctx, const uint8_t *d_text, const int64_t *d_toff, const int64_t *d_tlen,
                  int64_t nchunks, const int32_t *d_cfile, const int64_t *d_cstart, const int32_t *d_cfirst,
                  int64_t nfiles, int32_t *d_cnl, int64_t *d_cline0, int32_t *d_flags, const int32_t *d_fstatus);
/* the reference file (one file, nlines lines): its kept keys in line order -> the key list
 * d_K ((start, end) int64 pairs, *h_nK of them), d_kidx[line] = K index or -1; *h_unsorted = 1
 * when the keys are not strictly increasing (the caller then uses the host parser) */
int grid_md_parse_ref(grid_ctx *ctx, const uint8_t *d_text, const int64_t *d_toff, const int64_t *d_tlen,
                      int64_t nchunks, const int32_t *d_cfile, const int64_t *d_cstart, const int64_t *d_cline0,
                      const grid_md_opts *opts, int32_t *d_flags, int64_t nlines, uint8_t *d_kept_line,
                      void *d_keys_line, void *d_K, int32_t *d_kidx, int64_t *h_nK, int32_t *h_unsorted);
/* every file of the batch: d_Q[d_qrow[f] * ldq + K index] = depth hundredths, d_kept[f] += records */
int grid_md_parse_map(grid_ctx *ctx, const uint8_t *d_text, const int64_t *d_toff, const int64_t *d_tlen,
                      int64_t nchunks, const int32_t *d_cfile, const int64_t *d_cstart, const int64_t *d_cline0,
                      const grid_md_opts *opts, int32_t *d_flags, const void *d_K, int64_t nK,
                      const int32_t *d_kidx, int64_t ref_nlines, int32_t *d_Q, int64_t ldq, const int32_t *d_qrow,
                      uint64_t *d_kept, const int32_t *d_fstatus);
/* d_fstatus (may be NULL in grid_md_count / grid_md_parse_map: every file parsed) = per batch
 * file, nonzero when any of its inflate units failed (the file is dropped, as the reference
 * drops a sample whose gzip does not read): grid_file_status folds the units' statuses of a
 * grid_gunzip_batch launch (d_owner[u] = the unit's batch file) on the stream, so the parse
 * needs no host round trip to know which files inflated */
int grid_file_status(grid_ctx *ctx, const int32_t *d_unit_status, const int64_t *d_owner, int64_t n_units,
                     int32_t *d_fstatus, int64_t n_files);
int grid_fill_i32(grid_ctx *ctx, int32_t *d_p, int64_t n, int32_t v);
/* population means over the rows d_rows (file order), valid columns, their positions
 * (*h_m valid), per row: entries present and entries present in valid columns */
int grid_md_finish(grid_ctx *ctx, const int32_t *d_Q, int64_t ldq, int64_t nK, int64_t nfiles,
                   const int32_t *d_rows, int32_t nrows, double min_depth, double max_depth, double *d_mean,
                   int32_t *d_valid, int64_t *d_cpos, uint64_t *d_present, uint64_t *d_nvalid, int64_t *h_m);
/* Distributed ingest (`grid wgs` under torch.distributed: rank r parses a
 * contiguous slice of the files in file order into its own d_Q over the same
 * key list K; normalize_mosdepth.py:218-301 sums the population depths in
 * that file order).  The sum is a chain over the ranks: rank r continues
 * (d_sum, d_cnt) from rank r-1 over its rows (grid_md_popsum: the same
 * sequential fp64 adds as grid_md_finish's, q / 100.0 exact); the last rank's
 * totals give the valid flags (grid_md_popvalid: mean = sum / count, the
 * min/max window, bit for bit grid_md_finish's).  Then per rank, with the
 * global valid flags: column positions (exclusive scan) and per-row counts
 * (grid_md_rowstats = grid_md_finish without the means), and the rows sent to
 * every rank's 8192-aligned column shard (grid_md_pack_shards: shard s =
 * valid columns [d_bounds[s], d_bounds[s+1]), written as [nrows][width_s] at
 * d_out + nrows * d_bounds[s], row i taken from d_Q row d_src_rows[i]). */
int grid_md_popsum(grid_ctx *ctx, const int32_t *d_Q, int64_t ldq, int64_t nK, const int32_t *d_rows,
                   int32_t nrows, double *d_sum, int64_t *d_cnt);
int grid_md_popvalid(grid_ctx *ctx, const double *d_sum, const int64_t *d_cnt, int64_t nK, double min_depth,
                     double max_depth, int32_t *d_valid);
int grid_md_rowstats(grid_ctx *ctx, const int32_t *d_Q, int64_t ldq, int64_t nK, int64_t nfiles,
                     const int32_t *d_valid, int64_t *d_cpos, uint64_t *d_present, uint64_t *d_nvalid, int64_t *h_m);
int grid_md_pack_shards(grid_ctx *ctx, const int32_t *d_Q, int64_t ldq, int64_t nK, const int32_t *d_valid,
                        const int64_t *d_cpos, const int32_t *d_src_rows, int32_t nrows, const int64_t *d_bounds,
                        int32_t nshards, int32_t *d_out);
/* the matrix: d_out[d_dst_row[f] * ldo + column] for the valid columns; their (start, end) */
int grid_md_gather(grid_ctx *ctx, const int32_t *d_Q, int64_t ldq, int64_t nK, int64_t nfiles,
                   const int32_t *d_valid, const int64_t *d_cpos, const int32_t *d_dst_row, int32_t *d_out,
                   int64_t ldo, const void *d_K, int64_t *d_starts, int64_t *d_ends);
/* host: the inflated size of a gzip file in memory (BGZF: the members' sizes; else the
 * trailer's ISIZE of a single member); GRID_EUNSUPPORTED if it is not gzip */
int grid_gz_text_size(const uint8_t *h_buf, int64_t n, int64_t *size, int32_t *members);
/* host: the BGZF members of a gzip file in memory -- byte offset, length and ISIZE of each
 * (zero padding between members skipped) -- *count of them, at most cap written (a larger
 * *count: call again with more room); GRID_EUNSUPPORTED if the file is not BGZF throughout */
int grid_gz_members(const uint8_t *h_buf, int64_t n, int64_t *h_start, int64_t *h_len, uint32_t *h_isize,
                    int32_t cap, int32_t *count);
/* host: inflate a gzip file in memory (every member, zero padding after a member skipped, as
 * CPython's gzip reader) into h_out[0, cap): libdeflate when the system library loads, else
 * zlib; *out_len bytes; *status 0, or GRID_GZ_ESPACE (cap too small), GRID_GZ_EHEADER (not
 * gzip), GRID_GZ_EDATA (anything else: corrupt, truncated, CRC); *crc (may be NULL) = the
 * CRC-32 of the whole text, combined from the members' trailers -- what the device ingest
 * checks the text against once it sits in HBM (grid_text_crc32) */
int grid_gunzip_host(const uint8_t *h_in, int64_t n, uint8_t *h_out, int64_t cap, int64_t *out_len,
                     int32_t *status, uint32_t *crc);
/* CRC-32 (gzip) of n byte ranges of device memory, d_base + h_off[i] for h_len[i] bytes
 * (host arrays), into h_crc[i]: one wave per <= 1 MiB piece, the pieces folded on the host.
 * Synchronises the stream.  The device ingest's guard over host-inflated text in HBM. */
int grid_text_crc32(grid_ctx *ctx, const uint8_t *d_base, const int64_t *h_off, const int64_t *h_len, int64_t n,
                    uint32_t *h_crc);
/* Inflate n_files gzip streams (each: every member back to back) in one launch,
 * one wave per stream (a whole file, or one BGZF member of one).  d_src +
 * d_in_off[f] (4-B aligned) holds d_in_len[f] bytes; the text goes to d_out +
 * d_out_off[f], at most d_out_cap[f] bytes; d_mem[f * mcap ...] receives the
 * members.  Per stream: d_status (0 or GRID_GZ_E*), d_out_len, d_nmem.
 * Asynchronous on the stream. */
int grid_gunzip_batch(grid_ctx *ctx, const uint8_t *d_src, const int64_t *d_in_off, const int64_t *d_in_len,
                      int64_t n_files, uint8_t *d_out, const int64_t *d_out_off, const int64_t *d_out_cap,
                      grid_gz_member *d_mem, int32_t mcap, int32_t *d_status, int64_t *d_out_len,
                      int32_t *d_nmem);

#ifdef __cplusplus
}
#endif
#endif
