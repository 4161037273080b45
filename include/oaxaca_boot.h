/*
 * oaxaca_boot.h -- C ABI of the MI355X bootstrap-inference engine for Oaxaca-Blinder.
 *
 * Drop-in boundary for the bootstrap driver of `OaxacaBuilder::run()` in
 * dot-comma-hyphen/oaxaca-blinder-rs (paths below are relative to oaxaca_blinder/src/).
 * Plain C types only: no torch, no HIP types (a hipStream_t is passed as void*).
 * INTEGRATION.md shows the Rust `extern "C"` block and the edited run() a maintainer adds.
 *
 * Layering:
 *   1. hot path   ob_panel_* / ob_point_estimate / ob_boot_run*   replaces builder.rs:808-847
 *   2. inference  ob_bootstrap_stats / ob_rif                      inference.rs:4-34, math/rif.rs:14-88
 *   3. builder    ob_builder_* / ob_prepared_* / ob_results_*      OaxacaBuilder (builder.rs:37-983)
 *                 for hosts without a Rust toolchain (the Python front end binds these).
 *
 * All calls are blocking unless named *_device. One ob_ctx per thread, or external locking.
 * Errors: return code (OB_OK = 0) + thread-local message from ob_last_error().
 */
#ifndef OAXACA_BOOT_H
#define OAXACA_BOOT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- errors: one code per OaxacaError variant (error.rs:6-19) plus engine codes ---------- */
#define OB_OK 0
#define OB_E_POLARS 1        /* OaxacaError::PolarsError: dtype / frame errors */
#define OB_E_COLUMN 2        /* OaxacaError::ColumnNotFound */
#define OB_E_GROUP 3         /* OaxacaError::InvalidGroupVariable (also negative weights, ols.rs:60-66) */
#define OB_E_LINALG 4        /* OaxacaError::NalgebraError (Cholesky failure, ols.rs:107-111) */
#define OB_E_DIAG 5          /* OaxacaError::DiagnosticError */
#define OB_E_INSUFFICIENT 6  /* OaxacaError::InsufficientData (n <= k, ols.rs:98-105) */
#define OB_E_HIP 7           /* HIP runtime failure / no GPU: the engine never falls back to the CPU */
#define OB_E_INVALID 8       /* bad argument */
#define OB_E_UNSUPPORTED 9   /* outside the engine's scope (Heckman selection, sizes over limits) */
#define OB_E_OVERFLOW 10     /* a resample count exceeded the Gram's range in one row: 127 on the default i8
                                path (probability ~1e-215 per row and replicate), 255 on the f64 path */
#define OB_E_RCCL 11         /* RCCL missing or a collective failed (multi-GPU entry points) */

const char* ob_last_error(void);
const char* ob_version(void);

/* ---- ReferenceCoefficients (decomposition.rs:5-20) ---------------------------------------- */
#define OB_REF_GROUP_A 0
#define OB_REF_GROUP_B 1
#define OB_REF_POOLED 2   /* == Neumark */
#define OB_REF_WEIGHTED 3 /* == Cotton  */
#define OB_REF_COTTON 4
#define OB_REF_NEUMARK 5

/* ---- per-replicate row layout (Kd = K + n_base, K = p + 1 incl. the intercept) ------------ */
#define OB_ROW_EXPLAINED 0
#define OB_ROW_UNEXPLAINED 1
#define OB_ROW_ENDOWMENTS 2
#define OB_ROW_COEFFICIENTS 3
#define OB_ROW_INTERACTION 4
#define OB_ROW_TOTAL_GAP 5
#define OB_ROW_DETAILED 6 /* [6, 6+Kd) explained, [6+Kd, 6+2Kd) unexplained, then
                             beta_a[K], beta_b[K], xa_mean[K], xb_mean[K], beta_star[K] */

/* ---- device context ---------------------------------------------------------------------- */
typedef struct ob_ctx ob_ctx;
int ob_device_count(int* n);
int ob_ctx_create(int device, ob_ctx** out);
void ob_ctx_destroy(ob_ctx* ctx);

/* ---- hot path: the two groups' design, resident in HBM -------------------------------------
 * Replaces the per-replicate polars resample + prepare_data + OlsEstimator of builder.rs:816-839.
 * The caller builds X as in prepare_data (builder.rs:294-378) WITHOUT the intercept column:
 * column-major n x p, predictors then dummy columns (builder.rs:325-327). */
typedef struct {
  int64_t n;       /* rows (df_a.height() / df_b.height()) */
  const double* x; /* column-major, ldx >= n */
  int64_t ldx;
  const double* y; /* outcome */
  const double* w; /* weights or NULL */
} ob_group_desc;

typedef struct {
  int32_t p;        /* predictor columns (numeric + dummies); K = p + 1 */
  int32_t n_num;    /* numeric predictors: the pooled group indicator is inserted at 1 + n_num
                       (builder.rs:560-564 -> prepare_data extra_predictors) */
  int32_t weighted; /* 1 if .weights() was set */
  ob_group_desc a;  /* advantaged group A */
  ob_group_desc b;  /* reference group B */
  /* categorical normalization (estimation.rs:76-91, normalization.rs:5-51, builder.rs:634-674);
     n_norm = 0 disables it. Column indices count the intercept as column 0. */
  int32_t n_norm;
  const int32_t* norm_start;   /* n_norm + 1 offsets into norm_idx */
  const int32_t* norm_idx;     /* columns named "{var}_*" (normalization.rs:11-16) */
  const int32_t* norm_m;       /* category_counts[var], or -1 for a non-categorical var
                                  (then matches + 1, normalization.rs:28-31) */
  const int32_t* pooled_start; /* the same on the pooled predictor list (indicator inserted) */
  const int32_t* pooled_idx;
  const int32_t* has_base;     /* 1 if var has a base category (adds a detailed term) */
  /* outcomes (RIF multi-tau): 0 or 1 = one outcome; n_y > 1: each group's
     y is an n x n_y column-major block with leading dimension ldx, and every replicate yields
     n_y rows (one per outcome) from one Gram pass. */
  int32_t n_y;
  /* Heckman two-step (builder .heckman_selection; estimation.rs:114-260, heckman.rs:38-108):
     heckman = 1 runs a probit of s on [1, z] (math/probit.rs:25-170) and the outcome OLS on the
     rows with s = 1 augmented by the inverse Mills ratio. z: n x n_zsel column-major with
     leading dimension ldx (intercept implicit, n_zsel <= 7); s: the 0/1 selection outcome.
     With heckman = 1 the group w (if weighted) only feeds the total gap and the Cotton weights
     (the Heckman OLS is unweighted), n_norm must be 0, n_y 1, and rows carry K' = K + 1
     coefficients (IMR last) then 1 + n_zsel selection components (OB_ROW_* with K'). */
  int32_t heckman;
  int32_t n_zsel;
  const double* za;
  const double* zb;
  const double* sa;
  const double* sb;
} ob_panel_desc;

typedef struct ob_panel ob_panel;

/* Copies the design into HBM (the caller keeps ownership of its buffers). Fails with
   OB_E_GROUP on negative weights (ols.rs:60-66) and OB_E_HIP without a GPU. */
int ob_panel_create(ob_ctx* ctx, const ob_panel_desc* desc, ob_panel** out);
void ob_panel_destroy(ob_panel* panel);
int ob_panel_row_len(const ob_panel* panel);
int ob_panel_k(const ob_panel* panel);
int ob_panel_n_base(const ob_panel* panel);
int ob_panel_n_y(const ob_panel* panel);

/* Point estimate: run_single_pass on the unresampled data (builder.rs:810-811).
   resid_b (n_b entries, may be NULL) receives y_B - X_B beta_B (OaxacaResults::residuals).
   With n_y outcomes: row holds n_y x row_len, resid_b n_y x n_b (outcome-major). */
int ob_point_estimate(ob_panel* panel, int ref_mode, double* row, double* resid_b);

/* Bootstrap replicates [first_rep, first_rep + n_reps) of the OBRS-3 stream keyed by seed.
   rows: n_reps x ob_panel_row_len(); ok[r] = 0 marks a replicate the reference would drop
   (filter_map + .ok(), builder.rs:816-839): Cholesky failure or zero total weight. Results are
   a pure function of (seed, replicate id): identical on 1 or 8 GPUs. With n_y outcomes rows
   holds n_y x n_reps x row_len and ok n_y x n_reps (outcome-major blocks); each outcome's block
   is bitwise the rows a one-outcome panel of that y gives. */
int ob_boot_run(ob_panel* panel, uint64_t seed, uint64_t first_rep, uint64_t n_reps, int ref_mode,
                double* rows, uint8_t* ok);
/* Same, rows/ok in device memory, enqueued on hip_stream (hipStream_t; NULL = engine stream).
   Returns after enqueueing; synchronize the stream before reading. */
int ob_boot_run_device(ob_panel* panel, uint64_t seed, uint64_t first_rep, uint64_t n_reps,
                       int ref_mode, double* d_rows, uint8_t* d_ok, void* hip_stream);

/* HIP-event timings of the last boot run (ms summed over its launches; 0 if not run). */
typedef struct {
  double level1_ms; /* level-1 tile counts */
  double gram_ms;   /* X^T diag(c w) X MFMA kernel over the count images (the dominant kernel) */
  double reduce_ms;
  double solve_ms;  /* Cholesky solves + OB algebra */
  int32_t gram_launches;
  int32_t chunks;
  int32_t blocks;
  double counts_ms; /* level-2 count images (ob_count_kernel) */
  double heckman_ms; /* Heckman panels: probit iterations + IMR sums + two-step solve (in solve_ms too) */
  int32_t probit_iterations; /* Heckman panels: probit iterations of the last segment */
  double mm_assemble_ms;     /* ob_mm_run: mm_assemble kernel time (HIP events), summed */
  double mm_fit_rows;        /* ob_mm_run: live (fit, row) pairs those launches processed */
  int32_t mm_iterations;     /* ob_mm_run: most IPM iterations of a batch */
  double mm_ms;              /* ob_mm_run: whole call, host clock */
  double gather_ms;          /* sharded runs: the RCCL all-gather of the per-replicate rows (HIP events) */
  int32_t gram_path;         /* last boot run: 1 = f64 MFMA Gram, 2 = exact integer-sliced i8 MFMA Gram */
  double probit_ms;          /* Heckman panels: ob_probit_kernel time (HIP events), summed over iterations */
  int32_t probit_launches;   /* Heckman panels: ob_probit_kernel launches in those ms */
  double heck_sums_ms;       /* Heckman panels: ob_heck_sums_kernel (IMR sums) time */
  int32_t mm_reduced;        /* ob_mm_run: 1 if the row reduction ran (subsample, bands, reduced LPs) */
  int64_t mm_retried;        /* ob_mm_run: fits the reduction solved again on all rows (phase 3) */
  double prep_ms;            /* i8 Gram: building the panel's digit images + exception rows (HIP events;
                                nonzero only on the boot run that built them, the first of a panel) */
  int32_t oz_exceptions;     /* i8 Gram: exception rows, summed in f64 beside the integer Gram */
  int32_t oz_bits;           /* i8 Gram: a row is an exception when some |v_c| >= 2^oz_bits x its chunk's
                                scale for column c (geometric mean over nonzero rows), or not finite */
  int32_t oz_tiles6;         /* i8 Gram: (chunk, 32-pair column tile) blocks that run 6 of the 7 digit
                                slices (pairs of narrow magnitude range) */
  int32_t oz_tiles;          /* i8 Gram: all (chunk, column tile) blocks */
  int32_t oz_wide;           /* i8 Gram, last launch: 1 = the wide-tile kernel (4 waves, 256 replicates x 64
                                pairs per block), 2 = the wide tile with each chunk split over two blocks,
                                0 = the 8-wave kernel (32 pairs); option gram_tile */
} ob_timing;
int ob_panel_last_timing(const ob_panel* panel, ob_timing* out);
/* Synchronize the stream used by the last *_device call and collect its timings. */
int ob_panel_sync(ob_panel* panel);

/* ---- multi-GPU: replicates sharded over GPUs, one RCCL all-gather ----------
 * Replaces the Rayon into_par_iter of builder.rs:816-839 across devices. Replicates are
 * independent and a replicate's row is a pure function of (seed, replicate id), so the rows are
 * bitwise the same on 1, 2, 4 or 8 GPUs. Shard of rank r of W over [first_rep, first_rep + n):
 * per = ceil(n / W) replicates starting at first_rep + r * per (the last shard may be short or
 * empty). The per-replicate rows of every rank are then all-gathered over RCCL (xGMI), so every
 * rank ends with all n rows in replicate order; the caller aggregates them (ob_aggregate /
 * ob_prepared_finish) on one rank.
 *
 * One process per GPU (the torchrun / MPI shape): rank 0 calls ob_get_unique_id, sends the 128
 * bytes to every rank out of band, and each rank calls ob_ctx_create_rank with its GPU. Panels
 * created in a rank context run sharded through ob_boot_run_sharded[_device]. A plain ob_ctx acts
 * as rank 0 of 1 (no collective). */
typedef struct {
  char internal[128]; /* ncclUniqueId */
} ob_unique_id;
int ob_get_unique_id(ob_unique_id* id);
int ob_ctx_create_rank(int device, int rank, int world, const ob_unique_id* id, ob_ctx** out);
int ob_ctx_rank(const ob_ctx* ctx, int* rank, int* world);
/* This rank's shard + the all-gather; rows/ok (host) receive all n_reps rows on every rank
   (n_y outcome-major blocks as in ob_boot_run). Collective: every rank of the context calls it
   with the same seed, first_rep, n_reps and ref_mode. */
int ob_boot_run_sharded(ob_panel* panel, uint64_t seed, uint64_t first_rep, uint64_t n_reps, int ref_mode,
                        double* rows, uint8_t* ok);
/* Same into device buffers (n_reps x row_len doubles, n_reps bytes; x n_y) enqueued on hip_stream
   (NULL = engine stream); ob_panel_sync waits and fills ob_timing.gather_ms. */
int ob_boot_run_sharded_device(ob_panel* panel, uint64_t seed, uint64_t first_rep, uint64_t n_reps, int ref_mode,
                               double* d_rows, uint8_t* d_ok, void* hip_stream);
/* One process driving several GPUs: panels[i] (the same design, each created in an ob_ctx on a
   distinct device) takes shard i of n_panels; the shards are all-gathered over an RCCL clique of
   those devices (ncclCommInitAll, cached per device list) and rows/ok (host) receive all n_reps
   rows. */
int ob_boot_run_multi(ob_panel* const* panels, int n_panels, uint64_t seed, uint64_t first_rep, uint64_t n_reps,
                      int ref_mode, double* rows, uint8_t* ok);

/* The row columns the sharded entry points move over RCCL (ascending offsets into a row; n = 0 or
   every column: whole rows, the default). Aggregation reads only the component columns (two-fold,
   three-fold, total gap, detailed: [0, 6 + 2 Kd), plus the selection terms of a Heckman row), so a
   caller that only aggregates gathers those: 48 of 153 f64 per replicate at K = 21. Delivered rows
   then hold the other columns for this rank's own replicates only (NaN for the other ranks'). */
int ob_panel_set_gather_columns(ob_panel* panel, const int32_t* cols, int32_t n);
/* Test hook: a sharded run of `world` ranks simulated on this panel's one GPU -- each rank's shard
   computed and packed in turn and copied to where ncclAllGather would place it -- then delivered to
   host rows/ok as rank self_rank would receive them (the layout arithmetic of ob_shard_layout.h and
   the pack / unpack kernels of the real path, without the collective). */
int ob_debug_shard_sim(ob_panel* panel, int world, int self_rank, uint64_t seed, uint64_t first_rep, uint64_t n_reps,
                       int ref_mode, double* rows, uint8_t* ok);

/* ---- test hook: the OBRS-3 resample counts themselves (bitwise parity, builder.rs:822-827) ----
 * For replicates [first_rep, first_rep + n_reps) of `group` (0 = A, 1 = B): level1 receives
 * n_reps x ceil(n_g / 256) tile counts and row_counts n_reps x n_g per-row draw counts, exactly
 * as the Gram kernel consumes them. Either output may be NULL. */
int ob_debug_counts(ob_panel* panel, uint64_t seed, uint64_t first_rep, uint32_t n_reps, int group,
                    uint32_t* level1, uint8_t* row_counts);
/* Test hook: the reduced extended Grams G_r = sum_i c_ri v_i v_i^T (upper triangle, row-major pairs,
   e_pad per group) of replicates [first_rep, first_rep + n_reps <= 16384), gram: n_reps x 2 x e_pad,
   computed by path 1 (f64 MFMA) or 2 (exact integer-sliced i8 MFMA); 0 = the default choice. */
int ob_debug_gram(ob_panel* panel, int path, uint64_t seed, uint64_t first_rep, uint32_t n_reps, double* gram);
/* Test hook: the i8 Gram's exception rows once the panel's digit images exist:
   *bits = the threshold B, *n_exc = the number of exception rows, rows[0 .. min(cap, n_exc)) =
   (group << 31 | row) ascending. */
int ob_debug_gram_exceptions(ob_panel* panel, int32_t* bits, int32_t* n_exc, uint32_t* rows, int32_t cap);
/* Test hook: the panel's row chunking (a function of the panel only): *n_chunks chunks, and
   table[3 c .. 3 c + 2] = (group, first 256-row tile, end tile) for c < min(cap, *n_chunks).
   Host only; the Gram kernels, the exception rule and the reduce all use this table. */
int ob_debug_chunks(const ob_panel* panel, uint32_t* table, int32_t cap, int32_t* n_chunks);
/* Test hook: one Machado-Mata pass of replicate `rep` (0xFFFFFFFF: the point pass on the
   unresampled panel) and the coefficients of its quantile regressions: betas[(g S + s) K + k] for
   group g, simulation s < S = simulations (tau_s of MM-1), NaN where the fit failed; done[g S + s] = 1
   where it converged. For checks of LP optimality (objective, residual signs) on degenerate data. */
int ob_debug_mm_betas(ob_panel* panel, uint64_t seed, int32_t simulations, uint64_t rep, double* betas,
                      uint8_t* done);
/* Process-wide engine options (no reference counterpart: test and A/B switches). The library reads
   no environment variable; a caller sets these explicitly. value NaN restores the default.
     "gram_path"   1: f64 MFMA Gram, 2: i8 Gram (OB_E_UNSUPPORTED if its images do not fit)
     "gram_digits" 7: seven digit slices on every i8 column tile
     "hk_erfc"     0: library erfc in the Heckman probit/IMR kernels (default: npdf_ncdf)
     "mm_reduce"   0: no Machado-Mata row reduction, 1: always (default: both groups >= 2^16 rows)
     "mm_trace"    nonzero: Machado-Mata per-iteration trace on stderr
     "mm_state_gb", "mm_delta1", "mm_delta2", "mm_tol1", "mm_fit_stride", "mm_kappa", "mm_band0":
                   Machado-Mata tuning (the verification keeps results exact)
     "gram_diag", "l1_diag": timing ablations, tuning builds only (OB_E_UNSUPPORTED otherwise)
     "gram_tile"   1: the 8-wave i8 Gram kernel, 2: the wide-tile one, 3: the wide tile split (default: whichever the launch's
                   block count favours; their Grams are bitwise equal)
     "debug_count_overflow" nonzero: the resample's count-overflow word is raised after every
                   count kernel of a Machado-Mata run or ob_debug_counts (tests the OB_E_OVERFLOW path)
     "rs_double"   1: two level-1 / count-image buffers per panel, so each boot segment's resample
                   runs under the previous segment's Gram (rows bitwise unchanged; twice the image HBM),
                   0: one buffer (default: the engine's rule)
     "rs_pieces"   n > 1: level 1 and counts of a segment in n replicate pieces, each piece's counts beside
                   the next piece's level 1 (default 1; rows bitwise unchanged)
     "tail_stream" 1: the Gram and the reduce / solve on engine streams, the caller's stream waiting for
                   them at the end of the call (default 0; rows bitwise unchanged)
   Unknown names are OB_E_INVALID. ob_get_option reads back what ob_set_option stored (NaN: unset). ob_tuning_build() is 1 in a -DOB_TUNING=1 build (`make tuning`),
   which also reads OB_<NAME> from the environment for options nobody set. */
int ob_set_option(const char* name, double value);
int ob_get_option(const char* name, double* value);
/* Test hook: the Heckman kernels' normal pdf and cdf (npdf_ncdf: W. J. Cody's rational erfc with
   the pdf's exponential shared, ob_heckman.hip) on the device at z[0 .. n). */
int ob_debug_normal(int device, const double* z, int64_t n, double* pdf, double* cdf);
int ob_tuning_build(void);

/* ---- inference (host) --------------------------------------------------------------------- */
/* inference.rs:4-34: out = {std_err, p_value, ci_lower, ci_upper}; n = 0 gives NaNs. */
int ob_bootstrap_stats(const double* estimates, int64_t n, double point_estimate, double out[4]);
/* process_component over replicate rows (builder.rs:849-865): bootstrap_stats of row column
   cols[c] over the rows with ok != 0, in replicate order; out: n_cols x {std_err, p_value,
   ci_lower, ci_upper}. Multithreaded on the host. */
int ob_aggregate(const double* rows, const uint8_t* ok, uint64_t n_reps, int32_t row_len, const int32_t* cols,
                 int32_t n_cols, double* out);
/* math/rif.rs:14-88 (R type-7 quantile, Silverman bandwidth, Gaussian KDE). */
int ob_rif(const double* y, int64_t n, double tau, double* out);

/* ---- builder: OaxacaBuilder over a column frame ------------------------------------------- */
#define OB_COL_F64 0
#define OB_COL_I64 1
#define OB_COL_STR 2

typedef struct {
  const char* name;
  int32_t kind;
  const double* f64;       /* OB_COL_F64 */
  const int64_t* i64;      /* OB_COL_I64 */
  const char* const* str;  /* OB_COL_STR; a NULL entry is a null */
  const uint8_t* valid;    /* numeric kinds: 1 = valid, 0 = null; NULL = all valid */
} ob_column;

/* ---- CSV front end (the reference CLI's LazyCsvReader, main.rs:161-165) ------------------
 * Header row; dtypes from the first 100 rows (i64, else f64, else str); empty field = null;
 * RFC 4180 quotes. ob_csv_column views stay valid until ob_csv_free. */
typedef struct ob_csv ob_csv;
int ob_csv_read(const char* path, ob_csv** out);
int ob_csv_dims(const ob_csv* csv, int64_t* nrows, int32_t* ncols);
int ob_csv_column(const ob_csv* csv, int32_t i, ob_column* out);
void ob_csv_free(ob_csv* csv);

typedef struct {
  const char* outcome;
  const char* group;
  const char* reference_group;
  const char* const* predictors;
  int32_t n_predictors;
  const char* const* categorical;
  int32_t n_categorical;
  const char* const* normalize;
  int32_t n_normalize;
  const char* weights;           /* NULL: unweighted */
  const char* selection_outcome; /* Heckman two-step (builder .heckman_selection): the 0/1 outcome */
  uint64_t bootstrap_reps;       /* builder default 20 (builder.rs:122) */
  int32_t reference_coeffs;      /* builder default OB_REF_GROUP_A (builder.rs:123) */
  int32_t has_seed;              /* 0: fresh entropy per run, like the unseeded reference */
  uint64_t seed;
  const char* const* selection_predictors; /* Heckman: z (intercept implicit), at most 7 */
  int32_t n_selection_predictors;
} ob_builder_config;

typedef struct ob_prepared ob_prepared;
typedef struct ob_results ob_results;
typedef struct ob_matrices ob_matrices;

/* clean_dataframe -> dummies -> split_groups -> prepare_data -> HBM upload -> point estimate
   (builder.rs:787-814). */
int ob_builder_prepare(ob_ctx* ctx, const ob_column* cols, int32_t n_cols, int64_t n_rows,
                       const ob_builder_config* cfg, ob_prepared** out);
int ob_prepared_row_len(const ob_prepared* prep);
int ob_prepared_n_y(const ob_prepared* prep);
uint64_t ob_prepared_seed(const ob_prepared* prep);
ob_panel* ob_prepared_panel(ob_prepared* prep);
int ob_prepared_boot(ob_prepared* prep, uint64_t first_rep, uint64_t n_reps, double* rows, uint8_t* ok);
/* ob_boot_run_sharded over the prepared panel (its seed and reference coefficients): with a rank
   context (ob_ctx_create_rank) each rank runs its shard and every rank receives all rows. Only the
   columns ob_prepared_finish aggregates travel (ob_panel_set_gather_columns): the coefficient and
   mean columns of the other ranks' replicates arrive as NaN. */
int ob_prepared_boot_sharded(ob_prepared* prep, uint64_t first_rep, uint64_t n_reps, double* rows, uint8_t* ok);
int ob_prepared_boot_device(ob_prepared* prep, uint64_t first_rep, uint64_t n_reps, double* d_rows,
                            uint8_t* d_ok, void* hip_stream);
/* Aggregation of builder.rs:841-950 over the successful rows (ok != 0), in replicate order. */
int ob_prepared_finish(ob_prepared* prep, const double* rows, const uint8_t* ok, uint64_t n_reps,
                       ob_results** out);
void ob_prepared_destroy(ob_prepared* prep);

/* prepare + all replicates + finish: OaxacaBuilder::run() (builder.rs:787). */
int ob_builder_run(ob_ctx* ctx, const ob_column* cols, int32_t n_cols, int64_t n_rows,
                   const ob_builder_config* cfg, ob_results** out);
/* OaxacaBuilder::decompose_quantile (builder.rs:711-757). */
int ob_builder_decompose_quantile(ob_ctx* ctx, const ob_column* cols, int32_t n_cols, int64_t n_rows,
                                  const ob_builder_config* cfg, double quantile, ob_results** out);
/* Several quantiles in one run: out[t] = decompose_quantile(taus[t]),
   bitwise, from one panel whose outcomes are the n_taus RIF columns, so one Gram pass and one
   resample per replicate serve every tau. out must hold n_taus slots. */
int ob_builder_decompose_quantiles(ob_ctx* ctx, const ob_column* cols, int32_t n_cols, int64_t n_rows,
                                   const ob_builder_config* cfg, const double* taus, int32_t n_taus,
                                   ob_results** out);
/* OaxacaBuilder::get_data_matrices (builder.rs:252-291). Host only: needs no GPU. */
int ob_builder_data_matrices(const ob_column* cols, int32_t n_cols, int64_t n_rows,
                             const ob_builder_config* cfg, ob_matrices** out);

/* ---- results (types.rs:8-47,160-180) ------------------------------------------------------ */
#define OB_TABLE_TWO_FOLD 0            /* two_fold.aggregate: explained, unexplained */
#define OB_TABLE_DETAILED_EXPLAINED 1
#define OB_TABLE_DETAILED_UNEXPLAINED 2
#define OB_TABLE_DETAILED_SELECTION 3  /* Heckman only: intercept + selection predictors */
#define OB_TABLE_THREE_FOLD 4          /* endowments, coefficients, interaction */

typedef struct {
  const char* name; /* valid until ob_results_free */
  double estimate, std_err, t_stat, p_value, ci_lower, ci_upper;
} ob_component;

#define OB_VEC_RESIDUALS 0 /* point-estimate residuals of group B */
#define OB_VEC_XA_MEAN 1
#define OB_VEC_XB_MEAN 2
#define OB_VEC_BETA_STAR 3

double ob_results_total_gap(const ob_results* r);
int64_t ob_results_n_a(const ob_results* r);
int64_t ob_results_n_b(const ob_results* r);
int64_t ob_results_n_failed(const ob_results* r); /* dropped replicates (builder.rs:841-847) */
int ob_results_count(const ob_results* r, int32_t table);
int ob_results_component(const ob_results* r, int32_t table, int32_t i, ob_component* out);
int ob_results_vector(const ob_results* r, int32_t which, const double** data, int64_t* len);
void ob_results_free(ob_results* r);

/* get_data_matrices: X column-major n x K including the intercept column. */
int ob_matrices_dims(const ob_matrices* m, int64_t* n_a, int64_t* n_b, int32_t* k);
int ob_matrices_get(const ob_matrices* m, const double** x_a, const double** y_a, const double** x_b,
                    const double** y_b);
const char* ob_matrices_name(const ob_matrices* m, int32_t i);
void ob_matrices_free(ob_matrices* m);

/* ---- Machado-Mata (QuantileDecompositionBuilder, quantile_decomposition.rs:21-445) ---------
 * A pass (run_single_pass, :173-279): `simulations` quantile regressions per group at the MM-1
 * quantiles (csrc/ob_spec.h; the reference draws from an unseeded thread_rng), one MM-1 row pick
 * per group per successful simulation, predictions x_A b_A, x_B b_B, x_A b_B, and empirical
 * quantiles. Each QR (math/quantile_regression.rs:22-129, Clarabel LP) is solved on the GPU by an
 * interior-point method on its dual LP; the replicates are OBRS-3 resamples. */

/* Runs the point pass (every row once; with_point != 0) then one pass per replicate of
   [first_rep, first_rep + n_reps). rows: (with_point + n_reps) x 3 n_quantiles host doubles,
   [gap, characteristics, coefficients] per quantile; ok[r] = 0 where the pass failed (fewer than
   simulations / 2 successful fits in a group, :231-236). panel: unweighted, one outcome, at most
   31 predictor columns. Replaces run_single_pass + the bootstrap loop (:173-354). */
int ob_mm_run(ob_panel* panel, uint64_t seed, int32_t simulations, const double* quantiles,
              int32_t n_quantiles, uint64_t first_rep, uint64_t n_reps, int32_t with_point, double* rows,
              uint8_t* ok);
/* Test hook: make chosen quantile-regression fits count as failed, as Clarabel's non-Solved statuses
   do in the reference (quantile_regression.rs:120-128), to pin the pass's failure semantics
   (quantile_decomposition.rs:221-259): each group drops its failed fits independently, the
   survivors pair by index, and a pass with fewer than simulations / 2 successes in a group fails.
   mask: 2 x sims bytes [group][simulation]; fit (g, s) of pass rep fails when bit (rep & 7) of
   mask[g * sims + s] is set (the point pass has rep = 2^32 - 1, bit 7). sims = 0 clears it. */
int ob_debug_mm_fail(ob_panel* panel, const uint8_t* mask, int32_t sims);

typedef struct {
  const char* outcome;
  const char* group;
  const char* reference_group;
  const char* const* predictors;
  int32_t n_predictors;
  const char* const* categorical;
  int32_t n_categorical;
  const double* quantiles; /* NULL: the builder default {0.1, 0.25, 0.5, 0.75, 0.9} */
  int32_t n_quantiles;
  int32_t simulations;     /* builder default 200 */
  uint64_t bootstrap_reps; /* builder default 20 */
  int32_t has_seed;        /* 0: fresh entropy per run, like the reference's thread_rng */
  uint64_t seed;
} ob_qd_config;

typedef struct ob_qd_results ob_qd_results;
/* QuantileDecompositionBuilder::run over a column frame (quantile_decomposition.rs:281-445). */
int ob_quantile_decomposition_run(ob_ctx* ctx, const ob_column* cols, int32_t n_cols, int64_t n_rows,
                                  const ob_qd_config* cfg, ob_qd_results** out);
/* results_by_quantile: n entries keyed "q{floor(100 tau)}" (a repeated key keeps the later
   quantile, as the reference's HashMap does), in first-appearance order of the keys. */
int ob_qd_results_dims(const ob_qd_results* r, int32_t* n_entries, int64_t* n_a, int64_t* n_b);
/* comps[0..2] = Total Gap, Characteristics, Coefficients (QuantileDecompositionDetail). */
int ob_qd_results_get(const ob_qd_results* r, int32_t i, const char** key, ob_component* comps);
int64_t ob_qd_results_n_failed(const ob_qd_results* r);
void ob_qd_results_free(ob_qd_results* r);

#ifdef __cplusplus
}
#endif
#endif /* OAXACA_BOOT_H */
