/* Sanitizer driver for the oracle restatement (oracle/ob_oracle.c, test infrastructure): the
 * Random123 Philox KAT, the reference's OLS known answers (ols.rs:151-209), the OBRS-1 index
 * stream and a small threaded bootstrap, built with -fsanitize=address,undefined
 * (tests/asan/Makefile) and run by tests/test_asan.py. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

typedef struct {
  int k, pool_pos, ref_mode, weighted, n_norm;
  const int *norm_start, *norm_idx, *norm_m, *pooled_start, *pooled_idx, *has_base;
} orc_cfg;
void orc_philox4x32_10(const uint32_t ctr_in[4], const uint32_t key_in[2], uint32_t out[4]);
void orc_resample_indices(uint64_t seed, uint32_t rep, uint32_t g, uint32_t n, uint32_t* idx_out);
int orc_ols(const double* y, const double* x, int64_t n, int k, const double* w, double* beta, double* resid_out,
            int full);
int orc_row_len(int k, int n_base);
void orc_boot_ref(const orc_cfg* cfg, const double* xa, const double* ya, const double* wa, int64_t na,
                  const double* xb, const double* yb, const double* wb, int64_t nb, uint64_t seed, uint32_t first_rep,
                  uint32_t n_reps, int full, int nthreads, double* rows, uint8_t* ok);
void orc_bootstrap_stats(const double* v, int64_t n, double* out);
void orc_rif(const double* y, int64_t n, double tau, double* out);

static int failures = 0;
#define CHECK(c)                                                     \
  do {                                                               \
    if (!(c)) {                                                      \
      fprintf(stderr, "CHECK failed at %d: %s\n", __LINE__, #c);    \
      ++failures;                                                    \
    }                                                                \
  } while (0)

int main(void) {
  const uint32_t ctr[4] = {0, 0, 0, 0}, key[2] = {0, 0};
  uint32_t out[4];
  orc_philox4x32_10(ctr, key, out); /* Random123 kat_vectors */
  CHECK(out[0] == 1713891541u && out[1] == 3781805453u && out[2] == 3159862348u && out[3] == 2600524760u);

  /* ols.rs:151-162: y = 1 + 2 x exactly */
  const double x[8] = {1, 1, 1, 1, 1, 2, 3, 4}, y[4] = {3, 5, 7, 9};
  double beta[2];
  CHECK(orc_ols(y, x, 4, 2, NULL, beta, NULL, 1) == 0);
  CHECK(fabs(beta[0] - 1.0) < 1e-12 && fabs(beta[1] - 2.0) < 1e-12);
  /* ols.rs:164-181: collinear columns */
  const double xs[12] = {1, 1, 1, 1, 1, 2, 3, 4, 2, 4, 6, 8};
  CHECK(orc_ols(y, xs, 4, 3, NULL, beta, NULL, 1) != 0);

  /* OBRS-1 index stream: every index in range, several shapes */
  const uint32_t ns[4] = {1, 255, 257, 70001};
  for (int t = 0; t < 4; ++t) {
    uint32_t* idx = (uint32_t*)malloc(sizeof(uint32_t) * ns[t]);
    orc_resample_indices(0x0B5EEDull, 7u, 1u, ns[t], idx);
    for (uint32_t i = 0; i < ns[t]; ++i) CHECK(idx[i] < ns[t]);
    free(idx);
  }

  /* a small threaded bootstrap (2 groups x 500 rows, intercept + 2 predictors, weighted) */
  enum { N = 500, K = 3, R = 24 };
  double *xa = malloc(sizeof(double) * N * K), *xb = malloc(sizeof(double) * N * K);
  double ya[N], yb[N], wa[N], wb[N];
  for (int i = 0; i < N; ++i) {
    xa[i] = xb[i] = 1.0;
    xa[N + i] = sin(0.1 * i) * 3 + 10;
    xb[N + i] = cos(0.1 * i) * 3 + 9;
    xa[2 * N + i] = (i % 17) * 0.5;
    xb[2 * N + i] = (i % 13) * 0.5;
    ya[i] = 1 + 0.5 * xa[N + i] + 0.2 * xa[2 * N + i] + 0.01 * (i % 7);
    yb[i] = 0.8 + 0.4 * xb[N + i] + 0.25 * xb[2 * N + i] + 0.01 * (i % 5);
    wa[i] = 0.5 + (i % 3) * 0.5;
    wb[i] = 1.5 - (i % 4) * 0.25;
  }
  orc_cfg cfg = {K, 3, 0, 1, 0, NULL, NULL, NULL, NULL, NULL, NULL};
  const int rl = orc_row_len(K, 0);
  double* rows = (double*)malloc(sizeof(double) * R * rl);
  uint8_t ok[R];
  orc_boot_ref(&cfg, xa, ya, wa, N, xb, yb, wb, N, 0x0B5EEDull, 0, R, 1, 4, rows, ok);
  double col[R], st[4];
  int n = 0;
  for (int r = 0; r < R; ++r) {
    CHECK(ok[r]);
    if (ok[r]) col[n++] = rows[r * rl];
  }
  orc_bootstrap_stats(col, n, st);
  CHECK(isfinite(st[0]) && st[0] >= 0.0);
  double rif[N];
  orc_rif(ya, N, 0.5, rif);
  CHECK(isfinite(rif[0]));
  free(rows);
  free(xa);
  free(xb);
  printf("oracle_asan: %s (%d failed checks)\n", failures ? "FAIL" : "ok", failures);
  return failures ? 1 : 0;
}
