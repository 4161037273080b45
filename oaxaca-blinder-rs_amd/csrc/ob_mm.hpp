// ob_mm.hpp -- Machado-Mata passes on the GPU (ob_mm.hip): batched quantile regressions by a
// Mehrotra predictor-corrector interior-point method, then the MM draws and empirical quantiles.
#pragma once
#include <cstdint>

#include "ob_engine.hpp"

namespace ob {
constexpr int kMmMaxK = 32;      // intercept + predictors (LDS row stride 34, two X'v column blocks)
constexpr int kMmMaxSims = 4096;  // simulations per pass (LDS sort in the finish kernel)
constexpr int kMmMaxIter = 200;   // IPM iterations per fit (Clarabel's default max_iter)

// One MM pass per replicate of [first_rep, first_rep + n_reps) (OBRS-3 resamples), preceded by
// the point estimate (every row once, MM-1 replicate OB_MM_POINT_REP) when with_point. Rows:
// [gap, characteristics, coefficients] per quantile, the point row first; ok[r] = 1 where the
// pass succeeded (quantile_decomposition.rs:231-236 failure otherwise). Host buffers.
int mm_run(ob_panel* p, uint64_t seed, int sims, const double* quantiles, int n_q, uint64_t first_rep,
           uint64_t n_reps, bool with_point, double* rows, uint8_t* ok, int* max_iters);
}  // namespace ob
