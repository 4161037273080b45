// ob_heckman.hpp -- the Heckman two-step stage of a bootstrap segment (ob_heckman.hip), run after
// the selected-row Gram (weights := [s == 1]) has been reduced by the engine.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

// Panel column layout of a Heckman panel (per group, [col][ld]):
//   x_1..x_p | y | ind = [s == 1] (the Gram's weight column) | s | z_1..z_{ks-1} | (w)
struct ob_heck_seg {
  const double* cols[2];
  int64_t ld[2];
  uint32_t n[2];
  uint32_t tiles0;
  int p, ks, weighted;  // ks = 1 + selection predictors; weighted: the w column is present
  // resampling: level-2 count images (NULL = every row once: the point estimate) and chunks
  const uint32_t* counts;
  int counts_i8;  // 1: the i8 Gram's A-fragment images (ob_count_kernel<true>), 0: the f64 Gram's
  uint32_t nb_rep;
  const uint32_t* chunks;
  int n_chunks;
  uint32_t rep_pad, n_reps;
  // the selected-row extended Gram [rep][2][e_pad] over v = ind * [1, x, y]
  const double* gram;
  int e_pad, k1;
  // workspace
  double* gamma;     // [2][rep_pad][ks]
  uint32_t* hflags;  // [2][rep_pad]
  double* partial;   // [chunk][rep_pad][max(probit, sums) values]
  uint32_t* active;  // one word
  // output rows (ob_heck_row_len) and status
  int ref_mode;
  double* rows;
  uint8_t* ok;
  int row_len;
  int raw_status;  // 1: ok[] receives the status code (ob_heck_status)
  int max_iter;    // probit iterations (probit.rs: 100)
};

enum ob_heck_status {
  OB_HS_CHOLESKY = 0,  // outcome OLS: Cholesky failed (NalgebraError)
  OB_HS_OK = 1,
  OB_HS_ZERO_WEIGHT = 2,   // Weighted/Cotton: no weight in either group
  OB_HS_NO_OUTCOMES = 3,   // "No observed outcomes in group"
  OB_HS_INSUFFICIENT = 4,  // outcome OLS: selected rows <= K + 1
  OB_HS_PROBIT = 5,        // "Failed to solve Hessian system in Probit"
};

namespace ob {
constexpr int kHeckMaxKs = 8;
// Values per (chunk, replicate) of the sums kernel for K = p + 1 outcome columns.
__host__ __device__ inline int heck_sums_len(int k) { return 13 + k; }
__host__ __device__ inline int heck_probit_len(int ks) { return ks * (ks + 1) / 2 + ks; }
__host__ __device__ inline int heck_row_len(int k, int ks) { return 6 + 7 * (k + 1) + ks; }
// Largest p the register-resident sums kernel takes (13 + K <= 64).
constexpr int kHeckMaxP = 50;
// Kernel timings of one segment (HIP events on the segment's stream).
struct ob_heck_times {
  double probit_ms = 0.0;  // ob_probit_kernel, summed over the iterations
  int probit_launches = 0;
  double sums_ms = 0.0;    // ob_heck_sums_kernel
};
// Runs the probit iterations, the IMR sums and the two-step solve for one segment; on return
// (after a stream sync) rows/ok are final. iters: the probit iterations run; tm (optional): the
// kernel timings, added to.
int heckman_segment(const ob_heck_seg& h, hipStream_t s, int* iters, ob_heck_times* tm = nullptr);
}  // namespace ob
