// ob_engine.hpp -- device-side state of the bootstrap engine (HBM panel, workspaces, streams).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <vector>

#include "ob_common.hpp"

// Level-2 count images in HBM (ob_count_kernel): [tile (A then B)][replicate batch][sub-tile]
// [kCimgWords]; replicate r's counts for the sub-tile's 64 rows are the 16 words at r * 17 (+1 pad
// word), row i of the sub-tile in byte (i & 3) of word (i >> 2).
constexpr int kCimgStride = 17;               // u32 words per replicate row of a sub-tile image
constexpr int kCimgWords = 64 * kCimgStride;  // one sub-tile: 64 replicates x 64 rows (u8)

struct ob_ctx {
  int device = 0;
  int cus = 0;
  hipStream_t stream = nullptr;
  // rank contexts (ob_ctx_create_rank, ob_shard.cpp): this process's RCCL communicator
  int rank = 0, world = 1;
  void* comm = nullptr;             // ncclComm_t
  void (*comm_free)(void*) = nullptr;
};

// Normalization lists (normalization.rs:5-51) in the layout the solve kernel reads.
struct ob_norm_cfg {
  int n_norm = 0;
  int n_base = 0;
  std::vector<int32_t> start, idx, m, pstart, pidx, has_base;
};

struct ob_panel {
  ob_ctx* ctx = nullptr;
  int p = 0;        // predictor columns
  int k = 0;        // p + 1 (intercept)
  int n_y = 1;     // outcome columns (RIF multi-tau: one per quantile)
  int k1 = 0;       // p + 1 + n_y: v = [1, x, y_1..y_n_y]
  int e = 0;        // extended-Gram pairs
  int e_pad = 0;    // multiple of 16
  int ncb = 0;      // 16-wide column blocks
  int n_num = 0;
  int weighted = 0;  // the Gram's weight column is present (Heckman panels: [s == 1])
  // Heckman two-step panels (ob_heckman.hpp column layout): ks = 1 + selection predictors
  int heckman = 0, ks = 0, h_weighted = 0;
  uint32_t n[2] = {0, 0};
  int64_t ld[2] = {0, 0};      // padded rows (multiple of OB_TILE_ROWS)
  uint32_t ntiles[2] = {0, 0};
  double* d_cols[2] = {nullptr, nullptr};   // [col][ld]: x_1..x_p, y_1..y_n_y, (w)
  double* d_gpanel[2] = {nullptr, nullptr};  // Gram panel: [ld/64][k1 - c_first][96] staged images
  ob_norm_cfg norm;
  int32_t* d_norm = nullptr;               // packed norm lists
  int row_len = 0;

  // workspace, sized for `cap_reps` replicates per segment
  uint32_t* d_m1 = nullptr;      // [replicate][tile]
  uint32_t* d_counts = nullptr;  // level-2 count images [tile][batch][sub-tile][17 x 64]
  double* d_partial = nullptr;   // [chunk][rep_pad][e_pad]
  double* d_gram = nullptr;      // [rep_pad][2][e_pad]
  uint32_t* d_chunks = nullptr;  // [chunk][3] = (g, t0, t1)
  uint32_t* d_flags = nullptr;   // [0] = count overflow
  double* d_rows_tmp = nullptr;  // host-API staging
  uint8_t* d_ok_tmp = nullptr;
  uint64_t tmp_reps = 0;

  double* d_hgamma = nullptr;     // Heckman: [2][rep_pad][ks] probit coefficients
  uint32_t* d_hflags = nullptr;   // Heckman: [2][rep_pad] done / failed
  double* d_hpartial = nullptr;   // Heckman: [chunk][rep_pad][values]
  uint32_t* d_hactive = nullptr;  // Heckman: replicates still iterating
  size_t cap_hgamma = 0, cap_hflags = 0, cap_hpartial = 0;
  size_t cap_m1 = 0, cap_partial = 0, cap_gram = 0, cap_chunks = 0, cap_counts = 0;
  void* mm_ws = nullptr;  // Machado-Mata workspace (ob_mm.hip), freed by mm_ws_free
  void (*mm_ws_free)(void*) = nullptr;
  // sharded runs (ob_shard.cpp): this rank's rows, the all-gathered rows, the gather's events
  double* d_shard_rows = nullptr;
  uint8_t* d_shard_ok = nullptr;
  double* d_gather_rows = nullptr;
  uint8_t* d_gather_ok = nullptr;
  size_t cap_shard = 0, cap_gather = 0, cap_shard_ok = 0, cap_gather_ok = 0;
  hipEvent_t gather_ev[2] = {nullptr, nullptr};
  bool gather_timed = false;
  // integer-sliced Gram (ob_gram_i8.hip): digit images per group, pair exponents per chunk
  int oz_state = 0;  // 0 not built, 1 ready, -1 unavailable (the f64 MFMA Gram is used)
  int gram_force = 0;  // 0: i8 when available; 1: f64 MFMA Gram; 2: i8 (ob_debug_gram, OB_GRAM_PATH)
  int oz_n_ct = 0;
  void* d_oz_b[2] = {nullptr, nullptr};
  int32_t* d_oz_pexp = nullptr;
  std::vector<hipEvent_t> seg_events;  // 6 per segment of the last boot run
  ob_timing timing = {};
  bool timing_pending = false;
  hipStream_t last_stream = nullptr;
  int pending_segments = 0;
};

namespace ob {
int engine_point_estimate(ob_panel* p, int ref_mode, double* row, double* resid_b);
int engine_boot(ob_panel* p, uint64_t seed, uint64_t first_rep, uint64_t n_reps, int ref_mode,
                double* d_rows, uint8_t* d_ok, hipStream_t stream);
int engine_collect(ob_panel* p);
int engine_counts(ob_panel* p, uint64_t seed, uint64_t first_rep, uint32_t n_reps, hipStream_t s,
                  uint32_t* nb_rep, uint32_t* rep_pad);
// ob_gram_i8.hip
int oz_prepare(ob_panel* p, const std::vector<uint32_t>& chunks);
int oz_gram(ob_panel* p, const uint32_t* d_chunks, int n_chunks, const uint32_t* counts, uint32_t nb_rep,
            uint32_t rep_pad, uint32_t n_reps, double* partial, hipStream_t s);
}  // namespace ob
