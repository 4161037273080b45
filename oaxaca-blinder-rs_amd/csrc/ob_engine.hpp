// ob_engine.hpp -- device-side state of the bootstrap engine (HBM panel, workspaces, streams).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <vector>

#include "ob_common.hpp"
#include "ob_shard_layout.h"

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
  double* d_pe = nullptr;        // point estimate scratch (unit-Gram partials, Gram, rows, beta, residuals)
  uint8_t* d_pe_ok = nullptr;
  size_t cap_pe = 0, cap_pe_ok = 0;

  double* d_hgamma = nullptr;     // Heckman: [2][rep_pad][ks] probit coefficients
  uint32_t* d_hflags = nullptr;   // Heckman: [2][rep_pad] done / failed
  double* d_hpartial = nullptr;   // Heckman: [chunk][rep_pad][values]
  uint32_t* d_hactive = nullptr;  // Heckman: replicates still iterating
  size_t cap_hgamma = 0, cap_hflags = 0, cap_hpartial = 0;
  size_t cap_m1 = 0, cap_partial = 0, cap_gram = 0, cap_chunks = 0, cap_counts = 0;
  void* mm_ws = nullptr;  // Machado-Mata workspace (ob_mm.hip), freed by mm_ws_free
  void (*mm_ws_free)(void*) = nullptr;
  uint8_t* d_mm_fail = nullptr;  // ob_debug_mm_fail: forced fit failures [2][mm_fail_sims]
  int mm_fail_sims = 0;
  // sharded runs (ob_shard.cpp, buffer layouts in ob_shard_layout.h): this rank's rows, the packed
  // send block, the all-gathered block, host-delivery staging, the gathered columns, the events
  double* d_shard_rows = nullptr;
  uint8_t* d_shard_ok = nullptr;
  double* d_send = nullptr;
  uint8_t* d_send_ok = nullptr;
  double* d_gather_rows = nullptr;
  uint8_t* d_gather_ok = nullptr;
  double* d_deliver_rows = nullptr;
  uint8_t* d_deliver_ok = nullptr;
  double* d_own_rows = nullptr;  // ob_debug_shard_sim: the simulated rank's own shard rows
  size_t cap_shard = 0, cap_gather = 0, cap_shard_ok = 0, cap_gather_ok = 0, cap_send = 0, cap_send_ok = 0;
  size_t cap_deliver = 0, cap_deliver_ok = 0, cap_own = 0;
  std::vector<int32_t> gather_cols;   // gathered row columns, ascending (empty: every column)
  int32_t* d_gather_map = nullptr;    // [row_len] slot of each column or -1, then [nc] the columns
  bool gather_map_ready = false;
  std::vector<hipEvent_t> gather_evs;  // 2 per RCCL gather (start, end) since the last collect
  int pending_gathers = 0;
  // integer-sliced Gram (ob_gram_i8.hip): digit images per group, pair exponents per chunk
  int oz_state = 0;  // 0 not built, 1 ready, -1 unavailable (the f64 MFMA Gram is used)
  int gram_force = 0;  // 0: i8 when available; 1: f64 MFMA Gram; 2: i8 (ob_debug_gram, OB_GRAM_PATH)
  int oz_n_ct = 0;
  void* d_oz_b[2] = {nullptr, nullptr};
  int32_t* d_oz_pexp = nullptr;
  int64_t* d_oz_psum = nullptr;  // [chunk][pair][2]: exponent sum and count of the nonzero |P| (digit choice)
  uint8_t* d_oz_nsl = nullptr;   // [chunk][column tile]: digit slices the Gram runs (6 or 7)
  long long* d_oz_pint = nullptr;  // split wide launches: the halves' int64 slice-group sums
  size_t cap_oz_pint = 0;
  uint8_t* d_oz_pnsl = nullptr;  // [chunk][pair]: 6 = the pair's seventh digit is written as zero
  int oz_tiles6 = 0, oz_tiles = 0;  // (chunk, column tile) blocks on 6 slices / all (read with the meta)
  // exception rows (ob_gram_i8.hip): rows whose magnitude dwarfs their chunk's
  // typical one (or that are not finite) are left out of the digit images and summed in f64
  int8_t* d_oz_dev[2] = {nullptr, nullptr};  // per row: max over columns of (exponent - chunk scale)
  int32_t* d_oz_tile_chunk[2] = {nullptr, nullptr};
  int64_t* d_oz_acc = nullptr;   // [chunk][k1][2]: exponent sums and nonzero counts
  int32_t* d_oz_meta = nullptr;  // oz_meta layout (ob_gram_i8.hip)
  uint32_t* d_oz_exc = nullptr;  // [kOzExcCap] (g << 31 | row), sorted
  double* d_oz_excp = nullptr;   // [kOzExcCap][e_pad] their f64 pair products
  std::vector<int32_t> oz_tile_chunk[2];  // host copies (the async uploads read them)
  hipEvent_t oz_ev[2] = {nullptr, nullptr};
  bool oz_timed = false;  // the last boot run built the digit images (timing.prep_ms)
  int oz_nexc = -1;       // exception rows (-1: not read back yet), their threshold bits
  int oz_bits = 0;
  bool oz_overflow = false;
  // the panel's chunk table (a function of the panel only), uploaded once into d_chunks
  std::vector<uint32_t> chunks;
  bool chunks_ready = false;
  // timing and the overflow flag accumulate over every boot call since the last engine_collect
  // (ob_panel_sync), so a caller may enqueue several calls before it synchronizes
  std::vector<hipEvent_t> seg_events;  // 6 per segment of the boot calls since the last collect
  ob_timing timing = {};
  bool timing_pending = false;
  hipStream_t last_stream = nullptr;
  int pending_segments = 0;
  // cross-stream order of the calls on one panel: every boot shares the panel's scratch buffers,
  // digit images and chunk table, so a boot on another stream than the previous one first waits
  // for order_ev, recorded after the previous call's last kernel (engine_order / engine_mark)
  hipEvent_t order_ev = nullptr;
  hipStream_t order_stream = nullptr;
  // A boot's level-1 and count kernels run on the panel's resample stream (rs_stream), so that they
  // start as soon as the previous call has stopped reading the count images (scratch_ev: after its
  // Gram, or the end of a call of another kind) and overlap that call's reduce / solve / gather;
  // the Gram waits for them (rs_ev). Heckman panels keep one stream (their passes read the images
  // after the Gram).
  hipStream_t rs_stream = nullptr;
  hipEvent_t rs_ev = nullptr, scratch_ev = nullptr;
  bool scratch_recorded = false;
  // Double-buffered resample (option rs_double): a second m1 / count-image pair, so segment k + 1's
  // level 1 and counts (buffer (k + 1) & 1) wait only for the Gram of segment k - 1 (scratch_ev2
  // marks the second buffer's last read) and run under the Gram of segment k. rs_parity is the
  // buffer of the next boot segment.
  uint32_t* d_m1b = nullptr;
  uint32_t* d_countsb = nullptr;
  size_t cap_m1b = 0, cap_countsb = 0;
  hipEvent_t scratch_ev2 = nullptr;
  int rs_parity = 0;
  // Pieced resample (option rs_pieces): level 1 of replicate piece k + 1 on rs_stream beside the
  // count kernel of piece k on cnt_stream (cnt_ev[k]: piece k's level 1 is done)
  hipStream_t cnt_stream = nullptr;
  hipEvent_t cnt_ev[8] = {};
  // Tail stream (option tail_stream): the Gram on g_stream, the reduce / exceptions / solve on
  // t_stream, the caller's stream waiting only for t_ev at the end of the call, so segment k + 1's
  // Gram (partial buffer part_parity) runs under segment k's tail. red_ev[b]: the last reduce that
  // read partial buffer b; user_ev: the caller's stream at the call (the rows buffers); prep_ev: work
  // this call put on the caller's stream before its first Gram (chunk table, digit images).
  hipStream_t g_stream = nullptr, t_stream = nullptr;
  hipEvent_t g_ev = nullptr, t_ev = nullptr, user_ev = nullptr, prep_ev = nullptr, red_ev[2] = {};
  double* d_partialb = nullptr;
  size_t cap_partialb = 0;
  int part_parity = 0;
};

namespace ob {
int engine_point_estimate(ob_panel* p, int ref_mode, double* row, double* resid_b);
int engine_boot(ob_panel* p, uint64_t seed, uint64_t first_rep, uint64_t n_reps, int ref_mode,
                double* d_rows, uint8_t* d_ok, hipStream_t stream);
int engine_collect(ob_panel* p);
// make stream s wait for the panel's previous call when that ran on another stream / mark s as it
int engine_order(ob_panel* p, hipStream_t s);
// scratch: also mark the end of this call's use of d_m1 / d_counts (a boot marks that itself, after
// its last Gram, so its reduce / solve / gather overlap the next boot's resample)
int engine_mark(ob_panel* p, hipStream_t s, bool scratch = true);
int engine_counts(ob_panel* p, uint64_t seed, uint64_t first_rep, uint32_t n_reps, hipStream_t s,
                  uint32_t* nb_rep, uint32_t* rep_pad);
// ob_gram_i8.hip
int oz_prepare(ob_panel* p, hipStream_t s);
int oz_gram(ob_panel* p, const uint32_t* d_chunks, int n_chunks, const uint32_t* counts, uint32_t nb_rep,
            uint32_t rep_pad, uint32_t n_reps, double* partial, hipStream_t s);
// adds the exception rows' f64 terms to the reduced Grams [rep][2][e_pad] of a segment
bool oz_exceptions_pending(const ob_panel* p);
// whether oz_gram runs the wide-tile kernel for a launch of nb_rep 64-replicate batches
bool oz_wide(const ob_panel* p, int n_chunks, uint32_t nb_rep);
int oz_exceptions(ob_panel* p, const uint32_t* counts, uint32_t nb_rep, uint32_t n_reps, double* gram, hipStream_t s);
// after the stream is synchronized: exception count / bits into p->timing, overflow -> error
int oz_collect(ob_panel* p);
void oz_free(ob_panel* p);
// ob_shard.cpp
void shard_free(ob_panel* p);
// ob_shard_kernels.hip (layouts: ob_shard_layout.h)
int shard_pack(const double* rows, const uint8_t* ok, const ob_shard_range& s, int rl, int nc, const int32_t* cols,
               int n_y, double* send, uint8_t* send_ok, hipStream_t st);
int shard_unpack(const double* recv, const uint8_t* recv_ok, const ob_shard_range& s, int world, uint64_t n_reps,
                 int rl, int nc, const int32_t* cmap, int n_y, const double* own, double* rows, uint8_t* ok, hipStream_t st);
}  // namespace ob
