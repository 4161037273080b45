// ob_shard_layout.h -- where a sharded run's rows live between the shard computation, the RCCL
// all-gather and the delivery (ob_shard.cpp). Pure host arithmetic, no HIP: the CPU/ASan suite
// (tests/asan/host_asan.cpp) drives exactly these functions through a simulated gather.
//
// Replicates [first_rep, first_rep + n) split into W shards of per = ceil(n / W): rank r runs ids
// [first_rep + lo_r, first_rep + lo_r + count_r) with lo_r = min(r per, n) and count_r =
// min(n, lo_r + per) - lo_r, so the last shards may be short or empty (n < W).
//
// Buffers, with nc = the gathered row columns (all row_len of them by default; the aggregation's
// component columns when the panel narrows the gather) and n_y outcome blocks:
//   shard rows   engine_boot's output     [t][count][row_len]   (outcome-major blocks of count)
//   send         packed, padded           [t][per][nc]          (rows past count: zeros, ok 0)
//   recv         ncclAllGather of send    [t][W per][nc]        rank r's block at (t W + r) per nc
//   delivered    the caller's rows        [t][n][row_len]       replicate j of outcome t is recv
//                                                               row t W per + j (j < n): rank
//                                                               j / per, position j % per
// A column outside the gathered set is delivered from this rank's own shard rows for its own
// replicates and as NaN for the other ranks' replicates.
#pragma once
#include <stddef.h>
#include <stdint.h>

#if defined(__HIPCC__)
#define OB_SL_HD __attribute__((host, device)) static inline
#else
#define OB_SL_HD static inline
#endif

struct ob_shard_range {
  uint64_t per;    // shard stride: ceil(n / W)
  uint64_t lo;     // this rank's first replicate, relative to first_rep
  uint64_t first;  // first_rep + lo
  uint64_t count;  // replicates this rank computes (0 for an empty tail shard)
};

OB_SL_HD ob_shard_range ob_shard_of(uint64_t first_rep, uint64_t n_reps, int rank, int world) {
  ob_shard_range s;
  s.per = world > 0 ? (n_reps + (uint64_t)world - 1) / (uint64_t)world : n_reps;
  const uint64_t lo = (uint64_t)rank * s.per < n_reps ? (uint64_t)rank * s.per : n_reps;
  s.lo = lo;
  s.first = first_rep + lo;
  s.count = (n_reps < lo + s.per ? n_reps : lo + s.per) - lo;
  return s;
}

// shard rows: replicate i (< count) of outcome t, column c
OB_SL_HD size_t ob_shard_row_off(const ob_shard_range& s, int t, uint64_t i, int row_len, int c) {
  return ((size_t)t * s.count + i) * (size_t)row_len + (size_t)c;
}
OB_SL_HD size_t ob_shard_ok_off(const ob_shard_range& s, int t, uint64_t i) { return (size_t)t * s.count + i; }

// send buffer: position i (< per) of outcome t, gathered column slot q (< nc)
OB_SL_HD size_t ob_send_off(const ob_shard_range& s, int t, uint64_t i, int nc, int q) {
  return ((size_t)t * s.per + i) * (size_t)nc + (size_t)q;
}
OB_SL_HD size_t ob_send_ok_off(const ob_shard_range& s, int t, uint64_t i) { return (size_t)t * s.per + i; }
// elements one rank contributes per outcome (the all-gather's count)
OB_SL_HD size_t ob_send_elems(const ob_shard_range& s, int nc) { return (size_t)s.per * (size_t)nc; }

// recv buffer: where rank r's send block of outcome t lands, and where replicate j (< n) sits
OB_SL_HD size_t ob_recv_block_off(const ob_shard_range& s, int world, int t, int r, int nc) {
  return (((size_t)t * (size_t)world + (size_t)r) * s.per) * (size_t)nc;
}
OB_SL_HD size_t ob_recv_off(const ob_shard_range& s, int world, int t, uint64_t j, int nc, int q) {
  return ((size_t)t * (size_t)world * s.per + j) * (size_t)nc + (size_t)q;
}
OB_SL_HD size_t ob_recv_ok_off(const ob_shard_range& s, int world, int t, uint64_t j) {
  return (size_t)t * (size_t)world * s.per + j;
}

// delivered rows: replicate j of outcome t, column c
OB_SL_HD size_t ob_deliver_off(uint64_t n_reps, int t, uint64_t j, int row_len, int c) {
  return ((size_t)t * n_reps + j) * (size_t)row_len + (size_t)c;
}
