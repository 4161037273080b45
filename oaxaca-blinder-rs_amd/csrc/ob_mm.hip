// ob_mm.hip -- Machado-Mata on the GPU (QuantileDecompositionBuilder, quantile_decomposition.rs:21-445).
//
// A pass (run_single_pass, :173-279) solves `simulations` quantile regressions per group at the
// MM-1 quantiles (csrc/ob_spec.h), draws one row per group per successful simulation, and takes
// empirical quantiles of the three predictions. The reference solves each QR as a sparse LP with
// Clarabel (math/quantile_regression.rs:22-129); here every fit of a replicate runs at once as a
// Mehrotra predictor-corrector interior-point method on the bounded dual LP
//     max y'x  s.t.  X'x = (1 - tau) X'c,  0 <= x <= c        (c = the replicate's row counts)
// whose equality multipliers are the QR coefficients beta (tools/qr_ipm_proto.py is the numpy
// statement of the same iteration). The start is primal and dual feasible (x = (1 - tau) c, beta =
// weighted OLS, z - w = X beta - y), so every iteration only drives the complementarity gap.
//
// Layout: lane = (fit, list row) in the A-fragment shape of v_mfma_f64_16x16x4 (below); the IPM
// state (x, z, w) is stored per (fit, entry of the replicate's nonzero-row list), so every pass
// streams it as dense 512-byte wave loads (state_at). Per iteration, three passes over the rows, each writing per-(chunk, fit) partials that are
// reduced in a fixed chunk order (bitwise reproducible), and one-wave-per-fit solves:
//   mm_assemble<K>   (apply the last step,) M = X'QX, X'Q r, gap, objective
//   mm_affine<K>     affine direction: step-length bounds, mu_aff terms, corrector right-hand sides
//   mm_final<K>      corrector direction, step-length bounds; stores the direction
//   mm_finish        per replicate: successful fits in quantile order, MM-1 row picks (through
//                    the count images for resamples), predictions, LDS bitonic sorts, quantiles
//
// Row reduction (large groups; Portnoy & Koenker 1997, "the Gaussian hare and the Laplacian
// tortoise"; tools/qr_pk_proto.py). Phase 1 solves every fit on a fixed subsample (every 8th row,
// relative gap 1e-6) -> beta_hat. mm_band_kernel takes the residual band [lo, hi] of each fit at
// the tau -/+ delta quantiles of 4096 sampled residuals (delta = 4 sqrt(tau (1 - tau) K / m) +
// 0.01). mm_classify_kernel keeps, per 64-fit block, the rows inside some fit's band and fixes the
// others at their optimal bound (x_i = c_i above the band, 0 below), folding them into each fit's
// right-hand side b = (1 - tau) X'c - sum_above c_i x_i. Phase 2 solves the reduced LPs
// (X'x = b, infeasible centred start). mm_verify_kernel checks every fixed row's residual sign at
// the reduced optimum; a fit with a wrong sign (or a phase-2 failure) is solved again on all rows
// (phase 3). When every sign holds, the reduced optimum is the full LP's optimum.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "ob_device.hpp"
#include "ob_engine.hpp"
#include "ob_mm.hpp"
#include "ob_options.hpp"
#include "ob_spec.h"

namespace {

constexpr double kEta = 0.99995;  // fraction of the distance to the boundary per step
constexpr double kTol = 1e-12;    // relative duality gap at convergence
constexpr uint32_t kDone = 1u, kFailed = 2u, kRetry = 4u;
// Chunk geometry (a function of the panel only: determinism). A chunk's nonzero-count rows form one
// list (per fit block after the reduction); a block walks one list.
constexpr uint32_t kRc = 2048;       // rows per chunk without the row reduction
constexpr uint32_t kRcF = 8192;      // with it: the full and reduced lists (longer walks, 4x fewer partials)
constexpr uint32_t kCap = 8192;      // list capacity bound (LDS copies of a list)
constexpr uint32_t kSubStride = 8;   // phase 1 of the row reduction: every 8th row ...
constexpr uint32_t kRc1 = 4096;      // ... in chunks of 4096 rows (512 candidates: short walks)
static_assert(kRc <= kCap && kRcF <= kCap && kRc1 / kSubStride <= kCap, "lists fit the LDS copies");
constexpr double kPhase1Tol = 1e-4;  // phase-1 relative gap (beta_hat only centres the bands; 1e-6 until round 4)
constexpr int kFitStride = 16;       // phase 1 solves every 16th quantile (tau order) and the last ...
constexpr int kFitStrideMin = 64;    // ... when a group has at least 64 simulations; the rest interpolate
constexpr double kBandKappa = 3.5;   // band half-width in rank units: kappa sqrt(tau (1 - tau) K / m) + kBand0
constexpr double kBand0 = 0.01;      // (options mm_kappa, mm_band0: tuning knobs)
constexpr int kBandSamples = 4096;   // residuals per fit behind its band quantiles
// Start offsets of the IPM's z/w (the shifted start's 0.01 (1 + rms) offset, FS_DELTA, times dscale):
constexpr double kDelta1 = 3.0;      // phase 1: 3x FS_DELTA (48 -> 36 iterations at configs[4])
constexpr double kDelta2 = 2.0;      // phases 2/3 (reduced_round's a2, built from the unscaled args):
                                     // 2x FS_DELTA, not 2x phase 1's offset; all fits converge 3
                                     // iterations sooner (sweeps: profiles/r04_mm_delta.txt)
// These tuning defaults (phase-1 tolerance, fit stride, band width, start offsets) move iteration
// counts and which rows the reduction keeps, not the optimum a converged fit reaches (the sign
// verification keeps the reduced optimum the full LP's). That holds only while every fit converges:
// a fit pushed past kMmMaxIter is dropped like a failed solve_qr and changes the MM quantiles.
// tests/test_gpu_fullsize.py::test_configs4_machado_mata_full_size checks that every fit of the point
// pass and of two replicates converges at configs[4] under these defaults.

enum { FS_TAU, FS_GAP, FS_OBJ, FS_MU, FS_SIGMU, FS_AP, FS_AD, FS_NACT, FS_DELTA, FS_LO, FS_HI, FS_EXT, FS_OBJFIX, kFs };

// Assemble partial layout per fit: NP pairs of X'QX, X'Q r (K), gap, objective, X'x (K; phase 2).
__host__ __device__ constexpr int nv_asm(int K) { return K * (K + 1) / 2 + 2 * K + 2; }
// Classify partial layout per fit: sum_above c x (K), sum_all c x (K), sum_above c y, kept rows.
__host__ __device__ constexpr int nv_cls(int K) { return 2 * K + 2; }

#define MM_OK(expr)                                                                      \
  do {                                                                                   \
    hipError_t e_ = (expr);                                                              \
    if (e_ != hipSuccess)                                                                \
      return ob::fail(OB_E_HIP, "HIP error %s at %s:%d", hipGetErrorString(e_), __FILE__, \
                      __LINE__);                                                         \
  } while (0)

struct MmArgs {
  const double* cols[2];  // [col][ld]: x_1..x_p, y (intercept implicit)
  int64_t ld[2];
  uint32_t n[2];
  uint32_t tiles0;
  int p;
  int S, S_pad;
  uint32_t n_rb;           // replicates in this batch
  uint32_t rep0;           // MM-1 replicate id of slot 0 (OB_MM_POINT_REP: every row once)
  uint32_t seg0;           // slot 0's position in the count-image segment
  const uint32_t* counts;  // level-2 count images (ob_engine.hpp layout); null for the point
  const uint32_t* m1;      // level-1 tile counts [replicate][tile]
  uint32_t nb_rep, rep_pad;
  uint32_t nch[2];
  size_t rep_rows;         // n0 + n1: state rows per replicate
  double *x, *z, *w;                 // [slot][row (A then B)][S_pad]
  double *beta, *bprev, *dba, *db;   // [fit][K]; bprev: beta the last directions were taken at
  double* L;                         // [fit][K*K]
  double* fs;                        // [fit][kFs]
  uint32_t* fstat;                   // [fit]
  double* partial;                   // [slot][chunk (A then B)][S_pad][nv]
  double* red;                       // [slot][group][S_pad][nv]
  uint32_t* active;
  unsigned long long* active_rows;   // live (fit, row) pairs of the next passes
  uint32_t* tprefix;                 // [slot][group][tiles + 1] (finish kernel scratch)
  uint32_t* lane_of;                 // [slot][group][simulation] -> fit lane (lanes in ascending tau)
  uint32_t* rowlist;                 // [slot][chunk (A then B)][cap] nonzero-count rows (mm_rows_kernel)
  uint32_t* nrows;                   // [slot][chunk] list lengths
  uint32_t rc;                       // rows per chunk of this phase (kRc; kRcF / kRc1 with the reduction)
  uint32_t stride;                   // mm_rows_kernel: every stride-th row (phase 1) or all (1)
  uint32_t cap;                      // list capacity: rc / stride entries (a multiple of 256)
  uint32_t block_lists;              // lists per (slot, chunk, fit block) (phase 2/3) instead of per chunk
  int rp;                            // X'x = b per fit (phase 2/3): primal residual in the solves
  double tol;                        // relative duality gap at convergence
  int trace;                         // option mm_trace: device-side printf of rare events
  uint32_t* blist;                   // mm_classify_kernel output: [slot][chunk][fit block][cap]
  uint32_t* bnrows;                  // [slot][chunk][fit block]
  double *bvec, *rpv, *bhat;         // [fit][K]: b, b - X'x of the iterate, phase-1 beta (band centres)
  uint32_t* samp;                    // [slot][group][2][kBandSamples]: sampled rows, counts
  uint32_t* nsamp;                   // [slot][group]
  double* gchol;                     // [slot][group][K * K + 1]: Cholesky factor of the phase-1 OLS Gram, sum c
  double* lev;                       // [slot][chunk][cap]: leverage sqrt(n x_i' G^-1 x_i) per full-list entry
  uint32_t* xmask;                   // [slot][chunk][fit block][cap / 32]: rows added to the block's list
                                     // after a wrong-signed verification (mm_verify)
  uint32_t key0, key1;
  int n_q;
  const double* quantiles;
  double* rows;  // [slot][3 n_q]
  uint8_t* ok;
  // ob_debug_mm_fail (tests only): fit (g, s) of pass `rep` counts as failed when bit (rep & 7) of
  // fail_mask[g * fail_sims + s] is set -- the reference's dropped Clarabel fits, on demand
  const uint8_t* fail_mask;
  int fail_sims;
  double dscale;  // scale of the start's z/w offset (0: 1): phase 1 OB_MM_DELTA1, phases 2/3 kDelta2
  int list_stat;  // OB_MM_TRACE: the classify pass counts block-list entries against each wave's own needs
};

// OB_MM_TRACE statistics of the classify pass: [0] (wave, block-list entry) pairs, [1] those whose
// entry some fit of the wave keeps itself (what per-wave lists would walk)
__device__ unsigned long long g_mm_list_stat[2];

__device__ __forceinline__ size_t fit_index(const MmArgs& a, uint32_t slot, uint32_t g, int s) {
  return ((size_t)slot * 2 + g) * a.S_pad + s;
}

// Count of `row` of group g in replicate slot `slot` (1 for the point estimate).
__device__ __forceinline__ uint32_t row_count(const MmArgs& a, uint32_t slot, uint32_t g, uint32_t row) {
  if (!a.counts) return 1u;
  const uint32_t pos = a.seg0 + slot;
  const size_t tt = (g ? a.tiles0 : 0u) + (row >> 8);
  const uint32_t word =
      a.counts[((tt * a.nb_rep + (pos >> 6)) * 4 + ((row & 255u) >> 6)) * kCimgWords + (pos & 63u) * kCimgStride +
               ((row & 63u) >> 2)];
  return (word >> ((row & 3u) * 8u)) & 255u;
}

// Each pass walks a chunk's rows through a list of the replicate's nonzero-count rows
// (mm_rows_kernel, once per batch: the counts do not change across iterations). Block = 4
// waves x 16 fits (fit = lane & 15) on one chunk; a wave step takes 4 list rows (row = lane >> 4),
// so a lane holds one (fit, row) pair per step -- the A-fragment layout of v_mfma_f64_16x16x4
// (m = fit, k = row), and X'QX / X'Q r / X'q rho are MFMAs with B = the rows' pair products or
// values from LDS. The rows' design values are gathered 64 list rows at a time into
// double-buffered LDS (loaded one sub-tile ahead); the (fit, row) state streams into registers
// kRing steps ahead of use, across sub-tile seams.
// LDS stride of a staged row: [1, x_1..x_p, 0.., y at S - 2, 0 at S - 1]; 18 doubles up to K = 16
// (odd in 8-byte units: conflict-free row reads), 34 up to K = 32.
template <int K>
struct Xs {
  static_assert(K >= 1 && K <= 32, "Machado-Mata panels take at most 32 columns");
  static constexpr int S = K <= 16 ? 18 : 34;
  static constexpr int Y = S - 2, Z = S - 1;
  static constexpr int Stage = (64 * S + 255) / 256;  // staging values per thread (kSub = 64 rows)
  static constexpr int NXB = (K + 15) / 16;           // 16-column blocks of X' v products
};
constexpr int kSub = 64;    // list rows per staged sub-tile (16 wave steps of 4 rows)
#ifndef OB_MM_RING
#define OB_MM_RING 4
#endif
#ifndef OB_MM_RING_A
#define OB_MM_RING_A 4
#endif
#ifndef OB_MM_PASS_BLOCKS
#define OB_MM_PASS_BLOCKS 3  // affine / final blocks per CU the compiler sizes registers for (K <= 16)
#endif
constexpr int kRing = OB_MM_RING;     // wave steps of state in flight (affine / final)
constexpr int kRingA = OB_MM_RING_A;  // the same for the assemble pass (its fragments sit in LDS to make room)
constexpr int kStoreAt = 4; // step after which the next sub-tile's staged values are written
typedef double mm_d4 __attribute__((ext_vector_type(4)));
static_assert(16 % kRing == 0, "ring slots are static per unrolled step");

// Nonzero-count rows of each (slot, chunk) in ascending order: (row - chunk start) << 8 | count.
// A chunk spans a.rc rows, of which every a.stride-th is a candidate (a.cap candidates: a.cap / 256
// consecutive ones per thread, counted, scanned, then written).
__global__ __launch_bounds__(256) void mm_rows_kernel(const MmArgs a) {
  __shared__ uint32_t scan[256];
  const uint32_t gch = blockIdx.x, slot = blockIdx.z, nch = a.nch[0] + a.nch[1];
  const uint32_t g = gch >= a.nch[0] ? 1u : 0u;
  const uint32_t r0 = (gch - (g ? a.nch[0] : 0u)) * a.rc, nr = min(a.n[g] - r0, a.rc);
  const uint32_t per = a.cap / 256, i0 = threadIdx.x * per;
  uint32_t k = 0;
  for (uint32_t i = 0; i < per; ++i) {
    const uint32_t off = (i0 + i) * a.stride;
    k += (off < nr && row_count(a, slot, g, r0 + off) != 0u) ? 1u : 0u;
  }
  scan[threadIdx.x] = k;
  __syncthreads();
  for (int d = 1; d < 256; d <<= 1) {  // inclusive scan of the per-thread counts
    const uint32_t v = (int)threadIdx.x >= d ? scan[threadIdx.x - d] : 0u;
    __syncthreads();
    scan[threadIdx.x] += v;
    __syncthreads();
  }
  uint32_t o = scan[threadIdx.x] - k;
  uint32_t* L = a.rowlist + ((size_t)slot * nch + gch) * a.cap;
  for (uint32_t i = 0; i < per; ++i) {
    const uint32_t off = (i0 + i) * a.stride;
    const uint32_t c = off < nr ? row_count(a, slot, g, r0 + off) : 0u;
    if (c) L[o++] = (off << 8) | c;
  }
  if (threadIdx.x == 255) a.nrows[(size_t)slot * nch + gch] = scan[255];
}

struct Blk {
  uint32_t g, gch, slot, fb, r0, n_ent;
  int wave, lane, fl, rl, s;
  size_t F, sb;  // fit index; state index of (this lane's fit, list entry 0)
  bool live, wave_live, any;  // any: some fit of the block is live (else the block exits)
  const double* X;
  int64_t ld;
};

// Block context; copies the chunk's row list into lst (caller syncs).
__device__ __forceinline__ Blk blk_ctx(const MmArgs& a, uint32_t* lst, bool all_live) {
  Blk b;
  b.lane = threadIdx.x & 63;
  b.wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  b.fl = b.lane & 15;
  b.rl = b.lane >> 4;
  b.gch = blockIdx.x;
  b.fb = blockIdx.y;
  b.slot = blockIdx.z;
  b.g = b.gch >= a.nch[0] ? 1u : 0u;
  b.r0 = (b.gch - (b.g ? a.nch[0] : 0u)) * a.rc;
  b.s = (int)b.fb * 64 + b.wave * 16 + b.fl;
  b.F = fit_index(a, b.slot, b.g, b.s);
  b.live = all_live ? b.s < a.S_pad : (b.s < a.S && !(a.fstat[b.F] & (kDone | kFailed)));
  b.wave_live = __ballot(b.live) != 0;
  b.X = a.cols[b.g];
  b.ld = a.ld[b.g];
  const size_t li = (size_t)b.slot * (a.nch[0] + a.nch[1]) + b.gch;
  b.sb = (li * (a.S_pad / 64) + b.fb) * ((size_t)a.cap * 64) + b.wave * 64 + b.fl;
  b.any = __syncthreads_or(b.live) != 0;
  const size_t lli = a.block_lists ? li * (a.S_pad / 64) + b.fb : li;  // this block's row list
  b.n_ent = b.any ? a.nrows[lli] : 0u;
  const uint32_t* L = a.rowlist + lli * a.cap;
  for (uint32_t i = threadIdx.x; i < b.n_ent; i += 256) lst[i] = L[i];
  return b;
}

// Sub-tile t's design values -> registers (unconditional loads at clamped addresses, then a
// select: no branch around a load) ...
template <int K>
__device__ __forceinline__ void xs_load(const MmArgs& a, const Blk& b, const uint32_t* lst, uint32_t t,
                                        double (&v)[Xs<K>::Stage]) {
  constexpr int S = Xs<K>::S;
#pragma unroll
  for (int j = 0; j < Xs<K>::Stage; ++j) {
    const int i = threadIdx.x + 256 * j;
    const int rr = i / S, col = i % S;
    const uint32_t e = t * kSub + rr;
    const bool in = i < kSub * S && e < b.n_ent;
    const uint32_t row = b.r0 + (lst[min(e, b.n_ent - 1)] >> 8);
    const int src = (col >= 1 && col < K) ? col - 1 : (col == Xs<K>::Y ? a.p : 0);
    const double x = b.X[(size_t)src * b.ld + row];
    v[j] = !in ? 0.0 : (col == 0 ? 1.0 : ((col < K || col == Xs<K>::Y) ? x : 0.0));
  }
}
// ... -> LDS.
template <int K>
__device__ __forceinline__ void xs_store(double* xs, const double (&v)[Xs<K>::Stage]) {
#pragma unroll
  for (int j = 0; j < Xs<K>::Stage; ++j) {
    const int i = threadIdx.x + 256 * j;
    if (i < kSub * Xs<K>::S) xs[i] = v[j];
  }
}

// State index of this lane's fit at list entry e (clamped to the list). The state is stored by
// list entry, not by row, in units of 4 entries x the block's 64 fits: [slot][chunk][fit block]
// [entry / 4][wave][entry % 4][fit % 16], so a wave step (4 entries x 16 fits) is one contiguous
// 512-byte load and a block streams one dense region per pass.
__device__ __forceinline__ size_t state_at(const Blk& b, uint32_t e) {
  e = min(e, b.n_ent - 1);
  return b.sb + (size_t)(e >> 2) * 256 + (e & 3u) * 16;
}

// Sum (or min) over the 4 row lanes of each fit (lanes fl, fl + 16, fl + 32, fl + 48).
__device__ __forceinline__ double rows_sum(double v) {
  v += __shfl_xor(v, 16);
  return v + __shfl_xor(v, 32);
}
__device__ __forceinline__ double rows_min(double v) {
  v = fmin(v, __shfl_xor(v, 16));
  return fmin(v, __shfl_xor(v, 32));
}

// Per-fit vectors as MFMA B fragments: f[kb] = v[fit][4 kb + rl] (zero past K or for dead lanes).
template <int K>
__device__ __forceinline__ void bfrag(const double* v, const Blk& b, bool on, double (&f)[(K + 3) / 4]) {
#pragma unroll
  for (int kb = 0; kb < (K + 3) / 4; ++kb) {
    const int k = 4 * kb + b.rl;
    f[kb] = (on && k < K) ? v[b.F * K + k] : 0.0;
  }
}

// x_i . v for the 16 rows of step group G (steps 4G..4G+3 of a sub-tile) against each lane's fit,
// on f64 MFMA: A = the staged rows (m = row 16G + fl, k), B = the fragments (k, n = fit). D element
// i is this lane's row of step 4G + i (row 16G + rl + 4i), the (fit, row) pair the step holds.
template <int K, int NV>
__device__ __forceinline__ void group_dots(const double* X, int G, const Blk& b,
                                           const double (&f)[NV][(K + 3) / 4], mm_d4 (&d)[NV]) {
#pragma unroll
  for (int v = 0; v < NV; ++v) d[v] = (mm_d4){0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int kb = 0; kb < (K + 3) / 4; ++kb) {
    const double av = X[(16 * G + b.fl) * Xs<K>::S + 4 * kb + b.rl];
#pragma unroll
    for (int v = 0; v < NV; ++v) d[v] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, f[v][kb], d[v], 0, 0, 0);
  }
}

// group_dots with the fragments read from LDS ([vector][fit of the block][K + 1], odd stride).
template <int K, int NV>
__device__ __forceinline__ void group_dots_lds(const double* X, int G, const Blk& b, const double* fbl,
                                               mm_d4 (&d)[NV]) {
#pragma unroll
  for (int v = 0; v < NV; ++v) d[v] = (mm_d4){0.0, 0.0, 0.0, 0.0};
  const int fit = b.wave * 16 + b.fl;
#pragma unroll
  for (int kb = 0; kb < (K + 3) / 4; ++kb) {
    const double av = X[(16 * G + b.fl) * Xs<K>::S + 4 * kb + b.rl];
    const int k = 4 * kb + b.rl;
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const double bv = k < K ? fbl[(v * 64 + fit) * (K + 1) + k] : 0.0;
      d[v] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, d[v], 0, 0, 0);
    }
  }
}

// 1/v within ~1 ulp without the IEEE division sequence (div_scale / div_fmas / div_fixup):
// v_rcp_f64 and two Newton steps. The operands are normal numbers (interior iterates, nonzero
// direction components), so the scaling that sequence guards against is never needed.
__device__ __forceinline__ double mm_rcp(double v) {
  double r = __builtin_amdgcn_rcp(v);
  r = fma(fma(-v, r, 1.0), r, r);
  return fma(fma(-v, r, 1.0), r, r);
}

// The box variable x in [0, c] is stored by its distance to the nearer bound: d = x while x <= s,
// d = -s otherwise (s = c - x, the upper slack). Both x and s then keep full relative precision
// near either bound; derived as c - x, s lost it: a 500k-row fit whose rows sat at x = c (1 - 1e-16)
// got s = 0 in a few rows, and the iteration's next direction turned NaN (configs[4],
// tests/test_gpu_fullsize.py). Where the representation switches (x = s = c/2) the subtraction is
// exact (Sterbenz).
// (By value, with selects: the by-reference form left the assemble pass's x, s in a stack slot.)
struct XS {
  double x, s;
};
__device__ __forceinline__ XS xs_decode(double d, double c) {
  const bool lo = d >= 0.0;
  const double m = lo ? d : -d;  // the precise one
  const double o = c - m;
  return {lo ? m : o, lo ? o : m};
}
__device__ __forceinline__ double xs_encode(XS v) { return v.x <= v.s ? v.x : -v.s; }
// x += t from the precise (x, s): the smaller of the two takes the step, the other follows.
__device__ __forceinline__ XS xs_step(XS v, double c, double t) {
  const bool lo = v.x <= v.s;
  const double m = lo ? v.x + t : v.s - t;
  const double o = c - m;
  return {lo ? m : o, lo ? o : m};
}

// Per-row affine direction from the current state (shared by mm_affine, mm_final and the step
// replay of mm_assemble); xd is the stored (bound-distance) x.
struct Affine {
  double xv, zv, wv, sv, ix, is, q, r, dxa, dza, dwa;  // ix = 1/x, is = 1/s (divisions shared)
};

// xb = x_i . beta, xd = x_i . dba (group_dots).
__device__ __forceinline__ Affine affine_row(double xv, double zv, double wv, double c, double y, double xb,
                                             double xd) {
  Affine f;
  const XS v = xs_decode(xv, c);
  f.xv = v.x;
  f.sv = v.s;
  f.zv = zv;
  f.wv = wv;
  f.r = y - xb;
  f.ix = mm_rcp(f.xv);
  f.is = mm_rcp(f.sv);
  f.q = mm_rcp(f.zv * f.ix + f.wv * f.is);
  f.dxa = f.q * (f.r - xd);
  f.dza = -f.zv - f.zv * f.dxa * f.ix;
  f.dwa = -f.wv + f.wv * f.dxa * f.is;
  return f;
}

// Per-row corrector direction (mm_final for the step bounds; mm_assemble replays it to take the
// step, so the direction is never stored). xd = x_i . db (group_dots).
struct Corrector {
  double dx, dz, dw;
};
__device__ __forceinline__ Corrector corrector_row(const Affine& f, double xd, double sigmu) {
  Corrector o;
  const double rho = f.r - f.dxa * (f.dwa * f.is + f.dza * f.ix) + sigmu * (f.ix - f.is);
  o.dx = f.q * (rho - xd);
  const double rxz = sigmu - f.xv * f.zv - f.dxa * f.dza;
  const double rsw = sigmu - f.sv * f.wv + f.dxa * f.dwa;
  o.dz = (rxz - f.zv * o.dx) * f.ix;
  o.dw = (rsw + f.wv * o.dx) * f.is;
  return o;
}

// mm_assemble: mode 0: weighted OLS of the replicate (q = c, rho = y) -> M, X'Cy, sum c y^2, n_act;
// mode 1: start point (x = (1 - tau) c, z/w from the OLS residual) + assemble; mode 2 (STEP): replay
// the last corrector direction from (bprev, dba, db, sigma mu) and take the step (x += ap dx,
// z += ad dz, w += ad dw) + assemble; mode 3: centred start at beta (phase 2/3 of the row
// reduction: z/w from the residual, x = c w / (z + w), so x z = s w) + assemble. Only x, z, w
// cross HBM. M = X'QX and X'Q r on f64 MFMA: column block cb < NCB has B = x_i x_j of pair
// columns cb*16.. (ob_pair_index order), block NCB has A = q r and B = x; with a.rp, the start
// point's X'x too (a Newton step keeps X'dx = b - X'x, so afterwards b - X'x shrinks by 1 - ap
// per step and is tracked per fit, not reassembled).
template <int K, bool STEP>
__global__ __launch_bounds__(256, K <= 16 ? 2 : 1) void mm_assemble_mfma_kernel(const MmArgs a, int mode) {
  constexpr int NP = K * (K + 1) / 2, NV = nv_asm(K);
  constexpr int NCB = (NP + 15) / 16;
  constexpr int NXB = Xs<K>::NXB;  // X'Q r column blocks
  __shared__ __attribute__((aligned(16))) double xs[2][kSub * Xs<K>::S];
  __shared__ uint32_t lst[kCap];
  const Blk b = blk_ctx(a, lst, mode == 0);
  if (!b.any) return;  // partials of dead fits are never reduced
  constexpr int NDOT = STEP ? 3 : 1;  // x_i . (bprev, dba, db) or x_i . beta
  // the per-fit vectors live in LDS (registers go to a deeper state prefetch): [vector][fit][K + 1]
  __shared__ double fbl[NDOT * 64 * (K + 1)];
  {
    const double* src[3] = {STEP ? a.bprev : a.beta, a.dba, a.db};
    const int fit = b.wave * 16 + b.fl;
#pragma unroll
    for (int v = 0; v < NDOT; ++v)
      for (int k = b.rl; k < K; k += 4) fbl[(v * 64 + fit) * (K + 1) + k] = (b.live && mode) ? src[v][b.F * K + k] : 0.0;
  }
  mm_d4 dots[NDOT];
  double tau = 0.0, ap = 0.0, ad = 0.0, delta = 0.0, sigmu = 0.0;
  if (b.live && mode) {
    tau = a.fs[b.F * kFs + FS_TAU];
    ap = a.fs[b.F * kFs + FS_AP];
    ad = a.fs[b.F * kFs + FS_AD];
    delta = a.fs[b.F * kFs + FS_DELTA] * (a.dscale > 0.0 ? a.dscale : 1.0);
    sigmu = a.fs[b.F * kFs + FS_SIGMU];
  }
  // B-operand columns (i, j) of this lane (n = fl) per pair block, packed i | j << 8; the zero
  // slot past the last pair
  uint32_t pp[NCB];
#pragma unroll
  for (int cb = 0; cb < NCB; ++cb) {
    const int e = cb * 16 + b.fl;
    pp[cb] = Xs<K>::Z | (Xs<K>::Z << 8);
    if (e < NP) {
      int i = 0, e0 = 0;
      while (e >= e0 + (K - i)) {
        e0 += K - i;
        ++i;
      }
      pp[cb] = (uint32_t)i | (uint32_t)(i + (e - e0)) << 8;
    }
  }
  mm_d4 acc[NCB + NXB];
#pragma unroll
  for (int cb = 0; cb < NCB + NXB; ++cb) acc[cb] = (mm_d4){0.0, 0.0, 0.0, 0.0};
  mm_d4 axx[NXB];  // X'x (a.rp)
#pragma unroll
  for (int xb = 0; xb < NXB; ++xb) axx[xb] = (mm_d4){0.0, 0.0, 0.0, 0.0};
  const bool rp = !STEP && a.rp != 0;  // X'x of the start point (later steps track b - X'x exactly)
  double gap = 0.0, obj = 0.0;
  __syncthreads();  // lst
  const uint32_t nsub = (b.n_ent + kSub - 1) / kSub;
  if (__syncthreads_or(b.live) && nsub) {
    double stg[Xs<K>::Stage];
    xs_load<K>(a, b, lst, 0, stg);
    xs_store<K>(xs[0], stg);
    double rx[kRingA], rz[kRingA], rw[kRingA];
    auto load = [&](int k, uint32_t e) {
      if (STEP) {
        const size_t si = state_at(b, e);
        rx[k] = a.x[si];
        rz[k] = a.z[si];
        rw[k] = a.w[si];
      }
    };
#pragma unroll
    for (int k = 0; k < kRingA; ++k) load(k, 4 * k + b.rl);
    __syncthreads();
    for (uint32_t t = 0; t < nsub; ++t) {
      const double* X = xs[t & 1];
      xs_load<K>(a, b, lst, t + 1, stg);
      auto step = [&](int j) {
          if ((j & 3) == 0 && mode) group_dots_lds<K, NDOT>(X, j >> 2, b, fbl, dots);
          const int k = j % kRingA;
          const double cx = rx[k], cz = rz[k], cw = rw[k];
          const uint32_t e = t * kSub + 4 * j + b.rl;
          load(k, e + 4 * kRingA);
          const bool valid = e < b.n_ent && b.live;
          const double c = valid ? (double)(lst[e] & 255u) : 0.0;
          const double* xr = X + (4 * j + b.rl) * Xs<K>::S;
          const double y = xr[Xs<K>::Y];
          double q = 0.0, qr = 0.0, xq = 0.0;
          if (valid) {
            if (mode == 0) {
              q = c;
              qr = c * y;
              gap += c * y * y;
              obj += 1.0;
            } else {
              double xv, sv, zv, wv, r;
              if (!STEP) {
                r = y - dots[0][j & 3];
                zv = fmax(-r, 0.0) + delta;
                wv = fmax(r, 0.0) + delta;
                if (mode == 3) {
                  const double iz = c / (zv + wv);
                  xv = wv * iz;
                  sv = zv * iz;
                } else {
                  xv = (1.0 - tau) * c;
                  sv = tau * c;
                }
              } else {
                const Affine f = affine_row(cx, cz, cw, c, y, dots[0][j & 3], dots[NDOT > 1 ? 1 : 0][j & 3]);
                const double xdb = dots[NDOT > 2 ? 2 : 0][j & 3];
                const Corrector d = corrector_row(f, xdb, sigmu);
                const XS v = xs_step({f.xv, f.sv}, c, ap * d.dx);
                xv = v.x;
                sv = v.s;
                zv = cz + ad * d.dz;
                wv = cw + ad * d.dw;
                r = f.r - ad * xdb;  // y - x_i . (bprev + ad db)
              }
              const size_t si = state_at(b, e);
              a.x[si] = xs_encode({xv, sv});
              a.z[si] = zv;
              a.w[si] = wv;
              q = xv * sv * mm_rcp(zv * sv + wv * xv);  // 1 / (z/x + w/s)
              qr = q * r;                          // rho_aff = r_d + w - z = y - X beta
              xq = xv;
              gap += xv * zv + sv * wv;
              obj += y * xv;
            }
          }
#pragma unroll
          for (int cb = 0; cb < NCB; ++cb)
            acc[cb] = __builtin_amdgcn_mfma_f64_16x16x4f64(q, xr[pp[cb] & 255u] * xr[pp[cb] >> 8], acc[cb], 0, 0, 0);
#pragma unroll
          for (int xb = 0; xb < NXB; ++xb)
            acc[NCB + xb] = __builtin_amdgcn_mfma_f64_16x16x4f64(qr, xr[16 * xb + b.fl], acc[NCB + xb], 0, 0, 0);
          if (rp)
#pragma unroll
            for (int xb = 0; xb < NXB; ++xb)
              axx[xb] = __builtin_amdgcn_mfma_f64_16x16x4f64(xq, xr[16 * xb + b.fl], axx[xb], 0, 0, 0);
      };
      // the next sub-tile's values go to the other buffer after a few steps (registers freed)
      if (b.wave_live)
#pragma unroll
        for (int j = 0; j < kStoreAt; ++j) step(j);
      xs_store<K>(xs[(t + 1) & 1], stg);
      if (b.wave_live)
#pragma unroll
        for (int j = kStoreAt; j < 16; ++j) step(j);
      __syncthreads();
    }
  }
  // partials: D row = fit (rl + 4 r of the wave's 16), column = fl
  double* P = a.partial + ((size_t)b.slot * (a.nch[0] + a.nch[1]) + b.gch) * a.S_pad * NV;
  const size_t fw = (size_t)b.fb * 64 + b.wave * 16;
#pragma unroll
  for (int cb = 0; cb < NCB + NXB; ++cb)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const size_t fit = fw + b.rl + 4 * r;
      const int col = cb * 16 + b.fl;
      if (cb < NCB && col < NP) P[fit * NV + col] = acc[cb][r];
      const int xc = (cb - NCB) * 16 + b.fl;
      if (cb >= NCB && xc < K) P[fit * NV + NP + xc] = acc[cb][r];
    }
  if (rp)
#pragma unroll
    for (int xb = 0; xb < NXB; ++xb)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (16 * xb + b.fl < K) P[(fw + b.rl + 4 * r) * NV + NP + K + 2 + 16 * xb + b.fl] = axx[xb][r];
  gap = rows_sum(gap);
  obj = rows_sum(obj);
  if (b.rl == 0) {
    P[(fw + b.fl) * NV + NP + K] = gap;
    P[(fw + b.fl) * NV + NP + K + 1] = obj;
  }
}

// The affine / final passes share the walk: state (x, z, w) streamed kRing steps ahead, the
// design values from the double-buffered sub-tiles, x_i . v for the fragments fb on MFMA once per
// 4 steps. body(j-th step's state, valid, count, xr, dots).
template <int K, int NDOT, typename Body>
__device__ __forceinline__ void state_walk(const MmArgs& a, const Blk& b, const uint32_t* lst, double (*xs)[kSub * Xs<K>::S],
                                           const double (&fb)[NDOT][(K + 3) / 4], Body&& body) {
  mm_d4 dots[NDOT];
  const uint32_t nsub = (b.n_ent + kSub - 1) / kSub;
  if (!__syncthreads_or(b.live) || !nsub) return;
  double stg[Xs<K>::Stage];
  xs_load<K>(a, b, lst, 0, stg);
  xs_store<K>(xs[0], stg);
  double rx[kRing], rz[kRing], rw[kRing];
  auto load = [&](int k, uint32_t e) {
    const size_t si = state_at(b, e);
    rx[k] = a.x[si];
    rz[k] = a.z[si];
    rw[k] = a.w[si];
  };
#pragma unroll
  for (int k = 0; k < kRing; ++k) load(k, 4 * k + b.rl);
  __syncthreads();
  for (uint32_t t = 0; t < nsub; ++t) {
    const double* X = xs[t & 1];
    xs_load<K>(a, b, lst, t + 1, stg);
    auto step = [&](int j) {
      if ((j & 3) == 0) group_dots<K, NDOT>(X, j >> 2, b, fb, dots);
      const int k = j % kRing;
      const double xv = rx[k], zv = rz[k], wv = rw[k];
      const uint32_t e = t * kSub + 4 * j + b.rl;
      load(k, e + 4 * kRing);
      const bool valid = e < b.n_ent && b.live;
      double dv[NDOT];
#pragma unroll
      for (int v = 0; v < NDOT; ++v) dv[v] = dots[v][j & 3];
      body(xv, zv, wv, valid, valid ? (double)(lst[e] & 255u) : 1.0, X + (4 * j + b.rl) * Xs<K>::S, dv);
    };
    if (b.wave_live)
#pragma unroll
      for (int j = 0; j < kStoreAt; ++j) step(j);
    xs_store<K>(xs[(t + 1) & 1], stg);
    if (b.wave_live)
#pragma unroll
      for (int j = kStoreAt; j < 16; ++j) step(j);
    __syncthreads();
  }
}

// [0] primal step bound, [1] dual step bound, [2..4] mu_aff terms, then X'q rho0, X'q rho1.
template <int K>
__global__ __launch_bounds__(256, K <= 16 ? OB_MM_PASS_BLOCKS : 2) void mm_affine_kernel(const MmArgs a) {
  constexpr int NV = 5 + 2 * K;
  constexpr int NXB = Xs<K>::NXB;
  __shared__ __attribute__((aligned(16))) double xs[2][kSub * Xs<K>::S];
  __shared__ uint32_t lst[kCap];
  const Blk b = blk_ctx(a, lst, false);
  if (!b.any) return;  // partials of dead fits are never reduced
  double fb[2][(K + 3) / 4];
  bfrag<K>(a.beta, b, b.live, fb[0]);
  bfrag<K>(a.dba, b, b.live, fb[1]);
  double acc[5] = {1e300, 1e300, 0.0, 0.0, 0.0};
  mm_d4 m0[NXB], m1[NXB];
#pragma unroll
  for (int xb = 0; xb < NXB; ++xb) m0[xb] = m1[xb] = (mm_d4){0.0, 0.0, 0.0, 0.0};
  __syncthreads();  // lst
  state_walk<K, 2>(a, b, lst, xs, fb, [&](double xv, double zv, double wv, bool valid, double c, const double* xr,
                                          const double (&dv)[2]) {
    double q0 = 0.0, q1 = 0.0;
    if (valid) {
      const Affine f = affine_row(xv, zv, wv, c, xr[Xs<K>::Y], dv[0], dv[1]);
      if (f.dxa != 0.0) acc[0] = fmin(acc[0], (f.dxa < 0.0 ? -f.xv : f.sv) * mm_rcp(f.dxa));
      if (f.dza < 0.0) acc[1] = fmin(acc[1], -f.zv * mm_rcp(f.dza));
      if (f.dwa < 0.0) acc[1] = fmin(acc[1], -f.wv * mm_rcp(f.dwa));
      acc[2] += f.xv * f.dza + f.sv * f.dwa;
      acc[3] += f.zv * f.dxa - f.wv * f.dxa;
      acc[4] += f.dxa * f.dza - f.dxa * f.dwa;
      q0 = f.q * (f.r - f.dxa * (f.dwa * f.is + f.dza * f.ix));
      q1 = f.q * (f.ix - f.is);
    }
#pragma unroll
    for (int xb = 0; xb < NXB; ++xb) {
      const double bx = xr[16 * xb + b.fl];  // B: row rl, column 16 xb + fl (zero past K)
      m0[xb] = __builtin_amdgcn_mfma_f64_16x16x4f64(q0, bx, m0[xb], 0, 0, 0);
      m1[xb] = __builtin_amdgcn_mfma_f64_16x16x4f64(q1, bx, m1[xb], 0, 0, 0);
    }
  });
  double* P = a.partial + ((size_t)b.slot * (a.nch[0] + a.nch[1]) + b.gch) * a.S_pad * NV;
  const size_t fw = (size_t)b.fb * 64 + b.wave * 16;
#pragma unroll
  for (int xb = 0; xb < NXB; ++xb)
    if (16 * xb + b.fl < K)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const size_t fit = fw + b.rl + 4 * r;
        P[fit * NV + 5 + 16 * xb + b.fl] = m0[xb][r];
        P[fit * NV + 5 + K + 16 * xb + b.fl] = m1[xb][r];
      }
  acc[0] = rows_min(acc[0]);
  acc[1] = rows_min(acc[1]);
#pragma unroll
  for (int i = 2; i < 5; ++i) acc[i] = rows_sum(acc[i]);
  if (b.rl == 0)
#pragma unroll
    for (int i = 0; i < 5; ++i) P[(fw + b.fl) * NV + i] = acc[i];
}

// Step-length bounds of the corrector direction (the next assemble replays the direction).
template <int K>
__global__ __launch_bounds__(256, K <= 16 ? OB_MM_PASS_BLOCKS : 2) void mm_final_kernel(const MmArgs a) {
  __shared__ __attribute__((aligned(16))) double xs[2][kSub * Xs<K>::S];
  __shared__ uint32_t lst[kCap];
  const Blk b = blk_ctx(a, lst, false);
  if (!b.any) return;  // partials of dead fits are never reduced
  double fb[3][(K + 3) / 4];
  bfrag<K>(a.beta, b, b.live, fb[0]);
  bfrag<K>(a.dba, b, b.live, fb[1]);
  bfrag<K>(a.db, b, b.live, fb[2]);
  const double sigmu = b.live ? a.fs[b.F * kFs + FS_SIGMU] : 0.0;
  double acc[2] = {1e300, 1e300};
  __syncthreads();  // lst
  state_walk<K, 3>(a, b, lst, xs, fb, [&](double xv, double zv, double wv, bool valid, double c, const double* xr,
                                          const double (&dv)[3]) {
    if (!valid) return;
    const Affine f = affine_row(xv, zv, wv, c, xr[Xs<K>::Y], dv[0], dv[1]);
    const Corrector d = corrector_row(f, dv[2], sigmu);
    const double dx = d.dx, dz = d.dz, dw = d.dw;
    if (dx != 0.0) acc[0] = fmin(acc[0], (dx < 0.0 ? -f.xv : f.sv) * mm_rcp(dx));
    if (dz < 0.0) acc[1] = fmin(acc[1], -f.zv * mm_rcp(dz));
    if (dw < 0.0) acc[1] = fmin(acc[1], -f.wv * mm_rcp(dw));
  });
  acc[0] = rows_min(acc[0]);
  acc[1] = rows_min(acc[1]);
  if (b.rl == 0) {
    double* P = a.partial + (((size_t)b.slot * (a.nch[0] + a.nch[1]) + b.gch) * a.S_pad + b.s) * 2;
    P[0] = acc[0];
    P[1] = acc[1];
  }
}

// Chunk partials -> per-fit values, chunks in a fixed order; the first n_min values are minima.
__global__ __launch_bounds__(256) void mm_reduce_kernel(const MmArgs a, int nv, int n_min, int skip_dead) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  const size_t per_slot = (size_t)2 * a.S_pad * nv;
  if (i >= (size_t)a.n_rb * per_slot) return;
  const uint32_t slot = (uint32_t)(i / per_slot);
  const size_t rem = i % per_slot;
  const uint32_t g = (uint32_t)(rem / ((size_t)a.S_pad * nv));
  const size_t sv = rem % ((size_t)a.S_pad * nv);
  const uint32_t c0 = g ? a.nch[0] : 0u, nc = a.nch[g];
  const size_t stride = (size_t)a.S_pad * nv;
  const double* P = a.partial + ((size_t)slot * (a.nch[0] + a.nch[1]) + c0) * stride + sv;
  if (skip_dead && (a.fstat[((size_t)slot * 2 + g) * a.S_pad + sv / nv] & (kDone | kFailed))) return;
  const bool is_min = (int)(sv % nv) < n_min;
  double v = is_min ? 1e300 : 0.0;
  for (uint32_t c = 0; c < nc; ++c) v = is_min ? fmin(v, P[c * stride]) : v + P[c * stride];
  a.red[((size_t)slot * 2 + g) * stride + sv] = v;
}

// Weighted OLS of each (slot, group) -> the start of all its fits (wave per (slot, group)).
__global__ __launch_bounds__(64) void mm_start_kernel(const MmArgs a, int K) {
  extern __shared__ __attribute__((aligned(16))) double sm[];
  const int lane = threadIdx.x;
  const uint32_t slot = blockIdx.x >> 1, g = blockIdx.x & 1;
  const int NP = K * (K + 1) / 2, NV = nv_asm(K);
  const double* R = a.red + (((size_t)slot * 2 + g) * a.S_pad) * NV;  // fit 0 holds the sums
  double* M = sm;
  double* v = sm + K * K;
  for (int i = lane; i < K * K; i += 64) {
    const int r = i % K, c = i / K;
    M[i] = R[r <= c ? ob_pair_index(r, c, K) : ob_pair_index(c, r, K)];
  }
  for (int i = lane; i < K; i += 64) v[i] = R[NP + i];
  __syncthreads();
  const bool chol = wave_cholesky(M, K, lane);
  if (chol) wave_chol_solve(M, K, v, lane);
  __syncthreads();
  if (a.gchol) {  // the row reduction's leverages (mm_lev_kernel)
    double* gc = a.gchol + ((size_t)slot * 2 + g) * (K * K + 1);
    for (int i = lane; i < K * K; i += 64) gc[i] = M[i];
    if (lane == 0) gc[K * K] = chol ? R[0] : 0.0;
  }
  double delta = 0.0;
  if (chol) {
    double bv = 0.0;
    for (int k = 0; k < K; ++k) bv += v[k] * R[NP + k];
    const double ssr = fmax(R[NP + K] - bv, 0.0), sc = R[0];
    delta = ssr / sc;  // residual mean square; mm_shift_kernel makes the per-fit dual offset
  }
  for (int s = lane; s < a.S_pad; s += 64) {
    const size_t F = ((size_t)slot * 2 + g) * a.S_pad + s;
    if (s >= a.S) {
      a.fstat[F] = kDone | kFailed;
      continue;
    }
    a.fstat[F] = chol ? 0u : kFailed;
    for (int k = 0; k < K; ++k) a.beta[F * K + k] = chol ? v[k] : 0.0;
    double* f = a.fs + F * kFs;
    f[FS_DELTA] = delta;
    f[FS_NACT] = R[NP + K + 1];
    f[FS_AP] = f[FS_AD] = 0.0;
  }
  if (lane == 0 && chol) atomicAdd(a.active_rows, (unsigned long long)a.S * (unsigned long long)R[NP + K + 1]);
}

// MM-1 quantiles of each (slot, group), lanes in ascending tau (block per (slot, group)): the
// extreme quantiles, which need the most iterations, share fit batches, so the batches of the
// others stop costing passes early. lane_of maps simulation -> lane for the finish kernel.
__global__ __launch_bounds__(256) void mm_order_kernel(const MmArgs a, int m2) {
  extern __shared__ __attribute__((aligned(16))) double sm[];
  double* key = sm;
  uint32_t* val = reinterpret_cast<uint32_t*>(sm + m2);
  const uint32_t slot = blockIdx.x >> 1, g = blockIdx.x & 1;
  const uint32_t rep = a.rep0 == OB_MM_POINT_REP ? OB_MM_POINT_REP : a.rep0 + slot;
  for (int i = threadIdx.x; i < m2; i += blockDim.x) {
    key[i] = i < a.S ? ob_mm_tau((uint32_t)i, rep, a.key0, a.key1) : INFINITY;
    val[i] = (uint32_t)i;
  }
  __syncthreads();
  for (int k = 2; k <= m2; k <<= 1)
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = threadIdx.x; i < m2; i += blockDim.x) {
        const int l = i ^ j;
        if (l > i) {
          const bool up = (i & k) == 0;
          const double x = key[i], y = key[l];
          if ((x > y || (x == y && val[i] > val[l])) == up) {
            key[i] = y;
            key[l] = x;
            const uint32_t t = val[i];
            val[i] = val[l];
            val[l] = t;
          }
        }
      }
      __syncthreads();
    }
  const size_t base = ((size_t)slot * 2 + g) * a.S_pad;
  for (int j = threadIdx.x; j < a.S; j += blockDim.x) {
    a.fs[(base + j) * kFs + FS_TAU] = key[j];
    a.lane_of[base + val[j]] = (uint32_t)j;
  }
}

// Per-fit start (block per (slot, group)): the intercept of the OLS start moves to the fit's
// tau-quantile of the OLS residuals, and the dual offset shrinks to 0.01 (1 + rms of the shifted
// residual). At n = 250k this takes the extreme quantiles from ~85 to ~30 iterations and leaves the
// middle unchanged (tools/qr_ipm_proto.py --start). The quantile is a count-weighted one over
// kShiftSamples list entries taken at a fixed stride of the replicate's nonzero-count rows, so it
// is a function of the replicate alone.
constexpr int kShiftSamples = 4096;
constexpr double kDeltaScale = 0.01;
__global__ __launch_bounds__(1024) void mm_shift_kernel(const MmArgs a, int K) {
  __shared__ double key[kShiftSamples];
  __shared__ double wt[kShiftSamples];
  __shared__ uint32_t pre[1024 + 1];
  __shared__ double beta[ob::kMmMaxK];
  const uint32_t slot = blockIdx.x >> 1, g = blockIdx.x & 1;
  const uint32_t nch = a.nch[0] + a.nch[1], c0 = g ? a.nch[0] : 0u, ncg = a.nch[g];
  const size_t F0 = fit_index(a, slot, g, 0);
  if (a.fstat[F0] & kFailed) return;  // no OLS start for this group: every fit failed already
  const size_t li0 = (size_t)slot * nch + c0;
  // inclusive prefix of the chunk list lengths (ncg <= 1024 chunks)
  for (uint32_t c = threadIdx.x; c < ncg; c += blockDim.x) pre[c + 1] = a.nrows[li0 + c];
  if (threadIdx.x == 0) pre[0] = 0;
  if (threadIdx.x < (unsigned)K) beta[threadIdx.x] = a.beta[F0 * K + threadIdx.x];
  __syncthreads();
  if (threadIdx.x == 0)
    for (uint32_t c = 1; c <= ncg; ++c) pre[c] += pre[c - 1];
  __syncthreads();
  const uint32_t tot = pre[ncg];
  const int m = (int)min<uint32_t>(tot, (uint32_t)kShiftSamples);
  for (int j = threadIdx.x; j < kShiftSamples; j += blockDim.x) {
    double r = INFINITY, c = 0.0;
    if (j < m) {
      const uint32_t e = (uint32_t)(((uint64_t)j * tot) / (uint32_t)m);
      uint32_t lo = 0, hi = ncg;  // chunk with pre[lo] <= e < pre[lo + 1]
      while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (pre[mid] <= e) lo = mid;
        else hi = mid;
      }
      const uint32_t ent = a.rowlist[(li0 + lo) * a.cap + (e - pre[lo])];
      const uint32_t row = lo * a.rc + (ent >> 8);
      const double* X = a.cols[g];
      double xb = beta[0];
      for (int k = 1; k < K; ++k) xb += X[(size_t)(k - 1) * a.ld[g] + row] * beta[k];
      r = X[(size_t)a.p * a.ld[g] + row] - xb;
      c = (double)(ent & 255u);
    }
    key[j] = r;
    wt[j] = c;
  }
  __syncthreads();
  for (int k = 2; k <= kShiftSamples; k <<= 1)  // bitonic sort by residual, weights along
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = threadIdx.x; i < kShiftSamples; i += blockDim.x) {
        const int l = i ^ j;
        if (l > i) {
          const bool up = (i & k) == 0;
          const double x = key[i], y = key[l];
          if ((x > y) == up) {
            key[i] = y;
            key[l] = x;
            const double t = wt[i];
            wt[i] = wt[l];
            wt[l] = t;
          }
        }
      }
      __syncthreads();
    }
  if (threadIdx.x == 0)  // inclusive prefix of the weights (in place, serial: 4096 adds once per batch)
    for (int i = 1; i < m; ++i) wt[i] += wt[i - 1];
  __syncthreads();
  const double W = m ? wt[m - 1] : 0.0;
  for (int s = threadIdx.x; s < a.S; s += blockDim.x) {
    const size_t F = F0 + s;
    double* f = a.fs + F * kFs;
    double q = 0.0;
    if (m) {
      const double target = f[FS_TAU] * W;
      int lo = 0, hi = m - 1;  // first i with wt[i] >= target
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (wt[mid] >= target) hi = mid;
        else lo = mid + 1;
      }
      q = key[lo];
    }
    a.beta[F * K] = beta[0] + q;
    f[FS_DELTA] = kDeltaScale * (1.0 + sqrt(f[FS_DELTA] + q * q));
  }
}

// Convergence test, Cholesky of M, affine direction (wave per fit). rp_mode (phase 2/3, X'x = b):
// 1 = primal residual b - X'x from the start assemble, 2 = the last one times (1 - ap).
__global__ __launch_bounds__(64) void mm_solve_affine_kernel(const MmArgs a, int K, int rp_mode) {
  extern __shared__ __attribute__((aligned(16))) double sm[];
  const int lane = threadIdx.x;
  const size_t F = blockIdx.x;
  if (a.fstat[F] & (kDone | kFailed)) return;
  const int NP = K * (K + 1) / 2, NV = nv_asm(K);
  const double* R = a.red + F * NV;
  double* f = a.fs + F * kFs;
  const double gap = R[NP + K], obj = R[NP + K + 1] + (rp_mode ? f[FS_OBJFIX] : 0.0);
  double rpk = 0.0, bk = 0.0;  // lane k < K: b_k - (X'x)_k, b_k
  if (rp_mode && lane < K) {
    bk = a.bvec[F * K + lane];
    rpk = rp_mode == 1 ? bk - R[NP + K + 2 + lane] : (1.0 - f[FS_AP]) * a.rpv[F * K + lane];
  }
  double rpm = fabs(rpk), bm = fabs(bk);
  for (int o = 32; o > 0; o >>= 1) {
    rpm = fmax(rpm, __shfl_xor(rpm, o));
    bm = fmax(bm, __shfl_xor(bm, o));
  }
  if (lane == 0) {
    f[FS_GAP] = gap;
    f[FS_OBJ] = obj;
  }
  if (gap < a.tol * (1.0 + fabs(obj)) && rpm <= 1e-10 * (1.0 + bm)) {  // converged: beta is the QR solution
    if (lane == 0) a.fstat[F] = kDone;
    return;
  }
  if (rp_mode && lane < K) a.rpv[F * K + lane] = rpk;
  double* M = sm;
  double* v = sm + K * K;
  // Late in a solve the weights Q = 1 / (z/x + w/s) spread over many decades and M = X'QX can lose
  // positive definiteness in f64 (a 500k-row fit at tau 0.54 did after 114 iterations). As
  // Clarabel does (its static regularization, 1e-8 relative), the factorization is then retried on
  // M + delta max_i M_ii I for delta = 1e-14, 1e-12, 1e-10, 1e-8: the Newton direction becomes
  // slightly inexact, while the step lengths, the gap and the stopping rule stay exact.
  double dmax = 0.0;
  for (int i = lane; i < K; i += 64) dmax = fmax(dmax, R[ob_pair_index(i, i, K)]);
  for (int o = 32; o > 0; o >>= 1) dmax = fmax(dmax, __shfl_xor(dmax, o));
  bool chol = false;
  for (int attempt = 0; attempt < 5 && !chol; ++attempt) {
    const double reg = attempt ? dmax * (attempt == 1 ? 1e-14 : attempt == 2 ? 1e-12 : attempt == 3 ? 1e-10 : 1e-8) : 0.0;
    for (int i = lane; i < K * K; i += 64) {
      const int r = i % K, c = i / K;
      M[i] = R[r <= c ? ob_pair_index(r, c, K) : ob_pair_index(c, r, K)] + (r == c ? reg : 0.0);
    }
    __syncthreads();
    chol = wave_cholesky(M, K, lane);
    __syncthreads();
  }
  if (!chol) {  // no usable direction: accept the point at Clarabel's own Solved tolerance (1e-8), else fail
    if (lane == 0 && a.trace)
      printf("[mm] fit %zu: no Cholesky of M (K %d, max diag %.3e), gap %.3e obj %.6e rp %.3e\n", F, K, dmax, gap, obj, rpm);
    if (lane == 0) a.fstat[F] = gap < 1e-8 * (1.0 + fabs(obj)) && rpm <= 1e-8 * (1.0 + bm) ? kDone : (kDone | kFailed);
    return;
  }
  for (int i = lane; i < K; i += 64) v[i] = R[NP + i] - rpk;  // M dba = X'Q rho_aff - (b - X'x)
  __syncthreads();
  wave_chol_solve(M, K, v, lane);
  for (int i = lane; i < K * K; i += 64) a.L[F * K * K + i] = M[i];
  for (int i = lane; i < K; i += 64) a.dba[F * K + i] = v[i];
  if (lane == 0) {
    f[FS_MU] = gap / (2.0 * f[FS_NACT]);
    atomicAdd(a.active, 1u);
    atomicAdd(a.active_rows, (unsigned long long)f[FS_NACT]);
  }
}

// sigma from the affine step, corrector direction (wave per fit).
__global__ __launch_bounds__(64) void mm_solve_corrector_kernel(const MmArgs a, int K) {
  extern __shared__ __attribute__((aligned(16))) double sm[];
  const int lane = threadIdx.x;
  const size_t F = blockIdx.x;
  if (a.fstat[F] & (kDone | kFailed)) return;
  const int NV = 5 + 2 * K;
  const double* R = a.red + F * NV;
  double* f = a.fs + F * kFs;
  const double ap = fmin(1.0, R[0]), ad = fmin(1.0, R[1]);
  const double n2 = 2.0 * f[FS_NACT];
  const double mu_aff = (f[FS_GAP] + ad * R[2] + ap * R[3] + ap * ad * R[4]) / n2;
  const double mu = f[FS_MU];
  const double ratio = mu_aff / mu;
  const double sigmu = ratio * ratio * ratio * mu;
  double* Lm = sm;
  double* v = sm + K * K;
  for (int i = lane; i < K * K; i += 64) Lm[i] = a.L[F * K * K + i];
  for (int i = lane; i < K; i += 64) v[i] = R[5 + i] + sigmu * R[5 + K + i] - (a.rp ? a.rpv[F * K + i] : 0.0);
  __syncthreads();
  wave_chol_solve(Lm, K, v, lane);
  for (int i = lane; i < K; i += 64) a.db[F * K + i] = v[i];
  if (lane == 0) f[FS_SIGMU] = sigmu;
}

// Step lengths and the dual update of beta (thread per fit).
__global__ __launch_bounds__(256) void mm_step_kernel(const MmArgs a, int K, size_t n_fits) {
  const size_t F = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (F >= n_fits || (a.fstat[F] & (kDone | kFailed))) return;
  const double* R = a.red + F * 2;
  const double ap = fmin(1.0, kEta * R[0]), ad = fmin(1.0, kEta * R[1]);
  for (int k = 0; k < K; ++k) {
    a.bprev[F * K + k] = a.beta[F * K + k];
    a.beta[F * K + k] += ad * a.db[F * K + k];
  }
  a.fs[F * kFs + FS_AP] = ap;
  a.fs[F * kFs + FS_AD] = ad;
}

// ---- row reduction (phases 2 and 3) ----

// Phase 1 solves S1 quantiles per (slot, group): sorted lanes 0, f, 2f, ... and S - 1 (f = 1: all).
__host__ __device__ inline int sub_lane(int k, int S, int f) { return min(k * f, S - 1); }

// Phase-1 fit k's tau = the full fit's at sub_lane(k) (thread per phase-1 fit).
__global__ __launch_bounds__(256) void mm_subtau_kernel(const MmArgs a, const MmArgs a1, int f) {
  const size_t F1 = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (F1 >= (size_t)a1.n_rb * 2 * a1.S_pad) return;
  const size_t sg = F1 / a1.S_pad;
  const int k = (int)(F1 % a1.S_pad);
  if (k >= a1.S) return;
  a1.fs[F1 * kFs + FS_TAU] = a.fs[(sg * a.S_pad + sub_lane(k, a.S, f)) * kFs + FS_TAU];
}

// Every full fit's phase-1 result: linear in tau between the two phase-1 fits around its lane
// (a copy when f = 1). It only centres the fit's band, so interpolation error moves no result
// (the fixed rows are verified). Padding fits are retired.
__global__ __launch_bounds__(256) void mm_interp_kernel(const MmArgs a, const MmArgs a1, int K, int f) {
  const size_t F = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (F >= (size_t)a.n_rb * 2 * a.S_pad) return;
  const size_t sg = F / a.S_pad;
  const int s = (int)(F % a.S_pad);
  if (s >= a.S) {
    a.fstat[F] = kDone | kFailed;
    return;
  }
  const int k = a1.S > 1 ? min(s / f, a1.S - 2) : 0;
  const size_t Fa = sg * a1.S_pad + k, Fb = a1.S > 1 ? Fa + 1 : Fa;
  const double ta = a1.fs[Fa * kFs + FS_TAU], tb = a1.fs[Fb * kFs + FS_TAU], tau = a.fs[F * kFs + FS_TAU];
  const double t = (f > 1 && tb > ta) ? fmin(fmax((tau - ta) / (tb - ta), 0.0), 1.0) : 0.0;
  const bool failed = a1.fstat[Fa] != kDone || (t > 0.0 && a1.fstat[Fb] != kDone);
  a.fstat[F] = failed ? (kDone | kFailed) : kDone;
  for (int j = 0; j < K; ++j) {
    const double ba = a1.beta[Fa * K + j], bb = a1.beta[Fb * K + j];
    a.beta[F * K + j] = t > 0.0 ? (1.0 - t) * ba + t * bb : ba;
  }
  const double da = a1.fs[Fa * kFs + FS_DELTA], db = a1.fs[Fb * kFs + FS_DELTA];
  a.fs[F * kFs + FS_DELTA] = t > 0.0 ? (1.0 - t) * da + t * db : da;
  a.fs[F * kFs + FS_NACT] = a1.fs[Fa * kFs + FS_NACT];
}

// kBandSamples list entries of each (slot, group) at a fixed stride over the full nonzero-row lists:
// the rows behind every fit's band quantiles (a function of the replicate alone).
__global__ __launch_bounds__(1024) void mm_sample_kernel(const MmArgs a) {
  __shared__ uint32_t pre[1024 + 1];
  const uint32_t slot = blockIdx.x >> 1, g = blockIdx.x & 1;
  const uint32_t nch = a.nch[0] + a.nch[1], c0 = g ? a.nch[0] : 0u, ncg = a.nch[g];
  const size_t li0 = (size_t)slot * nch + c0;
  for (uint32_t c = threadIdx.x; c < ncg; c += blockDim.x) pre[c + 1] = a.nrows[li0 + c];
  if (threadIdx.x == 0) pre[0] = 0;
  __syncthreads();
  if (threadIdx.x == 0)
    for (uint32_t c = 1; c <= ncg; ++c) pre[c] += pre[c - 1];
  __syncthreads();
  const uint32_t tot = pre[ncg];
  const uint32_t m = min<uint32_t>(tot, (uint32_t)kBandSamples);
  uint32_t* out = a.samp + ((size_t)slot * 2 + g) * 2 * kBandSamples;
  for (uint32_t j = threadIdx.x; j < m; j += blockDim.x) {
    const uint32_t e = (uint32_t)(((uint64_t)j * tot) / m);
    uint32_t lo = 0, hi = ncg;  // chunk with pre[lo] <= e < pre[lo + 1]
    while (hi - lo > 1) {
      const uint32_t mid = (lo + hi) >> 1;
      if (pre[mid] <= e) lo = mid;
      else hi = mid;
    }
    const uint32_t ent = a.rowlist[(li0 + lo) * a.cap + (e - pre[lo])];
    out[j] = lo * a.rc + (ent >> 8);
    out[kBandSamples + j] = ent & 255u;
  }
  if (threadIdx.x == 0) a.nsamp[(size_t)slot * 2 + g] = m;
}

// Leverage of every full-list entry: lev_i = sqrt(n x_i' G^-1 x_i) with G = X'CX of the phase-1
// subsample and n = its sum of counts (about sqrt(K) for a typical row). The error of beta_hat
// moves a row's residual in proportion to it, so the bands widen for high-leverage rows.
__global__ __launch_bounds__(256) void mm_lev_kernel(const MmArgs a, int K) {
  __shared__ double L[ob::kMmMaxK * ob::kMmMaxK];
  const uint32_t gch = blockIdx.x, slot = blockIdx.z, nch = a.nch[0] + a.nch[1];
  const uint32_t g = gch >= a.nch[0] ? 1u : 0u;
  const double* gc = a.gchol + ((size_t)slot * 2 + g) * (K * K + 1);
  for (int i = threadIdx.x; i < K * K; i += 256) L[i] = gc[i];
  __syncthreads();
  const double n = gc[K * K];
  const size_t li = (size_t)slot * nch + gch;
  const uint32_t ne = a.nrows[li], r0 = (gch - (g ? a.nch[0] : 0u)) * a.rc;
  const double* X = a.cols[g];
  for (uint32_t e = threadIdx.x; e < ne; e += 256) {
    const uint32_t row = r0 + (a.rowlist[li * a.cap + e] >> 8);
    double v[ob::kMmMaxK], q = 0.0;
    for (int i = 0; i < K; ++i) {  // L v = x (forward substitution), q = |v|^2
      double t = i ? X[(size_t)(i - 1) * a.ld[g] + row] : 1.0;
      for (int j = 0; j < i; ++j) t -= L[i + j * K] * v[j];
      v[i] = t / L[i + i * K];
      q += v[i] * v[i];
    }
    a.lev[li * a.cap + e] = n > 0.0 ? sqrt(n * q) : sqrt((double)K);
  }
}

// Per fit (block of 256): beta_hat <- the phase-1 beta (zero if not finite), and the residual band
// [lo, hi] = the count-weighted tau -/+ delta quantiles of the sampled residuals at beta_hat, with
// delta = kappa sqrt(tau (1 - tau) K / m) + 0.01 (m = the phase-1 sample's rows). A fit whose
// phase 1 failed keeps every row (band = the real line); padding fits keep none.
__global__ __launch_bounds__(256) void mm_band_kernel(const MmArgs a, int K, double kappa, double band0) {
  __shared__ double key[kBandSamples];
  __shared__ double wt[kBandSamples];
  __shared__ double beta[ob::kMmMaxK];
  __shared__ double part[256];
  __shared__ int finite;
  const size_t F = blockIdx.x;
  const uint32_t slot = (uint32_t)(F / (2 * (size_t)a.S_pad)), g = (uint32_t)((F / a.S_pad) & 1);
  const int s = (int)(F % a.S_pad), t = threadIdx.x;
  double* f = a.fs + F * kFs;
  if (s >= a.S) {
    if (t == 0) {
      f[FS_LO] = INFINITY;
      f[FS_HI] = -INFINITY;
      f[FS_EXT] = 0.0;
    }
    return;
  }
  if (t == 0) finite = 1;
  __syncthreads();
  if (t < K) {
    beta[t] = a.beta[F * K + t];
    if (!isfinite(beta[t])) finite = 0;
  }
  __syncthreads();
  if (t < K) {
    if (!finite) beta[t] = 0.0;
    a.bhat[F * K + t] = beta[t];
  }
  const double tau = f[FS_TAU];
  const double delta = kappa * sqrt(tau * (1.0 - tau) * K / fmax(f[FS_NACT], 1.0)) + band0;
  if ((a.fstat[F] & kFailed) || (tau - delta <= 0.0 && tau + delta >= 1.0)) {
    if (t == 0) {
      f[FS_LO] = -INFINITY;
      f[FS_HI] = INFINITY;
      f[FS_EXT] = 0.0;
    }
    return;
  }
  __syncthreads();
  const uint32_t ns = a.nsamp[(size_t)slot * 2 + g];
  const uint32_t* sr = a.samp + ((size_t)slot * 2 + g) * 2 * kBandSamples;
  const double* X = a.cols[g];
  const int64_t ld = a.ld[g];
  for (int j = t; j < kBandSamples; j += 256) {
    double r = INFINITY, c = 0.0;
    if ((uint32_t)j < ns) {
      const uint32_t row = sr[j];
      double xb = beta[0];
      for (int k = 1; k < K; ++k) xb += X[(size_t)(k - 1) * ld + row] * beta[k];
      r = X[(size_t)a.p * ld + row] - xb;
      c = (double)sr[kBandSamples + j];
    }
    key[j] = r;
    wt[j] = c;
  }
  __syncthreads();
  for (int k = 2; k <= kBandSamples; k <<= 1)  // bitonic sort by residual, weights along
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = t; i < kBandSamples; i += 256) {
        const int l = i ^ j;
        if (l > i) {
          const bool up = (i & k) == 0;
          const double x = key[i], y = key[l];
          if ((x > y) == up) {
            key[i] = y;
            key[l] = x;
            const double w = wt[i];
            wt[i] = wt[l];
            wt[l] = w;
          }
        }
      }
      __syncthreads();
    }
  constexpr int kPer = kBandSamples / 256;  // inclusive prefix of the weights: 16 per thread
  double run = 0.0;
  for (int i = 0; i < kPer; ++i) run += wt[t * kPer + i];
  part[t] = run;
  __syncthreads();
  if (t == 0)
    for (int i = 1; i < 256; ++i) part[i] += part[i - 1];
  __syncthreads();
  run = t ? part[t - 1] : 0.0;
  for (int i = 0; i < kPer; ++i) {
    run += wt[t * kPer + i];
    wt[t * kPer + i] = run;
  }
  __syncthreads();
  if (t == 0) {
    const int m = (int)ns;
    const double W = m ? wt[m - 1] : 0.0;
    auto quant = [&](double target) {  // first i with wt[i] >= target
      int lo = 0, hi = m - 1;
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (wt[mid] >= target) hi = mid;
        else lo = mid + 1;
      }
      return key[lo];
    };
    const double lo = (m && tau - delta > 0.0) ? quant((tau - delta) * W) : -INFINITY;
    const double hi = (m && tau + delta < 1.0) ? quant((tau + delta) * W) : INFINITY;
    const double mid = m ? quant(tau * W) : 0.0;
    // residual units per rank unit (1 / density at the quantile), from the band's finite sides
    const double slope = isfinite(lo) && isfinite(hi) ? (hi - lo) / (2.0 * delta)
                         : isfinite(hi)               ? (hi - mid) / delta
                         : isfinite(lo)               ? (mid - lo) / delta
                                                      : 0.0;
    f[FS_LO] = lo;
    f[FS_HI] = hi;
    // per unit of leverage above sqrt(K): kappa standard errors of x_i beta_hat
    f[FS_EXT] = kappa * sqrt(tau * (1.0 - tau) / fmax(f[FS_NACT], 1.0)) * slope;
  }
}

// One walk over a chunk's full nonzero-row list per 64-fit block. Each lane's fit classifies its
// rows at beta_hat: inside the band [lo, hi] (kept: the row joins the block's reduced list if any
// fit of the block keeps it), above (x_i = c_i) or below (x_i = 0).
// !VERIFY: writes the block's list and per-fit partials: sum_above c x, sum_all c x, sum_above c y
//          (the fixed rows' objective), the kept entries (nv_cls layout).
// VERIFY:  at the reduced optimum beta, a fixed row whose residual has the wrong sign flags its fit
//          for phase 3 (kRetry).
template <int K, bool VERIFY>
__global__ __launch_bounds__(256, 2) void mm_classify_kernel(const MmArgs a) {
  constexpr int NXB = Xs<K>::NXB, S = Xs<K>::S, NVC = nv_cls(K), ND = VERIFY ? 2 : 1;
  __shared__ __attribute__((aligned(16))) double xs[2][kSub * S];
  __shared__ uint32_t lst[kCap];
  __shared__ uint32_t keep[2][kSub];
  __shared__ double levs[2][kSub];  // the sub-tile's leverages and added-row bits, staged with xs
  __shared__ uint32_t xbits[2][kSub];
  __shared__ uint32_t nkeep;
  const Blk b = blk_ctx(a, lst, true);
  const bool part = b.s < a.S;
  double lo = INFINITY, hi = -INFINITY, ext = 0.0;
  if (part) {
    lo = a.fs[b.F * kFs + FS_LO];
    hi = a.fs[b.F * kFs + FS_HI];
    ext = a.fs[b.F * kFs + FS_EXT];
  }
  const double sqk = sqrt((double)K);
  const size_t li = (size_t)b.slot * (a.nch[0] + a.nch[1]) + b.gch;
  double fb[ND][(K + 3) / 4];
  bfrag<K>(a.bhat, b, part, fb[0]);
  if (VERIFY) bfrag<K>(a.beta, b, part, fb[ND - 1]);
  mm_d4 A[NXB], T[NXB];
#pragma unroll
  for (int xb = 0; xb < NXB; ++xb) A[xb] = T[xb] = (mm_d4){0.0, 0.0, 0.0, 0.0};
  double objfix = 0.0;
  bool bad = false;
  uint32_t cnt = 0;  // wave 0: entries of the block's list so far
  const size_t oi = li * (a.S_pad / 64) + b.fb;
  uint32_t* out = a.blist + oi * a.cap;
  uint32_t* xm = a.xmask + oi * (a.cap / 32);
  const bool mine = part && lo <= hi;  // a fit of this round (the others have empty bands)
  const bool check = VERIFY && mine;
  if (!__syncthreads_or(mine)) {  // no fit of the block takes part: an empty list
    if (!VERIFY && threadIdx.x == 0) a.bnrows[oi] = 0u;
    return;
  }
  const uint32_t nsub = (b.n_ent + kSub - 1) / kSub;
  uint32_t st_need = 0, st_all = 0;  // a.list_stat
  double stg[Xs<K>::Stage], lv = 0.0;
  uint32_t xb1 = 0u;
  auto side_load = [&](uint32_t t) {  // threads < 64: row t * kSub + tid's leverage and added bit
    const uint32_t e = t * kSub + threadIdx.x;
    if (threadIdx.x < kSub && e < b.n_ent) {
      lv = a.lev[li * a.cap + e];
      xb1 = (xm[e >> 5] >> (e & 31u)) & 1u;
    }
  };
  auto side_store = [&](int buf) {
    if (threadIdx.x < kSub) {
      levs[buf][threadIdx.x] = lv;
      xbits[buf][threadIdx.x] = xb1;
      keep[buf][threadIdx.x] = 0u;
    }
  };
  xs_load<K>(a, b, lst, 0, stg);  // lst: published by the barrier above
  side_load(0);
  xs_store<K>(xs[0], stg);
  side_store(0);
  __syncthreads();
  for (uint32_t t = 0; t < nsub; ++t) {
    const double* X = xs[t & 1];
    uint32_t* kp = keep[t & 1];
    xs_load<K>(a, b, lst, t + 1, stg);  // the next sub-tile's values, in flight during this one
    side_load(t + 1);
    const double* LV = levs[t & 1];
    const uint32_t* XB = xbits[t & 1];
    uint32_t side = 0, wrong = 0;  // wrong: bit j = step j's residual at beta has the other sign (VERIFY)
    mm_d4 dots[ND];
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      if ((j & 3) == 0) group_dots<K, ND>(X, j >> 2, b, fb, dots);
      const uint32_t e = t * kSub + 4 * j + b.rl;
      const bool valid = part && e < b.n_ent;
      const double y = X[(4 * j + b.rl) * S + Xs<K>::Y];
      const double rh = y - dots[0][j & 3];
      const double x = valid ? ext * fmax(LV[4 * j + b.rl] - sqk, 0.0) : 0.0;  // leverage widening
      const bool in = valid && rh >= lo - x && rh <= hi + x;
      side |= (in ? 1u : (rh > hi + x ? 2u : 0u)) << (2 * j);
      // rows added after an earlier verification are in the list too (a row flagged in this pass
      // is set after the barrier below, so within a sub-tile the bits read here are the old ones)
      if (in || (e < b.n_ent && XB[4 * j + b.rl])) kp[4 * j + b.rl] = 1u;
      if (!VERIFY && a.list_stat) {
        const unsigned long long m = __ballot(in || (valid && XB[4 * j + b.rl]));
#pragma unroll
        for (int r = 0; r < 4; ++r) st_need += ((m >> (16 * r)) & 0xffffull) != 0ull ? 1u : 0u;
      }
      if (VERIFY) {
        const double rv = y - dots[ND - 1][j & 3], eps = 1e-9 * (1.0 + fabs(y));
        const uint32_t sd = in ? 1u : (rh > hi + x ? 2u : 0u);
        wrong |= (sd == 2u ? rv < -eps : (sd == 0u && rv > eps)) ? 1u << j : 0u;
      }
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const uint32_t e = t * kSub + 4 * j + b.rl;
      const bool valid = part && e < b.n_ent;
      const bool kept = kp[4 * j + b.rl] != 0u;
      const uint32_t sd = (side >> (2 * j)) & 3u;
      if (!VERIFY && a.list_stat) {  // entries of the block's list
        const unsigned long long m = __ballot(kept && e < b.n_ent);
#pragma unroll
        for (int r = 0; r < 4; ++r) st_all += ((m >> (16 * r)) & 0xffffull) != 0ull ? 1u : 0u;
      }
      const double* xr = X + (4 * j + b.rl) * S;
      const double y = xr[Xs<K>::Y];
      if (!VERIFY) {
        const double c = valid ? (double)(lst[e] & 255u) : 0.0;
        const double ab = (!kept && sd == 2u) ? c : 0.0;
        objfix += ab * y;
#pragma unroll
        for (int xb = 0; xb < NXB; ++xb) {
          const double bx = xr[16 * xb + b.fl];
          A[xb] = __builtin_amdgcn_mfma_f64_16x16x4f64(ab, bx, A[xb], 0, 0, 0);
          T[xb] = __builtin_amdgcn_mfma_f64_16x16x4f64(c, bx, T[xb], 0, 0, 0);
        }
      } else if (check && valid && !kept && ((wrong >> j) & 1u)) {  // the row joins the block's list next round
        bad = true;
        atomicOr(&xm[e >> 5], 1u << (e & 31u));
      }
    }
    if (!VERIFY && b.wave == 0) {  // the kept rows of this sub-tile, in row order
      const uint32_t e = t * kSub + b.lane;
      const bool f = e < b.n_ent && kp[b.lane] != 0u;
      const unsigned long long m = __ballot(f);
      const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
      if (f) out[cnt + below] = lst[e];
      cnt += (uint32_t)__popcll(m);
    }
    xs_store<K>(xs[(t + 1) & 1], stg);  // the other buffers were last read before the previous barrier
    side_store((t + 1) & 1);
    __syncthreads();
  }
  const bool wpart = __ballot(part) != 0ull;  // the wave has a fit in this round
  if (!VERIFY && a.list_stat && b.lane == 0 && wpart) {
    atomicAdd(&g_mm_list_stat[0], (unsigned long long)st_all);
    atomicAdd(&g_mm_list_stat[1], (unsigned long long)st_need);
  }
  if (!VERIFY) {
    if (threadIdx.x == 0) {
      a.bnrows[oi] = cnt;
      nkeep = cnt;
    }
    __syncthreads();
    double* P = a.partial + li * a.S_pad * NVC;
    const size_t fw = (size_t)b.fb * 64 + b.wave * 16;
#pragma unroll
    for (int xb = 0; xb < NXB; ++xb)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const size_t fit = fw + b.rl + 4 * r;
        const int col = 16 * xb + b.fl;
        if (col < K) {
          P[fit * NVC + col] = A[xb][r];
          P[fit * NVC + K + col] = T[xb][r];
        }
      }
    objfix = rows_sum(objfix);
    if (b.rl == 0) {
      P[(fw + b.fl) * NVC + 2 * K] = objfix;
      P[(fw + b.fl) * NVC + 2 * K + 1] = (double)nkeep;
    }
  } else {
    bad = rows_sum(bad ? 1.0 : 0.0) != 0.0;
    if (b.rl == 0 && part && bad) atomicOr(&a.fstat[b.F], kRetry);
  }
}

// Reduced right-hand sides from the classify partials (thread per fit): b = (1 - tau) X'c -
// sum_above c x; the fixed rows' objective; the reduced problem's rows. reset (phase 2): every fit
// restarts at beta_hat; a reduced list too short to hold a fit goes straight to phase 3.
__global__ __launch_bounds__(256) void mm_bvec_kernel(const MmArgs a, int K, size_t n_fits, int reset) {
  const size_t F = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (F >= n_fits || (int)(F % a.S_pad) >= a.S) return;
  const double* R = a.red + F * nv_cls(K);
  double* f = a.fs + F * kFs;
  const double tau = f[FS_TAU];
  for (int k = 0; k < K; ++k) a.bvec[F * K + k] = (1.0 - tau) * R[K + k] - R[k];
  f[FS_OBJFIX] = R[2 * K];
  f[FS_NACT] = R[2 * K + 1];
  if (reset) {
    a.fstat[F] = R[2 * K + 1] < (double)(2 * K) ? (kDone | kFailed) : 0u;
    for (int k = 0; k < K; ++k) a.beta[F * K + k] = a.bhat[F * K + k];
  }
  if (a.fstat[F] == 0u) {
    f[FS_AP] = f[FS_AD] = 0.0;
    atomicAdd(a.active_rows, (unsigned long long)R[2 * K + 1]);
  }
}

// After a reduced round and mm_verify: a fit with a wrong-signed fixed row or a failure restarts at
// beta_hat, after round 0 with its band plus the wrong-signed rows (mm_verify's xmask; the
// Portnoy-Koenker fix-up), after round 1 on all its rows (band = the real line); the others keep
// their result and an empty band.
__global__ __launch_bounds__(256) void mm_retry_kernel(const MmArgs a, int K, size_t n_fits, int all_rows) {
  const size_t F = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (F >= n_fits || (int)(F % a.S_pad) >= a.S) return;
  double* f = a.fs + F * kFs;
  if (a.fstat[F] == kDone) {
    f[FS_LO] = INFINITY;
    f[FS_HI] = -INFINITY;
    return;
  }
  a.fstat[F] = 0u;
  if (all_rows) {
    f[FS_LO] = -INFINITY;
    f[FS_HI] = INFINITY;
  }
  for (int k = 0; k < K; ++k) a.beta[F * K + k] = a.bhat[F * K + k];
  atomicAdd(a.active, 1u);
}

__global__ __launch_bounds__(256) void mm_expire_kernel(const MmArgs a, size_t n_fits) {
  const size_t F = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (F < n_fits && !(a.fstat[F] & (kDone | kFailed))) a.fstat[F] = kDone | kFailed;  // no convergence
}

// In-place ascending bitonic sort of v[0, m) (m a power of two) by the block.
__device__ void block_sort(double* v, int m) {
  for (int k = 2; k <= m; k <<= 1)
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = threadIdx.x; i < m; i += blockDim.x) {
        const int l = i ^ j;
        if (l > i) {
          const bool up = (i & k) == 0;
          const double x = v[i], y = v[l];
          if ((x > y) == up) {
            v[i] = y;
            v[l] = x;
          }
        }
      }
      __syncthreads();
    }
}

// Sample position -> row of group g in replicate slot (rows in order, each repeated by count).
__device__ uint32_t position_row(const MmArgs& a, uint32_t slot, uint32_t g, uint32_t j, const uint32_t* pre,
                                 uint32_t ntiles) {
  if (!a.counts) return j;
  uint32_t lo = 0, hi = ntiles;  // last tile t with pre[t] <= j
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (pre[mid] <= j)
      lo = mid;
    else
      hi = mid;
  }
  uint32_t rem = j - pre[lo];
  const uint32_t base = lo * OB_TILE_ROWS, rows = min(OB_TILE_ROWS, a.n[g] - base);
  for (uint32_t r = 0; r < rows; ++r) {
    const uint32_t c = row_count(a, slot, g, base + r);
    if (rem < c) return base + r;
    rem -= c;
  }
  return base + rows - 1;  // unreachable when the counts are consistent
}

// One block per replicate slot: run_single_pass (quantile_decomposition.rs:221-279) after the fits.
__global__ __launch_bounds__(256) void mm_finish_kernel(const MmArgs a, int K, int m2) {
  extern __shared__ __attribute__((aligned(16))) double sm[];
  double* yaa = sm;
  double* ybb = yaa + m2;
  double* yab = ybb + m2;
  uint16_t* ia = reinterpret_cast<uint16_t*>(yab + m2);
  uint16_t* ib = ia + m2;
  __shared__ uint32_t cnt[2];
  const uint32_t slot = blockIdx.x;
  const uint32_t rep = a.rep0 == OB_MM_POINT_REP ? OB_MM_POINT_REP : a.rep0 + slot;
  double* row = a.rows + (size_t)slot * 3 * a.n_q;
  if (threadIdx.x < 2) {  // successful fits in simulation order (filter_map, :221-229)
    const uint32_t g = threadIdx.x;
    uint16_t* idx = g ? ib : ia;
    uint32_t k = 0;
    const uint32_t* lanes = a.lane_of + ((size_t)slot * 2 + g) * a.S_pad;
    for (int s = 0; s < a.S; ++s) {
      const uint32_t j = lanes[s];
      const bool forced = a.fail_mask && s < a.fail_sims && ((a.fail_mask[g * a.fail_sims + s] >> (rep & 7u)) & 1u);
      if (a.fstat[fit_index(a, slot, g, (int)j)] == kDone && !forced) idx[k++] = (uint16_t)j;
    }
    cnt[g] = k;
  }
  // exclusive tile prefixes of the replicate's level-1 counts (both groups)
  const uint32_t nt[2] = {(a.n[0] + OB_TILE_ROWS - 1) / OB_TILE_ROWS, (a.n[1] + OB_TILE_ROWS - 1) / OB_TILE_ROWS};
  uint32_t* pre[2] = {a.tprefix + ((size_t)slot * 2) * (a.tiles0 + 1 + nt[1] + 1),
                      a.tprefix + ((size_t)slot * 2) * (a.tiles0 + 1 + nt[1] + 1) + nt[0] + 1};
  if (a.counts && threadIdx.x < 2) {
    const uint32_t g = threadIdx.x, pos = a.seg0 + slot;
    uint32_t s = 0;
    for (uint32_t t = 0; t < nt[g]; ++t) {
      pre[g][t] = s;
      s += a.m1[(size_t)pos * (a.tiles0 + nt[1]) + (g ? a.tiles0 : 0u) + t];
    }
    pre[g][nt[g]] = s;
  }
  __syncthreads();
  const uint32_t na = cnt[0], nb = cnt[1];
  if ((int)na < a.S / 2 || (int)nb < a.S / 2) {  // :231-236
    if (threadIdx.x == 0) {
      a.ok[slot] = 0;
      for (int i = 0; i < 3 * a.n_q; ++i) row[i] = __builtin_nan("");
    }
    return;
  }
  const uint32_t num = min(na, nb);
  const double* XA = a.cols[0];
  const double* XB = a.cols[1];
  for (uint32_t i = threadIdx.x; i < (uint32_t)m2; i += blockDim.x) {
    if (i >= num) {
      yaa[i] = ybb[i] = yab[i] = INFINITY;
      continue;
    }
    const uint32_t ra = position_row(a, slot, 0, ob_mm_pick(i, rep, 0, a.n[0], a.key0, a.key1), pre[0], nt[0]);
    const uint32_t rb = position_row(a, slot, 1, ob_mm_pick(i, rep, 1, a.n[1], a.key0, a.key1), pre[1], nt[1]);
    const double* ba = a.beta + fit_index(a, slot, 0, ia[i]) * K;
    const double* bb = a.beta + fit_index(a, slot, 1, ib[i]) * K;
    double vaa = ba[0], vbb = bb[0], vab = bb[0];  // x_i . beta with x_0 = 1 (:249-255)
    for (int k = 1; k < K; ++k) {
      const double xa = XA[(size_t)(k - 1) * a.ld[0] + ra], xb = XB[(size_t)(k - 1) * a.ld[1] + rb];
      vaa += xa * ba[k];
      vbb += xb * bb[k];
      vab += xa * bb[k];
    }
    yaa[i] = vaa;
    ybb[i] = vbb;
    yab[i] = vab;
  }
  __syncthreads();
  block_sort(yaa, m2);
  block_sort(ybb, m2);
  block_sort(yab, m2);
  if (threadIdx.x == 0) {  // empirical_quantile (:164-171) per target quantile
    for (int j = 0; j < a.n_q; ++j) {
      const uint32_t k = min((uint32_t)((double)num * a.quantiles[j]), num - 1);
      row[3 * j + 0] = yaa[k] - ybb[k];
      row[3 * j + 1] = yab[k] - ybb[k];
      row[3 * j + 2] = yaa[k] - yab[k];
    }
    a.ok[slot] = 1;
  }
}

template <int K>
struct Kernels {
  static void assemble(const MmArgs& a, dim3 grid, int mode, hipStream_t s) {
    if (mode == 2)
      hipLaunchKernelGGL((mm_assemble_mfma_kernel<K, true>), grid, dim3(256), 0, s, a, mode);
    else
      hipLaunchKernelGGL((mm_assemble_mfma_kernel<K, false>), grid, dim3(256), 0, s, a, mode);
  }
  static void affine(const MmArgs& a, dim3 grid, hipStream_t s) {
    hipLaunchKernelGGL(mm_affine_kernel<K>, grid, dim3(256), 0, s, a);
  }
  static void final_(const MmArgs& a, dim3 grid, hipStream_t s) {
    hipLaunchKernelGGL(mm_final_kernel<K>, grid, dim3(256), 0, s, a);
  }
  static void classify(const MmArgs& a, dim3 grid, bool verify, hipStream_t s) {
    if (verify)
      hipLaunchKernelGGL((mm_classify_kernel<K, true>), grid, dim3(256), 0, s, a);
    else
      hipLaunchKernelGGL((mm_classify_kernel<K, false>), grid, dim3(256), 0, s, a);
  }
};

// which: 0 assemble (mode), 1 affine, 2 final, 3 classify, 4 verify
template <int K>
void launch_pass(int which, const MmArgs& a, dim3 grid, int mode, hipStream_t s) {
  if (which == 0)
    Kernels<K>::assemble(a, grid, mode, s);
  else if (which == 1)
    Kernels<K>::affine(a, grid, s);
  else if (which == 2)
    Kernels<K>::final_(a, grid, s);
  else
    Kernels<K>::classify(a, grid, which == 4, s);
}

void pass(int K, int which, const MmArgs& a, dim3 grid, int mode, hipStream_t s) {
  switch (K) {
#define OB_MM_K(k) \
  case k: launch_pass<k>(which, a, grid, mode, s); break;
#ifdef OB_MM_ISA_K  // ISA inspection builds (tools/mm_isa.sh): one width only
    OB_MM_K(OB_MM_ISA_K)
#else
    OB_MM_K(1) OB_MM_K(2) OB_MM_K(3) OB_MM_K(4) OB_MM_K(5) OB_MM_K(6) OB_MM_K(7) OB_MM_K(8)
    OB_MM_K(9) OB_MM_K(10) OB_MM_K(11) OB_MM_K(12) OB_MM_K(13) OB_MM_K(14) OB_MM_K(15) OB_MM_K(16)
    OB_MM_K(17) OB_MM_K(18) OB_MM_K(19) OB_MM_K(20) OB_MM_K(21) OB_MM_K(22) OB_MM_K(23) OB_MM_K(24)
    OB_MM_K(25) OB_MM_K(26) OB_MM_K(27) OB_MM_K(28) OB_MM_K(29) OB_MM_K(30) OB_MM_K(31) OB_MM_K(32)
#endif
#undef OB_MM_K
    default: break;
  }
}

// MM workspace, kept on the panel between calls and grown on demand (the IPM state alone is
// tens of GB: allocating and freeing it per call cost more than the passes at configs[4]).
struct Buffers {
  double *x = nullptr, *z = nullptr, *w = nullptr;
  double *beta = nullptr, *bprev = nullptr, *dba = nullptr, *db = nullptr, *L = nullptr, *fs = nullptr;
  double *partial = nullptr, *red = nullptr, *quant = nullptr, *rows = nullptr;
  uint32_t *fstat = nullptr, *active = nullptr, *tprefix = nullptr, *lane_of = nullptr, *rowlist = nullptr,
           *nrows = nullptr;
  unsigned long long* active_rows = nullptr;
  uint8_t* ok = nullptr;
  double *bvec = nullptr, *rpv = nullptr, *bhat = nullptr;  // row reduction
  uint32_t *samp = nullptr, *nsamp = nullptr;
  double *gchol = nullptr, *lev = nullptr;
  uint32_t* xmask = nullptr;
  static constexpr int kSlots = 29;
  size_t cap[kSlots] = {};
  void** slot(int i) {
    void** v[kSlots] = {(void**)&x, (void**)&z, (void**)&w, (void**)&beta, (void**)&bprev,
                    (void**)&dba, (void**)&db, (void**)&L, (void**)&fs, (void**)&partial, (void**)&red,
                    (void**)&quant, (void**)&rows, (void**)&fstat, (void**)&active, (void**)&active_rows,
                    (void**)&tprefix, (void**)&lane_of, (void**)&rowlist, (void**)&nrows, (void**)&ok,
                    (void**)&bvec, (void**)&rpv, (void**)&bhat, (void**)&samp, (void**)&nsamp,
                    (void**)&gchol, (void**)&lev, (void**)&xmask};
    return v[i];
  }
  // bytes[i] for slot i; reallocates the slots that are too small
  hipError_t reserve(const size_t (&bytes)[kSlots]) {
    for (int i = 0; i < kSlots; ++i) {
      if (bytes[i] <= cap[i]) continue;
      void** q = slot(i);
      (void)hipFree(*q);
      *q = nullptr;
      cap[i] = 0;
      const hipError_t e = hipMalloc(q, bytes[i]);
      if (e != hipSuccess) return e;
      cap[i] = bytes[i];
    }
    return hipSuccess;
  }
  ~Buffers() {
    for (int i = 0; i < kSlots; ++i) (void)hipFree(*slot(i));
  }
};

void free_workspace(void* b) { delete static_cast<Buffers*>(b); }

// Option mm_trace (ob_set_option): per-iteration active fits and the final fit statuses on stderr.
bool trace() { return ob::opt_int(ob::Opt::MmTrace, 0) != 0; }

struct MmStats {
  double assemble_ms = 0.0, fit_rows = 0.0, sync_ms = 0.0;
  int iterations = 0;
  uint64_t retried = 0;  // fits solved again on all rows (row reduction, phase 3)
  std::vector<hipEvent_t> ev;  // pairs around the assemble launches of one ipm() call
  hipError_t events(size_t n) {
    while (ev.size() < n) {
      hipEvent_t e = nullptr;
      const hipError_t r = hipEventCreate(&e);
      if (r != hipSuccess) return r;
      ev.push_back(e);
    }
    return hipSuccess;
  }
  ~MmStats() {
    for (hipEvent_t e : ev) (void)hipEventDestroy(e);
  }
};
constexpr int kCheckEvery = 3;  // iterations between host checks for live fits (extra ones are no-ops)

struct Reduction {  // the row reduction's phase-1 geometry and list regions (mm_run)
  bool on = false;
  uint32_t nch1[2] = {0, 0};
  uint32_t *list1 = nullptr, *nrows1 = nullptr;
  double* gchol = nullptr;
  double *beta1 = nullptr, *bprev1 = nullptr, *dba1 = nullptr, *db1 = nullptr, *L1 = nullptr, *fs1 = nullptr;
  uint32_t* fstat1 = nullptr;  // phase 1's fit arrays (past the full fits' in the same buffers)
};

hipError_t reduce_partials(const MmArgs& a, int nv, int n_min, int skip_dead, hipStream_t s) {
  const size_t tot = (size_t)a.n_rb * 2 * a.S_pad * nv;
  hipLaunchKernelGGL(mm_reduce_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, a, nv, n_min, skip_dead);
  return hipGetLastError();
}

// Row lists, the OLS start per (slot, group), the tau order and the shifted start (phase 1, or the
// whole solve without the reduction); a.active_rows <- the live (fit, row) pairs of the first assemble.
// With the reduction, `full` holds every quantile: the order kernel sorts them there and phase 1 (a)
// takes every f-th lane's tau (mm_subtau_kernel).
int start_fits(const MmArgs& a, int K, hipStream_t s, const MmArgs* full = nullptr, int f = 1) {
  const uint32_t nch = a.nch[0] + a.nch[1];
  const size_t lds_solve = sizeof(double) * ((size_t)K * K + K);
  hipLaunchKernelGGL(mm_rows_kernel, dim3(nch, 1, a.n_rb), dim3(256), 0, s, a);
  MM_OK(hipGetLastError());
  MM_OK(hipMemsetAsync(a.active_rows, 0, sizeof(unsigned long long), s));
  pass(K, 0, a, dim3(nch, 1, a.n_rb), 0, s);
  MM_OK(hipGetLastError());
  MM_OK(reduce_partials(a, nv_asm(K), 0, 0, s));  // the OLS sums sit in fit 0 (the statuses are not set yet)
  hipLaunchKernelGGL(mm_start_kernel, dim3(a.n_rb * 2), dim3(64), lds_solve, s, a, K);
  MM_OK(hipGetLastError());
  const MmArgs& ao = full ? *full : a;
  int m2 = 1;
  while (m2 < ao.S) m2 <<= 1;
  const size_t lds_ord = (size_t)m2 * (sizeof(double) + sizeof(uint32_t));
  MM_OK(hipFuncSetAttribute((const void*)mm_order_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_ord));
  hipLaunchKernelGGL(mm_order_kernel, dim3(ao.n_rb * 2), dim3(256), lds_ord, s, ao, m2);
  MM_OK(hipGetLastError());
  if (full) {
    hipLaunchKernelGGL(mm_subtau_kernel, dim3((unsigned)(((size_t)a.n_rb * 2 * a.S_pad + 255) / 256)), dim3(256), 0, s,
                       *full, a, f);
    MM_OK(hipGetLastError());
  }
  hipLaunchKernelGGL(mm_shift_kernel, dim3(a.n_rb * 2), dim3(1024), 0, s, a, K);
  MM_OK(hipGetLastError());
  return OB_OK;
}

// Interior-point iterations over the live fits (first assemble in first_mode: 1 shifted start, 3
// centred start) until none is active or kMmMaxIter; the fits still live then fail. The host
// looks at the live count every kCheckEvery iterations (converged fits skip every kernel, so the
// iterations past the last live fit cost only launches). a.active_rows accumulates the live
// (fit, row) pairs of the assembles (the caller seeds it with the first one's).
int ipm(const MmArgs& a, int K, int first_mode, hipStream_t s, MmStats& st) {
  const uint32_t nch = a.nch[0] + a.nch[1];
  const int nv1 = nv_asm(K), nv2 = 5 + 2 * K;
  const size_t n_fits = (size_t)a.n_rb * 2 * a.S_pad;
  const dim3 grid(nch, a.S_pad / 64, a.n_rb);
  const size_t lds_solve = sizeof(double) * ((size_t)K * K + K);
  MM_OK(st.events(2 * (size_t)ob::kMmMaxIter));
  int it = 0;
  for (it = 1; it <= ob::kMmMaxIter; ++it) {
    MM_OK(hipEventRecord(st.ev[2 * (it - 1)], s));
    pass(K, 0, a, grid, it == 1 ? first_mode : 2, s);
    MM_OK(hipGetLastError());
    MM_OK(hipEventRecord(st.ev[2 * (it - 1) + 1], s));
    MM_OK(reduce_partials(a, nv1, 0, 1, s));
    MM_OK(hipMemsetAsync(a.active, 0, sizeof(uint32_t), s));
    hipLaunchKernelGGL(mm_solve_affine_kernel, dim3((unsigned)n_fits), dim3(64), lds_solve, s, a, K,
                       a.rp ? (it == 1 ? 1 : 2) : 0);
    MM_OK(hipGetLastError());
    if (it % kCheckEvery == 0 || it == ob::kMmMaxIter) {
      uint32_t active = 0;
      MM_OK(hipMemcpyAsync(&active, a.active, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
      const auto ts = std::chrono::steady_clock::now();
      MM_OK(hipStreamSynchronize(s));
      st.sync_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - ts).count();
      if (trace()) {
        fprintf(stderr, "[mm] iteration %d: %u of %zu fits active\n", it, active, n_fits);
        if (active && active <= 4) {  // the last live fits: where they stand
          std::vector<uint32_t> fst(n_fits);
          std::vector<double> fsh(n_fits * kFs);
          MM_OK(hipMemcpy(fst.data(), a.fstat, sizeof(uint32_t) * n_fits, hipMemcpyDeviceToHost));
          MM_OK(hipMemcpy(fsh.data(), a.fs, sizeof(double) * n_fits * kFs, hipMemcpyDeviceToHost));
          for (size_t f = 0; f < n_fits; ++f)
            if ((int)(f % a.S_pad) < a.S && !(fst[f] & (kDone | kFailed))) {
              const double* q = fsh.data() + f * kFs;
              fprintf(stderr, "[mm]   live fit %zu tau %.5f gap %.3e obj %.6e rel %.3e mu %.3e ap %.3e ad %.3e nact %.0f\n",
                      f, q[FS_TAU], q[FS_GAP], q[FS_OBJ], q[FS_GAP] / (1 + fabs(q[FS_OBJ])), q[FS_MU], q[FS_AP],
                      q[FS_AD], q[FS_NACT]);
            }
        }
      }
      if (active == 0) break;
    }
    pass(K, 1, a, grid, 0, s);
    MM_OK(hipGetLastError());
    MM_OK(reduce_partials(a, nv2, 2, 1, s));
    hipLaunchKernelGGL(mm_solve_corrector_kernel, dim3((unsigned)n_fits), dim3(64), lds_solve, s, a, K);
    MM_OK(hipGetLastError());
    pass(K, 2, a, grid, 0, s);
    MM_OK(hipGetLastError());
    MM_OK(reduce_partials(a, 2, 2, 1, s));
    hipLaunchKernelGGL(mm_step_kernel, dim3((unsigned)((n_fits + 255) / 256)), dim3(256), 0, s, a, K, n_fits);
    MM_OK(hipGetLastError());
  }
  {
    unsigned long long rows = 0;
    MM_OK(hipMemcpyAsync(&rows, a.active_rows, sizeof(rows), hipMemcpyDeviceToHost, s));
    MM_OK(hipStreamSynchronize(s));
    st.fit_rows += (double)rows;
    for (int i = 0; i < std::min(it, ob::kMmMaxIter); ++i) {
      float ms = 0.f;
      MM_OK(hipEventElapsedTime(&ms, st.ev[2 * i], st.ev[2 * i + 1]));
      st.assemble_ms += ms;
    }
  }
  if (trace()) {
    MM_OK(hipStreamSynchronize(s));
    std::vector<uint32_t> fst(n_fits);
    std::vector<double> fsh(n_fits * kFs);
    MM_OK(hipMemcpy(fst.data(), a.fstat, sizeof(uint32_t) * n_fits, hipMemcpyDeviceToHost));
    MM_OK(hipMemcpy(fsh.data(), a.fs, sizeof(double) * n_fits * kFs, hipMemcpyDeviceToHost));
    size_t done = 0, failed = 0, live = 0;
    for (size_t f = 0; f < n_fits; ++f) {
      if ((int)(f % a.S_pad) >= a.S) continue;
      if (fst[f] == kDone) ++done;
      else if (fst[f] & kFailed) ++failed;
      else {
        if (live < 8)
          fprintf(stderr, "[mm] live fit %zu tau %.4f gap %.3e obj %.3e rel %.3e\n", f, fsh[f * kFs + FS_TAU],
                  fsh[f * kFs + FS_GAP], fsh[f * kFs + FS_OBJ], fsh[f * kFs + FS_GAP] / (1 + fabs(fsh[f * kFs + FS_OBJ])));
        ++live;
      }
    }
    fprintf(stderr, "[mm] after %d iterations: %zu converged, %zu failed, %zu still live\n", it, done, failed, live);
  }
  hipLaunchKernelGGL(mm_expire_kernel, dim3((unsigned)((n_fits + 255) / 256)), dim3(256), 0, s, a, n_fits);
  MM_OK(hipGetLastError());
  st.iterations = std::max(st.iterations, std::min(it, ob::kMmMaxIter));
  return OB_OK;
}

// Phases 2 (round 0: reduced problems from the bands) and 3 (round 1: the flagged fits on all rows).
int reduced_round(const MmArgs& a, int K, int round, hipStream_t s, MmStats& st) {
  const uint32_t nch = a.nch[0] + a.nch[1];
  const size_t n_fits = (size_t)a.n_rb * 2 * a.S_pad;
  const dim3 grid(nch, a.S_pad / 64, a.n_rb);
  const unsigned fit_blocks = (unsigned)((n_fits + 255) / 256);
  MM_OK(hipMemsetAsync(a.active_rows, 0, sizeof(unsigned long long), s));
  MmArgs ac = a;
  ac.list_stat = trace() && round == 0;
  if (ac.list_stat) {
    const unsigned long long z[2] = {0ull, 0ull};
    MM_OK(hipMemcpyToSymbolAsync(HIP_SYMBOL(g_mm_list_stat), z, sizeof(z), 0, hipMemcpyHostToDevice, s));
  }
  pass(K, 3, ac, grid, 0, s);  // classify: block lists + fixed-row sums
  MM_OK(hipGetLastError());
  if (ac.list_stat) {
    unsigned long long v[2];
    MM_OK(hipMemcpyFromSymbolAsync(v, HIP_SYMBOL(g_mm_list_stat), sizeof(v), 0, hipMemcpyDeviceToHost, s));
    MM_OK(hipStreamSynchronize(s));
    fprintf(stderr, "[mm] block lists: %llu (wave, entry) pairs, %llu (%.1f %%) needed by a fit of the wave\n", v[0],
            v[1], v[0] ? 100.0 * (double)v[1] / (double)v[0] : 0.0);
  }
  MM_OK(reduce_partials(a, nv_cls(K), 0, 0, s));
  hipLaunchKernelGGL(mm_bvec_kernel, dim3(fit_blocks), dim3(256), 0, s, a, K, n_fits, round == 0 ? 1 : 0);
  MM_OK(hipGetLastError());
  MmArgs a2 = a;
  a2.block_lists = 1;
  a2.rowlist = a.blist;
  a2.nrows = a.bnrows;
  a2.rp = 1;
  const double d2 = ob::opt_double(ob::Opt::MmDelta2, 0.0);  // option mm_delta2: tuning
  a2.dscale = d2 > 0.0 ? d2 : kDelta2;
  return ipm(a2, K, 3, s, st);
}

// ob_debug_mm_betas (tests only): the per-fit coefficients of slot 0 of the next batch run, per group
// in simulation order (NaN where the fit failed), and the fit statuses (1 converged).
struct MmCapture {
  bool on = false;
  double* beta = nullptr;  // [2][S][K]
  uint8_t* done = nullptr;  // [2][S]
};
MmCapture g_capture;

int capture_fits(const MmArgs& a, int K, hipStream_t s) {
  const size_t nf = (size_t)2 * a.S_pad;  // slot 0: fit_index(a, 0, g, j) = g S_pad + j
  std::vector<uint32_t> lane(nf), fst(nf);
  std::vector<double> beta(nf * K);
  MM_OK(hipStreamSynchronize(s));
  MM_OK(hipMemcpy(lane.data(), a.lane_of, sizeof(uint32_t) * nf, hipMemcpyDeviceToHost));
  MM_OK(hipMemcpy(fst.data(), a.fstat, sizeof(uint32_t) * nf, hipMemcpyDeviceToHost));
  MM_OK(hipMemcpy(beta.data(), a.beta, sizeof(double) * nf * K, hipMemcpyDeviceToHost));
  for (int g = 0; g < 2; ++g)
    for (int sm = 0; sm < a.S; ++sm) {
      const size_t f = (size_t)g * a.S_pad + lane[(size_t)g * a.S_pad + sm];
      const bool ok = fst[f] == kDone;
      g_capture.done[(size_t)g * a.S + sm] = ok ? 1 : 0;
      for (int k = 0; k < K; ++k)
        g_capture.beta[((size_t)g * a.S + sm) * K + k] = ok ? beta[f * K + k] : __builtin_nan("");
    }
  g_capture.on = false;
  return OB_OK;
}

// One batch of replicate slots: start, IPM iterations (with the row reduction: phase 1 on the
// subsample, bands, phase 2 on the reduced lists, verification, phase 3 for flagged fits),
// finish. Rows/ok -> host.
int run_batch(MmArgs a, int K, hipStream_t s, double* rows_h, uint8_t* ok_h, MmStats& st, const Reduction& rd) {
  const size_t n_fits = (size_t)a.n_rb * 2 * a.S_pad;
  const uint32_t nch = a.nch[0] + a.nch[1];
  int m2 = 1;
  while (m2 < a.S) m2 <<= 1;
  if (!rd.on) {
    OB_TRY(start_fits(a, K, s));
    OB_TRY(ipm(a, K, 1, s, st));
  } else {
    hipLaunchKernelGGL(mm_rows_kernel, dim3(nch, 1, a.n_rb), dim3(256), 0, s, a);  // the full lists
    MM_OK(hipGetLastError());
    MmArgs a1 = a;  // phase 1: every kSubStride-th row, chunks of kRc1 rows
    a1.rc = kRc1;
    a1.cap = kRc1 / kSubStride;
    a1.stride = kSubStride;
    a1.nch[0] = rd.nch1[0];
    a1.nch[1] = rd.nch1[1];
    a1.rowlist = rd.list1;
    a1.nrows = rd.nrows1;
    const double tol1 = ob::opt_double(ob::Opt::MmTol1, 0.0);  // option mm_tol1 (the verification keeps results exact)
    a1.tol = tol1 > 0.0 ? tol1 : kPhase1Tol;
    a1.gchol = rd.gchol;
    const double d1 = ob::opt_double(ob::Opt::MmDelta1, 0.0);  // option mm_delta1: tuning
    a1.dscale = d1 > 0.0 ? d1 : kDelta1;
    // phase 1 solves S1 of the S quantiles (their own fit arrays); the others interpolate
    const int fs_opt = ob::opt_int(ob::Opt::MmFitStride, 0);  // option mm_fit_stride: tuning
    const int fstride = fs_opt > 0 ? fs_opt : kFitStride;
    const int f = a.S >= kFitStrideMin ? fstride : 1;
    a1.S = f > 1 ? (a.S - 1 + f - 1) / f + 1 : a.S;
    a1.S_pad = (a1.S + 63) / 64 * 64;
    a1.beta = rd.beta1;
    a1.bprev = rd.bprev1;
    a1.dba = rd.dba1;
    a1.db = rd.db1;
    a1.L = rd.L1;
    a1.fs = rd.fs1;
    a1.fstat = rd.fstat1;
    const auto tb = std::chrono::steady_clock::now();
    OB_TRY(start_fits(a1, K, s, &a, f));
    OB_TRY(ipm(a1, K, 1, s, st));
    hipLaunchKernelGGL(mm_interp_kernel, dim3((unsigned)((n_fits + 255) / 256)), dim3(256), 0, s, a, a1, K, f);
    MM_OK(hipGetLastError());
    if (trace()) {
      MM_OK(hipStreamSynchronize(s));
      fprintf(stderr, "[mm] phase 1 done at %.1f ms\n",
              std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tb).count());
    }
    hipLaunchKernelGGL(mm_sample_kernel, dim3(a.n_rb * 2), dim3(1024), 0, s, a);
    MM_OK(hipGetLastError());
    MmArgs al = a;
    al.gchol = rd.gchol;
    hipLaunchKernelGGL(mm_lev_kernel, dim3(nch, 1, a.n_rb), dim3(256), 0, s, al, K);
    MM_OK(hipGetLastError());
    const double kappa_opt = ob::opt_double(ob::Opt::MmKappa, 0.0);  // options mm_kappa, mm_band0: tuning
    const double kappa = kappa_opt > 0.0 ? kappa_opt : kBandKappa;
    const double band0 = ob::opt_double(ob::Opt::MmBand0, kBand0);
    hipLaunchKernelGGL(mm_band_kernel, dim3((unsigned)n_fits), dim3(256), 0, s, a, K, kappa, band0);
    MM_OK(hipGetLastError());
    MM_OK(hipMemsetAsync(a.xmask, 0, sizeof(uint32_t) * (size_t)a.n_rb * nch * (a.S_pad / 64) * (a.cap / 32), s));
    // round 0: the bands; round 1: flagged fits, their bands plus the wrong-signed rows; round 2:
    // fits flagged again, on all rows (no verification: nothing is fixed)
    for (int round = 0; round < 3; ++round) {
      OB_TRY(reduced_round(a, K, round, s, st));
      if (round == 2) break;
      MM_OK(hipMemsetAsync(a.active, 0, sizeof(uint32_t), s));
      pass(K, 4, a, dim3(nch, a.S_pad / 64, a.n_rb), 0, s);  // verify the fixed rows' signs
      MM_OK(hipGetLastError());
      if (trace()) {  // why fits go to the next round: wrong-signed fixed rows or failures (with tau)
        MM_OK(hipStreamSynchronize(s));
        std::vector<uint32_t> fst(n_fits);
        std::vector<double> fsh(n_fits * kFs);
        MM_OK(hipMemcpy(fst.data(), a.fstat, sizeof(uint32_t) * n_fits, hipMemcpyDeviceToHost));
        MM_OK(hipMemcpy(fsh.data(), a.fs, sizeof(double) * n_fits * kFs, hipMemcpyDeviceToHost));
        int nv = 0, nf = 0;
        for (size_t f = 0; f < n_fits; ++f) {
          if ((int)(f % a.S_pad) >= a.S || fst[f] == kDone) continue;
          const bool v = fst[f] & kRetry;
          nv += v;
          nf += !v;
          if (nv + nf <= 6)
            fprintf(stderr, "[mm]   fit %zu tau %.4f %s nact %.0f lo %.3g hi %.3g ext %.3g\n", f, fsh[f * kFs + FS_TAU],
                    v ? "sign" : "failed", fsh[f * kFs + FS_NACT], fsh[f * kFs + FS_LO], fsh[f * kFs + FS_HI],
                    fsh[f * kFs + FS_EXT]);
        }
        fprintf(stderr, "[mm] round %d at %.1f ms: %d fits with a wrong-signed fixed row, %d failures\n", round,
                std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tb).count(), nv, nf);
      }
      hipLaunchKernelGGL(mm_retry_kernel, dim3((unsigned)((n_fits + 255) / 256)), dim3(256), 0, s, a, K, n_fits,
                         round == 1 ? 1 : 0);
      MM_OK(hipGetLastError());
      uint32_t retry = 0;
      MM_OK(hipMemcpyAsync(&retry, a.active, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
      MM_OK(hipStreamSynchronize(s));
      st.retried += retry;
      if (!retry) break;
    }
    if (trace()) {
      MM_OK(hipStreamSynchronize(s));
      fprintf(stderr, "[mm] batch done at %.1f ms\n",
              std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tb).count());
    }
  }
  const size_t lds_fin = (size_t)m2 * (3 * sizeof(double) + 2 * sizeof(uint16_t));
  MM_OK(hipFuncSetAttribute((const void*)mm_finish_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_fin));
  hipLaunchKernelGGL(mm_finish_kernel, dim3(a.n_rb), dim3(256), lds_fin, s, a, K, m2);
  MM_OK(hipGetLastError());
  MM_OK(hipMemcpyAsync(rows_h, a.rows, sizeof(double) * a.n_rb * 3 * a.n_q, hipMemcpyDeviceToHost, s));
  MM_OK(hipMemcpyAsync(ok_h, a.ok, a.n_rb, hipMemcpyDeviceToHost, s));
  MM_OK(hipStreamSynchronize(s));
  if (g_capture.on) OB_TRY(capture_fits(a, K, s));
  return OB_OK;
}

}  // namespace

namespace ob {

static int mm_run_impl(ob_panel* p, uint64_t seed, int sims, const double* quantiles, int n_q, uint64_t first_rep,
                       uint64_t n_reps, bool with_point, double* rows, uint8_t* ok, int* max_iters);

// Machado-Mata on the context stream, ordered after any call on this panel from another stream
// (engine_order: an async boot on a user stream may still read the count images and flags this
// run rewrites) and marked so that the next call on another stream waits for it.
int mm_run(ob_panel* p, uint64_t seed, int sims, const double* quantiles, int n_q, uint64_t first_rep,
           uint64_t n_reps, bool with_point, double* rows, uint8_t* ok, int* max_iters) {
  MM_OK(hipSetDevice(p->ctx->device));
  OB_TRY(ob::engine_order(p, p->ctx->stream));
  const int rc = mm_run_impl(p, seed, sims, quantiles, n_q, first_rep, n_reps, with_point, rows, ok, max_iters);
  const int rm = ob::engine_mark(p, p->ctx->stream);
  return rc != OB_OK ? rc : rm;
}

static int mm_run_impl(ob_panel* p, uint64_t seed, int sims, const double* quantiles, int n_q, uint64_t first_rep,
                       uint64_t n_reps, bool with_point, double* rows, uint8_t* ok, int* max_iters) {
  ob_ctx* ctx = p->ctx;
  MM_OK(hipSetDevice(ctx->device));
  const int K = p->k;
  if (K > kMmMaxK) return ob::fail(OB_E_UNSUPPORTED, "Machado-Mata takes at most %d columns (intercept included), got %d", kMmMaxK, K);
  if (p->weighted || p->heckman || p->n_y != 1) return ob::fail(OB_E_INVALID, "Machado-Mata panels are unweighted, one outcome");
  if (sims < 1 || sims > kMmMaxSims) return ob::fail(OB_E_UNSUPPORTED, "simulations must be in [1, %d]", kMmMaxSims);
  if (n_q < 1) return ob::fail(OB_E_INVALID, "no target quantiles");
  if (p->n[0] < 1 || p->n[1] < 1) return ob::fail(OB_E_GROUP, "%sOne group has insufficient data", error_prefix(OB_E_GROUP));
  if (first_rep + n_reps >= 0xFFFFFFFFull) return ob::fail(OB_E_INVALID, "replicate ids must stay below 2^32 - 1");
  hipStream_t s = ctx->stream;
  const int S_pad = (sims + 63) / 64 * 64;
  const size_t rep_rows = (size_t)p->n[0] + p->n[1];
  if (p->n[0] > 1024u * kRc || p->n[1] > 1024u * kRc)  // mm_shift_kernel's chunk prefix (1024 chunks)
    return ob::fail(OB_E_UNSUPPORTED, "Machado-Mata groups take at most %u rows", 1024u * kRc);
  // Row reduction: option mm_reduce 0 off, 1 on; by default on when both groups have >= 2^16 rows.
  Reduction rd;
  {
    const int r = ob::opt_int(ob::Opt::MmReduce, -1);
    rd.on = r >= 0 ? r != 0 : (p->n[0] >= 65536u && p->n[1] >= 65536u);
  }
  const uint32_t rcF = rd.on ? kRcF : kRc;  // the full lists' chunk rows (= their capacity)
  const uint32_t nch0 = (p->n[0] + rcF - 1) / rcF, nch1 = (p->n[1] + rcF - 1) / rcF;
  // replicate slots per batch: IPM state (x, z, w: 3 f64 per fit and list entry, rcF entries per
  // chunk) within option mm_state_gb (default 160 of the 288 GB): a batch's tail iterations (few
  // live fits) and phase 1 cost about the same time for 2 or 12 replicates, so wider batches
  // amortize them
  const double sgb = ob::opt_double(ob::Opt::MmStateGb, 0.0);
  const uint64_t state_budget = (uint64_t)((sgb > 0.0 ? sgb : 160.0) * (double)(1ull << 30));
  const size_t state_rows = (size_t)(nch0 + nch1) * rcF;
  const size_t state_per_rep = 3 * state_rows * S_pad * sizeof(double);
  const uint64_t want = std::max<uint64_t>(n_reps, 1);
  size_t free_b = 0, total_b = 0;
  MM_OK(hipMemGetInfo(&free_b, &total_b));
  size_t held = 0;  // this panel's state slots from an earlier call count as free
  if (p->mm_ws)
    for (int i = 0; i < 3; ++i) held += static_cast<Buffers*>(p->mm_ws)->cap[i];
  const uint64_t budget = std::min<uint64_t>(state_budget, (uint64_t)((free_b + held) * 0.8));
  const uint32_t rb_cap = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>({want, 256, budget / state_per_rep}));
  const size_t fits = (size_t)rb_cap * 2 * S_pad;
  const size_t fitsx = 2 * fits;  // fit arrays: the full fits, then phase 1's (at most as many)
  const int nv_max = nv_asm(K);  // >= 5 + 2 K (affine) and nv_cls(K)
  const uint32_t rc1 = kRc1;
  rd.nch1[0] = (p->n[0] + rc1 - 1) / rc1;
  rd.nch1[1] = (p->n[1] + rc1 - 1) / rc1;
  const size_t nfb = (size_t)S_pad / 64;
  const size_t lists_full = (size_t)rb_cap * (nch0 + nch1), lists_blk = rd.on ? lists_full * nfb : 0,
               lists_p1 = rd.on ? (size_t)rb_cap * (rd.nch1[0] + rd.nch1[1]) : 0;
  const size_t cap1 = kRc1 / kSubStride;
  const size_t list_words = (lists_full + lists_blk) * rcF + lists_p1 * cap1;
  const size_t nch_max = std::max<size_t>(nch0 + nch1, rd.on ? rd.nch1[0] + rd.nch1[1] : 0);  // partials
  const size_t n_lists = lists_full + lists_blk + lists_p1;
  if (!p->mm_ws) {
    p->mm_ws = new Buffers();
    p->mm_ws_free = free_workspace;
  }
  Buffers& b = *static_cast<Buffers*>(p->mm_ws);
  const size_t st_elems = (size_t)rb_cap * state_rows * S_pad;
  const uint32_t nt1 = (p->n[1] + OB_TILE_ROWS - 1) / OB_TILE_ROWS;
  const size_t d8 = sizeof(double), u4 = sizeof(uint32_t);
  const size_t need[Buffers::kSlots] = {d8 * st_elems, d8 * st_elems, d8 * st_elems, d8 * fitsx * K,
                           d8 * fitsx * K, d8 * fitsx * K, d8 * fitsx * K, d8 * fitsx * K * K,
                           d8 * fitsx * kFs, d8 * (size_t)rb_cap * nch_max * S_pad * nv_max,
                           d8 * fits * nv_max, d8 * n_q, d8 * rb_cap * 3 * n_q, u4 * fitsx, u4,
                           sizeof(unsigned long long), u4 * rb_cap * 2 * (p->ntiles[0] + 1 + nt1 + 1), u4 * fits,
                           u4 * list_words, u4 * n_lists, rb_cap, d8 * fits * K, d8 * fits * K,
                           d8 * fits * K, u4 * (size_t)rb_cap * 2 * 2 * kBandSamples, u4 * (size_t)rb_cap * 2,
                           d8 * (size_t)rb_cap * 2 * (K * K + 1), d8 * lists_full * rcF,
                           u4 * (lists_blk ? lists_blk : 1) * (rcF / 32)};
  MM_OK(b.reserve(need));
  MM_OK(hipMemcpy(b.quant, quantiles, sizeof(double) * n_q, hipMemcpyHostToDevice));

  // the overflow word of this call's count images (engine_counts ORs into d_flags[2] over every
  // segment; word 0 is the boot calls' and may belong to an async boot not yet collected)
  MM_OK(hipMemsetAsync(p->d_flags + 2, 0, sizeof(uint32_t), s));
  MmArgs a{};
  for (int g = 0; g < 2; ++g) {
    a.cols[g] = p->d_cols[g];
    a.ld[g] = p->ld[g];
    a.n[g] = p->n[g];
  }
  a.tiles0 = p->ntiles[0];
  a.p = p->p;
  a.S = sims;
  a.S_pad = S_pad;
  a.nch[0] = nch0;
  a.nch[1] = nch1;
  a.rep_rows = rep_rows;
  a.x = b.x;
  a.z = b.z;
  a.w = b.w;
  a.beta = b.beta;
  a.bprev = b.bprev;
  a.dba = b.dba;
  a.db = b.db;
  a.L = b.L;
  a.fs = b.fs;
  a.fstat = b.fstat;
  a.partial = b.partial;
  a.red = b.red;
  a.active = b.active;
  a.active_rows = b.active_rows;
  a.tprefix = b.tprefix;
  a.lane_of = b.lane_of;
  a.rowlist = b.rowlist;
  a.nrows = b.nrows;
  a.rc = rcF;
  a.stride = 1;
  a.cap = rcF;
  a.tol = kTol;
  a.trace = trace() ? 1 : 0;
  a.blist = b.rowlist + lists_full * rcF;
  a.bnrows = b.nrows + lists_full;
  rd.list1 = b.rowlist + (lists_full + lists_blk) * rcF;
  rd.nrows1 = b.nrows + lists_full + lists_blk;
  rd.gchol = b.gchol;
  rd.beta1 = b.beta + fits * K;
  rd.bprev1 = b.bprev + fits * K;
  rd.dba1 = b.dba + fits * K;
  rd.db1 = b.db + fits * K;
  rd.L1 = b.L + fits * K * K;
  rd.fs1 = b.fs + fits * kFs;
  rd.fstat1 = b.fstat + fits;
  a.bvec = b.bvec;
  a.rpv = b.rpv;
  a.bhat = b.bhat;
  a.samp = b.samp;
  a.nsamp = b.nsamp;
  a.lev = b.lev;
  a.xmask = b.xmask;
  a.key0 = (uint32_t)seed;
  a.key1 = (uint32_t)(seed >> 32);
  a.n_q = n_q;
  a.quantiles = b.quant;
  a.rows = b.rows;
  a.ok = b.ok;
  a.fail_mask = p->d_mm_fail;
  a.fail_sims = p->mm_fail_sims;
  const auto t0 = std::chrono::steady_clock::now();
  MmStats st;
  size_t out = 0;
  if (with_point) {  // every row once, MM-1 replicate OB_MM_POINT_REP
    MmArgs pa = a;
    pa.n_rb = 1;
    pa.rep0 = OB_MM_POINT_REP;
    pa.counts = nullptr;
    OB_TRY(run_batch(pa, K, s, rows, ok, st, rd));
    out = 1;
  }
  // resamples: OBRS-3 count images per segment, then batches of rb_cap slots
  const uint64_t seg_cap = 4096;
  for (uint64_t s0 = 0; s0 < n_reps; s0 += seg_cap) {
    const uint32_t ns = (uint32_t)std::min<uint64_t>(seg_cap, n_reps - s0);
    uint32_t nb_rep = 0, rep_pad = 0;
    OB_TRY(engine_counts(p, seed, first_rep + s0, ns, s, &nb_rep, &rep_pad));
    for (uint32_t b0 = 0; b0 < ns; b0 += rb_cap) {
      MmArgs ba = a;
      ba.n_rb = std::min(rb_cap, ns - b0);
      ba.rep0 = (uint32_t)(first_rep + s0 + b0);
      ba.seg0 = b0;
      ba.counts = p->d_counts;
      ba.m1 = p->d_m1;
      ba.nb_rep = nb_rep;
      ba.rep_pad = rep_pad;
      OB_TRY(run_batch(ba, K, s, rows + (out + s0 + b0) * 3 * n_q, ok + out + s0 + b0, st, rd));
    }
  }
  uint32_t flag = 0;
  MM_OK(hipMemcpy(&flag, p->d_flags + 2, sizeof(uint32_t), hipMemcpyDeviceToHost));
  if (flag) return ob::fail(OB_E_OVERFLOW, "a resampled row was drawn more than 255 times in one replicate");
  p->timing.mm_assemble_ms = st.assemble_ms;
  p->timing.mm_fit_rows = st.fit_rows;
  p->timing.mm_iterations = st.iterations;
  p->timing.mm_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  p->timing.mm_reduced = rd.on ? 1 : 0;
  p->timing.mm_retried = (int64_t)st.retried;
  if (trace())
    fprintf(stderr, "[mm] call: %.1f ms, %.1f ms waiting in per-iteration syncs, assemble %.1f ms\n", p->timing.mm_ms,
            st.sync_ms, st.assemble_ms);
  if (max_iters) *max_iters = st.iterations;
  return OB_OK;
}

}  // namespace ob

extern "C" int ob_mm_run(ob_panel* panel, uint64_t seed, int32_t simulations, const double* quantiles,
                         int32_t n_quantiles, uint64_t first_rep, uint64_t n_reps, int32_t with_point,
                         double* rows, uint8_t* ok) {
  if (!panel || !quantiles || !rows || !ok) return ob::fail(OB_E_INVALID, "null pointer");
  return ob::mm_run(panel, seed, simulations, quantiles, n_quantiles, first_rep, n_reps, with_point != 0, rows, ok,
                    nullptr);
}

// Test hook (include/oaxaca_boot.h): one MM pass (rep = OB_MM_POINT_REP for the point pass) and
// the coefficients of its 2 x sims quantile regressions.
extern "C" int ob_debug_mm_betas(ob_panel* p, uint64_t seed, int32_t simulations, uint64_t rep, double* betas,
                                 uint8_t* done) {
  if (!p || !betas || !done) return ob::fail(OB_E_INVALID, "null pointer");
  const double q = 0.5;
  double row[3];
  uint8_t ok = 0;
  g_capture.on = true;
  g_capture.beta = betas;
  g_capture.done = done;
  const bool point = rep == OB_MM_POINT_REP;
  const int rc = ob::mm_run(p, seed, simulations, &q, 1, point ? 0 : rep, point ? 0 : 1, point, row, &ok, nullptr);
  g_capture.on = false;
  return rc;
}

extern "C" int ob_debug_mm_fail(ob_panel* p, const uint8_t* mask, int32_t sims) {
  if (!p || sims < 0 || (sims && !mask)) return ob::fail(OB_E_INVALID, "bad arguments");
  MM_OK(hipSetDevice(p->ctx->device));
  (void)hipFree(p->d_mm_fail);
  p->d_mm_fail = nullptr;
  p->mm_fail_sims = 0;
  if (sims == 0) return OB_OK;
  MM_OK(hipMalloc(&p->d_mm_fail, 2 * (size_t)sims));
  MM_OK(hipMemcpy(p->d_mm_fail, mask, 2 * (size_t)sims, hipMemcpyHostToDevice));
  p->mm_fail_sims = sims;
  return OB_OK;
}
