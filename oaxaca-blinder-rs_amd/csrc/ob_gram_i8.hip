// ob_gram_i8.hip -- the counts-weighted extended Gram as an exact integer GEMM on i8 MFMA.
//
// Same quantity as ob_gram_kernel (ob_engine.hip): per replicate r and row chunk,
//   G_r[e] = sum_i c_{r,i} P_i[e],   P_i[e] = v_i[a(e)] v_i[b(e)],  v = sqrt(w) [1, x, y]
// (the reference's own sqrt(w) scaling, ols.rs:68-78; X^T W X, X^T W y, sum w and the weighted
// sums of estimation.rs:56-71 are all entries of G). Counts are small integers, so the
// resample weighting is exact in int8; the pair products are written once per panel as S = 7
// balanced 8-bit digits (Ozaki-style splitting) of a 54-bit fixed-point value relative to the
// per-(chunk, pair) power of two 2^E with 2^(E-1) <= max |P| < 2^E:
//     m = rint(P 2^(54-E)),  |m| <= 2^54,   m = sum_s d_s 2^(8 (6 - s)),  d_s in [-128, 127]
// (|d_0| <= 64), so |P - m 2^(E-54)| <= 2^(E-55) <= 2^-54 max |P| -- finer than f64's own
// rounding of the chunk's largest product. Then
//     sum_i c_i P_i = 2^(E-54) sum_s 2^(8 (6 - s)) sum_i c_i d_{s,i},
// each inner sum an exact int32 (|c| <= 127, |d| <= 128, sum_i c_i <= n_g < 2^24 (oz_prepare), so
// |sum| < 2^31). The slices meet in int64, two f64 roundings per chunk partial, so the Gram
// equals the f64 MFMA Gram to ~1e-15 relative (tests/test_gpu_gram_i8.py holds it to 1e-12).
//
// v_mfma_i32_16x16x64_i8 issues in 16 cycles like v_mfma_f32_16x16x32_bf16 (MI355X_MICROARCH.md,
// Matrix cores): 64x the f64 MFMA rate, so 7 slices cost 7x the f64 multiply count and still
// leave 9x headroom. Layouts (HBM, built once per panel):
//   B (digits): per group [sub-tile 64 rows][col tile: 32 pairs][slice][pair block h][lane][16 B]
//               -- lane l holds pair 16 h + (l & 15), rows 16 (l >> 4) + j: the B fragment of
//               16x16x64_i8 (probed: tools/mfma_i8_probe.hip), one 14 KB DMA per sub-tile.
//   A (counts): ob_count_kernel<true> writes [tile][64-rep batch][sub-tile][rep block m][lane][16 B]
//               -- lane l holds replicate 16 m + (l & 15), the same rows: the A fragment.
// Kernel: 8 waves (two per SIMD), one block per CU, block tile 256 replicates x 32 pairs x 7
// slices; wave w owns replicate batch w & 3 (4 x 16 replicates) and slice group w >> 2 (slices
// 0-3 or 4-6): 16 or 12 accumulators of 16 x 16 i32 per pair block. B arrives in LDS by DMA four
// sub-tiles ahead; A goes straight from HBM/L2 into registers three sub-tiles ahead. The loop runs
// in half-steps (sub-tile, pair block): the B fragments of the next half-step are read from LDS
// while the MFMAs of this one issue, and one barrier per sub-tile (between its two halves)
// publishes the next sub-tile and frees the oldest ring stage.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

#include "ob_common.hpp"
#include "ob_engine.hpp"
#include "ob_spec.h"

typedef int ob_v4i __attribute__((ext_vector_type(4)));
typedef int ob_v16i __attribute__((ext_vector_type(16)));

namespace {

constexpr int kS = 7;                  // balanced 8-bit digits per pair product (54-bit fixed point)
constexpr int kFracBits = 54;          // m = rint(P 2^(kFracBits - E))
constexpr int kPairsPerTile = 32;      // pairs per column tile (one 32-wide MFMA column block)
constexpr int kSubUnits = kS * 2 * 64; // 16-byte units of one (sub-tile, column tile) B image (14 KB)
constexpr int kSlo = 4;                // slices of slice group 0 (waves 0-3); group 1 has kS - kSlo
#ifndef OB_OZ_A_NT
// A fragments by ordinary loads, so that the 8 column-tile blocks of a (chunk, replicate tile),
// which run together on one XCD, share them through its L2. Nontemporal loads (OB_OZ_A_NT=1,
// tools/build_alt.sh) measured 14.6 ms per Gram launch against 13.4 ms at configs[1].
#define OB_OZ_A_NT 0
#endif

#define OZ_HIP(expr)                                                                                  \
  do {                                                                                                \
    hipError_t e_ = (expr);                                                                           \
    if (e_ != hipSuccess)                                                                             \
      return ob::fail(OB_E_HIP, "HIP error %s at %s:%d", hipGetErrorString(e_), __FILE__, __LINE__); \
  } while (0)

// v_c of a row (ob_panel_kernel's formula): weighted sqrt(w) [1, x, y], else [1, x, y].
__device__ __forceinline__ double oz_v(const double* cols, int64_t ld, int nxy, int weighted, size_t row, int c) {
  if (weighted) {
    const double sw = sqrt(cols[(size_t)nxy * ld + row]);
    return c == 0 ? sw : sw * cols[(size_t)(c - 1) * ld + row];
  }
  return c == 0 ? 1.0 : cols[(size_t)(c - 1) * ld + row];
}

__device__ __forceinline__ void oz_pair_cols(int pair, int k1, int* a, int* b) {
  int aa = 0, rem = pair;
  while (rem >= k1 - aa) {
    rem -= k1 - aa;
    ++aa;
  }
  *a = aa;
  *b = aa + rem;
}

// Per (chunk, pair): the exponent E with 2^(E-1) <= max |P| < 2^E over the chunk's rows (0 if all
// zero or a padding pair). Same product expression as oz_digits_kernel.
__global__ __launch_bounds__(256) void oz_pairexp_kernel(const double* cols0, const double* cols1, int64_t ld0,
                                                         int64_t ld1, uint32_t n0, uint32_t n1, int nxy, int weighted,
                                                         const uint32_t* chunks, int k1, int e, int n_pairs_pad,
                                                         int32_t* pexp) {
  __shared__ double red[256];
  const int chunk = blockIdx.x, pair = blockIdx.y, tid = threadIdx.x;
  if (pair >= e) {
    if (tid == 0) pexp[chunk * n_pairs_pad + pair] = 0;
    return;
  }
  int ca, cb;
  oz_pair_cols(pair, k1, &ca, &cb);
  const uint32_t g = chunks[3 * chunk];
  const double* cols = g ? cols1 : cols0;
  const int64_t ld = g ? ld1 : ld0;
  const uint32_t n = g ? n1 : n0;
  const size_t r0 = (size_t)chunks[3 * chunk + 1] * OB_TILE_ROWS;
  const size_t r1 = std::min<size_t>((size_t)chunks[3 * chunk + 2] * OB_TILE_ROWS, n);
  double m = 0.0;
  for (size_t r = r0 + tid; r < r1; r += 256)
    m = fmax(m, fabs(oz_v(cols, ld, nxy, weighted, r, ca) * oz_v(cols, ld, nxy, weighted, r, cb)));
  red[tid] = m;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (tid < o) red[tid] = fmax(red[tid], red[tid + o]);
    __syncthreads();
  }
  if (tid == 0) {
    int ex = 0;
    if (red[0] > 0.0) (void)frexp(red[0], &ex);  // red[0] = f 2^ex, f in [0.5, 1)
    pexp[chunk * n_pairs_pad + pair] = ex;
  }
}

// B digits of one group: grid (sub-tile, column tile), 256 threads = (slice group, pair block, lane).
__global__ __launch_bounds__(256) void oz_digits_kernel(const double* cols, int64_t ld, uint32_t n, int nxy,
                                                        int weighted, int k1, int e, int n_ct, int n_pairs_pad,
                                                        const int32_t* tile_chunk, const int32_t* pexp,
                                                        ob_v4i* B) {
  const uint32_t sub = blockIdx.x;
  const int ct = blockIdx.y, t = threadIdx.x, lane = t & 63, nb = (t >> 6) & 1, grp = t >> 7;
  const int pair = ct * kPairsPerTile + 16 * nb + (lane & 15);
  int a = 0, b = 0;
  const bool live = pair < e;
  if (live) oz_pair_cols(pair, k1, &a, &b);
  const int E = live ? pexp[tile_chunk[sub >> 2] * n_pairs_pad + pair] : 0;
  int8_t dig[16][kS];
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const size_t row = (size_t)sub * 64 + 16 * (lane >> 4) + j;
    double P = 0.0;
    if (live && row < n) P = oz_v(cols, ld, nxy, weighted, row, a) * oz_v(cols, ld, nxy, weighted, row, b);
    long long m = (long long)rint(ldexp(P, kFracBits - E));  // |m| <= 2^54: exact
#pragma unroll
    for (int sl = kS - 1; sl >= 0; --sl) {  // balanced digits, least significant first
      const int8_t d = (int8_t)(m & 0xff);
      dig[j][sl] = d;
      m = (m - d) >> 8;
    }
  }
  const int sl0 = grp ? kSlo : 0, sl1 = grp ? kS : kSlo;
  for (int sl = sl0; sl < sl1; ++sl) {
    uint32_t w[4] = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int j = 0; j < 16; ++j) w[j >> 2] |= (uint32_t)(uint8_t)dig[j][sl] << (8 * (j & 3));
    B[(((size_t)sub * n_ct + ct) * kS + sl) * 2 * 64 + nb * 64 + lane] = (ob_v4i){(int)w[0], (int)w[1], (int)w[2], (int)w[3]};
  }
}

struct OzArgs {
  const ob_v4i* B0;
  const ob_v4i* B1;
  const ob_v4i* counts;    // I8 count images (ob_count_kernel<true>): [tile][batch][1024 units]
  const uint32_t* chunks;  // [chunk][3] = (group, first tile, end tile)
  const int32_t* pexp;     // [chunk][n_pairs_pad]
  double* partial;         // [chunk][rep_pad][e_pad]
  uint32_t n0, n1, tiles0, nb_rep, n_reps, rep_pad, n_rt;
  int n_ct, e_pad, n_pairs_pad;
};

constexpr int kWaves = 8;                         // 2 per SIMD: (replicate batch, slice group)
constexpr int kNbuf = 4;                          // LDS ring stages (sub-tiles)
constexpr int kBDma = (kSubUnits + 64 * kWaves - 1) / (64 * kWaves);  // B DMA instructions per wave (<=)
constexpr int kBDmaTotal = kSubUnits / 64;        // 14 per sub-tile, spread over the waves
constexpr size_t kLdsB = kNbuf * (size_t)kSubUnits * 16;      // B ring (56 KB)
constexpr size_t kLdsX = 4 * 64 * (size_t)kPairsPerTile * 8;  // slice-group exchange (64 KB, over the ring)
constexpr size_t kLdsBytes = kLdsB > kLdsX ? kLdsB : kLdsX;
static_assert(kBDma == 2 && kBDmaTotal == 14, "B DMA split below assumes 14 instructions over 8 waves");

// One 16-byte-per-lane LDS-DMA (global_load_lds_dwordx4: lane l lands at lds + 16 l). Issued from
// inline asm so the compiler does not track it: its wait model counts LDS-DMA against the LDS
// counter and would then drain every fragment read (lgkmcnt(0)) before the next MFMAs. The
// kernel waits for these loads itself (counted vmcnt before each publishing barrier).
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"  // m0 is reserved, and this asm does overwrite it
__device__ __forceinline__ void oz_dma16(const void* src, uint32_t lds) {
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(src), "s"(lds) : "memory", "m0");
}
#pragma clang diagnostic pop

__device__ __forceinline__ void oz_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

template <int N>
struct IC {
  static constexpr int value = N;
};

// Half-step h of a sub-tile: pair block h (16 pairs) of every slice q < NQ against the four
// 16-replicate blocks: 4 NQ v_mfma_i32_16x16x64_i8, K = the whole 64-row sub-tile.
template <int NQ>
__device__ __forceinline__ void oz_mfmas(ob_v4i (&acc)[4][kSlo][2], int h, const ob_v4i (&af)[4],
                                         const ob_v4i (&bf)[kSlo]) {
#pragma unroll
  for (int q = 0; q < NQ; ++q)
#pragma unroll
    for (int m = 0; m < 4; ++m)
      acc[m][q][h] = __builtin_amdgcn_mfma_i32_16x16x64_i8(af[m], bf[q], acc[m][q][h], 0, 0, 0);
}

// Block: (chunk, replicate tile of 4 batches, column tile). NQ = slices of this wave's group, NB =
// its B DMA pieces per sub-tile, LIVE = its replicate batch exists. All are wave-uniform template
// constants, so the loop has no divergent control flow and the compiler's LDS-counter bookkeeping
// stays exact (a wait only for the fragments an MFMA consumes). DIAG (OB_GRAM_DIAG, timing
// ablations only, wrong results): 2 no MFMAs, 4 no sub-tile loads after the prologue, 8 no barrier.
// MFMA shape: v_mfma_i32_16x16x64_i8 (the 16x16 forms hold a higher clock than the 32x32 forms on
// random operands at equal cycles per op, MI355X_MICROARCH.md 'DVFS give-back' item 7). Lane l of
// an A fragment holds replicate 16 m + (l & 15), rows 16 (l >> 4) + j of the sub-tile; lane l of a B
// fragment pair 16 h + (l & 15) of the column tile, the same rows; D: pair 16 h + (l & 15),
// replicates 16 m + 4 (l >> 4) + i.
template <int NQ, int NB, bool LIVE, int DIAG>
__device__ __forceinline__ void oz_gram_body(const OzArgs& a, unsigned char* smem, int wave) {
  constexpr int PER = NB + (LIVE ? 4 : 0);  // this wave's vector-memory ops per sub-tile
  const ob_v4i* bs = reinterpret_cast<const ob_v4i*>(smem);  // [kNbuf][kSubUnits]
  const int lane = threadIdx.x & 63;
  const int wb = wave & 3, grp = wave >> 2;  // replicate batch in the tile, slice group
  const int slo = grp ? kSlo : 0;
  // XCD-aware remap (as ob_gram_kernel's map_work): consecutive work items -- the column tiles of
  // one replicate tile, then the replicate tiles of one chunk -- share an XCD's L2.
  const uint32_t nwg = gridDim.x, bid = blockIdx.x;
  const uint32_t xcd = bid & 7u, slot = bid >> 3, q8 = nwg >> 3, r8 = nwg & 7u;
  const uint32_t wi = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + slot;
  const int ct = (int)(wi % (uint32_t)a.n_ct);
  const uint32_t tq = wi / (uint32_t)a.n_ct;
  const uint32_t rt = tq % a.n_rt, chunk = tq / a.n_rt;
  const uint32_t g = a.chunks[3 * chunk];
  const uint32_t n = g ? a.n1 : a.n0, tg0 = g ? a.tiles0 : 0u;
  const uint32_t s0 = a.chunks[3 * chunk + 1] * 4u;
  const uint32_t s1 = min(a.chunks[3 * chunk + 2] * 4u, (n + 63u) >> 6);
  const ob_v4i* Bg = g ? a.B1 : a.B0;
  const uint32_t batch = rt * 4u + (uint32_t)wb;
  auto dma = [&](int buf, uint32_t s) {
    const ob_v4i* src = Bg + ((size_t)s * a.n_ct + ct) * kSubUnits;  // B: 14 KB
#pragma unroll
    for (int t = 0; t < NB; ++t) {
      const int piece = t * kWaves + wave;
      oz_dma16(src + piece * 64 + lane, (uint32_t)(buf * kSubUnits + piece * 64) * 16u);
    }
  };
  // A fragments in registers: three slots, sub-tile s in slot (s - s0) % 3; this wave's batch of
  // sub-tile s is 4 x 1 KB, [replicate block][lane]
  ob_v4i ar[3][4];
  auto aload = [&](ob_v4i (&dst)[4], uint32_t s) {
    const ob_v4i* src_a = a.counts + (((size_t)(tg0 + (s >> 2)) * a.nb_rep + batch) * 4 + (s & 3)) * 256 + lane;
#pragma unroll
    for (int m = 0; m < 4; ++m) dst[m] = OB_OZ_A_NT ? __builtin_nontemporal_load(src_a + m * 64) : src_a[m * 64];
  };
  // B fragments of half-step h (sub-tile in ring stage buf)
  auto read = [&](int buf, int h, ob_v4i (&bf)[kSlo]) {
    const ob_v4i* bb = bs + buf * kSubUnits + (slo * 2 + h) * 64 + lane;
#pragma unroll
    for (int q = 0; q < NQ; ++q) bf[q] = bb[q * 128];
  };

  ob_v4i acc[4][kSlo][2];
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int q = 0; q < kSlo; ++q) acc[m][q][0] = acc[m][q][1] = (ob_v4i){};
  // prologue: B of sub-tiles s0 .. s0 + 3 and A of s0 .. s0 + 2 in flight; publish s0
  // (A loads unconditional, clamped to the last sub-tile, so that the three register slots are
  // loaded in the same order on entry to the loop as on its back edge)
  if constexpr (LIVE) {
    aload(ar[0], s0);
    aload(ar[1], min(s0 + 1, s1 - 1));
    aload(ar[2], min(s0 + 2, s1 - 1));
  }
#pragma unroll
  for (int j = 0; j < kNbuf; ++j)
    if (s0 + j < s1) dma(j, s0 + j);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every prologue load: once per block
  __syncthreads();
  ob_v4i fb0[kSlo], fb1[kSlo];
  if constexpr (LIVE) read(0, 0, fb0);

  // Half-step (s, 0): read (s, 1); MFMAs on (s, 0). Barrier B_s: sub-tile s + 1 landed (own loads,
  // then everyone's), every read of sub-tile s done. Refill stage s with B of s + 4. Half-step
  // (s, 1): read (s + 1, 0) (after the last sub-tile: a stale stage, never used); MFMAs on (s, 1);
  // then A of s + 3 into the register slot s frees. Issue order per sub-tile t: B(t + 4) after
  // B_t, A(t + 3) at the end of step t, so at B_s the loads newer than those of s + 1 are
  // B(s + 3), A(s + 2) (after step s - 1) and B(s + 2) is older than A(s + 1): the wait leaves
  // PER in flight while two or more sub-tiles follow.
  auto step = [&](uint32_t s, auto J) {
    constexpr int j = decltype(J)::value;
    const int buf = (int)((s - s0) & (kNbuf - 1));
    if constexpr (LIVE) {
      read(buf, 1, fb1);
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (!(DIAG & 2)) oz_mfmas<NQ>(acc, 0, ar[j], fb0);
      __builtin_amdgcn_sched_barrier(0);
    }
    const uint32_t ahead = (DIAG & 4) ? 0u : s1 - 1 - s;  // sub-tiles after s
    if (ahead >= 3) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PER) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if constexpr (DIAG & 8) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // timing only: no barrier
    else oz_barrier();
    if (!(DIAG & 4) && s + kNbuf < s1) dma(buf, s + kNbuf);
    if constexpr (LIVE) {
      read((buf + 1) & (kNbuf - 1), 0, fb0);
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (!(DIAG & 2)) oz_mfmas<NQ>(acc, 1, ar[j], fb1);
      __builtin_amdgcn_sched_barrier(0);
      // unconditional (past the end: a re-read of the last sub-tile, never used), so the compiler's
      // count of outstanding A loads is exact at every MFMA
      if constexpr (!(DIAG & 4)) aload(ar[j], min(s + 3, s1 - 1));
    }
  };
  uint32_t s = s0;
  for (; s + 3 <= s1; s += 3) {
    step(s, IC<0>{});
    step(s + 1, IC<1>{});
    step(s + 2, IC<2>{});
  }
  if (s < s1) step(s, IC<0>{});
  if (s + 1 < s1) step(s + 1, IC<1>{});
  // slices -> f64: this wave's digits meet exactly in int64, one ldexp each; group 1 goes through
  // LDS to its group-0 partner, which adds (one rounding) and stores.
  int E[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int pair = ct * kPairsPerTile + 16 * h + (lane & 15);
    E[h] = a.pexp[chunk * a.n_pairs_pad + min(pair, a.n_pairs_pad - 1)];
  }
  double v[4][2][4];
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int shift = E[h] - kFracBits + 8 * (kS - slo - NQ);  // weight of this group's last slice
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        long long part = 0;
#pragma unroll
        for (int q = 0; q < NQ; ++q) part = part * 256 + acc[m][q][h][i];
        v[m][h][i] = ldexp((double)part, shift);
      }
    }
  __syncthreads();  // every wave is done with the ring: the exchange overlays it
  double* xch = reinterpret_cast<double*>(smem);  // [batch in tile][64 reps][32 pairs]
  if (grp) {
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int i = 0; i < 4; ++i)
          xch[(wb * 64 + 16 * m + 4 * (lane >> 4) + i) * kPairsPerTile + 16 * h + (lane & 15)] = v[m][h][i];
  }
  __syncthreads();
  if (grp || !LIVE) return;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int pair = ct * kPairsPerTile + 16 * h + (lane & 15);
    if (pair >= a.e_pad) continue;
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int rl = 16 * m + 4 * (lane >> 4) + i;
        const uint32_t rep = batch * 64u + (uint32_t)rl;
        const double val = v[m][h][i] + xch[(wb * 64 + rl) * kPairsPerTile + 16 * h + (lane & 15)];
        if (rep < a.n_reps) a.partial[((size_t)chunk * a.rep_pad + rep) * a.e_pad + pair] = val;
      }
  }
}

template <int DIAG>
__global__ __launch_bounds__(kWaves * 64, 1) void oz_gram_kernel(const OzArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // the replicate tile of this block (same map as the body) decides which batches exist
  const uint32_t nwg = gridDim.x, bid = blockIdx.x;
  const uint32_t xcd = bid & 7u, slot = bid >> 3, q8 = nwg >> 3, r8 = nwg & 7u;
  const uint32_t wi = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + slot;
  const uint32_t rt = (wi / (uint32_t)a.n_ct) % a.n_rt;
  const bool live = rt * 4u + (uint32_t)(wave & 3) < a.nb_rep;
  // waves 0-3: slices 0-3, two B pieces; 4-5: slices 4-6, two B pieces; 6-7: slices 4-6, one piece
  if (wave < 4) {
    if (live) oz_gram_body<kSlo, 2, true, DIAG>(a, smem, wave);
    else oz_gram_body<kSlo, 2, false, DIAG>(a, smem, wave);
  } else if (wave < 6) {
    if (live) oz_gram_body<kS - kSlo, 2, true, DIAG>(a, smem, wave);
    else oz_gram_body<kS - kSlo, 2, false, DIAG>(a, smem, wave);
  } else {
    if (live) oz_gram_body<kS - kSlo, 1, true, DIAG>(a, smem, wave);
    else oz_gram_body<kS - kSlo, 1, false, DIAG>(a, smem, wave);
  }
}

}  // namespace

namespace ob {

// Build (once per panel) the digit images and exponents for the panel's chunking. Returns OB_OK
// with p->oz_state = 1, or OB_OK with p->oz_state = -1 when the digit images would not fit (the
// caller keeps the f64 MFMA Gram).
int oz_prepare(ob_panel* p, const std::vector<uint32_t>& chunks) {
  if (p->oz_state != 0) return OB_OK;
  // exact int32 slice sums need 128 x (a chunk's draws) < 2^31: a group's draws bound a chunk's
  if (p->n[0] >= (1u << 24) || p->n[1] >= (1u << 24)) {
    p->oz_state = -1;
    return OB_OK;
  }
  const int n_chunks = (int)(chunks.size() / 3);
  const int n_ct = (p->e + kPairsPerTile - 1) / kPairsPerTile;
  const int npp = n_ct * kPairsPerTile;
  size_t bytes = 0;
  for (int g = 0; g < 2; ++g) bytes += (size_t)(p->ld[g] >> 6) * n_ct * kSubUnits * 16;
  size_t free_b = 0, total_b = 0;
  OZ_HIP(hipSetDevice(p->ctx->device));
  OZ_HIP(hipMemGetInfo(&free_b, &total_b));
  if (bytes > free_b / 2 || bytes > (96ull << 30)) {
    p->oz_state = -1;
    return OB_OK;
  }
  for (int g = 0; g < 2; ++g)
    OZ_HIP(hipMalloc(&p->d_oz_b[g], std::max<size_t>((size_t)(p->ld[g] >> 6) * n_ct * kSubUnits * 16, 16)));
  OZ_HIP(hipMalloc(&p->d_oz_pexp, sizeof(int32_t) * (size_t)n_chunks * npp));
  int32_t* d_tc = nullptr;
  uint32_t* d_chunks = nullptr;
  int rc = OB_OK;
  do {
#define OZ_TRY(expr)                                                                                     \
  {                                                                                                      \
    hipError_t e_ = (expr);                                                                              \
    if (e_ != hipSuccess) {                                                                              \
      rc = ob::fail(OB_E_HIP, "HIP error %s at %s:%d", hipGetErrorString(e_), __FILE__, __LINE__);      \
      break;                                                                                             \
    }                                                                                                    \
  }
    OZ_TRY(hipMalloc(&d_chunks, sizeof(uint32_t) * chunks.size()));
    OZ_TRY(hipMemcpy(d_chunks, chunks.data(), sizeof(uint32_t) * chunks.size(), hipMemcpyHostToDevice));
    const int nxy = p->p + p->n_y;
    hipLaunchKernelGGL(oz_pairexp_kernel, dim3(n_chunks, npp), dim3(256), 0, 0, (const double*)p->d_cols[0],
                       (const double*)p->d_cols[1], p->ld[0], p->ld[1], p->n[0], p->n[1], nxy, p->weighted,
                       (const uint32_t*)d_chunks, p->k1, p->e, npp, p->d_oz_pexp);
    OZ_TRY(hipGetLastError());
    for (int g = 0; g < 2 && rc == OB_OK; ++g) {
      const uint32_t nsub = (uint32_t)(p->ld[g] >> 6);
      if (nsub == 0) continue;
      std::vector<int32_t> tc(p->ntiles[g] ? p->ntiles[g] : 1, 0);
      for (int c = 0; c < n_chunks; ++c)
        if (chunks[3 * c] == (uint32_t)g)
          for (uint32_t t = chunks[3 * c + 1]; t < chunks[3 * c + 2]; ++t) tc[t] = c;
      OZ_TRY(hipMalloc(&d_tc, sizeof(int32_t) * tc.size()));
      OZ_TRY(hipMemcpy(d_tc, tc.data(), sizeof(int32_t) * tc.size(), hipMemcpyHostToDevice));
      hipLaunchKernelGGL(oz_digits_kernel, dim3(nsub, n_ct), dim3(256), 0, 0, (const double*)p->d_cols[g], p->ld[g],
                         p->n[g], nxy, p->weighted, p->k1, p->e, n_ct, npp, (const int32_t*)d_tc,
                         (const int32_t*)p->d_oz_pexp, reinterpret_cast<ob_v4i*>(p->d_oz_b[g]));
      OZ_TRY(hipGetLastError());
      OZ_TRY(hipDeviceSynchronize());
      (void)hipFree(d_tc);
      d_tc = nullptr;
    }
    if (rc == OB_OK) OZ_TRY(hipDeviceSynchronize());
#undef OZ_TRY
  } while (0);
  (void)hipFree(d_tc);
  (void)hipFree(d_chunks);
  if (rc != OB_OK) return rc;
  p->oz_n_ct = n_ct;
  p->oz_state = 1;
  return OB_OK;
}

// One segment's Gram partials: d_chunks holds the panel's chunk table, counts the I8 images of
// the segment's nb_rep replicate batches.
int oz_gram(ob_panel* p, const uint32_t* d_chunks, int n_chunks, const uint32_t* counts, uint32_t nb_rep,
            uint32_t rep_pad, uint32_t n_reps, double* partial, hipStream_t s) {
  OzArgs a{};
  a.B0 = reinterpret_cast<const ob_v4i*>(p->d_oz_b[0]);
  a.B1 = reinterpret_cast<const ob_v4i*>(p->d_oz_b[1]);
  a.counts = reinterpret_cast<const ob_v4i*>(counts);
  a.chunks = d_chunks;
  a.pexp = p->d_oz_pexp;
  a.partial = partial;
  a.n0 = p->n[0];
  a.n1 = p->n[1];
  a.tiles0 = p->ntiles[0];
  a.nb_rep = nb_rep;
  a.n_reps = n_reps;
  a.rep_pad = rep_pad;
  a.n_rt = (nb_rep + 3) / 4;
  a.n_ct = p->oz_n_ct;
  a.e_pad = p->e_pad;
  a.n_pairs_pad = p->oz_n_ct * kPairsPerTile;
  static const int diag = [] {
    const char* e = getenv("OB_GRAM_DIAG");
    return e ? atoi(e) & 14 : 0;
  }();
  const uint32_t blocks = (uint32_t)n_chunks * a.n_rt * (uint32_t)a.n_ct;
  auto launch = [&](auto kern) -> hipError_t {
    hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kLdsBytes);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(kWaves * 64), kLdsBytes, s, a);
    return hipGetLastError();
  };
  switch (diag) {
    case 2: OZ_HIP(launch(oz_gram_kernel<2>)); break;
    case 4: OZ_HIP(launch(oz_gram_kernel<4>)); break;
    case 6: OZ_HIP(launch(oz_gram_kernel<6>)); break;
    case 8: OZ_HIP(launch(oz_gram_kernel<8>)); break;
    default: OZ_HIP(launch(oz_gram_kernel<0>)); break;
  }
  return OB_OK;
}

}  // namespace ob
