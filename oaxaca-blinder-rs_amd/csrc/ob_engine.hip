// ob_engine.hip -- the MI355X bootstrap engine: OBRS-3 resampling + X^T diag(c w) X on f64 MFMA
// + wave-parallel Cholesky solves + Oaxaca-Blinder algebra, all resident in HBM.
//
// Replaces, per replicate, builder.rs:816-839 (polars resample + vstack + run_single_pass):
//   split_groups/prepare_data (builder.rs:294-378) -> the panel stays in HBM, column-major;
//   OlsEstimator::estimate + ols (estimation.rs:51-111, math/ols.rs:44-144) -> ob_gram_kernel
//   (counts-weighted extended Gram) + ob_solve_kernel (Cholesky, solve, means);
//   beta* + decomposition (builder.rs:536-684, decomposition.rs:56-122) -> ob_solve_kernel.
//
// Kernels (DESIGN.md §4 has the rooflines):
//   ob_level1_kernel   one block per (replicate, group): n_g Philox draws -> LDS tile histogram
//   ob_gram_kernel     one block per (row chunk, 64-replicate batch, column group), two per CU:
//                      per 256-row tile, level-2 draws -> u8 count image in LDS (pipelined one
//                      tile ahead), then G[r][e] += sum_i c[r][i] v_i[a(e)] v_i[b(e)] with
//                      v_mfma_f64_16x16x4_f64 (A = counts, 16 replicates x 4 rows; B = pair
//                      products of the staged rows, 4 rows x 16 pairs; v = sqrt(w) [1, x, y])
//   ob_reduce_kernel   sums the per-chunk partial Grams in a fixed order (deterministic)
//   ob_solve_kernel    one wave per replicate: normal equations, Cholesky, beta*, OB terms
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <vector>

#include "ob_device.hpp"
#include "ob_engine.hpp"
#include "ob_heckman.hpp"
#include "ob_options.hpp"
#include "ob_spec.h"

typedef double ob_d4 __attribute__((ext_vector_type(4)));

namespace {

constexpr int kBlock = 256;
// The count kernel's LDS u8 image of a (tile, 64-replicate batch) is replicate-minor: row word q
// (rows 4q .. 4q+3 of the tile) of replicate r is word q * kImgRow + r. A wave whose lanes draw
// for 64 distinct replicates then hits 32 distinct banks per lane group (bank = r mod 32).
constexpr int kImgRow = 64;                            // words per row word (one per replicate)
constexpr int kImgWords = (OB_TILE_ROWS / 4) * kImgRow;  // 4096
constexpr uint64_t kSegReps = 16384;
constexpr uint64_t kCountBudget = 24ull << 30;  // bytes of level-2 count images per segment
// rows per group: 2^20 tiles (level 1 walks groups past 40960 tiles as subtrees, whose LDS
// buffers are bounded; the count images then cap a segment's replicates via kCountBudget)
constexpr int64_t kMaxGroupRows = (int64_t)1 << 28;
#ifndef OB_BOOT_OVERLAP
#define OB_BOOT_OVERLAP 1  // 0: level 1 and counts on the boot stream (A/B builds, tools/build_alt.sh)
#endif
constexpr size_t kSegEvents = 7;  // level-1 start / end, counts end (resample stream), Gram start / end, reduce end, solve end
constexpr int kColStride = 96;  // doubles per staged column: 64 rows rotated by (c mod 32), wrap duplicated

#define HIP_OK(expr)                                                                     \
  do {                                                                                   \
    hipError_t e_ = (expr);                                                              \
    if (e_ != hipSuccess)                                                                \
      return ob::fail(OB_E_HIP, "HIP error %s at %s:%d", hipGetErrorString(e_), __FILE__, \
                      __LINE__);                                                         \
  } while (0)

struct GramArgs {
  const double* gcols0;  // Gram panel of group A (ob_panel_kernel layout: [sub-tile][c_first..k1-1][96])
  const double* gcols1;
  int64_t ld0, ld1;
  uint32_t n0, n1;
  int k1, c_first, e, ncb, n_cg;
  uint32_t nb_rep;
  const uint32_t* chunks;  // [chunk][3] = (group, first tile, end tile)
  const uint32_t* m1;      // [replicate][tile (group 0 then group 1)]
  uint32_t tiles0;
  uint32_t rep_pad;
  uint32_t n_reps;
  uint32_t first_rep;
  uint32_t key0, key1;
  double* partial;  // [chunk][rep_pad][e_pad]
  int e_pad;
  uint32_t* flags;
  const uint32_t* counts;  // level-2 count images [tile (A then B)][batch][sub-tile][kCimgWords]
  uint32_t tiles_total;
  int diag;  // OB_GRAM_DIAG bits: 2 no MFMAs, 4 no sub-tile DMA (tools/gram_ablate.py), 8 raw Heckman
             // statuses; count kernel timing ablations (wrong counts): 32 no LDS atomics, 64 no Philox
  int dbl;   // ob_gram_kernel: 1 = two staged sub-tile buffers (prefetch), 0 = one (k1 > kGramDblMaxK1)
  uint32_t rb0;  // ob_count_kernel: the launch's first 64-replicate batch (a piece of the segment)
};

// ---------------------------------------------------------------------------------------------
// Level 1: tile counts m_j for one (replicate, group) by binomial splitting (OBRS-3, ob_spec.h:
// popcounts below 4096 draws, Knuth-Yao samples above; oracle orc_level1_counts). Level l of the
// dyadic tile tree lives in LDS buffer (D - l) & 1.
// Levels l < 8 have at most 2^l nodes and give each 256 >> l threads (popcounts summed by LDS
// atomics); deeper levels give a thread whole nodes. T <= 256 tiles ("small") keeps the tile
// level and the running counts in LDS; larger T sends the last split straight to m1, the
// thread that owns node k of level D-1 owning tiles 2k, 2k+1 in every round, so later rounds
// add to m1 without atomics. The <= 256 direct draws finish with atomics (LDS or global).
// ---------------------------------------------------------------------------------------------
static_assert(kBlock == 256, "level 1 maps 256 threads onto the top tree levels");
__host__ __device__ inline uint32_t l1_depth(uint32_t ntiles) { return ntiles > 1 ? 32u - __builtin_clz(ntiles - 1) : 0u; }
__host__ __device__ inline bool l1_small(uint32_t ntiles) { return ntiles <= 256u; }
// Groups of more than kL1FlatTiles tiles run the tree as subtrees of depth kL1SubDepth under the
// nodes of level J = D - kL1SubDepth (the "top", at most 2^J <= 512 nodes): the per-level LDS
// buffers then hold one subtree at a time. Node streams depend on (round, level, global index)
// only, so the order subtrees are walked in does not change a count.
constexpr uint32_t kL1FlatTiles = 40960;
constexpr uint32_t kL1SubDepth = 15;
constexpr uint32_t kL1TopWords = 512;
__host__ __device__ inline uint32_t l1_top_levels(uint32_t ntiles) {
  return ntiles > kL1FlatTiles ? l1_depth(ntiles) - kL1SubDepth : 0u;
}
__host__ __device__ inline uint32_t l1_sub_tiles(uint32_t ntiles) {
  return ntiles > kL1FlatTiles ? (1u << kL1SubDepth) : ntiles;
}
__host__ __device__ inline uint32_t l1_buf0_words(uint32_t ntiles) {
  return l1_small(ntiles) ? 256u : (l1_sub_tiles(ntiles) + 3) / 4;
}
__host__ __device__ inline uint32_t l1_lds_words(uint32_t ntiles) {
  if (l1_small(ntiles)) return 256u + 128u + 256u;
  const uint32_t t = l1_sub_tiles(ntiles);
  return (t + 3) / 4 + (t + 1) / 2 + (ntiles > kL1FlatTiles ? 2 * kL1TopWords : 0u);
}

// OBRS-2 split on the device (ob_spec.h; oracle orc_split_left). The hot columns of every table
// live in LDS, so a walk that ends within OB_KY_HOT columns of its first (p > 0.99) makes no
// global access; deeper columns read the global tables.
struct KyLds {
  uint32_t i0[OB_KY_TABLES], obase[OB_KY_TABLES], lbase[OB_KY_TABLES];
  uint32_t hoff[OB_KY_TABLES][OB_KY_HOT + 1];  // positions in hlist
  uint16_t hlist[OB_KY_HOT_CAP];
};

__device__ __forceinline__ void ky_stage(KyLds& L, const ob_ky_tables& g, uint32_t tid) {
  if (tid < OB_KY_TABLES) {
    L.i0[tid] = g.i0[tid];
    L.obase[tid] = g.off_base[tid];
    L.lbase[tid] = g.list_base[tid];
  }
  for (uint32_t i = tid; i < OB_KY_TABLES * (OB_KY_HOT + 1); i += kBlock) (&L.hoff[0][0])[i] = g.hot[i];
  const uint32_t* he = g.hot + OB_KY_TABLES * (OB_KY_HOT + 1);
  for (uint32_t i = tid; 2 * i < g.hot_entries; i += kBlock) reinterpret_cast<uint32_t*>(L.hlist)[i] = he[i];
}

// One B(2^(t + 7), 1/2) sample: the Knuth-Yao walk (ob_spec.h), one stream bit per column.
__device__ __forceinline__ uint32_t ky_walk(ob_bitstream& s, const KyLds& L, int t, const uint32_t* __restrict__ goff,
                                            const uint16_t* __restrict__ glist) {
  const uint32_t i0 = L.i0[t];
  uint32_t d = ob_bs_take_msb(s, i0 - 1u);  // columns 1 .. i0 - 1 hold no entries
  for (uint32_t c = 0;; ++c) {
    d = 2u * d + ob_bs_bit(s);
    if (c < OB_KY_HOT) {
      const uint32_t lo = L.hoff[t][c], cnt = L.hoff[t][c + 1] - lo;
      if (d < cnt) return L.hlist[lo + d];
      d -= cnt;
    } else {
      const uint32_t* off = goff + L.obase[t];
      const uint32_t i = i0 + c, lo = off[i], cnt = off[i + 1] - lo;
      if (d < cnt) return glist[L.lbase[t] + lo + d];
      d -= cnt;
    }
  }
}

// Work item q of the split of a node holding c draws (ob_spec.h, OBRS-2): a popcount word below
// OB_KY_MIN_C draws, else one stream (one Knuth-Yao sample or the low popcount). rl = (round << 5)
// + level.
__device__ __forceinline__ uint32_t l1_split_item(uint32_t q, uint32_t c, uint32_t rep, uint32_t c2, uint32_t rl,
                                                  uint32_t k0, uint32_t k1, const KyLds& L,
                                                  const uint32_t* __restrict__ goff,
                                                  const uint16_t* __restrict__ glist) {
  if (c < OB_KY_MIN_C) return ob_l1_split_bits(q, c, rep, c2, OB_TAG_L1T + rl, k0, k1);
  const uint32_t c4 = c >> 12;
  ob_bitstream s = {q << 12, rep, c2, OB_TAG_L1K + rl, k0, k1, 0u, 0u, 0u, 0u, 0u};
  if (q < c4) return ky_walk(s, L, OB_KY_TABLES - 1, goff, glist);
  const uint32_t i = q - c4, nd = (uint32_t)__builtin_popcount((c >> 7) & 31u);
  if (i < nd) return ky_walk(s, L, (int)ob_l1_digit_log(c, i) - OB_KY_MIN_LOG, goff, glist);
  return ob_bs_popcount(s, c & 127u);
}

// DIAG (OB_L1_DIAG, timing ablations only, wrong counts): 1 no random bits (left = c / 2),
// 2 one round only, 4 no Knuth-Yao staging, 8 no m1 stores, 16 return after the staging barrier,
// 32 no random bits for the one-thread-per-node levels' nodes below 128 draws.
template <int DIAG>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(8, 8))) void ob_level1_kernel(uint32_t n0, uint32_t n1, uint32_t tiles0,
                                                           uint32_t first_rep, uint32_t stride,
                                                           uint32_t key0, uint32_t key1, uint32_t* m1,
                                                           const ob_ky_tables ky_g) {
  extern __shared__ __attribute__((aligned(16))) uint32_t l1s[];
  __shared__ uint32_t s_rej, s_tail, s_acc;
  __shared__ KyLds kyl;  // the Knuth-Yao tables' hot columns and bases
  const uint32_t g = blockIdx.y, rl = blockIdx.x, rep = first_rep + rl, tid = threadIdx.x;
  const uint32_t n = g ? n1 : n0;
  if (n == 0) return;
  if constexpr (!(DIAG & 4)) ky_stage(kyl, ky_g, tid);  // published by the first barrier of the round loop
  if constexpr ((DIAG & 16) != 0) {
    __syncthreads();
    if (tid == 0 && kyl.hlist[7] == 0xFFFFu) m1[0] = 0u;  // keeps the staging
    return;
  }
  const uint32_t T = (n + OB_TILE_ROWS - 1) >> OB_TILE_SHIFT, D = l1_depth(T), J = l1_top_levels(T);
  const uint32_t tail = n - (T - 1) * OB_TILE_ROWS;
  const bool small = l1_small(T), partial = tail < OB_TILE_ROWS;
  uint32_t* buf[2] = {l1s, l1s + l1_buf0_words(T)};
  uint32_t* top[2] = {buf[1] + (l1_sub_tiles(T) + 1) / 2, buf[1] + (l1_sub_tiles(T) + 1) / 2 + kL1TopWords};
  uint32_t* mt = l1s + 256u + 128u;  // small: running tile counts
  uint32_t* mcol = m1 + (size_t)rl * stride + (g ? tiles0 : 0u);  // [rep][tile]: one row per block
  const uint32_t tail_owner = ((T - 1) >> 1) & (kBlock - 1);
  if (small && tid < T) mt[tid] = 0;
  uint32_t todo = n;
  for (uint32_t round = 0;; ++round) {
    if (tid == 0) {
      if (J) top[0][0] = todo;
      else buf[D & 1][0] = todo;
      s_rej = 0;
      s_tail = 0;
      s_acc = 0;
    }
    __syncthreads();
    uint32_t rej = 0;
    // large T, round r: tile t of the last split gets c (tail tile: parked for acceptance)
    auto emit = [&](uint32_t t, uint32_t c) {
      if constexpr ((DIAG & 8) != 0) return;
      if (partial && t == T - 1) s_tail = c;
      else if (round == 0) mcol[t] = c;
      else if (c) mcol[t] += c;
    };
    // Level l over `nodes` nodes starting at global index kb (cur: their counts, local index),
    // children into nxt (local 2k, 2k + 1) or rejected past the last tile; ll = the level within
    // the current (sub)tree decides the thread mapping (at most 2^ll nodes).
    auto level = [&](uint32_t l, uint32_t ll, uint32_t kb, uint32_t nodes, const uint32_t* cur, uint32_t* nxt) {
      const uint32_t span = 1u << (D - l - 1);  // tiles per child
      const uint32_t nnext = (T + span - 1) / span;
      const uint32_t rl = (round << 5) + l;
      if (ll < 8) {  // nodes <= 2^ll: 256 >> ll threads per node; never the large last level
        const uint32_t sh = 8 - ll, k = tid >> sh, j = tid & ((1u << sh) - 1);
        if (j == 0 && k < nodes) nxt[2 * k] = 0;
        __syncthreads();
        if (k < nodes) {
          const uint32_t c = cur[k];
          uint32_t left = 0;
          const uint32_t ns = c ? ob_l1_items(c) : 0u;
          if constexpr (DIAG & 1) left = j == 0 ? c >> 1 : 0u;
          else
            for (uint32_t q = j; q < ns; q += 1u << sh)
              left += l1_split_item(q, c, rep, ((kb + k) << 1) | g, rl, key0, key1, kyl, ky_g.off, ky_g.list);
          if (left) atomicAdd(&nxt[2 * k], left);
        }
        __syncthreads();
        if (j == 0 && k < nodes) {
          const uint32_t c = cur[k], right = c - nxt[2 * k];
          if (2 * (kb + k) + 1 < nnext) nxt[2 * k + 1] = right;
          else rej += right;
        }
        __syncthreads();
      } else {
        const bool to_m1 = l + 1 == D && !small;
        for (uint32_t k = tid; k < nodes; k += kBlock) {
          const uint32_t c = cur[k], kg = kb + k;
          uint32_t left = 0;
          const uint32_t ns = c ? ob_l1_items(c) : 0u;
          if constexpr (DIAG & 1) left = c >> 1;
          else if ((DIAG & 32) && c < 128u) left = c >> 1;
          else
            for (uint32_t q = 0; q < ns; ++q)
              left += l1_split_item(q, c, rep, (kg << 1) | g, rl, key0, key1, kyl, ky_g.off, ky_g.list);
          const uint32_t right = c - left;
          if (to_m1) {
            emit(2 * kg, left);
            if (2 * kg + 1 < T) emit(2 * kg + 1, right);
            else rej += right;
          } else {
            nxt[2 * k] = left;
            if (2 * kg + 1 < nnext) nxt[2 * k + 1] = right;
            else rej += right;
          }
        }
        __syncthreads();
      }
    };
    for (uint32_t l = 0; l < J; ++l) {  // the top of a large tree: every node of levels 0 .. J - 1
      const uint32_t span2 = 2u << (D - l - 1);
      level(l, l, 0, (T + span2 - 1) / span2, top[l & 1], top[(l + 1) & 1]);
    }
    // one subtree per node of level J (the whole tree when J = 0)
    const uint32_t nsub = J ? (T + (1u << (D - J)) - 1) >> (D - J) : 1u;
    for (uint32_t K = 0; K < nsub; ++K) {
      if (J) {
        if (tid == 0) buf[(D - J) & 1][0] = top[J & 1][K];
        __syncthreads();
      }
      for (uint32_t l = J; l < D; ++l) {
        const uint32_t ll = l - J, kb = K << ll, span2 = 2u << (D - l - 1);
        const uint32_t nodes = min(1u << ll, (T + span2 - 1) / span2 - kb);
        level(l, ll, kb, nodes, buf[(D - l) & 1], buf[(D - l - 1) & 1]);
      }
    }
    if (small) {  // tile level D is buf[0]
      const uint32_t* tl = buf[0];
      if (tid < T) {
        if (partial && tid == T - 1) s_tail = tl[tid];
        else mt[tid] += tl[tid];
      }
      __syncthreads();
    }
    if (partial && tid < 64) {  // the tail tile accepts draw i iff its byte < tail
      const uint32_t c = s_tail;
      uint32_t acc = 0;
      for (uint32_t q = tid; 16 * q < c; q += 64) {
        const ob_u32x4 u = ob_philox(q, rep, g, OB_TAG_L1S + round, key0, key1);
        const uint32_t wd[4] = {u.x, u.y, u.z, u.w};
        const uint32_t m = min(16u, c - 16 * q);
#pragma unroll
        for (uint32_t i = 0; i < 16; ++i) acc += (i < m && ((wd[i >> 2] >> (8 * (i & 3))) & 0xFFu) < tail) ? 1u : 0u;
      }
      if (acc) atomicAdd(&s_acc, acc);
    }
    __syncthreads();
    if (partial) {
      const uint32_t a = s_acc;
      if (tid == 0) rej += s_tail - a;
      if (small) {
        if (tid == 0) mt[T - 1] += a;
      } else if (tid == tail_owner) {
        if (round == 0) mcol[T - 1] = a;
        else if (a) mcol[T - 1] += a;
      }
    }
    if (rej) atomicAdd(&s_rej, rej);
    __syncthreads();
    todo = s_rej;
    __syncthreads();
    if (todo <= OB_L1_DIRECT) break;
    if constexpr ((DIAG & 2) != 0) {
      todo = 0;
      break;
    }
  }
  // The direct draws' global atomics (L2) add to m1 words other threads of this block stored:
  // __syncthreads() waits for this wave's stores (vmcnt(0)) before the barrier, which is all the
  // ordering a block on one CU needs. A device-scope __threadfence() here compiled to an L2
  // write-back and invalidate per block (buffer_wbl2 / buffer_inv): 1.6 of the kernel's 3.4 ms.
  // (Round 6 measured drawing up to 65,536 rejects directly, four per Philox call, into an LDS
  // histogram -- configs[1]'s whole second round: level 1 1.743 against 1.729 ms, no gain: the
  // direct draws take 32 random bits each where the tree's popcount splits take one per level.)
  __syncthreads();
  for (uint32_t r = tid; r < todo; r += kBlock) {  // direct draws: Lemire over [0, n)
    const uint32_t thresh = (0u - n) % n;
    uint64_t x;
    for (uint32_t j = 0;; ++j) {
      const ob_u32x4 u = ob_philox(r, rep, g, OB_TAG_L1D + (j >> 2), key0, key1);
      const uint32_t wd[4] = {u.x, u.y, u.z, u.w};
      x = (uint64_t)wd[j & 3] * n;
      if ((uint32_t)x >= thresh) break;
    }
    const uint32_t t = (uint32_t)(x >> 32) >> OB_TILE_SHIFT;
    if (small) atomicAdd(&mt[t], 1u);
    else atomicAdd(&mcol[t], 1u);
  }
  if (small) {
    __syncthreads();
    if (tid < T) mcol[tid] = mt[tid];
  }
}

// ---------------------------------------------------------------------------------------------
// Pieces of the Gram kernel.
//
// v = [1, x_1..x_p, y] scaled by sqrt(w) when weighted (the reference's own WLS formulation,
// ols.rs:68-78), so G[r][e] = sum_i c[r][i] v_i[a(e)] v_i[b(e)] with A = counts only.
// Staged sub-tile image: column-major [col][kColStride = 96] doubles. Row r of the 64-row
// sub-tile has slot q = (r & 3) * 16 + (r >> 2) (the 4 rows of a k-step 16 slots = 32 banks
// apart), and column c stores slot q at position q + (c mod 32), positions past 63 + (c mod 32)
// wrapping (duplicated), so the B read of (column c, k-step ks, row group g) is at
// c * 96 + g * 16 + (c mod 32) + ks: an immediate offset, and the 16 pair columns a 16-lane
// group reads fall on distinct banks. The Gram panel in HBM holds exactly this image per
// sub-tile ([sub-tile][column][96], ob_panel_kernel), so staging is one contiguous LDS-DMA copy.
// Column 0 is the intercept: ones (unweighted, filled once in LDS) or sqrt(w) (weighted).
// ---------------------------------------------------------------------------------------------
struct Work {
  uint32_t rb, cg, chunk, g, t0, t1, n, rep0;
  const double* X;
  int64_t ld;
};

__device__ __forceinline__ Work map_work(const GramArgs& a) {
  // XCD-aware bijective remap: consecutive work items (same chunk, successive replicate
  // batches) land on one XCD so the chunk's sub-tiles are shared through that XCD's L2.
  const uint32_t nwg = gridDim.x, bid = blockIdx.x;
  const uint32_t xcd = bid & 7u, slot = bid >> 3, q8 = nwg >> 3, r8 = nwg & 7u;
  const uint32_t wi = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + slot;
  Work w;
  w.rb = wi % a.nb_rep;
  const uint32_t tq = wi / a.nb_rep;
  w.cg = tq % (uint32_t)a.n_cg;
  w.chunk = tq / (uint32_t)a.n_cg;
  w.g = a.chunks[w.chunk * 3];
  w.t0 = a.chunks[w.chunk * 3 + 1];
  w.t1 = a.chunks[w.chunk * 3 + 2];
  w.X = w.g ? a.gcols1 : a.gcols0;
  w.ld = w.g ? a.ld1 : a.ld0;
  w.n = w.g ? a.n1 : a.n0;
  w.rep0 = w.rb * 64;
  return w;
}

// Block barrier for LDS hand-offs only. __syncthreads() also drains this wave's global loads
// (s_waitcnt vmcnt(0)), which would stall the producers on the sub-tile DMA they just issued;
// the DMA is waited for explicitly (vmcnt) before the barrier that publishes it.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// Per-lane LDS offsets of the pair (a(e), b(e)) for each of the wave's CB column blocks.
template <int CB>
__device__ __forceinline__ void pair_offsets(const GramArgs& a, int cb0, int lane, int (&offa)[CB], int (&offb)[CB]) {
#pragma unroll
  for (int c = 0; c < CB; ++c) {
    const int e = (cb0 + c) * 16 + (lane & 15);
    int pa = 0, pb = 0;
    if (e < a.e) {
      int rem = e;
      while (rem >= a.k1 - pa) {
        rem -= a.k1 - pa;
        ++pa;
      }
      pb = pa + rem;
    }
    offa[c] = pa * kColStride + (lane >> 4) * 16 + (pa & 31);
    offb[c] = pb * kColStride + (lane >> 4) * 16 + (pb & 31);
  }
}

// LDS-DMA of one 64-row sub-tile: the Gram panel holds each sub-tile's staged image
// contiguously ([column][96] from column c_first), so it is one copy of (k1 - c_first) x 768 B in
// 1 KiB wave-instructions (16 B per lane), waves [w_lo, w_lo + nw) round-robin.
__device__ __forceinline__ void stage_dma(const GramArgs& a, const Work& w, uint32_t xt_byte_off, size_t gbase,
                                          int wave, int w_lo, int nw, int lane,
                                          __attribute__((address_space(3))) unsigned char* lds3) {
  const int ncl = a.k1 - a.c_first;
  const uint32_t bytes = (uint32_t)ncl * kColStride * 8;
  const char* src = reinterpret_cast<const char*>(w.X + (gbase >> 6) * (size_t)ncl * kColStride);
  const uint32_t dst = xt_byte_off + (uint32_t)a.c_first * kColStride * 8;
  for (uint32_t t = wave - w_lo; t * 1024 < bytes; t += nw)
    if (t * 1024 + lane * 16 < bytes)
      __builtin_amdgcn_global_load_lds(src + t * 1024 + lane * 16,
                                       (__attribute__((address_space(3))) void*)(lds3 + dst + t * 1024), 16, 0, 0);
}

// Level-2 draws of `tile` into a u8 count image (OBRS-2, ob_spec.h: full tiles take sixteen
// 8-bit draws per Philox call, the partial last tile two 64-bit ones). Wave wv of nw owns
// replicates [64 wv / nw, 64 (wv+1) / nw). Full tile: replicate r's draws are floor(m/16) whole
// calls plus, when m % 16 != 0, one part call (index floor(m/16)). The whole calls of the wave's
// replicates form one list (cum = its prefix, publish_counts) walked by the 64 lanes in stride,
// unmasked; part k of nparts takes the slice [C k / nparts, C (k+1) / nparts), and the last part
// also takes the part calls, one lane per replicate. A lane finds its replicate with a uniform
// cursor plus the few boundaries inside its 64-call window (readlane, no LDS chains). The
// atomics return nothing: check_counts catches overflow.
static_assert(OB_TILE_ROWS == 256u, "full-tile draws are bytes");
__device__ __forceinline__ bool full_tile(const Work& w, uint32_t tile) {
  return w.n - tile * OB_TILE_ROWS >= OB_TILE_ROWS;
}

__device__ __forceinline__ void add_draw(uint32_t* img, uint32_t r, uint32_t lr) {
  atomicAdd(&img[(lr >> 2) * kImgRow + r], 1u << ((lr & 3u) * 8u));
}

// The four draws of one Philox word (byte b = a row of the tile). The LDS byte address of row b of
// replicate r is (b >> 2) * 4 kImgRow + 4 r = ((b & 0xFC) << 6) + 4 r: with lo = (w << 6) &
// 0x3F003F00 (16-bit halves = bytes 0 and 2 of w, so placed) and hi = (w >> 2) & 0x3F003F00 (bytes
// 1 and 3), a draw's address is one SDWA add (4 r + half h of lo or hi), and with m = (w << 3) &
// 0x18181818 (byte b = its byte lane x 8) its increment one SDWA shift (1 << byte b of m), where the
// compiler would emit a shift-and-mask chain for each. The shifts read only byte b of their
// operand, so no mask per draw is needed.
template <int H>
__device__ __forceinline__ uint32_t sdwa_add_half(uint32_t base, uint32_t a) {
  uint32_t r;
  if constexpr (H == 0)
    asm("v_add_u32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0" : "=v"(r) : "v"(base), "v"(a));
  else
    asm("v_add_u32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1" : "=v"(r) : "v"(base), "v"(a));
  return r;
}

template <int B>
__device__ __forceinline__ uint32_t sdwa_shl_byte(uint32_t m, uint32_t one) {
  uint32_t r;
  if constexpr (B == 0)
    asm("v_lshlrev_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_0 src1_sel:DWORD" : "=v"(r) : "v"(m), "v"(one));
  else if constexpr (B == 1)
    asm("v_lshlrev_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:DWORD" : "=v"(r) : "v"(m), "v"(one));
  else if constexpr (B == 2)
    asm("v_lshlrev_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_2 src1_sel:DWORD" : "=v"(r) : "v"(m), "v"(one));
  else
    asm("v_lshlrev_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_3 src1_sel:DWORD" : "=v"(r) : "v"(m), "v"(one));
  return r;
}

template <int B>
__device__ __forceinline__ void add_draw_byte(uint32_t* img, uint32_t rep_off, uint32_t a, uint32_t m, uint32_t one) {
  atomicAdd(reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(img) + sdwa_add_half<(B >> 1)>(rep_off, a)),
            sdwa_shl_byte<B>(m, one));
}

#ifndef OB_CNT_PERM
#define OB_CNT_PERM 1  // 1: a draw's LDS address by one v_perm_b32 (byte 0 = 4 r, byte 1 = its row word)
#endif
template <int B>
__device__ __forceinline__ void add_draw_perm(uint32_t* img, uint32_t rep_off, uint32_t q, uint32_t m, uint32_t one) {
  // bytes of the address: rep_off's byte 0 (< 256), byte B of q (the row word), zero, zero
  const uint32_t addr = __builtin_amdgcn_perm(q, rep_off, 0x0C0C0000u | ((4u + B) << 8));
  atomicAdd(reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(img) + addr), sdwa_shl_byte<B>(m, one));
}

// rep_off = 4 r, the replicate's byte offset in every row word
__device__ __forceinline__ void add_draws_word(uint32_t* img, uint32_t rep_off, uint32_t w, uint32_t one) {
  const uint32_t m = (w << 3) & 0x18181818u;
  if (OB_CNT_PERM) {
    const uint32_t q = (w >> 2) & 0x3F3F3F3Fu;  // byte b = the row word of draw b
    add_draw_perm<0>(img, rep_off, q, m, one);
    add_draw_perm<1>(img, rep_off, q, m, one);
    add_draw_perm<2>(img, rep_off, q, m, one);
    add_draw_perm<3>(img, rep_off, q, m, one);
    return;
  }
  const uint32_t lo = (w << 6) & 0x3F003F00u, hi = (w >> 2) & 0x3F003F00u;
  add_draw_byte<0>(img, rep_off, lo, m, one);
  add_draw_byte<1>(img, rep_off, hi, m, one);
  add_draw_byte<2>(img, rep_off, lo, m, one);
  add_draw_byte<3>(img, rep_off, hi, m, one);
}

__device__ __forceinline__ void level2_draws(const GramArgs& a, const Work& w, uint32_t tile, uint32_t* cnt,
                                             const uint32_t* mc, const uint32_t* cum, int k, int nparts, int wv,
                                             int nw, int lane) {
  const uint32_t S = min(OB_TILE_ROWS, w.n - tile * OB_TILE_ROWS);
  const bool full = S == OB_TILE_ROWS;
  const int r_lo = 64 * wv / nw, r_hi = 64 * (wv + 1) / nw, nr = r_hi - r_lo;
  if (nr <= 0) return;
  const uint32_t c_lo = cum[r_lo], C = cum[r_hi] - c_lo;
  const uint32_t f_lo = c_lo + C * (uint32_t)k / (uint32_t)nparts;
  const uint32_t f_hi = c_lo + C * (uint32_t)(k + 1) / (uint32_t)nparts;
  const uint32_t bnd = lane < nr ? cum[r_lo + 1 + lane] : 0xFFFFFFFFu;  // end of replicate r_lo + lane
  const uint32_t c2 = (tile << 1) | w.g;
  const uint32_t rep0 = a.first_rep + w.rep0;
  const uint32_t one = 1u;  // the SDWA shifts' operand (a VGPR)
  int rr = r_lo;  // uniform: replicate of the window's first call
  for (uint32_t f0 = f_lo; f0 < f_hi; f0 += 64) {
    while (rr < r_hi - 1 && (uint32_t)__builtin_amdgcn_readlane(bnd, rr - r_lo) <= f0) ++rr;
    const uint32_t f = f0 + lane;
    int r = rr;
    uint32_t base = rr > r_lo ? (uint32_t)__builtin_amdgcn_readlane(bnd, rr - r_lo - 1) : c_lo;
    for (int i = rr; i < r_hi - 1; ++i) {
      const uint32_t b = (uint32_t)__builtin_amdgcn_readlane(bnd, i - r_lo);
      if (b > f0 + 63) break;
      if (f >= b) {
        r = i + 1;
        base = b;
      }
    }
    if (f < f_hi) {
      const uint32_t pp = f - base;
      ob_u32x4 u;
      if (a.diag & 64)  // timing ablation (OB_GRAM_DIAG 64): no Philox, wrong draws
        u = ob_u32x4{pp * 0x9E3779B9u ^ r, pp * 0x85EBCA6Bu ^ c2, pp * 0xC2B2AE35u, pp ^ 0x27D4EB2Fu};
      else
        u = ob_philox_x3(pp, rep0 + r, c2, OB_TAG_L2, a.key0, a.key1);
      if (full && (a.diag & 32)) {  // timing ablation (OB_GRAM_DIAG 32): no LDS atomics
        if ((u.x ^ u.y ^ u.z ^ u.w) == 0x5EED5EEDu) cnt[r] = 1u;
      } else if (full) {
        const uint32_t wd[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
        for (int i = 0; i < 4; ++i) add_draws_word(cnt, (uint32_t)r * 4u, wd[i], one);
      } else {
        add_draw(cnt, (uint32_t)r, ob_mulhi64(u.x, u.y, S));
        if (2 * pp + 1 < mc[r]) add_draw(cnt, (uint32_t)r, ob_mulhi64(u.z, u.w, S));
      }
    }
  }
  if (full && k == nparts - 1 && lane < nr) {  // the part calls
    const int r = r_lo + lane;
    const uint32_t m = mc[r], nd = m & 15u;
    if (nd) {
      const ob_u32x4 u = ob_philox_x3(m >> 4, rep0 + r, c2, OB_TAG_L2, a.key0, a.key1);
      const uint32_t wd[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
      for (uint32_t d = 0; d < 15; ++d)
        if (d < nd) add_draw(cnt, (uint32_t)r, (wd[d >> 2] >> (8 * (d & 3))) & 0xFFu);
    }
  }
}

// Full tiles of the count kernel (OB_CNT_MAP): the whole calls of all 64 replicates form one list
// that the block's waves walk in 64-call windows, window j on wave j mod 4, one lane per call. The
// list is call-major: call index p of every replicate that has one, replicates ascending, then p + 1.
// The first cmin = min_r(calls) indices hold all 64 replicates, so window p < cmin is call p of
// replicate `lane` (no lookup); past them an LDS call map (word = p << 6 | r, written by wave 0
// when it publishes the tile's counts) lists the rest. Either way the lanes of a window draw for
// distinct replicates (up to the seam between two indices past cmin), and with the replicate-minor
// image (kImgRow) their atomics fall on distinct banks. The part calls (m % 16 draws, one per
// replicate) form one extra window, one lane per replicate. Same (call, replicate) -> draws as
// level2_draws, so the same counts.
#ifndef OB_CNT_MAPCAP
#define OB_CNT_MAPCAP 2048
#endif
constexpr uint32_t kCallMapCap = OB_CNT_MAPCAP;  // calls past the dense prefix a (tile, batch) map holds

__device__ __forceinline__ void level2_map_draws(const GramArgs& a, const Work& w, uint32_t tile, uint32_t* cnt,
                                                 const uint32_t* mc, const uint32_t* cmap, uint32_t C,
                                                 uint32_t cmin, int wv, int lane) {
  const uint32_t nwin = (C + 63u) >> 6;
  const uint32_t c2 = (tile << 1) | w.g;
  const uint32_t rep0 = a.first_rep + w.rep0;
  const uint32_t one = 1u;
  for (uint32_t win = (uint32_t)wv; win <= nwin; win += 4) {
    if (win < nwin) {
      const uint32_t f = win * 64u + (uint32_t)lane;
      if (f < C) {
        uint32_t r = (uint32_t)lane, pp = win;
        if (win >= cmin) {
          const uint32_t e = cmap[f - cmin * 64u];
          r = e & 63u;
          pp = e >> 6;
        }
        ob_u32x4 u;
        if (a.diag & 64)  // timing ablation (OB_GRAM_DIAG 64): no Philox, wrong draws
          u = ob_u32x4{pp * 0x9E3779B9u ^ r, pp * 0x85EBCA6Bu ^ c2, pp * 0xC2B2AE35u, pp ^ 0x27D4EB2Fu};
        else
          u = ob_philox_x3(pp, rep0 + r, c2, OB_TAG_L2, a.key0, a.key1);
        if (a.diag & 32) {  // timing ablation (OB_GRAM_DIAG 32): no LDS atomics
          if ((u.x ^ u.y ^ u.z ^ u.w) == 0x5EED5EEDu) cnt[r] = 1u;
        } else {
          const uint32_t wd[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
          for (int i = 0; i < 4; ++i) add_draws_word(cnt, r * 4u, wd[i], one);
        }
      }
    } else {  // the part calls
      const uint32_t m = mc[lane], nd = m & 15u;
      if (nd) {
        const ob_u32x4 u = ob_philox_x3(m >> 4, rep0 + (uint32_t)lane, c2, OB_TAG_L2, a.key0, a.key1);
        const uint32_t wd[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
        for (uint32_t d = 0; d < 15; ++d)
          if (d < nd) add_draw(cnt, (uint32_t)lane, (wd[d >> 2] >> (8 * (d & 3))) & 0xFFu);
      }
    }
  }
}

#ifndef OB_CNT_NT
#define OB_CNT_NT 0  // 1: the i8 count images are written with nontemporal stores
#endif
// A row drawn 256+ times wraps its byte and carries into the next one, which lowers the
// replicate's byte sum below m: comparing sums with the level-1 counts is an exact check.
// Thread (r = lane, sub-tile part = wave) reads replicate r's 16 words of sub-tile `part` (bank r
// mod 32: conflict-free), stores them straight to the HBM image (the tile's first ns sub-tiles),
// clears them in LDS, recycling the image without another pass, and adds its byte sum to the
// replicate's LDS sum; wave 0 compares the sums with m after the next barrier (check_sums).
// I8: the A-fragment units of ob_gram_i8.hip ([sub-tile][16-replicate block][lane][16 B], lane
// = replicate 16 m + (l & 15) holding rows 16 (l >> 4) .. + 15), i.e. word group q of the thread
// is unit sb * 256 + (r >> 4) * 64 + q * 16 + (r & 15). f64: replicate r's 16 words at r * 17 of
// the sub-tile image, then its zero pad word.
template <bool I8>
__device__ __forceinline__ void check_store_counts(const GramArgs& a, uint32_t* cnt, uint32_t* lsum, int my,
                                                   uint32_t tt, uint32_t rb, uint32_t ns) {
  const int r = my & 63, part = my >> 6;
  uint32_t* col = cnt + part * 16 * kImgRow + r;
  uint32_t v[16];
  uint32_t sum = 0, hib = 0;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    v[i] = col[i * kImgRow];
    sum = __builtin_amdgcn_sad_u8(v[i], 0u, sum);
    hib |= v[i] & 0x80808080u;
  }
  if (I8 && hib && !(a.diag & 1632)) atomicOr(a.flags, 2u);  // the i8 Gram reads counts as signed bytes: at most 127
  if ((uint32_t)part < ns && !(a.diag & 512)) {  // timing ablation (gram_diag 512): no image stores
    if constexpr (I8) {
      uint4* out = reinterpret_cast<uint4*>(const_cast<uint32_t*>(a.counts)) + ((size_t)tt * a.nb_rep + rb) * 1024 +
                   part * 256 + (r >> 4) * 64 + (r & 15);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (OB_CNT_NT) {
          typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
          const u32x4_t u4 = {v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]};
          __builtin_nontemporal_store(u4, reinterpret_cast<u32x4_t*>(out + q * 16));
        } else {
          out[q * 16] = make_uint4(v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]);
        }
      }
    } else {
      uint32_t* out = const_cast<uint32_t*>(a.counts) + ((size_t)tt * a.nb_rep + rb) * 4 * kCimgWords +
                      part * kCimgWords + r * kCimgStride;
#pragma unroll
      for (int i = 0; i < 16; ++i) out[i] = v[i];
      out[16] = 0u;
    }
  }
#pragma unroll
  for (int i = 0; i < 16; ++i) col[i * kImgRow] = 0u;
  atomicAdd(&lsum[r], sum);
}

// Wave 0, after the barrier that follows a tile's check_store_counts: the tile's byte sums against
// its level-1 counts, then the sums cleared for the tile after next.
__device__ __forceinline__ void check_sums(const GramArgs& a, uint32_t* lsum, const uint32_t* mc, int lane) {
  if (lsum[lane] != mc[lane] && !(a.diag & 1632)) atomicOr(a.flags, 1u);
  lsum[lane] = 0u;
}

// Level-1 count of global tile tt (group 0's tiles, then group 1's) for batch replicate r.
__device__ __forceinline__ uint32_t level1_count(const GramArgs& a, uint32_t rep0, uint32_t tt, uint32_t r) {
  const uint32_t rep = rep0 + r;
  return rep < a.n_reps ? a.m1[(size_t)rep * a.tiles_total + tt] : 0u;
}

__device__ __forceinline__ void publish_counts(const Work& w, uint32_t tile, uint32_t m, uint32_t* mc, uint32_t* cum,
                                               int lane, uint32_t* cmap, uint32_t* cminp) {
  mc[lane] = m;
  // calls in the whole-call list: full tile floor(m/16) (the part call goes apart), else ceil(m/2)
  const bool full = full_tile(w, tile);
  const uint32_t c = full ? m >> 4 : (m + 1) >> 1;
  uint32_t v = c;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t t = __shfl_up(v, o);
    if (lane >= o) v += t;
  }
  cum[lane + 1] = v;
  if (lane == 0) cum[0] = 0;
  // the call map of a full tile (level2_map_draws): call-major past the dense prefix of cmin
  // indices, when those calls fit it
  if (cmap && full) {
    uint32_t cmin = c, cmax = c;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      cmin = min(cmin, (uint32_t)__shfl_xor(cmin, o));
      cmax = max(cmax, (uint32_t)__shfl_xor(cmax, o));
    }
    const uint32_t total = (uint32_t)__builtin_amdgcn_readlane(v, 63);
    if (total - cmin * 64u <= kCallMapCap) {
      uint32_t base = 0;
      for (uint32_t j = cmin; j < cmax; ++j) {
        const uint64_t mask = __ballot(c > j);
        if (c > j)
          cmap[base + __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u))] =
              (j << 6) | (uint32_t)lane;
        base += (uint32_t)__popcll(mask);
      }
    }
    if (lane == 0) *cminp = cmin;
  }
}

template <int CB>
__device__ __forceinline__ void store_partials(const GramArgs& a, const Work& w, int cb0, int lane,
                                               const ob_d4 (&acc)[4][CB]) {
#pragma unroll
  for (int c = 0; c < CB; ++c) {
    if (cb0 + c >= a.ncb) continue;
    const int e = (cb0 + c) * 16 + (lane & 15);
#pragma unroll
    for (int q4 = 0; q4 < 4; ++q4)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const uint32_t rep = w.rep0 + q4 * 16 + (lane >> 4) + 4 * r;
        if (rep < a.n_reps) a.partial[((size_t)w.chunk * a.rep_pad + rep) * a.e_pad + e] = acc[q4][c][r];
      }
  }
}

// ---------------------------------------------------------------------------------------------
// Level-2 counts: one block per (64-replicate batch, run of tiles). Per tile: the batch's level-1
// counts and call prefix, the level-2 draws into an LDS u8 image, the exact overflow check, then
// the image written to HBM in the Gram kernel's sub-tile layout: per 64-row sub-tile, replicate
// r's 16 count words at r * 17 (+1 pad word: odd stride, conflict-free A-fragment reads), so the
// Gram kernel fetches a sub-tile with a plain LDS-DMA copy. Counts are drawn once per replicate
// batch, whatever the number of column groups.
// ---------------------------------------------------------------------------------------------
#ifndef OB_CNT_MAP
#define OB_CNT_MAP 1  // full tiles walk one call list through an LDS call map (level2_map_draws)
#endif
#ifndef OB_CNT_TILES
#define OB_CNT_TILES 8  // tiles per count block (A/B builds: tools/build_alt.sh ... -DOB_CNT_TILES=n)
#endif
constexpr int kCntTilesPerBlock = OB_CNT_TILES;

// I8: the image is written in the A-fragment order of ob_gram_i8.hip instead (v_mfma_i32_16x16x64_i8):
// per (tile, batch) [sub-tile][16-replicate block m][lane][16 B], lane l = replicate 16 m + (l & 15),
// rows 16 (l >> 4) + j of the sub-tile -- 16 KB, one 16-byte store per thread and unit.
template <bool I8>
__global__ __launch_bounds__(kBlock) void ob_count_kernel(const GramArgs a) {
  __shared__ uint32_t img[kImgWords];
  __shared__ uint32_t mcb[2][64], cumb[2][65], lsumb[2][64], cminb[2];
  __shared__ uint32_t cmap[OB_CNT_MAP ? kCallMapCap : 1];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  Work w{};
  w.rb = a.rb0 + blockIdx.y;
  w.rep0 = w.rb * 64;
  const uint32_t tt0 = blockIdx.x * kCntTilesPerBlock;
  const uint32_t tt1 = min(a.tiles_total, tt0 + kCntTilesPerBlock);
  // wave 0 loads tile tt+1's level-1 counts while the block draws tile tt
  uint32_t m_next = (wave == 0 && tt0 < tt1) ? level1_count(a, w.rep0, tt0, lane) : 0u;
  // the image starts zeroed once; check_store_counts clears what it read
  for (int i = tid; i < kImgWords; i += kBlock) img[i] = 0u;
  if (tid < 128) lsumb[tid >> 6][tid & 63] = 0u;
  // Two barriers per tile: the call prefix, counts and sums are double-buffered, so publishing
  // tile tt + 1's (buffer (tt + 1) & 1) never races the checks of tile tt (buffer tt & 1), and the
  // image clears of tile tt complete before the barrier that follows that publish.
  for (uint32_t tt = tt0; tt < tt1; ++tt) {
    uint32_t* mc = mcb[tt & 1];
    uint32_t* cum = cumb[tt & 1];
    w.g = tt >= a.tiles0 ? 1u : 0u;
    w.n = w.g ? a.n1 : a.n0;
    const uint32_t tile = tt - (w.g ? a.tiles0 : 0u);
    if (wave == 0) {
      publish_counts(w, tile, m_next, mc, cum, lane, OB_CNT_MAP ? cmap : nullptr, &cminb[tt & 1]);
      if (tt + 1 < tt1) m_next = level1_count(a, w.rep0, tt + 1, lane);
    }
    __syncthreads();
    if (wave == 0 && tt > tt0) check_sums(a, lsumb[(tt - 1) & 1], mcb[(tt - 1) & 1], lane);
    const uint32_t C = cum[64];
    const uint32_t cmin = cminb[tt & 1];
    if (a.diag & 1024) {  // timing ablation (gram_diag 1024): no level-2 draws at all
    } else if (OB_CNT_MAP && full_tile(w, tile) && C - cmin * 64u <= kCallMapCap)
      level2_map_draws(a, w, tile, img, mc, cmap, C, cmin, wave, lane);
    else
      level2_draws(a, w, tile, img, mc, cum, 0, 1, wave, 4, lane);
    __syncthreads();
    const uint32_t ns = (min(OB_TILE_ROWS, w.n - tile * OB_TILE_ROWS) + 63) >> 6;
    check_store_counts<I8>(a, img, lsumb[tt & 1], tid, tt, w.rb, ns);
  }
  if (tt0 < tt1) {
    __syncthreads();
    if (wave == 0) check_sums(a, lsumb[(tt1 - 1) & 1], mcb[(tt1 - 1) & 1], lane);
  }
}

// ---------------------------------------------------------------------------------------------
// Gram: 4 waves (one per SIMD) per block, two blocks per CU, CB column blocks per wave; the two
// blocks on a CU drift apart, so one block's barrier never drains a SIMD's MFMA pipe. One 64-row
// sub-tile per step, one LDS barrier per step. The next sub-tile's staged rows and its count
// image arrive by LDS-DMA issued at the start of the step; A fragments are count bytes
// (ds_read_b32 + convert) and B fragments pair products of staged values, both read one k-step
// ahead of their MFMAs (register double buffer). No draws here: ob_count_kernel made the counts.
// ---------------------------------------------------------------------------------------------
constexpr int kXtOff = 2 * kCimgWords * 4;
static_assert(kXtOff % 16 == 0, "staged sub-tiles must stay 16-byte aligned");

template <int CB, bool UNIT>
__global__ __launch_bounds__(kBlock, 2) void ob_gram_kernel(const GramArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  uint32_t* cimg = reinterpret_cast<uint32_t*>(smem);      // [2][kCimgWords]
  double* xt = reinterpret_cast<double*>(smem + kXtOff);  // [2][k1][kColStride]
  __attribute__((address_space(3))) unsigned char* lds3 = (__attribute__((address_space(3))) unsigned char*)smem;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const Work w = map_work(a);
  const int cb0 = ((int)w.cg * 4 + wave) * CB;
  const bool mma = cb0 < a.ncb && !(a.diag & 2);
  const bool dma = !(a.diag & 4);
  const int buf_dbl = a.k1 * kColStride;
  const uint32_t tg0 = w.g ? a.tiles0 : 0u;
  auto tile_rows = [&](uint32_t t) { return min(OB_TILE_ROWS, w.n - t * OB_TILE_ROWS); };
  // LDS-DMA of one sub-tile's count image: 16 bytes per lane, 1 KiB per wave-instruction
  // (kCimgWords = 4.25 KiB: waves 0..3 one piece each, wave 0 the quarter piece too)
  auto stage_counts = [&](int buf, uint32_t tile, uint32_t s) {
    if (UNIT) return;
    const uint32_t* src = a.counts + (((size_t)(tg0 + tile) * a.nb_rep + w.rb) * 4 + s) * kCimgWords;
    for (int t = wave; t * 256 < kCimgWords; t += 4)
      if (t * 256 + lane * 4 < kCimgWords)
        __builtin_amdgcn_global_load_lds(src + t * 256 + lane * 4,
                                         (__attribute__((address_space(3))) void*)(lds3 + (buf * kCimgWords + t * 256) * 4),
                                         16, 0, 0);
  };

  const bool dbl = a.dbl != 0;
  if (w.t0 < w.t1) {
    if (a.c_first == 1)
      for (int i = tid; i < kColStride; i += kBlock) {
        xt[i] = 1.0;
        if (dbl) xt[buf_dbl + i] = 1.0;
      }
    stage_dma(a, w, kXtOff, (size_t)w.t0 * OB_TILE_ROWS, wave, 0, 4, lane, lds3);
    stage_counts(0, w.t0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  int offa[CB], offb[CB];
  pair_offsets<CB>(a, cb0, lane, offa, offb);
  ob_d4 acc[4][CB];
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int c = 0; c < CB; ++c) acc[r][c] = (ob_d4){0.0, 0.0, 0.0, 0.0};
  const uint32_t sh = (uint32_t)(lane >> 4) * 8u;
  // A fragment of replicate block q4, k-step ks: count byte of (rep q4*16 + lane&15, row 4ks + lane>>4)
  uint32_t aw[4];
  double bf[CB];
  size_t gbase = 0;
  auto read_k = [&](const uint32_t* cw, const double* xb, int ks, uint32_t (&w4)[4], double (&va)[CB],
                    double (&vb)[CB]) {
#pragma unroll
    for (int q4 = 0; q4 < 4; ++q4) w4[q4] = UNIT ? 0u : cw[q4 * 16 * kCimgStride + ks];
#pragma unroll
    for (int c = 0; c < CB; ++c) {
      va[c] = xb[offa[c] + ks];
      vb[c] = xb[offb[c] + ks];
    }
  };

  int j = 0;
  for (uint32_t tile = w.t0; tile < w.t1; ++tile) {
    const uint32_t ns = (tile_rows(tile) + 63) >> 6;
    for (uint32_t s = 0; s < ns; ++s, ++j) {
      const int cur = j & 1;
      const bool last_sub = s + 1 == ns;
      const bool has_next = !last_sub || tile + 1 < w.t1;
      const uint32_t ntile = last_sub ? tile + 1 : tile, nsub = last_sub ? 0u : s + 1;
      gbase = (size_t)tile * OB_TILE_ROWS + s * 64;
      if (has_next && dma && dbl) {
        stage_dma(a, w, kXtOff + (cur ^ 1) * buf_dbl * 8, (size_t)ntile * OB_TILE_ROWS + nsub * 64, wave, 0, 4, lane,
                  lds3);
        stage_counts(cur ^ 1, ntile, nsub);
      }
      const int cb_ = dbl ? cur : 0;
      const uint32_t* cw = cimg + cb_ * kCimgWords + (lane & 15) * kCimgStride;
      const double* xb = xt + cb_ * buf_dbl;
      if (mma) {
        {
          double va[CB], vb[CB];
          read_k(cw, xb, 0, aw, va, vb);
#pragma unroll
          for (int c = 0; c < CB; ++c) bf[c] = va[c] * vb[c];
        }
#pragma unroll
        for (int ks = 0; ks < 16; ++ks) {
          uint32_t an[4];
          double na[CB], nb[CB];
          if (ks < 15) read_k(cw, xb, ks + 1, an, na, nb);
          __builtin_amdgcn_sched_barrier(0);
          double af[4];
#pragma unroll
          for (int q4 = 0; q4 < 4; ++q4)
            af[q4] = UNIT ? ((gbase + ks * 4 + (lane >> 4) < w.n) ? 1.0 : 0.0) : (double)((aw[q4] >> sh) & 0xFFu);
#pragma unroll
          for (int q4 = 0; q4 < 4; ++q4)
#pragma unroll
            for (int c = 0; c < CB; ++c)
              acc[q4][c] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[q4], bf[c], acc[q4][c], 0, 0, 0);
          __builtin_amdgcn_sched_barrier(0);
          if (ks < 15) {
#pragma unroll
            for (int q4 = 0; q4 < 4; ++q4) aw[q4] = an[q4];
#pragma unroll
            for (int c = 0; c < CB; ++c) bf[c] = na[c] * nb[c];
          }
          __builtin_amdgcn_sched_barrier(0);
        }
      }
      if (!dbl && has_next && dma) {  // one buffer: every read of this sub-tile done, then refill it
        lds_barrier();
        stage_dma(a, w, kXtOff, (size_t)ntile * OB_TILE_ROWS + nsub * 64, wave, 0, 4, lane, lds3);
        stage_counts(0, ntile, nsub);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the next sub-tile has landed
      lds_barrier();
    }
  }
  if (mma) store_partials<CB>(a, w, cb0, lane, acc);
}

// Sum of partial Grams over each group's chunks, chunk order fixed -> bitwise reproducible.
__global__ __launch_bounds__(kBlock) void ob_reduce_kernel(const double* partial, const uint32_t* chunks,
                                                           int n_chunks, uint32_t rep_pad, int e_pad,
                                                           uint32_t n_reps, double* gram) {
  const size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= (size_t)n_reps * e_pad) return;
  const uint32_t rep = (uint32_t)(i / e_pad);
  const int e = (int)(i % e_pad);
  double s0 = 0.0, s1 = 0.0;
  for (int c = 0; c < n_chunks; ++c) {
    const double v = partial[((size_t)c * rep_pad + rep) * e_pad + e];
    if (chunks[c * 3] == 0)
      s0 += v;
    else
      s1 += v;
  }
  gram[((size_t)rep * 2 + 0) * e_pad + e] = s0;
  gram[((size_t)rep * 2 + 1) * e_pad + e] = s1;
}

// ---------------------------------------------------------------------------------------------
// Solve: one 64-lane wave per replicate, matrices in LDS.
// ---------------------------------------------------------------------------------------------
struct SolveArgs {
  const double* gram;  // [rep][2][e_pad]
  int e_pad, k1, k, pool_pos, ref_mode, weighted;
  int yc;  // the outcome's column in the extended Gram (p + 1 + t)
  double rows_a, rows_b;
  int n_norm, n_base;
  const int32_t* norm;  // start[n_norm+1] | idx | m[n_norm] | pstart[n_norm+1] | pidx | has_base[n_norm]
  int off_idx, off_m, off_pstart, off_pidx, off_has;
  double* rows;
  uint8_t* ok;
  int row_len;
  uint32_t n_reps;
  double* gram_out;    // optional copy of the replicate-0 extended Grams (point estimate)
  double* raw_beta_b;  // optional: replicate-0 beta_B before normalization (ols.rs residuals)
  int raw_status;      // 1: ok[] receives the status code (1 ok, 0 Cholesky, 2 zero weight)
};

// normalization.rs:5-51
__device__ void normalize_coeffs(double* beta, const SolveArgs& a, const int32_t* starts,
                                 const int32_t* idx, double* base) {
  for (int v = 0; v < a.n_norm; ++v) {
    const int s = starts[v], e = starts[v + 1];
    base[v] = 0.0;
    if (e == s) continue;
    double sum = 0.0;
    for (int t = s; t < e; ++t) sum += beta[idx[t]];
    const int cat = a.norm[a.off_m + v];  // category count, or -1: matches + 1 (normalization.rs:28-31)
    const int mm = cat >= 0 ? cat : (e - s) + 1;
    if (mm == 0) continue;
    const double mean = sum / (double)mm;
    base[v] = -mean;
    beta[0] += mean;
    for (int t = s; t < e; ++t) beta[idx[t]] -= mean;
  }
}

// One block per replicate. DUAL (two waves, when both groups' matrices fit in LDS together): wave g
// factors group g's normal equations while the other wave factors the other group's, each with
// wave-local synchronization; then wave 0 picks beta* (the pooled system's own factorization
// included) and writes the row with its lanes. Otherwise one wave does the two groups in turn.
template <bool DUAL>
__global__ __launch_bounds__(128) void ob_solve_kernel(const SolveArgs a) {
  extern __shared__ __attribute__((aligned(16))) double sm[];
  __shared__ int st_sh[2];
  const int lane = threadIdx.x & 63, w = DUAL ? (int)(threadIdx.x >> 6) : 0;
  const uint32_t rep = blockIdx.x;
  if (rep >= a.n_reps) return;
  const int k = a.k, k1 = a.k1, kp = k + 1;
  double* M = sm;                              // kp * kp (group A, then the pooled system)
  double* M1 = M + kp * kp;                    // DUAL: k * k (group B)
  double* rhs = M1 + (DUAL ? k * k : 0);       // kp
  double* rhs1 = rhs + kp;                     // kp
  double* beta_a = rhs1 + kp;                  // k
  double* beta_b = beta_a + kp;                // k
  double* xam = beta_b + kp;                   // k
  double* xbm = xam + kp;                      // k
  double* bstar = xbm + kp;                    // kp (pooled before removal)
  double* base = bstar + kp;                   // 3 * n_norm: a, b, star
  const double* GA = a.gram + (size_t)rep * 2 * a.e_pad;
  const double* GB = GA + a.e_pad;
  double* row = a.rows + (size_t)rep * a.row_len;
  if (a.gram_out && rep == 0)
    for (int i = threadIdx.x; i < 2 * a.e_pad; i += blockDim.x) a.gram_out[i] = GA[i];

  // OLS for both groups (estimation.rs:53-54 -> ols.rs:44-144)
  int ok_g = 1;
  for (int g = w; g < 2; g += DUAL ? 2 : 1) {
    const double* G = g ? GB : GA;
    double* beta = g ? beta_b : beta_a;
    double* Mg = (DUAL && g) ? M1 : M;
    double* rg = (DUAL && g) ? rhs1 : rhs;
    for (int i = lane; i < k * k; i += 64) {
      const int r = i % k, c = i / k;
      Mg[r + c * k] = gpair(G, r, c, k1);
    }
    for (int i = lane; i < k; i += 64) rg[i] = gpair(G, i, a.yc, k1);
    ob_sync<DUAL>();
    if (!wave_cholesky<DUAL>(Mg, k, lane)) {
      ok_g = 0;
      break;
    }
    wave_chol_solve<DUAL>(Mg, k, rg, lane);
    if (g == 1 && a.raw_beta_b && rep == 0)
      for (int i = lane; i < k; i += 64) a.raw_beta_b[i] = rg[i];
    const double sw = G[0];
    for (int i = lane; i < k; i += 64) {
      beta[i] = rg[i];
      (g ? xbm : xam)[i] = gpair(G, 0, i, k1) / sw;  // estimation.rs:56-71 (weighted or row mean)
    }
  }
  if (lane == 0) st_sh[w] = ok_g;
  __syncthreads();
  if (w != 0) return;
  uint8_t status = (st_sh[0] && (!DUAL || st_sh[1])) ? 1 : 0;
  const int32_t* nst = a.norm;
  const int32_t* nidx = a.norm + a.off_idx;
  const int32_t* pst = a.norm + a.off_pstart;
  const int32_t* pidx = a.norm + a.off_pidx;
  const int32_t* has = a.norm + a.off_has;
  double* base_a = base;
  double* base_b = base + a.n_norm;
  double* base_s = base + 2 * a.n_norm;
  if (status == 1 && a.n_norm > 0) {  // estimation.rs:76-91
    if (lane == 0) {
      normalize_coeffs(beta_a, a, nst, nidx, base_a);
      normalize_coeffs(beta_b, a, nst, nidx, base_b);
      for (int v = 0; v < a.n_norm; ++v) base_s[v] = 0.0;
    }
    ob_sync<DUAL>();
  }
  // beta* (builder.rs:536-621)
  if (status == 1) {
    if (a.ref_mode == OB_REF_GROUP_A || a.ref_mode == OB_REF_GROUP_B) {
      const double* src = a.ref_mode == OB_REF_GROUP_A ? beta_a : beta_b;
      for (int i = lane; i < k; i += 64) bstar[i] = src[i];
      if (lane == 0)
        for (int v = 0; v < a.n_norm; ++v) base_s[v] = a.ref_mode == OB_REF_GROUP_A ? base_a[v] : base_b[v];
    } else if (a.ref_mode == OB_REF_WEIGHTED || a.ref_mode == OB_REF_COTTON) {
      const double sa = a.weighted ? GA[0] : a.rows_a;
      const double sb = a.weighted ? GB[0] : a.rows_b;
      const double tot = sa + sb;
      if (tot == 0.0) {
        status = 2;
      } else {
        const double wA = sa / tot, wB = 1.0 - wA;
        for (int i = lane; i < k; i += 64) bstar[i] = beta_a[i] * wA + beta_b[i] * wB;
        if (lane == 0)
          for (int v = 0; v < a.n_norm; ++v) base_s[v] = base_a[v] * wA + base_b[v] * wB;
      }
    } else {  // Pooled / Neumark: [A; B] with the group indicator at pool_pos
      const int ip = a.pool_pos;
      for (int i = lane; i < kp * kp; i += 64) {
        const int u = i % kp, v = i / kp;
        double val;
        if (u == ip && v == ip) {
          val = GA[0];
        } else if (u == ip || v == ip) {
          const int o = (u == ip) ? (v < ip ? v : v - 1) : (u < ip ? u : u - 1);
          val = gpair(GA, 0, o, k1);
        } else {
          const int ou = u < ip ? u : u - 1, ov = v < ip ? v : v - 1;
          val = gpair(GA, ou, ov, k1) + gpair(GB, ou, ov, k1);
        }
        M[u + v * kp] = val;
      }
      for (int u = lane; u < kp; u += 64) {
        if (u == ip) {
          rhs[u] = gpair(GA, 0, a.yc, k1);
        } else {
          const int o = u < ip ? u : u - 1;
          rhs[u] = gpair(GA, o, a.yc, k1) + gpair(GB, o, a.yc, k1);
        }
      }
      ob_sync<DUAL>();
      if (!wave_cholesky<DUAL>(M, kp, lane)) {
        status = 0;
      } else {
        wave_chol_solve<DUAL>(M, kp, rhs, lane);
        if (lane == 0) {
          if (a.n_norm > 0) normalize_coeffs(rhs, a, pst, pidx, base_s);
          for (int u = 0, d = 0; u < kp; ++u)
            if (u != ip) bstar[d++] = rhs[u];
        }
      }
    }
  }
  ob_sync<DUAL>();
  if (status != 1) {
    for (int i = lane; i < a.row_len; i += 64) row[i] = __builtin_nan("");
  } else {
    // decomposition.rs:56-122 with the lanes over the coefficients; the six sums by a wave reduction
    const int kd = k + a.n_base;
    double* dex = row + 6;
    double* dun = row + 6 + kd;
    double sum[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};  // explained, x_A b_A, x_B b_B, endowments, coefficients, interaction
    double* tail = row + 6 + 2 * kd;
    for (int j = lane; j < k; j += 64) {
      const double xa = xam[j], xb = xbm[j], ba = beta_a[j], bb = beta_b[j], bs = bstar[j];
      const double dx = xa - xb, db = ba - bb;
      sum[0] += dx * bs;
      sum[1] += xa * ba;
      sum[2] += xb * bb;
      sum[3] += dx * bb;
      sum[4] += xb * db;
      sum[5] += dx * db;
      dex[j] = dx * bs;
      dun[j] = xa * (ba - bs) + xb * (bs - bb);
      tail[j] = ba;
      tail[k + j] = bb;
      tail[2 * k + j] = xa;
      tail[3 * k + j] = xb;
      tail[4 * k + j] = bs;
    }
#pragma unroll
    for (int q = 0; q < 6; ++q)
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) sum[q] += __shfl_xor(sum[q], off);
    if (lane == 0) {
      double expl = sum[0], unexpl = (sum[1] - sum[2]) - sum[0];
      for (int v = 0, bi = 0; v < a.n_norm; ++v) {  // builder.rs:634-674
        if (!has[v]) continue;
        double sa = 0.0, sb = 0.0;
        for (int t = nst[v]; t < nst[v + 1]; ++t) {
          sa += xam[nidx[t]];
          sb += xbm[nidx[t]];
        }
        const double xa0 = 1.0 - sa, xb0 = 1.0 - sb;
        const double cu = xa0 * (base_a[v] - base_s[v]) + xb0 * (base_s[v] - base_b[v]);
        const double ce = (xa0 - xb0) * base_s[v];
        dun[k + bi] = cu;
        dex[k + bi] = ce;
        expl += ce;
        unexpl += cu;
        ++bi;
      }
      row[0] = expl;
      row[1] = unexpl;
      row[2] = sum[3];
      row[3] = sum[4];
      row[4] = sum[5];
      row[5] = gpair(GA, 0, a.yc, k1) / GA[0] - gpair(GB, 0, a.yc, k1) / GB[0];  // builder.rs:676-684
    }
  }
  if (lane == 0) a.ok[rep] = a.raw_status ? status : (uint8_t)(status == 1);
}

// y_B - X_B beta_B on the unresampled group B (ols.rs:118-119; OaxacaResults::residuals).
__global__ __launch_bounds__(kBlock) void ob_residual_kernel(const double* cols, int64_t ld, uint32_t n, int p,
                                                             int ycol, const double* beta, double* out) {
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  double yh = beta[0];
  for (int c = 0; c < p; ++c) yh += cols[(size_t)c * ld + i] * beta[1 + c];
  out[i] = cols[(size_t)ycol * ld + i] - yh;
}

// ---------------------------------------------------------------------------------------------
// Unit Gram of the point estimate (run_single_pass on the unresampled groups, builder.rs:810-811):
// G_g = V_g^T V_g over every row once, V = sqrt(w) [1, x, y] (ols.rs:68-78). With unit counts the
// count-weighted GEMM of the bootstrap collapses to a SYRK, so it runs as one: D(I, J) =
// V[:, 16I..]^T V[:, 16J..] on v_mfma_f64_16x16x4f64 with A = the staged rows of column block I
// and B those of block J (the same staged image the Gram kernels read, ob_panel_kernel). Each
// block sums a fixed run of 64-row sub-tiles of one group -- a function of the group's size only,
// so multi-outcome panels and their one-outcome slices agree bitwise -- and writes one partial
// per pair; ob_unit_reduce_kernel adds the partials in block order. 168 MB of panel at 1M x 20
// WLS, read once: the launch needs thousands of blocks, not the boot's 32 chunks.
// ---------------------------------------------------------------------------------------------
constexpr int kUgMaxBlocks = 1024;  // per group
constexpr int kUgMaxPairs = 9;      // column-block pairs per wave: 4 waves x 9 >= 36 (k1 <= 128)

struct UnitGramArgs {
  const double* gp[2];  // Gram panels (ob_panel_kernel layout)
  uint32_t n[2];
  uint32_t subs[2];     // sub-tiles per block
  uint32_t blocks0;     // blocks of group 0 (group 1 follows)
  int k1, c_first, e, nbk;
  double* partial;      // [e][total blocks]
  uint32_t nblocks;
};

__global__ __launch_bounds__(kBlock) void ob_unit_gram_kernel(const UnitGramArgs a) {
  extern __shared__ __attribute__((aligned(16))) double xs[];  // [k1][kColStride]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const uint32_t g = blockIdx.x < a.blocks0 ? 0u : 1u;
  const uint32_t bi = g ? blockIdx.x - a.blocks0 : blockIdx.x;
  const uint32_t n = a.n[g], nsub = (n + 63) >> 6;
  const uint32_t s0 = bi * a.subs[g], s1 = min(nsub, s0 + a.subs[g]);
  const int ncl = a.k1 - a.c_first;
  const int npairs = a.nbk * (a.nbk + 1) / 2;
  // this wave's column-block pairs (I <= J), dealt round-robin over the 4 waves
  int pI[kUgMaxPairs], pJ[kUgMaxPairs];
#pragma unroll
  for (int q = 0; q < kUgMaxPairs; ++q) {
    int t = wave + 4 * q, I = 0;
    while (t >= a.nbk - I && I < a.nbk) {
      t -= a.nbk - I;
      ++I;
    }
    pI[q] = I;
    pJ[q] = I + t;
  }
  ob_d4 acc[kUgMaxPairs];
#pragma unroll
  for (int q = 0; q < kUgMaxPairs; ++q) acc[q] = (ob_d4){0.0, 0.0, 0.0, 0.0};
  const int kq = lane >> 4, li = lane & 15;
  for (uint32_t s = s0; s < s1; ++s) {
    const double2* src = reinterpret_cast<const double2*>(a.gp[g] + (size_t)s * ncl * kColStride);
    double2* dst = reinterpret_cast<double2*>(xs + a.c_first * kColStride);
    for (int i = tid; i < ncl * kColStride / 2; i += kBlock) dst[i] = src[i];
    if (a.c_first == 1)  // the intercept's ones (LDS-resident in the Gram kernels), zero past n
      for (int pos = tid; pos < kColStride; pos += kBlock) {
        const int q = pos & 63;
        xs[pos] = (s * 64u + (uint32_t)(((q & 15) << 2) | (q >> 4)) < n) ? 1.0 : 0.0;
      }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < kUgMaxPairs; ++q) {
      if (wave + 4 * q >= npairs) break;
      const int ca = pI[q] * 16 + li, cb = pJ[q] * 16 + li;
      const double* pa = xs + ca * kColStride + kq * 16 + (ca & 31);
      const double* pb = xs + cb * kColStride + kq * 16 + (cb & 31);
      const bool va = ca < a.k1, vb = cb < a.k1;
#pragma unroll
      for (int ks = 0; ks < 16; ++ks)
        acc[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(va ? pa[ks] : 0.0, vb ? pb[ks] : 0.0, acc[q], 0, 0, 0);
    }
    __syncthreads();
  }
  // D(I, J)[i][j] sits in lane (i % 4) * 16 + j, element i / 4: pair (16I + i, 16J + j), upper triangle
#pragma unroll
  for (int q = 0; q < kUgMaxPairs; ++q) {
    if (wave + 4 * q >= npairs) break;
    const int b = pJ[q] * 16 + li;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int c = pI[q] * 16 + kq + 4 * r;
      if (c <= b && b < a.k1) {
        const int e = c * a.k1 - c * (c - 1) / 2 + (b - c);
        a.partial[(size_t)e * a.nblocks + blockIdx.x] = acc[q][r];
      }
    }
  }
}

// gram[g][e] = the sum of group g's block partials of pair e, in block order then a fixed LDS tree
// (deterministic); pairs e_pad > e >= E are zero. One block per (group, pair).
__global__ __launch_bounds__(kBlock) void ob_unit_reduce_kernel(const double* partial, uint32_t nblocks,
                                                                uint32_t blocks0, int e, int e_pad, double* gram) {
  __shared__ double red[kBlock];
  const int tid = threadIdx.x;
  const int g = blockIdx.x >= (unsigned)e_pad ? 1 : 0;
  const int ei = (int)blockIdx.x - g * e_pad;
  double s = 0.0;
  if (ei < e) {
    const uint32_t b0 = g ? blocks0 : 0u, b1 = g ? nblocks : blocks0;
    for (uint32_t b = b0 + tid; b < b1; b += kBlock) s += partial[(size_t)ei * nblocks + b];
  }
  red[tid] = s;
  __syncthreads();
  for (int h = kBlock / 2; h > 0; h >>= 1) {
    if (tid < h) red[tid] += red[tid + h];
    __syncthreads();
  }
  if (tid == 0) gram[g * e_pad + ei] = red[0];
}

// ---------------------------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------------------------
// Knuth-Yao tables of B(2^j, 1/2) for OBRS-2's level-1 split (ob_spec.h): W_k = C(2^j, k) exactly
// (multi-limb integers, C(n, k + 1) = C(n, k) (n - k) / (k + 1)); column i = 1 .. n lists the k
// with bit n - i of W_k set. Built once per process, uploaded once per device (~22 MB).
struct KyHost {
  std::vector<uint32_t> off;   // all tables' column offsets, table t at off_base[t]
  std::vector<uint16_t> list;  // all tables' lists, table t at list_base[t]
  std::vector<uint32_t> hot;   // [tables][OB_KY_HOT + 1] hot offsets, then the hot entries as uint16 pairs
  uint32_t off_base[OB_KY_TABLES] = {}, list_base[OB_KY_TABLES] = {}, i0[OB_KY_TABLES] = {};
  uint32_t hot_entries = 0;
};

const KyHost& ky_host() {
  static const KyHost h = [] {
    KyHost t;
    std::vector<uint16_t> hot_list;
    std::vector<uint32_t> hot_off;
    for (int j = OB_KY_MIN_LOG; j <= OB_KY_MAX_LOG; ++j) {
      const uint32_t n = 1u << j, L = n / 64 + 1;
      std::vector<uint64_t> w((size_t)(n + 1) * L, 0);
      w[0] = 1;
      for (uint32_t k = 0; k < n; ++k) {
        const uint64_t* a = &w[(size_t)k * L];
        uint64_t* b = &w[(size_t)(k + 1) * L];
        unsigned __int128 carry = 0;
        for (uint32_t i = 0; i < L; ++i) {
          const unsigned __int128 v = (unsigned __int128)a[i] * (n - k) + carry;
          b[i] = (uint64_t)v;
          carry = v >> 64;
        }
        unsigned __int128 rem = 0;
        for (uint32_t i = L; i-- > 0;) {
          const unsigned __int128 v = (rem << 64) | b[i];
          b[i] = (uint64_t)(v / (k + 1));
          rem = v % (k + 1);
        }
      }
      const int x = j - OB_KY_MIN_LOG;
      t.off_base[x] = (uint32_t)t.off.size();
      t.list_base[x] = (uint32_t)t.list.size();
      std::vector<uint32_t> off(n + 2, 0);
      std::vector<uint16_t> list;
      for (uint32_t i = 1; i <= n; ++i) {
        off[i] = (uint32_t)list.size();
        const uint32_t bit = n - i;
        for (uint32_t k = 0; k <= n; ++k)
          if ((w[(size_t)k * L + bit / 64] >> (bit % 64)) & 1u) list.push_back((uint16_t)k);
        if (!t.i0[x] && list.size() > off[i]) t.i0[x] = i;
      }
      off[n + 1] = (uint32_t)list.size();
      for (uint32_t c = 0; c <= OB_KY_HOT; ++c) hot_off.push_back((uint32_t)hot_list.size() + off[t.i0[x] + c] - off[t.i0[x]]);
      hot_list.insert(hot_list.end(), list.begin() + off[t.i0[x]], list.begin() + off[t.i0[x] + OB_KY_HOT]);
      t.off.insert(t.off.end(), off.begin(), off.end());
      t.list.insert(t.list.end(), list.begin(), list.end());
    }
    t.hot_entries = (uint32_t)hot_list.size();
    if (hot_list.size() % 2) hot_list.push_back(0);
    t.hot = hot_off;
    for (size_t i = 0; i < hot_list.size(); i += 2) t.hot.push_back((uint32_t)hot_list[i] | ((uint32_t)hot_list[i + 1] << 16));
    return t;
  }();
  return h;
}

int ky_device(int device, ob_ky_tables* out) {
  static std::mutex mu;
  static std::map<int, ob_ky_tables> cache;
  std::lock_guard<std::mutex> lk(mu);
  auto it = cache.find(device);
  if (it == cache.end()) {
    const KyHost& h = ky_host();
    if (h.hot_entries > OB_KY_HOT_CAP) return ob::fail(OB_E_INVALID, "internal: Knuth-Yao hot columns exceed the LDS stage");
    ob_ky_tables t{};
    uint32_t *off = nullptr, *hot = nullptr;
    uint16_t* list = nullptr;
    HIP_OK(hipMalloc(&off, sizeof(uint32_t) * h.off.size()));
    HIP_OK(hipMalloc(&list, sizeof(uint16_t) * h.list.size()));
    HIP_OK(hipMalloc(&hot, sizeof(uint32_t) * h.hot.size()));
    HIP_OK(hipMemcpy(off, h.off.data(), sizeof(uint32_t) * h.off.size(), hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(list, h.list.data(), sizeof(uint16_t) * h.list.size(), hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(hot, h.hot.data(), sizeof(uint32_t) * h.hot.size(), hipMemcpyHostToDevice));
    t.off = off;
    t.list = list;
    t.hot = hot;
    for (int x = 0; x < OB_KY_TABLES; ++x) {
      t.off_base[x] = h.off_base[x];
      t.list_base[x] = h.list_base[x];
      t.i0[x] = h.i0[x];
    }
    t.hot_entries = h.hot_entries;
    it = cache.emplace(device, t).first;
  }
  *out = it->second;
  return OB_OK;
}

struct Plan {
  uint32_t nb_rep, rep_pad, n_cg;
  int cb;
  std::vector<uint32_t> chunks;  // (g, t0, t1)
  int n_chunks() const { return (int)(chunks.size() / 3); }
};

// Timing ablations (gram_diag, tools/gram_ablate.py): tuning builds only, 0 otherwise (ob_options.hpp).
int diag_mode() { return ob::opt_int(ob::Opt::GramDiag, 0); }

// Two staged sub-tiles (the next one's DMA under this one's MFMAs) while they fit in the 160 KB of
// LDS (k1 <= 101); wider panels (p up to 120) stage one at a time.
constexpr size_t kLdsMax = 160 * 1024;
bool gram_dbl(const ob_panel* p) { return (size_t)kXtOff + 2 * (size_t)p->k1 * kColStride * 8 <= kLdsMax; }
size_t gram_lds_bytes(const ob_panel* p) {
  return (size_t)kXtOff + (gram_dbl(p) ? 2 : 1) * (size_t)p->k1 * kColStride * 8;
}

// The chunking is a function of the panel only (never of the replicate count or the launch),
// so a replicate's Gram -- summed over chunks in a fixed order -- is bitwise the same however
// the replicates are segmented or sharded. Each group splits into balanced chunks; about
// kTargetChunks in all, so a 16384-replicate segment (256 batches of 64) is a whole number of
// rounds over 256 CUs. 32 rather than 64 (round 3, profiles/r03_ab_chunks.txt): half the chunk
// partials to write and reduce, Gram 12.5 -> 12.3 ms and reduce 0.27 -> 0.14 ms at configs[1].
#ifndef OB_TARGET_CHUNKS
#define OB_TARGET_CHUNKS 32
#endif
constexpr uint32_t kTargetChunks = OB_TARGET_CHUNKS;

Plan make_plan(const ob_panel* p, uint64_t n_reps, bool unit) {
  Plan pl;
  pl.nb_rep = (uint32_t)((n_reps + 63) / 64);
  pl.rep_pad = pl.nb_rep * 64;
  if (unit) {  // the unit (point-estimate) variant stays at CB <= 2
    pl.cb = p->ncb > 4 ? 2 : 1;
  } else {      // fewest column groups (each re-reads the rows), then the smallest CB that covers
    const int groups = (p->ncb + 19) / 20;
    pl.cb = std::max(1, (p->ncb + 4 * groups - 1) / (4 * groups));
  }
  pl.n_cg = (uint32_t)((p->ncb + 4 * pl.cb - 1) / (4 * pl.cb));
  const uint32_t tT = p->ntiles[0] + p->ntiles[1];
  for (uint32_t g = 0; g < 2; ++g) {
    const uint32_t tg = p->ntiles[g];
    if (tg == 0) continue;
    const uint32_t want = (uint32_t)std::max<uint64_t>(1, ((uint64_t)kTargetChunks * tg + tT / 2) / std::max(tT, 1u));
    const uint32_t nc = std::min(tg, std::max(want, (tg + 4095) / 4096));
    for (uint32_t c = 0; c < nc; ++c) {
      pl.chunks.push_back(g);
      pl.chunks.push_back((uint32_t)((uint64_t)tg * c / nc));
      pl.chunks.push_back((uint32_t)((uint64_t)tg * (c + 1) / nc));
    }
  }
  return pl;
}

size_t solve_lds_bytes_t(const ob_panel* p, bool dual) {
  const int k = p->k, kp = k + 1;
  return sizeof(double) * ((size_t)kp * kp + (dual ? (size_t)k * k : 0) + 7 * (size_t)kp +
                           3 * (size_t)std::max(p->norm.n_norm, 1));
}
// Two waves per replicate (ob_solve_kernel<true>) while both groups' matrices fit in 64 KB of LDS.
bool solve_dual(const ob_panel* p) { return solve_lds_bytes_t(p, true) <= 64 * 1024; }
size_t solve_lds_bytes(const ob_panel* p) { return solve_lds_bytes_t(p, solve_dual(p)); }

hipError_t launch_solve(const ob_panel* p, const SolveArgs& sa, uint32_t blocks, hipStream_t s) {
  const bool dual = solve_dual(p);
  const size_t lds = solve_lds_bytes(p);
  const void* fn = dual ? (const void*)ob_solve_kernel<true> : (const void*)ob_solve_kernel<false>;
  hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return e;
  if (dual) hipLaunchKernelGGL(ob_solve_kernel<true>, dim3(blocks), dim3(128), lds, s, sa);
  else hipLaunchKernelGGL(ob_solve_kernel<false>, dim3(blocks), dim3(64), lds, s, sa);
  return hipGetLastError();
}

template <int CB, bool U>
hipError_t launch_gram_t(const GramArgs& ga, uint32_t blocks, size_t lds, hipStream_t s) {
  hipError_t e = hipFuncSetAttribute((const void*)ob_gram_kernel<CB, U>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                     (int)lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((ob_gram_kernel<CB, U>), dim3(blocks), dim3(kBlock), lds, s, ga);
  return hipGetLastError();
}

template <bool U>
hipError_t launch_gram_u(const ob_panel* p, int cb, const GramArgs& ga, uint32_t blocks, hipStream_t s) {
  const size_t lds = gram_lds_bytes(p);
  switch (cb) {
    case 5:
      if constexpr (!U) return launch_gram_t<5, U>(ga, blocks, lds, s);
      [[fallthrough]];
    case 4:
      if constexpr (!U) return launch_gram_t<4, U>(ga, blocks, lds, s);
      [[fallthrough]];
    case 2: return launch_gram_t<2, U>(ga, blocks, lds, s);
    default: return launch_gram_t<1, U>(ga, blocks, lds, s);
  }
}

hipError_t launch_gram(const ob_panel* p, int cb, bool unit, const GramArgs& ga, uint32_t blocks, hipStream_t s) {
  return unit ? launch_gram_u<true>(p, cb, ga, blocks, s) : launch_gram_u<false>(p, cb, ga, blocks, s);
}

// Gram panel (the staged-image layout of stage_dma): [sub-tile][column c_first..k1-1][96].
// Columns: weighted sqrt(w) * [1, x_1..x_p, y_1..] (ols.rs:68-78), else [x, y] (the intercept's
// ones are LDS-resident). cols: [x_1..x_p, y_1..y_n_y, (w)] x ld, zero rows past n.
__global__ __launch_bounds__(kBlock) void ob_panel_kernel(const double* cols, int64_t ld, int nxy, int weighted,
                                                          double* gp) {
  const int ncl = weighted ? nxy + 1 : nxy, c_first = weighted ? 0 : 1;
  const size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x;
  const size_t per_sub = (size_t)ncl * kColStride;
  if (i >= (size_t)(ld >> 6) * per_sub) return;
  const size_t sub = i / per_sub;
  const int cc = (int)((i % per_sub) / kColStride), pos = (int)(i % kColStride);
  const int c = cc + c_first;
  const int q = (pos - (c & 31)) & 63;
  const size_t row = sub * 64 + (size_t)(((q & 15) << 2) | (q >> 4));
  double v;
  if (weighted) {
    const double sw = sqrt(cols[(size_t)nxy * ld + row]);
    v = c == 0 ? sw : sw * cols[(size_t)(c - 1) * ld + row];
  } else {
    v = cols[(size_t)(c - 1) * ld + row];
  }
  gp[i] = v;
}

template <typename T>
int ensure_buf(T** ptr, size_t& cap_elems, size_t need_elems) {
  if (*ptr && cap_elems >= need_elems) return OB_OK;
  if (*ptr) (void)hipFree(*ptr);
  *ptr = nullptr;
  cap_elems = 0;
  HIP_OK(hipMalloc((void**)ptr, std::max<size_t>(need_elems, 1) * sizeof(T)));
  cap_elems = need_elems;
  return OB_OK;
}

SolveArgs solve_args(const ob_panel* p, int ref_mode) {
  SolveArgs sa{};
  sa.e_pad = p->e_pad;
  sa.k1 = p->k1;
  sa.k = p->k;
  sa.pool_pos = 1 + p->n_num;
  sa.ref_mode = ref_mode;
  sa.weighted = p->weighted;
  sa.yc = p->p + 1;
  sa.rows_a = (double)p->n[0];
  sa.rows_b = (double)p->n[1];
  sa.n_norm = p->norm.n_norm;
  sa.n_base = p->norm.n_base;
  sa.norm = p->d_norm;
  const int nn = p->norm.n_norm;
  sa.off_idx = nn + 1;
  sa.off_m = sa.off_idx + (int)p->norm.idx.size();
  sa.off_pstart = sa.off_m + nn;
  sa.off_pidx = sa.off_pstart + nn + 1;
  sa.off_has = sa.off_pidx + (int)p->norm.pidx.size();
  sa.row_len = p->row_len;
  return sa;
}

GramArgs gram_args(const ob_panel* p, const Plan& pl) {
  GramArgs ga{};
  ga.gcols0 = p->d_gpanel[0];
  ga.gcols1 = p->d_gpanel[1];
  ga.c_first = p->weighted ? 0 : 1;
  ga.ld0 = p->ld[0];
  ga.ld1 = p->ld[1];
  ga.n0 = p->n[0];
  ga.n1 = p->n[1];
  ga.k1 = p->k1;
  ga.e = p->e;
  ga.ncb = p->ncb;
  ga.n_cg = (int)pl.n_cg;
  ga.nb_rep = pl.nb_rep;
  ga.tiles0 = p->ntiles[0];
  ga.rep_pad = pl.rep_pad;
  ga.e_pad = p->e_pad;
  ga.flags = p->d_flags;
  ga.dbl = gram_dbl(p) ? 1 : 0;
  return ga;
}

int ensure_heck(ob_panel* p, const Plan& pl) {
  const int vals = std::max(ob::heck_probit_len(p->ks), ob::heck_sums_len(p->k));
  OB_TRY(ensure_buf(&p->d_hgamma, p->cap_hgamma, (size_t)2 * pl.rep_pad * p->ks));
  OB_TRY(ensure_buf(&p->d_hflags, p->cap_hflags, (size_t)2 * pl.rep_pad));
  OB_TRY(ensure_buf(&p->d_hpartial, p->cap_hpartial, (size_t)pl.n_chunks() * pl.rep_pad * vals));
  if (!p->d_hactive) HIP_OK(hipMalloc(&p->d_hactive, sizeof(uint32_t)));
  return OB_OK;
}

ob_heck_seg heck_seg(const ob_panel* p, const Plan& pl, const uint32_t* d_chunks, const double* d_gram,
                     int ref_mode) {
  ob_heck_seg h{};
  for (int g = 0; g < 2; ++g) {
    h.cols[g] = p->d_cols[g];
    h.ld[g] = p->ld[g];
    h.n[g] = p->n[g];
  }
  h.tiles0 = p->ntiles[0];
  h.p = p->p;
  h.ks = p->ks;
  h.weighted = p->h_weighted;
  h.nb_rep = pl.nb_rep;
  h.chunks = d_chunks;
  h.n_chunks = pl.n_chunks();
  h.rep_pad = pl.rep_pad;
  h.gram = d_gram;
  h.e_pad = p->e_pad;
  h.k1 = p->k1;
  h.gamma = p->d_hgamma;
  h.hflags = p->d_hflags;
  h.partial = p->d_hpartial;
  h.active = p->d_hactive;
  h.ref_mode = ref_mode;
  h.row_len = p->row_len;
  h.max_iter = 100;  // heckman.rs:46
  return h;
}

}  // namespace

namespace ob {

int engine_point_estimate(ob_panel* p, int ref_mode, double* row, double* resid_b) {
  ob_ctx* ctx = p->ctx;
  HIP_OK(hipSetDevice(ctx->device));
  hipStream_t s = ctx->stream;
  Plan pl = make_plan(p, 1, true);
  // the unit Gram's blocks: a run of sub-tiles per block, at most kUgMaxBlocks per group
  UnitGramArgs ua{};
  uint32_t nblk[2];
  for (int g = 0; g < 2; ++g) {
    const uint32_t nsub = (p->n[g] + 63) / 64;
    ua.subs[g] = std::max<uint32_t>(2u, (nsub + kUgMaxBlocks - 1) / kUgMaxBlocks);
    nblk[g] = (nsub + ua.subs[g] - 1) / ua.subs[g];
    ua.gp[g] = p->d_gpanel[g];
    ua.n[g] = p->n[g];
  }
  ua.blocks0 = nblk[0];
  ua.nblocks = nblk[0] + nblk[1];
  ua.k1 = p->k1;
  ua.c_first = p->weighted ? 0 : 1;
  ua.e = p->e;
  ua.nbk = (p->k1 + 15) / 16;
  if (ua.nbk * (ua.nbk + 1) / 2 > 4 * kUgMaxPairs) return ob::fail(OB_E_UNSUPPORTED, "point estimate: k1 > 128");
  // persistent per-panel scratch (no hipMalloc / hipFree per call): partials, then the Gram
  // [rep_pad][2][e_pad] (rep 0 used), the rows, the first outcome's reduced Grams, beta, residuals
  const size_t o_part = 0, n_part = (size_t)p->e * std::max(ua.nblocks, 1u);
  const size_t o_gram = o_part + n_part, n_gram = (size_t)2 * pl.rep_pad * p->e_pad;
  const size_t o_row = o_gram + n_gram, n_row = (size_t)p->row_len * p->n_y;
  const size_t o_gout = o_row + n_row, n_gout = (size_t)2 * p->e_pad;
  const size_t o_beta = o_gout + n_gout, n_beta = (size_t)p->k * p->n_y;
  const size_t o_res = o_beta + n_beta, n_res = std::max<uint32_t>(p->n[1], 1);
  OB_TRY(ensure_buf(&p->d_pe, p->cap_pe, o_res + (resid_b ? n_res : 0)));
  OB_TRY(ensure_buf(&p->d_pe_ok, p->cap_pe_ok, (size_t)std::max(p->n_y, 1)));
  double* d_gram = p->d_pe + o_gram;
  double* d_row = p->d_pe + o_row;
  double* d_gout = p->d_pe + o_gout;
  double* d_beta = p->d_pe + o_beta;
  uint8_t* d_ok = p->d_pe_ok;
  ua.partial = p->d_pe + o_part;
  const size_t lds = sizeof(double) * (size_t)p->k1 * kColStride;
  HIP_OK(hipFuncSetAttribute((const void*)ob_unit_gram_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  if (ua.nblocks) {
    hipLaunchKernelGGL(ob_unit_gram_kernel, dim3(ua.nblocks), dim3(kBlock), lds, s, ua);
    HIP_OK(hipGetLastError());
  }
  hipLaunchKernelGGL(ob_unit_reduce_kernel, dim3(2 * p->e_pad), dim3(kBlock), 0, s, (const double*)ua.partial,
                     ua.nblocks, ua.blocks0, p->e, p->e_pad, d_gram);
  HIP_OK(hipGetLastError());
  if (p->heckman) {  // estimation.rs:114-172 on the whole groups (every row once)
    if (!p->chunks_ready) {  // the probit/IMR passes walk the panel's chunk table
      p->chunks = pl.chunks;
      OB_TRY(ensure_buf(&p->d_chunks, p->cap_chunks, p->chunks.size()));
      HIP_OK(hipMemcpyAsync(p->d_chunks, p->chunks.data(), sizeof(uint32_t) * p->chunks.size(), hipMemcpyHostToDevice, s));
      p->chunks_ready = true;
    }
    OB_TRY(ensure_heck(p, pl));
    ob_heck_seg hs = heck_seg(p, pl, p->d_chunks, d_gram, ref_mode);
    hs.counts = nullptr;
    hs.n_reps = 1;
    hs.rows = d_row;
    hs.ok = d_ok;
    hs.raw_status = 1;
    int it = 0;
    OB_TRY(ob::heckman_segment(hs, s, &it));
    uint8_t okh = 0;
    HIP_OK(hipMemcpyAsync(row, d_row, sizeof(double) * p->row_len, hipMemcpyDeviceToHost, s));
    HIP_OK(hipMemcpyAsync(&okh, d_ok, 1, hipMemcpyDeviceToHost, s));
    HIP_OK(hipStreamSynchronize(s));
    p->timing.probit_iterations = it;
    switch (okh) {
      case OB_HS_OK: return OB_OK;  // residuals: zeros over B's selected rows (estimation.rs:152-153), the caller's
      case OB_HS_NO_OUTCOMES:
        return ob::fail(OB_E_GROUP, "%sNo observed outcomes in group", error_prefix(OB_E_GROUP));
      case OB_HS_PROBIT:
        return ob::fail(OB_E_LINALG, "%sFailed to solve Hessian system in Probit", error_prefix(OB_E_LINALG));
      case OB_HS_INSUFFICIENT:
        return ob::fail(OB_E_INSUFFICIENT, "%sInsufficient data for OLS calculation: n_obs must be strictly greater than k",
                        error_prefix(OB_E_INSUFFICIENT));
      case OB_HS_ZERO_WEIGHT:
        return ob::fail(OB_E_GROUP, "%sNo data in groups for weighted coefficients.", error_prefix(OB_E_GROUP));
      default:
        return ob::fail(OB_E_LINALG,
                        "%sFailed to perform Cholesky decomposition. Matrix may be singular or not positive "
                        "definite due to multicollinearity.",
                        error_prefix(OB_E_LINALG));
    }
  }
  for (int t = 0; t < p->n_y; ++t) {
    SolveArgs sa = solve_args(p, ref_mode);
    sa.yc = p->p + 1 + t;
    sa.gram = d_gram;
    sa.rows = d_row + (size_t)t * p->row_len;
    sa.ok = d_ok + t;
    sa.n_reps = 1;
    sa.gram_out = t == 0 ? d_gout : nullptr;
    sa.raw_status = 1;
    sa.raw_beta_b = d_beta + (size_t)t * p->k;
    HIP_OK(launch_solve(p, sa, 1, s));
  }
  // the residuals (only when asked for) are computed before the one host synchronization
  if (resid_b && p->n[1] > 0) {
    double* d_res = p->d_pe + o_res;
    for (int t = 0; t < p->n_y; ++t) {  // the kernel-stream order serializes d_res reuse
      hipLaunchKernelGGL(ob_residual_kernel, dim3((p->n[1] + kBlock - 1) / kBlock), dim3(kBlock), 0, s,
                         (const double*)p->d_cols[1], p->ld[1], p->n[1], p->p, p->p + t,
                         (const double*)(d_beta + (size_t)t * p->k), d_res);
      HIP_OK(hipGetLastError());
      HIP_OK(hipMemcpyAsync(resid_b + (size_t)t * p->n[1], d_res, sizeof(double) * p->n[1], hipMemcpyDeviceToHost, s));
    }
  }
  uint8_t okh = 0;
  HIP_OK(hipMemcpyAsync(row, d_row, sizeof(double) * p->row_len * p->n_y, hipMemcpyDeviceToHost, s));
  HIP_OK(hipMemcpyAsync(&okh, d_ok, 1, hipMemcpyDeviceToHost, s));
  HIP_OK(hipStreamSynchronize(s));
  if (okh == 2) return ob::fail(OB_E_GROUP, "%sNo data in groups for weighted coefficients.", error_prefix(OB_E_GROUP));
  if (okh != 1)
    return ob::fail(OB_E_LINALG,
                    "%sFailed to perform Cholesky decomposition. Matrix may be singular or not positive "
                    "definite due to multicollinearity.",
                    error_prefix(OB_E_LINALG));
  return OB_OK;
}

// OBRS-3 resample counts for replicates [first_rep, first_rep + n_reps) without the Gram: level-1
// tile counts into d_m1 ([replicate][tile]) and the level-2 count images into d_counts (the
// ob_engine.hpp layout, replicate batches of 64). Used by the Machado-Mata driver (ob_mm.hip).
int engine_counts(ob_panel* p, uint64_t seed, uint64_t first_rep, uint32_t n_reps, hipStream_t s,
                  uint32_t* nb_rep, uint32_t* rep_pad) {
  HIP_OK(hipSetDevice(p->ctx->device));
  if (n_reps == 0) return OB_OK;
  if (first_rep + n_reps > 0xFFFFFFFFull)
    return ob::fail(OB_E_INVALID, "replicate ids must stay below 2^32 - 1 (OBRS-3 / MM-1 counter word)");
  const uint32_t tiles = p->ntiles[0] + p->ntiles[1];
  Plan pl = make_plan(p, n_reps, false);
  OB_TRY(ensure_buf(&p->d_m1, p->cap_m1, (size_t)tiles * pl.rep_pad));
  OB_TRY(ensure_buf(&p->d_counts, p->cap_counts, (size_t)tiles * pl.nb_rep * 4 * kCimgWords));
  // Overflow goes to its own word, d_flags[2] (word 0 belongs to boot calls that may still be
  // pending). The caller clears it once before its first call and reads it after its last: the
  // count kernel only ever ORs into it, so an overflow in any segment survives to the check.
  const uint32_t key0 = (uint32_t)seed, key1 = (uint32_t)(seed >> 32);
  const size_t lds_l1 = sizeof(uint32_t) * std::max(l1_lds_words(p->ntiles[0]), l1_lds_words(p->ntiles[1]));
  HIP_OK(hipFuncSetAttribute((const void*)ob_level1_kernel<0>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_l1));
  ob_ky_tables ky{};
  OB_TRY(ky_device(p->ctx->device, &ky));
  hipLaunchKernelGGL(ob_level1_kernel<0>, dim3(n_reps, 2), dim3(kBlock), lds_l1, s, p->n[0], p->n[1], p->ntiles[0],
                     (uint32_t)first_rep, tiles, key0, key1, p->d_m1, ky);
  HIP_OK(hipGetLastError());
  GramArgs ga = gram_args(p, pl);
  ga.flags = p->d_flags + 2;
  ga.m1 = p->d_m1;
  ga.n_reps = n_reps;
  ga.first_rep = (uint32_t)first_rep;
  ga.key0 = key0;
  ga.key1 = key1;
  ga.counts = p->d_counts;
  ga.tiles_total = tiles;
  hipLaunchKernelGGL(ob_count_kernel<false>, dim3((tiles + kCntTilesPerBlock - 1) / kCntTilesPerBlock, pl.nb_rep),
                     dim3(kBlock), 0, s, ga);
  HIP_OK(hipGetLastError());
  if (opt_int(Opt::DebugCountOverflow, 0)) HIP_OK(hipMemsetAsync(p->d_flags + 2, 0xFF, sizeof(uint32_t), s));
  *nb_rep = pl.nb_rep;
  *rep_pad = pl.rep_pad;
  return OB_OK;
}

int engine_order(ob_panel* p, hipStream_t s) {
  if (p->order_stream && p->order_stream != s) HIP_OK(hipStreamWaitEvent(s, p->order_ev, 0));
  return OB_OK;
}

int engine_mark(ob_panel* p, hipStream_t s, bool scratch) {
  if (!p->order_ev) HIP_OK(hipEventCreateWithFlags(&p->order_ev, hipEventDisableTiming));
  HIP_OK(hipEventRecord(p->order_ev, s));
  p->order_stream = s;
  if (scratch) {
    if (!p->scratch_ev) HIP_OK(hipEventCreateWithFlags(&p->scratch_ev, hipEventDisableTiming));
    HIP_OK(hipEventRecord(p->scratch_ev, s));
    if (p->scratch_ev2) HIP_OK(hipEventRecord(p->scratch_ev2, s));
    p->scratch_recorded = true;
  }
  return OB_OK;
}

int engine_boot(ob_panel* p, uint64_t seed, uint64_t first_rep, uint64_t n_reps, int ref_mode, double* d_rows,
                uint8_t* d_ok, hipStream_t stream) {
  ob_ctx* ctx = p->ctx;
  HIP_OK(hipSetDevice(ctx->device));
  if (n_reps == 0) return OB_OK;
  if (first_rep + n_reps > 0x100000000ull)
    return ob::fail(OB_E_INVALID, "replicate ids must stay below 2^32 (OBRS-3 counter word)");
  hipStream_t s = stream ? stream : ctx->stream;
  OB_TRY(engine_order(p, s));  // a previous call on another stream (the digit images, scratch buffers)
  const uint32_t tiles = p->ntiles[0] + p->ntiles[1];
  // segment: at most kSegReps replicates, and a count-image buffer within kCountBudget
  const uint64_t batch_bytes = (uint64_t)std::max(tiles, 1u) * 4 * kCimgWords * sizeof(uint32_t);
  const uint64_t seg_cap = std::max<uint64_t>(64, (kCountBudget / batch_bytes) * 64);
  const uint64_t seg = std::min<uint64_t>(n_reps, std::min<uint64_t>(kSegReps, seg_cap));
  Plan pl = make_plan(p, seg, false);
  const uint64_t tail = n_reps % seg;
  Plan pl_tail = tail ? make_plan(p, tail, false) : pl;  // same chunks, fewer replicate batches
  const int nch = pl.n_chunks();
  const size_t need_partial = std::max((size_t)nch * pl.rep_pad, (size_t)pl_tail.n_chunks() * pl_tail.rep_pad);
  OB_TRY(ensure_buf(&p->d_m1, p->cap_m1, (size_t)tiles * pl.rep_pad));
  OB_TRY(ensure_buf(&p->d_counts, p->cap_counts, (size_t)tiles * pl.nb_rep * 4 * kCimgWords));
  OB_TRY(ensure_buf(&p->d_partial, p->cap_partial, need_partial * p->e_pad));
  OB_TRY(ensure_buf(&p->d_gram, p->cap_gram, (size_t)2 * pl.rep_pad * p->e_pad));
  bool s_work = false;  // this call put work on s that its Gram reads (tail_stream: g_stream waits for it)
  if (!p->chunks_ready) {  // the chunk table depends on the panel only: uploaded once, never rewritten
    s_work = true;
    p->chunks = pl.chunks;
    OB_TRY(ensure_buf(&p->d_chunks, p->cap_chunks, p->chunks.size()));
    HIP_OK(hipMemcpyAsync(p->d_chunks, p->chunks.data(), sizeof(uint32_t) * p->chunks.size(), hipMemcpyHostToDevice, s));
    p->chunks_ready = true;
  }
  if (pl.chunks != p->chunks || pl_tail.chunks != p->chunks)
    return ob::fail(OB_E_INVALID, "internal: the chunk table changed with the replicate count");
  if (p->heckman) OB_TRY(ensure_heck(p, pl));
  // Gram path: the exact integer-sliced i8 GEMM (ob_gram_i8.hip) unless forced to f64 MFMA
  // (option gram_path = 1, ob_set_option) or the digit images do not fit. Heckman's kernels read
  // either image layout.
  int force = p->gram_force;
  if (!force) force = ob::opt_int(ob::Opt::GramPath, 0);
  bool use_i8 = force != 1;
  if (!p->timing_pending) {  // the first call since the last collect: its timings start from zero
    std::memset(&p->timing, 0, sizeof(p->timing));
    p->pending_segments = 0;
    p->pending_gathers = 0;
  }
  if (use_i8) {
    if (p->oz_state == 0) s_work = true;
    OB_TRY(ob::oz_prepare(p, s));
    use_i8 = p->oz_state == 1;
    if (!use_i8 && force == 2) return ob::fail(OB_E_UNSUPPORTED, "the i8 Gram's digit images do not fit in HBM");
  }
  // the overflow flag (d_flags[0]) is sticky over the calls since the last collect, which reads and
  // clears it: no per-call reset, so an enqueued call never erases a pending one's flag

  const size_t lds_l1 = sizeof(uint32_t) * std::max(l1_lds_words(p->ntiles[0]), l1_lds_words(p->ntiles[1]));
  ob_ky_tables ky{};
  OB_TRY(ky_device(ctx->device, &ky));
  using L1Kernel = void (*)(uint32_t, uint32_t, uint32_t, uint32_t, uint32_t, uint32_t, uint32_t, uint32_t*,
                            const ob_ky_tables);
#if OB_TUNING  // timing ablations of level 1 (l1_diag, tools/l1_ablate.sh)
  const int l1_diag = ob::opt_int(ob::Opt::L1Diag, 0) & 63;
  const L1Kernel l1k = l1_diag == 0    ? ob_level1_kernel<0>
                       : l1_diag == 1  ? ob_level1_kernel<1>
                       : l1_diag == 2  ? ob_level1_kernel<2>
                       : l1_diag == 32 ? ob_level1_kernel<32>
                       : l1_diag == 3  ? ob_level1_kernel<3>
                       : l1_diag == 11 ? ob_level1_kernel<11>
                       : l1_diag == 16 ? ob_level1_kernel<16>
                       : l1_diag == 20 ? ob_level1_kernel<20>
                                       : ob_level1_kernel<0>;
#else
  const L1Kernel l1k = ob_level1_kernel<0>;
#endif
  HIP_OK(hipFuncSetAttribute((const void*)l1k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_l1));
  p->timing.chunks = nch;
  p->timing.blocks = use_i8 ? (int32_t)((uint32_t)nch * ((pl.nb_rep + 3) / 4) * (uint32_t)p->oz_n_ct)
                            : (int32_t)(pl.nb_rep * pl.n_cg * (uint32_t)nch);
  p->timing.gram_path = use_i8 ? 2 : 1;
  const uint32_t key0 = (uint32_t)seed, key1 = (uint32_t)(seed >> 32);
  const size_t nseg = (size_t)((n_reps + seg - 1) / seg);
  while (p->seg_events.size() < kSegEvents * (nseg + (size_t)p->pending_segments)) {
    hipEvent_t e;
    HIP_OK(hipEventCreate(&e));
    p->seg_events.push_back(e);
  }
  // the resample stream (ob_engine.hpp): level 1 and counts wait only for the previous call's last
  // read of the count images, not for its reduce / solve / gather
  const bool overlap = OB_BOOT_OVERLAP && !p->heckman;
  if (overlap) {
    if (!p->rs_stream) HIP_OK(hipStreamCreateWithFlags(&p->rs_stream, hipStreamNonBlocking));
    if (!p->rs_ev) HIP_OK(hipEventCreateWithFlags(&p->rs_ev, hipEventDisableTiming));
    if (!p->scratch_ev) HIP_OK(hipEventCreateWithFlags(&p->scratch_ev, hipEventDisableTiming));
    if (!p->scratch_recorded) {  // no engine call on this panel yet: start where s is
      HIP_OK(hipEventRecord(p->scratch_ev, s));
      p->scratch_recorded = true;
    }
  }
  const hipStream_t sr = overlap ? p->rs_stream : s;
  // two m1 / count-image buffers (ob_engine.hpp): a segment's resample then waits only for the Gram
  // two segments back and runs under the previous one's. By default only under the 8-wave i8 Gram:
  // its partial last rounds leave CUs to the resample (configs[2]'s 1,250 share: 536-545k -> 561-562k
  // replicates/s), while a wide-tile block needs a whole CU's LDS, so resample blocks there delay
  // the Gram more than they hide (5,000 / 2,500 / 10k replicates: -9 / -11 / -4.5 %;
  // profiles/r06_ab_rs_double.txt)
  const int rs_pieces = ob::opt_int(ob::Opt::RsPieces, 1);
  if (overlap && rs_pieces > 1) {
    if (!p->cnt_stream) HIP_OK(hipStreamCreateWithFlags(&p->cnt_stream, hipStreamNonBlocking));
    for (hipEvent_t& e : p->cnt_ev)
      if (!e) HIP_OK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  }
  const int rs_opt = ob::opt_int(ob::Opt::RsDouble, -1);
  const bool dbl = overlap && (rs_opt == 1 || (rs_opt < 0 && use_i8 && !ob::oz_wide(p, nch, pl.nb_rep)));
  if (dbl) {
    OB_TRY(ensure_buf(&p->d_m1b, p->cap_m1b, (size_t)tiles * pl.rep_pad));
    OB_TRY(ensure_buf(&p->d_countsb, p->cap_countsb, (size_t)tiles * pl.nb_rep * 4 * kCimgWords));
    if (!p->scratch_ev2) {
      HIP_OK(hipEventCreateWithFlags(&p->scratch_ev2, hipEventDisableTiming));
      HIP_OK(hipEventRecord(p->scratch_ev2, s));
    }
  }
  const bool tov = overlap && ob::opt_int(ob::Opt::TailStream, 0) == 1;
  if (tov) {
    if (!p->g_stream) HIP_OK(hipStreamCreateWithFlags(&p->g_stream, hipStreamNonBlocking));
    if (!p->t_stream) HIP_OK(hipStreamCreateWithFlags(&p->t_stream, hipStreamNonBlocking));
    for (hipEvent_t* e : {&p->g_ev, &p->t_ev, &p->user_ev, &p->prep_ev})
      if (!*e) HIP_OK(hipEventCreateWithFlags(e, hipEventDisableTiming));
    for (hipEvent_t& e : p->red_ev)
      if (!e) {
        HIP_OK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        HIP_OK(hipEventRecord(e, s));
      }
    OB_TRY(ensure_buf(&p->d_partialb, p->cap_partialb, need_partial * p->e_pad));
    HIP_OK(hipEventRecord(p->user_ev, s));
    if (s_work) {
      HIP_OK(hipEventRecord(p->prep_ev, s));
      HIP_OK(hipStreamWaitEvent(p->g_stream, p->prep_ev, 0));
    }
  }
  const hipStream_t sg = tov ? p->g_stream : s;  // the Gram
  const hipStream_t st = tov ? p->t_stream : s;  // reduce, exceptions, solve
  for (uint64_t s0 = 0; s0 < n_reps; s0 += seg) {
    const uint32_t ns = (uint32_t)std::min<uint64_t>(seg, n_reps - s0);
    const Plan& plx = (ns == seg) ? pl : pl_tail;
    const int nchx = plx.n_chunks();
    const uint32_t frep = (uint32_t)(first_rep + s0);
    hipEvent_t* ev = p->seg_events.data() + kSegEvents * (size_t)p->pending_segments;
    const bool timed = true;
    const int buf = dbl ? p->rs_parity : 0;
    uint32_t* const m1 = buf ? p->d_m1b : p->d_m1;
    uint32_t* const counts = buf ? p->d_countsb : p->d_counts;
    const hipEvent_t sev = buf ? p->scratch_ev2 : p->scratch_ev;  // the last read of this buffer
    if (dbl) p->rs_parity ^= 1;
    const int pb = tov ? p->part_parity : 0;
    if (tov) p->part_parity ^= 1;
    double* const partial = pb ? p->d_partialb : p->d_partial;
    if (overlap) HIP_OK(hipStreamWaitEvent(sr, sev, 0));
    if (timed) HIP_OK(hipEventRecord(ev[0], sr));
    // pieces (option rs_pieces): level 1 over replicate batches [b0, b1) of piece k, then (below) the
    // count kernel of each piece on cnt_stream once its level 1 is done, beside the next piece's
    const int npc = overlap ? std::max(1, std::min({rs_pieces, 8, (int)plx.nb_rep})) : 1;
    for (int k = 0; k < npc; ++k) {
      const uint32_t r0 = std::min<uint32_t>(64u * (plx.nb_rep * k / npc), ns);
      const uint32_t r1 = std::min<uint32_t>(64u * (plx.nb_rep * (k + 1) / npc), ns);
      if (r1 > r0)
        hipLaunchKernelGGL(l1k, dim3(r1 - r0, 2), dim3(kBlock), lds_l1, sr, p->n[0], p->n[1], p->ntiles[0],
                           frep + r0, tiles, key0, key1, m1 + (size_t)r0 * tiles, ky);
      HIP_OK(hipGetLastError());
      if (npc > 1) HIP_OK(hipEventRecord(p->cnt_ev[k], sr));
    }
    if (timed) HIP_OK(hipEventRecord(ev[1], sr));
    GramArgs ga = gram_args(p, plx);
    ga.chunks = p->d_chunks;
    ga.m1 = m1;
    ga.n_reps = ns;
    ga.first_rep = frep;
    ga.key0 = key0;
    ga.key1 = key1;
    ga.partial = partial;
    ga.counts = counts;
    ga.tiles_total = tiles;
    ga.diag = diag_mode();
    const hipStream_t sc = npc > 1 ? p->cnt_stream : sr;
    for (int k = 0; k < npc; ++k) {
      const uint32_t b0 = plx.nb_rep * k / npc, b1 = plx.nb_rep * (k + 1) / npc;
      if (npc > 1) HIP_OK(hipStreamWaitEvent(sc, p->cnt_ev[k], 0));
      if (b1 == b0) continue;
      ga.rb0 = b0;
      const dim3 cgrid((tiles + kCntTilesPerBlock - 1) / kCntTilesPerBlock, b1 - b0);
      if (use_i8) hipLaunchKernelGGL(ob_count_kernel<true>, cgrid, dim3(kBlock), 0, sc, ga);
      else hipLaunchKernelGGL(ob_count_kernel<false>, cgrid, dim3(kBlock), 0, sc, ga);
      HIP_OK(hipGetLastError());
    }
    ga.rb0 = 0;
    if (timed) HIP_OK(hipEventRecord(ev[2], sc));
    if (overlap) {
      HIP_OK(hipEventRecord(p->rs_ev, sc));
      HIP_OK(hipStreamWaitEvent(sg, p->rs_ev, 0));
    }
    if (tov) HIP_OK(hipStreamWaitEvent(sg, p->red_ev[pb], 0));  // the reduce two segments back read it
    if (timed) HIP_OK(hipEventRecord(ev[3], sg));
    if (use_i8) {
      OB_TRY(ob::oz_gram(p, p->d_chunks, nchx, counts, plx.nb_rep, plx.rep_pad, ns, partial, sg));
    } else {
      const uint32_t blocks = plx.nb_rep * plx.n_cg * (uint32_t)nchx;
      HIP_OK(launch_gram(p, plx.cb, false, ga, blocks, sg));
    }
    if (timed) HIP_OK(hipEventRecord(ev[4], sg));
    const bool exc = use_i8 && ob::oz_exceptions_pending(p);
    if (overlap && !exc) HIP_OK(hipEventRecord(sev, sg));  // the count images are free again
    if (tov) {
      HIP_OK(hipEventRecord(p->g_ev, sg));
      HIP_OK(hipStreamWaitEvent(st, p->g_ev, 0));
      HIP_OK(hipStreamWaitEvent(st, p->user_ev, 0));  // the caller's use of the rows buffers so far
    }
    const size_t nred = (size_t)ns * p->e_pad;
    hipLaunchKernelGGL(ob_reduce_kernel, dim3((unsigned)((nred + kBlock - 1) / kBlock)), dim3(kBlock), 0, st,
                       (const double*)partial, (const uint32_t*)p->d_chunks, nchx, plx.rep_pad, p->e_pad, ns,
                       p->d_gram);
    HIP_OK(hipGetLastError());
    if (tov) HIP_OK(hipEventRecord(p->red_ev[pb], st));
    if (exc) {
      OB_TRY(ob::oz_exceptions(p, counts, plx.nb_rep, ns, p->d_gram, st));
      if (overlap) HIP_OK(hipEventRecord(sev, st));
    }
    if (timed) HIP_OK(hipEventRecord(ev[5], st));
    if (p->heckman) {  // probit iterations + IMR sums + two-step solve (synchronizes the stream)
      ob_heck_seg hs = heck_seg(p, plx, p->d_chunks, p->d_gram, ref_mode);
      hs.counts = counts;
      hs.counts_i8 = use_i8 ? 1 : 0;
      hs.n_reps = ns;
      hs.rows = d_rows + s0 * p->row_len;
      hs.ok = d_ok + s0;
      hs.raw_status = (diag_mode() & 8) ? 1 : 0;  // OB_GRAM_DIAG bit 8: ok[] = ob_heck_status codes
      int it = 0;
      ob::ob_heck_times ht;
      OB_TRY(ob::heckman_segment(hs, s, &it, &ht));
      p->timing.probit_iterations = std::max(p->timing.probit_iterations, it);
      p->timing.probit_ms += ht.probit_ms;
      p->timing.probit_launches += ht.probit_launches;
      p->timing.heck_sums_ms += ht.sums_ms;
    }
    for (int t = 0; t < p->n_y && !p->heckman; ++t) {  // outcome-major row blocks
      SolveArgs sa = solve_args(p, ref_mode);
      sa.yc = p->p + 1 + t;
      sa.gram = p->d_gram;
      sa.rows = d_rows + ((size_t)t * n_reps + s0) * p->row_len;
      sa.ok = d_ok + (size_t)t * n_reps + s0;
      sa.n_reps = ns;
      sa.gram_out = nullptr;
      sa.raw_beta_b = nullptr;
      sa.raw_status = 0;
      HIP_OK(launch_solve(p, sa, ns, st));
    }
    if (timed) HIP_OK(hipEventRecord(ev[6], st));
    p->timing.gram_launches += 1;
    p->pending_segments += 1;
  }
  if (tov) {  // the caller's stream sees the rows complete, as without the tail stream
    HIP_OK(hipEventRecord(p->t_ev, st));
    HIP_OK(hipStreamWaitEvent(s, p->t_ev, 0));
  }
  p->timing_pending = true;
  p->last_stream = s;
  return engine_mark(p, s, !overlap);
}

// Synchronize the last boot run, sum its per-segment kernel timings and check the
// count-overflow flag.
int engine_collect(ob_panel* p) {
  if (!p->timing_pending) return OB_OK;
  HIP_OK(hipSetDevice(p->ctx->device));
  HIP_OK(hipStreamSynchronize(p->last_stream));
  p->timing_pending = false;
  // (ev[2] -> ev[3] is the Gram's wait for the previous call's tail on the boot stream: not a kernel)
  double* dst[kSegEvents - 1] = {&p->timing.level1_ms, &p->timing.counts_ms, nullptr, &p->timing.gram_ms,
                                 &p->timing.reduce_ms, &p->timing.solve_ms};
  for (int sg = 0; sg < p->pending_segments; ++sg) {
    hipEvent_t* ev = p->seg_events.data() + kSegEvents * (size_t)sg;
    for (size_t i = 0; i + 1 < kSegEvents; ++i) {
      if (!dst[i]) continue;
      float t = 0.f;
      HIP_OK(hipEventElapsedTime(&t, ev[i], ev[i + 1]));
      *dst[i] += t;
    }
  }
  if (p->heckman) p->timing.heckman_ms = p->timing.solve_ms;
  for (int k = 0; k < p->pending_gathers; ++k) {  // ob_shard.cpp: the RCCL all-gathers
    float t = 0.f;
    HIP_OK(hipEventElapsedTime(&t, p->gather_evs[2 * k], p->gather_evs[2 * k + 1]));
    p->timing.gather_ms += t;
  }
  p->pending_gathers = 0;
  p->pending_segments = 0;
  if (p->timing.gram_path == 2) OB_TRY(ob::oz_collect(p));
  uint32_t flag = 0;
  HIP_OK(hipMemcpy(&flag, p->d_flags, sizeof(uint32_t), hipMemcpyDeviceToHost));
  if (flag) HIP_OK(hipMemset(p->d_flags, 0, sizeof(uint32_t)));  // collected: the next calls start clean
  // a count of 256+ wraps its byte (bit 0: byte sums differ from the tile counts); on the i8 path
  // the bound is 127 either way
  if ((flag & 1u) && p->timing.gram_path != 2)
    return ob::fail(OB_E_OVERFLOW, "a resampled row was drawn more than 255 times in one replicate");
  if (flag & 3u)  // p ~ 1e-215 per row and replicate; the f64 Gram path takes counts up to 255
    return ob::fail(OB_E_OVERFLOW, "a resampled row was drawn more than 127 times in one replicate "
                                   "(the i8 Gram's range; option gram_path = 1 runs the f64 MFMA Gram)");
  return OB_OK;
}

}  // namespace ob

// ---------------------------------------------------------------------------------------------
// panel lifecycle (C ABI parts that touch HIP)
// ---------------------------------------------------------------------------------------------
extern "C" {

int ob_device_count(int* n) {
  if (!n) return ob::fail(OB_E_INVALID, "null pointer");
  *n = 0;
  hipError_t e = hipGetDeviceCount(n);
  if (e != hipSuccess) {
    *n = 0;
    return ob::fail(OB_E_HIP, "no HIP device: %s", hipGetErrorString(e));
  }
  return OB_OK;
}

int ob_ctx_create(int device, ob_ctx** out) {
  if (!out) return ob::fail(OB_E_INVALID, "null pointer");
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n == 0)
    return ob::fail(OB_E_HIP, "no HIP device visible: the MI355X engine has no CPU fallback");
  if (device < 0 || device >= n) return ob::fail(OB_E_INVALID, "device %d out of range (%d devices)", device, n);
  HIP_OK(hipSetDevice(device));
  hipDeviceProp_t prop;
  HIP_OK(hipGetDeviceProperties(&prop, device));
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
    return ob::fail(OB_E_HIP, "device %d is %s; this engine is built for gfx950 (MI355X) only", device,
                    prop.gcnArchName);
  ob_ctx* c = new ob_ctx();
  c->device = device;
  c->cus = prop.multiProcessorCount;
  hipError_t e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
  if (e != hipSuccess) {
    delete c;
    return ob::fail(OB_E_HIP, "hipStreamCreate: %s", hipGetErrorString(e));
  }
  *out = c;
  return OB_OK;
}

void ob_ctx_destroy(ob_ctx* ctx) {
  if (!ctx) return;
  (void)hipSetDevice(ctx->device);
  if (ctx->comm && ctx->comm_free) ctx->comm_free(ctx->comm);
  if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
  delete ctx;
}

int ob_panel_create(ob_ctx* ctx, const ob_panel_desc* d, ob_panel** out) {
  if (!ctx || !d || !out) return ob::fail(OB_E_INVALID, "null pointer");
  *out = nullptr;
  if (d->p < 0 || d->p > 120) return ob::fail(OB_E_UNSUPPORTED, "predictor columns must be in [0, 120], got %d", d->p);
  if (d->n_y < 0 || d->p + std::max(1, (int)d->n_y) > 121)
    return ob::fail(OB_E_UNSUPPORTED, "outcome columns must be in [1, %d], got %d", 121 - d->p, d->n_y);
  if (d->n_num < 0 || d->n_num > d->p) return ob::fail(OB_E_INVALID, "n_num out of range");
  const ob_group_desc* gd[2] = {&d->a, &d->b};
  const bool heck = d->heckman != 0;
  if (heck) {
    if (d->n_zsel < 0 || d->n_zsel > ob::kHeckMaxKs - 1)
      return ob::fail(OB_E_UNSUPPORTED, "Heckman selection predictors must be in [0, %d], got %d", ob::kHeckMaxKs - 1,
                      d->n_zsel);
    if (d->p > ob::kHeckMaxP)
      return ob::fail(OB_E_UNSUPPORTED, "Heckman panels take at most %d predictor columns, got %d", ob::kHeckMaxP, d->p);
    if (d->n_y > 1 || d->n_norm > 0)
      return ob::fail(OB_E_UNSUPPORTED, "Heckman panels take one outcome and no normalization");
    const double* sp[2] = {d->sa, d->sb};
    const double* zp[2] = {d->za, d->zb};
    for (int g = 0; g < 2; ++g)
      if (gd[g]->n > 0 && (!sp[g] || (d->n_zsel > 0 && !zp[g])))
        return ob::fail(OB_E_INVALID, "missing selection column pointer");
  }
  for (int g = 0; g < 2; ++g) {
    if (gd[g]->n < 0 || gd[g]->n > kMaxGroupRows)
      return ob::fail(OB_E_UNSUPPORTED, "group rows must be in [0, %lld]", (long long)kMaxGroupRows);
    if (gd[g]->n > 0 && ((d->p > 0 && !gd[g]->x) || !gd[g]->y || (d->weighted && !gd[g]->w)))
      return ob::fail(OB_E_INVALID, "missing column pointer");
    if (gd[g]->ldx < gd[g]->n) return ob::fail(OB_E_INVALID, "ldx < n");
    if (d->weighted && !heck)  // the Heckman OLS is unweighted: weights only scale the gap / Cotton
      for (int64_t i = 0; i < gd[g]->n; ++i)
        if (gd[g]->w[i] < 0.0)
          return ob::fail(OB_E_GROUP, "%sWeights cannot be negative", ob::error_prefix(OB_E_GROUP));
  }
  HIP_OK(hipSetDevice(ctx->device));
  ob_panel* p = new ob_panel();
  p->ctx = ctx;
  p->p = d->p;
  p->k = d->p + 1;
  p->n_y = std::max(1, (int)d->n_y);
  p->k1 = d->p + 1 + p->n_y;
  p->e = p->k1 * (p->k1 + 1) / 2;
  p->ncb = (p->e + 15) / 16;
  p->e_pad = p->ncb * 16;
  p->n_num = d->n_num;
  p->heckman = heck ? 1 : 0;
  p->ks = heck ? 1 + d->n_zsel : 0;
  p->h_weighted = heck && d->weighted ? 1 : 0;
  p->weighted = (d->weighted || heck) ? 1 : 0;
  ob_norm_cfg& nc = p->norm;
  nc.n_norm = d->n_norm;
  if (d->n_norm > 0) {
    nc.start.assign(d->norm_start, d->norm_start + d->n_norm + 1);
    nc.idx.assign(d->norm_idx, d->norm_idx + nc.start.back());
    nc.m.assign(d->norm_m, d->norm_m + d->n_norm);
    nc.pstart.assign(d->pooled_start, d->pooled_start + d->n_norm + 1);
    nc.pidx.assign(d->pooled_idx, d->pooled_idx + nc.pstart.back());
    nc.has_base.assign(d->has_base, d->has_base + d->n_norm);
    for (int v = 0; v < d->n_norm; ++v) nc.n_base += nc.has_base[v] ? 1 : 0;
  } else {
    nc.start.assign(1, 0);
    nc.pstart.assign(1, 0);
  }
  p->row_len = heck ? ob::heck_row_len(p->k, p->ks) : ob_row_len(p->k, nc.n_base);
  int rc = OB_OK;
  auto bad = [&](hipError_t e, int line) {
    rc = ob::fail(OB_E_HIP, "HIP error %s at %s:%d", hipGetErrorString(e), __FILE__, line);
  };
  for (int g = 0; g < 2 && rc == OB_OK; ++g) {
    p->n[g] = (uint32_t)gd[g]->n;
    p->ntiles[g] = (p->n[g] + OB_TILE_ROWS - 1) / OB_TILE_ROWS;
    p->ld[g] = (int64_t)std::max<uint32_t>(p->ntiles[g], 1) * OB_TILE_ROWS;
    const int ncols = heck ? p->p + 3 + (p->ks - 1) + p->h_weighted : p->p + p->n_y + p->weighted;
    const size_t bytes = sizeof(double) * (size_t)ncols * p->ld[g];
    hipError_t e = hipMalloc(&p->d_cols[g], bytes);
    if (e != hipSuccess) { bad(e, __LINE__); break; }
    e = hipMemset(p->d_cols[g], 0, bytes);
    if (e != hipSuccess) { bad(e, __LINE__); break; }
    const int64_t n = gd[g]->n;
    if (n > 0) {
      if (p->p > 0) {
        e = hipMemcpy2D(p->d_cols[g], sizeof(double) * p->ld[g], gd[g]->x, sizeof(double) * gd[g]->ldx,
                        sizeof(double) * n, p->p, hipMemcpyHostToDevice);
        if (e != hipSuccess) { bad(e, __LINE__); break; }
      }
      e = hipMemcpy2D(p->d_cols[g] + (size_t)p->p * p->ld[g], sizeof(double) * p->ld[g], gd[g]->y,
                      sizeof(double) * gd[g]->ldx, sizeof(double) * n, p->n_y, hipMemcpyHostToDevice);
      if (e != hipSuccess) { bad(e, __LINE__); break; }
      if (heck) {  // ob_heckman.hpp layout: x | y | [s == 1] | s | z | (w)
        const double* sg = g ? d->sb : d->sa;
        const double* zg = g ? d->zb : d->za;
        std::vector<double> ind((size_t)n);
        for (int64_t i = 0; i < n; ++i) ind[i] = sg[i] == 1.0 ? 1.0 : 0.0;  // estimation.rs:203-206 (== 1)
        double* c0 = p->d_cols[g] + (size_t)(p->p + 1) * p->ld[g];
        e = hipMemcpy(c0, ind.data(), sizeof(double) * n, hipMemcpyHostToDevice);
        if (e == hipSuccess) e = hipMemcpy(c0 + p->ld[g], sg, sizeof(double) * n, hipMemcpyHostToDevice);
        if (e == hipSuccess && p->ks > 1)
          e = hipMemcpy2D(c0 + 2 * p->ld[g], sizeof(double) * p->ld[g], zg, sizeof(double) * gd[g]->ldx,
                          sizeof(double) * n, p->ks - 1, hipMemcpyHostToDevice);
        if (e == hipSuccess && p->h_weighted)
          e = hipMemcpy(c0 + (size_t)(1 + p->ks) * p->ld[g], gd[g]->w, sizeof(double) * n, hipMemcpyHostToDevice);
        if (e != hipSuccess) { bad(e, __LINE__); break; }
      } else if (p->weighted) {
        e = hipMemcpy(p->d_cols[g] + (size_t)(p->p + p->n_y) * p->ld[g], gd[g]->w, sizeof(double) * n,
                      hipMemcpyHostToDevice);
        if (e != hipSuccess) { bad(e, __LINE__); break; }
      }
    }
  }
  for (int g = 0; g < 2 && rc == OB_OK; ++g) {
    const int ncl = p->k1 - (p->weighted ? 0 : 1);
    const size_t elems = (size_t)(p->ld[g] >> 6) * ncl * kColStride;
    hipError_t e = hipMalloc(&p->d_gpanel[g], sizeof(double) * std::max<size_t>(elems, 1));
    if (e == hipSuccess && elems) {
      hipLaunchKernelGGL(ob_panel_kernel, dim3((unsigned)((elems + kBlock - 1) / kBlock)), dim3(kBlock), 0, 0,
                         (const double*)p->d_cols[g], p->ld[g], p->p + p->n_y, p->weighted, p->d_gpanel[g]);
      e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (e != hipSuccess) bad(e, __LINE__);
  }
  if (rc == OB_OK) {
    std::vector<int32_t> packed;
    packed.insert(packed.end(), nc.start.begin(), nc.start.end());
    packed.insert(packed.end(), nc.idx.begin(), nc.idx.end());
    packed.insert(packed.end(), nc.m.begin(), nc.m.end());
    packed.insert(packed.end(), nc.pstart.begin(), nc.pstart.end());
    packed.insert(packed.end(), nc.pidx.begin(), nc.pidx.end());
    packed.insert(packed.end(), nc.has_base.begin(), nc.has_base.end());
    packed.push_back(0);
    hipError_t e = hipMalloc(&p->d_norm, sizeof(int32_t) * packed.size());
    if (e == hipSuccess) e = hipMemcpy(p->d_norm, packed.data(), sizeof(int32_t) * packed.size(), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMalloc(&p->d_flags, sizeof(uint32_t) * 4);
    if (e == hipSuccess) e = hipMemset(p->d_flags, 0, sizeof(uint32_t) * 4);  // read by calls that draw nothing
    if (e != hipSuccess) bad(e, __LINE__);
  }
  if (rc != OB_OK) {
    ob_panel_destroy(p);
    return rc;
  }
  *out = p;
  return OB_OK;
}

void ob_panel_destroy(ob_panel* p) {
  if (!p) return;
  (void)hipSetDevice(p->ctx->device);
  if (p->timing_pending) (void)hipStreamSynchronize(p->last_stream);
  for (int g = 0; g < 2; ++g) {
    (void)hipFree(p->d_cols[g]);
    (void)hipFree(p->d_gpanel[g]);
  }
  (void)hipFree(p->d_norm);
  (void)hipFree(p->d_m1);
  (void)hipFree(p->d_counts);
  (void)hipFree(p->d_m1b);
  (void)hipFree(p->d_countsb);
  (void)hipFree(p->d_partial);
  (void)hipFree(p->d_gram);
  (void)hipFree(p->d_chunks);
  (void)hipFree(p->d_flags);
  (void)hipFree(p->d_hgamma);
  (void)hipFree(p->d_hflags);
  (void)hipFree(p->d_hpartial);
  (void)hipFree(p->d_hactive);
  (void)hipFree(p->d_rows_tmp);
  (void)hipFree(p->d_ok_tmp);
  (void)hipFree(p->d_pe);
  (void)hipFree(p->d_pe_ok);
  if (p->rs_stream) (void)hipStreamSynchronize(p->rs_stream);
  if (p->rs_ev) (void)hipEventDestroy(p->rs_ev);
  if (p->scratch_ev) (void)hipEventDestroy(p->scratch_ev);
  if (p->scratch_ev2) (void)hipEventDestroy(p->scratch_ev2);
  for (hipStream_t x : {p->g_stream, p->t_stream})
    if (x) (void)hipStreamSynchronize(x);
  for (hipEvent_t e : {p->g_ev, p->t_ev, p->user_ev, p->prep_ev, p->red_ev[0], p->red_ev[1]})
    if (e) (void)hipEventDestroy(e);
  for (hipStream_t x : {p->g_stream, p->t_stream})
    if (x) (void)hipStreamDestroy(x);
  (void)hipFree(p->d_partialb);
  if (p->cnt_stream) (void)hipStreamSynchronize(p->cnt_stream);
  for (hipEvent_t e : p->cnt_ev)
    if (e) (void)hipEventDestroy(e);
  if (p->cnt_stream) (void)hipStreamDestroy(p->cnt_stream);
  if (p->rs_stream) (void)hipStreamDestroy(p->rs_stream);
  ob::shard_free(p);
  ob::oz_free(p);
  (void)hipFree(p->d_mm_fail);
  for (hipEvent_t e : p->seg_events) (void)hipEventDestroy(e);
  if (p->order_ev) (void)hipEventDestroy(p->order_ev);
  if (p->mm_ws_free) p->mm_ws_free(p->mm_ws);
  delete p;
}

int ob_panel_row_len(const ob_panel* p) { return p ? p->row_len : 0; }
int ob_panel_k(const ob_panel* p) { return p ? p->k : 0; }
int ob_panel_n_base(const ob_panel* p) { return p ? p->norm.n_base : 0; }
int ob_panel_n_y(const ob_panel* p) { return p ? p->n_y : 0; }

static bool valid_ref(int m) { return m >= OB_REF_GROUP_A && m <= OB_REF_NEUMARK; }

int ob_point_estimate(ob_panel* p, int ref_mode, double* row, double* resid_b) {
  if (!p || !row) return ob::fail(OB_E_INVALID, "null pointer");
  if (!valid_ref(ref_mode)) return ob::fail(OB_E_INVALID, "unknown reference coefficients %d", ref_mode);
  if (p->n[0] == 0 || p->n[1] == 0)
    return ob::fail(OB_E_GROUP, "%sOne group has no data", ob::error_prefix(OB_E_GROUP));
  for (int g = 0; g < 2; ++g)  // ols.rs:98-105 (row count, not sum of weights)
    if ((double)p->n[g] <= (double)p->k)
      return ob::fail(OB_E_INSUFFICIENT,
                      "%sInsufficient data for OLS calculation: n_obs (%u) must be strictly greater than k (%d)",
                      ob::error_prefix(OB_E_INSUFFICIENT), p->n[g], p->k);
  if (ref_mode == OB_REF_POOLED || ref_mode == OB_REF_NEUMARK) {
    if ((double)(p->n[0] + p->n[1]) <= (double)(p->k + 1))
      return ob::fail(OB_E_INSUFFICIENT,
                      "%sInsufficient data for OLS calculation: n_obs (%u) must be strictly greater than k (%d)",
                      ob::error_prefix(OB_E_INSUFFICIENT), p->n[0] + p->n[1], p->k + 1);
  }
  // ordered after any call on this panel from another stream (an async boot on a user
  // stream may still read the buffers the point estimate rewrites), and marked for the next one
  HIP_OK(hipSetDevice(p->ctx->device));
  hipStream_t s = p->ctx->stream;
  OB_TRY(ob::engine_order(p, s));
  const int rc = ob::engine_point_estimate(p, ref_mode, row, resid_b);
  const int rm = ob::engine_mark(p, s);
  return rc != OB_OK ? rc : rm;
}

int ob_boot_run_device(ob_panel* p, uint64_t seed, uint64_t first_rep, uint64_t n_reps, int ref_mode,
                       double* d_rows, uint8_t* d_ok, void* hip_stream) {
  if (!p || (n_reps && (!d_rows || !d_ok))) return ob::fail(OB_E_INVALID, "null pointer");
  if (!valid_ref(ref_mode)) return ob::fail(OB_E_INVALID, "unknown reference coefficients %d", ref_mode);
  if (p->n[0] == 0 || p->n[1] == 0)
    return ob::fail(OB_E_GROUP, "%sOne group has no data", ob::error_prefix(OB_E_GROUP));
  if (p->ntiles[0] > kMaxGroupRows / OB_TILE_ROWS || p->ntiles[1] > kMaxGroupRows / OB_TILE_ROWS)
    return ob::fail(OB_E_UNSUPPORTED, "groups take at most %lld rows", (long long)kMaxGroupRows);
  return ob::engine_boot(p, seed, first_rep, n_reps, ref_mode, d_rows, d_ok,
                         reinterpret_cast<hipStream_t>(hip_stream));
}

int ob_boot_run(ob_panel* p, uint64_t seed, uint64_t first_rep, uint64_t n_reps, int ref_mode, double* rows,
                uint8_t* ok) {
  if (!p || (n_reps && (!rows || !ok))) return ob::fail(OB_E_INVALID, "null pointer");
  if (n_reps == 0) return OB_OK;
  HIP_OK(hipSetDevice(p->ctx->device));
  if (p->tmp_reps < n_reps) {
    (void)hipFree(p->d_rows_tmp);
    (void)hipFree(p->d_ok_tmp);
    p->d_rows_tmp = nullptr;
    p->d_ok_tmp = nullptr;
    p->tmp_reps = 0;
    HIP_OK(hipMalloc(&p->d_rows_tmp, sizeof(double) * n_reps * p->row_len * p->n_y));
    HIP_OK(hipMalloc(&p->d_ok_tmp, n_reps * p->n_y));
    p->tmp_reps = n_reps;
  }
  OB_TRY(ob_boot_run_device(p, seed, first_rep, n_reps, ref_mode, p->d_rows_tmp, p->d_ok_tmp, nullptr));
  OB_TRY(ob::engine_collect(p));
  HIP_OK(hipMemcpy(rows, p->d_rows_tmp, sizeof(double) * n_reps * p->row_len * p->n_y, hipMemcpyDeviceToHost));
  HIP_OK(hipMemcpy(ok, p->d_ok_tmp, n_reps * p->n_y, hipMemcpyDeviceToHost));
  return OB_OK;
}

// Test hook (include/oaxaca_boot.h): the panel's chunk table, as make_plan builds it.
int ob_debug_chunks(const ob_panel* p, uint32_t* table, int32_t cap, int32_t* n_chunks) {
  if (!p || !n_chunks || (cap > 0 && !table)) return ob::fail(OB_E_INVALID, "null pointer");
  const Plan pl = make_plan(p, 64, false);
  *n_chunks = pl.n_chunks();
  for (int32_t i = 0; i < 3 * std::min(cap, *n_chunks); ++i) table[i] = pl.chunks[i];
  return OB_OK;
}

// Test hook (include/oaxaca_boot.h): the OBRS-2 counts of replicates [first_rep, first_rep + n)
// exactly as ob_count_kernel leaves them for the Gram kernel, unpacked on the host.
int ob_debug_counts(ob_panel* p, uint64_t seed, uint64_t first_rep, uint32_t n_reps, int group, uint32_t* level1,
                    uint8_t* row_counts) {
  if (!p || (group != 0 && group != 1)) return ob::fail(OB_E_INVALID, "bad arguments");
  if (n_reps == 0) return OB_OK;
  if (n_reps > 16384) return ob::fail(OB_E_INVALID, "at most 16384 replicates per call");
  HIP_OK(hipSetDevice(p->ctx->device));
  hipStream_t s = p->ctx->stream;
  uint32_t nb = 0, rep_pad = 0;
  OB_TRY(ob::engine_order(p, s));  // after any call on this panel from another stream
  HIP_OK(hipMemsetAsync(p->d_flags + 2, 0, sizeof(uint32_t), s));  // engine_counts' overflow word
  const int rc = ob::engine_counts(p, seed, first_rep, n_reps, s, &nb, &rep_pad);
  OB_TRY(ob::engine_mark(p, s));
  OB_TRY(rc);
  HIP_OK(hipStreamSynchronize(s));
  uint32_t flag = 0;
  HIP_OK(hipMemcpy(&flag, p->d_flags + 2, sizeof(uint32_t), hipMemcpyDeviceToHost));  // engine_counts' word
  if (flag & 1u) return ob::fail(OB_E_OVERFLOW, "a resampled row was drawn more than 255 times in one replicate");
  const uint32_t tiles = p->ntiles[0] + p->ntiles[1], tg = p->ntiles[group], t0 = group ? p->ntiles[0] : 0u;
  const uint32_t n = p->n[group];
  if (level1) {
    std::vector<uint32_t> m1((size_t)tiles * n_reps);
    HIP_OK(hipMemcpy(m1.data(), p->d_m1, sizeof(uint32_t) * m1.size(), hipMemcpyDeviceToHost));
    for (uint32_t r = 0; r < n_reps; ++r)
      for (uint32_t t = 0; t < tg; ++t) level1[(size_t)r * tg + t] = m1[(size_t)r * tiles + t0 + t];
  }
  if (row_counts && n) {
    const size_t per_tile = (size_t)nb * 4 * kCimgWords;
    std::vector<uint32_t> img((size_t)tg * per_tile);
    HIP_OK(hipMemcpy(img.data(), p->d_counts + (size_t)t0 * per_tile, sizeof(uint32_t) * img.size(),
                     hipMemcpyDeviceToHost));
    for (uint32_t r = 0; r < n_reps; ++r) {
      const uint32_t b = r >> 6, lr = r & 63u;
      for (uint32_t i = 0; i < n; ++i) {
        const uint32_t t = i / OB_TILE_ROWS, within = i % OB_TILE_ROWS, sub = within >> 6, q = within & 63u;
        const uint32_t word = img[(size_t)t * per_tile + ((size_t)b * 4 + sub) * kCimgWords + lr * kCimgStride + (q >> 2)];
        row_counts[(size_t)r * n + i] = (uint8_t)((word >> (8 * (q & 3u))) & 0xFFu);
      }
    }
  }
  return OB_OK;
}

// Test hook: the reduced extended Grams [n_reps][2 groups][e_pad] of replicates
// [first_rep, first_rep + n_reps) through the requested Gram path (0 auto, 1 f64 MFMA, 2 i8).
int ob_debug_gram(ob_panel* p, int path, uint64_t seed, uint64_t first_rep, uint32_t n_reps, double* gram) {
  if (!p || !gram || path < 0 || path > 2) return ob::fail(OB_E_INVALID, "bad arguments");
  if (n_reps == 0) return OB_OK;
  if (n_reps > 16384) return ob::fail(OB_E_INVALID, "at most 16384 replicates per call (one segment)");
  if (p->heckman) return ob::fail(OB_E_UNSUPPORTED, "Heckman panels use the f64 Gram only");
  HIP_OK(hipSetDevice(p->ctx->device));
  double* d_rows = nullptr;
  uint8_t* d_ok = nullptr;
  HIP_OK(hipMalloc(&d_rows, sizeof(double) * n_reps * p->row_len * p->n_y));
  HIP_OK(hipMalloc(&d_ok, (size_t)n_reps * p->n_y));
  const int saved = p->gram_force;
  p->gram_force = path;
  int rc = ob_boot_run_device(p, seed, first_rep, n_reps, OB_REF_GROUP_A, d_rows, d_ok, nullptr);
  p->gram_force = saved;
  if (rc == OB_OK) rc = ob::engine_collect(p);
  if (rc == OB_OK && hipMemcpy(gram, p->d_gram, sizeof(double) * 2 * (size_t)n_reps * p->e_pad,
                               hipMemcpyDeviceToHost) != hipSuccess)
    rc = ob::fail(OB_E_HIP, "copy of the Gram failed");
  (void)hipFree(d_rows);
  (void)hipFree(d_ok);
  return rc;
}

int ob_panel_sync(ob_panel* p) {
  if (!p) return ob::fail(OB_E_INVALID, "null pointer");
  return ob::engine_collect(p);
}

int ob_panel_last_timing(const ob_panel* p, ob_timing* out) {
  if (!p || !out) return ob::fail(OB_E_INVALID, "null pointer");
  *out = p->timing;
  return OB_OK;
}

}  // extern "C"
