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
// Pairs of narrow magnitude range take six digits (the seventh written as zero, oz_nsl_kernel:
// error bound below a quarter of an f64 summation's), and column tiles of such pairs run 6 slices.
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
#include "ob_options.hpp"
#include "ob_spec.h"

typedef int ob_v4i __attribute__((ext_vector_type(4)));
typedef int ob_v16i __attribute__((ext_vector_type(16)));

namespace {

constexpr int kS = 7;                  // balanced 8-bit digits per pair product (54-bit fixed point)
constexpr int kFracBits = 54;          // m = rint(P 2^(kFracBits - E))
constexpr int kPairsPerTile = 32;      // pairs per column tile (one 32-wide MFMA column block)
constexpr int kSubUnits = kS * 2 * 64; // 16-byte units of one (sub-tile, column tile) B image (14 KB)
constexpr int kSlo = 4;                // slices of slice group 0 (waves 0-3); group 1 has kS - kSlo
#ifndef OB_OZ_SIX0
#define OB_OZ_SIX0 4
#endif
constexpr int kSix0 = OB_OZ_SIX0;      // six-slice blocks: slices of group 0 (group 1: 6 - kSix0)
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

// ---------------------------------------------------------------------------------------------
// Panel preparation (once per panel, on the boot stream; no host synchronization).
//
// Exception rows. A fixed-point exponent per (chunk, pair) rounds every product of the chunk to
// 2^(E-55): a row whose magnitude dwarfs the chunk's (a top-coded 99,999,999, a sentinel, a
// heavy-tail draw) would set E for all the others and cost every replicate that does not draw it
// up to (max / typical)^2 2^-55 of relative accuracy. So, per (chunk, column c), the scale s_c is
// the rounded mean binary exponent of the column's nonzero finite |v_c| (the log of its geometric
// mean: one outlier in 15k rows moves it by 27 / 15k), and a row is an exception when some
// |v_c| >= 2^(s_c + B), or some v_c is not finite. Exception rows get zero digits and enter every
// replicate's Gram as c_ri P_i in f64 (oz_exc_kernel, zero counts skipped -- the gathered rows of
// the reference, builder.rs:822-829, never touch an undrawn row, NaN or not). For the others
// |v_c| < 2^(s_c + B) <= 2^(B + 1) rms(v_c) (rms >= geometric mean), so the rounding of any Gram
// entry stays below 2^(2B - 53) sqrt(G_aa G_bb) in the worst case (every rounding the same sign;
// ~ sqrt(n) smaller in practice): 2^-37 at B = 8. B starts at kOzBitsMin and rises only if more
// than kOzExcCap rows would be exceptions; more than kOzExcCap non-finite rows is an error.
// ---------------------------------------------------------------------------------------------
constexpr int kOzExcCap = 4096;  // exception rows per panel (both groups)
constexpr int kOzBitsMin = 8;
constexpr int kOzMaxK1 = 128;
constexpr int kExpBias = 4096;  // pair exponents while being reduced: ex + kExpBias, 0 = all zero
// d_oz_meta (int32): [0] B, [1] exceptions X (<= cap), [2] group-A exceptions, [3] overflow,
// [4] append cursor, [kMetaHist + d + 128] rows of deviation d (d in [-128, 127], 127 = non-finite)
constexpr int kMetaHist = 8;
constexpr int kMetaWords = kMetaHist + 256;

// Per (chunk, column): sum of the binary exponents (frexp) of the nonzero finite v_c and their
// count. Grid: the group's tiles (a tile lies in one chunk), one row per thread.
__global__ __launch_bounds__(256) void oz_scale_kernel(const double* cols, int64_t ld, uint32_t n, int nxy,
                                                       int weighted, int k1, const int32_t* tile_chunk,
                                                       unsigned long long* acc) {
  const uint32_t tile = blockIdx.x, row = tile * 256u + threadIdx.x;
  const int chunk = tile_chunk[tile], lane = threadIdx.x & 63;
  for (int c = 0; c < k1; ++c) {
    const double v = row < n ? oz_v(cols, ld, nxy, weighted, row, c) : 0.0;
    int ex = 0, nz = 0;
    if (v != 0.0 && isfinite(v)) {
      (void)frexp(v, &ex);
      nz = 1;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      ex += __shfl_xor(ex, o);
      nz += __shfl_xor(nz, o);
    }
    if (lane == 0 && nz) {
      atomicAdd(&acc[((size_t)chunk * k1 + c) * 2], (unsigned long long)(long long)ex);
      atomicAdd(&acc[((size_t)chunk * k1 + c) * 2 + 1], (unsigned long long)nz);
    }
  }
}

// Per row: d = max over columns of (exponent of v_c - s_c), clamped to [-128, 126]; 127 if some v_c
// is not finite; -128 for all-zero and padding rows. Histogram into meta.
__global__ __launch_bounds__(256) void oz_dev_kernel(const double* cols, int64_t ld, uint32_t n, int nxy, int weighted,
                                                     int k1, const int32_t* tile_chunk, const long long* acc,
                                                     int8_t* dev, int32_t* meta) {
  __shared__ int sc[kOzMaxK1];
  __shared__ uint32_t hist[256];
  const int tid = threadIdx.x;
  const uint32_t tile = blockIdx.x, row = tile * 256u + tid;
  const int chunk = tile_chunk[tile];
  hist[tid] = 0u;
  for (int c = tid; c < k1; c += 256) {
    const long long s = acc[((size_t)chunk * k1 + c) * 2], m = acc[((size_t)chunk * k1 + c) * 2 + 1];
    sc[c] = m ? (int)floor((double)s / (double)m + 0.5) : 0;
  }
  __syncthreads();
  int d = -128;
  if (row < n) {
    for (int c = 0; c < k1; ++c) {
      const double v = oz_v(cols, ld, nxy, weighted, row, c);
      if (v == 0.0) continue;
      if (!isfinite(v)) {
        d = 127;
        break;
      }
      int ex = 0;
      (void)frexp(v, &ex);
      d = max(d, min(ex - sc[c], 126));
    }
  }
  dev[row] = (int8_t)d;  // the grid covers the padded rows ld = 256 x tiles exactly
  atomicAdd(&hist[d + 128], 1u);
  __syncthreads();
  if (hist[tid]) atomicAdd(reinterpret_cast<uint32_t*>(meta) + kMetaHist + tid, hist[tid]);
}

// B = the smallest bits >= kOzBitsMin that leaves at most kOzExcCap exception rows.
__global__ void oz_choose_kernel(int32_t* meta) {
  if (threadIdx.x != 0) return;
  const uint32_t* h = reinterpret_cast<const uint32_t*>(meta) + kMetaHist;
  int b = kOzBitsMin;
  unsigned long long x = 0;
  for (;; ++b) {
    x = 0;
    for (int d = b + 1; d <= 127; ++d) x += h[d + 128];
    if (x <= (unsigned long long)kOzExcCap || b >= 126) break;
  }
  meta[0] = b;
  meta[1] = (int32_t)min(x, (unsigned long long)kOzExcCap);
  meta[3] = x > (unsigned long long)kOzExcCap ? 1 : 0;
  meta[4] = 0;
}

__global__ __launch_bounds__(256) void oz_collect_kernel(const int8_t* dev, uint32_t n, uint32_t g, int32_t* meta,
                                                         uint32_t* exc) {
  const uint32_t row = blockIdx.x * 256u + threadIdx.x;
  if (row >= n || dev[row] <= meta[0]) return;
  const int slot = atomicAdd(&meta[4], 1);
  if (slot < kOzExcCap) exc[slot] = (g << 31) | row;
}

// One block: bitonic sort of the exception list (padding 0xFFFFFFFF sorts last), so the f64 sums
// run in a fixed order (group A rows ascending, then group B's); meta[2] = group A's count.
__global__ __launch_bounds__(1024) void oz_sort_kernel(uint32_t* exc, int32_t* meta) {
  __shared__ uint32_t s[kOzExcCap];
  const int tid = threadIdx.x;
  for (int i = tid; i < kOzExcCap; i += 1024) s[i] = exc[i];
  __syncthreads();
  for (int k = 2; k <= kOzExcCap; k <<= 1)
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = tid; i < kOzExcCap; i += 1024) {
        const int ixj = i ^ j;
        if (ixj > i) {
          const uint32_t a = s[i], b = s[ixj];
          if ((a > b) == ((i & k) == 0)) {
            s[i] = b;
            s[ixj] = a;
          }
        }
      }
      __syncthreads();
    }
  for (int i = tid; i < kOzExcCap; i += 1024) {
    exc[i] = s[i];
    const bool here = s[i] < 0x80000000u, next = i + 1 < kOzExcCap && s[i + 1] < 0x80000000u;
    if (here && !next) meta[2] = i + 1;
  }
  if (tid == 0 && s[0] >= 0x80000000u) meta[2] = 0;
}

// f64 pair products of the exception rows: excp[x][e] = v_a v_b (NaN / inf kept).
__global__ __launch_bounds__(256) void oz_excp_kernel(const double* cols0, const double* cols1, int64_t ld0,
                                                      int64_t ld1, int nxy, int weighted, int k1, int e, int e_pad,
                                                      const uint32_t* exc, const int32_t* meta, double* excp) {
  const int x = blockIdx.x;
  if (x >= meta[1]) return;
  const uint32_t ent = exc[x], g = ent >> 31, row = ent & 0x7FFFFFFFu;
  const double* cols = g ? cols1 : cols0;
  const int64_t ld = g ? ld1 : ld0;
  for (int q = threadIdx.x; q < e_pad; q += 256) {
    double P = 0.0;
    if (q < e) {
      int a, b;
      oz_pair_cols(q, k1, &a, &b);
      P = oz_v(cols, ld, nxy, weighted, row, a) * oz_v(cols, ld, nxy, weighted, row, b);
    }
    excp[(size_t)x * e_pad + q] = P;
  }
}

// Stage the 64 rows [row0, row0 + 64) of every v column into vs[r * k1p + c], exception and
// padding rows as zeros. Coalesced: 64 consecutive rows of one column per wave instruction.
__device__ __forceinline__ void oz_stage(double* vs, int k1p, const double* cols, int64_t ld, uint32_t n, int nxy,
                                         int weighted, int k1, const int8_t* dev, int bits, size_t row0) {
  for (int i = threadIdx.x; i < 64 * k1; i += 256) {
    const int r = i & 63, c = i >> 6;
    const size_t row = row0 + r;
    vs[r * k1p + c] = (row < n && dev[row] <= bits) ? oz_v(cols, ld, nxy, weighted, row, c) : 0.0;
  }
}

// Per (chunk, pair): the largest |P| over the chunk's regular rows, as the raw exponent
// ex + kExpBias (atomicMax; 2^(ex-1) <= max |P| < 2^ex). Grid: (the group's tiles, pair blocks of
// kPexpPairs): the per-pair accumulators of a block stay within 18 * kPexpPairs bytes of LDS
// whatever the panel's width (p <= 120: e <= 7,503 pairs).
constexpr int kPexpPairs = 1024;
__global__ __launch_bounds__(256) void oz_pexp_kernel(const double* cols, int64_t ld, uint32_t n, int nxy,
                                                      int weighted, int k1, int e, int npp, const int32_t* tile_chunk,
                                                      const int8_t* dev, const int32_t* meta, int32_t* raw,
                                                      unsigned long long* psum) {
  extern __shared__ __attribute__((aligned(16))) double ozs[];
  const int k1p = k1 | 1, tid = threadIdx.x;
  const int q0 = (int)blockIdx.y * kPexpPairs, ne = min(kPexpPairs, e - q0);  // this block's pairs
  double* vs = ozs;               // [64][k1p]
  double* mx = ozs + 64 * k1p;    // [ne]
  int32_t* xs = reinterpret_cast<int32_t*>(mx + ne);  // [ne] exponent sums of the nonzero |P|
  int32_t* xc = xs + ne;                              // [ne] their count
  uint8_t* pa = reinterpret_cast<uint8_t*>(xc + ne);
  uint8_t* pb = pa + ne;
  const uint32_t tile = blockIdx.x;
  const int chunk = tile_chunk[tile], bits = meta[0];
  for (int q = tid; q < ne; q += 256) {
    int a, b;
    oz_pair_cols(q0 + q, k1, &a, &b);
    pa[q] = (uint8_t)a;
    pb[q] = (uint8_t)b;
    mx[q] = 0.0;
    xs[q] = 0;
    xc[q] = 0;
  }
  for (int sub = 0; sub < 4; ++sub) {
    __syncthreads();
    oz_stage(vs, k1p, cols, ld, n, nxy, weighted, k1, dev, bits, (size_t)tile * 256 + sub * 64);
    __syncthreads();
    for (int q = tid; q < ne; q += 256) {
      const int a = pa[q], b = pb[q];
      double m = mx[q];
      int sx = 0, sc = 0;
#pragma unroll 8
      for (int r = 0; r < 64; ++r) {
        const double P = fabs(vs[r * k1p + a] * vs[r * k1p + b]);
        m = fmax(m, P);
        if (P > 0.0) {
          int ex = 0;
          (void)frexp(P, &ex);
          sx += ex;
          ++sc;
        }
      }
      mx[q] = m;
      xs[q] += sx;
      xc[q] += sc;
    }
  }
  for (int q = tid; q < ne; q += 256)
    if (mx[q] > 0.0) {
      int ex = 0;
      (void)frexp(mx[q], &ex);
      const size_t x = (size_t)chunk * npp + q0 + q;
      atomicMax(&raw[x], ex + kExpBias);
      atomicAdd(&psum[2 * x], (unsigned long long)(long long)xs[q]);
      atomicAdd(&psum[2 * x + 1], (unsigned long long)xc[q]);
    }
}

// Digit slices per (chunk, column tile): 6 when every pair of the tile has a narrow range, else 7.
// Dropping the last of the 7 balanced digits moves each product by at most 2^(E-47) (E: the pair's
// chunk exponent, 2^(E-1) <= max |P| < 2^E). Summed over the chunk that is at most 2^(E-47) sum c,
// against the f64 rounding bound n u sum c |P| (u = 2^-53) of summing the same terms in f64; with
// 2^(r-1) <= (geometric mean of the nonzero |P|) <= their mean, r = floor(mean frexp exponent),
// the ratio is at most 2^(E - r + 7) / n. A pair takes six digits when that is <= 1/4:
// E - r <= floor(log2 n) - 9 (n = the group's rows); its seventh digit is then written as zero, so
// its Gram entries do not depend on the other pairs of its tile (a multi-outcome panel's entries
// equal the single-outcome panel's bitwise). A tile whose pairs all take six runs six slices.
// force7 (OB_GRAM_DIGITS=7) keeps seven everywhere. pnsl: [chunk][pair]; nsl: [chunk][column tile].
__global__ __launch_bounds__(256) void oz_nsl_kernel(const int32_t* pexp, const long long* psum, const uint32_t* chunks,
                                                     uint32_t n0, uint32_t n1, int e, int n_ct, int npp, int n_chunks,
                                                     int force7, uint8_t* pnsl, uint8_t* nsl, int32_t* meta) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n_chunks * n_ct) return;
  const int chunk = i / n_ct, ct = i - chunk * n_ct;
  const uint32_t n = chunks[3 * chunk] ? n1 : n0;
  const int thr = n ? (31 - __builtin_clz(n)) - 9 : -1;
  bool all6 = true;
  for (int q = 0; q < kPairsPerTile; ++q) {
    const int pair = ct * kPairsPerTile + q;
    const size_t x = (size_t)chunk * npp + pair;
    bool six = true;  // padding pairs and all-zero pairs are exact in any number of slices
    if (pair < e) {
      const long long sum = psum[2 * x], cnt = psum[2 * x + 1];
      if (force7 || thr < 0) six = false;
      else if (cnt > 0) {
        const long long r = sum >= 0 ? sum / cnt : -((-sum + cnt - 1) / cnt);  // floor
        six = (long long)pexp[x] - r <= thr;
      }
    }
    pnsl[x] = six ? 6 : 7;
    all6 = all6 && six;
  }
  nsl[i] = all6 ? 6 : 7;
  if (all6) atomicAdd(&meta[5], 1);
}

__global__ __launch_bounds__(256) void oz_pexp_finish_kernel(int32_t* pexp, int count) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < count) pexp[i] = pexp[i] ? pexp[i] - kExpBias : 0;
}

// B digits of one 64-row sub-tile for every column tile: grid = the group's sub-tiles. Unit u =
// (column tile, pair block, lane): lane l holds pair 16 nb + (l & 15), rows 16 (l >> 4) + j -- the B
// fragment -- and writes one 16-byte word per slice (consecutive units: consecutive 16 B).
__global__ __launch_bounds__(256) void oz_digits_kernel(const double* cols, int64_t ld, uint32_t n, int nxy,
                                                        int weighted, int k1, int e, int n_ct, int n_pairs_pad,
                                                        const int32_t* tile_chunk, const int8_t* dev,
                                                        const int32_t* meta, const int32_t* pexp, const uint8_t* pnsl,
                                                        ob_v4i* B) {
  extern __shared__ __attribute__((aligned(16))) double ozs[];
  const int k1p = k1 | 1;
  const uint32_t sub = blockIdx.x;
  const int chunk = tile_chunk[sub >> 2];
  oz_stage(ozs, k1p, cols, ld, n, nxy, weighted, k1, dev, meta[0], (size_t)sub * 64);
  __syncthreads();
  for (int u = threadIdx.x; u < n_ct * 128; u += 256) {
    const int ct = u >> 7, nb = (u >> 6) & 1, lane = u & 63;
    const int pair = ct * kPairsPerTile + 16 * nb + (lane & 15);
    int a = 0, b = 0;
    const bool live = pair < e;
    if (live) oz_pair_cols(pair, k1, &a, &b);
    const int E = live ? pexp[(size_t)chunk * n_pairs_pad + pair] : 0;
    const bool six = live && pnsl[(size_t)chunk * n_pairs_pad + pair] == 6;  // digit 6 written as zero
    const double* v0 = ozs + 16 * (lane >> 4) * k1p;
    long long m[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const double P = live ? v0[j * k1p + a] * v0[j * k1p + b] : 0.0;
      m[j] = (long long)rint(ldexp(P, kFracBits - E));  // |m| <= 2^54: exact
    }
    ob_v4i* dst = B + ((size_t)sub * n_ct + ct) * kS * 128 + nb * 64 + lane;
#pragma unroll
    for (int sl = kS - 1; sl >= 0; --sl) {  // balanced digits, least significant first
      uint32_t w[4] = {0u, 0u, 0u, 0u};
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const int8_t d = (int8_t)(m[j] & 0xff);
        w[j >> 2] |= (uint32_t)(uint8_t)d << (8 * (j & 3));
        m[j] = (m[j] - d) >> 8;
      }
      if (sl == kS - 1 && six) w[0] = w[1] = w[2] = w[3] = 0u;
      dst[sl * 128] = (ob_v4i){(int)w[0], (int)w[1], (int)w[2], (int)w[3]};
    }
  }
}

// The exception rows' terms of a segment: gram[rep][g][e] += sum_x c(rep, x) P_x[e] over the
// group's exception rows in list order, zero counts skipped. Grid: (64-replicate batch, group).
// c(rep, row) is byte (j & 15) of A-fragment unit ((tile * nb_rep + batch) * 4 + sub-tile) * 256 +
// (r >> 4) * 64 + (j >> 4) * 16 + (r & 15) (ob_count_kernel<true>; j = row & 63, r = rep & 63).
__global__ __launch_bounds__(256) void oz_exc_kernel(const uint8_t* counts, uint32_t nb_rep, uint32_t tiles0,
                                                     const uint32_t* exc, const double* excp, const int32_t* meta,
                                                     int e, int e_pad, uint32_t n_reps, double* gram) {
  __shared__ uint8_t cnt[64][64];  // [exception][replicate]
  __shared__ double pv[64][64];    // [exception][pair]
  const uint32_t rb = blockIdx.x, g = blockIdx.y;
  const int nx_all = meta[1], na = meta[2];
  const int x0 = g ? na : 0, x1 = g ? nx_all : na;
  if (x0 >= x1) return;
  const int tid = threadIdx.x, el = tid & 63, rq = tid >> 6;
  for (int eb = 0; eb < e; eb += 64) {
    double acc[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = 0.0;
    for (int xb = x0; xb < x1; xb += 64) {
      const int nx = min(64, x1 - xb);
      __syncthreads();
      for (int i = tid; i < 64 * nx; i += 256) {
        const int j = i >> 6, r = i & 63;
        const uint32_t row = exc[xb + j] & 0x7FFFFFFFu, jr = row & 63u;
        const size_t unit = (((size_t)(g ? tiles0 : 0u) + (row >> 8)) * nb_rep + rb) * 1024 + ((row >> 6) & 3u) * 256 +
                            (r >> 4) * 64 + (jr >> 4) * 16 + (r & 15);
        cnt[j][r] = counts[unit * 16 + (jr & 15u)];
        pv[j][r] = eb + r < e ? excp[(size_t)(xb + j) * e_pad + eb + r] : 0.0;
      }
      __syncthreads();
      for (int j = 0; j < nx; ++j) {
        const double pj = pv[j][el];
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const uint32_t c = cnt[j][rq * 16 + i];
          if (c) acc[i] += (double)c * pj;
        }
      }
    }
    if (eb + el < e)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const uint32_t rep = rb * 64u + (uint32_t)(rq * 16 + i);
        if (rep < n_reps) gram[((size_t)rep * 2 + g) * e_pad + eb + el] += acc[i];
      }
  }
}

struct OzArgs {
  const ob_v4i* B0;
  const ob_v4i* B1;
  const ob_v4i* counts;    // I8 count images (ob_count_kernel<true>): [tile][batch][1024 units]
  const uint32_t* chunks;  // [chunk][3] = (group, first tile, end tile)
  const int32_t* pexp;     // [chunk][n_pairs_pad]
  const uint8_t* nsl;      // [chunk][column tile]: 6 or 7 digit slices (oz_nsl_kernel)
  double* partial;         // [chunk][rep_pad][e_pad]
  uint32_t n0, n1, tiles0, nb_rep, n_reps, rep_pad, n_rt;
  int n_ct, e_pad, n_pairs_pad;
  int n_dct;  // oz_gram_w_kernel: column-tile pairs (64 pairs)
  int ksplit;  // oz_gram_w_kernel: 2 = each (chunk, tiles) block pair splits the chunk's sub-tiles
  long long* pint;  // ksplit 2: [half][chunk][rep_pad][e_pad][2] int64 slice-group sums
  int n_chunks;
};

constexpr int kWaves = 8;                         // 2 per SIMD: (replicate batch, slice group)
#ifndef OB_OZ_SUB2
// 1: two 64-row sub-tiles per barrier (one barrier per 128 rows) over an 8-stage ring; 0: one
// sub-tile per barrier over a 4-stage ring
#define OB_OZ_SUB2 1
#endif
constexpr int kNbuf = OB_OZ_SUB2 ? 8 : 4;         // LDS ring stages (sub-tiles)
constexpr int kBDma = (kSubUnits + 64 * kWaves - 1) / (64 * kWaves);  // B DMA instructions per wave (<=)
constexpr int kBDmaTotal = kSubUnits / 64;        // 14 per sub-tile, spread over the waves
constexpr size_t kLdsB = kNbuf * (size_t)kSubUnits * 16;      // B ring (56 KB; 112 KB with OB_OZ_SUB2)
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

// The same DMA with a wave-uniform SGPR base and a per-lane 32-bit offset (global saddr form): the
// address arithmetic stays on the scalar unit, which issues beside the MFMAs.
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
__device__ __forceinline__ void oz_dma16s(uint32_t voff, const void* sbase, uint32_t lds) {
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1" ::"v"(voff), "s"(sbase), "s"(lds)
               : "memory", "m0");
}
#pragma clang diagnostic pop

__device__ __forceinline__ void oz_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

#ifndef OB_OZ_RASTER
#define OB_OZ_RASTER 1
#endif
// Block -> (column tile, replicate tile, chunk). A "group" is the n_ct column tiles of one
// (chunk, replicate tile); its blocks share that tile's count images, so they run on one XCD
// (blocks b and b + 8 share an XCD under round-robin dispatch: speed only, never correctness).
// OB_OZ_RASTER 1: groups are dealt to the 8 XCDs in turn (8 consecutive groups = one "super group"
// of 8 n_ct blocks, group = bid mod 8 inside it), so all XCDs sweep the chunks together and the
// chunk's digit block (47 MB at configs[1]) is re-read from the Infinity Cache by every replicate
// tile. 0: each XCD sweeps a contiguous eighth of the groups (8 chunks in flight at once).
__device__ __forceinline__ void oz_map(const OzArgs& a, uint32_t* ct, uint32_t* rt, uint32_t* chunk) {
  const uint32_t nwg = gridDim.x, bid = blockIdx.x, nct = (uint32_t)a.n_ct;
  uint32_t grp, c;
#if OB_OZ_RASTER
  const uint32_t sgb = 8u * nct, sg = bid / sgb, r = bid - sg * sgb;
  const uint32_t left = nwg - sg * sgb;  // blocks from this super group on
  if (left >= sgb) {
    grp = sg * 8u + (r & 7u);
    c = r >> 3;
  } else {  // the last, partial super group: left / n_ct groups
    const uint32_t ng = left / nct;
    grp = sg * 8u + r % ng;
    c = r / ng;
  }
#else
  const uint32_t xcd = bid & 7u, slot = bid >> 3, q8 = nwg >> 3, r8 = nwg & 7u;
  const uint32_t wi = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + slot;
  grp = wi / nct;
  c = wi - grp * nct;
#endif
  *ct = c;
  *rt = grp % a.n_rt;
  *chunk = grp / a.n_rt;
}

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
// ablations only, wrong results): 2 no MFMAs, 4 no sub-tile loads after the prologue, 8 no barrier,
// 16 the MFMAs on zeroed B fragments (same instructions and traffic, no multiplier toggling: the
// power the data costs).
// MFMA shape: v_mfma_i32_16x16x64_i8 (the 16x16 forms hold a higher clock than the 32x32 forms on
// random operands at equal cycles per op, MI355X_MICROARCH.md 'DVFS give-back' item 7). Lane l of
// an A fragment holds replicate 16 m + (l & 15), rows 16 (l >> 4) + j of the sub-tile; lane l of a B
// fragment pair 16 h + (l & 15) of the column tile, the same rows; D: pair 16 h + (l & 15),
// replicates 16 m + 4 (l >> 4) + i.
template <int NQ, int SLO, int NB, bool LIVE, int DIAG>
__device__ __forceinline__ void oz_gram_body(const OzArgs& a, unsigned char* smem, int wave) {
  constexpr int PER = NB + (LIVE ? 4 : 0);  // this wave's vector-memory ops per sub-tile
  const ob_v4i* bs = reinterpret_cast<const ob_v4i*>(smem);  // [kNbuf][kSubUnits]
  const int lane = threadIdx.x & 63;
  const int wb = wave & 3, grp = wave >> 2;  // replicate batch in the tile, slice group
  constexpr int slo = SLO;                    // this wave's first slice
  // XCD-aware remap (as ob_gram_kernel's map_work): consecutive work items -- the column tiles of
  // one replicate tile, then the replicate tiles of one chunk -- share an XCD's L2.
  uint32_t ctu, rt, chunk;
  oz_map(a, &ctu, &rt, &chunk);
  const int ct = (int)ctu;
  const uint32_t g = a.chunks[3 * chunk];
  const uint32_t n = g ? a.n1 : a.n0, tg0 = g ? a.tiles0 : 0u;
  const uint32_t s0 = a.chunks[3 * chunk + 1] * 4u;
  // OB_OZ_SUB2: an odd sub-tile count (a group's last chunk) runs one padding sub-tile more, whose
  // count image and digits exist (tiles are 4 sub-tiles, s0 a multiple of 4) and hold zeros
  const uint32_t s1 = OB_OZ_SUB2 ? (min(a.chunks[3 * chunk + 2] * 4u, (n + 63u) >> 6) + 1u) & ~1u
                                 : min(a.chunks[3 * chunk + 2] * 4u, (n + 63u) >> 6);
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
    if constexpr (DIAG & 16) {
      int z;
      asm volatile("v_mov_b32 %0, 0" : "=v"(z));  // opaque zero: the reads and MFMAs stay
#pragma unroll
      for (int q = 0; q < NQ; ++q) bf[q] &= z;
    }
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
  // PER in flight. Every step issues the same loads (past the end: the last sub-tile again, into a
  // stage nobody reads, and a dead A slot), so every step waits the same count and the wait
  // pattern is a property of the code, not of the chunk length (tools/isa_vmem_check.py checks it
  // on the built ISA: no DMA older than two barriers at a barrier, no register of an un-waited load
  // touched). Round 4 measured the alternatives to this schedule and kept none.
  auto step = [&](uint32_t s, auto J) {
    constexpr int j = decltype(J)::value;
    const int buf = (int)((s - s0) & (kNbuf - 1));
    if constexpr (LIVE) {
      read(buf, 1, fb1);
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (!(DIAG & 2)) oz_mfmas<NQ>(acc, 0, ar[j], fb0);
      __builtin_amdgcn_sched_barrier(0);
    }
    if constexpr (DIAG & 4) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PER) : "memory");
    if constexpr (DIAG & 8) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // timing only: no barrier
    else oz_barrier();
    if constexpr (!(DIAG & 4)) dma(buf, min(s + kNbuf, s1 - 1));
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
  // groups of three steps, then the one or two left: every step, the tail's included, issues the
  // same loads and waits, so each path through the loop presents the same queue at each barrier.
  // (Ghost steps past the end with branch-guarded MFMAs, the round-4 first form, read 5 GB more
  // per launch and ran 1.5 % slower: profiles/r04_ab_gram_tail.txt.)
#if OB_OZ_SUB2
  // Two sub-tiles (s, s + 1) per barrier. Sub-tile u uses A slot (u - s0) % 3 and ring stage
  // (u - s0) % 8. Order: MFMAs (s, 0) | read (s, 1); MFMAs (s, 1) | read (s + 1, 0); A(s + 3) into
  // s's slot; MFMAs (s + 1, 0) | read (s + 1, 1); wait + barrier: stages s + 2, s + 3 landed (their
  // DMA was issued three barriers earlier), every read of s, s + 1 done; refill those two stages
  // with s + 8, s + 9; read (s + 2, 0); MFMAs (s + 1, 1); A(s + 4) into s + 1's slot. Newer than the
  // DMA of s + 2, s + 3 at the barrier: A(s - 2); A(s - 1), 2 NB DMA, A(s); A(s + 1), 2 NB DMA,
  // A(s + 2); A(s + 3) = 24 + 4 NB (LIVE) or 4 NB loads.
  constexpr int PER2 = 4 * NB + (LIVE ? 24 : 0);
  auto step2 = [&](uint32_t s, auto J0, auto J1) {
    constexpr int j0 = decltype(J0)::value, j1 = decltype(J1)::value;
    const int b0 = (int)((s - s0) & (kNbuf - 1)), b1 = (b0 + 1) & (kNbuf - 1), b2 = (b0 + 2) & (kNbuf - 1);
    if constexpr (LIVE) {
      read(b0, 1, fb1);
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (!(DIAG & 2)) oz_mfmas<NQ>(acc, 0, ar[j0], fb0);
      __builtin_amdgcn_sched_barrier(0);
      read(b1, 0, fb0);
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (!(DIAG & 2)) oz_mfmas<NQ>(acc, 1, ar[j0], fb1);
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (!(DIAG & 4)) aload(ar[j0], min(s + 3, s1 - 1));
      read(b1, 1, fb1);
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (!(DIAG & 2)) oz_mfmas<NQ>(acc, 0, ar[j1], fb0);
      __builtin_amdgcn_sched_barrier(0);
    }
    if constexpr (DIAG & 4) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PER2) : "memory");
    oz_barrier();
    if constexpr (!(DIAG & 4)) {
      dma(b0, min(s + kNbuf, s1 - 1));
      dma(b1, min(s + kNbuf + 1, s1 - 1));
    }
    if constexpr (LIVE) {
      read(b2, 0, fb0);
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (!(DIAG & 2)) oz_mfmas<NQ>(acc, 1, ar[j1], fb1);
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (!(DIAG & 4)) aload(ar[j1], min(s + 4, s1 - 1));
    }
  };
  uint32_t s = s0;  // s1 - s0 is even here
  for (; s + 6 <= s1; s += 6) {
    step2(s, IC<0>{}, IC<1>{});
    step2(s + 2, IC<2>{}, IC<0>{});
    step2(s + 4, IC<1>{}, IC<2>{});
  }
  if (s < s1) step2(s, IC<0>{}, IC<1>{});
  if (s + 2 < s1) step2(s + 2, IC<2>{}, IC<0>{});
#else
  uint32_t s = s0;
  for (; s + 3 <= s1; s += 3) {
    step(s, IC<0>{});
    step(s + 1, IC<1>{});
    step(s + 2, IC<2>{});
  }
  if (s < s1) step(s, IC<0>{});
  if (s + 1 < s1) step(s + 1, IC<1>{});
#endif
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
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the trailing DMAs (past the end) have landed
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
  uint32_t ct, rt, chunk;
  oz_map(a, &ct, &rt, &chunk);
  const bool live = rt * 4u + (uint32_t)(wave & 3) < a.nb_rep;
  const bool six = a.nsl[chunk * (uint32_t)a.n_ct + ct] == 6;
  // B piece t of wave w is 8 t + w. Waves 0-3: slices 0-3, two B pieces; 4-5: slices 4-6, two B pieces; 6-7: slices 4-6, one piece.
  // Six slices: waves 0-3 take slices 0 .. kSix0 - 1, waves 4-7 the rest of 0-5, one piece each;
  // pieces 12-13 (slice 6) are not loaded.
  if (six) {
    if (wave < 4) {
      if (live) oz_gram_body<kSix0, 0, 2, true, DIAG>(a, smem, wave);
      else oz_gram_body<kSix0, 0, 2, false, DIAG>(a, smem, wave);
    } else {
      if (live) oz_gram_body<6 - kSix0, kSix0, 1, true, DIAG>(a, smem, wave);
      else oz_gram_body<6 - kSix0, kSix0, 1, false, DIAG>(a, smem, wave);
    }
  } else if (wave < 4) {
    if (live) oz_gram_body<kSlo, 0, 2, true, DIAG>(a, smem, wave);
    else oz_gram_body<kSlo, 0, 2, false, DIAG>(a, smem, wave);
  } else if (wave < 6) {
    if (live) oz_gram_body<kS - kSlo, kSlo, 2, true, DIAG>(a, smem, wave);
    else oz_gram_body<kS - kSlo, kSlo, 2, false, DIAG>(a, smem, wave);
  } else {
    if (live) oz_gram_body<kS - kSlo, kSlo, 1, true, DIAG>(a, smem, wave);
    else oz_gram_body<kS - kSlo, kSlo, 1, false, DIAG>(a, smem, wave);
  }
}

// ---------------------------------------------------------------------------------------------
// Wide tile (round 6): one wave per SIMD, a block = 4 waves = (chunk, 256 replicates, 64 pairs),
// per 64-row sub-tile 4 replicate batches x 6 slices x 4 pair blocks = 384 v_mfma_i32_16x16x64_i8
// against 16 KB of A (the four batches' count fragments) and 24 KB of B (both column tiles' six
// slices), all by LDS-DMA into a 4-stage ring, one barrier per sub-tile. The block tile is twice the
// 8-wave kernel's, so each operand byte meets twice the MFMAs: 40 KB per 384 MFMAs against 44 KB per
// 192. 384 accumulator registers per wave (256 in AGPRs). The waves split the tile as a 2 x 2 grid
// (oz_gram_w2_body). The slice sums meet exactly as in oz_gram_body (slices 0-3 and 4-5 / 4-6 in
// int64, one rounding each, then their sum): the partials are bitwise the 8-wave kernel's. A
// column-tile pair whose tiles do not both run six slices takes its tiles one pass each (NH = 2).
// (Round 6 first ran the tile as 1 x 4 -- wave w = replicate batch w x all 64 pairs -- with the
// same ring and interleaved schedule: 4 A + 24 B fragment reads per 96 MFMAs against the grid's
// 8 + 12, 5 % slower; removed after the grid)
// ---------------------------------------------------------------------------------------------
#ifndef OB_OZ_W_NBUF
#define OB_OZ_W_NBUF 4
#endif
constexpr int kWNbuf = OB_OZ_W_NBUF;  // ring stages (sub-tiles): 4 x 40 KB fill the 160 KB of LDS
constexpr int kWAgprTiles = 64;  // accumulator tiles (4 registers each) pinned to AGPRs
// 4 stages of B (two six-slice tiles: 24 KB; one seven-slice tile: 14 KB) + A (16 KB)
constexpr size_t kWLds = kWNbuf * (size_t)(2 * 6 * 2 * 64 + 4 * 4 * 64) * 16;

#ifndef OB_OZ_W_AFIRST
#define OB_OZ_W_AFIRST 0  // 1: after the barrier, read the next step's A 0..3 with its first B block
#endif
#ifndef OB_OZ_W_SPLIT
#define OB_OZ_W_SPLIT 1  // the engine may split a wide launch's chunks over two blocks (oz_gram_mode)
#endif
#ifndef OB_OZ_W_RASTER
#define OB_OZ_W_RASTER 0
#endif
// Block -> (column-tile pair, replicate tile, chunk); a group is the n_dct blocks of one (chunk,
// replicate tile) and shares that tile's count images. OB_OZ_W_RASTER 0: each XCD sweeps a
// contiguous eighth of the groups, so its 32 CUs hold 32 / n_dct consecutive replicate tiles of
// one chunk at once and read each B sub-tile of the chunk from L2 that many times per fetch;
// 1: oz_map's chunk-major deal of groups over the XCDs (every XCD streams the chunk's B).
__device__ __forceinline__ void oz_map_w(const OzArgs& a, uint32_t* dct, uint32_t* rt, uint32_t* chunk) {
  // ksplit 2: blocks 2i and 2i + 1 are the two halves of work item i (different XCDs)
  const uint32_t nwg = gridDim.x / (uint32_t)a.ksplit, bid = blockIdx.x / (uint32_t)a.ksplit, nct = (uint32_t)a.n_dct;
  uint32_t grp, c;
#if OB_OZ_W_RASTER
  const uint32_t sgb = 8u * nct, sg = bid / sgb, r = bid - sg * sgb;
  const uint32_t left = nwg - sg * sgb;
  if (left >= sgb) {
    grp = sg * 8u + (r & 7u);
    c = r >> 3;
  } else {
    const uint32_t ng = left / nct;
    grp = sg * 8u + r % ng;
    c = r / ng;
  }
#else
  const uint32_t xcd = bid & 7u, slot = bid >> 3, q8 = nwg >> 3, r8 = nwg & 7u;
  const uint32_t wi = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + slot;
  grp = wi / nct;
  c = wi - grp * nct;
#endif
  *dct = c;
  *rt = grp % a.n_rt;
  *chunk = grp / a.n_rt;
}

// NS digit slices (6 or 7), NH 16-pair blocks per pass (4: column tiles ct0, ct0 + 1; 2: ct0 only),
// NB this wave's B DMA pieces per sub-tile. The waves as a 2 x 2 grid: wave w = (wr = w & 1,
// wc = w >> 1) owns replicate batches 2 wr, 2 wr + 1 (8 replicate blocks) and pair blocks
// wc NHW .. wc NHW + NHW - 1 (NHW = NH / 2: column tile ct0 + wc when NH = 4, one half of ct0 when
// NH = 2): per sub-tile 8 A and NHW NS B fragment reads for its 8 x NS x NHW MFMAs (20 reads per 96
// MFMAs; a 1 x 4 split needs 28, and the B reads are what the gram_diag 128 ablation found costly).
// Wave w DMAs B pieces t * 4 + w and its own batch w's A (DLIVE: batch w exists); the step DMAs
// sub-tile t + 3 into the stage freed at barrier t - 1, one or two instructions after each slice's
// MFMAs before the barrier (address arithmetic on the scalar unit, in the MFMAs' shadow), and the
// stage published at barrier t was issued before barrier t - 2, so the wait is vmcnt((N - 2) T) for
// N stages, the same at every step (past the end the last sub-tile is fetched again). A step is 2 NHW
// units (pair block h, replicate half mh) of 4 NS MFMAs, h-major; the last unit (the last two when
// NHW = 2) runs after the barrier and reads the next sub-tile's first B block and A. MLIVE: batch
// 2 wr exists (the wave computes; a dead second batch computes on stale LDS and is never stored).
template <int NS, int NH, int NB, bool DLIVE, bool MLIVE, int DIAG>
__device__ __forceinline__ void oz_gram_w2_body(const OzArgs& a, unsigned char* smem, int wave, uint32_t ct0,
                                                uint32_t rt, uint32_t chunk) {
  constexpr int NHW = NH / 2;                // pair blocks per wave
  constexpr int U = 2 * NHW;                 // units per step
  constexpr int POST = NHW > 1 ? 2 : 1;      // units after the barrier
  constexpr int NC = NH / 2;
  constexpr int PIECES = NC * NS * 2;
  constexpr int STAGE_B = PIECES * 64;
  constexpr int STAGE = STAGE_B + 4 * 4 * 64;
  constexpr int T = NB + (DLIVE ? 4 : 0);
  constexpr int PER = (kWNbuf - 2) * T;
  constexpr int PRE_SLOTS = (U - POST) * NS;  // DMA slots before the barrier
  static_assert(PRE_SLOTS >= 1, "at least one unit before the barrier");
  const ob_v4i* bs = reinterpret_cast<const ob_v4i*>(smem);
  const int lane = threadIdx.x & 63;
  const int wr = wave & 1, wc = wave >> 1;
  const uint32_t g = a.chunks[3 * chunk];
  const uint32_t n = g ? a.n1 : a.n0, tg0 = g ? a.tiles0 : 0u;
  const uint32_t c0 = a.chunks[3 * chunk + 1] * 4u;
  const uint32_t c1 = min(a.chunks[3 * chunk + 2] * 4u, (n + 63u) >> 6);
  // ksplit 2: this block takes half `half` of the chunk's sub-tiles (integer slice sums add exactly)
  const uint32_t half = blockIdx.x % (uint32_t)a.ksplit, cmid = c0 + (c1 - c0) / 2u;
  const uint32_t s0 = a.ksplit == 1 ? c0 : (half ? cmid : c0);
  const uint32_t s1 = a.ksplit == 1 ? c1 : (half ? c1 : cmid);
  const ob_v4i* Bg = g ? a.B1 : a.B0;
  const uint32_t dbatch = rt * 4u + (uint32_t)wave;  // the batch whose A this wave DMAs
  auto dma = [&](int buf, uint32_t s, auto LO, auto HI) {
    constexpr int lo = decltype(LO)::value, hi = decltype(HI)::value;
#pragma unroll
    for (int t = lo; t < hi; ++t) {
      if (t < NB) {
        const int piece = t * 4 + wave, c = piece / (NS * 2), q = piece - c * (NS * 2);
        const ob_v4i* src = Bg + ((size_t)s * a.n_ct + ct0 + c) * kSubUnits + q * 64;
        oz_dma16(src + lane, (uint32_t)(buf * STAGE + piece * 64) * 16u);
      } else {
        const int m = t - NB;
        const ob_v4i* src_a = a.counts + (((size_t)(tg0 + (s >> 2)) * a.nb_rep + dbatch) * 4 + (s & 3)) * 256;
        oz_dma16(src_a + m * 64 + lane, (uint32_t)(buf * STAGE + STAGE_B + (wave * 4 + m) * 64) * 16u);
      }
    }
  };
  auto dma1 = [&](int buf, uint32_t s, auto TT) {
    constexpr int t = decltype(TT)::value;
    if constexpr (t < NB) {
      const int piece = t * 4 + wave, c = piece / (NS * 2), q = piece - c * (NS * 2);
      const ob_v4i* src = Bg + ((size_t)s * a.n_ct + ct0 + c) * kSubUnits + q * 64;
      oz_dma16s((uint32_t)lane * 16u, src, (uint32_t)(buf * STAGE + piece * 64) * 16u);
    } else {
      constexpr int m = t - NB;
      const ob_v4i* src_a = a.counts + (((size_t)(tg0 + (s >> 2)) * a.nb_rep + dbatch) * 4 + (s & 3)) * 256 + m * 64;
      oz_dma16s((uint32_t)lane * 16u, src_a, (uint32_t)(buf * STAGE + STAGE_B + (wave * 4 + m) * 64) * 16u);
    }
  };
  // this wave's 8 A fragments: batches 2 wr, 2 wr + 1, blocks 0..3 each
  auto aread1 = [&](int buf, int m) { return bs[buf * STAGE + STAGE_B + (8 * wr + m) * 64 + lane]; };
  // B fragment q of this wave's pair block h
  auto bread1 = [&](int buf, int h, int q) {
    const int hg = wc * NHW + h;
    return bs[buf * STAGE + ((hg >> 1) * NS * 2 + (hg & 1)) * 64 + q * 128 + lane];
  };
  ob_v4i ar[2][8];
  ob_v4i fb[2][NS];
  ob_v4i acc[8][NS][NHW];
#pragma unroll
  for (int m = 0; m < 8; ++m)
#pragma unroll
    for (int q = 0; q < NS; ++q)
#pragma unroll
      for (int h = 0; h < NHW; ++h) acc[m][q][h] = (ob_v4i){};
  auto mfma1 = [&](int m, int q, int h, const ob_v4i& af, const ob_v4i& bf) {
    if ((m * NS + q) * NHW + h < kWAgprTiles)
      asm volatile("v_mfma_i32_16x16x64_i8 %0, %1, %2, %0" : "+a"(acc[m][q][h]) : "v"(af), "v"(bf));
    else
      asm volatile("v_mfma_i32_16x16x64_i8 %0, %1, %2, %0" : "+v"(acc[m][q][h]) : "v"(af), "v"(bf));
  };
  constexpr int AHEAD = kWNbuf - 1;
#pragma unroll
  for (int j = 0; j < AHEAD; ++j)
    if (s0 + j < s1) dma(j, s0 + j, IC<0>{}, IC<T>{});
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (MLIVE && s0 < s1) {
#pragma unroll
    for (int q = 0; q < NS; ++q) fb[0][q] = bread1(0, 0, q);
#pragma unroll
    for (int m = 0; m < 8; ++m) ar[0][m] = aread1(0, m);
  }
  // unit u = (h = u >> 1, mh = u & 1) of a step with parity j: 4 NS MFMAs on ar[j][4 mh ..] and
  // fb[(h + j NHW) & 1]; slot q (after the 4 MFMAs of slice q) issues this unit's reads and DMAs
  auto unit = [&](auto J, auto UU, int buf, int bnext, uint32_t snext) {
    constexpr int j = decltype(J)::value, u = decltype(UU)::value;
    constexpr int h = u >> 1, mh = u & 1;
    constexpr int fcur = (h + j * NHW) & 1, fnext = (h + 1 + j * NHW) & 1;
    constexpr bool pre = u < U - POST;
    auto slot = [&](auto Q) {
      constexpr int q = decltype(Q)::value;
#pragma unroll
      for (int m = 0; m < 4; ++m) mfma1(4 * mh + m, q, h, ar[j][4 * mh + m], fb[fcur][q]);
      if constexpr (pre) {
        // the next pair block of this sub-tile, during its first unit; the step's DMAs one or two per slot
        if constexpr (mh == 0 && h + 1 < NHW && !(DIAG & 128)) fb[fnext][q] = bread1(buf, h + 1, q);
        constexpr int k = u * NS + q;  // slot index before the barrier
        if constexpr (k < T && !(DIAG & 4)) dma1(bnext, snext, IC<k>{});
        if constexpr (k + PRE_SLOTS < T && !(DIAG & 4)) dma1(bnext, snext, IC<k + PRE_SLOTS>{});
      } else {
        // after the barrier: the next sub-tile's first B block, then its A
        constexpr int pu = u - (U - POST);  // 0 .. POST - 1
        const int nbuf = (buf + 1) % kWNbuf;
        constexpr bool rb = !(DIAG & 128), ra = !(DIAG & 256);  // timing ablations: no B / A reads
        if constexpr (POST == 2 && OB_OZ_W_AFIRST) {
          // in the order the next step needs them: A 0..3 and its first B block in the first unit,
          // A 4..7 (its second replicate half) in the second
          if constexpr (pu == 0) {
            if constexpr (ra && q < 4) ar[j ^ 1][q] = aread1(nbuf, q);
            if constexpr (rb) fb[fnext][q] = bread1(nbuf, 0, q);
          } else if constexpr (ra && q < 4) {
            ar[j ^ 1][q + 4] = aread1(nbuf, q + 4);
          }
        } else if constexpr (POST == 2) {
          if constexpr (pu == 0) {
            if constexpr (rb) fb[fnext][q] = bread1(nbuf, 0, q);
          } else if constexpr (ra) {
            ar[j ^ 1][q] = aread1(nbuf, q);
            if constexpr (q + NS < 8) ar[j ^ 1][q + NS] = aread1(nbuf, q + NS);
          }
        } else {
          if constexpr (rb) fb[fnext][q] = bread1(nbuf, 0, q);
          if constexpr (ra) {
            ar[j ^ 1][q] = aread1(nbuf, q);
            if constexpr (q + NS < 8) ar[j ^ 1][q + NS] = aread1(nbuf, q + NS);
          }
        }
      }
    };
    __builtin_amdgcn_sched_barrier(0);
    slot(IC<0>{}); slot(IC<1>{}); slot(IC<2>{}); slot(IC<3>{}); slot(IC<4>{}); slot(IC<5>{});
    if constexpr (NS > 6) slot(IC<6>{});
    __builtin_amdgcn_sched_barrier(0);
  };
  static_assert(2 * PRE_SLOTS >= T, "the pre-barrier slots hold every DMA of a step");
  auto step = [&](uint32_t s, auto J) {
    const int buf = (int)((s - s0) % kWNbuf);
    const uint32_t snext = min(s + AHEAD, s1 - 1);
    const int bnext = (buf + AHEAD) % kWNbuf;
    if constexpr (MLIVE && !(DIAG & 2)) {
      unit(J, IC<0>{}, buf, bnext, snext);
      if constexpr (U - POST > 1) unit(J, IC<1>{}, buf, bnext, snext);
      if constexpr (DIAG & 4) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PER) : "memory");
      if constexpr (DIAG & 8) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // timing only: no barrier
      else oz_barrier();
      if constexpr (POST == 2) {
        unit(J, IC<U - 2>{}, buf, bnext, snext);
        unit(J, IC<U - 1>{}, buf, bnext, snext);
      } else {
        unit(J, IC<U - 1>{}, buf, bnext, snext);
      }
      return;
    }
    // dead waves (and gram_diag 2): no MFMAs, the step's DMA in one burst before the barrier
    if constexpr (!(DIAG & 4)) dma(bnext, snext, IC<0>{}, IC<T>{});
    if constexpr (DIAG & 4) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PER) : "memory");
    if constexpr (DIAG & 8) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // as the live waves
    else oz_barrier();
  };
  uint32_t s = s0;
  for (; s + 2 <= s1; s += 2) {
    step(s, IC<0>{});
    step(s + 1, IC<1>{});
  }
  if (s < s1) step(s, IC<0>{});
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if constexpr (MLIVE) {
    // slices -> f64 exactly as oz_gram_body: slices 0-3 and 4 .. NS - 1 each in int64, one ldexp each, then
    // their sum; four replicate blocks at a time through this wave's quarter of the ring (a lane reads
    // back only its own words), so the int64 arithmetic never holds every accumulator in VGPRs at once
    ob_v4i* st = reinterpret_cast<ob_v4i*>(smem) + (size_t)wave * (4 * NS * 64);
#pragma unroll
    for (int h = 0; h < NHW; ++h) {
      const int hg = wc * NHW + h;
      const int pair = (int)(ct0 + (hg >> 1)) * kPairsPerTile + 16 * (hg & 1) + (lane & 15);
      const int E = a.pexp[chunk * a.n_pairs_pad + min(pair, a.n_pairs_pad - 1)];
      const int sh0 = E - kFracBits + 8 * (kS - 0 - kSlo), sh1 = E - kFracBits + 8 * (kS - kSlo - (NS - kSlo));
#pragma unroll
      for (int mh = 0; mh < 2; ++mh) {
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int m = 0; m < 4; ++m)
#pragma unroll
          for (int q = 0; q < NS; ++q) st[(m * NS + q) * 64 + lane] = acc[4 * mh + m][q][h];
        __builtin_amdgcn_sched_barrier(0);
        const uint32_t batch = rt * 4u + 2u * (uint32_t)wr + (uint32_t)mh;
#pragma unroll
        for (int m = 0; m < 4; ++m)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            long long p0 = 0, p1 = 0;
#pragma unroll
            for (int q = 0; q < kSlo; ++q) p0 = p0 * 256 + st[(m * NS + q) * 64 + lane][i];
#pragma unroll
            for (int q = kSlo; q < NS; ++q) p1 = p1 * 256 + st[(m * NS + q) * 64 + lane][i];
            const uint32_t rep = batch * 64u + (uint32_t)(16 * m + 4 * (lane >> 4) + i);
            if (pair < a.e_pad && rep < a.n_reps) {
              if (a.ksplit == 1) {
                a.partial[((size_t)chunk * a.rep_pad + rep) * a.e_pad + pair] = ldexp((double)p0, sh0) + ldexp((double)p1, sh1);
              } else {  // the two halves meet in oz_split_combine_kernel, in int64, before the roundings
                long long* d = a.pint + ((((size_t)half * a.n_chunks + chunk) * a.rep_pad + rep) * a.e_pad + pair) * 2;
                d[0] = p0;
                d[1] = p1;
              }
            }
          }
      }
    }
  }
  __syncthreads();
}

template <int NS, int NH, bool DLIVE, bool MLIVE, int DIAG>
__device__ __forceinline__ void oz_gram_w2_pass(const OzArgs& a, unsigned char* smem, int wave, uint32_t ct0,
                                                uint32_t rt, uint32_t chunk) {
  constexpr int P = (NH / 2) * NS * 2;
  if (wave < P % 4 || P % 4 == 0) oz_gram_w2_body<NS, NH, (P + 3) / 4, DLIVE, MLIVE, DIAG>(a, smem, wave, ct0, rt, chunk);
  else oz_gram_w2_body<NS, NH, P / 4, DLIVE, MLIVE, DIAG>(a, smem, wave, ct0, rt, chunk);
}

template <int NS, int NH, int DIAG>
__device__ __forceinline__ void oz_gram_w_pass_live(const OzArgs& a, unsigned char* smem, int wave, uint32_t ct0,
                                                    uint32_t rt, uint32_t chunk, bool live) {
  const bool mlive = rt * 4u + 2u * (uint32_t)(wave & 1) < a.nb_rep;
  if (live && mlive) oz_gram_w2_pass<NS, NH, true, true, DIAG>(a, smem, wave, ct0, rt, chunk);
  else if (live) oz_gram_w2_pass<NS, NH, true, false, DIAG>(a, smem, wave, ct0, rt, chunk);
  else if (mlive) oz_gram_w2_pass<NS, NH, false, true, DIAG>(a, smem, wave, ct0, rt, chunk);
  else oz_gram_w2_pass<NS, NH, false, false, DIAG>(a, smem, wave, ct0, rt, chunk);
}

template <int DIAG>
__global__ __launch_bounds__(256, 1) __attribute__((amdgpu_waves_per_eu(1, 1))) void oz_gram_w_kernel(const OzArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  uint32_t dct, rt, chunk;
  oz_map_w(a, &dct, &rt, &chunk);
  const bool live = rt * 4u + (uint32_t)wave < a.nb_rep;
  const uint32_t ct0 = 2u * dct;
  const bool two = (int)ct0 + 1 < a.n_ct;
  const bool six0 = a.nsl[chunk * (uint32_t)a.n_ct + ct0] == 6;
  const bool six1 = two && a.nsl[chunk * (uint32_t)a.n_ct + ct0 + 1] == 6;
  if (two && six0 && six1) {
    oz_gram_w_pass_live<6, 4, DIAG>(a, smem, wave, ct0, rt, chunk, live);
    return;
  }
  // a seven-slice tile (or a lone last tile): one column tile per pass
  if (six0) oz_gram_w_pass_live<6, 2, DIAG>(a, smem, wave, ct0, rt, chunk, live);
  else oz_gram_w_pass_live<7, 2, DIAG>(a, smem, wave, ct0, rt, chunk, live);
  if (!two) return;
  if (six1) oz_gram_w_pass_live<6, 2, DIAG>(a, smem, wave, ct0 + 1, rt, chunk, live);
  else oz_gram_w_pass_live<7, 2, DIAG>(a, smem, wave, ct0 + 1, rt, chunk, live);
}

}  // namespace

namespace ob {

// Build (once per panel, on stream s) the digit images, the pair exponents and the exception
// rows for the panel's chunking (p->chunks, already in p->d_chunks). Returns OB_OK with
// p->oz_state = 1, or OB_OK with p->oz_state = -1 when the digit images would not fit (the
// caller keeps the f64 MFMA Gram). Enqueue only: nothing here waits for the device.
int oz_prepare(ob_panel* p, hipStream_t s) {
  if (p->oz_state != 0) return OB_OK;
  // exact int32 slice sums need 128 x (a chunk's draws) < 2^31: a group's draws bound a chunk's
  if (p->n[0] >= (1u << 24) || p->n[1] >= (1u << 24) || p->k1 > kOzMaxK1 || !p->chunks_ready) {
    p->oz_state = -1;
    return OB_OK;
  }
  const std::vector<uint32_t>& chunks = p->chunks;
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
  for (int g = 0; g < 2; ++g) {
    if (!p->d_oz_b[g])
      OZ_HIP(hipMalloc(&p->d_oz_b[g], std::max<size_t>((size_t)(p->ld[g] >> 6) * n_ct * kSubUnits * 16, 16)));
    if (!p->d_oz_dev[g]) OZ_HIP(hipMalloc(&p->d_oz_dev[g], std::max<size_t>((size_t)p->ld[g], 1)));
    if (!p->d_oz_tile_chunk[g]) OZ_HIP(hipMalloc(&p->d_oz_tile_chunk[g], sizeof(int32_t) * std::max(p->ntiles[g], 1u)));
    p->oz_tile_chunk[g].assign(std::max(p->ntiles[g], 1u), 0);
  }
  if (!p->d_oz_pexp) OZ_HIP(hipMalloc(&p->d_oz_pexp, sizeof(int32_t) * (size_t)n_chunks * npp));
  if (!p->d_oz_psum) OZ_HIP(hipMalloc(&p->d_oz_psum, sizeof(int64_t) * 2 * (size_t)n_chunks * npp));
  if (!p->d_oz_nsl) OZ_HIP(hipMalloc(&p->d_oz_nsl, (size_t)n_chunks * n_ct));
  if (!p->d_oz_pnsl) OZ_HIP(hipMalloc(&p->d_oz_pnsl, (size_t)n_chunks * npp));
  if (!p->d_oz_acc) OZ_HIP(hipMalloc(&p->d_oz_acc, sizeof(int64_t) * 2 * (size_t)n_chunks * p->k1));
  if (!p->d_oz_meta) OZ_HIP(hipMalloc(&p->d_oz_meta, sizeof(int32_t) * kMetaWords));
  if (!p->d_oz_exc) OZ_HIP(hipMalloc(&p->d_oz_exc, sizeof(uint32_t) * kOzExcCap));
  if (!p->d_oz_excp) OZ_HIP(hipMalloc(&p->d_oz_excp, sizeof(double) * kOzExcCap * (size_t)p->e_pad));
  for (int i = 0; i < 2; ++i)
    if (!p->oz_ev[i]) OZ_HIP(hipEventCreate(&p->oz_ev[i]));
  for (int c = 0; c < n_chunks; ++c)
    for (uint32_t t = chunks[3 * c + 1]; t < chunks[3 * c + 2]; ++t) p->oz_tile_chunk[chunks[3 * c]][t] = c;

  OZ_HIP(hipEventRecord(p->oz_ev[0], s));
  for (int g = 0; g < 2; ++g)
    OZ_HIP(hipMemcpyAsync(p->d_oz_tile_chunk[g], p->oz_tile_chunk[g].data(), sizeof(int32_t) * p->oz_tile_chunk[g].size(),
                          hipMemcpyHostToDevice, s));
  OZ_HIP(hipMemsetAsync(p->d_oz_acc, 0, sizeof(int64_t) * 2 * (size_t)n_chunks * p->k1, s));
  OZ_HIP(hipMemsetAsync(p->d_oz_meta, 0, sizeof(int32_t) * kMetaWords, s));
  OZ_HIP(hipMemsetAsync(p->d_oz_pexp, 0, sizeof(int32_t) * (size_t)n_chunks * npp, s));
  OZ_HIP(hipMemsetAsync(p->d_oz_psum, 0, sizeof(int64_t) * 2 * (size_t)n_chunks * npp, s));
  OZ_HIP(hipMemsetAsync(p->d_oz_exc, 0xFF, sizeof(uint32_t) * kOzExcCap, s));
  const int nxy = p->p + p->n_y;
  const double* cols[2] = {p->d_cols[0], p->d_cols[1]};
  for (int g = 0; g < 2; ++g)
    if (p->ntiles[g]) {
      hipLaunchKernelGGL(oz_scale_kernel, dim3(p->ntiles[g]), dim3(256), 0, s, cols[g], p->ld[g], p->n[g], nxy,
                         p->weighted, p->k1, (const int32_t*)p->d_oz_tile_chunk[g],
                         reinterpret_cast<unsigned long long*>(p->d_oz_acc));
      OZ_HIP(hipGetLastError());
    }
  for (int g = 0; g < 2; ++g)
    if (p->ntiles[g]) {
      hipLaunchKernelGGL(oz_dev_kernel, dim3(p->ntiles[g]), dim3(256), 0, s, cols[g], p->ld[g], p->n[g], nxy,
                         p->weighted, p->k1, (const int32_t*)p->d_oz_tile_chunk[g], (const long long*)p->d_oz_acc,
                         p->d_oz_dev[g], p->d_oz_meta);
      OZ_HIP(hipGetLastError());
    }
  hipLaunchKernelGGL(oz_choose_kernel, dim3(1), dim3(64), 0, s, p->d_oz_meta);
  OZ_HIP(hipGetLastError());
  for (int g = 0; g < 2; ++g)
    if (p->ntiles[g]) {
      hipLaunchKernelGGL(oz_collect_kernel, dim3(p->ntiles[g]), dim3(256), 0, s, (const int8_t*)p->d_oz_dev[g], p->n[g],
                         (uint32_t)g, p->d_oz_meta, p->d_oz_exc);
      OZ_HIP(hipGetLastError());
    }
  hipLaunchKernelGGL(oz_sort_kernel, dim3(1), dim3(1024), 0, s, p->d_oz_exc, p->d_oz_meta);
  OZ_HIP(hipGetLastError());
  hipLaunchKernelGGL(oz_excp_kernel, dim3(kOzExcCap), dim3(256), 0, s, cols[0], cols[1], p->ld[0], p->ld[1], nxy,
                     p->weighted, p->k1, p->e, p->e_pad, (const uint32_t*)p->d_oz_exc, (const int32_t*)p->d_oz_meta,
                     p->d_oz_excp);
  OZ_HIP(hipGetLastError());
  const int k1p = p->k1 | 1;
  const int pexp_pairs = std::min(p->e, kPexpPairs), pexp_blocks = (p->e + kPexpPairs - 1) / kPexpPairs;
  const size_t lds_pexp =
      sizeof(double) * ((size_t)64 * k1p + pexp_pairs) + (2 * sizeof(int32_t) + 2) * (size_t)pexp_pairs;
  const size_t lds_dig = sizeof(double) * (size_t)64 * k1p;
  OZ_HIP(hipFuncSetAttribute((const void*)oz_pexp_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_pexp));
  OZ_HIP(hipFuncSetAttribute((const void*)oz_digits_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_dig));
  for (int g = 0; g < 2; ++g)
    if (p->ntiles[g]) {
      hipLaunchKernelGGL(oz_pexp_kernel, dim3(p->ntiles[g], pexp_blocks), dim3(256), lds_pexp, s, cols[g], p->ld[g],
                         p->n[g], nxy,
                         p->weighted, p->k1, p->e, npp, (const int32_t*)p->d_oz_tile_chunk[g],
                         (const int8_t*)p->d_oz_dev[g], (const int32_t*)p->d_oz_meta, p->d_oz_pexp,
                         reinterpret_cast<unsigned long long*>(p->d_oz_psum));
      OZ_HIP(hipGetLastError());
    }
  const int npe = n_chunks * npp;
  hipLaunchKernelGGL(oz_pexp_finish_kernel, dim3((npe + 255) / 256), dim3(256), 0, s, p->d_oz_pexp, npe);
  OZ_HIP(hipGetLastError());
  const int force7 = ob::opt_int(ob::Opt::GramDigits, 0) == 7 ? 1 : 0;
  const int nct_all = n_chunks * n_ct;
  hipLaunchKernelGGL(oz_nsl_kernel, dim3((nct_all + 255) / 256), dim3(256), 0, s, (const int32_t*)p->d_oz_pexp,
                     (const long long*)p->d_oz_psum, (const uint32_t*)p->d_chunks, p->n[0], p->n[1], p->e, n_ct, npp,
                     n_chunks, force7, p->d_oz_pnsl, p->d_oz_nsl, p->d_oz_meta);
  OZ_HIP(hipGetLastError());
  p->oz_tiles = nct_all;
  for (int g = 0; g < 2; ++g) {
    const uint32_t nsub = (uint32_t)(p->ld[g] >> 6);
    if (p->ntiles[g] == 0 || nsub == 0) continue;
    hipLaunchKernelGGL(oz_digits_kernel, dim3(nsub), dim3(256), lds_dig, s, cols[g], p->ld[g], p->n[g], nxy,
                       p->weighted, p->k1, p->e, n_ct, npp, (const int32_t*)p->d_oz_tile_chunk[g],
                       (const int8_t*)p->d_oz_dev[g], (const int32_t*)p->d_oz_meta, (const int32_t*)p->d_oz_pexp,
                       (const uint8_t*)p->d_oz_pnsl, reinterpret_cast<ob_v4i*>(p->d_oz_b[g]));
    OZ_HIP(hipGetLastError());
  }
  OZ_HIP(hipEventRecord(p->oz_ev[1], s));
  p->oz_timed = true;
  p->oz_nexc = -1;
  p->oz_n_ct = n_ct;
  p->oz_state = 1;
  return OB_OK;
}

// Whether oz_exceptions launches a kernel (which reads the count images after the reduce).
bool oz_exceptions_pending(const ob_panel* p) { return p->oz_state == 1 && p->oz_nexc != 0; }

// The exception rows' f64 terms of one segment (after ob_reduce_kernel). Skipped once a synchronized
// run has shown the panel has none.
int oz_exceptions(ob_panel* p, const uint32_t* counts, uint32_t nb_rep, uint32_t n_reps, double* gram, hipStream_t s) {
  if (p->oz_state != 1 || p->oz_nexc == 0 || n_reps == 0) return OB_OK;
  hipLaunchKernelGGL(oz_exc_kernel, dim3(nb_rep, 2), dim3(256), 0, s, reinterpret_cast<const uint8_t*>(counts), nb_rep,
                     p->ntiles[0], (const uint32_t*)p->d_oz_exc, (const double*)p->d_oz_excp,
                     (const int32_t*)p->d_oz_meta, p->e, p->e_pad, n_reps, gram);
  OZ_HIP(hipGetLastError());
  return OB_OK;
}

// After the boot stream is synchronized: the preparation's time and exception statistics into
// p->timing; more non-finite rows than the exception list holds is an error (their rows would
// be missing from every Gram).
int oz_collect(ob_panel* p) {
  if (p->oz_state != 1) return OB_OK;
  if (p->oz_timed) {
    float t = 0.f;
    OZ_HIP(hipEventElapsedTime(&t, p->oz_ev[0], p->oz_ev[1]));
    p->timing.prep_ms = t;
    p->oz_timed = false;
  }
  if (p->oz_nexc < 0) {
    int32_t meta[6] = {0, 0, 0, 0, 0, 0};
    OZ_HIP(hipMemcpy(meta, p->d_oz_meta, sizeof(meta), hipMemcpyDeviceToHost));
    p->oz_bits = meta[0];
    p->oz_nexc = meta[1];
    p->oz_overflow = meta[3] != 0;
    p->oz_tiles6 = meta[5];
  }
  p->timing.oz_bits = p->oz_bits;
  p->timing.oz_exceptions = p->oz_nexc;
  p->timing.oz_tiles6 = p->oz_tiles6;
  p->timing.oz_tiles = p->oz_tiles;
  if (p->oz_overflow)
    return ob::fail(OB_E_UNSUPPORTED, "more than %d rows hold non-finite values (NaN or inf); the i8 Gram keeps at most "
                                      "that many exception rows (option gram_path = 1 runs the f64 MFMA Gram)",
                    kOzExcCap);
  return OB_OK;
}

void oz_free(ob_panel* p) {
  for (int g = 0; g < 2; ++g) {
    (void)hipFree(p->d_oz_b[g]);
    (void)hipFree(p->d_oz_dev[g]);
    (void)hipFree(p->d_oz_tile_chunk[g]);
  }
  (void)hipFree(p->d_oz_pexp);
  (void)hipFree(p->d_oz_psum);
  (void)hipFree(p->d_oz_nsl);
  (void)hipFree(p->d_oz_pnsl);
  (void)hipFree(p->d_oz_pint);
  (void)hipFree(p->d_oz_acc);
  (void)hipFree(p->d_oz_meta);
  (void)hipFree(p->d_oz_exc);
  (void)hipFree(p->d_oz_excp);
  for (hipEvent_t e : p->oz_ev)
    if (e) (void)hipEventDestroy(e);
}

// One segment's Gram partials: d_chunks holds the panel's chunk table, counts the I8 images of
// the segment's nb_rep replicate batches.
// ksplit 2: each chunk partial from its two halves' int64 slice-group sums, exactly as one block
// would have rounded them (oz_gram_w2_body's epilogue): bitwise the unsplit partial.
__global__ __launch_bounds__(256) void oz_split_combine_kernel(const OzArgs a) {
  const size_t per = (size_t)a.rep_pad * a.e_pad;
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (size_t)a.n_chunks * per) return;
  const uint32_t chunk = (uint32_t)(i / per);
  const uint32_t rem = (uint32_t)(i - (size_t)chunk * per), rep = rem / (uint32_t)a.e_pad, pair = rem % (uint32_t)a.e_pad;
  if (rep >= a.n_reps) return;
  const long long* h0 = a.pint + i * 2;
  const long long* h1 = a.pint + ((size_t)a.n_chunks * per + i) * 2;
  const long long p0 = h0[0] + h1[0], p1 = h0[1] + h1[1];
  const int E = a.pexp[chunk * a.n_pairs_pad + min((int)pair, a.n_pairs_pad - 1)];
  const int NS = a.nsl[chunk * (uint32_t)a.n_ct + pair / kPairsPerTile];
  const int sh0 = E - kFracBits + 8 * (kS - 0 - kSlo), sh1 = E - kFracBits + 8 * (kS - kSlo - (NS - kSlo));
  a.partial[i] = ldexp((double)p0, sh0) + ldexp((double)p1, sh1);
}

// 0: the 8-wave kernel, 1: the wide tile, 2: the wide tile with each block's chunk split over two
// blocks (ksplit 2). Option gram_tile forces one (1, 2, 3); unset, split when the wide launch is a
// few rounds over the CUs with a last round at least a quarter empty (configs[2]'s 1,250 share: 640
// blocks = 2.5 rounds -> 1,280 half blocks = 5), else rounds x cost between the other two.
int oz_gram_mode(const ob_panel* p, int n_chunks, uint32_t nb_rep) {
  const uint32_t n_rt = (nb_rep + 3) / 4, n_ct = (uint32_t)p->oz_n_ct, n_dct = (n_ct + 1) / 2;
  const uint32_t wblocks = (uint32_t)n_chunks * n_rt * n_dct, blocks8 = (uint32_t)n_chunks * n_rt * n_ct;
  const uint32_t cus = (uint32_t)std::max(p->ctx->cus, 1);
  const int tile = ob::opt_int(ob::Opt::GramTile, 0);
  if (tile >= 1 && tile <= 3) return tile - 1;
  const uint32_t wrounds = (wblocks + cus - 1) / cus;
  if (OB_OZ_W_SPLIT && wrounds <= 4 && wrounds * cus - wblocks >= cus / 4) return 2;
  const double kWideCost = 1.85;
  return kWideCost * (double)wrounds <= (double)((blocks8 + cus - 1) / cus) ? 1 : 0;
}

bool oz_wide(const ob_panel* p, int n_chunks, uint32_t nb_rep) { return oz_gram_mode(p, n_chunks, nb_rep) != 0; }

int oz_gram(ob_panel* p, const uint32_t* d_chunks, int n_chunks, const uint32_t* counts, uint32_t nb_rep,
            uint32_t rep_pad, uint32_t n_reps, double* partial, hipStream_t s) {
  OzArgs a{};
  a.B0 = reinterpret_cast<const ob_v4i*>(p->d_oz_b[0]);
  a.B1 = reinterpret_cast<const ob_v4i*>(p->d_oz_b[1]);
  a.counts = reinterpret_cast<const ob_v4i*>(counts);
  a.chunks = d_chunks;
  a.pexp = p->d_oz_pexp;
  a.nsl = p->d_oz_nsl;
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
  a.n_dct = (a.n_ct + 1) / 2;
  // Which kernel: the wide tile does a block's work (twice the 8-wave kernel's) in kWideCost of the
  // 8-wave kernel's block time, but has half as many blocks, so a launch whose last round over the
  // CUs is partial wastes more of it. Rounds x cost decides; both kernels give bitwise the same
  // partials. Measured with the interleaved schedule (profiles/r06_ab_gram_tile_choice2.txt,
  // r06_ab_gram_half.txt): configs[1] 10.68-10.90 against 11.57 ms; configs[3] (5,000 x 3 outcomes,
  // 12.5 rounds) 7.03 against 7.16; 2,500 replicates (5 rounds) 2.65-2.75 against 2.93-3.00;
  // configs[2]'s 1,250 share (640 wide blocks, 2.5 rounds) 1.53-1.60 against 1.54-1.56. (A half-wide
  // tile, the same schedule on 128 replicates x 64 pairs for twice the blocks, measured 12.97 ms at
  // configs[1] and 1.57-1.66 at 1,250, slower than both: half the MFMAs per sub-tile for the same
  // barrier and DMA work, with one wave per SIMD.)
  const uint32_t wblocks = (uint32_t)n_chunks * a.n_rt * (uint32_t)a.n_dct;
  const uint32_t blocks8 = (uint32_t)n_chunks * a.n_rt * (uint32_t)a.n_ct;
  const int mode = oz_gram_mode(p, n_chunks, nb_rep);
  const bool wide = mode != 0;
  p->timing.oz_wide = mode;
  if (wide) {  // oz_gram_w_kernel: 4 waves, 256 replicates x 64 pairs per block
    a.ksplit = mode == 2 ? 2 : 1;
    a.n_chunks = n_chunks;
    if (mode == 2) {
      const size_t need = (size_t)2 * n_chunks * rep_pad * (size_t)p->e_pad * 2;
      if (need > p->cap_oz_pint) {
        (void)hipFree(p->d_oz_pint);
        p->d_oz_pint = nullptr;
        p->cap_oz_pint = 0;
        OZ_HIP(hipMalloc(&p->d_oz_pint, need * sizeof(long long)));
        p->cap_oz_pint = need;
      }
      a.pint = p->d_oz_pint;
    }
    auto wlaunch = [&](auto kern) -> hipError_t {
      hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kWLds);
      if (e != hipSuccess) return e;
      hipLaunchKernelGGL(kern, dim3(wblocks * (uint32_t)a.ksplit), dim3(256), kWLds, s, a);
      if (a.ksplit == 2) {
        const size_t n = (size_t)n_chunks * rep_pad * (size_t)p->e_pad;
        hipLaunchKernelGGL(oz_split_combine_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, a);
      }
      return hipGetLastError();
    };
#if OB_TUNING  // timing ablations (gram_diag): wrong results by design
    switch (ob::opt_int(ob::Opt::GramDiag, 0) & 398) {
      case 2: OZ_HIP(wlaunch(oz_gram_w_kernel<2>)); break;
      case 128: OZ_HIP(wlaunch(oz_gram_w_kernel<128>)); break;
      case 256: OZ_HIP(wlaunch(oz_gram_w_kernel<256>)); break;
      case 384: OZ_HIP(wlaunch(oz_gram_w_kernel<384>)); break;
      case 4: OZ_HIP(wlaunch(oz_gram_w_kernel<4>)); break;
      case 8: OZ_HIP(wlaunch(oz_gram_w_kernel<8>)); break;
      case 6: OZ_HIP(wlaunch(oz_gram_w_kernel<6>)); break;
      default: OZ_HIP(wlaunch(oz_gram_w_kernel<0>)); break;
    }
#else
    OZ_HIP(wlaunch(oz_gram_w_kernel<0>));
#endif
    return OB_OK;
  }
  const uint32_t blocks = blocks8;
  auto launch = [&](auto kern) -> hipError_t {
    hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kLdsBytes);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(kWaves * 64), kLdsBytes, s, a);
    return hipGetLastError();
  };
#if OB_TUNING  // timing ablations (gram_diag): wrong results by design
  switch (ob::opt_int(ob::Opt::GramDiag, 0) & 30) {
    case 2: OZ_HIP(launch(oz_gram_kernel<2>)); break;
    case 4: OZ_HIP(launch(oz_gram_kernel<4>)); break;
    case 6: OZ_HIP(launch(oz_gram_kernel<6>)); break;
    case 8: OZ_HIP(launch(oz_gram_kernel<8>)); break;
    case 16: OZ_HIP(launch(oz_gram_kernel<16>)); break;
    default: OZ_HIP(launch(oz_gram_kernel<0>)); break;
  }
#else
  OZ_HIP(launch(oz_gram_kernel<0>));
#endif
  return OB_OK;
}

}  // namespace ob

extern "C" {

// Test hook (include/oaxaca_boot.h): the exception rows of the panel's i8 Gram, once built.
int ob_debug_gram_exceptions(ob_panel* p, int32_t* bits, int32_t* n_exc, uint32_t* rows, int32_t cap) {
  if (!p || !bits || !n_exc) return ob::fail(OB_E_INVALID, "null pointer");
  if (p->oz_state != 1) return ob::fail(OB_E_INVALID, "the panel's i8 Gram is not built (run a boot on the i8 path first)");
  OZ_HIP(hipSetDevice(p->ctx->device));
  OZ_HIP(hipDeviceSynchronize());
  int32_t meta[4] = {0, 0, 0, 0};
  OZ_HIP(hipMemcpy(meta, p->d_oz_meta, sizeof(meta), hipMemcpyDeviceToHost));
  *bits = meta[0];
  *n_exc = meta[1];
  if (rows && cap > 0 && meta[1] > 0)
    OZ_HIP(hipMemcpy(rows, p->d_oz_exc, sizeof(uint32_t) * (size_t)std::min(cap, meta[1]), hipMemcpyDeviceToHost));
  return meta[3] ? ob::fail(OB_E_UNSUPPORTED, "more than %d non-finite rows", kOzExcCap) : OB_OK;
}

}  // extern "C"
