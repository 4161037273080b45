// ob_gram_i8.hip -- the counts-weighted extended Gram as an exact integer GEMM on i8 MFMA.
//
// Same quantity as ob_gram_kernel (ob_engine.hip): per replicate r and row chunk,
//   G_r[e] = sum_i c_{r,i} P_i[e],   P_i[e] = v_i[a(e)] v_i[b(e)],  v = sqrt(w) [1, x, y]
// (the reference's own sqrt(w) scaling, ols.rs:68-78; X^T W X, X^T W y, sum w and the weighted
// sums of estimation.rs:56-71 are all entries of G). Counts are small integers, so the
// resample weighting is exact in int8; the pair products are written once per panel as S = 8
// fixed-point digits of 7 bits each (Ozaki-style splitting) relative to a per-(chunk, pair)
// power of two 2^E > max |P|:
//     P = sign * sum_s d_s 2^(E - 7 (s + 1)),   d_s in [0, 127]      (56 bits; |error| <= 2^(E-57))
// and  sum_i c_i P_i = sum_s 2^(E - 7 (s + 1)) sum_i c_i (sign d_s)_i,  each inner sum an exact
// int32 (|c| <= 127, sum_i c_i <= n_g, so |sum| <= 127 n_g < 2^31). The slices meet in int64 and
// one f64 rounding per chunk partial. The representation error is at most 2^-57 of the chunk's
// max |P| per row, below f64 summation error, so the Gram equals the f64 MFMA Gram to ~1e-15
// relative (tests/test_gpu_gram_i8.py holds it to 1e-12).
//
// v_mfma_i32_32x32x32_i8 runs 64x the f64 MFMA rate (MI355X_MICROARCH.md, Matrix cores): 8
// slices cost 8x the f64 multiply count and still leave 8x headroom. Layouts (HBM, built once):
//   B (digits): per group [sub-tile 64 rows][col tile: 32 pairs][slice][k-half 32 rows][lane][16 B]
//               -- lane l holds pair (l & 31), rows 16 (l >> 5) + j of the k-half: the B fragment
//               of 32x32x32_i8 (probed: tools/mfma_i8_probe.hip), one 16 KB DMA per sub-tile.
//   A (counts): ob_count_kernel<true> writes [tile][64-rep batch][sub-tile][k-half][rep half][lane][16 B]
//               -- lane l holds replicate (l & 31) of the half, the same rows: the A fragment.
// Kernel: 8 waves (two per SIMD), one block per CU, block tile 256 replicates x 32 pairs x S
// slices; wave w owns replicate batch 4 rt + (w & 3) (2 x 32 replicates) and slice half w >> 2
// (S/2 x 32 columns): 8 accumulators of 32 x 32 i32. Per 64-row sub-tile a wave issues S x 2
// MFMAs (A from HBM straight into registers, prefetched one sub-tile ahead; B from the block's
// LDS copy, DMA'd one sub-tile ahead). The two slice halves meet through LDS at the end.
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

constexpr int kS = 8;                  // 7-bit digits per pair product (56 bits)
constexpr int kPairsPerTile = 32;      // pairs per column tile (one 32-wide MFMA column block)
constexpr int kSubUnits = kS * 2 * 64; // 16-byte units of one (sub-tile, column tile) B image

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

// Per (chunk, column): the exponent e with max |v_c| < 2^e over the chunk's rows (0 if all zero).
__global__ __launch_bounds__(256) void oz_colexp_kernel(const double* cols0, const double* cols1, int64_t ld0,
                                                        int64_t ld1, uint32_t n0, uint32_t n1, int nxy, int weighted,
                                                        const uint32_t* chunks, int k1, int32_t* colexp) {
  __shared__ double red[256];
  const int chunk = blockIdx.x, c = blockIdx.y, tid = threadIdx.x;
  const uint32_t g = chunks[3 * chunk];
  const double* cols = g ? cols1 : cols0;
  const int64_t ld = g ? ld1 : ld0;
  const uint32_t n = g ? n1 : n0;
  const size_t r0 = (size_t)chunks[3 * chunk + 1] * OB_TILE_ROWS;
  const size_t r1 = std::min<size_t>((size_t)chunks[3 * chunk + 2] * OB_TILE_ROWS, n);
  double m = 0.0;
  for (size_t r = r0 + tid; r < r1; r += 256) m = fmax(m, fabs(oz_v(cols, ld, nxy, weighted, r, c)));
  red[tid] = m;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (tid < o) red[tid] = fmax(red[tid], red[tid + o]);
    __syncthreads();
  }
  if (tid == 0) {
    int e = 0;
    if (red[0] > 0.0) (void)frexp(red[0], &e);  // red[0] = f 2^e, f in [0.5, 1): max < 2^e
    colexp[chunk * k1 + c] = e;
  }
}

// Pair exponents E[chunk][pair] = e_a + e_b (max |v_a v_b| <= max|v_a| max|v_b| < 2^(e_a + e_b)).
__global__ void oz_pairexp_kernel(const int32_t* colexp, int k1, int e, int n_pairs_pad, int n_chunks, int32_t* pexp) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_chunks * n_pairs_pad) return;
  const int chunk = i / n_pairs_pad, q = i % n_pairs_pad;
  int v = 0;
  if (q < e) {
    int a = 0, rem = q;
    while (rem >= k1 - a) {
      rem -= k1 - a;
      ++a;
    }
    v = colexp[chunk * k1 + a] + colexp[chunk * k1 + a + rem];
  }
  pexp[i] = v;
}

// B digits of one group: grid (sub-tile, column tile), 256 threads = (slice half, k-half, lane).
__global__ __launch_bounds__(256) void oz_digits_kernel(const double* cols, int64_t ld, uint32_t n, int nxy,
                                                        int weighted, int k1, int e, int n_ct, int n_pairs_pad,
                                                        const int32_t* tile_chunk, const int32_t* pexp,
                                                        ob_v4i* B) {
  const uint32_t sub = blockIdx.x;
  const int ct = blockIdx.y, t = threadIdx.x, lane = t & 63, k2 = (t >> 6) & 1, half = t >> 7;
  const int pair = ct * kPairsPerTile + (lane & 31);
  int a = 0, b = 0;
  const bool live = pair < e;
  if (live) {
    int rem = pair;
    while (rem >= k1 - a) {
      rem -= k1 - a;
      ++a;
    }
    b = a + rem;
  }
  const int E = live ? pexp[tile_chunk[sub >> 2] * n_pairs_pad + pair] : 0;
  long long mag[16];
  bool neg[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const size_t row = (size_t)sub * 64 + k2 * 32 + 16 * (lane >> 5) + j;
    double P = 0.0;
    if (live && row < n) P = oz_v(cols, ld, nxy, weighted, row, a) * oz_v(cols, ld, nxy, weighted, row, b);
    const double m = rint(ldexp(P, 7 * kS - E));  // |m| < 2^56: exact, already integral when >= 2^53
    neg[j] = m < 0.0;
    mag[j] = (long long)fabs(m);
  }
  for (int sl = half * (kS / 2); sl < (half + 1) * (kS / 2); ++sl) {
    const int sh = 7 * (kS - 1 - sl);
    uint32_t w[4] = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int d = (int)((mag[j] >> sh) & 127);
      const uint32_t byte = (uint32_t)(uint8_t)(int8_t)(neg[j] ? -d : d);
      w[j >> 2] |= byte << (8 * (j & 3));
    }
    B[(((size_t)sub * n_ct + ct) * kS + sl) * 2 * 64 + k2 * 64 + lane] = (ob_v4i){(int)w[0], (int)w[1], (int)w[2], (int)w[3]};
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

__device__ __forceinline__ void oz_lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

constexpr int kWaves = 8;                        // 2 per SIMD: (replicate batch, slice half)
constexpr int kHalf = kS / 2;                      // slices per wave
constexpr int kDist = 3;                           // sub-tiles in flight ahead of the MFMAs
constexpr int kNbuf = kDist + 1;                   // B ring in LDS
static_assert(kNbuf == 4, "the main loop below is unrolled over a 4-stage ring");
constexpr int kDmaPerWave = kSubUnits / (64 * kWaves);        // 1 KB B-DMA instructions per wave and sub-tile
constexpr int kAUnits = 4 * 256;                               // 16-byte units of a sub-tile's A (4 batches x 4 KB)
constexpr int kADmaPerWave = 2;                                // each wave DMAs half of its batch's 4 KB
constexpr size_t kLdsB = kNbuf * (size_t)kSubUnits * 16;      // B ring (64 KB)
constexpr size_t kLdsA = kNbuf * (size_t)kAUnits * 16;        // A ring (64 KB)
constexpr size_t kLdsX = 4 * 64 * (size_t)kPairsPerTile * 8;  // low-half exchange (64 KB, over the B ring)
constexpr size_t kLdsBytes = (kLdsB > kLdsX ? kLdsB : kLdsX) + kLdsA;

template <int N>
struct IC {
  static constexpr int value = N;
};

// Both operands arrive by LDS-DMA (global_load_lds), kDist sub-tiles ahead: the compiler does not
// track those loads in registers, so it inserts no vmcnt(0) before the MFMAs; the only waits are
// the explicit vmcnt(n) + barrier that publish sub-tile s + 1.
__global__ __launch_bounds__(kWaves * 64, 1) void oz_gram_kernel(const OzArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const size_t a_off = kLdsB > kLdsX ? kLdsB : kLdsX;
  const ob_v4i* bs = reinterpret_cast<const ob_v4i*>(smem);          // [kNbuf][kSubUnits]
  const ob_v4i* as = reinterpret_cast<const ob_v4i*>(smem + a_off);  // [kNbuf][4 batches][256]
  __attribute__((address_space(3))) unsigned char* lds3 = (__attribute__((address_space(3))) unsigned char*)smem;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wb = wave & 3, half = wave >> 2;  // replicate batch in the tile, slice half
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
  const bool live = batch < a.nb_rep;

  auto dma = [&](int buf, uint32_t s) {
    const ob_v4i* src = Bg + ((size_t)s * a.n_ct + ct) * kSubUnits;  // B: 16 KB
#pragma unroll
    for (int t = 0; t < kDmaPerWave; ++t) {
      const int u = (t * kWaves + wave) * 64;
      __builtin_amdgcn_global_load_lds(src + u + lane,
                                       (__attribute__((address_space(3))) void*)(lds3 + (size_t)(buf * kSubUnits + u) * 16),
                                       16, 0, 0);
    }
    if (live) {  // A: this wave's half of its batch's 4 KB
      const ob_v4i* asrc = a.counts + (((size_t)(tg0 + (s >> 2)) * a.nb_rep + batch) * 4 + (s & 3)) * 256;
#pragma unroll
      for (int t = 0; t < kADmaPerWave; ++t) {
        const int u = (half * kADmaPerWave + t) * 64;
        __builtin_amdgcn_global_load_lds(
            asrc + u + lane,
            (__attribute__((address_space(3))) void*)(lds3 + a_off + (size_t)(buf * kAUnits + wb * 256 + u) * 16), 16, 0,
            0);
      }
    }
  };
  auto wait_ahead = [&]() {  // everything but the kDist - 1 newest sub-tiles has landed
    if (live) asm volatile("s_waitcnt vmcnt(%0)" ::"n"((kDist - 1) * (kDmaPerWave + kADmaPerWave)) : "memory");
    else asm volatile("s_waitcnt vmcnt(%0)" ::"n"((kDist - 1) * kDmaPerWave) : "memory");
  };

  ob_v16i acc[2][kHalf];
#pragma unroll
  for (int rb = 0; rb < 2; ++rb)
#pragma unroll
    for (int q = 0; q < kHalf; ++q) acc[rb][q] = (ob_v16i){};
  // prologue: sub-tiles s0 .. s0 + kDist - 1 in flight; publish s0
#pragma unroll
  for (int j = 0; j < kDist; ++j)
    if (s0 + j < s1) dma(j, s0 + j);
  if (s0 + kDist <= s1) wait_ahead();
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  auto step = [&](uint32_t s, auto J) {
    constexpr int j = decltype(J)::value;
    const uint32_t sp = s + kDist;
    const bool issue = sp < s1;
    if (issue) dma((j + kDist) % kNbuf, sp);  // into the stage freed by s - 1 (every wave is past its barrier)
    if (live) {
      const ob_v4i* bb = bs + j * kSubUnits + half * kHalf * 2 * 64 + lane;
      const ob_v4i* ab = as + j * kAUnits + wb * 256 + lane;
      ob_v4i af[2][2], bf[2][kHalf];  // every fragment of the sub-tile is read before the MFMAs
#pragma unroll
      for (int k2 = 0; k2 < 2; ++k2) {
        af[k2][0] = ab[(k2 * 2 + 0) * 64];
        af[k2][1] = ab[(k2 * 2 + 1) * 64];
#pragma unroll
        for (int q = 0; q < kHalf; ++q) bf[k2][q] = bb[(q * 2 + k2) * 64];
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int k2 = 0; k2 < 2; ++k2)
#pragma unroll
        for (int q = 0; q < kHalf; ++q) {
          acc[0][q] = __builtin_amdgcn_mfma_i32_32x32x32_i8(af[k2][0], bf[k2][q], acc[0][q], 0, 0, 0);
          acc[1][q] = __builtin_amdgcn_mfma_i32_32x32x32_i8(af[k2][1], bf[k2][q], acc[1][q], 0, 0, 0);
        }
    }
    // sub-tile s + 1 must have landed; the kDist - 1 later ones may stay in flight
    if (issue) wait_ahead();
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    oz_lds_barrier();
  };
  for (uint32_t s = s0; s < s1; s += kNbuf) {
    step(s, IC<0>{});
    if (s + 1 < s1) step(s + 1, IC<1>{});
    if (s + 2 < s1) step(s + 2, IC<2>{});
    if (s + 3 < s1) step(s + 3, IC<3>{});
  }
  // slices -> f64: this wave's 4 digits meet exactly in int64 (< 2^52), one ldexp each; the low
  // half goes through LDS to its high-half partner, which adds (one rounding) and stores.
  const int pair = ct * kPairsPerTile + (lane & 31);
  const int E = a.pexp[chunk * a.n_pairs_pad + min(pair, a.n_pairs_pad - 1)];
  const int shift = E - 7 * kS + (half ? 0 : 7 * kHalf);
  double* xch = reinterpret_cast<double*>(smem);  // [batch in tile][64 reps][32 pairs]
  double v[2][16];
#pragma unroll
  for (int rb = 0; rb < 2; ++rb)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      long long part = 0;
#pragma unroll
      for (int q = 0; q < kHalf; ++q) part = part * 128 + acc[rb][q][r];
      v[rb][r] = ldexp((double)part, shift);
    }
  if (half) {
#pragma unroll
    for (int rb = 0; rb < 2; ++rb)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int rl = rb * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        xch[(wb * 64 + rl) * kPairsPerTile + (lane & 31)] = v[rb][r];
      }
  }
  __syncthreads();
  if (half || !live || pair >= a.e_pad) return;
#pragma unroll
  for (int rb = 0; rb < 2; ++rb)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int rl = rb * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
      const uint32_t rep = batch * 64u + (uint32_t)rl;
      const double val = v[rb][r] + xch[(wb * 64 + rl) * kPairsPerTile + (lane & 31)];
      if (rep < a.n_reps) a.partial[((size_t)chunk * a.rep_pad + rep) * a.e_pad + pair] = val;
    }
}

}  // namespace

namespace ob {

// Build (once per panel) the digit images and exponents for the panel's chunking. Returns OB_OK
// with p->oz_state = 1, or OB_OK with p->oz_state = -1 when the digit images would not fit (the
// caller keeps the f64 MFMA Gram).
int oz_prepare(ob_panel* p, const std::vector<uint32_t>& chunks) {
  if (p->oz_state != 0) return OB_OK;
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
  int32_t *d_colexp = nullptr, *d_tc = nullptr;
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
    OZ_TRY(hipMalloc(&d_colexp, sizeof(int32_t) * (size_t)n_chunks * p->k1));
    OZ_TRY(hipMalloc(&d_chunks, sizeof(uint32_t) * chunks.size()));
    OZ_TRY(hipMemcpy(d_chunks, chunks.data(), sizeof(uint32_t) * chunks.size(), hipMemcpyHostToDevice));
    const int nxy = p->p + p->n_y;
    hipLaunchKernelGGL(oz_colexp_kernel, dim3(n_chunks, p->k1), dim3(256), 0, 0, (const double*)p->d_cols[0],
                       (const double*)p->d_cols[1], p->ld[0], p->ld[1], p->n[0], p->n[1], nxy, p->weighted,
                       (const uint32_t*)d_chunks, p->k1, d_colexp);
    OZ_TRY(hipGetLastError());
    const int tot = n_chunks * npp;
    hipLaunchKernelGGL(oz_pairexp_kernel, dim3((tot + 255) / 256), dim3(256), 0, 0, (const int32_t*)d_colexp, p->k1,
                       p->e, npp, n_chunks, p->d_oz_pexp);
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
  (void)hipFree(d_colexp);
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
  OZ_HIP(hipFuncSetAttribute((const void*)oz_gram_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kLdsBytes));
  const uint32_t blocks = (uint32_t)n_chunks * a.n_rt * (uint32_t)a.n_ct;
  hipLaunchKernelGGL(oz_gram_kernel, dim3(blocks), dim3(kWaves * 64), kLdsBytes, s, a);
  OZ_HIP(hipGetLastError());
  return OB_OK;
}

}  // namespace ob
