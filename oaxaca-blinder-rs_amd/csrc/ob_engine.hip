// ob_engine.hip -- the MI355X bootstrap engine: OBRS-1 resampling + X^T diag(c w) X on f64 MFMA
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
//   ob_gram_kernel     one block per (row chunk, 64-replicate batch, column group): per 512-row
//                      tile, level-2 draws -> u8 count image in LDS, then
//                      G[r][e] += sum_i c[r][i] w_i v_i[a(e)] v_i[b(e)] with
//                      v_mfma_f64_16x16x4_f64 (A = counts x weight, 16 replicates x 4 rows;
//                      B = pair products, 4 rows x 16 pairs)
//   ob_reduce_kernel   sums the per-chunk partial Grams in a fixed order (deterministic)
//   ob_solve_kernel    one wave per replicate: normal equations, Cholesky, beta*, OB terms
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

#include "ob_engine.hpp"
#include "ob_spec.h"

typedef double ob_d4 __attribute__((ext_vector_type(4)));

namespace {

constexpr int kBlock = 256;
constexpr int kCntStride = 129;  // u32 words per replicate row of the u8 count image (+1 pad)
constexpr int kCntBytes = 64 * kCntStride * 4;
constexpr int kAuxBytes = 1024;  // prefix sums + level-1 counts of the batch
constexpr int kXtOffset = kCntBytes + kAuxBytes;
constexpr uint64_t kSegReps = 16384;

#define HIP_OK(expr)                                                                     \
  do {                                                                                   \
    hipError_t e_ = (expr);                                                              \
    if (e_ != hipSuccess)                                                                \
      return ob::fail(OB_E_HIP, "HIP error %s at %s:%d", hipGetErrorString(e_), __FILE__, \
                      __LINE__);                                                         \
  } while (0)

// LDS row stride (doubles) of the staged 64-row sub-tile: >= k1 + 1 (w) and == 17 mod 32, so
// the ds_write_b64 of a column (rows on lanes) and the ds_read_b64 of 16 consecutive pair
// columns on two rows are both conflict-free.
inline int lds_row_stride(int k1) {
  int rs = 17;
  while (rs < k1 + 1) rs += 32;
  return rs;
}

struct GramArgs {
  const double* cols0;
  const double* cols1;
  int64_t ld0, ld1;
  uint32_t n0, n1;
  int p, k1, e, ncb, rs, n_cg;
  uint32_t nb_rep;
  const uint32_t* chunks;  // [chunk][3] = (group, first tile, end tile)
  const uint32_t* m1;      // [tile (group 0 then group 1)][rep_pad]
  uint32_t tiles0;
  uint32_t rep_pad;
  uint32_t n_reps;
  uint32_t first_rep;
  uint32_t key0, key1;
  double* partial;  // [chunk][rep_pad][e_pad]
  int e_pad;
  uint32_t* flags;
};

// ---------------------------------------------------------------------------------------------
// Level 1: tile counts m_j for one (replicate, group) from n_g draws (OBRS-1, ob_spec.h).
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void ob_level1_kernel(uint32_t n0, uint32_t n1, uint32_t tiles0,
                                                           uint32_t first_rep, uint32_t rep_pad,
                                                           uint32_t key0, uint32_t key1, uint32_t* m1) {
  extern __shared__ __attribute__((aligned(16))) uint32_t hist[];
  const uint32_t g = blockIdx.y;
  const uint32_t rl = blockIdx.x;
  const uint32_t rep = first_rep + rl;
  const uint32_t n = g ? n1 : n0;
  const uint32_t ntiles = (n + OB_TILE_ROWS - 1) >> OB_TILE_SHIFT;
  for (uint32_t i = threadIdx.x; i < ntiles; i += kBlock) hist[i] = 0;
  __syncthreads();
  const uint32_t npairs = (n + 1) >> 1;
  for (uint32_t p = threadIdx.x; p < npairs; p += kBlock) {
    const ob_u32x4 u = ob_philox(p, rep, g, OB_TAG_L1, key0, key1);
    atomicAdd(&hist[ob_mulhi64(u.x, u.y, n) >> OB_TILE_SHIFT], 1u);
    if (2 * p + 1 < n) atomicAdd(&hist[ob_mulhi64(u.z, u.w, n) >> OB_TILE_SHIFT], 1u);
  }
  __syncthreads();
  const uint32_t toff = g ? tiles0 : 0;
  for (uint32_t i = threadIdx.x; i < ntiles; i += kBlock) m1[(size_t)(toff + i) * rep_pad + rl] = hist[i];
}

// ---------------------------------------------------------------------------------------------
// Gram: per block 64 replicates x (4 * CB * 16) pair columns x one row chunk of one group.
// ---------------------------------------------------------------------------------------------
template <int CB, bool WEIGHTED, bool UNIT>
__global__ __launch_bounds__(kBlock, 2) void ob_gram_kernel(const GramArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  uint32_t* cnt = reinterpret_cast<uint32_t*>(smem);
  uint32_t* pref = reinterpret_cast<uint32_t*>(smem + kCntBytes);  // 65 entries
  uint32_t* mcnt = pref + 72;                                       // 64 entries
  double* xt = reinterpret_cast<double*>(smem + kXtOffset);         // [64][rs]

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;

  // XCD-aware bijective remap: consecutive work items (same chunk, successive replicate
  // batches) land on one XCD so their X sub-tiles are shared through that XCD's L2.
  const uint32_t nwg = gridDim.x, bid = blockIdx.x;
  const uint32_t xcd = bid & 7u, slot = bid >> 3, q8 = nwg >> 3, r8 = nwg & 7u;
  const uint32_t wi = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + slot;
  const uint32_t rb = wi % a.nb_rep;
  const uint32_t tq = wi / a.nb_rep;
  const uint32_t cg = tq % (uint32_t)a.n_cg;
  const uint32_t chunk = tq / (uint32_t)a.n_cg;
  const uint32_t g = a.chunks[chunk * 3], t0 = a.chunks[chunk * 3 + 1], t1 = a.chunks[chunk * 3 + 2];
  const double* X = g ? a.cols1 : a.cols0;
  const int64_t ld = g ? a.ld1 : a.ld0;
  const uint32_t n = g ? a.n1 : a.n0;
  const uint32_t rep0 = rb * 64;
  const int rs = a.rs;

  const int cb0 = ((int)cg * 4 + wave) * CB;
  const bool wave_active = cb0 < a.ncb;
  int offa[CB], offb[CB];
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
    offa[c] = pa;
    offb[c] = pb;
  }
  ob_d4 acc[4][CB];
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int c = 0; c < CB; ++c) acc[r][c] = (ob_d4){0.0, 0.0, 0.0, 0.0};

  if (tid < 64) xt[tid * rs] = 1.0;  // v[0] = intercept, never overwritten
  const int ncl = a.p + 1 + (WEIGHTED ? 1 : 0);

  for (uint32_t tile = t0; tile < t1; ++tile) {
    const uint32_t row0 = tile * OB_TILE_ROWS;
    const uint32_t S = min(OB_TILE_ROWS, n - row0);
    if (!UNIT) {
      for (int i = tid; i < 64 * kCntStride; i += kBlock) cnt[i] = 0u;
      if (tid < 64) {
        const uint32_t rep = rep0 + tid;
        const uint32_t m =
            rep < a.n_reps ? a.m1[(size_t)(g ? a.tiles0 + tile : tile) * a.rep_pad + rep] : 0u;
        mcnt[tid] = m;
        uint32_t s = (m + 1) >> 1;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
          const uint32_t o = __shfl_up(s, off);
          if (lane >= off) s += o;
        }
        pref[tid + 1] = s;
        if (tid == 0) pref[0] = 0u;
      }
      __syncthreads();
      const uint32_t total = pref[64];
      int r = 0;
      uint32_t ovf = 0;
      for (uint32_t gp = tid; gp < total; gp += kBlock) {
        while (pref[r + 1] <= gp) ++r;
        const uint32_t pp = gp - pref[r];
        const ob_u32x4 u =
            ob_philox(pp, a.first_rep + rep0 + r, (tile << 1) | g, OB_TAG_L2, a.key0, a.key1);
        uint32_t lr = ob_mulhi64(u.x, u.y, S);
        uint32_t sh = (lr & 3u) * 8u;
        uint32_t old = atomicAdd(&cnt[r * kCntStride + (lr >> 2)], 1u << sh);
        ovf |= ((old >> sh) & 0xFFu) == 0xFFu;
        if (2 * pp + 1 < mcnt[r]) {
          lr = ob_mulhi64(u.z, u.w, S);
          sh = (lr & 3u) * 8u;
          old = atomicAdd(&cnt[r * kCntStride + (lr >> 2)], 1u << sh);
          ovf |= ((old >> sh) & 0xFFu) == 0xFFu;
        }
      }
      if (ovf) atomicOr(a.flags, 1u);
      __syncthreads();
    }
    const uint32_t nsub = (S + 63) >> 6;
    for (uint32_t s = 0; s < nsub; ++s) {
      const size_t gbase = (size_t)row0 + s * 64;
      for (int idx = tid; idx < ncl * 64; idx += kBlock) {
        const int c = idx >> 6, rr = idx & 63;
        xt[rr * rs + 1 + c] = X[(size_t)c * ld + gbase + rr];
      }
      __syncthreads();
      if (wave_active) {
#pragma unroll 1
        for (int ks = 0; ks < 16; ++ks) {
          const int rloc = ks * 4 + (lane >> 4);
          const double* xr = xt + rloc * rs;
          const double wv = WEIGHTED ? xr[a.k1] : 1.0;
          double af[4];
#pragma unroll
          for (int q4 = 0; q4 < 4; ++q4) {
            double cv;
            if (UNIT) {
              cv = (gbase + rloc < n) ? 1.0 : 0.0;
            } else {
              const int rep = q4 * 16 + (lane & 15);
              const uint32_t trow = s * 64 + rloc;
              const uint32_t word = cnt[rep * kCntStride + (trow >> 2)];
              cv = (double)((word >> ((trow & 3u) * 8u)) & 0xFFu);
            }
            af[q4] = cv * wv;
          }
          double bf[CB];
#pragma unroll
          for (int c = 0; c < CB; ++c) bf[c] = xr[offa[c]] * xr[offb[c]];
#pragma unroll
          for (int q4 = 0; q4 < 4; ++q4)
#pragma unroll
            for (int c = 0; c < CB; ++c)
              acc[q4][c] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[q4], bf[c], acc[q4][c], 0, 0, 0);
        }
      }
      __syncthreads();
    }
  }

  if (wave_active) {
#pragma unroll
    for (int c = 0; c < CB; ++c) {
      if (cb0 + c >= a.ncb) continue;
      const int e = (cb0 + c) * 16 + (lane & 15);
#pragma unroll
      for (int q4 = 0; q4 < 4; ++q4)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const uint32_t rep = rep0 + q4 * 16 + (lane >> 4) + 4 * r;
          if (rep < a.n_reps) a.partial[((size_t)chunk * a.rep_pad + rep) * a.e_pad + e] = acc[q4][c][r];
        }
    }
  }
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

__device__ __forceinline__ double gpair(const double* g, int a, int b, int k1) {
  return a <= b ? g[ob_pair_index(a, b, k1)] : g[ob_pair_index(b, a, k1)];
}

// nalgebra Cholesky::new order (left-looking, per-element updates in column order).
// Fails iff a pivot is zero, negative or NaN (!is_zero && try_sqrt). m: n x n col-major.
__device__ bool wave_cholesky(double* m, int n, int lane) {
  for (int j = 0; j < n; ++j) {
    for (int i = j + lane; i < n; i += 64) {
      double v = m[i + j * n];
      for (int c = 0; c < j; ++c) v = -m[j + c * n] * m[i + c * n] + v;
      m[i + j * n] = v;
    }
    __syncthreads();
    const double diag = m[j + j * n];
    if (!(diag != 0.0 && diag >= 0.0)) return false;
    const double den = sqrt(diag);
    __syncthreads();
    for (int i = j + lane; i < n; i += 64) m[i + j * n] = (i == j) ? den : m[i + j * n] / den;
    __syncthreads();
  }
  return true;
}

__device__ void wave_chol_solve(const double* l, int n, double* b, int lane) {
  for (int i = 0; i < n; ++i) {
    const double coeff = b[i] / l[i + i * n];
    __syncthreads();
    for (int r = i + 1 + lane; r < n; r += 64) b[r] -= coeff * l[r + i * n];
    if (lane == 0) b[i] = coeff;
    __syncthreads();
  }
  for (int i = n - 1; i >= 0; --i) {
    double part = 0.0;
    for (int r = i + 1 + lane; r < n; r += 64) part += l[r + i * n] * b[r];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) part += __shfl_xor(part, off);
    if (lane == 0) b[i] = (b[i] - part) / l[i + i * n];
    __syncthreads();
  }
}

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

__global__ __launch_bounds__(64) void ob_solve_kernel(const SolveArgs a) {
  extern __shared__ __attribute__((aligned(16))) double sm[];
  const int lane = threadIdx.x;
  const uint32_t rep = blockIdx.x;
  if (rep >= a.n_reps) return;
  const int k = a.k, k1 = a.k1, kp = k + 1;
  double* M = sm;                 // kp * kp
  double* rhs = M + kp * kp;      // kp
  double* beta_a = rhs + kp;      // k
  double* beta_b = beta_a + kp;   // k
  double* xam = beta_b + kp;      // k
  double* xbm = xam + kp;         // k
  double* bstar = xbm + kp;       // kp (pooled before removal)
  double* base = bstar + kp;      // 3 * n_norm: a, b, star
  const double* GA = a.gram + (size_t)rep * 2 * a.e_pad;
  const double* GB = GA + a.e_pad;
  double* row = a.rows + (size_t)rep * a.row_len;
  if (a.gram_out && rep == 0)
    for (int i = lane; i < 2 * a.e_pad; i += 64) a.gram_out[i] = GA[i];

  uint8_t status = 1;
  // OLS for both groups (estimation.rs:53-54 -> ols.rs:44-144)
  for (int g = 0; g < 2 && status == 1; ++g) {
    const double* G = g ? GB : GA;
    double* beta = g ? beta_b : beta_a;
    for (int i = lane; i < k * k; i += 64) {
      const int r = i % k, c = i / k;
      M[r + c * k] = gpair(G, r, c, k1);
    }
    for (int i = lane; i < k; i += 64) rhs[i] = gpair(G, i, k1 - 1, k1);
    __syncthreads();
    if (!wave_cholesky(M, k, lane)) {
      status = 0;
      break;
    }
    wave_chol_solve(M, k, rhs, lane);
    if (g == 1 && a.raw_beta_b && rep == 0)
      for (int i = lane; i < k; i += 64) a.raw_beta_b[i] = rhs[i];
    const double sw = G[0];
    for (int i = lane; i < k; i += 64) {
      beta[i] = rhs[i];
      (g ? xbm : xam)[i] = gpair(G, 0, i, k1) / sw;  // estimation.rs:56-71 (weighted or row mean)
    }
    __syncthreads();
  }
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
    __syncthreads();
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
          rhs[u] = gpair(GA, 0, k1 - 1, k1);
        } else {
          const int o = u < ip ? u : u - 1;
          rhs[u] = gpair(GA, o, k1 - 1, k1) + gpair(GB, o, k1 - 1, k1);
        }
      }
      __syncthreads();
      if (!wave_cholesky(M, kp, lane)) {
        status = 0;
      } else {
        wave_chol_solve(M, kp, rhs, lane);
        if (lane == 0) {
          if (a.n_norm > 0) normalize_coeffs(rhs, a, pst, pidx, base_s);
          for (int u = 0, d = 0; u < kp; ++u)
            if (u != ip) bstar[d++] = rhs[u];
        }
      }
    }
  }
  __syncthreads();
  if (lane == 0) {
    if (status != 1) {
      for (int i = 0; i < a.row_len; ++i) row[i] = __builtin_nan("");
    } else {
      const int kd = k + a.n_base;
      double* dex = row + 6;
      double* dun = row + 6 + kd;
      double expl = 0.0, ta = 0.0, tb = 0.0, endow = 0.0, coef = 0.0, inter = 0.0;
      for (int j = 0; j < k; ++j) {  // decomposition.rs:56-89
        const double dx = xam[j] - xbm[j], db = beta_a[j] - beta_b[j];
        expl += dx * bstar[j];
        ta += xam[j] * beta_a[j];
        tb += xbm[j] * beta_b[j];
        endow += dx * beta_b[j];
        coef += xbm[j] * db;
        inter += dx * db;
      }
      double unexpl = (ta - tb) - expl;
      for (int j = 0; j < k; ++j) {  // decomposition.rs:92-122
        dex[j] = (xam[j] - xbm[j]) * bstar[j];
        dun[j] = xam[j] * (beta_a[j] - bstar[j]) + xbm[j] * (bstar[j] - beta_b[j]);
      }
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
      row[2] = endow;
      row[3] = coef;
      row[4] = inter;
      row[5] = gpair(GA, 0, k1 - 1, k1) / GA[0] - gpair(GB, 0, k1 - 1, k1) / GB[0];  // builder.rs:676-684
      double* tail = row + 6 + 2 * kd;
      for (int j = 0; j < k; ++j) {
        tail[j] = beta_a[j];
        tail[k + j] = beta_b[j];
        tail[2 * k + j] = xam[j];
        tail[3 * k + j] = xbm[j];
        tail[4 * k + j] = bstar[j];
      }
    }
    a.ok[rep] = a.raw_status ? status : (uint8_t)(status == 1);
  }
}

// y_B - X_B beta_B on the unresampled group B (ols.rs:118-119; OaxacaResults::residuals).
__global__ __launch_bounds__(kBlock) void ob_residual_kernel(const double* cols, int64_t ld, uint32_t n, int p,
                                                             const double* beta, double* out) {
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  double yh = beta[0];
  for (int c = 0; c < p; ++c) yh += cols[(size_t)c * ld + i] * beta[1 + c];
  out[i] = cols[(size_t)p * ld + i] - yh;
}

// ---------------------------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------------------------
struct Plan {
  uint32_t nb_rep, rep_pad, n_cg;
  int cb;
  std::vector<uint32_t> chunks;  // (g, t0, t1)
  int n_chunks() const { return (int)(chunks.size() / 3); }
};

int pick_cb(int ncb) { return ncb > 8 ? 4 : (ncb > 4 ? 2 : 1); }

Plan make_plan(const ob_panel* p, uint64_t n_reps) {
  Plan pl;
  pl.nb_rep = (uint32_t)((n_reps + 63) / 64);
  pl.rep_pad = pl.nb_rep * 64;
  pl.cb = pick_cb(p->ncb);
  pl.n_cg = (uint32_t)((p->ncb + 4 * pl.cb - 1) / (4 * pl.cb));
  const uint32_t tA = p->ntiles[0], tB = p->ntiles[1], tT = tA + tB;
  const double conc = (double)std::max(p->ctx->cus, 1) * 2.0;
  // chunk size in tiles: pick the one whose grid fills whole rounds of resident blocks
  uint32_t best_tpc = tT;
  double best = -1.0;
  for (uint32_t c = 2; c <= std::min<uint32_t>(tT, 96); ++c) {
    const uint32_t tpc = (tT + c - 1) / c;
    const uint32_t nch = (tA + tpc - 1) / tpc + (tB + tpc - 1) / tpc;
    const double blocks = (double)pl.nb_rep * pl.n_cg * nch;
    const double rounds = std::ceil(blocks / conc);
    const double score = blocks / (rounds * conc) - 0.002 * nch;
    if (score > best + 1e-12) {
      best = score;
      best_tpc = tpc;
    }
  }
  if (tT < 2) best_tpc = 1;
  for (uint32_t g = 0; g < 2; ++g) {
    const uint32_t tg = g ? tB : tA;
    for (uint32_t t = 0; t < tg; t += best_tpc) {
      pl.chunks.push_back(g);
      pl.chunks.push_back(t);
      pl.chunks.push_back(std::min(tg, t + best_tpc));
    }
  }
  return pl;
}

size_t gram_lds_bytes(const ob_panel* p) { return (size_t)kXtOffset + (size_t)64 * lds_row_stride(p->k1) * 8; }
size_t solve_lds_bytes(const ob_panel* p) {
  const int kp = p->k + 1;
  return sizeof(double) * ((size_t)kp * kp + 6 * kp + 3 * (size_t)std::max(p->norm.n_norm, 1));
}

template <int CB, bool W, bool U>
hipError_t launch_gram_t(const GramArgs& ga, uint32_t blocks, size_t lds, hipStream_t s) {
  auto kern = ob_gram_kernel<CB, W, U>;
  hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(kBlock), lds, s, ga);
  return hipGetLastError();
}

template <bool W, bool U>
hipError_t launch_gram_w(int cb, const GramArgs& ga, uint32_t blocks, size_t lds, hipStream_t s) {
  switch (cb) {
    case 4: return launch_gram_t<4, W, U>(ga, blocks, lds, s);
    case 2: return launch_gram_t<2, W, U>(ga, blocks, lds, s);
    default: return launch_gram_t<1, W, U>(ga, blocks, lds, s);
  }
}

hipError_t launch_gram(int cb, bool weighted, bool unit, const GramArgs& ga, uint32_t blocks, size_t lds,
                       hipStream_t s) {
  if (weighted) return unit ? launch_gram_w<true, true>(cb, ga, blocks, lds, s) : launch_gram_w<true, false>(cb, ga, blocks, lds, s);
  return unit ? launch_gram_w<false, true>(cb, ga, blocks, lds, s) : launch_gram_w<false, false>(cb, ga, blocks, lds, s);
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
  ga.cols0 = p->d_cols[0];
  ga.cols1 = p->d_cols[1];
  ga.ld0 = p->ld[0];
  ga.ld1 = p->ld[1];
  ga.n0 = p->n[0];
  ga.n1 = p->n[1];
  ga.p = p->p;
  ga.k1 = p->k1;
  ga.e = p->e;
  ga.ncb = p->ncb;
  ga.rs = lds_row_stride(p->k1);
  ga.n_cg = (int)pl.n_cg;
  ga.nb_rep = pl.nb_rep;
  ga.tiles0 = p->ntiles[0];
  ga.rep_pad = pl.rep_pad;
  ga.e_pad = p->e_pad;
  ga.flags = p->d_flags;
  return ga;
}

}  // namespace

namespace ob {

int engine_point_estimate(ob_panel* p, int ref_mode, double* row, double* resid_b) {
  ob_ctx* ctx = p->ctx;
  HIP_OK(hipSetDevice(ctx->device));
  hipStream_t s = ctx->stream;
  Plan pl = make_plan(p, 1);
  const int nch = pl.n_chunks();
  double *d_partial = nullptr, *d_gram = nullptr, *d_row = nullptr, *d_gout = nullptr, *d_beta = nullptr,
         *d_res = nullptr;
  uint32_t* d_chunks = nullptr;
  uint8_t* d_ok = nullptr;
  auto cleanup = [&]() {
    (void)hipFree(d_partial);
    (void)hipFree(d_gram);
    (void)hipFree(d_row);
    (void)hipFree(d_gout);
    (void)hipFree(d_beta);
    (void)hipFree(d_res);
    (void)hipFree(d_chunks);
    (void)hipFree(d_ok);
  };
  int rc = OB_OK;
  do {
#define PE_OK(expr)                                                                            \
  {                                                                                            \
    hipError_t e_ = (expr);                                                                    \
    if (e_ != hipSuccess) {                                                                    \
      rc = ob::fail(OB_E_HIP, "HIP error %s at %s:%d", hipGetErrorString(e_), __FILE__, __LINE__); \
      break;                                                                                   \
    }                                                                                          \
  }
    PE_OK(hipMalloc(&d_partial, sizeof(double) * (size_t)nch * pl.rep_pad * p->e_pad));
    PE_OK(hipMalloc(&d_gram, sizeof(double) * 2 * (size_t)pl.rep_pad * p->e_pad));
    PE_OK(hipMalloc(&d_row, sizeof(double) * p->row_len));
    PE_OK(hipMalloc(&d_gout, sizeof(double) * 2 * p->e_pad));
    PE_OK(hipMalloc(&d_chunks, sizeof(uint32_t) * pl.chunks.size()));
    PE_OK(hipMalloc(&d_ok, 1));
    PE_OK(hipMemcpyAsync(d_chunks, pl.chunks.data(), sizeof(uint32_t) * pl.chunks.size(), hipMemcpyHostToDevice, s));
    GramArgs ga = gram_args(p, pl);
    ga.chunks = d_chunks;
    ga.m1 = nullptr;
    ga.n_reps = 1;
    ga.first_rep = 0;
    ga.partial = d_partial;
    const uint32_t blocks = pl.nb_rep * pl.n_cg * (uint32_t)nch;
    PE_OK(launch_gram(pl.cb, p->weighted != 0, true, ga, blocks, gram_lds_bytes(p), s));
    const size_t nred = (size_t)1 * p->e_pad;
    hipLaunchKernelGGL(ob_reduce_kernel, dim3((unsigned)((nred + kBlock - 1) / kBlock)), dim3(kBlock), 0, s,
                       (const double*)d_partial, (const uint32_t*)d_chunks, nch, pl.rep_pad, p->e_pad, 1u, d_gram);
    PE_OK(hipGetLastError());
    SolveArgs sa = solve_args(p, ref_mode);
    sa.gram = d_gram;
    sa.rows = d_row;
    sa.ok = d_ok;
    sa.n_reps = 1;
    sa.gram_out = d_gout;
    sa.raw_status = 1;
    PE_OK(hipMalloc(&d_beta, sizeof(double) * p->k));
    sa.raw_beta_b = d_beta;
    hipLaunchKernelGGL(ob_solve_kernel, dim3(1), dim3(64), solve_lds_bytes(p), s, sa);
    PE_OK(hipGetLastError());
    uint8_t okh = 0;
    std::vector<double> gout(2 * p->e_pad);
    PE_OK(hipMemcpyAsync(row, d_row, sizeof(double) * p->row_len, hipMemcpyDeviceToHost, s));
    PE_OK(hipMemcpyAsync(&okh, d_ok, 1, hipMemcpyDeviceToHost, s));
    PE_OK(hipMemcpyAsync(gout.data(), d_gout, sizeof(double) * gout.size(), hipMemcpyDeviceToHost, s));
    PE_OK(hipStreamSynchronize(s));
    if (okh == 2) {
      rc = ob::fail(OB_E_GROUP, "%sNo data in groups for weighted coefficients.", error_prefix(OB_E_GROUP));
      break;
    }
    if (okh != 1) {
      rc = ob::fail(OB_E_LINALG,
                    "%sFailed to perform Cholesky decomposition. Matrix may be singular or not positive "
                    "definite due to multicollinearity.",
                    error_prefix(OB_E_LINALG));
      break;
    }
    if (resid_b) {
      PE_OK(hipMalloc(&d_res, sizeof(double) * std::max<uint32_t>(p->n[1], 1)));
      if (p->n[1] > 0) {
        hipLaunchKernelGGL(ob_residual_kernel, dim3((p->n[1] + kBlock - 1) / kBlock), dim3(kBlock), 0, s,
                           (const double*)p->d_cols[1], p->ld[1], p->n[1], p->p, (const double*)d_beta, d_res);
        PE_OK(hipGetLastError());
        PE_OK(hipMemcpyAsync(resid_b, d_res, sizeof(double) * p->n[1], hipMemcpyDeviceToHost, s));
      }
      PE_OK(hipStreamSynchronize(s));
    }
#undef PE_OK
  } while (0);
  cleanup();
  return rc;
}

int engine_boot(ob_panel* p, uint64_t seed, uint64_t first_rep, uint64_t n_reps, int ref_mode, double* d_rows,
                uint8_t* d_ok, hipStream_t stream) {
  ob_ctx* ctx = p->ctx;
  HIP_OK(hipSetDevice(ctx->device));
  if (n_reps == 0) return OB_OK;
  if (first_rep + n_reps > 0x100000000ull)
    return ob::fail(OB_E_INVALID, "replicate ids must stay below 2^32 (OBRS-1 counter word)");
  hipStream_t s = stream ? stream : ctx->stream;
  const uint64_t seg = std::min<uint64_t>(n_reps, kSegReps);
  Plan pl = make_plan(p, seg);
  const int nch = pl.n_chunks();
  const uint32_t tiles = p->ntiles[0] + p->ntiles[1];
  OB_TRY(ensure_buf(&p->d_m1, p->cap_m1, (size_t)tiles * pl.rep_pad));
  OB_TRY(ensure_buf(&p->d_partial, p->cap_partial, (size_t)nch * pl.rep_pad * p->e_pad));
  OB_TRY(ensure_buf(&p->d_gram, p->cap_gram, (size_t)2 * pl.rep_pad * p->e_pad));
  OB_TRY(ensure_buf(&p->d_chunks, p->cap_chunks, pl.chunks.size()));
  HIP_OK(hipMemcpyAsync(p->d_chunks, pl.chunks.data(), sizeof(uint32_t) * pl.chunks.size(), hipMemcpyHostToDevice, s));
  HIP_OK(hipStreamSynchronize(s));  // the host vector dies with this call
  HIP_OK(hipMemsetAsync(p->d_flags, 0, sizeof(uint32_t), s));

  const size_t lds_l1 = sizeof(uint32_t) * std::max(p->ntiles[0], p->ntiles[1]);
  HIP_OK(hipFuncSetAttribute((const void*)ob_level1_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_l1));
  HIP_OK(hipFuncSetAttribute((const void*)ob_solve_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                             (int)solve_lds_bytes(p)));
  std::memset(&p->timing, 0, sizeof(p->timing));
  p->timing.chunks = nch;
  p->timing.blocks = (int32_t)(pl.nb_rep * pl.n_cg * (uint32_t)nch);
  p->pending_segments = 0;
  const uint32_t key0 = (uint32_t)seed, key1 = (uint32_t)(seed >> 32);
  const size_t nseg = (size_t)((n_reps + seg - 1) / seg);
  while (p->seg_events.size() < 5 * nseg) {
    hipEvent_t e;
    HIP_OK(hipEventCreate(&e));
    p->seg_events.push_back(e);
  }
  for (uint64_t s0 = 0; s0 < n_reps; s0 += seg) {
    const uint32_t ns = (uint32_t)std::min<uint64_t>(seg, n_reps - s0);
    Plan plx = (ns == seg) ? pl : make_plan(p, ns);
    if (plx.chunks != pl.chunks || plx.rep_pad != pl.rep_pad) {
      HIP_OK(hipStreamSynchronize(s));
      HIP_OK(hipMemcpyAsync(p->d_chunks, plx.chunks.data(), sizeof(uint32_t) * plx.chunks.size(),
                            hipMemcpyHostToDevice, s));
      HIP_OK(hipStreamSynchronize(s));
    }
    const int nchx = plx.n_chunks();
    const uint32_t frep = (uint32_t)(first_rep + s0);
    hipEvent_t* ev = p->seg_events.data() + 5 * (size_t)p->pending_segments;
    const bool timed = true;
    if (timed) HIP_OK(hipEventRecord(ev[0], s));
    hipLaunchKernelGGL(ob_level1_kernel, dim3(ns, 2), dim3(kBlock), lds_l1, s, p->n[0], p->n[1], p->ntiles[0], frep,
                       plx.rep_pad, key0, key1, p->d_m1);
    HIP_OK(hipGetLastError());
    if (timed) HIP_OK(hipEventRecord(ev[1], s));
    GramArgs ga = gram_args(p, plx);
    ga.chunks = p->d_chunks;
    ga.m1 = p->d_m1;
    ga.n_reps = ns;
    ga.first_rep = frep;
    ga.key0 = key0;
    ga.key1 = key1;
    ga.partial = p->d_partial;
    const uint32_t blocks = plx.nb_rep * plx.n_cg * (uint32_t)nchx;
    HIP_OK(launch_gram(plx.cb, p->weighted != 0, false, ga, blocks, gram_lds_bytes(p), s));
    if (timed) HIP_OK(hipEventRecord(ev[2], s));
    const size_t nred = (size_t)ns * p->e_pad;
    hipLaunchKernelGGL(ob_reduce_kernel, dim3((unsigned)((nred + kBlock - 1) / kBlock)), dim3(kBlock), 0, s,
                       (const double*)p->d_partial, (const uint32_t*)p->d_chunks, nchx, plx.rep_pad, p->e_pad, ns,
                       p->d_gram);
    HIP_OK(hipGetLastError());
    if (timed) HIP_OK(hipEventRecord(ev[3], s));
    SolveArgs sa = solve_args(p, ref_mode);
    sa.gram = p->d_gram;
    sa.rows = d_rows + (size_t)s0 * p->row_len;
    sa.ok = d_ok + s0;
    sa.n_reps = ns;
    sa.gram_out = nullptr;
    sa.raw_beta_b = nullptr;
    sa.raw_status = 0;
    hipLaunchKernelGGL(ob_solve_kernel, dim3(ns), dim3(64), solve_lds_bytes(p), s, sa);
    HIP_OK(hipGetLastError());
    if (timed) HIP_OK(hipEventRecord(ev[4], s));
    p->timing.gram_launches += 1;
    p->pending_segments += 1;
  }
  p->timing_pending = true;
  p->last_stream = s;
  return OB_OK;
}

// Synchronize the last boot run, sum its per-segment kernel timings and check the
// count-overflow flag.
int engine_collect(ob_panel* p) {
  if (!p->timing_pending) return OB_OK;
  HIP_OK(hipSetDevice(p->ctx->device));
  HIP_OK(hipStreamSynchronize(p->last_stream));
  p->timing_pending = false;
  double* dst[4] = {&p->timing.level1_ms, &p->timing.gram_ms, &p->timing.reduce_ms, &p->timing.solve_ms};
  for (int sg = 0; sg < p->pending_segments; ++sg) {
    hipEvent_t* ev = p->seg_events.data() + 5 * (size_t)sg;
    for (int i = 0; i < 4; ++i) {
      float t = 0.f;
      HIP_OK(hipEventElapsedTime(&t, ev[i], ev[i + 1]));
      *dst[i] += t;
    }
  }
  uint32_t flag = 0;
  HIP_OK(hipMemcpy(&flag, p->d_flags, sizeof(uint32_t), hipMemcpyDeviceToHost));
  if (flag) return ob::fail(OB_E_OVERFLOW, "a resampled row was drawn more than 255 times in one replicate");
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
  if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
  delete ctx;
}

int ob_panel_create(ob_ctx* ctx, const ob_panel_desc* d, ob_panel** out) {
  if (!ctx || !d || !out) return ob::fail(OB_E_INVALID, "null pointer");
  *out = nullptr;
  if (d->p < 0 || d->p > 126) return ob::fail(OB_E_UNSUPPORTED, "predictor columns must be in [0, 126], got %d", d->p);
  if (d->n_num < 0 || d->n_num > d->p) return ob::fail(OB_E_INVALID, "n_num out of range");
  const ob_group_desc* gd[2] = {&d->a, &d->b};
  for (int g = 0; g < 2; ++g) {
    if (gd[g]->n < 0 || gd[g]->n > 16000000) return ob::fail(OB_E_UNSUPPORTED, "group rows must be in [0, 16e6]");
    if (gd[g]->n > 0 && ((d->p > 0 && !gd[g]->x) || !gd[g]->y || (d->weighted && !gd[g]->w)))
      return ob::fail(OB_E_INVALID, "missing column pointer");
    if (gd[g]->ldx < gd[g]->n) return ob::fail(OB_E_INVALID, "ldx < n");
    if (d->weighted)
      for (int64_t i = 0; i < gd[g]->n; ++i)
        if (gd[g]->w[i] < 0.0)
          return ob::fail(OB_E_GROUP, "%sWeights cannot be negative", ob::error_prefix(OB_E_GROUP));
  }
  HIP_OK(hipSetDevice(ctx->device));
  ob_panel* p = new ob_panel();
  p->ctx = ctx;
  p->p = d->p;
  p->k = d->p + 1;
  p->k1 = d->p + 2;
  p->e = p->k1 * (p->k1 + 1) / 2;
  p->ncb = (p->e + 15) / 16;
  p->e_pad = p->ncb * 16;
  p->n_num = d->n_num;
  p->weighted = d->weighted ? 1 : 0;
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
  p->row_len = ob_row_len(p->k, nc.n_base);
  int rc = OB_OK;
  auto bad = [&](hipError_t e, int line) {
    rc = ob::fail(OB_E_HIP, "HIP error %s at %s:%d", hipGetErrorString(e), __FILE__, line);
  };
  for (int g = 0; g < 2 && rc == OB_OK; ++g) {
    p->n[g] = (uint32_t)gd[g]->n;
    p->ntiles[g] = (p->n[g] + OB_TILE_ROWS - 1) / OB_TILE_ROWS;
    p->ld[g] = (int64_t)std::max<uint32_t>(p->ntiles[g], 1) * OB_TILE_ROWS;
    const int ncols = p->p + 1 + p->weighted;
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
      e = hipMemcpy(p->d_cols[g] + (size_t)p->p * p->ld[g], gd[g]->y, sizeof(double) * n, hipMemcpyHostToDevice);
      if (e != hipSuccess) { bad(e, __LINE__); break; }
      if (p->weighted) {
        e = hipMemcpy(p->d_cols[g] + (size_t)(p->p + 1) * p->ld[g], gd[g]->w, sizeof(double) * n,
                      hipMemcpyHostToDevice);
        if (e != hipSuccess) { bad(e, __LINE__); break; }
      }
    }
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
  for (int g = 0; g < 2; ++g) (void)hipFree(p->d_cols[g]);
  (void)hipFree(p->d_norm);
  (void)hipFree(p->d_m1);
  (void)hipFree(p->d_partial);
  (void)hipFree(p->d_gram);
  (void)hipFree(p->d_chunks);
  (void)hipFree(p->d_flags);
  (void)hipFree(p->d_rows_tmp);
  (void)hipFree(p->d_ok_tmp);
  for (hipEvent_t e : p->seg_events) (void)hipEventDestroy(e);
  delete p;
}

int ob_panel_row_len(const ob_panel* p) { return p ? p->row_len : 0; }
int ob_panel_k(const ob_panel* p) { return p ? p->k : 0; }
int ob_panel_n_base(const ob_panel* p) { return p ? p->norm.n_base : 0; }

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
  return ob::engine_point_estimate(p, ref_mode, row, resid_b);
}

int ob_boot_run_device(ob_panel* p, uint64_t seed, uint64_t first_rep, uint64_t n_reps, int ref_mode,
                       double* d_rows, uint8_t* d_ok, void* hip_stream) {
  if (!p || (n_reps && (!d_rows || !d_ok))) return ob::fail(OB_E_INVALID, "null pointer");
  if (!valid_ref(ref_mode)) return ob::fail(OB_E_INVALID, "unknown reference coefficients %d", ref_mode);
  if (p->n[0] == 0 || p->n[1] == 0)
    return ob::fail(OB_E_GROUP, "%sOne group has no data", ob::error_prefix(OB_E_GROUP));
  if (p->ntiles[0] > 40000 || p->ntiles[1] > 40000)
    return ob::fail(OB_E_UNSUPPORTED, "group too large for the LDS level-1 histogram");
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
    HIP_OK(hipMalloc(&p->d_rows_tmp, sizeof(double) * n_reps * p->row_len));
    HIP_OK(hipMalloc(&p->d_ok_tmp, n_reps));
    p->tmp_reps = n_reps;
  }
  OB_TRY(ob_boot_run_device(p, seed, first_rep, n_reps, ref_mode, p->d_rows_tmp, p->d_ok_tmp, nullptr));
  OB_TRY(ob::engine_collect(p));
  HIP_OK(hipMemcpy(rows, p->d_rows_tmp, sizeof(double) * n_reps * p->row_len, hipMemcpyDeviceToHost));
  HIP_OK(hipMemcpy(ok, p->d_ok_tmp, n_reps, hipMemcpyDeviceToHost));
  return OB_OK;
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
