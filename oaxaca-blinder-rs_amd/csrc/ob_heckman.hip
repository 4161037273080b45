// ob_heckman.hip -- the Heckman two-step per replicate (builder .heckman_selection):
//   probit of s on [1, z] by Fisher scoring from 0 (math/probit.rs:25-170),
//   IMR lambda = phi/Phi on the selected rows, OLS of y on [1, x, lambda] over them
//   (heckman.rs:38-108, estimation.rs:114-260), beta* and the decomposition over K + 1 terms,
//   and the selection terms theta_ref delta_ref gamma_ref,j (zbar_A,j - zbar_B,j) (builder.rs:477-534).
//
// A replicate's resample enters through the same level-2 count images as the Gram kernel: every
// sum below is sum_i c_i f(row i). The selected-row normal matrix [X'X | X'y] is the engine's
// extended Gram with weights [s == 1]; only the IMR column needs per-replicate transcendental work.
//
// Kernels (one block per (row chunk, 64-replicate batch) unless noted; lane = replicate, wave =
// 64-row sub-tile of each 256-row tile, so a wave's panel reads are uniform and count reads are
// one word per 4 rows):
//   ob_probit_kernel<KS>      per iteration: sum c w z z', sum c lambda z (w, lambda per probit.rs)
//   ob_probit_step_kernel<KS> thread per (replicate, group): chunk sums in a fixed order, the
//                             nalgebra Cholesky step (LU fallback), convergence flag
//   ob_heck_sums_kernel<NB>   sum c lambda [1, x, y], c lambda^2, c lambda (lambda + z'gamma) over
//                             selected rows; sum c z, c w y, c w over all rows
//   ob_heck_solve_kernel      wave per replicate: [X'X, X'lambda; lambda'X, lambda'lambda] Cholesky,
//                             beta*, decomposition, selection terms
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <type_traits>

#include "ob_device.hpp"
#include "ob_engine.hpp"
#include "ob_heckman.hpp"
#include "ob_options.hpp"
#include "ob_spec.h"

namespace {

constexpr int kHB = 256;
constexpr uint32_t kDone = 1u, kFailed = 2u;

#define HK_OK(expr)                                                                      \
  do {                                                                                   \
    hipError_t e_ = (expr);                                                              \
    if (e_ != hipSuccess)                                                                \
      return ob::fail(OB_E_HIP, "HIP error %s at %s:%d", hipGetErrorString(e_), __FILE__, \
                      __LINE__);                                                         \
  } while (0)

// statrs Normal(0, 1): pdf = exp(-z^2 / 2) / sqrt(2 pi), cdf = erfc(-z / sqrt 2) / 2.
// (The constant divisions are multiplications by the reciprocals: a last-bit difference.)
__device__ __forceinline__ double npdf(double z) { return exp(-0.5 * z * z) * 0.3989422804014327; }
__device__ __forceinline__ double ncdf(double z) { return 0.5 * erfc(-z * 0.7071067811865476); }

// pdf and cdf together from one exp(-z^2 / 2) (OB_HK_ERFC=1): erfc(x), x = -z / sqrt 2, by W. J.
// Cody's rational Chebyshev approximations (Math. Comp. 23 (1969), the CALERF regions |x| < 0.46875,
// <= 4, > 4), whose two outer regions are exp(-x^2) times a rational function -- exp(-x^2) is the
// pdf's exp(-z^2 / 2). Checked against scipy's erfc on z in [-12, 12]: at most 3e-14 relative (the
// rounding of z^2 inside the shared exp, amplified at large |z|; about 1e-15 where the clamped
// probabilities are used).
__device__ __forceinline__ double nd_rcp(double v) {  // 1/v within ~1 ulp (as hk_rcp below)
  double r = __builtin_amdgcn_rcp(v);
  r = fma(fma(-v, r, 1.0), r, r);
  return fma(fma(-v, r, 1.0), r, r);
}
__device__ __forceinline__ void npdf_ncdf(double z, double& pdf, double& cdf) {
  const double x = -z * 0.7071067811865476, y = fabs(x);
  const double e = exp(-0.5 * z * z);
  pdf = e * 0.3989422804014327;
  double r;
  if (y <= 0.46875) {
    const double ysq = y * y;
    double xn = 1.85777706184603153e-1 * ysq, xd = ysq;
    xn = (xn + 3.16112374387056560e00) * ysq;
    xd = (xd + 2.36012909523441209e01) * ysq;
    xn = (xn + 1.13864154151050156e02) * ysq;
    xd = (xd + 2.44024637934444173e02) * ysq;
    xn = (xn + 3.77485237685302021e02) * ysq;
    xd = (xd + 1.28261652607737228e03) * ysq;
    cdf = 0.5 * (1.0 - x * (xn + 3.20937758913846947e03) * nd_rcp(xd + 2.84423683343917062e03));
    return;
  }
  if (y <= 4.0) {
    double xn = 2.15311535474403846e-8 * y, xd = y;
    xn = (xn + 5.64188496988670089e-1) * y;
    xd = (xd + 1.57449261107098347e01) * y;
    xn = (xn + 8.88314979438837594e00) * y;
    xd = (xd + 1.17693950891312499e02) * y;
    xn = (xn + 6.61191906371416295e01) * y;
    xd = (xd + 5.37181101862009858e02) * y;
    xn = (xn + 2.98635138197400131e02) * y;
    xd = (xd + 1.62138957456669019e03) * y;
    xn = (xn + 8.81952221241769090e02) * y;
    xd = (xd + 3.29079923573345963e03) * y;
    xn = (xn + 1.71204761263407058e03) * y;
    xd = (xd + 4.36261909014324716e03) * y;
    xn = (xn + 2.05107837782607147e03) * y;
    xd = (xd + 3.43936767414372164e03) * y;
    r = (xn + 1.23033935479799725e03) * nd_rcp(xd + 1.23033935480374942e03) * e;
  } else {
    const double iy = nd_rcp(y), ysq = iy * iy;
    double xn = 1.63153871373020978e-2 * ysq, xd = ysq;
    xn = (xn + 3.05326634961232344e-1) * ysq;
    xd = (xd + 2.56852019228982242e00) * ysq;
    xn = (xn + 3.60344899949804439e-1) * ysq;
    xd = (xd + 1.87295284992346725e00) * ysq;
    xn = (xn + 1.25781726111229246e-1) * ysq;
    xd = (xd + 5.27905102951428412e-1) * ysq;
    xn = (xn + 1.60837851487422766e-2) * ysq;
    xd = (xd + 6.05183413124413191e-2) * ysq;
    r = ysq * (xn + 6.58749161529837803e-4) * nd_rcp(xd + 2.33520497626869185e-3);
    r = (5.6418958354775628695e-1 - r) * iy * e;
  }
  cdf = 0.5 * (x >= 0.0 ? r : 2.0 - r);
}

// The probit and sums kernels take pdf and cdf from npdf_ncdf (one exp per row; probit launch 11.8
// -> 9.0 ms at configs[1] + selection, profiles/r04_ab_heckman_erfc.txt) unless option hk_erfc = 0
// (ob_set_option), which keeps the library's erfc beside a second exp.
inline bool hk_cody() { return ob::opt_int(ob::Opt::HkErfc, 1) != 0; }

// 1/v within ~1 ulp: v_rcp_f64 and two Newton steps instead of the IEEE division sequence (the
// operands are normal numbers: clamped probabilities).
__device__ __forceinline__ double hk_rcp(double v) {
  double r = __builtin_amdgcn_rcp(v);
  r = fma(fma(-v, r, 1.0), r, r);
  return fma(fma(-v, r, 1.0), r, r);
}

// f64::clamp: NaN stays NaN.
__device__ __forceinline__ double clamp_phi(double v) {
  return v < 1e-10 ? 1e-10 : (v > 1.0 - 1e-10 ? 1.0 - 1e-10 : v);
}

struct Lanes {
  uint32_t g, t0, t1, rep, rb;
  int wave, lane;
};

__device__ __forceinline__ Lanes lanes(const ob_heck_seg& a) {
  Lanes l;
  l.lane = threadIdx.x & 63;
  l.wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t chunk = blockIdx.x;
  l.rb = blockIdx.y;
  l.g = a.chunks[3 * chunk];
  l.t0 = a.chunks[3 * chunk + 1];
  l.t1 = a.chunks[3 * chunk + 2];
  l.rep = l.rb * 64 + l.lane;
  return l;
}

// This lane's count words for the wave's sub-tile of a tile (NULL: every row once). f64 Gram
// images: 16 consecutive words at lane * 17. I8 images (ob_count_kernel<true>, the A fragments of
// ob_gram_i8.hip: per sub-tile [16-replicate block][lane][16 B], lane = replicate 16 m + (l & 15),
// rows 16 (l >> 4) + j): the lane's rows 16 q .. 16 q + 15 are the 16-byte unit 16 q past the
// returned one (count_word).
__device__ __forceinline__ const uint32_t* count_row(const ob_heck_seg& a, const Lanes& l, uint32_t tile) {
  if (!a.counts) return nullptr;
  const size_t tt = (l.g ? a.tiles0 : 0u) + tile;
  if (a.counts_i8)
    return a.counts + ((tt * a.nb_rep + l.rb) * 1024 + l.wave * 256 + (l.lane >> 4) * 64 + (l.lane & 15)) * 4;
  return a.counts + ((tt * a.nb_rep + l.rb) * 4 + l.wave) * kCimgWords + l.lane * kCimgStride;
}

// Count bytes of the lane's rows ri .. ri + 3 of its sub-tile (ri % 4 == 0).
__device__ __forceinline__ uint32_t count_word(const ob_heck_seg& a, const uint32_t* cw, uint32_t ri) {
  if (!cw) return 0x01010101u;
  return a.counts_i8 ? cw[(ri >> 4) * 64 + ((ri >> 2) & 3u)] : cw[ri >> 2];
}

// Fixed-order block sum of acc over the 4 waves into LDS row `lane` (wave 3 + 2 + 1, then + 0).
template <int N>
__device__ __forceinline__ void block_sum(double (&acc)[N], double* red, const Lanes& l) {
#pragma unroll 1
  for (int w = 3; w >= 1; --w) {
    if (l.wave == w)
#pragma unroll
      for (int i = 0; i < N; ++i) red[l.lane * (N + 1) + i] = (w == 3 ? 0.0 : red[l.lane * (N + 1) + i]) + acc[i];
    __syncthreads();
  }
  if (l.wave == 0)
#pragma unroll
    for (int i = 0; i < N; ++i) acc[i] = red[l.lane * (N + 1) + i] + acc[i];
}

// The wave's 64-row sub-tile of `ncol` consecutive panel columns (from `src`) -> LDS [col][64]: one
// coalesced load per column instead of a scalar load per row and column; the wave then reads its
// rows at uniform LDS addresses. Wave-local (LDS operations of one wave complete in order).
__device__ __forceinline__ void wave_stage(double* stg, const double* src, int64_t ld, uint32_t r0, uint32_t nr,
                                           int ncol, int lane) {
  __builtin_amdgcn_wave_barrier();
  for (int c = 0; c < ncol; ++c) stg[c * 64 + lane] = (uint32_t)lane < nr ? src[(size_t)c * ld + r0 + lane] : 0.0;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

template <int KS, bool CODY>
__global__ __launch_bounds__(kHB) void ob_probit_kernel(const ob_heck_seg a) {
  constexpr int NH = KS * (KS + 1) / 2, NP = NH + KS;
  __shared__ double red[64 * (NP + 1)];
  __shared__ double stage[4 * KS * 64];  // per wave: s, z_1..z_{KS-1} of its sub-tile
  const Lanes l = lanes(a);
  const size_t st = (size_t)l.g * a.rep_pad + l.rep;
  const bool act = l.rep < a.n_reps && !(a.hflags[st] & kDone);
  if (!__syncthreads_or(act)) return;
  double gam[KS];
#pragma unroll
  for (int j = 0; j < KS; ++j) gam[j] = act ? a.gamma[st * KS + j] : 0.0;
  double acc[NP];
#pragma unroll
  for (int i = 0; i < NP; ++i) acc[i] = 0.0;
  const double* X = a.cols[l.g];
  const int64_t ld = a.ld[l.g];
  const uint32_t n = a.n[l.g];
  const double* SZ = X + (size_t)(a.p + 2) * ld;  // s, then z_1..z_{KS-1}: consecutive columns
  double* stg = stage + l.wave * (KS * 64);
  for (uint32_t tile = l.t0; tile < l.t1; ++tile) {
    const uint32_t r0 = tile * OB_TILE_ROWS + l.wave * 64;
    if (r0 >= n) break;
    const uint32_t nr = min(64u, n - r0);
    wave_stage(stg, SZ, ld, r0, nr, KS, l.lane);
    const uint32_t* cw = count_row(a, l, tile);
    uint32_t word = 0;
    for (uint32_t ri = 0; ri < nr; ++ri) {
      if ((ri & 3) == 0) word = count_word(a, cw, ri);
      const uint32_t cu = (word >> ((ri & 3) * 8)) & 255u;
      if (!act || cu == 0) continue;
      const double c = (double)cu;
      double z[KS];
      z[0] = 1.0;
#pragma unroll
      for (int j = 1; j < KS; ++j) z[j] = stg[j * 64 + ri];
      double zg = 0.0;
#pragma unroll
      for (int j = 0; j < KS; ++j) zg += z[j] * gam[j];
      double phi, bp;
      if constexpr (CODY) {
        npdf_ncdf(zg, phi, bp);
        bp = clamp_phi(bp);
      } else {
        phi = npdf(zg);
        bp = clamp_phi(ncdf(zg));
      }
      // one reciprocal: r = 1 / (Phi (1 - Phi)), so 1 / Phi = (1 - Phi) r, 1 / (1 - Phi) = Phi r and
      // the weight phi^2 / (Phi (1 - Phi)) = phi^2 r
      const double qb = 1.0 - bp, r = hk_rcp(bp * qb);
      const double lam = stg[ri] > 0.5 ? phi * (qb * r) : -phi * (bp * r);  // probit.rs:66-70
      const double cwt = c * (phi * phi * r), cl = c * lam;  // sqrt_w^2 of probit.rs:75-76
      int e = 0;
#pragma unroll
      for (int j = 0; j < KS; ++j) {
        const double t = cwt * z[j];
#pragma unroll
        for (int k = 0; k <= j; ++k) acc[e++] += t * z[k];
      }
#pragma unroll
      for (int j = 0; j < KS; ++j) acc[NH + j] += cl * z[j];
    }
  }
  block_sum(acc, red, l);
  if (l.wave == 0 && l.rep < a.n_reps)
#pragma unroll
    for (int i = 0; i < NP; ++i) a.partial[((size_t)blockIdx.x * a.rep_pad + l.rep) * NP + i] = acc[i];
}

// nalgebra LU (partial pivoting on the first largest |pivot|) + solve; false if U is singular.
template <int KS>
__device__ bool lu_solve(double (&m)[KS * KS], double (&b)[KS]) {
  int perm[KS];
#pragma unroll
  for (int i = 0; i < KS; ++i) perm[i] = i;
  bool ok = true;
#pragma unroll
  for (int i = 0; i < KS; ++i) {
    int piv = i;
    double best = fabs(m[i + i * KS]);
#pragma unroll
    for (int r = i + 1; r < KS; ++r)
      if (fabs(m[r + i * KS]) > best) {
        best = fabs(m[r + i * KS]);
        piv = r;
      }
    // select-based swaps keep every index compile-time (registers, no scratch)
#pragma unroll
    for (int r = i + 1; r < KS; ++r)
      if (r == piv) {
#pragma unroll
        for (int c = 0; c < KS; ++c) {
          const double t = m[i + c * KS];
          m[i + c * KS] = m[r + c * KS];
          m[r + c * KS] = t;
        }
        const int t = perm[i];
        perm[i] = perm[r];
        perm[r] = t;
      }
    const double d = m[i + i * KS];
    if (d == 0.0) {
      ok = false;
      continue;
    }
#pragma unroll
    for (int r = i + 1; r < KS; ++r) m[r + i * KS] /= d;
#pragma unroll
    for (int c = i + 1; c < KS; ++c)
#pragma unroll
      for (int r = i + 1; r < KS; ++r) m[r + c * KS] += -m[i + c * KS] * m[r + i * KS];
  }
  if (!ok) return false;
  double x[KS];
#pragma unroll
  for (int i = 0; i < KS; ++i) {
    double v = 0.0;
#pragma unroll
    for (int r = 0; r < KS; ++r)
      if (perm[i] == r) v = b[r];
    x[i] = v;
  }
#pragma unroll
  for (int i = 0; i < KS; ++i)
#pragma unroll
    for (int r = i + 1; r < KS; ++r) x[r] += -x[i] * m[r + i * KS];
#pragma unroll
  for (int i = KS - 1; i >= 0; --i) {
    x[i] /= m[i + i * KS];
#pragma unroll
    for (int r = 0; r < i; ++r) x[r] += -x[i] * m[r + i * KS];
  }
#pragma unroll
  for (int i = 0; i < KS; ++i) b[i] = x[i];
  return true;
}

template <int KS>
__global__ __launch_bounds__(64) void ob_probit_step_kernel(const ob_heck_seg a) {
  constexpr int NH = KS * (KS + 1) / 2, NP = NH + KS;
  const uint32_t rep = blockIdx.x * 64 + threadIdx.x, g = blockIdx.y;
  if (rep >= a.n_reps) return;
  const size_t st = (size_t)g * a.rep_pad + rep;
  const uint32_t fl = a.hflags[st];
  if (fl & kDone) return;
  double sum[NP];
#pragma unroll
  for (int i = 0; i < NP; ++i) sum[i] = 0.0;
  for (int c = 0; c < a.n_chunks; ++c) {
    if (a.chunks[3 * c] != g) continue;
    const double* pp = a.partial + ((size_t)c * a.rep_pad + rep) * NP;
#pragma unroll
    for (int i = 0; i < NP; ++i) sum[i] += pp[i];
  }
  // -H = sum c w z z' + 1e-9 I (probit.rs:95-118), g = sum c lambda z
  double m[KS * KS], l[KS * KS], b[KS];
  int e = 0;
#pragma unroll
  for (int j = 0; j < KS; ++j)
#pragma unroll
    for (int k = 0; k <= j; ++k) {
      m[j + k * KS] = sum[e];
      m[k + j * KS] = sum[e];
      ++e;
    }
#pragma unroll
  for (int j = 0; j < KS; ++j) {
    m[j + j * KS] += 1e-9;
    b[j] = sum[NH + j];
  }
#pragma unroll
  for (int i = 0; i < KS * KS; ++i) l[i] = m[i];
  bool chol = true;
#pragma unroll
  for (int j = 0; j < KS; ++j) {  // nalgebra Cholesky::new order
#pragma unroll
    for (int i = j; i < KS; ++i) {
      double v = l[i + j * KS];
#pragma unroll
      for (int c = 0; c < j; ++c) v = -l[j + c * KS] * l[i + c * KS] + v;
      l[i + j * KS] = v;
    }
    const double diag = l[j + j * KS];
    if (!(diag != 0.0 && diag >= 0.0)) chol = false;
    const double den = sqrt(diag);
#pragma unroll
    for (int i = j + 1; i < KS; ++i) l[i + j * KS] /= den;
    l[j + j * KS] = den;
  }
  double step[KS];
#pragma unroll
  for (int i = 0; i < KS; ++i) step[i] = b[i];
  if (chol) {
#pragma unroll
    for (int i = 0; i < KS; ++i) {
      const double coeff = step[i] / l[i + i * KS];
#pragma unroll
      for (int r = i + 1; r < KS; ++r) step[r] -= coeff * l[r + i * KS];
      step[i] = coeff;
    }
#pragma unroll
    for (int i = KS - 1; i >= 0; --i) {
      double part = 0.0;
#pragma unroll
      for (int r = i + 1; r < KS; ++r) part += l[r + i * KS] * step[r];
      step[i] = (step[i] - part) / l[i + i * KS];
    }
  } else if (!lu_solve<KS>(m, step)) {  // probit.rs:124-137: -(H^-1 g) = (-H)^-1 g
    a.hflags[st] = kDone | kFailed;
    return;
  }
  double nrm = 0.0;
#pragma unroll
  for (int i = 0; i < KS; ++i) {
    a.gamma[st * KS + i] += step[i];
    nrm += step[i] * step[i];
  }
  if (sqrt(nrm) < 1e-6)
    a.hflags[st] = kDone;
  else
    atomicAdd(a.active, 1u);
}

// Staged columns per row of the sums kernel: x_1..x_p, y, [s == 1], s, z_1..z_{ks-1}, (w).
__host__ __device__ inline int heck_sums_cols(int p, int ks, int weighted) { return p + 2 + ks + (weighted ? 1 : 0); }

template <int NB, bool CODY>
__global__ __launch_bounds__(kHB) void ob_heck_sums_kernel(const ob_heck_seg a) {
  extern __shared__ __attribute__((aligned(16))) double hsm[];
  double* red = hsm;  // [64][NB + 1], then the waves' staged sub-tiles
  const Lanes l = lanes(a);
  const bool act = l.rep < a.n_reps;
  if (!__syncthreads_or(act)) return;
  const int K = a.p + 1, nhs = ob::heck_sums_len(K), ks = a.ks;
  const size_t st = (size_t)l.g * a.rep_pad + l.rep;
  double gam[ob::kHeckMaxKs];
#pragma unroll
  for (int j = 0; j < ob::kHeckMaxKs; ++j) gam[j] = (act && j < ks) ? a.gamma[st * ks + j] : 0.0;
  double acc[NB];
#pragma unroll
  for (int i = 0; i < NB; ++i) acc[i] = 0.0;
  const double* X = a.cols[l.g];
  const int64_t ld = a.ld[l.g];
  const uint32_t n = a.n[l.g];
  const int ncol = heck_sums_cols(a.p, ks, a.weighted), cy = a.p, cind = a.p + 1, cz = a.p + 2, cw8 = a.p + 2 + ks;
  double* stg = hsm + 64 * (NB + 1) + l.wave * (ncol * 64);
  for (uint32_t tile = l.t0; tile < l.t1; ++tile) {
    const uint32_t r0 = tile * OB_TILE_ROWS + l.wave * 64;
    if (r0 >= n) break;
    const uint32_t nr = min(64u, n - r0);
    wave_stage(stg, X, ld, r0, nr, ncol, l.lane);
    const uint32_t* cw = count_row(a, l, tile);
    uint32_t word = 0;
    for (uint32_t ri = 0; ri < nr; ++ri) {
      if ((ri & 3) == 0) word = count_word(a, cw, ri);
      const uint32_t cu = (word >> ((ri & 3) * 8)) & 255u;
      if (!act || cu == 0) continue;
      const double c = (double)cu;
      double z[ob::kHeckMaxKs];
      z[0] = 1.0;
#pragma unroll
      for (int j = 1; j < ob::kHeckMaxKs; ++j) z[j] = j < ks ? stg[(cz + j) * 64 + ri] : 0.0;
      double zg = 0.0;
#pragma unroll
      for (int j = 0; j < ob::kHeckMaxKs; ++j)
        if (j < ks) zg += z[j] * gam[j];
#pragma unroll
      for (int j = 0; j < ob::kHeckMaxKs; ++j) acc[5 + j] += c * z[j];  // selection means (all rows)
      const double y = stg[cy * 64 + ri], w = a.weighted ? stg[cw8 * 64 + ri] : 1.0;
      acc[3] += c * w * y;  // total gap (builder.rs:676-684, all rows)
      acc[4] += c * w;
      if (stg[cind * 64 + ri] == 1.0) {  // heckman.rs:56-69: lambda = phi / Phi, 0 when Phi < 1e-10
        double pd, bp;
        if constexpr (CODY) {
          npdf_ncdf(zg, pd, bp);
        } else {
          pd = npdf(zg);
          bp = ncdf(zg);
        }
        const double lam = bp < 1e-10 ? 0.0 : pd * hk_rcp(bp);
        const double cl = c * lam;
        acc[0] += cl * y;
        acc[1] += cl * lam;
        acc[2] += cl * (lam + zg);
        acc[13] += cl;
#pragma unroll
        for (int j = 1; j < NB - 13; ++j)
          if (j < K) acc[13 + j] += cl * stg[(j - 1) * 64 + ri];
      }
    }
  }
  block_sum(acc, red, l);
  if (l.wave == 0 && act)
#pragma unroll
    for (int i = 0; i < NB; ++i)
      if (i < nhs) a.partial[((size_t)blockIdx.x * a.rep_pad + l.rep) * nhs + i] = acc[i];
}

size_t heck_solve_lds(const ob_heck_seg& a) {
  const int K = a.p + 1, kp = K + 1;
  return sizeof(double) * ((size_t)kp * kp + 7 * (size_t)kp + 2 * (size_t)ob::heck_sums_len(K) + 4);
}

// Sums layout (per group): [0] c lam y, [1] c lam^2, [2] c lam (lam + z'g), [3] c w y, [4] c w,
// [5..13) c z_j, [13..13+K) c lam x_j (x_0 = 1).
__global__ __launch_bounds__(64) void ob_heck_solve_kernel(const ob_heck_seg a) {
  extern __shared__ __attribute__((aligned(16))) double sm[];
  const int lane = threadIdx.x;
  const uint32_t rep = blockIdx.x;
  if (rep >= a.n_reps) return;
  const int K = a.p + 1, kp = K + 1, nhs = ob::heck_sums_len(K), ks = a.ks;
  double* M = sm;
  double* rhs = M + kp * kp;
  double* beta_a = rhs + kp;
  double* beta_b = beta_a + kp;
  double* xam = beta_b + kp;
  double* xbm = xam + kp;
  double* bstar = xbm + kp;
  double* S = bstar + kp;      // [2][nhs]
  double* delta = S + 2 * nhs;  // [2]
  for (int i = lane; i < 2 * nhs; i += 64) {
    const uint32_t g = (uint32_t)(i / nhs);
    const int j = i % nhs;
    double v = 0.0;
    for (int c = 0; c < a.n_chunks; ++c)
      if (a.chunks[3 * c] == g) v += a.partial[((size_t)c * a.rep_pad + rep) * nhs + j];
    S[i] = v;
  }
  __syncthreads();
  const double* GA = a.gram + (size_t)rep * 2 * a.e_pad;
  const double* GB = GA + a.e_pad;
  double* row = a.rows + (size_t)rep * a.row_len;
  uint8_t status = OB_HS_OK;
  if (GA[0] == 0.0 || GB[0] == 0.0) status = OB_HS_NO_OUTCOMES;  // estimation.rs:124-125
  for (int g = 0; g < 2 && status == OB_HS_OK; ++g) {
    if (a.hflags[(size_t)g * a.rep_pad + rep] & kFailed) {
      status = OB_HS_PROBIT;
      break;
    }
    const double* G = g ? GB : GA;
    const double* Sg = S + g * nhs;
    const double nsel = G[0];
    if (nsel <= (double)kp) {  // ols.rs:98-104
      status = OB_HS_INSUFFICIENT;
      break;
    }
    for (int i = lane; i < kp * kp; i += 64) {
      const int r = i % kp, c = i / kp;
      double v;
      if (r < K && c < K)
        v = gpair(G, r, c, a.k1);
      else if (r == K && c == K)
        v = Sg[1];
      else
        v = Sg[13 + (r == K ? c : r)];
      M[r + c * kp] = v;
    }
    for (int i = lane; i < kp; i += 64) rhs[i] = i < K ? gpair(G, i, K, a.k1) : Sg[0];
    __syncthreads();
    if (!wave_cholesky(M, kp, lane)) {
      status = OB_HS_CHOLESKY;
      break;
    }
    wave_chol_solve(M, kp, rhs, lane);
    double* beta = g ? beta_b : beta_a;
    double* xm = g ? xbm : xam;
    for (int i = lane; i < kp; i += 64) {
      beta[i] = rhs[i];
      xm[i] = i < K ? gpair(G, 0, i, a.k1) / nsel : Sg[13] / nsel;  // row means + IMR mean
    }
    if (lane == 0) delta[g] = -Sg[2] / nsel;  // heckman.rs:92-99
    __syncthreads();
  }
  if (status == OB_HS_OK) {  // beta* (builder.rs:536-621; Pooled/Neumark are refused on the host)
    if (a.ref_mode == OB_REF_GROUP_A || a.ref_mode == OB_REF_GROUP_B) {
      const double* src = a.ref_mode == OB_REF_GROUP_A ? beta_a : beta_b;
      for (int i = lane; i < kp; i += 64) bstar[i] = src[i];
    } else {
      const double sa = S[4], sb = S[nhs + 4];
      const double tot = sa + sb;
      if (tot == 0.0) {
        status = OB_HS_ZERO_WEIGHT;
      } else {
        const double wA = sa / tot, wB = 1.0 - wA;
        for (int i = lane; i < kp; i += 64) bstar[i] = beta_a[i] * wA + beta_b[i] * wB;
      }
    }
  }
  __syncthreads();
  if (lane == 0) {
    if (status != OB_HS_OK) {
      for (int i = 0; i < a.row_len; ++i) row[i] = __builtin_nan("");
    } else {
      double* dex = row + 6;
      double* dun = row + 6 + kp;
      double expl = 0.0, ta = 0.0, tb = 0.0, endow = 0.0, coef = 0.0, inter = 0.0;
      for (int j = 0; j < kp; ++j) {  // decomposition.rs:56-89
        const double dx = xam[j] - xbm[j], db = beta_a[j] - beta_b[j];
        expl += dx * bstar[j];
        ta += xam[j] * beta_a[j];
        tb += xbm[j] * beta_b[j];
        endow += dx * beta_b[j];
        coef += xbm[j] * db;
        inter += dx * db;
      }
      for (int j = 0; j < kp; ++j) {  // decomposition.rs:92-122
        dex[j] = (xam[j] - xbm[j]) * bstar[j];
        dun[j] = xam[j] * (beta_a[j] - bstar[j]) + xbm[j] * (bstar[j] - beta_b[j]);
      }
      row[0] = expl;
      row[1] = (ta - tb) - expl;
      row[2] = endow;
      row[3] = coef;
      row[4] = inter;
      row[5] = S[3] / S[4] - S[nhs + 3] / S[nhs + 4];
      double* tail = row + 6 + 2 * kp;
      for (int j = 0; j < kp; ++j) {
        tail[j] = beta_a[j];
        tail[kp + j] = beta_b[j];
        tail[2 * kp + j] = xam[j];
        tail[3 * kp + j] = xbm[j];
        tail[4 * kp + j] = bstar[j];
      }
      // selection terms (builder.rs:510-530): A's (theta, delta, gamma) for GroupA, else B's
      const int gr = a.ref_mode == OB_REF_GROUP_A ? 0 : 1;
      const double theta = gr ? beta_b[K] : beta_a[K];
      const double* gam = a.gamma + ((size_t)gr * a.rep_pad + rep) * ks;
      double* sel = tail + 5 * kp;
      for (int j = 0; j < ks; ++j) {
        const double za = S[5 + j] / S[5], zb = S[nhs + 5 + j] / S[nhs + 5];
        sel[j] = theta * delta[gr] * gam[j] * (za - zb);
      }
    }
    a.ok[rep] = a.raw_status ? status : (uint8_t)(status == OB_HS_OK);
  }
}

template <int KS>
hipError_t launch_probit_iter(const ob_heck_seg& a, hipStream_t s, hipEvent_t* ev) {
  if (ev) (void)hipEventRecord(ev[0], s);
  if (hk_cody())
    hipLaunchKernelGGL((ob_probit_kernel<KS, true>), dim3(a.n_chunks, a.rep_pad / 64), dim3(kHB), 0, s, a);
  else
    hipLaunchKernelGGL((ob_probit_kernel<KS, false>), dim3(a.n_chunks, a.rep_pad / 64), dim3(kHB), 0, s, a);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  if (ev) (void)hipEventRecord(ev[1], s);
  hipLaunchKernelGGL(ob_probit_step_kernel<KS>, dim3(a.rep_pad / 64, 2), dim3(64), 0, s, a);
  return hipGetLastError();
}

hipError_t probit_iter(const ob_heck_seg& a, hipStream_t s, hipEvent_t* ev) {
  switch (a.ks) {
    case 1: return launch_probit_iter<1>(a, s, ev);
    case 2: return launch_probit_iter<2>(a, s, ev);
    case 3: return launch_probit_iter<3>(a, s, ev);
    case 4: return launch_probit_iter<4>(a, s, ev);
    case 5: return launch_probit_iter<5>(a, s, ev);
    case 6: return launch_probit_iter<6>(a, s, ev);
    case 7: return launch_probit_iter<7>(a, s, ev);
    default: return launch_probit_iter<8>(a, s, ev);
  }
}

}  // namespace

namespace ob {

int heckman_segment(const ob_heck_seg& a, hipStream_t s, int* iters, ob_heck_times* tm) {
  if (a.ks < 1 || a.ks > kHeckMaxKs || a.p > kHeckMaxP || a.rep_pad % 64 != 0)
    return ob::fail(OB_E_INVALID, "heckman segment: bad shape");
  struct Events {  // [0, 1] around each probit pass, [2, 3] around the sums pass
    hipEvent_t e[4] = {};
    ~Events() {
      for (hipEvent_t x : e)
        if (x) (void)hipEventDestroy(x);
    }
  } ev;
  if (tm)
    for (hipEvent_t& x : ev.e) HK_OK(hipEventCreate(&x));
  HK_OK(hipMemsetAsync(a.gamma, 0, sizeof(double) * 2 * a.rep_pad * a.ks, s));
  HK_OK(hipMemsetAsync(a.hflags, 0, sizeof(uint32_t) * 2 * a.rep_pad, s));
  int it = 0;
  while (it < a.max_iter) {  // probit.rs:48-147, each replicate stopping on its own
    HK_OK(hipMemsetAsync(a.active, 0, sizeof(uint32_t), s));
    HK_OK(probit_iter(a, s, tm ? ev.e : nullptr));
    ++it;
    uint32_t active = 0;
    HK_OK(hipMemcpyAsync(&active, a.active, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    HK_OK(hipStreamSynchronize(s));
    if (tm) {
      float ms = 0.f;
      HK_OK(hipEventElapsedTime(&ms, ev.e[0], ev.e[1]));
      tm->probit_ms += ms;
      tm->probit_launches += 1;
    }
    if (active == 0) break;
  }
  if (iters) *iters = it;
  const dim3 grid(a.n_chunks, a.rep_pad / 64);
  const int nhs = heck_sums_len(a.p + 1);
  const int nb = nhs <= 32 ? 32 : (nhs <= 40 ? 40 : 64);
  const size_t lds_sums =
      sizeof(double) * (64 * (size_t)(nb + 1) + 4 * 64 * (size_t)heck_sums_cols(a.p, a.ks, a.weighted));
  const bool cody = hk_cody();
  auto sums = [&](auto nbc, auto cc) {
    constexpr int NB = decltype(nbc)::value;
    constexpr bool C = decltype(cc)::value;
    return (const void*)ob_heck_sums_kernel<NB, C>;
  };
  using T = std::true_type;
  using F = std::false_type;
  const void* fn = nb == 32   ? (cody ? sums(std::integral_constant<int, 32>{}, T{}) : sums(std::integral_constant<int, 32>{}, F{}))
                   : nb == 40 ? (cody ? sums(std::integral_constant<int, 40>{}, T{}) : sums(std::integral_constant<int, 40>{}, F{}))
                              : (cody ? sums(std::integral_constant<int, 64>{}, T{}) : sums(std::integral_constant<int, 64>{}, F{}));
  HK_OK(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_sums));
  if (tm) HK_OK(hipEventRecord(ev.e[2], s));
  void* args[] = {const_cast<ob_heck_seg*>(&a)};
  HK_OK(hipLaunchKernel(fn, grid, dim3(kHB), args, lds_sums, s));
  HK_OK(hipGetLastError());
  if (tm) HK_OK(hipEventRecord(ev.e[3], s));
  const size_t lds = heck_solve_lds(a);
  HK_OK(hipFuncSetAttribute((const void*)ob_heck_solve_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipLaunchKernelGGL(ob_heck_solve_kernel, dim3(a.n_reps), dim3(64), lds, s, a);
  HK_OK(hipGetLastError());
  if (tm) {  // the events die with this call: read the sums pass now
    float ms = 0.f;
    HK_OK(hipEventSynchronize(ev.e[3]));
    HK_OK(hipEventElapsedTime(&ms, ev.e[2], ev.e[3]));
    tm->sums_ms += ms;
  }
  return OB_OK;
}

}  // namespace ob

namespace {
__global__ void ob_normal_kernel(const double* z, int64_t n, double* pdf, double* cdf) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  double p, c;
  npdf_ncdf(z[i], p, c);
  pdf[i] = p;
  cdf[i] = c;
}
}  // namespace

// Test hook (include/oaxaca_boot.h): npdf_ncdf, the probit's phi and Phi (Cody's erfc with one
// shared exponential), evaluated on the device at z[0 .. n).
extern "C" int ob_debug_normal(int device, const double* z, int64_t n, double* pdf, double* cdf) {
  if (n < 0 || (n && (!z || !pdf || !cdf))) return ob::fail(OB_E_INVALID, "bad arguments");
  if (n == 0) return OB_OK;
  HK_OK(hipSetDevice(device));
  double* d = nullptr;
  HK_OK(hipMalloc(&d, sizeof(double) * 3 * (size_t)n));
  int rc = OB_OK;
  do {
    if (hipMemcpy(d, z, sizeof(double) * n, hipMemcpyHostToDevice) != hipSuccess) { rc = ob::fail(OB_E_HIP, "copy"); break; }
    hipLaunchKernelGGL(ob_normal_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, d, n, d + n, d + 2 * n);
    if (hipGetLastError() != hipSuccess || hipDeviceSynchronize() != hipSuccess) { rc = ob::fail(OB_E_HIP, "launch"); break; }
    if (hipMemcpy(pdf, d + n, sizeof(double) * n, hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(cdf, d + 2 * n, sizeof(double) * n, hipMemcpyDeviceToHost) != hipSuccess)
      rc = ob::fail(OB_E_HIP, "copy back");
  } while (0);
  (void)hipFree(d);
  return rc;
}
