// ob_device.hpp -- device helpers shared by the engine's kernel files: extended-Gram pair
// lookup and the one-wave Cholesky factor/solve in LDS (the solve kernels of ob_engine.hip and
// ob_heckman.hip).
#pragma once
#include <hip/hip_runtime.h>

#include "ob_spec.h"

namespace {

__device__ __forceinline__ double gpair(const double* g, int a, int b, int k1) {
  return a <= b ? g[ob_pair_index(a, b, k1)] : g[ob_pair_index(b, a, k1)];
}

// Synchronization of the one-wave routines below: the whole block (__syncthreads, one wave per
// block), or only the calling wave (WAVE: several waves of a block factor different matrices; LDS
// operations of one wave complete in issue order, so waiting for its own ones suffices).
template <bool WAVE>
__device__ __forceinline__ void ob_sync() {
  if constexpr (WAVE) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  else __syncthreads();
}

// nalgebra Cholesky::new order (left-looking, per-element updates in column order).
// Fails iff a pivot is zero, negative or NaN (!is_zero && try_sqrt). m: n x n col-major.
template <bool WAVE = false>
__device__ bool wave_cholesky(double* m, int n, int lane) {
  for (int j = 0; j < n; ++j) {
    for (int i = j + lane; i < n; i += 64) {
      double v = m[i + j * n];
      for (int c = 0; c < j; ++c) v = -m[j + c * n] * m[i + c * n] + v;
      m[i + j * n] = v;
    }
    ob_sync<WAVE>();
    const double diag = m[j + j * n];
    if (!(diag != 0.0 && diag >= 0.0)) return false;
    const double den = sqrt(diag);
    ob_sync<WAVE>();
    for (int i = j + lane; i < n; i += 64) m[i + j * n] = (i == j) ? den : m[i + j * n] / den;
    ob_sync<WAVE>();
  }
  return true;
}

template <bool WAVE = false>
__device__ void wave_chol_solve(const double* l, int n, double* b, int lane) {
  for (int i = 0; i < n; ++i) {
    const double coeff = b[i] / l[i + i * n];
    ob_sync<WAVE>();
    for (int r = i + 1 + lane; r < n; r += 64) b[r] -= coeff * l[r + i * n];
    if (lane == 0) b[i] = coeff;
    ob_sync<WAVE>();
  }
  for (int i = n - 1; i >= 0; --i) {
    double part = 0.0;
    for (int r = i + 1 + lane; r < n; r += 64) part += l[r + i * n] * b[r];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) part += __shfl_xor(part, off);
    if (lane == 0) b[i] = (b[i] - part) / l[i + i * n];
    ob_sync<WAVE>();
  }
}

}  // namespace
