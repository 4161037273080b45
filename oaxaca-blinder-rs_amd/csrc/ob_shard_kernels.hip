// ob_shard_kernels.hip -- the pack / unpack kernels around the sharded run's RCCL all-gather
// (ob_shard.cpp; buffer layouts and offsets: ob_shard_layout.h, shared with the CPU tests).
#include <hip/hip_runtime.h>

#include <algorithm>

#include "ob_engine.hpp"
#include "ob_shard_layout.h"

namespace {

using Shard = ob_shard_range;

// shard rows [t][count][rl] -> send [t][per][nc] (the gathered columns; positions past count are
// zero rows with ok 0). Offsets: ob_shard_layout.h.
__global__ __launch_bounds__(256) void sh_pack_kernel(const double* rows, const uint8_t* ok, Shard s, int rl, int nc,
                                                      const int32_t* cols, int n_y, double* send, uint8_t* send_ok) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  const size_t per_t = s.per * (size_t)nc;
  if (i < (size_t)n_y * per_t) {
    const int t = (int)(i / per_t), q = (int)(i % (size_t)nc);
    const uint64_t pos = (i % per_t) / (size_t)nc;
    send[ob_send_off(s, t, pos, nc, q)] = pos < s.count ? rows[ob_shard_row_off(s, t, pos, rl, cols[q])] : 0.0;
  }
  if (i < (size_t)n_y * s.per) {
    const int t = (int)(i / s.per);
    const uint64_t pos = i % s.per;
    send_ok[ob_send_ok_off(s, t, pos)] = pos < s.count ? ok[ob_shard_ok_off(s, t, pos)] : (uint8_t)0;
  }
}

// recv [t][W per][nc] -> the caller's rows [t][n][rl]: gathered columns from recv, the others from
// this rank's own shard rows (own replicates) or NaN (the other ranks').
__global__ __launch_bounds__(256) void sh_unpack_kernel(const double* recv, const uint8_t* recv_ok, Shard s, int world,
                                                        uint64_t n_reps, int rl, int nc, const int32_t* cmap, int n_y,
                                                        const double* own, double* rows, uint8_t* ok) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  const size_t per_t = n_reps * (size_t)rl;
  if (i < (size_t)n_y * per_t) {
    const int t = (int)(i / per_t), c = (int)(i % (size_t)rl);
    const uint64_t j = (i % per_t) / (size_t)rl;
    const int q = cmap[c];
    double v;
    if (q >= 0) v = recv[ob_recv_off(s, world, t, j, nc, q)];
    else if (own && j >= s.lo && j < s.lo + s.count) v = own[ob_shard_row_off(s, t, j - s.lo, rl, c)];
    else v = __builtin_nan("");
    rows[ob_deliver_off(n_reps, t, j, rl, c)] = v;
  }
  if (i < (size_t)n_y * n_reps) {
    const int t = (int)(i / n_reps);
    const uint64_t j = i % n_reps;
    ok[(size_t)t * n_reps + j] = recv_ok[ob_recv_ok_off(s, world, t, j)];
  }
}

unsigned blocks_for(size_t n) { return (unsigned)std::max<size_t>(1, (n + 255) / 256); }

}  // namespace

namespace ob {

int shard_pack(const double* rows, const uint8_t* ok, const ob_shard_range& s, int rl, int nc, const int32_t* cols, int n_y,
               double* send, uint8_t* send_ok, hipStream_t st) {
  hipLaunchKernelGGL(sh_pack_kernel, dim3(blocks_for((size_t)n_y * s.per * nc)), dim3(256), 0, st, rows, ok, s, rl, nc,
                     cols, n_y, send, send_ok);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? OB_OK : ob::fail(OB_E_HIP, "HIP error %s at %s:%d", hipGetErrorString(e), __FILE__, __LINE__);
}

int shard_unpack(const double* recv, const uint8_t* recv_ok, const ob_shard_range& s, int world, uint64_t n_reps, int rl,
                 int nc, const int32_t* cmap, int n_y, const double* own, double* rows, uint8_t* ok, hipStream_t st) {
  hipLaunchKernelGGL(sh_unpack_kernel, dim3(blocks_for((size_t)n_y * n_reps * rl)), dim3(256), 0, st, recv, recv_ok, s,
                     world, n_reps, rl, nc, cmap, n_y, own, rows, ok);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? OB_OK : ob::fail(OB_E_HIP, "HIP error %s at %s:%d", hipGetErrorString(e), __FILE__, __LINE__);
}

}  // namespace ob
