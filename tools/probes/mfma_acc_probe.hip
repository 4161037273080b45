// Register-allocation probe for the wide i8 Gram (round 6): one wave per SIMD holding 4 x NS x NH
// v_mfma_i32_16x16x64_i8 accumulator tiles through a K loop, then the int64 slice combination.
// Build: hipcc --offload-arch=gfx950 -O3 -c mfma_acc_probe.hip -Rpass-analysis=kernel-resource-usage
// Measured (ROCm 7.2 hipcc): <6, 2> (192 accumulators) 256 VGPRs + 227 AGPRs, no spill; <6, 3> 162
// VGPRs spilled; <6, 4> (384) 324 spilled; <4, 4> 116; <5, 4> 25. The compiler keeps copies of
// accumulators in both register files around the int64 epilogue. With inline-asm MFMAs pinning 64
// tiles to AGPRs ("+a") and the epilogue staged through LDS one pair block at a time, <6, 4> holds in
// 174 VGPRs + 256 AGPRs (oz_gram_w_kernel, ob_gram_i8.hip: 228 VGPRs with its operand buffers).
#include <hip/hip_runtime.h>
typedef int v4i __attribute__((ext_vector_type(4)));
template <int NS, int NH>
__global__ __launch_bounds__(256, 1) __attribute__((amdgpu_waves_per_eu(1, 1))) void k(const v4i* A, const v4i* B, int* out, int n) {
  v4i acc[4][NS][NH];
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int q = 0; q < NS; ++q)
#pragma unroll
      for (int h = 0; h < NH; ++h) acc[m][q][h] = (v4i){};
  const int lane = threadIdx.x & 63;
  for (int s = 0; s < n; ++s) {
    v4i af[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) af[m] = A[(s * 4 + m) * 64 + lane];
#pragma unroll
    for (int h = 0; h < NH; ++h) {
      v4i bf[NS];
#pragma unroll
      for (int q = 0; q < NS; ++q) bf[q] = B[((s * NH + h) * NS + q) * 64 + lane];
#pragma unroll
      for (int q = 0; q < NS; ++q)
#pragma unroll
        for (int m = 0; m < 4; ++m) acc[m][q][h] = __builtin_amdgcn_mfma_i32_16x16x64_i8(af[m], bf[q], acc[m][q][h], 0, 0, 0);
    }
  }
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int h = 0; h < NH; ++h)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        long long p = 0;
#pragma unroll
        for (int q = 0; q < NS; ++q) p = p * 256 + acc[m][q][h][i];
        out[((m * NH + h) * 4 + i) * 64 + lane] = (int)(p >> 13);
      }
}
template __global__ void k<6, 4>(const v4i*, const v4i*, int*, int);
