// i8 MFMA probe for the integer-sliced Gram:
//  1. operand layout of v_mfma_i32_32x32x32_i8 / 16x16x64_i8 with exact integer data: lane l is
//     assumed to hold A[row l&31][k = 16 (l>>5) + j] and B[k = 16 (l>>5) + j][col l&31] (32x32x32;
//     16x16x64: row/col l&15, k = 16 (l>>4) + j), C/D: col = lane&31, row = (r&3) + 8 (r>>2) + 4 (lane>>5);
//  2. back-to-back throughput (one wave per SIMD, independent accumulators).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

__global__ void layout32(const int8_t* A, const int8_t* B, int* D) {  // A 32x32 row-major [m][k], B [k][n]
  const int l = threadIdx.x;
  int8_t a[16], b[16];
  for (int j = 0; j < 16; ++j) {
    a[j] = A[(l & 31) * 32 + 16 * (l >> 5) + j];
    b[j] = B[(16 * (l >> 5) + j) * 32 + (l & 31)];
  }
  v4i av, bv;
  __builtin_memcpy(&av, a, 16);
  __builtin_memcpy(&bv, b, 16);
  v16i c = {};
  c = __builtin_amdgcn_mfma_i32_32x32x32_i8(av, bv, c, 0, 0, 0);
  for (int r = 0; r < 16; ++r) D[((r & 3) + 8 * (r >> 2) + 4 * (l >> 5)) * 32 + (l & 31)] = c[r];
}

__global__ void layout16(const int8_t* A, const int8_t* B, int* D) {  // A 16x64 [m][k], B 64x16 [k][n]
  const int l = threadIdx.x;
  int8_t a[16], b[16];
  for (int j = 0; j < 16; ++j) {
    a[j] = A[(l & 15) * 64 + 16 * (l >> 4) + j];
    b[j] = B[(16 * (l >> 4) + j) * 16 + (l & 15)];
  }
  v4i av, bv;
  __builtin_memcpy(&av, a, 16);
  __builtin_memcpy(&bv, b, 16);
  v4i c = {};
  c = __builtin_amdgcn_mfma_i32_16x16x64_i8(av, bv, c, 0, 0, 0);
  for (int r = 0; r < 4; ++r) D[((l >> 4) * 4 + r) * 16 + (l & 15)] = c[r];
}

template <int NACC>
__global__ __launch_bounds__(256, 1) void rate32(int* sink, int iters) {
  v16i acc[NACC];
  for (int a = 0; a < NACC; ++a) acc[a] = (v16i){};
  v4i x = {(int)threadIdx.x, 3, 5, 7}, y = {1, 2, (int)threadIdx.x, 4};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int a = 0; a < NACC; ++a) acc[a] = __builtin_amdgcn_mfma_i32_32x32x32_i8(x, y, acc[a], 0, 0, 0);
    x.x += 1;
  }
  int s = 0;
  for (int a = 0; a < NACC; ++a)
    for (int r = 0; r < 16; ++r) s += acc[a][r];
  if (s == 12345) sink[threadIdx.x] = s;
}

int main() {
  int8_t hA[32 * 64], hB[64 * 32];
  srand(7);
  for (auto& v : hA) v = (int8_t)(rand() % 255 - 127);
  for (auto& v : hB) v = (int8_t)(rand() % 255 - 127);
  int8_t *dA, *dB;
  int* dD;
  CK(hipMalloc(&dA, sizeof(hA)));
  CK(hipMalloc(&dB, sizeof(hB)));
  CK(hipMalloc(&dD, 32 * 32 * 4));
  CK(hipMemcpy(dA, hA, sizeof(hA), hipMemcpyHostToDevice));
  CK(hipMemcpy(dB, hB, sizeof(hB), hipMemcpyHostToDevice));
  int D[32 * 32];
  hipLaunchKernelGGL(layout32, dim3(1), dim3(64), 0, 0, dA, dB, dD);
  CK(hipMemcpy(D, dD, sizeof(D), hipMemcpyDeviceToHost));
  int bad = 0;
  for (int m = 0; m < 32; ++m)
    for (int n = 0; n < 32; ++n) {
      int s = 0;
      for (int k = 0; k < 32; ++k) s += hA[m * 32 + k] * hB[k * 32 + n];
      bad += s != D[m * 32 + n];
    }
  printf("32x32x32_i8 layout: %s (%d mismatches)\n", bad ? "WRONG" : "ok", bad);
  hipLaunchKernelGGL(layout16, dim3(1), dim3(64), 0, 0, dA, dB, dD);
  CK(hipMemcpy(D, dD, 16 * 16 * 4, hipMemcpyDeviceToHost));
  bad = 0;
  for (int m = 0; m < 16; ++m)
    for (int n = 0; n < 16; ++n) {
      int s = 0;
      for (int k = 0; k < 64; ++k) s += hA[m * 64 + k] * hB[k * 16 + n];
      bad += s != D[m * 16 + n];
    }
  printf("16x16x64_i8 layout: %s (%d mismatches)\n", bad ? "WRONG" : "ok", bad);
  hipDeviceProp_t p;
  CK(hipGetDeviceProperties(&p, 0));
  int* sink;
  CK(hipMalloc(&sink, 4096));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
#define RUN(NACC)                                                                                          \
  {                                                                                                        \
    const int iters = 20000;                                                                               \
    hipLaunchKernelGGL(rate32<NACC>, dim3(p.multiProcessorCount), dim3(256), 0, 0, sink, 10);              \
    CK(hipEventRecord(e0));                                                                                \
    hipLaunchKernelGGL(rate32<NACC>, dim3(p.multiProcessorCount), dim3(256), 0, 0, sink, iters);           \
    CK(hipEventRecord(e1));                                                                                \
    CK(hipEventSynchronize(e1));                                                                           \
    float ms;                                                                                              \
    CK(hipEventElapsedTime(&ms, e0, e1));                                                                  \
    const double ops = (double)p.multiProcessorCount * 4 * iters * NACC * 65536.0;                         \
    printf("32x32x32_i8 nacc=%d: %.0f TOPS (%.1f cycles/MFMA at 2.4 GHz)\n", NACC, ops / ms / 1e9,          \
           ms * 1e-3 * 2.4e9 / ((double)iters * NACC));                                                   \
  }
  RUN(4) RUN(8) RUN(16)
  return 0;
}
