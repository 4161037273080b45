// How much of the f64 MFMA peak can N waves per SIMD sustain with NACC independent accumulators?
// Operands in registers; 1 block per CU is forced with a large dynamic LDS request.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d4 __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

template <int NACC, int WPS>
__global__ __launch_bounds__(256 * WPS, WPS) void k(double* sink, int iters) {
  extern __shared__ double lds[];
  d4 acc[NACC];
#pragma unroll
  for (int a = 0; a < NACC; ++a) acc[a] = (d4){0, 0, 0, 0};
  double x = 1.0 + 1e-9 * threadIdx.x, y = 1.0 - 1e-9 * threadIdx.x;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int a = 0; a < NACC; ++a) acc[a] = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, acc[a], 0, 0, 0);
    x = x + 1e-12;  // keep operands live but dependent only once per iteration
  }
  double s = 0;
#pragma unroll
  for (int a = 0; a < NACC; ++a) s += acc[a][0] + acc[a][1] + acc[a][2] + acc[a][3];
  if (s == 1234.5) sink[threadIdx.x] = s + lds[0];
}

int main() {
  hipDeviceProp_t p; CK(hipGetDeviceProperties(&p, 0));
  double* sink; CK(hipMalloc(&sink, 1 << 20));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const size_t lds = 100 * 1024;
#define RUN(NACC, WPS) { \
    auto kern = k<NACC, WPS>; \
    CK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds)); \
    int iters = 40000 / NACC * 8 / WPS; \
    hipLaunchKernelGGL(kern, dim3(p.multiProcessorCount), dim3(256 * WPS), lds, 0, sink, 10); \
    CK(hipEventRecord(e0)); hipLaunchKernelGGL(kern, dim3(p.multiProcessorCount), dim3(256 * WPS), lds, 0, sink, iters); \
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1)); float ms; CK(hipEventElapsedTime(&ms, e0, e1)); \
    double flops = (double)p.multiProcessorCount * 4 * WPS * iters * NACC * 2048.0; \
    printf("waves/SIMD=%d nacc=%d: %.1f TFLOP/s\n", WPS, NACC, flops / ms / 1e9); }
  RUN(4, 1) RUN(8, 1) RUN(16, 1) RUN(4, 2) RUN(8, 2) RUN(16, 2)
  return 0;
}
