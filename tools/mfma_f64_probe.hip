// Probe for the gfx950 f64 matrix/vector rates and the v_mfma_f64_16x16x4_f64 lane maps.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/mfma_f64_probe tools/mfma_f64_probe.hip
// The Gram kernel's design depends on these numbers, so they are measured, not assumed.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <vector>

typedef double d4 __attribute__((ext_vector_type(4)));

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1);} } while (0)

// Layout check: A[i][k] = 1 + i + 100*k (16x4), B[k][j] = 3 + 7*j - 11*k (4x16), asymmetric.
__global__ void layout_kernel(double* out) {
  int l = threadIdx.x;
  int i = l & 15, k = l >> 4;
  double a = 1.0 + i + 100.0 * k;          // assumed A map: lane -> A[l&15][l>>4]
  double b = 3.0 + 7.0 * i - 11.0 * k;     // assumed B map: lane -> B[l>>4][l&15]
  d4 c = {0, 0, 0, 0};
  c = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
  for (int r = 0; r < 4; ++r) out[l * 4 + r] = c[r];
}

template <int NACC>
__global__ __launch_bounds__(256) void mfma_rate(double* sink, int iters) {
  d4 acc[NACC];
  for (int a = 0; a < NACC; ++a) acc[a] = (d4){0, 0, 0, 0};
  double x = 1.0 + 1e-9 * threadIdx.x, y = 1.0 - 1e-9 * threadIdx.x;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int a = 0; a < NACC; ++a) acc[a] = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, acc[a], 0, 0, 0);
  }
  double s = 0;
  for (int a = 0; a < NACC; ++a) s += acc[a][0] + acc[a][1] + acc[a][2] + acc[a][3];
  if (s == 12345.678) sink[threadIdx.x] = s;
}

// waves with (wave & 1)==0 issue MFMA, odd waves issue VALU fma: do the two f64 pipes add up?
__global__ __launch_bounds__(512) void mixed_rate(double* sink, int iters, int valu_iters) {
  int w = threadIdx.x >> 6;
  double s = 0;
  if ((w & 1) == 0) {
    d4 acc[8];
    for (int a = 0; a < 8; ++a) acc[a] = (d4){0, 0, 0, 0};
    double x = 1.0 + 1e-9 * threadIdx.x, y = 1.0 - 1e-9 * threadIdx.x;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int a = 0; a < 8; ++a) acc[a] = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, acc[a], 0, 0, 0);
    }
    for (int a = 0; a < 8; ++a) s += acc[a][0] + acc[a][1] + acc[a][2] + acc[a][3];
  } else {
    double a0 = threadIdx.x * 1e-3, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const double m = 0.999999, c = 1e-7;
    for (int it = 0; it < valu_iters; ++it) {
      a0 = fma(a0, m, c); a1 = fma(a1, m, c); a2 = fma(a2, m, c); a3 = fma(a3, m, c);
      a4 = fma(a4, m, c); a5 = fma(a5, m, c); a6 = fma(a6, m, c); a7 = fma(a7, m, c);
    }
    s = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
  }
  if (s == 12345.678) sink[threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void fma_rate(double* sink, int iters) {
  double a0 = threadIdx.x * 1e-3, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  const double m = 0.999999, c = 1e-7;
  for (int it = 0; it < iters; ++it) {
    a0 = fma(a0, m, c); a1 = fma(a1, m, c); a2 = fma(a2, m, c); a3 = fma(a3, m, c);
    a4 = fma(a4, m, c); a5 = fma(a5, m, c); a6 = fma(a6, m, c); a7 = fma(a7, m, c);
  }
  double s = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
  if (s == 12345.678) sink[threadIdx.x] = s;
}

int main() {
  hipDeviceProp_t p; CK(hipGetDeviceProperties(&p, 0));
  printf("device %s CUs %d clock %d kHz\n", p.gcnArchName, p.multiProcessorCount, p.clockRate);
  double* d; CK(hipMalloc(&d, 64 * 4 * sizeof(double)));
  layout_kernel<<<1, 64>>>(d);
  std::vector<double> h(256); CK(hipMemcpy(h.data(), d, 256 * 8, hipMemcpyDeviceToHost));
  // expected D[r][c] = sum_k A[r][k] * B[k][c]
  auto A = [](int i, int k) { return 1.0 + i + 100.0 * k; };
  auto B = [](int k, int j) { return 3.0 + 7.0 * j - 11.0 * k; };
  int bad_doc = 0, bad_alt = 0;
  for (int l = 0; l < 64; ++l) for (int r = 0; r < 4; ++r) {
    int col = l & 15, row_doc = (l >> 4) + 4 * r, row_alt = (l >> 4) * 4 + r;
    double e_doc = 0, e_alt = 0;
    for (int k = 0; k < 4; ++k) { e_doc += A(row_doc, k) * B(k, col); e_alt += A(row_alt, k) * B(k, col); }
    if (h[l * 4 + r] != e_doc) ++bad_doc;
    if (h[l * 4 + r] != e_alt) ++bad_alt;
  }
  printf("layout: row=(lane>>4)+4*r mismatches %d ; row=(lane>>4)*4+r mismatches %d\n", bad_doc, bad_alt);

  double* sink; CK(hipMalloc(&sink, 1 << 20));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  int cus = p.multiProcessorCount;
#define MFMA_RUN(NA) for (int wpc : {4, 8, 16}) { \
    int blocks = cus * wpc / 4, iters = 160000 / NA; \
    mfma_rate<NA><<<blocks, 256>>>(sink, 100); \
    CK(hipEventRecord(e0)); mfma_rate<NA><<<blocks, 256>>>(sink, iters); CK(hipEventRecord(e1)); \
    CK(hipEventSynchronize(e1)); float ms; CK(hipEventElapsedTime(&ms, e0, e1)); \
    double flops = (double)blocks * 4 * iters * NA * 16 * 16 * 4 * 2; \
    printf("mfma_f64_16x16x4 nacc=%d waves/CU=%d: %.2f TFLOP/s (%.3f ms)\n", NA, wpc, flops / ms / 1e9, ms); }
  MFMA_RUN(4) MFMA_RUN(8) MFMA_RUN(16)
  for (int vi : {0, 20000, 40000, 80000}) {
    int blocks = cus * 2, iters = 20000;
    mixed_rate<<<blocks, 512>>>(sink, 10, 10);
    CK(hipEventRecord(e0)); mixed_rate<<<blocks, 512>>>(sink, iters, vi); CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1)); float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    double mf = (double)blocks * 4 * iters * 8 * 16 * 16 * 4 * 2, vf = (double)blocks * 256 * vi * 8 * 2;
    printf("mixed valu_iters=%d: mfma %.2f TF + valu %.2f TF = %.2f TF (%.3f ms)\n", vi, mf / ms / 1e9, vf / ms / 1e9, (mf + vf) / ms / 1e9, ms);
  }
  for (int wpc : {4, 8, 16}) {
    int blocks = cus * wpc / 4, iters = 200000;
    fma_rate<<<blocks, 256>>>(sink, 100);
    CK(hipEventRecord(e0)); fma_rate<<<blocks, 256>>>(sink, iters); CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1)); float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    double flops = (double)blocks * 256 * iters * 8 * 2;
    printf("v_fma_f64 waves/CU=%d: %.2f TFLOP/s (%.3f ms)\n", wpc, flops / ms / 1e9, ms);
  }
  return 0;
}
