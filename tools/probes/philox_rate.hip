// Philox4x32-10 issue-rate probe (round 6): the same function written three ways, timed by HIP
// events over a grid that fills the chip, with an xor of every output into one word per thread so
// nothing is dead. V0: the 32x32 -> 64 products as uint64 multiplies (v_mad_u64_u32, ob_spec.h's
// ob_philox_x3); V1: __umulhi + a 32-bit multiply (v_mul_hi_u32 + v_mul_lo_u32); V2: the products
// from 16-bit halves on the full-rate 24-bit multipliers. All three give identical outputs (checked
// on the host against the first). Standalone:
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/philox_rate tools/probes/philox_rate.hip && /tmp/philox_rate
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <vector>

__device__ __forceinline__ uint32_t x3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

template <int V>
__device__ __forceinline__ void mul32(uint32_t a, uint32_t M, uint32_t& lo, uint32_t& hi) {
  if constexpr (V == 0) {
    const uint64_t p = (uint64_t)M * a;
    lo = (uint32_t)p;
    hi = (uint32_t)(p >> 32);
  } else if constexpr (V == 1) {
    lo = a * M;
    hi = __umulhi(a, M);
  } else {
    // a = ah 2^16 + al, M = Mh 2^16 + Ml: a M = ah Mh 2^32 + (ah Ml + al Mh) 2^16 + al Ml
    const uint32_t al = a & 0xFFFFu, ah = a >> 16, Ml = M & 0xFFFFu, Mh = M >> 16;
    const uint32_t p0 = al * Ml, p1 = ah * Ml, p2 = al * Mh, p3 = ah * Mh;
    const uint64_t mid = (uint64_t)p1 + p2;  // 33 bits
    const uint64_t t = (uint64_t)p0 + (mid << 16);
    lo = (uint32_t)t;
    hi = p3 + (uint32_t)(t >> 32);
  }
}

template <int V>
__device__ __forceinline__ uint4 philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    uint32_t l0, h0, l1, h1;
    mul32<V>(c0, 0xD2511F53u, l0, h0);
    mul32<V>(c2, 0xCD9E8D57u, l1, h1);
    const uint32_t n0 = x3(h1, c1, k0), n2 = x3(h0, c3, k1);
    c1 = l1;
    c3 = l0;
    c0 = n0;
    c2 = n2;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return make_uint4(c0, c1, c2, c3);
}

template <int V>
__global__ __launch_bounds__(256) void k(uint32_t* out, uint32_t calls, uint32_t key0, uint32_t key1) {
  const uint32_t t = blockIdx.x * 256 + threadIdx.x;
  uint32_t acc = 0;
  for (uint32_t q = 0; q < calls; ++q) {
    const uint4 u = philox<V>(q, t, 0x1234u, 0x4F425232u, key0, key1);
    acc = x3(acc, u.x ^ u.y, u.z ^ u.w);
  }
  out[t] = acc;
}

int main() {
  const uint32_t blocks = 256 * 8 * 4, calls = 256;
  const size_t n = (size_t)blocks * 256;
  uint32_t* d;
  hipMalloc(&d, n * 4 * 3);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  std::vector<uint32_t> h[3];
  for (int rep = 0; rep < 2; ++rep)
    for (int V = 0; V < 3; ++V) {
      uint32_t* o = d + V * n;
      hipEventRecord(e0);
      if (V == 0) hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(256), 0, 0, o, calls, 0xB5EEDu, 0x51u);
      if (V == 1) hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(256), 0, 0, o, calls, 0xB5EEDu, 0x51u);
      if (V == 2) hipLaunchKernelGGL(k<2>, dim3(blocks), dim3(256), 0, 0, o, calls, 0xB5EEDu, 0x51u);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      const double wave_calls = (double)n * calls / 64.0;
      printf("V%d pass %d: %.3f ms, %.2f G calls/s, %.1f ns per wave-call per SIMD\n", V, rep, ms,
             n * (double)calls / ms / 1e6, ms * 1e6 * 1024.0 / wave_calls);
      h[V].resize(n);
      hipMemcpy(h[V].data(), o, n * 4, hipMemcpyDeviceToHost);
    }
  for (int V = 1; V < 3; ++V) {
    size_t bad = 0;
    for (size_t i = 0; i < n; ++i) bad += h[V][i] != h[0][i];
    printf("V%d vs V0: %zu differing words of %zu\n", V, bad, n);
  }
  hipFree(d);
  return 0;
}
