// Microbenchmark: Philox4x32-10 throughput on gfx950, three exact formulations of the round's
// 32x32->64 products (the parallel phase of k_sim computes one or two draws per offered packet).
//   A  v_mad_u64_u32 (one 64-bit product per multiplier, the engine's form)
//   B  v_mul_hi_u32 + v_mul_lo_u32
//   C  pairs of lanes' counters... (not used) -- C: A with the two rounds' products interleaved
// Every variant must produce identical words (checked against A).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

template <int V>
__device__ __forceinline__ void philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1,
                                       uint32_t r[4]) {
  __asm__ volatile("" : "+s"(k0), "+s"(k1));
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    uint32_t h0, l0, h1, l1;
    if constexpr (V == 0) {
      const uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
      h0 = (uint32_t)(p0 >> 32); l0 = (uint32_t)p0;
      h1 = (uint32_t)(p1 >> 32); l1 = (uint32_t)p1;
    } else {
      h0 = __umulhi(0xD2511F53u, c0); l0 = 0xD2511F53u * c0;
      h1 = __umulhi(0xCD9E8D57u, c2); l1 = 0xCD9E8D57u * c2;
    }
    const uint32_t n0 = h1 ^ c1 ^ k0, n2 = h0 ^ c3 ^ k1;
    c0 = n0; c1 = l1; c2 = n2; c3 = l0;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  r[0] = c0; r[1] = c1; r[2] = c2; r[3] = c3;
}

template <int V, int ILP>
__global__ __launch_bounds__(64) void k_bench(uint32_t* out, uint32_t iters, uint32_t k0, uint32_t k1) {
  const uint32_t id = blockIdx.x * 64 + threadIdx.x;
  uint32_t acc[ILP] = {};
  for (uint32_t it = 0; it < iters; ++it) {
#pragma unroll
    for (int j = 0; j < ILP; ++j) {
      uint32_t r[4];
      philox<V>(id, it, j, acc[j], k0, k1, r);
      acc[j] ^= r[0] ^ r[1] ^ r[2] ^ r[3];
    }
  }
  uint32_t x = 0;
#pragma unroll
  for (int j = 0; j < ILP; ++j) x ^= acc[j];
  out[id] = x;
}

template <int V, int ILP>
float run(uint32_t* d, int blocks, uint32_t iters, uint32_t* host) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  k_bench<V, ILP><<<blocks, 64>>>(d, iters, 0x12345678u, 0x9ABCDEF0u);
  hipEventRecord(a);
  k_bench<V, ILP><<<blocks, 64>>>(d, iters, 0x12345678u, 0x9ABCDEF0u);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  hipMemcpy(host, d, sizeof(uint32_t) * blocks * 64, hipMemcpyDeviceToHost);
  return ms;
}

int main() {
  const int blocks = 256 * 4 * 8;  // 8 waves per SIMD
  const uint32_t iters = 4096;
  uint32_t* d;
  hipMalloc(&d, sizeof(uint32_t) * blocks * 64);
  static uint32_t h0[256 * 4 * 8 * 64], h1[256 * 4 * 8 * 64];
  const double draws = (double)blocks * 64 * iters;
#define ONE(V, ILP, H)                                                                                   \
  {                                                                                                     \
    const float ms = run<V, ILP>(d, blocks, iters / ILP, H);                                           \
    printf("variant %d ilp %d: %.3f ms, %.2f G draws/s, %.1f SIMD cycles per wave-draw @2.4GHz\n", V, ILP, \
           ms, draws / ms / 1e6, 2.4e9 * ms * 1e-3 * 1024 / (draws / 64));                             \
  }
  ONE(0, 1, h0) ONE(1, 1, h1)
  int bad = 0;
  for (int i = 0; i < blocks * 64; ++i) bad += h0[i] != h1[i];
  printf("mismatches A vs B: %d\n", bad);
  ONE(0, 2, h0) ONE(1, 2, h1) ONE(0, 4, h0) ONE(1, 4, h1)
  return 0;
}
