// FETCH_SIZE probe: the x2 correction of gfx950's FETCH_SIZE
// (MI355X_MICROARCH.md: 64 B counted per 128 B request) is established for coalesced streaming
// reads; the 1M-peer gossip window reads scattered 16-B items.  Four kernels over one 1 GiB array,
// each dispatched once, so a rocprofv3 --pmc FETCH_SIZE pass reports each one's counter:
//   k_stream   every 16-B item once, coalesced                           (1 GiB requested)
//   k_scatter  N random 16-B items, one per thread                       (N x 16 B requested)
//   k_scatter4 N/4 random 64-B blocks, 4 lanes read the block's 16-B quarters (N x 16 B requested)
//   k_pair     N/2 random 128-B lines, 2 lanes read 16 B at offsets 0 and 64 (both halves of a line)
// k_pair against k_scatter4 tells the L2's fill granularity: a raw FETCH_SIZE of 64 B per 128-B line
// means whole-line fills counted at half (the x2 correction holds for scattered reads too); 128 B
// per line means 64-B sector fills counted exactly (then scattered reads need no correction).
// The random indices come from a hash of the thread id (no index array is read).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

constexpr uint64_t kItems = 1ull << 26;  // 16-B items: 1 GiB
constexpr uint32_t kN = 1u << 22;        // scattered reads

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
  x ^= x >> 16; x *= 0x7FEB352Du; x ^= x >> 15; x *= 0x846CA68Bu; x ^= x >> 16;
  return x;
}

__global__ void k_stream(const uint4* a, uint32_t* out) {
  uint32_t acc = 0;
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < kItems; i += (uint64_t)gridDim.x * 256) {
    const uint4 v = a[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) out[0] = acc;
}

__global__ void k_scatter(const uint4* a, uint32_t* out) {
  const uint32_t t = blockIdx.x * 256 + threadIdx.x;
  const uint4 v = a[hash32(t) & (kItems - 1)];
  const uint32_t acc = v.x ^ v.y ^ v.z ^ v.w;
  if (acc == 0x12345678u) out[0] = acc;
}

__global__ void k_scatter4(const uint4* a, uint32_t* out) {
  const uint32_t t = blockIdx.x * 256 + threadIdx.x;
  const uint64_t line = hash32(t >> 2) & (kItems / 4 - 1);
  const uint4 v = a[line * 4 + (t & 3)];
  const uint32_t acc = v.x ^ v.y ^ v.z ^ v.w;
  if (acc == 0x12345678u) out[0] = acc;
}

__global__ void k_pair(const uint4* a, uint32_t* out) {
  const uint32_t t = blockIdx.x * 256 + threadIdx.x;
  const uint64_t line = hash32(t >> 1) & (kItems / 8 - 1);
  const uint4 v = a[line * 8 + (t & 1) * 4];
  const uint32_t acc = v.x ^ v.y ^ v.z ^ v.w;
  if (acc == 0x12345678u) out[0] = acc;
}

int main() {
  uint4* a;
  uint32_t* out;
  hipMalloc(&a, kItems * 16);
  hipMalloc(&out, 64);
  hipMemset(a, 1, kItems * 16);
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  float ms;
  hipEventRecord(e0);
  k_stream<<<8192, 256>>>(a, out);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  hipEventElapsedTime(&ms, e0, e1);
  printf("k_stream   requested %llu B  %.3f ms\n", (unsigned long long)(kItems * 16), ms);
  hipEventRecord(e0);
  k_scatter<<<kN / 256, 256>>>(a, out);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  hipEventElapsedTime(&ms, e0, e1);
  printf("k_scatter  requested %llu B  %.3f ms\n", (unsigned long long)kN * 16, ms);
  hipEventRecord(e0);
  k_scatter4<<<kN / 256, 256>>>(a, out);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  hipEventElapsedTime(&ms, e0, e1);
  printf("k_scatter4 requested %llu B  %.3f ms\n", (unsigned long long)kN * 16, ms);
  hipEventRecord(e0);
  k_pair<<<kN / 256, 256>>>(a, out);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  hipEventElapsedTime(&ms, e0, e1);
  printf("k_pair     requested %llu B in %u lines  %.3f ms\n", (unsigned long long)kN * 16, kN / 2, ms);
  return 0;
}
