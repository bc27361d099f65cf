// Residency census: how many 64-thread workgroups with k_sim's LDS footprint (16 KiB) and a given
// VGPR load are resident per GPU at once.  Each workgroup holds its slot for a bounded ~30 us.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int NV, int NL>
__global__ __launch_bounds__(64) void census(unsigned* active, unsigned* peak, unsigned* sink) {
  __shared__ uint4 lds[NL];
  const unsigned lane = threadIdx.x;
  unsigned now = 0;
  if (lane == 0) {
    now = atomicAdd(active, 1u) + 1;
    atomicMax(peak, now);
  }
  float v[NV];
#pragma unroll
  for (int i = 0; i < NV; ++i) v[i] = (float)(lane * (i + 1) + blockIdx.x);
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < 3000ull) {  // 100 MHz clock: 30 us, always ends
#pragma unroll
    for (int i = 0; i < NV; ++i) v[i] = v[i] * 1.0001f + v[(i + 1) % NV];
  }
  float acc = 0;
#pragma unroll
  for (int i = 0; i < NV; ++i) acc += v[i];
  lds[lane] = make_uint4(__float_as_uint(acc), 0, 0, 0);
  __syncthreads();
  if (lds[(lane + 1) & 63].x == 0x7fffffffu) sink[blockIdx.x] = 1;  // keep v live
  if (lane == 0) atomicSub(active, 1u);
}

template <int NV, int NL>
void run(const char* name) {
  unsigned *a, *p, *s;
  hipMalloc(&a, 4); hipMalloc(&p, 4); hipMalloc(&s, 4 * 10000);
  hipMemset(a, 0, 4); hipMemset(p, 0, 4);
  census<NV, NL><<<10000, 64>>>(a, p, s);
  hipDeviceSynchronize();
  unsigned peak = 0;
  hipMemcpy(&peak, p, 4, hipMemcpyDeviceToHost);
  printf("%s: peak resident workgroups %u (%.2f per CU)\n", name, peak, peak / 256.0);
  hipFree(a); hipFree(p); hipFree(s);
}

int main() {
  run<16, 1024>("LDS 16 KiB, 34 VGPR");
  run<16, 1000>("LDS 15.6 KiB, 34 VGPR");
  run<16, 512>("LDS 8 KiB, 34 VGPR");
  run<100, 1024>("LDS 16 KiB, 100+ VGPR");
  run<100, 512>("LDS 8 KiB, 100+ VGPR");
  return 0;
}
