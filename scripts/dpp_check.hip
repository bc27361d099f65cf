// Checks k_sim's DPP wave-scan helpers against plain loops (diagnostic; not part of the product).
#include "../testground_amd/csrc/tgsim_kernels.hip"
#include <stdio.h>
using namespace tgsim;
__global__ void k(const uint64_t* in, uint64_t* out) {
  const uint32_t l = threadIdx.x;
  uint64_t a = in[l] & 0xFFFF, b = in[l] >> 20;
  scan_maxplus(a, b);
  out[l * 8 + 0] = a; out[l * 8 + 1] = b;
  out[l * 8 + 2] = (uint64_t)(int64_t)scan_sum_i32((int32_t)(in[l] % 7) - 3);
  out[l * 8 + 3] = (uint64_t)(int64_t)scan_max_i32((int32_t)(in[l] % 1000) - 700);
  out[l * 8 + 4] = scan_max_u32((uint32_t)in[l] & 0xFFF);
  out[l * 8 + 5] = scan_min_u64(in[l]);
  out[l * 8 + 6] = shr1_u64(in[l], 12345);
  out[l * 8 + 7] = shr1_u32((uint32_t)in[l], 77u);
}
int main() {
  uint64_t h[64], o[512];
  for (int i = 0; i < 64; ++i) h[i] = (0x9E3779B97F4A7C15ull * (i + 1)) >> 8;
  uint64_t *d, *dout;
  (void)hipMalloc(&d, sizeof h); (void)hipMalloc(&dout, sizeof o);
  (void)hipMemcpy(d, h, sizeof h, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, dout);
  (void)hipMemcpy(o, dout, sizeof o, hipMemcpyDeviceToHost);
  uint64_t A = 0, B = 0; int64_t S = 0, M = INT64_MIN; uint64_t MU = 0, MN = ~0ull; int bad = 0;
  for (int i = 0; i < 64; ++i) {
    uint64_t a = h[i] & 0xFFFF, b = h[i] >> 20;
    uint64_t nb = B + a; B = nb > b ? nb : b; A = A + a;
    S += (int64_t)(h[i] % 7) - 3;
    int64_t mv = (int64_t)(h[i] % 1000) - 700; M = M > mv ? M : mv;
    uint64_t mu = (uint32_t)h[i] & 0xFFF; MU = MU > mu ? MU : mu;
    MN = MN < h[i] ? MN : h[i];
    uint64_t e[8] = {A, B, (uint64_t)S, (uint64_t)M, MU, MN, i ? h[i - 1] : 12345, i ? (uint32_t)h[i - 1] : 77u};
    for (int k = 0; k < 8; ++k)
      if (o[i * 8 + k] != e[k]) { if (bad < 12) printf("lane %d fn %d: got %llu want %llu\n", i, k, (unsigned long long)o[i * 8 + k], (unsigned long long)e[k]); bad++; }
  }
  printf("dpp check: %d mismatches\n", bad);
  return bad != 0;
}
