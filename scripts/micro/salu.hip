// Scalar-unit throughput: how many SALU instructions per cycle does one CU retire, and does
// VALU work of the same waves overlap it? Each wave runs ITERS iterations of NS independent
// s_add_u32 and NV independent v_add_u32 (inline asm: nothing folded); waves per SIMD set by
// the grid (blocks of 256 threads = 4 waves, one per SIMD, BPC blocks per CU).
// Build: hipcc -O3 --offload-arch=gfx950 -o salu salu.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

template <int NS, int NV>
__global__ __launch_bounds__(256) void k(uint32_t *out, int iters) {
  uint32_t s0 = blockIdx.x, s1 = 1, s2 = 2, s3 = 3, s4 = 4, s5 = 5, s6 = 6, s7 = 7;
  uint32_t v0 = threadIdx.x, v1 = 1, v2 = 2, v3 = 3, v4 = 4, v5 = 5, v6 = 6, v7 = 7;
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int r = 0; r < 4; r++) {
      if (NS >= 1) asm volatile("s_add_u32 %0, %0, 1" : "+s"(s0) : : "scc");
      if (NS >= 2) asm volatile("s_add_u32 %0, %0, 3" : "+s"(s1) : : "scc");
      if (NS >= 3) asm volatile("s_add_u32 %0, %0, 5" : "+s"(s2) : : "scc");
      if (NS >= 4) asm volatile("s_add_u32 %0, %0, 7" : "+s"(s3) : : "scc");
      if (NS >= 5) asm volatile("s_add_u32 %0, %0, 9" : "+s"(s4) : : "scc");
      if (NS >= 6) asm volatile("s_add_u32 %0, %0, 11" : "+s"(s5) : : "scc");
      if (NS >= 7) asm volatile("s_add_u32 %0, %0, 13" : "+s"(s6) : : "scc");
      if (NS >= 8) asm volatile("s_add_u32 %0, %0, 15" : "+s"(s7) : : "scc");
      if (NV >= 1) asm volatile("v_add_u32 %0, %0, 1" : "+v"(v0));
      if (NV >= 2) asm volatile("v_add_u32 %0, %0, 3" : "+v"(v1));
      if (NV >= 3) asm volatile("v_add_u32 %0, %0, 5" : "+v"(v2));
      if (NV >= 4) asm volatile("v_add_u32 %0, %0, 7" : "+v"(v3));
      if (NV >= 5) asm volatile("v_add_u32 %0, %0, 9" : "+v"(v4));
      if (NV >= 6) asm volatile("v_add_u32 %0, %0, 11" : "+v"(v5));
      if (NV >= 7) asm volatile("v_add_u32 %0, %0, 13" : "+v"(v6));
      if (NV >= 8) asm volatile("v_add_u32 %0, %0, 15" : "+v"(v7));
    }
  }
  out[blockIdx.x * 256 + threadIdx.x] = s0 + s1 + s2 + s3 + s4 + s5 + s6 + s7 + v0 + v1 + v2 + v3 + v4 + v5 + v6 + v7;
}

int main() {
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, 0) != hipSuccess) return 1;
  const int cus = prop.multiProcessorCount;
  uint32_t *out;
  (void)hipMalloc(&out, 4ull * cus * 8 * 256);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const int iters = 4096;
  float ms;
  printf("CUs %d; per CU per cycle at 2.4 GHz (clock under load may be lower)\n", cus);
#define RUN(NS, NV, BPC)                                                                                   \
  for (int rep = 0; rep < 2; rep++) {                                                                      \
    (void)hipEventRecord(e0);                                                                              \
    k<NS, NV><<<cus * (BPC), 256>>>(out, iters);                                                           \
    (void)hipEventRecord(e1);                                                                              \
    (void)hipEventSynchronize(e1);                                                                         \
    (void)hipEventElapsedTime(&ms, e0, e1);                                                                \
    const double waves = (double)cus * (BPC) * 4, cyc = ms * 1e-3 * 2.4e9;                                 \
    if (hipGetLastError() != hipSuccess) printf("launch error\n");                                    \
    if (rep)                                                                                               \
      printf("NS %d NV %d waves/SIMD %d: %8.3f ms  SALU/CU/cyc %.3f  VALU/SIMD/cyc %.3f\n", NS, NV, BPC, ms, \
             waves / cus * iters * 4 * (NS) / cyc, waves / cus / 4 * iters * 4 * (NV) / cyc);             \
  }
  RUN(8, 0, 1) RUN(8, 0, 2) RUN(8, 0, 4) RUN(8, 0, 8)
  RUN(0, 8, 1) RUN(0, 8, 2) RUN(0, 8, 4)
  RUN(4, 8, 2) RUN(4, 8, 4) RUN(8, 8, 4) RUN(2, 8, 4) RUN(8, 4, 4)
  return 0;
}
