// Microbenchmark: does a wave64 VALU op with only one 32-lane half active (exec) cost
// less than a full one on gfx950? 8 independent fma chains per lane, all SIMDs busy.
// mode 0: all 64 lanes; 1: lanes 0-31 only; 2: the two halves one after the other,
// each on its own data (= the cost of feeding two half-waves different operands).
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ __launch_bounds__(256) void chains(float *out, int iters, int mode) {
  const int lane = threadIdx.x & 63;
  float a0 = lane, a1 = lane + 1, a2 = lane + 2, a3 = lane + 3, a4 = lane + 4, a5 = lane + 5, a6 = lane + 6,
        a7 = lane + 7;
  const float m = 1.0000001f, c = 1e-7f;
#define BODY                                                                                       \
  for (int i = 0; i < iters; i++) {                                                                \
    a0 = fmaf(a0, m, c); a1 = fmaf(a1, m, c); a2 = fmaf(a2, m, c); a3 = fmaf(a3, m, c);            \
    a4 = fmaf(a4, m, c); a5 = fmaf(a5, m, c); a6 = fmaf(a6, m, c); a7 = fmaf(a7, m, c);            \
  }
  if (mode == 0) {
    BODY
  } else if (mode == 1) {
    if (lane < 32) { BODY }
  } else {
    if (lane < 32) { BODY }
    if (lane >= 32) { BODY }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
}

int main() {
  const int blocks = 256 * 8 * 4, threads = 256, iters = 4096;
  float *out;
  hipMalloc(&out, sizeof(float) * blocks * threads);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int rep = 0; rep < 2; rep++)
    for (int mode = 0; mode < 3; mode++) {
      hipEventRecord(e0);
      chains<<<blocks, threads>>>(out, iters, mode);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      const double ops = (double)blocks * threads / 64 * iters * 8;  // wave-instructions
      printf("mode %d: %.3f ms, %.3f ns per wave-fma per CU-SIMD slot\n", mode, ms,
             ms * 1e6 / (ops / 1024.0));
    }
  return 0;
}
