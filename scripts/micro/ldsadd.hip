// Is the per-candidate LDS histogram add (ds_add_u32, every lane) an issue cost or an LDS
// throughput limit? Body of NV VALU ops per slot with and without one ds_add per slot;
// if the LDS is the limit the ds_add variants flatten at the LDS rate as NV grows.
// PAIR: lanes l and l+32 add to the same dword (the knn_grid pair histogram layout).
// Build: hipcc -O3 --offload-arch=gfx950 -o ldsadd ldsadd.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

constexpr int kThreads = 256;

template <int NV, int ADD>  // ADD 0: none, 1: own dword per lane, 2: pair dword, 3: ds_write_b32
__global__ __launch_bounds__(kThreads) void k(uint32_t *out, int iters) {
  __shared__ uint32_t lds[4][41 * 64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int i = lane; i < 41 * 64; i += 64) lds[w][i] = 0;
  uint32_t v[4] = {(uint32_t)lane * 2654435761u, (uint32_t)lane * 40503u + 7u, (uint32_t)lane ^ 0x55u,
                   (uint32_t)lane * 97u};
  const uint32_t base = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint32_t *)lds[w];
  uint32_t acc = 0;
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int s = 0; s < 16; s++) {
#pragma unroll
      for (int j = 0; j < NV; j++) {
        v[j & 3] = (v[j & 3] ^ (uint32_t)(s * 31 + j)) + (uint32_t)it;
        asm volatile("" : "+v"(v[j & 3]));
      }
      const uint32_t bin = (v[s & 3] & 31u) + ((v[s & 3] >> 5) & 7u);
      if (ADD == 1 || ADD == 3) {
        const uint32_t a = base + (bin * 64u + (uint32_t)lane) * 4u;
        if (ADD == 1)
          __atomic_fetch_add((__attribute__((address_space(3))) uint32_t *)(uintptr_t)a, 1u, __ATOMIC_RELAXED);
        else
          *(__attribute__((address_space(3))) uint32_t *)(uintptr_t)a = v[s & 3];
      } else if (ADD == 2) {
        const uint32_t a = base + (bin * 32u + ((uint32_t)lane & 31u)) * 4u;
        __atomic_fetch_add((__attribute__((address_space(3))) uint32_t *)(uintptr_t)a,
                           1u << (((uint32_t)lane & 32u) >> 1), __ATOMIC_RELAXED);
      } else {
        acc += bin;
      }
    }
  }
  __syncthreads();
  out[blockIdx.x * kThreads + threadIdx.x] = acc + lds[w][lane] + v[0] + v[1] + v[2] + v[3];
}

int main() {
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, 0) != hipSuccess) return 1;
  const int cus = prop.multiProcessorCount, blocks = cus * 8;
  uint32_t *out;
  (void)hipMalloc(&out, 4 * blocks * kThreads);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const int iters = 1024;
  const double units = (double)blocks * 4 * iters * 16;
  float ms;
#define RUN(label, ...)                                                                          \
  for (int rep = 0; rep < 2; rep++) {                                                            \
    (void)hipEventRecord(e0);                                                                    \
    __VA_ARGS__;                                                                                 \
    (void)hipEventRecord(e1);                                                                    \
    (void)hipEventSynchronize(e1);                                                               \
    (void)hipEventElapsedTime(&ms, e0, e1);                                                      \
    if (rep) printf("%-34s %7.3f ms %7.2f SIMD-cyc/slot\n", label, ms, ms * 1e-3 * 2.4e9 * 4 * cus / units); \
  }
  RUN("NV 4, none", k<4, 0><<<blocks, kThreads>>>(out, iters));
  RUN("NV 4, ds_add own", k<4, 1><<<blocks, kThreads>>>(out, iters));
  RUN("NV 4, ds_add pair", k<4, 2><<<blocks, kThreads>>>(out, iters));
  RUN("NV 4, ds_write", k<4, 3><<<blocks, kThreads>>>(out, iters));
  RUN("NV 8, none", k<8, 0><<<blocks, kThreads>>>(out, iters));
  RUN("NV 8, ds_add own", k<8, 1><<<blocks, kThreads>>>(out, iters));
  RUN("NV 8, ds_add pair", k<8, 2><<<blocks, kThreads>>>(out, iters));
  RUN("NV 12, none", k<12, 0><<<blocks, kThreads>>>(out, iters));
  RUN("NV 12, ds_add own", k<12, 1><<<blocks, kThreads>>>(out, iters));
  RUN("NV 12, ds_add pair", k<12, 2><<<blocks, kThreads>>>(out, iters));
  RUN("NV 16, none", k<16, 0><<<blocks, kThreads>>>(out, iters));
  RUN("NV 16, ds_add pair", k<16, 2><<<blocks, kThreads>>>(out, iters));
  RUN("NV 24, none", k<24, 0><<<blocks, kThreads>>>(out, iters));
  RUN("NV 24, ds_add pair", k<24, 2><<<blocks, kThreads>>>(out, iters));
  return 0;
}
