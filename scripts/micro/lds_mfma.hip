// Microbenchmarks behind the round-5 k-NN kernel design (MFMA screening + band lists):
//  1. cost of an exec-masked ds_write_b32 per wave-instruction at lane densities 64..0,
//     beside a fixed VALU body (the "append" of a band value);
//  2. cost of a ds_add_u32 (all lanes, per-lane bin address) beside the same body (the
//     per-candidate histogram update of knn_grid.hip);
//  3. v_mfma_f32_32x32x2_f32 beside N VALU ops per MFMA (is the matrix pipe free?);
//  4. the 32x32x2 f32 MFMA's lane layout and numerics: D = fma chain over k, checked
//     against a host fmaf chain bit for bit.
// Build: hipcc -O3 --offload-arch=gfx950 -o lds_mfma lds_mfma.hip
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kThreads = 256;

// 16 value slots per iteration; per slot 6 VALU of "work" (a canonical-d²-like chain),
// then (APPEND) a masked ds_write of the value into the lane's 32-entry ring, the mask
// being lanes whose rotating id is below D.
template <int MODE>  // 0: body only, 1: + masked ds_write_b32, 2: + ds_add_u32 (all lanes)
__global__ __launch_bounds__(kThreads) void slots_kernel(float *out, int iters, int dens) {
  __shared__ uint32_t lds[4][64 * 33];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t *my = lds[w];
  float q = lane * 0.001f, acc = 0.f;
  uint32_t cnt = 0;
  uint32_t rot = (uint32_t)lane;
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int s = 0; s < 16; s++) {
      const float p = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(q + s)));
      const float dx = q - p, dy = q - 2.f * p, dz = q + p;
      const float d2 = fmaf(dz, dz, fmaf(dy, dy, dx * dx));
      acc += d2;
      if (MODE == 1) {
        const bool in = ((rot + (uint32_t)s * 5u) & 63u) < (uint32_t)dens;
        if (in) {
          my[(cnt & 31u) * 64u + (uint32_t)lane] = __float_as_uint(d2);
          cnt++;
        }
      } else if (MODE == 2) {
        const uint32_t bin = (__float_as_uint(d2) >> 20) & 31u;
        __atomic_fetch_add(&my[bin * 64u + (uint32_t)lane], 1u, __ATOMIC_RELAXED);
      }
    }
    rot += 7u;
    q += 1e-6f;
  }
  __syncthreads();
  out[blockIdx.x * kThreads + threadIdx.x] = acc + (float)my[lane] + (float)cnt;
}

// one MFMA per step with NV independent VALU fmas (8 chains) beside it
template <int NV, bool MF>
__global__ __launch_bounds__(kThreads) void mfma_kernel(float *out, int iters) {
  const int lane = threadIdx.x & 63;
  f32x16 c0 = {}, c1 = {};
  float a = lane * 0.5f, b = lane * 0.25f;
  float v[8];
#pragma unroll
  for (int i = 0; i < 8; i++) v[i] = lane + i;
  for (int it = 0; it < iters; it++) {
    if (MF) {
      c0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_32x32x2f32(b, a, c1, 0, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < NV / 8; j++)
#pragma unroll
      for (int i = 0; i < 8; i++) v[i] = fmaf(v[i], 1.0000001f, 1e-7f);
  }
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 16; i++) s += c0[i] + c1[i];
#pragma unroll
  for (int i = 0; i < 8; i++) s += v[i];
  out[blockIdx.x * kThreads + threadIdx.x] = s;
}

// layout / numerics: A[i][k] lane l: i = l & 31, k = l >> 5; B[k][j] lane l: k = l >> 5,
// j = l & 31; D[i][j] lane l reg r: j = l & 31, i = (r & 3) + 8 (r >> 2) + 4 (l >> 5)
__global__ void layout_kernel(const float *A, const float *B, const float *C, float *D) {
  const int l = threadIdx.x;
  const float a = A[(l & 31) * 2 + (l >> 5)];
  const float b = B[(l >> 5) * 32 + (l & 31)];
  f32x16 c;
  for (int r = 0; r < 16; r++) c[r] = C[((r & 3) + 8 * (r >> 2) + 4 * (l >> 5)) * 32 + (l & 31)];
  c = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
  for (int r = 0; r < 16; r++) D[((r & 3) + 8 * (r >> 2) + 4 * (l >> 5)) * 32 + (l & 31)] = c[r];
}

static float frand(uint64_t &s) {
  s = s * 6364136223846793005ull + 1442695040888963407ull;
  return (float)((s >> 40) & 0xffffff) / 16777216.0f * 2.f - 1.f;
}

int main() {
  int ndev = 0;
  hipGetDeviceCount(&ndev);
  if (ndev < 1) {
    printf("no GPU\n");
    return 1;
  }
  hipDeviceProp_t prop;
  hipGetDeviceProperties(&prop, 0);
  const int cus = prop.multiProcessorCount;
  const int blocks = cus * 8;  // 32 waves per CU
  float *out;
  hipMalloc(&out, sizeof(float) * blocks * kThreads);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const double ghz = 2.4;
  auto report = [&](const char *name, float ms, double wave_units) {
    // SIMD-cycles per wave-unit at 2.4 GHz: every SIMD of the chip busy
    const double simds = 4.0 * cus;
    printf("%-40s %8.3f ms  %7.2f SIMD-cyc/unit\n", name, ms, ms * 1e-3 * ghz * 1e9 * simds / wave_units);
  };
  const int iters = 2048;
  const double slots = (double)blocks * 4 * iters * 16;
  for (int rep = 0; rep < 2; rep++) {
    float ms;
#define RUN(label, ...)                            \
  hipEventRecord(e0);                              \
  __VA_ARGS__;                                     \
  hipEventRecord(e1);                              \
  hipEventSynchronize(e1);                         \
  hipEventElapsedTime(&ms, e0, e1);                \
  if (rep) report(label, ms, slots);
    RUN("body only (per slot)", slots_kernel<0><<<blocks, kThreads>>>(out, iters, 0));
    RUN("masked ds_write dens 64", slots_kernel<1><<<blocks, kThreads>>>(out, iters, 64));
    RUN("masked ds_write dens 16", slots_kernel<1><<<blocks, kThreads>>>(out, iters, 16));
    RUN("masked ds_write dens 4", slots_kernel<1><<<blocks, kThreads>>>(out, iters, 4));
    RUN("masked ds_write dens 1", slots_kernel<1><<<blocks, kThreads>>>(out, iters, 1));
    RUN("masked ds_write dens 0", slots_kernel<1><<<blocks, kThreads>>>(out, iters, 0));
    RUN("ds_add all lanes", slots_kernel<2><<<blocks, kThreads>>>(out, iters, 0));
#undef RUN
  }
  const int mit = 4096;
  const double steps = (double)blocks * 4 * mit;  // per wave-step: 2 MFMA + NV VALU
  for (int rep = 0; rep < 2; rep++) {
    float ms;
#define RUN(label, ...)                            \
  hipEventRecord(e0);                              \
  __VA_ARGS__;                                     \
  hipEventRecord(e1);                              \
  hipEventSynchronize(e1);                         \
  hipEventElapsedTime(&ms, e0, e1);                \
  if (rep) report(label, ms, steps);
    RUN("2 mfma32x32x2 only (per step)", mfma_kernel<0, true><<<blocks, kThreads>>>(out, mit));
    RUN("32 VALU only", mfma_kernel<32, false><<<blocks, kThreads>>>(out, mit));
    RUN("2 mfma + 32 VALU", mfma_kernel<32, true><<<blocks, kThreads>>>(out, mit));
    RUN("64 VALU only", mfma_kernel<64, false><<<blocks, kThreads>>>(out, mit));
    RUN("2 mfma + 64 VALU", mfma_kernel<64, true><<<blocks, kThreads>>>(out, mit));
    RUN("128 VALU only", mfma_kernel<128, false><<<blocks, kThreads>>>(out, mit));
    RUN("2 mfma + 128 VALU", mfma_kernel<128, true><<<blocks, kThreads>>>(out, mit));
#undef RUN
  }
  // layout / numerics check
  float hA[64], hB[64], hC[1024], hD[1024];
  uint64_t s = 12345;
  for (int i = 0; i < 64; i++) hA[i] = frand(s);
  for (int i = 0; i < 64; i++) hB[i] = frand(s);
  for (int i = 0; i < 1024; i++) hC[i] = frand(s);
  float *dA, *dB, *dC, *dD;
  hipMalloc(&dA, 256);
  hipMalloc(&dB, 256);
  hipMalloc(&dC, 4096);
  hipMalloc(&dD, 4096);
  hipMemcpy(dA, hA, 256, hipMemcpyHostToDevice);
  hipMemcpy(dB, hB, 256, hipMemcpyHostToDevice);
  hipMemcpy(dC, hC, 4096, hipMemcpyHostToDevice);
  layout_kernel<<<1, 64>>>(dA, dB, dC, dD);
  hipMemcpy(hD, dD, 4096, hipMemcpyDeviceToHost);
  int bad_chain = 0, bad_rev = 0;
  for (int i = 0; i < 32; i++)
    for (int j = 0; j < 32; j++) {
      const float a0 = hA[i * 2], a1 = hA[i * 2 + 1], b0 = hB[j], b1 = hB[32 + j], c = hC[i * 32 + j];
      const float chain = fmaf(a1, b1, fmaf(a0, b0, c));
      const float rev = fmaf(a0, b0, fmaf(a1, b1, c));
      bad_chain += chain != hD[i * 32 + j];
      bad_rev += rev != hD[i * 32 + j];
    }
  printf("layout 32x32x2f32: %d / 1024 differ from fma(a1,b1,fma(a0,b0,c)), %d from the reverse chain\n",
         bad_chain, bad_rev);
  return 0;
}
