// Microbenchmarks for the round-5 k-NN design (f16 hi/lo split MFMA screening):
//  1. v_mfma_f32_32x32x16_f16 beside N VALU ops per MFMA in the same wave (does the
//     matrix pipe run under the VALU?);
//  2. the band-append loop: per 16-value tile, a below-L count, an in-band bit mask,
//     then a loop that appends each lane's in-band entries to its LDS list (iterations =
//     the wave's max per-lane count), at in-band densities 1/8, 1/16, 1/32, 0;
//  3. numerics: d² of centred, power-of-2-scaled points through the split-f16 fragments
//     (q·p = (qh+ql)(ph+pl) in 4 products per axis, |p|² and |q|² as hi+lo) against fp64.
// Build: hipcc -O3 --offload-arch=gfx950 -o mfma16 mfma16.hip
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

constexpr int kThreads = 256;

template <int NV, bool MF>
__global__ __launch_bounds__(kThreads) void mfma_kernel(float *out, int iters) {
  const int lane = threadIdx.x & 63;
  f32x16 c0 = {}, c1 = {};
  f16x8 a, b;
  for (int i = 0; i < 8; i++) {
    a[i] = (_Float16)(lane * 0.01f + i);
    b[i] = (_Float16)(lane * 0.02f - i);
  }
  float v[8];
#pragma unroll
  for (int i = 0; i < 8; i++) v[i] = lane + i;
  for (int it = 0; it < iters; it++) {
    if (MF) {
      c0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(b, a, c1, 0, 0, 0);
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


template <int NV, bool MF>
__global__ __launch_bounds__(kThreads) void mfma_int_kernel(float *out, int iters) {
  const int lane = threadIdx.x & 63;
  f32x16 c0 = {}, c1 = {};
  f16x8 a, b;
  for (int i = 0; i < 8; i++) {
    a[i] = (_Float16)(lane * 0.01f + i);
    b[i] = (_Float16)(lane * 0.02f - i);
  }
  uint32_t v[8];
#pragma unroll
  for (int i = 0; i < 8; i++) v[i] = lane * 77u + i;
  for (int it = 0; it < iters; it++) {
    if (MF) {
      c0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(b, a, c1, 0, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < NV / 8; j++)
#pragma unroll
      for (int i = 0; i < 8; i++) {
        v[i] = (v[i] ^ (uint32_t)(j * 0x9e3779b9u + i)) + (uint32_t)it;
        asm volatile("" : "+v"(v[i]));
      }
  }
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 16; i++) s += c0[i] + c1[i];
#pragma unroll
  for (int i = 0; i < 8; i++) s += (float)v[i];
  out[blockIdx.x * kThreads + threadIdx.x] = s;
}

// MODE 0: values + below count + in-band bits only; 1: + the append loop
template <int MODE>
__global__ __launch_bounds__(kThreads) void append_kernel(uint32_t *out, int iters, uint32_t dens_shift) {
  __shared__ uint32_t lds[4][64 * 65];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t *my = lds[w] + lane;
  uint32_t below = 0, cnt = 0, h = (uint32_t)lane * 2654435761u + blockIdx.x;
  const uint32_t L = 0x10000000u, H = L + (0x10000000u >> dens_shift);
  for (int it = 0; it < iters; it++) {
    uint32_t bits = 0;
#pragma unroll
    for (int r = 0; r < 16; r++) {
      const uint32_t v = (h ^ (h >> 13)) * 0x5bd1e995u;  // "value" bits, uniform
      h += 0x9e3779b9u;
      const bool cl = v < L;
      below += cl ? 1u : 0u;
      bits |= (!cl && v < H) ? (1u << r) : 0u;
    }
    if (MODE == 1) {
      while (bits) {
        const uint32_t r = (uint32_t)__builtin_ctz(bits);
        bits &= bits - 1u;
        my[(cnt & 63u) * 65u] = (uint32_t)it * 16u + r;
        cnt++;
      }
    } else {
      cnt += (uint32_t)__builtin_popcount(bits);
    }
  }
  __syncthreads();
  out[blockIdx.x * kThreads + threadIdx.x] = below + cnt + my[0];
}

// split-f16 fragments (see header); p, q centred and scaled
struct Frag {
  f16x8 a, b;
};
__device__ __forceinline__ void split(float x, _Float16 &hi, _Float16 &lo) {
  hi = (_Float16)x;
  lo = (_Float16)(x - (float)hi);
}
__device__ __forceinline__ f16x8 frag_a(float px, float py, float pz, int h) {
  f16x8 a;
  if (h == 0) {
    _Float16 xh, xl, yh, yl;
    split(px, xh, xl);
    split(py, yh, yl);
    a[0] = xh; a[1] = xl; a[2] = xh; a[3] = xl;
    a[4] = yh; a[5] = yl; a[6] = yh; a[7] = yl;
  } else {
    _Float16 zh, zl, ph, pl;
    split(pz, zh, zl);
    split(fmaf(pz, pz, fmaf(py, py, px * px)), ph, pl);
    a[0] = zh; a[1] = zl; a[2] = zh; a[3] = zl;
    a[4] = ph; a[5] = pl; a[6] = (_Float16)1.f; a[7] = (_Float16)1.f;
  }
  return a;
}
__device__ __forceinline__ f16x8 frag_b(float qx, float qy, float qz, int h) {
  f16x8 b;
  if (h == 0) {
    _Float16 xh, xl, yh, yl;
    split(qx, xh, xl);
    split(qy, yh, yl);
    b[0] = -2 * xh; b[1] = -2 * xh; b[2] = -2 * xl; b[3] = -2 * xl;
    b[4] = -2 * yh; b[5] = -2 * yh; b[6] = -2 * yl; b[7] = -2 * yl;
  } else {
    _Float16 zh, zl, qh, ql;
    split(qz, zh, zl);
    split(fmaf(qz, qz, fmaf(qy, qy, qx * qx)), qh, ql);
    b[0] = -2 * zh; b[1] = -2 * zh; b[2] = -2 * zl; b[3] = -2 * zl;
    b[4] = (_Float16)1.f; b[5] = (_Float16)1.f; b[6] = qh; b[7] = ql;
  }
  return b;
}

// one wave per 32 queries x 32 candidates; D[i=cand][j=query] -> out[j*32+i]
__global__ void numerics_kernel(const float *q, const float *p, float *out, int ntiles) {
  const int l = threadIdx.x, h = l >> 5, i = l & 31;
  const int t = blockIdx.x;
  const float *qq = q + 3 * (t * 32 + i), *pp = p + 3 * (t * 32 + i);
  const f16x8 a = frag_a(pp[0], pp[1], pp[2], h);
  const f16x8 b = frag_b(qq[0], qq[1], qq[2], h);
  f32x16 c = {};
  c = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
  for (int r = 0; r < 16; r++) {
    const int row = (r & 3) + 8 * (r >> 2) + 4 * h;  // candidate
    out[(size_t)t * 1024 + (size_t)i * 32 + row] = c[r];
  }
}

static double drand(uint64_t &s) {
  s = s * 6364136223846793005ull + 1442695040888963407ull;
  return (double)((s >> 11) & ((1ull << 53) - 1)) / 9007199254740992.0;
}

int main() {
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, 0) != hipSuccess) {
    printf("no GPU\n");
    return 1;
  }
  const int cus = prop.multiProcessorCount;
  const int blocks = cus * 8;
  float *out;
  (void)hipMalloc(&out, sizeof(float) * blocks * kThreads);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const double ghz = 2.4, simds = 4.0 * cus;
  auto report = [&](const char *name, float ms, double units) {
    printf("%-44s %8.3f ms  %7.2f SIMD-cyc/unit\n", name, ms, ms * 1e-3 * ghz * 1e9 * simds / units);
  };
  float ms;
#define RUN(rep, label, units, ...)              \
  (void)hipEventRecord(e0);                      \
  __VA_ARGS__;                                   \
  (void)hipEventRecord(e1);                      \
  (void)hipEventSynchronize(e1);                 \
  (void)hipEventElapsedTime(&ms, e0, e1);        \
  if (rep) report(label, ms, units);
  const int mit = 4096;
  const double steps = (double)blocks * 4 * mit;
  for (int rep = 0; rep < 2; rep++) {
    RUN(rep, "2 mfma32x32x16f16 only (per step)", steps, mfma_kernel<0, true><<<blocks, kThreads>>>(out, mit));
    RUN(rep, "32 VALU only", steps, mfma_kernel<32, false><<<blocks, kThreads>>>(out, mit));
    RUN(rep, "2 mfma16 + 32 VALU", steps, mfma_kernel<32, true><<<blocks, kThreads>>>(out, mit));
    RUN(rep, "64 VALU only", steps, mfma_kernel<64, false><<<blocks, kThreads>>>(out, mit));
    RUN(rep, "2 mfma16 + 64 VALU", steps, mfma_kernel<64, true><<<blocks, kThreads>>>(out, mit));
    RUN(rep, "128 VALU only", steps, mfma_kernel<128, false><<<blocks, kThreads>>>(out, mit));
    RUN(rep, "2 mfma16 + 128 VALU", steps, mfma_kernel<128, true><<<blocks, kThreads>>>(out, mit));
    RUN(rep, "int: 64 VALU only", steps, mfma_int_kernel<32, false><<<blocks, kThreads>>>(out, mit));
    RUN(rep, "int: 2 mfma16 + 64 VALU", steps, mfma_int_kernel<32, true><<<blocks, kThreads>>>(out, mit));
    RUN(rep, "int: 128 VALU only", steps, mfma_int_kernel<64, false><<<blocks, kThreads>>>(out, mit));
    RUN(rep, "int: 2 mfma16 + 128 VALU", steps, mfma_int_kernel<64, true><<<blocks, kThreads>>>(out, mit));
  }
  const int ait = 1024;
  const double slots = (double)blocks * 4 * ait * 16;
  uint32_t *uout = (uint32_t *)out;
  for (int rep = 0; rep < 2; rep++) {
    RUN(rep, "tile: count+bits only (per slot)", slots, append_kernel<0><<<blocks, kThreads>>>(uout, ait, 3));
    RUN(rep, "tile + append loop, in-band 1/8", slots, append_kernel<1><<<blocks, kThreads>>>(uout, ait, 1));
    RUN(rep, "tile + append loop, in-band 1/16", slots, append_kernel<1><<<blocks, kThreads>>>(uout, ait, 2));
    RUN(rep, "tile + append loop, in-band 1/32", slots, append_kernel<1><<<blocks, kThreads>>>(uout, ait, 3));
    RUN(rep, "tile + append loop, in-band 1/64", slots, append_kernel<1><<<blocks, kThreads>>>(uout, ait, 4));
    RUN(rep, "tile + append loop, in-band 0", slots, append_kernel<1><<<blocks, kThreads>>>(uout, ait, 31));
  }
  // numerics
  const int nt = 4096;
  const size_t nq = (size_t)nt * 32;
  float *hq = (float *)malloc(nq * 12), *hp = (float *)malloc(nq * 12), *hd = (float *)malloc(nq * 32 * 4);
  uint64_t s = 7;
  for (int scen = 0; scen < 3; scen++) {
    // queries in a box of half-side qs, candidates in a ball-ish box of half-side ps (scaled units)
    const double qs = scen == 0 ? 0.3 : scen == 1 ? 0.6 : 0.05, ps = scen == 2 ? 0.2 : 1.0;
    for (size_t i = 0; i < nq * 3; i++) {
      hq[i] = (float)((drand(s) * 2 - 1) * qs);
      hp[i] = (float)((drand(s) * 2 - 1) * ps);
    }
    float *dq, *dp, *dd;
    (void)hipMalloc(&dq, nq * 12);
    (void)hipMalloc(&dp, nq * 12);
    (void)hipMalloc(&dd, nq * 32 * 4);
    (void)hipMemcpy(dq, hq, nq * 12, hipMemcpyHostToDevice);
    (void)hipMemcpy(dp, hp, nq * 12, hipMemcpyHostToDevice);
    numerics_kernel<<<nt, 64>>>(dq, dp, dd, nt);
    (void)hipMemcpy(hd, dd, nq * 32 * 4, hipMemcpyDeviceToHost);
    double worst_m = 0, worst_rel = 0;
    for (int t = 0; t < nt; t++) {
      double qm = 0, pm = 0;
      for (int i = 0; i < 32; i++) {
        const float *a = hq + 3 * (t * 32 + i), *b = hp + 3 * (t * 32 + i);
        qm = fmax(qm, sqrt((double)a[0] * a[0] + (double)a[1] * a[1] + (double)a[2] * a[2]));
        pm = fmax(pm, sqrt((double)b[0] * b[0] + (double)b[1] * b[1] + (double)b[2] * b[2]));
      }
      const double M2 = (qm + pm) * (qm + pm);
      for (int j = 0; j < 32; j++)
        for (int i = 0; i < 32; i++) {
          const float *a = hq + 3 * (t * 32 + j), *b = hp + 3 * (t * 32 + i);
          const double dx = (double)a[0] - b[0], dy = (double)a[1] - b[1], dz = (double)a[2] - b[2];
          const double d2 = dx * dx + dy * dy + dz * dz;
          const double err = fabs((double)hd[(size_t)t * 1024 + j * 32 + i] - d2);
          worst_m = fmax(worst_m, err / M2);
          if (d2 > 1e-3 * M2) worst_rel = fmax(worst_rel, err / d2);
        }
    }
    printf("numerics scenario %d (q half-side %.2f, p half-side %.2f): max |err|/M^2 = %.3e (2^%.1f), "
           "max |err|/d^2 (d^2 > 1e-3 M^2) = %.3e\n",
           scen, qs, ps, worst_m, log2(worst_m), worst_rel);
    (void)hipFree(dq);
    (void)hipFree(dp);
    (void)hipFree(dd);
  }
  return 0;
}
