// Device-side helpers shared by the lsknn gfx950 kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>

#include "../common.h"
#include "lsk_hip.h"

namespace lsk {

constexpr int kWave = 64;
constexpr int kBucket = 64;  // points per tree leaf == queries per wave group

// Constant-address-space view of read-only global data: uniform-address loads through
// it become scalar (SMEM) loads, so wave-uniform candidate points arrive in SGPRs and
// cost no VALU or LDS issue slots.
typedef const __attribute__((address_space(4))) float *cfloat_p;
typedef float v4f __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(4))) v4f *cfloat4_p;
typedef const __attribute__((address_space(4))) uint32_t *cuint_p;

__device__ __forceinline__ cfloat_p as_const(const float *p) { return (cfloat_p)(p); }
__device__ __forceinline__ cfloat4_p as_const4(const float *p) { return (cfloat4_p)(p); }

__device__ __forceinline__ uint32_t uniform(uint32_t v) {
  return __builtin_amdgcn_readfirstlane(v);
}
__device__ __forceinline__ float uniform_f(float v) {
  return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v)));
}
__device__ __forceinline__ int lane_id() { return __lane_id(); }

// Wave reductions. The result is equal in every lane; the final readfirstlane makes it
// provably uniform (an SGPR): without it, control flow that depends on the value is
// compiled as divergent (exec-masked loops, per-lane copies of scalar state).
__device__ __forceinline__ float wave_min(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fminf(v, __shfl_xor(v, o));
  return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v)));
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
  return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v)));
}
__device__ __forceinline__ float wave_sum_f(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v)));
}
__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return (uint32_t)__builtin_amdgcn_readfirstlane((int)v);
}

// K-th smallest (1-based) of a per-lane uint32 over the wave, by a bitwise ballot
// search (32 rounds of compare + ballot + popcount); uniform result.
__device__ __forceinline__ uint32_t wave_kth_smallest(uint32_t v, uint32_t K) {
  uint32_t lo = 0;  // largest value with count(v < lo) < K
#pragma unroll
  for (int b = 31; b >= 0; --b) {
    const uint32_t cand = lo | (1u << b);
    if ((uint32_t)__popcll(__ballot(v < cand)) < K) lo = cand;
  }
  return (uint32_t)__builtin_amdgcn_readfirstlane((int)lo);
}

// Bijective XCD-aware block remap (cdna_hip_programming.md §5.5 T1): blocks are dealt
// round-robin over the 8 XCDs; give each XCD a contiguous range of logical blocks so
// spatially adjacent query groups share an L2.
__device__ __forceinline__ uint32_t xcd_remap(uint32_t bid, uint32_t nblk) {
  const uint32_t q = nblk / 8, r = nblk % 8;
  const uint32_t xcd = bid % 8, local = bid / 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + local;
}

// Blocks of a launch that have work. A launch over a group list whose length is counted
// on the device (A.groups + A.ngroups_dev: a rank's interior / boundary groups) is sized by
// the list's bound and most of its tail blocks return at once; remapping over the whole
// grid would give the XCDs holding the tail ranges almost nothing to do (a 95 % list: the
// other XCDs carry 0.125 of the work each instead of 0.119). Blocks at or past the result
// must return without work (the remap is a bijection on [0, result) only).
template <class Args>
__device__ __forceinline__ uint32_t list_blocks(const Args &A, uint32_t nblk, uint32_t waves_per_block) {
  if (!(A.groups && A.ngroups_dev)) return nblk;
  const uint64_t cnt = min((uint64_t)A.ngroups, (uint64_t)*A.ngroups_dev);
  const uint64_t base = (uint32_t)A.wave_base;
  const uint64_t need = cnt > base ? (cnt - base + waves_per_block - 1) / waves_per_block : 0;
  return (uint32_t)min(need, (uint64_t)nblk);
}

// Next group of a persistent launch with a work queue (lsk_knn_args.wq, zeroed per
// launch): lane 0 takes it with one global atomic, the wave shares it. Waves take groups
// as they finish the previous one, so groups of very different cost (a short device-
// counted list: the halo re-query) balance across the GPU instead of striding statically.
__device__ __forceinline__ uint64_t wq_next(uint32_t *wq, uint32_t base) {
  uint32_t w = 0;
  if (lane_id() == 0) w = atomicAdd(wq, 1u);
  return (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)w) + base;
}

}  // namespace lsk

// -------------------------------------------------------------------- host-side errors
namespace lsk {
void set_last_error(const std::string &msg);
}

#define LSK_CHECK_LAUNCH(name)                                                        \
  do {                                                                                \
    hipError_t e__ = hipGetLastError();                                               \
    if (e__ != hipSuccess) {                                                          \
      lsk::set_last_error(std::string(name) + ": " + hipGetErrorString(e__));         \
      return (int)e__;                                                                \
    }                                                                                 \
  } while (0)

#define LSK_HIP(call)                                                                 \
  do {                                                                                \
    hipError_t e__ = (call);                                                          \
    if (e__ != hipSuccess) {                                                          \
      lsk::set_last_error(std::string(#call) + ": " + hipGetErrorString(e__));        \
      return (int)e__;                                                                \
    }                                                                                 \
  } while (0)

static inline unsigned lsk_blocks(int64_t n, int per_block, unsigned cap = 0) {
  int64_t b = (n + per_block - 1) / per_block;
  if (b < 1) b = 1;
  if (cap && b > (int64_t)cap) b = cap;
  return (unsigned)b;
}

// Fill nwords 32-bit words with v by a kernel instead of hipMemsetAsync: memset nodes in a
// captured HIP graph were seen not to re-run on later replays (ROCm 7.0: the 88-byte and
// 4-byte ones of the level census, and the grid's slot table — tests/test_gpu_graph.py read
// a stale table after a replay on other data); a kernel node always does.
__global__ __launch_bounds__(256) static void lsk_fill32_kernel(uint32_t *__restrict__ p, uint32_t v,
                                                                int64_t nwords) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nwords; i += stride) p[i] = v;
}

static inline hipError_t lsk_fill32(void *p, uint32_t v, int64_t nwords, hipStream_t st) {
  if (nwords <= 0) return hipSuccess;
  lsk_fill32_kernel<<<lsk_blocks(nwords, 256 * 4, 4096), 256, 0, st>>>((uint32_t *)p, v, nwords);
  return hipGetLastError();
}
