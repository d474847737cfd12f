// Hand-written LSD radix sort of (uint32 key, uint32 value) pairs for gfx950.
//
// Used for the Morton sort that precedes the bucket k-d tree build (the reference's
// cukd::buildTree sorts with thrust, unorderedDataVariant.cu:161 [inferred]; SURVEY
// §7.5 H5) and for the destination-rank partition of the spatial redistribution.
//
// Per 8-bit digit pass (reduce-then-scan, stable):
//   upsweep   : each block histograms its contiguous chunk          -> counts[d][blk]
//   scan      : one 1024-thread block scans counts (digit-major)     -> global offsets
//   downsweep : each block walks its chunk in 4096-element tiles; a wave ranks its 64
//               lanes per row with 8 ballots (wave-64 multisplit), waves are combined
//               through LDS prefix sums, the tile is staged in LDS in digit order and
//               written out in coalesced digit runs.
#include "dev.h"

namespace {

constexpr int kThreads = 256;
constexpr int kWaves = kThreads / lsk::kWave;
constexpr int kRadix = 256;
#ifndef LSK_SORT_ROWS
#define LSK_SORT_ROWS 16
#endif
constexpr int kRows = LSK_SORT_ROWS;  // rows of 64 per wave per tile (8: 36.5 vs 33.6 ms for 1B keys)
constexpr int kTile = kWaves * lsk::kWave * kRows;     // 4096 elements
constexpr unsigned kMaxBlocks = 2048;

__device__ __forceinline__ int64_t chunk_begin(int64_t n, unsigned b, unsigned nb) {
  return (int64_t)(((__uint128_t)n * b) / nb);
}

// The chunk's aligned middle is read as 16-byte vectors, four per lane in flight: 0.71 ms
// per pass over 1B keys (5.6 TB/s; one dword per lane and iteration: 1.12 ms alone, and
// 5.4 ms beside the stream's copies, profiles/r5_sort/).
__global__ __launch_bounds__(kThreads) void upsweep_kernel(const uint32_t *__restrict__ keys,
                                                           int64_t n, int shift,
                                                           uint32_t *__restrict__ counts) {
  __shared__ uint32_t h[kWaves][kRadix];
  const int t = threadIdx.x, w = t >> 6;
  for (int i = t; i < kWaves * kRadix; i += kThreads) (&h[0][0])[i] = 0;
  __syncthreads();
  const int64_t cb = chunk_begin(n, blockIdx.x, gridDim.x);
  const int64_t ce = chunk_begin(n, blockIdx.x + 1, gridDim.x);
  auto add = [&](uint32_t k) { atomicAdd(&h[w][(k >> shift) & 255u], 1u); };
  // [a0, a1): the 16-byte-aligned middle (keys may start at any dword); head and tail by dwords
  const int64_t off = (int64_t)(((uintptr_t)keys >> 2) & 3u);
  const int64_t a0 = min(ce, cb + ((4 - ((cb + off) & 3)) & 3));
  const int64_t a1 = max(a0, ce - ((ce + off) & 3));
  auto add4 = [&](uint4 v) { add(v.x); add(v.y); add(v.z); add(v.w); };
  for (int64_t i = cb + t; i < a0; i += kThreads) add(keys[i]);
  for (int64_t i = a1 + t; i < ce; i += kThreads) add(keys[i]);
  const uint4 *k4 = reinterpret_cast<const uint4 *>(keys + a0);
  const int64_t n4 = (a1 - a0) >> 2;
  int64_t j = t;
  for (; j + 3 * kThreads < n4; j += 4 * kThreads) {
    const uint4 v0 = k4[j], v1 = k4[j + kThreads], v2 = k4[j + 2 * kThreads], v3 = k4[j + 3 * kThreads];
    add4(v0); add4(v1); add4(v2); add4(v3);
  }
  for (; j < n4; j += kThreads) add4(k4[j]);
  __syncthreads();
  uint32_t s = 0;
  for (int j = 0; j < kWaves; j++) s += h[j][t];
  counts[(size_t)t * gridDim.x + blockIdx.x] = s;
}

// Block-wide exclusive scan of one value per thread (kThreads threads).
template <int NT>
__device__ __forceinline__ uint32_t block_exclusive_scan(uint32_t v, uint32_t *wave_tot,
                                                         uint32_t *total) {
  const int lane = lsk::lane_id(), w = threadIdx.x >> 6;
  uint32_t x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    uint32_t y = __shfl_up(x, o);
    if (lane >= o) x += y;
  }
  if (lane == 63) wave_tot[w] = x;
  __syncthreads();
  uint32_t pre = 0, tot = 0;
  for (int j = 0; j < NT / 64; j++) {
    uint32_t c = wave_tot[j];
    if (j < w) pre += c;
    tot += c;
  }
  if (total) *total = tot;
  __syncthreads();
  return pre + x - v;
}

// In-place exclusive scan of the digit-major counts by one 1024-thread block, in
// coalesced chunks of 8 consecutive counts per thread (two 16-byte loads), carrying the
// running total between chunks. (A per-thread contiguous segment instead makes every
// wave touch 64 cache lines per step: 0.6-0.75 ms per pass at 2048 blocks.)
constexpr int kScanThreads = 1024;
constexpr int kScanPer = 8;
__global__ __launch_bounds__(kScanThreads) void scan_kernel(uint32_t *__restrict__ counts,
                                                            int64_t total) {
  __shared__ uint32_t wave_tot[kScanThreads / 64];
  __shared__ uint32_t carry_s;
  const int t = threadIdx.x;
  if (t == 0) carry_s = 0;
  __syncthreads();
  for (int64_t base = 0; base < total; base += (int64_t)kScanThreads * kScanPer) {
    const int64_t i0 = base + (int64_t)t * kScanPer;
    uint32_t v[kScanPer];
    if (i0 + kScanPer <= total) {
      const uint4 a = *(const uint4 *)(counts + i0), b = *(const uint4 *)(counts + i0 + 4);
      v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
      v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
    } else {
#pragma unroll
      for (int j = 0; j < kScanPer; j++) v[j] = i0 + j < total ? counts[i0 + j] : 0u;
    }
    uint32_t s = 0;
#pragma unroll
    for (int j = 0; j < kScanPer; j++) s += v[j];
    uint32_t tot;
    const uint32_t carry = carry_s;
    uint32_t run = carry + block_exclusive_scan<kScanThreads>(s, wave_tot, &tot);
#pragma unroll
    for (int j = 0; j < kScanPer; j++) {
      const uint32_t c = v[j];
      v[j] = run;
      run += c;
    }
    if (i0 + kScanPer <= total) {
      *(uint4 *)(counts + i0) = make_uint4(v[0], v[1], v[2], v[3]);
      *(uint4 *)(counts + i0 + 4) = make_uint4(v[4], v[5], v[6], v[7]);
    } else {
#pragma unroll
      for (int j = 0; j < kScanPer; j++)
        if (i0 + j < total) counts[i0 + j] = v[j];
    }
    if (t == 0) carry_s = carry + tot;  // every thread read carry_s before the scan's barriers
    __syncthreads();
  }
}

// 6.6 ms per pass for 1B pairs (2.4 TB/s). Loading tile t+1 while tile t is written out
// (208 VGPRs) and a 4-waves/SIMD occupancy hint (66 VGPRs spilled) measured the same
// (profiles/r5_sort/).
// GATHER (the last pass of lsk_hip_sort_keys_iota_gather): the values are the points'
// input rows; every element's point is read from pin and written at its sorted position
// in pout as the pair is scattered (the separate gather3 pass and its read of the
// permutation fused into the sort).
template <bool GATHER>
__global__ __launch_bounds__(kThreads) void downsweep_kernel(
    const uint32_t *__restrict__ kin, const uint32_t *__restrict__ vin,
    uint32_t *__restrict__ kout, uint32_t *__restrict__ vout, int64_t n, int shift,
    const uint32_t *__restrict__ offsets, const float *__restrict__ pin, float *__restrict__ pout) {
  __shared__ uint32_t wave_cnt[kWaves][kRadix];
  __shared__ uint32_t run_base[kRadix];
  __shared__ uint32_t tile_start[kRadix];
  __shared__ uint32_t tile_total[kRadix];
  __shared__ uint32_t wave_tot[kWaves];
  __shared__ uint32_t stage_k[kTile];
  __shared__ uint32_t stage_v[kTile];

  const int t = threadIdx.x, w = t >> 6, lane = lsk::lane_id();
  const uint64_t lt_mask = (1ull << lane) - 1ull;
  const int64_t cb = chunk_begin(n, blockIdx.x, gridDim.x);
  const int64_t ce = chunk_begin(n, blockIdx.x + 1, gridDim.x);
  run_base[t] = offsets[(size_t)t * gridDim.x + blockIdx.x];

  for (int64_t tb = cb; tb < ce; tb += kTile) {
    const int tn = (int)((ce - tb) < kTile ? (ce - tb) : kTile);
    for (int i = t; i < kWaves * kRadix; i += kThreads) (&wave_cnt[0][0])[i] = 0;
    __syncthreads();

    uint32_t kr[kRows], vr[kRows], offr[kRows];
#pragma unroll
    for (int r = 0; r < kRows; r++) {
      const int e = w * (lsk::kWave * kRows) + r * lsk::kWave + lane;
      const bool valid = e < tn;
      kr[r] = valid ? kin[tb + e] : 0u;
      // vin == NULL (the first pass of lsk_hip_sort_keys_iota): the value is the index
      vr[r] = valid ? (vin ? vin[tb + e] : (uint32_t)(tb + e)) : 0u;
    }
#pragma unroll
    for (int r = 0; r < kRows; r++) {
      const int e = w * (lsk::kWave * kRows) + r * lsk::kWave + lane;
      const bool valid = e < tn;
      const uint32_t d = (kr[r] >> shift) & 255u;
      uint64_t match = __ballot(valid);
#pragma unroll
      for (int bit = 0; bit < 8; bit++) {
        const bool on = (d >> bit) & 1u;
        const uint64_t b = __ballot(on);
        match &= on ? b : ~b;
      }
      const uint32_t before = valid ? wave_cnt[w][d] : 0u;
      offr[r] = before + (uint32_t)__popcll(match & lt_mask);
      // the highest lane of each digit group publishes the new running count
      if (valid && (match >> lane) == 1ull) wave_cnt[w][d] = before + (uint32_t)__popcll(match);
    }
    __syncthreads();
    {
      uint32_t s = 0;
#pragma unroll
      for (int j = 0; j < kWaves; j++) {
        uint32_t c = wave_cnt[j][t];
        wave_cnt[j][t] = s;
        s += c;
      }
      tile_total[t] = s;
      tile_start[t] = block_exclusive_scan<kThreads>(s, wave_tot, nullptr);
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kRows; r++) {
      const int e = w * (lsk::kWave * kRows) + r * lsk::kWave + lane;
      if (e < tn) {
        const uint32_t d = (kr[r] >> shift) & 255u;
        const uint32_t lp = tile_start[d] + wave_cnt[w][d] + offr[r];
        stage_k[lp] = kr[r];
        stage_v[lp] = vr[r];
      }
    }
    __syncthreads();
    if (GATHER) {
      // four elements per thread in flight: their random 12-byte point reads overlap
      constexpr int kU = 4;
      for (int i0 = t; i0 < tn; i0 += kU * kThreads) {
        uint32_t gg[kU], vv[kU];
        float x[kU], y[kU], z[kU];
#pragma unroll
        for (int u = 0; u < kU; u++) {
          const int i = i0 + u * kThreads;
          const uint32_t k = i < tn ? stage_k[i] : 0u;
          const uint32_t d = (k >> shift) & 255u;
          gg[u] = run_base[d] + (uint32_t)i - tile_start[d];
          vv[u] = i < tn ? stage_v[i] : 0u;
          if (i < tn) {
            kout[gg[u]] = k;
            vout[gg[u]] = vv[u];
          }
        }
#pragma unroll
        for (int u = 0; u < kU; u++) {
          const float *p = pin + 3ull * vv[u];  // (row 0 for the padding slots: in bounds)
          x[u] = p[0];
          y[u] = p[1];
          z[u] = p[2];
        }
#pragma unroll
        for (int u = 0; u < kU; u++) {
          if (i0 + u * kThreads < tn) {
            float *q = pout + 3ull * gg[u];
            q[0] = x[u];
            q[1] = y[u];
            q[2] = z[u];
          }
        }
      }
    } else {
      for (int i = t; i < tn; i += kThreads) {
        const uint32_t k = stage_k[i];
        const uint32_t d = (k >> shift) & 255u;
        const uint32_t g = run_base[d] + (uint32_t)i - tile_start[d];
        kout[g] = k;
        vout[g] = stage_v[i];
      }
    }
    __syncthreads();
    run_base[t] += tile_total[t];
    __syncthreads();
  }
}

unsigned sort_blocks(int64_t n) { return lsk_blocks(n, kTile, kMaxBlocks); }

}  // namespace

extern "C" size_t lsk_hip_sort_ws_bytes(int64_t n) {
  return (size_t)kRadix * sort_blocks(n) * sizeof(uint32_t) + 256;
}

static int sort_impl(uint32_t *keys, uint32_t *vals, uint32_t *keys_alt, uint32_t *vals_alt, int64_t n,
                     int key_bits, void *ws, int *result_in_alt, bool iota, void *stream,
                     const float *pin = nullptr, float *pout = nullptr) {
  hipStream_t s = (hipStream_t)stream;
  *result_in_alt = 0;
  if (n <= 1 || key_bits <= 0) return 0;
  if (n >= (int64_t(1) << 32)) {
    lsk::set_last_error("sort_pairs: n must be < 2^32");
    return 1;
  }
  const unsigned nb = sort_blocks(n);
  uint32_t *counts = (uint32_t *)ws;
  uint32_t *ki = keys, *vi = vals, *ko = keys_alt, *vo = vals_alt;
  int passes = 0;
  for (int shift = 0; shift < key_bits; shift += 8, passes++) {
    upsweep_kernel<<<nb, kThreads, 0, s>>>(ki, n, shift, counts);
    LSK_CHECK_LAUNCH("sort_upsweep");
    scan_kernel<<<1, 1024, 0, s>>>(counts, (int64_t)kRadix * nb);
    LSK_CHECK_LAUNCH("sort_scan");
    const uint32_t *vsrc = (iota && passes == 0) ? nullptr : vi;
    if (pin && shift + 8 >= key_bits)  // the last pass: scatter the points too
      downsweep_kernel<true><<<nb, kThreads, 0, s>>>(ki, vsrc, ko, vo, n, shift, counts, pin, pout);
    else
      downsweep_kernel<false><<<nb, kThreads, 0, s>>>(ki, vsrc, ko, vo, n, shift, counts, nullptr, nullptr);
    LSK_CHECK_LAUNCH("sort_downsweep");
    std::swap(ki, ko);
    std::swap(vi, vo);
  }
  *result_in_alt = passes & 1;
  return 0;
}

extern "C" int lsk_hip_sort_pairs(uint32_t *keys, uint32_t *vals, uint32_t *keys_alt, uint32_t *vals_alt,
                                  int64_t n, int key_bits, void *ws, int *result_in_alt, void *stream) {
  return sort_impl(keys, vals, keys_alt, vals_alt, n, key_bits, ws, result_in_alt, false, stream);
}

// As lsk_hip_sort_pairs with the values 0..n-1 generated by the first pass (vals is only
// a ping-pong buffer: its contents are not read) — no iota array to write and read back.
extern "C" int lsk_hip_sort_keys_iota(uint32_t *keys, uint32_t *vals, uint32_t *keys_alt, uint32_t *vals_alt,
                                      int64_t n, int key_bits, void *ws, int *result_in_alt, void *stream) {
  if (n == 1) {  // (no pass runs: the single value must still be written)
    hipStream_t s = (hipStream_t)stream;
    LSK_HIP(lsk_fill32(vals, 0u, 1, s));
    *result_in_alt = 0;
    return 0;
  }
  return sort_impl(keys, vals, keys_alt, vals_alt, n, key_bits, ws, result_in_alt, true, stream);
}

// As lsk_hip_sort_keys_iota, and pout[j] = pin[perm[j]] (float3 rows) for the sorted
// order, written by the last pass (no separate gather). n >= 2 (one point: gather3).
extern "C" int lsk_hip_sort_keys_iota_gather(uint32_t *keys, uint32_t *vals, uint32_t *keys_alt, uint32_t *vals_alt,
                                             int64_t n, int key_bits, void *ws, int *result_in_alt, const float *pin,
                                             float *pout, void *stream) {
  if (n < 2 || key_bits <= 0 || !pin || !pout) {
    lsk::set_last_error("sort_keys_iota_gather: n >= 2, key_bits > 0 and both point arrays required");
    return 1;
  }
  return sort_impl(keys, vals, keys_alt, vals_alt, n, key_bits, ws, result_in_alt, true, stream, pin, pout);
}
