// Bounds, Morton keys, gathers/scatters and small partitioning helpers (gfx950).
//
// Replaces the reference's host-side O(N) bounds loop (prePartitionedDataVariant.cu:
// 230-232) with a device reduction, and provides the Morton/partition primitives the
// spatial redistribution (unordered variant) is built from.
#include "dev.h"

#include <cstdio>
#include <mutex>

namespace lsk {
static std::mutex g_err_mu;
static std::string g_err;
void set_last_error(const std::string &msg) {
  std::lock_guard<std::mutex> g(g_err_mu);
  g_err = msg;
}
}  // namespace lsk

extern "C" int lsk_hip_abi_version(void) { return 10; }

extern "C" const char *lsk_hip_last_error(void) {
  static thread_local std::string copy;
  std::lock_guard<std::mutex> g(lsk::g_err_mu);
  copy = lsk::g_err;
  return copy.c_str();
}

extern "C" int lsk_hip_device_info(int device, char *buf, int buflen) {
  hipDeviceProp_t p;
  LSK_HIP(hipGetDeviceProperties(&p, device));
  std::snprintf(buf, (size_t)buflen, "%s arch=%s CUs=%d lds/block=%zu mem=%zu", p.name,
                p.gcnArchName, p.multiProcessorCount, (size_t)p.sharedMemPerBlock,
                (size_t)p.totalGlobalMem);
  return 0;
}

namespace {

constexpr int kBoundsThreads = 256;
constexpr unsigned kBoundsMaxBlocks = 2048;

__global__ __launch_bounds__(kBoundsThreads) void bounds_partial_kernel(
    const float *__restrict__ pts, int64_t n, float *__restrict__ partial) {
  const float inf = __builtin_inff();
  float l0 = inf, l1 = inf, l2 = inf, h0 = -inf, h1 = -inf, h2 = -inf;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const float x = pts[3 * i], y = pts[3 * i + 1], z = pts[3 * i + 2];
    l0 = fminf(l0, x); l1 = fminf(l1, y); l2 = fminf(l2, z);
    h0 = fmaxf(h0, x); h1 = fmaxf(h1, y); h2 = fmaxf(h2, z);
  }
  l0 = lsk::wave_min(l0); l1 = lsk::wave_min(l1); l2 = lsk::wave_min(l2);
  h0 = lsk::wave_max(h0); h1 = lsk::wave_max(h1); h2 = lsk::wave_max(h2);
  __shared__ float red[kBoundsThreads / lsk::kWave][6];
  const int w = threadIdx.x >> 6;
  if (lsk::lane_id() == 0) {
    red[w][0] = l0; red[w][1] = l1; red[w][2] = l2;
    red[w][3] = h0; red[w][4] = h1; red[w][5] = h2;
  }
  __syncthreads();
  if (threadIdx.x < 6) {
    float v = red[0][threadIdx.x];
    for (int j = 1; j < kBoundsThreads / lsk::kWave; j++)
      v = threadIdx.x < 3 ? fminf(v, red[j][threadIdx.x]) : fmaxf(v, red[j][threadIdx.x]);
    partial[6 * blockIdx.x + threadIdx.x] = v;
  }
}

__device__ void finalize_box(float *box) {
  const float ex = fmaxf(fmaxf(box[3] - box[0], box[4] - box[1]), box[5] - box[2]);
  const bool ok = ex > 0.f && ex < __builtin_inff();
  box[6] = ok ? 1024.f / ex : 0.f;
  box[7] = ok ? ex : 0.f;
}

__global__ void bounds_final_kernel(const float *__restrict__ partial, int nb,
                                    float *__restrict__ box) {
  const int t = threadIdx.x;  // 64 threads
  const float inf = __builtin_inff();
  float v[6] = {inf, inf, inf, -inf, -inf, -inf};
  for (int b = t; b < nb; b += 64) {
    for (int a = 0; a < 3; a++) v[a] = fminf(v[a], partial[6 * b + a]);
    for (int a = 3; a < 6; a++) v[a] = fmaxf(v[a], partial[6 * b + a]);
  }
  for (int a = 0; a < 3; a++) v[a] = lsk::wave_min(v[a]);
  for (int a = 3; a < 6; a++) v[a] = lsk::wave_max(v[a]);
  if (t == 0) {
    for (int a = 0; a < 6; a++) box[a] = v[a];
    finalize_box(box);
  }
}

__global__ void box_finalize_kernel(float *box) {
  if (threadIdx.x == 0) finalize_box(box);
}

// k-th-distance estimate for uniform density over the box's non-degenerate axes
// (knn_engine.radius_hint2; only used by groups of zero extent, so it need not match the
// host value bit for bit). 1 when nothing is known.
__global__ void radius_hint_kernel(const float *box, int64_t n_total, int32_t k, float *out) {
  if (threadIdx.x != 0) return;
  double measure = 1.0;
  int dim = 0;
  bool ok = n_total > 0;
  for (int a = 0; a < 3; a++) {
    const double e = (double)box[3 + a] - (double)box[a];
    if (!(e == e) || e == __builtin_inf() || e == -__builtin_inf()) ok = false;
    if (e > 0.0) {
      measure *= e;
      dim++;
    }
  }
  float r2 = 1.f;
  if (ok && dim > 0) {
    const double unit = dim == 1 ? 2.0 : dim == 2 ? 3.14159265358979323846 : 4.0 * 3.14159265358979323846 / 3.0;
    const double r = pow((double)k / (unit * ((double)n_total / measure)), 1.0 / dim);
    r2 = (float)(r * r);
  }
  out[0] = r2;
}

// keys (and vals = base + i) of pts in the cube of `box`; with `flag` the kernel does
// nothing unless *flag != 0 (a device-side decision inside a captured step: the
// streamed single-rank upload re-keys only when a point fell outside its provisional box)
__global__ __launch_bounds__(256) void morton_kernel(const float *__restrict__ pts, int64_t n,
                                                     const float *__restrict__ box,
                                                     uint32_t *__restrict__ keys,
                                                     uint32_t *__restrict__ vals, int curve,
                                                     uint32_t base, const int *__restrict__ flag) {
  if (flag && *flag == 0) return;
  const float ox = box[0], oy = box[1], oz = box[2], s = box[6];
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const uint32_t ix = lsk::morton_quant(pts[3 * i], ox, s);
    const uint32_t iy = lsk::morton_quant(pts[3 * i + 1], oy, s);
    const uint32_t iz = lsk::morton_quant(pts[3 * i + 2], oz, s);
    keys[i] = lsk::curve3(curve, ix, iy, iz);
    if (vals) vals[i] = base + (uint32_t)i;
  }
}

// dst[i] = src[idx[i]] for float3 rows. The reads are random 12-byte rows (the Hilbert
// order is unrelated to the input order), the writes contiguous: each block gathers a
// tile of kG3Per x 256 rows — all index loads first, then all row loads, so every lane
// has kG3Per random loads in flight — stages it in LDS and writes it out as float4s
// (fully coalesced, instead of three stride-12 dword stores per row). Partial last tile:
// direct stores.
constexpr int kG3Per = 4;  // 8 / 16 rows per lane: same 26.1-26.7 ms at 1B (profiles/r5_sort/gather_tile_1b.txt)
constexpr int kG3Tile = 256 * kG3Per;

__global__ __launch_bounds__(256) void gather3_kernel(const float *__restrict__ src,
                                                      const uint32_t *__restrict__ idx,
                                                      int64_t n, float *__restrict__ dst) {
  __shared__ float4 tile[kG3Tile * 3 / 4];
  float *tf = reinterpret_cast<float *>(tile);
  const int t = threadIdx.x;
  const int64_t base = (int64_t)blockIdx.x * kG3Tile;
  uint32_t j[kG3Per];
#pragma unroll
  for (int u = 0; u < kG3Per; u++) {
    const int64_t i = base + u * 256 + t;
    j[u] = i < n ? idx[i] : 0u;
  }
  float x[kG3Per], y[kG3Per], z[kG3Per];
#pragma unroll
  for (int u = 0; u < kG3Per; u++) {
    const float *p = src + 3 * (int64_t)j[u];
    x[u] = p[0]; y[u] = p[1]; z[u] = p[2];
  }
  if (base + kG3Tile <= n) {
#pragma unroll
    for (int u = 0; u < kG3Per; u++) {
      const int r = u * 256 + t;
      tf[3 * r] = x[u]; tf[3 * r + 1] = y[u]; tf[3 * r + 2] = z[u];
    }
    __syncthreads();
    float4 *d4 = reinterpret_cast<float4 *>(dst + 3 * base);
#pragma unroll
    for (int v = t; v < kG3Tile * 3 / 4; v += 256) d4[v] = tile[v];
  } else {
#pragma unroll
    for (int u = 0; u < kG3Per; u++) {
      const int64_t i = base + u * 256 + t;
      if (i < n) { dst[3 * i] = x[u]; dst[3 * i + 1] = y[u]; dst[3 * i + 2] = z[u]; }
    }
  }
}

__global__ __launch_bounds__(256) void scatter1_kernel(const float *__restrict__ src,
                                                       const uint32_t *__restrict__ idx,
                                                       int64_t n, float *__restrict__ dst,
                                                       int fin) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const float v = src[i];
    dst[idx[i]] = fin ? lsk::final_distance(v) : v;
  }
}

__global__ __launch_bounds__(256) void finalize_kernel(const float *__restrict__ src,
                                                       int64_t n, float *__restrict__ dst) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    dst[i] = lsk::final_distance(src[i]);
}

__global__ __launch_bounds__(256) void dest_rank_kernel(const uint32_t *__restrict__ morton,
                                                        int64_t n,
                                                        const uint32_t *__restrict__ split,
                                                        int nsplit, int shift,
                                                        uint32_t *__restrict__ dest,
                                                        uint32_t *__restrict__ vals) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const uint32_t key = morton[i] >> shift;
    // number of splitters <= key (splitters are ascending bin starts of ranks 1..P-1)
    int lo = 0, hi = nsplit;
    while (lo < hi) {
      int mid = (lo + hi) >> 1;
      if (split[mid] <= key) lo = mid + 1; else hi = mid;
    }
    dest[i] = (uint32_t)lo;
    if (vals) vals[i] = (uint32_t)i;
  }
}

// hist[keys[i * sample] >> shift] += 1: a strided sample is enough for the splitters
// (they only balance the load; exactness does not depend on them), and device-scope
// atomics on a histogram shared by all 8 XCDs are slow (125M keys: 5 ms unsampled).
__global__ __launch_bounds__(256) void key_hist_kernel(const uint32_t *__restrict__ keys,
                                                       int64_t n, int shift, int sample,
                                                       uint32_t *__restrict__ hist) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t m = (n + sample - 1) / sample;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += stride)
    atomicAdd(&hist[keys[i * sample] >> shift], 1u);
}

__global__ __launch_bounds__(256) void count_dest_kernel(const uint32_t *__restrict__ dest,
                                                         int64_t n, int ndest,
                                                         uint32_t *__restrict__ counts) {
  __shared__ uint32_t loc[1024];
  for (int i = threadIdx.x; i < ndest; i += blockDim.x) loc[i] = 0;
  __syncthreads();
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const uint32_t d = dest[i];
    if (d < (uint32_t)ndest) atomicAdd(&loc[d], 1u);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < ndest; i += blockDim.x)
    if (loc[i]) atomicAdd(&counts[i], loc[i]);
}

}  // namespace

extern "C" size_t lsk_hip_bounds_ws_bytes(int64_t) { return kBoundsMaxBlocks * 6 * sizeof(float); }

extern "C" int lsk_hip_bounds(const float *pts, int64_t n, float *box_out, void *ws,
                              void *stream) {
  hipStream_t s = (hipStream_t)stream;
  unsigned nb = lsk_blocks(n, kBoundsThreads * 8, kBoundsMaxBlocks);
  bounds_partial_kernel<<<nb, kBoundsThreads, 0, s>>>(pts, n, (float *)ws);
  LSK_CHECK_LAUNCH("bounds_partial");
  bounds_final_kernel<<<1, 64, 0, s>>>((const float *)ws, (int)nb, box_out);
  LSK_CHECK_LAUNCH("bounds_final");
  return 0;
}

extern "C" int lsk_hip_radius_hint(const float *box, int64_t n_total, int32_t k, float *out,
                                   void *stream) {
  radius_hint_kernel<<<1, 64, 0, (hipStream_t)stream>>>(box, n_total, k, out);
  LSK_CHECK_LAUNCH("radius_hint");
  return 0;
}

extern "C" int lsk_hip_box_finalize(float *box, void *stream) {
  box_finalize_kernel<<<1, 64, 0, (hipStream_t)stream>>>(box);
  LSK_CHECK_LAUNCH("box_finalize");
  return 0;
}

extern "C" int lsk_hip_morton(const float *pts, int64_t n, const float *box, uint32_t *keys,
                              uint32_t *vals, int curve, void *stream) {
  if (n <= 0) return 0;
  morton_kernel<<<lsk_blocks(n, 256 * 4, 8192), 256, 0, (hipStream_t)stream>>>(pts, n, box,
                                                                             keys, vals, curve, 0u,
                                                                             nullptr);
  LSK_CHECK_LAUNCH("morton");
  return 0;
}

extern "C" int lsk_hip_morton_ex(const float *pts, int64_t n, const float *box, uint32_t *keys,
                                 uint32_t *vals, int curve, int64_t base, const int *flag, void *stream) {
  if (n <= 0) return 0;
  if (base < 0 || base + n > ((int64_t)1 << 32)) {
    lsk::set_last_error("morton_ex: indices must fit in 32 bits");
    return 1;
  }
  morton_kernel<<<lsk_blocks(n, 256 * 4, 8192), 256, 0, (hipStream_t)stream>>>(
      pts, n, box, keys, vals, curve, (uint32_t)base, flag);
  LSK_CHECK_LAUNCH("morton_ex");
  return 0;
}

extern "C" int lsk_hip_gather3(const float *src, const uint32_t *idx, int64_t n, float *dst,
                               void *stream) {
  if (n <= 0) return 0;
  if (((uintptr_t)dst & 15u) != 0) {
    lsk::set_last_error("gather3: dst must be 16-byte aligned");
    return 1;
  }
  gather3_kernel<<<lsk_blocks(n, kG3Tile), 256, 0, (hipStream_t)stream>>>(src, idx, n, dst);
  LSK_CHECK_LAUNCH("gather3");
  return 0;
}

extern "C" int lsk_hip_scatter1(const float *src, const uint32_t *idx, int64_t n, float *dst,
                                int finalize_sqrt, void *stream) {
  if (n <= 0) return 0;
  scatter1_kernel<<<lsk_blocks(n, 256 * 4, 8192), 256, 0, (hipStream_t)stream>>>(
      src, idx, n, dst, finalize_sqrt);
  LSK_CHECK_LAUNCH("scatter1");
  return 0;
}

extern "C" int lsk_hip_finalize(const float *src, int64_t n, float *dst, void *stream) {
  if (n <= 0) return 0;
  finalize_kernel<<<lsk_blocks(n, 256 * 4, 8192), 256, 0, (hipStream_t)stream>>>(src, n, dst);
  LSK_CHECK_LAUNCH("finalize");
  return 0;
}

extern "C" int lsk_hip_dest_rank(const uint32_t *morton, int64_t n, const uint32_t *splitters,
                                 int nsplit, int shift, uint32_t *dest, uint32_t *vals,
                                 void *stream) {
  if (n <= 0) return 0;
  dest_rank_kernel<<<lsk_blocks(n, 256 * 4, 8192), 256, 0, (hipStream_t)stream>>>(
      morton, n, splitters, nsplit, shift, dest, vals);
  LSK_CHECK_LAUNCH("dest_rank");
  return 0;
}

extern "C" int lsk_hip_key_histogram(const uint32_t *keys, int64_t n, int shift, int sample,
                                     uint32_t *hist, void *stream) {
  if (n <= 0) return 0;
  if (sample < 1) {
    lsk::set_last_error("key_histogram: sample must be >= 1");
    return 1;
  }
  const int64_t m = (n + sample - 1) / sample;
  key_hist_kernel<<<lsk_blocks(m, 256 * 8, 4096), 256, 0, (hipStream_t)stream>>>(keys, n, shift,
                                                                               sample, hist);
  LSK_CHECK_LAUNCH("key_histogram");
  return 0;
}

extern "C" int lsk_hip_count_dest(const uint32_t *dest, int64_t n, int ndest, uint32_t *counts,
                                  void *stream) {
  if (n <= 0) return 0;
  if (ndest > 1024) {
    lsk::set_last_error("count_dest: ndest > 1024");
    return 1;
  }
  count_dest_kernel<<<lsk_blocks(n, 256 * 16, 2048), 256, 0, (hipStream_t)stream>>>(dest, n, ndest,
                                                                                  counts);
  LSK_CHECK_LAUNCH("count_dest");
  return 0;
}

// ---- per-segment bounding boxes (heavy-cell refinement, knn_engine.refine_heavy_cells)
namespace {

// order-preserving float <-> uint map (atomicMin/Max on uint = float min/max)
__device__ __forceinline__ uint32_t ord_of(float f) {
  const uint32_t b = __float_as_uint(f);
  return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}

constexpr int kSegPer = 16;  // elements per lane

// Segments are contiguous runs of equal seg ids. A wave takes 64 x kSegPer consecutive
// elements; lanes reduce their own elements while the id stays the same, then a wave
// reduction per distinct id (wave-uniform loop over the few ids in the window) and one
// atomic per (wave, id, component): a 1e7-point segment costs ~1e4 atomics per address,
// not 1e7 contended compare-and-swaps (torch.scatter_reduce).
__global__ __launch_bounds__(256) void segment_bounds_kernel(const float *__restrict__ p,
                                                             const uint32_t *__restrict__ seg,
                                                             int64_t m, uint32_t *__restrict__ lo,
                                                             uint32_t *__restrict__ hi) {
  const int lane = lsk::lane_id();
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t w = (((int64_t)blockIdx.x * blockDim.x) >> 6) + (threadIdx.x >> 6);
       w * 64 * kSegPer < m; w += nwaves) {
    const int64_t base = w * 64 * kSegPer;
    const int64_t end = base + 64 * kSegPer < m ? base + 64 * kSegPer : m;
    // lane l handles elements base + l*kSegPer ... (contiguous per lane)
    const int64_t b0 = base + (int64_t)lane * kSegPer;
    uint32_t cur = 0xffffffffu;
    uint32_t l0 = 0xffffffffu, l1 = 0xffffffffu, l2 = 0xffffffffu, h0 = 0, h1 = 0, h2 = 0;
    auto flush = [&]() {
      if (cur != 0xffffffffu) {
        atomicMin(&lo[3 * (int64_t)cur], l0); atomicMin(&lo[3 * (int64_t)cur + 1], l1);
        atomicMin(&lo[3 * (int64_t)cur + 2], l2);
        atomicMax(&hi[3 * (int64_t)cur], h0); atomicMax(&hi[3 * (int64_t)cur + 1], h1);
        atomicMax(&hi[3 * (int64_t)cur + 2], h2);
      }
    };
    // fast path: the whole window is one segment -> one wave reduction, lane 0 flushes
    const uint32_t s_first = seg[base], s_last = seg[end - 1];
    if (s_first == s_last) {
      for (int j = 0; j < kSegPer; j++) {
        const int64_t i = b0 + j;
        if (i < end) {
          const uint32_t x = ord_of(p[3 * i]), y = ord_of(p[3 * i + 1]), z = ord_of(p[3 * i + 2]);
          l0 = min(l0, x); l1 = min(l1, y); l2 = min(l2, z);
          h0 = max(h0, x); h1 = max(h1, y); h2 = max(h2, z);
        }
      }
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        l0 = min(l0, (uint32_t)__shfl_xor((int)l0, o)); l1 = min(l1, (uint32_t)__shfl_xor((int)l1, o));
        l2 = min(l2, (uint32_t)__shfl_xor((int)l2, o)); h0 = max(h0, (uint32_t)__shfl_xor((int)h0, o));
        h1 = max(h1, (uint32_t)__shfl_xor((int)h1, o)); h2 = max(h2, (uint32_t)__shfl_xor((int)h2, o));
      }
      if (lane == 0) {
        cur = s_first;
        flush();
      }
      continue;
    }
    // boundary window: per-lane runs, one flush per lane-run
    for (int j = 0; j < kSegPer; j++) {
      const int64_t i = b0 + j;
      if (i >= end) break;
      const uint32_t s = seg[i];
      if (s != cur) {
        flush();
        cur = s;
        l0 = l1 = l2 = 0xffffffffu;
        h0 = h1 = h2 = 0u;
      }
      const uint32_t x = ord_of(p[3 * i]), y = ord_of(p[3 * i + 1]), z = ord_of(p[3 * i + 2]);
      l0 = min(l0, x); l1 = min(l1, y); l2 = min(l2, z);
      h0 = max(h0, x); h1 = max(h1, y); h2 = max(h2, z);
    }
    flush();
  }
}

__global__ __launch_bounds__(256) void ord_to_float_kernel(uint32_t *__restrict__ v, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const uint32_t u = v[i];
    v[i] = (u & 0x80000000u) ? (u & 0x7fffffffu) : ~u;
  }
}

}  // namespace

extern "C" int lsk_hip_segment_bounds(const float *pts, const uint32_t *seg, int64_t m, int64_t nseg,
                                      float *lo, float *hi, void *stream) {
  hipStream_t s = (hipStream_t)stream;
  if (nseg <= 0) return 0;
  LSK_HIP(lsk_fill32(lo, 0xffffffffu, nseg * 3, s));
  LSK_HIP(lsk_fill32(hi, 0u, nseg * 3, s));
  if (m > 0) {
    segment_bounds_kernel<<<lsk_blocks(m, 256 * kSegPer, 8192), 256, 0, s>>>(
        pts, seg, m, (uint32_t *)lo, (uint32_t *)hi);
    LSK_CHECK_LAUNCH("segment_bounds");
  }
  const int64_t tot = nseg * 3;
  ord_to_float_kernel<<<lsk_blocks(tot, 256 * 4, 8192), 256, 0, s>>>((uint32_t *)lo, tot);
  LSK_CHECK_LAUNCH("segment_bounds_lo");
  ord_to_float_kernel<<<lsk_blocks(tot, 256 * 4, 8192), 256, 0, s>>>((uint32_t *)hi, tot);
  LSK_CHECK_LAUNCH("segment_bounds_hi");
  return 0;
}
