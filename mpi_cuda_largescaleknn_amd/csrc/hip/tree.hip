// Bucket k-d tree over Morton-sorted points (gfx950).
//
// The reference builds a left-balanced object-median k-d tree in place with
// cukd::buildTree (unorderedDataVariant.cu:161, prePartitionedDataVariant.cu:271,
// [inferred]). Here the tree comes from the Morton sort: sorted points are cut into
// 64-point buckets (one wavefront of candidates per leaf), and an implicit complete
// binary tree over the buckets stores one AABB per node. Consecutive Morton buckets
// are spatially coherent, so each node's box is tight; splits follow the Morton
// (spatial-median, round-robin axis) order of the keys.
#include "dev.h"

namespace {

// 16-lane row reductions on DPP (VALU, a few cycles each) instead of LDS-routed
// shuffles: quad_perm [1,0,3,2], quad_perm [2,3,0,1], row_ror:4, row_ror:8 — afterwards
// every lane of the row holds the row's min / max.
template <int CTRL>
__device__ __forceinline__ float dppf(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xf, 0xf, false));
}
__device__ __forceinline__ float min16(float v) {
  v = fminf(v, dppf<0xB1>(v));
  v = fminf(v, dppf<0x4E>(v));
  v = fminf(v, dppf<0x124>(v));
  return fminf(v, dppf<0x128>(v));
}
__device__ __forceinline__ float max16(float v) {
  v = fmaxf(v, dppf<0xB1>(v));
  v = fmaxf(v, dppf<0x4E>(v));
  v = fmaxf(v, dppf<0x124>(v));
  return fmaxf(v, dppf<0x128>(v));
}
// bucket value from the four row values (lanes 0, 16, 32, 48), on the scalar side
__device__ __forceinline__ float rows_min(float v) {
  const float a = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 0));
  const float b = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 16));
  const float c = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 32));
  const float d = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 48));
  return fminf(fminf(a, b), fminf(c, d));
}
__device__ __forceinline__ float rows_max(float v) {
  const float a = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 0));
  const float b = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 16));
  const float c = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 32));
  const float d = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 48));
  return fmaxf(fmaxf(a, b), fmaxf(c, d));
}

// One wave per 64-point bucket: the leaf box and (optionally) the four 16-point
// quarter boxes used for per-row culling by the k-NN kernel.
__global__ __launch_bounds__(256) void leaf_kernel(const float *__restrict__ pts, int64_t n,
                                                   float *__restrict__ nodes,
                                                   float *__restrict__ qnodes, int depth,
                                                   int64_t nleaf_slots) {
  const int64_t leaf = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (leaf >= nleaf_slots) return;
  const int lane = lsk::lane_id();
  const int64_t i = leaf * lsk::kBucket + lane;
  const float inf = __builtin_inff();
  float lx = inf, ly = inf, lz = inf, hx = -inf, hy = -inf, hz = -inf;
  if (i < n) {
    lx = hx = pts[3 * i];
    ly = hy = pts[3 * i + 1];
    lz = hz = pts[3 * i + 2];
  }
  // quarter (16-lane row) boxes first, then the bucket box from them
  lx = min16(lx); ly = min16(ly); lz = min16(lz);
  hx = max16(hx); hy = max16(hy); hz = max16(hz);
  if (qnodes && (lane & 15) == 0) {
    float4 *qd = (float4 *)qnodes + 2 * (leaf * 4 + (lane >> 4));
    qd[0] = make_float4(lx, ly, lz, 0.f);
    qd[1] = make_float4(hx, hy, hz, 0.f);
  }
  lx = rows_min(lx); ly = rows_min(ly); lz = rows_min(lz);
  hx = rows_max(hx); hy = rows_max(hy); hz = rows_max(hz);
  if (lane == 0) {
    float4 *nd = (float4 *)nodes + 2 * (((int64_t)1 << depth) + leaf);
    nd[0] = make_float4(lx, ly, lz, 0.f);
    nd[1] = make_float4(hx, hy, hz, 0.f);
  }
}

__global__ __launch_bounds__(256) void levelup_kernel(float *__restrict__ nodes, int level,
                                                      int radii_only) {
  const int64_t cnt = (int64_t)1 << level;
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= cnt) return;
  const int64_t node = cnt + j;
  float4 *nd = (float4 *)nodes;
  const float4 al = nd[2 * (2 * node)], ah = nd[2 * (2 * node) + 1];
  const float4 bl = nd[2 * (2 * node + 1)], bh = nd[2 * (2 * node + 1) + 1];
  if (radii_only) {
    nd[2 * node].w = fmaxf(al.w, bl.w);
  } else {
    nd[2 * node] = make_float4(fminf(al.x, bl.x), fminf(al.y, bl.y), fminf(al.z, bl.z),
                               fmaxf(al.w, bl.w));
    nd[2 * node + 1] = make_float4(fmaxf(ah.x, bh.x), fmaxf(ah.y, bh.y), fmaxf(ah.z, bh.z), 0.f);
  }
}

__global__ __launch_bounds__(256) void leaf_radius_kernel(const float *__restrict__ d2,
                                                          int64_t n, float *__restrict__ nodes,
                                                          int depth, int64_t nleaf_slots) {
  const int64_t leaf = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (leaf >= nleaf_slots) return;
  const int64_t i = leaf * lsk::kBucket + lsk::lane_id();
  float r = i < n ? d2[i] : 0.f;
  // an unresolved (NaN) radius must widen the published halo bound, never vanish in
  // fmaxf: treat it as +inf (the exact backstop normally replaces every NaN first)
  r = r == r ? r : __builtin_inff();
  r = rows_max(max16(r));
  if (lsk::lane_id() == 0) nodes[8 * (((int64_t)1 << depth) + leaf) + 3] = r;
}

// A-priori upper bound of every leaf's k-th squared radius, before any k-NN runs (the
// overlapped halo exchange publishes it while the local k-NN is still running). The
// W = ceil(k/64) + 1 consecutive buckets around the leaf hold >= k points (the query
// itself included). For a window point p let m(p) = the farthest-corner distance from p
// to the leaf box: every query q of the leaf has |q - p| <= m(p), so the k-th smallest
// m(p) over the window bounds every query's k-th neighbour distance. One wave per leaf,
// W values per lane, k-th smallest by bisection on the float bits (ballot counts).
// Beyond kUbMaxW buckets (k > 448) the cheaper, looser farthest-corner pair of the leaf
// box and the window's union box is used. Padded by 2^-16 relative (far above the
// rounding of the canonical d2 the kernels compare). n < k: +inf (fewer than k local
// points: the local k-th is infinite).
constexpr int kUbMaxW = 8;

__global__ __launch_bounds__(256) void leaf_radius_ub_kernel(const float *__restrict__ pts, int64_t n, int k,
                                                             float *__restrict__ nodes, int depth,
                                                             int64_t nleaf_slots) {
  const int64_t leaf = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (leaf >= nleaf_slots) return;
  const int lane = lsk::lane_id();
  const int64_t nb = (n + lsk::kBucket - 1) / lsk::kBucket;
  const int64_t slots = (int64_t)1 << depth;
  const float4 *nd = (const float4 *)nodes;
  float r = 0.f;
  if (leaf < nb) {
    if (n < (int64_t)k) {
      r = __builtin_inff();
    } else {
      const int64_t W = min(nb, (int64_t)(k + lsk::kBucket - 1) / lsk::kBucket + 1);
      int64_t st = leaf - (W - 1) / 2;
      st = st < 0 ? 0 : (st > nb - W ? nb - W : st);
      const float4 lo = nd[2 * (slots + leaf)], hi = nd[2 * (slots + leaf) + 1];
      if (W <= kUbMaxW) {
        uint32_t v[kUbMaxW];
#pragma unroll
        for (int j = 0; j < kUbMaxW; j++) {
          const int64_t i = (st + j) * lsk::kBucket + lane;
          v[j] = 0xffffffffu;
          if (j < W && i < n) {
            const float px = pts[3 * i], py = pts[3 * i + 1], pz = pts[3 * i + 2];
            const float ex = fmaxf(px - lo.x, hi.x - px), ey = fmaxf(py - lo.y, hi.y - py),
                        ez = fmaxf(pz - lo.z, hi.z - pz);
            v[j] = __float_as_uint(lsk::dist2(ex, ey, ez));
          }
        }
        uint32_t sel = 0;  // largest value with count(v < sel) < k = the k-th smallest
        for (int b = 31; b >= 0; --b) {
          const uint32_t cand = sel | (1u << b);
          uint32_t c = 0;
#pragma unroll
          for (int j = 0; j < kUbMaxW; j++) c += (uint32_t)__popcll(__ballot(v[j] < cand));
          if (c < (uint32_t)k) sel = cand;
        }
        r = __uint_as_float(sel);
      } else {
        const float inf = __builtin_inff();
        float wlx = inf, wly = inf, wlz = inf, whx = -inf, why = -inf, whz = -inf;
        for (int64_t b = st; b < st + W; b++) {
          const float4 bl = nd[2 * (slots + b)], bh = nd[2 * (slots + b) + 1];
          wlx = fminf(wlx, bl.x); wly = fminf(wly, bl.y); wlz = fminf(wlz, bl.z);
          whx = fmaxf(whx, bh.x); why = fmaxf(why, bh.y); whz = fmaxf(whz, bh.z);
        }
        const float ex = fmaxf(whx - lo.x, hi.x - wlx), ey = fmaxf(why - lo.y, hi.y - wly),
                    ez = fmaxf(whz - lo.z, hi.z - wlz);
        r = lsk::dist2(ex, ey, ez);
      }
      r *= 1.f + 0x1p-16f;
    }
  }
  if (lane == 0) nodes[8 * (slots + leaf) + 3] = r;
}

}  // namespace

extern "C" int lsk_hip_tree_set_radii_ub(float *nodes, const float *sorted_pts, int64_t n, int k, void *stream) {
  hipStream_t s = (hipStream_t)stream;
  const int depth = lsk_hip_tree_depth(n);
  const int64_t slots = (int64_t)1 << depth;
  leaf_radius_ub_kernel<<<lsk_blocks(slots, 4), 256, 0, s>>>(sorted_pts, n, k, nodes, depth, slots);
  LSK_CHECK_LAUNCH("tree_leaf_radius_ub");
  for (int l = depth - 1; l >= 0; l--) {
    levelup_kernel<<<lsk_blocks((int64_t)1 << l, 256), 256, 0, s>>>(nodes, l, 1);
    LSK_CHECK_LAUNCH("tree_levelup_radius");
  }
  return 0;
}

extern "C" int lsk_hip_tree_depth(int64_t n) {
  int64_t nb = (n + lsk::kBucket - 1) / lsk::kBucket;
  int d = 0;
  while (((int64_t)1 << d) < nb) d++;
  return d;
}

extern "C" int64_t lsk_hip_tree_nodes(int64_t n) {
  return (int64_t)2 << lsk_hip_tree_depth(n);
}

extern "C" int lsk_hip_build_tree(const float *sorted_pts, int64_t n, float *nodes,
                                  float *qnodes, void *stream) {
  hipStream_t s = (hipStream_t)stream;
  const int depth = lsk_hip_tree_depth(n);
  const int64_t slots = (int64_t)1 << depth;
  leaf_kernel<<<lsk_blocks(slots, 4), 256, 0, s>>>(sorted_pts, n, nodes, qnodes, depth, slots);
  LSK_CHECK_LAUNCH("tree_leaf");
  for (int l = depth - 1; l >= 0; l--) {
    levelup_kernel<<<lsk_blocks((int64_t)1 << l, 256), 256, 0, s>>>(nodes, l, 0);
    LSK_CHECK_LAUNCH("tree_levelup");
  }
  return 0;
}

extern "C" int lsk_hip_tree_set_radii(float *nodes, int64_t n, const float *d2_sorted,
                                      void *stream) {
  hipStream_t s = (hipStream_t)stream;
  const int depth = lsk_hip_tree_depth(n);
  const int64_t slots = (int64_t)1 << depth;
  leaf_radius_kernel<<<lsk_blocks(slots, 4), 256, 0, s>>>(d2_sorted, n, nodes, depth, slots);
  LSK_CHECK_LAUNCH("tree_leaf_radius");
  for (int l = depth - 1; l >= 0; l--) {
    levelup_kernel<<<lsk_blocks((int64_t)1 << l, 256), 256, 0, s>>>(nodes, l, 1);
    LSK_CHECK_LAUNCH("tree_levelup_radius");
  }
  return 0;
}
