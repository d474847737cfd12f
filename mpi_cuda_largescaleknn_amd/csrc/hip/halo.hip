// Halo (boundary-candidate) selection kernels for the cross-rank exchange (gfx950).
//
// The reference ships whole shard trees between ranks — a ring of every tree
// (unorderedDataVariant.cu:178-196) or whole-tree pulls culled by rank-AABB distance
// against a single max-radius over all queries (prePartitionedDataVariant.cu:150-174,
// 315-345). cuBQL is declared for this but never used (CMakeLists.txt:47). Here each
// rank publishes the top levels of its bucket tree with per-node max k-NN radius, and
// every other rank tests its own points against that BVH: a point is sent to rank j
// only if it lies strictly inside the radius-inflated box of some node of rank j.
// Because box_dist2(p, box) <= dist2(p, q) for every q in the box (canonical monotone
// formula, common.h), the filter never drops a point that could change a result.
#include "dev.h"

namespace {

constexpr int kStack = 64;

// nodes: 8 floats per node (lo.xyz, r2, hi.xyz, pad); root = 1; leaves at `depth`.
__device__ __forceinline__ bool pub_need(const lsk::vec3f &p, const float *nd) {
  return lsk::box_dist2(p, {nd[0], nd[1], nd[2]}, {nd[4], nd[5], nd[6]}) < nd[3];
}

__global__ __launch_bounds__(256) void halo_mask_kernel(const float *__restrict__ pts, int64_t n,
                                                        const float *__restrict__ pub,
                                                        const int64_t *__restrict__ pub_off,
                                                        const int32_t *__restrict__ pub_depth,
                                                        int nranks, int self,
                                                        uint64_t *__restrict__ mask) {
  __shared__ uint32_t stack[4][kStack];
  const int wid = threadIdx.x >> 6, lane = lsk::lane_id();
  const int64_t i = ((int64_t)lsk::xcd_remap(blockIdx.x, gridDim.x) * 4 + wid) * 64 + lane;
  if (__ballot(i < n) == 0) return;
  const bool valid = i < n;
  const lsk::vec3f p = valid ? lsk::vec3f{pts[3 * i], pts[3 * i + 1], pts[3 * i + 2]}
                             : lsk::vec3f{__builtin_inff(), __builtin_inff(), __builtin_inff()};
  uint64_t m = 0;
  for (int j = 0; j < nranks; j++) {
    if (j == self) continue;
    const float *nodes = pub + pub_off[j];
    const uint32_t depth = (uint32_t)pub_depth[j];
    const uint32_t leaf0 = 1u << depth;
    bool hit = false;
    uint32_t sp = 0;
    if (lane == 0) stack[wid][0] = 1u;
    sp = 1;
    while (sp > 0) {
      sp--;
      const uint32_t node = lsk::uniform(stack[wid][sp]);
      const float *nd = nodes + 8 * (size_t)node;
      const bool need = valid && !hit && pub_need(p, nd);
      if (!__ballot(need)) continue;
      if (node >= leaf0) {
        hit = hit || need;
        if (__ballot(valid && !hit) == 0) break;  // every lane already routed to j
        continue;
      }
      if (sp + 2 > kStack) break;  // cannot happen for depth < 32
      if (lane == 0) {
        stack[wid][sp] = 2 * node + 1;
        stack[wid][sp + 1] = 2 * node;
      }
      sp += 2;
    }
    if (hit) m |= (1ull << j);
  }
  if (valid) mask[i] = m;
}

// One wave per local bucket: lanes are the bucket's queries with their current k-th
// squared radius (lo.w of the local leaf is the bucket max); the group is flagged when
// some halo leaf box is strictly closer than a lane's radius.
__global__ __launch_bounds__(256) void flag_groups_kernel(const float *__restrict__ qpts,
                                                          const float *__restrict__ qd2,
                                                          int64_t nq,
                                                          const float *__restrict__ hnodes,
                                                          int32_t hdepth, int64_t nhalo,
                                                          uint32_t *__restrict__ flags) {
  __shared__ uint32_t stack[4][kStack];
  const int wid = threadIdx.x >> 6, lane = lsk::lane_id();
  const int64_t g = (int64_t)blockIdx.x * 4 + wid;
  const int64_t ngroups = (nq + 63) / 64;
  if (g >= ngroups) return;
  const int64_t qi = g * 64 + lane;
  const bool valid = qi < nq;
  const lsk::vec3f q = valid ? lsk::vec3f{qpts[3 * qi], qpts[3 * qi + 1], qpts[3 * qi + 2]}
                             : lsk::vec3f{0.f, 0.f, 0.f};
  const float r2 = valid ? qd2[qi] : 0.f;
  lsk::cfloat4_p nodes = lsk::as_const4(hnodes);
  const uint32_t leaf0 = 1u << hdepth;
  bool flagged = false;
  if (nhalo > 0) {
    uint32_t sp = 0;
    if (lane == 0) stack[wid][0] = 1u;
    sp = 1;
    while (sp > 0) {
      sp--;
      const uint32_t node = lsk::uniform(stack[wid][sp]);
      const lsk::v4f lo = nodes[2 * node], hi = nodes[2 * node + 1];
      const bool need = lsk::box_dist2(q, {lo.x, lo.y, lo.z}, {hi.x, hi.y, hi.z}) < r2;
      if (!__ballot(need)) continue;
      if (node >= leaf0) {
        flagged = true;
        break;
      }
      if (lane == 0) {
        stack[wid][sp] = 2 * node + 1;
        stack[wid][sp + 1] = 2 * node;
      }
      sp += 2;
    }
  }
  if (lane == 0) flags[g] = flagged ? 1u : 0u;
}

// Inverse flagging: one lane per halo point walks the LOCAL tree, whose node boxes carry
// the max k-th squared radius of their queries (lo.w, set by tree_set_radii), and marks
// every bucket (= query group) whose radius-inflated box contains the point. A group can
// only change if some halo point lies within some query's radius, and box_dist2 <=
// dist2 for every query of the bucket, so the flags are a superset of what must be
// re-queried. Unlike testing groups against the halo tree, the outcome does not depend
// on the halo tree's boxes (halo points form thin slabs, whose Morton buckets often span
// Z-order jumps and have huge boxes).
__global__ __launch_bounds__(256) void flag_groups_inverse_kernel(const float *__restrict__ hpts,
                                                                  int64_t nh,
                                                                  const float *__restrict__ lnodes,
                                                                  int32_t depth, int64_t ngroups,
                                                                  uint32_t *__restrict__ flags) {
  __shared__ uint32_t stack[4][kStack];
  const int wid = threadIdx.x >> 6, lane = lsk::lane_id();
  const int64_t i = ((int64_t)lsk::xcd_remap(blockIdx.x, gridDim.x) * 4 + wid) * 64 + lane;
  if (__ballot(i < nh) == 0) return;
  const bool valid = i < nh;
  const lsk::vec3f p = valid ? lsk::vec3f{hpts[3 * i], hpts[3 * i + 1], hpts[3 * i + 2]}
                             : lsk::vec3f{__builtin_inff(), __builtin_inff(), __builtin_inff()};
  const uint32_t leaf0 = 1u << depth;
  uint32_t sp = 0;
  if (lane == 0) stack[wid][0] = 1u;
  sp = 1;
  while (sp > 0) {
    sp--;
    const uint32_t node = lsk::uniform(stack[wid][sp]);
    const float *nd = lnodes + 8 * (size_t)node;
    const bool need = valid && pub_need(p, nd);
    if (!__ballot(need)) continue;
    if (node >= leaf0) {
      const int64_t b = (int64_t)(node - leaf0);
      if (need && b < ngroups) flags[b] = 1u;
      continue;
    }
    if (sp + 2 > kStack) break;  // cannot happen for depth < 32
    if (lane == 0) {
      stack[wid][sp] = 2 * node + 1;
      stack[wid][sp + 1] = 2 * node;
    }
    sp += 2;
  }
}

// gap² between two node boxes (8 floats each: lo.xyz, -, hi.xyz, -). For q in box a and
// p in box b every axis gap is at most |q - p| on that axis after rounding (float
// subtraction is monotone), so with the canonical dist2 the result is <= dist2(q, p).
__device__ __forceinline__ float box_box_gap2(const float *a, const float *b) {
  const float gx = fmaxf(0.f, fmaxf(a[0] - b[4], b[0] - a[4]));
  const float gy = fmaxf(0.f, fmaxf(a[1] - b[5], b[1] - a[5]));
  const float gz = fmaxf(0.f, fmaxf(a[2] - b[6], b[2] - a[6]));
  return lsk::dist2(gx, gy, gz);
}

// One lane per local bucket (query group): its leaf box and squared radius bound (lo.w)
// against every other rank's published tree, wave-uniform DFS as halo_mask_kernel.
__global__ __launch_bounds__(256) void boundary_groups_kernel(const float *__restrict__ lnodes, int32_t depth,
                                                              int64_t ngroups, const float *__restrict__ pub,
                                                              const int64_t *__restrict__ pub_off,
                                                              const int32_t *__restrict__ pub_depth, int nranks,
                                                              int self, uint32_t *__restrict__ flags) {
  __shared__ uint32_t stack[4][kStack];
  const int wid = threadIdx.x >> 6, lane = lsk::lane_id();
  const int64_t g = ((int64_t)lsk::xcd_remap(blockIdx.x, gridDim.x) * 4 + wid) * 64 + lane;
  if (__ballot(g < ngroups) == 0) return;
  const bool valid = g < ngroups;
  float box[8];
  const float *lf = lnodes + 8 * (size_t)(((int64_t)1 << depth) + (valid ? g : 0));
#pragma unroll
  for (int t = 0; t < 8; t++) box[t] = lf[t];
  const float r2 = valid ? box[3] : 0.f;
  bool hit = false;
  for (int j = 0; j < nranks; j++) {
    if (j == self) continue;
    const float *nodes = pub + pub_off[j];
    const uint32_t leaf0 = 1u << (uint32_t)pub_depth[j];
    uint32_t sp = 0;
    if (lane == 0) stack[wid][0] = 1u;
    sp = 1;
    while (sp > 0) {
      sp--;
      const uint32_t node = lsk::uniform(stack[wid][sp]);
      const float *nd = nodes + 8 * (size_t)node;
      const bool need = valid && !hit && box_box_gap2(box, nd) < r2;
      if (!__ballot(need)) continue;
      if (node >= leaf0) {
        hit = hit || need;
        if (__ballot(valid && !hit) == 0) break;
        continue;
      }
      if (sp + 2 > kStack) break;  // cannot happen for depth < 32
      if (lane == 0) {
        stack[wid][sp] = 2 * node + 1;
        stack[wid][sp + 1] = 2 * node;
      }
      sp += 2;
    }
    if (__ballot(valid && !hit) == 0) break;
  }
  if (valid) flags[g] = hit ? 1u : 0u;
}

__global__ __launch_bounds__(256) void compact_kernel(const uint32_t *__restrict__ flags,
                                                      int64_t n, uint32_t *__restrict__ list,
                                                      uint32_t *__restrict__ count) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool on = i < n && flags[i] != 0u;
  const uint64_t b = __ballot(on);
  if (b == 0) return;
  const int lane = lsk::lane_id();
  uint32_t base = 0;
  if (lane == 0) base = atomicAdd(count, (uint32_t)__popcll(b));
  base = __shfl(base, 0);
  if (on) list[base + __popcll(b & ((1ull << lane) - 1ull))] = (uint32_t)i;
}

__global__ __launch_bounds__(256) void mask_counts_kernel(const uint64_t *__restrict__ mask,
                                                          int64_t n, int nranks,
                                                          uint32_t *__restrict__ counts) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t m = i < n ? mask[i] : 0ull;
  for (int j = 0; j < nranks; j++) {
    const uint64_t b = __ballot((m >> j) & 1ull);
    if (b && lsk::lane_id() == 0) atomicAdd(&counts[j], (uint32_t)__popcll(b));
  }
}

__global__ __launch_bounds__(256) void halo_pack_kernel(const float *__restrict__ pts,
                                                        const uint64_t *__restrict__ mask,
                                                        int64_t n, int nranks,
                                                        const int64_t *__restrict__ offsets,
                                                        uint32_t *__restrict__ cursors,
                                                        float *__restrict__ send) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int lane = lsk::lane_id();
  const uint64_t m = i < n ? mask[i] : 0ull;
  if (__ballot(m != 0ull) == 0) return;
  float x = 0.f, y = 0.f, z = 0.f;
  if (m) {
    x = pts[3 * i];
    y = pts[3 * i + 1];
    z = pts[3 * i + 2];
  }
  for (int j = 0; j < nranks; j++) {
    const bool on = (m >> j) & 1ull;
    const uint64_t b = __ballot(on);
    if (!b) continue;
    uint32_t base = 0;
    if (lane == 0) base = atomicAdd(&cursors[j], (uint32_t)__popcll(b));
    base = __shfl(base, 0);
    if (on) {
      const int64_t pos = offsets[j] + base + __popcll(b & ((1ull << lane) - 1ull));
      send[3 * pos] = x;
      send[3 * pos + 1] = y;
      send[3 * pos + 2] = z;
    }
  }
}

}  // namespace

extern "C" int lsk_hip_halo_mask(const float *pts, int64_t n, const float *pub,
                                 const int64_t *pub_off, const int32_t *pub_depth, int nranks,
                                 int self, uint64_t *mask, void *stream) {
  if (n <= 0) return 0;
  if (nranks > 64) {
    lsk::set_last_error("halo_mask: at most 64 ranks");
    return 1;
  }
  halo_mask_kernel<<<lsk_blocks(n, 256), 256, 0, (hipStream_t)stream>>>(pts, n, pub, pub_off,
                                                                      pub_depth, nranks, self,
                                                                      mask);
  LSK_CHECK_LAUNCH("halo_mask");
  return 0;
}

extern "C" int lsk_hip_boundary_groups(const float *local_nodes, int32_t depth, int64_t ngroups, const float *pub,
                                       const int64_t *pub_off, const int32_t *pub_depth, int nranks, int self,
                                       uint32_t *flags, void *stream) {
  if (ngroups <= 0) return 0;
  if (nranks > 64 || depth < 0 || depth > 30) {
    lsk::set_last_error("boundary_groups: at most 64 ranks, tree depth in [0, 30]");
    return 1;
  }
  boundary_groups_kernel<<<lsk_blocks(ngroups, 256), 256, 0, (hipStream_t)stream>>>(
      local_nodes, depth, ngroups, pub, pub_off, pub_depth, nranks, self, flags);
  LSK_CHECK_LAUNCH("boundary_groups");
  return 0;
}

extern "C" int lsk_hip_flag_query_groups(const float *qpts, const float *qd2, int64_t nq,
                                         const float *halo_nodes, int32_t halo_depth,
                                         int64_t nhalo, uint32_t *flags, void *stream) {
  if (nq <= 0) return 0;
  const int64_t ng = (nq + 63) / 64;
  flag_groups_kernel<<<lsk_blocks(ng, 4), 256, 0, (hipStream_t)stream>>>(
      qpts, qd2, nq, halo_nodes, halo_depth, nhalo, flags);
  LSK_CHECK_LAUNCH("flag_groups");
  return 0;
}

extern "C" int lsk_hip_flag_groups_inverse(const float *halo_pts, int64_t nh,
                                           const float *local_nodes, int32_t depth,
                                           int64_t ngroups, uint32_t *flags, void *stream) {
  if (nh <= 0 || ngroups <= 0) return 0;
  if (depth < 0 || depth > 30) {
    lsk::set_last_error("flag_groups_inverse: bad tree depth");
    return 1;
  }
  flag_groups_inverse_kernel<<<lsk_blocks(nh, 256), 256, 0, (hipStream_t)stream>>>(
      halo_pts, nh, local_nodes, depth, ngroups, flags);
  LSK_CHECK_LAUNCH("flag_groups_inverse");
  return 0;
}

extern "C" int lsk_hip_compact_flags(const uint32_t *flags, int64_t n, uint32_t *list,
                                     uint32_t *count, void *stream) {
  if (n <= 0) return 0;
  compact_kernel<<<lsk_blocks(n, 256), 256, 0, (hipStream_t)stream>>>(flags, n, list, count);
  LSK_CHECK_LAUNCH("compact_flags");
  return 0;
}

extern "C" int lsk_hip_mask_counts(const uint64_t *mask, int64_t n, int nranks,
                                   uint32_t *counts, void *stream) {
  if (n <= 0) return 0;
  mask_counts_kernel<<<lsk_blocks(n, 256), 256, 0, (hipStream_t)stream>>>(mask, n, nranks,
                                                                        counts);
  LSK_CHECK_LAUNCH("mask_counts");
  return 0;
}

extern "C" int lsk_hip_halo_pack(const float *pts, const uint64_t *mask, int64_t n, int nranks,
                                 const int64_t *offsets, uint32_t *cursors, float *send,
                                 void *stream) {
  if (n <= 0) return 0;
  halo_pack_kernel<<<lsk_blocks(n, 256), 256, 0, (hipStream_t)stream>>>(pts, mask, n, nranks,
                                                                      offsets, cursors, send);
  LSK_CHECK_LAUNCH("halo_pack");
  return 0;
}
