// "ref-algo": the reference's algorithm re-implemented on gfx950 (baseline + fidelity
// modes), 64-bit safe. SURVEY §6.3 / §2.2 E01-E03, [inferred] cudaKDTree semantics:
//
//  * left-balanced, object-median, round-robin-axis implicit k-d tree built in place
//    (cukd::buildTree, unorderedDataVariant.cu:161): node i has children 2i+1, 2i+2 and
//    the float3 array *is* the tree. Built with Wald's tag-update scheme: per level, sort
//    by (tag, coord[level%3]) (two stable passes of our radix sort) and retag each point
//    by its rank in its subtree's segment; segment starts are closed-form.
//  * stack-free traversal (cukd::stackFree::knn, U:86): (prev, curr) state machine, no
//    stack, revisits parents;
//  * FlexHeapCandidateList (U:84-85, U:97): a k-entry max-heap per query in GLOBAL memory,
//    AoS [query][k] of uint64 (d2 bits << 32 | point id), initialised with (cutoff², -1)
//    on round 0 and resumed on later rounds — indexed with 64-bit offsets here (the
//    reference's int k*tid overflows past 21.4M points per rank at k=100).
//  * runQuery's radius reduction (prePartitionedDataVariant.cu:91-94): max over queries of
//    sqrt(heap top), one float atomicMax per wave instead of one contended per thread.
#include "dev.h"

namespace {

// cukd's float3 is 12 B; tree[i] is point i of the left-balanced order.
__device__ __forceinline__ uint32_t ordered_bits(float f) {
  const uint32_t u = lsk::fbits(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);  // total order for finite floats
}

// Number of nodes in the subtree rooted at t of the left-balanced tree with n nodes.
__device__ __forceinline__ int64_t subtree_size(int64_t t, int64_t n) {
  int64_t size = 0, first = t, last = t;
  while (first < n) {
    size += (last < n ? last : n - 1) - first + 1;
    first = 2 * first + 1;
    last = 2 * last + 2;
  }
  return size;
}

__global__ __launch_bounds__(256) void lbt_keys_kernel(const float *__restrict__ pts, int64_t n,
                                                       int dim, uint32_t *__restrict__ keys,
                                                       uint32_t *__restrict__ vals) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    keys[i] = ordered_bits(pts[3 * i + dim]);
    vals[i] = (uint32_t)i;
  }
}

// Points are sorted by (tag, coord[level%3]); tags of level `level` are active.
__global__ __launch_bounds__(256) void lbt_retag_kernel(uint32_t *__restrict__ tags, int64_t n,
                                                        int level) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t lvl_first = ((int64_t)1 << level) - 1;   // first node id of this level
  const int64_t done = lvl_first < n ? lvl_first : n;      // nodes fixed on earlier levels
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const int64_t t = tags[i];
    if (t < lvl_first) continue;  // already a fixed node
    // start of t's segment: all fixed nodes, then the subtrees of level nodes left of t
    int64_t start = done;
    const int64_t left_nodes = t - lvl_first;
    if (left_nodes > 0) {
      int64_t f = lvl_first;
      for (int l = level;; l++) {
        const int64_t avail = n - f;
        if (avail <= 0) break;
        const int64_t want = left_nodes << (l - level);
        start += want < avail ? want : avail;
        f = 2 * f + 1;
      }
    }
    const int64_t pos = i - start;
    const int64_t lsize = subtree_size(2 * t + 1, n);
    tags[i] = (uint32_t)(pos < lsize ? 2 * t + 1 : (pos == lsize ? t : 2 * t + 2));
  }
}

__global__ __launch_bounds__(256) void gather_u32_kernel(const uint32_t *__restrict__ src,
                                                         const uint32_t *__restrict__ idx,
                                                         int64_t n, uint32_t *__restrict__ dst) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    dst[i] = src[idx[i]];
}

// ---------------------------------------------------------------------------------- query
struct FlexHeap {
  unsigned long long *h;  // k entries in global memory (AoS row of this query)
  int k;
  __device__ float max_radius2() const { return lsk::bitsf((uint32_t)(h[0] >> 32)); }
  __device__ void push(float d2, uint32_t id) {
    const unsigned long long v = ((unsigned long long)lsk::fbits(d2) << 32) | id;
    if (!(v < h[0])) return;
    int i = 0;
    for (;;) {
      const int l = 2 * i + 1, r = l + 1;
      int c = i;
      unsigned long long cv = v;
      if (l < k && h[l] > cv) { c = l; cv = h[l]; }
      if (r < k && h[r] > cv) { c = r; cv = h[r]; }
      if (c == i) break;
      h[i] = cv;
      i = c;
    }
    h[i] = v;
  }
};

__global__ __launch_bounds__(256) void refalgo_knn_kernel(
    const float *__restrict__ tree, int64_t n, const float *__restrict__ qpts, int64_t nq,
    unsigned long long *__restrict__ heaps, int k, float cut2, int init, float *__restrict__ rmax,
    uint32_t id_base) {
  const int64_t qi = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  float r = 0.f;
  if (qi < nq) {
    FlexHeap cl{heaps + qi * (int64_t)k, k};
    if (init) {
      const unsigned long long e = ((unsigned long long)lsk::fbits(cut2) << 32) | 0xffffffffull;
      for (int i = 0; i < k; i++) cl.h[i] = e;
    }
    const float qx = qpts[3 * qi], qy = qpts[3 * qi + 1], qz = qpts[3 * qi + 2];
    // stack-free traversal of the left-balanced tree
    int64_t prev = -1, curr = 0;
    if (n > 0) {
      for (;;) {
        const int64_t parent = (curr + 1) / 2 - 1;
        if (curr >= n) {  // non-existent child: go back up
          prev = curr;
          curr = parent;
          continue;
        }
        const bool from_parent = prev < curr;
        const float px = tree[3 * curr], py = tree[3 * curr + 1], pz = tree[3 * curr + 2];
        if (from_parent) {
          const float d2 = lsk::dist2(qx - px, qy - py, qz - pz);
          if (d2 < cl.max_radius2()) cl.push(d2, id_base + (uint32_t)curr);
        }
        const int level = 63 - __clzll((unsigned long long)(curr + 1));
        const int dim = level % 3;
        const float split = dim == 0 ? px : (dim == 1 ? py : pz);
        const float qd = dim == 0 ? qx : (dim == 1 ? qy : qz);
        const float diff = qd - split;
        const int side = diff >= 0.f ? 1 : 0;
        const int64_t close = 2 * curr + 1 + side, far = 2 * curr + 2 - side;
        int64_t next;
        if (from_parent) {
          next = close;
        } else if (prev == close) {
          next = (diff * diff < cl.max_radius2()) ? far : parent;
        } else {
          next = parent;
        }
        if (next == -1) break;
        prev = curr;
        curr = next;
      }
    }
    const float top = cl.max_radius2();
    r = isinf(top) ? top : sqrtf(top);
  }
  if (rmax) {
    r = lsk::wave_max(r);
    if (lsk::lane_id() == 0 && r > 0.f) {
      // float max on non-negative values == unsigned max on their bits
      atomicMax((unsigned int *)rmax, lsk::fbits(r));
    }
  }
}

__global__ __launch_bounds__(256) void refalgo_extract_kernel(const unsigned long long *__restrict__ heaps,
                                                              int64_t nq, int k,
                                                              float *__restrict__ out) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t qi = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; qi < nq; qi += stride) {
    const float d2 = lsk::bitsf((uint32_t)(heaps[qi * (int64_t)k] >> 32));
    out[qi] = lsk::final_distance(d2);
  }
}

}  // namespace

extern "C" int lsk_hip_lbt_keys(const float *pts, int64_t n, int dim, uint32_t *keys,
                                uint32_t *vals, void *stream) {
  if (n <= 0) return 0;
  lbt_keys_kernel<<<lsk_blocks(n, 1024, 8192), 256, 0, (hipStream_t)stream>>>(pts, n, dim, keys,
                                                                            vals);
  LSK_CHECK_LAUNCH("lbt_keys");
  return 0;
}

extern "C" int lsk_hip_lbt_retag(uint32_t *tags, int64_t n, int level, void *stream) {
  if (n <= 0) return 0;
  lbt_retag_kernel<<<lsk_blocks(n, 1024, 8192), 256, 0, (hipStream_t)stream>>>(tags, n, level);
  LSK_CHECK_LAUNCH("lbt_retag");
  return 0;
}

extern "C" int lsk_hip_gather_u32(const uint32_t *src, const uint32_t *idx, int64_t n,
                                  uint32_t *dst, void *stream) {
  if (n <= 0) return 0;
  gather_u32_kernel<<<lsk_blocks(n, 1024, 8192), 256, 0, (hipStream_t)stream>>>(src, idx, n, dst);
  LSK_CHECK_LAUNCH("gather_u32");
  return 0;
}

extern "C" int lsk_hip_refalgo_knn(const float *tree, int64_t n, const float *qpts, int64_t nq,
                                   unsigned long long *heaps, int k, float cut2, int init,
                                   float *rmax, uint32_t id_base, void *stream) {
  if (nq <= 0) return 0;
  if (n >= ((int64_t)1 << 32)) {
    lsk::set_last_error("refalgo_knn: tree must have < 2^32 points");
    return 1;
  }
  const int64_t nb = (nq + 255) / 256;
  refalgo_knn_kernel<<<(unsigned)nb, 256, 0, (hipStream_t)stream>>>(tree, n, qpts, nq, heaps, k,
                                                                   cut2, init, rmax, id_base);
  LSK_CHECK_LAUNCH("refalgo_knn");
  return 0;
}

extern "C" int lsk_hip_refalgo_extract(const unsigned long long *heaps, int64_t nq, int k,
                                       float *out, void *stream) {
  if (nq <= 0) return 0;
  refalgo_extract_kernel<<<lsk_blocks(nq, 1024, 8192), 256, 0, (hipStream_t)stream>>>(heaps, nq, k,
                                                                                    out);
  LSK_CHECK_LAUNCH("refalgo_extract");
  return 0;
}
