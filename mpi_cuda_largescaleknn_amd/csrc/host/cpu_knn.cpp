// CPU exact k-th-distance oracle + CPU backend ops (bounds, Morton, halo mask).
//
// The oracle defines the result the GPU must reproduce bit-for-bit:
// out[q] = k-th smallest of { dist2(q,p) < cut2 } ∪ { cut2 × k }, which is exactly what
// the reference's FlexHeapCandidateList (initialised with cutOff², strict '<' push;
// unorderedDataVariant.cu:84-86, 97-98) leaves on top of its heap.
#include "lsk_host.h"
#include "../common.h"

#include <algorithm>
#include <array>
#include <mutex>
#include <atomic>
#include <cmath>
#include <limits>
#include <thread>
#include <vector>

using lsk::vec3f;

namespace {

template <typename F>
void parallel_for(int64_t n, int nthreads, F &&fn) {
  if (n <= 0) return;
  if (nthreads < 1) nthreads = 1;
  int64_t nt = std::min<int64_t>(nthreads, n);
  if (nt == 1) {
    fn(0, n);
    return;
  }
  // Dynamic chunking: query costs vary a lot with local density.
  std::atomic<int64_t> next{0};
  const int64_t chunk = std::max<int64_t>(1, std::min<int64_t>(4096, n / (nt * 16) + 1));
  std::vector<std::thread> th;
  for (int64_t t = 0; t < nt; t++) {
    th.emplace_back([&] {
      for (;;) {
        int64_t b = next.fetch_add(chunk);
        if (b >= n) break;
        fn(b, std::min(n, b + chunk));
      }
    });
  }
  for (auto &x : th) x.join();
}

// k-max-heap over squared distances, initialised with k copies of cut2.
struct KHeap {
  std::vector<float> h;
  void reset(int k, float cut2) { h.assign((size_t)k, cut2); }
  float top() const { return h[0]; }
  void push(float v) {  // precondition: v < top()
    const int n = (int)h.size();
    int i = 0;
    for (;;) {
      int l = 2 * i + 1, r = l + 1, c = i;
      float cv = v;
      if (l < n && h[l] > cv) { c = l; cv = h[l]; }
      if (r < n && h[r] > cv) { c = r; cv = h[r]; }
      if (c == i) break;
      h[i] = h[c];
      i = c;
    }
    h[i] = v;
  }
};

struct KdNode {
  float lo[3], hi[3];
  int64_t begin, end;   // point range (leaf) or children
  int64_t left, right;  // -1 for leaf
};

struct KdTree {
  std::vector<vec3f> pts;
  std::vector<KdNode> nodes;
  static constexpr int kLeaf = 16;

  int64_t build(int64_t b, int64_t e) {
    KdNode nd;
    for (int a = 0; a < 3; a++) {
      nd.lo[a] = std::numeric_limits<float>::infinity();
      nd.hi[a] = -std::numeric_limits<float>::infinity();
    }
    for (int64_t i = b; i < e; i++) {
      const float c[3] = {pts[i].x, pts[i].y, pts[i].z};
      for (int a = 0; a < 3; a++) {
        nd.lo[a] = std::min(nd.lo[a], c[a]);
        nd.hi[a] = std::max(nd.hi[a], c[a]);
      }
    }
    nd.begin = b;
    nd.end = e;
    nd.left = nd.right = -1;
    int64_t id = (int64_t)nodes.size();
    nodes.push_back(nd);
    if (e - b > kLeaf) {
      int axis = 0;
      float w = nd.hi[0] - nd.lo[0];
      for (int a = 1; a < 3; a++)
        if (nd.hi[a] - nd.lo[a] > w) { w = nd.hi[a] - nd.lo[a]; axis = a; }
      int64_t m = (b + e) / 2;
      std::nth_element(pts.begin() + b, pts.begin() + m, pts.begin() + e,
                       [axis](const vec3f &p, const vec3f &q) {
                         return (&p.x)[axis] < (&q.x)[axis];
                       });
      int64_t l = build(b, m);
      int64_t r = build(m, e);
      nodes[id].left = l;
      nodes[id].right = r;
    }
    return id;
  }

  float node_dist2(const KdNode &n, const vec3f &q) const {
    return lsk::box_dist2(q, vec3f{n.lo[0], n.lo[1], n.lo[2]}, vec3f{n.hi[0], n.hi[1], n.hi[2]});
  }

  float query(const vec3f &q, int k, float cut2, KHeap &heap,
              std::vector<std::pair<int64_t, float>> &stack) const {
    heap.reset(k, cut2);
    if (nodes.empty()) return heap.top();
    stack.clear();
    stack.push_back({0, node_dist2(nodes[0], q)});
    while (!stack.empty()) {
      auto [ni, bd] = stack.back();
      stack.pop_back();
      if (!(bd < heap.top())) continue;
      const KdNode &n = nodes[ni];
      if (n.left < 0) {
        for (int64_t i = n.begin; i < n.end; i++) {
          float d2 = lsk::dist2(q, pts[i]);
          if (d2 < heap.top()) heap.push(d2);
        }
        continue;
      }
      float dl = node_dist2(nodes[n.left], q), dr = node_dist2(nodes[n.right], q);
      if (dl <= dr) {
        stack.push_back({n.right, dr});
        stack.push_back({n.left, dl});
      } else {
        stack.push_back({n.left, dl});
        stack.push_back({n.right, dr});
      }
    }
    return heap.top();
  }
};

}  // namespace

extern "C" void lsk_cpu_kth_brute(const float *pts, int64_t n, const float *qry, int64_t nq,
                                  int k, float cut2, float *out_d2, int nthreads) {
  const vec3f *P = (const vec3f *)pts;
  const vec3f *Q = (const vec3f *)qry;
  parallel_for(nq, nthreads, [&](int64_t b, int64_t e) {
    std::vector<float> d;
    d.reserve((size_t)n);
    for (int64_t qi = b; qi < e; qi++) {
      d.clear();
      for (int64_t i = 0; i < n; i++) {
        float v = lsk::dist2(Q[qi], P[i]);
        if (v < cut2) d.push_back(v);
      }
      if ((int64_t)d.size() < k) {
        out_d2[qi] = cut2;
      } else {
        std::nth_element(d.begin(), d.begin() + (k - 1), d.end());
        out_d2[qi] = d[(size_t)k - 1];
      }
    }
  });
}

extern "C" void lsk_cpu_count_below(const float *pts, int64_t n, const float *qry,
                                    const float *thr, int nq, unsigned long long *counts,
                                    int nthreads) {
  const vec3f *P = (const vec3f *)pts;
  const vec3f *Q = (const vec3f *)qry;
  parallel_for(nq, nthreads, [&](int64_t b, int64_t e) {
    for (int64_t j = b; j < e; j++) {
      unsigned long long lt = 0, le = 0;
      for (int64_t i = 0; i < n; i++) {
        const float v = lsk::dist2(Q[j], P[i]);
        lt += v < thr[2 * j];
        le += v < thr[2 * j + 1];
      }
      counts[2 * j] += lt;
      counts[2 * j + 1] += le;
    }
  });
}

extern "C" void lsk_cpu_kth_kdtree(const float *pts, int64_t n, const float *qry, int64_t nq,
                                   int k, float cut2, float *out_d2, int nthreads) {
  KdTree t;
  t.pts.assign((const vec3f *)pts, (const vec3f *)pts + n);
  if (n > 0) t.nodes.reserve((size_t)(2 * n / KdTree::kLeaf + 16)), t.build(0, n);
  const vec3f *Q = (const vec3f *)qry;
  parallel_for(nq, nthreads, [&](int64_t b, int64_t e) {
    KHeap heap;
    std::vector<std::pair<int64_t, float>> stack;
    for (int64_t qi = b; qi < e; qi++) out_d2[qi] = t.query(Q[qi], k, cut2, heap, stack);
  });
}

extern "C" void lsk_cpu_bounds(const float *pts, int64_t n, float *box, int nthreads) {
  const float inf = std::numeric_limits<float>::infinity();
  float lo[3] = {inf, inf, inf}, hi[3] = {-inf, -inf, -inf};
  std::vector<std::array<float, 6>> part;
  std::mutex mu;
  parallel_for(n, nthreads, [&](int64_t b, int64_t e) {
    float l[3] = {inf, inf, inf}, h[3] = {-inf, -inf, -inf};
    for (int64_t i = b; i < e; i++)
      for (int a = 0; a < 3; a++) {
        l[a] = std::min(l[a], pts[3 * i + a]);
        h[a] = std::max(h[a], pts[3 * i + a]);
      }
    std::lock_guard<std::mutex> g(mu);
    for (int a = 0; a < 3; a++) {
      lo[a] = std::min(lo[a], l[a]);
      hi[a] = std::max(hi[a], h[a]);
    }
  });
  for (int a = 0; a < 3; a++) {
    box[a] = lo[a];
    box[3 + a] = hi[a];
  }
}

extern "C" void lsk_cpu_morton(const float *pts, int64_t n, const float *origin, float scale,
                               uint32_t *keys, int curve, int nthreads) {
  parallel_for(n, nthreads, [&](int64_t b, int64_t e) {
    for (int64_t i = b; i < e; i++) {
      uint32_t ix = lsk::morton_quant(pts[3 * i + 0], origin[0], scale);
      uint32_t iy = lsk::morton_quant(pts[3 * i + 1], origin[1], scale);
      uint32_t iz = lsk::morton_quant(pts[3 * i + 2], origin[2], scale);
      keys[i] = lsk::curve3(curve, ix, iy, iz);
    }
  });
}

extern "C" void lsk_cpu_halo_mask(const float *pts, int64_t n, const float *boxes,
                                  const int64_t *box_offsets, int nsets, int skip_set,
                                  uint64_t *mask, int nthreads) {
  parallel_for(n, nthreads, [&](int64_t b, int64_t e) {
    for (int64_t i = b; i < e; i++) {
      vec3f p{pts[3 * i], pts[3 * i + 1], pts[3 * i + 2]};
      uint64_t m = 0;
      for (int s = 0; s < nsets && s < 64; s++) {
        if (s == skip_set) continue;
        for (int64_t j = box_offsets[s]; j < box_offsets[s + 1]; j++) {
          const float *bx = boxes + 8 * j;
          float d2 = lsk::box_dist2(p, vec3f{bx[0], bx[1], bx[2]}, vec3f{bx[4], bx[5], bx[6]});
          if (d2 < bx[3]) {
            m |= (1ull << s);
            break;
          }
        }
      }
      mask[i] = m;
    }
  });
}
