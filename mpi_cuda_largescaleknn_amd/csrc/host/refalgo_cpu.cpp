// CPU twin of csrc/hip/refalgo.hip ("ref-algo" baseline: left-balanced k-d tree,
// stack-free traversal, persisted global k-max-heaps). Used by the CPU/gloo tests of the
// reference-faithful ring and peer schedules and by `--device cpu --mode ring|peer`.
#include "lsk_host.h"
#include "../common.h"

#include <algorithm>
#include <atomic>
#include <cmath>
#include <thread>
#include <vector>

using lsk::vec3f;

namespace {

int64_t subtree_size(int64_t t, int64_t n) {
  int64_t size = 0, first = t, last = t;
  while (first < n) {
    size += std::min(last, n - 1) - first + 1;
    first = 2 * first + 1;
    last = 2 * last + 2;
  }
  return size;
}

struct Item {
  vec3f p;
  uint32_t id;
};

// Place the items of subtree t (already gathered in [b, e)) into out[] recursively.
void build_rec(std::vector<Item> &v, int64_t b, int64_t e, int64_t t, int level, int64_t n,
               std::vector<Item> &out) {
  if (b >= e) return;
  const int dim = level % 3;
  const int64_t lsize = subtree_size(2 * t + 1, n);
  std::nth_element(v.begin() + b, v.begin() + b + lsize, v.begin() + e,
                   [dim](const Item &x, const Item &y) { return (&x.p.x)[dim] < (&y.p.x)[dim]; });
  out[(size_t)t] = v[(size_t)(b + lsize)];
  build_rec(v, b, b + lsize, 2 * t + 1, level + 1, n, out);
  build_rec(v, b + lsize + 1, e, 2 * t + 2, level + 1, n, out);
}

struct Heap {
  unsigned long long *h;
  int k;
  float top() const { return lsk::bitsf((uint32_t)(h[0] >> 32)); }
  void push(float d2, uint32_t id) {
    const unsigned long long v = ((unsigned long long)lsk::fbits(d2) << 32) | id;
    if (!(v < h[0])) return;
    int i = 0;
    for (;;) {
      int l = 2 * i + 1, r = l + 1, c = i;
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

}  // namespace

extern "C" void lsk_cpu_lbt_build(const float *pts, int64_t n, float *out_pts, uint32_t *out_ids) {
  std::vector<Item> v((size_t)n), out((size_t)n);
  for (int64_t i = 0; i < n; i++) v[(size_t)i] = Item{{pts[3 * i], pts[3 * i + 1], pts[3 * i + 2]}, (uint32_t)i};
  build_rec(v, 0, n, 0, 0, n, out);
  for (int64_t i = 0; i < n; i++) {
    out_pts[3 * i] = out[(size_t)i].p.x;
    out_pts[3 * i + 1] = out[(size_t)i].p.y;
    out_pts[3 * i + 2] = out[(size_t)i].p.z;
    if (out_ids) out_ids[i] = out[(size_t)i].id;
  }
}

extern "C" void lsk_cpu_refalgo_knn(const float *tree, int64_t n, const float *qpts, int64_t nq,
                                    unsigned long long *heaps, int k, float cut2, int init,
                                    float *rmax, uint32_t id_base, int nthreads) {
  std::atomic<uint32_t> rbits{0};
  std::atomic<int64_t> next{0};
  auto work = [&] {
    uint32_t local = 0;
    for (;;) {
      const int64_t b = next.fetch_add(1024);
      if (b >= nq) break;
      const int64_t e = std::min(nq, b + 1024);
      for (int64_t qi = b; qi < e; qi++) {
        Heap cl{heaps + qi * (int64_t)k, k};
        if (init) {
          const unsigned long long ent = ((unsigned long long)lsk::fbits(cut2) << 32) | 0xffffffffull;
          for (int i = 0; i < k; i++) cl.h[i] = ent;
        }
        const float qx = qpts[3 * qi], qy = qpts[3 * qi + 1], qz = qpts[3 * qi + 2];
        int64_t prev = -1, curr = 0;
        if (n > 0) {
          for (;;) {
            const int64_t parent = (curr + 1) / 2 - 1;
            if (curr >= n) {
              prev = curr;
              curr = parent;
              continue;
            }
            const bool from_parent = prev < curr;
            const float px = tree[3 * curr], py = tree[3 * curr + 1], pz = tree[3 * curr + 2];
            if (from_parent) {
              const float d2 = lsk::dist2(qx - px, qy - py, qz - pz);
              if (d2 < cl.top()) cl.push(d2, id_base + (uint32_t)curr);
            }
            int level = 0;
            while (((curr + 1) >> (level + 1)) != 0) level++;
            const int dim = level % 3;
            const float split = dim == 0 ? px : (dim == 1 ? py : pz);
            const float qd = dim == 0 ? qx : (dim == 1 ? qy : qz);
            const float diff = qd - split;
            const int side = diff >= 0.f ? 1 : 0;
            const int64_t close = 2 * curr + 1 + side, far = 2 * curr + 2 - side;
            int64_t nxt;
            if (from_parent) nxt = close;
            else if (prev == close) nxt = (diff * diff < cl.top()) ? far : parent;
            else nxt = parent;
            if (nxt == -1) break;
            prev = curr;
            curr = nxt;
          }
        }
        const float top = cl.top();
        const float r = std::isinf(top) ? top : std::sqrt(top);
        local = std::max(local, lsk::fbits(r));
      }
    }
    uint32_t cur = rbits.load();
    while (local > cur && !rbits.compare_exchange_weak(cur, local)) {
    }
  };
  if (nthreads < 1) nthreads = 1;
  std::vector<std::thread> th;
  for (int t = 0; t < nthreads; t++) th.emplace_back(work);
  for (auto &x : th) x.join();
  if (rmax) {
    const uint32_t cur = lsk::fbits(*rmax);
    if (rbits.load() > cur) *rmax = lsk::bitsf(rbits.load());
  }
}

extern "C" void lsk_cpu_refalgo_extract(const unsigned long long *heaps, int64_t nq, int k,
                                        float *out) {
  for (int64_t qi = 0; qi < nq; qi++)
    out[qi] = lsk::final_distance(lsk::bitsf((uint32_t)(heaps[qi * (int64_t)k] >> 32)));
}
