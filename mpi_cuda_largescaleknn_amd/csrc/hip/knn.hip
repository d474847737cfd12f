// k-th-nearest-neighbour distance selection on gfx950 — the hot kernel.
//
// Reference behaviour reproduced: runQuery + extractFinalResult
// (unorderedDataVariant.cu:75-103, prePartitionedDataVariant.cu:76-112): for every query,
// the k-th smallest squared distance among all points (self included), where only
// distances < cutOff² count and cutOff² fills the list when fewer than k qualify.
// The reference keeps a k-entry max-heap per query in global memory (N·k·8 B,
// uncoalesced) and walks a left-balanced tree stack-free, one thread per
// query. This kernel is designed for CDNA4 instead:
//
//  * A wavefront owns 64 consecutive Morton-sorted queries (= one tree bucket), so the
//    traversal is wave-uniform: one LDS-resident node stack per wave, node boxes come
//    through scalar loads, and a leaf's 64 candidates are loaded with one vector load
//    (prefetched one leaf ahead) and broadcast lane by lane with v_readlane — every
//    candidate costs the 64 lanes one distance each, with no divergence and no LDS
//    traffic for candidates.
//  * Selection is a two-pass radix select on the bits of d² instead of a k-heap:
//      pass 1 builds a per-lane 64-bin histogram (1/8-octave bins of d², 16-bit counts
//             packed in LDS, lane-interleaved -> conflict-free ds_add_u32, branch-free
//             updates) and shrinks each lane's search radius as soon as k candidates
//             lie below a bin edge; afterwards the k-th value lies in one narrow bin and
//             the exact count c_lo of smaller values is known;
//      pass 2 replays the leaves recorded in pass 1 (LDS leaf list) that cut some
//             lane's shell [band_lo, band_hi), collects the values inside that bin into a
//             per-wave LDS pool, and each lane runs a (k-c_lo)-max-heap over its few
//             collected values in LDS.
//    Pass 1 is seeded with the group's own bucket and its Morton neighbours, so most
//    lanes start the tree walk with a radius close to the final one.
//    Out-of-range estimates (under/overflow), oversized bins (refinement by 6 more bits)
//    and duplicate-heavy data are handled by bounded extra passes, so the result is
//    exact for any input: it equals the CPU oracle bit for bit.
#include "dev.h"

namespace {

using lsk::bitsf;
using lsk::fbits;

constexpr int kWavesPerBlock = 4;
constexpr int kThreads = kWavesPerBlock * lsk::kWave;
constexpr int kPool = 2048;      // dwords per wave: 32-dword histogram x 64 lanes, or collect pool
constexpr int kStackCap = 64;    // DFS stack (depth <= 32 -> <= 33 live entries)
constexpr int kLeafCap = 256;    // leaves recorded in pass 1 for replay
constexpr int kBatch = 8;        // leaves gathered per processing batch
constexpr int kBins = lsk::kSelBins;        // 64
constexpr uint32_t kShift0 = 20;            // 1/8-octave bins of d²
constexpr uint32_t kMaxPasses = 96;         // hard bound on passes per wave (never hang)

enum : uint32_t { ST_HIST = 0, ST_READY = 1, ST_DONE = 2 };
enum { MODE_HIST = 0, MODE_COLLECT = 1 };

struct WaveLds {
  uint32_t pool[kPool];
  uint32_t stack[kStackCap];
  uint32_t leaves[kLeafCap];
  uint32_t batch[kBatch];
};

struct Lane {
  float qx, qy, qz;
  uint32_t state;
  // histogram pass state
  uint32_t lo_b, hi_b, shift;
  int32_t bin_hi;
  uint32_t c_hi, zc;
  uint32_t cut_lim;  // min(cut2 bits, +inf bits)
  // band state (READY)
  uint32_t band_lo, band_w, m, bc;
  uint32_t coff, ccnt;
  uint32_t ans;
};

__device__ __forceinline__ void set_range(Lane &s, uint32_t lo_b, uint32_t shift, uint32_t top_limit) {
  s.lo_b = lo_b;
  s.shift = shift;
  uint64_t top = (uint64_t)lo_b + ((uint64_t)kBins << shift);
  uint64_t hi = top < (uint64_t)top_limit ? top : (uint64_t)top_limit;
  s.hi_b = (uint32_t)hi;
  s.bin_hi = hi > lo_b ? (int32_t)((hi - lo_b + ((1ull << shift) - 1)) >> shift) : 0;
  s.c_hi = 0;
  s.zc = 0;
}

__device__ __forceinline__ uint32_t hist_read(const uint32_t *pool, uint32_t b, int lane) {
  return (pool[(b >> 1) * lsk::kWave + lane] >> ((b & 1u) << 4)) & 0xffffu;
}

// Count in the current top bin (the underflow bin once every bin is dropped).
__device__ __forceinline__ uint32_t top_count(const Lane &s, const uint32_t *pool, int lane) {
  return s.bin_hi > 0 ? hist_read(pool, (uint32_t)s.bin_hi - 1u, lane) : s.c_hi;
}

// Drop top bins while the bins below them already hold >= k values: every value in a
// dropped bin is beyond the k-th, so the lane's search radius shrinks to that edge.
__device__ __forceinline__ void hist_shrink(Lane &s, const uint32_t *pool, int lane, uint32_t k) {
  while (s.bin_hi > 0) {
    const uint32_t top = hist_read(pool, (uint32_t)s.bin_hi - 1u, lane);
    if (s.c_hi - top < k) break;
    s.c_hi -= top;
    s.bin_hi--;
    s.hi_b = s.lo_b + ((uint32_t)s.bin_hi << s.shift);
  }
}

__device__ __forceinline__ float bcast(float v, uint32_t j) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), (int)j));
}

// One leaf: lane j holds candidate j in (px,py,pz); candidates are broadcast with
// v_readlane (no LDS traffic) and processed in chunks of 8. Histogram updates are
// branch-free (a lane that does not count a value adds 0 to a valid bin).
template <int MODE, bool ZC>
__device__ __forceinline__ void process_points(Lane &s, float px, float py, float pz,
                                               uint32_t cnt, uint32_t *pool, int lane,
                                               uint32_t k) {
  for (uint32_t j0 = 0; j0 < cnt; j0 += 8) {
    uint32_t u[8];
    uint32_t umin = 0xffffffffu;
#pragma unroll
    for (int t = 0; t < 8; t++) {
      const uint32_t j = j0 + (uint32_t)t;
      const float d2 = lsk::dist2(s.qx - bcast(px, j), s.qy - bcast(py, j), s.qz - bcast(pz, j));
      u[t] = (j < cnt) ? fbits(d2) : 0xffffffffu;
      umin = min(umin, u[t]);
    }
    if (MODE == MODE_HIST) {
      if (!__ballot(umin < s.hi_b)) continue;
      const uint32_t hb = s.hi_b, lb = s.lo_b, sh = s.shift;
#pragma unroll
      for (int t = 0; t < 8; t++) {
        const uint32_t v = u[t];
        const bool in = v < hb;
        const uint32_t b = min((v - lb) >> sh, 63u);
        const uint32_t inc = (in && v >= lb) ? (1u << ((b & 1u) << 4)) : 0u;
        atomicAdd(&pool[(b >> 1) * lsk::kWave + lane], inc);
        s.c_hi += in ? 1u : 0u;
        if (ZC) s.zc += (v == 0u) ? 1u : 0u;
      }
    } else {
      const uint32_t bl = s.band_lo, bw = s.band_w;
      bool any = false;
#pragma unroll
      for (int t = 0; t < 8; t++) any = any || (u[t] - bl < bw);
      if (!__ballot(any)) continue;
#pragma unroll
      for (int t = 0; t < 8; t++) {
        if (u[t] - bl < bw) {
          if (s.ccnt < s.bc) pool[s.coff + s.ccnt] = u[t];
          s.ccnt++;
        }
      }
    }
  }
  // one shrink check per leaf (the bound lags at most 64 candidates behind)
  if (MODE == MODE_HIST && __ballot(s.c_hi >= k)) hist_shrink(s, pool, lane, k);
}

__device__ __forceinline__ float lane_bound(const Lane &s, int mode) {
  return bitsf(mode == MODE_HIST ? s.hi_b : (s.band_w ? s.band_lo + s.band_w : 0u));
}

struct WaveCtx {
  WaveLds *L;
  int lane;
  uint32_t k;
  uint32_t g;          // group id (== tree-0 bucket when queries are tree 0's points)
  int32_t seed;        // neighbour buckets seeded on each side (0 = off)
  float cx, cy, cz;    // group centre (near-first ordering)
  uint32_t nleaves;
  bool list_ok;
  bool count_zero;     // count exact zeros (only after an underflow)
  uint32_t evals, leaves_visited, nodes_visited;
};

__device__ __forceinline__ lsk_tree_view pick_tree(const lsk_knn_args &A, uint32_t t) {
  return t ? A.tree[1] : A.tree[0];
}

// Leaf entry = (tree << 31) | bucket. Loads lane's candidate (vector load, padded array).
__device__ __forceinline__ uint32_t load_leaf(const lsk_knn_args &A, uint32_t e, int lane,
                                              float &px, float &py, float &pz) {
  const lsk_tree_view T = pick_tree(A, e >> 31);
  const int64_t base = (int64_t)(e & 0x7fffffffu) * lsk::kBucket;
  const int64_t rem = T.n - base;
  const float *p = T.pts + 3 * (base + lane);
  px = p[0];
  py = p[1];
  pz = p[2];
  return rem < lsk::kBucket ? (uint32_t)rem : (uint32_t)lsk::kBucket;
}

// Processes the leaves queued in the wave's LDS batch; the next leaf's candidates are
// loaded while the current one is being processed.
template <int MODE>
__device__ void process_batch(Lane &s, WaveCtx &W, const lsk_knn_args &A, uint32_t nb) {
  float px, py, pz;
  uint32_t cnt = load_leaf(A, lsk::uniform(W.L->batch[0]), W.lane, px, py, pz);
  for (uint32_t i = 0; i < nb; i++) {
    const float cx = px, cy = py, cz = pz;
    const uint32_t ccnt = cnt;
    if (i + 1 < nb) cnt = load_leaf(A, lsk::uniform(W.L->batch[i + 1]), W.lane, px, py, pz);
    W.leaves_visited++;
    W.evals += ccnt;
    if (MODE == MODE_HIST && W.count_zero)
      process_points<MODE, true>(s, cx, cy, cz, ccnt, W.L->pool, W.lane, W.k);
    else
      process_points<MODE, false>(s, cx, cy, cz, ccnt, W.L->pool, W.lane, W.k);
  }
}

__device__ __forceinline__ void batch_push(WaveCtx &W, uint32_t &nb, uint32_t e, bool record) {
  if (W.lane == 0) W.L->batch[nb] = e;
  nb++;
  if (record) {
    if (W.nleaves < kLeafCap) {
      if (W.lane == 0) W.L->leaves[W.nleaves] = e;
      W.nleaves++;
    } else {
      W.list_ok = false;
    }
  }
}

// Leaf test per lane. HIST: box closer than the lane's radius. COLLECT: the box cuts
// the lane's shell [band_lo, band_hi) — a box entirely inside band_lo holds only values
// already counted in c_lo (max-distance is monotone like box_dist2, common.h).
template <int MODE>
__device__ __forceinline__ bool leaf_needed(const Lane &s, const lsk::v4f &lo, const lsk::v4f &hi) {
  const lsk::vec3f q{s.qx, s.qy, s.qz};
  const bool near = lsk::box_dist2(q, {lo.x, lo.y, lo.z}, {hi.x, hi.y, hi.z}) < lane_bound(s, MODE);
  if (MODE == MODE_HIST) return near;
  const float fx = fmaxf(fabsf(lo.x - s.qx), fabsf(hi.x - s.qx));
  const float fy = fmaxf(fabsf(lo.y - s.qy), fabsf(hi.y - s.qy));
  const float fz = fmaxf(fabsf(lo.z - s.qz), fabsf(hi.z - s.qz));
  return near && fbits(lsk::dist2(fx, fy, fz)) >= s.band_lo;
}

// Depth-first, near-child-first walk of every tree with a per-wave LDS stack; needed
// leaves are gathered into batches of kBatch and processed with load prefetching.
// With seeding, tree 0's buckets [g-seed, g+seed] are processed first (nearest first)
// and skipped by the walk.
template <int MODE>
__device__ void traverse(Lane &s, WaveCtx &W, const lsk_knn_args &A, bool record) {
  const lsk::vec3f q{s.qx, s.qy, s.qz};
  const lsk::vec3f c{W.cx, W.cy, W.cz};
  for (uint32_t t = 0; t < (uint32_t)A.ntrees; t++) {
    const lsk_tree_view T = pick_tree(A, t);
    if (T.n <= 0) continue;
    lsk::cfloat4_p nodes = lsk::as_const4(T.nodes);
    const uint32_t leaf0 = 1u << T.depth;
    const uint32_t nbuckets = (uint32_t)((T.n + lsk::kBucket - 1) / lsk::kBucket);
    int64_t skip_lo = 1, skip_hi = 0;  // empty
    if (t == 0 && W.seed > 0) {
      skip_lo = (int64_t)W.g - W.seed;
      skip_hi = (int64_t)W.g + W.seed;
      uint32_t nb = 0;
      for (int32_t d = 0; d <= W.seed; d++) {
        for (int32_t sgn = 0; sgn < (d ? 2 : 1); sgn++) {
          const int64_t b = sgn ? (int64_t)W.g + d : (int64_t)W.g - d;
          if (b < 0 || b >= (int64_t)nbuckets) continue;
          batch_push(W, nb, (uint32_t)b, record);
          if (nb == (uint32_t)kBatch) {
            process_batch<MODE>(s, W, A, nb);
            nb = 0;
          }
        }
      }
      if (nb) process_batch<MODE>(s, W, A, nb);
    }
    uint32_t sp = 0;
    if (W.lane == 0) W.L->stack[0] = 1u;
    sp = 1;
    while (sp > 0) {
      uint32_t nb = 0;
      const float lim = lane_bound(s, MODE);
      while (sp > 0 && nb < (uint32_t)kBatch) {
        sp--;
        const uint32_t node = lsk::uniform(W.L->stack[sp]);
        W.nodes_visited++;
        if (node >= leaf0) {
          const uint32_t b = node - leaf0;
          if (b >= nbuckets || ((int64_t)b >= skip_lo && (int64_t)b <= skip_hi)) continue;
          const lsk::v4f lo = nodes[2 * node], hi = nodes[2 * node + 1];
          if (__ballot(leaf_needed<MODE>(s, lo, hi))) batch_push(W, nb, (t << 31) | b, record);
          continue;
        }
        const lsk::v4f lo = nodes[2 * node], hi = nodes[2 * node + 1];
        if (!__ballot(lsk::box_dist2(q, {lo.x, lo.y, lo.z}, {hi.x, hi.y, hi.z}) < lim)) continue;
        const uint32_t c0 = 2 * node, c1 = c0 + 1;
        const lsk::v4f l0 = nodes[2 * c0], h0 = nodes[2 * c0 + 1];
        const lsk::v4f l1 = nodes[2 * c1], h1 = nodes[2 * c1 + 1];
        const bool n0 = __ballot(lsk::box_dist2(q, {l0.x, l0.y, l0.z}, {h0.x, h0.y, h0.z}) < lim) != 0;
        const bool n1 = __ballot(lsk::box_dist2(q, {l1.x, l1.y, l1.z}, {h1.x, h1.y, h1.z}) < lim) != 0;
        const float g0 = lsk::box_dist2(c, {l0.x, l0.y, l0.z}, {h0.x, h0.y, h0.z});
        const float g1 = lsk::box_dist2(c, {l1.x, l1.y, l1.z}, {h1.x, h1.y, h1.z});
        const bool first0 = g0 <= g1;  // near child popped first => pushed last
        const uint32_t a = first0 ? c1 : c0, b = first0 ? c0 : c1;
        const bool na = first0 ? n1 : n0, nbb = first0 ? n0 : n1;
        if (na) {
          if (W.lane == 0) W.L->stack[sp] = a;
          sp++;
        }
        if (nbb) {
          if (W.lane == 0) W.L->stack[sp] = b;
          sp++;
        }
      }
      if (nb) process_batch<MODE>(s, W, A, nb);
    }
  }
}

// Re-walk only the leaves recorded in the first histogram pass (valid while every
// lane's bound is <= its pass-1 bound).
template <int MODE>
__device__ void replay(Lane &s, WaveCtx &W, const lsk_knn_args &A) {
  uint32_t i = 0;
  while (i < W.nleaves) {
    uint32_t nb = 0;
    for (; i < W.nleaves && nb < (uint32_t)kBatch; i++) {
      const uint32_t e = lsk::uniform(W.L->leaves[i]);
      const lsk_tree_view T = pick_tree(A, e >> 31);
      lsk::cfloat4_p nodes = lsk::as_const4(T.nodes);
      const uint32_t node = (1u << T.depth) + (e & 0x7fffffffu);
      const lsk::v4f lo = nodes[2 * node], hi = nodes[2 * node + 1];
      if (__ballot(leaf_needed<MODE>(s, lo, hi))) batch_push(W, nb, e, false);
    }
    if (nb) process_batch<MODE>(s, W, A, nb);
  }
}

__device__ void heap_sift(uint32_t *h, uint32_t i, uint32_t m) {
  const uint32_t v = h[i];
  for (;;) {
    uint32_t l = 2 * i + 1, r = l + 1, c = i;
    uint32_t cv = v;
    if (l < m && h[l] > cv) { c = l; cv = h[l]; }
    if (r < m && h[r] > cv) { c = r; cv = h[r]; }
    if (c == i) break;
    h[i] = cv;
    i = c;
  }
  h[i] = v;
}

// Per-lane estimate of the k-th squared distance from the group's own points (pass 0):
// the m0-th smallest squared distance to the group's queries (self included, broadcast
// from the lanes that hold them), scaled by (k/m0)^(2/3) (uniform local density).
__device__ __forceinline__ float own_group_estimate(const Lane &s, uint32_t nvalid, uint32_t k) {
  constexpr int M = 8;
  float best[M];
#pragma unroll
  for (int i = 0; i < M; i++) best[i] = __builtin_inff();
  for (uint32_t j0 = 0; j0 < nvalid; j0 += 8) {
#pragma unroll
    for (int t = 0; t < 8; t++) {
      const uint32_t j = j0 + (uint32_t)t;
      float v = lsk::dist2(s.qx - bcast(s.qx, j), s.qy - bcast(s.qy, j), s.qz - bcast(s.qz, j));
      v = (j < nvalid) ? v : __builtin_inff();
#pragma unroll
      for (int i = 0; i < M; i++) {  // sorted insertion network
        const float lo = fminf(best[i], v);
        v = fmaxf(best[i], v);
        best[i] = lo;
      }
    }
  }
  const uint32_t m0 = k < (uint32_t)M ? k : (uint32_t)M;
  float dm = best[0];
#pragma unroll
  for (int i = 1; i < M; i++) dm = (i + 1 == (int)m0) ? best[i] : dm;
  return dm * cbrtf(((float)k / (float)m0) * ((float)k / (float)m0));
}

enum : uint32_t {
  QS_OVERFLOW = 1, QS_UNDERFLOW = 2, QS_REFINE = 4, QS_LIST_INVALID = 8, QS_COLLECTED = 16,
  QS_DONE_BAND1 = 32, QS_DONE_CUT = 64, QS_DONE_ZERO = 128, QS_LIMIT = 256, QS_MISMATCH = 512,
  QS_HINT = 1024
};

__global__ __launch_bounds__(kThreads) void knn_kernel(const lsk_knn_args A) {
  __shared__ WaveLds lds[kWavesPerBlock];
  const int wid = threadIdx.x >> 6;
  const int lane = lsk::lane_id();
  const uint32_t blk = lsk::xcd_remap(blockIdx.x, gridDim.x);
  const uint64_t wave = (uint64_t)blk * kWavesPerBlock + wid;
  const uint64_t ngroups = A.groups ? (uint64_t)A.ngroups : (uint64_t)((A.nq + 63) / 64);
  if (wave >= ngroups) return;
  const uint32_t g = lsk::uniform(A.groups ? A.groups[wave] : (uint32_t)wave);
  const int64_t q0 = (int64_t)g * lsk::kBucket;
  const int64_t qi = q0 + lane;
  const bool valid = qi < A.nq;
  const uint32_t nvalid = (uint32_t)((A.nq - q0) < lsk::kBucket ? (A.nq - q0) : lsk::kBucket);
  const uint32_t k = (uint32_t)A.k;

  WaveCtx W;
  W.L = &lds[wid];
  W.lane = lane;
  W.k = k;
  W.g = g;
  W.seed = A.seed;
  W.nleaves = 0;
  W.list_ok = true;
  W.count_zero = false;
  W.evals = W.leaves_visited = W.nodes_visited = 0;

  Lane s;
  s.qx = valid ? A.qpts[3 * qi] : 0.f;
  s.qy = valid ? A.qpts[3 * qi + 1] : 0.f;
  s.qz = valid ? A.qpts[3 * qi + 2] : 0.f;
  uint32_t qs = 0;

  // group bounding box -> centre for near-child-first ordering
  const float inf = __builtin_inff();
  const float lx = lsk::wave_min(valid ? s.qx : inf), hx = lsk::wave_max(valid ? s.qx : -inf);
  const float ly = lsk::wave_min(valid ? s.qy : inf), hy = lsk::wave_max(valid ? s.qy : -inf);
  const float lz = lsk::wave_min(valid ? s.qz : inf), hz = lsk::wave_max(valid ? s.qz : -inf);
  W.cx = 0.5f * (lx + hx);
  W.cy = 0.5f * (ly + hy);
  W.cz = 0.5f * (lz + hz);

  float r_est2 = own_group_estimate(s, nvalid, k);
  {
    // Robust cap: a group straddling a Morton discontinuity has lanes with few
    // same-side neighbours in the group, whose estimate is then orders of magnitude too
    // large (range far above the k-th value: huge first-pass bound, one slow wave).
    // Cap at 16x (4 octaves of d2) the wave's lower-quartile estimate.
    const bool ok = valid && r_est2 > 0.f && r_est2 < inf;
    const uint32_t kq = max(1u, nvalid / 4u);
    const uint32_t pb = lsk::wave_kth_smallest(ok ? fbits(r_est2) : 0xffffffffu, kq);
    if (pb < lsk::kInfBits) r_est2 = fminf(r_est2, 16.f * bitsf(pb));
  }
  if (!(r_est2 > 0.f) || !(r_est2 < inf)) {
    r_est2 = A.r_hint2 >= 0.f ? A.r_hint2 : A.tree[0].nodes[3];
    qs |= QS_HINT;
  }
  if (!(r_est2 > 0.f) || !(r_est2 < inf)) r_est2 = 1.f;

  const uint32_t cut_b = (A.cut2 == A.cut2) ? fbits(fmaxf(A.cut2, 0.f)) : lsk::kInfBits;
  s.cut_lim = cut_b < lsk::kInfBits ? cut_b : lsk::kInfBits;
  s.band_lo = s.band_w = s.m = s.bc = s.coff = s.ccnt = 0;
  // every lane's histogram state is defined (lanes that never histogram included:
  // the wave-wide shrink step reads bin_hi / c_hi of all lanes)
  s.lo_b = s.hi_b = s.shift = s.c_hi = 0;
  s.bin_hi = 0;
  s.zc = 0;
  s.ans = cut_b;

  int64_t total_pts = 0;
  for (int t = 0; t < A.ntrees; t++) total_pts += pick_tree(A, t).n;

  uint32_t hist_passes = 0, limit = 0;

  if (!valid || total_pts < (int64_t)k) {
    s.state = ST_DONE;  // fewer than k points overall -> cutoff value (reference: heap init)
    s.hi_b = 0;
    qs |= QS_DONE_CUT;
  } else {
    s.state = ST_HIST;
    // range = 8 octaves of d^2 ending 2 octaves (2x in distance) above the estimate:
    // the own-group estimate is biased high (a group holds only part of a query's
    // neighbourhood), so a tight top keeps the first pass's search region small
    const uint32_t est_b = fbits(r_est2);
    const uint32_t off = 48u << kShift0;
    const uint32_t lo0 = est_b > off ? est_b - off : 0u;
    set_range(s, lo0, kShift0, s.cut_lim);
  }

  uint32_t pool_off = 0;
  bool first = true;
  uint32_t passes = 0;
  for (;;) {
    while (__ballot(s.state == ST_HIST)) {
      if (++passes > kMaxPasses) {
        limit = 1;
        if (s.state == ST_HIST) {
          s.state = ST_DONE;
          s.ans = 0x7fc00000u;  // NaN marks failure (never expected; counted in stats)
          qs |= QS_LIMIT;
        }
        break;
      }
      hist_passes++;
      if (s.state != ST_HIST) {  // not histogramming this pass: count nothing
        s.hi_b = 0;
        s.c_hi = 0;
        s.bin_hi = 0;
      }
#pragma unroll 8
      for (int j = 0; j < kPool / lsk::kWave; j++) W.L->pool[j * lsk::kWave + lane] = 0u;
      if (first || !W.list_ok) traverse<MODE_HIST>(s, W, A, first);
      else replay<MODE_HIST>(s, W, A);
      first = false;
      bool ovf = false, udf = false;
      if (s.state == ST_HIST) {
        const uint32_t top = top_count(s, W.L->pool, lane);
        if (s.c_hi < k) {
          if (s.hi_b >= s.cut_lim) {
            s.state = ST_DONE;
            s.ans = cut_b;
            qs |= QS_DONE_CUT;
          } else {  // estimate too small: next 8 octaves up (pass-1 leaf list now too small)
            ovf = true;
            qs |= QS_OVERFLOW;
            set_range(s, s.hi_b, kShift0, s.cut_lim);
          }
        } else if (s.bin_hi == 0) {
          if (W.count_zero && s.zc >= k) {
            s.state = ST_DONE;
            s.ans = 0u;
            qs |= QS_DONE_ZERO;
          } else {  // estimate too large: next 8 octaves down, counting exact zeros
            udf = true;
            qs |= QS_UNDERFLOW;
            const uint32_t topb = s.lo_b;
            set_range(s, topb > (64u << kShift0) ? topb - (64u << kShift0) : 0u, kShift0, topb);
          }
        } else {
          const uint32_t bl = s.lo_b + ((uint32_t)(s.bin_hi - 1) << s.shift);
          const uint32_t bw = s.hi_b - bl;
          if (bw <= 1u) {
            s.state = ST_DONE;
            s.ans = bl;
            qs |= QS_DONE_BAND1;
          } else {
            s.state = ST_READY;
            s.band_lo = bl;
            s.band_w = bw;
            s.m = k - (s.c_hi - top);
            s.bc = top;
          }
        }
      }
      if (__ballot(ovf)) W.list_ok = false;
      if (__ballot(udf)) W.count_zero = true;
    }
    if (limit) break;
    // carve the collect pool; refine the biggest bands if it does not fit
    const uint32_t need = s.state == ST_READY ? s.bc : 0u;
    uint32_t x = need;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(x, o);
      if (lane >= o) x += y;
    }
    const uint32_t total = __shfl(x, 63);
    pool_off = x - need;
    if (total <= (uint32_t)kPool) break;
    if (s.state == ST_READY && s.bc > (uint32_t)(kPool / lsk::kWave)) {
      qs |= QS_REFINE;
      const uint32_t sh = s.shift >= 6u ? s.shift - 6u : 0u;
      set_range(s, s.band_lo, sh, s.band_lo + s.band_w);
      s.band_lo = s.band_w = 0;
      s.state = ST_HIST;
    }
  }

  if (!W.list_ok) qs |= QS_LIST_INVALID;
  if (!limit && __ballot(s.state == ST_READY)) {
    if (s.state != ST_READY) s.band_lo = s.band_w = 0;
    s.coff = pool_off;
    s.ccnt = 0;
    if (W.list_ok) replay<MODE_COLLECT>(s, W, A);
    else traverse<MODE_COLLECT>(s, W, A, false);
    if (s.state == ST_READY) {
      qs |= QS_COLLECTED;
      if (s.ccnt != s.bc) qs |= QS_MISMATCH;
      uint32_t *h = W.L->pool + s.coff;
      const uint32_t c = min(s.ccnt, s.bc), m = s.m;
      if (m >= 1 && m <= c) {
        for (int i = (int)(m / 2) - 1; i >= 0; i--) heap_sift(h, (uint32_t)i, m);
        for (uint32_t i = m; i < c; i++) {
          const uint32_t v = h[i];
          if (v < h[0]) {
            h[0] = v;
            heap_sift(h, 0, m);
          }
        }
        s.ans = h[0];
      } else {
        qs |= QS_MISMATCH;
        s.ans = 0x7fc00000u;
      }
    }
  }

  if (valid) {
    if (A.out_perm) A.out_final[A.out_perm[qi]] = lsk::final_distance(bitsf(s.ans));
    if (A.out_d2) A.out_d2[qi] = bitsf(s.ans);
    if (A.qstatus) A.qstatus[qi] = qs | (hist_passes << 16);
  }

  if (A.stats) {
    auto cnt = [&](uint32_t bit) {
      return (unsigned long long)__popcll(__ballot(valid && (qs & bit)));
    };
    const unsigned long long c_ovf = cnt(QS_OVERFLOW), c_udf = cnt(QS_UNDERFLOW),
                             c_ref = cnt(QS_REFINE), c_mm = cnt(QS_MISMATCH), c_hint = cnt(QS_HINT);
    if (lane == 0) {
      atomicAdd(&A.stats[0], (unsigned long long)W.evals);
      atomicAdd(&A.stats[1], (unsigned long long)W.leaves_visited);
      atomicAdd(&A.stats[2], (unsigned long long)W.nodes_visited);
      atomicAdd(&A.stats[3], (unsigned long long)hist_passes);
      atomicAdd(&A.stats[4], c_ovf);
      atomicAdd(&A.stats[5], c_udf);
      atomicAdd(&A.stats[6], c_ref);
      atomicAdd(&A.stats[7], c_mm);
      atomicAdd(&A.stats[8], (unsigned long long)limit);
      atomicAdd(&A.stats[9], W.list_ok ? 0ull : 1ull);
      atomicAdd(&A.stats[10], 1ull);
      atomicAdd(&A.stats[11], c_hint);
      atomicAdd(&A.stats[12], (unsigned long long)W.nleaves);
    }
  }
}

}  // namespace

extern "C" int lsk_hip_knn(const lsk_knn_args *args, void *stream) {
  const lsk_knn_args &A = *args;
  if (A.k < 1 || A.k > 65535) {
    lsk::set_last_error("knn: k must be in [1, 65535] for the radix-select kernel");
    return 1;
  }
  if (A.nq >= ((int64_t)1 << 32) || A.ntrees < 0 || A.ntrees > 2 || A.seed < 0 || A.seed > 64) {
    lsk::set_last_error("knn: nq must be < 2^32, ntrees in [0,2], seed in [0,64]");
    return 1;
  }
  for (int t = 0; t < A.ntrees; t++) {
    if (A.tree[t].n >= ((int64_t)1 << 31) || A.tree[t].depth > 26) {
      lsk::set_last_error("knn: tree too large (n < 2^31 per tree)");
      return 1;
    }
  }
  const int64_t ngroups = A.groups ? A.ngroups : (A.nq + 63) / 64;
  if (ngroups <= 0) return 0;
  const unsigned nblk = lsk_blocks(ngroups, kWavesPerBlock);
  knn_kernel<<<nblk, kThreads, 0, (hipStream_t)stream>>>(A);
  LSK_CHECK_LAUNCH("knn");
  return 0;
}
