// Exact k-th-distance backstop: wave-per-query radix select with 32-bit LDS counters.
//
// The production kernel (knn_rows.hip) keeps two 16-bit histogram bins per LDS dword and
// a bounded number of passes: that is what buys its occupancy, and it gives up on a
// query when a bin would overflow (more than 65535 values in one 1/8-octave bin: massive
// duplication, a far query looking at a tiny dense cluster), when it runs out of passes
// or when its collect count disagrees with the histogram. It never emits such a value:
// it appends the query to a failure list, and this kernel recomputes every listed query
// exactly, for any input and any k (also k > 65535, which the 16-bit kernel rejects).
// This is the exactness guarantee of the reference's FlexHeapCandidateList +
// stackFree::knn (unorderedDataVariant.cu:84-86, 97-102), without its N*k heap memory.
//
// Per query (one wave, all control flow wave-uniform; a failure list gives each query a
// block of 16 waves that split every tree's buckets and share the histogram; mixed-scale
// 2e7 k=100 with 4 / 8 / 16 waves: 379 / 448 / 505 Mpts/s, profiles/r6_listwaves/):
//  1. Upper bound: the max d² over k points taken around the query's position in
//     tree 0 (queries are tree points in curve order, so these are spatial neighbours;
//     any k distinct points give a valid bound), tightened by init_d2 when given, and
//     clipped at the -r cutoff.
//  2. Radix select on the float bits of d² in [lo, hi): every pass walks the bucket
//     trees (DFS, 64-ary expansion tested by 64 lanes, stack in LDS), prunes boxes whose
//     distance is >= hi and boxes whose farthest corner is closer than lo (their values
//     were counted by an earlier pass: a thin shell through a dense far cluster visits
//     only the buckets it cuts), counts a whole box at once when its [near, far] range
//     falls in one bin (subtree point count from the implicit tree), and counts the values
//     of each remaining 64-point bucket (one point per lane, one wave-wide atomic when
//     they share a bin) into 256 32-bit LDS bins. The bin holding the k-th value becomes the next
//     [lo, hi); a range of width 1 is the answer. <= 4 counting passes (8 bits each).
// Same canonical dist² (common.h) as the oracle and the production kernel: bit-identical.
#include "dev.h"

namespace {

using lsk::bitsf;
using lsk::fbits;

constexpr int kWaves = 4;      // waves per block, one query each (whole-set runs)
#ifndef LSK_EXACT_LIST_WAVES
#define LSK_EXACT_LIST_WAVES 16
#endif
constexpr int kListWaves = LSK_EXACT_LIST_WAVES;  // waves per block, all on one query (failure lists)
constexpr int kBins = 256;
// levels per tree expansion: 3 = the 8 children of a node tested by 8 lanes, 6 = its 64
// grandchildren by all 64 lanes (half the dependent node loads of a walk: the failure-list
// walks are latency-bound; mixed-scale 2e7 k=100 at 16 waves 504 -> 512 Mpts/s)
#ifndef LSK_EXACT_STEP
#define LSK_EXACT_STEP 6
#endif
constexpr int kStep = LSK_EXACT_STEP;
static_assert(kStep >= 1 && kStep <= 6, "a wave tests at most 64 boxes per expansion");
// DFS stack entries per wave: <= ceil(30 / step) expansions of 2^step - 1 siblings + 1
constexpr int kStack = ((30 + kStep - 1) / kStep * ((1 << kStep) - 1) + 1 + 31) / 32 * 32 < 128
                           ? 128
                           : ((30 + kStep - 1) / kStep * ((1 << kStep) - 1) + 1 + 31) / 32 * 32;

// W = 1: each wave owns its query (hist per wave). W > 1: the block's W waves share one
// query and one histogram, each walking a contiguous 1/W of every tree's buckets: the
// hard failures (a far query resolving a dense cluster point by point) are latency-bound
// walks, W waves in flight on them instead of one.
template <int W>
struct ExactLds {
  uint32_t hist[kBins];
  uint32_t stk[W][kStack];
};

template <int W>
__device__ __forceinline__ void qbarrier() {
  if constexpr (W == 1)
    __builtin_amdgcn_wave_barrier();
  else
    __syncthreads();
}

__device__ __forceinline__ uint32_t cand_bits(float qx, float qy, float qz, const float *p) {
  return fbits(lsk::dist2(qx - p[0], qy - p[1], qz - p[2]));
}

// Histogram every value v in [lo, hi) of the points of buckets [b0, b1) of one tree into
// hist[(v-lo)>>shift].
// (bx, by, bz): the query in the tree's frame for the box tests (= qx.. unless the tree was
// built in a rotated frame, lsk_knn_args.qrot); distances use qx..
__device__ void count_tree(const lsk_tree_view &T, float qx, float qy, float qz, float bx, float by, float bz,
                           uint32_t lo, uint32_t hi, uint32_t shift, uint32_t *hist, uint32_t *stk, int64_t b0,
                           int64_t b1, int lane) {
  if (T.n <= 0 || b0 >= b1) return;
  const int32_t depth = T.depth;
  const float lim = bitsf(hi);  // a box at distance >= bitsf(hi) holds no value < hi
  const lsk::vec3f q{bx, by, bz};
  const float4 *nodes = (const float4 *)T.nodes;
  uint32_t sp = 1;
  if (lane == 0) stk[0] = 1u;
  __builtin_amdgcn_wave_barrier();
  while (sp > 0) {
    sp--;
    const uint32_t node = lsk::uniform(stk[sp]);
    const int32_t lvl = 31 - __clz(node);
    if (lvl >= depth) {  // a bucket: one point per lane
      const int64_t b = (int64_t)node - ((int64_t)1 << depth);
      const int64_t i = b * lsk::kBucket + lane;
      const uint32_t v = i < T.n ? cand_bits(qx, qy, qz, T.pts + 3 * i) : hi;
      const bool in = v >= lo && v < hi;
      const uint32_t bin = (v - lo) >> shift;
      // a far query sees a dense bucket's values in one or a few bins: one atomic for
      // the wave when they all share a bin (same-address LDS atomics serialise)
      const uint64_t m = __ballot(in);
      if (m) {
        const uint32_t bf = lsk::uniform((uint32_t)__shfl((int)bin, (int)__builtin_ctzll(m)));
        if (__ballot(in && bin == bf) == m) {
          if (lane == 0) atomicAdd(&hist[bf], (uint32_t)__popcll(m));
        } else if (in) {
          atomicAdd(&hist[bin], 1u);
        }
      }
      continue;
    }
    // expand to the descendants `step` levels down (at most the bucket level): lanes
    // 0..2^step-1 test one box each, the needed ones are pushed
    const int32_t step = min(kStep, depth - lvl);
    const uint32_t nc = 1u << step;
    const uint32_t child = (node << step) + (uint32_t)lane;
    bool need = false;
    if ((uint32_t)lane < nc) {
      // the child's buckets, clipped to this wave's share
      const int32_t span_lg = depth - (lvl + step);
      const int64_t first = ((int64_t)child - ((int64_t)1 << (lvl + step))) << span_lg;
      const int64_t c0 = max(first, b0), c1 = min(first + ((int64_t)1 << span_lg), b1);
      const float4 lo4 = nodes[2 * child], hi4 = nodes[2 * child + 1];
      const float nd = lsk::box_dist2(q, {lo4.x, lo4.y, lo4.z}, {hi4.x, hi4.y, hi4.z});
      need = c0 < c1 && nd < lim;
      if (need) {
        // farthest corner (per-axis float differences, squares and fma are monotone: no
        // point inside is farther)
        const float fx = fmaxf(fabsf(lo4.x - bx), fabsf(hi4.x - bx));
        const float fy = fmaxf(fabsf(lo4.y - by), fabsf(hi4.y - by));
        const float fz = fmaxf(fabsf(lo4.z - bz), fabsf(hi4.z - bz));
        const uint32_t fb = fbits(lsk::dist2(fx, fy, fz)), nb = fbits(nd);
        if (fb < lo) {
          // shell test: only values below lo, counted by the previous passes
          need = false;
        } else if (nb >= lo && fb < hi && ((nb - lo) >> shift) == ((fb - lo) >> shift)) {
          // the whole (clipped) subtree falls in one bin: count it without visiting its
          // points (a far query looking at a dense cluster resolves coarse passes per box)
          const int64_t p0 = c0 * lsk::kBucket, p1 = min(T.n, c1 * lsk::kBucket);
          if (p1 > p0) atomicAdd(&hist[(nb - lo) >> shift], (uint32_t)(p1 - p0));
          need = false;
        }
      }
    }
    const uint64_t m = __ballot(need);
    if (need) {
      const uint32_t r = __popcll(m & ((1ull << lane) - 1ull));
      stk[sp + r] = child;
    }
    sp += (uint32_t)__popcll(m);
    __builtin_amdgcn_wave_barrier();
  }
}

// Upper bound (exclusive, in float bits) of the k-th value: max d² over k points around
// position `pos` of tree 0 (rest from tree 1 when tree 0 is smaller than k).
__device__ uint32_t window_bound(const lsk_knn_args &A, int64_t pos, float qx, float qy, float qz,
                                 uint32_t k, int lane) {
  const int64_t n0 = A.ntrees > 0 ? A.tree[0].n : 0;
  const int64_t m0 = n0 < (int64_t)k ? n0 : (int64_t)k;
  int64_t w0 = pos - (int64_t)(k / 2);
  if (w0 > n0 - m0) w0 = n0 - m0;
  if (w0 < 0) w0 = 0;
  uint32_t vmax = 0;
  for (int64_t j = lane; j < (int64_t)k; j += lsk::kWave) {
    const float *p = j < m0 ? A.tree[0].pts + 3 * (w0 + j) : A.tree[1].pts + 3 * (j - m0);
    vmax = max(vmax, cand_bits(qx, qy, qz, p));
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) vmax = max(vmax, (uint32_t)__shfl_xor((int)vmax, o));
  return lsk::uniform(vmax);
}

// The k-th value of query qi; every wave of the query's group (W) returns it.
template <int W>
__device__ uint32_t exact_kth(const lsk_knn_args &A, int64_t qi, ExactLds<W> &L, int wq, int lane) {
  const uint32_t k = (uint32_t)A.k;
  const float qx = lsk::uniform_f(A.qpts[3 * qi]);
  const float qy = lsk::uniform_f(A.qpts[3 * qi + 1]);
  const float qz = lsk::uniform_f(A.qpts[3 * qi + 2]);
  const float bx = A.qrot ? lsk::uniform_f(A.qrot[3 * qi]) : qx;
  const float by = A.qrot ? lsk::uniform_f(A.qrot[3 * qi + 1]) : qy;
  const float bz = A.qrot ? lsk::uniform_f(A.qrot[3 * qi + 2]) : qz;
  const uint32_t cut_b = (A.cut2 == A.cut2) ? fbits(fmaxf(A.cut2, 0.f)) : lsk::kInfBits;
  const uint32_t cut_lim = cut_b < lsk::kInfBits ? cut_b : lsk::kInfBits;
  int64_t total = 0;
  for (int t = 0; t < A.ntrees; t++) total += A.tree[t].n;
  if (total < (int64_t)k) return cut_b;
  // 1. upper bound hi (count(< hi) >= k is known when hi_ok)
  const uint32_t wb = window_bound(A, qi, qx, qy, qz, k, lane);
  uint32_t hi = cut_lim;
  bool hi_ok = false;
  if (wb < cut_lim) {
    hi = wb + 1u;
    hi_ok = true;
  }
  if (A.init_d2) {
    const float ub = A.init_d2[qi];
    if (ub >= 0.f && ub < __builtin_inff() && fbits(ub) + 1u < hi) {
      hi = fbits(ub) + 1u;
      hi_ok = true;
    }
  }
  // 2. radix select on [lo, hi)
  uint32_t lo = 0, below = 0;  // below = count of values < lo
  for (int pass = 0; pass < 8; pass++) {
    const uint32_t width = hi - lo;
    if (hi_ok && width == 1u) return lo;
    if (width == 0u) return cut_b;  // (not reached: hi > lo always holds)
    uint32_t shift = 0;
    while (((width - 1u) >> shift) >= (uint32_t)kBins) shift++;
    qbarrier<W>();  // (the previous pass's reads of hist are done)
    for (int j = wq * lsk::kWave + lane; j < kBins; j += W * lsk::kWave) L.hist[j] = 0u;
    qbarrier<W>();
    for (int t = 0; t < A.ntrees; t++) {
      const int64_t nb = (A.tree[t].n + lsk::kBucket - 1) / lsk::kBucket;
      count_tree(A.tree[t], qx, qy, qz, bx, by, bz, lo, hi, shift, L.hist, L.stk[wq], nb * wq / W, nb * (wq + 1) / W,
                 lane);
    }
    qbarrier<W>();
    // lane l owns bins 4l .. 4l+3
    const uint32_t c0 = L.hist[4 * lane], c1 = L.hist[4 * lane + 1];
    const uint32_t c2 = L.hist[4 * lane + 2], c3 = L.hist[4 * lane + 3];
    const uint32_t s = c0 + c1 + c2 + c3;
    uint32_t incl = s;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = (uint32_t)__shfl_up((int)incl, o);
      if (lane >= o) incl += y;
    }
    const uint32_t sum = lsk::uniform((uint32_t)__shfl((int)incl, 63));
    if ((uint64_t)below + sum < (uint64_t)k) return cut_b;  // < k values below the cutoff
    const uint32_t need = k - below;
    const uint32_t excl = incl - s;
    const bool mine = excl < need && incl >= need;
    const int src = (int)__builtin_ctzll(__ballot(mine));
    // bin inside the owning lane and the count below it
    uint32_t bsel = 3u, before = excl + c0 + c1 + c2;
    if (excl + c0 >= need) {
      bsel = 0u;
      before = excl;
    } else if (excl + c0 + c1 >= need) {
      bsel = 1u;
      before = excl + c0;
    } else if (excl + c0 + c1 + c2 >= need) {
      bsel = 2u;
      before = excl + c0 + c1;
    }
    const uint32_t b = 4u * (uint32_t)src + (uint32_t)__shfl((int)bsel, src);
    below += (uint32_t)__shfl((int)before, src);
    below = lsk::uniform(below);
    const uint32_t nlo = lo + (lsk::uniform(b) << shift);
    const uint64_t nhi = (uint64_t)nlo + (1ull << shift);
    hi = nhi < (uint64_t)hi ? (uint32_t)nhi : hi;
    lo = nlo;
    hi_ok = true;
  }
  return 0x7fc00000u;  // unreachable: width shrinks 256x per pass
}

__device__ __forceinline__ void write_answer(const lsk_knn_args &A, int64_t qi, uint32_t ans) {
  if (A.out_d2) A.out_d2[qi] = bitsf(ans);
  if (A.out_perm) A.out_final[A.out_perm[qi]] = lsk::final_distance(bitsf(ans));
}

// Whole-set runs (no list): one query per wave, grid-stride over the queries / groups.
__global__ __launch_bounds__(kWaves * 64) void knn_exact_kernel(const lsk_knn_args A) {
  __shared__ ExactLds<1> lds[kWaves];
  const int wid = threadIdx.x >> 6;
  const int lane = lsk::lane_id();
  ExactLds<1> &L = lds[wid];
  const int64_t gw = (int64_t)blockIdx.x * kWaves + wid;
  const int64_t tw = (int64_t)gridDim.x * kWaves;
  int64_t ng = A.ngroups;
  if (A.groups && A.ngroups_dev) ng = min(ng, (int64_t)A.ngroups_dev[0]);
  const int64_t total = A.groups ? ng * lsk::kBucket : A.nq;
  for (int64_t i = gw; i < total; i += tw) {
    int64_t qi = A.groups ? (int64_t)A.groups[i / lsk::kBucket] * lsk::kBucket + (i % lsk::kBucket) : i;
    qi = (int64_t)lsk::uniform((uint32_t)qi);
    if (qi >= A.nq) continue;
    const uint32_t ans = exact_kth<1>(A, qi, L, 0, lane);
    if (lane == 0) write_answer(A, qi, ans);
  }
}

// Failure lists: the block's kListWaves waves on one listed query at a time.
__global__ __launch_bounds__(kListWaves * 64) void knn_exact_list_kernel(const lsk_knn_args A,
                                                                         const uint32_t *__restrict__ list,
                                                                         const uint32_t *__restrict__ count,
                                                                         int64_t cap) {
  __shared__ ExactLds<kListWaves> L;
  const int wid = threadIdx.x >> 6;
  const int lane = lsk::lane_id();
  const int64_t c = (int64_t)count[0];
  const int64_t total = c < cap ? c : cap;
  for (int64_t i = blockIdx.x; i < total; i += gridDim.x) {
    const int64_t qi = (int64_t)lsk::uniform(list[i]);
    if (qi >= A.nq) continue;  // (uniform over the block)
    const uint32_t ans = exact_kth<kListWaves>(A, qi, L, wid, lane);
    if (wid == 0 && lane == 0) write_answer(A, qi, ans);
  }
}

}  // namespace

extern "C" int lsk_hip_knn_exact(const lsk_knn_args *args, const uint32_t *list,
                                 const uint32_t *count, int64_t cap, void *stream) {
  const lsk_knn_args &A = *args;
  if (A.k < 1 || A.nq >= ((int64_t)1 << 32) || A.ntrees < 0 || A.ntrees > 2) {
    lsk::set_last_error("knn_exact: k >= 1, nq < 2^32, ntrees in [0,2]");
    return 1;
  }
  for (int t = 0; t < A.ntrees; t++) {
    if (A.tree[t].depth > 30 || !A.tree[t].nodes || !A.tree[t].pts) {
      lsk::set_last_error("knn_exact: tree view incomplete");
      return 1;
    }
  }
  if (list && (!count || cap <= 0)) return 0;
  const int64_t work = list ? cap : (A.groups ? A.ngroups * lsk::kBucket : A.nq);
  if (work <= 0) return 0;
  // persistent grid-stride loops (every wave exits at the end of the list; with an empty
  // failure list the launch is a few microseconds)
  if (list) {
    const unsigned nblk = lsk_blocks(work, 1, 1024);
    knn_exact_list_kernel<<<nblk, kListWaves * 64, 0, (hipStream_t)stream>>>(A, list, count, cap);
  } else {
    const unsigned nblk = lsk_blocks(work, kWaves, 2048);
    knn_exact_kernel<<<nblk, kWaves * 64, 0, (hipStream_t)stream>>>(A);
  }
  LSK_CHECK_LAUNCH("knn_exact");
  return 0;
}
