// k-th-NN distance selection over the bucket tree (knn_rows_kernel): the tree-walk k-NN
// pass — the path for skewed data (clustered, planar, exact copies, mixed scale) and for
// halo re-queries against two trees; near-uniform local passes use knn_grid.hip, which
// shares the selection algorithm below. Contract: reference runQuery +
// extractFinalResult (unorderedDataVariant.cu:75-103): for every query, the k-th smallest
// canonical squared distance (common.h dist2) to the tree points, self included, or the
// cutoff when fewer than k points lie below it.
//
// Selection: a radix select on the float bits of d² (non-negative floats order like their
// bits). Pass 1 (HIST) counts each lane's values in 40 bins of 1/8 octave of d² in LDS
// (two 16-bit counters per dword) over a range placed by an estimate of the k-th value;
// the range top shrinks online as soon as k values lie below a bin edge, which is what
// culls the walk. Pass 2 (COLLECT) gathers the values of the bin holding the k-th into a
// per-wave LDS pool, where a per-lane (k - below)-max-heap yields the exact value. Lanes
// whose range was wrong (overflow / underflow / too-full bin) run further passes; lanes
// the 16-bit counters cannot resolve exactly go to the failure list (knn_exact.hip).
//
// SIMD decomposition:
//  * a wave owns 64 consecutive Hilbert-sorted queries split into 4 ROWS of 16 (the
//    16-lane rows of CDNA4 DPP). The tree walk is wave-uniform: best-first over the
//    implicit bucket tree (64-entry priority list in two VGPRs, DFS stack in one VGPR as
//    bounded overflow, 4-ary steps with scalar node loads); at the level above the
//    buckets each row tests the 8 16-point QUARTER boxes of the node's two buckets with
//    its own 16 lanes and queues the quarters it needs. Quarter boxes of 4 such nodes are
//    fetched with one vector load per node (one memory latency per batch) and broadcast
//    with v_readlane;
//  * rows consume their queues in lockstep: one step = one quarter per row, the 16
//    candidates of each row's quarter are loaded by the row's 16 lanes (one vector load,
//    prefetched one step ahead) and broadcast inside the row with DPP row_newbcast, which
//    the compiler folds into v_subrev_f32_dpp — the broadcast costs nothing;
//  * so a query evaluates only candidates of quarters its own 16-query row needs (small
//    union of balls, 16-point culling granularity) instead of everything its 64-query
//    group needs;
//  * walk and processing alternate (fill the row queues until every row has a batch
//    pending, then drain in lockstep); pass 1 logs the visited nodes with the rows that
//    took each quarter (a private-memory log striped over the lanes), and the later
//    passes (collect, retries) replay that log instead of walking the tree again;
//  * histogram bin index = sat(d²bits - lo) >> shift: values below the range land in bin
//    0 (no separate compare), and c_base tracks how many of them are known to be below;
//  * the per-lane estimate that places the first range is capped by the wave's lower
//    quartile: groups straddling a curve discontinuity otherwise produce a few waves
//    with absurd first-pass bounds that dominate the kernel's tail.
//  Inner-loop cost per candidate and lane: 6 VALU for d² (DPP broadcast folded into the
//  subtracts) + 5 VALU + 1 exec-masked ds_add for the histogram when in range (compiled
//  with -fno-slp-vectorize: packed-math ops cannot take DPP operands). 7 waves/SIMD
//  (72 VGPRs, 5.6 KB LDS per wave, 2-wave blocks).
#include "dev.h"

namespace {

using lsk::bitsf;
using lsk::fbits;

// waves per workgroup: a block holds its LDS until its last wave ends, so 2-wave blocks
// free slots sooner when waves differ in length (1B bench 633.5/633.9 vs 629.7/631.5
// Mpts/s with 4; 1 wave per block is slower: profiles/archive/r2_s3_wpb)
#ifndef LSK_ROWS_WPB
#define LSK_ROWS_WPB 2
#endif
constexpr int kWavesPerBlock = LSK_ROWS_WPB;
constexpr int kThreads = kWavesPerBlock * lsk::kWave;
#ifndef LSK_ROWS_BINS
#define LSK_ROWS_BINS 40
#endif
#ifndef LSK_ROWS_MINW
// 7 waves/SIMD: 40 bins keep the LDS at 5.6 KB per wave (28 waves/CU) and the allocator fits
// 72 VGPRs with 4-candidate batches (its spills sit in per-pass code, not in the inner
// loops). 1e8 pts, k=100 (round 1): 5 waves 0.166 s, 6 waves 0.149-0.152 s, 7 waves
// 0.147 s, 8 waves (36 bins) 0.155 s; round 2: 8 waves 0.137 vs 7 waves 0.126 s. The
// final kernel is VALU-issue bound (VALUBusy 74 %, profiles/archive/r2_pmc_final).
#define LSK_ROWS_MINW 7
#endif
// 40 bins of 1/8 octave of d² (kShift0) around the estimate (48 bins: 0.150 s at 6
// waves/SIMD; 36 bins: more refine passes, 0.153 s at 7; 32 bins: 0.225 s).
// Measured on 1e8 uniform points, k=100.
constexpr int kBins = LSK_ROWS_BINS;  // histogram bins (1/8 octave of d² each at kShift0)
static_assert(kBins % 2 == 0 && kBins <= 64, "two 16-bit bins per dword, <= 32 dwords");
// As knn_grid.hip: lanes l and l+32 share a dword (low / high half) of each bin row, so a
// lane's increment is a per-lane constant and every candidate adds without a branch — in
// range to its bin, otherwise to a trash row (kBins) that nothing reads (mixed_scale 2e7
// k=100 77.6 -> 85.8 Mpts/s over exec-masked adds, profiles/r3_rows_hist).
constexpr int kPool = (kBins + 1) * 32;  // dwords per wave: histogram + trash row, or collect pool
// 16 bins (2 octaves of d²) above the estimate: with Hilbert-sorted groups fewer
// overflow retries than 12 (1e8 uniform, k=100: 0.155 vs 0.159 s; 8: 0.179 s)
// (with the blended estimate below: 12 bins = 1.5 octaves; 1e8 uniform, k=100: 8 bins
// 0.137 s with 82K overflow lanes, 10 bins 0.135 s / 6.8K, 12 bins 0.135 s / 623; the
// lane-only estimate needed 16)
#ifndef LSK_TOP_BINS
#define LSK_TOP_BINS 12
#endif
// first-range placement from a blend of the lane estimate and the wave median
#ifndef LSK_EST_CALIB
#define LSK_EST_CALIB 0.8
#endif
// a pass aborts and restarts with finer bins as soon as the bin holding some lane's k-th
// value has more than this many times k entries (0 = off)
#ifndef LSK_CROWD_ABORT
#define LSK_CROWD_ABORT 64
#endif
// walk/process alternation: the walk fills the row queues until every row has this
// many entries pending (then one lockstep drain)
#ifndef LSK_FILL_MIN
#define LSK_FILL_MIN 8
#endif
// Fixed design choices (each measured on 1e8 uniform points, k=100, one MI355X; the
// alternatives were removed once rejected — profiles/archive/r1_*, profiles/archive/r2_kernel):
//  * best-first walk: inner nodes popped in order of their box distance to the centre of
//    the wave's queries from a 64-entry priority list in two VGPRs, a DFS stack as
//    bounded overflow (DFS by bucket-index gap 0.135 s, query-box key 0.129 s, centre
//    key 0.126 s);
//  * the pass-1 log is pruned: (quarter, row) pairs whose pass-1 processing found no
//    value below any lane's bound are dropped before the collect / later replays; the
//    replay appends the logged quarters without re-testing their boxes (re-test 0.169 s);
//  * wave-level box-box prefilter of the 8 quarter tests of a pre-leaf node: one VALU
//    pass (lanes 0-7) decides which quarters need the per-lane tests at all; the accepted
//    set is unchanged (0.147 -> 0.143 s);
//  * candidates in batches of 4 (vs 8: frees the VGPRs of the 7th wave per SIMD);
//  * exec-masked histogram update (5 VALU + ds_add per in-range candidate) with a
//    wave-uniform skip when no lane is in range (0.154 vs 0.159 s);
//  * no entry prefetch (0.129 vs 0.124 s), no early drain of a long row queue.
constexpr int kTopBins = LSK_TOP_BINS;  // bins of the initial range above the estimate
constexpr uint32_t kLogBins = kBins >= 64 ? 6 : kBins >= 32 ? 5 : 4;  // floor(log2(kBins))
#ifndef LSK_ROWS_SHIFT0
#define LSK_ROWS_SHIFT0 20
#endif
constexpr uint32_t kShift0 = LSK_ROWS_SHIFT0;
constexpr uint32_t kMaxPasses = 96;
constexpr uint32_t kGuardRounds = 1u << 22;
// Step budget of a wave (all passes): max(kStepBudget, kStepsPerK * k) row-steps, ~16x
// what a uniform wave takes at k = 100 (~500). A wave beyond it hands its unresolved
// queries to the exact backstop, which runs one wave per query with 64 candidates per
// step: queries next to a dense core far below their own scale (mixed_scale) would
// otherwise stream millions of candidates through ONE wave, pass after pass, while the
// rest of the GPU idles (2e7 points, k = 100: 0.26 s for the whole set).
#ifndef LSK_STEP_BUDGET
#define LSK_STEP_BUDGET 8192
#endif
#ifndef LSK_STEPS_PER_K
#define LSK_STEPS_PER_K 64
#endif
constexpr uint32_t kStepBudget = LSK_STEP_BUDGET;
constexpr uint32_t kStepsPerK = LSK_STEPS_PER_K;

// LSK_PROFILE builds (tuning only) accumulate per-wave shader-clock cycles per activity
// into stats[16..23]: proc hist, proc collect, traverse hist, traverse collect, replay
// hist, replay collect, final select, whole wave.
#ifdef LSK_PROFILE
#define LSK_PT(v) const uint64_t v = __builtin_readcyclecounter()
#define LSK_PADD(acc, t0) (acc) += __builtin_readcyclecounter() - (t0)
#else
#define LSK_PT(v)
#define LSK_PADD(acc, t0)
#endif
constexpr uint32_t kInvalid = 0xffffffffu;
constexpr uint32_t kUnknown = 0xffffffffu;

enum : uint32_t { ST_HIST = 0, ST_READY = 1, ST_DONE = 2 };
enum { MODE_HIST = 0, MODE_COLLECT = 1 };

struct WaveLds {
  uint32_t pool[kPool];
};
// + per-row quarter lists (RCAP entries per row), a kernel template parameter: it sets
// the LDS footprint and so the occupancy
template <int RCAP>
struct WaveLdsR {
  WaveLds w;
  uint32_t rl[4 * RCAP];
};

struct Lane {
  float qx, qy, qz;  // the query (NT == 3: in the trees' rotated frame, for the box tests)
  float ox, oy, oz;  // NT == 3 only: the query's own coordinates (the canonical distances)
  uint32_t state;
  uint32_t lo_b, hi_b, shift;  // histogram range; lo_b = the answer once DONE
  int32_t bin_hi;
  uint32_t c_hi;
  uint32_t c_base;  // exact count of values < lo_b, or kUnknown
  uint32_t nudf;    // underflow retries so far
  uint32_t band_lo, band_w, bc;  // (READY: c_base holds the count below the band)
  uint32_t coff, ccnt;
  // (no separate answer register: once a lane is DONE — or READY and collected — its
  // lo_b is dead and holds the answer bits, see done())
#ifdef LSK_PROFILE
  uint32_t pdead, pslots;  // HIST candidate slots with no lane in range / all slots
  bool pband;              // COLLECT: this lane had a value in its band this step
#endif
};

// Histogram range [lo_b, hi_b) in 64 bins of 2^shift float bits. Values below lo_b are
// counted in bin 0 (saturating bin index), so bin 0 is [0, lo_b + 2^shift); c_base is
// the exact number of values below lo_b when a previous pass established it.
__device__ __forceinline__ void set_range(Lane &s, uint32_t lo_b, uint32_t shift, uint32_t top_limit,
                                          uint32_t c_base) {
  s.lo_b = lo_b;
  s.c_base = lo_b == 0 ? 0u : c_base;
  s.shift = shift;
  uint64_t top = (uint64_t)lo_b + ((uint64_t)kBins << shift);
  uint64_t hi = top < (uint64_t)top_limit ? top : (uint64_t)top_limit;
  s.hi_b = (uint32_t)hi;
  s.bin_hi = hi > lo_b ? (int32_t)((hi - lo_b + ((1ull << shift) - 1)) >> shift) : 0;
  s.c_hi = 0;
}

__device__ __forceinline__ uint32_t hist_read(const uint32_t *pool, uint32_t b, int lane) {
  return (pool[b * 32u + ((uint32_t)lane & 31u)] >> (((uint32_t)lane & 32u) >> 1)) & 0xffffu;
}

typedef __attribute__((address_space(3))) uint32_t lds_u32;
__device__ __forceinline__ uint32_t lds_addr(uint32_t *p) { return (uint32_t)(uintptr_t)(lds_u32 *)p; }
__device__ __forceinline__ void lds_add(uint32_t addr, uint32_t v) {
  __atomic_fetch_add((lds_u32 *)(uintptr_t)addr, v, __ATOMIC_RELAXED);
}

__device__ __forceinline__ uint32_t top_count(const Lane &s, const uint32_t *pool, int lane) {
  return s.bin_hi > 0 ? hist_read(pool, (uint32_t)s.bin_hi - 1u, lane) : s.c_hi;
}

// A crowded k-th bin can be narrowed when shift > 0 (finer bins), or — bin 0 with an
// unknown count below lo_b, the k-th may lie below the range — by one underflow restart.
// Every restart lowers the shift or spends the one underflow: a lane restarts a bounded
// number of times.
__device__ __forceinline__ bool crowd_refinable(const Lane &s) {
  return s.bin_hi >= 2 ? s.shift > 0u
                       : (s.bin_hi == 1 && (s.shift > 0u || (s.c_base == kUnknown && s.nudf == 0)));
}

// Underflow restart: the k-th lies below lo_b (or bin 0 is too coarse to say). First time
// the 5 octaves below the top; again (or a crowded bin 0: the values may lie any number
// of octaves below, e.g. a dense cluster next to a far-off estimate): everything below in
// kBins coarse bins.
__device__ __forceinline__ void underflow_restart(Lane &s, bool coarse) {
  const uint32_t topb = s.hi_b;  // = lo_b + 2^shift, or the clipped top
  if (!coarse && s.nudf == 0 && topb > ((uint32_t)kBins << kShift0)) {
    set_range(s, topb - ((uint32_t)kBins << kShift0), kShift0, topb, kUnknown);
  } else {
    uint32_t sh = 0;
    while (((uint64_t)kBins << sh) < (uint64_t)topb) sh++;
    set_range(s, 0u, sh, topb, 0u);
  }
  s.nudf++;
}

// Returns true when the bin now holding the k-th seen value is CROWDED (more than
// kCrowd values, refinable: shift > 0, not the saturating bin 0): a dense cluster seen
// from outside puts millions of candidates into one 1/8-octave bin, and the walk would
// visit all of them (and overflow the 16-bit bin) before the pass could narrow the range.
__device__ __forceinline__ bool hist_shrink(Lane &s, const uint32_t *pool, int lane, uint32_t k) {
  uint32_t top = 0;
  while (s.bin_hi > 0) {
    top = hist_read(pool, (uint32_t)s.bin_hi - 1u, lane);
    if (s.c_hi - top < k) break;
    s.c_hi -= top;
    s.bin_hi--;
    s.hi_b = s.lo_b + ((uint32_t)s.bin_hi << s.shift);
  }
  // bin 0 of a range starting at 0 with shift 0 holds exactly the d² = +0 values: k of
  // them make the k-th 0 and nothing can be closer — the radius closes (hi_b = 0: every
  // box and candidate is culled), so k + duplicates of a point cost k candidates, not all
  // of them (and bin 0's 16-bit counter cannot overflow)
  if (s.bin_hi == 1 && s.lo_b == 0u && s.shift == 0u && s.c_hi >= k) s.hi_b = 0u;
  return top > (uint32_t)LSK_CROWD_ABORT * k && crowd_refinable(s);
}

// Wave min / max of NON-NEGATIVE floats without LDS round trips: DPP
// reductions inside each 16-lane row (quad_perm [1,0,3,2], [2,3,0,1], row_ror:4,
// row_ror:8), then the four row values combined on the scalar unit (non-negative float
// bits order as unsigned integers). The generic lsk::wave_min is six dependent
// ds_bpermute round trips — on the priority-list pop of every node visit.
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xf, 0xf, false));
}
__device__ __forceinline__ float wave_min_nonneg(float v) {
  v = fminf(v, dpp_f<0xB1>(v));
  v = fminf(v, dpp_f<0x4E>(v));
  v = fminf(v, dpp_f<0x124>(v));
  v = fminf(v, dpp_f<0x128>(v));
  const uint32_t a = (uint32_t)__builtin_amdgcn_readlane(__float_as_int(v), 0);
  const uint32_t b = (uint32_t)__builtin_amdgcn_readlane(__float_as_int(v), 16);
  const uint32_t c = (uint32_t)__builtin_amdgcn_readlane(__float_as_int(v), 32);
  const uint32_t d = (uint32_t)__builtin_amdgcn_readlane(__float_as_int(v), 48);
  return __uint_as_float(min(min(a, b), min(c, d)));
}
__device__ __forceinline__ float wave_max_nonneg(float v) {
  v = fmaxf(v, dpp_f<0xB1>(v));
  v = fmaxf(v, dpp_f<0x4E>(v));
  v = fmaxf(v, dpp_f<0x124>(v));
  v = fmaxf(v, dpp_f<0x128>(v));
  const uint32_t a = (uint32_t)__builtin_amdgcn_readlane(__float_as_int(v), 0);
  const uint32_t b = (uint32_t)__builtin_amdgcn_readlane(__float_as_int(v), 16);
  const uint32_t c = (uint32_t)__builtin_amdgcn_readlane(__float_as_int(v), 32);
  const uint32_t d = (uint32_t)__builtin_amdgcn_readlane(__float_as_int(v), 48);
  return __uint_as_float(max(max(a, b), max(c, d)));
}

// DPP row_newbcast:J — lane J of each 16-lane row to the whole row (folded into the
// consuming VALU op as a DPP source).
template <int J>
__device__ __forceinline__ float rowb(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x150 + J, 0xf, 0xf, false));
}

// Candidate J of the row's quarter (padding lanes hold +inf coordinates: d² = inf,
// which is above every histogram range and collect band).
// NT: tree count of the kernel instance; 3 = one tree built in a rotated frame (the query's
// own coordinates are then s.ox.., s.qx.. being the rotated ones its box tests use).
template <int J, int NT>
__device__ __forceinline__ uint32_t cand(const Lane &s, float px, float py, float pz) {
  const float qx = NT == 3 ? s.ox : s.qx, qy = NT == 3 ? s.oy : s.qy, qz = NT == 3 ? s.oz : s.qz;
  const float d2 = lsk::dist2(qx - rowb<J>(px), qy - rowb<J>(py), qz - rowb<J>(pz));
  return fbits(d2);
}

template <int MODE, int G>
__device__ __forceinline__ bool update8(Lane &s, const uint32_t (&u)[G], uint32_t *pool, int lane,
                                        uint32_t trash) {
  uint32_t umin = u[0];
#pragma unroll
  for (int t = 1; t < G; t++) umin = min(umin, u[t]);
  const bool lane_in = umin < s.hi_b;  // (profiling: this lane had a value in range)
#ifdef LSK_PROFILE
  if (MODE == MODE_HIST) {
#pragma unroll
    for (int t = 0; t < G; t++) s.pdead += __ballot(u[t] < s.hi_b) == 0 ? 1u : 0u;
    s.pslots += G;
  } else {
#pragma unroll
    for (int t = 0; t < G; t++) s.pband = s.pband || (u[t] - s.band_lo < s.band_w);
  }
#endif
  if (MODE == MODE_HIST) {
    if (!__ballot(lane_in)) return false;
    // bin = sat(v - lo_b) >> shift (< 64 for every v < hi_b); bins 2j, 2j+1 share the
    // lane's dword j as two 16-bit counters
    const uint32_t hb = s.hi_b, lb = s.lo_b, sh = s.shift;
    // branch-free: a value below hi_b to its bin, any other to the lane's trash row
    // (`trash`, an opaque per-lane LDS address, so the select is between addresses); the
    // compare also counts c_hi. 6 VALU per candidate, no exec-mask round trip.
    const uint32_t inc = 1u << (((uint32_t)lane & 32u) >> 1);
    const uint32_t row0 = lds_addr(pool) + ((uint32_t)lane & 31u) * 4u;
#pragma unroll
    for (int t = 0; t < G; t++) {
      const uint32_t v = u[t];
      const bool in = v < hb;
      lds_add(in ? row0 + ((__builtin_elementwise_sub_sat(v, lb) >> sh) << 7) : trash, inc);
      s.c_hi += in ? 1u : 0u;
    }
  } else {
    const uint32_t bl = s.band_lo, bw = s.band_w;
    bool any = false;
#pragma unroll
    for (int t = 0; t < G; t++) any = any || (u[t] - bl < bw);
    if (!__ballot(any)) return lane_in;
#pragma unroll
    for (int t = 0; t < G; t++) {
      if (u[t] - bl < bw) {
        if (s.ccnt < s.bc) pool[s.coff + s.ccnt] = u[t];
        s.ccnt++;
      }
    }
  }
  return lane_in;
}

// The 16 candidates of this lane's row quarter (lane i of the row holds candidate i).
template <int MODE, int NT>
__device__ __forceinline__ bool process16(Lane &s, float px, float py, float pz, uint32_t cnt,
                                          uint32_t *pool, int lane, uint32_t trash, uint32_t k, bool &crowd) {
  bool lane_in;
  // groups of 4 candidates: 4 fewer live VGPRs in the hot loop than groups of 8
  {
    uint32_t u[4] = {cand<0, NT>(s, px, py, pz), cand<1, NT>(s, px, py, pz), cand<2, NT>(s, px, py, pz),
                     cand<3, NT>(s, px, py, pz)};
    lane_in = update8<MODE, 4>(s, u, pool, lane, trash);
  }
  {
    uint32_t u[4] = {cand<4, NT>(s, px, py, pz), cand<5, NT>(s, px, py, pz), cand<6, NT>(s, px, py, pz),
                     cand<7, NT>(s, px, py, pz)};
    lane_in = update8<MODE, 4>(s, u, pool, lane, trash) || lane_in;
  }
  if (__ballot(cnt > 8u)) {
    {
      uint32_t u[4] = {cand<8, NT>(s, px, py, pz), cand<9, NT>(s, px, py, pz), cand<10, NT>(s, px, py, pz),
                       cand<11, NT>(s, px, py, pz)};
      lane_in = update8<MODE, 4>(s, u, pool, lane, trash) || lane_in;
    }
    {
      uint32_t u[4] = {cand<12, NT>(s, px, py, pz), cand<13, NT>(s, px, py, pz), cand<14, NT>(s, px, py, pz),
                       cand<15, NT>(s, px, py, pz)};
      lane_in = update8<MODE, 4>(s, u, pool, lane, trash) || lane_in;
    }
  }
  if (MODE == MODE_HIST && __ballot(s.c_hi >= k)) crowd = __ballot(hist_shrink(s, pool, lane, k)) != 0 || crowd;
  return lane_in;
}

struct WaveCtx {
  WaveLds *L;
  uint32_t *rl;
  uint32_t rcap;
  uint32_t trash;  // LDS byte address of this lane's trash-row counter (opaque)
  int lane, row;
  uint32_t k;
  uint32_t g;
  int32_t seed;
  float cx, cy, cz;
  float wlx, wly, wlz, whx, why, whz;  // bounding box of the wave's queries (uniform)
  float rmax2;                         // wave max of the lanes' current bounds (per flush)
  // Row queues are circular (RCAP entries, a power of two) with their own heads: a step
  // consumes the head entry of every row that has one, so a row that got ahead does not
  // force the others to idle until a reset (lockstep idle only when a row is empty).
  uint32_t len0, len1, len2, len3;  // row queue tails = entries appended (wave-uniform)
  uint32_t hd0, hd1, hd2, hd3;      // row queue heads = entries consumed (wave-uniform)
  uint32_t rlen, rhead;             // this lane's row's tail / head (per lane; no select
                                    // chain: the compiler turns one into a scratch table)
  // pass-1 log of the visited pre-leaf nodes: entry n = (first quarter | tree << 31,
  // 4 row bits per quarter) held by lane n % 64 of word n / 64 of two private arrays
  uint32_t logn;
  bool logging, log_ok;
  bool crowd;  // a lane's k-th bin got crowded: abort the pass (see hist_shrink)
  // pass-1 "dead row-step" stream: bit h of row r (lane 16r + h/32, bit h%32) is set when
  // the row's h-th queue entry gave no lane of the row a value below its bound; after
  // pass 1 those (quarter, row) pairs are removed from the log (they cannot hold a value
  // below any later bound or inside the collect band: bounds only shrink)
  uint32_t *dead;  // private (scratch) word: keeps the stream out of the VGPR budget
  uint32_t nseed;  // seed quarters appended to every row before the logged ones
  uint32_t *logq, *logm;
  const float *p0, *p1, *pdef;  // tree point arrays (pdef: one that is non-empty)
  uint32_t n0, n1;
  uint32_t guard;  // bit 0: watchdog trip of the walk (never expected; see traverse);
                   // bit 1: the wave's step budget ran out (kStepBudget)
#ifdef LSK_PROFILE
  uint64_t prof[8];
  uint32_t prof_rows_entry, prof_rows_in;  // pass-1 row-steps with an entry / with a value in range
  uint32_t prof_crows_entry, prof_crows_in;  // collect row-steps with an entry / with a band value
#endif
  uint32_t steps, quarters, nodes_visited, csteps, cnodes;
};

// pending (appended, not yet processed) entries of the longest / shortest row queue
__device__ __forceinline__ uint32_t max_pend(const WaveCtx &W) {
  return max(max(W.len0 - W.hd0, W.len1 - W.hd1), max(W.len2 - W.hd2, W.len3 - W.hd3));
}
__device__ __forceinline__ uint32_t min_pend(const WaveCtx &W) {
  return min(min(W.len0 - W.hd0, W.len1 - W.hd1), min(W.len2 - W.hd2, W.len3 - W.hd3));
}

__device__ __forceinline__ lsk_tree_view pick_tree(const lsk_knn_args &A, uint32_t t) {
  return t ? A.tree[1] : A.tree[0];
}

// Entry = (tree << 31) | quarter id. Loads this lane's candidate of its row's quarter.
// Branch-free (the load is always issued, from a clamped in-bounds address), so the
// compiler can count outstanding loads and the prefetch is not serialised by vmcnt(0).
// 32-bit index math (trees hold < 2^31 points, checked on the host).
// NT = number of trees the kernel instance handles (1: no per-lane tree selects; 3: one
// tree in a rotated frame).
template <int NT>
__device__ __forceinline__ uint32_t load_quarter(const WaveCtx &W, uint32_t e, float &px, float &py,
                                                 float &pz) {
  const bool ok = e != kInvalid;
  const bool t1 = NT == 2 && (e >> 31) != 0;
  const uint32_t n = t1 ? W.n1 : W.n0;
  const uint32_t q16 = (e & 0x7fffffffu) << 4;
  const uint32_t idx = q16 | (uint32_t)(W.lane & 15);
  const bool live = ok && idx < n;
  // dead lanes read point 0 of a non-empty tree
  const float *p = NT != 2 ? W.p0 + 3u * (live ? idx : 0u)
                           : (live ? (t1 ? W.p1 : W.p0) + 3u * idx : W.pdef);
  px = p[0];  // raw: the consumer substitutes +inf for padding lanes (see process_steps)
  py = p[1];
  pz = p[2];
  return ok ? min(n - q16, 16u) : 0u;
}

// Entry number `h` of this lane's row queue (kInvalid past the tail).
__device__ __forceinline__ uint32_t row_entry(const WaveCtx &W, uint32_t h) {
  const uint32_t v = W.rl[(uint32_t)W.row * W.rcap + (h & (W.rcap - 1u))];
  return h < W.rlen ? v : kInvalid;
}

__device__ __forceinline__ uint32_t row_bits(uint64_t ballot) {
  return ((ballot & 0xffffull) ? 1u : 0u) | ((ballot & 0xffff0000ull) ? 2u : 0u) |
         ((ballot & 0xffff00000000ull) ? 4u : 0u) | ((ballot & 0xffff000000000000ull) ? 8u : 0u);
}

// n lockstep steps: every row consumes its head entry (rows with an empty queue idle).
template <int MODE, int NT>
__device__ __forceinline__ void process_steps(Lane &s, WaveCtx &W, const lsk_knn_args &A,
                                              uint32_t n) {
  n = lsk::uniform(n);  // wave-uniform loop (lets the compiler keep it scalar)
  if (n == 0) return;
  // one step of prefetch; loads are unconditional (the entry after the last step is
  // fetched too, harmlessly) so no branch breaks the compiler's count of outstanding loads
  float px, py, pz;
  uint32_t cnt = load_quarter<NT>(W, row_entry(W, W.rhead), px, py, pz);
  // (two steps of prefetch: 0.155 vs 0.152 s at 6 waves/SIMD with 10 spilled VGPRs,
  // 0.166 s at 5 waves/SIMD — occupancy, not the candidate-load distance, is what counts)
  const float inf = __builtin_inff();
  for (uint32_t st = 0; st < n; st++) {
    const uint32_t ccnt = cnt;
    const uint32_t hcur = W.rhead;  // queue position of the entry processed by this step
    const bool live = (uint32_t)(W.lane & 15) < ccnt;
    const float cx = live ? px : inf, cy = live ? py : inf, cz = live ? pz : inf;
    W.rhead += W.rhead < W.rlen ? 1u : 0u;
    cnt = load_quarter<NT>(W, row_entry(W, W.rhead), px, py, pz);
    W.steps++;
    if (MODE == MODE_COLLECT) W.csteps++;
#ifdef LSK_PROFILE
    s.pband = false;
#endif
    const bool lin = process16<MODE, NT>(s, cx, cy, cz, ccnt, W.L->pool, W.lane, W.trash, W.k, W.crowd);
    if (W.steps >= max(kStepBudget, kStepsPerK * W.k)) W.guard |= 2u;
#ifdef LSK_PROFILE
    if (MODE == MODE_HIST) {
      const uint32_t re = row_bits(__ballot(ccnt > 0u)), ri = row_bits(__ballot(lin));
      W.prof_rows_entry += __popc(re);
      W.prof_rows_in += __popc(re & ri);
    } else {
      const uint32_t re = row_bits(__ballot(ccnt > 0u)), ri = row_bits(__ballot(s.pband));
      W.prof_crows_entry += __popc(re);
      W.prof_crows_in += __popc(re & ri);
    }
#endif
    if (MODE == MODE_HIST && W.logging) {
      const uint32_t rin = row_bits(__ballot(lin)), rent = row_bits(__ballot(ccnt > 0u));
      const uint32_t dead = ((rent & ~rin) >> W.row) & 1u;
      if (dead && hcur < 512u && (uint32_t)(W.lane & 15) == (hcur >> 5))
        W.dead[hcur >> 9] |= 1u << (hcur & 31u);  // (index 0: dynamic, so it stays in scratch)
    }
    if ((MODE == MODE_HIST && W.crowd) || W.guard) break;  // crowded bin: the pass restarts narrower
  }
  W.hd0 = min(W.hd0 + n, W.len0);
  W.hd1 = min(W.hd1 + n, W.len1);
  W.hd2 = min(W.hd2 + n, W.len2);
  W.hd3 = min(W.hd3 + n, W.len3);
}

__device__ __forceinline__ float hist_bound(const Lane &s) { return bitsf(s.hi_b); }

// per-lane need of a box in a given mode. HIST: closer than the lane's radius; COLLECT:
// box cuts the lane's shell [band_lo, band_hi) (max-distance is monotone, common.h).
template <int MODE>
__device__ __forceinline__ bool box_needed(const Lane &s, float lx, float ly, float lz, float hx,
                                           float hy, float hz) {
  const lsk::vec3f q{s.qx, s.qy, s.qz};
  if (MODE == MODE_HIST) return lsk::box_dist2(q, {lx, ly, lz}, {hx, hy, hz}) < hist_bound(s);
  if (s.band_w == 0) return false;
  const bool near = lsk::box_dist2(q, {lx, ly, lz}, {hx, hy, hz}) < bitsf(s.band_lo + s.band_w);
  const float fx = fmaxf(fabsf(lx - s.qx), fabsf(hx - s.qx));
  const float fy = fmaxf(fabsf(ly - s.qy), fabsf(hy - s.qy));
  const float fz = fmaxf(fabsf(lz - s.qz), fabsf(hz - s.qz));
  return near && fbits(lsk::dist2(fx, fy, fz)) >= s.band_lo;
}

// Box kept by a replay filter: any future use (HIST lanes: radius, READY lanes: shell).
template <int MODE>
__device__ __forceinline__ bool box_retained(const Lane &s, float lx, float ly, float lz, float hx,
                                             float hy, float hz) {
  if (MODE == MODE_COLLECT) return box_needed<MODE_COLLECT>(s, lx, ly, lz, hx, hy, hz);
  if (s.state == ST_HIST) return box_needed<MODE_HIST>(s, lx, ly, lz, hx, hy, hz);
  if (s.state == ST_READY) return box_needed<MODE_COLLECT>(s, lx, ly, lz, hx, hy, hz);
  return false;
}


// Append entry e to the lists of the rows in rowmask: the leader lane of each such row
// writes at its row's length (one vector LDS store), the lengths stay scalar.
__device__ __forceinline__ void rows_append(WaveCtx &W, uint32_t rowmask, uint32_t e) {
  const uint32_t mine = (rowmask >> W.row) & 1u;
  if ((W.lane & 15) == 0 && mine) W.rl[(uint32_t)W.row * W.rcap + (W.rlen & (W.rcap - 1u))] = e;
  W.rlen += mine;
  W.len0 += rowmask & 1u;
  W.len1 += (rowmask >> 1) & 1u;
  W.len2 += (rowmask >> 2) & 1u;
  W.len3 += (rowmask >> 3) & 1u;
  W.quarters += __popc(rowmask);
}

// Quarter boxes of up to kPend pre-leaf nodes (8 quarters = 64 floats each, one dword
// per lane) are loaded together — one memory latency per batch instead of per node —
// and broadcast with v_readlane for the per-row tests.
#ifndef LSK_PEND
#define LSK_PEND 4
#endif
constexpr uint32_t kPend = LSK_PEND;
constexpr uint32_t kLogWords = 8;  // log capacity 512 pre-leaf entries (private memory)
constexpr uint32_t kLogCap = kLogWords * 64;

__device__ __forceinline__ float lanef(float v, uint32_t l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), (int)l));
}

// One pre-leaf node's 8 quarters, already loaded one float per lane in `blk`; lmask
// restricts the rows per quarter (4 bits each; all ones for a walk). Returns the rows
// that took each quarter (same layout).
template <int MODE>
__device__ __forceinline__ uint32_t test_block(Lane &s, WaveCtx &W, float blk, uint32_t t, uint32_t q0,
                                               uint32_t lmask, uint32_t nquarters, int64_t skip_lo,
                                               int64_t skip_hi) {
  uint32_t took = 0;
  // wave-level prefilter: lane j < 8 tests quarter j's box against the box of the wave's
  // queries and the largest lane bound (box-box distance <= every query's box distance,
  // so a quarter some lane needs always passes); the exact per-lane tests then run only
  // for the quarters that pass
  uint32_t pm;
  {
    const int src = (W.lane & 7) * 8;
    const float qlx = __shfl(blk, src), qly = __shfl(blk, src + 1), qlz = __shfl(blk, src + 2);
    const float qhx = __shfl(blk, src + 4), qhy = __shfl(blk, src + 5), qhz = __shfl(blk, src + 6);
    const lsk::box3f wb{{W.wlx, W.wly, W.wlz}, {W.whx, W.why, W.whz}};
    const lsk::box3f qb{{qlx, qly, qlz}, {qhx, qhy, qhz}};
    pm = (uint32_t)__ballot(W.lane < 8 && lsk::box_box_dist2(wb, qb) < W.rmax2) & 0xffu;
  }
#pragma unroll
  for (uint32_t j = 0; j < 8; j++) {
    const uint32_t qid = q0 + j;
    const int64_t b = (int64_t)(qid >> 2);
    const uint32_t lm = (lmask >> (4 * j)) & 0xfu;
    if (lm == 0 || qid >= nquarters || (b >= skip_lo && b <= skip_hi)) continue;
    if (!((pm >> j) & 1u)) continue;
    const float lx = lanef(blk, 8 * j), ly = lanef(blk, 8 * j + 1), lz = lanef(blk, 8 * j + 2);
    const float hx = lanef(blk, 8 * j + 4), hy = lanef(blk, 8 * j + 5), hz = lanef(blk, 8 * j + 6);
    const uint32_t rm = row_bits(__ballot(box_needed<MODE>(s, lx, ly, lz, hx, hy, hz))) & lm;
    rows_append(W, rm, (t << 31) | qid);
    took |= rm << (4 * j);
  }
  return took;
}

__device__ __forceinline__ void log_put(WaveCtx &W, uint32_t e, uint32_t mask) {
  if (W.logn >= kLogCap) {
    W.log_ok = false;
    return;
  }
  const uint32_t slot = W.logn >> 6;
  if (W.lane == (int)(W.logn & 63u)) {
    W.logq[slot] = e;
    W.logm[slot] = mask;
  }
  W.logn++;
}

// Pending pre-leaf nodes p[0..kPend) (first quarter ids; scalars — an indexed array
// would live in scratch).
struct Pend {
  uint32_t p0, p1, p2, p3, n;
  uint32_t m0, m1, m2, m3;  // row masks (replay; all ones for a walk)
};

template <int MODE>
__device__ __forceinline__ void flush_pending(Lane &s, WaveCtx &W, const float *qf, uint32_t t,
                                              const Pend &P, uint32_t nquarters, int64_t skip_lo,
                                              int64_t skip_hi, uint32_t qfloats) {
  const uint32_t l = (uint32_t)W.lane, last = qfloats - 1u;
  {
    const float bnd = MODE == MODE_HIST ? hist_bound(s) : (s.band_w ? bitsf(s.band_lo + s.band_w) : 0.f);
    W.rmax2 = wave_max_nonneg(bnd);
  }
  // all loads first (one latency for the batch), then the tests
#define LSK_LD(i) const float b##i = qf[min((P.n > i ? P.p##i : P.p0) * 8u + l, last)];
  LSK_LD(0) LSK_LD(1) LSK_LD(2) LSK_LD(3)
#undef LSK_LD
#define LSK_TB(i)                                                                          \
  if (P.n > i) {                                                                           \
    const uint32_t took = test_block<MODE>(s, W, b##i, t, P.p##i, P.m##i, nquarters, skip_lo, \
                                           skip_hi);                                     \
    if (W.logging && took) log_put(W, P.p##i | (t << 31), took);                           \
  }
  LSK_TB(0) LSK_TB(1) LSK_TB(2) LSK_TB(3)
#undef LSK_TB
}

__device__ __forceinline__ uint32_t ubits(float v) {  // uniform, order-preserving for v >= 0
  return (uint32_t)__builtin_amdgcn_readfirstlane((int)__float_as_uint(v));
}

// Drop from the pass-1 log every (quarter, row) pair whose pass-1 step gave no lane of the
// row a value below its bound (WaveCtx::dead). Row r's queue held the seeds first, then
// the logged quarters in log order (quarter order inside an entry), so the stream index
// of a logged pair is nseed + (row-r pairs in earlier entries) + (row-r pairs of earlier
// quarters of the same entry). One 64-entry log word per iteration, all lanes at once.
// Out of line with scalar arguments: WaveCtx stays in registers and the prune's own
// temporaries do not raise the kernel's register pressure (0.1245 s; out of line taking
// WaveCtx& forces WaveCtx to scratch: 0.127 s; inlined: 0.149 s).
__device__ __attribute__((noinline)) void log_prune_impl(uint32_t *logm, uint32_t logn, uint32_t dw,
                                                          uint32_t nseed, int lane) {
  uint32_t base01 = 0, base23 = 0;  // row pairs before this word (rows 0|1, 2|3: 16-bit fields)
#pragma unroll 1
  for (uint32_t w = 0; w < kLogWords; w++) {
    if ((w << 6) >= logn) break;
    const bool have = (w << 6) + (uint32_t)lane < logn;
    const uint32_t mk = have ? logm[w] : 0u;
    const uint32_t c01 = __popc(mk & 0x11111111u) | (__popc(mk & 0x22222222u) << 16);
    const uint32_t c23 = __popc(mk & 0x44444444u) | (__popc(mk & 0x88888888u) << 16);
    uint32_t x01 = c01, x23 = c23;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y01 = __shfl_up(x01, o), y23 = __shfl_up(x23, o);
      if (lane >= o) {
        x01 += y01;
        x23 += y23;
      }
    }
    const uint32_t e01 = base01 + x01 - c01, e23 = base23 + x23 - c23;  // exclusive
    uint32_t keep = mk;
#pragma unroll 1
    for (uint32_t b = 0; b < 32; b++) {  // bit b: quarter b / 4, row b % 4
      const uint32_t r = b & 3u;
      const uint32_t prev = ((r < 2u ? e01 : e23) >> (16u * (r & 1u))) & 0xffffu;
      const uint32_t idx = nseed + prev + (uint32_t)__popc(mk & (0x11111111u << r) & ((1u << b) - 1u));
      const uint32_t word = (uint32_t)__shfl((int)dw, (int)(16u * r + min(idx >> 5, 15u)));
      if (((mk >> b) & 1u) && idx < 512u && ((word >> (idx & 31u)) & 1u)) keep &= ~(1u << b);
    }
    if (have) logm[w] = keep;
    base01 += (uint32_t)__shfl((int)x01, 63);
    base23 += (uint32_t)__shfl((int)x23, 63);
  }
}
__device__ __forceinline__ void log_prune(WaveCtx &W) {
  log_prune_impl(W.logm, W.logn, W.dead[0], W.nseed, W.lane);
}

// Tree walk (wave-uniform DFS, near child first) building the per-row quarter lists,
// alternating with lockstep processing of what every row has pending (one processing
// call site per pass keeps the kernel's register allocation tight).
//  * 4-ary steps: a popped node at level l tests its four grandchildren (level l+2,
//    contiguous in the implicit tree: one 128-byte scalar load) — half the dependent
//    pop -> load -> test rounds of a binary walk; a binary step lands on level depth-1
//    when needed. Nodes at level depth-1 test the 8 quarter boxes of their two buckets
//    directly (one 256-byte load), so buckets are never pushed.
//  * Seeding: tree 0's buckets [g-seed, g+seed] are queued for every row first and
//    skipped by the walk.
//  * A list that would overflow forces a drain and a reset (replay then disabled).
//  * replay (pass > 1 with a complete pass-1 log): the pre-leaf nodes and per-quarter
//    row masks come from the log instead of the walk (bounds only shrink after pass 1,
//    so the log is a superset of what later passes need).
template <int MODE, bool replay, int NT>
__device__ __forceinline__ void traverse(Lane &s, WaveCtx &W, const lsk_knn_args &A) {
  const lsk::vec3f q{s.qx, s.qy, s.qz};
  const lsk::vec3f c{W.cx, W.cy, W.cz};
  W.len0 = W.len1 = W.len2 = W.len3 = W.rlen = 0;
  W.hd0 = W.hd1 = W.hd2 = W.hd3 = W.rhead = 0;
  uint32_t t = 0, sp = 0;
  // DFS stack in one VGPR (lane i = entry i; < 64 entries): v_readlane to pop, a
  // lane select to push, instead of an LDS round trip per node
  uint32_t stk = 0;
  // priority list: lane i holds (node, key) entry i; empty = (any, +inf); npq entries
  uint32_t pqn = 0u;
  float pqk = __builtin_inff();
  uint32_t npq = 0;
  const lsk::box3f wbox{{W.wlx, W.wly, W.wlz}, {W.whx, W.why, W.whz}};
  // a node popped from the DFS stack pushes its children back onto the stack (depth-first
  // inside an overflowed subtree), and the stack is drained before the list is popped
  // again: the stack then never holds more than 4 + 3 per level entries (< 64), while
  // the list holds at most 64
  bool dfs_mode = false;
  auto pq_push = [&](uint32_t cn, lsk::v4f lo, lsk::v4f hi) {
    if (!dfs_mode && npq < 64u) {
      // key: squared distance from the wave's query-box centre to the node box
      const float key = lsk::uniform_f(lsk::box_dist2(c, {lo.x, lo.y, lo.z}, {hi.x, hi.y, hi.z}));
      const uint64_t fr = __ballot(pqk == __builtin_inff());
      const int l = (int)__builtin_ctzll(fr);
      if (W.lane == l) {
        pqn = cn;
        pqk = key < __builtin_inff() ? key : 3.0e38f;  // never store the empty marker
      }
      npq++;
    } else {
      stk = W.lane == (int)sp++ ? cn : stk;
    }
  };
  bool started = false, finished = false;
  int32_t seed_d = W.seed > 0 ? 0 : -1;  // next seed distance (tree 0 only)
  lsk_tree_view T = pick_tree(A, 0);
  uint32_t nquarters = 0, nbuckets = 0;
  int32_t depth = 0;
  int64_t skip_lo = 1, skip_hi = 0;
  uint32_t fill_rounds = 0;
  Pend P{0, 0, 0, 0, 0, ~0u, ~0u, ~0u, ~0u};  // pending pre-leaf nodes
  uint32_t ri = 0, lq = 0, lmk = 0;  // replay cursor, cached log words
  bool force_flush = false;           // replay: a tree switch needs the batch flushed
  if (!replay && W.logging) {
    W.logn = 0;
    W.dead[0] = 0;
    W.nseed = 0;
  }
  while (!finished) {
    bool overflow = false;
    if (++fill_rounds > kGuardRounds) {  // watchdog: never spin on the GPU
      W.guard |= 1u;
      break;
    }
    // ---- fill until every row has a batch pending, a list is nearly full or the walk ends
    for (;;) {
      // room for the pending batch (8 entries per node per row) plus one more node
      const bool room_short = max_pend(W) + 8u * (P.n + 1u) > W.rcap;
      const bool walk_empty = sp == 0 && npq == 0;
      if (P.n && (P.n == kPend || room_short || (started && walk_empty) || force_flush ||
                  (replay && ri >= W.logn))) {
        force_flush = false;
        LSK_PT(tq0);  // the one flush site (keeps a single inlined copy)
        flush_pending<MODE>(s, W, T.qnodes, t, P, nquarters, skip_lo, skip_hi, 32u << depth);
        LSK_PADD(W.prof[4], tq0);
        P.n = 0;
        continue;
      }
      if (room_short) {
        overflow = true;
        break;
      }
      if (min_pend(W) >= (uint32_t)LSK_FILL_MIN) break;
      if (!started) {
        if (t >= (uint32_t)A.ntrees) {
          finished = true;
          break;
        }
        T = pick_tree(A, t);
        if (T.n <= 0) {
          t++;
          continue;
        }
        depth = T.depth;
        nquarters = (uint32_t)((T.n + 15) / 16);
        nbuckets = (uint32_t)((T.n + lsk::kBucket - 1) / lsk::kBucket);
        skip_lo = 1;
        skip_hi = 0;
        if (t == 0 && W.seed > 0) {
          skip_lo = (int64_t)W.g - W.seed;
          skip_hi = (int64_t)W.g + W.seed;
        }
        if (W.lane == 0) {  // the root enters the priority list
          pqn = 1u;
          pqk = 0.f;
        }
        npq = 1;
        started = true;
      }
      if (t == 0 && seed_d >= 0) {  // seed buckets g, g-1, g+1, g-2, g+2, ... for every row
        for (int32_t sgn = 0; sgn < (seed_d ? 2 : 1); sgn++) {
          const int64_t b = sgn ? (int64_t)W.g + seed_d : (int64_t)W.g - seed_d;
          if (b < 0 || b >= (int64_t)nbuckets) continue;
          for (uint32_t qq = 0; qq < 4; qq++) {
            const uint32_t qid = (uint32_t)b * 4 + qq;
            if (qid < nquarters) {
              rows_append(W, 0xfu, qid);
              if (!replay) W.nseed++;
            }
          }
        }
        seed_d = seed_d < W.seed ? seed_d + 1 : -1;
        continue;
      }
      if (replay) {
        if (ri >= W.logn) {  // (nothing pending here: flushed above)
          finished = true;
          break;
        }
        if ((ri & 63u) == 0) {  // next 64 log entries, one per lane
          lq = W.logq[ri >> 6];
          lmk = W.logm[ri >> 6];
        }
        const uint32_t e = __builtin_amdgcn_readlane(lq, (int)(ri & 63u));
        const uint32_t mk = __builtin_amdgcn_readlane(lmk, (int)(ri & 63u));
        const uint32_t tq = e & 0x80000000u, q0 = e & 0x7fffffffu;
        // the logged rows per quarter are appended as they are: they are a superset of
        // what any later pass needs (bounds only shrink), and skipping the re-test keeps
        // replay free of box loads
#pragma unroll
        for (uint32_t j = 0; j < 8; j++) {
          const uint32_t rm = (mk >> (4 * j)) & 0xfu;
          if (rm) rows_append(W, rm, tq | (q0 + j));
        }
        ri++;
        continue;
      }
      if (sp == 0 && npq == 0) {  // (nothing pending here: flushed above)
        t++;
        started = false;
        continue;
      }
      uint32_t node;
      dfs_mode = sp != 0;
      if (!dfs_mode) {
        const float m = wave_min_nonneg(pqk);
        const int l = (int)__builtin_ctzll(__ballot(pqk == m));
        node = __builtin_amdgcn_readlane(pqn, l);
        if (W.lane == l) pqk = __builtin_inff();
        npq--;
      } else {
        sp--;
        node = __builtin_amdgcn_readlane(stk, (int)sp);
      }
      W.nodes_visited++;
      if (MODE == MODE_COLLECT) W.cnodes++;
      const int32_t lvl = 31 - __clz(node);
      if (lvl == depth - 1 || depth == 0) {  // two buckets = 8 quarters (depth 0: the root)
        const uint32_t q0 = depth == 0 ? 0u : (node - (1u << lvl)) * 8u;
        P.p0 = P.n == 0 ? q0 : P.p0;
        P.p1 = P.n == 1 ? q0 : P.p1;
        P.p2 = P.n == 2 ? q0 : P.p2;
        P.p3 = P.n == 3 ? q0 : P.p3;
        P.n++;
        continue;
      }
      LSK_PT(tn0);
      lsk::cfloat4_p nodes = lsk::as_const4(T.nodes);
      const float lim = MODE == MODE_HIST ? hist_bound(s)
                                          : (s.band_w ? bitsf(s.band_lo + s.band_w) : 0.f);
      if (lvl + 2 <= depth - 1) {
        const uint32_t g0 = 4u * node;
        // bucket-index gap of each child's subtree to the wave's own bucket (the DFS
        // visiting order before the best-first walk; unused, kept for an identical build)
        const uint32_t csh = (uint32_t)(depth - lvl - 2);
        auto korder = [&](uint32_t ch, uint32_t j) -> uint32_t {
          if (t != 0) return 3u - j;
          const uint32_t b0 = (ch - (1u << (lvl + 2))) << csh, b1 = b0 + (1u << csh);
          const uint32_t gap = W.g < b0 ? b0 - W.g : (W.g >= b1 ? W.g - b1 + 1u : 0u);
          return (min(gap, 0x3fffffffu) << 2) | j;
        };
        // test the 4 grandchildren; key = (center distance bits & ~3) | index, so the
        // nearest is pushed last (popped first); scalar variables only (no arrays: an
        // array here ends up in scratch and makes the stack index divergent)
        uint32_t need = 0, k0, k1, k2, k3;
        {
          const lsk::v4f lo = nodes[2 * g0], hi = nodes[2 * g0 + 1];
          const lsk::vec3f bl{lo.x, lo.y, lo.z}, bh{hi.x, hi.y, hi.z};
          need |= __ballot(lsk::box_dist2(q, bl, bh) < lim) != 0 ? 1u : 0u;
          k0 = korder(g0 + 0u, 0u);
        }
        {
          const lsk::v4f lo = nodes[2 * g0 + 2], hi = nodes[2 * g0 + 3];
          const lsk::vec3f bl{lo.x, lo.y, lo.z}, bh{hi.x, hi.y, hi.z};
          need |= __ballot(lsk::box_dist2(q, bl, bh) < lim) != 0 ? 2u : 0u;
          k1 = korder(g0 + 1u, 1u);
        }
        {
          const lsk::v4f lo = nodes[2 * g0 + 4], hi = nodes[2 * g0 + 5];
          const lsk::vec3f bl{lo.x, lo.y, lo.z}, bh{hi.x, hi.y, hi.z};
          need |= __ballot(lsk::box_dist2(q, bl, bh) < lim) != 0 ? 4u : 0u;
          k2 = korder(g0 + 2u, 2u);
        }
        {
          const lsk::v4f lo = nodes[2 * g0 + 6], hi = nodes[2 * g0 + 7];
          const lsk::vec3f bl{lo.x, lo.y, lo.z}, bh{hi.x, hi.y, hi.z};
          need |= __ballot(lsk::box_dist2(q, bl, bh) < lim) != 0 ? 8u : 0u;
          k3 = korder(g0 + 3u, 3u);
        }
        need = (uint32_t)__builtin_amdgcn_readfirstlane((int)need);
        (void)k0; (void)k1; (void)k2; (void)k3;
        for (uint32_t j = 0; j < 4u; j++)
          if ((need >> j) & 1u) {
            const lsk::v4f lo = nodes[2 * (g0 + j)], hi = nodes[2 * (g0 + j) + 1];
            pq_push(g0 + j, lo, hi);
          }
      } else {  // binary step onto level depth-1
        const uint32_t c0 = 2 * node, c1 = c0 + 1;
        const lsk::v4f l0 = nodes[2 * c0], h0 = nodes[2 * c0 + 1];
        const lsk::v4f l1 = nodes[2 * c1], h1 = nodes[2 * c1 + 1];
        const bool n0 = __ballot(lsk::box_dist2(q, {l0.x, l0.y, l0.z}, {h0.x, h0.y, h0.z}) < lim) != 0;
        const bool n1 = __ballot(lsk::box_dist2(q, {l1.x, l1.y, l1.z}, {h1.x, h1.y, h1.z}) < lim) != 0;
        // near child first: the one whose buckets contain / precede the wave's bucket
        const uint32_t mid = ((c1 - (1u << (lvl + 1))) << (uint32_t)(depth - lvl - 1));
        const bool first0 = t != 0 || W.g < mid;
        const uint32_t a = first0 ? c1 : c0, bb = first0 ? c0 : c1;
        const bool na = first0 ? n1 : n0, nbb = first0 ? n0 : n1;
        (void)a; (void)bb; (void)na; (void)nbb;
        if (n0) pq_push(c0, l0, h0);
        if (n1) pq_push(c1, l1, h1);
      }
      LSK_PADD(W.prof[5], tn0);
    }
    // ---- drain (single processing call site)
    // fill: the steps every row can take; overflow: at least enough to make room for one
    // more node's 8 quarters in the longest queue; end of walk: everything pending
    const uint32_t mxp = max_pend(W), mnp = min_pend(W);
    const uint32_t nsteps = finished ? mxp : overflow ? max(mnp, mxp + 8u - min(mxp + 8u, W.rcap)) : mnp;
    LSK_PT(tp0);
    process_steps<MODE, NT>(s, W, A, nsteps);
    LSK_PADD(W.prof[MODE], tp0);
    if ((MODE == MODE_HIST && W.crowd) || W.guard) break;  // aborted pass (the caller restarts it)
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

__device__ __forceinline__ float bcast64(float v, uint32_t j) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), (int)j));
}

// Local dimension of a group (64 curve-consecutive points) from the shape of its
// covariance C, scaled to trace 1: 3-D groups keep det(C) >= ~1e-3 (uniform, clustered,
// mixed-scale data: 99.99 % of groups >= 3.5e-3, worst 7e-7), points on a plane give
// det ~ 0 (<= 2e-11 tilted, exactly 0 axis-aligned) and points on a line also give the sum
// of the 2x2 principal minors ~ 0 (<= 7e-9; planes >= 1e-4). 3, 2 or 1.
#ifndef LSK_DIM2_MIN
#define LSK_DIM2_MIN 1e-5
#endif
__device__ __forceinline__ uint32_t group_dimension(const Lane &s, bool valid, uint32_t nvalid) {
  const float inv = 1.f / (float)(nvalid > 0 ? nvalid : 1u);
  const float mx = lsk::wave_sum_f(valid ? s.qx : 0.f) * inv, my = lsk::wave_sum_f(valid ? s.qy : 0.f) * inv,
              mz = lsk::wave_sum_f(valid ? s.qz : 0.f) * inv;
  const float dx = valid ? s.qx - mx : 0.f, dy = valid ? s.qy - my : 0.f, dz = valid ? s.qz - mz : 0.f;
  float cxx = lsk::wave_sum_f(dx * dx), cyy = lsk::wave_sum_f(dy * dy), czz = lsk::wave_sum_f(dz * dz);
  float cxy = lsk::wave_sum_f(dx * dy), cxz = lsk::wave_sum_f(dx * dz), cyz = lsk::wave_sum_f(dy * dz);
  const float tr = cxx + cyy + czz;
  if (!(tr > 0.f) || !(tr < __builtin_inff())) return 3u;
  const float it = 1.f / tr;
  cxx *= it; cyy *= it; czz *= it; cxy *= it; cxz *= it; cyz *= it;
  const float m_xy = cxx * cyy - cxy * cxy, m_xz = cxx * czz - cxz * cxz, m_yz = cyy * czz - cyz * cyz;
  const float det = cxx * m_yz - cxy * (cxy * czz - cyz * cxz) + cxz * (cxy * cyz - cyy * cxz);
  if (det >= 1e-6f) return 3u;
  // (LSK_DIM2_MIN, round 6: 1e-2 / 1e-3 classify a line of float-quantised points — its
  // coordinates rounded by up to half an ulp across it, ~1e-3 here — as 1-D: 2e7 line,
  // k = 100, 702 -> 785 / 746 Mpts/s, but clustered 594 -> 405 / 410: groups that straddle
  // a curve discontinuity between two clumps look like lines too and get the 1-D scale;
  // kept at 1e-5, profiles/r6_nonuniform/)
  return m_xy + m_xz + m_yz >= (float)LSK_DIM2_MIN ? 2u : 1u;
}

__device__ __forceinline__ float own_group_estimate(const Lane &s, uint32_t nvalid, uint32_t k,
                                                     bool &dup) {
#ifndef LSK_EST_M
#define LSK_EST_M 8
#endif
  constexpr int M = LSK_EST_M;  // nearest group members kept for the estimate
  float best[M];
#pragma unroll
  for (int i = 0; i < M; i++) best[i] = __builtin_inff();
  for (uint32_t j0 = 0; j0 < nvalid; j0 += 8) {
#pragma unroll
    for (int t = 0; t < 8; t++) {
      const uint32_t j = j0 + (uint32_t)t;
      float v = lsk::dist2(s.qx - bcast64(s.qx, j), s.qy - bcast64(s.qy, j), s.qz - bcast64(s.qz, j));
      v = (j < nvalid) ? v : __builtin_inff();
#pragma unroll
      for (int i = 0; i < M; i++) {
        const float lo = fminf(best[i], v);
        v = fmaxf(best[i], v);
        best[i] = lo;
      }
    }
  }
  dup = best[1] == 0.f;  // an exact copy of the query besides itself
  const uint32_t m0 = k < (uint32_t)M ? k : (uint32_t)M;
  float dm = best[0];
#pragma unroll
  for (int i = 1; i < M; i++) dm = (i + 1 == (int)m0) ? best[i] : dm;
  return dm * cbrtf(((float)k / (float)m0) * ((float)k / (float)m0));
}

enum : uint32_t {
  QS_OVERFLOW = 1, QS_UNDERFLOW = 2, QS_REFINE = 4, QS_LIST_INVALID = 8, QS_COLLECTED = 16,
  QS_DONE_BAND1 = 32, QS_DONE_CUT = 64, QS_DONE_ZERO = 128, QS_LIMIT = 256, QS_MISMATCH = 512,
  QS_HINT = 1024, QS_BINOVF = 2048,
  QS_FAIL = 4096  // not resolved here: NaN placeholder + failure list (knn_exact.hip)
};
constexpr uint32_t kNaNBits = 0x7fc00000u;

// 16-bit bin checksum of a lane's histogram: c_hi (a 32-bit register) is exactly the
// number of counted values in bins [0, bin_hi), and every wrap of a 16-bit counter
// (an even bin carrying into its odd neighbour, an odd bin carrying out of the dword)
// changes the sum of the counters by -65535 or -65536 — so the sum equals c_hi iff no
// bin overflowed during the pass (values of dropped top bins were subtracted from c_hi
// as read, which preserves the identity).
__device__ __forceinline__ bool hist_consistent(const Lane &s, const uint32_t *pool, int lane) {
  uint32_t sum = 0;
#pragma unroll
  for (int b = 0; b < kBins; b++) sum += b < s.bin_hi ? hist_read(pool, (uint32_t)b, lane) : 0u;
  return sum == s.c_hi;
}


// STRIDE = false: one wave per group (the normal launch). STRIDE = true: a small persistent
// grid strides over the groups — the form launched beside the grid kernel when the device
// gate is expected to pick the grid: every wave returns at once when it does, instead of
// millions of blocks each being dispatched only to return (1B points: ~16 ms per launch).
template <int RCAP, int NT, bool STRIDE>
__global__ __launch_bounds__(kThreads, RCAP <= 32 ? LSK_ROWS_MINW : 4) void knn_rows_kernel(const lsk_knn_args A) {
  __shared__ WaveLdsR<RCAP> lds[kWavesPerBlock];
  const int wid = threadIdx.x >> 6;
  const int lane = lsk::lane_id();
  if (!STRIDE) {
    const uint32_t nb = lsk::list_blocks(A, gridDim.x, kWavesPerBlock);
    if (blockIdx.x >= nb) return;
    const uint32_t blk = lsk::xcd_remap(blockIdx.x, nb);
    const uint64_t wave = (uint64_t)blk * kWavesPerBlock + wid + (uint32_t)A.wave_base;
#include "knn_rows_wave.inc"
  } else {
    if (A.gate && *A.gate != A.gate_on) return;
    uint64_t nwaves = A.groups ? (uint64_t)A.ngroups : (uint64_t)((A.nq + 63) / 64);
    if (A.groups && A.ngroups_dev) nwaves = min(nwaves, (uint64_t)*A.ngroups_dev);
    if (A.wave_end > 0) nwaves = min(nwaves, (uint64_t)A.wave_end);
    // groups: strided, or from the work queue when the launch has one (A.wq)
    const bool dyn = A.wq != nullptr;
    uint64_t w = dyn ? lsk::wq_next(A.wq, (uint32_t)A.wave_base)
                     : (uint64_t)blockIdx.x * kWavesPerBlock + wid + (uint32_t)A.wave_base;
    while (w < nwaves) {
      [&](const uint64_t wave) {
#include "knn_rows_wave.inc"
      }(w);
      w = dyn ? lsk::wq_next(A.wq, (uint32_t)A.wave_base) : w + (uint64_t)gridDim.x * kWavesPerBlock;
    }
  }
}

}  // namespace

#ifndef LSK_RCAP
#define LSK_RCAP 32  // row queue capacity (entries per row, a power of two <= 32)
#endif
constexpr unsigned kStrideBlocks = 1024;  // persistent form: 2048 waves, 2 per SIMD
constexpr unsigned kStrideBlocksFull = 4096;  // ... over a short group list (pad2 = 2)

extern "C" int lsk_hip_knn_rows(const lsk_knn_args *args, void *stream) {
  const lsk_knn_args &A = *args;
  if (A.k < 1 || A.k > 65535) {
    lsk::set_last_error("knn_rows: k must be in [1, 65535] for the radix-select kernel");
    return 1;
  }
  if (A.nq >= ((int64_t)1 << 32) || A.ntrees < 0 || A.ntrees > 2 || A.seed < 0 || A.seed > 64 ||
      (A.qrot && A.ntrees != 1)) {
    lsk::set_last_error("knn_rows: nq must be < 2^32, ntrees in [0,2], seed in [0,64]; a rotated frame "
                        "(qrot) with one tree");
    return 1;
  }
  for (int t = 0; t < A.ntrees; t++) {
    if (A.tree[t].n >= ((int64_t)1 << 31) || A.tree[t].depth > 26 || !A.tree[t].qnodes) {
      lsk::set_last_error("knn_rows: tree too large or quarter boxes missing");
      return 1;
    }
  }
  const int64_t ngroups = A.groups ? A.ngroups : (A.nq + 63) / 64;
  // this launch's waves: [wave_base, wave_end or ngroups)
  const int64_t wend = A.wave_end > 0 && A.wave_end < ngroups ? A.wave_end : ngroups;
  if (A.wave_base < 0 || wend - A.wave_base <= 0) return 0;
  const unsigned nblk = lsk_blocks(wend - A.wave_base, kWavesPerBlock);
  // Row work-queue capacity 32 entries per row: 5.6 KB of LDS per wave, 28 waves
  // per CU. One instance per tree count: the single-tree one (every local pass) has no
  // per-lane tree selects in its step loop; the two-tree one serves halo re-queries.
  hipStream_t st = (hipStream_t)stream;
  if (A.pad2 >= 1) {  // persistent strided form (see knn_rows_kernel); 2: a short list
    const unsigned cap = A.pad2 == 2 ? kStrideBlocksFull : kStrideBlocks;
    const unsigned sblk = nblk < cap ? nblk : cap;
    if (A.ntrees > 1)
      knn_rows_kernel<LSK_RCAP, 2, true><<<sblk, kThreads, 0, st>>>(A);
    else if (A.qrot)
      knn_rows_kernel<LSK_RCAP, 3, true><<<sblk, kThreads, 0, st>>>(A);
    else
      knn_rows_kernel<LSK_RCAP, 1, true><<<sblk, kThreads, 0, st>>>(A);
  } else if (A.ntrees > 1) {
    knn_rows_kernel<LSK_RCAP, 2, false><<<nblk, kThreads, 0, st>>>(A);
  } else if (A.qrot) {
    knn_rows_kernel<LSK_RCAP, 3, false><<<nblk, kThreads, 0, st>>>(A);
  } else {
    knn_rows_kernel<LSK_RCAP, 1, false><<<nblk, kThreads, 0, st>>>(A);
  }
  LSK_CHECK_LAUNCH("knn_rows");
  return 0;
}
