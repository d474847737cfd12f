// k-th-NN distance selection with a cell-grid candidate source (the near-uniform fast path).
//
// Same contract and selection algorithm as knn_rows.hip (two-pass radix select on the
// float bits of d² with a per-lane 16-bit LDS histogram, LDS collect pool and a per-lane
// (k - below)-max-heap, exact on every input through the failure list + knn_exact.hip
// backstop; reference runQuery / extractFinalResult, unorderedDataVariant.cu:75-103). What
// differs is where the candidates come from and how they are broadcast:
//
//  * the curve-sorted points are indexed by an octree grid: every cell of level `lc` has
//    64 slots, one per grandchild (level lc+2) IN CURVE ORDER — which is memory order —
//    holding the grandchild's contiguous run of the sorted array and its coordinates.
//    Built in one pass over the sorted points and keys (grid_build_kernel: a grandchild's
//    slot is the 6 key bits below its cell's prefix);
//  * a wave owns 64 curve-consecutive queries. A pass enumerates the level-lc cells
//    around the wave's query box ARITHMETICALLY (cell coordinates from the quantised box
//    ± the current radius; no pointer chasing), NEAREST FIRST: the cells' gaps to the box
//    sit in the lanes and each round takes the smallest one still within the (shrinking)
//    radius, so the bounds tighten before farther cells are reached;
//  * per cell, one 16-byte vector load gives each lane one grandchild slot (prefetched one
//    cell ahead) and one VALU pass tests all 64 against the box; runs of needed (or empty)
//    slots are contiguous in memory and become one segment each;
//  * a cell's segments are one candidate stream read with SCALAR loads (wave-uniform
//    addresses through the constant address space): the candidates arrive in SGPRs and
//    every VALU op of the canonical d² takes them as an operand — 6 VALU per candidate and
//    lane, no broadcast, no per-row queues or logs; the next batch's loads (across segment
//    boundaries) are issued before the current batch is computed;
//  * the histogram update is branch-free: lanes l and l+32 share one dword per bin row,
//    and every candidate adds to the row of its value CLAMPED into the lane's range with
//    one v_med3_u32 — values past the range top land in the row just above the top bin
//    (the "clamp row"), values below it in bin 0. The count below the top (c_hi) is not
//    counted per candidate: it is derived once per cell from the wave's add count minus
//    the clamp row (read and zeroed, "fold"). 3 VALU per candidate (med3, shift,
//    shift-add) instead of 6 (round 6; round 3's form selected between a bin and a trash
//    address and counted c_hi with a carry-add). The kernel is VALU-cycle bound: a wave64
//    op takes 2 cycles on the 32-lane SIMD, packed f32 ops take 4 (no gain), and an
//    exec-masked half wave costs a full op (profiles/r3_pairs, profiles/r3_hist).
//
// Every cull is conservative: cell boxes are the quantisation intervals widened by a
// few ulps of the cube, the radius is inflated by 2^-16 (relative) over the largest lane
// bound, so a skipped point always has canonical d² >= every lane's bound.
//
// Measured on one MI355X, uniform points, k = 100, this pass vs the bucket-tree kernel on
// the same index (bit-identical outputs): 1e8 0.088 vs 0.125 s, 1B 0.932 vs 1.29 s
// (profiles/r3_hist, profiles/r3_s2); GRID=auto keeps clustered, planar, duplicate and
// mixed-scale data on knn_rows (knn_engine.grid_applies).
#include "dev.h"

namespace {

using lsk::bitsf;
using lsk::fbits;

#ifndef LSK_GRID_MINW
// waves per SIMD the register budget is sized for. 6 (80 VGPRs; 132 SGPRs / 52 VGPRs
// spilled with 8-candidate batches) against 7 (72 VGPRs; 152 / 89 spilled): 1e8 k=100
// 79.6 -> 77.7 ms (profiles/r5_kernel_ab/minw6_vs_7_1e8.txt)
#define LSK_GRID_MINW 6
#endif
#ifndef LSK_GRID_BATCH
#define LSK_GRID_BATCH 8  // candidates per scalar-load batch of the cell stream (4 or 8; 8: 1B stream 952.6 -> 941.9-943.3 ms, profiles/r5_kernel_ab)
#endif
#ifndef LSK_GRID_WPB
// waves per workgroup: 1 (1e8 k=100 at 6 waves/SIMD: 77.0 ms; 2: 78.1; 4: 79.6,
// profiles/r5_kernel_ab/wpb_batch_1e8.txt)
#define LSK_GRID_WPB 1
#endif
constexpr int kWPB = LSK_GRID_WPB;
constexpr int kThreads = kWPB * lsk::kWave;
#ifndef LSK_GRID_BINS
#define LSK_GRID_BINS 40
#endif
constexpr int kBins = LSK_GRID_BINS;      // 16-bit bins
// Lanes l and l+32 share a dword (low / high half) of each bin row, so a lane's increment
// is a per-lane constant and every candidate adds without a branch (values past the range
// go to a trash row, kBins).
constexpr int kPool = (kBins + 1) * 32;   // dwords per wave: histogram + trash row, or collect pool
// Grandchild culling by ROWS: a grandchild is needed when it lies within the cull radius
// of one of the wave's four 16-query rows (each with its own box and radius, kept in LDS)
// instead of the whole wave's box and largest radius: the union of the rows' regions is
// smaller (0.918x the evaluations at 1e8 uniform, k = 100; 4 gap tests per grandchild):
// 0.088 -> 0.085 s, 1B stream 1005 Mpts/s (profiles/r3_rowcull). With the row boxes in
// SGPRs the extra pressure put spill reloads into the candidate loop and it was slower
// (0.091 s); eight groups of 8 queries cut 11.9 % of the evaluations but spent it on twice
// the gap tests (0.086 s).
constexpr int kCullGroups = 4;
constexpr int kCullLanes = 64 / kCullGroups;

// max inside each 16-lane row (DPP: quads, then the row); every lane of a row ends with
// the row's value
__device__ __forceinline__ float group_max(float v) {
  v = fmaxf(v, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xB1, 0xf, 0xf, false)));
  v = fmaxf(v, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x4E, 0xf, 0xf, false)));
  v = fmaxf(v, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x124, 0xf, 0xf, false)));
  v = fmaxf(v, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x128, 0xf, 0xf, false)));
  return v;
}
__device__ __forceinline__ float group_min(float v) { return -group_max(-v); }
// band selection: a bitonic network over up to kNet band values in registers (1e8, k=100:
// 0.082 -> 0.079 s against the LDS heap for every band; 16 values: no gain, bands of
// 17..32 then take the heap and the wave runs both)
#ifndef LSK_GRID_NET
#define LSK_GRID_NET 16  // (round 6, with first_range's finer bins; rounds 3-5: 32)
#endif
#ifndef LSK_GRID_NETMIN
#define LSK_GRID_NETMIN 4
#endif
constexpr int kNet = LSK_GRID_NET;
constexpr int kNetMin = LSK_GRID_NETMIN;  // the network serves a wave only if some band holds more values
#ifndef LSK_GRID_ABL
#define LSK_GRID_ABL 0  // tuning ablations (wrong results): 1 no wrap check, 2 no band network
#endif
#ifndef LSK_GRID_TOPBINS
#define LSK_GRID_TOPBINS 0  // 0: by k (first_range); else fixed (tuning)
#endif
constexpr uint32_t kLogBins = 5;          // floor(log2(kBins))
#ifndef LSK_GRID_SHIFT0
#define LSK_GRID_SHIFT0 0  // 0: by k (first_range); else fixed (tuning)
#endif
// First-range resolution and top by k (round 6). The k-th's d² spreads ~2/(3 sqrt k)
// around the density estimate (6.7 % at k = 100), so the bins of the first range (and of
// every restart) narrow as k grows: bins of 2^shift0 float ulps (20: 1/8 octave of d², 19:
// 1/16, 18: 1/32) and a top kTop bins above the estimate. Finer bins make the final band
// (the k-th's bin) narrower: fewer values to collect and select (16-value network instead
// of 32) and a smaller collect radius; a lower top makes the first cells cull harder. 1e8
// uniform, k = 100, bit-identical outputs (profiles/r6_bins): 20 / +10 bins (rounds 3-5)
// 74.9 ms, 19 / +14 72.6, 18 / +22 70.5; 1B: 773.6 -> 730.3 ms; k in {8..128} at 1e8 in
// profiles/r6_bins/k_sweep_1e8.txt.
struct FirstRange {
  uint32_t shift, top;
};
__device__ __forceinline__ FirstRange first_range(uint32_t k) {
  if (LSK_GRID_SHIFT0 != 0) return FirstRange{(uint32_t)LSK_GRID_SHIFT0, (uint32_t)LSK_GRID_TOPBINS};
  if (k >= 96u) return FirstRange{18u, 22u};  // (k = 64: 19 / +14 65.4 ms, 18 / +22 66.1)
  if (k >= 12u) return FirstRange{19u, 14u};  // (k = 8: 19 / +14 38.9 ms, 20 / +10 36.6)
  return FirstRange{20u, 10u};
}
constexpr uint32_t kMaxPasses = 24;
constexpr uint32_t kUnknown = 0xffffffffu;
constexpr uint32_t kNaNBits = 0x7fc00000u;

// LSK_GRID_PROFILE builds (tuning only): shader-clock cycles per wave in candidate
// processing / cell enumeration of each pass kind, and the whole wave, into
// stats[16..19] and [23] (knn_engine.KnnStats prof_* names), evals per pass kind in
// stats[12] (HIST) and [13] (COLLECT).
#ifdef LSK_GRID_PROFILE
#define LSK_GT(v) const uint64_t v = __builtin_readcyclecounter()
#define LSK_GADD(acc, t0) (acc) += __builtin_readcyclecounter() - (t0)
#else
#define LSK_GT(v)
#define LSK_GADD(acc, t0)
#endif

enum : uint32_t { ST_HIST = 0, ST_READY = 1, ST_DONE = 2 };
enum { MODE_HIST = 0, MODE_COLLECT = 1 };
enum : uint32_t {
  QS_OVERFLOW = 1, QS_UNDERFLOW = 2, QS_REFINE = 4, QS_COLLECTED = 16, QS_DONE_BAND1 = 32,
  QS_DONE_CUT = 64, QS_LIMIT = 256, QS_MISMATCH = 512, QS_HINT = 1024, QS_BINOVF = 2048,
  QS_FAIL = 4096
};

struct Lane {
  float qx, qy, qz;
  uint32_t state;
  // histogram range [lo_b, hi_b) in bins of 2^shift: lo_b is a multiple of 2^shift and
  // hi_b = lo_b + bin_hi << shift (a whole number of bins; a cutoff is applied to the
  // result, not to the range). lo_b holds the answer once DONE. hi_b = 0: nothing more
  // can count (the zero probe's k exact copies).
  uint32_t lo_b, hi_b, shift;
  int32_t bin_hi;
  uint32_t c_hi;     // values < hi_b this pass (exact, 32-bit; derived: adds - above)
  uint32_t above;    // values of this pass at or above the top: folded clamp row + dropped bins
  uint32_t c_base;   // exact count below lo_b, or kUnknown (READY: count below the band)
  uint32_t nudf;
  uint32_t band_lo, band_w, bc;
  uint32_t coff, ccnt;
  // operands of the histogram add (hist_regs): clamp top, row base, per-lane increment
  uint32_t chi, hbase, inc;
};

__device__ __forceinline__ void set_range(Lane &s, uint32_t lo_b, uint32_t shift, uint32_t top_limit,
                                          uint32_t c_base) {
  // bins start at a multiple of 2^shift (the histogram add then needs no subtraction);
  // a lower start than asked for loses the exact count below it
  const uint32_t lo = lo_b & ~((1u << shift) - 1u);
  s.lo_b = lo;
  s.c_base = lo == 0 ? 0u : (lo == lo_b ? c_base : kUnknown);
  s.shift = shift;
  // the fewest whole bins (<= kBins) that reach top_limit, ending at or below +inf (a value
  // at or past the top — +inf padding included — lands in the clamp row)
  const uint64_t span = top_limit > lo ? (uint64_t)(top_limit - lo) : 0ull;
  uint64_t nb = (span + ((1ull << shift) - 1)) >> shift;
  const uint64_t nb_inf = lo < lsk::kInfBits ? (uint64_t)(lsk::kInfBits - lo) >> shift : 0ull;
  nb = nb < nb_inf ? nb : nb_inf;
  s.bin_hi = (int32_t)(nb < (uint64_t)kBins ? nb : (uint64_t)kBins);
  s.hi_b = lo + ((uint32_t)s.bin_hi << shift);
  s.c_hi = 0;
  s.above = 0;
}

// A range that starts at an estimate: if the cutoff lies at or below its (aligned) start,
// the range would be empty (bin_hi = 0) and a value below the start — the query's own
// zero at k = 1 — would land in the clamp row, uncounted; such a range starts at 0 instead
// with bins wide enough that kBins of them reach the cutoff (everything counts below it).
__device__ __forceinline__ void start_range(Lane &s, uint32_t lo_b, uint32_t shift, uint32_t top_limit) {
  if ((lo_b & ~((1u << shift) - 1u)) < top_limit) {
    set_range(s, lo_b, shift, top_limit, kUnknown);
    return;
  }
  uint32_t sh = 0;
  while (((uint64_t)kBins << sh) < (uint64_t)top_limit) sh++;
  set_range(s, 0u, sh, top_limit, 0u);
}

typedef __attribute__((address_space(3))) uint32_t lds_u32;
typedef __attribute__((address_space(3))) uint16_t lds_u16;
__device__ __forceinline__ uint32_t lds_addr(uint32_t *p) { return (uint32_t)(uintptr_t)(lds_u32 *)p; }
__device__ __forceinline__ void lds_add(uint32_t addr, uint32_t v) {
  __atomic_fetch_add((lds_u32 *)(uintptr_t)addr, v, __ATOMIC_RELAXED);
}
// this lane's 16-bit half of a histogram dword (byte address)
__device__ __forceinline__ uint32_t lds_read16(uint32_t addr) { return *(lds_u16 *)(uintptr_t)addr; }
__device__ __forceinline__ void lds_zero16(uint32_t addr) { *(lds_u16 *)(uintptr_t)addr = 0; }
// LDS byte address of the histogram row of v clamped into [lo, hi]: base + ((med3 >> sh) << 7).
// One asm block: the compiler forms med3 only for constant bounds (else max + min), and a
// lone asm med3 gets an s_nop before its VALU consumer (it might be a transcendental).
__device__ __forceinline__ uint32_t hist_row_addr(uint32_t v, uint32_t lo, uint32_t hi, uint32_t sh,
                                                  uint32_t base) {
  uint32_t r;
  asm("v_med3_u32 %0, %1, %2, %3\n\tv_lshrrev_b32 %0, %4, %0\n\tv_lshl_add_u32 %0, %0, 7, %5"
      : "=&v"(r)
      : "v"(v), "v"(lo), "v"(hi), "v"(sh), "v"(base));
  return r;
}

__device__ __forceinline__ uint32_t hist_read(const uint32_t *pool, uint32_t b, int lane) {
  return (pool[b * 32u + ((uint32_t)lane & 31u)] >> (((uint32_t)lane & 32u) >> 1)) & 0xffffu;
}

__device__ __forceinline__ uint32_t top_count(const Lane &s, const uint32_t *pool, int lane) {
  return s.bin_hi > 0 ? hist_read(pool, (uint32_t)s.bin_hi - 1u, lane) : s.c_hi;
}

__device__ __forceinline__ void underflow_restart(Lane &s, uint32_t shift0) {
  const uint32_t topb = s.hi_b;
  if (s.nudf == 0 && topb > ((uint32_t)kBins << shift0)) {
    set_range(s, topb - ((uint32_t)kBins << shift0), shift0, topb, kUnknown);
  } else {
    uint32_t sh = 0;
    while (((uint64_t)kBins << sh) < (uint64_t)topb) sh++;
    set_range(s, 0u, sh, topb, 0u);
  }
  s.nudf++;
}


// 16-bit bin checksum (see knn_rows.hip hist_consistent): the counter sum over [0, bin_hi)
// equals c_hi iff no counter wrapped.
__device__ __forceinline__ bool hist_consistent(const Lane &s, const uint32_t *pool, int lane) {
  uint32_t sum = 0;
#pragma unroll
  for (int b = 0; b < kBins; b++) sum += b < s.bin_hi ? hist_read(pool, (uint32_t)b, lane) : 0u;
  return sum == s.c_hi;
}

template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xf, 0xf, false));
}
// wave max of non-negative floats (DPP inside rows, scalar combine of the 4 rows)
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

__device__ __forceinline__ float bcast64(float v, uint32_t j) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), (int)j));
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

// Wave-uniform grid context.
struct GridCtx {
  const float *pts;        // sorted points (packed float3, padded)
  const float *inf4;       // 4 x +inf (tail padding of a candidate batch)
  const uint4 *slots;      // [8^lc][64] grandchild runs (start, end, coords, -) in Hilbert order
  float ox, oy, oz;        // cube origin
  float scale;             // 1024 / extent (the sort keys' quantisation)
  float step;              // extent / 1024: one level-10 quantum
  float eps;               // absolute slack of cell boundaries and the cull radius
  uint32_t lc;             // cell level
  float wlx, wly, wlz, whx, why, whz;  // box of the wave's queries
  float *rbox;             // LDS, per row r: [8r..8r+5] box of its 16 queries (lo xyz, hi
                           // xyz), [8r+6] its squared cull radius (cull_r2); read per cell
                           // (in SGPRs they pushed spill reloads into the candidate loop)
  uint32_t *pool;
  uint32_t row0;           // LDS byte address of this lane's dword in histogram row 0
  uint32_t hoff;           // byte offset of this lane's 16-bit half (lanes l, l+32 share a dword)
  uint32_t inc;            // this lane's histogram increment: 1 or 1 << 16
  int lane;
  uint32_t k;
  uint32_t adds;           // histogram adds per lane this pass (wave-uniform)
  uint32_t evals, cells_n, segs;
#ifdef LSK_ROWQ_STATS
  uint32_t rq_steps, rq_took, rq_refills;
#endif
#ifdef LSK_GRID_PROFILE
  uint64_t prof[8];
  uint32_t ev_mode[2];
#endif
};

// The grid fields of G from a view: the sorted points it indexes, its slots, the cube of
// its keys (origin, quantisation) and the slack of its cell boundaries.
__device__ __forceinline__ void load_grid(GridCtx &G, const lsk_grid_view &V, const float *pts) {
  G.pts = pts;
  G.inf4 = V.inf4;
  G.slots = (const uint4 *)V.slots;
  const lsk::cfloat_p bx = lsk::as_const(V.box);
  G.ox = bx[0];
  G.oy = bx[1];
  G.oz = bx[2];
  G.scale = bx[6];
  const float ext = bx[7];
  G.step = ext * (1.f / 1024.f);
  const float mag = fmaxf(fmaxf(fabsf(G.ox), fabsf(G.oy)), fmaxf(fabsf(G.oz), 0.f)) + ext;
  G.eps = mag * 0x1p-19f;
  G.lc = (uint32_t)V.level;
}

// The histogram add's operands after a change of the lane's range or state. A lane that
// is not histogramming adds 0 (to its row 0).
__device__ __forceinline__ void hist_regs(Lane &s, const GridCtx &G) {
  const bool h = s.state == ST_HIST;
  s.chi = h ? s.lo_b + ((uint32_t)s.bin_hi << s.shift) : s.lo_b;
  s.hbase = G.row0 - ((s.lo_b >> s.shift) << 7);
  s.inc = h ? G.inc : 0u;
}

// Fold the clamp row (row bin_hi: every value at or above the top since the last fold)
// into `above` and zero it, then c_hi = adds - above. Called once per cell, so the clamp
// row never holds more than one cell's values (no 16-bit wrap on long passes).
__device__ __forceinline__ void hist_fold(Lane &s, const GridCtx &G) {
  if (s.state == ST_HIST) {
    const uint32_t a = G.row0 + G.hoff + ((uint32_t)s.bin_hi << 7);
    s.above += lds_read16(a);
    lds_zero16(a);
    s.c_hi = G.adds - s.above;
  }
}

// Drop top bins while at least k counted values stay below: the lane's bound shrinks. A
// dropped bin becomes the clamp row (its values move to `above`, the row is zeroed).
__device__ __forceinline__ void hist_shrink(Lane &s, const GridCtx &G) {
  const uint32_t k = G.k;
  while (s.bin_hi > 0) {
    const uint32_t top = hist_read(G.pool, (uint32_t)s.bin_hi - 1u, G.lane);
    if (s.c_hi - top < k) break;
    s.c_hi -= top;
    s.above += top;
    s.bin_hi--;
    lds_zero16(G.row0 + G.hoff + ((uint32_t)s.bin_hi << 7));
    s.hi_b = s.lo_b + ((uint32_t)s.bin_hi << s.shift);
  }
  // k exact zeros: the k-th is 0 and nothing can be closer (knn_rows zero probe)
  if (s.bin_hi == 1 && s.lo_b == 0u && s.shift == 0u && s.c_hi >= k) s.hi_b = 0u;
  hist_regs(s, G);
}

// Cell coordinate at level l (monotone in v: a point with coordinate v' <= v never lies in
// a later cell — the same float ops as the sort keys, common.h morton_quant).
__device__ __forceinline__ uint32_t cell_of(float v, float o, float scale, uint32_t sh) {
  return lsk::morton_quant(v, o, scale) >> sh;
}

// Conservative [lo, hi] of cell c (level-10 quanta [c << sh, (c+1) << sh)) on one axis.
__device__ __forceinline__ void cell_span(const GridCtx &G, float o, uint32_t c, uint32_t sh, uint32_t last,
                                          float &lo, float &hi) {
  lo = c == 0 ? -__builtin_inff() : o + (float)(c << sh) * G.step - G.eps;
  hi = c >= last ? __builtin_inff() : o + (float)((c + 1u) << sh) * G.step + G.eps;
}

__device__ __forceinline__ float gap1(float lo, float hi, float wl, float wh) {
  return fmaxf(0.f, fmaxf(lo - wh, wl - hi));
}

// gap² between the cell (x, y, z) of level (10 - sh) and the wave's query box
__device__ __forceinline__ float cell_gap2(const GridCtx &G, uint32_t x, uint32_t y, uint32_t z, uint32_t sh) {
  const uint32_t last = (1023u >> sh);
  float lx, hx, ly, hy, lz, hz;
  cell_span(G, G.ox, x, sh, last, lx, hx);
  cell_span(G, G.oy, y, sh, last, ly, hy);
  cell_span(G, G.oz, z, sh, last, lz, hz);
  return lsk::dist2(gap1(lx, hx, G.wlx, G.whx), gap1(ly, hy, G.wly, G.why), gap1(lz, hz, G.wlz, G.whz));
}

// Per-lane bound of the current pass (HIST: range top; COLLECT: band top; else 0).
template <int MODE>
__device__ __forceinline__ float lane_bound(const Lane &s) {
  if (MODE == MODE_HIST) return s.state == ST_HIST ? bitsf(s.hi_b) : 0.f;
  return s.band_w ? bitsf(s.band_lo + s.band_w) : 0.f;
}

// Squared cull radius over the wave: every lane's bound, inflated so that a point whose
// true distance to the query box is at least this radius has canonical d² >= the bound
// (relative 2^-16 covers the rounding of d² and of the gap arithmetic; eps covers the
// absolute rounding of coordinates).
__device__ __forceinline__ float inflate_r2(float b, float eps) {
  if (fbits(b) == 0u) return 0.f;  // (bits: a denormal bound is still a bound)
  const float r = sqrtf(b) * (1.f + 0x1p-16f) + eps;
  return r * r;
}

template <int MODE>
__device__ __forceinline__ float cull_r2(const Lane &s, GridCtx &G) {
  // row maxima (DPP inside the 16-lane rows), each row's radius, the wave's = the largest
  const float v = group_max(lane_bound<MODE>(s));
  const float r2 = inflate_r2(v, G.eps);  // this lane's row's radius
  if ((G.lane & (kCullLanes - 1)) == 0) G.rbox[(G.lane / kCullLanes) * 8 + 6] = r2;
  const uint32_t a = (uint32_t)__builtin_amdgcn_readlane(__float_as_int(r2), 0);
  const uint32_t b = (uint32_t)__builtin_amdgcn_readlane(__float_as_int(r2), 16);
  const uint32_t c = (uint32_t)__builtin_amdgcn_readlane(__float_as_int(r2), 32);
  const uint32_t d = (uint32_t)__builtin_amdgcn_readlane(__float_as_int(r2), 48);
  return __uint_as_float(max(max(a, b), max(c, d)));
}

#ifndef LSK_GRID_HSKIP
#define LSK_GRID_HSKIP 0  // 1: skip a 4-candidate histogram step when no lane has a value below its top (1e8 k=100: 80.3 vs 74.3 ms, profiles/r6_hist)
#endif
template <int MODE>
__device__ __forceinline__ void update4(Lane &s, GridCtx &G, uint32_t u0, uint32_t u1, uint32_t u2, uint32_t u3) {
  if (MODE == MODE_HIST) {
    if (LSK_GRID_HSKIP) {
      const uint32_t um = min(min(u0, u1), min(u2, u3));
      if (!__ballot(um < s.hi_b)) return;
    }
    const uint32_t u[4] = {u0, u1, u2, u3};
    // every slot adds, without a branch or a compare: the value clamped into [lo_b, top]
    // (v_med3_u32) picks the row — its bin, bin 0 below the range, the clamp row (bin_hi)
    // at or above the top — and lo_b being a multiple of 2^shift folds the bin offset into
    // the per-lane row base: med3, shift, shift-add (3 VALU; round 3-5: 6). The count below
    // the top is derived per cell (hist_fold). A 16-bit wrap (65536 adds to one in-range
    // bin in a pass) is caught by hist_consistent (the clamp row is zeroed every cell).
    G.adds += 4u;
#pragma unroll
    for (int t = 0; t < 4; t++) {
      lds_add(hist_row_addr(u[t], s.lo_b, s.chi, s.shift, s.hbase), s.inc);
    }
  } else {
    const uint32_t bl = s.band_lo, bw = s.band_w;
    const bool any = (u0 - bl < bw) || (u1 - bl < bw) || (u2 - bl < bw) || (u3 - bl < bw);
    if (!__ballot(any)) return;
    const uint32_t u[4] = {u0, u1, u2, u3};
#pragma unroll
    for (int t = 0; t < 4; t++) {
      if (u[t] - bl < bw) {
        if (s.ccnt < s.bc) G.pool[s.coff + s.ccnt] = u[t];
        s.ccnt++;
      }
    }
  }
}

// Points [i0, i1) of the sorted array (process_segment: 4 per batch; the cell stream:
// LSK_GRID_BATCH, 8 — half the per-batch scalar work per candidate) through scalar loads, software
// pipelined: the wait for batch i (lgkmcnt(0): scalar loads may return out of order, so
// only an empty queue proves a batch complete) comes BEFORE batch i+1's loads are issued,
// which then fly while batch i is computed. Reads past i1 stay inside the array's
// 64-point readable pad (i < i1 <= n).
struct Batch {
  float x0, y0, z0, x1, y1, z1, x2, y2, z2, x3, y3, z3;
};
// 4 consecutive points: 12 dwords in two scalar loads (x8 + x4)
__device__ __forceinline__ Batch load_batch(lsk::cfloat_p P, uint32_t i) {
  const lsk::cfloat_p p = P + 3ull * (uint64_t)i;
  return Batch{p[0], p[1], p[2], p[3], p[4], p[5], p[6], p[7], p[8], p[9], p[10], p[11]};
}
constexpr unsigned kWaitLgkm0 = 0xC07F;  // s_waitcnt lgkmcnt(0) (vmcnt / expcnt untouched)

constexpr uint32_t kSegCheck = 1024;  // candidates between bound checks in a long segment

template <int MODE>
__device__ __forceinline__ void shrink_all(Lane &s, GridCtx &G) {
  if (MODE == MODE_HIST) {
    hist_fold(s, G);
    if (__ballot(s.state == ST_HIST && s.c_hi >= G.k)) {
      if (s.state == ST_HIST && s.c_hi >= G.k) hist_shrink(s, G);
    }
  }
}

template <int MODE>
__device__ __forceinline__ void eval4(Lane &s, GridCtx &G, const Batch &b) {
  const uint32_t u0 = fbits(lsk::dist2(s.qx - b.x0, s.qy - b.y0, s.qz - b.z0));
  const uint32_t u1 = fbits(lsk::dist2(s.qx - b.x1, s.qy - b.y1, s.qz - b.z1));
  const uint32_t u2 = fbits(lsk::dist2(s.qx - b.x2, s.qy - b.y2, s.qz - b.z2));
  const uint32_t u3 = fbits(lsk::dist2(s.qx - b.x3, s.qy - b.y3, s.qz - b.z3));
  update4<MODE>(s, G, u0, u1, u2, u3);
}

// The 64 grandchild slots of one level-lc cell, fetched ahead of use (one 16-byte vector
// load per lane: its counter retires in order, so the wait lands at the first use, one
// cell later): lane j holds the j-th grandchild (level lc+2) IN HILBERT ORDER — the
// order of the sorted array — as (start, end, packed coordinates); empty: (0, 0).
struct CellLoad {
  uint32_t a, e, xyz;  // per lane
};
__device__ __forceinline__ CellLoad fetch_cell(const GridCtx &G, uint32_t x, uint32_t y, uint32_t z) {
  const uint32_t mc = lsk::morton3(x, y, z);
  const uint4 v = G.slots[64u * mc + (uint32_t)G.lane];
  return CellLoad{v.x, v.y, v.z};
}

template <int MODE>
__device__ __forceinline__ void count_batch(GridCtx &G) {
  G.evals += (uint32_t)LSK_GRID_BATCH;
#ifdef LSK_GRID_PROFILE
  G.ev_mode[MODE] += (uint32_t)LSK_GRID_BATCH;
#endif
}

// The last batch of a segment: slots past its end count nowhere.
template <int MODE>
__device__ __forceinline__ void eval4_tail(Lane &s, GridCtx &G, const Batch &b, uint32_t left) {
  const uint32_t u0 = fbits(lsk::dist2(s.qx - b.x0, s.qy - b.y0, s.qz - b.z0));
  const uint32_t u1 = left > 1u ? fbits(lsk::dist2(s.qx - b.x1, s.qy - b.y1, s.qz - b.z1)) : ~0u;
  const uint32_t u2 = left > 2u ? fbits(lsk::dist2(s.qx - b.x2, s.qy - b.y2, s.qz - b.z2)) : ~0u;
  update4<MODE>(s, G, u0, u1, u2, ~0u);
}

#if LSK_GRID_BATCH == 8
struct Batch8 {
  Batch a, b;
};
__device__ __forceinline__ Batch8 load_batch8(lsk::cfloat_p P, uint32_t i) {
  const lsk::cfloat_p p = P + 3ull * (uint64_t)i;
  return Batch8{Batch{p[0], p[1], p[2], p[3], p[4], p[5], p[6], p[7], p[8], p[9], p[10], p[11]},
                Batch{p[12], p[13], p[14], p[15], p[16], p[17], p[18], p[19], p[20], p[21], p[22], p[23]}};
}
template <int MODE>
__device__ __forceinline__ void eval8(Lane &s, GridCtx &G, const Batch8 &b, uint32_t left) {
  if (left >= 4u) eval4<MODE>(s, G, b.a); else eval4_tail<MODE>(s, G, b.a, left);
  if (left >= 8u) eval4<MODE>(s, G, b.b); else if (left > 4u) eval4_tail<MODE>(s, G, b.b, left - 4u);
}
#endif

// The candidates of one cell as ONE stream over its needed runs of grandchildren, 4 per
// batch. Slots are in memory order, so a run of needed (or empty) slots is one
// contiguous segment of the sorted array. The next batch's scalar loads — the next
// segment's first batch at a segment end — are issued before the current batch is
// computed, so short segments do not each pay a cold load latency. Unrolled by two with
// A / B batch registers (a loop-carried copy would make the compiler wait for the prefetch
// right after issuing it).
//   need: needed non-empty slots; free: needed or empty slots (runs of `free` that hold
//   a needed slot are the segments).
template <int MODE>
__device__ __forceinline__ void process_cell_stream(Lane &s, GridCtx &G, const CellLoad &c, uint64_t need,
                                                    uint64_t free) {
  const lsk::cfloat_p P = lsk::as_const(G.pts);
  // pops the next segment: [start of its first needed slot, end of its last needed slot)
  auto pop = [&](uint32_t &a, uint32_t &b) {
    const uint32_t t0 = (uint32_t)__builtin_ctzll(need);
    const uint64_t after = ~free >> t0;  // first slot past the run of free slots
    const uint32_t len = after ? (uint32_t)__builtin_ctzll(after) : 64u - t0;
    const uint64_t run = (len >= 64u ? ~0ull : ((1ull << len) - 1ull)) << t0;
    const uint64_t in = need & run;
    const uint32_t t1 = 63u - (uint32_t)__builtin_clzll(in);
    need &= ~run;
    a = lsk::uniform((uint32_t)__builtin_amdgcn_readlane((int)c.a, (int)t0));
    b = lsk::uniform((uint32_t)__builtin_amdgcn_readlane((int)c.e, (int)t1));
    G.segs++;
  };
  uint32_t i, e;
  pop(i, e);
  uint32_t chk = i + kSegCheck;
  // position after batch i of [.., e): next batch of the segment, else the next segment
  auto advance = [&](uint32_t &ni, uint32_t &ne) -> bool {
    ni = i + (uint32_t)LSK_GRID_BATCH;
    ne = e;
    if (ni < e) return true;
    if (!need) {
      ni = i;  // (a dummy reload of the current batch: in flight, unused)
      return false;
    }
    pop(ni, ne);
    return true;
  };
#if LSK_GRID_BATCH == 8
  Batch8 A = load_batch8(P, i);
#else
  Batch A = load_batch(P, i);
#endif
  for (;;) {
    uint32_t ni, ne;
    bool more = advance(ni, ne);
    __builtin_amdgcn_s_waitcnt(kWaitLgkm0);
#if LSK_GRID_BATCH == 8
    Batch8 B = load_batch8(P, ni);
    __builtin_amdgcn_sched_barrier(0);
    eval8<MODE>(s, G, A, e - i);
#else
    Batch B = load_batch(P, ni);
    __builtin_amdgcn_sched_barrier(0);
    if (e - i >= 4u) eval4<MODE>(s, G, A); else eval4_tail<MODE>(s, G, A, e - i);
#endif
    count_batch<MODE>(G);
    if (!more) break;
    i = ni;
    e = ne;
    more = advance(ni, ne);
    __builtin_amdgcn_s_waitcnt(kWaitLgkm0);
#if LSK_GRID_BATCH == 8
    A = load_batch8(P, ni);
    __builtin_amdgcn_sched_barrier(0);
    eval8<MODE>(s, G, B, e - i);
#else
    A = load_batch(P, ni);
    __builtin_amdgcn_sched_barrier(0);
    if (e - i >= 4u) eval4<MODE>(s, G, B); else eval4_tail<MODE>(s, G, B, e - i);
#endif
    count_batch<MODE>(G);
    if (!more) break;
    i = ni;
    e = ne;
    if (MODE == MODE_HIST && i >= chk) {
      // long stream (a crowded cell): once every lane's bound has closed (k exact copies:
      // the k-th is 0) the rest of it cannot count
      chk = i + kSegCheck;
      shrink_all<MODE>(s, G);
      if (!__ballot(s.state == ST_HIST && s.hi_b > 0u)) break;
    }
  }
}

// Unrolled by two with separate A / B batch registers: a loop-carried copy of the batch
// would make the compiler wait for the prefetch right after issuing it.
template <int MODE>
__device__ __forceinline__ void process_segment(Lane &s, GridCtx &G, uint32_t i0, uint32_t i1) {
  const lsk::cfloat_p P = lsk::as_const(G.pts);
  i0 = lsk::uniform(i0);
  i1 = lsk::uniform(i1);
  uint32_t i = i0;
  Batch A = load_batch(P, i);
  uint32_t chk = i0 + kSegCheck;
  for (;;) {  // A holds batch i (in flight)
    if (i + 4u > i1) break;
    if (MODE == MODE_HIST && i >= chk) {
      // long segment (a crowded sub-cell): once every lane's bound has closed (k exact
      // copies: the k-th is 0) the rest of it cannot count
      chk = i + kSegCheck;
      shrink_all<MODE>(s, G);
      if (!__ballot(s.state == ST_HIST && s.hi_b > 0u)) break;
    }
    __builtin_amdgcn_s_waitcnt(kWaitLgkm0);
    Batch B = load_batch(P, i + 4u < i1 ? i + 4u : i);
    __builtin_amdgcn_sched_barrier(0);
    eval4<MODE>(s, G, A);
    i += 4u;
    if (i + 4u > i1) {
      A = B;  // (tail: once per segment)
      break;
    }
    __builtin_amdgcn_s_waitcnt(kWaitLgkm0);
    A = load_batch(P, i + 4u < i1 ? i + 4u : i);
    __builtin_amdgcn_sched_barrier(0);
    eval4<MODE>(s, G, B);
    i += 4u;
  }
  if (i < i1) {  // 1-3 tail points (already loaded): slots past the end count nowhere
    __builtin_amdgcn_s_waitcnt(kWaitLgkm0);
    const uint32_t left = i1 - i;
    const Batch &b = A;
    const uint32_t u0 = fbits(lsk::dist2(s.qx - b.x0, s.qy - b.y0, s.qz - b.z0));
    const uint32_t u1 = left > 1u ? fbits(lsk::dist2(s.qx - b.x1, s.qy - b.y1, s.qz - b.z1)) : ~0u;
    const uint32_t u2 = left > 2u ? fbits(lsk::dist2(s.qx - b.x2, s.qy - b.y2, s.qz - b.z2)) : ~0u;
    update4<MODE>(s, G, u0, u1, u2, ~0u);
  }
  G.evals += (i1 - i0 + 3u) & ~3u;  // (an early stop counts the whole segment)
  G.segs++;
#ifdef LSK_GRID_PROFILE
  G.ev_mode[MODE] += (i1 - i0 + 3u) & ~3u;
#endif
}

// One level-lc cell: lane j tests grandchild j against the wave box.
template <int MODE>
__device__ __forceinline__ void process_cell(Lane &s, GridCtx &G, const CellLoad &c, float r2) {
  const bool ne = c.e > c.a;
  const uint64_t nonempty = __ballot(ne);
  if (!nonempty) return;
  G.cells_n++;
  const uint32_t sh = 10u - (G.lc + 2u);
  (void)r2;
  const uint32_t last = (1023u >> sh);
  float lx, hx, ly, hy, lz, hz;
  cell_span(G, G.ox, c.xyz & 1023u, sh, last, lx, hx);
  cell_span(G, G.oy, (c.xyz >> 10) & 1023u, sh, last, ly, hy);
  cell_span(G, G.oz, c.xyz >> 20, sh, last, lz, hz);
  bool in_any = false;
#pragma unroll
  for (int r = 0; r < kCullGroups; r++) {
    const float *b = G.rbox + 8 * r;
    const float g2 = lsk::dist2(gap1(lx, hx, b[0], b[3]), gap1(ly, hy, b[1], b[4]), gap1(lz, hz, b[2], b[5]));
    in_any = in_any || g2 <= b[6];
  }
  const uint64_t need = __ballot(ne && in_any);
  if (!need) return;
  LSK_GT(tp0);
  process_cell_stream<MODE>(s, G, c, need, need | ~nonempty);
  shrink_all<MODE>(s, G);
  LSK_GADD(G.prof[MODE], tp0);
}

// One pass over every cell within the cull radius of the wave's query box (cells that
// hold the queries first). The radius is re-read after every cell (bounds only shrink).
// Cells are enumerated in 4x4x4 blocks, lane l taking cell (l & 3, (l >> 2) & 3, l >> 4) of
// the block (no integer division). A range of more than kMaxCells cells (a bound far above
// the local spacing: k beyond the local point count, or an estimate far off) is served by
// one scan of all points when the tree is small, else the wave hands its unresolved
// queries to the exact backstop (returns false).
constexpr unsigned kStrideBlocks = 2048 / kWPB;  // persistent form: 2048 waves, 2 per SIMD
constexpr unsigned kStrideBlocksFull = 8192 / kWPB;  // persistent form over a short group list: 8192
                                              // waves, the kernel's full occupancy
constexpr uint32_t kMaxCells = 4096;
// Candidate budget of a wave, checked before each pass: max(kEvalBudget, kEvalsPerK * k),
// ~80x a uniform wave at k = 100 (~3.4K). Beyond it the wave's unresolved queries go to
// the exact backstop (one wave per query, 64 candidates per step) instead of one wave
// streaming a dense cluster pass after pass (the grid is only chosen for near-uniform
// data; GRID=on forces it). A check per cell instead cost 16 B/lane more scratch.
constexpr uint32_t kEvalBudget = 1u << 18;
constexpr uint32_t kEvalsPerK = 2048;
constexpr uint32_t kScanAll = 1u << 16;

template <int MODE>
__device__ bool grid_pass_impl(Lane &s, GridCtx &G, uint32_t n);

#ifndef LSK_GRID_ROWQ
#define LSK_GRID_ROWQ 0
#endif
#ifndef LSK_ROWQ_LOW
#define LSK_ROWQ_LOW 1  // a row with at most this many queued segments asks for the next cell
#endif
#if LSK_GRID_ROWQ
// ------------------------------------------------------------------ per-row candidate streams
// Each 16-query row streams ITS OWN candidates (round 6; the SGPR form above streams the
// union of the four rows' needs to all 64 lanes). Cells are still taken nearest first by
// the wave, tested per row (process_cell's row boxes and radii), and each row's runs of
// needed grandchildren ("segments") are appended to that row's queue; a step takes the
// next 16 candidates of every row at once: lane j of row r loads candidate j of its row
// (one vector load, issued a step ahead) and the row's 16 lanes read it with a DPP
// row_newbcast folded into the distance's v_subrev_f32_dpp. Rows consume their queues
// independently across cells, so a row never pays for another row's candidates.
//
// Queue of row r: lanes 16r + t of (qa, qe) hold its t-th segment [qa, qe) of the sorted
// points (t = 0: the head, partly consumed: qa advances); qn = segments queued (the same
// in every lane of the row). A full queue (16) blocks the next cell; within one cell, the
// segments past the 16th are merged into the 16th (the slots between them are unneeded by
// that row and lie in the same cell: extra candidates, never a repeated one).
template <int J>
__device__ __forceinline__ float rowb(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x150 + J, 0xf, 0xf, false));
}
template <int J>
__device__ __forceinline__ uint32_t rowb_u(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x150 + J, 0xf, 0xf, false);
}
// lane j of each row <- lane j + 1 (lane 15 <- 0)
__device__ __forceinline__ uint32_t row_shl1(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x101, 0xf, 0xf, true);
}

struct RowQ {
  uint32_t qa, qe, qn;
};
struct RowPts {
  float x, y, z;
};

// The next (up to) 16 candidates of this lane's row: lane j loads candidate j (padding:
// the +inf point, d² = +inf, at or past every range top and collect band). At most one
// segment boundary per step; a consumed head segment is popped (the queue shifts down).
__device__ __forceinline__ RowPts rowq_take(RowQ &Q, GridCtx &G) {
  const uint32_t j = (uint32_t)G.lane & 15u;
  const uint32_t a0 = rowb_u<0>(Q.qa), e0 = rowb_u<0>(Q.qe), a1 = rowb_u<1>(Q.qa), e1 = rowb_u<1>(Q.qe);
  const uint32_t l0 = e0 - a0, l1 = e1 - a1;
  const uint32_t took = min(l0 + l1, 16u);
#ifdef LSK_ROWQ_STATS
  G.rq_steps++;
  G.rq_took += (uint32_t)__builtin_amdgcn_readlane((int)took, 0) + (uint32_t)__builtin_amdgcn_readlane((int)took, 16) +
               (uint32_t)__builtin_amdgcn_readlane((int)took, 32) + (uint32_t)__builtin_amdgcn_readlane((int)took, 48);
#endif
  const uint32_t idx = j < l0 ? a0 + j : a1 + (j - l0);
  const float *p = j < took ? G.pts + 3ull * idx : G.inf4;
  const RowPts r{p[0], p[1], p[2]};
  const bool pop = took >= l0 && Q.qn > 0u;
  const uint32_t sa = row_shl1(Q.qa), se = row_shl1(Q.qe);
  Q.qa = pop ? sa : Q.qa;
  Q.qe = pop ? se : Q.qe;
  if (j == 0u) Q.qa = pop ? a1 + (took - l0) : a0 + took;
  Q.qn -= pop ? 1u : 0u;
  return r;
}

template <int J>
__device__ __forceinline__ uint32_t rcand(const Lane &s, const RowPts &p) {
  return fbits(lsk::dist2(s.qx - rowb<J>(p.x), s.qy - rowb<J>(p.y), s.qz - rowb<J>(p.z)));
}

template <int MODE>
__device__ __forceinline__ void rowq_eval(Lane &s, GridCtx &G, const RowPts &p) {
  update4<MODE>(s, G, rcand<0>(s, p), rcand<1>(s, p), rcand<2>(s, p), rcand<3>(s, p));
  update4<MODE>(s, G, rcand<4>(s, p), rcand<5>(s, p), rcand<6>(s, p), rcand<7>(s, p));
  update4<MODE>(s, G, rcand<8>(s, p), rcand<9>(s, p), rcand<10>(s, p), rcand<11>(s, p));
  update4<MODE>(s, G, rcand<12>(s, p), rcand<13>(s, p), rcand<14>(s, p), rcand<15>(s, p));
  G.evals += 16u;
#ifdef LSK_GRID_PROFILE
  G.ev_mode[MODE] += 16u;
#endif
}

// One level-lc cell: every row's segments are appended to its queue.
__device__ __forceinline__ void cell_rows(GridCtx &G, const CellLoad &c, RowQ &Q) {
  const bool ne = c.e > c.a;
  const uint64_t nonempty = __ballot(ne);
  if (!nonempty) return;
  G.cells_n++;
  const uint32_t sh = 10u - (G.lc + 2u);
  const uint32_t last = (1023u >> sh);
  float lx, hx, ly, hy, lz, hz;
  cell_span(G, G.ox, c.xyz & 1023u, sh, last, lx, hx);
  cell_span(G, G.oy, (c.xyz >> 10) & 1023u, sh, last, ly, hy);
  cell_span(G, G.oz, c.xyz >> 20, sh, last, lz, hz);
  uint64_t need[kCullGroups];
#pragma unroll
  for (int r = 0; r < kCullGroups; r++) {
    const float *b = G.rbox + 8 * r;
    const float g2 = lsk::dist2(gap1(lx, hx, b[0], b[3]), gap1(ly, hy, b[1], b[4]), gap1(lz, hz, b[2], b[5]));
    need[r] = __ballot(ne && g2 <= b[6]);
  }
  uint32_t qa = Q.qa, qe = Q.qe, qn = Q.qn;
#pragma unroll
  for (int r = 0; r < kCullGroups; r++) {
    uint64_t nd = need[r];
    if (!nd) continue;
    const uint64_t fr = nd | ~nonempty;  // runs of needed or empty slots are contiguous in memory
    uint32_t t = lsk::uniform((uint32_t)__builtin_amdgcn_readlane((int)qn, 16 * r));
    do {
      const uint32_t t0 = (uint32_t)__builtin_ctzll(nd);
      const uint64_t after = ~fr >> t0;
      const uint32_t len = after ? (uint32_t)__builtin_ctzll(after) : 64u - t0;
      const uint64_t run = (len >= 64u ? ~0ull : ((1ull << len) - 1ull)) << t0;
      const uint32_t t1 = 63u - (uint32_t)__builtin_clzll(nd & run);
      nd &= ~run;
      const uint32_t a = lsk::uniform((uint32_t)__builtin_amdgcn_readlane((int)c.a, (int)t0));
      const uint32_t e = lsk::uniform((uint32_t)__builtin_amdgcn_readlane((int)c.e, (int)t1));
      // lane 16r + t takes the segment; past 16 entries lane 16r + 15 extends its end
      const bool at = (uint32_t)G.lane == 16u * r + min(t, 15u);
      qa = at && t < 16u ? a : qa;
      qe = at ? e : qe;
      t += t < 16u ? 1u : 0u;
      G.segs++;
    } while (nd);
    qn = ((uint32_t)G.lane >> 4) == (uint32_t)r ? t : qn;
  }
  Q.qa = qa;
  Q.qe = qe;
  Q.qn = qn;
}

// One pass with per-row streams. The cells in range are visited in chunks of at most
// 16 x 16 x (256 / 256..) cells (one chunk for a normal range), nearest first inside a
// chunk: lane l holds chunk cells l, l+64, l+128, l+192 with their gap to the wave box.
// A range of more than kMaxCells cells is one segment of all points per row (n <= kScanAll)
// or the backstop (returns false).
template <int MODE>
__device__ __forceinline__ bool grid_pass_rows(Lane &s, GridCtx &G, uint32_t n) {
  float r2 = cull_r2<MODE>(s, G);
  if (fbits(r2) == 0u) return true;
  const uint32_t sh = 10u - G.lc;
  const float r = sqrtf(r2);
  const uint32_t x0 = cell_of(G.wlx - r, G.ox, G.scale, sh), x1 = cell_of(G.whx + r, G.ox, G.scale, sh);
  const uint32_t y0 = cell_of(G.wly - r, G.oy, G.scale, sh), y1 = cell_of(G.why + r, G.oy, G.scale, sh);
  const uint32_t z0 = cell_of(G.wlz - r, G.oz, G.scale, sh), z1 = cell_of(G.whz + r, G.oz, G.scale, sh);
  const uint32_t nx = x1 - x0 + 1u, ny = y1 - y0 + 1u, nz = z1 - z0 + 1u;
  const bool scan_all = (uint64_t)nx * ny * nz > kMaxCells;
  if (scan_all && n > kScanAll) return false;
  const uint32_t cxn = min(nx, 16u), cyn = min(ny, 16u), czn = max(1u, min(nz, 256u / (cxn * cyn)));
  const uint32_t ncx = (nx + cxn - 1u) / cxn, ncy = (ny + cyn - 1u) / cyn, ncz = (nz + czn - 1u) / czn;
  const uint32_t nchunks = scan_all ? 0u : ncx * ncy * ncz;
  uint32_t chunk = 0, bx = 0, by = 0, bz = 0, tx = 1, ty = 1, tot = 0, inx = 0, iny = 0;
  const uint32_t l = (uint32_t)G.lane;
  float g0 = __builtin_inff(), g1 = g0, g2 = g0, g3 = g0;
  // chunk k: its origin and size (clipped at the range end) and the gaps of its cells
  auto load_chunk = [&](uint32_t k) {
    const uint32_t kx = k % ncx, ky = (k / ncx) % ncy, kz = k / (ncx * ncy);
    bx = x0 + kx * cxn;
    by = y0 + ky * cyn;
    bz = z0 + kz * czn;
    tx = min(cxn, x1 + 1u - bx);
    ty = min(cyn, y1 + 1u - by);
    const uint32_t tz = min(czn, z1 + 1u - bz);
    tot = tx * ty * tz;
    inx = (65536u + tx - 1u) / tx;  // exact for c < 256
    iny = (65536u + ty - 1u) / ty;
    auto gap_of = [&](uint32_t c) {
      const uint32_t q = (c * inx) >> 16, rr = (q * iny) >> 16;
      return c < tot ? cell_gap2(G, bx + c - q * tx, by + q - rr * ty, bz + rr, sh) : __builtin_inff();
    };
    g0 = gap_of(l);
    g1 = tot > 64u ? gap_of(l + 64u) : __builtin_inff();
    g2 = tot > 128u ? gap_of(l + 128u) : __builtin_inff();
    g3 = tot > 192u ? gap_of(l + 192u) : __builtin_inff();
  };
  if (nchunks) load_chunk(0);
  CellLoad pend{0u, 0u, 0u};
  // the nearest cell still within the radius (next chunks when one is exhausted): its
  // slots are fetched into pend
  auto next_cell = [&]() -> bool {
    for (;;) {
      const float m = wave_min_nonneg(fminf(fminf(g0, g1), fminf(g2, g3)));
      if (m <= r2) {
        const uint64_t b0 = __ballot(g0 == m), b1 = __ballot(g1 == m), b2 = __ballot(g2 == m);
        const uint32_t c = b0 ? (uint32_t)__builtin_ctzll(b0)
                              : b1 ? 64u + (uint32_t)__builtin_ctzll(b1)
                                   : b2 ? 128u + (uint32_t)__builtin_ctzll(b2)
                                        : 192u + (uint32_t)__builtin_ctzll(__ballot(g3 == m));
        if (l == (c & 63u)) {
          const uint32_t slot = c >> 6;
          g0 = slot == 0u ? __builtin_inff() : g0;
          g1 = slot == 1u ? __builtin_inff() : g1;
          g2 = slot == 2u ? __builtin_inff() : g2;
          g3 = slot == 3u ? __builtin_inff() : g3;
        }
        const uint32_t q = (c * inx) >> 16, rr = (q * iny) >> 16;
        pend = fetch_cell(G, bx + c - q * tx, by + q - rr * ty, bz + rr);
        return true;
      }
      if (++chunk >= nchunks) return false;
      load_chunk(chunk);
    }
  };
  RowQ Q{0u, 0u, 0u};
  bool have = false;
  if (scan_all) {
    // every row streams all points
    Q.qe = (l & 15u) == 0u ? n : 0u;
    Q.qn = 1u;
  } else {
    have = next_cell();
    if (!have) return true;
  }

  // cells while a row runs low and no row's queue is full (the radius is re-read first)
  auto refill = [&]() {
    while (have && !__ballot(Q.qn >= 16u) && __ballot(Q.qn <= (uint32_t)LSK_ROWQ_LOW)) {
      if (MODE == MODE_HIST) r2 = cull_r2<MODE>(s, G);
#ifdef LSK_ROWQ_STATS
      G.rq_refills++;
#endif
      cell_rows(G, pend, Q);
      have = fbits(r2) != 0u && next_cell();
    }
    return __ballot(Q.qn > 0u) != 0ull;
  };
  if (!refill()) return true;
  RowPts A = rowq_take(Q, G);
  for (;;) {
    bool more = refill();
    RowPts B = rowq_take(Q, G);
    rowq_eval<MODE>(s, G, A);
    if (MODE == MODE_HIST) {
      shrink_all<MODE>(s, G);
      if (!__ballot(s.state == ST_HIST && s.hi_b > 0u)) break;
    }
    if (!more) break;
    more = refill();
    A = rowq_take(Q, G);
    rowq_eval<MODE>(s, G, B);
    if (MODE == MODE_HIST) {
      shrink_all<MODE>(s, G);
      if (!__ballot(s.state == ST_HIST && s.hi_b > 0u)) break;
    }
    if (!more) break;
  }
  return true;
}
#endif

template <int MODE>
__device__ __forceinline__ bool grid_pass(Lane &s, GridCtx &G, uint32_t n) {
  LSK_GT(tw0);
#if LSK_GRID_ROWQ
  const bool ok = grid_pass_rows<MODE>(s, G, n);
#else
  const bool ok = grid_pass_impl<MODE>(s, G, n);
#endif
  LSK_GADD(G.prof[2 + MODE], tw0);
  return ok;
}

template <int MODE>
__device__ bool grid_pass_impl(Lane &s, GridCtx &G, uint32_t n) {
  float r2 = cull_r2<MODE>(s, G);
  if (fbits(r2) == 0u) return true;
  const uint32_t sh = 10u - G.lc;
  const float r = sqrtf(r2);
  const uint32_t x0 = cell_of(G.wlx - r, G.ox, G.scale, sh), x1 = cell_of(G.whx + r, G.ox, G.scale, sh);
  const uint32_t y0 = cell_of(G.wly - r, G.oy, G.scale, sh), y1 = cell_of(G.why + r, G.oy, G.scale, sh);
  const uint32_t z0 = cell_of(G.wlz - r, G.oz, G.scale, sh), z1 = cell_of(G.whz + r, G.oz, G.scale, sh);
  if ((uint64_t)(x1 - x0 + 1u) * (y1 - y0 + 1u) * (z1 - z0 + 1u) > kMaxCells) {
    if (n > kScanAll) return false;
    process_segment<MODE>(s, G, 0u, n);
    shrink_all<MODE>(s, G);
    return true;
  }
  CellLoad pend{0u, 0u, 0u};
  bool have = false;
  const uint32_t nx = x1 - x0 + 1u, ny = y1 - y0 + 1u, nz = z1 - z0 + 1u;
  if (nx <= 16u && ny <= 16u && nx * ny * nz <= 256u) {
    // Nearest first: lane l holds range cells l, l+64, l+128, l+192 with their gap to the
    // wave box; each round takes the smallest gap still within the (shrinking) radius, so
    // the bounds tighten before the farther cells are reached.
    const uint32_t tot = nx * ny * nz;
    const uint32_t inx = (65536u + nx - 1u) / nx, iny = (65536u + ny - 1u) / ny;  // exact for c < 256
    auto gap_of = [&](uint32_t c) {
      const uint32_t q = (c * inx) >> 16, r = (q * iny) >> 16;
      return c < tot ? cell_gap2(G, x0 + c - q * nx, y0 + q - r * ny, z0 + r, sh) : __builtin_inff();
    };
    const uint32_t l = (uint32_t)G.lane;
    float g0 = gap_of(l), g1 = gap_of(l + 64u), g2 = tot > 128u ? gap_of(l + 128u) : __builtin_inff();
    float g3 = tot > 192u ? gap_of(l + 192u) : __builtin_inff();
    for (;;) {
      const float m = wave_min_nonneg(fminf(fminf(g0, g1), fminf(g2, g3)));
      if (!(m <= r2)) break;
      // the first slot holding the minimum; marked taken (+inf)
      const uint64_t b0 = __ballot(g0 == m), b1 = __ballot(g1 == m), b2 = __ballot(g2 == m);
      const uint32_t c = b0 ? (uint32_t)__builtin_ctzll(b0)
                            : b1 ? 64u + (uint32_t)__builtin_ctzll(b1)
                                 : b2 ? 128u + (uint32_t)__builtin_ctzll(b2)
                                      : 192u + (uint32_t)__builtin_ctzll(__ballot(g3 == m));
      if (l == (c & 63u)) {
        const uint32_t slot = c >> 6;
        g0 = slot == 0u ? __builtin_inff() : g0;
        g1 = slot == 1u ? __builtin_inff() : g1;
        g2 = slot == 2u ? __builtin_inff() : g2;
        g3 = slot == 3u ? __builtin_inff() : g3;
      }
      const uint32_t q = (c * inx) >> 16, r = (q * iny) >> 16;
      const CellLoad cl = fetch_cell(G, x0 + c - q * nx, y0 + q - r * ny, z0 + r);
      if (have) {
        process_cell<MODE>(s, G, pend, r2);
        if (MODE == MODE_HIST) r2 = cull_r2<MODE>(s, G);
        if (fbits(r2) == 0u) return true;
      }
      pend = cl;
      have = true;
    }
    if (have) process_cell<MODE>(s, G, pend, r2);
    return true;
  }
  const uint32_t bx0 = cell_of(G.wlx, G.ox, G.scale, sh), bx1 = cell_of(G.whx, G.ox, G.scale, sh);
  const uint32_t by0 = cell_of(G.wly, G.oy, G.scale, sh), by1 = cell_of(G.why, G.oy, G.scale, sh);
  const uint32_t bz0 = cell_of(G.wlz, G.oz, G.scale, sh), bz1 = cell_of(G.whz, G.oz, G.scale, sh);
  const uint32_t lx = (uint32_t)G.lane & 3u, ly = ((uint32_t)G.lane >> 2) & 3u, lz = (uint32_t)G.lane >> 4;
  for (int phase = 0; phase < 2; phase++) {
    const uint32_t ax = phase ? x0 : bx0, ay = phase ? y0 : by0, az = phase ? z0 : bz0;
    const uint32_t ex = phase ? x1 : bx1, ey = phase ? y1 : by1, ez = phase ? z1 : bz1;
    for (uint32_t oz = az; oz <= ez; oz += 4u)
      for (uint32_t oy = ay; oy <= ey; oy += 4u)
        for (uint32_t ox = ax; ox <= ex; ox += 4u) {
          const uint32_t cx = ox + lx, cy = oy + ly, cz = oz + lz;
          const bool core = cx >= bx0 && cx <= bx1 && cy >= by0 && cy <= by1 && cz >= bz0 && cz <= bz1;
          const bool valid = cx <= ex && cy <= ey && cz <= ez && (phase == 0 || !core);
          const float g2 = valid ? cell_gap2(G, cx, cy, cz, sh) : __builtin_inff();
          uint64_t m = __ballot(g2 <= r2);
          while (m) {
            const int b = __builtin_ctzll(m);
            m &= m - 1ull;
            const float gb = bcast64(g2, (uint32_t)b);
            if (!(gb <= r2)) continue;  // the radius shrank since the test
            // fetch this cell's entries, then process the one fetched before it
            const CellLoad c = fetch_cell(G, ox + ((uint32_t)b & 3u), oy + (((uint32_t)b >> 2) & 3u),
                                          oz + ((uint32_t)b >> 4));
            if (have) {
              process_cell<MODE>(s, G, pend, r2);
                    if (MODE == MODE_HIST) r2 = cull_r2<MODE>(s, G);
              if (fbits(r2) == 0u) return true;
            }
            pend = c;
            have = true;
          }
        }
  }
  if (have) process_cell<MODE>(s, G, pend, r2);
  return true;
}

// One pass over every candidate source: the index's own grid, then (NG = 2: the halo
// re-query of a distributed run) the grid of the received halo points, whose
// cells are walked the same way from the same wave box and (shrinking) radius; the
// histogram / collect pool spans both. G ends on the first grid.
template <int MODE, int NG>
__device__ __forceinline__ bool grid_pass_n(Lane &s, GridCtx &G, const lsk_knn_args &A, const lsk_grid_view &V,
                                            const lsk_grid_view &V1) {
  bool ok = grid_pass<MODE>(s, G, (uint32_t)A.tree[0].n);
  if (NG > 1) {
    load_grid(G, V1, A.tree[1].pts);
    ok = ok && grid_pass<MODE>(s, G, (uint32_t)A.tree[1].n);
    load_grid(G, V, A.tree[0].pts);
  }
  return ok;
}

// STRIDE = false: one wave per group (the normal launch). STRIDE = true: a small persistent
// grid strides over the groups — the form launched when the device gate is expected to
// pick knn_rows: every wave returns at once when it does, instead of millions of blocks
// each being dispatched only to return (1B points: ~16 ms per launch); and, at full
// occupancy, over a group list whose device-side length is far below its bound (a rank's
// boundary groups: ~5 % of its groups).
#ifndef LSK_GRID2_MINW
#define LSK_GRID2_MINW 4  // waves/SIMD of the two-source form (at 6: 393 SGPR / 146 VGPR spills)
#endif
#ifndef LSK_GRID_STRIDE_MINW
#define LSK_GRID_STRIDE_MINW LSK_GRID_MINW
#endif
template <bool STRIDE, int NG>
__global__ __launch_bounds__(kThreads, NG > 1 ? LSK_GRID2_MINW : (STRIDE ? LSK_GRID_STRIDE_MINW : LSK_GRID_MINW)) void knn_grid_kernel(const lsk_knn_args A, const lsk_grid_view V,
                                                                          const lsk_grid_view V1) {
  __shared__ uint32_t lds[kWPB][kPool + 8 * kCullGroups];
  const int wid = threadIdx.x >> 6;
  const int lane = lsk::lane_id();
  if (!STRIDE) {
    const uint32_t nb = lsk::list_blocks(A, gridDim.x, kWPB);
    if (blockIdx.x >= nb) return;
    const uint32_t blk = lsk::xcd_remap(blockIdx.x, nb);
    const uint64_t wave = (uint64_t)blk * kWPB + wid + (uint32_t)A.wave_base;
#include "knn_grid_wave.inc"
  } else {
    if (A.gate && *A.gate != A.gate_on) return;
    uint64_t nwaves = A.groups ? (uint64_t)A.ngroups : (uint64_t)((A.nq + 63) / 64);
    if (A.groups && A.ngroups_dev) nwaves = min(nwaves, (uint64_t)*A.ngroups_dev);
    if (A.wave_end > 0) nwaves = min(nwaves, (uint64_t)A.wave_end);
    // groups: strided, or from the work queue when the launch has one (A.wq)
    const bool dyn = A.wq != nullptr;
    uint64_t w = dyn ? lsk::wq_next(A.wq, (uint32_t)A.wave_base)
                     : (uint64_t)blockIdx.x * kWPB + wid + (uint32_t)A.wave_base;
    while (w < nwaves) {
      [&](const uint64_t wave) {
#include "knn_grid_wave.inc"
      }(w);
      w = dyn ? lsk::wq_next(A.wq, (uint32_t)A.wave_base) : w + (uint64_t)gridDim.x * kWPB;
    }
  }
}

// ------------------------------------------------------------------ grid build
// Runs of the level-g grandchildren (g = lc + 2) along the sorted points. A grandchild's
// slot inside its level-lc cell is bits [6g-..] of its curve key: the 6 key bits below
// the cell's prefix = its rank in curve order among the cell's 64 grandchildren, i.e. in
// memory order (Hilbert and Morton keys alike: every aligned block of 8^l keys is one
// octree cell). Slot = (start, end, x | y << 10 | z << 20 of the grandchild, 0).
__global__ __launch_bounds__(256) void grid_build_kernel(const float *__restrict__ pts,
                                                         const uint32_t *__restrict__ keys, int64_t n,
                                                         const float *__restrict__ box, uint32_t g,
                                                         uint4 *__restrict__ slots) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t ks = 3u * (10u - g);
  const uint32_t kg = keys[i] >> ks;
  const bool first = i == 0 || (keys[i - 1] >> ks) != kg;
  const bool last = i + 1 == n || (keys[i + 1] >> ks) != kg;
  if (!first && !last) return;
  const float ox = box[0], oy = box[1], oz = box[2], sc = box[6];
  const uint32_t sh = 10u - g;
  const uint32_t x = lsk::morton_quant(pts[3 * i], ox, sc) >> sh;
  const uint32_t y = lsk::morton_quant(pts[3 * i + 1], oy, sc) >> sh;
  const uint32_t z = lsk::morton_quant(pts[3 * i + 2], oz, sc) >> sh;
  uint32_t *slot = (uint32_t *)(slots + 64u * lsk::morton3(x >> 2, y >> 2, z >> 2) + (kg & 63u));
  if (first) {
    slot[0] = (uint32_t)i;
    slot[2] = x | (y << 10) | (z << 20);
  }
  if (last) slot[1] = (uint32_t)(i + 1);
}

// counts[l] += number of i in [1, n) whose key prefix at level l (top 3l bits of the
// 30-bit key) differs from key i-1's: distinct cells of level l = counts[l] + 1.
// run > 0: also heavy[0] = 1 if some key equals the key `run` positions before it (an
// over-full cell, knn_engine.refine_heavy_cells) — the same pass over the keys.
// Grid-stride: per-thread counts in registers, wave sums, one atomic per level and block.
constexpr int kLevelsBlocks = 8192;  // 8 waves per SIMD: the key pass is a latency-bound stream (1024: 3.6 ms at 1B)
__global__ __launch_bounds__(256) void key_levels_kernel(const uint32_t *__restrict__ keys, int64_t n,
                                                         unsigned long long *__restrict__ counts, int64_t run,
                                                         int32_t *__restrict__ heavy) {
  uint32_t c[11];
#pragma unroll
  for (int l = 0; l <= 10; l++) c[l] = 0;
  bool hv = false;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x + 1; i < n; i += stride) {
    const uint32_t ki = keys[i];
    const uint32_t x = keys[i - 1] ^ ki;  // differing bits
#pragma unroll
    for (int l = 1; l <= 10; l++) c[l] += (x >> (3 * (10 - l))) != 0u ? 1u : 0u;
    if (run > 0 && i >= run) hv = hv || keys[i - run] == ki;
  }
  if (run > 0 && __ballot(hv) && lsk::lane_id() == 0) heavy[0] = 1;
  __shared__ uint32_t part[11][4];
  const int w = threadIdx.x >> 6;
#pragma unroll
  for (int l = 1; l <= 10; l++) {
    const uint32_t v = lsk::wave_sum(c[l]);
    if (lsk::lane_id() == 0) part[l][w] = v;
  }
  __syncthreads();
  if (threadIdx.x >= 1 && threadIdx.x <= 10) {
    const int l = threadIdx.x;
    const uint32_t v = part[l][0] + part[l][1] + part[l][2] + part[l][3];
    if (v) atomicAdd(&counts[l], (unsigned long long)v);
  }
}

// sum over grandchild slots of (end - start)^2: the mean grandchild population seen by a
// point is this / n (uniform data: about the mean population + 1). Grid-stride, one
// atomic per block.
__global__ __launch_bounds__(256) void grid_sq_kernel(const uint4 *__restrict__ slots, int64_t nslot,
                                                      unsigned long long *__restrict__ out) {
  unsigned long long v = 0;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nslot; i += stride) {
    const uint4 t = slots[i];
    const unsigned long long d = t.y > t.x ? (unsigned long long)(t.y - t.x) : 0ull;
    v += d * d;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  __shared__ unsigned long long part[4];
  if (lsk::lane_id() == 0) part[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned long long t = part[0] + part[1] + part[2] + part[3];
    if (t) atomicAdd(out, t);
  }
}

__global__ void grid_decide_kernel(const unsigned long long *__restrict__ counts,
                                   const unsigned long long *__restrict__ sq, int64_t n, int32_t g, float crowd,
                                   int32_t check, int32_t *__restrict__ gate) {
  if (threadIdx.x != 0) return;
  int32_t ok = 1;
  if (check) {
    // distinct cells of level l = counts[l] + 1 (adjacent sorted keys that differ)
    const double dg = (double)counts[g] + 1.0, dg1 = g >= 2 ? (double)counts[g - 1] + 1.0 : 1.0;
    const double mean = (double)n / dg;
    const double seen = (double)sq[0] / (double)(n > 0 ? n : 1);
    ok = (dg >= 6.0 * dg1 && mean >= 2.0 && mean <= 256.0 && seen <= (double)crowd * (mean + 1.0)) ? 1 : 0;
  }
  gate[0] = ok;
}

}  // namespace

extern "C" int lsk_hip_grid_decide(const unsigned long long *counts, const unsigned long long *sq, int64_t n,
                                   int32_t g, float crowd, int32_t check, int32_t *gate, void *stream) {
  if (g < 2 || g > 10) {
    lsk::set_last_error("grid_decide: grandchild level must be in [2, 10]");
    return 1;
  }
  grid_decide_kernel<<<1, 64, 0, (hipStream_t)stream>>>(counts, sq, n, g, crowd, check, gate);
  LSK_CHECK_LAUNCH("grid_decide");
  return 0;
}

extern "C" int lsk_hip_grid_build(const float *sorted_pts, const uint32_t *sorted_keys, int64_t n,
                                  const float *box, int32_t level, uint32_t *slots, void *stream) {
  if (level < 0 || level > 8) {
    lsk::set_last_error("grid_build: level must be in [0, 8] (grandchildren at level + 2 <= 10)");
    return 1;
  }
  if (n >= ((int64_t)1 << 32)) {
    lsk::set_last_error("grid_build: n must be < 2^32");
    return 1;
  }
  const size_t nslot = (size_t)64 << (3 * level);
  hipStream_t st = (hipStream_t)stream;
  LSK_HIP(lsk_fill32(slots, 0u, (int64_t)nslot * 4, st));
  if (n <= 0) return 0;
  grid_build_kernel<<<lsk_blocks(n, 256), 256, 0, st>>>(sorted_pts, sorted_keys, n, box, (uint32_t)level + 2u,
                                                        (uint4 *)slots);
  LSK_CHECK_LAUNCH("grid_build");
  return 0;
}

extern "C" int lsk_hip_key_levels(const uint32_t *keys, int64_t n, unsigned long long *counts, void *stream) {
  hipStream_t st = (hipStream_t)stream;
  LSK_HIP(lsk_fill32(counts, 0u, 22, st));
  if (n <= 1) return 0;
  key_levels_kernel<<<lsk_blocks(n, 256, kLevelsBlocks), 256, 0, st>>>(keys, n, counts, 0, nullptr);
  LSK_CHECK_LAUNCH("key_levels");
  return 0;
}

// (counts and heavy are zeroed by the caller: tiny hipMemsetAsync nodes in a captured HIP
// graph were seen not to re-zero them on later replays — ROCm 7.0, 88 and 4 bytes)
extern "C" int lsk_hip_key_census(const uint32_t *keys, int64_t n, unsigned long long *counts, int64_t run,
                                  int32_t *heavy, void *stream) {
  hipStream_t st = (hipStream_t)stream;
  if (n <= 1) return 0;
  key_levels_kernel<<<lsk_blocks(n, 256, kLevelsBlocks), 256, 0, st>>>(keys, n, counts, run, heavy);
  LSK_CHECK_LAUNCH("key_census");
  return 0;
}

extern "C" int lsk_hip_grid_sq(const uint32_t *slots, int64_t nslot, unsigned long long *out, void *stream) {
  hipStream_t st = (hipStream_t)stream;
  if (nslot <= 0) return 0;
  grid_sq_kernel<<<lsk_blocks(nslot, 256, kLevelsBlocks), 256, 0, st>>>((const uint4 *)slots, nslot, out);
  LSK_CHECK_LAUNCH("grid_sq");
  return 0;
}

static int knn_grid_launch(const lsk_knn_args *args, const lsk_grid_view *grid, const lsk_grid_view *grid1,
                           void *stream) {
  const lsk_knn_args &A = *args;
  if (A.k < 1 || A.k > 65535) {
    lsk::set_last_error("knn_grid: k must be in [1, 65535]");
    return 1;
  }
  const int ng = grid1 ? 2 : 1;
  if (A.nq >= ((int64_t)1 << 32) || A.ntrees != ng || (ng == 1 && A.init_d2) || A.tree[0].n >= ((int64_t)1 << 32) ||
      (ng == 2 && A.tree[1].n >= ((int64_t)1 << 32)) || !grid || grid->level < 0 || grid->level > 8 ||
      (grid1 && (grid1->level < 0 || grid1->level > 8))) {
    lsk::set_last_error("knn_grid: one tree and grid (< 2^32 points, the queries' own; no init_d2), or two "
                        "(knn_grid2: + the halo's), grid levels in [0, 8]");
    return 1;
  }
  const int64_t ngroups = A.groups ? A.ngroups : (A.nq + 63) / 64;
  // this launch's waves: [wave_base, wave_end or ngroups)
  const int64_t wend = A.wave_end > 0 && A.wave_end < ngroups ? A.wave_end : ngroups;
  if (A.wave_base < 0 || wend - A.wave_base <= 0) return 0;
  const unsigned nblk = lsk_blocks(wend - A.wave_base, kWPB);
  const unsigned cap = A.pad2 == 2 ? kStrideBlocksFull : kStrideBlocks;
  const unsigned sblk = nblk < cap ? nblk : cap;
  hipStream_t st = (hipStream_t)stream;
  if (ng == 2) {  // (the halo re-query: a device-counted list, persistent or full form)
    if (A.pad2 >= 1)
      knn_grid_kernel<true, 2><<<sblk, kThreads, 0, st>>>(A, *grid, *grid1);
    else
      knn_grid_kernel<false, 2><<<nblk, kThreads, 0, st>>>(A, *grid, *grid1);
  } else if (A.pad2 >= 1) {  // persistent strided form (see knn_grid_kernel); 2: a short list
    knn_grid_kernel<true, 1><<<sblk, kThreads, 0, st>>>(A, *grid, *grid);
  } else {
    knn_grid_kernel<false, 1><<<nblk, kThreads, 0, st>>>(A, *grid, *grid);
  }
  LSK_CHECK_LAUNCH("knn_grid");
  return 0;
}

extern "C" int lsk_hip_knn_grid(const lsk_knn_args *args, const lsk_grid_view *grid, void *stream) {
  return knn_grid_launch(args, grid, nullptr, stream);
}

// The halo re-query on the grid: args->tree[1] / grid1 are the received halo
// points' index and grid; args->init_d2 (optional) the local k-th as an upper bound.
extern "C" int lsk_hip_knn_grid2(const lsk_knn_args *args, const lsk_grid_view *grid, const lsk_grid_view *grid1,
                                 void *stream) {
  if (!grid1) {
    lsk::set_last_error("knn_grid2: the halo grid view is required");
    return 1;
  }
  return knn_grid_launch(args, grid, grid1, stream);
}
