// k-th-NN distance on the cell grid with MFMA-screened candidates (round 5).
//
// Same contract as knn_grid.hip (one tree whose points are the queries, the octree grid
// of grandchild runs, the failure list + knn_exact.hip backstop, fused output scatter;
// reference runQuery / extractFinalResult, unorderedDataVariant.cu:75-103), a different
// inner loop:
//
//  * a wave owns 32 curve-consecutive queries (half a 64-query group; a 2-wave block is one
//    group). Lanes l and l+32 hold query l & 31;
//  * candidates come in TILES of 32 points (runs of the sorted array: the needed
//    grandchild runs of the grid cells around the queries, packed across runs and cells);
//    one v_mfma_f32_32x32x16_f16 gives all 32 x 32 squared distances of a tile at once:
//    d² = |q|² + |p|² - 2 q·p on wave-centred, power-of-2-scaled coordinates, each split
//    into two f16 halves (x = xh + xl, RTZ), so every product is exact in f32 and the sum
//    carries ~2^-20 of relative error. The VALU does no distance arithmetic at all;
//  * the MFMA value a is an APPROXIMATION. It is biased by +delta (a bound on its error
//    against the canonical fp32 d², from the pass's largest |q'| + |p'|), so a >= S²·d²
//    canonical and a <= S²·d² + 2 delta. Per query the pass has a band [L, H) of squared
//    distances (from the density prior, sized so that the k-th lies inside with high
//    probability): a < L·S² counts as certainly below L; a in [L·S², H·S² + 2 delta)
//    appends the candidate's index to the query's band list in LDS; anything above is
//    certainly >= H. Per value: 2 compares, a carry-add, a shift-add (4 VALU);
//  * after the pass every band entry gets its EXACT canonical d² (gathered point,
//    common.h dist2); with the exact count below L the k-th is selected among the exact
//    band values (8 sub-bands, then a 32-value bitonic network) — bit-identical to the CPU
//    oracle. A query whose k-th is outside its band (or whose list overflowed) runs
//    another pass with a moved band; the other queries of the wave stay done, and the
//    pass streams only the cells around the unresolved queries. After kMaxPasses the
//    query goes to the failure list (exact backstop).
//
// Measured micro facts behind the design (scripts/micro/, profiles/r5_micro): the f32
// MFMA shares the VALU's datapath (no overlap), the f16 MFMA costs ~35 SIMD-cycles per
// 1024 pairs beside VALU work, an exec-masked ds_write costs the same at any lane density
// (so appends go through a per-lane bit mask and a loop over the wave's max count), and
// the f16 products are exact (hi/lo splits with explicit RTZ conversion: two conversion
// paths can round a tie differently).
#include "dev.h"

namespace {

using lsk::bitsf;
using lsk::fbits;

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

#ifndef LSK_MF_CAPQ
#define LSK_MF_CAPQ 96
#endif
#ifndef LSK_MF_Z10
#define LSK_MF_Z10 35  // band half-width in tenths of sqrt(k) standard deviations
#endif
#ifndef LSK_MF_MINW
#define LSK_MF_MINW 3
#endif
// LSK_MF_PROFILE builds (tuning only): shader-clock cycles per wave in pass setup, the
// tile stream, the exact values, decide + selection, and append-loop rounds / tiles, into
// stats[16..21] (knn_engine.KnnStats prof_* names).
#ifdef LSK_MF_PROFILE
#define MF_T(v) const uint64_t v = __builtin_readcyclecounter()
#define MF_ADD(i, t0) prof[i] += __builtin_readcyclecounter() - (t0)
#else
#define MF_T(v)
#define MF_ADD(i, t0)
#endif
#ifndef LSK_MF_EXP
#define LSK_MF_EXP 0  // tuning experiments (wrong results): 1 no point loads, 2 no band work, 3 both
#endif
constexpr int kQ = 32;                      // queries per wave
constexpr int kWPB = 2;                     // waves per block (= one 64-query group)
constexpr int kThreads = kWPB * lsk::kWave;
constexpr uint32_t kCapQ = LSK_MF_CAPQ;     // band entries per query (both halves)
constexpr uint32_t kStride = kCapQ + 1;     // LDS dwords per query (bank spread)
constexpr uint32_t kMaxPasses = 6;
constexpr uint32_t kMaxCells = 4096;
constexpr uint32_t kNaNBits = 0x7fc00000u;
constexpr unsigned kStrideBlocks = 2048;
constexpr unsigned kStrideBlocksFull = 8192;

enum : uint32_t {
  QS_OVERFLOW = 1, QS_UNDERFLOW = 2, QS_REFINE = 4, QS_DONE_BAND1 = 32, QS_DONE_CUT = 64, QS_LIMIT = 256,
  QS_MISMATCH = 512, QS_HINT = 1024, QS_BINOVF = 2048, QS_FAIL = 4096
};

// ---------------------------------------------------------------- small wave helpers
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xf, 0xf, false));
}
// the value of the partner lane (l ^ 32)
__device__ __forceinline__ uint32_t partner_u(uint32_t v) { return (uint32_t)__shfl_xor((int)v, 32); }
__device__ __forceinline__ float umax_f(float v) {  // wave max of non-negative floats
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
  return lsk::uniform_f(v);
}

// -------------------------------------------------------------------- grid geometry
struct Geo {
  const float *pts;
  const uint4 *slots;
  float ox, oy, oz, scale, step, eps;
  uint32_t lc;
};

__device__ __forceinline__ uint32_t cell_of(float v, float o, float scale, uint32_t sh) {
  return lsk::morton_quant(v, o, scale) >> sh;
}
__device__ __forceinline__ void cell_span(const Geo &G, float o, uint32_t c, uint32_t sh, float &lo, float &hi) {
  const uint32_t last = 1023u >> sh;
  lo = c == 0 ? -__builtin_inff() : o + (float)(c << sh) * G.step - G.eps;
  hi = c >= last ? __builtin_inff() : o + (float)((c + 1u) << sh) * G.step + G.eps;
}
__device__ __forceinline__ float gap1(float lo, float hi, float wl, float wh) {
  return fmaxf(0.f, fmaxf(lo - wh, wl - hi));
}

struct QBox {
  float lx, ly, lz, hx, hy, hz;
};
__device__ __forceinline__ float cell_gap2(const Geo &G, const QBox &B, uint32_t x, uint32_t y, uint32_t z,
                                           uint32_t sh) {
  float lx, hx, ly, hy, lz, hz;
  cell_span(G, G.ox, x, sh, lx, hx);
  cell_span(G, G.oy, y, sh, ly, hy);
  cell_span(G, G.oz, z, sh, lz, hz);
  return lsk::dist2(gap1(lx, hx, B.lx, B.hx), gap1(ly, hy, B.ly, B.hy), gap1(lz, hz, B.lz, B.hz));
}

// ------------------------------------------------------------ split-f16 fragments
__device__ __forceinline__ uint32_t pk_rtz(float a, float b) {
  return __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_pkrtz(a, b));
}
__device__ __forceinline__ float lo16f(uint32_t p) {
  return (float)__builtin_bit_cast(_Float16, (uint16_t)(p & 0xffffu));
}
__device__ __forceinline__ float hi16f(uint32_t p) {
  return (float)__builtin_bit_cast(_Float16, (uint16_t)(p >> 16));
}
// (u, v) -> hi = (uh, vh), lo = (ul, vl), RTZ both: u = uh + ul + e, |e| < 2^-20 |u| (+2^-24)
__device__ __forceinline__ void split2(float u, float v, uint32_t &hi, uint32_t &lo) {
  hi = pk_rtz(u, v);
  lo = pk_rtz(u - lo16f(hi), v - hi16f(hi));
}
__device__ __forceinline__ f16x8 as_frag(uint32_t d0, uint32_t d1, uint32_t d2, uint32_t d3) {
  u32x4 v = {d0, d1, d2, d3};
  return __builtin_bit_cast(f16x8, v);
}
constexpr uint32_t kOnes16 = 0x3C003C00u;  // (1.0, 1.0) in f16

// Point loads the compiler does not see as loads: issued unconditionally (it cannot sink a
// load into the one path that uses it, which would leave other paths with fewer younger
// loads and force vmcnt(0)), waited for by hand with a count that holds on every path.
// Valid only in a build without VGPR spills (the compiler could spill the destination
// before the hand-placed wait): the production build has none (MINW 3); a MINW 6 probe
// with 58 spilled VGPRs faulted (profiles/r5_mfma/occupancy_gband.log).
typedef float f32x3 __attribute__((ext_vector_type(3)));
__device__ __forceinline__ f32x3 ld_point(const float *pts, uint32_t i) {
  f32x3 v;
  asm volatile("global_load_dwordx3 %0, %1, off" : "=v"(v) : "v"(pts + 3ull * i) : "memory");
  return v;
}
// all but the two youngest vector-memory operations done; the operands are the registers
// the wait makes valid (no use of them can move above it)
__device__ __forceinline__ void wait_vm2(f32x3 &a, f32x3 &b) {
  asm volatile("s_waitcnt vmcnt(2)" : "+v"(a), "+v"(b) : : "memory");
}

// A fragment of candidate (px, py, pz) (centred, scaled) for this lane's half h of K:
// h = 0: [xh xl xh xl yh yl yh yl]; h = 1: [zh zl zh zl pph ppl 1 1] (pp = |p|²).
__device__ __forceinline__ f16x8 frag_a(float px, float py, float pz, bool upper) {
  const float pp = lsk::dist2(px, py, pz);
  const float u = upper ? pz : px, v = upper ? pp : py;
  uint32_t hi, lo;
  split2(u, v, hi, lo);
  const uint32_t du = __builtin_amdgcn_perm(lo, hi, 0x05040100u);  // (uh, ul)
  const uint32_t dv = __builtin_amdgcn_perm(lo, hi, 0x07060302u);  // (vh, vl)
  return as_frag(du, du, dv, upper ? kOnes16 : dv);
}
// B fragment of query (qx, qy, qz) (centred, scaled), qq = |q|² + delta:
// h = 0: [-2xh -2xh -2xl -2xl -2yh -2yh -2yl -2yl]; h = 1: [-2zh -2zh -2zl -2zl 1 1 qqh qql]
__device__ __forceinline__ f16x8 frag_b(float qx, float qy, float qz, float qq, bool upper) {
  const float u = -2.f * (upper ? qz : qx), v = -2.f * qy;
  uint32_t hi, lo;
  split2(u, v, hi, lo);
  const uint32_t uh2 = __builtin_amdgcn_perm(hi, hi, 0x01000100u);  // (uh, uh)
  const uint32_t ul2 = __builtin_amdgcn_perm(lo, lo, 0x01000100u);  // (ul, ul)
  const uint32_t vh2 = __builtin_amdgcn_perm(hi, hi, 0x03020302u);
  const uint32_t vl2 = __builtin_amdgcn_perm(lo, lo, 0x03020302u);
  uint32_t qh, ql;
  split2(qq, 0.f, qh, ql);
  const uint32_t qd = (qh & 0xffffu) | (ql << 16);  // (qqh, qql)
  return as_frag(uh2, ul2, upper ? kOnes16 : vh2, upper ? qd : vl2);
}

// -------------------------------------------------------------- candidate stream
// Cells of level lc around the box, culled by their gap to the box; per cell the 64
// grandchild slots (lane j: slot j, curve order = memory order), the needed ones (gap to
// the box <= R) form runs; runs are packed into 32-point tiles (up to 4 pieces per tile).
struct CellIter {
  uint32_t x0, y0, z0, x1, y1, z1;  // cell range (inclusive)
  uint32_t bx, by, bz;              // next 4x4x4 block to test
  uint32_t mx, my, mz;              // origin of the block bmask belongs to
  uint64_t bmask;                   // culled cells of that block not yet taken
  bool done;
};

struct Stream {
  // current cell (its masks) and the next two (slots in flight: a cell change inside the
  // tile builder waits for its slots, and with them for every older load)
  uint64_t need, free_;
  uint32_t ca, ce, cxyz;     // per lane: slots of the current cell
  uint32_t na, ne, nxyz;     // per lane: slots of the next cell
  uint32_t ma, me, mxyz;     // per lane: slots of the cell after it
  bool have_next, have_next2;
  uint32_t si, se;  // current segment (sorted-array range)
};

}  // namespace

namespace {

struct Wave {
  Geo G;
  QBox B;
  float R2;
  uint32_t sh_c, sh_g;  // cell / grandchild quantisation shifts
  uint32_t nmax;        // last valid point index
  int lane;
};

__device__ __forceinline__ bool next_cell(Wave &W, CellIter &I, uint32_t &cx, uint32_t &cy, uint32_t &cz) {
  for (;;) {
    if (I.bmask) {
      const uint32_t b = (uint32_t)__builtin_ctzll(I.bmask);
      I.bmask &= I.bmask - 1ull;
      cx = I.mx + (b & 3u);
      cy = I.my + ((b >> 2) & 3u);
      cz = I.mz + (b >> 4);
      return true;
    }
    if (I.done) return false;
    // next block
    const uint32_t l = (uint32_t)W.lane;
    const uint32_t x = I.bx + (l & 3u), y = I.by + ((l >> 2) & 3u), z = I.bz + (l >> 4);
    const bool in = x <= I.x1 && y <= I.y1 && z <= I.z1;
    const float g2 = in ? cell_gap2(W.G, W.B, x, y, z, W.sh_c) : __builtin_inff();
    I.bmask = __ballot(g2 <= W.R2);
    I.mx = I.bx;
    I.my = I.by;
    I.mz = I.bz;
    I.bx += 4u;
    if (I.bx > I.x1) {
      I.bx = I.x0;
      I.by += 4u;
      if (I.by > I.y1) {
        I.by = I.y0;
        I.bz += 4u;
        if (I.bz > I.z1) I.done = true;
      }
    }
  }
}

__device__ __forceinline__ void fetch_cell(const Wave &W, uint32_t cx, uint32_t cy, uint32_t cz, uint32_t &a,
                                           uint32_t &e, uint32_t &xyz) {
  // (cells come from the clamped range: the guard only keeps a bad coordinate in bounds)
  const uint32_t cmax = (1u << W.G.lc) - 1u;
  const uint4 v = W.G.slots[64u * lsk::morton3(min(cx, cmax), min(cy, cmax), min(cz, cmax)) + (uint32_t)W.lane];
  a = v.x;
  e = v.y;
  xyz = v.z;
}

// masks of the current cell: needed = non-empty and within R of the box
__device__ __forceinline__ void cell_masks(const Wave &W, Stream &S) {
  const bool ne = S.ce > S.ca;
  const uint64_t nonempty = __ballot(ne);
  float lx, hx, ly, hy, lz, hz;
  cell_span(W.G, W.G.ox, S.cxyz & 1023u, W.sh_g, lx, hx);
  cell_span(W.G, W.G.oy, (S.cxyz >> 10) & 1023u, W.sh_g, ly, hy);
  cell_span(W.G, W.G.oz, S.cxyz >> 20, W.sh_g, lz, hz);
  const float g2 = lsk::dist2(gap1(lx, hx, W.B.lx, W.B.hx), gap1(ly, hy, W.B.ly, W.B.hy),
                              gap1(lz, hz, W.B.lz, W.B.hz));
  S.need = __ballot(ne && g2 <= W.R2);
  S.free_ = S.need | ~nonempty;
}

// advance to the next cell with something needed; false at the end of the stream
__device__ __forceinline__ bool advance_cell(Wave &W, CellIter &I, Stream &S) {
  for (;;) {
    if (!S.have_next) return false;
    S.ca = S.na;
    S.ce = S.ne;
    S.cxyz = S.nxyz;
    S.na = S.ma;
    S.ne = S.me;
    S.nxyz = S.mxyz;
    S.have_next = S.have_next2;
    uint32_t cx, cy, cz;
    S.have_next2 = S.have_next2 && next_cell(W, I, cx, cy, cz);
    if (S.have_next2) fetch_cell(W, cx, cy, cz, S.ma, S.me, S.mxyz);
    cell_masks(W, S);
    if (S.need) return true;
  }
}

// next segment [si, se) of the stream; false at the end
__device__ __forceinline__ bool next_segment(Wave &W, CellIter &I, Stream &S) {
  if (!S.need && !advance_cell(W, I, S)) return false;
  const uint32_t t0 = (uint32_t)__builtin_ctzll(S.need);
  const uint64_t after = ~S.free_ >> t0;
  const uint32_t len = after ? (uint32_t)__builtin_ctzll(after) : 64u - t0;
  const uint64_t run = (len >= 64u ? ~0ull : ((1ull << len) - 1ull)) << t0;
  const uint64_t in = S.need & run;
  const uint32_t t1 = 63u - (uint32_t)__builtin_clzll(in);
  S.need &= ~run;
  S.si = lsk::uniform((uint32_t)__builtin_amdgcn_readlane((int)S.ca, (int)t0));
  S.se = lsk::uniform((uint32_t)__builtin_amdgcn_readlane((int)S.ce, (int)t1));
  return true;
}

// One tile: up to 32 stream positions in up to 4 pieces; row i of the tile is candidate
// base(i) + i, base(i) = b_p of the last piece p with o_p <= i (o_0 = 0). Lane i (= lane &
// 31) gets its candidate index; false (no tile) at the end of the stream.
struct Tile {  // (kept as scalars: a struct the compiler spills gets selected through scratch)
  uint32_t o1, o2, o3, b0, b1, b2, b3;
};
__device__ __forceinline__ uint32_t tile_base(uint32_t o1, uint32_t o2, uint32_t o3, uint32_t b0, uint32_t b1,
                                              uint32_t b2, uint32_t b3, uint32_t row) {
  // b_p of the last piece with o_p <= row, as a sum of deltas (values, not a lookup)
  return b0 + (row >= o1 ? b1 - b0 : 0u) + (row >= o2 ? b2 - b1 : 0u) + (row >= o3 ? b3 - b2 : 0u);
}
__device__ __forceinline__ bool next_tile(Wave &W, CellIter &I, Stream &S, uint32_t &o1, uint32_t &o2,
                                          uint32_t &o3, uint32_t &b0, uint32_t &b1, uint32_t &b2, uint32_t &b3,
                                          uint32_t &idx, bool &cv) {
  uint32_t o = 0, k = 0;
  uint32_t t1 = 32u, t2 = 32u, t3 = 32u, c0 = 0u, c1 = 0u, c2 = 0u, c3 = 0u;
  while (o < 32u && k < 4u) {
    if (S.si >= S.se && !next_segment(W, I, S)) break;
    const uint32_t m = min(32u - o, S.se - S.si);
    const uint32_t base = S.si - o;
    if (k == 0) c0 = base;
    else if (k == 1) { t1 = o; c1 = base; }
    else if (k == 2) { t2 = o; c2 = base; }
    else { t3 = o; c3 = base; }
    S.si += m;
    o += m;
    k++;
  }
  o1 = lsk::uniform(t1);
  o2 = lsk::uniform(t2);
  o3 = lsk::uniform(t3);
  b0 = lsk::uniform(c0);
  b1 = lsk::uniform(c1);
  b2 = lsk::uniform(c2);
  b3 = lsk::uniform(c3);
  if (o == 0) return false;
  const uint32_t i = (uint32_t)W.lane & 31u;
  cv = i < o;
  idx = cv ? tile_base(o1, o2, o3, b0, b1, b2, b3, i) + i : b0;
  idx = min(idx, W.nmax);  // (runs come from the grid: only a corrupt table reaches past n)
  return true;
}

}  // namespace

namespace {

// band of a query: [L, H) of squared distances (floats)
__device__ __forceinline__ void band_from(float E, float kf, float z, float &L, float &H) {
  const float s = z * sqrtf(kf);
  const float lo = fmaxf(kf - s, 0.f) / kf, hi = (kf + s) / kf;
  L = E * __builtin_powf(lo, 2.f / 3.f);
  H = E * __builtin_powf(hi, 2.f / 3.f);
}

// Expected k-th squared distance of a query near the data box's faces: the ball of
// radius r loses a spherical cap (volume fraction (1-t)^2 (2+t) / 4, t = d / r) beyond each
// face closer than r, so r grows by f^(-1/3) (f = the product of the kept fractions; one
// fixed-point step from the uniform estimate). Interior queries keep E.
__device__ __forceinline__ float boundary_est(float E, const float q[3], const float lo[3], const float hi[3]) {
  const float r0 = sqrtf(E);
  float r = r0, f = 1.f;
#pragma unroll
  for (int it = 0; it < 2; it++) {
    f = 1.f;
#pragma unroll
    for (int a = 0; a < 3; a++) {
      const float d = fmaxf(fminf(q[a] - lo[a], hi[a] - q[a]), 0.f);
      const float t = fminf(d / r, 1.f);
      f *= 1.f - (1.f - t) * (1.f - t) * (2.f + t) * 0.25f;
    }
    f = fmaxf(f, 0.125f);
    r = r0 * __builtin_powf(f, -1.f / 3.f);
  }
  return E * __builtin_powf(f, -2.f / 3.f);
}

__device__ __forceinline__ void net32_select(uint32_t *v, uint32_t m, uint32_t &out) {
#pragma unroll
  for (int kk = 2; kk <= 32; kk <<= 1) {
#pragma unroll
    for (int j = kk >> 1; j > 0; j >>= 1) {
#pragma unroll
      for (int i = 0; i < 32; i++) {
        const int l = i ^ j;
        if (l > i) {
          const uint32_t a = v[i], b = v[l];
          const bool up = (i & kk) == 0;
          v[i] = up ? min(a, b) : max(a, b);
          v[l] = up ? max(a, b) : min(a, b);
        }
      }
    }
  }
  uint32_t r = v[0];
#pragma unroll
  for (int i = 1; i < 32; i++) r = ((uint32_t)i == m - 1u) ? v[i] : r;
  out = r;
}

#ifndef LSK_MF_GBAND
#define LSK_MF_GBAND 0  // tuning: band lists in global memory (an occupancy probe: no LDS limit)
#endif
#if LSK_MF_GBAND
#define BAND(jj, e) gband[(size_t)(e) * kQ + (jj)]
#else
#define BAND(jj, e) region[(jj) * kStride + (e)]
#endif

template <bool STRIDE>
__global__ __launch_bounds__(kThreads, LSK_MF_MINW) void knn_mfma_kernel(const lsk_knn_args A, const lsk_grid_view V,
                                                                         uint32_t *gband_all) {
  // per wave: the band lists (32 queries x kStride dwords), then the current tile's points
  // (32 x float3: the append loop computes the exact d² of a band candidate from it)
#ifndef LSK_MF_LDSPAD
#define LSK_MF_LDSPAD 0  // tuning: extra LDS dwords per wave (an occupancy probe)
#endif
#if LSK_MF_GBAND
  __shared__ uint32_t lds[kWPB][6 * kQ + LSK_MF_LDSPAD];
#else
  __shared__ uint32_t lds[kWPB][kQ * kStride + 6 * kQ + LSK_MF_LDSPAD];
#endif
  const int wid = threadIdx.x >> 6;
  const int lane = lsk::lane_id();
  if (A.gate && *A.gate != A.gate_on) return;  // the device chose another kernel
  const uint64_t ngroups = A.groups ? (uint64_t)A.ngroups : (uint64_t)((A.nq + 63) / 64);
  uint64_t gend = ngroups;
  if (A.groups && A.ngroups_dev) gend = min(gend, (uint64_t)*A.ngroups_dev);
  if (A.wave_end > 0) gend = min(gend, (uint64_t)A.wave_end);
  const uint32_t nb = STRIDE ? gridDim.x : lsk::list_blocks(A, gridDim.x, 1u);
  if (blockIdx.x >= nb) return;
  uint64_t g = STRIDE ? (uint64_t)blockIdx.x + (uint32_t)A.wave_base
                      : (uint64_t)lsk::xcd_remap(blockIdx.x, nb) + (uint32_t)A.wave_base;
  uint64_t gstep = gridDim.x;
#if LSK_MF_GBAND
  // persistent blocks, XCD-aware: the blocks of XCD x (blockIdx % 8, the dispatch order)
  // walk the x-th eighth of the groups
  if (STRIDE && (gridDim.x & 7u) == 0u) {
    const uint64_t nall = gend - (uint64_t)(uint32_t)A.wave_base, x = blockIdx.x & 7u;
    const uint64_t lo = (uint32_t)A.wave_base + nall * x / 8u, hi = (uint32_t)A.wave_base + nall * (x + 1u) / 8u;
    g = lo + (blockIdx.x >> 3);
    gend = hi;
    gstep = gridDim.x >> 3;
  }
#endif
#if LSK_MF_GBAND
  uint32_t *gband = gband_all + ((size_t)blockIdx.x * kWPB + (size_t)wid) * kQ * kCapQ;
  float *stage = (float *)lds[wid];
#else
  (void)gband_all;
  uint32_t *region = lds[wid];
  float *stage = (float *)(lds[wid] + kQ * kStride);
#endif
  const bool upper = lane >= 32;
  const uint32_t j = (uint32_t)lane & 31u;
  const uint32_t k = (uint32_t)A.k;
  const float kf = (float)k;
  const float z = (float)LSK_MF_Z10 * 0.1f;

  Wave W;
  W.lane = lane;
  W.G.pts = A.tree[0].pts;
  W.G.slots = (const uint4 *)V.slots;
  {
    const lsk::cfloat_p bx = lsk::as_const(V.box);
    W.G.ox = bx[0];
    W.G.oy = bx[1];
    W.G.oz = bx[2];
    W.G.scale = bx[6];
    const float ext = bx[7];
    W.G.step = ext * (1.f / 1024.f);
    const float mag = fmaxf(fmaxf(fabsf(W.G.ox), fabsf(W.G.oy)), fabsf(W.G.oz)) + ext;
    W.G.eps = mag * 0x1p-19f;
  }
  W.G.lc = (uint32_t)V.level;
  W.nmax = (uint32_t)(A.tree[0].n > 0 ? A.tree[0].n - 1 : 0);
  W.sh_c = 10u - W.G.lc;
  W.sh_g = 10u - (W.G.lc + 2u);
  // grandchild cell diagonal (an upper bound on any candidate's distance to its own cell)
  const float gdiag = 1.7320508f * W.G.step * (float)(1u << W.sh_g) + 2.f * W.G.eps;
  float r_est2 = A.r_hint2 >= 0.f ? A.r_hint2 : A.tree[0].nodes[3];
  if (!(r_est2 > 0.f) || !(r_est2 < __builtin_inff())) r_est2 = 1.f;
  const float cut2 = (A.cut2 == A.cut2) ? fmaxf(A.cut2, 0.f) : __builtin_inff();
  const uint32_t cut_b = fbits(cut2);

  for (; g < gend; g += STRIDE ? gstep : gend) {
    const uint32_t grp = lsk::uniform(A.groups ? A.groups[g] : (uint32_t)g);
    const int64_t q0 = (int64_t)grp * lsk::kBucket + (int64_t)wid * kQ;
    const int64_t qi = q0 + (int64_t)j;
    const bool valid = qi < A.nq;
    const float qx = valid ? A.qpts[3 * qi] : 0.f, qy = valid ? A.qpts[3 * qi + 1] : 0.f,
                qz = valid ? A.qpts[3 * qi + 2] : 0.f;
    uint32_t qs = QS_HINT;
    // state: 0 active, 1 done; res = answer bits
    bool done = !valid;
    uint32_t res = 0;
    float L = 0.f, H = 0.f;
    if (valid) {
      if (A.tree[0].n < (int64_t)k) {
        done = true;
        res = cut_b;
        qs |= QS_DONE_CUT;
      } else {
        const float qv[3] = {qx, qy, qz}, blo[3] = {V.box[0], V.box[1], V.box[2]},
                    bhi[3] = {V.box[3], V.box[4], V.box[5]};
        band_from(boundary_est(r_est2, qv, blo, bhi), kf, z, L, H);
        if (H >= cut2) H = cut2;
        if (!(H > L)) L = 0.f;
      }
    }
    uint32_t passes = 0, evals = 0;
#ifdef LSK_MF_PROFILE
    uint64_t prof[6] = {0, 0, 0, 0, 0, 0};
#endif
    for (;;) {
      const bool act = !done;
      if (!__ballot(act)) break;
      if (passes >= kMaxPasses) {
        if (act) {
          done = true;
          res = kNaNBits;
          qs |= QS_LIMIT | QS_FAIL;
        }
        break;
      }
      passes++;
      MF_T(tp0);
      // ---- pass geometry: box of the unresolved queries, radius = their largest H
      const float inf = __builtin_inff();
      W.B.lx = lsk::wave_min(act ? qx : inf);
      W.B.ly = lsk::wave_min(act ? qy : inf);
      W.B.lz = lsk::wave_min(act ? qz : inf);
      W.B.hx = lsk::wave_max(act ? qx : -inf);
      W.B.hy = lsk::wave_max(act ? qy : -inf);
      W.B.hz = lsk::wave_max(act ? qz : -inf);
      const float Hmax = umax_f(act ? H : 0.f);
      const float R = sqrtf(Hmax) * (1.f + 0x1p-16f) + W.G.eps;
      W.R2 = R * R;
      const float cx = 0.5f * (W.B.lx + W.B.hx), cy = 0.5f * (W.B.ly + W.B.hy), cz = 0.5f * (W.B.lz + W.B.hz);
      const float hd = 0.5f * sqrtf(lsk::dist2(W.B.hx - W.B.lx, W.B.hy - W.B.ly, W.B.hz - W.B.lz));
      // every candidate streamed lies within hd + R + gdiag of the centre; queries within hd
      const float M = (2.f * hd + R + gdiag) * (1.f + 0x1p-10f) + W.G.eps;
      // scale S = 2^-e with M * S <= 1 (exact power of 2: no rounding in the scaling)
      int e2;
      (void)frexpf(fmaxf(M, 1e-30f), &e2);
      const float S = ldexpf(1.f, -e2);
      const float S2 = S * S;
      // |a - S² d²| <= 2^-16 (analysis in the header; M·S <= 1): bias and band margin
      const float delta = 0x1p-14f;
      const float qxs = (qx - cx) * S, qys = (qy - cy) * S, qzs = (qz - cz) * S;
      const f16x8 bfrag = frag_b(qxs, qys, qzs, lsk::dist2(qxs, qys, qzs) + delta, upper);
      const float La = act ? L * S2 : -1.f;
      const float Ha = act ? H * S2 + 2.5f * delta : -1.f;
      uint32_t below = 0, cnt = 0;
      // ---- stream
      MF_ADD(0, tp0);
      MF_T(tp1);
      CellIter I;
      I.x0 = cell_of(W.B.lx - R, W.G.ox, W.G.scale, W.sh_c);
      I.x1 = cell_of(W.B.hx + R, W.G.ox, W.G.scale, W.sh_c);
      I.y0 = cell_of(W.B.ly - R, W.G.oy, W.G.scale, W.sh_c);
      I.y1 = cell_of(W.B.hy + R, W.G.oy, W.G.scale, W.sh_c);
      I.z0 = cell_of(W.B.lz - R, W.G.oz, W.G.scale, W.sh_c);
      I.z1 = cell_of(W.B.hz + R, W.G.oz, W.G.scale, W.sh_c);
      if ((uint64_t)(I.x1 - I.x0 + 1u) * (I.y1 - I.y0 + 1u) * (I.z1 - I.z0 + 1u) > kMaxCells) {
        // a range the grid cannot serve (a band far above the local spacing): backstop
        if (act) {
          done = true;
          res = kNaNBits;
          qs |= QS_FAIL;
        }
        break;
      }
      I.bx = I.x0;
      I.by = I.y0;
      I.bz = I.z0;
      I.bmask = 0;
      I.done = false;
      Stream S_;
      S_.need = 0;
      S_.si = S_.se = 0;
      {
        uint32_t fx, fy, fz;
        S_.have_next = next_cell(W, I, fx, fy, fz);
        if (S_.have_next) fetch_cell(W, fx, fy, fz, S_.na, S_.ne, S_.nxyz);
        S_.have_next2 = S_.have_next && next_cell(W, I, fx, fy, fz);
        if (S_.have_next2) fetch_cell(W, fx, fy, fz, S_.ma, S_.me, S_.mxyz);
      }
      // Pipeline over PAIRS of tiles, two pairs in flight: pair X is processed while pair
      // Y's loads are outstanding, and X's registers take the pair after Y (loads issued
      // under X's MFMAs, consumed two half-steps later). The loop is unrolled by two (X, Y)
      // so no loaded register is copied (a copy would wait for its load), and every point
      // load is issued unconditionally (a clamped index when there is no tile): with equal
      // load counts on every path the waits for a pair are vmcnt(2), not vmcnt(0). Band
      // candidates of the pair get their exact canonical d² in one append loop over a
      // 32-bit mask (the pair's points staged in LDS): below L -> counted, in [L, H) -> the
      // band list holds the exact bits.
      const uint32_t Lb = fbits(L), Hb = fbits(H);
      uint32_t o1, o2, o3, b0, b1, b2, b3;
      const uint32_t LaB = fbits(fmaxf(La, 0.f)), HaB = fbits(fmaxf(Ha, 0.f));
      const uint32_t hrow = (uint32_t)upper << 2;
      uint32_t belowx = 0;
      const f32x16 zero = {};
      const float *pts = W.G.pts;
      bool more = true;  // the stream has not ended (the last tile built existed)
      // build the next pair and issue its loads (unconditionally) into (h, v, p) of a set
      auto build_pair = [&](bool &ha_, bool &va_, f32x3 &pa_, bool &hb_, bool &vb_, f32x3 &pb_)
                            __attribute__((always_inline)) {
        uint32_t i0 = 0, i1 = 0;
        bool v0 = false, v1 = false;
        const bool h0 = more && next_tile(W, I, S_, o1, o2, o3, b0, b1, b2, b3, i0, v0);
        const bool h1 = h0 && next_tile(W, I, S_, o1, o2, o3, b0, b1, b2, b3, i1, v1);
        more = h1;
        pa_ = ld_point(pts, h0 ? i0 : 0u);
        pb_ = ld_point(pts, h1 ? i1 : 0u);
        ha_ = h0;
        va_ = v0;
        hb_ = h1;
        vb_ = v1;
      };
      auto step = [&](bool &ha, bool &va, f32x3 &pa, bool &hb, bool &vb, f32x3 &pb) __attribute__((always_inline)) {
        wait_vm2(pa, pb);  // this pair's loads (the other set's two are younger)
        const float pax = pa.x, pay = pa.y, paz = pa.z, pbx = pb.x, pby = pb.y, pbz = pb.z;
        // tile A and tile B (dummy rows, and a missing tile B: |p|² = 8, far above any band)
        const float ax = va ? (pax - cx) * S : 0.f, ay = va ? (pay - cy) * S : 0.f, az = va ? (paz - cz) * S : 0.f;
        f16x8 fa = frag_a(ax, ay, az, upper);
        if (!va && upper) fa = as_frag(0u, 0u, 0x00004800u, kOnes16);  // (pp h, l) = (8, 0)
        const f32x16 accA = __builtin_amdgcn_mfma_f32_32x32x16_f16(fa, bfrag, zero, 0, 0, 0);
        const float bx_ = vb ? (pbx - cx) * S : 0.f, by_ = vb ? (pby - cy) * S : 0.f, bz_ = vb ? (pbz - cz) * S : 0.f;
        f16x8 fb = frag_a(bx_, by_, bz_, upper);
        if (!vb && upper) fb = as_frag(0u, 0u, 0x00004800u, kOnes16);
        const f32x16 accB = __builtin_amdgcn_mfma_f32_32x32x16_f16(fb, bfrag, zero, 0, 0, 0);
        if (!upper) {
          stage[3 * j] = pax;
          stage[3 * j + 1] = pay;
          stage[3 * j + 2] = paz;
          stage[96 + 3 * j] = pbx;
          stage[96 + 3 * j + 1] = pby;
          stage[96 + 3 * j + 2] = pbz;
        }
        evals += hb ? 64u : 32u;
        // this set's registers take the pair after the other set's (built under the MFMAs;
        // both tiles are built before either's loads are issued: a cell change inside the
        // builder waits for the slot loads, and with them for every older load)
        build_pair(ha, va, pa, hb, vb, pb);
        // per value 4 VALU, no lane masks: the sign of (a - La) / (a - Ha) on the float bits
        // (a >= 0 by the bias) shifted into two bit masks with v_alignbit; bit r < 16:
        // tile A value r, bit 16 + r: tile B value r
        uint32_t ltL = 0, ltH = 0;
#pragma unroll
        for (int r = 15; r >= 0; r--) {
          const uint32_t ab = fbits(accB[r]);
          ltL = __builtin_amdgcn_alignbit(ltL, ab - LaB, 31);
          ltH = __builtin_amdgcn_alignbit(ltH, ab - HaB, 31);
        }
#pragma unroll
        for (int r = 15; r >= 0; r--) {
          const uint32_t ab = fbits(accA[r]);
          ltL = __builtin_amdgcn_alignbit(ltL, ab - LaB, 31);
          ltH = __builtin_amdgcn_alignbit(ltH, ab - HaB, 31);
        }
        below += (uint32_t)__builtin_popcount(ltL);
        uint32_t bits = ltH & ~ltL;
        // (the counters as locals: captured by reference, the two increments below became
        // one store through a selected pointer, in scratch)
        uint32_t nbx = belowx, nc = cnt;
        if (LSK_MF_EXP & 2) {
          nbx += __builtin_popcount(bits);
          bits = 0;
        }
        // band candidates, two per round (rounds = the wave's largest count / 2), branch
        // free: a candidate that is not in the band stores into the query's pad dword
        while (__ballot(bits != 0u)) {
#ifdef LSK_MF_PROFILE
          prof[4]++;
#endif
          const bool h0 = bits != 0u;
          const uint32_t r0 = (uint32_t)__builtin_ctz(bits | 0x80000000u);
          bits &= bits - 1u;
          const bool h1 = bits != 0u;
          const uint32_t r1 = (uint32_t)__builtin_ctz(bits | 0x80000000u);
          bits &= bits - 1u;
          // staged point of value r: tile (r >> 4), row (r & 3) + 8 ((r >> 2) & 3) + 4 h
          const uint32_t q0 = r0 & 15u, q1 = r1 & 15u;
          const uint32_t w0 = 3u * (q0 + (q0 & 12u) + hrow) + ((r0 >> 4) * 96u);
          const uint32_t w1 = 3u * (q1 + (q1 & 12u) + hrow) + ((r1 >> 4) * 96u);
          const float e0 = lsk::dist2(qx - stage[w0], qy - stage[w0 + 1], qz - stage[w0 + 2]);
          const float e1 = lsk::dist2(qx - stage[w1], qy - stage[w1 + 1], qz - stage[w1 + 2]);
          const uint32_t eb0 = fbits(e0), eb1 = fbits(e1);
          const bool lo0 = h0 && eb0 < Lb, lo1 = h1 && eb1 < Lb;
          const bool in0 = h0 && !lo0 && eb0 < Hb, in1 = h1 && !lo1 && eb1 < Hb;
          nbx += (uint32_t)lo0 + (uint32_t)lo1;
          const uint32_t c0 = min(nc, kCapQ - 1u);
          nc += (uint32_t)in0;
          const uint32_t c1 = min(nc, kCapQ - 1u);
          nc += (uint32_t)in1;
#if LSK_MF_GBAND
          if (in0) BAND(j, upper ? kCapQ - 1u - c0 : c0) = eb0;
          if (in1) BAND(j, upper ? kCapQ - 1u - c1 : c1) = eb1;
#else
          const uint32_t qb = j * kStride;
          region[qb + (in0 ? (upper ? kCapQ - 1u - c0 : c0) : kCapQ)] = eb0;
          region[qb + (in1 ? (upper ? kCapQ - 1u - c1 : c1) : kCapQ)] = eb1;
#endif
        }
        belowx = nbx;
        cnt = nc;
      };
      bool hxa, vxa, hxb, vxb, hya, vya, hyb, vyb;
      f32x3 xa, xb, ya, yb;
      build_pair(hxa, vxa, xa, hxb, vxb, xb);
      build_pair(hya, vya, ya, hyb, vyb, yb);
      while (hxa) {
        step(hxa, vxa, xa, hxb, vxb, xb);
        if (!hya) break;
        step(hya, vya, ya, hyb, vyb, yb);
      }
      // the loads still in flight land in registers nothing reads again: keep all four
      // live up to a full drain, so no other value takes them while a load is pending
      asm volatile("s_waitcnt vmcnt(0)" : "+v"(xa), "+v"(xb), "+v"(ya), "+v"(yb) : : "memory");
      const uint32_t pcnt = partner_u(cnt);
      const bool ovf = cnt + pcnt > kCapQ;
      const uint32_t kept = min(cnt, kCapQ);
      // ---- decide per query (both halves agree: they combine the same two numbers)
      MF_ADD(1, tp1);
      MF_T(tp3);
      const uint32_t btot = below + belowx + partner_u(below + belowx);
      const uint32_t pkept = partner_u(kept);
      const uint32_t ktot = kept + pkept;
      bool sel = false;
      if (act) {
        // every count is exact (the band candidates were classified by their canonical d²
        // as they came, stored or not): btot below L, cnt + pcnt in [L, H)
        const uint32_t tot_in = cnt + pcnt;
        if (btot >= k) {
          qs |= QS_UNDERFLOW;
          // k-th below L: the band just below, sized from the count
          const float nH = L;
          const float want = fmaxf(kf - 1.5f * z * sqrtf(kf), 0.f);
          L = L * __builtin_powf(want / (float)btot, 2.f / 3.f);
          H = nH;
          if (!(H > L)) L = 0.f;
        } else if (btot + tot_in < k) {
          if (fbits(H) >= cut_b) {
            done = true;
            res = cut_b;
            qs |= QS_DONE_CUT;
          } else {
            qs |= QS_REFINE;
            const float nL = H;
            const float have_c = fmaxf((float)(btot + tot_in), 1.f);
            float nH = H * __builtin_powf((kf + 1.5f * z * sqrtf(kf)) / have_c, 2.f / 3.f);
            nH = fminf(nH, H * 64.f);
            L = nL;
            H = fminf(nH, cut2);
            if (!(H > L)) H = bitsf(fbits(L) + 1u);
          }
        } else if (ovf) {
          qs |= QS_OVERFLOW;
          // the k-th is in the band but the list dropped values: a narrower band around
          // its position (the band's values taken as uniform in r³)
          const float l3 = L * sqrtf(L), h3 = H * sqrtf(H);
          const float f = (float)(k - btot) / (float)tot_in;
          const float c3 = l3 + f * (h3 - l3), w3 = (h3 - l3) * ((float)kCapQ * 0.3f / (float)tot_in);
          const float nl3 = fmaxf(c3 - w3, l3), nh3 = fminf(c3 + w3, h3);
          L = __builtin_powf(nl3, 2.f / 3.f);
          H = fmaxf(__builtin_powf(nh3, 2.f / 3.f), L);
          if (fbits(H) <= fbits(L)) H = bitsf(fbits(L) + 1u);
        } else {
          sel = true;
        }
      }
      // ---- selection of the m-th exact band value (m = k - below, 1-based)
#if LSK_MF_GBAND
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the band stores are done
#endif
      if (__ballot(sel)) {
        uint32_t m = sel ? k - btot : 1u;
        uint32_t lo = Lb, w = Hb - Lb;
        uint32_t inr = ktot;  // values of the query in [lo, lo + w)
        // narrow by 8 sub-bands until <= 32 values remain (both halves in lockstep)
        for (int it = 0; it < 6; it++) {
          const bool more = sel && inr > 32u && w > 1u;
          if (!__ballot(more)) break;
          const uint32_t nb = 32u - (uint32_t)__builtin_clz(w - 1u);  // bits of w - 1
          const uint32_t sh = nb > 3u ? nb - 3u : 0u;
          uint32_t c0 = 0, c1 = 0;  // 8 byte counters: sub-bands 0-3, 4-7
          uint32_t nk = 0;
          {
            uint32_t km = kept;
            uint32_t kmax = km;
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) kmax = max(kmax, (uint32_t)__shfl_xor((int)kmax, o));
            kmax = lsk::uniform(kmax);
            for (uint32_t e = 0; e < kmax; e++) {
              if (more && e < km) {
                const uint32_t v = BAND(j, (upper ? kCapQ - 1u - e : e));
                const uint32_t d = v - lo;
                if (d < w) {
                  const uint32_t sb = d >> sh;
                  const uint32_t inc = 1u << ((sb & 3u) << 3);
                  if (sb < 4u) c0 += inc; else c1 += inc;
                }
              }
            }
            (void)nk;
          }
          c0 += partner_u(c0);
          c1 += partner_u(c1);
          if (more) {
            uint32_t acc = 0, b = 0, cb = 0;
            for (uint32_t t = 0; t < 8u; t++) {
              const uint32_t c = ((t < 4u ? c0 : c1) >> ((t & 3u) << 3)) & 0xffu;
              if (acc + c >= m) {
                b = t;
                cb = c;
                break;
              }
              acc += c;
            }
            m -= acc;
            lo += b << sh;
            const uint32_t nw = 1u << sh;
            w = min(nw, w - (b << sh));
            inr = cb;
          }
        }
        // gather the <= 32 values in [lo, lo + w): each half compacts its own to its end
        uint32_t mine = 0;
        {
          uint32_t km = kept;
          uint32_t kmax = km;
#pragma unroll
          for (int o = 32; o > 0; o >>= 1) kmax = max(kmax, (uint32_t)__shfl_xor((int)kmax, o));
          kmax = lsk::uniform(kmax);
          for (uint32_t e = 0; e < kmax; e++) {
            if (sel && e < km) {
              const uint32_t v = BAND(j, (upper ? kCapQ - 1u - e : e));
              if (v - lo < w) {
                BAND(j, (upper ? kCapQ - 1u - mine : mine)) = v;
                mine++;
              }
            }
          }
        }
        const uint32_t other = partner_u(mine);
#if LSK_MF_GBAND
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the partner's compaction stores
#endif
        if (sel && !upper) {
          if (w <= 1u || mine + other > 32u) {
            // all equal (w == 1) or still crowded (pathological ties): lo is exact for w == 1
            if (w <= 1u) {
              res = lo;
              done = true;
            } else {
              res = kNaNBits;
              done = true;
              qs |= QS_FAIL | QS_BINOVF;
            }
          } else {
            uint32_t v[32];
#pragma unroll
            for (int i = 0; i < 32; i++) {
              const uint32_t ui = (uint32_t)i;
              v[i] = ui < mine ? BAND(j, ui) : (ui < mine + other ? BAND(j, kCapQ - 1u - (ui - mine)) : 0xffffffffu);
            }
            uint32_t r;
            net32_select(v, m, r);
            res = r;
            done = true;
          }
        }
        // the upper half takes the lower half's answer
        const uint32_t pres = partner_u(res);
        const uint32_t pdone = partner_u(done ? 1u : 0u);
        const uint32_t pqs = partner_u(qs);
        if (sel && upper) {
          res = pres;
          done = pdone != 0u;
          qs = pqs;
        }
      }
      MF_ADD(3, tp3);
    }
    // ---- output (the lower half writes)
#ifdef LSK_MF_PROFILE
    if (A.stats && lane == 0) {
      atomicAdd(&A.stats[16], (unsigned long long)prof[0]);
      atomicAdd(&A.stats[17], (unsigned long long)prof[1]);
      atomicAdd(&A.stats[18], (unsigned long long)prof[2]);
      atomicAdd(&A.stats[19], (unsigned long long)prof[3]);
      atomicAdd(&A.stats[20], (unsigned long long)prof[4]);
      atomicAdd(&A.stats[21], (unsigned long long)(evals / 32u));
    }
#endif
    if (A.debug_fail_mod > 0 && qi % A.debug_fail_mod == 0) qs |= QS_FAIL;
    const bool failed = valid && !upper && (qs & QS_FAIL);
    if (failed) res = kNaNBits;
    if (A.fail_count) {
      const uint64_t fm = __ballot(failed);
      if (fm) {
        uint32_t base = 0;
        if (lane == 0) base = atomicAdd(A.fail_count, (uint32_t)__popcll(fm));
        base = lsk::uniform(base);
        const uint64_t slot = (uint64_t)base + (uint64_t)__popcll(fm & ((1ull << lane) - 1ull));
        if (failed && slot < (uint64_t)A.fail_cap) A.fail_list[slot] = (uint32_t)qi;
      }
    }
    if (valid && !upper) {
      if (A.out_perm) A.out_final[A.out_perm[qi]] = lsk::final_distance(bitsf(res));
      if (A.out_d2) A.out_d2[qi] = bitsf(res);
      if (A.qstatus) A.qstatus[qi] = qs | (passes << 16);
    }
    if (A.stats) {
      const unsigned long long c_ovf = __popcll(__ballot(valid && !upper && (qs & QS_OVERFLOW)));
      const unsigned long long c_udf = __popcll(__ballot(valid && !upper && (qs & QS_UNDERFLOW)));
      const unsigned long long c_ref = __popcll(__ballot(valid && !upper && (qs & QS_REFINE)));
      const unsigned long long c_fail = __popcll(__ballot(valid && !upper && (qs & QS_FAIL)));
      if (lane == 0) {
        atomicAdd(&A.stats[0], (unsigned long long)evals * 2ull);  // candidates per query (x 64 lanes / 32 queries)
        atomicAdd(&A.stats[3], (unsigned long long)passes);
        atomicAdd(&A.stats[4], c_ovf);
        atomicAdd(&A.stats[5], c_udf);
        atomicAdd(&A.stats[6], c_ref);
        atomicAdd(&A.stats[10], 1ull);
        atomicAdd(&A.stats[26], c_fail);
      }
    }
    if (!STRIDE) break;
  }
}

}  // namespace

extern "C" int lsk_hip_knn_mfma(const lsk_knn_args *args, const lsk_grid_view *grid, void *stream) {
  const lsk_knn_args &A = *args;
  if (A.k < 1 || A.k > 65535) {
    lsk::set_last_error("knn_mfma: k must be in [1, 65535]");
    return 1;
  }
  if (A.nq >= ((int64_t)1 << 32) || A.ntrees != 1 || A.init_d2 || A.tree[0].n >= ((int64_t)1 << 32) || !grid ||
      grid->level < 0 || grid->level > 8) {
    lsk::set_last_error("knn_mfma: one tree (< 2^32 points, the queries' own), no init_d2, grid level in [0, 8]");
    return 1;
  }
  const int64_t ngroups = A.groups ? A.ngroups : (A.nq + 63) / 64;
  const int64_t gend = A.wave_end > 0 && A.wave_end < ngroups ? A.wave_end : ngroups;
  if (A.wave_base < 0 || gend - A.wave_base <= 0) return 0;
  const unsigned nblk = lsk_blocks(gend - A.wave_base, 1);
#if LSK_MF_GBAND
  // (tuning build only: one static buffer, not safe for concurrent launches)
  static uint32_t *gband = nullptr;
  if (!gband) LSK_HIP(hipMalloc(&gband, (size_t)kStrideBlocksFull * kWPB * kQ * kCapQ * sizeof(uint32_t)));
  {
    const unsigned cap = kStrideBlocksFull;
    unsigned nb = nblk < cap ? nblk : cap;
    if (nb >= 8u) nb &= ~7u;
    knn_mfma_kernel<true><<<nb, kThreads, 0, (hipStream_t)stream>>>(A, *grid, gband);
  }
#else
  if (A.pad2 >= 1) {
    const unsigned cap = A.pad2 == 2 ? kStrideBlocksFull : kStrideBlocks;
    knn_mfma_kernel<true><<<nblk < cap ? nblk : cap, kThreads, 0, (hipStream_t)stream>>>(A, *grid, nullptr);
  } else {
    knn_mfma_kernel<false><<<nblk, kThreads, 0, (hipStream_t)stream>>>(A, *grid, nullptr);
  }
#endif
  LSK_CHECK_LAUNCH("knn_mfma");
  return 0;
}
