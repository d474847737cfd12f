// lsknn — shared host/device definitions.
//
// Everything numeric that must agree bit-for-bit between the gfx950 kernels and the
// CPU oracle lives here: the 12-byte point type, the 24-byte box type, the canonical
// squared-distance formula, Morton encoding and the float<->bits helpers used by the
// radix-select k-th-distance kernels.
//
// Reference parity: the reference's float3 / cukd::box_t<float3> (24 B, sent as
// 6 MPI_FLOAT at prePartitionedDataVariant.cu:290) and cukd's squared distance used
// inside stackFree::knn (unorderedDataVariant.cu:86). The reference leaves the
// association of dx*dx+dy*dy+dz*dz to the compiler; we pin it.
#pragma once
#include <stdint.h>
#include <math.h>

#if defined(__HIPCC__)
#define LSK_HD __host__ __device__ __forceinline__
#else
#define LSK_HD inline
#endif

namespace lsk {

// 12-byte packed point, identical layout to the reference's float3 input records.
struct vec3f {
  float x, y, z;
};
static_assert(sizeof(vec3f) == 12, "vec3f must be 12 bytes (file format)");

// 24-byte AABB, identical layout to cukd::box_t<float3> (lower, upper).
struct box3f {
  vec3f lo, hi;
};
static_assert(sizeof(box3f) == 24, "box3f must be 24 bytes");

// Canonical squared distance. The product/fma association is fixed so that the GPU
// kernels and the CPU oracle produce identical bits; every translation unit that uses
// it is compiled with -ffp-contract=off.
LSK_HD float dist2(float dx, float dy, float dz) {
  return fmaf(dz, dz, fmaf(dy, dy, dx * dx));
}

LSK_HD float dist2(const vec3f &a, const vec3f &b) {
  return dist2(a.x - b.x, a.y - b.y, a.z - b.z);
}

// Squared distance from a point to a box. For every point p inside the box, the
// value computed here is <= dist2(q, p) computed above (float subtraction, squaring
// and fma are monotone in their non-negative arguments), so pruning with it is exact.
LSK_HD float box_dist2(const vec3f &q, const vec3f &lo, const vec3f &hi) {
  float dx = fmaxf(fmaxf(lo.x - q.x, q.x - hi.x), 0.f);
  float dy = fmaxf(fmaxf(lo.y - q.y, q.y - hi.y), 0.f);
  float dz = fmaxf(fmaxf(lo.z - q.z, q.z - hi.z), 0.f);
  return dist2(dx, dy, dz);
}

// Box-to-box gap (reference computeDistance, prePartitionedDataVariant.cu:150-155):
// per-axis max(0, a.lo-b.hi, b.lo-a.hi), then sqrt of the sum of squares.
LSK_HD float box_box_dist2(const box3f &a, const box3f &b) {
  float dx = fmaxf(0.f, fmaxf(a.lo.x - b.hi.x, b.lo.x - a.hi.x));
  float dy = fmaxf(0.f, fmaxf(a.lo.y - b.hi.y, b.lo.y - a.hi.y));
  float dz = fmaxf(0.f, fmaxf(a.lo.z - b.hi.z, b.lo.z - a.hi.z));
  return dist2(dx, dy, dz);
}

// --- Morton (Z-order) keys: 10 bits per axis, 30-bit key ------------------------
LSK_HD uint32_t morton_spread10(uint32_t v) {
  v &= 0x3ffu;
  v = (v | (v << 16)) & 0x030000FFu;
  v = (v | (v << 8)) & 0x0300F00Fu;
  v = (v | (v << 4)) & 0x030C30C3u;
  v = (v | (v << 2)) & 0x09249249u;
  return v;
}

// Quantise a coordinate into [0, 1023] given the cube origin and 1024/extent scale.
LSK_HD uint32_t morton_quant(float v, float origin, float scale) {
  float f = (v - origin) * scale;
  f = fminf(fmaxf(f, 0.f), 1023.f);
  return (uint32_t)f;
}

LSK_HD uint32_t morton3(uint32_t ix, uint32_t iy, uint32_t iz) {
  return (morton_spread10(ix) << 2) | (morton_spread10(iy) << 1) | morton_spread10(iz);
}

// --- Hilbert keys: 10 bits per axis, 30-bit key ------------------------------------
// Skilling's transform (axes -> transposed Hilbert index, then bit interleave). Like
// Morton, every aligned block of 8^l consecutive keys is one octree cell of level 10-l
// (what the splitter snapping relies on), but consecutive cells are always face
// neighbours: 16-point runs have ~3x smaller boxes than Z-order runs (uniform data:
// mean box volume 1.1x vs 3.3x the ideal cube), so rows and buckets cull much better.
LSK_HD uint32_t hilbert3(uint32_t x, uint32_t y, uint32_t z) {
  x &= 0x3ffu;
  y &= 0x3ffu;
  z &= 0x3ffu;
  for (uint32_t q = 1u << 9; q > 1u; q >>= 1) {
    const uint32_t p = q - 1u;
    // axis 0: invert low bits of x when its bit is set (exchange with itself = no-op)
    if (x & q) x ^= p;
    if (y & q) {
      x ^= p;
    } else {
      const uint32_t t = (x ^ y) & p;
      x ^= t;
      y ^= t;
    }
    if (z & q) {
      x ^= p;
    } else {
      const uint32_t t = (x ^ z) & p;
      x ^= t;
      z ^= t;
    }
  }
  y ^= x;  // Gray encode
  z ^= y;
  uint32_t t = 0;
  for (uint32_t q = 1u << 9; q > 1u; q >>= 1)
    if (z & q) t ^= q - 1u;
  return morton3(x ^ t, y ^ t, z ^ t);
}

enum : int { kCurveMorton = 0, kCurveHilbert = 1 };

LSK_HD uint32_t curve3(int curve, uint32_t ix, uint32_t iy, uint32_t iz) {
  return curve == kCurveHilbert ? hilbert3(ix, iy, iz) : morton3(ix, iy, iz);
}

// --- float <-> ordered bits (non-negative floats order like their bit patterns) ---
LSK_HD uint32_t fbits(float f) {
  union { float f; uint32_t u; } c; c.f = f; return c.u;
}
LSK_HD float bitsf(uint32_t u) {
  union { float f; uint32_t u; } c; c.u = u; return c.f;
}

// The radix-select histogram geometry shared by kernel and oracle tests.
constexpr int kSelBins = 64;          // bins per histogram pass
constexpr int kSelShift0 = 21;        // first pass: 2 mantissa bits -> 1/4-octave bins of d^2
constexpr int kSelRefine = 6;         // each refinement pass resolves log2(kSelBins) more bits
constexpr uint32_t kInfBits = 0x7f800000u;

// Results of the k-th-distance selection are returned as squared distances; the
// reference output is sqrtf of that value unless it is +inf
// (extractFinalResult, unorderedDataVariant.cu:97-102).
LSK_HD float final_distance(float d2) {
  return isinf(d2) ? d2 : sqrtf(d2);
}

}  // namespace lsk
