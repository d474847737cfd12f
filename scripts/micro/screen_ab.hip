// MFMA vs VALU candidate screening: the measured A/B behind the decision to keep the
// k-NN distance math on the VALU (no counterpart in the reference,
// whose stackFree::knn evaluates one candidate per thread, unorderedDataVariant.cu:84-86).
//
// Both kernels do the pass-1 inner work of knn_rows.hip on the same data layout: a wave
// holds 64 consecutive (curve-ordered) queries as 4 rows of 16; per step every row takes
// one 16-point quarter of the sorted points and every (query, candidate) pair of the row
// is tested against the query's squared-radius threshold. A row visits the quarters of
// the neighbouring buckets (quarter r of bucket g + s - S/2 in step s), like a walk.
//
//  * VALU (the production form): the row's candidates are broadcast lane to lane with DPP
//    row_newbcast and every lane computes the canonical d² of its own query to each of
//    the 16 — exact, the value the histogram bins need.
//  * MFMA: per row one v_mfma_f32_16x16x4_f32 computes the 16x16 tile
//    |q'|² - 2 q'·p' + |p'|² on row-centred coordinates (A = [q'x q'y q'z 1] per query,
//    B = [-2p'x -2p'y -2p'z |p'|²] per candidate, C = |q'|²), an APPROXIMATE d². It can
//    only screen: a pair is kept when  D < thr (1 + 2^-20) + (qn² + |p'|²) 2^-18, a
//    bound that covers the f32 rounding of the centring, of the fma chain and of the
//    canonical formula (qn = largest |q'| of the row), so no pair with canonical
//    d² < thr is ever dropped. The result sits in the MFMA C layout (lane l holds
//    queries 4(l>>4)..+3 of candidate l&15), not one query per lane.
//
// Output: per lane the number of kept pairs (VALU: its query's; MFMA: its C elements'),
// and for the MFMA check form the number of pairs the screen dropped although their
// canonical d² is below thr (must be 0).
#include "dev.h"

namespace {

constexpr int kThreads = 256;

template <int J>
__device__ __forceinline__ float rowb(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x150 + J, 0xf, 0xf, false));
}

__device__ __forceinline__ int64_t quarter_of(int64_t g, int r, int s, int steps, int64_t nq4) {
  int64_t qid = 4 * (g + s - steps / 2) + r;
  qid = qid < 0 ? (qid & 3) : qid;
  return qid >= nq4 ? nq4 - 4 + (qid & 3) : qid;
}

template <int J>
__device__ __forceinline__ uint32_t valu_pair(float qx, float qy, float qz, float px, float py, float pz,
                                              uint32_t thrb) {
  const float d2 = lsk::dist2(qx - rowb<J>(px), qy - rowb<J>(py), qz - rowb<J>(pz));
  return __float_as_uint(d2) < thrb ? 1u : 0u;
}

__global__ __launch_bounds__(kThreads) void screen_valu_kernel(const float *__restrict__ pts, int64_t n,
                                                               const float *__restrict__ thr, int steps,
                                                               uint32_t *__restrict__ out) {
  const int lane = lsk::lane_id();
  const int64_t g = ((int64_t)blockIdx.x * kThreads + threadIdx.x) >> 6;
  if (g * 64 >= n) return;
  const int64_t qi = g * 64 + lane;
  const float qx = pts[3 * qi], qy = pts[3 * qi + 1], qz = pts[3 * qi + 2];
  const uint32_t thrb = __float_as_uint(thr[qi]);
  const int64_t nq4 = n / 16;
  const int r = lane >> 4;
  uint32_t cnt = 0;
  for (int s = 0; s < steps; s++) {
    const int64_t c = 16 * quarter_of(g, r, s, steps, nq4) + (lane & 15);
    const float px = pts[3 * c], py = pts[3 * c + 1], pz = pts[3 * c + 2];
    cnt += valu_pair<0>(qx, qy, qz, px, py, pz, thrb) + valu_pair<1>(qx, qy, qz, px, py, pz, thrb) +
           valu_pair<2>(qx, qy, qz, px, py, pz, thrb) + valu_pair<3>(qx, qy, qz, px, py, pz, thrb) +
           valu_pair<4>(qx, qy, qz, px, py, pz, thrb) + valu_pair<5>(qx, qy, qz, px, py, pz, thrb) +
           valu_pair<6>(qx, qy, qz, px, py, pz, thrb) + valu_pair<7>(qx, qy, qz, px, py, pz, thrb) +
           valu_pair<8>(qx, qy, qz, px, py, pz, thrb) + valu_pair<9>(qx, qy, qz, px, py, pz, thrb) +
           valu_pair<10>(qx, qy, qz, px, py, pz, thrb) + valu_pair<11>(qx, qy, qz, px, py, pz, thrb) +
           valu_pair<12>(qx, qy, qz, px, py, pz, thrb) + valu_pair<13>(qx, qy, qz, px, py, pz, thrb) +
           valu_pair<14>(qx, qy, qz, px, py, pz, thrb) + valu_pair<15>(qx, qy, qz, px, py, pz, thrb);
  }
  out[qi] = cnt;
}

typedef float f32x4 __attribute__((ext_vector_type(4)));

template <bool CHECK>
__global__ __launch_bounds__(kThreads) void screen_mfma_kernel(const float *__restrict__ pts, int64_t n,
                                                               const float *__restrict__ thr, int steps,
                                                               uint32_t *__restrict__ out,
                                                               uint32_t *__restrict__ viol) {
  const int lane = lsk::lane_id();
  const int64_t g = ((int64_t)blockIdx.x * kThreads + threadIdx.x) >> 6;
  if (g * 64 >= n) return;
  const int64_t qi = g * 64 + lane;
  const float qx = pts[3 * qi], qy = pts[3 * qi + 1], qz = pts[3 * qi + 2];
  const float qt = thr[qi];
  const int k = lane >> 4, j = lane & 15;
  const int64_t nq4 = n / 16;
  // per row r: centre (its first query), A operand, C init (|q'|^2), thresholds, qn^2
  float cx[4], cy[4], cz[4], a[4], qn2[4];
  f32x4 cin[4], th[4];
  float ex[4][4], ey[4][4], ez[4][4];  // CHECK: the C elements' query coordinates
#pragma unroll
  for (int r = 0; r < 4; r++) {
    cx[r] = __shfl(qx, 16 * r);
    cy[r] = __shfl(qy, 16 * r);
    cz[r] = __shfl(qz, 16 * r);
    const float dx = qx - cx[r], dy = qy - cy[r], dz = qz - cz[r];  // lane's own query, centred on row r
    const float n2 = lsk::dist2(dx, dy, dz);
    // A[i][k] = comp k of query 16r + i, from lane 16r + i
    const int src = 16 * r + j;
    const float sx = __shfl(dx, src), sy = __shfl(dy, src), sz = __shfl(dz, src);
    a[r] = k == 0 ? sx : k == 1 ? sy : k == 2 ? sz : 1.f;
    float m = (lane >> 4) == r ? n2 : 0.f;
    m = fmaxf(m, __shfl_xor(m, 1)); m = fmaxf(m, __shfl_xor(m, 2)); m = fmaxf(m, __shfl_xor(m, 4));
    m = fmaxf(m, __shfl_xor(m, 8)); m = fmaxf(m, __shfl_xor(m, 16)); m = fmaxf(m, __shfl_xor(m, 32));
    qn2[r] = m;
#pragma unroll
    for (int v = 0; v < 4; v++) {
      const int e = 16 * r + 4 * k + v;  // query of C element (row 4k + v)
      cin[r][v] = __shfl(n2, e);
      th[r][v] = __shfl(qt, e);
      if (CHECK) {
        ex[r][v] = __shfl(qx, e);
        ey[r][v] = __shfl(qy, e);
        ez[r][v] = __shfl(qz, e);
      }
    }
  }
  uint32_t cnt = 0, bad = 0;
  for (int s = 0; s < steps; s++) {
#pragma unroll
    for (int r = 0; r < 4; r++) {
      const int64_t c = 16 * quarter_of(g, r, s, steps, nq4) + j;  // candidate j of row r
      const float px = pts[3 * c], py = pts[3 * c + 1], pz = pts[3 * c + 2];
      const float dx = px - cx[r], dy = py - cy[r], dz = pz - cz[r];
      const float pn2 = lsk::dist2(dx, dy, dz);
      const float b = k == 0 ? -2.f * dx : k == 1 ? -2.f * dy : k == 2 ? -2.f * dz : pn2;
      const f32x4 d = __builtin_amdgcn_mfma_f32_16x16x4f32(a[r], b, cin[r], 0, 0, 0);
      const float e = (qn2[r] + pn2) * 0x1p-18f;
#pragma unroll
      for (int v = 0; v < 4; v++) {
        const bool keep = d[v] < fmaf(th[r][v], 0x1p-20f, th[r][v]) + e;
        cnt += keep ? 1u : 0u;
        if (CHECK) {
          const float x = lsk::dist2(ex[r][v] - px, ey[r][v] - py, ez[r][v] - pz);
          bad += (!keep && x < th[r][v]) ? 1u : 0u;
        }
      }
    }
  }
  out[qi] = cnt;
  if (CHECK) {
    const uint32_t w = lsk::wave_sum(bad);
    if (lane == 0 && w) atomicAdd(viol, w);
  }
}

}  // namespace

// mode 0: VALU canonical; 1: MFMA screen; 2: MFMA screen + violation check (viol).
extern "C" int lsk_hip_screen_ab(const float *pts, int64_t n, const float *thr, int steps, int mode,
                                 uint32_t *out, uint32_t *viol, void *stream) {
  if (n < 64 || n % 64 != 0 || steps < 1 || mode < 0 || mode > 2) {
    return 1;  // n must be a positive multiple of 64, steps >= 1, mode 0..2
  }
  const unsigned nb = lsk_blocks(n, kThreads);
  hipStream_t st = (hipStream_t)stream;
  if (mode == 0)
    screen_valu_kernel<<<nb, kThreads, 0, st>>>(pts, n, thr, steps, out);
  else if (mode == 1)
    screen_mfma_kernel<false><<<nb, kThreads, 0, st>>>(pts, n, thr, steps, out, viol);
  else
    screen_mfma_kernel<true><<<nb, kThreads, 0, st>>>(pts, n, thr, steps, out, viol);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
