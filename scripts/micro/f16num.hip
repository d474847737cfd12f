// Numerics probe of v_mfma_f32_32x32x16_f16: which part of the split-f16 d² loses
// precision? Case 1: D = xh*1 + xl*1 (the hi/lo split of x alone). Case 2: products
// xh*yh + xh*yl + xl*yh + xl*yl. Case 3: 16 equal-magnitude terms. Each against fp64.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdint.h>

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ void split(float x, _Float16 &hi, _Float16 &lo) {
  hi = (_Float16)x;
  lo = (_Float16)(x - (float)hi);
}

// lane l: A row i = l & 31, k = 8h + j; B col j = l & 31, k = 8h + j. Only h = 0 lanes'
// slots 0..3 carry data; D[i][j] = sum over k of A[i][k] B[k][j].
__global__ void probe(const float *xs, const float *ys, int mode, float *out, float *split_out) {
  const int l = threadIdx.x, h = l >> 5, i = l & 31;
  f16x8 a = {}, b = {};
  const float x = xs[i], y = ys[i];
  _Float16 xh, xl, yh, yl;
  split(x, xh, xl);
  split(y, yh, yl);
  if (h == 0) {
    if (mode == 0) {  // D[i][j] = xh_i + xl_i
      a[0] = xh; a[1] = xl;
      b[0] = (_Float16)1.f; b[1] = (_Float16)1.f;
    } else if (mode == 1) {  // D[i][j] = x_i * y_j
      a[0] = xh; a[1] = xl; a[2] = xh; a[3] = xl;
      b[0] = yh; b[1] = yh; b[2] = yl; b[3] = yl;
    } else {  // D[i][j] = xh_i * yh_j only
      a[0] = xh;
      b[0] = yh;
    }
  }
  if (h == 0) {
    split_out[4 * i] = (float)xh;
    split_out[4 * i + 1] = (float)xl;
    split_out[4 * i + 2] = (float)yh;
    split_out[4 * i + 3] = (float)yl;
  }
  f32x16 c = {};
  c = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
  for (int r = 0; r < 16; r++) {
    const int row = (r & 3) + 8 * (r >> 2) + 4 * h;
    out[row * 32 + i] = c[r];
  }
}


// full split-f16 d² of query j (col) and candidate i (row), both halves of K used; also
// writes the fragments so the host can form the exact sum of the MFMA's own inputs
__global__ void probe_d2(const float *q, const float *p, float *out, _Float16 *fa, _Float16 *fb) {
  const int l = threadIdx.x, h = l >> 5, i = l & 31;
  q += 96 * blockIdx.x; p += 96 * blockIdx.x; out += 1024 * blockIdx.x; fa += 512 * blockIdx.x; fb += 512 * blockIdx.x;
  const float px = p[3 * i], py = p[3 * i + 1], pz = p[3 * i + 2];
  const float qx = q[3 * i], qy = q[3 * i + 1], qz = q[3 * i + 2];
  f16x8 a, b;
  _Float16 t0, t1, t2, t3;
  if (h == 0) {
    split(px, t0, t1); split(py, t2, t3);
    a[0] = t0; a[1] = t1; a[2] = t0; a[3] = t1; a[4] = t2; a[5] = t3; a[6] = t2; a[7] = t3;
    split(qx, t0, t1); split(qy, t2, t3);
    b[0] = -2 * t0; b[1] = -2 * t0; b[2] = -2 * t1; b[3] = -2 * t1;
    b[4] = -2 * t2; b[5] = -2 * t2; b[6] = -2 * t3; b[7] = -2 * t3;
  } else {
    split(pz, t0, t1); split(fmaf(pz, pz, fmaf(py, py, px * px)), t2, t3);
    a[0] = t0; a[1] = t1; a[2] = t0; a[3] = t1; a[4] = t2; a[5] = t3; a[6] = (_Float16)1.f; a[7] = (_Float16)1.f;
    split(qz, t0, t1); split(fmaf(qz, qz, fmaf(qy, qy, qx * qx)), t2, t3);
    b[0] = -2 * t0; b[1] = -2 * t0; b[2] = -2 * t1; b[3] = -2 * t1;
    b[4] = (_Float16)1.f; b[5] = (_Float16)1.f; b[6] = t2; b[7] = t3;
  }
  for (int j = 0; j < 8; j++) {
    fa[i * 16 + 8 * h + j] = a[j];
    fb[i * 16 + 8 * h + j] = b[j];
  }
  f32x16 c = {};
  c = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
  for (int r = 0; r < 16; r++) {
    const int row = (r & 3) + 8 * (r >> 2) + 4 * h;
    out[row * 32 + i] = c[r];
  }
}

int main() {
  float hx[32], hy[32], hd[1024], hs[128];
  for (int i = 0; i < 32; i++) {
    hx[i] = 0.3f + 0.0123457f * i + 1e-5f * (float)(i * i % 7);
    hy[i] = 1.7f - 0.0312345f * i;
  }
  float *dx, *dy, *dd, *ds;
  (void)hipMalloc(&dx, 128);
  (void)hipMalloc(&dy, 128);
  (void)hipMalloc(&dd, 4096);
  (void)hipMalloc(&ds, 512);
  (void)hipMemcpy(dx, hx, 128, hipMemcpyHostToDevice);
  (void)hipMemcpy(dy, hy, 128, hipMemcpyHostToDevice);
  for (int mode = 0; mode < 3; mode++) {
    probe<<<1, 64>>>(dx, dy, mode, dd, ds);
    (void)hipMemcpy(hd, dd, 4096, hipMemcpyDeviceToHost);
    (void)hipMemcpy(hs, ds, 512, hipMemcpyDeviceToHost);
    double worst = 0, worst_split = 0;
    for (int i = 0; i < 32; i++) {
      worst_split = fmax(worst_split, fabs((double)hs[4 * i] + hs[4 * i + 1] - hx[i]) / fabs(hx[i]));
      for (int j = 0; j < 32; j++) {
        double want = mode == 0 ? (double)hx[i] : mode == 1 ? (double)hx[i] * hy[j] : (double)hs[4 * i] * hs[4 * j + 2];
        worst = fmax(worst, fabs(hd[i * 32 + j] - want) / fabs(want));
      }
    }
    printf("mode %d: max rel err of D %.3e (2^%.1f); split hi+lo rel err %.3e; x0 = %.9g hi %.9g lo %.9g D00 %.9g\n",
           mode, worst, log2(worst + 1e-30), worst_split, hx[0], hs[0], hs[1], hd[0]);
  }

  {
    const int NT = 2048;
    float *hq = new float[96 * NT], *hp = new float[96 * NT], *hd2 = new float[1024 * NT];
    _Float16 *ha = new _Float16[512 * NT], *hb = new _Float16[512 * NT];
    uint64_t s = 7;
    auto rnd = [&]() { s = s * 6364136223846793005ull + 1442695040888963407ull; return (double)(s >> 11) / 9007199254740992.0; };
    for (int i = 0; i < 96 * NT; i++) {
      hq[i] = (float)((rnd() * 2 - 1) * 0.3);
      hp[i] = (float)((rnd() * 2 - 1) * 1.0);
    }
    float *dq, *dp, *dd2;
    _Float16 *da, *db;
    (void)hipMalloc(&dq, 384 * NT); (void)hipMalloc(&dp, 384 * NT); (void)hipMalloc(&dd2, 4096 * NT);
    (void)hipMalloc(&da, 1024 * NT); (void)hipMalloc(&db, 1024 * NT);
    (void)hipMemcpy(dq, hq, 384 * NT, hipMemcpyHostToDevice);
    (void)hipMemcpy(dp, hp, 384 * NT, hipMemcpyHostToDevice);
    probe_d2<<<NT, 64>>>(dq, dp, dd2, da, db);
    (void)hipMemcpy(hd2, dd2, 4096 * NT, hipMemcpyDeviceToHost);
    (void)hipMemcpy(ha, da, 1024 * NT, hipMemcpyDeviceToHost);
    (void)hipMemcpy(hb, db, 1024 * NT, hipMemcpyDeviceToHost);
    double w_in = 0, w_true = 0, w_split = 0;
    int wt = 0, wi = 0, wj = 0;
    for (int t = 0; t < NT; t++)
    for (int i = 0; i < 32; i++)
      for (int j = 0; j < 32; j++) {
        double sm = 0, mag = 0, sx = 0;
        for (int k = 0; k < 16; k++) {
          const double tt = (double)(float)ha[t*512 + i * 16 + k] * (double)(float)hb[t*512 + j * 16 + k];
          sm += tt; mag = fmax(mag, fabs(tt));
        }
        const float *Q = hq + 96*t + 3*j, *P = hp + 96*t + 3*i;
        const double dx = (double)Q[0] - P[0], dy = (double)Q[1] - P[1], dz = (double)Q[2] - P[2];
        const double tr = dx*dx + dy*dy + dz*dz;
        const double D = hd2[t*1024 + i * 32 + j];
        const double e_in = fabs(D - sm) / mag, e_tr = fabs(D - tr) / mag, e_sp = fabs(sm - tr) / mag;
        if (e_in > w_in) w_in = e_in;
        if (e_tr > w_true) { wt = t; wi = i; wj = j; }
        w_true = fmax(w_true, e_tr);
        w_split = fmax(w_split, e_sp);
      }
    printf("d2 x%d tiles: max |D - fragment sum|/max term %.3e (2^%.1f) [t %d c %d q %d]; |D - true| %.3e; |fragment sum - true| %.3e\n",
           NT, w_in, log2(w_in + 1e-30), wt, wi, wj, w_true, w_split);
    for (int k = 0; k < 16; k++) printf("  k%2d a=%.8g b=%.8g\n", k, (double)(float)ha[wt*512+wi*16+k], (double)(float)hb[wt*512+wj*16+k]);
    printf("  D=%.9g q=(%.9g %.9g %.9g) p=(%.9g %.9g %.9g)\n", hd2[wt*1024+wi*32+wj], hq[96*wt+3*wj], hq[96*wt+3*wj+1], hq[96*wt+3*wj+2], hp[96*wt+3*wi], hp[96*wt+3*wi+1], hp[96*wt+3*wi+2]);
  }
  return 0;
}
