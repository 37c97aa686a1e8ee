// MEASURED AND NOT KEPT (round 6, scripts/gpu_r6h.sh, profiles/r06_enc_sincos_ab.txt): the library's sincosf is
// faster on gfx950 (0.35-0.43 ms per 16M samples x 30 against 0.50-0.54 for the float64 kernels below) and the
// headline forward ran 0.8 % slower with this in every encoding site.  Kept here with its accuracy check.
//
// The positional encoding's sines and cosines (models.py:27-41: sin(2^k x), cos(2^k x), k = 0..9, x in fp32) with
// ONE argument reduction per coordinate instead of one per frequency.
//
// 2^k x is exact in fp32, so every frequency's quarter-turn count is 2^k t with t = x (2/pi).  t is formed once in
// double-double (x C1 exactly split by an fma, plus x C2), and for each k the reduced angle r = 2^k t - rint(2^k t)
// (|r| <= 1/2 quarter turn, exact subtraction, the tail added after) is accurate to ~2^-60 absolute -- so the angle
// handed to the fp32 kernels is the correctly rounded reduction of the fp32 argument, as a full-range sincosf's
// Payne-Hanek path gives it, for |x| up to ~2^20 (positions here are metres; the KITTI / MaiCity scenes span < 100).
// The |a| <= pi/4 kernels are the Cephes single-precision minimax polynomials (|error| < 1 ulp over the range).
// Cost per frequency: six float64 ops and ~12 fp32 fma instead of the library's per-call large-argument reduction
// (~100 instructions, the encoding prologue's time in the query and the moment pass).
#pragma once

#include <hip/hip_runtime.h>

namespace pcn {

// sin / cos of the angle a + da (a fp32, da its rounding residual) plus n quarter turns
__host__ __device__ __forceinline__ void enc_sincos_kernel(float a, float da, int n, float& s, float& c) {
  const float z = a * a;
  // sin a = a + a z (S1 + z (S2 + z S3)),  cos a = 1 - z/2 + z^2 (C1 + z (C2 + z C3)); then the residual:
  // sin(a + da) = sin a + da cos a, cos(a + da) = cos a - da sin a (|da| <= 2^-25 |a|)
  const float ps = fmaf(fmaf(-1.9515295891e-4f, z, 8.3321608736e-3f), z, -1.6666654611e-1f);
  const float pc = fmaf(fmaf(2.443315711809948e-5f, z, -1.388731625493765e-3f), z, 4.166664568298827e-2f);
  const float ca0 = fmaf(z * z, pc, fmaf(-0.5f, z, 1.0f));
  const float sa = fmaf(a * z, ps, fmaf(da, ca0, a));
  const float ca = fmaf(-da, a, ca0);
  // quadrant n: (s, c) = (sa, ca), (ca, -sa), (-sa, -ca), (-ca, sa)
  const bool sw = n & 1;
  const float s0 = sw ? ca : sa, c0 = sw ? sa : ca;
  s = (n & 2) ? -s0 : s0;
  c = ((n + 1) & 2) ? -c0 : c0;
}

// the same kernel in float64 (Taylor to a^11 / a^12 on |a| <= pi/4: truncation < 1e-11 relative), rounded once
__host__ __device__ __forceinline__ void enc_sincos_kernel_d(double a, int n, float& s, float& c) {
  const double z = a * a;
  const double ps = fma(fma(fma(fma(-1.0 / 39916800.0, z, 1.0 / 362880.0), z, -1.0 / 5040.0), z, 1.0 / 120.0), z,
                        -1.0 / 6.0);
  const double pc = fma(fma(fma(fma(fma(1.0 / 479001600.0, z, -1.0 / 3628800.0), z, 1.0 / 40320.0), z, -1.0 / 720.0), z,
                            1.0 / 24.0), z, -0.5);
  const float sa = (float)fma(a * z, ps, a), ca = (float)fma(z, pc, 1.0);
  const bool sw = n & 1;
  const float s0 = sw ? ca : sa, c0 = sw ? sa : ca;
  s = (n & 2) ? -s0 : s0;
  c = ((n + 1) & 2) ? -c0 : c0;
}

// s[k] = sin(2^k x), c[k] = cos(2^k x), k = 0 .. NF - 1
template <int NF, bool D64 = false>
__host__ __device__ __forceinline__ void enc_sincos(float x, float (&s)[NF], float (&c)[NF]) {
  const double C1 = 0x1.45f306dc9c883p-1;    // fl64(2 / pi)
  const double C2 = -0x1.6b01ec5417056p-55;  // 2 / pi - C1
  const double PIO2 = 0x1.921fb54442d18p+0;  // fl64(pi / 2)
  const double xd = (double)x;
  const double th = xd * C1;
  const double tl = fma(xd, C1, -th) + xd * C2;   // x (2/pi) = th + tl to ~2^-100 relative
#pragma unroll
  for (int k = 0; k < NF; ++k) {
    const double sc = (double)(1 << k);
    const double u = th * sc, q = rint(u);
    const double r = (u - q) + tl * sc;        // quarter turns, |r| <= 1/2 (+ the tail)
    const int n = (int)(long long)q & 3;
    const double ad = r * PIO2;
    if (D64) {
      enc_sincos_kernel_d(ad, n, s[k], c[k]);
    } else {
      const float a = (float)ad;
      enc_sincos_kernel(a, (float)(ad - (double)a), n, s[k], c[k]);
    }
  }
}

// one frequency: sin(2^k x), cos(2^k x) (the per-feature staging forms)
__host__ __device__ __forceinline__ void enc_sincos1(float x, int k, float& s, float& c) {
  const double C1 = 0x1.45f306dc9c883p-1, C2 = -0x1.6b01ec5417056p-55, PIO2 = 0x1.921fb54442d18p+0;
  const double xd = (double)x;
  const double th = xd * C1;
  const double tl = fma(xd, C1, -th) + xd * C2;
  const double sc = (double)(1 << k);
  const double u = th * sc, q = rint(u);
  const double r = (u - q) + tl * sc;
  enc_sincos_kernel_d(r * PIO2, (int)(long long)q & 3, s, c);
}

}  // namespace pcn
