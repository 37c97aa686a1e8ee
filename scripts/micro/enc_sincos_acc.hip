// Host-side accuracy check of pcn::enc_sincos (csrc/enc_sincos.h) against long-double sin/cos of the exact fp32
// arguments 2^k x, and of libm's sinf/cosf for comparison: max error in ulps of the fp32 result over random x in
// [-R, R].   build: hipcc -O2 -I. enc_sincos_acc.hip -o /tmp/esa && /tmp/esa
#include <cmath>
#include <cstdio>
#include <random>
#include "enc_sincos.h"

static double ulp_err(float got, long double ref) {
  const float rf = (float)ref;
  const float u = std::nextafter(std::fabs(rf), INFINITY) - std::fabs(rf);
  return (double)(std::fabs((long double)got - ref) / (long double)u);
}

int main() {
  std::mt19937_64 g(7);
  for (float R : {1.0f, 10.0f, 100.0f, 1000.0f}) {
    std::uniform_real_distribution<float> d(-R, R);
    double me = 0, le = 0, mae = 0, de = 0;
    for (int i = 0; i < 500000; ++i) {
      const float x = d(g);
      float s[10], c[10];
      float s2[10], c2[10];
      pcn::enc_sincos<10>(x, s, c);
      pcn::enc_sincos<10, true>(x, s2, c2);
      for (int k = 0; k < 10; ++k) {
        const float a = std::ldexp(x, k);
        const long double rs = sinl((long double)a), rc = cosl((long double)a);
        me = std::fmax(me, std::fmax(ulp_err(s[k], rs), ulp_err(c[k], rc)));
        de = std::fmax(de, std::fmax(ulp_err(s2[k], rs), ulp_err(c2[k], rc)));
        le = std::fmax(le, std::fmax(ulp_err(sinf(a), rs), ulp_err(cosf(a), rc)));
        mae = std::fmax(mae, (double)std::fmax(std::fabs(s[k] - rs), std::fabs(c[k] - rc)));
      }
    }
    std::printf("|x| <= %6.0f: enc_sincos max %.3f ulp (max abs %.3g), float64 kernel %.3f ulp, libm sinf/cosf %.3f ulp\n", R, me, mae, de, le);
  }
  return 0;
}
