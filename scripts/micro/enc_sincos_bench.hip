// GPU timing + accuracy of the encoding's 30 sines/cosines per sample: the library's sincosf per frequency (what
// encode_full did) vs pcn::enc_sincos (one reduction per coordinate; fp32 or float64 kernels).  Prints ms per
// 16M samples and the max |difference| of each against the float64 kernel (correctly rounded on the host check).
// build: hipcc -O3 --offload-arch=gfx950 -I. enc_sincos_bench.hip -o enc_sincos_bench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include "enc_sincos.h"

template <int MODE>
__global__ __launch_bounds__(256) void k_enc(const float* __restrict__ p, int n, float* __restrict__ out,
                                             float* __restrict__ dump) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  float acc = 0.0f;
#pragma unroll
  for (int m = 0; m < 3; ++m) {
    const float x = p[3 * i + m];
    float s[10], c[10];
    if (MODE == 0) {
#pragma unroll
      for (int k = 0; k < 10; ++k) sincosf((float)(1 << k) * x, &s[k], &c[k]);
    } else {
      pcn::enc_sincos<10, MODE == 2>(x, s, c);
    }
#pragma unroll
    for (int k = 0; k < 10; ++k) {
      acc += s[k] * (float)(k + 1) + c[k];
      if (dump && i < 65536) {
        dump[((size_t)i * 3 + m) * 20 + k] = s[k];
        dump[((size_t)i * 3 + m) * 20 + 10 + k] = c[k];
      }
    }
  }
  out[i] = acc;
}

int main() {
  const int n = 1 << 24;
  std::vector<float> hp(3 * (size_t)n);
  unsigned st = 12345u;
  for (auto& v : hp) {
    st = st * 1664525u + 1013904223u;
    v = ((st >> 8) * (1.0f / 16777216.0f) - 0.5f) * 100.0f;   // metres, +-50
  }
  float *p, *out, *dump[3];
  hipMalloc(&p, hp.size() * 4);
  hipMalloc(&out, (size_t)n * 4);
  for (auto& d : dump) hipMalloc(&d, (size_t)65536 * 60 * 4);
  hipMemcpy(p, hp.data(), hp.size() * 4, hipMemcpyHostToDevice);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  auto run = [&](auto kern, float* d) {
    hipLaunchKernelGGL(kern, dim3(n / 256), dim3(256), 0, 0, p, n, out, d);
  };
  run(k_enc<0>, dump[0]);
  run(k_enc<1>, dump[1]);
  run(k_enc<2>, dump[2]);
  hipDeviceSynchronize();
  for (int rep = 0; rep < 3; ++rep) {
    float ms[3];
    for (int m = 0; m < 3; ++m) {
      hipEventRecord(e0);
      for (int it = 0; it < 10; ++it) {
        if (m == 0) run(k_enc<0>, nullptr);
        if (m == 1) run(k_enc<1>, nullptr);
        if (m == 2) run(k_enc<2>, nullptr);
      }
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      hipEventElapsedTime(&ms[m], e0, e1);
    }
    std::printf("ms per 16M samples: library sincosf %.3f, enc_sincos fp32 kernel %.3f, float64 kernel %.3f\n",
                ms[0] / 10, ms[1] / 10, ms[2] / 10);
  }
  std::vector<float> a(65536 * 60), b(65536 * 60), c(65536 * 60);
  hipMemcpy(a.data(), dump[0], a.size() * 4, hipMemcpyDeviceToHost);
  hipMemcpy(b.data(), dump[1], b.size() * 4, hipMemcpyDeviceToHost);
  hipMemcpy(c.data(), dump[2], c.size() * 4, hipMemcpyDeviceToHost);
  double d0 = 0, d1 = 0;
  size_t n0 = 0, n1 = 0;
  for (size_t i = 0; i < a.size(); ++i) {
    d0 = std::max(d0, (double)std::fabs(a[i] - c[i]));
    d1 = std::max(d1, (double)std::fabs(b[i] - c[i]));
    n0 += a[i] != c[i];
    n1 += b[i] != c[i];
  }
  std::printf("vs the float64 kernel: library max |diff| %.3g (%zu of %zu differ), fp32 kernel %.3g (%zu differ)\n", d0,
              n0, a.size(), d1, n1);
  return 0;
}
