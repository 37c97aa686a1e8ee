// Microbenchmark (diagnostic): v_mfma_f32_32x32x16_f16 throughput with ONE dependent accumulator chain per wave vs
// two / four independent chains, at 1 and 2 waves per SIMD (k_train_h runs one chain per wave, 2 waves per SIMD).
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

template <int CH>
__global__ __launch_bounds__(512) void k(const float* in, float* out, int iters) {
  const int t = threadIdx.x, g = blockIdx.x * blockDim.x + t;
  f16x8 a[4], b[4];
  for (int i = 0; i < 4; ++i)
    for (int e = 0; e < 8; ++e) { a[i][e] = (_Float16)in[(g * 64 + i * 8 + e) & 65535]; b[i][e] = (_Float16)in[(g * 64 + 32 + i * 8 + e) & 65535]; }
  f32x16 acc[CH] = {};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k2 = 0; k2 < 12; ++k2)
#pragma unroll
      for (int c = 0; c < CH; ++c) acc[c] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[(k2 + c) & 3], b[k2 & 3], acc[c], 0, 0, 0);
  }
  float s = 0;
  for (int c = 0; c < CH; ++c) for (int r = 0; r < 16; ++r) s += acc[c][r];
  out[g] = s;
}

template <int CH>
void run(const float* in, float* out, int threads, int iters) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  std::vector<float> ms;
  for (int r = 0; r < 30; ++r) {
    hipEventRecord(e0);
    hipLaunchKernelGGL(k<CH>, dim3(256), dim3(threads), 0, 0, in, out, iters / CH);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float m; hipEventElapsedTime(&m, e0, e1); if (r >= 10) ms.push_back(m);
  }
  std::sort(ms.begin(), ms.end());
  const double t = ms[ms.size() / 2] * 1e-3;
  const double mf = 256.0 * (threads / 64) * (double)(iters / CH) * 12 * CH;
  printf("chains %d waves/SIMD %d: %.3f ms  %.1f cycles per MFMA per SIMD at 2.4 GHz (%.0f TF fp16)\n", CH, threads / 256,
         t * 1e3, t * 2.4e9 / (mf / 1024.0), mf * 32768.0 / t / 1e12);
}

int main() {
  float *in, *out;
  hipMalloc(&in, 65536 * 4); hipMalloc(&out, 256 * 512 * 4);
  std::vector<float> h(65536);
  for (int i = 0; i < 65536; ++i) h[i] = (float)((i * 2654435761u) % 1000) / 1000.0f - 0.5f;
  hipMemcpy(in, h.data(), 65536 * 4, hipMemcpyHostToDevice);
  for (int th : {256, 512}) { run<1>(in, out, th, 2400); run<2>(in, out, th, 2400); run<4>(in, out, th, 2400); }
  return 0;
}
