// Microbenchmark (diagnostic, not part of the library): fp16 MFMA shape v_mfma_f32_32x32x16_f16 vs
// v_mfma_f32_16x16x32_f16 on random operands, equal FLOPs per wave, one wave per SIMD, operands in registers
// (optionally re-read from LDS per MFMA, as the eval query does).  Prints TFLOP/s and the in-kernel clock after
// >= 2 s of back-to-back launches (MI355X_MICROARCH 'DVFS give-back' items 6-7).
#include <hip/hip_runtime.h>
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

constexpr int ITERS = 2048;

// S = 32: 6 accumulators of 32x32 (one k-step of 16 for 2 neuron blocks x 3 tiles); S = 16: 24 accumulators of 16x16
// (the same 64 neurons x 96 samples, K = 32 per MFMA, so half the MFMAs per k-step pair)
template <int S, bool LDS>
__global__ __launch_bounds__(256, 1) void k(const float* in, float* out, unsigned long long* clk) {
  __shared__ f16x8 sb[8][256];
  const int t = threadIdx.x, g = blockIdx.x * blockDim.x + t;
  f16x8 a[4], b[8];
  for (int i = 0; i < 4; ++i)
    for (int e = 0; e < 8; ++e) a[i][e] = (_Float16)in[(g * 64 + i * 8 + e) & 65535];
  for (int i = 0; i < 8; ++i) {
    for (int e = 0; e < 8; ++e) b[i][e] = (_Float16)in[(g * 64 + 32 + i * 8 + e) & 65535];
    sb[i][t] = b[i];
  }
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  if constexpr (S == 32) {
    f32x16 acc[6] = {};
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)   // two k-steps of 16 = 32 features, 3 products each
#pragma unroll
        for (int p = 0; p < 3; ++p)
#pragma unroll
          for (int c = 0; c < 6; ++c) {
            const f16x8 bb = LDS ? sb[(c + p + kk) & 7][t] : b[(c + p + kk) & 7];
            acc[c] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[(p + kk) & 3], bb, acc[c], 0, 0, 0);
          }
    }
    float s = 0;
    for (int c = 0; c < 6; ++c)
      for (int r = 0; r < 16; ++r) s += acc[c][r];
    out[g] = s;
  } else {
    f32x4 acc[24] = {};
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
      for (int p = 0; p < 3; ++p)   // one k-step of 32 features, 3 products
#pragma unroll
        for (int c = 0; c < 24; ++c) {
          const f16x8 bb = LDS ? sb[(c + p) & 7][t] : b[(c + p) & 7];
          acc[c] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[(p + c) & 3], bb, acc[c], 0, 0, 0);
        }
    }
    float s = 0;
    for (int c = 0; c < 24; ++c)
      for (int r = 0; r < 4; ++r) s += acc[c][r];
    out[g] = s;
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  if (t == 0) {
    clk[2 * blockIdx.x] = t1 - t0;
    clk[2 * blockIdx.x + 1] = r1 - r0;
  }
}

template <int S, bool LDS>
void run(const float* in, float* out, unsigned long long* clk) {
  auto t0 = std::chrono::steady_clock::now();
  int n = 0;
  while (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() < 2.0) {
    hipLaunchKernelGGL((k<S, LDS>), dim3(256), dim3(256), 0, 0, in, out, clk);
    if (++n % 16 == 0) (void)hipDeviceSynchronize();
  }
  (void)hipDeviceSynchronize();
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  std::vector<float> ms;
  for (int r = 0; r < 20; ++r) {
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL((k<S, LDS>), dim3(256), dim3(256), 0, 0, in, out, clk);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float m;
    (void)hipEventElapsedTime(&m, e0, e1);
    ms.push_back(m);
  }
  std::sort(ms.begin(), ms.end());
  std::vector<unsigned long long> h(512);
  (void)hipMemcpy(h.data(), clk, 512 * 8, hipMemcpyDeviceToHost);
  std::vector<double> mhz;
  for (int b = 0; b < 256; ++b) mhz.push_back((double)h[2 * b] / (double)h[2 * b + 1] * 100.0);
  std::sort(mhz.begin(), mhz.end());
  // FLOP per launch: 256 blocks x 4 waves x ITERS x (64 neurons x 96 samples x 32 features x 2 x 3)
  const double flop = 256.0 * 4 * ITERS * (64.0 * 96 * 32 * 2 * 3);
  printf("{\"shape\": \"%s\", \"lds_B\": %d, \"ms\": %.3f, \"TFLOPs\": %.1f, \"clock_MHz\": %.0f}\n",
         S == 32 ? "32x32x16" : "16x16x32", (int)LDS, ms[10], flop / (ms[10] * 1e-3) / 1e12, mhz[128]);
}

int main() {
  float *in, *out;
  unsigned long long* clk;
  (void)hipMalloc(&in, 65536 * 4);
  (void)hipMalloc(&out, 256 * 256 * 4);
  (void)hipMalloc(&clk, 512 * 8);
  std::vector<float> h(65536);
  unsigned s = 12345;
  for (int i = 0; i < 65536; ++i) {
    s = s * 1664525u + 1013904223u;
    h[i] = (float)(s >> 8) / 16777216.0f - 0.5f;
  }
  (void)hipMemcpy(in, h.data(), 65536 * 4, hipMemcpyHostToDevice);
  run<32, false>(in, out, clk);
  run<16, false>(in, out, clk);
  run<32, true>(in, out, clk);
  run<16, true>(in, out, clk);
  run<32, false>(in, out, clk);
  run<16, false>(in, out, clk);
  return 0;
}
