// Microbenchmark (diagnostic, not part of the library): one wave per SIMD issuing v_mfma_f32_32x32x16_f16 on C
// independent accumulators with N independent VALU instructions (fma / cvt_pk / fma_mix: the split epilogue's mix)
// placed in every MFMA gap by sched_group_barrier.  Prints cycles per MFMA (in-kernel s_memtime) per (C, N).
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

template <int C, int N>
__global__ __launch_bounds__(256, 1) void k(const float* in, float* out, unsigned long long* clk, int iters) {
  const int t = threadIdx.x, g = blockIdx.x * blockDim.x + t;
  f16x8 a[2], b[2];
  for (int i = 0; i < 2; ++i)
    for (int e = 0; e < 8; ++e) {
      a[i][e] = (_Float16)in[(g * 32 + i * 8 + e) & 65535];
      b[i][e] = (_Float16)in[(g * 32 + 16 + i * 8 + e) & 65535];
    }
  float v[16];
  for (int i = 0; i < 16; ++i) v[i] = in[(g + 97 * i) & 65535];
  f32x16 acc[C] = {};
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int m = 0; m < 24; ++m) {
      const int c = m % C;
      acc[c] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[m & 1], b[(m >> 1) & 1], acc[c], 0, 0, 0);
#pragma unroll
      for (int q = 0; q < N; ++q) {
        const int i = (m * N + q) & 15;
        v[i] = __builtin_fmaf(v[i], 1.0001f, 0.5f);
      }
    }
#pragma unroll
    for (int m = 0; m < 24; ++m) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      if (N) __builtin_amdgcn_sched_group_barrier(0x002, N, 0);
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0;
  for (int c = 0; c < C; ++c)
    for (int r = 0; r < 16; ++r) s += acc[c][r];
  for (int i = 0; i < 16; ++i) s += v[i];
  out[g] = s;
  if (t == 0) clk[blockIdx.x] = t1 - t0;
}

template <int C, int N>
void run(const float* in, float* out, unsigned long long* clk, int iters) {
  std::vector<double> cyc;
  for (int r = 0; r < 20; ++r) {
    hipLaunchKernelGGL((k<C, N>), dim3(256), dim3(256), 0, 0, in, out, clk, iters);
    hipDeviceSynchronize();
    if (r < 5) continue;
    std::vector<unsigned long long> h(256);
    hipMemcpy(h.data(), clk, 256 * 8, hipMemcpyDeviceToHost);
    std::sort(h.begin(), h.end());
    cyc.push_back((double)h[128] / (iters * 24.0));
  }
  std::sort(cyc.begin(), cyc.end());
  printf("{\"chains\": %d, \"valu_per_gap\": %d, \"cycles_per_mfma\": %.2f}\n", C, N, cyc[cyc.size() / 2]);
}

int main() {
  float *in, *out;
  unsigned long long* clk;
  (void)hipMalloc(&in, 65536 * 4);
  (void)hipMalloc(&out, 256 * 256 * 4);
  (void)hipMalloc(&clk, 256 * 8);
  std::vector<float> h(65536);
  for (int i = 0; i < 65536; ++i) h[i] = (float)((i * 2654435761u) % 1000) / 1000.0f - 0.5f;
  (void)hipMemcpy(in, h.data(), 65536 * 4, hipMemcpyHostToDevice);
  const int it = 400;
  run<2, 0>(in, out, clk, it); run<2, 2>(in, out, clk, it); run<2, 4>(in, out, clk, it); run<2, 6>(in, out, clk, it);
  run<6, 0>(in, out, clk, it); run<6, 4>(in, out, clk, it); run<1, 0>(in, out, clk, it); run<1, 4>(in, out, clk, it);
  return 0;
}
