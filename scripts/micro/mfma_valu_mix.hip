// Microbenchmark (diagnostic, not part of the library): does the fp32 MFMA pipe (v_mfma_f32_32x32x2_f32, 64
// FLOP/clk/SIMD) run concurrently with fp32 VALU FMAs (v_fma_f32 / v_pk_fma_f32, also 64 FLOP/clk/SIMD) of
// OTHER waves on the same SIMD?  If yes, an fp32 GEMM split between MFMA waves and VALU waves can exceed the fp32
// MFMA peak with exact fp32 arithmetic.
// Workgroups of 256 CUs x (MW + VW) waves per SIMD: waves 0..4MW-1 run MFMA chains (2 independent accumulators),
// the rest run VALU FMA chains (16 independent accumulators), random operands.  Prints, per mix, the wall time of a
// launch (median of the last 20 of 200 back-to-back launches), the in-kernel clock, and TFLOP/s per role.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>

typedef float f32x16 __attribute__((ext_vector_type(16)));

#define CHECK(x)                                                              \
  do {                                                                        \
    hipError_t e = (x);                                                       \
    if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } \
  } while (0)

template <int MW, int VW>
__global__ __launch_bounds__(256 * (MW + VW)) void k_mix(const float* __restrict__ in, float* __restrict__ out,
                                                         unsigned long long* clk, int iters_m, int iters_v) {
  const int t = threadIdx.x, wid = t >> 6;
  const int g = blockIdx.x * blockDim.x + t;
  float a[8], b[8];
  for (int i = 0; i < 8; ++i) { a[i] = in[(g * 16 + i) & 1048575]; b[i] = in[(g * 16 + 8 + i) & 1048575]; }
  float s = 0.f;
  unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  if (wid < 4 * MW) {
    f32x16 acc0 = {}, acc1 = {};
    for (int it = 0; it < iters_m; ++it) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a[k], b[k], acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a[k], b[(k + 1) & 7], acc1, 0, 0, 0);
      }
    }
    for (int r = 0; r < 16; ++r) s += acc0[r] + acc1[r];
  } else {
    float x[16];
    for (int c = 0; c < 16; ++c) x[c] = a[c & 7] * 0.5f + (float)c;
    for (int it = 0; it < iters_v; ++it) {
#pragma unroll
      for (int r = 0; r < 32; ++r)
#pragma unroll
        for (int c = 0; c < 16; ++c) x[c] = fmaf(x[c], a[r & 7], b[(r + c) & 7]);
    }
    for (int c = 0; c < 16; ++c) s += x[c];
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  out[g] = s;
  if ((t & 63) == 0) { clk[2 * (blockIdx.x * 32 + wid)] = t1 - t0; clk[2 * (blockIdx.x * 32 + wid) + 1] = r1 - r0; }
}

template <int MW, int VW>
int run(const float* in, float* out, unsigned long long* clk, int iters_m, int iters_v) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  std::vector<float> ms;
  for (int rep = 0; rep < 200; ++rep) {
    CHECK(hipEventRecord(e0));
    hipLaunchKernelGGL((k_mix<MW, VW>), dim3(256), dim3(256 * (MW + VW)), 0, 0, in, out, clk, iters_m, iters_v);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float m;
    CHECK(hipEventElapsedTime(&m, e0, e1));
    if (rep >= 180) ms.push_back(m);
  }
  std::sort(ms.begin(), ms.end());
  const double t = ms[ms.size() / 2] * 1e-3;
  std::vector<unsigned long long> h(2 * 256 * 32);
  CHECK(hipMemcpy(h.data(), clk, h.size() * 8, hipMemcpyDeviceToHost));
  std::vector<double> f;
  for (int i = 0; i < 256 * 32; ++i)
    if (h[2 * i + 1]) f.push_back((double)h[2 * i] / (double)h[2 * i + 1] * 100.0);
  std::sort(f.begin(), f.end());
  const double fm = 256.0 * 4 * MW * (double)iters_m * 16 * 32 * 32 * 2 * 2;   // MFMA FLOP
  const double fv = 256.0 * 4 * VW * 64 * (double)iters_v * 32 * 16 * 2;       // VALU FLOP
  printf("MFMA waves/SIMD %d  VALU waves/SIMD %d : %8.3f ms  clock %4.0f MHz  MFMA %6.1f TF  VALU %6.1f TF  "
         "total %6.1f TF\n", MW, VW, t * 1e3, f.empty() ? 0.0 : f[f.size() / 2], fm / t / 1e12, fv / t / 1e12,
         (fm + fv) / t / 1e12);
  return 0;
}

int main() {
  float *in, *out;
  unsigned long long* clk;
  CHECK(hipMalloc(&in, 1048576 * 4));
  CHECK(hipMalloc(&out, 256 * 1024 * 4));
  CHECK(hipMalloc(&clk, 2 * 256 * 32 * 8));
  std::vector<float> h(1048576);
  unsigned s = 12345;
  for (auto& v : h) { s = s * 1664525u + 1013904223u; v = ((s >> 8) & 0xFFFF) / 65536.0f - 0.5f; }
  CHECK(hipMemcpy(in, h.data(), h.size() * 4, hipMemcpyHostToDevice));
  // iteration counts with equal FLOP per wave: 16 MFMA (65,536 FLOP) per MFMA iteration, 512 v_fma x 64 lanes
  // (65,536 FLOP) per VALU iteration
  const int IM = 3000, IV = 3000;
  int rc = 0;
  rc |= run<1, 0>(in, out, clk, IM, IV);
  rc |= run<2, 0>(in, out, clk, IM, IV);
  rc |= run<0, 1>(in, out, clk, IM, IV);
  rc |= run<0, 2>(in, out, clk, IM, IV);
  rc |= run<1, 1>(in, out, clk, IM, IV);
  rc |= run<1, 2>(in, out, clk, IM, IV);
  rc |= run<2, 2>(in, out, clk, IM, IV);
  rc |= run<1, 1>(in, out, clk, IM, IV / 2);
  rc |= run<1, 2>(in, out, clk, IM, IV / 2);
  return rc;
}
