// Microbenchmark (diagnostic, not part of the library): fp32 MFMA shape 32x32x2 vs 16x16x4 on random operands,
// same FLOPs per wave, operands in registers, 2 waves per SIMD.  Prints TFLOP/s and the in-kernel clock
// (s_memtime / s_memrealtime x 100 MHz) after >= 2 s of back-to-back launches (MI355X_MICROARCH 'DVFS give-back').
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int ITERS = 4096;
#ifndef BARRIER
#define BARRIER 0
#endif

__global__ __launch_bounds__(512, 1) void k32(const float* __restrict__ in, float* __restrict__ out,
                                               unsigned long long* clk) {
  const int t = threadIdx.x;
  float a[8], b[8];
  for (int i = 0; i < 8; ++i) { a[i] = in[(blockIdx.x * 512 + t) * 16 + i]; b[i] = in[(blockIdx.x * 512 + t) * 16 + 8 + i]; }
  f32x16 acc[4] = {};
  unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int k = 0; k < 8; ++k)
#pragma unroll
      for (int c = 0; c < 4; ++c) acc[c] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[k], b[(k + c) & 7], acc[c], 0, 0, 0);
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  float s = 0.f;
  for (int c = 0; c < 4; ++c) for (int r = 0; r < 16; ++r) s += acc[c][r];
  out[blockIdx.x * 512 + t] = s;
  if (t == 0) { clk[2 * blockIdx.x] = t1 - t0; clk[2 * blockIdx.x + 1] = r1 - r0; }
}

// 16x16x4: 4 FLOP-equivalents: one 32x32x2 = 4096 FLOP, one 16x16x4 = 2048 FLOP -> twice the instructions
__global__ __launch_bounds__(512, 1) void k16(const float* __restrict__ in, float* __restrict__ out,
                                               unsigned long long* clk) {
  const int t = threadIdx.x;
  float a[8], b[8];
  for (int i = 0; i < 8; ++i) { a[i] = in[(blockIdx.x * 512 + t) * 16 + i]; b[i] = in[(blockIdx.x * 512 + t) * 16 + 8 + i]; }
  f32x4 acc[8] = {};
  unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int k = 0; k < 8; ++k)
#pragma unroll
      for (int c = 0; c < 8; ++c) acc[c] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[k], b[(k + c) & 7], acc[c], 0, 0, 0);
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  float s = 0.f;
  for (int c = 0; c < 8; ++c) for (int r = 0; r < 4; ++r) s += acc[c][r];
  out[blockIdx.x * 512 + t] = s;
  if (t == 0) { clk[2 * blockIdx.x] = t1 - t0; clk[2 * blockIdx.x + 1] = r1 - r0; }
}


// one accumulator chain per wave (k_train_ws's k-loop), operands in registers
__global__ __launch_bounds__(512, 1) void k32c1(const float* __restrict__ in, float* __restrict__ out,
                                                 unsigned long long* clk) {
  const int t = threadIdx.x;
  float a[8], b[8];
  for (int i = 0; i < 8; ++i) { a[i] = in[(blockIdx.x * 512 + t) * 16 + i]; b[i] = in[(blockIdx.x * 512 + t) * 16 + 8 + i]; }
  f32x16 acc = {};
  unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int k = 0; k < 8; ++k)
#pragma unroll
      for (int c = 0; c < 4; ++c) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[k], b[(k + c) & 7], acc, 0, 0, 0);
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  float s = 0.f;
  for (int r = 0; r < 16; ++r) s += acc[r];
  out[blockIdx.x * 512 + t] = s;
  if (t == 0) { clk[2 * blockIdx.x] = t1 - t0; clk[2 * blockIdx.x + 1] = r1 - r0; }
}

// one chain per wave, B operand from LDS: one ds_read_b128 per 4 MFMAs, read 3 k-groups ahead (k_train_ws)
__global__ __launch_bounds__(512, 1) void k32lds(const float* __restrict__ in, float* __restrict__ out,
                                                  unsigned long long* clk) {
  __shared__ f32x4 xs[32 * 64];
  const int t = threadIdx.x, lane = t & 63;
  for (int i = t; i < 32 * 64; i += 512) xs[i] = f32x4{in[i * 4], in[i * 4 + 1], in[i * 4 + 2], in[i * 4 + 3]};
  f32x4 w[32];
  for (int i = 0; i < 32; ++i) w[i] = f32x4{in[(blockIdx.x * 512 + t) * 16 + (i & 15)], in[t + i], in[t + 2 * i], in[t + 3 * i]};
  __syncthreads();
  f32x16 acc = {};
  unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < ITERS / 4; ++it) {
    const f32x4* xb = &xs[lane];
    f32x4 xr[4];
#pragma unroll
    for (int d = 0; d < 3; ++d) xr[d] = xb[d * 64];
#pragma unroll
    for (int kg = 0; kg < 32; ++kg) {
      if (kg + 3 < 32) xr[(kg + 3) % 4] = xb[(kg + 3) * 64];
#pragma unroll
      for (int q = 0; q < 4; ++q) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(w[kg][q], xr[kg % 4][q], acc, 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
    if (BARRIER) __syncthreads();
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  float s = 0.f;
  for (int r = 0; r < 16; ++r) s += acc[r];
  out[blockIdx.x * 512 + t] = s;
  if (t == 0) { clk[2 * blockIdx.x] = t1 - t0; clk[2 * blockIdx.x + 1] = r1 - r0; }
}

int main() {
  const int blocks = 256;
  const size_t nin = (size_t)blocks * 512 * 16;
  std::vector<float> h(nin);
  unsigned s = 12345;
  for (auto& x : h) { s = s * 1664525u + 1013904223u; x = (float)((s >> 8) & 0xffff) / 65536.0f - 0.5f; }
  float *din, *dout;
  unsigned long long* dclk;
  hipMalloc(&din, nin * 4);
  hipMalloc(&dout, (size_t)blocks * 512 * 4);
  hipMalloc(&dclk, (size_t)blocks * 16);
  hipMemcpy(din, h.data(), nin * 4, hipMemcpyHostToDevice);
  const double flop = (double)blocks * 8 * ITERS * 8 * 4 * 4096.0;   // waves x iters x 32 MFMA x 4096
  const char* names[4] = {"32x32x2 4 chains", "16x16x4 8 chains", "32x32x2 1 chain", "32x32x2 1 chain, B from LDS"};
  for (int which = 0; which < 4; ++which) {
    auto launch = [&]() {
      if (which == 0) hipLaunchKernelGGL(k32, dim3(blocks), dim3(512), 0, 0, din, dout, dclk);
      else if (which == 1) hipLaunchKernelGGL(k16, dim3(blocks), dim3(512), 0, 0, din, dout, dclk);
      else if (which == 2) hipLaunchKernelGGL(k32c1, dim3(blocks), dim3(512), 0, 0, din, dout, dclk);
      else hipLaunchKernelGGL(k32lds, dim3(blocks), dim3(512), 0, 0, din, dout, dclk);
    };
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    // warm: >= 2 s back to back
    hipEventRecord(e0);
    int warm = 0;
    float ms = 0.f;
    do { for (int i = 0; i < 20; ++i) launch(); warm += 20; hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms, e0, e1); } while (ms < 2000.f);
    hipEventRecord(e0);
    const int reps = 20;
    for (int i = 0; i < reps; ++i) launch();
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
    std::vector<unsigned long long> c(2 * blocks);
    hipMemcpy(c.data(), dclk, c.size() * 8, hipMemcpyDeviceToHost);
    std::vector<double> f;
    for (int b = 0; b < blocks; ++b) f.push_back((double)c[2 * b] / (double)c[2 * b + 1] * 100.0);
    std::sort(f.begin(), f.end());
    printf("%s: %.1f TFLOP/s, %.3f ms/launch, clock %.0f MHz (median over workgroups), warm launches %d\n",
           names[which], flop / (ms / reps * 1e-3) / 1e12, ms / reps, f[f.size() / 2], warm);
  }
  return 0;
}
