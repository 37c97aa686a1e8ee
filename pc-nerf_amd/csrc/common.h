// Shared device helpers for the PC-NeRF render path (gfx950 / CDNA4, wave64).
//
// Compiled with -ffp-contract=off: the reference rounds every eager torch op separately
// (nof/render.py:432,458), and the positional encoding reaches sin(512 x) (nof/networks/models.py:23), so a
// fused multiply-add in z = near*(1-s)+far*s or p = o+d*z would move sample features by ~1e-3.  Where an FMA
// *is* the reference's arithmetic (torch.linspace's upper half) it is written explicitly with fmaf().
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <atomic>

#define PCN_WAVE 64

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

namespace pcn {

// torch.linspace(0, 1, n) on CPU, value i (verified bit-exact for n in 2..8192):
// step = 1/(n-1); lower half i*step, upper half fma(-(n-1-i), step, 1).
__device__ __forceinline__ float linspace01(int i, int n) {
  if (n == 1) return 0.0f;
  const float step = 1.0f / (float)(n - 1);
  if (i < n / 2) return (float)i * step;
  return fmaf(-(float)(n - 1 - i), step, 1.0f);
}

// z = near*(1-s) + far*s, rounded op by op (render.py:432).
__device__ __forceinline__ float lerp_z(float near, float far, float s) {
  const float a = near * (1.0f - s);
  const float b = far * s;
  return a + b;
}

__device__ __forceinline__ float wave_sum_f(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max_f(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// max |alpha(n) W[n][k]| over one layer's out_f x in_f weights by the whole block of NT threads (16-byte loads, eight
// in flight per thread: two or three rounds for a 256 x 256..319 layer; fmaxf drops NaN weights, in any order)
template <int NT, typename Alpha>
__device__ __forceinline__ float block_layer_absmax(const float* __restrict__ w, int out_f, int in_f, Alpha alpha) {
  const int total = out_f * in_f;
  float m = 0.0f;
  const int n4 = ((uintptr_t)w & 15) == 0 ? total >> 2 : 0;   // (an unaligned layer takes the scalar loop)
  const f32x4* __restrict__ w4 = reinterpret_cast<const f32x4*>(w);
  for (int i0 = threadIdx.x; i0 < n4; i0 += NT * 8) {
    f32x4 v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int i = i0 + NT * e;
      v[e] = i < n4 ? w4[i] : f32x4{};
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int i = i0 + NT * e;
      if (i < n4) {
#pragma unroll
        for (int q = 0; q < 4; ++q) m = fmaxf(m, fabsf(alpha((4 * i + q) / in_f) * v[e][q]));
      }
    }
  }
  for (int i = 4 * n4 + (int)threadIdx.x; i < total; i += NT) m = fmaxf(m, fabsf(alpha(i / in_f) * w[i]));
  m = wave_max_f(m);
  __shared__ float red[NT / 64];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  float r = 0.0f;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) r = fmaxf(r, red[i]);
  return r;
}

// torch sigmoid on CPU: 1 / (1 + exp(-x)).
__device__ __forceinline__ float sigmoid_ref(float x) { return 1.0f / (1.0f + expf(-x)); }

// nn.SmoothL1Loss(beta=1) element term on already-scaled inputs.
__device__ __forceinline__ float smooth_l1(float a, float b) {
  const float d = fabsf(a - b);
  return d < 1.0f ? 0.5f * d * d : d - 0.5f;
}


// ---- float64 64 x 64 tiles on v_mfma_f64_16x16x4_f64 (A[l&15][k=l>>4], B[k=l>>4][l&15], D[(l>>4)+4r][l&15]).
// Four waves per workgroup, wave w owns the 32 x 32 quadrant (rows 32(w>>1), columns 32(w&1)) as 2 x 2 blocks.
typedef double f64x4 __attribute__((ext_vector_type(4)));
constexpr int TP = 65;   // LDS pitch (doubles) of a 64-wide tile: odd, so 16 lanes' 8-byte reads are conflict-free

// acc += A B over k in [0, 64): A(r, k) = ATR ? As[k TP + r] : As[r TP + k], B(k, c) = BTR ? Bs[c TP + k] : Bs[k TP + c]
template <bool ATR, bool BTR>
__device__ __forceinline__ void mfma64_quad(const double* As, const double* Bs, int R, int Cc, int lane,
                                            f64x4 (&acc)[2][2]) {
  const int li = lane & 15, lk = lane >> 4;
#pragma unroll 4
  for (int k0 = 0; k0 < 64; k0 += 4) {
    const int k = k0 + lk;
    double a[2], b[2];
#pragma unroll
    for (int x = 0; x < 2; ++x) {
      const int r = R + 16 * x + li, c = Cc + 16 * x + li;
      a[x] = ATR ? As[k * TP + r] : As[r * TP + k];
      b[x] = BTR ? Bs[c * TP + k] : Bs[k * TP + c];
    }
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int y = 0; y < 2; ++y) acc[x][y] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[x], b[y], acc[x][y], 0, 0, 0);
  }
}

__device__ __forceinline__ int q_row(int R, int x, int r, int lane) { return R + 16 * x + (lane >> 4) + 4 * r; }
__device__ __forceinline__ int q_col(int Cc, int y, int lane) { return Cc + 16 * y + (lane & 15); }

}  // namespace pcn

// hipFuncSetAttribute (the dynamic-LDS cap) is per DEVICE: a launcher sets it the first time it runs on each device
// of the process, tracked by a bit per device id (a per-process flag left a second device's launches at
// the default cap).
inline bool pcn_attr_needed(const std::atomic<uint64_t>& mask) {
  int d = 0;
  (void)hipGetDevice(&d);
  return !(mask.load(std::memory_order_acquire) & (1ull << (d & 63)));
}
inline void pcn_attr_done(std::atomic<uint64_t>& mask) {
  int d = 0;
  (void)hipGetDevice(&d);
  mask.fetch_or(1ull << (d & 63), std::memory_order_release);
}
