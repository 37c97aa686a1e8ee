// Checks on the GPU that the fp16 split's low part formed by v_fma_mixlo/hi_f16 (one mixed-precision fma,
// mid = f16(v - f32(hi)), one rounding) is bit-identical to the two-step form the kernels used before
// (f32 subtraction, then a conversion): the subtraction is exact in f32 (hi is v rounded to 11 bits), so both round
// the same real number once.  Random fp32 values over the whole finite range plus edge cases (fp16 subnormal /
// overflow neighbourhoods, zeros, powers of two).   build: hipcc -O3 --offload-arch=gfx950 split_mix.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <vector>

typedef _Float16 h2 __attribute__((ext_vector_type(2)));

__global__ void k_split(const float* __restrict__ in, int64_t n, unsigned* __restrict__ ref, unsigned* __restrict__ mix) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (2 * i + 1 >= n) return;
  const float v0 = in[2 * i], v1 = in[2 * i + 1];
  h2 hi;
  hi[0] = (_Float16)v0;
  hi[1] = (_Float16)v1;
  h2 m;
  m[0] = (_Float16)(v0 - (float)hi[0]);
  m[1] = (_Float16)(v1 - (float)hi[1]);
  const unsigned hb = __builtin_bit_cast(unsigned, hi);
  ref[i] = __builtin_bit_cast(unsigned, m);
  unsigned mid;
  asm("v_fma_mixlo_f16 %0, %1, -1.0, %2 op_sel_hi:[1,0,0]" : "=v"(mid) : "v"(hb), "v"(v0));
  asm("v_fma_mixhi_f16 %0, %1, -1.0, %2 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "+v"(mid) : "v"(hb), "v"(v1));
  mix[i] = mid;
}

int main() {
  const int64_t n = 1 << 26;
  std::vector<float> h(n);
  uint64_t s = 0x9E3779B97F4A7C15ull;
  auto rnd = [&]() { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; };
  int64_t i = 0;
  // edge cases: around fp16's subnormal range, its largest finite values, zeros, powers of two
  const float edges[] = {0.0f, -0.0f, 6.1035156e-05f, 5.9604645e-08f, 2.9802322e-08f, 65504.0f, 65519.99f, 1.0f,
                         -1.0f, 3.0517578e-05f, 1e-10f, -1e-10f, 4096.0001f, 1.00048828125f};
  for (float e : edges) h[i++] = e;
  for (; i < n; ++i) {
    uint32_t b = (uint32_t)rnd();
    // exponents concentrated where the split is used (|v| < 2^16): biased exponent 90..142
    const uint32_t ex = 90 + (uint32_t)(rnd() % 53);
    b = (b & 0x807FFFFFu) | (ex << 23);
    std::memcpy(&h[i], &b, 4);
  }
  float* d;
  unsigned *r, *m;
  hipMalloc(&d, n * 4);
  hipMalloc(&r, n * 2);
  hipMalloc(&m, n * 2);
  hipMemcpy(d, h.data(), n * 4, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k_split, dim3((unsigned)((n / 2 + 255) / 256)), dim3(256), 0, 0, d, n, r, m);
  std::vector<unsigned> hr(n / 2), hm(n / 2);
  hipMemcpy(hr.data(), r, n * 2, hipMemcpyDeviceToHost);
  hipMemcpy(hm.data(), m, n * 2, hipMemcpyDeviceToHost);
  int64_t bad = 0;
  for (int64_t j = 0; j < n / 2; ++j)
    if (hr[j] != hm[j]) {
      if (bad < 5) printf("mismatch at %lld: %08x vs %08x (v %g %g)\n", (long long)j, hr[j], hm[j], h[2 * j], h[2 * j + 1]);
      ++bad;
    }
  printf("{\"values\": %lld, \"mismatches\": %lld}\n", (long long)n, (long long)bad);
  return bad != 0;
}
