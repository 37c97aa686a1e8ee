// Microbenchmark (diagnostic, not part of the library): k_bwd_fused's LDS access patterns (nof_train.hip fb_off
// swizzle) timed per wave-instruction with s_memtime, one wave per SIMD, 4096 back-to-back instructions per
// pattern: the data gradient's ds_read_b128, the weight gradient's ds_read_b64_tr_b16 (g and x images), the split
// writes (ds_write_b64), the epilogue's ds_read_b64.  Prints cycles per instruction (ideal: b128 4, b64 2).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

template <int P>
__device__ __forceinline__ int off(int r, int c, int mode) {
  if (mode == 0) {   // fb_off: XOR swizzle of 16-B chunks by row
    const int swz = 2 * ((r & 3) | ((r & 8) >> 1));
    return r * P + 16 * ((c >> 3) ^ swz) + 2 * (c & 7);
  }
  if (mode == 3) {   // nof_train.hip's fb_swz (round 4 final)
    const int f = 2 * ((r & 3) | ((((r >> 2) ^ (r >> 3)) & 1) << 2)) | ((r >> 2) & 1);
    return r * P + 16 * ((c >> 3) ^ f) + 2 * (c & 7);
  }
  // mode 1: rows padded by 16 B, no swizzle; mode 2: rows padded by 16 B + the XOR swizzle
  const int swz = mode == 2 ? 2 * ((r & 3) | ((r & 8) >> 1)) : 0;
  return r * (P + 16) + 16 * ((c >> 3) ^ swz) + 2 * (c & 7);
}

typedef int i32x2 __attribute__((ext_vector_type(2)));
typedef int i32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256, 1) void k(int pattern, int mode, unsigned long long* out, int* sink) {
  __shared__ __attribute__((aligned(16))) char lds[65536];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6, kg = lane >> 4, lm = lane & 15;
  for (int i = t; i < 65536 / 4; i += 256) reinterpret_cast<int*>(lds)[i] = i;
  __syncthreads();
  int acc = 0;
  unsigned a0;
  // per pattern: one address per lane (wave-dependent), instruction repeated with alternating immediates
  if (pattern == 0) a0 = off<512>(lm, 8 * kg, mode);                                  // dgrad b128 (ks 0, sb 0)
  else if (pattern == 1) a0 = off<512>(8 * kg + (lm >> 2), 32 * wv + 4 * (lm & 3), mode);   // tr read, g
  else if (pattern == 2) a0 = off<256>(8 * kg + (lm >> 2), 4 * (lm & 3), mode);       // tr read, x
  else if (pattern == 3 && mode < 3) a0 = off<512>(lane & 31, 8 * wv + 4 * ((lane >> 5) & 1), mode);   // split write, g
  else if (pattern == 3) a0 = off<512>(lm, 8 * (4 * wv + (lane >> 5)) + 4 * ((lane >> 4) & 1), mode);   // its final map
  else a0 = off<256>(lm, 16 * wv + 4 * kg, mode);                                      // epilogue read x
  const unsigned base = (unsigned)(uintptr_t)(__attribute__((address_space(3))) char*)lds;
  const unsigned addr = base + a0;
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < 512; ++it) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      if (pattern == 0) {
        i32x4 v;
        asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(addr));
        acc += v[0];
      } else if (pattern == 1 || pattern == 2) {
        i32x2 v;
        asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(v) : "v"(addr));
        acc += v[0];
      } else if (pattern == 3) {
        i32x2 v = {acc, it};
        asm volatile("ds_write_b64 %0, %1" ::"v"(addr), "v"(v));
      } else {
        i32x2 v;
        asm volatile("ds_read_b64 %0, %1" : "=v"(v) : "v"(addr));
        acc += v[0];
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)");
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) out[blockIdx.x * 4 + wv] = t1 - t0;
  sink[blockIdx.x * 256 + t] = acc;
}

int main() {
  unsigned long long* out;
  int* sink;
  (void)hipMalloc(&out, 256 * 4 * 8);
  (void)hipMalloc(&sink, 256 * 256 * 4);
  const char* names[] = {"dgrad ds_read_b128", "tr read g", "tr read x", "split ds_write_b64", "epilogue ds_read_b64"};
  for (int mode = 0; mode < 4; ++mode)
    for (int p = 0; p < 5; ++p) {
      hipLaunchKernelGGL(k, dim3(256), dim3(256), 0, 0, p, mode, out, sink);
      (void)hipDeviceSynchronize();
      std::vector<unsigned long long> h(1024);
      (void)hipMemcpy(h.data(), out, 1024 * 8, hipMemcpyDeviceToHost);
      double s = 0;
      for (auto v : h) s += (double)v;
      // s_memtime ticks at the shader clock; 4096 instructions per wave, 4 waves per CU share the LDS
      printf("{\"mode\": %d, \"pattern\": \"%s\", \"cycles_per_instr_per_CU\": %.2f}\n", mode, names[p],
             s / 1024 / 4096 / 4);
    }
  return 0;
}
