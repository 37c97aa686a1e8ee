// Optional per-kernel timing with HIP events, recorded on the launch stream around the library's kernels.
// Off by default (zero cost); bench.py turns it on over its timed region to measure the dominant kernel's
// average launch duration live (the rocprofv3 summary under profiles/ must agree with it).
#include <algorithm>
#include <vector>

#include "pcnerf_internal.h"
#include "prof.h"

namespace pcn {

struct ProfRec {
  hipEvent_t a, b;
  int tag;
  double flops, bytes;
};
static std::vector<ProfRec> g_recs;
static std::vector<hipEvent_t> g_pool;
bool g_prof_on = false;

static hipEvent_t get_event() {
  if (!g_pool.empty()) {
    hipEvent_t e = g_pool.back();
    g_pool.pop_back();
    return e;
  }
  // timing-only events (read by hipEventElapsedTime after a device synchronise): no system-scope fence, whose L2
  // writeback + invalidate at every record put ~10 us between the instrumented step's kernels (and a cold L2 in
  // front of each), where the uninstrumented steps run them back to back
  hipEvent_t e;
  PCN_HIP(hipEventCreateWithFlags(&e, hipEventDisableSystemFence));
  return e;
}

ProfScope::ProfScope(hipStream_t s, int tag, double flops, double bytes) : s_(s), idx_(-1) {
  if (!g_prof_on) return;
  ProfRec r{get_event(), get_event(), tag, flops, bytes};
  PCN_HIP(hipEventRecord(r.a, s));
  g_recs.push_back(r);
  idx_ = (int)g_recs.size() - 1;
}
ProfScope::~ProfScope() {
  if (idx_ >= 0) (void)hipEventRecord(g_recs[idx_].b, s_);
}

}  // namespace pcn

using namespace pcn;

extern "C" int pcnerf_prof_enable(int on) {
  PCN_API_BEGIN
  for (auto& r : g_recs) {
    g_pool.push_back(r.a);
    g_pool.push_back(r.b);
  }
  g_recs.clear();
  g_prof_on = on != 0;
  PCN_API_END
}

extern "C" int pcnerf_prof_read(int tag, double* total_ms, int64_t* launches, double* flops, double* bytes) {
  PCN_API_BEGIN
  PCN_CHECK(total_ms && launches && flops && bytes, "pcnerf_prof_read: null argument");
  double t = 0.0, f = 0.0, b = 0.0;
  int64_t n = 0;
  for (auto& r : g_recs) {
    if (r.tag != tag) continue;
    PCN_HIP(hipEventSynchronize(r.b));
    float ms = 0.0f;
    PCN_HIP(hipEventElapsedTime(&ms, r.a, r.b));
    t += ms;
    f += r.flops;
    b += r.bytes;
    ++n;
  }
  *total_ms = t;
  *launches = n;
  *flops = f;
  *bytes = b;
  PCN_API_END
}

// ---------------------------------------------------------------------------------------------------------------
// What the fp16 matrix pipe sustains on this board right now (bench.py's roofline: "ceiling_measured_TFLOPs").
// The headline query issues v_mfma_f32_16x16x32_f16 at one wave per SIMD with its B operands read from LDS; this
// kernel is that loop and nothing else: random fp16 operands (the power the pipe draws depends on the data), 24
// accumulators of 16x16 per wave (64 neurons x 96 samples), 3 products per k-step of 32, 256 workgroups of 4 waves.
// Run back to back for `seconds` so the board settles at its power-limited clock (MI355X_MICROARCH 'DVFS
// give-back'), then timed with HIP events over the second half; the shader clock from s_memtime / s_memrealtime.
namespace pcn {
typedef _Float16 h16x8 __attribute__((ext_vector_type(8)));
constexpr int CEIL_ITERS = 1024;
constexpr int CEIL_BLOCKS = 256;

__global__ __launch_bounds__(256) void k_ceiling_init(float* __restrict__ in) {
  const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned s = i * 2654435761u + 12345u;
  s ^= s >> 13;
  s *= 1664525u;
  s += 1013904223u;
  s ^= s >> 16;
  in[i] = (float)(s >> 8) / 16777216.0f - 0.5f;
}

__global__ __launch_bounds__(256, 1) void k_ceiling(const float* __restrict__ in, float* __restrict__ out,
                                                    unsigned long long* __restrict__ clk) {
  __shared__ h16x8 sb[8][256];
  const int t = threadIdx.x, g = blockIdx.x * blockDim.x + t;
  h16x8 a[4];
  for (int i = 0; i < 4; ++i)
    for (int e = 0; e < 8; ++e) a[i][e] = (_Float16)in[(g * 64 + i * 8 + e) & 65535];
  for (int i = 0; i < 8; ++i) {
    h16x8 b;
    for (int e = 0; e < 8; ++e) b[e] = (_Float16)in[(g * 64 + 32 + i * 8 + e) & 65535];
    sb[i][t] = b;
  }
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  f32x4 acc[24] = {};
  for (int it = 0; it < CEIL_ITERS; ++it) {
#pragma unroll
    for (int p = 0; p < 3; ++p)
#pragma unroll
      for (int c = 0; c < 24; ++c)
        acc[c] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[(p + c) & 3], sb[(c + p) & 7][t], acc[c], 0, 0, 0);
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  float s = 0.0f;
  for (int c = 0; c < 24; ++c)
    for (int r = 0; r < 4; ++r) s += acc[c][r];
  out[g] = s;
  if (t == 0) {
    clk[2 * blockIdx.x] = t1 - t0;
    clk[2 * blockIdx.x + 1] = r1 - r0;
  }
}
}  // namespace pcn

extern "C" int pcnerf_mfma_ceiling(double seconds, double* tflops, double* clock_mhz, void* stream) {
  PCN_API_BEGIN
  PCN_CHECK(tflops && clock_mhz, "pcnerf_mfma_ceiling: null argument");
  PCN_CHECK(seconds > 0.0 && seconds <= 30.0, "pcnerf_mfma_ceiling: seconds must be in (0, 30]");
  hipStream_t s = (hipStream_t)stream;
  float *in = nullptr, *out = nullptr;
  unsigned long long* clk = nullptr;
  PCN_HIP(hipMalloc(&in, 65536 * sizeof(float)));
  PCN_HIP(hipMalloc(&out, CEIL_BLOCKS * 256 * sizeof(float)));
  PCN_HIP(hipMalloc(&clk, 2 * CEIL_BLOCKS * sizeof(unsigned long long)));
  hipLaunchKernelGGL(k_ceiling_init, dim3(256), dim3(256), 0, s, in);
  hipEvent_t e0, e1;
  PCN_HIP(hipEventCreate(&e0));
  PCN_HIP(hipEventCreate(&e1));
  // one launch: 256 x 4 waves x CEIL_ITERS x 3 products x 24 MFMAs x (16 x 16 x 32 x 2) FLOP
  const double flop = (double)CEIL_BLOCKS * 4 * CEIL_ITERS * 3 * 24 * (16.0 * 16 * 32 * 2);
  // settle: launches for the first half of `seconds`, in batches of 8 so the queue never runs dry
  float ms = 0.0f;
  double settled = 0.0;
  while (settled < 0.5e3 * seconds) {
    PCN_HIP(hipEventRecord(e0, s));
    for (int i = 0; i < 8; ++i) hipLaunchKernelGGL(k_ceiling, dim3(CEIL_BLOCKS), dim3(256), 0, s, in, out, clk);
    PCN_HIP(hipEventRecord(e1, s));
    PCN_HIP(hipEventSynchronize(e1));
    PCN_HIP(hipEventElapsedTime(&ms, e0, e1));
    settled += ms;
  }
  // measure: the same batches over the second half
  const int per = (int)std::max(8.0, 8.0 * (0.5e3 * seconds) / std::max((double)ms, 1e-3));
  PCN_HIP(hipEventRecord(e0, s));
  for (int i = 0; i < per; ++i) hipLaunchKernelGGL(k_ceiling, dim3(CEIL_BLOCKS), dim3(256), 0, s, in, out, clk);
  PCN_HIP(hipEventRecord(e1, s));
  PCN_HIP(hipEventSynchronize(e1));
  PCN_HIP(hipEventElapsedTime(&ms, e0, e1));
  PCN_LAUNCH_CHECK("pcnerf_mfma_ceiling");
  std::vector<unsigned long long> h(2 * CEIL_BLOCKS);
  PCN_HIP(hipMemcpy(h.data(), clk, h.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
  std::vector<double> mhz;
  for (int b = 0; b < CEIL_BLOCKS; ++b)
    if (h[2 * b + 1] > 0) mhz.push_back((double)h[2 * b] / (double)h[2 * b + 1] * 100.0);   // memrealtime: 100 MHz
  std::sort(mhz.begin(), mhz.end());
  *tflops = flop * per / (ms * 1e-3) / 1e12;
  *clock_mhz = mhz.empty() ? 0.0 : mhz[mhz.size() / 2];
  PCN_HIP(hipEventDestroy(e0));
  PCN_HIP(hipEventDestroy(e1));
  PCN_HIP(hipFree(in));
  PCN_HIP(hipFree(out));
  PCN_HIP(hipFree(clk));
  PCN_API_END
}
