// Optional per-kernel timing with HIP events, recorded on the launch stream around the library's kernels.
// Off by default (zero cost); bench.py turns it on over its timed region to measure the dominant kernel's
// average launch duration live (the rocprofv3 summary under profiles/ must agree with it).
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
  hipEvent_t e;
  PCN_HIP(hipEventCreate(&e));
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
