// Per-ray stages of the render path: coarse sampling, perturbation, occupancy compositing with the child
// masks and loss terms, importance resampling + merge, and the loss reductions (nof/render.py).
// These stages read/write a few bytes per sample and are bound by HBM, not by arithmetic: one wave per ray,
// samples of a ray in contiguous per-lane blocks, scans in registers + cross-lane shuffles, no atomics on
// the per-ray path.
#include <stdio.h>

#include <mutex>
#include <string>

#include "common.h"
#include "pcnerf_internal.h"
#include "prof.h"

namespace pcn {

static thread_local std::string g_last_error;
void set_error(const std::string& msg) { g_last_error = msg; }

bool to_dev_params(const pcnerf_nof_params* p, float eps, NofParamsDev* d) {
  for (int i = 0; i < 8; ++i) {
    if (!p->lin_w[i] || !p->lin_b[i] || !p->bn_w[i] || !p->bn_b[i] || !p->bn_rm[i] || !p->bn_rv[i]) return false;
    d->lin_w[i] = p->lin_w[i];
    d->lin_b[i] = p->lin_b[i];
    d->bn_w[i] = p->bn_w[i];
    d->bn_b[i] = p->bn_b[i];
    d->bn_rm[i] = p->bn_rm[i];
    d->bn_rv[i] = p->bn_rv[i];
  }
  if (!p->out_w || !p->out_b) return false;
  d->out_w = p->out_w;
  d->out_b = p->out_b;
  d->eps = eps;
  return true;
}

// ------------------------------------------------------------------------------- coarse sampling
// render.py:429-442.  One wave per ray; segmented sampling merges the parent and child linspace lists by
// rank (count of smaller values + equal values with a lower index), which is the sorted order for any input.
__device__ __forceinline__ float seg_value(int a, int sp, int sc, float near, float far, float cn, float cf) {
  return a < sp ? lerp_z(near, far, linspace01(a, sp)) : lerp_z(cn, cf, linspace01(a - sp, sc));
}

__global__ __launch_bounds__(256) void k_sample_coarse(const float* __restrict__ rays, int64_t n_rays, int stride,
                                                       int near_col, int far_col, int cn_col, int cf_col, int S,
                                                       int sp, int disparity, float* __restrict__ z) {
  const int lane = threadIdx.x & 63;
  const int64_t ray = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (ray >= n_rays) return;
  const float* r = rays + ray * stride;
  const float near = r[near_col], far = r[far_col];
  float* zr = z + ray * S;
  if (disparity) {  // render.py:565-567: z = 1 / (1/near*(1-s) + 1/far*s)
    const float in = 1.0f / near, inf_ = 1.0f / far;
    for (int i = lane; i < S; i += 64) {
      const float sv = linspace01(i, S);
      const float a = in * (1.0f - sv);
      const float b = inf_ * sv;
      zr[i] = 1.0f / (a + b);
    }
    return;
  }
  if (sp >= S) {
    for (int i = lane; i < S; i += 64) zr[i] = lerp_z(near, far, linspace01(i, S));
    return;
  }
  const float cn = r[cn_col], cf = r[cf_col];
  const int sc = S - sp;
  // Both lists are linspaces, so (after rounding) almost always non-decreasing; then the rank of a parent value
  // is its index plus the child values strictly below it (equal child values have higher indices), and the rank
  // of a child value its index plus the parent values <= it -- two binary searches instead of S comparisons.
  // The wave checks monotonicity first and falls back to the all-pairs rank otherwise (identical output).
  // A NaN bound (NaN values compare false) makes the list non-monotone, so such rays take the rank path, which
  // orders NaNs last like torch.sort.
  bool mono = true;
  for (int a = lane; a < S; a += 64) {
    const float va = seg_value(a, sp, sc, near, far, cn, cf);
    if (!(va == va) || (a + 1 < S && a + 1 != sp && !(va <= seg_value(a + 1, sp, sc, near, far, cn, cf))))
      mono = false;
  }
  if (__all(mono)) {
    for (int a = lane; a < S; a += 64) {
      const float va = seg_value(a, sp, sc, near, far, cn, cf);
      int lo, hi;   // search [lo, hi) of the other list for the first element not counted
      if (a < sp) {
        lo = 0, hi = sc;
        while (lo < hi) {
          const int mid = (lo + hi) >> 1;
          if (seg_value(sp + mid, sp, sc, near, far, cn, cf) < va) lo = mid + 1; else hi = mid;
        }
        zr[a + lo] = va;
      } else {
        lo = 0, hi = sp;
        while (lo < hi) {
          const int mid = (lo + hi) >> 1;
          if (seg_value(mid, sp, sc, near, far, cn, cf) <= va) lo = mid + 1; else hi = mid;
        }
        zr[(a - sp) + lo] = va;
      }
    }
    return;
  }
  for (int a = lane; a < S; a += 64) {
    const float va = seg_value(a, sp, sc, near, far, cn, cf);
    int rank = 0;
    const bool na = !(va == va);
    for (int b = 0; b < S; ++b) {
      const float vb = seg_value(b, sp, sc, near, far, cn, cf);
      const bool nb = !(vb == vb);
      rank += (vb < va) || (na && !nb) || ((vb == va || (na && nb)) && b < a);   // NaNs after every number
    }
    zr[rank] = va;
  }
}

// render.py:449-454 (and :506-511): z' = lower + (upper - lower) * (perturb * rand)
__global__ void k_perturb(const float* __restrict__ z, int64_t total, int S, float perturb,
                          const float* __restrict__ rnd, float* __restrict__ zo) {
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= total) return;
  const int i = (int)(g % S);
  const float zi = z[g];
  const float lower = i == 0 ? zi : 0.5f * (z[g - 1] + zi);
  const float upper = i == S - 1 ? zi : 0.5f * (zi + z[g + 1]);
  const float pr = perturb * rnd[g];
  zo[g] = lower + (upper - lower) * pr;
}

// ------------------------------------------------------------------------------- compositing
// Exclusive multiplicative scan of one double per lane across the wave.
__device__ __forceinline__ double wave_excl_prod(double v, int lane) {
  double incl = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const double n = __shfl_up(incl, o, 64);
    if (lane >= o) incl *= n;
  }
  const double ex = __shfl_up(incl, 1, 64);
  return lane == 0 ? 1.0 : ex;
}
__device__ __forceinline__ double wave_excl_sum(double v, int lane) {
  double incl = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const double n = __shfl_up(incl, o, 64);
    if (lane >= o) incl += n;
  }
  const double ex = __shfl_up(incl, 1, 64);
  return lane == 0 ? 0.0 : ex;
}

// A ray's compositing group: one wave (G = 64, four rays per 256-thread workgroup: the many-ray batches) or one
// whole workgroup (G = 256: batches of a few hundred long rays, e.g. the reference shell's 256 rays x 2,304 fine
// samples, where a wave per ray kept 64 of 256 CUs busy and 36 samples per lane spilled).  Thread t of the group
// holds samples t B .. t B + B - 1; the group primitives below combine the per-thread values -- wave shuffles, and
// for G = 256 the four waves' partials through LDS (sh: 8 doubles).
template <int G>
struct Grp {
  static_assert(G == 64 || G == 256, "one wave or one 256-thread workgroup per ray");
  static constexpr int NW = G / 64;
  __device__ static int tid() { return G == 64 ? (int)(threadIdx.x & 63) : (int)threadIdx.x; }
  __device__ static int64_t ray() {
    return G == 64 ? (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6) : (int64_t)blockIdx.x;
  }
  __device__ static double sum(double v, double* sh) {
    v = wave_sum_d(v);
    if constexpr (G == 64) {
      return v;
    } else {
      if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
      __syncthreads();
      double t = 0.0;
#pragma unroll
      for (int i = 0; i < NW; ++i) t += sh[i];
      __syncthreads();
      return t;
    }
  }
  // exclusive product over the group's threads in order
  __device__ static double excl_prod(double v, double* sh) {
    const int lane = threadIdx.x & 63;
    const double ex = wave_excl_prod(v, lane);
    if constexpr (G == 64) {
      return ex;
    } else {
      const int w = threadIdx.x >> 6;
      const double tot = __shfl(ex * v, 63, 64);
      if (lane == 0) sh[w] = tot;
      __syncthreads();
      double base = 1.0;
      for (int i = 0; i < w; ++i) base *= sh[i];
      __syncthreads();
      return base * ex;
    }
  }
  __device__ static bool any(bool b) {
    if constexpr (G == 64) return __any(b);
    else return __syncthreads_or(b ? 1 : 0) != 0;
  }
  __device__ static float bcast(float v, int src, double* sh) {
    if constexpr (G == 64) {
      return __shfl(v, src, 64);
    } else {
      if ((int)threadIdx.x == src) sh[0] = (double)v;
      __syncthreads();
      const float r = (float)sh[0];
      __syncthreads();
      return r;
    }
  }
  // U entering each thread's block from above: the composition of threads t + 1 .. G - 1's affine maps
  // (Y = A + Bm Y_next) applied to 0
  __device__ static double suffix_affine(double A, double Bm, double* sh) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const double An = __shfl_down(A, o, 64), Bn = __shfl_down(Bm, o, 64);
      if (lane + o < 64) {
        A = A + Bm * An;
        Bm = Bm * Bn;
      }
    }
    double Y = 0.0;   // entering this wave's last lane
    if constexpr (G == 256) {
      const int w = threadIdx.x >> 6;
      if (lane == 0) {
        sh[w] = A;
        sh[4 + w] = Bm;
      }
      __syncthreads();
      for (int i = NW - 1; i > w; --i) Y = sh[i] + sh[4 + i] * Y;
      __syncthreads();
    }
    const double An1 = __shfl_down(A, 1, 64), Bn1 = __shfl_down(Bm, 1, 64);
    return lane == 63 ? Y : An1 + Bn1 * Y;
  }
};

// Smallest thr = thr0 + k*0.01 (Python float64 accumulation) for which a sample of the ray lies in
// [fl32(near - fl32(thr)), fl32(far + fl32(thr))] (inclusive: render.py:80-84,94-97) or the open interval
// (strict: render.py:255-263).  Returns fl32 bounds.
template <bool STRICT, int MAXB, int G = 64>
__device__ __forceinline__ void expand_bounds(const float (&zv)[MAXB], int nb, float near, float far, double thr0,
                                              float& lo, float& hi, int* err) {
  double thr = thr0;
  for (int it = 0; it < 4000000; ++it) {
    const float t32 = (float)thr;
    lo = near - t32;
    hi = far + t32;
    bool any = false;
#pragma unroll
    for (int j = 0; j < MAXB; ++j)
      if (j < nb) any |= STRICT ? (lo < zv[j] && zv[j] < hi) : (lo <= zv[j] && zv[j] <= hi);
    if (Grp<G>::any(any)) return;
    thr = thr + 0.01;
  }
  if (err) *err = 1;
}

// ATen's KeyValueCompDesc (sort descending): NaN first, then a > b
__device__ __forceinline__ bool kv_desc(float a, float b) { return (isnan(a) && !isnan(b)) || a > b; }

// torch CPU's argsort(descending=True) (render.py:598) runs libstdc++'s std::sort -- introsort: median-of-three
// quicksort with unguarded Hoare partitions down to ranges of 16, heapsort past 2 lg n levels, then one insertion
// sort -- over (value, index) pairs with KeyValueCompDesc; the order it leaves equal keys in is this algorithm's, so
// it is restated step by step (checked against torch's argsort on tie-heavy rows, tests/test_parity_gpu.py).
// V / I: the row's values and indices (LDS), n entries; one thread.
__device__ void introsort_desc(float* V, int* I, int n) {
  auto swp = [&](int a, int b) {
    const float tv = V[a];
    V[a] = V[b];
    V[b] = tv;
    const int ti = I[a];
    I[a] = I[b];
    I[b] = ti;
  };
  auto push_heap = [&](int first, int hole, int top, float vv, int vi) {
    int parent = (hole - 1) / 2;
    while (hole > top && kv_desc(V[first + parent], vv)) {
      V[first + hole] = V[first + parent];
      I[first + hole] = I[first + parent];
      hole = parent;
      parent = (hole - 1) / 2;
    }
    V[first + hole] = vv;
    I[first + hole] = vi;
  };
  auto adjust_heap = [&](int first, int hole, int len, float vv, int vi) {
    const int top = hole;
    int second = hole;
    while (second < (len - 1) / 2) {
      second = 2 * (second + 1);
      if (kv_desc(V[first + second], V[first + second - 1])) --second;
      V[first + hole] = V[first + second];
      I[first + hole] = I[first + second];
      hole = second;
    }
    if ((len & 1) == 0 && second == (len - 2) / 2) {
      second = 2 * (second + 1);
      V[first + hole] = V[first + second - 1];
      I[first + hole] = I[first + second - 1];
      hole = second - 1;
    }
    push_heap(first, hole, top, vv, vi);
  };
  auto heap_sort = [&](int first, int last) {   // __partial_sort(first, last, last): make_heap + sort_heap
    const int len = last - first;
    if (len >= 2) {
      for (int parent = (len - 2) / 2;; --parent) {
        adjust_heap(first, parent, len, V[first + parent], I[first + parent]);
        if (parent == 0) break;
      }
    }
    while (last - first > 1) {
      --last;
      const float vv = V[last];
      const int vi = I[last];
      V[last] = V[first];
      I[last] = I[first];
      adjust_heap(first, 0, last - first, vv, vi);
    }
  };
  auto median_to_first = [&](int res, int a, int b, int c) {
    if (kv_desc(V[a], V[b])) {
      if (kv_desc(V[b], V[c])) swp(res, b);
      else if (kv_desc(V[a], V[c])) swp(res, c);
      else swp(res, a);
    } else if (kv_desc(V[a], V[c])) swp(res, a);
    else if (kv_desc(V[b], V[c])) swp(res, c);
    else swp(res, b);
  };
  auto linear_insert = [&](int last) {   // __unguarded_linear_insert
    const float vv = V[last];
    const int vi = I[last];
    int next = last - 1;
    while (kv_desc(vv, V[next])) {
      V[last] = V[next];
      I[last] = I[next];
      last = next;
      --next;
    }
    V[last] = vv;
    I[last] = vi;
  };
  auto insertion_sort = [&](int first, int last) {
    for (int i = first + 1; i < last; ++i) {
      if (kv_desc(V[i], V[first])) {
        const float vv = V[i];
        const int vi = I[i];
        for (int k = i; k > first; --k) {
          V[k] = V[k - 1];
          I[k] = I[k - 1];
        }
        V[first] = vv;
        I[first] = vi;
      } else {
        linear_insert(i);
      }
    }
  };
  if (n < 2) return;
  // __introsort_loop with its recursion on [cut, last) as an explicit stack (the ranges are disjoint, so the
  // order they are processed in does not change the result)
  int sf[64], sl[64], sd[64], sp = 1;
  sf[0] = 0;
  sl[0] = n;
  sd[0] = 2 * (31 - __clz(n));
  while (sp > 0) {
    --sp;
    int first = sf[sp], last = sl[sp], depth = sd[sp];
    while (last - first > 16) {
      if (depth == 0) {
        heap_sort(first, last);
        break;
      }
      --depth;
      median_to_first(first, first + 1, first + (last - first) / 2, last - 1);
      int lo = first + 1, hi = last;   // __unguarded_partition(first + 1, last, pivot = first)
      while (true) {
        while (kv_desc(V[lo], V[first])) ++lo;
        --hi;
        while (kv_desc(V[first], V[hi])) --hi;
        if (!(lo < hi)) break;
        swp(lo, hi);
        ++lo;
      }
      if (sp < 64) {
        sf[sp] = lo;
        sl[sp] = last;
        sd[sp] = depth;
        ++sp;
      }
      last = lo;
    }
  }
  if (n > 16) {   // __final_insertion_sort
    insertion_sort(0, 16);
    for (int i = 16; i < n; ++i) linear_insert(i);
  } else {
    insertion_sort(0, n);
  }
}

// render.py:598-600 on the rows where w[S-1] ties with another weight: one wave per row (the others exit at once),
// the row staged in LDS, lane 0 sorts it as torch does and takes the position of index S-1.
__global__ __launch_bounds__(256) void k_depth2_ties(const float* __restrict__ W, const float* __restrict__ Z,
                                                     int64_t n_rays, int S, float* __restrict__ depth2) {
  extern __shared__ float sm_row[];
  const int wq = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t ray = (int64_t)blockIdx.x * 4 + wq;
  if (ray >= n_rays) return;
  float* V = sm_row + (size_t)wq * S;
  int* I = reinterpret_cast<int*>(sm_row + (size_t)4 * S) + (size_t)wq * S;
  const float* wr = W + ray * S;
  const float wl = wr[S - 1];
  bool tie = false;
  for (int j = lane; j < S; j += 64) {
    const float x = wr[j];
    V[j] = x;
    I[j] = j;
    if (j < S - 1) tie = tie || !(kv_desc(x, wl) || kv_desc(wl, x));
  }
  if (__ballot(tie) == 0) return;   // (wave-uniform)
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  if (lane == 0) {
    introsort_desc(V, I, S);
    int pos = 0;
    while (I[pos] != S - 1) ++pos;
    depth2[ray] = Z[ray * S + pos];
  }
}

template <int MAXB, int G>
__global__ __launch_bounds__(256) void k_composite(const float* __restrict__ P, const float* __restrict__ Z,
                                                   int64_t n_rays, int S, const float* __restrict__ noise,
                                                   float noise_std, float eps, const float* __restrict__ rays,
                                                   int stride, int cn_col, int cf_col, int rg_col,
                                                   float* __restrict__ Wout, float* __restrict__ depth,
                                                   float* __restrict__ free_ray, float* __restrict__ sl1_ray,
                                                   double* __restrict__ opac_row, float* __restrict__ depth2,
                                                   int* __restrict__ err) {
  using Gp = Grp<G>;
  __shared__ double gsh[8];
  const int lane = Gp::tid();
  const int64_t ray = Gp::ray();
  if (ray >= n_rays) return;   // (G = 256: one workgroup per ray, never taken)
  const int B = (S + G - 1) / G;
  const int i0 = lane * B;
  const int nb = max(0, min(B, S - i0));
  const float* pr = P + ray * S + i0;
  const float* zr = Z + ray * S + i0;
  float pv[MAXB], zv[MAXB], wv[MAXB];
  double loc = 1.0;
#pragma unroll
  for (int j = 0; j < MAXB; ++j) {
    if (j < nb) {
      pv[j] = pr[j];
      zv[j] = zr[j];
      loc *= (double)(1.0f - pv[j]);
    } else {
      pv[j] = 0.0f;
      zv[j] = 0.0f;
    }
  }
  // transmittance: cumprod of [1, 1-p] in float64, each prefix rounded to fp32 (render.py:52-55)
  double T = Gp::excl_prod(loc, gsh);
  double sw = 0.0;
#pragma unroll
  for (int j = 0; j < MAXB; ++j) {
    if (j < nb) {
      float w = (float)T * pv[j];
      if (noise) w = w + noise[ray * S + i0 + j] * noise_std;
      wv[j] = w;
      sw += (double)w;
      T *= (double)(1.0f - pv[j]);
    } else {
      wv[j] = 0.0f;
    }
  }
  const float den = (float)Gp::sum(sw, gsh) + eps;  // render.py:60
  double sd = 0.0;
#pragma unroll
  for (int j = 0; j < MAXB; ++j) {
    if (j < nb) {
      wv[j] = wv[j] / den;
      sd += (double)(wv[j] * zv[j]);
    }
  }
  const float d = (float)Gp::sum(sd, gsh);
  if (Wout) {
    float* wr = Wout + ray * S + i0;
#pragma unroll
    for (int j = 0; j < MAXB; ++j)
      if (j < nb) wr[j] = wv[j];
  }
  if (lane == 0) depth[ray] = d;
  if (opac_row) {  // render.py:224: log(0.1 + p) + log(0.1 + (1 - p)) + 2.20727, summed per ray
    double op = 0.0;
#pragma unroll
    for (int j = 0; j < MAXB; ++j)
      if (j < nb) op += (double)((logf(0.1f + pv[j]) + logf(0.1f + (1.0f - pv[j]))) + 2.20727f);
    op = Gp::sum(op, gsh);
    if (lane == 0) opac_row[ray] = op;
  }
  if (depth2) {  // render.py:598-600: z at the position of sample S-1 in argsort(w, descending=True)
    // the count of weights a stable descending sort orders before it: every greater weight, and every equal one
    // (all have smaller indices) -- torch's sort on the GPU, where the reference runs this (the rows it sorts are
    // > 32 long: merge / radix sort, stable).  Under pcnerf_set_depth2_order(1) rows with a tie are redone by
    // k_depth2_ties (torch CPU's std::sort order of equal keys)
    const int last_lane = (S - 1) / B, last_j = (S - 1) % B;
    float wl = 0.0f;
#pragma unroll
    for (int j = 0; j < MAXB; ++j)
      if (j == last_j) wl = wv[j];
    wl = Gp::bcast(wl, last_lane, gsh);
    int cnt = 0;
#pragma unroll
    for (int j = 0; j < MAXB; ++j)
      if (j < nb && i0 + j < S - 1) cnt += kv_desc(wv[j], wl) || !kv_desc(wl, wv[j]);
    cnt = (int)Gp::sum((double)cnt, gsh);
    if (lane == 0) depth2[ray] = Z[ray * S + cnt];
  }
  if (!rays) return;

  // child masks and loss terms (render.py:75-159)
  const float* r = rays + ray * stride;
  const float cn = r[cn_col], cf = r[cf_col], rg = r[rg_col];
  float lo0, hi0, lo2, hi2;
  expand_bounds<false, MAXB, G>(zv, nb, cn, cf, 0.0, lo0, hi0, err);
  expand_bounds<false, MAXB, G>(zv, nb, cn, cf, 2.0, lo2, hi2, err);
  double fr = 0.0, sc = 0.0;
#pragma unroll
  for (int j = 0; j < MAXB; ++j) {
    if (j < nb) {
      const bool m0 = lo0 <= zv[j] && zv[j] <= hi0;
      const float wf = wv[j] * (m0 ? 0.0f : 1.0f);
      fr += (double)(wf * wf);
      const bool m2 = lo2 <= zv[j] && zv[j] <= hi2;
      sc += (double)(wv[j] * (m2 ? 1.0f : 0.0f));
    }
  }
  const float denc = (float)Gp::sum(sc, gsh) + eps;  // render.py:129
  double dcs = 0.0;
#pragma unroll
  for (int j = 0; j < MAXB; ++j) {
    if (j < nb) {
      const float m2 = (lo2 <= zv[j] && zv[j] <= hi2) ? 1.0f : 0.0f;
      const float wc = (wv[j] * m2) / denc;
      dcs += (double)(wc * (zv[j] * m2));
    }
  }
  const float dc = (float)Gp::sum(dcs, gsh);
  const float frs = (float)Gp::sum(fr, gsh);
  if (lane == 0) {
    free_ray[ray] = frs;
    sl1_ray[ray] = smooth_l1(10.0f * dc, 10.0f * rg);
  }
}

// ------------------------------------------------------------------------------- importance resampling
// sample_pdf (render.py:371-412) for one ray by one wave: bins[0..nb), weights w[0..nb-1) (already sliced),
// cdf scratch of nb floats in LDS, n draws -> out[k] (unsorted).  Sums run in float64: every pdf value is
// >= 1e-5/sum, so all partial sums are exact in float64 and the cdf equals the reference's cumsum (which
// accumulates in float64 on CPU) bit for bit; the normaliser is the float64 sum rounded once.
__device__ void pdf_samples(const float* bins, const float* w, int nb, float* cdf, int n, const float* u_row,
                            float* out, int lane) {
  const int npdf = nb - 1;
  const int B = (npdf + 63) / 64;
  const int i0 = lane * B;
  double ls = 0.0;
  for (int j = 0; j < B; ++j) {
    const int i = i0 + j;
    if (i < npdf) ls += (double)(w[i] + 1e-5f);
  }
  const float tot = (float)wave_sum_d(ls);
  double lp = 0.0;
  for (int j = 0; j < B; ++j) {
    const int i = i0 + j;
    if (i < npdf) lp += (double)((w[i] + 1e-5f) / tot);
  }
  double run = wave_excl_sum(lp, lane);
  if (lane == 0) cdf[0] = 0.0f;
  for (int j = 0; j < B; ++j) {
    const int i = i0 + j;
    if (i < npdf) {
      run += (double)((w[i] + 1e-5f) / tot);
      cdf[i + 1] = (float)run;
    }
  }
  __syncthreads();
  for (int k = lane; k < n; k += 64) {
    const float u = u_row ? u_row[k] : linspace01(k, n);
    int lo = 0, hi = nb;  // first index with cdf > u  (searchsorted right=True)
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (cdf[mid] <= u) lo = mid + 1; else hi = mid;
    }
    const int below = max(lo - 1, 0), above = min(lo, nb - 1);
    const float c0 = cdf[below], c1 = cdf[above];
    float denom = c1 - c0;
    if (denom < 1e-5f) denom = 1.0f;
    const float t = (u - c0) / denom;
    const float b0 = bins[below], b1 = bins[above];
    out[k] = b0 + t * (b1 - b0);
  }
}

// standalone sample_pdf(bins (R,nb), weights (R,nb-1)) -> (R,n), one wave per ray; LDS: bins | w | cdf
__global__ __launch_bounds__(256) void k_sample_pdf(const float* __restrict__ bins_g, const float* __restrict__ w_g,
                                                    int64_t n_rays, int nb, int n, const float* __restrict__ U,
                                                    float* __restrict__ out) {
  extern __shared__ float lds[];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const int64_t ray0 = (int64_t)blockIdx.x * nw + wid;
  const bool active = ray0 < n_rays;
  const int64_t ray = active ? ray0 : n_rays - 1;
  float* bins = lds + (size_t)wid * 3 * nb;
  float* w = bins + nb;
  float* cdf = w + nb;
  for (int i = lane; i < nb; i += 64) bins[i] = bins_g[ray * nb + i];
  for (int i = lane; i < nb - 1; i += 64) w[i] = w_g[ray * (nb - 1) + i];
  __syncthreads();
  if (active) {
    pdf_samples(bins, w, nb, cdf, n, U ? U + ray * n : nullptr, out + ray * n, lane);
  } else {
    pdf_samples(bins, w, nb, cdf, 0, nullptr, nullptr, lane);
  }
}

// float64 block sum / exclusive scan over NT threads (NT / 64 waves; sh holds NT / 64 doubles).  The pdf sums
// they serve are exact in float64 (see pdf_samples), so the grouping does not change a bit of the result.
template <int NT>
__device__ __forceinline__ double blk_sum_d(double v, double* sh) {
  v = wave_sum_d(v);
  if constexpr (NT == 64) {
    return v;
  } else {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if (lane == 0) sh[wid] = v;
    __syncthreads();
    double t = 0.0;
    for (int i = 0; i < NT / 64; ++i) t += sh[i];
    __syncthreads();
    return t;
  }
}
template <int NT>
__device__ __forceinline__ double blk_excl_d(double v, double* sh) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const double ex = wave_excl_sum(v, lane);
  if constexpr (NT == 64) {
    return ex;
  } else {
    const double wt = __shfl(ex + v, 63, 64);
    if (lane == 0) sh[wid] = wt;
    __syncthreads();
    double base = 0.0;
    for (int i = 0; i < wid; ++i) base += sh[i];
    __syncthreads();
    return base + ex;
  }
}

// ascending bitonic sort of a[0..n) in LDS (n a power of two) by NT threads, comparator c of each stage on the
// pair (i, i | j) with i = c with a zero bit inserted at j; NaN sorts after every number (torch.sort's order)
template <int NT>
__device__ void blk_bitonic(float* a, int n) {
  for (int k = 2; k <= n; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int c = threadIdx.x; c < (n >> 1); c += NT) {
        const int i = ((c & ~(j - 1)) << 1) | (c & (j - 1)), ixj = i | j;
        const float x = a[i], y = a[ixj];
        const bool up = (i & k) == 0;
        const bool gt = (x == x) ? (x > y) : (y == y);
        if (gt == up) {
          a[i] = y;
          a[ixj] = x;
        }
      }
      __syncthreads();
    }
  }
}

// render.py:371-412 + :463-467, one ray per workgroup of NT threads.  LDS: z (S) | fine (PF = pow2 >= I) | w (S) |
// bins (S) | cdf (S), the full-sort buffer (P2 = pow2 >= S + I) aliasing w / bins / cdf, which are dead once the
// fine values are drawn: (S + PF + max(3S, P2)) floats, 112 KiB at the reference eval shells' 4096 + 8192.  sample_pdf's draws are unsorted whenever the uniforms
// are (perturb: torch.rand), so the fine list is bitonic-sorted on its own and merged with the coarse z (sorted by
// construction, render.py:433-442) by binary search: a coarse value lands at its index plus the fine values
// strictly below it, a fine value at its index plus the coarse values <= it.  A coarse list out of order or a NaN
// anywhere sends the ray through the bitonic sort of the whole concatenation instead; the sorted values are the
// same either way.
template <int NT>
__global__ __launch_bounds__(NT) void k_resample(const float* __restrict__ Z, const float* __restrict__ Wt, int S,
                                                 int I, int PF, int P2, const float* __restrict__ U,
                                                 float* __restrict__ ZF) {
  extern __shared__ float lds[];
  __shared__ double sh[NT / 64];
  const int tid = threadIdx.x;
  const int64_t ray = blockIdx.x;
  float* zs = lds;
  float* fs = zs + S;
  float* ws = fs + PF;
  float* bins = ws + S;
  float* cdf = bins + S;
  float* sb = ws;   // (after the draws: the barrier below orders the last cdf / bins read before its first write)
  for (int i = tid; i < S; i += NT) {
    zs[i] = Z[ray * S + i];
    ws[i] = Wt[ray * S + i];
  }
  __syncthreads();
  const int nb = S - 1, npdf = nb - 1;   // bins = mid-points, weights w[1:-1] (render.py:456-458)
  for (int i = tid; i < nb; i += NT) bins[i] = 0.5f * (zs[i + 1] + zs[i]);
  const float* w = ws + 1;
  const int B = (npdf + NT - 1) / NT, i0 = tid * B;
  double ls = 0.0;
  for (int j = 0; j < B; ++j) {
    const int i = i0 + j;
    if (i < npdf) ls += (double)(w[i] + 1e-5f);
  }
  const float tot = (float)blk_sum_d<NT>(ls, sh);
  double lp = 0.0;
  for (int j = 0; j < B; ++j) {
    const int i = i0 + j;
    if (i < npdf) lp += (double)((w[i] + 1e-5f) / tot);
  }
  double run = blk_excl_d<NT>(lp, sh);
  if (tid == 0) cdf[0] = 0.0f;
  for (int j = 0; j < B; ++j) {
    const int i = i0 + j;
    if (i < npdf) {
      run += (double)((w[i] + 1e-5f) / tot);
      cdf[i + 1] = (float)run;
    }
  }
  __syncthreads();
  const float* u_row = U ? U + ray * I : nullptr;
  for (int k = tid; k < I; k += NT) {
    const float u = u_row ? u_row[k] : linspace01(k, I);
    int lo = 0, hi = nb;   // first index with cdf > u  (searchsorted right=True)
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (cdf[mid] <= u) lo = mid + 1; else hi = mid;
    }
    const int below = max(lo - 1, 0), above = min(lo, nb - 1);
    const float c0 = cdf[below], c1 = cdf[above];
    float denom = c1 - c0;
    if (denom < 1e-5f) denom = 1.0f;
    const float t = (u - c0) / denom;
    const float b0 = bins[below], b1 = bins[above];
    fs[k] = b0 + t * (b1 - b0);
  }
  for (int k = I + tid; k < PF; k += NT) fs[k] = __builtin_nanf("");
  bool ok = true;
  for (int i = tid; i < S; i += NT) ok = ok && (zs[i] == zs[i]) && (i + 1 >= S || zs[i] <= zs[i + 1]);
  __syncthreads();
  for (int i = tid; i < I; i += NT) ok = ok && (fs[i] == fs[i]);
  float* out = ZF + ray * (S + I);
  if (__syncthreads_or(ok ? 0 : 1)) {
    for (int i = tid; i < S; i += NT) sb[i] = zs[i];
    for (int i = tid; i < I; i += NT) sb[S + i] = fs[i];
    for (int i = S + I + tid; i < P2; i += NT) sb[i] = __builtin_nanf("");
    __syncthreads();
    blk_bitonic<NT>(sb, P2);
    for (int i = tid; i < S + I; i += NT) out[i] = sb[i];
    return;
  }
  blk_bitonic<NT>(fs, PF);
  for (int i = tid; i < S; i += NT) {
    const float v = zs[i];
    int lo = 0, hi = I;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (fs[mid] < v) lo = mid + 1; else hi = mid;
    }
    out[i + lo] = v;
  }
  for (int i = tid; i < I; i += NT) {
    const float v = fs[i];
    int lo = 0, hi = S;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (zs[mid] <= v) lo = mid + 1; else hi = mid;
    }
    out[i + lo] = v;
  }
}

// ------------------------------------------------------------------------------- loss reductions
__device__ __forceinline__ double block_sum_d(double v, double* sh) {
  v = wave_sum_d(v);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) sh[wid] = v;
  __syncthreads();
  double t = 0.0;
  if (threadIdx.x == 0) {
    for (int i = 0; i < (int)(blockDim.x >> 6); ++i) t += sh[i];
    sh[0] = t;
  }
  __syncthreads();
  t = sh[0];
  __syncthreads();
  return t;
}

// plain branch: free = fl32(sum) / R (render.py:121); depth = fl32((1/R)*0.1) * mean(SmoothL1) (render.py:155)
__global__ void k_child_loss_plain(const float* __restrict__ fr, const float* __restrict__ sl, int64_t n,
                                   float* __restrict__ out) {
  __shared__ double sh[16];
  double a = 0.0, b = 0.0;
  for (int64_t i = threadIdx.x; i < n; i += blockDim.x) {
    a += (double)fr[i];
    b += (double)sl[i];
  }
  a = block_sum_d(a, sh);
  b = block_sum_d(b, sh);
  if (threadIdx.x == 0) {
    const float nf = (float)n;
    out[0] = (float)a / nf;
    const float mean = (float)b / nf;
    out[1] = (float)((1.0 / (double)n) * 0.1) * mean;
  }
}

// divide branch: per child id c in 1..N (render.py:111-119, :140-152)
__global__ void k_child_loss_scatter(const float* __restrict__ fr, const float* __restrict__ sl, int64_t n,
                                     const float* __restrict__ cid, int stride, int N, double* __restrict__ acc) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float c = cid[i * stride];
  const int k = (int)floorf(c - 0.5f);  // candidate child slot: c in (k+0.5, k+1.5)
  if (k < 0 || k >= N) return;
  if (!(c > (float)k + 0.5f && c < (float)k + 1.5f)) return;
  atomicAdd(acc + 3 * k + 0, (double)fr[i]);
  atomicAdd(acc + 3 * k + 1, (double)sl[i]);
  atomicAdd(acc + 3 * k + 2, 1.0);
}

__global__ void k_child_loss_divide(const double* __restrict__ acc, int N, float* __restrict__ out) {
  __shared__ double sh[16];
  double a = 0.0, b = 0.0;
  for (int k = threadIdx.x; k < N; k += blockDim.x) {
    const double cnt = acc[3 * k + 2];
    if (cnt >= 1.0) {
      const float c32 = (float)cnt;
      a += (double)((float)acc[3 * k + 0] / c32);
      const float inv = 1.0f / c32;
      b += (double)((inv * 0.1f) * ((float)acc[3 * k + 1] / c32));
    }
  }
  a = block_sum_d(a, sh);
  b = block_sum_d(b, sh);
  if (threadIdx.x == 0) {
    out[0] = (float)a;
    out[1] = (float)b;
  }
}

// Per-child range loss (train_kitti.py:125-142, use_child_nerf_divide == 1): for each child id c in 1..N,
// post * mean_c loss(pre*pred, pre*target); the reference sums these over the children that own >= 1 ray.
// Scatter: per-child float64 sums of the element losses and counts (child slot as in k_child_loss_scatter).
__device__ __forceinline__ int child_slot(const float* cid, int64_t i, int stride, int N) {
  const float c = cid[i * stride];
  const int k = (int)floorf(c - 0.5f);
  if (k < 0 || k >= N) return -1;
  return (c > (float)k + 0.5f && c < (float)k + 1.5f) ? k : -1;
}

__global__ void k_child_range_scatter(const float* __restrict__ a, const float* __restrict__ b, int64_t n,
                                      const float* __restrict__ cid, int stride, int N, int kind, float pre,
                                      double* __restrict__ acc) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int k = child_slot(cid, i, stride, N);
  if (k < 0) return;
  const float x = pre * a[i], y = pre * b[i];
  const float d = x - y;
  const float v = kind == 0 ? d * d : kind == 1 ? fabsf(d) : smooth_l1(x, y);
  atomicAdd(acc + 2 * k + 0, (double)v);
  atomicAdd(acc + 2 * k + 1, 1.0);
}

__global__ void k_child_range_reduce(const double* __restrict__ acc, int N, float post, float* __restrict__ out) {
  __shared__ double sh[16];
  double a = 0.0;
  for (int k = threadIdx.x; k < N; k += blockDim.x) {
    const double cnt = acc[2 * k + 1];
    if (cnt >= 1.0) a += (double)(post * ((float)acc[2 * k + 0] / (float)cnt));
  }
  a = block_sum_d(a, sh);
  if (threadIdx.x == 0) out[0] = (float)a;
}

// d/dpred_i = gout * post * pre * loss'(pre*pred - pre*target) / count_c(i); 0 for rays of no child slot.
__global__ void k_child_range_bwd(const float* __restrict__ a, const float* __restrict__ b, int64_t n,
                                  const float* __restrict__ cid, int stride, int N, int kind, float pre, float post,
                                  const double* __restrict__ acc, const float* __restrict__ gout,
                                  float* __restrict__ ga) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int k = child_slot(cid, i, stride, N);
  if (k < 0) {
    ga[i] = 0.0f;
    return;
  }
  const float d = pre * a[i] - pre * b[i];
  const float sg = d > 0.0f ? 1.0f : (d < 0.0f ? -1.0f : 0.0f);
  const float g = kind == 0 ? 2.0f * d : kind == 1 ? sg : (fabsf(d) < 1.0f ? d : sg);
  ga[i] = ((gout[0] * post) / (float)acc[2 * k + 1]) * g * pre;
}

__global__ void k_sum_f64(const double* __restrict__ x, int64_t n, double denom, float* __restrict__ out) {
  __shared__ double sh[16];
  double a = 0.0;
  for (int64_t i = threadIdx.x; i < n; i += blockDim.x) a += x[i];
  a = block_sum_d(a, sh);
  if (threadIdx.x == 0) out[0] = (float)(a / denom);
}

__global__ void k_pointwise_loss(const float* __restrict__ a, const float* __restrict__ b,
                                 const uint8_t* __restrict__ m, int64_t n, int kind, float* __restrict__ out) {
  __shared__ double sh[16];
  double s = 0.0, c = 0.0;
  for (int64_t i = threadIdx.x; i < n; i += blockDim.x) {
    if (m && !m[i]) continue;
    const float d = a[i] - b[i];
    float v;
    if (kind == 0) v = d * d;
    else if (kind == 1) v = fabsf(d);
    else v = smooth_l1(a[i], b[i]);
    s += (double)v;
    c += 1.0;
  }
  s = block_sum_d(s, sh);
  c = block_sum_d(c, sh);
  if (threadIdx.x == 0) out[0] = (float)s / (float)c;  // mean of an empty selection is nan, like torch
}

// d mean(loss(pred, target)) / d pred, scaled by the upstream scalar gradient; zero outside the mask
// (torch's backward of index-select + mean: grad / count at the selected elements).
__global__ void k_pointwise_loss_bwd(const float* __restrict__ a, const float* __restrict__ b,
                                     const uint8_t* __restrict__ m, int64_t n, int kind,
                                     const float* __restrict__ gout, float* __restrict__ ga) {
  __shared__ double sh[16];
  double c = 0.0;
  if (m) {
    for (int64_t i = threadIdx.x; i < n; i += blockDim.x) c += m[i] ? 1.0 : 0.0;
    c = block_sum_d(c, sh);
  } else {
    c = (double)n;
  }
  const float scale = gout[0] / (float)c;
  for (int64_t i = threadIdx.x; i < n; i += blockDim.x) {
    if (m && !m[i]) {
      ga[i] = 0.0f;
      continue;
    }
    const float d = a[i] - b[i];
    const float sg = d > 0.0f ? 1.0f : (d < 0.0f ? -1.0f : 0.0f);
    const float g = kind == 0 ? 2.0f * d : kind == 1 ? sg : (fabsf(d) < 1.0f ? d : sg);
    ga[i] = g * scale;
  }
}


// ------------------------------------------------------------------------------- compositing backward
// Gradient of the compositing + child-loss terms (render.py:51-61, 75-159) with respect to the occupancy
// logits, from the upstream gradients autograd hands the render step: dL/ddepth per ray and dL/d(free loss),
// dL/d(child depth loss) as scalars.  One wave per ray, the forward values recomputed exactly as k_composite
// does.  All backward arithmetic runs in float64 and rounds once, so the result is the exact derivative of the
// fp32 forward up to that final rounding (torch's autograd rounds each backward op in fp32).
//   w~_j = T_j p_j (+ noise),  W = sum w~ + eps,  w_j = w~_j / W,  depth = sum w_j z_j
//   dL/dw~_j = (dL/dw_j - sum_k dL/dw_k w_k) / W
//   dL/dp_j  = T_j (dL/dw~_j - U_j),  U_j = sum_{k>j} dL/dw~_k p_k prod_{j<i<k}(1-p_i)
// U is the reverse affine recurrence U_{j-1} = g~_j p_j + (1-p_j) U_j (no division by 1-p, exact when
// p saturates at 1): each lane composes the map over its block, a wave suffix scan composes the lanes.
// Child terms: free = sum (w*!M0)^2 / R (or per child / count), depth loss c * mean SL1(10 dc, 10 range),
// dc = sum_j w_j M2_j z_j / (sum w M2 + eps).
template <int MAXB, int G>
__global__ __launch_bounds__(256) void k_composite_bwd(
    const float* __restrict__ P, const float* __restrict__ Z, int64_t n_rays, int S, const float* __restrict__ noise,
    float noise_std, float eps, const float* __restrict__ rays, int stride, int cn_col, int cf_col, int rg_col,
    int cid_col, int n_child, const double* __restrict__ counts, const float* __restrict__ g_depth,
    const float* __restrict__ g_free, const float* __restrict__ g_dl, float* __restrict__ g_logit,
    int* __restrict__ err) {
  using Gp = Grp<G>;
  __shared__ double gsh[8];
  const int lane = Gp::tid();
  const int64_t ray = Gp::ray();
  if (ray >= n_rays) return;   // (G = 256: one workgroup per ray, never taken)
  const int B = (S + G - 1) / G;
  const int i0 = lane * B;
  const int nb = max(0, min(B, S - i0));
  const float* pr = P + ray * S + i0;
  const float* zr = Z + ray * S + i0;
  float pv[MAXB], zv[MAXB], wv[MAXB], tv[MAXB];
  double loc = 1.0;
#pragma unroll
  for (int j = 0; j < MAXB; ++j) {
    if (j < nb) {
      pv[j] = pr[j];
      zv[j] = zr[j];
      loc *= (double)(1.0f - pv[j]);
    } else {
      pv[j] = 0.0f;
      zv[j] = 0.0f;
    }
  }
  double T = Gp::excl_prod(loc, gsh);
  double sw = 0.0;
#pragma unroll
  for (int j = 0; j < MAXB; ++j) {
    tv[j] = 0.0f;
    wv[j] = 0.0f;
    if (j < nb) {
      tv[j] = (float)T;
      float w = tv[j] * pv[j];
      if (noise) w = w + noise[ray * S + i0 + j] * noise_std;
      wv[j] = w;
      sw += (double)w;
      T *= (double)(1.0f - pv[j]);
    }
  }
  const float den = (float)Gp::sum(sw, gsh) + eps;
#pragma unroll
  for (int j = 0; j < MAXB; ++j)
    if (j < nb) wv[j] = wv[j] / den;

  // dL/dw_j
  const double gd = g_depth ? (double)g_depth[ray] : 0.0;
  double gw[MAXB];
#pragma unroll
  for (int j = 0; j < MAXB; ++j) gw[j] = gd * (double)zv[j];
  if (rays) {
    const float* r = rays + ray * stride;
    const float cn = r[cn_col], cf = r[cf_col], rg = r[rg_col];
    double kf = 0.0, kd = 0.0;  // d loss / d (w_j^2 summand) and d loss / d dc
    const double gf = g_free ? (double)g_free[0] : 0.0, gl = g_dl ? (double)g_dl[0] : 0.0;
    if (n_child <= 0) {
      kf = gf / (double)(float)n_rays;
      kd = gl * (double)(float)((1.0 / (double)n_rays) * 0.1) / (double)(float)n_rays * 10.0;
    } else {
      const float c = r[cid_col];
      const int k = (int)floorf(c - 0.5f);
      if (k >= 0 && k < n_child && c > (float)k + 0.5f && c < (float)k + 1.5f && counts[k] >= 1.0) {
        const float c32 = (float)counts[k];
        kf = gf / (double)c32;
        kd = gl * (double)((1.0f / c32) * 0.1f) / (double)c32 * 10.0;
      }
    }
    float lo0, hi0, lo2, hi2;
    expand_bounds<false, MAXB, G>(zv, nb, cn, cf, 0.0, lo0, hi0, err);
    expand_bounds<false, MAXB, G>(zv, nb, cn, cf, 2.0, lo2, hi2, err);
    double sc = 0.0;
#pragma unroll
    for (int j = 0; j < MAXB; ++j) {
      if (j < nb) {
        const bool m2 = lo2 <= zv[j] && zv[j] <= hi2;
        sc += (double)(wv[j] * (m2 ? 1.0f : 0.0f));
      }
    }
    const float denc = (float)Gp::sum(sc, gsh) + eps;
    double dcs = 0.0;
#pragma unroll
    for (int j = 0; j < MAXB; ++j) {
      if (j < nb) {
        const float m2 = (lo2 <= zv[j] && zv[j] <= hi2) ? 1.0f : 0.0f;
        const float wc = (wv[j] * m2) / denc;
        dcs += (double)(wc * (zv[j] * m2));
      }
    }
    const float dc = (float)Gp::sum(dcs, gsh);
    const float x = 10.0f * dc - 10.0f * rg;
    const double sl1g = fabsf(x) < 1.0f ? (double)x : (x > 0.0f ? 1.0 : -1.0);  // SmoothL1 (beta 1) derivative
    const double gdc = kd * sl1g;
#pragma unroll
    for (int j = 0; j < MAXB; ++j) {
      if (j < nb) {
        const bool m0 = lo0 <= zv[j] && zv[j] <= hi0;
        const bool m2 = lo2 <= zv[j] && zv[j] <= hi2;
        if (!m0) gw[j] += 2.0 * kf * (double)wv[j];
        if (m2) gw[j] += gdc * ((double)zv[j] - (double)dc) / (double)denc;
      }
    }
  }
  // normalisation backward
  double dot = 0.0;
#pragma unroll
  for (int j = 0; j < MAXB; ++j)
    if (j < nb) dot += gw[j] * (double)wv[j];
  dot = Gp::sum(dot, gsh);
  const double rden = 1.0 / (double)den;
#pragma unroll
  for (int j = 0; j < MAXB; ++j) gw[j] = (gw[j] - dot) * rden;  // now dL/dw~
  // this lane's affine map U_{end} -> U_{i0 - 1}: U_{j-1} = a_j + b_j U_j
  double A = 0.0, Bm = 1.0;
#pragma unroll
  for (int j = MAXB - 1; j >= 0; --j) {
    if (j < nb) {
      const double a = gw[j] * (double)pv[j], b = (double)(1.0f - pv[j]);
      A = a + b * A;
      Bm = b * Bm;
    }
  }
  // suffix composition over the group's threads: Y_t = A_t + B_t Y_{t+1}
  double U = Gp::suffix_affine(A, Bm, gsh);
  float* go = g_logit + ray * S + i0;
#pragma unroll
  for (int j = MAXB - 1; j >= 0; --j) {
    if (j < nb) {
      const double gp = (double)tv[j] * (gw[j] - U);
      U = gw[j] * (double)pv[j] + (double)(1.0f - pv[j]) * U;
      go[j] = (float)(gp * (double)(1.0f - pv[j]) * (double)pv[j]);  // sigmoid backward
    }
  }
}

// rays per child id c in 1..N (the divide branch's sub_nerf_tmp.sum(), render.py:111-119)
__global__ void k_child_counts(const float* __restrict__ cid, int stride, int64_t n, int N, double* __restrict__ acc) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float c = cid[i * stride];
  const int k = (int)floorf(c - 0.5f);
  if (k < 0 || k >= N) return;
  if (!(c > (float)k + 0.5f && c < (float)k + 1.5f)) return;
  atomicAdd(acc + k, 1.0);
}

}  // namespace pcn

using namespace pcn;

extern "C" int pcnerf_abi_version(void) { return PCNERF_ABI_VERSION; }
extern "C" const char* pcnerf_last_error(void) { return g_last_error.c_str(); }

static inline unsigned nblk(int64_t n, int per) { return (unsigned)((n + per - 1) / per); }

// a workgroup per ray (Grp<256>) when a wave per ray would leave most CUs idle: fewer rays than two 4-ray workgroups
// per CU (2048), with rows long enough (>= 512 samples) that 256 threads each hold >= 2 of them.  Override for
// A/B: pcnerf_set_composite_group(64 | 256 | 0 = this rule).
static int g_comp_group = 0;
static inline bool composite_block_per_ray(int64_t n_rays, int n_samples) {
  if (g_comp_group == 64) return false;
  if (g_comp_group == 256) return true;
  return n_rays < 2048 && n_samples >= 512;
}
extern "C" int pcnerf_set_composite_group(int g) {
  if (g != 0 && g != 64 && g != 256) {
    pcn::set_error("pcnerf_set_composite_group: 0 (automatic), 64 (a wave per ray) or 256 (a workgroup per ray)");
    return -1;
  }
  const int prev = g_comp_group;
  g_comp_group = g;
  return prev;
}

extern "C" int pcnerf_sample_coarse(const float* rays, int64_t n_rays, int ray_stride, int near_col, int far_col,
                                    int child_near_col, int child_far_col, int n_samples, int n_parent,
                                    int disparity, float* z, void* stream) {
  PCN_API_BEGIN
  PCN_CHECK(rays && z, "pcnerf_sample_coarse: null argument");
  PCN_CHECK(n_rays > 0 && n_samples > 0, "pcnerf_sample_coarse: empty input");
  PCN_CHECK(n_parent >= 1 && n_parent <= n_samples, "pcnerf_sample_coarse: n_parent out of range");
  const int maxc = near_col > far_col ? near_col : far_col;
  PCN_CHECK(maxc < ray_stride && child_near_col < ray_stride && child_far_col < ray_stride,
            "pcnerf_sample_coarse: column outside ray row");
  ProfScope ps((hipStream_t)stream, PT_SAMPLE, 0.0, (double)n_rays * (4.0 * ray_stride + 4.0 * n_samples));
  hipLaunchKernelGGL(k_sample_coarse, dim3(nblk(n_rays, 4)), dim3(256), 0, (hipStream_t)stream, rays, n_rays,
                     ray_stride, near_col, far_col, child_near_col, child_far_col, n_samples, n_parent, disparity,
                     z);
  PCN_LAUNCH_CHECK("pcnerf_sample_coarse");
  PCN_API_END
}

extern "C" int pcnerf_perturb(const float* z, int64_t n_rays, int n_samples, float perturb, const float* rand,
                              float* z_out, void* stream) {
  PCN_API_BEGIN
  PCN_CHECK(z && rand && z_out && z != z_out, "pcnerf_perturb: null or aliased argument");
  PCN_CHECK(n_rays > 0 && n_samples > 0, "pcnerf_perturb: empty input");
  const int64_t total = n_rays * (int64_t)n_samples;
  hipLaunchKernelGGL(k_perturb, dim3(nblk(total, 256)), dim3(256), 0, (hipStream_t)stream, z, total, n_samples,
                     perturb, rand, z_out);
  PCN_LAUNCH_CHECK("pcnerf_perturb");
  PCN_API_END
}

// render_rays' depth2 tie order: 0 = stable (torch's sort on the GPU, default), 1 = torch CPU's std::sort
static int g_depth2_order = 0;

extern "C" int pcnerf_set_depth2_order(int order) {
  PCN_API_BEGIN
  PCN_CHECK(order == 0 || order == 1, "pcnerf_set_depth2_order: order must be 0 (stable) or 1 (torch CPU)");
  g_depth2_order = order;
  PCN_API_END
}

extern "C" int pcnerf_composite(const float* p, const float* z, int64_t n_rays, int n_samples, const float* noise,
                                float noise_std, float eps, const float* rays, int ray_stride, int child_near_col,
                                int child_far_col, int range_col, float* weights, float* depth, float* free_ray,
                                float* sl1_ray, double* opac_row, float* depth2, void* stream) {
  PCN_API_BEGIN
  PCN_CHECK(p && z && depth, "pcnerf_composite: null argument");
  PCN_CHECK(!depth2 || weights, "pcnerf_composite: depth2 needs the weights output");
  PCN_CHECK(n_rays > 0 && n_samples > 0, "pcnerf_composite: empty input");
  if (rays) {
    PCN_CHECK(free_ray && sl1_ray, "pcnerf_composite: child losses need free_ray and sl1_ray");
    PCN_CHECK(child_near_col < ray_stride && child_far_col < ray_stride && range_col < ray_stride,
              "pcnerf_composite: column outside ray row");
  }
  PCN_CHECK(!depth2 || g_depth2_order == 0 || n_samples <= 2048,
            "pcnerf_composite: depth2 in torch CPU's tie order (pcnerf_set_depth2_order(1)) supports at most 2048 "
            "samples per ray");
  hipStream_t s = (hipStream_t)stream;
  const dim3 b(256);
  const double ns = (double)n_rays * n_samples;
  ProfScope ps(s, PT_COMPOSITE, 0.0, ns * (weights ? 12.0 : 8.0) + (rays ? 60.0 * n_rays : 0.0) + 12.0 * n_rays);
#define PCN_COMP(MB, G, GRID)                                                                                 \
  hipLaunchKernelGGL((k_composite<MB, G>), GRID, b, 0, s, p, z, n_rays, n_samples, noise, noise_std, eps,     \
                     rays, ray_stride, child_near_col, child_far_col, range_col, weights, depth, free_ray,    \
                     sl1_ray, opac_row, depth2, (int*)nullptr)
  if (composite_block_per_ray(n_rays, n_samples)) {
    const int B = (n_samples + 255) / 256;
    const dim3 g((unsigned)n_rays);
    if (B <= 2) PCN_COMP(2, 256, g);
    else if (B <= 6) PCN_COMP(6, 256, g);
    else if (B <= 16) PCN_COMP(16, 256, g);
    else if (B <= 64) PCN_COMP(64, 256, g);
    else PCN_CHECK(false, "pcnerf_composite: more than 16384 samples per ray");
  } else {
    const int B = (n_samples + 63) / 64;
    const dim3 g(nblk(n_rays, 4));
    if (B <= 2) PCN_COMP(2, 64, g);
    else if (B <= 6) PCN_COMP(6, 64, g);
    else if (B <= 16) PCN_COMP(16, 64, g);
    else if (B <= 64) PCN_COMP(64, 64, g);
    else if (B <= 256) PCN_COMP(256, 64, g);
    else PCN_CHECK(false, "pcnerf_composite: more than 16384 samples per ray");
  }
#undef PCN_COMP
  if (depth2 && g_depth2_order == 1)   // rows whose w[S-1] ties: torch CPU's order of equal keys
    hipLaunchKernelGGL(k_depth2_ties, dim3(nblk(n_rays, 4)), b, (size_t)8 * 4 * n_samples, s, weights, z, n_rays,
                       n_samples, depth2);
  PCN_LAUNCH_CHECK("pcnerf_composite");
  PCN_API_END
}

extern "C" int pcnerf_resample(const float* z, const float* weights, int64_t n_rays, int n_samples, int n_importance,
                               const float* u, float* z_fine, void* stream) {
  PCN_API_BEGIN
  PCN_CHECK(z && weights && z_fine, "pcnerf_resample: null argument");
  PCN_CHECK(n_rays > 0 && n_samples >= 3 && n_importance > 0, "pcnerf_resample: need n_samples >= 3");
  PCN_CHECK(n_rays <= 0x7fffffff, "pcnerf_resample: more than 2^31 - 1 rays in one call");
  const int F = n_samples + n_importance;
  int P2 = 1, PF = 1;
  while (P2 < F) P2 <<= 1;
  while (PF < n_importance) PF <<= 1;
  const size_t lds = (size_t)(n_samples + PF + std::max(3 * n_samples, P2)) * sizeof(float);
  // about four comparators per thread in each bitonic stage of the fine sort
  const int nt = PF >= 2048 ? 512 : PF >= 1024 ? 256 : PF >= 512 ? 128 : 64;
  // (+ the static float64 block-scan slots, NT / 64 of them)
  PCN_CHECK(lds + (size_t)(nt / 64) * sizeof(double) <= 160 * 1024,
            "pcnerf_resample: n_samples + n_importance too large for one workgroup's LDS");
  ProfScope ps((hipStream_t)stream, PT_RESAMPLE, 0.0,
               (double)n_rays * (8.0 * n_samples + 4.0 * F + (u ? 4.0 * n_importance : 0.0)));
#define PCN_RS(NT)                                                                                                \
  do {                                                                                                            \
    if (lds > 64 * 1024)                                                                                          \
      PCN_HIP(hipFuncSetAttribute((const void*)k_resample<NT>, hipFuncAttributeMaxDynamicSharedMemorySize,       \
                                  (int)lds));                                                                     \
    hipLaunchKernelGGL(k_resample<NT>, dim3((unsigned)n_rays), dim3(NT), lds, (hipStream_t)stream, z, weights,   \
                       n_samples, n_importance, PF, P2, u, z_fine);                                               \
  } while (0)
  if (nt == 512) PCN_RS(512);
  else if (nt == 256) PCN_RS(256);
  else if (nt == 128) PCN_RS(128);
  else PCN_RS(64);
#undef PCN_RS
  PCN_LAUNCH_CHECK("pcnerf_resample");
  PCN_API_END
}

extern "C" int pcnerf_sample_pdf(const float* bins, const float* weights, int64_t n_rays, int n_bins, int n_samples,
                                 const float* u, float* out, void* stream) {
  PCN_API_BEGIN
  PCN_CHECK(bins && weights && out, "pcnerf_sample_pdf: null argument");
  PCN_CHECK(n_rays > 0 && n_bins >= 2 && n_samples > 0, "pcnerf_sample_pdf: need n_bins >= 2");
  const size_t per_wave = (size_t)3 * n_bins * sizeof(float);
  PCN_CHECK(per_wave <= 64 * 1024, "pcnerf_sample_pdf: too many bins");
  int nw = (int)((64 * 1024) / per_wave);
  if (nw > 4) nw = 4;
  hipLaunchKernelGGL(k_sample_pdf, dim3(nblk(n_rays, nw)), dim3(64 * nw), per_wave * nw, (hipStream_t)stream, bins,
                     weights, n_rays, n_bins, n_samples, u, out);
  PCN_LAUNCH_CHECK("pcnerf_sample_pdf");
  PCN_API_END
}

extern "C" size_t pcnerf_child_loss_workspace_bytes(int n) { return (size_t)(n > 0 ? n : 1) * 3 * sizeof(double); }

extern "C" int pcnerf_child_loss_reduce(const float* free_ray, const float* sl1_ray, int64_t n_rays,
                                        const float* child_id, int id_stride, int sub_nerf_test_num, void* workspace,
                                        float* out, void* stream) {
  PCN_API_BEGIN
  PCN_CHECK(free_ray && sl1_ray && out, "pcnerf_child_loss_reduce: null argument");
  PCN_CHECK(n_rays > 0, "pcnerf_child_loss_reduce: empty input");
  hipStream_t s = (hipStream_t)stream;
  if (sub_nerf_test_num <= 0) {
    hipLaunchKernelGGL(k_child_loss_plain, dim3(1), dim3(1024), 0, s, free_ray, sl1_ray, n_rays, out);
  } else {
    PCN_CHECK(child_id && workspace, "pcnerf_child_loss_reduce: divide branch needs child ids and workspace");
    PCN_HIP(hipMemsetAsync(workspace, 0, pcnerf_child_loss_workspace_bytes(sub_nerf_test_num), s));
    hipLaunchKernelGGL(k_child_loss_scatter, dim3(nblk(n_rays, 256)), dim3(256), 0, s, free_ray, sl1_ray, n_rays,
                       child_id, id_stride, sub_nerf_test_num, (double*)workspace);
    hipLaunchKernelGGL(k_child_loss_divide, dim3(1), dim3(1024), 0, s, (const double*)workspace, sub_nerf_test_num,
                       out);
  }
  PCN_LAUNCH_CHECK("pcnerf_child_loss_reduce");
  PCN_API_END
}

extern "C" size_t pcnerf_child_range_loss_workspace_bytes(int n) { return (size_t)(n > 0 ? n : 1) * 2 * sizeof(double); }

extern "C" int pcnerf_child_range_loss(const float* pred, const float* target, int64_t n, const float* child_id,
                                       int id_stride, int sub_nerf_test_num, int kind, float pre_scale,
                                       float post_scale, void* workspace, float* out, void* stream) {
  PCN_API_BEGIN
  PCN_CHECK(pred && target && child_id && workspace && out, "pcnerf_child_range_loss: null argument");
  PCN_CHECK(n > 0 && sub_nerf_test_num > 0, "pcnerf_child_range_loss: empty input or no children");
  PCN_CHECK(kind >= 0 && kind <= 2, "pcnerf_child_range_loss: kind must be 0, 1 or 2");
  hipStream_t s = (hipStream_t)stream;
  PCN_HIP(hipMemsetAsync(workspace, 0, pcnerf_child_range_loss_workspace_bytes(sub_nerf_test_num), s));
  hipLaunchKernelGGL(k_child_range_scatter, dim3(nblk(n, 256)), dim3(256), 0, s, pred, target, n, child_id, id_stride,
                     sub_nerf_test_num, kind, pre_scale, (double*)workspace);
  hipLaunchKernelGGL(k_child_range_reduce, dim3(1), dim3(1024), 0, s, (const double*)workspace, sub_nerf_test_num,
                     post_scale, out);
  PCN_LAUNCH_CHECK("pcnerf_child_range_loss");
  PCN_API_END
}

extern "C" int pcnerf_child_range_loss_backward(const float* pred, const float* target, int64_t n,
                                                const float* child_id, int id_stride, int sub_nerf_test_num, int kind,
                                                float pre_scale, float post_scale, const void* workspace,
                                                const float* grad_out, float* grad_pred, void* stream) {
  PCN_API_BEGIN
  PCN_CHECK(pred && target && child_id && workspace && grad_out && grad_pred,
            "pcnerf_child_range_loss_backward: null argument");
  PCN_CHECK(n > 0 && sub_nerf_test_num > 0, "pcnerf_child_range_loss_backward: empty input or no children");
  PCN_CHECK(kind >= 0 && kind <= 2, "pcnerf_child_range_loss_backward: kind must be 0, 1 or 2");
  hipLaunchKernelGGL(k_child_range_bwd, dim3(nblk(n, 256)), dim3(256), 0, (hipStream_t)stream, pred, target, n,
                     child_id, id_stride, sub_nerf_test_num, kind, pre_scale, post_scale, (const double*)workspace,
                     grad_out, grad_pred);
  PCN_LAUNCH_CHECK("pcnerf_child_range_loss_backward");
  PCN_API_END
}

extern "C" int pcnerf_mean_f64(const double* x, int64_t n, double denom, float* out, void* stream) {
  PCN_API_BEGIN
  PCN_CHECK(x && out && n > 0, "pcnerf_mean_f64: bad argument");
  hipLaunchKernelGGL(k_sum_f64, dim3(1), dim3(1024), 0, (hipStream_t)stream, x, n, denom, out);
  PCN_LAUNCH_CHECK("pcnerf_mean_f64");
  PCN_API_END
}

extern "C" int pcnerf_pointwise_loss(const float* pred, const float* target, const uint8_t* mask, int64_t n,
                                     int kind, float* out, void* stream) {
  PCN_API_BEGIN
  PCN_CHECK(pred && target && out, "pcnerf_pointwise_loss: null argument");
  PCN_CHECK(n > 0, "pcnerf_pointwise_loss: empty input");
  PCN_CHECK(kind >= 0 && kind <= 2, "pcnerf_pointwise_loss: kind must be 0 (mse), 1 (l1) or 2 (smoothl1)");
  hipLaunchKernelGGL(k_pointwise_loss, dim3(1), dim3(1024), 0, (hipStream_t)stream, pred, target, mask, n, kind,
                     out);
  PCN_LAUNCH_CHECK("pcnerf_pointwise_loss");
  PCN_API_END
}

extern "C" size_t pcnerf_composite_backward_workspace_bytes(int sub_nerf_test_num) {
  return (size_t)(sub_nerf_test_num > 0 ? sub_nerf_test_num : 1) * sizeof(double);
}

extern "C" int pcnerf_composite_backward(const float* p, const float* z, int64_t n_rays, int n_samples,
                                         const float* noise, float noise_std, float eps, const float* rays,
                                         int ray_stride, int child_near_col, int child_far_col, int range_col,
                                         int child_id_col, int sub_nerf_test_num, const float* grad_depth,
                                         const float* grad_free_loss, const float* grad_depth_loss, void* workspace,
                                         float* grad_logit, void* stream) {
  PCN_API_BEGIN
  PCN_CHECK(p && z && grad_logit, "pcnerf_composite_backward: null argument");
  PCN_CHECK(n_rays > 0 && n_samples > 0, "pcnerf_composite_backward: empty input");
  hipStream_t s = (hipStream_t)stream;
  const double* counts = nullptr;
  if (rays && sub_nerf_test_num > 0) {
    PCN_CHECK(workspace, "pcnerf_composite_backward: divide branch needs a workspace");
    PCN_HIP(hipMemsetAsync(workspace, 0, pcnerf_composite_backward_workspace_bytes(sub_nerf_test_num), s));
    hipLaunchKernelGGL(k_child_counts, dim3(nblk(n_rays, 256)), dim3(256), 0, s, rays + child_id_col, ray_stride,
                       n_rays, sub_nerf_test_num, (double*)workspace);
    counts = (const double*)workspace;
  }
  const dim3 b(256);
  ProfScope ps(s, PT_COMPOSITE_BWD, 0.0, (double)n_rays * n_samples * (12.0 + (noise ? 4.0 : 0.0)));
#define PCN_CB(MB, G, GRID)                                                                                   \
  hipLaunchKernelGGL((k_composite_bwd<MB, G>), GRID, b, 0, s, p, z, n_rays, n_samples, noise, noise_std, eps, \
                     rays, ray_stride, child_near_col, child_far_col, range_col, child_id_col,               \
                     rays ? sub_nerf_test_num : 0, counts, grad_depth, grad_free_loss, grad_depth_loss,       \
                     grad_logit, (int*)nullptr)
  if (composite_block_per_ray(n_rays, n_samples)) {
    const int B = (n_samples + 255) / 256;
    const dim3 g((unsigned)n_rays);
    if (B <= 2) PCN_CB(2, 256, g);
    else if (B <= 6) PCN_CB(6, 256, g);
    else if (B <= 16) PCN_CB(16, 256, g);
    else PCN_CHECK(false, "pcnerf_composite_backward: more than 4096 samples per ray");
  } else {
    const int B = (n_samples + 63) / 64;
    const dim3 g(nblk(n_rays, 4));
    if (B <= 2) PCN_CB(2, 64, g);
    else if (B <= 6) PCN_CB(6, 64, g);
    else if (B <= 16) PCN_CB(16, 64, g);
    else if (B <= 64) PCN_CB(64, 64, g);
    else PCN_CHECK(false, "pcnerf_composite_backward: more than 4096 samples per ray");
  }
#undef PCN_CB
  PCN_LAUNCH_CHECK("pcnerf_composite_backward");
  PCN_API_END
}

extern "C" int pcnerf_pointwise_loss_backward(const float* pred, const float* target, const uint8_t* mask, int64_t n,
                                              int kind, const float* grad_out, float* grad_pred, void* stream) {
  PCN_API_BEGIN
  PCN_CHECK(pred && target && grad_out && grad_pred, "pcnerf_pointwise_loss_backward: null argument");
  PCN_CHECK(n > 0, "pcnerf_pointwise_loss_backward: empty input");
  PCN_CHECK(kind >= 0 && kind <= 2, "pcnerf_pointwise_loss_backward: kind must be 0, 1 or 2");
  hipLaunchKernelGGL(k_pointwise_loss_bwd, dim3(1), dim3(1024), 0, (hipStream_t)stream, pred, target, mask, n, kind,
                     grad_out, grad_pred);
  PCN_LAUNCH_CHECK("pcnerf_pointwise_loss_backward");
  PCN_API_END
}
