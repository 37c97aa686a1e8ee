// Two-step (coarse-to-fine) inference stages of render_rays_view_0525_2_2 (nof/render.py:229-368, 614-699):
// per-row compositing, the strict child mask with its expansion loop, the Gaussian-smoothed weight peak
// (scipy.ndimage.gaussian_filter, sigma 5, reflect, render.py:306), child-sum, method-0/2 depth, opacity and
// points (k_view_rows, one wave per row); then the ray-group walk that flags one effective row per ray group
// (render.py:317-340; k_view_walk).
#include <stdint.h>

#include "common.h"
#include "pcnerf_internal.h"

namespace pcn {

__device__ __forceinline__ double view_excl_prod(double v, int lane) {
  double incl = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const double n = __shfl_up(incl, o, 64);
    if (lane >= o) incl *= n;
  }
  const double ex = __shfl_up(incl, 1, 64);
  return lane == 0 ? 1.0 : ex;
}

// scipy 'reflect' extension (d c b a | a b c d | d c b a), any distance
__device__ __forceinline__ int reflect_index(int j, int n) {
  const int p = 2 * n;
  int m = j % p;
  if (m < 0) m += p;
  return m < n ? m : p - 1 - m;
}

template <int MAXB>
__global__ __launch_bounds__(256) void k_view_rows(const float* __restrict__ P, const float* __restrict__ Z,
                                                   int64_t n_rows, int S, const float* __restrict__ rows, int stride,
                                                   int cn_col, int cf_col, int method, float eps,
                                                   const double* __restrict__ gw, int radius,
                                                   float* __restrict__ Wout, float* __restrict__ depth,
                                                   uint8_t* __restrict__ at_peak, float* __restrict__ wsum,
                                                   double* __restrict__ opac_row, float* __restrict__ points) {
  extern __shared__ float lds_rows[];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const int64_t row0 = (int64_t)blockIdx.x * nw + wid;
  if (row0 >= n_rows) return;  // no block-level barrier below: waves are independent
  const int64_t row = row0;
  float* lrow = lds_rows + (size_t)wid * S;
  const int B = (S + 63) / 64;
  const int i0 = lane * B;
  const int nb = max(0, min(B, S - i0));
  const float* pr = P + row * S + i0;
  const float* zr = Z + row * S + i0;
  float pv[MAXB], zv[MAXB], wv[MAXB];
  double loc = 1.0, op = 0.0;
#pragma unroll
  for (int j = 0; j < MAXB; ++j) {
    if (j < nb) {
      pv[j] = pr[j];
      zv[j] = zr[j];
      const float fr = 1.0f - pv[j];
      loc *= (double)fr;
      // opacity term (render.py:354): log(0.1 + p) + log(0.1 + (1 - p)) + 2.20727
      op += (double)((logf(0.1f + pv[j]) + logf(0.1f + fr)) + 2.20727f);
    } else {
      pv[j] = zv[j] = 0.0f;
    }
  }
  double T = view_excl_prod(loc, lane);
  double sw = 0.0;
#pragma unroll
  for (int j = 0; j < MAXB; ++j) {
    if (j < nb) {
      wv[j] = (float)T * pv[j];
      sw += (double)wv[j];
      T *= (double)(1.0f - pv[j]);
    } else {
      wv[j] = 0.0f;
    }
  }
  const float den = (float)wave_sum_d(sw) + eps;  // render.py:246
#pragma unroll
  for (int j = 0; j < MAXB; ++j)
    if (j < nb) {
      wv[j] = wv[j] / den;
      lrow[i0 + j] = wv[j];
      if (Wout) Wout[row * S + i0 + j] = wv[j];
    }
  // strict child mask, expanded by 0.01 from 0.01 until it holds a sample (render.py:252-263)
  const float* r = rows + row * stride;
  const float cn = r[cn_col], cf = r[cf_col];
  double thr = 0.01;
  float lo = 0.0f, hi = 0.0f;
  for (int it = 0; it < 4000000; ++it) {
    const float t32 = (float)thr;
    lo = cn - t32;
    hi = cf + t32;
    bool any = false;
#pragma unroll
    for (int j = 0; j < MAXB; ++j)
      if (j < nb) any |= (lo < zv[j] && zv[j] < hi);
    if (__any(any)) break;
    thr = thr + 0.01;
  }
  double sc = 0.0, sd = 0.0;
#pragma unroll
  for (int j = 0; j < MAXB; ++j)
    if (j < nb) {
      const float m = (lo < zv[j] && zv[j] < hi) ? 1.0f : 0.0f;
      sc += (double)(wv[j] * m);
      if (method != 2) sd += (double)(wv[j] * zv[j]);
    }
  const float csum = (float)wave_sum_d(sc);
  if (method == 2) {  // render.py:346-348: child re-normalised weights
    const float denc = csum + eps;
#pragma unroll
    for (int j = 0; j < MAXB; ++j)
      if (j < nb) {
        const float m = (lo < zv[j] && zv[j] < hi) ? 1.0f : 0.0f;
        sd += (double)(((wv[j] * m) / denc) * zv[j]);
      }
  }
  const float d = (float)wave_sum_d(sd);
  // Gaussian smoothing of the weight row (scipy correlate1d, symmetric kernel: x[k]*w0 + sum over the outer
  // taps first of (x[k-j] + x[k+j]) * w_j, in float64, rounded to float32) and its first argmax
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  float best = -__builtin_inff();
  int bidx = 0x7fffffff;
  for (int j = 0; j < nb; ++j) {
    const int k = i0 + j;
    double t = (double)lrow[k] * gw[radius];
    for (int q = -radius; q < 0; ++q)
      t = t + ((double)lrow[reflect_index(k + q, S)] + (double)lrow[reflect_index(k - q, S)]) * gw[radius + q];
    const float v = (float)t;
    if (v > best) {
      best = v;
      bidx = k;
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(best, o, 64);
    const int oi = __shfl_xor(bidx, o, 64);
    if (ov > best || (ov == best && oi < bidx)) {
      best = ov;
      bidx = oi;
    }
  }
  const double opw = wave_sum_d(op);
  if (lane == 0) {
    const float zp = Z[row * S + bidx];
    at_peak[row] = (lo < zp && zp < hi) ? 1 : 0;
    wsum[row] = csum;
    depth[row] = d;
    opac_row[row] = opw;
  }
  if (points && lane < 3) points[row * 3 + lane] = r[lane] + d * r[3 + lane];  // render.py:674-684
}

// Ray-group walk (render.py:317-340): i = 0; while i < R: other[i] == 0 -> flag i, i += 1; other[i] > 0 ->
// pick the first row of the group i..i+other[i] whose smoothed peak lies in its child mask, else the row with
// the largest child weight sum (strict >, starting from i), i += other[i] + 1; other[i] < 0 -> i += 1.
// Well-formed batches (every group's inner rows have other == 0, groups disjoint and complete) are processed in
// parallel over the grid -- the walk then visits exactly the rows no group covers; anything else falls back to
// the literal sequential walk.  Three launches (the kernel boundaries order the phases across workgroups):
//   k_walk_cover  every group head marks its inner rows covered and flags a malformed list; per-block partial
//                 sums of the opacity terms;
//   k_walk_pick   (well-formed) every uncovered row: flag it (other == 0) or pick its group's row;
//   k_walk_finish one thread: the opacity mean from the partials in block order (deterministic), and the
//                 sequential walk when the list was malformed.
__device__ __forceinline__ void pick_group(const uint8_t* __restrict__ at_peak, const float* __restrict__ wsum,
                                           uint8_t* __restrict__ flag, int64_t i, int64_t o) {
  int64_t pick = i;
  if (!at_peak[i]) {
    bool found = false;
    for (int64_t j = 0; j < o; ++j)
      if (at_peak[i + j + 1]) {
        pick = i + j + 1;
        found = true;
        break;
      }
    if (!found)
      for (int64_t j = 0; j < o; ++j)
        if (wsum[i + j + 1] > wsum[pick]) pick = i + j + 1;
  }
  flag[pick] = 1;
}

constexpr int WALK_THREADS = 256;

__global__ __launch_bounds__(WALK_THREADS) void k_walk_cover(const int64_t* __restrict__ other, int64_t n,
                                                             int* __restrict__ covered, int* __restrict__ bad,
                                                             const double* __restrict__ opac_row,
                                                             double* __restrict__ partial) {
  __shared__ double red[WALK_THREADS / 64];
  const int64_t i = (int64_t)blockIdx.x * WALK_THREADS + threadIdx.x;
  double os = 0.0;
  if (i < n) {
    os = opac_row[i];
    const int64_t o = other[i];
    if (o > 0) {
      if (i + o >= n) atomicOr(bad, 1);
      for (int64_t j = i + 1; j <= i + o && j < n; ++j) {
        if (other[j] != 0) atomicOr(bad, 1);
        if (atomicAdd(&covered[j], 1) != 0) atomicOr(bad, 1);
      }
    }
  }
  os = wave_sum_d(os);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = os;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0.0;
    for (int w = 0; w < WALK_THREADS / 64; ++w) t += red[w];
    partial[blockIdx.x] = t;
  }
}

__global__ __launch_bounds__(WALK_THREADS) void k_walk_pick(const int64_t* __restrict__ other, int64_t n,
                                                            const int* __restrict__ covered,
                                                            const int* __restrict__ bad,
                                                            const uint8_t* __restrict__ at_peak,
                                                            const float* __restrict__ wsum,
                                                            uint8_t* __restrict__ flag) {
  if (*bad) return;
  const int64_t i = (int64_t)blockIdx.x * WALK_THREADS + threadIdx.x;
  if (i >= n || covered[i]) return;
  const int64_t o = other[i];
  if (o == 0) flag[i] = 1;
  else if (o > 0) pick_group(at_peak, wsum, flag, i, o);
}

__global__ void k_walk_finish(const int64_t* __restrict__ other, int64_t n, const int* __restrict__ bad,
                              const uint8_t* __restrict__ at_peak, const float* __restrict__ wsum,
                              uint8_t* __restrict__ flag, const double* __restrict__ partial, int nblocks,
                              double n_elems, float* __restrict__ opac_out) {
  if (threadIdx.x != 0) return;
  double t = 0.0;
  for (int b = 0; b < nblocks; ++b) t += partial[b];
  opac_out[0] = (float)(t / n_elems);
  if (!*bad) return;
  int64_t i = 0;
  while (i < n) {
    const int64_t o = other[i];
    if (o == 0) {
      flag[i] = 1;
      i += 1;
    } else if (o > 0) {
      if (i + o >= n) break;  // the reference would raise IndexError here
      pick_group(at_peak, wsum, flag, i, o);
      i += o + 1;
    } else {
      i += 1;
    }
  }
}

}  // namespace pcn

using namespace pcn;

extern "C" int pcnerf_view_rows(const float* p, const float* z, int64_t n_rows, int n_samples, const float* rows,
                                int row_stride, int child_near_col, int child_far_col, int method, float eps,
                                const double* gauss, int radius, float* weights, float* depth, uint8_t* at_peak,
                                float* child_sum, double* opac_row, float* points, void* stream) {
  PCN_API_BEGIN
  PCN_CHECK(p && z && rows && gauss && depth && at_peak && child_sum && opac_row, "pcnerf_view_rows: null argument");
  PCN_CHECK(n_rows > 0 && n_samples > 0 && radius >= 0, "pcnerf_view_rows: empty input");
  PCN_CHECK(child_near_col < row_stride && child_far_col < row_stride && row_stride >= 6,
            "pcnerf_view_rows: column outside row");
  const size_t per_wave = (size_t)n_samples * sizeof(float);
  PCN_CHECK(per_wave <= 64 * 1024, "pcnerf_view_rows: more than 16384 samples per row");
  int nw = (int)((64 * 1024) / per_wave);
  if (nw > 4) nw = 4;
  const int B = (n_samples + 63) / 64;
  const dim3 g((unsigned)((n_rows + nw - 1) / nw)), b(64 * nw);
  hipStream_t s = (hipStream_t)stream;
#define PCN_VIEW(MB)                                                                                        \
  hipLaunchKernelGGL(k_view_rows<MB>, g, b, per_wave * nw, s, p, z, n_rows, n_samples, rows, row_stride,   \
                     child_near_col, child_far_col, method, eps, gauss, radius, weights, depth, at_peak,   \
                     child_sum, opac_row, points)
  if (B <= 2) PCN_VIEW(2);
  else if (B <= 6) PCN_VIEW(6);
  else if (B <= 16) PCN_VIEW(16);
  else if (B <= 64) PCN_VIEW(64);
  else PCN_VIEW(256);
#undef PCN_VIEW
  PCN_LAUNCH_CHECK("pcnerf_view_rows");
  PCN_API_END
}

static int64_t walk_blocks(int64_t n) { return (n + WALK_THREADS - 1) / WALK_THREADS; }

// covered[n] (int) | bad (int, padded to 16 B) | per-block opacity partials (double)
extern "C" size_t pcnerf_view_walk_workspace_bytes(int64_t n_rows) {
  const int64_t n = n_rows > 0 ? n_rows : 1;
  return (((size_t)n * 4 + 15) & ~(size_t)15) + 16 + (size_t)walk_blocks(n) * 8;
}

extern "C" int pcnerf_view_walk(const int64_t* other, int64_t n_rows, const uint8_t* at_peak, const float* child_sum,
                                const double* opac_row, int n_samples, void* workspace, uint8_t* flags,
                                float* opacity, void* stream) {
  PCN_API_BEGIN
  PCN_CHECK(other && at_peak && child_sum && opac_row && workspace && flags && opacity,
            "pcnerf_view_walk: null argument");
  PCN_CHECK(n_rows > 0, "pcnerf_view_walk: empty input");
  hipStream_t s = (hipStream_t)stream;
  const int64_t nb = walk_blocks(n_rows);
  PCN_CHECK(nb < (int64_t)1 << 31, "pcnerf_view_walk: too many rows");
  char* w = (char*)workspace;
  int* covered = (int*)w;
  int* bad = (int*)(w + (((size_t)n_rows * 4 + 15) & ~(size_t)15));
  double* partial = (double*)((char*)bad + 16);
  PCN_HIP(hipMemsetAsync(workspace, 0, (((size_t)n_rows * 4 + 15) & ~(size_t)15) + 16, s));
  PCN_HIP(hipMemsetAsync(flags, 0, (size_t)n_rows, s));
  hipLaunchKernelGGL(k_walk_cover, dim3((unsigned)nb), dim3(WALK_THREADS), 0, s, other, n_rows, covered, bad, opac_row,
                     partial);
  hipLaunchKernelGGL(k_walk_pick, dim3((unsigned)nb), dim3(WALK_THREADS), 0, s, other, n_rows, covered, bad, at_peak,
                     child_sum, flags);
  hipLaunchKernelGGL(k_walk_finish, dim3(1), dim3(64), 0, s, other, n_rows, bad, at_peak, child_sum, flags, partial,
                     (int)nb, (double)n_rows * n_samples, opacity);
  PCN_LAUNCH_CHECK("pcnerf_view_walk");
  PCN_API_END
}
