// Ray-table construction on the GPU: ray/AABB intersection against the parent block and the child boxes
// (SURVEY.md 8(a) a3-a5).  float64 throughout, like the reference's numpy; one thread per LiDAR point.
//   train/val rows (nof/dataset/ipb2dmapping.py:736-768): KD-tree child lookup (find_aabb_box :174-197, the
//     first of the 10 nearest centres whose box holds the point), child near/far from the face-hit test
//     (compute_far_bound0606 :119-172), +-surface_expand, parent far (compute_far_bound :36-77), 15 columns;
//   two-step rows (eval_kitti_render.py:675-803): parent far by slab (ray_aabb_distances :213-235), children whose
//     centre lies within 0.65 m of the ray line (distance_to_ray :237-244), exactly-two-face-hit test
//     (compute_far_bound0429 :170-211), cumulative 0.05 m expansion retries, hits sorted by near, 13 columns.
// Variable-length outputs: pass 0 counts rows per point, a one-block scan gives offsets, pass 1 recomputes and
// writes (the work is cheap next to the memory it would take to keep every point's hits).
#include <stdint.h>

#include "common.h"
#include "pcnerf_internal.h"

namespace pcn {

constexpr int KNN = 10;      // find_aabb_box: tree.query(k=10)
constexpr int HIT_MAX = 64;  // max child hits kept per ray (KITTI logs: <= 28)
constexpr int CTILE = 1024;  // child centres per LDS tile

__device__ __forceinline__ int face_hits(const double (&p)[3], const double (&d)[3], const double* lo,
                                         const double* hi, double (&out)[6]) {
  int n = 0;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const double b = s == 0 ? lo[i] : hi[i];
      if (d[i] * (b - p[i]) > 0) {
        const double dist = (b - p[i]) / d[i];
        int cnt = 0;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          if (k == i) continue;
          const double pe = p[k] + dist * d[k];
          cnt += (pe >= lo[k] && pe <= hi[k]) ? 1 : 0;
        }
        if (cnt >= 2) out[n++] = dist;
      }
    }
  }
  return n;
}

__device__ __forceinline__ double parent_far_train(const double (&o)[3], const double (&d)[3], const double* P6) {
  // compute_far_bound: x_max, x_min, y_max, y_min, z_max, z_min planes; t < 0 or d == 0 -> inf; all inf -> None
  double t = __builtin_inf();
#pragma unroll
  for (int a = 0; a < 3; ++a) {
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const double b = s == 0 ? P6[3 + a] : P6[a];
      double ti = __builtin_inf();
      if (d[a] != 0) {
        ti = (b - o[a]) / d[a];
        if (ti < 0) ti = __builtin_inf();
      }
      t = ti < t ? ti : t;
    }
  }
  return t == __builtin_inf() ? __builtin_nan("") : t;
}

__device__ __forceinline__ void ray_of(const double* q, const double (&o)[3], double (&d)[3], double& rng) {
  const double v0 = q[0] - o[0], v1 = q[1] - o[1], v2 = q[2] - o[2];
  rng = sqrt(v0 * v0 + v1 * v1 + v2 * v2);
  d[0] = v0 / rng;
  d[1] = v1 / rng;
  d[2] = v2 / rng;
}

// ------------------------------------------------------------------------------- train/val rows
// pass 0: cnt[i] = 1 if point i yields a row; pass 1: rows[off[i]] = the row.
__global__ __launch_bounds__(256) void k_train_rays(int pass, const double* __restrict__ pts, int64_t n,
                                                    const double* __restrict__ origin, const double* __restrict__ ctr,
                                                    const double* __restrict__ b6, int64_t C,
                                                    const double* __restrict__ P6, double se, int rule,
                                                    int* __restrict__ cnt, const int64_t* __restrict__ off,
                                                    float* __restrict__ rows, int* __restrict__ nshort) {
  __shared__ double sc[CTILE * 3];
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool act = i < n;
  const double o[3] = {origin[0], origin[1], origin[2]};
  double q[3] = {0, 0, 0};
  if (act) {
    q[0] = pts[3 * i];
    q[1] = pts[3 * i + 1];
    q[2] = pts[3 * i + 2];
  }
  // the KNN nearest child centres (squared Euclidean distance, ties by index), sorted ascending
  double kd[KNN];
  int ki[KNN];
#pragma unroll
  for (int k = 0; k < KNN; ++k) {
    kd[k] = __builtin_inf();
    ki[k] = -1;
  }
  for (int64_t c0 = 0; c0 < C; c0 += CTILE) {
    const int nt = (int)(C - c0 < CTILE ? C - c0 : CTILE);
    __syncthreads();
    for (int t = threadIdx.x; t < nt * 3; t += blockDim.x) sc[t] = ctr[c0 * 3 + t];
    __syncthreads();
    if (!act) continue;
    for (int t = 0; t < nt; ++t) {
      const double a = q[0] - sc[3 * t], b = q[1] - sc[3 * t + 1], e = q[2] - sc[3 * t + 2];
      const double ds = a * a + b * b + e * e;
      if (ds < kd[KNN - 1]) {
        int pos = KNN - 1;
        const int ci = (int)(c0 + t);
#pragma unroll
        for (int k = KNN - 1; k > 0; --k) {
          if (kd[k - 1] > ds) {
            kd[k] = kd[k - 1];
            ki[k] = ki[k - 1];
            pos = k - 1;
          } else {
            break;
          }
        }
        kd[pos] = ds;
        ki[pos] = ci;
      }
    }
  }
  if (!act) return;
  int child = -1;
#pragma unroll
  for (int k = 0; k < KNN; ++k) {
    const int c = ki[k];
    if (child < 0 && c >= 0) {
      const double* b = b6 + 6 * c;
      if (q[0] >= b[0] && q[1] >= b[1] && q[2] >= b[2] && q[0] <= b[3] && q[1] <= b[4] && q[2] <= b[5]) child = c;
    }
  }
  int ok = 0;
  double near = 0, far = 0, d[3], rng;
  ray_of(q, o, d, rng);
  if (child >= 0) {
    double h[6];
    const int nh = face_hits(o, d, b6 + 6 * child, b6 + 6 * child + 3, h);
    if (rule == 1) {
      // compute_far_bound0406 (MaiCity, ipb2dmapping.py:82-114): the first two hits in face order; every point in a
      // child box yields a row; fewer than two hits is the reference's IndexError (counted, the caller raises)
      ok = 1;
      if (nh >= 2) {
        near = h[0] < h[1] ? h[0] : h[1];
        far = h[0] < h[1] ? h[1] : h[0];
      } else if (pass == 0) {
        atomicAdd(nshort, 1);
      }
    } else if (nh > 0) {  // compute_far_bound0606 (KITTI, :119-172): min / max over all hits, none -> dropped
      ok = 1;
      near = h[0];
      far = h[0];
      for (int k = 1; k < nh; ++k) {
        near = h[k] < near ? h[k] : near;
        far = h[k] > far ? h[k] : far;
      }
    }
  }
  if (pass == 0) {
    cnt[i] = ok;
    return;
  }
  if (!ok) return;
  near = near - se;
  far = far + se;
  double pf = parent_far_train(o, d, P6);
  if (pf < far) pf = far;
  float* r = rows + 15 * off[i];
  r[0] = (float)o[0];
  r[1] = (float)o[1];
  r[2] = (float)o[2];
  r[3] = (float)d[0];
  r[4] = (float)d[1];
  r[5] = (float)d[2];
  r[6] = 0.0f;
  r[7] = (float)pf;
  r[8] = 3.0f;
  r[9] = (float)(child + 1);
  r[10] = (float)near;
  r[11] = (float)far;
  r[12] = (float)(rng - se);
  r[13] = (float)far;  // ipb2dmapping.py:815: the point-far column takes the child far bound
  r[14] = (float)rng;
}

// ------------------------------------------------------------------------------- two-step rows
struct ViewHit {
  double near, far, col7;
  int tin;
};

__global__ __launch_bounds__(256) void k_view_rays(int pass, const double* __restrict__ pts, int64_t n,
                                                   const double* __restrict__ origin, const double* __restrict__ b6,
                                                   int64_t C, const double* __restrict__ P6, int method, int rule,
                                                   double radius, int* __restrict__ cnt,
                                                   const int64_t* __restrict__ off, float* __restrict__ rows,
                                                   float* __restrict__ ranges, int64_t* __restrict__ other,
                                                   uint8_t* __restrict__ tin, int* __restrict__ overflow) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double o[3] = {origin[0], origin[1], origin[2]};
  const double q[3] = {pts[3 * i], pts[3 * i + 1], pts[3 * i + 2]};
  double d[3], rng;
  ray_of(q, o, d, rng);
  // parent far: slab exit (NaN-propagating min/max like numpy), inf when the slabs miss
  double tmin = -__builtin_inf(), tmax = __builtin_inf();
  {
    double lo_t[3], hi_t[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      const double t1 = (P6[a] - o[a]) / d[a], t2 = (P6[3 + a] - o[a]) / d[a];
      const bool nan = t1 != t1 || t2 != t2;
      lo_t[a] = nan ? __builtin_nan("") : (t1 < t2 ? t1 : t2);
      hi_t[a] = nan ? __builtin_nan("") : (t1 > t2 ? t1 : t2);
    }
    bool nan = false;
    for (int a = 0; a < 3; ++a) nan |= lo_t[a] != lo_t[a];
    tmin = nan ? __builtin_nan("") : fmax(fmax(lo_t[0], lo_t[1]), lo_t[2]);
    nan = false;
    for (int a = 0; a < 3; ++a) nan |= hi_t[a] != hi_t[a];
    tmax = nan ? __builtin_nan("") : fmin(fmin(hi_t[0], hi_t[1]), hi_t[2]);
  }
  const double pfar = tmax >= tmin ? tmax : __builtin_inf();
  const double pnear = 0.0;
  ViewHit hits[HIT_MAX];
  int nh = 0;
  // expansion rounds: ext_r = ext_{r-1} + step (float64; KITTI 0.05, MaiCity 0.005), the filtered boxes grow by
  // ext_1, then ext_2, ... (the reference updates them in place); give up once ext > 0.5
  const double step = rule == 1 ? 0.005 : 0.05;
  double ext_now = 0.0;
  int rounds = 0;
  bool drop = false;
  for (;;) {
    for (int64_t c = 0; c < C && !(method == 1 && nh > 0); ++c) {
      const double* b = b6 + 6 * c;
      // distance_to_ray of the centre of the ORIGINAL box
      const double cx = (b[0] + b[3]) / 2, cy = (b[1] + b[4]) / 2, cz = (b[2] + b[5]) / 2;
      const double v0 = cx - o[0], v1 = cy - o[1], v2 = cz - o[2];
      const double dist = sqrt(v0 * v0 + v1 * v1 + v2 * v2);
      const double cs = (v0 * d[0] + v1 * d[1] + v2 * d[2]) / dist;
      const double dr = dist * sqrt(1 - cs * cs);
      if (!(dr <= radius)) continue;
      double lo[3] = {b[0], b[1], b[2]}, hi[3] = {b[3], b[4], b[5]};
      double e = 0.0;
      for (int r = 1; r <= rounds; ++r) {
        e = e + step;
        for (int a = 0; a < 3; ++a) {
          lo[a] = lo[a] - e;
          hi[a] = hi[a] + e;
        }
      }
      double h[6];
      if (face_hits(o, d, lo, hi, h) != 2) continue;
      const double a0 = h[0] < h[1] ? h[0] : h[1], a1 = h[0] < h[1] ? h[1] : h[0];
      if (nh >= HIT_MAX) {
        atomicAdd(overflow, 1);
        break;
      }
      ViewHit& H = hits[nh++];
      H.near = method == 1 ? pnear : a0;
      H.far = method == 1 ? pfar : a1;
      H.col7 = rule == 1 ? pfar : (pfar < a1 ? a1 : pfar);   // MaiCity keeps the parent far bound as is
      H.tin = (q[0] >= lo[0] && q[0] <= hi[0] && q[1] >= lo[1] && q[1] <= hi[1] && q[2] >= lo[2] && q[2] <= hi[2]);
    }
    if (nh > 0) break;
    if (ext_now > 0.5) {
      drop = true;
      break;
    }
    ext_now = ext_now + step;
    ++rounds;
  }
  const int k = drop ? 0 : nh;
  if (pass == 0) {
    cnt[i] = k;
    return;
  }
  if (k == 0) return;
  // sort by near (stable insertion sort)
  for (int a = 1; a < k; ++a) {
    const ViewHit t = hits[a];
    int b = a - 1;
    while (b >= 0 && hits[b].near > t.near) {
      hits[b + 1] = hits[b];
      --b;
    }
    hits[b + 1] = t;
  }
  const int64_t base = off[i];
  for (int j = 0; j < k; ++j) {
    float* r = rows + 13 * (base + j);
    r[0] = (float)o[0];
    r[1] = (float)o[1];
    r[2] = (float)o[2];
    r[3] = (float)d[0];
    r[4] = (float)d[1];
    r[5] = (float)d[2];
    r[6] = (float)hits[j].near;
    r[7] = (float)hits[j].far;
    r[8] = 3.0f;
    r[9] = (float)pnear;
    r[10] = (float)hits[j].col7;
    r[11] = (float)(j + 1);
    r[12] = j == 0 ? (float)(k - 1) : -1.0f;
    ranges[base + j] = (float)rng;
    other[base + j] = j == 0 ? (int64_t)(k - 1) : 0;
    tin[base + j] = (uint8_t)hits[j].tin;
  }
}

// exclusive scan of int counts -> int64 offsets, total in off[n]; one block
__global__ __launch_bounds__(1024) void k_scan_counts(const int* __restrict__ cnt, int64_t n,
                                                      int64_t* __restrict__ off) {
  __shared__ int64_t part[1024];
  const int t = threadIdx.x;
  const int64_t per = (n + 1023) / 1024;
  const int64_t a = t * per, b = a + per < n ? a + per : n;
  int64_t s = 0;
  for (int64_t i = a; i < b; ++i) s += cnt[i];
  part[t] = s;
  __syncthreads();
  if (t == 0) {
    int64_t run = 0;
    for (int k = 0; k < 1024; ++k) {
      const int64_t v = part[k];
      part[k] = run;
      run += v;
    }
    off[n] = run;
  }
  __syncthreads();
  int64_t run = part[t];
  for (int64_t i = a; i < b; ++i) {
    off[i] = run;
    run += cnt[i];
  }
}

}  // namespace pcn

using namespace pcn;

extern "C" size_t pcnerf_rays_workspace_bytes(int64_t n_points) {
  return (size_t)((n_points + 1) * 8 + n_points * 4 + 64 + 255) & ~(size_t)255;
}

extern "C" int pcnerf_build_train_rays(const double* points, int64_t n_points, const double* origin,
                                       const double* centers, const double* bounds6, int64_t n_children,
                                       const double* parent6, double surface_expand, int face_rule, void* workspace,
                                       float* rows, int64_t* n_rows, int* n_short, void* stream) {
  PCN_API_BEGIN
  PCN_CHECK(points && origin && centers && bounds6 && parent6 && workspace && rows && n_rows,
            "pcnerf_build_train_rays: null argument");
  PCN_CHECK(n_points > 0 && n_children >= KNN, "pcnerf_build_train_rays: need points and >= 10 child boxes");
  PCN_CHECK(face_rule == 0 || (face_rule == 1 && n_short),
            "pcnerf_build_train_rays: face_rule must be 0 (0606) or 1 (0406, with n_short)");
  hipStream_t s = (hipStream_t)stream;
  int64_t* off = (int64_t*)workspace;
  int* cnt = (int*)(off + n_points + 1);
  const dim3 g((unsigned)((n_points + 255) / 256)), b(256);
  if (n_short) PCN_HIP(hipMemsetAsync(n_short, 0, sizeof(int), s));
  hipLaunchKernelGGL(k_train_rays, g, b, 0, s, 0, points, n_points, origin, centers, bounds6, n_children, parent6,
                     surface_expand, face_rule, cnt, (const int64_t*)nullptr, rows, n_short);
  hipLaunchKernelGGL(k_scan_counts, dim3(1), dim3(1024), 0, s, cnt, n_points, off);
  hipLaunchKernelGGL(k_train_rays, g, b, 0, s, 1, points, n_points, origin, centers, bounds6, n_children, parent6,
                     surface_expand, face_rule, cnt, off, rows, n_short);
  PCN_HIP(hipMemcpyAsync(n_rows, off + n_points, sizeof(int64_t), hipMemcpyDeviceToDevice, s));
  PCN_LAUNCH_CHECK("pcnerf_build_train_rays");
  PCN_API_END
}

extern "C" int pcnerf_count_view_rows(const double* points, int64_t n_points, const double* origin,
                                      const double* bounds6, int64_t n_children, const double* parent6, int method,
                                      int rule, void* workspace, int64_t* n_rows, void* stream) {
  PCN_API_BEGIN
  PCN_CHECK(points && origin && bounds6 && parent6 && workspace && n_rows, "pcnerf_count_view_rows: null argument");
  PCN_CHECK(n_points > 0 && n_children > 0, "pcnerf_count_view_rows: empty input");
  PCN_CHECK(rule == 0 || rule == 1, "pcnerf_count_view_rows: rule must be 0 (KITTI) or 1 (MaiCity)");
  hipStream_t s = (hipStream_t)stream;
  int64_t* off = (int64_t*)workspace;
  int* cnt = (int*)(off + n_points + 1);
  int* ovf = (int*)(cnt + n_points);
  PCN_HIP(hipMemsetAsync(ovf, 0, sizeof(int), s));
  hipLaunchKernelGGL(k_view_rays, dim3((unsigned)((n_points + 255) / 256)), dim3(256), 0, s, 0, points, n_points,
                     origin, bounds6, n_children, parent6, method, rule, 0.65, cnt, (const int64_t*)nullptr,
                     (float*)nullptr, (float*)nullptr, (int64_t*)nullptr, (uint8_t*)nullptr, ovf);
  hipLaunchKernelGGL(k_scan_counts, dim3(1), dim3(1024), 0, s, cnt, n_points, off);
  PCN_HIP(hipMemcpyAsync(n_rows, off + n_points, sizeof(int64_t), hipMemcpyDeviceToDevice, s));
  PCN_LAUNCH_CHECK("pcnerf_count_view_rows");
  PCN_API_END
}

extern "C" int pcnerf_emit_view_rows(const double* points, int64_t n_points, const double* origin,
                                     const double* bounds6, int64_t n_children, const double* parent6, int method,
                                     int rule, void* workspace, float* rows, float* ranges, int64_t* other,
                                     uint8_t* true_in, void* stream) {
  PCN_API_BEGIN
  PCN_CHECK(points && origin && bounds6 && parent6 && workspace && rows && ranges && other && true_in,
            "pcnerf_emit_view_rows: null argument");
  int64_t* off = (int64_t*)workspace;
  int* cnt = (int*)(off + n_points + 1);
  int* ovf = (int*)(cnt + n_points);
  hipLaunchKernelGGL(k_view_rays, dim3((unsigned)((n_points + 255) / 256)), dim3(256), 0, (hipStream_t)stream, 1,
                     points, n_points, origin, bounds6, n_children, parent6, method, rule, 0.65, cnt,
                     (const int64_t*)off, rows, ranges, other, true_in, ovf);
  PCN_LAUNCH_CHECK("pcnerf_emit_view_rows");
  PCN_API_END
}
