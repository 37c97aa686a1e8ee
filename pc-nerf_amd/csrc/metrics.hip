// Point-cloud metrics of the evaluation step (nof/criteria/pointcloud_metrics.py:5-49,
// logs/*/render_result/print_metrics.py:31-52): nearest-neighbour distances between a rendered and a reference
// cloud, Chamfer distance, precision/recall/F-score at a threshold, range error and accuracy.
//
// The reference builds an open3d KD-tree per cloud and queries it point by point from Python.  Here the search
// is exhaustive on the GPU, in float64 (open3d and scipy compute squared distances of float64 coordinates), so
// the nearest distance is the exact minimum: ~10^10 point pairs per 100k-point frame, one query per lane, the
// reference cloud streamed through LDS in tiles that every lane of the block reads by broadcast.
#include "common.h"
#include "pcnerf_internal.h"

namespace pcn {

constexpr int NN_TILE = 1024;

// dist[i] = min_j |q_i - r_j| (float64), q/r float32 xyz rows
__global__ __launch_bounds__(256) void k_nn_dist(const float* __restrict__ ref, int64_t n_ref,
                                                 const float* __restrict__ qry, int64_t n_qry,
                                                 double* __restrict__ dist) {
  __shared__ double rx[NN_TILE], ry[NN_TILE], rz[NN_TILE];
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool active = i < n_qry;
  const double qx = active ? (double)qry[3 * i] : 0.0, qy = active ? (double)qry[3 * i + 1] : 0.0,
               qz = active ? (double)qry[3 * i + 2] : 0.0;
  double best = INFINITY;
  for (int64_t t0 = 0; t0 < n_ref; t0 += NN_TILE) {
    const int cnt = (int)(n_ref - t0 < NN_TILE ? n_ref - t0 : NN_TILE);
    __syncthreads();
    for (int k = threadIdx.x; k < cnt; k += blockDim.x) {
      rx[k] = (double)ref[3 * (t0 + k)];
      ry[k] = (double)ref[3 * (t0 + k) + 1];
      rz[k] = (double)ref[3 * (t0 + k) + 2];
    }
    __syncthreads();
    int k = 0;
    for (; k + 4 <= cnt; k += 4) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const double dx = qx - rx[k + u], dy = qy - ry[k + u], dz = qz - rz[k + u];
        const double d2 = dx * dx + dy * dy + dz * dz;
        best = d2 < best ? d2 : best;
      }
    }
    for (; k < cnt; ++k) {
      const double dx = qx - rx[k], dy = qy - ry[k], dz = qz - rz[k];
      const double d2 = dx * dx + dy * dy + dz * dz;
      best = d2 < best ? d2 : best;
    }
  }
  if (active) dist[i] = sqrt(best);
}

__device__ __forceinline__ double block_sum(double v, double* sh) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  const int w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) sh[w] = v;
  __syncthreads();
  double s = 0.0;
  for (int k = 0; k < nw; ++k) s += sh[k];
  return s;
}

// out[0] = sum d, out[1] = count(d < threshold)   (one block)
__global__ void k_dist_stats(const double* __restrict__ d, int64_t n, double threshold, double* __restrict__ out) {
  __shared__ double sh[16];
  double s = 0.0, c = 0.0;
  for (int64_t i = threadIdx.x; i < n; i += blockDim.x) {
    s += d[i];
    c += d[i] < threshold ? 1.0 : 0.0;
  }
  s = block_sum(s, sh);
  c = block_sum(c, sh);
  if (threadIdx.x == 0) {
    out[0] = s;
    out[1] = c;
  }
}

// print_metrics.py:44-52 over n aligned points: |range_pred - range_gt| with ranges from `origin`
// out[0] = sum |e|, out[1] = count(|e| < threshold)
__global__ void k_range_stats(const float* __restrict__ pred, const float* __restrict__ gt,
                              const float* __restrict__ origin, int64_t n, double threshold,
                              double* __restrict__ out) {
  __shared__ double sh[16];
  const double ox = origin[0], oy = origin[1], oz = origin[2];
  double s = 0.0, c = 0.0;
  for (int64_t i = threadIdx.x; i < n; i += blockDim.x) {
    const double px = (double)pred[3 * i] - ox, py = (double)pred[3 * i + 1] - oy, pz = (double)pred[3 * i + 2] - oz;
    const double gx = (double)gt[3 * i] - ox, gy = (double)gt[3 * i + 1] - oy, gz = (double)gt[3 * i + 2] - oz;
    const double e = fabs(sqrt(px * px + py * py + pz * pz) - sqrt(gx * gx + gy * gy + gz * gz));
    s += e;
    c += e < threshold ? 1.0 : 0.0;
  }
  s = block_sum(s, sh);
  c = block_sum(c, sh);
  if (threadIdx.x == 0) {
    out[0] = s;
    out[1] = c;
  }
}

// print_metrics.py:37-41: precision over the reference points' distances, recall over the rendered points'
__global__ void k_eval_finish(const double* __restrict__ acc, int64_t n_gt, int64_t n_pred, double* __restrict__ out) {
  const double precision = acc[1] / (double)n_gt, recall = acc[3] / (double)n_pred;
  out[0] = acc[0] / (double)n_gt + acc[2] / (double)n_pred;
  out[1] = 2.0 * precision * recall / (precision + recall);
  out[2] = precision;
  out[3] = recall;
}

}  // namespace pcn

using namespace pcn;

extern "C" int pcnerf_nn_distance(const float* ref, int64_t n_ref, const float* query, int64_t n_query,
                                  double* dist, void* stream) {
  PCN_API_BEGIN
  PCN_CHECK(ref && query && dist, "pcnerf_nn_distance: null argument");
  PCN_CHECK(n_ref > 0 && n_query > 0, "pcnerf_nn_distance: empty cloud");
  hipLaunchKernelGGL(k_nn_dist, dim3((unsigned)((n_query + 255) / 256)), dim3(256), 0, (hipStream_t)stream, ref,
                     n_ref, query, n_query, dist);
  PCN_LAUNCH_CHECK("pcnerf_nn_distance");
  PCN_API_END
}

extern "C" size_t pcnerf_eval_pts_workspace_bytes(int64_t n_pred, int64_t n_gt) {
  return (size_t)(n_pred + n_gt) * sizeof(double) + 4 * sizeof(double);
}

extern "C" int pcnerf_eval_pts(const float* pred, int64_t n_pred, const float* gt, int64_t n_gt, double threshold,
                               void* workspace, double* out, void* stream) {
  PCN_API_BEGIN
  PCN_CHECK(pred && gt && workspace && out, "pcnerf_eval_pts: null argument");
  PCN_CHECK(n_pred > 0 && n_gt > 0, "pcnerf_eval_pts: empty cloud");
  hipStream_t s = (hipStream_t)stream;
  double* d1 = (double*)workspace;   // for each gt point, nearest pred point (pointcloud_metrics.py:39)
  double* d2 = d1 + n_gt;            // for each pred point, nearest gt point (:40)
  double* acc = d2 + n_pred;
  hipLaunchKernelGGL(k_nn_dist, dim3((unsigned)((n_gt + 255) / 256)), dim3(256), 0, s, pred, n_pred, gt, n_gt, d1);
  hipLaunchKernelGGL(k_nn_dist, dim3((unsigned)((n_pred + 255) / 256)), dim3(256), 0, s, gt, n_gt, pred, n_pred, d2);
  hipLaunchKernelGGL(k_dist_stats, dim3(1), dim3(1024), 0, s, d1, n_gt, threshold, acc);
  hipLaunchKernelGGL(k_dist_stats, dim3(1), dim3(1024), 0, s, d2, n_pred, threshold, acc + 2);
  hipLaunchKernelGGL(k_eval_finish, dim3(1), dim3(1), 0, s, acc, n_gt, n_pred, out);
  PCN_LAUNCH_CHECK("pcnerf_eval_pts");
  PCN_API_END
}

extern "C" int pcnerf_range_metrics(const float* pred, const float* gt, const float* origin, int64_t n,
                                    double threshold, double* out, void* stream) {
  PCN_API_BEGIN
  PCN_CHECK(pred && gt && origin && out, "pcnerf_range_metrics: null argument");
  PCN_CHECK(n > 0, "pcnerf_range_metrics: empty input");
  hipLaunchKernelGGL(k_range_stats, dim3(1), dim3(1024), 0, (hipStream_t)stream, pred, gt, origin, n, threshold, out);
  PCN_LAUNCH_CHECK("pcnerf_range_metrics");
  PCN_API_END
}
