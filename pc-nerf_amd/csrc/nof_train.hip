// Train-mode NOF query: BatchNorm1d with batch statistics over each chunk of `chunk` flattened ray-major
// samples (nof/render.py:47-50 chunk loop; nn.BatchNorm1d train semantics; models.py:183-203).
//
// Every BatchNorm needs the statistics of its whole chunk before the next Linear may run, so the network is
// evaluated layer by layer per chunk:
//   k_train_layer  : h_L = W'_L x + b'_L on MFMA for the chunk, written raw (pre-BN) to HBM, with per-neuron
//                    sums of (h - c) and (h - c)^2 (shift c = the expected mean) reduced in the epilogue;
//   k_bn_fold      : mean / biased var -> alpha = gamma/sqrt(var+eps), beta' = beta - mean*alpha; running
//                    stats updated (momentum, unbiased var); the BN is folded into the NEXT Linear:
//                    W'_{L+1} = W_{L+1} diag(alpha), b'_{L+1} = b_{L+1} + W_{L+1} beta' (packed for MFMA);
//   k_train_out    : occ_out Linear(256,1) on the folded last BN + sigmoid.
// The activations LeakyReLU(True) are identities (negative_slope == 1) and are not applied.
//
// MFMA mapping (v_mfma_f32_32x32x2_f32), samples on rows: out[sample][neuron] = act[sample][:] . W^T[:][neuron]
//   A (lane l) = act[sample l&31][feature(t, l>>5)],  B (lane l) = W'[32*ob + (l&31)][feature(t, l>>5)]
//   D (block ob, reg r, lane l) = out[sample (r&3) + 8*(r>>2) + 4*(l>>5)][neuron 32*ob + (l&31)]
// so each lane owns one neuron per block and the per-neuron statistics are register sums (no cross-lane
// reduction).  feature(t, h) = 8*(t>>2) + 4*h + (t&3): k-steps 4g..4g+3 read one float4 per lane from the
// activation tile stored as [tile][g][lane][4] (1 KiB per wave-instruction).
#include "common.h"
#include "pcnerf_internal.h"
#include "prof.h"

namespace pcn {

constexpr int KG_E = 8, KG_H = 32;
constexpr size_t SZ_E = (size_t)KG_E * 8 * 64 * 4;
constexpr size_t SZ_H = (size_t)KG_H * 8 * 64 * 4;
constexpr size_t TILE_FLOATS = 32 * 256;

__host__ __device__ inline size_t packed_index(int n, int f) {
  // neuron n, input feature f (0..255 or 0..63) -> position in a [kg][ob][lane][q] part
  const int ob = n >> 5, i = n & 31, g = f >> 3, hh = (f >> 2) & 1, q = f & 3;
  return (((size_t)g * 8 + ob) * 64 + (i + 32 * hh)) * 4 + q;
}

template <int KG, int NX>
__device__ __forceinline__ void gemm_n_regs(f32x16 (&acc)[8], const float (&x)[NX], const float* __restrict__ wp,
                                            int lane) {
  static_assert(NX == 4 * KG, "operand count");
  const f32x4* __restrict__ w4 = reinterpret_cast<const f32x4*>(wp) + lane;
  f32x4 wa[8];
#pragma unroll
  for (int ob = 0; ob < 8; ++ob) wa[ob] = w4[ob * 64];
#pragma unroll
  for (int kg = 0; kg < KG; ++kg) {
    f32x4 wb[8];
    if (kg + 1 < KG) {
#pragma unroll
      for (int ob = 0; ob < 8; ++ob) wb[ob] = w4[((kg + 1) * 8 + ob) * 64];
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
#pragma unroll
      for (int ob = 0; ob < 8; ++ob)
        acc[ob] = __builtin_amdgcn_mfma_f32_32x32x2f32(x[4 * kg + q], wa[ob][q], acc[ob], 0, 0, 0);
    }
    if (kg + 1 < KG) {
#pragma unroll
      for (int ob = 0; ob < 8; ++ob) wa[ob] = wb[ob];
    }
  }
}

template <int KG>
__device__ __forceinline__ void gemm_n_mem(f32x16 (&acc)[8], const float* __restrict__ xt,
                                           const float* __restrict__ wp, int lane) {
  const f32x4* __restrict__ w4 = reinterpret_cast<const f32x4*>(wp) + lane;
  const f32x4* __restrict__ x4 = reinterpret_cast<const f32x4*>(xt) + lane;
  f32x4 wa[8];
  f32x4 xa = x4[0];
#pragma unroll
  for (int ob = 0; ob < 8; ++ob) wa[ob] = w4[ob * 64];
#pragma unroll
  for (int kg = 0; kg < KG; ++kg) {
    f32x4 wb[8];
    f32x4 xb;
    if (kg + 1 < KG) {
      xb = x4[(kg + 1) * 64];
#pragma unroll
      for (int ob = 0; ob < 8; ++ob) wb[ob] = w4[((kg + 1) * 8 + ob) * 64];
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
#pragma unroll
      for (int ob = 0; ob < 8; ++ob)
        acc[ob] = __builtin_amdgcn_mfma_f32_32x32x2f32(xa[q], wa[ob][q], acc[ob], 0, 0, 0);
    }
    if (kg + 1 < KG) {
      xa = xb;
#pragma unroll
      for (int ob = 0; ob < 8; ++ob) wa[ob] = wb[ob];
    }
  }
}

// One pre-BN Linear over a chunk [c0, c0 + n) of flattened samples.  EP: the encoding half (layer 1 and the
// skip half of layer 5) computed from positions; HP: the 256 BN'd features read from `hin`.
template <bool EP, bool HP>
__global__ __launch_bounds__(256, 2) void k_train_layer(const float* __restrict__ rays, int stride,
                                                        const float* __restrict__ z, int S, int64_t c0, int64_t n,
                                                        const float* __restrict__ ein, const float* __restrict__ hin, const float* __restrict__ Wp,
                                                        const float* __restrict__ bias,
                                                        const float* __restrict__ shift, float* __restrict__ hout,
                                                        double* __restrict__ stats) {
  __shared__ double st[512];
  for (int i = threadIdx.x; i < 512; i += blockDim.x) st[i] = 0.0;
  __syncthreads();
  const int lane = threadIdx.x & 63, h = lane >> 5, wv = threadIdx.x >> 6;
  const int64_t ntiles = (n + 31) / 32;
  // activation tile offset of this lane's neuron column (see the [tile][g][lane][4] layout above)
  const int li = lane & 31;
  const int lane_off = ((li >> 3) * 64 + 32 * ((li >> 2) & 1) + 4 * h) * 4 + (li & 3);
  for (int64_t tile = (int64_t)blockIdx.x * 4 + wv; tile < ntiles; tile += (int64_t)gridDim.x * 4) {
    // opaque per-iteration copy of the weight pointer: without it the compiler hoists all 256 weight
    // float4s of the layer out of the tile loop (loop-invariant) and spills them to scratch
    const float* wpt = Wp;
    asm volatile("" : "+s"(wpt));
    f32x16 acc[8];
#pragma unroll
    for (int ob = 0; ob < 8; ++ob)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[ob][r] = 0.0f;
    if (EP) {
      int64_t sl = tile * 32 + li;
      if (sl >= n) sl = n - 1;
      const int64_t g = c0 + sl;
      float e[32];
      if (ein) {
        load_embedding<1>(ein + g * 63, h, e);
      } else {
        const float* r = rays + (g / S) * stride;
        float p[3];
        sample_point(r, z[g], p);
        encode_half<1>(p, h, e);
      }
      gemm_n_regs<KG_E>(acc, e, wpt, lane);
    }
    if (HP) gemm_n_mem<KG_H>(acc, hin + tile * TILE_FLOATS, wpt + (EP ? SZ_E : 0), lane);
    // epilogue: + bias, raw h to the next layer's tile layout, shifted statistics of the valid samples
    float* ho = hout + tile * TILE_FLOATS + lane_off;
    const int64_t base = tile * 32;
#pragma unroll
    for (int ob = 0; ob < 8; ++ob) {
      const int nn = 32 * ob + li;
      const float bo = bias[nn], so = shift[nn];
      float s1 = 0.0f, s2 = 0.0f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int s = (r & 3) + 8 * (r >> 2) + 4 * h;
        const float v = acc[ob][r] + bo;
        ho[1024 * ob + 4 * ((r & 3) + 8 * (r >> 2))] = v;
        if (base + s < n) {
          const float d = v - so;
          s1 += d;
          s2 += d * d;
        }
      }
      atomicAdd(&st[2 * nn], (double)s1);
      atomicAdd(&st[2 * nn + 1], (double)s2);
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 512; i += blockDim.x) atomicAdd(&stats[i], st[i]);
}

// BatchNorm L's statistics -> folded next layer (L < 7) or folded occ_out (L == 7).
// grid: 256 blocks (one per neuron of layer L+1), or 1 block for L == 7; block: 256 threads (one per feature).
__global__ __launch_bounds__(256) void k_bn_fold(NofParamsDev P, int L, const double* __restrict__ stats,
                                                 const float* __restrict__ shift, int64_t n, float momentum,
                                                 float* __restrict__ Wp, float* __restrict__ bias_next,
                                                 float* __restrict__ shift_next) {
  __shared__ double red[2][4];
  const int k = threadIdx.x;
  const double s1 = stats[2 * k], s2 = stats[2 * k + 1];
  const double m = s1 / (double)n;
  const double mean = (double)shift[k] + m;
  double var = s2 / (double)n - m * m;
  if (var < 0.0) var = 0.0;
  // ATen batch_norm_cpu_update_stats: invstd = 1/sqrt(var + eps) in double, stored as float;
  // transform: alpha = invstd * gamma, beta' = beta - mean * alpha (float)
  const float invstd = (float)(1.0 / sqrt(var + (double)P.eps));
  const float a = invstd * P.bn_w[L][k];
  const float bp = P.bn_b[L][k] - (float)mean * a;
  if (blockIdx.x == 0) {
    const double mom = (double)momentum;
    P.bn_rm[L][k] = (float)(mom * mean + (1.0 - mom) * (double)P.bn_rm[L][k]);
    const double unb = n > 1 ? var * (double)n / (double)(n - 1) : var;
    P.bn_rv[L][k] = (float)(mom * unb + (1.0 - mom) * (double)P.bn_rv[L][k]);
  }
  const int lane = k & 63, wid = k >> 6;
  if (L == 7) {
    const float w = P.out_w[k];
    Wp[k] = w * a;
    double dp = wave_sum_d((double)w * (double)bp);
    if (lane == 0) red[0][wid] = dp;
    __syncthreads();
    if (k == 0) bias_next[0] = (float)((double)P.out_b[0] + red[0][0] + red[0][1] + red[0][2] + red[0][3]);
    return;
  }
  const int nxt = L + 1;
  const int nn = blockIdx.x;
  const int in_f = nxt == 4 ? 319 : 256;
  const int hc0 = nxt == 4 ? 63 : 0;
  const float* Wn = P.lin_w[nxt] + (size_t)nn * in_f;
  const float w = Wn[hc0 + k];
  Wp[(nxt == 4 ? SZ_E : 0) + packed_index(nn, k)] = w * a;
  if (nxt == 4 && k < 64) Wp[packed_index(nn, k)] = k < 63 ? Wn[k] : 0.0f;
  const double dp = wave_sum_d((double)w * (double)bp);
  const double dc = wave_sum_d((double)w * (double)P.bn_b[L][k]);
  if (lane == 0) {
    red[0][wid] = dp;
    red[1][wid] = dc;
  }
  __syncthreads();
  if (k == 0) {
    const double b = (double)P.lin_b[nxt][nn];
    bias_next[nn] = (float)(b + red[0][0] + red[0][1] + red[0][2] + red[0][3]);
    shift_next[nn] = (float)(b + red[1][0] + red[1][1] + red[1][2] + red[1][3]);
  }
}

// Layer 1's raw weights in the train-mode operand order (encoding features, feature 63 = zero padding).
__global__ void k_pack_train_first(const float* __restrict__ W1, float* __restrict__ Wp) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (int)SZ_E) return;
  const int q = idx & 3, lane = (idx >> 2) & 63, ob = (idx >> 8) & 7, kg = idx >> 11;
  const int f = 8 * kg + 4 * (lane >> 5) + q, nn = 32 * ob + (lane & 31);
  Wp[idx] = f < 63 ? W1[nn * 63 + f] : 0.0f;
}

// occ_out on the folded last BatchNorm + sigmoid; one wave per 32-sample tile.
__global__ __launch_bounds__(256) void k_train_out(const float* __restrict__ hin, int64_t n,
                                                   const float* __restrict__ wout, const float* __restrict__ bout,
                                                   float* __restrict__ p_out) {
  const int lane = threadIdx.x & 63, h = lane >> 5;
  const int64_t tile = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t ntiles = (n + 31) / 32;
  if (tile >= ntiles) return;
  const f32x4* x4 = reinterpret_cast<const f32x4*>(hin + tile * TILE_FLOATS) + lane;
  float part = 0.0f;
#pragma unroll 8
  for (int g = 0; g < 32; ++g) {
    const f32x4 x = x4[g * 64];
    const f32x4 w = *reinterpret_cast<const f32x4*>(wout + 8 * g + 4 * h);
    part = fmaf(x[0], w[0], part);
    part = fmaf(x[1], w[1], part);
    part = fmaf(x[2], w[2], part);
    part = fmaf(x[3], w[3], part);
  }
  const float logit = part + __shfl_xor(part, 32, 64) + bout[0];
  const int64_t s = tile * 32 + (lane & 31);
  if (lane < 32 && s < n) p_out[s] = sigmoid_ref(logit);
}

struct TrainWs {
  float* bufA;
  float* bufB;
  float* wp1;
  float* wp;
  float* bias;
  float* shift[2];  // c_L and c_{L+1} ping-pong: k_bn_fold reads one and writes the other
  float* wout;
  float* bout;
  double* stats;
  size_t bytes;
};

static TrainWs carve(void* base, int64_t chunk) {
  const size_t tiles = (size_t)((chunk + 31) / 32);
  size_t off = 0;
  auto take = [&](size_t bytes) {
    const size_t o = off;
    off += (bytes + 255) & ~(size_t)255;
    return o;
  };
  const size_t oA = take(tiles * TILE_FLOATS * 4), oB = take(tiles * TILE_FLOATS * 4);
  const size_t o1 = take(SZ_E * 4), ow = take((SZ_E + SZ_H) * 4), ob = take(256 * 4), os = take(2 * 256 * 4);
  const size_t owo = take(256 * 4), obo = take(16), ost = take(8 * 512 * 8);
  char* b = (char*)base;
  TrainWs w;
  w.bufA = (float*)(b + oA);
  w.bufB = (float*)(b + oB);
  w.wp1 = (float*)(b + o1);
  w.wp = (float*)(b + ow);
  w.bias = (float*)(b + ob);
  w.shift[0] = (float*)(b + os);
  w.shift[1] = (float*)(b + os) + 256;
  w.wout = (float*)(b + owo);
  w.bout = (float*)(b + obo);
  w.stats = (double*)(b + ost);
  w.bytes = off;
  return w;
}

}  // namespace pcn

using namespace pcn;

extern "C" size_t pcnerf_nof_train_workspace_bytes(int64_t chunk) { return carve(nullptr, chunk).bytes; }

static void query_train(const float* rays, int ray_stride, const float* z, int n_samples, const float* ein,
                        int64_t total, int64_t chunk, const pcnerf_nof_params* params, float momentum, float eps,
                        void* workspace, size_t workspace_bytes, float* p_out, void* stream) {
  const TrainWs ws = carve(workspace, chunk);
  PCN_CHECK(workspace_bytes >= ws.bytes, "pcnerf_nof_query_train: workspace too small");
  NofParamsDev P;
  PCN_CHECK(to_dev_params(params, eps, &P), "pcnerf_nof_query_train: null parameter pointer");
  // nn.BatchNorm1d raises for a chunk of one sample (render.py:47-50 would hit it on a 1-sample tail)
  PCN_CHECK(total % chunk != 1 && total != 1, "Expected more than 1 value per channel when training");
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(k_pack_train_first, dim3((unsigned)((SZ_E + 255) / 256)), dim3(256), 0, s, P.lin_w[0], ws.wp1);
  for (int64_t c0 = 0; c0 < total; c0 += chunk) {
    const int64_t n = total - c0 < chunk ? total - c0 : chunk;
    const int64_t ntiles = (n + 31) / 32;
    const unsigned grid = (unsigned)(ntiles / 4 + 1 < 512 ? ntiles / 4 + 1 : 512);
    PCN_HIP(hipMemsetAsync(ws.stats, 0, 8 * 512 * sizeof(double), s));
    float* hin = ws.bufA;
    float* hout = ws.bufB;
    // layer 1: encoding -> h1
    const double dn = (double)n;
    {
      ProfScope ps(s, PT_TRAIN_FIRST, 2.0 * 63 * 256 * dn, (4.0 + 1024.0) * dn);
      hipLaunchKernelGGL((k_train_layer<true, false>), dim3(grid), dim3(256), 0, s, rays, ray_stride, z, n_samples,
                         c0, n, ein, (const float*)nullptr, ws.wp1, P.lin_b[0], P.lin_b[0], hin, ws.stats);
    }
    for (int L = 0; L < 7; ++L) {
      const float* c_cur = L == 0 ? P.lin_b[0] : ws.shift[L & 1];
      float* c_next = ws.shift[(L + 1) & 1];
      {
        ProfScope ps(s, PT_BN_FOLD, 0.0, 4.0 * 256 * 320);
        hipLaunchKernelGGL(k_bn_fold, dim3(256), dim3(256), 0, s, P, L, ws.stats + 512 * L, c_cur, n, momentum,
                           ws.wp, ws.bias, c_next);
      }
      if (L + 1 == 4) {
        ProfScope ps(s, PT_TRAIN_SKIP, 2.0 * 319 * 256 * dn, (4.0 + 2048.0) * dn);
        hipLaunchKernelGGL((k_train_layer<true, true>), dim3(grid), dim3(256), 0, s, rays, ray_stride, z, n_samples,
                           c0, n, ein, hin, ws.wp, ws.bias, c_next, hout, ws.stats + 512 * (L + 1));
      } else {
        // algorithmic: 2*256*256 FLOP and 1 KiB in + 1 KiB out per sample
        ProfScope ps(s, PT_TRAIN_HIDDEN, 2.0 * 256 * 256 * dn, 2048.0 * dn);
        hipLaunchKernelGGL((k_train_layer<false, true>), dim3(grid), dim3(256), 0, s, rays, ray_stride, z,
                           n_samples, c0, n, ein, hin, ws.wp, ws.bias, c_next, hout, ws.stats + 512 * (L + 1));
      }
      float* t = hin;
      hin = hout;
      hout = t;
    }
    hipLaunchKernelGGL(k_bn_fold, dim3(1), dim3(256), 0, s, P, 7, ws.stats + 512 * 7, ws.shift[7 & 1], n, momentum,
                       ws.wout, ws.bout, (float*)nullptr);
    {
      ProfScope ps(s, PT_TRAIN_OUT, 2.0 * 256 * dn, 1028.0 * dn);
      hipLaunchKernelGGL(k_train_out, dim3((unsigned)((ntiles + 3) / 4)), dim3(256), 0, s, hin, n, ws.wout, ws.bout,
                         p_out + c0);
    }
  }
  PCN_LAUNCH_CHECK("pcnerf_nof_query_train");
}

extern "C" int pcnerf_nof_query_train(const float* rays, int64_t n_rays, int ray_stride, const float* z,
                                      int n_samples, int64_t chunk, const pcnerf_nof_params* params, float momentum,
                                      float eps, void* workspace, size_t workspace_bytes, float* p_out,
                                      void* stream) {
  PCN_API_BEGIN
  PCN_CHECK(rays && z && params && workspace && p_out, "pcnerf_nof_query_train: null argument");
  PCN_CHECK(n_rays > 0 && n_samples > 0 && chunk > 0, "pcnerf_nof_query_train: empty input");
  PCN_CHECK(ray_stride >= 6, "pcnerf_nof_query_train: ray_stride < 6");
  query_train(rays, ray_stride, z, n_samples, nullptr, n_rays * (int64_t)n_samples, chunk, params, momentum, eps,
              workspace, workspace_bytes, p_out, stream);
  PCN_API_END
}

extern "C" int pcnerf_nof_forward_train(const float* emb, int64_t n, const pcnerf_nof_params* params,
                                        float momentum, float eps, void* workspace, size_t workspace_bytes,
                                        float* p_out, void* stream) {
  PCN_API_BEGIN
  PCN_CHECK(emb && params && workspace && p_out, "pcnerf_nof_forward_train: null argument");
  PCN_CHECK(n > 0, "pcnerf_nof_forward_train: empty input");
  query_train(nullptr, 0, nullptr, 1, emb, n, n, params, momentum, eps, workspace, workspace_bytes, p_out, stream);
  PCN_API_END
}
