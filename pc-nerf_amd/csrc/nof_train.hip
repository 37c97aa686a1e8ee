// Train-mode NOF query: BatchNorm1d with batch statistics over each chunk of `chunk` flattened ray-major
// samples (nof/render.py:47-50 chunk loop; nn.BatchNorm1d train semantics; models.py:183-203).
//
// Every BatchNorm needs the statistics of its whole chunk before the next Linear may run, so the network is
// evaluated layer by layer per chunk, one launch per Linear:
//   k_train_layer<EP,HP> : prologue: BatchNorm L-1's coefficients from the chunk statistics of h_{L-1},
//                          alpha = gamma/sqrt(var+eps), beta' = beta - mean*alpha (ATen's transform form; block 0
//                          also updates running_mean/var with momentum and the unbiased variance);
//                          body: h_L = W_L (alpha*h_{L-1} + beta') + b_L on MFMA, the BatchNorm applied as the
//                          activations are loaded; h_L written raw (pre-BN) to HBM with per-neuron sums of
//                          (h - b) and (h - b)^2 reduced in the epilogue;
//   k_train_out          : the same prologue for BatchNorm 8, occ_out Linear(256,1) + sigmoid.
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

// tuning knobs (variant builds for A/B timing; defaults are the shipped configuration)
#ifndef PCN_TRAIN_WAVES
#define PCN_TRAIN_WAVES 1  // waves per SIMD the layer kernel is compiled for (launch bounds)
#endif
#ifndef PCN_XD
#define PCN_XD 4  // activation prefetch depth in k-groups (divides 32)
#endif
#ifndef PCN_WD
#define PCN_WD 2  // weight prefetch depth in k-groups (divides 32)
#endif

constexpr int KG_E = 8, KG_H = 32;
constexpr size_t SZ_E = (size_t)KG_E * 8 * 64 * 4;
constexpr size_t SZ_H = (size_t)KG_H * 8 * 64 * 4;
constexpr size_t TILE_FLOATS = 32 * 256;
constexpr int LDS_ROW = 260;


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
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
#pragma unroll
      for (int ob = 0; ob < 8; ++ob)
        acc[ob] = __builtin_amdgcn_mfma_f32_32x32x2f32(x[4 * kg + q], wa[ob][q], acc[ob], 0, 0, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
    if (kg + 1 < KG) {
#pragma unroll
      for (int ob = 0; ob < 8; ++ob) wa[ob] = wb[ob];
    }
  }
}

// Packed train-mode weights: the eval image's layout (off_w) with raw weights (no BatchNorm folding) in the
// samples-on-rows operand order, feature(t, h) = 8*(t>>2) + 4*h + (t&3).
__host__ __device__ constexpr size_t off_w(int layer, bool epart) {
  return layer == 0 ? 0
       : layer <= 3 ? SZ_E + (size_t)(layer - 1) * SZ_H
       : layer == 4 ? (epart ? SZ_E + 3 * SZ_H : 2 * SZ_E + 3 * SZ_H)
                    : 2 * SZ_E + (size_t)(layer - 1) * SZ_H;
}
constexpr size_t TRAIN_W_FLOATS = 2 * SZ_E + 7 * SZ_H;

__global__ void k_pack_train(NofParamsDev P, float* __restrict__ out) {
  const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= TRAIN_W_FLOATS) return;
  int layer;
  bool epart;
  size_t base;
  if (idx < SZ_E) { layer = 0; epart = true; base = 0; }
  else if (idx < SZ_E + 3 * SZ_H) { layer = 1 + (int)((idx - SZ_E) / SZ_H); epart = false; base = off_w(layer, false); }
  else if (idx < 2 * SZ_E + 3 * SZ_H) { layer = 4; epart = true; base = off_w(4, true); }
  else if (idx < 2 * SZ_E + 4 * SZ_H) { layer = 4; epart = false; base = off_w(4, false); }
  else { layer = 5 + (int)((idx - (2 * SZ_E + 4 * SZ_H)) / SZ_H); epart = false; base = off_w(layer, false); }
  const size_t j = idx - base;
  const int q = (int)(j & 3), lane = (int)((j >> 2) & 63), ob = (int)((j >> 8) & 7), kg = (int)(j >> 11);
  const int f = 8 * kg + 4 * (lane >> 5) + q, nn = 32 * ob + (lane & 31);
  const int in_f = layer == 0 ? 63 : layer == 4 ? 319 : 256;
  int col;
  if (epart) col = f < 63 ? f : -1;
  else col = (layer == 4 ? 63 : 0) + f;
  out[idx] = col < 0 ? 0.0f : P.lin_w[layer][(size_t)nn * in_f + col];
}

struct BnPrev {  // the BatchNorm whose output a layer consumes
  const float* gamma;
  const float* beta;
  float* rm;
  float* rv;
  const float* lin_bias;   // bias of the Linear that produced the statistics (the stats are of h - bias)
  const double* stats;     // [256][2]: sum(h - bias), sum((h - bias)^2) over the chunk
};

// alpha/beta' of one BatchNorm for feature k = threadIdx.x (256 threads); block 0 updates the running stats.
// ATen batch_norm_cpu_update_stats/transform: mean and biased var in float64, invstd = 1/sqrt(var+eps) stored as
// float, alpha = invstd*gamma, beta' = beta - mean*alpha; running = momentum*x + (1-momentum)*running with the
// unbiased variance.
__device__ __forceinline__ void bn_coeffs(const BnPrev& B, int64_t n, float momentum, float eps, float* al,
                                          float* be) {
  const int k = threadIdx.x;
  const double s1 = B.stats[2 * k], s2 = B.stats[2 * k + 1];
  const double m = s1 / (double)n;
  double var = s2 / (double)n - m * m;
  if (var < 0.0) var = 0.0;
  const double mean = (double)B.lin_bias[k] + m;
  const float invstd = (float)(1.0 / sqrt(var + (double)eps));
  const float a = invstd * B.gamma[k];
  al[k] = a;
  be[k] = B.beta[k] - (float)mean * a;
  if (blockIdx.x == 0) {
    const double mom = (double)momentum;
    B.rm[k] = (float)(mom * mean + (1.0 - mom) * (double)B.rm[k]);
    const double unb = n > 1 ? var * (double)n / (double)(n - 1) : var;
    B.rv[k] = (float)(mom * unb + (1.0 - mom) * (double)B.rv[k]);
  }
}

// 256-wide input streamed from HBM with the previous BatchNorm applied on load (x*alpha + beta').
// Software pipeline (one wave per SIMD has no partner to hide latency, so every load is issued ahead):
//   activations: ring of XD k-groups, weights: ring of WD k-groups, alpha/beta': one group ahead (LDS).
// Both rings are carried across tiles -- their last loads of a tile fetch the first groups of the next tile
// (the weights' addresses repeat), so a tile starts with its operands in flight.  KG_H % XD == KG_H % WD == 0
// keeps the ring slot of group g equal to g % depth in every tile.  sched_barrier pins the loads where they
// are issued (otherwise the scheduler sinks them next to their first use).
constexpr int XD = PCN_XD;
constexpr int WD = PCN_WD;
static_assert(KG_H % XD == 0 && KG_H % WD == 0, "ring depths must divide the k-group count");

struct HRing {
  f32x4 x[XD];
  f32x4 w[WD][8];
  f32x4 a, b;  // alpha/beta' of the next group
};

__device__ __forceinline__ void ring_fill(HRing& R, const f32x4* __restrict__ x4, const f32x4* __restrict__ w4,
                                          const float* __restrict__ al, const float* __restrict__ be, int h4) {
#pragma unroll
  for (int d = 0; d < XD; ++d) R.x[d] = x4[d * 64];
#pragma unroll
  for (int d = 0; d < WD; ++d)
#pragma unroll
    for (int ob = 0; ob < 8; ++ob) R.w[d][ob] = w4[(d * 8 + ob) * 64];
  R.a = *reinterpret_cast<const f32x4*>(al + h4);
  R.b = *reinterpret_cast<const f32x4*>(be + h4);
}

// `prev_out` (nullable): the previous tile's output, staged in LDS rows `stage_row`, is written to HBM one
// 1 KiB group per k-group (vmcnt retires in issue order: a burst of 32 stores at the end of a tile would hold
// back the waits of the next tile's first loads until the whole burst is acknowledged).
__device__ __forceinline__ void gemm_n_mem(f32x16 (&acc)[8], HRing& R, const f32x4* __restrict__ x4,
                                           const f32x4* __restrict__ x4_next, const f32x4* __restrict__ w4,
                                           const float* __restrict__ al, const float* __restrict__ be, int h4,
                                           f32x4* __restrict__ prev_out, const float* __restrict__ stage_row) {
#pragma unroll
  for (int kg = 0; kg < KG_H; ++kg) {
    f32x4 xa;
#pragma unroll
    for (int q = 0; q < 4; ++q) xa[q] = R.x[kg % XD][q] * R.a[q] + R.b[q];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
#pragma unroll
      for (int ob = 0; ob < 8; ++ob)
        acc[ob] = __builtin_amdgcn_mfma_f32_32x32x2f32(xa[q], R.w[kg % WD][ob][q], acc[ob], 0, 0, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
    const int gw = (kg + WD) % KG_H;  // group kg+WD of this tile, or the first groups of the next tile
#pragma unroll
    for (int ob = 0; ob < 8; ++ob) R.w[kg % WD][ob] = w4[(gw * 8 + ob) * 64];
    R.x[kg % XD] = kg + XD < KG_H ? x4[(kg + XD) * 64] : x4_next[(kg + XD - KG_H) * 64];
    const int ga = (kg + 1) % KG_H;
    R.a = *reinterpret_cast<const f32x4*>(al + 8 * ga + h4);
    R.b = *reinterpret_cast<const f32x4*>(be + 8 * ga + h4);
    if (prev_out) prev_out[kg * 64] = *reinterpret_cast<const f32x4*>(stage_row + 8 * kg);
    __builtin_amdgcn_sched_barrier(0);
  }
}

// One Linear over a chunk [c0, c0 + n) of flattened samples.  EP: the encoding half (layer 1, skip half of
// layer 5) computed from positions (or read from `ein`); HP: the 256 BatchNorm'd features of the previous layer.
template <bool EP, bool HP>
__global__ __launch_bounds__(256, PCN_TRAIN_WAVES) void k_train_layer(
    const float* __restrict__ rays, int stride, const float* __restrict__ z, int S, int64_t c0, int64_t n,
    const float* __restrict__ ein, const float* __restrict__ hin, const float* __restrict__ Wp,
    const float* __restrict__ bias, BnPrev prev, float momentum, float eps, float* __restrict__ hout,
    double* __restrict__ stats) {
  __shared__ double st[512];
  __shared__ __attribute__((aligned(16))) float al[256];
  __shared__ __attribute__((aligned(16))) float be[256];
  // per-wave output staging: 32 samples x 256 neurons, rows padded to 260 floats (conflict-free writes by
  // neuron, conflict-free 16-byte reads by sample)
  __shared__ __attribute__((aligned(16))) float stage[4][32 * LDS_ROW];
  for (int i = threadIdx.x; i < 512; i += blockDim.x) st[i] = 0.0;
  if (HP) bn_coeffs(prev, n, momentum, eps, al, be);
  __syncthreads();
  const int lane = threadIdx.x & 63, h = lane >> 5, wv = threadIdx.x >> 6;
  const int li = lane & 31;
  const int64_t ntiles = (n + 31) / 32;
  const int64_t tstride = (int64_t)gridDim.x * 4;
  const int64_t tile0 = (int64_t)blockIdx.x * 4 + wv;
  const f32x4* __restrict__ wh4 = reinterpret_cast<const f32x4*>(Wp + (EP ? SZ_E : 0)) + lane;
  HRing ring;
  if (HP && tile0 < ntiles)
    ring_fill(ring, reinterpret_cast<const f32x4*>(hin + tile0 * TILE_FLOATS) + lane, wh4, al, be, 4 * h);
  f32x4* prev_out = nullptr;  // previous tile's output, still staged in LDS
  for (int64_t tile = tile0; tile < ntiles; tile += tstride) {
    // opaque per-iteration offset: keeps the compiler from hoisting all of the layer's weight loads out of the
    // tile loop (an integer, not the pointer: a laundered pointer loses its global address space -> flat loads)
    int wofs = 0;
    asm volatile("" : "+s"(wofs));
    const float* wpt = Wp + wofs;
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
    float* lt = stage[wv];
    const float* lrow = lt + li * LDS_ROW + 4 * h;
    if (HP) {
      const int64_t nxt = tile + tstride < ntiles ? tile + tstride : tile;
      gemm_n_mem(acc, ring, reinterpret_cast<const f32x4*>(hin + tile * TILE_FLOATS) + lane,
                 reinterpret_cast<const f32x4*>(hin + nxt * TILE_FLOATS) + lane, wh4 + wofs, al, be, 4 * h,
                 prev_out, lrow);
      prev_out = nullptr;
    }
    if (prev_out) {  // EP-only layer: no k-group loop to hide the stores in
#pragma unroll
      for (int g = 0; g < 32; ++g) prev_out[g * 64] = *reinterpret_cast<const f32x4*>(lrow + 8 * g);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // epilogue: + bias -> LDS stage [sample][neuron]; statistics of (h - bias) over valid samples
    const int64_t base = tile * 32;
#pragma unroll
    for (int ob = 0; ob < 8; ++ob) {
      const int nn = 32 * ob + li;
      const float bo = bias[nn];
      float s1 = 0.0f, s2 = 0.0f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int s = (r & 3) + 8 * (r >> 2) + 4 * h;
        const float d = acc[ob][r];
        lt[s * LDS_ROW + nn] = d + bo;
        if (base + s < n) {
          s1 += d;
          s2 += d * d;
        }
      }
      atomicAdd(&st[2 * nn], (double)s1);
      atomicAdd(&st[2 * nn + 1], (double)s2);
    }
    // the raw h of this tile goes to the next layer's [g][lane][4] layout (1 KiB dwordx4 stores) during the
    // next tile's k-group loop, or below after the last tile
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    prev_out = reinterpret_cast<f32x4*>(hout + tile * TILE_FLOATS) + lane;
  }
  if (prev_out) {
    const float* lrow = stage[wv] + li * LDS_ROW + 4 * h;
#pragma unroll
    for (int g = 0; g < 32; ++g) prev_out[g * 64] = *reinterpret_cast<const f32x4*>(lrow + 8 * g);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 512; i += blockDim.x) atomicAdd(&stats[i], st[i]);
}

// occ_out on BatchNorm 8 (applied on load) + sigmoid; one wave per 32-sample tile.
__global__ __launch_bounds__(256) void k_train_out(const float* __restrict__ hin, int64_t n, BnPrev prev,
                                                   float momentum, float eps, const float* __restrict__ wout,
                                                   const float* __restrict__ bout, float* __restrict__ p_out) {
  __shared__ __attribute__((aligned(16))) float al[256];
  __shared__ __attribute__((aligned(16))) float be[256];
  bn_coeffs(prev, n, momentum, eps, al, be);
  __syncthreads();
  const int lane = threadIdx.x & 63, h = lane >> 5;
  const int64_t tile = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t ntiles = (n + 31) / 32;
  if (tile >= ntiles) return;
  const f32x4* x4 = reinterpret_cast<const f32x4*>(hin + tile * TILE_FLOATS) + lane;
  float part = 0.0f;
#pragma unroll 8
  for (int g = 0; g < 32; ++g) {
    const f32x4 x = x4[g * 64];
    const int f = 8 * g + 4 * h;
    const f32x4 w = *reinterpret_cast<const f32x4*>(wout + f);
    const f32x4 a = *reinterpret_cast<const f32x4*>(al + f);
    const f32x4 b = *reinterpret_cast<const f32x4*>(be + f);
#pragma unroll
    for (int q = 0; q < 4; ++q) part = fmaf(x[q] * a[q] + b[q], w[q], part);
  }
  const float logit = part + __shfl_xor(part, 32, 64) + bout[0];
  const int64_t s = tile * 32 + (lane & 31);
  if (lane < 32 && s < n) p_out[s] = sigmoid_ref(logit);
}

struct TrainWs {
  float* bufA;
  float* bufB;
  float* wp;
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
  const size_t ow = take(TRAIN_W_FLOATS * 4), ost = take(8 * 512 * 8);
  char* b = (char*)base;
  TrainWs w;
  w.bufA = (float*)(b + oA);
  w.bufB = (float*)(b + oB);
  w.wp = (float*)(b + ow);
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
  hipLaunchKernelGGL(k_pack_train, dim3((unsigned)((TRAIN_W_FLOATS + 255) / 256)), dim3(256), 0, s, P, ws.wp);
  for (int64_t c0 = 0; c0 < total; c0 += chunk) {
    const int64_t n = total - c0 < chunk ? total - c0 : chunk;
    const int64_t ntiles = (n + 31) / 32;
    const unsigned maxg = 256u * PCN_TRAIN_WAVES;
    const unsigned grid = (unsigned)(ntiles / 4 + 1 < maxg ? ntiles / 4 + 1 : maxg);
    const double dn = (double)n;
    PCN_HIP(hipMemsetAsync(ws.stats, 0, 8 * 512 * sizeof(double), s));
    float* hin = ws.bufA;
    float* hout = ws.bufB;
    {
      const BnPrev none{};
      ProfScope ps(s, PT_TRAIN_FIRST, 2.0 * 63 * 256 * dn, (4.0 + 1024.0) * dn);
      hipLaunchKernelGGL((k_train_layer<true, false>), dim3(grid), dim3(256), 0, s, rays, ray_stride, z, n_samples,
                         c0, n, ein, (const float*)nullptr, ws.wp + off_w(0, true), P.lin_b[0], none, momentum, eps,
                         hin, ws.stats);
    }
    for (int L = 1; L < 8; ++L) {
      const BnPrev prev{P.bn_w[L - 1], P.bn_b[L - 1], P.bn_rm[L - 1], P.bn_rv[L - 1], P.lin_b[L - 1],
                        ws.stats + 512 * (L - 1)};
      if (L == 4) {
        ProfScope ps(s, PT_TRAIN_SKIP, 2.0 * 319 * 256 * dn, (4.0 + 2048.0) * dn);
        hipLaunchKernelGGL((k_train_layer<true, true>), dim3(grid), dim3(256), 0, s, rays, ray_stride, z, n_samples,
                           c0, n, ein, hin, ws.wp + off_w(4, true), P.lin_b[L], prev, momentum, eps, hout,
                           ws.stats + 512 * L);
      } else {
        // algorithmic: 2*256*256 FLOP and 1 KiB in + 1 KiB out per sample
        ProfScope ps(s, PT_TRAIN_HIDDEN, 2.0 * 256 * 256 * dn, 2048.0 * dn);
        hipLaunchKernelGGL((k_train_layer<false, true>), dim3(grid), dim3(256), 0, s, rays, ray_stride, z,
                           n_samples, c0, n, ein, hin, ws.wp + off_w(L, false), P.lin_b[L], prev, momentum, eps,
                           hout, ws.stats + 512 * L);
      }
      float* t = hin;
      hin = hout;
      hout = t;
    }
    {
      const BnPrev prev{P.bn_w[7], P.bn_b[7], P.bn_rm[7], P.bn_rv[7], P.lin_b[7], ws.stats + 512 * 7};
      ProfScope ps(s, PT_TRAIN_OUT, 2.0 * 256 * dn, 1028.0 * dn);
      hipLaunchKernelGGL(k_train_out, dim3((unsigned)((ntiles + 3) / 4)), dim3(256), 0, s, hin, n, prev, momentum,
                         eps, P.out_w, P.out_b, p_out + c0);
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
