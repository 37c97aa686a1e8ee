// Train-mode NOF query: BatchNorm1d with batch statistics over each chunk of `chunk` flattened ray-major
// samples (nof/render.py:47-50 chunk loop; nn.BatchNorm1d train semantics; models.py:183-203), and its backward.
//
// Every BatchNorm needs the statistics of its whole chunk before the next Linear may run, so the network is
// evaluated layer by layer, one launch per Linear (k_train_ws), then k_train_out:
//   prologue: BatchNorm L-1's coefficients from the chunk statistics of h_{L-1}, alpha = gamma/sqrt(var+eps),
//             beta' = beta - mean*alpha (ATen's transform form; block 0 also updates running_mean/var with momentum
//             and the unbiased variance);
//   body:     h_L = W_L (alpha*h_{L-1} + beta') + b_L on MFMA, the BatchNorm applied while the input tile is
//             staged; h_L written raw (pre-BN) to HBM with per-neuron sums of (h - b) and (h - b)^2.
// The activations LeakyReLU(True) are identities (negative_slope == 1) and are not applied.
//
// Activation layout (HBM and LDS): tiles of 32 samples, [tile][g][lane][4] with lane = sample + 32 h holding
// features 8g + 4h + q (1 KiB per wave-instruction).  MFMA v_mfma_f32_32x32x2_f32 with samples on COLUMNS
// (D = W x^T): A (lane l) = W[neuron 32b + (l&31)][feature(t, l>>5)], B (lane l) = x[sample l&31][feature(t, l>>5)]
// (the tile's float4 itself), D (reg r, lane l) = out[neuron 32b + (r&3) + 8(r>>2) + 4(l>>5)][sample l&31], so
// registers 4j..4j+3 are the output tile's float4 at group 4b+j.  feature(t, h) = 8(t>>2) + 4h + (t&3).
#include <algorithm>
#include <array>
#include <cstring>
#include <string>
#include <type_traits>
#include <vector>

#include "common.h"
#include "pcnerf_internal.h"
#include "prof.h"

namespace pcn {

// Schedule constants (each measured against its alternatives in same-process A/Bs; DESIGN.md, git history):
constexpr int WS_XD_SKIP = 2;    // k_train_ws, skip layer: LDS read ring depth in k-groups
constexpr int WS_XD = 4;         // k_train_ws / k_dgrad_ws: LDS read ring depth in k-groups
constexpr int S12_COPIES = 8;    // k_wgrad_reduce: copies of the BatchNorm-backward sums (block m adds to copy m % COPIES)
// k_train_h: ring depth of B-operand reads (hidden / skip), k-step of the next tile's raw loads, staging k-steps
// counted from the end, k-step of the previous tile's epilogue, raw loads one tile ahead
constexpr int H_XD = 3, H_XD_SKIP = 2, H_LOAD = 2, H_STAGE = 4, H_EPI = 1, H_AHEAD = 1;
constexpr int H1_XD = H_XD;      // k_train_h1's B-operand read ring depth
// k_wgrad_b3 schedule (column blocks of a half tile): the block that reads the next half tile's A values (split two
// blocks later), the block of the first staging piece, the blocks between staging pieces
constexpr int WB3_AREAD = 3, WB3_STAGE = 0, WB3_SPACE = 2;

#ifndef PCN_RB_CLK
#define PCN_RB_CLK 0   // diagnostic builds: per-wave shader cycles of the layer-2 launch's phases (pcnerf_debug_rbclk)
#endif
#if PCN_RB_CLK
// [block * 8 + wave]: cycles summed over the tiles of: phase A (D: data-gradient MFMAs; W: remat), phase B (D:
// epilogue; W: weight-gradient MFMAs), the end-of-tile wait + barrier; the loop; the tile count
__device__ unsigned long long g_rbclk[4096][5];
#define RB_T(v) do { __builtin_amdgcn_sched_barrier(0); v = __builtin_amdgcn_s_memtime(); __builtin_amdgcn_sched_barrier(0); } while (0)
#else
#define RB_T(v) do { } while (0)
#endif
#ifndef PCN_CLOCK_STAMP
#define PCN_CLOCK_STAMP 0  // diagnostic builds only: phase stamps of 1 k_train_ws, 2 k_wgrad (pcnerf_debug_clock)
#endif
#if PCN_CLOCK_STAMP
// per workgroup: s_memrealtime (100 MHz, global) at entry / loop begin / loop end / exit (after its atomics
// completed), s_memtime (shader clock) at loop begin / end
__device__ unsigned long long g_clk[4096][6];
#define CLK_ENTRY unsigned long long clk_e = __builtin_amdgcn_s_memrealtime();
#define CLK_ON(k) (PCN_CLOCK_STAMP == (k))
#define CLK_BEGIN                                                   \
  unsigned long long clk_t0 = __builtin_amdgcn_s_memtime();         \
  unsigned long long clk_r0 = __builtin_amdgcn_s_memrealtime();
#define CLK_END                                                     \
  unsigned long long clk_t1 = __builtin_amdgcn_s_memtime();         \
  unsigned long long clk_r1 = __builtin_amdgcn_s_memrealtime();
#define CLK_EXIT(k)                                                               \
  __builtin_amdgcn_s_waitcnt(0);                                                  \
  if (CLK_ON(k) && threadIdx.x == 0 && blockIdx.x < 4096) {                       \
    unsigned long long* g = g_clk[blockIdx.x];                                    \
    g[0] = clk_e; g[1] = clk_r0; g[2] = clk_r1; g[3] = __builtin_amdgcn_s_memrealtime(); \
    g[4] = clk_t0; g[5] = clk_t1;                                                 \
  }
#else
#define CLK_ENTRY
#define CLK_BEGIN
#define CLK_END
#define CLK_EXIT(k)
#define CLK_ON(k) 0
#endif

constexpr int KG_E = 8, KG_H = 32;
constexpr size_t SZ_E = (size_t)KG_E * 8 * 64 * 4;
constexpr size_t SZ_H = (size_t)KG_H * 8 * 64 * 4;
constexpr size_t TILE_FLOATS = 32 * 256;
constexpr int LDS_ROW = 260;

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
  if (blockIdx.x == 0 && B.rm) {  // (the backward's forward recomputation passes no running stats)
    const double mom = (double)momentum;
    B.rm[k] = (float)(mom * mean + (1.0 - mom) * (double)B.rm[k]);
    const double unb = n > 1 ? var * (double)n / (double)(n - 1) : var;
    B.rv[k] = (float)(mom * unb + (1.0 - mom) * (double)B.rv[k]);
  }
}


// Encoding feature group g (features 8g + 4h + q, q = 0..3) of a sample at p for lane half h: Embedding(3, 10) as
// in encode_half (2^k * x exact, full-range sincosf), computed per feature so one thread stages one float4.
__device__ __forceinline__ f32x4 enc_feats(const float (&p)[3], int h, int g) {
  f32x4 e;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int f = 8 * g + 4 * h + q;
    const int fk = f < 3 ? 0 : (f - 3) / 6, fr = f < 3 ? 0 : (f - 3) - 6 * fk;
    const int m = fr < 3 ? fr : fr - 3;
    const float pm = m == 0 ? p[0] : m == 1 ? p[1] : p[2];
    float sn, cs;
    sincosf(__int_as_float((127 + fk) << 23) * pm, &sn, &cs);   // (float)(1 << fk) * p[m]
    const float pf = f == 0 ? p[0] : f == 1 ? p[1] : p[2];
    e[q] = f < 3 ? pf : f >= 63 ? 0.0f : fr < 3 ? sn : cs;
  }
  return e;
}

// The same group from a stored (., 63) embedding row.
__device__ __forceinline__ f32x4 enc_feats_row(const float* __restrict__ row, int h, int g) {
  f32x4 e;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int f = 8 * g + 4 * h + q;
    e[q] = f < 63 ? row[f] : 0.0f;
  }
  return e;
}

// ---- k_train_ws<KE, HP>: weight-stationary train-mode Linear, samples on COLUMNS (D = W x^T).
//   KE = 8: the 63 (+1 pad) encoding features are input k-groups 0..7 (computed from positions, or read from
//   `ein`); HP: the 256 BatchNorm'd features of the previous layer are k-groups KE..KE+31.  Instances: first
//   layer <8,false> (63 -> 256), hidden layers <0,true> (256 -> 256), skip layer 5 <8,true> ([e, h4] 319 -> 256).
// A workgroup of 8 waves (two per SIMD) computes all 256 neurons of one 32-sample tile at a time; wave b owns
// neurons 32b..32b+31, whose weights are its MFMA A operand, loaded ONCE per launch into registers (the packed
// B-operand image of the samples-on-rows kernels has exactly the per-lane content the A operand of the
// transposed product wants).  The B operand is the input tile's [g][lane][4] float4 itself, staged once per
// workgroup in LDS (double buffered; previous BatchNorm applied while staging; encoding groups computed while
// staging, one float4 per thread).  In this orientation accumulator registers 4j..4j+3 of wave b ARE the output
// tile's float4 at group 4b+j, so the raw h goes to HBM straight from registers (no LDS transpose), and each lane
// owns one sample: the per-neuron statistics are per-lane running sums (kept in an LDS slot of the lane's own)
// across all the workgroup's tiles, reduced across lanes once at the end -- one coalesced float64 atomic per
// (neuron, moment) and workgroup.  No weight traffic inside the tile loop at all.
// Software pipeline over tiles: tile t's MFMAs run into one accumulator set while the other set's epilogue (tile
// t-1: + bias, statistics, 4 x 1 KiB stores) goes out at k-groups 1-2 and tile t+1's input is staged into the
// other LDS buffer (activation loads at k-group 3, BatchNorm'd at KGT-10/KGT-9; ray rows loaded at k-group KGT-8
// (first layer: 0), encoding computed at the last k-group), so the only thing left between two tiles' MFMA
// streams is the barrier.
// Hidden layer: 265 us per chunk of 262,144 samples (the previous samples-on-rows kernel: 299 us); one wave per
// SIMD owning 64 neurons measured 295 us.
template <int KE, bool HP>
__global__ __launch_bounds__(512, 1) void k_train_ws(const float* __restrict__ rays, int stride,
                                                     const float* __restrict__ z, int S, int64_t c0,
                                                     const float* __restrict__ ein, const float* __restrict__ hin,
                                                     int64_t n, const float* __restrict__ Wp,
                                                     const float* __restrict__ bias, BnPrev prev, float momentum,
                                                     float eps, float* __restrict__ hout,
                                                     double* __restrict__ stats,
                                                     const f32x4* __restrict__ etin, f32x4* __restrict__ etout) {
  // etout (first layer): every tile's encoding float4s, [tile][g 0..7][lane] (8 KiB per tile), as staged;
  // etin (skip layer): the same tiles read back instead of recomputing the sincosf from the ray rows (every
  // caller runs the first layer of the chunk before its skip layer with the same buffer)
  constexpr bool ETIN = KE && HP, ETOUT = KE && !HP;
  constexpr int KGT = KE + (HP ? KG_H : 0);
  constexpr int XD = (KE && HP) ? WS_XD_SKIP : WS_XD;   // the skip layer's 160 weight registers leave less
  __shared__ __attribute__((aligned(16))) float al[256];
  __shared__ __attribute__((aligned(16))) float be[256];
  __shared__ __attribute__((aligned(16))) float bs[256];
  __shared__ f32x4 xs[2][KGT * 64];
  // per-lane running statistics (its sample's d and d^2 summed over the launch's tiles) for the wave's 16
  // neurons of its half: [wave][lane][8 float4 chunks], chunk 2j = sum d, 2j+1 = sum d^2 of registers 4j..4j+3,
  // stored at position chunk ^ ((lane >> 1) & 7) (conflict-free 16-byte accesses)
  __shared__ f32x4 sred[8 * 64 * 8];   // 64 KiB
  CLK_ENTRY
  const int t = threadIdx.x;
  if (t < 256) {
    if (HP) bn_coeffs(prev, n, momentum, eps, al, be);
    bs[t] = bias[t];
  }
  const int nt = (int)((n + 31) / 32);
  const int gstride = (int)gridDim.x;
  const int lane = t & 63, h = lane >> 5, li = lane & 31;
  const int blk = __builtin_amdgcn_readfirstlane(t >> 6);
  f32x4 wr[KGT];
  {
    const f32x4* __restrict__ w4 = reinterpret_cast<const f32x4*>(Wp) + lane;
#pragma unroll
    for (int kg = 0; kg < KGT; ++kg) wr[kg] = w4[(kg * 8 + blk) * 64];
  }
  f32x4* const my_st = sred + (blk * 64 + lane) * 8;
  const int st_sw = (lane >> 1) & 7;
#pragma unroll
  for (int c = 0; c < 8; ++c) my_st[c] = f32x4{};
  __syncthreads();
  // all weights resident before the tile loop: otherwise the waitcnt pass cannot tell them from the loop's own
  // loads and waits on the next tile's activations inside the k-loop
  __builtin_amdgcn_s_waitcnt(0);
  int buf = 0;
  // staging: thread t owns the activation float4s t + 512 m (m = 0..3) of a tile: group KE + (t >> 6) + 8 m,
  // lane t & 63; and (KE) the encoding float4 of group t >> 6, lane t & 63
  auto stage = [&](int b, const f32x4 (&v)[4], int m) {
    const int g = (t >> 6) + 8 * m;
    const f32x4 a = *reinterpret_cast<const f32x4*>(al + 8 * g + 4 * h);
    const f32x4 c = *reinterpret_cast<const f32x4*>(be + 8 * g + 4 * h);
    f32x4 x;
#pragma unroll
    for (int q = 0; q < 4; ++q) x[q] = v[m][q] * a[q] + c[q];
    xs[b][KE * 64 + t + 512 * m] = x;
  };
  auto sample_of = [&](int tile) {
    int64_t sl = (int64_t)tile * 32 + li;
    if (sl >= n) sl = n - 1;
    return c0 + sl;
  };
  int tl = __builtin_amdgcn_readfirstlane((int)blockIdx.x);
  if (tl < nt) {
    if (HP) {
      f32x4 v[4];
#pragma unroll
      for (int m = 0; m < 4; ++m)
        v[m] = reinterpret_cast<const f32x4*>(hin + (size_t)tl * TILE_FLOATS + (size_t)m * 2048)[t];
#pragma unroll
      for (int m = 0; m < 4; ++m) stage(0, v, m);
    }
    if (KE) {
      const int64_t gs = sample_of(tl);
      f32x4 e;
      if (ETIN) {
        e = etin[(size_t)tl * 512 + t];
      } else if (ein) {
        e = enc_feats_row(ein + gs * 63, h, t >> 6);
      } else {
        float p[3];
        sample_point(rays + ray_of(gs, S) * stride, z[gs], p);
        e = enc_feats(p, h, t >> 6);
      }
      xs[0][t] = e;
      if (ETOUT) etout[(size_t)tl * 512 + t] = e;
    }
  }
  __syncthreads();
  CLK_BEGIN
  auto epi = [&](const f32x16& pacc, int ptile, int j) {
    const bool valid = (int64_t)ptile * 32 + li < n;
    const f32x4 bj = *reinterpret_cast<const f32x4*>(bs + 32 * blk + 8 * j + 4 * h);
    f32x4 s1 = my_st[(2 * j) ^ st_sw], s2 = my_st[(2 * j + 1) ^ st_sw];
    f32x4 o;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float d = pacc[4 * j + q];
      o[q] = d + bj[q];
      const float dv = valid ? d : 0.0f;
      s1[q] += dv;
      s2[q] += dv * dv;
    }
    my_st[(2 * j) ^ st_sw] = s1;
    my_st[(2 * j + 1) ^ st_sw] = s2;
    float* base = hout + (size_t)ptile * TILE_FLOATS + (size_t)(4 * blk + j) * 256;
    reinterpret_cast<f32x4*>(base)[lane] = o;
  };
  auto body = [&](f32x16& acc, const f32x16& pacc, int tile, int ptile) {
    const int nxt = __builtin_amdgcn_readfirstlane(tile + gstride);
    const bool more = nxt < nt;
    const f32x4* xb = &xs[buf][lane];
    f32x4 xr[XD];
    f32x4 v[4];    // HP: the next tile's raw activations, k-groups 3 to KGT-9 only
    float rr[7];   // KE: the next tile's ray origin/direction and z for this lane's sample (last 8 k-groups)
    f32x4 ev;      // ETIN: the next tile's stored encoding float4
#pragma unroll
    for (int d = 0; d < XD - 1; ++d) xr[d] = xb[d * 64];
#pragma unroll
    for (int kg = 0; kg < KGT; ++kg) {
      if (kg + XD - 1 < KGT) xr[(kg + XD - 1) % XD] = xb[(kg + XD - 1) * 64];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const f32x16 c = (kg == 0 && q == 0) ? f32x16{} : acc;
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(wr[kg][q], xr[kg % XD][q], c, 0, 0, 0);
      }
      if (ETIN && kg == KGT - 8 && more) ev = etin[(size_t)nxt * 512 + t];
      if (ETOUT && kg == 0 && more && !ein) {   // after the activations' registers are free
        const int64_t gs = sample_of(nxt);
        const float* r = rays + ray_of(gs, S) * stride;
#pragma unroll
        for (int c = 0; c < 6; ++c) rr[c] = r[c];
        rr[6] = z[gs];
      }
      if (kg == 1 && ptile >= 0) {
        epi(pacc, ptile, 0);
        epi(pacc, ptile, 1);
      }
      if (kg == 2 && ptile >= 0) {
        epi(pacc, ptile, 2);
        epi(pacc, ptile, 3);
      }
      if (HP && kg == 3 && more) {
#pragma unroll
        for (int m = 0; m < 4; ++m)
          v[m] = reinterpret_cast<const f32x4*>(hin + (size_t)nxt * TILE_FLOATS + (size_t)m * 2048)[t];
      }
      if (HP && kg == KGT - 10 && more) {
        stage(buf ^ 1, v, 0);
        stage(buf ^ 1, v, 1);
      }
      if (HP && kg == KGT - 9 && more) {
        stage(buf ^ 1, v, 2);
        stage(buf ^ 1, v, 3);
      }
      if (KE && kg == KGT - 1 && more) {
        f32x4 e;
        if (ETIN) {
          e = ev;
        } else if (ein) {
          e = enc_feats_row(ein + sample_of(nxt) * 63, h, t >> 6);
        } else {   // sample_point on the prefetched ray row
          float p[3];
#pragma unroll
          for (int c = 0; c < 3; ++c) p[c] = rr[c] + rr[3 + c] * rr[6];
          e = enc_feats(p, h, t >> 6);
        }
        xs[buf ^ 1][t] = e;
        if (ETOUT) etout[(size_t)nxt * 512 + t] = e;
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    __syncthreads();
    buf ^= 1;
  };
  f32x16 accA, accB;
  int ptile = -1;
  while (tl < nt) {
    body(accA, accB, tl, ptile);
    ptile = tl;
    tl = __builtin_amdgcn_readfirstlane(tl + gstride);
    if (tl >= nt) {
#pragma unroll
      for (int j = 0; j < 4; ++j) epi(accA, ptile, j);
      break;
    }
    body(accB, accA, tl, ptile);
    ptile = tl;
    tl = __builtin_amdgcn_readfirstlane(tl + gstride);
    if (tl >= nt) {
#pragma unroll
      for (int j = 0; j < 4; ++j) epi(accB, ptile, j);
    }
  }
  CLK_END
  // per-neuron sums, once per launch: thread t = 2 n + moment sums its (neuron, moment) over the 32 lanes of the
  // half that holds neuron n, in float64, and adds it with one coalesced atomic
  __syncthreads();
  {
    const int nn = t >> 1, mo = t & 1, ib = nn & 31, wb = nn >> 5;
    const int hh = (ib >> 2) & 1, jj = ib >> 3, qq = ib & 3;
    double a = 0.0;
#pragma unroll 8
    for (int l = 0; l < 32; ++l) {
      const int ln = 32 * hh + l;
      a += (double)sred[(wb * 64 + ln) * 8 + ((2 * jj + mo) ^ ((ln >> 1) & 7))][qq];
    }
    atomicAdd(&stats[t], a);
  }
  CLK_EXIT(1)
}

// ---- k_train_h<KE, HP>: k_train_ws with the fp32 products taken on the fp16 matrix pipe (opt-in,
// pcnerf_set_train_math(1)).  Each fp32 operand is split into two fp16 parts, v = hi + mid (hi = fp16(v),
// mid = fp16(v - hi): 22 significant bits, relative representation error <= 2^-23), and
// W x = Wh xh + Wh xm + Wm xh (+ Wm xm when NT == 4) on v_mfma_f32_32x32x16_f16: every fp16 x fp16 product is
// exact in the fp32 accumulator, so the only departures from an fp32 FMA chain are the operands' 2^-23
// representation error and the dropped term(s) (Wm xm ~ 2^-22 relative, NT == 3).  Power-of-two scales keep
// the mid parts out of the fp16 subnormal range and the operands below 2^15: the packed weights of layer L carry
// 2^sw[L] (max |W| 2^sw in [2^14, 2^15)), the staged activations 2^sx with sx chosen per launch from the
// BatchNorm's own bound |x| <= sqrt(n) |gamma| + |beta| (Samuelson: no sample lies more than sqrt(n-1) standard
// deviations from its chunk mean); the epilogue multiplies by 2^-(sw+sx) (exact).
// Same tiles, layouts, statistics and pipeline as k_train_ws; the B operand (the staged tile) lives in LDS as
// [k-step s][part][lane][8 halves], lane = sample + 32 (G & 1) holding features 16 s + 8 (G & 1) + 0..7 of 16-byte
// feature group G = 2 s + (G & 1).
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));

constexpr int KS_E = 4, KS_H = 16;   // k-steps of 16 features: encoding (64 incl. pad), hidden (256)
constexpr size_t HW_E = (size_t)KS_E * 8 * 2 * 64;   // f16x8 per encoding part of a layer's image
constexpr size_t HW_H = (size_t)KS_H * 8 * 2 * 64;
// layer images in f16x8 units: [k-step][out-block 8][part 2][lane 64]
__host__ __device__ constexpr size_t off_h(int layer, bool epart) {
  return layer == 0 ? 0
       : layer <= 3 ? HW_E + (size_t)(layer - 1) * HW_H
       : layer == 4 ? (epart ? HW_E + 3 * HW_H : 2 * HW_E + 3 * HW_H)
                    : 2 * HW_E + (size_t)(layer - 1) * HW_H;
}
constexpr size_t TRAIN_H_VECS = 2 * HW_E + 7 * HW_H;

// per-layer weight scale exponents: sw[L] with max|W_L| 2^sw in [2^14, 2^15); grid 8, 1024 threads
__global__ __launch_bounds__(1024) void k_wscale(NofParamsDev P, int* __restrict__ sw) {
  const int L = blockIdx.x;
  const float m = block_layer_absmax<1024>(P.lin_w[L], 256, L == 0 ? 63 : L == 4 ? 319 : 256, [](int) { return 1.0f; });
  if (threadIdx.x == 0) sw[L] = m > 0.0f && m == m && m < 3.0e38f ? 14 - ilogbf(m) : 0;
}

__global__ void k_pack_train_h(NofParamsDev P, const int* __restrict__ sw, f16x8* __restrict__ out) {
  const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= TRAIN_H_VECS) return;
  int layer;
  bool epart;
  size_t base;
  if (idx < HW_E) { layer = 0; epart = true; base = 0; }
  else if (idx < HW_E + 3 * HW_H) { layer = 1 + (int)((idx - HW_E) / HW_H); epart = false; base = off_h(layer, false); }
  else if (idx < 2 * HW_E + 3 * HW_H) { layer = 4; epart = true; base = off_h(4, true); }
  else if (idx < 2 * HW_E + 4 * HW_H) { layer = 4; epart = false; base = off_h(4, false); }
  else { layer = 5 + (int)((idx - (2 * HW_E + 4 * HW_H)) / HW_H); epart = false; base = off_h(layer, false); }
  const size_t j = idx - base;
  const int lane = (int)(j & 63), part = (int)((j >> 6) & 1), ob = (int)((j >> 7) & 7), ks = (int)(j >> 10);
  const int nn = 32 * ob + (lane & 31);
  const int in_f = layer == 0 ? 63 : layer == 4 ? 319 : 256;
  const float sc = ldexpf(1.0f, sw[layer]);
  f16x8 v;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int f = 16 * ks + 8 * (lane >> 5) + e;
    int col;
    if (epart) col = f < 63 ? f : -1;
    else col = (layer == 4 ? 63 : 0) + f;
    const float w = col < 0 ? 0.0f : P.lin_w[layer][(size_t)nn * in_f + col] * sc;
    const _Float16 hi = (_Float16)w;
    v[e] = part == 0 ? hi : (_Float16)(w - (float)hi);
  }
  out[idx] = v;
}

// hi / mid halves of 4 scaled fp32 values
__device__ __forceinline__ void split4(const f32x4& x, f16x4& hi, f16x4& mid) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const _Float16 a = (_Float16)x[q];
    hi[q] = a;
    mid[q] = (_Float16)(x[q] - (float)a);
  }
}

template <int KE, bool HP, int NT>
// hin / hout are NOT restrict-qualified: the split forward without activation store runs every layer in place
// (hin == hout, query_train's in-place forward)
__global__ __launch_bounds__(512, 1) void k_train_h(const float* __restrict__ rays, int stride,
                                                    const float* __restrict__ z, int S, int64_t c0,
                                                    const float* __restrict__ ein, const float* hin,
                                                    int64_t n, const f16x8* __restrict__ Wp, const int* __restrict__ swp,
                                                    int layer, const float* __restrict__ bias, BnPrev prev,
                                                    float momentum, float eps, float* hout,
                                                    double* __restrict__ stats, const f32x4* __restrict__ etin,
                                                    f32x4* __restrict__ etout) {
  constexpr bool ETIN = KE && HP, ETOUT = KE && !HP;
  constexpr int KSE = KE ? KS_E : 0;               // encoding k-steps
  constexpr int KS = KSE + (HP ? KS_H : 0);        // k-steps of 16 features
  constexpr int XD = (KE && HP) ? H_XD_SKIP : H_XD;   // LDS read ring depth in k-steps
  // HP: the next tile's raw loads, their staging (BatchNorm + split + LDS), the previous tile's epilogue
  constexpr int S_LOAD = H_LOAD, S_STAGE0 = KS - H_STAGE, S_STAGE1 = S_STAGE0 + 1;
  constexpr int S_EPI = H_EPI;
  constexpr int AHEAD = (KE && HP) ? 1 : H_AHEAD;   // the skip layer's weight registers leave no room
  // REGSTAT: each tile's epilogue right after its MFMAs, the per-lane running statistics in registers (no LDS
  // read-modify-write per tile, one accumulator set); the B buffers double as the final reduction area
  // WENC (skip layer): the encoding k-steps' weights live in LDS, read two k-steps ahead, instead of 32 registers --
  // which lets the skip layer take the REGSTAT form as well
  constexpr bool WENC = KE && HP;   // skip layer: encoding weights in LDS
  constexpr bool REGSTAT = HP;      // running statistics in registers, epilogue after each tile's MFMAs
  // NWL: k-steps whose weights come from LDS (two k-steps ahead) -- the skip layer's encoding k-steps (WENC)
  constexpr int NWL = WENC ? KSE : 0;
  constexpr int NBUF = 2;
  __shared__ __attribute__((aligned(16))) float al[256];
  __shared__ __attribute__((aligned(16))) float be[256];
  __shared__ __attribute__((aligned(16))) float bs[256];
  __shared__ float smax[8];
  __shared__ f16x8 xs[NBUF][KS][2][64];
  __shared__ f32x4 sred_[REGSTAT ? 1 : 8 * 64 * 8];   // per-lane running statistics, as k_train_ws
  __shared__ f16x8 wenc_[NWL ? NWL * 8 * 2 * 64 : 1];
  static_assert(!REGSTAT || sizeof(xs) >= 8 * 64 * 8 * sizeof(f32x4), "reduction area");
  f32x4* const sred = REGSTAT ? reinterpret_cast<f32x4*>(&xs[0][0][0][0]) : sred_;
  const int t = threadIdx.x;
  if (t < 256) {
    if (HP) bn_coeffs(prev, n, momentum, eps, al, be);
    bs[t] = bias[t];
  }
  // activation scale 2^sx: the largest power of two keeping sqrt(n) |gamma| + |beta| below 2^15 (never above
  // 2^0 for the skip layer, whose encoding part is not scaled)
  int sx = 0;
  if (HP) {
    float bnd = 0.0f;
    if (t < 256) bnd = sqrtf((float)n) * fabsf(prev.gamma[t]) + fabsf(prev.beta[t]);
    bnd = wave_max_f(bnd);
    if ((t & 63) == 0) smax[t >> 6] = bnd;
    __syncthreads();
    float m = smax[0];
#pragma unroll
    for (int i = 1; i < 8; ++i) m = fmaxf(m, smax[i]);
    sx = (m > 0.0f && m < 3.0e38f) ? 14 - ilogbf(m) : 0;
    if (KE && sx > 0) sx = 0;
    sx = sx > 24 ? 24 : sx;
    if (t < 256) {   // 2^sx into the BatchNorm coefficients (exact: a power of two)
      al[t] = ldexpf(al[t], sx);
      be[t] = ldexpf(be[t], sx);
    }
  }
  const float xscale = ldexpf(1.0f, sx);
  const float unscale = ldexpf(1.0f, -(swp[layer & 255] + sx));
  const int nt = (int)((n + 31) / 32);
  const int gstride = (int)gridDim.x;
  // tile order: odd layers walk the chunk backwards, so a layer first reads the tiles its predecessor wrote last
  // (still in the memory-side cache) -- P maps the loop's tile to the tile of the chunk
  const bool rev = !KE && ((layer >> 8) & 1);   // (the first and skip layers keep the forward walk: registers)
  auto P = [&](int x) { return rev ? nt - 1 - x : x; };
  const int lane = t & 63, h = lane >> 5, li = lane & 31;
  // staging identity: the HBM lane (sample ls + 32 hs) whose float4s this thread stages
  const int sln = lane, ls = sln & 31, hs = sln >> 5;
  const int blk = __builtin_amdgcn_readfirstlane(t >> 6);
  if (blk >= 4) __builtin_amdgcn_s_setprio(1);   // MI355X_MICROARCH two-waves item 4
  f16x8 wr[KS][2];
  {
    const f16x8* __restrict__ w8 = Wp + lane;
#pragma unroll
    for (int ks = NWL; ks < KS; ++ks)
#pragma unroll
      for (int p = 0; p < 2; ++p) wr[ks][p] = w8[((ks * 8 + blk) * 2 + p) * 64];
    if (NWL)
      for (int j = t; j < NWL * 8 * 2 * 64; j += 512) wenc_[j] = Wp[j];
  }
  auto wenc = [&](int ks, int p) { return wenc_[((ks * 8 + blk) * 2 + p) * 64 + lane]; };
  f32x4* const my_st = sred + (blk * 64 + lane) * 8;
  const int st_sw = (lane >> 1) & 7;
  f32x4 rs[8];   // REGSTAT: chunk 2j = sum d, 2j+1 = sum d^2 of accumulator registers 4j..4j+3
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    rs[c] = f32x4{};
    if (!REGSTAT) my_st[c] = f32x4{};
  }
  __syncthreads();
  __builtin_amdgcn_s_waitcnt(0);
  int buf = 0;
  // staging: thread t owns the activation float4s t + 512 m (m = 0..3) of a tile: feature group G = KE + (t >> 6)
  // + 8 m, lane t & 63 (sample li, half h) -> LDS [s = G >> 1][part][li + 32 (G & 1)][4 h .. 4 h + 3]
  auto put = [&](int b, int G, const f32x4& x) {
    f16x4 hi, mid;
    split4(x, hi, mid);
    const int s = G >> 1, ln = ls + 32 * (G & 1);
    *reinterpret_cast<f16x4*>(reinterpret_cast<_Float16*>(&xs[b][s][0][ln]) + 4 * hs) = hi;
    *reinterpret_cast<f16x4*>(reinterpret_cast<_Float16*>(&xs[b][s][1][ln]) + 4 * hs) = mid;
  };
  auto stage = [&](int b, const f32x4 (&v)[4], int m) {
    const int g = (t >> 6) + 8 * m;
    const f32x4 a = *reinterpret_cast<const f32x4*>(al + 8 * g + 4 * hs);
    const f32x4 c = *reinterpret_cast<const f32x4*>(be + 8 * g + 4 * hs);
    f32x4 x;
#pragma unroll
    for (int q = 0; q < 4; ++q) x[q] = v[m][q] * a[q] + c[q];
    put(b, KE + g, x);
  };
  auto put_enc = [&](int b, const f32x4& e) {   // encoding group t >> 6 (not scaled: sx <= 0 -> x 2^sx only if < 1)
    f32x4 x = e;
    if (sx != 0) {
#pragma unroll
      for (int q = 0; q < 4; ++q) x[q] *= xscale;
    }
    put(b, t >> 6, x);
  };
  // the raw activation float4s of a tile this thread stages ([g][HBM lane][4], g = (t >> 6) + 8 m)
  auto load_tile = [&](f32x4 (&v)[4], int tile) {
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const f32x4* src = reinterpret_cast<const f32x4*>(hin + (size_t)P(tile) * TILE_FLOATS) + (t & ~63) + sln + 512 * m;
      v[m] = *src;
    }
  };
  const int etix = (t & ~63) + sln;   // this thread's encoding float4 in a stored tile [g][HBM lane]
  auto sample_of = [&](int tile) {
    int64_t sl = (int64_t)P(tile) * 32 + ls;
    if (sl >= n) sl = n - 1;
    return c0 + sl;
  };
  int tl = __builtin_amdgcn_readfirstlane((int)blockIdx.x);
  if (tl < nt) {
    if (HP) {
      f32x4 v[4];
      load_tile(v, tl);
#pragma unroll
      for (int m = 0; m < 4; ++m) stage(0, v, m);
    }
    if (KE) {
      const int64_t gs = sample_of(tl);
      f32x4 e;
      if (ETIN) {
        e = etin[(size_t)P(tl) * 512 + etix];
      } else if (ein) {
        e = enc_feats_row(ein + gs * 63, hs, t >> 6);
      } else {
        float p[3];
        sample_point(rays + ray_of(gs, S) * stride, z[gs], p);
        e = enc_feats(p, hs, t >> 6);
      }
      put_enc(0, e);
      if (ETOUT) etout[(size_t)P(tl) * 512 + etix] = e;
    }
  }
  __syncthreads();
  auto epi = [&](const f32x16& pacc, int ptile_l, int j) {
    const int ptile = P(ptile_l);
    const bool valid = (int64_t)ptile * 32 + li < n;
    const f32x4 bj = *reinterpret_cast<const f32x4*>(bs + 32 * blk + 8 * j + 4 * h);
    f32x4 s1 = my_st[(2 * j) ^ st_sw], s2 = my_st[(2 * j + 1) ^ st_sw];
    f32x4 o;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float d = pacc[4 * j + q] * unscale;
      o[q] = d + bj[q];
      const float dv = valid ? d : 0.0f;
      s1[q] += dv;
      s2[q] += dv * dv;
    }
    my_st[(2 * j) ^ st_sw] = s1;
    my_st[(2 * j + 1) ^ st_sw] = s2;
    if (hout) {   // (the first layer runs statistics-only when k_train_h1 recomputes its output)
      float* base = hout + (size_t)ptile * TILE_FLOATS + (size_t)(4 * blk + j) * 256;
      reinterpret_cast<f32x4*>(base)[lane] = o;
    }
  };
  // AHEAD == 2: the raw loads run two tiles ahead (vload gets tile + 2 gstride while vstage, loaded one
  // tile earlier, is staged for tile + gstride); == 1: loaded and staged within the same tile
  auto epir = [&](const f32x16& acc, int tile_l, int j) {   // REGSTAT epilogue
    const int tile = P(tile_l);
    const bool valid = (int64_t)tile * 32 + li < n;
    const f32x4 bj = *reinterpret_cast<const f32x4*>(bs + 32 * blk + 8 * j + 4 * h);
    f32x4 o;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float d = acc[4 * j + q] * unscale;
      o[q] = d + bj[q];
      const float dv = valid ? d : 0.0f;
      rs[2 * j][q] += dv;
      rs[2 * j + 1][q] += dv * dv;
    }
    float* base = hout + (size_t)tile * TILE_FLOATS + (size_t)(4 * blk + j) * 256;
    reinterpret_cast<f32x4*>(base)[lane] = o;
  };
  auto body = [&](f32x16& acc, const f32x16& pacc, int tile, int ptile, f32x4 (&vstage)[4], f32x4 (&vload)[4],
                  bool sync) {
    const int nxt = __builtin_amdgcn_readfirstlane(tile + gstride);
    const bool more = nxt < nt;
    const int nxt2 = __builtin_amdgcn_readfirstlane(tile + 2 * gstride);
    const int bnext = buf ^ 1;   // the buffer this tile stages into
    const int tst = nxt;         // ... for this tile
    const bool mst = tst < nt;
    f16x8 xr[XD][2];
    f32x4 vloc[4];   // AHEAD == 1: this tile's loads of the next tile
    float rr[7];
    f32x4 ev;
    f16x8 we[2][2];   // NWL: weights of LDS k-steps ks, ks + 1
    if (NWL) {
#pragma unroll
      for (int d = 0; d < 2; ++d)
#pragma unroll
        for (int p = 0; p < 2; ++p) we[d][p] = wenc(d, p);
    }
#pragma unroll
    for (int d = 0; d < XD - 1; ++d) {
      xr[d][0] = xs[buf][d][0][lane];
      xr[d][1] = xs[buf][d][1][lane];
    }
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      if (ks + XD - 1 < KS) {
        xr[(ks + XD - 1) % XD][0] = xs[buf][ks + XD - 1][0][lane];
        xr[(ks + XD - 1) % XD][1] = xs[buf][ks + XD - 1][1][lane];
      }
      const f16x8 xh = xr[ks % XD][0], xm = xr[ks % XD][1];
      const bool wl = ks < NWL;
      const f16x8 w0 = wl ? we[ks & 1][0] : wr[ks][0], w1 = wl ? we[ks & 1][1] : wr[ks][1];
      acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(w0, xh, ks == 0 ? f32x16{} : acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(w0, xm, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(w1, xh, acc, 0, 0, 0);
      if (NT == 4) acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(w1, xm, acc, 0, 0, 0);
      if (ks + 2 < NWL) {
        we[ks & 1][0] = wenc(ks + 2, 0);
        we[ks & 1][1] = wenc(ks + 2, 1);
      }
      if (ETIN && ks == KS - 4 && more) ev = etin[(size_t)P(nxt) * 512 + etix];
      if (ETOUT && ks == 0 && more && !ein) {
        const int64_t gs = sample_of(nxt);
        const float* r = rays + ray_of(gs, S) * stride;
#pragma unroll
        for (int c = 0; c < 6; ++c) rr[c] = r[c];
        rr[6] = z[gs];
      }
      if (!REGSTAT && ks == S_EPI && ptile >= 0) {
        epi(pacc, ptile, 0);
        epi(pacc, ptile, 1);
      }
      if (!REGSTAT && ks == S_EPI + 1 && ptile >= 0) {
        epi(pacc, ptile, 2);
        epi(pacc, ptile, 3);
      }
      if constexpr (HP && AHEAD == 2) {
        if (ks == S_LOAD && nxt2 < nt) load_tile(vload, nxt2);
        if (ks == S_STAGE0 && more) {
          stage(buf ^ 1, vstage, 0);
          stage(buf ^ 1, vstage, 1);
        }
        if (ks == S_STAGE1 && more) {
          stage(buf ^ 1, vstage, 2);
          stage(buf ^ 1, vstage, 3);
        }
      } else if constexpr (HP) {
        if (ks == S_LOAD && mst) load_tile(vloc, tst);
        if (ks == S_STAGE0 && mst) {
          stage(bnext, vloc, 0);
          stage(bnext, vloc, 1);
        }
        if (ks == S_STAGE1 && mst) {
          stage(bnext, vloc, 2);
          stage(bnext, vloc, 3);
        }
      }
      if (KE && ks == KS - 1 && more) {
        f32x4 e;
        if (ETIN) {
          e = ev;
        } else if (ein) {
          e = enc_feats_row(ein + sample_of(nxt) * 63, hs, t >> 6);
        } else {
          float p[3];
#pragma unroll
          for (int c = 0; c < 3; ++c) p[c] = rr[c] + rr[3 + c] * rr[6];
          e = enc_feats(p, hs, t >> 6);
        }
        put_enc(buf ^ 1, e);
        if (ETOUT) etout[(size_t)P(nxt) * 512 + etix] = e;
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    if (REGSTAT) {
#pragma unroll
      for (int j = 0; j < 4; ++j) epir(acc, tile, j);
    }
    if (sync) __syncthreads();
    buf ^= 1;
  };
  f32x16 accA, accB;
  f32x4 vA[4], vB[4];
  if (HP && AHEAD == 2) {
    const int t1 = __builtin_amdgcn_readfirstlane(tl + gstride);
    if (t1 < nt) load_tile(vA, t1);
  }
  int ptile = -1;
  if (REGSTAT) {
    while (tl < nt) {
      body(accA, accA, tl, -1, vA, vB, true);
      tl = __builtin_amdgcn_readfirstlane(tl + gstride);
      if (tl >= nt) break;
      body(accA, accA, tl, -1, vB, vA, true);
      tl = __builtin_amdgcn_readfirstlane(tl + gstride);
    }
    tl = nt;
#pragma unroll
    for (int c = 0; c < 8; ++c) my_st[c ^ st_sw] = rs[c];
  }
  while (tl < nt) {
    body(accA, accB, tl, ptile, vA, vB, true);
    ptile = tl;
    tl = __builtin_amdgcn_readfirstlane(tl + gstride);
    if (tl >= nt) {
#pragma unroll
      for (int j = 0; j < 4; ++j) epi(accA, ptile, j);
      break;
    }
    body(accB, accA, tl, ptile, vB, vA, true);
    ptile = tl;
    tl = __builtin_amdgcn_readfirstlane(tl + gstride);
    if (tl >= nt) {
#pragma unroll
      for (int j = 0; j < 4; ++j) epi(accB, ptile, j);
    }
  }
  __syncthreads();
  {
    const int nn = t >> 1, mo = t & 1, ib = nn & 31, wb = nn >> 5;
    const int hh = (ib >> 2) & 1, jj = ib >> 3, qq = ib & 3;
    double a = 0.0;
#pragma unroll 8
    for (int l = 0; l < 32; ++l) {
      const int ln = 32 * hh + l;
      a += (double)sred[(wb * 64 + ln) * 8 + ((2 * jj + mo) ^ ((ln >> 1) & 7))][qq];
    }
    atomicAdd(&stats[t], a);
  }
}

// ---- k_train_h1<NT>: hidden layer 1 straight from the chunk's encoding tiles.  The first layer's output h0 is a
// 268 MB round trip per chunk (written by layer 0, read back here) although it is W0 e + b0 of the 67 MB of
// encoding tiles layer 0 also writes.  So layer 0 runs statistics-only (no h0 store), and this kernel recomputes
// each tile's h0 with the first layer's own instruction sequence (the same split products in the same order on
// the same split operands: bit-identical h0), applies BatchNorm 0 and stages it as the B operand of W1 -- 8 KiB
// read per tile instead of 32 KiB.  Structure = k_train_h's hidden REGSTAT form; per tile: W1 products of tile T
// (16 k-steps), its epilogue, then W0 products of tile T + 1 (4 k-steps, W0 in LDS, reusing the accumulator) and
// their BatchNorm + split into the other B buffer; the encoding tile of T + 2 is loaded during T's k-loop and
// staged (split) into a two-slot LDS ring.  One barrier per tile.
template <int NT>
__global__ __launch_bounds__(512, 1) void k_train_h1(const f32x4* __restrict__ etin, int64_t n,
                                                     const f16x8* __restrict__ W1p, const f16x8* __restrict__ W0p,
                                                     const int* __restrict__ swp, int layer,
                                                     const float* __restrict__ bias, BnPrev prev, float momentum,
                                                     float eps, float* __restrict__ hout,
                                                     double* __restrict__ stats) {
  constexpr int KS = KS_H, XD = H1_XD;
  constexpr int S_ELOAD = 2, S_EPUT = KS - 4;
  __shared__ __attribute__((aligned(16))) float al[256];
  __shared__ __attribute__((aligned(16))) float be[256];
  __shared__ __attribute__((aligned(16))) float bs[256];
  __shared__ __attribute__((aligned(16))) float b0s[256];
  __shared__ float smax[8];
  __shared__ f16x8 xs[2][KS][2][64];
  __shared__ f16x8 eb[2][KS_E][2][64];   // split encoding tiles (B operand of W0), two slots
  __shared__ f16x8 w0s[HW_E];            // W0's image [k-step][out-block][part][lane]
  static_assert(sizeof(xs) >= 8 * 64 * 8 * sizeof(f32x4), "reduction area");
  f32x4* const sred = reinterpret_cast<f32x4*>(&xs[0][0][0][0]);
  const int t = threadIdx.x;
  if (t < 256) {
    bn_coeffs(prev, n, momentum, eps, al, be);   // BatchNorm 0
    bs[t] = bias[t];
    b0s[t] = prev.lin_bias[t];
  }
  int sx;
  {
    float bnd = 0.0f;
    if (t < 256) bnd = sqrtf((float)n) * fabsf(prev.gamma[t]) + fabsf(prev.beta[t]);
    bnd = wave_max_f(bnd);
    if ((t & 63) == 0) smax[t >> 6] = bnd;
    __syncthreads();
    float m = smax[0];
#pragma unroll
    for (int i = 1; i < 8; ++i) m = fmaxf(m, smax[i]);
    sx = (m > 0.0f && m < 3.0e38f) ? 14 - ilogbf(m) : 0;
    sx = sx > 24 ? 24 : sx;
    if (t < 256) {   // 2^sx into BatchNorm 0's coefficients (exact), as k_train_h
      al[t] = ldexpf(al[t], sx);
      be[t] = ldexpf(be[t], sx);
    }
  }
  const float unscale = ldexpf(1.0f, -(swp[layer & 255] + sx));
  const float unscale0 = ldexpf(1.0f, -swp[0]);   // layer 0: unscaled encoding operand (its sx is 0)
  const int nt = (int)((n + 31) / 32);
  const int gstride = (int)gridDim.x;
  const bool rev = (layer >> 8) & 1;
  auto P = [&](int x) { return rev ? nt - 1 - x : x; };
  const int lane = t & 63, h = lane >> 5, li = lane & 31;
  const int blk = __builtin_amdgcn_readfirstlane(t >> 6);
  if (blk >= 4) __builtin_amdgcn_s_setprio(1);
  f16x8 wr[KS][2];
  {
    const f16x8* __restrict__ w8 = W1p + lane;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int p = 0; p < 2; ++p) wr[ks][p] = w8[((ks * 8 + blk) * 2 + p) * 64];
    for (int j = t; j < (int)HW_E; j += 512) w0s[j] = W0p[j];
  }
  f32x4 rs[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) rs[c] = f32x4{};
  // split 4 values into the B layout [k-step G >> 1][part][li + 32 (G & 1)][4 h ..] of feature group G
  auto putb = [&](f16x8 (*dst)[2][64], int G, const f32x4& x) {
    f16x4 hi, mid;
    split4(x, hi, mid);
    const int ln = li + 32 * (G & 1);
    *reinterpret_cast<f16x4*>(reinterpret_cast<_Float16*>(&dst[G >> 1][0][ln]) + 4 * h) = hi;
    *reinterpret_cast<f16x4*>(reinterpret_cast<_Float16*>(&dst[G >> 1][1][ln]) + 4 * h) = mid;
  };
  auto load_enc = [&](int tile) { return etin[(size_t)P(tile) * 512 + t]; };   // group t >> 6, lane
  auto put_enc = [&](int slot, const f32x4& e) { putb(eb[slot], t >> 6, e); };
  // h0 of the wave's 32 neurons for `tile` (W0 products exactly as k_train_h<8,false>), BatchNorm 0, split into
  // B buffer b at groups 4 blk + j
  // operands of W0 k-step ks for encoding slot `slot`: {w hi, w mid, x hi, x mid}
  auto h0_ops = [&](f16x8 (&o)[4], int slot, int ks) {
    o[0] = w0s[((ks * 8 + blk) * 2 + 0) * 64 + lane];
    o[1] = w0s[((ks * 8 + blk) * 2 + 1) * 64 + lane];
    o[2] = eb[slot][ks][0][lane];
    o[3] = eb[slot][ks][1][lane];
  };
  // one W0 k-step of h0 (ops: its operands)
  auto h0_mfma = [&](f32x16& acc, const f16x8 (&o)[4], int ks) {
    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(o[0], o[2], ks == 0 ? f32x16{} : acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(o[0], o[3], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(o[1], o[2], acc, 0, 0, 0);
    if (NT == 4) acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(o[1], o[3], acc, 0, 0, 0);
  };
  // h0 part j (accumulator registers 4j..4j+3) + b0, BatchNorm 0, split into B buffer b at group 4 blk + j
  auto h0_epi = [&](const f32x16& acc, int b, int j) {
    const int f0 = 32 * blk + 8 * j + 4 * h;
    const f32x4 bj = *reinterpret_cast<const f32x4*>(b0s + f0);
    const f32x4 a = *reinterpret_cast<const f32x4*>(al + f0), c = *reinterpret_cast<const f32x4*>(be + f0);
    f32x4 x;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float hv = acc[4 * j + q] * unscale0 + bj[q];   // k_train_h's epilogue: o = d + b
      x[q] = hv * a[q] + c[q];   // its staging: (v alpha + beta') 2^sx, the scale folded into alpha / beta' 
    }
    putb(xs[b], 4 * blk + j, x);
  };
  // (ops0: k-step 0's operands, read ahead by the caller)
  auto h0_stage = [&](f32x16& acc, int slot, int b, const f16x8 (&ops0)[4]) {
    f16x8 op[2][4];
#pragma unroll
    for (int i = 0; i < 4; ++i) op[0][i] = ops0[i];
#pragma unroll
    for (int ks = 0; ks < KS_E; ++ks) {
      if (ks + 1 < KS_E) h0_ops(op[(ks + 1) & 1], slot, ks + 1);
      h0_mfma(acc, op[ks & 1], ks);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) h0_epi(acc, b, j);
  };
  int tl = __builtin_amdgcn_readfirstlane((int)blockIdx.x);
  f32x16 acc;
  if (tl < nt) {
    put_enc(0, load_enc(tl));
    const int t1 = tl + gstride;
    if (t1 < nt) put_enc(1, load_enc(t1));
  }
  __syncthreads();
  __builtin_amdgcn_s_waitcnt(0);   // W1 resident
  if (tl < nt) {
    f16x8 o0[4];
    h0_ops(o0, 0, 0);
    h0_stage(acc, 0, 0, o0);
  }
  __syncthreads();
  int buf = 0;
  while (tl < nt) {
    const int nxt = __builtin_amdgcn_readfirstlane(tl + gstride);
    const int nxt2 = __builtin_amdgcn_readfirstlane(tl + 2 * gstride);
    const bool more = nxt < nt, more2 = nxt2 < nt;
    f16x8 xr[XD][2];
    f32x4 ev;
    f16x8 o0[4];   // W0 k-step 0 operands of tile + 1, read during the last W1 k-step
#pragma unroll
    for (int d = 0; d < XD - 1; ++d) {
      xr[d][0] = xs[buf][d][0][lane];
      xr[d][1] = xs[buf][d][1][lane];
    }
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      if (ks + XD - 1 < KS) {
        xr[(ks + XD - 1) % XD][0] = xs[buf][ks + XD - 1][0][lane];
        xr[(ks + XD - 1) % XD][1] = xs[buf][ks + XD - 1][1][lane];
      }
      const f16x8 xh = xr[ks % XD][0], xm = xr[ks % XD][1];
      acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(wr[ks][0], xh, ks == 0 ? f32x16{} : acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(wr[ks][0], xm, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(wr[ks][1], xh, acc, 0, 0, 0);
      if (NT == 4) acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(wr[ks][1], xm, acc, 0, 0, 0);
      if (ks == S_ELOAD && more2) ev = load_enc(nxt2);
      if (ks == S_EPUT && more2) put_enc(buf, ev);   // slot of tile + 2 = this tile's slot (read one tile ago)
      if (ks == KS - 1) h0_ops(o0, buf ^ 1, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
    {   // epilogue of this tile (as k_train_h's REGSTAT epilogue)
      const int tile = P(tl);
      const bool valid = (int64_t)tile * 32 + li < n;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const f32x4 bj = *reinterpret_cast<const f32x4*>(bs + 32 * blk + 8 * j + 4 * h);
        f32x4 o;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float d = acc[4 * j + q] * unscale;
          o[q] = d + bj[q];
          const float dv = valid ? d : 0.0f;
          rs[2 * j][q] += dv;
          rs[2 * j + 1][q] += dv * dv;
        }
        f32x4* dst = reinterpret_cast<f32x4*>(hout + (size_t)tile * TILE_FLOATS + (size_t)(4 * blk + j) * 256) + lane;
        *dst = o;
      }
    }
    if (more) h0_stage(acc, buf ^ 1, buf ^ 1, o0);   // tile + 1's encoding sits in the other slot
    __syncthreads();
    buf ^= 1;
    tl = nxt;
  }
  f32x4* const my_st = sred + (blk * 64 + lane) * 8;
  const int st_sw = (lane >> 1) & 7;
#pragma unroll
  for (int c = 0; c < 8; ++c) my_st[c ^ st_sw] = rs[c];
  __syncthreads();
  {
    const int nn = t >> 1, mo = t & 1, ib = nn & 31, wb = nn >> 5;
    const int hh = (ib >> 2) & 1, jj = ib >> 3, qq = ib & 3;
    double a = 0.0;
#pragma unroll 8
    for (int l = 0; l < 32; ++l) {
      const int ln = 32 * hh + l;
      a += (double)sred[(wb * 64 + ln) * 8 + ((2 * jj + mo) ^ ((ln >> 1) & 7))][qq];
    }
    atomicAdd(&stats[t], a);
  }
}

// ---- layer 0 from the encoding's moments (split forward without activation store, k_train_h1 after it).
// Layer 0's only remaining outputs there are the chunk's encoding tiles and BatchNorm 0's statistics, and those
// statistics are exact functions of the chunk's encoding mean ebar and covariance Sigma (h0 = W0 e + b0 feeds
// BatchNorm 0 directly, models.py:183-203, whatever the activations further on):
// sum_s (W0 e_s)_i = n w_i.ebar, sum_s (W0 e_s)_i^2 = n (w_i^T Sigma w_i + (w_i.ebar)^2).
//   k_enc_gram    each sample's encoding once (encode_full: 30 sincosf, not 64 as the per-float4 form of the first
//                 layer), stored as the chunk's encoding tiles ([tile][g][lane][4]; padded lanes carry the last
//                 sample, as k_train_h's), and sum d d^T with d = [e - e0, 1] (e0 = the chunk's first encoding, a
//                 shift against cancellation) in k_tf_moments' form: fp16 hi/mid parts in a wave-private
//                 [feature][sample] LDS tile, three exact products per pair on v_mfma_f32_32x32x16_f16, fp32 per
//                 64-sample unit, float64 across units, one partial per workgroup (blocks 00, 01, 11 of 64 x 64);
//   k_gram_sum    the partials summed in a fixed order;
//   k_gram_stats  ebar, Sigma and the 256 neurons' sums in float64 -> BatchNorm 0's statistics (bn_coeffs' input).
// The 256-neuron product of the first layer (99 us per chunk of 262,144, VALU-bound) becomes a 64 x 64 one.
constexpr int GR_P = 72;          // LDS pitch (halves): 16 lanes' 16-byte operand reads hit disjoint bank groups
constexpr int GR_BLOCKS = 512;    // k_enc_gram workgroups per chunk (two per CU)
constexpr int GR_PART = 3072;     // doubles per partial: blocks 00, 01, 11 as [block][register 16][lane 64]
constexpr size_t GR_DOUBLES = (size_t)(GR_BLOCKS + 1) * GR_PART + 64;

// feature f of Embedding(3, 10) at p: encode_full's value, one sincosf per feature (wave-parallel shift vector)
__device__ __forceinline__ float enc_feat1(const float (&p)[3], int f) {
  const int fk = f < 3 ? 0 : (f - 3) / 6, fr = f < 3 ? 0 : (f - 3) - 6 * fk;
  const int m = fr < 3 ? fr : fr - 3;
  const float pm = m == 0 ? p[0] : m == 1 ? p[1] : p[2];
  float sn, cs;
  sincosf(__int_as_float((127 + fk) << 23) * pm, &sn, &cs);
  const float pf = f == 0 ? p[0] : f == 1 ? p[1] : p[2];
  return f < 3 ? pf : f >= 63 ? 0.0f : fr < 3 ? sn : cs;
}

__device__ __forceinline__ void gram_lds_sync() {   // wave-private tiles: order one wave's LDS writes and reads
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__global__ __launch_bounds__(256, 2) void k_enc_gram(const float* __restrict__ rays, int stride,
                                                     const float* __restrict__ z, int S, int64_t c0,
                                                     const float* __restrict__ ein, int64_t n,
                                                     f32x4* __restrict__ etout, double* __restrict__ part,
                                                     double* __restrict__ e0out) {
  __shared__ __attribute__((aligned(16))) _Float16 th[4][2][64 * GR_P];
  __shared__ float sh0[64];
  static_assert(sizeof(th) >= GR_PART * sizeof(double), "reduction area");
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  if (tid < 64) {   // e0 = the encoding of the chunk's first sample, one feature per lane
    float v;
    if (ein) {
      v = tid < 63 ? ein[c0 * 63 + tid] : 0.0f;
    } else {
      float p[3];
      sample_point(rays + ray_of(c0, S) * stride, z[c0], p);
      v = enc_feat1(p, tid);
    }
    sh0[tid] = v;
    if (blockIdx.x == 0) e0out[tid] = (double)v;
  }
  __syncthreads();
  const int64_t nu = (n + 63) / 64, ntiles = (n + 31) / 32;
  f32x16 a00 = {}, a01 = {}, a11 = {};
  double d00[16], d01[16], d11[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) d00[r] = d01[r] = d11[r] = 0.0;
  _Float16* const hi = th[wave][0];
  _Float16* const mi = th[wave][1];
  for (int64_t u = (int64_t)blockIdx.x * 4 + wave; u < nu; u += (int64_t)gridDim.x * 4) {
    const int64_t s = u * 64 + lane;
    const bool ok = s < n;
    const int64_t se = ok ? s : n - 1;   // padded lanes: the last sample (k_train_h's sample_of)
    float f[64];
    if (ein) {
      const float* r = ein + (c0 + se) * 63;
#pragma unroll
      for (int k = 0; k < 63; ++k) f[k] = r[k];
      f[63] = 0.0f;
    } else {
      float p[3];
      sample_point(rays + ray_of(c0 + se, S) * stride, z[c0 + se], p);
      encode_full(p, f);
    }
    const int64_t tile = s >> 5;
    if (tile < ntiles) {   // [tile][g][lane (s & 31) + 32 h][4]: features 8 g + 4 h + q
      f32x4* dst = etout + (size_t)tile * 512 + (lane & 31);
#pragma unroll
      for (int g = 0; g < 8; ++g)
#pragma unroll
        for (int h = 0; h < 2; ++h)
          dst[g * 64 + 32 * h] = f32x4{f[8 * g + 4 * h], f[8 * g + 4 * h + 1], f[8 * g + 4 * h + 2], f[8 * g + 4 * h + 3]};
    }
    // fp16 range: a unit whose largest |d| reaches 2^15 (positions spread over more than 32 km) is split at 2^-ks,
    // the count column included, and its products rescaled by 2^(2 ks) in float64 (exact powers of two; ks = 0 for
    // every realistic scene, so the common path is unchanged)
    float dm = 0.0f;
#pragma unroll
    for (int k = 0; k < 63; ++k) dm = fmaxf(dm, ok ? fabsf(f[k] - sh0[k]) : 0.0f);
    dm = wave_max_f(dm);
    int ks = (dm >= 32768.0f && dm < 3.0e38f) ? ilogbf(dm) - 14 : 0;
    ks = ks > 24 ? 24 : ks;
    const float dsc = ldexpf(1.0f, -ks);
#pragma unroll
    for (int k = 0; k < 63; ++k) {
      const float d = ok ? (f[k] - sh0[k]) * dsc : 0.0f;
      const _Float16 a = (_Float16)d;
      hi[k * GR_P + lane] = a;
      mi[k * GR_P + lane] = (_Float16)(d - (float)a);
    }
    hi[63 * GR_P + lane] = ok ? (_Float16)dsc : (_Float16)0.0f;
    mi[63 * GR_P + lane] = (_Float16)0.0f;
    gram_lds_sync();
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const int o = (lane & 31) * GR_P + 16 * ks + 8 * (lane >> 5);
      const f16x8 h0 = *reinterpret_cast<const f16x8*>(hi + o);
      const f16x8 m0 = *reinterpret_cast<const f16x8*>(mi + o);
      const f16x8 h1 = *reinterpret_cast<const f16x8*>(hi + 32 * GR_P + o);
      const f16x8 m1 = *reinterpret_cast<const f16x8*>(mi + 32 * GR_P + o);
      a00 = __builtin_amdgcn_mfma_f32_32x32x16_f16(h0, h0, a00, 0, 0, 0);
      a01 = __builtin_amdgcn_mfma_f32_32x32x16_f16(h0, h1, a01, 0, 0, 0);
      a11 = __builtin_amdgcn_mfma_f32_32x32x16_f16(h1, h1, a11, 0, 0, 0);
      a00 = __builtin_amdgcn_mfma_f32_32x32x16_f16(h0, m0, a00, 0, 0, 0);
      a01 = __builtin_amdgcn_mfma_f32_32x32x16_f16(h0, m1, a01, 0, 0, 0);
      a11 = __builtin_amdgcn_mfma_f32_32x32x16_f16(h1, m1, a11, 0, 0, 0);
      a00 = __builtin_amdgcn_mfma_f32_32x32x16_f16(m0, h0, a00, 0, 0, 0);
      a01 = __builtin_amdgcn_mfma_f32_32x32x16_f16(m0, h1, a01, 0, 0, 0);
      a11 = __builtin_amdgcn_mfma_f32_32x32x16_f16(m1, h1, a11, 0, 0, 0);
    }
    const double usc = ldexp(1.0, 2 * ks);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      d00[r] += (double)a00[r] * usc;
      d01[r] += (double)a01[r] * usc;
      d11[r] += (double)a11[r] * usc;
      a00[r] = a01[r] = a11[r] = 0.0f;
    }
    gram_lds_sync();
  }
  // the four waves' partials summed in a fixed order through LDS (aliasing the tiles), one coalesced store
  __syncthreads();
  double* red = reinterpret_cast<double*>(&th[0][0][0]);
  for (int wv = 0; wv < 4; ++wv) {
    if (wave == wv) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int x = r * 64 + lane;
        red[x] = wv ? red[x] + d00[r] : d00[r];
        red[1024 + x] = wv ? red[1024 + x] + d01[r] : d01[r];
        red[2048 + x] = wv ? red[2048 + x] + d11[r] : d11[r];
      }
    }
    __syncthreads();
  }
  double* out = part + (size_t)blockIdx.x * GR_PART;
  for (int k = tid; k < GR_PART; k += 256) out[k] = red[k];
}

// grid GR_PART / 16, 512 threads: block x0 owns moments x0 .. x0 + 15; thread (q = tid >> 4, x) sums partials
// q, q + 32, .. (all its loads in flight at once: the partials were written by every XCD, so each load is a trip
// to the memory side), then the 32 q-sums are added in order -> mom[x]
__global__ __launch_bounds__(512) void k_gram_sum(const double* __restrict__ part, int nb, double* __restrict__ mom) {
  __shared__ double red[32][16];
  const int xl = threadIdx.x & 15, q = threadIdx.x >> 4, x = blockIdx.x * 16 + xl;
  double s = 0.0;
  int b = q;
  for (; b + 32 * 15 < nb; b += 32 * 16) {
    double v[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) v[k] = part[(size_t)(b + 32 * k) * GR_PART + x];
#pragma unroll
    for (int k = 0; k < 16; ++k) s += v[k];
  }
  for (; b < nb; b += 32) s += part[(size_t)b * GR_PART + x];
  red[q][xl] = s;
  __syncthreads();
  if (q == 0) {
    double t = red[0][xl];
#pragma unroll
    for (int k = 1; k < 32; ++k) t += red[k][xl];
    mom[x] = t;
  }
}

// grid 32, 256 threads: block b -> neurons 8 b .. 8 b + 7.  M = sum d d^T, n = M[63][63], dbar = M[k][63] / n,
// Sigma = M / n - dbar dbar^T, ebar = e0 + dbar; neuron i (32 threads, rows k = slice, slice + 32 of Sigma w_i):
// stats[2i] = n w_i.ebar, stats[2i+1] = n (w_i^T Sigma w_i + (w_i.ebar)^2)   (sums of h - b0, as k_train_h's)
constexpr int GS_BLOCKS = 32;
__global__ __launch_bounds__(256) void k_gram_stats(const double* __restrict__ mom, const double* __restrict__ e0,
                                                    const float* __restrict__ w0, double* __restrict__ stats) {
  __shared__ double M[64 * 65];
  __shared__ double Sg[63 * 65];
  __shared__ double eb[64], db[64];
  __shared__ float ws[8 * 64];
  const int tid = threadIdx.x;
  double mv[GR_PART / 256];   // every load in flight at once
#pragma unroll
  for (int j = 0; j < GR_PART / 256; ++j) mv[j] = mom[tid + 256 * j];
  float wv[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int x = tid + 256 * j, i = x >> 6, k = x & 63;
    wv[j] = k < 63 ? w0[(size_t)(8 * blockIdx.x + i) * 63 + k] : 0.0f;
  }
  const double e0v = tid < 63 ? e0[tid] : 0.0;
#pragma unroll
  for (int jx = 0; jx < GR_PART / 256; ++jx) {   // blocks 00, 01, 11 -> M (both triangles)
    const int x = tid + 256 * jx;
    const int b = x >> 10, r = (x >> 6) & 15, ln = x & 63;
    const int i = (r & 3) + 8 * (r >> 2) + 4 * (ln >> 5) + (b == 2 ? 32 : 0), j = (ln & 31) + (b ? 32 : 0);
    M[i * 65 + j] = mv[jx];
    M[j * 65 + i] = mv[jx];
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) ws[tid + 256 * j] = wv[j];
  // the chunk's other BatchNorm statistics start from zero (layers 1-7 add to them): the memset of the other path
  if (tid < 7 * 512 / GS_BLOCKS) stats[512 + (int)blockIdx.x * (7 * 512 / GS_BLOCKS) + tid] = 0.0;
  __syncthreads();
  const double n = M[63 * 65 + 63], inv_n = 1.0 / n;
  if (tid < 64) {
    db[tid] = tid < 63 ? M[tid * 65 + 63] * inv_n : 0.0;
    eb[tid] = tid < 63 ? e0v + M[tid * 65 + 63] * inv_n : 0.0;
  }
  __syncthreads();
#pragma unroll 4
  for (int j = 0; j < (63 * 63 + 255) / 256; ++j) {   // Sigma
    const int x = tid + 256 * j;
    if (x < 63 * 63) {
      const int k = x / 63, l = x - 63 * k;
      Sg[k * 65 + l] = M[k * 65 + l] * inv_n - db[k] * db[l];
    }
  }
  __syncthreads();
  const int i = tid >> 5, sl = tid & 31;
  const float* w = ws + i * 64;
  double v = 0.0, mu = 0.0;
#pragma unroll 1
  for (int k = sl; k < 63; k += 32) {
    double r[63];   // the row's loads issued together
#pragma unroll
    for (int l = 0; l < 63; ++l) r[l] = Sg[k * 65 + l];
    double t0 = 0.0, t1 = 0.0, t2 = 0.0;
#pragma unroll
    for (int l = 0; l < 63; l += 3) {
      t0 += r[l] * (double)w[l];
      t1 += r[l + 1] * (double)w[l + 1];
      t2 += r[l + 2] * (double)w[l + 2];
    }
    const double wk = (double)w[k];
    v += wk * ((t0 + t1) + t2);
    mu += wk * eb[k];
  }
#pragma unroll
  for (int o = 1; o < 32; o <<= 1) {
    v += __shfl_xor(v, o, 64);
    mu += __shfl_xor(mu, o, 64);
  }
  if (sl == 0) {
    const int nn = 8 * blockIdx.x + i;
    stats[2 * nn] = n * mu;
    stats[2 * nn + 1] = n * (v + mu * mu);
  }
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
  f32x4* enc;   // the chunk's encoding tiles: written by the first layer, read by the skip layer
  float* wp;
  f16x8* wh;    // split-fp16 weight image (train math 1/2)
  int* sw;      // its per-layer scale exponents
  double* stats;
  double* gram;  // k_enc_gram partials, their slice sums and the chunk's shift e0
  unsigned* pbound;   // k_pos_bound's result (float bits)
  size_t bytes;
};

// Train-mode MLP arithmetic: 0 = fp32 MFMA, 1 = split fp16 with 3 products (default), 2 = split fp16 with 4
// products (k_train_h).  Process-wide; pcnerf_set_train_math.  Mode 1 renders config 2 within 1.9e-5 of a float64
// evaluation of the same rays (fp32 MFMA: 2.2e-5; the reference itself: 1.1e-4) at 1.9x the speed.
static int g_train_math = 1;
// The rematerialised backward's layer kernel: 4 = k_bwd_remat3<true> (default: weight gradient over the encoding
// columns, projected by P'^T per chunk; BatchNorm-backward epilogue on the W waves), 3 = k_bwd_remat3<false> (the
// epilogue on the D waves), 2 = k_bwd_remat2 (round 5's: over the rematerialised x columns).  PCNERF_REMAT_VER
// selects it at load time (A/B measurements).
static int remat_ver_env() {
  const char* v = getenv("PCNERF_REMAT_VER");
  return (v && v[0] == '2') ? 2 : (v && v[0] == '3') ? 3 : 4;
}
static int g_remat_ver = remat_ver_env();
// version 4's layer-1 launch forms dW_0's encoding columns itself (k_bwd_remat3<true, true>; default); 0 keeps
// k_wgrad_enc on the stored g_0 (PCNERF_REMAT_FUSE0=0 / pcnerf_set_remat_fuse0, A/B)
// version 4's hidden layers with eight W waves (three waves per SIMD: each W wave half the epilogue / remat / G_d
// rows); PCNERF_REMAT_W8=1 (A/B)
#ifndef PCN_R3_W8_DEFAULT
#define PCN_R3_W8_DEFAULT 0
#endif
static int g_remat_w8 = [] {
  const char* v = getenv("PCNERF_REMAT_W8");
  return v ? (v[0] == '1' ? 1 : 0) : PCN_R3_W8_DEFAULT;
}();
static int g_remat_fuse0 = [] {
  const char* v = getenv("PCNERF_REMAT_FUSE0");
  return (v && v[0] == '0') ? 0 : 1;
}();

static TrainWs carve(void* base, int64_t chunk) {
  const size_t tiles = (size_t)((chunk + 31) / 32);
  size_t off = 0;
  auto take = [&](size_t bytes) {
    const size_t o = off;
    off += (bytes + 255) & ~(size_t)255;
    return o;
  };
  const size_t oA = take(tiles * TILE_FLOATS * 4), oB = take(tiles * TILE_FLOATS * 4);
  const size_t oE = take(tiles * 512 * sizeof(f32x4));
  const size_t ow = take(TRAIN_W_FLOATS * 4), ost = take(8 * 512 * 8);
  const size_t owh = take(TRAIN_H_VECS * sizeof(f16x8)), osw = take(16 * sizeof(int));
  const size_t ogr = take(GR_DOUBLES * sizeof(double)), opb = take(sizeof(unsigned));
  char* b = (char*)base;
  TrainWs w;
  w.bufA = (float*)(b + oA);
  w.bufB = (float*)(b + oB);
  w.enc = (f32x4*)(b + oE);
  w.wp = (float*)(b + ow);
  w.wh = (f16x8*)(b + owh);
  w.sw = (int*)(b + osw);
  w.stats = (double*)(b + ost);
  w.gram = (double*)(b + ogr);
  w.pbound = (unsigned*)(b + opb);
  w.bytes = off;
  return w;
}

}  // namespace pcn

using namespace pcn;

extern "C" size_t pcnerf_nof_train_workspace_bytes(int64_t chunk) { return carve(nullptr, chunk).bytes; }

extern "C" int pcnerf_set_train_math(int mode) {
  if (mode < 0 || mode > 2) {
    pcn::set_error("pcnerf_set_train_math: mode must be 0 (fp32 MFMA), 1 or 2 (split fp16, 3 / 4 products)");
    return -1;
  }
  const int prev = pcn::g_train_math;
  pcn::g_train_math = mode;
  return prev;
}

extern "C" int pcnerf_set_remat_version(int version) {
  if (version < 2 || version > 4) {
    pcn::set_error("pcnerf_set_remat_version: version must be 2 (k_bwd_remat2), 3 (k_bwd_remat3) or 4 "
                   "(k_bwd_remat3 with the epilogue on the W waves)");
    return -1;
  }
  const int prev = pcn::g_remat_ver;
  pcn::g_remat_ver = version;
  return prev;
}

// The train-mode layer launches of one chunk under the selected arithmetic (layer 0: KE_FIRST, hidden, skip).
namespace pcn {
struct TrainLayerLaunch {
  const float* rays;
  int stride;
  const float* z;
  int S;
  int64_t c0;
  const float* ein;
  int64_t n;
  unsigned gws;
  float mom, eps;
  hipStream_t s;
};

// Tile order of the split train layers: the odd hidden layers walk their chunk backwards, so each hidden layer
// first reads the tiles its predecessor wrote last.
static int tile_rev(int L) { return (0xAA >> L) & 1; }

template <int KE, bool HP>
static void launch_layer(const TrainLayerLaunch& q, const NofParamsDev& P, const float* wp, const f16x8* wh,
                         const int* sw, int L, const float* hin, const BnPrev& prev, float* hout, double* stats,
                         const f32x4* etin, f32x4* etout) {
  const int m = g_train_math;
  if (m == 0) {
    hipLaunchKernelGGL((k_train_ws<KE, HP>), dim3(q.gws), dim3(512), 0, q.s, q.rays, q.stride, q.z, q.S, q.c0, q.ein,
                       hin, q.n, wp + off_w(L, KE != 0), P.lin_b[L], prev, q.mom, q.eps, hout, stats, etin, etout);
  } else if (m == 1) {
    hipLaunchKernelGGL((k_train_h<KE, HP, 3>), dim3(q.gws), dim3(512), 0, q.s, q.rays, q.stride, q.z, q.S, q.c0,
                       q.ein, hin, q.n, wh + off_h(L, KE != 0), sw, L | (tile_rev(L) << 8), P.lin_b[L], prev, q.mom,
                       q.eps, hout, stats, etin, etout);
  } else {
    hipLaunchKernelGGL((k_train_h<KE, HP, 4>), dim3(q.gws), dim3(512), 0, q.s, q.rays, q.stride, q.z, q.S, q.c0,
                       q.ein, hin, q.n, wh + off_h(L, KE != 0), sw, L | (tile_rev(L) << 8), P.lin_b[L], prev, q.mom,
                       q.eps, hout, stats, etin, etout);
  }
}

static void pack_weights(const NofParamsDev& P, float* wp, f16x8* wh, int* sw, hipStream_t s) {
  if (g_train_math == 0) {
    hipLaunchKernelGGL(k_pack_train, dim3((unsigned)((TRAIN_W_FLOATS + 255) / 256)), dim3(256), 0, s, P, wp);
  } else {
    hipLaunchKernelGGL(k_wscale, dim3(8), dim3(1024), 0, s, P, sw);
    hipLaunchKernelGGL(k_pack_train_h, dim3((unsigned)((TRAIN_H_VECS + 255) / 256)), dim3(256), 0, s, P, sw, wh);
  }
}
}  // namespace pcn

#if PCN_RB_CLK
extern "C" int pcnerf_debug_rbclk(unsigned long long* out) {   // out: [4096][5] (g_rbclk)
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(pcn::g_rbclk), sizeof(pcn::g_rbclk)) == hipSuccess ? 0 : 1;
}
#endif

#if PCN_CLOCK_STAMP
// diagnostic builds: median over workgroups of the last hidden-layer launch's in-kernel clock (MHz) and cycles
extern "C" int pcnerf_debug_clock(double* out) {
  // out: [0] loop clock MHz, [1] kernel span us (last exit - first entry), median [2] prologue, [3] loop,
  // [4] epilogue us; [5] entry spread, [6] exit spread, [7] loop-end spread (us)
  static unsigned long long h[4096][6];
  if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_clk), sizeof(h)) != hipSuccess) return 1;
  std::vector<double> f, pro, loop, epi, en, ex, le;
  for (int i = 0; i < 4096; ++i)
    if (h[i][3] > h[i][0] && h[i][2] > h[i][1]) {
      f.push_back((double)(h[i][5] - h[i][4]) / (double)(h[i][2] - h[i][1]) * 100.0);
      pro.push_back((h[i][1] - h[i][0]) * 0.01);
      loop.push_back((h[i][2] - h[i][1]) * 0.01);
      epi.push_back((h[i][3] - h[i][2]) * 0.01);
      en.push_back((double)h[i][0]);
      ex.push_back((double)h[i][3]);
      le.push_back((double)h[i][2]);
    }
  if (f.empty()) return 2;
  auto med = [](std::vector<double> v) { std::sort(v.begin(), v.end()); return v[v.size() / 2]; };
  const double e0 = *std::min_element(en.begin(), en.end()), e1 = *std::max_element(en.begin(), en.end());
  const double x0 = *std::min_element(ex.begin(), ex.end()), x1 = *std::max_element(ex.begin(), ex.end());
  const double l0 = *std::min_element(le.begin(), le.end()), l1 = *std::max_element(le.begin(), le.end());
  out[0] = med(f); out[1] = (x1 - e0) * 0.01; out[2] = med(pro); out[3] = med(loop); out[4] = med(epi);
  out[5] = (e1 - e0) * 0.01; out[6] = (x1 - x0) * 0.01; out[7] = (l1 - l0) * 0.01;
  return 0;
}
#endif

// Activation store of the training step: per chunk the raw h of all 8 layers (the tile layout the backward
// consumes) and the chunk's BatchNorm statistics, written by the forward so the backward need not recompute.
struct StoreChunk {
  float* h[8];
  double* stats;
};

static_assert(TILE_FLOATS == 32 * 256, "store_layer_bytes (pcnerf_internal.h) assumes 32-sample tiles of 256");

extern "C" size_t pcnerf_nof_store_bytes(int64_t chunk) {
  return 8 * store_layer_bytes(chunk) + ((8 * 512 * 8 + 255) & ~(size_t)255);
}

static StoreChunk store_chunk(const void* store, int64_t chunk, int64_t ci) {
  char* b = (char*)store + (size_t)ci * pcnerf_nof_store_bytes(chunk);
  StoreChunk c;
  for (int L = 0; L < 8; ++L) c.h[L] = (float*)(b + L * store_layer_bytes(chunk));
  c.stats = (double*)(b + 8 * store_layer_bytes(chunk));
  return c;
}

// fp16 range of the layered split math: k_train_h1, the skip layer and the encoding-column weight gradients split
// the encoding's xyz features without a scale, so a sample position at or beyond 65,504 (fp16's largest finite
// value) from the block origin would turn into inf there and NaN downstream.  The fused forward, the eval query
// and the layer-0 moments scale per sample / per unit and have no such limit.  Before any launch, one pass over
// the call's sample positions (sample_point's arithmetic, or the embedded batch's xyz columns) is read back and
// the call raises instead of returning NaN.
__global__ __launch_bounds__(256) void k_pos_bound(const float* __restrict__ rays, int stride,
                                                   const float* __restrict__ z, int S, const float* __restrict__ ein,
                                                   int64_t total, unsigned* __restrict__ out) {
  float m = 0.0f;
  for (int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x; g < total; g += (int64_t)gridDim.x * 256) {
    float p[3];
    if (ein) {
      p[0] = ein[g * 63], p[1] = ein[g * 63 + 1], p[2] = ein[g * 63 + 2];
    } else {
      sample_point(rays + ray_of(g, S) * stride, z[g], p);
    }
    m = fmaxf(m, fmaxf(fabsf(p[0]), fmaxf(fabsf(p[1]), fabsf(p[2]))));   // fmaxf drops NaN positions
  }
  m = wave_max_f(m);
  __shared__ float red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  // one atomic per workgroup (a few hundred in all: same-address atomics serialise at one L2 channel)
  if (threadIdx.x == 0) atomicMax(out, __float_as_uint(fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]))));
}

static void pos_bound_async(const float* rays, int stride, const float* z, int S, const float* ein, int64_t total,
                            unsigned* dev, hipStream_t s) {
  PCN_HIP(hipMemsetAsync(dev, 0, sizeof(unsigned), s));
  const int64_t blocks = std::min<int64_t>(512, (total + 255) / 256);
  hipLaunchKernelGGL(k_pos_bound, dim3((unsigned)blocks), dim3(256), 0, s, rays, stride, z, S, ein, total, dev);
}

static void check_split_range(const float* rays, int stride, const float* z, int S, const float* ein, int64_t total,
                              unsigned* dev, hipStream_t s, const char* who) {
  if (g_train_math == 0) return;   // fp32 MFMA: no fp16 operand
  pos_bound_async(rays, stride, z, S, ein, total, dev, s);
  unsigned h = 0;
  PCN_HIP(hipMemcpyAsync(&h, dev, sizeof(unsigned), hipMemcpyDeviceToHost, s));
  PCN_HIP(hipStreamSynchronize(s));
  float m;
  memcpy(&m, &h, sizeof(m));
  if (!(m < 65504.0f))
    throw std::runtime_error(std::string(who) + ": a sample position lies " + std::to_string(m) +
                             " from the block origin, beyond fp16's range (65,504) that the layered split train "
                             "math's encoding operand needs; use set_train_math('fp32') for such blocks");
}

static void query_train(const float* rays, int ray_stride, const float* z, int n_samples, const float* ein,
                        int64_t total, int64_t chunk, const pcnerf_nof_params* params, float momentum, float eps,
                        void* workspace, size_t workspace_bytes, float* p_out, void* stream,
                        void* store = nullptr, int64_t store_chunks = 0) {
  const TrainWs ws = carve(workspace, chunk);
  PCN_CHECK(workspace_bytes >= ws.bytes, "pcnerf_nof_query_train: workspace too small");
  NofParamsDev P;
  PCN_CHECK(to_dev_params(params, eps, &P), "pcnerf_nof_query_train: null parameter pointer");
  // nn.BatchNorm1d raises for a chunk of one sample (render.py:47-50 would hit it on a 1-sample tail)
  PCN_CHECK(total % chunk != 1 && total != 1, "Expected more than 1 value per channel when training");
  hipStream_t s = (hipStream_t)stream;
  check_split_range(rays, ray_stride, z, n_samples, ein, total, ws.pbound, s, "pcnerf_nof_query_train");
  pack_weights(P, ws.wp, ws.wh, ws.sw, s);
  for (int64_t c0 = 0; c0 < total; c0 += chunk) {
    const int64_t n = total - c0 < chunk ? total - c0 : chunk;
    const int64_t ntiles = (n + 31) / 32;
    const unsigned gws = (unsigned)(ntiles < 256 ? ntiles : 256);   // k_train_ws: one workgroup per CU
    const double dn = (double)n;
    // stored chunk: every layer writes its own buffer of the store (kept for the backward); else ping-pong
    const int64_t ci = c0 / chunk;
    const bool keep = store && ci < store_chunks;
    const StoreChunk sc = keep ? store_chunk(store, chunk, ci) : StoreChunk{};
    double* stats = keep ? sc.stats : ws.stats;
    float* hin = keep ? sc.h[0] : ws.bufA;
    float* hout = keep ? sc.h[1] : ws.bufB;
    // the encoding tiles the skip layer reads back: written by THIS chunk's first-layer launch just below
    const f32x4* enc_of_chunk = nullptr;
    // split math, nothing kept for a backward: layer 0 statistics-only, layer 1 recomputes h0 from the encoding
    // tiles (k_train_h1)
    const bool h1 = !keep && g_train_math != 0;
    if (!h1) PCN_HIP(hipMemsetAsync(stats, 0, 8 * 512 * sizeof(double), s));   // (else k_gram_stats)
    // in place: every layer of the chunk overwrites its input tile by tile (a tile is read only by the workgroup
    // that writes its output, which staged it before its MFMAs): one 268 MB footprint instead of two.  k_train_h
    // declares hin / hout without __restrict__ for this; k_train_h1 reads the encoding tiles, not hin.
    if (h1) hout = hin;
    if (h1) {
      // algorithmic: the 64 x 64 moment product per sample; 4 B of z in, 256 B of encoding out
      ProfScope ps(s, PT_TRAIN_FIRST, 2.0 * 64 * 64 * dn, (4.0 + 256.0) * dn);
      const int64_t nu = (n + 63) / 64;
      const int gb = (int)std::min<int64_t>(GR_BLOCKS, (nu + 3) / 4);
      double* mom = ws.gram + (size_t)GR_BLOCKS * GR_PART;
      double* e0 = mom + GR_PART;
      hipLaunchKernelGGL(k_enc_gram, dim3((unsigned)gb), dim3(256), 0, s, rays, ray_stride, z, n_samples, c0, ein, n,
                         ws.enc, ws.gram, e0);
      hipLaunchKernelGGL(k_gram_sum, dim3(GR_PART / 16), dim3(512), 0, s, ws.gram, gb, mom);
      hipLaunchKernelGGL(k_gram_stats, dim3(GS_BLOCKS), dim3(256), 0, s, mom, e0, P.lin_w[0], stats);
      enc_of_chunk = ws.enc;
    } else {
      const BnPrev none{};
      ProfScope ps(s, PT_TRAIN_FIRST, 2.0 * 63 * 256 * dn, (4.0 + (h1 ? 256.0 : 1024.0 + 256.0)) * dn);
      const TrainLayerLaunch q{rays, ray_stride, z, n_samples, c0, ein, n, gws, momentum, eps, s};
      launch_layer<KG_E, false>(q, P, ws.wp, ws.wh, ws.sw, 0, nullptr, none, h1 ? nullptr : hin, stats, nullptr,
                                ws.enc);
      enc_of_chunk = ws.enc;
    }
    for (int L = 1; L < 8; ++L) {
      if (keep) {
        hin = sc.h[L - 1];
        hout = sc.h[L];
      }
      const BnPrev prev{P.bn_w[L - 1], P.bn_b[L - 1], P.bn_rm[L - 1], P.bn_rv[L - 1], P.lin_b[L - 1],
                        stats + 512 * (L - 1)};
      if (L == 1 && h1) {
        ProfScope ps(s, PT_TRAIN_H1, 2.0 * (63 + 256) * 256 * dn, (256.0 + 1024.0) * dn);
        if (g_train_math == 1)
          hipLaunchKernelGGL(k_train_h1<3>, dim3(gws), dim3(512), 0, s, enc_of_chunk, n, ws.wh + off_h(1, false),
                             ws.wh + off_h(0, true), ws.sw, 1 | (tile_rev(1) << 8), P.lin_b[1], prev, momentum, eps,
                             hout, stats + 512);
        else
          hipLaunchKernelGGL(k_train_h1<4>, dim3(gws), dim3(512), 0, s, enc_of_chunk, n, ws.wh + off_h(1, false),
                             ws.wh + off_h(0, true), ws.sw, 1 | (tile_rev(1) << 8), P.lin_b[1], prev, momentum, eps,
                             hout, stats + 512);
      } else if (L == 4) {
        PCN_CHECK(enc_of_chunk, "skip layer launched without this chunk's first-layer encoding tiles");
        ProfScope ps(s, PT_TRAIN_SKIP, 2.0 * 319 * 256 * dn, (4.0 + 2048.0) * dn);
        const TrainLayerLaunch q{rays, ray_stride, z, n_samples, c0, ein, n, gws, momentum, eps, s};
        launch_layer<KG_E, true>(q, P, ws.wp, ws.wh, ws.sw, 4, hin, prev, hout, stats + 512 * L, enc_of_chunk,
                                 nullptr);
      } else {
        // algorithmic: 2*256*256 FLOP and 1 KiB in + 1 KiB out per sample
        ProfScope ps(s, PT_TRAIN_HIDDEN, 2.0 * 256 * 256 * dn, 2048.0 * dn);
        const TrainLayerLaunch q{rays, ray_stride, z, n_samples, c0, ein, n, gws, momentum, eps, s};
        launch_layer<0, true>(q, P, ws.wp, ws.wh, ws.sw, L, hin, prev, hout, stats + 512 * L, nullptr, nullptr);
      }
      float* t = hin;
      hin = hout;
      hout = t;
    }
    {
      const BnPrev prev{P.bn_w[7], P.bn_b[7], P.bn_rm[7], P.bn_rv[7], P.lin_b[7], stats + 512 * 7};
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

extern "C" int pcnerf_nof_query_train_store(const float* rays, int64_t n_rays, int ray_stride, const float* z,
                                            int n_samples, int64_t chunk, const pcnerf_nof_params* params,
                                            float momentum, float eps, void* workspace, size_t workspace_bytes,
                                            float* p_out, void* store, int64_t store_chunks, void* stream) {
  PCN_API_BEGIN
  PCN_CHECK(rays && z && params && workspace && p_out, "pcnerf_nof_query_train_store: null argument");
  PCN_CHECK(n_rays > 0 && n_samples > 0 && chunk > 0, "pcnerf_nof_query_train_store: empty input");
  PCN_CHECK(ray_stride >= 6, "pcnerf_nof_query_train_store: ray_stride < 6");
  PCN_CHECK(store_chunks == 0 || store, "pcnerf_nof_query_train_store: store_chunks > 0 needs a store");
  query_train(rays, ray_stride, z, n_samples, nullptr, n_rays * (int64_t)n_samples, chunk, params, momentum, eps,
              workspace, workspace_bytes, p_out, stream, store, store_chunks);
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

// =============================================================================================== backward
// dL/dparams of the train-mode query (loss.backward() through render.py:47-50 and models.py:183-203), given
// dL/dlogit per sample (or dL/dp with p).  Per chunk:
//   1. the forward's raw h_L of all 8 layers (1 KiB/sample each) and chunk statistics: from the activation store,
//      or recomputed with k_train_ws (running stats untouched); k_bn_save stores mean/invstd/alpha/beta;
//   2. occ_out + BatchNorm 8 backward (k_out_bwd_stats1, k_out_bwd_grad) -> dL/dh_7;
//   3. for L = 7..1: k_wgrad: G_L = sum_s dL/dh_L[s] (x) (h_{L-1}[s] - mean_{L-1})   (+ the encoding part at L=4)
//                    on MFMA, partials per block;  k_wgrad_reduce: dW_L = alpha*G + beta (x) db, db_L, and the
//                    statistics BatchNorm L-1's backward needs, which are algebraic in G and db:
//                      sum_s dL/dy = W^T db,   sum_s dL/dy (h - mean) = colsum(W o G);
//                    k_dgrad_ws: dL/dh_{L-1} = BN_back(W_L^T dL/dh_L) on MFMA, the BatchNorm backward fused into
//                    the epilogue (ATen's formula: (dy - mean(dy) - (h - mean) * k) * invstd * gamma);
//   4. k_wgrad / k_wgrad_reduce for layer 0 on the recomputed encoding.
// Parameter gradients accumulate in float64 across chunks and are added to the caller's fp32 buffers at the
// end (k_grad_emit).
namespace pcn {

constexpr size_t DGRAD_W_FLOATS = 7 * SZ_H;
constexpr int GMAX_SLOTS = 64;                     // per layer: atomicMax targets of the |dL/dh| maxima
constexpr int GMAX_DBL = 8 * GMAX_SLOTS / 2;       // their doubles in the per-chunk s12 region
constexpr int WG_BLOCKS = 256;  // weight-gradient partials per chunk (one 8-wave block per CU)

__host__ __device__ constexpr int in_features(int L) { return L == 0 ? 63 : L == 4 ? 319 : 256; }

// transposed weights for the data-gradient GEMM (neurons of layer L-1 on MFMA rows, samples on columns):
//   A (k-group kg, block ob, lane l, component q) = W_L[m = 8kg + 4(l>>5) + q][col0 + 32 ob + (l&31)]
__global__ void k_pack_dgrad(NofParamsDev P, float* __restrict__ out) {
  const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= DGRAD_W_FLOATS) return;
  const int L = 1 + (int)(idx / SZ_H);
  const size_t j = idx % SZ_H;
  const int q = (int)(j & 3), lane = (int)((j >> 2) & 63), ob = (int)((j >> 8) & 7), kg = (int)(j >> 11);
  const int m = 8 * kg + 4 * (lane >> 5) + q, nn = 32 * ob + (lane & 31);
  out[idx] = P.lin_w[L][(size_t)m * in_features(L) + (L == 4 ? 63 : 0) + nn];
}

// per layer: [mean(256), invstd(256), alpha = invstd*gamma (256), beta (256)] -- bn_coeffs' arithmetic
__global__ void k_bn_save(NofParamsDev P, const double* __restrict__ stats, int64_t n, float eps,
                          float* __restrict__ coef) {
  const int L = blockIdx.x, k = threadIdx.x;
  const double s1 = stats[512 * L + 2 * k], s2 = stats[512 * L + 2 * k + 1];
  const double m = s1 / (double)n;
  double var = s2 / (double)n - m * m;
  if (var < 0.0) var = 0.0;
  const float invstd = (float)(1.0 / sqrt(var + (double)eps));
  float* c = coef + 1024 * L;
  c[k] = (float)((double)P.lin_b[L][k] + m);
  c[256 + k] = invstd;
  c[512 + k] = invstd * P.bn_w[L][k];
  c[768 + k] = P.bn_b[L][k];
}

__device__ __forceinline__ float logit_grad(const float* __restrict__ g, const float* __restrict__ p, int64_t i) {
  if (!p) return g[i];
  const float pv = p[i];
  return g[i] * (1.0f - pv) * pv;  // sigmoid backward
}

// acc[f] += sum_s g_s (h7[s][f] - mean7[f]), acc[256] += sum_s g_s in one pass: each lane keeps all 128 of its
// half's feature sums over its tiles (two 16-load batches per tile in flight), reduces them across its 32 lanes with shuffles once at the end, and the
// block adds its totals to copy (block % OSTAT_COPIES) of acc (fewer blocks per address); k_out_bwd_grad sums the
// copies.
constexpr int OSTAT_COPIES = 8;
__global__ __launch_bounds__(256) void k_out_bwd_stats1(const float* __restrict__ g, const float* __restrict__ pin,
                                                        const float* __restrict__ h7, int64_t n,
                                                        const float* __restrict__ coef7, double* __restrict__ acc) {
  __shared__ __attribute__((aligned(16))) float mu[256];
  __shared__ float wsum[4][257];
  const int t = threadIdx.x, lane = t & 63, h = lane >> 5, li = lane & 31, wv = t >> 6;
  mu[t] = coef7[t];
  __syncthreads();
  const int64_t ntiles = (n + 31) / 32;
  float a[128];
#pragma unroll
  for (int i = 0; i < 128; ++i) a[i] = 0.0f;
  float gs = 0.0f;
  for (int64_t tile = (int64_t)blockIdx.x * 4 + wv; tile < ntiles; tile += (int64_t)gridDim.x * 4) {
    const int64_t s = tile * 32 + li;
    const float gv = s < n ? logit_grad(g, pin, s) : 0.0f;
    if (h == 0) gs += gv;
    const f32x4* x4 = reinterpret_cast<const f32x4*>(h7 + tile * TILE_FLOATS) + lane;
#pragma unroll
    for (int hb = 0; hb < 2; ++hb) {
      f32x4 x[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) x[j] = x4[(16 * hb + j) * 64];
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const int gq = 16 * hb + j;
        const f32x4 m = *reinterpret_cast<const f32x4*>(mu + 8 * gq + 4 * h);
#pragma unroll
        for (int q = 0; q < 4; ++q) a[4 * gq + q] += gv * (x[j][q] - m[q]);
      }
    }
  }
#pragma unroll
  for (int i = 0; i < 128; ++i) {
    float v = a[i];
#pragma unroll
    for (int o = 16; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);   // over the 32 lanes of this half
    a[i] = v;
  }
  if (li == 0) {
#pragma unroll
    for (int i = 0; i < 128; ++i) wsum[wv][8 * (i >> 2) + 4 * h + (i & 3)] = a[i];
  }
  gs = wave_sum_f(gs);
  if (lane == 0) wsum[wv][256] = gs;
  __syncthreads();
  double* ac = acc + (size_t)(blockIdx.x % OSTAT_COPIES) * 257;
  const double tot = (((double)wsum[0][t] + (double)wsum[1][t]) + ((double)wsum[2][t] + (double)wsum[3][t]));
  atomicAdd(&ac[t], tot);
  if (t == 0)
    atomicAdd(&ac[256], ((double)wsum[0][256] + (double)wsum[1][256]) + ((double)wsum[2][256] + (double)wsum[3][256]));
}

// dL/dh_7 = BN8_back(g_s * w_out); block 0 also accumulates d gamma_8, d beta_8, d w_out, d b_out.
__global__ __launch_bounds__(256) void k_out_bwd_grad(const float* __restrict__ g, const float* __restrict__ pin,
                                                      const float* __restrict__ h7, int64_t n,
                                                      const float* __restrict__ coef7, const float* __restrict__ gamma,
                                                      const float* __restrict__ wout, const double* __restrict__ acc,
                                                      double* __restrict__ d_gamma, double* __restrict__ d_beta,
                                                      double* __restrict__ d_wout, double* __restrict__ d_bout,
                                                      float* __restrict__ gout, float* __restrict__ tmax,
                                                      unsigned* __restrict__ gmax, int ncopies) {
  __shared__ __attribute__((aligned(16))) float cgm[256];
  __shared__ __attribute__((aligned(16))) float ckk[256];
  __shared__ __attribute__((aligned(16))) float cmu[256];
  __shared__ __attribute__((aligned(16))) float cis[256];
  __shared__ __attribute__((aligned(16))) float cga[256];
  __shared__ __attribute__((aligned(16))) float cwo[256];
  {
    const int k = threadIdx.x;
    double A = 0.0, G0 = 0.0;
#pragma unroll
    for (int c = 0; c < ncopies; ++c) {   // k_out_bwd_stats1's copies (or the fold's one)
      A += acc[257 * c + k];
      G0 += acc[257 * c + 256];
    }
    const float wo = wout[k], invstd = coef7[256 + k];
    const double S1 = (double)wo * G0, dotp = (double)wo * A;
    cgm[k] = (float)(S1 / (double)n);
    ckk[k] = (((float)dotp * invstd) * invstd) / (float)n;
    cmu[k] = coef7[k];
    cis[k] = invstd;
    cga[k] = gamma[k];
    cwo[k] = wo;
    if (blockIdx.x == 0) {
      d_gamma[k] += dotp * (double)invstd;
      d_beta[k] += S1;
      d_wout[k] += (double)coef7[512 + k] * A + (double)coef7[768 + k] * G0;
      if (k == 0) d_bout[0] += G0;
    }
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, h = lane >> 5, li = lane & 31;
  const int64_t ntiles = (n + 31) / 32;
  float gm = 0.0f;   // the wave's largest |dL/dh_7| over its tiles
  for (int64_t tile = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); tile < ntiles; tile += (int64_t)gridDim.x * 4) {
    const int64_t s = tile * 32 + li;
    const bool valid = s < n;
    const float gv = valid ? logit_grad(g, pin, s) : 0.0f;
    const f32x4* x4 = reinterpret_cast<const f32x4*>(h7 + tile * TILE_FLOATS) + lane;
    f32x4* o4 = reinterpret_cast<f32x4*>(gout + tile * TILE_FLOATS) + lane;
    f32x4 mq = {};   // per-q running maxima (four short dependency chains, not one of 128)
#pragma unroll 8
    for (int gq = 0; gq < 32; ++gq) {
      const f32x4 x = x4[gq * 64];
      const int f0 = 8 * gq + 4 * h;
      f32x4 o;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int f = f0 + q;
        o[q] = valid ? ((gv * cwo[f] - cgm[f]) - (x[q] - cmu[f]) * ckk[f]) * cis[f] * cga[f] : 0.0f;
        mq[q] = fmaxf(mq[q], fabsf(o[q]));
      }
      o4[gq * 64] = o;
    }
    if (tmax || gmax) {   // the tile's largest |dL/dh_7| (k_dgrad_h's per-tile operand scale) and the chunk's
      float mx = fmaxf(fmaxf(mq[0], mq[1]), fmaxf(mq[2], mq[3]));
      mx = wave_max_f(mx);
      if (tmax && lane < 8) tmax[tile * 8 + lane] = mx;
      gm = fmaxf(gm, mx);
    }
  }
  // non-negative floats order as their bits; one of GMAX_SLOTS addresses per wave (a single address would
  // serialise thousands of atomics), the consumer takes the max over the slots
  if (gmax && lane == 0) atomicMax(gmax + ((blockIdx.x * 4 + (threadIdx.x >> 6)) & (GMAX_SLOTS - 1)), __float_as_uint(gm));
}

// ---- weight gradient: G[m][n] = sum_s dL/dh_L[s][m] * X[s][n] over one chunk, partials per block.
// 8 waves per block, wave w owns rows m in [32w, 32w+32).  Per 32-sample tile both operands are staged in LDS
// as [sample][feature] (rows padded to 260 floats) so the MFMA reads contract over samples:
//   A (lane l, k-step t) = dL/dh[2t + (l>>5)][32w + (l&31)],  B (lane l) = X[2t + (l>>5)][32nb + (l&31)]
// X = h_{L-1} - mean_{L-1} (MODE 0), the encoding (MODE 1, 64 columns), or both (MODE 2, layer 4).  The next
// tile's operands are loaded into registers while the current one is multiplied (double-buffered LDS, one
// barrier per tile).  db[m] = sum_s dL/dh[s][m] comes free from the A reads.
constexpr int ES_ROW = 68;

template <int MODE>
struct WgradCfg {
  static constexpr bool HX = MODE != 1, EX = MODE != 0;
  static constexpr int C = (EX ? 64 : 0) + (HX ? 256 : 0);
  static constexpr int GS = 32 * LDS_ROW;
  static constexpr int BUF = GS + (HX ? GS : 0) + (EX ? 32 * ES_ROW : 0);
  static constexpr size_t LDS_BYTES = (size_t)(2 * BUF + 256 + 64) * sizeof(float);   // + mu, + encoding shift
  static constexpr size_t PART = (size_t)256 * C + 256;
  // k_wgrad_reduce: SPLIT slices of the partial list per column, RT threads per block
  static constexpr int SPLIT = C >= 1024 ? 1 : 1024 / C;
  static constexpr int RT = C * SPLIT;
};

// the chunk's encoding mean as float64 column sums (atomics into a zeroed acc[64]): k_wgrad's centring constant
__global__ __launch_bounds__(256) void k_enc_mean(const float* __restrict__ rays, int stride,
                                                  const float* __restrict__ z, int S, int64_t c0, int64_t n,
                                                  const float* __restrict__ ein, double* __restrict__ acc) {
  __shared__ double sh[4][64];
  double a[63];
#pragma unroll
  for (int k = 0; k < 63; ++k) a[k] = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    float f[64];
    if (ein) {
#pragma unroll
      for (int k = 0; k < 63; ++k) f[k] = ein[(c0 + i) * 63 + k];
    } else {
      float p[3];
      sample_point(rays + ray_of(c0 + i, S) * stride, z[c0 + i], p);
      encode_full(p, f);
    }
#pragma unroll
    for (int k = 0; k < 63; ++k) a[k] += (double)f[k];
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < 63; ++k) {
    const double v = wave_sum_d(a[k]);
    if (lane == 0) sh[w][k] = v;
  }
  __syncthreads();
  if (threadIdx.x < 63) {
    const int k = threadIdx.x;
    atomicAdd(acc + k, ((sh[0][k] + sh[1][k]) + (sh[2][k] + sh[3][k])));
  }
}

template <int MODE>
__global__ __launch_bounds__(512, 1) void k_wgrad(const float* __restrict__ rays, int stride,
                                                  const float* __restrict__ z, int S, int64_t c0, int64_t n,
                                                  const float* __restrict__ ein, const float* __restrict__ gin,
                                                  const float* __restrict__ hprev, const float* __restrict__ mu,
                                                  float* __restrict__ part, const double* __restrict__ esum) {
  using Cfg = WgradCfg<MODE>;
  constexpr bool HX = Cfg::HX, EX = Cfg::EX;
  constexpr int GS = Cfg::GS, BUF = Cfg::BUF, C = Cfg::C;
  CLK_ENTRY
  extern __shared__ __attribute__((aligned(16))) float lds[];
  float* mus = lds + 2 * BUF;
  // the encoding columns are contracted as g (x) (e - ebar), ebar the chunk's encoding mean (k_enc_mean; esum null:
  // 0): sum_s g = 0 exactly (BatchNorm follows the Linear), so the sum is the same, while a constant offset in g (the
  // fp32 rounding of its chunk mean) no longer multiplies n ebar -- it cancels, as in the fused paths' G = g (x) d
  float* esh = mus + 256;
  const int t = threadIdx.x, lane = t & 63, h = lane >> 5, li = lane & 31, wv = t >> 6;
  if (HX && t < 256) mus[t] = mu[t];
  if (EX && t < 64) esh[t] = (esum && t < 63) ? (float)(esum[t] / (double)n) : 0.0f;
  __syncthreads();
  const int64_t ntiles = (n + 31) / 32;
  f32x16 ah[8], ae[2];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
#pragma unroll
    for (int b = 0; b < 8; ++b) ah[b][r] = 0.0f;
    ae[0][r] = 0.0f;
    ae[1][r] = 0.0f;
  }
  float dbacc = 0.0f;
  f32x4 rg[4], rx[4];
  auto gload = [&](int64_t tile) {
    const f32x4* g4 = reinterpret_cast<const f32x4*>(gin + tile * TILE_FLOATS);
    const f32x4* x4 = reinterpret_cast<const f32x4*>((HX ? hprev : gin) + tile * TILE_FLOATS);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      rg[j] = g4[t + 512 * j];
      if (HX) rx[j] = x4[t + 512 * j];
    }
  };
  auto lstore = [&](float* buf, int64_t tile) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int i = t + 512 * j, g = i >> 6, lp = i & 63;
      const int off = (lp & 31) * LDS_ROW + 8 * g + 4 * (lp >> 5);
      *reinterpret_cast<f32x4*>(buf + off) = rg[j];
      if (HX) {
        const f32x4 m = *reinterpret_cast<const f32x4*>(mus + 8 * g + 4 * (lp >> 5));
        f32x4 x;
#pragma unroll
        for (int q = 0; q < 4; ++q) x[q] = rx[j][q] - m[q];
        *reinterpret_cast<f32x4*>(buf + GS + off) = x;
      }
    }
    if (EX) {
      float* row = buf + GS + (HX ? GS : 0) + (t >> 4) * ES_ROW;
      const int jj = t & 15;
      int64_t sl = tile * 32 + (t >> 4);
      if (sl >= n) sl = n - 1;
      const int64_t gi = c0 + sl;
      if (ein) {
        const float* er = ein + gi * 63;
        for (int f = jj; f < 64; f += 16) row[f] = f < 63 ? er[f] - esh[f] : 0.0f;
      } else {
        float p[3];
        sample_point(rays + ray_of(gi, S) * stride, z[gi], p);
        if (jj == 0) {
          row[0] = p[0] - esh[0];
          row[1] = p[1] - esh[1];
          row[2] = p[2] - esh[2];
          row[63] = 0.0f;
        }
        for (int q = jj; q < 30; q += 16) {
          const int k = q / 3, m = q - 3 * k;
          float sv, cv;
          sincosf((float)(1 << k) * p[m], &sv, &cv);  // encode_half's arithmetic
          row[3 + 6 * k + m] = sv - esh[3 + 6 * k + m];
          row[6 + 6 * k + m] = cv - esh[6 + 6 * k + m];
        }
      }
    }
  };
  int64_t tile = blockIdx.x;
  if (tile < ntiles) gload(tile);
  int bsel = 0;
  CLK_BEGIN
  for (; tile < ntiles; tile += gridDim.x) {
    float* buf = lds + bsel * BUF;
    lstore(buf, tile);
    __syncthreads();
    if (tile + gridDim.x < ntiles) gload(tile + gridDim.x);
    const float* xs = buf + GS;
    const float* xe = buf + GS + (HX ? GS : 0);
#pragma unroll
    for (int kt = 0; kt < 16; ++kt) {
      const int s = 2 * kt + h;
      const float a = buf[s * LDS_ROW + 32 * wv + li];
      dbacc += a;
      if (HX) {
#pragma unroll
        for (int nb = 0; nb < 8; ++nb)
          ah[nb] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, xs[s * LDS_ROW + 32 * nb + li], ah[nb], 0, 0, 0);
      }
      if (EX) {
#pragma unroll
        for (int nb = 0; nb < 2; ++nb)
          ae[nb] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, xe[s * ES_ROW + 32 * nb + li], ae[nb], 0, 0, 0);
      }
    }
    bsel ^= 1;
  }
  CLK_END
  float* pb = part + (size_t)blockIdx.x * Cfg::PART;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int m = 32 * wv + (r & 3) + 8 * (r >> 2) + 4 * h;
    if (EX) {
#pragma unroll
      for (int nb = 0; nb < 2; ++nb) pb[(size_t)m * C + 32 * nb + li] = ae[nb][r];
    }
    if (HX) {
#pragma unroll
      for (int nb = 0; nb < 8; ++nb) pb[(size_t)m * C + (EX ? 64 : 0) + 32 * nb + li] = ah[nb][r];
    }
  }
  dbacc += __shfl_xor(dbacc, 32, 64);
  if (h == 0) pb[(size_t)256 * C + 32 * wv + li] = dbacc;
  CLK_EXIT(MODE == 0 ? 2 : -1)
}

// Sum the partials of row m (block m; thread = column + C * slice, SPLIT slices of the partial list so every
// layer puts ~1024 threads, 8 loads each in flight, on the latency-bound sum), accumulate dW/db in float64 and the
// statistics of the BatchNorm below: s12[n] = (sum_m W[m][n] db[m], sum_m W[m][n] G[m][n]).
template <int MODE>
__device__ __forceinline__ void wgrad_reduce_body(const float* __restrict__ part, int nblk, const float* __restrict__ W,
                                                  const float* __restrict__ coefp, double* __restrict__ dW,
                                                  double* __restrict__ db, double* __restrict__ s12, int nblk_e,
                                                  int ldw) {
  // ldw: dW's row stride when it is not the layer's own (MODE 1 summing the skip layer's encoding columns: 319);
  // db may be null (no bias sum)
  using Cfg = WgradCfg<MODE>;
  constexpr int C = Cfg::C;
  constexpr int SPLIT = Cfg::SPLIT;
  const int in_f = ldw > 0 ? ldw : MODE == 0 ? 256 : MODE == 1 ? 63 : 319;
  constexpr int wcol_h = MODE == 2 ? 63 : 0, col_h = Cfg::EX ? 64 : 0;
  static_assert(C * SPLIT % 64 == 0, "whole waves");
  __shared__ double red[C * SPLIT];
  __shared__ double redw[C * SPLIT / 64];
  const int m = blockIdx.x, tt = threadIdx.x, t = tt % C, sl = tt / C;
  // the column sums first (32 loads per thread in flight at once: the sum is latency-bound otherwise), then the bias
  // row, reduced by wave shuffles -- one barrier
  double Gp[8] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
  const float* pc = part + (size_t)m * C + t;
  const int nbc = (Cfg::EX && t < 64) ? nblk_e : nblk;   // the encoding columns' own partial count (MODE 2)
  const int b0 = sl * ((nbc + SPLIT - 1) / SPLIT), b1 = min(nbc, b0 + (nbc + SPLIT - 1) / SPLIT);
  int b = b0;
  for (; b + 32 <= b1; b += 32) {
    float v[32];
#pragma unroll
    for (int j = 0; j < 32; ++j) v[j] = pc[(size_t)(b + j) * Cfg::PART];
#pragma unroll
    for (int j = 0; j < 32; ++j) Gp[j & 7] += (double)v[j];
  }
  for (; b + 8 <= b1; b += 8) {
#pragma unroll
    for (int j = 0; j < 8; ++j) Gp[j] += (double)pc[(size_t)(b + j) * Cfg::PART];
  }
  for (; b < b1; ++b) Gp[0] += (double)pc[(size_t)b * Cfg::PART];
  double G = ((Gp[0] + Gp[1]) + (Gp[2] + Gp[3])) + ((Gp[4] + Gp[5]) + (Gp[6] + Gp[7]));
  double d = 0.0;
  for (int bb = tt; bb < nblk; bb += C * SPLIT) d += (double)part[(size_t)bb * Cfg::PART + (size_t)256 * C + m];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) d += __shfl_xor(d, o, 64);
  if ((tt & 63) == 0) redw[tt >> 6] = d;
  if (SPLIT > 1) red[tt] = G;
  __syncthreads();
  double dbm = 0.0;
#pragma unroll
  for (int i = 0; i < C * SPLIT / 64; ++i) dbm += redw[i];
  if (SPLIT > 1) {
    if (sl != 0) return;
    for (int k = 1; k < SPLIT; ++k) G += red[t + C * k];
  }
  if (Cfg::EX && t < 64) {
    if (t < 63) dW[(size_t)m * in_f + t] += G;
  } else {
    const int nn = t - col_h;
    const size_t wi = (size_t)m * in_f + wcol_h + nn;
    dW[wi] += (double)coefp[512 + nn] * G + (double)coefp[768 + nn] * dbm;
    if (s12) {   // (the two-pass backward's BatchNorm-backward sums; the one-pass backward passes none)
      const double w = (double)W[wi];
      double* s12c = s12 + (m % S12_COPIES) * 512;   // 256 / COPIES blocks per address instead of 256
      atomicAdd(&s12c[2 * nn], w * dbm);
      atomicAdd(&s12c[2 * nn + 1], w * G);
    }
  }
  if (t == 0 && db) db[m] += dbm;
}

template <int MODE>
__global__ __launch_bounds__(1024) void k_wgrad_reduce(const float* __restrict__ part, int nblk, const float* __restrict__ W,
                               const float* __restrict__ coefp, double* __restrict__ dW, double* __restrict__ db,
                               double* __restrict__ s12, int nblk_e, int ldw = 0) {
  wgrad_reduce_body<MODE>(part, nblk, W, coefp, dW, db, s12, nblk_e, ldw);
}

// The one-pass backward's last sums of a chunk in one launch (blockIdx.y): layer 1's partials (k_wgrad_reduce<0>),
// layer 0's and the skip layer's encoding columns (k_wgrad_reduce<1>, the latter into rows of 319)
__global__ __launch_bounds__(1024) void k_fb_reduce_tail(const float* __restrict__ part1, const float* __restrict__ coef1,
                                                         double* __restrict__ dW1, double* __restrict__ db1,
                                                         const float* __restrict__ pe0, double* __restrict__ dW0,
                                                         double* __restrict__ db0, const float* __restrict__ pe4,
                                                         double* __restrict__ dW4, int np, int we) {
  static_assert(WgradCfg<0>::RT == 1024 && WgradCfg<1>::RT == 1024, "one block size for both sums");
  if (blockIdx.y == 0) wgrad_reduce_body<0>(part1, np, nullptr, coef1, dW1, db1, nullptr, np, 0);
  else if (blockIdx.y == 1) wgrad_reduce_body<1>(pe0, we, nullptr, nullptr, dW0, db0, nullptr, we, 0);
  else wgrad_reduce_body<1>(pe4, we, nullptr, nullptr, dW4, nullptr, nullptr, we, in_features(4));
}

// ---- k_dgrad_ws: the data gradient in the weight-stationary form of k_train_ws<0,true>.  A workgroup of 8 waves (two per
// SIMD) computes all 256 input features of one 32-sample tile at a time; wave b holds the W^T rows of features
// 32b..32b+31 (128 registers, loaded once per launch) as the A operand, the dL/dh tile is staged raw in LDS
// (double buffered, next tile's loads in flight), and the BatchNorm backward runs on the accumulators: register
// float4 4j..4j+3 of wave b is the output float4 at group 4b+j, whose h_{L-1} operand is the same [g][lane]
// float4 of the h tile (one 16-byte load per lane, issued during the k-loop), and the result goes to HBM straight
// from registers.  The previous tile's epilogue runs at k-groups 1-2 of the next tile's k-loop.
__global__ __launch_bounds__(512, 1) void k_dgrad_ws(
    const float* __restrict__ gin, const float* __restrict__ Wt, const float* __restrict__ hprev, int64_t n,
    const double* __restrict__ s12, const float* __restrict__ coefp, const float* __restrict__ gamma,
    double* __restrict__ d_gamma, double* __restrict__ d_beta, float* __restrict__ gout) {
  __shared__ __attribute__((aligned(16))) float cgm[256];
  __shared__ __attribute__((aligned(16))) float ckk[256];
  __shared__ __attribute__((aligned(16))) float cmu[256];
  __shared__ __attribute__((aligned(16))) float cis[256];
  __shared__ __attribute__((aligned(16))) float cga[256];
  __shared__ f32x4 xs[2][KG_H * 64];   // 2 x 32 KiB
  const int t = threadIdx.x;
  if (t < 256) {
    const int k = t;
    double S1 = 0.0, dotp = 0.0;
#pragma unroll
    for (int c = 0; c < S12_COPIES; ++c) {
      S1 += s12[512 * c + 2 * k];
      dotp += s12[512 * c + 2 * k + 1];
    }
    const float invstd = coefp[256 + k];
    cgm[k] = (float)(S1 / (double)n);
    ckk[k] = (((float)dotp * invstd) * invstd) / (float)n;
    cmu[k] = coefp[k];
    cis[k] = invstd;
    cga[k] = gamma[k];
    if (blockIdx.x == 0) {
      d_gamma[k] += dotp * (double)invstd;
      d_beta[k] += S1;
    }
  }
  const int nt = (int)((n + 31) / 32);
  const int gstride = (int)gridDim.x;
  const int lane = t & 63, h = lane >> 5, li = lane & 31;
  const int blk = __builtin_amdgcn_readfirstlane(t >> 6);
  f32x4 wr[KG_H];
  {
    const f32x4* __restrict__ w4 = reinterpret_cast<const f32x4*>(Wt) + lane;
#pragma unroll
    for (int kg = 0; kg < KG_H; ++kg) wr[kg] = w4[(kg * 8 + blk) * 64];
  }
  int tl = __builtin_amdgcn_readfirstlane((int)blockIdx.x);
  if (tl < nt) {
    f32x4 v[4];
#pragma unroll
    for (int m = 0; m < 4; ++m)
      v[m] = reinterpret_cast<const f32x4*>(gin + (size_t)tl * TILE_FLOATS + (size_t)m * 2048)[t];
#pragma unroll
    for (int m = 0; m < 4; ++m) xs[0][t + 512 * m] = v[m];
  }
  __syncthreads();
  __builtin_amdgcn_s_waitcnt(0);   // weights resident before the tile loop (see k_train_ws)
  int buf = 0;
  auto epi = [&](const f32x16& pacc, const f32x4 (&hx)[4], int ptile, int j) {
    const bool valid = (int64_t)ptile * 32 + li < n;
    const int f0 = 8 * (4 * blk + j) + 4 * h;
    const f32x4 gm = *reinterpret_cast<const f32x4*>(cgm + f0), kk = *reinterpret_cast<const f32x4*>(ckk + f0);
    const f32x4 mu = *reinterpret_cast<const f32x4*>(cmu + f0), is = *reinterpret_cast<const f32x4*>(cis + f0);
    const f32x4 ga = *reinterpret_cast<const f32x4*>(cga + f0);
    f32x4 o;
#pragma unroll
    for (int q = 0; q < 4; ++q)
      o[q] = valid ? ((pacc[4 * j + q] - gm[q]) - (hx[j][q] - mu[q]) * kk[q]) * is[q] * ga[q] : 0.0f;
    reinterpret_cast<f32x4*>(gout + (size_t)ptile * TILE_FLOATS + (size_t)(4 * blk + j) * 256)[lane] = o;
  };
  auto body = [&](f32x16& acc, f32x4 (&hx)[4], const f32x16& pacc, const f32x4 (&phx)[4], int tile, int ptile) {
    const int nxt = __builtin_amdgcn_readfirstlane(tile + gstride);
    const bool more = nxt < nt;
    const f32x4* xb = &xs[buf][lane];
    f32x4 xr[WS_XD];
    f32x4 v[4];
#pragma unroll
    for (int d = 0; d < WS_XD - 1; ++d) xr[d] = xb[d * 64];
#pragma unroll
    for (int kg = 0; kg < KG_H; ++kg) {
      if (kg + WS_XD - 1 < KG_H) xr[(kg + WS_XD - 1) % WS_XD] = xb[(kg + WS_XD - 1) * 64];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const f32x16 c = (kg == 0 && q == 0) ? f32x16{} : acc;
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(wr[kg][q], xr[kg % WS_XD][q], c, 0, 0, 0);
      }
      if (kg == 1 && ptile >= 0) {
        epi(pacc, phx, ptile, 0);
        epi(pacc, phx, ptile, 1);
      }
      if (kg == 2 && ptile >= 0) {
        epi(pacc, phx, ptile, 2);
        epi(pacc, phx, ptile, 3);
      }
      if (kg == 3 && more) {
#pragma unroll
        for (int m = 0; m < 4; ++m)
          v[m] = reinterpret_cast<const f32x4*>(gin + (size_t)nxt * TILE_FLOATS + (size_t)m * 2048)[t];
      }
      if (kg == 22 && more) {
        xs[buf ^ 1][t] = v[0];
        xs[buf ^ 1][t + 512] = v[1];
      }
      if (kg == 23 && more) {
        xs[buf ^ 1][t + 1024] = v[2];
        xs[buf ^ 1][t + 1536] = v[3];
      }
      if (kg == 24) {   // this tile's h_{L-1} operand of the BatchNorm backward (epilogue at the next tile)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          hx[j] = reinterpret_cast<const f32x4*>(hprev + (size_t)tile * TILE_FLOATS + (size_t)(4 * blk + j) * 256)[lane];
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    __syncthreads();
    buf ^= 1;
  };
  f32x16 accA, accB;
  f32x4 hxA[4], hxB[4];
  int ptile = -1;
  while (tl < nt) {
    body(accA, hxA, accB, hxB, tl, ptile);
    ptile = tl;
    tl = __builtin_amdgcn_readfirstlane(tl + gstride);
    if (tl >= nt) {
#pragma unroll
      for (int j = 0; j < 4; ++j) epi(accA, hxA, ptile, j);
      break;
    }
    body(accB, hxB, accA, hxA, tl, ptile);
    ptile = tl;
    tl = __builtin_amdgcn_readfirstlane(tl + gstride);
    if (tl >= nt) {
#pragma unroll
      for (int j = 0; j < 4; ++j) epi(accB, hxB, ptile, j);
    }
  }
}

// ---- Backward under the split train math (pcnerf_set_train_math 1/2).
//
// k_dgrad_h<NT>: k_dgrad_ws's product dL/dy = W^T dL/dh on the fp16 matrix pipe, in k_train_h's form (W^T resident
// as hi/mid fp16 parts x 2^sw, the dL/dh tile staged split into LDS, NT products per k-step).  dL/dh has no bound
// known before it exists, so its producer (k_out_bwd_grad, or the previous k_dgrad_h) records every tile's largest
// |value| (tmax[tile][8], one entry per wave) and the staging scales the tile by 2^sg with that max x 2^sg in
// [2^14, 2^15): a per-tile scale factors out of the tile's own product (the accumulator is per tile) and is undone
// in its epilogue.  The epilogue is k_dgrad_ws's BatchNorm backward; it records the output tile's max for the next
// layer.
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ int tile_scale_exp(float m) {
  if (!(m > 0.0f) || !(m < 3.0e38f)) return 0;   // zero, NaN or inf tiles: unscaled
  int e = 14 - ilogbf(m);
  return e < -100 ? -100 : e > 100 ? 100 : e;
}

// W^T image for k_dgrad_h: layer L (1..7) at (L-1) HW_H, [ks][out-block 8][part 2][lane 64] f16x8, row i = input
// feature 32 ob + (lane & 31) of layer L, k = neuron 16 ks + 8 (lane >> 5) + e; scaled by 2^sw[L] like the forward
__global__ void k_pack_dgrad_h(NofParamsDev P, const int* __restrict__ sw, f16x8* __restrict__ out) {
  const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= 7 * HW_H) return;
  const int L = 1 + (int)(idx / HW_H);
  const size_t j = idx % HW_H;
  const int lane = (int)(j & 63), part = (int)((j >> 6) & 1), ob = (int)((j >> 7) & 7), ks = (int)(j >> 10);
  const int i = 32 * ob + (lane & 31), in_f = in_features(L), col = (L == 4 ? 63 : 0) + i;
  const float sc = ldexpf(1.0f, sw[L]);
  f16x8 v;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int k = 16 * ks + 8 * (lane >> 5) + e;
    const float w = P.lin_w[L][(size_t)k * in_f + col] * sc;
    const _Float16 hi = (_Float16)w;
    v[e] = part == 0 ? hi : (_Float16)(w - (float)hi);
  }
  out[idx] = v;
}

template <int NT>
__global__ __launch_bounds__(512, 1) void k_dgrad_h(
    const float* __restrict__ gin, const float* __restrict__ tmax_in, const f16x8* __restrict__ Wt,
    const int* __restrict__ swp, int layer, const float* __restrict__ hprev, int64_t n,
    const double* __restrict__ s12, const float* __restrict__ coefp, const float* __restrict__ gamma,
    double* __restrict__ d_gamma, double* __restrict__ d_beta, float* __restrict__ gout,
    float* __restrict__ tmax_out, unsigned* __restrict__ gmax_out) {
  constexpr int KS = KS_H, XD = H_XD;
  float gm = 0.0f;   // the wave's largest |dL/dh_{L-1}| over its tiles (k_wgrad_b3's chunk-wide scale)
  constexpr int S_LOAD = H_LOAD, S_STAGE0 = KS - H_STAGE, S_STAGE1 = S_STAGE0 + 1, S_HX = 8;
  __shared__ __attribute__((aligned(16))) float cgm[256];
  __shared__ __attribute__((aligned(16))) float ckk[256];
  __shared__ __attribute__((aligned(16))) float cmu[256];
  __shared__ __attribute__((aligned(16))) float cis[256];
  __shared__ __attribute__((aligned(16))) float cga[256];
  __shared__ f16x8 xs[2][KS][2][64];
  const int t = threadIdx.x;
  if (t < 256) {
    const int k = t;
    double S1 = 0.0, dotp = 0.0;
#pragma unroll
    for (int c = 0; c < S12_COPIES; ++c) {
      S1 += s12[512 * c + 2 * k];
      dotp += s12[512 * c + 2 * k + 1];
    }
    const float invstd = coefp[256 + k];
    cgm[k] = (float)(S1 / (double)n);
    ckk[k] = (((float)dotp * invstd) * invstd) / (float)n;
    cmu[k] = coefp[k];
    cis[k] = invstd;
    cga[k] = gamma[k];
    if (blockIdx.x == 0) {
      d_gamma[k] += dotp * (double)invstd;
      d_beta[k] += S1;
    }
  }
  const float wunscale = ldexpf(1.0f, -swp[layer]);
  const int nt = (int)((n + 31) / 32);
  const int gstride = (int)gridDim.x;
  const int lane = t & 63, h = lane >> 5, li = lane & 31;
  const int blk = __builtin_amdgcn_readfirstlane(t >> 6);
  if (blk >= 4) __builtin_amdgcn_s_setprio(1);
  f16x8 wr[KS][2];
  {
    const f16x8* __restrict__ w8 = Wt + lane;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int p = 0; p < 2; ++p) wr[ks][p] = w8[((ks * 8 + blk) * 2 + p) * 64];
  }
  auto tile_exp = [&](int tile) {
    const f32x4* tm = reinterpret_cast<const f32x4*>(tmax_in + (size_t)tile * 8);
    const f32x4 a = tm[0], b = tm[1];
    const float m = fmaxf(fmaxf(fmaxf(a[0], a[1]), fmaxf(a[2], a[3])), fmaxf(fmaxf(b[0], b[1]), fmaxf(b[2], b[3])));
    return __builtin_amdgcn_readfirstlane(tile_scale_exp(m));
  };
  // staging: thread t's float4s t + 512 m of the tile (feature group g = (t >> 6) + 8 m, lane t & 63), scaled by
  // 2^sg and split -> LDS [s = g >> 1][part][li + 32 (g & 1)][4 h ..], as k_train_h's put
  auto stage = [&](int b, const f32x4 (&v)[4], int m, float xscale) {
    const int g = (t >> 6) + 8 * m;
    f32x4 x;
#pragma unroll
    for (int q = 0; q < 4; ++q) x[q] = v[m][q] * xscale;
    f16x4 hi, mid;
    split4(x, hi, mid);
    const int s = g >> 1, ln = li + 32 * (g & 1);
    *reinterpret_cast<f16x4*>(reinterpret_cast<_Float16*>(&xs[b][s][0][ln]) + 4 * h) = hi;
    *reinterpret_cast<f16x4*>(reinterpret_cast<_Float16*>(&xs[b][s][1][ln]) + 4 * h) = mid;
  };
  auto load_tile = [&](f32x4 (&v)[4], int tile) {
#pragma unroll
    for (int m = 0; m < 4; ++m) v[m] = reinterpret_cast<const f32x4*>(gin + (size_t)tile * TILE_FLOATS)[t + 512 * m];
  };
  int tl = __builtin_amdgcn_readfirstlane((int)blockIdx.x);
  int sg = 0;
  if (tl < nt) {
    sg = tile_exp(tl);
    f32x4 v[4];
    load_tile(v, tl);
    const float xscale = ldexpf(1.0f, sg);
#pragma unroll
    for (int m = 0; m < 4; ++m) stage(0, v, m, xscale);
  }
  __syncthreads();
  __builtin_amdgcn_s_waitcnt(0);
  int buf = 0;
  auto epi = [&](const f32x16& acc, const f32x4 (&hx)[4], int tile, float unscale) {
    const bool valid = (int64_t)tile * 32 + li < n;
    float mx = 0.0f;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int f0 = 8 * (4 * blk + j) + 4 * h;
      const f32x4 gm = *reinterpret_cast<const f32x4*>(cgm + f0), kk = *reinterpret_cast<const f32x4*>(ckk + f0);
      const f32x4 mu = *reinterpret_cast<const f32x4*>(cmu + f0), is = *reinterpret_cast<const f32x4*>(cis + f0);
      const f32x4 ga = *reinterpret_cast<const f32x4*>(cga + f0);
      f32x4 o;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float d = (acc[4 * j + q] * wunscale) * unscale;
        o[q] = valid ? ((d - gm[q]) - (hx[j][q] - mu[q]) * kk[q]) * is[q] * ga[q] : 0.0f;
        mx = fmaxf(mx, fabsf(o[q]));
      }
      reinterpret_cast<f32x4*>(gout + (size_t)tile * TILE_FLOATS + (size_t)(4 * blk + j) * 256)[lane] = o;
    }
    mx = wave_max_f(mx);
    if (lane == 0) tmax_out[(size_t)tile * 8 + blk] = mx;
    gm = fmaxf(gm, mx);
  };
  while (tl < nt) {
    const int nxt = __builtin_amdgcn_readfirstlane(tl + gstride);
    const bool more = nxt < nt;
    const float unscale = ldexpf(1.0f, -sg);
    int sgn = 0;
    f32x16 acc;
    f16x8 xr[XD][2];
    f32x4 vloc[4], hx[4];
#pragma unroll
    for (int d = 0; d < XD - 1; ++d) {
      xr[d][0] = xs[buf][d][0][lane];
      xr[d][1] = xs[buf][d][1][lane];
    }
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      if (ks + XD - 1 < KS) {
        xr[(ks + XD - 1) % XD][0] = xs[buf][ks + XD - 1][0][lane];
        xr[(ks + XD - 1) % XD][1] = xs[buf][ks + XD - 1][1][lane];
      }
      const f16x8 xh = xr[ks % XD][0], xm = xr[ks % XD][1];
      acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(wr[ks][0], xh, ks == 0 ? f32x16{} : acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(wr[ks][0], xm, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(wr[ks][1], xh, acc, 0, 0, 0);
      if (NT == 4) acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(wr[ks][1], xm, acc, 0, 0, 0);
      if (ks == S_LOAD && more) {
        load_tile(vloc, nxt);
        sgn = tile_exp(nxt);
      }
      if (ks == S_HX) {   // this tile's h_{L-1} operand of the BatchNorm backward
#pragma unroll
        for (int j = 0; j < 4; ++j)
          hx[j] = reinterpret_cast<const f32x4*>(hprev + (size_t)tl * TILE_FLOATS + (size_t)(4 * blk + j) * 256)[lane];
      }
      if (ks == S_STAGE0 && more) {
        const float xscale = ldexpf(1.0f, sgn);
        stage(buf ^ 1, vloc, 0, xscale);
        stage(buf ^ 1, vloc, 1, xscale);
      }
      if (ks == S_STAGE1 && more) {
        const float xscale = ldexpf(1.0f, sgn);
        stage(buf ^ 1, vloc, 2, xscale);
        stage(buf ^ 1, vloc, 3, xscale);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    epi(acc, hx, tl, unscale);
    __syncthreads();
    buf ^= 1;
    sg = sgn;
    tl = nxt;
  }
  if (gmax_out && lane == 0) atomicMax(gmax_out + ((blockIdx.x * 8 + blk) & (GMAX_SLOTS - 1)), __float_as_uint(gm));
}

// k_wgrad_b3<RB, MODE>: k_wgrad<MODE>'s G = sum_s dL/dh (x) x with each fp32 operand split into three bf16 parts
// (v = hi + mid + lo: all 24 bits of the fp32 value, bf16 keeps fp32's exponent range, so no scaling) and the six
// products down to 2^-16 (hh, hm, mh, hl, lh, mm) on v_mfma_f32_32x32x16_bf16: the dropped ml, lm, ll are
// <= 2^-23 relative, like fp32 rounding.  x = h_{L-1} - mean (MODE 0, hidden layers), the encoding (MODE 1, layer
// 0) or both (MODE 2, the skip layer: encoding columns first, as k_wgrad).  The contraction runs over samples, 16
// per k-step, so the unit of work is a half tile (16 samples, one k-step), and an operand lane needs 8 consecutive
// samples of one feature.  Every thread loads 2 float4 of each operand per half tile (256-byte coalesced runs of
// the tile's [g][lane][4] order) and stages them into a ring of three LDS buffers, two half tiles ahead:
//   x (B operand, read by all 8 waves): split, each part stored as [sample 16][feature] bf16 rows (pitch 2 x the
//     feature count + 64 B); 16-byte chunk c of row r at (c ^ ((r >> 1) & 3)) and its 8-byte halves swapped when
//     r & 8: conflict-free 8-byte writes, and ds_read_b64_tr_b16 reads (4 consecutive samples of the lane's
//     feature, two per part) that are conflict-free and affine in the column block (immediate offsets); the
//     encoding columns are computed while staging (enc_feats from the ray row, or the stored embedding row);
//   dL/dh (A operand, read by its wave only): copied raw ([g][half][sample ^ c][4], c = 2 (g & 3) + half:
//     conflict-free 4-byte reads), each wave splitting its 8 values per half tile itself.
// One barrier per half tile.  Partials and db in k_wgrad<MODE>'s layout (k_wgrad_reduce<MODE> sums them).
// MODE 3 (DUAL): the encoding columns of TWO layers in one pass -- layer 0's G on dL/dh_0 (gin) and the skip layer's
// encoding columns on dL/dh_4 (gin2, a second partial set part2 in layer 0's layout, no db) -- sharing the staged
// encoding (one sincos pass) and each half tile's barrier.
template <int MODE, bool H2 = false>
struct Wb3Cfg {
  static constexpr bool HX = MODE != 1 && MODE != 3, EX = MODE != 0, DUAL = MODE == 3;
  static constexpr int NPART = H2 ? 2 : 3;                         // operand parts: f16 hi/mid or bf16 hi/mid/lo
  static constexpr int NBLK = (EX ? 2 : 0) + (HX ? 8 : 0);        // 32-column blocks of G
  static constexpr int PITCH = 64 * NBLK + 64;                     // x row bytes: 576, 192, 704
  static constexpr int XPART = 16 * PITCH;
  static constexpr int GB1 = 16 * 256 * 4;                         // raw dL/dh bytes per half tile (per source)
  static constexpr int GB = (DUAL ? 2 : 1) * GB1;
  static constexpr size_t BUF = (size_t)GB + NPART * XPART;
  static constexpr size_t LDS = 3 * BUF;
};

typedef short s16x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void split3_bf16(const float (&v)[8], bf16x8& hi, bf16x8& mid, bf16x8& lo) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const __bf16 a = (__bf16)v[j];
    const float r = v[j] - (float)a;   // exact (Sterbenz)
    const __bf16 b = (__bf16)r;
    hi[j] = a;
    mid[j] = b;
    lo[j] = (__bf16)(r - (float)b);
  }
}

__device__ __forceinline__ void split3_x4(const f32x4& v, s16x4& p0, s16x4& p1, s16x4& p2) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const __bf16 a = (__bf16)v[q];
    const float r = v[q] - (float)a;
    const __bf16 bb = (__bf16)r;
    p0[q] = __builtin_bit_cast(short, a);
    p1[q] = __builtin_bit_cast(short, bb);
    p2[q] = __builtin_bit_cast(short, (__bf16)(r - (float)bb));
  }
}

// hi = fp16(v), mid = fp16(v - hi) for a pair of values: the pair's hi parts by one packed conversion, each mid by
// ONE mixed-precision fma (v_fma_mix{lo,hi}_f16 with the f16 hi operand selected by op_sel): v - hi is exact in
// fp32, so this is the same single rounding as converting the fp32 difference, bit for bit (nof_eval.hip's
// eh_split8; scripts/micro/split_mix.hip checked it over 67M values) -- 3 instructions a pair instead of ~10
__device__ __forceinline__ void split2_pair(float a, float b, unsigned& hb, unsigned& mb) {
  typedef _Float16 h2 __attribute__((ext_vector_type(2)));
  h2 hp;
  hp[0] = (_Float16)a;
  hp[1] = (_Float16)b;
  hb = __builtin_bit_cast(unsigned, hp);
  asm("v_fma_mixlo_f16 %0, %1, -1.0, %2 op_sel_hi:[1,0,0]" : "=v"(mb) : "v"(hb), "v"(a));
  asm("v_fma_mixhi_f16 %0, %1, -1.0, %2 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "+v"(mb) : "v"(hb), "v"(b));
}

__device__ __forceinline__ void split2_x4(const f32x4& v, s16x4& p0, s16x4& p1) {
  typedef unsigned u32x2_ __attribute__((ext_vector_type(2)));
  unsigned h0, m0, h1, m1;
  split2_pair(v[0], v[1], h0, m0);
  split2_pair(v[2], v[3], h1, m1);
  p0 = __builtin_bit_cast(s16x4, u32x2_{h0, h1});
  p1 = __builtin_bit_cast(s16x4, u32x2_{m0, m1});
}

__device__ __forceinline__ void split2_f16(const float (&v)[8], f16x8& hi, f16x8& mid) {
  typedef unsigned u32x4_ __attribute__((ext_vector_type(4)));
  unsigned h[4], m[4];
#pragma unroll
  for (int p = 0; p < 4; ++p) split2_pair(v[2 * p], v[2 * p + 1], h[p], m[p]);
  hi = __builtin_bit_cast(f16x8, u32x4_{h[0], h[1], h[2], h[3]});
  mid = __builtin_bit_cast(f16x8, u32x4_{m[0], m[1], m[2], m[3]});
}

// byte offset of features f .. f+3 (f % 4 == 0) of row r (sample within the half tile) in one x part
template <int PITCH>
__device__ __forceinline__ int wb3_xoff(int r, int f) {
  const int c = (f >> 3) ^ ((r >> 1) & 3);
  const int half = ((f >> 2) & 1) ^ ((r >> 3) & 1);
  return r * PITCH + 16 * c + 8 * half;
}

// RB: row blocks (32 features of dL/dh) per wave; 8 / RB waves per workgroup.  LAY: the k_wgrad mode whose partial
// layout is written -- the skip layer (LAY 2) runs MODE 0 (its h columns, at column 64, and db) and MODE 1 (its
// encoding columns): its 10 column blocks would not fit the accumulator registers of one launch
// H2: the f16x2 form (NT products of two fp16 parts, as the forward): dL/dh scaled by 2^sg from the chunk's
// largest |dL/dh| (`gmax`, recorded by the producer), x per column by 2^sx from its own bound (the Samuelson bound
// sqrt(n) / invstd of h - mean; 2^14 for the encoding's sin/cos, 1 for its xyz), both undone on the partials.
template <int RB, int MODE, int LAY, bool H2, int NTP>
__global__ __launch_bounds__(512 / RB, 1) void k_wgrad_b3(const float* __restrict__ rays, int stride,
                                                          const float* __restrict__ z, int S, int64_t c0,
                                                          const float* __restrict__ ein,
                                                          const float* __restrict__ gin,
                                                          const float* __restrict__ hprev,
                                                          const float* __restrict__ mu, int64_t n,
                                                          const unsigned* __restrict__ gmax,
                                                          float* __restrict__ part,
                                                          const unsigned* __restrict__ pbound,
                                                          const float* __restrict__ gin2,
                                                          const unsigned* __restrict__ gmax2,
                                                          float* __restrict__ part2) {
  using Cfg = Wb3Cfg<MODE, H2>;
  constexpr int NPART = Cfg::NPART;
  constexpr bool HX = Cfg::HX, EX = Cfg::EX, DUAL = Cfg::DUAL;
  constexpr int GB1 = Cfg::GB1;
  constexpr int NBLK = Cfg::NBLK, PITCH = Cfg::PITCH, XPART = Cfg::XPART, GB = Cfg::GB;
  constexpr int NT = 512 / RB, NI = 2 * RB;   // threads; float4 per thread per operand and half tile
  constexpr int HOFF = EX ? 64 : 0;           // first h feature column in the x image
  using P8 = std::conditional_t<H2, f16x8, bf16x8>;   // operand part type
  extern __shared__ __attribute__((aligned(16))) float wb3[];
  const int t = threadIdx.x, lane = t & 63, h = lane >> 5, li = lane & 31;
  // H2: per-column scales of G (x operand) after the three buffers; dL/dh's chunk-wide scale
  float* const csc = wb3 + 3 * Cfg::BUF / 4;
  float* const cun = csc + NBLK * 32;
  float gsc = 1.0f, gun = 1.0f, gsc2 = 1.0f, gun2 = 1.0f;
  if constexpr (H2) {
    for (int c = t; c < NBLK * 32; c += 512 / RB) {
      int e;
      if (EX && c < 64) {
        // |sin|, |cos| <= 1; xyz by the call's largest |position| (k_pos_bound, on the device: no host sync)
        e = (c >= 3 && c < 63) ? 14 : 0;
        if (c < 3 && pbound) {
          const float pm = __uint_as_float(*pbound);
          e = (pm > 0.0f && pm < 3.0e38f) ? 14 - ilogbf(pm) : 0;
          e = e < -60 ? -60 : e > 60 ? 60 : e;
        }
      } else {
        const float invstd = mu[256 + (c - HOFF)];
        const float bnd = sqrtf((float)n) / invstd;   // Samuelson: |h - mean| <= sqrt(n) sigma
        e = (bnd > 0.0f && bnd < 3.0e38f) ? 14 - ilogbf(bnd) : 0;
        e = e < -60 ? -60 : e > 60 ? 60 : e;
      }
      csc[c] = ldexpf(1.0f, e);
      cun[c] = ldexpf(1.0f, -e);
    }
    unsigned gm = 0;
    for (int i = 0; i < GMAX_SLOTS; ++i) gm = max(gm, gmax[i]);   // (uniform loads)
    const int eg = tile_scale_exp(__uint_as_float(gm));
    gsc = ldexpf(1.0f, eg);
    gun = ldexpf(1.0f, -eg);
    if constexpr (DUAL) {
      unsigned gm2 = 0;
      for (int i = 0; i < GMAX_SLOTS; ++i) gm2 = max(gm2, gmax2[i]);
      const int eg2 = tile_scale_exp(__uint_as_float(gm2));
      gsc2 = ldexpf(1.0f, eg2);
      gun2 = ldexpf(1.0f, -eg2);
    }
    __syncthreads();
  }
  const int wv = __builtin_amdgcn_readfirstlane(t >> 6);
  const int nt = (int)((n + 31) / 32);
  const int gstride = (int)gridDim.x;
  const int tb = (int)(TILE_FLOATS * 4);
  // staging map: float4 idx = t + NT i (i < NI) of a half tile hs: feature group sg = idx >> 5, HBM lane
  // 32 shh + 16 hs + sl (shh = (idx >> 4) & 1, sl = idx & 15); buffer loads, offsets in SGPRs + one VGPR
  const int sl = t & 15, shh = (t >> 4) & 1, sg0 = t >> 5;   // sg = sg0 + (NT / 32) i
  // encoding staging (EX): row er = t & 15, sincos task ej = t >> 4
  const int er = t & 15, ej = t >> 4;
  const __amdgpu_buffer_rsrc_t rg = __builtin_amdgcn_make_buffer_rsrc((void*)gin, (short)0, nt * tb, 0x00020000);
  const __amdgpu_buffer_rsrc_t rx =   // (DUAL: the second dL/dh)
      __builtin_amdgcn_make_buffer_rsrc((void*)(HX ? hprev : DUAL ? gin2 : gin), (short)0, nt * tb, 0x00020000);
  const int voff = (sg0 * 64 + 32 * shh + sl) * 16;
  constexpr int NR = 2 * NI + (EX ? 2 : 0);   // staging registers (float4): dL/dh, x, ray row + z
  auto sample_of = [&](int tile, int hs) {
    int64_t s = (int64_t)tile * 32 + 16 * hs + er;
    if (s >= n) s = n - 1;
    return c0 + s;
  };
  auto load_half = [&](f32x4 (&rv)[NR], int tile, int hs) {
    const int so = tile * tb + hs * 256;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      rv[i] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rg, voff, so + NT * 32 * i, 0));
      if (HX || DUAL)
        rv[NI + i] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rx, voff, so + NT * 32 * i, 0));
    }
    if constexpr (EX) {   // the sample's ray origin, direction and z
      if (ein) return;
      const int64_t gs = sample_of(tile, hs);
      // (32-bit division when it fits: the 64-bit one is a long emulated sequence per thread and half tile; the
      // ray row's first four floats as one 4-byte-aligned vector load)
      const int64_t ray = ray_of(gs, S);
      const float* r = rays + ray * stride;
      typedef float f32x4u __attribute__((ext_vector_type(4), aligned(4)));
      const f32x4u r4 = *reinterpret_cast<const f32x4u*>(r);
      rv[2 * NI] = f32x4{r4[0], r4[1], r4[2], r4[3]};
      rv[2 * NI + 1] = f32x4{r[4], r[5], z[gs], 0.0f};
    }
  };
  f32x4 mu2[NI];
#pragma unroll
  for (int i = 0; i < NI; ++i)
    mu2[i] = HX ? *reinterpret_cast<const f32x4*>(mu + 8 * (sg0 + (NT / 32) * i) + 4 * shh) : f32x4{};
  // staging pieces of a half tile: k < NI the dL/dh float4 k; NI <= k < 2 NI the x float4 k - NI (HX); the
  // encoding piece last (EX)
  constexpr int NP = NI * (HX || DUAL ? 2 : 1) + (EX ? 1 : 0);
  auto stage_piece = [&](int b, const f32x4 (&rv)[NR], int tile, int hs, int k) {
    char* base = reinterpret_cast<char*>(wb3) + (size_t)b * Cfg::BUF;
    char* xb = base + GB;
    if (k < NI || (DUAL && k < 2 * NI)) {   // raw dL/dh (DUAL: the second source GB1 further)
      const int kk = k < NI ? k : k - NI;
      const int g = sg0 + (NT / 32) * kk, c = 2 * (g & 3) + shh;
      char* bb = base + (k < NI ? 0 : GB1);
      *reinterpret_cast<f32x4*>(reinterpret_cast<float*>(bb) + g * 128 + shh * 64 + (sl ^ c) * 4) = rv[k];
      return;
    }
    s16x4 p0 = {}, p1 = {}, p2 = {};
    int off = 0;
    if (HX && k < 2 * NI) {
      const int i = (k - NI) & (NI - 1), g = sg0 + (NT / 32) * i;
      const bool valid = (int64_t)tile * 32 + 16 * hs + sl < n;
      f32x4 v;
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] = valid ? rv[(NI + i) % NR][q] - mu2[i][q] : 0.0f;
      if constexpr (H2) {
        const f32x4 sc = *reinterpret_cast<const f32x4*>(csc + HOFF + 8 * g + 4 * shh);
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] *= sc[q];
        split2_x4(v, p0, p1);
      } else {
        split3_x4(v, p0, p1, p2);
      }
      off = wb3_xoff<PITCH>(sl, HOFF + 8 * g + 4 * shh);
    } else if constexpr (EX) {
      // one sincos per thread: row er, task ej < 30 -> 2^k p[m] (k = ej / 3, m = ej % 3) feeding features
      // 3 + 6 k + m (sin) and 6 + 6 k + m (cos); ej == 30: x, y, z and the zero pad 63; ej == 31 idle
      const bool valid = (int64_t)tile * 32 + 16 * hs + er < n;
      const int64_t gs = sample_of(tile, hs);
      float pp[3];
      if (!ein) {
        const f32x4 ra = rv[2 * NI], rb2 = rv[2 * NI + 1];   // {o0, o1, o2, d0}, {d1, d2, z, -}
        const float zz = rb2[2];
        pp[0] = ra[0] + ra[3] * zz;   // sample_point
        pp[1] = ra[1] + rb2[0] * zz;
        pp[2] = ra[2] + rb2[1] * zz;
      }
      auto put1 = [&](int f, float v) {
        s16x4 q0, q1, q2 = {};
        const f32x4 v4 = f32x4{valid ? (H2 ? v * csc[f] : v) : 0.0f, 0.0f, 0.0f, 0.0f};
        if constexpr (H2) split2_x4(v4, q0, q1);
        else split3_x4(v4, q0, q1, q2);
        const int o = wb3_xoff<PITCH>(er, f & ~3) + 2 * (f & 3);
        *reinterpret_cast<short*>(xb + o) = q0[0];
        *reinterpret_cast<short*>(xb + XPART + o) = q1[0];
        if (!H2) *reinterpret_cast<short*>(xb + 2 * XPART + o) = q2[0];
      };
      if (ej < 30) {
        const int k = ej / 3, m = ej - 3 * k;
        float sn, cs;
        if (ein) {
          sn = ein[gs * 63 + 3 + 6 * k + m];
          cs = ein[gs * 63 + 6 + 6 * k + m];
        } else {
          const float pm = m == 0 ? pp[0] : m == 1 ? pp[1] : pp[2];
          sincosf(__int_as_float((127 + k) << 23) * pm, &sn, &cs);   // encode_half's (float)(1 << k) * p[m]
        }
        put1(3 + 6 * k + m, sn);
        put1(6 + 6 * k + m, cs);
      } else if (ej == 30) {
#pragma unroll
        for (int c = 0; c < 3; ++c) put1(c, ein ? ein[gs * 63 + c] : pp[c]);
        put1(63, 0.0f);
      }
      return;
    }
    *reinterpret_cast<s16x4*>(xb + off) = p0;
    *reinterpret_cast<s16x4*>(xb + XPART + off) = p1;
    if (!H2) *reinterpret_cast<s16x4*>(xb + 2 * XPART + off) = p2;
  };
  f32x16 acc[RB][NBLK], acc2[DUAL ? RB : 1][DUAL ? NBLK : 1];
#pragma unroll
  for (int rb = 0; rb < RB; ++rb)
#pragma unroll
    for (int nb = 0; nb < NBLK; ++nb) acc[rb][nb] = f32x16{};
  if constexpr (DUAL)
#pragma unroll
    for (int rb = 0; rb < RB; ++rb)
#pragma unroll
      for (int nb = 0; nb < NBLK; ++nb) acc2[rb][nb] = f32x16{};
  float dbacc[RB] = {};
  // A read: feature m = 32 (RB wv + rb) + li -> g = 4 (RB wv + rb) + (li >> 3), half (li >> 2) & 1, q = li & 3;
  // row 8 h + j (the swizzle c = 2 (g & 3) + half does not depend on rb)
  const int ag = 4 * RB * wv + (li >> 3), ahh = (li >> 2) & 1, aq = li & 3, ac = 2 * (ag & 3) + ahh;
  const int abase = ag * 128 + ahh * 64 + aq;
  // B transposed reads: 16-lane group (h, column half ch); lane 4 q + pp supplies row 8 h + 4 r + q, features
  // 32 nb + 16 ch + 4 pp, and receives column (lane & 15) of the 4 rows
  const int trq = (lane >> 2) & 3, trp = lane & 3, trch = (lane >> 4) & 1;
  const int trow0 = 8 * h + trq;   // + 4 r
  const int troff0 = wb3_xoff<PITCH>(trow0, 16 * trch + 4 * trp);
  const int troff1 = wb3_xoff<PITCH>(trow0 + 4, 16 * trch + 4 * trp);
  // half tiles of this workgroup: u = 0, 1, ... -> tile blockIdx + (u >> 1) gridDim, half u & 1
  const int tl0 = __builtin_amdgcn_readfirstlane((int)blockIdx.x);
  const int nh = tl0 < nt ? 2 * ((nt - 1 - tl0) / gstride + 1) : 0;
  auto tile_of = [&](int u) { return tl0 + (u >> 1) * gstride; };
  auto bufp = [&](int b) { return reinterpret_cast<const char*>(wb3) + (size_t)b * Cfg::BUF; };
  auto readA = [&](float (&av)[RB][8], int b, int src = 0) {
    const float* gbuf = reinterpret_cast<const float*>(bufp(b) + src * GB1);
#pragma unroll
    for (int rb = 0; rb < RB; ++rb)
#pragma unroll
      for (int j = 0; j < 8; ++j) av[rb][j] = gbuf[abase + 512 * rb + ((8 * h + j) ^ ac) * 4];
  };
  auto splitA = [&](float (&av)[RB][8], P8 (&a)[RB][NPART], bool count, float sc) {
#pragma unroll
    for (int rb = 0; rb < RB; ++rb) {
#pragma unroll
      for (int j = 0; j < 8; ++j) dbacc[rb] += count ? av[rb][j] : 0.0f;
      if constexpr (H2) {
        float sv[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) sv[j] = av[rb][j] * sc;
        split2_f16(sv, a[rb][0], a[rb][1]);
      } else {
        split3_bf16(av[rb], a[rb][0], a[rb][1], a[rb][2]);
      }
    }
  };
  auto readB = [&](P8 (&bv)[NPART], int b, int nb) {
    const char* xb = bufp(b) + GB;
#pragma unroll
    for (int p = 0; p < NPART; ++p) {
      const char* pb = xb + p * XPART + 64 * nb;
      const s16x4 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
          (__attribute__((address_space(3))) s16x4*)(__attribute__((address_space(3))) void*)(pb + troff0));
      const s16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
          (__attribute__((address_space(3))) s16x4*)(__attribute__((address_space(3))) void*)(pb + troff1));
      bv[p] = __builtin_bit_cast(P8, __builtin_shufflevector(v0, v1, 0, 1, 2, 3, 4, 5, 6, 7));
    }
  };
  // Pipeline: half tile u computes from buffer u % 3 while half tile u + 2 is staged into buffer (u + 2) % 3 from
  // registers loaded during u - 1 (pieces at column blocks S_P0 + k S_PD), the loads of u + 3 go out after the last
  // piece, and u + 1's A operand and first B block are read (already staged and fenced) before the barrier.
  // DEEP (the two-layer encoding form): two register sets, the loads of half tile u + 4 issued at u (two half tiles
  // of latency instead of one; nh is even): 131.3 -> 128.1 us per launch (profiles/r04_variants_enc_wgrad_deep.txt)
  constexpr bool DEEP = DUAL;
  f32x4 rv[NR], rv1[DEEP ? NR : 1];
#pragma unroll
  for (int u = 0; u < 2; ++u)
    if (u < nh) {
      load_half(rv, tile_of(u), u & 1);
#pragma unroll
      for (int k = 0; k < NP; ++k) stage_piece(u, rv, tile_of(u), u & 1, k);
    }
  if (2 < nh) load_half(rv, tile_of(2), 0);
  if constexpr (DEEP)
    if (3 < nh) load_half(rv1, tile_of(3), 1);
  __syncthreads();
  constexpr int S_PD = NBLK / NP < WB3_SPACE ? NBLK / NP : WB3_SPACE;
  constexpr int S_P0 = WB3_STAGE + (NP - 1) * S_PD < NBLK ? WB3_STAGE : 0;
  constexpr int S_APF = WB3_AREAD < NBLK ? WB3_AREAD : NBLK - 1;
  constexpr int S_ASP = S_APF + 2 < NBLK ? S_APF + 2 : NBLK - 1;
  P8 Acur[RB][NPART], Anext[RB][NPART], B[2][NPART];
  P8 Acur2[DUAL ? RB : 1][NPART], Anext2[DUAL ? RB : 1][NPART];
  if (nh > 0) {
    float av[RB][8];
    readA(av, 0);
    splitA(av, Acur, true, gsc);
    if constexpr (DUAL) {
      readA(av, 0, 1);
      splitA(av, Acur2, false, gsc2);
    }
    readB(B[0], 0, 0);
  }
  int bcur = 0;
  // the loop body is branch-free (a branch would split the scheduling regions the MFMA chains are interleaved in):
  // past the end, the reads of half tile u + 1 and the staging of u + 2 touch buffers nobody reads afterwards, and
  // the loads of u + 3 (DEEP: u + 4) re-read the last half tile
  auto body = [&](int u, f32x4 (&rvs)[NR]) __attribute__((always_inline)) {
    const int bn1 = bcur == 2 ? 0 : bcur + 1, bn2 = bcur == 0 ? 2 : bcur - 1;
    const int u2 = u + 2 < nh ? u + 2 : nh - 1, u3 = u + (DEEP ? 4 : 3) < nh ? u + (DEEP ? 4 : 3) : nh - 1;
    float av[RB][8], av2[RB][8];
#pragma unroll
    for (int nb = 0; nb < NBLK; ++nb) {
      if (nb + 1 < NBLK) readB(B[(nb + 1) & 1], bcur, nb + 1);
      else readB(B[0], bn1, 0);
      if (nb == S_APF) {
        readA(av, bn1);
        if constexpr (DUAL) readA(av2, bn1, 1);
      }
      if (nb == S_ASP) {
        splitA(av, Anext, u + 1 < nh, gsc);
        if constexpr (DUAL) splitA(av2, Anext2, false, gsc2);
      }
      const P8* bo = B[nb & 1];
      if constexpr (DUAL)
#pragma unroll
        for (int rb = 0; rb < RB; ++rb) {
          const P8* a = Acur2[rb];
          f32x16 c = acc2[rb][nb];
          c = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[1], bo[0], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[0], bo[1], c, 0, 0, 0);
          if (NTP == 4) c = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[1], bo[1], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[0], bo[0], c, 0, 0, 0);
          acc2[rb][nb] = c;
        }
#pragma unroll
      for (int rb = 0; rb < RB; ++rb) {
        const P8* a = Acur[rb];
        f32x16 c = acc[rb][nb];
        if constexpr (H2) {
          c = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[1], bo[0], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[0], bo[1], c, 0, 0, 0);
          if (NTP == 4) c = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[1], bo[1], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[0], bo[0], c, 0, 0, 0);
        } else {
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], bo[1], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2], bo[0], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], bo[2], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], bo[0], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], bo[1], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], bo[0], c, 0, 0, 0);
        }
        acc[rb][nb] = c;
      }
#pragma unroll
      for (int k = 0; k < NP; ++k)
        if (nb == S_P0 + k * S_PD) stage_piece(bn2, rvs, tile_of(u2), u2 & 1, k);
      if (nb == S_P0 + (NP - 1) * S_PD) load_half(rvs, tile_of(u3), u3 & 1);
      __builtin_amdgcn_sched_barrier(0);
    }
    __syncthreads();
#pragma unroll
    for (int rb = 0; rb < RB; ++rb)
#pragma unroll
      for (int p = 0; p < NPART; ++p) {
        Acur[rb][p] = Anext[rb][p];
        if constexpr (DUAL) Acur2[rb][p] = Anext2[rb][p];
      }
    bcur = bn1;
  };
  if constexpr (DEEP) {
    for (int u = 0; u < nh; u += 2) {   // (half tiles u and u + 1: the register sets by parity)
      body(u, rv);
      body(u + 1, rv1);
    }
  } else {
    for (int u = 0; u < nh; ++u) body(u, rv);
  }
  static_assert(!DUAL || (H2 && LAY == 1), "the two-layer encoding form: f16x2, both partial sets in layer 0's layout");
  static_assert(MODE != 2 && (LAY == MODE || LAY == 2 || DUAL), "partial layouts");
  constexpr int C = WgradCfg<LAY>::C, COL = (LAY == 2 && MODE == 0) ? 64 : 0;
  constexpr bool DB = MODE == 0 || LAY == 1;
  float* pb = part + (size_t)blockIdx.x * WgradCfg<LAY>::PART;
#pragma unroll
  for (int rb = 0; rb < RB; ++rb) {
#pragma unroll
    for (int rr = 0; rr < 16; ++rr) {
      const int m = 32 * (RB * wv + rb) + (rr & 3) + 8 * (rr >> 2) + 4 * h;
#pragma unroll
      for (int nb = 0; nb < NBLK; ++nb)
        pb[(size_t)m * C + COL + 32 * nb + li] = H2 ? (acc[rb][nb][rr] * gun) * cun[32 * nb + li] : acc[rb][nb][rr];
    }
    float d = dbacc[rb] + __shfl_xor(dbacc[rb], 32, 64);
    if (DB && h == 0) pb[(size_t)256 * C + 32 * (RB * wv + rb) + li] = d;
  }
  if constexpr (DUAL) {   // the skip layer's encoding columns (no db: its dL/dh_4 sum comes with its h columns)
    float* pb2 = part2 + (size_t)blockIdx.x * WgradCfg<LAY>::PART;
#pragma unroll
    for (int rb = 0; rb < RB; ++rb)
#pragma unroll
      for (int rr = 0; rr < 16; ++rr) {
        const int m = 32 * (RB * wv + rb) + (rr & 3) + 8 * (rr >> 2) + 4 * h;
#pragma unroll
        for (int nb = 0; nb < NBLK; ++nb)
          pb2[(size_t)m * C + 32 * nb + li] = (acc2[rb][nb][rr] * gun2) * cun[32 * nb + li];
      }
  }
}

// ---- k_bwd_fused: one layer's backward over a chunk of stored tiles in ONE pass -- the data gradient with the
// BatchNorm backward below it AND the weight gradient (5 -> 3 KiB of HBM per sample and layer).
// What used to force two passes is the chunk-wide statistics of BatchNorm L-1's backward, Sigma_s dL/dy and
// Sigma_s dL/dy (h - mean), which the weight-gradient GEMM's result gave; here they come before the backward from
// the fused forward's fold state (fold_bn_backward: exact float64 functions of the chunk's encoding and gradient
// moments -- the premise, identity activations, the forward's statistics already rest on), so each tile's
//   dy = W_L^T g_L  (data gradient)   ->   g_{L-1} = ((dy - mean dy) - (h - mean) kk) invstd gamma
// is final in the tile's epilogue, and G_L += g_L (x) (h_{L-1} - mean) (weight gradient) uses the same operands.
//
// Work split: the 256 input features i of layer L in two halves; a PAIR of workgroups (blocks b and b + 8: the same
// XCD, so the second read of a g tile is an L2 hit) takes the same tiles, each computing its half of dy and of G's
// columns -- W^T for 16 features per wave stays in 64 registers and G's 32 x 128 slice per wave in 64, which two
// waves per SIMD can hold.  8 waves; per 32-sample tile and wave: 48 v_mfma_f32_16x16x32_f16 of data gradient (its
// 16 features x 2 sample blocks, 8 k-steps of 32 neurons, 3 products) + 48 of weight gradient (2 x 8 blocks of
// 16 x 16 over the tile's 32 samples, 3 products).  Operands in LDS per tile (double-buffered, one barrier a tile):
// g_L scaled by its chunk-wide 2^sg (the producer's gmax) and h - mean per column by 2^sx (Samuelson), each split
// into fp16 hi + mid, stored [sample][feature] with 16-byte chunks swizzled by row (fb_off): conflict-free for the
// data gradient's 16-byte reads (8 neurons of a sample) and the weight gradient's transposed ds_read_b64_tr_b16
// reads (8 samples of a feature).  g_{L-1} is written in place over h_{L-1} (each workgroup reads exactly the
// columns it writes); the weight-gradient partial per pair in k_wgrad<LAY>'s layout (summed at the end of the next
// layer's launch, fb_reduce_row; layer 1's by k_fb_reduce_tail).
constexpr int FB_GP = 512, FB_XP = 256;                   // g / x part row bytes (256 / 128 halves)
constexpr int FB_GPART = 32 * FB_GP, FB_XPART = 32 * FB_XP;
constexpr int FB_BUF = 2 * FB_GPART + 2 * FB_XPART;       // 48 KiB per tile
constexpr int FB_PAIRS = 128;
constexpr size_t FB_LDS = 3 * (size_t)FB_BUF + 7 * 128 * sizeof(float);   // split + 2 raw tiles + constants
constexpr size_t FB_LDS_OUT = FB_LDS + (4 * 256 + 8 * 64) * sizeof(float);  // + occ_out / BatchNorm 7 constants,
                                                                            //   dL/dlogit slots

// The rematerialised backward (k_bwd_remat, the default since round 5) moves g between layers PRE-SPLIT, scaled by
// 2^gexp[L], in the byte layout its consumer's LDS holds it, so it is DMA'd with no conversion: per 32-sample tile
// [part 2][octet o 32][cell][8 fp16] (32 KiB), cell = sample ^ (12 (o & 1)) holding features 8 o .. 8 o + 7 of that
// sample (gs_off).  That one layout makes the data gradient's 16-byte B-operand reads (16 samples of one octet per
// lane group), the weight gradient's transposed reads (4 samples x 16 features per 16 lanes) and the producer's
// 8-byte stores (16 samples x 2 halves: 256 contiguous bytes per octet) conflict-free / contiguous.  The chunk's
// encoding image (FB_ENC bytes per tile, k_remat_enc) is DMA'd the same way: row r's 16-byte chunk ch sits at
// ch ^ ((r >> 1) & 7) (conflict-free 16-byte B-operand reads, lanes = 16 samples x 4 chunks).
constexpr int FB_ENC = 8192;
constexpr int GS_TILE = 2 * FB_GPART;
__device__ __forceinline__ int fb_eoff(int r, int ch) { return r * 128 + 16 * (ch ^ ((r >> 1) & 7)); }
__device__ __forceinline__ int gs_off(int s, int o) { return (o * 32 + (s ^ (12 * (o & 1)))) * 16; }

// 16-byte chunk c of row r sits at c ^ f(r), f(r) = 2 (r & 3 | b << 2) | p with p = bit 2 of r and b = bit 2 ^ bit 3:
// sixteen distinct values over a row block of 16 (the split writes: 32 lanes = 16 rows x two 8-byte halves of one
// chunk), distinct f >> 1 over rows {0..3, 8..11} and over {4..7, 12..15} (the transposed reads: 8 rows x 2 chunks),
// and {f(A)} u {f(B) ^ 1} distinct for A = {0..3, 12..15}, B = {4..11} (the 16-byte reads' lane groups of 16, two
// k-groups each) -- every pattern conflict-free (scripts/micro/lds_fb.hip)
__device__ __forceinline__ int fb_swz(int r) {
  return 2 * ((r & 3) | ((((r >> 2) ^ (r >> 3)) & 1) << 2)) | ((r >> 2) & 1);
}
template <int P>
__device__ __forceinline__ int fb_off(int r, int c) {   // 16-bit element c of row r
  return r * P + 16 * ((c >> 3) ^ fb_swz(r)) + 2 * (c & 7);
}
// ds_read_b64_tr_b16 of four 16-bit elements at p (LDS) + OFF.  Inline asm: hipcc waits vmcnt(0) before every
// ds_read_tr16 builtin while an LDS-DMA is in flight (it cannot tell the DMA's destination from the read's), which
// would drain k_bwd_fused's two-tiles-ahead prefetch.  The compiler does not count these reads: the caller waits
// lgkmcnt before using the result (fb_lgkm).
typedef int fb_i32x2 __attribute__((ext_vector_type(2)));
template <int OFF>
__device__ __forceinline__ s16x4 fb_tr(unsigned addr) {
  fb_i32x2 r;
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(r) : "v"(addr), "i"(OFF));
  return __builtin_bit_cast(s16x4, r);
}
// s_waitcnt lgkmcnt(N), then the values that wait made ready pass through an (ordered) empty asm: the compiler
// cannot read their registers before the wait
template <int N, size_t K>
__device__ __forceinline__ void fb_lgkm(std::array<s16x4, 4> (&ready)[K]) {
  asm volatile("s_waitcnt lgkmcnt(%0)" ::"i"(N));
#pragma unroll
  for (size_t k = 0; k < K; ++k)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      fb_i32x2 v = __builtin_bit_cast(fb_i32x2, ready[k][i]);
      asm volatile("" : "+v"(v));
      ready[k][i] = __builtin_bit_cast(s16x4, v);
    }
}
__device__ __forceinline__ unsigned fb_lds_addr(const void* p) {
  return (unsigned)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
}

// W_L^T image for k_bwd_fused: layer L (1..7) at (L-1) HW_H, [ks 8][input block 16][part 2][lane 64] f16x8: row
// i = 16 iblk + (lane & 15) (input feature of layer L, the skip layer's h columns), k = neuron 32 ks + 8 (lane >> 4)
// + e; scaled by 2^sw[L] like the forward
__global__ void k_pack_dgrad_h16(NofParamsDev P, const int* __restrict__ sw, f16x8* __restrict__ out) {
  const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= 7 * HW_H) return;
  const int L = 1 + (int)(idx / HW_H);
  const size_t j = idx % HW_H;
  const int lane = (int)(j & 63), part = (int)((j >> 6) & 1), ib = (int)((j >> 7) & 15), ks = (int)(j >> 11);
  const int i = 16 * ib + (lane & 15), in_f = in_features(L), col = (L == 4 ? 63 : 0) + i;
  const float sc = ldexpf(1.0f, sw[L]);
  f16x8 v;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int k = 32 * ks + 8 * (lane >> 4) + e;
    const float w = P.lin_w[L][(size_t)k * in_f + col] * sc;
    const _Float16 hi = (_Float16)w;
    v[e] = part == 0 ? hi : (_Float16)(w - (float)hi);
  }
  out[idx] = v;
}

// max |dL/dlogit| over the chunk (float bits, into a zeroed word): k_fb_prep's bound on |g_7|
// (one atomic per workgroup: 4 per workgroup onto the one word cost ~10 us per chunk in L2 serialisation)
__global__ __launch_bounds__(256) void k_out_gabs(const float* __restrict__ g, int64_t n, unsigned* __restrict__ out) {
  __shared__ float wm[4];
  float m = 0.0f;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    m = fmaxf(m, fabsf(g[i]));
  m = wave_max_f(m);
  if ((threadIdx.x & 63) == 0) wm[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) atomicMax(out, __float_as_uint(fmaxf(fmaxf(wm[0], wm[1]), fmaxf(wm[2], wm[3]))));
}

// Everything a stored chunk's one-pass backward needs before its first layer, in ONE launch of 8 blocks x 256
// threads (block L, thread k = neuron k of layer L): BatchNorm L's forward coefficients from the chunk's stored
// statistics (k_bn_save's arithmetic), then
//   L < 7: BatchNorm L's backward constants from the fold (mean(dL/dy) = 0 exactly: dL/dy = W_{L+1}^T g_{L+1} and
//          g_{L+1} is a BatchNorm backward's output, zero-mean over the chunk; kk = Sigma dL/dy (h - mean) invstd^2 / n
//          with Sigma dL/dy (h - mean) = dgamma / fl64(1/sqrt(var+eps)) from the fold; dgamma_L += that sum x invstd),
//   L = 7: occ_out + BatchNorm 7 (k_out_bwd_grad's prologue on the fold's occ_out statistics acc = (Sigma dL/dlogit
//          (h_7 - mean_7), Sigma dL/dlogit)): k_bwd_fused<0, true>'s per-column constants, the output layer's and
//          BatchNorm 7's parameter gradients, and the bound |g_7[f]| <= ((|gvmax w_out| + |gm|) + sqrt(n) sigma |kk|)
//          invstd |gamma| (|h_7 - mean_7| <= sqrt(n) sigma, Samuelson) as layer 7's operand-scale maximum;
// and layer L's |dL/dh| maximum slots zeroed for this chunk (block 7 after reading gvmax also re-zeroes it for the
// next chunk's k_out_gabs).
struct FbPrepOut {
  int64_t g[8];                        // gacc offsets of dgamma per layer
  double *d_beta7, *d_wout, *d_bout;   // occ_out / BatchNorm 7 parameter gradients
};
__global__ __launch_bounds__(256) void k_fb_prep(NofParamsDev P, const double* __restrict__ stats, int64_t n,
                                                 float eps, float* __restrict__ coef, FoldBnBwd F, int64_t c,
                                                 float* __restrict__ bnb, double* __restrict__ gacc, FbPrepOut o,
                                                 const double* __restrict__ oacc, unsigned* __restrict__ gvmax,
                                                 float* __restrict__ ocst, unsigned* __restrict__ gmax) {
  __shared__ float wmax[4];
  const int L = blockIdx.x, k = threadIdx.x;
  double m, var;
  if (stats) {
    const double s1 = stats[512 * L + 2 * k], s2 = stats[512 * L + 2 * k + 1];
    m = s1 / (double)n;
    var = s2 / (double)n - m * m;
  } else {   // no store (rematerialised backward): the fold's exact statistics, as the forward's coefficients
    m = F.pp[(((int64_t)L * F.C + c) * 256 + k) * 64 + 63];
    var = F.sr[((int64_t)L * F.C + c) * 1024 + 768 + k];
  }
  if (var < 0.0) var = 0.0;
  const float invstd = (float)(1.0 / sqrt(var + (double)eps));
  float* cf = coef + 1024 * L;
  cf[k] = (float)((double)P.lin_b[L][k] + m);
  cf[256 + k] = invstd;
  cf[512 + k] = invstd * P.bn_w[L][k];
  cf[768 + k] = P.bn_b[L][k];
  if (k < GMAX_SLOTS) gmax[L * GMAX_SLOTS + k] = 0u;
  if (L < 7) {
    const double rinv = F.sr[((int64_t)L * F.C + c) * 1024 + 256 + k];
    const double dotp = F.dg[((int64_t)L * F.C + c) * 256 + k] / rinv;
    bnb[512 * L + k] = 0.0f;
    bnb[512 * L + 256 + k] = (((float)dotp * invstd) * invstd) / (float)n;
    gacc[o.g[L] + k] += dotp * (double)invstd;
    return;
  }
  const double A = oacc[k], G0 = oacc[256];
  const float wo = P.out_w[k], ga = P.bn_w[7][k], mu = cf[k], al = cf[512 + k], be = cf[768 + k];
  const double S1 = (double)wo * G0, dotp = (double)wo * A;
  const float gm = (float)(S1 / (double)n), kk = (((float)dotp * invstd) * invstd) / (float)n;
  const float sg = invstd * ga;
  ocst[k] = wo * sg;
  ocst[256 + k] = gm * sg;
  ocst[512 + k] = mu;
  ocst[768 + k] = kk * sg;
  gacc[o.g[7] + k] += dotp * (double)invstd;
  o.d_beta7[k] += S1;
  o.d_wout[k] += (double)al * A + (double)be * G0;
  if (k == 0) o.d_bout[0] += G0;
  const float gvm = __uint_as_float(*gvmax);
  float bd = ((fabsf(gvm * wo) + fabsf(gm)) + sqrtf((float)n) / invstd * fabsf(kk)) * invstd * fabsf(ga) * 1.001f;
  bd = wave_max_f(bd);
  if ((k & 63) == 0) wmax[k >> 6] = bd;
  __syncthreads();   // (also: every thread has read gvmax)
  if (k == 0) {
    gmax[7 * GMAX_SLOTS] = __float_as_uint(fmaxf(fmaxf(wmax[0], wmax[1]), fmaxf(wmax[2], wmax[3])));
    *gvmax = 0u;
  }
}

// The rematerialised backward's operand images (k_bwd_fused<., ., true>).  Column scale 2^s_k of the encoding
// image: the sin / cos features (and their chunk means) lie in [-1, 1], so |e - ebar| <= 2 -> 2^13; the xyz features
// |e - ebar| <= 2 max |position| (k_pos_bound) -> 2^(13 - ilogb max|position|); every scaled value below 2^15.
__device__ __forceinline__ int remat_sx(int k, float pmax) {
  if (k >= 3) return 13;
  int e = (pmax > 0.0f && pmax < 3.0e38f) ? 13 - ilogbf(pmax) : 13;
  return e < -60 ? -60 : e > 60 ? 60 : e;
}

// grid (8 layers, C chunks), 256 threads (row i of P'_L for chunk c): the row scaled by 2^(t_i - s_k), t_i putting
// its largest entry in [2^14, 2^15), split into fp16 hi / mid in k_bwd_fused's A-operand order, and 2^-t_i
__global__ __launch_bounds__(256) void k_remat_pimg(FoldBnBwd F, const unsigned* __restrict__ pbound,
                                                    f16x8* __restrict__ img, float* __restrict__ scl) {
  const int L = blockIdx.x, i = threadIdx.x;
  const int64_t c = blockIdx.y, li = ((int64_t)L * F.C + c) * 256 + i;
  const int sxyz = remat_sx(0, __uint_as_float(*pbound));
  const double* row = F.pp + li * 64;
  double mx = 0.0;
  for (int k = 0; k < 63; ++k) mx = fmax(mx, fabs(ldexp(row[k], -(k < 3 ? sxyz : 13))));
  int t = (mx > 0.0 && mx < 1.0e300) ? 14 - ilogb(mx) : 0;
  t = t < -100 ? -100 : t > 100 ? 100 : t;
  scl[li] = ldexpf(1.0f, -t);
  f16x8* o = img + li * 16;
#pragma unroll
  for (int ks = 0; ks < 2; ++ks)
#pragma unroll
    for (int kg = 0; kg < 4; ++kg) {
      f16x8 h, m;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int k = 32 * ks + 8 * kg + e;
        const float a = k < 63 ? (float)ldexp(row[k], t - (k < 3 ? sxyz : 13)) : 0.0f;
        h[e] = (_Float16)a;
        m[e] = (_Float16)(a - (float)h[e]);
      }
      o[(2 * ks) * 4 + kg] = h;
      o[(2 * ks + 1) * 4 + kg] = m;
    }
}

// One chunk's encoding image: per sample d = fl32(e - ebar) (encode_full, the forward's features; ebar float64),
// times 2^s_k, split into fp16 hi / mid at [tile][part][row = sample & 31][chunk ch ^ ((row >> 1) & 7)][8]; samples
// past the chunk (the last tile's tail) are zero.  One thread per sample; a workgroup's four tiles are assembled in
// LDS and written as whole 16-byte lanes (1 KiB per wave store).  Block 0 also zeroes k_g7's |g_7| slots (gm7) for
// this chunk (the previous chunk's layer 7 has read them: stream order).
constexpr int RE_TILES = 4;
__global__ __launch_bounds__(32 * RE_TILES) void k_remat_enc(const float* __restrict__ rays, int stride,
                                                           const float* __restrict__ z, int S, int64_t c0, int64_t n,
                                                           const double* __restrict__ eb,
                                                           const unsigned* __restrict__ pbound,
                                                           char* __restrict__ out, unsigned* __restrict__ gm7) {
  __shared__ __attribute__((aligned(16))) char img[RE_TILES * FB_ENC];
  __shared__ double ebs[64];
  const int t = threadIdx.x;
  if (t < 64) ebs[t] = t < 63 ? eb[t] : 0.0;
  if (blockIdx.x == 0 && t < GMAX_SLOTS) gm7[t] = 0u;
  __syncthreads();
  const int64_t i = (int64_t)blockIdx.x * (32 * RE_TILES) + t;
  const int64_t nrow = (n + 31) / 32 * 32;
  float f[64];
  if (i < n) {
    float p[3];
    sample_point(rays + ray_of(c0 + i, S) * stride, z[c0 + i], p);
    encode_full(p, f);
  }
  const int sxyz = remat_sx(0, __uint_as_float(*pbound));
  char* tb = img + (t >> 5) * FB_ENC;
  const int r = t & 31;
#pragma unroll
  for (int ch = 0; ch < 8; ++ch) {
    f16x8 h, m;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int k = 8 * ch + e;
      const float d = (i < n && k < 63) ? (float)((double)f[k] - ebs[k]) : 0.0f;
      const float a = ldexpf(d, k < 3 ? sxyz : 13);
      h[e] = (_Float16)a;
      m[e] = (_Float16)(a - (float)h[e]);
    }
    *reinterpret_cast<f16x8*>(tb + fb_eoff(r, ch)) = h;
    *reinterpret_cast<f16x8*>(tb + FB_ENC / 2 + fb_eoff(r, ch)) = m;
  }
  __syncthreads();
  const int64_t b0 = (int64_t)blockIdx.x * RE_TILES * FB_ENC;
  const int64_t bend = nrow / 32 * FB_ENC;
#pragma unroll
  for (int j = 0; j < RE_TILES * FB_ENC / 16 / (32 * RE_TILES); ++j) {
    const int o = 16 * (t + 32 * RE_TILES * j);
    if (b0 + o < bend) *reinterpret_cast<f32x4*>(out + b0 + o) = *reinterpret_cast<const f32x4*>(img + o);
  }
}

// grid 7 (layers 1..7), 256 threads: sum_j |W_L[j][i]| over the 256 outputs j, for the 256 input columns i that
// k_bwd_remat's data gradient takes (the skip layer's h columns) -- its bound on |W_L^T g_L|
__global__ __launch_bounds__(256) void k_wcol(NofParamsDev P, float* __restrict__ wcol) {
  const int L = 1 + blockIdx.x, i = threadIdx.x, in_f = in_features(L), col = (L == 4 ? 63 : 0) + i;
  float s = 0.0f;
  for (int j = 0; j < 256; ++j) s += fabsf(P.lin_w[L][(size_t)j * in_f + col]);
  wcol[(L - 1) * 256 + i] = s;
}

template <int AUX = 0>
__device__ __forceinline__ void fb_glds16(const void* g, void* l) {   // 16 B per lane -> l + 16 lane (LDS-DMA)
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                   (__attribute__((address_space(3))) void*)l, 16, 0, AUX);
}

__device__ __forceinline__ constexpr int fb_vmcnt(int n) {   // s_waitcnt vmcnt(n) alone (gfx9 encoding)
  return (n & 15) | ((n >> 4) << 14) | 0x0F70;
}

// The previous layer's weight-gradient partials, summed at the end of a k_bwd_fused launch (k_wgrad_reduce's sum,
// one row per workgroup of the 256) instead of by a launch of its own: mode 0 none, 1 the 256-column layout
// (WgradCfg<0>), 2 the skip layer's (WgradCfg<2>: hidden columns at 64, dW rows of 319)
struct FbRed {
  const float* part;
  const float* coef;   // that layer's coefp (alpha at 512, beta'' at 768)
  double* dW;
  double* db;
  int mode;
};

// Row m = blockIdx.x of dW += alpha G + beta'' (x) db over FB_PAIRS partials; red: 640 doubles of LDS
__device__ __forceinline__ void fb_reduce_row(const FbRed& R, double* red, int t) {
  const int m = (int)blockIdx.x;
  const int C = R.mode == 2 ? WgradCfg<2>::C : WgradCfg<0>::C, colh = R.mode == 2 ? 64 : 0;
  const size_t PART = (size_t)256 * C + 256;
  const int c = t & 255, hv = t >> 8;
  const float* pc = R.part + (size_t)m * C + colh + c;
  double Gp[8] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
  {   // all 64 of the thread's loads in flight (32 at a time: +0.3 % step)
    float v[FB_PAIRS / 2];
#pragma unroll
    for (int j = 0; j < FB_PAIRS / 2; ++j) v[j] = pc[(size_t)(FB_PAIRS / 2 * hv + j) * PART];
#pragma unroll
    for (int j = 0; j < FB_PAIRS / 2; ++j) Gp[j & 7] += (double)v[j];
  }
  red[t] = ((Gp[0] + Gp[1]) + (Gp[2] + Gp[3])) + ((Gp[4] + Gp[5]) + (Gp[6] + Gp[7]));
  if (t < FB_PAIRS) {
    double d = (double)R.part[(size_t)t * PART + (size_t)256 * C + m];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) d += __shfl_xor(d, o, 64);
    if ((t & 63) == 0) red[512 + (t >> 6)] = d;
  }
  __syncthreads();
  if (t < 256) {
    const double dbm = red[512] + red[513];
    const double G = red[t] + red[t + 256];
    const int in_f = R.mode == 2 ? 319 : 256, wcol = R.mode == 2 ? 63 : 0;
    R.dW[(size_t)m * in_f + wcol + c] += (double)R.coef[512 + c] * G + (double)R.coef[768 + c] * dbm;
    if (t == 0) R.db[m] += dbm;
  }
  __syncthreads();
}
static_assert(FB_PAIRS == 128 && 2 * FB_PAIRS == 256, "fb_reduce_row: one row per workgroup, two 64-pair halves");

// OUT (layer 7 only): g_7 = dL/dh_7 is not read from HBM but made in LDS from h_7 (gin, DMA'd as the raw tile) and
// the chunk's dL/dlogit (ograd): g_7 = (dL/dlogit A - B) - (h_7 - mean_7) K with k_fb_prep's per-column A = w_out s,
// B = gm s, K = kk s, s = invstd gamma_7 (k_out_bwd_grad's terms, the same cancellation order), and the operand scale
// comes from k_fb_prep's bound on |g_7| instead of a recorded maximum: 1 KiB per sample less written and read than
// producing g_7 first.
template <int LAY, bool OUT>
__global__ __launch_bounds__(512, 1) void k_bwd_fused(const float* __restrict__ gin, float* hio,
                                                       const f16x8* __restrict__ wt, const int* __restrict__ sw,
                                                       int layer, int64_t n, const float* __restrict__ coefp,
                                                       const float* __restrict__ bnb,
                                                       const float* __restrict__ gamma,
                                                       const unsigned* __restrict__ gmax_in,
                                                       unsigned* __restrict__ gmax_out, float* __restrict__ part,
                                                       const float* __restrict__ ograd,
                                                       const float* __restrict__ ocst, FbRed red) {
  constexpr int C = WgradCfg<LAY>::C, COL = LAY == 2 ? 64 : 0;
  extern __shared__ __attribute__((aligned(16))) char fb[];
  // LDS: split operands of tiles k & 1 (two buffers), the raw tile (one buffer), constants
  float* const cst = reinterpret_cast<float*>(fb + 3 * FB_BUF);     // [csc | cun | gm | kk | invstd | gamma | mu][128]
  float* const ocs = cst + 7 * 128;   // OUT: [A | B | mean | K][256], then per wave 64 dL/dlogit
  const int t = threadIdx.x, lane = t & 63, kg = lane >> 4, lm = lane & 15;
  const int wv = __builtin_amdgcn_readfirstlane(t >> 6);
  const int bid = (int)blockIdx.x, hf = (bid >> 3) & 1, pr = ((bid >> 4) << 3) | (bid & 7);
  const int npair = (int)gridDim.x >> 1;
  const int nt = (int)((n + 31) / 32);
  const int nk = pr < nt ? (nt - 1 - pr) / npair + 1 : 0;   // this pair's tiles: pr + k npair, k < nk
  if (t < 128) {
    const int c = 128 * hf + t;
    const float invstd = coefp[256 + c];
    const float bnd = sqrtf((float)n) / invstd;   // Samuelson: |h - mean| <= sqrt(n) sigma
    int e = (bnd > 0.0f && bnd < 3.0e38f) ? 14 - ilogbf(bnd) : 0;
    e = e < -60 ? -60 : e > 60 ? 60 : e;
    cst[t] = ldexpf(1.0f, e);
    cst[128 + t] = ldexpf(1.0f, -e);
    cst[256 + t] = bnb[c];
    cst[384 + t] = bnb[256 + c];
    cst[512 + t] = invstd;
    cst[640 + t] = gamma[c];
    cst[768 + t] = coefp[c];
  }
  if constexpr (OUT)
    for (int i = t; i < 4 * 256; i += 512) ocs[i] = ocst[i];
  unsigned gmx = 0;
  for (int i = 0; i < GMAX_SLOTS; ++i) gmx = max(gmx, gmax_in[i]);   // (uniform loads)
  const int eg = tile_scale_exp(__uint_as_float(gmx));
  const float gsc = ldexpf(1.0f, eg), gun = ldexpf(1.0f, -eg);
  const float dun = ldexpf(1.0f, -sw[layer]) * gun;   // data-gradient accumulator -> dL/dy
  // this wave's W^T rows: input features 128 hf + 16 wv + (lane & 15), all 8 k-steps, hi / mid
  f16x8 wr[8][2];
  {
    const f16x8* __restrict__ w8 = wt + lane;
#pragma unroll
    for (int ks = 0; ks < 8; ++ks)
#pragma unroll
      for (int p = 0; p < 2; ++p) wr[ks][p] = w8[((ks * 16 + 8 * hf + wv) * 2 + p) * 64];
  }
  // Raw tiles by LDS-DMA, two ahead: raw buffer k & 1 holds the pair's tile k as it lies in HBM -- 32 rows (feature
  // groups) of 1 KiB of g_L, then the 16 rows of this half's h_{L-1}.  Wave w moves g rows 4 w + m and x rows
  // 2 w + m and later splits exactly those rows, so a wave waits only for its own DMA.  Split map of wave w's
  // instruction m: lane l takes sample 16 sb + (l & 15) (sb = m & 1), half (l >> 4) & 1 of row 4 w + 2 (m >> 1) +
  // (l >> 5) (g) or 2 w + (l >> 5) (x, sb = m): the raw reads and the split writes conflict-free
  // OUT: the tile's 32 dL/dlogit, DMA'd with the raw rows into this wave's own 256-byte slot (lane l: sample l & 31)
  float* const gvs = ocs + 4 * 256 + 64 * wv;
  auto issue_raw = [&](int k) {
    const int tl = pr + k * npair;
    char* rb = fb + 2 * (size_t)FB_BUF;
    int ln = lane;
    asm volatile("" : "+v"(ln));   // lane addresses recomputed per tile: held across the loop they would spill
    if constexpr (OUT) {
      const int64_t s0 = (int64_t)tl * 32 + (ln & 31);
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(ograd + (s0 < n ? s0 : n - 1)),
                                       (__attribute__((address_space(3))) void*)gvs, 4, 0, 0);
    }
    const float* gsrc = gin + (size_t)tl * TILE_FLOATS + ln * 4;
    const float* xsrc = hio + (size_t)tl * TILE_FLOATS + 16 * hf * 256 + ln * 4;
#pragma unroll
    for (int m = 0; m < 4; ++m) fb_glds16(gsrc + (4 * wv + m) * 256, rb + (4 * wv + m) * 1024);
#pragma unroll
    for (int m = 0; m < 2; ++m)
      fb_glds16<2>(xsrc + (2 * wv + m) * 256, rb + 32 * 1024 + (2 * wv + m) * 1024);   // (nt: read once)
  };
  const int sl = lane & 15, sh = (lane >> 4) & 1, sr = lane >> 5;
  auto convert = [&](int k) {   // raw tile k -> split buffer k & 1 (this wave's rows)
    const int tl = pr + k * npair;
    const char* rb = fb + 2 * (size_t)FB_BUF;
    char* const sp = fb + (size_t)(k & 1) * FB_BUF;
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const int row = 4 * wv + 2 * (m >> 1) + sr, sm = 16 * (m & 1) + sl;
      const bool valid = (int64_t)tl * 32 + sm < n;
      const f32x4 r = *reinterpret_cast<const f32x4*>(rb + (row * 64 + sm + 32 * sh) * 16);
      f32x4 v;
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] = valid ? r[q] * gsc : 0.0f;
      s16x4 p0, p1;
      split2_x4(v, p0, p1);
      const int o = fb_off<FB_GP>(sm, 8 * row + 4 * sh);
      *reinterpret_cast<s16x4*>(sp + o) = p0;
      *reinterpret_cast<s16x4*>(sp + FB_GPART + o) = p1;
    }
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      const int row = 2 * wv + sr, sm = 16 * m + sl, cl = 8 * row + 4 * sh;   // column within the half
      const bool valid = (int64_t)tl * 32 + sm < n;
      const f32x4 r = *reinterpret_cast<const f32x4*>(rb + 32 * 1024 + (row * 64 + sm + 32 * sh) * 16);
      const f32x4 mu = *reinterpret_cast<const f32x4*>(cst + 768 + cl);
      const f32x4 sc = *reinterpret_cast<const f32x4*>(cst + cl);
      f32x4 v;
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] = valid ? (r[q] - mu[q]) * sc[q] : 0.0f;
      s16x4 p0, p1;
      split2_x4(v, p0, p1);
      const int o = fb_off<FB_XP>(sm, cl);
      *reinterpret_cast<s16x4*>(sp + 2 * FB_GPART + o) = p0;
      *reinterpret_cast<s16x4*>(sp + 2 * FB_GPART + FB_XPART + o) = p1;
    }
  };
  // OUT: this wave's raw rows of tile k (h_7, as DMA'd) -> g_7 in place, before convert splits them; run where
  // the data-gradient accumulators are not live yet (the top of the tile before k)
  auto out_rows = [&]() {
    char* rb = fb + 2 * (size_t)FB_BUF;
    int ln = lane;
    asm volatile("" : "+v"(ln));   // addresses recomputed here, not held in registers across the tile loop
    const float gv = gvs[ln & 31];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int row = 4 * wv + j, f = 8 * row + 4 * (ln >> 5);
      f32x4* rp = reinterpret_cast<f32x4*>(rb + (row * 64 + ln) * 16);
      const f32x4 r = *rp;
      const f32x4 ca = *reinterpret_cast<const f32x4*>(ocs + f), cb = *reinterpret_cast<const f32x4*>(ocs + 256 + f);
      const f32x4 mu = *reinterpret_cast<const f32x4*>(ocs + 512 + f), ck = *reinterpret_cast<const f32x4*>(ocs + 768 + f);
      f32x4 o;
#pragma unroll
      for (int q = 0; q < 4; ++q) o[q] = (gv * ca[q] - cb[q]) - (r[q] - mu[q]) * ck[q];
      *rp = o;
    }
  };
  f32x4 aw[2][8];
#pragma unroll
  for (int jb = 0; jb < 2; ++jb)
#pragma unroll
    for (int ib = 0; ib < 8; ++ib) aw[jb][ib] = f32x4{};
  float dbacc[2] = {0.0f, 0.0f};
  float gmo = 0.0f;
  const int trq = lm >> 2, trp = lm & 3;   // transposed reads: lane lm = 4 q + pp of 16-lane group kg
  __syncthreads();   // cst
  // Pipeline, one barrier per tile: tile k computes from split buffer k & 1 while each wave splits ITS rows of tile
  // k + 1 (raw, DMA'd during tile k - 1) into buffer (k + 1) & 1 between the data- and weight-gradient MFMAs, then
  // DMAs its rows of tile k + 2 into the raw buffer it has just read
  if (nk > 0) {
    issue_raw(0);
    __builtin_amdgcn_s_waitcnt(fb_vmcnt(0));
    if constexpr (OUT) out_rows();
    convert(0);
    if (nk > 1) issue_raw(1);
  }
  __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0)
  __builtin_amdgcn_s_barrier();
  // one tile: data gradient, split of tile k + 1, weight gradient, epilogue (the second wave of each SIMD running
  // the phases in another order -- weight gradient first, or split first -- measured +2 %,
  // profiles/r04_variants_bwd_*.txt)
  auto tile = [&](int k) {
    const int tl = pr + k * npair;
    const char* const sp = fb + (size_t)(k & 1) * FB_BUF;
    const char* gb = sp;
    const char* xb = sp + 2 * FB_GPART;
    // data gradient: this wave's 16 input features x 32 samples
    f32x4 ad[2] = {f32x4{}, f32x4{}};
    auto dgrad = [&]() {
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
#pragma unroll
      for (int sb = 0; sb < 2; ++sb) {
        const int o = fb_off<FB_GP>(16 * sb + lm, 32 * ks + 8 * kg);
        const f16x8 bh = *reinterpret_cast<const f16x8*>(gb + o);
        const f16x8 bm = *reinterpret_cast<const f16x8*>(gb + FB_GPART + o);
        ad[sb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wr[ks][0], bh, ad[sb], 0, 0, 0);
        ad[sb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wr[ks][0], bm, ad[sb], 0, 0, 0);
        ad[sb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wr[ks][1], bh, ad[sb], 0, 0, 0);
      }
    }
    };
    auto split_next = [&]() {
    if (k + 1 < nk) {   // this wave's rows of tile k + 1 (its DMA, then the stores of tile k - 1: vmcnt(2))
      if (k > 0) __builtin_amdgcn_s_waitcnt(fb_vmcnt(2));
      else __builtin_amdgcn_s_waitcnt(fb_vmcnt(0));
      if constexpr (OUT) out_rows();   // (OUT: g_7 rows of tile k + 1 from its h_7 rows, in place)
      convert(k + 1);
      __builtin_amdgcn_s_waitcnt(0xC07F);   // its raw reads done before the raw buffer is refilled
      if (k + 2 < nk) issue_raw(k + 2);
    }
    };
    auto wgrad = [&]() {
    // weight gradient: rows j = 32 wv + 16 jb + lm, the tile's 32 samples, 8 column blocks of this half.  Operands
    // by transposed reads (rows +4: the same swizzle, so an immediate offset; the mid part FB_*PART further), the
    // next column block's read while the current one multiplies
    auto read8 = [&](unsigned a0, unsigned a1, auto part) {   // rows 8 kg + q (a0) and + 4 (a1), hi and mid
      constexpr int Q = decltype(part)::value;
      const s16x4 h0 = fb_tr<0>(a0), h1 = fb_tr<0>(a1), m0 = fb_tr<Q>(a0), m1 = fb_tr<Q>(a1);
      return std::array<s16x4, 4>{h0, h1, m0, m1};
    };
    auto join = [](const s16x4& a, const s16x4& b) {
      return __builtin_bit_cast(f16x8, __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7));
    };
    using QG = std::integral_constant<int, FB_GPART>;
    using QX = std::integral_constant<int, FB_XPART>;
    const unsigned ga = fb_lds_addr(gb), xa = fb_lds_addr(xb);
    const int tr0 = 8 * kg + trq, tr1 = tr0 + 4;
    auto xrd = [&](int ib) {
      const int col = 16 * ib + 4 * trp;
      return read8(xa + fb_off<FB_XP>(tr0, col), xa + fb_off<FB_XP>(tr1, col), QX{});
    };
    std::array<s16x4, 4> ra[2], rbx[2];
#pragma unroll
    for (int jb = 0; jb < 2; ++jb) {
      const int col = 32 * wv + 16 * jb + 4 * trp;
      ra[jb] = read8(ga + fb_off<FB_GP>(tr0, col), ga + fb_off<FB_GP>(tr1, col), QG{});
    }
    rbx[0] = xrd(0);
    fb_lgkm<4>(ra);   // A landed (the first column block's four reads may still fly)
    f16x8 A[2][2];
#pragma unroll
    for (int jb = 0; jb < 2; ++jb) {
      A[jb][0] = join(ra[jb][0], ra[jb][1]);
      A[jb][1] = join(ra[jb][2], ra[jb][3]);
    }
    if (hf == 0) {
#pragma unroll
      for (int jb = 0; jb < 2; ++jb)
#pragma unroll
        for (int e = 0; e < 8; ++e) dbacc[jb] += (float)A[jb][0][e] + (float)A[jb][1][e];
    }
#pragma unroll
    for (int ib = 0; ib < 8; ++ib) {
      std::array<s16x4, 4> cur[1] = {rbx[ib & 1]};
      if (ib + 1 < 8) {
        rbx[(ib + 1) & 1] = xrd(ib + 1);
        fb_lgkm<4>(cur);
      } else {
        fb_lgkm<0>(cur);
      }
      rbx[ib & 1] = cur[0];
      const f16x8 B0 = join(rbx[ib & 1][0], rbx[ib & 1][1]), B1 = join(rbx[ib & 1][2], rbx[ib & 1][3]);
#pragma unroll
      for (int jb = 0; jb < 2; ++jb) {
        aw[jb][ib] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A[jb][0], B0, aw[jb][ib], 0, 0, 0);
        aw[jb][ib] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A[jb][0], B1, aw[jb][ib], 0, 0, 0);
        aw[jb][ib] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A[jb][1], B0, aw[jb][ib], 0, 0, 0);
      }
    }
    };
    auto epilogue = [&]() {
    // epilogue: dL/dy -> BatchNorm L-1 backward -> g_{L-1} over this tile's h_{L-1} (input features
    // 128 hf + 16 wv + 4 kg .. + 3 of sample 16 sb + lm): two 16-byte stores per lane
    {
      const int il = 16 * wv + 4 * kg;   // column within the half
      const f32x4 cun = *reinterpret_cast<const f32x4*>(cst + 128 + il);
      const f32x4 cgm = *reinterpret_cast<const f32x4*>(cst + 256 + il);
      const f32x4 ckk = *reinterpret_cast<const f32x4*>(cst + 384 + il);
      const f32x4 cis = *reinterpret_cast<const f32x4*>(cst + 512 + il);
      const f32x4 cga = *reinterpret_cast<const f32x4*>(cst + 640 + il);
      const int i = 128 * hf + il;
#pragma unroll
      for (int sb = 0; sb < 2; ++sb) {
        const int sm = 16 * sb + lm;
        const bool valid = (int64_t)tl * 32 + sm < n;
        const int o = fb_off<FB_XP>(sm, il);
        const f16x4 xh = *reinterpret_cast<const f16x4*>(xb + o);
        const f16x4 xm = *reinterpret_cast<const f16x4*>(xb + FB_XPART + o);
        f32x4 v;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float d = ad[sb][q] * dun;
          const float xc = ((float)xh[q] + (float)xm[q]) * cun[q];   // h - mean (hi + mid: 22 bits)
          v[q] = valid ? ((d - cgm[q]) - xc * ckk[q]) * cis[q] * cga[q] : 0.0f;
          gmo = fmaxf(gmo, fabsf(v[q]));
        }
        f32x4* dst = reinterpret_cast<f32x4*>(hio + (size_t)tl * TILE_FLOATS) + (i >> 3) * 64 + sm + 32 * ((i >> 2) & 1);
        __builtin_nontemporal_store(v, dst);   // streamed past L2, which keeps the g tiles for the pair
      }
    }
    };
    // the MFMA phases at raised wave priority, so a SIMD's other wave (in its split / epilogue) does not delay their
    // issue: -1.0 % per launch (the split and epilogue raised instead: +0.3 %; profiles/r04_variants_bwd_prio.txt)
    __builtin_amdgcn_s_setprio(1);
    dgrad();
    __builtin_amdgcn_s_setprio(0);
    split_next();
    __builtin_amdgcn_s_setprio(1);
    wgrad();
    __builtin_amdgcn_s_setprio(0);
    epilogue();
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_s_barrier();   // every wave done with split buffer k & 1 and has filled (k + 1) & 1
    };
  for (int k = 0; k < nk; ++k) tile(k);
  gmo = wave_max_f(gmo);
  if (lane == 0) atomicMax(gmax_out + ((bid * 8 + wv) & (GMAX_SLOTS - 1)), __float_as_uint(gmo));
  // G partial of pair pr: rows j = 32 wv + 16 jb + 4 kg + r, columns 128 hf + 16 ib + lm (x scale undone per column)
  float* pb = part + (size_t)pr * WgradCfg<LAY>::PART;
#pragma unroll
  for (int ib = 0; ib < 8; ++ib) {
    const float cu = cst[128 + 16 * ib + lm] * gun;
#pragma unroll
    for (int jb = 0; jb < 2; ++jb)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        pb[(size_t)(32 * wv + 16 * jb + 4 * kg + r) * C + COL + 128 * hf + 16 * ib + lm] = aw[jb][ib][r] * cu;
  }
  if (hf == 0) {
#pragma unroll
    for (int jb = 0; jb < 2; ++jb) {
      float d = dbacc[jb];
      d += __shfl_xor(d, 16, 64);
      d += __shfl_xor(d, 32, 64);
      if (kg == 0) pb[(size_t)256 * C + 32 * wv + 16 * jb + lm] = d * gun;
    }
  }
  // the previous layer's partials (split buffer 0 as scratch; after the loop, where the registers are free and
  // other workgroups' loops still run: -0.3 % step against the prologue, profiles/r04_variants_bwd_reductions.txt)
  __syncthreads();
  if (red.mode != 0) fb_reduce_row(red, reinterpret_cast<double*>(fb), t);
}

// ---- The rematerialised backward (the default training backward since round 5; no activation store).
//
// Every layer input is made per tile from the chunk's encoding instead of read from a store:
//   h_{L-1} - mean_{L-1} = P'_{L-1} (e - ebar),   P'_L = W_L P_{L-1}   (the fold state's float64 layer maps)
// -- the identity-activation premise (models.py:72) the BatchNorm statistics already rest on -- so the forward
// writes nothing for the backward and every chunk takes this path whatever its size.  Operands: the encoding image
// (k_remat_enc: d = e - ebar scaled by 2^s_k, fp16 hi / mid, 256 B per sample) and P' rows scaled by 2^(t_i - s_k)
// and split (k_remat_pimg); the product d -> x is 3 fp16 products per fp32 product like every other.
//
// k_g7: g_7 = dL/dh_7 per tile, (dL/dlogit A - B) - (h_7 - mean_7) K (k_out_bwd_grad's terms and order; A, B, K
// from k_fb_prep), h_7 - mean_7 = P'_7 d on the matrix pipe (wave w: features 32 w .. + 31, 24 MFMAs a tile, P'_7's
// rows in registers, the encoding by LDS-DMA into two slots), written pre-split at 2^gexp[7] (k_fb_prep's bound on
// |g_7|), its largest |g_7| recorded (gm7) for layer 7's bound on g_6.
__global__ __launch_bounds__(512, 1) void k_g7(const char* __restrict__ enc, const float* __restrict__ ograd,
                                               int64_t n, const f16x8* __restrict__ p7, const float* __restrict__ p7s,
                                               const float* __restrict__ ocst, const unsigned* __restrict__ gbound,
                                               int* __restrict__ gexp, unsigned* __restrict__ gm7,
                                               char* __restrict__ gout) {
  extern __shared__ __attribute__((aligned(16))) char g7l[];
  float* const ocs = reinterpret_cast<float*>(g7l + 2 * FB_ENC);   // [A | B | 2^-t | K][256]
  const int t = threadIdx.x, lane = t & 63, kg = lane >> 4, lm = lane & 15;
  const int wv = __builtin_amdgcn_readfirstlane(t >> 6);
  const int nt = (int)((n + 31) / 32), grid = (int)gridDim.x, bid = (int)blockIdx.x;
  const int nk = bid < nt ? (nt - 1 - bid) / grid + 1 : 0;
  for (int i = t; i < 1024; i += 512) ocs[i] = (i >= 512 && i < 768) ? p7s[i - 512] : ocst[i];
  const int eg = tile_scale_exp(__uint_as_float(*gbound));
  const float gsc = ldexpf(1.0f, eg);
  if (bid == 0 && t == 0) gexp[7] = eg;
  f16x8 pa[2][2][2];   // [rb][ks][part]: rows 32 wv + 16 rb + lm
#pragma unroll
  for (int rb = 0; rb < 2; ++rb)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int p = 0; p < 2; ++p) pa[rb][ks][p] = p7[((size_t)(32 * wv + 16 * rb + lm) * 4 + 2 * ks + p) * 4 + kg];
  auto dma = [&](int k) {
    int ln = lane;
    asm volatile("" : "+v"(ln));
    fb_glds16(enc + (size_t)(bid + k * grid) * FB_ENC + wv * 1024 + ln * 16, g7l + (k & 1) * FB_ENC + wv * 1024);
  };
  if (nk > 0) dma(0);
  __builtin_amdgcn_s_waitcnt(fb_vmcnt(0));
  __syncthreads();
  float gmo = 0.0f;
  for (int k = 0; k < nk; ++k) {
    const int tl = bid + k * grid;
    float gv[2];
#pragma unroll
    for (int sb = 0; sb < 2; ++sb) {
      const int64_t s = (int64_t)tl * 32 + 16 * sb + lm;
      gv[sb] = ograd[s < n ? s : n - 1];
    }
    if (k + 1 < nk) dma(k + 1);   // slot (k + 1) & 1: tile k - 1's, read before the last barrier
    const char* eb = g7l + (k & 1) * FB_ENC;
    f32x4 ah[2][2] = {{f32x4{}, f32x4{}}, {f32x4{}, f32x4{}}};
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int sb = 0; sb < 2; ++sb) {
        const int o = fb_eoff(16 * sb + lm, 4 * ks + kg);
        const f16x8 bh = *reinterpret_cast<const f16x8*>(eb + o);
        const f16x8 bm = *reinterpret_cast<const f16x8*>(eb + FB_ENC / 2 + o);
#pragma unroll
        for (int rb = 0; rb < 2; ++rb) {
          ah[rb][sb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(pa[rb][ks][0], bh, ah[rb][sb], 0, 0, 0);
          ah[rb][sb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(pa[rb][ks][0], bm, ah[rb][sb], 0, 0, 0);
          ah[rb][sb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(pa[rb][ks][1], bh, ah[rb][sb], 0, 0, 0);
        }
      }
    char* gt = gout + (size_t)tl * GS_TILE;
#pragma unroll
    for (int sb = 0; sb < 2; ++sb) {
      const int sm = 16 * sb + lm;
      const bool valid = (int64_t)tl * 32 + sm < n;
#pragma unroll
      for (int rb = 0; rb < 2; ++rb) {
        const int f = 32 * wv + 16 * rb + 4 * kg;
        const f32x4 ca = *reinterpret_cast<const f32x4*>(ocs + f), cb = *reinterpret_cast<const f32x4*>(ocs + 256 + f);
        const f32x4 ts = *reinterpret_cast<const f32x4*>(ocs + 512 + f), ck = *reinterpret_cast<const f32x4*>(ocs + 768 + f);
        f32x4 v;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float g7 = (gv[sb] * ca[q] - cb[q]) - (ah[rb][sb][q] * ts[q]) * ck[q];
          v[q] = valid ? g7 : 0.0f;
          gmo = fmaxf(gmo, fabsf(v[q]));
          v[q] *= gsc;
        }
        s16x4 p0, p1;
        split2_x4(v, p0, p1);
        // one 16-byte cell per lane, as k_bwd_remat2's epilogue: kg even / odd (features f .. f+3, f+4 .. f+7 of
        // one octet) swap halves, the even row storing the octet's hi part and the odd row its mid part
        const fb_i32x2 hv = __builtin_bit_cast(fb_i32x2, p0), mv = __builtin_bit_cast(fb_i32x2, p1);
        const auto s0 = __builtin_amdgcn_permlane16_swap(hv[0], mv[0], false, false);
        const auto s1 = __builtin_amdgcn_permlane16_swap(hv[1], mv[1], false, false);
        typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
        const u32x4 cell = {s0[0], s1[0], s0[1], s1[1]};
        __builtin_nontemporal_store(cell, reinterpret_cast<u32x4*>(gt + (kg & 1) * FB_GPART + gs_off(sm, f >> 3)));
      }
    }
    __builtin_amdgcn_s_waitcnt(fb_vmcnt(4));   // this wave's DMA of tile k + 1 (the 4 stores may still fly)
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_s_barrier();
  }
  gmo = wave_max_f(gmo);
  if (lane == 0) atomicMax(gm7 + ((bid * 8 + wv) & (GMAX_SLOTS - 1)), __float_as_uint(gmo));
}
constexpr size_t G7_LDS = 2 * FB_ENC + 1024 * sizeof(float);
// k_g7's grid: two workgroups per CU (96 VGPRs, 20 KiB of LDS each) -- -6 % against one (256), 1024 no better
// (profiles/r05_g7_ab.txt)
constexpr int G7_BLOCKS = 512;

// The rematerialised layer launch (k_bwd_remat2 below): one layer's backward over a chunk in one pass, as k_bwd_fused
// (a pair of workgroups per tile, halves of the input features, 8 waves; W_L^T rows in registers; one barrier a
// tile), with
//   * g_L arriving PRE-SPLIT by LDS-DMA straight into the tile's split buffer (no raw buffer, no conversion: its
//     producer wrote it at 2^gexp[L]), one tile ahead;
//   * the layer input x = h_{L-1} - mean made on the matrix pipe from the encoding image (two LDS slots, one tile
//     deeper) and the half's P'_{L-1} rows (LDS, staged once: 12 MFMAs per wave and tile), split into the x half of
//     the next tile's buffer between the data- and weight-gradient MFMAs;
//   * g_{L-1} = ((dy - gm) - x kk) invstd gamma written pre-split at 2^gexp[L-1] from a bound fixed in the prologue:
//     |g_{L-1,i}| <= (sum_j |W_L[j][i]| max|g_L| + |gm_i| + sqrt(n) sigma_i |kk_i|) invstd_i |gamma_i|.
// HBM per sample: 1 KiB of g_L, 256 B of encoding in, 1 KiB of g_{L-1} out (2.25 KiB; the store path moved 3).
constexpr size_t RB_PX = 128 * 256;   // the half's P' rows (128 x 16 f16x8), slot q of row r at q ^ (r & 15)
constexpr size_t RB_LDS = 2 * (size_t)FB_BUF + 2 * FB_ENC + RB_PX + 8 * 128 * sizeof(float);
static_assert(RB_LDS <= 160 * 1024, "k_bwd_remat2 LDS");
// k_bwd_remat2<LAY>: that work split by ROLE between the two waves of each SIMD (waves w and w + 4 share a SIMD): waves 0-3 ("D") the data gradient of 32 input features
// each (W_L^T rows in registers: 2 row blocks, so every 16-byte g read feeds 6 MFMAs instead of 3) and the BatchNorm
// backward epilogue with the g_{L-1} stores; waves 4-7 ("W") the rematerialisation of 32 x columns each and the
// weight gradient of 64 neuron rows each (G's 64 x 128 slice in 128 registers).  Per tile a D wave runs MFMAs then
// VALU (dgrad, epilogue), a W wave VALU-heavy then MFMAs (remat, wgrad), so each SIMD's two waves are in
// complementary phases between the tile's barriers; the g / encoding DMAs stay spread over all eight waves.
template <int LAY>
__global__ __launch_bounds__(512, 1) void k_bwd_remat2(const char* __restrict__ gin, char* __restrict__ gout,
                                                        const f16x8* __restrict__ wt,
                                                        const int* __restrict__ sw, int layer, int64_t n,
                                                        const float* __restrict__ coefp, const float* __restrict__ bnb,
                                                        const float* __restrict__ gamma, int* __restrict__ gexp,
                                                        const float* __restrict__ wcol,
                                                        const unsigned* __restrict__ gmax_in,
                                                        unsigned* __restrict__ gmax_out, float* __restrict__ part,
                                                        FbRed red, const char* __restrict__ enc,
                                                        const f16x8* __restrict__ px, const float* __restrict__ pxs) {
  constexpr int C = WgradCfg<LAY>::C, COL = LAY == 2 ? 64 : 0;
  constexpr int NST = 4;   // a D wave's global stores per tile
  extern __shared__ __attribute__((aligned(16))) char fb[];
  char* const enb = fb + 2 * FB_BUF;
  char* const pxl = enb + 2 * FB_ENC;
  float* const cst = reinterpret_cast<float*>(pxl + RB_PX);   // [csc | cun | gm | kk | invstd | gamma | xs | bound]
  const int t = threadIdx.x, lane = t & 63, kg = lane >> 4, lm = lane & 15;
  const int wv = __builtin_amdgcn_readfirstlane(t >> 6);
  const int rw = wv & 3;   // index within the role
  const int bid = (int)blockIdx.x, hf = (bid >> 3) & 1, pr = ((bid >> 4) << 3) | (bid & 7);
  const int npair = (int)gridDim.x >> 1;
  const int nt = (int)((n + 31) / 32);
  const int nk = pr < nt ? (nt - 1 - pr) / npair + 1 : 0;
  const float rn = sqrtf((float)n);
  if (t < 128) {
    const int c = 128 * hf + t;
    const float invstd = coefp[256 + c];
    const float bnd = rn / invstd;   // Samuelson: |h - mean| <= sqrt(n) sigma
    int e = (bnd > 0.0f && bnd < 3.0e38f) ? 14 - ilogbf(bnd) : 0;
    e = e < -60 ? -60 : e > 60 ? 60 : e;
    cst[t] = ldexpf(1.0f, e);
    cst[128 + t] = ldexpf(1.0f, -e);
    cst[256 + t] = bnb[c];
    cst[384 + t] = bnb[256 + c];
    cst[512 + t] = invstd;
    cst[640 + t] = gamma[c];
    cst[768 + t] = ldexpf(pxs[c], e);
  }
  unsigned gmx = 0;
  for (int i = 0; i < GMAX_SLOTS; ++i) gmx = max(gmx, gmax_in[i]);
  {
    const int c = t & 255;
    const float invstd = coefp[256 + c];
    float ob = ((wcol[c] * __uint_as_float(gmx) + fabsf(bnb[c])) + rn / invstd * fabsf(bnb[256 + c])) * invstd *
               fabsf(gamma[c]) * 1.01f;
    ob = wave_max_f(ob);
    if (lane == 0) cst[896 + wv] = ob;
  }
  for (int j = t; j < 128 * 16; j += 512) {
    const int r = j >> 4, q = j & 15;
    *reinterpret_cast<f16x8*>(pxl + r * 256 + 16 * (q ^ (r & 15))) = px[(size_t)(128 * hf + r) * 16 + q];
  }
  const int eg = gexp[layer];
  const float gun = ldexpf(1.0f, -eg);
  __syncthreads();
  float obm = cst[896];
#pragma unroll
  for (int i = 1; i < 8; ++i) obm = fmaxf(obm, cst[896 + i]);
  const int eo = tile_scale_exp(obm);
  const float gso = ldexpf(1.0f, eo);
  if (bid == 0 && t == 0) gexp[layer - 1] = eo;
  // the epilogue's per-feature constants folded (read by the D waves after the barrier below):
  //   2^eo g_{L-1} = (dy A - B) - (xh + xm) C,  A = dun invstd gamma 2^eo,  B = gm invstd gamma 2^eo,
  //   C = 2^-e kk invstd gamma 2^eo   (slots 640 / 256 / 384; cun at 128 stays for the W waves)
  const float dun = ldexpf(1.0f, -sw[layer]) * gun;
  if (t < 128) {
    const float sc = cst[512 + t] * cst[640 + t] * gso;
    const float cb = cst[256 + t] * sc, cc = cst[128 + t] * cst[384 + t] * sc;
    cst[640 + t] = dun * sc;
    cst[256 + t] = cb;
    cst[384 + t] = cc;
  }
  auto dma_g = [&](int k) {
    const int tl = pr + k * npair;
    char* const sb = fb + (size_t)(k & 1) * FB_BUF;
    int ln = lane;
    asm volatile("" : "+v"(ln));
#pragma unroll
    for (int m = 0; m < 4; ++m)
      fb_glds16(gin + (size_t)tl * GS_TILE + (4 * wv + m) * 1024 + 16 * ln, sb + (4 * wv + m) * 1024);
  };
  auto dma_enc = [&](int k) {
    const int tl = pr + k * npair;
    int ln = lane;
    asm volatile("" : "+v"(ln));
    fb_glds16(enc + (size_t)tl * FB_ENC + wv * 1024 + ln * 16, enb + (k & 1) * FB_ENC + wv * 1024);
  };
  // W waves: x of tile k, columns 32 rw .. 32 rw + 31 of the half (2 row blocks of P'), slot k & 1 -> buffer k & 1
  auto remat_x = [&](int k) {
    const char* eb = enb + (k & 1) * FB_ENC;
    char* const xb = fb + (size_t)(k & 1) * FB_BUF + 2 * FB_GPART;
    f32x4 ax[2][2] = {{f32x4{}, f32x4{}}, {f32x4{}, f32x4{}}};
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      f16x8 pa[2][2];
#pragma unroll
      for (int rb = 0; rb < 2; ++rb)
#pragma unroll
        for (int p = 0; p < 2; ++p) {
          const int r = 32 * rw + 16 * rb + lm, q = (2 * ks + p) * 4 + kg;
          pa[rb][p] = *reinterpret_cast<const f16x8*>(pxl + r * 256 + 16 * (q ^ (r & 15)));
        }
#pragma unroll
      for (int sb = 0; sb < 2; ++sb) {
        const int o = fb_eoff(16 * sb + lm, 4 * ks + kg);
        const f16x8 bh = *reinterpret_cast<const f16x8*>(eb + o);
        const f16x8 bm = *reinterpret_cast<const f16x8*>(eb + FB_ENC / 2 + o);
#pragma unroll
        for (int rb = 0; rb < 2; ++rb) {
          ax[rb][sb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(pa[rb][0], bh, ax[rb][sb], 0, 0, 0);
          ax[rb][sb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(pa[rb][0], bm, ax[rb][sb], 0, 0, 0);
          ax[rb][sb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(pa[rb][1], bh, ax[rb][sb], 0, 0, 0);
        }
      }
    }
#pragma unroll
    for (int rb = 0; rb < 2; ++rb) {
      const int il = 32 * rw + 16 * rb + 4 * kg;
      const f32x4 xs = *reinterpret_cast<const f32x4*>(cst + 768 + il);
#pragma unroll
      for (int sb = 0; sb < 2; ++sb) {
        f32x4 v;
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = ax[rb][sb][q] * xs[q];
        s16x4 p0, p1;
        split2_x4(v, p0, p1);
        const int o = fb_off<FB_XP>(16 * sb + lm, il);
        *reinterpret_cast<s16x4*>(xb + o) = p0;
        *reinterpret_cast<s16x4*>(xb + FB_XPART + o) = p1;
      }
    }
  };
  if (nk > 0) {
    dma_g(0);
    dma_enc(0);
    if (nk > 1) dma_enc(1);
    __builtin_amdgcn_s_waitcnt(fb_vmcnt(0));
    __builtin_amdgcn_s_barrier();
    if (wv >= 4) remat_x(0);
  }
  __builtin_amdgcn_s_waitcnt(0xC07F);
  __builtin_amdgcn_s_barrier();
  if (wv < 4) {
    // ---- D: data gradient of input features 128 hf + 32 rw + 16 rb + lm, epilogue, g_{L-1} stores
    const float gui = ldexpf(1.0f, -eo);
    f16x8 wr[8][2][2];
    {
      const f16x8* __restrict__ w8 = wt + lane;
#pragma unroll
      for (int ks = 0; ks < 8; ++ks)
#pragma unroll
        for (int rb = 0; rb < 2; ++rb)
#pragma unroll
          for (int p = 0; p < 2; ++p) wr[ks][rb][p] = w8[((ks * 16 + 8 * hf + 2 * rw + rb) * 2 + p) * 64];
    }
    // the W^T rows used once before the loop: otherwise the waitcnt pass sees their loads pending at the loop header
    // and waits vmcnt(0) at every tile's first MFMA -- i.e. for the DMAs the tile has just issued
#pragma unroll
    for (int ks = 0; ks < 8; ++ks)
      asm volatile("" ::"v"(wr[ks][0][0]), "v"(wr[ks][0][1]), "v"(wr[ks][1][0]), "v"(wr[ks][1][1]));
    float gmo = 0.0f;
    typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
    u32x4 pcell[2][2] = {{u32x4{}, u32x4{}}, {u32x4{}, u32x4{}}};
    // a cell's g_{L-1} store (tile tq): the split pair as one 16-byte cell
    auto store_cell = [&](int rb, int sb, int tq, const u32x4& cell) {
      const int i = 128 * hf + 32 * rw + 16 * rb + 4 * kg, sm = 16 * sb + lm;
      char* gt = gout + (size_t)tq * GS_TILE + (kg & 1) * FB_GPART + gs_off(sm, i >> 3);
#if PCN_RB_NOSTORE
      if (cell[0] == 12345u && cell[3] == 4321u)
#endif
      __builtin_nontemporal_store(cell, reinterpret_cast<u32x4*>(gt));   // streaming: keep L2 for the g / encoding tiles the other half re-reads
    };
    // tile k's g_{L-1} cells are stored during tile k + 1's data-gradient MFMAs, one cell after every second k-step
    // (pinned there by scheduling barriers: left to the scheduler they sink to the phase's end), so the D waves'
    // stores do not meet every CU's at the epilogue: -1.6 % per launch (profiles/r05_variants_remat2_defer.txt)
    // (tile 0: zero cells to tile 0's own slots, rewritten by this wave's later stores of its real cells -- same
    // addresses, program order; they also keep NST stores behind every tile's DMAs for the vmcnt(NST) below)
    [[maybe_unused]] unsigned long long ck0 = 0, ck1 = 0, ck2 = 0, ck3 = 0, cA = 0, cB = 0, cW = 0, cL0 = 0, cL1 = 0;
    RB_T(cL0);
    for (int k = 0; k < nk; ++k) {
      const int tl = pr + k * npair;
      const int ptl = k > 0 ? tl - npair : tl;
      RB_T(ck0);
#if !PCN_RB_NODMA
      if (k + 1 < nk) dma_g(k + 1);
      if (k + 2 < nk) dma_enc(k + 2);
#endif
      const char* const sp = fb + (size_t)(k & 1) * FB_BUF;
      const char* xb = sp + 2 * FB_GPART;
      f32x4 ad[2][2] = {{f32x4{}, f32x4{}}, {f32x4{}, f32x4{}}};
#pragma unroll
      for (int ks = 0; ks < 8; ++ks)
#pragma unroll
        for (int sb = 0; sb < 2; ++sb) {
          const int o = gs_off(16 * sb + lm, 4 * ks + kg);
          const f16x8 bh = *reinterpret_cast<const f16x8*>(sp + o);
          const f16x8 bm = *reinterpret_cast<const f16x8*>(sp + FB_GPART + o);
#pragma unroll
          for (int rb = 0; rb < 2; ++rb) {
#if PCN_RB_NODG
            ad[rb][sb] += __builtin_bit_cast(f32x4, bh) + __builtin_bit_cast(f32x4, bm);
#else
            ad[rb][sb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wr[ks][rb][0], bh, ad[rb][sb], 0, 0, 0);
            ad[rb][sb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wr[ks][rb][0], bm, ad[rb][sb], 0, 0, 0);
            ad[rb][sb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wr[ks][rb][1], bh, ad[rb][sb], 0, 0, 0);
#endif
          }
          if ((ks & 1) && sb == 1) {
            store_cell((ks >> 2) & 1, (ks >> 1) & 1, ptl, pcell[(ks >> 2) & 1][(ks >> 1) & 1]);
            __builtin_amdgcn_sched_barrier(0);
          }
        }
      RB_T(ck1);
#pragma unroll
      for (int rb = 0; rb < 2; ++rb) {
        const int il = 32 * rw + 16 * rb + 4 * kg;
        const f32x4 cA = *reinterpret_cast<const f32x4*>(cst + 640 + il);
        const f32x4 cB = *reinterpret_cast<const f32x4*>(cst + 256 + il);
        const f32x4 cC = *reinterpret_cast<const f32x4*>(cst + 384 + il);
#pragma unroll
        for (int sb = 0; sb < 2; ++sb) {
          const int sm = 16 * sb + lm;
          const bool valid = (int64_t)tl * 32 + sm < n;
          const int o = fb_off<FB_XP>(sm, il);
          const f16x4 xh = *reinterpret_cast<const f16x4*>(xb + o);
          const f16x4 xm = *reinterpret_cast<const f16x4*>(xb + FB_XPART + o);
          f32x4 vs;   // 2^eo g_{L-1}
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const float xs = (float)xh[q] + (float)xm[q];   // exact: the split's two parts
            vs[q] = valid ? fmaf(-xs, cC[q], fmaf(ad[rb][sb][q], cA[q], -cB[q])) : 0.0f;
            gmo = fmaxf(gmo, fabsf(vs[q]));
          }
          s16x4 p0, p1;
          split2_x4(vs, p0, p1);
          // one 16-byte cell per lane: the lanes of 16-lane rows 2r / 2r+1 (kg even / odd: features i .. i+3 and
          // i+4 .. i+7 of one octet) swap halves (v_permlane16_swap: the odd row's first operand <-> the even
          // row's second), so the even row stores the octet's hi part and the odd row its mid part
          const fb_i32x2 hv = __builtin_bit_cast(fb_i32x2, p0), mv = __builtin_bit_cast(fb_i32x2, p1);
          const auto s0 = __builtin_amdgcn_permlane16_swap(hv[0], mv[0], false, false);
          const auto s1 = __builtin_amdgcn_permlane16_swap(hv[1], mv[1], false, false);
          pcell[rb][sb] = u32x4{s0[0], s1[0], s0[1], s1[1]};
        }
      }
      RB_T(ck2);
#if !PCN_RB_NOWAIT
      __builtin_amdgcn_s_waitcnt(fb_vmcnt(NST));   // this wave's DMAs (its stores may fly)
#endif
      __builtin_amdgcn_s_waitcnt(0xC07F);
      __builtin_amdgcn_s_barrier();
      RB_T(ck3);
      cA += ck1 - ck0;
      cB += ck2 - ck1;
      cW += ck3 - ck2;
    }
    RB_T(cL1);
#if PCN_RB_CLK
    if (layer == 2 && lane == 0 && bid < 512) {
      unsigned long long* g = g_rbclk[bid * 8 + wv];
      g[0] = cA; g[1] = cB; g[2] = cW; g[3] = cL1 - cL0; g[4] = (unsigned long long)nk;
    }
#endif
    if (nk > 0) {   // the last tile's cells
#pragma unroll
      for (int rb = 0; rb < 2; ++rb)
#pragma unroll
        for (int sb = 0; sb < 2; ++sb) store_cell(rb, sb, pr + (nk - 1) * npair, pcell[rb][sb]);
    }
    gmo = wave_max_f(gmo) * gui;
    if (lane == 0) atomicMax(gmax_out + ((bid * 4 + rw) & (GMAX_SLOTS - 1)), __float_as_uint(gmo));
  } else {
    // ---- W: x of tile k + 1, weight gradient rows j = 64 rw + 16 jb + lm (4 blocks) x the half's 128 columns
    f32x4 aw[4][8];
#pragma unroll
    for (int jb = 0; jb < 4; ++jb)
#pragma unroll
      for (int ib = 0; ib < 8; ++ib) aw[jb][ib] = f32x4{};
    const int trq = lm >> 2, trp = lm & 3;
    [[maybe_unused]] unsigned long long ck0 = 0, ck1 = 0, ck2 = 0, ck3 = 0, cA = 0, cB = 0, cW = 0, cL0 = 0, cL1 = 0;
    RB_T(cL0);
    for (int k = 0; k < nk; ++k) {
      RB_T(ck0);
#if !PCN_RB_NODMA
      if (k + 1 < nk) dma_g(k + 1);
      if (k + 2 < nk) dma_enc(k + 2);
#endif
#if !PCN_RB_NORM
      if (k + 1 < nk) remat_x(k + 1);
#endif
      RB_T(ck1);
      const char* const sp = fb + (size_t)(k & 1) * FB_BUF;
      auto read8 = [&](unsigned a0, unsigned a1, auto partc) {
        constexpr int Q = decltype(partc)::value;
        const s16x4 h0 = fb_tr<0>(a0), h1 = fb_tr<0>(a1), m0 = fb_tr<Q>(a0), m1 = fb_tr<Q>(a1);
        return std::array<s16x4, 4>{h0, h1, m0, m1};
      };
      auto join = [](const s16x4& a, const s16x4& b) {
        return __builtin_bit_cast(f16x8, __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7));
      };
      using QG = std::integral_constant<int, FB_GPART>;
      using QX = std::integral_constant<int, FB_XPART>;
      const unsigned ga = fb_lds_addr(sp), xa = fb_lds_addr(sp + 2 * FB_GPART);
      const int tr0 = 8 * kg + trq, tr1 = tr0 + 4;
      auto xrd = [&](int ib) {
        const int col = 16 * ib + 4 * trp;
        return read8(xa + fb_off<FB_XP>(tr0, col), xa + fb_off<FB_XP>(tr1, col), QX{});
      };
      std::array<s16x4, 4> ra[4], rbx[2];
#pragma unroll
      for (int jb = 0; jb < 4; ++jb) {
        const int col = 64 * rw + 16 * jb + 4 * trp;
        ra[jb] = read8(ga + gs_off(tr0, col >> 3) + 2 * (col & 7), ga + gs_off(tr1, col >> 3) + 2 * (col & 7), QG{});
      }
      rbx[0] = xrd(0);
      fb_lgkm<4>(ra);
      f16x8 A[4][2];
#pragma unroll
      for (int jb = 0; jb < 4; ++jb) {
        A[jb][0] = join(ra[jb][0], ra[jb][1]);
        A[jb][1] = join(ra[jb][2], ra[jb][3]);
      }
#pragma unroll
      for (int ib = 0; ib < 8; ++ib) {
        std::array<s16x4, 4> cur[1] = {rbx[ib & 1]};
        if (ib + 1 < 8) {
          rbx[(ib + 1) & 1] = xrd(ib + 1);
          fb_lgkm<4>(cur);
        } else {
          fb_lgkm<0>(cur);
        }
        rbx[ib & 1] = cur[0];
        const f16x8 B0 = join(rbx[ib & 1][0], rbx[ib & 1][1]), B1 = join(rbx[ib & 1][2], rbx[ib & 1][3]);
#pragma unroll
        for (int jb = 0; jb < 4; ++jb) {
#if PCN_RB_NOWG
          aw[jb][ib] += __builtin_bit_cast(f32x4, B0) + __builtin_bit_cast(f32x4, A[jb][1]);
#else
          aw[jb][ib] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A[jb][0], B0, aw[jb][ib], 0, 0, 0);
          aw[jb][ib] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A[jb][0], B1, aw[jb][ib], 0, 0, 0);
          aw[jb][ib] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A[jb][1], B0, aw[jb][ib], 0, 0, 0);
#endif
        }
      }
      RB_T(ck2);
#if !PCN_RB_NOWAIT
      __builtin_amdgcn_s_waitcnt(fb_vmcnt(0));
#endif
      __builtin_amdgcn_s_waitcnt(0xC07F);
      __builtin_amdgcn_s_barrier();
      RB_T(ck3);
      cA += ck1 - ck0;
      cB += ck2 - ck1;
      cW += ck3 - ck2;
    }
    RB_T(cL1);
#if PCN_RB_CLK
    if (layer == 2 && lane == 0 && bid < 512) {
      unsigned long long* g = g_rbclk[bid * 8 + wv];
      g[0] = cA; g[1] = cB; g[2] = cW; g[3] = cL1 - cL0; g[4] = (unsigned long long)nk;
    }
#endif
    float* pb = part + (size_t)pr * WgradCfg<LAY>::PART;
#pragma unroll
    for (int ib = 0; ib < 8; ++ib) {
      const float cu = cst[128 + 16 * ib + lm] * gun;
#pragma unroll
      for (int jb = 0; jb < 4; ++jb)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          pb[(size_t)(64 * rw + 16 * jb + 4 * kg + r) * C + COL + 128 * hf + 16 * ib + lm] = aw[jb][ib][r] * cu;
    }
    // sum_s g_L (the Linear bias gradient, and the beta_{L-1} term of dW_L in the reduction): exactly zero -- BatchNorm
    // L's backward leaves every neuron's g with zero chunk mean (models.py:183-203: Linear -> BatchNorm); the
    // reference's autograd carries rounding noise there, the fold path an exact zero like this one
    if (hf == 0 && kg == 0) {
#pragma unroll
      for (int jb = 0; jb < 4; ++jb) pb[(size_t)256 * C + 64 * rw + 16 * jb + lm] = 0.0f;
    }
  }
  __syncthreads();
  if (red.mode != 0) fb_reduce_row(red, reinterpret_cast<double*>(fb), t);
}

// ---- k_bwd_remat3: the rematerialised layer launch with the weight gradient taken over the ENCODING columns
// (VERDICT r5 item 2).  Inside a chunk every layer input is x = h_{L-1} - mean_{L-1} = P'_{L-1} d (d = e - ebar, the
// identity-activation premise the remat already rests on) and sum_s g_L = 0 (BatchNorm L's backward), so
//   G_L = sum_s g_L (x) x = (sum_s g_L (x) d) P'_{L-1}^T :
// the tile loop contracts g_L with the 64 encoding columns (24 MFMAs per W wave and tile instead of 96 over the 256
// x columns) and k_gd_proj applies P'_{L-1}^T in float64 once per chunk and layer (256 x 64 x 256).  x itself is
// still made per tile (the BatchNorm backward's x kk term), but only as that term: the W waves write
// xc = x (kk invstd gamma 2^eo) + gm invstd gamma 2^eo in fp32 (no hi / mid split: x is no longer an MFMA operand),
// and the D waves' epilogue is one fma, 2^eo g_{L-1} = dy A - xc.  Per SIMD and tile the matrix pipe carries 96 + 24
// + 24 MFMA groups instead of 96 + 24 + 96.  The weight-gradient partials (per pair: 256 rows x the half's 32 encoding
// columns, in k_wgrad_enc's 64-column layout) are 4x smaller; the next launch's tail sums them per row into the
// chunk's float64 G_d (gd_reduce_row), k_gd_tail sums layer 1's.  The skip layer's encoding columns ARE its G_d, so
// k_wgrad_enc is left with g_0 alone.
constexpr int R3_XC = 32 * 128 * 4;                      // xc: [32 samples][32 chunks of 4 features] fp32
static_assert(2 * FB_GPART + R3_XC == FB_BUF, "remat3 keeps k_bwd_remat2's tile buffer size");
constexpr int R3_ENC_SLOTS = 3;                          // remat of tile k + 1 and wgrad of tile k, DMA of k + 2
constexpr size_t R3_LDS = 2 * (size_t)FB_BUF + R3_ENC_SLOTS * FB_ENC + 8 * 128 * sizeof(float);
static_assert(R3_LDS <= 160 * 1024, "k_bwd_remat3 LDS");
// layer 1's launch with dW_0's encoding columns fused (LAST): a fourth encoding slot (tile k - 1's image stays until
// its G_0 is formed) and the half's g_0 tile, split, in the g layout (2 parts x 16 octets x 32 cells x 16 B)
constexpr int R3_G0 = 2 * 16 * 32 * 16;
constexpr size_t R3L_LDS = 2 * (size_t)FB_BUF + 4 * FB_ENC + 8 * 128 * sizeof(float) + R3_G0;
static_assert(R3L_LDS <= 160 * 1024, "k_bwd_remat3<true, true> LDS");
constexpr size_t GD_PART = WgradCfg<1>::PART;            // 256 x 64 + 256 floats per pair
constexpr int GD_LAYER = 256 * 64;                       // doubles of one layer's G_d
// 16-byte chunk c4 (features 4 c4 .. 4 c4 + 3) of sample s: 16 lanes of one k-group (16 samples) on 16 distinct bank
// groups for the W waves' stores and the D waves' reads alike
__device__ __forceinline__ int r3_xoff(int s, int c4) { return s * 512 + 16 * (c4 ^ (s & 15)); }

// Row m = blockIdx.x of a layer's G_d over np pair partials (WgradCfg<1> layout), float64, by NT threads: column
// t & 63, NT / 64 slices of the pairs; red: NT doubles of LDS
template <int NT>
__device__ __forceinline__ void gd_reduce_row(const float* __restrict__ part, int np, double* __restrict__ gd,
                                              double* red, int t) {
  constexpr int NS = NT / 64;
  const int m = (int)blockIdx.x, c = t & 63, sl = t >> 6;
  const int per = (np + NS - 1) / NS, b0 = sl * per, b1 = min(np, b0 + per);
  const float* pc = part + (size_t)m * 64 + c;
  double a[4] = {0.0, 0.0, 0.0, 0.0};
  int b = b0;
  for (; b + 16 <= b1; b += 16) {
    float v[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) v[j] = pc[(size_t)(b + j) * GD_PART];
#pragma unroll
    for (int j = 0; j < 16; ++j) a[j & 3] += (double)v[j];
  }
  for (; b < b1; ++b) a[0] += (double)pc[(size_t)b * GD_PART];
  red[t] = (a[0] + a[1]) + (a[2] + a[3]);
  __syncthreads();
  if (t < 64) {
    double s = 0.0;
#pragma unroll
    for (int i = 0; i < NS; ++i) s += red[64 * i + t];
    gd[(size_t)m * 64 + t] = s;
  }
  __syncthreads();
}

// WEPI (version 4): the BatchNorm-backward epilogue and the g_{L-1} stores move from the D to the W waves, which
// hold x in registers from their own rematerialisation: a D wave runs only the 96 data-gradient MFMAs of a tile and
// writes its fp32 accumulators to LDS (the xc slot's 16 KiB), a W wave takes tile k - 1's accumulators there after
// the barrier, finishes g_{L-1} = dy A - (x X + B) and stores it, then makes x of tile k and G_d of tile k (48 MFMAs):
// per SIMD 96 MFMAs against 48 + the epilogue's VALU, instead of 96 + epilogue against 48.
//
// LAST (layer 1, with WEPI): g_0 is consumed in the launch that makes it -- its only use is dW_0's encoding columns
// G_0 = sum_s g_0 (x) d -- so the W waves write their g_0 cells of tile k - 1 to the LDS g_0 tile instead of HBM and
// form G_0 there (24 more MFMAs: their 32 rows x the 64 encoding columns), one partial set per pair in
// k_wgrad_enc's layout (part0): k_wgrad_enc and g_0's 1 KiB/sample round trip through HBM are gone.
#ifndef PCN_R3_ABL
#define PCN_R3_ABL 0    // timing-only ablations of k_bwd_remat3<true> (wrong results): 1 W waves idle, 2 D waves
                        // without MFMAs, 3 D waves' B operands from registers instead of LDS, 4 no DMA waits
#endif
#ifndef PCN_R3_WORDER
#define PCN_R3_WORDER 2   // W waves: G_d's transposed reads issued 1 after the epilogue / 2 before it (0: after remat)
#endif
#ifndef PCN_R3_DPF
#define PCN_R3_DPF 0      // D waves: the next k-step's B operands read one k-step ahead into registers
#endif
#ifndef PCN_R3_KREG
#define PCN_R3_KREG 1   // the W waves' per-feature epilogue / remat constants in registers (0: read from LDS, A/B)
#endif
template <bool WEPI, bool LAST = false, int NW = 4>
__global__ __launch_bounds__(64 * (4 + NW), 1) void k_bwd_remat3(const char* __restrict__ gin, char* __restrict__ gout,
                                                        const f16x8* __restrict__ wt,
                                                        const int* __restrict__ sw, int layer, int64_t n,
                                                        const float* __restrict__ coefp, const float* __restrict__ bnb,
                                                        const float* __restrict__ gamma, int* __restrict__ gexp,
                                                        const float* __restrict__ wcol,
                                                        const unsigned* __restrict__ gmax_in,
                                                        unsigned* __restrict__ gmax_out, float* __restrict__ part,
                                                        const float* __restrict__ rpart, double* __restrict__ rgd,
                                                        const char* __restrict__ enc,
                                                        const f16x8* __restrict__ px, const float* __restrict__ pxs,
                                                        const unsigned* __restrict__ pbound, float* __restrict__ part0) {
  static_assert(!LAST || WEPI, "the fused layer-0 columns need the W-wave epilogue");
  static_assert(NW == 4 || (NW == 8 && WEPI && !LAST), "eight W waves: the W-wave epilogue, hidden layers");
  // NW W waves: FW features of the half each (RBW row blocks of 16) and GR rows of G_d (JBW blocks of 16)
  constexpr int FW = 128 / NW, RBW = FW / 16, GR = 256 / NW, JBW = GR / 16;
  constexpr int NST = LAST ? 0 : 2 * RBW;   // a g-storing wave's global stores per tile
  constexpr int NS = LAST ? 4 : R3_ENC_SLOTS;   // encoding slots
  extern __shared__ __attribute__((aligned(16))) char fb[];
  char* const enb = fb + 2 * FB_BUF;
  float* const cst = reinterpret_cast<float*>(enb + NS * FB_ENC);   // [. | 2^-e | B | . | invstd | A | X | bound]
  char* const g0i = enb + NS * FB_ENC + 8 * 128 * sizeof(float);   // LAST: the half's g_0 tile
  const int t = threadIdx.x, lane = t & 63, kg = lane >> 4, lm = lane & 15;
  const int wv = __builtin_amdgcn_readfirstlane(t >> 6);
  const int rw = wv & 3;   // index within the role (D waves)
  const int rwW = wv - 4;  // index within the W role
  const int bid = (int)blockIdx.x, hf = (bid >> 3) & 1, pr = ((bid >> 4) << 3) | (bid & 7);
  const int npair = (int)gridDim.x >> 1;
  const int nt = (int)((n + 31) / 32);
  const int nk = pr < nt ? (nt - 1 - pr) / npair + 1 : 0;
  const float rn = sqrtf((float)n);
  if (t < 128) {
    const int c = 128 * hf + t;
    const float invstd = coefp[256 + c];
    const float bnd = rn / invstd;   // Samuelson: |h - mean| <= sqrt(n) sigma
    int e = (bnd > 0.0f && bnd < 3.0e38f) ? 14 - ilogbf(bnd) : 0;
    e = e < -60 ? -60 : e > 60 ? 60 : e;
    cst[128 + t] = ldexpf(1.0f, -e);
    cst[256 + t] = bnb[c];
    cst[384 + t] = bnb[256 + c];
    cst[512 + t] = invstd;
    cst[640 + t] = gamma[c];
    cst[768 + t] = ldexpf(pxs[c], e);
  }
  unsigned gmx = 0;
  for (int i = 0; i < GMAX_SLOTS; ++i) gmx = max(gmx, gmax_in[i]);
  {
    const int c = t & 255;
    const float invstd = coefp[256 + c];
    float ob = ((wcol[c] * __uint_as_float(gmx) + fabsf(bnb[c])) + rn / invstd * fabsf(bnb[256 + c])) * invstd *
               fabsf(gamma[c]) * 1.01f;
    ob = wave_max_f(ob);
    if (lane == 0) cst[896 + wv] = ob;
  }
  // W waves: their P' rows (features 32 rw .. 32 rw + 31 of the half, 64 columns, hi / mid) in registers for the
  // whole launch -- the same 8 f16x8 every tile (the LDS copy cost 8 KiB of reads per wave and tile)
  f16x8 pa_r[2][RBW][2];   // [ks][rb][part]
  if (wv >= 4) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int rb = 0; rb < RBW; ++rb)
#pragma unroll
        for (int p = 0; p < 2; ++p)
          pa_r[ks][rb][p] = px[(size_t)(128 * hf + FW * rwW + 16 * rb + lm) * 16 + (2 * ks + p) * 4 + kg];
  }
  const int eg = gexp[layer];
  const float gun = ldexpf(1.0f, -eg);
  __syncthreads();
  float obm = cst[896];
#pragma unroll
  for (int i = 1; i < 4 + NW; ++i) obm = fmaxf(obm, cst[896 + i]);
  const int eo = tile_scale_exp(obm);
  const float gso = ldexpf(1.0f, eo);
  if (bid == 0 && t == 0) gexp[layer - 1] = eo;
  // the epilogue's per-feature constants folded:
  //   2^eo g_{L-1} = dy A - xc,  A = dun invstd gamma 2^eo  (slot 640),
  //   xc = m X + B,  m = the remat MFMA's output,  X = x scale 2^-e kk invstd gamma 2^eo (slot 768),
  //   B = gm invstd gamma 2^eo (slot 256)
  const float dun = ldexpf(1.0f, -sw[layer]) * gun;
  if (t < 128) {
    const float sc = cst[512 + t] * cst[640 + t] * gso;
    const float cb = cst[256 + t] * sc, cc = cst[128 + t] * cst[384 + t] * sc;
    cst[640 + t] = dun * sc;
    cst[256 + t] = cb;
    cst[768 + t] = cst[768 + t] * cc;   // (a power of two times cc: exact)
  }
  auto dma_g = [&](int k) {
    const int tl = pr + k * npair;
    char* const sb = fb + (size_t)(k & 1) * FB_BUF;
    int ln = lane;
    asm volatile("" : "+v"(ln));
#pragma unroll
    for (int m = 0; m < 4; ++m)
      fb_glds16(gin + (size_t)tl * GS_TILE + (4 * wv + m) * 1024 + 16 * ln, sb + (4 * wv + m) * 1024);
  };
  auto dma_enc = [&](int k) {
    const int tl = pr + k * npair;
    int ln = lane;
    asm volatile("" : "+v"(ln));
    fb_glds16(enc + (size_t)tl * FB_ENC + wv * 1024 + ln * 16, enb + (k % NS) * FB_ENC + wv * 1024);
  };
  // W waves: xc of tile k, features 32 rw .. 32 rw + 31 of the half (2 row blocks of P'), enc slot k % 3 -> buffer k & 1
  auto remat_xc = [&](int k) {
    const char* eb = enb + (k % NS) * FB_ENC;
    char* const xb = fb + (size_t)(k & 1) * FB_BUF + 2 * FB_GPART;
    f32x4 ax[RBW][2];
#pragma unroll
    for (int rb = 0; rb < RBW; ++rb) ax[rb][0] = ax[rb][1] = f32x4{};
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const auto& pa = pa_r[ks];
#pragma unroll
      for (int sb = 0; sb < 2; ++sb) {
        const int o = fb_eoff(16 * sb + lm, 4 * ks + kg);
        const f16x8 bh = *reinterpret_cast<const f16x8*>(eb + o);
        const f16x8 bm = *reinterpret_cast<const f16x8*>(eb + FB_ENC / 2 + o);
#pragma unroll
        for (int rb = 0; rb < RBW; ++rb) {
          ax[rb][sb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(pa[rb][0], bh, ax[rb][sb], 0, 0, 0);
          ax[rb][sb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(pa[rb][0], bm, ax[rb][sb], 0, 0, 0);
          ax[rb][sb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(pa[rb][1], bh, ax[rb][sb], 0, 0, 0);
        }
      }
    }
#pragma unroll
    for (int rb = 0; rb < RBW; ++rb) {
      const int il = FW * rwW + 16 * rb + 4 * kg;
      const f32x4 X = *reinterpret_cast<const f32x4*>(cst + 768 + il);
      const f32x4 B = *reinterpret_cast<const f32x4*>(cst + 256 + il);
#pragma unroll
      for (int sb = 0; sb < 2; ++sb) {
        f32x4 v;
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = fmaf(ax[rb][sb][q], X[q], B[q]);
        *reinterpret_cast<f32x4*>(xb + r3_xoff(16 * sb + lm, il >> 2)) = v;
      }
    }
  };
  if (nk > 0) {
    if (wv < 8) {   // (waves 8.. of the eight-W-wave form issue no DMA)
      dma_g(0);
      dma_enc(0);
      if (nk > 1) dma_enc(1);
    }
    __builtin_amdgcn_s_waitcnt(fb_vmcnt(0));
    __builtin_amdgcn_s_barrier();
    if (!WEPI && wv >= 4) remat_xc(0);
  }
  __builtin_amdgcn_s_waitcnt(0xC07F);
  __builtin_amdgcn_s_barrier();
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  if constexpr (WEPI) {
    if (wv < 4) {
      // ---- D: the data-gradient MFMAs of features 128 hf + 32 rw + 16 rb + lm; accumulators to LDS
      f16x8 wr[8][2][2];
      {
        const f16x8* __restrict__ w8 = wt + lane;
#pragma unroll
        for (int ks = 0; ks < 8; ++ks)
#pragma unroll
          for (int rb = 0; rb < 2; ++rb)
#pragma unroll
            for (int p = 0; p < 2; ++p) wr[ks][rb][p] = w8[((ks * 16 + 8 * hf + 2 * rw + rb) * 2 + p) * 64];
      }
#pragma unroll
      for (int ks = 0; ks < 8; ++ks)
        asm volatile("" ::"v"(wr[ks][0][0]), "v"(wr[ks][0][1]), "v"(wr[ks][1][0]), "v"(wr[ks][1][1]));
      constexpr int ABL = LAST ? 0 : PCN_R3_ABL;
      for (int k = 0; k < nk; ++k) {
        if (k + 1 < nk) dma_g(k + 1);
        if (k + 2 < nk) dma_enc(k + 2);
        char* const sp = fb + (size_t)(k & 1) * FB_BUF;
        f32x4 ad[2][2] = {{f32x4{}, f32x4{}}, {f32x4{}, f32x4{}}};
        constexpr bool DPF = !LAST && PCN_R3_DPF;
        f16x8 bq[2][2][2];   // DPF: [k-step parity][sb][part], the next k-step's operands read ahead
        auto bload = [&](int ks) {
#pragma unroll
          for (int sb = 0; sb < 2; ++sb) {
            const int o = gs_off(16 * sb + lm, 4 * ks + kg);
            bq[ks & 1][sb][0] = *reinterpret_cast<const f16x8*>(sp + o);
            bq[ks & 1][sb][1] = *reinterpret_cast<const f16x8*>(sp + FB_GPART + o);
          }
        };
        if (DPF) bload(0);
#pragma unroll
        for (int ks = 0; ks < (ABL == 2 ? 0 : 8); ++ks) {
          if (DPF && ks + 1 < 8) bload(ks + 1);
#pragma unroll
          for (int sb = 0; sb < 2; ++sb) {
            const int o = gs_off(16 * sb + lm, 4 * ks + kg);
            const f16x8 bh = DPF ? bq[ks & 1][sb][0] : ABL == 3 ? wr[(ks + 1) & 7][sb][0]
                                                               : *reinterpret_cast<const f16x8*>(sp + o);
            const f16x8 bm = DPF ? bq[ks & 1][sb][1] : ABL == 3 ? wr[(ks + 2) & 7][sb][1]
                                                               : *reinterpret_cast<const f16x8*>(sp + FB_GPART + o);
#pragma unroll
            for (int rb = 0; rb < 2; ++rb) {
              ad[rb][sb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wr[ks][rb][0], bh, ad[rb][sb], 0, 0, 0);
              ad[rb][sb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wr[ks][rb][0], bm, ad[rb][sb], 0, 0, 0);
              ad[rb][sb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wr[ks][rb][1], bh, ad[rb][sb], 0, 0, 0);
            }
          }
        }
#pragma unroll
        for (int rb = 0; rb < 2; ++rb)
#pragma unroll
          for (int sb = 0; sb < 2; ++sb)
            *reinterpret_cast<f32x4*>(sp + 2 * FB_GPART + r3_xoff(16 * sb + lm, (32 * rw + 16 * rb + 4 * kg) >> 2)) =
                ad[rb][sb];
        if (ABL != 4) __builtin_amdgcn_s_waitcnt(fb_vmcnt(0));
        __builtin_amdgcn_s_waitcnt(0xC07F);
        __builtin_amdgcn_s_barrier();
      }
    } else {
      // ---- W: epilogue + stores of tile k - 1, x of tile k (registers), G_d of tile k
      const float gui = ldexpf(1.0f, -eo);
      float gmo = 0.0f;
      f32x4 xr[RBW][2];   // x X + B of the previous tile
#pragma unroll
      for (int rb = 0; rb < RBW; ++rb) xr[rb][0] = xr[rb][1] = f32x4{};
      f32x4 aw[JBW][2];
#pragma unroll
      for (int jb = 0; jb < JBW; ++jb)
#pragma unroll
        for (int ib = 0; ib < 2; ++ib) aw[jb][ib] = f32x4{};
      const int trq = lm >> 2, trp = lm & 3, tr0 = 8 * kg + trq, tr1 = tr0 + 4;
      auto join = [](const s16x4& a, const s16x4& b) {
        return __builtin_bit_cast(f16x8, __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7));
      };
      auto eoff = [](int r, int c) { return r * 128 + 16 * ((c >> 3) ^ ((r >> 1) & 7)) + 2 * (c & 7); };
      // the epilogue's and the remat's per-feature constants A, X, B of this wave's 2 x 4 features: in registers
      // for the launch (24 VGPRs; 6 KiB of LDS reads per wave and tile saved), except in layer 1's fused launch,
      // whose G_0 accumulators take those registers
      f32x4 kA[RBW], kX[RBW], kB[RBW];
#pragma unroll
      for (int rb = 0; rb < RBW; ++rb) {
        const int il = FW * rwW + 16 * rb + 4 * kg;
        kA[rb] = *reinterpret_cast<const f32x4*>(cst + 640 + il);
        kX[rb] = *reinterpret_cast<const f32x4*>(cst + 768 + il);
        kB[rb] = *reinterpret_cast<const f32x4*>(cst + 256 + il);
      }
      constexpr bool KREG = PCN_R3_KREG && !LAST;
      auto cA_of = [&](int rb, int il) { return KREG ? kA[rb] : *reinterpret_cast<const f32x4*>(cst + 640 + il); };
      auto cX_of = [&](int rb, int il) { return KREG ? kX[rb] : *reinterpret_cast<const f32x4*>(cst + 768 + il); };
      auto cB_of = [&](int rb, int il) { return KREG ? kB[rb] : *reinterpret_cast<const f32x4*>(cst + 256 + il); };
      // tile kq's g_{L-1}: its accumulators (LDS) and xr; kq < 0: zero cells to tile 0's own slots (rewritten by
      // this wave's later stores -- same addresses, program order), so every tile has NST stores behind its DMAs
      auto epilogue = [&](int kq) {
        if (LAST && kq < 0) return;
        const int tq = pr + (kq < 0 ? 0 : kq) * npair;
        const char* adb = fb + (size_t)((kq < 0 ? 0 : kq) & 1) * FB_BUF + 2 * FB_GPART;
#pragma unroll
        for (int rb = 0; rb < RBW; ++rb) {
          const int il = FW * rwW + 16 * rb + 4 * kg, i = 128 * hf + il;
          const f32x4 cA = cA_of(rb, il);
#pragma unroll
          for (int sb = 0; sb < 2; ++sb) {
            const int sm = 16 * sb + lm;
            const bool valid = kq >= 0 && (int64_t)tq * 32 + sm < n;
            const f32x4 ad = *reinterpret_cast<const f32x4*>(adb + r3_xoff(sm, il >> 2));
            f32x4 vs;   // 2^eo g_{L-1}
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              vs[q] = valid ? fmaf(ad[q], cA[q], -xr[rb][sb][q]) : 0.0f;
              gmo = fmaxf(gmo, fabsf(vs[q]));
            }
            s16x4 p0, p1;
            split2_x4(vs, p0, p1);
            const fb_i32x2 hv = __builtin_bit_cast(fb_i32x2, p0), mv = __builtin_bit_cast(fb_i32x2, p1);
            const auto s0 = __builtin_amdgcn_permlane16_swap(hv[0], mv[0], false, false);
            const auto s1 = __builtin_amdgcn_permlane16_swap(hv[1], mv[1], false, false);
            const u32x4 cell = {s0[0], s1[0], s0[1], s1[1]};
            if constexpr (LAST) {
              *reinterpret_cast<u32x4*>(g0i + (kg & 1) * (R3_G0 / 2) + gs_off(sm, il >> 3)) = cell;
            } else {
              char* gt = gout + (size_t)tq * GS_TILE + (kg & 1) * FB_GPART + gs_off(sm, i >> 3);
              __builtin_nontemporal_store(cell, reinterpret_cast<u32x4*>(gt));
            }
          }
        }
      };
      // LAST: G_0 of tile kq, rows 32 rw + 16 jb + 4 kg + r of the half's g_0 (this wave's own epilogue rows, read
      // back transposed from the g_0 tile) x the 64 encoding columns of tile kq's image (slot kq % 4)
      f32x4 a0w[2][4];
#pragma unroll
      for (int jb = 0; jb < 2; ++jb)
#pragma unroll
        for (int ib = 0; ib < 4; ++ib) a0w[jb][ib] = f32x4{};
      auto gd0 = [&](int kq) {
        asm volatile("" ::: "memory");   // the g_0 cell stores above, before the transposed reads
        const unsigned g0a = fb_lds_addr(g0i), ea = fb_lds_addr(enb + (kq % NS) * FB_ENC);
        std::array<s16x4, 4> ra[2], rx[4];
#pragma unroll
        for (int jb = 0; jb < 2; ++jb) {
          const int col = 32 * rw + 16 * jb + 4 * trp;
          const unsigned a0 = g0a + gs_off(tr0, col >> 3) + 2 * (col & 7), a1 = g0a + gs_off(tr1, col >> 3) + 2 * (col & 7);
          ra[jb] = std::array<s16x4, 4>{fb_tr<0>(a0), fb_tr<0>(a1), fb_tr<R3_G0 / 2>(a0), fb_tr<R3_G0 / 2>(a1)};
        }
#pragma unroll
        for (int ib = 0; ib < 4; ++ib) {
          const int c = 16 * ib + 4 * trp;
          const unsigned a0 = ea + eoff(tr0, c), a1 = ea + eoff(tr1, c);
          rx[ib] = std::array<s16x4, 4>{fb_tr<0>(a0), fb_tr<0>(a1), fb_tr<FB_ENC / 2>(a0), fb_tr<FB_ENC / 2>(a1)};
        }
        fb_lgkm<0>(ra);
        fb_lgkm<0>(rx);
#pragma unroll
        for (int ib = 0; ib < 4; ++ib) {
          const f16x8 B0 = join(rx[ib][0], rx[ib][1]), B1 = join(rx[ib][2], rx[ib][3]);
#pragma unroll
          for (int jb = 0; jb < 2; ++jb) {
            const f16x8 A0 = join(ra[jb][0], ra[jb][1]), A1 = join(ra[jb][2], ra[jb][3]);
            a0w[jb][ib] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A0, B0, a0w[jb][ib], 0, 0, 0);
            a0w[jb][ib] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A0, B1, a0w[jb][ib], 0, 0, 0);
            a0w[jb][ib] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A1, B0, a0w[jb][ib], 0, 0, 0);
          }
        }
        asm volatile("" ::: "memory");   // the reads above, before the next tile's cell stores
      };
      auto remat_reg = [&](int k) {
        const char* eb = enb + (k % NS) * FB_ENC;
        f32x4 ax[RBW][2];
#pragma unroll
        for (int rb = 0; rb < RBW; ++rb) ax[rb][0] = ax[rb][1] = f32x4{};
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          const auto& pa = pa_r[ks];
#pragma unroll
          for (int sb = 0; sb < 2; ++sb) {
            const int o = fb_eoff(16 * sb + lm, 4 * ks + kg);
            const f16x8 bh = *reinterpret_cast<const f16x8*>(eb + o);
            const f16x8 bm = *reinterpret_cast<const f16x8*>(eb + FB_ENC / 2 + o);
#pragma unroll
            for (int rb = 0; rb < RBW; ++rb) {
              ax[rb][sb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(pa[rb][0], bh, ax[rb][sb], 0, 0, 0);
              ax[rb][sb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(pa[rb][0], bm, ax[rb][sb], 0, 0, 0);
              ax[rb][sb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(pa[rb][1], bh, ax[rb][sb], 0, 0, 0);
            }
          }
        }
#pragma unroll
        for (int rb = 0; rb < RBW; ++rb) {
          const int il = FW * rwW + 16 * rb + 4 * kg;
          const f32x4 X = cX_of(rb, il), B = cB_of(rb, il);
#pragma unroll
          for (int sb = 0; sb < 2; ++sb)
#pragma unroll
            for (int q = 0; q < 4; ++q) xr[rb][sb][q] = fmaf(ax[rb][sb][q], X[q], B[q]);
        }
      };
      constexpr int ABLW = LAST ? 0 : PCN_R3_ABL;
      for (int k = 0; k < nk; ++k) {
        if (wv < 8 && k + 1 < nk) dma_g(k + 1);
        if (wv < 8 && k + 2 < nk) dma_enc(k + 2);
        if (ABLW == 1) {
          __builtin_amdgcn_s_waitcnt(fb_vmcnt(0));
          __builtin_amdgcn_s_waitcnt(0xC07F);
          __builtin_amdgcn_s_barrier();
          continue;
        }
        const char* const sp = fb + (size_t)(k & 1) * FB_BUF;
        const unsigned ga = fb_lds_addr(sp), ea = fb_lds_addr(enb + (k % NS) * FB_ENC);
        std::array<s16x4, 4> ra[JBW], rx[2];
        auto gd_reads = [&]() {
#pragma unroll
          for (int jb = 0; jb < JBW; ++jb) {
            const int col = GR * rwW + 16 * jb + 4 * trp;
            const unsigned a0 = ga + gs_off(tr0, col >> 3) + 2 * (col & 7), a1 = ga + gs_off(tr1, col >> 3) + 2 * (col & 7);
            ra[jb] = std::array<s16x4, 4>{fb_tr<0>(a0), fb_tr<0>(a1), fb_tr<FB_GPART>(a0), fb_tr<FB_GPART>(a1)};
          }
#pragma unroll
          for (int ib = 0; ib < 2; ++ib) {
            const int c = 32 * hf + 16 * ib + 4 * trp;
            const unsigned a0 = ea + eoff(tr0, c), a1 = ea + eoff(tr1, c);
            rx[ib] = std::array<s16x4, 4>{fb_tr<0>(a0), fb_tr<0>(a1), fb_tr<FB_ENC / 2>(a0), fb_tr<FB_ENC / 2>(a1)};
          }
          asm volatile("" ::: "memory");   // (issued before the LDS reads that follow)
        };
        constexpr int WO = LAST ? 0 : PCN_R3_WORDER;
        if (WO == 2) gd_reads();
        epilogue(k - 1);
        if (LAST && k > 0) gd0(k - 1);
        if (WO == 1) gd_reads();
        remat_reg(k);
        if (WO == 0) gd_reads();
        fb_lgkm<0>(ra);
        fb_lgkm<0>(rx);
#pragma unroll
        for (int ib = 0; ib < 2; ++ib) {
          const f16x8 B0 = join(rx[ib][0], rx[ib][1]), B1 = join(rx[ib][2], rx[ib][3]);
#pragma unroll
          for (int jb = 0; jb < JBW; ++jb) {
            const f16x8 A0 = join(ra[jb][0], ra[jb][1]), A1 = join(ra[jb][2], ra[jb][3]);
            aw[jb][ib] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A0, B0, aw[jb][ib], 0, 0, 0);
            aw[jb][ib] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A0, B1, aw[jb][ib], 0, 0, 0);
            aw[jb][ib] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A1, B0, aw[jb][ib], 0, 0, 0);
          }
        }
        if (ABLW != 4) __builtin_amdgcn_s_waitcnt(fb_vmcnt(NST));   // this wave's DMAs (its stores may fly)
        __builtin_amdgcn_s_waitcnt(0xC07F);
        __builtin_amdgcn_s_barrier();
      }
      if (nk > 0) epilogue(nk - 1);   // (the loop's last barrier: D's accumulators of tile nk - 1 are in LDS)
      if (LAST && nk > 0) gd0(nk - 1);
      gmo = wave_max_f(gmo) * gui;
      if (lane == 0) atomicMax(gmax_out + ((bid * 4 + rwW) & (GMAX_SLOTS - 1)), __float_as_uint(gmo));
      float* const pb = part + (size_t)pr * GD_PART;
      const int sxyz = remat_sx(0, __uint_as_float(*pbound));
#pragma unroll
      for (int ib = 0; ib < 2; ++ib) {
        const int col = 32 * hf + 16 * ib + lm;
        const float cu = ldexpf(gun, -(col < 3 ? sxyz : 13));
#pragma unroll
        for (int jb = 0; jb < JBW; ++jb)
#pragma unroll
          for (int r = 0; r < 4; ++r) pb[(size_t)(GR * rwW + 16 * jb + 4 * kg + r) * 64 + col] = aw[jb][ib][r] * cu;
      }
      if constexpr (LAST) {   // G_0, unscaled (2^-eo of the g_0 tile, 2^-s of the column); the bias row: exact 0
        float* const p0 = part0 + (size_t)pr * GD_PART;
#pragma unroll
        for (int ib = 0; ib < 4; ++ib) {
          const int col = 16 * ib + lm;
          const float cu = ldexpf(gui, -(col < 3 ? sxyz : 13));
#pragma unroll
          for (int jb = 0; jb < 2; ++jb)
#pragma unroll
            for (int r = 0; r < 4; ++r)
              p0[(size_t)(128 * hf + 32 * rw + 16 * jb + 4 * kg + r) * 64 + col] = a0w[jb][ib][r] * cu;
        }
        if (lane < 32) p0[(size_t)256 * 64 + 128 * hf + 32 * rw + lane] = 0.0f;
      }
    }
  } else if (wv < 4) {
    // ---- D: data gradient of input features 128 hf + 32 rw + 16 rb + lm, epilogue, g_{L-1} stores
    const float gui = ldexpf(1.0f, -eo);
    f16x8 wr[8][2][2];
    {
      const f16x8* __restrict__ w8 = wt + lane;
#pragma unroll
      for (int ks = 0; ks < 8; ++ks)
#pragma unroll
        for (int rb = 0; rb < 2; ++rb)
#pragma unroll
          for (int p = 0; p < 2; ++p) wr[ks][rb][p] = w8[((ks * 16 + 8 * hf + 2 * rw + rb) * 2 + p) * 64];
    }
#pragma unroll
    for (int ks = 0; ks < 8; ++ks)
      asm volatile("" ::"v"(wr[ks][0][0]), "v"(wr[ks][0][1]), "v"(wr[ks][1][0]), "v"(wr[ks][1][1]));
    float gmo = 0.0f;
    typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
    u32x4 pcell[2][2] = {{u32x4{}, u32x4{}}, {u32x4{}, u32x4{}}};
    auto store_cell = [&](int rb, int sb, int tq, const u32x4& cell) {
      const int i = 128 * hf + 32 * rw + 16 * rb + 4 * kg, sm = 16 * sb + lm;
      char* gt = gout + (size_t)tq * GS_TILE + (kg & 1) * FB_GPART + gs_off(sm, i >> 3);
      __builtin_nontemporal_store(cell, reinterpret_cast<u32x4*>(gt));
    };
    // tile k's g_{L-1} cells are stored during tile k + 1's data-gradient MFMAs (k_bwd_remat2's schedule)
    for (int k = 0; k < nk; ++k) {
      const int tl = pr + k * npair;
      const int ptl = k > 0 ? tl - npair : tl;
      if (k + 1 < nk) dma_g(k + 1);
      if (k + 2 < nk) dma_enc(k + 2);
      const char* const sp = fb + (size_t)(k & 1) * FB_BUF;
      const char* xb = sp + 2 * FB_GPART;
      f32x4 ad[2][2] = {{f32x4{}, f32x4{}}, {f32x4{}, f32x4{}}};
#pragma unroll
      for (int ks = 0; ks < 8; ++ks)
#pragma unroll
        for (int sb = 0; sb < 2; ++sb) {
          const int o = gs_off(16 * sb + lm, 4 * ks + kg);
          const f16x8 bh = *reinterpret_cast<const f16x8*>(sp + o);
          const f16x8 bm = *reinterpret_cast<const f16x8*>(sp + FB_GPART + o);
#pragma unroll
          for (int rb = 0; rb < 2; ++rb) {
            ad[rb][sb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wr[ks][rb][0], bh, ad[rb][sb], 0, 0, 0);
            ad[rb][sb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wr[ks][rb][0], bm, ad[rb][sb], 0, 0, 0);
            ad[rb][sb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wr[ks][rb][1], bh, ad[rb][sb], 0, 0, 0);
          }
          if ((ks & 1) && sb == 1) {
            store_cell((ks >> 2) & 1, (ks >> 1) & 1, ptl, pcell[(ks >> 2) & 1][(ks >> 1) & 1]);
            __builtin_amdgcn_sched_barrier(0);
          }
        }
#pragma unroll
      for (int rb = 0; rb < 2; ++rb) {
        const int il = 32 * rw + 16 * rb + 4 * kg;
        const f32x4 cA = *reinterpret_cast<const f32x4*>(cst + 640 + il);
#pragma unroll
        for (int sb = 0; sb < 2; ++sb) {
          const int sm = 16 * sb + lm;
          const bool valid = (int64_t)tl * 32 + sm < n;
          const f32x4 xc = *reinterpret_cast<const f32x4*>(xb + r3_xoff(sm, il >> 2));
          f32x4 vs;   // 2^eo g_{L-1}
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            vs[q] = valid ? fmaf(ad[rb][sb][q], cA[q], -xc[q]) : 0.0f;
            gmo = fmaxf(gmo, fabsf(vs[q]));
          }
          s16x4 p0, p1;
          split2_x4(vs, p0, p1);
          const fb_i32x2 hv = __builtin_bit_cast(fb_i32x2, p0), mv = __builtin_bit_cast(fb_i32x2, p1);
          const auto s0 = __builtin_amdgcn_permlane16_swap(hv[0], mv[0], false, false);
          const auto s1 = __builtin_amdgcn_permlane16_swap(hv[1], mv[1], false, false);
          pcell[rb][sb] = u32x4{s0[0], s1[0], s0[1], s1[1]};
        }
      }
      __builtin_amdgcn_s_waitcnt(fb_vmcnt(NST));   // this wave's DMAs (its stores may fly)
      __builtin_amdgcn_s_waitcnt(0xC07F);
      __builtin_amdgcn_s_barrier();
    }
    if (nk > 0) {   // the last tile's cells
#pragma unroll
      for (int rb = 0; rb < 2; ++rb)
#pragma unroll
        for (int sb = 0; sb < 2; ++sb) store_cell(rb, sb, pr + (nk - 1) * npair, pcell[rb][sb]);
    }
    gmo = wave_max_f(gmo) * gui;
    if (lane == 0) atomicMax(gmax_out + ((bid * 4 + rw) & (GMAX_SLOTS - 1)), __float_as_uint(gmo));
  } else {
    // ---- W: xc of tile k + 1; G_d rows j = 64 rw + 16 jb + lm (4 blocks) x the half's 32 encoding columns
    f32x4 aw[4][2];
#pragma unroll
    for (int jb = 0; jb < 4; ++jb)
#pragma unroll
      for (int ib = 0; ib < 2; ++ib) aw[jb][ib] = f32x4{};
    const int trq = lm >> 2, trp = lm & 3, tr0 = 8 * kg + trq, tr1 = tr0 + 4;
    auto join = [](const s16x4& a, const s16x4& b) {
      return __builtin_bit_cast(f16x8, __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7));
    };
    auto eoff = [](int r, int c) { return r * 128 + 16 * ((c >> 3) ^ ((r >> 1) & 7)) + 2 * (c & 7); };
    for (int k = 0; k < nk; ++k) {
      if (k + 1 < nk) dma_g(k + 1);
      if (k + 2 < nk) dma_enc(k + 2);
      if (k + 1 < nk) remat_xc(k + 1);
      const char* const sp = fb + (size_t)(k & 1) * FB_BUF;
      const unsigned ga = fb_lds_addr(sp), ea = fb_lds_addr(enb + (k % NS) * FB_ENC);
      std::array<s16x4, 4> ra[4], rx[2];
#pragma unroll
      for (int jb = 0; jb < 4; ++jb) {
        const int col = 64 * rw + 16 * jb + 4 * trp;
        const unsigned a0 = ga + gs_off(tr0, col >> 3) + 2 * (col & 7), a1 = ga + gs_off(tr1, col >> 3) + 2 * (col & 7);
        ra[jb] = std::array<s16x4, 4>{fb_tr<0>(a0), fb_tr<0>(a1), fb_tr<FB_GPART>(a0), fb_tr<FB_GPART>(a1)};
      }
#pragma unroll
      for (int ib = 0; ib < 2; ++ib) {
        const int c = 32 * hf + 16 * ib + 4 * trp;
        const unsigned a0 = ea + eoff(tr0, c), a1 = ea + eoff(tr1, c);
        rx[ib] = std::array<s16x4, 4>{fb_tr<0>(a0), fb_tr<0>(a1), fb_tr<FB_ENC / 2>(a0), fb_tr<FB_ENC / 2>(a1)};
      }
      fb_lgkm<0>(ra);
      fb_lgkm<0>(rx);
#pragma unroll
      for (int ib = 0; ib < 2; ++ib) {
        const f16x8 B0 = join(rx[ib][0], rx[ib][1]), B1 = join(rx[ib][2], rx[ib][3]);
#pragma unroll
        for (int jb = 0; jb < 4; ++jb) {
          const f16x8 A0 = join(ra[jb][0], ra[jb][1]), A1 = join(ra[jb][2], ra[jb][3]);
          aw[jb][ib] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A0, B0, aw[jb][ib], 0, 0, 0);
          aw[jb][ib] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A0, B1, aw[jb][ib], 0, 0, 0);
          aw[jb][ib] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A1, B0, aw[jb][ib], 0, 0, 0);
        }
      }
      __builtin_amdgcn_s_waitcnt(fb_vmcnt(0));
      __builtin_amdgcn_s_waitcnt(0xC07F);
      __builtin_amdgcn_s_barrier();
    }
    // this pair's G_d partial, unscaled (2^-gexp[L] of g_L, 2^-s_k of the column): Sigma_s g_L d_k
    float* const pb = part + (size_t)pr * GD_PART;
    const int sxyz = remat_sx(0, __uint_as_float(*pbound));
#pragma unroll
    for (int ib = 0; ib < 2; ++ib) {
      const int col = 32 * hf + 16 * ib + lm;
      const float cu = ldexpf(gun, -(col < 3 ? sxyz : 13));
#pragma unroll
      for (int jb = 0; jb < 4; ++jb)
#pragma unroll
        for (int r = 0; r < 4; ++r) pb[(size_t)(64 * rw + 16 * jb + 4 * kg + r) * 64 + col] = aw[jb][ib][r] * cu;
    }
  }
  // the previous layer's G_d partials, one row per workgroup (LDS as scratch)
  __syncthreads();
  if (rpart) gd_reduce_row<64 * (4 + NW)>(rpart, FB_PAIRS, rgd, reinterpret_cast<double*>(fb), t);
}

// after layer 1's launch: layer 1's G_d (grid.y 0) and layer 0's encoding columns from k_wgrad_enc's g_0 sets
// (grid.y 1: dW_0, db_0), one row per block of 1024
__global__ __launch_bounds__(1024) void k_gd_tail(const float* __restrict__ part1, double* __restrict__ gd1,
                                                  const float* __restrict__ pe0, double* __restrict__ dW0,
                                                  double* __restrict__ db0, int we) {
  __shared__ double red[1024];
  if (blockIdx.y == 0) gd_reduce_row<1024>(part1, FB_PAIRS, gd1, red, threadIdx.x);
  else wgrad_reduce_body<1>(pe0, we, nullptr, nullptr, dW0, db0, nullptr, we, 0);
}

// dW_L[j][i] += alpha_i sum_k G_d[L][j][k] P'_{L-1}[i][k] for the chunk (float64; alpha = invstd gamma of BatchNorm
// L-1, the Linear's input scale), L = 1..7; the skip layer also takes its encoding columns dW_4[j][k] += G_d[4][j][k]
// (its input there is e itself).
struct GdProj {
  double* dW[8];
  const float* coef;   // ws.coef: layer L's BatchNorm constants at 1024 L (alpha at 512)
  const double* gd;    // [8][256][64]
  const double* pp;    // the fold's P' maps [8][C][256][64]
  int64_t C, ci;
};
__global__ __launch_bounds__(256) void k_gd_proj(GdProj g) {
  // one 64 x 64 block of dW_L per workgroup: grid (16 = 4 row blocks x 4 column blocks, 7 layers).  G_d rows
  // j0..j0+63 and P'_{L-1} rows i0..i0+63 (64 encoding columns, the 64th zero) staged in LDS -- every thread's 32
  // loads issued before its first LDS store -- then the 64 x 64 x 64 product on v_mfma_f64_16x16x4_f64, a 32 x 32
  // quadrant per wave (mfma64_quad; the VALU form's 1,008 dependent fma per thread and 16 serialised load rounds
  // took 39 us per chunk)
  __shared__ double gs[64 * TP];
  __shared__ double ps[64 * TP];
  const int L = 1 + (int)blockIdx.y, j0 = 64 * ((int)blockIdx.x >> 2), i0 = 64 * ((int)blockIdx.x & 3);
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const double* gdl = g.gd + (size_t)L * GD_LAYER + (size_t)j0 * 64;
  const double* pp = g.pp + (((size_t)(L - 1) * g.C + g.ci) * 256 + i0) * 64;
  double vg[16], vp[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int idx = t + 256 * q;
    vg[q] = gdl[idx];
    vp[q] = (idx & 63) < 63 ? pp[idx] : 0.0;
  }
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int idx = t + 256 * q, r = idx >> 6, c = idx & 63;
    gs[r * TP + c] = vg[q];
    ps[r * TP + c] = vp[q];
  }
  __syncthreads();
  const int R = 32 * (w >> 1), Cc = 32 * (w & 1);
  f64x4 acc[2][2];
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int y = 0; y < 2; ++y) acc[x][y] = f64x4{0.0, 0.0, 0.0, 0.0};
  // acc(r, c) = sum_k G_d[j0 + r][k] P'[i0 + c][k]
  mfma64_quad<false, true>(gs, ps, R, Cc, lane, acc);
  const int in_f = in_features(L), wc = L == 4 ? 63 : 0;
  double* const dW = g.dW[L];
  // the read-modify-writes of the float64 accumulators: every load issued before the first store (the compiler
  // cannot tell the addresses apart, so interleaved += serialised 16 round trips: 20 us per launch)
  double old[2][2][4];
#pragma unroll
  for (int y = 0; y < 2; ++y)
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        old[x][y][r] = dW[(size_t)(j0 + q_row(R, x, r, lane)) * in_f + wc + i0 + q_col(Cc, y, lane)];
  double ek[16];
  const bool skip = L == 4 && i0 == 0;   // the skip layer's encoding columns: its input there is e itself
  if (skip) {
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int idx = t + 256 * q, r = idx / 63, c = idx - 63 * r;
      ek[q] = idx < 64 * 63 ? dW[(size_t)(j0 + r) * in_f + c] : 0.0;
    }
  }
#pragma unroll
  for (int y = 0; y < 2; ++y) {
    const int i = i0 + q_col(Cc, y, lane);
    const double alpha = (double)g.coef[1024 * (L - 1) + 512 + i];
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        dW[(size_t)(j0 + q_row(R, x, r, lane)) * in_f + wc + i] = old[x][y][r] + alpha * acc[x][y][r];
  }
  if (skip) {
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int idx = t + 256 * q, r = idx / 63, c = idx - 63 * r;
      if (idx < 64 * 63) dW[(size_t)(j0 + r) * in_f + c] = ek[q] + gs[r * TP + c];
    }
  }
}

// k_wgrad_enc: the encoding columns of dW_0 and of the skip layer's dW_4, G = sum_s g (x) d, from the PRE-SPLIT g_0 and
// g_4 images (k_bwd_remat2's output layout, gs_off) and the chunk's encoding image (k_remat_enc: d = e - ebar, fb_eoff),
// DMA'd straight into LDS -- no sincos, no conversion.  d in place of e: sum_s g_L = 0 exactly (BatchNorm follows
// both Linears), so sum g (x) e = sum g (x) d; the layer-0 bias gradient sum_s g_0 is that exact 0.  The two sources
// split between the workgroups of a pair (blocks b and b + 8: the same XCD, so the encoding tile's second read is an
// L2 hit): 40 KiB per tile (one g image + the encoding), a ring of three slots, DMA two tiles ahead (-5 % against
// one workgroup taking both sources at 72 KiB per tile, double-buffered; four slots: no change;
// profiles/r05_wgrad_enc_ab.txt).  8 waves x 32 rows (2 x 16) x the 64 columns in 32 registers; per tile and wave
// 24 transposed reads (ds_read_b64_tr_b16) and 24 v_mfma_f32_16x16x32_f16 (hi.hi + hi.mid + mid.hi).  Partials in
// k_wgrad<1>'s layout, one set per pair and source, unscaled (2^-gexp of the image, 2^-s of the column), summed by
// k_fb_reduce_tail.  HBM per sample: 2 KiB of g + 256 B of encoding.
constexpr int WE_SLOTS = 3, WE_AHEAD = WE_SLOTS - 1;
constexpr size_t WE_BUF = (size_t)GS_TILE + FB_ENC;
constexpr size_t WE_LDS = WE_SLOTS * WE_BUF;
static_assert(WE_LDS <= 160 * 1024, "k_wgrad_enc LDS");
__global__ __launch_bounds__(512, 1) void k_wgrad_enc(const char* __restrict__ g0, const char* __restrict__ g4,
                                                       const char* __restrict__ enc, int64_t n,
                                                       const int* __restrict__ gexp, const unsigned* __restrict__ pbound,
                                                       float* __restrict__ part0, float* __restrict__ part4) {
  extern __shared__ __attribute__((aligned(16))) char wel[];
  const int t = threadIdx.x, lane = t & 63, kg = lane >> 4, lm = lane & 15;
  const int wv = __builtin_amdgcn_readfirstlane(t >> 6);
  // g4 null (the default, k_bwd_remat3 takes the skip layer's encoding columns): every workgroup its own tiles of
  // g_0 and its own partial set; otherwise the pairs split by source
  const bool one = g4 == nullptr;
  const int bid = (int)blockIdx.x, src = one ? 0 : (bid >> 3) & 1;
  const int pr = one ? bid : ((bid >> 4) << 3) | (bid & 7);
  const int npair = one ? (int)gridDim.x : (int)gridDim.x >> 1;
  const int nt = (int)((n + 31) / 32);
  const int nk = pr < nt ? (nt - 1 - pr) / npair + 1 : 0;
  const char* const gsrc = src == 0 ? g0 : g4;
  // one tile: 40 pieces of 1 KiB (g 0..31, encoding 32..39), 5 per wave, into slot k % 3
  auto dma = [&](int k) {
    const size_t tl = (size_t)(pr + k * npair);
    char* const b = wel + (size_t)(k % WE_SLOTS) * WE_BUF;
    int ln = lane;
    asm volatile("" : "+v"(ln));
#pragma unroll
    for (int i = 0; i < 5; ++i) {
      const int p = 5 * wv + i;
      const char* a = p < 32 ? gsrc + tl * GS_TILE + p * 1024 : enc + tl * FB_ENC + (p - 32) * 1024;
      fb_glds16(a + 16 * ln, b + p * 1024);
    }
  };
  auto eoff = [](int r, int c) { return r * 128 + 16 * ((c >> 3) ^ ((r >> 1) & 7)) + 2 * (c & 7); };
  auto join = [](const s16x4& a, const s16x4& b) {
    return __builtin_bit_cast(f16x8, __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7));
  };
  f32x4 aw[2][4];
#pragma unroll
  for (int jb = 0; jb < 2; ++jb)
#pragma unroll
    for (int ib = 0; ib < 4; ++ib) aw[jb][ib] = f32x4{};
  const int trq = lm >> 2, trp = lm & 3, tr0 = 8 * kg + trq, tr1 = tr0 + 4;
  // this wave's DMAs done but for the last m tiles' (5 each)
  auto wait_ahead = [](int m) {
    if (m >= 2) __builtin_amdgcn_s_waitcnt(fb_vmcnt(10));
    else if (m == 1) __builtin_amdgcn_s_waitcnt(fb_vmcnt(5));
    else __builtin_amdgcn_s_waitcnt(fb_vmcnt(0));
  };
  static_assert(WE_AHEAD <= 3, "wait_ahead");
#pragma unroll
  for (int j = 0; j < WE_AHEAD; ++j)
    if (j < nk) dma(j);
  wait_ahead(min(WE_AHEAD - 1, nk - 1));
  __builtin_amdgcn_s_barrier();
  for (int k = 0; k < nk; ++k) {
    if (k + WE_AHEAD < nk) dma(k + WE_AHEAD);
    const char* const b = wel + (size_t)(k % WE_SLOTS) * WE_BUF;
    const unsigned ga = fb_lds_addr(b), ea = fb_lds_addr(b + GS_TILE);
    std::array<s16x4, 4> ra[2], rx[4];
#pragma unroll
    for (int jb = 0; jb < 2; ++jb) {
      const int col = 32 * wv + 16 * jb + 4 * trp;
      const unsigned a0 = ga + gs_off(tr0, col >> 3) + 2 * (col & 7), a1 = ga + gs_off(tr1, col >> 3) + 2 * (col & 7);
      ra[jb] = std::array<s16x4, 4>{fb_tr<0>(a0), fb_tr<0>(a1), fb_tr<FB_GPART>(a0), fb_tr<FB_GPART>(a1)};
    }
#pragma unroll
    for (int ib = 0; ib < 4; ++ib) {
      const int c = 16 * ib + 4 * trp;
      const unsigned a0 = ea + eoff(tr0, c), a1 = ea + eoff(tr1, c);
      rx[ib] = std::array<s16x4, 4>{fb_tr<0>(a0), fb_tr<0>(a1), fb_tr<FB_ENC / 2>(a0), fb_tr<FB_ENC / 2>(a1)};
    }
    fb_lgkm<0>(ra);
    fb_lgkm<0>(rx);
#pragma unroll
    for (int ib = 0; ib < 4; ++ib) {
      const f16x8 B0 = join(rx[ib][0], rx[ib][1]), B1 = join(rx[ib][2], rx[ib][3]);
#pragma unroll
      for (int jb = 0; jb < 2; ++jb) {
        const f16x8 A0 = join(ra[jb][0], ra[jb][1]), A1 = join(ra[jb][2], ra[jb][3]);
        aw[jb][ib] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A0, B0, aw[jb][ib], 0, 0, 0);
        aw[jb][ib] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A0, B1, aw[jb][ib], 0, 0, 0);
        aw[jb][ib] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A1, B0, aw[jb][ib], 0, 0, 0);
      }
    }
    wait_ahead(max(0, min(k + WE_AHEAD, nk - 1) - (k + 1)));   // tile k + 1's DMA landed (later tiles' may fly)
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_s_barrier();
  }
  constexpr int C = WgradCfg<1>::C;
  float* const pb = (src == 0 ? part0 : part4) + (size_t)pr * WgradCfg<1>::PART;
  const float gu = ldexpf(1.0f, -gexp[src == 0 ? 0 : 4]);
  const int sxyz = remat_sx(0, __uint_as_float(*pbound));
#pragma unroll
  for (int ib = 0; ib < 4; ++ib) {
    const int col = 16 * ib + lm;
    const float cu = ldexpf(gu, -(col < 3 ? sxyz : 13));
#pragma unroll
    for (int jb = 0; jb < 2; ++jb)
#pragma unroll
      for (int r = 0; r < 4; ++r) pb[(size_t)(32 * wv + 16 * jb + 4 * kg + r) * C + col] = aw[jb][ib][r] * cu;
  }
  if (kg == 0) {
#pragma unroll
    for (int jb = 0; jb < 2; ++jb) pb[(size_t)256 * C + 32 * wv + 16 * jb + lm] = 0.0f;
  }
}

struct GradTable {
  float* dst[34];
  int64_t off[34];
  int len[34];
};

__global__ void k_grad_emit(GradTable T, const double* __restrict__ acc) {
  const int k = blockIdx.y;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (T.dst[k] && i < T.len[k]) T.dst[k][i] += (float)acc[T.off[k] + i];
}

struct GaccLayout {
  int64_t w[8], b[8], g[8], be[8], wo, bo, total;
};

static GaccLayout gacc_layout() {
  GaccLayout G;
  int64_t o = 0;
  for (int L = 0; L < 8; ++L) {
    G.w[L] = o;
    o += 256 * (int64_t)in_features(L);
    G.b[L] = o;
    o += 256;
    G.g[L] = o;
    o += 256;
    G.be[L] = o;
    o += 256;
  }
  G.wo = o;
  o += 256;
  G.bo = o;
  o += 1;
  G.total = o;
  return G;
}

constexpr int S12_LAYER = S12_COPIES * 512;

struct BwdWs {
  float* h[8];
  float* g[2];
  float* wp;
  float* wt;
  double* stats;
  float* coef;
  float* part;
  double* s12;
  double* ostat;
  double* gacc;
  f32x4* enc;   // encoding tiles of a recomputed chunk (first layer -> skip layer)
  f16x8* wh;    // split-fp16 weight image for recomputation under train math 1/2
  int* sw;
  f16x8* wth;   // split-fp16 W^T image of k_dgrad_h (train math 1/2)
  float* tmax[2];   // per-tile max |dL/dh| of g[0] / g[1] ([tile][8])
  unsigned* gmax;   // per layer L: GMAX_SLOTS partial maxima of the chunk's |dL/dh_L| (float bits; zeroed per chunk)
  unsigned* pbound;   // k_pos_bound's result (float bits)
  f16x8* wth16;       // W^T image of k_bwd_fused (7 layers)
  float* bnb;         // BatchNorm 0..6 backward constants of the chunk (k_fb_prep)
  float* ocst;        // occ_out / BatchNorm 7 backward constants of the chunk (k_fb_prep: [A | B | mean | K][256])
  int* gexp;          // rematerialised backward: scale exponents of the pre-split g images, per layer
  unsigned* gm7;      // rematerialised backward: |g_7| maximum slots (k_g7)
  float* wcol;        // rematerialised backward: column abs sums of W_1..W_7 (k_wcol)
  double* gd;         // k_bwd_remat3: the chunk's G_d = sum_s g_L (x) d per layer [8][256][64]
  size_t bytes;
};

static BwdWs carve_bwd(void* base, int64_t chunk) {
  const size_t tiles = (size_t)((chunk + 31) / 32);
  size_t off = 0;
  auto take = [&](size_t bytes) {
    const size_t o = off;
    off += (bytes + 255) & ~(size_t)255;
    return o;
  };
  size_t oh[8], og[2];
  for (int L = 0; L < 8; ++L) oh[L] = take(tiles * TILE_FLOATS * 4);
  for (int i = 0; i < 2; ++i) og[i] = take(tiles * TILE_FLOATS * 4);
  const size_t oenc = take(tiles * 512 * sizeof(f32x4));
  const size_t ow = take(TRAIN_W_FLOATS * 4), ot = take(DGRAD_W_FLOATS * 4), ost = take(8 * 512 * 8);
  // partials: up to 2 WG_BLOCKS records of the skip layer's layout (its encoding columns, two workgroups per CU)
  // partials: the layered path's 2 x WG_BLOCKS sets; the one-pass path's two hidden-layer sets (FB_PAIRS each) and
  // the two encoding-column sets (WG_BLOCKS each) fit in the same space
  static_assert(2 * FB_PAIRS * WgradCfg<2>::PART + 2 * WG_BLOCKS * WgradCfg<1>::PART <= 2 * WG_BLOCKS * WgradCfg<2>::PART,
                "one-pass backward partial sets");
  const size_t oc = take(8 * 1024 * 4), op = take(2 * WG_BLOCKS * WgradCfg<2>::PART * 4);
  const size_t os = take((8 * S12_LAYER + OSTAT_COPIES * 257 + GMAX_DBL) * 8), oa = take((size_t)gacc_layout().total * 8);
  const size_t owh = take(TRAIN_H_VECS * sizeof(f16x8)), osw = take(16 * sizeof(int));
  const size_t owt = take(7 * HW_H * sizeof(f16x8));
  const size_t otm0 = take(tiles * 8 * sizeof(float)), otm1 = take(tiles * 8 * sizeof(float));
  const size_t opb = take(sizeof(unsigned));
  const size_t owt16 = take(7 * HW_H * sizeof(f16x8)), obnb = take(7 * 512 * sizeof(float));
  const size_t oocst = take(4 * 256 * sizeof(float));
  const size_t ogexp = take(16 * sizeof(int)), ogm7 = take(GMAX_SLOTS * sizeof(unsigned));
  const size_t owcol = take(7 * 256 * sizeof(float));
  const size_t ogd = take(8 * (size_t)GD_LAYER * sizeof(double));
  char* b = (char*)base;
  BwdWs w;
  w.wth = (f16x8*)(b + owt);
  w.tmax[0] = (float*)(b + otm0);
  w.tmax[1] = (float*)(b + otm1);
  w.wh = (f16x8*)(b + owh);
  w.sw = (int*)(b + osw);
  for (int L = 0; L < 8; ++L) w.h[L] = (float*)(b + oh[L]);
  for (int i = 0; i < 2; ++i) w.g[i] = (float*)(b + og[i]);
  w.wp = (float*)(b + ow);
  w.wt = (float*)(b + ot);
  w.stats = (double*)(b + ost);
  w.coef = (float*)(b + oc);
  w.part = (float*)(b + op);
  w.s12 = (double*)(b + os);
  w.ostat = w.s12 + 8 * S12_LAYER;   // s12 per layer [8][COPIES][512], then the output layer's statistics
  w.gmax = (unsigned*)(w.ostat + OSTAT_COPIES * 257);
  w.gacc = (double*)(b + oa);
  w.enc = (f32x4*)(b + oenc);
  w.pbound = (unsigned*)(b + opb);
  w.wth16 = (f16x8*)(b + owt16);
  w.bnb = (float*)(b + obnb);
  w.ocst = (float*)(b + oocst);
  w.gexp = (int*)(b + ogexp);
  w.gm7 = (unsigned*)(b + ogm7);
  w.wcol = (float*)(b + owcol);
  w.gd = (double*)(b + ogd);
  w.bytes = off;
  return w;
}

template <int MODE>
static void launch_wgrad(unsigned blocks, hipStream_t s, const float* rays, int stride, const float* z, int S,
                         int64_t c0, int64_t n, const float* ein, const float* gin, const float* hprev,
                         const float* mu, float* part, const double* esum = nullptr) {
  static std::atomic<uint64_t> attr{0};
  const size_t lds = WgradCfg<MODE>::LDS_BYTES;
  if (pcn_attr_needed(attr)) {
    PCN_HIP(hipFuncSetAttribute((const void*)k_wgrad<MODE>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    pcn_attr_done(attr);
  }
  hipLaunchKernelGGL(k_wgrad<MODE>, dim3(blocks), dim3(512), lds, s, rays, stride, z, S, c0, n, ein, gin, hprev,
                     mu, part, esum);
}

template <int MODE, int LAY, bool H2, int NTP>
static void launch_wgrad_b3_one(unsigned blocks, hipStream_t s, const float* rays, int stride, const float* z, int S,
                                int64_t c0, int64_t n, const float* ein, const float* gin, const float* hprev,
                                const float* mu, const unsigned* gmax, float* part, const unsigned* pbound,
                                const float* gin2 = nullptr, const unsigned* gmax2 = nullptr,
                                float* part2 = nullptr) {
  constexpr int RB = 1;
  using Cfg = Wb3Cfg<MODE, H2>;
  constexpr size_t lds = 3 * Cfg::BUF + (H2 ? 2 * Cfg::NBLK * 32 * sizeof(float) : 0);
  static_assert(lds <= 160 * 1024, "LDS");
  static std::atomic<uint64_t> attr{0};
  if (pcn_attr_needed(attr)) {
    PCN_HIP(hipFuncSetAttribute((const void*)k_wgrad_b3<RB, MODE, LAY, H2, NTP>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    pcn_attr_done(attr);
  }
  hipLaunchKernelGGL((k_wgrad_b3<RB, MODE, LAY, H2, NTP>), dim3(blocks), dim3(512 / RB), lds, s, rays, stride, z, S,
                     c0, ein, gin, hprev, mu, n, gmax, part, pbound, gin2, gmax2, part2);
}

// the weight-gradient partials of k_wgrad<MODE> under the split train math: f16x2 with the forward's product count
template <int MODE>
static void launch_wgrad_b3(unsigned blocks, hipStream_t s, const float* rays, int stride, const float* z, int S,
                            int64_t c0, int64_t n, const float* ein, const float* gin, const float* hprev,
                            const float* mu, const unsigned* gmax, float* part, const unsigned* pbound,
                            bool h_cols = true, bool e_cols = true) {
  auto one = [&](auto mode, auto lay) {
    constexpr int M = decltype(mode)::value, LY = decltype(lay)::value;
    if (g_train_math == 1)
      launch_wgrad_b3_one<M, LY, true, 3>(blocks, s, rays, stride, z, S, c0, n, ein, gin, hprev, mu, gmax, part,
                                          pbound);
    else
      launch_wgrad_b3_one<M, LY, true, 4>(blocks, s, rays, stride, z, S, c0, n, ein, gin, hprev, mu, gmax, part,
                                          pbound);
  };
  if constexpr (MODE != 1) if (h_cols) one(std::integral_constant<int, 0>{}, std::integral_constant<int, MODE>{});
  if constexpr (MODE != 0) if (e_cols) one(std::integral_constant<int, 1>{}, std::integral_constant<int, MODE>{});
}

}  // namespace pcn

extern "C" size_t pcnerf_nof_backward_workspace_bytes(int64_t chunk) { return carve_bwd(nullptr, chunk).bytes; }

// One stored chunk through the one-pass backward: max |dL/dlogit| (k_out_gabs), then in one launch (k_fb_prep) the
// BatchNorm coefficients from the chunk's stored statistics, the BatchNorm-backward constants from the fold and
// occ_out + BatchNorm 7 on the fold's occ_out statistics (no statistics pass); then layers 7..1 each in ONE
// k_bwd_fused launch (g_{L-1} in place over h_{L-1}; layer 7 makes g_7 from h_7) + the partial reduction, the skip
// layer's and layer 0's encoding columns (k_wgrad_b3 MODE 1 on g_4 and g_0, which stay in their store slots).
static void fused_chunk(const NofParamsDev& P, const GaccLayout& G, const BwdWs& ws, const FoldBnBwd& FB, int64_t ci,
                        int64_t c0, int64_t n, const double* stats, float* const (&hh)[8], const float* rays,
                        int ray_stride, const float* z, int n_samples, const float* ein, float eps, const float* grad,
                        hipStream_t s) {
  static std::atomic<uint64_t> attr{0};
  if (pcn_attr_needed(attr)) {
    PCN_HIP(hipFuncSetAttribute((const void*)k_bwd_fused<0, false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)FB_LDS));
    PCN_HIP(hipFuncSetAttribute((const void*)k_bwd_fused<2, false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)FB_LDS));
    PCN_HIP(hipFuncSetAttribute((const void*)k_bwd_fused<0, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)FB_LDS_OUT));
    pcn_attr_done(attr);
  }
  const double dn = (double)n;
  const int64_t ntiles = (n + 31) / 32;
  const unsigned eg = (unsigned)((ntiles + 3) / 4 < 1024 ? (ntiles + 3) / 4 : 1024);
  {
    // max |dL/dlogit| (into the first word of the output-statistics copies, which the one-pass backward does not
    // use: it takes those statistics from the fold; zero before the first chunk, re-zeroed by k_fb_prep), then
    // every constant of the chunk's layers in one launch (k_fb_prep); g_7 itself is made inside layer 7's
    // k_bwd_fused.  Bytes: k_out_gabs reads 4 B of dL/dlogit per sample; k_fb_prep's are per chunk (a few KB)
    ProfScope ps(s, PT_BWD_MISC, 0.0, 4.0 * dn);
    unsigned* gvmax = reinterpret_cast<unsigned*>(ws.ostat);
    hipLaunchKernelGGL(k_out_gabs, dim3(eg < 256 ? eg : 256), dim3(256), 0, s, grad + c0, n, gvmax);
    FbPrepOut po;
    for (int L = 0; L < 8; ++L) po.g[L] = G.g[L];
    po.d_beta7 = ws.gacc + G.be[7];
    po.d_wout = ws.gacc + G.wo;
    po.d_bout = ws.gacc + G.bo;
    hipLaunchKernelGGL(k_fb_prep, dim3(8), dim3(256), 0, s, P, stats, n, eps, ws.coef, FB, ci, ws.bnb, ws.gacc, po,
                       FB.oacc + ci * 257, gvmax, ws.ocst, ws.gmax);
  }
  const unsigned fbg = (unsigned)(2 * FB_PAIRS);
  // two partial sets, by layer parity: layer L's launch writes set L & 1 and sums layer L + 1's set in its prologue
  float* const pset[2] = {ws.part, ws.part + (size_t)FB_PAIRS * WgradCfg<2>::PART};
  for (int L = 7; L >= 1; --L) {
    const float* coefp = ws.coef + 1024 * (L - 1);
    const float* gin = hh[L];   // layer 7: h_7, from which k_bwd_fused<0, true> makes g_7
    FbRed red{nullptr, nullptr, nullptr, nullptr, 0};
    if (L < 7)
      red = FbRed{pset[(L + 1) & 1], ws.coef + 1024 * L, ws.gacc + G.w[L + 1], ws.gacc + G.b[L + 1], L + 1 == 4 ? 2 : 1};
    ProfScope ps(s, PT_BWD_FUSED, 2.0 * 2.0 * 256.0 * 256.0 * dn, 3072.0 * dn);
    auto launch = [&](auto kern, size_t lds) {
      hipLaunchKernelGGL(kern, dim3(fbg), dim3(512), lds, s, gin, hh[L - 1], ws.wth16 + (size_t)(L - 1) * HW_H,
                         ws.sw, L, n, coefp, ws.bnb + 512 * (L - 1), P.bn_w[L - 1], ws.gmax + L * GMAX_SLOTS,
                         ws.gmax + (L - 1) * GMAX_SLOTS, pset[L & 1], grad + c0, (const float*)ws.ocst, red);
    };
    if (L == 7)
      launch(k_bwd_fused<0, true>, FB_LDS_OUT);
    else if (L == 4)
      launch(k_bwd_fused<2, false>, FB_LDS);
    else
      launch(k_bwd_fused<0, false>, FB_LDS);
  }
  // layer 0 and the skip layer's encoding columns in ONE pass over the staged encoding (k_wgrad_b3 MODE 3: g_0 and
  // g_4 in their store slots), one workgroup per CU, two partial sets in layer 0's layout (after the two hidden sets)
  const unsigned we = (unsigned)std::min<int64_t>(ntiles, WG_BLOCKS);
  float* const part_e0 = ws.part + 2 * (size_t)FB_PAIRS * WgradCfg<2>::PART;
  float* const part_e4 = part_e0 + (size_t)WG_BLOCKS * WgradCfg<1>::PART;
  {
    ProfScope ps(s, PT_BWD_WGRAD_H, 2.0 * 2.0 * 256.0 * 64 * dn, 2048.0 * dn);
    launch_wgrad_b3_one<3, 1, true, 3>(we, s, rays, ray_stride, z, n_samples, c0, n, ein, hh[0], nullptr, nullptr,
                                       ws.gmax + 0 * GMAX_SLOTS, part_e0, ws.pbound, hh[4], ws.gmax + 4 * GMAX_SLOTS,
                                       part_e4);
  }
  ProfScope ps(s, PT_BWD_MISC, 0.0, (double)FB_PAIRS * WgradCfg<0>::PART * 4.0 + 2.0 * we * WgradCfg<1>::PART * 4.0);
  hipLaunchKernelGGL(k_fb_reduce_tail, dim3(256, 3), dim3(1024), 0, s, pset[1], (const float*)ws.coef,
                     ws.gacc + G.w[1], ws.gacc + G.b[1], part_e0, ws.gacc + G.w[0], ws.gacc + G.b[0], part_e4,
                     ws.gacc + G.w[4], FB_PAIRS, (int)we);
}

// k_bwd_remat3's layers of one chunk (after k_g7): layers 7..1 (each launch's tail sums the previous layer's G_d
// partials into ws.gd), k_wgrad_enc on g_0 alone, k_gd_tail (layer 1's G_d, dW_0), k_gd_proj (every layer's
// dW_L += alpha (G_d P'^T), and the skip layer's encoding columns)
template <class PR, class PS>
static void remat3_layers(const NofParamsDev& P, const GaccLayout& G, const BwdWs& ws, const FoldBnBwd& FB, const f16x8*,
                          const float*, int64_t ci, int64_t n, const float*, hipStream_t s, char* encimg,
                          const PR& prow, const PS& psrow, char* const (&S)[2], char* S2, float* const (&pset)[2]) {
  const double dn = (double)n;
  const int64_t ntiles = (n + 31) / 32;
  const unsigned fbg = (unsigned)(2 * FB_PAIRS);
  float* const part_e0 = ws.part + 2 * (size_t)FB_PAIRS * WgradCfg<2>::PART;
  const bool fuse0 = g_remat_ver == 4 && g_remat_fuse0;   // layer 1's launch forms dW_0's encoding columns
  for (int L = 7; L >= 1; --L) {
    const float* coefp = ws.coef + 1024 * (L - 1);
    const char* gin = L == 4 ? S2 : S[(7 - L) & 1];
    char* gout = L == 5 ? S2 : S[(8 - L) & 1];
    const unsigned* gmin = L == 7 ? ws.gm7 : ws.gmax + L * GMAX_SLOTS;
    const float* rpart = L < 7 ? pset[(L + 1) & 1] : nullptr;
    double* rgd = ws.gd + (size_t)(L + 1) * GD_LAYER;
    // algorithmic work: the layer's backward as written, data gradient (2 x 256 x 256) + weight gradient
    // (2 x 256 x 256: G_L = sum g (x) x, formed here as (sum g (x) d) P'^T); issued on the matrix pipe per sample:
    // 2 x 256 x 256 + 2 x 256 x 64 (G_d) + 2 x 256 x 64 (x), x 3 products.  Bytes: g_L in (1 KiB), the encoding
    // image (256 B), g_{L-1} out (1 KiB)
    // (layer 1 fused: + 2 x 256 x 64 of dW_0's encoding columns; g_0 stays in LDS: 1 KiB less out)
    const bool last = fuse0 && L == 1;
    ProfScope ps(s, last ? PT_BWD_FUSED_L1 : PT_BWD_FUSED,
                 (2.0 * 2.0 * 256.0 * 256.0 + (last ? 2.0 * 256.0 * 64.0 : 0.0)) * dn,
                 (1024.0 + 256.0 + (last ? 0.0 : 1024.0)) * dn);
    auto launch = [&](auto kern, size_t lds, unsigned threads = 512) {
      hipLaunchKernelGGL(kern, dim3(fbg), dim3(threads), lds, s, gin, gout, ws.wth16 + (size_t)(L - 1) * HW_H,
                         (const int*)ws.sw, L, n, coefp, (const float*)(ws.bnb + 512 * (L - 1)), P.bn_w[L - 1],
                         ws.gexp, (const float*)(ws.wcol + (L - 1) * 256), gmin, ws.gmax + (L - 1) * GMAX_SLOTS,
                         pset[L & 1], rpart, rgd, (const char*)encimg, prow(L - 1), psrow(L - 1),
                         (const unsigned*)ws.pbound, last ? part_e0 : (float*)nullptr);
    };
    if (last) launch(k_bwd_remat3<true, true>, R3L_LDS);
    else if (g_remat_ver == 4 && g_remat_w8) launch(k_bwd_remat3<true, false, 8>, R3_LDS, 768);
    else if (g_remat_ver == 4) launch(k_bwd_remat3<true>, R3_LDS);
    else launch(k_bwd_remat3<false>, R3_LDS);
  }
  // g_0's partial sets: one per pair from the fused layer-1 launch, else one per workgroup of k_wgrad_enc
  const int ne = fuse0 ? FB_PAIRS : (int)std::min<int64_t>(ntiles, 2 * FB_PAIRS);
  if (!fuse0) {
    // 2 x 256 x 64 fp32-FLOP per sample; 1 KiB of g + 256 B of encoding in
    ProfScope ps(s, PT_BWD_WGRAD_H, 2.0 * 256.0 * 64 * dn, (1024.0 + 256.0) * dn);
    hipLaunchKernelGGL(k_wgrad_enc, dim3(2 * FB_PAIRS), dim3(512), WE_LDS, s, (const char*)S[1], (const char*)nullptr,
                       (const char*)encimg, n, (const int*)ws.gexp, (const unsigned*)ws.pbound, part_e0,
                       (float*)nullptr);
  }
  ProfScope ps(s, PT_BWD_MISC, 0.0, (double)FB_PAIRS * GD_PART * 4.0 + ne * WgradCfg<1>::PART * 4.0);
  hipLaunchKernelGGL(k_gd_tail, dim3(256, 2), dim3(1024), 0, s, (const float*)pset[1], ws.gd + GD_LAYER,
                     (const float*)part_e0, ws.gacc + G.w[0], ws.gacc + G.b[0], ne);
  GdProj gp;
  for (int L = 0; L < 8; ++L) gp.dW[L] = ws.gacc + G.w[L];
  gp.coef = ws.coef;
  gp.gd = ws.gd;
  gp.pp = FB.pp;
  gp.C = FB.C;
  gp.ci = ci;
  hipLaunchKernelGGL(k_gd_proj, dim3(16, 7), dim3(256), 0, s, gp);
}

// One chunk through the rematerialised backward (no activation store): max |dL/dlogit|, k_fb_prep on the fold's
// statistics, the chunk's encoding image, g_7 (k_g7), layers 7..1 each in ONE k_bwd_remat2 launch, the encoding
// columns of layers 0 and 4 (k_wgrad_enc on the pre-split g_0 and g_4 and the encoding image), the last partial sums.
// g buffers, all pre-split: S0 / S1 alternate (g_7, g_5, g_3, g_1 in S0; g_6, g_2, g_0 in S1), g_4 in S2 (kept to
// the end for k_wgrad_enc).
static void remat_chunk(const NofParamsDev& P, const GaccLayout& G, const BwdWs& ws, const FoldBnBwd& FB,
                        const f16x8* pimg, const float* pscl, int64_t ci, int64_t c0, int64_t n, const float* rays,
                        int ray_stride, const float* z, int n_samples, float eps, const float* grad, hipStream_t s) {
  static std::atomic<uint64_t> attr{0};
  if (pcn_attr_needed(attr)) {
    PCN_HIP(hipFuncSetAttribute((const void*)k_bwd_remat2<0>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)RB_LDS));
    PCN_HIP(hipFuncSetAttribute((const void*)k_bwd_remat2<2>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)RB_LDS));
    PCN_HIP(hipFuncSetAttribute((const void*)k_bwd_remat3<false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)R3_LDS));
    PCN_HIP(hipFuncSetAttribute((const void*)k_bwd_remat3<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)R3_LDS));
    PCN_HIP(hipFuncSetAttribute((const void*)k_bwd_remat3<true, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)R3L_LDS));
    PCN_HIP(hipFuncSetAttribute((const void*)k_bwd_remat3<true, false, 8>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)R3_LDS));
    PCN_HIP(hipFuncSetAttribute((const void*)k_g7, hipFuncAttributeMaxDynamicSharedMemorySize, (int)G7_LDS));
    PCN_HIP(hipFuncSetAttribute((const void*)k_wgrad_enc, hipFuncAttributeMaxDynamicSharedMemorySize, (int)WE_LDS));
    pcn_attr_done(attr);
  }
  const double dn = (double)n;
  const int64_t ntiles = (n + 31) / 32;
  const unsigned eg = (unsigned)((ntiles + 3) / 4 < 1024 ? (ntiles + 3) / 4 : 1024);
  {
    // k_out_gabs reads 4 B per sample; k_fb_prep's traffic is per chunk (a few KB)
    ProfScope ps(s, PT_BWD_MISC, 0.0, 4.0 * dn);
    unsigned* gvmax = reinterpret_cast<unsigned*>(ws.ostat);
    hipLaunchKernelGGL(k_out_gabs, dim3(eg < 256 ? eg : 256), dim3(256), 0, s, grad + c0, n, gvmax);
    FbPrepOut po;
    for (int L = 0; L < 8; ++L) po.g[L] = G.g[L];
    po.d_beta7 = ws.gacc + G.be[7];
    po.d_wout = ws.gacc + G.wo;
    po.d_bout = ws.gacc + G.bo;
    hipLaunchKernelGGL(k_fb_prep, dim3(8), dim3(256), 0, s, P, (const double*)nullptr, n, eps, ws.coef, FB, ci,
                       ws.bnb, ws.gacc, po, FB.oacc + ci * 257, gvmax, ws.ocst, ws.gmax);
  }
  char* const encimg = reinterpret_cast<char*>(ws.enc);
  const int64_t C = FB.C;
  auto prow = [&](int L) { return pimg + ((size_t)L * C + ci) * 256 * 16; };
  auto psrow = [&](int L) { return pscl + ((size_t)L * C + ci) * 256; };
  char* const S[2] = {reinterpret_cast<char*>(ws.h[0]), reinterpret_cast<char*>(ws.h[1])};
  char* const S2 = reinterpret_cast<char*>(ws.h[2]);
  {
    // the encoding (30 sincosf per sample): 4 B of z in, 256 B of image out per sample
    ProfScope ps(s, PT_BWD_REMAT, 0.0, (4.0 + 256.0) * dn);
    hipLaunchKernelGGL(k_remat_enc, dim3((unsigned)((ntiles + RE_TILES - 1) / RE_TILES)), dim3(32 * RE_TILES), 0, s,
                       rays, ray_stride, z, n_samples, c0, n, FB.eb + ci * 64, ws.pbound, encimg, ws.gm7);
  }
  {
    // g_7: 2 x 256 x 64 fp32-FLOP per sample (h_7 - mean_7); 256 B of image + 4 B in, 1 KiB out
    ProfScope ps(s, PT_BWD_REMAT, 2.0 * 256.0 * 64.0 * dn, (260.0 + 1024.0) * dn);
    hipLaunchKernelGGL(k_g7, dim3((unsigned)std::min<int64_t>(ntiles, G7_BLOCKS)), dim3(512), G7_LDS, s, encimg,
                       grad + c0, n, prow(7), psrow(7), (const float*)ws.ocst, ws.gmax + 7 * GMAX_SLOTS, ws.gexp,
                       ws.gm7, S[0]);
  }
  const unsigned fbg = (unsigned)(2 * FB_PAIRS);
  float* const pset[2] = {ws.part, ws.part + (size_t)FB_PAIRS * WgradCfg<2>::PART};
  if (g_remat_ver >= 3) {
    remat3_layers(P, G, ws, FB, pimg, pscl, ci, n, grad, s, encimg, prow, psrow, S, S2, pset);
    return;
  }
  for (int L = 7; L >= 1; --L) {
    const float* coefp = ws.coef + 1024 * (L - 1);
    FbRed red{nullptr, nullptr, nullptr, nullptr, 0};
    if (L < 7)
      red = FbRed{pset[(L + 1) & 1], ws.coef + 1024 * L, ws.gacc + G.w[L + 1], ws.gacc + G.b[L + 1], L + 1 == 4 ? 2 : 1};
    const char* gin = L == 4 ? S2 : S[(7 - L) & 1];
    char* gout = L == 5 ? S2 : S[(8 - L) & 1];
    const unsigned* gmin = L == 7 ? ws.gm7 : ws.gmax + L * GMAX_SLOTS;
    // algorithmic work: data and weight gradient (2 x 2 x 256 x 256) + the input's rematerialisation (2 x 256 x 64);
    // bytes: g_L in (1 KiB), the encoding image (256 B), g_{L-1} out (1 KiB)
    ProfScope ps(s, PT_BWD_FUSED, (2.0 * 2.0 * 256.0 * 256.0 + 2.0 * 256.0 * 64.0) * dn, (1024.0 + 256.0 + 1024.0) * dn);
    auto launch = [&](auto kern) {
      hipLaunchKernelGGL(kern, dim3(fbg), dim3(512), RB_LDS, s, gin, gout, ws.wth16 + (size_t)(L - 1) * HW_H,
                         (const int*)ws.sw, L, n, coefp, (const float*)(ws.bnb + 512 * (L - 1)), P.bn_w[L - 1],
                         ws.gexp, (const float*)(ws.wcol + (L - 1) * 256), gmin, ws.gmax + (L - 1) * GMAX_SLOTS,
                         pset[L & 1], red, (const char*)encimg, prow(L - 1), psrow(L - 1));
    };
    if (L == 4) launch(k_bwd_remat2<2>);
    else launch(k_bwd_remat2<0>);
  }
  const int ne = (int)std::min<int64_t>(ntiles, FB_PAIRS);   // encoding-column partial sets (one per pair)
  float* const part_e0 = ws.part + 2 * (size_t)FB_PAIRS * WgradCfg<2>::PART;
  float* const part_e4 = part_e0 + (size_t)WG_BLOCKS * WgradCfg<1>::PART;
  {
    // 2 x 2 x 256 x 64 fp32-FLOP per sample; 2 KiB of g + 256 B of encoding in
    ProfScope ps(s, PT_BWD_WGRAD_H, 2.0 * 2.0 * 256.0 * 64 * dn, (2048.0 + 256.0) * dn);
    hipLaunchKernelGGL(k_wgrad_enc, dim3(2 * FB_PAIRS), dim3(512), WE_LDS, s, (const char*)S[1], (const char*)S2,
                       (const char*)encimg, n, (const int*)ws.gexp, (const unsigned*)ws.pbound, part_e0, part_e4);
  }
  // the partial sums read (k_fb_reduce_tail): layer 1's pair partials and the two encoding-column sets
  ProfScope ps(s, PT_BWD_MISC, 0.0, (double)FB_PAIRS * WgradCfg<0>::PART * 4.0 + 2.0 * ne * WgradCfg<1>::PART * 4.0);
  hipLaunchKernelGGL(k_fb_reduce_tail, dim3(256, 3), dim3(1024), 0, s, pset[1], (const float*)ws.coef,
                     ws.gacc + G.w[1], ws.gacc + G.b[1], part_e0, ws.gacc + G.w[0], ws.gacc + G.b[0], part_e4,
                     ws.gacc + G.w[4], FB_PAIRS, ne);
}

static void emit_grads(const GaccLayout& G, const BwdWs& ws, const pcnerf_nof_grads* grads, hipStream_t s) {
  GradTable T;
  int k = 0;
  for (int L = 0; L < 8; ++L) {
    T.dst[k] = grads->lin_w[L], T.off[k] = G.w[L], T.len[k++] = 256 * in_features(L);
    T.dst[k] = grads->lin_b[L], T.off[k] = G.b[L], T.len[k++] = 256;
    T.dst[k] = grads->bn_w[L], T.off[k] = G.g[L], T.len[k++] = 256;
    T.dst[k] = grads->bn_b[L], T.off[k] = G.be[L], T.len[k++] = 256;
  }
  T.dst[k] = grads->out_w, T.off[k] = G.wo, T.len[k++] = 256;
  T.dst[k] = grads->out_b, T.off[k] = G.bo, T.len[k++] = 1;
  hipLaunchKernelGGL(k_grad_emit, dim3((256 * 319 + 255) / 256, 34), dim3(256), 0, s, T, ws.gacc);
}

// The default training backward (train math f16x2_3 with the fused forward): every chunk through remat_chunk, on
// the state the forward kept (pcnerf_nof_query_train_fused_state) -- no activation store, no recomputed forward, no
// host synchronisation.
static void backward_remat(const float* rays, int ray_stride, const float* z, int n_samples, int64_t total,
                           int64_t chunk, const pcnerf_nof_params* params, float eps, const float* grad,
                           void* workspace, size_t workspace_bytes, const pcnerf_nof_grads* grads, hipStream_t s,
                           void* fstate, size_t fstate_bytes) {
  PCN_CHECK(g_train_math == 1, "pcnerf_nof_query_train_backward_remat: needs train math 1 (f16x2_3)");
  const BwdWs ws = carve_bwd(workspace, chunk);
  PCN_CHECK(workspace_bytes >= ws.bytes, "pcnerf_nof_query_train_backward_remat: workspace too small");
  NofParamsDev P;
  PCN_CHECK(to_dev_params(params, eps, &P), "pcnerf_nof_query_train_backward_remat: null parameter pointer");
  PCN_CHECK(total % chunk != 1 && total != 1, "Expected more than 1 value per channel when training");
  const GaccLayout G = gacc_layout();
  pos_bound_async(rays, ray_stride, z, n_samples, nullptr, total, ws.pbound, s);
  hipLaunchKernelGGL(k_wscale, dim3(8), dim3(1024), 0, s, P, ws.sw);
  hipLaunchKernelGGL(k_pack_dgrad_h16, dim3((unsigned)((7 * HW_H + 255) / 256)), dim3(256), 0, s, P, ws.sw,
                     ws.wth16);
  hipLaunchKernelGGL(k_wcol, dim3(7), dim3(256), 0, s, P, ws.wcol);
  PCN_HIP(hipMemsetAsync(ws.gacc, 0, (size_t)G.total * 8, s));
  PCN_HIP(hipMemsetAsync(ws.ostat, 0, sizeof(unsigned), s));   // k_out_gabs's word (k_fb_prep re-zeroes it)
  const FoldBnBwd FB = fold_bn_backward(rays, ray_stride, z, n_samples, total, chunk, P, grad, fstate, fstate_bytes, s);
  // every chunk's P' images at once, into the Sigma products' space (free now)
  f16x8* const pimg = static_cast<f16x8*>(FB.scratch);
  float* const pscl = reinterpret_cast<float*>(pimg + (size_t)8 * FB.C * 256 * 16);
  hipLaunchKernelGGL(k_remat_pimg, dim3(8, (unsigned)FB.C), dim3(256), 0, s, FB, ws.pbound, pimg, pscl);
  for (int64_t c0 = 0; c0 < total; c0 += chunk) {
    const int64_t n = total - c0 < chunk ? total - c0 : chunk;
    remat_chunk(P, G, ws, FB, pimg, pscl, c0 / chunk, c0, n, rays, ray_stride, z, n_samples, eps, grad, s);
  }
  emit_grads(G, ws, grads, s);
  PCN_LAUNCH_CHECK("pcnerf_nof_query_train_backward_remat");
}

static void backward_train(const float* rays, int ray_stride, const float* z, int n_samples, const float* ein,
                           int64_t total, int64_t chunk, const pcnerf_nof_params* params, float eps,
                           const float* grad, const float* p, void* workspace, size_t workspace_bytes,
                           const pcnerf_nof_grads* grads, hipStream_t s, const void* store = nullptr,
                           int64_t store_chunks = 0, void* fstate = nullptr, size_t fstate_bytes = 0) {
  const BwdWs ws = carve_bwd(workspace, chunk);
  PCN_CHECK(workspace_bytes >= ws.bytes, "pcnerf_nof_backward: workspace too small");
  NofParamsDev P;
  PCN_CHECK(to_dev_params(params, eps, &P), "pcnerf_nof_backward: null parameter pointer");
  PCN_CHECK(total % chunk != 1 && total != 1, "Expected more than 1 value per channel when training");
  const GaccLayout G = gacc_layout();
  const int64_t n_chunks = (total + chunk - 1) / chunk;
  // the one-pass backward (k_bwd_fused) on the chunks the fused forward stored, under the split math of the fused
  // forward (f16x2, 3 products); every other chunk (recomputed) and every other math: the two-pass backward
  const bool fused = fstate && store && g_train_math == 1;
  bool fused_zeroed = false;
  const bool recompute = !store || store_chunks < n_chunks || !fused;
  // the encoding operand's xyz columns are scaled by the largest |position| (device-side, k_pos_bound); the
  // layered forward that recomputes chunks splits them unscaled and needs the host-side range check
  if (recompute) check_split_range(rays, ray_stride, z, n_samples, ein, total, ws.pbound, s, "pcnerf_nof_backward");
  else pos_bound_async(rays, ray_stride, z, n_samples, ein, total, ws.pbound, s);
  hipLaunchKernelGGL(k_pack_train, dim3((unsigned)((TRAIN_W_FLOATS + 255) / 256)), dim3(256), 0, s, P, ws.wp);
  const bool split = g_train_math != 0;
  if (split) {   // the forward's arithmetic for recomputation, and k_dgrad_h's W^T image
    pack_weights(P, nullptr, ws.wh, ws.sw, s);
    hipLaunchKernelGGL(k_pack_dgrad_h, dim3((unsigned)((7 * HW_H + 255) / 256)), dim3(256), 0, s, P, ws.sw, ws.wth);
  }
  hipLaunchKernelGGL(k_pack_dgrad, dim3((unsigned)((DGRAD_W_FLOATS + 255) / 256)), dim3(256), 0, s, P, ws.wt);
  PCN_HIP(hipMemsetAsync(ws.gacc, 0, (size_t)G.total * 8, s));
  FoldBnBwd FB{};
  if (fused) {
    hipLaunchKernelGGL(k_pack_dgrad_h16, dim3((unsigned)((7 * HW_H + 255) / 256)), dim3(256), 0, s, P, ws.sw,
                       ws.wth16);
    FB = fold_bn_backward(rays, ray_stride, z, n_samples, total, chunk, P, grad, fstate, fstate_bytes, s);
  }
  const float mom = 0.0f;  // unused: the recomputation passes no running stats
  for (int64_t c0 = 0; c0 < total; c0 += chunk) {
    const int64_t n = total - c0 < chunk ? total - c0 : chunk;
    const int64_t ntiles = (n + 31) / 32;
    const double dn = (double)n;
    const unsigned gws = (unsigned)(ntiles < 256 ? ntiles : 256);   // k_train_ws / k_dgrad_ws
    const unsigned eg = (unsigned)((ntiles + 3) / 4 < 1024 ? (ntiles + 3) / 4 : 1024);
    const unsigned wblocks = (unsigned)(ntiles < WG_BLOCKS ? ntiles : WG_BLOCKS);
    // 1. the forward's layer outputs and statistics: from the activation store, or recomputed here
    const int64_t ci = c0 / chunk;
    const bool kept = store && ci < store_chunks;
    const StoreChunk sc = kept ? store_chunk(store, chunk, ci) : StoreChunk{};
    float* hh[8];
    for (int L = 0; L < 8; ++L) hh[L] = kept ? sc.h[L] : ws.h[L];
    const double* stats = kept ? sc.stats : ws.stats;
    if (kept && fused) {
      if (!fused_zeroed) {   // k_out_gabs's word (k_fb_prep re-zeroes it after every chunk)
        PCN_HIP(hipMemsetAsync(ws.ostat, 0, sizeof(unsigned), s));
        fused_zeroed = true;
      }
      fused_chunk(P, G, ws, FB, ci, c0, n, stats, hh, rays, ray_stride, z, n_samples, ein, eps, grad, s);
      continue;
    }
    if (!kept) PCN_HIP(hipMemsetAsync(ws.stats, 0, 8 * 512 * sizeof(double), s));
    const f32x4* enc_of_chunk = nullptr;   // written by this chunk's recomputed first layer, read by its skip layer
    if (!kept) {
      const BnPrev none{};
      ProfScope ps(s, PT_TRAIN_FIRST, 2.0 * 63 * 256 * dn, (4.0 + 1024.0) * dn);
      const TrainLayerLaunch q{rays, ray_stride, z, n_samples, c0, ein, n, gws, mom, eps, s};
      launch_layer<KG_E, false>(q, P, ws.wp, ws.wh, ws.sw, 0, nullptr, none, ws.h[0], ws.stats, nullptr, ws.enc);
      enc_of_chunk = ws.enc;
    }
    for (int L = 1; L < 8 && !kept; ++L) {
      const BnPrev prev{P.bn_w[L - 1], P.bn_b[L - 1], nullptr, nullptr, P.lin_b[L - 1], ws.stats + 512 * (L - 1)};
      if (L == 4) {
        PCN_CHECK(enc_of_chunk, "skip layer launched without this chunk's first-layer encoding tiles");
        ProfScope ps(s, PT_TRAIN_SKIP, 2.0 * 319 * 256 * dn, (4.0 + 2048.0) * dn);
        const TrainLayerLaunch q{rays, ray_stride, z, n_samples, c0, ein, n, gws, mom, eps, s};
        launch_layer<KG_E, true>(q, P, ws.wp, ws.wh, ws.sw, 4, ws.h[3], prev, ws.h[4], ws.stats + 512 * 4,
                                 enc_of_chunk, nullptr);
      } else {
        ProfScope ps(s, PT_TRAIN_HIDDEN, 2.0 * 256 * 256 * dn, 2048.0 * dn);
        const TrainLayerLaunch q{rays, ray_stride, z, n_samples, c0, ein, n, gws, mom, eps, s};
        launch_layer<0, true>(q, P, ws.wp, ws.wh, ws.sw, L, ws.h[L - 1], prev, ws.h[L], ws.stats + 512 * L, nullptr,
                              nullptr);
      }
    }
    {
      ProfScope ps(s, PT_BWD_MISC, 0.0, 2.0 * 1024.0 * dn);
      hipLaunchKernelGGL(k_bn_save, dim3(8), dim3(256), 0, s, P, stats, n, eps, ws.coef);
      // 2. occ_out + BatchNorm 8
      PCN_HIP(hipMemsetAsync(ws.s12, 0, (8 * S12_LAYER + OSTAT_COPIES * 257 + GMAX_DBL) * sizeof(double), s));  // per chunk
      {
        const unsigned sg = (unsigned)((ntiles + 3) / 4 < 256 ? (ntiles + 3) / 4 : 256);
        hipLaunchKernelGGL(k_out_bwd_stats1, dim3(sg), dim3(256), 0, s, grad + c0, p ? p + c0 : nullptr, hh[7], n,
                           ws.coef + 7 * 1024, ws.ostat);
      }
      hipLaunchKernelGGL(k_out_bwd_grad, dim3(eg), dim3(256), 0, s, grad + c0, p ? p + c0 : nullptr, hh[7], n,
                         ws.coef + 7 * 1024, P.bn_w[7], P.out_w, ws.ostat, ws.gacc + G.g[7], ws.gacc + G.be[7],
                         ws.gacc + G.wo, ws.gacc + G.bo, ws.g[0], split ? ws.tmax[0] : nullptr,
                         split ? ws.gmax + 7 * GMAX_SLOTS : nullptr, OSTAT_COPIES);
    }
    // the chunk's encoding mean (fp32 MFMA math: k_wgrad's centring of the encoding columns of layers 0 and 4)
    const double* emean = nullptr;
    if (!split) {
      PCN_HIP(hipMemsetAsync(ws.gd, 0, 64 * sizeof(double), s));
      hipLaunchKernelGGL(k_enc_mean, dim3((unsigned)std::min<int64_t>((n + 255) / 256, 256)), dim3(256), 0, s, rays,
                         ray_stride, z, n_samples, c0, n, ein, ws.gd);
      emean = ws.gd;
    }
    // 3. layers 7..1
    int cur = 0;
    for (int L = 7; L >= 1; --L) {
      const float* coefp = ws.coef + 1024 * (L - 1);
      {
        ProfScope ps(s, split ? PT_BWD_WGRAD_H : PT_BWD_WGRAD, 2.0 * 256.0 * (L == 4 ? 320 : 256) * dn,
                     2048.0 * dn);
        if (split && L == 4)
          launch_wgrad_b3<2>(wblocks, s, rays, ray_stride, z, n_samples, c0, n, ein, ws.g[cur], hh[3], coefp,
                             ws.gmax + L * GMAX_SLOTS, ws.part, ws.pbound);
        else if (split)
          launch_wgrad_b3<0>(wblocks, s, rays, ray_stride, z, n_samples, c0, n, ein, ws.g[cur], hh[L - 1], coefp,
                             ws.gmax + L * GMAX_SLOTS, ws.part, ws.pbound);
        else if (L == 4)
          launch_wgrad<2>(wblocks, s, rays, ray_stride, z, n_samples, c0, n, ein, ws.g[cur], hh[3], coefp, ws.part,
                          emean);
        else
          launch_wgrad<0>(wblocks, s, rays, ray_stride, z, n_samples, c0, n, ein, ws.g[cur], hh[L - 1], coefp,
                          ws.part);
      }
      {
        ProfScope ps(s, PT_BWD_MISC, 0.0, (double)wblocks * WgradCfg<0>::PART * 4.0);
        if (L == 4)
          hipLaunchKernelGGL(k_wgrad_reduce<2>, dim3(256), dim3(WgradCfg<2>::RT), 0, s, ws.part, (int)wblocks,
                             P.lin_w[4], coefp, ws.gacc + G.w[4], ws.gacc + G.b[4], ws.s12 + S12_LAYER * L, (int)wblocks);
        else
          hipLaunchKernelGGL(k_wgrad_reduce<0>, dim3(256), dim3(WgradCfg<0>::RT), 0, s, ws.part, (int)wblocks,
                             P.lin_w[L], coefp, ws.gacc + G.w[L], ws.gacc + G.b[L], ws.s12 + S12_LAYER * L, (int)wblocks);
      }
      {
        ProfScope ps(s, PT_BWD_DGRAD, 2.0 * 256 * 256 * dn, 3072.0 * dn);
        if (split && g_train_math == 1)
          hipLaunchKernelGGL(k_dgrad_h<3>, dim3(gws), dim3(512), 0, s, ws.g[cur], ws.tmax[cur],
                             ws.wth + (size_t)(L - 1) * HW_H, ws.sw, L, hh[L - 1], n, ws.s12 + S12_LAYER * L, coefp,
                             P.bn_w[L - 1], ws.gacc + G.g[L - 1], ws.gacc + G.be[L - 1], ws.g[cur ^ 1],
                             ws.tmax[cur ^ 1], ws.gmax + (L - 1) * GMAX_SLOTS);
        else if (split)
          hipLaunchKernelGGL(k_dgrad_h<4>, dim3(gws), dim3(512), 0, s, ws.g[cur], ws.tmax[cur],
                             ws.wth + (size_t)(L - 1) * HW_H, ws.sw, L, hh[L - 1], n, ws.s12 + S12_LAYER * L, coefp,
                             P.bn_w[L - 1], ws.gacc + G.g[L - 1], ws.gacc + G.be[L - 1], ws.g[cur ^ 1],
                             ws.tmax[cur ^ 1], ws.gmax + (L - 1) * GMAX_SLOTS);
        else
          hipLaunchKernelGGL(k_dgrad_ws, dim3(gws), dim3(512), 0, s, ws.g[cur], ws.wt + (size_t)(L - 1) * SZ_H,
                             hh[L - 1], n, ws.s12 + S12_LAYER * L, coefp, P.bn_w[L - 1], ws.gacc + G.g[L - 1],
                             ws.gacc + G.be[L - 1], ws.g[cur ^ 1]);
      }
      cur ^= 1;
    }
    // 4. layer 0 on the encoding.  Under the split math at TWO workgroups per CU: the
    // encoding-column launch is latency-bound on its sincosf staging at one 8-wave workgroup per CU, and its
    // 127 VGPRs and 66 KiB of LDS let a second one share the CU (its partials: 2 x WG_BLOCKS slots of k_wgrad<1>'s
    // layout, within the buffer sized for WG_BLOCKS of k_wgrad<2>'s)
    static_assert(2 * WG_BLOCKS * WgradCfg<1>::PART <= WG_BLOCKS * WgradCfg<2>::PART, "layer-0 partial slots");
    const unsigned wb0 = split ? (unsigned)std::min<int64_t>(2 * ntiles, 2 * WG_BLOCKS) : wblocks;
    {
      ProfScope ps(s, split ? PT_BWD_WGRAD_H : PT_BWD_WGRAD, 2.0 * 256.0 * 64 * dn, 1024.0 * dn);
      if (split)
        launch_wgrad_b3<1>(wb0, s, rays, ray_stride, z, n_samples, c0, n, ein, ws.g[cur], nullptr, nullptr,
                           ws.gmax + 0 * GMAX_SLOTS, ws.part, ws.pbound);
      else
        launch_wgrad<1>(wblocks, s, rays, ray_stride, z, n_samples, c0, n, ein, ws.g[cur], nullptr, nullptr,
                        ws.part, emean);
    }
    {
      ProfScope ps(s, PT_BWD_MISC, 0.0, (double)wb0 * WgradCfg<1>::PART * 4.0);
      hipLaunchKernelGGL(k_wgrad_reduce<1>, dim3(256), dim3(WgradCfg<1>::RT), 0, s, ws.part, (int)wb0,
                         P.lin_w[0], (const float*)nullptr, ws.gacc + G.w[0], ws.gacc + G.b[0], (double*)nullptr, (int)wb0);
    }
  }
  emit_grads(G, ws, grads, s);
  PCN_LAUNCH_CHECK("pcnerf_nof_backward");
}

extern "C" int pcnerf_nof_query_train_backward_store(const float* rays, int64_t n_rays, int ray_stride,
                                                     const float* z, int n_samples, int64_t chunk,
                                                     const pcnerf_nof_params* params, float eps,
                                                     const float* grad_logit, void* workspace,
                                                     size_t workspace_bytes, const pcnerf_nof_grads* grads,
                                                     const void* store, int64_t store_chunks, void* stream) {
  PCN_API_BEGIN
  PCN_CHECK(rays && z && params && grad_logit && workspace && grads,
            "pcnerf_nof_query_train_backward_store: null argument");
  PCN_CHECK(n_rays > 0 && n_samples > 0 && chunk > 0, "pcnerf_nof_query_train_backward_store: empty input");
  PCN_CHECK(ray_stride >= 6, "pcnerf_nof_query_train_backward_store: ray_stride < 6");
  PCN_CHECK(store_chunks == 0 || store, "pcnerf_nof_query_train_backward_store: store_chunks > 0 needs a store");
  backward_train(rays, ray_stride, z, n_samples, nullptr, n_rays * (int64_t)n_samples, chunk, params, eps,
                 grad_logit, nullptr, workspace, workspace_bytes, grads, (hipStream_t)stream, store, store_chunks);
  PCN_API_END
}

extern "C" int pcnerf_nof_query_train_backward_fused(const float* rays, int64_t n_rays, int ray_stride,
                                                     const float* z, int n_samples, int64_t chunk,
                                                     const pcnerf_nof_params* params, float eps,
                                                     const float* grad_logit, void* state, size_t state_bytes,
                                                     void* workspace, size_t workspace_bytes,
                                                     const pcnerf_nof_grads* grads, void* store,
                                                     int64_t store_chunks, void* stream) {
  PCN_API_BEGIN
  PCN_CHECK(rays && z && params && grad_logit && state && workspace && grads,
            "pcnerf_nof_query_train_backward_fused: null argument");
  PCN_CHECK(n_rays > 0 && n_samples > 0 && chunk > 0, "pcnerf_nof_query_train_backward_fused: empty input");
  PCN_CHECK(ray_stride >= 6, "pcnerf_nof_query_train_backward_fused: ray_stride < 6");
  PCN_CHECK(store_chunks == 0 || store, "pcnerf_nof_query_train_backward_fused: store_chunks > 0 needs a store");
  backward_train(rays, ray_stride, z, n_samples, nullptr, n_rays * (int64_t)n_samples, chunk, params, eps,
                 grad_logit, nullptr, workspace, workspace_bytes, grads, (hipStream_t)stream, store, store_chunks,
                 state, state_bytes);
  PCN_API_END
}

extern "C" int pcnerf_nof_query_train_backward_remat(const float* rays, int64_t n_rays, int ray_stride,
                                                     const float* z, int n_samples, int64_t chunk,
                                                     const pcnerf_nof_params* params, float eps,
                                                     const float* grad_logit, void* state, size_t state_bytes,
                                                     void* workspace, size_t workspace_bytes,
                                                     const pcnerf_nof_grads* grads, void* stream) {
  PCN_API_BEGIN
  PCN_CHECK(rays && z && params && grad_logit && state && workspace && grads,
            "pcnerf_nof_query_train_backward_remat: null argument");
  PCN_CHECK(n_rays > 0 && n_samples > 0 && chunk > 0, "pcnerf_nof_query_train_backward_remat: empty input");
  PCN_CHECK(ray_stride >= 6, "pcnerf_nof_query_train_backward_remat: ray_stride < 6");
  const int64_t total = n_rays * (int64_t)n_samples;
  backward_remat(rays, ray_stride, z, n_samples, total, std::min(chunk, total), params, eps, grad_logit, workspace,
                 workspace_bytes, grads, (hipStream_t)stream, state, state_bytes);
  PCN_API_END
}

extern "C" int pcnerf_nof_query_train_backward(const float* rays, int64_t n_rays, int ray_stride, const float* z,
                                               int n_samples, int64_t chunk, const pcnerf_nof_params* params,
                                               float eps, const float* grad_logit, void* workspace,
                                               size_t workspace_bytes, const pcnerf_nof_grads* grads, void* stream) {
  PCN_API_BEGIN
  PCN_CHECK(rays && z && params && grad_logit && workspace && grads, "pcnerf_nof_query_train_backward: null argument");
  PCN_CHECK(n_rays > 0 && n_samples > 0 && chunk > 0, "pcnerf_nof_query_train_backward: empty input");
  PCN_CHECK(ray_stride >= 6, "pcnerf_nof_query_train_backward: ray_stride < 6");
  backward_train(rays, ray_stride, z, n_samples, nullptr, n_rays * (int64_t)n_samples, chunk, params, eps,
                 grad_logit, nullptr, workspace, workspace_bytes, grads, (hipStream_t)stream);
  PCN_API_END
}

extern "C" int pcnerf_nof_forward_train_backward(const float* emb, int64_t n, const pcnerf_nof_params* params,
                                                 float eps, const float* p, const float* grad_p, void* workspace,
                                                 size_t workspace_bytes, const pcnerf_nof_grads* grads,
                                                 void* stream) {
  PCN_API_BEGIN
  PCN_CHECK(emb && params && p && grad_p && workspace && grads, "pcnerf_nof_forward_train_backward: null argument");
  PCN_CHECK(n > 0, "pcnerf_nof_forward_train_backward: empty input");
  backward_train(nullptr, 0, nullptr, 1, emb, n, n, params, eps, grad_p, p, workspace, workspace_bytes, grads,
                 (hipStream_t)stream);
  PCN_API_END
}
