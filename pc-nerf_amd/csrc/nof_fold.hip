// Opt-in exact affine fold of the TRAIN-mode network, forward and backward (SURVEY fact 1, §7 "alternative exact
// route").  Never the default: the drop-in evaluates the module as written (nof_train.hip).
//
// Every LeakyReLU(True) of NOF is the identity (negative_slope = 1, models.py:72,152,232), so within one BatchNorm
// chunk (render.py:47-50) every layer output is an affine map of the sample's encoding e (models.py:27-41):
//   x_L = P_L (e - ebar) + beta_L,   P_L = s_L (.) P'_L,   P'_L = W_L P_{L-1}   (skip layer: W_e + W_h P_3)
// and BatchNorm's batch statistics follow exactly from the chunk's encoding mean ebar and covariance Sigma:
//   mean(h_L) = W_L mean(x_{L-1}) + b_L,  var(h_L)_i = p'_i^T Sigma p'_i,  s_L = gamma / sqrt(var + eps)
// (models.py:183-203; nn.BatchNorm1d train: biased variance for the normalisation, unbiased for running_var).
// The chunk's network is then sigmoid(a_c . e + c_c) with a_c = w_out P_7, c_c = w_out . beta_7 + b_out - a_c . ebar.
// Rounding differs from the layer-by-layer fp32 network (the algebra runs in float64), so the path is opt-in and
// reported as its own bench line.
//
// Forward per query (all chunks of one render pass batched into each launch):
//   k_tf_moments   per chunk: sum over samples of d d^T, d = [e - e0, 1] (e0 = the chunk's first encoding,
//                  a shift against cancellation), fp16 hi/mid parts on the matrix pipe per 64-sample tile (three
//                  exact products, fp32 accumulation), float64 across tiles
//   k_tf_stats     ebar, Sigma per chunk (float64)
//   k_tf_layer16<L> P'_L, Q_L = P'_L Sigma, var, s, the pre-BN mean (float64 GEMMs on v_mfma_f64_16x16x4_f64,
//                  16-row tiles x chunks)
//   k_tf_out       (a_c, c_c);  launch_fold_logits: p = sigmoid(a_c . e + c_c) per sample
//   k_tf_running   running_mean / running_var, chunk by chunk in order (bn_coeffs' arithmetic)
// Backward (dL/dlogit per sample):
//   k_tf_gmoments  per chunk: abar = sum_s g_s (e_s - ebar), gbar = sum_s g_s
//   k_tf_bwd_out   occ_out / beta_7 gradients, adjoint of P_7 -> through BatchNorm 7 to the adjoint A'_7 of P'_7
//   per layer L = 7..0: k_tf_dw<L> (dW_L = sum_c A'_L P_{L-1}^T, chunk-group partials), k_tf_dw_reduce<L>,
//                  k_tf_bwd_layer16<L> (A_{L-1} = W_L^T A'_L, then BatchNorm L-1's backward:
//                  ds = A.p', dgamma += ds / sqrt(var+eps), dvar = -ds gamma / (2 (var+eps)^1.5),
//                  A'_{L-1} = s A + 2 dvar Q_{L-1})
//   k_tf_vec_reduce gamma / out gradients summed over chunks.
// The Linear biases and the shifts of every BatchNorm that feeds Linear->BatchNorm get exactly zero gradient (the
// next BatchNorm removes the mean); the reference's autograd gives rounding noise there.
#include <algorithm>

#include "common.h"
#include "pcnerf_internal.h"
#include "prof.h"

namespace pcn {

constexpr int TF_WPC_MIN = 16;   // moment workgroups per chunk: at least this many (when the chunk has the tiles),
constexpr int TF_WPC_MAX = 256;  //   enough for ~512 workgroups over all chunks when there are few, at most this
constexpr int TF_G_MAX = 16;     // chunk groups of the weight-gradient partials

struct FoldDev {   // device views of the fold state (float64 throughout)
  int64_t C;       // BatchNorm chunks of the query
  int wpc, G;
  double* mom;     // [C][wpc][64][64] moment partials (blocks 00, 01, 11 of d d^T)
  double* sig;     // [C][64][64] Sigma (row / column 63 zero)
  double* eb;      // [C][64] ebar (63 used)
  double* e0;      // [C][64] the chunk's shift
  double* pp;      // [8][C][256][64] P'_L (column 63: W_L mean(x_{L-1}))
  double* q;       // [8][C][256][64] P'_L Sigma
  double* sr;      // [8][C][4][256] s, 1/sqrt(var+eps), mean(h_L), var(h_L)
  double* fold;    // [C][64] (a_c, c_c)
  double* gm;      // [C][wpc][64] backward moment partials
  double* ab;      // [2][C][256][64] forward: P_L = s_L (.) P'_L | beta_L ping-pong; backward: A'_L ping-pong
  double* dg;      // [8][C][256] dgamma per chunk
  double* dw;      // [G][256][256] weight-gradient partials (h columns)
  double* vec;     // [C][576] d out_w (256), d beta_7 (256), d out_b (1)
  float* coef;     // [C][TQ_COEF_FLOATS] the chunks' BatchNorm coefficients and operand scales (train-mode query)
  float* img;      // the train-mode query's weight image (train_query_image_floats)
  double* oacc;    // [C][257] sum_s g_s (h_7 - mean_7) and sum_s g_s (the per-sample backward's occ_out statistics)
};

constexpr int FOLD_PIECES = 16;
struct FoldLayout {
  int64_t C;
  int wpc, G;
  size_t off[FOLD_PIECES];
  size_t doubles;
};

// fwd_only: the fused train query's state (pcnerf_nof_train_fused_bytes) -- the backward-only pieces (gm, dg, dw, vec:
// about 2.2 MB per chunk) and the fold's logits are empty, so its size does not grow with them; ab is kept (the
// forward's P_L ping-pong, k_tf_layer16)
static FoldLayout fold_layout(int64_t total, int64_t chunk, bool fwd_only = false) {
  FoldLayout F{};
  F.C = (total + chunk - 1) / chunk;
  const int64_t tiles = (std::min(chunk, total) + 63) / 64;
  // a few large chunks (the reference's shell setting: 1 coarse and 3 fine chunks) would leave most CUs idle at
  // 16 workgroups per chunk: ~512 workgroups in all, each at least 4 tiles of 64 samples (one per wave)
  const int64_t want = std::max<int64_t>(TF_WPC_MIN, (512 + F.C - 1) / F.C);
  F.wpc = (int)std::max<int64_t>(1, std::min<int64_t>(std::min<int64_t>(want, TF_WPC_MAX), tiles / 4));
  F.G = (int)std::min<int64_t>(F.C, TF_G_MAX);
  const size_t C = (size_t)F.C, wpc = (size_t)F.wpc, G = (size_t)F.G;
  const size_t b = fwd_only ? 0 : 1;
  const size_t n[FOLD_PIECES] = {C * wpc * 4096, C * 4096, C * 64, C * 64, 8 * C * 256 * 64, 8 * C * 256 * 64,
                                 8 * C * 1024, b * C * 64, b * C * wpc * 64, 2 * C * 256 * 64, b * 8 * C * 256,
                                 b * G * 256 * 256, b * C * 576, C * TQ_COEF_FLOATS / 2,
                                 (train_query_image_floats() + 1) / 2, b * C * 257};
  size_t o = 0;
  for (int i = 0; i < FOLD_PIECES; ++i) {
    F.off[i] = o;
    o += (n[i] + 31) & ~(size_t)31;   // 256-byte aligned pieces
  }
  F.doubles = o;
  return F;
}

static FoldDev fold_dev(const FoldLayout& L, void* state) {
  double* b = (double*)state;
  FoldDev F;
  F.C = L.C;
  F.wpc = L.wpc;
  F.G = L.G;
  double** dst[13] = {&F.mom, &F.sig, &F.eb, &F.e0, &F.pp, &F.q, &F.sr, &F.fold, &F.gm, &F.ab, &F.dg, &F.dw, &F.vec};
  for (int i = 0; i < 13; ++i) *dst[i] = b + L.off[i];
  F.coef = (float*)(b + L.off[13]);
  F.img = (float*)(b + L.off[14]);
  F.oacc = b + L.off[15];
  return F;
}

struct SampleSrc {   // the query's flattened ray-major samples (rays + z) or an embedded batch (ein)
  const float* rays;
  int stride;
  const float* z;
  int S;
  const float* ein;
  int64_t total, chunk;
};

__device__ __forceinline__ void sample_enc(const SampleSrc& q, int64_t g, float (&f)[64]) {
  if (q.ein) {
    const float* r = q.ein + g * 63;
#pragma unroll
    for (int k = 0; k < 63; ++k) f[k] = r[k];
    f[63] = 0.0f;
  } else {
    float p[3];
    sample_point(q.rays + ray_of(g, q.S) * q.stride, q.z[g], p);
    encode_full(p, f);
  }
}

__device__ __forceinline__ int64_t chunk_len(const SampleSrc& q, int64_t c) {
  const int64_t r = q.total - c * q.chunk;
  return r < q.chunk ? r : q.chunk;
}

// ------------------------------------------------------------------------------------------------- forward
// grid (wpc, C), 256 threads.  Each wave stages 64 samples' d = [e - e0, 1] (zero past the chunk) as two fp16
// parts (hi = fp16(d), mid = fp16(d - hi): 22 significant bits) in a [feature][sample] LDS tile, and accumulates
// d d^T (blocks 00, 01, 11 of 64 x 64) on v_mfma_f32_32x32x16_f16 as hi.hi + hi.mid + mid.hi (exact products,
// fp32 accumulation over the 64-sample tile, float64 across tiles).  The tile rows are 72 halves apart, so the
// operand reads (16 bytes: 8 samples of one feature) of 16 lanes hit 16 disjoint bank groups.
typedef _Float16 tf_f16x8 __attribute__((ext_vector_type(8)));

// orders one wave's LDS writes before its reads of the same tile (and the reads before the next tile's writes):
// the tiles are wave-private, so no workgroup barrier is needed and the four waves run out of phase
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
constexpr int TM_P = 72;

__global__ __launch_bounds__(256) void k_tf_moments(SampleSrc q, FoldDev F) {
  __shared__ __attribute__((aligned(16))) _Float16 th[4][2][64 * TM_P];
  __shared__ float sh0[64];
  const int c = blockIdx.y, w = blockIdx.x, tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int64_t c0 = (int64_t)c * q.chunk, n = chunk_len(q, c);
  if (tid == 0) {
    float f[64];
    sample_enc(q, c0, f);
#pragma unroll
    for (int k = 0; k < 63; ++k) sh0[k] = f[k];
    sh0[63] = 0.0f;
  }
  __syncthreads();
  if (w == 0 && tid < 64) F.e0[(int64_t)c * 64 + tid] = (double)sh0[tid];
  const int64_t ntile = (n + 63) / 64, per = (ntile + F.wpc - 1) / F.wpc;
  const int64_t t0 = std::min(ntile, (int64_t)w * per), t1 = std::min(ntile, t0 + per);
  f32x16 a00 = {}, a01 = {}, a11 = {};
  double d00[16], d01[16], d11[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) d00[r] = d01[r] = d11[r] = 0.0;
  _Float16* hi = th[wave][0];
  _Float16* mi = th[wave][1];
  for (int64_t t = t0 + wave; t < t1; t += 4) {   // waves independent: wave-local LDS tiles
    const int64_t i = t * 64 + lane;
    const bool ok = i < n;
    // fp16 range (k_enc_gram's guard): a tile whose largest |d| reaches 2^15 (positions spread over more than
    // 32 km; the sin/cos features differ by at most 2) is split at 2^-sk, the count column included, and its
    // products rescaled by 2^(2 sk) in float64 -- exact powers of two, sk = 0 for every realistic scene
    const float* r = q.ein ? q.ein + (c0 + (ok ? i : 0)) * 63 : nullptr;
    float p[3] = {0.0f, 0.0f, 0.0f};
    float dm = 0.0f;
    if (q.ein) {
      if (ok)
        for (int f = 0; f < 63; ++f) dm = fmaxf(dm, fabsf(r[f] - sh0[f]));
    } else if (ok) {
      sample_point(q.rays + ray_of(c0 + i, q.S) * q.stride, q.z[c0 + i], p);
#pragma unroll
      for (int m = 0; m < 3; ++m) dm = fmaxf(dm, fabsf(p[m] - sh0[m]));
    }
    dm = wave_max_f(dm);
    int sk = (dm >= 32768.0f && dm < 3.0e38f) ? ilogbf(dm) - 14 : 0;
    sk = sk > 24 ? 24 : sk;
    const float dsc = ldexpf(1.0f, -sk);
    auto put = [&](int f, float v) {
      const float d = ok ? (v - sh0[f]) * dsc : 0.0f;
      const _Float16 h = (_Float16)d;
      hi[f * TM_P + lane] = h;
      mi[f * TM_P + lane] = (_Float16)(d - (float)h);
    };
    if (q.ein) {
#pragma unroll 7
      for (int f = 0; f < 63; ++f) put(f, r[f]);
    } else {
#pragma unroll
      for (int m = 0; m < 3; ++m) put(m, p[m]);
#pragma unroll 2
      for (int k = 0; k < 10; ++k) {
        const float sc = (float)(1 << k);
#pragma unroll
        for (int m = 0; m < 3; ++m) {
          float sv, cv;
          sincosf(sc * p[m], &sv, &cv);
          put(3 + 6 * k + m, sv);
          put(6 + 6 * k + m, cv);
        }
      }
    }
    hi[63 * TM_P + lane] = ok ? (_Float16)dsc : (_Float16)0.0f;
    mi[63 * TM_P + lane] = (_Float16)0.0f;
    wave_lds_sync();
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const int o = (lane & 31) * TM_P + 16 * ks + 8 * (lane >> 5);
      const tf_f16x8 h0 = *reinterpret_cast<const tf_f16x8*>(hi + o);
      const tf_f16x8 m0 = *reinterpret_cast<const tf_f16x8*>(mi + o);
      const tf_f16x8 h1 = *reinterpret_cast<const tf_f16x8*>(hi + 32 * TM_P + o);
      const tf_f16x8 m1 = *reinterpret_cast<const tf_f16x8*>(mi + 32 * TM_P + o);
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
    const double usc = ldexp(1.0, 2 * sk);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      d00[r] += (double)a00[r] * usc;
      d01[r] += (double)a01[r] * usc;
      d11[r] += (double)a11[r] * usc;
      a00[r] = a01[r] = a11[r] = 0.0f;
    }
    wave_lds_sync();
  }
  // the four waves' blocks summed in a fixed order through LDS (aliasing the tiles, once every wave is done with
  // its own), then one coalesced store
  __syncthreads();
  double* red = reinterpret_cast<double*>(&th[0][0][0]);
  for (int wv = 0; wv < 4; ++wv) {
    if (wave == wv) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int i = (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5), j = lane & 31;
        if (wv == 0) {
          red[i * 64 + j] = d00[r];
          red[i * 64 + 32 + j] = d01[r];
          red[(32 + i) * 64 + 32 + j] = d11[r];
          red[(32 + i) * 64 + j] = 0.0;
        } else {
          red[i * 64 + j] += d00[r];
          red[i * 64 + 32 + j] += d01[r];
          red[(32 + i) * 64 + 32 + j] += d11[r];
        }
      }
    }
    __syncthreads();
  }
  double* out = F.mom + ((int64_t)c * F.wpc + w) * 4096;
  for (int k = tid; k < 4096; k += 256) out[k] = red[k];
}

// grid (64, C), 256 threads (wpc > 1): the moment partials of a chunk summed in a fixed order into partial 0 --
// thread group g (4 of 64 threads) adds partials g, g + 4, ... of entry 64 blockIdx.x + lane, then the four group
// sums are added in order (the partials come from every XCD: 4 independent chains of loads in flight per entry)
__global__ __launch_bounds__(256) void k_tf_msum(FoldDev F) {
  __shared__ double red[4][64];
  const int g = threadIdx.x >> 6, lane = threadIdx.x & 63, k = blockIdx.x * 64 + lane;
  double* m = F.mom + (int64_t)blockIdx.y * F.wpc * 4096 + k;
  double s = 0.0;
#pragma unroll 8
  for (int w = g; w < F.wpc; w += 4) s += m[(int64_t)w * 4096];
  red[g][lane] = s;
  __syncthreads();
  if (g == 0) m[0] = (red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]);
}

// grid C, 256 threads: n = sum d_63^2, dbar = sum d / n, Sigma = sum d d^T / n - dbar dbar^T, ebar = e0 + dbar.
__global__ __launch_bounds__(256) void k_tf_stats(FoldDev F) {
  __shared__ double G[4096];
  const int c = blockIdx.x, tid = threadIdx.x;
  const double* m = F.mom + (int64_t)c * F.wpc * 4096;
  for (int k = tid; k < 4096; k += 256) G[k] = m[k];
  __syncthreads();
  const double n = G[63 * 64 + 63];
  for (int k = tid; k < 4096; k += 256) {
    const int i = k >> 6, j = k & 63;
    double v = 0.0;
    if (i < 63 && j < 63) {
      const int lo = i < j ? i : j, hi = i < j ? j : i;   // blocks 00, 01, 11 hold the upper triangle
      v = G[lo * 64 + hi] / n - (G[i * 64 + 63] / n) * (G[j * 64 + 63] / n);
    }
    F.sig[(int64_t)c * 4096 + k] = v;
  }
  if (tid < 64) F.eb[(int64_t)c * 64 + tid] = tid < 63 ? F.e0[(int64_t)c * 64 + tid] + G[tid * 64 + 63] / n : 0.0;
}

// (float64 64 x 64 tiles on v_mfma_f64_16x16x4_f64: mfma64_quad, common.h)

// ---- 16-row tiles (the layer algebra's kernels): wave w owns the tile's columns 16 w .. 16 w + 15, one 16 x 16
// block on v_mfma_f64_16x16x4_f64: acc += A B over k in [0, 64) with A(r, k) = ATR ? As[k TP + r] : As[r TP + k]
// (r < 16), B(k, col) = Bs[k TP + col].  Four times the workgroups of the 64-row form and a quarter of its MFMA
// chain per wave: the reference's shell setting has 1-3 chunks, so the chain's latency was the cost.
template <bool ATR>
__device__ __forceinline__ void mfma16_rows(const double* As, const double* Bs, int wave, int lane, f64x4& acc) {
  const int li = lane & 15, lk = lane >> 4;
#pragma unroll 4
  for (int k0 = 0; k0 < 64; k0 += 4) {
    const int k = k0 + lk;
    const double a = ATR ? As[k * TP + li] : As[li * TP + k];
    const double b = Bs[k * TP + 16 * wave + li];
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
  }
}

// sum over the wave's 16 columns of v[r] (row (lane >> 4) + 4 r of the tile) into red[wave][row]
__device__ __forceinline__ void row_sum16(const double (&v)[4], int wave, int lane, double (*red)[16]) {
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    double t = v[r];
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) t += __shfl_xor(t, o, 64);
    if ((lane & 15) == 0) red[wave][(lane >> 4) + 4 * r] = t;
  }
}

// k_tf_layer in 16-row tiles, grid (16, C): rows R0..R0+15 of P'_L, Q_L = P'_L Sigma, var, s, the pre-BN mean, and
// P_L = s_L (.) P'_L with beta_L in column 63 (F.ab[L & 1]: the next layer's B operand as a plain copy; the backward
// reuses the buffer for its adjoints).  Thread t stages B rows k0 + (t >> 6) + 4 it, column t & 63, through
// registers one K step ahead of the matrix products.
template <int L>
__global__ __launch_bounds__(256) void k_tf_layer16(NofParamsDev P, FoldDev F, double eps) {
  constexpr int IN = L == 0 ? 63 : L == 4 ? 319 : 256;
  constexpr int KE = (L == 0 || L == 4) ? 63 : 0;
  __shared__ double As[16 * TP];
  __shared__ double Bs[64 * TP];
  __shared__ double red[4][16];
  __shared__ double sv[16];
  const int64_t C = F.C;
  const int c = blockIdx.y, R0 = blockIdx.x * 16, tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int col = tid & 63, rr = tid >> 6;
  const float* __restrict__ W = P.lin_w[L];
  const double* eb = F.eb + (int64_t)c * 64;
  const double* pbp = F.ab + ((int64_t)((L + 1) & 1) * C + c) * 256 * 64;   // P_{L-1} | beta_{L-1}
  const double* sg = F.sig + (int64_t)c * 4096;
  double bv[16];
  float av[4];
  auto load = [&](int k0) {
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      const int e = tid + 256 * it, k = k0 + (e & 63);
      av[it] = k < IN ? W[(int64_t)(R0 + (e >> 6)) * IN + k] : 0.0f;
    }
#pragma unroll
    for (int it = 0; it < 16; ++it) {
      const int kr = k0 + rr + 4 * it;
      double x = 0.0;
      if (kr < KE) x = col < 63 ? (kr == col ? 1.0 : 0.0) : eb[kr];
      else if (kr < IN) x = pbp[(kr - KE) * 64 + col];
      bv[it] = x;
    }
  };
  load(0);
  f64x4 acc = f64x4{0.0, 0.0, 0.0, 0.0};
  for (int k0 = 0; k0 < IN; k0 += 64) {
#pragma unroll
    for (int it = 0; it < 4; ++it) As[(rr + 4 * it) * TP + col] = (double)av[it];
#pragma unroll
    for (int it = 0; it < 16; ++it) Bs[(rr + 4 * it) * TP + col] = bv[it];
    __syncthreads();
    if (k0 + 64 < IN) {
      load(k0 + 64);
    } else {
#pragma unroll
      for (int it = 0; it < 16; ++it) bv[it] = sg[(rr + 4 * it) * 64 + col];   // Sigma for Q_L
    }
    mfma16_rows<false>(As, Bs, wave, lane, acc);
    __syncthreads();
  }
  const int ocol = 16 * wave + (lane & 15);
  const int64_t base = (((int64_t)L * C + c) * 256 + R0) * 64;
  double* pp = F.pp + base;
  double* qo = F.q + base;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int row = (lane >> 4) + 4 * r;
    pp[row * 64 + ocol] = acc[r];
    As[row * TP + ocol] = acc[r];
  }
#pragma unroll
  for (int it = 0; it < 16; ++it) Bs[(rr + 4 * it) * TP + col] = bv[it];
  __syncthreads();
  f64x4 qa = f64x4{0.0, 0.0, 0.0, 0.0};
  mfma16_rows<false>(As, Bs, wave, lane, qa);
  double v[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int row = (lane >> 4) + 4 * r;
    qo[row * 64 + ocol] = qa[r];
    v[r] = qa[r] * acc[r];   // column 63: Sigma's row 63 is zero, so Q[:, 63] = 0
  }
  row_sum16(v, wave, lane, red);
  __syncthreads();
  if (tid < 16) {
    const int row = R0 + tid;
    double var = (red[0][tid] + red[1][tid]) + (red[2][tid] + red[3][tid]);
    if (var < 0.0) var = 0.0;
    const double rinv = 1.0 / sqrt(var + eps);
    const double sc = (double)P.bn_w[L][row] * rinv;
    double* sr = F.sr + ((int64_t)L * C + c) * 1024;
    sr[row] = sc;
    sr[256 + row] = rinv;
    sr[512 + row] = As[tid * TP + 63] + (double)P.lin_b[L][row];
    sr[768 + row] = var;
    sv[tid] = sc;
  }
  __syncthreads();
  double* pb = F.ab + ((int64_t)(L & 1) * C + c) * 256 * 64 + (int64_t)R0 * 64;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int row = (lane >> 4) + 4 * r;
    pb[row * 64 + ocol] = ocol < 63 ? sv[row] * acc[r] : (double)P.bn_b[L][R0 + row];
  }
}

// grid C, 256 threads: a_c = sum_i w_i s_7i P'_7[i][:63], c_c = w . beta_7 + b_out - a_c . ebar.
__global__ __launch_bounds__(256) void k_tf_out(NofParamsDev P, FoldDev F) {
  __shared__ double u[256];
  __shared__ double part[4][64];
  __shared__ double cw[4];
  const int c = blockIdx.x, tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int64_t C = F.C;
  const double* sr7 = F.sr + (7 * C + c) * 1024;
  u[tid] = (double)P.out_w[tid] * sr7[tid];
  const double cb = wave_sum_d((double)P.out_w[tid] * (double)P.bn_b[7][tid]);
  if (lane == 0) cw[wave] = cb;
  __syncthreads();
  const double* pp7 = F.pp + (7 * C + c) * 256 * 64;
  double s = 0.0;
  for (int i = 64 * wave; i < 64 * wave + 64; ++i) s += u[i] * pp7[i * 64 + lane];
  part[wave][lane] = s;
  __syncthreads();
  if (wave == 0) {
    const double a = lane < 63 ? (part[0][lane] + part[1][lane]) + (part[2][lane] + part[3][lane]) : 0.0;
    const double t = wave_sum_d(a * F.eb[(int64_t)c * 64 + lane]);
    F.fold[(int64_t)c * 64 + lane] =
        lane < 63 ? a : ((cw[0] + cw[1]) + (cw[2] + cw[3])) + (double)P.out_b[0] - t;
  }
}

// grid C, 256 threads: each chunk's BatchNorm coefficients for the train-mode query, bn_coeffs' (nof_train.hip)
// arithmetic on the chunk's exact batch statistics: invstd = fl32(1 / sqrt(var + eps)) (biased variance), alpha =
// invstd * gamma, and beta'' = beta - mean(W x) alpha with mean(W x) = P'[:, 63] -- the Linear's bias cancels
// inside BatchNorm, so the query's epilogue is (W x) alpha + beta''.  Then the operand scale of each layer's output:
// BatchNorm output k has batch mean beta_k and batch variance gamma_k^2 var / (var + eps) <= gamma_k^2, so by
// Samuelson's inequality no sample of the chunk exceeds sqrt(n) |gamma_k| + |beta_k|; sxB[L] puts the layer's
// largest such bound in [2^14, 2^15) (fp16's range with a factor-2 margin for rounding).
__global__ __launch_bounds__(256) void k_tf_coeffs(NofParamsDev P, FoldDev F, SampleSrc q) {
  __shared__ float red[4];
  const int c = blockIdx.x, k = threadIdx.x;
  const int64_t C = F.C;
  const float rn = sqrtf((float)chunk_len(q, c));
  float* o = F.coef + (int64_t)c * TQ_COEF_FLOATS;
  for (int L = 0; L < 8; ++L) {
    const double* sr = F.sr + ((int64_t)L * C + c) * 1024;
    const double m = F.pp[(((int64_t)L * C + c) * 256 + k) * 64 + 63];
    const float invstd = (float)(1.0 / sqrt(sr[768 + k] + (double)P.eps));
    const float a = invstd * P.bn_w[L][k];
    o[L * 512 + k] = a;
    o[L * 512 + 256 + k] = (float)((double)P.bn_b[L][k] - m * (double)a);
    float bnd = wave_max_f(rn * fabsf(P.bn_w[L][k]) + fabsf(P.bn_b[L][k]));
    if ((k & 63) == 0) red[k >> 6] = bnd;
    __syncthreads();
    if (k == 0) {
      bnd = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
      int sx = (bnd > 0.0f && bnd < 3.0e38f) ? 14 - ilogbf(bnd) : 0;
      sx = sx > 64 ? 64 : sx < -64 ? -64 : sx;
      reinterpret_cast<int*>(o + 16 * 256)[L] = sx;
    }
    __syncthreads();
  }
}

// grid (8 layers, store_chunks), 256 threads: a stored chunk's BatchNorm sums in the activation store's layout
// (nof_train.hip k_bn_save reads them): sum h and sum h^2 of the raw layer output h = W x (no Linear bias) over the
// chunk's n samples, from the exact statistics the query's coefficients come from (mean = P'_L's column 63, biased
// variance): n m and n (var + m^2) in float64.
__global__ void k_tf_store_stats(FoldDev F, SampleSrc q, char* __restrict__ store, size_t chunk_bytes,
                                 size_t stats_off) {
  const int L = blockIdx.x, k = threadIdx.x;
  const int64_t c = blockIdx.y, C = F.C;
  const double n = (double)chunk_len(q, c);
  const double m = F.pp[(((int64_t)L * C + c) * 256 + k) * 64 + 63];
  const double var = F.sr[((int64_t)L * C + c) * 1024 + 768 + k];
  double* st = reinterpret_cast<double*>(store + (size_t)c * chunk_bytes + stats_off);
  st[512 * L + 2 * k] = n * m;
  st[512 * L + 2 * k + 1] = n * (var + m * m);
}

// grid 8, 256 threads: running stats chunk by chunk, bn_coeffs' arithmetic (float64 update, stored as float).
__global__ void k_tf_running(NofParamsDev P, FoldDev F, SampleSrc q, double mom) {
  const int L = blockIdx.x, k = threadIdx.x;
  if (!P.bn_rm[L]) return;
  float rm = P.bn_rm[L][k], rv = P.bn_rv[L][k];
  for (int64_t c0 = 0; c0 < F.C; c0 += 8) {   // eight chunks' statistics loaded before the sequential updates
    double mean[8], var[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int64_t c = c0 + j < F.C ? c0 + j : F.C - 1;
      const double* sr = F.sr + ((int64_t)L * F.C + c) * 1024;
      mean[j] = sr[512 + k];
      var[j] = sr[768 + k];
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (c0 + j >= F.C) break;
      const int64_t n = chunk_len(q, c0 + j);
      rm = (float)(mom * mean[j] + (1.0 - mom) * (double)rm);
      const double unb = n > 1 ? var[j] * (double)n / (double)(n - 1) : var[j];
      rv = (float)(mom * unb + (1.0 - mom) * (double)rv);
    }
  }
  P.bn_rm[L][k] = rm;
  P.bn_rv[L][k] = rv;
}

// grid 8, 256 threads: the running statistics after n chunks' batch statistics applied in order, k_tf_running's
// arithmetic -- st [n][8][2][256] (mean of h_L with its bias, biased variance), ns [n] the chunks' sample counts.
// The data-parallel BatchNorm sync (nof/bn_sync.py) replays every rank's chunks in global order with it.
__global__ void k_bn_replay(NofParamsDev P, const double* __restrict__ st, const int64_t* __restrict__ ns, int64_t n,
                            double mom) {
  const int L = blockIdx.x, k = threadIdx.x;
  if (!P.bn_rm[L]) return;
  float rm = P.bn_rm[L][k], rv = P.bn_rv[L][k];
#pragma unroll 8
  for (int64_t c = 0; c < n; ++c) {
    const double mean = st[(c * 8 + L) * 512 + k], var = st[(c * 8 + L) * 512 + 256 + k];
    const int64_t m = ns[c];
    rm = (float)(mom * mean + (1.0 - mom) * (double)rm);
    const double unb = m > 1 ? var * (double)m / (double)(m - 1) : var;
    rv = (float)(mom * unb + (1.0 - mom) * (double)rv);
  }
  P.bn_rm[L][k] = rm;
  P.bn_rv[L][k] = rv;
}

// ------------------------------------------------------------------------------------------------- backward
__device__ __forceinline__ float fold_logit_grad(const float* __restrict__ g, const float* __restrict__ p,
                                                 int64_t i) {
  if (!p) return g[i];
  const float pv = p[i];
  return g[i] * (1.0f - pv) * pv;   // sigmoid backward (as nof_train.hip's logit_grad)
}

// grid (wpc, C), 256 threads: sum g_s d_s (d as in k_tf_moments, fp32 here; d_63 = 1).  Each wave stages 64
// samples' d as a [sample][feature] fp32 tile (one lane per sample, its encoding written as computed) and g in
// LDS; then lane f accumulates sum_s g_s d_s[f] over the tile in float64 (exact products, one register).
__global__ __launch_bounds__(256) void k_tf_gmoments(SampleSrc q, FoldDev F, const float* __restrict__ g,
                                                     const float* __restrict__ p) {
  __shared__ float tile[4][64 * 65];
  __shared__ float gs[4][64];
  __shared__ float sh0[64];
  __shared__ double red[4][64];
  const int c = blockIdx.y, w = blockIdx.x, tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int64_t c0 = (int64_t)c * q.chunk, n = chunk_len(q, c);
  if (tid < 64) sh0[tid] = (float)F.e0[(int64_t)c * 64 + tid];
  __syncthreads();
  const int64_t ntile = (n + 63) / 64, per = (ntile + F.wpc - 1) / F.wpc;
  const int64_t t0 = std::min(ntile, (int64_t)w * per), t1 = std::min(ntile, t0 + per);
  float* my = tile[wave];
  double acc = 0.0;
  for (int64_t t = t0 + wave; t < t1; t += 4) {   // waves independent: wave-local LDS tiles
    const int64_t i = t * 64 + lane;
    const bool ok = i < n;
    auto put = [&](int f, float v) { my[lane * 65 + f] = ok ? v - sh0[f] : 0.0f; };
    if (q.ein) {
      const float* r = q.ein + (c0 + (ok ? i : 0)) * 63;
#pragma unroll 7
      for (int f = 0; f < 63; ++f) put(f, r[f]);
    } else {
      float pt[3] = {0.0f, 0.0f, 0.0f};
      if (ok) sample_point(q.rays + ray_of(c0 + i, q.S) * q.stride, q.z[c0 + i], pt);
#pragma unroll
      for (int m = 0; m < 3; ++m) put(m, pt[m]);
#pragma unroll 2
      for (int k = 0; k < 10; ++k) {
        const float sc = (float)(1 << k);
#pragma unroll
        for (int m = 0; m < 3; ++m) {
          float sv, cv;
          sincosf(sc * pt[m], &sv, &cv);
          put(3 + 6 * k + m, sv);
          put(6 + 6 * k + m, cv);
        }
      }
    }
    my[lane * 65 + 63] = ok ? 1.0f : 0.0f;
    gs[wave][lane] = ok ? fold_logit_grad(g, p, c0 + i) : 0.0f;
    wave_lds_sync();
#pragma unroll 16
    for (int s = 0; s < 64; ++s) acc += (double)gs[wave][s] * (double)my[s * 65 + lane];
    wave_lds_sync();
  }
  red[wave][lane] = acc;
  __syncthreads();
  if (tid < 64)
    F.gm[((int64_t)c * F.wpc + w) * 64 + tid] = (red[0][tid] + red[1][tid]) + (red[2][tid] + red[3][tid]);
}

// grid (4, C), 256 threads (rows I0..I0+63 of layer 7): abar = sum g (d - dbar), gbar = sum g; occ_out / beta_7
// gradient partials; the adjoint of P_7 is w_i abar_j, taken through BatchNorm 7 to A'_7 (ab[1]).
__global__ __launch_bounds__(256) void k_tf_bwd_out(NofParamsDev P, FoldDev F) {
  __shared__ double ab[64];
  __shared__ double dot[64], coef[64], dvv[64];
  __shared__ double gbar_s;
  __shared__ double gred[4][64];
  const int c = blockIdx.y, I0 = blockIdx.x * 64, tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int64_t C = F.C;
  {   // the gradient-moment partials: wave v adds partials v, v + 4, ..., then the four sums in order
    double G = 0.0;
    for (int w = wave; w < F.wpc; w += 4) G += F.gm[((int64_t)c * F.wpc + w) * 64 + lane];
    gred[wave][lane] = G;
  }
  __syncthreads();
  if (wave == 0) {
    const double G = (gred[0][lane] + gred[1][lane]) + (gred[2][lane] + gred[3][lane]);
    const double gb = __shfl(G, 63, 64);
    ab[lane] = lane < 63 ? G - gb * (F.eb[(int64_t)c * 64 + lane] - F.e0[(int64_t)c * 64 + lane]) : 0.0;
    if (lane == 0) gbar_s = gb;
  }
  __syncthreads();
  const double* pp7 = F.pp + (7 * C + c) * 256 * 64;
  const double* q7 = F.q + (7 * C + c) * 256 * 64;
  for (int r = wave; r < 64; r += 4) {
    const double d = wave_sum_d(ab[lane] * pp7[(I0 + r) * 64 + lane]);
    if (lane == 0) dot[r] = d;
  }
  __syncthreads();
  const double* sr7 = F.sr + (7 * C + c) * 1024;
  if (tid < 64) {
    const int i = I0 + tid;
    const double gb = gbar_s, s7 = sr7[i], rinv = sr7[256 + i], gam = (double)P.bn_w[7][i];
    const double w = (double)P.out_w[i], beta = (double)P.bn_b[7][i];
    double* v = F.vec + (int64_t)c * 576;
    v[i] = s7 * dot[tid] + beta * gb;
    v[256 + i] = w * gb;
    if (i == 0) v[512] = gb;
    const double ds = w * dot[tid];
    F.dg[(7 * C + c) * 256 + i] = ds * rinv;
    if (F.oacc) {   // sum_s g_s (h_7 - mean_7)_i and sum_s g_s, for the per-sample backward (nof_train.hip)
      F.oacc[c * 257 + i] = dot[tid];
      if (i == 0) F.oacc[c * 257 + 256] = gb;
    }
    dvv[tid] = -0.5 * ds * gam * rinv * rinv * rinv;
    coef[tid] = s7 * w;
  }
  __syncthreads();
  double* out = F.ab + (1 * C + c) * 256 * 64;
  for (int r = wave; r < 64; r += 4)
    out[(I0 + r) * 64 + lane] = lane < 63 ? coef[r] * ab[lane] + 2.0 * dvv[r] * q7[(I0 + r) * 64 + lane] : 0.0;
}

// k_tf_bwd_layer in 16-row tiles, grid (16, C): rows k0..k0+15 of A_{L-1} = W_L^T A'_L, BatchNorm L-1's backward
// to A'_{L-1} and dgamma_{L-1} per chunk.  Staging through registers one K step ahead, as k_tf_layer16.
template <int L>
__global__ __launch_bounds__(256) void k_tf_bwd_layer16(NofParamsDev P, FoldDev F) {
  constexpr int IN = L == 4 ? 319 : 256, OFF = L == 4 ? 63 : 0;
  constexpr int LP = L - 1;
  __shared__ double As[64 * TP];   // W_L[i][OFF + K0 + kk], kk < 16 (read transposed)
  __shared__ double Bs[64 * TP];
  __shared__ double red[4][16];
  __shared__ double dsv[16];
  const int64_t C = F.C;
  const int c = blockIdx.y, K0 = blockIdx.x * 16, tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int col = tid & 63, rr = tid >> 6;
  const float* __restrict__ W = P.lin_w[L];
  const double* abin = F.ab + ((int64_t)(L & 1) * C + c) * 256 * 64;
  const double* ppp = F.pp + ((int64_t)LP * C + c) * 256 * 64;
  const double* qq = F.q + ((int64_t)LP * C + c) * 256 * 64;
  const double* srp = F.sr + ((int64_t)LP * C + c) * 1024;
  const int ocol = 16 * wave + (lane & 15);
  double pv[4], qv[4];   // the epilogue's operands, loaded while the products run
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int k = K0 + (lane >> 4) + 4 * r;
    pv[r] = ppp[k * 64 + ocol];
    qv[r] = qq[k * 64 + ocol];
  }
  double bv[16];
  float av[4];
  auto load = [&](int i0) {
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      const int e = tid + 256 * it;
      av[it] = W[(int64_t)(i0 + (e >> 4)) * IN + OFF + K0 + (e & 15)];
    }
#pragma unroll
    for (int it = 0; it < 16; ++it) bv[it] = abin[(i0 + rr + 4 * it) * 64 + col];
  };
  load(0);
  f64x4 acc = f64x4{0.0, 0.0, 0.0, 0.0};
  for (int i0 = 0; i0 < 256; i0 += 64) {
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      const int e = tid + 256 * it;
      As[(e >> 4) * TP + (e & 15)] = (double)av[it];
    }
#pragma unroll
    for (int it = 0; it < 16; ++it) Bs[(rr + 4 * it) * TP + col] = bv[it];
    __syncthreads();
    if (i0 + 64 < 256) load(i0 + 64);
    mfma16_rows<true>(As, Bs, wave, lane, acc);
    __syncthreads();
  }
  double v[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) v[r] = ocol < 63 ? acc[r] * pv[r] : 0.0;
  row_sum16(v, wave, lane, red);
  __syncthreads();
  if (tid < 16) {
    const int k = K0 + tid;
    const double ds = (red[0][tid] + red[1][tid]) + (red[2][tid] + red[3][tid]);
    F.dg[((int64_t)LP * C + c) * 256 + k] = ds * srp[256 + k];
    dsv[tid] = ds;
  }
  __syncthreads();
  double* out = F.ab + ((int64_t)(LP & 1) * C + c) * 256 * 64;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int kl = (lane >> 4) + 4 * r, k = K0 + kl;
    const double sk = srp[k], rinv = srp[256 + k], gam = (double)P.bn_w[LP][k];
    const double dv = -0.5 * dsv[kl] * gam * rinv * rinv * rinv;
    out[k * 64 + ocol] = ocol < 63 ? sk * acc[r] + 2.0 * dv * qv[r] : 0.0;
  }
}

// grid (16, G), 256 threads: partial g of dW_L's h columns, sum over the group's chunks of
// A'_L[i][j] * s_{L-1,k} P'_{L-1}[k][j] (j < 63), one 64 x 64 tile (rows I0, columns K0) per workgroup
// (both operands staged in their natural [row][j] layout, B read transposed).
template <int L>
__global__ __launch_bounds__(256) void k_tf_dw(FoldDev F) {
  __shared__ double As[64 * TP];
  __shared__ double Bs[64 * TP];
  const int64_t C = F.C;
  const int I0 = (blockIdx.x >> 2) * 64, K0 = (blockIdx.x & 3) * 64, g = blockIdx.y;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int R = 32 * (wave >> 1), Cc = 32 * (wave & 1);
  const int64_t cg0 = C * g / F.G, cg1 = C * (g + 1) / F.G;
  f64x4 acc[2][2];
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int y = 0; y < 2; ++y) acc[x][y] = f64x4{0.0, 0.0, 0.0, 0.0};
  for (int64_t c = cg0; c < cg1; ++c) {
    const double* abin = F.ab + ((int64_t)(L & 1) * C + c) * 256 * 64;
    const double* pp = F.pp + ((int64_t)(L - 1) * C + c) * 256 * 64;
    const double* s = F.sr + ((int64_t)(L - 1) * C + c) * 1024;
    for (int e = tid; e < 4096; e += 256) {
      const int r = e >> 6, j = e & 63;
      As[r * TP + j] = abin[(I0 + r) * 64 + j];
      Bs[r * TP + j] = j < 63 ? s[K0 + r] * pp[(K0 + r) * 64 + j] : 0.0;
    }
    __syncthreads();
    mfma64_quad<false, true>(As, Bs, R, Cc, lane, acc);
    __syncthreads();
  }
  double* out = F.dw + (int64_t)g * 65536;
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int y = 0; y < 2; ++y)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        out[(I0 + q_row(R, x, r, lane)) * 256 + K0 + q_col(Cc, y, lane)] = acc[x][y][r];
}

// grid 256 (rows i), 320 threads (columns): dW_L[i][col] += encoding columns: sum_c A'_L[i][col]; h columns: the
// chunk-group partials, in a fixed order.
template <int L>
__global__ __launch_bounds__(320) void k_tf_dw_reduce(FoldDev F, float* __restrict__ gw) {
  constexpr int IN = L == 0 ? 63 : L == 4 ? 319 : 256;
  constexpr int KE = (L == 0 || L == 4) ? 63 : 0;
  const int i = blockIdx.x, col = threadIdx.x;
  if (col >= IN) return;
  double s = 0.0;
  if (col < KE) {
    for (int64_t c = 0; c < F.C; ++c) s += F.ab[((int64_t)(L & 1) * F.C + c) * 256 * 64 + i * 64 + col];
  } else {
    for (int g = 0; g < F.G; ++g) s += F.dw[(int64_t)g * 65536 + i * 256 + col - KE];
  }
  gw[(int64_t)i * IN + col] += (float)s;
}

// grid 10, 256 threads: blocks 0-7 dgamma_L, block 8 d out_w, block 9 d beta_7 and d out_b, summed over chunks.
__global__ void k_tf_vec_reduce(FoldDev F, pcnerf_nof_grads G) {
  const int b = blockIdx.x, k = threadIdx.x;
  double s = 0.0;
  if (b < 8) {
    if (!G.bn_w[b]) return;
    for (int64_t c = 0; c < F.C; ++c) s += F.dg[((int64_t)b * F.C + c) * 256 + k];
    G.bn_w[b][k] += (float)s;
  } else if (b == 8) {
    if (!G.out_w) return;
    for (int64_t c = 0; c < F.C; ++c) s += F.vec[c * 576 + k];
    G.out_w[k] += (float)s;
  } else {
    if (G.bn_b[7]) {
      for (int64_t c = 0; c < F.C; ++c) s += F.vec[c * 576 + 256 + k];
      G.bn_b[7][k] += (float)s;
    }
    if (k == 0 && G.out_b) {
      double t = 0.0;
      for (int64_t c = 0; c < F.C; ++c) t += F.vec[c * 576 + 512];
      G.out_b[0] += (float)t;
    }
  }
}

// ------------------------------------------------------------------------------------------------- host
template <int L>
static void launch_layer(const NofParamsDev& P, const FoldDev& F, double eps, hipStream_t s) {
  hipLaunchKernelGGL(k_tf_layer16<L>, dim3(16, (unsigned)F.C), dim3(256), 0, s, P, F, eps);
}

static void fold_forward(const SampleSrc& q, const pcnerf_nof_params* params, float momentum, float eps,
                         void* state, size_t state_bytes, float* p_out, hipStream_t s) {
  PCN_CHECK(q.total > 0 && q.chunk > 0, "train fold: empty input");
  // nn.BatchNorm1d raises for a chunk of one sample (render.py:47-50 would hit it on a 1-sample tail)
  PCN_CHECK(q.total % q.chunk != 1 && q.total != 1, "Expected more than 1 value per channel when training");
  const FoldLayout Lo = fold_layout(q.total, q.chunk);
  PCN_CHECK(state_bytes >= Lo.doubles * sizeof(double), "train fold: state buffer too small");
  PCN_CHECK(Lo.C < 65536, "train fold: too many chunks for one query");
  NofParamsDev P;
  PCN_CHECK(to_dev_params(params, eps, &P), "train fold: null parameter pointer");
  const FoldDev F = fold_dev(Lo, state);
  const double ep = (double)eps;
  {
    // algorithmic work per sample: the encoding + 3 x 32 x 32 x 2 flops per k-step pair; bytes: z in, ray rows
    ProfScope ps(s, PT_FOLD_MOMENTS, 6144.0 * (double)q.total, 4.0 * (double)q.total);
    hipLaunchKernelGGL(k_tf_moments, dim3(F.wpc, (unsigned)F.C), dim3(256), 0, s, q, F);
  }
  {
    ProfScope ps(s, PT_FOLD_ALGEBRA, 0.0, 0.0);
    if (F.wpc > 1) hipLaunchKernelGGL(k_tf_msum, dim3(64, (unsigned)F.C), dim3(256), 0, s, F);
    hipLaunchKernelGGL(k_tf_stats, dim3((unsigned)F.C), dim3(256), 0, s, F);
    launch_layer<0>(P, F, ep, s);
    launch_layer<1>(P, F, ep, s);
    launch_layer<2>(P, F, ep, s);
    launch_layer<3>(P, F, ep, s);
    launch_layer<4>(P, F, ep, s);
    launch_layer<5>(P, F, ep, s);
    launch_layer<6>(P, F, ep, s);
    launch_layer<7>(P, F, ep, s);
    hipLaunchKernelGGL(k_tf_out, dim3((unsigned)F.C), dim3(256), 0, s, P, F);
  }
  {
    ProfScope ps(s, PT_EVAL_FOLD, 126.0 * (double)q.total, 8.0 * (double)q.total);
    launch_fold_logits(q.rays, q.stride, q.z, q.total, q.S, q.ein, F.fold, q.chunk, p_out, s);
  }
  hipLaunchKernelGGL(k_tf_running, dim3(8), dim3(256), 0, s, P, F, q, (double)momentum);
}

// The train-mode query evaluated per sample (the network as written, one BatchNorm coefficient set per chunk):
// the chunk statistics from the encoding moments and the float64 layer algebra above, then k_nof_eval_h3<true>.
static void fused_forward(const SampleSrc& q, const pcnerf_nof_params* params, float momentum, float eps,
                          void* state, size_t state_bytes, float* p_out, hipStream_t s, void* store = nullptr,
                          int64_t store_chunks = 0, bool keep = false) {
  PCN_CHECK(q.total > 0 && q.chunk > 0, "train query: empty input");
  // nn.BatchNorm1d raises for a chunk of one sample (render.py:47-50 would hit it on a 1-sample tail)
  PCN_CHECK(q.total % q.chunk != 1 && q.total != 1, "Expected more than 1 value per channel when training");
  // with an activation store, or kept for the rematerialised backward (keep), the state is the backward's too
  // (fold_bn_backward): the full layout
  const FoldLayout Lo = fold_layout(q.total, q.chunk, store == nullptr && !keep);
  PCN_CHECK(state_bytes >= Lo.doubles * sizeof(double), "train query: state buffer too small");
  PCN_CHECK(Lo.C < 65536, "train query: too many chunks for one query");
  NofParamsDev P;
  PCN_CHECK(to_dev_params(params, eps, &P), "train query: null parameter pointer");
  const FoldDev F = fold_dev(Lo, state);
  const double ep = (double)eps;
  pack_train_query(P, F.img, s);
  {
    ProfScope ps(s, PT_FOLD_MOMENTS, 6144.0 * (double)q.total, 4.0 * (double)q.total);
    hipLaunchKernelGGL(k_tf_moments, dim3(F.wpc, (unsigned)F.C), dim3(256), 0, s, q, F);
  }
  {
    ProfScope ps(s, PT_FOLD_ALGEBRA, 0.0, 0.0);
    if (F.wpc > 1) hipLaunchKernelGGL(k_tf_msum, dim3(64, (unsigned)F.C), dim3(256), 0, s, F);
    hipLaunchKernelGGL(k_tf_stats, dim3((unsigned)F.C), dim3(256), 0, s, F);
    launch_layer<0>(P, F, ep, s);
    launch_layer<1>(P, F, ep, s);
    launch_layer<2>(P, F, ep, s);
    launch_layer<3>(P, F, ep, s);
    launch_layer<4>(P, F, ep, s);
    launch_layer<5>(P, F, ep, s);
    launch_layer<6>(P, F, ep, s);
    launch_layer<7>(P, F, ep, s);
    hipLaunchKernelGGL(k_tf_coeffs, dim3((unsigned)F.C), dim3(256), 0, s, P, F, q);
  }
  {
    // algorithmic work: 982,528 FLOP per sample (9 Linear layers); bytes: z in, p out, ray rows
    ProfScope ps(s, PT_TRAIN_QUERY, 982528.0 * (double)q.total, 8.0 * (double)q.total);
    const int64_t sc = store ? std::min<int64_t>(store_chunks, F.C) : 0;
    const size_t cb = pcnerf_nof_store_bytes(q.chunk), lb = store_layer_bytes(q.chunk);
    launch_train_query(q.rays, q.stride, q.z, q.total, q.S, q.ein, F.img, F.coef, q.chunk, p_out, s,
                       sc > 0 ? static_cast<float*>(store) : nullptr, (int64_t)(cb / 4), (int64_t)(lb / 4), sc);
    if (sc > 0)
      hipLaunchKernelGGL(k_tf_store_stats, dim3(8, (unsigned)sc), dim3(256), 0, s, F, q, static_cast<char*>(store),
                         cb, 8 * lb);
  }
  hipLaunchKernelGGL(k_tf_running, dim3(8), dim3(256), 0, s, P, F, q, (double)momentum);
}

template <int L>
static void backward_layer(const NofParamsDev& P, const FoldDev& F, const pcnerf_nof_grads* G, hipStream_t s) {
  if constexpr (L > 0) hipLaunchKernelGGL(k_tf_dw<L>, dim3(16, F.G), dim3(256), 0, s, F);
  if (G->lin_w[L]) hipLaunchKernelGGL(k_tf_dw_reduce<L>, dim3(256), dim3(320), 0, s, F, G->lin_w[L]);
  if constexpr (L > 0) hipLaunchKernelGGL(k_tf_bwd_layer16<L>, dim3(16, (unsigned)F.C), dim3(256), 0, s, P, F);
}

static void fold_backward(const SampleSrc& q, const pcnerf_nof_params* params, float eps, const float* g,
                          const float* p, void* state, size_t state_bytes, const pcnerf_nof_grads* G,
                          hipStream_t s) {
  PCN_CHECK(q.total > 0 && q.chunk > 0, "train fold backward: empty input");
  PCN_CHECK(q.total % q.chunk != 1 && q.total != 1, "Expected more than 1 value per channel when training");
  const FoldLayout Lo = fold_layout(q.total, q.chunk);
  PCN_CHECK(state_bytes >= Lo.doubles * sizeof(double), "train fold backward: state buffer too small");
  NofParamsDev P;
  PCN_CHECK(to_dev_params(params, eps, &P), "train fold backward: null parameter pointer");
  const FoldDev F = fold_dev(Lo, state);
  {
    ProfScope ps(s, PT_FOLD_MOMENTS, 126.0 * (double)q.total, 8.0 * (double)q.total);
    hipLaunchKernelGGL(k_tf_gmoments, dim3(F.wpc, (unsigned)F.C), dim3(256), 0, s, q, F, g, p);
  }
  ProfScope ps(s, PT_FOLD_ALGEBRA, 0.0, 0.0);
  hipLaunchKernelGGL(k_tf_bwd_out, dim3(4, (unsigned)F.C), dim3(256), 0, s, P, F);
  backward_layer<7>(P, F, G, s);
  backward_layer<6>(P, F, G, s);
  backward_layer<5>(P, F, G, s);
  backward_layer<4>(P, F, G, s);
  backward_layer<3>(P, F, G, s);
  backward_layer<2>(P, F, G, s);
  backward_layer<1>(P, F, G, s);
  backward_layer<0>(P, F, G, s);
  hipLaunchKernelGGL(k_tf_vec_reduce, dim3(10), dim3(256), 0, s, F, *G);
}

// The per-sample training backward's BatchNorm statistics (nof_train.hip, backward_train with a fold state): the
// state the store-writing fused forward left (full layout), the gradient moments of g_logit, and the fold's layer
// algebra down to every BatchNorm's dgamma per chunk (Sigma_s dL/dy (h - mean) / sqrt(var + eps)) and the occ_out
// statistics -- no weight gradient (the per-sample passes compute those as written).
FoldBnBwd fold_bn_backward(const float* rays, int stride, const float* z, int S, int64_t total, int64_t chunk,
                           const NofParamsDev& P, const float* g_logit, void* state, size_t state_bytes,
                           hipStream_t s) {
  const SampleSrc q{rays, stride, z, S, nullptr, total, std::min(chunk, total)};
  const FoldLayout Lo = fold_layout(q.total, q.chunk);
  PCN_CHECK(state_bytes >= Lo.doubles * sizeof(double), "train backward: fold state buffer too small");
  const FoldDev F = fold_dev(Lo, state);
  {
    ProfScope ps(s, PT_FOLD_MOMENTS, 126.0 * (double)q.total, 8.0 * (double)q.total);
    hipLaunchKernelGGL(k_tf_gmoments, dim3(F.wpc, (unsigned)F.C), dim3(256), 0, s, q, F, g_logit,
                       (const float*)nullptr);
  }
  ProfScope ps(s, PT_FOLD_ALGEBRA, 0.0, 0.0);
  hipLaunchKernelGGL(k_tf_bwd_out, dim3(4, (unsigned)F.C), dim3(256), 0, s, P, F);
  hipLaunchKernelGGL(k_tf_bwd_layer16<7>, dim3(16, (unsigned)F.C), dim3(256), 0, s, P, F);
  hipLaunchKernelGGL(k_tf_bwd_layer16<6>, dim3(16, (unsigned)F.C), dim3(256), 0, s, P, F);
  hipLaunchKernelGGL(k_tf_bwd_layer16<5>, dim3(16, (unsigned)F.C), dim3(256), 0, s, P, F);
  hipLaunchKernelGGL(k_tf_bwd_layer16<4>, dim3(16, (unsigned)F.C), dim3(256), 0, s, P, F);
  hipLaunchKernelGGL(k_tf_bwd_layer16<3>, dim3(16, (unsigned)F.C), dim3(256), 0, s, P, F);
  hipLaunchKernelGGL(k_tf_bwd_layer16<2>, dim3(16, (unsigned)F.C), dim3(256), 0, s, P, F);
  hipLaunchKernelGGL(k_tf_bwd_layer16<1>, dim3(16, (unsigned)F.C), dim3(256), 0, s, P, F);
  return FoldBnBwd{F.dg, F.sr, F.oacc, F.C, F.pp, F.eb, F.q};
}

}  // namespace pcn

using namespace pcn;

extern "C" size_t pcnerf_nof_train_fold_bytes(int64_t total_samples, int64_t chunk) {
  if (total_samples <= 0 || chunk <= 0) return 0;
  return fold_layout(total_samples, std::min(chunk, total_samples)).doubles * sizeof(double);
}

extern "C" size_t pcnerf_nof_train_fused_bytes(int64_t total_samples, int64_t chunk) {
  if (total_samples <= 0 || chunk <= 0) return 0;
  return fold_layout(total_samples, std::min(chunk, total_samples), true).doubles * sizeof(double);
}

// Per-chunk BatchNorm batch statistics of a fused / fold train query (or embedded forward) from its state, while
// the state is still the forward's (before any backward): out [C][8][2][256] doubles = each chunk's mean of h_L
// (bias included) and biased variance -- what k_tf_running applied to running_mean / running_var.
extern "C" int pcnerf_nof_train_bn_stats(const void* state, size_t state_bytes, int64_t total_samples, int64_t chunk,
                                         double* out, void* stream) {
  PCN_API_BEGIN
  PCN_CHECK(state && out, "pcnerf_nof_train_bn_stats: null argument");
  PCN_CHECK(total_samples > 0 && chunk > 0, "pcnerf_nof_train_bn_stats: empty input");
  // the statistics' offset is the same in the forward-only and the full layout (pieces before it do not change)
  const FoldLayout Lo = fold_layout(total_samples, std::min(chunk, total_samples), true);
  PCN_CHECK(state_bytes >= Lo.doubles * sizeof(double), "pcnerf_nof_train_bn_stats: state buffer too small");
  const double* sr = static_cast<const double*>(state) + Lo.off[6];
  for (int L = 0; L < 8; ++L)
    PCN_HIP(hipMemcpy2DAsync(out + L * 512, 8 * 512 * sizeof(double), sr + (size_t)L * Lo.C * 1024 + 512,
                             1024 * sizeof(double), 512 * sizeof(double), (size_t)Lo.C, hipMemcpyDeviceToDevice,
                             (hipStream_t)stream));
  PCN_API_END
}

// running_mean / running_var of `params` advanced over n_chunks chunks' statistics in order (k_bn_replay):
// stats [n_chunks][8][2][256] as pcnerf_nof_train_bn_stats writes them, ns [n_chunks] (device) their sample counts.
extern "C" int pcnerf_bn_running_replay(const pcnerf_nof_params* params, float momentum, const double* stats,
                                        const int64_t* ns, int64_t n_chunks, void* stream) {
  PCN_API_BEGIN
  PCN_CHECK(params && stats && ns, "pcnerf_bn_running_replay: null argument");
  PCN_CHECK(n_chunks >= 0, "pcnerf_bn_running_replay: negative chunk count");
  NofParamsDev P;
  PCN_CHECK(to_dev_params(params, 1e-5f, &P), "pcnerf_bn_running_replay: null parameter pointer");
  if (n_chunks > 0)
    hipLaunchKernelGGL(k_bn_replay, dim3(8), dim3(256), 0, (hipStream_t)stream, P, stats, ns, n_chunks,
                       (double)momentum);
  PCN_LAUNCH_CHECK("pcnerf_bn_running_replay");
  PCN_API_END
}

extern "C" int pcnerf_nof_query_train_fused(const float* rays, int64_t n_rays, int ray_stride, const float* z,
                                            int n_samples, int64_t chunk, const pcnerf_nof_params* params,
                                            float momentum, float eps, void* state, size_t state_bytes, float* p_out,
                                            void* stream) {
  PCN_API_BEGIN
  PCN_CHECK(rays && z && params && state && p_out, "pcnerf_nof_query_train_fused: null argument");
  PCN_CHECK(n_rays > 0 && n_samples > 0 && chunk > 0, "pcnerf_nof_query_train_fused: empty input");
  PCN_CHECK(ray_stride >= 6, "pcnerf_nof_query_train_fused: ray_stride < 6");
  const int64_t total = n_rays * (int64_t)n_samples;
  const SampleSrc q{rays, ray_stride, z, n_samples, nullptr, total, std::min(chunk, total)};
  fused_forward(q, params, momentum, eps, state, state_bytes, p_out, (hipStream_t)stream);
  PCN_LAUNCH_CHECK("pcnerf_nof_query_train_fused");
  PCN_API_END
}

// The training step's forward: the fused query, its state in the full layout (pcnerf_nof_train_fold_bytes) kept for
// pcnerf_nof_query_train_backward_remat -- nothing else is written for the backward.
extern "C" int pcnerf_nof_query_train_fused_state(const float* rays, int64_t n_rays, int ray_stride, const float* z,
                                                  int n_samples, int64_t chunk, const pcnerf_nof_params* params,
                                                  float momentum, float eps, void* state, size_t state_bytes,
                                                  float* p_out, void* stream) {
  PCN_API_BEGIN
  PCN_CHECK(rays && z && params && state && p_out, "pcnerf_nof_query_train_fused_state: null argument");
  PCN_CHECK(n_rays > 0 && n_samples > 0 && chunk > 0, "pcnerf_nof_query_train_fused_state: empty input");
  PCN_CHECK(ray_stride >= 6, "pcnerf_nof_query_train_fused_state: ray_stride < 6");
  const int64_t total = n_rays * (int64_t)n_samples;
  const SampleSrc q{rays, ray_stride, z, n_samples, nullptr, total, std::min(chunk, total)};
  fused_forward(q, params, momentum, eps, state, state_bytes, p_out, (hipStream_t)stream, nullptr, 0, true);
  PCN_LAUNCH_CHECK("pcnerf_nof_query_train_fused_state");
  PCN_API_END
}

extern "C" int pcnerf_nof_query_train_fused_store(const float* rays, int64_t n_rays, int ray_stride, const float* z,
                                                  int n_samples, int64_t chunk, const pcnerf_nof_params* params,
                                                  float momentum, float eps, void* state, size_t state_bytes,
                                                  float* p_out, void* store, int64_t store_chunks, void* stream) {
  PCN_API_BEGIN
  PCN_CHECK(rays && z && params && state && p_out, "pcnerf_nof_query_train_fused_store: null argument");
  PCN_CHECK(n_rays > 0 && n_samples > 0 && chunk > 0, "pcnerf_nof_query_train_fused_store: empty input");
  PCN_CHECK(ray_stride >= 6, "pcnerf_nof_query_train_fused_store: ray_stride < 6");
  PCN_CHECK(store_chunks == 0 || store, "pcnerf_nof_query_train_fused_store: store_chunks > 0 needs a store");
  const int64_t total = n_rays * (int64_t)n_samples;
  const SampleSrc q{rays, ray_stride, z, n_samples, nullptr, total, std::min(chunk, total)};
  fused_forward(q, params, momentum, eps, state, state_bytes, p_out, (hipStream_t)stream, store, store_chunks);
  PCN_LAUNCH_CHECK("pcnerf_nof_query_train_fused_store");
  PCN_API_END
}

extern "C" int pcnerf_nof_forward_train_fused(const float* emb, int64_t n, const pcnerf_nof_params* params,
                                              float momentum, float eps, void* state, size_t state_bytes,
                                              float* p_out, void* stream) {
  PCN_API_BEGIN
  PCN_CHECK(emb && params && state && p_out, "pcnerf_nof_forward_train_fused: null argument");
  PCN_CHECK(n > 1, "pcnerf_nof_forward_train_fused: Expected more than 1 value per channel when training");
  const SampleSrc q{nullptr, 0, nullptr, 1, emb, n, n};
  fused_forward(q, params, momentum, eps, state, state_bytes, p_out, (hipStream_t)stream);
  PCN_LAUNCH_CHECK("pcnerf_nof_forward_train_fused");
  PCN_API_END
}

extern "C" int pcnerf_nof_query_train_fold(const float* rays, int64_t n_rays, int ray_stride, const float* z,
                                           int n_samples, int64_t chunk, const pcnerf_nof_params* params,
                                           float momentum, float eps, void* state, size_t state_bytes, float* p_out,
                                           void* stream) {
  PCN_API_BEGIN
  PCN_CHECK(rays && z && params && state && p_out, "pcnerf_nof_query_train_fold: null argument");
  PCN_CHECK(n_rays > 0 && n_samples > 0 && chunk > 0, "pcnerf_nof_query_train_fold: empty input");
  PCN_CHECK(ray_stride >= 6, "pcnerf_nof_query_train_fold: ray_stride < 6");
  const int64_t total = n_rays * (int64_t)n_samples;
  const SampleSrc q{rays, ray_stride, z, n_samples, nullptr, total, std::min(chunk, total)};
  fold_forward(q, params, momentum, eps, state, state_bytes, p_out, (hipStream_t)stream);
  PCN_LAUNCH_CHECK("pcnerf_nof_query_train_fold");
  PCN_API_END
}

extern "C" int pcnerf_nof_forward_train_fold(const float* emb, int64_t n, const pcnerf_nof_params* params,
                                             float momentum, float eps, void* state, size_t state_bytes,
                                             float* p_out, void* stream) {
  PCN_API_BEGIN
  PCN_CHECK(emb && params && state && p_out, "pcnerf_nof_forward_train_fold: null argument");
  PCN_CHECK(n > 1, "pcnerf_nof_forward_train_fold: Expected more than 1 value per channel when training");
  const SampleSrc q{nullptr, 0, nullptr, 1, emb, n, n};
  fold_forward(q, params, momentum, eps, state, state_bytes, p_out, (hipStream_t)stream);
  PCN_LAUNCH_CHECK("pcnerf_nof_forward_train_fold");
  PCN_API_END
}

extern "C" int pcnerf_nof_query_train_fold_backward(const float* rays, int64_t n_rays, int ray_stride,
                                                    const float* z, int n_samples, int64_t chunk,
                                                    const pcnerf_nof_params* params, float eps,
                                                    const float* grad_logit, void* state, size_t state_bytes,
                                                    const pcnerf_nof_grads* grads, void* stream) {
  PCN_API_BEGIN
  PCN_CHECK(rays && z && params && grad_logit && state && grads,
            "pcnerf_nof_query_train_fold_backward: null argument");
  PCN_CHECK(n_rays > 0 && n_samples > 0 && chunk > 0, "pcnerf_nof_query_train_fold_backward: empty input");
  PCN_CHECK(ray_stride >= 6, "pcnerf_nof_query_train_fold_backward: ray_stride < 6");
  const int64_t total = n_rays * (int64_t)n_samples;
  const SampleSrc q{rays, ray_stride, z, n_samples, nullptr, total, std::min(chunk, total)};
  fold_backward(q, params, eps, grad_logit, nullptr, state, state_bytes, grads, (hipStream_t)stream);
  PCN_LAUNCH_CHECK("pcnerf_nof_query_train_fold_backward");
  PCN_API_END
}

extern "C" int pcnerf_nof_forward_train_fold_backward(const float* emb, int64_t n, const pcnerf_nof_params* params,
                                                      float eps, const float* p, const float* grad_p, void* state,
                                                      size_t state_bytes, const pcnerf_nof_grads* grads,
                                                      void* stream) {
  PCN_API_BEGIN
  PCN_CHECK(emb && params && p && grad_p && state && grads, "pcnerf_nof_forward_train_fold_backward: null argument");
  PCN_CHECK(n > 1, "pcnerf_nof_forward_train_fold_backward: empty input");
  const SampleSrc q{nullptr, 0, nullptr, 1, emb, n, n};
  fold_backward(q, params, eps, grad_p, p, state, state_bytes, grads, (hipStream_t)stream);
  PCN_LAUNCH_CHECK("pcnerf_nof_forward_train_fold_backward");
  PCN_API_END
}
