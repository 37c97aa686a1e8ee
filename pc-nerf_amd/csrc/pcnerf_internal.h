// Internal glue shared by the translation units: error reporting, the device-side parameter struct and the
// per-sample front end (sample position + positional encoding) used by every NOF query kernel.
#pragma once
#include <stdexcept>
#include <string>

#include "common.h"
#include "pcnerf_hip.h"

namespace pcn {

struct NofParamsDev {
  const float* lin_w[8];
  const float* lin_b[8];
  const float* bn_w[8];
  const float* bn_b[8];
  float* bn_rm[8];
  float* bn_rv[8];
  const float* out_w;
  const float* out_b;
  float eps;
};

bool to_dev_params(const pcnerf_nof_params* p, float eps, NofParamsDev* d);
void set_error(const std::string& msg);
// p_out[g] = sigmoid(fl32(a_c . Embedding(sample g) + c_c)), (a_c, c_c) = fold[64 c .. 64 c + 63] for the
// BatchNorm chunk c = g / chunk (nof_eval.hip: the eval fold with chunk >= total, the train fold per chunk)
void launch_fold_logits(const float* rays, int stride, const float* z, int64_t total, int S, const float* ein,
                        const double* fold, int64_t chunk, float* p_out, hipStream_t s);

// The train-mode query in k_nof_eval_h3's form (nof_eval.hip): the image (train_query_image_floats floats) holds
// the raw split weights and occ_out; coef[chunk] (TQ_COEF_FLOATS) each chunk's BatchNorm coefficients and the
// per-layer operand scales of its bound.
size_t train_query_image_floats();
// the activation store's bytes per layer of a chunk ([tile of 32 samples][32 k-groups][64 lanes][4] floats, 256-B
// aligned; nof_train.hip StoreChunk, pcnerf_nof_store_bytes): the chunk rounded up to 96 samples, so the train
// query's 48-sample blocks write whole tiles unconditionally (the tail's extra tiles are never read)
inline size_t store_layer_bytes(int64_t chunk) {
  return (size_t)((chunk + 95) / 96) * 3 * (32 * 256) * 4;
}
constexpr int TQ_COEF_FLOATS = 16 * 256 + 16;   // per chunk: [L][alpha 256 | beta'' 256], then sxB[8] (int)
void pack_train_query(const NofParamsDev& P, float* img, hipStream_t s);
void launch_train_query(const float* rays, int stride, const float* z, int64_t total, int S, const float* ein,
                        const float* img, const float* coef, int64_t chunk, float* p_out, hipStream_t s,
                        float* hst = nullptr, int64_t hst_chunk = 0, int64_t hst_layer = 0,
                        int64_t store_chunks = 0);

// The per-sample training backward's BatchNorm statistics from the fused forward's fold state (nof_fold.hip):
// dg [8][C][256] each BatchNorm's dgamma per chunk, sr [8][C][1024] (s, 1/sqrt(var+eps), mean, var per layer and
// chunk), oacc [C][257] (sum_s g_s (h_7 - mean_7), sum_s g_s).
struct FoldBnBwd {
  const double* dg;
  const double* sr;
  const double* oacc;
  int64_t C;
  const double* pp;   // [8][C][256][64] P'_L (column 63: the pre-BatchNorm mean without the Linear bias)
  const double* eb;   // [C][64] the chunks' encoding means
  void* scratch;      // the layer maps' Sigma products (P'_L Sigma, 1 MiB per chunk): free once fold_bn_backward ran
};
FoldBnBwd fold_bn_backward(const float* rays, int stride, const float* z, int S, int64_t total, int64_t chunk,
                           const NofParamsDev& P, const float* g_logit, void* state, size_t state_bytes,
                           hipStream_t s);

// p = o + d*z, one rounding per op (render.py:458; built with -ffp-contract=off).
// ray of flattened sample g (ray-major, S samples per ray): a 32-bit division when g fits (the 64-bit one is a long
// emulated sequence)
__device__ __forceinline__ int64_t ray_of(int64_t g, int S) {
  return g < 0x7fffffff ? (int64_t)((unsigned)g / (unsigned)S) : g / S;
}
__device__ __forceinline__ void sample_point(const float* __restrict__ r, float z, float (&p)[3]) {
  p[0] = r[0] + r[3] * z;
  p[1] = r[1] + r[4] * z;
  p[2] = r[2] + r[5] * z;
}

// Embedding(3, 10) (models.py:27-41): feature f of [x(3), sin(2^0 x)(3), cos(2^0 x)(3), ..., cos(2^9 x)(3)],
// f = 63 is zero padding.  freq_bands = 2**linspace(0,9,10) are exact powers of two, so 2^k * x is exact
// and only sinf/cosf rounding remains (full-range ocml sincosf, never the __sinf fast path).
// Lane half h receives, for k-step t = 0..31, feature 2t + h (MAP 0: eval chain) or 8(t>>2) + 4h + (t&3)
// (MAP 1: train-mode layer kernels, whose memory-resident activations use 16-byte feature groups).
__device__ __forceinline__ void encode_full(const float (&p)[3], float (&f)[64]) {
  f[0] = p[0];
  f[1] = p[1];
  f[2] = p[2];
#pragma unroll
  for (int k = 0; k < 10; ++k) {
    const float sc = (float)(1 << k);
#pragma unroll
    for (int m = 0; m < 3; ++m) {
      float s, c;
      sincosf(sc * p[m], &s, &c);
      f[3 + 6 * k + m] = s;
      f[6 + 6 * k + m] = c;
    }
  }
  f[63] = 0.0f;
}

template <int MAP = 0>
__device__ __forceinline__ void encode_half(const float (&p)[3], int h, float (&e)[32]) {
  float f[64];
  encode_full(p, f);
#pragma unroll
  for (int t = 0; t < 32; ++t) {
    if (MAP == 0) e[t] = h ? f[2 * t + 1] : f[2 * t];
    else e[t] = h ? f[8 * (t >> 2) + 4 + (t & 3)] : f[8 * (t >> 2) + (t & 3)];
  }
}

// The same operand selection from a stored (., 63) embedding row.
template <int MAP = 0>
__device__ __forceinline__ void load_embedding(const float* __restrict__ row, int h, float (&e)[32]) {
#pragma unroll
  for (int t = 0; t < 32; ++t) {
    const int f = MAP == 0 ? 2 * t + h : 8 * (t >> 2) + 4 * h + (t & 3);
    e[t] = f < 63 ? row[f] : 0.0f;
  }
}

}  // namespace pcn

#define PCN_API_BEGIN try {
#define PCN_API_END                                       \
  return 0;                                               \
  }                                                       \
  catch (const std::exception& ex__) {                    \
    pcn::set_error(ex__.what());                          \
    return 1;                                             \
  }
#define PCN_CHECK(cond, msg)                              \
  do {                                                    \
    if (!(cond)) throw std::runtime_error(msg);           \
  } while (0)
#define PCN_LAUNCH_CHECK(name)                                                                 \
  do {                                                                                         \
    hipError_t e__ = hipGetLastError();                                                        \
    if (e__ != hipSuccess) throw std::runtime_error(std::string(name) + ": " + hipGetErrorString(e__)); \
  } while (0)
#define PCN_HIP(call)                                                                          \
  do {                                                                                         \
    hipError_t e__ = (call);                                                                   \
    if (e__ != hipSuccess) throw std::runtime_error(std::string(#call) + ": " + hipGetErrorString(e__)); \
  } while (0)
