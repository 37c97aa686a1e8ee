// Kernel timing scope: records a HIP event pair around the enclosed launch when profiling is enabled.
#pragma once
#include <hip/hip_runtime.h>

namespace pcn {
// tags reported by pcnerf_prof_read
enum ProfTag {
  PT_EVAL_QUERY = 0,   // k_nof_eval: fused 9-layer eval query
  PT_TRAIN_HIDDEN = 1, // k_train_ws<0,true>: 256 -> 256 pre-BN Linear (6 per chunk)
  PT_TRAIN_FIRST = 2,  // k_train_ws<8,false>: encoding -> 256
  PT_TRAIN_SKIP = 3,   // k_train_ws<8,true>: [encoding, 256] -> 256
  PT_TRAIN_OUT = 4,    // k_train_out
  PT_BN_FOLD = 5,      // k_bn_fold
  PT_COMPOSITE = 6,    // k_composite
  PT_RESAMPLE = 7,     // k_resample
  PT_SAMPLE = 8,       // k_sample_coarse / k_perturb
  PT_COMPOSITE_BWD = 9,// k_composite_bwd
  PT_BWD_WGRAD = 10,   // k_wgrad: weight-gradient GEMM partials (sum over samples on MFMA)
  PT_BWD_DGRAD = 11,   // k_dgrad_ws / k_dgrad_h: data-gradient GEMM + BatchNorm backward
  PT_BWD_MISC = 12,    // output-layer backward, partial reduction, BN statistics
  PT_EVAL_FOLD = 13,   // k_nof_eval_fold: exact affine fold of the eval network (opt-in)
  PT_BWD_WGRAD_H = 14, // k_wgrad_b3: weight gradients under the split train math
  PT_TRAIN_H1 = 15,    // k_train_h1: layer 1 from the encoding tiles (h0 recomputed)
  PT_FOLD_MOMENTS = 16,// train fold: k_tf_moments / k_tf_gmoments (per-sample encoding moments)
  PT_FOLD_ALGEBRA = 17,// train fold: the per-chunk float64 layer algebra (forward or backward)
  PT_TRAIN_QUERY = 18, // k_nof_eval_h3<true>: the fused train-mode query (per-chunk BatchNorm coefficients)
  PT_BWD_FUSED = 19,   // k_bwd_remat / k_bwd_fused: one layer's data + weight gradient in one pass
  PT_BWD_REMAT = 20,   // the rematerialised backward's per-chunk operands: encoding image (k_remat_enc), g_7 (k_g7)
  PT_BWD_FUSED_L1 = 21,// k_bwd_remat3<true, true>: layer 1 with dW_0's encoding columns formed in LDS
};
extern bool g_prof_on;
class ProfScope {
 public:
  ProfScope(hipStream_t s, int tag, double flops, double bytes);
  ~ProfScope();

 private:
  hipStream_t s_;
  int idx_;
};
}  // namespace pcn
