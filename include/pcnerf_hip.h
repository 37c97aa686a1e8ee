/* pcnerf_hip.h -- C ABI of the MI355X (gfx950) PC-NeRF render + loss path.
 *
 * The reference (biter0088/pc-nerf) has no FFI: its hot path is eager PyTorch called from Python
 * (nof/render.py, nof/networks/models.py, nof/criteria/loss.py).  This library is what that Python
 * boundary binds to: the drop-in modules under pc-nerf_amd/nof/ keep the reference's names and signatures
 * and call these entry points through ctypes.  Every entry point below names the
 * reference code it replaces.
 *
 * Conventions
 *   - every pointer is a device pointer (hipMalloc'd / torch CUDA tensor) unless stated otherwise;
 *   - `stream` is a hipStream_t (NULL = legacy default stream); all work is enqueued asynchronously on it;
 *   - arrays are contiguous, fp32 unless stated; "rays" rows are `ray_stride` floats apart;
 *   - return value 0 = success; nonzero = failure, with a message from pcnerf_last_error()
 *     (argument errors are detected on the host before anything is launched).
 */
#ifndef PCNERF_HIP_H
#define PCNERF_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PCNERF_ABI_VERSION 1
#define PCNERF_FEATURES 256 /* NOF feature_size supported by the kernels (models.py:45 default) */
#define PCNERF_IN_CH 63     /* 3 + 3*2*L_pos with L_pos = 10 (train_kitti.py:25-28)            */

int pcnerf_abi_version(void);
const char* pcnerf_last_error(void);

/* ---------------------------------------------------------------- NOF network (models.py:44-359)
 * Parameters in reference state_dict order: Linear weights [256,63],[256,256]x3,[256,319],[256,256]x3
 * (layer1.{0,3,6,9}, layer2.{0,2,4,6}), BatchNorm1d gamma/beta/running_mean/running_var
 * (layer1.{1,4,7,10}, layer2.{1,3,5,7}), occ_out.0 weight [1,256] and bias [1]. */
typedef struct pcnerf_nof_params {
  const float* lin_w[8];
  const float* lin_b[8];
  const float* bn_w[8];
  const float* bn_b[8];
  float* bn_rm[8]; /* running_mean: read in eval mode, updated in place in train mode */
  float* bn_rv[8]; /* running_var:  idem */
  const float* out_w;
  const float* out_b;
} pcnerf_nof_params;

/* Eval-mode network image: BatchNorm (running stats) folded into each Linear, weights repacked into the
 * MFMA operand order of the fused query kernels -- the fp32 image followed by the split-fp16 image (per-layer
 * power-of-two scales, hi/mid fp16 parts).  Replaces the per-call nn.Module forward in eval mode. */
size_t pcnerf_nof_eval_packed_floats(void);
int pcnerf_nof_pack_eval(const pcnerf_nof_params* params, float* packed, void* stream);

/* Arithmetic of the fused eval-mode query (pcnerf_nof_query_eval / pcnerf_nof_forward_eval), process-wide;
 * returns the previous mode, or -1 for an invalid one.  0: fp32 MFMA (v_mfma_f32_32x32x2_f32).  1 (default): each
 * fp32 operand as two fp16 parts (22 significant bits; weights scaled per layer, activations per sample by powers
 * of two) and hi*hi + hi*mid + mid*hi on v_mfma_f32_32x32x16_f16 (exact products, fp32 accumulation), as
 * pcnerf_set_train_math mode 1. */
int pcnerf_set_eval_math(int mode);

/* Fused eval-mode query: for every flattened sample g = ray*n_samples + s computes
 *   p_out[g] = NOF(Embedding(o + d*z[g]))        (render.py:18-25 chunk loop, models.py:27-41, :183-203)
 * with o = rays[ray, 0:3], d = rays[ray, 3:6]. */
int pcnerf_nof_query_eval(const float* rays, int64_t n_rays, int ray_stride, const float* z, int n_samples,
                          const float* packed, float* p_out, void* stream);

/* NOF.forward on an already embedded batch: p_out[i] = NOF(emb[i, 0:63]) (eval mode, packed image). */
int pcnerf_nof_forward_eval(const float* emb, int64_t n, const float* packed, float* p_out, void* stream);

/* Exact affine fold of the eval network (opt-in fast path): LeakyReLU(True) is the identity
 * (models.py:72,152,232) and eval BatchNorm is affine, so NOF(e) = sigmoid(a . e + c).  Writes fold[0..62] = a,
 * fold[63] = c (64 doubles), composed in float64 from the module's parameters (models.py:44-123, :183-203). */
int pcnerf_nof_fold_eval(const pcnerf_nof_params* params, double* fold, void* stream);

/* pcnerf_nof_query_eval through the fold: p_out[g] = sigmoid(fl32(a . Embedding(o + d*z[g]) + c)).  Replaces the
 * same eval chunk loop (render.py:18-25); rounding differs from the layer-by-layer network (~1e-7 rel logit). */
int pcnerf_nof_query_eval_fold(const float* rays, int64_t n_rays, int ray_stride, const float* z, int n_samples,
                               const double* fold, float* p_out, void* stream);

/* pcnerf_nof_forward_eval through the fold: p_out[i] = sigmoid(fl32(a . emb[i, 0:63] + c)). */
int pcnerf_nof_forward_eval_fold(const float* emb, int64_t n, const double* fold, float* p_out, void* stream);

/* Embedding(3, 10).forward (models.py:27-41): out[i, 0:63] = [x, sin(2^k x), cos(2^k x)]_k for x = pts[i, 0:3]. */
int pcnerf_embed(const float* pts, int64_t n, float* out, void* stream);

/* Train-mode query (BatchNorm batch statistics per chunk of `chunk` flattened ray-major samples, running
 * stats updated once per chunk with `momentum`; render.py:47-50 + nn.BatchNorm1d train semantics).
 * `workspace` must hold pcnerf_nof_train_workspace_bytes(chunk) bytes. */
size_t pcnerf_nof_train_workspace_bytes(int64_t chunk);
int pcnerf_nof_query_train(const float* rays, int64_t n_rays, int ray_stride, const float* z, int n_samples,
                           int64_t chunk, const pcnerf_nof_params* params, float momentum, float eps,
                           void* workspace, size_t workspace_bytes, float* p_out, void* stream);

/* Arithmetic of the train-mode Linear layers (forward and the backward's forward recomputation), process-wide;
 * returns the previous mode, or -1 for an invalid one.  0: fp32 MFMA (v_mfma_f32_32x32x2_f32, an fp32 FMA chain).
 * 1 (default) / 2: each fp32 operand split into two fp16 parts (22 significant bits, power-of-two scaled) and the
 * products taken on the fp16 matrix pipe (v_mfma_f32_32x32x16_f16: exact products, fp32 accumulation):
 * hi*hi + hi*mid + mid*hi (1) or + mid*mid (2).  Measured against a float64 evaluation of the render:
 * as accurate as mode 0.  The reference's own GPU runs used TF32 matmuls (train_kitti.py:267). */
int pcnerf_set_train_math(int mode);

/* The default training backward's layer kernel, process-wide; returns the previous one, or -1 for an invalid one.
 * 4 (default): k_bwd_remat3<true> -- each hidden layer's weight gradient contracted over the 64 encoding columns,
 * (sum_s g_L (x) (e - ebar)) P'_{L-1}^T, with P'_{L-1} the chunk's float64 layer map (x = h_{L-1} - mean = P' (e - ebar)
 * under identity activations, models.py:72) applied once per chunk; the BatchNorm-backward epilogue and the g stores
 * on the weight-gradient waves.  3: the same with the epilogue on the data-gradient waves.  2: k_bwd_remat2 (round 5: over the 256 rematerialised input
 * columns).  Same gradients within the parity envelope (tests/test_backward_gpu.py). */
int pcnerf_set_remat_version(int version);

/* NOF.forward in train mode on an embedded batch of n rows (one BatchNorm chunk; running stats updated). */
int pcnerf_nof_forward_train(const float* emb, int64_t n, const pcnerf_nof_params* params, float momentum,
                             float eps, void* workspace, size_t workspace_bytes, float* p_out, void* stream);

/* ---------------------------------------------------------------- training backward (loss.backward())
 * Parameter gradients of the train-mode query, i.e. what autograd produces through render.py:47-50 and
 * models.py:183-203 (Linear -> BatchNorm1d(train) x 8, skip concat, occ_out, sigmoid) in the reference's
 * training step (train_kitti.py:155 `loss` returned to Lightning, which calls backward).  The chunks are
 * recomputed (same BatchNorm batches as the forward, running stats untouched).  Gradients are ADDED to the
 * non-NULL buffers of `grads` (torch .grad accumulation semantics); each has the shape of its parameter. */
typedef struct pcnerf_nof_grads {
  float* lin_w[8];
  float* lin_b[8];
  float* bn_w[8];
  float* bn_b[8];
  float* out_w;
  float* out_b;
} pcnerf_nof_grads;
size_t pcnerf_nof_backward_workspace_bytes(int64_t chunk);
/* grad_logit[g] = dL/d(occupancy logit) of flattened sample g (pcnerf_composite_backward's output). */
int pcnerf_nof_query_train_backward(const float* rays, int64_t n_rays, int ray_stride, const float* z,
                                    int n_samples, int64_t chunk, const pcnerf_nof_params* params, float eps,
                                    const float* grad_logit, void* workspace, size_t workspace_bytes,
                                    const pcnerf_nof_grads* grads, void* stream);
/* Activation store (the training step without the backward's recomputation): pcnerf_nof_store_bytes(chunk) bytes
 * per chunk hold that chunk's raw layer outputs h_1..h_8 and BatchNorm statistics.  The _store forward writes
 * chunks 0..store_chunks-1 into `store` (results otherwise identical to pcnerf_nof_query_train); the _store
 * backward reads them instead of recomputing those chunks (the rest are recomputed).  The caller sizes
 * store_chunks to the HBM it can spare (nof._autograd: what is free after the backward workspace). */
size_t pcnerf_nof_store_bytes(int64_t chunk);
int pcnerf_nof_query_train_store(const float* rays, int64_t n_rays, int ray_stride, const float* z, int n_samples,
                                 int64_t chunk, const pcnerf_nof_params* params, float momentum, float eps,
                                 void* workspace, size_t workspace_bytes, float* p_out, void* store,
                                 int64_t store_chunks, void* stream);
int pcnerf_nof_query_train_backward_store(const float* rays, int64_t n_rays, int ray_stride, const float* z,
                                          int n_samples, int64_t chunk, const pcnerf_nof_params* params, float eps,
                                          const float* grad_logit, void* workspace, size_t workspace_bytes,
                                          const pcnerf_nof_grads* grads, const void* store, int64_t store_chunks,
                                          void* stream);
/* NOF.forward(emb) in train mode (one batch): grad_p = dL/dp for p = the forward's output. */
int pcnerf_nof_forward_train_backward(const float* emb, int64_t n, const pcnerf_nof_params* params, float eps,
                                      const float* p, const float* grad_p, void* workspace, size_t workspace_bytes,
                                      const pcnerf_nof_grads* grads, void* stream);

/* ---------------------------------------------------------------- opt-in train-mode affine fold
 * Exact affine fold of the TRAIN-mode network (SURVEY fact 1 with BatchNorm batch statistics; not the default --
 * the drop-in evaluates the module as written).  Every LeakyReLU(True) is the identity (models.py:72,152,232), so
 * within one BatchNorm chunk (render.py:47-50) every layer's batch mean and variance follow exactly from the
 * chunk's encoding mean and covariance, and NOF(e) = sigmoid(a_c . e + c_c) per chunk c (models.py:183-203).  The
 * forward computes those per-chunk moments, the float64 layer algebra, p_out and the running-stat updates (chunk by
 * chunk, as pcnerf_nof_query_train); `state` (pcnerf_nof_train_fold_bytes(total_samples, chunk) bytes) keeps what
 * the backward needs and must stay unchanged until it runs.  The backward ADDS the parameter gradients (the
 * Linear biases and the shifts of BatchNorms 0-6 are exactly zero there: the next BatchNorm removes the mean). */
size_t pcnerf_nof_train_fold_bytes(int64_t total_samples, int64_t chunk);
int pcnerf_nof_query_train_fold(const float* rays, int64_t n_rays, int ray_stride, const float* z, int n_samples,
                                int64_t chunk, const pcnerf_nof_params* params, float momentum, float eps,
                                void* state, size_t state_bytes, float* p_out, void* stream);
int pcnerf_nof_forward_train_fold(const float* emb, int64_t n, const pcnerf_nof_params* params, float momentum,
                                  float eps, void* state, size_t state_bytes, float* p_out, void* stream);
int pcnerf_nof_query_train_fold_backward(const float* rays, int64_t n_rays, int ray_stride, const float* z,
                                         int n_samples, int64_t chunk, const pcnerf_nof_params* params, float eps,
                                         const float* grad_logit, void* state, size_t state_bytes,
                                         const pcnerf_nof_grads* grads, void* stream);
/* ---------------------------------------------------------------- train-mode query without activations
 * The render+loss forward's train-mode query (render.py:38-50 chunk loop over models.py:183-203 with BatchNorm batch
 * statistics per chunk; replaces the layer-by-layer pcnerf_nof_query_train where no backward needs the layer
 * outputs).  The network is evaluated AS WRITTEN, per sample, in one fused kernel (the 9 Linear layers on split-fp16
 * products, BatchNorm applied in each layer's epilogue); only the chunk statistics it needs come from the chunk's
 * encoding moments through the float64 layer algebra above -- exact because every LeakyReLU(True) is the identity
 * (negative_slope = 1, models.py:72,92).  Running stats are updated chunk by chunk as nn.BatchNorm1d does.  `state`:
 * pcnerf_nof_train_fused_bytes(total_samples, chunk) bytes of scratch (the fold's forward pieces only: no
 * backward state). */
size_t pcnerf_nof_train_fused_bytes(int64_t total_samples, int64_t chunk);
int pcnerf_nof_query_train_fused(const float* rays, int64_t n_rays, int ray_stride, const float* z, int n_samples,
                                 int64_t chunk, const pcnerf_nof_params* params, float momentum, float eps,
                                 void* state, size_t state_bytes, float* p_out, void* stream);
/* The same query writing chunks 0..store_chunks-1 into an activation store (pcnerf_nof_store_bytes(chunk) bytes per
 * chunk, the layout pcnerf_nof_query_train_store writes: raw layer outputs W_L x and BatchNorm sums) for
 * pcnerf_nof_query_train_backward_fused (or _store).  Here `state` is pcnerf_nof_train_fold_bytes(total_samples,
 * chunk) bytes and must stay untouched until that backward: it holds the chunks' encoding moments and layer maps. */
int pcnerf_nof_query_train_fused_store(const float* rays, int64_t n_rays, int ray_stride, const float* z,
                                       int n_samples, int64_t chunk, const pcnerf_nof_params* params, float momentum,
                                       float eps, void* state, size_t state_bytes, float* p_out, void* store,
                                       int64_t store_chunks, void* stream);
/* The training backward after pcnerf_nof_query_train_fused_store (the autograd of render.py:47-50 / models.py:183-203
 * in train_kitti.py:155's loss.backward(), as pcnerf_nof_query_train_backward): `state` is that forward's state.
 * Each stored chunk's layers run ONE pass each (data gradient, BatchNorm backward and weight gradient together,
 * g_{L-1} written over h_{L-1} in the store, which the call CONSUMES: a second backward on the same store would read
 * gradients as activations -- recompute instead); the BatchNorm-backward statistics per chunk
 * come from the state (the chunk's encoding and gradient moments, float64).  Chunks beyond store_chunks are
 * recomputed and take the two-pass backward.  Gradients are ADDED to `grads`. */
int pcnerf_nof_query_train_backward_fused(const float* rays, int64_t n_rays, int ray_stride, const float* z,
                                          int n_samples, int64_t chunk, const pcnerf_nof_params* params, float eps,
                                          const float* grad_logit, void* state, size_t state_bytes, void* workspace,
                                          size_t workspace_bytes, const pcnerf_nof_grads* grads, void* store,
                                          int64_t store_chunks, void* stream);
/* Data-parallel BatchNorm running statistics (replaces, for DP training, the per-process running-stat update of
 * nn.BatchNorm1d in train mode, models.py:183-203 under render.py:47-50's chunk loop; Lightning's DDP leaves them
 * per rank).  pcnerf_nof_train_bn_stats: each chunk's batch statistics of a fused / fold train query (or embedded
 * forward) read from its `state` right after the forward -- out [C][8][2][256] doubles, C = ceil(total / chunk):
 * the mean of h_L (bias included) and the biased variance.  pcnerf_bn_running_replay: running_mean / running_var of
 * `params` advanced over `n_chunks` such records in order with the forward's own update arithmetic; `ns` (device,
 * int64) holds each chunk's sample count.  nof/bn_sync.py gathers every rank's records and replays them in global
 * chunk order, so every rank ends with the same statistics. */
int pcnerf_nof_train_bn_stats(const void* state, size_t state_bytes, int64_t total_samples, int64_t chunk,
                              double* out, void* stream);
int pcnerf_bn_running_replay(const pcnerf_nof_params* params, float momentum, const double* stats, const int64_t* ns,
                             int64_t n_chunks, void* stream);
/* The training step's forward and backward without any activation store (the default training path since round 5;
 * replaces the autograd of render.py:47-50 / models.py:183-203 that train_kitti.py:155's loss.backward() runs).
 * pcnerf_nof_query_train_fused_state: the fused query above, keeping its `state` (pcnerf_nof_train_fold_bytes
 * (total_samples, chunk) bytes: the chunks' encoding moments and layer maps) for the backward; nothing else is
 * written.  pcnerf_nof_query_train_backward_remat: every chunk's layers in ONE pass each (data gradient, BatchNorm
 * backward, weight gradient), each layer's input h_{L-1} - mean rematerialised per tile from the chunk's encoding
 * through its exact layer map P'_{L-1} (identity activations, models.py:72: the premise of the statistics); `state`
 * is consumed (its Sigma products are overwritten), `workspace` is pcnerf_nof_backward_workspace_bytes(chunk) bytes;
 * train math 1 (f16x2_3) only.  Gradients are ADDED to `grads`. */
int pcnerf_nof_query_train_fused_state(const float* rays, int64_t n_rays, int ray_stride, const float* z,
                                       int n_samples, int64_t chunk, const pcnerf_nof_params* params, float momentum,
                                       float eps, void* state, size_t state_bytes, float* p_out, void* stream);
int pcnerf_nof_query_train_backward_remat(const float* rays, int64_t n_rays, int ray_stride, const float* z,
                                          int n_samples, int64_t chunk, const pcnerf_nof_params* params, float eps,
                                          const float* grad_logit, void* state, size_t state_bytes, void* workspace,
                                          size_t workspace_bytes, const pcnerf_nof_grads* grads, void* stream);
/* NOF.forward(emb) in train mode on an embedded batch of n rows (one chunk), the same way. */
int pcnerf_nof_forward_train_fused(const float* emb, int64_t n, const pcnerf_nof_params* params, float momentum,
                                   float eps, void* state, size_t state_bytes, float* p_out, void* stream);
/* NOF.forward(emb) through the fold (one chunk of n rows); grad_p = dL/dp of its output p. */
int pcnerf_nof_forward_train_fold_backward(const float* emb, int64_t n, const pcnerf_nof_params* params, float eps,
                                           const float* p, const float* grad_p, void* state, size_t state_bytes,
                                           const pcnerf_nof_grads* grads, void* stream);

/* ---------------------------------------------------------------- sampling (render.py:429-454, :497-511)
 * z[ray, :] = linspace sampling of [rays[near_col], rays[far_col]] with n_samples points; if
 * n_parent < n_samples the segmented scheme is used: n_parent points over [near, far] and
 * n_samples - n_parent over [rays[child_near_col], rays[child_far_col]], merged by sort.  disparity != 0:
 * linear in inverse depth, z = 1/(1/near*(1-s) + 1/far*s) (render.py:565-567, use_disp). */
int pcnerf_sample_coarse(const float* rays, int64_t n_rays, int ray_stride, int near_col, int far_col,
                         int child_near_col, int child_far_col, int n_samples, int n_parent, int disparity, float* z,
                         void* stream);
/* Stratified perturbation z' = lower + (upper - lower) * (perturb * rand) (render.py:449-454). */
int pcnerf_perturb(const float* z, int64_t n_rays, int n_samples, float perturb, const float* rand, float* z_out,
                   void* stream);

/* The compositing kernels' ray group, process-wide; returns the previous setting, or -1 for an invalid one.
 * 0 (default): a whole 256-thread workgroup per ray when the batch has fewer than 2,048 rays of >= 512 samples (the
 * reference shell's 256 rays x 2,304 fine samples: all CUs busy, 9 samples per thread), one wave per ray otherwise;
 * 64 / 256 force either (A/B, tests).  Same results: every sum and scan runs in float64 and rounds once. */
int pcnerf_set_composite_group(int group);

/* ---------------------------------------------------------------- compositing + child losses
 * (render.py:51-61 and :75-159).  Per ray: w = p * cumprod(1-p) (+ noise_std*noise if noise != NULL),
 * w /= sum(w) + eps; depth = sum(w z).  If `rays` != NULL, also the child masks (inclusive, expansion
 * from 0 and from 2 m by 0.01 steps) and the per-ray loss terms:
 *   free_ray[r] = sum_s (w * !M0)^2,   sl1_ray[r] = SmoothL1(10 * depth_child, 10 * range). */
int pcnerf_composite(const float* p, const float* z, int64_t n_rays, int n_samples, const float* noise,
                     float noise_std, float eps, const float* rays, int ray_stride, int child_near_col,
                     int child_far_col, int range_col, float* weights, float* depth, float* free_ray,
                     float* sl1_ray, double* opac_row, float* depth2, void* stream);
/* (opac_row, nullable: per-ray sum of log(0.1+p)+log(1.1-p)+2.20727, render.py:224; depth2, nullable: z at the
 * rank of the last sample in the descending weight order, render.py:598-600.) */
/* depth2's order of equal weights (render.py:598 argsort(descending=True)): 0 (default) = stable, as torch sorts
 * these rows on the GPU where the reference runs render_rays (rows > 32 long: merge / radix sort); 1 = torch CPU's
 * std::sort (introsort) order, reproduced per tied row (at most 2048 samples per ray; checked before any launch). */
int pcnerf_set_depth2_order(int order);
/* mean = sum(x[0:n]) / denom, one float written to out (used for the opacity means). */
int pcnerf_mean_f64(const double* x, int64_t n, double denom, float* out, void* stream);

/* Backward of pcnerf_composite + the child losses (render.py:51-61, 75-159) to the occupancy logits:
 * grad_logit[r, s] = dL/d logit(p[r, s]) given grad_depth[r] = dL/d depth[r] (nullable = 0) and the device
 * scalars grad_free_loss = dL/d child_free_loss, grad_depth_loss = dL/d child_depth_loss (nullable = 0;
 * ignored when rays == NULL).  sub_nerf_test_num > 0 selects the divide branch (child ids in
 * rays[:, child_id_col]); `workspace` then needs pcnerf_composite_backward_workspace_bytes(sub_nerf_test_num).
 * The weights are not differentiated through sample_pdf (render.py:466 detaches the fine samples). */
size_t pcnerf_composite_backward_workspace_bytes(int sub_nerf_test_num);
int pcnerf_composite_backward(const float* p, const float* z, int64_t n_rays, int n_samples, const float* noise,
                              float noise_std, float eps, const float* rays, int ray_stride, int child_near_col,
                              int child_far_col, int range_col, int child_id_col, int sub_nerf_test_num,
                              const float* grad_depth, const float* grad_free_loss, const float* grad_depth_loss,
                              void* workspace, float* grad_logit, void* stream);

/* ---------------------------------------------------------------- importance resampling
 * z_fine[ray, :] = sort(cat(z, sample_pdf(mid(z), weights[:, 1:-1], n_importance, det = (u == NULL))))
 * (render.py:371-412, :463-467).  `u` [n_rays, n_importance] replaces torch.rand when not NULL. */
int pcnerf_resample(const float* z, const float* weights, int64_t n_rays, int n_samples, int n_importance,
                    const float* u, float* z_fine, void* stream);

/* Standalone sample_pdf(bins (R, n_bins), weights (R, n_bins-1), n_samples, det = (u == NULL)) -> out
 * (R, n_samples), unsorted (render.py:371-412). */
int pcnerf_sample_pdf(const float* bins, const float* weights, int64_t n_rays, int n_bins, int n_samples,
                      const float* u, float* out, void* stream);

/* ---------------------------------------------------------------- losses
 * Child free / depth losses from the per-ray terms (render.py:102-159).  sub_nerf_test_num == 0 selects
 * the plain branch (sum / n_rays, 0.1/n_rays * mean); > 0 the per-child "divide" branch over child ids
 * 1..sub_nerf_test_num read from child_id[r * id_stride].  out[0] = free loss, out[1] = depth loss.
 * `workspace` needs pcnerf_child_loss_workspace_bytes(sub_nerf_test_num) bytes. */
size_t pcnerf_child_loss_workspace_bytes(int sub_nerf_test_num);
int pcnerf_child_loss_reduce(const float* free_ray, const float* sl1_ray, int64_t n_rays, const float* child_id,
                             int id_stride, int sub_nerf_test_num, void* workspace, float* out, void* stream);

/* mean(loss(pred, target)) over elements where mask != 0 (mask may be NULL); kind 0 = MSE, 1 = L1,
 * 2 = SmoothL1(beta 1) (nof/criteria/loss.py:12-50 with nn.*Loss(reduction='mean')).  out: one float. */
int pcnerf_pointwise_loss(const float* pred, const float* target, const uint8_t* mask, int64_t n, int kind,
                          float* out, void* stream);
/* Its backward: grad_pred[i] = grad_out * d loss_i / d pred_i / count (0 where mask == 0); grad_out is a
 * device scalar. */
int pcnerf_pointwise_loss_backward(const float* pred, const float* target, const uint8_t* mask, int64_t n, int kind,
                                   const float* grad_out, float* grad_pred, void* stream);

/* Per-child range loss, the use_child_nerf_divide branch of train_kitti.py:125-142 (replaces its Python loop over
 * sub_nerf_test_num children): out = sum over child ids c in 1..N owning >= 1 ray of
 * post_scale * mean_{i in c} loss(pre_scale*pred_i, pre_scale*target_i) (the reference: pre 10, post 0.1*lambda).
 * Child ids are read from child_id[i * id_stride] (ray column 9).  The backward needs the forward's workspace
 * (per-child sums and counts, pcnerf_child_range_loss_workspace_bytes) unchanged; grad_out is a device scalar. */
size_t pcnerf_child_range_loss_workspace_bytes(int sub_nerf_test_num);
int pcnerf_child_range_loss(const float* pred, const float* target, int64_t n, const float* child_id, int id_stride,
                            int sub_nerf_test_num, int kind, float pre_scale, float post_scale, void* workspace,
                            float* out, void* stream);
int pcnerf_child_range_loss_backward(const float* pred, const float* target, int64_t n, const float* child_id,
                                     int id_stride, int sub_nerf_test_num, int kind, float pre_scale, float post_scale,
                                     const void* workspace, const float* grad_out, float* grad_pred, void* stream);

/* ---------------------------------------------------------------- two-step inference (render_rays_view_0525_2_2)
 * Per row (render.py:241-354 after the query): weights = composite(p) normalised with eps, the strict child
 * mask [rows[child_near_col], rows[child_far_col]] expanded from 0.01 by 0.01, the argmax of the weights
 * smoothed by `gauss` (2*radius+1 float64 taps = scipy gaussian_filter(sigma=5), reflect), at_peak = mask at
 * that argmax, child_sum = sum(w * mask), depth (method 2: child re-normalised, else sum(w z)), the per-row
 * opacity sum and points = o + depth * d (points may be NULL, weights may be NULL). */
int pcnerf_view_rows(const float* p, const float* z, int64_t n_rows, int n_samples, const float* rows, int row_stride,
                     int child_near_col, int child_far_col, int method, float eps, const double* gauss, int radius,
                     float* weights, float* depth, uint8_t* at_peak, float* child_sum, double* opac_row,
                     float* points, void* stream);
/* Ray-group walk (render.py:317-340) over other_interest_sub_nerf_number (int64, k-1 on a group's first row):
 * flags[r] = 1 for the effective row of every group; *opacity = mean opacity term over n_rows * n_samples. */
size_t pcnerf_view_walk_workspace_bytes(int64_t n_rows);
int pcnerf_view_walk(const int64_t* other, int64_t n_rows, const uint8_t* at_peak, const float* child_sum,
                     const double* opac_row, int n_samples, void* workspace, uint8_t* flags, float* opacity,
                     void* stream);

/* ---------------------------------------------------------------- ray tables (ray/AABB intersection)
 * float64 inputs: points (n,3) and origin (3) of one LiDAR frame in the block frame, child boxes as bounds6
 * (C,6) = [xmin,ymin,zmin,xmax,ymax,zmax] (already grown by 0.025), centers (C,3), parent6 (6) the parent block.
 * Train/val 15-column rows (nof/dataset/ipb2dmapping.py:736-768): rows needs n_points*15 floats; the row count
 * is written to *n_rows (device int64).  face_rule 0 = compute_far_bound0606 (KITTI, :119-172: min/max of every
 * face hit, rays that hit no face are dropped); 1 = compute_far_bound0406 (MaiCity, :82-114, :383-395: the first
 * two hits, every point in a child box yields a row; rays with fewer than two hits -- the reference's IndexError
 * -- are counted in *n_short, a device int, so the caller can raise). */
size_t pcnerf_rays_workspace_bytes(int64_t n_points);
int pcnerf_build_train_rays(const double* points, int64_t n_points, const double* origin, const double* centers,
                            const double* bounds6, int64_t n_children, const double* parent6, double surface_expand,
                            int face_rule, void* workspace, float* rows, int64_t* n_rows, int* n_short,
                            void* stream);
/* Two-step 13-column rows grouped per ray (eval_kitti_render.py:675-803; method 2 = every child hit, method 1 =
 * first hit with parent bounds): count pass (writes *n_rows, device int64) then emit pass with the same workspace;
 * rule 0 = KITTI (expansion step 0.05, column 10 = max(parent far, child far)), 1 = MaiCity (multi_frame_maicity,
 * eval_kitti_render.py:344-431: step 0.005, column 10 = parent far; pass its child boxes grown by 0.025);
 * ranges (M), other_interest_sub_nerf_number (M, int64), true_in (M, bool). */
int pcnerf_count_view_rows(const double* points, int64_t n_points, const double* origin, const double* bounds6,
                           int64_t n_children, const double* parent6, int method, int rule, void* workspace,
                           int64_t* n_rows, void* stream);
int pcnerf_emit_view_rows(const double* points, int64_t n_points, const double* origin, const double* bounds6,
                          int64_t n_children, const double* parent6, int method, int rule, void* workspace,
                          float* rows, float* ranges, int64_t* other, uint8_t* true_in, void* stream);

/* ---------------------------------------------------------------- evaluation metrics
 * (nof/criteria/pointcloud_metrics.py:5-49, logs/.../render_result/print_metrics.py:31-133; exhaustive float64
 * nearest-neighbour search instead of open3d's KD-tree).  Clouds are (n, 3) float32 rows.
 * pcnerf_nn_distance: dist[i] = min_j |query[i] - ref[j]| (float64).
 * pcnerf_eval_pts: out = {cd, fscore, precision, recall} of eval_pts(pred, gt, threshold): precision over the
 *   gt points' nearest-pred distances, recall over the pred points' nearest-gt distances, cd = sum of the two
 *   means; `workspace` needs pcnerf_eval_pts_workspace_bytes(n_pred, n_gt) bytes.  out is device memory.
 * pcnerf_range_metrics: out = {sum |r_pred - r_gt|, count(|.| < threshold)} with ranges from `origin` (3 floats)
 *   over n aligned points (abs_error / acc_thres before the division by n). */
int pcnerf_nn_distance(const float* ref, int64_t n_ref, const float* query, int64_t n_query, double* dist,
                       void* stream);
size_t pcnerf_eval_pts_workspace_bytes(int64_t n_pred, int64_t n_gt);
int pcnerf_eval_pts(const float* pred, int64_t n_pred, const float* gt, int64_t n_gt, double threshold,
                    void* workspace, double* out, void* stream);
int pcnerf_range_metrics(const float* pred, const float* gt, const float* origin, int64_t n, double threshold,
                         double* out, void* stream);

/* ---------------------------------------------------------------- kernel timing (bench / profiling)
 * pcnerf_prof_enable(1) makes every subsequent launch record a HIP event pair on its stream; tags:
 * 0 eval query, 1 train hidden Linear, 2 train first Linear, 3 train skip Linear, 4 train occ_out,
 * 5 BN fold, 6 composite, 7 resample, 8 sampling, 9 composite backward, 10 weight-gradient GEMM,
 * 11 data-gradient GEMM, 12 other backward kernels, 13 eval/train fold per-sample query, 14 split-math weight
 * gradients, 15 fused first layers, 16 train-fold moments, 17 train-fold layer algebra.  pcnerf_prof_read synchronises the tag's events and returns
 * the summed duration, launch count and algorithmic FLOPs / bytes of those launches. */
int pcnerf_prof_enable(int on);
int pcnerf_prof_read(int tag, double* total_ms, int64_t* launches, double* flops, double* bytes);

/* What the fp16 matrix pipe sustains on this board: the headline query's instruction (v_mfma_f32_16x16x32_f16, B
 * operands from LDS, one wave per SIMD, 24 accumulators per wave) in a bare loop on random operands, launched back
 * to back for `seconds` (settle for the first half, timed with HIP events over the second).  *tflops = dense fp16
 * TFLOP/s, *clock_mhz = median shader clock of the timed launches.  No reference counterpart (measurement only). */
int pcnerf_mfma_ceiling(double seconds, double* tflops, double* clock_mhz, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* PCNERF_HIP_H */
