/*
 * gr_amd.h — C ABI of the MI355X (gfx950) hot-path library libgr_amd.so.
 *
 * The reference (CatchMan1/AI-education-generative-recommendation) has no native layer: its hot
 * paths are sequences of ATen ops inside two nn.Modules.  This ABI is what those modules' methods
 * bottom out in here; each entry point names the reference code it replaces (paths relative to the
 * reference root).  The Python drop-in modules (RQVAE, SASRec) bind these through ctypes.
 *
 * Conventions
 *  - Every pointer argument named x/w/z/... is a DEVICE pointer to contiguous row-major data in the
 *    layout PyTorch uses (nn.Linear weight = [out, in], nn.Embedding weight = [rows, dim]).
 *    Arguments documented as "host array" are host arrays OF device pointers / sizes.
 *  - All work is enqueued on `stream` (a hipStream_t; NULL = the default stream).  No call
 *    synchronises, allocates or frees device memory: scratch comes from the caller's workspace
 *    (size from the matching *_workspace_bytes query).  Calls are reentrant and stateless.
 *  - Return 0 (GR_OK) on success, a negative GR_ERR_* code otherwise; gr_last_error() returns a
 *    thread-local message for the last failure on the calling thread.  No exceptions cross the ABI.
 *  - Floating point is fp32 throughout (f32-input MFMA, f32 accumulate); indices are int64.
 */
#ifndef GR_AMD_H
#define GR_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GR_OK 0
#define GR_ERR_ARG (-1)          /* bad shape / null pointer / misalignment                   */
#define GR_ERR_UNSUPPORTED (-2)  /* shape outside what the kernels are built for               */
#define GR_ERR_HIP (-3)          /* a HIP runtime error at launch                              */
#define GR_ERR_WORKSPACE (-4)    /* workspace too small                                        */

#define GR_MAX_LEVELS 8          /* RQ levels supported by one gr_rq_* call                    */
#define GR_MAX_LINEAR 8          /* encoder Linear layers supported by gr_rq_encode_f32        */

#define GR_ACT_NONE 0
#define GR_ACT_RELU 1
#define GR_ACT_SIGMOID 2         /* the activations of RQ-VAE/models/layers.py:45-67 besides   */
#define GR_ACT_TANH 3            /* ReLU (nn.Sigmoid / nn.Tanh / nn.LeakyReLU(0.01)); gr_linear */
#define GR_ACT_LEAKYRELU 4       /* only, without a residual                                     */

/* Library identification ("gr_amd <version> gfx950"). */
const char* gr_version(void);
/* Message of the last failed call on this thread ("" if none). */
const char* gr_last_error(void);
/* Process-wide path switches (no reference counterpart).  Each selects between two kernel paths
 * that give BITWISE identical results, so the tests can run both; no option changes numerics, and
 * the defaults are what every caller wants.  (Round 5 removed the A/B knobs of slower variants and
 * the two numerics-changing ones: the final SASRec block of a last-position forward always runs
 * the H form below.)
 *   "rq_fused"      1 (default): gr_rq_encode_f32 runs the fused persistent kernel when the encoder
 *                   shape is in -> 256 -> 128 -> 32; 0: the layer-wise path (exact gr_linear +
 *                   quantize).
 *   "sas_fused"     2 (default): gr_sasrec_forward_f32 / gr_sasrec_predict_f32 run the fused
 *                   register-resident forward kernel when n <= 64, d <= 64 (d and the head width
 *                   multiples of 8), mlp <= 128, num_blocks <= 8: one wave per sequence, or two
 *                   (one per 32-token tile) when n > 32 and the batch size favours it; 3: two
 *                   waves whenever n > 32; 1: always one; 0: the layer-wise pipeline (the
 *                   workspace query follows the option in force when it is called).  The fused
 *                   forms give bitwise the same results.
 *   "sas_rowtile"   1 (default): d = 128 forwards on the row-tile kernels; 0: one kernel per op.
 *   "lin_wres"      1 (default): gr_linear_f32 with k = 128, n % 128 == 0, no residual and
 *                   m >= 96 x 256 runs a persistent kernel that keeps each wave's 32 columns of w in
 *                   registers (the C5 block-0 in-projection); 0: the tiled kernel.
 *   "emb_proj"      1 (default): the d = 128 forward's block 0 (embedding gather + LN_a0 +
 *                   in-projection) runs as one persistent kernel with W_in in registers; 0: the
 *                   embed_ln kernel then gr_linear_f32.
 *   "topk_half"     2 (default): gr_score_topk_f32's tile pass records the max of every 16-row
 *                   half tile when the catalog is below ~3,700 64-row chunks per 128 features (the
 *                   select kernel then re-scores half as many rows), else of every 32-row tile;
 *                   1: always half tiles; 0: never.
 *   "attn_k16"      1 (default): head width 128 attention on 32-query tiles over 16-key steps at
 *                   two waves per SIMD; 0: 32 x 32 steps at one wave per SIMD.  Different fp32
 *                   chains of the same attention (both within the logits tolerance).
 * A last-position forward (predict, last_hidden) runs its final block as the one-query tail on
 * LN_a(X): q . K_j = (W_k^T q) . H_j (+ a term constant over j that cancels in the softmax) and
 * p . V = W_v (p . H) + b_v, so K|V of the B n rows are never projected (sas_tail_h2_kernel; the
 * fused d <= 64 kernel likewise).  The reassociated sums round differently from the reference
 * formulation: logits within the 1e-5 row-scaled tolerance (tests/test_sasrec_gpu.py::
 * test_tail_h_form_vs_full_block_and_oracle).
 * gr_set_option returns GR_ERR_ARG for an unknown name/value; gr_get_option returns -1 for an
 * unknown name. */
int gr_set_option(const char* name, int64_t value);
int64_t gr_get_option(const char* name);

/* ------------------------------------------------------------------------------------------ */
/* Dense layer  y[m, n] = act(x[m, k] . w[n, k]^T + bias[n]) (+ residual[m, n])
 * Replaces nn.Linear -> F.linear -> addmm (+ nn.ReLU): RQ-VAE/models/layers.py:23-30 (encoder),
 * SASRec/model.py:37-45 (FFN), torch functional.py:5785-5830 / :6600 (MHA in/out projections) and
 * SASRec/model.py:107 (scoring: w = item table, bias = NULL).
 * bias, residual may be NULL.  `residual` may alias `y` (in-place residual add).  act: GR_ACT_*
 * (SIGMOID / TANH / LEAKYRELU only with residual = NULL).
 * Requires k % 4 == 0 and 16-byte aligned x, w.  ldy / ldr are row strides (elements) of y / residual. */
int gr_linear_f32(const float* x, int64_t m, int32_t k, const float* w, int32_t n,
                  const float* bias, const float* residual, int64_t ldr, int32_t act,
                  float* y, int64_t ldy, void* stream);

/* ------------------------------------------------------------------------------------------ */
/* RQ-VAE encode.
 * Squared norms of codebook rows, cn[c] = sum_k C[c,k]^2 (the `torch.sum(self.embedding.weight**2,
 * dim=1)` term of RQ-VAE/models/vq.py:72), computed once per codebook. */
int gr_rq_codebook_norms_f32(const float* codebook, int32_t K, int32_t e, float* cn_out, void* stream);

/* Residual quantization of latents z[n, e] over L levels (RQ-VAE/models/rq.py:39-56 with
 * VectorQuantizer.forward(use_sk=False), vq.py:63-99):
 *   d = (||r||^2 + ||C_l||^2) - 2 r.C_l^T ;  idx = first argmin ;  r <- r - (r + (C_l[idx] - r))
 * Every fp32 rounding is the reference's CPU one (r.C: one fma chain over k in order, as MKL's
 * sgemm at K = e; the squared norms in ATen's vectorised row-sum order; oracle/rq_exact.c), so
 * idx_out equals the reference's, exact ties included.
 * K, codebooks: host arrays of length L.  code_norms: accepted for ABI stability and ignored (may be
 * NULL); the kernel recomputes each code's norm from its LDS copy of the codebook.
 * idx_out[n, L] int64 row-major (the stacked `indices` of rq.py:54).
 * best_out[n, L], gap_out[n, L] (optional, may be NULL): the best fp32 distance and the gap to the
 * second best per level.
 * Supports 1 <= e <= 4096 (e > 64 and one-row calls on the per-row kernel), 1 <= L <= GR_MAX_LEVELS,
 * any K >= 1; z and the codebooks must be 16-byte aligned when e is 16, 32 or 64. */
int gr_rq_quantize_f32(const float* z, int64_t n, int32_t e, int32_t L, const int32_t* K,
                       const float* const* codebooks, const float* const* code_norms,
                       int64_t* idx_out, float* best_out, float* gap_out, void* stream);

/* Workspace for gr_rq_encode_f32 (bytes).  dims: host array of n_linear+1 layer widths
 * (in_dim, hidden..., e_dim) = RQVAE.encode_layer_dims (RQ-VAE/models/rqvae.py:45). */
size_t gr_rq_encode_workspace_bytes(int64_t n, int32_t n_linear, const int32_t* dims,
                                    int32_t L, const int32_t* K);

/* RQVAE.get_indices(xs, use_sk=False) (RQ-VAE/models/rqvae.py:67-71): encoder MLP
 * (layers.py:42-43; ReLU after every Linear but the last) followed by gr_rq_quantize_f32.
 * The encoder and the quantizer's r . c reproduce the reference's CPU sgemm order for a call of n
 * rows (gr_mkl_plan: k-block chains of >= 16-row calls on the MFMA kernels, the one-row and 2-15-row
 * 16-lane orders on a per-row kernel; widths whose order is not pinned, in_features % 4 != 0 and
 * e_dim > 64 also run there); any width is accepted. 
 * weights/biases: host arrays (n_linear) of device pointers; codebooks, K: host arrays (L).
 * best_out, gap_out: as gr_rq_quantize_f32 (optional).
 * z_out (optional, may be NULL): the encoder output [n, e]. */
int gr_rq_encode_f32(const float* x, int64_t n, int32_t n_linear, const int32_t* dims,
                     const float* const* weights, const float* const* biases, int32_t L,
                     const int32_t* K, const float* const* codebooks, int64_t* idx_out,
                     float* best_out, float* gap_out, float* z_out, void* workspace,
                     size_t workspace_bytes, void* stream);

/* The fused encoder's packed weight image (in -> 256 -> 128 -> 32 encoders; 0 floats otherwise):
 * W1 / W2 with every 32-deep k group in the order the 32x32x2 MFMA chains consume (feature
 * 8j + 2s + h at 16h + 4j + s), W3 in the 16x16x4 chain's (feature 4t + g of a 16-block at 4g + t).
 * gr_rq_encode_f32 writes it into its workspace on every call; a caller that keeps the weights
 * fixed between calls packs once (gr_rq_encoder_pack_f32, `packed` 16-byte aligned) and passes it
 * to gr_rq_encode_packed_f32 (same arguments as gr_rq_encode_f32 otherwise; packed = NULL: pack
 * per call), which saves a launch per call. */
size_t gr_rq_encoder_pack_floats(int32_t n_linear, const int32_t* dims);
int gr_rq_encoder_pack_f32(int32_t n_linear, const int32_t* dims, const float* const* weights,
                           float* packed, void* stream);
int gr_rq_encode_packed_f32(const float* x, int64_t n, int32_t n_linear, const int32_t* dims,
                            const float* const* weights, const float* const* biases,
                            const float* packed, int32_t L, const int32_t* K,
                            const float* const* codebooks, int64_t* idx_out, float* best_out,
                            float* gap_out, float* z_out, void* workspace, size_t workspace_bytes,
                            void* stream);

/* MLPLayers.forward in eval mode (RQ-VAE/models/layers.py:42-43): z_out[n, dims[n_linear]] = the
 * encoder output alone (ReLU after every Linear but the last).  Same kernels as gr_rq_encode_f32. */
size_t gr_rq_mlp_workspace_bytes(int64_t n, int32_t n_linear, const int32_t* dims);
int gr_rq_mlp_f32(const float* x, int64_t n, int32_t n_linear, const int32_t* dims,
                  const float* const* weights, const float* const* biases, float* z_out,
                  void* workspace, size_t workspace_bytes, void* stream);

/* MLPLayers.forward in eval mode with the general layer options of RQ-VAE/models/layers.py:18-43,
 * in the reference's exact CPU order: per layer Linear, then (all but the last) an eval
 * BatchNorm1d when bn_mean / bn_var are given (host arrays of n_linear - 1 device pointers; bn_w /
 * bn_b may be NULL arrays = affine off; torch's CPU formula a = w / sqrt(var + eps),
 * y = fma(y, a, fma(-mean, a, b))) and act (GR_ACT_RELU / GR_ACT_LEAKYRELU / GR_ACT_NONE).
 * Workspace: gr_rq_mlp_workspace_bytes. */
int gr_mlp_exact_f32(const float* x, int64_t n, int32_t n_linear, const int32_t* dims,
                     const float* const* weights, const float* const* biases,
                     const float* const* bn_mean, const float* const* bn_var,
                     const float* const* bn_w, const float* const* bn_b, float bn_eps,
                     int32_t act, float* z_out, void* workspace, size_t workspace_bytes,
                     void* stream);

/* MLPLayers.forward (eval) for consecutive row groups, each ONE reference call with its own MKL
 * accumulation order (the call's row count selects it, see gr_mkl_plan): the encoder half of
 * RQVAE.get_indices(group, use_sk=True) per collision group (RQ-VAE/infer.py:116-127).  group_ptr:
 * device int64 [n_groups + 1] offsets as gr_rq_encode_sk_f32.  Other arguments as gr_mlp_exact_f32
 * (no workspace). */
int gr_mlp_exact_groups_f32(const float* x, int64_t n, int32_t n_linear, const int32_t* dims,
                            const float* const* weights, const float* const* biases,
                            const float* const* bn_mean, const float* const* bn_var,
                            const float* const* bn_w, const float* const* bn_b, float bn_eps,
                            int32_t act, const int64_t* group_ptr, int64_t n_groups, float* z_out,
                            void* stream);

/* The accumulation order the reference's CPU sgemm (torch 2.10 / MKL 2024.2, 8 threads, AVX-512:
 * the golden-fixture host) uses for ONE call of M rows, inner size K, N outputs -- nn.Linear
 * (RQ-VAE/models/layers.py:23) and the quantizer's matmul (vq.py:73, K = e_dim, N = codebook size):
 *   *kind 0 = k-block chain of width *kb, 1 = one-row 16-lane gemv, 2 = 2-15-row 16-lane small
 * kernel (oracle/rq_exact.c rqx_plan).  Every gr_rq_* / gr_mlp_* entry point computes each call in
 * this order.  Returns 1 when (M, K, N) lies in the envelope checked bit for bit against torch on
 * that host, 0 outside it (the order is then mkl_plan's best restatement, parity unpinned). */
int32_t gr_mkl_plan(int64_t M, int32_t K, int32_t N, int32_t* kind, int32_t* kb);

/* MLPLayers.forward in train mode (RQ-VAE/models/layers.py:18-43, [Dropout -> Linear -> ReLU] x
 * (n_linear - 1), then Dropout -> Linear; RQVAE.forward under RQ-VAE/train.py:113).  Dropout p_drop
 * on every layer input, masks from a counter-based hash of (*seed_dev, layer, element) -- torch's
 * distribution, not its random stream (seed_dev and xd0 may be null when p_drop = 0).  Outputs:
 * xd0[M, dims[0]] = the dropped input (p_drop > 0), outs[i][M, dims[i+1]] = the next layer's dropped
 * input drop(relu(X_i W_i^T + b_i)) for i < n_linear - 1 and the MLP output for the last layer --
 * the tensors the backward reads. */
int gr_mlp_train_fwd_f32(const float* x, int64_t M, int32_t n_linear, const int32_t* dims,
                         const float* const* weights, const float* const* biases, float p_drop,
                         const uint64_t* seed_dev, float* xd0, float* const* outs, void* stream);

/* Backward of layer i of such an MLP (the autograd of layers.py's Linear / ReLU / Dropout,
 * train.py:116), one launch, on the layer's dropped input xd_in (xd0, or outs[i-1] of the forward):
 * dweight[N, K] = dz^T xd_in, dbias[N] = column sums of dz (rows in order), and (dx_out non-null)
 * dx_out[M, K] = (dz W) * mask, mask per dx_mode: 1 = (xd_in > 0 ? 1 / (1 - p) : 0) (the input came
 * through ReLU: ReLU' and dropout), 2 = the dropout hash mask of `site` (the first layer), 0 = none.
 * dz[M, N] is the gradient of this layer's pre-activation output. */
int gr_mlp_train_bwd_layer_f32(const float* xd_in, int64_t M, int32_t K, const float* weight, int32_t N,
                               const float* dz, int32_t dx_mode, float p_drop, const uint64_t* seed_dev,
                               int32_t site, float* dweight, float* dbias, float* dx_out, void* stream);

/* RQVAE.get_indices(xs, use_sk=True) over independent row groups (the collision re-encode of
 * RQ-VAE/infer.py:108-130; vq.py:52-61, 76-84; layers.py:85-108).  z[n, e]: encoder outputs (as
 * gr_rq_encode_f32's z_out), rows grouped contiguously: group g = rows [group_ptr[g],
 * group_ptr[g+1]) (device int64 array of n_groups + 1, group_ptr[0] = 0, group_ptr[n_groups] = n).
 * Each group is one reference call: a level with sk_eps[l] > 0 (host array, float64) assigns by
 * sk_iters Sinkhorn iterations over the group's [rows, K] distances (batch-coupled), a level with
 * sk_eps[l] <= 0 by the plain argmin.  idx_out[n, L] int64.  K[l] <= 1024. */
size_t gr_rq_encode_sk_workspace_bytes(int64_t n, int32_t e, int32_t L, const int32_t* K);
int gr_rq_encode_sk_f32(const float* z, int64_t n, int32_t e, int32_t L, const int32_t* K,
                        const float* const* codebooks, const double* sk_eps, int32_t sk_iters,
                        const int64_t* group_ptr, int64_t n_groups, int64_t* idx_out,
                        void* workspace, size_t workspace_bytes, void* stream);

/* The quantizer's training forward (RQ-VAE/models/rq.py:39-56, vq.py:63-99 under
 * RQ-VAE/train.py:113): gr_rq_encode_sk_f32's assignment (one group per call for a training batch)
 * plus, when non-null, xq_out[n, e] = x_q = sum_l (r_l + (C_l[idx_l] - r_l)) and
 * sq_out[n, L] = sum_j (C_l[idx_l] - r_l)^2 per row and level (the mse numerators).  Same
 * workspace as gr_rq_encode_sk_f32. */
int gr_rq_quantize_sk_train_f32(const float* z, int64_t n, int32_t e, int32_t L, const int32_t* K,
                                const float* const* codebooks, const double* sk_eps, int32_t sk_iters,
                                const int64_t* group_ptr, int64_t n_groups, int64_t* idx_out,
                                float* xq_out, float* sq_out, void* workspace, size_t workspace_bytes,
                                void* stream);

/* Its backward for rq_loss = mean_l(mse(x_q_l, r_l.detach()) + beta * mse(x_q_l.detach(), r_l))
 * (vq.py:88-92) and the straight-through x_q (vq.py:95): dz_out[n, e] = g_xq + g * beta * 2 *
 * (z - C_0[idx_0]) / (n e L) (g_xq may be null: zero), dcodebooks_out[l][K_l, e] =
 * g * 2 / (n e L) * sum over the rows assigned to each code of (C_l[k] - r_l), rows in index order
 * (deterministic).  g_rq: device float scalar, the gradient of rq_loss. */
int gr_rq_quantize_sk_train_bwd_f32(const float* z, int64_t n, int32_t e, int32_t L, const int32_t* K,
                                    const float* const* codebooks, const int64_t* idx, const float* g_xq,
                                    const float* g_rq, float beta, float* dz_out,
                                    float* const* dcodebooks_out, void* stream);

/* ------------------------------------------------------------------------------------------ */
/* SASRec.  Parameters of one model, as device pointers to the tensors of SASRec.state_dict()
 * (SASRec/model.py:17-47).  Per-block fields are host arrays of length n_blocks.  The dead
 * W_Q/W_K/W_V projections (model.py:23-25, 63-65) do not affect any output and are not passed. */
typedef struct gr_sasrec_params {
  int32_t d;            /* hidden size                          params['d']            */
  int32_t n_blocks;     /* params['num_blocks']                                        */
  int32_t n_heads;      /* params['num_heads'] (d % n_heads == 0)                      */
  int32_t mlp;          /* params['mlp_layer']                                         */
  int32_t max_len;      /* rows of pos_emb                      params['max_len']      */
  float eps;            /* params['layernorm_eps']                                     */
  int64_t item_rows;    /* item_num + 1 (row 0 = padding)                              */
  const float* item_emb;          /* [item_rows, d]   item_emb.weight                  */
  const float* pos_emb;           /* [max_len, d]     pos_emb.weight                   */
  const float* const* attn_ln_w;  /* attention_layernorms.{i}.weight  [d]              */
  const float* const* attn_ln_b;  /* attention_layernorms.{i}.bias    [d]              */
  const float* const* in_proj_w;  /* attention_layers.{i}.in_proj_weight  [3d, d]      */
  const float* const* in_proj_b;  /* attention_layers.{i}.in_proj_bias    [3d]         */
  const float* const* out_proj_w; /* attention_layers.{i}.out_proj.weight [d, d]       */
  const float* const* out_proj_b; /* attention_layers.{i}.out_proj.bias   [d]          */
  const float* const* ffn_ln_w;   /* forward_layernorms.{i}.weight  [d]                */
  const float* const* ffn_ln_b;   /* forward_layernorms.{i}.bias    [d]                */
  const float* const* ffn1_w;     /* forward_layers.{i}.0.weight [mlp, d]              */
  const float* const* ffn1_b;     /* forward_layers.{i}.0.bias   [mlp]                 */
  const float* const* ffn2_w;     /* forward_layers.{i}.3.weight [d, mlp]              */
  const float* const* ffn2_b;     /* forward_layers.{i}.3.bias   [d]                   */
  const float* last_ln_w;         /* last_layernorm.weight [d]                         */
  const float* last_ln_b;         /* last_layernorm.bias   [d]                         */
} gr_sasrec_params;

/* Workspace (bytes) for gr_sasrec_forward_f32 / gr_sasrec_predict_f32 at batch B, length n. */
size_t gr_sasrec_workspace_bytes(const gr_sasrec_params* p, int64_t B, int32_t n);

/* SASRec.forward(log_seqs) (SASRec/model.py:49-96) in eval mode: seqs[B, n] int64 ids ->
 * out[B, n, d] (last_only = 0) or only the last position out[B, d] (last_only = 1, the
 * `final_feats[:, -1, :]` of model.py:104).  err_flag (optional device int32, may be NULL) is set
 * to 1 when an id is outside [0, item_rows) (such ids read the zero padding row instead). */
int gr_sasrec_forward_f32(const gr_sasrec_params* p, const int64_t* seqs, int64_t B, int32_t n,
                          float* out, int32_t last_only, void* workspace, size_t workspace_bytes,
                          int32_t* err_flag, void* stream);

/* SASRec.predict(log_seqs) (SASRec/model.py:98-108): logits[B, item_rows] = h_last . item_emb^T. */
int gr_sasrec_predict_f32(const gr_sasrec_params* p, const int64_t* seqs, int64_t B, int32_t n,
                          float* logits, void* workspace, size_t workspace_bytes,
                          int32_t* err_flag, void* stream);

/* Same, logits rows ld floats apart (ld >= item_rows).  SASRec.predict allocates ld = item_rows
 * rounded up to 32 floats, so every row starts on a 128-byte line and the scoring kernel stores
 * whole lines straight from its accumulators; the caller gets the [B, item_rows]
 * view, on which evaluate.py:27-32 (in-place column-0 mask, gather, '>' count) work unchanged. */
int gr_sasrec_predict_ld_f32(const gr_sasrec_params* p, const int64_t* seqs, int64_t B, int32_t n,
                             float* logits, int64_t ld, void* workspace, size_t workspace_bytes,
                             int32_t* err_flag, void* stream);

/* One batch of SASRec/evaluate.py:26-32 in one call, the logits never written: ranks_out[b] =
 * #{j : l[b, j] > l[b, targets[b]]} + 1 with l = predict(seqs) and column 0 taken as -1e9 when
 * mask_col0 (evaluate.py:27) -- the forward's last hidden states, then the target logit and the
 * strict count on the scoring kernel's exact fp32 chain (gr_score_pairs_f32 /
 * gr_score_count_gt_ws_f32 below; bitwise the ranks of the materialised sequence).  d in {16, 32,
 * 64, 128}.  workspace: gr_sasrec_rank_workspace_bytes; count_ws (optional, may be NULL): zero on
 * entry and left zero, gr_score_count_workspace_bytes(B).  err_flag as gr_sasrec_forward_f32 (also
 * set for a target outside [0, item_rows)). */
size_t gr_sasrec_rank_workspace_bytes(const gr_sasrec_params* p, int64_t B, int32_t n);
int gr_sasrec_rank_f32(const gr_sasrec_params* p, const int64_t* seqs, int64_t B, int32_t n,
                       const int64_t* targets, int32_t mask_col0, int64_t* ranks_out, void* workspace,
                       size_t workspace_bytes, void* count_ws, size_t count_ws_bytes, int32_t* err_flag,
                       void* stream);

/* SASRec training, the transformer part of one step (SASRec/train.py:131 `model.forward` in train
 * mode and the backward that `loss.backward()`, train.py:161-172, runs through model.py:49-96).
 * One workgroup per sequence; n <= 64, d <= 64 (d % num_heads == 0), mlp_layer <= 128, <= 8 blocks.
 * Dropout p (params['dropout']) on the attention probabilities, the FFN hidden layer and the FFN
 * output, as nn.MultiheadAttention / nn.Dropout apply it; masks from a counter-based hash keyed by
 * seed ^ *seed_dev (seed_dev optional), the same for the forward and the backward of one step.
 * Buffers (device, caller-allocated, fp32): nb = n_blocks, R = B * n rows (sequence-major). */
typedef struct gr_sasrec_train_bufs {
  float* xin;    /* [nb, R, d]    LN_a input of each block       (written by the forward) */
  float* hs;     /* [nb, R, d]    LN_a output = in-projection input                       */
  float* qkv;    /* [nb, R, 3d]   in-projection output q | k | v                          */
  float* prob;   /* [nb, B, H, n, n] softmax probabilities before dropout                 */
  float* os;     /* [nb, R, d]    attention output = out-projection input                 */
  float* x1;     /* [nb, R, d]    residual after attention = LN_f input                   */
  float* fs;     /* [nb, R, d]    LN_f output = FFN1 input                                */
  float* zs;     /* [nb, R, mlp]  FFN1 output before the ReLU                             */
  float* us;     /* [nb, R, mlp]  dropout(relu(FFN1)) = FFN2 input                        */
  float* xl;     /* [R, d]        last LayerNorm input                                    */
  float* g_vec;  /* [B, gr_sasrec_train_vec_width] (written by the backward) per-sequence partial
                    gradients in SASRec's parameter order: per block [ln_a w, ln_a b, in_proj w
                    (3d x d), in_proj b, out_proj w (d x d), out_proj b, ln_f w, ln_f b, ffn1 w
                    (mlp x d), ffn1 b, ffn2 w (d x mlp), ffn2 b], then [last ln w, last ln b], then
                    pos_emb rows [n, d]; the parameter gradients are its sum over B             */
} gr_sasrec_train_bufs;

/* Floats per sequence in gr_sasrec_train_bufs.g_vec: n_blocks * (4d^2 + 2 d mlp + 9d + mlp) + 2d + n*d. */
int32_t gr_sasrec_train_vec_width(const gr_sasrec_params* p, int32_t n);

/* Train-mode forward: seqs[B, n] -> out[B, n, d] (model.py:49-96 with dropout p), saving the
 * activations in bufs.  err_flag (optional) gets 1 for an id outside [0, item_rows). */
int gr_sasrec_train_fwd_f32(const gr_sasrec_params* p, const int64_t* seqs, int64_t B, int32_t n,
                            float p_drop, uint64_t seed, const uint64_t* seed_dev,
                            const gr_sasrec_train_bufs* bufs, float* out, int32_t* err_flag, void* stream);

/* Backward of the forward above (same seqs, p_drop, seed, bufs): d_out[B, n, d] -> the
 * per-sequence partial gradients in bufs.g_vec (sum over B = every parameter's gradient except
 * the item table's); item-embedding rows are added (atomically) into g_item[item_rows, d]
 * (optional; padding row 0 is left untouched). */
int gr_sasrec_train_bwd_f32(const gr_sasrec_params* p, const int64_t* seqs, int64_t B, int32_t n,
                            float p_drop, uint64_t seed, const uint64_t* seed_dev,
                            const gr_sasrec_train_bufs* bufs, const float* d_out, float* g_item,
                            void* stream);

/* Full-catalog (or catalog-shard) scoring logits[B, rows] = h[B, d] . table[rows, d]^T
 * (SASRec/model.py:107).  ld = row stride of logits. */
int gr_score_f32(const float* h, int64_t B, int32_t d, const float* table, int64_t rows,
                 float* logits, int64_t ld, void* stream);

/* Strict rank of each user's target (SASRec/evaluate.py:27-32) without mutating logits:
 * with column 0 taken as -1e9 (when mask_col0), rank[b] = #{j : l[b,j] > l[b,t_b]} + 1.
 * ld = row stride of logits, cols = number of columns. */
int gr_rank_f32(const float* logits, int64_t B, int64_t cols, int64_t ld, const int64_t* targets,
                int32_t mask_col0, int64_t* ranks_out, void* stream);

/* Catalog-shard helpers.  count: cnt[b] = #{j < cols : l[b,j] > thresholds[b]}
 * (the strict '>' of SASRec/evaluate.py:32; summed over shards it gives rank - 1).  B <= 65535. */
int gr_count_gt_f32(const float* logits, int64_t B, int64_t cols, int64_t ld,
                    const float* thresholds, int64_t* counts_out, void* stream);

/* Per-row top-k (k <= 64) of logits[B, cols]: values descending, ties to the lower column;
 * ids_out = column + id_offset (the shard's first catalog row); -1 pads rows with < k entries.
 * When thresholds / counts_out are given (both or neither), the same single pass over the logits
 * also produces gr_count_gt_f32's counts.  Rows are cut into segments (one workgroup each, local
 * top-k to the workspace) and merged per row.  B <= 65535. */
size_t gr_topk_workspace_bytes(int64_t B, int64_t cols, int32_t k);
int gr_topk_f32(const float* logits, int64_t B, int64_t cols, int64_t ld, int32_t k,
                int64_t id_offset, float* vals_out, int64_t* ids_out, const float* thresholds,
                int64_t* counts_out, void* workspace, size_t workspace_bytes, void* stream);

/* ------------------------------------------------------------------------------------------ */
/* Fused rank without materialising logits (SASRec/evaluate.py:26-32).  Every
 * logit is evaluated with exactly the instruction sequence of gr_score_f32 (d in {16, 32, 64, 128}), so
 * the values below are bitwise the entries gr_score_f32 / gr_sasrec_predict_f32 would write.
 *
 * Target logits: out[b] = h[b] . table[ids[b]] (-1e9 when mask_col0 and ids[b] == 0, the
 * evaluate.py:27 mask).  err_flag (optional device int32) is set when an id is outside [0, rows). */
int gr_score_pairs_f32(const float* h, int64_t B, int32_t d, const float* table, int64_t rows,
                       const int64_t* ids, int32_t mask_col0, float* out, int32_t* err_flag,
                       void* stream);

/* counts_out[b] = #{j < rows : l[b, j] > thresholds[b]}, l = h . table^T with column 0 taken as
 * -1e9 when mask_col0 (strict '>', evaluate.py:32).  With thresholds = gr_score_pairs_f32 of the
 * targets, counts + 1 is the reference's rank.  On a catalog shard (rows = the shard's rows,
 * mask_col0 only on the shard holding row 0) the counts of all shards sum to the global count. */
int gr_score_count_gt_f32(const float* h, int64_t B, int32_t d, const float* table, int64_t rows,
                          const float* thresholds, int32_t mask_col0, int64_t* counts_out,
                          void* stream);

/* The same counts with a caller workspace of gr_score_count_workspace_bytes(B) bytes that must be
 * ZERO on entry and is left zero on return (one zeroed buffer serves every call on a stream).  Short
 * batches split the catalog over every CU, so hundreds of workgroups add into each user's word;
 * with the workspace the adds are spread over 16 copies and one more launch sums them (in copy
 * order: exact) -- at B 128 x 100k rows 65 -> ~25 us.  Null / short workspace: the form above. */
size_t gr_score_count_workspace_bytes(int64_t B);
int gr_score_count_gt_ws_f32(const float* h, int64_t B, int32_t d, const float* table, int64_t rows,
                             const float* thresholds, int32_t mask_col0, int64_t* counts_out,
                             void* workspace, size_t workspace_bytes, void* stream);

/* Fused top-k (+ strict counts) over the full catalog or a catalog shard without materialising
 * logits (SASRec/model.py:107 + evaluate.py:27-32; the per-shard candidate lists of SURVEY §8(e)).
 * Logits are l = h . table^T evaluated with exactly gr_score_f32's instruction sequence, column 0
 * taken as -1e9 when mask_col0.  vals_out[B, k] / ids_out[B, k]: the k largest, value descending,
 * ties to the lower column, ids = column + id_offset (-1 / -inf pad rows with fewer than k
 * columns).  thresholds / counts_out (both or neither): counts_out[b] = #{j : l[b, j] > thr[b]}.
 * d in {16, 32, 64, 128}, 1 <= k <= 16, rows < 2^31, B <= 65535.  Replaces gr_score_f32 + gr_topk_f32
 * (which read the logits back) when only the top-k / ranks are needed. */
size_t gr_score_topk_workspace_bytes(int64_t B, int32_t d, int64_t rows, int32_t k);
int gr_score_topk_f32(const float* h, int64_t B, int32_t d, const float* table, int64_t rows,
                      int64_t id_offset, int32_t mask_col0, int32_t k, const float* thresholds,
                      int64_t* counts_out, float* vals_out, int64_t* ids_out, void* workspace,
                      size_t workspace_bytes, void* stream);

/* ------------------------------------------------------------------------------------------ */
/* Merge of catalog shards' top-k lists (the catalog-sharded counterpart of
 * SASRec/evaluate.py's per-user ranking): per row b, the k best of C candidates (cand_vals[b, c],
 * cand_ids[b, c]) by (value desc, id asc) -- the id order compares all 64 bits, so any id in
 * [0, INT64_MAX) orders exactly; ids < 0 and NaN values are padding, emitted as (-inf, -1) when
 * fewer than k real candidates remain (the output always has k columns).  k >= 1, C <= 256.
 * ldv / ldi: row strides (elements). */
int gr_merge_topk_f32(const float* cand_vals, int64_t ldv, const int64_t* cand_ids, int64_t ldi,
                      int64_t B, int32_t C, int32_t k, float* vals_out, int64_t* ids_out, void* stream);
/* The same merge straight from the all-gathered exchange buffer: packed [world][B][2 kk] int64, per
 * (rank, row) kk ids then kk values (float bits in the low 32 bits of each word).  world kk <= 256. */
int gr_merge_topk_packed(const int64_t* packed, int32_t world, int64_t B, int32_t kk, int32_t k,
                         float* vals_out, int64_t* ids_out, void* stream);

/* Training-side scoring (SASRec/train.py:131-160) without the [B, n, rows]
 * score matrix.  feats[B, n, d] = model.forward(input_seqs), table[rows, d] = item_emb.weight,
 * targets[B, n] = o_t (0 = padding, masked), negs[B, num_neg] (shared by the user's n positions,
 * train.py:143-150).  With S = feats . table^T:
 *   row_loss[b*n+t] = m*(-log(sigmoid(S[b,t,o_t]) + eps)) + sum_j m*(-log(1 - sigmoid(S[b,t,neg_j]) + eps)),
 *   m = (o_t != 0);  sums[0] = batch_loss = sum of row_loss, sums[1] = mask.sum()  (train.py:155-158).
 * coef[B*n*(1+num_neg)] receives d row_loss / d S at the gathered entries (target first), the
 * saved state for the backward.  err_flag (optional device int32) is set for an id outside [0, rows). */
int gr_sampled_bce_fwd_f32(const float* feats, int64_t B, int32_t n, int32_t d, const float* table,
                           int64_t rows, const int64_t* targets, const int64_t* negs,
                           int32_t num_neg, float eps, float* row_loss, float* coef, float* sums,
                           int32_t* err_flag, void* stream);

/* Backward of batch_loss scaled by *grad_scale (device fp32 scalar, e.g. 1/valid of
 * `loss = batch_loss / batch_valid_t`): dfeats[B, n, d] (written) and dtable[rows, d] (zeroed,
 * then the gathered rows accumulated with fp32 atomics, so the summation order is not fixed). */
int gr_sampled_bce_bwd_f32(const float* feats, int64_t B, int32_t n, int32_t d, const float* table,
                           int64_t rows, const int64_t* targets, const int64_t* negs,
                           int32_t num_neg, const float* coef, const float* grad_scale,
                           float* dfeats, float* dtable, void* stream);

/* Negative items for SASRec training (SASRec/train.py:15-30 get_neg_samples): out[b, 0..num_neg)
 * = num_neg distinct items drawn uniformly from [1, item_num] minus the non-zero items of
 * seqs[b, 0..n) (the reference's np.random.choice(setdiff1d(...), num_neg, replace=False): same
 * distribution, own counter-based random stream keyed by seed).  num_neg <= 1024.  err_flag
 * (optional device int32) is set to 2 when a row has fewer than num_neg valid items (the reference
 * raises ValueError there); that row's ids are all -1. */
int gr_neg_samples(const int64_t* seqs, int64_t B, int32_t n, int64_t item_num, int32_t num_neg,
                   uint64_t seed, int64_t* out, int32_t* err_flag, void* stream);

/* gr_neg_samples keyed by seed ^ *seed_dev (a device uint64 the kernel only reads): the form a
 * captured graph (hipGraph / torch.cuda.graph) replays with fresh negatives, the caller advancing
 * *seed_dev on the stream between replays (SasTrainStep in the Python package does). */
int gr_neg_samples_dseed(const int64_t* seqs, int64_t B, int32_t n, int64_t item_num, int32_t num_neg,
                         uint64_t seed, const uint64_t* seed_dev, int64_t* out, int32_t* err_flag,
                         void* stream);

#ifdef __cplusplus
}
#endif
#endif /* GR_AMD_H */
