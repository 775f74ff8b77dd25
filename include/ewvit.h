/*
 * ewvit.h — C-ABI of the MI355X (gfx950) hot path of Efficient-Wavelet-ViT.
 *
 * The reference (Sheldon-Xiao9/efficient-wavelet-vit) is pure Python and has
 * no FFI; its boundary is the nn.Module surface of network/{mwt,sfe,dama}.py.
 * Each entry point below replaces the reference operation cited next to it;
 * the Python host side (efficient-wavelet-vit_amd/ewvit/) binds them through
 * ctypes and keeps the reference's module/attribute/state-dict surface.
 *
 * Conventions (all entry points):
 *  - plain device pointers and sizes, no framework types; every tensor is
 *    dense in the layout stated; the caller owns all memory;
 *  - `dtype` codes: EWVIT_F32 = 0, EWVIT_BF16 = 1;
 *  - `stream` is a hipStream_t passed as void* (NULL = default stream); every
 *    launch is asynchronous on it, no entry point synchronises or allocates,
 *    so calls are capturable into a hipGraph and re-entrant across threads;
 *  - return 0 on success, otherwise a hipError_t value or EWVIT_EINVAL for a
 *    rejected argument; ewvit_last_error() then describes it (thread-local).
 */
#ifndef EWVIT_H
#define EWVIT_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define EWVIT_ABI_VERSION 3
#define EWVIT_F32 0
#define EWVIT_BF16 1
#define EWVIT_EINVAL 1000
#define EWVIT_ADAM_MAX 48   /* tensors per ewvit_adam_step launch */
#define EWVIT_PACK_MAX 32   /* weights per ewvit_conv2d_pack_weights launch */

int ewvit_abi_version(void);
const char *ewvit_last_error(void);

/* ---------------------------------------------------------------- DWT ---
 * Multi-level 2-D Haar analysis, mode 'zero' — replaces the J=1
 * DWTForward(wave='haar', mode='zero') built at network/mwt.py:20 and called
 * once per level at network/mwt.py:76 inside the level loop mwt.py:107-111.
 * One HBM read of x yields every level.
 *   x   [N, C, H, W]                       (x_dtype)
 *   yh  levels planes, level l (1-based) at yh + off_l:
 *       [N, C, 3, h_l, w_l], h_l = ceil(h_{l-1}/2), band order
 *       (W-lo,H-hi), (W-hi,H-lo), (W-hi,H-hi) = pytorch_wavelets yh[0][:, :, b]
 *       off_1 = 0, off_{l+1} = off_l + N*C*3*h_l*w_l           (out_dtype)
 *   ll  [N, C, h_L, w_L] the final level's low band          (out_dtype)
 * levels in [1, 5].
 */
int ewvit_dwt_haar_fwd(const void *x, void *yh, void *ll, int64_t N, int64_t C, int64_t H,
                       int64_t W, int levels, int x_dtype, int out_dtype, void *stream);

/* Bilinear (align_corners=False) upsample of every level's HF bands to
 * (OH, OW), channels-last — replaces network/mwt.py:77-81 (reshape of yh[0]
 * to channel c*3+band, then F.interpolate(size=target_size, mode='bilinear')).
 *   yh  as produced by ewvit_dwt_haar_fwd (in_dtype)
 *   out [levels, N, OH, OW, 3C]  channel = c*3 + band          (out_dtype)
 * (OH, OW) == (h_l, w_l) is an exact copy (the reference skips the interpolate
 * when MWT.levels == 1, mwt.py:79; the caller passes (h_1, w_1) then).
 */
int ewvit_hf_upsample(const void *yh, void *out, int64_t N, int64_t C, int64_t H, int64_t W,
                      int levels, int64_t OH, int64_t OW, int in_dtype, int out_dtype,
                      int64_t out_channels, void *stream);
/* out_channels: channel stride of `out` (0 = 3C); channels 3C .. out_channels-1 are
 * written as zeros (the 16-channel-aligned input of the hf_conv MFMA conv). */

/* Fused ewvit_dwt_haar_fwd + ewvit_hf_upsample for the MWT's hf_conv input (SURVEY §7.4;
 * network/mwt.py:76-81 per level, all levels at once as mwt.py:101-110 loops them): x
 * [N, 3, H, W] (fp32/bf16) -> out [levels, N, H/2, W/2, out_channels] channels-last, the 9
 * band channels (colour-major, bands LH/HL/HH) bilinearly upsampled to level-1 resolution
 * and channels 9.. zero.  Bit-identical to the two-launch path with band_dtype = out_dtype;
 * the bands never reach HBM (one launch, 1 x frames in + the output).  Applies when
 * ewvit_dwt_hf_fused_ok(): C == 3, levels <= 3, H and W multiples of 2^levels,
 * (OH, OW) == (H/2, W/2), W/2 <= 112, 9 <= out_channels <= 16 (wider frames: the two
 * launches measured faster). */
int ewvit_dwt_hf_fused_ok(int64_t N, int64_t C, int64_t H, int64_t W, int levels, int64_t OH, int64_t OW,
                          int64_t out_channels);
int ewvit_dwt_hf_upsample_fused(const void *x, void *out, int64_t N, int64_t C, int64_t H, int64_t W,
                                int levels, int x_dtype, int out_dtype, int64_t out_channels, void *stream);

/* --------------------------------------------------------------- GEMM ---
 * C[m,n] = epilogue( alpha * sum_k A(m,k) * B(k,n) )   bf16 MFMA, fp32 accumulate
 * — the projection GEMMs of network/sfe.py:44-55,29-40 (to_qkv, to_out,
 * FeedForward), network/dama.py:25-31 (to_q, to_kv, to_out),
 * sfe.py:127,155 (patch_to_embedding, split-K) and their backward products.
 *   A(m,k) = A[m*lda_m + k*lda_k]   (exactly one of lda_m, lda_k equals 1)
 *   B(k,n) = B[k*ldb_k + n*ldb_n]   (exactly one of ldb_k, ldb_n equals 1)
 *   C[m*ldc + n]                    (c_dtype)
 * epilogue, in order: + bias[n] (f32, may be NULL)
 *                     ; act: 0 none, 1 GELU(erf), 2 ReLU, 3 multiply by GELU'(aux[m,n])
 *                       (act 1/2 also store the pre-activation to aux when aux != NULL)
 *                     ; dropout: if drop_p > 0, keep with prob 1-drop_p from
 *                       hash(seed', m*N+n), scale 1/(1-drop_p), where
 *                       seed' = seed + *seed_offset * 0xD1B54A32D192ED03 (seed_offset:
 *                       device int64 advanced once per step — a graph-replayed
 *                       launch draws a new mask each replay — or NULL: seed' = seed)
 *                     ; + resid[m*ldr + n] (f32 or bf16 per resid_dtype, may be NULL)
 *                     ; if beta != 0: C = beta*C_old + value (f32 C only)
 *   aux[m*ldc + n] (bf16) — pre-activation for act 1/3
 * splitk > 1 partitions K over blockIdx.z; workspace must then hold
 * splitk*M*N floats and the epilogue runs in a second launch.
 */
int ewvit_gemm(const void *A, int a_dtype, int64_t lda_m, int64_t lda_k, const void *B,
               int b_dtype, int64_t ldb_k, int64_t ldb_n, void *C, int c_dtype, int64_t ldc,
               int64_t M, int64_t N, int64_t K, float alpha, float beta, const float *bias,
               int act, void *aux, float drop_p, uint64_t seed, const int64_t *seed_offset,
               const void *resid, int resid_dtype, int64_t ldr, int splitk, float *workspace,
               void *stream);

/* fp8 (BASELINE configs[4]): ewvit_gemm with MXFP8 operands — each run of 32 consecutive K
 * elements of a row of A (and of a column of B) quantized to OCP e4m3fn with one shared E8M0
 * scale 2^X, X the smallest with max|run| <= 448 * 2^X (round to nearest even, no saturation
 * needed) — multiplied on v_mfma_scale_f32_16x16x128_f8f6f4 with fp32 accumulation:
 * C = epi(alpha * sum_k q(A)(m,k) sa(m,k/32) q(B)(k,n) sb(k/32,n)).  The scales are computed
 * from the operands as they are staged (no amax pass; graph-capturable).  Replaces the bf16
 * GEMMs of the ViT attention / MLP (sfe.py:29-70), the cross-attention projections
 * (dama.py:15-53) and patch_to_embedding / feat_map (sfe.py:127,155,168) when the model runs in
 * fp8 (network.set_gemm_precision) on the module path; same arguments as ewvit_gemm. */
int ewvit_gemm_mx8(const void *A, int a_dtype, int64_t lda_m, int64_t lda_k, const void *B, int b_dtype,
                   int64_t ldb_k, int64_t ldb_n, void *C, int c_dtype, int64_t ldc, int64_t M, int64_t N, int64_t K,
                   float alpha, float beta, const float *bias, int act, void *aux, float drop_p, uint64_t seed,
                   const int64_t *seed_offset, const void *resid, int resid_dtype, int64_t ldr, int splitk,
                   float *workspace, void *stream);

/* Column sums: out[n] (+)= sum_m X[m*ldx + n]  (bias gradients).  accumulate!=0 adds. */
/* C[M][N] f32 = A[M][K] (bf16, row stride lda) x W[N][K]^T (fp32, rounded to bf16) + bias (may be
 * NULL) for M <= 64, N % 256 == 0, K % 256 == 0: the patch_to_embedding forward (sfe.py:155,
 * [64 x 62720] x [62720 x 512]).  A workgroup per (256-wide K slice, 256 columns) leaves a fp32
 * partial in `workspace` (ewvit_gemm_tallk_workspace bytes), a second launch adds the slices
 * in a fixed order. */
int64_t ewvit_gemm_tallk_workspace(int64_t M, int64_t N, int64_t K);
int ewvit_gemm_tallk(const void *A, int64_t lda, const float *W, const float *bias, float *C, int64_t ldc, int64_t M,
                     int64_t N, int64_t K, float *workspace, void *stream);
int ewvit_colsum(const void *X, int x_dtype, int64_t ldx, int64_t M, int64_t N, float *out,
                 int accumulate, void *stream);

/* Dropout mask regeneration for backward: g[i] *= keep(seed', i)/(1-p), i < n. */
int ewvit_dropout_bwd(void *g, int g_dtype, int64_t rows, int64_t cols, int64_t ldg, float p,
                      uint64_t seed, const int64_t *seed_offset, void *stream);

/* Backward of the GEMM epilogue: out[m*N+n] = dy[m*lddy+n] * keep(seed', m*N+n)/(1-p)
 * * act'(aux[m*N+n]);  act 0 none, 1 GELU(erf) (aux = pre-activation), 2 ReLU. */
int ewvit_act_bwd(const void *dy, int dy_dtype, int64_t lddy, const void *aux, int act,
                  float drop_p, uint64_t seed, const int64_t *seed_offset, void *out, int out_dtype,
                  int64_t M, int64_t N, void *stream);

/* ---------------------------------------------------------- LayerNorm ---
 * y = (x - mean) * rstd * gamma + beta over the last dim D, eps — nn.LayerNorm
 * of network/sfe.py:23 (PreNorm) and network/dama.py:62,64.
 *   x [M, D] (x_dtype, row stride ldx); y [M, D] (y_dtype); mean/rstd [M] f32.
 */
int ewvit_layernorm_fwd(const void *x, int x_dtype, int64_t ldx, const float *gamma,
                        const float *beta, void *y, int y_dtype, float *mean, float *rstd,
                        int64_t M, int64_t D, float eps, void *stream);
/* dx = LN backward (x_dtype input, dy dy_dtype); dgamma/dbeta written (=) in f32 (either may be
 * null); dx written (f32) or added to (accumulate_dx != 0). */
int ewvit_layernorm_bwd(const void *dy, int dy_dtype, const void *x, int x_dtype, int64_t ldx,
                        const float *gamma, const float *mean, const float *rstd, float *dx,
                        int accumulate_dx, float *dgamma, float *dbeta, float *workspace, int64_t M, int64_t D,
                        void *stream);
/* bytes of `workspace` ewvit_layernorm_bwd needs: per-block dgamma / dbeta partials, added in
 * block order by a second launch (deterministic; dgamma / dbeta need no zero-fill) */
int64_t ewvit_layernorm_bwd_workspace(int64_t M, int64_t D);

/* ------------------------------------------------- short-sequence attention ---
 * softmax(q k^T * scale) v per (batch, head) for the degenerate sequence
 * lengths of this model: ViT n=2 (sfe.py:59-70: 'b n (h d) -> b h n d', einsum,
 * Softmax(-1), einsum, merge) and the cross-attention 1 query x 2 keys
 * (dama.py:33-53 with kv_include_self).  nq, nk <= 8, head dim d <= 128.
 *   q (b, i, h, :) at q + b*sq_b + i*sq_n + h*d      (bf16)
 *   k (b, j, h, :) at k + b*sk_b + j*sk_n + h*d      (bf16); v likewise (sv_*)
 *   o (b, i, h, :) at o + b*so_b + i*so_n + h*d      (bf16)
 *   p [B, H, nq, nk] softmax probabilities saved for backward (f32)
 */
int ewvit_attn_fwd(const void *q, int64_t sq_b, int64_t sq_n, const void *k, int64_t sk_b,
                   int64_t sk_n, const void *v, int64_t sv_b, int64_t sv_n, void *o,
                   int64_t so_b, int64_t so_n, float *p, int64_t B, int64_t H, int nq, int nk,
                   int d, float scale, void *stream);
/* dq, dk, dv (bf16, same strides as q/k/v; written, not accumulated) from do. */
int ewvit_attn_bwd(const void *dout, int64_t sdo_b, int64_t sdo_n, const void *q, int64_t sq_b,
                   int64_t sq_n, const void *k, int64_t sk_b, int64_t sk_n, const void *v,
                   int64_t sv_b, int64_t sv_n, const float *p, void *dq, void *dk, void *dv,
                   int64_t B, int64_t H, int nq, int nk, int d, float scale, void *stream);

/* ------------------------------------------- depthwise 3x3 conv (backbone) ---
 * The MBConv depthwise convolutions of EfficientNetV2-S (groups = channels,
 * kernel 3, stride 1|2, pad 1, no bias) — the backbone the reference reaches
 * through network/sfe.py:111-113,150 (torchvision Conv2dNormActivation).
 * Channels-last: x [N, H, W, C], y [N, Ho, Wo, C] (dtype), w [C, 3, 3] f32;
 * C % 8 == 0; Ho = (H + 2*pad - 3)/stride + 1.
 */
int ewvit_dwconv3x3_fwd(const void *x, const float *w, void *y, int64_t N, int64_t H, int64_t W,
                        int64_t C, int stride, int pad, int dtype, void *stream);
/* dx [N, H, W, C] from dy [N, Ho, Wo, C] (written). */
int ewvit_dwconv3x3_bwd_data(const void *dy, const float *w, void *dx, int64_t N, int64_t H, int64_t W,
                             int64_t C, int stride, int pad, int dtype, void *stream);
/* bytes of f32 workspace ewvit_dwconv3x3_bwd_weight needs (per-slab partials). */
int64_t ewvit_dwconv3x3_bwd_weight_workspace(int64_t N, int64_t H, int64_t W, int64_t C, int stride,
                                             int pad);
/* dw [C, 3, 3] f32 (= or += when accumulate) = sum over N*Ho*Wo of dy * x-tap;
 * deterministic two-pass reduction through `workspace`. */
int ewvit_dwconv3x3_bwd_weight(const void *x, const void *dy, float *dw, int accumulate, int64_t N,
                               int64_t H, int64_t W, int64_t C, int stride, int pad, int dtype,
                               float *workspace, void *stream);
/* The same convs with the training-mode BatchNorm sums of what they store (bf16, pad 1),
 * so the MBConv block's BatchNorm around the depthwise conv (torchvision
 * Conv2dNormActivation, sfe.py:111-113,150) runs no statistics pass of its own.  One partial
 * row per 32 output rows n*Ho + ho: ewvit_dwconv3x3_bn_rows(N, H, W, C, stride, bwd) rows
 * (0 = shape not supported; bwd: the stride-1 input gradient, rows of dx).
 * fwd_bn: part [rows][2C] = (sum (y - K), sum (y - K)^2) per channel, K = shift (a running
 *   mean estimate, NULL: 0), shift_out [C] = K — what ewvit_bn_fwd_partials finalises.
 * bwd_data_bn (stride 1): dx as ewvit_dwconv3x3_bwd_data, and part [rows][2C] = (sum g,
 *   sum g*xhat) of the BatchNorm(+act) that produced the conv's input: xhat = (bx - mean)
 *   * invstd (bx: that BN's input [N, H, W, C] bf16), g = dx * act'(xhat*gamma + beta)
 *   (act 0/1/2; gamma / beta NULL = 1 / 0) — what ewvit_bn_bwd_partials finalises. */
int64_t ewvit_dwconv3x3_bn_rows(int64_t N, int64_t H, int64_t W, int64_t C, int stride, int bwd);
int ewvit_dwconv3x3_fwd_bn(const void *x, const float *w, void *y, int64_t N, int64_t H, int64_t W, int64_t C,
                           int stride, const float *shift, float *part, float *shift_out, void *stream);
int ewvit_dwconv3x3_bwd_data_bn(const void *dy, const float *w, void *dx, int64_t N, int64_t H, int64_t W,
                                int64_t C, const void *bx, const float *mean, const float *invstd,
                                const float *gamma, const float *beta, int act, float *part, void *stream);
/* The whole stride-1 pad-1 backward in one pass: dx and part as bwd_data_bn, plus
 * dw [C, 3, 3] f32 (= or += when accumulate) as ewvit_dwconv3x3_bwd_weight from x (the conv's
 * bf16 input [N, H, W, C]), reading dy once; C % 8 == 0.  workspace: ..._bwd_fused_workspace
 * bytes (one [C][9] slab per partial row). */
int64_t ewvit_dwconv3x3_bwd_fused_workspace(int64_t N, int64_t H, int64_t W, int64_t C);
int ewvit_dwconv3x3_bwd_fused(const void *dy, const float *w, void *dx, const void *x, float *dw, int accumulate,
                              int64_t N, int64_t H, int64_t W, int64_t C, const void *bx, const float *mean,
                              const float *invstd, const float *gamma, const float *beta, int act, float *part,
                              float *workspace, void *stream);
/* ewvit_dwconv3x3_bwd_fused with the backward of the BatchNorm(+act se_act) + squeeze-excitation
 * that consumed the conv's OUTPUT folded in (MBConv: depthwise conv -> BN -> SiLU -> SE): dy is
 * the SE output gradient; the conv's output gradient dz = gamma*invstd*(act'(zhat*gamma+beta)*
 * (dy*s + g) - row[c]/n - zhat*row[C+c]/n), zhat = (z - se_mean)*se_invstd, n = N*H*W, is formed
 * per window element (zero outside the map) and rounded to bf16 — the same operations as
 * ewvit_bn_se_bwd's dx pass, so the same bits — and never stored.  z: the BN input (the conv's
 * output) [N,H,W,C] bf16; se_row: the sums row ewvit_bn_se_bwd (dx NULL) leaves in its workspace
 * at ewvit_bn_se_bwd_row_offset floats; se_s / se_g [N][C]: the excitation and squeeze term. */
int ewvit_dwconv3x3_bwd_fused_se(const void *dy, const float *w, void *dx, const void *x, float *dw,
                                 int accumulate, int64_t N, int64_t H, int64_t W, int64_t C, const void *bx,
                                 const float *mean, const float *invstd, const float *gamma, const float *beta,
                                 int act, float *part, float *workspace, const void *z, const float *se_mean,
                                 const float *se_invstd, const float *se_gamma, const float *se_beta, int se_act,
                                 const float *se_row, const float *se_s, const float *se_g, void *stream);

/* ---------------------------------------------- BatchNorm2d + activation ---
 * BatchNorm2d (batch statistics in training, running statistics in eval) fused
 * with the activation that follows it: act 0 none, 1 ReLU (the MWT conv stack,
 * network/mwt.py:23-72), 2 SiLU (the EfficientNetV2-S backbone's
 * Conv2dNormActivation, reached via network/sfe.py:111-113).  Channels-last
 * x, y [M = N*H*W][C] (dtype), C % 8 == 0, C <= 2048; gamma/beta/running stats f32.
 * Training also writes save_mean / save_invstd [C] (biased variance) and
 * updates running_mean/var in place with `momentum` (unbiased variance), as
 * torch does.  `groups` > 1 splits the M rows into equal consecutive groups
 * with their OWN batch statistics (save_mean/invstd [groups][C]) and applies
 * the running-stat update once per group in order — the MWT calls its shared
 * hf_conv BatchNorms once per wavelet level (network/mwt.py:107-111), here all
 * levels are one launch.  `num_batches_tracked` (int64 on the device, or NULL) is
 * incremented by `groups` in training, like the module's counter.
 * `workspace` holds ewvit_bn_workspace(M, C, groups) bytes.
 */
int64_t ewvit_bn_workspace(int64_t M, int64_t C, int groups);
int ewvit_bn_fwd(const void *x, void *y, int dtype, int64_t M, int64_t C, const float *gamma,
                 const float *beta, float *running_mean, float *running_var, int training,
                 float momentum, float eps, int act, float *save_mean, float *save_invstd,
                 int groups, int64_t *num_batches_tracked, float *workspace, void *stream);
/* Training forward from precomputed partial statistics: part [nrc][2C] rows of
 * (sum (x-K), sum (x-K)^2) and shifts K [C] — what ewvit_conv2d_fwd_bn leaves in
 * its epilogue — so only the apply pass runs (one group). */
int ewvit_bn_fwd_partials(const void *x, void *y, int dtype, int64_t M, int64_t C, const float *gamma,
                          const float *beta, float *running_mean, float *running_var, float momentum,
                          float eps, int act, float *save_mean, float *save_invstd,
                          int64_t *num_batches_tracked, const float *part, const float *shifts, int nrc,
                          int groups, void *stream);
/* ewvit_bn_fwd_partials without the apply pass: the same finalisation (batch statistics,
 * running statistics, counter += groups, save_mean / save_invstd) writing the apply pass's
 * coefficients coef[g][0][c] = gamma * invstd, coef[g][1][c] = beta - mean * gamma * invstd,
 * for an op that applies y = act(x * coef0 + coef1) itself (ewvit_conv2d_fwd_bn_xf). */
int ewvit_bn_coef(int64_t M, int64_t C, const float *gamma, const float *beta, float *running_mean,
                  float *running_var, float momentum, float eps, float *save_mean, float *save_invstd,
                  int64_t *num_batches_tracked, const float *part, const float *shifts, int nrc, int groups,
                  float *coef, void *stream);
/* part_out[g][k] = sum of part_in[g][k*ch .. k*ch + ch - 1] (ch = ceil(nin / nout); rows
 * of 2C floats, fixed order) and shift_out[g][:] = shift_in[:]: brings a large conv's
 * per-tile partial rows down to what the apply pass finalises from. */
int ewvit_bn_fold_partials(const float *part_in, int nin, const float *shift_in, float *part_out, int nout,
                           float *shift_out, int64_t C, int groups, void *stream);
/* MBConv block tail in one pass (training, no activation, one group): y = bn(x) *
 * scale[n] + skip, n = row / HW, scale[n] = (u < keep_prob) / keep_prob with u the
 * counter hash of (seed + *seed_offset * golden, n) as ewvit dropout draws it;
 * scale_out[n] receives the factors.  Statistics from part/shifts/nrc (as
 * ewvit_bn_fwd_partials) or, with part == NULL, computed into `workspace`
 * (ewvit_bn_workspace(M, C, 1) bytes). */
int ewvit_bn_fwd_drop_add(const void *x, void *y, int dtype, int64_t M, int64_t C, const float *gamma,
                          const float *beta, float *running_mean, float *running_var, float momentum, float eps,
                          float *save_mean, float *save_invstd, int64_t *num_batches_tracked, const float *part,
                          const float *shifts, int nrc, const void *skip, int64_t HW, float keep_prob,
                          uint64_t seed, const int64_t *seed_offset, float *scale_out, float *workspace,
                          void *stream);
/* Its backward: dx of the BatchNorm for g = dy * row_scale[row / HW]; dgamma / dbeta
 * overwritten (may be NULL); the skip's gradient is dy. */
int ewvit_bn_bwd_scaled(const void *dy, const void *x, void *dx, int dtype, int64_t M, int64_t C,
                        const float *gamma, const float *beta, const float *save_mean, const float *save_invstd,
                        float *dgamma, float *dbeta, const float *row_scale, int64_t HW, float *workspace,
                        void *stream);
/* Backward of BatchNorm(+act) followed by squeeze-excitation (MBConv's depthwise BN + SiLU
 * then SE, torchvision Conv2dNormActivation + SqueezeExcitation, network/sfe.py:111-113):
 * the BatchNorm's output gradient dy*se_s[n][c] + se_g[n][c] (se_s the excitation [N][C],
 * se_g the squeeze term from ewvit_se_squeeze_mlp_bwd, HW rows per frame) is formed from the
 * SE output gradient dy inside both passes — the SE input-gradient pass never runs.
 * dgamma / dbeta overwritten. */
int ewvit_bn_bwd_se(const void *dy, const void *x, void *dx, int dtype, int64_t M, int64_t C, const float *gamma,
                    const float *beta, const float *save_mean, const float *save_invstd, int act, float *dgamma,
                    float *dbeta, const float *se_s, const float *se_g, int64_t HW, float *workspace, void *stream);
/* Training-mode backward whose reduction pass already ran in the kernel that produced dy
 * (ewvit_conv2d_bwd_data_bn, ewvit_dwconv3x3_bwd_data_bn): part [groups][nrc][2C] rows of
 * (sum g, sum g*xhat), g = dy * act'(...) or, with row_scale [M / HW] (act 0, one group: the
 * MBConv tail of ewvit_bn_fwd_drop_add), g = dy * row_scale[row / HW].  `groups` as in
 * ewvit_bn_bwd (consecutive row slices with their own statistics).  Only the dx pass runs;
 * dgamma / dbeta summed over the groups, overwritten (may be NULL).  Replaces the reduce
 * launch of ewvit_bn_bwd / ewvit_bn_bwd_scaled (BatchNorm2d backward of the backbone,
 * sfe.py:111-113, and of the MWT's hf_conv / multiscale_fusion, mwt.py:60-72). */
int ewvit_bn_bwd_partials(const void *dy, const void *x, void *dx, int dtype, int64_t M, int64_t C,
                          const float *gamma, const float *beta, const float *save_mean, const float *save_invstd,
                          int act, float *dgamma, float *dbeta, const float *row_scale, int64_t HW,
                          const float *part, int nrc, int groups, void *stream);
/* MBConv's depthwise BatchNorm + act (training, statistics from partial rows as
 * ewvit_bn_fwd_partials: the depthwise conv's, ewvit_dwconv3x3_fwd_bn) and the squeeze of the
 * squeeze-excitation after it (torchvision Conv2dNormActivation + SqueezeExcitation,
 * sfe.py:111-113) in one pass over x [N][HW][C]: y = act(bn(x)), s0[n][c] = mean_hw y (of
 * the stored values), part [N][ceil(C / 64)][Csq] = the SE MLP's first-layer partials
 * sum_{c in chunk} w1[j][c] s0[n][c] (w1 [Csq][C] f32) for ewvit_se_gate_excite; running
 * statistics / saved mean, invstd / counter as ewvit_bn_fwd_partials.  The same bits as
 * ewvit_bn_fwd_partials + ewvit_se_squeeze_mlp_fwd's first launch. */
int ewvit_bn_act_se_squeeze(const void *x, void *y, int dtype, int64_t N, int64_t HW, int64_t C, const float *gamma,
                            const float *beta, float *running_mean, float *running_var, float momentum, float eps,
                            int act, float *save_mean, float *save_invstd, int64_t *num_batches_tracked,
                            const float *part, const float *shifts, int nrc, const float *w1, int64_t Csq, float *s0,
                            float *hpart, void *stream);
/* dx (dtype) from dy and the saved x/statistics (training-mode backward);
 * dgamma/dbeta f32 summed over groups (= or += when accumulate), either may be NULL. */
int ewvit_bn_bwd(const void *dy, const void *x, void *dx, int dtype, int64_t M, int64_t C,
                 const float *gamma, const float *beta, const float *save_mean,
                 const float *save_invstd, int act, float *dgamma, float *dbeta, int accumulate,
                 int groups, float *workspace, void *stream);

/* ------------------------------------------ dense conv, implicit GEMM ---
 * Conv2d(kernel 1|3, pad kernel/2, stride 1|2, bias) — the MWT conv stack:
 * hf_conv['fusion'] (mwt.py:60-64), multiscale_fusion (mwt.py:68-72), freq_conv
 * (mwt.py:23-36), freq_pool's conv (mwt.py:38-44) — and the EfficientNetV2-S
 * backbone's dense convs (sfe.py:111-113 -> torchvision Conv2dNormActivation).
 * Replaces the cuDNN nn.Conv2d calls behind those modules.
 * bf16 MFMA, fp32 accumulate, channels-last: x [N, H, W, Cin], y [N, Ho, Wo, Cout]
 * (bf16); Cin, Cout % 8 == 0; Ho = (H-1)/stride + 1.  Weights are packed once per
 * step from the fp32 master [Cout][Cin][k][k] (element (co, ci, kh*k+kw) at
 * co*s_co + ci*s_ci + (kh*k+kw)*s_tap: contiguous or channels-last parameters) by
 * ewvit_conv2d_pack_weight into wp [Cout][k*k][Cin_pad] (fwd) and/or
 * wp_t [Cin_pad][k*k][Cout] (bwd_data), either may be NULL; input channels
 * ci >= Cin are zero-filled up to Cin_pad.
 * Grouped channels-last operands (x of fwd / bwd_weight, dx of bwd_data): channel c
 * of pixel p lives at (c / group_c) * group_stride + p * group_c + c % group_c
 * (elements); group_c = 0 means plain NHWC.  group_c must divide Cin and be a
 * multiple of 32 — e.g. the MWT's per-level outputs [L][N][H][W][128] consumed as
 * their channel concatenation (mwt.py:112) without a copy.
 */
int ewvit_conv2d_pack_weight(const float *w, int64_t s_co, int64_t s_ci, int64_t s_tap, void *wp,
                             void *wp_t, int64_t Cout, int64_t Cin, int64_t Cin_pad, int ksize,
                             void *stream);
/* ewvit_conv2d_pack_weight for n <= EWVIT_PACK_MAX weights in ONE launch (arrays of the
 * same per-weight arguments; ksize[i] 1 or 3): the training step packs every conv
 * weight of the model once, after the optimizer update, instead of once per conv. */
int ewvit_conv2d_pack_weights(int n, const float *const *w, const int64_t *s_co, const int64_t *s_ci,
                              const int64_t *s_tap, void *const *wp, void *const *wp_t, const int64_t *Cout,
                              const int64_t *Cin, const int64_t *Cin_pad, const int *ksize, void *stream);
/* At most `max_workgroups` (rounded up to a multiple of 8; 0 = no cap, the default) per
 * launch of the big-grid kernels from now on: LDS-DMA conv fwd / dgrad walk their tiles
 * persistently, conv wgrad uses fewer pixel splits, the BatchNorm passes take more rows per
 * workgroup.  For a branch sharing the GPU with another stream (DAMA's MWT beside the
 * backbone: its big launches then leave most CUs to the backbone's latency-bound kernels).
 * Host-side state of the CALLING THREAD, read at launch time (so a HIP graph records the
 * capped grids; nn.DataParallel's replica threads, reference train.py:249-251, each keep their
 * own).  Returns the previous cap.  ewvit_conv2d_set_grid_cap is the same call. */
int ewvit_set_grid_cap(int max_workgroups);
/* Timeline probe (diagnostics): when `stream` reaches it, stamps[idx] = the device wall clock,
 * ewvit_wall_clock_khz() ticks per millisecond (0 when the device cannot be queried). */
int ewvit_probe(long long *stamps, int idx, void *stream);
int ewvit_wall_clock_khz(void);
int ewvit_conv2d_set_grid_cap(int max_workgroups);

/* Kernel-family test switch (not needed for correctness): 0 runs every shape on the
 * register-staged kernels — the fallback of the shapes the LDS-DMA kernels refuse — so a test
 * can check both on one case; 1 (default) the LDS-DMA kernels wherever the shape allows.
 * Returns the previous setting.  Replaces nothing in the reference. */
int ewvit_conv2d_set_glds(int variant);
/* Windowed 3x3 stride-1 kernel switch (test / A-B switch, csrc/convwin.hip): 1 (default) the
 * forward and input gradient of 3x3 stride-1 convs over maps whose sides are multiples of 16,
 * with 64-channel input blocks and 128-column output tiles (the MWT's multiscale_fusion and
 * hf_conv fusion, reference network/mwt.py:60-72,112-114), run one workgroup per 16 x 16
 * output block with the block's 18 x 18 input window staged once per channel block; 0 the
 * generic LDS-DMA kernel (bit-identical results).  The forward's BatchNorm partials then
 * come one row per 16 x 16 block (ewvit_conv2d_fwd_bn_rows answers 256).  Returns the
 * previous setting.  Replaces nothing in the reference. */
int ewvit_conv2d_set_win(int variant);
/* 1 = the windowed kernels request the CU's whole 160 KB of LDS (no co-resident workgroup of
 * another stream on a CU they hold; the default), 0 = their own footprint.  Returns the previous. */
int ewvit_conv2d_set_lds_pad(int on);
/* The windowed 3x3 weight gradient's tap-split 8-wave variant (two waves per SIMD, taps 0-4 and
 * 5-8 on separate waves; 1 on, the default, 0 the 4-wave kernel, 2 a 12-wave form with one kernel
 * row per wave group); returns the previous setting.  Results are bit-identical in every form
 * (same per-output MFMA chain).  Env: EWVIT_WGWIN_TS=0 / 2. */
int ewvit_conv2d_set_wgrad_tap_split(int on);
/* The non-temporal cache hint on the windowed MWT convs' activation-window DMAs, taken only
 * under a grid cap (beside the backbone): a mask, 1 the fwd / dgrad windows, 2 the wgrad dy
 * tiles, 4 the wgrad x windows (7, the default, all; 0 none); returns the previous setting.
 * Env: EWVIT_WIN_NT. */
int ewvit_conv2d_set_win_nt(int mask);
/* A/B: level-1 pixels per thread in flight in ewvit_dwt_hf_upsample_fused (2, the default, or 4); returns the previous. */
int ewvit_dwt_set_pf(int pf);
/* Weight-gradient n'-tile width (test switch): 4 (default) auto — 256-column tiles (each wave
 * 64 x 128, 32 pixels per K-tile) for n' = k*k*Cin >= 2048 over >= 64K output pixels, else
 * 128-column tiles; 2 = 256-column tiles whenever n' >= 256 and the last tile wastes <= 1/8 of
 * it; 0 = never.  Returns the previous setting.  Replaces nothing in the reference. */
int ewvit_conv2d_set_wgrad_wide(int variant);
/* The 1x1 stride-1 weight-gradient kernel (plain NHWC x, no bias gradient): workgroup target of
 * its pixel splits (0 = never: the generic kernel), fewest 64-pixel K-tiles per split, LDS ring
 * depth (2 | 3).  Test / tuning switch; returns the previous target.  min_ktiles < 1 and a ring
 * other than 2 / 3 keep the current value. */
int ewvit_conv2d_set_wgrad_1x1(int target_wg, int min_ktiles, int ring);
/* The current 1x1 weight-gradient knobs: which = 0 workgroup target, 1 min K-tiles, 2 ring
 * (defaults 256, 8, 2).  Replaces nothing in the reference. */
int ewvit_conv2d_wgrad_1x1_config(int which);
/* LDS-DMA fwd / dgrad on grids of < 128 row tiles: 64-row (and 64-column) tiles, 1 (default),
 * or the 128-row tiles everywhere, 0 (test switch).  Returns the previous setting. */
int ewvit_conv2d_set_small_tiles(int on);
/* Split K (default OFF: measured slower in the step) for the LDS-DMA 1x1 forward / input
 * gradient over fewer than 256 tiles with >= 8 K-tiles per split (the backbone's long-K 1x1
 * convs at 7^2): fp32 partials in a per-stream scratch buffer the library owns (allocated
 * outside stream capture), summed by an epilogue launch that also forms the BatchNorm
 * statistics.  on > 1 sets the limits too (max splits = on & 15, min K-tiles = on >> 4).
 * Returns the previous on / off setting. */
int ewvit_conv2d_set_ksplit(int on);
/* Input channels per tap the forward expects its packed weights to have (the Cin_pad
 * of ewvit_conv2d_pack_weight for the fwd pack): Cin, or Cin rounded up to 64 when a
 * plain-NHWC input's channel count is not a multiple of 64 and the LDS-DMA kernel runs
 * the shape with zero lanes for the missing channels. */
int64_t ewvit_conv2d_fwd_pack_cin(int64_t N, int64_t H, int64_t W, int64_t Cin, int64_t Cout, int ksize,
                                  int stride);
/* y = conv(x, W) + bias (bias f32 [Cout] or NULL); wp packed with
 * ewvit_conv2d_fwd_pack_cin(...) input channels (grouped x: Cin). */
/* ewvit_conv2d_fwd (plain NHWC x, Cin % 64 == 0) that also leaves the BatchNorm
 * statistics of its bf16 output for ewvit_bn_fwd_partials (grouped x as in ewvit_conv2d_fwd,
 * group width a multiple of 64): per tile of R output rows
 * (R = ewvit_conv2d_fwd_bn_rows(...), 0 when the shape is not supported) bn_part[t]
 * gets (sum (y - K), sum (y - K)^2) over its rows per channel, K = bn_shift[c] (a
 * running-mean estimate; NULL: 0), and bn_shift_out receives K. */
int64_t ewvit_conv2d_fwd_bn_rows(int64_t N, int64_t H, int64_t W, int64_t Cin, int64_t Cout, int ksize,
                                 int stride);
int ewvit_conv2d_fwd_bn(const void *x, const void *wp, const float *bias, void *y, int64_t N, int64_t H,
                        int64_t W, int64_t Cin, int64_t Cout, int ksize, int stride, int64_t x_group_c,
                        int64_t x_group_stride, const float *bn_shift, float *bn_part, float *bn_shift_out,
                        void *stream);
int ewvit_conv2d_fwd(const void *x, const void *wp, const float *bias, void *y, int64_t N, int64_t H,
                     int64_t W, int64_t Cin, int64_t Cout, int ksize, int stride, int64_t x_group_c,
                     int64_t x_group_stride, void *stream);
/* Convs that read relu(x * scale + shift) instead of x: the training BatchNorm + ReLU of x's
 * producer (the MWT hf_conv['fusion'] BN, reference network/mwt.py:60-65, ahead of
 * multiscale_fusion, mwt.py:68-72,114) applied inside the windowed kernels' operand staging,
 * so the normalised map is never written.  xf: [groups][2][x_group_c] fp32 = per channel group
 * of x (scale row, shift row), as ewvit_bn_coef writes them; the result is bit-identical to
 * ewvit_bn_fwd_partials(act = relu) followed by ewvit_conv2d_fwd_bn / ewvit_conv2d_bwd_weight.
 * 3x3 stride 1 only, where the windowed kernels take the shape (ewvit_conv2d_xf_ok: 1 / 0;
 * Cin <= 512).  The input gradient of such a conv is the plain ewvit_conv2d_bwd_data. */
/* The windowed 3x3 stride-1 input gradient with the backward statistics of the BatchNorm(+act)
 * whose output the conv read (as ewvit_conv2d_bwd_data_bn, but one partial row per 16 x 16 dx
 * block: part [groups][N*H*W/256][2 group_c], BatchNorm groups = dx's channel groups, mean /
 * invstd [groups][group_c], gamma / beta [group_c] or NULL) — the MWT hf fusion BN's backward
 * sums taken by multiscale_fusion's input gradient (reference network/mwt.py:60-72,114).  A
 * plain dx (dx_group_c = Cin, dx_group_stride 0) may instead carry BatchNorm row groups:
 * bn_group_rows > 0 rows per slice (whole images, slices * Cin <= 768), mean / invstd
 * [slices][Cin], part [slices][bn_group_rows/256][2 Cin] — the seperate BNs' per-level
 * statistics taken by hf_conv['fusion']'s input gradient (a 64-column dx: the k-split form,
 * reference network/mwt.py:48-65,84-88).
 * Limits: Cin <= 512 columns (row groups: slices * Cin <= 768), group_c <= 256.
 * ewvit_conv2d_bwd_bn_win_rows: N*H*W/256 (the rows per channel group; with row groups, the
 * total over the slices), 0 when the windowed kernel does not take it. */
int64_t ewvit_conv2d_bwd_bn_win_rows(int64_t N, int64_t H, int64_t W, int64_t Cin, int64_t Cout, int ksize, int stride,
                                     int64_t dx_group_c, int64_t dx_group_stride, int64_t bn_group_rows);
int ewvit_conv2d_bwd_data_bn_win(const void *dy, const void *wp_t, void *dx, int64_t N, int64_t H, int64_t W,
                                 int64_t Cin, int64_t Cout, int64_t dx_group_c, int64_t dx_group_stride,
                                 const void *bx, const float *mean, const float *invstd, const float *gamma,
                                 const float *beta, int act, int64_t bn_group_rows, float *part, void *stream);
int ewvit_conv2d_xf_ok(int64_t N, int64_t H, int64_t W, int64_t Cin, int64_t Cout, int ksize, int stride,
                       int64_t x_group_c, int64_t x_group_stride);
int ewvit_conv2d_fwd_bn_xf(const void *x, const void *wp, const float *bias, void *y, int64_t N, int64_t H,
                           int64_t W, int64_t Cin, int64_t Cout, int64_t x_group_c, int64_t x_group_stride,
                           const float *xf, const float *bn_shift, float *bn_part, float *bn_shift_out, void *stream);
int ewvit_conv2d_bwd_weight_xf(const void *x, const void *dy, float *dw, float *dbias, int accumulate, int64_t N,
                               int64_t H, int64_t W, int64_t Cin, int64_t Cout, int64_t x_group_c,
                               int64_t x_group_stride, const float *xf, int64_t dw_cin, int64_t dw_s_co,
                               int64_t dw_s_ci, int64_t dw_s_tap, float *workspace, void *stream);
/* The backbone stem, forward only (replaces the library conv of the frozen
 * features.0.0 = Conv2d(3, 24, 3, stride 2, pad 1), reference network/sfe.py:111-119):
 * y [N, Ho, Wo, Cout] bf16 channels-last = conv(x, w) + bias (fp32 operands and accumulation,
 * the output rounded once) for x f32 or bf16 at any element strides (sx_*: the frames'
 * NCHW; x spans < 2 GiB).  w: fp32 tap-major [Cin*9][Cout] (the weight permuted to
 * [Cin][3][3][Cout]), then, if has_bias, one more row [Cout] holding the bias, then >= 64
 * readable floats (scalar loads read 64 bytes at a time).  Cin 1..4, Cout 8/16/24/32,
 * stride 1|2.  bn_part (or NULL) [P][2][Cout] receives per workgroup the shifted
 * BatchNorm sums of the bf16 output as ewvit_conv2d_fwd_bn leaves them,
 * P = ewvit_conv2d_stem_parts(N, H, W, stride); bn_shift_out receives K. */
int64_t ewvit_conv2d_stem_parts(int64_t N, int64_t H, int64_t W, int stride);
int ewvit_conv2d_stem_fwd(const void *x, int x_dtype, int64_t N, int64_t Cin, int64_t H, int64_t W,
                          int64_t sx_n, int64_t sx_c, int64_t sx_h, int64_t sx_w, const float *w,
                          int has_bias, void *y, int64_t Cout, int stride, const float *bn_shift,
                          float *bn_part, float *bn_shift_out, void *stream);
/* dx [N, H, W, Cin] from dy [N, Ho, Wo, Cout] and the transposed pack. */
int ewvit_conv2d_bwd_data(const void *dy, const void *wp_t, void *dx, int64_t N, int64_t H, int64_t W,
                          int64_t Cin, int64_t Cout, int ksize, int stride, int64_t dx_group_c,
                          int64_t dx_group_stride, void *stream);
/* dx = dgrad(dy) + addend (plain NHWC bf16, same layout as dx): a residual block's skip
 * gradient added in the epilogue of its first conv's input gradient (no separate add).
 * Supported when ewvit_conv2d_bwd_data_add_ok(...) returns 1 (the LDS-DMA kernel). */
int64_t ewvit_conv2d_bwd_data_add_ok(int64_t N, int64_t H, int64_t W, int64_t Cin, int64_t Cout, int ksize,
                                     int stride);
int ewvit_conv2d_bwd_data_add(const void *dy, const void *wp_t, void *dx, const void *addend, int64_t N, int64_t H,
                              int64_t W, int64_t Cin, int64_t Cout, int ksize, int stride, void *stream);
/* Stride-1 input gradient (+ addend when not NULL, plain dx, as ewvit_conv2d_bwd_data_add;
 * dx_group_c / dx_group_stride as ewvit_conv2d_bwd_data) that also sums, over its
 * bf16-rounded dx, the backward statistics of the BatchNorm whose output was this conv's
 * input — the MBConv tail / Conv2dNormActivation before the next block's first conv
 * (sfe.py:111-113), the MWT's seperate / fusion BatchNorms before the fusion / multiscale
 * convs (mwt.py:60-72, 112): bx that BN's input in dx's layout (bf16), mean / invstd its saved
 * statistics, gamma / beta or NULL, act 0/1/2, rscale [N] (act 0) the drop-path factor per
 * frame or NULL.  BatchNorm groups: one per channel group of a grouped dx (mean / invstd
 * [groups][group_c]), or, plain dx with bn_group_rows > 0 (a multiple of 128 dividing
 * N*H*W), one per slice of that many rows (mean / invstd [groups][Cin]).  part [groups][rows
 * per group][2 C] gets per 128-row m-tile (sum g, sum g*xhat) as ewvit_dwconv3x3_bwd_data_bn
 * defines them; *nrc_out = rows per group (for ewvit_bn_bwd_partials; fold them with
 * ewvit_bn_fold_partials beyond a few hundred).  Works under a workgroup cap (the persistent
 * walk).  ewvit_conv2d_bwd_bn_rows: m-tiles of 128 dx rows, 0 = shape not supported. */
int64_t ewvit_conv2d_bwd_bn_rows(int64_t N, int64_t H, int64_t W, int64_t Cin, int64_t Cout, int ksize, int stride);
int ewvit_conv2d_bwd_data_bn(const void *dy, const void *wp_t, void *dx, const void *addend, int64_t N, int64_t H,
                             int64_t W, int64_t Cin, int64_t Cout, int ksize, int stride, int64_t dx_group_c,
                             int64_t dx_group_stride, const void *bx, const float *mean, const float *invstd,
                             const float *gamma, const float *beta, int act, const float *rscale,
                             int64_t bn_group_rows, float *part, int *nrc_out, void *stream);
/* bytes of f32 split-K workspace for ewvit_conv2d_bwd_weight. */
int64_t ewvit_conv2d_bwd_weight_workspace(int64_t N, int64_t H, int64_t W, int64_t Cin, int64_t Cout,
                                          int ksize, int stride);
/* dw f32 and, when dbias != NULL, the bias gradient dbias[Cout] = sum of dy over
 * pixels (fused: read from the dy tiles already staged), both (= or +=);
 * deterministic split-K + reduction.  dW element (co, ci, kh*k + kw) for the first
 * dw_cin input channels (the rest are zero padding of x) is written at
 * co*dw_s_co + ci*dw_s_ci + tap*dw_s_tap: the weight parameter's own memory format
 * (contiguous or channels-last), so no layout copy follows. */
int ewvit_conv2d_bwd_weight(const void *x, const void *dy, float *dw, float *dbias, int accumulate,
                            int64_t N, int64_t H, int64_t W, int64_t Cin, int64_t Cout, int ksize,
                            int stride, int64_t x_group_c, int64_t x_group_stride, int64_t dw_cin,
                            int64_t dw_s_co, int64_t dw_s_ci, int64_t dw_s_tap, float *workspace, void *stream);

/* ------------------------------ deferred weight-gradient reductions ---
 * The split-K weight gradients (ewvit_conv2d_bwd_weight's 1x1 and LDS-DMA forms, no bias) and
 * ewvit_dwconv3x3_bwd_fused finish with a reduce launch over their fp32 partial slabs.
 * ewvit_reduce_defer_next(1) marks the calling thread's NEXT such call: its reduce is queued on
 * its stream instead of launched (the call's workspace must then stay allocated, and dw must not
 * be read, until the job has run).  Every later ewvit_conv2d_bwd_weight launch of those two
 * forms on the same stream runs up to 2 queued jobs in extra workgroups ahead of its own tiles;
 * ewvit_reduce_flush(stream) launches whatever is still queued on `stream`.  Summation order
 * is the reduce kernel's: results are bit-identical to the immediate form.  The mark is
 * consumed by the next ewvit_conv2d_bwd_weight / ewvit_dwconv3x3_bwd_fused call whatever path
 * it takes.  ewvit_reduce_pending(stream) counts queued jobs (stream NULL: all streams).
 * Replaces the per-call reduce of torch's weight-gradient convs (reached through
 * network/sfe.py:111-113, the EfficientNetV2-S backbone). */
int ewvit_reduce_defer_next(int on);
int ewvit_reduce_flush(void *stream);
int ewvit_reduce_pending(void *stream);

/* ------------------------------ squeeze-excitation / stochastic-depth add ---
 * The MBConv block tail of the EfficientNetV2-S backbone (torchvision
 * SqueezeExcitation + StochasticDepth, reached via network/sfe.py:111-113) on
 * channels-last [N][HW][C] tensors (dtype bf16 or f32), C % 8 == 0.
 * out[n][c] = scale * sum_hw a (b == NULL) or scale * sum_hw a*b (b != NULL), f32;
 * deterministic; `workspace` holds ewvit_se_reduce_workspace(N, HW, C) bytes.
 *   squeeze: a = x, scale = 1/HW;  excite backward: a = dy, b = x, scale = 1. */
int64_t ewvit_se_reduce_workspace(int64_t N, int64_t HW, int64_t C);
int ewvit_se_reduce(const void *a, const void *b, int dtype, int64_t N, int64_t HW, int64_t C,
                    float scale, float *out, float *workspace, void *stream);
/* y = x * s[n][c] (+ g[n][c] when g != NULL); s, g f32 [N][C].
 *   excite: x, s;  backward: dx = dy * s + dsqueeze / HW. */
int ewvit_se_scale(const void *x, int dtype, const float *s, const float *g, void *y, int64_t N,
                   int64_t HW, int64_t C, void *stream);

/* Squeeze MLP of SqueezeExcitation (torchvision fc1/fc2 1x1 convs + SiLU + Sigmoid on the
 * squeezed [N, C] vector, fp32): h1 = W1 s0 + b1 [N, Csq], s = sigmoid(W2 silu(h1) + b2)
 * [N, C].  W1 [Csq][C], W2 [C][Csq] (the conv weights' memory), b1/b2 may be NULL.
 * Replaces addmm + silu + addmm + sigmoid of the reference block. */
int64_t ewvit_se_mlp_fwd_workspace(int64_t N, int64_t C, int64_t Csq);
int ewvit_se_mlp_fwd(const float *s0, const float *w1, const float *b1, const float *w2, const float *b2,
                     float *h1, float *s, int64_t N, int64_t C, int64_t Csq, float *workspace, void *stream);
int64_t ewvit_se_mlp_bwd_workspace(int64_t N, int64_t C, int64_t Csq);
/* Backward of the squeeze MLP given ds[n, c] = sum_hw dy * x: g = (dL/ds0) * inv_hw (the
 * squeeze's share of dx, consumed by ewvit_se_scale), dW1 [Csq][C], db1, dW2 [C][Csq],
 * db2 (overwritten; db1/db2 may be NULL).  Deterministic (fixed-order sums over N). */
int ewvit_se_mlp_bwd(const float *ds, const float *s, const float *h1, const float *s0, const float *w1,
                     const float *w2, float inv_hw, float *g, float *dw1, float *db1, float *dw2, float *db2,
                     int64_t N, int64_t C, int64_t Csq, float *workspace, void *stream);
/* The squeeze folded into the MLP: s0 = mean_hw x (written out) -> h1, s exactly as
 * ewvit_se_mlp_fwd (workspace ewvit_se_mlp_fwd_workspace bytes), 2 launches; and the
 * backward with ds = sum_hw dy * x computed inside its first kernel, then g, dW1, db1,
 * dW2, db2 as ewvit_se_mlp_bwd (workspace ewvit_se_mlp_bwd_workspace bytes). */
int ewvit_se_squeeze_mlp_fwd(const void *x, int dtype, int64_t N, int64_t HW, int64_t C, const float *w1,
                             const float *b1, const float *w2, const float *b2, int64_t Csq, float *s0, float *h1,
                             float *s, float *workspace, void *stream);
/* The whole squeeze-excitation forward (torchvision SqueezeExcitation, sfe.py:111-113): the
 * squeeze + MLP of ewvit_se_squeeze_mlp_fwd (s0, h1, s written out for the backward) and the
 * excite pass y = x * s[n, c] ([N][HW][C], dtype) — the gates and the excite pass share one
 * launch (2 in all; bit-identical to ewvit_se_squeeze_mlp_fwd + ewvit_se_scale). */
int ewvit_se_forward(const void *x, int dtype, int64_t N, int64_t HW, int64_t C, const float *w1, const float *b1,
                     const float *w2, const float *b2, int64_t Csq, float *s0, float *h1, float *s, void *y,
                     float *workspace, void *stream);
/* ewvit_se_forward's second launch alone: the SE gates from the MLP's first-layer partials part
 * [N][ceil(C / 64)][Csq] (h1, s written out) and the excite pass y = x * s[n, c]. */
int ewvit_se_gate_excite(const float *part, const float *b1, const float *w2, const float *b2, const void *x,
                         int dtype, int64_t N, int64_t HW, int64_t C, int64_t Csq, float *h1, float *s, void *y,
                         void *stream);
int ewvit_se_squeeze_mlp_bwd(const void *dy, const void *x, int dtype, int64_t N, int64_t HW, int64_t C,
                             const float *s, const float *h1, const float *s0, const float *w1, const float *w2,
                             int64_t Csq, float *g, float *dw1, float *db1, float *dw2, float *db2,
                             float *workspace, void *stream);
/* The backward of SE(act(BatchNorm(z))) (MBConv's depthwise BN + act + SE, network/sfe.py:111-113)
 * in one call, 4 launches: ewvit_se_squeeze_mlp_bwd's outputs (g, dw1, db1, dw2, db2) and
 * ewvit_bn_bwd_se's (dx, dgamma, dbeta overwritten), with the BatchNorm's two channel sums split
 * per frame (sum over rows of (dy s + g) act' = sum_n s A_n + g B_n, likewise for the xhat
 * moment) and formed in the SE squeeze pass that streams dy and a anyway — the BN's own
 * reduction pass over dy and z never runs.  a: the SE input act(BN(z)) as the forward stored
 * it; z: the BN input; save_mean / save_invstd from the forward.  C % 8 == 0, C <= 4096.
 * workspace: ewvit_bn_se_bwd_workspace(N, C, Csq) bytes.  dx NULL: 3 launches, no dx pass —
 * dgamma / dbeta are written by the sums pass and the sums row [2C] stays in the workspace at
 * ewvit_bn_se_bwd_row_offset(N, C, Csq) floats for ewvit_dwconv3x3_bwd_fused_se (or
 * ewvit_bn_se_bwd_dx, the dx pass alone). */
int64_t ewvit_bn_se_bwd_workspace(int64_t N, int64_t C, int64_t Csq);
int64_t ewvit_bn_se_bwd_row_offset(int64_t N, int64_t C, int64_t Csq);
int ewvit_bn_se_bwd(const void *dy, const void *a, const void *z, void *dx, int dtype, int64_t N, int64_t HW,
                    int64_t C, const float *gamma, const float *beta, const float *save_mean,
                    const float *save_invstd, int act, float *dgamma, float *dbeta, const float *s,
                    const float *h1, const float *s0, const float *w1, const float *w2, int64_t Csq, float *g,
                    float *dw1, float *db1, float *dw2, float *db2, float *workspace, void *stream);
int ewvit_bn_se_bwd_dx(const void *dy, const void *z, void *dx, int dtype, int64_t N, int64_t HW, int64_t C,
                       const float *gamma, const float *beta, const float *save_mean, const float *save_invstd,
                       int act, const float *s, const float *g, const float *row, void *stream);
/* y = r * scale[n] (+ x when x != NULL) over N rows of row_elems elements (row_elems % 8 == 0):
 * StochasticDepth(mode='row') with its keep/(1-p) factor fused with the skip add. */
int ewvit_scale_add(const void *r, const void *x, int dtype, const float *scale, void *y, int64_t N,
                    int64_t row_elems, void *stream);
/* The same add with the StochasticDepth(row) keep mask drawn in-kernel: scale[n] =
 * (u < keep_prob) / keep_prob, u uniform in [0,1) from the counter hash of (seed +
 * *seed_offset * golden, n) as ewvit dropout draws it; scale_out[n] receives the
 * factors (the backward's ewvit_scale_add scale). */
int ewvit_scale_add_drop(const void *r, const void *x, int dtype, float keep_prob, uint64_t seed,
                         const int64_t *seed_offset, float *scale_out, void *y, int64_t N, int64_t row_elems,
                         void *stream);

/* ------------------------------------------------------ pooling ---
 * MaxPool2d(2) (kernel 2, stride 2, floor mode) of the MWT freq_pool (mwt.py:38-44) on
 * channels-last [N, H, W, C] (C % 8 == 0): y [N, H/2, W/2, C] and argmax (uint8 window
 * slot 0..3 per output element, torch's first-maximum / NaN rule); the backward writes
 * every dx element once (dy at the slot, 0 elsewhere and in a floor-mode remainder). */
int ewvit_maxpool2_fwd(const void *x, void *y, uint8_t *argmax, int dtype, int64_t N, int64_t H, int64_t W,
                       int64_t C, void *stream);
int ewvit_maxpool2_bwd(const void *dy, const uint8_t *argmax, void *dx, int dtype, int64_t N, int64_t H, int64_t W,
                       int64_t C, void *stream);

/* ------------------------------------------------------ optimizer ---
 * Adam exactly as torch.optim.Adam (amsgrad=False, maximize=False): g += wd*p;
 * m = b1 m + (1-b1) g; v = b2 v + (1-b2) g^2; p -= lr/(1-b1^t) * m / (sqrt(v)/sqrt(1-b2^t) + eps)
 * with t = *steps[i] (per-tensor device f32, advanced by the caller first) and lr = *lr_dev when
 * lr_dev is non-null (device f64, so a replayed HIP graph follows an LR schedule the caller
 * writes between replays: CosineAnnealingLR of train.py:274,300), else `lr` — the optimizer of the
 * reference's training step (train.py:273-275).  n <= EWVIT_ADAM_MAX f32 tensors per
 * launch (pointers by value: capturable although autograd reallocates the gradients);
 * p, g, m, v of a tensor share one memory order (any dense layout), numel elements. */
int ewvit_adam_step(int n, float *const *params, const float *const *grads, float *const *exp_avg,
                    float *const *exp_avg_sq, const int64_t *numel, const float *const *steps, double lr,
                    const double *lr_dev, double beta1, double beta2, float eps, float weight_decay, void *stream);
/* The same update for any number of tensors in ONE launch: `table` is a DEVICE array of n
 * entries of EWVIT_ADAM_ENTRY int64 words {p, g, m, v, step (pointers), numel, first chunk},
 * first chunks ascending from 0 with ewvit_adam_chunks(numel) chunks per tensor, nchunks the
 * total.  A caller whose tensors keep their addresses builds the table once (a replayed HIP
 * graph then runs the whole group as one kernel). */
#define EWVIT_ADAM_ENTRY 7
int64_t ewvit_adam_chunks(int64_t numel);
int ewvit_adam_step_table(const int64_t *table, int n, int64_t nchunks, double lr, const double *lr_dev, double beta1,
                          double beta2, float eps, float weight_decay, void *stream);

/* ------------------------------------------------------ loss ---
 * combined_loss of train.py:69-91 with orthogonal_loss of train.py:55-67, forward and all input
 * gradients in one launch: out[0] = cls + w * orth, out[1] = cls = BCEWithLogits(logits, labels,
 * pos_weight, mean), out[2] = orth = ||offdiag(normalize(space)^T normalize(freq))||_F^2 /
 * (D (D - 1)); d_logits / d_space / d_freq = d out[0] / d input.  w = *weight (device f32) when
 * weight is non-null (the curriculum weight a replayed step reads), else lam.  logits / labels
 * [B], space / freq / d_* [B, D] f32 row-major, pos_weight device f32[1] or NULL (1);
 * 1 <= B <= 64, 4 * B * D floats <= 64 KB. */
int ewvit_combined_loss(const float *logits, const float *labels, const float *space, const float *freq, int64_t B,
                        int64_t D, const float *pos_weight, const float *weight, float lam, float *out,
                        float *d_logits, float *d_space, float *d_freq, void *stream);

/* ----------------------------------------------------- MWT seperate convs (csrc/hfsep.hip) ---
 * hf_conv['seperate'][g] for g = 0..2 (reference network/mwt.py:48-59: Conv2d(3, 18, 3, pad 1) per
 * colour, applied to channels 3g..3g+2 of the level's HF input at mwt.py:84-86, weights shared by the
 * levels, mwt.py:108) for every level in one launch — the grouped conv it is (1458 MACs per pixel).
 *   x   [L*N][H][W][x_channels] bf16 channels-last, level-major (ewvit_dwt_hf_upsample_fused's
 *       output: channel 3g+ci real for g, ci < 3; x_channels 16: channels 9..15 zero, x_channels 9:
 *       the 9 band channels only, W even — the kernels zero-pad K in LDS)
 *   y   [L*N][H][W][64] bf16: channel 18g+o for o < 18; channels 54..63 written as zero
 *   w_g [18][3][3][3] fp32, b_g [18] fp32 (the three modules' parameters, contiguous)
 * ewvit_hfsep_fwd also leaves, when bn_part is not NULL, the BatchNorm partial statistics of the
 * bf16 y per level for ewvit_bn_fwd_partials (groups = L): bn_part [L][nparts][128] (sum (y - K),
 * sum (y - K)^2 per channel, K = bn_shift[c] for c < 54 (NULL: 0), else 0) and bn_shift_out [L][64]
 * = K; nparts must equal ewvit_hfsep_fwd_parts(L, N, H, W) under the same grid cap.
 * ewvit_hfsep_bwd_weight overwrites dw_g [18][3][3][3] and db_g [18] (any may be NULL) from dy
 * [L*N][H][W][64] bf16 and x; workspace: ewvit_hfsep_bwd_weight_workspace(L*N, H, W) bytes.
 * W <= 512. */
int64_t ewvit_hfsep_fwd_parts(int64_t L, int64_t N, int64_t H, int64_t W);
int ewvit_hfsep_fwd(const void *x, void *y, int64_t L, int64_t N, int64_t H, int64_t W, int x_channels, const float *w0,
                    const float *w1, const float *w2, const float *b0, const float *b1, const float *b2,
                    const float *bn_shift, float *bn_part, float *bn_shift_out, int nparts, void *stream);
int64_t ewvit_hfsep_bwd_weight_workspace(int64_t NI, int64_t H, int64_t W);
int ewvit_hfsep_bwd_weight(const void *x, const void *dy, int64_t NI, int64_t H, int64_t W, int x_channels, float *dw0, float *dw1,
                           float *dw2, float *db0, float *db1, float *db2, float *workspace, void *stream);

/* The seperate conv's weight gradients THROUGH the grouped BatchNorm + ReLU that follows it
 * (mwt.py:48-59: Conv -> BatchNorm2d(18) -> ReLU per colour; per-level batch statistics): the
 * BN backward's dx pass is recomputed per element inside the weight-gradient pass instead of
 * being written out.  y: the conv output / BN input [L*N][H][W][64] bf16; dz: the gradient of
 * the BN + ReLU output (same layout); mean / invstd [L][64] the BN forward's batch statistics;
 * gamma / beta [64]; part [L][nrc][128]: per channel sum g' and sum g' xhat (g' = dz masked by
 * the ReLU), as the consumer conv's input-gradient epilogue leaves them (ewvit_bn_fold_partials
 * shape).  Writes dw_g, db_g as ewvit_hfsep_bwd_weight and dgamma = sum g' xhat, dbeta = sum g'
 * [64] (summed over the levels); any output may be NULL.  workspace:
 * ewvit_hfsep_bn_bwd_weight_workspace(L, N, H, W) bytes. */
/* The reduction pass of ewvit_bn_bwd alone, for a consumer that forms the BN's dx itself:
 * part [groups][nrc][2][C] = per channel sum g and sum g * xhat (g = dy * act'(BN output)),
 * nrc = ewvit_bn_bwd_reduce_rows(M, C, groups) (0: bad shape). */
int ewvit_bn_bwd_reduce_rows(int64_t M, int64_t C, int groups);
int ewvit_bn_bwd_reduce(const void *dy, const void *x, int dtype, int64_t M, int64_t C, const float *gamma,
                        const float *beta, const float *save_mean, const float *save_invstd, int act, int groups,
                        float *part, void *stream);
int64_t ewvit_hfsep_bn_bwd_weight_workspace(int64_t L, int64_t N, int64_t H, int64_t W);
int ewvit_hfsep_bn_bwd_weight(const void *x, const void *y, const void *dz, int64_t L, int64_t N, int64_t H, int64_t W,
                              int x_channels, const float *mean, const float *invstd, const float *gamma, const float *beta,
                              const float *part, int nrc, float *dw0, float *dw1, float *dw2, float *db0, float *db1,
                              float *db2, float *dgamma, float *dbeta, float *workspace, void *stream);

/* ------------------------------------------------------ frames (input side) ---
 * The per-frame transform chain of config/transforms.py:81-113 applied by the datasets'
 * __getitem__ (config/data_loader.py:325-337: cv2.imread -> BGR2RGB -> transform(frame) per
 * frame -> torch.stack), on a batch of frames at once and bit-identical to Pillow +
 * torchvision: crop box (FaceAlignTransform, transforms.py:28-79) -> Resize(450) (Pillow
 * bilinear, 8-bpc fixed point) -> CenterCrop(S) -> [ColorJitter(brightness, contrast)] ->
 * ToTensor -> Normalize(mean, std).
 *   frames  one buffer of nbytes uint8 holding the RGB frames, HWC, each at its own offset
 *   geom    [n][10] int64: byte offset of the frame, bytes per frame row, crop box left, top,
 *           width, height (inside the frame), Resize output width, height (torchvision's
 *           short-side rule), CenterCrop offsets x, y (round((size - S) / 2))
 *   mean_std  host float[6]: mean[3], std[3]
 * ewvit_frames_plan (host-only, geom in HOST memory): validates every frame (box inside the
 * buffer, S <= 256, crop inside the resized image, downscale <= 8x) and fills plan[4] (output
 * rows per workgroup, taps, source rows per workgroup, staged dwords per source row) for
 * ewvit_frames_resize_crop; returns 0 or EWVIT_EINVAL.
 * ewvit_frames_resize_crop (geom in DEVICE memory, plan in host memory): out = to_f32 ?
 * [n][3][S][S] normalised f32 : [n][S][S][3] uint8 (the PIL image after CenterCrop).
 * ewvit_frames_jitter_normalize: ColorJitter + ToTensor + Normalize of that uint8 image;
 * jitter [n][4] f32 device: brightness factor, contrast factor (< 0: absent), order (0:
 * brightness first, 1: contrast first — torchvision's randperm(4) restricted to ids 0 / 1),
 * unused; out [n][3][S][S] f32. */
int ewvit_frames_plan(const int64_t *geom, int64_t n, int S, int64_t nbytes, int *plan);
int ewvit_frames_resize_crop(const uint8_t *frames, const int64_t *geom, int64_t n, int S, const int *plan,
                             int to_f32, const float *mean_std, void *out, void *stream);
int ewvit_frames_jitter_normalize(const uint8_t *img, const float *jitter, int64_t n, int S, const float *mean_std,
                                  float *out, void *stream);

/* ------------------------------------------------ DAMA frame head ---
 * Everything of DAMA._process_frame after its two branches (reference network/dama.py:143-169):
 * the BidirectionalCrossTransformer (depth 2: per layer s = s + CA(LN(s), f), then
 * f = f + CA(LN(f), s); CrossAttention dama.py:15-53 with kv_include_self, 4 heads of 32,
 * to_out + Dropout), the fusion gate (Conv3x3(256 -> 128, pad 1) on the 1x1 map = its centre
 * tap, + BatchNorm2d + ReLU, dama.py:124-128), the gate net (Linear 256 -> 64, ReLU, Dropout,
 * Linear 64 -> 3, Softmax, dama.py:105-113) and the weighted sum (dama.py:159-163), for
 * N <= 64 frames of dim 128.  Replaces ~90 module-level launches of the forward and backward.
 * The fp32 master parameters are read in place (bf16 MFMA operands, fp32 accumulation). */
typedef struct {
  const float *ln_w, *ln_b;   /* the block's pre-norm LayerNorm(128) weight / bias */
  const float *wq;            /* to_q.weight [128][128] */
  const float *wkv;           /* to_kv.weight [256][128] */
  const float *wo, *bo;       /* to_out[0].weight [128][128], bias [128] */
} ewvit_head_ca;
typedef struct {
  ewvit_head_ca ca[4];        /* layer 0 space, layer 0 freq, layer 1 space, layer 1 freq */
  const float *wfg;           /* fusion_gate[0].weight [128][256][3][3]: element (o, i, tap) at */
  int64_t fg_so, fg_si, fg_tap; /*   o * fg_so + i * fg_si + tap * fg_tap (centre tap 4) */
  const float *bfg;           /* fusion_gate[0].bias [128] */
  const float *bn_w, *bn_b;   /* fusion_gate[1] BatchNorm2d affine */
  float *bn_rm, *bn_rv;       /* its running statistics (updated in training) */
  int64_t *bn_nbt;            /* its num_batches_tracked (incremented in training; may be NULL) */
  float bn_mom, bn_eps;
  const float *g1w, *g1b;     /* gate_net[2]: Linear(256, 64) */
  const float *g2w, *g2b;     /* gate_net[5]: Linear(64, 3) */
  float p_ca, p_gate;         /* dropout probabilities (to_out, gate_net[4]; 0 in eval) */
  uint64_t seed;              /* dropout: counter hash of (seed + *seed_off * golden, site, n, c) */
  const int64_t *seed_off;
  int training;               /* BatchNorm batch statistics + running-stat update */
  float ln_eps;
  void *packed;               /* ewvit_head_pack_bytes() of scratch: the weights as bf16, packed
                               * by ewvit_head_fwd and read by it and by ewvit_head_bwd */
  void *packed_mx;            /* NULL: bf16 attention GEMMs; else ewvit_head_pack_bytes_mx() of
                               * scratch: to_q / to_kv / to_out as MXFP8 (ewvit_gemm_mx8's
                               * format, both orientations), packed by ewvit_head_fwd — every
                               * attention-block GEMM (fwd, input and weight gradients) then runs
                               * on MXFP8 operands (configs[4]); the fusion conv / gate stay bf16 */
} ewvit_head_params;
/* bytes of fp32 workspace the head needs (what the forward saves for the backward) */
int64_t ewvit_head_workspace(void);
/* bytes of the bf16 weight pack (ewvit_head_params.packed) */
int64_t ewvit_head_pack_bytes(void);
/* bytes of the MXFP8 attention-weight pack (ewvit_head_params.packed_mx) */
int64_t ewvit_head_pack_bytes_mx(void);
/* s0, f0 [N][128] f32: the space / freq tokens (one per frame) -> fused, s_out, f_out [N][128]
 * (dama.py:165-169's fused / space / freq per frame); the workspace keeps what the backward
 * reads; one workgroup. */
int ewvit_head_fwd(const ewvit_head_params *p, const float *s0, const float *f0, int N, float *workspace,
                   float *fused, float *s_out, float *f_out, void *stream);
/* Backward from the forward's workspace: g_fused, g_s, g_f [N][128] -> ds0, df0 [N][128] and
 * every parameter gradient (overwritten): per attention block i (arrays of 4) to_q / to_kv /
 * to_out weight and bias, LayerNorm weight / bias; the fusion conv's full [128][256][3][3]
 * gradient at wfg with strides (fg_so, fg_si, fg_tap) (the 8 dead taps: 0), its bias, the
 * BatchNorm affine, gate_net's two linears.  One workgroup for the activation gradients, then
 * one grid for the weight gradients (fp32 sums over the frames in a fixed order). */
int ewvit_head_bwd(const ewvit_head_params *p, const float *workspace, int N, const float *g_fused,
                   const float *g_s, const float *g_f, float *ds0, float *df0, float *const *wq,
                   float *const *wkv, float *const *wo, float *const *bo, float *const *lnw,
                   float *const *lnb, float *wfg, int64_t fg_so, int64_t fg_si, int64_t fg_tap, float *bfg,
                   float *bn_w, float *bn_b, float *g1w, float *g1b, float *g2w, float *g2b, void *stream);

/* ------------------------------------------------ ViT encoder layer ---
 * One pre-norm layer of the spatial branch's Transformer (reference network/sfe.py:72-85):
 *   x1 = x0 + Dropout(to_out(Attention(LayerNorm(x0))))      (sfe.py:20-27, 42-70)
 *   x2 = x1 + Linear2(GELU(Linear1(LayerNorm(x1))))         (sfe.py:29-40, FeedForward dropout 0)
 * at the hot path's shape: dim 512, 8 heads of 64, mlp 2048, 2 tokens per frame (CLS + the one
 * 7x7 patch), R = 2 * frames <= 128 rows (row 2b + i = token i of frame b).  Replaces the 11
 * forward / ~25 backward module-level launches of the layer (LayerNorm, to_qkv, attention,
 * to_out, LayerNorm, two Linears, the split-K reduces, act / dropout backward, column sums)
 * with 4 forward / 5 backward launches.  fp32 master parameters read in place (bf16 MFMA
 * operands, fp32 accumulation, the module path's roundings); the dropout mask of to_out is the
 * module path's: keep(seed + *seed_off * golden, row * 512 + col). */
typedef struct {
  const float *ln1_w, *ln1_b;   /* layers[i][0].norm: LayerNorm(512) */
  const float *wqkv;            /* to_qkv.weight [1536][512] (no bias) */
  const float *wo, *bo;         /* to_out[0]: [512][512], [512] */
  const float *ln2_w, *ln2_b;   /* layers[i][1].norm */
  const float *w1, *b1;         /* net[0]: [2048][512], [2048] */
  const float *w2, *b2;         /* net[3]: [512][2048], [512] */
  float ln_eps, drop_p;         /* LayerNorm eps; to_out dropout probability (0 in eval) */
  uint64_t seed;
  const int64_t *seed_off;
  const void *packed;           /* this layer's block of ewvit_vit_pack's output (bf16 weights), or
                                   of ewvit_vit_pack_mx's when mx != 0 */
  int mx;                       /* 1: every GEMM of the layer on MXFP8 operands (configs[4]; see
                                   ewvit_gemm_mx8): weights from the MX pack, activations and
                                   gradients block-quantized by the kernels that form their
                                   fragments, fp32 accumulation; 0: bf16 */
} ewvit_vit_layer;
typedef struct {                /* parameter gradients (overwritten), parameter layouts */
  float *ln1_w, *ln1_b, *wqkv, *wo, *bo, *ln2_w, *ln2_b, *w1, *b1, *w2, *b2;
} ewvit_vit_grads;
/* bytes of the forward's saved state (which = 0), of the backward's scratch (which = 1), of
 * one layer's packed bf16 weights (which = 2) and of one layer's MXFP8 pack (which = 3) */
int64_t ewvit_vit_layer_workspace(int which);
#define EWVIT_VIT_PACK_MAX 8
/* The n <= EWVIT_VIT_PACK_MAX layers' to_qkv / to_out / Linear1 / Linear2 weights (fp32, read
 * from layers[i]) as bf16, each in its own layout and transposed, into n consecutive blocks of
 * ewvit_vit_layer_workspace(2) bytes: the GEMM operands of ewvit_vit_layer_fwd / _bwd, packed
 * once per step (the module path rounds the same weights to bf16 inside every GEMM). */
int ewvit_vit_pack(const ewvit_vit_layer *layers, int n, void *packed, void *stream);
/* The same weights as MXFP8 (ewvit_gemm_mx8's format) into n blocks of
 * ewvit_vit_layer_workspace(3) bytes: per weight W [out][in] the e4m3 image with one E8M0 scale
 * per 32 consecutive `in` elements, and W^T [in][out] with one per 32 `out` elements (the K of
 * the forward and of the input-gradient GEMMs), quantized once per step from the fp32 masters. */
int ewvit_vit_pack_mx(const ewvit_vit_layer *layers, int n, void *packed, void *stream);
/* x0 [R][512] f32 -> x2 [R][512] f32; `saved` (ewvit_vit_layer_workspace(0) bytes) keeps what
 * the backward reads (LayerNorm statistics, qkv, softmax weights, the GEMM operands). */
int ewvit_vit_layer_fwd(const ewvit_vit_layer *p, int R, const float *x0, void *saved, float *x2, void *stream);
/* g = dL/dx2 [R][512] f32 -> dx0 [R][512] f32 and every parameter gradient. */
int ewvit_vit_layer_bwd(const ewvit_vit_layer *p, int R, const float *x0, const void *saved, const float *g,
                        void *scratch, float *dx0, const ewvit_vit_grads *grads, void *stream);
/* The token sequence of sfe.py:155-160 for one 7x7 patch per frame: tok [B][2][512] f32 with
 * tok[b][0] = cls + pos[b], tok[b][1] = y[b] + pos[b] (y = patch_to_embedding output [B][512],
 * cls [512], pos = pos_embedding rows [npos >= B][512], EINVAL otherwise), then Dropout(drop_p) (emb_dropout; keep mask
 * keep(seed + *seed_off * golden, (2 b + i) * 512 + c)).  Replaces torch.cat + add + nn.Dropout. */
int ewvit_vit_embed_fwd(const float *y, const float *cls, const float *pos, int B, int npos, float drop_p,
                        uint64_t seed, const int64_t *seed_off, float *tok, void *stream);
/* Backward: dtok [B][2][512] -> dy [B][512], dcls [512] (sum over frames, fixed order), dpos [npos][512]
 * (npos <= 64; rows >= B written 0: the pos_embedding[0:B] slice's gradient). */
int ewvit_vit_embed_bwd(const float *dtok, int B, int npos, float drop_p, uint64_t seed, const int64_t *seed_off,
                        float *dy, float *dcls, float *dpos, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* EWVIT_H */
