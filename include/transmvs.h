/*
 * transmvs.h -- C-ABI of the MI355X-native TransMVSNet depth-inference hot path.
 *
 * The reference (delldu/TransMVSNet) is pure PyTorch; its "operator API" for this path is
 * the set of Python callables the north star names. Each entry point below replaces one of
 * them (reference file:line cited) and is what a ctypes / cffi / pybind binding binds
 * (see INTEGRATION.md). Conventions, identical for every entry point:
 *
 *   - extern "C", stateless, re-entrant; no allocation and no host synchronisation inside
 *     a call (graph-capturable); scratch memory is passed in by the caller.
 *   - every tensor argument is a DEVICE pointer to fp32 data unless marked HOST; sizes and
 *     strides are explicit ints; layouts are stated per argument. "NHWC" = channels-last.
 *   - `stream` is a hipStream_t passed as void* (NULL = legacy default stream).
 *   - return value: TMVS_OK (0) or a negative status (bad argument, unsupported shape,
 *     HIP launch error); tmvs_status_string() names it. A failing call launches nothing
 *     on bad arguments/shapes.
 */
#ifndef TRANSMVS_H_
#define TRANSMVS_H_

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TMVS_ABI_VERSION 9

#define TMVS_OK 0
#define TMVS_ERR_ARG (-1)    /* null pointer / non-positive size / bad enum        */
#define TMVS_ERR_SHAPE (-2)  /* shape the kernels do not support (e.g. D % 8 != 0) */
#define TMVS_ERR_HIP (-3)    /* hipGetLastError() reported a launch failure       */

#define TMVS_MAX_VIEWS 16    /* source views per warp_corr launch                  */

int tmvs_abi_version(void);
const char* tmvs_status_string(int status);

/* ------------------------------------------------------------------ host helpers
 * Eval-mode BatchNorm as the reference's PyTorch-CPU kernel evaluates it
 * (nn.BatchNorm{2,3}d, models/module.py:132,173,218):
 *   alpha = (1 / sqrtf(var + eps)) * gamma;   shift = fmaf(-mean, alpha, beta);
 *   y     = fmaf(x, alpha, shift).
 * All pointers HOST. */
int tmvs_bn_fold(const float* gamma, const float* beta, const float* mean, const float* var, int n, float eps,
                 float* alpha, float* shift);

/* ------------------------------------------------------------------ stage glue
 * Depth hypotheses of one cascade stage: get_depth_samples (models/module.py:606-634) plus
 * the bilinear up-sampling of the previous stage's depth and the trilinear resampling to
 * the stage resolution (models/TransMVSNet.py:147-149,174-204), fused, without the
 * full-resolution [B,D,H,W] intermediate.
 *   depth_values : [B][n_values]     (the forward's depth_values input; [0,0] and [0,-1] of
 *                                     batch 0 give depth_interval, as at TransMVSNet.py:147-149)
 *   prev_depth   : [B][prev_h][prev_w] previous stage's UNCLAMPED WTA depth, or NULL (stage 1)
 *   ndepth, ratio: this stage's hypothesis count and interval ratio (TransMVSNet.py:113-114)
 *   full_h/full_w: image size; stage_scale: 4, 2 or 1 (TransMVSNet.py:128-132)
 *   hyp_out      : [B][ndepth][full_h/stage_scale][full_w/stage_scale]                      */
int tmvs_stage_hypotheses(const float* depth_values, int n_values, const float* prev_depth, int prev_h, int prev_w,
                          int batch, int ndepth, float ratio, int full_h, int full_w, int stage_scale,
                          float* hyp_out, void* stream);

/* ------------------------------------------------------------------ cost volume
 * Fused DepthNet steps 1-2 (models/TransMVSNet.py:58-93): for every source view the
 * homography warp + bilinear grid_sample of homo_warping (models/module.py:284-322), the
 * single-group correlation (warped*ref).mean(C) (TransMVSNet.py:80), the stage-1 view
 * weight PixelwiseNet (TransMVSNet.py:10-30) or the given up-sampled weights (:86), and the
 * weighted view aggregation Σ w·sim / (1e-5 + Σ w) (:71-72,88-93). The [C,D,H,W] warped
 * volume is never materialised.
 *   ref_fea      : [B][H][W][C] (NHWC)      src_fea : [B][V][H][W][C] (NHWC)
 *   proj         : HOST [B][V][12] = rows of (P_src · P_ref^-1)[:3,:4]  (module.py:295-297)
 *   hyp          : [B][D][H][W]
 *   view_w_in    : NULL (stage 1: compute with PixelwiseNet) or [B][vw_total][H>>vw_shift][W>>vw_shift]
 *                  (stages 2/3: nearest x2^vw_shift up-sampling, TransMVSNet.py:194);
 *                  this call's views are vw_offset .. vw_offset+V-1 of it
 *   pw_params    : HOST, TMVS_PW_NPARAMS floats (layout below), used when view_w_in == NULL
 *   flags        : TMVS_WARP_PARTIAL -> write sim_out = Σ_v w_v·sim_v and wsum_out = Σ_v w_v
 *                  undivided (view-sharded mode; finish with tmvs_aggregate_finalize after the
 *                  all-reduce); 0 -> sim_out = the reference's normalised similarity.
 *                  TMVS_WARP_ROT_PLAIN -> rot·(x,y,1) as (r0·x + r1·y) + r2, the rounding of the
 *                  reference's torch.matmul (module.py:303) where the host BLAS does not contract
 *                  it (MKL on AMD EPYC); without it fmaf(r1, y, r0·x) + r2 (MKL on AVX-512 Xeons).
 *                  The two differ by up to 1.2e-4 px in the sample coordinate.
 *   sim_out      : [B][D][H][W]       wsum_out : [B][H][W] (PARTIAL only, else may be NULL)
 *   view_w_out   : [B][vw_total][H][W] written at vw_offset.. when view_w_in == NULL
 * Supported: C in {8,16,32}; D in {8,16,24,32,48,64}; 1 <= V <= TMVS_MAX_VIEWS;
 *            V*H*W*C*4 < 2^30 bytes per sample (32-bit buffer offsets); H, W <= 32766.      */
#define TMVS_WARP_PARTIAL 1
#define TMVS_WARP_ROT_PLAIN 2
#define TMVS_WARP_BWD_PLANES 4 /* tmvs_warp_corr_backward: hyp[d] is one depth per plane (stage 1) */
#define TMVS_PW_NPARAMS 201 /* w0[16] a0[16] s0[16] w1[8][16] a1[8] s1[8] w2[8] b2 */
int tmvs_warp_corr(const float* ref_fea, const float* src_fea, const float* proj, const float* hyp,
                   const float* view_w_in, int vw_shift, int vw_offset, int vw_total, const float* pw_params,
                   int batch, int n_src, int channels, int ndepth, int height, int width, int flags,
                   float* sim_out, float* wsum_out, float* view_w_out, void* stream);

/* sim = sim_sum / (1e-5 + w_sum) after a cross-rank all-reduce of both (TransMVSNet.py:72,93). */
int tmvs_aggregate_finalize(float* sim_sum, const float* w_sum, int batch, int ndepth, int height, int width,
                            void* stream);

/* Materialising homo_warping (models/module.py:284-322) for the reference seam / tests:
 *   src_fea [B][C][H][W] (NCHW), proj HOST [B][12], hyp [B][D][H][W] -> out [B][C][D][H][W];
 *   flags: TMVS_WARP_ROT_PLAIN as for tmvs_warp_corr. */
int tmvs_homo_warping(const float* src_fea, const float* proj, const float* hyp, int batch, int channels,
                      int ndepth, int height, int width, int flags, float* out, void* stream);

/* ------------------------------------------------------------------ CostRegNet
 * 3-D U-Net of models/module.py:425-456 on an NDHWC volume, eval-mode BN folded into a
 * per-channel (alpha, shift) epilogue (tmvs_bn_fold). Weight packing ("packed" below):
 *   Conv3d weight [Co][Ci][3][3][3]          -> [27][Co][Ci]  (tap = kd*9+kh*3+kw)
 *   ConvTranspose3d weight [Ci][Co][3][3][3] -> [27][Co][Ci]
 * (conv0, Ci=1, is thus [27][Co].) prob (Co=1, Ci=C) is packed per kh row:
 *   [kh][ {W[c][kd=1][kh][kw], W[c][kd=2][kh][kw]} for (kw, c) | W[c][kd=0][kh][kw] for (kw, c) ]  */
typedef struct {
  const float* w[11];      /* conv0..conv6, conv7, conv9, conv11 (packed), prob [3][72]     */
  const float* alpha[10];  /* BN alpha of the first 10 layers                              */
  const float* shift[10];  /* BN shift                                                     */
  int base_ch;             /* cr_base_chs (models/TransMVSNet.py:115), 8                   */
} TmvsCostRegWeights;

/* bytes of scratch tmvs_costregnet needs for a [B][D][H][W] volume */
size_t tmvs_costregnet_workspace(int batch, int depth, int height, int width, int base_ch);
/* x: [B][D][H][W] (=NDHWC with C=1), logits: [B][D][H][W]. Needs D,H,W % 8 == 0. */
int tmvs_costregnet(const float* x, int batch, int depth, int height, int width, const TmvsCostRegWeights* w,
                    void* workspace, size_t workspace_bytes, float* logits, void* stream);
/* CostRegNet + softmax/WTA in one call (models/TransMVSNet.py:97-103,214-221): for ndepth <= 32
 * the prob conv, the softmax over D and the winner-take-all run as one kernel (the logits stay in
 * LDS and never reach HBM); for 48 and 64 the depth-chunked prob kernel + tmvs_softmax_wta. Outputs and their bits are those of tmvs_costregnet -> tmvs_softmax_wta.
 * Same workspace as tmvs_costregnet; ndepth in {8, 16, 24, 32, 48, 64}.                        */
int tmvs_costregnet_wta(const float* x, const float* hyp, int batch, int depth, int height, int width,
                        const TmvsCostRegWeights* w, void* workspace, size_t workspace_bytes, float clamp_lo,
                        float clamp_hi, float* prob, float* depth_out, float* depth_raw, float* conf, void* stream);

/* Single layers (Conv3d / Deconv3d blocks, models/module.py:108-191), NDHWC in and out.
 * conv: stride 1 or 2, padding 1;  y = relu(fmaf(conv, alpha, shift)).
 * deconv: ConvTranspose3d k3 s2 p1 op1 (output 2x input);  y = skip + relu(fmaf(...)).    */
int tmvs_conv3d_bn_relu(const float* x, int batch, int cin, int d, int h, int w, const float* wpk, const float* alpha,
                        const float* shift, int cout, int stride, float* y, void* stream);
int tmvs_deconv3d_bn_relu_add(const float* x, int batch, int cin, int d, int h, int w, const float* wpk,
                              const float* alpha, const float* shift, int cout, const float* skip, float* y,
                              void* stream);

/* ------------------------------------------------------------------ regression
 * prob = exp(log_softmax(logits, D)) (TransMVSNet.py:99); winner-take-all
 * argmax (first maximum) + gather (module.py:474-482, TransMVSNet.py:217-218);
 * photo_confidence = max_D prob (:103); depth clamped to [clamp_lo, clamp_hi] (:221).
 *   logits, hyp, prob: [B][D][H][W];  depth (clamped), depth_raw (unclamped), conf: [B][H][W] */
int tmvs_softmax_wta(const float* logits, const float* hyp, int batch, int ndepth, int height, int width,
                     float clamp_lo, float clamp_hi, float* prob, float* depth, float* depth_raw, float* conf,
                     void* stream);

/* ------------------------------------------------------------------ FMT
 * Feature Matching Transformer (models/FMT.py), d_model 32, 8 heads x 4, linear attention.
 * Tokens are [nv][L][32] (= NHWC of the stage-1 map). Packed EncoderLayer weights
 * (TMVS_ENC_NPARAMS floats, offsets TMVS_ENC_*); nn.Linear weights are [out][in] except the
 * K/V projections and linear2, stored transposed ([in][out]) for the rank-1-update kernels:
 *   Wq[32][32] bq[32] WkT[32][32] bk[32] WvT[32][32] bv[32] Wo[32][32] bo[32]
 *   W1[64][32] b1[64] W2T[64][32] b2[32] ln1_g[32] ln1_b[32] ln2_g[32] ln2_b[32]            */
#define TMVS_ENC_WQ 0
#define TMVS_ENC_BQ 1024
#define TMVS_ENC_WK 1056
#define TMVS_ENC_BK 2080
#define TMVS_ENC_WV 2112
#define TMVS_ENC_BV 3136
#define TMVS_ENC_WO 3168
#define TMVS_ENC_BO 4192
#define TMVS_ENC_W1 4224
#define TMVS_ENC_B1 6272
#define TMVS_ENC_W2T 6336
#define TMVS_ENC_B2 8384
#define TMVS_ENC_LN1G 8416
#define TMVS_ENC_LN1B 8448
#define TMVS_ENC_LN2G 8480
#define TMVS_ENC_LN2B 8512
#define TMVS_ENC_NPARAMS 8544
#define TMVS_KV_NFLOATS 160 /* per view: KV[8 heads][4 m][4 d] then Ksum[8][4] */

/* x + PositionEncodingSine (models/position_encoding.py:55-60) and 'n c h w -> n (h w) c'
 * (FMT.py:152,168):  feat [nv][C][H][W] (NCHW, per-view stride feat_view_stride floats),
 * pe [C][pe_h][pe_w] -> tokens [nv][H*W][C]. */
int tmvs_fmt_embed(const float* feat, long feat_view_stride, const float* pe, int pe_h, int pe_w, int nv,
                   int channels, int height, int width, float* tokens, void* stream);
/* bytes of scratch for tmvs_fmt_kv over nv views of S tokens */
size_t tmvs_fmt_kv_workspace(int nv, int s_tokens);
/* K = elu(Wk x + bk) + 1, V = Wv x + bv over the source tokens; KV = Σ_s K⊗V, Ksum = Σ_s K
 * (FMT.py:23-32). source [nv][S][32] -> kv [nv][TMVS_KV_NFLOATS]. */
int tmvs_fmt_kv(const float* source, int nv, int s_tokens, const float* enc_w, void* workspace,
                size_t workspace_bytes, float* kv, void* stream);
/* tmvs_fmt_kv with the partial-sum grouping of a group_nv-view launch: each view's kv is bitwise what a
 * tmvs_fmt_kv over group_nv views (this view among them) gives, for any subset of views (FMT.py:23-32). */
size_t tmvs_fmt_kv_grouped_workspace(int nv, int group_nv, int s_tokens);
int tmvs_fmt_kv_grouped(const float* source, int nv, int group_nv, int s_tokens, const float* enc_w, void* workspace,
                        size_t workspace_bytes, float* kv, void* stream);
/* The rest of EncoderLayer.forward (FMT.py:96-111, AttentionLayer :56-75, LinearAttention
 * :22-37) per query token, in place on x [nv][L][32]. kv_view_stride = 0 shares one kv
 * (cross layers: the ref view's K/V serve every source view). */
int tmvs_fmt_apply(float* x, int nv, int l_tokens, const float* kv, long kv_view_stride, const float* enc_w,
                   void* stream);

/* FMT_with_pathway lateral step (models/FMT.py:221-228): out = smooth(up2(reduce(coarse)) + lateral)
 *   coarse [nv][h][w][cc] (NHWC), lateral [nv][cf][2h][2w] (NCHW, per-view stride lat_view_stride),
 *   w_reduce [cc][cf] (1x1 conv weight [cf][cc] transposed), w_smooth [cf_in][3][3][cf_out]
 *   (3x3 conv weight [cf_out][cf_in][3][3] permuted (1,2,3,0)); both convs have no bias
 *   -> out [nv][2h][2w][cf] (NHWC).  Supported (cc,cf): (32,16), (16,8).                  */
int tmvs_fmt_pathway(const float* coarse, const float* lateral, long lat_view_stride, const float* w_reduce,
                     const float* w_smooth, int nv, int cc, int cf, int h, int w, float* out, void* stream);

/* ------------------------------------------------------------------ native orchestration
 * Whole-FMT forward (models/FMT.py:147-177 inside FMT_with_pathway :212-226): embedding + PE,
 * the reference view's 4 self layers (the K/V of each output is reduced once for the matching
 * cross layer), then views 1..nv-1 through all 8 layers, batched.
 *   stage1 [nv][32][H][W] (NCHW, per-view stride view_stride floats), pe [32][pe_h][pe_w],
 *   enc_w  HOST array of 8 DEVICE pointers (packed EncoderLayer weights, layer order 0..7)
 *   tokens [nv][H*W][32] out (NHWC stage-1 features after the FMT).                         */
size_t tmvs_fmt_forward_workspace(int nv, int l_tokens);
int tmvs_fmt_forward(const float* stage1, long view_stride, const float* pe, int pe_h, int pe_w, int nv, int height,
                     int width, const float* const* enc_w, void* workspace, size_t workspace_bytes, float* tokens,
                     void* stream);
/* tmvs_fmt_forward with the reference view's chain -- its self layers 0,2,4,6 and the K/V of their outputs
 * for the cross layers (FMT.py:155-158,173-174) -- on side_stream, concurrent with the source views' 8
 * layers on stream. Bitwise the tokens of tmvs_fmt_forward. side_stream forks from stream after the
 * embedding and is joined back into stream before the call returns (one fork level: graph-capturable).
 * side_stream NULL (or == stream, or nv < 2) runs tmvs_fmt_forward. */
size_t tmvs_fmt_forward_split_workspace(int nv, int l_tokens);
int tmvs_fmt_forward_split(const float* stage1, long view_stride, const float* pe, int pe_h, int pe_w, int nv,
                           int height, int width, const float* const* enc_w, void* workspace, size_t workspace_bytes,
                           float* tokens, void* stream, void* side_stream);

/* One cascade stage of TransMVSNet.forward for ONE sample (models/TransMVSNet.py:174-221):
 * tmvs_stage_hypotheses -> tmvs_warp_corr -> tmvs_costregnet -> tmvs_softmax_wta.
 *   feat [n_views][h][w][channels] NHWC, reference view first; proj HOST [n_views-1][12];
 *   pw_params HOST (stage 1: view_w [n_views-1][h][w] is written) or NULL (view_w is read at
 *   1/2^vw_shift resolution); warp_flags: TMVS_WARP_ROT_PLAIN or 0 (tmvs_warp_corr);
 *   outputs hyp/prob [ndepth][h][w], depth/depth_raw/conf [h][w]. */
size_t tmvs_depth_stage_workspace(int ndepth, int height, int width, int base_ch);
int tmvs_depth_stage(const float* depth_values, int n_values, const float* prev_depth, int prev_h, int prev_w,
                     const float* feat, int n_views, int channels, int ndepth, float ratio, int full_h, int full_w,
                     int stage_scale, const float* proj, const float* pw_params, float* view_w, int vw_shift,
                     int warp_flags, const TmvsCostRegWeights* cr, void* workspace, size_t workspace_bytes, float clamp_lo,
                     float clamp_hi, float* hyp_out, float* prob_out, float* depth_out, float* depth_raw_out,
                     float* conf_out, void* stream);

/* ------------------------------------------------------------------ CostRegNet training
 * Train-mode forward and backward of CostRegNet (models/module.py:425-456, Conv3d :108-147,
 * Deconv3d :150-191, nn.BatchNorm3d with batch statistics), the pieces torch.autograd needs.
 * Activations NDHWC [B][D][H][W][C]; weights packed [27][Cout][Cin] (tap = kd*9+kh*3+kw) in the
 * arrangement each use needs (transmvsnet_amd/train.py packs them). C in {1, 8, 16, 32, 64}.
 *
 * tmvs_conv3d_generic: y = conv of x, no bias. Without TMVS_CONV_TRANSPOSED: y[o] = sum W[k]
 *   x[o*s - 1 + k] (Conv3d k3 p1 stride s; the dgrad of a ConvTranspose3d); with it: y[o] = sum
 *   W[k] x[(o + 1 - k)/s] over the k with s | o + 1 - k (ConvTranspose3d k3 s2 p1 op1; the dgrad
 *   of a Conv3d). TMVS_CONV_ACCUMULATE: y += the result. Output dims are explicit; taps outside
 *   the input grid contribute nothing.                                                          */
#define TMVS_CONV_TRANSPOSED 1
#define TMVS_CONV_ACCUMULATE 2
int tmvs_conv3d_generic(const float* x, int batch, int cin, int d_in, int h_in, int w_in, const float* w, int cout,
                        int d_out, int h_out, int w_out, int stride, int flags, float* y, void* stream);

/* The same convolutions on the inference layers' MFMA kernels (tmvs_conv3d_bn_relu /
 * tmvs_deconv3d_bn_relu_add) with the raw epilogue (no BN, no ReLU): y = conv(x) (+ skip).
 * transposed = 0: Conv3d k3 p1, stride 1 or 2 (the train forward of conv1..conv6; the dgrad of
 * conv7/9/11 with their ConvTranspose weight tensor read as a Conv3d [Ci_t][Co_t] weight);
 * transposed = 1: ConvTranspose3d k3 s2 p1 op1, output 2x input (the train forward of conv7/9/11;
 * the dgrad of the stride-2 Conv3d layers, whose weight read as ConvTranspose [Co][Ci] is the
 * adjoint), skip (nullable, transposed only, must not alias y) added. wpk [27][cout][cin].
 * Shapes: the inference layers' (cin, cout) pairs -- stride 1: 16->16, 32->32, 64->64; stride 2:
 * 8->16, 16->32, 32->64; transposed: 64->32, 32->16, 16->8 -- else TMVS_ERR_SHAPE; and conv0's and
 * prob's VALU kernels, stride 1: 1->8 (wpk [27][8]) and 8->1 (wpk in the prob packing of
 * TmvsCostRegWeights.w[10], [3][72]).                                                           */
int tmvs_conv3d_mfma(const float* x, int batch, int cin, int d, int h, int w, const float* wpk, int cout, int stride,
                     int transposed, const float* skip, float* y, void* stream);

/* dw[k][a][b] = sum_p direct[p][a] * gathered[p*stride - 1 + k][b] over every voxel p of direct
 * [B][pd][ph][pw][a_ch] (taps outside gathered [B][gd][gh][gw][b_ch] are zero): the weight
 * gradient of a Conv3d (direct = dz, gathered = x) or of a ConvTranspose3d (direct = x,
 * gathered = dz, stride 2). Block partials + fixed-order combine (deterministic).            */
size_t tmvs_conv3d_wgrad_workspace(int batch, int d, int h, int w, int a_ch, int b_ch);
int tmvs_conv3d_wgrad(const float* direct, int a_ch, int batch, int pd, int ph, int pw, const float* gathered,
                      int b_ch, int gd, int gh, int gw, int stride, void* workspace, size_t workspace_bytes,
                      float* dw, void* stream);

/* Backward of the per-view similarity (homo_warping + (warped*ref).mean(1), module.py:284-322,
 * TransMVSNet.py:80) for the training path: given dsim [V][D][H][W] (d loss / d sim_v), writes
 *   dref [H][W][C] = sum_v sum_d dsim/C * bilinear(src_v)          (NHWC, overwritten)
 *   dsrc [V][H][W][C] = the bilinear scatter of dsim/C * ref          (NHWC, overwritten)
 * ref/src/hyp/proj/flags as tmvs_warp_corr (one sample, C in {8,16,32}). The scatter is summed
 * in fixed point with 64-bit integer atomics (deterministic); the unit is chosen per call from
 * max|dsim| and max|ref| so that no texel's sum can overflow (ABI 5; it was a fixed 2^-40). The
 * workspace's int after the buffer is set to 1 when dsim or ref holds a non-finite value. One
 * thread per (pixel, view, chunk of 8 planes); dref is the fixed-order sum of those partials.
 * ABI 3: the workspace size takes ndepth (the d ref partials live in it).
 * flags & TMVS_WARP_BWD_PLANES (ABI 7; hyp[d][p] = hyp[d][0] for every p, i.e. fronto-parallel
 * depth planes, D <= 64): dsrc is GATHERED instead -- per source texel, the reference pixels in the
 * preimage of its tap square under the plane homography, re-projected with the forward's rounding --
 * in fp32 with a fixed order, no atomics; a pixel whose hyp differs from its plane's sets bit 2 of
 * the workspace flag int.                                                                        */
size_t tmvs_warp_corr_backward_workspace(int n_src, int channels, int height, int width, int ndepth);
int tmvs_warp_corr_backward(const float* ref_fea, const float* src_fea, const float* proj, const float* hyp,
                            const float* dsim, int n_src, int channels, int ndepth, int height, int width, int flags,
                            void* workspace, size_t workspace_bytes, float* dref, float* dsrc, void* stream);

/* DepthNet view aggregation + stage-1 PixelwiseNet in train mode (TransMVSNet.py:10-30, 71-93),
 * one sample, per-view similarity volumes sims [V][D][H][W] (tmvs_warp_corr per view):
 *   pwp [201] (device): w0[16] gamma0[16] beta0[16] W1[8][16] gamma1[8] beta1[8] w2[8] b2.
 *   tmvs_pixelwise_train_forward: per view, BatchNorm batch statistics (stats [V][48]: mean0[16]
 *     var0[16] mean1[8] var1[8], biased) and the view weight view_w [V][H][W] = max over D of the
 *     sigmoid output, with its first argmax dstar [V][H][W] (int32).
 *   tmvs_aggregate_train: sim [D][H][W] = sum_v sims_v w_v / (1e-5 + sum_v w_v) (views in order),
 *     wsum [H][W]; view_w read at (y >> vw_shift, x >> vw_shift) of [V][H>>s][W>>s].
 *   tmvs_aggregate_train_backward: dsims = dsim / wsum * w_v, and (dview_w non-NULL)
 *     dview_w = sum_d dsim / wsum * (sims_v - sim).
 *   tmvs_pixelwise_train_backward: adds the PixelwiseNet path to dsims and its parameter gradients
 *     to dpwp [201] (accumulated: zero it first).
 * All reductions: fp64 block partials + fixed-order combines (deterministic).                  */
size_t tmvs_pixelwise_train_workspace(void);
int tmvs_pixelwise_train_forward(const float* sims, int n_views, int ndepth, int height, int width, const float* pwp,
                                 void* workspace, size_t workspace_bytes, float* stats, float* view_w, int* dstar,
                                 void* stream);
int tmvs_aggregate_train(const float* sims, const float* view_w, int n_views, int ndepth, int height, int width,
                         int vw_shift, float* sim, float* wsum, void* stream);
int tmvs_aggregate_train_backward(const float* dsim, const float* sims, const float* sim, const float* wsum,
                                  const float* view_w, int n_views, int ndepth, int height, int width, int vw_shift,
                                  float* dsims, float* dview_w, void* stream);
int tmvs_pixelwise_train_backward(const float* sims, int n_views, int ndepth, int height, int width, const float* pwp,
                                  const float* stats, const float* view_w, const int* dstar, const float* dview_w,
                                  void* workspace, size_t workspace_bytes, float* dsims, float* dpwp, void* stream);

/* FMT_with_pathway lateral step for training (FMT.py:201-209, 221-228), NHWC, C in {8, 16}:
 *   tmvs_upsample2_add_nhwc: u [n][2h][2w][C] = bilinear x2 (align_corners=False) of r [n][h][w][C]
 *     + lateral [n][C][2h][2w] (NCHW);  tmvs_upsample2_backward_nhwc: dr [n][h][w][C] = the adjoint
 *     of the interpolation applied to du [n][2h][2w][C] (gather, deterministic).
 * The 1x1 reduction and the 3x3 smoothing run on tmvs_conv3d_generic / tmvs_conv3d_wgrad with
 * depth 1 (kd = 1 taps).                                                                       */
int tmvs_upsample2_add_nhwc(const float* r, const float* lateral, int n, int h, int w, int channels, float* u,
                            void* stream);
int tmvs_upsample2_backward_nhwc(const float* du, int n, int h, int w, int channels, float* dr, void* stream);

/* FMT EncoderLayer backward for training (FMT.py:96-111, 56-75, 22-37), tokens [T][C] fp32,
 * C in {32, 64}; every cross-token sum is fp64 with a fixed combine order (no atomics).
 *   tmvs_token_linear:   y = x W^T + b (W [out][in], torch Linear), or with transpose_w y = x W
 *     (W [in'][out'] = the Linear's weight: the data gradient); relu_of (nullable, [T][out])
 *     zeroes y where relu_of <= 0; accumulate adds into y. (in, out) in {(32,32), (32,64), (64,32)}.
 *   tmvs_token_wgrad:    dw [a][b] = sum_t dy[t][a] x[t][b], db [a] = sum_t dy[t][a].
 *   tmvs_layer_norm_fwd / _bwd: LayerNorm(32, eps 1e-5); the backward takes the LN input x,
 *     gives dx and dgb = {dgamma[32], dbeta[32]} (statistics recomputed per token).
 *   tmvs_linattn_fwd:    msg = linear attention of q (pre-elu) against kv [groups][TMVS_KV_NFLOATS]
 *     (token t uses group t / tokens_per_group; kv_stride 0 shares one group).
 *   tmvs_linattn_bwd_q:  dq through the elu and dkv [groups][TMVS_KV_NFLOATS] = dKV, dKsum summed
 *     over each group's query tokens (tokens % tokens_per_group == 0).
 *   tmvs_linattn_bwd_kv: dk (through the elu), dv of the source tokens from k (pre-elu), v, dkv. */
int tmvs_token_linear(const float* x, long tokens, int in_features, int out_features, const float* w,
                      const float* b, int transpose_w, const float* relu_of, int accumulate, float* y,
                      void* stream);
/* tmvs_token_linear_res: y = residual + tmvs_token_linear(x) (the residual [T][out] read, y written: the
 *   accumulate form without first copying the residual into y; residual must not alias y). */
int tmvs_token_linear_res(const float* x, long tokens, int in_features, int out_features, const float* w,
                          const float* b, int transpose_w, const float* relu_of, const float* residual, float* y,
                          void* stream);
size_t tmvs_token_wgrad_workspace(long tokens, int a, int b);
int tmvs_token_wgrad(const float* dy, int a, const float* x, int b, long tokens, void* workspace,
                     size_t workspace_bytes, float* dw, float* db, int accumulate, void* stream);
int tmvs_layer_norm_fwd(const float* x, long tokens, const float* g, const float* b, float* y, void* stream);
size_t tmvs_layer_norm_bwd_workspace(long tokens);
int tmvs_layer_norm_bwd(const float* dy, const float* x, long tokens, const float* g, void* workspace,
                        size_t workspace_bytes, float* dx, float* dgb, int accumulate, void* stream);
int tmvs_linattn_fwd(const float* q, long tokens, long tokens_per_group, const float* kv, long kv_stride,
                     float* msg, void* stream);
size_t tmvs_linattn_bwd_workspace(long tokens, long tokens_per_group);
int tmvs_linattn_bwd_q(const float* q, const float* dmsg, long tokens, long tokens_per_group, const float* kv,
                       long kv_stride, void* workspace, size_t workspace_bytes, float* dq, float* dkv,
                       void* stream);
int tmvs_linattn_bwd_kv(const float* k, const float* v, long tokens, long tokens_per_group, const float* dkv,
                        float* dk, float* dv, void* stream);

/* Adam over one flat fp32 buffer (finetune.py:324: torch.optim.Adam, L2 weight decay, no amsgrad),
 * torch's single-tensor update order; step >= 1 is the 1-based step count (bias corrections).
 * Scalars are doubles, as the Python floats torch receives (1 - beta is formed before rounding).  */
int tmvs_adam_step(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, long n, double lr,
                   double beta1, double beta2, double eps, double weight_decay, int step, void* stream);
/* The same with the step number on the device (a captured HIP graph replays it): *step_counter
 * (int, device) is advanced by the launch itself; scalars: 2 device floats of scratch. lr_dev
 * (ABI 8): NULL = use lr; else the launch reads the learning rate from that device double when it
 * runs, so a graph replay follows the schedule the caller writes there (finetune.py:58-72).     */
int tmvs_adam_step_dev(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, long n, double lr,
                       const double* lr_dev, double beta1, double beta2, double eps, double weight_decay,
                       int* step_counter, float* scalars, void* stream);

/* BatchNorm3d in train mode over z [nvox][C] (C divides 256): batch mean and biased variance
 * (fp64 partials, fixed-order combine); y = relu(fmaf(z, a, b)) [+ skip] with a = gamma /
 * sqrt(var + eps), b = beta - mean * a; the backward of that (incl. the ReLU mask) gives dz,
 * dgamma = sum g * xhat, dbeta = sum g. The running-statistics update is the caller's.        */
size_t tmvs_bn_train_workspace(long nvox, int channels);
int tmvs_bn_stats(const float* z, long nvox, int channels, void* workspace, size_t workspace_bytes, float* mean,
                  float* var, void* stream);
int tmvs_bn_relu_train(const float* z, long nvox, int channels, const float* mean, const float* var,
                       const float* gamma, const float* beta, float eps, const float* skip, float* out, void* stream);
int tmvs_bn_relu_backward(const float* dy, const float* z, long nvox, int channels, const float* mean,
                          const float* var, const float* gamma, const float* beta, float eps, void* workspace,
                          size_t workspace_bytes, float* dz, float* dgamma, float* dbeta, void* stream);
/* The same over `groups` consecutive [nvox][C] slabs with statistics per group (FeatureNet's BatchNorm2d
 * runs once per view: models/TransMVSNet.py:165-166 calls FeatureNet per view) in one launch each:
 * mean / var [groups][C]; dgamma / dbeta are the per-group sums added over the groups in order.   */
size_t tmvs_bn_train_workspace_grouped(int groups, long nvox, int channels);
int tmvs_bn_stats_grouped(const float* z, int groups, long nvox, int channels, void* workspace, size_t workspace_bytes,
                          float* mean, float* var, void* stream);
int tmvs_bn_relu_train_grouped(const float* z, int groups, long nvox, int channels, const float* mean,
                               const float* var, const float* gamma, const float* beta, float eps, const float* skip,
                               float* out, void* stream);
int tmvs_bn_relu_backward_grouped(const float* dy, const float* z, int groups, long nvox, int channels,
                                  const float* mean, const float* var, const float* gamma, const float* beta,
                                  float eps, void* workspace, size_t workspace_bytes, float* dz, float* dgamma,
                                  float* dbeta, void* stream);

/* ------------------------------------------------------------------ FeatureNet heads
 * Modulated deformable convolution of DCN.forward (models/dcn.py:66-80; torchvision.ops.deform_conv2d,
 * torchvision 0.10.1): 3x3, stride 1, padding 1, dilation 1, one offset group, with the head's bias,
 * optional eval BatchNorm (tmvs_bn_fold's alpha/shift) and ReLU fused (models/module.py:362-395).
 *   x_nhwc      : [B][H][W][cin] (cin = 32)
 *   offset_mask : [B][27][H][W] = conv_offset_mask(x) (NCHW): channels 2k / 2k+1 = dy / dx of tap k,
 *                 18+k = mask logit of tap k (sigmoid applied inside)
 *   w_packed    : tmvs_deform_conv2d_packed_floats(cout) floats from tmvs_deform_conv2d_pack (HOST
 *                 packing of the [cout][cin][3][3] weight; copy to the device once per load_state_dict)
 *   bias        : [cout]; bn_alpha / bn_shift: [cout] or both NULL; relu: 0/1
 *   out         : [B][cout][H][W] (NCHW);  out_nhwc: optional [B][H][W][cout] copy, or NULL
 * Supported: cin = 32, cout in {8, 16, 32}; H*W*cin*4 < 2^31; H, W <= 32766. tmvs_deform_conv2d_pack also
 * takes cout = 27 (a conv_offset_mask weight, for tmvs_dcn_fused).                                */
size_t tmvs_deform_conv2d_packed_floats(int cout);
int tmvs_deform_conv2d_pack(const float* weight, int cout, int cin, float* packed);
int tmvs_deform_conv2d(const float* x_nhwc, const float* offset_mask, const float* w_packed, const float* bias,
                       const float* bn_alpha, const float* bn_shift, int relu, int batch, int cin, int cout,
                       int height, int width, float* out, float* out_nhwc, void* stream);

/* The whole DCN.forward (models/dcn.py:66-80) in one launch: conv_offset_mask (3x3, 32 -> 27, bias;
 * models/dcn.py:58-64) computed in-kernel from the same staged input window, then the modulated
 * deformable convolution as above. The [B][27][H][W] offset/mask tensor never reaches HBM.
 *   wom_packed : tmvs_deform_conv2d_packed_floats(27) floats = tmvs_deform_conv2d_pack(conv_offset_mask.weight,
 *                27, 32, ...);  bom: conv_offset_mask.bias [27]
 *   out (NCHW) and out_nhwc are both optional (at least one).                                        */
int tmvs_dcn_fused(const float* x_nhwc, const float* wom_packed, const float* bom, const float* w_packed,
                   const float* bias, const float* bn_alpha, const float* bn_shift, int relu, int batch, int cin,
                   int cout, int height, int width, float* out, float* out_nhwc, void* stream);

/* FeatureNet heads' first layer Conv2d(32, 32, 3, 1, 1, bias=False) -> BatchNorm -> ReLU
 * (models/module.py:24-61 as used at :373 / :385), NHWC: x_nhwc [B][H][W][32] -> out [B][32][H][W]
 * and/or out_nhwc [B][H][W][32] (either may be NULL, not both). w_packed = tmvs_deform_conv2d_pack of
 * the [32][32][3][3] weight; bias optional (NULL for the reference's bias-free conv).            */
int tmvs_conv3x3_nhwc(const float* x_nhwc, const float* w_packed, const float* bias, const float* bn_alpha,
                      const float* bn_shift, int relu, int batch, int cin, int cout, int height, int width,
                      float* out, float* out_nhwc, void* stream);

/* out_nhwc [B][H][W][32] += conv3x3(x_nhwc) with tmvs_conv3x3_nhwc's kernel and no bias / BN / ReLU
 * (each element out + conv, the operand order of torch's out += conv): the FeatureNet backward's data
 * gradient of the DCN offset/mask conv added into the DCN's input gradient in the conv's epilogue. */
int tmvs_conv3x3_nhwc_acc(const float* x_nhwc, const float* w_packed, int batch, int cin, int cout, int height,
                          int width, float* out_nhwc, void* stream);

/* FeatureNet FPN merge (models/module.py:409-417): intra = interpolate(prev, 2, nearest) + inner(lat),
 * inner = Conv2d(lat_channels, 32, 1, bias=True) with w_inner [32][lat_channels], b_inner [32].
 * prev_nhwc [B][height][width][32], lat_nhwc [B][2 height][2 width][lat_channels] (8 or 16),
 * out_nhwc [B][2 height][2 width][32].                                                            */
int tmvs_fpn_merge(const float* prev_nhwc, const float* lat_nhwc, int lat_channels, const float* w_inner,
                   const float* b_inner, int batch, int height, int width, float* out_nhwc, void* stream);

/* FeatureNet Conv2d(bias=False) -> eval BatchNorm -> ReLU blocks (models/module.py:24-61) of the trunk
 * (:349-360) and the stage-1 head's 1x1 (:362), NHWC out. Shapes (cin, cout, k, stride): (3,8,3,1) --
 * x is the NCHW image [B][3][H][W] --, (8,8,3,1), (8,16,5,2), (16,16,3,1), (16,32,5,2), (32,32,3,1),
 * (32,32,1,1) -- x is NHWC [B][H][W][cin]; padding k/2; out_nhwc [B][Ho][Wo][cout].
 * w_packed = tmvs_conv2d_packed_floats(cout, cin, k) floats from tmvs_conv2d_pack (HOST).            */
size_t tmvs_conv2d_packed_floats(int cout, int cin, int k);
int tmvs_conv2d_pack(const float* weight, int cout, int cin, int k, float* packed);
int tmvs_conv2d_bn_relu(const float* x, int batch, int cin, int height, int width, const float* w_packed, int cout,
                        int k, int stride, const float* bn_alpha, const float* bn_shift, int relu, float* out_nhwc,
                        void* stream);

/* ------------------------------------------------------------------ output side
 * gipuma depth-map fusion kernel (gipuma/fusibile/fusibile.cu:89-173) for one reference camera:
 *   rgbd    : [V][H][W][4] float (B, G, R, depth), depth = 425 + 512 * alpha / 255 (main.cpp:136)
 *   cams    : [V][32] float: P (3x4 row-major), inv(P[:, :3]) (3x3), camera centre (3), fx, pad
 *   coord / texture : [H][W][4] point buffer; pixels fused with >= consistent_threshold agreeing
 *             views are overwritten with the averaged point / colour (.w = 0), others are left as
 *             they are (the reference reuses one buffer across cameras).                         */
int tmvs_fusibile(const float* rgbd, const float* cams, int n_views, int height, int width, int ref_view,
                  int consistent_threshold, float depth_threshold, float* coord, float* texture, void* stream);

/* ------------------------------------------------------------------ training losses
 * entropy_loss (models/module.py:495-531) of one stage, as trans_mvsnet_loss / focal_loss_bld
 * (:532-588) call it, fused with the backward through the stage's softmax (:prob = softmax(logits)).
 *   prob        [batch][ndepth][H][W]   softmax probability volume (outputs[stage]["prob_volume"])
 *   depth_values [batch][ndepth][H][W] (dv_per_pixel = 1) or [batch][ndepth] (0, module.py:503-504)
 *   depth_gt, mask [batch][H][W]        mask > 0.5 is valid (module.py:540)
 *   out (device, 2 floats): out[0] = entropy loss (unweighted, :522), out[1] = smooth-L1 depth_loss of
 *             the WTA depth over the masked pixels (:545; NaN for an empty mask, as torch)
 *   wta_depth / photo_conf [batch][H][W] (nullable): WTA depth (:524-525) and max prob (:528)
 *   grad_logits [batch][ndepth][H][W] (nullable): d(grad_scale * loss)/d(logits); grad_scale is the
 *             caller's weight of this stage's loss (entropy_weight 2.0 x dlossw[stage], :547-553).
 *   workspace: tmvs_entropy_loss_workspace(batch, H, W) bytes of device memory.                   */
size_t tmvs_entropy_loss_workspace(int batch, int height, int width);
int tmvs_entropy_loss(const float* prob, const float* depth_values, int dv_per_pixel, const float* depth_gt,
                      const float* mask, int batch, int ndepth, int height, int width, float grad_scale,
                      void* workspace, size_t workspace_bytes, float* out, float* wta_depth, float* photo_conf,
                      float* grad_logits, void* stream);
/* focal_loss_bld's metrics (module.py:581-587): err = |gt - depth| / (depth_interval * 192 / 128) over
 * the n masked elements; out (device, 3 floats) = {epe, less1, less3}; NaN for an empty mask.      */
size_t tmvs_depth_metrics_workspace(int n);
int tmvs_depth_metrics(const float* depth, const float* depth_gt, const float* mask, int n, float depth_interval,
                       void* workspace, size_t workspace_bytes, float* out, void* stream);

/* ------------------------------------------------------------------ FeatureNet training
 * The backward of FeatureNet (models/module.py:343-422) and of its DCNs (models/dcn.py:66-80 ->
 * torchvision.ops.deform_conv2d), and of the softmax of prob_volume (models/TransMVSNet.py:99).
 * NHWC fp32 activations; every pixel reduction is block partials + a fixed-order fp64 combine.
 *
 * tmvs_conv2d_generic: y [B][h_out][w_out][cout] = bias + conv (k x k taps, weights w [k*k][cout][cin]):
 *   strided (flags 0): y[o] = sum_k W[k] x[o*stride - pad + k]       (Conv2d; replaces cuDNN's forward)
 *   TMVS_CONV_TRANSPOSED: y[i] = sum_k W[k] x[(i + pad - k)/stride] where stride divides (the data
 *   gradient of a Conv2d with W[k][ci][co] = its weight transposed); TMVS_CONV_ACCUMULATE: y +=.
 *   bias nullable. cin in {3, 8, 16, 27, 32}; cout a multiple of 8, or 27 (cin 8/16/32).
 * tmvs_conv2d_wgrad: dw [k*k][a_ch][b_ch] = sum_p direct[p][a] gathered[p*stride - pad + k][b] (a Conv2d's
 *   weight gradient: direct = dz [B][ph][pw][a], gathered = x [B][gh][gw][b]). (a, b) in {8,16,27,32} x
 *   {8,16,32} with a <= 32, or (8, 3).
 * tmvs_colsum: out[c] = sum_p x[p][c] over x [n][channels] (a bias gradient), channels <= 32.
 * tmvs_dcn_forward_train: tmvs_dcn_fused without BatchNorm / ReLU that also writes the offset/mask
 *   tensor the backward needs: offset_mask_out [B][27][H][W] (= conv_offset_mask(x) + bias).
 * tmvs_dcn_backward: given dy_nhwc [B][H][W][cout] (d loss / d DCN output) and the forward's
 *   x_nhwc [B][H][W][32], offset_mask [B][27][H][W], w_taps [9][cout][32] (the weight [cout][32][3][3]
 *   as [tap][co][ci]):
 *     dx_nhwc  [B][H][W][32]  += the bilinear scatter of mask * dcol (fp32 atomics, as torchvision)
 *     dom_nhwc [B][H][W][32]   = d offsets (channels 2k, 2k+1) and d mask logits (18 + k); channels
 *                                27..31 are written 0 (aligned rows for the offset/mask conv's gradients)
 *     dw_taps  [9][cout][32]   = the weight gradient (the bias gradient is tmvs_colsum of dy).
 *   cout in {8, 16, 32}. The offset/mask conv's gradients are tmvs_conv2d_wgrad / _generic of dom.
 * tmvs_dcn_backward_set: the same, but dx_nhwc is WRITTEN (need not be initialised): the corners
 *   beyond the LDS windows are added with fp32 atomics into far_zeroed [B][H][W][32], which must be all
 *   zero on entry and is all zero again on return (the gather pass folds it into dx and clears it, only
 *   when a far corner occurred) -- so the caller keeps one zeroed buffer instead of a zero fill of dx per
 *   call. One far buffer per stream: concurrent calls must not share it.
 * tmvs_nearest_up2_backward_nhwc: dprev [n][h][w][C] (+)= the 2x2 sums of d [n][2h][2w][C] (the
 *   adjoint of interpolate(scale 2, nearest), models/module.py:413,417).
 * tmvs_softmax_backward: dlogits = prob * (dprob - sum_d prob * dprob), [B][D][H][W].            */
int tmvs_conv2d_generic(const float* x, int batch, int cin, int h_in, int w_in, const float* w, const float* bias,
                        int cout, int h_out, int w_out, int k, int stride, int pad, int flags, float* y, void* stream);
size_t tmvs_conv2d_wgrad_workspace(int batch, int h, int w, int a_ch, int b_ch, int k);
int tmvs_conv2d_wgrad(const float* direct, int a_ch, int batch, int ph, int pw, const float* gathered, int b_ch,
                      int gh, int gw, int k, int stride, int pad, void* workspace, size_t workspace_bytes, float* dw,
                      void* stream);
size_t tmvs_colsum_workspace(long n, int channels);
int tmvs_colsum(const float* x, long n, int channels, void* workspace, size_t workspace_bytes, float* out,
                void* stream);
int tmvs_dcn_forward_train(const float* x_nhwc, const float* wom_packed, const float* bom, const float* w_packed,
                           const float* bias, int batch, int cin, int cout, int height, int width, float* out,
                           float* out_nhwc, float* offset_mask_out, void* stream);
size_t tmvs_dcn_backward_workspace(int batch, int cout, int height, int width);
int tmvs_dcn_backward(const float* x_nhwc, const float* offset_mask, const float* w_taps, const float* dy_nhwc,
                      int batch, int cin, int cout, int height, int width, void* workspace, size_t workspace_bytes,
                      float* dx_nhwc, float* dom_nhwc, float* dw_taps, void* stream);
int tmvs_dcn_backward_set(const float* x_nhwc, const float* offset_mask, const float* w_taps, const float* dy_nhwc,
                          int batch, int cin, int cout, int height, int width, void* workspace, size_t workspace_bytes,
                          float* dx_nhwc, float* dom_nhwc, float* dw_taps, float* far_zeroed, void* stream);
int tmvs_nearest_up2_backward_nhwc(const float* d, int n, int h, int w, int channels, int accumulate, float* dprev,
                                   void* stream);
int tmvs_softmax_backward(const float* prob, const float* dprob, int batch, int ndepth, int height, int width,
                          float* dlogits, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* TRANSMVS_H_ */
