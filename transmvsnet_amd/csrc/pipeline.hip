// Native orchestration of the hot path: whole-FMT and whole-DepthNet-stage entry points that
// enqueue their kernels back to back on one stream (no per-kernel host round trip).
#include "common.h"

static size_t align_up256(size_t v) { return (v + 255) & ~(size_t)255; }
static size_t fmt_kv_slab(int nv, int l_tokens) {  // self K/V runs on nv views, cross K/V on one
  const size_t a = tmvs_fmt_kv_workspace(nv, l_tokens), b = tmvs_fmt_kv_workspace(1, l_tokens);
  return align_up256(a > b ? a : b);
}

extern "C" size_t tmvs_fmt_forward_workspace(int nv, int l_tokens) {
  // kv slabs (one per layer application in flight) + 4 cross-layer kv + per-view kv
  return fmt_kv_slab(nv, l_tokens) + align_up256((size_t)(4 + nv) * TMVS_KV_NFLOATS * 4);
}

// FMT of FMT_with_pathway (models/FMT.py:147-177, 212-226), all views batched on the launch
// grid's y dimension.
extern "C" int tmvs_fmt_forward(const float* stage1, long view_stride, const float* pe, int pe_h, int pe_w, int nv,
                                int height, int width, const float* const* enc_w, void* workspace,
                                size_t workspace_bytes, float* tokens, void* stream) {
  if (!stage1 || !pe || !enc_w || !workspace || !tokens || nv <= 0) return TMVS_ERR_ARG;
  for (int i = 0; i < 8; ++i)
    if (!enc_w[i]) return TMVS_ERR_ARG;
  const int L = height * width;
  if (workspace_bytes < tmvs_fmt_forward_workspace(nv, L)) return TMVS_ERR_ARG;
  char* ws = (char*)workspace;
  const size_t slab = fmt_kv_slab(nv, L);
  void* kv_ws = ws;
  float* kv_cross = (float*)(ws + slab);
  float* kv_self = kv_cross + 4 * TMVS_KV_NFLOATS;
  int rc;
  if ((rc = tmvs_fmt_embed(stage1, view_stride, pe, pe_h, pe_w, nv, 32, height, width, tokens, stream))) return rc;
  // Self layers 0,2,4,6 carry the same weights for the reference view (FMT.py:155-158) and the
  // source views (:171-172): each runs on all nv views in one launch (per-view K/V). The
  // reference output of self layer 2j is ref_feature_list[j], the K/V source of cross layer 2j+1.
  float* src = tokens + (size_t)L * 32;
  for (int j = 0; j < 4; ++j) {
    const int i = 2 * j;
    if ((rc = tmvs_fmt_kv(tokens, nv, L, enc_w[i], kv_ws, slab, kv_self, stream))) return rc;
    if ((rc = tmvs_fmt_apply(tokens, nv, L, kv_self, TMVS_KV_NFLOATS, enc_w[i], stream))) return rc;
    if (nv == 1) continue;
    if ((rc = tmvs_fmt_kv(tokens, 1, L, enc_w[i + 1], kv_ws, slab, kv_cross + j * TMVS_KV_NFLOATS, stream))) return rc;
    if ((rc = tmvs_fmt_apply(src, nv - 1, L, kv_cross + j * TMVS_KV_NFLOATS, 0, enc_w[i + 1], stream))) return rc;
  }
  return TMVS_OK;
}

// The same FMT with the reference view's chain on a second stream (tmvs_fmt_forward_split). Workspace:
// [main K/V slab][side K/V slab][4 cross K/V][ref self K/V][source views' self K/V].
static size_t fmt_split_slab_main(int nv, int l_tokens) {
  return align_up256(tmvs_fmt_kv_grouped_workspace(nv - 1, nv, l_tokens));
}
static size_t fmt_split_slab_side(int nv, int l_tokens) {
  const size_t a = tmvs_fmt_kv_grouped_workspace(1, nv, l_tokens), b = tmvs_fmt_kv_workspace(1, l_tokens);
  return align_up256(a > b ? a : b);
}

extern "C" size_t tmvs_fmt_forward_split_workspace(int nv, int l_tokens) {
  if (nv < 2) return tmvs_fmt_forward_workspace(nv, l_tokens);
  return fmt_split_slab_main(nv, l_tokens) + fmt_split_slab_side(nv, l_tokens) +
         align_up256((size_t)(4 + 1 + (nv - 1)) * TMVS_KV_NFLOATS * 4);
}

#ifndef TMVS_FMT_SPLIT_ORDER
#define TMVS_FMT_SPLIT_ORDER 0
#endif
#ifndef TMVS_SPLIT_REF_TPW
// tiles per wave of the reference view's applies (0: occupancy-sized, as if the launch were alone). Beside the
// source views' launches a 1-view apply of 2 tiles per wave (half the waves) measured 297.8 vs 296.6 depth maps/s
// (4: 297.4, 8: 293.6; profiles/r22/reftpw_ab.txt); the tokens are the same either way
#define TMVS_SPLIT_REF_TPW 2
#endif

namespace {
// fork / cross-layer / join events of tmvs_fmt_forward_split, created once per host thread and device
// (thread_local: concurrent host threads never share an event; within one thread every record is
// followed by its waits in the same call, so a wait always binds to this call's record)
struct SplitEvents {
  hipEvent_t ev[6];
  bool ok;
};
SplitEvents* split_events() {
  constexpr int kMaxDev = 16;
  thread_local SplitEvents cache[kMaxDev] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDev) return nullptr;
  SplitEvents& e = cache[dev];
  if (!e.ok) {
    for (int i = 0; i < 6; ++i)
      if (hipEventCreateWithFlags(&e.ev[i], hipEventDisableTiming) != hipSuccess) return nullptr;
    e.ok = true;
  }
  return &e;
}
}  // namespace

// models/FMT.py:147-177 as two dependency chains: the reference view's self layers 0,2,4,6 (FMT.py:155-158)
// and the K/V reductions of its outputs for the cross layers (:173-174) on side_stream; the source views'
// 8 layers (:168-175) on stream, each cross layer waiting for its K/V. Self-layer K/V keep the nv-view
// launch's partial grouping (tmvs_fmt_kv_grouped) and the applies are per token, so the tokens are bitwise
// those of tmvs_fmt_forward. side_stream forks from stream after the embedding and joins before return.
extern "C" int tmvs_fmt_forward_split(const float* stage1, long view_stride, const float* pe, int pe_h, int pe_w,
                                      int nv, int height, int width, const float* const* enc_w, void* workspace,
                                      size_t workspace_bytes, float* tokens, void* stream, void* side_stream) {
  if (!side_stream || nv < 2 || side_stream == stream)
    return tmvs_fmt_forward(stage1, view_stride, pe, pe_h, pe_w, nv, height, width, enc_w, workspace, workspace_bytes,
                            tokens, stream);
  if (!stage1 || !pe || !enc_w || !workspace || !tokens) return TMVS_ERR_ARG;
  for (int i = 0; i < 8; ++i)
    if (!enc_w[i]) return TMVS_ERR_ARG;
  const int L = height * width;
  if (workspace_bytes < tmvs_fmt_forward_split_workspace(nv, L)) return TMVS_ERR_ARG;
  SplitEvents* e = split_events();
  if (!e) return TMVS_ERR_HIP;
  hipStream_t ms = (hipStream_t)stream, ss = (hipStream_t)side_stream;
  char* ws = (char*)workspace;
  const size_t sm = fmt_split_slab_main(nv, L), sd = fmt_split_slab_side(nv, L);
  void* slab_main = ws;
  void* slab_side = ws + sm;
  float* kv_cross = (float*)(ws + sm + sd);
  float* kv_ref = kv_cross + 4 * TMVS_KV_NFLOATS;
  float* kv_src = kv_ref + TMVS_KV_NFLOATS;
  int rc;
  if ((rc = tmvs_fmt_embed(stage1, view_stride, pe, pe_h, pe_w, nv, 32, height, width, tokens, stream))) return rc;
  if (hipEventRecord(e->ev[0], ms) != hipSuccess || hipStreamWaitEvent(ss, e->ev[0], 0) != hipSuccess)
    return TMVS_ERR_HIP;
  float* src = tokens + (size_t)L * 32;
  auto ref_layer = [&](int j) -> int {  // reference view: self layer 2j, then its output's K/V for cross layer 2j+1
    const int i = 2 * j;
    int r;
    if ((r = tmvs_fmt_kv_grouped(tokens, 1, nv, L, enc_w[i], slab_side, sd, kv_ref, ss))) return r;
    if ((r = tmvs_fmt_apply_tiled(tokens, 1, L, kv_ref, TMVS_KV_NFLOATS, enc_w[i], TMVS_SPLIT_REF_TPW, ss))) return r;
    if ((r = tmvs_fmt_kv(tokens, 1, L, enc_w[i + 1], slab_side, sd, kv_cross + j * TMVS_KV_NFLOATS, ss))) return r;
    return hipEventRecord(e->ev[1 + j], ss) != hipSuccess ? TMVS_ERR_HIP : TMVS_OK;
  };
  auto src_self = [&](int j) -> int {  // source views: self layer 2j
    const int i = 2 * j;
    int r;
    if ((r = tmvs_fmt_kv_grouped(src, nv - 1, nv, L, enc_w[i], slab_main, sm, kv_src, ms))) return r;
    return tmvs_fmt_apply(src, nv - 1, L, kv_src, TMVS_KV_NFLOATS, enc_w[i], ms);
  };
  auto src_cross = [&](int j) -> int {  // source views: cross layer 2j+1 (waits for the reference's K/V)
    if (hipStreamWaitEvent(ms, e->ev[1 + j], 0) != hipSuccess) return TMVS_ERR_HIP;
    return tmvs_fmt_apply(src, nv - 1, L, kv_cross + j * TMVS_KV_NFLOATS, 0, enc_w[2 * j + 1], ms);
  };
  if (TMVS_FMT_SPLIT_ORDER == 0) {  // the reference chain enqueued whole, then the source views'
    for (int j = 0; j < 4; ++j)
      if ((rc = ref_layer(j))) return rc;
    for (int j = 0; j < 4; ++j)
      if ((rc = src_self(j)) || (rc = src_cross(j))) return rc;
  } else {  // layer by layer
    for (int j = 0; j < 4; ++j)
      if ((rc = src_self(j)) || (rc = ref_layer(j)) || (rc = src_cross(j))) return rc;
  }
  if (hipEventRecord(e->ev[5], ss) != hipSuccess) return TMVS_ERR_HIP;
  if (hipStreamWaitEvent(ms, e->ev[5], 0) != hipSuccess) return TMVS_ERR_HIP;
  return TMVS_OK;
}

extern "C" size_t tmvs_depth_stage_workspace(int ndepth, int height, int width, int base_ch) {
  const size_t vol = (size_t)ndepth * height * width * 4;
  return align_up256(vol) + align_up256(tmvs_costregnet_workspace(1, ndepth, height, width, base_ch));
}

// One cascade stage of TransMVSNet.forward for one sample (models/TransMVSNet.py:174-221):
// hypotheses -> fused cost volume -> CostRegNet -> softmax / winner-take-all.
extern "C" int tmvs_depth_stage(const float* depth_values, int n_values, const float* prev_depth, int prev_h,
                                int prev_w, const float* feat, int n_views, int channels, int ndepth, float ratio,
                                int full_h, int full_w, int stage_scale, const float* proj, const float* pw_params,
                                float* view_w, int vw_shift, int warp_flags, const TmvsCostRegWeights* cr, void* workspace,
                                size_t workspace_bytes, float clamp_lo, float clamp_hi, float* hyp_out,
                                float* prob_out, float* depth_out, float* depth_raw_out, float* conf_out,
                                void* stream) {
  if (!feat || !view_w || !cr || !workspace || !hyp_out || n_views < 2) return TMVS_ERR_ARG;
  const int h = full_h / stage_scale, w = full_w / stage_scale;
  if (workspace_bytes < tmvs_depth_stage_workspace(ndepth, h, w, cr->base_ch)) return TMVS_ERR_ARG;
  const size_t vol = (size_t)ndepth * h * w;
  char* ws = (char*)workspace;
  float* sim = (float*)ws;
  char* crws = ws + align_up256(vol * 4);
  const size_t crbytes = workspace_bytes - align_up256(vol * 4);
  const int V = n_views - 1;
  int rc;
  if ((rc = tmvs_stage_hypotheses(depth_values, n_values, prev_depth, prev_h, prev_w, 1, ndepth, ratio, full_h, full_w,
                                  stage_scale, hyp_out, stream)))
    return rc;
  const float* ref = feat;
  const float* src = feat + (size_t)h * w * channels;
  if (pw_params)
    rc = tmvs_warp_corr(ref, src, proj, hyp_out, nullptr, 0, 0, V, pw_params, 1, V, channels, ndepth, h, w,
                        warp_flags & TMVS_WARP_ROT_PLAIN, sim,
                        nullptr, view_w, stream);
  else
    rc = tmvs_warp_corr(ref, src, proj, hyp_out, view_w, vw_shift, 0, V, nullptr, 1, V, channels, ndepth, h, w,
                        warp_flags & TMVS_WARP_ROT_PLAIN, sim, nullptr, nullptr, stream);
  if (rc) return rc;
  return tmvs_costregnet_wta(sim, hyp_out, 1, ndepth, h, w, cr, crws, crbytes, clamp_lo, clamp_hi, prob_out, depth_out,
                             depth_raw_out, conf_out, stream);
}
