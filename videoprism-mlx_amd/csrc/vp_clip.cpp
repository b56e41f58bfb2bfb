// C-ABI of the LvT video-text model, FactorizedVideoCLIP (encoders.py:762-910), on top of the
// FactorizedEncoder handle (vp_abi.cpp) and the shared layer schedule (vp_internal.h).
//
//   video: vision encoder (vp_forward) -> auxiliary encoder (2 pre-LN layers over all T*N
//          tokens, attention_long_bf16) -> contrastive pooler (query folded into the key
//          projection, clip_kernels.hip) -> LayerNorm -> L2 normalise
//   text:  token embedding * sqrt(D) + sinusoidal positions, CLS appended -> 12 causal pre-LN
//          ReLU layers (attention_masked) -> unimodal_ln on the CLS row -> L2 normalise
#include "vp_internal.h"

using namespace vpi;

namespace {
constexpr int kMaxTextLen = 1024;  // L + 1 (CLS) tokens; TEXT_MAX_LEN is 64 (models.py:53)
}

// AttenTokenPoolingLayer weights, packed (see pack_pooler): U [H][D] (query folded into the key
// projection), Ut = bf16 hi|lo halves of U for the MFMA logits, Wv^T [H][D][dp], bv [H][dp],
// Wpost^T [H*dp][D], bpost [D], LayerNorm gamma (1 + scale) / beta
struct PoolerW {
  void* Ut = nullptr;
  float *U = nullptr, *WvT = nullptr, *bv = nullptr, *WpT = nullptr, *bp = nullptr;
  float *ln_g = nullptr, *ln_b = nullptr;
  int dp = 0;
};

struct vp_clip {
  vp_clip_config cfg;
  int device = 0;
  bool finalized = false;
  vp_handle* video = nullptr;  // 'vision_encoder/' leaves
  std::map<std::string, vpi::HostParam> host;
  std::vector<std::string> names;
  std::map<std::string, std::vector<int64_t>> expected;
  std::vector<vpi::DevBuf> allocs;
  bool bf16() const { return cfg.video.fprop_dtype == VP_BF16; }
  std::vector<vpi::LayerW> aux, text;
  PoolerW pool;  // contrastive_vision_pooler (hidden 4D)
  // text tower: token table [V][D] (fprop dtype), cls [D], sinusoidal table [kMaxTextLen][D]
  void* tok = nullptr;
  float *cls = nullptr, *tpos = nullptr, *uln_g = nullptr, *uln_b = nullptr;
};

namespace {

struct ClipVideoWs {
  size_t inner = 0, feat = 0, logits = 0, stats = 0, zpart = 0, z = 0, enc = 0, pooled = 0, total = 0;
};

// vision features + pooler scratch for G <= B*T groups; dp = the pooler's dim_per_head
ClipVideoWs pool_video_ws(const vp_config& v, int64_t B, int64_t T, int64_t H, int64_t W, size_t inner_bytes,
                          int64_t dp) {
  const int64_t P = v.patch_size, N = (H / P) * (W / P), M = B * T * N;
  const int64_t Mp = (M + 255) / 256 * 256;  // the auxiliary encoder's GEMM rows (clip_video_chunk)
  const int64_t D = v.model_dim, NH = v.num_heads;
  const size_t es = v.fprop_dtype == VP_BF16 ? 2 : 4;
  const int64_t gc = std::max<int64_t>(B * vp::pool_chunks((int)(T * N)), B * T * vp::pool_chunks((int)N));
  ClipVideoWs L;
  size_t off = 0;
  L.inner = off; off = align256(off + inner_bytes);
  L.feat = off; off = align256(off + (size_t)Mp * D * es);
  L.logits = off; off = align256(off + (size_t)M * NH * 4);
  L.stats = off; off = align256(off + (size_t)B * T * NH * 8);
  L.zpart = off; off = align256(off + (size_t)gc * NH * D * 4);
  L.z = off; off = align256(off + (size_t)B * T * NH * D * 4);
  L.enc = off; off = align256(off + (size_t)B * T * NH * dp * 4);
  L.pooled = off; off = align256(off + (size_t)B * T * D * 4);
  L.total = off;
  return L;
}

ClipVideoWs clip_video_ws(const vp_clip* c, int64_t B, int64_t T, int64_t H, int64_t W, size_t inner_bytes) {
  return pool_video_ws(c->cfg.video, B, T, H, W, inner_bytes, 4 * c->cfg.video.model_dim / c->cfg.video.num_heads);
}

struct ClipTextWs {
  size_t x = 0, hb = 0, big = 0, pad = 0, total = 0;
  int64_t Mt = 0;
  bool small = false;  // bf16 GEMMs on the small-M kernel (64-row tiles)
};

ClipTextWs clip_text_ws(const vp_clip* c, int64_t Q, int64_t L) {
  const int64_t D = c->cfg.video.model_dim;
  const size_t es = c->bf16() ? 2 : 4;
  ClipTextWs w;
  // up to 4096 rows (63 queries) the bf16 GEMMs take the small-M kernel, whose tiles are 64 rows; the
  // 256 x 256-tile kernels would leave at least three quarters of the CUs idle
  w.small = c->bf16() && Q * (L + 1) <= 4096 && D % 256 == 0;
  const int64_t rt = w.small ? 64 : 256;
  w.Mt = (Q * (L + 1) + rt - 1) / rt * rt;
  size_t off = 0;
  w.x = off; off = align256(off + (size_t)w.Mt * D * 4);  // fp32 residual stream
  w.hb = off; off = align256(off + (size_t)w.Mt * D * es);
  w.big = off; off = align256(off + (size_t)w.Mt * 4 * D * es);
  w.pad = off; off = align256(off + (size_t)w.Mt * 4);
  w.total = off;
  return w;
}

// the 12 leaves of an AttenTokenPoolingLayer (layers.py:1044-1136, layers_test.py:283)
template <class Hd>
void add_pooler_expected(Hd* c, const std::string& pre, int64_t D, int64_t NH, int64_t dp) {
  add_expected(c, pre + "pooling_attention_query", {1, D});
  add_expected(c, pre + "pooling_attention/per_dim_scale/per_dim_scale", {dp});
  for (const char* q : {"query", "key", "value"}) {
    add_expected(c, pre + "pooling_attention/" + q + "/w", {D, NH, dp});
    add_expected(c, pre + "pooling_attention/" + q + "/b", {NH, dp});
  }
  add_expected(c, pre + "pooling_attention/post/w", {D, NH, dp});
  add_expected(c, pre + "pooling_attention/post/b", {D});
  add_expected(c, pre + "pooling_attention_layer_norm/scale", {D});
  add_expected(c, pre + "pooling_attention_layer_norm/bias", {D});
}

void build_clip_expected(vp_clip* c) {
  const vp_clip_config& cc = c->cfg;
  const int64_t D = cc.video.model_dim, NH = cc.video.num_heads, dp = 4 * D / NH;
  if (cc.num_auxiliary_layers > 0)
    add_stack_expected(c, "auxiliary_encoder/transformers_stack/x_layers/", cc.num_auxiliary_layers, D,
                       cc.video.mlp_dim, NH);
  add_pooler_expected(c, "contrastive_vision_pooler/", D, NH, dp);
  add_expected(c, "text_encoder/token_emb/emb_var", {(int64_t)cc.vocabulary_size, D});
  add_expected(c, "text_encoder/cls_emb", {1, 1, D});
  add_stack_expected(c, "text_encoder/unimodal_transformer/x_layers/", cc.num_unimodal_layers, D, 4 * D, NH);
  add_expected(c, "text_encoder/unimodal_ln/scale", {D});
  add_expected(c, "text_encoder/unimodal_ln/bias", {D});
}

// AttenTokenPoolingLayer (layers.py:1044-1136) with the query folded into the key projection
// (see clip_kernels.hip): host packing in fp64.
template <class Hd>
int pack_pooler(Hd* c, const std::string& root, int64_t D, int64_t H, int64_t dp, PoolerW& pw) {
  const std::string pre = root + "pooling_attention/";
  pw.dp = (int)dp;
  const auto& query = param_data(c, root + "pooling_attention_query");
  const auto& wq = param_data(c, pre + "query/w");
  const auto& bq = param_data(c, pre + "query/b");
  const auto& wk = param_data(c, pre + "key/w");
  const auto& wv = param_data(c, pre + "value/w");
  const auto& bv = param_data(c, pre + "value/b");
  const auto& wp = param_data(c, pre + "post/w");
  const auto& bp = param_data(c, pre + "post/b");
  const auto& pds = param_data(c, pre + "per_dim_scale/per_dim_scale");
  // q~[h][j] = (query . Wq[:, h, j] + bq[h][j]) * 1.442695041/sqrt(dp) * softplus(pds[j])  (:502-527)
  std::vector<double> qt((size_t)H * dp);
  const double r_softplus_0 = 1.442695041 / std::sqrt((double)dp);
  for (int64_t h = 0; h < H; ++h)
    for (int64_t j = 0; j < dp; ++j) {
      double a = bq[(size_t)h * dp + j];
      for (int64_t d = 0; d < D; ++d) a += (double)query[d] * wq[((size_t)d * H + h) * dp + j];
      const double x = pds[j];
      const double sp = x > 30.0 ? x : std::log1p(std::exp(x));
      qt[(size_t)h * dp + j] = a * r_softplus_0 * sp;
    }
  std::vector<float> U((size_t)H * D), wvt((size_t)H * D * dp), wpt((size_t)H * dp * D);
  for (int64_t h = 0; h < H; ++h)
    for (int64_t d = 0; d < D; ++d) {
      double a = 0.0;
      for (int64_t j = 0; j < dp; ++j) a += (double)wk[((size_t)d * H + h) * dp + j] * qt[(size_t)h * dp + j];
      U[(size_t)h * D + d] = (float)a;
      for (int64_t j = 0; j < dp; ++j) wvt[((size_t)h * D + d) * dp + j] = wv[((size_t)d * H + h) * dp + j];
    }
  for (int64_t n = 0; n < D; ++n)
    for (int64_t k = 0; k < H * dp; ++k) wpt[(size_t)k * D + n] = wp[(size_t)n * H * dp + k];
  std::vector<float> g(D);
  const auto& sc = param_data(c, root + "pooling_attention_layer_norm/scale");
  for (int64_t d = 0; d < D; ++d) g[d] = sc[d] + 1.0f;
  // bf16 hi/lo split of U for the MFMA logits kernel
  std::vector<uint16_t> ut((size_t)32 * D, 0);
  for (int64_t h = 0; h < H; ++h)
    for (int64_t d = 0; d < D; ++d) {
      const float u = U[(size_t)h * D + d];
      const uint16_t hi = host_f2bf(u);
      uint32_t hb = (uint32_t)hi << 16;
      float hf;
      std::memcpy(&hf, &hb, 4);
      ut[(size_t)h * D + d] = hi;
      ut[(size_t)(H + h) * D + d] = host_f2bf(u - hf);
    }
  int rc;
  if ((rc = dev_alloc(c, ut.size() * 2, &pw.Ut))) return rc;
  VP_HIP(hipMemcpy(pw.Ut, ut.data(), ut.size() * 2, hipMemcpyHostToDevice));
  if ((rc = upload_f32(c, U, &pw.U)) || (rc = upload_f32(c, wvt, &pw.WvT)) || (rc = upload_f32(c, bv, &pw.bv)) ||
      (rc = upload_f32(c, wpt, &pw.WpT)) || (rc = upload_f32(c, bp, &pw.bp)) || (rc = upload_f32(c, g, &pw.ln_g)) ||
      (rc = upload_f32(c, param_data(c, root + "pooling_attention_layer_norm/bias"), &pw.ln_b)))
    return rc;
  return VP_OK;
}

// pooler over G groups of Sg rows of feat [G*Sg][D] -> dst [G][D] fp32 (LayerNorm, then L2 if do_l2)
struct PoolScratch {
  float *logits, *stats, *zpart, *z, *enc, *pooled;
  size_t zpart_floats;  // capacity of zpart (the output projection's split-K partials reuse it)
};

int run_pooler(Fwd& f, const PoolerW& pw, const void* feat, int M, int G, int Sg, int D, int NH,
               const PoolScratch& sc, int do_l2, float* dst) {
  using namespace vp;
  const int dp = pw.dp;
  const double bytes = 2.0 * M * D * (f.bf ? 2 : 4);  // two streaming passes over the tokens
  VP_HIP(f.rec(PC_POOL, 2.0 * 2.0 * M * D * NH, bytes, [&] {
    hipError_t e = pool_logits(feat, f.bf, M, Sg, D, pw.U, (const bf16_t*)pw.Ut, NH, sc.logits, f.s);
    if (e != hipSuccess) return e;
    return pool_softmax_wsum(feat, f.bf, G, Sg, D, NH, sc.logits, sc.stats, sc.zpart, sc.z, f.s); }));
  // the value projection per head, then the output projection over K = NH * dp split 8 ways into zpart (free
  // again once z is summed; sized for >= G * NH * D floats), then LayerNorm (+ L2)
  const int splits = NH >= 8 && (NH * dp) % (8 * 128) == 0 && (size_t)8 * G * D <= sc.zpart_floats ? 8 : 1;
  VP_HIP(f.rec(PC_POOL, 2.0 * G * D * (double)dp * NH * 2.0, 4.0 * (double)NH * D * dp * 2.0, [&] {
    hipError_t e = small_gemm(sc.z, (int64_t)NH * D, D, pw.WvT, (int64_t)D * dp, pw.bv, dp, sc.enc, (int64_t)NH * dp,
                              dp, G, dp, D, NH, f.s);
    if (e != hipSuccess) return e;
    e = splits > 1 ? small_gemm_splitk(sc.enc, (int64_t)NH * dp, pw.WpT, pw.bp, sc.pooled, D, G, D, NH * dp, splits,
                                       sc.zpart, f.s)
                   : small_gemm(sc.enc, (int64_t)NH * dp, 0, pw.WpT, 0, pw.bp, 0, sc.pooled, D, 0, G, D, NH * dp, 1, f.s);
    if (e != hipSuccess) return e;
    return ln_l2_rows(sc.pooled, 0, D, G, D, pw.ln_g, pw.ln_b, do_l2, dst, f.s); }));
  return VP_OK;
}

int pack_text(vp_clip* c) {
  const int64_t D = c->cfg.video.model_dim;
  int rc;
  if ((rc = upload_mat(c, param_data(c, "text_encoder/token_emb/emb_var"), &c->tok))) return rc;
  if ((rc = upload_f32(c, param_data(c, "text_encoder/cls_emb"), &c->cls))) return rc;
  // PositionalEmbedding (encoders.py:190-224): [sin(t * inv) | cos(t * inv)], zero column for odd D
  std::vector<float> pos((size_t)kMaxTextLen * D, 0.0f);
  const int64_t nts = D / 2;
  const double inc = std::log(10000.0) / std::max<double>((double)nts - 1.0, 1.0);
  for (int t = 0; t < kMaxTextLen; ++t)
    for (int64_t i = 0; i < nts; ++i) {
      const double st = t * std::exp(-(double)i * inc);
      pos[(size_t)t * D + i] = (float)std::sin(st);
      pos[(size_t)t * D + nts + i] = (float)std::cos(st);
    }
  if ((rc = upload_f32(c, pos, &c->tpos))) return rc;
  std::vector<float> g(D);
  const auto& sc = param_data(c, "text_encoder/unimodal_ln/scale");
  for (int64_t d = 0; d < D; ++d) g[d] = sc[d] + 1.0f;
  if ((rc = upload_f32(c, g, &c->uln_g)) || (rc = upload_f32(c, param_data(c, "text_encoder/unimodal_ln/bias"), &c->uln_b)))
    return rc;
  const int NH = c->cfg.video.num_heads;
  return pack_stack(c, "text_encoder/unimodal_transformer/x_layers/", c->cfg.num_unimodal_layers, D, 4 * D, NH,
                    false, c->text);
}

}  // namespace

extern "C" {

int vp_clip_create(const vp_clip_config* cfg, int device, vp_clip** out) {
  if (!cfg || !out) return fail(VP_EINVAL, "null argument");
  *out = nullptr;
  if (cfg->num_auxiliary_layers < 0 || cfg->num_unimodal_layers < 0 || cfg->vocabulary_size < 1)
    return fail(VP_EINVAL, "bad LvT configuration");
  if (cfg->video.num_heads > 16) return fail(VP_ENOTSUP, "pooler kernels support up to 16 heads");
  vp_handle* v = nullptr;
  int rc = vp_create(&cfg->video, device, &v);
  if (rc) return rc;
  v->prefix = "vision_encoder/";
  v->names.clear();
  v->expected.clear();
  build_expected(v);
  vp_clip* c = new vp_clip();
  c->cfg = *cfg;
  c->device = device;
  c->video = v;
  build_clip_expected(c);
  *out = c;
  return VP_OK;
}

int vp_clip_destroy(vp_clip* c) {
  if (!c) return VP_OK;
  vp_destroy(c->video);
  hipSetDevice(c->device);
  for (auto& a : c->allocs) hipFree(a.p);
  delete c;
  return VP_OK;
}

int vp_clip_set_param(vp_clip* c, const char* name, const float* host_data, const int64_t* shape, int ndim) {
  if (!c || !name || !host_data || (ndim > 0 && !shape)) return fail(VP_EINVAL, "null argument");
  if (c->finalized) return fail(VP_ESTATE, "handle already finalized");
  if (!std::strncmp(name, "vision_encoder/", 15)) return vp_set_param(c->video, name, host_data, shape, ndim);
  auto it = c->expected.find(name);
  if (it == c->expected.end()) return fail(VP_EINVAL, std::string("unexpected parameter: ") + name);
  const auto& exp = it->second;
  bool ok = (int)exp.size() == ndim;
  for (int i = 0; ok && i < ndim; ++i) ok = exp[i] == shape[i];
  if (!ok) {
    std::string e = std::string("shape mismatch for ") + name + ": expected (";
    for (size_t i = 0; i < exp.size(); ++i) e += std::to_string(exp[i]) + (i + 1 < exp.size() ? ", " : "");
    e += ") got (";
    for (int i = 0; i < ndim; ++i) e += std::to_string(shape[i]) + (i + 1 < ndim ? ", " : "");
    return fail(VP_EINVAL, e + ")");
  }
  size_t n = 1;
  for (int i = 0; i < ndim; ++i) n *= (size_t)shape[i];
  HostParam hp;
  hp.shape.assign(shape, shape + ndim);
  hp.data.assign(host_data, host_data + n);
  c->host[name] = std::move(hp);
  return VP_OK;
}

int vp_clip_param_count(const vp_clip* c, int* count) {
  if (!c || !count) return fail(VP_EINVAL, "null argument");
  *count = (int)(c->video->names.size() + c->names.size());
  return VP_OK;
}

int vp_clip_param_name(const vp_clip* c, int index, const char** name) {
  if (!c || !name || index < 0) return fail(VP_EINVAL, "bad index");
  const int nv = (int)c->video->names.size();
  if (index < nv) {
    *name = c->video->names[index].c_str();
    return VP_OK;
  }
  if (index - nv >= (int)c->names.size()) return fail(VP_EINVAL, "bad index");
  *name = c->names[index - nv].c_str();
  return VP_OK;
}

int vp_clip_finalize(vp_clip* c) {
  if (!c) return fail(VP_EINVAL, "null handle");
  if (c->finalized) return VP_OK;
  for (const auto& n : c->names)
    if (!c->host.count(n)) return fail(VP_ESTATE, "missing parameter: " + n);
  int rc = vp_finalize(c->video);
  if (rc) return rc;
  VP_HIP(hipSetDevice(c->device));
  const vp_config& v = c->cfg.video;
  if (c->cfg.num_auxiliary_layers > 0 &&
      (rc = pack_stack(c, "auxiliary_encoder/transformers_stack/x_layers/", c->cfg.num_auxiliary_layers, v.model_dim,
                       v.mlp_dim, v.num_heads, c->bf16(), c->aux)))
    return rc;
  if ((rc = pack_pooler(c, "contrastive_vision_pooler/", v.model_dim, v.num_heads, 4 * v.model_dim / v.num_heads,
                        c->pool)) ||
      (rc = pack_text(c)))
    return rc;
  c->host.clear();
  c->finalized = true;
  return VP_OK;
}

int vp_clip_video_handle(vp_clip* c, vp_handle** video) {
  if (!c || !video) return fail(VP_EINVAL, "null argument");
  *video = c->video;
  return VP_OK;
}

int vp_clip_video_workspace_bytes(const vp_clip* c, int64_t B, int64_t T, int64_t H, int64_t W, size_t* bytes) {
  if (!c || !bytes) return fail(VP_EINVAL, "null argument");
  size_t inner = 0;
  int rc = vp_workspace_bytes(c->video, B, T, H, W, &inner);
  if (rc) return rc;
  *bytes = clip_video_ws(c, chunk_of(c->video, B, T, H, W), T, H, W, inner).total;
  return VP_OK;
}

}  // extern "C"

namespace {

// video side of FactorizedVideoCLIP over one chunk of B <= chunk_clips clips
int clip_video_chunk(vp_clip* c, const void* video, int in_dtype, int64_t B, int64_t T, int64_t H, int64_t W,
                     const float* frame_paddings, int normalize, float* video_emb, float* frame_emb,
                     void* spatial_out, void* spatiotemporal_out, void* workspace, void* stream) {
  using namespace vp;
  const bool bf = c->bf16();
  const int fdt = bf ? VP_BF16 : VP_F32;
  size_t inner = 0;
  int rc = vp_workspace_bytes(c->video, B, T, H, W, &inner);
  if (rc) return rc;
  const ClipVideoWs L = clip_video_ws(c, B, T, H, W, inner);

  const vp_config& v = c->cfg.video;
  const int P = v.patch_size, N = (int)((H / P) * (W / P)), D = v.model_dim, NH = v.num_heads;
  const int S = (int)T * N;
  const int64_t M64 = B * T * N;
  if (M64 > 0x7fffffff) return fail(VP_ENOTSUP, "too many tokens");
  const int M = (int)M64;
  // the auxiliary encoder's GEMM rows: B*T*N padded to the tile (as the vision encoder's, vp_internal.h
  // padded_rows); the padding rows of feat are zeroed, ride through the row-independent GEMM / LayerNorm
  // kernels and are never attended to or pooled (every sequence and pooling group is a block of M rows)
  const int Mp = (int)padded_rows(c->video, M64);
  char* ws = static_cast<char*>(workspace);
  void* feat = ws + L.feat;
  hipStream_t s = static_cast<hipStream_t>(stream);
  // 1. vision encoder -> vision_features [B, T*N, D] (encoders.py:833-845)
  rc = vp_forward(c->video, video, in_dtype, B, T, H, W, frame_paddings, feat, fdt, spatial_out, ws + L.inner,
                  inner, stream);
  if (rc) return rc;
  VP_HIP(hipSetDevice(c->device));
  const size_t es = bf ? 2 : 4;
  if (spatiotemporal_out)
    VP_HIP(hipMemcpyAsync(spatiotemporal_out, feat, (size_t)M * D * es, hipMemcpyDeviceToDevice, s));
  // the vision encoder's scratch regions are free again (stream order): reuse them
  const WsLayout Lv = ws_layout(c->video, B, T, H, W);
  char* wsv = ws + L.inner;
  Fwd f;
  f.s = s; f.bf = bf; f.M = Mp; f.D = D; f.NH = NH; f.cap = v.atten_logit_cap;
  f.hb = wsv + Lv.hbuf; f.big = wsv + Lv.big;
  f.st_part = reinterpret_cast<float*>(wsv + Lv.st_part);
  f.ln_rs = reinterpret_cast<float*>(wsv + Lv.ln_rs);
  f.pf = &c->video->prof;
  // 2. auxiliary encoder over all T*N tokens of each clip (encoders.py:846-857; paddings None)
  if (c->cfg.num_auxiliary_layers > 0) {
    if (Mp > M) VP_HIP(hipMemsetAsync(static_cast<char*>(feat) + (size_t)M * D * es, 0, (size_t)(Mp - M) * D * es, s));
    if (bf)
      VP_HIP(f.rec(PC_LAYERNORM, 0.0, (double)M * D * 2, [&] {
        return ln_row_stats((const bf16_t*)feat, Mp, D, f.ln_rs, s); }));
    rc = f.run_stack(c->aux, feat, (int)B, S, nullptr, v.mlp_dim, PC_ATTN_AUX, ATT_LONG, bf, false);
    if (rc) return rc;
  }
  // 3. contrastive pooler + L2 (encoders.py:859-872), and per frame (:874-885)
  float* logits = reinterpret_cast<float*>(ws + L.logits);
  float* stats = reinterpret_cast<float*>(ws + L.stats);
  float* zpart = reinterpret_cast<float*>(ws + L.zpart);
  float* z = reinterpret_cast<float*>(ws + L.z);
  float* enc = reinterpret_cast<float*>(ws + L.enc);
  float* pooled = reinterpret_cast<float*>(ws + L.pooled);
  const PoolScratch sc{logits, stats, zpart, z, enc, pooled, (L.z - L.zpart) / 4};
  auto pool = [&](int G, int Sg, float* dst) -> int {
    return run_pooler(f, c->pool, feat, M, G, Sg, D, NH, sc, normalize, dst);
  };
  if ((rc = pool((int)B, S, video_emb))) return rc;
  if (frame_emb && (rc = pool((int)(B * T), N, frame_emb))) return rc;
  return VP_OK;
}

}  // namespace

extern "C" {

int vp_clip_encode_video(vp_clip* c, const void* video, int in_dtype, int64_t B, int64_t T, int64_t H, int64_t W,
                         const float* frame_paddings, int normalize, float* video_emb, float* frame_emb,
                         void* spatial_out, void* spatiotemporal_out, int out_dtype, void* workspace,
                         size_t ws_bytes, void* stream) {
  if (!c || !video || !video_emb || !workspace) return fail(VP_EINVAL, "null argument");
  if (!c->finalized) return fail(VP_ESTATE, "vp_clip_finalize has not been called");
  const int fdt = c->bf16() ? VP_BF16 : VP_F32;
  if (spatiotemporal_out && out_dtype != fdt)
    return fail(VP_EINVAL, "spatiotemporal_features are returned in the fprop dtype");
  if ((in_dtype != VP_F32 && in_dtype != VP_BF16 && in_dtype != VP_U8) ||
      (out_dtype != VP_F32 && out_dtype != VP_BF16))
    return fail(VP_EINVAL, "bad dtype");
  size_t need = 0;
  int rc = vp_clip_video_workspace_bytes(c, B, T, H, W, &need);
  if (rc) return rc;
  if (ws_bytes < need) return fail(VP_EINVAL, "workspace too small: need " + std::to_string(need));
  // the batch in chunks of independent clips (vp_internal.h chunk_clips)
  const int64_t Bc = chunk_of(c->video, B, T, H, W);
  const vp_config& v = c->cfg.video;
  const int64_t N = (H / v.patch_size) * (W / v.patch_size), D = v.model_dim;
  const size_t in_clip = (size_t)(T * H * W * 3) * (in_dtype == VP_U8 ? 1 : in_dtype == VP_BF16 ? 2 : 4);
  // spatial and spatio-temporal features are written in the fprop dtype (vp_forward's out dtype)
  const size_t st_clip = (size_t)(T * N * D) * (c->bf16() ? 2 : 4);
  for (int64_t b0 = 0; b0 < B; b0 += Bc) {
    const int64_t nb = std::min(Bc, B - b0);
    rc = clip_video_chunk(c, static_cast<const char*>(video) + b0 * in_clip, in_dtype, nb, T, H, W,
                          frame_paddings ? frame_paddings + b0 * T : nullptr, normalize, video_emb + b0 * D,
                          frame_emb ? frame_emb + b0 * T * D : nullptr,
                          spatial_out ? static_cast<char*>(spatial_out) + b0 * st_clip : nullptr,
                          spatiotemporal_out ? static_cast<char*>(spatiotemporal_out) + b0 * st_clip : nullptr,
                          workspace, stream);
    if (rc) return rc;
  }
  return VP_OK;
}

int vp_clip_text_workspace_bytes(const vp_clip* c, int64_t Q, int64_t L, size_t* bytes) {
  if (!c || !bytes) return fail(VP_EINVAL, "null argument");
  if (Q < 1 || L < 1 || L + 1 > kMaxTextLen) return fail(VP_EINVAL, "text ids must be [Q, L] with 1 <= L < 1024");
  *bytes = clip_text_ws(c, Q, L).total;
  return VP_OK;
}

int vp_clip_encode_text(vp_clip* c, const int32_t* ids, const float* paddings, int64_t Q, int64_t L, int normalize,
                        float* text_emb, void* workspace, size_t ws_bytes, void* stream) {
  using namespace vp;
  if (!c || !ids || !paddings || !text_emb || !workspace) return fail(VP_EINVAL, "null argument");
  if (!c->finalized) return fail(VP_ESTATE, "vp_clip_finalize has not been called");
  if (Q < 1 || L < 1 || L + 1 > kMaxTextLen) return fail(VP_EINVAL, "text ids must be [Q, L] with 1 <= L < 1024");
  const ClipTextWs w = clip_text_ws(c, Q, L);
  if (ws_bytes < w.total) return fail(VP_EINVAL, "workspace too small: need " + std::to_string(w.total));
  if (w.Mt > 0x7fffffff) return fail(VP_ENOTSUP, "too many text tokens");
  VP_HIP(hipSetDevice(c->device));
  hipStream_t s = static_cast<hipStream_t>(stream);
  const bool bf = c->bf16();
  const vp_config& v = c->cfg.video;
  const int D = v.model_dim;
  char* ws = static_cast<char*>(workspace);
  void* x = ws + w.x;
  float* pad = reinterpret_cast<float*>(ws + w.pad);
  // The text tower keeps its residual stream in fp32 in both modes (bf16 GEMM operands, fp32
  // sums): its Q*(L+1) rows cost nothing, and it removes the stream's per-layer bf16 rounding.
  // Rows past Q*(L+1) only pad the GEMMs' M to a tile multiple: keep them finite.
  VP_HIP(hipMemsetAsync(x, 0, (size_t)w.Mt * D * 4, s));
  VP_HIP(hipMemsetAsync(pad, 0, (size_t)w.Mt * 4, s));
  VP_HIP(text_embed(ids, (int)Q, (int)L, c->tok, bf, c->cfg.vocabulary_size, c->cls, c->tpos, std::sqrt((float)D), D,
                    x, 0, paddings, pad, s));
  Fwd f;
  f.s = s; f.bf = bf; f.M = (int)w.Mt; f.D = D; f.NH = v.num_heads; f.cap = v.atten_logit_cap;
  f.causal = c->cfg.enable_causal_atten ? 1 : 0;
  f.xs_f32 = true;
  f.small_m = w.small;
  f.hb = ws + w.hb; f.big = ws + w.big;
  f.pf = &c->video->prof;
  f.cls_all = PC_ATTN_TEXT;  // the whole text tower in one profiler class ("text_tower"), so the vision GEMM
                             // classes (and bench.py's dominant-kernel roofline) hold the vision launches only
  int rc = f.run_stack(c->text, x, (int)Q, (int)L + 1, pad, 4 * D, PC_ATTN_TEXT, ATT_TEXT, false, true);
  if (rc) return rc;
  // unimodal_ln on the CLS rows, then L2 (encoders.py:752-758, :905-908)
  VP_HIP(ln_l2_rows(static_cast<float*>(x) + (size_t)L * D, 0, (int64_t)(L + 1) * D, (int)Q, D, c->uln_g,
                    c->uln_b, normalize, text_emb, s));
  return VP_OK;
}

}  // extern "C"

// ------------------------------------------------------------------------------------------
// FactorizedVideoClassifier (encoders.py:583-653): encoder -> AttenTokenPoolingLayer(hidden D,
// dim_per_head D/heads, paddings None) -> Dense(num_classes)
// ------------------------------------------------------------------------------------------
struct vp_classifier {
  vp_config cfg;
  int num_classes = 0;
  int device = 0;
  bool finalized = false;
  vp_handle* video = nullptr;  // 'encoder/' leaves
  std::map<std::string, vpi::HostParam> host;
  std::vector<std::string> names;
  std::map<std::string, std::vector<int64_t>> expected;
  std::vector<vpi::DevBuf> allocs;
  bool bf16() const { return cfg.fprop_dtype == VP_BF16; }
  PoolerW pool;                  // atten_pooler
  float *wproj = nullptr, *bproj = nullptr;  // projection kernel [D][C] (= Wt of small_gemm), bias [C]
};

extern "C" {

int vp_classifier_create(const vp_config* cfg, int num_classes, int device, vp_classifier** out) {
  if (!cfg || !out) return fail(VP_EINVAL, "null argument");
  *out = nullptr;
  if (num_classes < 1) return fail(VP_EINVAL, "num_classes must be positive");
  if (cfg->num_heads > 16) return fail(VP_ENOTSUP, "pooler kernels support up to 16 heads");
  vp_handle* v = nullptr;
  int rc = vp_create(cfg, device, &v);
  if (rc) return rc;
  v->prefix = "encoder/";
  v->names.clear();
  v->expected.clear();
  build_expected(v);
  vp_classifier* c = new vp_classifier();
  c->cfg = *cfg;
  c->num_classes = num_classes;
  c->device = device;
  c->video = v;
  const int64_t D = cfg->model_dim, NH = cfg->num_heads;
  add_pooler_expected(c, "atten_pooler/", D, NH, D / NH);
  add_expected(c, "projection/linear/kernel", {D, (int64_t)num_classes});
  add_expected(c, "projection/linear/bias", {(int64_t)num_classes});
  *out = c;
  return VP_OK;
}

int vp_classifier_destroy(vp_classifier* c) {
  if (!c) return VP_OK;
  vp_destroy(c->video);
  hipSetDevice(c->device);
  for (auto& a : c->allocs) hipFree(a.p);
  delete c;
  return VP_OK;
}

int vp_classifier_set_param(vp_classifier* c, const char* name, const float* host_data, const int64_t* shape,
                            int ndim) {
  if (!c || !name || !host_data || (ndim > 0 && !shape)) return fail(VP_EINVAL, "null argument");
  if (c->finalized) return fail(VP_ESTATE, "handle already finalized");
  if (!std::strncmp(name, "encoder/", 8)) return vp_set_param(c->video, name, host_data, shape, ndim);
  auto it = c->expected.find(name);
  if (it == c->expected.end()) return fail(VP_EINVAL, std::string("unexpected parameter: ") + name);
  const auto& exp = it->second;
  bool ok = (int)exp.size() == ndim;
  for (int i = 0; ok && i < ndim; ++i) ok = exp[i] == shape[i];
  if (!ok) return fail(VP_EINVAL, std::string("shape mismatch for ") + name);
  size_t n = 1;
  for (int i = 0; i < ndim; ++i) n *= (size_t)shape[i];
  HostParam hp;
  hp.shape.assign(shape, shape + ndim);
  hp.data.assign(host_data, host_data + n);
  c->host[name] = std::move(hp);
  return VP_OK;
}

int vp_classifier_param_count(const vp_classifier* c, int* count) {
  if (!c || !count) return fail(VP_EINVAL, "null argument");
  *count = (int)(c->video->names.size() + c->names.size());
  return VP_OK;
}

int vp_classifier_param_name(const vp_classifier* c, int index, const char** name) {
  if (!c || !name || index < 0) return fail(VP_EINVAL, "bad index");
  const int nv = (int)c->video->names.size();
  if (index < nv) {
    *name = c->video->names[index].c_str();
    return VP_OK;
  }
  if (index - nv >= (int)c->names.size()) return fail(VP_EINVAL, "bad index");
  *name = c->names[index - nv].c_str();
  return VP_OK;
}

int vp_classifier_finalize(vp_classifier* c) {
  if (!c) return fail(VP_EINVAL, "null handle");
  if (c->finalized) return VP_OK;
  for (const auto& n : c->names)
    if (!c->host.count(n)) return fail(VP_ESTATE, "missing parameter: " + n);
  int rc = vp_finalize(c->video);
  if (rc) return rc;
  VP_HIP(hipSetDevice(c->device));
  const int64_t D = c->cfg.model_dim, NH = c->cfg.num_heads;
  if ((rc = pack_pooler(c, "atten_pooler/", D, NH, D / NH, c->pool)) ||
      (rc = upload_f32(c, param_data(c, "projection/linear/kernel"), &c->wproj)) ||
      (rc = upload_f32(c, param_data(c, "projection/linear/bias"), &c->bproj)))
    return rc;
  c->host.clear();
  c->finalized = true;
  return VP_OK;
}

int vp_classifier_video_handle(vp_classifier* c, vp_handle** video) {
  if (!c || !video) return fail(VP_EINVAL, "null argument");
  *video = c->video;
  return VP_OK;
}

int vp_classifier_workspace_bytes(const vp_classifier* c, int64_t B, int64_t T, int64_t H, int64_t W,
                                  size_t* bytes) {
  if (!c || !bytes) return fail(VP_EINVAL, "null argument");
  size_t inner = 0;
  int rc = vp_workspace_bytes(c->video, B, T, H, W, &inner);
  if (rc) return rc;
  const int64_t Bc = chunk_of(c->video, B, T, H, W);
  const ClipVideoWs L = pool_video_ws(c->cfg, Bc, T, H, W, inner, c->cfg.model_dim / c->cfg.num_heads);
  *bytes = L.total + align256((size_t)Bc * c->cfg.model_dim * 4);
  return VP_OK;
}

}  // extern "C"

namespace {

// FactorizedVideoClassifier over one chunk of B <= chunk_clips clips
int classifier_chunk(vp_classifier* c, const void* video, int in_dtype, int64_t B, int64_t T, int64_t H,
                     int64_t W, const float* frame_paddings, float* logits, float* embeddings,
                     void* spatial_out, void* spatiotemporal_out, void* workspace, void* stream) {
  using namespace vp;
  const bool bf = c->bf16();
  const int fdt = bf ? VP_BF16 : VP_F32;
  size_t inner = 0;
  int rc = vp_workspace_bytes(c->video, B, T, H, W, &inner);
  if (rc) return rc;
  const vp_config& v = c->cfg;
  const int D = v.model_dim, NH = v.num_heads;
  const ClipVideoWs L = pool_video_ws(v, B, T, H, W, inner, D / NH);
  const int P = v.patch_size, N = (int)((H / P) * (W / P));
  const int M = (int)(B * T * N);
  char* ws = static_cast<char*>(workspace);
  void* feat = ws + L.feat;
  hipStream_t s = static_cast<hipStream_t>(stream);
  // 1. encoder -> features [B, T*N, D] (encoders.py:621-630)
  rc = vp_forward(c->video, video, in_dtype, B, T, H, W, frame_paddings, feat, fdt, spatial_out, ws + L.inner,
                  inner, stream);
  if (rc) return rc;
  VP_HIP(hipSetDevice(c->device));
  if (spatiotemporal_out)
    VP_HIP(hipMemcpyAsync(spatiotemporal_out, feat, (size_t)M * D * (bf ? 2 : 4), hipMemcpyDeviceToDevice, s));
  Fwd f;
  f.s = s; f.bf = bf; f.M = M; f.D = D; f.NH = NH; f.cap = v.atten_logit_cap;
  f.pf = &c->video->prof;
  // 2. atten_pooler over all T*N tokens, paddings None (:634-641); 3. projection (:646-652)
  float* emb = embeddings ? embeddings : reinterpret_cast<float*>(ws + L.total);
  const PoolScratch sc{reinterpret_cast<float*>(ws + L.logits), reinterpret_cast<float*>(ws + L.stats),
                       reinterpret_cast<float*>(ws + L.zpart), reinterpret_cast<float*>(ws + L.z),
                       reinterpret_cast<float*>(ws + L.enc), reinterpret_cast<float*>(ws + L.pooled),
                       (L.z - L.zpart) / 4};
  if ((rc = run_pooler(f, c->pool, feat, M, (int)B, (int)(T * N), D, NH, sc, 0, emb))) return rc;
  VP_HIP(small_gemm(emb, D, 0, c->wproj, 0, c->bproj, 0, logits, c->num_classes, 0, (int)B, c->num_classes, D, 1, s));
  return VP_OK;
}

}  // namespace

extern "C" {

int vp_classifier_forward(vp_classifier* c, const void* video, int in_dtype, int64_t B, int64_t T, int64_t H,
                          int64_t W, const float* frame_paddings, float* logits, float* embeddings,
                          void* spatial_out, void* spatiotemporal_out, int out_dtype, void* workspace,
                          size_t ws_bytes, void* stream) {
  if (!c || !video || !logits || !workspace) return fail(VP_EINVAL, "null argument");
  if (!c->finalized) return fail(VP_ESTATE, "vp_classifier_finalize has not been called");
  const int fdt = c->bf16() ? VP_BF16 : VP_F32;
  if (spatiotemporal_out && out_dtype != fdt)
    return fail(VP_EINVAL, "spatiotemporal_features are returned in the fprop dtype");
  if ((in_dtype != VP_F32 && in_dtype != VP_BF16 && in_dtype != VP_U8) ||
      (out_dtype != VP_F32 && out_dtype != VP_BF16))
    return fail(VP_EINVAL, "bad dtype");
  size_t need = 0;
  int rc = vp_classifier_workspace_bytes(c, B, T, H, W, &need);
  if (rc) return rc;
  if (ws_bytes < need) return fail(VP_EINVAL, "workspace too small: need " + std::to_string(need));
  const int64_t Bc = chunk_of(c->video, B, T, H, W);
  const int64_t N = (H / c->cfg.patch_size) * (W / c->cfg.patch_size), D = c->cfg.model_dim;
  const size_t in_clip = (size_t)(T * H * W * 3) * (in_dtype == VP_U8 ? 1 : in_dtype == VP_BF16 ? 2 : 4);
  const size_t st_clip = (size_t)(T * N * D) * (c->bf16() ? 2 : 4);  // features in the fprop dtype
  for (int64_t b0 = 0; b0 < B; b0 += Bc) {
    const int64_t nb = std::min(Bc, B - b0);
    rc = classifier_chunk(c, static_cast<const char*>(video) + b0 * in_clip, in_dtype, nb, T, H, W,
                          frame_paddings ? frame_paddings + b0 * T : nullptr, logits + b0 * c->num_classes,
                          embeddings ? embeddings + b0 * D : nullptr,
                          spatial_out ? static_cast<char*>(spatial_out) + b0 * st_clip : nullptr,
                          spatiotemporal_out ? static_cast<char*>(spatiotemporal_out) + b0 * st_clip : nullptr,
                          workspace, stream);
    if (rc) return rc;
  }
  return VP_OK;
}

}  // extern "C"
