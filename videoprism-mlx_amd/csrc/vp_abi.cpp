// C-ABI implementation (include/videoprism_hip.h): parameter intake in the reference's
// Flax layout, packing into kernel-ready device buffers, and the FactorizedEncoder
// forward schedule (encoders.py:411-580) over the HIP kernels.
#include "../../include/videoprism_hip.h"

#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "vp_kernels.h"

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define VP_HIP(expr)                                                                   \
  do {                                                                                 \
    hipError_t _e = (expr);                                                            \
    if (_e != hipSuccess)                                                              \
      return fail(VP_EHIP, std::string(#expr) + ": " + hipGetErrorString(_e));        \
  } while (0)

uint16_t host_f2bf(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  if ((u & 0x7F800000u) == 0x7F800000u) return (uint16_t)(u >> 16);  // inf / nan
  u += 0x7FFFu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

// jax.image.resize(method='bilinear') weights W[in][out] (restated in oracle/ and DESIGN.md:
// triangle kernel, half-pixel centres, antialiased when downsampling, normalised columns).
std::vector<double> resize_weights(int in_size, int out_size) {
  std::vector<double> w((size_t)in_size * out_size, 0.0);
  const double scale = (double)out_size / in_size;
  const double inv_scale = 1.0 / scale;
  const double kscale = std::max(inv_scale, 1.0);
  for (int o = 0; o < out_size; ++o) {
    const double sf = (o + 0.5) * inv_scale - 0.5;
    double tot = 0.0;
    for (int i = 0; i < in_size; ++i) {
      const double x = std::fabs(sf - i) / kscale;
      const double v = std::max(0.0, 1.0 - x);
      w[(size_t)i * out_size + o] = v;
      tot += v;
    }
    const bool inside = sf >= -0.5 && sf <= in_size - 0.5;
    for (int i = 0; i < in_size; ++i) {
      double& v = w[(size_t)i * out_size + o];
      if (!inside || !(std::fabs(tot) > 1000.0 * 1.1920928955078125e-07)) v = 0.0;
      else v = v / (tot != 0.0 ? tot : 1.0);
    }
  }
  return w;
}

struct HostParam {
  std::vector<int64_t> shape;
  std::vector<float> data;
};

struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
};

struct LayerW {  // one transformer layer, packed
  void* wqkv = nullptr;  // [3D][D]   rows (q|k|v, head, dh); q rows scaled by dh^-0.5
  float* bqkv = nullptr; // [3D]
  void* wpost = nullptr; // [D][D]    (out d, in n*H+h)
  float* bpost = nullptr;
  float *ln1_g = nullptr, *ln1_b = nullptr, *ln2_g = nullptr, *ln2_b = nullptr;
  void* w1 = nullptr;    // [F][D]
  float* b1 = nullptr;
  // bf16 handles fold LN1 / LN2 into the consuming GEMM (EPI_*_LN): wqkv / w1 hold
  // W' = W diag(1+scale), bqkv / b1 hold b + W beta, and c = row sums of bf16(W')
  float* cqkv = nullptr;
  float* c1 = nullptr;
  void* w2 = nullptr;    // [D][F]
  float* b2 = nullptr;
};

constexpr int kMaxT = 32;

enum ProfClass {
  PC_PATCHIFY = 0, PC_GEMM_PATCH, PC_LAYERNORM, PC_GEMM_QKV, PC_ATTN_SPATIAL, PC_ATTN_TEMPORAL,
  PC_GEMM_POST, PC_GEMM_FFN1, PC_GEMM_FFN2, PC_MISC, PC_COUNT
};
const char* kProfNames[PC_COUNT] = {"patchify", "gemm_patch_embed", "layernorm", "gemm_qkv",
                                    "attention_spatial", "attention_temporal", "gemm_post",
                                    "gemm_ffn1_gelu", "gemm_ffn2", "misc"};

// HIP-event profiler: start/stop events around each launch on the launch stream.
struct Profiler {
  int cap = 0, used = 0;
  std::vector<hipEvent_t> ev;
  std::vector<int> cls;
  std::vector<double> flops, bytes;
};

}  // namespace

struct vp_handle {
  vp_config cfg;
  int device = 0;
  bool finalized = false;
  std::map<std::string, HostParam> host;
  std::vector<std::string> names;
  std::map<std::string, std::vector<int64_t>> expected;
  std::vector<DevBuf> allocs;
  // packed device weights
  int kpad = 0;
  void* wpatch = nullptr;      // [D][kpad]
  float* bpatch = nullptr;
  float* spatial_pos = nullptr;    // [pos_h*pos_w][D]
  float* temporal_pos = nullptr;   // [kMaxT+1][kMaxT][D]: table for T at offset T*kMaxT*D
  std::vector<LayerW> spatial, temporal;
  float *sln_g = nullptr, *sln_b = nullptr, *tln_g = nullptr, *tln_b = nullptr;
  Profiler prof;
};

namespace {

bool is_bf16(const vp_handle* h) { return h->cfg.fprop_dtype == VP_BF16; }

int dev_alloc(vp_handle* h, size_t bytes, void** out) {
  void* p = nullptr;
  if (hipMalloc(&p, bytes) != hipSuccess) return fail(VP_ENOMEM, "hipMalloc failed");
  h->allocs.push_back({p, bytes});
  *out = p;
  return VP_OK;
}

int upload_f32(vp_handle* h, const std::vector<float>& v, float** out) {
  void* p;
  int rc = dev_alloc(h, v.size() * 4, &p);
  if (rc) return rc;
  VP_HIP(hipMemcpy(p, v.data(), v.size() * 4, hipMemcpyHostToDevice));
  *out = static_cast<float*>(p);
  return VP_OK;
}

// matrix in the handle's compute dtype
int upload_mat(vp_handle* h, const std::vector<float>& v, void** out) {
  if (!is_bf16(h)) {
    float* p;
    int rc = upload_f32(h, v, &p);
    *out = p;
    return rc;
  }
  std::vector<uint16_t> b(v.size());
  for (size_t i = 0; i < v.size(); ++i) b[i] = host_f2bf(v[i]);
  void* p;
  int rc = dev_alloc(h, b.size() * 2, &p);
  if (rc) return rc;
  VP_HIP(hipMemcpy(p, b.data(), b.size() * 2, hipMemcpyHostToDevice));
  *out = p;
  return VP_OK;
}

void add_expected(vp_handle* h, const std::string& n, std::vector<int64_t> s) {
  h->names.push_back(n);
  h->expected[n] = std::move(s);
}

void build_expected(vp_handle* h) {
  const vp_config& c = h->cfg;
  const int64_t D = c.model_dim, F = c.mlp_dim, NH = c.num_heads, DH = c.model_dim / c.num_heads;
  const int64_t P = c.patch_size;
  add_expected(h, "patch_projection/linear/kernel", {P * P * 3, D});
  add_expected(h, "patch_projection/linear/bias", {D});
  add_expected(h, "spatial_pos_emb/emb_var", {(int64_t)c.pos_emb_h * c.pos_emb_w, D});
  const char* stacks[2] = {"spatial_encoder", "temporal_encoder"};
  const int64_t Ls[2] = {c.num_spatial_layers, c.num_temporal_layers};
  for (int s = 0; s < 2; ++s) {
    const std::string pre = std::string(stacks[s]) + "/transformers_stack/x_layers/";
    const int64_t L = Ls[s];
    add_expected(h, pre + "layer_norm/scale", {L, D});
    add_expected(h, pre + "layer_norm/bias", {L, D});
    for (const char* qkv : {"query", "key", "value"}) {
      add_expected(h, pre + "self_attention/" + qkv + "/w", {L, D, NH, DH});
      add_expected(h, pre + "self_attention/" + qkv + "/b", {L, NH, DH});
    }
    add_expected(h, pre + "self_attention/post/w", {L, D, NH, DH});
    add_expected(h, pre + "self_attention/post/b", {L, D});
    add_expected(h, pre + "ff_layer/layer_norm/scale", {L, D});
    add_expected(h, pre + "ff_layer/layer_norm/bias", {L, D});
    add_expected(h, pre + "ff_layer/ffn_layer1/linear/kernel", {L, D, F});
    add_expected(h, pre + "ff_layer/ffn_layer1/linear/bias", {L, F});
    add_expected(h, pre + "ff_layer/ffn_layer2/linear/kernel", {L, F, D});
    add_expected(h, pre + "ff_layer/ffn_layer2/linear/bias", {L, D});
    if (s == 0) {
      add_expected(h, "spatial_ln/scale", {D});
      add_expected(h, "spatial_ln/bias", {D});
      add_expected(h, "temporal_pos_emb/emb_var", {(int64_t)c.pos_emb_t, D});
    }
  }
  add_expected(h, "temporal_ln/scale", {D});
  add_expected(h, "temporal_ln/bias", {D});
}

const std::vector<float>& param_data(vp_handle* h, const std::string& n) { return h->host.at(n).data; }

// LayerNorm folded into the following GEMM (bf16 handles): w [N][K] *= gamma[k],
// b[n] += sum_k w[n][k] beta[k] (before scaling, fp64), c[n] = sum_k bf16(w'[n][k]) (fp64).
// LN(x).W + b = rstd * (x.W') - mean*rstd * c + b'   (layers.py:208-270 with :273-313)
std::vector<float> fold_ln(std::vector<float>& w, std::vector<float>& b, const std::vector<float>& gamma,
                           const std::vector<float>& beta, int64_t N, int64_t K) {
  std::vector<float> c(N);
  for (int64_t n = 0; n < N; ++n) {
    double bb = b[n], cs = 0.0;
    float* row = w.data() + (size_t)n * K;
    for (int64_t k = 0; k < K; ++k) {
      bb += (double)row[k] * beta[k];
      row[k] = row[k] * gamma[k];
      const uint16_t r = host_f2bf(row[k]);
      uint32_t u = (uint32_t)r << 16;
      float rf;
      std::memcpy(&rf, &u, 4);
      cs += rf;
    }
    b[n] = (float)bb;
    c[n] = (float)cs;
  }
  return c;
}

int pack_stack(vp_handle* h, const std::string& stack, int L, std::vector<LayerW>& out) {
  const int64_t D = h->cfg.model_dim, F = h->cfg.mlp_dim;
  const float qscale = 1.0f / std::sqrt((float)(D / h->cfg.num_heads));  // layers.py:576-583
  const std::string pre = stack + "/transformers_stack/x_layers/";
  const auto& lng = param_data(h, pre + "layer_norm/scale");
  const auto& lnb = param_data(h, pre + "layer_norm/bias");
  const auto& ln2g = param_data(h, pre + "ff_layer/layer_norm/scale");
  const auto& ln2b = param_data(h, pre + "ff_layer/layer_norm/bias");
  const std::vector<float>* wq[3] = {&param_data(h, pre + "self_attention/query/w"),
                                     &param_data(h, pre + "self_attention/key/w"),
                                     &param_data(h, pre + "self_attention/value/w")};
  const std::vector<float>* bq[3] = {&param_data(h, pre + "self_attention/query/b"),
                                     &param_data(h, pre + "self_attention/key/b"),
                                     &param_data(h, pre + "self_attention/value/b")};
  const auto& wpost = param_data(h, pre + "self_attention/post/w");
  const auto& bpost = param_data(h, pre + "self_attention/post/b");
  const auto& w1 = param_data(h, pre + "ff_layer/ffn_layer1/linear/kernel");
  const auto& b1 = param_data(h, pre + "ff_layer/ffn_layer1/linear/bias");
  const auto& w2 = param_data(h, pre + "ff_layer/ffn_layer2/linear/kernel");
  const auto& b2 = param_data(h, pre + "ff_layer/ffn_layer2/linear/bias");
  out.resize(L);
  for (int l = 0; l < L; ++l) {
    LayerW& lw = out[l];
    std::vector<float> t((size_t)3 * D * D), tb((size_t)3 * D);
    for (int which = 0; which < 3; ++which) {
      const float sc = which == 0 ? qscale : 1.0f;
      const float* w = wq[which]->data() + (size_t)l * D * D;  // [D_in][N*H]
      for (int64_t k = 0; k < D; ++k)
        for (int64_t n = 0; n < D; ++n) t[((size_t)which * D + n) * D + k] = w[k * D + n] * sc;
      const float* b = bq[which]->data() + (size_t)l * D;
      for (int64_t n = 0; n < D; ++n) tb[(size_t)which * D + n] = b[n] * sc;
    }
    int rc;
    std::vector<float> g1(D), be1(D), g2(D), be2(D);
    for (int64_t i = 0; i < D; ++i) {
      g1[i] = lng[(size_t)l * D + i] + 1.0f;   // direct_scale=False (layers.py:259-260)
      be1[i] = lnb[(size_t)l * D + i];
      g2[i] = ln2g[(size_t)l * D + i] + 1.0f;
      be2[i] = ln2b[(size_t)l * D + i];
    }
    if (is_bf16(h)) {
      const std::vector<float> c = fold_ln(t, tb, g1, be1, 3 * D, D);
      if ((rc = upload_f32(h, c, &lw.cqkv))) return rc;
    }
    if ((rc = upload_mat(h, t, &lw.wqkv)) || (rc = upload_f32(h, tb, &lw.bqkv))) return rc;
    // post: w[d][n][h] is already [out D][in N*H]
    std::vector<float> wp(wpost.begin() + (size_t)l * D * D, wpost.begin() + (size_t)(l + 1) * D * D);
    std::vector<float> bp(bpost.begin() + (size_t)l * D, bpost.begin() + (size_t)(l + 1) * D);
    if ((rc = upload_mat(h, wp, &lw.wpost)) || (rc = upload_f32(h, bp, &lw.bpost))) return rc;
    if ((rc = upload_f32(h, g1, &lw.ln1_g)) || (rc = upload_f32(h, be1, &lw.ln1_b)) ||
        (rc = upload_f32(h, g2, &lw.ln2_g)) || (rc = upload_f32(h, be2, &lw.ln2_b)))
      return rc;
    std::vector<float> t1((size_t)F * D), t2((size_t)D * F);
    const float* w1l = w1.data() + (size_t)l * D * F;  // [D][F]
    for (int64_t k = 0; k < D; ++k)
      for (int64_t n = 0; n < F; ++n) t1[(size_t)n * D + k] = w1l[k * F + n];
    const float* w2l = w2.data() + (size_t)l * F * D;  // [F][D]
    for (int64_t k = 0; k < F; ++k)
      for (int64_t n = 0; n < D; ++n) t2[(size_t)n * F + k] = w2l[k * D + n];
    std::vector<float> bb1(b1.begin() + (size_t)l * F, b1.begin() + (size_t)(l + 1) * F);
    std::vector<float> bb2(b2.begin() + (size_t)l * D, b2.begin() + (size_t)(l + 1) * D);
    if (is_bf16(h)) {
      const std::vector<float> c = fold_ln(t1, bb1, g2, be2, F, D);
      if ((rc = upload_f32(h, c, &lw.c1))) return rc;
    }
    if ((rc = upload_mat(h, t1, &lw.w1)) || (rc = upload_f32(h, bb1, &lw.b1)) ||
        (rc = upload_mat(h, t2, &lw.w2)) || (rc = upload_f32(h, bb2, &lw.b2)))
      return rc;
  }
  return VP_OK;
}

// workspace carve-up (all offsets 256-B aligned)
struct WsLayout {
  size_t x = 0, x2 = 0, hbuf = 0, big = 0, pad_btn = 0, pad_bnt = 0, st_part = 0, ln_rs = 0, total = 0;
};

size_t align256(size_t v) { return (v + 255) & ~(size_t)255; }

WsLayout ws_layout(const vp_handle* h, int64_t B, int64_t T, int64_t H, int64_t W) {
  const int64_t P = h->cfg.patch_size;
  const int64_t Nsp = (H / P) * (W / P);
  const int64_t M = B * T * Nsp;
  const int64_t D = h->cfg.model_dim, F = h->cfg.mlp_dim;
  const size_t es = is_bf16(h) ? 2 : 4;
  const int64_t kpad = ((P * P * 3 + 63) / 64) * 64;
  const int64_t bigcols = std::max(std::max(3 * D, F), kpad);
  WsLayout L;
  size_t off = 0;
  // residual streams: fp32, or bf16 when fprop_dtype is bf16 (Flax keeps activations in
  // fprop_dtype between layers, models.py:301-302)
  L.x = off; off = align256(off + (size_t)M * D * es);
  L.x2 = off; off = align256(off + (size_t)M * D * es);
  L.hbuf = off; off = align256(off + (size_t)M * D * es);
  L.big = off; off = align256(off + (size_t)M * bigcols * es);
  L.pad_btn = off; off = align256(off + (size_t)M * 4);
  L.pad_bnt = off; off = align256(off + (size_t)M * 4);
  // GEMM-folded LayerNorm (bf16): per-row partial statistics and (rstd, -mean*rstd)
  L.st_part = off; off = align256(off + (size_t)(D / 128) * M * 8);
  L.ln_rs = off; off = align256(off + (size_t)M * 8);
  L.total = off;
  return L;
}

int check_geometry(const vp_handle* h, int64_t B, int64_t T, int64_t H, int64_t W) {
  const int64_t P = h->cfg.patch_size;
  if (B < 1 || T < 1 || H < 1 || W < 1) return fail(VP_EINVAL, "inputs must be [B, T, H, W, 3] with positive sizes");
  if (H != W) return fail(VP_EINVAL, "assert h == w failed (encoders.py:435)");
  if (H % P || W % P)
    return fail(VP_EINVAL, "Image height (" + std::to_string(H) + ") and width (" + std::to_string(W) +
                               ") should be multiples of patch_size (" + std::to_string(P) + ").");
  if (H / P != h->cfg.pos_emb_h || W / P != h->cfg.pos_emb_w)
    return fail(VP_ENOTSUP, "patch grid must equal pos_emb_shape[1:] (no spatial interpolation yet)");
  if (T > kMaxT) return fail(VP_ENOTSUP, "T > 32 frames not supported");
  if (is_bf16(h)) {
    if (h->cfg.pos_emb_h * h->cfg.pos_emb_w != 256)
      return fail(VP_ENOTSUP, "bf16 spatial attention kernel needs a 16x16 patch grid");
    if (T > 16) return fail(VP_ENOTSUP, "bf16 temporal attention kernel needs T <= 16");
  }
  return VP_OK;
}

}  // namespace

extern "C" {

const char* vp_last_error(void) { return g_err.c_str(); }
int vp_abi_version(void) { return VP_ABI_VERSION; }

int vp_create(const vp_config* cfg, int device, vp_handle** out) {
  if (!cfg || !out) return fail(VP_EINVAL, "null argument");
  *out = nullptr;
  if (cfg->num_heads <= 0 || cfg->model_dim % cfg->num_heads)
    return fail(VP_EINVAL, "model_dim must be divisible by num_heads");
  if (cfg->model_dim / cfg->num_heads != 64) return fail(VP_ENOTSUP, "dim_per_head must be 64");
  if (cfg->model_dim % 256 || cfg->mlp_dim % 256)
    return fail(VP_ENOTSUP, "model_dim and mlp_dim must be multiples of 256");
  if (cfg->fprop_dtype != VP_F32 && cfg->fprop_dtype != VP_BF16)
    return fail(VP_EINVAL, "fprop_dtype must be VP_F32 or VP_BF16");
  if (cfg->patch_size <= 0 || cfg->pos_emb_t <= 0 || cfg->pos_emb_h <= 0 || cfg->pos_emb_w <= 0)
    return fail(VP_EINVAL, "bad patch_size / pos_emb_shape");
  if (cfg->num_spatial_layers < 0 || cfg->num_temporal_layers < 0)
    return fail(VP_EINVAL, "negative layer count");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev)
    return fail(VP_EINVAL, "invalid HIP device " + std::to_string(device));
  vp_handle* h = new vp_handle();
  h->cfg = *cfg;
  h->device = device;
  build_expected(h);
  *out = h;
  return VP_OK;
}

int vp_destroy(vp_handle* h) {
  if (!h) return VP_OK;
  hipSetDevice(h->device);
  for (auto& a : h->allocs) hipFree(a.p);
  for (auto& e : h->prof.ev) hipEventDestroy(e);
  delete h;
  return VP_OK;
}

int vp_param_count(const vp_handle* h, int* count) {
  if (!h || !count) return fail(VP_EINVAL, "null argument");
  *count = (int)h->names.size();
  return VP_OK;
}

int vp_param_name(const vp_handle* h, int index, const char** name) {
  if (!h || !name || index < 0 || index >= (int)h->names.size()) return fail(VP_EINVAL, "bad index");
  *name = h->names[index].c_str();
  return VP_OK;
}

int vp_set_param(vp_handle* h, const char* name, const float* host_data, const int64_t* shape,
                 int ndim) {
  if (!h || !name || !host_data || (ndim > 0 && !shape)) return fail(VP_EINVAL, "null argument");
  if (h->finalized) return fail(VP_ESTATE, "handle already finalized");
  auto it = h->expected.find(name);
  if (it == h->expected.end()) return fail(VP_EINVAL, std::string("unexpected parameter: ") + name);
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
  h->host[name] = std::move(hp);
  return VP_OK;
}

int vp_finalize(vp_handle* h) {
  if (!h) return fail(VP_EINVAL, "null handle");
  if (h->finalized) return VP_OK;
  for (const auto& n : h->names)
    if (!h->host.count(n)) return fail(VP_ESTATE, "missing parameter: " + n);
  VP_HIP(hipSetDevice(h->device));
  const vp_config& c = h->cfg;
  const int64_t D = c.model_dim, P = c.patch_size;
  const int64_t kreal = P * P * 3;
  h->kpad = (int)(((kreal + 63) / 64) * 64);
  int rc;
  {  // patch projection: kernel [kreal][D] -> [D][kpad]
    const auto& k = param_data(h, "patch_projection/linear/kernel");
    std::vector<float> t((size_t)D * h->kpad, 0.0f);
    for (int64_t i = 0; i < kreal; ++i)
      for (int64_t n = 0; n < D; ++n) t[(size_t)n * h->kpad + i] = k[(size_t)i * D + n];
    if ((rc = upload_mat(h, t, &h->wpatch))) return rc;
    if ((rc = upload_f32(h, param_data(h, "patch_projection/linear/bias"), &h->bpatch))) return rc;
  }
  if ((rc = upload_f32(h, param_data(h, "spatial_pos_emb/emb_var"), &h->spatial_pos))) return rc;
  {  // temporal positional tables for every T in 1..kMaxT (encoders.py:543-553)
    const auto& e = param_data(h, "temporal_pos_emb/emb_var");
    const int Tp = c.pos_emb_t;
    std::vector<float> tab((size_t)(kMaxT + 1) * kMaxT * D, 0.0f);
    for (int T = 1; T <= kMaxT; ++T) {
      float* dst = tab.data() + (size_t)T * kMaxT * D;
      if (T == Tp) {
        std::memcpy(dst, e.data(), (size_t)T * D * 4);
      } else {
        const auto w = resize_weights(Tp, T);
        for (int t = 0; t < T; ++t)
          for (int64_t d = 0; d < D; ++d) {
            double s = 0.0;
            for (int i = 0; i < Tp; ++i) s += w[(size_t)i * T + t] * e[(size_t)i * D + d];
            dst[(size_t)t * D + d] = (float)s;
          }
      }
    }
    if ((rc = upload_f32(h, tab, &h->temporal_pos))) return rc;
  }
  if ((rc = pack_stack(h, "spatial_encoder", c.num_spatial_layers, h->spatial))) return rc;
  if ((rc = pack_stack(h, "temporal_encoder", c.num_temporal_layers, h->temporal))) return rc;
  std::vector<float> g(D);
  const char* lns[2] = {"spatial_ln", "temporal_ln"};
  for (int i = 0; i < 2; ++i) {
    const auto& sc = param_data(h, std::string(lns[i]) + "/scale");
    for (int64_t d = 0; d < D; ++d) g[d] = sc[d] + 1.0f;
    float** gp = i == 0 ? &h->sln_g : &h->tln_g;
    float** bp = i == 0 ? &h->sln_b : &h->tln_b;
    if ((rc = upload_f32(h, g, gp)) || (rc = upload_f32(h, param_data(h, std::string(lns[i]) + "/bias"), bp)))
      return rc;
  }
  h->host.clear();
  h->finalized = true;
  return VP_OK;
}

int vp_workspace_bytes(const vp_handle* h, int64_t B, int64_t T, int64_t H, int64_t W,
                       size_t* bytes) {
  if (!h || !bytes) return fail(VP_EINVAL, "null argument");
  int rc = check_geometry(h, B, T, H, W);
  if (rc) return rc;
  *bytes = ws_layout(h, B, T, H, W).total;
  return VP_OK;
}

int vp_forward(vp_handle* h, const void* video, int in_dtype, int64_t B, int64_t T, int64_t H,
               int64_t W, const float* frame_paddings, void* out, int out_dtype,
               void* spatial_out, void* workspace, size_t ws_bytes, void* stream) {
  using namespace vp;
  if (!h || !video || !out || !workspace) return fail(VP_EINVAL, "null argument");
  if (!h->finalized) return fail(VP_ESTATE, "vp_finalize has not been called");
  if ((in_dtype != VP_F32 && in_dtype != VP_BF16) || (out_dtype != VP_F32 && out_dtype != VP_BF16))
    return fail(VP_EINVAL, "bad dtype");
  int rc = check_geometry(h, B, T, H, W);
  if (rc) return rc;
  const WsLayout L = ws_layout(h, B, T, H, W);
  if (ws_bytes < L.total) return fail(VP_EINVAL, "workspace too small: need " + std::to_string(L.total));
  VP_HIP(hipSetDevice(h->device));
  hipStream_t s = static_cast<hipStream_t>(stream);
  const vp_config& c = h->cfg;
  const bool bf = is_bf16(h);
  const int P_ = c.patch_size;
  const int Nsp = (int)((H / P_) * (W / P_));
  const int M = (int)(B * T * Nsp);
  const int D = c.model_dim, F = c.mlp_dim, NH = c.num_heads;
  const size_t es = bf ? 2 : 4;
  char* ws = static_cast<char*>(workspace);
  void* x = ws + L.x;
  void* x2 = ws + L.x2;
  void* hb = ws + L.hbuf;
  void* big = ws + L.big;
  float* pad_btn = nullptr;
  float* pad_bnt = nullptr;
  if (frame_paddings) {
    pad_btn = reinterpret_cast<float*>(ws + L.pad_btn);
    pad_bnt = reinterpret_cast<float*>(ws + L.pad_bnt);
    VP_HIP(expand_paddings(frame_paddings, (int)B, (int)T, Nsp, pad_btn, pad_bnt, s));
  }
  // bf16: LayerNorms inside the layers are folded into the consuming GEMMs (EPI_*_LN); the
  // residual-stream producers emit row statistics (EPI_*_ST) that ln_stats_finalize turns into
  // (rstd, -mean*rstd) per row
  float* st_part = reinterpret_cast<float*>(ws + L.st_part);
  float* ln_rs = reinterpret_cast<float*>(ws + L.ln_rs);
  auto gemm = [&](int epi, const void* A, int K, const void* Wt, int N, void* o, int64_t ldo,
                  const float* bias, const void* resid, const float* pos, int pos_rows,
                  const float* rowpad, const float* lnc = nullptr) -> hipError_t {
    EpiArgs ep;
    ep.out = o; ep.ldo = ldo; ep.bias = bias; ep.resid = resid; ep.ldr = ldo;
    ep.pos = pos; ep.pos_rows = pos_rows; ep.rowpad = rowpad;
    ep.ln_rs = ln_rs; ep.ln_c = lnc; ep.st_part = st_part; ep.st_rows = M;
    if (bf) return gemm_bf16_auto(epi, (const bf16_t*)A, K, (const bf16_t*)Wt, K, M, N, K, ep, s);
    return gemm_f32(epi, (const float*)A, K, (const float*)Wt, K, M, N, K, ep, s);
  };
  // residual-stream epilogues in the stream's dtype
  const int epi_pos = bf ? EPI_POS_BF16 : EPI_POS_F32;
  const int epi_resid = bf ? EPI_RESID_BF16 : EPI_RESID_F32;
  const int epi_resid_ffn = bf ? EPI_RESID_FFN_BF16 : EPI_RESID_FFN;
  const char* ge = bf ? gemm_bf16_check(M, 3 * D, D, D, D) : gemm_f32_check(M, 3 * D, D);
  if (ge) return fail(VP_ENOTSUP, ge);
  // profiled launch: records events around `fn` when vp_profile_enable() is active
  Profiler& pf = h->prof;
  auto rec = [&](int cls, double flops, double bytes, auto&& fn) -> hipError_t {
    if (pf.used >= pf.cap) return fn();
    const int i = pf.used++;
    hipError_t e = hipEventRecord(pf.ev[2 * i], s);
    if (e != hipSuccess) return e;
    e = fn();
    if (e != hipSuccess) return e;
    pf.cls[i] = cls; pf.flops[i] = flops; pf.bytes[i] = bytes;
    return hipEventRecord(pf.ev[2 * i + 1], s);
  };
  const double dM = M, dD = D, dF = F, dE = (double)es;
  auto gbytes = [&](double K, double N, double outb, double resid) {  // algorithmic GEMM bytes
    return dM * K * dE + N * K * dE + dM * N * outb + dM * N * resid;
  };

  // 1. tokenisation + patch projection + spatial pos-emb (encoders.py:436-514)
  const double kreal = (double)P_ * P_ * 3;
  VP_HIP(rec(PC_PATCHIFY, 0.0, dM * kreal * (in_dtype == VP_BF16 ? 2 : 4) + dM * h->kpad * dE, [&] {
    return patchify(video, in_dtype == VP_BF16, big, bf, (int)(B * T), (int)H, (int)W, 3, P_, h->kpad, s); }));
  const bool fold = bf && c.num_spatial_layers > 0;  // LN1 of spatial layer 0 folded
  VP_HIP(rec(PC_GEMM_PATCH, 2.0 * dM * kreal * dD, gbytes(kreal, dD, dE, 0), [&] {
    return gemm(fold ? EPI_POS_BF16_ST : epi_pos, big, h->kpad, h->wpatch, D, x, D, h->bpatch, nullptr,
                h->spatial_pos, Nsp, nullptr); }));
  const double ln_bytes = dM * dD * dE + dM * dD * dE;
  const double fin_bytes = dM * (D / 128) * 8.0 + dM * 8.0;
  auto finalize = [&]() {
    return rec(PC_LAYERNORM, 0.0, fin_bytes, [&] { return ln_stats_finalize(st_part, D / 128, M, ln_rs, s); });
  };
  if (fold) VP_HIP(finalize());

  auto run_stack = [&](std::vector<LayerW>& layers, void* xs, int num_seq, int S,
                       const float* pad) -> int {
    const int acls = num_seq == (int)(B * T) ? PC_ATTN_SPATIAL : PC_ATTN_TEMPORAL;
    const double aflops = 4.0 * num_seq * (double)S * S * dD;
    const double abytes = dM * 3 * dD * dE + dM * dD * dE;
    for (size_t li = 0; li < layers.size(); ++li) {
      LayerW& lw = layers[li];
      const bool last = li + 1 == layers.size();
      if (bf) {  // LN1 folded: A = the residual stream, (rstd, -mean*rstd) in ln_rs
        VP_HIP(rec(PC_GEMM_QKV, 2.0 * dM * dD * 3 * dD, gbytes(dD, 3 * dD, dE, 0), [&] {
          return gemm(EPI_BF16_LN, xs, D, lw.wqkv, 3 * D, big, 3 * D, lw.bqkv, nullptr, nullptr, 1, nullptr,
                      lw.cqkv); }));
      } else {
        VP_HIP(rec(PC_LAYERNORM, 0.0, ln_bytes, [&] {
          return layernorm(xs, bf, M, D, lw.ln1_g, lw.ln1_b, hb, bf, PERM_NONE, 1, 1, nullptr, s); }));
        VP_HIP(rec(PC_GEMM_QKV, 2.0 * dM * dD * 3 * dD, gbytes(dD, 3 * dD, dE, 0), [&] {
          return gemm(EPI_BF16, hb, D, lw.wqkv, 3 * D, big, 3 * D, lw.bqkv, nullptr, nullptr, 1, nullptr); }));
      }
      VP_HIP(rec(acls, aflops, abytes, [&] {
        if (!bf) return attention_f32((const float*)big, (float*)hb, num_seq, S, NH, c.atten_logit_cap, pad, s);
        if (S == 256) return attention_spatial_bf16((const bf16_t*)big, (bf16_t*)hb, num_seq, NH, c.atten_logit_cap, pad, s);
        return attention_temporal_bf16((const bf16_t*)big, (bf16_t*)hb, num_seq, S, NH, c.atten_logit_cap, pad, s); }));
      VP_HIP(rec(PC_GEMM_POST, 2.0 * dM * dD * dD, gbytes(dD, dD, dE, dE), [&] {
        return gemm(bf ? EPI_RESID_BF16_ST : epi_resid, hb, D, lw.wpost, D, xs, D, lw.bpost, xs, nullptr, 1,
                    nullptr); }));
      if (bf) {  // LN2 folded into ffn_layer1
        VP_HIP(finalize());
        VP_HIP(rec(PC_GEMM_FFN1, 2.0 * dM * dD * dF, gbytes(dD, dF, dE, 0), [&] {
          return gemm(EPI_GELU_BF16_LN, xs, D, lw.w1, F, big, F, lw.b1, nullptr, nullptr, 1, pad, lw.c1); }));
      } else {
        VP_HIP(rec(PC_LAYERNORM, 0.0, ln_bytes, [&] {
          return layernorm(xs, bf, M, D, lw.ln2_g, lw.ln2_b, hb, bf, PERM_NONE, 1, 1, nullptr, s); }));
        VP_HIP(rec(PC_GEMM_FFN1, 2.0 * dM * dD * dF, gbytes(dD, dF, dE, 0), [&] {
          return gemm(EPI_GELU_BF16, hb, D, lw.w1, F, big, F, lw.b1, nullptr, nullptr, 1, pad); }));
      }
      const bool st = bf && !last;  // the next layer's LN1 statistics
      VP_HIP(rec(PC_GEMM_FFN2, 2.0 * dM * dF * dD, gbytes(dF, dD, dE, dE), [&] {
        return gemm(st ? EPI_RESID_FFN_BF16_ST : epi_resid_ffn, big, F, lw.w2, D, xs, D, lw.b2, xs, nullptr, 1,
                    pad); }));
      if (st) VP_HIP(finalize());
    }
    return VP_OK;
  };
  // 2. spatial encoder over (b t) sequences of Nsp tokens
  if ((rc = run_stack(h->spatial, x, (int)(B * T), Nsp, pad_btn))) return rc;
  // 3. spatial_ln (+ optional spatial_features), transpose to (b n) t, + temporal pos-emb
  if (spatial_out)
    VP_HIP(rec(PC_LAYERNORM, 0.0, dM * dD * dE + dM * dD * (out_dtype == VP_BF16 ? 2 : 4), [&] {
      return layernorm(x, bf, M, D, h->sln_g, h->sln_b, spatial_out, out_dtype == VP_BF16, PERM_NONE, 1, 1, nullptr, s); }));
  const float* tpos = h->temporal_pos + (size_t)T * kMaxT * D;
  VP_HIP(rec(PC_LAYERNORM, 0.0, ln_bytes, [&] {
    return layernorm(x, bf, M, D, h->sln_g, h->sln_b, x2, bf, PERM_BTN_TO_BNT, (int)T, Nsp, tpos, s,
                     bf && c.num_temporal_layers > 0 ? ln_rs : nullptr); }));
  // 4. temporal encoder over (b n) sequences of T tokens
  if ((rc = run_stack(h->temporal, x2, (int)(B * Nsp), (int)T, pad_bnt))) return rc;
  // 5. temporal_ln and '(bn)td->b(tn)d'
  VP_HIP(rec(PC_LAYERNORM, 0.0, dM * dD * dE + dM * dD * (out_dtype == VP_BF16 ? 2 : 4), [&] {
    return layernorm(x2, bf, M, D, h->tln_g, h->tln_b, out, out_dtype == VP_BF16, PERM_BNT_TO_BTN, (int)T, Nsp, nullptr, s); }));
  (void)es;
  return VP_OK;
}

// ----------------------------------- profiling ----------------------------------------

int vp_profile_enable(vp_handle* h, int capacity) {
  if (!h || capacity < 0) return fail(VP_EINVAL, "bad argument");
  VP_HIP(hipSetDevice(h->device));
  Profiler& p = h->prof;
  for (auto& e : p.ev) hipEventDestroy(e);
  p.ev.clear();
  p.cap = 0;
  p.used = 0;
  p.ev.resize((size_t)capacity * 2);
  for (auto& e : p.ev) VP_HIP(hipEventCreate(&e));
  p.cls.assign(capacity, PC_MISC);
  p.flops.assign(capacity, 0.0);
  p.bytes.assign(capacity, 0.0);
  p.cap = capacity;
  return VP_OK;
}

int vp_profile_read(vp_handle* h, int nclass, double* ms, double* flops, double* bytes,
                    int64_t* launches) {
  if (!h || nclass < PC_COUNT || !ms || !flops || !bytes || !launches)
    return fail(VP_EINVAL, "bad argument");
  for (int c = 0; c < nclass; ++c) { ms[c] = 0; flops[c] = 0; bytes[c] = 0; launches[c] = 0; }
  Profiler& p = h->prof;
  if (p.used > 0) VP_HIP(hipEventSynchronize(p.ev[2 * p.used - 1]));
  for (int i = 0; i < p.used; ++i) {
    float t = 0.f;
    VP_HIP(hipEventElapsedTime(&t, p.ev[2 * i], p.ev[2 * i + 1]));
    ms[p.cls[i]] += t;
    flops[p.cls[i]] += p.flops[i];
    bytes[p.cls[i]] += p.bytes[i];
    launches[p.cls[i]] += 1;
  }
  p.used = 0;
  return VP_OK;
}

int vp_profile_class_name(int cls, const char** name) {
  if (cls < 0 || cls >= PC_COUNT || !name) return fail(VP_EINVAL, "bad class");
  *name = kProfNames[cls];
  return VP_OK;
}

int vp_profile_class_count(void) { return PC_COUNT; }

// ----------------------------------- op level -----------------------------------------

int vp_op_gemm(int precision, int epilogue, const void* A, int64_t lda, const void* W, int64_t ldw,
               int64_t M, int64_t N, int64_t K, void* out, int64_t ldo, const float* bias,
               const void* resid, int64_t ldr, const float* pos, int64_t pos_rows,
               const float* rowpad, void* stream) {
  using namespace vp;
  if (!A || !W || !out || !bias) return fail(VP_EINVAL, "null argument");
  if (epilogue < 0 || epilogue > 7) return fail(VP_EINVAL, "bad epilogue");
  const bool needs_resid = epilogue == EPI_RESID_F32 || epilogue == EPI_RESID_FFN ||
                           epilogue == EPI_RESID_BF16 || epilogue == EPI_RESID_FFN_BF16;
  if (needs_resid && !resid) return fail(VP_EINVAL, "resid required");
  if ((epilogue == EPI_POS_F32 || epilogue == EPI_POS_BF16) && (!pos || pos_rows < 1))
    return fail(VP_EINVAL, "pos required");
  if (precision == VP_F32 && epilogue > 4) return fail(VP_EINVAL, "bf16 residual epilogues need precision VP_BF16");
  EpiArgs ep;
  ep.out = out; ep.ldo = ldo; ep.bias = bias; ep.resid = resid; ep.ldr = ldr;
  ep.pos = pos; ep.pos_rows = (int)pos_rows; ep.rowpad = rowpad;
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (precision == VP_BF16) {
    const char* e = gemm_bf16_check((int)M, (int)N, (int)K, lda, ldw);
    if (e) return fail(VP_EINVAL, e);
    VP_HIP(gemm_bf16_auto(epilogue, (const bf16_t*)A, lda, (const bf16_t*)W, ldw, (int)M, (int)N, (int)K, ep, s));
  } else if (precision == VP_F32) {
    const char* e = gemm_f32_check((int)M, (int)N, (int)K);
    if (e) return fail(VP_EINVAL, e);
    VP_HIP(gemm_f32(epilogue, (const float*)A, lda, (const float*)W, ldw, (int)M, (int)N, (int)K, ep, s));
  } else {
    return fail(VP_EINVAL, "bad precision");
  }
  return VP_OK;
}

// Not in the public header: ablation builds of the bf16 GEMM (tools/gemm_bench.py).
int vp_dev_gemm_diag(int diag, const void* A, const void* W, int64_t M, int64_t N, int64_t K,
                     void* out, const float* bias, void* stream) {
  using namespace vp;
  const char* e = gemm_bf16_check((int)M, (int)N, (int)K, K, K);
  if (e) return fail(VP_EINVAL, e);
  EpiArgs ep;
  ep.out = out; ep.ldo = N; ep.bias = bias;
  VP_HIP(gemm_bf16_diag(diag, (const bf16_t*)A, K, (const bf16_t*)W, K, (int)M, (int)N, (int)K, ep,
                        static_cast<hipStream_t>(stream)));
  return VP_OK;
}

// Not in the public header: one named bf16 GEMM kernel (which = 2: gemm_bf16_ov, 4: gemm_bf16_w4,
// 8: gemm_bf16)
// with any epilogue, for kernel A/B tests (tests/test_gpu_kernels.py) and tools/gemm_bench.py.
// epi >= 1000 selects the 4-wave kernel's ablation builds.
int vp_dev_gemm_kernel(int which, int epi, const void* A, const void* W, int64_t M, int64_t N,
                       int64_t K, void* out, const float* bias, const void* resid, const float* pos,
                       int64_t pos_rows, const float* rowpad, void* stream) {
  using namespace vp;
  if (which != 2) {
    const char* e = gemm_bf16_check((int)M, (int)N, (int)K, K, K);
    if (e) return fail(VP_EINVAL, e);
  }
  EpiArgs ep;
  ep.out = out; ep.ldo = N; ep.bias = bias; ep.resid = resid; ep.ldr = N;
  ep.pos = pos; ep.pos_rows = (int)(pos_rows > 0 ? pos_rows : 1); ep.rowpad = rowpad;
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (which == 4)
    VP_HIP(gemm_bf16_w4(epi, (const bf16_t*)A, K, (const bf16_t*)W, K, (int)M, (int)N, (int)K, ep, s));
  else if (which == 8)
    VP_HIP(gemm_bf16(epi, (const bf16_t*)A, K, (const bf16_t*)W, K, (int)M, (int)N, (int)K, ep, s));
  else if (which == 2) {
    if (!gemm_bf16_ov_ok(epi >= 1000 ? 0 : epi, (int)M, (int)N, (int)K, K, K))
      return fail(VP_EINVAL, "shape/epilogue not supported by gemm_bf16_ov");
    VP_HIP(gemm_bf16_ov(epi, (const bf16_t*)A, K, (const bf16_t*)W, K, (int)M, (int)N, (int)K, ep, s));
  } else
    return fail(VP_EINVAL, "which must be 2, 4 or 8");
  return VP_OK;
}

// Not in the public header: the GEMM-folded LayerNorm pieces (tests/test_gpu_kernels.py).
// vp_dev_gemm_ln: EPI_BF16_LN / EPI_GELU_BF16_LN with (rstd, -mean*rstd) rows ln_rs and column
// sums ln_c, or EPI_*_ST writing partial row statistics to st_part ([N/128][M][2]).
int vp_dev_gemm_ln(int epi, const void* A, const void* W, int64_t M, int64_t N, int64_t K, void* out,
                   const float* bias, const void* resid, const float* pos, int64_t pos_rows,
                   const float* rowpad, const float* ln_rs, const float* ln_c, float* st_part,
                   void* stream) {
  using namespace vp;
  if (epi < EPI_BF16_LN || epi > EPI_POS_BF16_ST) return fail(VP_EINVAL, "epilogue must be 8..12");
  const char* e = gemm_bf16_check((int)M, (int)N, (int)K, K, K);
  if (e) return fail(VP_EINVAL, e);
  EpiArgs ep;
  ep.out = out; ep.ldo = N; ep.bias = bias; ep.resid = resid; ep.ldr = N;
  ep.pos = pos; ep.pos_rows = (int)(pos_rows > 0 ? pos_rows : 1); ep.rowpad = rowpad;
  ep.ln_rs = ln_rs; ep.ln_c = ln_c; ep.st_part = st_part; ep.st_rows = M;
  VP_HIP(gemm_bf16_w4(epi, (const bf16_t*)A, K, (const bf16_t*)W, K, (int)M, (int)N, (int)K, ep,
                      static_cast<hipStream_t>(stream)));
  return VP_OK;
}

// ablation builds of the spatial attention kernel (tools/attn_bench.py)
int vp_dev_attention_diag(int diag, const void* qkv, void* o, int64_t num_seq, int64_t heads, float cap,
                          void* stream) {
  VP_HIP(vp::attention_spatial_diag(diag, (const vp::bf16_t*)qkv, (vp::bf16_t*)o, (int)num_seq, (int)heads, cap,
                                    static_cast<hipStream_t>(stream)));
  return VP_OK;
}

// which = 0: ln_stats_finalize(src = st_part [D/128][M][2]); 1: ln_row_stats(src = bf16 [M][D])
int vp_dev_ln_stats(int which, const void* src, int64_t M, int64_t D, float* ln_rs, void* stream) {
  using namespace vp;
  if (D % 128 || D < 128) return fail(VP_EINVAL, "D must be a multiple of 128");
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (which == 0) VP_HIP(ln_stats_finalize((const float*)src, (int)(D / 128), M, ln_rs, s));
  else VP_HIP(ln_row_stats((const bf16_t*)src, M, (int)D, ln_rs, s));
  return VP_OK;
}

int vp_op_attention(int precision, const void* qkv, void* o, int64_t num_seq, int64_t S,
                    int64_t heads, float cap, const float* key_pad, void* stream) {
  using namespace vp;
  if (!qkv || !o || num_seq < 1 || heads < 1) return fail(VP_EINVAL, "bad argument");
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (precision == VP_BF16) {
    if (!(cap > 0.0f)) return fail(VP_ENOTSUP, "bf16 attention requires atten_logit_cap > 0");
    if (S == 256)
      VP_HIP(attention_spatial_bf16((const bf16_t*)qkv, (bf16_t*)o, (int)num_seq, (int)heads, cap, key_pad, s));
    else if (S >= 1 && S <= 16)
      VP_HIP(attention_temporal_bf16((const bf16_t*)qkv, (bf16_t*)o, (int)num_seq, (int)S, (int)heads, cap, key_pad, s));
    else
      return fail(VP_ENOTSUP, "bf16 attention supports S == 256 or S <= 16");
  } else if (precision == VP_F32) {
    if (S < 1 || S > 256) return fail(VP_ENOTSUP, "fp32 attention supports S <= 256");
    VP_HIP(attention_f32((const float*)qkv, (float*)o, (int)num_seq, (int)S, (int)heads, cap, key_pad, s));
  } else {
    return fail(VP_EINVAL, "bad precision");
  }
  return VP_OK;
}

int vp_op_layernorm(const void* x, int in_dtype, int64_t rows, int64_t D, const float* gamma,
                    const float* beta, void* out, int out_dtype, int perm, int64_t T, int64_t Nsp,
                    const float* add, void* stream) {
  using namespace vp;
  if (!x || !gamma || !beta || !out) return fail(VP_EINVAL, "null argument");
  if ((in_dtype != VP_F32 && in_dtype != VP_BF16) || (out_dtype != VP_F32 && out_dtype != VP_BF16))
    return fail(VP_EINVAL, "bad dtype");
  if (perm && (T < 1 || Nsp < 1 || rows % (T * Nsp))) return fail(VP_EINVAL, "bad permutation geometry");
  hipError_t e = layernorm(x, in_dtype == VP_BF16, (int)rows, (int)D, gamma, beta, out, out_dtype == VP_BF16,
                           perm, (int)T, (int)Nsp, add, static_cast<hipStream_t>(stream));
  if (e == hipErrorInvalidValue) return fail(VP_ENOTSUP, "layernorm: D must be 256*k, k in {1..6, 8}");
  VP_HIP(e);
  return VP_OK;
}

int vp_op_patchify(const void* video, int in_dtype, void* patches, int out_dtype, int64_t BT,
                   int64_t H, int64_t W, int64_t C, int64_t P, int64_t kpad, void* stream) {
  using namespace vp;
  if (!video || !patches || P <= 0) return fail(VP_EINVAL, "bad argument");
  if (H % P || W % P)
    return fail(VP_EINVAL, "Image height (" + std::to_string(H) + ") and width (" + std::to_string(W) +
                               ") should be multiples of patch_size (" + std::to_string(P) + ").");
  if (kpad % 8 || kpad < P * P * C) return fail(VP_EINVAL, "kpad must be >= P*P*C and a multiple of 8");
  VP_HIP(patchify(video, in_dtype == VP_BF16, patches, out_dtype == VP_BF16, (int)BT, (int)H, (int)W,
                  (int)C, (int)P, (int)kpad, static_cast<hipStream_t>(stream)));
  return VP_OK;
}

int vp_op_pool_l2(const void* emb, int dtype, int64_t B, int64_t L, int64_t D, float* out,
                  void* stream) {
  using namespace vp;
  if (!emb || !out || B < 1 || L < 1 || D < 1) return fail(VP_EINVAL, "bad argument");
  VP_HIP(pool_l2(emb, dtype == VP_BF16, (int)B, (int)L, (int)D, out, static_cast<hipStream_t>(stream)));
  return VP_OK;
}

}  // extern "C"
