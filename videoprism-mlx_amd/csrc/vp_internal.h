// Host-side internals shared by the C-ABI translation units (vp_abi.cpp: FactorizedEncoder,
// vp_clip.cpp: FactorizedVideoCLIP): parameter intake, weight packing, workspace layout and the
// pre-LN transformer-stack schedule over the HIP kernels.
#pragma once
#include "../../include/videoprism_hip.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "vp_kernels.h"

namespace vpi {

inline thread_local std::string g_err;

inline int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define VP_HIP(expr)                                                                   \
  do {                                                                                 \
    hipError_t _e = (expr);                                                            \
    if (_e != hipSuccess)                                                              \
      return fail(VP_EHIP, std::string(#expr) + ": " + hipGetErrorString(_e));        \
  } while (0)

inline uint16_t host_f2bf(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  if ((u & 0x7F800000u) == 0x7F800000u) return (uint16_t)(u >> 16);  // inf / nan
  u += 0x7FFFu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

// jax.image.resize(method='bilinear') weights W[in][out] (restated in oracle/ and DESIGN.md:
// triangle kernel, half-pixel centres, antialiased when downsampling, normalised columns).
inline std::vector<double> resize_weights(int in_size, int out_size) {
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
  // temporal layers (bf16, folded): the q and k rows of wqkv regrouped per head, [q_h | k_h] for
  // h = 0..heads-1 ([2D][D]), with their b' and c -- the first launch of the fused temporal
  // attention (EPI_QK_TATTN_LN); the v rows stay at wqkv + 2 D rows
  void* wqk = nullptr;
  float* bqk = nullptr;
  float* cqk = nullptr;
  // bf16, folded, F % 256 == 0: w1 / b1 / c1 rows permuted within each 32-row group (W row 16h + 4g + i
  // holds column 8g + 4h + i) for the FFN pair over the row-blocked hidden activation (EPI_*_BLK)
  bool ffn_blk = false;
  // spatial stacks (bf16, folded, 3D % 256 == 0): a copy of wqkv / b' / c with the rows permuted the same
  // way, for the q|k|v projection into the row-blocked layout the spatial attention reads (EPI_BF16_LN_BLK)
  void* wqkv_blk = nullptr;
  float* bqkv_blk = nullptr;
  float* cqkv_blk = nullptr;
};

// temporal positional tables precomputed by vp_finalize (T = 1..kPrecomputedT); longer clips get
// theirs from vp_prepare_frames (encoders.py:543-553 interpolates to any T)
constexpr int kPrecomputedT = 32;

enum ProfClass {
  PC_PATCHIFY = 0, PC_GEMM_PATCH, PC_LAYERNORM, PC_GEMM_QKV, PC_ATTN_SPATIAL, PC_ATTN_TEMPORAL,
  PC_GEMM_POST, PC_GEMM_FFN1, PC_GEMM_FFN2, PC_ATTN_AUX, PC_ATTN_TEXT, PC_POOL, PC_MISC,
  PC_GEMM_QKV_TATTN, PC_COUNT
};
inline const char* kProfNames[PC_COUNT] = {"patchify", "gemm_patch_embed", "layernorm", "gemm_qkv",
                                    "attention_spatial", "attention_temporal", "gemm_post",
                                    "gemm_ffn1_gelu", "gemm_ffn2", "attention_aux", "text_tower",
                                    "pooler", "misc", "gemm_qkv_temporal_attn"};

// HIP-event profiler: start/stop events around each launch on the launch stream.
struct Profiler {
  const void* kfn[PC_COUNT] = {};  // host function of the last kernel launched per class
  std::string kname[PC_COUNT];    // its demangled name (vp_profile_kernel_name)
  int cap = 0, used = 0;
  uint32_t mask = 0xffffffffu;  // kernel classes that get events (vp_profile_set_mask)
  std::vector<hipEvent_t> ev;
  std::vector<int> cls;
  std::vector<double> flops, bytes;
};

}  // namespace

struct vp_handle {
  vp_config cfg;
  int device = 0;
  std::string prefix;  // "" for a FactorizedEncoder, "vision_encoder/" inside a vp_clip
  bool bf16() const { return cfg.fprop_dtype == VP_BF16; }
  bool finalized = false;
  std::map<std::string, vpi::HostParam> host;
  std::vector<std::string> names;
  std::map<std::string, std::vector<int64_t>> expected;
  std::vector<vpi::DevBuf> allocs;
  // packed device weights
  int kpad = 0;
  void* wpatch = nullptr;      // [D][kpad]
  void* wpatch_v = nullptr;    // bf16, vp::video_patch_ok(P) (even P, 4..20): [D][video_patch_k(P)] in the frames' chunk order (fused
                               // patch embedding straight from the frames, gemm_bf16_w4_video)
  float* bpatch = nullptr;
  float* spatial_pos = nullptr;    // [pos_h*pos_w][D]
  std::vector<float> spatial_pos_host;                   // kept for other patch grids
  std::map<std::pair<int, int>, float*> grid_pos;        // interpolated tables (vp_prepare_geometry)
  std::vector<float> temporal_pos_host;                  // temporal_pos_emb/emb_var [pos_t][D]
  std::map<int, float*> temporal_pos;                    // T -> [T][D] (resampled when T != pos_t)
  std::vector<vpi::LayerW> spatial, temporal;
  float *sln_g = nullptr, *sln_b = nullptr, *tln_g = nullptr, *tln_b = nullptr;
  vpi::Profiler prof;
};

namespace vpi {

inline bool is_bf16(const vp_handle* h) { return h->bf16(); }

// device buffers owned by a handle (vp_handle or vp_clip: members allocs, bf16())
template <class H>
int dev_alloc(H* h, size_t bytes, void** out) {
  void* p = nullptr;
  if (hipMalloc(&p, bytes) != hipSuccess) return fail(VP_ENOMEM, "hipMalloc failed");
  h->allocs.push_back({p, bytes});
  *out = p;
  return VP_OK;
}

template <class H>
int upload_f32(H* h, const std::vector<float>& v, float** out) {
  void* p;
  int rc = dev_alloc(h, v.size() * 4, &p);
  if (rc) return rc;
  VP_HIP(hipMemcpy(p, v.data(), v.size() * 4, hipMemcpyHostToDevice));
  *out = static_cast<float*>(p);
  return VP_OK;
}

// matrix in the handle's compute dtype
template <class H>
int upload_mat(H* h, const std::vector<float>& v, void** out) {
  if (!h->bf16()) {
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

template <class H>
void add_expected(H* h, const std::string& n, std::vector<int64_t> s) {
  h->names.push_back(n);
  h->expected[n] = std::move(s);
}

// the 16 leaves of a scanned StackedTransformer (layers.py:940-1041) under `pre` (".../x_layers/")
template <class H>
void add_stack_expected(H* h, const std::string& pre, int64_t L, int64_t D, int64_t F, int64_t NH) {
  const int64_t DH = D / NH;
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
}

inline void build_expected(vp_handle* h) {
  const vp_config& c = h->cfg;
  const int64_t D = c.model_dim, F = c.mlp_dim, NH = c.num_heads;
  const int64_t P = c.patch_size;
  const std::string& px = h->prefix;
  add_expected(h, px + "patch_projection/linear/kernel", {P * P * 3, D});
  add_expected(h, px + "patch_projection/linear/bias", {D});
  add_expected(h, px + "spatial_pos_emb/emb_var", {(int64_t)c.pos_emb_h * c.pos_emb_w, D});
  const char* stacks[2] = {"spatial_encoder", "temporal_encoder"};
  const int64_t Ls[2] = {c.num_spatial_layers, c.num_temporal_layers};
  for (int s = 0; s < 2; ++s) {
    add_stack_expected(h, px + stacks[s] + "/transformers_stack/x_layers/", Ls[s], D, F, NH);
    if (s == 0) {
      add_expected(h, px + "spatial_ln/scale", {D});
      add_expected(h, px + "spatial_ln/bias", {D});
      add_expected(h, px + "temporal_pos_emb/emb_var", {(int64_t)c.pos_emb_t, D});
    }
  }
  add_expected(h, px + "temporal_ln/scale", {D});
  add_expected(h, px + "temporal_ln/bias", {D});
}

template <class H>
const std::vector<float>& param_data(H* h, const std::string& n) { return h->host.at(n).data; }

// LayerNorm folded into the following GEMM (bf16 handles): w [N][K] *= gamma[k],
// b[n] += sum_k w[n][k] beta[k] (before scaling, fp64), c[n] = sum_k bf16(w'[n][k]) (fp64).
// LN(x).W + b = rstd * (x.W') - mean*rstd * c + b'   (layers.py:208-270 with :273-313)
inline std::vector<float> fold_ln(std::vector<float>& w, std::vector<float>& b, const std::vector<float>& gamma,
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

// extra copies of the folded q|k|v rows a stack's attention path reads (pack_stack)
enum QkvExtra {
  QKV_PLAIN = 0,    // row-major [3D][D] only (auxiliary / text stacks)
  QKV_PER_HEAD = 1, // + [q_h | k_h] per head (temporal stacks: the fused temporal attention)
  QKV_BLOCKED = 2,  // + the row-blocked copy (spatial stacks: EPI_BF16_LN_BLK -> attn_spatial<.., true>)
};

// one scanned stack `pre` (".../x_layers/") -> L packed layers.  fold: LayerNorms folded into
// the consuming GEMMs (bf16 handles, EPI_*_LN); otherwise W / b are the plain projections and the
// LayerNorms run as kernels (ln*_g / ln*_b).  The row-major q|k|v copy is always kept: it serves the
// unfused attention paths (other patch grids, frame paddings, caps outside the fast range).
template <class H>
int pack_stack(H* h, const std::string& pre, int L, int64_t D, int64_t F, int NH, bool fold,
               std::vector<LayerW>& out, QkvExtra extra = QKV_PLAIN) {
  const bool qk_perm = extra == QKV_PER_HEAD;
  const float qscale = 1.0f / std::sqrt((float)(D / NH));  // layers.py:576-583
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
    if (fold) {
      const std::vector<float> c = fold_ln(t, tb, g1, be1, 3 * D, D);
      if ((rc = upload_f32(h, c, &lw.cqkv))) return rc;
      if (extra == QKV_BLOCKED && (3 * D) % 256 == 0) {  // the row-blocked copy (LayerW::wqkv_blk)
        const int64_t N3 = 3 * D;
        std::vector<float> pt((size_t)N3 * D), pb(N3), pc(N3);
        for (int64_t r = 0; r < N3; ++r) {
          const int64_t w = r & 31, src = (r & ~31LL) + 8 * ((w >> 2) & 3) + 4 * (w >> 4) + (w & 3);
          std::memcpy(pt.data() + (size_t)r * D, t.data() + (size_t)src * D, (size_t)D * 4);
          pb[r] = tb[src];
          pc[r] = c[src];
        }
        if ((rc = upload_mat(h, pt, &lw.wqkv_blk)) || (rc = upload_f32(h, pb, &lw.bqkv_blk)) ||
            (rc = upload_f32(h, pc, &lw.cqkv_blk)))
          return rc;
      }
      if (qk_perm) {  // [q_h | k_h] per head (rows of the folded t, b', c)
        const int64_t DH = D / NH;
        std::vector<float> tq((size_t)2 * D * D), bq((size_t)2 * D), cq((size_t)2 * D);
        for (int64_t hh = 0; hh < NH; ++hh)
          for (int which = 0; which < 2; ++which)
            for (int64_t i = 0; i < DH; ++i) {
              const int64_t src = which * D + hh * DH + i, dst = hh * 2 * DH + which * DH + i;
              std::memcpy(tq.data() + (size_t)dst * D, t.data() + (size_t)src * D, (size_t)D * 4);
              bq[dst] = tb[src];
              cq[dst] = c[src];
            }
        if ((rc = upload_mat(h, tq, &lw.wqk)) || (rc = upload_f32(h, bq, &lw.bqk)) ||
            (rc = upload_f32(h, cq, &lw.cqk)))
          return rc;
      }
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
    if (fold) {
      std::vector<float> c = fold_ln(t1, bb1, g2, be2, F, D);
      if (F % 256 == 0) {  // rows of W', b', c in the blocked FFN pair's order (LayerW::ffn_blk)
        std::vector<float> pt((size_t)F * D), pb(F), pc(F);
        for (int64_t r = 0; r < F; ++r) {
          const int64_t w = r & 31, src = (r & ~31LL) + 8 * ((w >> 2) & 3) + 4 * (w >> 4) + (w & 3);
          std::memcpy(pt.data() + (size_t)r * D, t1.data() + (size_t)src * D, (size_t)D * 4);
          pb[r] = bb1[src];
          pc[r] = c[src];
        }
        t1.swap(pt);
        bb1.swap(pb);
        c.swap(pc);
        lw.ffn_blk = true;
      }
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

inline size_t align256(size_t v) { return (v + 255) & ~(size_t)255; }

// GEMM row count: B*T*N padded to the GEMM tile (256 rows bf16, 128 fp32); the padding rows
// ride through the row-independent GEMM / LayerNorm kernels and are never read back
inline int64_t padded_rows(const vp_handle* h, int64_t M) {
  const int64_t t = is_bf16(h) ? 256 : 128;
  return (M + t - 1) / t * t;
}

inline WsLayout ws_layout(const vp_handle* h, int64_t B, int64_t T, int64_t H, int64_t W) {
  const int64_t P = h->cfg.patch_size;
  const int64_t Nsp = (H / P) * (W / P);
  const int64_t M = padded_rows(h, B * T * Nsp);
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

// Clips per forward chunk: the forward entry points process any B as consecutive chunks of at most this
// many clips (clips are independent, encoders.py:411-580), each in the same workspace, which bounds the
// workspace at about 4 GiB of FFN hidden activation (170 clips of 16 x 288 x 288).  A single clip always
// fits a chunk: the GEMMs walk an operand past the 32-bit buffer range in row ranges (gemm_bf16_w4.hip),
// so clip length is bounded by device memory only.
inline int64_t chunk_clips(const vp_config& c, int64_t T, int64_t H, int64_t W) {
  const int64_t P = c.patch_size;
  const int64_t tok = T * (H / P) * (W / P);
  const int64_t kpad = ((P * P * 3 + 63) / 64) * 64;
  const int64_t lda = std::max<int64_t>(std::max<int64_t>(c.model_dim, c.mlp_dim), kpad);
  const int64_t max_rows = (int64_t)(0xFFFFFFF0ull / (uint64_t)(2 * lda)) / 256 * 256;
  return tok > 0 ? std::max<int64_t>(1, max_rows / tok) : 1;
}

inline int check_geometry(const vp_handle* h, int64_t B, int64_t T, int64_t H, int64_t W) {
  const int64_t P = h->cfg.patch_size;
  if (B < 1 || T < 1 || H < 1 || W < 1) return fail(VP_EINVAL, "inputs must be [B, T, H, W, 3] with positive sizes");
  if (H != W) return fail(VP_EINVAL, "assert h == w failed (encoders.py:435)");
  if (H % P || W % P)
    return fail(VP_EINVAL, "Image height (" + std::to_string(H) + ") and width (" + std::to_string(W) +
                               ") should be multiples of patch_size (" + std::to_string(P) + ").");
  if (T * (H / P) * (W / P) > ((int64_t)1 << 30))
    return fail(VP_EINVAL, "one clip of " + std::to_string(T) + "x" + std::to_string(H) + "x" + std::to_string(W) +
                               " has more than 2^30 tokens (32-bit row indices)");
  return VP_OK;
}

// clips per chunk for a forward over B clips
inline int64_t chunk_of(const vp_handle* h, int64_t B, int64_t T, int64_t H, int64_t W) {
  return std::min<int64_t>(B, chunk_clips(h->cfg, T, H, W));
}

}  // namespace

namespace vpi {

// The bf16 attention kernels compute the capped softmax without a running max: every numerator
// is exp(l) with |l| <= cap, and both the row sum and the unnormalised O = sum_s exp(l_s) v_s are
// accumulated in fp32.  With cap <= 50 (the reference's value for every VideoPrism config,
// models.py:91) and S keys, |O| <= e^50 * S * max|v| stays below FLT_MAX for any |v| < 1.6e13 at
// S = 4096 (16 frames) and |v| < 1e12 at S = 65536 (256 frames of the auxiliary encoder) --
// bf16 activations of a trained model are nowhere near.  (Round 2 allowed 80,
// priced on the row sum alone: e^80 * S * |v| overflows for |v| > ~1.5 at S = 4096.)  Any other
// cap (<= 0: no capping, layers.py:586-589; > 50) takes the online-softmax kernel.
constexpr float kMaxFastCap = 50.0f;
inline bool fast_cap(float cap) { return cap > 0.0f && cap <= kMaxFastCap; }

// which attention kernel a stack uses (the rest of the pre-LN layer is shared)
enum AttnKind {
  ATT_VIDEO = 0,  // factorized encoder: S == 256 spatial / S <= 16 temporal (bf16), any S <= 256 (fp32)
  ATT_LONG = 1,   // auxiliary encoder over T*N tokens, no masks
  ATT_TEXT = 2,   // text tower: causal + key paddings (layers.py:155-179)
};

// One forward pass's launch context: stream, dtype, row count, scratch buffers and the profiler.
// hipEventRecord on `s`; inside a stream capture an event-record node of the graph instead (a
// plain record during capture only orders the capture, so a replay would not re-record it)
inline hipError_t record_event(hipEvent_t ev, hipStream_t s) {
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  hipGraph_t g = nullptr;
  const hipGraphNode_t* deps = nullptr;
  size_t nd = 0;
  hipError_t e = hipStreamGetCaptureInfo_v2(s, &cs, nullptr, &g, &deps, &nd);
  if (e != hipSuccess) return e;
  if (cs != hipStreamCaptureStatusActive) return hipEventRecord(ev, s);
  hipGraphNode_t node = nullptr;
  e = hipGraphAddEventRecordNode(&node, g, deps, nd, ev);
  if (e != hipSuccess) return e;
  return hipStreamUpdateCaptureDependencies(s, &node, 1, hipStreamSetCaptureDependencies);
}

struct Fwd {
  hipStream_t s = nullptr;
  bool bf = false;
  int M = 0, D = 0, NH = 0;
  float cap = 0.0f;
  int causal = 1;            // ATT_TEXT: merged causal + padding mask (enable_causal_atten)
  bool xs_f32 = false;       // bf16 GEMMs over an fp32 residual stream (text tower; no folding)
  bool small_m = false;      // few rows (text tower): 64 x 64-tile GEMM, K split over the waves (gemm_bf16_small.hip)
  void* hb = nullptr;        // [M][D] LayerNorm / attention output
  void* big = nullptr;       // [M][max(3D, F)] q|k|v, FFN hidden
  float* st_part = nullptr;  // [D/128][M][2] partial row statistics (folded LayerNorm)
  float* ln_rs = nullptr;    // [M][2] (rstd, -mean*rstd)
  Profiler* pf = nullptr;
  int cls_all = -1;          // >= 0: every launch of this context counts in that class (the text tower)

  // profiled launch: records events around `fn` when vp_profile_enable() is active
  template <class Fn>
  hipError_t rec(int cls, double flops, double bytes, Fn&& fn) {
    if (cls_all >= 0) cls = cls_all;
    auto launch = [&]() {
      vp::g_last_kernel = nullptr;
      const hipError_t e = fn();
      if (pf && vp::g_last_kernel) pf->kfn[cls] = vp::g_last_kernel;
      return e;
    };
    if (!pf || pf->used >= pf->cap || !((pf->mask >> cls) & 1u)) return launch();
    const int i = pf->used++;
    hipError_t e = record_event(pf->ev[2 * i], s);
    if (e != hipSuccess) return e;
    e = launch();
    if (e != hipSuccess) return e;
    pf->cls[i] = cls; pf->flops[i] = flops; pf->bytes[i] = bytes;
    return record_event(pf->ev[2 * i + 1], s);
  }

  hipError_t gemm(int epi, const void* A, int K, const void* Wt, int N, void* o, int64_t ldo, const float* bias,
                  const void* resid, const float* pos, int pos_rows, const float* rowpad,
                  const float* lnc = nullptr) const {
    vp::EpiArgs ep;
    ep.out = o; ep.ldo = ldo; ep.bias = bias; ep.resid = resid; ep.ldr = ldo;
    ep.pos = pos; ep.pos_rows = pos_rows; ep.rowpad = rowpad;
    ep.ln_rs = ln_rs; ep.ln_c = lnc; ep.st_part = st_part; ep.st_rows = M;
    if (bf && small_m) {
      // the text tower's rows are padded to 64 only (clip_text_ws): the 256-row kernels cannot take
      // them, so an epilogue the small-M kernel lacks is an error here, not a fallback
      if (!vp::gemm_bf16_small_ok(epi, M, N, K, K, K)) return hipErrorNotSupported;
      return vp::gemm_bf16_small(epi, (const vp::bf16_t*)A, K, (const vp::bf16_t*)Wt, K, M, N, K, ep, s);
    }
    if (bf) return vp::gemm_bf16_auto(epi, (const vp::bf16_t*)A, K, (const vp::bf16_t*)Wt, K, M, N, K, ep, s);
    return vp::gemm_f32(epi, (const float*)A, K, (const float*)Wt, K, M, N, K, ep, s);
  }

  // (rstd, -mean*rstd) of the residual stream from the producers' partial statistics
  hipError_t finalize() {
    const double b = (double)M * (D / 128) * 8.0 + (double)M * 8.0;
    return rec(PC_LAYERNORM, 0.0, b, [&] { return vp::ln_stats_finalize(st_part, D / 128, M, ln_rs, s); });
  }

  // pre-LN transformer layers (layers.py:749-872) over num_seq contiguous sequences of S rows of
  // the residual stream xs (in place).  fold: LN1/LN2 folded into the q|k|v / ffn1 GEMMs, with
  // (rstd, -mean*rstd) of xs already in ln_rs on entry.  relu: ReLU FFN (text tower), else GELU.
  int run_stack(std::vector<LayerW>& layers, void* xs, int num_seq, int S, const float* pad, int F, int acls,
                int kind, bool fold, bool relu) {
    using namespace vp;
    const double dM = M, dD = D, dF = F, dE = bf ? 2.0 : 4.0;
    auto gbytes = [&](double K, double N, double outb, double resid) {  // algorithmic GEMM bytes
      return dM * K * dE + N * K * dE + dM * N * outb + dM * N * resid;
    };
    const double aflops = 4.0 * num_seq * (double)S * S * dD;
    const double abytes = dM * 3 * dD * dE + dM * dD * dE;
    const double ln_bytes = 2.0 * dM * dD * dE;
    const bool xbf = bf && !xs_f32;  // residual stream dtype
    const int epi_resid = xbf ? EPI_RESID_BF16 : EPI_RESID_F32;
    const int epi_resid_ffn = xbf ? EPI_RESID_FFN_BF16 : EPI_RESID_FFN;
    // temporal attention fused into the q|k|v projection (vp_kernels.h EPI_*_TATTN_LN): T = 16
    // frames (one 16-row MFMA block per sequence), dh = 64, no key paddings, max-free cap; the
    // unfused pair stays for every other temporal case (frame paddings, T != 16, other caps)
    const bool tattn = fold && xbf && kind == ATT_VIDEO && S == 16 && !pad && fast_cap(cap) && D == NH * 64 &&
                       !layers.empty() && layers[0].wqk && M % 256 == 0;
    for (size_t li = 0; li < layers.size(); ++li) {
      LayerW& lw = layers[li];
      const bool last = li + 1 == layers.size();
      // spatial layers: q|k|v in the row-blocked layout for the spatial attention kernel
      const bool sblk = fold && xbf && lw.wqkv_blk && kind == ATT_VIDEO && S == 256 && fast_cap(cap) && !tattn;
      if (tattn) {
        // P (normalised bf16 probabilities, 512 B per (sequence, head)) goes to `big`; O to hb
        vp::EpiArgs ep;
        ep.ln_rs = ln_rs; ep.cap = cap; ep.heads = NH;
        ep.cap_c1 = 2.0f * 1.4426950408889634f / cap;  // the same IEEE division the kernel did
        ep.cap_c2 = cap * 1.4426950408889634f;
        ep.out = big; ep.bias = lw.bqk; ep.ln_c = lw.cqk;
        VP_HIP(rec(PC_GEMM_QKV_TATTN, 2.0 * dM * dD * 2 * dD + 4.0 * num_seq * (double)S * S * dD,
                   gbytes(dD, 2 * dD, 0, 0) + dM * NH * 32.0, [&] {
          return gemm_bf16_w4(EPI_QK_TATTN_LN, (const bf16_t*)xs, D, (const bf16_t*)lw.wqk, D, M, 2 * D, D, ep, s); }));
        vp::EpiArgs ev;
        ev.ln_rs = ln_rs; ev.cap = cap; ev.heads = NH;
        ev.out = hb; ev.ldo = D; ev.resid = big;
        ev.bias = lw.bqkv + 2 * D; ev.ln_c = lw.cqkv + 2 * D;
        const bf16_t* wv = static_cast<const bf16_t*>(lw.wqkv) + (size_t)2 * D * D;
        VP_HIP(rec(PC_GEMM_QKV_TATTN, 2.0 * dM * dD * dD, gbytes(dD, dD, dE, 0) + dM * NH * 32.0, [&] {
          return gemm_bf16_w4(EPI_V_TATTN_LN, (const bf16_t*)xs, D, wv, D, M, D, D, ev, s); }));
      } else if (fold) {  // LN1 folded: A = the residual stream, (rstd, -mean*rstd) in ln_rs
        VP_HIP(rec(PC_GEMM_QKV, 2.0 * dM * dD * 3 * dD, gbytes(dD, 3 * dD, dE, 0), [&] {
          if (sblk) return gemm(EPI_BF16_LN_BLK, xs, D, lw.wqkv_blk, 3 * D, big, 3 * D, lw.bqkv_blk, nullptr, nullptr, 1,
                                nullptr, lw.cqkv_blk);
          return gemm(EPI_BF16_LN, xs, D, lw.wqkv, 3 * D, big, 3 * D, lw.bqkv, nullptr, nullptr, 1, nullptr,
                      lw.cqkv); }));
      } else {
        VP_HIP(rec(PC_LAYERNORM, 0.0, ln_bytes, [&] {
          return layernorm(xs, xbf, M, D, lw.ln1_g, lw.ln1_b, hb, bf, PERM_NONE, 1, 1, nullptr, s); }));
        VP_HIP(rec(PC_GEMM_QKV, 2.0 * dM * dD * 3 * dD, gbytes(dD, 3 * dD, dE, 0), [&] {
          return gemm(EPI_BF16, hb, D, lw.wqkv, 3 * D, big, 3 * D, lw.bqkv, nullptr, nullptr, 1, nullptr); }));
      }
      // fp32 sequences longer than 256 (the auxiliary encoder, long clips' temporal attention, large patch grids): the
      // MFMA kernel for 0 < cap <= 50, else the generic online-softmax one
      auto attention_f32_long = [&](int ns, int len, const float* kpad) {
        const hipError_t e = attention_f32_mfma((const float*)big, (float*)hb, ns, len, NH, cap, kpad, s);
        return e != hipErrorNotSupported ? e : attention_masked(big, hb, 0, ns, len, NH, cap, kpad, 0, s);
      };
      if (!tattn) VP_HIP(rec(acls, aflops, abytes, [&] {
        if (kind == ATT_TEXT) {
          if (bf && fast_cap(cap) && S > 16 && S <= 256)
            return attention_seq_bf16((const bf16_t*)big, (bf16_t*)hb, num_seq, S, NH, cap, pad, s, causal);
          return attention_masked(big, hb, bf, num_seq, S, NH, cap, pad, causal, s);
        }
        // the bf16 kernels' max-free softmax needs 0 < cap <= kMaxFastCap; cap <= 0 (no capping,
        // layers.py:586-589) or a larger cap runs the online-softmax kernel
        if (bf && !fast_cap(cap)) return attention_masked(big, hb, 1, num_seq, S, NH, cap, pad, 0, s);
        if (kind == ATT_LONG) {  // no masks (encoders.py:855); any T*N
          if (!bf) return attention_f32_long(num_seq, S, nullptr);
          if (S >= 256) return attention_long_bf16((const bf16_t*)big, (bf16_t*)hb, num_seq, S, NH, cap, s);
          if (S > 16) return attention_seq_bf16((const bf16_t*)big, (bf16_t*)hb, num_seq, S, NH, cap, nullptr, s);
          return attention_temporal_bf16((const bf16_t*)big, (bf16_t*)hb, num_seq, S, NH, cap, nullptr, s);
        }
        // 16 < S <= 256 (T > 16 frames, other patch grids) on the sequence-packed MFMA kernel; longer sequences
        // on the generic fp32-math kernel
        if (!bf) {
          if (S <= 256) return attention_f32((const float*)big, (float*)hb, num_seq, S, NH, cap, pad, s);
          return attention_f32_long(num_seq, S, pad);
        }
        if (S == 256) return attention_spatial_bf16((const bf16_t*)big, (bf16_t*)hb, num_seq, NH, cap, pad, s, sblk);
        if (S <= 16) return attention_temporal_bf16((const bf16_t*)big, (bf16_t*)hb, num_seq, S, NH, cap, pad, s);
        if (S <= 256) return attention_seq_bf16((const bf16_t*)big, (bf16_t*)hb, num_seq, S, NH, cap, pad, s);
        return attention_masked(big, hb, 1, num_seq, S, NH, cap, pad, 0, s); }));
      VP_HIP(rec(PC_GEMM_POST, 2.0 * dM * dD * dD, gbytes(dD, dD, dE, dE), [&] {
        return gemm(fold ? EPI_RESID_BF16_ST : epi_resid, hb, D, lw.wpost, D, xs, D, lw.bpost, xs, nullptr, 1,
                    nullptr); }));
      if (fold) {  // LN2 folded into ffn_layer1
        VP_HIP(finalize());
        VP_HIP(rec(PC_GEMM_FFN1, 2.0 * dM * dD * dF, gbytes(dD, dF, dE, 0), [&] {
          return gemm(lw.ffn_blk ? EPI_GELU_BF16_LN_BLK : EPI_GELU_BF16_LN, xs, D, lw.w1, F, big, F, lw.b1, nullptr,
                      nullptr, 1, pad, lw.c1); }));
      } else {
        VP_HIP(rec(PC_LAYERNORM, 0.0, ln_bytes, [&] {
          return layernorm(xs, xbf, M, D, lw.ln2_g, lw.ln2_b, hb, bf, PERM_NONE, 1, 1, nullptr, s); }));
        VP_HIP(rec(PC_GEMM_FFN1, 2.0 * dM * dD * dF, gbytes(dD, dF, dE, 0), [&] {
          return gemm(relu ? EPI_RELU_BF16 : EPI_GELU_BF16, hb, D, lw.w1, F, big, F, lw.b1, nullptr, nullptr, 1,
                      pad); }));
      }
      const bool st = fold && !last;  // the next layer's LN1 statistics
      const int epi_ffn2 = lw.ffn_blk && fold ? (st ? EPI_RESID_FFN_BF16_ST_BLK : EPI_RESID_FFN_BF16_BLK)
                                              : st ? EPI_RESID_FFN_BF16_ST : epi_resid_ffn;
      VP_HIP(rec(PC_GEMM_FFN2, 2.0 * dM * dF * dD, gbytes(dF, dD, dE, dE), [&] {
        return gemm(epi_ffn2, big, F, lw.w2, D, xs, D, lw.b2, xs, nullptr, 1, pad); }));
      if (st) VP_HIP(finalize());
    }
    return VP_OK;
  }
};

}  // namespace vpi
