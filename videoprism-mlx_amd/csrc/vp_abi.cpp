// C-ABI implementation (include/videoprism_hip.h): parameter intake in the reference's
// Flax layout, packing into kernel-ready device buffers, and the FactorizedEncoder
// forward schedule (encoders.py:411-580) over the HIP kernels.
#include "../../include/videoprism_hip.h"

#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdlib>
#include <cxxabi.h>
#include <cstdio>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "vp_kernels.h"

#include "vp_internal.h"

using namespace vpi;

namespace {

// the temporal positional table for T frames, [T][D]: temporal_pos_emb/emb_var itself when T ==
// pos_emb_t, else _interpolate_emb_1d (encoders.py:107-130: jax.image.resize 'bilinear', antialiased
// when shrinking), fp64 on the host
std::vector<float> temporal_table(const vp_handle* h, int T) {
  const int64_t D = h->cfg.model_dim;
  const int Tp = h->cfg.pos_emb_t;
  const std::vector<float>& e = h->temporal_pos_host;
  std::vector<float> dst((size_t)T * D);
  if (T == Tp) {
    std::memcpy(dst.data(), e.data(), (size_t)T * D * 4);
    return dst;
  }
  const auto w = resize_weights(Tp, T);
  for (int t = 0; t < T; ++t)
    for (int64_t d = 0; d < D; ++d) {
      double s = 0.0;
      for (int i = 0; i < Tp; ++i) s += w[(size_t)i * T + t] * e[(size_t)i * D + d];
      dst[(size_t)t * D + d] = (float)s;
    }
  return dst;
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
  if (!std::isfinite(cfg->atten_logit_cap)) return fail(VP_EINVAL, "atten_logit_cap must be finite");
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
  const std::string& px = h->prefix;
  {  // patch projection: kernel [kreal][D] -> [D][kpad]
    const auto& k = param_data(h, px + "patch_projection/linear/kernel");
    std::vector<float> t((size_t)D * h->kpad, 0.0f);
    for (int64_t i = 0; i < kreal; ++i)
      for (int64_t n = 0; n < D; ++n) t[(size_t)n * h->kpad + i] = k[(size_t)i * D + n];
    if ((rc = upload_mat(h, t, &h->wpatch))) return rc;
    if (is_bf16(h) && vp::video_patch_ok((int)P)) {  // the frames' chunk order (gemm_bf16_w4_video, vp_kernels.h)
      const int64_t cpr = vp::video_patch_cpr((int)P), kv = vp::video_patch_k((int)P);
      std::vector<float> tv((size_t)D * kv, 0.0f);
      for (int64_t py = 0; py < P; ++py)
        for (int64_t cr = 0; cr < cpr; ++cr) {
          const int64_t vo = std::min<int64_t>(8 * cr, 3 * P - 8);
          for (int64_t e = 0; e < 8; ++e) {
            const int64_t v = vo + e;
            if (cr == cpr - 1 && v < 8 * (cpr - 1)) continue;  // overlap with the row's previous chunk
            for (int64_t n = 0; n < D; ++n) tv[(size_t)n * kv + 64 * py + 8 * cr + e] = k[(size_t)(py * 3 * P + v) * D + n];
          }
        }
      if ((rc = upload_mat(h, tv, &h->wpatch_v))) return rc;
    }
    if ((rc = upload_f32(h, param_data(h, px + "patch_projection/linear/bias"), &h->bpatch))) return rc;
  }
  if ((rc = upload_f32(h, param_data(h, px + "spatial_pos_emb/emb_var"), &h->spatial_pos))) return rc;
  h->spatial_pos_host = param_data(h, px + "spatial_pos_emb/emb_var");
  {  // temporal positional tables for T = 1..kPrecomputedT in one buffer (encoders.py:543-553)
    h->temporal_pos_host = param_data(h, px + "temporal_pos_emb/emb_var");
    std::vector<float> tab;
    std::vector<size_t> off(kPrecomputedT + 1);
    for (int T = 1; T <= kPrecomputedT; ++T) {
      off[T] = tab.size();
      const std::vector<float> t = temporal_table(h, T);
      tab.insert(tab.end(), t.begin(), t.end());
    }
    float* dev = nullptr;
    if ((rc = upload_f32(h, tab, &dev))) return rc;
    for (int T = 1; T <= kPrecomputedT; ++T) h->temporal_pos[T] = dev + off[T];
  }
  const bool fold = is_bf16(h);
  if ((rc = pack_stack(h, px + "spatial_encoder/transformers_stack/x_layers/", c.num_spatial_layers, D, c.mlp_dim,
                       c.num_heads, fold, h->spatial, QKV_BLOCKED)))
    return rc;
  if ((rc = pack_stack(h, px + "temporal_encoder/transformers_stack/x_layers/", c.num_temporal_layers, D,
                       c.mlp_dim, c.num_heads, fold, h->temporal,
                       fold && c.model_dim == c.num_heads * 64 ? QKV_PER_HEAD : QKV_PLAIN)))
    return rc;
  std::vector<float> g(D);
  const char* lns[2] = {"spatial_ln", "temporal_ln"};
  for (int i = 0; i < 2; ++i) {
    const auto& sc = param_data(h, px + lns[i] + "/scale");
    for (int64_t d = 0; d < D; ++d) g[d] = sc[d] + 1.0f;
    float** gp = i == 0 ? &h->sln_g : &h->tln_g;
    float** bp = i == 0 ? &h->sln_b : &h->tln_b;
    if ((rc = upload_f32(h, g, gp)) || (rc = upload_f32(h, param_data(h, px + lns[i] + "/bias"), bp)))
      return rc;
  }
  h->host.clear();
  h->finalized = true;
  return VP_OK;
}

int vp_prepare_geometry(vp_handle* h, int64_t H, int64_t W) {
  if (!h) return fail(VP_EINVAL, "null handle");
  if (!h->finalized) return fail(VP_ESTATE, "vp_finalize has not been called");
  const vp_config& c = h->cfg;
  const int64_t P = c.patch_size, D = c.model_dim;
  if (H < 1 || W < 1 || H % P || W % P)
    return fail(VP_EINVAL, "Image height (" + std::to_string(H) + ") and width (" + std::to_string(W) +
                               ") should be multiples of patch_size (" + std::to_string(P) + ").");
  const int gm = (int)(H / P), gn = (int)(W / P);
  if ((gm == c.pos_emb_h && gn == c.pos_emb_w) || h->grid_pos.count({gm, gn})) return VP_OK;
  // _interpolate_emb_2d (encoders.py:133-165): separable jax.image.resize 'bilinear' (antialiased
  // when shrinking) of the [pos_h, pos_w, D] table, fp64 on the host
  const int ph = c.pos_emb_h, pw = c.pos_emb_w;
  const auto wh = resize_weights(ph, gm), ww = resize_weights(pw, gn);
  const auto& e = h->spatial_pos_host;
  std::vector<float> out((size_t)gm * gn * D);
  std::vector<double> acc(D);
  for (int i = 0; i < gm; ++i)
    for (int j = 0; j < gn; ++j) {
      std::fill(acc.begin(), acc.end(), 0.0);
      for (int a = 0; a < ph; ++a) {
        const double wa = wh[(size_t)a * gm + i];
        if (wa == 0.0) continue;
        for (int b = 0; b < pw; ++b) {
          const double w = wa * ww[(size_t)b * gn + j];
          if (w == 0.0) continue;
          const float* src = e.data() + ((size_t)a * pw + b) * D;
          for (int64_t d = 0; d < D; ++d) acc[d] += w * src[d];
        }
      }
      for (int64_t d = 0; d < D; ++d) out[((size_t)i * gn + j) * D + d] = (float)acc[d];
    }
  VP_HIP(hipSetDevice(h->device));
  float* dev = nullptr;
  int rc = upload_f32(h, out, &dev);
  if (rc) return rc;
  h->grid_pos[{gm, gn}] = dev;
  return VP_OK;
}

int vp_prepare_frames(vp_handle* h, int64_t T) {
  if (!h) return fail(VP_EINVAL, "null handle");
  if (!h->finalized) return fail(VP_ESTATE, "vp_finalize has not been called");
  if (T < 1 || T > (int64_t)1 << 20) return fail(VP_EINVAL, "T must be in [1, 2^20]");
  if (h->temporal_pos.count((int)T)) return VP_OK;
  VP_HIP(hipSetDevice(h->device));
  float* dev = nullptr;
  int rc = upload_f32(h, temporal_table(h, (int)T), &dev);
  if (rc) return rc;
  h->temporal_pos[(int)T] = dev;
  return VP_OK;
}

int vp_workspace_bytes(const vp_handle* h, int64_t B, int64_t T, int64_t H, int64_t W,
                       size_t* bytes) {
  if (!h || !bytes) return fail(VP_EINVAL, "null argument");
  int rc = check_geometry(h, B, T, H, W);
  if (rc) return rc;
  *bytes = ws_layout(h, chunk_of(h, B, T, H, W), T, H, W).total;
  return VP_OK;
}

}  // extern "C"

namespace {

// FactorizedEncoder.__call__ over one chunk of B clips (B <= chunk_clips: a workspace of about 4 GiB of
// FFN hidden activation); vp_forward below walks the batch chunk by chunk
int forward_chunk(vp_handle* h, const void* video, int in_dtype, int64_t B, int64_t T, int64_t H,
                  int64_t W, const float* frame_paddings, void* out, int out_dtype,
                  void* spatial_out, void* workspace, void* stream) {
  using namespace vp;
  int rc;
  const WsLayout L = ws_layout(h, B, T, H, W);

  VP_HIP(hipSetDevice(h->device));
  hipStream_t s = static_cast<hipStream_t>(stream);
  const vp_config& c = h->cfg;
  const bool bf = is_bf16(h);
  const int P_ = c.patch_size;
  const int Nsp = (int)((H / P_) * (W / P_));
  const int M = (int)(B * T * Nsp);  // tokens
  const int Mp = (int)padded_rows(h, M);  // GEMM rows
  const float* sp_pos = h->spatial_pos;
  if (Nsp != c.pos_emb_h * c.pos_emb_w || H / P_ != c.pos_emb_h) {  // encoders.py:497-512
    auto it = h->grid_pos.find({(int)(H / P_), (int)(W / P_)});
    if (it == h->grid_pos.end())
      return fail(VP_ESTATE, "patch grid differs from pos_emb_shape[1:]: call vp_prepare_geometry first");
    sp_pos = it->second;
  }
  const auto tp = h->temporal_pos.find((int)T);
  if (tp == h->temporal_pos.end())
    return fail(VP_ESTATE, "no temporal positional table for T = " + std::to_string(T) + ": call vp_prepare_frames first");
  const float* tpos = tp->second;
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
    if (Mp > M) {
      VP_HIP(hipMemsetAsync(pad_btn + M, 0, (size_t)(Mp - M) * 4, s));
      VP_HIP(hipMemsetAsync(pad_bnt + M, 0, (size_t)(Mp - M) * 4, s));
    }
    VP_HIP(expand_paddings(frame_paddings, (int)B, (int)T, Nsp, pad_btn, pad_bnt, s));
  }
  // bf16: LayerNorms inside the layers are folded into the consuming GEMMs (EPI_*_LN); the
  // residual-stream producers emit row statistics (EPI_*_ST) that ln_stats_finalize turns into
  // (rstd, -mean*rstd) per row
  Fwd f;
  f.s = s; f.bf = bf; f.M = Mp; f.D = D; f.NH = NH; f.cap = c.atten_logit_cap;
  f.hb = hb; f.big = big;
  f.st_part = reinterpret_cast<float*>(ws + L.st_part);
  f.ln_rs = reinterpret_cast<float*>(ws + L.ln_rs);
  f.pf = &h->prof;
  float* ln_rs = f.ln_rs;
  const int epi_pos = bf ? EPI_POS_BF16 : EPI_POS_F32;
  const char* ge = bf ? gemm_bf16_check(Mp, 3 * D, D, D, D) : gemm_f32_check(Mp, 3 * D, D, D, D);
  if (ge) return fail(VP_ENOTSUP, ge);
  const double dM = M, dD = D, dE = (double)es;
  auto gbytes = [&](double K, double N, double outb, double resid) {  // algorithmic GEMM bytes
    return dM * K * dE + N * K * dE + dM * N * outb + dM * N * resid;
  };

  // 1. tokenisation + patch projection + spatial pos-emb (encoders.py:436-514)
  const double kreal = (double)P_ * P_ * 3;
  const double in_es = in_dtype == VP_U8 ? 1 : in_dtype == VP_BF16 ? 2 : 4;
  const bool fold = bf && c.num_spatial_layers > 0;  // LN1 of spatial layer 0 folded
  // bf16 on a 16x16 patch grid: the patch embedding reads the frames themselves (no patch
  // tensor); f32 / uint8 frames are converted to bf16 frames first (the patchify kernels' per-value
  // conversion, so every input dtype gives bitwise the bf16 caller's result)
  // the fused path reads bf16 frames in 16-B chunks at 4-B granularity, and video_to_bf16 reads
  // float4 / uchar4: frames at a less aligned address (a sliced caller buffer) take patchify + GEMM
  const uintptr_t vmis = reinterpret_cast<uintptr_t>(video) & (in_dtype == VP_F32 ? 15 : 3);
  if (h->wpatch_v && H / P_ == 16 && W / P_ == 16 && Mp == M && vmis == 0) {
    const bf16_t* frames = static_cast<const bf16_t*>(video);
    if (in_dtype != VP_BF16) {
      VP_HIP(f.rec(PC_PATCHIFY, 0.0, dM * kreal * (in_es + dE), [&] {
        return video_to_bf16(video, in_dtype, static_cast<bf16_t*>(big), (int64_t)B * T * H * W * 3, s); }));
      frames = static_cast<const bf16_t*>(big);
    }
    EpiArgs ep;
    ep.out = x; ep.ldo = D; ep.bias = h->bpatch; ep.pos = sp_pos; ep.pos_rows = Nsp;
    ep.st_part = f.st_part; ep.st_rows = Mp;
    VP_HIP(f.rec(PC_GEMM_PATCH, 2.0 * dM * kreal * dD, gbytes(kreal, dD, dE, 0), [&] {
      return gemm_bf16_w4_video(fold ? EPI_POS_BF16_ST : EPI_POS_BF16, frames, P_, (const bf16_t*)h->wpatch_v, Mp, D,
                                ep, s); }));
  } else {
    if (Mp > M) VP_HIP(hipMemsetAsync(static_cast<char*>(big) + (size_t)M * h->kpad * es, 0,
                                      (size_t)(Mp - M) * h->kpad * es, s));
    VP_HIP(f.rec(PC_PATCHIFY, 0.0, dM * kreal * in_es + dM * h->kpad * dE, [&] {
      return patchify(video, in_dtype, big, bf, (int)(B * T), (int)H, (int)W, 3, P_, h->kpad, s); }));
    VP_HIP(f.rec(PC_GEMM_PATCH, 2.0 * dM * kreal * dD, gbytes(kreal, dD, dE, 0), [&] {
      return f.gemm(fold ? EPI_POS_BF16_ST : epi_pos, big, h->kpad, h->wpatch, D, x, D, h->bpatch, nullptr,
                    sp_pos, Nsp, nullptr); }));
  }
  const double ln_bytes = dM * dD * dE + dM * dD * dE;
  if (fold) VP_HIP(f.finalize());
  auto run_stack = [&](std::vector<LayerW>& layers, void* xs, int num_seq, int S, const float* pad) -> int {
    const int acls = num_seq == (int)(B * T) ? PC_ATTN_SPATIAL : PC_ATTN_TEMPORAL;
    return f.run_stack(layers, xs, num_seq, S, pad, F, acls, ATT_VIDEO, bf, false);
  };
  auto rec = [&](int cls, double flops, double bytes, auto&& fn) { return f.rec(cls, flops, bytes, fn); };
  // 2. spatial encoder over (b t) sequences of Nsp tokens
  if ((rc = run_stack(h->spatial, x, (int)(B * T), Nsp, pad_btn))) return rc;
  // 3. spatial_ln (+ optional spatial_features), transpose to (b n) t, + temporal pos-emb
  if (spatial_out)
    VP_HIP(rec(PC_LAYERNORM, 0.0, dM * dD * dE + dM * dD * (out_dtype == VP_BF16 ? 2 : 4), [&] {
      return layernorm(x, bf, M, D, h->sln_g, h->sln_b, spatial_out, out_dtype == VP_BF16, PERM_NONE, 1, 1, nullptr, s); }));
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

}  // namespace

extern "C" {

int vp_forward(vp_handle* h, const void* video, int in_dtype, int64_t B, int64_t T, int64_t H,
               int64_t W, const float* frame_paddings, void* out, int out_dtype,
               void* spatial_out, void* workspace, size_t ws_bytes, void* stream) {
  if (!h || !video || !out || !workspace) return fail(VP_EINVAL, "null argument");
  if (!h->finalized) return fail(VP_ESTATE, "vp_finalize has not been called");
  if ((in_dtype != VP_F32 && in_dtype != VP_BF16 && in_dtype != VP_U8) ||
      (out_dtype != VP_F32 && out_dtype != VP_BF16))
    return fail(VP_EINVAL, "bad dtype");
  int rc = check_geometry(h, B, T, H, W);
  if (rc) return rc;
  const int64_t Bc = chunk_of(h, B, T, H, W);
  const size_t need = ws_layout(h, Bc, T, H, W).total;
  if (ws_bytes < need) return fail(VP_EINVAL, "workspace too small: need " + std::to_string(need));
  // per-clip strides of the caller's buffers
  const int64_t P = h->cfg.patch_size, D = h->cfg.model_dim;
  const size_t in_clip = (size_t)(T * H * W * 3) * (in_dtype == VP_U8 ? 1 : in_dtype == VP_BF16 ? 2 : 4);
  const size_t out_clip = (size_t)(T * (H / P) * (W / P) * D) * (out_dtype == VP_BF16 ? 2 : 4);
  for (int64_t b0 = 0; b0 < B; b0 += Bc) {
    const int64_t nb = std::min(Bc, B - b0);
    rc = forward_chunk(h, static_cast<const char*>(video) + b0 * in_clip, in_dtype, nb, T, H, W,
                       frame_paddings ? frame_paddings + b0 * T : nullptr, static_cast<char*>(out) + b0 * out_clip,
                       out_dtype, spatial_out ? static_cast<char*>(spatial_out) + b0 * out_clip : nullptr,
                       workspace, stream);
    if (rc) return rc;
  }
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

int vp_profile_set_mask(vp_handle* h, uint32_t class_mask) {
  if (!h) return fail(VP_EINVAL, "null handle");
  h->prof.mask = class_mask;
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

int vp_profile_kernel_name(vp_handle* h, int cls, const char** name) {
  if (!h || cls < 0 || cls >= PC_COUNT || !name) return fail(VP_EINVAL, "bad argument");
  Profiler& p = h->prof;
  p.kname[cls].clear();
  if (p.kfn[cls]) {
    const char* raw = hipKernelNameRefByPtr(p.kfn[cls], nullptr);
    if (raw) {
      int st = 0;
      char* dm = abi::__cxa_demangle(raw, nullptr, nullptr, &st);
      p.kname[cls] = (st == 0 && dm) ? dm : raw;
      std::free(dm);
    }
  }
  *name = p.kname[cls].c_str();
  return VP_OK;
}

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
    const char* e = gemm_f32_check((int)M, (int)N, (int)K, lda, ldw);
    if (e) return fail(VP_EINVAL, e);
    VP_HIP(gemm_f32(epilogue, (const float*)A, lda, (const float*)W, ldw, (int)M, (int)N, (int)K, ep, s));
  } else {
    return fail(VP_EINVAL, "bad precision");
  }
  return VP_OK;
}

// Not in the public header: one named bf16 GEMM kernel (4: gemm_bf16_w4, 8: gemm_bf16) with any
// epilogue, for kernel A/B tests (tests/test_gpu_kernels.py) and tools/gemm_bench.py.
int vp_dev_gemm_kernel(int which, int epi, const void* A, const void* W, int64_t M, int64_t N,
                       int64_t K, void* out, const float* bias, const void* resid, const float* pos,
                       int64_t pos_rows, const float* rowpad, void* stream) {
  using namespace vp;
  const char* e = which == 1 ? nullptr : (which == 32 || which == 33) ? gemm_f32_check((int)M, (int)N, (int)K, K, K)
                                                                       : gemm_bf16_check((int)M, (int)N, (int)K, K, K);
  if (e) return fail(VP_EINVAL, e);
  EpiArgs ep;
  ep.out = out; ep.ldo = N; ep.bias = bias; ep.resid = resid; ep.ldr = N;
  ep.pos = pos; ep.pos_rows = (int)(pos_rows > 0 ? pos_rows : 1); ep.rowpad = rowpad;
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (which == 4)
    VP_HIP(gemm_bf16_w4(epi, (const bf16_t*)A, K, (const bf16_t*)W, K, (int)M, (int)N, (int)K, ep, s));
  else if (which == 8)
    VP_HIP(gemm_bf16(epi, (const bf16_t*)A, K, (const bf16_t*)W, K, (int)M, (int)N, (int)K, ep, s));
  else if (which == 1) {  // the small-M kernel (text tower)
    if (!gemm_bf16_small_ok(epi, (int)M, (int)N, (int)K, K, K))
      return fail(VP_EINVAL, "small-M GEMM: epilogue 0, 1, 2, 4, 5, 7 or 13 and K % 256 == 0");
    VP_HIP(gemm_bf16_small(epi, (const bf16_t*)A, K, (const bf16_t*)W, K, (int)M, (int)N, (int)K, ep, s));
  } else if (which == 32 || which == 33) {  // fp32: round 1's 16x16x4 kernel (32) / the 32x32x2 kernel (33)
    VP_HIP(gemm_f32(epi, (const float*)A, K, (const float*)W, K, (int)M, (int)N, (int)K, ep, s, which - 31));
  } else
    return fail(VP_EINVAL, "which must be 1, 4, 8, 32 or 33");
  return VP_OK;
}

// Not in the public header: the GEMM-folded LayerNorm pieces (tests/test_gpu_kernels.py).
// vp_dev_gemm_ln: EPI_BF16_LN / EPI_GELU_BF16_LN with (rstd, -mean*rstd) rows ln_rs and column
// sums ln_c, or EPI_*_ST writing partial row statistics to st_part ([N/128][M][2]); EPI_*_BLK: the FFN
// pair over the row-blocked hidden activation (vp_kernels.h).
int vp_dev_gemm_ln(int epi, const void* A, const void* W, int64_t M, int64_t N, int64_t K, void* out,
                   const float* bias, const void* resid, const float* pos, int64_t pos_rows,
                   const float* rowpad, const float* ln_rs, const float* ln_c, float* st_part,
                   void* stream) {
  using namespace vp;
  if (!((epi >= EPI_BF16_LN && epi <= EPI_POS_BF16_ST) || (epi >= EPI_GELU_BF16_LN_BLK && epi <= EPI_BF16_LN_BLK)))
    return fail(VP_EINVAL, "epilogue must be 8..12 or 16..19");
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

// Not in the public header: the spatial attention (S = 256) over q|k|v in the row-blocked layout of
// EPI_BF16_LN_BLK (tests: bitwise the row-major path).
int vp_dev_attention_spatial_blk(const void* qkv, void* o, int64_t num_seq, int64_t heads, float cap,
                                 const float* key_pad, void* stream) {
  using namespace vp;
  if (!qkv || !o || num_seq < 1 || heads < 1) return fail(VP_EINVAL, "bad argument");
  VP_HIP(attention_spatial_bf16((const bf16_t*)qkv, (bf16_t*)o, (int)num_seq, (int)heads, cap, key_pad,
                                static_cast<hipStream_t>(stream), true));
  return VP_OK;
}

// Not in the public header: the two launches of the fused temporal attention (EPI_QK_TATTN_LN,
// EPI_V_TATTN_LN; vp_kernels.h) for kernel-level tests (tests/test_gpu_kernels.py).  which = 0: A = x
// [M][K], W = the [q_h | k_h]-regrouped LN-folded rows [2K][K] -> P (512 B per (sequence, head));
// which = 1: W = the v rows [K][K], p = P -> O [M][K].  K = heads * 64, M % 256 == 0.
int vp_dev_gemm_tattn(int which, const void* A, const void* W, int64_t M, int64_t K, void* out, const float* bias,
                      const float* ln_rs, const float* ln_c, const void* p, int64_t heads, float cap, void* stream) {
  using namespace vp;
  if (which < 0 || which > 1 || !A || !W || !out || !bias || !ln_rs || !ln_c || (which == 1 && !p))
    return fail(VP_EINVAL, "bad argument");
  if (K != heads * 64 || M % 256 || !vpi::fast_cap(cap)) return fail(VP_EINVAL, "needs K = heads*64, M % 256, 0 < cap <= 50");
  const int64_t N = which == 0 ? 2 * K : K;
  const char* e = gemm_bf16_check((int)M, (int)N, (int)K, K, K);
  if (e) return fail(VP_EINVAL, e);
  EpiArgs ep;
  ep.out = out; ep.ldo = K; ep.bias = bias; ep.ln_rs = ln_rs; ep.ln_c = ln_c; ep.resid = p;
  ep.cap = cap; ep.heads = (int)heads;
  ep.cap_c1 = 2.0f * 1.4426950408889634f / cap;
  ep.cap_c2 = cap * 1.4426950408889634f;
  VP_HIP(gemm_bf16_w4(which == 0 ? EPI_QK_TATTN_LN : EPI_V_TATTN_LN, (const bf16_t*)A, K, (const bf16_t*)W, K, (int)M,
                      (int)N, (int)K, ep, static_cast<hipStream_t>(stream)));
  return VP_OK;
}

// Not in the public header: the fused patch embedding (gemm_bf16_w4_video, EPI_POS_BF16) for kernel
// tests: bf16 frames [frames][16P][16P][3], wv [N][video_patch_k(P)] in the frames' chunk order
// (vp_kernels.h), pos [256][N] fp32 -> out [frames*256][N] bf16.
int vp_dev_patch_embed(const void* video, int64_t frames, int64_t P, const void* wv, int64_t N, const float* bias,
                       const float* pos, void* out, void* stream) {
  using namespace vp;
  if (!video || !wv || !bias || !pos || !out || frames < 1 || N % 256) return fail(VP_EINVAL, "bad argument");
  if (!video_patch_ok((int)P)) return fail(VP_EINVAL, "fused patch embedding needs an even patch size, 4 <= P <= 21");
  EpiArgs ep;
  ep.out = out; ep.ldo = N; ep.bias = bias; ep.pos = pos; ep.pos_rows = 256;
  VP_HIP(gemm_bf16_w4_video(EPI_POS_BF16, (const bf16_t*)video, (int)P, (const bf16_t*)wv, (int)(frames * 256), (int)N,
                            ep, static_cast<hipStream_t>(stream)));
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
    if (!fast_cap(cap)) {  // the max-free kernels need 0 < cap <= kMaxFastCap: online softmax
      if (S < 1) return fail(VP_EINVAL, "bad S");
      VP_HIP(attention_masked(qkv, o, 1, (int)num_seq, (int)S, (int)heads, cap, key_pad, 0, s));
    } else if (S == 256)
      VP_HIP(attention_spatial_bf16((const bf16_t*)qkv, (bf16_t*)o, (int)num_seq, (int)heads, cap, key_pad, s));
    else if (S > 256 && !key_pad)  // the auxiliary encoder's kernel (any S; a partial last query block)
      VP_HIP(attention_long_bf16((const bf16_t*)qkv, (bf16_t*)o, (int)num_seq, (int)S, (int)heads, cap, s));
    else if (S > 256)  // key paddings beyond 256 keys: the forward's choice (run_stack), the generic kernel
      VP_HIP(attention_masked(qkv, o, 1, (int)num_seq, (int)S, (int)heads, cap, key_pad, 0, s));
    else if (S >= 1 && S <= 16)
      VP_HIP(attention_temporal_bf16((const bf16_t*)qkv, (bf16_t*)o, (int)num_seq, (int)S, (int)heads, cap, key_pad, s));
    else if (S > 16 && S < 256)
      VP_HIP(attention_seq_bf16((const bf16_t*)qkv, (bf16_t*)o, (int)num_seq, (int)S, (int)heads, cap, key_pad, s));
    else
      return fail(VP_EINVAL, "bad S");
  } else if (precision == VP_F32) {
    if (S < 1) return fail(VP_EINVAL, "bad S");
    if (S <= 256) {
      VP_HIP(attention_f32((const float*)qkv, (float*)o, (int)num_seq, (int)S, (int)heads, cap, key_pad, s));
    } else {  // the forward's choice for long sequences (run_stack): the MFMA kernel, else online softmax
      const hipError_t e = attention_f32_mfma((const float*)qkv, (float*)o, (int)num_seq, (int)S, (int)heads, cap,
                                              key_pad, s);
      if (e != hipErrorNotSupported) VP_HIP(e);
      else VP_HIP(attention_masked(qkv, o, 0, (int)num_seq, (int)S, (int)heads, cap, key_pad, 0, s));
    }
  } else {
    return fail(VP_EINVAL, "bad precision");
  }
  return VP_OK;
}

int vp_op_attention_masked(int precision, const void* qkv, void* o, int64_t num_seq, int64_t S,
                           int64_t heads, float cap, const float* key_pad, int causal, void* stream) {
  using namespace vp;
  if (!qkv || !o || num_seq < 1 || heads < 1 || S < 1) return fail(VP_EINVAL, "bad argument");
  if (precision != VP_F32 && precision != VP_BF16) return fail(VP_EINVAL, "bad precision");
  // the forward's choice (vp_internal.h run_stack, ATT_TEXT): bf16 16 < S <= 256 on the MFMA sequence kernel
  if (precision == VP_BF16 && fast_cap(cap) && S > 16 && S <= 256)
    VP_HIP(attention_seq_bf16((const bf16_t*)qkv, (bf16_t*)o, (int)num_seq, (int)S, (int)heads, cap, key_pad,
                              static_cast<hipStream_t>(stream), causal ? 1 : 0));
  else
    VP_HIP(attention_masked(qkv, o, precision == VP_BF16, (int)num_seq, (int)S, (int)heads, cap, key_pad, causal,
                            static_cast<hipStream_t>(stream)));
  return VP_OK;
}

int vp_op_similarity(const float* video_emb, const float* text_emb, int64_t B, int64_t Q, int64_t D,
                     float* out, void* stream) {
  if (!video_emb || !text_emb || !out || B < 1 || Q < 1 || D < 1) return fail(VP_EINVAL, "bad argument");
  VP_HIP(vp::similarity(video_emb, text_emb, (int)B, (int)Q, (int)D, out, static_cast<hipStream_t>(stream)));
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
  if (in_dtype != VP_F32 && in_dtype != VP_BF16 && in_dtype != VP_U8) return fail(VP_EINVAL, "bad dtype");
  VP_HIP(patchify(video, in_dtype, patches, out_dtype == VP_BF16, (int)BT, (int)H, (int)W,
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
