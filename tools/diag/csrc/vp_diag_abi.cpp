// C entry points of the tools' diag library (`make diag` -> videoprism/libvideoprism_hip_diag.so,
// loaded only with VP_DIAG_LIB=1 by tools/): the experiment-only kernels and the ablation builds of
// the product 4-wave GEMM.  Not part of include/videoprism_hip.h.
#include "../../../videoprism-mlx_amd/csrc/vp_internal.h"
#include "vp_diag.h"

using vpi::fail;

extern "C" {

// ablation builds of the product 4-wave GEMM (EPI_BF16): abl 2 = no ds_reads, 4 = no staging loads,
// 8 = no epilogue (bits combine); s3 selects the three-A-buffer staging
int vp_dev_gemm_w4_abl(int abl, int s3, const void* A, const void* W, int64_t M, int64_t N, int64_t K, void* out,
                       const float* bias, void* stream) {
  using namespace vp;
  const char* e = gemm_bf16_check((int)M, (int)N, (int)K, K, K);
  if (e) return fail(VP_EINVAL, e);
  EpiArgs ep;
  ep.out = out; ep.ldo = N; ep.bias = bias;
  VP_HIP(gemm_bf16_w4_abl(abl, s3, (const bf16_t*)A, K, (const bf16_t*)W, K, (int)M, (int)N, (int)K, ep,
                          static_cast<hipStream_t>(stream)));
  return VP_OK;
}

// the fused temporal attention launches with ablation bits (vp_dev_gemm_tattn of the product ABI + abl)
int vp_dev_gemm_tattn_abl(int which, int abl, const void* A, const void* W, int64_t M, int64_t K, void* out,
                          const float* bias, const float* ln_rs, const float* ln_c, const void* p, int64_t heads,
                          float cap, void* stream) {
  using namespace vp;
  EpiArgs ep;
  ep.out = out; ep.ldo = K; ep.bias = bias; ep.ln_rs = ln_rs; ep.ln_c = ln_c; ep.resid = p;
  ep.cap = cap; ep.heads = (int)heads;
  ep.cap_c1 = 2.0f * 1.4426950408889634f / cap;
  ep.cap_c2 = cap * 1.4426950408889634f;
  VP_HIP(gemm_bf16_w4_tattn_abl(which, abl, (const bf16_t*)A, (const bf16_t*)W, (int)M, (int)(which == 0 ? 2 * K : K),
                                (int)K, ep, static_cast<hipStream_t>(stream)));
  return VP_OK;
}

// the overlapped-epilogue GEMM (gemm_bf16_ov.hip) with the plain bf16-output epilogues
int vp_dev_gemm_ov(int epi, const void* A, const void* W, int64_t M, int64_t N, int64_t K, void* out,
                   const float* bias, const void* resid, void* stream) {
  using namespace vp;
  if (!gemm_bf16_ov_ok(epi, (int)M, (int)N, (int)K, K, K))
    return fail(VP_EINVAL, "shape/epilogue not supported by gemm_bf16_ov");
  EpiArgs ep;
  ep.out = out; ep.ldo = N; ep.bias = bias; ep.resid = resid; ep.ldr = N;
  VP_HIP(gemm_bf16_ov(epi, (const bf16_t*)A, K, (const bf16_t*)W, K, (int)M, (int)N, (int)K, ep,
                      static_cast<hipStream_t>(stream)));
  return VP_OK;
}

// the 8-wave GEMM with the 4-wave pipeline (gemm_bf16_w8b.hip), EPI_BF16 / EPI_GELU_BF16_LN, for
// tools/ab_tests.py and tools/gemm_bench.py w8b (diag 8: no epilogue)
int vp_dev_gemm_w8b(int epi, int diag, const void* A, const void* W, int64_t M, int64_t N, int64_t K, void* out,
                    const float* bias, const float* rowpad, const float* ln_rs, const float* ln_c, void* stream) {
  using namespace vp;
  const char* e = gemm_bf16_check((int)M, (int)N, (int)K, K, K);
  if (e) return fail(VP_EINVAL, e);
  EpiArgs ep;
  ep.out = out; ep.ldo = N; ep.bias = bias; ep.rowpad = rowpad; ep.ln_rs = ln_rs; ep.ln_c = ln_c;
  VP_HIP(gemm_bf16_w8b(epi, (const bf16_t*)A, K, (const bf16_t*)W, K, (int)M, (int)N, (int)K, ep, diag,
                       static_cast<hipStream_t>(stream)));
  return VP_OK;
}

// the fused q|k|v projection + spatial attention kernel (an experiment that measured no faster than
// the unfused pair; tools/qa_bench.py checks it bitwise against vp_dev_gemm_ln(EPI_BF16_LN)
// + vp_op_attention)
int vp_dev_qkv_attention(const void* x, const float* ln_rs, const void* wqkv, const float* bias, const float* lnc,
                         void* out, int64_t frames, int64_t heads, float cap, void* stream) {
  using namespace vp;
  if (!qkv_attention_spatial_ok((int)frames, (int)heads, cap < -1000.f ? 50.f : cap))
    return fail(VP_EINVAL, "qkv_attention: needs heads*64 == 768, cap > 0 and frames*256 rows in range");
  if (cap < -1000.f) {  // ablation builds: cap = -1000 - diag (tools/qa_bench.py)
    VP_HIP(qkv_attention_spatial_diag((int)(-1000.f - cap), (const bf16_t*)x, ln_rs, (const bf16_t*)wqkv, bias, lnc,
                                      (bf16_t*)out, (int)frames, (int)heads, 50.f, static_cast<hipStream_t>(stream)));
    return VP_OK;
  }
  VP_HIP(qkv_attention_spatial_bf16((const bf16_t*)x, ln_rs, (const bf16_t*)wqkv, bias, lnc, (bf16_t*)out,
                                    (int)frames, (int)heads, cap, static_cast<hipStream_t>(stream)));
  return VP_OK;
}

}  // extern "C"
