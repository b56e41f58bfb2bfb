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

// the product ffn_layer1 launch (EPI_GELU_BF16_LN_BLK) with ablation bits; out [M/16][N/32][16][32] bf16
int vp_dev_gemm_ffn1_abl(int abl, const void* A, const void* W, int64_t M, int64_t N, int64_t K, void* out,
                         const float* bias, const float* ln_rs, const float* ln_c, void* stream) {
  using namespace vp;
  EpiArgs ep;
  ep.out = out; ep.ldo = N; ep.bias = bias; ep.ln_rs = ln_rs; ep.ln_c = ln_c;
  VP_HIP(gemm_bf16_w4_ffn1_abl(abl, (const bf16_t*)A, (const bf16_t*)W, (int)M, (int)N, (int)K, ep,
                               static_cast<hipStream_t>(stream)));
  return VP_OK;
}

// the product ffn_layer2 launch with ablation bits: A [M/16][K/32][16][32] bf16 (row-blocked), out = resid
// [M][N] bf16 in place, st_part [N/128][M][2]
int vp_dev_gemm_ffn2_abl(int abl, const void* A, const void* W, int64_t M, int64_t N, int64_t K, void* out,
                         const float* bias, float* st_part, void* stream) {
  using namespace vp;
  EpiArgs ep;
  ep.out = out; ep.ldo = N; ep.bias = bias; ep.resid = out; ep.ldr = N; ep.st_part = st_part; ep.st_rows = M;
  VP_HIP(gemm_bf16_w4_ffn2_abl(abl, (const bf16_t*)A, (const bf16_t*)W, (int)M, (int)N, (int)K, ep,
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

// fp32 GEMM variants (gemm_f32_var.hip): out [M][N] fp32 = A [M][K] . W [N][K]^T + bias (GELU for epi 1)
int vp_dev_gemm_f32_var(int var, int abl, int epi, const float* A, const float* W, int64_t M, int64_t N, int64_t K,
                        float* out, const float* bias, void* stream) {
  using namespace vp;
  EpiArgs ep;
  ep.out = out; ep.ldo = N; ep.bias = bias;
  VP_HIP(gemm_f32_var(var, abl, epi, A, W, (int)M, (int)N, (int)K, ep, static_cast<hipStream_t>(stream)));
  return VP_OK;
}

}  // extern "C"
