// Ablation builds of the product 4-wave GEMM (videoprism-mlx_amd/csrc/gemm_w4_kernel.h) for the
// tools' diag library only: the same template with parts of the pipeline switched off, to price
// them (tools/gemm_bench.py ablate).  Results are garbage.
#include "gemm_w4_kernel.h"
#include "vp_diag.h"

namespace vp {

hipError_t gemm_bf16_w4_abl(int abl, int s3, const bf16_t* A, int64_t lda, const bf16_t* W, int64_t ldw, int M,
                            int N, int K, const EpiArgs& ep, hipStream_t s) {
  if (K % BK || M % BM || N % BN) return hipErrorInvalidValue;
#define VP_ABL(S3, X) \
  case X: return launch_w4<EPI_BF16, false, S3, X>(A, lda, W, ldw, M, N, K, ep, s);
  if (s3) {
    switch (abl) { VP_ABL(true, 0) VP_ABL(true, 2) VP_ABL(true, 4) VP_ABL(true, 6) VP_ABL(true, 8) VP_ABL(true, 14) }
  } else {
    switch (abl) { VP_ABL(false, 0) VP_ABL(false, 2) VP_ABL(false, 4) VP_ABL(false, 6) VP_ABL(false, 8) VP_ABL(false, 14) }
  }
#undef VP_ABL
  return hipErrorInvalidValue;
}

hipError_t gemm_bf16_w4_ffn1_abl(int abl, const bf16_t* A, const bf16_t* W, int M, int N, int K, const EpiArgs& ep,
                                 hipStream_t s) {
  if (K % BK || M % BM || N % BN) return hipErrorInvalidValue;
  switch (abl) {
    case 0: return launch_w4<EPI_GELU_BF16_LN_BLK, true, false, 0>(A, K, W, K, M, N, K, ep, s);
    case 2: return launch_w4<EPI_GELU_BF16_LN_BLK, true, false, 2>(A, K, W, K, M, N, K, ep, s);
    case 4: return launch_w4<EPI_GELU_BF16_LN_BLK, true, false, 4>(A, K, W, K, M, N, K, ep, s);
    case 8: return launch_w4<EPI_GELU_BF16_LN_BLK, true, false, 8>(A, K, W, K, M, N, K, ep, s);
    case 14: return launch_w4<EPI_GELU_BF16_LN_BLK, true, false, 14>(A, K, W, K, M, N, K, ep, s);
  }
  return hipErrorInvalidValue;
}

// the product ffn_layer2 launch (EPI_RESID_FFN_BF16_ST_BLK: A = the row-blocked hidden, S3, residual + row
// statistics) with ABL bits as above
hipError_t gemm_bf16_w4_ffn2_abl(int abl, const bf16_t* A, const bf16_t* W, int M, int N, int K, const EpiArgs& ep,
                                 hipStream_t s) {
  if (K % BK || M % BM || N % BN || K < 2048) return hipErrorInvalidValue;
  switch (abl) {
    case 0: return launch_w4<EPI_RESID_FFN_BF16_ST_BLK, false, true, 0>(A, K, W, K, M, N, K, ep, s);
    case 2: return launch_w4<EPI_RESID_FFN_BF16_ST_BLK, false, true, 2>(A, K, W, K, M, N, K, ep, s);
    case 4: return launch_w4<EPI_RESID_FFN_BF16_ST_BLK, false, true, 4>(A, K, W, K, M, N, K, ep, s);
    case 8: return launch_w4<EPI_RESID_FFN_BF16_ST_BLK, false, true, 8>(A, K, W, K, M, N, K, ep, s);
    case 14: return launch_w4<EPI_RESID_FFN_BF16_ST_BLK, false, true, 14>(A, K, W, K, M, N, K, ep, s);
  }
  return hipErrorInvalidValue;
}

// the fused temporal attention launches (which 0: EPI_QK_TATTN_LN, 1: EPI_V_TATTN_LN) with ABL bits
// (8: no epilogue, prices it)
hipError_t gemm_bf16_w4_tattn_abl(int which, int abl, const bf16_t* A, const bf16_t* W, int M, int N, int K,
                                  const EpiArgs& ep, hipStream_t s) {
  if (K % BK || M % BM || N % BN) return hipErrorInvalidValue;
  if (which == 0 && abl == 0) return launch_w4<EPI_QK_TATTN_LN, false, true, 0>(A, K, W, K, M, N, K, ep, s);
  if (which == 1 && abl == 0) return launch_w4<EPI_V_TATTN_LN, false, true, 0>(A, K, W, K, M, N, K, ep, s);
  if (which == 0 && abl == 8) return launch_w4<EPI_QK_TATTN_LN, false, true, 8>(A, K, W, K, M, N, K, ep, s);
  if (which == 1 && abl == 8) return launch_w4<EPI_V_TATTN_LN, false, true, 8>(A, K, W, K, M, N, K, ep, s);
  return hipErrorInvalidValue;
}

}  // namespace vp
