// Production instantiations and dispatch of the 4-wave bf16 GEMM (kernel template and design notes:
// gemm_w4_kernel.h).  Only production configurations are compiled here; the ablation builds live
// in the tools' diag library (tools/diag/csrc/gemm_w4_abl.hip).
#include "gemm_w4_kernel.h"

namespace vp {

// N-tile group size (see coords): the whole W when it is small (<= 2 MB) or when the GEMM streams
// A from HBM (K >= 2048: a group sweep would re-read A per group); else groups whose W rows take
// <= 2.5 MB (W > 4 MB: Base ffn_layer1 6 of 12 N-tiles, Large ffn_layer1 / q|k|v 4) or <= half of
// W (Base q|k|v, 3.5 MB: 3 of 9; forward 6.39 -> 6.29 ms/step, one box, alternating runs)
int w4_ngrp(int M, int N, int K, int grid) {
  const int tilesN = N / BN;
  const int64_t w_tile = (int64_t)BN * K * 2;  // W bytes per N-tile
  const int64_t w_all = (int64_t)tilesN * w_tile;
  if (w_all <= (2ll << 20) || K >= 2048 || (M / BM) % 8 || grid % 8) return tilesN;
  const int64_t budget = w_all > (4ll << 20) ? (5ll << 19) : w_all / 2;
  int g = tilesN;
  for (int d = tilesN; d >= 1; --d)
    if (tilesN % d == 0 && (int64_t)d * w_tile <= budget) { g = d; break; }
  return g;
}

hipError_t gemm_bf16_w4(int epi, const bf16_t* A, int64_t lda, const bf16_t* W, int64_t ldw, int M,
                        int N, int K, const EpiArgs& ep, hipStream_t s) {
  // byte offsets into A / W must fit the 32-bit buffer range
  if ((uint64_t)M * (uint64_t)lda * 2 >= 0xFFFFFFF0ull || (uint64_t)N * (uint64_t)ldw * 2 >= 0xFFFFFFF0ull)
    return hipErrorInvalidValue;
  if (K % BK || M % BM || N % BN) return hipErrorInvalidValue;
  // Every configuration stores its output nontemporally: +1.7 % on the whole forward vs plain stores
  // (same device, back-to-back: 947.8 vs 931.7 clips/s); plain stores on the residual-stream producers
  // (x in the Infinity Cache for the next GEMM) and on the q|k|v projection (for the spatial attention)
  // measured no faster (profiles/HISTORY.md).
  constexpr bool S3 = true, S2 = false;
  // the S3 residual epilogues peel their last K-tile (gemm_w4_kernel.h kEarly: K >= 2 BK); the
  // other bf16-residual epilogues take S3 only for K >= 2048
  if (K < 2 * BK && epi == EPI_RESID_BF16_ST) return hipErrorInvalidValue;
  switch (epi) {
    case EPI_BF16: return launch_w4<EPI_BF16, false, S2>(A, lda, W, ldw, M, N, K, ep, s);
    case EPI_GELU_BF16: return launch_w4<EPI_GELU_BF16, false, S2>(A, lda, W, ldw, M, N, K, ep, s);
    case EPI_RESID_F32: return launch_w4<EPI_RESID_F32, false, S2>(A, lda, W, ldw, M, N, K, ep, s);
    case EPI_POS_F32: return launch_w4<EPI_POS_F32, false, S2>(A, lda, W, ldw, M, N, K, ep, s);
    case EPI_RESID_FFN: return launch_w4<EPI_RESID_FFN, false, S2>(A, lda, W, ldw, M, N, K, ep, s);
    case EPI_RESID_BF16: return launch_w4<EPI_RESID_BF16, false, S2>(A, lda, W, ldw, M, N, K, ep, s);
    case EPI_POS_BF16: return launch_w4<EPI_POS_BF16, false, S2>(A, lda, W, ldw, M, N, K, ep, s);
    case EPI_RESID_FFN_BF16:
      if (K >= 2048) return launch_w4<EPI_RESID_FFN_BF16, false, S3>(A, lda, W, ldw, M, N, K, ep, s);
      return launch_w4<EPI_RESID_FFN_BF16, false, S2>(A, lda, W, ldw, M, N, K, ep, s);
    // q|k|v projection and post projection: S3 staging (forward, one box, alternating runs: qkv
    // 6.74-6.76 -> 6.50-6.54 ms/step, post 2.82-2.83 -> 2.69-2.71); ffn_layer1 measured no gain
    case EPI_BF16_LN: return launch_w4<EPI_BF16_LN, false, S3>(A, lda, W, ldw, M, N, K, ep, s);
    // ffn_layer1 launches without padded rows take the no-(1 - rowpad) build (bitwise equal; ffn1
    // 11.0-11.26 -> 10.9-11.0 ms/step)
    case EPI_GELU_BF16_LN:
      if (!ep.rowpad) return launch_w4<EPI_GELU_BF16_LN, true, S2>(A, lda, W, ldw, M, N, K, ep, s);
      return launch_w4<EPI_GELU_BF16_LN, false, S2>(A, lda, W, ldw, M, N, K, ep, s);
    case EPI_RESID_BF16_ST: return launch_w4<EPI_RESID_BF16_ST, false, S3>(A, lda, W, ldw, M, N, K, ep, s);
    case EPI_RESID_FFN_BF16_ST:
      if (K >= 2048) return launch_w4<EPI_RESID_FFN_BF16_ST, false, S3>(A, lda, W, ldw, M, N, K, ep, s);
      return launch_w4<EPI_RESID_FFN_BF16_ST, false, S2>(A, lda, W, ldw, M, N, K, ep, s);
    case EPI_POS_BF16_ST: return launch_w4<EPI_POS_BF16_ST, false, S2>(A, lda, W, ldw, M, N, K, ep, s);
    case EPI_RELU_BF16: return launch_w4<EPI_RELU_BF16, false, S2>(A, lda, W, ldw, M, N, K, ep, s);
    // the FFN pair over the row-blocked hidden activation (vp_kernels.h EPI_*_BLK): row-major A / W
    // for ffn_layer1, A blocked for ffn_layer2 (lda = K, K % 64 == 0)
    case EPI_GELU_BF16_LN_BLK:
      if (N % 32 || ldw != K) return hipErrorInvalidValue;
      if (!ep.rowpad) return launch_w4<EPI_GELU_BF16_LN_BLK, true, S2>(A, lda, W, ldw, M, N, K, ep, s);
      return launch_w4<EPI_GELU_BF16_LN_BLK, false, S2>(A, lda, W, ldw, M, N, K, ep, s);
    case EPI_BF16_LN_BLK:
      if (N % 32 || ldw != K) return hipErrorInvalidValue;
      return launch_w4<EPI_BF16_LN_BLK, true, S3>(A, lda, W, ldw, M, N, K, ep, s);
    case EPI_RESID_FFN_BF16_ST_BLK:
      if (lda != K) return hipErrorInvalidValue;
      if (K >= 2048) return launch_w4<EPI_RESID_FFN_BF16_ST_BLK, false, S3>(A, lda, W, ldw, M, N, K, ep, s);
      return launch_w4<EPI_RESID_FFN_BF16_ST_BLK, false, S2>(A, lda, W, ldw, M, N, K, ep, s);
    case EPI_RESID_FFN_BF16_BLK:
      if (lda != K) return hipErrorInvalidValue;
      if (K >= 2048) return launch_w4<EPI_RESID_FFN_BF16_BLK, false, S3>(A, lda, W, ldw, M, N, K, ep, s);
      return launch_w4<EPI_RESID_FFN_BF16_BLK, false, S2>(A, lda, W, ldw, M, N, K, ep, s);
    // temporal layers' q|k|v projection with the attention fused (T = 16): S3 as the q|k|v GEMM
    // (their last K-tile is peeled: K >= 2 BK)
    case EPI_QK_TATTN_LN:
      if (K < 2 * BK) return hipErrorInvalidValue;
      return launch_w4<EPI_QK_TATTN_LN, false, S3>(A, lda, W, ldw, M, N, K, ep, s);
    case EPI_V_TATTN_LN:
      if (K < 2 * BK) return hipErrorInvalidValue;
      return launch_w4<EPI_V_TATTN_LN, false, S3>(A, lda, W, ldw, M, N, K, ep, s);
  }
  return hipErrorInvalidValue;
}

hipError_t gemm_bf16_w4_video(int epi, const bf16_t* video, int P, const bf16_t* W, int M, int N, const EpiArgs& ep,
                              hipStream_t s) {
  if (!video_patch_ok(P) || M % BM || N % BN) return hipErrorInvalidValue;
  const int64_t lda = 16LL * P * 3;  // elements of one pixel row
  const int K = video_patch_k(P);
  if ((uint64_t)(M / BM) * 16 * P * lda * 2 >= 0xFFFFFFF0ull || (uint64_t)N * K * 2 >= 0xFFFFFFF0ull)
    return hipErrorInvalidValue;
  if (epi == EPI_POS_BF16_ST) return launch_w4<EPI_POS_BF16_ST, false, false, 0, true>(video, lda, W, K, M, N, K, ep, s);
  if (epi == EPI_POS_BF16) return launch_w4<EPI_POS_BF16, false, false, 0, true>(video, lda, W, K, M, N, K, ep, s);
  return hipErrorInvalidValue;
}

}  // namespace vp
