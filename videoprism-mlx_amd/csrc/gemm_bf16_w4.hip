// Production instantiations and dispatch of the 4-wave bf16 GEMM (kernel template and design notes:
// gemm_w4_kernel.h).  Only production configurations are compiled here; the ablation builds live
// in the tools' diag library (tools/diag/csrc/gemm_w4_abl.hip).
#include <algorithm>

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

namespace {

// one launch: the byte offsets into A / W must fit the 32-bit buffer range
hipError_t gemm_bf16_w4_launch(int epi, const bf16_t* A, int64_t lda, const bf16_t* W, int64_t ldw, int M,
                               int N, int K, const EpiArgs& ep, hipStream_t s) {
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

}  // namespace

// Rows are independent in every epilogue, so an A operand past the 32-bit buffer range (a long clip:
// the FFN hidden of one 16 x 288 x 288 clip is 4096 x 3072 x 2 B = 24 MiB, 4 GiB at ~2730 frames) runs
// as consecutive row ranges, each a launch whose row-indexed arguments start at its first row: out /
// resid by rows (the row-blocked layouts too: a 16-row block row is N elements), ln_rs / rowpad /
// st_part by rows (st_rows stays the full stride of the partial planes), the fused temporal
// attention's P by 16-row sequences, pos unchanged (ranges are multiples of pos_rows).  Each output
// element is still one tile's K-ordered sum: bitwise the single launch.
hipError_t gemm_bf16_w4(int epi, const bf16_t* A, int64_t lda, const bf16_t* W, int64_t ldw, int M,
                        int N, int K, const EpiArgs& ep, hipStream_t s) {
  const uint64_t rowb = (uint64_t)lda * 2;
  if (M <= 0 || (uint64_t)M * rowb < 0xFFFFFFF0ull) return gemm_bf16_w4_launch(epi, A, lda, W, ldw, M, N, K, ep, s);
  const bool f32_io = epi == EPI_RESID_F32 || epi == EPI_RESID_FFN || epi == EPI_POS_F32;  // fp32 out / resid
  const bool pos = epi == EPI_POS_F32 || epi == EPI_POS_BF16 || epi == EPI_POS_BF16_ST;
  int64_t unit = BM;  // row ranges: multiples of the tile (and of the positional table's period)
  if (pos) {
    int64_t a = BM, b = ep.pos_rows > 0 ? ep.pos_rows : 1;
    while (b) { const int64_t t = a % b; a = b; b = t; }
    unit = (int64_t)BM / a * (ep.pos_rows > 0 ? ep.pos_rows : 1);
  }
  const int64_t max_rows = (int64_t)(0xFFFFFFF0ull / rowb) / unit * unit;
  if (max_rows < unit) return hipErrorInvalidValue;
  for (int64_t r0 = 0; r0 < M; r0 += max_rows) {
    const int rows = (int)std::min<int64_t>(max_rows, M - r0);
    const int64_t pel = (r0 / 16) * ep.heads * 256;  // fused temporal P: 16 x 16 bf16 per (sequence, head)
    EpiArgs e = ep;
    if (epi == EPI_QK_TATTN_LN) e.out = static_cast<bf16_t*>(ep.out) + pel;
    else e.out = static_cast<char*>(ep.out) + r0 * ep.ldo * (f32_io ? 4 : 2);
    if (ep.resid) {
      if (epi == EPI_V_TATTN_LN) e.resid = static_cast<const bf16_t*>(ep.resid) + pel;
      else e.resid = static_cast<const char*>(ep.resid) + r0 * ep.ldr * (f32_io ? 4 : 2);
    }
    if (ep.rowpad) e.rowpad = ep.rowpad + r0;
    if (ep.ln_rs) e.ln_rs = ep.ln_rs + 2 * r0;
    if (ep.st_part) e.st_part = ep.st_part + 2 * r0;  // st_rows: the full stride of the partial planes
    const hipError_t err = gemm_bf16_w4_launch(epi, A + r0 * lda, lda, W, ldw, rows, N, K, e, s);
    if (err != hipSuccess) return err;
  }
  return hipSuccess;
}

hipError_t gemm_bf16_w4_video(int epi, const bf16_t* video, int P, const bf16_t* W, int M, int N, const EpiArgs& ep,
                              hipStream_t s) {
  if (!video_patch_ok(P) || M % BM || N % BN) return hipErrorInvalidValue;
  const int64_t lda = 16LL * P * 3;  // elements of one pixel row
  const int K = video_patch_k(P);
  if ((uint64_t)N * K * 2 >= 0xFFFFFFF0ull || (epi != EPI_POS_BF16_ST && epi != EPI_POS_BF16) || ep.pos_rows != 256)
    return hipErrorInvalidValue;
  // one frame = 16 P pixel rows = one 256-row tile; frames past the 32-bit buffer range run as consecutive
  // frame ranges (rows independent, the position table's period is the frame: bitwise one launch)
  const int64_t frame_elems = 16LL * P * lda;
  const int64_t max_frames = (int64_t)(0xFFFFFFF0ull / (uint64_t)(frame_elems * 2));
  const int64_t frames = M / BM;
  for (int64_t f0 = 0; f0 < frames; f0 += max_frames) {
    const int rows = (int)(std::min<int64_t>(max_frames, frames - f0) * BM);
    const int64_t r0 = f0 * BM;
    EpiArgs e = ep;
    e.out = static_cast<bf16_t*>(ep.out) + r0 * ep.ldo;
    if (ep.st_part) e.st_part = ep.st_part + 2 * r0;
    const bf16_t* v = video + f0 * frame_elems;
    const hipError_t err = epi == EPI_POS_BF16_ST
                               ? launch_w4<EPI_POS_BF16_ST, false, false, 0, true>(v, lda, W, K, rows, N, K, e, s)
                               : launch_w4<EPI_POS_BF16, false, false, 0, true>(v, lda, W, K, rows, N, K, e, s);
    if (err != hipSuccess) return err;
  }
  return hipSuccess;
}

}  // namespace vp
