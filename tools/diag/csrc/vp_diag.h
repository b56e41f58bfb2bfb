// Declarations of the experiment-only kernels of the tools' diag library (`make diag`).  None of
// them is part of the product library; DESIGN.md records why each was not kept.
#pragma once
#include "vp_kernels.h"

namespace vp {

// 8-wave form of the 4-wave kernel's pipeline (two 128x64 waves per SIMD, gemm_bf16_w8b.hip):
// EPI_BF16 / EPI_GELU_BF16_LN; diag 8 = no epilogue
hipError_t gemm_bf16_w8b(int epi, const bf16_t* A, int64_t lda, const bf16_t* W, int64_t ldw, int M, int N,
                         int K, const EpiArgs& ep, int diag, hipStream_t s);
// 4-wave, 256x128 tile, two accumulator sets: the epilogue of tile j runs under the MFMAs of tile j+1
// (gemm_bf16_ov.hip).  bf16-output epilogues, M % 256, N % 128, K % 64, K >= 704.
bool gemm_bf16_ov_ok(int epi, int M, int N, int K, int64_t lda, int64_t ldw);
hipError_t gemm_bf16_ov(int epi, const bf16_t* A, int64_t lda, const bf16_t* W, int64_t ldw, int M,
                        int N, int K, const EpiArgs& ep, hipStream_t s);
// ablation builds of the product 4-wave GEMM template (gemm_w4_abl.hip): abl 2 = no ds_reads in the
// K-loop, 4 = no staging loads after the prologue, 8 = no epilogue, EPI_BF16 (S3 when s3 != 0)
hipError_t gemm_bf16_w4_abl(int abl, int s3, const bf16_t* A, int64_t lda, const bf16_t* W, int64_t ldw, int M,
                            int N, int K, const EpiArgs& ep, hipStream_t s);
hipError_t gemm_bf16_w4_tattn_abl(int which, int abl, const bf16_t* A, const bf16_t* W, int M, int N, int K,
                                  const EpiArgs& ep, hipStream_t s);
// q|k|v projection (LN1 folded, EPI_BF16_LN arithmetic) + spatial attention (S = 256, dh = 64,
// D = 768, no key paddings) fused per (frame, head) (qkv_attention.hip); bitwise equal to
// gemm_bf16_w4(EPI_BF16_LN) followed by attention_spatial_bf16.
bool qkv_attention_spatial_ok(int frames, int heads, float cap);
hipError_t qkv_attention_spatial_bf16(const bf16_t* x, const float* ln_rs, const bf16_t* wqkv, const float* bias,
                                      const float* lnc, bf16_t* o, int frames, int heads, float cap,
                                      hipStream_t s);
hipError_t qkv_attention_spatial_diag(int diag, const bf16_t* x, const float* ln_rs, const bf16_t* wqkv,
                                      const float* bias, const float* lnc, bf16_t* o, int frames, int heads,
                                      float cap, hipStream_t s);

}  // namespace vp
