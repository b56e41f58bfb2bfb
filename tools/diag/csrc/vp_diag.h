// Declarations of the experiment-only kernels of the tools' diag library (`make diag`).  None of
// them is part of the product library; DESIGN.md records why each was not kept.
#pragma once
#include "vp_kernels.h"

namespace vp {

// ablation builds of the product 4-wave GEMM template (gemm_w4_abl.hip): abl 2 = no ds_reads in the
// K-loop, 4 = no staging loads after the prologue, 8 = no epilogue, EPI_BF16 (S3 when s3 != 0)
hipError_t gemm_bf16_w4_abl(int abl, int s3, const bf16_t* A, int64_t lda, const bf16_t* W, int64_t ldw, int M,
                            int N, int K, const EpiArgs& ep, hipStream_t s);
// the product ffn_layer1 launch (EPI_GELU_BF16_LN_BLK, no padded rows, 2-stage) with ABL bits: 2 = no ds_reads,
// 4 = no staging loads, 8 = no epilogue (prices the LN fold + GELU against the K-loop)
hipError_t gemm_bf16_w4_ffn1_abl(int abl, const bf16_t* A, const bf16_t* W, int M, int N, int K, const EpiArgs& ep,
                                 hipStream_t s);
hipError_t gemm_bf16_w4_ffn2_abl(int abl, const bf16_t* A, const bf16_t* W, int M, int N, int K, const EpiArgs& ep,
                                 hipStream_t s);
hipError_t gemm_bf16_w4_tattn_abl(int which, int abl, const bf16_t* A, const bf16_t* W, int M, int N, int K,
                                  const EpiArgs& ep, hipStream_t s);

// fp32 GEMM variants (gemm_f32_var.hip): var 0 = the product schedule, 1 = mid-K-tile barrier; abl bits
// 2 = no LDS reads, 4 = no staging, 8 = no epilogue, 16 = no barrier; epi EPI_BF16 / EPI_GELU_BF16 (fp32 out)
hipError_t gemm_f32_var(int var, int abl, int epi, const float* A, const float* W, int M, int N, int K,
                        const EpiArgs& ep, hipStream_t s);

}  // namespace vp
