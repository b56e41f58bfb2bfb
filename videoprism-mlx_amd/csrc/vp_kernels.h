// Internal (C++) launch interface of the HIP kernels.  The public C-ABI lives in
// include/videoprism_hip.h and is implemented in vp_abi.cpp on top of these.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace vp {

typedef uint16_t bf16_t;

// host function of the kernel most recently launched by this thread through the launchers below
// (vp_profile_kernel_name names the kernel behind each profiled class, so bench.py can match the
// PMC traffic of exactly that kernel symbol)
extern thread_local const void* g_last_kernel;
#define VP_NOTE_KERNEL(fn) (::vp::g_last_kernel = reinterpret_cast<const void*>(fn))

enum Epilogue {
  EPI_BF16 = 0,       // out_bf16 = acc + bias                       (fused q|k|v projection)
  EPI_GELU_BF16 = 1,  // out_bf16 = gelu(acc + bias) * (1 - rowpad)  (ffn_layer1)
  EPI_RESID_F32 = 2,  // out_f32  = resid + (acc + bias) * (1 - rowpad)   (post, ffn_layer2)
  EPI_POS_F32 = 3,    // out_f32  = acc + bias + pos[m % pos_rows]   (patch_projection + pos emb)
  EPI_RESID_FFN = 4,  // = EPI_RESID_F32, separate kernel symbol for ffn_layer2 (profiling)
  // bf16 residual stream (bf16 GEMM only): same as 2 / 3 / 4 with bf16 resid and output
  EPI_RESID_BF16 = 5,
  EPI_POS_BF16 = 6,
  EPI_RESID_FFN_BF16 = 7,
  // LayerNorm folded into the consuming GEMM (bf16 path): A = the raw residual stream x,
  // W' = diag(1+scale) W, bias' = b + W.beta, and per row (rstd, -mean*rstd) from ln_rs:
  //   out = rstd * acc + (-mean*rstd) * c[n] + bias'[n],   c[n] = sum_k W'[n][k]
  EPI_BF16_LN = 8,       // as EPI_BF16   (q|k|v of LN1(x))
  EPI_GELU_BF16_LN = 9,  // as EPI_GELU   (ffn_layer1 of LN2(x))
  // residual-stream producers that also emit the row statistics of the bf16 values they
  // store: per 128-column partial p = (n / 128), st_part[p][row] = (sum, sum of squares about
  // the partial mean); ln_stats_finalize() combines them into ln_rs
  EPI_RESID_BF16_ST = 10,
  EPI_RESID_FFN_BF16_ST = 11,
  EPI_POS_BF16_ST = 12,
  // ReLU FFN of the text tower (encoders.py:743): out = relu(acc + bias) * (1 - rowpad);
  // bf16 out on the bf16 GEMM, fp32 out on the fp32 GEMM
  EPI_RELU_BF16 = 13,
  // temporal self-attention (T = 16 frames, dh = 64, no key paddings) fused into the LN1-folded
  // q|k|v projection of a temporal layer (layers.py:601-661 over sequences of 16 rows, which are
  // aligned 16-row blocks of the (b n) t row order): two launches over the same A = x2
  //  EPI_QK_TATTN_LN: W rows [q_h | k_h] per head (a 256-column tile = 2 heads); the epilogue
  //    rounds q, k to bf16 (as the reference's bf16 projections), forms the 16x16 logits of every
  //    (sequence, head) on MFMA, the capped softmax in fp32, and stores the normalised probabilities
  //    in bf16 -- P^T fragments, 512 B per (sequence, head) at out + ((seq * heads + h) * 256) --
  //    instead of q and k;
  //  EPI_V_TATTN_LN: W rows = the v projection; the epilogue rounds v to bf16 and stores
  //    O = P . V (P from `resid`, the first launch's output) in v's place, so the attention output
  //    [M][D] comes out of the GEMM and q|k|v never reach HBM.
  EPI_QK_TATTN_LN = 14,
  EPI_V_TATTN_LN = 15,
  // The FFN pair with the hidden activation h in a row-blocked layout [M/16][F/32][16][32] (4-wave
  // kernel, bf16): ffn_layer1's epilogue stores straight from the accumulator layout -- a lane's
  // 8 values of one row are 8 natural columns because W1's rows (and b', c) are permuted within each
  // 32-row group on the host (W-row 16h + 4g + i holds column 8g + 4h + i), and one store
  // instruction writes one whole 1 KiB block -- so no LDS transposition; ffn_layer2 stages its A
  // K-tiles from that layout.  Bitwise the row-major pair.
  EPI_GELU_BF16_LN_BLK = 16,       // ffn_layer1 (as EPI_GELU_BF16_LN), h blocked
  EPI_RESID_FFN_BF16_ST_BLK = 17,  // ffn_layer2 (as EPI_RESID_FFN_BF16_ST), A = blocked h
  EPI_RESID_FFN_BF16_BLK = 18,     // ffn_layer2 (as EPI_RESID_FFN_BF16), A = blocked h
  // the spatial layers' q|k|v projection (as EPI_BF16_LN) into the row-blocked layout [M/16][3D/32][16][32]
  // (Wqkv / b' / c rows permuted the same way, a separate copy), read by attention_spatial_bf16(blk)
  EPI_BF16_LN_BLK = 19,
};

struct EpiArgs {
  void* out = nullptr;
  int64_t ldo = 0;
  const float* bias = nullptr;    // [N]
  const void* resid = nullptr;    // EPI_RESID_*: fp32 or bf16 by epilogue (may alias out)
  int64_t ldr = 0;
  const float* pos = nullptr;     // EPI_POS_F32: [pos_rows][N]
  int pos_rows = 1;
  const float* rowpad = nullptr;  // optional [M], 1 = padded token
  const float* ln_rs = nullptr;   // EPI_*_LN: [M][2] (rstd, -mean*rstd)
  const float* ln_c = nullptr;    // EPI_*_LN: [N] column sums of W'
  float* st_part = nullptr;       // EPI_*_ST: [N/128][M][2] partial (sum, M2) of each row
  int64_t st_rows = 0;            // EPI_*_ST: M (partial stride)
  float cap = 0.0f;               // EPI_*_TATTN_LN: logit cap (0 < cap <= 50)
  // EPI_QK_TATTN_LN: 2 log2(e) / cap and cap log2(e), the capped-exp constants (host-computed: a
  // kernel argument lives in SGPRs, the in-kernel division's result in two VGPRs across the loop)
  float cap_c1 = 0.0f, cap_c2 = 0.0f;
  int heads = 0;                  // EPI_*_TATTN_LN: heads of the whole projection (P indexing)
};

// ---- bf16 MFMA GEMM (gemm_bf16.hip) ----
const char* gemm_bf16_check(int M, int N, int K, int64_t lda, int64_t ldw);
hipError_t gemm_bf16(int epi, const bf16_t* A, int64_t lda, const bf16_t* W, int64_t ldw, int M,
                     int N, int K, const EpiArgs& ep, hipStream_t s);

// small M (the text tower, gemm_bf16_small.hip): 64 x 64 tiles, K split over 4 waves; epilogues EPI_BF16,
// EPI_GELU_BF16, EPI_RELU_BF16, EPI_RESID_F32/_FFN, EPI_RESID_BF16/_FFN_BF16; M, N % 64 == 0, K % 256 == 0
bool gemm_bf16_small_ok(int epi, int M, int N, int K, int64_t lda, int64_t ldw);
hipError_t gemm_bf16_small(int epi, const bf16_t* A, int64_t lda, const bf16_t* W, int64_t ldw, int M, int N, int K,
                           const EpiArgs& ep, hipStream_t s);
// 4-wave (one wave per SIMD, 128x128 per wave, 16x16x32 MFMA, full-line buffer_load..lds
// staging) decomposition; needs N*ldw*2 < 4 GiB (32-bit buffer offsets); an A operand past that range
// runs as consecutive row ranges (gemm_bf16_w4.hip)
hipError_t gemm_bf16_w4(int epi, const bf16_t* A, int64_t lda, const bf16_t* W, int64_t ldw, int M,
                        int N, int K, const EpiArgs& ep, hipStream_t s);
// patch embedding straight from bf16 frames (no patch tensor): video [M/256 frames]
// [16P][16P][3] (a 16x16 patch grid, so one 256-row tile is one frame), 3 <= P <= 21, epi
// EPI_POS_BF16(_ST).  W [N][video_patch_k(P) = 64 P]: patch pixel row py is K-tile py, read as cpr =
// ceil(3P/8) chunks of 8 values at value offsets min(8 j, 3P - 8) in slots j < cpr; W holds the
// patch-kernel row (py, vo + e) at column 64 py + 8 j + e except where the last chunk overlaps its
// predecessor and in the slots j >= cpr (zeros; video_patch_w packs it)
inline int video_patch_cpr(int P) { return (3 * P + 7) / 8; }
inline int video_patch_k(int P) { return 64 * P; }
// patch sizes the fused path takes: a patch pixel row (3P values) fits one 64-wide K-tile, and P is
// even so every 16-B chunk starts 4-B aligned in the frame (byte offsets 6P px + 16 j and 6P - 16 for
// the overlapping last chunk; P = 18 is the models' size).  Odd P would put chunks at 2-B offsets:
// those grids take patchify + GEMM instead
inline bool video_patch_ok(int P) { return P >= 4 && P % 2 == 0 && 3 * P <= 64; }
hipError_t gemm_bf16_w4_video(int epi, const bf16_t* video, int P, const bf16_t* W, int M, int N, const EpiArgs& ep,
                              hipStream_t s);
// N-tile group size of the persistent tile order (gemm_bf16_w4.hip; shared by the diag kernels)
int w4_ngrp(int M, int N, int K, int grid);
// picks gemm_bf16_w4 or gemm_bf16 by epilogue and shape
hipError_t gemm_bf16_auto(int epi, const bf16_t* A, int64_t lda, const bf16_t* W, int64_t ldw, int M,
                          int N, int K, const EpiArgs& ep, hipStream_t s);

// ---- fp32 GEMM for fprop_dtype=float32 (gemm_f32.hip) ----
const char* gemm_f32_check(int M, int N, int K, int64_t lda, int64_t ldw);
// version 2 (default): the 32x32x2 kernel; 1: round 1's 16x16x4 kernel (A/B through vp_dev_gemm_kernel)
hipError_t gemm_f32(int epi, const float* A, int64_t lda, const float* W, int64_t ldw, int M,
                    int N, int K, const EpiArgs& ep, hipStream_t s, int version = 2);

// ---- attention (attention.hip) ----
// qkv: rows of [q(D) | k(D) | v(D)], row r = seq * S + s; q pre-scaled by dh^-0.5.
// o: rows of D = heads*64.  key_pad: optional [num_seq * S] (1 = padded key).
// blk: qkv in the row-blocked layout of EPI_BF16_LN_BLK ([M/16][3D/32][16][32])
hipError_t attention_spatial_bf16(const bf16_t* qkv, bf16_t* o, int num_seq, int heads,
                                  float cap, const float* key_pad, hipStream_t s, bool blk = false);
// 16 < S <= 256 (temporal attention of clips longer than 16 frames, other patch grids, the text tower with
// causal = 1), key paddings optional (attention.hip)
hipError_t attention_seq_bf16(const bf16_t* qkv, bf16_t* o, int num_seq, int S, int heads, float cap,
                              const float* key_pad, hipStream_t s, int causal = 0);
hipError_t attention_temporal_bf16(const bf16_t* qkv, bf16_t* o, int num_seq, int S, int heads,
                                   float cap, const float* key_pad, hipStream_t s);
// fp32, S <= 256: S >= 128 with 0 < cap <= 50 on the MFMA (attention_f32_mfma), else the generic kernel
hipError_t attention_f32(const float* qkv, float* o, int num_seq, int S, int heads, float cap,
                         const float* key_pad, hipStream_t s);
// fp32 on v_mfma_f32_32x32x2f32, any S, no causal mask: hipErrorNotSupported unless 0 < cap <= 50 (the
// max-free softmax); the callers then take the generic online-softmax kernels
hipError_t attention_f32_mfma(const float* qkv, float* o, int num_seq, int S, int heads, float cap,
                              const float* key_pad, hipStream_t s);

// ---- elementwise / normalisation (elementwise.hip) ----
enum RowPerm { PERM_NONE = 0, PERM_BTN_TO_BNT = 1, PERM_BNT_TO_BTN = 2 };
// video [BT, H, W, C] (in_dtype 0 f32, 1 bf16, 2 uint8 normalised /255) -> patches [BT*np, kpad]
// (bf16 or f32), zero-padded K.
hipError_t patchify(const void* video, int in_dtype, void* patches, int out_is_bf16, int BT,
                    int H, int W, int C, int P, int kpad, hipStream_t s);
// LayerNorm over D of fp32 or bf16 rows; gamma already holds (1 + scale).  Output row r goes
// to row perm(r); `add` (optional, fp32 [add_rows][D]) is added by the *output* row's t index.
// out_rs (optional): (rstd, -mean*rstd) of each stored output row (as ln_rs above), by
// output row index
hipError_t layernorm(const void* x, int in_is_bf16, int rows, int D, const float* gamma,
                     const float* beta, void* out, int out_is_bf16, int perm, int T, int Nsp,
                     const float* add, hipStream_t s, float* out_rs = nullptr);
// f32 (in_dtype 0) / uint8 (2, normalised /255) frames -> bf16 frames, n values, the patchify kernels'
// per-value conversion (for the fused patch embedding)
hipError_t video_to_bf16(const void* video, int in_dtype, bf16_t* out, int64_t n, hipStream_t s);
// fp32 -> bf16 cast (weights are pre-packed on the host; this is for activations)
hipError_t cast_f32_bf16(const float* x, bf16_t* y, int64_t n, hipStream_t s);
// per-token padding vector expansion: frame_pad [B*T] -> token pads in both orders
hipError_t expand_paddings(const float* frame_pad, int B, int T, int Nsp, float* pad_btn,
                           float* pad_bnt, hipStream_t s);

// (rstd, -mean*rstd) of every row from the P partial (sum, M2) pairs of 128 columns each
// (Chan's combination), D = 128 * P, LayerNorm eps 1e-6 (layers.py:240-243)
hipError_t ln_stats_finalize(const float* st_part, int P, int64_t M, float* ln_rs, hipStream_t s);
// same statistics straight from bf16 rows [M][D] (two-pass), for tests and the op API
hipError_t ln_row_stats(const bf16_t* x, int64_t M, int D, float* ln_rs, hipStream_t s);

// ---- LvT video-text path (attention_long.hip, clip_kernels.hip) ----
// auxiliary-encoder self-attention over S = T*N tokens (S % 256 == 0), capped, no masks
hipError_t attention_long_bf16(const bf16_t* qkv, bf16_t* o, int num_seq, int S, int heads, float cap,
                               hipStream_t s);
// generic fp32-math attention (any S, dh 64) with key paddings and the causal merge of
// layers.py:111-179; qkv / o in bf16 (in_is_bf16) or fp32
hipError_t attention_masked(const void* qkv, void* o, int in_is_bf16, int num_seq, int S, int heads,
                            float cap, const float* key_pad, int causal, hipStream_t s);
// contrastive pooler: logits[g][h][s] = x[g*S+s] . U[h]; then softmax per (g,h) and
// z[g][h][:] = sum_s p x (zpart scratch: [G][pool_chunks(S)][H][D], stats [G*H][2])
// (bf16 x with Ut = [32][D] bf16 (U_hi | U_lo | 0) and S % 32 == 0: MFMA kernel)
hipError_t pool_logits(const void* x, int in_bf16, int64_t rows, int S, int D, const float* U, const bf16_t* Ut,
                       int H, float* logits, hipStream_t s);
hipError_t pool_softmax_wsum(const void* x, int in_bf16, int G, int S, int D, int H, const float* logits,
                             float* stats, float* zpart, float* z, hipStream_t s);
int pool_chunks(int S);
// out[b][m][n] = A[b][m][:] . Wt[b][:][n] + bias[b][n] (fp32, small M), batch strides sA/sW/sB/sO
hipError_t small_gemm(const float* A, int64_t lda, int64_t sA, const float* Wt, int64_t sW, const float* bias,
                      int64_t sB, float* out, int64_t ldo, int64_t sO, int M, int N, int K, int batch,
                      hipStream_t s);
hipError_t small_gemm_splitk(const float* A, int64_t lda, const float* Wt, const float* bias, float* out, int64_t ldo,
                             int M, int N, int K, int splits, float* part, hipStream_t s);
// rows r of x (stride elements apart): optional LayerNorm (gamma = 1 + scale) then optional
// L2 normalisation, fp32 out [rows][D]
hipError_t ln_l2_rows(const void* x, int in_bf16, int64_t stride, int rows, int D, const float* gamma,
                      const float* beta, int do_l2, float* out, hipStream_t s);
// text tokens: out[q*(L+1)+t] = table[ids[q][t]]*scale + pos[t] (t < L), cls*scale (t = L);
// pad_out[q*(L+1)+t] = pad_in[q][t] (t < L), 0 (t = L)
hipError_t text_embed(const int32_t* ids, int Q, int L, const void* table, int table_bf16, int V, const float* cls,
                      const float* pos, float scale, int D, void* out, int out_bf16, const float* pad_in,
                      float* pad_out, hipStream_t s);
// out[i][j] = a[i] . b[j]
hipError_t similarity(const float* a, const float* b, int B, int Q, int D, float* out, hipStream_t s);

hipError_t pool_l2(const void* emb, int is_bf16, int B, int L, int D, float* out, hipStream_t s);

}  // namespace vp
