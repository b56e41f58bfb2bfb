// A/B builds of the auxiliary (4096-token) attention kernel (videoprism-mlx_amd/csrc/
// attention_long_kernel.h) for the tools' diag library: var 0 = the product kernel, 1 = the
// polynomial numerator in scalar instead of packed fp32 (bitwise the same output), 2 = without the
// quadratic tier for small logits, 4 = the row sum one value at a time, 8 = without the linear tier
// (round 4's product kernel), 16 = the row sum on the MFMA, 32 = the row sum by v_dot2_f32_bf16,
// 64 = the LIN / QUAD tiers and the row sum in unpaired scalar fp32, 128 = the LIN tier packed, 256 = s_setprio 1
// for waves 4-7, 1024 = round 5's chunk loop (addresses per tile; the product unrolls over the LDS stages)
// (bits combine: 6 = round 3's kernel).
#include "attention_long_kernel.h"
#include "attention_long_pp.h"

extern "C" int vp_dev_attention_long_var(int var, const void* qkv, void* o, int64_t num_seq, int64_t S,
                                         int64_t heads, float cap, void* stream) {
  using namespace vp;
  hipStream_t s = static_cast<hipStream_t>(stream);
  hipError_t e = hipErrorInvalidValue;
  if (var == 0) e = launch_attn_long<0>((const bf16_t*)qkv, (bf16_t*)o, (int)num_seq, (int)S, (int)heads, cap, s);
  if (var == 1) e = launch_attn_long<1>((const bf16_t*)qkv, (bf16_t*)o, (int)num_seq, (int)S, (int)heads, cap, s);
  if (var == 2) e = launch_attn_long<2>((const bf16_t*)qkv, (bf16_t*)o, (int)num_seq, (int)S, (int)heads, cap, s);
  if (var == 4) e = launch_attn_long<4>((const bf16_t*)qkv, (bf16_t*)o, (int)num_seq, (int)S, (int)heads, cap, s);
  if (var == 6) e = launch_attn_long<6>((const bf16_t*)qkv, (bf16_t*)o, (int)num_seq, (int)S, (int)heads, cap, s);
  if (var == 8) e = launch_attn_long<8>((const bf16_t*)qkv, (bf16_t*)o, (int)num_seq, (int)S, (int)heads, cap, s);
  if (var == 16) e = launch_attn_long<16>((const bf16_t*)qkv, (bf16_t*)o, (int)num_seq, (int)S, (int)heads, cap, s);
  if (var == 32) e = launch_attn_long<32>((const bf16_t*)qkv, (bf16_t*)o, (int)num_seq, (int)S, (int)heads, cap, s);
  if (var == 64) e = launch_attn_long<64>((const bf16_t*)qkv, (bf16_t*)o, (int)num_seq, (int)S, (int)heads, cap, s);
  if (var == 80) e = launch_attn_long<80>((const bf16_t*)qkv, (bf16_t*)o, (int)num_seq, (int)S, (int)heads, cap, s);
  if (var == 96) e = launch_attn_long<96>((const bf16_t*)qkv, (bf16_t*)o, (int)num_seq, (int)S, (int)heads, cap, s);
  if (var == 128) e = launch_attn_long<128>((const bf16_t*)qkv, (bf16_t*)o, (int)num_seq, (int)S, (int)heads, cap, s);
  if (var == 256) e = launch_attn_long<256>((const bf16_t*)qkv, (bf16_t*)o, (int)num_seq, (int)S, (int)heads, cap, s);
  if (var == 384) e = launch_attn_long<384>((const bf16_t*)qkv, (bf16_t*)o, (int)num_seq, (int)S, (int)heads, cap, s);
  if (var == 1024) e = launch_attn_long<1024>((const bf16_t*)qkv, (bf16_t*)o, (int)num_seq, (int)S, (int)heads, cap, s);
  // 512 + bits: the two-waves-per-SIMD alternating kernel (attn_long_pp_kernel) with those VAR bits
  if (var == 512) e = launch_attn_long_pp<0>((const bf16_t*)qkv, (bf16_t*)o, (int)num_seq, (int)S, (int)heads, cap, s);
  if (var == 640) e = launch_attn_long_pp<128>((const bf16_t*)qkv, (bf16_t*)o, (int)num_seq, (int)S, (int)heads, cap, s);
  if (var == 768) e = launch_attn_long_pp<256>((const bf16_t*)qkv, (bf16_t*)o, (int)num_seq, (int)S, (int)heads, cap, s);
  if (var == 7) e = launch_attn_long<7>((const bf16_t*)qkv, (bf16_t*)o, (int)num_seq, (int)S, (int)heads, cap, s);
  return e == hipSuccess ? 0 : -1;
}
