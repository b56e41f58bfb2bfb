// Fused GEMM epilogues shared by the bf16 GEMM kernels (gemm_bf16.hip, gemm_bf16_w4.hip).
//
// Every lane owns 4 consecutive output columns n..n+3 of one output row (operand-swapped
// MFMA), so each epilogue is one 8-byte (bf16) or 16-byte (fp32) store per row, and the
// residual / position reads are the same width.  Semantics (layers.py line refs):
//   EPI_BF16            out_bf16 = acc + bias                                   (:273-313)
//   EPI_GELU_BF16       out_bf16 = gelu(acc + bias) * keep                      (:370-400)
//   EPI_RESID_F32/_FFN  out_f32  = resid_f32 + (acc + bias) * keep              (:855, :425)
//   EPI_POS_F32         out_f32  = acc + bias + pos[row % pos_rows]     (encoders.py:505-514)
//   EPI_RESID_BF16/_FFN_BF16, EPI_POS_BF16: the same with a bf16 residual stream (fprop_dtype
//   bf16 keeps activations in bf16 between layers, models.py:301-302); fp32 math, one rounding.
// keep = 1 - rowpad[row] (padded tokens, layers.py:405-420) where the epilogue takes it.
#pragma once
#include "vp_common.h"
#include "vp_kernels.h"

namespace vp {

template <int EPI>
struct EpiTraits {
  static constexpr bool kGelu = EPI == EPI_GELU_BF16;
  static constexpr bool kResidF32 = EPI == EPI_RESID_F32 || EPI == EPI_RESID_FFN;
  static constexpr bool kResidBf16 = EPI == EPI_RESID_BF16 || EPI == EPI_RESID_FFN_BF16;
  static constexpr bool kPos = EPI == EPI_POS_F32 || EPI == EPI_POS_BF16;
  static constexpr bool kExtra = kResidF32 || kResidBf16 || kPos;
  static constexpr bool kKeep = kGelu || kResidF32 || kResidBf16;
  static constexpr bool kOutBf16 = !(EPI == EPI_RESID_F32 || EPI == EPI_RESID_FFN || EPI == EPI_POS_F32);
};

// A&S 7.1.26 erf (|err| <= 1.5e-7) folded into GELU: 0.5*(x + |x|*erf(|x|/sqrt2)).
__device__ __forceinline__ float gelu_fast(float x) {
  const float ax = fabsf(x);
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f * 0.70710678118654752f, ax, 1.0f));
  float p = fmaf(t, 1.061405429f, -1.453152027f);
  p = fmaf(t, p, 1.421413741f);
  p = fmaf(t, p, -0.284496736f);
  p = fmaf(t, p, 0.254829592f);
  p *= t;
  const float e = __builtin_amdgcn_exp2f(x * x * (-0.5f * 1.4426950408889634f));
  return 0.5f * fmaf(ax, fmaf(-p, e, 1.0f), x);
}

__device__ __forceinline__ float4 bf16x4_to_f32(uint2 u) {
  return make_float4(__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u),
                     __uint_as_float(u.y << 16), __uint_as_float(u.y & 0xffff0000u));
}

// residual or position term of row `row`, columns n..n+3
template <int EPI>
__device__ __forceinline__ float4 epi_extra(const EpiArgs& ep, int row, int n, int N) {
  using Tr = EpiTraits<EPI>;
  if constexpr (Tr::kResidF32) {
    return *reinterpret_cast<const float4*>(static_cast<const float*>(ep.resid) + (int64_t)row * ep.ldr + n);
  } else if constexpr (Tr::kResidBf16) {
    return bf16x4_to_f32(
        *reinterpret_cast<const uint2*>(static_cast<const bf16_t*>(ep.resid) + (int64_t)row * ep.ldr + n));
  } else if constexpr (Tr::kPos) {
    return *reinterpret_cast<const float4*>(ep.pos + (int64_t)(row % ep.pos_rows) * N + n);
  } else {
    return make_float4(0.f, 0.f, 0.f, 0.f);
  }
}

// v = acc + bias (4 columns); applies GELU / keep / extra and stores
template <int EPI>
__device__ __forceinline__ void epi_store(const EpiArgs& ep, int row, int n, float4 v, float keep,
                                          float4 extra) {
  using Tr = EpiTraits<EPI>;
  if constexpr (Tr::kGelu) {
    v.x = gelu_fast(v.x); v.y = gelu_fast(v.y); v.z = gelu_fast(v.z); v.w = gelu_fast(v.w);
  }
  if constexpr (Tr::kKeep) {
    v.x *= keep; v.y *= keep; v.z *= keep; v.w *= keep;
  }
  if constexpr (Tr::kExtra) {
    v.x += extra.x; v.y += extra.y; v.z += extra.z; v.w += extra.w;
  }
  if constexpr (Tr::kOutBf16) {
    *reinterpret_cast<uint2*>(static_cast<bf16_t*>(ep.out) + (int64_t)row * ep.ldo + n) =
        make_uint2(pack_bf16x2(v.x, v.y), pack_bf16x2(v.z, v.w));
  } else {
    *reinterpret_cast<float4*>(static_cast<float*>(ep.out) + (int64_t)row * ep.ldo + n) = v;
  }
}

}  // namespace vp
