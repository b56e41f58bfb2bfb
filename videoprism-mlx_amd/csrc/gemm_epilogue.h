// Fused GEMM epilogues shared by the bf16 GEMM kernels (gemm_bf16.hip, gemm_bf16_w4.hip).
//
// Every lane owns 4 consecutive output columns n..n+3 of one output row (operand-swapped
// MFMA), so each epilogue is one 8-byte (bf16) or 16-byte (fp32) store per row, and the
// residual / position reads are the same width.  Semantics (layers.py line refs):
//   EPI_BF16            out_bf16 = acc + bias                                   (:273-313)
//   EPI_GELU_BF16       out_bf16 = gelu(acc + bias) * keep                      (:370-400)
//   EPI_RELU_BF16       out_bf16 = relu(acc + bias) * keep   (text tower ffn_layer1, encoders.py:743)
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
  static constexpr bool kLn = EPI == EPI_BF16_LN || EPI == EPI_GELU_BF16_LN;
  static constexpr bool kStats = EPI == EPI_RESID_BF16_ST || EPI == EPI_RESID_FFN_BF16_ST || EPI == EPI_POS_BF16_ST ||
                                 EPI == EPI_RESID_FFN_BF16_ST_BLK;
  static constexpr bool kGelu = EPI == EPI_GELU_BF16 || EPI == EPI_GELU_BF16_LN || EPI == EPI_GELU_BF16_LN_BLK;
  static constexpr bool kResidF32 = EPI == EPI_RESID_F32 || EPI == EPI_RESID_FFN;
  static constexpr bool kResidBf16 = EPI == EPI_RESID_BF16 || EPI == EPI_RESID_FFN_BF16 ||
                                     EPI == EPI_RESID_BF16_ST || EPI == EPI_RESID_FFN_BF16_ST ||
                                     EPI == EPI_RESID_FFN_BF16_ST_BLK || EPI == EPI_RESID_FFN_BF16_BLK;
  // the FFN pair over the row-blocked hidden activation (vp_kernels.h EPI_*_BLK)
  static constexpr bool kBlkOut = EPI == EPI_GELU_BF16_LN_BLK || EPI == EPI_BF16_LN_BLK;
  static constexpr bool kABlk = EPI == EPI_RESID_FFN_BF16_ST_BLK || EPI == EPI_RESID_FFN_BF16_BLK;
  static constexpr bool kPos = EPI == EPI_POS_F32 || EPI == EPI_POS_BF16 || EPI == EPI_POS_BF16_ST;
  static constexpr bool kExtra = kResidF32 || kResidBf16 || kPos;
  // residual-stream producers (bf16 path): their A (the attention output / the FFN hidden activation)
  // is read once, so it is staged with nontemporal loads, and the residual stream they write in place
  // is stored with default-policy (cache-allocating) stores -- the next readers of the residual stream
  // (the LN-folded consumer GEMM, the next residual epilogue) then find it in the Infinity Cache, which
  // the once-read streams (q|k|v, attention output, hidden activation) no longer displace
  static constexpr bool kResidStream = EPI == EPI_RESID_BF16_ST || EPI == EPI_RESID_FFN_BF16_ST ||
                                       EPI == EPI_RESID_FFN_BF16_ST_BLK;
  static constexpr bool kRelu = EPI == EPI_RELU_BF16;
  static constexpr bool kKeep = kGelu || kRelu || kResidF32 || kResidBf16;
  static constexpr bool kOutBf16 = !(EPI == EPI_RESID_F32 || EPI == EPI_RESID_FFN || EPI == EPI_POS_F32);
  // fused temporal attention (EPI_QK_TATTN_LN / EPI_V_TATTN_LN): LN-fold values per tile as kLn,
  // custom epilogue in gemm_bf16_w4.hip
  static constexpr bool kQkAttn = EPI == EPI_QK_TATTN_LN;
  static constexpr bool kVAttn = EPI == EPI_V_TATTN_LN;
  static constexpr bool kLnVals = kLn || kQkAttn || kVAttn;
};

// GELU(x) = x * Phi(x) (exact-erf form, layers.py:31) in one transcendental:
//   gelu(x) = max(x, 0) - t * Phi(-t),   t = min(|x|, GELU_TMAX),
//   Phi(-t) = exp2(P(t)),  P = degree-6 fit of log2 Phi(-t) on [0, 5.3] (tools/fit_gelu.py log2).
// fp32 result vs x*Phi(x) in fp64: relative error <= 2.2e-5 where |gelu| > 1e-6, absolute
// <= 3.0e-6 (checked on [-30, 30] with fp32 Horner, tests/test_epilogue_math.py): 1 % of the bf16
// output's half-ulp (2^-9).  Per value pair: 2 min, 6 packed FMA, 2 exp2, 2 max, 1 packed FMA = 11
// VALU + 2 transcendental issues.  (Degree 7 on [0, 5.6], relative 5.7e-6, took one packed FMA more
// per pair: ffn_layer1 598.9 -> 588.1 us with degree 6, tools/gemm_bench.py; the A&S 7.1.26 form
// before it needed 13 + 4 issues.)
// The clamp and max(x, 0) are IEEE-754-2019 minimum / maximum (gfx950 v_minimum3_f32 /
// v_maximum3_f32, same issue cost as v_min / v_max): a NaN pre-activation stays NaN, as in the
// reference's x * Phi(x), instead of being absorbed by minNum / maxNum; +inf gives +inf.  -inf gives the
// clamp's value gelu(-5.3) = -3.1e-7 by design, where the reference's -inf * Phi(-inf) = -inf * 0 is
// NaN: matching it would cost a select per value in the hot epilogue for an input a finite bf16
// activation stream never produces (tests/test_epilogue_math.py pins the behaviour).
constexpr float GELU_TMAX = 5.3f;
#define VP_GELU_P6 2.7470525310491212e-05f
#define VP_GELU_P5 -0.000680534983985126f
#define VP_GELU_P4 0.007596395444124937f
#define VP_GELU_P3 -0.05224345251917839f
#define VP_GELU_P2 -0.46002063155174255f
#define VP_GELU_P1 -1.1507104635238647f
#define VP_GELU_P0 -1.0000278949737549f

__device__ __forceinline__ float gelu_fast(float x) {
  const float t = __builtin_elementwise_minimum(__builtin_fabsf(x), GELU_TMAX);
  float p = fmaf(t, VP_GELU_P6, VP_GELU_P5);
  p = fmaf(t, p, VP_GELU_P4);
  p = fmaf(t, p, VP_GELU_P3);
  p = fmaf(t, p, VP_GELU_P2);
  p = fmaf(t, p, VP_GELU_P1);
  p = fmaf(t, p, VP_GELU_P0);
  return fmaf(-t, __builtin_amdgcn_exp2f(p), __builtin_elementwise_maximum(x, 0.0f));
}

// The same operation sequence on two values with packed fp32 math (v_pk_fma_f32):
// bit-identical to two gelu_fast calls, fewer VALU issue slots.
typedef float f32x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f32x2_t gelu_fast2(f32x2_t x) {
  const f32x2_t t = {__builtin_elementwise_minimum(__builtin_fabsf(x.x), GELU_TMAX),
                     __builtin_elementwise_minimum(__builtin_fabsf(x.y), GELU_TMAX)};
  f32x2_t p = __builtin_elementwise_fma(t, f32x2_t(VP_GELU_P6), f32x2_t(VP_GELU_P5));
  p = __builtin_elementwise_fma(t, p, f32x2_t(VP_GELU_P4));
  p = __builtin_elementwise_fma(t, p, f32x2_t(VP_GELU_P3));
  p = __builtin_elementwise_fma(t, p, f32x2_t(VP_GELU_P2));
  p = __builtin_elementwise_fma(t, p, f32x2_t(VP_GELU_P1));
  p = __builtin_elementwise_fma(t, p, f32x2_t(VP_GELU_P0));
  const f32x2_t e = {__builtin_amdgcn_exp2f(p.x), __builtin_amdgcn_exp2f(p.y)};
  const f32x2_t m = {__builtin_elementwise_maximum(x.x, 0.0f), __builtin_elementwise_maximum(x.y, 0.0f)};
  return __builtin_elementwise_fma(-t, e, m);
}

__device__ __forceinline__ float4 gelu4(float4 v) {
  const f32x2_t a = gelu_fast2(f32x2_t{v.x, v.y});
  const f32x2_t b = gelu_fast2(f32x2_t{v.z, v.w});
  return make_float4(a.x, a.y, b.x, b.y);
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
  if constexpr (Tr::kGelu) v = gelu4(v);
  if constexpr (Tr::kRelu) v = make_float4(relu_nan(v.x), relu_nan(v.y), relu_nan(v.z), relu_nan(v.w));
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

// ---- 8-column forms: a lane owns columns n..n+7 of one row (LDS-transposed epilogue) ----
struct F8 {
  float4 lo, hi;
};

template <int EPI>
__device__ __forceinline__ F8 epi_extra8(const EpiArgs& ep, int row, int n, int N) {
  using Tr = EpiTraits<EPI>;
  F8 e;
  if constexpr (Tr::kResidF32) {
    const float* r = static_cast<const float*>(ep.resid) + (int64_t)row * ep.ldr + n;
    e.lo = *reinterpret_cast<const float4*>(r);
    e.hi = *reinterpret_cast<const float4*>(r + 4);
  } else if constexpr (Tr::kResidBf16) {
    const uint4 u = *reinterpret_cast<const uint4*>(static_cast<const bf16_t*>(ep.resid) + (int64_t)row * ep.ldr + n);
    e.lo = bf16x4_to_f32(make_uint2(u.x, u.y));
    e.hi = bf16x4_to_f32(make_uint2(u.z, u.w));
  } else if constexpr (Tr::kPos) {
    const float* p = ep.pos + (int64_t)(row % ep.pos_rows) * N + n;
    e.lo = *reinterpret_cast<const float4*>(p);
    e.hi = *reinterpret_cast<const float4*>(p + 4);
  } else {
    e.lo = e.hi = make_float4(0.f, 0.f, 0.f, 0.f);
  }
  return e;
}

__device__ __forceinline__ float4 epi_math4(float4 v, float keep, float4 extra, bool gelu, bool kp, bool ex,
                                           bool relu = false) {
  if (gelu) v = gelu4(v);
  if (relu) v = make_float4(relu_nan(v.x), relu_nan(v.y), relu_nan(v.z), relu_nan(v.w));
  if (kp) { v.x *= keep; v.y *= keep; v.z *= keep; v.w *= keep; }
  if (ex) { v.x += extra.x; v.y += extra.y; v.z += extra.z; v.w += extra.w; }
  return v;
}

// v = acc + bias (8 columns); same math and single rounding as epi_store
typedef unsigned epi_u32x4 __attribute__((ext_vector_type(4)));
// NT: nontemporal output stores (global_store ... nt).  Measured on the w4 kernel at the
// encoder's shapes in isolation: qkv 432 -> 379 us, post 147 -> 130 us, ffn1 579 -> 502 us
// (tools/gemm_bench.py nt); inside the full forward within +-1 %.
// returns the stored bf16 values (packed) for the row-statistics epilogues
// KEEP = false: the launch has no padded rows (rowpad == nullptr), so the (1 - rowpad) factor is
// skipped -- bitwise the same result, one packed multiply per value pair less
template <int EPI, bool NT = true, bool KEEP = true>
__device__ __forceinline__ epi_u32x4 epi_store8(const EpiArgs& ep, int row, int n, F8 v, float keep, F8 extra) {
  using Tr = EpiTraits<EPI>;
  v.lo = epi_math4(v.lo, keep, extra.lo, Tr::kGelu, Tr::kKeep && KEEP, Tr::kExtra, Tr::kRelu);
  v.hi = epi_math4(v.hi, keep, extra.hi, Tr::kGelu, Tr::kKeep && KEEP, Tr::kExtra, Tr::kRelu);
  epi_u32x4 pk = {0u, 0u, 0u, 0u};
  if constexpr (Tr::kOutBf16) {
    pk = epi_u32x4{pack_bf16x2(v.lo.x, v.lo.y), pack_bf16x2(v.lo.z, v.lo.w), pack_bf16x2(v.hi.x, v.hi.y),
                   pack_bf16x2(v.hi.z, v.hi.w)};
    epi_u32x4* dst = reinterpret_cast<epi_u32x4*>(static_cast<bf16_t*>(ep.out) + (int64_t)row * ep.ldo + n);
    if constexpr (NT) __builtin_nontemporal_store(pk, dst);
    else *dst = pk;
  } else {
    typedef float f4_t __attribute__((ext_vector_type(4)));
    f4_t* o = reinterpret_cast<f4_t*>(static_cast<float*>(ep.out) + (int64_t)row * ep.ldo + n);
    const f4_t lo = {v.lo.x, v.lo.y, v.lo.z, v.lo.w}, hi = {v.hi.x, v.hi.y, v.hi.z, v.hi.w};
    if constexpr (NT) {
      __builtin_nontemporal_store(lo, o);
      __builtin_nontemporal_store(hi, o + 1);
    } else {
      o[0] = lo;
      o[1] = hi;
    }
  }
  return pk;
}

// sum over the 8 consecutive lanes (lane & ~7) of a wave; every lane gets the same bits
__device__ __forceinline__ float sum8_lanes(float x) {
  x += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0xB1, 0xF, 0xF, false));   // quad_perm 1,0,3,2
  x += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0x4E, 0xF, 0xF, false));   // quad_perm 2,3,0,1
  x += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0x141, 0xF, 0xF, false));  // row_half_mirror
  return x;
}

}  // namespace vp
