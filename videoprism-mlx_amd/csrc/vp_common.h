// Shared device/host helpers for the VideoPrism MI355X (gfx950) kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace vp {

typedef uint16_t bf16_t;                                            // raw bf16 bits
typedef short bf16x4 __attribute__((ext_vector_type(4)));
typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

#define VP_LDS_PTR(p) ((__attribute__((address_space(3))) void*)(p))
#define VP_GLB_PTR(p) ((const __attribute__((address_space(1))) void*)(p))

__device__ __forceinline__ float bf2f(bf16_t v) {
  return __uint_as_float(((uint32_t)v) << 16);
}

// round-to-nearest-even f32 -> bf16 (inputs on this path are finite)
__device__ __forceinline__ bf16_t f2bf(float f) {
  uint32_t u = __float_as_uint(f);
  u += 0x7FFFu + ((u >> 16) & 1u);
  return (bf16_t)(u >> 16);
}

// two f32 -> packed bf16 (round to nearest even): one v_cvt_pk_bf16_f32 on gfx950
__device__ __forceinline__ uint32_t pack_bf16x2(float lo, float hi) {
  typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
  typedef float f32x2_v __attribute__((ext_vector_type(2)));
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2_v{lo, hi}, bf16x2_t));
}

// Exact-erf GELU (layers.py:31).  erff from the device libm.
__device__ __forceinline__ float gelu_erf(float x) {
  return 0.5f * x * (1.0f + erff(x * 0.70710678118654752f));
}

// nontemporal (streaming) stores of 8 / 16 bytes: outputs that the next kernel reads back from
// HBM anyway go past L2 instead of being written back from it later
typedef unsigned nt_u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned nt_u32x4 __attribute__((ext_vector_type(4)));
typedef float nt_f32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void st_nt(void* p, uint2 v) {
  __builtin_nontemporal_store(nt_u32x2{v.x, v.y}, reinterpret_cast<nt_u32x2*>(p));
}
__device__ __forceinline__ void st_nt(void* p, uint4 v) {
  __builtin_nontemporal_store(nt_u32x4{v.x, v.y, v.z, v.w}, reinterpret_cast<nt_u32x4*>(p));
}
__device__ __forceinline__ void st_nt(void* p, float4 v) {
  __builtin_nontemporal_store(nt_f32x4{v.x, v.y, v.z, v.w}, reinterpret_cast<nt_f32x4*>(p));
}

__device__ __forceinline__ int wave_id() {
  return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
}

__device__ __forceinline__ void wait_vmcnt0() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

}  // namespace vp
