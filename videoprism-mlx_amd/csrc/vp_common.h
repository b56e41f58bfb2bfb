// Shared device/host helpers for the VideoPrism MI355X (gfx950) kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <atomic>
#include <mutex>
#include <set>
#include <utility>

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

// Exact-erf GELU without the libm call, on a pair of values (the fp32 GEMM's epilogue): erfc(|z|) =
// t exp(-z^2 + P(t)), t = 1 / (1 + |z| / 2), P of degree 9 (the Chebyshev fit of Numerical Recipes' erfcc,
// relative error <= 1.2e-7), one Newton step on the reciprocal; Phi(x) = 1 - erfc / 2 (x >= 0) or erfc / 2.
// Branch-free (libm's erff runs several branches per wave), two transcendentals per value, the polynomial on
// packed FMAs.  Error vs fp64 on [-12, 12] (emulated, tools/gelu_erfc_accuracy.py): max 2.3e-7 / mean 5.9e-8 on
// [1, 4), the same band as a correctly rounded fp32 erf's (2.9e-7 / 6.6e-8); at the ffn_layer1 GEMM 5.19e-6 max /
// 1.950e-7 mean vs the libm form's 5.14e-6 / 1.943e-7 (profiles/r06/fp32_gemm_var.txt).
typedef float f32x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f32x2_t gelu_erfc_fit2(f32x2_t x) {
  const f32x2_t za = __builtin_elementwise_abs(x) * f32x2_t(0.70710678118654752f);
  const f32x2_t d = __builtin_elementwise_fma(f32x2_t(0.5f), za, f32x2_t(1.0f));
  f32x2_t t = f32x2_t{__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
  t = __builtin_elementwise_fma(t, __builtin_elementwise_fma(-d, t, f32x2_t(1.0f)), t);
  f32x2_t p = f32x2_t(0.17087277f);
  p = __builtin_elementwise_fma(p, t, f32x2_t(-0.82215223f));
  p = __builtin_elementwise_fma(p, t, f32x2_t(1.48851587f));
  p = __builtin_elementwise_fma(p, t, f32x2_t(-1.13520398f));
  p = __builtin_elementwise_fma(p, t, f32x2_t(0.27886807f));
  p = __builtin_elementwise_fma(p, t, f32x2_t(-0.18628806f));
  p = __builtin_elementwise_fma(p, t, f32x2_t(0.09678418f));
  p = __builtin_elementwise_fma(p, t, f32x2_t(0.37409196f));
  p = __builtin_elementwise_fma(p, t, f32x2_t(1.00002368f));
  p = __builtin_elementwise_fma(p, t, f32x2_t(-1.26551223f));
  const f32x2_t y = __builtin_elementwise_fma(-za, za, p) * f32x2_t(1.4426950408889634f);
  const f32x2_t hec = f32x2_t(0.5f) * t * f32x2_t{__builtin_amdgcn_exp2f(y.x), __builtin_amdgcn_exp2f(y.y)};
  const f32x2_t phi = f32x2_t{x.x >= 0.0f ? 1.0f - hec.x : hec.x, x.y >= 0.0f ? 1.0f - hec.y : hec.y};
  return x * phi;
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

// ---- capped-softmax numerators exp(cap * tanh(x / cap)) (layers.py:586-594, :650-654) ----
// exact form: tanh(y) = 1 - 2 / (exp(2y) + 1), three transcendentals, saturates correctly
__device__ __forceinline__ float capped_exp_exact(float x, float two_log2e_over_cap, float cap_log2e) {
  const float t = __builtin_amdgcn_exp2f(x * two_log2e_over_cap);
  const float r = __builtin_amdgcn_rcpf(t + 1.0f);
  return __builtin_amdgcn_exp2f(cap_log2e - 2.0f * cap_log2e * r);
}

// One transcendental where every logit of the wave's 32x32 tile has |x| <= 0.48 cap:
// cap*tanh(x/cap) = x*T((x/cap)^2), T(v) = tanh(sqrt v)/sqrt v fitted on v in [0, 0.48^2] by a
// cubic (relative error 4.5e-7, tools/fit_gelu.py fit_tanh), so the numerator is
// exp2(x * P(x^2)) with k_i = log2e t_i / cap^(2i) folded on the host (make_cap_poly); tiles
// holding a larger logit take the exact path (wave-uniform branch).
// QUAD tier (tiles whose logits all satisfy |x| <= 0.24 cap): T fitted by a quadratic on v in
// [0, 0.24^2] (relative error 3.5e-7, tools/fit_gelu.py fit_tanh(0.24, 2)), coefficients q0..q2.
// LIN tier (tiles whose logits all satisfy |x| <= 0.10 cap): T fitted by a line on v in [0, 0.10^2]
// (relative error 1.7e-6, tools/fit_gelu.py fit_tanh(0.10, 1): exponent error <= 1.2e-5, 0.3 % of a
// bf16 ulp of the numerator), coefficients l0, l1 -- three VALU operations per logit instead of four.
struct CapPoly {
  float k0, k1, k2, k3, x0;
  float q0, q1, q2, x1;
  float l0, l1, x2;
};

inline CapPoly make_cap_poly(float cap) {
  const double t[4] = {0.9999995827674866, -0.33327752351760864, 0.1321016252040863, -0.045063190162181854};
  const double u[3] = {0.9999996877028773, -0.33323595618512314, 0.12879159575308177};
  const double w[2] = {0.9999983358095185, -0.33200482774291656};
  const double l2e = 1.4426950408889634, c2 = (double)cap * cap;
  return CapPoly{(float)(l2e * t[0]), (float)(l2e * t[1] / c2), (float)(l2e * t[2] / (c2 * c2)),
                 (float)(l2e * t[3] / (c2 * c2 * c2)), 0.48f * cap,
                 (float)(l2e * u[0]), (float)(l2e * u[1] / c2), (float)(l2e * u[2] / (c2 * c2)), 0.24f * cap,
                 (float)(l2e * w[0]), (float)(l2e * w[1] / c2), 0.10f * cap};
}

// PACKED: the polynomial in pairs of packed fp32 (v_pk_mul_f32 / v_pk_fma_f32), else scalar fp32
// (the same IEEE operations per value, so bitwise the same result; packed fp32 VALU beside another
// wave's MFMAs is priced as an anti-lever in MI355X_MICROARCH.md's price list)
// scalar VALU the SLP vectorizer cannot pair into v_pk_* (A/B builds only: SCALAR below)
__device__ __forceinline__ float mul_s(float a, float b) {
  float r;
  asm("v_mul_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ float fma_s(float a, float b, float c) {
  float r;
  asm("v_fma_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}

// SCALAR (A/B builds): the LIN / QUAD tiers in unpaired scalar fp32 (the same IEEE operations); PKLIN (A/B
// builds): the LIN tier in packed pairs (the same IEEE operations, half the instructions)
template <bool PACKED = true, bool QUAD = false, bool LIN = false, bool SCALAR = false, bool PKLIN = false>
__device__ __forceinline__ void capped_exp16(const f32x16& x, float* p, float c1, float c2, const CapPoly& cp) {
  float mx = 0.0f;
#pragma unroll
  for (int i = 0; i < 16; ++i) mx = fmaxf(mx, fabsf(x[i]));
  if (LIN && __builtin_amdgcn_ballot_w64(mx > cp.x2) == 0) {
    if constexpr (PKLIN) {
      typedef float f2_t __attribute__((ext_vector_type(2)));
#pragma unroll
      for (int i = 0; i < 16; i += 2) {
        const f2_t xv = {x[i], x[i + 1]};
        const f2_t g = xv * __builtin_elementwise_fma(f2_t(cp.l1), xv * xv, f2_t(cp.l0));
        p[i] = __builtin_amdgcn_exp2f(g.x);
        p[i + 1] = __builtin_amdgcn_exp2f(g.y);
      }
    } else {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        if constexpr (SCALAR) p[i] = __builtin_amdgcn_exp2f(mul_s(x[i], fma_s(cp.l1, mul_s(x[i], x[i]), cp.l0)));
        else p[i] = __builtin_amdgcn_exp2f(x[i] * fmaf(cp.l1, x[i] * x[i], cp.l0));
      }
    }
  } else if (QUAD && __builtin_amdgcn_ballot_w64(mx > cp.x1) == 0) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      if constexpr (SCALAR) {
        const float u = mul_s(x[i], x[i]);
        p[i] = __builtin_amdgcn_exp2f(mul_s(x[i], fma_s(fma_s(cp.q2, u, cp.q1), u, cp.q0)));
      } else {
        const float u = x[i] * x[i];
        const float P = fmaf(fmaf(cp.q2, u, cp.q1), u, cp.q0);
        p[i] = __builtin_amdgcn_exp2f(x[i] * P);
      }
    }
  } else if (__builtin_amdgcn_ballot_w64(mx > cp.x0) == 0) {
    if constexpr (PACKED) {
      typedef float f2_t __attribute__((ext_vector_type(2)));
#pragma unroll
      for (int i = 0; i < 16; i += 2) {
        const f2_t xv = {x[i], x[i + 1]};
        const f2_t u = xv * xv;
        f2_t P = __builtin_elementwise_fma(f2_t(cp.k3), u, f2_t(cp.k2));
        P = __builtin_elementwise_fma(P, u, f2_t(cp.k1));
        P = __builtin_elementwise_fma(P, u, f2_t(cp.k0));
        const f2_t g = xv * P;
        p[i] = __builtin_amdgcn_exp2f(g.x);
        p[i + 1] = __builtin_amdgcn_exp2f(g.y);
      }
    } else {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const float u = x[i] * x[i];
        float P = fmaf(cp.k3, u, cp.k2);
        P = fmaf(P, u, cp.k1);
        P = fmaf(P, u, cp.k0);
        p[i] = __builtin_amdgcn_exp2f(x[i] * P);
      }
    }
  } else {
#pragma unroll
    for (int i = 0; i < 16; ++i) p[i] = capped_exp_exact(x[i], c1, c2);
  }
}

// LayerNorm statistics of one row from P partials (sum S_p, sum of squares about the partial mean Q_p)
// over 128 columns each (Chan): M2 = sum Q_p + 128 (S_p / 128 - mean)^2 -> (rstd, -mean * rstd),
// eps 1e-6 (layers.py:225-243).  Shared by ln_stats_finalize and the GEMMs that combine the partials
// themselves, so both give the same bits.
template <int PMAX>
__device__ __forceinline__ float2 ln_combine(const float2 (&pt)[PMAX], int P) {
  float tot = 0.f;
#pragma unroll
  for (int p = 0; p < PMAX; ++p)
    if (p < P) tot += pt[p].x;
  const float D = 128.0f * P;
  const float mean = tot / D;
  float m2 = 0.f;
#pragma unroll
  for (int p = 0; p < PMAX; ++p)
    if (p < P) {
      const float d = fmaf(pt[p].x, 1.0f / 128.0f, -mean);
      m2 = m2 + fmaf(128.0f * d, d, pt[p].y);
    }
  const float rs = 1.0f / sqrtf(m2 / D + 1e-6f);
  return make_float2(rs, -mean * rs);
}

__device__ __forceinline__ void wait_vmcnt0() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// ---- LDS reads hipcc must not wait for with vmcnt (the attention kernels' K/V chunks land by
// LDS-DMA while earlier chunks are read; a compiler-visible read there gets a vmcnt(0) in front
// of it).  Each helper issues its reads AND their lgkmcnt(0) in ONE asm statement with
// early-clobber outputs (cdna_hip_programming.md §5.7 item 1, form (i)): the destination
// registers are defined only after the data has landed, so no compiler copy, spill or reuse can
// touch them while a read is in flight.  tools/check_kernels.py rejects any asm load with a VGPR
// destination that does not carry its wait in the same statement. ----
typedef short s16x4 __attribute__((ext_vector_type(4)));

// 8 transposed reads (ds_read_b64_tr_b16) at ad[s][dh] and ad[s][dh] + 1024 -> v[s][dh][0 / 1]
__device__ __forceinline__ void lds_tr_read8(s16x4 (&v)[2][2][2], const uint32_t (&ad)[2][2]) {
  asm volatile(
      "ds_read_b64_tr_b16 %0, %8\n\t"
      "ds_read_b64_tr_b16 %1, %8 offset:1024\n\t"
      "ds_read_b64_tr_b16 %2, %9\n\t"
      "ds_read_b64_tr_b16 %3, %9 offset:1024\n\t"
      "ds_read_b64_tr_b16 %4, %10\n\t"
      "ds_read_b64_tr_b16 %5, %10 offset:1024\n\t"
      "ds_read_b64_tr_b16 %6, %11\n\t"
      "ds_read_b64_tr_b16 %7, %11 offset:1024\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&v"(v[0][0][0]), "=&v"(v[0][0][1]), "=&v"(v[0][1][0]), "=&v"(v[0][1][1]), "=&v"(v[1][0][0]),
        "=&v"(v[1][0][1]), "=&v"(v[1][1][0]), "=&v"(v[1][1][1])
      : "v"(ad[0][0]), "v"(ad[0][1]), "v"(ad[1][0]), "v"(ad[1][1])
      : "memory");
}

// 4 reads of 16 B (ds_read_b128) at ad[i] -> v[i]
__device__ __forceinline__ void lds_read4_b128(bf16x8 (&v)[4], const uint32_t (&ad)[4]) {
  asm volatile(
      "ds_read_b128 %0, %4\n\t"
      "ds_read_b128 %1, %5\n\t"
      "ds_read_b128 %2, %6\n\t"
      "ds_read_b128 %3, %7\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&v"(v[0]), "=&v"(v[1]), "=&v"(v[2]), "=&v"(v[3])
      : "v"(ad[0]), "v"(ad[1]), "v"(ad[2]), "v"(ad[3])
      : "memory");
}

// the same reads from per-lane base addresses plus a compile-time offset (loops unrolled so a tile's stage and key
// offsets are immediates: the per-tile address arithmetic disappears); same form (i): reads and wait in one statement
template <int OFF>
__device__ __forceinline__ void lds_read4_b128_o(bf16x8 (&v)[4], const uint32_t (&ad)[4]) {
  asm volatile(
      "ds_read_b128 %0, %4 offset:%8\n\t"
      "ds_read_b128 %1, %5 offset:%8\n\t"
      "ds_read_b128 %2, %6 offset:%8\n\t"
      "ds_read_b128 %3, %7 offset:%8\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&v"(v[0]), "=&v"(v[1]), "=&v"(v[2]), "=&v"(v[3])
      : "v"(ad[0]), "v"(ad[1]), "v"(ad[2]), "v"(ad[3]), "n"(OFF)
      : "memory");
}
// v[s][dh][hf] <- ad[dh] + OFF + 2048 s + 1024 hf
template <int OFF>
__device__ __forceinline__ void lds_tr_read8_o(s16x4 (&v)[2][2][2], const uint32_t (&ad)[2]) {
  asm volatile(
      "ds_read_b64_tr_b16 %0, %8 offset:%10\n\t"
      "ds_read_b64_tr_b16 %1, %8 offset:%11\n\t"
      "ds_read_b64_tr_b16 %2, %9 offset:%10\n\t"
      "ds_read_b64_tr_b16 %3, %9 offset:%11\n\t"
      "ds_read_b64_tr_b16 %4, %8 offset:%12\n\t"
      "ds_read_b64_tr_b16 %5, %8 offset:%13\n\t"
      "ds_read_b64_tr_b16 %6, %9 offset:%12\n\t"
      "ds_read_b64_tr_b16 %7, %9 offset:%13\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&v"(v[0][0][0]), "=&v"(v[0][0][1]), "=&v"(v[0][1][0]), "=&v"(v[0][1][1]), "=&v"(v[1][0][0]),
        "=&v"(v[1][0][1]), "=&v"(v[1][1][0]), "=&v"(v[1][1][1])
      : "v"(ad[0]), "v"(ad[1]), "n"(OFF), "n"(OFF + 1024), "n"(OFF + 2048), "n"(OFF + 3072)
      : "memory");
}

// ---- per-device launch state (host) ----
// The header allows one handle per device, driven from any host thread (include/videoprism_hip.h), so
// a kernel's dynamic-LDS attribute and the CU count are kept per (device, kernel) / per device, set under
// a lock the first time, and read lock-free afterwards (a thread-local cache of the pairs already set).
inline hipError_t ensure_dyn_lds(const void* fn, int bytes) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  const std::pair<int, const void*> key{dev, fn};
  thread_local std::set<std::pair<int, const void*>> seen;
  if (seen.count(key)) return hipSuccess;
  static std::mutex mu;
  static std::set<std::pair<int, const void*>> done;
  std::lock_guard<std::mutex> lk(mu);
  if (!done.count(key)) {
    e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
    if (e != hipSuccess) return e;
    done.insert(key);
  }
  seen.insert(key);
  return hipSuccess;
}

// CUs of the current device (256 on MI355X; the persistent GEMM grids are sized by it)
inline int device_cu_count() {
  constexpr int kMaxDev = 64;
  static std::atomic<int> cus[kMaxDev];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0) return 256;
  if (dev < kMaxDev) {
    const int c = cus[dev].load(std::memory_order_relaxed);
    if (c > 0) return c;
  }
  int n = 0;
  if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
  if (dev < kMaxDev) cus[dev].store(n, std::memory_order_relaxed);
  return n;
}

// ReLU that keeps a NaN a NaN like jax.nn.relu (text tower ffn_layer1, encoders.py:743): IEEE-754-2019
// maximum (gfx950 v_maximum3_f32), not maxNum
__device__ __forceinline__ float relu_nan(float x) { return __builtin_elementwise_maximum(x, 0.0f); }

}  // namespace vp
