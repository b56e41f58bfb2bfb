// Measured bf16 MFMA peak of this GPU (the spec's 2.5 PF dense is confirmed
// by an in-repo microbenchmark and both figures are stated).  Measurement infrastructure for bench.py's
// `roofline.peak_measured`, not part of the product library.
//
// Every CU runs one 256-thread workgroup (one wave per SIMD); each wave keeps its A / B fragments (random
// bf16 from a per-lane hash: the chip holds a lower clock on random operands than on zeros,
// MI355X_MICROARCH.md "DVFS give-back") and independent accumulators in registers (8 of 16x16, 4 of 32x32) and
// issues `iters` x 8 / 4 back-to-back MFMAs of one shape: v_mfma_f32_16x16x32_bf16 (the GEMMs' instruction) or
// v_mfma_f32_32x32x16_bf16 (the attention kernels').  TFLOP/s = FLOPs / event time of the launch.
// Wave 0 of each workgroup stamps s_memtime (shader clock) and s_memrealtime (100 MHz) around its loop
// into a buffer of its own (nothing reads it back on the device): clock = d(memtime) / d(realtime) x 100 MHz.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <vector>

namespace {

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
  return x;
}

// random bf16 in about [-1, 1): sign, exponent 126 - (0..1), random mantissa
__device__ __forceinline__ bf16x8 rand_frag(uint32_t seed) {
  bf16x8 v;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const uint32_t h = hash32(seed * 8u + j);
    v[j] = (short)(((h & 0x8000u)) | ((126u - ((h >> 7) & 1u)) << 7) | (h & 0x7fu));
  }
  return v;
}

template <int SHAPE>  // 0: 16x16x32 bf16, 1: 32x32x16 bf16, 2: 16x16x4 f32, 3: 32x32x2 f32
__global__ __launch_bounds__(256) void mfma_peak_kernel(int iters, float* sink, unsigned long long* stamps) {
  const uint32_t gid = blockIdx.x * 256u + threadIdx.x;
  const bf16x8 a = rand_frag(gid * 2u + 1u), b = rand_frag(gid * 2u + 2u);
  unsigned long long t0 = 0, r0 = 0;
  if (threadIdx.x == 0) {
    t0 = __builtin_amdgcn_s_memtime();
    r0 = __builtin_amdgcn_s_memrealtime();
  }
  // the MFMAs as asm statements: the compiler, given an accumulator array in a loop, rotates it through
  // AGPR copies between iterations (measured 874 TF); each statement here is exactly one MFMA on a fixed
  // register quad / block, and an accumulator recurs every NACC MFMAs (128 cycles, past any latency)
  float s = 0.0f;
  if constexpr (SHAPE == 0) {
    f32x4 a0 = {0.f}, a1 = {1.f}, a2 = {2.f}, a3 = {3.f}, a4 = {4.f}, a5 = {5.f}, a6 = {6.f}, a7 = {7.f};
#pragma unroll 1
    for (int it = 0; it < iters; ++it) {
#define VP_M16(acc) asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+v"(acc) : "v"(a), "v"(b))
      VP_M16(a0); VP_M16(a1); VP_M16(a2); VP_M16(a3); VP_M16(a4); VP_M16(a5); VP_M16(a6); VP_M16(a7);
#undef VP_M16
    }
    const f32x4 t = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
    s = t[0] + t[1] + t[2] + t[3];
  } else if constexpr (SHAPE == 2) {  // fp32 operands: one random float per lane in about [-1, 1)
    const float fa = __uint_as_float((hash32(gid * 2u + 1u) & 0x807fffffu) | 0x3f000000u);
    const float fb = __uint_as_float((hash32(gid * 2u + 2u) & 0x807fffffu) | 0x3f000000u);
    f32x4 a0 = {0.f}, a1 = {1.f}, a2 = {2.f}, a3 = {3.f}, a4 = {4.f}, a5 = {5.f}, a6 = {6.f}, a7 = {7.f};
#pragma unroll 1
    for (int it = 0; it < iters; ++it) {
#define VP_F16(acc) asm volatile("v_mfma_f32_16x16x4_f32 %0, %1, %2, %0" : "+v"(acc) : "v"(fa), "v"(fb))
      VP_F16(a0); VP_F16(a1); VP_F16(a2); VP_F16(a3); VP_F16(a4); VP_F16(a5); VP_F16(a6); VP_F16(a7);
#undef VP_F16
    }
    const f32x4 t = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
    s = t[0] + t[1] + t[2] + t[3];
  } else if constexpr (SHAPE == 3) {
    const float fa = __uint_as_float((hash32(gid * 2u + 1u) & 0x807fffffu) | 0x3f000000u);
    const float fb = __uint_as_float((hash32(gid * 2u + 2u) & 0x807fffffu) | 0x3f000000u);
    f32x16 a0 = {0.f}, a1 = {1.f}, a2 = {2.f}, a3 = {3.f};
#pragma unroll 1
    for (int it = 0; it < iters; ++it) {
#define VP_F32(acc) asm volatile("v_mfma_f32_32x32x2_f32 %0, %1, %2, %0" : "+v"(acc) : "v"(fa), "v"(fb))
      VP_F32(a0); VP_F32(a1); VP_F32(a2); VP_F32(a3);
#undef VP_F32
    }
    const f32x16 t = a0 + a1 + a2 + a3;
#pragma unroll
    for (int j = 0; j < 16; ++j) s += t[j];
  } else {
    f32x16 a0 = {0.f}, a1 = {1.f}, a2 = {2.f}, a3 = {3.f};
#pragma unroll 1
    for (int it = 0; it < iters; ++it) {
#define VP_M32(acc) asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(acc) : "v"(a), "v"(b))
      VP_M32(a0); VP_M32(a1); VP_M32(a2); VP_M32(a3);
#undef VP_M32
    }
    const f32x16 t = a0 + a1 + a2 + a3;
#pragma unroll
    for (int j = 0; j < 16; ++j) s += t[j];
  }
  if (threadIdx.x == 0) {
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
    stamps[2 * blockIdx.x] = t1 - t0;
    stamps[2 * blockIdx.x + 1] = r1 - r0;
  }
  sink[gid] = s;
}

}  // namespace

extern "C" {

// shape 0: v_mfma_f32_16x16x32_bf16, 1: v_mfma_f32_32x32x16_bf16, 2: v_mfma_f32_16x16x4_f32 (the fp32 GEMMs'),
// 3: v_mfma_f32_32x32x2_f32 (the fp32 attention's).  Runs `reps` timed launches of `iters`
// loop iterations after one warm-up launch on every CU of device `device`; writes the best and the median
// TFLOP/s, the median in-kernel clock (GHz) over the workgroups of the last launch, and the ms per launch.
// Returns 0 or a hipError_t.
int mfma_peak_run(int device, int shape, int iters, int reps, double* tflops_best, double* tflops_median,
                  double* clock_ghz, double* ms_median) {
  if (shape < 0 || shape > 3) return hipErrorInvalidValue;
  hipError_t e = hipSetDevice(device);
  if (e != hipSuccess) return e;
  int cus = 0;
  if ((e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device)) != hipSuccess) return e;
  float* sink = nullptr;
  unsigned long long* stamps = nullptr;
  if ((e = hipMalloc(&sink, (size_t)cus * 256 * 4)) != hipSuccess) return e;
  if ((e = hipMalloc(&stamps, (size_t)cus * 16)) != hipSuccess) { hipFree(sink); return e; }
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  // FLOPs per MFMA: 2 * 16 * 16 * 32 = 16384 (8 per iteration) or 2 * 32 * 32 * 16 = 32768 (4 per iteration)
  const double per_iter[4] = {8.0 * 16384.0, 4.0 * 32768.0, 8.0 * 2048.0, 4.0 * 4096.0};
  const double flops = (double)cus * 4 * iters * per_iter[shape];
  std::vector<double> tf;
  for (int r = 0; r <= reps && e == hipSuccess; ++r) {
    hipEventRecord(a, nullptr);
    if (shape == 0)
      hipLaunchKernelGGL(mfma_peak_kernel<0>, dim3(cus), dim3(256), 0, nullptr, iters, sink, stamps);
    else if (shape == 1)
      hipLaunchKernelGGL(mfma_peak_kernel<1>, dim3(cus), dim3(256), 0, nullptr, iters, sink, stamps);
    else if (shape == 2)
      hipLaunchKernelGGL(mfma_peak_kernel<2>, dim3(cus), dim3(256), 0, nullptr, iters, sink, stamps);
    else
      hipLaunchKernelGGL(mfma_peak_kernel<3>, dim3(cus), dim3(256), 0, nullptr, iters, sink, stamps);
    hipEventRecord(b, nullptr);
    e = hipEventSynchronize(b);
    float ms = 0.f;
    hipEventElapsedTime(&ms, a, b);
    if (r > 0) tf.push_back(flops / (ms * 1e-3) / 1e12);
  }
  if (e == hipSuccess && !tf.empty()) {
    std::vector<unsigned long long> st((size_t)cus * 2);
    e = hipMemcpy(st.data(), stamps, st.size() * 8, hipMemcpyDeviceToHost);
    std::vector<double> clk;
    for (int i = 0; i < cus; ++i)
      if (st[2 * i + 1] > 0) clk.push_back((double)st[2 * i] / (double)st[2 * i + 1] * 0.1);
    std::sort(clk.begin(), clk.end());
    std::vector<double> s = tf;
    std::sort(s.begin(), s.end());
    *tflops_best = s.back();
    *tflops_median = s[s.size() / 2];
    *ms_median = flops / (*tflops_median * 1e12) * 1e3;
    *clock_ghz = clk.empty() ? 0.0 : clk[clk.size() / 2];
  }
  hipEventDestroy(a);
  hipEventDestroy(b);
  hipFree(sink);
  hipFree(stamps);
  return e;
}

}  // extern "C"
