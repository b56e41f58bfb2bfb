// Attention kernels of the LvT video-text path.
//
// attention_long_bf16: the auxiliary encoder's self-attention over all T*N spatio-temporal
//   tokens of a clip (encoders.py:846-857, S = 4096 at 16 frames): DotProductAttention
//   (layers.py:601-661) with q pre-scaled by dh^-0.5, logits capped by cap*tanh(x/cap) and an
//   fp32 softmax.  As in attention.hip the cap bounds every logit to [-cap, cap], so the
//   softmax needs no running max: numerators are exp(logit) and the fp32 row sum is exact.
//   Flash-style: a workgroup owns 256 queries of one (sequence, head) -- 8 waves x 32, each
//   query on one lane column of v_mfma_f32_32x32x16_bf16 -- and streams K and V through LDS in
//   64-key chunks, 4 stages deep (buffer_load..lds style global_load_lds pieces of 8 rows x
//   128 B, swizzled), one barrier per chunk.  The numerators never touch LDS: they are the B
//   operand of O^T = V^T.P^T (V read transposed with ds_read_b64_tr_b16).  Workgroups of one
//   (sequence, head) are mapped onto one XCD so its K/V (1 MiB at S = 4096) stays in that
//   XCD's L2.  No masks: the auxiliary encoder is called without paddings (:855).
//
// attention_masked: generic fp32-math attention with key paddings and the causal merge of
//   layers.py:111-179 (a padded *query* row is fully masked when causal, and a fully masked
//   row gets uniform weights, as the reference's where(mask, logits, -0.7*FLT_MAX) + softmax
//   produce).  Used by the text tower (S = L+1 = 65, causal + paddings, both dtypes) and by
//   the fp32 auxiliary encoder.  Online softmax (cap may be 0), exact tanhf / expf.
#include "attention_long_kernel.h"

namespace vp {

namespace {

// ------------------------------------------------------------------------------------
// generic masked attention, fp32 math (dh = 64)
// ------------------------------------------------------------------------------------
constexpr int kGnQ = 64;      // queries per workgroup (4 lanes each)
constexpr int kGnChunk = 64;  // keys per LDS stage

template <typename T>
__device__ __forceinline__ float ld_f(const T* p, int64_t i) {
  if constexpr (sizeof(T) == 2) return bf2f(reinterpret_cast<const bf16_t*>(p)[i]);
  else return reinterpret_cast<const float*>(p)[i];
}

template <typename T>
__global__ __launch_bounds__(256) void attn_masked_kernel(const T* __restrict__ qkv, T* __restrict__ o, int S,
                                                         int heads, int nqb, float cap,
                                                         const float* __restrict__ key_pad, int causal) {
  __shared__ float Ks[kGnChunk][65];
  __shared__ float Vs[kGnChunk][64];
  __shared__ float kp[kGnChunk];
  __shared__ int any_valid_key;
  const int qb = blockIdx.x % nqb;
  const int sh = blockIdx.x / nqb;
  const int seq = sh / heads;
  const int h = sh % heads;
  const int D = heads * 64;
  const int64_t ld = 3 * (int64_t)D;
  const T* base = qkv + (int64_t)seq * S * ld + h * 64;
  const int t = threadIdx.x;
  const int qi = qb * kGnQ + (t >> 2);
  const int part = t & 3;
  const bool qvalid = qi < S;
  float q[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) q[j] = qvalid ? ld_f(base, (int64_t)qi * ld + 16 * part + j) : 0.0f;
  // rows whose every key is masked get uniform weights (equal logits)
  if (t == 0) any_valid_key = 0;
  __syncthreads();
  if (key_pad && !causal) {
    for (int s = t; s < S; s += 256)
      if (key_pad[(int64_t)seq * S + s] == 0.0f) any_valid_key = 1;
  }
  __syncthreads();
  bool all_masked = false;
  if (key_pad) {
    if (causal) all_masked = qvalid && key_pad[(int64_t)seq * S + qi] != 0.0f;
    else all_masked = any_valid_key == 0;
  }
  float m = -INFINITY, l = 0.0f;
  float acc[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) acc[j] = 0.0f;
  // every thread runs the same key loop (barriers inside); masked keys are skipped per query
  for (int k0 = 0; k0 < S; k0 += kGnChunk) {
    __syncthreads();
    for (int i = t; i < kGnChunk * 64; i += 256) {
      const int r = i >> 6, d = i & 63;
      const bool in = k0 + r < S;
      Ks[r][d] = in ? ld_f(base, (int64_t)(k0 + r) * ld + D + d) : 0.0f;
      Vs[r][d] = in ? ld_f(base, (int64_t)(k0 + r) * ld + 2 * D + d) : 0.0f;
    }
    if (t < kGnChunk) kp[t] = (key_pad && k0 + t < S) ? key_pad[(int64_t)seq * S + k0 + t] : 0.0f;
    __syncthreads();
    const int n = S - k0 < kGnChunk ? S - k0 : kGnChunk;
    for (int j = 0; j < n; ++j) {
      float d = 0.0f;
#pragma unroll
      for (int e = 0; e < 16; ++e) d = fmaf(q[e], Ks[j][16 * part + e], d);
      d += __shfl_xor(d, 1);
      d += __shfl_xor(d, 2);
      const int key = k0 + j;
      bool valid = kp[j] == 0.0f && (!causal || key <= qi);
      float logit = cap > 0.0f ? cap * tanhf(d / cap) : d;
      if (all_masked) {
        valid = true;
        logit = 0.0f;
      }
      if (!valid) continue;
      const float mn = fmaxf(m, logit);
      const float sc = __expf(m - mn);
      const float pe = __expf(logit - mn);
      l = l * sc + pe;
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[e] = fmaf(pe, Vs[j][16 * part + e], acc[e] * sc);
      m = mn;
    }
  }
  if (!qvalid) return;
  const float inv = 1.0f / l;
  T* op = o + ((int64_t)seq * S + qi) * D + h * 64 + 16 * part;
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    const float v = acc[e] * inv;
    if constexpr (sizeof(T) == 2) reinterpret_cast<bf16_t*>(op)[e] = f2bf(v);
    else reinterpret_cast<float*>(op)[e] = v;
  }
}

}  // namespace

hipError_t attention_long_bf16(const bf16_t* qkv, bf16_t* o, int num_seq, int S, int heads, float cap,
                               hipStream_t s) {
  return launch_attn_long<0>(qkv, o, num_seq, S, heads, cap, s);
}

hipError_t attention_masked(const void* qkv, void* o, int in_is_bf16, int num_seq, int S, int heads,
                            float cap, const float* key_pad, int causal, hipStream_t s) {
  if (S < 1 || num_seq < 1) return hipErrorInvalidValue;
  const int nqb = (S + kGnQ - 1) / kGnQ;
  const int64_t grid = (int64_t)num_seq * heads * nqb;
  if (grid > 0x7fffffff) return hipErrorInvalidValue;
  VP_NOTE_KERNEL(in_is_bf16 ? (const void*)attn_masked_kernel<bf16_t> : (const void*)attn_masked_kernel<float>);
  if (in_is_bf16)
    hipLaunchKernelGGL(attn_masked_kernel<bf16_t>, dim3((unsigned)grid), dim3(256), 0, s,
                       (const bf16_t*)qkv, (bf16_t*)o, S, heads, nqb, cap, key_pad, causal);
  else
    hipLaunchKernelGGL(attn_masked_kernel<float>, dim3((unsigned)grid), dim3(256), 0, s, (const float*)qkv,
                       (float*)o, S, heads, nqb, cap, key_pad, causal);
  return hipGetLastError();
}

}  // namespace vp
