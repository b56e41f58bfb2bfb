// The auxiliary (4096-token) attention kernel of the LvT video path, as a template shared by the
// product library (attention_long.hip: VAR = 0) and the tools' diag library (tools/diag/csrc:
// variants for A/B).  Design notes: attention_long.hip.
#pragma once
#include <type_traits>

#include "vp_common.h"
#include "vp_kernels.h"

namespace vp {

namespace {

constexpr float kLog2e = 1.4426950408889634f;

__device__ __forceinline__ float capped_exp(float x, float two_log2e_over_cap, float cap_log2e) {
  const float t = __builtin_amdgcn_exp2f(x * two_log2e_over_cap);
  const float r = __builtin_amdgcn_rcpf(t + 1.0f);
  return __builtin_amdgcn_exp2f(cap_log2e - 2.0f * cap_log2e * r);
}

__device__ __forceinline__ int swzK(int row) { return (row >> 1) & 7; }
__device__ __forceinline__ int swzV(int row) { return ((row >> 1) & 1) << 2; }

constexpr int kLgThreads = 512;          // 8 waves x 32 queries
constexpr int kLgQ = 256;                // queries per workgroup
constexpr int kLgChunk = 64;             // keys per LDS stage
constexpr int kLgStages = 4;
constexpr int kLgStageBytes = 2 * kLgChunk * 128;  // K then V, 128 B per key row
constexpr int kLgLds = kLgStages * kLgStageBytes;  // 64 KiB

// The numerator takes the linear tier on tiles whose logits all satisfy |x| <= 0.10 cap (vp_common.h
// capped_exp16 LIN), else the quadratic tier for |x| <= 0.24 cap (QUAD: as accurate as the cubic), and
// the row sum accumulates in packed pairs; with logits of std 0.5 / 6 (tools/attn_bench.py long,
// LvT-Large shape) 2.606 / 2.926 ms vs 2.828 / 2.953 without the quadratic tier and the packed sum.
// VAR (A/B builds of the diag library; the product uses 0): 1 = the polynomial numerator in scalar
// instead of packed fp32 arithmetic (bitwise the same values); 2 = no quadratic tier; 4 = the row sum
// one value at a time; 8 = no linear tier; 16 = the row sum on the MFMA (a ones A operand against the
// bf16 numerators, so the sum of the rounded values P.V uses); 32 = the row sum by v_dot2_f32_bf16 of
// the bf16 numerator pairs; 64 = the LIN / QUAD tiers and the row sum in unpaired scalar fp32; 128 = the LIN
// tier in packed pairs; 256 = s_setprio 1 for waves 4-7 (MI355X_MICROARCH.md, two waves per SIMD, item 4); 1024 =
// round 5's chunk loop with the stage and the K / V read addresses computed per tile (the product unrolls the chunk
// loop over the 4 LDS stages, so the reads take per-lane bases + immediate offsets: bitwise the same, 2.4-3.7 %
// faster at logit std 0.5 / 2 / 6, profiles/r06/aux_attention_stage_unroll.txt).
// TAIL: S % 256 != 0 (S > 256; frame sizes whose T*N is not a multiple of 256, encoders.py:846-857 takes any
// T*N): nqb = ceil(S / 256) and ceil(S / 64) chunks; a query or key row past S is read from row S - 1 (so
// every load stays inside the sequence), the numerators of keys past S are zeroed before the row sum and
// P.V, and queries past S are not stored.  S % 256 == 0 takes TAIL = false: the product instantiation as before
template <int VAR = 0, bool TAIL = false>
__global__ __launch_bounds__(kLgThreads, 4) void attn_long_kernel(const bf16_t* __restrict__ qkv,
                                                                  bf16_t* __restrict__ o, int S,
                                                                  int heads, int nqb, float cap,
                                                                  int xcd_map, CapPoly cp) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int D = heads * 64;
  const int64_t ld = 3 * (int64_t)D;
  // XCD-aware work id: hardware places workgroup b on XCD b % 8; give every XCD a contiguous
  // range of work ids so the q-blocks of one (sequence, head) share that XCD's L2
  int bid = (int)blockIdx.x;
  if (xcd_map) bid = (bid & 7) * ((int)gridDim.x >> 3) + (bid >> 3);
  const int qb = bid % nqb;
  const int sh = bid / nqb;
  const int seq = sh / heads;
  const int h = sh % heads;
  const int lane = threadIdx.x & 63;
  const int w = wave_id();
  const bf16_t* base = qkv + (int64_t)seq * S * ld + h * 64;
  const int q0 = qb * kLgQ + w * 32;
  const int half = lane >> 5;

  // this wave's 32 queries as the B operand (lane: q = l&31, d = 16kd + 8(l>>5) + j): asm loads
  // (hipcc cannot count a plain load against the LDS-DMA pieces behind it and would drain the
  // stream with vmcnt(0)), retired by the prologue's wait statement that names qf (form (ii) of
  // cdna_hip_programming.md §5.7 item 1; audited by tools/check_kernels.py)
  bf16x8 qf[4];
  {
    const int qr = TAIL ? min(q0 + (lane & 31), S - 1) : q0 + (lane & 31);
    const bf16_t* qp = base + (int64_t)qr * ld + 8 * half;
#pragma unroll
    for (int kd = 0; kd < 4; ++kd)
      asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(qf[kd]) : "v"(qp + 16 * kd));
  }
  // chunk c -> stage c % 4: wave w loads piece w of the stage's 16 pieces (8 K pieces, then
  // 8 V pieces; a piece = 8 key rows x 128 B = 1 KiB) and piece w + 8
  const int nchunks = TAIL ? (S + kLgChunk - 1) / kLgChunk : S / kLgChunk;
  auto issue = [&](int c) {
    char* st = smem + (c & (kLgStages - 1)) * kLgStageBytes;
#pragma unroll
    for (int isV = 0; isV < 2; ++isV) {
      const int row = w * 8 + (lane >> 3);  // key row within the chunk
      const int ch = (lane & 7) ^ (isV ? swzV(row) : swzK(row));
      const int key = TAIL ? min(c * kLgChunk + row, S - 1) : c * kLgChunk + row;
      const bf16_t* src = base + (int64_t)key * ld + (isV ? 2 * D : D) + ch * 8;
      __builtin_amdgcn_global_load_lds(VP_GLB_PTR(src), VP_LDS_PTR(st + isV * kLgChunk * 128 + w * 1024),
                                       16, 0, 0);
    }
  };
#pragma unroll
  for (int c = 0; c < kLgStages - 1; ++c) issue(c);  // nchunks >= 4 (S % 256 == 0, checked by the launcher)
  // Q and chunk 0 landed (chunks 1, 2 -- 4 pieces -- may still be in flight); the loop's own
  // chunk-0 wait is then a no-op
  asm volatile("s_waitcnt vmcnt(4)" : "+v"(qf[0]), "+v"(qf[1]), "+v"(qf[2]), "+v"(qf[3]) : : "memory");

  const float c1 = 2.0f * kLog2e / cap;
  const float c2 = cap * kLog2e;
  f32x16 y0 = {}, y1 = {};
  [[maybe_unused]] f32x16 ysum = {};
  float lsum = 0.0f;
  typedef float f2_t __attribute__((ext_vector_type(2)));
  f2_t lsum2 = {0.0f, 0.0f};
  const int krow_l = lane & 31;
  const int g = lane >> 4;
  const int li = lane & 15;
  const int trq = li >> 2, trp = li & 3;
  if constexpr ((VAR & 256) != 0) {
    if (w >= 4) __builtin_amdgcn_s_setprio(1);  // static priority for the second-dispatched half
  }

  // per-lane K / V read bases of the stage-unrolled loop (stage and key offsets are immediates there): krow = kt 32 + krow_l, so
  // swzK(krow) = (krow_l >> 1) & 7 and, for key = kt 32 + 16 s + 4 half + trq, swzV(key) = ((trq >> 1) & 1) << 2
  [[maybe_unused]] uint32_t kb[4], vb[2];
  if constexpr ((VAR & 1024) == 0) {
    const uint32_t sb = (uint32_t)(uintptr_t)VP_LDS_PTR(smem);
#pragma unroll
    for (int kd = 0; kd < 4; ++kd) kb[kd] = sb + krow_l * 128 + (((2 * kd + half) ^ ((krow_l >> 1) & 7)) << 4);
#pragma unroll
    for (int dh = 0; dh < 2; ++dh) {
      const int col = 32 * dh + 16 * (g & 1) + 4 * trp;
      vb[dh] = sb + (4 * half + trq) * 128 + (((col >> 3) ^ (((trq >> 1) & 1) << 2)) << 4) + (col & 7) * 2;
    }
  }
  // one 64-key chunk: STG = its LDS stage as a compile-time constant (the product), or -1 (c % 4 at run time, VAR 1024)
  auto chunk = [&](int c, auto STG) {
    constexpr int stg = decltype(STG)::value;
    // this wave's pieces of chunk c have landed when at most the younger chunks' pieces
    // (2 per chunk) are outstanding; then one barrier makes every wave's pieces visible and
    // retires all reads of stage (c - 1) % 4, which chunk c + 3 overwrites
    const int younger = nchunks - 1 - c < kLgStages - 2 ? nchunks - 1 - c : kLgStages - 2;
    if (younger >= 2) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else if (younger == 1) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (c + kLgStages - 1 < nchunks) issue(c + kLgStages - 1);
    const char* Ks = smem + (c & (kLgStages - 1)) * kLgStageBytes;
    [[maybe_unused]] const char* Vs = Ks + kLgChunk * 128;
    auto tile = [&](auto KT) {
      constexpr int kt = decltype(KT)::value;
      f32x16 x = {};
      const int krow = kt * 32 + krow_l;
      // K and V reads: inline asm (a visible LDS read would get a vmcnt(0) for the chunks still
      // landing), reads and wait in one statement (vp_common.h lds_read4_b128 / lds_tr_read8)
      bf16x8 kf[4];
      if constexpr (stg >= 0) {
        lds_read4_b128_o<stg * kLgStageBytes + kt * 4096>(kf, kb);
      } else {
        uint32_t kad[4];
#pragma unroll
        for (int kd = 0; kd < 4; ++kd) {
          const int cc = 2 * kd + half;
          kad[kd] = (uint32_t)(uintptr_t)VP_LDS_PTR(Ks + krow * 128 + ((cc ^ swzK(krow)) << 4));
        }
        lds_read4_b128(kf, kad);
      }
#pragma unroll
      for (int kd = 0; kd < 4; ++kd) x = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf[kd], qf[kd], x, 0, 0, 0);
      float p[16];
      capped_exp16<(VAR & 1) == 0, (VAR & 2) == 0, (VAR & 8) == 0, (VAR & 64) != 0, (VAR & 128) != 0>(x, p, c1, c2,
                                                                                                     cp);
      if constexpr (TAIL) {
        // keys past S (the last chunk only): weight 0.  Lane l, value i holds key row
        // 8 (i / 4) + 4 (l / 32) + i % 4 of the 32-key tile (the 32x32 MFMA output layout)
        const int kbase = c * kLgChunk + kt * 32 + 4 * half;
        if (kbase + 28 >= S) {
#pragma unroll
          for (int i = 0; i < 16; ++i)
            if (kbase + 8 * (i >> 2) + (i & 3) >= S) p[i] = 0.0f;
        }
      }
      if constexpr ((VAR & 48) != 0) {
        // row sum from the bf16 numerators below
      } else if constexpr ((VAR & 64) != 0) {
#pragma unroll
        for (int i = 0; i < 16; i += 2) {
          float t;
          asm("v_add_f32 %0, %1, %2" : "=v"(t) : "v"(p[i]), "v"(p[i + 1]));
          asm("v_add_f32 %0, %1, %2" : "=v"(lsum) : "v"(lsum), "v"(t));
        }
      } else if constexpr ((VAR & 4) == 0) {  // row sum in packed pairs
#pragma unroll
        for (int i = 0; i < 16; i += 2) lsum2 += f2_t{p[i], p[i + 1]};
      } else {
#pragma unroll
        for (int i = 0; i < 16; ++i) lsum += p[i];
      }
      bf16x8 pf[2];
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        uint32_t u[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) u[j] = pack_bf16x2(p[8 * s + 2 * j], p[8 * s + 2 * j + 1]);
        pf[s] = *reinterpret_cast<bf16x8*>(u);
        if constexpr ((VAR & 32) != 0) {
#pragma unroll
          for (int j = 0; j < 4; ++j)
            asm("v_dot2_f32_bf16 %0, %1, %2, %3" : "=v"(lsum) : "v"(u[j]), "v"(0x3f803f80u), "v"(lsum));
        }
      }
      if constexpr ((VAR & 16) != 0) {
        const bf16x8 ones = {0x3f80, 0x3f80, 0x3f80, 0x3f80, 0x3f80, 0x3f80, 0x3f80, 0x3f80};
        ysum = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ones, pf[0], ysum, 0, 0, 0);
        ysum = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ones, pf[1], ysum, 0, 0, 0);
      }
      s16x4 vr[2][2][2];
      if constexpr (stg >= 0) {
        lds_tr_read8_o<stg * kLgStageBytes + kLgChunk * 128 + kt * 4096>(vr, vb);
      } else {
        uint32_t vad[2][2];
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const int key = kt * 32 + 16 * s + 4 * half + trq;
#pragma unroll
          for (int dh = 0; dh < 2; ++dh) {
            const int col = 32 * dh + 16 * (g & 1) + 4 * trp;
            const int cc = col >> 3;
            vad[s][dh] = (uint32_t)(uintptr_t)VP_LDS_PTR(Vs + key * 128 + ((cc ^ swzV(key)) << 4) + (col & 7) * 2);
          }
        }
        lds_tr_read8(vr, vad);
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int s = 0; s < 2; ++s) {
#pragma unroll
        for (int dh = 0; dh < 2; ++dh) {
          const s16x4 lo = vr[s][dh][0], hi = vr[s][dh][1];
          const bf16x8 vf = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
          if (dh == 0) y0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, pf[s], y0, 0, 0, 0);
          else y1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, pf[s], y1, 0, 0, 0);
        }
      }
    };
    tile(std::integral_constant<int, 0>{});
    tile(std::integral_constant<int, 1>{});
  };
  if constexpr ((VAR & 1024) == 0) {
#pragma unroll 1
    for (int c0 = 0; c0 < nchunks; c0 += kLgStages) {
      chunk(c0, std::integral_constant<int, 0>{});
      if (c0 + 1 < nchunks) chunk(c0 + 1, std::integral_constant<int, 1>{});
      if (c0 + 2 < nchunks) chunk(c0 + 2, std::integral_constant<int, 2>{});
      if (c0 + 3 < nchunks) chunk(c0 + 3, std::integral_constant<int, 3>{});
    }
  } else {
#pragma unroll 1
    for (int c = 0; c < nchunks; ++c) chunk(c, std::integral_constant<int, -1>{});
  }
  if constexpr ((VAR & 16) != 0) {
    lsum = ysum[0];  // every row of the ones product holds the full sum of its query column
  } else {
    if constexpr ((VAR & 100) == 0) lsum = lsum2.x + lsum2.y;
    lsum += __shfl_xor(lsum, 32);
  }
  const float inv = 1.0f / lsum;
  if (TAIL && q0 + (lane & 31) >= S) return;
  bf16_t* op = o + ((int64_t)seq * S + q0 + (lane & 31)) * D + h * 64 + 4 * half;
#pragma unroll
  for (int g4 = 0; g4 < 4; ++g4) {
    uint2 v0 = make_uint2(pack_bf16x2(y0[4 * g4] * inv, y0[4 * g4 + 1] * inv),
                          pack_bf16x2(y0[4 * g4 + 2] * inv, y0[4 * g4 + 3] * inv));
    uint2 v1 = make_uint2(pack_bf16x2(y1[4 * g4] * inv, y1[4 * g4 + 1] * inv),
                          pack_bf16x2(y1[4 * g4 + 2] * inv, y1[4 * g4 + 3] * inv));
    *reinterpret_cast<uint2*>(op + 8 * g4) = v0;
    *reinterpret_cast<uint2*>(op + 32 + 8 * g4) = v1;
  }
}

template <int VAR, bool TAIL>
hipError_t launch_attn_long_t(const bf16_t* qkv, bf16_t* o, int num_seq, int S, int heads, float cap, hipStream_t s) {
  const void* fn = reinterpret_cast<const void*>(attn_long_kernel<VAR, TAIL>);
  hipError_t e = ensure_dyn_lds(fn, kLgLds);
  if (e != hipSuccess) return e;
  const int nqb = (S + kLgQ - 1) / kLgQ;
  const int64_t grid = (int64_t)num_seq * heads * nqb;
  if (grid > 0x7fffffff) return hipErrorInvalidValue;
  const int xcd_map = grid % 8 == 0 ? 1 : 0;
  const CapPoly cp = make_cap_poly(cap);
  VP_NOTE_KERNEL(fn);
  hipLaunchKernelGGL((attn_long_kernel<VAR, TAIL>), dim3((unsigned)grid), dim3(kLgThreads), kLgLds, s, qkv, o, S,
                     heads, nqb, cap, xcd_map, cp);
  return hipGetLastError();
}

// S % 256 == 0 (S >= 256) or any S > 256 (TAIL: the prologue's three chunks exist)
template <int VAR>
hipError_t launch_attn_long(const bf16_t* qkv, bf16_t* o, int num_seq, int S, int heads, float cap, hipStream_t s) {
  if (S < kLgQ || !(cap > 0.0f) || num_seq < 1) return hipErrorInvalidValue;
  if (S % kLgQ == 0) return launch_attn_long_t<VAR, false>(qkv, o, num_seq, S, heads, cap, s);
  return launch_attn_long_t<VAR, true>(qkv, o, num_seq, S, heads, cap, s);
}


}  // namespace

}  // namespace vp
