// Diag-only (tools' A/B library): the auxiliary attention as two waves per SIMD alternating MFMA and VALU
// segments -- built, bitwise equal to the product kernel, and measured 33-38 % slower at the LvT-Large shape
// (tools/attn_bench.py long, var 512; profiles/r06/aux_attention_pp.txt): with one VALU wave per SIMD at a time
// the numerators issue at the lone-wave rate (4 cycles per VALU op instead of 2 with two VALU-issuing waves),
// and this kernel is VALU-bound.  Kept for the record; the product keeps attn_long_kernel.
#pragma once
#include "attention_long_kernel.h"

namespace vp {

namespace {

// ---------------------------------------------------------------------------------------------------------
// Two waves per SIMD, alternating (MI355X_MICROARCH.md "Two waves per SIMD"): one 512-thread workgroup per
// CU, waves w and w + 4 share SIMD w.  A wave owns 64 queries (two 32-query blocks sharing every K / V
// fragment read) and walks 32-key tiles in two kinds of segment separated by a workgroup barrier:
//   C(t): the MFMA segment -- P(t-1).V(t-1) into O, then the logits K(t).Q -> x;
//   V(t): the VALU segment -- the capped numerators of x, the row sums, bf16 P, and one LDS-DMA piece of the
//         chunk two ahead.
// Waves 0-3 run C(t) while waves 4-7 run V(t-1), then the roles swap: each SIMD pairs one wave's MFMAs with
// its partner's exponentials.  Phase p: waves 0-3 run C(p/2) (p even) / V((p-1)/2) (p odd), waves 4-7 one
// phase later.  K / V stream through a 4-stage ring of 64-key chunks (16 KiB; a chunk's last read is
// C(2c+2) of waves 4-7 at phase 4c+5, its stage is refilled from phase 4c+9 on); chunk c must have landed
// when waves 0-3 open it at phase 4c.  Per (query, tile) the arithmetic is the one-wave kernel's -- the
// same MFMA chains in the same order, the same tier decision per 32 x 32 tile, the same row-sum pairs --
// so the output is bitwise attn_long_kernel's.  TAIL as there (S % 512 != 0).
constexpr int kPpThreads = 512;
constexpr int kPpQ = 512;  // queries per workgroup: 8 waves x 64
constexpr int kPpLds = kLgStages * kLgStageBytes;  // 64 KiB

template <int VAR = 0, bool TAIL = false>
__global__ __launch_bounds__(kPpThreads, 2) void attn_long_pp_kernel(const bf16_t* __restrict__ qkv,
                                                                     bf16_t* __restrict__ o, int S, int heads,
                                                                     int nqb, float cap, int xcd_map, CapPoly cp) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int D = heads * 64;
  const int64_t ld = 3 * (int64_t)D;
  int bid = (int)blockIdx.x;
  if (xcd_map) bid = (bid & 7) * ((int)gridDim.x >> 3) + (bid >> 3);
  const int qb = bid % nqb;
  const int sh = bid / nqb;
  const int seq = sh / heads;
  const int h = sh % heads;
  const int lane = threadIdx.x & 63;
  const int w = wave_id();
  const int grp = w >> 2;  // 0: waves 0-3 (lead), 1: waves 4-7 (one phase behind)
  const bf16_t* base = qkv + (int64_t)seq * S * ld + h * 64;
  const int q0 = qb * kPpQ + w * 64;
  const int half = lane >> 5;

  // the wave's two 32-query blocks as B operands (form (ii) asm loads, retired by the prologue's wait)
  bf16x8 qf[2][4];
#pragma unroll
  for (int b = 0; b < 2; ++b) {
    const int qr = TAIL ? min(q0 + 32 * b + (lane & 31), S - 1) : q0 + 32 * b + (lane & 31);
    const bf16_t* qp = base + (int64_t)qr * ld + 8 * half;
#pragma unroll
    for (int kd = 0; kd < 4; ++kd)
      asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(qf[b][kd]) : "v"(qp + 16 * kd));
  }
  const int nchunks = TAIL ? (S + kLgChunk - 1) / kLgChunk : S / kLgChunk;
  // piece isV of chunk c: this wave's 8 key rows (K rows 8w.., then V rows 8w..), 1 KiB
  auto issue = [&](int c, int isV) {
    char* st = smem + (c & (kLgStages - 1)) * kLgStageBytes;
    const int row = w * 8 + (lane >> 3);
    const int ch = (lane & 7) ^ (isV ? swzV(row) : swzK(row));
    const int key = TAIL ? min(c * kLgChunk + row, S - 1) : c * kLgChunk + row;
    const bf16_t* src = base + (int64_t)key * ld + (isV ? 2 * D : D) + ch * 8;
    __builtin_amdgcn_global_load_lds(VP_GLB_PTR(src), VP_LDS_PTR(st + isV * kLgChunk * 128 + w * 1024), 16, 0, 0);
  };
  issue(0, 0);
  issue(0, 1);
  if (nchunks > 1) {
    issue(1, 0);
    issue(1, 1);
    asm volatile("s_waitcnt vmcnt(2)"
                 : "+v"(qf[0][0]), "+v"(qf[0][1]), "+v"(qf[0][2]), "+v"(qf[0][3]), "+v"(qf[1][0]), "+v"(qf[1][1]),
                   "+v"(qf[1][2]), "+v"(qf[1][3])
                 :
                 : "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)"
                 : "+v"(qf[0][0]), "+v"(qf[0][1]), "+v"(qf[0][2]), "+v"(qf[0][3]), "+v"(qf[1][0]), "+v"(qf[1][1]),
                   "+v"(qf[1][2]), "+v"(qf[1][3])
                 :
                 : "memory");
  }
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  if constexpr ((VAR & 256) != 0) {
    if (grp) __builtin_amdgcn_s_setprio(1);
  }

  const float c1 = 2.0f * kLog2e / cap;
  const float c2 = cap * kLog2e;
  f32x16 y[2][2] = {};
  f32x16 x[2] = {};
  bf16x8 pf[2][2] = {};
  typedef float f2_t __attribute__((ext_vector_type(2)));
  f2_t lsum2[2] = {{0.0f, 0.0f}, {0.0f, 0.0f}};
  const int krow_l = lane & 31;
  const int g = lane >> 4;
  const int li = lane & 15;
  const int trq = li >> 2, trp = li & 3;
  const int ntiles = 2 * nchunks;
  const int nphase = 2 * ntiles + 2;

#pragma unroll 1
  for (int p = 0; p < nphase; ++p) {
    if (((p + grp) & 1) == 0) {
      // ---- C(t): P(t-1).V(t-1), then K(t).Q ----
      const int t = (p - grp) >> 1;
      if (t >= 1) {
        const int tp = t - 1;
        const char* Vs = smem + ((tp >> 1) & (kLgStages - 1)) * kLgStageBytes + kLgChunk * 128;
        uint32_t vad[2][2];
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const int key = (tp & 1) * 32 + 16 * s + 4 * half + trq;
#pragma unroll
          for (int dh = 0; dh < 2; ++dh) {
            const int col = 32 * dh + 16 * (g & 1) + 4 * trp;
            const int cc = col >> 3;
            vad[s][dh] = (uint32_t)(uintptr_t)VP_LDS_PTR(Vs + key * 128 + ((cc ^ swzV(key)) << 4) + (col & 7) * 2);
          }
        }
        s16x4 vr[2][2][2];
        lds_tr_read8(vr, vad);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int s = 0; s < 2; ++s) {
#pragma unroll
          for (int dh = 0; dh < 2; ++dh) {
            const s16x4 lo = vr[s][dh][0], hi = vr[s][dh][1];
            const bf16x8 vf = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
#pragma unroll
            for (int b = 0; b < 2; ++b) y[b][dh] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, pf[b][s], y[b][dh], 0, 0, 0);
          }
        }
      }
      if (t < ntiles) {
        const char* Ks = smem + ((t >> 1) & (kLgStages - 1)) * kLgStageBytes;
        const int krow = (t & 1) * 32 + krow_l;
        bf16x8 kf[4];
        uint32_t kad[4];
#pragma unroll
        for (int kd = 0; kd < 4; ++kd) {
          const int cc = 2 * kd + half;
          kad[kd] = (uint32_t)(uintptr_t)VP_LDS_PTR(Ks + krow * 128 + ((cc ^ swzK(krow)) << 4));
        }
        lds_read4_b128(kf, kad);
#pragma unroll
        for (int b = 0; b < 2; ++b) {
          x[b] = f32x16{};
#pragma unroll
          for (int kd = 0; kd < 4; ++kd) x[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf[kd], qf[b][kd], x[b], 0, 0, 0);
        }
      }
    } else {
      // ---- V(t): numerators, row sums, bf16 P; one piece of chunk t/2 + 2 ----
      const int t = (p - 1 - grp) >> 1;
      if (t >= 0 && t < ntiles) {
#pragma unroll
        for (int b = 0; b < 2; ++b) {
          float pv[16];
          capped_exp16<true, true, true, false, (VAR & 128) != 0>(x[b], pv, c1, c2, cp);
          if constexpr (TAIL) {
            const int kbase = t * 32 + 4 * half;
            if (kbase + 28 >= S) {
#pragma unroll
              for (int i = 0; i < 16; ++i)
                if (kbase + 8 * (i >> 2) + (i & 3) >= S) pv[i] = 0.0f;
            }
          }
#pragma unroll
          for (int i = 0; i < 16; i += 2) lsum2[b] += f2_t{pv[i], pv[i + 1]};
#pragma unroll
          for (int s = 0; s < 2; ++s) {
            uint32_t u[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) u[j] = pack_bf16x2(pv[8 * s + 2 * j], pv[8 * s + 2 * j + 1]);
            pf[b][s] = *reinterpret_cast<bf16x8*>(u);
          }
        }
        const int cn = (t >> 1) + 2;
        if (cn < nchunks) issue(cn, t & 1);
      }
    }
    // chunk c is first read by waves 0-3 at phase 4c: before that phase every wave's pieces of it have
    // landed (younger pieces: those of chunk c + 1 issued so far, two by waves 0-3 and one by waves 4-7)
    if (((p + 1) & 3) == 0) {
      const int c = (p + 1) >> 2;
      if (c + 1 < nchunks) {
        if (grp == 0) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  }
#pragma unroll
  for (int b = 0; b < 2; ++b) {
    float lsum = lsum2[b].x + lsum2[b].y;
    lsum += __shfl_xor(lsum, 32);
    const float inv = 1.0f / lsum;
    const int q = q0 + 32 * b + (lane & 31);
    if (TAIL && q >= S) continue;
    bf16_t* op = o + ((int64_t)seq * S + q) * D + h * 64 + 4 * half;
#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4) {
      uint2 v0 = make_uint2(pack_bf16x2(y[b][0][4 * g4] * inv, y[b][0][4 * g4 + 1] * inv),
                            pack_bf16x2(y[b][0][4 * g4 + 2] * inv, y[b][0][4 * g4 + 3] * inv));
      uint2 v1 = make_uint2(pack_bf16x2(y[b][1][4 * g4] * inv, y[b][1][4 * g4 + 1] * inv),
                            pack_bf16x2(y[b][1][4 * g4 + 2] * inv, y[b][1][4 * g4 + 3] * inv));
      *reinterpret_cast<uint2*>(op + 8 * g4) = v0;
      *reinterpret_cast<uint2*>(op + 32 + 8 * g4) = v1;
    }
  }
}

template <int VAR, bool TAIL>
hipError_t launch_attn_long_pp_t(const bf16_t* qkv, bf16_t* o, int num_seq, int S, int heads, float cap,
                                 hipStream_t s) {
  const void* fn = reinterpret_cast<const void*>(attn_long_pp_kernel<VAR, TAIL>);
  hipError_t e = ensure_dyn_lds(fn, kPpLds);
  if (e != hipSuccess) return e;
  const int nqb = (S + kPpQ - 1) / kPpQ;
  const int64_t grid = (int64_t)num_seq * heads * nqb;
  if (grid > 0x7fffffff) return hipErrorInvalidValue;
  const int xcd_map = grid % 8 == 0 ? 1 : 0;
  const CapPoly cp = make_cap_poly(cap);
  VP_NOTE_KERNEL(fn);
  hipLaunchKernelGGL((attn_long_pp_kernel<VAR, TAIL>), dim3((unsigned)grid), dim3(kPpThreads), kPpLds, s, qkv, o, S,
                     heads, nqb, cap, xcd_map, cp);
  return hipGetLastError();
}

// S >= 512: S % 512 == 0, or TAIL
template <int VAR>
hipError_t launch_attn_long_pp(const bf16_t* qkv, bf16_t* o, int num_seq, int S, int heads, float cap,
                               hipStream_t s) {
  if (S < kPpQ || !(cap > 0.0f) || num_seq < 1) return hipErrorInvalidValue;
  if (S % kPpQ == 0) return launch_attn_long_pp_t<VAR, false>(qkv, o, num_seq, S, heads, cap, s);
  return launch_attn_long_pp_t<VAR, true>(qkv, o, num_seq, S, heads, cap, s);
}


}  // namespace

}  // namespace vp
