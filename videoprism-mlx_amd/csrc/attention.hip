// Capped dot-product attention for the factorized encoder.
//
// Reference semantics (layers.py:601-661, _cap_logits :586-594, masks :51-89):
//   logits = q.k (q pre-scaled by dh^-0.5, folded into the q projection weights)
//   logits = cap * tanh(logits / cap); softmax in fp32; probs . v
// Because |cap*tanh(.)| <= cap (= 50 on every VideoPrism config), exp(logit) lies in
// [e^-50, e^50] and the softmax needs no running max: numerators are exp(x) directly and
// the row sum is exact in fp32.  Padded keys (key_pad = 1) contribute 0; if every key of a
// row is padded, the reference's where(mask, logits, -0.7*FLT_MAX) makes all logits equal
// and softmax uniform -- reproduced by treating every key as weight 1.
//
// attention_spatial_bf16: S = 256 (one frame's patch grid), dh = 64.  One workgroup per
//   (frame, head); K and V (32 KiB each) land in LDS by global_load_lds; 8 waves x 32
//   queries.  S^T = K.Q^T on v_mfma_f32_32x32x16_bf16 puts one query per lane column; the
//   bf16 numerators are fed straight back as the B operand of O^T = V^T.P^T (V read with
//   ds_read_b64_tr_b16), so P never touches LDS and the row sum is lane-local.
// attention_temporal_bf16: S = T <= 16 frames.  One wave per (sequence, head), 16x16x32 for
//   Q.K^T and 16x16x16 for P.V; memory-bound on the qkv rows.
// attention_f32: fp32 path (fprop_dtype=float32): S = 256 with 0 < cap <= 50 on v_mfma_f32_32x32x2f32
//   (attn_f32_mfma_kernel), any other S <= 256 / cap on a generic online-softmax kernel; exact tanhf/expf.
#include <type_traits>

#include "vp_common.h"
#include "vp_kernels.h"

namespace vp {

namespace {

constexpr float kLog2e = 1.4426950408889634f;

// exp(cap * tanh(x / cap)) with tanh(y) = 1 - 2 / (exp(2y) + 1); saturates correctly.
__device__ __forceinline__ float capped_exp(float x, float two_log2e_over_cap, float cap_log2e) {
  const float t = __builtin_amdgcn_exp2f(x * two_log2e_over_cap);
  const float r = __builtin_amdgcn_rcpf(t + 1.0f);
  return __builtin_amdgcn_exp2f(cap_log2e - 2.0f * cap_log2e * r);
}

__device__ __forceinline__ int swzK(int row) { return (row >> 1) & 7; }
__device__ __forceinline__ int swzV(int row) { return ((row >> 1) & 1) << 2; }

__device__ __forceinline__ bf16x4 tr_read(const char* p) {
  s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) s16x4*)(p));
  return bf16x4{v[0], v[1], v[2], v[3]};
}

// ------------------------------------------------------------------------------------
// spatial: S = 256, dh = 64
// ------------------------------------------------------------------------------------
constexpr int kSpS = 256;
constexpr int kSpThreads = 512;
constexpr int kSpLds = 2 * kSpS * 128 + kSpS * 4 + 16;

// q|k|v layout by strides (elements): row rs, head hs, section (q -> k -> v) sec; the row-major
// fused projection output is (3D, 64, D).  O goes through LDS and leaves as whole 128-B row
// segments (8 rows per store); O is written with nontemporal stores (read once, by the post
// projection), so it does not displace the residual stream from the Infinity Cache (gemm_epilogue.h
// kResidStream).  (Nontemporal q|k|v loads measured slower: 2.45 vs 2.37-2.40 ms per step.)
// BLK: q|k|v in the row-blocked layout of the q|k|v GEMM's EPI_BF16_LN_BLK ([M/16][3D/32][16][32],
// element (row, col) at ((row >> 4) * 3D/32 + (col >> 5)) * 512 + (row & 15) * 32 + (col & 31)): a K / V
// piece (8 keys x 64 dims) is then two 512-B runs instead of 8 rows of 128 B
template <bool MASK, bool BLK = false>
__global__ __launch_bounds__(kSpThreads, 4) void attn_spatial_kernel(
    const bf16_t* __restrict__ qkv, bf16_t* __restrict__ o, int heads, float cap,
    const float* __restrict__ key_pad, int rev, int64_t rs, int64_t hs, int64_t sec) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* Ks = smem;
  char* Vs = smem + kSpS * 128;
  float* kp = reinterpret_cast<float*>(smem + 2 * kSpS * 128);
  int* allmask = reinterpret_cast<int*>(kp + kSpS);

  const int D = heads * 64;
  const int64_t ld = rs;
  // rev: sequences in reverse order, so the last-written (Infinity-Cache resident) q|k|v rows
  // of the producing GEMM are read first
  const int bid = rev ? (int)gridDim.x - 1 - (int)blockIdx.x : (int)blockIdx.x;
  const int seq = bid / heads;
  const int h = bid % heads;
  const int lane = threadIdx.x & 63;
  const int w = wave_id();
  const bf16_t* base = qkv + (int64_t)seq * kSpS * ld + h * hs;
  // BLK: element (row r of this sequence, column col of the q|k|v row)
  auto blk_at = [&](int r, int col) {
    return qkv + (((int64_t)seq * 16 + (r >> 4)) * (ld >> 5) + (col >> 5)) * 512 + (r & 15) * 32 + (col & 31);
  };

  // ---- this wave's 32 queries as the B operand (lane: q = l&31, d = 16kd + 8(l>>5) + j),
  // requested ahead of the K/V stream.  hipcc cannot count a plain load against the LDS-DMA
  // pieces behind it (mixed event kinds: it emits vmcnt(0), draining the stream before the first
  // key tile), so these are asm loads retired by chunk 0's wait statement, which names qf as
  // operands (cdna_hip_programming.md §5.7 item 1, form (ii)); tools/check_kernels.py audits the
  // assembly for any compiler access to those registers in between, and the build refuses
  // scratch or spills in every product kernel ----
  const int q0 = w * 32;
  const int half = lane >> 5;
  bf16x8 qf[4];
  {
    const bf16_t* qp = base + (int64_t)(q0 + (lane & 31)) * ld + 8 * half;
#pragma unroll
    for (int kd = 0; kd < 4; ++kd) {
      const bf16_t* qa = BLK ? blk_at(q0 + (lane & 31), h * 64 + 16 * kd + 8 * half) : qp + 16 * kd;
      asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(qf[kd]) : "v"(qa));
    }
  }
  // ---- stage K and V in 4 chunks of 64 keys, chunk-major: wave w loads K piece c*8+w and
  // V piece 32+c*8+w of chunk c (a piece = 8 keys x 128 B), so key tiles 2c, 2c+1 can start as
  // soon as chunk c has landed while the later chunks are still in flight ----
#pragma unroll
  for (int cc = 0; cc < 4; ++cc)
#pragma unroll
    for (int isV = 0; isV < 2; ++isV) {
      const int piece = isV * 32 + cc * 8 + w;
      const int row = (piece & 31) * 8 + (lane >> 3);
      const int c = (lane & 7) ^ (isV ? swzV(row) : swzK(row));
      const bf16_t* src = BLK ? blk_at(row, (isV ? 2 : 1) * (int)sec + h * 64 + c * 8)
                              : base + (int64_t)row * ld + (isV ? 2 * sec : sec) + c * 8;
      __builtin_amdgcn_global_load_lds(VP_GLB_PTR(src), VP_LDS_PTR(smem + piece * 1024), 16, 0, 0);
    }
  if constexpr (MASK) {  // (padded batches: no streaming)
    if (threadIdx.x < kSpS) kp[threadIdx.x] = key_pad[(int64_t)seq * kSpS + threadIdx.x];
    if (threadIdx.x == 0) *allmask = 1;
    asm volatile("s_waitcnt vmcnt(0)" : "+v"(qf[0]), "+v"(qf[1]), "+v"(qf[2]), "+v"(qf[3]) : : "memory");
    __syncthreads();
  }
  // chunk cc of every wave has landed: this wave's vmcnt leaves only its younger chunks in
  // flight, then one barrier
  auto chunk_ready = [&](auto CC) {
    constexpr int cc = decltype(CC)::value;
    if constexpr (!MASK) {
      if constexpr (cc == 0)  // also retires the Q loads (issued before every piece)
        asm volatile("s_waitcnt vmcnt(6)" : "+v"(qf[0]), "+v"(qf[1]), "+v"(qf[2]), "+v"(qf[3]) : : "memory");
      else
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * (3 - cc)) : "memory");
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  bool all_masked = false;
  if constexpr (MASK) {
    if (threadIdx.x < kSpS && kp[threadIdx.x] == 0.0f) *allmask = 0;
    __syncthreads();
    all_masked = *allmask != 0;
  }

  const float c1 = 2.0f * kLog2e / cap;
  const float c2 = cap * kLog2e;
  f32x16 y0 = {}, y1 = {};
  float lsum = 0.0f;
  const int krow_l = lane & 31;
  const int g = lane >> 4;
  const int li = lane & 15;
  const int trq = li >> 2, trp = li & 3;

  // S^T tile of keys kt*32 .. +31: X[key][q]
  auto qk = [&](int kt) {
    f32x16 x = {};
    const int krow = kt * 32 + krow_l;
#pragma unroll
    for (int kd = 0; kd < 4; ++kd) {
      const int c = 2 * kd + half;
      const bf16x8 kf = *reinterpret_cast<const bf16x8*>(Ks + krow * 128 + ((c ^ swzK(krow)) << 4));
      x = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[kd], x, 0, 0, 0);
    }
    return x;
  };
  // per-lane V read bases (lds_tr_read8_o): for key = kt 32 + 16 s + 4 half + trq, swzV(key) = ((trq >> 1) & 1) << 2,
  // so a tile's V addresses are these plus the immediate kt 4096 (+ 2048 s, + 1024 for the upper 4 rows)
  [[maybe_unused]] uint32_t vb[2];
#pragma unroll
  for (int dh = 0; dh < 2; ++dh) {
    const int col = 32 * dh + 16 * (g & 1) + 4 * trp;
    vb[dh] = (uint32_t)(uintptr_t)VP_LDS_PTR(Vs + (4 * half + trq) * 128 + (((col >> 3) ^ (((trq >> 1) & 1) << 2)) << 4) +
                                             (col & 7) * 2);
  }
  // numerators of tile kt, then O^T += V^T . X
  // OFFT: the tile's V offset kt * 4096 as a compile-time constant (the unrolled unmasked form), or -1 (run time)
  auto pv = [&](int kt, auto OFFT, const f32x16& x) {
    constexpr int voff = decltype(OFFT)::value;
    // numerators: register i <-> key kt*32 + (i&3) + 8(i>>2) + 4*half (exact three-transcendental
    // form: the one-transcendental polynomial moved the full-depth LvT-B bf16 embedding across the
    // 1e-3 bar)
    float p[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) p[i] = capped_exp(x[i], c1, c2);
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      float e = p[i];
      if constexpr (MASK) {
        const int key = kt * 32 + (i & 3) + 8 * (i >> 2) + 4 * half;
        e = all_masked ? 1.0f : (kp[key] != 0.0f ? 0.0f : e);
      }
      p[i] = e;
      lsum += e;
    }
    bf16x8 pf[2];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      uint32_t u[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) u[j] = pack_bf16x2(p[8 * s + 2 * j], p[8 * s + 2 * j + 1]);
      pf[s] = *reinterpret_cast<bf16x8*>(u);
    }
    // O^T += V^T . X  (A = V^T via transposed reads, B = P^T numerators).  hipcc puts a vmcnt(0)
    // for the in-flight K/V chunks in front of a visible ds_read_tr (it cannot tell it from a read
    // of a chunk still landing), so the 8 reads are inline asm -- issued together with their
    // lgkmcnt(0) in ONE statement with early-clobber outputs: the destinations are defined only
    // once the data has landed, so no compiler copy or spill can touch them in flight
    // (cdna_hip_programming.md §5.7 item 1, form (i))
    s16x4 vr[2][2][2];
    if constexpr (voff >= 0) {
      lds_tr_read8_o<voff>(vr, vb);
    } else {
      uint32_t ad[2][2];
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int key = kt * 32 + 16 * s + 4 * half + trq;
#pragma unroll
        for (int dh = 0; dh < 2; ++dh) {
          const int col = 32 * dh + 16 * (g & 1) + 4 * trp;
          const int c = col >> 3;
          ad[s][dh] = (uint32_t)(uintptr_t)VP_LDS_PTR(Vs + key * 128 + ((c ^ swzV(key)) << 4) + (col & 7) * 2);
        }
      }
      lds_tr_read8(vr, ad);
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

  // (a software-pipelined form -- the S^T MFMAs of tile kt+1 issued ahead of tile kt's
  // numerators -- is bitwise equal but measured 289.8 vs 206.8 us: at 128 VGPRs it spills inside
  // the loop; profiles/HISTORY.md round 3.)  Unmasked (round 6): the 8 tiles written out, so every K / V read address
  // is a per-lane base plus an immediate offset (no per-tile address arithmetic); the masked form keeps the loop (its
  // key-padding reads would spill written out)
  chunk_ready(std::integral_constant<int, 0>{});
  if constexpr (!MASK) {
    using std::integral_constant;
    pv(0, integral_constant<int, 0 * 4096>{}, qk(0));
    pv(1, integral_constant<int, 1 * 4096>{}, qk(1));
    chunk_ready(integral_constant<int, 1>{});
    pv(2, integral_constant<int, 2 * 4096>{}, qk(2));
    pv(3, integral_constant<int, 3 * 4096>{}, qk(3));
    chunk_ready(integral_constant<int, 2>{});
    pv(4, integral_constant<int, 4 * 4096>{}, qk(4));
    pv(5, integral_constant<int, 5 * 4096>{}, qk(5));
    chunk_ready(integral_constant<int, 3>{});
    pv(6, integral_constant<int, 6 * 4096>{}, qk(6));
    pv(7, integral_constant<int, 7 * 4096>{}, qk(7));
  } else {
#pragma unroll 1
    for (int cc = 0; cc < 4; ++cc) {
#pragma unroll 2
      for (int kt = 2 * cc; kt < 2 * cc + 2; ++kt) pv(kt, std::integral_constant<int, -1>{}, qk(kt));
    }
  }
  lsum += __shfl_xor(lsum, 32);
  const float inv = 1.0f / lsum;
  // y_dh[i] = O^T[d = 32dh + (i&3) + 8(i>>2) + 4*half][q = q0 + (l&31)].  Every wave is done with
  // K/V: the wave's 32 x 64 output tile goes to its 4 KiB of the K region ([q][16-B chunk ^ (q & 7)]),
  // then 8 lanes per row store whole 128-B segments
  __syncthreads();
  char* st = smem + w * 4096;
  const int ql = lane & 31;
#pragma unroll
  for (int g4 = 0; g4 < 4; ++g4) {
    const uint2 v0 = make_uint2(pack_bf16x2(y0[4 * g4] * inv, y0[4 * g4 + 1] * inv),
                                pack_bf16x2(y0[4 * g4 + 2] * inv, y0[4 * g4 + 3] * inv));
    const uint2 v1 = make_uint2(pack_bf16x2(y1[4 * g4] * inv, y1[4 * g4 + 1] * inv),
                                pack_bf16x2(y1[4 * g4 + 2] * inv, y1[4 * g4 + 3] * inv));
    *reinterpret_cast<uint2*>(st + ql * 128 + (((g4) ^ (ql & 7)) << 4) + 8 * half) = v0;
    *reinterpret_cast<uint2*>(st + ql * 128 + (((4 + g4) ^ (ql & 7)) << 4) + 8 * half) = v1;
  }
  __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const int r = p * 8 + (lane >> 3), c = lane & 7;
    const uint4 v = *reinterpret_cast<const uint4*>(st + r * 128 + ((c ^ (r & 7)) << 4));
    st_nt(o + ((int64_t)seq * kSpS + q0 + r) * D + h * 64 + c * 8, v);
  }
}

// ------------------------------------------------------------------------------------
// sequences of 16 < S <= 256 (temporal attention of clips longer than 16 frames): the spatial
// kernel's tiles over 256 query / key slots per workgroup, holding 256 / Sp sequences of one head,
// Sp = S rounded up to 32, 64, 128 or 256.  Wave w's 32 queries lie in one sequence and run over that
// sequence's Sp / 32 key tiles; slots past S are masked keys and unstored queries.  K and V are
// staged whole (LDS-DMA, then one barrier: no chunk pipelining), the numerators are the spatial
// kernel's exact capped form, P is rounded to bf16 for O^T = V^T.P^T and the row sum is fp32.
// ------------------------------------------------------------------------------------
constexpr int kSqLds = 2 * kSpS * 128 + kSpS * 4 + 8 * 4;  // K, V, key paddings, 8 all-masked flags

template <bool MASK>
__global__ __launch_bounds__(kSpThreads, 4) void attn_seq_kernel(const bf16_t* __restrict__ qkv,
                                                                bf16_t* __restrict__ o, int num_seq, int S,
                                                                int Sp, int heads, float cap,
                                                                const float* __restrict__ key_pad, int causal) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* Ks = smem;
  char* Vs = smem + kSpS * 128;
  float* kp = reinterpret_cast<float*>(smem + 2 * kSpS * 128);  // [slot] key padding (MASK)
  int* allmask = reinterpret_cast<int*>(kp + kSpS);              // [sequence of the workgroup]
  const int D = heads * 64;
  const int64_t ld = 3 * (int64_t)D;
  const int per = kSpS / Sp;  // sequences per workgroup
  const int h = (int)blockIdx.x % heads;
  const int seq0 = (int)blockIdx.x / heads * per;
  const int lane = threadIdx.x & 63;
  const int w = wave_id();
  // slot -> q|k|v row of this head (slots past S or past the last sequence read a valid row, unused)
  auto row_of = [&](int slot) {
    const int j = slot / Sp, t = slot - j * Sp;
    const int sq = seq0 + j < num_seq ? seq0 + j : num_seq - 1;
    return (int64_t)sq * S + (t < S ? t : S - 1);
  };
  // K and V: 64 pieces of 8 slots x 128 B, 8 per wave; the bank swizzle goes on the source address
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int piece = i * 8 + w;
    const int isV = piece >> 5;
    const int slot = (piece & 31) * 8 + (lane >> 3);
    const int c = (lane & 7) ^ (isV ? swzV(slot) : swzK(slot));
    const bf16_t* src = qkv + row_of(slot) * ld + (isV ? 2 * D : D) + h * 64 + c * 8;
    __builtin_amdgcn_global_load_lds(VP_GLB_PTR(src), VP_LDS_PTR(smem + piece * 1024), 16, 0, 0);
  }
  const int q0 = w * 32;
  const int half = lane >> 5;
  const int j = q0 / Sp;  // this wave's sequence in the workgroup
  bf16x8 qf[4];
  {
    const bf16_t* qp = qkv + row_of(q0 + (lane & 31)) * ld + h * 64 + 8 * half;
#pragma unroll
    for (int kd = 0; kd < 4; ++kd) qf[kd] = *reinterpret_cast<const bf16x8*>(qp + 16 * kd);
  }
  if constexpr (MASK) {
    if (threadIdx.x < kSpS) {
      const int jj = threadIdx.x / Sp, t = threadIdx.x - jj * Sp;
      kp[threadIdx.x] = (t < S && seq0 + jj < num_seq) ? key_pad[(int64_t)(seq0 + jj) * S + t] : 1.0f;
    }
    if (threadIdx.x < 8) allmask[threadIdx.x] = 1;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if constexpr (MASK) {
    if (threadIdx.x < kSpS && (threadIdx.x % Sp) < S && kp[threadIdx.x] == 0.0f) allmask[threadIdx.x / Sp] = 0;
    __syncthreads();
  }
  // causal (text tower, layers.py:111-179 merged with the key paddings): key t <= query t; a padded query's row is
  // fully masked, so its weights are uniform over all S keys (as attention_masked and the reference's softmax of
  // equal logits); otherwise a sequence with every key padded gets uniform weights
  const int qt = q0 + (lane & 31) - j * Sp;
  const bool all_masked = MASK && (causal ? kp[q0 + (lane & 31)] != 0.0f : allmask[j] != 0);

  const float c1 = 2.0f * kLog2e / cap;
  const float c2 = cap * kLog2e;
  f32x16 y0 = {}, y1 = {};
  float lsum = 0.0f;
  const int krow_l = lane & 31;
  const int g = lane >> 4;
  const int li = lane & 15;
  const int trq = li >> 2, trp = li & 3;
  const int kt0 = j * Sp / 32, kt1 = kt0 + Sp / 32;
#pragma unroll 1
  for (int kt = kt0; kt < kt1; ++kt) {
    f32x16 x = {};
    const int krow = kt * 32 + krow_l;
#pragma unroll
    for (int kd = 0; kd < 4; ++kd) {
      const int c = 2 * kd + half;
      const bf16x8 kf = *reinterpret_cast<const bf16x8*>(Ks + krow * 128 + ((c ^ swzK(krow)) << 4));
      x = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[kd], x, 0, 0, 0);
    }
    // register i <-> key slot kt*32 + (i&3) + 8(i>>2) + 4*half
    float p[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int slot = kt * 32 + (i & 3) + 8 * (i >> 2) + 4 * half;
      float e = capped_exp(x[i], c1, c2);
      if (causal && slot - j * Sp > qt) e = 0.0f;
      if constexpr (MASK) e = all_masked ? 1.0f : (kp[slot] != 0.0f ? 0.0f : e);
      if (slot - j * Sp >= S) e = 0.0f;
      p[i] = e;
      lsum += e;
    }
    bf16x8 pf[2];
#pragma unroll
    for (int sidx = 0; sidx < 2; ++sidx) {
      uint32_t u[4];
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) u[jj] = pack_bf16x2(p[8 * sidx + 2 * jj], p[8 * sidx + 2 * jj + 1]);
      pf[sidx] = *reinterpret_cast<bf16x8*>(u);
    }
#pragma unroll
    for (int sidx = 0; sidx < 2; ++sidx) {
      const int key = kt * 32 + 16 * sidx + 4 * half + trq;
#pragma unroll
      for (int dh = 0; dh < 2; ++dh) {
        const int col = 32 * dh + 16 * (g & 1) + 4 * trp;
        const int c = col >> 3;
        const char* a = Vs + key * 128 + ((c ^ swzV(key)) << 4) + (col & 7) * 2;
        const bf16x4 lo = tr_read(a), hi = tr_read(a + 8 * 128);
        const bf16x8 vf = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        if (dh == 0) y0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, pf[sidx], y0, 0, 0, 0);
        else y1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, pf[sidx], y1, 0, 0, 0);
      }
    }
  }
  lsum += __shfl_xor(lsum, 32);
  const float inv = 1.0f / lsum;
  const int slot = q0 + (lane & 31);
  const int t = slot - j * Sp;
  if (t >= S || seq0 + j >= num_seq) return;
  // y_dh[i] = O^T[d = 32dh + (i&3) + 8(i>>2) + 4*half][query]: 4 consecutive dims per register quad
  bf16_t* op = o + ((int64_t)(seq0 + j) * S + t) * D + h * 64 + 4 * half;
#pragma unroll
  for (int g4 = 0; g4 < 4; ++g4) {
    *reinterpret_cast<uint2*>(op + 8 * g4) = make_uint2(pack_bf16x2(y0[4 * g4] * inv, y0[4 * g4 + 1] * inv),
                                                        pack_bf16x2(y0[4 * g4 + 2] * inv, y0[4 * g4 + 3] * inv));
    *reinterpret_cast<uint2*>(op + 32 + 8 * g4) = make_uint2(pack_bf16x2(y1[4 * g4] * inv, y1[4 * g4 + 1] * inv),
                                                             pack_bf16x2(y1[4 * g4 + 2] * inv, y1[4 * g4 + 3] * inv));
  }
}

// ------------------------------------------------------------------------------------
// temporal: S <= 16, dh = 64; one wave per (sequence, head)
// ------------------------------------------------------------------------------------
constexpr int kTpWaves = 4;

template <bool MASK>
__global__ __launch_bounds__(kTpWaves * 64) void attn_temporal_kernel(
    const bf16_t* __restrict__ qkv, bf16_t* __restrict__ o, int num_pairs, int S, int heads,
    float cap, const float* __restrict__ key_pad) {
  __shared__ __attribute__((aligned(16))) char vlds[kTpWaves * 16 * 128];
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int pair = blockIdx.x * kTpWaves + w;
  if (pair >= num_pairs) return;  // whole wave exits together
  const int seq = pair / heads;
  const int h = pair % heads;
  const int D = heads * 64;
  const int64_t ld = 3 * (int64_t)D;
  const bf16_t* base = qkv + (int64_t)seq * S * ld + h * 64;
  char* vs = vlds + w * 16 * 128;

  const int r16 = lane & 15;
  const int g = lane >> 4;
  // Q/K fragments (16x16x32): lane row r16, d = 32ks + 8g + j
  bf16x8 qf[2], kf[2];
  const bool rv = r16 < S;
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) {
    if (rv) {
      qf[ks] = *reinterpret_cast<const bf16x8*>(base + (int64_t)r16 * ld + 32 * ks + 8 * g);
      kf[ks] = *reinterpret_cast<const bf16x8*>(base + (int64_t)r16 * ld + D + 32 * ks + 8 * g);
    } else {
      qf[ks] = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
      kf[ks] = qf[ks];
    }
  }
  // V rows -> LDS [16][64] (row 128 B): lane covers row lane>>3 (+8), chunk lane&7
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = i * 8 + (lane >> 3);
    bf16x8 v = {0, 0, 0, 0, 0, 0, 0, 0};
    if (row < S) v = *reinterpret_cast<const bf16x8*>(base + (int64_t)row * ld + 2 * D + (lane & 7) * 8);
    *reinterpret_cast<bf16x8*>(vs + row * 128 + (lane & 7) * 16) = v;
  }
  f32x4 x = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) x = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf[ks], qf[ks], x, 0, 0, 0);
  // x[r] = S^T[key = 4g + r][q = r16]
  bool all_masked = false;
  float kpad[4] = {0.f, 0.f, 0.f, 0.f};
  if constexpr (MASK) {
    // every lane evaluates the whole key set of its sequence (S <= 16 floats)
    int nvalid = 0;
    for (int k = 0; k < S; ++k) nvalid += key_pad[(int64_t)seq * S + k] == 0.0f;
    all_masked = nvalid == 0;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int key = 4 * g + r;
      kpad[r] = key < S ? key_pad[(int64_t)seq * S + key] : 1.0f;
    }
  }
  const float c1 = 2.0f * kLog2e / cap;
  const float c2 = cap * kLog2e;
  float p[4];
  float lsum = 0.f;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int key = 4 * g + r;
    float e = key < S ? capped_exp(x[r], c1, c2) : 0.0f;
    if constexpr (MASK) e = key < S ? (all_masked ? 1.0f : (kpad[r] != 0.0f ? 0.0f : e)) : 0.0f;
    p[r] = e;
    lsum += e;
  }
  lsum += __shfl_xor(lsum, 16);
  lsum += __shfl_xor(lsum, 32);
  const float inv = 1.0f / lsum;
  uint32_t pu[2] = {pack_bf16x2(p[0], p[1]), pack_bf16x2(p[2], p[3])};
  const bf16x4 pb = *reinterpret_cast<bf16x4*>(pu);
  __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): V rows written by this wave
  __builtin_amdgcn_wave_barrier();
  const int trq = r16 >> 2, trp = r16 & 3;
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) {
    // A = V^T: lane (d = 16dt + r16) x keys 4g..4g+3 via transposed read
    const bf16x4 vf = tr_read(vs + (4 * g + trq) * 128 + (16 * dt + 4 * trp) * 2);
    f32x4 y = {0.f, 0.f, 0.f, 0.f};
    y = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(vf, pb, y, 0, 0, 0);
    // y[r] = O^T[d = 16dt + 4g + r][q = r16]
    if (rv) {
      uint2 st = make_uint2(pack_bf16x2(y[0] * inv, y[1] * inv), pack_bf16x2(y[2] * inv, y[3] * inv));
      *reinterpret_cast<uint2*>(o + ((int64_t)seq * S + r16) * D + h * 64 + 16 * dt + 4 * g) = st;
    }
  }
}

// ------------------------------------------------------------------------------------
// fp32 generic (fprop_dtype=float32): one workgroup per (sequence, head), one query per
// thread, K/V of the sequence in LDS, online softmax with exact tanhf/expf.
// ------------------------------------------------------------------------------------
constexpr int kF32MaxS = 256;

__global__ __launch_bounds__(256) void attn_f32_kernel(const float* __restrict__ qkv,
                                                        float* __restrict__ o, int S, int heads,
                                                        float cap,
                                                        const float* __restrict__ key_pad) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* Ks = reinterpret_cast<float*>(smem);        // [S][64]
  float* Vs = Ks + S * 64;                            // [S][64]
  float* kp = Vs + S * 64;                            // [S]
  int& nvalid = *reinterpret_cast<int*>(kp + S);
  const int D = heads * 64;
  const int64_t ld = 3 * (int64_t)D;
  const int seq = blockIdx.x / heads;
  const int h = blockIdx.x % heads;
  const float* base = qkv + (int64_t)seq * S * ld + h * 64;
  if (threadIdx.x == 0) nvalid = 0;
  for (int i = threadIdx.x; i < S * 16; i += blockDim.x) {
    const int row = i >> 4, c4 = (i & 15) * 4;
    *reinterpret_cast<float4*>(Ks + row * 64 + c4) =
        *reinterpret_cast<const float4*>(base + (int64_t)row * ld + D + c4);
    *reinterpret_cast<float4*>(Vs + row * 64 + c4) =
        *reinterpret_cast<const float4*>(base + (int64_t)row * ld + 2 * D + c4);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < S; i += blockDim.x) {
    const float pv = key_pad ? key_pad[(int64_t)seq * S + i] : 0.0f;
    kp[i] = pv;
    if (pv == 0.0f) atomicAdd(&nvalid, 1);
  }
  __syncthreads();
  const bool all_masked = nvalid == 0;
  const int qi = threadIdx.x;
  if (qi >= S) return;
  float q[64];
#pragma unroll
  for (int d = 0; d < 64; d += 4) {
    const float4 t = *reinterpret_cast<const float4*>(base + (int64_t)qi * ld + d);
    q[d] = t.x; q[d + 1] = t.y; q[d + 2] = t.z; q[d + 3] = t.w;
  }
  float acc[64];
#pragma unroll
  for (int d = 0; d < 64; ++d) acc[d] = 0.f;
  float m = -INFINITY, l = 0.f;
  for (int j = 0; j < S; ++j) {
    if (!all_masked && kp[j] != 0.0f) continue;
    float s = 0.f;
    if (!all_masked) {
#pragma unroll
      for (int d = 0; d < 64; ++d) s = fmaf(q[d], Ks[j * 64 + d], s);
      if (cap > 0.f) s = cap * tanhf(s / cap);
    }
    const float mn = fmaxf(m, s);
    const float sc = expf(m - mn);
    const float e = expf(s - mn);
    l = l * sc + e;
#pragma unroll
    for (int d = 0; d < 64; ++d) acc[d] = fmaf(acc[d], sc, e * Vs[j * 64 + d]);
    m = mn;
  }
  const float inv = 1.0f / l;
  float* op = o + ((int64_t)seq * S + qi) * D + h * 64;
#pragma unroll
  for (int d = 0; d < 64; d += 4)
    *reinterpret_cast<float4*>(op + d) =
        make_float4(acc[d] * inv, acc[d + 1] * inv, acc[d + 2] * inv, acc[d + 3] * inv);
}

// ------------------------------------------------------------------------------------
// fp32 (fprop_dtype=float32, the reference's default precision) on v_mfma_f32_32x32x2f32, any S: the
// spatial attention (S = 256), other patch grids (S >= 128), long clips' temporal attention and the LvT
// auxiliary encoder (S = T*N).  Exact fp32 products summed in fp32; the numerators exp(cap * tanh(x / cap))
// from capped_exp_f32x16 (a few fp32 ulp from exp(cap tanh(x / cap))).  With 0 < cap <= 50 every capped logit lies in [-cap, cap],
// so the softmax needs no running max (the bf16 kernels' argument, vp_internal.h kMaxFastCap).
// A workgroup owns 256 queries of one (sequence, head), 8 waves x 32 queries; K and V stream through LDS in
// 128-key chunks, double-buffered (chunk c + 1's loads in flight in registers while chunk c is consumed; one
// barrier per chunk), rows padded to 68 floats so the b128 K reads and the b64 V reads are conflict-free.
// S^T = K.Q^T puts one query per lane column; the contraction index d is permuted per lane half
// (d = 32 (l / 32) + step) so a lane's K operands are 32 consecutive floats of its key row (numerators:
// capped_exp_f32x16).  O^T = V^T.P^T
// takes the numerators straight from the S^T accumulators: MFMA step r sums keys 8 (r / 4) + 4 (l / 32) + r % 4
// -- the keys register r of each lane half holds -- and output row i of block b is d = 2 i + b, so a lane's
// V operands are one 8-byte read.  Padded keys (MASK) weigh 0, a fully padded sequence gives uniform weights
// (as attn_f32_kernel); TAIL (S % 256 != 0): query and key rows past S read row S - 1, keys past S weigh 0,
// queries past S are not stored.
// ------------------------------------------------------------------------------------
// exp(cap * tanh(x / cap)) in fp32 for the 16 logits of a 32x32 tile (the MFMA kernel's numerators), accurate
// to a few fp32 ulp without the libm calls (≈ 14 VALU operations and one transcendental per logit instead of ≈ 56):
// cap tanh(x / cap) = x T(t^2), t = x / cap, with T(u) = tanh(sqrt u) / sqrt u fitted on u <= 0.55^2 by a
// degree-5 polynomial (relative error 9.4e-10; 4.6e-8 evaluated in fp32); tiles holding a larger |t| take
// tanh |t| = 1 - 2 / (e^{2|t|} + 1) there (no cancellation past 0.55: the result is >= 0.5; one Newton step on the
// reciprocal).  The exponential keeps the rounding error of g log2e: exp(g) = 2^p (1 + ln2 (g log2e - p)), the
// product's error recovered by an FMA against log2e split into fp32 hi + lo.  Emulated in fp32 against fp64 on
// |x| <= 200, cap 50: max relative error 5.4e-6 (rms 1.3e-6) vs 4.1e-6 (1.2e-6) for fp32 tanhf / expf -- both set by
// the fp32 rounding of cap tanh(.) itself, ~1.9e-6 of the exponent at 50.
__device__ __forceinline__ void capped_exp_f32x16(const f32x16& x, float* e, float cap, float inv_cap) {
  constexpr float c0 = 0.9999999990601012f, c1 = -0.33333310932806975f, c2 = 0.13332460381965514f,
                  c3 = -0.05384268765140977f, c4 = 0.021039637749701284f, c5 = -0.00623554674883513f;
  constexpr float kL = 1.4426950216293335f, kLlo = 1.92596298909109e-08f, kLn2 = 0.6931471805599453f;
  float mx = 0.0f;
#pragma unroll
  for (int i = 0; i < 16; ++i) mx = fmaxf(mx, fabsf(x[i]));
  const float xthr = 0.55f * cap, k2 = 2.0f * kL * inv_cap;
  const bool big = __builtin_amdgcn_ballot_w64(mx >= xthr) != 0;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const float t = x[i] * inv_cap;
    const float u = t * t;
    float P = fmaf(c5, u, c4);
    P = fmaf(P, u, c3);
    P = fmaf(P, u, c2);
    P = fmaf(P, u, c1);
    P = fmaf(P, u, c0);
    float g = x[i] * P;
    if (big) {
      const float a2 = fminf(fabsf(x[i]) * k2, 64.0f);  // 2 |t| log2e, clamped: e^{44} already gives tanh = 1
      const float d = __builtin_amdgcn_exp2f(a2) + 1.0f;
      const float r0 = __builtin_amdgcn_rcpf(d);
      const float r = fmaf(r0, fmaf(-d, r0, 1.0f), r0);
      const float gl = copysignf(cap * fmaf(-2.0f, r, 1.0f), x[i]);
      g = fabsf(x[i]) < xthr ? g : gl;
    }
    const float p = g * kL;
    const float lo = fmaf(g, kLlo, fmaf(g, kL, -p));
    const float E = __builtin_amdgcn_exp2f(p);
    e[i] = fmaf(E, lo * kLn2, E);
  }
}

constexpr int kF32Chunk = 128, kF32Row = 68;
constexpr int kF32BufFloats = 2 * kF32Chunk * kF32Row + kF32Chunk;  // K, V, key paddings of one chunk
constexpr int kF32MfmaLds = 2 * kF32BufFloats * 4 + 16;

template <bool MASK, bool TAIL>
__global__ __launch_bounds__(512) void attn_f32_mfma_kernel(const float* __restrict__ qkv, float* __restrict__ o,
                                                            int S, int heads, int nqb, float cap,
                                                            const float* __restrict__ key_pad) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* bufs = reinterpret_cast<float*>(smem);
  const int D = heads * 64;
  const int64_t ld = 3 * (int64_t)D;
  const int qb = blockIdx.x % nqb;
  const int sh = blockIdx.x / nqb;
  const int seq = sh / heads;
  const int h = sh % heads;
  const float* base = qkv + (int64_t)seq * S * ld + h * 64;
  const int t = threadIdx.x, lane = t & 63, w = wave_id();
  const int half = lane >> 5, l32 = lane & 31;
  const int q = qb * 256 + 32 * w + l32;

  // this wave's 32 queries as the B operand: lane l holds Q[q][32 (l / 32) + s], s = 0..31
  float qf[32];
  {
    const float* qp = base + (int64_t)(TAIL ? min(q, S - 1) : q) * ld + 32 * half;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float4 v = *reinterpret_cast<const float4*>(qp + 4 * i);
      qf[4 * i] = v.x; qf[4 * i + 1] = v.y; qf[4 * i + 2] = v.z; qf[4 * i + 3] = v.w;
    }
  }
  bool all_masked = false;
  if constexpr (MASK) {
    int valid = 0;
    for (int i = t; i < S; i += 512) valid |= key_pad[(int64_t)seq * S + i] == 0.0f;
    all_masked = __syncthreads_or(valid) == 0;
  }
  // chunk c: 128 key rows x 16 float4 of K and of V, 4 of each per thread (+ the chunk's key paddings)
  f32x4 kr[4], vr[4];  // (native vectors: arrays of HIP's float4 struct stay in scratch here)
  float pr = 0.0f;
  auto stage = [&](int c) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int idx = t + 512 * i, row = idx >> 4, c4 = (idx & 15) * 4;
      const int key = TAIL ? min(c * kF32Chunk + row, S - 1) : c * kF32Chunk + row;
      kr[i] = *reinterpret_cast<const f32x4*>(base + (int64_t)key * ld + D + c4);
      vr[i] = *reinterpret_cast<const f32x4*>(base + (int64_t)key * ld + 2 * D + c4);
    }
    if constexpr (MASK) {
      const int key = c * kF32Chunk + t;
      if (t < kF32Chunk) pr = key < S ? key_pad[(int64_t)seq * S + key] : 1.0f;
    }
  };
  auto store = [&](int c) __attribute__((always_inline)) {
    float* Kb = bufs + (c & 1) * kF32BufFloats;
    float* Vb = Kb + kF32Chunk * kF32Row;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int idx = t + 512 * i, row = idx >> 4, c4 = (idx & 15) * 4;
      *reinterpret_cast<f32x4*>(Kb + row * kF32Row + c4) = kr[i];
      *reinterpret_cast<f32x4*>(Vb + row * kF32Row + c4) = vr[i];
    }
    if constexpr (MASK) {
      if (t < kF32Chunk) Vb[kF32Chunk * kF32Row + t] = pr;
    }
  };

  f32x16 y0 = {}, y1 = {};  // O^T blocks b = 0 / 1: row i <-> d = 2 i + b
  float lsum = 0.0f;
  const float inv_cap = 1.0f / cap;
  const int nch = (S + kF32Chunk - 1) / kF32Chunk;
  stage(0);
  store(0);
  __syncthreads();
#pragma unroll 1
  for (int c = 0; c < nch; ++c) {
    if (c + 1 < nch) stage(c + 1);  // in flight while chunk c is consumed
    const float* Kb = bufs + (c & 1) * kF32BufFloats;
    const float* Vb = Kb + kF32Chunk * kF32Row;
    const float* kp = Vb + kF32Chunk * kF32Row;
#pragma unroll 1
    for (int kt = 0; kt < kF32Chunk / 32; ++kt) {
      // S^T tile: x[r] = logit(key c 128 + kt 32 + 8 (r / 4) + 4 half + r % 4, query q)
      f32x16 x = {};
      const float* kq = Kb + (kt * 32 + l32) * kF32Row + 32 * half;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float4 kv = *reinterpret_cast<const float4*>(kq + 4 * i);
        x = __builtin_amdgcn_mfma_f32_32x32x2f32(kv.x, qf[4 * i], x, 0, 0, 0);
        x = __builtin_amdgcn_mfma_f32_32x32x2f32(kv.y, qf[4 * i + 1], x, 0, 0, 0);
        x = __builtin_amdgcn_mfma_f32_32x32x2f32(kv.z, qf[4 * i + 2], x, 0, 0, 0);
        x = __builtin_amdgcn_mfma_f32_32x32x2f32(kv.w, qf[4 * i + 3], x, 0, 0, 0);
      }
      float ev[16];
      capped_exp_f32x16(x, ev, cap, inv_cap);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int kl = kt * 32 + 8 * (r >> 2) + 4 * half + (r & 3);  // key within the chunk
        float e = ev[r];
        if constexpr (MASK) e = all_masked ? 1.0f : (kp[kl] != 0.0f ? 0.0f : e);
        if constexpr (TAIL) e = c * kF32Chunk + kl < S ? e : 0.0f;
        lsum += e;
        const float2 vv = *reinterpret_cast<const float2*>(Vb + kl * kF32Row + 2 * l32);
        y0 = __builtin_amdgcn_mfma_f32_32x32x2f32(vv.x, e, y0, 0, 0, 0);
        y1 = __builtin_amdgcn_mfma_f32_32x32x2f32(vv.y, e, y1, 0, 0, 0);
      }
    }
    // buffer (c + 1) & 1 was last read in chunk c - 1, before the previous barrier
    if (c + 1 < nch) store(c + 1);
    __syncthreads();
  }
  lsum += __shfl_xor(lsum, 32);
  const float inv = 1.0f / lsum;
  if (TAIL && q >= S) return;
  // y_b[4 m + c] = O[q][d = 16 m + 8 half + 2 c + b]: 8 consecutive floats per m
  float* op = o + ((int64_t)seq * S + q) * D + h * 64 + 8 * half;
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    *reinterpret_cast<float4*>(op + 16 * m) =
        make_float4(y0[4 * m] * inv, y1[4 * m] * inv, y0[4 * m + 1] * inv, y1[4 * m + 1] * inv);
    *reinterpret_cast<float4*>(op + 16 * m + 4) =
        make_float4(y0[4 * m + 2] * inv, y1[4 * m + 2] * inv, y0[4 * m + 3] * inv, y1[4 * m + 3] * inv);
  }
}

}  // namespace

hipError_t attention_spatial_bf16(const bf16_t* qkv, bf16_t* o, int num_seq, int heads, float cap,
                                  const float* key_pad, hipStream_t s, bool blk) {
  if (!(cap > 0.0f)) return hipErrorInvalidValue;
  const int mi = (key_pad ? 1 : 0) + (blk ? 2 : 0);
  const void* fns[4] = {(const void*)attn_spatial_kernel<false, false>, (const void*)attn_spatial_kernel<true, false>,
                        (const void*)attn_spatial_kernel<false, true>, (const void*)attn_spatial_kernel<true, true>};
  const void* fn = fns[mi];
  hipError_t e = ensure_dyn_lds(fn, kSpLds);
  if (e != hipSuccess) return e;
  const dim3 grid(num_seq * heads);
  // frames in reverse order (the producing GEMM's last-written q|k|v rows first): 2.354-2.358 vs
  // 2.400-2.407 ms/step in the forward (round 3, one box, alternating; round 2 measured it neutral)
  const int rev = 1;
  // (a persistent variant -- one workgroup per CU walking (frame, head) pairs, next pair's
  // Q/K/V staged by LDS-DMA during the current one, 160 KiB LDS -- measured 255 vs 218 us: at
  // 2 waves per SIMD the softmax/P.V phase loses more than the continuous stream gains)
  // O leaves through LDS as whole 128-B row segments (217 -> 209 us at the bench shape); a
  // head-major q|k|v layout measured only 1 % faster and is not used
  const int64_t D = heads * 64;
  if (blk && (3 * D) % 32) return hipErrorInvalidValue;
  VP_NOTE_KERNEL(fn);
#define VP_SPATIAL(M, B)                                                                                        \
  hipLaunchKernelGGL((attn_spatial_kernel<M, B>), grid, dim3(kSpThreads), kSpLds, s, qkv, o, heads, cap, key_pad, \
                     rev, 3 * D, (int64_t)64, D)
  switch (mi) {
    case 0: VP_SPATIAL(false, false); break;
    case 1: VP_SPATIAL(true, false); break;
    case 2: VP_SPATIAL(false, true); break;
    default: VP_SPATIAL(true, true); break;
  }
#undef VP_SPATIAL
  return hipGetLastError();
}

hipError_t attention_temporal_bf16(const bf16_t* qkv, bf16_t* o, int num_seq, int S, int heads,
                                   float cap, const float* key_pad, hipStream_t s) {
  if (!(cap > 0.0f) || S < 1 || S > 16) return hipErrorInvalidValue;
  const int pairs = num_seq * heads;
  const dim3 grid((pairs + kTpWaves - 1) / kTpWaves);
  VP_NOTE_KERNEL(key_pad ? (const void*)attn_temporal_kernel<true> : (const void*)attn_temporal_kernel<false>);
  if (key_pad)
    hipLaunchKernelGGL(attn_temporal_kernel<true>, grid, dim3(kTpWaves * 64), 0, s, qkv, o, pairs, S, heads, cap, key_pad);
  else
    hipLaunchKernelGGL(attn_temporal_kernel<false>, grid, dim3(kTpWaves * 64), 0, s, qkv, o, pairs, S, heads, cap, key_pad);
  return hipGetLastError();
}

hipError_t attention_seq_bf16(const bf16_t* qkv, bf16_t* o, int num_seq, int S, int heads, float cap,
                              const float* key_pad, hipStream_t s, int causal) {
  if (!(cap > 0.0f) || S < 17 || S > kSpS || num_seq < 1) return hipErrorInvalidValue;
  const int Sp = S <= 32 ? 32 : S <= 64 ? 64 : S <= 128 ? 128 : 256;
  const int per = kSpS / Sp;
  const void* fn = key_pad ? (const void*)attn_seq_kernel<true> : (const void*)attn_seq_kernel<false>;
  hipError_t e = ensure_dyn_lds(fn, kSqLds);
  if (e != hipSuccess) return e;
  const int64_t grid = (int64_t)((num_seq + per - 1) / per) * heads;
  if (grid > 0x7fffffff) return hipErrorInvalidValue;
  VP_NOTE_KERNEL(fn);
  if (key_pad)
    hipLaunchKernelGGL(attn_seq_kernel<true>, dim3((unsigned)grid), dim3(kSpThreads), kSqLds, s, qkv, o, num_seq, S,
                       Sp, heads, cap, key_pad, causal);
  else
    hipLaunchKernelGGL(attn_seq_kernel<false>, dim3((unsigned)grid), dim3(kSpThreads), kSqLds, s, qkv, o, num_seq, S,
                       Sp, heads, cap, key_pad, causal);
  return hipGetLastError();
}

hipError_t attention_f32_mfma(const float* qkv, float* o, int num_seq, int S, int heads, float cap,
                              const float* key_pad, hipStream_t s) {
  if (!(cap > 0.0f && cap <= 50.0f)) return hipErrorNotSupported;
  if (S < 1 || num_seq < 1 || heads < 1) return hipErrorInvalidValue;
  const int nqb = (S + 255) / 256;
  const int64_t grid = (int64_t)num_seq * heads * nqb;
  if (grid > 0x7fffffff || (int64_t)num_seq * S > 0x7fffffff) return hipErrorInvalidValue;
  const int mi = (key_pad ? 1 : 0) + (S % 256 ? 2 : 0);
  const void* fns[4] = {(const void*)attn_f32_mfma_kernel<false, false>, (const void*)attn_f32_mfma_kernel<true, false>,
                        (const void*)attn_f32_mfma_kernel<false, true>, (const void*)attn_f32_mfma_kernel<true, true>};
  hipError_t e = ensure_dyn_lds(fns[mi], kF32MfmaLds);
  if (e != hipSuccess) return e;
  VP_NOTE_KERNEL(fns[mi]);
#define VP_F32M(M, T)                                                                                              \
  hipLaunchKernelGGL((attn_f32_mfma_kernel<M, T>), dim3((unsigned)grid), dim3(512), kF32MfmaLds, s, qkv, o, S, heads, \
                     nqb, cap, key_pad)
  switch (mi) {
    case 0: VP_F32M(false, false); break;
    case 1: VP_F32M(true, false); break;
    case 2: VP_F32M(false, true); break;
    default: VP_F32M(true, true); break;
  }
#undef VP_F32M
  return hipGetLastError();
}

hipError_t attention_f32(const float* qkv, float* o, int num_seq, int S, int heads, float cap,
                         const float* key_pad, hipStream_t s) {
  if (S < 1 || S > kF32MaxS) return hipErrorInvalidValue;
  if (S >= 128) {  // MFMA kernel (max-free softmax: 0 < cap <= 50); other caps fall through to the generic one
    const hipError_t e = attention_f32_mfma(qkv, o, num_seq, S, heads, cap, key_pad, s);
    if (e != hipErrorNotSupported) return e;
  }
  const int lds = (2 * S * 64 + S) * 4 + 16;
  hipError_t e = ensure_dyn_lds((const void*)attn_f32_kernel, (2 * kF32MaxS * 64 + kF32MaxS) * 4 + 16);
  if (e != hipSuccess) return e;
  VP_NOTE_KERNEL(attn_f32_kernel);
  hipLaunchKernelGGL(attn_f32_kernel, dim3(num_seq * heads), dim3(256), lds, s, qkv, o, S, heads, cap, key_pad);
  return hipGetLastError();
}

}  // namespace vp
