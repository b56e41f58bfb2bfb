// Fused q|k|v projection + spatial attention for the bf16 encoder (one launch per spatial layer).
//
// STATUS: diag library only (tools/qa_bench.py).  Bitwise equal to the unfused pair but measured
// no faster at B=32 (fused 659 us vs gemm_bf16_w4 + attn_spatial_kernel 651 us in isolation;
// in the forward 8.13 vs 7.56 ms/step): with two 56 KiB K-tile buffers the K-stream keeps one
// K-tile in flight and is latency-bound (~1.2 us per K-tile with no MFMAs at all: 350 us per
// layer for staging, fragment reads, hand-off and O stores), and the capped-softmax VALU at one
// wave per SIMD costs ~7 us per (frame, head) (172 us per layer).
//
// Replaces, per (frame, head):  q|k|v = LN1(x) . Wqkv + b   (layers.py:208-270, :433-499, the
// fused [3D][D] GEMM of vp_finalize with LN1 folded into its epilogue, gemm_bf16_w4 EPI_BF16_LN)
// and  o = softmax(cap*tanh(q.k^T / cap)) . v   (layers.py:586-661, attn_spatial_kernel).
// The unfused path writes the 604 MB q|k|v tensor of a B=32 layer to HBM in the GEMM's epilogue
// burst and streams it back in the attention kernel (HBM-bound at ~4 TB/s); here a frame's 192
// q|k|v columns of one head never leave the CU: the GEMM's accumulators go through the LN fold
// into LDS and the attention runs from there.
//
// Results are bitwise those of the unfused pair: the GEMM accumulates the same k32 steps in the
// same order with v_mfma_f32_16x16x32_bf16 and applies the same packed fp32 LN fold and single
// bf16 rounding; the attention is attn_spatial_kernel's per-32-query arithmetic (exact capped
// numerator, the same key order for the row sums, the same P.V MFMAs and output rounding).
//
// Layout and schedule (one persistent 256-thread workgroup per CU, one wave per SIMD):
//  * item = (frame f, head h); the 8 XCDs own contiguous item ranges (the 12 heads of a frame
//    share its 384 KiB A panel in that XCD's L2).
//  * GEMM tile 256 tokens x 192 columns (q, k, v of head h), K = 768 in 12 K-tiles of 64:
//    4 waves as 2 (tokens) x 2 (columns), 128 x 96 per wave = 6 x 8 blocks of 16x16x32 (192
//    accumulators); two 56 KiB K-tile buffers R0/R1, pieces of 8 rows x 128 B by
//    buffer_load_dwordx4 ... lds with the chunk ^ ((row >> 1) & 7) swizzle of gemm_bf16_w4, and
//    its h0/h1 k-half pipeline.
//  * hand-off: acc -> rstd*acc + (-mean*rstd*c + b') -> bf16 -> Q [120K, 152K), K [56K, 88K),
//    V [88K, 120K) (128-B token rows, the attention kernel's swizzles); the next item's K-tile 0
//    streams into R0 meanwhile.
//  * attention: wave w owns queries 64w .. 64w+63 as two 32-query groups that share every K
//    fragment and transposed V read; O is staged through the wave's own Q rows and leaves as
//    whole 128-B row segments after the next item's K-tile 1 loads have been issued (so the
//    next item's K-stream waits never wait behind these stores).
#include <cstdlib>
#include <type_traits>

#include "gemm_epilogue.h"

namespace vp {

namespace {

constexpr int kQaThreads = 256;
constexpr int kQaOpA = 256 * 128;          // 32 KiB: A K-tile (256 tokens x 64 k)
constexpr int kQaOpW = 192 * 128;          // 24 KiB: W K-tile (192 columns x 64 k)
constexpr int kQaBuf = kQaOpA + kQaOpW;    // 56 KiB
constexpr int kQaK = kQaBuf;               // 56 KiB: K [256][64] bf16
constexpr int kQaV = kQaK + 32768;         // 88 KiB
constexpr int kQaQ = kQaV + 32768;         // 120 KiB
constexpr int kQaC = kQaQ + 32768;         // 152 KiB: LN constants c'[192], b'[192], (rstd, -mean*rstd)[256]
constexpr int kQaLds = kQaC + 192 * 8 + 256 * 8;  // 159232 B
constexpr int kQaNk = 12;                  // K = 768 in K-tiles of 64
constexpr int kQaOStores = 8;              // 16-B O stores per lane per item

__device__ __forceinline__ int swzA(int row) { return (row >> 1) & 7; }   // GEMM operands, Q, K
__device__ __forceinline__ int swzV(int row) { return ((row >> 1) & 1) << 2; }
__device__ __forceinline__ void qa_fence() { __builtin_amdgcn_sched_barrier(0); }

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4_nt __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void store_nt16(bf16_t* p, uint4 v) {
  __builtin_nontemporal_store(u32x4_nt{v.x, v.y, v.z, v.w}, reinterpret_cast<u32x4_nt*>(p));
}

template <int DIAG = 0>
__global__ __launch_bounds__(kQaThreads, 1) void qkv_attn_spatial_kernel(
    const bf16_t* __restrict__ X, const float* __restrict__ ln_rs, const bf16_t* __restrict__ Wqkv,
    const float* __restrict__ bias, const float* __restrict__ lnc, bf16_t* __restrict__ O, int frames,
    int heads, float cap) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int D = heads * 64;
  const int items = frames * heads;
  const int G = gridDim.x, b = blockIdx.x;
  int first, stride, count;
  if ((G & 7) == 0) {  // XCD x owns items [x*I/8, (x+1)*I/8)
    const int xcd = b & 7, li = b >> 3, nx = G >> 3;
    const int lo = (int)(((int64_t)xcd * items) >> 3), hi = (int)(((int64_t)(xcd + 1) * items) >> 3);
    first = lo + li;
    stride = nx;
    count = first < hi ? (hi - first + nx - 1) / nx : 0;
  } else {
    first = b;
    stride = G;
    count = b < items ? (items - b + G - 1) / G : 0;
  }
  if (count == 0) return;
  const int lane = threadIdx.x & 63;
  const int w = wave_id();
  const int wm = w >> 1, wn = w & 1;

  // ---- staging (gemm_bf16_w4's scheme): wave w fills A pieces w*8+i (i < 8) and W pieces
  // w*6+i (i < 6); piece = 8 rows x 128 B; lane: row lane>>3, LDS chunk lane&7 <- source chunk
  // (lane&7) ^ swzA(row), which depends only on the piece's parity
  const uint32_t rb = (uint32_t)D * 2;  // A and W rows are both D elements
  const auto rsA = __builtin_amdgcn_make_buffer_rsrc((void*)X, 0, (int)(uint32_t)((uint64_t)frames * 256 * rb), 0x00020000);
  const auto rsW = __builtin_amdgcn_make_buffer_rsrc((void*)Wqkv, 0, (int)(uint32_t)((uint64_t)3 * D * rb), 0x00020000);
  const int prow = lane >> 3;
  const uint32_t cE = (uint32_t)((lane & 7) ^ swzA(prow)) * 16;
  const uint32_t cO = (uint32_t)((lane & 7) ^ swzA(prow + 8)) * 16;
  const uint32_t vo[2] = {prow * rb + cE, prow * rb + cO};
  typedef __attribute__((address_space(3))) void lds_void;
  auto stage_ktile = [&](int buf, int item, int kt) {  // 14 VMEM ops per lane
    const int f = item / heads, h = item - f * heads;
    char* base = smem + buf * kQaBuf;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int q = w * 8 + i;
      const uint32_t so = (uint32_t)(f * 256 + q * 8) * rb + kt * 128;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsA, (lds_void*)(base + q * 1024), 16, vo[i & 1], so, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < 6; ++i) {
      const int q = w * 6 + i;  // tile rows q*8 .. +7: section q>>3 (q, k, v), head dims (q&7)*8 ..
      const uint32_t so = (uint32_t)((q >> 3) * D + h * 64 + (q & 7) * 8) * rb + kt * 128;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsW, (lds_void*)(base + kQaOpA + q * 1024), 16, vo[i & 1], so, 0, 0);
    }
  };

  // ---- GEMM fragments: 16x16x32 operand = rows (lane&15), 16-byte chunk kh*4 + (lane>>4)
  const int frow = lane & 15;
  int aoff[2], woff[2];
#pragma unroll
  for (int kh = 0; kh < 2; ++kh) {
    const int ch = ((kh * 4 + (lane >> 4)) ^ swzA(frow)) * 16;
    aoff[kh] = (wm * 128 + frow) * 128 + ch;
    woff[kh] = kQaOpA + (wn * 96 + frow) * 128 + ch;
  }
  bf16x8 fa[2][8], fw[2][6];
  auto rd = [&](int set, int buf, int q) {  // q < 8: A fragment q, else W fragment q-8
    const char* base = smem + buf * kQaBuf;
    if (q < 8) fa[set][q] = *reinterpret_cast<const bf16x8*>(base + aoff[set] + q * 2048);
    else fw[set][q - 8] = *reinterpret_cast<const bf16x8*>(base + woff[set] + (q - 8) * 2048);
  };
  f32x4 acc[6][8];
  auto mfma = [&](int set, int idx, bool zero) {  // idx = nt*8 + mt
    const int nt = idx >> 3, mt = idx & 7;
    if constexpr (DIAG & 2) {
      asm volatile("" : "+v"(fw[set][nt]), "+v"(fa[set][mt]));
      if (zero) acc[nt][mt] = f32x4{0.f, 0.f, 0.f, 0.f};
      return;
    }
    acc[nt][mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
        fw[set][nt], fa[set][mt], zero ? f32x4{0.f, 0.f, 0.f, 0.f} : acc[nt][mt], 0, 0, 0);
  };
  auto h0 = [&](int cb, bool zero) {  // MFMAs on set 0, reads of set 1 (same K-tile)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    qa_fence();
#pragma unroll
    for (int q = 0; q < 14; ++q) rd(1, cb, q);
#pragma unroll
    for (int idx = 0; idx < 48; ++idx) mfma(0, idx, zero);
#pragma unroll
    for (int q = 0; q < 14; ++q) {
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
    }
    __builtin_amdgcn_sched_group_barrier(0x008, 6, 0);
    qa_fence();
  };
  // h1 of K-tile kt (buffer cb): wait until K-tile kt+1 has landed, barrier, MFMAs on set 1,
  // reads of set 0 <- (kt+1) from cb^1 (RD), loads of K-tile kt+2 -- or of the next item's
  // K-tile 0 at kt = 11 -- into cb (LD)
  bool o_pending = false;
  auto h1 = [&](int cb, int ldi, int ldk, auto wait_tag, auto rd_tag, auto ld_tag) {
    constexpr int kWait = decltype(wait_tag)::value;  // vmcnt(kWait); < 0: none
    constexpr bool RD = decltype(rd_tag)::value, LD = decltype(ld_tag)::value;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if constexpr (kWait == 1) {  // K-tile 0 of an item: the previous item's O stores are younger than K-tile 1
      if (o_pending) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kQaOStores) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else if constexpr (kWait >= 0) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kWait) : "memory");
    }
    qa_fence();
    mfma(1, 0, false);
    mfma(1, 1, false);
    qa_fence();
    __builtin_amdgcn_s_barrier();
    qa_fence();
    if constexpr (RD) {
#pragma unroll
      for (int q = 0; q < 14; ++q) rd(0, cb ^ 1, q);
    }
    if constexpr (LD) {  // kt <= 9: K-tile kt+2 into cb; kt = 11: the next item's K-tile 0 into R0
      if (ldi >= 0) stage_ktile(ldk == 0 ? 0 : cb, ldi, ldk);
    }
#pragma unroll
    for (int idx = 2; idx < 48; ++idx) mfma(1, idx, false);
    if constexpr (RD && LD) {
#pragma unroll
      for (int q = 0; q < 14; ++q) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      }
      __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
    } else if constexpr (RD) {
#pragma unroll
      for (int q = 0; q < 14; ++q) {
        __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      }
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
    }
    qa_fence();
  };
  using W0 = std::integral_constant<int, 0>;
  using WNone = std::integral_constant<int, -1>;
  using WO = std::integral_constant<int, 1>;  // see kWait == 1
  using T = std::integral_constant<bool, true>;
  using F = std::integral_constant<bool, false>;

  // ---- attention constants and lane roles (attn_spatial_kernel's)
  const float c1 = 2.0f * 1.4426950408889634f / cap;
  const float c2 = cap * 1.4426950408889634f;
  const int half = lane >> 5;
  const int krow_l = lane & 31;
  const int g16 = lane >> 4;
  const int trq = (lane & 15) >> 2, trp = lane & 3;
  char* const Ks = smem + kQaK;
  char* const Vs = smem + kQaV;
  char* const Qs = smem + kQaQ;

  // ---- LN constants of an item: thread t holds c'/b' of tile column t (t < 192) and the
  // (rstd, -mean*rstd) of token t; written to LDS at the item's start
  float lc = 0.f, lb = 0.f;
  float2 lr = make_float2(0.f, 0.f);
  const int tid = threadIdx.x;
  auto ln_fetch = [&](int it) {
    const int f = it / heads, h = it - f * heads;
    if (tid < 192) {
      const int gcol = (tid >> 6) * D + h * 64 + (tid & 63);
      lc = lnc[gcol];
      lb = bias[gcol];
    }
    lr = *reinterpret_cast<const float2*>(ln_rs + 2 * ((int64_t)f * 256 + tid));
  };
  float* const Cs = reinterpret_cast<float*>(smem + kQaC);  // c'[192] b'[192] rs[256][2]

  // ---- prologue: K-tile 0 of the first item into R0, its LN constants
  stage_ktile(0, first, 0);
  ln_fetch(first);

  for (int j = 0; j < count; ++j) {
    const int item = first + j * stride;
    const int f = item / heads, h = item - f * heads;
    const int next = j + 1 < count ? item + stride : -1;
    if (tid < 192) {
      Cs[tid] = lc;
      Cs[192 + tid] = lb;
    }
    *reinterpret_cast<float2*>(Cs + 384 + 2 * tid) = lr;
    // K-tile 1 -> R1 (free: the previous item's K/V reads ended before the barrier below)
    stage_ktile(1, item, 1);
    qa_fence();
    if (j > 0) {
      // O of the previous item (staged in this wave's own Q rows at the end of its attention):
      // whole 128-B row segments, issued after the K-tile 1 loads so the K-stream waits never
      // wait behind these stores
      const char* st = Qs + w * 64 * 128;
      const int pitem = item - stride;
      const int pf = pitem / heads, ph = pitem - pf * heads;
#pragma unroll
      for (int p = 0; p < 8; ++p) {
        const int r = p * 8 + (lane >> 3), c = lane & 7;
        const uint4 v = *reinterpret_cast<const uint4*>(st + r * 128 + ((c ^ (r & 7)) << 4));
        store_nt16(O + ((int64_t)pf * 256 + w * 64 + r) * D + ph * 64 + c * 8, v);
      }
      qa_fence();
      // K-tile 0 (loaded during the previous attention) has landed: the 14 K-tile 1 loads and
      // the 8 O stores are younger
      asm volatile("s_waitcnt vmcnt(22)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(14)" ::: "memory");
    }
    qa_fence();
    __builtin_amdgcn_s_barrier();
    qa_fence();
#pragma unroll
    for (int q = 0; q < 14; ++q) rd(0, 0, q);

    // ---- GEMM: 12 K-tiles, buffer kt & 1
    h0(0, true);
    o_pending = j > 0;
    h1(0, item, 2, WO{}, T{}, T{});
    for (int kt = 1; kt < 10; ++kt) {
      h0(kt & 1, false);
      h1(kt & 1, item, kt + 2, W0{}, T{}, T{});
    }
    h0(0, false);                                  // kt = 10
    h1(0, -1, 0, W0{}, T{}, F{});
    // the next item's LN constants (4 values per thread, written to LDS at its start)
    if (next >= 0) ln_fetch(next);
    h0(1, false);                                  // kt = 11: the next item's K-tile 0 -> R0
    h1(1, next, 0, WNone{}, F{}, T{});

    // ---- hand-off: LN fold, bf16, into Q / K / V.  acc[nt][mt]: token wm*128 + 16mt + (lane&15),
    // tile columns wn*96 + 16nt + 4(lane>>4) + 0..3 (one section: 4 | 64)
    float2 rsv[8];
#pragma unroll
    for (int mt = 0; mt < 8; ++mt) rsv[mt] = *reinterpret_cast<const float2*>(Cs + 384 + 2 * (wm * 128 + mt * 16 + frow));
#pragma unroll
    for (int nt = 0; nt < 6; ++nt) {
      const int col = wn * 96 + nt * 16 + 4 * g16;
      const int sec = col >> 6, d = col & 63;
      char* reg = smem + (sec == 0 ? kQaQ : sec == 1 ? kQaK : kQaV);
      const float4 ccv = *reinterpret_cast<const float4*>(Cs + col);
      const float4 bbv = *reinterpret_cast<const float4*>(Cs + 192 + col);
#pragma unroll
      for (int mt = 0; mt < 8; ++mt) {
        const int t = wm * 128 + mt * 16 + frow;
        const f32x2_t r = f32x2_t(rsv[mt].x), qv = f32x2_t(rsv[mt].y);
        const f32x4 a = acc[nt][mt];
        const f32x2_t o01 = __builtin_elementwise_fma(
            r, f32x2_t{a[0], a[1]}, __builtin_elementwise_fma(qv, f32x2_t{ccv.x, ccv.y}, f32x2_t{bbv.x, bbv.y}));
        const f32x2_t o23 = __builtin_elementwise_fma(
            r, f32x2_t{a[2], a[3]}, __builtin_elementwise_fma(qv, f32x2_t{ccv.z, ccv.w}, f32x2_t{bbv.z, bbv.w}));
        const int sw = sec == 2 ? swzV(t) : swzA(t);
        *reinterpret_cast<uint2*>(reg + t * 128 + (((d >> 3) ^ sw) << 4) + (d & 7) * 2) =
            make_uint2(pack_bf16x2(o01.x, o01.y), pack_bf16x2(o23.x, o23.y));
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    qa_fence();
    __builtin_amdgcn_s_barrier();
    qa_fence();

    // ---- attention: queries 64w + 32g2 + (lane&31); keys in tiles of 32
    bf16x8 qf[2][4];
#pragma unroll
    for (int g2 = 0; g2 < 2; ++g2) {
      const int qr = w * 64 + g2 * 32 + krow_l;
#pragma unroll
      for (int kd = 0; kd < 4; ++kd)
        qf[g2][kd] = *reinterpret_cast<const bf16x8*>(Qs + qr * 128 + (((2 * kd + half) ^ swzA(qr)) << 4));
    }
    float lsum[2] = {0.f, 0.f};
    f32x16 y[2][2];
#pragma unroll
    for (int g2 = 0; g2 < 2; ++g2) y[g2][0] = y[g2][1] = f32x16{};
#pragma unroll 1
    for (int kt = 0; kt < ((DIAG & 1) ? 0 : 8); ++kt) {
      f32x16 x[2] = {f32x16{}, f32x16{}};
      const int krow = kt * 32 + krow_l;
#pragma unroll
      for (int kd = 0; kd < 4; ++kd) {
        const int c = 2 * kd + half;
        const bf16x8 kf = *reinterpret_cast<const bf16x8*>(Ks + krow * 128 + ((c ^ swzA(krow)) << 4));
        x[0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[0][kd], x[0], 0, 0, 0);
        x[1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[1][kd], x[1], 0, 0, 0);
      }
      bf16x8 pf[2][2];
#pragma unroll
      for (int g2 = 0; g2 < 2; ++g2) {
        float p[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          p[i] = capped_exp_exact(x[g2][i], c1, c2);
          lsum[g2] += p[i];
        }
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          uint32_t u[4];
#pragma unroll
          for (int jj = 0; jj < 4; ++jj) u[jj] = pack_bf16x2(p[8 * s + 2 * jj], p[8 * s + 2 * jj + 1]);
          pf[g2][s] = *reinterpret_cast<bf16x8*>(u);
        }
      }
      // O^T += V^T . P^T (V^T by transposed reads, shared by both query groups)
      s16x4 vr[2][2][2];
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int key = kt * 32 + 16 * s + 4 * half + trq;
#pragma unroll
        for (int dh = 0; dh < 2; ++dh) {
          const int col = 32 * dh + 16 * (g16 & 1) + 4 * trp;
          const int c = col >> 3;
          const char* ad = Vs + key * 128 + ((c ^ swzV(key)) << 4) + (col & 7) * 2;
          vr[s][dh][0] = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(ad));
          vr[s][dh][1] = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(ad + 1024));
        }
      }
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int dh = 0; dh < 2; ++dh) {
          const s16x4 lo = vr[s][dh][0], hi = vr[s][dh][1];
          const bf16x8 vf = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
#pragma unroll
          for (int g2 = 0; g2 < 2; ++g2) y[g2][dh] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, pf[g2][s], y[g2][dh], 0, 0, 0);
        }
    }
    // O^T: y[g2][dh][i] = O[q = 64w + 32g2 + (lane&31)][d = 32dh + (i&3) + 8(i>>2) + 4*half] * lsum;
    // staged into this wave's own Q rows ([q][16-B chunk ^ (q & 7)]), stored at the next item's start
    {
      char* st = Qs + w * 64 * 128;
      const int ql = lane & 31;
#pragma unroll
      for (int g2 = 0; g2 < 2; ++g2) {
        const float inv = 1.0f / (lsum[g2] + __shfl_xor(lsum[g2], 32));
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          const int r = g2 * 32 + ql;
          const uint2 v0 = make_uint2(pack_bf16x2(y[g2][0][4 * g4] * inv, y[g2][0][4 * g4 + 1] * inv),
                                      pack_bf16x2(y[g2][0][4 * g4 + 2] * inv, y[g2][0][4 * g4 + 3] * inv));
          const uint2 v1 = make_uint2(pack_bf16x2(y[g2][1][4 * g4] * inv, y[g2][1][4 * g4 + 1] * inv),
                                      pack_bf16x2(y[g2][1][4 * g4 + 2] * inv, y[g2][1][4 * g4 + 3] * inv));
          *reinterpret_cast<uint2*>(st + r * 128 + ((g4 ^ (r & 7)) << 4) + 8 * half) = v0;
          *reinterpret_cast<uint2*>(st + r * 128 + (((4 + g4) ^ (r & 7)) << 4) + 8 * half) = v1;
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    // every wave is done with K / V before the next item's K-tile 1 lands in R1
    qa_fence();
    __builtin_amdgcn_s_barrier();
    qa_fence();
  }
  // O of the last item (staged like the others)
  {
    const int item = first + (count - 1) * stride;
    const int f = item / heads, h = item - f * heads;
    const char* st = Qs + w * 64 * 128;
#pragma unroll
    for (int p = 0; p < 8; ++p) {
      const int r = p * 8 + (lane >> 3), c = lane & 7;
      const uint4 v = *reinterpret_cast<const uint4*>(st + r * 128 + ((c ^ (r & 7)) << 4));
      store_nt16(O + ((int64_t)f * 256 + w * 64 + r) * D + h * 64 + c * 8, v);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

int num_cus_qa() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
  }
  return n;
}

}  // namespace

bool qkv_attention_spatial_ok(int frames, int heads, float cap) {
  const int64_t D = (int64_t)heads * 64;
  return frames > 0 && heads > 0 && cap > 0.0f && D == 768 &&
         (uint64_t)frames * 256 * D * 2 < 0xFFFFFFF0ull && (uint64_t)3 * D * D * 2 < 0xFFFFFFF0ull;
}

hipError_t qkv_attention_spatial_bf16(const bf16_t* x, const float* ln_rs, const bf16_t* wqkv, const float* bias,
                                      const float* lnc, bf16_t* o, int frames, int heads, float cap,
                                      hipStream_t s) {
  if (!qkv_attention_spatial_ok(frames, heads, cap)) return hipErrorInvalidValue;
  static bool attr = false;
  if (!attr) {
    hipError_t e = hipFuncSetAttribute((const void*)qkv_attn_spatial_kernel<0>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, kQaLds);
    if (e != hipSuccess) return e;
    attr = true;
  }
  const int items = frames * heads;
  const int grid = items < num_cus_qa() ? items : num_cus_qa();
  VP_NOTE_KERNEL(qkv_attn_spatial_kernel<0>);
  hipLaunchKernelGGL(qkv_attn_spatial_kernel<0>, dim3(grid), dim3(kQaThreads), kQaLds, s, x, ln_rs, wqkv, bias,
                     lnc, o, frames, heads, cap);
  return hipGetLastError();
}

#ifdef VP_DIAG
// ablation builds (tools/qa_bench.py; results garbage): 1 = no attention key loop, 2 = no GEMM MFMAs
hipError_t qkv_attention_spatial_diag(int diag, const bf16_t* x, const float* ln_rs, const bf16_t* wqkv,
                                      const float* bias, const float* lnc, bf16_t* o, int frames, int heads,
                                      float cap, hipStream_t s) {
  auto go = [&](const void* fn, auto kern) {
    hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, kQaLds);
    if (e != hipSuccess) return e;
    const int items = frames * heads;
    const int grid = items < num_cus_qa() ? items : num_cus_qa();
    hipLaunchKernelGGL(kern, dim3(grid), dim3(kQaThreads), kQaLds, s, x, ln_rs, wqkv, bias, lnc, o, frames, heads, cap);
    return hipGetLastError();
  };
  switch (diag) {
    case 1: return go((const void*)qkv_attn_spatial_kernel<1>, qkv_attn_spatial_kernel<1>);
    case 2: return go((const void*)qkv_attn_spatial_kernel<2>, qkv_attn_spatial_kernel<2>);
    case 3: return go((const void*)qkv_attn_spatial_kernel<3>, qkv_attn_spatial_kernel<3>);
  }
  return hipErrorInvalidValue;
}
#endif

}  // namespace vp
