// bf16 GEMM, 4-wave decomposition (one wave per SIMD, 128x128 per wave), persistent.
//
//   C[M,N] = A[M,K] . W[N,K]^T  (+ epilogue), 256x256 tile, BK = 64, 256 threads.
//
// Why this shape on MI355X (measured with tools/gemm_bench.py):
//  * 8 waves of 128x64 (gemm_bf16.hip) read 2x the LDS bytes per FLOP of 4 waves of
//    128x128 and every staging instruction competes with the partner wave's MFMAs.  Here the
//    512-entry register file of a SIMD belongs to one wave: 256 fp32 accumulators (8x8
//    blocks of v_mfma_f32_16x16x32_bf16) in AGPRs, two fragment sets (k-halves) in VGPRs.
//  * Staging moves FULL 128-byte lines: a piece is 8 rows x 128 B (one K-tile of 8 rows),
//    loaded by buffer_load_dwordx4 ... lds (SGPR descriptor, constant per-lane voffset, tile
//    and K offsets in soffset).  Half-line (64 B) pieces measured 15-18% slower.
//  * Two 64 KiB K-tile buffers.  K-tile g is computed as two k-halves h0/h1 of 64 MFMAs:
//      h0: MFMAs on set 0, ds_read set 1 <- (g, h1)                      (no barrier)
//      h1: lgkmcnt(0) vmcnt(0) barrier; MFMAs on set 1, ds_read set 0 <- (g+1, h0),
//          16 loads of K-tile g+2 into buffer g&1 (free: its last reads retired before the
//          barrier).  Those loads have ~1.5 halves before the next h1 barrier waits on them
//          (a 2-half window measured as good as 3; 1 half costs 10%).
//  * 128-byte LDS rows, swizzle chunk ^= (row >> 1) & 7 applied on the global source (the
//    LDS-DMA image is lane-linear) and undone on the ds_read_b128 (conflict-free for the
//    16x16x32 operand reads).
//  * W is the MFMA A-operand, so each lane's accumulators hold 4 consecutive N columns of
//    one M row (8-byte bf16 / 16-byte fp32 stores), as in gemm_bf16.hip.
//  * The K-tile stream runs across the persistent workgroup's tiles: the next tile's first
//    K-tiles load during this tile's last K-tiles and epilogue.
//  * S3 variant (q|k|v, post and ffn_layer2 in the forward): a third A buffer lets each
//    K-tile's A pieces go out in the h0 of the K-tile two before it (W pieces stay in h1), so the
//    A stream the previous kernel just wrote gets 1.5 K-tiles of lead and the VMEM issue is spread
//    over both phases; the epilogue's scratch lives in the A buffer its last K-tile freed.
//  * Tile order: XCD-contiguous tile ranges; where W outgrows the XCD's L2 share the XCD sweeps
//    its M-blocks once per group of N-tiles (w4_ngrp), so a group's W stays L2-resident.
#pragma once
#include <cstdlib>
#include <type_traits>

#include "gemm_epilogue.h"

namespace vp {

namespace {

constexpr int BM = 256, BN = 256, BK = 64;
constexpr int kThreads = 256;
constexpr int kOp = BM * BK * 2;             // 32 KiB: one operand's K-tile
constexpr int kBuf = 2 * kOp;                // A then W
constexpr int kLds = 2 * kBuf;               // 128 KiB
// per-wave epilogue scratch: two buffers of 16 rows x 64 fp32 columns (256-B rows), 16-B
// chunk c of row r stored at chunk c ^ (r & 7) (conflict-free for the ds_write_b128 and
// ds_read_b128 patterns below, brute-force checked)
constexpr int kScrBuf = 16 * 256;
constexpr int kScr = 2 * kScrBuf;            // 8 KiB per wave
constexpr int kLdsTotal = kLds + 4 * kScr;   // 163840 B = all 160 KiB

__device__ __forceinline__ int swz(int row) { return (row >> 1) & 7; }


__device__ __forceinline__ void sched_fence() { __builtin_amdgcn_sched_barrier(0); }

typedef short w4_s16x4 __attribute__((ext_vector_type(4)));
// 4 bf16 of one LDS column (rows +0..3 of 16-bit element p) as an MFMA operand
__device__ __forceinline__ bf16x4 w4_tr_read(const char* p) {
  const w4_s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) w4_s16x4*)(p));
  return bf16x4{v[0], v[1], v[2], v[3]};
}

// NOPAD: the launch has no padded rows (rowpad == nullptr), so the (1 - rowpad) factor is skipped --
// bitwise the same result (ffn_layer1: 651.7 -> 639.5 us; the same build of the residual epilogues
// measured slower in the forward, a different compiler schedule, so only ffn_layer1 uses it).
// S3 (ffn_layer2, whose A -- the 805 MB hidden activation -- streams from HBM; also the q|k|v and
// post projections, whose A the previous kernel wrote with nontemporal stores): three
// 32 KiB A buffers and two W buffers (all 160 KiB).  A K-tile's A pieces are issued in the h0 of
// the K-tile two before it (into the A buffer freed by the K-tile before that), its W pieces in
// the h1, so A gets 1.5 K-tiles of lead and the 16 pieces are spread over both phases.  The
// epilogue's scratch is the A buffer of the tile's last K-tile, refilled by the next h0.
// Bitwise equal to the 2-stage kernel; ffn_layer2 (statistics epilogue) 501.8 -> 485.6 us isolated,
// 7.78 -> 7.48 ms/step in the forward.  (Three A stages with all 16 pieces in h1 measured 468 vs
// 475 us isolated and nothing in the forward; the lead time alone is not it -- spreading the
// pieces over both phases is.)
// AVID: A is the video itself (patch embedding without a patch tensor): bf16 frames
// [frames][16P][16P][3] of a 16x16 patch grid, so a 256-row tile is one frame and a piece's 8 rows
// are 8 horizontally adjacent patches -- their pixel-row segments are contiguous in the frame, so a
// piece instruction reads one 8 x 6P-byte run.  K-tile kt is patch pixel row kt (K = 64 P): its 3P
// channels-last values are read as 16-B chunks at value offsets 0, 8, .., and min(8 j, 3P - 8) for the
// row's last chunk j = cpr - 1 (cpr = ceil(3P / 8); it overlaps its predecessor instead of running
// into the next patch), chunk slots j >= cpr re-read chunk 0; W is zero at the overlap and in those
// slots, so no read leaves the patch's row segment.  The lane offsets are K-tile independent.  lda =
// the pixel-row length in elements (48 P); the buffer descriptor spans the M / 256 frames.
// ABL: ablation builds for the tools' diag library only (tools/diag/csrc/gemm_w4_abl.hip; results
// are garbage; the product library instantiates ABL = 0 only): 2 = no ds_reads in the K-loop,
// 4 = no staging loads after the prologue, 8 = no epilogue (stores skipped at run time; the
// accumulators stay live).

// the LN fold of 4 accumulator values (r * a + (m * c + b)) in packed pairs: two IEEE fmas per value
// (the scalar form is bitwise equal and measured no faster beside the fused epilogues' MFMAs:
// QK launch 250.9 vs 246.5 us, V launch 161.8 vs 159.0, profiles/HISTORY.md)
__device__ __forceinline__ void fold4(const f32x4& a, float r, float m, const float4& c, const float4& b, f32x2_t& lo,
                                      f32x2_t& hi) {
  const f32x2_t rr = f32x2_t(r), mm = f32x2_t(m);
  lo = __builtin_elementwise_fma(rr, f32x2_t{a[0], a[1]}, __builtin_elementwise_fma(mm, f32x2_t{c.x, c.y}, f32x2_t{b.x, b.y}));
  hi = __builtin_elementwise_fma(rr, f32x2_t{a[2], a[3]}, __builtin_elementwise_fma(mm, f32x2_t{c.z, c.w}, f32x2_t{b.z, b.w}));
}

template <int EPI, bool NOPAD, bool S3, int ABL = 0, bool AVID = false>
__global__ __launch_bounds__(kThreads, 1) void gemm_bf16_w4_kernel(
    const bf16_t* __restrict__ A, int64_t lda, const bf16_t* __restrict__ W, int64_t ldw, int M,
    int N, int K, int ngrp, EpiArgs ep) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tilesN = N / BN;
  const int T = (M / BM) * tilesN;
  // tile index -> (M-block, N-tile).  ngrp == tilesN: N-tile fastest.  ngrp < tilesN (host: only
  // when every XCD owns whole M-blocks): each XCD sweeps its M-blocks once per group of ngrp
  // N-tiles, so the group's W rows (<= 2.5 MB) stay in the XCD's 4 MiB L2 instead of the whole W
  // being re-fetched from beyond it for every M-block (ffn_layer1: W = 4.7 MB)
  auto coords = [&](int t, int& tm, int& tn) {
    if (ngrp == tilesN) {
      tm = t / tilesN;
      tn = t - tm * tilesN;
      return;
    }
    const int mbx = (M / BM) >> 3;
    const int x = t / (mbx * tilesN);
    const int u = t - x * mbx * tilesN;
    const int gsz = mbx * ngrp;
    const int gi = u / gsz, r = u - gi * gsz;
    const int rm = r / ngrp;
    tm = x * mbx + rm;
    tn = gi * ngrp + (r - rm * ngrp);
  };
  const int G = gridDim.x;
  const int b = blockIdx.x;
  int first, stride, count;
  if ((G & 7) == 0) {  // XCD x owns tiles [x*T/8, (x+1)*T/8), tn fastest
    const int xcd = b & 7, li = b >> 3, nx = G >> 3;
    const int lo = (int)(((int64_t)xcd * T) >> 3), hi = (int)(((int64_t)(xcd + 1) * T) >> 3);
    first = lo + li;
    stride = nx;
    count = first < hi ? (hi - first + nx - 1) / nx : 0;
  } else {
    first = b;
    stride = G;
    count = b < T ? (T - b + G - 1) / G : 0;
  }
  if (count == 0) return;
  const int lane = threadIdx.x & 63;
  const int w = wave_id();
  const int wm = w >> 1, wn = w & 1;
  const int nk = K / BK;
  const int total = count * nk;

  // ---- staging: wave w fills pieces w*8+i (i = 0..7) of A and of W; piece = 8 rows x 128 B.
  // Lane: row (lane>>3) of the piece, LDS chunk (lane&7) <- source chunk (lane&7)^swz(row);
  // swz(row) of piece i depends only on i & 1.
  const uint32_t a_rb = (uint32_t)(lda * 2), w_rb = (uint32_t)(ldw * 2);
  // AVID: a_rb = one pixel row of a frame (48 P values), 16 P pixel rows per frame, K-tile = one
  // patch pixel row of 3P values in cpr 16-B chunks
  const int av_p = AVID ? K / BK : 0;
  const int av_cpr = AVID ? (3 * av_p + 7) >> 3 : 1;
  const uint32_t prow_b = AVID ? (uint32_t)(6 * av_p) : 0;    // bytes of one patch's pixel row
  const uint32_t frame_b = AVID ? (uint32_t)(16 * av_p) * a_rb : 0;
  const uint64_t a_bytes = AVID ? (uint64_t)(M / BM) * frame_b : (uint64_t)M * a_rb;
  const uint64_t w_bytes = (uint64_t)N * w_rb;
  const auto rsA = __builtin_amdgcn_make_buffer_rsrc((void*)A, 0, (int)(uint32_t)a_bytes, 0x00020000);
  const auto rsW = __builtin_amdgcn_make_buffer_rsrc((void*)W, 0, (int)(uint32_t)w_bytes, 0x00020000);
  const int prow = lane >> 3;
  const uint32_t cE = (uint32_t)((lane & 7) ^ swz(prow)) * 16;       // even pieces
  const uint32_t cO = (uint32_t)((lane & 7) ^ swz(prow + 8)) * 16;   // odd pieces
  // AVID: logical chunk j = (lane & 7) ^ swz of a K-tile row -> value offset within the patch row
  auto video_off = [&](int par) -> uint32_t {
    const int jj = (lane & 7) ^ swz(prow + 8 * par);
    const int vo = jj >= av_cpr ? 0 : min(8 * jj, 3 * av_p - 8);
    return prow * prow_b + (uint32_t)vo * 2;
  };
  // ABLK (A = the row-blocked hidden activation [M/16][K/32][16][32]): logical chunk j of a piece row
  // is 16 B of column block j >> 2 (1 KiB apart), row (piece parity * 8 + prow) of the block (64 B)
  auto ablk_off = [&](int par) -> uint32_t {
    const uint32_t jj = (uint32_t)((lane & 7) ^ swz(prow + 8 * par));
    return (jj >> 2) * 1024u + (uint32_t)prow * 64u + (jj & 3u) * 16u;
  };
  constexpr bool ABLK = EpiTraits<EPI>::kABlk;
  const uint32_t vA[2] = {AVID ? video_off(0) : ABLK ? ablk_off(0) : prow * a_rb + cE,
                          AVID ? video_off(1) : ABLK ? ablk_off(1) : prow * a_rb + cO};
  const uint32_t vW[2] = {prow * w_rb + cE, prow * w_rb + cO};
  typedef __attribute__((address_space(3))) void lds_void;
  // load stream: K-tile ld_g -> (tile ld_tm/ld_tn, K-tile ld_kt); the tail re-loads the last
  // K-tile (harmless), so every wait count stays uniform
  int ld_g = 0, ld_kt = 0, ld_tile = first;
  int ld_tm, ld_tn;
  coords(ld_tile, ld_tm, ld_tn);
  auto advance = [&]() {
    if (ld_g + 1 >= total) return;
    ++ld_g;
    if (++ld_kt == nk) {
      ld_kt = 0;
      ld_tile += stride;
      coords(ld_tile, ld_tm, ld_tn);
    }
  };
  // LDS: 2 x [A | W] K-tile buffers; S3: A buffers 0..2 then W buffers 0..1
  auto a_buf = [&](int ai) { return smem + ai * (S3 ? kOp : kBuf); };
  auto w_buf = [&](int wi) { return smem + (S3 ? 3 * kOp + wi * kOp : wi * kBuf + kOp); };
  // p: 0..7 A pieces into A buffer `buf`, 8..15 W pieces into W buffer `buf`
  auto stage_piece = [&](int buf, int p) {
    const int i = p & 7;
    char* dst = (p >= 8 ? w_buf(buf) : a_buf(buf)) + (w * 8 + i) * 1024;
    if (p < 8) {
      uint32_t so;
      if constexpr (AVID) {  // piece w*8+i: patch-grid row (w*8+i) >> 1, patches 8 ((w*8+i) & 1) + 0..7
        const int pc = w * 8 + i;
        so = (uint32_t)ld_tm * frame_b + (uint32_t)((pc >> 1) * av_p + ld_kt) * a_rb + (uint32_t)(pc & 1) * 8 * prow_b;
      } else if constexpr (ABLK) {  // piece rows 8 pc .. +7: block row pc >> 1, half pc & 1; K-tile = blocks 2 kt, +1
        const int pc = w * 8 + i;
        so = (uint32_t)((ld_tm * 16 + (pc >> 1)) * (K >> 5) + 2 * ld_kt) * 1024u + (uint32_t)(pc & 1) * 512u;
      } else {
        so = (uint32_t)(ld_tm * BM + (w * 8 + i) * 8) * a_rb + ld_kt * (BK * 2);
      }
      if constexpr (EpiTraits<EPI>::kResidStream)  // aux 2: nt
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsA, (lds_void*)dst, 16, vA[i & 1], so, 0, 2);
      else
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsA, (lds_void*)dst, 16, vA[i & 1], so, 0, 0);
    } else {
      const uint32_t so = (uint32_t)(ld_tn * BN + (w * 8 + i) * 8) * w_rb + ld_kt * (BK * 2);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsW, (lds_void*)dst, 16, vW[i & 1], so, 0, 0);
    }
  };

  // ---- fragments: 16x16x32 operand = rows (lane&15), 16-byte chunk kh*4 + (lane>>4)
  const int frow = lane & 15;
  int aoff[2], woff[2];
#pragma unroll
  for (int kh = 0; kh < 2; ++kh) {
    const int ch = ((kh * 4 + (lane >> 4)) ^ swz(frow)) * 16;
    aoff[kh] = (wm * 128 + frow) * 128 + ch;
    woff[kh] = (wn * 128 + frow) * 128 + ch;
  }
  bf16x8 fa[2][8], fw[2][8];
  // fragment q of A (q < 8, A buffer ab) or W (W buffer wb), k-half `set`
  auto rd = [&](int set, int ab, int wb, int q) {
    if constexpr (ABL & 2) {
      asm volatile("" : "+v"(fa[set][q & 7]), "+v"(fw[set][q & 7]));
      return;
    }
    if (q < 8) fa[set][q] = *reinterpret_cast<const bf16x8*>(a_buf(ab) + aoff[set] + q * 2048);
    else fw[set][q - 8] = *reinterpret_cast<const bf16x8*>(w_buf(wb) + woff[set] + (q - 8) * 2048);
  };

  f32x4 acc[8][8];
  // the first k-half of every tile starts its accumulators from 0 (C = inline constant)
  auto mfma = [&](int set, int idx, bool zero) {  // idx = nt*8 + mt
    const int nt = idx >> 3, mt = idx & 7;
    acc[nt][mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
        fw[set][nt], fa[set][mt], zero ? f32x4{0.f, 0.f, 0.f, 0.f} : acc[nt][mt], 0, 0, 0);
  };

  // ---- prologue: K-tiles 0, 1 into buffers 0, 1; fragments of (0, h0)
#pragma unroll
  for (int p = 0; p < 16; ++p) stage_piece(0, p);
  advance();
#pragma unroll
  for (int p = 0; p < 16; ++p) stage_piece(1, p);
  advance();
  asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  sched_fence();
  __builtin_amdgcn_s_barrier();
  sched_fence();
#pragma unroll
  for (int q = 0; q < 16; ++q) rd(0, 0, 0, q);
  int a3 = 0;  // S3: A buffer of the K-tile being computed (g % 3)

  auto h0 = [&](int cb, bool zero) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    sched_fence();
    const int a_ld = a3 == 0 ? 2 : a3 - 1;  // S3: A buffer of K-tile g+2 (freed by K-tile g-1)
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      rd(1, S3 ? a3 : cb, cb, q);
      if constexpr (S3) {
        if (q < 8) stage_piece(a_ld, q);
      }
    }
#pragma unroll
    for (int idx = 0; idx < 64; ++idx) mfma(0, idx, zero);
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      if constexpr (S3) {
        if (q < 8) __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
      }
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
    }
    sched_fence();
  };
  // h1 of K-tile g (buffer cb): MFMAs set 1, reads of set 0 <- (g+1, h0) from buffer cb^1,
  // 16 loads of K-tile g+2 into buffer cb.  DEFER (the fused temporal launches' last K-tile of a
  // tile): the reads of set 0 are left to the end of the epilogue, so their 64 registers are free in it
  // EARLY (kEarly's last K-tile): 4 residual loads were issued after this K-tile's h0 pieces
  auto h1 = [&](int cb, auto DEFER, auto EARLY) {
    constexpr bool defer = decltype(DEFER)::value;
    constexpr bool early = decltype(EARLY)::value;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    // S3: K-tile g+1 has landed once all but this K-tile's h0 A pieces (of g+2) are done
    if constexpr (S3 && early) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
    else if constexpr (S3) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    sched_fence();
    mfma(1, 0, false);
    mfma(1, 1, false);
    sched_fence();
    __builtin_amdgcn_s_barrier();
    sched_fence();
    const int an = a3 == 2 ? 0 : a3 + 1;  // S3: A buffer of K-tile g+1
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      if constexpr (!defer) rd(0, S3 ? an : (cb ^ 1), cb ^ 1, q);
      if constexpr (S3) {
        if (q >= 8) stage_piece(cb, q);  // W of K-tile g+2 into W buffer cb
      } else if constexpr (!(ABL & 4)) {
        stage_piece(cb, q);
      }
    }
#pragma unroll
    for (int idx = 2; idx < 64; ++idx) mfma(1, idx, false);
#pragma unroll
    for (int q = 0; q < 15; ++q) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
    }
    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
    __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
    __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
    sched_fence();
    if constexpr (S3) a3 = an;
    advance();  // after the scheduled block: its branch must not split it
  };

  int g = 0;
  const int er = lane >> 3, es = lane & 7;  // epilogue read-back: row pass*8 + er, column segment es
  for (int j = 0; j < count; ++j) {
    // this tile's bias columns, requested before any of the tile's K-stream loads: vmcnt
    // retires in issue order, so a bias load issued in the epilogue would wait for the next
    // tile's prefetch
    float4 bl[2], bh[2];
    float4 cl[2], ch[2];  // EPI_*_LN: column sums of W'
    float2 rs[8][2];      // EPI_*_LN: (rstd, -mean*rstd) of rows mt*16 + pass*8 + er
    float2 rsb[8];        // EPI_GELU_BF16_LN_BLK: (rstd, -mean*rstd) of rows mt*16 + (lane & 15)
    // S3 epilogues with a bf16 residual (post, ffn_layer2): the residual rows of the first row block are
    // requested inside the tile's last K-tile (after its h0 staging loads, so h1's vmcnt(8) still
    // names that K-tile's pieces) and kept raw until the epilogue uses them -- their memory latency
    // overlaps the last K-tile's MFMAs instead of opening the epilogue
    constexpr bool kEarly = EpiTraits<EPI>::kResidBf16 && S3;
    uint4 exr[2][2][2];   // kEarly: raw residual [buffer][nh][pass]
    int m0t = 0, n0t = 0;  // kEarly: this tile's wave origin (the epilogue's m0, n0)
    float keepb[8];       // EPI_GELU_BF16_LN_BLK with padded rows: 1 - rowpad of the same rows
    {
      int ttm, ttn;
      coords(first + j * stride, ttm, ttn);
      m0t = ttm * BM + wm * 128;
      n0t = ttn * BN + wn * 128;
      const int nb = ttn * BN + wn * 128 + es * 8;
#pragma unroll
      for (int nh = 0; nh < 2; ++nh) {
        bl[nh] = *reinterpret_cast<const float4*>(ep.bias + nb + nh * 64);
        bh[nh] = *reinterpret_cast<const float4*>(ep.bias + nb + nh * 64 + 4);
      }
      if constexpr (EpiTraits<EPI>::kBlkOut) {
        const int rb = ttm * BM + wm * 128 + (lane & 15);
#pragma unroll
        for (int mt = 0; mt < 8; ++mt) {
          rsb[mt] = *reinterpret_cast<const float2*>(ep.ln_rs + 2 * (int64_t)(rb + mt * 16));
          if constexpr (EpiTraits<EPI>::kKeep && !NOPAD) keepb[mt] = 1.0f - ep.rowpad[rb + mt * 16];
        }
      }
      if constexpr (EpiTraits<EPI>::kLn) {  // (the fused temporal epilogues load theirs in the epilogue)
#pragma unroll
        for (int nh = 0; nh < 2; ++nh) {
          cl[nh] = *reinterpret_cast<const float4*>(ep.ln_c + nb + nh * 64);
          ch[nh] = *reinterpret_cast<const float4*>(ep.ln_c + nb + nh * 64 + 4);
        }
        const int mb = ttm * BM + wm * 128 + er;
#pragma unroll
        for (int mt = 0; mt < 8; ++mt)
#pragma unroll
          for (int pass = 0; pass < 2; ++pass)
            rs[mt][pass] = *reinterpret_cast<const float2*>(ep.ln_rs + 2 * (int64_t)(mb + mt * 16 + pass * 8));
      }
    }
    if constexpr (EpiTraits<EPI>::kVAttn || EpiTraits<EPI>::kQkAttn) {  // last K-tile peeled (K >= 2 BK)
      h0(g & 1, true);
      h1(g & 1, std::false_type{}, std::false_type{});
      ++g;
      for (int kt = 1; kt < nk - 1; ++kt, ++g) {
        h0(g & 1, false);
        h1(g & 1, std::false_type{}, std::false_type{});
      }
      h0(g & 1, false);
      h1(g & 1, std::true_type{}, std::false_type{});
      ++g;
    } else {
      auto fetch_raw = [&](int bsel, int mt) {
#pragma unroll
        for (int nh = 0; nh < 2; ++nh)
#pragma unroll
          for (int pass = 0; pass < 2; ++pass)
            exr[bsel][nh][pass] = *reinterpret_cast<const uint4*>(
                static_cast<const bf16_t*>(ep.resid) + (int64_t)(m0t + mt * 16 + pass * 8 + er) * ep.ldr + n0t +
                nh * 64 + es * 8);
      };
      h0(g & 1, true);
      h1(g & 1, std::false_type{}, std::false_type{});
      ++g;
      if constexpr (kEarly) {  // last K-tile peeled (the launcher checks K >= 2 BK)
        for (int kt = 1; kt < nk - 1; ++kt, ++g) {
          h0(g & 1, false);
          h1(g & 1, std::false_type{}, std::false_type{});
        }
        h0(g & 1, false);
        fetch_raw(0, 0);
        h1(g & 1, std::false_type{}, std::true_type{});
        ++g;
      } else {
        for (int kt = 1; kt < nk; ++kt, ++g) {
          h0(g & 1, false);
          h1(g & 1, std::false_type{}, std::false_type{});
        }
      }
    }

    // ---- epilogue of tile j.  acc[nt][mt] holds D[row mb + 16*mt][cols nb + 16*nt + 4*(lane>>4)
    // + 0..3] (row mb = m0 + wm*128 + (lane&15)).  Each 16-row x 64-column block goes through the
    // wave's LDS scratch so that a lane owns 8 consecutive columns of one row: every store and
    // residual load instruction then covers 8 rows x 128 B (bf16) -- full lines instead of
    // 16 rows x 32 B.  Same fp32 math and single rounding as the direct epilogue.
    if constexpr (ABL & 8) {
      if (ep.ldo != -12345) continue;  // never false at run time: keeps acc live, skips stores
    }
    int etm, etn;
    coords(first + j * stride, etm, etn);
    const int m0 = etm * BM + wm * 128, n0 = etn * BN + wn * 128;
    using Tr = EpiTraits<EPI>;
    // S3: the A buffer of the tile's last K-tile (free since its h1 barrier; refilled in the next h0)
    char* scr = (S3 ? a_buf(a3 == 0 ? 2 : a3 - 1) : smem + kLds) + w * kScr;
    if constexpr (Tr::kBlkOut) {
      // ---- ffn_layer1 / the spatial q|k|v projection into a row-blocked layout (vp_kernels.h
      // EPI_GELU_BF16_LN_BLK, EPI_BF16_LN_BLK): the LN fold (+ GELU) where the accumulators stand (lane: row r16 of block mt, W rows 16 nt + 4 g4 ..
      // +3), the same IEEE operations as the row-major epilogue; nt pair (2p, 2p+1) gives the lane 8
      // natural columns 32 p + 8 g4 .. +7 (host row permutation), stored as 16 B at row r16 of the
      // 1 KiB block (row block, column block) -- one whole block per store instruction
      int lid = lane;
      asm volatile("" : "+v"(lid));
      const int r16 = lid & 15, g4 = lid >> 4;
#pragma unroll
      for (int nt = 0; nt < 8; ++nt)
#pragma unroll
        for (int mt = 0; mt < 8; ++mt) asm volatile("" : "+a"(acc[nt][mt]));
      char* lc = scr;  // c at +0, b' at +512 (the wave's 128 W rows)
      {
        const float* src = (lid < 32 ? ep.ln_c : ep.bias) + n0 + 4 * (lid & 31);
        *reinterpret_cast<float4*>(lc + (lid < 32 ? 0 : 512) + 16 * (lid & 31)) = *reinterpret_cast<const float4*>(src);
      }
      const int64_t nblk = N >> 5;
      bf16_t* outp = static_cast<bf16_t*>(ep.out);
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        const float4 c0 = *reinterpret_cast<const float4*>(lc + 4 * (32 * p + 4 * g4));
        const float4 c1 = *reinterpret_cast<const float4*>(lc + 4 * (32 * p + 16 + 4 * g4));
        const float4 b0 = *reinterpret_cast<const float4*>(lc + 512 + 4 * (32 * p + 4 * g4));
        const float4 b1 = *reinterpret_cast<const float4*>(lc + 512 + 4 * (32 * p + 16 + 4 * g4));
#pragma unroll
        for (int mt = 0; mt < 8; ++mt) {
          f32x2_t v[4];
          fold4(acc[2 * p][mt], rsb[mt].x, rsb[mt].y, c0, b0, v[0], v[1]);
          fold4(acc[2 * p + 1][mt], rsb[mt].x, rsb[mt].y, c1, b1, v[2], v[3]);
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            if constexpr (Tr::kGelu) v[q] = gelu_fast2(v[q]);
            if constexpr (Tr::kKeep && !NOPAD) v[q] = v[q] * f32x2_t(keepb[mt]);
          }
          const uint4 pk = make_uint4(pack_bf16x2(v[0].x, v[0].y), pack_bf16x2(v[1].x, v[1].y),
                                      pack_bf16x2(v[2].x, v[2].y), pack_bf16x2(v[3].x, v[3].y));
          const int64_t blk = (int64_t)((m0 >> 4) + mt) * nblk + ((n0 >> 5) + p);
          st_nt(outp + blk * 512 + r16 * 32 + 8 * g4, pk);
          __builtin_amdgcn_sched_barrier(0);  // one block's accumulator reads at a time
        }
      }
      continue;  // nothing else of this tile is stored
    }
    if constexpr (Tr::kQkAttn || Tr::kVAttn) {
      // ---- fused temporal attention (EPI_QK_TATTN_LN / EPI_V_TATTN_LN, see vp_kernels.h).  A
      // 16-row block mt of this wave's 128 rows is one (b n) sequence of T = 16 frames; the
      // wave's 128 columns are [q_h | k_h] of one head (QK launch) or v of two heads (V launch).
      // q, k, v are LN-folded and rounded to bf16 as the reference's bf16 projections are. ----
      // lane-derived addresses of these epilogues are computed here, per tile, from an opaque copy
      // of the lane id: hoisted out of the tile loop (the compiler's choice) they would all stay
      // live through the K-loop next to the fragment registers and spill
      int lid = lane;
      asm volatile("" : "+v"(lid));
      const int r16 = lid & 15, g4 = lid >> 4;
      // The accumulators stay in AGPRs through the K-loop: both epilogues read them with VALU where
      // they stand, and without this the allocator gives some of them VGPR homes and the K-loop's
      // fragment registers no longer fit (the QK launch spilled 5 VGPRs to scratch)
#pragma unroll
      for (int nt = 0; nt < 8; ++nt)
#pragma unroll
        for (int mt = 0; mt < 8; ++mt) asm volatile("" : "+a"(acc[nt][mt]));
      if constexpr (Tr::kQkAttn) {
        // logits^T = K Q^T (16x16x32 on the accumulator-layout operands, d in two halves), capped
        // softmax over the 16 keys in fp32, the normalised probabilities rounded to bf16 (the
        // reference's probs.astype(fprop)) and stored as this lane's P^T fragment: keys
        // 4*g4 .. +3 of query r16, 512 B per (sequence, head).  The LN fold runs on the
        // accumulators where they stand (lane: row mt*16 + r16, columns 16 nt + 4 g4 + 0..3), so
        // the operands need no LDS round trip: MFMA k-slot 8*g4 + i <-> column 16*(nt + (i >= 4)) +
        // 4*g4 + (i & 3), the same map on both operands of a dot product, which leaves it
        // unchanged.  The logits are summed over two 32-column halves of d (the LN constants of 4
        // blocks live at a time: 266 us per launch vs 301 with the scratch round trip).
        // The 8 sequences go in two groups of 4, so only 4 logit tiles are live next to the LN
        // constants, and the row statistics (rstd, -mean*rstd) of the accumulator rows are read here
        // rather than held through the K-loop (the first form spilled 5 VGPRs to scratch; the
        // constants are re-read per group from L1).
        const float c1 = ep.cap_c1, c2 = ep.cap_c2;
        const int head = n0 >> 7;
        const uint32_t lane_off = (uint32_t)lid * 8u;  // this lane's 8 B of a 512-B P block
        // the LN-fold constants of the wave's 128 columns go to LDS once (c at +0, b' at +512 of the
        // wave's scratch) and are read per k-half from there (global reads per k-half waited behind
        // the next tile's staging loads); the row statistics of all 8 sequences are read up front
        char* lc = scr;
        {
          const float* src = (lid < 32 ? ep.ln_c : ep.bias) + n0 + 4 * (lid & 31);
          *reinterpret_cast<float4*>(lc + (lid < 32 ? 0 : 512) + 16 * (lid & 31)) =
              *reinterpret_cast<const float4*>(src);
        }
        float2 rsA[8];  // (rstd, -mean*rstd) of rows mt*16 + (lane & 15)
#pragma unroll
        for (int mt = 0; mt < 8; ++mt)
          rsA[mt] = *reinterpret_cast<const float2*>(ep.ln_rs + 2 * (int64_t)(m0 + mt * 16 + (lane & 15)));
#pragma unroll
        for (int mh = 0; mh < 2; ++mh) {
          float4 cc[4], bb[4];
#pragma unroll
          for (int kk = 0; kk < 2; ++kk) {
#pragma unroll
            for (int hh = 0; hh < 2; ++hh)  // cc/bb[2*hh + i]: block 2kk + i of q (hh = 0) / k (hh = 1)
#pragma unroll
              for (int i = 0; i < 2; ++i) {
                const int cofs = 4 * (hh * 64 + 16 * (2 * kk + i) + 4 * g4);
                cc[2 * hh + i] = *reinterpret_cast<const float4*>(lc + cofs);
                bb[2 * hh + i] = *reinterpret_cast<const float4*>(lc + 512 + cofs);
              }
#pragma unroll
            for (int ml = 0; ml < 4; ++ml) {
              const int mt = mh * 4 + ml;
              auto fold2blk = [&](int hh) {  // operand of blocks (hh*4 + 2kk, +1), constants cc/bb[2hh..]
                uint32_t u[4];
#pragma unroll
                for (int i = 0; i < 2; ++i) {
                  f32x2_t lo, hi;
                  fold4(acc[hh * 4 + 2 * kk + i][mt], rsA[mt].x, rsA[mt].y, cc[2 * hh + i], bb[2 * hh + i], lo, hi);
                  u[2 * i] = pack_bf16x2(lo.x, lo.y);
                  u[2 * i + 1] = pack_bf16x2(hi.x, hi.y);
                }
                return *reinterpret_cast<const bf16x8*>(u);
              };
              // the logits accumulate in acc[0][mt] (q block 0, consumed at kk = 0), so they take
              // no registers beyond the accumulators (separate logit tiles spilled 5 VGPRs)
              acc[0][mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fold2blk(1), fold2blk(0),
                                                                   kk ? acc[0][mt] : f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
              __builtin_amdgcn_sched_barrier(0);  // one sequence's accumulator reads at a time
            }
            __builtin_amdgcn_sched_barrier(0);
          }
#pragma unroll
          for (int ml = 0; ml < 4; ++ml) {
            const int mt = mh * 4 + ml;
            // acc[0][mt][r] = logit[query r16][key 4*g4 + r]
            float p[4], lsum = 0.f;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              p[r] = capped_exp_exact(acc[0][mt][r], c1, c2);
              lsum += p[r];
            }
            lsum += __shfl_xor(lsum, 16);
            lsum += __shfl_xor(lsum, 32);
            const float inv = 1.0f / lsum;
            const int64_t sq = (int64_t)(m0 + mt * 16) >> 4;
            char* pblk = static_cast<char*>(ep.out) + (sq * ep.heads + head) * 512;  // wave-uniform
            *reinterpret_cast<uint2*>(pblk + lane_off) =
                make_uint2(pack_bf16x2(p[0] * inv, p[1] * inv), pack_bf16x2(p[2] * inv, p[3] * inv));
          }
        }
#pragma unroll
        for (int q = 0; q < 16; ++q) rd(0, a3, g & 1, q);  // the next tile's first fragments (deferred)
        continue;  // nothing else of this tile is stored
      } else {
        // O^T = V^T . P^T per (sequence mt, head nh) on 16x16x16 MFMAs: A = V^T by transposed
        // reads of the bf16 V block, B = this lane's P^T fragment; the result lands in the
        // accumulator layout (lane: query r16, d = 16 dt + 4 g4 + r) and replaces v there, so the
        // store path below writes O with whole-line stores.  One LDS pass: v is LN-folded where the
        // accumulators stand (lane: row r16, columns 16 q + 4 g4 .. +3 of block q), rounded to bf16
        // and written row-major with one ds_write_b64 per block into a 2 KiB V block whose 8-byte
        // units are swizzled by row (unit ^ (((row >> 1) & 3) << 2): conflict-free for these writes
        // and for the transposed reads, which read 8 B of one row per lane and so see the swizzle
        // only in their addresses).  (The first form took v through the fp32 scratch and back:
        // 168 us per launch at the bench shape.)
        const bf16_t* pin = static_cast<const bf16_t*>(ep.resid);
        const int trq = r16 >> 2, trp = r16 & 3;
        auto vunit = [](int row, int u) { return row * 128 + ((u ^ (((row >> 1) & 3) << 2)) << 3); };
        // the LN-fold constants of the wave's 128 columns go to LDS once (c at +4 KiB, b' at +4.5 KiB
        // of the wave's scratch) and are read into registers per head
        char* lc = scr + 4096;
        {
          const float* src = (lid < 32 ? ep.ln_c : ep.bias) + n0 + 4 * (lid & 31);
          *reinterpret_cast<float4*>(lc + (lid < 32 ? 0 : 512) + 16 * (lid & 31)) =
              *reinterpret_cast<const float4*>(src);
        }
        // P^T fragment of (sequence mt, head nh), two (sequence, head) steps ahead of its use, and
        // (rstd, -mean*rstd) of rows mt*16 + r16 (both heads)
        auto ld_p = [&](int st) {
          const int64_t sq = (int64_t)(m0 + (st & 7) * 16) >> 4;
          return *reinterpret_cast<const bf16x4*>(pin + (sq * ep.heads + ((n0 + (st >> 3) * 64) >> 6)) * 256 + lid * 4);
        };
        float2 rsv[8];
#pragma unroll
        for (int mt = 0; mt < 8; ++mt) rsv[mt] = *reinterpret_cast<const float2*>(ep.ln_rs + 2 * (int64_t)(m0 + mt * 16 + r16));
        bf16x4 pbq[2] = {ld_p(0), ld_p(1)};
        float4 cc[4], bb[4];
        auto ld_consts = [&](int nh) {
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int cofs = 4 * (nh * 64 + 16 * q + 4 * g4);
            cc[q] = *reinterpret_cast<const float4*>(lc + cofs);
            bb[q] = *reinterpret_cast<const float4*>(lc + 512 + cofs);
          }
        };
        // step st = (head st >> 3, sequence st & 7): v LN-folded, rounded and written to V block st & 1
        auto fold_write = [&](int st) {
          const int nh = st >> 3, mt = st & 7;
          char* vb = scr + (st & 1) * 2048;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            f32x2_t lo, hi;
            fold4(acc[nh * 4 + q][mt], rsv[mt].x, rsv[mt].y, cc[q], bb[q], lo, hi);
            *reinterpret_cast<uint2*>(vb + vunit(r16, 4 * q + g4)) = make_uint2(pack_bf16x2(lo.x, lo.y), pack_bf16x2(hi.x, hi.y));
          }
        };
        // software-pipelined over the 16 steps: the transposed reads of step st are issued, then step
        // st+1's block is folded and written (LDS executes one wave's operations in order, so no wait
        // separates a block's writes from its reads), then step st's MFMAs wait for their reads only
        ld_consts(0);
        fold_write(0);
#pragma unroll
        for (int st = 0; st < 16; ++st) {
          const int nh = st >> 3, mt = st & 7;
          const char* vb = scr + (st & 1) * 2048;
          bf16x4 vf[4];
#pragma unroll
          for (int dt = 0; dt < 4; ++dt) vf[dt] = w4_tr_read(vb + vunit(4 * g4 + trq, 4 * dt + trp));
          if (st + 1 < 16) {
            if (st + 1 == 8) ld_consts(1);
            fold_write(st + 1);
          }
          const bf16x4 pb = pbq[st & 1];
          if (st + 2 < 16) pbq[st & 1] = ld_p(st + 2);
#pragma unroll
          for (int dt = 0; dt < 4; ++dt)
            acc[nh * 4 + dt][mt] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(vf[dt], pb, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
    }
    // residual / position rows of block mt+1 are requested before block mt's stores, so a
    // load never waits behind the stores just issued (vmcnt retires in issue order)
    F8 ex[2][2][2];  // [buffer][nh][pass] (kEarly: exr, raw)
    auto fetch = [&](int bsel, int mt) {
#pragma unroll
      for (int nh = 0; nh < 2; ++nh)
#pragma unroll
        for (int pass = 0; pass < 2; ++pass) {
          if constexpr (kEarly)
            exr[bsel][nh][pass] = *reinterpret_cast<const uint4*>(
                static_cast<const bf16_t*>(ep.resid) + (int64_t)(m0 + mt * 16 + pass * 8 + er) * ep.ldr + n0 + nh * 64 +
                es * 8);
          else
            ex[bsel][nh][pass] = epi_extra8<EPI>(ep, m0 + mt * 16 + pass * 8 + er, n0 + nh * 64 + es * 8, N);
        }
    };
    // block G = (mt, nh): acc[nh*4 + q][mt], q = 0..3 -> scratch buffer G & 1.  Block G+1 is
    // written before block G is read back, so the LDS round trip overlaps the math and stores.
    auto put = [&](int G) {
      const int mt = G >> 1, nh = G & 1;
      char* sb = scr + (G & 1) * kScrBuf + frow * 256;
#pragma unroll
      for (int q = 0; q < 4; ++q)
        *reinterpret_cast<f32x4*>(sb + (((q * 4 + (lane >> 4)) ^ (frow & 7)) << 4)) = acc[nh * 4 + q][mt];
    };
    // EPI_*_ST: the stored row values of block (mt, nh=0), then per (mt, pass) the row's
    // partial over this wave's 128 columns: sum and sum of squares about the partial mean
    // (two passes over the 16 values a lane holds, each reduced over the row's 8 lanes); lane
    // es keeps the partials of mt == es, so the wave stores its 128 rows with 2 instructions
    float sv[2][8];
    float pS[2] = {0.f, 0.f}, pQ[2] = {0.f, 0.f};
    if constexpr (Tr::kExtra && !kEarly) fetch(0, 0);
    put(0);
#pragma unroll
    for (int G = 0; G < 16; ++G) {
      const int mt = G >> 1, nh = G & 1;
      if (G + 1 < 16) put(G + 1);
      if constexpr (Tr::kExtra) {
        if (nh == 0 && mt < 7) fetch((mt + 1) & 1, mt + 1);
      }
#pragma unroll
      for (int pass = 0; pass < 2; ++pass) {
        const int rl = pass * 8 + er;
        const int row = m0 + mt * 16 + rl;
        const int n = n0 + nh * 64 + es * 8;
        const char* sb = scr + (G & 1) * kScrBuf + rl * 256;
        F8 v;
        v.lo = *reinterpret_cast<const float4*>(sb + (((2 * es) ^ (rl & 7)) << 4));
        v.hi = *reinterpret_cast<const float4*>(sb + (((2 * es + 1) ^ (rl & 7)) << 4));
        if constexpr (Tr::kLn) {  // LN(x) . W + b = rstd * (x . W') - mean*rstd * c + b'
          // packed pairs (v_pk_fma_f32): the same two roundings per value as the scalar form
          const f32x2_t r = f32x2_t(rs[mt][pass].x), q = f32x2_t(rs[mt][pass].y);
          auto fold2 = [&](float& x0, float& x1, float c0, float c1, float b0, float b1) {
            const f32x2_t o = __builtin_elementwise_fma(
                r, f32x2_t{x0, x1}, __builtin_elementwise_fma(q, f32x2_t{c0, c1}, f32x2_t{b0, b1}));
            x0 = o.x;
            x1 = o.y;
          };
          fold2(v.lo.x, v.lo.y, cl[nh].x, cl[nh].y, bl[nh].x, bl[nh].y);
          fold2(v.lo.z, v.lo.w, cl[nh].z, cl[nh].w, bl[nh].z, bl[nh].w);
          fold2(v.hi.x, v.hi.y, ch[nh].x, ch[nh].y, bh[nh].x, bh[nh].y);
          fold2(v.hi.z, v.hi.w, ch[nh].z, ch[nh].w, bh[nh].z, bh[nh].w);
        } else if constexpr (!Tr::kVAttn) {  // (fused V launch: the values are O already)
          v.lo.x += bl[nh].x; v.lo.y += bl[nh].y; v.lo.z += bl[nh].z; v.lo.w += bl[nh].w;
          v.hi.x += bh[nh].x; v.hi.y += bh[nh].y; v.hi.z += bh[nh].z; v.hi.w += bh[nh].w;
        }
        float keep = 1.0f;
        if constexpr (Tr::kKeep && !NOPAD) {
          if (ep.rowpad) keep = 1.0f - ep.rowpad[row];
        }
        {
          F8 e;
          if constexpr (kEarly) {  // the same conversion as epi_extra8
            const uint4 u = exr[mt & 1][nh][pass];
            e.lo = bf16x4_to_f32(make_uint2(u.x, u.y));
            e.hi = bf16x4_to_f32(make_uint2(u.z, u.w));
          } else {
            e = ex[mt & 1][nh][pass];
          }
          const epi_u32x4 pk = epi_store8<EPI, !Tr::kResidStream, !NOPAD>(ep, row, n, v, keep, e);
          if constexpr (Tr::kStats) {
            float y[8];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              y[2 * i] = __uint_as_float(pk[i] << 16);
              y[2 * i + 1] = __uint_as_float(pk[i] & 0xffff0000u);
            }
            if (nh == 0) {
#pragma unroll
              for (int i = 0; i < 8; ++i) sv[pass][i] = y[i];
            } else {
              float s0 = 0.f;
#pragma unroll
              for (int i = 0; i < 8; ++i) s0 += sv[pass][i] + y[i];
              const float S = sum8_lanes(s0);
              const float mp = S * (1.0f / 128.0f);
              float q0 = 0.f;
#pragma unroll
              for (int i = 0; i < 8; ++i) {
                const float a = sv[pass][i] - mp, b2 = y[i] - mp;
                q0 = fmaf(a, a, fmaf(b2, b2, q0));
              }
              const float Q = sum8_lanes(q0);
              if (es == mt) { pS[pass] = S; pQ[pass] = Q; }
            }
          }
        }
      }
    }
    if constexpr (Tr::kStats) {
      const int p = (n0 >> 7);  // 128-column partial index of this wave
      float* dst = ep.st_part + 2 * ((int64_t)p * ep.st_rows + m0 + es * 16 + er);
#pragma unroll
      for (int pass = 0; pass < 2; ++pass) *reinterpret_cast<float2*>(dst + 16 * pass) = make_float2(pS[pass], pQ[pass]);
    }
    if constexpr (EpiTraits<EPI>::kVAttn) {  // the next tile's first fragments, deferred by its last h1
      // (also after the last tile, where they are not used: a conditional read would keep the
      // K-loop's stale set-0 registers live through the epilogue on the other path)
#pragma unroll
      for (int q = 0; q < 16; ++q) rd(0, a3, g & 1, q);
    }
  }
  // drain the tail's (clamped) loads before the workgroup's LDS is released
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

int num_cus_w4() { return device_cu_count(); }  // per device (vp_common.h)

template <int EPI, bool NOPAD, bool S3, int ABL = 0, bool AVID = false>
hipError_t launch_w4(const bf16_t* A, int64_t lda, const bf16_t* W, int64_t ldw, int M, int N,
                     int K, const EpiArgs& ep, hipStream_t s) {
  hipError_t e = ensure_dyn_lds((const void*)gemm_bf16_w4_kernel<EPI, NOPAD, S3, ABL, AVID>, kLdsTotal);
  if (e != hipSuccess) return e;
  const int tiles = (M / BM) * (N / BN);
  const int grid = tiles < num_cus_w4() ? tiles : num_cus_w4();
  const int ngrp = w4_ngrp(M, N, K, grid);
  VP_NOTE_KERNEL((gemm_bf16_w4_kernel<EPI, NOPAD, S3, ABL, AVID>));
  hipLaunchKernelGGL((gemm_bf16_w4_kernel<EPI, NOPAD, S3, ABL, AVID>), dim3(grid), dim3(kThreads), kLdsTotal, s, A, lda,
                     W, ldw, M, N, K, ngrp, ep);
  return hipGetLastError();
}

}  // namespace

}  // namespace vp
