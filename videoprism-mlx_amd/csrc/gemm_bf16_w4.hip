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
#include <cstdlib>

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

// DIAG (ablation builds for tools/gemm_bench.py only; results are garbage): 2 = no ds_reads
// in the K loop, 4 = no staging loads after the prologue, 8 = no epilogue (stores skipped at
// run time; the accumulators stay live), 16 = after an epilogue the next barrier waits vmcnt(32)
// (lets the stores drain behind the next tile; correct, measured no faster), 32 = epilogue
// without its global stores (LDS transposition and math kept), 64 = start skew: workgroup
// group (b>>3) % G of every XCD waits group * d before its first K-tile (G, d from
// ep.pos_rows), so the tiles' epilogue store bursts do not coincide across the chip, 128 = h1
// schedule with the 16 loads and 16 reads in its first 32 MFMAs, 256 = plain (temporal) output stores,
// 512 (production) = no padded rows: the epilogue skips the (1 - rowpad) factor, 1024 = GELU in
// unpacked fp32 arithmetic (A/B), 2048 / 4096 = epilogue without the LDS transposition's
// writes / read-backs.
// PF > 0: L2 prefetch of A, PF K-tiles beyond the K-tile being staged (one dword per A row per
// K-tile, the youngest VMEM op of an h1, so the next h1 waits vmcnt(1)).  ffn_layer2, K = 3072:
// 490 -> 471 us; costs on the K = 768 shapes (A mostly from the Infinity Cache).  Superseded for
// K >= 2048 by S3 (below; A/B build only).
// S3 (ffn_layer2, whose A -- the 805 MB hidden activation -- streams from HBM; also the q|k|v and
// post projections, whose A the previous kernel wrote with nontemporal stores): three
// 32 KiB A buffers and two W buffers (all 160 KiB).  A K-tile's A pieces are issued in the h0 of
// the K-tile two before it (into the A buffer freed by the K-tile before that), its W pieces in
// the h1, so A gets 1.5 K-tiles of lead and the 16 pieces are spread over both phases.  The
// epilogue's scratch is the A buffer of the tile's last K-tile, refilled by the next h0.
// Bitwise equal to the 2-stage kernel; ffn_layer2 (statistics epilogue) 501.8 -> 485.6 us isolated,
// 7.78 -> 7.48 ms/step in the forward (tools/gemm_bench.py s3).  (Three A stages with all 16
// pieces in h1 measured 468 vs 475 us isolated and nothing in the forward; the lead time alone is
// not it -- spreading the pieces over both phases is.)
template <int EPI, int DIAG = 0, int PF = 0, bool S3 = false>
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
    if (ngrp < 0) {  // A/B (diag): XCD pairs -- XCD x sweeps the M-blocks of pair x/2 over N-tile half x&1
      const int per = T >> 3, hn = tilesN >> 1;
      const int x = t / per, u = t - x * per;
      const int rm = u / hn;
      tm = (x >> 1) * ((M / BM) >> 2) + rm;
      tn = (x & 1) * hn + (u - rm * hn);
      return;
    }
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
  const uint64_t a_bytes = (uint64_t)M * a_rb, w_bytes = (uint64_t)N * w_rb;
  const auto rsA = __builtin_amdgcn_make_buffer_rsrc((void*)A, 0, (int)(uint32_t)a_bytes, 0x00020000);
  const auto rsW = __builtin_amdgcn_make_buffer_rsrc((void*)W, 0, (int)(uint32_t)w_bytes, 0x00020000);
  const int prow = lane >> 3;
  const uint32_t cE = (uint32_t)((lane & 7) ^ swz(prow)) * 16;       // even pieces
  const uint32_t cO = (uint32_t)((lane & 7) ^ swz(prow + 8)) * 16;   // odd pieces
  const uint32_t vA[2] = {prow * a_rb + cE, prow * a_rb + cO};
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
      const uint32_t so = (uint32_t)(ld_tm * BM + (w * 8 + i) * 8) * a_rb + ld_kt * (BK * 2);
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
    if constexpr (DIAG & 2) {
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

  uint32_t pf_dummy = 0;  // PF: destination of the L2-prefetch loads (never read)
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
  // 16 loads of K-tile g+2 into buffer cb
  // after_epi (DIAG 16): the tile's epilogue issued >= 32 VMEM ops (its stores) after the
  // K-stream loads this barrier needs, so vmcnt(32) retires those loads and lets the stores
  // drain behind the next tile's MFMAs
  auto h1 = [&](int cb, bool after_epi) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    // S3: K-tile g+1 has landed once all but this K-tile's h0 A pieces (of g+2) are done
    if constexpr (S3) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if (after_epi) asm volatile("s_waitcnt vmcnt(32)" ::: "memory");
    else if constexpr (PF > 0) asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
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
      rd(0, S3 ? an : (cb ^ 1), cb ^ 1, q);
      if constexpr (S3) {
        if (q >= 8) stage_piece(cb, q);  // W of K-tile g+2 into W buffer cb
      } else if constexpr (!(DIAG & 4)) {
        stage_piece(cb, q);
      }
    }
#pragma unroll
    for (int idx = 2; idx < 64; ++idx) mfma(1, idx, false);
    if constexpr (DIAG & 128) {  // front-loaded: loads and reads within the first 32 MFMAs
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      }
    } else {
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
    }
    sched_fence();
    if constexpr (PF > 0) {
      // L2 prefetch of A for K-tile (load position + PF); past the row end it touches the next
      // row (or returns 0 beyond the buffer): harmless
      const uint32_t voff = (uint32_t)(ld_tm * BM + w * 64 + lane) * a_rb + (ld_kt + PF) * (BK * 2);
      asm volatile("buffer_load_dword %0, %1, %2, 0 offen" : "+v"(pf_dummy) : "v"(voff), "s"(rsA));
      sched_fence();
    }
    if constexpr (S3) a3 = an;
    advance();  // after the scheduled block: its branch must not split it
  };

  int g = 0;
  if constexpr (DIAG & 64) {
    // ep.pos_rows (unused by EPI_BF16) = groups * 10000 + delay per group in 10-ns ticks
    const int ng = ep.pos_rows / 10000 > 0 ? ep.pos_rows / 10000 : 1;
    const uint64_t ticks = (uint64_t)((b >> 3) % ng) * (uint64_t)(ep.pos_rows % 10000);  // s_memrealtime: 100 MHz
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(2);
  }
  const int er = lane >> 3, es = lane & 7;  // epilogue read-back: row pass*8 + er, column segment es
  for (int j = 0; j < count; ++j) {
    // this tile's bias columns, requested before any of the tile's K-stream loads: vmcnt
    // retires in issue order, so a bias load issued in the epilogue would wait for the next
    // tile's prefetch
    float4 bl[2], bh[2];
    float4 cl[2], ch[2];  // EPI_*_LN: column sums of W'
    float2 rs[8][2];      // EPI_*_LN: (rstd, -mean*rstd) of rows mt*16 + pass*8 + er
    float2 rsA[8];        // EPI_*_TATTN_LN: the same for the accumulator rows mt*16 + (lane & 15)
    {
      int ttm, ttn;
      coords(first + j * stride, ttm, ttn);
      const int nb = ttn * BN + wn * 128 + es * 8;
#pragma unroll
      for (int nh = 0; nh < 2; ++nh) {
        bl[nh] = *reinterpret_cast<const float4*>(ep.bias + nb + nh * 64);
        bh[nh] = *reinterpret_cast<const float4*>(ep.bias + nb + nh * 64 + 4);
      }
      if constexpr (EpiTraits<EPI>::kQkAttn) {
        const int mb = ttm * BM + wm * 128 + (lane & 15);
#pragma unroll
        for (int mt = 0; mt < 8; ++mt)
          rsA[mt] = *reinterpret_cast<const float2*>(ep.ln_rs + 2 * (int64_t)(mb + mt * 16));
      } else if constexpr (EpiTraits<EPI>::kLnVals) {
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
    h0(g & 1, true);
    h1(g & 1, (DIAG & 16) && j > 0);
    ++g;
    for (int kt = 1; kt < nk; ++kt, ++g) {
      h0(g & 1, false);
      h1(g & 1, false);
    }

    // ---- epilogue of tile j.  acc[nt][mt] holds D[row mb + 16*mt][cols nb + 16*nt + 4*(lane>>4)
    // + 0..3] (row mb = m0 + wm*128 + (lane&15)).  Each 16-row x 64-column block goes through the
    // wave's LDS scratch so that a lane owns 8 consecutive columns of one row: every store and
    // residual load instruction then covers 8 rows x 128 B (bf16) -- full lines instead of
    // 16 rows x 32 B.  Same fp32 math and single rounding as the direct epilogue.
    if constexpr (DIAG & 8) {
      if (ep.ldo != -12345) continue;  // never false at run time: keeps acc live, skips stores
    }
    int etm, etn;
    coords(first + j * stride, etm, etn);
    const int m0 = etm * BM + wm * 128, n0 = etn * BN + wn * 128;
    using Tr = EpiTraits<EPI>;
    // S3: the A buffer of the tile's last K-tile (free since its h1 barrier; refilled in the next h0)
    char* scr = (S3 ? a_buf(a3 == 0 ? 2 : a3 - 1) : smem + kLds) + w * kScr;
    if constexpr (Tr::kQkAttn || Tr::kVAttn) {
      // ---- fused temporal attention (EPI_QK_TATTN_LN / EPI_V_TATTN_LN, see vp_kernels.h).  A
      // 16-row block mt of this wave's 128 rows is one (b n) sequence of T = 16 frames; the
      // wave's 128 columns are [q_h | k_h] of one head (QK launch) or v of two heads (V launch).
      // q, k, v are LN-folded and rounded to bf16 as the reference's bf16 projections are. ----
      const int r16 = lane & 15, g4 = lane >> 4;
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
        float4 cc[4], bb[4];
        f32x4 x[8];
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
#pragma unroll
          for (int hh = 0; hh < 2; ++hh)  // cc/bb[2*hh + i]: block 2kk + i of q (hh = 0) / k (hh = 1)
#pragma unroll
            for (int i = 0; i < 2; ++i) {
              const int n = n0 + hh * 64 + 16 * (2 * kk + i) + 4 * g4;
              cc[2 * hh + i] = *reinterpret_cast<const float4*>(ep.ln_c + n);
              bb[2 * hh + i] = *reinterpret_cast<const float4*>(ep.bias + n);
            }
#pragma unroll
          for (int mt = 0; mt < 8; ++mt) {
            auto fold2blk = [&](int hh) {  // operand of blocks (hh*4 + 2kk, +1), constants cc/bb[2hh..]
              uint32_t u[4];
#pragma unroll
              for (int i = 0; i < 2; ++i) {
                const f32x4& a = acc[hh * 4 + 2 * kk + i][mt];
                const float4 c = cc[2 * hh + i], b = bb[2 * hh + i];
                const f32x2_t r = f32x2_t(rsA[mt].x), m = f32x2_t(rsA[mt].y);
                const f32x2_t lo = __builtin_elementwise_fma(
                    r, f32x2_t{a[0], a[1]}, __builtin_elementwise_fma(m, f32x2_t{c.x, c.y}, f32x2_t{b.x, b.y}));
                const f32x2_t hi = __builtin_elementwise_fma(
                    r, f32x2_t{a[2], a[3]}, __builtin_elementwise_fma(m, f32x2_t{c.z, c.w}, f32x2_t{b.z, b.w}));
                u[2 * i] = pack_bf16x2(lo.x, lo.y);
                u[2 * i + 1] = pack_bf16x2(hi.x, hi.y);
              }
              return *reinterpret_cast<const bf16x8*>(u);
            };
            x[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fold2blk(1), fold2blk(0),
                                                            kk ? x[mt] : f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
          }
          __builtin_amdgcn_sched_barrier(0);
        }
        const float c1 = 2.0f * 1.4426950408889634f / ep.cap, c2 = ep.cap * 1.4426950408889634f;
        const int head = n0 >> 7;
        bf16_t* pout = static_cast<bf16_t*>(ep.out);
#pragma unroll
        for (int mt = 0; mt < 8; ++mt) {
          // x[mt][r] = logit[query r16][key 4*g4 + r]
          float p[4], lsum = 0.f;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            p[r] = capped_exp_exact(x[mt][r], c1, c2);
            lsum += p[r];
          }
          lsum += __shfl_xor(lsum, 16);
          lsum += __shfl_xor(lsum, 32);
          const float inv = 1.0f / lsum;
          const int64_t sq = (int64_t)(m0 + mt * 16) >> 4;
          *reinterpret_cast<uint2*>(pout + (sq * ep.heads + head) * 256 + lane * 4) =
              make_uint2(pack_bf16x2(p[0] * inv, p[1] * inv), pack_bf16x2(p[2] * inv, p[3] * inv));
        }
        continue;  // nothing else of this tile is stored
      } else {
        // O^T = V^T . P^T per (sequence mt, head nh) on 16x16x16 MFMAs: A = V^T by transposed
        // reads of the bf16 V block, B = this lane's P^T fragment; the result lands in the
        // accumulator layout (lane: query r16, d = 16 dt + 4 g4 + r) and replaces v there, so the
        // store path below writes O with whole-line stores.  The V values take the fp32 scratch
        // round trip of the store path (row segments, the LN constants of the put layout): folding
        // them where the accumulators stand measured slower here (register spills, 209 vs 168 us).
        char* sb0 = scr;
        char* sb1 = scr + kScrBuf;
        const bf16_t* pin = static_cast<const bf16_t*>(ep.resid);
        const int trq = r16 >> 2, trp = r16 & 3;
#pragma unroll
        for (int mt = 0; mt < 8; ++mt) {
          // both heads of sequence mt: V blocks at sb1 and sb1 + 2 KiB, one LDS wait per sequence
          const int64_t sq = (int64_t)(m0 + mt * 16) >> 4;
          bf16x4 pb[2];
#pragma unroll
          for (int nh = 0; nh < 2; ++nh)
            pb[nh] = *reinterpret_cast<const bf16x4*>(pin + (sq * ep.heads + ((n0 + nh * 64) >> 6)) * 256 + lane * 4);
#pragma unroll
          for (int nh = 0; nh < 2; ++nh) {
            {  // accumulator block -> fp32 scratch (put layout)
              char* sb = sb0 + frow * 256;
#pragma unroll
              for (int q = 0; q < 4; ++q)
                *reinterpret_cast<f32x4*>(sb + (((q * 4 + (lane >> 4)) ^ (frow & 7)) << 4)) = acc[nh * 4 + q][mt];
            }
#pragma unroll
            for (int pass = 0; pass < 2; ++pass) {  // row segments -> LN fold -> bf16 V rows
              const int rl = pass * 8 + er;
              const char* sb = sb0 + rl * 256;
              const float4 lo = *reinterpret_cast<const float4*>(sb + (((2 * es) ^ (rl & 7)) << 4));
              const float4 hi = *reinterpret_cast<const float4*>(sb + (((2 * es + 1) ^ (rl & 7)) << 4));
              const f32x2_t r = f32x2_t(rs[mt][pass].x), m = f32x2_t(rs[mt][pass].y);
              auto fold2 = [&](float x0, float x1, float c0, float c1, float b0, float b1) {
                const f32x2_t o = __builtin_elementwise_fma(
                    r, f32x2_t{x0, x1}, __builtin_elementwise_fma(m, f32x2_t{c0, c1}, f32x2_t{b0, b1}));
                return pack_bf16x2(o.x, o.y);
              };
              *reinterpret_cast<epi_u32x4*>(sb1 + nh * 2048 + rl * 128 + es * 16) =
                  epi_u32x4{fold2(lo.x, lo.y, cl[nh].x, cl[nh].y, bl[nh].x, bl[nh].y),
                            fold2(lo.z, lo.w, cl[nh].z, cl[nh].w, bl[nh].z, bl[nh].w),
                            fold2(hi.x, hi.y, ch[nh].x, ch[nh].y, bh[nh].x, bh[nh].y),
                            fold2(hi.z, hi.w, ch[nh].z, ch[nh].w, bh[nh].z, bh[nh].w)};
            }
          }
          __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
          __builtin_amdgcn_wave_barrier();
#pragma unroll
          for (int nh = 0; nh < 2; ++nh)
#pragma unroll
            for (int dt = 0; dt < 4; ++dt) {
              const bf16x4 vf = w4_tr_read(sb1 + nh * 2048 + (4 * g4 + trq) * 128 + (16 * dt + 4 * trp) * 2);
              acc[nh * 4 + dt][mt] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(vf, pb[nh], f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
            }
        }
      }
    }
    // residual / position rows of block mt+1 are requested before block mt's stores, so a
    // load never waits behind the stores just issued (vmcnt retires in issue order)
    F8 ex[2][2][2];  // [buffer][nh][pass]
    auto fetch = [&](int bsel, int mt) {
#pragma unroll
      for (int nh = 0; nh < 2; ++nh)
#pragma unroll
        for (int pass = 0; pass < 2; ++pass)
          ex[bsel][nh][pass] = epi_extra8<EPI>(ep, m0 + mt * 16 + pass * 8 + er, n0 + nh * 64 + es * 8, N);
    };
    // block G = (mt, nh): acc[nh*4 + q][mt], q = 0..3 -> scratch buffer G & 1.  Block G+1 is
    // written before block G is read back, so the LDS round trip overlaps the math and stores.
    auto put = [&](int G) {
      if constexpr (DIAG & 2048) {
        if (ep.ldo != -12345) return;  // never false at run time: ablation without the LDS writes
      }
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
    if constexpr (Tr::kExtra) fetch(0, 0);
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
        if ((DIAG & 4096) && ep.ldo != -12345) {  // ablation without the LDS read-back
          v.lo = make_float4((float)G, (float)pass, (float)rl, 0.f);
          v.hi = v.lo;
        } else {
          v.lo = *reinterpret_cast<const float4*>(sb + (((2 * es) ^ (rl & 7)) << 4));
          v.hi = *reinterpret_cast<const float4*>(sb + (((2 * es + 1) ^ (rl & 7)) << 4));
        }
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
        if constexpr (Tr::kKeep && !(DIAG & 512)) {
          if (ep.rowpad) keep = 1.0f - ep.rowpad[row];
        }
        if constexpr (DIAG & 32) {
          if (ep.ldo == -12345) epi_store8<EPI>(ep, row, n, v, keep, ex[mt & 1][nh][pass]);
          else asm volatile("" :: "v"(v.lo.x), "v"(v.lo.y), "v"(v.lo.z), "v"(v.lo.w), "v"(v.hi.x), "v"(v.hi.y), "v"(v.hi.z), "v"(v.hi.w));
        } else {
          const epi_u32x4 pk =
              epi_store8<EPI, !(DIAG & 256), !(DIAG & 512), (DIAG & 1024) != 0>(ep, row, n, v, keep,
                                                                                   ex[mt & 1][nh][pass]);
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
  }
  // drain the tail's (clamped) loads before the workgroup's LDS is released
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

[[maybe_unused]] constexpr int kPfLongK = 2;  // A prefetch distance (K-tiles) of the PF build (A/B; K >= 2048 uses S3)

int num_cus_w4() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
  }
  return n;
}

template <int EPI, int DIAG = 0, int PF = 0, bool S3 = false>
hipError_t launch_w4(const bf16_t* A, int64_t lda, const bf16_t* W, int64_t ldw, int M, int N,
                     int K, const EpiArgs& ep, hipStream_t s) {
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute((const void*)gemm_bf16_w4_kernel<EPI, DIAG, PF, S3>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, kLdsTotal);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  const int tiles = (M / BM) * (N / BN);
  const int grid = tiles < num_cus_w4() ? tiles : num_cus_w4();
  // DIAG 32768: ungrouped, 65536: XCD-pair split of W (A/B; needs (M/BM) % 4 == 0, (N/BN) even, grid % 8 == 0)
  const int ngrp = (DIAG & 32768) ? N / BN : (DIAG & 65536) ? -1 : w4_ngrp(M, N, K, grid);
  VP_NOTE_KERNEL((gemm_bf16_w4_kernel<EPI, DIAG, PF, S3>));
  hipLaunchKernelGGL((gemm_bf16_w4_kernel<EPI, DIAG, PF, S3>), dim3(grid), dim3(kThreads), kLdsTotal, s, A, lda, W,
                     ldw, M, N, K, ngrp, ep);
  return hipGetLastError();
}

}  // namespace

// N-tile group size (see coords): the whole W when it is small (<= 2 MB) or when the GEMM streams
// A from HBM (K >= 2048: a group sweep would re-read A per group); else groups whose W rows take
// <= 2.5 MB (W > 4 MB: Base ffn_layer1 6 of 12 N-tiles, Large ffn_layer1 / q|k|v 4) or <= half of
// W (Base q|k|v, 3.5 MB: 3 of 9; forward 6.39 -> 6.29 ms/step, one box, alternating runs)
int w4_ngrp(int M, int N, int K, int grid) {
  const int tilesN = N / BN;
  const int64_t w_tile = (int64_t)BN * K * 2;  // W bytes per N-tile
  const int64_t w_all = (int64_t)tilesN * w_tile;
  if (w_all <= (2ll << 20) || K >= 2048 || (M / BM) % 8 || grid % 8) return tilesN;
  const int64_t budget = w_all > (4ll << 20) ? (5ll << 19) : w_all / 2;
  int g = tilesN;
  for (int d = tilesN; d >= 1; --d)
    if (tilesN % d == 0 && (int64_t)d * w_tile <= budget) { g = d; break; }
  return g;
}

namespace {
// production epilogues; D = 0: nontemporal output stores, D = 256: plain stores (ablation)
template <int D>
hipError_t w4_dispatch_d(int epi, const bf16_t* A, int64_t lda, const bf16_t* W, int64_t ldw, int M, int N,
                       int K, const EpiArgs& ep, hipStream_t s) {
  switch (epi) {
    case EPI_BF16: return launch_w4<EPI_BF16, D>(A, lda, W, ldw, M, N, K, ep, s);
    case EPI_GELU_BF16: return launch_w4<EPI_GELU_BF16, D>(A, lda, W, ldw, M, N, K, ep, s);
    case EPI_RESID_F32: return launch_w4<EPI_RESID_F32, D>(A, lda, W, ldw, M, N, K, ep, s);
    case EPI_POS_F32: return launch_w4<EPI_POS_F32, D>(A, lda, W, ldw, M, N, K, ep, s);
    case EPI_RESID_FFN: return launch_w4<EPI_RESID_FFN, D>(A, lda, W, ldw, M, N, K, ep, s);
    case EPI_RESID_BF16: return launch_w4<EPI_RESID_BF16, D>(A, lda, W, ldw, M, N, K, ep, s);
    case EPI_POS_BF16: return launch_w4<EPI_POS_BF16, D>(A, lda, W, ldw, M, N, K, ep, s);
    case EPI_RESID_FFN_BF16:
      if (K >= 2048) return launch_w4<EPI_RESID_FFN_BF16, D, 0, true>(A, lda, W, ldw, M, N, K, ep, s);
      return launch_w4<EPI_RESID_FFN_BF16, D>(A, lda, W, ldw, M, N, K, ep, s);
    // q|k|v projection and post projection: S3 staging (forward, one box, alternating runs: qkv
    // 6.74-6.76 -> 6.50-6.54 ms/step, post 2.82-2.83 -> 2.69-2.71); ffn_layer1 measured no gain
    case EPI_BF16_LN: return launch_w4<EPI_BF16_LN, D, 0, true>(A, lda, W, ldw, M, N, K, ep, s);
    case EPI_GELU_BF16_LN: return launch_w4<EPI_GELU_BF16_LN, D>(A, lda, W, ldw, M, N, K, ep, s);
    case EPI_RESID_BF16_ST: return launch_w4<EPI_RESID_BF16_ST, D, 0, true>(A, lda, W, ldw, M, N, K, ep, s);
    case EPI_RESID_FFN_BF16_ST:
      if (K >= 2048) return launch_w4<EPI_RESID_FFN_BF16_ST, D, 0, true>(A, lda, W, ldw, M, N, K, ep, s);
      return launch_w4<EPI_RESID_FFN_BF16_ST, D>(A, lda, W, ldw, M, N, K, ep, s);
    case EPI_POS_BF16_ST: return launch_w4<EPI_POS_BF16_ST, D>(A, lda, W, ldw, M, N, K, ep, s);
    case EPI_RELU_BF16: return launch_w4<EPI_RELU_BF16, D>(A, lda, W, ldw, M, N, K, ep, s);
    // temporal layers' q|k|v projection with the attention fused (T = 16): S3 as the q|k|v GEMM
    case EPI_QK_TATTN_LN: return launch_w4<EPI_QK_TATTN_LN, D, 0, true>(A, lda, W, ldw, M, N, K, ep, s);
    case EPI_V_TATTN_LN: return launch_w4<EPI_V_TATTN_LN, D, 0, true>(A, lda, W, ldw, M, N, K, ep, s);
  }
  return hipErrorInvalidValue;
}
// ffn_layer1 launches without padded rows take the no-(1 - rowpad) build of the GELU epilogue
// (bitwise equal; ffn1 11.0-11.26 -> 10.9-11.0 ms/step).  The same build of the residual epilogues
// measured slower (post 2.78 -> 3.0, ffn2 7.87 -> 8.1 ms/step: different schedules), so they keep
// the multiply.
template <int D>
hipError_t w4_dispatch(int epi, const bf16_t* A, int64_t lda, const bf16_t* W, int64_t ldw, int M, int N,
                       int K, const EpiArgs& ep, hipStream_t s) {
  if (!ep.rowpad && epi == EPI_GELU_BF16_LN)
    return launch_w4<EPI_GELU_BF16_LN, D | 512>(A, lda, W, ldw, M, N, K, ep, s);
  return w4_dispatch_d<D>(epi, A, lda, W, ldw, M, N, K, ep, s);
}
}  // namespace

hipError_t gemm_bf16_w4(int epi, const bf16_t* A, int64_t lda, const bf16_t* W, int64_t ldw, int M,
                        int N, int K, const EpiArgs& ep, hipStream_t s) {
  // byte offsets into A / W must fit the 32-bit buffer range
  if ((uint64_t)M * (uint64_t)lda * 2 >= 0xFFFFFFF0ull || (uint64_t)N * (uint64_t)ldw * 2 >= 0xFFFFFFF0ull)
    return hipErrorInvalidValue;
  if (K % BK || M % BM || N % BN) return hipErrorInvalidValue;
#ifdef VP_DIAG
  if (epi >= 1000) {  // ablation builds (tools' diag library only), EPI_BF16 epilogue
    switch (epi - 1000) {
      case 2: return launch_w4<EPI_BF16, 2>(A, lda, W, ldw, M, N, K, ep, s);
      case 4: return launch_w4<EPI_BF16, 4>(A, lda, W, ldw, M, N, K, ep, s);
      case 6: return launch_w4<EPI_BF16, 6>(A, lda, W, ldw, M, N, K, ep, s);
      case 8: return launch_w4<EPI_BF16, 8>(A, lda, W, ldw, M, N, K, ep, s);
      case 14: return launch_w4<EPI_BF16, 14>(A, lda, W, ldw, M, N, K, ep, s);
      case 16: return launch_w4<EPI_BF16, 16>(A, lda, W, ldw, M, N, K, ep, s);
      case 32: return launch_w4<EPI_BF16, 32>(A, lda, W, ldw, M, N, K, ep, s);
      case 64: return launch_w4<EPI_BF16, 64>(A, lda, W, ldw, M, N, K, ep, s);
      case 80: return launch_w4<EPI_BF16, 80>(A, lda, W, ldw, M, N, K, ep, s);
      case 12: return launch_w4<EPI_BF16, 12>(A, lda, W, ldw, M, N, K, ep, s);
      case 128: return launch_w4<EPI_BF16, 128>(A, lda, W, ldw, M, N, K, ep, s);
      case 136: return launch_w4<EPI_BF16, 136>(A, lda, W, ldw, M, N, K, ep, s);
      case 256: return launch_w4<EPI_BF16, 256>(A, lda, W, ldw, M, N, K, ep, s);
      case 5000: return launch_w4<EPI_BF16, 2048>(A, lda, W, ldw, M, N, K, ep, s);
      case 5001: return launch_w4<EPI_BF16, 4096>(A, lda, W, ldw, M, N, K, ep, s);
      case 5002: return launch_w4<EPI_BF16, 6144>(A, lda, W, ldw, M, N, K, ep, s);
      case 5003: return launch_w4<EPI_BF16, 6144 | 32>(A, lda, W, ldw, M, N, K, ep, s);
      // S3 staging (production for K >= 2048) with the plain epilogue / without epilogue, and the
      // former K >= 2048 production (PF 2) with the statistics epilogue, for A/B
      case 9100: return launch_w4<EPI_BF16, 0, 0, true>(A, lda, W, ldw, M, N, K, ep, s);
      case 9108: return launch_w4<EPI_BF16, 8, 0, true>(A, lda, W, ldw, M, N, K, ep, s);
      case 9102: return launch_w4<EPI_BF16, 0, kPfLongK>(A, lda, W, ldw, M, N, K, ep, s);
      case 9111: return launch_w4<EPI_RESID_FFN_BF16_ST, 0, kPfLongK>(A, lda, W, ldw, M, N, K, ep, s);
      // the ffn_layer1 production epilogue without the N-tile grouping (A/B of w4_ngrp)
      case 2011: return launch_w4<EPI_GELU_BF16_LN, 512 | 32768>(A, lda, W, ldw, M, N, K, ep, s);
      // ... and with the XCD-pair order (each XCD of a pair holds half of W in its L2)
      case 2013: return launch_w4<EPI_GELU_BF16_LN, 512 | 65536>(A, lda, W, ldw, M, N, K, ep, s);
      case 1024: return launch_w4<EPI_BF16, 0, 2>(A, lda, W, ldw, M, N, K, ep, s);
      case 2048: return launch_w4<EPI_BF16, 0, 3>(A, lda, W, ldw, M, N, K, ep, s);
      case 4096: return launch_w4<EPI_BF16, 0, 4>(A, lda, W, ldw, M, N, K, ep, s);
      // ffn_layer1 epilogue with the (1 - rowpad) multiply kept (A/B of the DIAG 512 build)
      case 2009: return launch_w4<EPI_GELU_BF16_LN, 0>(A, lda, W, ldw, M, N, K, ep, s);
      // + scalar (unpacked) GELU arithmetic
      case 2010: return launch_w4<EPI_GELU_BF16_LN, 512 | 1024>(A, lda, W, ldw, M, N, K, ep, s);
    }
    return hipErrorInvalidValue;
  }
#endif
  // nontemporal output stores: +1.7 % on the whole forward vs plain stores (same device,
  // back-to-back runs: 947.8 vs 931.7 clips/s)
  // (also measured, no difference in the full forward: plain stores on the residual-stream
  // producers so x stays in the Infinity Cache, and the A prefetch on the LayerNorm-folded
  // consumers: 912-915 clips/s for all four combinations on one device)
  // (round 3: plain stores on the q|k|v projection, so the spatial attention could read the
  // last-written rows from the Infinity Cache, measured q|k|v 5.02-5.06 vs 4.87-4.89 ms/step and the
  // attention no faster, forward or reverse order)
  return w4_dispatch<0>(epi, A, lda, W, ldw, M, N, K, ep, s);
}

}  // namespace vp
