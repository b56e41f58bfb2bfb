// Variants of the product fp32 GEMM (videoprism-mlx_amd/csrc/gemm_f32.hip, gemm_f32_kernel2) for the
// tools' diag library only (tools/gemm_f32_var.py): the same 128x128x16 tile on v_mfma_f32_32x32x2_f32,
// with parts of the K-loop switched off (ABL, results garbage) or moved (VAR, same sums as the product).
//   ABL 2 = no LDS operand reads after the first K-tile, 4 = no staging loads / LDS stores after the
//   prologue, 8 = no epilogue stores (run-time skip: the accumulators stay live), 16 = no barrier;
//   bit 32 is not an ablation: the GELU epilogue computes erf without the libm call (gelu_erfc_fit).
//   VAR 0 = the product schedule; VAR 1 = the next K-tile's LDS stores and the barrier moved to the middle
//   of the K-tile (after step 3), and the next K-tile's first-half operand reads issued right after that
//   barrier, behind steps 4-7 (one barrier per K-tile still; every LDS read latency hidden behind MFMAs);
//   VAR 2 = the product schedule with the staging loads issued two K-tiles ahead (two register sets);
//   VAR 3 = the product schedule with LDS-DMA staging into swizzled unpadded tiles; VAR 5 / 6 = its persistent
//   form (gemm_f32_pers_kernel), 6 with a staggered start; VAR 7 = VAR 3 (+ packed GELU) in an N-grouped tile order
//   (abl = N-tiles per group); VAR 8 = VAR 3 + packed GELU with full-row stores through LDS; VAR 9 = VAR 8 N-grouped.
// Epilogues: EPI_BF16 (fp32 store + bias) and EPI_GELU_BF16 (erf GELU), as the product's epi_f32.
#include "vp_common.h"
#include "vp_diag.h"

#include <type_traits>

namespace vp {

namespace {

constexpr int VTM = 128, VTN = 128, VTK = 16, VROW = VTK + 4, VSPR = VTK / 4, VNST = VTM * VSPR / 256, VSH = VTK / 2;

// exact-erf GELU without the libm call (ABL bit 32): erfc(|z|) = t exp(-z^2 + P(t)), t = 1 / (1 + |z| / 2), P of
// degree 9 (the Chebyshev fit of Numerical Recipes' erfcc, relative error <= 1.2e-7), one Newton step on the
// reciprocal; Phi(x) = 1 - erfc / 2 (x >= 0) or erfc / 2 -- branch-free, two transcendentals
__device__ __forceinline__ float gelu_erfc_fit(float x) {
  const float za = __builtin_fabsf(x) * 0.70710678118654752f;
  const float d = __builtin_fmaf(0.5f, za, 1.0f);
  float t = __builtin_amdgcn_rcpf(d);
  t = __builtin_fmaf(t, __builtin_fmaf(-d, t, 1.0f), t);
  float p = 0.17087277f;
  p = __builtin_fmaf(p, t, -0.82215223f);
  p = __builtin_fmaf(p, t, 1.48851587f);
  p = __builtin_fmaf(p, t, -1.13520398f);
  p = __builtin_fmaf(p, t, 0.27886807f);
  p = __builtin_fmaf(p, t, -0.18628806f);
  p = __builtin_fmaf(p, t, 0.09678418f);
  p = __builtin_fmaf(p, t, 0.37409196f);
  p = __builtin_fmaf(p, t, 1.00002368f);
  p = __builtin_fmaf(p, t, -1.26551223f);
  const float y = __builtin_fmaf(-za, za, p);
  const float hec = 0.5f * t * __builtin_amdgcn_exp2f(y * 1.4426950408889634f);  // erfc(|z|) / 2
  const float phi = x >= 0.0f ? 1.0f - hec : hec;
  return x * phi;
}

// ABL bit 64: the product epilogue (vp_common.h gelu_erfc_fit2, packed; bitwise gelu_erfc_fit's results)
typedef f32x2_t vf2;

template <int EPI, int ABL, int VAR>
__global__ __launch_bounds__(256) void gemm_f32_var_kernel(const float* __restrict__ A, int64_t lda,
                                                           const float* __restrict__ W, int64_t ldw, int M, int N,
                                                           int K, EpiArgs ep) {
  __shared__ __attribute__((aligned(16))) float lds[2][2][VTM * VROW];
  const int tilesN = N / VTN;
  int bid = (int)blockIdx.x;
  if (gridDim.x % 8 == 0) bid = (bid & 7) * ((int)gridDim.x >> 3) + (bid >> 3);
  int m0 = (bid / tilesN) * VTM, n0 = (bid % tilesN) * VTN;
  if constexpr (VAR == 7 || VAR == 9) {
    // N-grouped order (ngrp = ep.ldr N-tiles, host: tilesN % ngrp == 0, M / 128 % 8 == 0): each XCD sweeps its
    // M-blocks once per group of ngrp N-tiles, so the group's W rows stay in the XCD's L2
    const int ngrp = (int)ep.ldr, mbx = (M / VTM) >> 3, x = bid / (mbx * tilesN), u = bid - x * mbx * tilesN;
    const int gi = u / (mbx * ngrp), r = u - gi * mbx * ngrp, rm = r / ngrp;
    m0 = (x * mbx + rm) * VTM;
    n0 = (gi * ngrp + (r - rm * ngrp)) * VTN;
  }
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int wm = w >> 1, wn = w & 1;
  const int half = lane >> 5, l32 = lane & 31;
  f32x4 ra[VNST], rw[VNST];
  auto gload = [&](int k0) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < VNST; ++i) {
      const int idx = t + 256 * i, row = idx / VSPR, c4 = (idx % VSPR) * 4;
      ra[i] = *reinterpret_cast<const f32x4*>(A + (int64_t)(m0 + row) * lda + k0 + c4);
      rw[i] = *reinterpret_cast<const f32x4*>(W + (int64_t)(n0 + row) * ldw + k0 + c4);
    }
  };
  auto sstore = [&](int buf) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < VNST; ++i) {
      const int idx = t + 256 * i, row = idx / VSPR, c4 = (idx % VSPR) * 4;
      *reinterpret_cast<f32x4*>(&lds[buf][0][row * VROW + c4]) = ra[i];
      *reinterpret_cast<f32x4*>(&lds[buf][1][row * VROW + c4]) = rw[i];
    }
  };
  auto barrier = [&]() __attribute__((always_inline)) {
    if constexpr (!(ABL & 16)) __syncthreads();
  };
  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x16{};
  f32x4 av[2][2], wv[2][2];  // [block][k half j]
  auto rd = [&](int buf, int j) __attribute__((always_inline)) {
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      av[b][j] = *reinterpret_cast<const f32x4*>(&lds[buf][0][(wm * 64 + b * 32 + l32) * VROW + VSH * half + 4 * j]);
      wv[b][j] = *reinterpret_cast<const f32x4*>(&lds[buf][1][(wn * 64 + b * 32 + l32) * VROW + VSH * half + 4 * j]);
    }
  };
  auto mm = [&](int st) __attribute__((always_inline)) {
#pragma unroll
    for (int nb = 0; nb < 2; ++nb)
#pragma unroll
      for (int mb = 0; mb < 2; ++mb)
        acc[nb][mb] = __builtin_amdgcn_mfma_f32_32x32x2f32(wv[nb][st >> 2][st & 3], av[mb][st >> 2][st & 3],
                                                           acc[nb][mb], 0, 0, 0);
  };
  const int nk = K / VTK;
  gload(0);
  sstore(0);
  __syncthreads();
  if constexpr (VAR == 0) {
#pragma unroll 1
    for (int kt = 0; kt < nk; ++kt) {
      const int cur = kt & 1;
      if (!(ABL & 4) && kt + 1 < nk) gload((kt + 1) * VTK);
      if (!(ABL & 2) || kt == 0) rd(cur, 0);
      __builtin_amdgcn_sched_barrier(0);
      mm(0);
      __builtin_amdgcn_sched_barrier(0);
      if (!(ABL & 2) || kt == 0) rd(cur, 1);
      __builtin_amdgcn_sched_barrier(0);
      mm(1); mm(2); mm(3);
      __builtin_amdgcn_sched_barrier(0);
      mm(4); mm(5); mm(6); mm(7);
      if (!(ABL & 4) && kt + 1 < nk) sstore(cur ^ 1);
      barrier();
    }
  } else if constexpr (VAR == 2) {
    // staging two K-tiles ahead: register sets alternate by K-tile parity (loop unrolled by 2, nk even), so
    // the stores into LDS wait for loads issued a whole K-tile earlier
    f32x4 sa[2][VNST], sw[2][VNST];
    auto gl2 = [&](int set, int k0) __attribute__((always_inline)) {
#pragma unroll
      for (int i = 0; i < VNST; ++i) {
        const int idx = t + 256 * i, row = idx / VSPR, c4 = (idx % VSPR) * 4;
        sa[set][i] = *reinterpret_cast<const f32x4*>(A + (int64_t)(m0 + row) * lda + k0 + c4);
        sw[set][i] = *reinterpret_cast<const f32x4*>(W + (int64_t)(n0 + row) * ldw + k0 + c4);
      }
    };
    auto st2 = [&](int set, int buf) __attribute__((always_inline)) {
#pragma unroll
      for (int i = 0; i < VNST; ++i) {
        const int idx = t + 256 * i, row = idx / VSPR, c4 = (idx % VSPR) * 4;
        *reinterpret_cast<f32x4*>(&lds[buf][0][row * VROW + c4]) = sa[set][i];
        *reinterpret_cast<f32x4*>(&lds[buf][1][row * VROW + c4]) = sw[set][i];
      }
    };
    gl2(1, VTK);
    auto body = [&](int kt, auto par) __attribute__((always_inline)) {
      constexpr int P = decltype(par)::value;  // kt & 1
      if (!(ABL & 4) && kt + 2 < nk) gl2(P, (kt + 2) * VTK);
      if (!(ABL & 2) || kt == 0) rd(P, 0);
      __builtin_amdgcn_sched_barrier(0);
      mm(0);
      __builtin_amdgcn_sched_barrier(0);
      if (!(ABL & 2) || kt == 0) rd(P, 1);
      __builtin_amdgcn_sched_barrier(0);
      mm(1); mm(2); mm(3);
      __builtin_amdgcn_sched_barrier(0);
      mm(4); mm(5); mm(6); mm(7);
      if (!(ABL & 4) && kt + 1 < nk) st2(P ^ 1, P ^ 1);
      barrier();
    };
#pragma unroll 1
    for (int kt = 0; kt < nk; kt += 2) {
      body(kt, std::integral_constant<int, 0>{});
      body(kt + 1, std::integral_constant<int, 1>{});
    }
  } else if constexpr (VAR == 3 || VAR == 7 || VAR == 8 || VAR == 9) {
    // LDS-DMA staging (buffer_load ... lds, 16 B per lane): no staging registers and no ds_write.  Tiles
    // unpadded, [row][4 chunks of 16 B] (64-B rows), chunk c of row r stored in slot c ^ ((r >> 2) & 3):
    // conflict-free for the operand reads' ds_read_b128 lane groups (MI355X_MICROARCH.md §LDS).  Wave w
    // stages pieces 2w, 2w+1 (16 rows = 1 KiB each) of A and of W; lane i of a piece: row i / 4, slot i % 4.
    typedef __attribute__((address_space(3))) void lds_void;
    float* L = &lds[0][0][0];
    auto opnd = [&](int buf, int x) { return L + (buf * 2 + x) * (VTM * VTK); };
    const int wu = __builtin_amdgcn_readfirstlane(w);
    const int prow = lane >> 2, pslot = lane & 3;
    const auto rsA = __builtin_amdgcn_make_buffer_rsrc((void*)(A + (int64_t)m0 * lda), 0, (int)(VTM * lda * 4), 0x00020000);
    const auto rsW = __builtin_amdgcn_make_buffer_rsrc((void*)(W + (int64_t)n0 * ldw), 0, (int)(VTN * ldw * 4), 0x00020000);
    uint32_t voA[2], voW[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int r = 16 * (2 * wu + i) + prow;
      const int c = pslot ^ ((r >> 2) & 3);
      voA[i] = (uint32_t)(r * lda * 4 + c * 16);
      voW[i] = (uint32_t)(r * ldw * 4 + c * 16);
    }
    auto dma = [&](int buf, int k0) __attribute__((always_inline)) {
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int q = 2 * wu + i;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsA, (lds_void*)(opnd(buf, 0) + q * 256), 16, voA[i], k0 * 4, 0, 0);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsW, (lds_void*)(opnd(buf, 1) + q * 256), 16, voW[i], k0 * 4, 0, 0);
      }
    };
    int offA[2][2], offW[2][2];  // [block][chunk j of this lane half] float offsets within an operand buffer
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int ra_ = wm * 64 + b * 32 + l32, rw_ = wn * 64 + b * 32 + l32, c = 2 * half + j;
        offA[b][j] = ra_ * VTK + 4 * (c ^ ((ra_ >> 2) & 3));
        offW[b][j] = rw_ * VTK + 4 * (c ^ ((rw_ >> 2) & 3));
      }
    auto rd3 = [&](int buf, int j) __attribute__((always_inline)) {
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        av[b][j] = *reinterpret_cast<const f32x4*>(opnd(buf, 0) + offA[b][j]);
        wv[b][j] = *reinterpret_cast<const f32x4*>(opnd(buf, 1) + offW[b][j]);
      }
    };
    __syncthreads();  // the register-staged prologue above wrote the padded layout: restage K-tile 0
    dma(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
#pragma unroll 1
    for (int kt = 0; kt < nk; ++kt) {
      const int cur = kt & 1;
      if (!(ABL & 4) && kt + 1 < nk) dma(cur ^ 1, (kt + 1) * VTK);
      if (!(ABL & 2) || kt == 0) rd3(cur, 0);
      __builtin_amdgcn_sched_barrier(0);
      mm(0);
      __builtin_amdgcn_sched_barrier(0);
      if (!(ABL & 2) || kt == 0) rd3(cur, 1);
      __builtin_amdgcn_sched_barrier(0);
      mm(1); mm(2); mm(3);
      __builtin_amdgcn_sched_barrier(0);
      mm(4); mm(5); mm(6); mm(7);
      __builtin_amdgcn_sched_barrier(0);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      barrier();
    }
  } else {
    rd(0, 0);
#pragma unroll 1
    for (int kt = 0; kt < nk; ++kt) {
      const int cur = kt & 1;
      const bool more = kt + 1 < nk;
      if (!(ABL & 4) && more) gload((kt + 1) * VTK);
      __builtin_amdgcn_sched_barrier(0);
      mm(0);
      __builtin_amdgcn_sched_barrier(0);
      if (!(ABL & 2) || kt == 0) rd(cur, 1);
      __builtin_amdgcn_sched_barrier(0);
      mm(1); mm(2); mm(3);
      __builtin_amdgcn_sched_barrier(0);
      // every wave's reads of `cur` were issued before this point, and its stores of `cur ^ 1` land before
      // the barrier: after it `cur ^ 1` may be read, and in the next K-tile `cur` may be overwritten
      if (!(ABL & 4) && more) sstore(cur ^ 1);
      barrier();
      if (!(ABL & 2) && more) rd(cur ^ 1, 0);
      __builtin_amdgcn_sched_barrier(0);
      mm(4); mm(5); mm(6); mm(7);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  if constexpr (ABL & 8) {
    if (ep.ldo != -12345) return;
  }
  if constexpr (VAR == 8 || VAR == 9) {
    // full-row stores: each 32-row x 64-column block goes through the wave's 8 KiB of LDS (free: the last K-tile's
    // barrier is behind every operand read) so that 16 lanes hold one row's 64 consecutive columns (256 B) per
    // store instruction instead of 2 lanes holding 32 B.  16-B chunk c of LDS row r at chunk c ^ (r & 7).
    float* stg = &lds[0][0][0] + w * 2048;
#pragma unroll
    for (int mb = 0; mb < 2; ++mb) {
#pragma unroll
      for (int nb = 0; nb < 2; ++nb)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int c = nb * 8 + 2 * q + half;
          const f32x16& a = acc[nb][mb];
          *reinterpret_cast<f32x4*>(stg + l32 * 64 + 4 * (c ^ (l32 & 7))) =
              f32x4{a[4 * q], a[4 * q + 1], a[4 * q + 2], a[4 * q + 3]};
        }
      __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's block is in LDS (wave-private region)
      __builtin_amdgcn_wave_barrier();
      const int c = lane & 15;
      const int n = n0 + wn * 64 + 4 * c;
      const float4 b = *reinterpret_cast<const float4*>(ep.bias + n);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int r = 4 * i + (lane >> 4);
        const f32x4 v = *reinterpret_cast<const f32x4*>(stg + r * 64 + 4 * (c ^ (r & 7)));
        float v0 = v[0] + b.x, v1 = v[1] + b.y, v2 = v[2] + b.z, v3 = v[3] + b.w;
        if constexpr (EPI == EPI_GELU_BF16) {
          const vf2 g0 = gelu_erfc_fit2(vf2{v0, v1}), g1 = gelu_erfc_fit2(vf2{v2, v3});
          v0 = g0.x; v1 = g0.y; v2 = g1.x; v3 = g1.y;
        }
        float* out = static_cast<float*>(ep.out) + (int64_t)(m0 + wm * 64 + mb * 32 + r) * ep.ldo + n;
        *reinterpret_cast<float4*>(out) = make_float4(v0, v1, v2, v3);
      }
      __builtin_amdgcn_s_waitcnt(0xc07f);
      __builtin_amdgcn_wave_barrier();  // the reads of this block are done before the next block's writes
    }
    return;
  }
#pragma unroll
  for (int nb = 0; nb < 2; ++nb)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int n = n0 + wn * 64 + nb * 32 + 8 * q + 4 * half;
      const float4 b = *reinterpret_cast<const float4*>(ep.bias + n);
#pragma unroll
      for (int mb = 0; mb < 2; ++mb) {
        const f32x16& a = acc[nb][mb];
        float v0 = a[4 * q] + b.x, v1 = a[4 * q + 1] + b.y, v2 = a[4 * q + 2] + b.z, v3 = a[4 * q + 3] + b.w;
        if constexpr (EPI == EPI_GELU_BF16 && (ABL & 64)) {
          const vf2 lo = gelu_erfc_fit2(vf2{v0, v1}), hi = gelu_erfc_fit2(vf2{v2, v3});
          v0 = lo.x; v1 = lo.y; v2 = hi.x; v3 = hi.y;
        } else if constexpr (EPI == EPI_GELU_BF16 && (ABL & 32)) {
          v0 = gelu_erfc_fit(v0); v1 = gelu_erfc_fit(v1); v2 = gelu_erfc_fit(v2); v3 = gelu_erfc_fit(v3);
        } else if constexpr (EPI == EPI_GELU_BF16) {
          v0 = gelu_erf(v0); v1 = gelu_erf(v1); v2 = gelu_erf(v2); v3 = gelu_erf(v3);
        }
        float* out = static_cast<float*>(ep.out) + (int64_t)(m0 + wm * 64 + mb * 32 + l32) * ep.ldo + n;
        *reinterpret_cast<float4*>(out) = make_float4(v0, v1, v2, v3);
      }
    }
}

// Persistent form of VAR 3 (+ the packed libm-free GELU): G workgroups (3 per CU) loop over XCD-contiguous tile
// ranges; the next tile's first K-tile is requested before this tile's epilogue.  stagger > 0: the workgroups of
// the second and third residency slot on a CU (li / 32 = 1, 2 within the XCD) sleep slot * stagger * 8128 cycles
// before their first tile, so the co-resident workgroups do not reach their epilogues together.
template <int EPI>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3, 3))) void gemm_f32_pers_kernel(const float* __restrict__ A, int64_t lda,
                                                            const float* __restrict__ W, int64_t ldw, int M, int N,
                                                            int K, EpiArgs ep, int stagger) {
  __shared__ __attribute__((aligned(16))) float L[2 * 2 * VTM * VTK];
  typedef __attribute__((address_space(3))) void lds_void;
  const int tilesN = N / VTN, T = (M / VTM) * tilesN;
  const int G = gridDim.x, b = blockIdx.x, xcd = b & 7, li = b >> 3, nx = G >> 3;
  const int lo = (int)(((int64_t)xcd * T) >> 3), hi = (int)(((int64_t)(xcd + 1) * T) >> 3);
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int wm = w >> 1, wn = w & 1;
  const int half = lane >> 5, l32 = lane & 31;
  const int wu = __builtin_amdgcn_readfirstlane(w);
  const int prow = lane >> 2, pslot = lane & 3;
  auto opnd = [&](int buf, int x) { return L + (buf * 2 + x) * (VTM * VTK); };
  uint32_t voA[2], voW[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int r = 16 * (2 * wu + i) + prow;
    const int c = pslot ^ ((r >> 2) & 3);
    voA[i] = (uint32_t)(r * lda * 4 + c * 16);
    voW[i] = (uint32_t)(r * ldw * 4 + c * 16);
  }
  int offA[2][2], offW[2][2];
#pragma unroll
  for (int bb = 0; bb < 2; ++bb)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int ra_ = wm * 64 + bb * 32 + l32, rw_ = wn * 64 + bb * 32 + l32, c = 2 * half + j;
      offA[bb][j] = ra_ * VTK + 4 * (c ^ ((ra_ >> 2) & 3));
      offW[bb][j] = rw_ * VTK + 4 * (c ^ ((rw_ >> 2) & 3));
    }
  auto rsrc = [&](const float* base, int64_t ld) {
    return __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, (int)(VTM * ld * 4), 0x00020000);
  };
  auto dma = [&](__amdgpu_buffer_rsrc_t rA, __amdgpu_buffer_rsrc_t rW, int buf, int k0) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int q = 2 * wu + i;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rA, (lds_void*)(opnd(buf, 0) + q * 256), 16, voA[i], k0 * 4, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rW, (lds_void*)(opnd(buf, 1) + q * 256), 16, voW[i], k0 * 4, 0, 0);
    }
  };
  f32x4 av[2][2], wv[2][2];
  auto rd3 = [&](int buf, int j) __attribute__((always_inline)) {
#pragma unroll
    for (int bb = 0; bb < 2; ++bb) {
      av[bb][j] = *reinterpret_cast<const f32x4*>(opnd(buf, 0) + offA[bb][j]);
      wv[bb][j] = *reinterpret_cast<const f32x4*>(opnd(buf, 1) + offW[bb][j]);
    }
  };
  f32x16 acc[2][2];
  auto mm = [&](int st) __attribute__((always_inline)) {
#pragma unroll
    for (int nb = 0; nb < 2; ++nb)
#pragma unroll
      for (int mb = 0; mb < 2; ++mb)
        acc[nb][mb] = __builtin_amdgcn_mfma_f32_32x32x2f32(wv[nb][st >> 2][st & 3], av[mb][st >> 2][st & 3],
                                                           acc[nb][mb], 0, 0, 0);
  };
  const int nk = K / VTK;
  int tile = lo + li;
  if (tile >= hi) return;
  if (stagger > 0) {
    const int slot = (li >> 5) % 3;
    for (int i = 0; i < slot * stagger; ++i) __builtin_amdgcn_s_sleep(127);
  }
  {
    const int m0 = (tile / tilesN) * VTM, n0 = (tile % tilesN) * VTN;
    dma(rsrc(A + (int64_t)m0 * lda, lda), rsrc(W + (int64_t)n0 * ldw, ldw), 0, 0);
  }
  for (; tile < hi; tile += nx) {
    const int m0 = (tile / tilesN) * VTM, n0 = (tile % tilesN) * VTN;
    const auto rA = rsrc(A + (int64_t)m0 * lda, lda), rW = rsrc(W + (int64_t)n0 * ldw, ldw);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = f32x16{};
#pragma unroll 1
    for (int kt = 0; kt < nk; ++kt) {
      const int cur = kt & 1;
      if (kt + 1 < nk) dma(rA, rW, cur ^ 1, (kt + 1) * VTK);
      rd3(cur, 0);
      __builtin_amdgcn_sched_barrier(0);
      mm(0);
      __builtin_amdgcn_sched_barrier(0);
      rd3(cur, 1);
      __builtin_amdgcn_sched_barrier(0);
      mm(1); mm(2); mm(3);
      __builtin_amdgcn_sched_barrier(0);
      mm(4); mm(5); mm(6); mm(7);
      __builtin_amdgcn_sched_barrier(0);
      if (kt + 1 < nk) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
      }
    }
    // every wave's reads of the last K-tile's buffer were waited on by its MFMAs; buffer 0 is free once all
    // waves are past them (nk even: the last K-tile used buffer 1, so only buffer 0's readers of K-tile nk-2
    // matter, and they are behind the last barrier)
    const int nt = tile + nx;
    if (nt < hi) {
      const int m1 = (nt / tilesN) * VTM, n1 = (nt % tilesN) * VTN;
      dma(rsrc(A + (int64_t)m1 * lda, lda), rsrc(W + (int64_t)n1 * ldw, ldw), 0, 0);
    }
#pragma unroll
    for (int nb = 0; nb < 2; ++nb)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int n = n0 + wn * 64 + nb * 32 + 8 * q + 4 * half;
        const float4 bs = *reinterpret_cast<const float4*>(ep.bias + n);
#pragma unroll
        for (int mb = 0; mb < 2; ++mb) {
          const f32x16& a = acc[nb][mb];
          float v0 = a[4 * q] + bs.x, v1 = a[4 * q + 1] + bs.y, v2 = a[4 * q + 2] + bs.z, v3 = a[4 * q + 3] + bs.w;
          if constexpr (EPI == EPI_GELU_BF16) {
            const vf2 g0 = gelu_erfc_fit2(vf2{v0, v1}), g1 = gelu_erfc_fit2(vf2{v2, v3});
            v0 = g0.x; v1 = g0.y; v2 = g1.x; v3 = g1.y;
          }
          float* out = static_cast<float*>(ep.out) + (int64_t)(m0 + wm * 64 + mb * 32 + l32) * ep.ldo + n;
          *reinterpret_cast<float4*>(out) = make_float4(v0, v1, v2, v3);
        }
      }
  }
}

template <int EPI, int ABL, int VAR>
hipError_t launch_var(const float* A, const float* W, int M, int N, int K, const EpiArgs& ep, hipStream_t s) {
  hipLaunchKernelGGL((gemm_f32_var_kernel<EPI, ABL, VAR>), dim3((M / VTM) * (N / VTN)), dim3(256), 0, s, A,
                     (int64_t)K, W, (int64_t)K, M, N, K, ep);
  return hipGetLastError();
}

template <int EPI, int VAR>
hipError_t by_abl(int abl, const float* A, const float* W, int M, int N, int K, const EpiArgs& ep, hipStream_t s) {
  switch (abl) {
    case 0: return launch_var<EPI, 0, VAR>(A, W, M, N, K, ep, s);
    case 2: return launch_var<EPI, 2, VAR>(A, W, M, N, K, ep, s);
    case 4: return launch_var<EPI, 4, VAR>(A, W, M, N, K, ep, s);
    case 8: return launch_var<EPI, 8, VAR>(A, W, M, N, K, ep, s);
    case 20: return launch_var<EPI, 20, VAR>(A, W, M, N, K, ep, s);
    case 14: return launch_var<EPI, 14, VAR>(A, W, M, N, K, ep, s);
    case 30: return launch_var<EPI, 30, VAR>(A, W, M, N, K, ep, s);
    case 32: return launch_var<EPI, 32, VAR>(A, W, M, N, K, ep, s);
    case 64: return launch_var<EPI, 64, VAR>(A, W, M, N, K, ep, s);
  }
  return hipErrorInvalidValue;
}

}  // namespace

hipError_t gemm_f32_var(int var, int abl, int epi, const float* A, const float* W, int M, int N, int K,
                        const EpiArgs& ep, hipStream_t s) {
  if (M <= 0 || N <= 0 || K < 2 * VTK || M % VTM || N % VTN || K % VTK) return hipErrorInvalidValue;
  if (epi != EPI_BF16 && epi != EPI_GELU_BF16) return hipErrorInvalidValue;
  if (var == 0)
    return epi == EPI_BF16 ? by_abl<EPI_BF16, 0>(abl, A, W, M, N, K, ep, s)
                           : by_abl<EPI_GELU_BF16, 0>(abl, A, W, M, N, K, ep, s);
  if (var == 1)
    return epi == EPI_BF16 ? by_abl<EPI_BF16, 1>(abl, A, W, M, N, K, ep, s)
                           : by_abl<EPI_GELU_BF16, 1>(abl, A, W, M, N, K, ep, s);
  if (var == 5 || var == 6) {  // persistent (6: staggered start, abl = the stagger in s_sleep(127) units)
    const int T = (M / VTM) * (N / VTN);
    if (T % 8 || (K / VTK) % 2) return hipErrorInvalidValue;
    const int G = T < 768 ? T : 768;
    const int st = var == 6 ? abl : 0;
    if (epi == EPI_BF16)
      hipLaunchKernelGGL((gemm_f32_pers_kernel<EPI_BF16>), dim3(G), dim3(256), 0, s, A, (int64_t)K, W, (int64_t)K, M, N,
                         K, ep, st);
    else
      hipLaunchKernelGGL((gemm_f32_pers_kernel<EPI_GELU_BF16>), dim3(G), dim3(256), 0, s, A, (int64_t)K, W, (int64_t)K,
                         M, N, K, ep, st);
    return hipGetLastError();
  }
  if (var == 8)  // VAR 3 (+ packed GELU) with full-row stores through LDS
    return epi == EPI_BF16 ? launch_var<EPI_BF16, 64, 8>(A, W, M, N, K, ep, s)
                           : launch_var<EPI_GELU_BF16, 64, 8>(A, W, M, N, K, ep, s);
  if (var == 9) {  // VAR 8 in N-grouped tile order, abl = ngrp
    const int tilesN = N / VTN;
    if (abl < 1 || tilesN % abl || (M / VTM) % 8) return hipErrorInvalidValue;
    EpiArgs e2 = ep;
    e2.ldr = abl;
    return epi == EPI_BF16 ? launch_var<EPI_BF16, 64, 9>(A, W, M, N, K, e2, s)
                           : launch_var<EPI_GELU_BF16, 64, 9>(A, W, M, N, K, e2, s);
  }
  if (var == 7) {  // VAR 3 in N-grouped tile order, abl = ngrp
    const int tilesN = N / VTN;
    if (abl < 1 || tilesN % abl || (M / VTM) % 8) return hipErrorInvalidValue;
    EpiArgs e2 = ep;
    e2.ldr = abl;
    return epi == EPI_BF16 ? launch_var<EPI_BF16, 64, 7>(A, W, M, N, K, e2, s)
                           : launch_var<EPI_GELU_BF16, 64, 7>(A, W, M, N, K, e2, s);
  }
  if (var == 3)
    return epi == EPI_BF16 ? by_abl<EPI_BF16, 3>(abl, A, W, M, N, K, ep, s)
                           : by_abl<EPI_GELU_BF16, 3>(abl, A, W, M, N, K, ep, s);
  if (var == 2 && (K / VTK) % 2 == 0)
    return epi == EPI_BF16 ? by_abl<EPI_BF16, 2>(abl, A, W, M, N, K, ep, s)
                           : by_abl<EPI_GELU_BF16, 2>(abl, A, W, M, N, K, ep, s);
  return hipErrorInvalidValue;
}

}  // namespace vp
