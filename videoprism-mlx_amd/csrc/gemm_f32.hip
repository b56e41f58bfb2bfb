// fp32 GEMM for fprop_dtype=float32 (the reference's default precision, models.py:268-303).
//
//   C[M,N] = A[M,K] . W[N,K]^T (+ epilogue), exact fp32 on v_mfma_f32_16x16x4_f32
//   (a k-ordered fmaf chain per output, no reduced-precision inner product).
//
// Tile 128x128x16, 4 waves (2x2, 64x64 each), register-staged double-buffered LDS
// stored k-major ([k][m], row stride 144 floats) so the 16x16x4 operand reads are
// conflict-free ds_read_b32.  Same operand swap as the bf16 kernel: each lane owns
// 4 consecutive N columns of one M row for 16-byte epilogue stores.
#include "vp_common.h"
#include "vp_kernels.h"

namespace vp {

namespace {

constexpr int TM = 128, TN = 128, TK = 16, LDSROW = 144;

// GFIT: the GELU as gelu_erfc_fit2 (v2 kernel) instead of the libm erff (v1 kernel)
template <int EPI, bool GFIT = false>
__device__ __forceinline__ void epi_f32(const EpiArgs& ep, int N, int m, int n, float v0, float v1,
                                        float v2, float v3) {
  float* out = static_cast<float*>(ep.out) + (int64_t)m * ep.ldo + n;
  if constexpr (EPI == EPI_BF16) {
    *reinterpret_cast<float4*>(out) = make_float4(v0, v1, v2, v3);
  } else if constexpr (EPI == EPI_GELU_BF16 || EPI == EPI_RELU_BF16) {
    if constexpr (EPI == EPI_GELU_BF16 && GFIT) {
      const f32x2_t g0 = gelu_erfc_fit2(f32x2_t{v0, v1}), g1 = gelu_erfc_fit2(f32x2_t{v2, v3});
      v0 = g0.x; v1 = g0.y; v2 = g1.x; v3 = g1.y;
    } else if constexpr (EPI == EPI_GELU_BF16) {
      v0 = gelu_erf(v0); v1 = gelu_erf(v1); v2 = gelu_erf(v2); v3 = gelu_erf(v3);
    } else {
      v0 = relu_nan(v0); v1 = relu_nan(v1); v2 = relu_nan(v2); v3 = relu_nan(v3);
    }
    if (ep.rowpad) {
      const float keep = 1.0f - ep.rowpad[m];
      v0 *= keep; v1 *= keep; v2 *= keep; v3 *= keep;
    }
    *reinterpret_cast<float4*>(out) = make_float4(v0, v1, v2, v3);
  } else if constexpr (EPI == EPI_RESID_F32 || EPI == EPI_RESID_FFN) {
    if (ep.rowpad) {
      const float keep = 1.0f - ep.rowpad[m];
      v0 *= keep; v1 *= keep; v2 *= keep; v3 *= keep;
    }
    const float4 r = *reinterpret_cast<const float4*>(static_cast<const float*>(ep.resid) + (int64_t)m * ep.ldr + n);
    *reinterpret_cast<float4*>(out) = make_float4(r.x + v0, r.y + v1, r.z + v2, r.w + v3);
  } else {
    const float4 p =
        *reinterpret_cast<const float4*>(ep.pos + (int64_t)(m % ep.pos_rows) * N + n);
    *reinterpret_cast<float4*>(out) = make_float4(v0 + p.x, v1 + p.y, v2 + p.z, v3 + p.w);
  }
}

template <int EPI>
__global__ __launch_bounds__(256) void gemm_f32_kernel(const float* __restrict__ A, int64_t lda,
                                                       const float* __restrict__ W, int64_t ldw,
                                                       int M, int N, int K, EpiArgs ep) {
  __shared__ __attribute__((aligned(16))) float lds[2][2][TK * LDSROW];
  const int tilesN = N / TN;
  const int m0 = (blockIdx.x / tilesN) * TM, n0 = (blockIdx.x % tilesN) * TN;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int wm = w >> 1, wn = w & 1;
  const int srow = t >> 2, sk = (t & 3) * 4;

  float4 ra[2], rw[2];
  auto gload = [&](int k0) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      ra[i] = *reinterpret_cast<const float4*>(A + (int64_t)(m0 + srow + 64 * i) * lda + k0 + sk);
      rw[i] = *reinterpret_cast<const float4*>(W + (int64_t)(n0 + srow + 64 * i) * ldw + k0 + sk);
    }
  };
  auto sstore = [&](int buf) {
    float* la = lds[buf][0];
    float* lw = lds[buf][1];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int r = srow + 64 * i;
      la[(sk + 0) * LDSROW + r] = ra[i].x; la[(sk + 1) * LDSROW + r] = ra[i].y;
      la[(sk + 2) * LDSROW + r] = ra[i].z; la[(sk + 3) * LDSROW + r] = ra[i].w;
      lw[(sk + 0) * LDSROW + r] = rw[i].x; lw[(sk + 1) * LDSROW + r] = rw[i].y;
      lw[(sk + 2) * LDSROW + r] = rw[i].z; lw[(sk + 3) * LDSROW + r] = rw[i].w;
    }
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = K / TK;
  gload(0);
  sstore(0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) gload((kt + 1) * TK);
    const float* la = lds[cur][0];
    const float* lw = lds[cur][1];
#pragma unroll
    for (int kk = 0; kk < TK / 4; ++kk) {
      const int k = kk * 4 + (lane >> 4);
      float av[4], wv[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        av[i] = la[k * LDSROW + wm * 64 + i * 16 + (lane & 15)];
        wv[i] = lw[k * LDSROW + wn * 64 + i * 16 + (lane & 15)];
      }
#pragma unroll
      for (int nt = 0; nt < 4; ++nt)
#pragma unroll
        for (int mt = 0; mt < 4; ++mt)
          acc[nt][mt] = __builtin_amdgcn_mfma_f32_16x16x4f32(wv[nt], av[mt], acc[nt][mt], 0, 0, 0);
    }
    if (kt + 1 < nk) sstore(cur ^ 1);
    __syncthreads();
  }
  const int mb = m0 + wm * 64 + (lane & 15);
  const int nb = n0 + wn * 64 + (lane >> 4) * 4;
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) {
    const int n = nb + nt * 16;
    const float4 b = *reinterpret_cast<const float4*>(ep.bias + n);
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      const f32x4 a = acc[nt][mt];
      epi_f32<EPI>(ep, N, mb + mt * 16, n, a[0] + b.x, a[1] + b.y, a[2] + b.z, a[3] + b.w);
    }
  }
}

// ---- v2 (round 6): v_mfma_f32_32x32x2_f32, K-tile 16 with a per-lane-half k permutation ----
// Same 128x128 workgroup tile and 2x2 waves of 64x64, but on 32x32x2 MFMAs (2 x 2 blocks per wave, 32 MFMAs
// per K-tile instead of 64) with operands read as whole 16-B runs: in K-tile step s (0..7) lane half h
// contracts k = 8 h + s, so a lane's 8 operands of a K-tile are 8 consecutive floats of its row (two
// ds_read_b128 per row).  Operands swapped as in v1 (D^T = W.A^T): register r of block (nb, mb) is output row
// m = l % 32, column n = 8 (r / 4) + 4 (l / 32) + r % 4, so each lane owns 4 consecutive columns of one row for
// the 16-byte epilogue stores.  XCD-contiguous tile ranges (workgroup b runs on XCD b % 8), M-block-major
// inside a range so an A block stays in its XCD's L2 across the N tiles.  Exact fp32 products summed in fp32
// (another order than v1: k-pairs, then steps).  Within a K-tile the second half's LDS reads are issued behind
// the first step's MFMAs, so only four reads' latency is exposed after each barrier.
// Staging by LDS-DMA (buffer_load_dwordx4 ... lds: 16 B per lane straight into LDS, no staging registers and no
// ds_write): each 1-KiB wave instruction fills 16 whole 64-B rows of a tile, so the tiles are unpadded
// [row][4 chunks of 16 B] with chunk c of row r in slot c ^ ((r >> 2) & 3) -- the lane picks its source chunk,
// and the operand reads undo the swizzle; conflict-free for the ds_read_b128 lane groups (MI355X_MICROARCH.md
// §LDS: per group the 4 lanes of each row residue mod 4 sit in 4 distinct slots).  Measured (tools/
// gemm_f32_var.py, Base B = 8 shapes, profiles/r06/fp32_gemm_var.txt): bitwise the register-staged kernel's
// sums, 5-9 % faster (q|k|v 818 vs 883 us, post 278 vs 302, ffn2 1057 vs 1151).  The register-staged form
// measured 0-8 % faster than v1 (profiles/r06/fp32_gemm_ab.txt); a K-tile of 32 (two workgroups per CU) was
// 8-38 % slower.  Its GELU epilogue is gelu_erfc_fit2 (no libm branches; ffn_layer1 1157 vs 1228 us).
template <int EPI>
__global__ __launch_bounds__(256) void gemm_f32_kernel2(const float* __restrict__ A, int64_t lda,
                                                        const float* __restrict__ W, int64_t ldw,
                                                        int M, int N, int K, int ngrp, EpiArgs ep) {
  constexpr int TK2 = 16;
  __shared__ __attribute__((aligned(16))) float lds[2][2][TM * TK2];  // [buffer][A | W][row][16 k, swizzled]
  typedef __attribute__((address_space(3))) void lds_void;
  const int tilesN = N / TN;
  int bid = (int)blockIdx.x;
  if (gridDim.x % 8 == 0) bid = (bid & 7) * ((int)gridDim.x >> 3) + (bid >> 3);
  int m0 = (bid / tilesN) * TM, n0 = (bid % tilesN) * TN;
  if (ngrp != tilesN) {
    // N-grouped order (host f32_ngrp: every XCD owns M / 1024 whole M-blocks): the XCD sweeps its M-blocks once
    // per group of ngrp N-tiles, so the group's W rows stay in its L2 instead of W being re-fetched per M-block
    const int mbx = (M / TM) >> 3, x = bid / (mbx * tilesN), u = bid - x * mbx * tilesN;
    const int gi = u / (mbx * ngrp), r = u - gi * mbx * ngrp, rm = r / ngrp;
    m0 = (x * mbx + rm) * TM;
    n0 = (gi * ngrp + (r - rm * ngrp)) * TN;
  }
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int wu = __builtin_amdgcn_readfirstlane(w);
  const int wm = w >> 1, wn = w & 1;
  const int half = lane >> 5, l32 = lane & 31;
  // staging: wave w fills rows 32 w .. 32 w + 31 of A and of W (pieces 2 w, 2 w + 1 of 16 rows); lane i of a
  // piece: row i / 4, slot i % 4 <- source chunk slot ^ swizzle.  The descriptors span the tile's 128 rows.
  const auto rsA = __builtin_amdgcn_make_buffer_rsrc((void*)(A + (int64_t)m0 * lda), 0, (int)(TM * lda * 4), 0x00020000);
  const auto rsW = __builtin_amdgcn_make_buffer_rsrc((void*)(W + (int64_t)n0 * ldw), 0, (int)(TN * ldw * 4), 0x00020000);
  uint32_t voA[2], voW[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int r = 16 * (2 * wu + i) + (lane >> 2);
    const int c = (lane & 3) ^ ((r >> 2) & 3);
    voA[i] = (uint32_t)(r * lda * 4 + c * 16);
    voW[i] = (uint32_t)(r * ldw * 4 + c * 16);
  }
  auto dma = [&](int buf, int k0) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int q = 2 * wu + i;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsA, (lds_void*)&lds[buf][0][q * 256], 16, voA[i], k0 * 4, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsW, (lds_void*)&lds[buf][1][q * 256], 16, voW[i], k0 * 4, 0, 0);
    }
  };
  // operand reads: block b's row of this lane, chunk 2 h + j (k = 8 h + 4 j .. + 3), through the swizzle
  int offA[2][2], offW[2][2];
#pragma unroll
  for (int b = 0; b < 2; ++b)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int ra = wm * 64 + b * 32 + l32, rw = wn * 64 + b * 32 + l32, c = 2 * half + j;
      offA[b][j] = ra * TK2 + 4 * (c ^ ((ra >> 2) & 3));
      offW[b][j] = rw * TK2 + 4 * (c ^ ((rw >> 2) & 3));
    }
  f32x16 acc[2][2];  // [n block][m block]
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x16{};
  const int nk = K / TK2;
  dma(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
#pragma unroll 1
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) dma(cur ^ 1, (kt + 1) * TK2);  // buffer cur ^ 1: every read of it was before the last barrier
    f32x4 av[2][2], wv[2][2];  // [block][chunk j]
    auto rd = [&](int j) __attribute__((always_inline)) {
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        av[b][j] = *reinterpret_cast<const f32x4*>(&lds[cur][0][offA[b][j]]);
        wv[b][j] = *reinterpret_cast<const f32x4*>(&lds[cur][1][offW[b][j]]);
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
    // the second half's reads issued behind the first step's MFMAs, so only 4 reads' latency is exposed
    rd(0);
    __builtin_amdgcn_sched_barrier(0);
    mm(0);
    __builtin_amdgcn_sched_barrier(0);
    rd(1);
    __builtin_amdgcn_sched_barrier(0);
    mm(1); mm(2); mm(3);
    __builtin_amdgcn_sched_barrier(0);
    mm(4); mm(5); mm(6); mm(7);
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the next K-tile has landed in LDS
    __syncthreads();
  }
  // epilogue through the wave's 8 KiB of LDS (free: every operand read is behind the last barrier): a 32-row x
  // 64-column block is written from the accumulator layout (a lane: 16 columns of one row in 16-B pieces) and read
  // back as 16 lanes per row of 64 consecutive columns, so each store / residual load instruction covers 4 rows x
  // 256 B -- whole lines instead of 32 rows x 32 B (ffn_layer1: 1.74x the output bytes written at the HBM side
  // before, 1.00x after).  16-B chunk c of row r sits at chunk c ^ (r & 7): conflict-free for the ds_write_b128
  // lane groups.  Same values and epilogue arithmetic as storing from the accumulators.
  float* stg = &lds[0][0][0] + w * 2048;
  const int c16 = lane & 15;
  const int n = n0 + wn * 64 + 4 * c16;
  const float4 b = *reinterpret_cast<const float4*>(ep.bias + n);
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
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the block is in LDS (a wave-private region)
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int r = 4 * i + (lane >> 4);
      const f32x4 v = *reinterpret_cast<const f32x4*>(stg + r * 64 + 4 * (c16 ^ (r & 7)));
      epi_f32<EPI, true>(ep, N, m0 + wm * 64 + mb * 32 + r, n, v[0] + b.x, v[1] + b.y, v[2] + b.z, v[3] + b.w);
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();  // this block's reads are done before the next block's writes
  }
}

// N-tile group size of the fp32 GEMM's tile order (kernel2): the whole W when it fits the XCD's L2 share
// (<= 3 MB) or when A is the stream that matters (K >= 2048: a group sweep would re-read A per group); else
// groups whose W rows take <= 2.5 MB (Base q|k|v and ffn_layer1: 6 N-tiles).  ffn_layer1 at B = 8: fetched
// bytes 1.86 -> 0.80 GB per launch, 5 % faster with the whole-line epilogue (profiles/r06/fp32_gemm_var.txt).
int f32_ngrp(int M, int N, int K) {
  const int tilesN = N / TN;
  const int64_t w_tile = (int64_t)TN * K * 4;
  if ((int64_t)tilesN * w_tile <= (3ll << 20) || K >= 2048 || (M / TM) % 8 || ((M / TM) * tilesN) % 8) return tilesN;
  for (int d = tilesN; d >= 1; --d)
    if (tilesN % d == 0 && (int64_t)d * w_tile <= (5ll << 19)) return d;
  return tilesN;
}

template <int EPI>
hipError_t launch(const float* A, int64_t lda, const float* W, int64_t ldw, int M, int N, int K,
                  const EpiArgs& ep, hipStream_t s, int version) {
  if (version == 1) {
    VP_NOTE_KERNEL(gemm_f32_kernel<EPI>);
    hipLaunchKernelGGL(gemm_f32_kernel<EPI>, dim3((M / TM) * (N / TN)), dim3(256), 0, s, A, lda, W,
                       ldw, M, N, K, ep);
  } else {
    VP_NOTE_KERNEL(gemm_f32_kernel2<EPI>);
    // 4 workgroups per CU fit (48-59 VGPRs, 32 KiB of LDS); at K >= 2048 (ffn_layer2, A streamed from HBM) 3 run
    // faster (1106 vs 1170 us at B = 8, same box; the K = 768 launches equal or faster at 4: q|k|v 833 vs 843):
    // 20 KiB of unused dynamic LDS caps them at 3
    const size_t cap3 = K >= 2048 ? 20480 : 0;
    hipLaunchKernelGGL(gemm_f32_kernel2<EPI>, dim3((M / TM) * (N / TN)), dim3(256), cap3, s, A, lda, W,
                       ldw, M, N, K, f32_ngrp(M, N, K), ep);
  }
  return hipGetLastError();
}

}  // namespace

const char* gemm_f32_check(int M, int N, int K, int64_t lda, int64_t ldw) {
  if (M <= 0 || N <= 0 || K <= 0) return "gemm_f32: non-positive dimension";
  if (M % TM) return "gemm_f32: M must be a multiple of 128";
  if (N % TN) return "gemm_f32: N must be a multiple of 128";
  if (K % TK) return "gemm_f32: K must be a multiple of 16";
  // the v2 kernel's LDS-DMA descriptors span 128 rows of A / W in bytes (int32) with 16-B row starts
  if (lda < K || ldw < K || lda % 4 || ldw % 4) return "gemm_f32: lda, ldw must be >= K and multiples of 4";
  if ((int64_t)TM * lda * 4 > 0x7fffffff || (int64_t)TN * ldw * 4 > 0x7fffffff) return "gemm_f32: lda, ldw too large";
  return nullptr;
}

hipError_t gemm_f32(int epi, const float* A, int64_t lda, const float* W, int64_t ldw, int M, int N,
                    int K, const EpiArgs& ep, hipStream_t s, int version) {
  switch (epi) {
    case EPI_BF16: return launch<EPI_BF16>(A, lda, W, ldw, M, N, K, ep, s, version);
    case EPI_GELU_BF16: return launch<EPI_GELU_BF16>(A, lda, W, ldw, M, N, K, ep, s, version);
    case EPI_RESID_F32: return launch<EPI_RESID_F32>(A, lda, W, ldw, M, N, K, ep, s, version);
    case EPI_POS_F32: return launch<EPI_POS_F32>(A, lda, W, ldw, M, N, K, ep, s, version);
    case EPI_RESID_FFN: return launch<EPI_RESID_FFN>(A, lda, W, ldw, M, N, K, ep, s, version);
    case EPI_RELU_BF16: return launch<EPI_RELU_BF16>(A, lda, W, ldw, M, N, K, ep, s, version);
  }
  return hipErrorInvalidValue;
}

}  // namespace vp
