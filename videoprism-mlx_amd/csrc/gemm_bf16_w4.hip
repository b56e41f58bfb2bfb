// bf16 GEMM, 4-wave decomposition (one wave per SIMD, 128x128 per wave).
//
//   C[M,N] = A[M,K] . W[N,K]^T  (+ epilogue), 256x256 tile, BK = 64, 256 threads.
//
// Why this shape on MI355X (measured, tools/gemm_bench.py ablations):
// with 8 waves of 128x64 the CU reads 224 KiB of LDS per K-tile and the LDS-DMA issue of
// the staging loads competes with it; removing the DMA instructions alone was worth +32%.
// 4 waves of 128x128 read 128 KiB per K-tile, and v_mfma_f32_32x32x16_bf16 (32 cycles,
// issue held for 8) leaves 24 free issue cycles per MFMA in which each wave's 16
// global_load_lds and 32 ds_read_b128 per K-tile are interleaved.  The 256 fp32
// accumulators live in the AGPR half of the 512-entry register file.
//
// Pipeline: 2 LDS buffers (2 x 64 KiB).  K-tile t+1 is staged into the other buffer while
// K-tile t is computed (its buffer was released by the barrier that ended t-1); fragments
// of k-step s+1 are read while the 16 MFMAs of k-step s run; one vmcnt(0) + barrier per
// K-tile.  Same source-side bank swizzle and epilogue conventions as gemm_bf16.hip.
#include <type_traits>

#include "vp_common.h"
#include "vp_kernels.h"

namespace vp {

namespace {

constexpr int BM = 256, BN = 256, BK = 64;
constexpr int kThreads = 256;
constexpr int kTileBytes = BM * BK * 2;      // 32 KiB per operand per K-tile
constexpr int kBuf = 2 * kTileBytes;         // A then W
constexpr int kLds = 2 * kBuf;               // 128 KiB

__device__ __forceinline__ int swz(int row) { return (row >> 1) & 7; }

__device__ __forceinline__ bf16x8 frag(const char* base, int row, int chunk) {
  return *reinterpret_cast<const bf16x8*>(base + row * 128 + ((chunk ^ swz(row)) << 4));
}

__device__ __forceinline__ float gelu_fast(float x) {
  const float ax = fabsf(x);
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f * 0.70710678118654752f, ax, 1.0f));
  float p = fmaf(t, 1.061405429f, -1.453152027f);
  p = fmaf(t, p, 1.421413741f);
  p = fmaf(t, p, -0.284496736f);
  p = fmaf(t, p, 0.254829592f);
  p *= t;
  const float e = __builtin_amdgcn_exp2f(x * x * (-0.5f * 1.4426950408889634f));
  return 0.5f * fmaf(ax, fmaf(-p, e, 1.0f), x);
}

template <int EPI>
__global__ __launch_bounds__(kThreads, 1) void gemm_bf16_w4_kernel(
    const bf16_t* __restrict__ A, int64_t lda, const bf16_t* __restrict__ W, int64_t ldw, int M,
    int N, int K, EpiArgs ep) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tilesN = N / BN;
  const int nwg = gridDim.x;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int m0 = (wgid / tilesN) * BM, n0 = (wgid % tilesN) * BN;
  const int lane = threadIdx.x & 63;
  const int w = wave_id();
  const int wm = w >> 1, wn = w & 1;

  // staging: wave w fills pieces w*8 + i (i = 0..7) of A and of W; piece = 8 rows x 128 B.
  // Row of piece i: w*64 + i*8 + (lane>>3); its swizzled chunk depends only on i & 1.
  const int r0 = w * 64 + (lane >> 3);
  const int c_even = (lane & 7) ^ swz(r0);
  const int c_odd = (lane & 7) ^ swz(r0 + 8);
  const bf16_t* a_even = A + (int64_t)(m0 + r0) * lda + c_even * 8;
  const bf16_t* a_odd = A + (int64_t)(m0 + r0 + 8) * lda + c_odd * 8;
  const bf16_t* w_even = W + (int64_t)(n0 + r0) * ldw + c_even * 8;
  const bf16_t* w_odd = W + (int64_t)(n0 + r0 + 8) * ldw + c_odd * 8;
  const int64_t a16 = 16 * lda, w16 = 16 * ldw;
  // piece p (0..15) of this wave for one K-tile: p < 8 -> A piece p, else W piece p-8
  auto stage_piece = [&](int buf, int kt, int p) {
    const int i = p & 7;
    const bool isW = p >= 8;
    const bf16_t* src = isW ? ((i & 1) ? w_odd : w_even) + (i >> 1) * w16
                            : ((i & 1) ? a_odd : a_even) + (i >> 1) * a16;
    char* dst = smem + buf * kBuf + (isW ? kTileBytes : 0) + (w * 8 + i) * 1024;
    __builtin_amdgcn_global_load_lds(VP_GLB_PTR(src + kt * BK), VP_LDS_PTR(dst), 16, 0, 0);
  };

  f32x16 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x16{};

  const int l32 = lane & 31, hi = lane >> 5;
  const int arow = wm * 128 + l32;
  const int wrow = wn * 128 + l32;
  bf16x8 fa[2][4], fw[2][4];
  auto read_frags = [&](const char* buf, int ks, bf16x8 (&a)[4], bf16x8 (&b)[4]) {
    const int c = ks * 2 + hi;
#pragma unroll
    for (int t = 0; t < 4; ++t) a[t] = frag(buf, arow + t * 32, c);
#pragma unroll
    for (int t = 0; t < 4; ++t) b[t] = frag(buf + kTileBytes, wrow + t * 32, c);
  };
  auto mma = [&](const bf16x8 (&a)[4], const bf16x8 (&b)[4]) {
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
        acc[nt][mt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b[nt], a[mt], acc[nt][mt], 0, 0, 0);
  };

  const int nk = K / BK;
#pragma unroll
  for (int p = 0; p < 16; ++p) stage_piece(0, 0, p);
  wait_vmcnt0();
  __builtin_amdgcn_s_barrier();

  // One K-tile: k-step ks runs its 16 MFMAs while the fragments of ks+1 (8 ds_read_b128)
  // and 4 of the 16 staging DMAs of K-tile t+1 are issued between them; the interleave is
  // pinned with sched_group_barrier so that no LDS wait lands in front of an MFMA block.
  auto ktile = [&](int t, auto pre_tag) {
    constexpr bool kPre = decltype(pre_tag)::value;
    const char* cur = smem + (t & 1) * kBuf;
    const int nb = (t & 1) ^ 1;
    read_frags(cur, 0, fa[0], fw[0]);
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      if (ks < 3) read_frags(cur, ks + 1, fa[(ks + 1) & 1], fw[(ks + 1) & 1]);
      if constexpr (kPre) {
#pragma unroll
        for (int p = 0; p < 4; ++p) stage_piece(nb, t + 1, ks * 4 + p);
      }
      mma(fa[ks & 1], fw[ks & 1]);
      // next k-step's 8 DS reads first (other register set), then 16 MFMA with the 4 DMA
      // issued behind the first four
      if (ks < 3) __builtin_amdgcn_sched_group_barrier(0x100, 8, 0);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        if (kPre) __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
      }
      __builtin_amdgcn_sched_group_barrier(0x008, 12, 0);
    }
    wait_vmcnt0();
    __builtin_amdgcn_s_barrier();
  };
  for (int t = 0; t + 1 < nk; ++t) ktile(t, std::true_type{});
  ktile(nk - 1, std::false_type{});

  // ---- epilogue: acc[nt][mt][r] = D[n = nb + nt*32 + 8*(r>>2) + 4*hi + (r&3)][m = mb + mt*32]
  const int mb = m0 + wm * 128 + l32;
  const int nbase = n0 + wn * 128 + 4 * hi;
  float keep[4] = {1.f, 1.f, 1.f, 1.f};
  if constexpr (EPI == EPI_GELU_BF16 || EPI == EPI_RESID_F32 || EPI == EPI_RESID_FFN) {
    if (ep.rowpad) {
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) keep[mt] = 1.0f - ep.rowpad[mb + mt * 32];
    }
  }
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) {
#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4) {
      const int n = nbase + nt * 32 + g4 * 8;
      const float4 bb = *reinterpret_cast<const float4*>(ep.bias + n);
      if constexpr (EPI == EPI_BF16 || EPI == EPI_GELU_BF16) {
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) {
          const f32x16& a = acc[nt][mt];
          float v0 = a[4 * g4] + bb.x, v1 = a[4 * g4 + 1] + bb.y, v2 = a[4 * g4 + 2] + bb.z,
                v3 = a[4 * g4 + 3] + bb.w;
          if constexpr (EPI == EPI_GELU_BF16) {
            v0 = gelu_fast(v0) * keep[mt]; v1 = gelu_fast(v1) * keep[mt];
            v2 = gelu_fast(v2) * keep[mt]; v3 = gelu_fast(v3) * keep[mt];
          }
          *reinterpret_cast<uint2*>(static_cast<bf16_t*>(ep.out) + (int64_t)(mb + mt * 32) * ep.ldo + n) =
              make_uint2(pack_bf16x2(v0, v1), pack_bf16x2(v2, v3));
        }
      } else if constexpr (EPI == EPI_RESID_F32 || EPI == EPI_RESID_FFN) {
        float4 r[4];
#pragma unroll
        for (int mt = 0; mt < 4; ++mt)
          r[mt] = *reinterpret_cast<const float4*>(ep.resid + (int64_t)(mb + mt * 32) * ep.ldr + n);
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) {
          const f32x16& a = acc[nt][mt];
          const float k = keep[mt];
          *reinterpret_cast<float4*>(static_cast<float*>(ep.out) + (int64_t)(mb + mt * 32) * ep.ldo + n) =
              make_float4(r[mt].x + (a[4 * g4] + bb.x) * k, r[mt].y + (a[4 * g4 + 1] + bb.y) * k,
                          r[mt].z + (a[4 * g4 + 2] + bb.z) * k, r[mt].w + (a[4 * g4 + 3] + bb.w) * k);
        }
      } else {  // EPI_POS_F32
        float4 pp[4];
#pragma unroll
        for (int mt = 0; mt < 4; ++mt)
          pp[mt] = *reinterpret_cast<const float4*>(ep.pos + (int64_t)((mb + mt * 32) % ep.pos_rows) * N + n);
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) {
          const f32x16& a = acc[nt][mt];
          *reinterpret_cast<float4*>(static_cast<float*>(ep.out) + (int64_t)(mb + mt * 32) * ep.ldo + n) =
              make_float4(a[4 * g4] + bb.x + pp[mt].x, a[4 * g4 + 1] + bb.y + pp[mt].y,
                          a[4 * g4 + 2] + bb.z + pp[mt].z, a[4 * g4 + 3] + bb.w + pp[mt].w);
        }
      }
    }
  }
}

template <int EPI>
hipError_t launch_w4(const bf16_t* A, int64_t lda, const bf16_t* W, int64_t ldw, int M, int N,
                     int K, const EpiArgs& ep, hipStream_t s) {
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute((const void*)gemm_bf16_w4_kernel<EPI>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, kLds);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  const int grid = (M / BM) * (N / BN);
  hipLaunchKernelGGL((gemm_bf16_w4_kernel<EPI>), dim3(grid), dim3(kThreads), kLds, s, A, lda, W,
                     ldw, M, N, K, ep);
  return hipGetLastError();
}

}  // namespace

hipError_t gemm_bf16_w4(int epi, const bf16_t* A, int64_t lda, const bf16_t* W, int64_t ldw, int M,
                        int N, int K, const EpiArgs& ep, hipStream_t s) {
  switch (epi) {
    case EPI_BF16: return launch_w4<EPI_BF16>(A, lda, W, ldw, M, N, K, ep, s);
    case EPI_GELU_BF16: return launch_w4<EPI_GELU_BF16>(A, lda, W, ldw, M, N, K, ep, s);
    case EPI_RESID_F32: return launch_w4<EPI_RESID_F32>(A, lda, W, ldw, M, N, K, ep, s);
    case EPI_POS_F32: return launch_w4<EPI_POS_F32>(A, lda, W, ldw, M, N, K, ep, s);
    case EPI_RESID_FFN: return launch_w4<EPI_RESID_FFN>(A, lda, W, ldw, M, N, K, ep, s);
  }
  return hipErrorInvalidValue;
}

}  // namespace vp
