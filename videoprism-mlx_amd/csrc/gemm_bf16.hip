// bf16 MFMA GEMM with fused epilogues for every Dense/einsum on the encoder path.
//
//   C[M,N] = A[M,K] . W[N,K]^T  (+ epilogue)     A, W bf16 row-major, fp32 accumulate
//
// Replaces: patch_projection  (encoders.py:488-494, layers.py:273-313)
//           q/k/v projection  (layers.py:433-499, 720-722) as ONE fused N=3*D GEMM
//           post projection   (layers.py:736-745) + residual add (:855)
//           ffn_layer1 + GELU (layers.py:370-393) and ffn_layer2 + residual (:400-425)
//
// Structure (MI355X-specific):
//  * 256x256 output tile per 512-thread workgroup, 8 waves = 2 (M) x 4 (N), each wave
//    128x64 = 8x4 accumulators of v_mfma_f32_16x16x32_bf16 (128 acc VGPRs).
//  * K-tile BK=64 is computed in 4 "phases", one per wave quadrant (qm, qn) of 64x32,
//    order (0,0) (0,1) (1,1) (1,0): 16 MFMAs per phase.  LDS holds 2 K-tile buffers, each
//    split in 4 regions A0/A1 (tile rows with qm = 0/1) and B0/B1 (cols with qn = 0/1) of
//    16 KiB.  A region is restaged by global_load_lds two phases after its last ds_read,
//    so the only VMEM wait is a counted vmcnt(4) once per K-tile (never vmcnt(0) in
//    steady state) and LDS reads retire under the barrier wait.
//  * Each phase = [ds_reads + 2 glds] barrier [lgkmcnt(0) + 16 MFMA] barrier.  Waves 4-7
//    run one barrier behind waves 0-3, so on every SIMD one wave's MFMAs overlap its
//    partner's LDS reads and DMA issue.
//  * LDS images are lane-linear for glds; the bank swizzle chunk ^= (row>>1)&7 is applied
//    to the per-lane SOURCE address and undone on the ds_read_b128 (conflict-free for the
//    16x16x32 operand pattern).
//  * W is the MFMA "A" operand, so each lane's accumulator holds 4 consecutive N columns
//    of one M row (16-byte fp32 / 8-byte bf16 stores); epilogue loads are batched.
//  * Persistent grid (one workgroup per CU) with a K-tile stream that runs across tiles,
//    so the next tile's loads overlap this tile's epilogue; each XCD owns a contiguous
//    tile chunk (L2 locality for A panels and W).
#include "gemm_epilogue.h"

#include <cstdlib>
#include <cstring>

namespace vp {

namespace {

constexpr int BM = 256, BN = 256, BK = 64;
constexpr int kGemmThreads = 512;
constexpr int kRegion = 128 * BK * 2;       // 16 KiB
constexpr int kBuf = 4 * kRegion;           // A0 A1 B0 B1
constexpr int kGemmLds = 2 * kBuf;          // 131072 B
enum { RA0 = 0, RA1 = 1, RB0 = 2, RB1 = 3 };

__device__ __forceinline__ int swz(int row) { return (row >> 1) & 7; }

__device__ __forceinline__ bf16x8 lds_frag(const char* region, int row, int chunk) {
  return *reinterpret_cast<const bf16x8*>(region + row * 128 + ((chunk ^ swz(row)) << 4));
}


__device__ __forceinline__ void sched_fence() { __builtin_amdgcn_sched_barrier(0); }

// Persistent: grid = min(tiles, CUs).  The 8 XCDs each own a contiguous chunk of the
// (tm, tn) tile range (tn fastest) and their workgroups sweep it together, so A panels and
// W stay in that XCD's L2.  The K-tile stream is global over a workgroup's tiles: the
// glds of the next tile's first K-tiles are issued during the last K-tiles of the current
// one, and its epilogue runs while they are in flight (no per-tile pipeline drain).
template <int EPI>
__global__ __launch_bounds__(kGemmThreads, 2) void gemm_bf16_tn_kernel(
    const bf16_t* __restrict__ A, int64_t lda, const bf16_t* __restrict__ W, int64_t ldw, int M,
    int N, int K, EpiArgs ep) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tilesN = N / BN;
  const int T = (M / BM) * tilesN;
  const int G = gridDim.x;
  const int b = blockIdx.x;
  int first, stride, count;
  if ((G & 7) == 0) {
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
  if (count == 0) return;  // uniform over the workgroup
  const int lane = threadIdx.x & 63;
  const int w = wave_id();
  const int wm = w >> 2, wn = w & 3;
  const int nk = K / BK;
  const int total = count * nk;

  // per-lane element offsets of this wave's 2 glds pieces per region (tile-relative):
  // region q of A holds tile rows (rl>>6)*128 + q*64 + (rl&63); of B tile cols (rl>>5)*64 +
  // q*32 + (rl&31); chunk swizzle c = (lane&7) ^ swz(rl) applied to the source.
  int64_t offA[2][2], offB[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int rl = (w * 2 + i) * 8 + (lane >> 3);
    const int c = (lane & 7) ^ swz(rl);
#pragma unroll
    for (int qq = 0; qq < 2; ++qq) {
      offA[qq][i] = (int64_t)(((rl >> 6) << 7) + qq * 64 + (rl & 63)) * lda + c * 8;
      offB[qq][i] = (int64_t)(((rl >> 5) << 6) + qq * 32 + (rl & 31)) * ldw + c * 8;
    }
  }
  auto tile_of = [&](int g, int& tm, int& tn, int& kt) {
    const int j = g / nk;
    kt = g - j * nk;
    const int tile = first + j * stride;
    tm = tile / tilesN;
    tn = tile - tm * tilesN;
  };
  auto stage = [&](int region, int g) {
    int tm, tn, kt;
    tile_of(g, tm, tn, kt);
    char* dst = smem + (g & 1) * kBuf + region * kRegion + w * 2048;
    const bf16_t* base = region < 2 ? A + (int64_t)tm * BM * lda + kt * BK
                                    : W + (int64_t)tn * BN * ldw + kt * BK;
    const int64_t o0 = region == RA0 ? offA[0][0] : region == RA1 ? offA[1][0]
                     : region == RB0 ? offB[0][0] : offB[1][0];
    const int64_t o1 = region == RA0 ? offA[0][1] : region == RA1 ? offA[1][1]
                     : region == RB0 ? offB[0][1] : offB[1][1];
    __builtin_amdgcn_global_load_lds(VP_GLB_PTR(base + o0), VP_LDS_PTR(dst), 16, 0, 0);
    __builtin_amdgcn_global_load_lds(VP_GLB_PTR(base + o1), VP_LDS_PTR(dst + 1024), 16, 0, 0);
  };

  f32x4 acc[4][8];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int l16 = lane & 15, cq = lane >> 4;
  const int arow = wm * 64 + l16;   // local row inside an A region
  const int brow = wn * 32 + l16;   // local row inside a B region
  bf16x8 af[8], bf[4];
  auto read_A = [&](const char* reg) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) af[kk * 4 + mt] = lds_frag(reg, arow + mt * 16, kk * 4 + cq);
  };
  auto read_B = [&](const char* reg) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) bf[kk * 2 + nt] = lds_frag(reg, brow + nt * 16, kk * 4 + cq);
  };
  auto mma = [&](int qm, int qn) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int nt = 0; nt < 2; ++nt)
#pragma unroll
        for (int mt = 0; mt < 4; ++mt)
          acc[qn * 2 + nt][qm * 4 + mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
              bf[kk * 2 + nt], af[kk * 4 + mt], acc[qn * 2 + nt][qm * 4 + mt], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };
  auto lgkm0 = [] { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); };
  auto barrier = [] {
    sched_fence();
    __builtin_amdgcn_s_barrier();
    sched_fence();
  };

  // Region schedule (global K-tile g in buffer g&1; phases P1..P4 read A0+B0, B1, A1, B0):
  //   P1(g): glds A1(g+1)   P2(g): glds B0(g+1)   P3(g): glds A0(g+2)   P4(g): glds B1(g+2)
  // Every region is restaged >= 2 phases after its last ds_read (so reads need not be
  // retired before the barrier), and P4's counted vmcnt(4) leaves only the two newest
  // half-tiles in flight: all of K-tile g+1 has landed before the barrier into P1(g+1).
  stage(RA0, 0); stage(RB0, 0); stage(RB1, 0); stage(RA1, 0);
  if (total > 1) {
    stage(RA0, 1); stage(RB1, 1);
    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  barrier();
  if (wm == 1) barrier();  // stagger: waves 4-7 run one barrier behind

  int kt = 0, j = 0;
  for (int g = 0; g < total; ++g) {
    const char* cur = smem + (g & 1) * kBuf;
    const bool s1 = g + 1 < total, s2 = g + 2 < total;
    // P1: quadrant (0,0)
    read_A(cur + RA0 * kRegion);
    read_B(cur + RB0 * kRegion);
    if (s1) stage(RA1, g + 1);
    barrier();
    lgkm0();
    mma(0, 0);
    barrier();
    // P2: quadrant (0,1)
    read_B(cur + RB1 * kRegion);
    if (s1) stage(RB0, g + 1);
    barrier();
    lgkm0();
    mma(0, 1);
    barrier();
    // P3: quadrant (1,1)
    read_A(cur + RA1 * kRegion);
    if (s2) stage(RA0, g + 2);
    barrier();
    lgkm0();
    mma(1, 1);
    barrier();
    // P4: quadrant (1,0)
    read_B(cur + RB0 * kRegion);
    if (s2) {
      stage(RB1, g + 2);
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    barrier();
    lgkm0();
    mma(1, 0);
    barrier();
    if (++kt < nk) continue;
    kt = 0;

    // ---- epilogue of tile j: lane holds D[n = nb + 16*ng + 4*(lane>>4) + r][m = mb + 16*mg] ----
    const int tile = first + j * stride;
    ++j;
    const int m0 = (tile / tilesN) * BM, n0 = (tile % tilesN) * BN;
    const int mb = m0 + wm * 128 + l16;
    const int nbase = n0 + wn * 64 + cq * 4;
    using Tr = EpiTraits<EPI>;
    float keep[8];
#pragma unroll
    for (int mg = 0; mg < 8; ++mg) keep[mg] = 1.0f;
    if constexpr (Tr::kKeep) {
      if (ep.rowpad) {
#pragma unroll
        for (int mg = 0; mg < 8; ++mg) keep[mg] = 1.0f - ep.rowpad[mb + mg * 16];
      }
    }
#pragma unroll
    for (int ng = 0; ng < 4; ++ng) {
      const int n = nbase + ng * 16;
      const float4 bb = *reinterpret_cast<const float4*>(ep.bias + n);
      float4 ex[8];  // residual / position rows, all issued before the first store
#pragma unroll
      for (int mg = 0; mg < 8; ++mg) ex[mg] = epi_extra<EPI>(ep, mb + mg * 16, n, N);
#pragma unroll
      for (int mg = 0; mg < 8; ++mg) {
        const f32x4 a = acc[ng][mg];
        epi_store<EPI>(ep, mb + mg * 16, n, make_float4(a[0] + bb.x, a[1] + bb.y, a[2] + bb.z, a[3] + bb.w),
                       keep[mg], ex[mg]);
      }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int jj = 0; jj < 8; ++jj) acc[i][jj] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  if (wm == 0) barrier();  // balance the stagger barrier
}

int num_cus() { return device_cu_count(); }  // per device (vp_common.h)

template <int EPI>
hipError_t launch_one(const bf16_t* A, int64_t lda, const bf16_t* W, int64_t ldw, int M, int N,
                      int K, const EpiArgs& ep, hipStream_t s) {
  hipError_t e = ensure_dyn_lds((const void*)gemm_bf16_tn_kernel<EPI>, kGemmLds);
  if (e != hipSuccess) return e;
  const int tiles = (M / BM) * (N / BN);
  const int grid = tiles < num_cus() ? tiles : num_cus();
  VP_NOTE_KERNEL((gemm_bf16_tn_kernel<EPI>));
  hipLaunchKernelGGL((gemm_bf16_tn_kernel<EPI>), dim3(grid), dim3(kGemmThreads), kGemmLds, s, A, lda,
                     W, ldw, M, N, K, ep);
  return hipGetLastError();
}

}  // namespace

const char* gemm_bf16_check(int M, int N, int K, int64_t lda, int64_t ldw) {
  if (M <= 0 || N <= 0 || K <= 0) return "gemm: non-positive dimension";
  if (M % BM) return "gemm: M must be a multiple of 256";
  if (N % BN) return "gemm: N must be a multiple of 256";
  if (K % BK) return "gemm: K must be a multiple of 64";
  if (lda < K || ldw < K || (lda % 8) || (ldw % 8)) return "gemm: bad leading dimension";
  return nullptr;
}

hipError_t gemm_bf16(int epi, const bf16_t* A, int64_t lda, const bf16_t* W, int64_t ldw, int M,
                     int N, int K, const EpiArgs& ep, hipStream_t s) {
  switch (epi) {
    case EPI_BF16: return launch_one<EPI_BF16>(A, lda, W, ldw, M, N, K, ep, s);
    case EPI_GELU_BF16: return launch_one<EPI_GELU_BF16>(A, lda, W, ldw, M, N, K, ep, s);
    case EPI_RESID_F32: return launch_one<EPI_RESID_F32>(A, lda, W, ldw, M, N, K, ep, s);
    case EPI_POS_F32: return launch_one<EPI_POS_F32>(A, lda, W, ldw, M, N, K, ep, s);
    case EPI_RESID_FFN: return launch_one<EPI_RESID_FFN>(A, lda, W, ldw, M, N, K, ep, s);
    case EPI_RESID_BF16: return launch_one<EPI_RESID_BF16>(A, lda, W, ldw, M, N, K, ep, s);
    case EPI_POS_BF16: return launch_one<EPI_POS_BF16>(A, lda, W, ldw, M, N, K, ep, s);
    case EPI_RESID_FFN_BF16: return launch_one<EPI_RESID_FFN_BF16>(A, lda, W, ldw, M, N, K, ep, s);
  }
  return hipErrorInvalidValue;
}

// Kernel choice for the forward and vp_op_gemm: the 4-wave kernel wherever its 32-bit buffer
// offsets reach W (A past them runs in row ranges), except the fp32-residual
// epilogues at K < 1024 (text tower), where the 8-wave kernel measured faster.
hipError_t gemm_bf16_auto(int epi, const bf16_t* A, int64_t lda, const bf16_t* W, int64_t ldw, int M,
                          int N, int K, const EpiArgs& ep, hipStream_t s) {
  // (gemm_bf16_w4 walks an A past the 32-bit buffer range in row ranges; W must fit one range)
  const bool w4_ok = (uint64_t)N * (uint64_t)ldw * 2 < 0xFFFFFFF0ull;
  if (epi >= EPI_BF16_LN) return w4_ok ? gemm_bf16_w4(epi, A, lda, W, ldw, M, N, K, ep, s) : hipErrorInvalidValue;
  if (w4_ok && !((epi == EPI_RESID_F32 || epi == EPI_RESID_FFN) && K < 1024))
    return gemm_bf16_w4(epi, A, lda, W, ldw, M, N, K, ep, s);
  return gemm_bf16(epi, A, lda, W, ldw, M, N, K, ep, s);
}

}  // namespace vp
