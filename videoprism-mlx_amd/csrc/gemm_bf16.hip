// bf16 MFMA GEMM with fused epilogues for every Dense/einsum on the encoder path.
//
//   C[M,N] = A[M,K] . W[N,K]^T  (+ epilogue)     A, W bf16 row-major, fp32 accumulate
//
// Replaces: patch_projection  (encoders.py:488-494, layers.py:273-313)
//           q/k/v projection  (layers.py:433-499, 720-722) as ONE fused N=3*D GEMM
//           post projection   (layers.py:736-745) + residual add (:855)
//           ffn_layer1 + GELU (layers.py:370-393) and ffn_layer2 + residual (:400-425)
//
// Tile 256x256x64, 8 waves (2 M x 4 N), each wave 128x64 = 8x4 tiles of
// v_mfma_f32_16x16x32_bf16.  Operands are staged global->LDS by
// global_load_lds_dwordx4 (lane-linear LDS image; the bank swizzle is applied to the
// per-lane SOURCE address and undone on the ds_read_b128), double buffered (128 KiB).
// The MFMA is issued with W as the "A" operand so that each lane's accumulator
// holds 4 consecutive N columns of one M row: 16-byte fp32 / 8-byte bf16 stores.
// Workgroups are remapped so that each XCD walks a contiguous range of output
// tiles (bijective for any grid size): A panels and W stay in that XCD's L2.
#include "vp_common.h"
#include "vp_kernels.h"

namespace vp {

namespace {

constexpr int BM = 256, BN = 256, BK = 64;
constexpr int kGemmThreads = 512;
constexpr int kGemmLds = 2 * (BM + BN) * BK * 2;  // 131072 B

__device__ __forceinline__ int swz(int row) { return (row >> 1) & 7; }

__device__ __forceinline__ bf16x8 lds_frag(const char* base, int row, int chunk) {
  return *reinterpret_cast<const bf16x8*>(base + row * 128 + ((chunk ^ swz(row)) << 4));
}

template <int EPI>
__device__ __forceinline__ void epilogue_store(const EpiArgs& ep, int N, int m, int n, float v0,
                                               float v1, float v2, float v3) {
  if constexpr (EPI == EPI_BF16) {
    uint2 o = make_uint2(pack_bf16x2(v0, v1), pack_bf16x2(v2, v3));
    *reinterpret_cast<uint2*>(static_cast<bf16_t*>(ep.out) + (int64_t)m * ep.ldo + n) = o;
  } else if constexpr (EPI == EPI_GELU_BF16) {
    v0 = gelu_erf(v0); v1 = gelu_erf(v1); v2 = gelu_erf(v2); v3 = gelu_erf(v3);
    if (ep.rowpad) {
      const float keep = 1.0f - ep.rowpad[m];
      v0 *= keep; v1 *= keep; v2 *= keep; v3 *= keep;
    }
    uint2 o = make_uint2(pack_bf16x2(v0, v1), pack_bf16x2(v2, v3));
    *reinterpret_cast<uint2*>(static_cast<bf16_t*>(ep.out) + (int64_t)m * ep.ldo + n) = o;
  } else if constexpr (EPI == EPI_RESID_F32 || EPI == EPI_RESID_FFN) {
    if (ep.rowpad) {
      const float keep = 1.0f - ep.rowpad[m];
      v0 *= keep; v1 *= keep; v2 *= keep; v3 *= keep;
    }
    const float4 r = *reinterpret_cast<const float4*>(ep.resid + (int64_t)m * ep.ldr + n);
    *reinterpret_cast<float4*>(static_cast<float*>(ep.out) + (int64_t)m * ep.ldo + n) =
        make_float4(r.x + v0, r.y + v1, r.z + v2, r.w + v3);
  } else {  // EPI_POS_F32
    const float4 p =
        *reinterpret_cast<const float4*>(ep.pos + (int64_t)(m % ep.pos_rows) * N + n);
    *reinterpret_cast<float4*>(static_cast<float*>(ep.out) + (int64_t)m * ep.ldo + n) =
        make_float4(v0 + p.x, v1 + p.y, v2 + p.z, v3 + p.w);
  }
}

template <int EPI>
__global__ __launch_bounds__(kGemmThreads, 2) void gemm_bf16_tn_kernel(
    const bf16_t* __restrict__ A, int64_t lda, const bf16_t* __restrict__ W, int64_t ldw, int M,
    int N, int K, EpiArgs ep) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tilesN = N / BN;
  const int nwg = gridDim.x;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  const int wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  const int m0 = (wgid / tilesN) * BM, n0 = (wgid % tilesN) * BN;
  const int lane = threadIdx.x & 63;
  const int w = wave_id();
  const int wm = w >> 2, wn = w & 3;

  // per-lane source rows/chunks of this wave's 4 glds pieces (8 rows x 128 B each)
  const int srow = lane >> 3;
  const bf16_t* srcA[4];
  const bf16_t* srcB[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int rr = (w * 4 + i) * 8 + srow;
    const int c = (lane & 7) ^ swz(rr);
    srcA[i] = A + (int64_t)(m0 + rr) * lda + c * 8;
    srcB[i] = W + (int64_t)(n0 + rr) * ldw + c * 8;
  }
  auto stage = [&](int buf, int k0) {
    char* baseA = smem + buf * 65536;
    char* baseB = baseA + 32768;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int piece = (w * 4 + i) * 1024;
      __builtin_amdgcn_global_load_lds(VP_GLB_PTR(srcA[i] + k0), VP_LDS_PTR(baseA + piece), 16, 0, 0);
      __builtin_amdgcn_global_load_lds(VP_GLB_PTR(srcB[i] + k0), VP_LDS_PTR(baseB + piece), 16, 0, 0);
    }
  };

  f32x4 acc[4][8];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = K / BK;
  stage(0, 0);
  wait_vmcnt0();
  __syncthreads();
  const int arow = wm * 128 + (lane & 15);
  const int brow = wn * 64 + (lane & 15);
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) stage(cur ^ 1, (kt + 1) * BK);
    const char* bA = smem + cur * 65536;
    const char* bB = bA + 32768;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int c = kk * 4 + (lane >> 4);
      bf16x8 af[8], wf[4];
#pragma unroll
      for (int mt = 0; mt < 8; ++mt) af[mt] = lds_frag(bA, arow + mt * 16, c);
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) wf[nt] = lds_frag(bB, brow + nt * 16, c);
#pragma unroll
      for (int nt = 0; nt < 4; ++nt)
#pragma unroll
        for (int mt = 0; mt < 8; ++mt)
          acc[nt][mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[nt], af[mt], acc[nt][mt], 0, 0, 0);
    }
    wait_vmcnt0();
    __syncthreads();
  }

  // epilogue: lane holds D[n = nb + 4*(lane>>4) + r][m = mb + (lane&15)], r = 0..3
  const int mb = m0 + wm * 128 + (lane & 15);
  const int nb = n0 + wn * 64 + (lane >> 4) * 4;
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) {
    const int n = nb + nt * 16;
    const float4 b = *reinterpret_cast<const float4*>(ep.bias + n);
#pragma unroll
    for (int mt = 0; mt < 8; ++mt) {
      const f32x4 a = acc[nt][mt];
      epilogue_store<EPI>(ep, N, mb + mt * 16, n, a[0] + b.x, a[1] + b.y, a[2] + b.z, a[3] + b.w);
    }
  }
}

template <int EPI>
hipError_t launch_one(const bf16_t* A, int64_t lda, const bf16_t* W, int64_t ldw, int M, int N,
                      int K, const EpiArgs& ep, hipStream_t s) {
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute((const void*)gemm_bf16_tn_kernel<EPI>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, kGemmLds);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  const int grid = (M / BM) * (N / BN);
  hipLaunchKernelGGL(gemm_bf16_tn_kernel<EPI>, dim3(grid), dim3(kGemmThreads), kGemmLds, s, A, lda,
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
  }
  return hipErrorInvalidValue;
}

}  // namespace vp
