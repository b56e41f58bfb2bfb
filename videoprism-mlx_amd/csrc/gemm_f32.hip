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

template <int EPI>
__device__ __forceinline__ void epi_f32(const EpiArgs& ep, int N, int m, int n, float v0, float v1,
                                        float v2, float v3) {
  float* out = static_cast<float*>(ep.out) + (int64_t)m * ep.ldo + n;
  if constexpr (EPI == EPI_BF16) {
    *reinterpret_cast<float4*>(out) = make_float4(v0, v1, v2, v3);
  } else if constexpr (EPI == EPI_GELU_BF16 || EPI == EPI_RELU_BF16) {
    if constexpr (EPI == EPI_GELU_BF16) {
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

template <int EPI>
hipError_t launch(const float* A, int64_t lda, const float* W, int64_t ldw, int M, int N, int K,
                  const EpiArgs& ep, hipStream_t s) {
  VP_NOTE_KERNEL(gemm_f32_kernel<EPI>);
  hipLaunchKernelGGL(gemm_f32_kernel<EPI>, dim3((M / TM) * (N / TN)), dim3(256), 0, s, A, lda, W,
                     ldw, M, N, K, ep);
  return hipGetLastError();
}

}  // namespace

const char* gemm_f32_check(int M, int N, int K) {
  if (M <= 0 || N <= 0 || K <= 0) return "gemm_f32: non-positive dimension";
  if (M % TM) return "gemm_f32: M must be a multiple of 128";
  if (N % TN) return "gemm_f32: N must be a multiple of 128";
  if (K % TK) return "gemm_f32: K must be a multiple of 16";
  return nullptr;
}

hipError_t gemm_f32(int epi, const float* A, int64_t lda, const float* W, int64_t ldw, int M, int N,
                    int K, const EpiArgs& ep, hipStream_t s) {
  switch (epi) {
    case EPI_BF16: return launch<EPI_BF16>(A, lda, W, ldw, M, N, K, ep, s);
    case EPI_GELU_BF16: return launch<EPI_GELU_BF16>(A, lda, W, ldw, M, N, K, ep, s);
    case EPI_RESID_F32: return launch<EPI_RESID_F32>(A, lda, W, ldw, M, N, K, ep, s);
    case EPI_POS_F32: return launch<EPI_POS_F32>(A, lda, W, ldw, M, N, K, ep, s);
    case EPI_RESID_FFN: return launch<EPI_RESID_FFN>(A, lda, W, ldw, M, N, K, ep, s);
    case EPI_RELU_BF16: return launch<EPI_RELU_BF16>(A, lda, W, ldw, M, N, K, ep, s);
  }
  return hipErrorInvalidValue;
}

}  // namespace vp
