// bf16 MFMA GEMM for small M (the LvT text tower: Q queries x 65 tokens, M = 768 rows at the bench's
// 8 queries), same operation and epilogues as gemm_bf16.hip / gemm_bf16_w4.hip:
//
//   C[M,N] = A[M,K] . W[N,K]^T  (+ epilogue)     A, W bf16 row-major, fp32 accumulate
//
// Replaces, for the text tower's 12 causal layers (encoders.py:656-759): q|k|v (layers.py:433-499),
// post + residual (:736-745, :855), ffn_layer1 + ReLU and ffn_layer2 + residual (:370-425).
//
// Why a second kernel: the 256 x 256-tile kernels give M = 768 three tile rows, so a text GEMM runs
// on 12-48 of the 256 CUs for its whole K loop (one tile's K = 4096 loop on one CU for ffn_layer2).
// Here a 256-thread workgroup owns a 64 x 64 tile and its 4 waves split K four ways (each wave a
// 64 x 64 fp32 partial over K/4, 16 accumulators of v_mfma_f32_16x16x32_bf16), so M = 768 gives
// 144-768 workgroups.  Operands go global -> VGPRs in MFMA fragment order (lane: row l & 15, k-group
// l >> 4, 16 contiguous bytes; no LDS staging: every byte is read once per workgroup), two 64-deep
// K-steps in flight per wave.  The four partials meet in LDS (64 KiB) and are summed in a fixed
// order, so the result does not depend on timing.  W is the MFMA A operand, so a lane's accumulator
// holds 4 consecutive output columns of one row: the epilogue is gemm_epilogue.h's epi_store.
#include "gemm_epilogue.h"

namespace vp {

namespace {

constexpr int kSmT = 64;     // tile rows and columns
constexpr int kSmKStep = 64;  // K per register stage (two 32-deep MFMA steps)

typedef float f32x4_t __attribute__((ext_vector_type(4)));

struct Stage {
  bf16x8 a[2][4];  // [32-deep half][16-row block]
  bf16x8 w[2][4];
};

template <int EPI>
__global__ __launch_bounds__(256) void gemm_bf16_small_kernel(const bf16_t* __restrict__ A, int64_t lda,
                                                              const bf16_t* __restrict__ W, int64_t ldw, int M,
                                                              int N, int K, EpiArgs ep) {
  __shared__ f32x4_t red[4][16][64];  // [wave][block ni*4 + mi][lane]
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  // XCD-aware tile order: workgroup b runs on XCD b % 8, and each XCD takes a contiguous range of the
  // tiles ordered column-block-major, so an XCD's L2 holds a slice of W (about 1/8) plus A, instead of
  // every XCD pulling all of A and W through the fabric (the grid is 8 x the largest range)
  const int tilesM = M / kSmT;
  const int T = tilesM * (N / kSmT);
  const int xcd = blockIdx.x & 7;
  const int lo = (int)(((int64_t)xcd * T) >> 3), hi = (int)(((int64_t)(xcd + 1) * T) >> 3);
  const int t = lo + (int)(blockIdx.x >> 3);
  if (t >= hi) return;  // whole workgroup
  const int m0 = (t % tilesM) * kSmT;
  const int n0 = (t / tilesM) * kSmT;
  const int r = lane & 15;
  const int kq = (lane >> 4) * 8;
  const int kw = K / 4;  // this wave's K range (K % 256 == 0: a multiple of kSmKStep)
  const int kbeg = wv * kw, kend = kbeg + kw;
  const bf16_t* ap = A + (int64_t)(m0 + r) * lda + kq;
  const bf16_t* wp = W + (int64_t)(n0 + r) * ldw + kq;

  auto load = [&](Stage& st, int k) {
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        st.a[h][b] = *reinterpret_cast<const bf16x8*>(ap + (int64_t)b * 16 * lda + k + 32 * h);
        st.w[h][b] = *reinterpret_cast<const bf16x8*>(wp + (int64_t)b * 16 * ldw + k + 32 * h);
      }
  };
  f32x4_t acc[4][4];  // [ni][mi]: rows n0 + 16 ni + 4 (l >> 4) + i, column m0 + 16 mi + (l & 15) of C^T
#pragma unroll
  for (int ni = 0; ni < 4; ++ni)
#pragma unroll
    for (int mi = 0; mi < 4; ++mi) acc[ni][mi] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  auto compute = [&](const Stage& st) {
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int ni = 0; ni < 4; ++ni)
#pragma unroll
        for (int mi = 0; mi < 4; ++mi)
          acc[ni][mi] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(st.w[h][ni], st.a[h][mi], acc[ni][mi], 0, 0, 0);
  };

  // two register stages, the next one's loads issued before this one's MFMAs.  (Three stages two ahead,
  // with exact vmcnt waits -- fenced bursts or loads spread between the MFMAs -- measured 10-15 % slower
  // in the LvT-Large forward, profiles/r05/text_tower_small_gemm.txt)
  Stage s0, s1;
  int k = kbeg;
  load(s0, k);
  for (; k + 2 * kSmKStep <= kend; k += 2 * kSmKStep) {
    load(s1, k + kSmKStep);
    compute(s0);
    if (k + 2 * kSmKStep < kend) load(s0, k + 2 * kSmKStep);
    compute(s1);
  }
  if (k < kend) compute(s0);  // an odd number of stages: the last one is in s0

#pragma unroll
  for (int ni = 0; ni < 4; ++ni)
#pragma unroll
    for (int mi = 0; mi < 4; ++mi) red[wv][ni * 4 + mi][lane] = acc[ni][mi];
  __syncthreads();

  // wave wv finishes column block ni = wv: the four K partials summed in wave order
  const int n = n0 + 16 * wv + 4 * (lane >> 4);
  const float4 bias = *reinterpret_cast<const float4*>(ep.bias + n);
#pragma unroll
  for (int mi = 0; mi < 4; ++mi) {
    const int b = wv * 4 + mi;
    const f32x4_t s = ((red[0][b][lane] + red[1][b][lane]) + red[2][b][lane]) + red[3][b][lane];
    const int row = m0 + 16 * mi + r;
    const float keep = ep.rowpad ? 1.0f - ep.rowpad[row] : 1.0f;
    const float4 v = make_float4(s[0] + bias.x, s[1] + bias.y, s[2] + bias.z, s[3] + bias.w);
    epi_store<EPI>(ep, row, n, v, keep, epi_extra<EPI>(ep, row, n, N));
  }
}

template <int EPI>
hipError_t launch_small(const bf16_t* A, int64_t lda, const bf16_t* W, int64_t ldw, int M, int N, int K,
                        const EpiArgs& ep, hipStream_t s) {
  VP_NOTE_KERNEL(gemm_bf16_small_kernel<EPI>);
  const int64_t T = (int64_t)(M / kSmT) * (N / kSmT);
  const int64_t grid = 8 * ((T + 7) / 8);  // 8 x the largest per-XCD range ((x + 1) T / 8 - x T / 8 <= ceil(T / 8))
  hipLaunchKernelGGL(gemm_bf16_small_kernel<EPI>, dim3((unsigned)grid), dim3(256), 0, s, A, lda, W, ldw, M, N, K, ep);
  return hipGetLastError();
}

}  // namespace

bool gemm_bf16_small_ok(int epi, int M, int N, int K, int64_t lda, int64_t ldw) {
  const bool epi_ok = epi == EPI_BF16 || epi == EPI_GELU_BF16 || epi == EPI_RESID_F32 || epi == EPI_RESID_FFN ||
                      epi == EPI_RESID_BF16 || epi == EPI_RESID_FFN_BF16 || epi == EPI_RELU_BF16;
  return epi_ok && M > 0 && M % kSmT == 0 && N % kSmT == 0 && K % 256 == 0 && lda % 8 == 0 && ldw % 8 == 0 &&
         lda >= K && ldw >= K;
}

hipError_t gemm_bf16_small(int epi, const bf16_t* A, int64_t lda, const bf16_t* W, int64_t ldw, int M, int N, int K,
                           const EpiArgs& ep, hipStream_t s) {
  if (!gemm_bf16_small_ok(epi, M, N, K, lda, ldw)) return hipErrorInvalidValue;
  switch (epi) {
    case EPI_BF16: return launch_small<EPI_BF16>(A, lda, W, ldw, M, N, K, ep, s);
    case EPI_GELU_BF16: return launch_small<EPI_GELU_BF16>(A, lda, W, ldw, M, N, K, ep, s);
    case EPI_RESID_F32: return launch_small<EPI_RESID_F32>(A, lda, W, ldw, M, N, K, ep, s);
    case EPI_RESID_FFN: return launch_small<EPI_RESID_FFN>(A, lda, W, ldw, M, N, K, ep, s);
    case EPI_RESID_BF16: return launch_small<EPI_RESID_BF16>(A, lda, W, ldw, M, N, K, ep, s);
    case EPI_RESID_FFN_BF16: return launch_small<EPI_RESID_FFN_BF16>(A, lda, W, ldw, M, N, K, ep, s);
    case EPI_RELU_BF16: return launch_small<EPI_RELU_BF16>(A, lda, W, ldw, M, N, K, ep, s);
  }
  return hipErrorInvalidValue;
}

}  // namespace vp
