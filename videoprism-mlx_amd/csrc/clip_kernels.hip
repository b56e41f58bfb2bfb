// Kernels of the LvT video-text path besides attention.
//
// Contrastive pooler (AttenTokenPoolingLayer, layers.py:1044-1136; num_queries = 1, no logit
// cap, per-dim scale on, paddings None).  Its single query is a parameter, so the projected
// and scaled query q~[h] (layers.py:502-527, :676-681) is a constant and the key projection
// folds into it on the host:  logit[g,h,s] = x[g,s,:].U[h,:] + q~[h].bk[h], U[h] = Wk[:,h,:] q~[h].
// The constant q~[h].bk[h] shifts every logit of a row equally and cancels in the softmax, so
// the pooler never materialises K (B*S x 4D) or V: with p = softmax(logit) and sum_s p = 1,
//   enc[g,h,:] = sum_s p[g,h,s] (x[g,s,:] Wv[:,h,:] + bv[h]) = z[g,h,:] Wv[:,h,:] + bv[h],
//   z[g,h,:]   = sum_s p[g,h,s] x[g,s,:]
// which turns the two [S x D] x [D x 4D] projections per clip into two streaming passes over x
// (HBM-bound: pool_logits, pool_wsum) and [G x D] x [D x dh] matrix products (small_gemm).
//   pool_logits : logits[g][h][s] = x[g*S+s] . U[h]       (bf16: skinny MFMA GEMM; fp32: U in LDS)
//   pool_stats  : (max, 1/sum exp(l - max)) per (g, h)    (fp32 softmax, layers.py:650-654)
//   pool_wsum   : zpart[g][c][h][:] = sum over the c-th 256-row chunk of p * x
//   pool_reduce : z[g][h][:] = sum_c zpart
//   small_gemm  : out[m][n] = A[m][:] . Wt[:][n] + bias[n], batched (enc per head, then post)
//   ln_l2_rows  : LayerNorm (layers.py:208-270) and/or _l2_normalize (encoders.py:50-67), fp32
// Text tower: text_embed = Embedding(ids)*sqrt(D) + sinusoidal PositionalEmbedding, with the
// CLS token appended (encoders.py:190-266, :700-740).  similarity = video_emb . text_emb^T.
#include "vp_common.h"
#include "vp_kernels.h"

namespace vp {

namespace {

__device__ __forceinline__ float ldx(const void* p, int in_bf16, int64_t i) {
  return in_bf16 ? bf2f(static_cast<const bf16_t*>(p)[i]) : static_cast<const float*>(p)[i];
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
  return v;
}

// block (256 threads) reductions through LDS
__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  return red[0] + red[1] + red[2] + red[3];
}

__device__ __forceinline__ float block_max(float v, float* red) {
  v = wave_max(v);
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  return fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
}

constexpr int kPlRows = 64;  // rows per workgroup (16 per wave)

__global__ __launch_bounds__(256) void pool_logits_kernel(const void* __restrict__ x, int in_bf16, int64_t rows,
                                                          int S, int D, const float* __restrict__ U, int H,
                                                          float* __restrict__ logits) {
  extern __shared__ float Us[];  // [H][D]
  for (int i = threadIdx.x; i < H * D; i += 256) Us[i] = U[i];
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int nj = D >> 6;
  for (int rr = 0; rr < kPlRows / 4; ++rr) {
    const int64_t r = (int64_t)blockIdx.x * kPlRows + w * (kPlRows / 4) + rr;
    if (r >= rows) break;  // uniform per wave
    float xv[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) xv[j] = j < nj ? ldx(x, in_bf16, r * D + lane + 64 * j) : 0.0f;
    const int64_t g = r / S, s = r % S;
    for (int h = 0; h < H; ++h) {
      float a = 0.0f;
#pragma unroll
      for (int j = 0; j < 16; ++j)
        if (j < nj) a = fmaf(xv[j], Us[h * D + lane + 64 * j], a);
      a = wave_sum(a);
      if (lane == 0) logits[(g * H + h) * S + s] = a;
    }
  }
}

// bf16 tokens: logits as a skinny GEMM on v_mfma_f32_32x32x16_bf16.  One wave owns 32 rows;
// the B operand is Ut [32][D] bf16 = (U_hi | U_lo | 0) with U = U_hi + U_lo split on the host, so
// the fp32 U survives the bf16 operands to ~2^-16 relative; lane c < H adds column H + c.
__global__ __launch_bounds__(256) void pool_logits_mfma_kernel(const bf16_t* __restrict__ x, int64_t rows, int S,
                                                               int D, const bf16_t* __restrict__ Ut, int H,
                                                               float* __restrict__ logits) {
  const int lane = threadIdx.x & 63;
  const int64_t r0 = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * 32;
  if (r0 >= rows) return;  // whole wave
  const int i = lane & 31, half = lane >> 5;
  const bf16_t* ap = x + (r0 + i) * D + 8 * half;
  const bf16_t* bp = Ut + (int64_t)i * D + 8 * half;
  f32x16 acc = {};
  const int nt = D >> 4;
  int t = 0;
  for (; t + 8 <= nt; t += 8) {
    bf16x8 a[8], b[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      a[u] = *reinterpret_cast<const bf16x8*>(ap + 16 * (t + u));
      b[u] = *reinterpret_cast<const bf16x8*>(bp + 16 * (t + u));
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[u], b[u], acc, 0, 0, 0);
  }
  for (; t < nt; ++t) {
    const bf16x8 a = *reinterpret_cast<const bf16x8*>(ap + 16 * t);
    const bf16x8 b = *reinterpret_cast<const bf16x8*>(bp + 16 * t);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc, 0, 0, 0);
  }
  // acc[r] = C[row = (r&3) + 8(r>>2) + 4*half][col = i]
  const int64_t g = r0 / S;
  const int64_t s0 = r0 % S;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const float v = acc[r] + __shfl_down(acc[r], H);
    if (i < H) logits[(g * H + i) * S + s0 + (r & 3) + 8 * (r >> 2) + 4 * half] = v;
  }
}

__global__ __launch_bounds__(256) void pool_stats_kernel(const float* __restrict__ logits, int S,
                                                         float* __restrict__ stats) {
  __shared__ float red[4];
  const float* l = logits + (int64_t)blockIdx.x * S;
  float m = -INFINITY;
  for (int s = threadIdx.x; s < S; s += 256) m = fmaxf(m, l[s]);
  m = block_max(m, red);
  float sum = 0.0f;
  for (int s = threadIdx.x; s < S; s += 256) sum += expf(l[s] - m);
  sum = block_sum(sum, red);
  if (threadIdx.x == 0) {
    stats[2 * blockIdx.x] = m;
    stats[2 * blockIdx.x + 1] = 1.0f / sum;
  }
}

constexpr int kPwRows = 256;  // rows per chunk
constexpr int kPwMaxH = 16;

// zpart[g][c][h][d] = sum over rows of chunk c of p[g,h,s] x[g*S+s][d]: a workgroup owns one
// (g, 256-row chunk, 256-column quarter) with 128 threads; a thread owns two adjacent columns (one 4-byte
// bf16 pair / 8-byte fp32 pair per row) and all 16 head sums of each, the probabilities of the chunk sit in
// LDS (float4 broadcast reads).  Each column is summed over the rows in row order.
__global__ __launch_bounds__(128) void pool_wsum_kernel(const void* __restrict__ x, int in_bf16, int S, int D,
                                                        int H, const float* __restrict__ logits,
                                                        const float* __restrict__ stats, int C,
                                                        float* __restrict__ zpart) {
  __shared__ __attribute__((aligned(16))) float ps[kPwRows][kPwMaxH];
  const int nq = D >> 8;
  const int q = blockIdx.x % nq;
  const int gc = blockIdx.x / nq;
  const int g = gc / C;
  const int c = gc % C;
  const int r0 = c * kPwRows;
  const int nr = S - r0 < kPwRows ? S - r0 : kPwRows;
  for (int i = threadIdx.x; i < kPwRows * kPwMaxH; i += 128) {
    const int r = i / kPwMaxH, h = i % kPwMaxH;
    float p = 0.0f;
    if (r < nr && h < H) {
      const int64_t gh = (int64_t)g * H + h;
      p = __expf(logits[gh * S + r0 + r] - stats[2 * gh]) * stats[2 * gh + 1];
    }
    ps[r][h] = p;
  }
  __syncthreads();
  const int d = q * 256 + 2 * threadIdx.x;
  float acc0[kPwMaxH], acc1[kPwMaxH];
#pragma unroll
  for (int h = 0; h < kPwMaxH; ++h) acc0[h] = acc1[h] = 0.0f;
  const int64_t rowbase = (int64_t)g * S + r0;
  auto ld2 = [&](int r) -> float2 {
    const int64_t i = (rowbase + r) * D + d;
    if (in_bf16) {
      const uint32_t u = *reinterpret_cast<const uint32_t*>(static_cast<const bf16_t*>(x) + i);
      return make_float2(__uint_as_float(u << 16), __uint_as_float(u & 0xffff0000u));
    }
    return *reinterpret_cast<const float2*>(static_cast<const float*>(x) + i);
  };
  auto row = [&](int r, float2 xv) {
    const float4* pr = reinterpret_cast<const float4*>(ps[r]);
#pragma unroll
    for (int h4 = 0; h4 < kPwMaxH / 4; ++h4) {
      const float4 p = pr[h4];
      acc0[4 * h4] = fmaf(p.x, xv.x, acc0[4 * h4]);
      acc0[4 * h4 + 1] = fmaf(p.y, xv.x, acc0[4 * h4 + 1]);
      acc0[4 * h4 + 2] = fmaf(p.z, xv.x, acc0[4 * h4 + 2]);
      acc0[4 * h4 + 3] = fmaf(p.w, xv.x, acc0[4 * h4 + 3]);
      acc1[4 * h4] = fmaf(p.x, xv.y, acc1[4 * h4]);
      acc1[4 * h4 + 1] = fmaf(p.y, xv.y, acc1[4 * h4 + 1]);
      acc1[4 * h4 + 2] = fmaf(p.z, xv.y, acc1[4 * h4 + 2]);
      acc1[4 * h4 + 3] = fmaf(p.w, xv.y, acc1[4 * h4 + 3]);
    }
  };
  int r = 0;
  for (; r + 16 <= nr; r += 16) {
    float2 xv[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) xv[u] = ld2(r + u);
#pragma unroll
    for (int u = 0; u < 16; ++u) row(r + u, xv[u]);
  }
  for (; r < nr; ++r) row(r, ld2(r));
  float* zp = zpart + ((int64_t)g * C + c) * H * D + d;
#pragma unroll
  for (int h = 0; h < kPwMaxH; ++h)
    if (h < H) *reinterpret_cast<float2*>(zp + (int64_t)h * D) = make_float2(acc0[h], acc1[h]);
}

__global__ __launch_bounds__(256) void pool_reduce_kernel(const float* __restrict__ zpart, int C, int64_t HD,
                                                          int64_t total, float* __restrict__ z) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  const int64_t g = i / HD, e = i % HD;
  const float* p = zpart + g * C * HD + e;
  float s = 0.0f;
  for (int c = 0; c < C; ++c) s += p[(int64_t)c * HD];
  z[i] = s;
}

// out[m][n] = A[m][:] . Wt[:][n] + bias[n] for small M (pooled vectors): a workgroup owns 64
// columns x 32 rows and splits K four ways (one quarter per wave, partial sums combined through
// LDS); A^T chunks are staged in LDS and read as float4 broadcasts, Wt rows are coalesced.
constexpr int kSgM = 32;
constexpr int kSgN = 64;
constexpr int kSgK = 128;

__global__ __launch_bounds__(256) void small_gemm_kernel(const float* __restrict__ A, int64_t lda, int64_t sA,
                                                         const float* __restrict__ Wt, int64_t sW,
                                                         const float* __restrict__ bias, int64_t sB,
                                                         float* __restrict__ out, int64_t ldo, int64_t sO, int M,
                                                         int N, int K) {
  __shared__ __attribute__((aligned(16))) float At[kSgK][kSgM];  // A^T chunk
  __shared__ float red[3][kSgM][kSgN];
  const int bz = blockIdx.z;
  A += bz * sA;
  Wt += bz * sW;
  out += bz * sO;
  const float* bb = bias ? bias + bz * sB : nullptr;
  const int col = threadIdx.x & 63;
  const int quarter = threadIdx.x >> 6;  // wave
  const int n = blockIdx.x * kSgN + col;
  const int m0 = blockIdx.y * kSgM;
  float acc[kSgM];
#pragma unroll
  for (int i = 0; i < kSgM; ++i) acc[i] = 0.0f;
  for (int k0 = 0; k0 < K; k0 += kSgK) {
    __syncthreads();
    for (int i = threadIdx.x; i < kSgM * kSgK; i += 256) {
      const int mi = i / kSgK, kk = i % kSgK;
      At[kk][mi] = (m0 + mi < M && k0 + kk < K) ? A[(int64_t)(m0 + mi) * lda + k0 + kk] : 0.0f;
    }
    __syncthreads();
    if (n < N) {
      const int kq0 = quarter * (kSgK / 4);
#pragma unroll 4
      for (int kk = kq0; kk < kq0 + kSgK / 4; ++kk) {
        const float w = k0 + kk < K ? Wt[(int64_t)(k0 + kk) * N + n] : 0.0f;
        const float4* ar = reinterpret_cast<const float4*>(At[kk]);
#pragma unroll
        for (int i4 = 0; i4 < kSgM / 4; ++i4) {
          const float4 a = ar[i4];
          acc[4 * i4] = fmaf(a.x, w, acc[4 * i4]);
          acc[4 * i4 + 1] = fmaf(a.y, w, acc[4 * i4 + 1]);
          acc[4 * i4 + 2] = fmaf(a.z, w, acc[4 * i4 + 2]);
          acc[4 * i4 + 3] = fmaf(a.w, w, acc[4 * i4 + 3]);
        }
      }
    }
  }
  if (quarter > 0) {
#pragma unroll
    for (int i = 0; i < kSgM; ++i) red[quarter - 1][i][col] = acc[i];
  }
  __syncthreads();
  if (quarter > 0 || n >= N) return;
  const float b = bb ? bb[n] : 0.0f;
#pragma unroll
  for (int i = 0; i < kSgM; ++i)
    if (m0 + i < M) out[(int64_t)(m0 + i) * ldo + n] = acc[i] + red[0][i][col] + red[1][i][col] + red[2][i][col] + b;
}

// out[m][n] = bias[n] + sum_z part[z][m][n] in z order (small_gemm_splitk)
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const float* __restrict__ part, int splits, int64_t MN,
                                                            int N, const float* __restrict__ bias,
                                                            float* __restrict__ out, int64_t ldo) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= MN) return;
  float v = part[i];
  for (int z = 1; z < splits; ++z) v += part[z * MN + i];
  const int64_t m = i / N;
  const int n = (int)(i % N);
  out[m * ldo + n] = v + (bias ? bias[n] : 0.0f);
}

__global__ __launch_bounds__(256) void ln_l2_rows_kernel(const void* __restrict__ x, int in_bf16, int64_t stride,
                                                         int D, const float* __restrict__ gamma,
                                                         const float* __restrict__ beta, int do_l2,
                                                         float* __restrict__ out) {
  __shared__ float red[4];
  const int64_t r = blockIdx.x;
  float v[4];
  const int nj = (D + 255) >> 8;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int d = threadIdx.x + 256 * j;
    v[j] = (j < nj && d < D) ? ldx(x, in_bf16, r * stride + d) : 0.0f;
  }
  if (gamma) {
    float s = 0.0f;
#pragma unroll
    for (int j = 0; j < 4; ++j) s += v[j];
    const float mean = block_sum(s, red) / (float)D;
    float q = 0.0f;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int d = threadIdx.x + 256 * j;
      const float c = (j < nj && d < D) ? v[j] - mean : 0.0f;
      q = fmaf(c, c, q);
    }
    const float rstd = rsqrtf(block_sum(q, red) / (float)D + 1e-6f);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int d = threadIdx.x + 256 * j;
      if (j < nj && d < D) v[j] = (v[j] - mean) * rstd * gamma[d] + beta[d];
      else v[j] = 0.0f;
    }
  }
  if (do_l2) {
    float q = 0.0f;
#pragma unroll
    for (int j = 0; j < 4; ++j) q = fmaf(v[j], v[j], q);
    const float inv = 1.0f / sqrtf(block_sum(q, red) + 1e-12f);
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] *= inv;
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int d = threadIdx.x + 256 * j;
    if (j < nj && d < D) out[r * D + d] = v[j];
  }
}

__global__ __launch_bounds__(256) void text_embed_kernel(const int32_t* __restrict__ ids, int L, const void* table,
                                                         int table_bf16, int V, const float* __restrict__ cls,
                                                         const float* __restrict__ pos, float scale, int D,
                                                         void* out, int out_bf16, const float* __restrict__ pad_in,
                                                         float* __restrict__ pad_out) {
  const int64_t r = blockIdx.x;  // q * (L + 1) + t
  const int64_t q = r / (L + 1);
  const int t = (int)(r % (L + 1));
  // paddings with the CLS token's zero appended (encoders.py:737-740)
  if (threadIdx.x == 0) pad_out[r] = t < L ? pad_in[q * L + t] : 0.0f;
  int id = 0;
  if (t < L) {
    id = ids[q * L + t];
    id = id < 0 ? 0 : (id >= V ? V - 1 : id);  // jnp indexing clamps out-of-range ids
  }
  for (int d = threadIdx.x; d < D; d += 256) {
    const float e = t < L ? ldx(table, table_bf16, (int64_t)id * D + d) * scale + pos[(int64_t)t * D + d]
                          : cls[d] * scale;
    if (out_bf16) static_cast<bf16_t*>(out)[r * D + d] = f2bf(e);
    else static_cast<float*>(out)[r * D + d] = e;
  }
}

__global__ __launch_bounds__(256) void similarity_kernel(const float* __restrict__ a, const float* __restrict__ b,
                                                         int B, int Q, int D, float* __restrict__ out) {
  __shared__ float red[4];
  const int i = blockIdx.x / Q, j = blockIdx.x % Q;
  float s = 0.0f;
  for (int d = threadIdx.x; d < D; d += 256) s = fmaf(a[(int64_t)i * D + d], b[(int64_t)j * D + d], s);
  s = block_sum(s, red);
  if (threadIdx.x == 0) out[blockIdx.x] = s;
}

}  // namespace

hipError_t pool_logits(const void* x, int in_bf16, int64_t rows, int S, int D, const float* U, const bf16_t* Ut,
                       int H, float* logits, hipStream_t s) {
  if (D % 64 || D > 1024 || H < 1 || H > kPwMaxH || rows % S) return hipErrorInvalidValue;
  if (in_bf16 && Ut && S % 32 == 0) {
    const int64_t grid = (rows / 32 + 3) / 4;
    hipLaunchKernelGGL(pool_logits_mfma_kernel, dim3((unsigned)grid), dim3(256), 0, s, (const bf16_t*)x, rows, S,
                       D, Ut, H, logits);
    return hipGetLastError();
  }
  const int64_t grid = (rows + kPlRows - 1) / kPlRows;
  hipLaunchKernelGGL(pool_logits_kernel, dim3((unsigned)grid), dim3(256), (size_t)H * D * 4, s, x, in_bf16, rows,
                     S, D, U, H, logits);
  return hipGetLastError();
}

hipError_t pool_softmax_wsum(const void* x, int in_bf16, int G, int S, int D, int H, const float* logits,
                             float* stats, float* zpart, float* z, hipStream_t s) {
  if (D % 256 || D > 1024 || H < 1 || H > kPwMaxH) return hipErrorInvalidValue;
  hipLaunchKernelGGL(pool_stats_kernel, dim3(G * H), dim3(256), 0, s, logits, S, stats);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  const int C = (S + kPwRows - 1) / kPwRows;
  hipLaunchKernelGGL(pool_wsum_kernel, dim3(G * C * (D / 256)), dim3(128), 0, s, x, in_bf16, S, D, H, logits, stats,
                     C, zpart);
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  const int64_t HD = (int64_t)H * D, total = (int64_t)G * HD;
  hipLaunchKernelGGL(pool_reduce_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, zpart, C, HD, total,
                     z);
  return hipGetLastError();
}

int pool_chunks(int S) { return (S + kPwRows - 1) / kPwRows; }

hipError_t small_gemm(const float* A, int64_t lda, int64_t sA, const float* Wt, int64_t sW, const float* bias,
                      int64_t sB, float* out, int64_t ldo, int64_t sO, int M, int N, int K, int batch,
                      hipStream_t s) {
  if (M < 1 || N < 1 || K < 1 || batch < 1) return hipErrorInvalidValue;
  hipLaunchKernelGGL(small_gemm_kernel, dim3((N + kSgN - 1) / kSgN, (M + kSgM - 1) / kSgM, batch), dim3(256), 0, s, A,
                     lda, sA, Wt, sW, bias, sB, out, ldo, sO, M, N, K);
  return hipGetLastError();
}

// K split `splits` ways as a batch of small_gemm over K slices (A columns / Wt rows), partials [splits][M][N]
// in `part`, then summed in slice order: the same bits for any M, and splits x the workgroups of one
// small_gemm (the pooler's output projection, K = heads x dim_per_head = 4096 on LvT-Large, otherwise ran on
// N / 64 = 16 workgroups)
hipError_t small_gemm_splitk(const float* A, int64_t lda, const float* Wt, const float* bias, float* out, int64_t ldo,
                             int M, int N, int K, int splits, float* part, hipStream_t s) {
  if (splits < 1 || K % splits) return hipErrorInvalidValue;
  const int Kc = K / splits;
  hipError_t e = small_gemm(A, lda, Kc, Wt, (int64_t)Kc * N, nullptr, 0, part, N, (int64_t)M * N, M, N, Kc, splits, s);
  if (e != hipSuccess) return e;
  const int64_t MN = (int64_t)M * N;
  hipLaunchKernelGGL(splitk_reduce_kernel, dim3((unsigned)((MN + 255) / 256)), dim3(256), 0, s, part, splits, MN, N,
                     bias, out, ldo);
  return hipGetLastError();
}

hipError_t ln_l2_rows(const void* x, int in_bf16, int64_t stride, int rows, int D, const float* gamma,
                      const float* beta, int do_l2, float* out, hipStream_t s) {
  if (D < 1 || D > 1024 || rows < 1) return hipErrorInvalidValue;
  hipLaunchKernelGGL(ln_l2_rows_kernel, dim3(rows), dim3(256), 0, s, x, in_bf16, stride, D, gamma, beta, do_l2, out);
  return hipGetLastError();
}

hipError_t text_embed(const int32_t* ids, int Q, int L, const void* table, int table_bf16, int V, const float* cls,
                      const float* pos, float scale, int D, void* out, int out_bf16, const float* pad_in,
                      float* pad_out, hipStream_t s) {
  if (Q < 1 || L < 0 || V < 1) return hipErrorInvalidValue;
  hipLaunchKernelGGL(text_embed_kernel, dim3(Q * (L + 1)), dim3(256), 0, s, ids, L, table, table_bf16, V, cls, pos,
                     scale, D, out, out_bf16, pad_in, pad_out);
  return hipGetLastError();
}

hipError_t similarity(const float* a, const float* b, int B, int Q, int D, float* out, hipStream_t s) {
  if (B < 1 || Q < 1 || D < 1) return hipErrorInvalidValue;
  hipLaunchKernelGGL(similarity_kernel, dim3(B * Q), dim3(256), 0, s, a, b, B, Q, D, out);
  return hipGetLastError();
}

}  // namespace vp
