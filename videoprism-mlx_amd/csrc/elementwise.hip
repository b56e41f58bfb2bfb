// HBM-bound kernels of the encoder path: patchify, LayerNorm (+row permutation and
// positional add), casts and padding expansion.
#include "vp_common.h"
#include "vp_kernels.h"

namespace vp {

thread_local const void* g_last_kernel = nullptr;


namespace {

// ---- patchify (encoders.py:70-104): '(m p)(n q) c -> (m n)(p q c)', K zero-padded ----
// One thread produces 8 consecutive K elements of one patch row (a 16-byte store); the
// 8 source elements are read from the NHWC frame (a run of P*C contiguous values per p).
template <typename TI, typename TO>
__global__ __launch_bounds__(256) void patchify_kernel(const TI* __restrict__ video,
                                                       TO* __restrict__ out, int BT, int H, int W,
                                                       int C, int P, int kpad) {
  const int gm = H / P, gn = W / P, np_ = gm * gn;
  const int kreal = P * P * C;
  const int64_t groups_per_row = kpad / 8;
  const int64_t total = (int64_t)BT * np_ * groups_per_row;
  for (int64_t gid = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; gid < total;
       gid += (int64_t)gridDim.x * blockDim.x) {
    const int64_t row = gid / groups_per_row;
    const int k0 = (int)(gid % groups_per_row) * 8;
    const int bt = (int)(row / np_);
    const int pidx = (int)(row % np_);
    const int mi = pidx / gn, ni = pidx % gn;
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = k0 + j;
      float x = 0.0f;
      if (k < kreal) {
        const int p = k / (P * C);
        const int rem = k - p * P * C;  // = q*C + c, contiguous in the source row
        const int64_t off = (((int64_t)bt * H + mi * P + p) * W + ni * P) * C + rem;
        if constexpr (sizeof(TI) == 1) x = (float)video[off] / 255.0f;  // video_utils.py:94
        else if constexpr (sizeof(TI) == 2) x = bf2f(video[off]);
        else x = video[off];
      }
      v[j] = x;
    }
    if constexpr (sizeof(TO) == 2) {
      uint4 o = make_uint4(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]),
                           pack_bf16x2(v[4], v[5]), pack_bf16x2(v[6], v[7]));
      *reinterpret_cast<uint4*>(out + row * kpad + k0) = o;
    } else {
      float4* op = reinterpret_cast<float4*>(out + row * kpad + k0);
      op[0] = make_float4(v[0], v[1], v[2], v[3]);
      op[1] = make_float4(v[4], v[5], v[6], v[7]);
    }
  }
}

// Band variant: one workgroup per (frame, patch row mi).  The P image rows of the band are one
// contiguous run of P*W*C values: read it with coalesced 16-byte loads into LDS (as fp32), then
// write the band's W/P patch rows [kpad] with 16-byte stores.  (The element-gather kernel above
// reads 2-byte values at a 108-byte stride: 2 TB/s at the bench shape.)
template <typename TI>
__device__ __forceinline__ float to_f(TI v) {
  if constexpr (sizeof(TI) == 1) return (float)v / 255.0f;  // video_utils.py:94
  else if constexpr (sizeof(TI) == 2) return bf2f(v);
  else return v;
}

template <typename TI, typename TO>
__global__ __launch_bounds__(256) void patchify_band_kernel(const TI* __restrict__ video, TO* __restrict__ out,
                                                            int H, int W, int C, int P, int kpad) {
  // the band is staged in the OUTPUT dtype: exact (the value is rounded once either way) and,
  // for bf16, 31 KiB per workgroup so five workgroups share a CU
  extern __shared__ __attribute__((aligned(16))) char band_raw[];
  TO* band = reinterpret_cast<TO*>(band_raw);
  const int gm = H / P, gn = W / P;
  const int bt = blockIdx.x / gm, mi = blockIdx.x % gm;
  const int rowlen = W * C;
  const int n = P * rowlen;
  const TI* src = video + ((int64_t)bt * H + (int64_t)mi * P) * rowlen;
  auto put = [&](int i, float v) {
    if constexpr (sizeof(TO) == 2) band[i] = f2bf(v);
    else band[i] = v;
  };
  constexpr int V = 16 / sizeof(TI);  // elements per 16-byte load
  if (rowlen % V == 0) {  // every row start (and the band) 16-byte aligned
    typedef TI vec_t __attribute__((ext_vector_type(V)));
    for (int i = threadIdx.x; i < n / V; i += 256) {
      const vec_t x = *reinterpret_cast<const vec_t*>(src + (int64_t)i * V);
#pragma unroll
      for (int j = 0; j < V; ++j) put(i * V + j, to_f<TI>(x[j]));
    }
  } else {
    for (int i = threadIdx.x; i < n; i += 256) put(i, to_f<TI>(src[i]));
  }
  __syncthreads();
  const int pc = P * C, kreal = P * pc, groups = kpad / 8;
  TO* dst = out + ((int64_t)bt * gm * gn + (int64_t)mi * gn) * kpad;
  for (int gi = threadIdx.x; gi < gn * groups; gi += 256) {
    const int ni = gi / groups, k0 = (gi % groups) * 8;
    TO v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = k0 + j;
      const int p = k / pc;
      v[j] = k < kreal ? band[p * rowlen + ni * pc + (k - p * pc)] : TO(0);
    }
    if constexpr (sizeof(TO) == 2) {
      *reinterpret_cast<uint4*>(dst + (int64_t)ni * kpad + k0) = *reinterpret_cast<const uint4*>(v);
    } else {
      float4* op = reinterpret_cast<float4*>(dst + (int64_t)ni * kpad + k0);
      op[0] = make_float4(v[0], v[1], v[2], v[3]);
      op[1] = make_float4(v[4], v[5], v[6], v[7]);
    }
  }
}

// ---- LayerNorm (layers.py:208-270) over fp32 or bf16 rows ----
// One wave owns RPW rows: all RPW x NCH loads are issued before the first reduction (memory-level
// parallelism for an HBM-bound kernel), and the RPW row reductions interleave.  NCH = D / 256
// 4-element chunks per lane.  gamma = 1 + scale (folded on the host).
template <int NCH, bool OUT_BF16, bool IN_BF16, int RPW>
__global__ __launch_bounds__(256) void layernorm_kernel(const void* __restrict__ x, int rows,
                                                        const float* __restrict__ gamma,
                                                        const float* __restrict__ beta,
                                                        void* __restrict__ out, int perm, int T,
                                                        int Nsp, const float* __restrict__ add,
                                                        float* __restrict__ out_rs) {
  constexpr int D = NCH * 256;
  const int lane = threadIdx.x & 63;
  const int row0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * RPW;
  if (row0 >= rows) return;
  float4 v[RPW][NCH];
#pragma unroll
  for (int r = 0; r < RPW; ++r) {
    const int row = row0 + r < rows ? row0 + r : rows - 1;  // tail rows: recomputed, not stored
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      if constexpr (IN_BF16) {
        const uint2 u = *reinterpret_cast<const uint2*>(static_cast<const bf16_t*>(x) + (int64_t)row * D +
                                                        c * 256 + lane * 4);
        v[r][c] = make_float4(__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u),
                              __uint_as_float(u.y << 16), __uint_as_float(u.y & 0xffff0000u));
      } else {
        v[r][c] = *reinterpret_cast<const float4*>(static_cast<const float*>(x) + (int64_t)row * D + c * 256 +
                                                   lane * 4);
      }
    }
  }
  float s[RPW];
#pragma unroll
  for (int r = 0; r < RPW; ++r) {
    s[r] = 0.f;
#pragma unroll
    for (int c = 0; c < NCH; ++c) s[r] += (v[r][c].x + v[r][c].y) + (v[r][c].z + v[r][c].w);
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1)
#pragma unroll
    for (int r = 0; r < RPW; ++r) s[r] += __shfl_xor(s[r], off);
  float ss[RPW];
#pragma unroll
  for (int r = 0; r < RPW; ++r) {
    const float mean = s[r] * (1.0f / D);
    ss[r] = 0.f;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      v[r][c].x -= mean; v[r][c].y -= mean; v[r][c].z -= mean; v[r][c].w -= mean;
      ss[r] += (v[r][c].x * v[r][c].x + v[r][c].y * v[r][c].y) + (v[r][c].z * v[r][c].z + v[r][c].w * v[r][c].w);
    }
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1)
#pragma unroll
    for (int r = 0; r < RPW; ++r) ss[r] += __shfl_xor(ss[r], off);

  float4 gm[NCH], bt[NCH];
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    gm[c] = *reinterpret_cast<const float4*>(gamma + c * 256 + lane * 4);
    bt[c] = *reinterpret_cast<const float4*>(beta + c * 256 + lane * 4);
  }
#pragma unroll
  for (int r = 0; r < RPW; ++r) {
    const int row = row0 + r;
    if (row >= rows) break;
    const float rstd = 1.0f / sqrtf(ss[r] * (1.0f / D) + 1e-6f);
    int64_t orow = row;
    int t_of_out = 0;
    if (perm == PERM_BTN_TO_BNT) {  // r = (b*T + t)*Nsp + n  ->  (b*Nsp + n)*T + t
      const int n = row % Nsp;
      const int btx = row / Nsp;
      const int t = btx % T, b = btx / T;
      orow = ((int64_t)b * Nsp + n) * T + t;
      t_of_out = t;
    } else if (perm == PERM_BNT_TO_BTN) {  // r = (b*Nsp + n)*T + t  ->  (b*T + t)*Nsp + n
      const int t = row % T;
      const int bn = row / T;
      const int n = bn % Nsp, b = bn / Nsp;
      orow = ((int64_t)b * T + t) * Nsp + n;
      t_of_out = t;
    }
    float4 ys[NCH];  // the stored values (bf16-rounded when OUT_BF16), for out_rs
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int col = c * 256 + lane * 4;
      float4 y = make_float4(v[r][c].x * rstd * gm[c].x + bt[c].x, v[r][c].y * rstd * gm[c].y + bt[c].y,
                             v[r][c].z * rstd * gm[c].z + bt[c].z, v[r][c].w * rstd * gm[c].w + bt[c].w);
      if (add) {
        const float4 a = *reinterpret_cast<const float4*>(add + (int64_t)t_of_out * D + col);
        y.x += a.x; y.y += a.y; y.z += a.z; y.w += a.w;
      }
      if constexpr (OUT_BF16) {
        const uint2 pk = make_uint2(pack_bf16x2(y.x, y.y), pack_bf16x2(y.z, y.w));
        *reinterpret_cast<uint2*>(static_cast<bf16_t*>(out) + orow * D + col) = pk;
        ys[c] = make_float4(__uint_as_float(pk.x << 16), __uint_as_float(pk.x & 0xffff0000u),
                            __uint_as_float(pk.y << 16), __uint_as_float(pk.y & 0xffff0000u));
      } else {
        *reinterpret_cast<float4*>(static_cast<float*>(out) + orow * D + col) = y;
        ys[c] = y;
      }
    }
    if (out_rs) {  // statistics of the stored row for the LayerNorm folded into the next GEMM
      float a = 0.f;
#pragma unroll
      for (int c = 0; c < NCH; ++c) a += (ys[c].x + ys[c].y) + (ys[c].z + ys[c].w);
#pragma unroll
      for (int off = 32; off >= 1; off >>= 1) a += __shfl_xor(a, off);
      const float mean = a * (1.0f / D);
      float q = 0.f;
#pragma unroll
      for (int c = 0; c < NCH; ++c) {
        const float dx = ys[c].x - mean, dy = ys[c].y - mean, dz = ys[c].z - mean, dw = ys[c].w - mean;
        q += (dx * dx + dy * dy) + (dz * dz + dw * dw);
      }
#pragma unroll
      for (int off = 32; off >= 1; off >>= 1) q += __shfl_xor(q, off);
      const float rs = 1.0f / sqrtf(q * (1.0f / D) + 1e-6f);
      if (lane == 0) *reinterpret_cast<float2*>(out_rs + 2 * orow) = make_float2(rs, -mean * rs);
    }
  }
}

// ---- LayerNorm statistics for the GEMM-folded LayerNorm (EPI_*_LN) ----
// partials: st[p][row] = (sum, M2) over columns [128p, 128p+128) of the stored bf16 row
// (vp_common.h ln_combine).  PP: the partial count as a compile-time constant (D = 768: 6, 1024: 8),
// so the P loads are all in flight at once -- with a run-time count each iteration waited for its load
// (6 serial memory latencies: 5.3 us per launch); PP = 0: run-time P <= 16
template <int PP>
__global__ __launch_bounds__(256) void ln_stats_finalize_kernel(const float* __restrict__ st, int P_rt,
                                                                int64_t M, float* __restrict__ rs_out) {
  constexpr int PMAX = PP > 0 ? PP : 16;
  const int P = PP > 0 ? PP : P_rt;
  const int64_t row = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (row >= M) return;
  float2 pt[PMAX];
#pragma unroll
  for (int p = 0; p < PMAX; ++p)
    pt[p] = p < P ? *reinterpret_cast<const float2*>(st + 2 * ((int64_t)p * M + row)) : make_float2(0.f, 0.f);
  *reinterpret_cast<float2*>(rs_out + 2 * row) = ln_combine(pt, P);
}

// two-pass statistics straight from bf16 rows, one wave per row.  NCH = D / 256 > 0: the row is held in
// registers (lane: 4 values of every 256-column chunk, NCH 8-byte loads in flight), both passes from
// there; NCH = 0: any D, element by element (each load waited for: 1.25 TB/s on the LvT-Large aux input)
template <int NCH>
__global__ __launch_bounds__(256) void ln_row_stats_vec_kernel(const bf16_t* __restrict__ x, int64_t M,
                                                               float* __restrict__ rs_out) {
  constexpr int D = NCH * 256;
  const int lane = threadIdx.x & 63;
  const int64_t row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  const bf16_t* r = x + row * D + 4 * lane;
  uint2 u[NCH];
#pragma unroll
  for (int j = 0; j < NCH; ++j) u[j] = *reinterpret_cast<const uint2*>(r + 256 * j);
  float v[NCH][4];
#pragma unroll
  for (int j = 0; j < NCH; ++j) {
    v[j][0] = __uint_as_float(u[j].x << 16);
    v[j][1] = __uint_as_float(u[j].x & 0xffff0000u);
    v[j][2] = __uint_as_float(u[j].y << 16);
    v[j][3] = __uint_as_float(u[j].y & 0xffff0000u);
  }
  float a = 0.f;
#pragma unroll
  for (int j = 0; j < NCH; ++j) a += (v[j][0] + v[j][1]) + (v[j][2] + v[j][3]);
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) a += __shfl_xor(a, off);
  const float mean = a / D;
  float q = 0.f;
#pragma unroll
  for (int j = 0; j < NCH; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float d = v[j][e] - mean;
      q = fmaf(d, d, q);
    }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) q += __shfl_xor(q, off);
  const float rs = 1.0f / sqrtf(q / D + 1e-6f);
  if (lane == 0) *reinterpret_cast<float2*>(rs_out + 2 * row) = make_float2(rs, -mean * rs);
}

__global__ __launch_bounds__(256) void ln_row_stats_kernel(const bf16_t* __restrict__ x, int64_t M, int D,
                                                           float* __restrict__ rs_out) {
  const int lane = threadIdx.x & 63;
  const int64_t row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  const bf16_t* r = x + row * D;
  float a = 0.f;
  for (int c = lane; c < D; c += 64) a += bf2f(r[c]);
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) a += __shfl_xor(a, off);
  const float mean = a / D;
  float q = 0.f;
  for (int c = lane; c < D; c += 64) {
    const float d = bf2f(r[c]) - mean;
    q += d * d;
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) q += __shfl_xor(q, off);
  const float rs = 1.0f / sqrtf(q / D + 1e-6f);
  if (lane == 0) *reinterpret_cast<float2*>(rs_out + 2 * row) = make_float2(rs, -mean * rs);
}

__global__ __launch_bounds__(256) void cast_f32_bf16_kernel(const float* __restrict__ x,
                                                            bf16_t* __restrict__ y, int64_t n4) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4;
       i += (int64_t)gridDim.x * blockDim.x) {
    const float4 v = reinterpret_cast<const float4*>(x)[i];
    reinterpret_cast<uint2*>(y)[i] = make_uint2(pack_bf16x2(v.x, v.y), pack_bf16x2(v.z, v.w));
  }
}

// f32 / uint8 frames -> bf16 frames in place of layout (the fused patch embedding reads bf16
// frames): the same conversion the patchify kernels apply per value (to_f, then one RNE rounding),
// so a forward over converted frames sees bitwise the values a bf16 caller would pass
template <typename TI>
__global__ __launch_bounds__(256) void video_bf16_kernel(const TI* __restrict__ x, bf16_t* __restrict__ y,
                                                         int64_t n) {
  const int64_t n4 = n >> 2;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
    float v[4];
    if constexpr (sizeof(TI) == 1) {
      const uchar4 u = reinterpret_cast<const uchar4*>(x)[i];
      v[0] = to_f<TI>(u.x); v[1] = to_f<TI>(u.y); v[2] = to_f<TI>(u.z); v[3] = to_f<TI>(u.w);
    } else {
      const float4 f = reinterpret_cast<const float4*>(x)[i];
      v[0] = f.x; v[1] = f.y; v[2] = f.z; v[3] = f.w;
    }
    reinterpret_cast<uint2*>(y)[i] = make_uint2((uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16),
                                                (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16));
  }
  for (int64_t i = (n4 << 2) + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    y[i] = f2bf(to_f<TI>(x[i]));
}

__global__ __launch_bounds__(256) void expand_paddings_kernel(const float* __restrict__ fp, int B,
                                                              int T, int Nsp,
                                                              float* __restrict__ pad_btn,
                                                              float* __restrict__ pad_bnt) {
  const int64_t total = (int64_t)B * T * Nsp;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    // i in (b, t, n) order
    const int n = (int)(i % Nsp);
    const int64_t bt = i / Nsp;
    const int t = (int)(bt % T), b = (int)(bt / T);
    const float v = fp[bt];
    pad_btn[i] = v;
    pad_bnt[((int64_t)b * Nsp + n) * T + t] = v;
  }
}


// ---- pooled clip embedding: out[b] = l2norm(mean_l emb[b, l, :]) (encoders.py:50-67) ----
template <typename T>
__global__ __launch_bounds__(256) void pool_l2_kernel(const T* __restrict__ emb, int L, int D,
                                                      float* __restrict__ out) {
  __shared__ float red[256 / 64];
  const int b = blockIdx.x;
  const T* e = emb + (int64_t)b * L * D;
  float sq = 0.f;
  for (int col = threadIdx.x; col < D; col += blockDim.x) {
    float s = 0.f;
    for (int l = 0; l < L; ++l) {
      if constexpr (sizeof(T) == 2) s += bf2f(e[(int64_t)l * D + col]); else s += e[(int64_t)l * D + col];
    }
    s *= 1.0f / L;
    out[(int64_t)b * D + col] = s;
    sq += s * s;
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) sq += __shfl_xor(sq, off);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = sq;
  __syncthreads();
  const float tot = red[0] + red[1] + red[2] + red[3];
  const float inv = 1.0f / sqrtf(tot + 1e-12f);
  for (int col = threadIdx.x; col < D; col += blockDim.x) out[(int64_t)b * D + col] *= inv;
}

int grid_for(int64_t work, int block) {
  int64_t g = (work + block - 1) / block;
  if (g > 8192) g = 8192;
  if (g < 1) g = 1;
  return (int)g;
}

template <int NCH>
hipError_t ln_launch(const void* x, int in_is_bf16, int rows, const float* gamma, const float* beta,
                     void* out, int out_is_bf16, int perm, int T, int Nsp, const float* add, hipStream_t s,
                     float* out_rs) {
  constexpr int RPW = NCH <= 4 ? 4 : 2;  // rows per wave
  const dim3 grid((rows + 4 * RPW - 1) / (4 * RPW));
  if (in_is_bf16) {
    if (out_is_bf16)
      hipLaunchKernelGGL((layernorm_kernel<NCH, true, true, RPW>), grid, dim3(256), 0, s, x, rows, gamma, beta,
                         out, perm, T, Nsp, add, out_rs);
    else
      hipLaunchKernelGGL((layernorm_kernel<NCH, false, true, RPW>), grid, dim3(256), 0, s, x, rows, gamma, beta,
                         out, perm, T, Nsp, add, out_rs);
  } else {
    if (out_is_bf16)
      hipLaunchKernelGGL((layernorm_kernel<NCH, true, false, RPW>), grid, dim3(256), 0, s, x, rows, gamma, beta,
                         out, perm, T, Nsp, add, out_rs);
    else
      hipLaunchKernelGGL((layernorm_kernel<NCH, false, false, RPW>), grid, dim3(256), 0, s, x, rows, gamma, beta,
                         out, perm, T, Nsp, add, out_rs);
  }
  return hipGetLastError();
}

}  // namespace

hipError_t patchify(const void* video, int in_dtype, void* patches, int out_is_bf16, int BT, int H,
                    int W, int C, int P, int kpad, hipStream_t s) {
  if (kpad % 8 || kpad < P * P * C || H % P || W % P || in_dtype < 0 || in_dtype > 2) return hipErrorInvalidValue;
  const int64_t work = (int64_t)BT * (H / P) * (W / P) * (kpad / 8);
  const int grid = grid_for(work, 256);
  const size_t band_bytes = (size_t)P * W * C * (out_is_bf16 ? 2 : 4);
  const bool aligned = ((uintptr_t)video & 15) == 0;
  auto go = [&](auto in_tag) {
    using TI = decltype(in_tag);
    if (band_bytes <= 65536 && aligned) {  // one workgroup per (frame, patch row)
      const dim3 g((unsigned)(BT * (H / P)));
      if (out_is_bf16)
        hipLaunchKernelGGL((patchify_band_kernel<TI, bf16_t>), g, dim3(256), band_bytes, s, (const TI*)video,
                           (bf16_t*)patches, H, W, C, P, kpad);
      else
        hipLaunchKernelGGL((patchify_band_kernel<TI, float>), g, dim3(256), band_bytes, s, (const TI*)video,
                           (float*)patches, H, W, C, P, kpad);
      return;
    }
    if (out_is_bf16)
      hipLaunchKernelGGL((patchify_kernel<TI, bf16_t>), dim3(grid), dim3(256), 0, s, (const TI*)video,
                         (bf16_t*)patches, BT, H, W, C, P, kpad);
    else
      hipLaunchKernelGGL((patchify_kernel<TI, float>), dim3(grid), dim3(256), 0, s, (const TI*)video,
                         (float*)patches, BT, H, W, C, P, kpad);
  };
  if (in_dtype == 1) go(bf16_t{});
  else if (in_dtype == 2) go(uint8_t{});
  else go(float{});
  return hipGetLastError();
}

hipError_t layernorm(const void* x, int in_is_bf16, int rows, int D, const float* gamma,
                     const float* beta, void* out, int out_is_bf16, int perm, int T, int Nsp,
                     const float* add, hipStream_t s, float* out_rs) {
  switch (D) {
    case 256: return ln_launch<1>(x, in_is_bf16, rows, gamma, beta, out, out_is_bf16, perm, T, Nsp, add, s, out_rs);
    case 512: return ln_launch<2>(x, in_is_bf16, rows, gamma, beta, out, out_is_bf16, perm, T, Nsp, add, s, out_rs);
    case 768: return ln_launch<3>(x, in_is_bf16, rows, gamma, beta, out, out_is_bf16, perm, T, Nsp, add, s, out_rs);
    case 1024: return ln_launch<4>(x, in_is_bf16, rows, gamma, beta, out, out_is_bf16, perm, T, Nsp, add, s, out_rs);
    case 1280: return ln_launch<5>(x, in_is_bf16, rows, gamma, beta, out, out_is_bf16, perm, T, Nsp, add, s, out_rs);
    case 1536: return ln_launch<6>(x, in_is_bf16, rows, gamma, beta, out, out_is_bf16, perm, T, Nsp, add, s, out_rs);
    case 2048: return ln_launch<8>(x, in_is_bf16, rows, gamma, beta, out, out_is_bf16, perm, T, Nsp, add, s, out_rs);
  }
  return hipErrorInvalidValue;
}

hipError_t ln_stats_finalize(const float* st_part, int P, int64_t M, float* ln_rs, hipStream_t s) {
  if (P < 1 || P > 16) return hipErrorInvalidValue;
  const dim3 g((unsigned)((M + 255) / 256));
  if (P == 6) hipLaunchKernelGGL(ln_stats_finalize_kernel<6>, g, dim3(256), 0, s, st_part, P, M, ln_rs);
  else if (P == 8) hipLaunchKernelGGL(ln_stats_finalize_kernel<8>, g, dim3(256), 0, s, st_part, P, M, ln_rs);
  else hipLaunchKernelGGL(ln_stats_finalize_kernel<0>, g, dim3(256), 0, s, st_part, P, M, ln_rs);
  return hipGetLastError();
}

hipError_t ln_row_stats(const bf16_t* x, int64_t M, int D, float* ln_rs, hipStream_t s) {
  const dim3 g((unsigned)((M + 3) / 4));
  switch (D) {
    case 768: hipLaunchKernelGGL(ln_row_stats_vec_kernel<3>, g, dim3(256), 0, s, x, M, ln_rs); break;
    case 1024: hipLaunchKernelGGL(ln_row_stats_vec_kernel<4>, g, dim3(256), 0, s, x, M, ln_rs); break;
    case 1536: hipLaunchKernelGGL(ln_row_stats_vec_kernel<6>, g, dim3(256), 0, s, x, M, ln_rs); break;
    case 2048: hipLaunchKernelGGL(ln_row_stats_vec_kernel<8>, g, dim3(256), 0, s, x, M, ln_rs); break;
    default: hipLaunchKernelGGL(ln_row_stats_kernel, g, dim3(256), 0, s, x, M, D, ln_rs);
  }
  return hipGetLastError();
}

hipError_t video_to_bf16(const void* video, int in_dtype, bf16_t* out, int64_t n, hipStream_t s) {
  const dim3 g(grid_for((n + 3) / 4, 256));
  if (in_dtype == 2) {
    VP_NOTE_KERNEL(video_bf16_kernel<uint8_t>);
    hipLaunchKernelGGL(video_bf16_kernel<uint8_t>, g, dim3(256), 0, s, (const uint8_t*)video, out, n);
  } else if (in_dtype == 0) {
    VP_NOTE_KERNEL(video_bf16_kernel<float>);
    hipLaunchKernelGGL(video_bf16_kernel<float>, g, dim3(256), 0, s, (const float*)video, out, n);
  } else {
    return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t cast_f32_bf16(const float* x, bf16_t* y, int64_t n, hipStream_t s) {
  if (n % 4) return hipErrorInvalidValue;
  hipLaunchKernelGGL(cast_f32_bf16_kernel, dim3(grid_for(n / 4, 256)), dim3(256), 0, s, x, y, n / 4);
  return hipGetLastError();
}

hipError_t expand_paddings(const float* frame_pad, int B, int T, int Nsp, float* pad_btn,
                           float* pad_bnt, hipStream_t s) {
  hipLaunchKernelGGL(expand_paddings_kernel, dim3(grid_for((int64_t)B * T * Nsp, 256)), dim3(256),
                     0, s, frame_pad, B, T, Nsp, pad_btn, pad_bnt);
  return hipGetLastError();
}

hipError_t pool_l2(const void* emb, int is_bf16, int B, int L, int D, float* out, hipStream_t s) {
  if (is_bf16)
    hipLaunchKernelGGL(pool_l2_kernel<bf16_t>, dim3(B), dim3(256), 0, s, (const bf16_t*)emb, L, D, out);
  else
    hipLaunchKernelGGL(pool_l2_kernel<float>, dim3(B), dim3(256), 0, s, (const float*)emb, L, D, out);
  return hipGetLastError();
}

}  // namespace vp
