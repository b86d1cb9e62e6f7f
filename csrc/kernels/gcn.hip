// Fused GeneralConv + BatchNorm + PReLU + node pooling (SURVEY §2.2 K1 + K2).
//
// The reference runs spektral GeneralConv (x@W+b -> BatchNorm -> PReLU -> mean
// over in-edges) on a block-diagonal graph with one edge-list copy per (sample,
// time step), then `timeseries_pooling` (dynamic_partition into batch_size
// partitions, mean over nodes) and a Concatenate with the flagged series
// (libs/create_model.py:8-41,215-223).
//
// For linear node pooling (mean / sum / selection) the aggregation and the pool
// collapse algebraically: pooled[b,t,:] = sum_j w[b,j] * act(x[b,t,j,:]) with
// per-sample node weights w = p^T (D^-1 A) (computed once per batch from the
// [N,N] adjacency, shared by all T steps). So the whole block is one streaming
// pass over x that writes the LSTM input [B,T,Ca+F] directly (flagged series
// first, like Concatenate([anom, pooled])).
//
// Training-mode BatchNorm needs batch statistics of z = xW+b over all valid node
// rows; since z is affine in the Cin-dim input they follow from the first and
// second moments of x (gcn_stats: Cin + Cin^2 + 1 sums, fp64 accumulation).
// Backward needs one more streaming pass (gcn_pool_bwd) whose per-block partial
// sums give dW, dgamma, dbeta, dalpha in closed form; gcn_pool_bwd_input gives
// d/dx for attribution (integrated gradients).
#include "common.h"

namespace gq {

constexpr int GCN_MAX_CIN = 8;

// ------------------------------------------------------------------ stats
// out[0:Cin] = sum m x_k ; out[Cin : Cin+Cin^2] = sum m x_k x_l ; out[last] = sum m
template <int Cin>
__global__ void gcn_stats_kernel(const float* __restrict__ x, const float* __restrict__ mask, double* out,
                                 int B, int T, int N) {
  constexpr int nstat = Cin + Cin * Cin + 1;
  double acc[nstat];
  _Pragma("unroll") for (int i = 0; i < nstat; ++i) acc[i] = 0.0;
  const long rows = (long)B * T * N;
  for (long r = blockIdx.x * (long)blockDim.x + threadIdx.x; r < rows; r += (long)gridDim.x * blockDim.x) {
    const int n = r % N;
    const int b = r / ((long)T * N);
    const float m = mask[b * N + n];
    if (m == 0.f) continue;
    float xv[Cin];
    _Pragma("unroll") for (int k = 0; k < Cin; ++k) xv[k] = x[r * Cin + k];
    _Pragma("unroll") for (int k = 0; k < Cin; ++k) {
      acc[k] += m * xv[k];
      _Pragma("unroll") for (int l = 0; l < Cin; ++l) acc[Cin + k * Cin + l] += (double)(m * xv[k]) * xv[l];
    }
    acc[nstat - 1] += m;
  }
  // wave reduction by shuffles, then one LDS slot per wave, one atomic per block
  __shared__ double red[4][nstat];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  _Pragma("unroll") for (int i = 0; i < nstat; ++i) {
    double v = acc[i];
    _Pragma("unroll") for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if (lane == 0) red[wv][i] = v;
  }
  __syncthreads();
  if (threadIdx.x < nstat) {
    double v = 0.0;
    for (int k = 0; k < (int)(blockDim.x >> 6); ++k) v += red[k][threadIdx.x];
    atomicAdd(&out[threadIdx.x], v);
  }
}

// ------------------------------------------------------------------ forward
// thread = one (b,t) row, all F channels in registers. A workgroup's 256 rows are ONE
// contiguous span of x ([B,T,N,Cin] with (b,t) consecutive), staged through LDS with
// coalesced float4 loads when it fits (N*Cin <= GCN_STAGE_MAX); each thread then walks its
// row's N nodes once (the old channel-per-thread layout re-read every row F times).
// Channel parameters live in LDS (wave-uniform broadcast reads).
constexpr int GCN_STAGE_MAX = 48;           // floats per row staged in LDS (48 KiB / 256 rows)

template <int Cin, int F>
__device__ __forceinline__ void gcn_load_params(const float* W, const float* bias, const float* scale,
                                                const float* shift, const float* alpha, float* sp) {
  // sp: [Cin+4][F] = W rows, bias, scale, shift, alpha
  for (int i = threadIdx.x; i < (Cin + 4) * F; i += blockDim.x) {
    const int r = i / F, f = i % F;
    float v;
    if (r < Cin) v = W[r * F + f];
    else if (r == Cin) v = bias[f];
    else if (r == Cin + 1) v = scale[f];
    else if (r == Cin + 2) v = shift[f];
    else v = alpha[f];
    sp[i] = v;
  }
}

// stage rows [row0, row0 + nrow) of a [rows, L] fp32 array into LDS (zero past `rows`)
__device__ __forceinline__ void gcn_stage_rows(const float* __restrict__ src, float* dst, long row0, int nrow,
                                               long rows, int L) {
  const long beg = row0 * L;
  const long end = min(rows, row0 + nrow) * (long)L;
  const int n = nrow * L;
  if ((beg & 3) == 0 && (L & 3) == 0) {
    for (int i = threadIdx.x * 4; i < n; i += blockDim.x * 4) {
      float4 v = beg + i < end ? *reinterpret_cast<const float4*>(src + beg + i) : make_float4(0.f, 0.f, 0.f, 0.f);
      *reinterpret_cast<float4*>(dst + i) = v;
    }
  } else {
    for (int i = threadIdx.x; i < n; i += blockDim.x) dst[i] = beg + i < end ? src[beg + i] : 0.f;
  }
}

// 4 threads per row (adjacent lanes), each owning F/4 channels whose parameters sit in VGPRs.
template <int Cin, int F>
__global__ __launch_bounds__(256) void gcn_pool_fwd_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                           const float* __restrict__ anom, const float* __restrict__ W,
                                                           const float* __restrict__ bias, const float* __restrict__ scale,
                                                           const float* __restrict__ shift, const float* __restrict__ alpha,
                                                           float* __restrict__ out, int B, int T, int N, int Ca,
                                                           int Mp, int Cp) {
  // Mp > 0: write the time-major LSTM input [T][Mp][Cp] directly (rows b >= B and channels
  // >= Ca + F zero), else [B][T][Ca + F]
  constexpr int FQ = F / 4, RPB = 64;             // channels per thread, rows per workgroup
  extern __shared__ __attribute__((aligned(16))) float sx[];   // RPB * N * Cin (if staged)
  const int L = N * Cin;
  const bool staged = L <= GCN_STAGE_MAX;
  const int Fo = Ca + F;
  const long rows = (long)B * T;
  const int r = threadIdx.x >> 2, q = threadIdx.x & 3, f0 = q * FQ;
  float pw[Cin][FQ], pb[FQ], psc[FQ], psh[FQ], pal[FQ];
#pragma unroll
  for (int j = 0; j < FQ; ++j) {
#pragma unroll
    for (int k = 0; k < Cin; ++k) pw[k][j] = W[k * F + f0 + j];
    pb[j] = bias[f0 + j];
    psc[j] = scale[f0 + j];
    psh[j] = shift[f0 + j];
    pal[j] = alpha[f0 + j];
  }
  const long vrows = Mp > 0 ? (long)Mp * T : rows;        // virtual rows incl. zero padding rows
  float* sw = sx + RPB * L;                         // staged: the node weights of the block's samples
  for (long row0 = (long)blockIdx.x * RPB; row0 < vrows; row0 += (long)gridDim.x * RPB) {
    const int b0 = (int)(row0 / T);
    if (staged) {
      __syncthreads();
      if (row0 < rows) {
        gcn_stage_rows(x, sx, row0, RPB, rows, L);
        // samples b0 .. of rows row0 .. row0 + RPB - 1 (<= RPB / T + 2 of them): the per-node
        // weight loads then leave the node loop (they were its serial memory round trips)
        const int nb = min((int)((min(row0 + RPB, rows) - 1) / T) - b0 + 1, RPB / T + 2);
        for (int i = threadIdx.x; i < nb * N; i += blockDim.x) sw[i] = w[(long)b0 * N + i];
      }
      __syncthreads();
    }
    const long row = row0 + r;
    if (row >= vrows) continue;
    const int b = (int)(row / T), t = (int)(row % T);
    float* o = Mp > 0 ? out + ((long)t * Mp + b) * Cp : out + row * Fo;
    if (row >= rows) {                            // (time-major only) padding row
      for (int c = q; c < Cp; c += 4) o[c] = 0.f;
      continue;
    }
    const float* xr = staged ? sx + r * L : x + row * (long)L;
    const float* wr = staged ? sw + (long)(b - b0) * N : w + (long)b * N;
    float acc[FQ];
#pragma unroll
    for (int j = 0; j < FQ; ++j) acc[j] = 0.f;
    for (int n = 0; n < N; ++n) {
      const float wn = wr[n];
      float xv[Cin];
#pragma unroll
      for (int k = 0; k < Cin; ++k) xv[k] = xr[n * Cin + k];
#pragma unroll
      for (int j = 0; j < FQ; ++j) {
        float z = pb[j];
#pragma unroll
        for (int k = 0; k < Cin; ++k) z += xv[k] * pw[k][j];
        const float y = z * psc[j] + psh[j];
        acc[j] += wn * (y > 0.f ? y : pal[j] * y);
      }
    }
    for (int c = q; c < Ca; c += 4) o[c] = anom[row * Ca + c];
#pragma unroll
    for (int j = 0; j < FQ; ++j) o[Ca + f0 + j] = acc[j];
    if (Mp > 0)
      for (int c = Fo + q; c < Cp; c += 4) o[c] = 0.f;
  }
}

// ------------------------------------------------------------------ backward (params)
// partial[blk][j*F + f] with j: 0 = sum dy, 1 = sum dy*z, 2 = sum da*y[y<=0], 3.. = sum x_k dy
template <int Cin>
__global__ void gcn_pool_bwd_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                    const float* __restrict__ dout, const float* __restrict__ W,
                                    const float* __restrict__ bias, const float* __restrict__ scale,
                                    const float* __restrict__ shift, const float* __restrict__ alpha,
                                    float* __restrict__ partial, int B, int T, int N, int F, int c_off,
                                    int dstride, int dmp) {
  // dmp > 0: dout is time-major [T][dmp][dstride] (row (b,t) at (t*dmp + b)*dstride)
  // block = 256 threads = (256/F) rows x F channels (F divides 256)
  const int f = threadIdx.x % F;
  const int rsub = threadIdx.x / F;
  const int rows_per_blk = blockDim.x / F;
  constexpr int nacc = 3 + Cin;
  float acc[nacc];
  _Pragma("unroll") for (int j = 0; j < nacc; ++j) acc[j] = 0.f;
  float wk[Cin];
  _Pragma("unroll") for (int k = 0; k < Cin; ++k) wk[k] = W[k * F + f];
  const float bb = bias[f], sc = scale[f], sh = shift[f], al = alpha[f];
  const long nrows = (long)B * T;
  // staged (N * Cin <= GCN_STAGE_MAX): the pass's x rows and its samples' node weights are
  // copied to LDS with coalesced loads first, so the node loop makes no memory round trips
  // (its per-node global loads, behind a data-dependent branch, were ~all of the kernel's time)
  extern __shared__ __attribute__((aligned(16))) float sbx[];
  const int L = N * Cin;
  const bool staged = L <= GCN_STAGE_MAX;
  float* sbw = sbx + rows_per_blk * L;
  // staged: a pass's x rows, node weights of its samples and upstream gradients are fetched
  // into registers one pass AHEAD (coalesced scalar loads), then parked in LDS, so the node loop
  // makes no memory round trips and each pass's loads overlap the previous pass's compute
  constexpr int XG = (32 * GCN_STAGE_MAX + 255) / 256, WG = (34 * GCN_STAGE_MAX + 255) / 256;   // F >= 8: <= 32 rows
  float px[XG], pw[WG], pg = 0.f;
  const long stride = (long)gridDim.x * rows_per_blk;
  auto fetch = [&](long r0) {
    const long xbeg = r0 * L, xend = min(nrows, r0 + rows_per_blk) * (long)L;
    const int b0 = (int)(r0 / T);
    const int nb = r0 < nrows ? min((int)((min(r0 + rows_per_blk, nrows) - 1) / T) - b0 + 1, rows_per_blk / T + 2) : 0;
#pragma unroll
    for (int j = 0; j < XG; ++j) {
      const long i = xbeg + threadIdx.x + 256 * j;
      px[j] = i < xend ? x[i] : 0.f;
    }
#pragma unroll
    for (int j = 0; j < WG; ++j) {
      const int i = threadIdx.x + 256 * j;
      pw[j] = i < nb * N ? w[(long)b0 * N + i] : 0.f;
    }
    const long row = r0 + rsub;
    if (row < nrows) {
      const long dro = dmp > 0 ? ((row % T) * dmp + row / T) * (long)dstride : row * (long)dstride;
      pg = dout[dro + c_off + f];
    }
  };
  if (staged) fetch((long)blockIdx.x * rows_per_blk);
  for (long r0 = (long)blockIdx.x * rows_per_blk; r0 < nrows; r0 += stride) {
    const long row = r0 + rsub;
    const int b0 = (int)(r0 / T);
    float g = 0.f;
    if (staged) {
      __syncthreads();
#pragma unroll
      for (int j = 0; j < XG; ++j)
        if (threadIdx.x + 256 * j < rows_per_blk * L) sbx[threadIdx.x + 256 * j] = px[j];
#pragma unroll
      for (int j = 0; j < WG; ++j)
        if (threadIdx.x + 256 * j < (rows_per_blk / T + 2) * N) sbw[threadIdx.x + 256 * j] = pw[j];
      __syncthreads();
      g = pg;
      if (r0 + stride < nrows) fetch(r0 + stride);
    }
    if (row >= nrows) continue;
    const int b = row / T;
    if (!staged) {
      const long dro = dmp > 0 ? ((row % T) * dmp + row / T) * (long)dstride : row * (long)dstride;
      g = dout[dro + c_off + f];
    }
    const float* xr = staged ? sbx + rsub * L : x + row * (long)L;
    const float* wr = staged ? sbw + (long)(b - b0) * N : w + (long)b * N;
    for (int n = 0; n < N; ++n) {
      const float wn = wr[n];                     // wn == 0 (masked / unpooled node): da = 0
      float xv[Cin];
      _Pragma("unroll") for (int k = 0; k < Cin; ++k) xv[k] = xr[n * Cin + k];
      float z = bb;
      _Pragma("unroll") for (int k = 0; k < Cin; ++k) z += xv[k] * wk[k];
      const float y = z * sc + sh;
      const float da = wn * g;
      const float dy = y > 0.f ? da : al * da;
      acc[0] += dy;
      acc[1] += dy * z;
      acc[2] += y > 0.f ? 0.f : da * y;
      _Pragma("unroll") for (int k = 0; k < Cin; ++k) acc[3 + k] += xv[k] * dy;
    }
  }
  // reduce over the rows of the block (threads with equal f): shuffles inside the
  // wave (lanes f, f+F, ...), then the 4 wave partials through LDS
  __shared__ float red[4][nacc][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  _Pragma("unroll") for (int j = 0; j < nacc; ++j) {
    float v = acc[j];
    for (int o = 32; o >= F; o >>= 1) v += __shfl_xor(v, o, 64);
    red[wv][j][lane] = v;
  }
  __syncthreads();
  for (int e = threadIdx.x; e < nacc * F; e += blockDim.x) {
    const int j = e / F, ff = e % F;
    float v = 0.f;
    for (int k = 0; k < (int)(blockDim.x >> 6); ++k) v += red[k][j][ff];
    partial[(long)blockIdx.x * nacc * F + j * F + ff] = v;
  }
}

// ------------------------------------------------------------------ backward (input)
// thread = one (b,t) row: its F upstream gradients are read once, then per node n
// dz_f = c1_f*dy_f + c0_f + c2_f*z_f (valid nodes), dx_k = sum_f W[k,f] dz_f.
// 4 adjacent lanes per row, F/4 channels each; dx_k reduced over the 4 lanes by shuffles.
template <int Cin, int F>
__global__ __launch_bounds__(256) void gcn_pool_bwd_input_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                                 const float* __restrict__ mask, const float* __restrict__ dout,
                                                                 const float* __restrict__ W, const float* __restrict__ bias,
                                                                 const float* __restrict__ scale, const float* __restrict__ shift,
                                                                 const float* __restrict__ alpha, const float* __restrict__ coef,
                                                                 float* __restrict__ dx, int B, int T, int N, int c_off,
                                                                 int dstride, int dmp) {
  constexpr int FQ = F / 4;
  const int q = threadIdx.x & 3, f0 = q * FQ;
  float pw[Cin][FQ], pb[FQ], psc[FQ], psh[FQ], pal[FQ], c0[FQ], c1[FQ], c2[FQ];
#pragma unroll
  for (int j = 0; j < FQ; ++j) {
#pragma unroll
    for (int k = 0; k < Cin; ++k) pw[k][j] = W[k * F + f0 + j];
    pb[j] = bias[f0 + j];
    psc[j] = scale[f0 + j];
    psh[j] = shift[f0 + j];
    pal[j] = alpha[f0 + j];
    c0[j] = coef[f0 + j];
    c1[j] = coef[F + f0 + j];
    c2[j] = coef[2 * F + f0 + j];
  }
  const long rows = (long)B * T;
  const long nthr = (long)gridDim.x * blockDim.x / 4;
  for (long row = (blockIdx.x * (long)blockDim.x + threadIdx.x) / 4; row < rows + 0; row += nthr) {
    // (all 4 lanes of a row take the same trip count: the shuffles below stay converged)
    const int b = (int)(row / T);
    const long dro = dmp > 0 ? ((row % T) * dmp + b) * (long)dstride : row * (long)dstride;
    float g[FQ];
#pragma unroll
    for (int j = 0; j < FQ; ++j) g[j] = dout[dro + c_off + f0 + j];
    const float* xr = x + row * (long)N * Cin;
    float* dxr = dx + row * (long)N * Cin;
    for (int n = 0; n < N; ++n) {
      float xv[Cin], dxv[Cin];
#pragma unroll
      for (int k = 0; k < Cin; ++k) {
        xv[k] = xr[n * Cin + k];
        dxv[k] = 0.f;
      }
      const float m = mask[b * N + n] != 0.f ? 1.f : 0.f;
      const float wn = w[b * N + n];
#pragma unroll
      for (int j = 0; j < FQ; ++j) {
        float z = pb[j];
#pragma unroll
        for (int k = 0; k < Cin; ++k) z += xv[k] * pw[k][j];
        const float y = z * psc[j] + psh[j];
        const float da = wn * g[j];
        const float dy = y > 0.f ? da : pal[j] * da;
        const float dz = m * (c1[j] * dy + c0[j] + c2[j] * z);
#pragma unroll
        for (int k = 0; k < Cin; ++k) dxv[k] += pw[k][j] * dz;
      }
#pragma unroll
      for (int k = 0; k < Cin; ++k) {
        float v = dxv[k];
        v += __shfl_xor(v, 1, 64);
        v += __shfl_xor(v, 2, 64);
        if (q == (k & 3)) dxr[n * Cin + k] = v;
      }
    }
  }
}

// Deterministic column sums of a [R, C] fp32 matrix (per-workgroup partials, R large, C
// small): workgroup = 8 columns x 32 row lanes, fixed-order LDS combine. (A torch sum over
// dim 0 of a [1448, 80] partial matrix took ~20 us on the backward critical path.)
__global__ __launch_bounds__(256) void colsum_kernel(const float* __restrict__ in, long R, int C,
                                                     float* __restrict__ out) {
  __shared__ float red[32][9];
  const int c8 = threadIdx.x & 7, l = threadIdx.x >> 3;
  const int c = min(blockIdx.x * 8 + c8, C - 1);
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  long r = l;
  for (; r + 96 < R; r += 128) {
    a0 += in[r * C + c];
    a1 += in[(r + 32) * C + c];
    a2 += in[(r + 64) * C + c];
    a3 += in[(r + 96) * C + c];
  }
  for (; r < R; r += 32) a0 += in[r * C + c];
  red[l][c8] = (a0 + a1) + (a2 + a3);
  __syncthreads();
  if (threadIdx.x < 8 && blockIdx.x * 8 + c8 < C) {
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 32; ++k) s += red[k][c8];
    out[c] = s;
  }
}

// sum over the leading dim of a contiguous [R, ...] fp32 tensor
at::Tensor colsum(const at::Tensor& partial) {
  check_f32_cuda(partial, "partial");
  const long R = partial.size(0);
  const int C = (int)(partial.numel() / std::max<long>(R, 1));
  std::vector<int64_t> shape(partial.sizes().begin() + 1, partial.sizes().end());
  at::Tensor out = at::empty(shape, partial.options());
  if (R == 0) return out.zero_();
  hipLaunchKernelGGL(colsum_kernel, dim3((C + 7) / 8), dim3(256), 0, stream(), partial.data_ptr<float>(), R, C,
                     out.data_ptr<float>());
  GQ_LAUNCH_CHECK();
  return out;
}

#define GQ_CIN_DISPATCH(CIN_RT, ...)                        \
  switch (CIN_RT) {                                         \
    case 1: { constexpr int CIN = 1; __VA_ARGS__; } break;  \
    case 2: { constexpr int CIN = 2; __VA_ARGS__; } break;  \
    case 3: { constexpr int CIN = 3; __VA_ARGS__; } break;  \
    case 4: { constexpr int CIN = 4; __VA_ARGS__; } break;  \
    case 5: { constexpr int CIN = 5; __VA_ARGS__; } break;  \
    case 6: { constexpr int CIN = 6; __VA_ARGS__; } break;  \
    case 7: { constexpr int CIN = 7; __VA_ARGS__; } break;  \
    case 8: { constexpr int CIN = 8; __VA_ARGS__; } break;  \
    default: TORCH_CHECK(false, "gcn: 1..8 input channels"); \
  }

static int grid_for(long work, int block, int cap = 2048) {
  long g = (work + block - 1) / block;
  return (int)std::max<long>(1, std::min<long>(g, cap));
}

at::Tensor gcn_stats(const at::Tensor& x, const at::Tensor& mask) {
  check_f32_cuda(x, "x");
  check_f32_cuda(mask, "mask");
  TORCH_CHECK(x.dim() == 4, "x must be [B,T,N,Cin]");
  const int B = x.size(0), T = x.size(1), N = x.size(2), Cin = x.size(3);
  TORCH_CHECK(Cin <= GCN_MAX_CIN, "gcn: at most 8 input channels");
  TORCH_CHECK(mask.size(0) == B && mask.size(1) == N, "mask must be [B,N]");
  c10::DeviceGuard guard(x.device());
  at::Tensor out = at::zeros({Cin + Cin * Cin + 1}, x.options().dtype(at::kDouble));
  const long rows = (long)B * T * N;
  GQ_CIN_DISPATCH(Cin, hipLaunchKernelGGL(gcn_stats_kernel<CIN>, dim3(deterministic_mode() ? 1 : grid_for(rows, 256, 512)), dim3(256), 0,
                                          stream(), x.data_ptr<float>(), mask.data_ptr<float>(),
                                          out.data_ptr<double>(), B, T, N));
  GQ_LAUNCH_CHECK();
  return out;
}

#define GQ_GCN_F_DISPATCH(F_RT, ...)                                   \
  switch (F_RT) {                                                      \
    case 8: { constexpr int FF = 8; __VA_ARGS__; } break;              \
    case 16: { constexpr int FF = 16; __VA_ARGS__; } break;            \
    case 32: { constexpr int FF = 32; __VA_ARGS__; } break;            \
    default: TORCH_CHECK(false, "gcn: 8, 16 or 32 output channels");  \
  }

at::Tensor gcn_pool_fwd(const at::Tensor& x, const at::Tensor& w, const at::Tensor& anom, const at::Tensor& W,
                        const at::Tensor& b, const at::Tensor& scale, const at::Tensor& shift,
                        const at::Tensor& alpha, int64_t Mp, int64_t Cp) {
  for (auto* p : {&x, &w, &W, &b, &scale, &shift, &alpha}) check_f32_cuda(*p, "gcn input");
  const int B = x.size(0), T = x.size(1), N = x.size(2), Cin = x.size(3), F = W.size(1);
  TORCH_CHECK(W.size(0) == Cin && Cin <= GCN_MAX_CIN, "W must be [Cin,F], Cin<=8");
  TORCH_CHECK(w.size(0) == B && w.size(1) == N, "w must be [B,N]");
  int Ca = 0;
  if (anom.numel() > 0) {
    check_f32_cuda(anom, "anom");
    TORCH_CHECK(anom.size(0) == B && anom.size(1) == T, "anom must be [B,T,Ca]");
    Ca = anom.size(2);
  }
  TORCH_CHECK(Mp == 0 || (Mp >= B && Mp % 16 == 0 && Cp >= Ca + F), "gcn_pool_fwd: time-major Mp / Cp");
  c10::DeviceGuard guard(x.device());
  at::Tensor out = Mp > 0 ? at::empty({T, Mp, Cp}, x.options()) : at::empty({B, T, Ca + F}, x.options());
  const long rows = Mp > 0 ? (long)Mp * T : (long)B * T;
  const float* anom_p = Ca ? anom.data_ptr<float>() : nullptr;
  const bool staged = N * Cin <= GCN_STAGE_MAX;
  const size_t smem = staged ? ((size_t)64 * N * Cin + (size_t)(64 / T + 2) * N) * sizeof(float) : 0;
  GQ_CIN_DISPATCH(Cin, GQ_GCN_F_DISPATCH(F,
      hipLaunchKernelGGL((gcn_pool_fwd_kernel<CIN, FF>), dim3(grid_for(rows, 64, 8192)), dim3(256), smem, stream(),
                         x.data_ptr<float>(), w.data_ptr<float>(), anom_p, W.data_ptr<float>(), b.data_ptr<float>(),
                         scale.data_ptr<float>(), shift.data_ptr<float>(), alpha.data_ptr<float>(),
                         out.data_ptr<float>(), B, T, N, Ca, (int)Mp, (int)Cp)));
  GQ_LAUNCH_CHECK();
  return out;
}

at::Tensor gcn_pool_bwd(const at::Tensor& x, const at::Tensor& w, const at::Tensor& dout, const at::Tensor& W,
                        const at::Tensor& b, const at::Tensor& scale, const at::Tensor& shift,
                        const at::Tensor& alpha, int64_t c_off, bool time_major) {
  for (auto* p : {&x, &w, &dout, &W, &b, &scale, &shift, &alpha}) check_f32_cuda(*p, "gcn bwd input");
  const int B = x.size(0), T = x.size(1), N = x.size(2), Cin = x.size(3), F = W.size(1);
  TORCH_CHECK(256 % F == 0, "gcn_pool_bwd: F must divide 256");
  TORCH_CHECK(time_major ? (dout.size(0) == T && dout.size(1) >= B && dout.size(2) >= c_off + F)
                         : (dout.size(0) == B && dout.size(1) == T && dout.size(2) >= c_off + F), "dout shape");
  c10::DeviceGuard guard(x.device());
  const int nacc = 3 + Cin;
  const int rows_per_blk = 256 / F;
  // a few passes per workgroup: fewer partial rows for gcn_bwd_finalize to sum
  const int nblk = grid_for((long)B * T, rows_per_blk, 512);
  at::Tensor partial = at::empty({nblk, nacc, F}, x.options());
  const bool staged = N * Cin <= GCN_STAGE_MAX;
  const size_t smem = staged ? ((size_t)rows_per_blk * N * Cin + (size_t)(rows_per_blk / T + 2) * N) * sizeof(float) : 0;
  GQ_CIN_DISPATCH(Cin, hipLaunchKernelGGL(gcn_pool_bwd_kernel<CIN>, dim3(nblk), dim3(256), smem, stream(), x.data_ptr<float>(),
                     w.data_ptr<float>(), dout.data_ptr<float>(), W.data_ptr<float>(), b.data_ptr<float>(),
                     scale.data_ptr<float>(), shift.data_ptr<float>(), alpha.data_ptr<float>(),
                     partial.data_ptr<float>(), B, T, N, F, (int)c_off, (int)dout.size(2),
                     time_major ? (int)dout.size(1) : 0));
  GQ_LAUNCH_CHECK();
  // [nblk, 3+Cin, F]: gcn_bwd_finalize sums the blocks in fixed order (deterministic)
  return partial;
}

at::Tensor gcn_pool_bwd_input(const at::Tensor& x, const at::Tensor& w, const at::Tensor& mask,
                              const at::Tensor& dout, const at::Tensor& W, const at::Tensor& b,
                              const at::Tensor& scale, const at::Tensor& shift, const at::Tensor& alpha,
                              const at::Tensor& coef, int64_t c_off, bool time_major) {
  for (auto* p : {&x, &w, &mask, &dout, &W, &b, &scale, &shift, &alpha, &coef}) check_f32_cuda(*p, "gcn bwd_input");
  const int B = x.size(0), T = x.size(1), N = x.size(2), Cin = x.size(3), F = W.size(1);
  TORCH_CHECK(coef.numel() == 3 * F, "coef must be [3,F]");
  c10::DeviceGuard guard(x.device());
  at::Tensor dx = at::empty_like(x);
  const long rows = (long)B * T;
  GQ_CIN_DISPATCH(Cin, GQ_GCN_F_DISPATCH(F,
      hipLaunchKernelGGL((gcn_pool_bwd_input_kernel<CIN, FF>), dim3(grid_for(rows, 64, 8192)), dim3(256), 0, stream(),
                         x.data_ptr<float>(), w.data_ptr<float>(), mask.data_ptr<float>(), dout.data_ptr<float>(),
                         W.data_ptr<float>(), b.data_ptr<float>(), scale.data_ptr<float>(), shift.data_ptr<float>(),
                         alpha.data_ptr<float>(), coef.data_ptr<float>(), dx.data_ptr<float>(), B, T, N,
                         (int)c_off, (int)dout.size(2), time_major ? (int)dout.size(1) : 0)));
  GQ_LAUNCH_CHECK();
  return dx;
}

}  // namespace gq

TORCH_LIBRARY_IMPL(gnnqc, CUDA, m) {
  m.impl("gcn_stats", &gq::gcn_stats);
  m.impl("gcn_pool_fwd", &gq::gcn_pool_fwd);
  m.impl("gcn_pool_bwd", &gq::gcn_pool_bwd);
  m.impl("gcn_pool_bwd_input", &gq::gcn_pool_bwd_input);
}
