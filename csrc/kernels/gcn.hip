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
// thread = (row=(b,t), f); loops over the N nodes of its sample.
template <int Cin>
__global__ void gcn_pool_fwd_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                    const float* __restrict__ anom, const float* __restrict__ W,
                                    const float* __restrict__ bias, const float* __restrict__ scale,
                                    const float* __restrict__ shift, const float* __restrict__ alpha,
                                    float* __restrict__ out, int B, int T, int N, int F, int Ca) {
  const int Fo = Ca + F;
  const long total = (long)B * T * Fo;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int f = i % Fo;
    const long row = i / Fo;          // b*T + t
    const int b = row / T;
    if (f < Ca) {
      out[i] = anom[row * Ca + f];
      continue;
    }
    const int ff = f - Ca;
    float wk[Cin];
    _Pragma("unroll") for (int k = 0; k < Cin; ++k) wk[k] = W[k * F + ff];
    const float bb = bias[ff], sc = scale[ff], sh = shift[ff], al = alpha[ff];
    const float* xr = x + row * (long)N * Cin;
    const float* wr = w + (long)b * N;
    float acc = 0.f;
    for (int n = 0; n < N; ++n) {
      const float wn = wr[n];
      if (wn == 0.f) continue;
      float z = bb;
      _Pragma("unroll") for (int k = 0; k < Cin; ++k) z += xr[n * Cin + k] * wk[k];
      const float y = z * sc + sh;
      acc += wn * (y > 0.f ? y : al * y);
    }
    out[i] = acc;
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
                                    int dstride) {
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
  for (long row = (long)blockIdx.x * rows_per_blk + rsub; row < nrows; row += (long)gridDim.x * rows_per_blk) {
    const int b = row / T;
    const float g = dout[row * dstride + c_off + f];
    const float* xr = x + row * (long)N * Cin;
    const float* wr = w + (long)b * N;
    for (int n = 0; n < N; ++n) {
      const float wn = wr[n];
      if (wn == 0.f) continue;
      float z = bb;
      _Pragma("unroll") for (int k = 0; k < Cin; ++k) z += xr[n * Cin + k] * wk[k];
      const float y = z * sc + sh;
      const float da = wn * g;
      const float dy = y > 0.f ? da : al * da;
      acc[0] += dy;
      acc[1] += dy * z;
      acc[2] += y > 0.f ? 0.f : da * y;
      _Pragma("unroll") for (int k = 0; k < Cin; ++k) acc[3 + k] += xr[n * Cin + k] * dy;
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
// thread = node row (b,t,n): dz_f = c1_f*dy_f + c0_f + c2_f*z_f (valid rows), dx_k = sum_f W[k,f] dz_f
template <int Cin>
__global__ void gcn_pool_bwd_input_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                          const float* __restrict__ mask, const float* __restrict__ dout,
                                          const float* __restrict__ W, const float* __restrict__ bias,
                                          const float* __restrict__ scale, const float* __restrict__ shift,
                                          const float* __restrict__ alpha, const float* __restrict__ coef,
                                          float* __restrict__ dx, int B, int T, int N, int F, int c_off,
                                          int dstride) {
  const long rows = (long)B * T * N;
  for (long r = blockIdx.x * (long)blockDim.x + threadIdx.x; r < rows; r += (long)gridDim.x * blockDim.x) {
    const int n = r % N;
    const long bt = r / N;
    const int b = bt / T;
    float xv[Cin], dxv[Cin];
    _Pragma("unroll") for (int k = 0; k < Cin; ++k) {
      xv[k] = x[r * Cin + k];
      dxv[k] = 0.f;
    }
    const float m = mask[b * N + n];
    if (m != 0.f) {
      const float wn = w[b * N + n];
      for (int f = 0; f < F; ++f) {
        float z = bias[f];
        _Pragma("unroll") for (int k = 0; k < Cin; ++k) z += xv[k] * W[k * F + f];
        const float y = z * scale[f] + shift[f];
        const float da = wn * dout[bt * dstride + c_off + f];
        const float dy = y > 0.f ? da : alpha[f] * da;
        const float dz = coef[F + f] * dy + coef[f] + coef[2 * F + f] * z;
        _Pragma("unroll") for (int k = 0; k < Cin; ++k) dxv[k] += W[k * F + f] * dz;
      }
    }
    _Pragma("unroll") for (int k = 0; k < Cin; ++k) dx[r * Cin + k] = dxv[k];
  }
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

at::Tensor gcn_pool_fwd(const at::Tensor& x, const at::Tensor& w, const at::Tensor& anom, const at::Tensor& W,
                        const at::Tensor& b, const at::Tensor& scale, const at::Tensor& shift,
                        const at::Tensor& alpha) {
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
  c10::DeviceGuard guard(x.device());
  at::Tensor out = at::empty({B, T, Ca + F}, x.options());
  const long total = (long)B * T * (Ca + F);
  const float* anom_p = Ca ? anom.data_ptr<float>() : nullptr;
  GQ_CIN_DISPATCH(Cin, hipLaunchKernelGGL(gcn_pool_fwd_kernel<CIN>, dim3(grid_for(total, 256, 4096)), dim3(256), 0,
                     stream(), x.data_ptr<float>(), w.data_ptr<float>(), anom_p,
                     W.data_ptr<float>(), b.data_ptr<float>(), scale.data_ptr<float>(), shift.data_ptr<float>(),
                     alpha.data_ptr<float>(), out.data_ptr<float>(), B, T, N, F, Ca));
  GQ_LAUNCH_CHECK();
  return out;
}

at::Tensor gcn_pool_bwd(const at::Tensor& x, const at::Tensor& w, const at::Tensor& dout, const at::Tensor& W,
                        const at::Tensor& b, const at::Tensor& scale, const at::Tensor& shift,
                        const at::Tensor& alpha, int64_t c_off) {
  for (auto* p : {&x, &w, &dout, &W, &b, &scale, &shift, &alpha}) check_f32_cuda(*p, "gcn bwd input");
  const int B = x.size(0), T = x.size(1), N = x.size(2), Cin = x.size(3), F = W.size(1);
  TORCH_CHECK(256 % F == 0, "gcn_pool_bwd: F must divide 256");
  TORCH_CHECK(dout.size(0) == B && dout.size(1) == T && dout.size(2) >= c_off + F, "dout shape");
  c10::DeviceGuard guard(x.device());
  const int nacc = 3 + Cin;
  const int rows_per_blk = 256 / F;
  const int nblk = grid_for((long)B * T, rows_per_blk, 2048);
  at::Tensor partial = at::empty({nblk, nacc, F}, x.options());
  GQ_CIN_DISPATCH(Cin, hipLaunchKernelGGL(gcn_pool_bwd_kernel<CIN>, dim3(nblk), dim3(256), 0, stream(), x.data_ptr<float>(),
                     w.data_ptr<float>(), dout.data_ptr<float>(), W.data_ptr<float>(), b.data_ptr<float>(),
                     scale.data_ptr<float>(), shift.data_ptr<float>(), alpha.data_ptr<float>(),
                     partial.data_ptr<float>(), B, T, N, F, (int)c_off, (int)dout.size(2)));
  GQ_LAUNCH_CHECK();
  return partial.sum(0);   // [3+Cin, F], fixed-order (deterministic) reduction
}

at::Tensor gcn_pool_bwd_input(const at::Tensor& x, const at::Tensor& w, const at::Tensor& mask,
                              const at::Tensor& dout, const at::Tensor& W, const at::Tensor& b,
                              const at::Tensor& scale, const at::Tensor& shift, const at::Tensor& alpha,
                              const at::Tensor& coef, int64_t c_off) {
  for (auto* p : {&x, &w, &mask, &dout, &W, &b, &scale, &shift, &alpha, &coef}) check_f32_cuda(*p, "gcn bwd_input");
  const int B = x.size(0), T = x.size(1), N = x.size(2), Cin = x.size(3), F = W.size(1);
  TORCH_CHECK(coef.numel() == 3 * F, "coef must be [3,F]");
  c10::DeviceGuard guard(x.device());
  at::Tensor dx = at::empty_like(x);
  const long rows = (long)B * T * N;
  GQ_CIN_DISPATCH(Cin, hipLaunchKernelGGL(gcn_pool_bwd_input_kernel<CIN>, dim3(grid_for(rows, 256, 4096)), dim3(256), 0, stream(),
                     x.data_ptr<float>(), w.data_ptr<float>(), mask.data_ptr<float>(), dout.data_ptr<float>(),
                     W.data_ptr<float>(), b.data_ptr<float>(), scale.data_ptr<float>(), shift.data_ptr<float>(),
                     alpha.data_ptr<float>(), coef.data_ptr<float>(), dx.data_ptr<float>(), B, T, N, F,
                     (int)c_off, (int)dout.size(2)));
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
