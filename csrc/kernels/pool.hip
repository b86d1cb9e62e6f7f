// MaxPooling1D (valid padding, stride = pool size) forward / backward for gfx950.
//
// Keras MaxPooling1D in the TimeLayer (libs/create_model.py:43-136) between LSTM
// stacks. Forward keeps the window argmax as one byte per output; backward routes
// the gradient to that position (TF's MaxPoolGrad picks the first maximum) and
// writes zeros elsewhere - one pass each instead of amax + eq/where/count chains.
// Layout [M, T, C] with C contiguous: a thread owns 4 consecutive channels (float4).
#include "common.h"

namespace gq {

__global__ __launch_bounds__(256) void maxpool1d_fwd_kernel(const float* __restrict__ x, float* __restrict__ y,
                                                            uint8_t* __restrict__ idx, long M, int T, int To,
                                                            int C4, int p) {
  const long n = M * To * C4;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < n; e += (long)gridDim.x * blockDim.x) {
    const int c4 = (int)(e % C4);
    const long mo = e / C4;                    // m * To + to
    const int to = (int)(mo % To);
    const long m = mo / To;
    const float4* src = reinterpret_cast<const float4*>(x + ((m * T + (long)to * p) * C4 + c4) * 4);
    float4 best = src[0];
    uchar4 bi = make_uchar4(0, 0, 0, 0);
    for (int k = 1; k < p; ++k) {
      const float4 v = src[(long)k * C4];
      if (v.x > best.x) { best.x = v.x; bi.x = k; }
      if (v.y > best.y) { best.y = v.y; bi.y = k; }
      if (v.z > best.z) { best.z = v.z; bi.z = k; }
      if (v.w > best.w) { best.w = v.w; bi.w = k; }
    }
    reinterpret_cast<float4*>(y)[e] = best;
    reinterpret_cast<uchar4*>(idx)[e] = bi;
  }
}

__global__ __launch_bounds__(256) void maxpool1d_bwd_kernel(const float* __restrict__ dy,
                                                            const uint8_t* __restrict__ idx, float* __restrict__ dx,
                                                            long M, int T, int To, int C4, int p) {
  // one thread per (m, t, c4) of dx: reads its pooled slot (or writes 0 past To*p)
  const long n = M * (long)T * C4;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < n; e += (long)gridDim.x * blockDim.x) {
    const int c4 = (int)(e % C4);
    const long mt = e / C4;
    const int t = (int)(mt % T);
    const long m = mt / T;
    const int to = t / p, k = t - to * p;
    float4 o = make_float4(0.f, 0.f, 0.f, 0.f);
    if (to < To) {
      const long s = (m * To + to) * C4 + c4;
      const float4 g = reinterpret_cast<const float4*>(dy)[s];
      const uchar4 b = reinterpret_cast<const uchar4*>(idx)[s];
      o.x = b.x == k ? g.x : 0.f;
      o.y = b.y == k ? g.y : 0.f;
      o.z = b.z == k ? g.z : 0.f;
      o.w = b.w == k ? g.w : 0.f;
    }
    reinterpret_cast<float4*>(dx)[e] = o;
  }
}

// Row-granular forms for wide rows (the time-major TimeLayer views a [T, Mp, C] tensor as one
// [1, T, Mp C] row set: C4 in the 10^4..10^5 range): a 3-D grid (float4 column block, output step,
// sequence) instead of a flat grid-stride loop, so no thread divides a 64-bit index (the flat form's
// e % C4, e / C4 per element cost more than its memory traffic)
__global__ __launch_bounds__(256) void maxpool1d_fwd_rows_kernel(const float* __restrict__ x, float* __restrict__ y,
                                                                 uint8_t* __restrict__ idx, int T, int To, long C4,
                                                                 int p) {
  const long c4 = blockIdx.x * 256L + threadIdx.x;
  if (c4 >= C4) return;
  const long m = blockIdx.z;
  const int to = blockIdx.y;
  const float4* src = reinterpret_cast<const float4*>(x) + (m * T + (long)to * p) * C4 + c4;
  float4 best = src[0];
  uchar4 bi = make_uchar4(0, 0, 0, 0);
  for (int k = 1; k < p; ++k) {
    const float4 v = src[(long)k * C4];
    if (v.x > best.x) { best.x = v.x; bi.x = k; }
    if (v.y > best.y) { best.y = v.y; bi.y = k; }
    if (v.z > best.z) { best.z = v.z; bi.z = k; }
    if (v.w > best.w) { best.w = v.w; bi.w = k; }
  }
  const long o = (m * To + to) * C4 + c4;
  reinterpret_cast<float4*>(y)[o] = best;
  reinterpret_cast<uchar4*>(idx)[o] = bi;
}

__global__ __launch_bounds__(256) void maxpool1d_bwd_rows_kernel(const float* __restrict__ dy,
                                                                 const uint8_t* __restrict__ idx,
                                                                 float* __restrict__ dx, int T, int To, long C4,
                                                                 int p) {
  const long c4 = blockIdx.x * 256L + threadIdx.x;
  if (c4 >= C4) return;
  const long m = blockIdx.z;
  const int t = blockIdx.y;
  const int to = t / p, k = t - to * p;            // (block-uniform)
  float4 o = make_float4(0.f, 0.f, 0.f, 0.f);
  if (to < To) {
    const long s = (m * To + to) * C4 + c4;
    const float4 g = reinterpret_cast<const float4*>(dy)[s];
    const uchar4 b = reinterpret_cast<const uchar4*>(idx)[s];
    o.x = b.x == k ? g.x : 0.f;
    o.y = b.y == k ? g.y : 0.f;
    o.z = b.z == k ? g.z : 0.f;
    o.w = b.w == k ? g.w : 0.f;
  }
  reinterpret_cast<float4*>(dx)[(m * T + t) * C4 + c4] = o;
}

static bool pool_rows_form(long M, long C4) { return C4 >= 256 && M <= 65535; }

static int ew_grid(long n) { return (int)std::max<long>(1, std::min<long>((n + 255) / 256, 4096)); }

std::vector<at::Tensor> maxpool1d_fwd(const at::Tensor& x, int64_t p) {
  check_f32_cuda(x, "x");
  TORCH_CHECK(x.dim() == 3 && x.size(2) % 4 == 0, "maxpool1d: x must be [M,T,C] with C % 4 == 0");
  TORCH_CHECK(p >= 1 && p <= 255, "maxpool1d: pool size");
  const long M = x.size(0);
  const int T = (int)x.size(1), C = (int)x.size(2), To = T / (int)p;
  c10::DeviceGuard guard(x.device());
  at::Tensor y = at::empty({M, To, C}, x.options());
  at::Tensor idx = at::empty({M, To, C}, x.options().dtype(at::kByte));
  const long n = M * To * (C / 4);
  if (n > 0 && pool_rows_form(M, C / 4)) {
    hipLaunchKernelGGL(maxpool1d_fwd_rows_kernel, dim3((unsigned)((C / 4 + 255) / 256), To, (unsigned)M), dim3(256), 0,
                       stream(), x.data_ptr<float>(), y.data_ptr<float>(), idx.data_ptr<uint8_t>(), T, To,
                       (long)(C / 4), (int)p);
    GQ_LAUNCH_CHECK();
  } else if (n > 0) {
    hipLaunchKernelGGL(maxpool1d_fwd_kernel, dim3(ew_grid(n)), dim3(256), 0, stream(), x.data_ptr<float>(),
                       y.data_ptr<float>(), idx.data_ptr<uint8_t>(), M, T, To, C / 4, (int)p);
    GQ_LAUNCH_CHECK();
  }
  return {y, idx};
}

at::Tensor maxpool1d_bwd(const at::Tensor& dy, const at::Tensor& idx, int64_t T, int64_t p) {
  check_f32_cuda(dy, "dy");
  TORCH_CHECK(idx.is_cuda() && idx.scalar_type() == at::kByte && idx.is_contiguous() && idx.sizes() == dy.sizes(),
              "maxpool1d_bwd: idx must be a contiguous uint8 tensor shaped like dy");
  const long M = dy.size(0);
  const int To = (int)dy.size(1), C = (int)dy.size(2);
  TORCH_CHECK(To == T / p, "maxpool1d_bwd: T / p mismatch");
  c10::DeviceGuard guard(dy.device());
  at::Tensor dx = at::empty({M, T, C}, dy.options());
  const long n = M * T * (C / 4);
  if (n > 0 && pool_rows_form(M, C / 4)) {
    hipLaunchKernelGGL(maxpool1d_bwd_rows_kernel, dim3((unsigned)((C / 4 + 255) / 256), (unsigned)T, (unsigned)M),
                       dim3(256), 0, stream(), dy.data_ptr<float>(), idx.data_ptr<uint8_t>(), dx.data_ptr<float>(),
                       (int)T, To, (long)(C / 4), (int)p);
    GQ_LAUNCH_CHECK();
  } else if (n > 0) {
    hipLaunchKernelGGL(maxpool1d_bwd_kernel, dim3(ew_grid(n)), dim3(256), 0, stream(), dy.data_ptr<float>(),
                       idx.data_ptr<uint8_t>(), dx.data_ptr<float>(), M, (int)T, To, C / 4, (int)p);
    GQ_LAUNCH_CHECK();
  }
  return dx;
}

}  // namespace gq

TORCH_LIBRARY_IMPL(gnnqc, CUDA, m) {
  m.impl("maxpool1d_fwd", &gq::maxpool1d_fwd);
  m.impl("maxpool1d_bwd", &gq::maxpool1d_bwd);
}
