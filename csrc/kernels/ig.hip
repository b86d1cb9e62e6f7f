// Integrated-gradients device steps (reference xai/libs/integrated_gradients.py
// :919-942 interpolation, :955-1004 per-step gradients, :1006-1015 trapezoid average, :1180-1208
// input scaling / negative-value policy).
//
// The explainer folds kk interpolation steps into the batch (gnnqc/xai/ig.py); these kernels are
// the elementwise ends of that pass, each ONE launch over all steps of a chunk:
//   ig_interp   out[i, b, e] = alpha[i] * v[b, e]                     (zero baseline path points)
//   ig_accum    acc[b, e]  += sum_i w[i] * g[i, b, e]                 (trapezoid weights, fixed
//                                                                     step order: deterministic)
//   ig_finalize out[b, e]   = policy(acc[b, e] * (scale ? v[b, e] : 1))  (keep / clip / abs)
// All three stream float4 granules when n % 4 == 0 (every step slice aligned), scalars otherwise.
#include "common.h"

namespace gq {

__global__ __launch_bounds__(256) void ig_interp_kernel(const float* __restrict__ v, const float* __restrict__ alpha,
                                                        float* __restrict__ out, int kk, long n) {
  const long stride = (long)gridDim.x * blockDim.x;
  // float4 slices only when every step's slice out + s n stays 16-byte aligned (n % 4 == 0)
  const long n4 = n % 4 == 0 ? n / 4 : 0;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4; i += stride) {
    const float4 x = reinterpret_cast<const float4*>(v)[i];
    for (int s = 0; s < kk; ++s) {
      const float a = alpha[s];
      reinterpret_cast<float4*>(out + (size_t)s * n)[i] = make_float4(a * x.x, a * x.y, a * x.z, a * x.w);
    }
  }
  for (long i = n4 * 4 + blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += stride)
    for (int s = 0; s < kk; ++s) out[(size_t)s * n + i] = alpha[s] * v[i];
}

__global__ __launch_bounds__(256) void ig_accum_kernel(float* __restrict__ acc, const float* __restrict__ g,
                                                       const float* __restrict__ w, int kk, long n) {
  const long stride = (long)gridDim.x * blockDim.x;
  const long n4 = n % 4 == 0 ? n / 4 : 0;          // (as ig_interp: aligned step slices only)
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 a = reinterpret_cast<float4*>(acc)[i];
    for (int s = 0; s < kk; ++s) {
      const float ws = w[s];
      const float4 x = reinterpret_cast<const float4*>(g + (size_t)s * n)[i];
      a.x += ws * x.x;
      a.y += ws * x.y;
      a.z += ws * x.z;
      a.w += ws * x.w;
    }
    reinterpret_cast<float4*>(acc)[i] = a;
  }
  for (long i = n4 * 4 + blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += stride) {
    float a = acc[i];
    for (int s = 0; s < kk; ++s) a += w[s] * g[(size_t)s * n + i];
    acc[i] = a;
  }
}

__global__ __launch_bounds__(256) void ig_finalize_kernel(const float* __restrict__ acc, const float* __restrict__ v,
                                                          float* __restrict__ out, long n, int mode) {
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += stride) {
    float r = acc[i] * (v != nullptr ? v[i] : 1.f);
    if (mode == 1) r = fmaxf(r, 0.f);
    else if (mode == 2) r = fabsf(r);
    out[i] = r;
  }
}

static int ig_grid(long n) { return (int)std::max<long>(1, std::min<long>((n / 4 + 255) / 256, 2048)); }

static void ig_check_aligned(const at::Tensor& t, const char* name) {
  check_f32_cuda(t, name);
  TORCH_CHECK(reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0, "ig: ", name, " must be 16-byte aligned");
}

// v [B, ...] fp32, alpha [kk] -> [kk * B, ...]
at::Tensor ig_interp(const at::Tensor& v, const at::Tensor& alpha) {
  ig_check_aligned(v, "v");
  check_f32_cuda(alpha, "alpha");
  const int kk = (int)alpha.numel();
  TORCH_CHECK(kk >= 1 && v.dim() >= 1, "ig_interp: shapes");
  c10::DeviceGuard guard(v.device());
  std::vector<int64_t> shape(v.sizes().begin(), v.sizes().end());
  shape[0] *= kk;
  at::Tensor out = at::empty(shape, v.options());
  const long n = v.numel();
  if (n > 0)
    hipLaunchKernelGGL(ig_interp_kernel, dim3(ig_grid(n)), dim3(256), 0, stream(), v.data_ptr<float>(),
                       alpha.data_ptr<float>(), out.data_ptr<float>(), kk, n);
  GQ_LAUNCH_CHECK();
  return out;
}

// acc [B, ...] += sum_i w[i] g[i] with g [kk * B, ...] (step-major), w [kk]
void ig_accum(at::Tensor acc, const at::Tensor& g, const at::Tensor& w) {
  ig_check_aligned(acc, "acc");
  ig_check_aligned(g, "g");
  check_f32_cuda(w, "w");
  const int kk = (int)w.numel();
  TORCH_CHECK(kk >= 1 && g.numel() == acc.numel() * kk, "ig_accum: g must hold kk x acc elements");
  c10::DeviceGuard guard(acc.device());
  const long n = acc.numel();
  if (n > 0)
    hipLaunchKernelGGL(ig_accum_kernel, dim3(ig_grid(n)), dim3(256), 0, stream(), acc.data_ptr<float>(),
                       g.data_ptr<float>(), w.data_ptr<float>(), kk, n);
  GQ_LAUNCH_CHECK();
}

// policy(acc * v) (v empty: no input scaling); mode 0 keep, 1 clip at 0, 2 abs
at::Tensor ig_finalize(const at::Tensor& acc, const at::Tensor& v, int64_t mode) {
  check_f32_cuda(acc, "acc");
  TORCH_CHECK(mode >= 0 && mode <= 2, "ig_finalize: mode 0 keep / 1 clip / 2 abs");
  const float* vp = nullptr;
  if (v.numel() > 0) {
    check_f32_cuda(v, "v");
    TORCH_CHECK(v.numel() == acc.numel(), "ig_finalize: v / acc sizes");
    vp = v.data_ptr<float>();
  }
  c10::DeviceGuard guard(acc.device());
  at::Tensor out = at::empty_like(acc);
  const long n = acc.numel();
  if (n > 0)
    hipLaunchKernelGGL(ig_finalize_kernel, dim3(ig_grid(n * 4)), dim3(256), 0, stream(), acc.data_ptr<float>(), vp,
                       out.data_ptr<float>(), n, (int)mode);
  GQ_LAUNCH_CHECK();
  return out;
}

}  // namespace gq

TORCH_LIBRARY_IMPL(gnnqc, CUDA, m) {
  m.impl("ig_interp", &gq::ig_interp);
  m.impl("ig_accum", &gq::ig_accum);
  m.impl("ig_finalize", &gq::ig_finalize);
}
