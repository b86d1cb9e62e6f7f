// Single-launch Adam over the flat fp32 parameter buffer.
//
// The reference uses Keras Adam (jit_compile XLA; beta1 .9, beta2 .999, eps 1e-7,
// libs/fit_model.py:71-74). Keras' update rule is the "epsilon hat" form:
//   m = b1 m + (1-b1) g ; v = b2 v + (1-b2) g^2
//   p -= lr * sqrt(1-b2^t)/(1-b1^t) * m / (sqrt(v) + eps)
// All trainables live in one contiguous buffer (parameters are views into it) so
// the optimiser is one kernel and the DP gradient all-reduce is one collective;
// grad_scale folds the 1/world averaging in. lr and step are device tensors so the
// launch can be captured in a HIP graph and replayed with a changing schedule.
#include "common.h"

namespace gq {

__global__ void adam_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                            float* __restrict__ v, const float* __restrict__ lr_p, const float* __restrict__ step_p,
                            long n, float b1, float b2, float eps, float gscale, float wd) {
  const float step = *step_p;
  const float lr = *lr_p;
  const float bc1 = 1.0f - powf(b1, step);
  const float bc2 = 1.0f - powf(b2, step);
  const float alpha = lr * sqrtf(bc2) / bc1;
  const long n4 = n / 4;
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 gg = reinterpret_cast<const float4*>(g)[i];
    float4 pp = reinterpret_cast<float4*>(p)[i];
    float4 mm = reinterpret_cast<float4*>(m)[i];
    float4 vv = reinterpret_cast<float4*>(v)[i];
#define GQ_ADAM_LANE(c)                                         \
    {                                                           \
      float gc = gg.c * gscale + wd * pp.c;                     \
      mm.c = b1 * mm.c + (1.f - b1) * gc;                       \
      vv.c = b2 * vv.c + (1.f - b2) * gc * gc;                  \
      pp.c -= alpha * mm.c / (sqrtf(vv.c) + eps);               \
    }
    GQ_ADAM_LANE(x) GQ_ADAM_LANE(y) GQ_ADAM_LANE(z) GQ_ADAM_LANE(w)
#undef GQ_ADAM_LANE
    reinterpret_cast<float4*>(p)[i] = pp;
    reinterpret_cast<float4*>(m)[i] = mm;
    reinterpret_cast<float4*>(v)[i] = vv;
  }
  for (long i = n4 * 4 + blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += stride) {
    float gc = g[i] * gscale + wd * p[i];
    m[i] = b1 * m[i] + (1.f - b1) * gc;
    v[i] = b2 * v[i] + (1.f - b2) * gc * gc;
    p[i] -= alpha * m[i] / (sqrtf(v[i]) + eps);
  }
}

__global__ void nonfinite_kernel(const float* __restrict__ x, long n, int* out) {
  int bad = 0;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    bad += !isfinite(x[i]);
  // wave-level reduce then one atomic per wave
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) bad += __shfl_xor(bad, o, 64);
  if ((threadIdx.x & 63) == 0 && bad) atomicAdd(out, bad);
}

void adam_step(at::Tensor p, const at::Tensor& g, at::Tensor m, at::Tensor v, const at::Tensor& lr,
               const at::Tensor& step, double b1, double b2, double eps, double gscale, double wd) {
  const at::Tensor* ops[] = {&p, &g, &m, &v, &lr, &step};
  for (const at::Tensor* t : ops) check_f32_cuda(*t, "adam operand");
  const long n = p.numel();
  TORCH_CHECK(g.numel() == n && m.numel() == n && v.numel() == n, "adam: size mismatch");
  TORCH_CHECK((reinterpret_cast<uintptr_t>(p.data_ptr()) % 16) == 0 && (reinterpret_cast<uintptr_t>(g.data_ptr()) % 16) == 0,
              "adam: buffers must be 16-byte aligned");
  c10::DeviceGuard guard(p.device());
  const int block = 256;
  const int grid = (int)std::max<long>(1, std::min<long>((n / 4 + block - 1) / block, 1024));
  hipLaunchKernelGGL(adam_kernel, dim3(grid), dim3(block), 0, stream(), p.data_ptr<float>(), g.data_ptr<float>(),
                     m.data_ptr<float>(), v.data_ptr<float>(), lr.data_ptr<float>(), step.data_ptr<float>(), n,
                     (float)b1, (float)b2, (float)eps, (float)gscale, (float)wd);
  GQ_LAUNCH_CHECK();
}

at::Tensor nonfinite_count(const at::Tensor& x) {
  check_f32_cuda(x, "x");
  c10::DeviceGuard guard(x.device());
  at::Tensor out = at::zeros({1}, x.options().dtype(at::kInt));
  const long n = x.numel();
  const int grid = (int)std::max<long>(1, std::min<long>((n + 255) / 256, 1024));
  hipLaunchKernelGGL(nonfinite_kernel, dim3(grid), dim3(256), 0, stream(), x.data_ptr<float>(), n,
                     out.data_ptr<int>());
  GQ_LAUNCH_CHECK();
  return out;
}

}  // namespace gq

TORCH_LIBRARY_IMPL(gnnqc, CUDA, m) {
  m.impl("adam_step", &gq::adam_step);
  m.impl("nonfinite_count", &gq::nonfinite_count);
}
