// Label-split score histograms for threshold sweeps and AUC.
//
// The reference sweeps np.unique(round(p, 3)) with sklearn's matthews_corrcoef
// (libs/test_model.py:9-17) and tracks Keras AUC with 200 thresholds. Both only
// need, per score bin, the count of positives and negatives: with bins = 1001 and
// bin = rint(p * 1000) every 3-decimal threshold's confusion matrix is a prefix
// sum. Per-block LDS histograms, one global atomic per non-empty bin per block.
#include "common.h"

namespace gq {

__global__ void score_hist_kernel(const float* __restrict__ s, const float* __restrict__ y,
                                  const float* __restrict__ mask, long n, int bins, float* out) {
  extern __shared__ float h[];   // [2 * bins]: negatives then positives
  for (int i = threadIdx.x; i < 2 * bins; i += blockDim.x) h[i] = 0.f;
  __syncthreads();
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const float m = mask ? mask[i] : 1.f;
    if (m == 0.f) continue;
    float p = s[i];
    p = fminf(fmaxf(p, 0.f), 1.f);
    int b = (int)rintf(p * (float)(bins - 1));
    b = b < 0 ? 0 : (b >= bins ? bins - 1 : b);
    const int pos = y[i] > 0.5f ? 1 : 0;
    atomicAdd(&h[pos * bins + b], m);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 2 * bins; i += blockDim.x)
    if (h[i] != 0.f) atomicAdd(&out[i], h[i]);
}

at::Tensor score_histogram(const at::Tensor& scores, const at::Tensor& labels, const at::Tensor& mask,
                           int64_t bins) {
  check_f32_cuda(scores, "scores");
  check_f32_cuda(labels, "labels");
  TORCH_CHECK(bins >= 2 && bins <= 16384, "bins must be in [2, 16384]");
  const long n = scores.numel();
  TORCH_CHECK(labels.numel() == n, "labels size");
  const float* mp = nullptr;
  if (mask.numel() > 0) {
    check_f32_cuda(mask, "mask");
    TORCH_CHECK(mask.numel() == n, "mask size");
    mp = mask.data_ptr<float>();
  }
  c10::DeviceGuard guard(scores.device());
  at::Tensor out = at::zeros({2, bins}, scores.options());
  const int grid = (int)std::max<long>(1, std::min<long>((n + 255) / 256, 512));
  hipLaunchKernelGGL(score_hist_kernel, dim3(grid), dim3(256), 2 * bins * sizeof(float), stream(),
                     scores.data_ptr<float>(), labels.data_ptr<float>(), mp, n, (int)bins, out.data_ptr<float>());
  GQ_LAUNCH_CHECK();
  return out;
}

}  // namespace gq

TORCH_LIBRARY_IMPL(gnnqc, CUDA, m) { m.impl("score_histogram", &gq::score_histogram); }
