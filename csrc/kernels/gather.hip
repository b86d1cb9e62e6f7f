// On-device window gather + normalisation.
//
// Replaces the reference's host-side TFRecord parse + ragged->dense conversion +
// normalisation (libs/preprocessing_functions.py:566-634) with one streaming
// kernel over HBM-resident series:
//   x[b,t,n,c] = (series[g, c0 - tb + t, n, c] - shift[g, tc, n, c]) * scale[g, tc, n, c] * valid[w, n]
// with g = win_group[w], c0 = win_center[w], tc = c0 (time-varying rolling stats) or 0,
// w = wids[b] (-1 = padding -> zeros). The (n, c) slab of one time step is
// contiguous in both source and destination, so the copy is fully coalesced.
#include "common.h"

namespace gq {

__global__ void window_gather_kernel(const float* __restrict__ series, const float* __restrict__ shift,
                                     const float* __restrict__ scale, const long* __restrict__ wg,
                                     const long* __restrict__ wc, const uint8_t* __restrict__ wv,
                                     const long* __restrict__ wids, float* __restrict__ out, int B, int Tw,
                                     int Ttot, int Tn, int NC, int C, int tb, int time_norm) {
  const long total = (long)B * Tw * NC;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int nc = i % NC;
    const long bt = i / NC;
    const int t = bt % Tw;
    const int b = bt / Tw;
    const long w = wids[b];
    float val = 0.f;
    if (w >= 0) {
      const int n = nc / C;
      const long N = NC / C;
      if (wv[w * N + n]) {
        const long g = wg[w];
        const long c0 = wc[w];
        const long ts = c0 - tb + t;
        const long tn = time_norm ? c0 : 0;
        const float x = series[(g * Ttot + ts) * NC + nc];
        const long k = (g * Tn + tn) * NC + nc;
        val = (x - shift[k]) * scale[k];
      }
    }
    out[i] = val;
  }
}

at::Tensor window_gather(const at::Tensor& series, const at::Tensor& shift, const at::Tensor& scale,
                         const at::Tensor& win_group, const at::Tensor& win_center, const at::Tensor& win_valid,
                         const at::Tensor& wids, int64_t tb, int64_t seq_len, bool time_norm) {
  check_f32_cuda(series, "series");
  check_f32_cuda(shift, "shift");
  check_f32_cuda(scale, "scale");
  TORCH_CHECK(series.dim() == 4, "series must be [G,Ttot,N,C]");
  TORCH_CHECK(win_group.scalar_type() == at::kLong && win_center.scalar_type() == at::kLong &&
                  wids.scalar_type() == at::kLong, "index tensors must be int64");
  TORCH_CHECK(win_valid.scalar_type() == at::kByte && win_valid.is_contiguous(), "win_valid must be uint8");
  const int G = series.size(0), Ttot = series.size(1), N = series.size(2), C = series.size(3);
  TORCH_CHECK(shift.size(0) == G && shift.size(2) == N && shift.size(3) == C, "shift shape");
  TORCH_CHECK(scale.sizes() == shift.sizes(), "scale shape");
  TORCH_CHECK(win_valid.size(1) == N, "win_valid must be [W,N]");
  const int B = wids.size(0);
  c10::DeviceGuard guard(series.device());
  at::Tensor out = at::empty({B, seq_len, N, C}, series.options());
  const long total = (long)B * seq_len * N * C;
  const int grid = (int)std::max<long>(1, std::min<long>((total + 255) / 256, 8192));
  hipLaunchKernelGGL(window_gather_kernel, dim3(grid), dim3(256), 0, stream(), series.data_ptr<float>(),
                     shift.data_ptr<float>(), scale.data_ptr<float>(), win_group.data_ptr<long>(),
                     win_center.data_ptr<long>(), win_valid.data_ptr<uint8_t>(), wids.data_ptr<long>(),
                     out.data_ptr<float>(), B, (int)seq_len, Ttot, (int)shift.size(1), N * C, C, (int)tb,
                     time_norm ? 1 : 0);
  GQ_LAUNCH_CHECK();
  return out;
}

}  // namespace gq

TORCH_LIBRARY_IMPL(gnnqc, CUDA, m) { m.impl("window_gather", &gq::window_gather); }
