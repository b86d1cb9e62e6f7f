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

// Everything else a batch needs, one workgroup per sample (replaces ~12 small indexing /
// masking launches): node mask, masked adjacency, flagged-node position, labels and label
// mask, and (CML) the flagged sensor's series cut from the gathered x.
//   vm[b,n]    = (w >= 0) * win_valid[w,n]
//   adj[b,i,j] = group_adj[g,i,j] * vm[b,i] * vm[b,j]
//   CML:     y[b] = win_label[w] * ok, y_mask[b] = ok, anom[b,t,c] = x[b,t,max(ap,0),c]
//   SoilNet: y[b,n] = win_label[w,n] * vm[b,n], y_mask[b,n] = win_label_valid[w,n] * ok
// with w = max(wids[b], 0), g = win_group[w], ok = (wids[b] >= 0) * valid_sample[b].
__global__ __launch_bounds__(256) void batch_meta_kernel(
    const long* __restrict__ wids, const long* __restrict__ wg, const uint8_t* __restrict__ wv,
    const float* __restrict__ gadj, const long* __restrict__ gap, const float* __restrict__ wlab,
    const float* __restrict__ wlabv, const float* __restrict__ vsample, const float* __restrict__ x,
    float* __restrict__ vm, float* __restrict__ adj, long* __restrict__ ap, float* __restrict__ y,
    float* __restrict__ ym, float* __restrict__ anom, int N, int T, int C, int soil) {
  const int b = blockIdx.x, tid = threadIdx.x;
  const long wraw = wids[b];
  const long w = wraw < 0 ? 0 : wraw;
  const float ok = (wraw >= 0 ? 1.f : 0.f) * (vsample != nullptr ? vsample[b] : 1.f);
  const long g = wg[w];
  const float live = wraw >= 0 ? 1.f : 0.f;
  __shared__ float svm[1024];
  for (int n = tid; n < N; n += 256) {
    const float v = live * (wv[w * N + n] ? 1.f : 0.f);
    svm[n] = v;
    vm[(long)b * N + n] = v;
    if (soil) {
      y[(long)b * N + n] = wlab[w * N + n] * v;
      ym[(long)b * N + n] = wlabv[w * N + n] * ok;
    }
  }
  __syncthreads();
  const float* A = gadj + g * (long)N * N;
  float* out = adj + (long)b * N * N;
  for (int e = tid; e < N * N; e += 256) out[e] = A[e] * svm[e / N] * svm[e % N];
  const long a = gap[g];
  if (tid == 0) {
    ap[b] = a;
    if (!soil) {
      y[b] = wlab[w] * ok;
      ym[b] = ok;
    }
  }
  if (!soil) {
    const long n0 = a < 0 ? 0 : a;
    for (int e = tid; e < T * C; e += 256) {
      const int t = e / C, c = e % C;
      anom[((long)b * T + t) * C + c] = x[(((long)b * T + t) * N + n0) * C + c];
    }
  }
}

// returns [vm, adj, anom_pos, y, y_mask, anom (CML; empty for SoilNet)]
std::vector<at::Tensor> batch_meta(const at::Tensor& wids, const at::Tensor& win_group, const at::Tensor& win_valid,
                                   const at::Tensor& group_adj, const at::Tensor& group_anom_pos,
                                   const at::Tensor& win_label, const at::Tensor& win_label_valid,
                                   const at::Tensor& valid_sample, const at::Tensor& x) {
  TORCH_CHECK(wids.scalar_type() == at::kLong && win_group.scalar_type() == at::kLong &&
                  group_anom_pos.scalar_type() == at::kLong, "batch_meta: index tensors must be int64");
  TORCH_CHECK(win_valid.scalar_type() == at::kByte && win_valid.is_contiguous(), "batch_meta: win_valid uint8");
  check_f32_cuda(group_adj, "group_adj");
  check_f32_cuda(win_label, "win_label");
  check_f32_cuda(x, "x");
  TORCH_CHECK(x.dim() == 4, "batch_meta: x must be [B,T,N,C]");
  const int B = wids.size(0), T = x.size(1), N = x.size(2), C = x.size(3);
  TORCH_CHECK(N <= 1024 && win_valid.size(1) == N && group_adj.size(1) == N && group_adj.size(2) == N,
              "batch_meta: node dimension");
  const bool soil = win_label.dim() == 2;
  if (soil) {
    check_f32_cuda(win_label_valid, "win_label_valid");
    TORCH_CHECK(win_label.size(1) == N && win_label_valid.sizes() == win_label.sizes(), "batch_meta: label shapes");
  }
  const float* vs = nullptr;
  if (valid_sample.numel() > 0) {
    check_f32_cuda(valid_sample, "valid_sample");
    TORCH_CHECK(valid_sample.numel() == B, "batch_meta: valid_sample must be [B]");
    vs = valid_sample.data_ptr<float>();
  }
  c10::DeviceGuard guard(x.device());
  auto fo = x.options();
  at::Tensor vm = at::empty({B, N}, fo), adj = at::empty({B, N, N}, fo);
  at::Tensor ap = at::empty({B}, wids.options());
  at::Tensor y = soil ? at::empty({B, N}, fo) : at::empty({B}, fo);
  at::Tensor ym = soil ? at::empty({B, N}, fo) : at::empty({B}, fo);
  at::Tensor anom = soil ? at::empty({0}, fo) : at::empty({B, T, C}, fo);
  hipLaunchKernelGGL(batch_meta_kernel, dim3(B), dim3(256), 0, stream(), wids.data_ptr<long>(),
                     win_group.data_ptr<long>(), win_valid.data_ptr<uint8_t>(), group_adj.data_ptr<float>(),
                     group_anom_pos.data_ptr<long>(), win_label.data_ptr<float>(),
                     soil ? win_label_valid.data_ptr<float>() : nullptr, vs, x.data_ptr<float>(),
                     vm.data_ptr<float>(), adj.data_ptr<float>(), ap.data_ptr<long>(), y.data_ptr<float>(),
                     ym.data_ptr<float>(), soil ? nullptr : anom.data_ptr<float>(), N, T, C, soil ? 1 : 0);
  GQ_LAUNCH_CHECK();
  return {vm, adj, ap, y, ym, anom};
}

// window_gather + batch_meta as ONE launch (one workgroup per sample): the sample's node mask
// goes to LDS first, then the window cut (4 elements per thread per round, loads issued before
// use; masked nodes read a valid address and are multiplied out), the flagged sensor's series
// (CML) taken from the values as they are cut, and the meta outputs. cursor (optional): the
// batch is row (cursor[0] % nrows) of the device table [nrows, B] (multi-step graphs); the
// window ids used are written to wid_out.
__global__ __launch_bounds__(256) void batch_gather_kernel(
    const float* __restrict__ series, const float* __restrict__ shift, const float* __restrict__ scale,
    const long* __restrict__ wg, const long* __restrict__ wc, const uint8_t* __restrict__ wv,
    const long* __restrict__ wids, const long* __restrict__ table, const long* __restrict__ cursor, long nrows,
    const float* __restrict__ gadj, const long* __restrict__ gap, const float* __restrict__ wlab,
    const float* __restrict__ wlabv, const float* __restrict__ vsample, float* __restrict__ x,
    float* __restrict__ vm, float* __restrict__ adj, long* __restrict__ ap, float* __restrict__ y,
    float* __restrict__ ym, float* __restrict__ anom, long* __restrict__ wid_out, int B, int Tw, int Ttot, int Tn,
    int N, int C, int tb, int time_norm, int soil) {
  // grid (B, NY): workgroup (b, y) cuts slice y of sample b's window; y == 0 also writes the meta
  const int b = blockIdx.x, tid = threadIdx.x;
  const bool meta = blockIdx.y == 0;
  const long* ids = cursor != nullptr ? table + (cursor[0] % nrows) * B : wids;
  const long wraw = ids[b];
  const long w = wraw < 0 ? 0 : wraw;
  const float ok = (wraw >= 0 ? 1.f : 0.f) * (vsample != nullptr ? vsample[b] : 1.f);
  const long g = wg[w];
  const float live = wraw >= 0 ? 1.f : 0.f;
  const long a = gap[g];
  const int n0 = a < 0 ? 0 : (int)a;
  const int NC = N * C;
  __shared__ float svm[1024];
  for (int n = tid; n < N; n += 256) {
    const float v = live * (wv[w * N + n] ? 1.f : 0.f);
    svm[n] = v;
    if (meta) {
      vm[(long)b * N + n] = v;
      if (soil) {
        y[(long)b * N + n] = wlab[w * N + n] * v;
        ym[(long)b * N + n] = wlabv[w * N + n] * ok;
      }
    }
  }
  if (meta && tid == 0) {
    ap[b] = a;
    wid_out[b] = wraw;
    if (!soil) {
      y[b] = wlab[w] * ok;
      ym[b] = ok;
    }
  }
  __syncthreads();
  if (meta) {
    const float* A = gadj + g * (long)N * N;
    float* out = adj + (long)b * N * N;
    for (int e = tid; e < N * N; e += 256) out[e] = A[e] * svm[e / N] * svm[e % N];
  }
  const long c0 = wc[w];
  const float* src = series + (g * Ttot + (c0 - tb)) * (long)NC;
  const long tn = time_norm ? c0 : 0;
  const float* sh = shift + (g * Tn + tn) * (long)NC;
  const float* sc = scale + (g * Tn + tn) * (long)NC;
  float* xo = x + (long)b * Tw * NC;
  const int total = Tw * NC;
  const int per = ((total + gridDim.y - 1) / gridDim.y + 1023) / 1024 * 1024;
  const int e_end = min(total, ((int)blockIdx.y + 1) * per);
  for (int e0 = (int)blockIdx.y * per + tid; e0 < e_end; e0 += 4 * 256) {
    float xv[4], sv[4], cv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = min(e0 + u * 256, e_end - 1);
      xv[u] = src[e];
      sv[u] = sh[e % NC];
      cv[u] = sc[e % NC];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = e0 + u * 256;
      if (e < e_end) {
        const int nc = e % NC, n = nc / C;
        const float val = (xv[u] - sv[u]) * cv[u] * svm[n];
        xo[e] = val;
        if (!soil && n == n0) anom[((long)b * Tw + e / NC) * C + (nc - n * C)] = val;
      }
    }
  }
}

// [x, vm, adj, anom_pos, y, y_mask, anom (CML; empty for SoilNet), wid] in one launch; ids from
// wids [B], or (cursor defined) from row cursor % table.size(0) of table [rows, B]
std::vector<at::Tensor> batch_gather(const at::Tensor& series, const at::Tensor& shift, const at::Tensor& scale,
                                     const at::Tensor& win_group, const at::Tensor& win_center,
                                     const at::Tensor& win_valid, const at::Tensor& wids, const at::Tensor& table,
                                     const c10::optional<at::Tensor>& cursor, const at::Tensor& group_adj,
                                     const at::Tensor& group_anom_pos, const at::Tensor& win_label,
                                     const at::Tensor& win_label_valid, const at::Tensor& valid_sample, int64_t tb,
                                     int64_t seq_len, bool time_norm) {
  check_f32_cuda(series, "series");
  check_f32_cuda(shift, "shift");
  check_f32_cuda(scale, "scale");
  check_f32_cuda(group_adj, "group_adj");
  check_f32_cuda(win_label, "win_label");
  TORCH_CHECK(series.dim() == 4, "batch_gather: series must be [G,Ttot,N,C]");
  TORCH_CHECK(win_group.scalar_type() == at::kLong && win_center.scalar_type() == at::kLong &&
                  group_anom_pos.scalar_type() == at::kLong, "batch_gather: index tensors must be int64");
  TORCH_CHECK(win_valid.scalar_type() == at::kByte && win_valid.is_contiguous(), "batch_gather: win_valid uint8");
  const int G = series.size(0), Ttot = series.size(1), N = series.size(2), C = series.size(3);
  TORCH_CHECK(shift.size(0) == G && shift.size(2) == N && shift.size(3) == C && scale.sizes() == shift.sizes(),
              "batch_gather: shift / scale shape");
  TORCH_CHECK(N <= 1024 && win_valid.size(1) == N && group_adj.size(1) == N && group_adj.size(2) == N,
              "batch_gather: node dimension");
  const long* wp = nullptr;
  const long* tp = nullptr;
  const long* cp = nullptr;
  long nrows = 1;
  int B;
  if (cursor.has_value() && cursor->defined()) {
    TORCH_CHECK(table.dim() == 2 && table.scalar_type() == at::kLong && table.is_contiguous() && table.is_cuda(),
                "batch_gather: table must be a contiguous int64 [rows, B] device tensor");
    TORCH_CHECK(cursor->scalar_type() == at::kLong && cursor->numel() >= 1 && cursor->is_cuda(),
                "batch_gather: cursor must be int64[1] on the device");
    B = table.size(1);
    nrows = table.size(0);
    tp = table.data_ptr<long>();
    cp = cursor->data_ptr<long>();
  } else {
    TORCH_CHECK(wids.scalar_type() == at::kLong && wids.is_contiguous() && wids.is_cuda(), "batch_gather: wids int64");
    B = wids.size(0);
    wp = wids.data_ptr<long>();
  }
  const bool soil = win_label.dim() == 2;
  if (soil) {
    check_f32_cuda(win_label_valid, "win_label_valid");
    TORCH_CHECK(win_label.size(1) == N && win_label_valid.sizes() == win_label.sizes(), "batch_gather: label shapes");
  }
  const float* vs = nullptr;
  if (valid_sample.numel() > 0) {
    check_f32_cuda(valid_sample, "valid_sample");
    TORCH_CHECK(valid_sample.numel() == B, "batch_gather: valid_sample must be [B]");
    vs = valid_sample.data_ptr<float>();
  }
  c10::DeviceGuard guard(series.device());
  auto fo = series.options();
  at::Tensor x = at::empty({B, seq_len, N, C}, fo);
  at::Tensor vm = at::empty({B, N}, fo), adj = at::empty({B, N, N}, fo);
  at::Tensor ap = at::empty({B}, win_group.options());
  at::Tensor y = soil ? at::empty({B, N}, fo) : at::empty({B}, fo);
  at::Tensor ym = soil ? at::empty({B, N}, fo) : at::empty({B}, fo);
  at::Tensor anom = soil ? at::empty({0}, fo) : at::empty({B, seq_len, C}, fo);
  at::Tensor wid = at::empty({B}, win_group.options());
  // one round of 4 elements per thread per workgroup: the cut is latency-bound per workgroup
  const int ny = (int)std::max<long>(1, std::min<long>(((long)seq_len * N * C + 1023) / 1024, 32));
  hipLaunchKernelGGL(batch_gather_kernel, dim3(B, ny), dim3(256), 0, stream(), series.data_ptr<float>(),
                     shift.data_ptr<float>(), scale.data_ptr<float>(), win_group.data_ptr<long>(),
                     win_center.data_ptr<long>(), win_valid.data_ptr<uint8_t>(), wp, tp, cp, nrows,
                     group_adj.data_ptr<float>(), group_anom_pos.data_ptr<long>(), win_label.data_ptr<float>(),
                     soil ? win_label_valid.data_ptr<float>() : nullptr, vs, x.data_ptr<float>(), vm.data_ptr<float>(),
                     adj.data_ptr<float>(), ap.data_ptr<long>(), y.data_ptr<float>(), ym.data_ptr<float>(),
                     soil ? nullptr : anom.data_ptr<float>(), wid.data_ptr<long>(), B, (int)seq_len, Ttot,
                     (int)shift.size(1), N, C, (int)tb, time_norm ? 1 : 0, soil ? 1 : 0);
  GQ_LAUNCH_CHECK();
  return {x, vm, adj, ap, y, ym, anom, wid};
}

}  // namespace gq

TORCH_LIBRARY_IMPL(gnnqc, CUDA, m) {
  m.impl("batch_gather", &gq::batch_gather);
  m.impl("window_gather", &gq::window_gather);
  m.impl("batch_meta", &gq::batch_meta);
}
