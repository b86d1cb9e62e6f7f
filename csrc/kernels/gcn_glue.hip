// Small fused kernels around the GeneralConv + pooling block (gcn.hip) for gfx950.
//
// Without these, each training step runs ~45 tiny PyTorch kernels between the
// streaming passes (adjacency degree / mask normalisation + bmm for the pooling
// weights; fp64 einsums for the BatchNorm batch statistics and the running-stat
// update; ~20 elementwise ops for the closed-form weight gradients). Each is a
// 1-5 us launch on a [16]-sized tensor. Here they are three launches:
//
//  gcn_pool_weights  w[b,j] = sum_i p[b,i] / deg[b,i] * A[b,i,j]   (one block / sample)
//  gcn_bn_prep       mu, 1/sigma, scale, shift (+ Keras running-stat update) from the
//                    x moments of gcn_stats, in fp64                  (one block)
//  gcn_bwd_finalize  dW, db, dgamma, dbeta, dalpha accumulated straight into the
//                    gradient buffers + the dx coefficients          (one block)
//
// Semantics: spektral GeneralConv + Keras BatchNormalization (momentum .99, eps 1e-3,
// biased batch variance), libs/create_model.py:184-189, :8-41.
#include "common.h"

namespace gq {

constexpr int GLUE_MAX_CIN = 8;

// pool: 0 mean over valid nodes, 1 sum, 2 selection of anom_pos ; agg_mean: divide by in-degree
__global__ __launch_bounds__(256) void gcn_pool_weights_kernel(const float* __restrict__ adj,
                                                               const float* __restrict__ mask,
                                                               const int64_t* __restrict__ anom_pos, int N,
                                                               int agg_mean, int pool, float* __restrict__ w) {
  extern __shared__ float coef[];       // [N]
  __shared__ float red[4];
  const int b = blockIdx.x;
  const float* A = adj + (long)b * N * N;
  const float* m = mask + (long)b * N;
  float ms = 0.f;
  for (int i = threadIdx.x; i < N; i += blockDim.x) ms += m[i];
  ms = wave_sum(ms);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = ms;
  __syncthreads();
  ms = red[0] + red[1] + red[2] + red[3];
  const long ap = anom_pos != nullptr ? anom_pos[b] : -1;
  for (int i = threadIdx.x; i < N; i += blockDim.x) {
    float p;
    if (pool == 0) p = m[i] / fmaxf(ms, 1.f);
    else if (pool == 1) p = m[i];
    else p = (i == (ap < 0 ? 0 : ap)) ? 1.f : 0.f;
    float c = p;
    if (agg_mean && p != 0.f) {
      float deg = 0.f;
      for (int j = 0; j < N; ++j) deg += A[(long)i * N + j];
      c = p / fmaxf(deg, 1.f);
    }
    coef[i] = c;
  }
  __syncthreads();
  for (int j = threadIdx.x; j < N; j += blockDim.x) {
    float s = 0.f;
    for (int i = 0; i < N; ++i) s += coef[i] * A[(long)i * N + j];
    w[(long)b * N + j] = s;
  }
}

// S: [Cin + Cin^2 + 1] fp64 moments (training) ; out: [4, F] = mu, invstd, scale, shift
__global__ __launch_bounds__(256) void gcn_bn_prep_kernel(const double* __restrict__ S, int Cin, int F,
                                                          const float* __restrict__ W, const float* __restrict__ b,
                                                          const float* __restrict__ gamma,
                                                          const float* __restrict__ beta, float* __restrict__ rmean,
                                                          float* __restrict__ rvar, int training, float momentum,
                                                          float eps, float* __restrict__ out) {
  for (int f = threadIdx.x; f < F; f += blockDim.x) {
    float mu, var;
    if (training) {
      const double cnt = fmax(S[Cin + Cin * Cin], 1.0);
      double ex[GLUE_MAX_CIN];
      for (int k = 0; k < Cin; ++k) ex[k] = S[k] / cnt;
      double m = b[f], v = 0.0;
      for (int k = 0; k < Cin; ++k) {
        const double wk = W[k * F + f];
        m += ex[k] * wk;
        for (int l = 0; l < Cin; ++l) {
          const double cov = S[Cin + k * Cin + l] / cnt - ex[k] * ex[l];
          v += wk * cov * (double)W[l * F + f];
        }
      }
      mu = (float)m;
      var = (float)fmax(v, 0.0);
      rmean[f] = rmean[f] * momentum + mu * (1.f - momentum);
      rvar[f] = rvar[f] * momentum + var * (1.f - momentum);
    } else {
      mu = rmean[f];
      var = rvar[f];
    }
    const float inv = rsqrtf(var + eps);
    const float sc = gamma[f] * inv;
    out[f] = mu;
    out[F + f] = inv;
    out[2 * F + f] = sc;
    out[3 * F + f] = beta[f] - mu * sc;
  }
}

// acc: [3 + Cin, F] = A, Z, P, Q (gcn_pool_bwd partial sums) ; st: [4, F] from gcn_bn_prep.
// Adds into dW [Cin,F], db, dgamma, dbeta, dalpha [F] (nullptr = not needed); coef: [3, F].
__global__ __launch_bounds__(256) void gcn_bwd_finalize_kernel(
    const float* __restrict__ acc, const double* __restrict__ S, int Cin, int F, const float* __restrict__ W,
    const float* __restrict__ b, const float* __restrict__ st, int training, float* __restrict__ dW,
    float* __restrict__ db, float* __restrict__ dgamma, float* __restrict__ dbeta, float* __restrict__ dalpha,
    float* __restrict__ coef) {
  for (int f = threadIdx.x; f < F; f += blockDim.x) {
    const float mu = st[f], inv = st[F + f], sc = st[2 * F + f];
    float c0 = 0.f, c2 = 0.f;
    if (acc != nullptr) {
      const float A = acc[f], Z = acc[F + f], P = acc[2 * F + f];
      const float dg = inv * (Z - mu * A);
      if (dbeta) dbeta[f] += A;
      if (dgamma) dgamma[f] += dg;
      if (dalpha) dalpha[f] += P;
      if (training) {
        const double n = fmax(S[Cin + Cin * Cin], 1.0);
        for (int k = 0; k < Cin; ++k) {
          double s2w = 0.0;
          for (int l = 0; l < Cin; ++l) s2w += S[Cin + k * Cin + l] * (double)W[l * F + f];
          const double s1 = S[k];
          const double sxx = inv * (s2w + s1 * ((double)b[f] - mu));
          const double q = acc[(3 + k) * F + f];
          if (dW) dW[k * F + f] += (float)(sc * (q - s1 * A / n - sxx * dg / n));
        }
        c0 = (float)(sc * (-A / n + mu * inv * dg / n));
        c2 = (float)(-sc * inv * dg / n);
      } else {
        for (int k = 0; k < Cin; ++k)
          if (dW) dW[k * F + f] += sc * acc[(3 + k) * F + f];
        if (db) db[f] += sc * A;
      }
    }
    coef[f] = c0;
    coef[F + f] = sc;
    coef[2 * F + f] = c2;
  }
}

at::Tensor gcn_pool_weights(const at::Tensor& adj, const at::Tensor& mask, const at::Tensor& anom_pos,
                            bool agg_mean, int64_t pool) {
  check_f32_cuda(adj, "adj");
  check_f32_cuda(mask, "mask");
  TORCH_CHECK(adj.dim() == 3 && adj.size(1) == adj.size(2), "adj must be [B,N,N]");
  const int B = (int)adj.size(0), N = (int)adj.size(1);
  TORCH_CHECK(mask.size(0) == B && mask.size(1) == N, "mask must be [B,N]");
  TORCH_CHECK(pool >= 0 && pool <= 2, "pool: 0 mean, 1 sum, 2 selection");
  TORCH_CHECK(N <= 16384, "gcn_pool_weights: too many nodes");
  const int64_t* ap = nullptr;
  if (pool == 2) {
    TORCH_CHECK(anom_pos.is_cuda() && anom_pos.scalar_type() == at::kLong && anom_pos.numel() == B &&
                    anom_pos.is_contiguous(), "anom_pos must be [B] int64");
    ap = anom_pos.data_ptr<int64_t>();
  }
  c10::DeviceGuard guard(adj.device());
  at::Tensor w = at::empty({B, N}, adj.options());
  if (B > 0)
    hipLaunchKernelGGL(gcn_pool_weights_kernel, dim3(B), dim3(256), N * sizeof(float), stream(),
                       adj.data_ptr<float>(), mask.data_ptr<float>(), ap, N, agg_mean ? 1 : 0, (int)pool,
                       w.data_ptr<float>());
  GQ_LAUNCH_CHECK();
  return w;
}

at::Tensor gcn_bn_prep(const at::Tensor& S, const at::Tensor& W, const at::Tensor& b, const at::Tensor& gamma,
                       const at::Tensor& beta, at::Tensor rmean, at::Tensor rvar, bool training, double momentum,
                       double eps) {
  const at::Tensor* ops[] = {&W, &b, &gamma, &beta, &rmean, &rvar};
  for (const at::Tensor* t : ops) check_f32_cuda(*t, "gcn_bn_prep operand");
  const int Cin = (int)W.size(0), F = (int)W.size(1);
  TORCH_CHECK(Cin <= GLUE_MAX_CIN, "gcn_bn_prep: at most 8 input channels");
  const double* sp = nullptr;
  if (training) {
    TORCH_CHECK(S.is_cuda() && S.scalar_type() == at::kDouble && S.numel() == Cin + Cin * Cin + 1,
                "gcn_bn_prep: S must be the fp64 gcn_stats output");
    sp = S.data_ptr<double>();
  }
  c10::DeviceGuard guard(W.device());
  at::Tensor out = at::empty({4, F}, W.options());
  hipLaunchKernelGGL(gcn_bn_prep_kernel, dim3(1), dim3(256), 0, stream(), sp, Cin, F, W.data_ptr<float>(),
                     b.data_ptr<float>(), gamma.data_ptr<float>(), beta.data_ptr<float>(), rmean.data_ptr<float>(),
                     rvar.data_ptr<float>(), training ? 1 : 0, (float)momentum, (float)eps, out.data_ptr<float>());
  GQ_LAUNCH_CHECK();
  return out;
}

static float* opt_ptr(const at::Tensor& t, long n, const char* name) {
  if (t.numel() == 0) return nullptr;
  check_f32_cuda(t, name);
  TORCH_CHECK(t.numel() == n, "gcn_bwd_finalize: ", name, " size");
  return t.data_ptr<float>();
}

at::Tensor gcn_bwd_finalize(const at::Tensor& acc, const at::Tensor& S, const at::Tensor& W, const at::Tensor& b,
                            const at::Tensor& st, bool training, at::Tensor dW, at::Tensor db, at::Tensor dgamma,
                            at::Tensor dbeta, at::Tensor dalpha) {
  check_f32_cuda(W, "W");
  check_f32_cuda(b, "b");
  check_f32_cuda(st, "st");
  const int Cin = (int)W.size(0), F = (int)W.size(1);
  TORCH_CHECK(st.numel() == 4 * F, "gcn_bwd_finalize: st must be [4,F]");
  const float* ap = nullptr;
  if (acc.numel() > 0) {
    check_f32_cuda(acc, "acc");
    TORCH_CHECK(acc.numel() == (long)(3 + Cin) * F, "gcn_bwd_finalize: acc must be [3+Cin,F]");
    ap = acc.data_ptr<float>();
  }
  const double* sp = nullptr;
  if (training) {
    TORCH_CHECK(ap != nullptr, "gcn_bwd_finalize: training mode needs acc");
    TORCH_CHECK(S.is_cuda() && S.scalar_type() == at::kDouble && S.numel() == Cin + Cin * Cin + 1, "S");
    sp = S.data_ptr<double>();
  }
  c10::DeviceGuard guard(W.device());
  at::Tensor coef = at::empty({3, F}, W.options());
  hipLaunchKernelGGL(gcn_bwd_finalize_kernel, dim3(1), dim3(256), 0, stream(), ap, sp, Cin, F, W.data_ptr<float>(),
                     b.data_ptr<float>(), st.data_ptr<float>(), training ? 1 : 0, opt_ptr(dW, (long)Cin * F, "dW"),
                     opt_ptr(db, F, "db"), opt_ptr(dgamma, F, "dgamma"), opt_ptr(dbeta, F, "dbeta"),
                     opt_ptr(dalpha, F, "dalpha"), coef.data_ptr<float>());
  GQ_LAUNCH_CHECK();
  return coef;
}

}  // namespace gq

TORCH_LIBRARY_IMPL(gnnqc, CUDA, m) {
  m.impl("gcn_pool_weights", &gq::gcn_pool_weights);
  m.impl("gcn_bn_prep", &gq::gcn_bn_prep);
  m.impl("gcn_bwd_finalize", &gq::gcn_bwd_finalize);
}
