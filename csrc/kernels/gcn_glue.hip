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
//  gcn_bwd_finalize  the column sums of the backward pass's per-block partials, then dW, db,
//                    dgamma, dbeta, dalpha accumulated straight into the gradient buffers
//                    + the dx coefficients                           (one block per channel)
//  gcn_prep          pool weights + x moments + BN prep of a training step in ONE launch
//
// Semantics: spektral GeneralConv + Keras BatchNormalization (momentum .99, eps 1e-3,
// biased batch variance), libs/create_model.py:184-189, :8-41.
#include "common.h"

namespace gq {

constexpr int GLUE_MAX_CIN = 8;
constexpr int GLUE_NSTAT_MAX = GLUE_MAX_CIN + GLUE_MAX_CIN * GLUE_MAX_CIN + 1;

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

// acc: [R][3 + Cin][F] per-block partial sums A, Z, P, Q of gcn_pool_bwd / gcn_node_bwd (R = 1:
// already reduced); st: [4, F] from the BN prep. Workgroup f sums column (j, f) over the R rows
// (fixed order: deterministic) and adds dW[:, f], db, dgamma, dbeta, dalpha (nullptr = not
// needed) into the gradient buffers; coef: [3, F]. (Replaces a separate column-sum launch.)
// First stage of the finalize for many partial rows (SoilNet's node backward: one row per
// (window, 2-step chunk) workgroup, 5,408 rows): workgroup p sums rows [p*chunk, (p+1)*chunk) of
// acc [R][ncol] for every column in a fixed order (coalesced rows; 256/ncol row lanes per column,
// combined in order), out [P][ncol]. The finalize then sums P rows instead of R (a workgroup per
// column striding 384 B between its R loads took 49 us).
__global__ __launch_bounds__(256) void gcn_acc_colsum_kernel(const float* __restrict__ acc, int R, int ncol,
                                                             int chunk, float* __restrict__ out) {
  __shared__ float part[256];
  const int p = blockIdx.x, tid = threadIdx.x;
  const int r0 = p * chunk, r1 = min(R, r0 + chunk);
  if (ncol <= 128) {
    const int nsub = 256 / ncol, c = tid % ncol, rs = tid / ncol;
    float a0 = 0.f, a1 = 0.f;
    if (rs < nsub) {
      int r = r0 + rs;
      for (; r + nsub < r1; r += 2 * nsub) {          // two independent loads in flight
        a0 += acc[(long)r * ncol + c];
        a1 += acc[(long)(r + nsub) * ncol + c];
      }
      if (r < r1) a0 += acc[(long)r * ncol + c];
    }
    part[tid] = a0 + a1;
    __syncthreads();
    if (tid < ncol) {
      float t = 0.f;
      for (int q = 0; q < nsub; ++q) t += part[q * ncol + tid];
      out[(long)p * ncol + tid] = t;
    }
  } else {
    for (int c = tid; c < ncol; c += 256) {
      float t = 0.f;
      for (int r = r0; r < r1; ++r) t += acc[(long)r * ncol + c];
      out[(long)p * ncol + c] = t;
    }
  }
}

__global__ __launch_bounds__(256) void gcn_bwd_finalize_kernel(
    const float* __restrict__ acc, int R, const double* __restrict__ S, int Cin, int F, const float* __restrict__ W,
    const float* __restrict__ b, const float* __restrict__ st, int training, float* __restrict__ dW,
    float* __restrict__ db, float* __restrict__ dgamma, float* __restrict__ dbeta, float* __restrict__ dalpha,
    float* __restrict__ coef) {
  const int f = blockIdx.x;
  const int nacc = 3 + Cin;
  __shared__ float red[4][GLUE_MAX_CIN + 3];
  __shared__ float tot[GLUE_MAX_CIN + 3];
  // the closed-form epilogue's operands, fetched up front so their loads overlap the reduction's
  // (thread 0 loading them after it was a chain of dependent memory round trips)
  __shared__ double sS[GLUE_NSTAT_MAX];
  __shared__ float sWf[GLUE_MAX_CIN], sst[3], sb;
  {
    const int t = threadIdx.x;
    const int nstat = Cin + Cin * Cin + 1;
    if (training && acc != nullptr && t < nstat) sS[t] = S[t];
    if (t >= 96 && t < 96 + Cin) sWf[t - 96] = W[(t - 96) * F + f];
    if (t >= 128 && t < 131) sst[t - 128] = st[(t - 128) * F + f];
    if (t == 192) sb = b[f];
  }
  if (acc != nullptr) {
    float a[GLUE_MAX_CIN + 3];
#pragma unroll
    for (int j = 0; j < GLUE_MAX_CIN + 3; ++j) a[j] = 0.f;
    for (int r = threadIdx.x; r < R; r += 256) {
#pragma unroll
      for (int j = 0; j < GLUE_MAX_CIN + 3; ++j)
        if (j < nacc) a[j] += acc[((long)r * nacc + j) * F + f];
    }
    // fixed-shape reduction: wave shuffles, then the 4 wave partials in order (deterministic)
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
    for (int j = 0; j < GLUE_MAX_CIN + 3; ++j) {
      float v = a[j];
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
      if (lane == 0) red[wv][j] = v;
    }
    __syncthreads();
    if ((int)threadIdx.x < nacc)
      tot[threadIdx.x] = (red[0][threadIdx.x] + red[1][threadIdx.x]) + (red[2][threadIdx.x] + red[3][threadIdx.x]);
    __syncthreads();
  }
  __syncthreads();
  if (threadIdx.x != 0) return;
  const float mu = sst[0], inv = sst[1], sc = sst[2];
  float c0 = 0.f, c2 = 0.f;
  if (acc != nullptr) {
    const float A = tot[0], Z = tot[1], P = tot[2];
    const float dg = inv * (Z - mu * A);
    if (dbeta) dbeta[f] += A;
    if (dgamma) dgamma[f] += dg;
    if (dalpha) dalpha[f] += P;
    if (training) {
      const double n = fmax(sS[Cin + Cin * Cin], 1.0);
      for (int k = 0; k < Cin; ++k) {
        double s2w = 0.0;
        for (int l = 0; l < Cin; ++l) s2w += sS[Cin + k * Cin + l] * (double)sWf[l];
        const double s1 = sS[k];
        const double sxx = inv * (s2w + s1 * ((double)sb - mu));
        const double q = tot[3 + k];
        if (dW) dW[k * F + f] += (float)(sc * (q - s1 * A / n - sxx * dg / n));
      }
      c0 = (float)(sc * (-A / n + mu * inv * dg / n));
      c2 = (float)(-sc * inv * dg / n);
    } else {
      for (int k = 0; k < Cin; ++k)
        if (dW) dW[k * F + f] += sc * tot[3 + k];
      if (db) db[f] += sc * A;
    }
  }
  coef[f] = c0;
  coef[F + f] = sc;
  coef[2 * F + f] = c2;
}

// ---- forward prep in ONE launch (was: a zero-fill, gcn_stats, gcn_bn_prep, gcn_pool_weights).
// Workgroup b: the pooling weights of sample b and (training) its fp64 x moments, stored as a
// record with sc1 stores; the workgroup whose arrival-counter add comes last sums the records in
// sample order (deterministic) and runs the BN prep (batch statistics, Keras running-stat
// update, scale / shift). Eval: workgroup 0 preps BN from the running statistics.
constexpr int GLUE_ADJ_LDS = 8192;      // adjacency floats staged in LDS (32 KiB)

__device__ __forceinline__ void glue_bn(const double* S, int Cin, int F, const float* __restrict__ W,
                                        const float* __restrict__ b, const float* __restrict__ gamma,
                                        const float* __restrict__ beta, float* __restrict__ rmean,
                                        float* __restrict__ rvar, int training, float momentum, float eps,
                                        float* __restrict__ out) {
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

template <int Cin>
__global__ __launch_bounds__(256) void gcn_prep_kernel(
    const float* __restrict__ x, const float* __restrict__ adj, const float* __restrict__ mask,
    const int64_t* __restrict__ anom_pos, int B, int T, int N, int agg_mean, int pool, float* __restrict__ w,
    double* __restrict__ part, double* __restrict__ Sout, int* __restrict__ ticket, int training, int F,
    const float* __restrict__ W, const float* __restrict__ bias, const float* __restrict__ gamma,
    const float* __restrict__ beta, float* __restrict__ rmean, float* __restrict__ rvar, float momentum, float eps,
    float* __restrict__ st) {
  constexpr int nstat = Cin + Cin * Cin + 1;
  extern __shared__ float coef[];       // [N], then (small graphs) the sample's [N, N] adjacency
  __shared__ float red[4];
  __shared__ double dred[4][nstat];
  __shared__ double Ssh[nstat];
  __shared__ int last;
  const int b = blockIdx.x;
  const float* A = adj + (long)b * N * N;
  const float* m = mask + (long)b * N;
  if (N * N <= GLUE_ADJ_LDS) {          // one coalesced pass: the loops below then read LDS
    float* sA = coef + N;
    for (int i = threadIdx.x; i < N * N; i += blockDim.x) sA[i] = A[i];
    A = sA;
  }
  {
    float* sM = coef + N + (N * N <= GLUE_ADJ_LDS ? N * N : 0);
    for (int i = threadIdx.x; i < N; i += blockDim.x) sM[i] = m[i];
  }
  // pooling weights w[b, j] = sum_i p_i / deg_i * A[i, j]
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
  if (!training) {
    if (b == 0) glue_bn(nullptr, Cin, F, W, bias, gamma, beta, rmean, rvar, 0, momentum, eps, st);
    return;
  }
  // this sample's moments over its T x N node rows (fp64), 4 rows per thread per round with all
  // their loads issued first (a load-then-branch loop made every row a serial memory round trip);
  // masked rows contribute zeros
  double acc[nstat];
#pragma unroll
  for (int i = 0; i < nstat; ++i) acc[i] = 0.0;
  const float* xb = x + (long)b * T * N * Cin;
  const int R = T * N;
  const float* sM = coef + N + (N * N <= GLUE_ADJ_LDS ? N * N : 0);   // the sample's mask (LDS)
  for (int r0 = threadIdx.x; r0 < R; r0 += 4 * blockDim.x) {
    float xv[4][Cin], mv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int r = r0 + u * (int)blockDim.x;
      const int rc = r < R ? r : 0;
#pragma unroll
      for (int k = 0; k < Cin; ++k) xv[u][k] = xb[(long)rc * Cin + k];
      mv[u] = r < R ? sM[rc % N] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
#pragma unroll
      for (int k = 0; k < Cin; ++k) {
        const float mx = mv[u] * xv[u][k];
        acc[k] += mx;
#pragma unroll
        for (int l = 0; l < Cin; ++l) acc[Cin + k * Cin + l] += (double)mx * xv[u][l];
      }
      acc[nstat - 1] += mv[u];
    }
  }
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < nstat; ++i) {
    double v = acc[i];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if (lane == 0) dred[wv][i] = v;
  }
  __syncthreads();
  // record -> sc1 stores; every storing wave's vmcnt(0); barrier; one lane's counter add
  if ((int)threadIdx.x < nstat) {
    const double v = (dred[0][threadIdx.x] + dred[1][threadIdx.x]) + (dred[2][threadIdx.x] + dred[3][threadIdx.x]);
    __hip_atomic_store(reinterpret_cast<unsigned long long*>(part) + (long)b * nstat + threadIdx.x,
                       (unsigned long long)__double_as_longlong(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) last = __hip_atomic_fetch_add(ticket, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == B - 1;
  __syncthreads();
  if (!last) return;
  // the last arrival: every record (sc1 loads; thread k takes records k, k + 256, ... so all
  // loads are in flight at once - a per-statistic loop over the B records was B serial memory
  // round trips), then a fixed-shape tree over the 256 thread partials (deterministic)
  double v[nstat];
#pragma unroll
  for (int i = 0; i < nstat; ++i) v[i] = 0.0;
  for (int k = threadIdx.x; k < B; k += blockDim.x) {
#pragma unroll
    for (int i = 0; i < nstat; ++i)
      v[i] += __longlong_as_double((long long)__hip_atomic_load(
          reinterpret_cast<const unsigned long long*>(part) + (long)k * nstat + i, __ATOMIC_RELAXED,
          __HIP_MEMORY_SCOPE_AGENT));
  }
#pragma unroll
  for (int i = 0; i < nstat; ++i) {
    double s = v[i];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    if (lane == 0) dred[wv][i] = s;
  }
  __syncthreads();
  if ((int)threadIdx.x < nstat) {
    const double s = (dred[0][threadIdx.x] + dred[1][threadIdx.x]) + (dred[2][threadIdx.x] + dred[3][threadIdx.x]);
    Ssh[threadIdx.x] = s;
    Sout[threadIdx.x] = s;
  }
  __syncthreads();
  glue_bn(Ssh, Cin, F, W, bias, gamma, beta, rmean, rvar, 1, momentum, eps, st);
  if (threadIdx.x == 0) __hip_atomic_store(ticket, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

static int* glue_ticket(int dev) {
  static int* t[64] = {nullptr};
  TORCH_CHECK(dev >= 0 && dev < 64, "gcn_prep: device index");
  if (!t[dev]) {
    hipStreamCaptureStatus cs;
    TORCH_CHECK(hipStreamIsCapturing(stream(), &cs) == hipSuccess && cs == hipStreamCaptureStatusNone,
                "gcn_prep: first use must not be inside a graph capture");
    TORCH_CHECK(hipMalloc(&t[dev], 4 * sizeof(int)) == hipSuccess, "gcn_prep: counter allocation");
    TORCH_CHECK(hipMemset(t[dev], 0, 4 * sizeof(int)) == hipSuccess, "gcn_prep: counter init");
  }
  return t[dev];
}

#define GQ_GLUE_CIN_DISPATCH(CIN_RT, ...)                       \
  switch (CIN_RT) {                                             \
    case 1: { constexpr int CIN = 1; __VA_ARGS__; } break;      \
    case 2: { constexpr int CIN = 2; __VA_ARGS__; } break;      \
    case 3: { constexpr int CIN = 3; __VA_ARGS__; } break;      \
    case 4: { constexpr int CIN = 4; __VA_ARGS__; } break;      \
    default: TORCH_CHECK(false, "gcn_prep: 1..4 input channels"); \
  }

// x [B,T,N,Cin], adj [B,N,N], mask [B,N]; returns [w [B,N], S [nstat] fp64 (training), st [4,F]].
std::vector<at::Tensor> gcn_prep(const at::Tensor& x, const at::Tensor& adj, const at::Tensor& mask,
                                 const at::Tensor& anom_pos, bool agg_mean, int64_t pool, const at::Tensor& W,
                                 const at::Tensor& b, const at::Tensor& gamma, const at::Tensor& beta,
                                 at::Tensor rmean, at::Tensor rvar, bool training, double momentum, double eps) {
  check_f32_cuda(x, "x");
  check_f32_cuda(adj, "adj");
  check_f32_cuda(mask, "mask");
  for (const at::Tensor* t : {&W, &b, &gamma, &beta, (const at::Tensor*)&rmean, (const at::Tensor*)&rvar})
    check_f32_cuda(*t, "gcn_prep operand");
  TORCH_CHECK(x.dim() == 4 && adj.dim() == 3, "gcn_prep: x [B,T,N,Cin], adj [B,N,N]");
  const int B = (int)x.size(0), T = (int)x.size(1), N = (int)x.size(2), Cin = (int)x.size(3), F = (int)W.size(1);
  TORCH_CHECK(adj.size(0) == B && adj.size(1) == N && adj.size(2) == N && mask.size(0) == B && mask.size(1) == N,
              "gcn_prep: adj / mask shapes");
  TORCH_CHECK(W.size(0) == Cin && Cin >= 1 && Cin <= 4, "gcn_prep: W must be [Cin<=4, F]");
  TORCH_CHECK(pool >= 0 && pool <= 2 && N <= 8192 && B >= 1, "gcn_prep: pool / sizes");
  const int64_t* ap = nullptr;
  if (pool == 2) {
    TORCH_CHECK(anom_pos.is_cuda() && anom_pos.scalar_type() == at::kLong && anom_pos.numel() == B &&
                    anom_pos.is_contiguous(), "anom_pos must be [B] int64");
    ap = anom_pos.data_ptr<int64_t>();
  }
  c10::DeviceGuard guard(x.device());
  const int nstat = Cin + Cin * Cin + 1;
  at::Tensor w = at::empty({B, N}, x.options());
  at::Tensor S = training ? at::empty({nstat}, x.options().dtype(at::kDouble)) : at::empty({0}, x.options().dtype(at::kDouble));
  at::Tensor part = training ? at::empty({(long)B * nstat}, x.options().dtype(at::kDouble)) : S;
  at::Tensor st = at::empty({4, F}, x.options());
  int* tk = glue_ticket(x.get_device());
  const size_t smem = (2 * N + (N * N <= GLUE_ADJ_LDS ? N * N : 0)) * sizeof(float);
  GQ_GLUE_CIN_DISPATCH(Cin, hipLaunchKernelGGL(gcn_prep_kernel<CIN>, dim3(B), dim3(256), smem, stream(),
      x.data_ptr<float>(), adj.data_ptr<float>(), mask.data_ptr<float>(), ap, B, T, N, agg_mean ? 1 : 0, (int)pool,
      w.data_ptr<float>(), training ? part.data_ptr<double>() : nullptr, training ? S.data_ptr<double>() : nullptr,
      tk, training ? 1 : 0, F, W.data_ptr<float>(), b.data_ptr<float>(), gamma.data_ptr<float>(),
      beta.data_ptr<float>(), rmean.data_ptr<float>(), rvar.data_ptr<float>(), (float)momentum, (float)eps,
      st.data_ptr<float>()));
  GQ_LAUNCH_CHECK();
  return {w, S, st};
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
  int R = 0;
  if (acc.numel() > 0) {
    check_f32_cuda(acc, "acc");
    TORCH_CHECK(acc.numel() % ((long)(3 + Cin) * F) == 0, "gcn_bwd_finalize: acc must be [R,3+Cin,F]");
    R = (int)(acc.numel() / ((long)(3 + Cin) * F));
    ap = acc.data_ptr<float>();
  }
  at::Tensor pre;
  if (R > 256) {        // two-stage fixed-order sum (still deterministic)
    const int ncol = (3 + Cin) * F;
    const int P = std::min(256, (R + 15) / 16), chunk = (R + P - 1) / P;
    const int Pn = (R + chunk - 1) / chunk;
    pre = at::empty({(long)Pn, ncol}, W.options());
    c10::DeviceGuard g0(W.device());
    hipLaunchKernelGGL(gcn_acc_colsum_kernel, dim3(Pn), dim3(256), 0, stream(), ap, R, ncol, chunk,
                       pre.data_ptr<float>());
    GQ_LAUNCH_CHECK();
    ap = pre.data_ptr<float>();
    R = Pn;
  }
  const double* sp = nullptr;
  if (training) {
    TORCH_CHECK(ap != nullptr, "gcn_bwd_finalize: training mode needs acc");
    TORCH_CHECK(S.is_cuda() && S.scalar_type() == at::kDouble && S.numel() == Cin + Cin * Cin + 1, "S");
    sp = S.data_ptr<double>();
  }
  c10::DeviceGuard guard(W.device());
  at::Tensor coef = at::empty({3, F}, W.options());
  hipLaunchKernelGGL(gcn_bwd_finalize_kernel, dim3(F), dim3(256), 0, stream(), ap, R, sp, Cin, F, W.data_ptr<float>(),
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
  m.impl("gcn_prep", &gq::gcn_prep);
}
