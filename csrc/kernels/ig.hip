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

// =====================================================================================
// Path-folded GeneralConv + BatchNorm (eval) + PReLU + node pooling for the CML GCN (K10: the
// alpha scaling folded into the input load). The zero-baseline path point s of window b is
// x_s = alpha_s x_b, so its GCN pre-activation is z = alpha_s (x_b W) + bias: x W is computed
// ONCE per (window, step, node) and no kk x B copy of x (ig_interp: 430 MB per CML batch) or of
// the static adjacency / mask tensors exists. Rows of the time-major LSTM input are step-major
// (row = s * B + b), as the explainer's path batch.
//
// forward: out [T][Mp][Cp] = [alpha_s anom_b | sum_n w_bn prelu((alpha_s xW_bn + bias) sc + sh) | 0]
// backward: the input gradients of every path point, trapezoid-weighted and summed over the
// chunk's steps in ONE pass (ig_accum folded in, fixed step order: deterministic):
//   acc_x[b,t,n,k]  += sum_s wt_s sum_f W[k,f] m_n w_bn sc_f prelu'(y) g_f(s)
//   acc_a[b,t,c]    += sum_s wt_s g_c(s)           (g = dL/d out, rows s * B + b)
// The workgroup of (t, 256 / F windows) first stages every step's output-gradient rows of its
// windows (contiguous per step) in LDS, so all those loads are in flight at once.
constexpr int IGG_NMAX = 32;      // nodes per window (lanes of the backward's node axis)
constexpr int IGG_SCH = 32;       // path points staged per LDS pass of the backward

constexpr int IGG_FSG = 8;        // path points per coalesced store pass of the forward

template <int Cin, int F, int NM>                  // NM >= N: node slots (unrolled)
__global__ __launch_bounds__(256) void ig_gcn_pool_fwd_kernel(
    const float* __restrict__ x, const float* __restrict__ w, const float* __restrict__ anom,
    const float* __restrict__ W, const float* __restrict__ bias, const float* __restrict__ scale,
    const float* __restrict__ shift, const float* __restrict__ prelu_a, const float* __restrict__ alphas,
    float* __restrict__ out, int B, int T, int N, int Ca, int kk, int Mp, int Cp) {
  constexpr int BB = 256 / F;                       // windows per workgroup
  extern __shared__ __attribute__((aligned(16))) float so[];   // [IGG_FSG][BB][Cp] output rows
  const int f = threadIdx.x % F, bl = threadIdx.x / F;
  const int t = blockIdx.y, b0 = blockIdx.x * BB, b = b0 + bl;
  const int nb = min(BB, B - b0);
  if (blockIdx.x == 0) {                            // zero the padding rows kk*B .. Mp-1 of step t
    const long z0 = ((long)t * Mp + (long)kk * B) * Cp, z1 = ((long)t + 1) * Mp * Cp;
    for (long e = z0 + threadIdx.x; e < z1; e += 256) out[e] = 0.f;
  }
  const bool live = b < B;
  float wk[Cin];
#pragma unroll
  for (int k = 0; k < Cin; ++k) wk[k] = W[k * F + f];
  const float sc = scale[f], A0 = bias[f] * sc + shift[f], al = prelu_a[f];
  // y_n(s) = alpha_s * xs_n + A0 with xs_n = (x_bn . W_f) sc
  float xs[NM], wn[NM];
  const float* xb = x + ((long)(live ? b : 0) * T + t) * (long)N * Cin;
#pragma unroll
  for (int n = 0; n < NM; ++n) {
    float z = 0.f;
    if (n < N) {
#pragma unroll
      for (int k = 0; k < Cin; ++k) z += xb[n * Cin + k] * wk[k];
    }
    xs[n] = z * sc;
    wn[n] = (live && n < N) ? w[(long)b * N + n] : 0.f;
  }
  const float a_in = (live && f < Ca) ? anom[((long)b * T + t) * Ca + f] : 0.f;
  // Piecewise-linear form over the path (see the backward): prelu(y_n(s)) = c_n(s) y_n(s) with
  // c_n in {1, al} flipping at most once, at j_n, so out(s) = alpha_s S1(s) + A0 S0(s) where
  // S1 = sum_n w_n c_n(s) xs_n and S0 = sum_n w_n c_n(s) change only at the flips: per node one
  // binary search, then a running sum over the steps (O(N log kk + kk) per thread, not O(N kk)).
  const float a_first = alphas[0], a_last = alphas[kk - 1];
  float S1 = 0.f, S0 = 0.f;
  int jn[NM];
  float d1[NM], d0[NM];
#pragma unroll
  for (int n = 0; n < NM; ++n) {
    const bool p0 = a_first * xs[n] + A0 > 0.f, p1 = a_last * xs[n] + A0 > 0.f;
    const float c0 = p0 ? 1.f : al, c1 = p1 ? 1.f : al;
    S1 += wn[n] * c0 * xs[n];
    S0 += wn[n] * c0;
    int j = kk;                                     // no flip along the path
    if (p0 != p1) {
      int lo = 0, hi = kk - 1;                      // p(lo) == p0, p(hi) != p0
      while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if ((alphas[mid] * xs[n] + A0 > 0.f) == p0) lo = mid;
        else hi = mid;
      }
      j = hi;
    }
    jn[n] = j;
    d1[n] = wn[n] * (c1 - c0) * xs[n];
    d0[n] = wn[n] * (c1 - c0);
  }
  float* D1 = so + IGG_FSG * BB * Cp + threadIdx.x;  // this thread's flip deltas [IGG_FSG][256]
  float* D0 = D1 + IGG_FSG * 256;
  const int rowf = nb * Cp;                         // floats of one step's rows (contiguous)
  for (int s0 = 0; s0 < kk; s0 += IGG_FSG) {
    const int ns = min(IGG_FSG, kk - s0);
#pragma unroll
    for (int q = 0; q < IGG_FSG; ++q) {
      D1[q * 256] = 0.f;
      D0[q * 256] = 0.f;
    }
#pragma unroll
    for (int n = 0; n < NM; ++n) {
      const int r = jn[n] - s0;
      if (r >= 0 && r < IGG_FSG) {
        D1[r * 256] += d1[n];
        D0[r * 256] += d0[n];
      }
    }
    for (int si = 0; si < ns; ++si) {
      const float a = alphas[s0 + si];
      S1 += D1[si * 256];
      S0 += D0[si * 256];
      float* o = so + (si * BB + bl) * Cp;
      o[Ca + f] = a * S1 + A0 * S0;
      if (f < Ca) o[f] = a * a_in;
      for (int c = Ca + F + f; c < Cp; c += F) o[c] = 0.f;
    }
    __syncthreads();
    // coalesced float4 stores of the ns x nb rows (Cp % 4 == 0: every row starts 16-byte aligned)
    const int r4 = rowf / 4;
    for (int e = threadIdx.x; e < ns * r4; e += 256) {
      const int si = e / r4, q = e - si * r4;
      const float4 v = reinterpret_cast<const float4*>(so + si * BB * Cp)[q];
      reinterpret_cast<float4*>(out + ((long)t * Mp + (long)(s0 + si) * B + b0) * Cp)[q] = v;
    }
    __syncthreads();
  }
}

// Backward in closed form over the path. For a node n and channel f, y(s) = alpha_s xw + A0 is
// monotone in s (alphas ascending), so prelu'(y(s)) takes one value c0 before a single flip index j
// and another, c1, after it. With the prefix sums P(j) = sum_{s<j} wt_s g_f(s) (Q = P(kk)):
//   sum_s wt_s prelu'(y(s)) g_f(s) = c0 P(j) + c1 (Q - P(j)),
// j found by a binary search on the same predicate (y > 0, same fma) the forward evaluated. Per
// (window, step) that is kk F prefix adds + N F log2(kk) compares instead of N F kk terms.
constexpr int IGG_KMAX = 128;     // path points per launch (the host splits longer chunks)
constexpr int IGG_BWB = 4;        // windows per backward workgroup (128 threads: lanes = nodes)

template <int Cin, int F>
__global__ __launch_bounds__(IGG_BWB * IGG_NMAX) void ig_gcn_pool_bwd_kernel(
    const float* __restrict__ x, const float* __restrict__ w, const float* __restrict__ mask,
    const float* __restrict__ g, const float* __restrict__ W, const float* __restrict__ bias,
    const float* __restrict__ scale, const float* __restrict__ shift, const float* __restrict__ prelu_a,
    const float* __restrict__ alphas, const float* __restrict__ wts, float* __restrict__ acc_x,
    float* __restrict__ acc_a, int B, int T, int N, int Ca, int kk, int s_off, int Mp, int Cp, int first) {
  constexpr int PC = F + 4;                         // prefix channels: F GCN + 4 anomaly slots
  extern __shared__ __attribute__((aligned(16))) float sP[];   // [IGG_BWB][kk + 1][PC]
  __shared__ float sA[IGG_KMAX];
  const int tid = threadIdx.x;
  const int n = tid % IGG_NMAX, bl = tid / IGG_NMAX;
  const int t = blockIdx.y, b0 = blockIdx.x * IGG_BWB, b = b0 + bl;
  const int rowp = (kk + 1) * PC;
  for (int e = tid; e < kk; e += IGG_BWB * IGG_NMAX) sA[e] = alphas[e];
  // prefix sums over the path points of wt_s g_c(s): thread (window, channel)
  for (int e = tid; e < IGG_BWB * PC; e += IGG_BWB * IGG_NMAX) {
    const int wb = e / PC, c = e - wb * PC, bb = b0 + wb;
    const int ch = c < F ? Ca + c : (c - F < Ca ? c - F : -1);
    float* P = sP + wb * rowp + c;
    float acc = 0.f;
    P[0] = 0.f;
    if (bb < B && ch >= 0) {
      const float* gp = g + ((long)t * Mp + (long)s_off * B + bb) * Cp + ch;
      const long stride = (long)B * Cp;
#pragma unroll 8
      for (int s = 0; s < kk; ++s) {
        acc += wts[s] * gp[s * stride];
        P[(s + 1) * PC] = acc;
      }
    } else {
      for (int s = 0; s < kk; ++s) P[(s + 1) * PC] = 0.f;
    }
  }
  __syncthreads();
  if (b >= B) return;
  const float* P = sP + bl * rowp;
  // (first: this launch writes the accumulators instead of adding - no zero-fill pass before it)
  if (n < Ca) {
    float* oa = acc_a + ((long)b * T + t) * Ca + n;
    *oa = (first ? 0.f : *oa) + P[kk * PC + F + n];
  }
  if (n >= N) return;
  float xv[Cin];
#pragma unroll
  for (int k = 0; k < Cin; ++k) xv[k] = x[(((long)b * T + t) * N + n) * Cin + k];
  const float mw = (mask[(long)b * N + n] != 0.f ? 1.f : 0.f) * w[(long)b * N + n];
  const float a_first = sA[0], a_last = sA[kk - 1];
  float d[Cin];
#pragma unroll
  for (int k = 0; k < Cin; ++k) d[k] = 0.f;
#pragma unroll 4
  for (int f = 0; f < F; ++f) {
    const float sc = scale[f];
    float z = 0.f;
    float wp[Cin];
#pragma unroll
    for (int k = 0; k < Cin; ++k) {
      const float wkf = W[k * F + f];
      z += xv[k] * wkf;
      wp[k] = wkf * sc;
    }
    const float xw = z * sc, A0 = bias[f] * sc + shift[f], al = prelu_a[f];
    const bool p0 = a_first * xw + A0 > 0.f;
    const bool p1 = a_last * xw + A0 > 0.f;
    int lo = 0, hi = kk;                            // p(lo) == p0; first flip in (lo, hi]
    if (p1 != p0) {
      hi = kk - 1;
      while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if ((sA[mid] * xw + A0 > 0.f) == p0) lo = mid;
        else hi = mid;
      }
    }
    const float Pj = P[hi * PC + f], Q = P[kk * PC + f];
    const float H = (p0 ? 1.f : al) * Pj + (p1 ? 1.f : al) * (Q - Pj);
#pragma unroll
    for (int k = 0; k < Cin; ++k) d[k] += wp[k] * H;
  }
  float* o = acc_x + (((long)b * T + t) * N + n) * Cin;
#pragma unroll
  for (int k = 0; k < Cin; ++k) o[k] = (first ? 0.f : o[k]) + mw * d[k];
}

#define GQ_IGG_DISPATCH(CIN_RT, F_RT, ...)                                                         \
  do {                                                                                             \
    if (CIN_RT == 2 && F_RT == 16) { constexpr int CIN = 2, FF = 16; __VA_ARGS__; }                \
    else if (CIN_RT == 1 && F_RT == 16) { constexpr int CIN = 1, FF = 16; __VA_ARGS__; }           \
    else if (CIN_RT == 3 && F_RT == 16) { constexpr int CIN = 3, FF = 16; __VA_ARGS__; }           \
    else if (CIN_RT == 2 && F_RT == 32) { constexpr int CIN = 2, FF = 32; __VA_ARGS__; }           \
    else if (CIN_RT == 2 && F_RT == 8) { constexpr int CIN = 2, FF = 8; __VA_ARGS__; }             \
    else TORCH_CHECK(false, "ig_gcn_pool: unsupported Cin ", CIN_RT, " / F ", F_RT);               \
  } while (0)

bool ig_gcn_shape_ok(int64_t Cin, int64_t F, int64_t N) {
  return N >= 1 && N <= IGG_NMAX &&
         ((Cin == 2 && (F == 8 || F == 16 || F == 32)) || ((Cin == 1 || Cin == 3) && F == 16));
}

// x [B,T,N,Cin], w [B,N] pool weights (gcn_prep), anom [B,T,Ca] (or empty), st rows 2/3 = BN scale /
// shift (eval), alphas [kk]. Returns [T, Mp, Cp] with Mp = kk*B rounded up to 16.
at::Tensor ig_gcn_pool_fwd(const at::Tensor& x, const at::Tensor& w, const at::Tensor& anom, const at::Tensor& W,
                           const at::Tensor& b, const at::Tensor& scale, const at::Tensor& shift,
                           const at::Tensor& alpha, const at::Tensor& alphas, int64_t Cp) {
  for (auto* p : {&x, &w, &W, &b, &scale, &shift, &alpha, &alphas}) check_f32_cuda(*p, "ig_gcn_pool_fwd input");
  TORCH_CHECK(x.dim() == 4, "ig_gcn_pool_fwd: x must be [B,T,N,Cin]");
  const int B = x.size(0), T = x.size(1), N = x.size(2), Cin = x.size(3), F = W.size(1);
  TORCH_CHECK(ig_gcn_shape_ok(Cin, F, N) && W.size(0) == Cin, "ig_gcn_pool_fwd: unsupported shape");
  TORCH_CHECK(w.size(0) == B && w.size(1) == N && b.numel() == F && scale.numel() == F && shift.numel() == F &&
                  alpha.numel() == F, "ig_gcn_pool_fwd: parameter shapes");
  int Ca = 0;
  if (anom.numel() > 0) {
    check_f32_cuda(anom, "anom");
    TORCH_CHECK(anom.dim() == 3 && anom.size(0) == B && anom.size(1) == T, "ig_gcn_pool_fwd: anom must be [B,T,Ca]");
    Ca = anom.size(2);
  }
  TORCH_CHECK(Ca <= F && Cp >= Ca + F && Cp % 4 == 0, "ig_gcn_pool_fwd: Cp / Ca");
  const int kk = (int)alphas.numel();
  TORCH_CHECK(kk >= 1, "ig_gcn_pool_fwd: no path points");
  const long Mp = ((long)kk * B + 15) / 16 * 16;
  c10::DeviceGuard guard(x.device());
  at::Tensor out = at::empty({T, Mp, Cp}, x.options());
#define GQ_IGG_FWD(NMV)                                                                                     \
  hipLaunchKernelGGL((ig_gcn_pool_fwd_kernel<CIN, FF, NMV>), dim3((B + 256 / FF - 1) / (256 / FF), T), dim3(256), \
                     ((size_t)IGG_FSG * (256 / FF) * Cp + 2 * IGG_FSG * 256) * sizeof(float), stream(),           \
                     x.data_ptr<float>(),                                                                           \
                     w.data_ptr<float>(), Ca ? anom.data_ptr<float>() : nullptr, W.data_ptr<float>(),               \
                     b.data_ptr<float>(), scale.data_ptr<float>(), shift.data_ptr<float>(), alpha.data_ptr<float>(), \
                     alphas.data_ptr<float>(), out.data_ptr<float>(), B, T, N, Ca, kk, (int)Mp, (int)Cp)
  GQ_IGG_DISPATCH(Cin, F,
      if (N <= 8) GQ_IGG_FWD(8); else if (N <= 16) GQ_IGG_FWD(16); else if (N <= 24) GQ_IGG_FWD(24);
      else GQ_IGG_FWD(32));
#undef GQ_IGG_FWD
  GQ_LAUNCH_CHECK();
  return out;
}

// g = dL/d out [T, Mp, Cp] of ig_gcn_pool_fwd; accumulates into acc_x [B,T,N,Cin] and acc_a [B,T,Ca]
// (overwrite: the first launch writes them - uninitialised accumulators need no zero fill).
void ig_gcn_pool_bwd(const at::Tensor& x, const at::Tensor& w, const at::Tensor& mask, const at::Tensor& g,
                     const at::Tensor& W, const at::Tensor& b, const at::Tensor& scale, const at::Tensor& shift,
                     const at::Tensor& alpha, const at::Tensor& alphas, const at::Tensor& wts, at::Tensor acc_x,
                     at::Tensor acc_a, bool overwrite) {
  for (auto* p : {&x, &w, &mask, &g, &W, &b, &scale, &shift, &alpha, &alphas, &wts})
    check_f32_cuda(*p, "ig_gcn_pool_bwd input");
  check_f32_cuda(acc_x, "ig_gcn_pool_bwd acc_x");
  const int B = x.size(0), T = x.size(1), N = x.size(2), Cin = x.size(3), F = W.size(1);
  TORCH_CHECK(ig_gcn_shape_ok(Cin, F, N), "ig_gcn_pool_bwd: unsupported shape");
  const int kk = (int)alphas.numel();
  TORCH_CHECK(wts.numel() == kk && kk >= 1, "ig_gcn_pool_bwd: weights per path point");
  TORCH_CHECK(acc_x.sizes() == x.sizes() && mask.numel() == (long)B * N && w.numel() == (long)B * N,
              "ig_gcn_pool_bwd: accumulator / mask shapes");
  TORCH_CHECK(g.dim() == 3 && g.size(0) == T && g.size(1) >= (long)kk * B, "ig_gcn_pool_bwd: g must be [T, Mp, Cp]");
  const int Cp = g.size(2);
  int Ca = 0;
  if (acc_a.numel() > 0) {
    check_f32_cuda(acc_a, "acc_a");
    TORCH_CHECK(acc_a.dim() == 3 && acc_a.size(0) == B && acc_a.size(1) == T, "ig_gcn_pool_bwd: acc_a [B,T,Ca]");
    Ca = acc_a.size(2);
  }
  TORCH_CHECK(Cp >= Ca + F && Ca <= 4, "ig_gcn_pool_bwd: Cp / Ca");
  c10::DeviceGuard guard(x.device());
  // path points in slices of at most IGG_KMAX (the prefix table of a workgroup lives in LDS)
  for (int s0 = 0; s0 < kk; s0 += IGG_KMAX) {
    const int ks = std::min(IGG_KMAX, kk - s0);
    const size_t smem = (size_t)IGG_BWB * (ks + 1) * (F + 4) * sizeof(float);
    GQ_IGG_DISPATCH(Cin, F,
        hipLaunchKernelGGL((ig_gcn_pool_bwd_kernel<CIN, FF>), dim3((B + IGG_BWB - 1) / IGG_BWB, T),
                           dim3(IGG_BWB * IGG_NMAX), smem, stream(), x.data_ptr<float>(), w.data_ptr<float>(),
                           mask.data_ptr<float>(), g.data_ptr<float>(), W.data_ptr<float>(), b.data_ptr<float>(),
                           scale.data_ptr<float>(), shift.data_ptr<float>(), alpha.data_ptr<float>(),
                           alphas.data_ptr<float>() + s0, wts.data_ptr<float>() + s0, acc_x.data_ptr<float>(),
                           Ca ? acc_a.data_ptr<float>() : nullptr, B, T, N, Ca, ks, s0, (int)g.size(1), Cp,
                           (overwrite && s0 == 0) ? 1 : 0));
    GQ_LAUNCH_CHECK();
  }
}
#undef GQ_IGG_DISPATCH

}  // namespace gq

TORCH_LIBRARY_IMPL(gnnqc, CUDA, m) {
  m.impl("ig_gcn_pool_fwd", &gq::ig_gcn_pool_fwd);
  m.impl("ig_gcn_pool_bwd", &gq::ig_gcn_pool_bwd);
  m.impl("ig_interp", &gq::ig_interp);
  m.impl("ig_accum", &gq::ig_accum);
  m.impl("ig_finalize", &gq::ig_finalize);
}
