// Temporal Conv1D + LeakyReLU (+ GlobalAveragePooling1D) for the CNN TimeLayer branch
// (reference create_model.py:80-101 - Keras Conv1D(padding='same'),
// LeakyReLU(alpha), GlobalAveragePooling1D after the last conv).
//
// Forward  z[m,t,o] = b[o] + sum_{tap,i} x[m, t+tap-left, i] W[tap,i,o]   (zero outside [0,T))
//          y = leaky(z) ; optionally g[m,o] = mean_t y[m,t,o]
// as an implicit GEMM on v_mfma_f32_16x16x32_bf16: rows = (m,t), K = tap*Cin + i, N = o.
//   * persistent grid; W^T [Cout][K] staged ONCE per workgroup into LDS (bf16);
//   * per 64-row tile the im2col A tile [64][K] is gathered straight into LDS with
//     branch-free clamped loads (no vmcnt drains, see lstm.hip), wave w owns rows 16w..;
//   * epilogue: bias + LeakyReLU + store, and the GAP as one atomic per (lane, sequence).
// Backward reuses the same kernel for dx = conv_same(dz, flip(W)) with mirrored padding,
// where the A loads form dz = dy * leaky'(y) on the fly (and broadcast dg/T for the GAP),
// plus conv1d_wgrad_kernel: dW^T/db over 32-row tiles (db = a ones row of the im2col).
#include "common.h"

namespace gq {

constexpr int CV_RT = 64;   // forward rows per tile (4 waves x 16)
constexpr int CV_PAD = 8;   // LDS row padding (bf16) against bank conflicts

struct ConvArgs {
  const float* a;      // A source: x [rows][lda] or (bcast) [M][lda]
  const float* gate;   // leaky' gate source [rows][Cin_a] (y of the layer; = a with slope 1 when unused)
  const float* W;      // [k][Cin_a][Cout]
  const float* bias;   // [Cout] or null
  float* y;            // [rows][Cout] or null
  float* g;            // [M][Cout] GAP accumulator (pre-zeroed) or null
  long rows;
  int T, Cin, Cout, k, left, lda, Kp;
  int KCH;             // K chunk staged per pass (multiple of 32; = Kp keeps W^T resident)
  float alpha;         // output activation slope (1 = identity)
  float gate_alpha;    // slope of the gating leaky'
  float a_scale;       // multiplier of A (1/T for the GAP backward)
  int bcast;           // A rows indexed by sequence only (GAP backward)
  float inv_T;
};

template <int NT>      // NT = ceil(Cout / 16) output tiles
__global__ __launch_bounds__(256) void conv1d_fwd_kernel(ConvArgs p) {
  extern __shared__ __attribute__((aligned(16))) __bf16 smem[];
  const int Kp = p.Kp, KCH = p.KCH, LD = KCH + CV_PAD;
  __bf16* Wt = smem;                          // [NT*16][LD]   W^T chunk
  __bf16* As = smem + NT * 16 * LD;           // [CV_RT][LD]   im2col chunk
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int col = lane & 15, quad = lane >> 4;
  const int KC = p.k * p.Cin;
  const int nch = (Kp + KCH - 1) / KCH;       // kernel-uniform

  float bias[NT];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    const int n = 16 * nt + col;
    bias[nt] = p.bias != nullptr ? p.bias[min(n, p.Cout - 1)] : 0.f;
  }

  const long ntiles = (p.rows + CV_RT - 1) / CV_RT;
  bool w_staged = false;
  for (long tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const long r0 = tile * CV_RT;
    f32x4_t acc[NT];
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) acc[nt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    for (int ch = 0; ch < nch; ++ch) {
      const int k0 = ch * KCH;
      __syncthreads();   // previous chunk / tile reads of As (and Wt) are done
      if (!w_staged) {   // W^T chunk: Wt[n][kk - k0] = W[tap][i][n]  (zero padded); once if resident
        for (int e = tid; e < NT * 16 * KCH; e += 256) {
          const int n = e / KCH, kk = k0 + e % KCH;
          const float m_ = (n < p.Cout && kk < KC) ? 1.f : 0.f;
          const float v = p.W[(size_t)min(kk, KC - 1) * p.Cout + min(n, p.Cout - 1)];
          Wt[n * LD + (kk - k0)] = (__bf16)(v * m_);
        }
        w_staged = nch == 1;
      }
      // ---- im2col A chunk [64][KCH]
      for (int e = tid; e < CV_RT * KCH; e += 256) {
        const int rr = e / KCH, kk = k0 + e % KCH;
        const long r = r0 + rr;
        const long rc = min(r, p.rows - 1);
        const long m = rc / p.T;
        const int t = (int)(rc - m * p.T);
        const int tap = kk / p.Cin, i = kk - tap * p.Cin;
        const int ts = t + tap - p.left;
        const bool ok = r < p.rows && kk < KC && ts >= 0 && ts < p.T;
        const int tsc = min(max(ts, 0), p.T - 1);
        const int ic = min(i, p.Cin - 1);
        const long src = p.bcast ? m : m * p.T + tsc;
        // unconditional loads (the forward passes gate = x with slope 1): no branch around VMEM
        const float v = p.a[(size_t)src * p.lda + ic];
        const float gy = p.gate[(size_t)(m * p.T + tsc) * p.Cin + ic];
        As[rr * LD + (kk - k0)] = (__bf16)(ok ? v * (gy > 0.f ? 1.f : p.gate_alpha) * p.a_scale : 0.f);
      }
      __syncthreads();
      const int kw = min(KCH, Kp - k0);
      for (int ks = 0; ks < kw; ks += 32) {
        const bf16x8_t a = *reinterpret_cast<const bf16x8_t*>(&As[(16 * w + col) * LD + ks + 8 * quad]);
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
          const bf16x8_t b = *reinterpret_cast<const bf16x8_t*>(&Wt[(16 * nt + col) * LD + ks + 8 * quad]);
          acc[nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc[nt], 0, 0, 0);
        }
      }
    }
    // ---- epilogue: lane holds rows 16w + 4quad + q of column 16nt + col
    const long rb = r0 + 16 * w + 4 * quad;
    const long m_first = min(rb, p.rows - 1) / p.T, m_last = min(rb + 3, p.rows - 1) / p.T;
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      const int n = 16 * nt + col;
      float gs = 0.f;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const long r = rb + q;
        const float z = acc[nt][q] + bias[nt];
        const float yv = z > 0.f ? z : p.alpha * z;
        if (r < p.rows && n < p.Cout) {
          if (p.y != nullptr) p.y[(size_t)r * p.Cout + n] = yv;
          if (p.g != nullptr && m_first != m_last) atomicAdd(&p.g[(size_t)(r / p.T) * p.Cout + n], yv * p.inv_T);
        }
        gs += (r < p.rows) ? yv : 0.f;
      }
      if (p.g != nullptr && m_first == m_last && rb < p.rows && n < p.Cout)
        atomicAdd(&p.g[(size_t)m_first * p.Cout + n], gs * p.inv_T);
    }
  }
}

// dW^T[o][tap*Cin+i] (+ db[o] as column KC) over 32-row tiles; grid = (Cout blocks of 64) x splits.
// dz[r][o] = dy * leaky'(y)   (dy = dg[m][o] / T with gap)
constexpr int CW_RT = 32;
constexpr int CW_LD = CW_RT + 8;

template <int DT>      // DT = ceil((k*Cin + 1) / 16) im2col column tiles (incl. the ones row)
__global__ __launch_bounds__(256) void conv1d_wgrad_kernel(const float* __restrict__ dy, const float* __restrict__ y,
                                                            const float* __restrict__ x, float* __restrict__ dW,
                                                            float* __restrict__ db, long rows, int T, int Cin,
                                                            int Cout, int k, int left, float alpha, int gap) {
  __shared__ __attribute__((aligned(16))) __bf16 dzT[64][CW_LD];
  __shared__ __attribute__((aligned(16))) __bf16 xT[DT * 16][CW_LD];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int col = lane & 15, quad = lane >> 4;
  const int o0 = blockIdx.x * 64;
  const int KC = k * Cin;
  const long ntiles = (rows + CW_RT - 1) / CW_RT;
  const float inv_T = 1.f / (float)T;
  f32x4_t acc[DT];
#pragma unroll
  for (int d = 0; d < DT; ++d) acc[d] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  for (long tile = blockIdx.y; tile < ntiles; tile += gridDim.y) {
    const long r0 = tile * CW_RT;
    for (int e = tid; e < CW_RT * 64; e += 256) {
      const int rr = e / 64, oo = e % 64;
      const long r = r0 + rr;
      const long rc = min(r, rows - 1);
      const int o = min(o0 + oo, Cout - 1);
      const float gy = y[(size_t)rc * Cout + o];
      const float d = dy[(size_t)(gap ? rc / T : rc) * Cout + o] * (gap ? inv_T : 1.f);
      const bool ok = r < rows && o0 + oo < Cout;
      dzT[oo][rr] = (__bf16)(ok ? d * (gy > 0.f ? 1.f : alpha) : 0.f);
    }
    for (int e = tid; e < CW_RT * DT * 16; e += 256) {
      const int rr = e / (DT * 16), kk = e % (DT * 16);
      const long r = r0 + rr;
      const long rc = min(r, rows - 1);
      const long m = rc / T;
      const int t = (int)(rc - m * T);
      const int tap = kk / Cin, i = kk - tap * Cin;
      const int ts = t + tap - left;
      const int tsc = min(max(ts, 0), T - 1);
      const float v = x[(size_t)(m * T + tsc) * Cin + min(i, Cin - 1)];
      const bool ok = r < rows && kk < KC && ts >= 0 && ts < T;
      xT[kk][rr] = (__bf16)(ok ? v : ((kk == KC && r < rows) ? 1.f : 0.f));
    }
    __syncthreads();
    const bf16x8_t a = *reinterpret_cast<const bf16x8_t*>(&dzT[16 * w + col][8 * quad]);
#pragma unroll
    for (int d = 0; d < DT; ++d) {
      const bf16x8_t b = *reinterpret_cast<const bf16x8_t*>(&xT[16 * d + col][8 * quad]);
      acc[d] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc[d], 0, 0, 0);
    }
    __syncthreads();
  }
  // flush: lane holds o = o0 + 16w + 4quad + q, kk = 16d + col
#pragma unroll
  for (int d = 0; d < DT; ++d) {
    const int kk = 16 * d + col;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int o = o0 + 16 * w + 4 * quad + q;
      if (o < Cout) {
        if (kk < KC) atomicAdd(&dW[(size_t)kk * Cout + o], acc[d][q]);
        else if (kk == KC) atomicAdd(&db[o], acc[d][q]);
      }
    }
  }
}

// ----------------------------------------------------------------------------- host
static int conv_kp(int k, int Cin) { return (k * Cin + 31) / 32 * 32; }

static int conv_ntp(int Cout) {
  const int NT = (Cout + 15) / 16;
  return NT <= 1 ? 1 : NT <= 2 ? 2 : NT <= 4 ? 4 : 8;
}

static size_t conv_lds(int NTp, int KCH) { return (size_t)(NTp * 16 + CV_RT) * (KCH + CV_PAD) * sizeof(__bf16); }

// K chunk: all of K (W^T resident) when it fits 80 KB (two workgroups per CU), else the
// largest multiple of 32 that does
static int conv_kch(int NTp, int Kp) {
  int kch = Kp;
  while (kch > 32 && conv_lds(NTp, kch) > 80 * 1024) kch -= 32;
  return kch;
}

bool conv1d_supported(int k, int Cin, int Cout) {
  // forward / dx: any K (chunked); dW: the im2col tile (k*Cin + 1 ones row) must fit 24 column tiles
  return k >= 1 && Cin >= 1 && Cout >= 1 && Cout <= 128 && Cin <= 128 && (k * Cin + 1 + 15) / 16 <= 24;
}

static void launch_conv_fwd(ConvArgs& a) {
  const int NTp = conv_ntp(a.Cout);
  a.KCH = conv_kch(NTp, a.Kp);
  const size_t lds = conv_lds(NTp, a.KCH);
  const long ntiles = (a.rows + CV_RT - 1) / CV_RT;
  const int per_cu = std::max<int>(1, std::min<int>(4, (int)((160 * 1024) / lds)));
  const int grid = (int)std::max<long>(1, std::min<long>(ntiles, 256L * per_cu));
  auto st = stream();
#define GQ_CV_NT(N)                                                                                  \
  case N:                                                                                            \
    if (lds > 64 * 1024)                                                                             \
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&conv1d_fwd_kernel<N>),                \
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);              \
    hipLaunchKernelGGL(conv1d_fwd_kernel<N>, dim3(grid), dim3(256), lds, st, a);                     \
    break;
  switch (NTp) {
    GQ_CV_NT(1) GQ_CV_NT(2) GQ_CV_NT(4) GQ_CV_NT(8)
    default: TORCH_CHECK(false, "conv1d: Cout too large");
  }
#undef GQ_CV_NT
  GQ_LAUNCH_CHECK();
}

// x [M,T,Cin], W [k,Cin,Cout], b [Cout]. Returns [y (M,T,Cout) or empty, g (M,Cout) or empty].
std::vector<at::Tensor> conv1d_fwd(const at::Tensor& x, const at::Tensor& W, const at::Tensor& b, double alpha,
                                   bool gap, bool store_y) {
  check_f32_cuda(x, "x");
  check_f32_cuda(W, "W");
  check_f32_cuda(b, "b");
  TORCH_CHECK(x.dim() == 3 && W.dim() == 3 && W.size(1) == x.size(2) && b.numel() == W.size(2),
              "conv1d_fwd: shapes x [M,T,Cin], W [k,Cin,Cout], b [Cout]");
  const int M = (int)x.size(0), T = (int)x.size(1), Cin = (int)x.size(2);
  const int k = (int)W.size(0), Cout = (int)W.size(2);
  TORCH_CHECK(conv1d_supported(k, Cin, Cout), "conv1d_fwd: unsupported (k, Cin, Cout)");
  c10::DeviceGuard guard(x.device());
  at::Tensor y = store_y ? at::empty({M, T, Cout}, x.options()) : at::empty({0}, x.options());
  at::Tensor g = gap ? at::zeros({M, Cout}, x.options()) : at::empty({0}, x.options());
  if ((long)M * T == 0) return {y, g};
  ConvArgs a{};
  a.a = x.data_ptr<float>();
  a.gate = x.data_ptr<float>();
  a.W = W.data_ptr<float>();
  a.bias = b.data_ptr<float>();
  a.y = store_y ? y.data_ptr<float>() : nullptr;
  a.g = gap ? g.data_ptr<float>() : nullptr;
  a.rows = (long)M * T;
  a.T = T; a.Cin = Cin; a.Cout = Cout; a.k = k; a.left = (k - 1) / 2; a.lda = Cin; a.Kp = conv_kp(k, Cin);
  a.alpha = (float)alpha; a.gate_alpha = 1.f; a.a_scale = 1.f; a.bcast = 0; a.inv_T = 1.f / (float)T;
  launch_conv_fwd(a);
  return {y, g};
}

// dy: [M,T,Cout] (or dg [M,Cout] when gap); y: the layer's output [M,T,Cout]; accumulates dW, db.
// Returns dx [M,T,Cin] if need_dx.
at::Tensor conv1d_bwd(const at::Tensor& dy, const at::Tensor& y, const at::Tensor& x, const at::Tensor& W,
                      double alpha, bool gap, at::Tensor dW, at::Tensor db, bool need_dx) {
  const at::Tensor* ops[] = {&dy, &y, &x, &W};
  for (const at::Tensor* t : ops) check_f32_cuda(*t, "conv1d_bwd operand");
  const int M = (int)x.size(0), T = (int)x.size(1), Cin = (int)x.size(2);
  const int k = (int)W.size(0), Cout = (int)W.size(2);
  TORCH_CHECK(y.dim() == 3 && y.size(0) == M && y.size(1) == T && y.size(2) == Cout, "conv1d_bwd: y shape");
  TORCH_CHECK(gap ? (dy.dim() == 2 && dy.size(0) == M && dy.size(1) == Cout) : dy.sizes() == y.sizes(),
              "conv1d_bwd: dy shape");
  TORCH_CHECK(conv1d_supported(k, Cin, Cout), "conv1d_bwd: unsupported shape");
  c10::DeviceGuard guard(x.device());
  const long rows = (long)M * T;
  at::Tensor dx = need_dx ? at::empty({M, T, Cin}, x.options()) : at::empty({0}, x.options());
  if (rows == 0) return need_dx ? dx.zero_() : dx;
  const bool wg = dW.numel() > 0;
  if (wg) {
    check_f32_cuda(dW, "dW");
    check_f32_cuda(db, "db");
    TORCH_CHECK(dW.numel() == W.numel() && db.numel() == Cout, "conv1d_bwd: gradient buffer shapes");
    const int DT = (k * Cin + 1 + 15) / 16;
    const long ntiles = (rows + CW_RT - 1) / CW_RT;
    const int ncb = (Cout + 63) / 64;
    const int splits = deterministic_mode() ? 1 : (int)std::max<long>(1, std::min<long>(ntiles, 256 / ncb));
    dim3 grid(ncb, splits);
    auto st = stream();
    switch (DT) {
#define GQ_CW_DT(D)                                                                                               \
  case D:                                                                                                         \
    hipLaunchKernelGGL(conv1d_wgrad_kernel<D>, grid, dim3(256), 0, st, dy.data_ptr<float>(), y.data_ptr<float>(), \
                       x.data_ptr<float>(), dW.data_ptr<float>(), db.data_ptr<float>(), rows, T, Cin, Cout, k,    \
                       (k - 1) / 2, (float)alpha, (int)gap);                                                      \
    break;
      GQ_CW_DT(1) GQ_CW_DT(2) GQ_CW_DT(3) GQ_CW_DT(4) GQ_CW_DT(5) GQ_CW_DT(6) GQ_CW_DT(7) GQ_CW_DT(8)
      GQ_CW_DT(9) GQ_CW_DT(10) GQ_CW_DT(11) GQ_CW_DT(12) GQ_CW_DT(13) GQ_CW_DT(14) GQ_CW_DT(15) GQ_CW_DT(16)
      GQ_CW_DT(17) GQ_CW_DT(18) GQ_CW_DT(19) GQ_CW_DT(20) GQ_CW_DT(21) GQ_CW_DT(22) GQ_CW_DT(23) GQ_CW_DT(24)
#undef GQ_CW_DT
      default: TORCH_CHECK(false, "conv1d_bwd: k*Cin too large");
    }
    GQ_LAUNCH_CHECK();
  }
  if (need_dx) {
    // dx = conv_same(dz, Wf) with Wf[tap'][o][i] = W[k-1-tap'][i][o] and left' = k-1-left
    at::Tensor Wf = W.flip(0).transpose(1, 2).contiguous();
    ConvArgs a{};
    a.a = dy.data_ptr<float>();
    a.gate = y.data_ptr<float>();
    a.W = Wf.data_ptr<float>();
    a.bias = nullptr;
    a.y = dx.data_ptr<float>();
    a.g = nullptr;
    a.rows = rows;
    a.T = T; a.Cin = Cout; a.Cout = Cin; a.k = k; a.left = k - 1 - (k - 1) / 2; a.lda = Cout;
    a.Kp = conv_kp(k, Cout);
    a.alpha = 1.f; a.gate_alpha = (float)alpha; a.a_scale = gap ? 1.f / (float)T : 1.f; a.bcast = gap ? 1 : 0;
    a.inv_T = 1.f / (float)T;
    launch_conv_fwd(a);
  }
  return dx;
}

}  // namespace gq

TORCH_LIBRARY_IMPL(gnnqc, CUDA, m) {
  m.impl("conv1d_fwd", &gq::conv1d_fwd);
  m.impl("conv1d_bwd", &gq::conv1d_bwd);
}
