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
  int wflip;           // W is the FORWARD layer's [k][Cout][Cin] (p.Cin / p.Cout swapped): read it as
                       // flip(0).transpose(1, 2), the dx pass's weights, without materialising them
};

// NT = output tiles of 16 columns per workgroup (grid.y splits Cout into groups of NT tiles when the
// row tiles alone would leave the chip idle). GATE: the A loads form dy * leaky'(y) (dx pass); the
// forward skips the second load.
// Index math is table-driven: per tile the 64 rows' (sequence start, t) and per K chunk the columns'
// (tap, channel) go to LDS once, so the gather loop has no integer division; each wave gathers its 16
// rows with the lanes on consecutive K columns (consecutive channels of one tap: contiguous loads).
template <int NT, bool GATE>
__global__ __launch_bounds__(256) void conv1d_fwd_kernel(ConvArgs p) {
  extern __shared__ __attribute__((aligned(16))) __bf16 smem[];
  const int Kp = p.Kp, KCH = p.KCH, LD = KCH + CV_PAD;
  constexpr int NTC = NT * 16;                    // output columns of this workgroup
  __bf16* Wt = smem;                              // [NTC][LD]   W^T chunk
  __bf16* As = smem + NTC * LD;                   // [CV_RT][LD] im2col chunk
  int* rinfo = reinterpret_cast<int*>(As + CV_RT * LD);      // [CV_RT]: sequence start row | -1 past rows
  int* tinfo = rinfo + CV_RT;                                 // [CV_RT]: t
  int* minfo = tinfo + CV_RT;                                 // [CV_RT]: sequence
  int* kinfo = minfo + CV_RT;                                 // [KCH]: (tap << 16) | channel, -1 past K
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int col = lane & 15, quad = lane >> 4;
  const int KC = p.k * p.Cin;
  const int nch = (Kp + KCH - 1) / KCH;           // kernel-uniform
  const int n0 = blockIdx.y * NTC;                // first output column of this workgroup

  float bias[NT];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    const int n = n0 + 16 * nt + col;
    bias[nt] = p.bias != nullptr ? p.bias[min(n, p.Cout - 1)] : 0.f;
  }

  const long ntiles = (p.rows + CV_RT - 1) / CV_RT;
  bool staged = false;
  for (long tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const long r0 = tile * CV_RT;
    f32x4_t acc[NT];
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) acc[nt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    __syncthreads();                              // previous tile's reads of the tables are done
    if (tid < CV_RT) {
      const long r = r0 + tid;
      const long rc = min(r, p.rows - 1);
      const long m = rc / p.T;
      rinfo[tid] = r < p.rows ? (int)(m * p.T) : -1;
      tinfo[tid] = (int)(rc - m * p.T);
      minfo[tid] = (int)m;
    }
    for (int ch = 0; ch < nch; ++ch) {
      const int k0 = ch * KCH;
      __syncthreads();                            // previous chunk's reads of As / Wt / kinfo are done
      if (!staged) {
        for (int kk = tid; kk < KCH; kk += 256) {
          const int kg = k0 + kk;
          const int tap = kg / p.Cin;
          kinfo[kk] = kg < KC ? ((tap << 16) | (kg - tap * p.Cin)) : -1;
        }
        // W^T chunk: Wt[n][kk] = W[k0 + kk][n0 + n] (zero padded); consecutive threads read
        // consecutive output columns (coalesced); once per workgroup when K fits one chunk
        for (int e = tid; e < NTC * KCH; e += 256) {
          const int n = e % NTC, kk = e / NTC;      // (NTC: a power of two)
          const int kg = k0 + kk, ng = n0 + n;
          const float m_ = (ng < p.Cout && kg < KC) ? 1.f : 0.f;
          const int kc = min(kg, KC - 1), nc = min(ng, p.Cout - 1);
          size_t wi = (size_t)kc * p.Cout + nc;
          if (p.wflip) {                            // W_fwd[k - 1 - tap][nc][i] ([k][Cout_fwd = p.Cin][Cin_fwd = p.Cout])
            const int tap = kc / p.Cin, i = kc - tap * p.Cin;
            wi = ((size_t)(p.k - 1 - tap) * p.Cout + nc) * p.Cin + i;
          }
          Wt[n * LD + kk] = (__bf16)(p.W[wi] * m_);
        }
        staged = nch == 1;
      }
      __syncthreads();
      // ---- im2col A chunk: wave w gathers rows 16w .. 16w+15, lanes on K columns
      for (int kb = 0; kb < KCH; kb += 64) {
        const int kk = kb + lane;
        const int ki = kk < KCH ? kinfo[kk] : -1;
        const int tap = ki >> 16, ic = ki & 0xffff;
        // (fully unrolled: the 16 rows' loads are in flight together; the gather is latency-bound)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int rr = 16 * w + r;
          const int rb = rinfo[rr], t = tinfo[rr];  // (LDS broadcast)
          const int ts = t + tap - p.left;
          const bool ok = ki >= 0 && rb >= 0 && ts >= 0 && ts < p.T;
          const int tsc = min(max(ts, 0), p.T - 1);
          const long src = p.bcast ? (long)minfo[rr] : (long)(rb >= 0 ? rb : 0) + tsc;
          const int icc = ki >= 0 ? ic : 0;
          float v = p.a[(size_t)src * p.lda + icc];
          if constexpr (GATE) {
            const float gy = p.gate[((size_t)(rb >= 0 ? rb : 0) + tsc) * p.Cin + icc];
            v *= (gy > 0.f ? 1.f : p.gate_alpha) * p.a_scale;
          }
          if (kk < KCH) As[rr * LD + kk] = (__bf16)(ok ? v : 0.f);
        }
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
    // ---- epilogue: lane holds rows 16w + 4quad + q of column n0 + 16nt + col
    const long rb = r0 + 16 * w + 4 * quad;
    const long m_first = min(rb, p.rows - 1) / p.T, m_last = min(rb + 3, p.rows - 1) / p.T;
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      const int n = n0 + 16 * nt + col;
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

// Each split (grid.y) leaves its partial dW^T | db tile in ws[split][CoutP][KT] with plain stores;
// conv1d_wgrad_reduce_kernel sums the splits in a fixed order (deterministic). (Flushed with atomics,
// all splits hit the same addresses and the L2 atomic unit serialised them: 40-55 us per call at 256
// splits, profiles/r6_cnn_kernel_stats_*.)
template <int DT>      // DT = ceil((k*Cin + 1) / 16) im2col column tiles (incl. the ones row)
__global__ __launch_bounds__(256) void conv1d_wgrad_kernel(const float* __restrict__ dy, const float* __restrict__ y,
                                                            const float* __restrict__ x, float* __restrict__ ws,
                                                            int CoutP, long rows, int T, int Cin,
                                                            int Cout, int k, int left, float alpha, int gap) {
  constexpr int KT = DT * 16;
  __shared__ __attribute__((aligned(16))) __bf16 dzT[64][CW_LD];
  __shared__ __attribute__((aligned(16))) __bf16 xT[KT][CW_LD];
  // index tables (no integer division in the staging loops): per im2col column (tap << 16 | channel;
  // -2 = the ones row of db, -1 = padding), per tile row (sequence start row, t, sequence)
  __shared__ int kinfo[KT];
  __shared__ int rbase[CW_RT], tinf[CW_RT], minf[CW_RT];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int col = lane & 15, quad = lane >> 4;
  const int o0 = blockIdx.x * 64;
  const int KC = k * Cin;
  const long ntiles = (rows + CW_RT - 1) / CW_RT;
  const float inv_T = 1.f / (float)T;
  for (int kk = tid; kk < KT; kk += 256) {
    const int tap = kk / Cin;
    kinfo[kk] = kk < KC ? ((tap << 16) | (kk - tap * Cin)) : (kk == KC ? -2 : -1);
  }
  f32x4_t acc[DT];
#pragma unroll
  for (int d = 0; d < DT; ++d) acc[d] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  for (long tile = blockIdx.y; tile < ntiles; tile += gridDim.y) {
    const long r0 = tile * CW_RT;
    __syncthreads();                              // previous tile's reads of the images / tables
    if (tid < CW_RT) {
      const long r = r0 + tid;
      const long rc = min(r, rows - 1);
      const long m = rc / T;
      rbase[tid] = r < rows ? (int)(m * T) : -1;
      tinf[tid] = (int)(rc - m * T);
      minf[tid] = (int)m;
    }
    __syncthreads();
#pragma unroll
    for (int e = tid; e < CW_RT * 64; e += 256) {
      const int rr = e >> 6, oo = e & 63;
      const int rb = rbase[rr];
      const long rc = rb >= 0 ? (long)rb + tinf[rr] : 0;
      const int o = min(o0 + oo, Cout - 1);
      const float gy = y[(size_t)rc * Cout + o];
      const float d = dy[(size_t)(gap ? minf[rr] : rc) * Cout + o] * (gap ? inv_T : 1.f);
      const bool ok = rb >= 0 && o0 + oo < Cout;
      dzT[oo][rr] = (__bf16)(ok ? d * (gy > 0.f ? 1.f : alpha) : 0.f);
    }
#pragma unroll 6
    for (int e = tid; e < CW_RT * KT; e += 256) {
      const int kk = e % KT, rr = e / KT;         // (KT: compile-time)
      const int ki = kinfo[kk];
      const int rb = rbase[rr], t = tinf[rr];
      const int tap = ki >> 16, i = ki & 0xffff;
      const int ts = t + tap - left;
      const int tsc = min(max(ts, 0), T - 1);
      const float v = x[((size_t)(rb >= 0 ? rb : 0) + tsc) * Cin + (ki >= 0 ? i : 0)];
      const bool ok = rb >= 0 && ki >= 0 && ts >= 0 && ts < T;
      xT[kk][rr] = (__bf16)(ok ? v : ((ki == -2 && rb >= 0) ? 1.f : 0.f));
    }
    __syncthreads();
    const bf16x8_t a = *reinterpret_cast<const bf16x8_t*>(&dzT[16 * w + col][8 * quad]);
#pragma unroll
    for (int d = 0; d < DT; ++d) {
      const bf16x8_t b = *reinterpret_cast<const bf16x8_t*>(&xT[16 * d + col][8 * quad]);
      acc[d] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc[d], 0, 0, 0);
    }
  }
  // partial record: lane holds o = o0 + 16w + 4quad + q, kk = 16d + col
  float* rec = ws + (size_t)blockIdx.y * CoutP * KT;
#pragma unroll
  for (int d = 0; d < DT; ++d) {
    const int kk = 16 * d + col;
#pragma unroll
    for (int q = 0; q < 4; ++q) rec[(size_t)(o0 + 16 * w + 4 * quad + q) * KT + kk] = acc[d][q];
  }
}

// dW[kk][o] += sum over splits of ws[split][o][kk] (kk < KC), db[o] += ... (kk == KC). A workgroup
// takes 16 consecutive elements; its 16 thread groups sum every 16th split (loads in flight together),
// then the 16 group sums are added in a fixed order (deterministic)
__global__ __launch_bounds__(256) void conv1d_wgrad_reduce_kernel(const float* __restrict__ ws, int splits, int CoutP,
                                                                   int KT, int KC, int Cout, float* __restrict__ dW,
                                                                   float* __restrict__ db) {
  __shared__ float part[16][17];
  const int el = threadIdx.x & 15, g = threadIdx.x >> 4;
  const long E = (long)CoutP * KT;
  const long e = (long)blockIdx.x * 16 + el;
  const long ec = e < E ? e : E - 1;
  float s0 = 0.f, s1 = 0.f;
  int sp = g;
#pragma unroll 4
  for (; sp + 16 < splits; sp += 32) {
    s0 += ws[(size_t)sp * E + ec];
    s1 += ws[(size_t)(sp + 16) * E + ec];
  }
  if (sp < splits) s0 += ws[(size_t)sp * E + ec];
  part[g][el] = s0 + s1;
  __syncthreads();
  if (g != 0 || e >= E) return;
  float s = 0.f;
#pragma unroll
  for (int q = 0; q < 16; ++q) s += part[q][el];
  const int o = (int)(e / KT), kk = (int)(e - (long)o * KT);
  if (o >= Cout || kk > KC) return;
  if (kk < KC) dW[(size_t)kk * Cout + o] += s;
  else db[o] += s;
}

// ----------------------------------------------------------------------------- host
static int conv_kp(int k, int Cin) { return (k * Cin + 31) / 32 * 32; }

static int conv_ntp(int Cout) {
  const int NT = (Cout + 15) / 16;
  return NT <= 1 ? 1 : NT <= 2 ? 2 : NT <= 4 ? 4 : 8;
}

static size_t conv_lds(int NTp, int KCH) {
  return (size_t)(NTp * 16 + CV_RT) * (KCH + CV_PAD) * sizeof(__bf16) + (3 * CV_RT + KCH) * sizeof(int);
}

// K chunk: all of K (W^T resident) when it fits 80 KB (two workgroups per CU), else the
// largest multiple of 32 that does
static int conv_kch(int NTp, int Kp, size_t limit = 80 * 1024) {
  int kch = Kp;
  while (kch > 32 && conv_lds(NTp, kch) > limit) kch -= 32;
  return kch;
}

bool conv1d_supported(int k, int Cin, int Cout) {
  // forward / dx: any K (chunked); dW: the im2col tile (k*Cin + 1 ones row) must fit 24 column tiles
  return k >= 1 && Cin >= 1 && Cout >= 1 && Cout <= 128 && Cin <= 128 && (k * Cin + 1 + 15) / 16 <= 24;
}

static void launch_conv_fwd(ConvArgs& a, bool gate) {
  const int NT = conv_ntp(a.Cout);
  const long ntiles = (a.rows + CV_RT - 1) / CV_RT;
  // few row tiles (the deep, short layers): split the output columns over grid.y so the launch has
  // enough workgroups (each gathers the same A tile, small next to the idle chip it fills)
  int NTW = NT;
  while (NTW > 1 && ntiles * (NT / NTW) < 256) NTW /= 2;
  // (a grid of at most one workgroup per CU may take the whole LDS: K in one chunk, one gather pass)
  a.KCH = conv_kch(NTW, a.Kp, ntiles * (NT / NTW) <= 256 ? 160 * 1024 : 80 * 1024);
  const size_t lds = conv_lds(NTW, a.KCH);
  const int per_cu = std::max<int>(1, std::min<int>(4, (int)((160 * 1024) / lds)));
  const int gx = (int)std::max<long>(1, std::min<long>(ntiles, 256L * per_cu / (NT / NTW)));
  dim3 grid(gx, NT / NTW);
  auto st = stream();
#define GQ_CV_NT(N, G)                                                                               \
  {                                                                                                  \
    if (lds > 64 * 1024)                                                                             \
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&conv1d_fwd_kernel<N, G>),             \
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);              \
    hipLaunchKernelGGL((conv1d_fwd_kernel<N, G>), grid, dim3(256), lds, st, a);                      \
  }
#define GQ_CV_G(N) case N: if (gate) GQ_CV_NT(N, true) else GQ_CV_NT(N, false) break;
  switch (NTW) {
    GQ_CV_G(1) GQ_CV_G(2) GQ_CV_G(4) GQ_CV_G(8)
    default: TORCH_CHECK(false, "conv1d: Cout too large");
  }
#undef GQ_CV_G
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
  launch_conv_fwd(a, false);
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
    // splits write partial records, reduced in a fixed order by a second launch (deterministic)
    const int splits = (int)std::max<long>(1, std::min<long>(ntiles, 256 / ncb));
    const int CoutP = ncb * 64, KT = DT * 16;
    at::Tensor ws = at::empty({(long)splits * CoutP * KT}, x.options());
    dim3 grid(ncb, splits);
    auto st = stream();
    switch (DT) {
#define GQ_CW_DT(D)                                                                                               \
  case D:                                                                                                         \
    hipLaunchKernelGGL(conv1d_wgrad_kernel<D>, grid, dim3(256), 0, st, dy.data_ptr<float>(), y.data_ptr<float>(), \
                       x.data_ptr<float>(), ws.data_ptr<float>(), CoutP, rows, T, Cin, Cout, k,                   \
                       (k - 1) / 2, (float)alpha, (int)gap);                                                      \
    break;
      GQ_CW_DT(1) GQ_CW_DT(2) GQ_CW_DT(3) GQ_CW_DT(4) GQ_CW_DT(5) GQ_CW_DT(6) GQ_CW_DT(7) GQ_CW_DT(8)
      GQ_CW_DT(9) GQ_CW_DT(10) GQ_CW_DT(11) GQ_CW_DT(12) GQ_CW_DT(13) GQ_CW_DT(14) GQ_CW_DT(15) GQ_CW_DT(16)
      GQ_CW_DT(17) GQ_CW_DT(18) GQ_CW_DT(19) GQ_CW_DT(20) GQ_CW_DT(21) GQ_CW_DT(22) GQ_CW_DT(23) GQ_CW_DT(24)
#undef GQ_CW_DT
      default: TORCH_CHECK(false, "conv1d_bwd: k*Cin too large");
    }
    GQ_LAUNCH_CHECK();
    hipLaunchKernelGGL(conv1d_wgrad_reduce_kernel, dim3((CoutP * KT + 15) / 16), dim3(256), 0, st,
                       ws.data_ptr<float>(), splits, CoutP, KT, k * Cin, Cout, dW.data_ptr<float>(),
                       db.data_ptr<float>());
    GQ_LAUNCH_CHECK();
  }
  if (need_dx) {
    // dx = conv_same(dz, Wf) with Wf[tap'][o][i] = W[k-1-tap'][i][o] and left' = k-1-left (read in place:
    // wflip)
    const at::Tensor Wc = W.contiguous();
    ConvArgs a{};
    a.a = dy.data_ptr<float>();
    a.gate = y.data_ptr<float>();
    a.W = Wc.data_ptr<float>();
    a.wflip = 1;
    a.bias = nullptr;
    a.y = dx.data_ptr<float>();
    a.g = nullptr;
    a.rows = rows;
    a.T = T; a.Cin = Cout; a.Cout = Cin; a.k = k; a.left = k - 1 - (k - 1) / 2; a.lda = Cout;
    a.Kp = conv_kp(k, Cout);
    a.alpha = 1.f; a.gate_alpha = (float)alpha; a.a_scale = gap ? 1.f / (float)T : 1.f; a.bcast = gap ? 1 : 0;
    a.inv_T = 1.f / (float)T;
    launch_conv_fwd(a, true);
  }
  return dx;
}

}  // namespace gq

TORCH_LIBRARY_IMPL(gnnqc, CUDA, m) {
  m.impl("conv1d_fwd", &gq::conv1d_fwd);
  m.impl("conv1d_bwd", &gq::conv1d_bwd);
}
