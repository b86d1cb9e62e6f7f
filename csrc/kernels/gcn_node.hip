// Per-node GeneralConv (+ BatchNorm + PReLU) writing the time-major LSTM input, for
// graphs whose nodes each keep their own sequence (SoilNet, SURVEY §2.2 K1 + K2s).
//
// Reference: spektral GeneralConv on the block-diagonal (sample, time step) graph, then
// Concatenate([gcn_out, features]) and `graph_reshape` into one sequence per node
// (libs/create_model.py:184-189, :225-233, :242-258). The eager equivalent here is
// einsum('bij,btjf->btif', D^-1 A, act(x W + b)) -> cat -> permute/reshape -> pad ->
// transpose, i.e. a dense [N,N] fp32 bmm over all B*T steps plus four full copies of a
// [B*N, T, 19] tensor. SoilNet neighbourhoods are sparse (same depth within a radius or
// the same profile within a depth range), so:
//
//  gcn_adj_bits      adjacency -> 32-bit row masks of A and A^T + row scales (1/deg)
//                    (once per batch; shared by every time step of the sample)
//  gcn_node_fwd      one workgroup per (sample, chunk of time steps): per step, the
//                    activations act(x_j W + b) of all nodes go to LDS, then every
//                    output (node i, channel c) sums its neighbours' LDS entries by
//                    walking the set bits of its row mask. The row written is the final
//                    LSTM-input row [T][Mp][Cp] (m = b*N + i): F aggregated channels, the
//                    Cin raw channels, zero padding up to Cp (float4 granules).
//  gcn_node_bwd      same traversal over A^T for da = A^T (D^-1 dagg); the per-channel
//                    partial sums (sum dy, sum dy*z, dalpha, sum x_k dy) feed the closed-form
//                    gcn_bwd_finalize of gcn_glue.hip (BatchNorm statistics come from the
//                    x moments of gcn_stats, exactly as on the CML path).
//  gcn_node_bwd_input  dx for attribution: dz from the finalize coefficients, reduced over
//                    channels with lane shuffles, plus the pass-through of the raw channels.
#include "common.h"

#include <cstdlib>

namespace gq {

at::Tensor colsum(const at::Tensor& partial);     // gcn.hip

// bits[b][i][w]: bit q of word w set iff A[b,i,32w+q] != 0 ; bitsT the same for A^T.
// rs[b][i] = 1/deg_i (mean aggregation; 0 for an isolated node) or 1 (sum).
__global__ void gcn_adj_bits_kernel(const float* __restrict__ adj, unsigned* __restrict__ bits,
                                    unsigned* __restrict__ bitsT, int B, int N, int NWd) {
  const long total = (long)B * N * NWd;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
    const int w = e % NWd;
    const long bi = e / NWd;
    const int i = bi % N, b = bi / N;
    const float* A = adj + (long)b * N * N;
    unsigned m = 0u, mt = 0u;
    for (int q = 0; q < 32; ++q) {
      const int j = 32 * w + q;
      if (j < N) {
        m |= (A[(long)i * N + j] != 0.f ? 1u : 0u) << q;
        mt |= (A[(long)j * N + i] != 0.f ? 1u : 0u) << q;
      }
    }
    bits[e] = m;
    bitsT[e] = mt;
  }
}

__global__ void gcn_row_scale_kernel(const unsigned* __restrict__ bits, float* __restrict__ rs, int rows, int NWd,
                                     int mean) {
  for (int r = blockIdx.x * blockDim.x + threadIdx.x; r < rows; r += gridDim.x * blockDim.x) {
    int d = 0;
    for (int w = 0; w < NWd; ++w) d += __popc(bits[(long)r * NWd + w]);
    rs[r] = mean ? (d > 0 ? 1.f / (float)d : 0.f) : 1.f;
  }
}

// sum over the set bits of one row mask of vals[j * F + f]
__device__ __forceinline__ float row_gather(const unsigned* __restrict__ row, int NWd, const float* __restrict__ vals,
                                            int F, int f) {
  float acc = 0.f;
  for (int w = 0; w < NWd; ++w) {
    unsigned m = row[w];
    while (m) {
      const int q = __builtin_ctz(m);
      m &= m - 1u;
      acc += vals[(32 * w + q) * F + f];
    }
  }
  return acc;
}

// V consecutive channels c0..c0+V-1 at once (one ds_read_b128 per neighbour when V == 4;
// vals 16-byte aligned, F and c0 multiples of V): one bit walk per V channels
template <int V>
__device__ __forceinline__ void row_gather_v(const unsigned* __restrict__ row, int NWd, const float* __restrict__ vals,
                                             int F, int c0, float (&acc)[V]) {
#pragma unroll
  for (int v = 0; v < V; ++v) acc[v] = 0.f;
  for (int w = 0; w < NWd; ++w) {
    unsigned m = row[w];
    while (m) {
      const int q = __builtin_ctz(m);
      m &= m - 1u;
      const float* p = vals + (32 * w + q) * F + c0;
      if constexpr (V == 4) {
        const float4 a = *reinterpret_cast<const float4*>(p);
        acc[0] += a.x; acc[1] += a.y; acc[2] += a.z; acc[3] += a.w;
      } else {
#pragma unroll
        for (int v = 0; v < V; ++v) acc[v] += p[v];
      }
    }
  }
}

struct NodeSmem {
  unsigned* bits;
  float* vals;
  float* rs;
  float* mk;
  float* xs;                                   // [2][N * Cin] staged node inputs of a step (Cin <= 4)
  __device__ NodeSmem(unsigned char* base, int N, int NWd, int F) {
    bits = reinterpret_cast<unsigned*>(base);
    vals = reinterpret_cast<float*>(bits + ((size_t)N * NWd + 3) / 4 * 4);   // 16-byte aligned rows
    rs = vals + (size_t)N * F;
    mk = rs + N;
    xs = mk + N;
  }
};

static size_t node_smem_bytes(int N, int NWd, int F) {
  return ((size_t)N * NWd + 3) / 4 * 16 + (size_t)N * F * 4 + (size_t)N * 8 + (size_t)N * 32;
}

// ------------------------------------------------------------------ forward
template <int Cin, int V>
__global__ __launch_bounds__(256) void gcn_node_fwd_kernel(
    const float* __restrict__ x, const unsigned* __restrict__ bits, const float* __restrict__ rs,
    const float* __restrict__ mask, const float* __restrict__ W, const float* __restrict__ bias,
    const float* __restrict__ scale, const float* __restrict__ shift, const float* __restrict__ alpha,
    float* __restrict__ out, int B, int T, int N, int F, int Cp, int Mp, int NWd, int tchunk) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  NodeSmem sm(smem_raw, N, NWd, F);
  const int tid = threadIdx.x, b = blockIdx.y, t0 = blockIdx.x * tchunk;
  for (int e = tid; e < N * NWd; e += 256) sm.bits[e] = bits[(long)b * N * NWd + e];
  for (int i = tid; i < N; i += 256) {
    sm.rs[i] = rs[(long)b * N + i];
    sm.mk[i] = mask[(long)b * N + i];
  }
  const int f = tid % F;                       // 256 % F == 0: fixed channel per thread
  float wk[Cin];
#pragma unroll
  for (int k = 0; k < Cin; ++k) wk[k] = W[k * F + f];
  const float bb = bias[f], sc = scale[f], sh = shift[f], al = alpha[f];
  const int t1 = min(t0 + tchunk, T);
  // x_t (N * Cin floats) is staged in LDS one step ahead, during the previous step's gather: the
  // activation loop below then reads LDS instead of issuing a dependent HBM load per item
  for (int e = tid; e < N * Cin; e += 256) sm.xs[e] = x[((long)b * T + t0) * (long)N * Cin + e];
  for (int t = t0; t < t1; ++t) {
    __syncthreads();                           // previous step's reads of vals are done, xs[t] written
    const float* xt = sm.xs + ((t - t0) & 1) * N * Cin;
    for (int e = tid; e < N * F; e += 256) {
      const int j = e / F;
      float z = bb;
#pragma unroll
      for (int k = 0; k < Cin; ++k) z += xt[j * Cin + k] * wk[k];
      const float y = z * sc + sh;
      sm.vals[e] = (y > 0.f ? y : al * y) * sm.mk[j];
    }
    __syncthreads();
    if (t + 1 < t1) {                          // stage x_{t+1} (its buffer was last read in step t-1)
      float* xn = sm.xs + ((t + 1 - t0) & 1) * N * Cin;
      for (int e = tid; e < N * Cin; e += 256) xn[e] = x[((long)b * T + t + 1) * (long)N * Cin + e];
    }
    float* ot = out + ((long)t * Mp + (long)b * N) * Cp;
    // V output channels per item (F, Cp multiples of V): aggregated groups walk the row mask once
    const int G = Cp / V;
    for (int e = tid; e < N * G; e += 256) {
      const int i = e / G, c0 = (e - i * G) * V;
      float v[V];
      if (c0 < F) {
        row_gather_v<V>(sm.bits + (size_t)i * NWd, NWd, sm.vals, F, c0, v);
        const float r = sm.rs[i];
#pragma unroll
        for (int u = 0; u < V; ++u) v[u] *= r;
      } else {
#pragma unroll
        for (int u = 0; u < V; ++u) v[u] = c0 + u < F + Cin ? xt[i * Cin + (c0 + u - F)] : 0.f;
      }
      if constexpr (V == 4) {
        *reinterpret_cast<float4*>(ot + (long)i * Cp + c0) = make_float4(v[0], v[1], v[2], v[3]);
      } else {
#pragma unroll
        for (int u = 0; u < V; ++u) ot[(long)i * Cp + c0 + u] = v[u];
      }
    }
  }
  if (b == B - 1) {                            // zero the padding rows B*N .. Mp-1
    const int npad = (Mp - B * N) * Cp;
    for (int t = t0; t < t1; ++t)
      for (int e = tid; e < npad; e += 256) out[((long)t * Mp + (long)B * N) * Cp + e] = 0.f;
  }
}

// ------------------------------------------------------------------ backward (params)
// partial[blk][q][f], q: 0 = sum dy, 1 = sum dy*z, 2 = sum da*y[y<=0], 3+k = sum x_k dy
template <int Cin, int V>
__global__ __launch_bounds__(256) void gcn_node_bwd_kernel(
    const float* __restrict__ x, const unsigned* __restrict__ bitsT, const float* __restrict__ rs,
    const float* __restrict__ mask, const float* __restrict__ dout, const float* __restrict__ W,
    const float* __restrict__ bias, const float* __restrict__ scale, const float* __restrict__ shift,
    const float* __restrict__ alpha, float* __restrict__ partial, int B, int T, int N, int F, int Cp, int Mp,
    int NWd, int tchunk) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  NodeSmem sm(smem_raw, N, NWd, F);
  constexpr int NACC = 3 + Cin;
  const int tid = threadIdx.x, b = blockIdx.y, t0 = blockIdx.x * tchunk;
  for (int e = tid; e < N * NWd; e += 256) sm.bits[e] = bitsT[(long)b * N * NWd + e];
  for (int i = tid; i < N; i += 256) {
    sm.rs[i] = rs[(long)b * N + i];
    sm.mk[i] = mask[(long)b * N + i];
  }
  const int f = tid % F;
  // gather phase: V channels c0..c0+V-1 per item (G = F / V groups; 256 % G == 0, so fixed per thread)
  const int G = F / V, c0 = (tid % G) * V;
  float wk[V][Cin], bb[V], sc[V], sh[V], al[V];
#pragma unroll
  for (int v = 0; v < V; ++v) {
#pragma unroll
    for (int k = 0; k < Cin; ++k) wk[v][k] = W[k * F + c0 + v];
    bb[v] = bias[c0 + v];
    sc[v] = scale[c0 + v];
    sh[v] = shift[c0 + v];
    al[v] = alpha[c0 + v];
  }
  float acc[V][NACC];
#pragma unroll
  for (int v = 0; v < V; ++v)
#pragma unroll
    for (int q = 0; q < NACC; ++q) acc[v][q] = 0.f;
  const int t1 = min(t0 + tchunk, T);
  for (int t = t0; t < t1; ++t) {
    __syncthreads();
    const float* dt = dout + ((long)t * Mp + (long)b * N) * Cp;
    if constexpr (V == 4) {                    // Cp % 4 == 0 (host): one 16-byte load per 4 channels
#pragma unroll 4
      for (int e = tid; e < N * G; e += 256) {
        const int i = e / G, cc = (e - i * G) * 4;
        float4 d = *reinterpret_cast<const float4*>(dt + (long)i * Cp + cc);
        const float r = sm.rs[i];
        d.x *= r; d.y *= r; d.z *= r; d.w *= r;          // dagg_i / deg_i
        *reinterpret_cast<float4*>(sm.vals + i * F + cc) = d;
      }
    } else {
      for (int e = tid; e < N * F; e += 256) {
        const int i = e / F;
        sm.vals[e] = dt[(long)i * Cp + f] * sm.rs[i];  // dagg_i / deg_i
      }
    }
    for (int e = tid; e < N * Cin; e += 256) sm.xs[e] = x[((long)b * T + t) * (long)N * Cin + e];
    __syncthreads();
    const float* xt = sm.xs;
    for (int e = tid; e < N * G; e += 256) {
      const int j = e / G;
      if (sm.mk[j] == 0.f) continue;               // masked node: activation forced to 0
      float da[V];
      row_gather_v<V>(sm.bits + (size_t)j * NWd, NWd, sm.vals, F, c0, da);
      float xv[Cin];
#pragma unroll
      for (int k = 0; k < Cin; ++k) xv[k] = xt[j * Cin + k];
#pragma unroll
      for (int v = 0; v < V; ++v) {
        float z = bb[v];
#pragma unroll
        for (int k = 0; k < Cin; ++k) z += xv[k] * wk[v][k];
        const float y = z * sc[v] + sh[v];
        const float dy = y > 0.f ? da[v] : al[v] * da[v];
        acc[v][0] += dy;
        acc[v][1] += dy * z;
        acc[v][2] += y > 0.f ? 0.f : da[v] * y;
#pragma unroll
        for (int k = 0; k < Cin; ++k) acc[v][3 + k] += xv[k] * dy;
      }
    }
  }
  __shared__ float red[4][NACC][64];
  const int lane = tid & 63, wv = tid >> 6;
#pragma unroll
  for (int v = 0; v < V; ++v)
#pragma unroll
    for (int q = 0; q < NACC; ++q) {
      float a = acc[v][q];
      for (int o = 32; o >= G; o >>= 1) a += __shfl_xor(a, o, 64);
      if (lane < G) red[wv][q][lane * V + v] = a;  // lane g holds channels g*V .. g*V+V-1
    }
  __syncthreads();
  const long blk = (long)blockIdx.y * gridDim.x + blockIdx.x;
  for (int e = tid; e < NACC * F; e += 256) {
    const int q = e / F, ff = e % F;
    partial[blk * NACC * F + e] = red[0][q][ff] + red[1][q][ff] + red[2][q][ff] + red[3][q][ff];
  }
}

// ------------------------------------------------------------------ backward (input)
// dx[b,t,j,k] = sum_f W[k,f] dz_f(j) + dout[t][b*N+j][F+k], dz_f = coef1 dy + coef0 + coef2 z
template <int Cin>
__global__ __launch_bounds__(256) void gcn_node_bwd_input_kernel(
    const float* __restrict__ x, const unsigned* __restrict__ bitsT, const float* __restrict__ rs,
    const float* __restrict__ mask, const float* __restrict__ dout, const float* __restrict__ W,
    const float* __restrict__ bias, const float* __restrict__ scale, const float* __restrict__ shift,
    const float* __restrict__ alpha, const float* __restrict__ coef, float* __restrict__ dx, int B, int T, int N,
    int F, int Cp, int Mp, int NWd, int tchunk) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  NodeSmem sm(smem_raw, N, NWd, F);
  const int tid = threadIdx.x, b = blockIdx.y, t0 = blockIdx.x * tchunk;
  for (int e = tid; e < N * NWd; e += 256) sm.bits[e] = bitsT[(long)b * N * NWd + e];
  for (int i = tid; i < N; i += 256) {
    sm.rs[i] = rs[(long)b * N + i];
    sm.mk[i] = mask[(long)b * N + i];
  }
  const int f = tid % F;
  float wk[Cin];
#pragma unroll
  for (int k = 0; k < Cin; ++k) wk[k] = W[k * F + f];
  const float bb = bias[f], sc = scale[f], sh = shift[f], al = alpha[f];
  const float c0 = coef[f], c1 = coef[F + f], c2 = coef[2 * F + f];
  const int NF = N * F, NFp = (NF + 255) / 256 * 256;  // every lane runs every iteration (shuffles)
  const int t1 = min(t0 + tchunk, T);
  for (int t = t0; t < t1; ++t) {
    __syncthreads();
    const float* dt = dout + ((long)t * Mp + (long)b * N) * Cp;
    for (int e = tid; e < NF; e += 256) {
      const int i = e / F;
      sm.vals[e] = dt[(long)i * Cp + f] * sm.rs[i];
    }
    __syncthreads();
    const float* xt = x + ((long)b * T + t) * (long)N * Cin;
    for (int e = tid; e < NFp; e += 256) {
      const int j = min(e / F, N - 1);
      const bool ok = e < NF && sm.mk[j] != 0.f;
      const float da = ok ? row_gather(sm.bits + (size_t)j * NWd, NWd, sm.vals, F, f) : 0.f;
      float xv[Cin];
      float z = bb;
#pragma unroll
      for (int k = 0; k < Cin; ++k) {
        xv[k] = xt[j * Cin + k];
        z += xv[k] * wk[k];
      }
      const float y = z * sc + sh;
      const float dy = y > 0.f ? da : al * da;
      const float dz = ok ? c1 * dy + c0 + c2 * z : 0.f;
#pragma unroll
      for (int k = 0; k < Cin; ++k) {
        float v = wk[k] * dz;
        for (int o = 1; o < F; o <<= 1) v += __shfl_xor(v, o, 64);
        if (f == 0 && e < NF) {
          dx[(((long)b * T + t) * N + j) * Cin + k] = v + dt[(long)j * Cp + F + k];
        }
      }
    }
  }
}

#define GQ_NODE_CIN_DISPATCH(CIN_RT, ...)                        \
  switch (CIN_RT) {                                              \
    case 1: { constexpr int CIN = 1; __VA_ARGS__; } break;       \
    case 2: { constexpr int CIN = 2; __VA_ARGS__; } break;       \
    case 3: { constexpr int CIN = 3; __VA_ARGS__; } break;       \
    case 4: { constexpr int CIN = 4; __VA_ARGS__; } break;       \
    default: TORCH_CHECK(false, "gcn_node: 1..4 input channels"); \
  }

#define GQ_NODE_V_DISPATCH(VEC, ...)                   \
  if (VEC) {                                           \
    constexpr int VV = 4;                              \
    __VA_ARGS__;                                       \
  } else {                                             \
    constexpr int VV = 1;                              \
    __VA_ARGS__;                                       \
  }

struct NodeGeom {
  int B, T, N, Cin, F, NWd, tchunk;
  size_t smem;
  dim3 grid;
};

static NodeGeom node_geom(const at::Tensor& x, const at::Tensor& bits, const at::Tensor& W, int tdef = 2) {
  NodeGeom g;
  TORCH_CHECK(x.dim() == 4, "gcn_node: x must be [B,T,N,Cin]");
  g.B = x.size(0);
  g.T = x.size(1);
  g.N = x.size(2);
  g.Cin = x.size(3);
  g.F = W.size(1);
  g.NWd = (g.N + 31) / 32;
  TORCH_CHECK(W.size(0) == g.Cin, "gcn_node: W must be [Cin,F]");
  TORCH_CHECK(g.F <= 64 && 64 % g.F == 0, "gcn_node: F must divide 64");
  TORCH_CHECK(bits.numel() == (long)g.B * g.N * g.NWd, "gcn_node: adjacency bit rows shape");
  g.smem = node_smem_bytes(g.N, g.NWd, g.F);
  TORCH_CHECK(g.smem <= 150 * 1024, "gcn_node: graph too large for LDS (N=", g.N, ")");
  // enough workgroups to fill 256 CUs several times over
  const long steps = (long)g.B * g.T;
  // steps per workgroup cap (A/B: GNNQC_NODE_TCHUNK overrides both). SoilNet, scripts/node_tchunk_sweep.sh:
  // forward 113 / 112 / 123 / 155 us and parameter backward 207 / 172 / 153 / 178 us at 1 / 2 / 4 / 8
  static const int tenv = [] {
    const char* e = std::getenv("GNNQC_NODE_TCHUNK");
    return e != nullptr ? std::max(1, std::atoi(e)) : 0;
  }();
  const int tmax = tenv > 0 ? tenv : tdef;
  g.tchunk = (int)std::max<long>(1, std::min<long>(tmax, steps / 1024));
  g.grid = dim3((g.T + g.tchunk - 1) / g.tchunk, g.B);
  return g;
}

template <typename K>
static void allow_smem(K kernel, size_t bytes) {
  if (bytes > 64 * 1024)
    TORCH_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                                    (int)bytes) == hipSuccess, "gcn_node: LDS attribute");
}

// returns [bits (int32 [B,N,NWd]), bitsT, rs (float [B,N])]
std::vector<at::Tensor> gcn_adj_bits(const at::Tensor& adj, bool agg_mean) {
  check_f32_cuda(adj, "adj");
  TORCH_CHECK(adj.dim() == 3 && adj.size(1) == adj.size(2), "gcn_adj_bits: adj must be [B,N,N]");
  const int B = adj.size(0), N = adj.size(1), NWd = (N + 31) / 32;
  c10::DeviceGuard guard(adj.device());
  auto io = adj.options().dtype(at::kInt);
  at::Tensor bits = at::empty({B, N, NWd}, io), bitsT = at::empty({B, N, NWd}, io);
  at::Tensor rs = at::empty({B, N}, adj.options());
  const long total = (long)B * N * NWd;
  const int grid = (int)std::max<long>(1, std::min<long>((total + 255) / 256, 2048));
  hipLaunchKernelGGL(gcn_adj_bits_kernel, dim3(grid), dim3(256), 0, stream(), adj.data_ptr<float>(),
                     reinterpret_cast<unsigned*>(bits.data_ptr<int>()), reinterpret_cast<unsigned*>(bitsT.data_ptr<int>()),
                     B, N, NWd);
  GQ_LAUNCH_CHECK();
  const int rows = B * N;
  hipLaunchKernelGGL(gcn_row_scale_kernel, dim3(std::max(1, std::min((rows + 255) / 256, 1024))), dim3(256), 0,
                     stream(), reinterpret_cast<const unsigned*>(bits.data_ptr<int>()), rs.data_ptr<float>(), rows, NWd,
                     (int)agg_mean);
  GQ_LAUNCH_CHECK();
  return {bits, bitsT, rs};
}

// out: [T, Mp, Cp] (m = b*N + i; channels [agg F | raw Cin | zeros]); rows >= B*N zero.
at::Tensor gcn_node_fwd(const at::Tensor& x, const at::Tensor& bits, const at::Tensor& rs, const at::Tensor& mask,
                        const at::Tensor& W, const at::Tensor& b, const at::Tensor& scale, const at::Tensor& shift,
                        const at::Tensor& alpha, int64_t Mp, int64_t Cp) {
  for (auto* p : {&x, &rs, &mask, &W, &b, &scale, &shift, &alpha}) check_f32_cuda(*p, "gcn_node_fwd input");
  TORCH_CHECK(bits.is_cuda() && bits.scalar_type() == at::kInt && bits.is_contiguous(), "gcn_node_fwd: bits");
  NodeGeom g = node_geom(x, bits, W);
  TORCH_CHECK(Mp >= (long)g.B * g.N && Mp % 16 == 0, "gcn_node_fwd: Mp must cover B*N rows, multiple of 16");
  TORCH_CHECK(Cp >= g.F + g.Cin, "gcn_node_fwd: Cp too small");
  TORCH_CHECK(rs.numel() == (long)g.B * g.N && mask.numel() == (long)g.B * g.N, "gcn_node_fwd: rs/mask shape");
  c10::DeviceGuard guard(x.device());
  at::Tensor out = at::empty({g.T, Mp, Cp}, x.options());
  const bool vec = g.F % 4 == 0 && Cp % 4 == 0;
  GQ_NODE_CIN_DISPATCH(g.Cin, GQ_NODE_V_DISPATCH(vec,
      allow_smem(gcn_node_fwd_kernel<CIN, VV>, g.smem);
      hipLaunchKernelGGL((gcn_node_fwd_kernel<CIN, VV>), g.grid, dim3(256), g.smem, stream(), x.data_ptr<float>(),
                         reinterpret_cast<const unsigned*>(bits.data_ptr<int>()), rs.data_ptr<float>(),
                         mask.data_ptr<float>(), W.data_ptr<float>(), b.data_ptr<float>(), scale.data_ptr<float>(),
                         shift.data_ptr<float>(), alpha.data_ptr<float>(), out.data_ptr<float>(), g.B, g.T, g.N, g.F,
                         (int)Cp, (int)Mp, g.NWd, g.tchunk)));
  GQ_LAUNCH_CHECK();
  return out;
}

// returns acc [3 + Cin, F] (fixed-order sum of per-workgroup partials)
at::Tensor gcn_node_bwd(const at::Tensor& x, const at::Tensor& bitsT, const at::Tensor& rs, const at::Tensor& mask,
                        const at::Tensor& dout, const at::Tensor& W, const at::Tensor& b, const at::Tensor& scale,
                        const at::Tensor& shift, const at::Tensor& alpha) {
  for (auto* p : {&x, &rs, &mask, &dout, &W, &b, &scale, &shift, &alpha}) check_f32_cuda(*p, "gcn_node_bwd input");
  NodeGeom g = node_geom(x, bitsT, W, 4);
  TORCH_CHECK(dout.dim() == 3 && dout.size(0) == g.T && dout.size(1) >= (long)g.B * g.N && dout.size(2) >= g.F + g.Cin,
              "gcn_node_bwd: dout must be [T, Mp, Cp]");
  c10::DeviceGuard guard(x.device());
  const int nacc = 3 + g.Cin;
  at::Tensor partial = at::empty({(long)g.grid.x * g.grid.y, nacc, g.F}, x.options());
  const bool vec = g.F % 4 == 0 && dout.size(2) % 4 == 0 && dout.stride(1) == dout.size(2) &&
                   (reinterpret_cast<uintptr_t>(dout.data_ptr()) % 16) == 0;
  GQ_NODE_CIN_DISPATCH(g.Cin, GQ_NODE_V_DISPATCH(vec,
      allow_smem(gcn_node_bwd_kernel<CIN, VV>, g.smem);
      hipLaunchKernelGGL((gcn_node_bwd_kernel<CIN, VV>), g.grid, dim3(256), g.smem, stream(), x.data_ptr<float>(),
                         reinterpret_cast<const unsigned*>(bitsT.data_ptr<int>()), rs.data_ptr<float>(),
                         mask.data_ptr<float>(), dout.data_ptr<float>(), W.data_ptr<float>(), b.data_ptr<float>(),
                         scale.data_ptr<float>(), shift.data_ptr<float>(), alpha.data_ptr<float>(),
                         partial.data_ptr<float>(), g.B, g.T, g.N, g.F, (int)dout.size(2), (int)dout.size(1), g.NWd,
                         g.tchunk)));
  GQ_LAUNCH_CHECK();
  return partial;      // [blocks, 3+Cin, F]: gcn_bwd_finalize sums the blocks (fixed order)
}

at::Tensor gcn_node_bwd_input(const at::Tensor& x, const at::Tensor& bitsT, const at::Tensor& rs,
                              const at::Tensor& mask, const at::Tensor& dout, const at::Tensor& W, const at::Tensor& b,
                              const at::Tensor& scale, const at::Tensor& shift, const at::Tensor& alpha,
                              const at::Tensor& coef) {
  for (auto* p : {&x, &rs, &mask, &dout, &W, &b, &scale, &shift, &alpha, &coef})
    check_f32_cuda(*p, "gcn_node_bwd_input input");
  NodeGeom g = node_geom(x, bitsT, W);
  TORCH_CHECK(coef.numel() == 3 * g.F, "gcn_node_bwd_input: coef must be [3,F]");
  TORCH_CHECK(dout.dim() == 3 && dout.size(0) == g.T && dout.size(1) >= (long)g.B * g.N && dout.size(2) >= g.F + g.Cin,
              "gcn_node_bwd_input: dout must be [T, Mp, Cp]");
  c10::DeviceGuard guard(x.device());
  at::Tensor dx = at::empty_like(x);
  GQ_NODE_CIN_DISPATCH(g.Cin,
      allow_smem(gcn_node_bwd_input_kernel<CIN>, g.smem);
      hipLaunchKernelGGL(gcn_node_bwd_input_kernel<CIN>, g.grid, dim3(256), g.smem, stream(), x.data_ptr<float>(),
                         reinterpret_cast<const unsigned*>(bitsT.data_ptr<int>()), rs.data_ptr<float>(),
                         mask.data_ptr<float>(), dout.data_ptr<float>(), W.data_ptr<float>(), b.data_ptr<float>(),
                         scale.data_ptr<float>(), shift.data_ptr<float>(), alpha.data_ptr<float>(),
                         coef.data_ptr<float>(), dx.data_ptr<float>(), g.B, g.T, g.N, g.F, (int)dout.size(2),
                         (int)dout.size(1), g.NWd, g.tchunk));
  GQ_LAUNCH_CHECK();
  return dx;
}

}  // namespace gq

TORCH_LIBRARY_IMPL(gnnqc, CUDA, m) {
  m.impl("gcn_adj_bits", &gq::gcn_adj_bits);
  m.impl("gcn_node_fwd", &gq::gcn_node_fwd);
  m.impl("gcn_node_bwd", &gq::gcn_node_bwd);
  m.impl("gcn_node_bwd_input", &gq::gcn_node_bwd_input);
}
