// Fused classifier head + weighted BCE + metric accumulation (forward) and its
// backward, for gfx950.
//
// Reference: the Keras head Dense(64) -> LeakyReLU(.3) -> Dense(64) -> LeakyReLU(.3)
// -> Dense(1, sigmoid) (libs/create_model.py:204-239, :356-376), compiled with
// binary_crossentropy + class_weight (libs/fit_model.py:76-111) and the metric list
// Recall/BinaryAccuracy/Precision/AUC/TP/FP/TN/FN (:79-86).
//
// On the eager path this is ~50 launches of 1-5 us each per training step (GEMMs
// with 128 rows, bias adds, activations, BCE pieces, metric reductions, histogram).
// Here: ONE forward kernel (activations, logits, loss, confusion counts, score
// histogram) and ONE backward kernel (all weight gradients + d features).
//
// Layout: rows are tiled by 64; 256 threads = 4 waves; thread (j = tid & 63,
// g = tid >> 6) owns output column j of rows g*RPG .. g*RPG+RPG-1. Input tiles and
// activations live in LDS; inner products read LDS with wave-uniform addresses
// (broadcast, conflict free) and weights with lane-contiguous addresses. The
// backward kernel is persistent over row tiles and keeps its weight-gradient
// partials in registers, flushing them once per block with coalesced atomics
// straight into the optimiser's flat gradient buffer (or a zeroed sink).
#include "common.h"

namespace gq {

int* chain_ctl(int dev);   // lstm_chain.hip: the device's chain control words

constexpr int HT = 16;     // rows per tile: 8 workgroups for a CML batch of 128 (LDS-bound loops
                           // spread over 8 CUs; 64-row tiles left 2 CUs doing 4x the work each)
constexpr int HU = 64;     // dense units (model_config dense.units)
constexpr int RPG = HT / 4;  // rows per wave group
constexpr int UPG = HU / 4;  // dense units per wave group (dW2 rows per thread)
constexpr int HEAD_HIST_LDS = 1024;   // score-histogram bins aggregated in LDS (engine: 1001)

__device__ __forceinline__ float leaky(float z, float a) { return z > 0.f ? z : a * z; }
__device__ __forceinline__ float dleaky(float z, float a) { return z > 0.f ? 1.f : a; }

// Copy N floats (N % 1024 == 0) global -> LDS rows of pitch P: every thread issues all of
// its float4 loads before the first LDS store, so the copy costs one memory latency.
template <int N, int COLS, int P>
__device__ __forceinline__ void stage_lds(float* __restrict__ dst, const float* __restrict__ src) {
  constexpr int PER = N / 4 / 256;
  static_assert(N % 1024 == 0 && COLS % 4 == 0, "stage_lds shape");
  float4 v[PER];
#pragma unroll
  for (int i = 0; i < PER; ++i) v[i] = reinterpret_cast<const float4*>(src)[threadIdx.x + 256 * i];
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int e = 4 * (threadIdx.x + 256 * i), r = e / COLS, c = e % COLS;
    float* d = dst + r * P + c;
    if constexpr (P % 4 == 0) {
      *reinterpret_cast<float4*>(d) = v[i];
    } else {
      d[0] = v[i].x; d[1] = v[i].y; d[2] = v[i].z; d[3] = v[i].w;
    }
  }
}

// mask sum over all rows (every block recomputes it: no cross-block dependency)
__device__ float block_mask_sum(const float* __restrict__ mask, int R, float* red) {
  // 8 independent loads in flight per thread (large R, e.g. SoilNet's 6,688 node rows: a
  // one-load-per-iteration loop paid one memory latency per 256 rows)
  float s = 0.f;
  int i = threadIdx.x;
  for (; i + 7 * 256 < R; i += 8 * 256) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = mask[i + 256 * u];
#pragma unroll
    for (int u = 0; u < 8; ++u) s += v[u];
  }
  for (; i < R; i += 256) s += mask[i];
  s = wave_sum(s);
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[w] = s;
  __syncthreads();
  s = red[0] + red[1] + red[2] + red[3];
  __syncthreads();
  return s;
}

// PROB (frozen-weight attribution, e.g. integrated gradients): logits[r] receives sigmoid(z_r), no
// loss, metrics or histogram (y, mask, aux, sums, hist unused)
template <int F, bool PROB = false>
__global__ __launch_bounds__(256) void head_fwd_kernel(
    const float* __restrict__ feat, int ldf, const float* __restrict__ W1, const float* __restrict__ b1,
    const float* __restrict__ W2, const float* __restrict__ b2, const float* __restrict__ W3,
    const float* __restrict__ b3, const float* __restrict__ y, const float* __restrict__ mask, int R,
    float alpha1, float alpha2, float w0, float w1, float* __restrict__ z1o, float* __restrict__ z2o,
    float* __restrict__ logits, float* __restrict__ aux, double* __restrict__ sums, float* __restrict__ hist,
    int bins) {
  __shared__ float sf[HT][F + 4];
  __shared__ float sW1[F][HU];
  __shared__ float sW2[HU][HU];
  __shared__ float sa1[HT][HU + 4];
  __shared__ float sa2[HT][HU + 4];
  __shared__ float red[4];
  __shared__ float mred[4][8];
  // the workgroup's score histogram, flushed with one global atomic per non-empty bin: per-row
  // global atomics all landed on the same few bins (an untrained model scores every node ~0.5)
  // and serialised - SoilNet's 6,688 node rows per step made this kernel ~50 us
  __shared__ float shist[2 * HEAD_HIST_LDS];
  const bool lds_hist = hist != nullptr && bins <= HEAD_HIST_LDS;
  const int tid = threadIdx.x, j = tid & 63, g = tid >> 6;
  if (lds_hist)
    for (int e = tid; e < 2 * bins; e += 256) shist[e] = 0.f;
  stage_lds<F * HU, HU, HU>(&sW1[0][0], W1);
  stage_lds<HU * HU, HU, HU>(&sW2[0][0], W2);
  const float bj1 = b1[j], bj2 = b2[j], w3 = W3[j], b3v = b3[0];
  const float nm = PROB ? 0.f : block_mask_sum(mask, R, red);
  const float inv = 1.f / fmaxf(nm, 1.f);
  if (!PROB && blockIdx.x == 0 && tid == 0) aux[1] = nm;
  float m_loss = 0.f, m_n = 0.f, m_tp = 0.f, m_tn = 0.f, m_fp = 0.f, m_fn = 0.f;
  const int ntiles = (R + HT - 1) / HT;
  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int row0 = tile * HT;
    // stage the feature tile (float4; rows past R are zero)
    for (int e = tid; e < HT * (F / 4); e += 256) {
      const int r = e / (F / 4), c4 = e % (F / 4);
      // clamped row + 0/1 scale instead of a guarded load (a branch around a load makes
      // hipcc drain vmcnt at the join)
      const float m_ = row0 + r < R ? 1.f : 0.f;
      float4 v = *reinterpret_cast<const float4*>(feat + (long)min(row0 + r, R - 1) * ldf + 4 * c4);
      v.x *= m_; v.y *= m_; v.z *= m_; v.w *= m_;
      *reinterpret_cast<float4*>(&sf[r][4 * c4]) = v;
    }
    __syncthreads();
    float acc[RPG];
    const float bj1 = b1[j];
#pragma unroll
    for (int i = 0; i < RPG; ++i) acc[i] = bj1;
    #pragma unroll 4
    for (int k = 0; k < F; ++k) {
      const float w = sW1[k][j];
#pragma unroll
      for (int i = 0; i < RPG; ++i) acc[i] += sf[g * RPG + i][k] * w;
    }
#pragma unroll
    for (int i = 0; i < RPG; ++i) {
      const int r = g * RPG + i;
      if (row0 + r < R) z1o[(long)(row0 + r) * HU + j] = acc[i];
      sa1[r][j] = leaky(acc[i], alpha1);
    }
    __syncthreads();
    const float bj2 = b2[j];
#pragma unroll
    for (int i = 0; i < RPG; ++i) acc[i] = bj2;
    #pragma unroll 4
    for (int k = 0; k < HU; ++k) {
      const float w = sW2[k][j];
#pragma unroll
      for (int i = 0; i < RPG; ++i) acc[i] += sa1[g * RPG + i][k] * w;
    }
#pragma unroll
    for (int i = 0; i < RPG; ++i) {
      const int r = g * RPG + i;
      if (row0 + r < R) z2o[(long)(row0 + r) * HU + j] = acc[i];
      sa2[r][j] = leaky(acc[i], alpha2);
    }
    __syncthreads();
    // output unit: wave g reduces its RPG rows; lane i < RPG keeps row g*RPG+i
    float zr = 0.f;
#pragma unroll
    for (int i = 0; i < RPG; ++i) {
      const float v = wave_sum(sa2[g * RPG + i][j] * w3);
      if (j == i) zr = v;
    }
    if constexpr (PROB) {
      const int row = row0 + g * RPG + (j % RPG);
      if (j < RPG && row < R) logits[row] = sigmoidf_fast(zr + b3v);
    } else {
      const int row = row0 + g * RPG + (j % RPG);
      const int rc = min(row, R - 1);
      const float yy_ = y[rc], m_ = mask[rc];        // loads outside any per-lane branch
      if (j < RPG && row < R) {
        const float z = zr + b3v;
        logits[row] = z;
        const float yy = yy_, m = m_;
        const float l = fmaxf(z, 0.f) - z * yy + log1pf(__expf(-fabsf(z)));
        const float wc = yy > 0.5f ? w1 : w0;
        m_loss += m * wc * l;
        m_n += m;
        const float p = sigmoidf_fast(z);
        const bool pos = yy > 0.5f, pp = p > 0.5f;
        m_tp += (pp && pos) ? m : 0.f;
        m_tn += (!pp && !pos) ? m : 0.f;
        m_fp += (pp && !pos) ? m : 0.f;
        m_fn += (!pp && pos) ? m : 0.f;
        if (hist != nullptr && m != 0.f) {
          int b = (int)rintf(fminf(fmaxf(p, 0.f), 1.f) * (float)(bins - 1));
          b = b < 0 ? 0 : (b >= bins ? bins - 1 : b);
          if (lds_hist) atomicAdd(&shist[(pos ? bins : 0) + b], m);
          else atomicAdd(&hist[(pos ? bins : 0) + b], m);
        }
      }
    }
    __syncthreads();
  }
  if constexpr (PROB) return;
  if (lds_hist)
    for (int e = tid; e < 2 * bins; e += 256)
      if (shist[e] != 0.f) atomicAdd(&hist[e], shist[e]);
  // block reduction of the loss / metric partials (lanes >= RPG hold zeros)
  float v[6] = {m_loss, m_n, m_tp, m_tn, m_fp, m_fn};
#pragma unroll
  for (int q = 0; q < 6; ++q) v[q] = wave_sum(v[q]);
  if (j == 0) {
#pragma unroll
    for (int q = 0; q < 6; ++q) mred[g][q] = v[q];
  }
  __syncthreads();
  if (tid == 0) {
    float t[6];
#pragma unroll
    for (int q = 0; q < 6; ++q) t[q] = mred[0][q] + mred[1][q] + mred[2][q] + mred[3][q];
    atomicAdd(&aux[0], t[0] * inv);
    if (sums != nullptr) {
      for (int q = 0; q < 6; ++q) atomicAdd(&sums[q], (double)t[q]);
    }
  }
}

// Backward. gout: device scalar dL/dloss; aux[1]: mask sum from the forward.
// PROB: the input gradient of sum_r sigmoid(z_r) (logits holds the forward's sigmoid(z)):
// dz3_r = s_r (1 - s_r); no weight gradients (gout, aux, y, mask and the gradient sinks unused)
template <int F, bool PROB = false>
__global__ __launch_bounds__(256) void head_bwd_kernel(
    const float* __restrict__ feat, int ldf, const float* __restrict__ W1, const float* __restrict__ W2,
    const float* __restrict__ W3, const float* __restrict__ z1, const float* __restrict__ z2,
    const float* __restrict__ logits, const float* __restrict__ y, const float* __restrict__ mask, int R,
    float alpha1, float alpha2, float w0, float w1, const float* __restrict__ gout, const float* __restrict__ aux,
    float* __restrict__ dfeat, int ldd, float* __restrict__ dW1, float* __restrict__ db1, float* __restrict__ dW2,
    float* __restrict__ db2, float* __restrict__ dW3, float* __restrict__ db3, int* __restrict__ nf) {
  constexpr int KPT = F / 4;            // dW1 rows per thread
  constexpr int RPT = HT * F / 256;     // dfeat rows per thread
  __shared__ float sf[HT][F + 4];
  __shared__ float sW1[F][HU + 1];
  __shared__ float sW2[HU][HU + 1];
  __shared__ float sa1[HT][HU + 4];      // a1 = leaky(z1)
  __shared__ float sz1[HT][HU + 4];      // z1, then dz1
  __shared__ float sz2[HT][HU + 4];      // z2, then dz2
  __shared__ float sdz3[HT];
  __shared__ float red[4][HU + 1];
  const int tid = threadIdx.x, j = tid & 63, g = tid >> 6;
  const float scale = PROB ? 1.f : gout[0] / fmaxf(aux[1], 1.f);
  stage_lds<F * HU, HU, HU + 1>(&sW1[0][0], W1);
  stage_lds<HU * HU, HU, HU + 1>(&sW2[0][0], W2);
  const float w3j = W3[j];
  float aW1[KPT], aW2[UPG], aW3 = 0.f, ab1 = 0.f, ab2 = 0.f, ab3 = 0.f;
#pragma unroll
  for (int q = 0; q < KPT; ++q) aW1[q] = 0.f;
#pragma unroll
  for (int q = 0; q < UPG; ++q) aW2[q] = 0.f;
  const int ntiles = (R + HT - 1) / HT;
  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int row0 = tile * HT;
    for (int e = tid; e < HT * (F / 4); e += 256) {
      const int r = e / (F / 4), c4 = e % (F / 4);
      // clamped row + 0/1 scale instead of a guarded load (a branch around a load makes
      // hipcc drain vmcnt at the join)
      const float m_ = row0 + r < R ? 1.f : 0.f;
      float4 v = *reinterpret_cast<const float4*>(feat + (long)min(row0 + r, R - 1) * ldf + 4 * c4);
      v.x *= m_; v.y *= m_; v.z *= m_; v.w *= m_;
      *reinterpret_cast<float4*>(&sf[r][4 * c4]) = v;
    }
#pragma unroll
    for (int i = 0; i < RPG; ++i) {
      const int r = g * RPG + i, row = row0 + r;
      const float rm = row < R ? 1.f : 0.f;
      const float a = z1[(long)min(row, R - 1) * HU + j] * rm;
      const float b = z2[(long)min(row, R - 1) * HU + j] * rm;
      sz1[r][j] = a;
      sa1[r][j] = leaky(a, alpha1);
      sz2[r][j] = b;
    }
    {
      const int row = row0 + (tid & (HT - 1));
      const int rc = min(row, R - 1);
      float d;
      if constexpr (PROB) {
        const float sp = logits[rc];
        d = (row < R ? 1.f : 0.f) * sp * (1.f - sp);
      } else {
        const float yy = y[rc];
        const float wc = yy > 0.5f ? w1 : w0;
        d = (row < R ? 1.f : 0.f) * scale * mask[rc] * wc * (sigmoidf_fast(logits[rc]) - yy);
      }
      if (tid < HT) {             // LDS / register only inside the branch
        sdz3[tid] = d;
        ab3 += d;
      }
    }
    __syncthreads();
    // dW3 / db... and dz2 = dz3 * W3 * leaky'(z2) (in place)
#pragma unroll
    for (int i = 0; i < RPG; ++i) {
      const int r = g * RPG + i;
      const float z = sz2[r][j], d3 = sdz3[r];
      aW3 += leaky(z, alpha2) * d3;
      sz2[r][j] = d3 * w3j * dleaky(z, alpha2);
    }
    __syncthreads();
    // dW2[i][j] = sum_r a1[r][i] dz2[r][j] ; db2 ; da1 -> dz1
    if constexpr (!PROB) {
      #pragma unroll 4
      for (int r = 0; r < HT; ++r) {
        const float d = sz2[r][j];
#pragma unroll
        for (int q = 0; q < UPG; ++q) aW2[q] += sa1[r][g * UPG + q] * d;
        if (g == 0) ab2 += d;
      }
    }
    float da[RPG];
#pragma unroll
    for (int q = 0; q < RPG; ++q) da[q] = 0.f;
    // thread owns unit i = j of rows g*RPG..: da1[r][i] = sum_k dz2[r][k] W2[i][k]
    #pragma unroll 4
    for (int k = 0; k < HU; ++k) {
      const float w = sW2[j][k];
#pragma unroll
      for (int q = 0; q < RPG; ++q) da[q] += sz2[g * RPG + q][k] * w;
    }
    __syncthreads();     // all reads of sz1 (raw z1) by other threads are per-owner: safe, but sz2 reads end here
#pragma unroll
    for (int q = 0; q < RPG; ++q) {
      const int r = g * RPG + q;
      sz1[r][j] = da[q] * dleaky(sz1[r][j], alpha1);
    }
    __syncthreads();
    // dW1[k][j] = sum_r feat[r][k] dz1[r][j] ; db1
    if constexpr (!PROB) {
      #pragma unroll 4
      for (int r = 0; r < HT; ++r) {
        const float d = sz1[r][j];
#pragma unroll
        for (int q = 0; q < KPT; ++q) aW1[q] += sf[r][g * KPT + q] * d;
        if (g == 0) ab1 += d;
      }
    }
    // dfeat[r][k] = sum_j dz1[r][j] W1[k][j]
    if (dfeat != nullptr) {
      const int k = tid % F, rg = tid / F;
      float o[RPT];
#pragma unroll
      for (int q = 0; q < RPT; ++q) o[q] = 0.f;
      #pragma unroll 4
      for (int jj = 0; jj < HU; ++jj) {
        const float w = sW1[k][jj];
#pragma unroll
        for (int q = 0; q < RPT; ++q) o[q] += sz1[rg * RPT + q][jj] * w;
      }
#pragma unroll
      for (int q = 0; q < RPT; ++q) {
        const int row = row0 + rg * RPT + q;
        if (row < R) dfeat[(long)row * ldd + k] = o[q];
      }
    }
    __syncthreads();
  }
  if constexpr (PROB) return;
  // flush: coalesced atomics (lanes = consecutive j); a non-finite partial raises the flag the
  // flag-driven Adam decides from (chain control word 7)
  bool fin = isfinite(aW3) && isfinite(ab1) && isfinite(ab2) && isfinite(ab3);
#pragma unroll
  for (int q = 0; q < KPT; ++q) {
    fin = fin && isfinite(aW1[q]);
    atomicAdd(&dW1[(g * KPT + q) * HU + j], aW1[q]);
  }
#pragma unroll
  for (int q = 0; q < UPG; ++q) {
    fin = fin && isfinite(aW2[q]);
    atomicAdd(&dW2[(g * UPG + q) * HU + j], aW2[q]);
  }
  if (!fin && nf != nullptr) __hip_atomic_store(nf, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  red[g][j] = aW3;
  __syncthreads();
  if (g == 0) {
    atomicAdd(&dW3[j], red[0][j] + red[1][j] + red[2][j] + red[3][j]);
    atomicAdd(&db1[j], ab1);
    atomicAdd(&db2[j], ab2);
    const float s3 = wave_sum(ab3);
    if (j == 0) atomicAdd(&db3[0], s3);
  }
}

// backward: persistent over at most 256 tiles (each workgroup flushes its weight-gradient
// partials once with atomics); forward: one tile per workgroup up to 512 (two 66 KB-LDS
// workgroups per CU: SoilNet's 418 node-row tiles run in one round instead of two)
static int head_grid(int R, bool fwd = false) {
  const int nt = (R + HT - 1) / HT;
  return deterministic_mode() ? 1 : std::max(1, std::min(nt, fwd ? 512 : 256));
}

#define GQ_HEAD_F_DISPATCH(F_, ...)                                 \
  switch (F_) {                                                      \
    case 32: { constexpr int FF = 32; __VA_ARGS__; break; }          \
    case 64: { constexpr int FF = 64; __VA_ARGS__; break; }          \
    case 128: { constexpr int FF = 128; __VA_ARGS__; break; }        \
    default: TORCH_CHECK(false, "gnnqc head: feature width must be 32, 64 or 128, got ", F_); \
  }

// returns [z1 (R,64), z2 (R,64), logits (R), aux (2): loss, mask-sum]
std::vector<at::Tensor> head_fwd(const at::Tensor& feat, const at::Tensor& W1, const at::Tensor& b1,
                                 const at::Tensor& W2, const at::Tensor& b2, const at::Tensor& W3,
                                 const at::Tensor& b3, const at::Tensor& y, const at::Tensor& mask, double alpha1,
                                 double alpha2, double w0, double w1, at::Tensor sums, at::Tensor hist) {
  TORCH_CHECK(feat.is_cuda() && feat.scalar_type() == at::kFloat && feat.dim() == 2 && feat.stride(1) == 1,
              "gnnqc head: feat must be a float32 GPU matrix with unit inner stride");
  const int R = (int)feat.size(0), F = (int)feat.size(1);
  TORCH_CHECK(feat.stride(0) % 4 == 0 && reinterpret_cast<uintptr_t>(feat.data_ptr()) % 16 == 0,
              "gnnqc head: feat rows must be 16-byte aligned");
  const at::Tensor* ops[] = {&W1, &b1, &W2, &b2, &W3, &b3, &y, &mask};
  for (const at::Tensor* t : ops) check_f32_cuda(*t, "head operand");
  TORCH_CHECK(W1.size(0) == F && W1.size(1) == HU && W2.size(0) == HU && W2.size(1) == HU &&
                  W3.numel() == HU && b1.numel() == HU && b2.numel() == HU && b3.numel() == 1,
              "gnnqc head: expected Dense(F,64)-Dense(64,64)-Dense(64,1)");
  TORCH_CHECK(y.numel() == R && mask.numel() == R, "gnnqc head: y/mask must have one entry per row");
  double* sp = nullptr;
  float* hp = nullptr;
  int bins = 2;
  if (sums.numel() > 0) {
    TORCH_CHECK(sums.is_cuda() && sums.scalar_type() == at::kDouble && sums.numel() == 6, "sums: 6 float64");
    sp = sums.data_ptr<double>();
  }
  if (hist.numel() > 0) {
    check_f32_cuda(hist, "hist");
    TORCH_CHECK(hist.dim() == 2 && hist.size(0) == 2, "hist must be [2, bins]");
    hp = hist.data_ptr<float>();
    bins = (int)hist.size(1);
  }
  c10::DeviceGuard guard(feat.device());
  auto opt = feat.options();
  at::Tensor z1 = at::empty({R, HU}, opt), z2 = at::empty({R, HU}, opt), lo = at::empty({R}, opt);
  at::Tensor aux = at::zeros({2}, opt);
  const int grid = head_grid(R, true);
  GQ_HEAD_F_DISPATCH(F, hipLaunchKernelGGL(head_fwd_kernel<FF>, dim3(grid), dim3(256), 0, stream(),
                                           feat.data_ptr<float>(), (int)feat.stride(0), W1.data_ptr<float>(),
                                           b1.data_ptr<float>(), W2.data_ptr<float>(), b2.data_ptr<float>(),
                                           W3.data_ptr<float>(), b3.data_ptr<float>(), y.data_ptr<float>(),
                                           mask.data_ptr<float>(), R, (float)alpha1, (float)alpha2, (float)w0,
                                           (float)w1, z1.data_ptr<float>(), z2.data_ptr<float>(),
                                           lo.data_ptr<float>(), aux.data_ptr<float>(), sp, hp, bins));
  GQ_LAUNCH_CHECK();
  return {z1, z2, lo, aux};
}

// Accumulates into dW1..db3 (which may be the optimiser's gradient views); returns dfeat.
at::Tensor head_bwd(const at::Tensor& feat, const at::Tensor& W1, const at::Tensor& W2, const at::Tensor& W3,
                    const at::Tensor& z1, const at::Tensor& z2, const at::Tensor& logits, const at::Tensor& y,
                    const at::Tensor& mask, double alpha1, double alpha2, double w0, double w1, const at::Tensor& gout,
                    const at::Tensor& aux, at::Tensor dW1, at::Tensor db1, at::Tensor dW2, at::Tensor db2,
                    at::Tensor dW3, at::Tensor db3, bool need_dfeat) {
  const int R = (int)feat.size(0), F = (int)feat.size(1);
  TORCH_CHECK(feat.stride(1) == 1 && feat.stride(0) % 4 == 0, "gnnqc head_bwd: feat layout");
  const at::Tensor* ops[] = {&W1, &W2, &W3, &z1, &z2, &logits, &y, &mask, &gout, &aux, &dW1, &db1, &dW2, &db2,
                             &dW3, &db3};
  for (const at::Tensor* t : ops) check_f32_cuda(*t, "head_bwd operand");
  TORCH_CHECK(z1.size(0) == R && z2.size(0) == R && logits.numel() == R, "gnnqc head_bwd: saved tensor rows");
  TORCH_CHECK(dW1.numel() == (long)F * HU && dW2.numel() == HU * HU && dW3.numel() == HU && db1.numel() == HU &&
                  db2.numel() == HU && db3.numel() == 1, "gnnqc head_bwd: gradient shapes");
  c10::DeviceGuard guard(feat.device());
  at::Tensor dfeat = need_dfeat ? at::empty({R, F}, feat.options()) : at::empty({0}, feat.options());
  const int grid = head_grid(R);
  GQ_HEAD_F_DISPATCH(F, hipLaunchKernelGGL(head_bwd_kernel<FF>, dim3(grid), dim3(256), 0, stream(),
                                           feat.data_ptr<float>(), (int)feat.stride(0), W1.data_ptr<float>(),
                                           W2.data_ptr<float>(), W3.data_ptr<float>(), z1.data_ptr<float>(),
                                           z2.data_ptr<float>(), logits.data_ptr<float>(), y.data_ptr<float>(),
                                           mask.data_ptr<float>(), R, (float)alpha1, (float)alpha2, (float)w0,
                                           (float)w1, gout.data_ptr<float>(), aux.data_ptr<float>(),
                                           need_dfeat ? dfeat.data_ptr<float>() : nullptr, F,
                                           dW1.data_ptr<float>(), db1.data_ptr<float>(), dW2.data_ptr<float>(),
                                           db2.data_ptr<float>(), dW3.data_ptr<float>(), db3.data_ptr<float>(),
                                           chain_ctl(feat.get_device()) + 7));
  GQ_LAUNCH_CHECK();
  return dfeat;
}

// Frozen-weight head for attribution: [z1 (R,64), z2 (R,64), prob (R) = sigmoid(logit)]
std::vector<at::Tensor> head_prob_fwd(const at::Tensor& feat, const at::Tensor& W1, const at::Tensor& b1,
                                      const at::Tensor& W2, const at::Tensor& b2, const at::Tensor& W3,
                                      const at::Tensor& b3, double alpha1, double alpha2) {
  TORCH_CHECK(feat.is_cuda() && feat.scalar_type() == at::kFloat && feat.dim() == 2 && feat.stride(1) == 1 &&
                  feat.stride(0) % 4 == 0 && reinterpret_cast<uintptr_t>(feat.data_ptr()) % 16 == 0,
              "gnnqc head_prob_fwd: feat must be a float32 GPU matrix with 16-byte aligned rows");
  const int R = (int)feat.size(0), F = (int)feat.size(1);
  const at::Tensor* ops[] = {&W1, &b1, &W2, &b2, &W3, &b3};
  for (const at::Tensor* t : ops) check_f32_cuda(*t, "head operand");
  TORCH_CHECK(R >= 1 && W1.size(0) == F && W1.size(1) == HU && W2.size(0) == HU && W2.size(1) == HU &&
                  W3.numel() == HU && b1.numel() == HU && b2.numel() == HU && b3.numel() == 1,
              "gnnqc head_prob_fwd: expected Dense(F,64)-Dense(64,64)-Dense(64,1)");
  c10::DeviceGuard guard(feat.device());
  auto opt = feat.options();
  at::Tensor z1 = at::empty({R, HU}, opt), z2 = at::empty({R, HU}, opt), pr = at::empty({R}, opt);
  const int grid = head_grid(R, true);
  GQ_HEAD_F_DISPATCH(F, hipLaunchKernelGGL((head_fwd_kernel<FF, true>), dim3(grid), dim3(256), 0, stream(),
                                           feat.data_ptr<float>(), (int)feat.stride(0), W1.data_ptr<float>(),
                                           b1.data_ptr<float>(), W2.data_ptr<float>(), b2.data_ptr<float>(),
                                           W3.data_ptr<float>(), b3.data_ptr<float>(), nullptr, nullptr, R,
                                           (float)alpha1, (float)alpha2, 0.f, 0.f, z1.data_ptr<float>(),
                                           z2.data_ptr<float>(), pr.data_ptr<float>(), nullptr, nullptr, nullptr, 2));
  GQ_LAUNCH_CHECK();
  return {z1, z2, pr};
}

// d sum_r sigmoid(z_r) / d feat of head_prob_fwd's rows (no weight gradients)
at::Tensor head_prob_bwd(const at::Tensor& feat, const at::Tensor& W1, const at::Tensor& W2, const at::Tensor& W3,
                         const at::Tensor& z1, const at::Tensor& z2, const at::Tensor& prob, double alpha1,
                         double alpha2) {
  const int R = (int)feat.size(0), F = (int)feat.size(1);
  TORCH_CHECK(feat.is_cuda() && feat.scalar_type() == at::kFloat && feat.stride(1) == 1 && feat.stride(0) % 4 == 0 &&
                  reinterpret_cast<uintptr_t>(feat.data_ptr()) % 16 == 0, "gnnqc head_prob_bwd: feat layout");
  const at::Tensor* ops[] = {&W1, &W2, &W3, &z1, &z2, &prob};
  for (const at::Tensor* t : ops) check_f32_cuda(*t, "head_prob_bwd operand");
  TORCH_CHECK(z1.size(0) == R && z2.size(0) == R && prob.numel() == R && W1.size(0) == F && W1.size(1) == HU &&
                  W2.numel() == HU * HU && W3.numel() == HU, "gnnqc head_prob_bwd: shapes");
  c10::DeviceGuard guard(feat.device());
  at::Tensor dfeat = at::empty({R, F}, feat.options());
  const int grid = head_grid(R);
  GQ_HEAD_F_DISPATCH(F, hipLaunchKernelGGL((head_bwd_kernel<FF, true>), dim3(grid), dim3(256), 0, stream(),
                                           feat.data_ptr<float>(), (int)feat.stride(0), W1.data_ptr<float>(),
                                           W2.data_ptr<float>(), W3.data_ptr<float>(), z1.data_ptr<float>(),
                                           z2.data_ptr<float>(), prob.data_ptr<float>(), nullptr, nullptr, R,
                                           (float)alpha1, (float)alpha2, 0.f, 0.f, nullptr, nullptr,
                                           dfeat.data_ptr<float>(), F, nullptr, nullptr, nullptr, nullptr, nullptr,
                                           nullptr, nullptr));
  GQ_LAUNCH_CHECK();
  return dfeat;
}

}  // namespace gq

TORCH_LIBRARY_IMPL(gnnqc, CUDA, m) {
  m.impl("head_fwd", &gq::head_fwd);
  m.impl("head_bwd", &gq::head_bwd);
  m.impl("head_prob_fwd", &gq::head_prob_fwd);
  m.impl("head_prob_bwd", &gq::head_prob_bwd);
}
