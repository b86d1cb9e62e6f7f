// Classifier head fused into the LSTM chain kernels (lstm_chain.hip), CML GCN.
//
// Reference: Dense(64) -> LeakyReLU(.3) -> Dense(64) -> LeakyReLU(.3) -> Dense(1, sigmoid) on the
// TimeLayer output (libs/create_model.py:204-239) trained with class-weighted binary
// cross-entropy, SUM_OVER_BATCH_SIZE (libs/fit_model.py:76-111), metrics :79-86.
//
// The head is tiny (16 rows x 128 -> 64 -> 64 -> 1 per tile) and the last chain stage (time4,
// H = 128) already holds its input rows in LDS, so instead of two more launches (head forward,
// head backward: 24 us per CML step, latency only) the work runs inside the chain kernels:
//   forward:  epilogue of the last stage's workgroups - logits, per-row loss, metric counts;
//             the workgroup that arrives last (ticket) sums the per-tile partials in tile
//             order (deterministic) into the loss and the metric accumulators.
//   backward: prologue of the first backward stage (time4) - recomputes the head forward of
//             its 16 rows, back-propagates dloss, leaves dh_{T-1} of time4 in LDS and writes the
//             tile's weight-gradient partials; the workgroup holding the last ticket sums them
//             in tile order after its own (6-step) recurrence and adds them to the gradients.
// Everything is fp32 on the FMA pipes (4 K FLOP per row: MFMA would not shorten the latency).
#pragma once
#include "common.h"

namespace gq {

constexpr int CH_HU = 64;              // Dense units (model_config dense.units)
constexpr int CH_AP = CH_HU + 4;       // activation tile pitch (floats)

struct ChainHead {
  const float *W1, *b1, *W2, *b2, *W3, *b3;   // W1 [F][64], W2 [64][64], W3 [64], b3 [1]
  const float *y, *mask;                      // [M]
  float* logits;                              // [M]
  float* part;                                // forward: [ntiles][8] per-tile partials
  float* loss;                                // forward: [1]
  double* sums;                               // MetricAccumulator [loss*n, n, tp, tn, fp, fn] (nullable)
  float* hist;                                // [2][bins] score histogram (nullable)
  int bins;
  int* ticket;                                // arrival counter (the last arrival re-arms it)
  int M;                                      // real rows (Mp - M padding rows are ignored)
  float alpha1, alpha2, w0, w1;
  // backward
  const float* hT;                            // time4 output at step T-1: [Mp][F]
  const float* dloss;                         // [1] dL/dloss
  float* gpart;                               // [ntiles][CH_NG] weight-gradient partials
  float *dW1, *db1, *dW2, *db2, *dW3, *db3;   // accumulated (+=): .grad views or zeroed sinks
};

// gradient record of one tile: dW1 [F*64] | db1 [64] | dW2 [64*64] | db2 [64] | dW3 [64] | db3 [1]
template <int F>
struct ChainHeadRec {
  static constexpr int N = F * CH_HU + CH_HU + CH_HU * CH_HU + CH_HU + CH_HU + 1;
  static constexpr int PITCH = (N + 3) / 4 * 4;
};

__device__ __forceinline__ float ch_leaky(float z, float a) { return z > 0.f ? z : a * z; }
__device__ __forceinline__ float ch_dleaky(float z, float a) { return z > 0.f ? 1.f : a; }

__device__ __forceinline__ float ch_load_acq(const float* p) {
  return __uint_as_float(__hip_atomic_load(reinterpret_cast<const unsigned*>(p), __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT));
}

// Sum of mask[0..M) over the 1024-thread workgroup (red: 16 floats of LDS).
__device__ __forceinline__ float ch_mask_sum(const float* __restrict__ mask, int M, float* red) {
  float s = 0.f;
  for (int i = threadIdx.x; i < M; i += 1024) s += mask[i];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  float t = 0.f;
#pragma unroll
  for (int k = 0; k < 16; ++k) t += red[k];
  return t;
}

// LDS bytes of the forward epilogue scratch
template <int F>
struct ChainHeadFwdLds {
  static constexpr int BYTES = (F * CH_HU + CH_HU * CH_HU + 16 * CH_AP + 16 * 8) * 4;
};

// Forward of the 16 rows of `tile` from hl [16][F + 4] (LDS). 1024 threads.
template <int F>
__device__ void chain_head_fwd(const ChainHead& hd, int tile, int ntiles, const float* hl, char* scratch) {
  constexpr int HLP = F + 4;
  float* sW1 = reinterpret_cast<float*>(scratch);     // [F][64]
  float* sW2 = sW1 + F * CH_HU;                       // [64][64]
  float* sa1 = sW2 + CH_HU * CH_HU;                   // [16][CH_AP]
  float* rowv = sa1 + 16 * CH_AP;                     // [16][8]
  const int tid = threadIdx.x, r = tid >> 6, j = tid & 63;
  constexpr int N1 = F * CH_HU / 4 / 1024;
  static_assert(F * CH_HU % 4096 == 0, "head W1 staging");
  float4 v1[N1];
#pragma unroll
  for (int i = 0; i < N1; ++i) v1[i] = reinterpret_cast<const float4*>(hd.W1)[tid + 1024 * i];
  const float4 v2 = reinterpret_cast<const float4*>(hd.W2)[tid];
  const float b1j = hd.b1[j], b2j = hd.b2[j], w3j = hd.W3[j], b3 = hd.b3[0];
  const int row = tile * 16 + r;
  const bool valid = row < hd.M;
  const int rc = min(row, hd.M - 1);
  const float yy = hd.y[rc], mm = hd.mask[rc];
#pragma unroll
  for (int i = 0; i < N1; ++i) reinterpret_cast<float4*>(sW1)[tid + 1024 * i] = v1[i];
  reinterpret_cast<float4*>(sW2)[tid] = v2;
  __syncthreads();
  float acc = b1j;
#pragma unroll 8
  for (int k = 0; k < F; ++k) acc += hl[r * HLP + k] * sW1[k * CH_HU + j];
  sa1[r * CH_AP + j] = ch_leaky(acc, hd.alpha1);
  __syncthreads();
  float acc2 = b2j;
#pragma unroll 8
  for (int k = 0; k < CH_HU; ++k) acc2 += sa1[r * CH_AP + k] * sW2[k * CH_HU + j];
  const float z = wave_sum(ch_leaky(acc2, hd.alpha2) * w3j) + b3;
  if (j == 0) {
    const float m = valid ? mm : 0.f;
    if (valid && hd.logits != nullptr) hd.logits[row] = z;
    const float l = fmaxf(z, 0.f) - z * yy + log1pf(__expf(-fabsf(z)));
    const float wc = yy > 0.5f ? hd.w1 : hd.w0;
    const float p = sigmoidf_fast(z);
    const bool pos = yy > 0.5f, pp = p > 0.5f;
    rowv[r * 8 + 0] = m * wc * l;
    rowv[r * 8 + 1] = m;
    rowv[r * 8 + 2] = (pp && pos) ? m : 0.f;
    rowv[r * 8 + 3] = (!pp && !pos) ? m : 0.f;
    rowv[r * 8 + 4] = (pp && !pos) ? m : 0.f;
    rowv[r * 8 + 5] = (!pp && pos) ? m : 0.f;
    if (hd.hist != nullptr && m != 0.f) {
      int b = (int)rintf(fminf(fmaxf(p, 0.f), 1.f) * (float)(hd.bins - 1));
      b = b < 0 ? 0 : (b >= hd.bins ? hd.bins - 1 : b);
      atomicAdd(&hd.hist[(pos ? hd.bins : 0) + b], m);
    }
  }
  __syncthreads();
  if (tid < 6) {
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) s += rowv[k * 8 + tid];
    hd.part[tile * 8 + tid] = s;
    __threadfence();
  }
  __syncthreads();
  if (tid == 0) {
    const int t = __hip_atomic_fetch_add(hd.ticket, 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (t == ntiles - 1) {              // every tile's partials are in: fixed-order sums
      double s[6] = {0, 0, 0, 0, 0, 0};
      for (int k = 0; k < ntiles; ++k)
        for (int q = 0; q < 6; ++q) s[q] += (double)ch_load_acq(hd.part + k * 8 + q);
      hd.loss[0] = (float)(s[0] / fmax(s[1], 1.0));
      if (hd.sums != nullptr)
        for (int q = 0; q < 6; ++q) hd.sums[q] += s[q];
      __hip_atomic_store(hd.ticket, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// LDS bytes of the backward prologue scratch (dh_{T-1} output tile excluded)
template <int F>
struct ChainHeadBwdLds {
  static constexpr int W1P = CH_HU + 1;     // odd pitches: row- and column-wise reads conflict free
  static constexpr int BYTES = (F * W1P + CH_HU * W1P + 16 * (F + 4) + 5 * 16 * CH_AP + 32) * 4;
};

// Backward of the head for the 16 rows of `tile`: dh_{T-1} -> dh [16][F + 4] (LDS), the tile's
// weight-gradient record -> hd.gpart[tile]. Returns (uniform) whether this workgroup took the
// last ticket, i.e. must reduce the records (chain_head_bwd_reduce) once all have been written.
template <int F>
__device__ bool chain_head_bwd(const ChainHead& hd, int tile, int ntiles, float* dh, char* scratch) {
  constexpr int W1P = ChainHeadBwdLds<F>::W1P, HLP = F + 4;
  using Rec = ChainHeadRec<F>;
  float* sW1 = reinterpret_cast<float*>(scratch);    // [F][W1P]
  float* sW2 = sW1 + F * W1P;                        // [64][W1P]
  float* sh = sW2 + CH_HU * W1P;                     // [16][HLP]
  float* sz1 = sh + 16 * HLP;                        // [16][CH_AP] z1
  float* sa1 = sz1 + 16 * CH_AP;                     // [16][CH_AP] leaky(z1)
  float* sz2 = sa1 + 16 * CH_AP;                     // [16][CH_AP] dz2
  float* sad = sz2 + 16 * CH_AP;                     // [16][CH_AP] leaky(z2) * d
  float* sdz1 = sad + 16 * CH_AP;                    // [16][CH_AP] dz1
  float* misc = sdz1 + 16 * CH_AP;                   // [32]: d per row, mask-sum reduction
  const int tid = threadIdx.x, r = tid >> 6, j = tid & 63;
  const int row0 = tile * 16;
  constexpr int N1 = F * CH_HU / 4 / 1024;
  float4 v1[N1];
#pragma unroll
  for (int i = 0; i < N1; ++i) v1[i] = reinterpret_cast<const float4*>(hd.W1)[tid + 1024 * i];
  const float4 v2 = reinterpret_cast<const float4*>(hd.W2)[tid];
  float4 vh = make_float4(0.f, 0.f, 0.f, 0.f);
  if (tid < 16 * F / 4) vh = reinterpret_cast<const float4*>(hd.hT + (size_t)row0 * F)[tid];
  const float b1j = hd.b1[j], b2j = hd.b2[j], w3j = hd.W3[j], b3 = hd.b3[0], gl = hd.dloss[0];
  const int row = row0 + r;
  const bool valid = row < hd.M;
  const int rc = min(row, hd.M - 1);
  const float yy = hd.y[rc], mm = hd.mask[rc];
#pragma unroll
  for (int i = 0; i < N1; ++i) {
    const int e = 4 * (tid + 1024 * i), k = e / CH_HU, c = e % CH_HU;
    float* d = sW1 + k * W1P + c;
    d[0] = v1[i].x; d[1] = v1[i].y; d[2] = v1[i].z; d[3] = v1[i].w;
  }
  {
    const int e = 4 * tid, k = e / CH_HU, c = e % CH_HU;
    float* d = sW2 + k * W1P + c;
    d[0] = v2.x; d[1] = v2.y; d[2] = v2.z; d[3] = v2.w;
  }
  if (tid < 16 * F / 4) {
    const int e = 4 * tid, rr = e / F, k = e % F;
    *reinterpret_cast<float4*>(sh + rr * HLP + k) = vh;
  }
  const float n = ch_mask_sum(hd.mask, hd.M, misc + 16);    // (contains a barrier)
  float acc = b1j;
#pragma unroll 8
  for (int k = 0; k < F; ++k) acc += sh[r * HLP + k] * sW1[k * W1P + j];
  sz1[r * CH_AP + j] = acc;
  sa1[r * CH_AP + j] = ch_leaky(acc, hd.alpha1);
  __syncthreads();
  float z2 = b2j;
#pragma unroll 8
  for (int k = 0; k < CH_HU; ++k) z2 += sa1[r * CH_AP + k] * sW2[k * W1P + j];
  const float a2 = ch_leaky(z2, hd.alpha2);
  const float z = wave_sum(a2 * w3j) + b3;
  const float wc = yy > 0.5f ? hd.w1 : hd.w0;
  const float d = valid ? gl / fmaxf(n, 1.f) * mm * wc * (sigmoidf_fast(z) - yy) : 0.f;
  sz2[r * CH_AP + j] = d * w3j * ch_dleaky(z2, hd.alpha2);
  sad[r * CH_AP + j] = a2 * d;
  if (j == 0) misc[r] = d;
  __syncthreads();
  {   // da1 = dz2 W2^T, dz1 = da1 * leaky'(z1)
    float da = 0.f;
#pragma unroll 8
    for (int k = 0; k < CH_HU; ++k) da += sz2[r * CH_AP + k] * sW2[j * W1P + k];
    sdz1[r * CH_AP + j] = da * ch_dleaky(sz1[r * CH_AP + j], hd.alpha1);
  }
  __syncthreads();
  float* rec = hd.gpart + (size_t)tile * Rec::PITCH;
#pragma unroll
  for (int q = 0; q < F / 16; ++q) {                 // dW1[k][j] = sum_r h[r][k] dz1[r][j]
    const int k = r + 16 * q;
    float s = 0.f;
#pragma unroll
    for (int rr = 0; rr < 16; ++rr) s += sh[rr * HLP + k] * sdz1[rr * CH_AP + j];
    rec[k * CH_HU + j] = s;
  }
  float* rec2 = rec + F * CH_HU + CH_HU;
#pragma unroll
  for (int q = 0; q < CH_HU / 16; ++q) {             // dW2[i][j] = sum_r a1[r][i] dz2[r][j]
    const int i = r + 16 * q;
    float s = 0.f;
#pragma unroll
    for (int rr = 0; rr < 16; ++rr) s += sa1[rr * CH_AP + i] * sz2[rr * CH_AP + j];
    rec2[i * CH_HU + j] = s;
  }
  if (tid < CH_HU) {
    float s1 = 0.f, s2 = 0.f, s3 = 0.f;
#pragma unroll
    for (int rr = 0; rr < 16; ++rr) {
      s1 += sdz1[rr * CH_AP + j];
      s2 += sz2[rr * CH_AP + j];
      s3 += sad[rr * CH_AP + j];
    }
    rec[F * CH_HU + j] = s1;                                    // db1
    rec2[CH_HU * CH_HU + j] = s2;                               // db2
    rec2[CH_HU * CH_HU + CH_HU + j] = s3;                       // dW3
  } else if (tid == CH_HU) {
    float s = 0.f;
#pragma unroll
    for (int rr = 0; rr < 16; ++rr) s += misc[rr];
    rec2[CH_HU * CH_HU + 2 * CH_HU] = s;                        // db3
  }
#pragma unroll
  for (int q = 0; q < F / 64; ++q) {                 // dh[r][k] = sum_j dz1[r][j] W1[k][j]
    const int k = j + 64 * q;
    float s = 0.f;
#pragma unroll 8
    for (int jj = 0; jj < CH_HU; ++jj) s += sdz1[r * CH_AP + jj] * sW1[k * W1P + jj];
    dh[r * HLP + k] = s;
  }
  __threadfence();
  __syncthreads();
  if (tid == 0) {
    const int t = __hip_atomic_fetch_add(hd.ticket, 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    misc[0] = t == ntiles - 1 ? 1.f : 0.f;
  }
  __syncthreads();
  return __builtin_amdgcn_readfirstlane((int)(misc[0] != 0.f)) != 0;
}

// The last-ticket workgroup: every tile's record, summed in tile order, added to the gradients.
template <int F>
__device__ void chain_head_bwd_reduce(const ChainHead& hd, int ntiles) {
  using Rec = ChainHeadRec<F>;
  for (int e = threadIdx.x; e < Rec::N; e += 1024) {
    float s = 0.f;
    for (int k = 0; k < ntiles; ++k) s += ch_load_acq(hd.gpart + (size_t)k * Rec::PITCH + e);
    int o = e;
    if (o < F * CH_HU) { hd.dW1[o] += s; continue; }
    o -= F * CH_HU;
    if (o < CH_HU) { hd.db1[o] += s; continue; }
    o -= CH_HU;
    if (o < CH_HU * CH_HU) { hd.dW2[o] += s; continue; }
    o -= CH_HU * CH_HU;
    if (o < CH_HU) { hd.db2[o] += s; continue; }
    o -= CH_HU;
    if (o < CH_HU) { hd.dW3[o] += s; continue; }
    hd.db3[0] += s;
  }
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_store(hd.ticket, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

}  // namespace gq
