// Classifier head of the CML GCN on one 16-row tile, for the time4 kernels (time4_head.hip).
//
// Reference: Dense(64) -> LeakyReLU(.3) -> Dense(64) -> LeakyReLU(.3) -> Dense(1, sigmoid) on the
// TimeLayer output (libs/create_model.py:204-239) trained with class-weighted binary
// cross-entropy, SUM_OVER_BATCH_SIZE (libs/fit_model.py:76-111), metrics :79-86.
//
// The head is tiny (16 rows x 128 -> 64 -> 64 -> 1 per tile) and the workgroup that ran the
// last LSTM layer (time4, H = 128) of a tile already holds its input rows, so the head runs as
// that kernel's epilogue (forward) / prologue (backward) instead of two more launches:
//   forward:  logits, per-row loss, metric counts; the workgroup that arrives last (ticket)
//             sums the per-tile partials in tile order (deterministic) into the loss and the
//             metric accumulators.
//   backward: recomputes the head forward of its 16 rows, back-propagates dloss, leaves
//             dh_{T-1} of time4 in LDS and writes the tile's weight-gradient record; the
//             workgroup holding the last ticket sums the records in tile order and adds them to
//             the gradients.
// 512 threads (8 waves); a thread owns unit j = tid & 63 of rows w = tid >> 6 and w + 8. The
// backward also runs in 1024-thread workgroups (the chain backward launch): there tid is taken
// modulo 512, so waves 8..15 repeat waves 0..7's work - the same values to the same LDS / global
// addresses - and join every barrier; counter atomics stay with thread 0 alone.
// The products run on the exact-f32 MFMA (v_mfma_f32_16x16x4_f32: lane l holds A[l&15][k=l>>4]
// and B[k=l>>4][l&15], D[4(l>>4)+j][l&15]): one output per thread on the FMA pipes needed two
// LDS reads per multiply-add (13 us forward / 23 us backward per tile, measured). Weights come
// straight from L2 as A fragments (all loads of a product issued before its MFMAs),
// activations from LDS as B fragments.
#pragma once
#include "common.h"

namespace gq {

constexpr int CH_HU = 64;              // Dense units (model_config dense.units)
constexpr int CH_AP = CH_HU + 4;       // activation tile pitch (floats)
constexpr int CH_NW = 8;               // waves of the head workgroup
constexpr int CH_WP = CH_HU + 4;       // pitch of the LDS images of W1 / W2 (floats)

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
  int* done;                                  // backward: workgroups past the gradient reduction
  int* ctl;                                   // chain control words ([2]: timeout flag)
  int M;                                      // real rows (Mp - M padding rows are ignored)
  float alpha1, alpha2, w0, w1;
  // backward
  const float* dloss;                         // [1] dL/dloss
  float* gpart;                               // [ntiles][ChainHeadRec::PITCH] weight-gradient records
  float *dW1, *db1, *dW2, *db2, *dW3, *db3;   // accumulated (+=): .grad views or zeroed sinks
};

// gradient record of one tile: dW1 [F*64] | db1 [64] | dW2 [64*64] | db2 [64] | dW3 [64] | db3 [1]
template <int F>
struct ChainHeadRec {
  static constexpr int N = F * CH_HU + CH_HU + CH_HU * CH_HU + CH_HU + CH_HU + 1;
  static constexpr int PITCH = (N + 3) / 4 * 4;
};

typedef float ch_f4 __attribute__((ext_vector_type(4)));

// agent-scope (sc1) store / load of a handed-off float: L1-bypassing, no fence needed
__device__ __forceinline__ void ch_st(float* p, float v) {
  __hip_atomic_store(reinterpret_cast<unsigned*>(p), __float_as_uint(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ch_ld(const float* p) {
  return __uint_as_float(__hip_atomic_load(reinterpret_cast<const unsigned*>(p), __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT));
}

__device__ __forceinline__ float ch_leaky(float z, float a) { return z > 0.f ? z : a * z; }
__device__ __forceinline__ float ch_dleaky(float z, float a) { return z > 0.f ? 1.f : a; }

// Sum of mask[0..M) over the workgroup (red: CH_NW floats of LDS). Contains a barrier.
__device__ __forceinline__ int ch_tid() { return threadIdx.x & (64 * CH_NW - 1); }

__device__ __forceinline__ float ch_mask_sum(const float* __restrict__ mask, int M, float* red) {
  float s = 0.f;
  for (int i = ch_tid(); i < M; i += 64 * CH_NW) s += ch_ld(mask + i);   // (agent scope: the labels may come from this launch's producers)
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[ch_tid() >> 6] = s;
  __syncthreads();
  float t = 0.f;
#pragma unroll
  for (int k = 0; k < CH_NW; ++k) t += red[k];
  return t;
}

// D^T tile (16 outputs x 16 rows) of out[r][o] = sum_k act[r][k] * Wt[k][o], o in [16 ot, +16),
// k in [k0, k0 + 4 NS): A[m][kk] = Wt[(k0 + 4s + kk) * ldw + 16 ot + m], B[kk][n] = act[n * lda + k0 + 4s + kk]
template <int NS>
__device__ __forceinline__ ch_f4 ch_mm_wk(const float* __restrict__ Wt, int ldw, int ot, int k0, const float* act,
                                          int lda) {
  const int l = threadIdx.x & 63, m = l & 15, kk = l >> 4;
  float a[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) a[s] = Wt[(size_t)(k0 + 4 * s + kk) * ldw + 16 * ot + m];
  ch_f4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < NS; ++s)
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s], act[m * lda + k0 + 4 * s + kk], acc, 0, 0, 0);
  return acc;
}

// the same with the weight read transposed: A[m][kk] = W[(16 ot + m) * ldw + k0 + 4s + kk]
template <int NS>
__device__ __forceinline__ ch_f4 ch_mm_wt(const float* __restrict__ W, int ldw, int ot, int k0, const float* act,
                                          int lda) {
  const int l = threadIdx.x & 63, m = l & 15, kk = l >> 4;
  float a[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) a[s] = W[(size_t)(16 * ot + m) * ldw + k0 + 4 * s + kk];
  ch_f4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < NS; ++s)
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s], act[m * lda + k0 + 4 * s + kk], acc, 0, 0, 0);
  return acc;
}

// store a D^T tile (outputs 16 ot + m, rows n) into part[n][16 ot + m] (pitch lp)
__device__ __forceinline__ void ch_put(float* part, int lp, int ot, const ch_f4& d) {
  const int l = threadIdx.x & 63, n = l & 15, q = l >> 4;
#pragma unroll
  for (int j = 0; j < 4; ++j) part[n * lp + 16 * ot + 4 * q + j] = d[j];
}

// W1 [F][64] / W2 [64][64] -> LDS images (pitch CH_WP): coalesced float4 loads, all in flight
// at once; the head's products then read their A fragments from LDS (one L2 round trip per
// product phase before). Ends with a barrier.
template <int F>
__device__ __forceinline__ void ch_stage_weights(const ChainHead& hd, float* sW1, float* sW2) {
  constexpr int N1 = F * CH_HU / 4, N2 = CH_HU * CH_HU / 4, NT = 64 * CH_NW;
  const int tid = ch_tid();
  float4 v1[(N1 + NT - 1) / NT], v2[(N2 + NT - 1) / NT];
#pragma unroll
  for (int i = 0; i < (N1 + NT - 1) / NT; ++i) v1[i] = reinterpret_cast<const float4*>(hd.W1)[min(tid + NT * i, N1 - 1)];
#pragma unroll
  for (int i = 0; i < (N2 + NT - 1) / NT; ++i) v2[i] = reinterpret_cast<const float4*>(hd.W2)[min(tid + NT * i, N2 - 1)];
#pragma unroll
  for (int i = 0; i < (N1 + NT - 1) / NT; ++i) {
    const int e = 4 * (tid + NT * i);
    *reinterpret_cast<float4*>(sW1 + (e / CH_HU) * CH_WP + e % CH_HU) = v1[i];
  }
#pragma unroll
  for (int i = 0; i < (N2 + NT - 1) / NT; ++i) {
    const int e = 4 * (tid + NT * i);
    *reinterpret_cast<float4*>(sW2 + (e / CH_HU) * CH_WP + e % CH_HU) = v2[i];
  }
  __syncthreads();
}

// z1 = h W1 + b1 (-> sz1 if non-null), a1 = leaky(z1) -> sa1; returns z2 = a1 W2 + b2 of this
// thread's two rows (w, w + 8) at unit j. part: [2][16][CH_AP] partial tiles; sW1 / sW2: the LDS
// weight images (ch_stage_weights).
template <int F>
__device__ __forceinline__ void ch_head_z2(const ChainHead& hd, const float* sW1, const float* sW2, const float* hl,
                                           float* part, float* sz1, float* sa1, float z2[2]) {
  constexpr int HLP = F + 4, PT = 16 * CH_AP;
  const int tid = ch_tid(), w = tid >> 6, j = tid & 63;
  const int ot = w & 3, kh = w >> 2;                // output tile, K half
  const float b1j = hd.b1[j], b2j = hd.b2[j];
  ch_put(part + kh * PT, CH_AP, ot, ch_mm_wk<F / 8>(sW1, CH_WP, ot, kh * (F / 2), hl, HLP));
  __syncthreads();
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int r = w + 8 * q;
    const float z1 = b1j + part[r * CH_AP + j] + part[PT + r * CH_AP + j];
    if (sz1 != nullptr) sz1[r * CH_AP + j] = z1;
    sa1[r * CH_AP + j] = ch_leaky(z1, hd.alpha1);
  }
  __syncthreads();
  ch_put(part + kh * PT, CH_AP, ot, ch_mm_wk<8>(sW2, CH_WP, ot, kh * 32, sa1, CH_AP));
  __syncthreads();
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int r = w + 8 * q;
    z2[q] = b2j + part[r * CH_AP + j] + part[PT + r * CH_AP + j];
  }
}

// LDS bytes of the forward epilogue scratch
template <int F>
struct ChainHeadFwdLds {
  static constexpr int BYTES = (2 * 16 * CH_AP + 16 * CH_AP + 16 * 8 + (F + CH_HU) * CH_WP) * 4;
};

// Forward of the 16 rows of `tile` from hl [16][F + 4] (LDS).
// (hd by value: a reference into a kernel's by-value argument struct makes the compiler copy the
// whole struct to scratch)
// staged: the weight images at ch_head_fwd_weights(scratch) were loaded earlier (ch_stage_weights,
// e.g. while the chain's time4 stage still waited for its input)
template <int F>
__device__ __forceinline__ float* ch_head_fwd_weights(char* scratch) {
  return reinterpret_cast<float*>(scratch) + 3 * 16 * CH_AP + 16 * 8;
}
template <int F>
__device__ __forceinline__ void chain_head_fwd_handoff(const ChainHead hd, int tile, int ntiles, char* scratch);
// handoff = false: stop before the tile's loss partials are handed off (the caller runs
// chain_head_fwd_handoff later, e.g. after more work whose latency hides the stores' acknowledgements)
template <int F>
__device__ __forceinline__ void chain_head_fwd(const ChainHead hd, int tile, int ntiles, const float* hl, char* scratch,
                                               bool staged = false, bool handoff = true) {
  float* part = reinterpret_cast<float*>(scratch);    // [2][16][CH_AP]
  float* sa1 = part + 2 * 16 * CH_AP;                 // [16][CH_AP]
  float* rowv = sa1 + 16 * CH_AP;                     // [16][8]
  float* sW1 = rowv + 16 * 8;                         // [F][CH_WP]
  float* sW2 = sW1 + F * CH_WP;                       // [64][CH_WP]
  if (!staged) ch_stage_weights<F>(hd, sW1, sW2);
  const int tid = threadIdx.x, w = tid >> 6, j = tid & 63;
  const float w3j = hd.W3[j], b3 = hd.b3[0];
  float yy[2], mm[2];
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int rc = min(tile * 16 + w + 8 * q, hd.M - 1);
    yy[q] = ch_ld(hd.y + rc);
    mm[q] = ch_ld(hd.mask + rc);
  }
  float z2[2];
  ch_head_z2<F>(hd, sW1, sW2, hl, part, nullptr, sa1, z2);
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int r = w + 8 * q, row = tile * 16 + r;
    const float z = wave_sum(ch_leaky(z2[q], hd.alpha2) * w3j) + b3;
    if (j == 0) {
      const bool valid = row < hd.M;
      const float m = valid ? mm[q] : 0.f, y = yy[q];
      if (valid && hd.logits != nullptr) hd.logits[row] = z;
      const float l = fmaxf(z, 0.f) - z * y + log1pf(__expf(-fabsf(z)));
      const float wc = y > 0.5f ? hd.w1 : hd.w0;
      const float p = sigmoidf_fast(z);
      const bool pos = y > 0.5f, pp = p > 0.5f;
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
  }
  __syncthreads();
  if (handoff) chain_head_fwd_handoff<F>(hd, tile, ntiles, scratch);
}

// the tile's loss / metric partials (rowv, in the head forward's scratch) -> hd.part, and the loss
// of the last tile to arrive
template <int F>
__device__ __forceinline__ void chain_head_fwd_handoff(const ChainHead hd, int tile, int ntiles, char* scratch) {
  const float* rowv = reinterpret_cast<const float*>(scratch) + 3 * 16 * CH_AP;
  const int tid = threadIdx.x;
  // hand-off without fences (MI355X_MICROARCH.md: an agent fence costs 1.7-3.5 us): sc1 stores,
  // the storing wave's vmcnt(0), a workgroup barrier, ONE lane's agent-scope counter add; the
  // workgroup whose add came last reads the partials with sc1 loads
  if (tid < 6) {
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) s += rowv[k * 8 + tid];
    ch_st(hd.part + tile * 8 + tid, s);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    const int t = __hip_atomic_fetch_add(hd.ticket, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (t == ntiles - 1) {              // every tile's partials are in: fixed-order sums
      double s[6] = {0, 0, 0, 0, 0, 0};
      for (int k = 0; k < ntiles; ++k)
        for (int q = 0; q < 6; ++q) s[q] += (double)ch_ld(hd.part + k * 8 + q);
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
  static constexpr int BYTES = (16 * (F + 4) + 2 * 16 * CH_AP + 5 * 16 * CH_AP + 32 + (F + CH_HU) * CH_WP) * 4;
};

// Backward of the head for the 16 rows of `tile`, whose time4 output hT ([16][F] rows of the
// tile, global) feeds it: dh_{T-1} -> dh [16][F + 4] (LDS), the tile's weight-gradient record ->
// hd.gpart[tile], then the tile's arrival is counted in hd.ticket (chain_head_bwd_reduce waits
// for all of them).
// Precompute mode (the chain FORWARD's time4 stage, right after the head forward; everything here
// is linear in dL/dloss): hld >= 0 reads hT as the [16][hld] LDS tile of h_{T-1}, unit_gl takes
// dL/dloss = 1 (the backward scales dh and the reduced records by the real one), count = false
// leaves the arrival ticket alone (the records are complete at the launch boundary), and nlive
// is the number of live waves that share the record tiles.
template <int F>
__device__ __forceinline__ void chain_head_bwd(const ChainHead hd, const float* __restrict__ hT, int tile, int ntiles,
                                               float* dh, char* scratch, int hld = -1, bool unit_gl = false,
                                               bool count = true, int nlive = 0, const float* pW1 = nullptr,
                                               const float* pW2 = nullptr) {
  constexpr int HLP = F + 4, PT = 16 * CH_AP;
  using Rec = ChainHeadRec<F>;
  float* sh = reinterpret_cast<float*>(scratch);     // [16][HLP]
  float* part = sh + 16 * HLP;                       // [2][16][CH_AP]
  float* sz1 = part + 2 * PT;                        // [16][CH_AP] z1
  float* sa1 = sz1 + PT;                             // [16][CH_AP] leaky(z1)
  float* sz2 = sa1 + PT;                             // [16][CH_AP] dz2
  float* sad = sz2 + PT;                             // [16][CH_AP] leaky(z2) * d
  float* sdz1 = sad + PT;                            // [16][CH_AP] dz1
  float* misc = sdz1 + PT;                           // [32]: d per row, mask-sum reduction
  // (pW1 / pW2: images already staged by the caller, e.g. the forward's head)
  float* sW1 = pW1 != nullptr ? const_cast<float*>(pW1) : misc + 32;   // [F][CH_WP]
  float* sW2 = pW2 != nullptr ? const_cast<float*>(pW2) : sW1 + F * CH_WP;   // [64][CH_WP]
  if (pW1 == nullptr) ch_stage_weights<F>(hd, sW1, sW2);
  const int tid = ch_tid(), w = tid >> 6, j = tid & 63;
  const int l = tid & 63, lm = l & 15, lq = l >> 4;
  const int row0 = tile * 16;
  const float* hsrc = hld < 0 ? hT + (size_t)row0 * F : hT;
  const int hp = hld < 0 ? F : hld;
  for (int e = tid; e < 16 * F / 4; e += 64 * CH_NW) {
    const int rr = 4 * e / F, k = 4 * e % F;
    const float4 v = *reinterpret_cast<const float4*>(hsrc + (size_t)rr * hp + k);
    *reinterpret_cast<float4*>(sh + rr * HLP + k) = v;
  }
  const float w3j = hd.W3[j], b3 = hd.b3[0], gl = unit_gl ? 1.f : hd.dloss[0];
  float yy[2], mm[2];
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int rc = min(row0 + w + 8 * q, hd.M - 1);
    yy[q] = ch_ld(hd.y + rc);
    mm[q] = ch_ld(hd.mask + rc);
  }
  const float n = ch_mask_sum(hd.mask, hd.M, misc + 16);    // (its barrier also publishes sh)
  float z2[2];
  ch_head_z2<F>(hd, sW1, sW2, sh, part, sz1, sa1, z2);
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int r = w + 8 * q;
    const float a2 = ch_leaky(z2[q], hd.alpha2);
    const float z = wave_sum(a2 * w3j) + b3;
    const float wc = yy[q] > 0.5f ? hd.w1 : hd.w0;
    const float d = (row0 + r < hd.M) ? gl / fmaxf(n, 1.f) * mm[q] * wc * (sigmoidf_fast(z) - yy[q]) : 0.f;
    sz2[r * CH_AP + j] = d * w3j * ch_dleaky(z2[q], hd.alpha2);
    sad[r * CH_AP + j] = a2 * d;
    if (j == 0) misc[r] = d;
  }
  __syncthreads();
  {   // da1 = dz2 W2^T (A = W2 rows), dz1 = da1 * leaky'(z1)
    const int ot = w & 3, kh = w >> 2;
    ch_put(part + kh * PT, CH_AP, ot, ch_mm_wt<8>(sW2, CH_WP, ot, kh * 32, sz2, CH_AP));
  }
  __syncthreads();
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int r = w + 8 * q;
    const float da = part[r * CH_AP + j] + part[PT + r * CH_AP + j];
    sdz1[r * CH_AP + j] = da * ch_dleaky(sz1[r * CH_AP + j], hd.alpha1);
  }
  __syncthreads();
  // dh = dz1 W1^T: output tiles of 16 features, the full K = 64 per wave (no partials)
#pragma unroll
  for (int q = 0; q < F / 16 / CH_NW; ++q) {
    const int ot = w + CH_NW * q;
    ch_put(dh, HLP, ot, ch_mm_wt<16>(sW1, CH_WP, ot, 0, sdz1, CH_AP));
  }
  // weight gradients over the tile's 16 rows (K = rows): A[m][kk] = act1[4s + kk][16 it + m],
  // B[kk][n] = act2[4s + kk][16 jt + n]
  auto wgrad = [&](const float* a1, int lda1, int it, const float* a2, int jt) {
    ch_f4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < 4; ++s)
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a1[(4 * s + lq) * lda1 + 16 * it + lm],
                                                 a2[(4 * s + lq) * CH_AP + 16 * jt + lm], acc, 0, 0, 0);
    return acc;
  };
  float* rec = hd.gpart + (size_t)tile * Rec::PITCH;
  float* rec2 = rec + F * CH_HU + CH_HU;
  // the record tiles are spread over ALL waves of the workgroup (8 or 16), each stored once
  const int wa = threadIdx.x >> 6, nwa = nlive > 0 ? nlive : (int)(blockDim.x >> 6);
  for (int t = wa; t < F / 16 * 4; t += nwa) {        // dW1 [F][64]: (F/16) x 4 tiles
    const int it = t >> 2, jt = t & 3;
    const ch_f4 acc = wgrad(sh, HLP, it, sdz1, jt);
#pragma unroll
    for (int k = 0; k < 4; ++k) ch_st(rec + (16 * it + 4 * lq + k) * CH_HU + 16 * jt + lm, acc[k]);
  }
  for (int t = wa; t < 16; t += nwa) {                // dW2 [64][64]: 16 tiles
    const int it = t >> 2, jt = t & 3;
    const ch_f4 acc = wgrad(sa1, CH_AP, it, sz2, jt);
#pragma unroll
    for (int k = 0; k < 4; ++k) ch_st(rec2 + (16 * it + 4 * lq + k) * CH_HU + 16 * jt + lm, acc[k]);
  }
  if (threadIdx.x < CH_HU) {
    float s1 = 0.f, s2 = 0.f, s3 = 0.f;
#pragma unroll
    for (int rr = 0; rr < 16; ++rr) {
      s1 += sdz1[rr * CH_AP + j];
      s2 += sz2[rr * CH_AP + j];
      s3 += sad[rr * CH_AP + j];
    }
    ch_st(rec + F * CH_HU + j, s1);                             // db1
    ch_st(rec2 + CH_HU * CH_HU + j, s2);                        // db2
    ch_st(rec2 + CH_HU * CH_HU + CH_HU + j, s3);                // dW3
  } else if (threadIdx.x == CH_HU) {
    float s = 0.f;
#pragma unroll
    for (int rr = 0; rr < 16; ++rr) s += misc[rr];
    ch_st(rec2 + CH_HU * CH_HU + 2 * CH_HU, s);                 // db3
  }
  if (!count) {
    __syncthreads();
    return;
  }
  // (sc1 stores, every wave's vmcnt(0), barrier, one lane's counter add: no fence)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_fetch_add(hd.ticket, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// After chain_head_bwd: once every tile's record is in (ticket == ntiles; the workgroups of the
// launch are all resident, and each has its own recurrence to run in between), workgroup `tile`
// sums its 1/ntiles slice of the records over the tiles in tile order (deterministic) and adds
// it to the gradients; the last one to finish re-arms both counters. One workgroup reducing all
// of it took ~60 us (25 rounds of 8 dependent-latency loads per thread).
// pre: the records come from an earlier launch (chain_head_bwd's precompute mode): no arrival wait,
// and every sum is scaled by `scale` (dL/dloss).
template <int F>
__device__ __forceinline__ void chain_head_bwd_reduce(const ChainHead hd, int tile, int ntiles, bool pre = false,
                                                      float scale = 1.f) {
  using Rec = ChainHeadRec<F>;
  __shared__ int bad;
  if (threadIdx.x == 0 && pre) bad = 0;
  if (threadIdx.x == 0 && !pre) {
    int nap = 1, it = 0;
    bad = 0;
    while (__hip_atomic_load(hd.ticket, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < ntiles) {
      for (int k = 0; k < nap; ++k) __builtin_amdgcn_s_sleep(8);
      nap = min(nap * 2, 8);
      if (++it > (1 << 22)) {             // never expected (8 co-resident workgroups): fail loudly
        __hip_atomic_store(hd.ctl + 2, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        bad = 1;
        break;
      }
    }
  }
  __syncthreads();
  if (!bad) {                             // (the records were stored sc1: sc1 loads, no acquire)
    const int chunk = (Rec::N + ntiles - 1) / ntiles;
    const int e1 = min(Rec::N, (tile + 1) * chunk);
    constexpr int RB = 4;                 // elements per thread per round: RB x ntiles loads in flight
    for (int e0 = tile * chunk + (int)threadIdx.x; e0 < e1; e0 += RB * blockDim.x) {
      float acc[RB];
#pragma unroll
      for (int q = 0; q < RB; ++q) acc[q] = 0.f;
      for (int k = 0; k < ntiles; ++k) {
        float v[RB];
#pragma unroll
        for (int q = 0; q < RB; ++q) v[q] = ch_ld(hd.gpart + (size_t)k * Rec::PITCH + min(e0 + q * (int)blockDim.x, e1 - 1));
#pragma unroll
        for (int q = 0; q < RB; ++q) acc[q] += v[q];
      }
#pragma unroll
      for (int q = 0; q < RB; ++q) {
      const int e = e0 + q * (int)blockDim.x;
      if (e >= e1) break;
      const float s = acc[q] * scale;
      // (adam_flagged decides the step from such flags instead of scanning the gradient buffer)
      if (!isfinite(s)) __hip_atomic_store(hd.ctl + 7, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
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
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const int d = __hip_atomic_fetch_add(hd.done, 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (d == ntiles - 1) {                // everyone has read the ticket: re-arm for the next launch
      __hip_atomic_store(hd.ticket, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(hd.done, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

}  // namespace gq
