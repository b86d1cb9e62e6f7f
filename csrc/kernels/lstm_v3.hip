// Cell-per-lane persistent LSTM forward / backward for H <= 64 (bf16 MFMA), gfx950.
// Same math as lstm.hip (v1); one barrier per step like v1, but 4x less VALU per lane.
//
// v1 gives each lane 4 units x 4 gates of one sequence (20 sigmoid/tanh = 40
// transcendentals per step), so the H = 16 recurrence is bound by one wave's VALU
// issue (8 cycles per transcendental, MI355X_MICROARCH constants) at ~1000 cycles /
// step. v3 permutes the rows of the MFMA A operand so that ONE 16x16 output tile
// holds (unit, gate) pairs: tile row 4q + g = gate g of unit 4w + q. With the C
// layout (col = lane & 15 -> sequence, rows 4 (lane >> 4) + r) every lane then gets
// the i, f, g, o pre-activations of exactly one cell and does that cell's update
// alone: 5 activations per lane per step, H/4 waves per 16-sequence tile.
//
// x_t is needed by every wave as the MFMA B operand: a few loader lanes keep a
// register ring of x rows in flight and drop the next step's tile into LDS (bf16)
// before the step barrier, so each x element is loaded once per tile (v2 loaded it
// once per wave and was address-unit bound).
//
// Gates are stored interleaved per cell ([M, T, H, 4]: one 16-byte store / load per
// lane per step); the backward kernel of this file is the only consumer.
//
// Backward: lane = cell again. dz (bf16) crosses LDS once per step; the recurrent
// gradient dh_{t-1}^T = U dz^T uses A rows 4q (unit 4w + q, all K = 4H) and zero
// rows 4q + 1..3, so acc[0] of a lane is the dh of its own cell.
#include "common.h"

namespace gq {

template <int H>
struct V3 {
  static constexpr int NW = H / 4;              // waves per 16-sequence tile
  static constexpr int NT = 64 * NW;            // == 16 * H threads: one per cell
  static constexpr int G4 = 4 * H;
  static constexpr int KPH = ((H + 31) / 32) * 32;
  static constexpr int KSH = KPH / 32;
};

// D: register-ring depth of the x loader (steps in flight)
template <int H, bool TRAIN, int KX, int D, int GR>
__global__ __launch_bounds__(16 * H) void lstm_fwd3_kernel(
    const float* __restrict__ x, const float* __restrict__ W, const float* __restrict__ U,
    const float* __restrict__ bias, float* __restrict__ hseq, float* __restrict__ cseq,
    float* __restrict__ gates, int M, int T, int Din, int ldx) {
  using C = V3<H>;
  constexpr int KPX = 32 * KX;
  __shared__ __attribute__((aligned(16))) __bf16 hs[2][16][C::KPH + 8];
  __shared__ __attribute__((aligned(16))) __bf16 xs[2][16][KPX + 8];

  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int col = lane & 15, quad = lane >> 4;
  const int row0 = blockIdx.x * 16;
  const int seq = row0 + col;                    // padded row of this lane's cell
  const int u = 4 * w + quad;                    // unit of this lane's cell
  // A-operand row supplied by this lane: tile row `col` = gate (col & 3) of unit 4w + (col >> 2)
  const int ar_unit = 4 * w + (col >> 2), ar_gate = col & 3;

  for (int i = threadIdx.x; i < 2 * 16 * (C::KPH + 8); i += C::NT) (&hs[0][0][0])[i] = (__bf16)0.0f;
  for (int i = threadIdx.x; i < 2 * 16 * (KPX + 8); i += C::NT) (&xs[0][0][0])[i] = (__bf16)0.0f;

  bf16x8_t ufr[C::KSH], wfr[KX];
#pragma unroll
  for (int s = 0; s < C::KSH; ++s) {
    bf16x8_t v;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = 32 * s + 8 * quad + j;
      v[j] = (__bf16)(U[min(k, H - 1) * C::G4 + ar_gate * H + ar_unit] * (k < H ? 1.0f : 0.0f));
    }
    ufr[s] = v;
  }
#pragma unroll
  for (int s = 0; s < KX; ++s) {
    bf16x8_t v;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = 32 * s + 8 * quad + j;
      v[j] = (__bf16)(W[min(k, Din - 1) * C::G4 + ar_gate * H + ar_unit] * (k < Din ? 1.0f : 0.0f));
    }
    wfr[s] = v;
  }
  const f32x4_t bias4 = {bias[0 * H + u], bias[1 * H + u], bias[2 * H + u], bias[3 * H + u]};

  // ---- x loader: granule e (GR floats) of the per-step tile [16 seq][Din]. Whole waves
  // load (the branch stays wave-uniform: no vmcnt drain at a divergent join); surplus
  // lanes duplicate the last granule, writing the same value to the same LDS word.
  const int per_seq = Din / GR;
  const int n_gran = 16 * per_seq;
  const bool loader = w < (n_gran + 63) / 64;
  const int lg = min((int)threadIdx.x, n_gran - 1);
  const int l_seq = lg / per_seq, l_k = (lg % per_seq) * GR;
  const float* lrow = x + (size_t)min(row0 + l_seq, M - 1) * T * ldx + l_k;
  float4 xr[D];
#define GQ_X3_LOAD(J, TT)                                                               \
  {                                                                                     \
    const float* p_ = lrow + (size_t)(TT) * ldx;                                        \
    if constexpr (GR == 4) xr[J] = *reinterpret_cast<const float4*>(p_);                 \
    else if constexpr (GR == 2) {                                                       \
      const float2 v_ = *reinterpret_cast<const float2*>(p_);                           \
      xr[J].x = v_.x; xr[J].y = v_.y;                                                   \
    } else xr[J].x = *p_;                                                               \
  }
#define GQ_X3_STAGE(J, BUF)                                                             \
  {                                                                                     \
    __bf16* d_ = &xs[BUF][l_seq][l_k];                                                  \
    d_[0] = (__bf16)xr[J].x;                                                            \
    if constexpr (GR >= 2) d_[1] = (__bf16)xr[J].y;                                     \
    if constexpr (GR == 4) { d_[2] = (__bf16)xr[J].z; d_[3] = (__bf16)xr[J].w; }         \
  }
  if (loader) {
#pragma unroll
    for (int j = 0; j < D; ++j) GQ_X3_LOAD(j, min(j, T - 1))
  }
  __syncthreads();   // zero-fill of xs done before the first staging
  if (loader) {
    GQ_X3_STAGE(0, 0)
    GQ_X3_LOAD(0, min(D, T - 1))
  }
  float c = 0.f;
  __syncthreads();

  int buf = 0;
  for (int t0 = 0; t0 < T; t0 += D) {
#pragma unroll
    for (int j = 0; j < D; ++j) {
      const int t = t0 + j;
      const int jn = (j + 1 == D) ? 0 : j + 1;   // ring slot holding step t + 1
      f32x4_t acc = bias4;
#pragma unroll
      for (int s = 0; s < KX; ++s) {
        const bf16x8_t bx = *reinterpret_cast<const bf16x8_t*>(&xs[buf][col][32 * s + 8 * quad]);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wfr[s], bx, acc, 0, 0, 0);
      }
#pragma unroll
      for (int s = 0; s < C::KSH; ++s) {
        const bf16x8_t bh = *reinterpret_cast<const bf16x8_t*>(&hs[buf][col][32 * s + 8 * quad]);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ufr[s], bh, acc, 0, 0, 0);
      }
      if (loader) {                               // next step's x tile -> the other LDS buffer
        GQ_X3_STAGE(jn, buf ^ 1)
        GQ_X3_LOAD(jn, min(t + 1 + D, T - 1))
      }
      const float iv = sigmoidf_fast(acc[0]);
      const float fv = sigmoidf_fast(acc[1]);
      const float gv = tanhf_fast(acc[2]);
      const float ov = sigmoidf_fast(acc[3]);
      c = fv * c + iv * gv;
      const float hv = ov * tanhf_fast(c);
      hs[buf ^ 1][col][u] = (__bf16)hv;
      if (t < T) {   // wave-uniform
        const size_t o = (size_t)seq * T + t;
        hseq[o * H + u] = hv;
        if constexpr (TRAIN) {
          cseq[o * H + u] = c;
          *reinterpret_cast<float4*>(gates + (o * H + u) * 4) = make_float4(iv, fv, gv, ov);
        }
      }
      lds_barrier();
      buf ^= 1;
    }
  }
#undef GQ_X3_LOAD
#undef GQ_X3_STAGE
}

template <int H, int D>
__global__ __launch_bounds__(16 * H) void lstm_bwd3_kernel(
    const float* __restrict__ dh_out, const float* __restrict__ gates, const float* __restrict__ cseq,
    const float* __restrict__ U, float* __restrict__ dz_out, int M, int T) {
  using C = V3<H>;
  constexpr int KB = C::G4 / 32;
  constexpr int LDZ = C::G4 + 8;
  __shared__ __attribute__((aligned(16))) __bf16 zs[2][16][LDZ];

  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int col = lane & 15, quad = lane >> 4;
  const int row0 = blockIdx.x * 16;
  const int seq = row0 + col;
  const int lseq = min(seq, M - 1);
  const float msk = seq < M ? 1.f : 0.f;
  const int u = 4 * w + quad;

  // A rows: tile row `col` = unit 4w + (col >> 2) when col % 4 == 0, zero otherwise
  bf16x8_t afr[KB];
#pragma unroll
  for (int s = 0; s < KB; ++s) {
    bf16x8_t v;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float val = U[(size_t)(4 * w + (col >> 2)) * C::G4 + 32 * s + 8 * quad + j];
      v[j] = (__bf16)(val * ((col & 3) == 0 ? 1.0f : 0.0f));
    }
    afr[s] = v;
  }

  float4 rg[D];
  float rc[D], rd[D];
#define GQ_B3_LOAD(J, SS)                                                   \
  {                                                                         \
    const int tt = max(T - 1 - (SS), 0);                                    \
    const size_t o = (size_t)lseq * T + tt;                                 \
    rg[J] = *reinterpret_cast<const float4*>(gates + (o * H + u) * 4);      \
    rc[J] = cseq[o * H + u];                                                \
    rd[J] = dh_out[o * H + u];                                              \
  }
#pragma unroll
  for (int j = 0; j < D; ++j) GQ_B3_LOAD(j, j)
  float dc = 0.f, dhr = 0.f;
  int buf = 0;
  for (int s0 = 0; s0 < T; s0 += D) {
#pragma unroll
    for (int j = 0; j < D; ++j) {
      const int s = s0 + j;
      const int t = T - 1 - s;
      const float cp = rc[(j + 1) % D] * (t > 0 ? 1.f : 0.f);   // c_{t-1}
      const float dh = rd[j] * msk + dhr;
      const float gi = rg[j].x, gf = rg[j].y, gg = rg[j].z, go = rg[j].w;
      const float tc = tanhf_fast(rc[j]);
      const float dct = dc + dh * go * (1.f - tc * tc);
      dc = dct * gf;
      const float zi = dct * gg * gi * (1.f - gi);
      const float zf = dct * cp * gf * (1.f - gf);
      const float zg = dct * gi * (1.f - gg * gg);
      const float zo = dh * tc * go * (1.f - go);
      GQ_B3_LOAD(j, s + D)
      zs[buf][col][0 * H + u] = (__bf16)zi;
      zs[buf][col][1 * H + u] = (__bf16)zf;
      zs[buf][col][2 * H + u] = (__bf16)zg;
      zs[buf][col][3 * H + u] = (__bf16)zo;
      if (t >= 0) {   // wave-uniform
        float* o = dz_out + ((size_t)seq * T + t) * C::G4 + u;
        o[0 * H] = zi;
        o[1 * H] = zf;
        o[2 * H] = zg;
        o[3 * H] = zo;
      }
      lds_barrier();
      // two accumulators halve the dependent MFMA chain
      f32x4_t a0 = {0.f, 0.f, 0.f, 0.f}, a1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int k = 0; k < KB; ++k) {
        const bf16x8_t bz = *reinterpret_cast<const bf16x8_t*>(&zs[buf][col][32 * k + 8 * quad]);
        if (k & 1) a1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(afr[k], bz, a1, 0, 0, 0);
        else a0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(afr[k], bz, a0, 0, 0, 0);
      }
      dhr = a0[0] + a1[0];
      buf ^= 1;
    }
  }
#undef GQ_B3_LOAD
}

// ---------------------------------------------------------------- launchers
// Granule of the x loader: 4 floats (16-B aligned rows), 2 (8-B) or 1.
int v3_granule(int Din, int ldx, const void* x) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(x);
  if (Din % 4 == 0 && ldx % 4 == 0 && a % 16 == 0) return 4;
  if (Din % 2 == 0 && ldx % 2 == 0 && a % 8 == 0) return 2;
  return 1;
}

// v3 handles H in {16, 32, 64} when the per-step x tile fits the loader lanes
// (16 * Din / granule <= 16 * H) and Din <= 128.
bool v3_supports(int H, int Din, int ldx, const void* x) {
  if (H != 16 && H != 32 && H != 64) return false;
  if (Din > 128 || Din < 1) return false;
  return Din / v3_granule(Din, ldx, x) <= H;
}

template <int H, bool TRAIN, int KX, int GR>
static void fwd3_cfg(int M, int T, int Din, int ldx, const float* x, const float* W, const float* U, const float* b,
                     float* h, float* c, float* g, hipStream_t st) {
  constexpr int D = 6;     // loader lanes carry one load per step: 6 steps in flight
  hipLaunchKernelGGL((lstm_fwd3_kernel<H, TRAIN, KX, D, GR>), dim3((M + 15) / 16), dim3(16 * H), 0, st, x, W, U,
                     b, h, c, g, M, T, Din, ldx);
}

template <int H, bool TRAIN>
static void fwd3_h(int M, int T, int Din, int ldx, const float* x, const float* W, const float* U, const float* b,
                   float* h, float* c, float* g, hipStream_t st) {
  const int kx = (Din + 31) / 32;
  const int gr = v3_granule(Din, ldx, x);
#define GQ_KX3(KXV)                                                                         \
  if (gr == 4) fwd3_cfg<H, TRAIN, KXV, 4>(M, T, Din, ldx, x, W, U, b, h, c, g, st);          \
  else if (gr == 2) fwd3_cfg<H, TRAIN, KXV, 2>(M, T, Din, ldx, x, W, U, b, h, c, g, st);     \
  else fwd3_cfg<H, TRAIN, KXV, 1>(M, T, Din, ldx, x, W, U, b, h, c, g, st);
  if (kx == 1) { GQ_KX3(1) }
  else if (kx == 2) { GQ_KX3(2) }
  else { GQ_KX3(4) }
#undef GQ_KX3
}

// Forward with the interleaved gate layout; call only when v3_supports(...) is true.
void launch_fwd_v3(int H, bool train, int M, int T, int Din, int ldx, const float* x, const float* W, const float* U,
                   const float* b, float* h, float* c, float* g, hipStream_t st) {
  switch (H) {
    case 16: train ? fwd3_h<16, true>(M, T, Din, ldx, x, W, U, b, h, c, g, st)
                   : fwd3_h<16, false>(M, T, Din, ldx, x, W, U, b, h, c, g, st); break;
    case 32: train ? fwd3_h<32, true>(M, T, Din, ldx, x, W, U, b, h, c, g, st)
                   : fwd3_h<32, false>(M, T, Din, ldx, x, W, U, b, h, c, g, st); break;
    default: train ? fwd3_h<64, true>(M, T, Din, ldx, x, W, U, b, h, c, g, st)
                   : fwd3_h<64, false>(M, T, Din, ldx, x, W, U, b, h, c, g, st); break;
  }
}

bool launch_bwd_v3(int H, int M, int T, const float* dh, const float* gates, const float* c, const float* U,
                   float* dz, hipStream_t st) {
  dim3 grid((M + 15) / 16);
  switch (H) {
    case 16: hipLaunchKernelGGL((lstm_bwd3_kernel<16, 6>), grid, dim3(256), 0, st, dh, gates, c, U, dz, M, T); return true;
    case 32: hipLaunchKernelGGL((lstm_bwd3_kernel<32, 6>), grid, dim3(512), 0, st, dh, gates, c, U, dz, M, T); return true;
    case 64: hipLaunchKernelGGL((lstm_bwd3_kernel<64, 6>), grid, dim3(1024), 0, st, dh, gates, c, U, dz, M, T); return true;
    default: return false;
  }
}

}  // namespace gq
