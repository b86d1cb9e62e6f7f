// Gate-split persistent LSTM forward / backward for small hidden sizes (H <= 64),
// gfx950. Same math and memory layouts as lstm.hip (v1), different work split.
//
// Why: in v1 one wave owns all four gates of 16 units x 16 sequences, so every
// lane evaluates 20 transcendentals (sigmoid/tanh = exp + rcp, quarter rate) per
// step; for H = 16 the whole workgroup is ONE wave and the recurrence is bound by
// that VALU chain (~1000 cycles / step measured, scripts/lstm_microbench.py).
//
// v2 spreads a 16-sequence tile over 4 * H/16 waves and splits each step in two
// phases around LDS barriers:
//   gate phase  wave (g, ub) computes z^T for gate g, units [16ub, 16ub+16):
//               one MFMA chain (h part; the x part of step t+1 is issued right
//               after it, off the serial chain), ONE activation kind per wave,
//               result -> LDS gl[g][seq][unit] (and the gate row to HBM).
//   cell phase  one thread per (sequence, unit): c = f c + i g, h = o tanh(c);
//               h -> LDS (bf16, next step's MFMA B operand) and HBM.
// Backward mirrors it: cell phase (one thread per cell) produces dz, then wave
// (g, ub) computes the K = H slice  U[:, gH:(g+1)H] dz_g^T  of dh_rec and the
// next cell phase sums the four partials.
#include "common.h"

namespace gq {

template <int H, bool TRAIN, int KX, int D, bool VEC>
__global__ __launch_bounds__(64 * 4 * (H / 16)) void lstm_fwd2_kernel(
    const float* __restrict__ x, const float* __restrict__ W, const float* __restrict__ U,
    const float* __restrict__ bias, float* __restrict__ hseq, float* __restrict__ cseq,
    float* __restrict__ gates, int M, int T, int Din, int ldx) {
  constexpr int NUB = H / 16, NT = 256 * NUB;   // NT == 16 * H: one thread per cell
  constexpr int G4 = 4 * H;
  constexpr int KP = ((H + 31) / 32) * 32;
  constexpr int KS = KP / 32;
  constexpr int LDH = KP + 8;
  __shared__ __attribute__((aligned(16))) __bf16 hs[2][16][LDH];
  __shared__ __attribute__((aligned(16))) float gl[4][16][H];

  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int g = w / NUB, ub = w % NUB;
  const int col = lane & 15, quad = lane >> 4;
  const int ua = 16 * ub + col;
  const int u0 = 16 * ub + 4 * quad;
  const int row0 = blockIdx.x * 16;
  const int seq = row0 + col;
  const int lseq = min(seq, M - 1);
  const int cs = threadIdx.x / H, cu = threadIdx.x % H;    // cell owned in the cell phase
  const int cseqp = row0 + cs;

  for (int i = threadIdx.x; i < 2 * 16 * LDH; i += NT) (&hs[0][0][0])[i] = (__bf16)0.0f;

  bf16x8_t ufr[KS], wfr[KX];
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    bf16x8_t v;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = 32 * s + 8 * quad + j;
      v[j] = (__bf16)(k < H ? U[min(k, H - 1) * G4 + g * H + ua] : 0.0f);
    }
    ufr[s] = v;
  }
#pragma unroll
  for (int s = 0; s < KX; ++s) {
    bf16x8_t v;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = 32 * s + 8 * quad + j;
      v[j] = (__bf16)(k < Din ? W[min(k, Din - 1) * G4 + g * H + ua] : 0.0f);
    }
    wfr[s] = v;
  }
  const f32x4_t bias4 = {bias[g * H + u0], bias[g * H + u0 + 1], bias[g * H + u0 + 2], bias[g * H + u0 + 3]};
  int kidx[KX][8];
#pragma unroll
  for (int s = 0; s < KX; ++s)
#pragma unroll
    for (int j = 0; j < 8; ++j) kidx[s][j] = min(32 * s + 8 * quad + j, Din - 1);

  float xr[D][KX][8];
  const float* xrow = x + (size_t)lseq * T * ldx;
#define GQ_FWD2_LOAD(J, TT)                                                                      \
  {                                                                                              \
    const float* xp_ = xrow + (size_t)(TT) * ldx;                                                \
    _Pragma("unroll") for (int s = 0; s < KX; ++s) {                                             \
      if constexpr (VEC) {                                                                       \
        const int kk = min(32 * s + 8 * quad, Din - 8);                                          \
        const float4 a_ = *reinterpret_cast<const float4*>(xp_ + kk);                            \
        const float4 b_ = *reinterpret_cast<const float4*>(xp_ + kk + 4);                        \
        xr[J][s][0] = a_.x; xr[J][s][1] = a_.y; xr[J][s][2] = a_.z; xr[J][s][3] = a_.w;          \
        xr[J][s][4] = b_.x; xr[J][s][5] = b_.y; xr[J][s][6] = b_.z; xr[J][s][7] = b_.w;          \
      } else {                                                                                   \
        _Pragma("unroll") for (int q = 0; q < 8; ++q) xr[J][s][q] = xp_[kidx[s][q]];             \
      }                                                                                          \
    }                                                                                            \
  }
#define GQ_FWD2_XPROJ(J, ACC)                                                                    \
  {                                                                                              \
    ACC = bias4;                                                                                 \
    _Pragma("unroll") for (int s = 0; s < KX; ++s) {                                             \
      bf16x8_t bx_;                                                                              \
      _Pragma("unroll") for (int q = 0; q < 8; ++q) bx_[q] = (__bf16)xr[J][s][q];                \
      ACC = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wfr[s], bx_, ACC, 0, 0, 0);                  \
    }                                                                                            \
  }
#pragma unroll
  for (int j = 0; j < D; ++j) GQ_FWD2_LOAD(j, min(j, T - 1))
  f32x4_t accx;
  GQ_FWD2_XPROJ(0, accx)
  GQ_FWD2_LOAD(0, min(D, T - 1))
  float c = 0.f;
  __syncthreads();

  int buf = 0;
  for (int t0 = 0; t0 < T; t0 += D) {
#pragma unroll
    for (int j = 0; j < D; ++j) {
      const int t = t0 + j;
      const int jn = (j + 1 == D) ? 0 : j + 1;    // ring slot of step t + 1
      f32x4_t acc = accx;
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        const bf16x8_t bh = *reinterpret_cast<const bf16x8_t*>(&hs[buf][col][32 * s + 8 * quad]);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ufr[s], bh, acc, 0, 0, 0);
      }
      GQ_FWD2_XPROJ(jn, accx)                     // input projection of step t + 1 (independent of h)
      GQ_FWD2_LOAD(jn, min(t + 1 + D, T - 1))     // slot jn refilled with step t + 1 + D
      float a[4];
      if (g == 2) {
#pragma unroll
        for (int r = 0; r < 4; ++r) a[r] = tanhf_fast(acc[r]);
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r) a[r] = sigmoidf_fast(acc[r]);
      }
      *reinterpret_cast<float4*>(&gl[g][col][u0]) = make_float4(a[0], a[1], a[2], a[3]);
      if (TRAIN && t < T)
        *reinterpret_cast<float4*>(gates + ((size_t)seq * T + t) * G4 + g * H + u0) = make_float4(a[0], a[1], a[2], a[3]);
      lds_barrier();
      const float iv = gl[0][cs][cu], fv = gl[1][cs][cu], gv = gl[2][cs][cu], ov = gl[3][cs][cu];
      c = fv * c + iv * gv;
      const float hv = ov * tanhf_fast(c);
      hs[buf ^ 1][cs][cu] = (__bf16)hv;
      if (t < T) {
        const size_t o = ((size_t)cseqp * T + t) * H + cu;
        hseq[o] = hv;
        if constexpr (TRAIN) cseq[o] = c;
      }
      lds_barrier();
      buf ^= 1;
    }
  }
#undef GQ_FWD2_LOAD
#undef GQ_FWD2_XPROJ
}

template <int H, int D>
__global__ __launch_bounds__(64 * 4 * (H / 16)) void lstm_bwd2_kernel(
    const float* __restrict__ dh_out, const float* __restrict__ gates, const float* __restrict__ cseq,
    const float* __restrict__ U, float* __restrict__ dz_out, int M, int T) {
  constexpr int NUB = H / 16, NT = 256 * NUB;
  constexpr int G4 = 4 * H;
  constexpr int KSB = (H + 31) / 32;               // k-steps of one gate block (K = H, padded to 32)
  constexpr int LDZ = G4 + 32;                     // zero pad: padded k reads past gate 3 stay finite
  __shared__ __attribute__((aligned(16))) __bf16 zs[2][16][LDZ];
  __shared__ __attribute__((aligned(16))) float pr[4][16][H];

  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int g = w / NUB, ub = w % NUB;
  const int col = lane & 15, quad = lane >> 4;
  const int ua = 16 * ub + col;
  const int u0 = 16 * ub + 4 * quad;
  const int row0 = blockIdx.x * 16;
  const int cs = threadIdx.x / H, cu = threadIdx.x % H;
  const int cseqp = row0 + cs;
  const int lcs = min(cseqp, M - 1);
  const float msk = cseqp < M ? 1.f : 0.f;

  for (int i = threadIdx.x; i < 2 * 16 * LDZ; i += NT) (&zs[0][0][0])[i] = (__bf16)0.0f;
  for (int i = threadIdx.x; i < 4 * 16 * H; i += NT) (&pr[0][0][0])[i] = 0.f;

  bf16x8_t afr[KSB];
#pragma unroll
  for (int s = 0; s < KSB; ++s) {
    bf16x8_t v;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = 32 * s + 8 * quad + j;
      v[j] = (__bf16)(k < H ? U[(size_t)ua * G4 + g * H + min(k, H - 1)] : 0.0f);
    }
    afr[s] = v;
  }

  float rg[D][4], rc[D], rd[D];
#define GQ_BWD2_LOAD(J, SS)                                                          \
  {                                                                                  \
    const int tt = max(T - 1 - (SS), 0);                                             \
    const size_t o = (size_t)lcs * T + tt;                                           \
    _Pragma("unroll") for (int q = 0; q < 4; ++q) rg[J][q] = gates[o * G4 + q * H + cu]; \
    rc[J] = cseq[o * H + cu];                                                        \
    rd[J] = dh_out[o * H + cu];                                                      \
  }
#pragma unroll
  for (int j = 0; j < D; ++j) GQ_BWD2_LOAD(j, j)
  float dc = 0.f;
  __syncthreads();

  int buf = 0;
  for (int s0 = 0; s0 < T; s0 += D) {
#pragma unroll
    for (int j = 0; j < D; ++j) {
      const int s = s0 + j;
      const int t = T - 1 - s;
      const float cp = rc[(j + 1) % D] * (t > 0 ? 1.f : 0.f);   // c_{t-1}: next reverse slot
      const float dhr = pr[0][cs][cu] + pr[1][cs][cu] + pr[2][cs][cu] + pr[3][cs][cu];
      const float dh = rd[j] * msk + dhr;
      const float gi = rg[j][0], gf = rg[j][1], gg = rg[j][2], go = rg[j][3];
      const float tc = tanhf_fast(rc[j]);
      const float dct = dc + dh * go * (1.f - tc * tc);
      dc = dct * gf;
      const float zi = dct * gg * gi * (1.f - gi);
      const float zf = dct * cp * gf * (1.f - gf);
      const float zg = dct * gi * (1.f - gg * gg);
      const float zo = dh * tc * go * (1.f - go);
      GQ_BWD2_LOAD(j, s + D)
      zs[buf][cs][0 * H + cu] = (__bf16)zi;
      zs[buf][cs][1 * H + cu] = (__bf16)zf;
      zs[buf][cs][2 * H + cu] = (__bf16)zg;
      zs[buf][cs][3 * H + cu] = (__bf16)zo;
      if (t >= 0) {
        float* o = dz_out + ((size_t)cseqp * T + t) * G4 + cu;
        o[0 * H] = zi;
        o[1 * H] = zf;
        o[2 * H] = zg;
        o[3 * H] = zo;
      }
      lds_barrier();
      f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int k = 0; k < KSB; ++k) {
        const bf16x8_t bz = *reinterpret_cast<const bf16x8_t*>(&zs[buf][col][g * H + 32 * k + 8 * quad]);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(afr[k], bz, acc, 0, 0, 0);
      }
      *reinterpret_cast<float4*>(&pr[g][col][u0]) = make_float4(acc[0], acc[1], acc[2], acc[3]);
      lds_barrier();
      buf ^= 1;
    }
  }
#undef GQ_BWD2_LOAD
}

// ---------------------------------------------------------------- launchers
// Ring depth: <= ~56 outstanding VMEM ops per wave and <= ~48 ring VGPRs.
template <int H, bool TRAIN, int KX, bool VEC>
static void fwd2_cfg(int M, int T, int Din, int ldx, const float* x, const float* W, const float* U, const float* b,
                     float* h, float* c, float* g, hipStream_t st) {
  constexpr int loads = VEC ? 2 * KX : 8 * KX;
  constexpr int ops = loads + (TRAIN ? 3 : 1);
  constexpr int d1 = 56 / ops, d2 = 48 / (8 * KX);
  constexpr int Dm = d1 < d2 ? d1 : d2;
  constexpr int D = Dm < 2 ? 2 : (Dm > 8 ? 8 : Dm);
  hipLaunchKernelGGL((lstm_fwd2_kernel<H, TRAIN, KX, D, VEC>), dim3((M + 15) / 16), dim3(256 * (H / 16)), 0, st, x,
                     W, U, b, h, c, g, M, T, Din, ldx);
}

template <int H, bool TRAIN>
static void fwd2_h(int M, int T, int Din, int ldx, const float* x, const float* W, const float* U, const float* b,
                   float* h, float* c, float* g, hipStream_t st) {
  const int kx = (Din + 31) / 32;
  const bool vec = Din % 8 == 0 && ldx % 4 == 0 && (reinterpret_cast<uintptr_t>(x) % 16) == 0;
#define GQ_KX2(KXV)                                                              \
  if (vec) fwd2_cfg<H, TRAIN, KXV, true>(M, T, Din, ldx, x, W, U, b, h, c, g, st); \
  else fwd2_cfg<H, TRAIN, KXV, false>(M, T, Din, ldx, x, W, U, b, h, c, g, st);
  if (kx == 1) { GQ_KX2(1) }
  else { GQ_KX2(2) }
#undef GQ_KX2
}

// returns false when v2 does not handle this configuration (caller falls back to v1)
bool launch_fwd_v2(int H, bool train, int M, int T, int Din, int ldx, const float* x, const float* W, const float* U,
                   const float* b, float* h, float* c, float* g, hipStream_t st) {
  // Din > 64 (KX = 4) and the scalar-load H = 64 KX = 2 case exceed the register budget: v1
  if (Din > 64) return false;
  const bool vec = Din % 8 == 0 && ldx % 4 == 0 && (reinterpret_cast<uintptr_t>(x) % 16) == 0;
  if (H == 64 && Din > 32 && !vec) return false;
  switch (H) {
    case 16: train ? fwd2_h<16, true>(M, T, Din, ldx, x, W, U, b, h, c, g, st)
                   : fwd2_h<16, false>(M, T, Din, ldx, x, W, U, b, h, c, g, st); return true;
    case 32: train ? fwd2_h<32, true>(M, T, Din, ldx, x, W, U, b, h, c, g, st)
                   : fwd2_h<32, false>(M, T, Din, ldx, x, W, U, b, h, c, g, st); return true;
    case 64: train ? fwd2_h<64, true>(M, T, Din, ldx, x, W, U, b, h, c, g, st)
                   : fwd2_h<64, false>(M, T, Din, ldx, x, W, U, b, h, c, g, st); return true;
    default: return false;
  }
}

bool launch_bwd_v2(int H, int M, int T, const float* dh, const float* gates, const float* c, const float* U,
                   float* dz, hipStream_t st) {
  dim3 grid((M + 15) / 16);
  switch (H) {
    case 16: hipLaunchKernelGGL((lstm_bwd2_kernel<16, 5>), grid, dim3(256), 0, st, dh, gates, c, U, dz, M, T); return true;
    case 32: hipLaunchKernelGGL((lstm_bwd2_kernel<32, 5>), grid, dim3(512), 0, st, dh, gates, c, U, dz, M, T); return true;
    case 64: hipLaunchKernelGGL((lstm_bwd2_kernel<64, 4>), grid, dim3(1024), 0, st, dh, gates, c, U, dz, M, T); return true;
    default: return false;
  }
}

}  // namespace gq
