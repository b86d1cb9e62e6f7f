// Persistent, register-resident LSTM layer for gfx950.
//
// Keras LSTM semantics (gate order i,f,c,o; sigmoid recurrent activation, tanh
// activation, zero initial state) as used by the reference TimeLayer
// (libs/create_model.py:61-79):
//   z_t = x_t W + h_{t-1} U + b ;  c_t = f c_{t-1} + i g ;  h_t = o tanh(c_t)
// One launch runs all T steps of a layer (the serial chain never leaves the CU).
//
// Transposed MFMA formulation: each step computes z^T[unit][seq] = W^T x_t^T +
// U^T h_{t-1}^T with v_mfma_f32_16x16x32_bf16, weights as the A operand and data
// as the B operand. A workgroup owns 16 sequences (MFMA columns); wave w owns
// units [16w, 16w+16) of ALL FOUR gates. With the 16x16 C layout (col = lane&15
// -> sequence, rows 4*(lane>>4)+r -> 4 consecutive units) every lane holds the
// i,f,g,o pre-activations of 4 consecutive units of ONE sequence, so
//   * the cell update is lane-local, c stays in 4 VGPRs for the whole sequence,
//   * every global access is a 16-byte vector op (h, c, 4 gates, dh, dz rows),
//   * h_{t-1} crosses LDS as one 8-byte write + one 16-byte read per lane.
// W^T, U^T and b are packed into MFMA fragments once and stay in VGPRs (the input
// projection is fused: no xp GEMM). x_t and the backward's saved activations
// stream through a D-deep register ring (load for step t+D issued when step t
// consumes its slot) sized so the <= 63 outstanding VMEM ops never saturate.
// Loads clamp rows/steps and outputs are padded to 16-row tiles: no per-lane
// branch surrounds a memory op (hipcc would drain vmcnt at every join). One
// LDS-only barrier per step (no vmcnt drain).
//
// BF16=false: exact f32-input MFMA (v_mfma_f32_16x16x4_f32), the numerics
// reference path.
//
// Backward (BPTT): reverse ring over (i,f,g,o, c_t, c_{t-1}, dh_t);
// dh_rec^T = U dz^T is a K = 4H MFMA chain with U rows as A fragments and dz
// (bf16) crossing LDS once per step; dz (fp32) is written for the weight-gradient
// GEMMs.
#include "common.h"
#include <cstdlib>

namespace gq {

template <int H, bool BF16>
struct LstmCfg {
  static constexpr int G4 = 4 * H;
  static constexpr int KP = BF16 ? ((H + 31) / 32) * 32 : H;
  static constexpr int KS = BF16 ? KP / 32 : H / 4;       // h k-steps (forward)
  static constexpr int KB = BF16 ? G4 / 32 : G4 / 4;      // dz k-steps (backward, K = 4H)
};

// k index of element j of this lane's B fragment in 32-wide chunk s
template <bool BF16>
__device__ __forceinline__ int b_k(int s, int quad, int j) {
  return BF16 ? 32 * s + 8 * quad + j : 32 * s + 4 * j + quad;
}

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ void st4(float* p, float a, float b, float c, float d) {
  *reinterpret_cast<float4*>(p) = make_float4(a, b, c, d);
}

// ---------------------------------------------------------------- forward
// VEC: x rows are 16-byte aligned and Din % 8 == 0 -> two float4 per chunk
// Saved gates: bf16 in BF16 mode (8 instead of 16 bytes per cell-step; the gates lie in (0, 1) / (-1, 1)
// and combine with bf16 MFMA operands in the backward), fp32 in the fp32 reference mode.
#ifndef LSTM_BF16_GATES
#define LSTM_BF16_GATES 1     // 0: fp32 saved gates in bf16 mode too (the round-5 form, for A/B builds)
#endif
template <bool BF16>
using gate_t = typename std::conditional<BF16 && LSTM_BF16_GATES, __bf16, float>::type;

template <int H, bool BF16, bool TRAIN, int KX, int D, bool VEC>
__global__ __launch_bounds__(64 * (H / 16)) void lstm_fwd_kernel(
    const float* __restrict__ x, const float* __restrict__ W, const float* __restrict__ U,
    const float* __restrict__ bias, float* __restrict__ hseq, float* __restrict__ cseq,
    gate_t<BF16>* __restrict__ gates, int M, int T, int Din, int ldx) {
  using C = LstmCfg<H, BF16>;
  constexpr int G4 = C::G4;
  constexpr int KS = C::KS;
  constexpr int LDH = BF16 ? C::KP + 8 : H + 1;
  using elem_t = typename std::conditional<BF16, __bf16, float>::type;
  __shared__ __attribute__((aligned(16))) elem_t hs[2][16][LDH];

  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int col = lane & 15;          // sequence column of B / C
  const int quad = lane >> 4;
  const int ua = 16 * w + col;        // unit row of this lane's A fragments
  const int u0 = 16 * w + 4 * quad;   // first of the 4 units this lane owns in C
  const int row0 = blockIdx.x * 16;
  const int seq = row0 + col;                  // padded row (stores)
  const int lseq = min(seq, M - 1);            // clamped row (loads)

  for (int i = threadIdx.x; i < 2 * 16 * LDH; i += blockDim.x) (&hs[0][0][0])[i] = elem_t(0.0f);

  // ---- register-resident A fragments: W^T and U^T rows of unit ua, per gate
  using frag_t = typename std::conditional<BF16, bf16x8_t, float>::type;
  constexpr int SUB = BF16 ? 1 : 8;
  frag_t ufr[4][KS];
  frag_t wfr[4][KX * SUB];
#pragma unroll
  for (int g = 0; g < 4; ++g) {
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      if constexpr (BF16) {
        bf16x8_t v;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int k = 32 * s + 8 * quad + j;
          v[j] = (__bf16)(U[min(k, H - 1) * G4 + g * H + ua] * (k < H ? 1.0f : 0.0f));
        }
        ufr[g][s] = v;
      } else {
        ufr[g][s] = U[(4 * s + quad) * G4 + g * H + ua];
      }
    }
#pragma unroll
    for (int s = 0; s < KX; ++s) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int k = b_k<BF16>(s, quad, j);
        const float v = W[min(k, Din - 1) * G4 + g * H + ua] * (k < Din ? 1.0f : 0.0f);
        if constexpr (BF16) wfr[g][s][j] = (__bf16)v;
        else wfr[g][s * 8 + j] = v;
      }
    }
  }
  float bg[4][4];
#pragma unroll
  for (int g = 0; g < 4; ++g)
#pragma unroll
    for (int r = 0; r < 4; ++r) bg[g][r] = bias[g * H + u0 + r];

  // clamped k indices (W rows >= Din are zero in the fragments, so the clamped
  // finite x values loaded there contribute nothing)
  int kidx[KX][8];
#pragma unroll
  for (int s = 0; s < KX; ++s)
#pragma unroll
    for (int j = 0; j < 8; ++j) kidx[s][j] = min(b_k<BF16>(s, quad, j), Din - 1);

  // ---- x ring: slot j holds step t0 + j
  float xr[D][KX][8];
  const float* xrow = x + (size_t)lseq * T * ldx;
#define GQ_FWD_LOAD(J, TT)                                                                       \
  {                                                                                              \
    const float* xp_ = xrow + (size_t)(TT) * ldx;                                                \
    _Pragma("unroll") for (int s = 0; s < KX; ++s) {                                             \
      if constexpr (VEC) {                                                                       \
        const int kk = min(32 * s + 8 * quad, Din - 8);                                          \
        const float4 a_ = ld4(xp_ + kk), b_ = ld4(xp_ + kk + 4);                                 \
        xr[J][s][0] = a_.x; xr[J][s][1] = a_.y; xr[J][s][2] = a_.z; xr[J][s][3] = a_.w;          \
        xr[J][s][4] = b_.x; xr[J][s][5] = b_.y; xr[J][s][6] = b_.z; xr[J][s][7] = b_.w;          \
      } else {                                                                                   \
        _Pragma("unroll") for (int q = 0; q < 8; ++q) xr[J][s][q] = xp_[kidx[s][q]];             \
      }                                                                                          \
    }                                                                                            \
  }
#pragma unroll
  for (int j = 0; j < D; ++j) GQ_FWD_LOAD(j, min(j, T - 1))

  float c[4] = {0.f, 0.f, 0.f, 0.f};
  __syncthreads();

  int buf = 0;
  for (int t0 = 0; t0 < T; t0 += D) {
#pragma unroll
    for (int j = 0; j < D; ++j) {
      const int t = t0 + j;
      f32x4_t acc[4];
#pragma unroll
      for (int g = 0; g < 4; ++g) acc[g] = f32x4_t{bg[g][0], bg[g][1], bg[g][2], bg[g][3]};
      // input projection from ring slot j (independent of h: off the serial chain)
#pragma unroll
      for (int s = 0; s < KX; ++s) {
        if constexpr (BF16) {
          bf16x8_t bx;
#pragma unroll
          for (int q = 0; q < 8; ++q) bx[q] = (__bf16)xr[j][s][q];
#pragma unroll
          for (int g = 0; g < 4; ++g) acc[g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wfr[g][s], bx, acc[g], 0, 0, 0);
        } else {
#pragma unroll
          for (int q = 0; q < 8; ++q)
#pragma unroll
            for (int g = 0; g < 4; ++g)
              acc[g] = __builtin_amdgcn_mfma_f32_16x16x4f32(wfr[g][s * 8 + q], xr[j][s][q], acc[g], 0, 0, 0);
        }
      }
      GQ_FWD_LOAD(j, min(t + D, T - 1))   // refill slot j: consumed D steps later
      // recurrent part: B = h_{t-1}^T from LDS
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        if constexpr (BF16) {
          const bf16x8_t bh = *reinterpret_cast<const bf16x8_t*>(&hs[buf][col][32 * s + 8 * quad]);
#pragma unroll
          for (int g = 0; g < 4; ++g) acc[g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ufr[g][s], bh, acc[g], 0, 0, 0);
        } else {
          const float bh = hs[buf][col][4 * s + quad];
#pragma unroll
          for (int g = 0; g < 4; ++g) acc[g] = __builtin_amdgcn_mfma_f32_16x16x4f32(ufr[g][s], bh, acc[g], 0, 0, 0);
        }
      }
      float hv[4], iv[4], fv[4], gv[4], ov[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        iv[r] = sigmoidf_fast(acc[0][r]);
        fv[r] = sigmoidf_fast(acc[1][r]);
        gv[r] = tanhf_fast(acc[2][r]);
        ov[r] = sigmoidf_fast(acc[3][r]);
        c[r] = fv[r] * c[r] + iv[r] * gv[r];
        hv[r] = ov[r] * tanhf_fast(c[r]);
      }
      if constexpr (BF16) {
        typedef __bf16 bf16x4_t __attribute__((ext_vector_type(4)));
        bf16x4_t hb = {(__bf16)hv[0], (__bf16)hv[1], (__bf16)hv[2], (__bf16)hv[3]};
        *reinterpret_cast<bf16x4_t*>(&hs[buf ^ 1][col][u0]) = hb;
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r) hs[buf ^ 1][col][u0 + r] = hv[r];
      }
      if (t < T) {   // wave-uniform: only the tail chunk skips
        const size_t o = (size_t)seq * T + t;
        st4(hseq + o * H + u0, hv[0], hv[1], hv[2], hv[3]);
        if constexpr (TRAIN) {
          st4(cseq + o * H + u0, c[0], c[1], c[2], c[3]);
          gate_t<BF16>* gp = gates + o * G4 + u0;
          if constexpr (BF16 && LSTM_BF16_GATES) {
            typedef __bf16 bf16x4_t __attribute__((ext_vector_type(4)));
            *reinterpret_cast<bf16x4_t*>(gp + 0 * H) = bf16x4_t{(__bf16)iv[0], (__bf16)iv[1], (__bf16)iv[2], (__bf16)iv[3]};
            *reinterpret_cast<bf16x4_t*>(gp + 1 * H) = bf16x4_t{(__bf16)fv[0], (__bf16)fv[1], (__bf16)fv[2], (__bf16)fv[3]};
            *reinterpret_cast<bf16x4_t*>(gp + 2 * H) = bf16x4_t{(__bf16)gv[0], (__bf16)gv[1], (__bf16)gv[2], (__bf16)gv[3]};
            *reinterpret_cast<bf16x4_t*>(gp + 3 * H) = bf16x4_t{(__bf16)ov[0], (__bf16)ov[1], (__bf16)ov[2], (__bf16)ov[3]};
          } else {
            st4(gp + 0 * H, iv[0], iv[1], iv[2], iv[3]);
            st4(gp + 1 * H, fv[0], fv[1], fv[2], fv[3]);
            st4(gp + 2 * H, gv[0], gv[1], gv[2], gv[3]);
            st4(gp + 3 * H, ov[0], ov[1], ov[2], ov[3]);
          }
        }
      }
      lds_barrier();
      buf ^= 1;
    }
  }
#undef GQ_FWD_LOAD
}

// ---------------------------------------------------------------- backward
template <int H, bool BF16, int D>
__global__ __launch_bounds__(64 * (H / 16)) void lstm_bwd_kernel(
    const float* __restrict__ dh_out, const gate_t<BF16>* __restrict__ gates, const float* __restrict__ cseq,
    const float* __restrict__ U, void* __restrict__ dz_out, int M, int T) {
  // BF16: dz is stored as bf16 (the weight-gradient / dx passes round it to bf16 for their MFMAs
  // anyway: same results, half the bytes); fp32 reference mode keeps fp32 dz
  using C = LstmCfg<H, BF16>;
  constexpr int G4 = C::G4;
  constexpr int KB = C::KB;
  constexpr int LDZ = BF16 ? G4 + 8 : G4 + 1;
  using elem_t = typename std::conditional<BF16, __bf16, float>::type;
  __shared__ __attribute__((aligned(16))) elem_t zs[2][16][LDZ];

  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int col = lane & 15;
  const int quad = lane >> 4;
  const int ua = 16 * w + col;
  const int u0 = 16 * w + 4 * quad;
  const int row0 = blockIdx.x * 16;
  const int seq = row0 + col;
  const int lseq = min(seq, M - 1);
  const float msk = seq < M ? 1.f : 0.f;

  // A fragments: U rows (dh_rec^T[u][seq] = sum_k U[u][k] dz[seq][k])
  using frag_t = typename std::conditional<BF16, bf16x8_t, float>::type;
  frag_t ua_fr[KB];
#pragma unroll
  for (int s = 0; s < KB; ++s) {
    if constexpr (BF16) {
      bf16x8_t v;
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = (__bf16)U[(size_t)ua * G4 + 32 * s + 8 * quad + j];
      ua_fr[s] = v;
    } else {
      ua_fr[s] = U[(size_t)ua * G4 + 4 * s + quad];
    }
  }

  // ring slot j: reverse step s = s0 + j (t = T-1-s): i,f,g,o, c_t, dh_t
  float4 rg[D][4], rc[D], rd[D];
  auto ld_gate4 = [](const gate_t<BF16>* p) -> float4 {
    if constexpr (BF16 && LSTM_BF16_GATES) {
      const uint2 u = *reinterpret_cast<const uint2*>(p);
      return make_float4(__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u), __uint_as_float(u.y << 16),
                         __uint_as_float(u.y & 0xffff0000u));
    } else {
      return ld4(p);
    }
  };
#define GQ_BWD_LOAD(J, SS)                                                 \
  {                                                                        \
    const int tt = max(T - 1 - (SS), 0);                                   \
    const size_t o = (size_t)lseq * T + tt;                                \
    _Pragma("unroll") for (int g = 0; g < 4; ++g) rg[J][g] = ld_gate4(gates + o * G4 + g * H + u0); \
    rc[J] = ld4(cseq + o * H + u0);                                        \
    rd[J] = ld4(dh_out + o * H + u0);                                      \
  }
#pragma unroll
  for (int j = 0; j < D; ++j) GQ_BWD_LOAD(j, j)

  float dc[4] = {0.f, 0.f, 0.f, 0.f};
  float dhr[4] = {0.f, 0.f, 0.f, 0.f};
  int buf = 0;
  for (int s0 = 0; s0 < T; s0 += D) {
#pragma unroll
    for (int j = 0; j < D; ++j) {
      const int s = s0 + j;
      const int t = T - 1 - s;
      // c_{t-1} lives in slot j+1 (for j = D-1: slot 0, already refilled with s+1)
      const float4 cp4 = rc[(j + 1) % D];
      const float hp = t > 0 ? 1.f : 0.f;
      const float cpv[4] = {cp4.x * hp, cp4.y * hp, cp4.z * hp, cp4.w * hp};
      const float ctv[4] = {rc[j].x, rc[j].y, rc[j].z, rc[j].w};
      const float dhv[4] = {rd[j].x * msk, rd[j].y * msk, rd[j].z * msk, rd[j].w * msk};
      const float giv[4] = {rg[j][0].x, rg[j][0].y, rg[j][0].z, rg[j][0].w};
      const float gfv[4] = {rg[j][1].x, rg[j][1].y, rg[j][1].z, rg[j][1].w};
      const float ggv[4] = {rg[j][2].x, rg[j][2].y, rg[j][2].z, rg[j][2].w};
      const float gov[4] = {rg[j][3].x, rg[j][3].y, rg[j][3].z, rg[j][3].w};
      float zi[4], zf[4], zg[4], zo[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float dh = dhv[r] + dhr[r];
        const float tc = tanhf_fast(ctv[r]);
        const float dc_t = dc[r] + dh * gov[r] * (1.f - tc * tc);
        dc[r] = dc_t * gfv[r];
        zi[r] = dc_t * ggv[r] * giv[r] * (1.f - giv[r]);
        zf[r] = dc_t * cpv[r] * gfv[r] * (1.f - gfv[r]);
        zg[r] = dc_t * giv[r] * (1.f - ggv[r] * ggv[r]);
        zo[r] = dh * tc * gov[r] * (1.f - gov[r]);
      }
      GQ_BWD_LOAD(j, s + D)    // slot j consumed: refill with reverse step s + D
      if constexpr (BF16) {
        typedef __bf16 bf16x4_t __attribute__((ext_vector_type(4)));
        *reinterpret_cast<bf16x4_t*>(&zs[buf][col][0 * H + u0]) = bf16x4_t{(__bf16)zi[0], (__bf16)zi[1], (__bf16)zi[2], (__bf16)zi[3]};
        *reinterpret_cast<bf16x4_t*>(&zs[buf][col][1 * H + u0]) = bf16x4_t{(__bf16)zf[0], (__bf16)zf[1], (__bf16)zf[2], (__bf16)zf[3]};
        *reinterpret_cast<bf16x4_t*>(&zs[buf][col][2 * H + u0]) = bf16x4_t{(__bf16)zg[0], (__bf16)zg[1], (__bf16)zg[2], (__bf16)zg[3]};
        *reinterpret_cast<bf16x4_t*>(&zs[buf][col][3 * H + u0]) = bf16x4_t{(__bf16)zo[0], (__bf16)zo[1], (__bf16)zo[2], (__bf16)zo[3]};
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          zs[buf][col][0 * H + u0 + r] = zi[r];
          zs[buf][col][1 * H + u0 + r] = zf[r];
          zs[buf][col][2 * H + u0 + r] = zg[r];
          zs[buf][col][3 * H + u0 + r] = zo[r];
        }
      }
      if (t >= 0) {   // wave-uniform
        if constexpr (BF16) {
          typedef __bf16 bf16x4_t __attribute__((ext_vector_type(4)));
          __bf16* o = reinterpret_cast<__bf16*>(dz_out) + ((size_t)seq * T + t) * G4 + u0;
          *reinterpret_cast<bf16x4_t*>(o + 0 * H) = bf16x4_t{(__bf16)zi[0], (__bf16)zi[1], (__bf16)zi[2], (__bf16)zi[3]};
          *reinterpret_cast<bf16x4_t*>(o + 1 * H) = bf16x4_t{(__bf16)zf[0], (__bf16)zf[1], (__bf16)zf[2], (__bf16)zf[3]};
          *reinterpret_cast<bf16x4_t*>(o + 2 * H) = bf16x4_t{(__bf16)zg[0], (__bf16)zg[1], (__bf16)zg[2], (__bf16)zg[3]};
          *reinterpret_cast<bf16x4_t*>(o + 3 * H) = bf16x4_t{(__bf16)zo[0], (__bf16)zo[1], (__bf16)zo[2], (__bf16)zo[3]};
        } else {
          float* o = reinterpret_cast<float*>(dz_out) + ((size_t)seq * T + t) * G4 + u0;
          st4(o + 0 * H, zi[0], zi[1], zi[2], zi[3]);
          st4(o + 1 * H, zf[0], zf[1], zf[2], zf[3]);
          st4(o + 2 * H, zg[0], zg[1], zg[2], zg[3]);
          st4(o + 3 * H, zo[0], zo[1], zo[2], zo[3]);
        }
      }
      lds_barrier();
      f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int k = 0; k < KB; ++k) {
        if constexpr (BF16) {
          const bf16x8_t bz = *reinterpret_cast<const bf16x8_t*>(&zs[buf][col][32 * k + 8 * quad]);
          acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ua_fr[k], bz, acc, 0, 0, 0);
        } else {
          const float bz = zs[buf][col][4 * k + quad];
          acc = __builtin_amdgcn_mfma_f32_16x16x4f32(ua_fr[k], bz, acc, 0, 0, 0);
        }
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) dhr[r] = acc[r];
      buf ^= 1;
    }
  }
#undef GQ_BWD_LOAD
}

// ---------------------------------------------------------------- host side
// Ring depth D: enough steps in flight to cover an L2/HBM miss, while
// D x (VMEM ops per step) stays below the 63-entry vmcnt counter.
template <int H, bool BF16, bool TRAIN, int KX, bool VEC>
void launch_fwd_cfg(dim3 grid, dim3 block, hipStream_t st, const float* x, const float* W, const float* U,
                    const float* b, float* h, float* c, void* g, int M, int T, int Din, int ldx) {
  constexpr int loads = VEC ? 2 * KX : 8 * KX;
  constexpr int ops = loads + (TRAIN ? 6 : 1);
  constexpr int Dv = 56 / ops < 2 ? 2 : (56 / ops > 8 ? 8 : 56 / ops);
  constexpr int D = (H >= 128 || !BF16) ? 2 : Dv;
  hipLaunchKernelGGL((lstm_fwd_kernel<H, BF16, TRAIN, KX, D, VEC>), grid, block, 0, st, x, W, U, b, h, c,
                     reinterpret_cast<gate_t<BF16>*>(g), M, T, Din, ldx);
}

template <int H, bool BF16, bool TRAIN>
void launch_fwd_h(const float* x, const float* W, const float* U, const float* b, float* h, float* c, void* g,
                  int M, int T, int Din, int ldx, hipStream_t st) {
  dim3 grid((M + 15) / 16), block(64 * (H / 16));
  const int kx = (Din + 31) / 32;
  const bool vec = BF16 && Din % 8 == 0 && ldx % 4 == 0 && (reinterpret_cast<uintptr_t>(x) % 16) == 0;
#define GQ_KX(KXV)                                                                                           \
  if (vec) launch_fwd_cfg<H, BF16, TRAIN, KXV, true>(grid, block, st, x, W, U, b, h, c, g, M, T, Din, ldx);  \
  else launch_fwd_cfg<H, BF16, TRAIN, KXV, false>(grid, block, st, x, W, U, b, h, c, g, M, T, Din, ldx);
  if (kx == 1) { GQ_KX(1) }
  else if (kx == 2) { GQ_KX(2) }
  else if (kx <= 4) { GQ_KX(4) }
  else TORCH_CHECK(false, "gnnqc lstm: input width ", Din, " > 128 is not supported by the fused kernel");
#undef GQ_KX
}

template <bool BF16, bool TRAIN>
void launch_fwd(int H, const float* x, const float* W, const float* U, const float* b, float* h, float* c, void* g,
                int M, int T, int Din, int ldx, hipStream_t st) {
  switch (H) {
    case 16: launch_fwd_h<16, BF16, TRAIN>(x, W, U, b, h, c, g, M, T, Din, ldx, st); break;
    case 32: launch_fwd_h<32, BF16, TRAIN>(x, W, U, b, h, c, g, M, T, Din, ldx, st); break;
    case 64: launch_fwd_h<64, BF16, TRAIN>(x, W, U, b, h, c, g, M, T, Din, ldx, st); break;
    case 128: launch_fwd_h<128, BF16, TRAIN>(x, W, U, b, h, c, g, M, T, Din, ldx, st); break;
    default: TORCH_CHECK(false, "gnnqc lstm: unsupported hidden size ", H, " (16, 32, 64, 128)");
  }
}

template <int H, bool BF16>
constexpr int bwd_ring() { return (H >= 128 || !BF16) ? 3 : 5; }   // 10 VMEM ops per step

template <bool BF16>
void launch_bwd(int H, const float* dh, const void* gv, const float* c, const float* U, void* dz, int M, int T,
                hipStream_t st) {
  const gate_t<BF16>* g = reinterpret_cast<const gate_t<BF16>*>(gv);
  dim3 grid((M + 15) / 16);
  switch (H) {
#define GQ_CASE(HH)                                                                                       \
  case HH:                                                                                                \
    hipLaunchKernelGGL((lstm_bwd_kernel<HH, BF16, bwd_ring<HH, BF16>()>), grid, dim3(64 * (HH / 16)), 0, st, \
                       dh, g, c, U, dz, M, T);                                                            \
    break;
    GQ_CASE(16) GQ_CASE(32) GQ_CASE(64) GQ_CASE(128)
#undef GQ_CASE
    default:
      TORCH_CHECK(false, "gnnqc lstm: unsupported hidden size ", H);
  }
}

std::vector<at::Tensor> lstm_fwd(const at::Tensor& x, const at::Tensor& W, const at::Tensor& U, const at::Tensor& b,
                                 bool train, bool bf16) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kFloat, "x must be a float32 GPU tensor");
  TORCH_CHECK(x.dim() == 3 && x.stride(2) == 1 && x.stride(0) == x.size(1) * x.stride(1),
              "x must be [M, T, Din] with unit inner stride (row padding allowed)");
  check_f32_cuda(W, "W");
  check_f32_cuda(U, "U");
  check_f32_cuda(b, "b");
  const int M = x.size(0), T = x.size(1), Din = x.size(2), H = U.size(0);
  const int ldx = x.stride(1);
  TORCH_CHECK(U.size(1) == 4 * H && W.size(0) == Din && W.size(1) == 4 * H && b.numel() == 4 * H,
              "lstm_fwd: weight shapes do not match x / U");
  TORCH_CHECK(Din >= 1, "lstm_fwd: empty input width");
  c10::DeviceGuard guard(x.device());
  auto opt = x.options();
  const int Mp = (M + 15) / 16 * 16;   // stores go to whole 16-row tiles
  at::Tensor h = at::empty({Mp, T, H}, opt);
  at::Tensor c = train ? at::empty({Mp, T, H}, opt) : at::empty({0}, opt);
  at::Tensor g = train ? at::empty({Mp, T, 4 * H}, (bf16 && LSTM_BF16_GATES) ? opt.dtype(at::kBFloat16) : opt)
                        : at::empty({0}, opt);
  auto cut = [&](at::Tensor t) { return (train && Mp != M) ? t.narrow(0, 0, M) : t; };
  if (M == 0 || T == 0) return {h.narrow(0, 0, M), cut(c), cut(g)};
  auto st = stream();
  const float *xp = x.data_ptr<float>(), *Wp = W.data_ptr<float>(), *Up = U.data_ptr<float>(), *bp = b.data_ptr<float>();
  float* hp = h.data_ptr<float>();
  float* cp = train ? c.data_ptr<float>() : nullptr;
  void* gp = train ? g.data_ptr() : nullptr;
  if (bf16) {
    if (train) launch_fwd<true, true>(H, xp, Wp, Up, bp, hp, cp, gp, M, T, Din, ldx, st);
    else launch_fwd<true, false>(H, xp, Wp, Up, bp, hp, cp, gp, M, T, Din, ldx, st);
  } else {
    if (train) launch_fwd<false, true>(H, xp, Wp, Up, bp, hp, cp, gp, M, T, Din, ldx, st);
    else launch_fwd<false, false>(H, xp, Wp, Up, bp, hp, cp, gp, M, T, Din, ldx, st);
  }
  GQ_LAUNCH_CHECK();
  return {Mp == M ? h : h.narrow(0, 0, M), cut(c), cut(g)};
}

at::Tensor lstm_bwd(const at::Tensor& dh, const at::Tensor& gates, const at::Tensor& cseq, const at::Tensor& U,
                    bool bf16) {
  check_f32_cuda(dh, "dh");
  TORCH_CHECK(gates.is_cuda() && gates.is_contiguous() &&
                  gates.scalar_type() == ((bf16 && LSTM_BF16_GATES) ? at::kBFloat16 : at::kFloat),
              "lstm_bwd: gates must be the forward's (bf16 in bf16 mode, fp32 otherwise)");
  check_f32_cuda(cseq, "cseq");
  check_f32_cuda(U, "U");
  const int M = dh.size(0), T = dh.size(1), H = U.size(0);
  TORCH_CHECK(dh.size(2) == H && gates.size(0) == M && gates.size(1) == T && gates.size(2) == 4 * H &&
                  cseq.size(0) == M && cseq.size(1) == T && cseq.size(2) == H, "lstm_bwd: shape mismatch");
  c10::DeviceGuard guard(dh.device());
  const int Mp = (M + 15) / 16 * 16;
  at::Tensor dz = at::empty({Mp, T, 4 * H}, dh.options().dtype(bf16 ? at::kBFloat16 : at::kFloat));
  if (M == 0 || T == 0) return dz.narrow(0, 0, M);
  auto st = stream();
  if (bf16) launch_bwd<true>(H, dh.data_ptr<float>(), gates.data_ptr(), cseq.data_ptr<float>(), U.data_ptr<float>(), dz.data_ptr(), M, T, st);
  else launch_bwd<false>(H, dh.data_ptr<float>(), gates.data_ptr(), cseq.data_ptr<float>(), U.data_ptr<float>(), dz.data_ptr(), M, T, st);
  GQ_LAUNCH_CHECK();
  return Mp == M ? dz : dz.narrow(0, 0, M);
}

}  // namespace gq

TORCH_LIBRARY_IMPL(gnnqc, CUDA, m) {
  m.impl("lstm_fwd", &gq::lstm_fwd);
  m.impl("lstm_bwd", &gq::lstm_bwd);
}
