// Persistent LSTM recurrence for gfx950.
//
// Keras LSTM semantics (gate order i,f,c,o; sigmoid recurrent activation, tanh
// activation, zero initial state) as used by the reference TimeLayer
// (libs/create_model.py:61-79). The input projection x@W+b for all T is one
// library GEMM done by the caller; this kernel runs the serial part:
//
//   forward : z_t = xp_t + h_{t-1} U ;  c_t = f c_{t-1} + i g ;  h_t = o tanh(c_t)
//   backward: BPTT producing dz_t (pre-activation gate grads) for all t; the
//             weight/input grads are then plain GEMMs over all (seq, t).
//
// Layout / mapping (one launch for all T steps, state in registers):
//   * workgroup = 16 sequences (MFMA rows) x all H units; wave w owns units
//     [16w, 16w+16) of ALL FOUR gates, so with the 16x16 MFMA C layout
//     (col = lane&15 -> unit, rows 4*(lane>>4)+r -> sequence) the cell update is
//     lane-local: c lives in 4 VGPRs per lane for the whole sequence.
//   * U is converted to bf16 MFMA B-fragments ONCE and kept in VGPRs
//     (<= 64 VGPRs at H = 128); only h_{t-1} (bf16, 16 x H) crosses LDS each step,
//     double buffered so one barrier per step suffices.
//   * BF16=false uses the exact f32-input MFMA (v_mfma_f32_16x16x4_f32) instead -
//     the numerics reference path.
//   * backward mirrors it: dz (bf16) goes through LDS and dh_rec = dz U^T is a
//     K = 4H MFMA chain against register-resident U^T fragments.
#include "common.h"

namespace gq {

template <int H, bool BF16>
struct LstmCfg {
  static constexpr int NW = H / 16;                  // waves per workgroup
  static constexpr int G4 = 4 * H;
  static constexpr int KP = BF16 ? ((H + 31) / 32) * 32 : H;   // padded K (forward)
  static constexpr int KS = BF16 ? KP / 32 : H / 4;             // k-steps forward
  static constexpr int KB = BF16 ? G4 / 32 : G4 / 4;            // k-steps backward (K = 4H)
};

// ---------------------------------------------------------------- forward
template <int H, bool BF16, bool TRAIN>
__global__ __launch_bounds__(64 * (H / 16)) void lstm_fwd_kernel(
    const float* __restrict__ xp, const float* __restrict__ U, float* __restrict__ hseq,
    float* __restrict__ cseq, float* __restrict__ gates, int M, int T) {
  using C = LstmCfg<H, BF16>;
  constexpr int G4 = C::G4;
  constexpr int LDH = BF16 ? C::KP + 8 : H + 1;   // LDS row stride (elements)
  using elem_t = typename std::conditional<BF16, __bf16, float>::type;
  __shared__ __attribute__((aligned(16))) elem_t hs[2][16][LDH];

  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int col = lane & 15;
  const int quad = lane >> 4;
  const int u = 16 * w + col;
  const int row0 = blockIdx.x * 16;

  // zero both h buffers (incl. padding)
  for (int i = threadIdx.x; i < 2 * 16 * LDH; i += blockDim.x) (&hs[0][0][0])[i] = elem_t(0.0f);

  // register-resident recurrent weights
  constexpr int KS = C::KS;
  typename std::conditional<BF16, bf16x8_t, float>::type bfr[4][KS];
#pragma unroll
  for (int g = 0; g < 4; ++g) {
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      if constexpr (BF16) {
        bf16x8_t v;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int k = 32 * s + 8 * quad + j;
          v[j] = (__bf16)(k < H ? U[k * G4 + g * H + u] : 0.0f);
        }
        bfr[g][s] = v;
      } else {
        const int k = 4 * s + quad;
        bfr[g][s] = U[k * G4 + g * H + u];
      }
    }
  }

  int seq[4];
  bool ok[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    seq[r] = row0 + 4 * quad + r;
    ok[r] = seq[r] < M;
  }
  float c[4] = {0.f, 0.f, 0.f, 0.f};
  float xn[4][4];
#pragma unroll
  for (int g = 0; g < 4; ++g)
#pragma unroll
    for (int r = 0; r < 4; ++r)
      xn[g][r] = ok[r] ? xp[((size_t)seq[r] * T + 0) * G4 + g * H + u] : 0.f;
  __syncthreads();

  int buf = 0;
  for (int t = 0; t < T; ++t) {
    f32x4_t acc[4];
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[g][r] = xn[g][r];
    // prefetch next step's input projection (latency hidden by the MFMA chain)
    if (t + 1 < T) {
#pragma unroll
      for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          xn[g][r] = ok[r] ? xp[((size_t)seq[r] * T + t + 1) * G4 + g * H + u] : 0.f;
    }
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      if constexpr (BF16) {
        const bf16x8_t a = *reinterpret_cast<const bf16x8_t*>(&hs[buf][col][32 * s + 8 * quad]);
#pragma unroll
        for (int g = 0; g < 4; ++g)
          acc[g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bfr[g][s], acc[g], 0, 0, 0);
      } else {
        const float a = hs[buf][col][4 * s + quad];
#pragma unroll
        for (int g = 0; g < 4; ++g)
          acc[g] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, bfr[g][s], acc[g], 0, 0, 0);
      }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float ig = sigmoidf_fast(acc[0][r]);
      const float fg = sigmoidf_fast(acc[1][r]);
      const float gg = tanhf_fast(acc[2][r]);
      const float og = sigmoidf_fast(acc[3][r]);
      c[r] = fg * c[r] + ig * gg;
      const float h = og * tanhf_fast(c[r]);
      hs[buf ^ 1][4 * quad + r][u] = elem_t(h);
      if (ok[r]) {
        const size_t o = ((size_t)seq[r] * T + t);
        hseq[o * H + u] = h;
        if constexpr (TRAIN) {
          cseq[o * H + u] = c[r];
          gates[o * G4 + 0 * H + u] = ig;
          gates[o * G4 + 1 * H + u] = fg;
          gates[o * G4 + 2 * H + u] = gg;
          gates[o * G4 + 3 * H + u] = og;
        }
      }
    }
    __syncthreads();
    buf ^= 1;
  }
}

// ---------------------------------------------------------------- backward
template <int H, bool BF16>
__global__ __launch_bounds__(64 * (H / 16)) void lstm_bwd_kernel(
    const float* __restrict__ dh_out, const float* __restrict__ gates, const float* __restrict__ cseq,
    const float* __restrict__ U, float* __restrict__ dz_out, int M, int T) {
  using C = LstmCfg<H, BF16>;
  constexpr int G4 = C::G4;
  constexpr int LDZ = BF16 ? G4 + 8 : G4 + 1;
  using elem_t = typename std::conditional<BF16, __bf16, float>::type;
  __shared__ __attribute__((aligned(16))) elem_t zs[2][16][LDZ];

  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int col = lane & 15;
  const int quad = lane >> 4;
  const int u = 16 * w + col;
  const int row0 = blockIdx.x * 16;

  // U^T fragments: B[k][n] = U[n][k] with n = u (this wave's unit), k over 4H
  constexpr int KB = C::KB;
  typename std::conditional<BF16, bf16x8_t, float>::type bt[KB];
#pragma unroll
  for (int s = 0; s < KB; ++s) {
    if constexpr (BF16) {
      bf16x8_t v;
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = (__bf16)U[(size_t)u * G4 + 32 * s + 8 * quad + j];
      bt[s] = v;
    } else {
      bt[s] = U[(size_t)u * G4 + 4 * s + quad];
    }
  }

  int seq[4];
  bool ok[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    seq[r] = row0 + 4 * quad + r;
    ok[r] = seq[r] < M;
  }
  float dc[4] = {0.f, 0.f, 0.f, 0.f};
  float dhr[4] = {0.f, 0.f, 0.f, 0.f};

  // register prefetch of step t's saved activations
  float gi[4], gf[4], gg[4], go[4], ct[4], cp[4], dho[4];
#define GQ_LOAD_STEP(TT)                                                    \
  _Pragma("unroll") for (int r = 0; r < 4; ++r) {                           \
    const size_t o = (size_t)(ok[r] ? seq[r] : 0) * T + (TT);               \
    const float msk = ok[r] ? 1.f : 0.f;                                    \
    gi[r] = msk * gates[o * G4 + 0 * H + u];                                \
    gf[r] = msk * gates[o * G4 + 1 * H + u];                                \
    gg[r] = msk * gates[o * G4 + 2 * H + u];                                \
    go[r] = msk * gates[o * G4 + 3 * H + u];                                \
    ct[r] = msk * cseq[o * H + u];                                          \
    cp[r] = (TT) > 0 ? msk * cseq[(o - 1) * H + u] : 0.f;                   \
    dho[r] = msk * dh_out[o * H + u];                                       \
  }
  GQ_LOAD_STEP(T - 1)
  int buf = 0;
  for (int t = T - 1; t >= 0; --t) {
    float zi[4], zf[4], zg[4], zo[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float dh = dho[r] + dhr[r];
      const float tc = tanhf_fast(ct[r]);
      const float dc_t = dc[r] + dh * go[r] * (1.f - tc * tc);
      const float d_o = dh * tc;
      const float d_i = dc_t * gg[r];
      const float d_g = dc_t * gi[r];
      const float d_f = dc_t * cp[r];
      dc[r] = dc_t * gf[r];
      zi[r] = d_i * gi[r] * (1.f - gi[r]);
      zf[r] = d_f * gf[r] * (1.f - gf[r]);
      zg[r] = d_g * (1.f - gg[r] * gg[r]);
      zo[r] = d_o * go[r] * (1.f - go[r]);
    }
    // stage dz: global (fp32, for weight GEMMs) and LDS (MFMA operand)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int rr = 4 * quad + r;
      zs[buf][rr][0 * H + u] = elem_t(zi[r]);
      zs[buf][rr][1 * H + u] = elem_t(zf[r]);
      zs[buf][rr][2 * H + u] = elem_t(zg[r]);
      zs[buf][rr][3 * H + u] = elem_t(zo[r]);
      if (ok[r]) {
        const size_t o = ((size_t)seq[r] * T + t) * G4;
        dz_out[o + 0 * H + u] = zi[r];
        dz_out[o + 1 * H + u] = zf[r];
        dz_out[o + 2 * H + u] = zg[r];
        dz_out[o + 3 * H + u] = zo[r];
      }
    }
    if (t > 0) { GQ_LOAD_STEP(t - 1) }
    __syncthreads();
    if (t > 0) {
      f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < KB; ++s) {
        if constexpr (BF16) {
          const bf16x8_t a = *reinterpret_cast<const bf16x8_t*>(&zs[buf][col][32 * s + 8 * quad]);
          acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bt[s], acc, 0, 0, 0);
        } else {
          const float a = zs[buf][col][4 * s + quad];
          acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, bt[s], acc, 0, 0, 0);
        }
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) dhr[r] = acc[r];
    }
    buf ^= 1;
  }
#undef GQ_LOAD_STEP
}

// ---------------------------------------------------------------- host side
template <bool BF16, bool TRAIN>
void launch_fwd(int H, const float* xp, const float* U, float* h, float* c, float* g, int M, int T,
                hipStream_t st) {
  dim3 grid((M + 15) / 16);
  switch (H) {
#define GQ_CASE(HH)                                                                            \
  case HH:                                                                                     \
    hipLaunchKernelGGL((lstm_fwd_kernel<HH, BF16, TRAIN>), grid, dim3(64 * (HH / 16)), 0, st, \
                       xp, U, h, c, g, M, T);                                                  \
    break;
    GQ_CASE(16) GQ_CASE(32) GQ_CASE(64) GQ_CASE(128)
    case 256:
      if constexpr (BF16) {
        hipLaunchKernelGGL((lstm_fwd_kernel<256, BF16, TRAIN>), grid, dim3(64 * 16), 0, st, xp, U, h, c, g, M, T);
        break;
      }
      [[fallthrough]];
#undef GQ_CASE
    default:
      TORCH_CHECK(false, "gnnqc lstm: unsupported hidden size ", H, BF16 ? "" : " (fp32 path supports 16..128)");
  }
}

template <bool BF16>
void launch_bwd(int H, const float* dh, const float* g, const float* c, const float* U, float* dz, int M,
                int T, hipStream_t st) {
  dim3 grid((M + 15) / 16);
  switch (H) {
#define GQ_CASE(HH)                                                                                  \
  case HH:                                                                                           \
    hipLaunchKernelGGL((lstm_bwd_kernel<HH, BF16>), grid, dim3(64 * (HH / 16)), 0, st, dh, g, c, U, \
                       dz, M, T);                                                                    \
    break;
    GQ_CASE(16) GQ_CASE(32) GQ_CASE(64) GQ_CASE(128)
    case 256:
      if constexpr (BF16) {
        hipLaunchKernelGGL((lstm_bwd_kernel<256, BF16>), grid, dim3(64 * 16), 0, st, dh, g, c, U, dz, M, T);
        break;
      }
      [[fallthrough]];
#undef GQ_CASE
    default:
      TORCH_CHECK(false, "gnnqc lstm: unsupported hidden size ", H, BF16 ? "" : " (fp32 path supports 16..128)");
  }
}

std::vector<at::Tensor> lstm_fwd(const at::Tensor& xp, const at::Tensor& U, bool train, bool bf16) {
  check_f32_cuda(xp, "xp");
  check_f32_cuda(U, "U");
  TORCH_CHECK(xp.dim() == 3, "xp must be [M, T, 4H]");
  const int M = xp.size(0), T = xp.size(1), H = U.size(0);
  TORCH_CHECK(U.size(1) == 4 * H && xp.size(2) == 4 * H, "shape mismatch between xp and U");
  TORCH_CHECK(H % 16 == 0 && H >= 16 && H <= 256, "hidden size must be 16..256, multiple of 16");
  c10::DeviceGuard guard(xp.device());
  auto opt = xp.options();
  at::Tensor h = at::empty({M, T, H}, opt);
  at::Tensor c = train ? at::empty({M, T, H}, opt) : at::empty({0}, opt);
  at::Tensor g = train ? at::empty({M, T, 4 * H}, opt) : at::empty({0}, opt);
  if (M == 0 || T == 0) return {h, c, g};
  auto st = stream();
  if (bf16) {
    if (train) launch_fwd<true, true>(H, xp.data_ptr<float>(), U.data_ptr<float>(), h.data_ptr<float>(), c.data_ptr<float>(), g.data_ptr<float>(), M, T, st);
    else launch_fwd<true, false>(H, xp.data_ptr<float>(), U.data_ptr<float>(), h.data_ptr<float>(), nullptr, nullptr, M, T, st);
  } else {
    if (train) launch_fwd<false, true>(H, xp.data_ptr<float>(), U.data_ptr<float>(), h.data_ptr<float>(), c.data_ptr<float>(), g.data_ptr<float>(), M, T, st);
    else launch_fwd<false, false>(H, xp.data_ptr<float>(), U.data_ptr<float>(), h.data_ptr<float>(), nullptr, nullptr, M, T, st);
  }
  GQ_LAUNCH_CHECK();
  return {h, c, g};
}

at::Tensor lstm_bwd(const at::Tensor& dh, const at::Tensor& gates, const at::Tensor& cseq, const at::Tensor& U,
                    bool bf16) {
  check_f32_cuda(dh, "dh");
  check_f32_cuda(gates, "gates");
  check_f32_cuda(cseq, "cseq");
  check_f32_cuda(U, "U");
  const int M = dh.size(0), T = dh.size(1), H = U.size(0);
  TORCH_CHECK(dh.size(2) == H && gates.size(2) == 4 * H && cseq.size(2) == H, "lstm_bwd shape mismatch");
  TORCH_CHECK(gates.size(0) == M && cseq.size(0) == M && gates.size(1) == T && cseq.size(1) == T,
              "lstm_bwd shape mismatch");
  c10::DeviceGuard guard(dh.device());
  at::Tensor dz = at::empty({M, T, 4 * H}, dh.options());
  if (M == 0 || T == 0) return dz;
  auto st = stream();
  if (bf16) launch_bwd<true>(H, dh.data_ptr<float>(), gates.data_ptr<float>(), cseq.data_ptr<float>(), U.data_ptr<float>(), dz.data_ptr<float>(), M, T, st);
  else launch_bwd<false>(H, dh.data_ptr<float>(), gates.data_ptr<float>(), cseq.data_ptr<float>(), U.data_ptr<float>(), dz.data_ptr<float>(), M, T, st);
  GQ_LAUNCH_CHECK();
  return dz;
}

}  // namespace gq

TORCH_LIBRARY_IMPL(gnnqc, CUDA, m) {
  m.impl("lstm_fwd", &gq::lstm_fwd);
  m.impl("lstm_bwd", &gq::lstm_bwd);
}
