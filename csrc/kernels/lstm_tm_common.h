// Pieces shared by the time-major LSTM kernels (lstm_tm.hip, lstm_chain.hip).
#pragma once
#include "common.h"

#include <type_traits>

namespace gq {

typedef __bf16 bf16x4_t __attribute__((ext_vector_type(4)));

// Saved LSTM gates (i, f, g, o of one cell and step) are stored as 4 x bf16 = 8 bytes: the
// forward's largest stream and the backward's largest read (was 16 bytes of fp32). Gate
// activations lie in (0, 1) / (-1, 1), so bf16 keeps ~3 significant digits, the precision of
// the bf16 MFMA operands they are combined with.
__device__ __forceinline__ uint2 gates_pack(float i, float f, float g, float o) {
  const bf16x4_t v = bf16x4_t{(__bf16)i, (__bf16)f, (__bf16)g, (__bf16)o};
  return *reinterpret_cast<const uint2*>(&v);
}
__device__ __forceinline__ float4 gates_unpack(uint2 u) {
  return make_float4(__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u), __uint_as_float(u.y << 16),
                     __uint_as_float(u.y & 0xffff0000u));
}

// A wave-uniform predicate the compiler can SEE is uniform (an SGPR): branches on it are
// scalar, so no exec-mask join -> no conservative s_waitcnt vmcnt(0) around the loads
// inside (measured: with threadIdx-derived predicates every step drained the load ring).
__device__ __forceinline__ bool wave_uniform(bool p) { return __builtin_amdgcn_readfirstlane((int)p) != 0; }

template <int H>
struct TMC {
  static constexpr int CPL = H > 64 ? H / 64 : 1;   // cells per lane
  static constexpr int NW = H / (4 * CPL);          // waves per 16-sequence tile (<= 16)
  static constexpr int NT = 64 * NW;
  static constexpr int G4 = 4 * H;
  static constexpr int KPH = ((H + 31) / 32) * 32;
  static constexpr int KSH = KPH / 32;              // K = H steps (forward recurrent part)
  static constexpr int KB = G4 / 32;                // K = 4H steps (backward)
  static constexpr int HP = H + 4;                  // row pitch of fp32 [16][H] LDS tiles: the
                                                    // per-cell accesses (16 rows x 4 units per
                                                    // wave) then hit 64 distinct banks
};

// ---- tile streamer: granules of GR floats of one contiguous tile, wave-uniform loaders
template <int GR>
struct Granule {
  float v[4];
  __device__ __forceinline__ void load(const float* p) {
    if constexpr (GR == 4) {
      const float4 a = *reinterpret_cast<const float4*>(p);
      v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
    } else if constexpr (GR == 2) {
      const float2 a = *reinterpret_cast<const float2*>(p);
      v[0] = a.x; v[1] = a.y;
    } else {
      v[0] = *p;
    }
  }
  __device__ __forceinline__ void zero() { v[0] = v[1] = v[2] = v[3] = 0.f; }
  __device__ __forceinline__ __bf16 bf(int q) const { return (__bf16)v[q]; }
};

// The same GR-element granule from bf16 data, kept as the raw bits: a ring slot's load is waited for
// where the value is used (staged into LDS as bf16), not at the load
template <int GR>
struct GranuleH {
  using R = std::conditional_t<GR == 4, uint2, std::conditional_t<GR == 2, unsigned, unsigned short>>;
  R r;
  __device__ __forceinline__ void load(const __bf16* p) { r = *reinterpret_cast<const R*>(p); }
  __device__ __forceinline__ __bf16 bf(int q) const {
    unsigned w;
    if constexpr (GR == 4) w = q < 2 ? r.x : r.y;
    else w = (unsigned)r;
    return __builtin_bit_cast(__bf16, (unsigned short)((q & 1) ? (w >> 16) : (w & 0xffffu)));
  }
};

// ---- fused MaxPooling1D(P) (valid, stride P) of a stored h sequence (the chain forward's last
// stage, lstm_chain.hip, whose pooled output leaves the chain). Each storer lane owns
// one float4 granule of the [16][H] tile for the whole sequence, so the running max and the
// byte argmax (first maximum wins, like TF's MaxPoolGrad) stay in its registers; the pooled
// granule and its 4 argmax bytes are written when a window closes. Layout = maxpool1d_fwd's
// on the time-major tensor: pooled [T/P][Mp][H] fp32, argmax [T/P][Mp][H] uint8.
struct PoolAcc {
  float4 m;
  unsigned idx;
  __device__ __forceinline__ void step(const float4& v, int t, int P, int To, float* __restrict__ pout,
                                       unsigned* __restrict__ iout, size_t off, size_t pstep) {
    const int r = t % P;                            // t, P wave-uniform: scalar branches
    if (r == 0) {
      m = v;
      idx = 0u;
    } else {
      const unsigned rb = (unsigned)r;
      if (v.x > m.x) { m.x = v.x; idx = (idx & 0xffffff00u) | rb; }
      if (v.y > m.y) { m.y = v.y; idx = (idx & 0xffff00ffu) | (rb << 8); }
      if (v.z > m.z) { m.z = v.z; idx = (idx & 0xff00ffffu) | (rb << 16); }
      if (v.w > m.w) { m.w = v.w; idx = (idx & 0x00ffffffu) | (rb << 24); }
    }
    if (r == P - 1 && t / P < To) {
      const size_t k = (size_t)(t / P);
      *reinterpret_cast<float4*>(pout + k * pstep + off) = m;
      iout[(k * pstep + off) / 4] = idx;
    }
  }
};

// fused-pool outputs of the chain forward (host)
struct TmPool {
  int P = 0;
  float* out = nullptr;
  unsigned* idx = nullptr;
};

inline TmPool tm_pool_outputs(int P, int T, int Mp, int H, const at::TensorOptions& opt, at::Tensor& pooled,
                              at::Tensor& pidx) {
  TmPool pl;
  if (P <= 0) {
    pooled = at::empty({0}, opt);
    pidx = at::empty({0}, opt.dtype(at::kByte));
    return pl;
  }
  TORCH_CHECK(P <= 255 && T / P >= 1, "lstm_tm: pool size must be 1..255 and <= T");
  pooled = at::empty({T / P, Mp, H}, opt);
  pidx = at::empty({T / P, Mp, H}, opt.dtype(at::kByte));
  pl.P = P;
  pl.out = pooled.data_ptr<float>();
  pl.idx = reinterpret_cast<unsigned*>(pidx.data_ptr<uint8_t>());
  return pl;
}

// ---- time4 (H = 128, Din <= 64) forward and backward A-fragment images (time4_head.hip's 512-thread layout:
// wave w of 8, cell cc of 4, lane = (quad, col)): U fragments [w][cc][s < 4][lane], then W
// fragments [w][cc][s < 2][lane], each 8 bf16. Gathering them from the [K][4H] weights touches 16
// cache lines per load instruction, so the chain forward's idle workgroups build this image once per
// step and the time4 kernel reads it with lane-contiguous 16-B loads.
constexpr int T4PK_U = 8 * 4 * 4 * 64;
constexpr int T4PK_W = 8 * 4 * 2 * 64;
constexpr int T4PK_N = T4PK_U + T4PK_W;
// backward image (time4_head.hip t4_head_bwd_kernel): U rows [w][s < 16][lane] = U[16w + col][32s + 8quad ..],
// then W rows [w][s < 8][lane] = W[16 (w & 3) + col][256 (w >> 2) + 32s + 8quad ..] (rows >= Dw zero)
constexpr int T4PK_BU = 8 * 16 * 64;
constexpr int T4PK_BW = 8 * 8 * 64;
constexpr int T4PK_ALL = T4PK_N + T4PK_BU + T4PK_BW;

__device__ __forceinline__ void t4_pack_one(int f, const float* __restrict__ U, const float* __restrict__ W, int Dw,
                                            bf16x8_t* __restrict__ out) {
  if (f >= T4PK_N) {                       // backward fragments: 8 contiguous floats per lane
    const int fb = f - T4PK_N;
    const bool isU = fb < T4PK_BU;
    const int f2 = isU ? fb : fb - T4PK_BU;
    const int lane = f2 & 63, col = lane & 15, quad = lane >> 4;
    const int s = isU ? (f2 >> 6) & 15 : (f2 >> 6) & 7;
    const int w = isU ? f2 >> 10 : f2 >> 9;
    const float* src;
    float m = 1.f;
    if (isU) {
      src = U + (size_t)(16 * w + col) * 512 + 32 * s + 8 * quad;
    } else {
      const int din = 16 * (w & 3) + col;
      m = din < Dw ? 1.f : 0.f;
      src = W + (size_t)min(din, Dw - 1) * 512 + 256 * (w >> 2) + 32 * s + 8 * quad;
    }
    const float4 a = *reinterpret_cast<const float4*>(src), b = *reinterpret_cast<const float4*>(src + 4);
    out[f] = bf16x8_t{(__bf16)(a.x * m), (__bf16)(a.y * m), (__bf16)(a.z * m), (__bf16)(a.w * m),
                      (__bf16)(b.x * m), (__bf16)(b.y * m), (__bf16)(b.z * m), (__bf16)(b.w * m)};
    return;
  }
  const bool isU = f < T4PK_U;
  const int f2 = isU ? f : f - T4PK_U;
  const int lane = f2 & 63;
  const int s = isU ? (f2 >> 6) & 3 : (f2 >> 6) & 1;
  const int cc = isU ? (f2 >> 8) & 3 : (f2 >> 7) & 3;
  const int w = isU ? f2 >> 10 : f2 >> 9;
  const int col = lane & 15, quad = lane >> 4;
  const int gi = w + 8 * cc, au = 4 * gi + (col >> 2), ag = col & 3;
  bf16x8_t v;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int k = 32 * s + 8 * quad + j;
    if (isU) v[j] = (__bf16)U[(size_t)k * 512 + ag * 128 + au];
    else v[j] = (__bf16)(W[(size_t)min(k, Dw - 1) * 512 + ag * 128 + au] * (k < Dw ? 1.f : 0.f));
  }
  out[f] = v;
}

}  // namespace gq
