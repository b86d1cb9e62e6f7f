// Last LSTM layer of the CML TimeLayer (time4: H = 128, last state only) fused with the classifier
// head and the weighted BCE, forward and backward, for gfx950 (libs/create_model.py:61-79 time4,
// :204-239 head; loss libs/fit_model.py:76-111).
//
// After the six pipelined layers (lstm_chain.hip) the CML step used to run time4 and the head as
// five launches (lstm_fwd<128>, head_fwd, head_bwd, lstm_bwd<128>, lstm_dx: ~82 us, latency only,
// plus pad / transpose copies between them). Here: ONE forward kernel (time4's six steps, then
// the head, the loss and the metric accumulation as the epilogue) and ONE backward kernel (the
// head backward as the prologue, then time4's reverse recurrence writing dz for the weight-
// gradient pass and dx - the gradient of the chain's pooled output - for the chain backward).
//
// One 512-thread workgroup per 16-sequence tile. 512 rather than 1024 threads: at 16 waves per
// CU a wave may hold 128 VGPRs, and an H = 128 layer with its recurrent weights resident (the
// forward's U fragments alone are 64 VGPRs at 4 cells per lane) spilled inside the step loop,
// and every spill reload drained the vector-memory counter. At 8 waves a wave holds 256.
//   forward   lane = 4 cells (unit 4(w + 8cc) + quad of sequence col); the MFMA A rows are
//             permuted so a 16x16 tile delivers the i, f, g, o pre-activations of the lane's own
//             cell (as lstm_tm.hip). The whole input sequence of the tile is staged in LDS once.
//   backward  dh_rec^T = U dz^T: wave w owns unit tile w over the full K = 4H (16 MFMAs, U
//             fragments resident); dx^T = W dz^T: din tile w % 4 over gate-column half w / 4.
//             The forward state (gates, c) streams through a 2-deep register ring.
#include "chain_head.h"
#include "common.h"
#include "lstm_tm_common.h"

namespace gq {

int* chain_ctl(int dev);     // lstm_chain.hip: per-device control words ([4] / [5]: head tickets)

constexpr int T4H = 128;                 // hidden size
constexpr int T4G = 4 * T4H;             // gate columns
constexpr int T4NT = 512;                // threads
constexpr int T4NW = T4NT / 64;          // waves
constexpr int T4CPL = T4H * 16 / T4NT;   // cells per lane (4)
constexpr int T4MAXT = 16;               // sequence length bound (the input tile lives in LDS)
constexpr int T4HP = T4H + 4;

struct T4Args {
  const float* x;                        // [T][Mp][Din] (time-major, 16-B aligned rows)
  const float *W, *U, *b;                // [Dw][4H], [H][4H], [4H]
  float* h;                              // [T][Mp][H] (hlast: [Mp][H], the last step only)
  float* g;                              // train: [T][tiles][NW][CPL][64][4]
  float* c;                              // train: [T][tiles][NW][CPL][64][2]: c_t, c_{t-1} (CG: [..][64] c_t)
  uint2* gb;                             // CG train: [T][tiles][NW][CPL][64] packed bf16 gates
  const float* dhT;                      // CG backward: [Mp][H] gradient of the last state
  const float* dhs;                      // CG backward (optional): row scales of dhT (rows >= dhs_n: 0)
  int dhs_n;
  float* prob;                           // CG forward with the head: [Mp] sigmoid outputs
  float* dhg;                            //   and [Mp][H] d prob / d h_{T-1}
  __bf16* dz;                            // backward: [T + 1][Mp][4H] bf16
  float* dx;                             // backward: [T][Mp][Din]
  int T, Mp, Din, Dw, ntiles;
  ChainHead hd;
  int head;
  int hlast;                             // forward: store h of the last step only ([Mp][H])
  long long* trace;                      // [blocks][16] s_memrealtime marks of the last launch (profiling)
  const bf16x8_t* pk;                    // forward: A-fragment image (lstm_tm_common.h), or nullptr
};

__device__ __forceinline__ void t4_mark(long long* tr, int i) {
  if (tr != nullptr && threadIdx.x == 0) tr[blockIdx.x * 16 + i] = (long long)__builtin_amdgcn_s_memrealtime();
}

__device__ __forceinline__ size_t t4_sidx(int t, int ntiles, int tile, int w, int cc, int lane) {
  return ((((size_t)t * ntiles + tile) * T4NW + w) * T4CPL + cc) * 64 + lane;
}

// ------------------------------------------------------------------------------------ forward
// LDS of the integrated-gradients head epilogue (t4_prob_head): part [2][16][AP], z1, a1 / dz1,
// dz2 [16][AP], dh [16][F + 4], the W1 / W2 images
template <int F>
struct T4ProbLds {
  static constexpr int BYTES = (5 * 16 * CH_AP + 16 * (F + 4) + (F + CH_HU) * CH_WP) * 4;
};

// Integrated-gradients epilogue of the standalone forward (CG with a head): the head's sigmoid
// output p of the tile's 16 rows (from h_{T-1} in hl [16][F + 4]) -> prob, and dp / dh_{T-1} ->
// dhg [Mp][F]: the seed of time4_bwd's recurrence for d sum(p) / dx (rows >= M: p = 0, dh = 0).
// Replaces head_prob_fwd / head_prob_bwd (two launches, ~90 us on a 32k-row IG pass). staged:
// the W1 / W2 images in the scratch are still those of an earlier tile of this workgroup.
template <int F>
__device__ __forceinline__ void t4_prob_head(const ChainHead hd, int tile, const float* hl, char* scratch, bool staged,
                                             float* __restrict__ prob, float* __restrict__ dhg) {
  constexpr int HLP = F + 4, PT = 16 * CH_AP;
  float* part = reinterpret_cast<float*>(scratch);   // [2][16][AP]
  float* sz1 = part + 2 * PT;                        // z1
  float* sa1 = sz1 + PT;                             // leaky(z1), then dz1
  float* sdz2 = sa1 + PT;                            // dz2
  float* dh = sdz2 + PT;                             // [16][HLP]
  float* sW1 = dh + 16 * HLP;                        // [F][WP]
  float* sW2 = sW1 + F * CH_WP;                      // [64][WP]
  if (!staged) ch_stage_weights<F>(hd, sW1, sW2);
  const int tid = ch_tid(), w = tid >> 6, j = tid & 63;
  const float w3j = hd.W3[j], b3 = hd.b3[0];
  float z2[2];
  ch_head_z2<F>(hd, sW1, sW2, hl, part, sz1, sa1, z2);
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int r = w + 8 * q, row = tile * 16 + r;
    const float z = wave_sum(ch_leaky(z2[q], hd.alpha2) * w3j) + b3;
    const float p = row < hd.M ? sigmoidf_fast(z) : 0.f;
    sdz2[r * CH_AP + j] = p * (1.f - p) * w3j * ch_dleaky(z2[q], hd.alpha2);
    if (j == 0) prob[row] = p;
  }
  __syncthreads();
  {   // da1 = dz2 W2^T
    const int ot = w & 3, kh = w >> 2;
    ch_put(part + kh * PT, CH_AP, ot, ch_mm_wt<8>(sW2, CH_WP, ot, kh * 32, sdz2, CH_AP));
  }
  __syncthreads();
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int r = w + 8 * q;
    const float da = part[r * CH_AP + j] + part[PT + r * CH_AP + j];
    sa1[r * CH_AP + j] = da * ch_dleaky(sz1[r * CH_AP + j], hd.alpha1);
  }
  __syncthreads();
#pragma unroll
  for (int q = 0; q < F / 16 / CH_NW; ++q) {          // dh = dz1 W1^T
    const int ot = w + CH_NW * q;
    ch_put(dh, HLP, ot, ch_mm_wt<16>(sW1, CH_WP, ot, 0, sa1, CH_AP));
  }
  __syncthreads();
  for (int e = tid; e < 16 * F / 4; e += 64 * CH_NW) {
    const int r = 4 * e / F, k = 4 * e % F;
    *reinterpret_cast<float4*>(dhg + (size_t)(tile * 16 + r) * F + k) = *reinterpret_cast<const float4*>(dh + r * HLP + k);
  }
}

template <int KX, bool CG = false>
struct T4FwdLds {
  static constexpr int XP = 32 * KX + 8;
  static constexpr int XS = T4MAXT * 16 * XP * 2;        // bf16 input tiles of every step
  static constexpr int HS = 2 * 16 * (T4H + 8) * 2;      // bf16 h_{t-1} (double buffer)
  static constexpr int HL = 16 * T4HP * 4;               // fp32 h_{T-1} for the head
  static constexpr int HEAD = CG ? T4ProbLds<T4H>::BYTES : ChainHeadFwdLds<T4H>::BYTES;
  static constexpr int WORK = XS + HS + HL + HEAD;
  static constexpr int STAGE = T4H * (T4G + 8) * 2;       // bf16 U (then W) staged for the fragments
  static constexpr int BYTES = WORK > STAGE ? WORK : STAGE;
};

// Weight rows [rows][4H] (fp32, global) -> bf16 LDS image [rows][4H + 8]: coalesced float4 loads,
// eight in flight per thread. (Gathering the permuted A fragments straight from global memory
// touched 16 cache lines per load instruction: 12 us of prologue per launch, measured.)
__device__ __forceinline__ void t4_stage_rows(__bf16* dst, const float* __restrict__ src, int rows) {
  const int n4 = rows * T4G / 4;
  for (int e0 = threadIdx.x; e0 < n4; e0 += 8 * T4NT) {
    float4 v[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int e = min(e0 + q * T4NT, n4 - 1);
      v[q] = reinterpret_cast<const float4*>(src)[e];
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int e = e0 + q * T4NT;
      if (e < n4) {
        const int k = 4 * e / T4G, c = 4 * e % T4G;
        typedef __bf16 bf4 __attribute__((ext_vector_type(4)));
        *reinterpret_cast<bf4*>(dst + k * (T4G + 8) + c) =
            bf4{(__bf16)v[q].x, (__bf16)v[q].y, (__bf16)v[q].z, (__bf16)v[q].w};
      }
    }
  }
}

// CG (the standalone layer, time4_fwd / time4_bwd): compact saved state - packed bf16 gates and
// c_t only (12 instead of 24 bytes per cell and step) - and workgroups that loop over tiles, so
// the weight fragments are staged once per workgroup rather than once per 16 sequences (an
// integrated-gradients pass runs 32k sequences: 2048 tiles on 256 workgroups). With the head
// (grid = tiles) the loop runs once.
template <bool TRAIN, int KX, bool CG = false>
__global__ __launch_bounds__(T4NT) void t4_head_fwd_kernel(T4Args A) {
  using L = T4FwdLds<KX, CG>;
  constexpr int XP = L::XP;
  __shared__ __attribute__((aligned(16))) char smem[L::BYTES];
  auto xs = reinterpret_cast<__bf16 (*)[16][XP]>(smem);
  auto hs = reinterpret_cast<__bf16 (*)[16][T4H + 8]>(smem + L::XS);
  float* hl = reinterpret_cast<float*>(smem + L::XS + L::HS);
  char* scratch = smem + L::XS + L::HS + L::HL;

  const int T = A.T, Mp = A.Mp, Din = A.Din, Dw = A.Dw, ntiles = A.ntiles;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int col = lane & 15, quad = lane >> 4;

  t4_mark(A.trace, 0);
  bf16x8_t ufr[T4CPL][T4H / 32], wfr[T4CPL][KX];
  f32x4_t bias4[T4CPL];
  int unit[T4CPL];
  if (A.pk != nullptr) {   // the fragment image the chain forward built: lane-contiguous 16-B loads
#pragma unroll
    for (int cc = 0; cc < T4CPL; ++cc) {
      const int gi = w + T4NW * cc;
      unit[cc] = 4 * gi + quad;
#pragma unroll
      for (int s = 0; s < T4H / 32; ++s) ufr[cc][s] = A.pk[((w * T4CPL + cc) * 4 + s) * 64 + lane];
#pragma unroll
      for (int s = 0; s < KX; ++s) wfr[cc][s] = A.pk[T4PK_U + ((w * T4CPL + cc) * 2 + s) * 64 + lane];
      const int u = unit[cc];
      bias4[cc] = f32x4_t{A.b[u], A.b[T4H + u], A.b[2 * T4H + u], A.b[3 * T4H + u]};
    }
  } else {   // weights -> permuted A fragments through an LDS image (see t4_stage_rows)
    __bf16* st = reinterpret_cast<__bf16*>(smem);
    constexpr int SP = T4G + 8;
    t4_stage_rows(st, A.U, T4H);
    __syncthreads();
#pragma unroll
    for (int cc = 0; cc < T4CPL; ++cc) {
      const int gi = w + T4NW * cc;
      const int au = 4 * gi + (col >> 2), ag = col & 3;
      unit[cc] = 4 * gi + quad;
#pragma unroll
      for (int s = 0; s < T4H / 32; ++s) {
        bf16x8_t v;
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = st[(32 * s + 8 * quad + j) * SP + ag * T4H + au];
        ufr[cc][s] = v;
      }
      const int u = unit[cc];
      bias4[cc] = f32x4_t{A.b[u], A.b[T4H + u], A.b[2 * T4H + u], A.b[3 * T4H + u]};
    }
    __syncthreads();
    t4_stage_rows(st, A.W, Dw);
    __syncthreads();
#pragma unroll
    for (int cc = 0; cc < T4CPL; ++cc) {
      const int gi = w + T4NW * cc;
      const int au = 4 * gi + (col >> 2), ag = col & 3;
#pragma unroll
      for (int s = 0; s < KX; ++s) {
        bf16x8_t v;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int k = 32 * s + 8 * quad + j;
          v[j] = (__bf16)((float)st[min(k, Dw - 1) * SP + ag * T4H + au] * (k < Dw ? 1.f : 0.f));
        }
        wfr[cc][s] = v;
      }
    }
    __syncthreads();
  }
  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
  const int row0 = tile * 16;
  // the tile's whole input sequence -> LDS (bf16, channels >= Din zero)
  for (int e = tid; e < T * 16 * XP; e += T4NT) (&xs[0][0][0])[e] = (__bf16)0.f;
  for (int e = tid; e < 2 * 16 * (T4H + 8); e += T4NT) (&hs[0][0][0])[e] = (__bf16)0.f;
  __syncthreads();
  {
    const int n4 = Din / 4, per = 16 * n4;
    for (int e = tid; e < T * per; e += T4NT) {
      const int t = e / per, r = (e % per) / n4, k = 4 * (e % n4);
      const float4 v = *reinterpret_cast<const float4*>(A.x + ((size_t)t * Mp + row0 + r) * Din + k);
      xs[t][r][k] = (__bf16)v.x;
      xs[t][r][k + 1] = (__bf16)v.y;
      xs[t][r][k + 2] = (__bf16)v.z;
      xs[t][r][k + 3] = (__bf16)v.w;
    }
  }
  float c[T4CPL];
#pragma unroll
  for (int cc = 0; cc < T4CPL; ++cc) c[cc] = 0.f;
  __syncthreads();
  t4_mark(A.trace, 1);

  for (int t = 0; t < T; ++t) {
    const int p = t & 1;
    // B fragments once per step (shared by the lane's cells), then the cells' MFMA chains
    // interleaved: 2 x CPL independent accumulators keep the MFMA pipe busy (one chain at a time
    // left each step latency-bound at ~2 us)
    bf16x8_t bx[KX], bh[T4H / 32];
#pragma unroll
    for (int s = 0; s < KX; ++s) bx[s] = *reinterpret_cast<const bf16x8_t*>(&xs[t][col][32 * s + 8 * quad]);
#pragma unroll
    for (int s = 0; s < T4H / 32; ++s) bh[s] = *reinterpret_cast<const bf16x8_t*>(&hs[p][col][32 * s + 8 * quad]);
    f32x4_t accx[T4CPL], acch[T4CPL];
#pragma unroll
    for (int cc = 0; cc < T4CPL; ++cc) {
      accx[cc] = bias4[cc];
      acch[cc] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int s = 0; s < KX; ++s)
#pragma unroll
      for (int cc = 0; cc < T4CPL; ++cc) accx[cc] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wfr[cc][s], bx[s], accx[cc], 0, 0, 0);
#pragma unroll
    for (int s = 0; s < T4H / 32; ++s)
#pragma unroll
      for (int cc = 0; cc < T4CPL; ++cc) acch[cc] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ufr[cc][s], bh[s], acch[cc], 0, 0, 0);
#pragma unroll
    for (int cc = 0; cc < T4CPL; ++cc) {
      const f32x4_t a = accx[cc] + acch[cc];
      const float iv = sigmoidf_fast(a[0]), fv = sigmoidf_fast(a[1]), gv = tanhf_fast(a[2]),
                  ov = sigmoidf_fast(a[3]);
      const float cold = c[cc];
      c[cc] = fv * cold + iv * gv;
      const float hv = ov * tanhf_fast(c[cc]);
      const int u = unit[cc];
      hs[p ^ 1][col][u] = (__bf16)hv;
      if (!A.hlast)
        A.h[((size_t)t * Mp + row0 + col) * T4H + u] = hv;
      else if (t == T - 1)
        A.h[(size_t)(row0 + col) * T4H + u] = hv;
      if (t == T - 1) hl[col * T4HP + u] = hv;
      if constexpr (TRAIN) {
        const size_t o = t4_sidx(t, ntiles, tile, w, cc, lane);
        if constexpr (CG) {
          A.gb[o] = gates_pack(iv, fv, gv, ov);
          A.c[o] = c[cc];
        } else {
          *reinterpret_cast<float4*>(A.g + o * 4) = make_float4(iv, fv, gv, ov);
          *reinterpret_cast<float2*>(A.c + o * 2) = make_float2(c[cc], cold);
        }
      }
    }
    lds_barrier();
    t4_mark(A.trace, 2 + min(t, 9));
  }
  __syncthreads();
  if constexpr (CG) {
    if (A.head) t4_prob_head<T4H>(A.hd, tile, hl, scratch, tile != (int)blockIdx.x, A.prob, A.dhg);
  } else {
    if (A.head) chain_head_fwd<T4H>(A.hd, tile, ntiles, hl, scratch);
  }
  __syncthreads();
  if constexpr (!CG) break;              // (grid = tiles)
  }
  t4_mark(A.trace, 15);
}

// ----------------------------------------------------------------------------------- backward
template <int KX>
struct T4BwdLds {
  static constexpr int DH = 16 * T4HP * 4;                       // dh_{T-1} from the head
  static constexpr int ZS = 16 * (T4G + 8) * 2;                  // bf16 dz tile
  static constexpr int DN = 16 * T4HP * 4;                       // fp32 dh_rec tile
  static constexpr int DX = 2 * 16 * (32 * KX + 4) * 4;          // fp32 dx partials
  static constexpr int STEP = ZS + DN + DX;
  static constexpr int BYTES = DH + (STEP > ChainHeadBwdLds<T4H>::BYTES ? STEP : ChainHeadBwdLds<T4H>::BYTES);
};

template <int KX, bool CG = false>
__global__ __launch_bounds__(T4NT) void t4_head_bwd_kernel(T4Args A) {
  using L = T4BwdLds<KX>;
  constexpr int DXP = 32 * KX + 4;
  __shared__ __attribute__((aligned(16))) char smem[L::BYTES];
  float* dhT = reinterpret_cast<float*>(smem);
  char* rs = smem + L::DH;
  auto zs = reinterpret_cast<__bf16 (*)[T4G + 8]>(rs);
  auto dhn = reinterpret_cast<float (*)[T4HP]>(rs + L::ZS);
  auto dxp = reinterpret_cast<float (*)[16][DXP]>(rs + L::ZS + L::DN);

  int tile = blockIdx.x;
  const int T = A.T, Mp = A.Mp, Din = A.Din, Dw = A.Dw, ntiles = A.ntiles;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int col = lane & 15, quad = lane >> 4;
  const int dt = w & 3, kh = w >> 2;

  int unit[T4CPL];
#pragma unroll
  for (int cc = 0; cc < T4CPL; ++cc) unit[cc] = 4 * (w + T4NW * cc) + quad;
  // forward state ring (2 reverse steps: gates, c_t, c_{t-1}); a slot is refilled right after the
  // cell phase that consumed it, before that step's stores (vmcnt retires in order, so a wait for
  // a slot then covers only stores issued two steps earlier)
  // (CG: packed bf16 gates, unpacked when consumed, and c_t / c_{t-1} from two step slots)
  using GR = std::conditional_t<CG, uint2, float4>;
  GR rg[2][T4CPL];
  float2 rcs[2][T4CPL];
  auto load_slot = [&](int j, int t) {
    const int tc = max(t, 0);
#pragma unroll
    for (int cc = 0; cc < T4CPL; ++cc) {
      const size_t o = t4_sidx(tc, ntiles, tile, w, cc, lane);
      if constexpr (CG) {
        rg[j][cc] = A.gb[o];
        rcs[j][cc] = make_float2(A.c[o], A.c[t4_sidx(max(t - 1, 0), ntiles, tile, w, cc, lane)]);
      } else {
        rg[j][cc] = *reinterpret_cast<const float4*>(A.g + o * 4);
        rcs[j][cc] = *reinterpret_cast<const float2*>(A.c + o * 2);
      }
    }
  };
  auto load_dhT = [&]() {   // CG: the last state's gradient [Mp][H] (x the row scales) -> LDS
    const float4* src = reinterpret_cast<const float4*>(A.dhT + (size_t)tile * 16 * T4H);
    for (int e = tid; e < 16 * T4H / 4; e += T4NT) {
      const int r = e / (T4H / 4), k = 4 * (e % (T4H / 4));
      float4 v = src[e];
      if (A.dhs != nullptr) {
        const int row = tile * 16 + r;
        const float sc = row < A.dhs_n ? A.dhs[min(row, A.dhs_n - 1)] : 0.f;
        v = make_float4(v.x * sc, v.y * sc, v.z * sc, v.w * sc);
      }
      *reinterpret_cast<float4*>(dhT + r * T4HP + k) = v;
    }
  };
  load_slot(0, T - 1);
  load_slot(1, T - 2);

  t4_mark(A.trace, 0);
  if constexpr (CG)
    load_dhT();
  else
    chain_head_bwd<T4H>(A.hd, A.h + (size_t)(T - 1) * Mp * T4H, tile, ntiles, dhT, rs);
  // recurrent / input weights as A fragments, after the head prologue (live through it they
  // pushed the kernel past 256 VGPRs into scratch): from the chain forward's backward image
  // (lane-contiguous 16-B loads), else gathered (16 rows per load instruction: ~10 us)
  bf16x8_t ufr[T4G / 32], wfr[8];
  if (A.pk != nullptr) {
    const bf16x8_t* pu = A.pk + T4PK_N + (size_t)w * 16 * 64 + lane;
    const bf16x8_t* pw = A.pk + T4PK_N + T4PK_BU + (size_t)w * 8 * 64 + lane;
#pragma unroll
    for (int s = 0; s < T4G / 32; ++s) ufr[s] = pu[s * 64];
#pragma unroll
    for (int s = 0; s < 8; ++s) wfr[s] = pw[s * 64];
  } else {
#pragma unroll
    for (int s = 0; s < T4G / 32; ++s) {
      const float* src = A.U + (size_t)(16 * w + col) * T4G + 32 * s + 8 * quad;
      const float4 a = *reinterpret_cast<const float4*>(src), b = *reinterpret_cast<const float4*>(src + 4);
      ufr[s] = bf16x8_t{(__bf16)a.x, (__bf16)a.y, (__bf16)a.z, (__bf16)a.w,
                        (__bf16)b.x, (__bf16)b.y, (__bf16)b.z, (__bf16)b.w};
    }
    const int din = 16 * dt + col;
    const float m = (dt < 2 * KX && din < Dw) ? 1.f : 0.f;
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      const float* src = A.W + (size_t)min(din, Dw - 1) * T4G + 256 * kh + 32 * s + 8 * quad;
      const float4 a = *reinterpret_cast<const float4*>(src), b = *reinterpret_cast<const float4*>(src + 4);
      wfr[s] = bf16x8_t{(__bf16)(a.x * m), (__bf16)(a.y * m), (__bf16)(a.z * m), (__bf16)(a.w * m),
                        (__bf16)(b.x * m), (__bf16)(b.y * m), (__bf16)(b.z * m), (__bf16)(b.w * m)};
    }
  }
  __syncthreads();                      // the head scratch becomes the step tiles
  t4_mark(A.trace, 1);

  const size_t zstep = (size_t)Mp * T4G;
  const int nx = 16 * Din;
  for (;;) {                            // tiles (one pass unless CG)
  const int row0 = tile * 16;
  float dc[T4CPL], dhr[T4CPL];
#pragma unroll
  for (int cc = 0; cc < T4CPL; ++cc) dc[cc] = dhr[cc] = 0.f;
  for (int s0 = 0; s0 < T; s0 += 2) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int s = s0 + j;
      if (s >= T) break;                 // (uniform)
      const int t = T - 1 - s;
#pragma unroll
      for (int cc = 0; cc < T4CPL; ++cc) {
        const int u = unit[cc];
        const float dh = dhr[cc] + (s == 0 ? dhT[col * T4HP + u] : 0.f);
        float4 g;
        if constexpr (CG)
          g = gates_unpack(rg[j][cc]);
        else
          g = rg[j][cc];
        // (0 at t = 0: the forward's initial state; CG reads a clamped slot there)
        const float cprev = (CG && t == 0) ? 0.f : rcs[j][cc].y;
        const float tc = tanhf_fast(rcs[j][cc].x);
        const float dct = dc[cc] + dh * g.w * (1.f - tc * tc);
        dc[cc] = dct * g.y;
        zs[col][0 * T4H + u] = (__bf16)(dct * g.z * g.x * (1.f - g.x));
        zs[col][1 * T4H + u] = (__bf16)(dct * cprev * g.y * (1.f - g.y));
        zs[col][2 * T4H + u] = (__bf16)(dct * g.x * (1.f - g.z * g.z));
        zs[col][3 * T4H + u] = (__bf16)(dh * tc * g.w * (1.f - g.w));
      }
      load_slot(j, t - 2);
      lds_barrier();
      if (!CG || A.dz != nullptr) {   // (uniform; CG: none without weight gradients)
#pragma unroll
        for (int q = 0; q < 16 * T4G / 4 / T4NT; ++q) {   // dz_t -> HBM, the bf16 values the MFMAs use
          const int e = tid + T4NT * q, sq = e / (T4G / 4), c4 = (e % (T4G / 4)) * 4;
          const bf16x4_t zv = *reinterpret_cast<const bf16x4_t*>(&zs[sq][c4]);
          *reinterpret_cast<bf16x4_t*>(A.dz + (size_t)t * zstep + (size_t)(row0 + sq) * T4G + c4) = zv;
        }
      }
      {   // dh_rec^T for unit tile w (full K) and dx^T for din tile dt over gate-column half kh,
          // as 4 + 2 interleaved accumulator chains
        f32x4_t a[4], b[2];
#pragma unroll
        for (int q = 0; q < 4; ++q) a[q] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int q = 0; q < 2; ++q) b[q] = f32x4_t{0.f, 0.f, 0.f, 0.f};
        const bool dxw = dt < 2 * KX;    // (uniform)
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {   // gate-column halves: one uniform branch per half for dx
          bf16x8_t bz[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) bz[j] = *reinterpret_cast<const bf16x8_t*>(&zs[col][32 * (8 * hh + j) + 8 * quad]);
#pragma unroll
          for (int j = 0; j < 8; ++j)
            a[j & 3] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ufr[8 * hh + j], bz[j], a[j & 3], 0, 0, 0);
          if (dxw && hh == kh) {
#pragma unroll
            for (int j = 0; j < 8; ++j) b[j & 1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wfr[j], bz[j], b[j & 1], 0, 0, 0);
          }
        }
        const f32x4_t as = (a[0] + a[1]) + (a[2] + a[3]);
#pragma unroll
        for (int r = 0; r < 4; ++r) dhn[col][16 * w + 4 * quad + r] = as[r];
        if (dxw) {
          const f32x4_t bs = b[0] + b[1];
#pragma unroll
          for (int r = 0; r < 4; ++r) dxp[kh][col][16 * dt + 4 * quad + r] = bs[r];
        }
      }
      lds_barrier();
#pragma unroll
      for (int cc = 0; cc < T4CPL; ++cc) dhr[cc] = dhn[col][unit[cc]];
      for (int e = tid; e < nx; e += T4NT) {
        const int r = e / Din, k = e % Din;
        A.dx[((size_t)t * Mp + row0 + r) * Din + k] = dxp[0][r][k] + dxp[1][r][k];
      }
      t4_mark(A.trace, 2 + min(s, 9));
    }
  }
  if constexpr (!CG) break;
  tile += gridDim.x;
  if (tile >= ntiles) break;
  load_slot(0, T - 1);                   // the next tile: state ring and last-state gradient
  load_slot(1, T - 2);
  load_dhT();
  __syncthreads();
  }
  if constexpr (!CG) chain_head_bwd_reduce<T4H>(A.hd, tile, ntiles);
  __syncthreads();
  t4_mark(A.trace, 15);
}

// --------------------------------------------------------------------------------------- host
static long long* t4_trace_buf(int dev) {
  static long long* tr[64] = {nullptr};
  TORCH_CHECK(dev >= 0 && dev < 64, "time4_head: device index");
  if (!tr[dev]) TORCH_CHECK(hipMalloc(&tr[dev], 256 * 16 * sizeof(long long)) == hipSuccess, "time4_head: trace");
  return tr[dev];
}

// [blocks * 16] s_memrealtime marks (100 MHz) of the last time4 launch: 0 start, 1 prologue done,
// 2.. after each step, 15 end (profiling)
at::Tensor time4_trace(const at::Tensor& like) {
  c10::DeviceGuard guard(like.device());
  at::Tensor o = at::empty({256 * 16}, like.options().dtype(at::kLong));
  TORCH_CHECK(hipMemcpyAsync(o.data_ptr<int64_t>(), t4_trace_buf(like.get_device()), 256 * 16 * sizeof(long long),
                             hipMemcpyDeviceToDevice, stream()) == hipSuccess, "time4_trace");
  return o;
}

static void t4_head_args(ChainHead& hd, at::TensorList head, const at::Tensor& y, const at::Tensor& mask, int64_t M,
                         int Mp, double alpha1, double alpha2, double w0, double w1) {
  TORCH_CHECK(head.size() == 6, "time4_head: expected W1, b1, W2, b2, W3, b3");
  for (const at::Tensor& t : head) check_f32_cuda(t, "time4_head head weight");
  TORCH_CHECK(head[0].numel() == (long)T4H * CH_HU && head[1].numel() == CH_HU && head[2].numel() == CH_HU * CH_HU &&
                  head[3].numel() == CH_HU && head[4].numel() == CH_HU && head[5].numel() == 1,
              "time4_head: expected Dense(128,64)-Dense(64,64)-Dense(64,1)");
  check_f32_cuda(y, "y");
  check_f32_cuda(mask, "mask");
  TORCH_CHECK(M >= 1 && M <= Mp && y.numel() >= M && mask.numel() >= M, "time4_head: y / mask rows");
  hd.W1 = head[0].data_ptr<float>();
  hd.b1 = head[1].data_ptr<float>();
  hd.W2 = head[2].data_ptr<float>();
  hd.b2 = head[3].data_ptr<float>();
  hd.W3 = head[4].data_ptr<float>();
  hd.b3 = head[5].data_ptr<float>();
  hd.y = y.data_ptr<float>();
  hd.mask = mask.data_ptr<float>();
  hd.M = (int)M;
  hd.alpha1 = (float)alpha1;
  hd.alpha2 = (float)alpha2;
  hd.w0 = (float)w0;
  hd.w1 = (float)w1;
}

static void t4_check(const at::Tensor& x, const at::Tensor& W, const at::Tensor& U, int& T, int& Mp, int& Din,
                     int& Dw) {
  check_f32_cuda(x, "x");
  check_f32_cuda(W, "W");
  check_f32_cuda(U, "U");
  TORCH_CHECK(x.dim() == 3, "time4_head: x must be [T, Mp, Din]");
  T = (int)x.size(0);
  Mp = (int)x.size(1);
  Din = (int)x.size(2);
  Dw = (int)W.size(0);
  TORCH_CHECK(T >= 1 && T <= T4MAXT, "time4_head: sequence length 1..", T4MAXT, " (got ", T, ")");
  TORCH_CHECK(Mp % 16 == 0 && Mp >= 16, "time4_head: Mp must be a positive multiple of 16");
  TORCH_CHECK(Din % 4 == 0 && Din >= 4 && Din <= 64 && Dw >= 1 && Dw <= Din,
              "time4_head: input width must be a multiple of 4 up to 64 (W rows <= width)");
  TORCH_CHECK(U.size(0) == T4H && U.size(1) == T4G && W.size(1) == T4G, "time4_head: H must be 128");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0, "time4_head: x must be 16-byte aligned");
}

// The forward head's arguments: weights, labels, outputs (logits [M], loss [1], per-tile partials
// allocated here), the metric accumulators (sums [6] fp64 / hist [2, bins], empty: none) and the
// arrival ticket (chain control word 4). Also used by lstm_chain_head_fwd (lstm_chain.hip).
void t4_head_fwd_args(ChainHead& hd, at::TensorList head, const at::Tensor& y, const at::Tensor& mask, int64_t M,
                      int Mp, double alpha1, double alpha2, double w0, double w1, const at::Tensor& sums,
                      const at::Tensor& hist, at::Tensor& logits, at::Tensor& loss, at::Tensor& part) {
  t4_head_args(hd, head, y, mask, M, Mp, alpha1, alpha2, w0, w1);
  auto opt = y.options();
  logits = at::empty({M}, opt);
  loss = at::empty({1}, opt);
  part = at::empty({Mp / 16 * 8}, opt);
  hd.logits = logits.data_ptr<float>();
  hd.loss = loss.data_ptr<float>();
  hd.part = part.data_ptr<float>();
  hd.ticket = chain_ctl(y.get_device()) + 4;
  if (sums.numel() > 0) {
    TORCH_CHECK(sums.is_cuda() && sums.scalar_type() == at::kDouble && sums.numel() == 6, "sums: 6 float64");
    hd.sums = sums.data_ptr<double>();
  }
  if (hist.numel() > 0) {
    check_f32_cuda(hist, "hist");
    TORCH_CHECK(hist.dim() == 2 && hist.size(0) == 2, "hist must be [2, bins]");
    hd.hist = hist.data_ptr<float>();
    hd.bins = (int)hist.size(1);
  }
}

// time4 + head + weighted BCE forward. x: [T, Mp, Din] (the pooled output of the chain); pk: the
// A-fragment image of (W, U) built by lstm_chain_fwd_pack (empty: built here through LDS);
// head = [W1, b1, W2, b2, W3, b3], y / mask [M]. Returns [h [T, Mp, 128], g, c, logits [M], loss [1]];
// with sums / hist non-empty the metric accumulators are updated.
std::vector<at::Tensor> time4_head_fwd(const at::Tensor& x, const at::Tensor& W, const at::Tensor& U,
                                       const at::Tensor& b, const at::Tensor& pk, bool train, at::TensorList head, const at::Tensor& y,
                                       const at::Tensor& mask, int64_t M, double alpha1, double alpha2, double w0,
                                       double w1, at::Tensor sums, at::Tensor hist) {
  int T, Mp, Din, Dw;
  t4_check(x, W, U, T, Mp, Din, Dw);
  check_f32_cuda(b, "b");
  c10::DeviceGuard guard(x.device());
  auto opt = x.options();
  const int ntiles = Mp / 16;
  T4Args A{};
  A.x = x.data_ptr<float>();
  A.W = W.data_ptr<float>();
  A.U = U.data_ptr<float>();
  A.b = b.data_ptr<float>();
  if (pk.numel() > 0) {
    TORCH_CHECK(pk.is_cuda() && pk.is_contiguous() && pk.nbytes() >= (size_t)T4PK_N * 16,
                "time4_head: fragment image size");
    A.pk = reinterpret_cast<const bf16x8_t*>(pk.data_ptr());
  }
  at::Tensor h = at::empty({T, Mp, T4H}, opt);
  at::Tensor g = train ? at::empty({(long)T * Mp * T4H * 4}, opt) : at::empty({0}, opt);
  at::Tensor c = train ? at::empty({(long)T * Mp * T4H * 2}, opt) : at::empty({0}, opt);
  at::Tensor logits, loss, part;
  A.h = h.data_ptr<float>();
  A.g = train ? g.data_ptr<float>() : nullptr;
  A.c = train ? c.data_ptr<float>() : nullptr;
  A.T = T;
  A.Mp = Mp;
  A.Din = Din;
  A.Dw = Dw;
  A.ntiles = ntiles;
  t4_head_fwd_args(A.hd, head, y, mask, M, Mp, alpha1, alpha2, w0, w1, sums, hist, logits, loss, part);
  A.head = 1;
  A.trace = t4_trace_buf(x.get_device());
  TORCH_CHECK(ntiles <= 256, "time4_head: at most 256 tiles");
  const int KX = (Din + 31) / 32;
#define GQ_T4F(TR, K) hipLaunchKernelGGL((t4_head_fwd_kernel<TR, K>), dim3(ntiles), dim3(T4NT), 0, stream(), A)
  if (train) { if (KX == 1) GQ_T4F(true, 1); else GQ_T4F(true, 2); }
  else { if (KX == 1) GQ_T4F(false, 1); else GQ_T4F(false, 2); }
#undef GQ_T4F
  GQ_LAUNCH_CHECK();
  return {h, g, c, logits, loss};
}

// The backward head's arguments: dloss [1], the head gradient sinks (accumulated), the per-tile
// record buffer (allocated here) and the chain control words' tickets ([5] arrivals, [8] reduce
// done; [7] is the non-finite gradient flag). Also used by lstm_chain_head_bwd (lstm_chain.hip).
void t4_head_bwd_args(ChainHead& hd, at::TensorList head, const at::Tensor& y, const at::Tensor& mask, int64_t M,
                      int Mp, double alpha1, double alpha2, double w0, double w1, const at::Tensor& dloss,
                      at::TensorList hgrads, at::Tensor& gpart) {
  check_f32_cuda(dloss, "dloss");
  TORCH_CHECK(dloss.numel() == 1, "time4_head_bwd: dloss must be a scalar");
  TORCH_CHECK(hgrads.size() == 6, "time4_head_bwd: head gradient list");
  t4_head_args(hd, head, y, mask, M, Mp, alpha1, alpha2, w0, w1);
  for (size_t i = 0; i < 6; ++i) {
    check_f32_cuda(hgrads[i], "head gradient");
    TORCH_CHECK(hgrads[i].numel() == head[i].numel(), "time4_head_bwd: head gradient ", i, " size");
  }
  gpart = at::empty({(long)(Mp / 16) * ChainHeadRec<T4H>::PITCH}, y.options());
  hd.dloss = dloss.data_ptr<float>();
  hd.gpart = gpart.data_ptr<float>();
  hd.dW1 = hgrads[0].data_ptr<float>();
  hd.db1 = hgrads[1].data_ptr<float>();
  hd.dW2 = hgrads[2].data_ptr<float>();
  hd.db2 = hgrads[3].data_ptr<float>();
  hd.dW3 = hgrads[4].data_ptr<float>();
  hd.db3 = hgrads[5].data_ptr<float>();
  const int dev = y.get_device();
  hd.ticket = chain_ctl(dev) + 5;
  hd.done = chain_ctl(dev) + 8;
  hd.ctl = chain_ctl(dev);
}

// Backward: dloss [1]; x / h / g / c from the forward. Adds the head's weight gradients to
// hgrads = [dW1, db1, dW2, db2, dW3, db3]; returns [dz [T + 1, Mp, 512], dx [T, Mp, Din]].
std::vector<at::Tensor> time4_head_bwd(const at::Tensor& dloss, const at::Tensor& x, const at::Tensor& h,
                                       const at::Tensor& g, const at::Tensor& c, const at::Tensor& W,
                                       const at::Tensor& U, const at::Tensor& pk, at::TensorList head, const at::Tensor& y,
                                       const at::Tensor& mask, int64_t M, double alpha1, double alpha2, double w0,
                                       double w1, at::TensorList hgrads) {
  int T, Mp, Din, Dw;
  t4_check(x, W, U, T, Mp, Din, Dw);
  for (const at::Tensor* t : {&dloss, &h, &g, &c}) check_f32_cuda(*t, "time4_head_bwd operand");
  TORCH_CHECK(dloss.numel() == 1, "time4_head_bwd: dloss must be a scalar");
  TORCH_CHECK(h.numel() == (long)T * Mp * T4H && g.numel() == (long)T * Mp * T4H * 4 && c.numel() == (long)T * Mp * T4H * 2,
              "time4_head_bwd: saved state shapes");
  c10::DeviceGuard guard(x.device());
  auto opt = x.options();
  const int ntiles = Mp / 16;
  T4Args A{};
  A.x = x.data_ptr<float>();
  A.W = W.data_ptr<float>();
  A.U = U.data_ptr<float>();
  A.h = const_cast<float*>(h.data_ptr<float>());
  A.g = const_cast<float*>(g.data_ptr<float>());
  A.c = const_cast<float*>(c.data_ptr<float>());
  at::Tensor dz = at::empty({T + 1, Mp, T4G}, opt.dtype(at::kBFloat16)), dx = at::empty({T, Mp, Din}, opt);
  A.dz = bf16_ptr(dz);
  A.dx = dx.data_ptr<float>();
  A.T = T;
  A.Mp = Mp;
  A.Din = Din;
  A.Dw = Dw;
  A.ntiles = ntiles;
  at::Tensor gpart;
  t4_head_bwd_args(A.hd, head, y, mask, M, Mp, alpha1, alpha2, w0, w1, dloss, hgrads, gpart);
  A.head = 1;
  A.trace = t4_trace_buf(x.get_device());
  if (pk.numel() > 0) {         // the chain forward's image including the backward fragments
    TORCH_CHECK(pk.is_cuda() && pk.is_contiguous() && pk.nbytes() == (size_t)T4PK_ALL * 16,
                "time4_head_bwd: pk must be the forward's full fragment image");
    A.pk = reinterpret_cast<const bf16x8_t*>(pk.data_ptr());
  }
  TORCH_CHECK(ntiles <= 256, "time4_head: at most 256 tiles");
  if ((Din + 31) / 32 == 1)
    hipLaunchKernelGGL((t4_head_bwd_kernel<1>), dim3(ntiles), dim3(T4NT), 0, stream(), A);
  else
    hipLaunchKernelGGL((t4_head_bwd_kernel<2>), dim3(ntiles), dim3(T4NT), 0, stream(), A);
  GQ_LAUNCH_CHECK();
  return {dz, dx};
}

// ------------------------------------------------------------- the layer alone (no head)
// time4 as a standalone time-major layer returning its last state, for passes with many
// sequences (integrated gradients: 32k path sequences per launch, where the seq-major
// lstm_fwd<128> / lstm_bwd / lstm_dx path plus its layout copies took ~0.7 ms). CG kernels:
// compact saved state, workgroups looping over tiles.
static int t4_grid(int ntiles, int64_t max_blocks) {
  int dev = 0;
  TORCH_CHECK(hipGetDevice(&dev) == hipSuccess, "time4: device");
  int cus = 0;
  TORCH_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess, "time4: CUs");
  int g = std::min(ntiles, std::max(cus, 1));       // one 512-thread workgroup per CU (LDS / VGPRs)
  if (max_blocks > 0) g = std::min<int64_t>(g, max_blocks);
  return std::max(g, 1);
}

// x [T, Mp, Din] time-major. Returns [h, g, c]: h = [T, Mp, 128] (all_h) or the last state
// [Mp, 128]; with train the compact saved state g (packed bf16 gates) and c for time4_bwd.
std::vector<at::Tensor> time4_fwd(const at::Tensor& x, const at::Tensor& W, const at::Tensor& U, const at::Tensor& b,
                                  bool train, bool all_h, int64_t max_blocks) {
  int T, Mp, Din, Dw;
  t4_check(x, W, U, T, Mp, Din, Dw);
  check_f32_cuda(b, "b");
  TORCH_CHECK(b.numel() == T4G, "time4_fwd: bias size");
  c10::DeviceGuard guard(x.device());
  auto opt = x.options();
  const int ntiles = Mp / 16;
  const long cells = (long)T * Mp * T4H;
  at::Tensor h = all_h ? at::empty({T, Mp, T4H}, opt) : at::empty({Mp, T4H}, opt);
  at::Tensor g = train ? at::empty({cells * 4}, opt.dtype(at::kBFloat16)) : at::empty({0}, opt);
  at::Tensor c = train ? at::empty({cells}, opt) : at::empty({0}, opt);
  T4Args A{};
  A.x = x.data_ptr<float>();
  A.W = W.data_ptr<float>();
  A.U = U.data_ptr<float>();
  A.b = b.data_ptr<float>();
  A.h = h.data_ptr<float>();
  A.gb = train ? reinterpret_cast<uint2*>(g.data_ptr()) : nullptr;
  A.c = train ? c.data_ptr<float>() : nullptr;
  A.T = T;
  A.Mp = Mp;
  A.Din = Din;
  A.Dw = Dw;
  A.ntiles = ntiles;
  A.hlast = all_h ? 0 : 1;
  const dim3 grid(t4_grid(ntiles, max_blocks));
  const int KX = (Din + 31) / 32;
#define GQ_T4F(TR, K) hipLaunchKernelGGL((t4_head_fwd_kernel<TR, K, true>), grid, dim3(T4NT), 0, stream(), A)
  if (train) { if (KX == 1) GQ_T4F(true, 1); else GQ_T4F(true, 2); }
  else { if (KX == 1) GQ_T4F(false, 1); else GQ_T4F(false, 2); }
#undef GQ_T4F
  GQ_LAUNCH_CHECK();
  return {h, g, c};
}

// time4 + the frozen Dense head for integrated gradients: x [T, Mp, Din]; head = [W1, b1, W2, b2, W3,
// b3] (Dense(128,64)-LeakyReLU(alpha1)-Dense(64,64)-LeakyReLU(alpha2)-Dense(64,1)-sigmoid). Returns
// [prob [Mp], dh [Mp, 128] = d prob / d h_{T-1} (rows >= M zero), g, c]: time4_bwd(dh, ...,
// row_scale = d loss / d prob) then gives the input gradient without a head backward launch.
std::vector<at::Tensor> time4_prob_fwd(const at::Tensor& x, const at::Tensor& W, const at::Tensor& U, const at::Tensor& b,
                                       at::TensorList head, double alpha1, double alpha2, int64_t M, bool train,
                                       int64_t max_blocks) {
  int T, Mp, Din, Dw;
  t4_check(x, W, U, T, Mp, Din, Dw);
  check_f32_cuda(b, "b");
  TORCH_CHECK(b.numel() == T4G, "time4_prob_fwd: bias size");
  TORCH_CHECK(head.size() == 6, "time4_prob_fwd: expected W1, b1, W2, b2, W3, b3");
  for (const at::Tensor& t : head) check_f32_cuda(t, "time4_prob_fwd head weight");
  TORCH_CHECK(head[0].numel() == (long)T4H * CH_HU && head[1].numel() == CH_HU && head[2].numel() == CH_HU * CH_HU &&
                  head[3].numel() == CH_HU && head[4].numel() == CH_HU && head[5].numel() == 1,
              "time4_prob_fwd: expected Dense(128,64)-Dense(64,64)-Dense(64,1)");
  TORCH_CHECK(M >= 1 && M <= Mp, "time4_prob_fwd: rows");
  c10::DeviceGuard guard(x.device());
  auto opt = x.options();
  const int ntiles = Mp / 16;
  const long cells = (long)T * Mp * T4H;
  at::Tensor h = at::empty({Mp, T4H}, opt), prob = at::empty({Mp}, opt), dh = at::empty({Mp, T4H}, opt);
  at::Tensor g = train ? at::empty({cells * 4}, opt.dtype(at::kBFloat16)) : at::empty({0}, opt);
  at::Tensor c = train ? at::empty({cells}, opt) : at::empty({0}, opt);
  T4Args A{};
  A.x = x.data_ptr<float>();
  A.W = W.data_ptr<float>();
  A.U = U.data_ptr<float>();
  A.b = b.data_ptr<float>();
  A.h = h.data_ptr<float>();
  A.gb = train ? reinterpret_cast<uint2*>(g.data_ptr()) : nullptr;
  A.c = train ? c.data_ptr<float>() : nullptr;
  A.T = T;
  A.Mp = Mp;
  A.Din = Din;
  A.Dw = Dw;
  A.ntiles = ntiles;
  A.hlast = 1;
  A.head = 1;
  A.prob = prob.data_ptr<float>();
  A.dhg = dh.data_ptr<float>();
  A.hd.W1 = head[0].data_ptr<float>();
  A.hd.b1 = head[1].data_ptr<float>();
  A.hd.W2 = head[2].data_ptr<float>();
  A.hd.b2 = head[3].data_ptr<float>();
  A.hd.W3 = head[4].data_ptr<float>();
  A.hd.b3 = head[5].data_ptr<float>();
  A.hd.M = (int)M;
  A.hd.alpha1 = (float)alpha1;
  A.hd.alpha2 = (float)alpha2;
  const dim3 grid(t4_grid(ntiles, max_blocks));
  const int KX = (Din + 31) / 32;
#define GQ_T4F(TR, K) hipLaunchKernelGGL((t4_head_fwd_kernel<TR, K, true>), grid, dim3(T4NT), 0, stream(), A)
  if (train) { if (KX == 1) GQ_T4F(true, 1); else GQ_T4F(true, 2); }
  else { if (KX == 1) GQ_T4F(false, 1); else GQ_T4F(false, 2); }
#undef GQ_T4F
  GQ_LAUNCH_CHECK();
  return {prob, dh, g, c};
}

// dh [Mp, 128]: gradient of the last state; x / g / c from time4_fwd(train). Returns [dz, dx]:
// dz [T + 1, Mp, 512] bf16 for lstm_tm_grads when need_dz (else empty), dx [T, Mp, Din].
std::vector<at::Tensor> time4_bwd(const at::Tensor& dh, const at::Tensor& x, const at::Tensor& g, const at::Tensor& c,
                                  const at::Tensor& W, const at::Tensor& U, bool need_dz, int64_t max_blocks,
                                  const c10::optional<at::Tensor>& row_scale) {
  int T, Mp, Din, Dw;
  t4_check(x, W, U, T, Mp, Din, Dw);
  check_f32_cuda(dh, "dh");
  check_f32_cuda(c, "c");
  const long cells = (long)T * Mp * T4H;
  TORCH_CHECK(dh.numel() == (long)Mp * T4H, "time4_bwd: dh must be [Mp, 128]");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(dh.data_ptr()) % 16 == 0, "time4_bwd: dh must be 16-byte aligned");
  TORCH_CHECK(g.is_cuda() && g.is_contiguous() && g.scalar_type() == at::kBFloat16 && g.numel() == cells * 4 &&
                  c.numel() == cells, "time4_bwd: saved state from time4_fwd(train=True)");
  c10::DeviceGuard guard(x.device());
  auto opt = x.options();
  const int ntiles = Mp / 16;
  at::Tensor dz = need_dz ? at::empty({T + 1, Mp, T4G}, opt.dtype(at::kBFloat16)) : at::empty({0}, opt);
  at::Tensor dx = at::empty({T, Mp, Din}, opt);
  T4Args A{};
  A.x = x.data_ptr<float>();
  A.W = W.data_ptr<float>();
  A.U = U.data_ptr<float>();
  A.gb = reinterpret_cast<uint2*>(const_cast<void*>(g.data_ptr()));
  A.c = const_cast<float*>(c.data_ptr<float>());
  A.dhT = dh.data_ptr<float>();
  if (row_scale.has_value() && row_scale->defined()) {
    check_f32_cuda(*row_scale, "row_scale");
    TORCH_CHECK(row_scale->numel() >= 1 && row_scale->numel() <= Mp && row_scale->is_contiguous(),
                "time4_bwd: row_scale must have 1..Mp entries (rows past them get 0)");
    A.dhs = row_scale->data_ptr<float>();
    A.dhs_n = (int)row_scale->numel();
  }
  A.dz = need_dz ? bf16_ptr(dz) : nullptr;
  A.dx = dx.data_ptr<float>();
  A.T = T;
  A.Mp = Mp;
  A.Din = Din;
  A.Dw = Dw;
  A.ntiles = ntiles;
  const dim3 grid(t4_grid(ntiles, max_blocks));
  if ((Din + 31) / 32 == 1)
    hipLaunchKernelGGL((t4_head_bwd_kernel<1, true>), grid, dim3(T4NT), 0, stream(), A);
  else
    hipLaunchKernelGGL((t4_head_bwd_kernel<2, true>), grid, dim3(T4NT), 0, stream(), A);
  GQ_LAUNCH_CHECK();
  return {dz, dx};
}

}  // namespace gq

TORCH_LIBRARY_IMPL(gnnqc, CUDA, m) {
  m.impl("time4_head_fwd", &gq::time4_head_fwd);
  m.impl("time4_head_bwd", &gq::time4_head_bwd);
  m.impl("time4_trace", &gq::time4_trace);
  m.impl("time4_fwd", &gq::time4_fwd);
  m.impl("time4_bwd", &gq::time4_bwd);
  m.impl("time4_prob_fwd", &gq::time4_prob_fwd);
}
