// Time-major persistent LSTM (forward + fused backward) for gfx950.
//
// Layout: every activation inside the TimeLayer is time-major, [T][Mp][C] with Mp a
// multiple of 16, so the per-step tile of a 16-sequence block is ONE contiguous run of
// 16*C floats. All global traffic in the recurrences is tile-granular and coalesced:
//   * loader lanes stream x_t / dh_t / h_{t-1} tiles (float4/float2 granules) through a
//     register ring and stage them into LDS one step ahead;
//   * storer lanes write whole h_t / dx_t tiles from an fp32 LDS copy;
//   * the training-only state (gates, c) is written and re-read in a lane-natural layout
//     ([T][tile][wave][cell][lane]) - one 1 KiB / 256 B contiguous run per wave and step.
// (Measured on the CML shapes, per-cell scattered accesses - 16 rows per instruction -
// were what bound lstm_v3; see profiles/r1_lstm_microbench.md.)
//
// Compute mapping (as lstm_v3): the rows of the MFMA A operand are permuted so one
// 16x16 output tile holds (unit, gate) pairs and every lane receives the i,f,g,o
// pre-activations of its own cell(s): 5 activations per cell and lane, one LDS
// barrier per step. H <= 64: one cell per lane, H/4 waves; H = 128: two cells per lane,
// 16 waves.
//
// The backward fuses what lstm_bwd + lstm_grads did: per reverse step
//   cell phase   dz of the lane's cells (dh = dh_out + U dz_{t+1}), dz -> LDS (bf16, both
//                row- and column-major)
//   MFMA phase   dh_rec = U dz^T (the serial chain), dx^T = W dz^T (tile -> HBM next step),
//                and the weight gradients dW^T += dz^T [x_t | 1], dU^T += dz^T h_{t-1}
//                with v_mfma_f32_16x16x16_bf16 (K = the 16 sequences of the tile), kept in
//                VGPRs for the whole sequence and flushed once with atomics.
// So dz never goes to HBM and no separate weight-gradient kernel runs.
#include "common.h"

#include <cstdlib>
#include "lstm_grads_body.h"
#include "gcn_fused.h"
#include "lstm_tm_common.h"

#ifndef TM_RG_BF16H
#define TM_RG_BF16H 1    // recompute-gates pairs save layer A's h in bf16 (its only readers stage it as bf16; A/B: 0)
#endif
#ifndef TM_RG_BF16C
#define TM_RG_BF16C 1    // recompute-gates layers save c_t in bf16 (the forward keeps fp32 in registers; A/B: 0)
#endif

namespace gq {

// lstm_grads.hip: weight gradients (+ dx) over flat rows, h_{t-1} hshift rows back
void lstm_grads_rows(const void* dz, int zbf, const float* x, const float* hseq, const float* W, float* dx, float* dW,
                     float* dU, float* db, long rows, long period, long hshift, int H, int Din, int ldx,
                     long dx_cb_stride, int lddx, long x_elems, hipStream_t st);
int lstm_grads_col_blocks(int H);
void lstm_grads_reduce_records(const at::Tensor& ws_t, int H, int Din, int splits, float* dW, float* dU, float* db,
                               hipStream_t st);
int* chain_ctl(int dev);   // lstm_chain.hip: the device's chain control words
void lstm_dx_rows(const void* dz, int zbf, const float* W, float* dx, long rows, int H, int Dw, int lddx,
                  hipStream_t st);

// =====================================================================================
// forward
// x: [T][Mp][Din]  hout: [T][Mp][H]  gbuf: [T][tiles][NW][CPL][64][4]  cbuf: [..][64]
// 1024-thread workgroups ask for 8 waves per SIMD, i.e. two workgroups per CU (at the default
// allocation, ~70-80 VGPRs, only one fits and a 418-tile grid - SoilNet, 6,688 sequences - runs in
// two rounds on 256 CUs) where that costs no spills: the H = 64 layer with a 32-channel input
// (70.6 vs 76.7 us on the SoilNet step) and the H = 32 pair (214.5 vs 221.5 us). The 64-channel
// input variant spills at 64 VGPRs (169 vs 105 us) and keeps the default.
template <int NT, int KX = 1>
struct TmOcc {
  static constexpr int W = (NT >= 1024 && KX == 1) ? 8 : 1;
};

// SG = false (train mode, recompute-gates backward, lstm_tm_bwd_body RG): only c is saved; the
// backward recomputes the gates from x_t and h_{t-1} (same bf16 operands, same MFMA order: bitwise the
// forward's pre-activations), which halves the forward's state stream (h + c + packed gates = 16 B per
// cell-step -> 8 B) and drops the backward's 8-byte gate read
template <int H, bool TRAIN, int KX, int GR, int D, bool SG = true>
__global__ __launch_bounds__(TMC<H>::NT, (TmOcc<TMC<H>::NT, KX>::W)) void lstm_tm_fwd_kernel(
    const float* __restrict__ x, const float* __restrict__ W, const float* __restrict__ U,
    const float* __restrict__ bias, float* __restrict__ hout, __bf16* __restrict__ gbuf,
    float* __restrict__ cbuf, int Mp, int T, int Din, int Dw) {
  // Din: channels of the x layout (row pitch); Dw <= Din: rows of W (padding channels of x are zero)
  using C = TMC<H>;
  constexpr int CPL = C::CPL, NW = C::NW, NT = C::NT, G4 = C::G4;
  constexpr int KPX = 32 * KX;
  __shared__ __attribute__((aligned(16))) __bf16 hs[2][16][C::KPH + 8];
  __shared__ __attribute__((aligned(16))) __bf16 xs[2][16][KPX + 8];
  __shared__ __attribute__((aligned(16))) float hf[2][16][C::HP];

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave index in an SGPR
  const int col = lane & 15, quad = lane >> 4;
  const int tile = blockIdx.x, ntiles = gridDim.x, row0 = tile * 16;

  for (int i = tid; i < 2 * 16 * (C::KPH + 8); i += NT) (&hs[0][0][0])[i] = (__bf16)0.0f;
  for (int i = tid; i < 2 * 16 * (KPX + 8); i += NT) (&xs[0][0][0])[i] = (__bf16)0.0f;

  // A fragments: tile row `col` of cell group gi = gate (col & 3) of unit 4 gi + (col >> 2)
  bf16x8_t ufr[CPL][C::KSH], wfr[CPL][KX];
  f32x4_t bias4[CPL];
  int unit[CPL];
#pragma unroll
  for (int cc = 0; cc < CPL; ++cc) {
    const int gi = w + NW * cc;
    const int au = 4 * gi + (col >> 2), ag = col & 3;
    unit[cc] = 4 * gi + quad;
#pragma unroll
    for (int s = 0; s < C::KSH; ++s) {
      bf16x8_t v;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int k = 32 * s + 8 * quad + j;
        v[j] = (__bf16)(U[min(k, H - 1) * G4 + ag * H + au] * (k < H ? 1.0f : 0.0f));
      }
      ufr[cc][s] = v;
    }
#pragma unroll
    for (int s = 0; s < KX; ++s) {
      bf16x8_t v;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int k = 32 * s + 8 * quad + j;
        v[j] = (__bf16)(W[min(k, Dw - 1) * G4 + ag * H + au] * (k < Dw ? 1.0f : 0.0f));
      }
      wfr[cc][s] = v;
    }
    const int u = unit[cc];
    bias4[cc] = f32x4_t{bias[u], bias[H + u], bias[2 * H + u], bias[3 * H + u]};
  }

  // x loader: every wave streams granule (tid mod n) of the contiguous [16][Din] tile and
  // stages it (identical duplicates across waves). No branch surrounds a memory op: with a
  // predicate around loads hipcc drained vmcnt at the join every step (seen in the ISA).
  const int n_gx = 16 * Din / GR;
  const int gx = (tid % n_gx) * GR;
  const int gx_seq = gx / Din, gx_k = gx % Din;
  const float* xbase = x + (size_t)row0 * Din + gx;
  const size_t xstep = (size_t)Mp * Din;
  Granule<GR> xr[D];
  // h storer: every wave stores granule (tid mod n) of the [16][H] tile; a step without an
  // h to store writes the scratch time row T.
  constexpr int n_gh = 16 * H / 4;
  const int gh = (tid % n_gh) * 4;
  float* hbase = hout + (size_t)row0 * H + gh;
  const size_t hstep = (size_t)Mp * H;

#pragma unroll
  for (int j = 0; j < D; ++j) xr[j].load(xbase + (size_t)min(j, T - 1) * xstep);
  __syncthreads();
#pragma unroll
  for (int q = 0; q < GR; ++q) xs[0][gx_seq][gx_k + q] = (__bf16)xr[0].v[q];
  xr[0].load(xbase + (size_t)min(D, T - 1) * xstep);
  float c[CPL];
#pragma unroll
  for (int cc = 0; cc < CPL; ++cc) c[cc] = 0.f;
  __syncthreads();

  // steps 0 .. T (step T only stores h_{T-1})
  for (int t0 = 0; t0 <= T; t0 += D) {
#pragma unroll
    for (int j = 0; j < D; ++j) {
      const int t = t0 + j;
      const int p = t & 1;
      const int jn = (j + 1 == D) ? 0 : j + 1;
      {                                             // h_{t-1}: one contiguous tile
        const int ts = (t >= 1 && t <= T) ? t - 1 : T;
        const float4 v = *reinterpret_cast<const float4*>(&hf[p ^ 1][gh / H][gh % H]);
        *reinterpret_cast<float4*>(hbase + (size_t)ts * hstep) = v;
      }
      f32x4_t acc[CPL];
#pragma unroll
      for (int cc = 0; cc < CPL; ++cc) {
        // x and h parts in independent accumulators: their MFMA chains overlap instead of
        // the h part waiting for the x part's result
        f32x4_t accx = bias4[cc], acch = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < KX; ++s) {
          const bf16x8_t bx = *reinterpret_cast<const bf16x8_t*>(&xs[p][col][32 * s + 8 * quad]);
          accx = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wfr[cc][s], bx, accx, 0, 0, 0);
        }
#pragma unroll
        for (int s = 0; s < C::KSH; ++s) {
          const bf16x8_t bh = *reinterpret_cast<const bf16x8_t*>(&hs[p][col][32 * s + 8 * quad]);
          acch = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ufr[cc][s], bh, acch, 0, 0, 0);
        }
        acc[cc] = accx + acch;
      }
      // stage x_{t+1}, refill the slot with x_{t+1+D}
#pragma unroll
      for (int q = 0; q < GR; ++q) xs[p ^ 1][gx_seq][gx_k + q] = (__bf16)xr[jn].v[q];
      xr[jn].load(xbase + (size_t)min(t + 1 + D, T - 1) * xstep);
#pragma unroll
      for (int cc = 0; cc < CPL; ++cc) {
        const float iv = sigmoidf_fast(acc[cc][0]);
        const float fv = sigmoidf_fast(acc[cc][1]);
        const float gv = tanhf_fast(acc[cc][2]);
        const float ov = sigmoidf_fast(acc[cc][3]);
        c[cc] = fv * c[cc] + iv * gv;
        const float hv = ov * tanhf_fast(c[cc]);
        const int u = unit[cc];
        hs[p ^ 1][col][u] = (__bf16)hv;
        hf[p][col][u] = hv;
        if constexpr (TRAIN) {                       // steps past T-1 write the scratch row T
          const size_t o = ((((size_t)min(t, T) * ntiles + tile) * NW + w) * CPL + cc) * 64 + lane;
          if constexpr (SG) *reinterpret_cast<uint2*>(gbuf + o * 4) = gates_pack(iv, fv, gv, ov);
          if constexpr (!SG && TM_RG_BF16C) reinterpret_cast<__bf16*>(cbuf)[o] = (__bf16)c[cc];
          else cbuf[o] = c[cc];
        }
      }
      lds_barrier();
    }
  }
}

// =====================================================================================
// forward of a layer PAIR (layer A: Din -> H, layer B: H -> H, both return_sequences),
// wavefront-pipelined inside one workgroup: waves [0, NW) run layer A at step s while waves
// [NW, 2 NW) run layer B at step s - 1, fed from A's bf16 h tile in LDS (no HBM round trip,
// no second launch). One LDS barrier per step for both layers, so the pair costs ~one
// recurrence of T + 1 steps instead of two of T. Outputs and saved state are exactly those
// of two lstm_tm_fwd_kernel launches (same bf16 operands, same accumulation order).
// (The reference stacks time1/time2 and time_layers[2i]/[2i+1], libs/create_model.py:61-79.)
// PL: MaxPooling1D(P) of layer B's output in the same launch - the storer lanes of layer B keep a
// running max + byte argmax of their h granule (PoolAcc) and write the pooled tile and its argmax
// when a window closes (the maxpool1d_fwd pass over hB is gone; hB itself is still stored for the
// backward)
template <int H, bool TRAIN, int KX, int GR, int D, bool SG = true, bool PL = false>
__global__ __launch_bounds__(2 * TMC<H>::NT, (TmOcc<2 * TMC<H>::NT, KX>::W)) void lstm_tm2_fwd_kernel(
    const float* __restrict__ x, const float* __restrict__ WA, const float* __restrict__ UA,
    const float* __restrict__ bA, const float* __restrict__ WB, const float* __restrict__ UB,
    const float* __restrict__ bB, float* __restrict__ hA, __bf16* __restrict__ gA, float* __restrict__ cA,
    float* __restrict__ hB, __bf16* __restrict__ gB, float* __restrict__ cB, int Mp, int T, int Din, int Dw,
    int P = 0, float* __restrict__ pout = nullptr, unsigned* __restrict__ iout = nullptr) {
  using C = TMC<H>;
  static_assert(C::CPL == 1, "pair kernel: one cell per lane (H <= 64)");
  constexpr int NW = C::NW, NTL = C::NT, G4 = C::G4;
  constexpr int KPX = 32 * KX;
  constexpr int KS = C::KSH;                       // K steps over an H-wide operand
  constexpr int KW = KX > KS ? KX : KS;
  // [layer][parity]: indexed (not pointer-selected) so every access stays a DS instruction
  __shared__ __attribute__((aligned(16))) __bf16 hs[2][2][16][C::KPH + 8];
  __shared__ __attribute__((aligned(16))) __bf16 xs[2][16][KPX + 8];
  __shared__ __attribute__((aligned(16))) float hf[2][2][16][C::HP];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const bool layerB = wv >= NW;                     // SGPR: branches on it are scalar
  const int L = layerB ? 1 : 0;
  const int w = layerB ? wv - NW : wv;
  const int tl = tid - (layerB ? NTL : 0);          // thread index within the layer
  const int col = lane & 15, quad = lane >> 4;
  const int tile = blockIdx.x, ntiles = gridDim.x, row0 = tile * 16;

  for (int i = tid; i < 2 * 2 * 16 * (C::KPH + 8); i += 2 * NTL) (&hs[0][0][0][0])[i] = (__bf16)0.0f;
  for (int i = tid; i < 2 * 16 * (KPX + 8); i += 2 * NTL) (&xs[0][0][0])[i] = (__bf16)0.0f;

  // A fragments (rows permuted as in lstm_tm_fwd_kernel): U and W of this wave's layer
  const float* Ul = layerB ? UB : UA;
  const float* Wl = layerB ? WB : WA;
  const float* bl = layerB ? bB : bA;
  const int Dl = layerB ? H : Dw;                   // rows of this layer's W
  bf16x8_t ufr[KS], wfr[KW];
  const int au = 4 * w + (col >> 2), ag = col & 3;
  const int unit = 4 * w + quad;
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    bf16x8_t v;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = 32 * s + 8 * quad + j;
      v[j] = (__bf16)(Ul[min(k, H - 1) * G4 + ag * H + au] * (k < H ? 1.0f : 0.0f));
    }
    ufr[s] = v;
  }
#pragma unroll
  for (int s = 0; s < KW; ++s) {
    bf16x8_t v;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = 32 * s + 8 * quad + j;
      v[j] = (__bf16)(Wl[min(k, Dl - 1) * G4 + ag * H + au] * (k < Dl ? 1.0f : 0.0f));
    }
    wfr[s] = v;
  }
  const f32x4_t bias4 = f32x4_t{bl[unit], bl[H + unit], bl[2 * H + unit], bl[3 * H + unit]};

  // x loader (all threads, granule tid mod n; duplicates are identical) and h storers
  const int n_gx = 16 * Din / GR;
  const int gx = (tid % n_gx) * GR;
  const int gx_seq = gx / Din, gx_k = gx % Din;
  const float* xbase = x + (size_t)row0 * Din + gx;
  const size_t xstep = (size_t)Mp * Din;
  Granule<GR> xr[D];
  constexpr int n_gh = 16 * H / 4;
  const int gh = (tl % n_gh) * 4;
  float* hbase = (layerB ? hB : hA) + (size_t)row0 * H + gh;
  // recompute-gates pairs (training without saved gates) store layer A's h in bf16: its readers are this
  // pair's backward (B's x stream, A's h_{t-1} stream), which stage it as bf16 MFMA operands anyway
  constexpr bool HBA = TRAIN && !SG && TM_RG_BF16H;
  __bf16* hbaseA = reinterpret_cast<__bf16*>(hA) + (size_t)row0 * H + gh;
  const size_t hstep = (size_t)Mp * H;
  __bf16* gbuf = layerB ? gB : gA;
  float* cbuf = layerB ? cB : cA;
  PoolAcc pacc{};
  const bool pooler = PL && layerB && wave_uniform(tl < n_gh);
  const int To = PL ? T / P : 0;
#pragma unroll
  for (int j = 0; j < D; ++j) xr[j].load(xbase + (size_t)min(j, T - 1) * xstep);
  __syncthreads();
#pragma unroll
  for (int q = 0; q < GR; ++q) xs[0][gx_seq][gx_k + q] = (__bf16)xr[0].v[q];
  xr[0].load(xbase + (size_t)min(D, T - 1) * xstep);
  float c = 0.f;
  __syncthreads();

  // steps 0 .. T+1: A computes t = s (s < T), B computes t = s - 1 (1 <= s <= T); each layer
  // stores the h tile of its previous step (A: s - 1, B: s - 2; invalid -> scratch row T)
  for (int t0 = 0; t0 <= T + 1; t0 += D) {
#pragma unroll
    for (int j = 0; j < D; ++j) {
      const int s = t0 + j;
      const int p = s & 1;
      const int jn = (j + 1 == D) ? 0 : j + 1;
      const int tc = layerB ? s - 1 : s;             // time step this layer computes
      {
        const int ts = (tc >= 1 && tc <= T) ? tc - 1 : T;
        const float4 v = *reinterpret_cast<const float4*>(&hf[L][p ^ 1][gh / H][gh % H]);
        if (HBA && !layerB)                        // (uniform) layer A's h in bf16, TM_RG_BF16H
          *reinterpret_cast<bf16x4_t*>(hbaseA + (size_t)ts * hstep) =
              bf16x4_t{(__bf16)v.x, (__bf16)v.y, (__bf16)v.z, (__bf16)v.w};
        else
          *reinterpret_cast<float4*>(hbase + (size_t)ts * hstep) = v;
        if constexpr (PL) {
          if (pooler && ts < T) pacc.step(v, ts, P, To, pout, iout, (size_t)row0 * H + gh, hstep);
        }
      }
      f32x4_t accx = bias4, acch = {0.f, 0.f, 0.f, 0.f};   // independent MFMA chains
      if (layerB) {
#pragma unroll
        for (int k = 0; k < KS; ++k) {
          const bf16x8_t bx = *reinterpret_cast<const bf16x8_t*>(&hs[0][p][col][32 * k + 8 * quad]);
          accx = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wfr[k], bx, accx, 0, 0, 0);
        }
      } else {
#pragma unroll
        for (int k = 0; k < KX; ++k) {
          const bf16x8_t bx = *reinterpret_cast<const bf16x8_t*>(&xs[p][col][32 * k + 8 * quad]);
          accx = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wfr[k], bx, accx, 0, 0, 0);
        }
      }
#pragma unroll
      for (int k = 0; k < KS; ++k) {
        const bf16x8_t bh = *reinterpret_cast<const bf16x8_t*>(&hs[L][p][col][32 * k + 8 * quad]);
        acch = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ufr[k], bh, acch, 0, 0, 0);
      }
      const f32x4_t acc = accx + acch;
      // stage x_{s+1}, refill the slot with x_{s+1+D}
#pragma unroll
      for (int q = 0; q < GR; ++q) xs[p ^ 1][gx_seq][gx_k + q] = (__bf16)xr[jn].v[q];
      xr[jn].load(xbase + (size_t)min(s + 1 + D, T - 1) * xstep);
      {
        // branch-free (a branch here makes the compiler drain the x prefetch ring at the join):
        // B's step s = 0 is masked to keep c = 0, h = 0
        const float m = tc >= 0 ? 1.f : 0.f;
        const float iv = sigmoidf_fast(acc[0]);
        const float fv = sigmoidf_fast(acc[1]);
        const float gv = tanhf_fast(acc[2]);
        const float ov = sigmoidf_fast(acc[3]);
        c = (fv * c + iv * gv) * m;
        const float hv = ov * tanhf_fast(c) * m;
        hs[L][p ^ 1][col][unit] = (__bf16)hv;
        hf[L][p][col][unit] = hv;
        if constexpr (TRAIN) {                       // invalid steps write the scratch row T
          const size_t o = (((size_t)(tc >= 0 ? min(tc, T) : T) * ntiles + tile) * NW + w) * 64 + lane;
          if constexpr (SG) *reinterpret_cast<uint2*>(gbuf + o * 4) = gates_pack(iv, fv, gv, ov);
          if constexpr (!SG && TM_RG_BF16C) reinterpret_cast<__bf16*>(cbuf)[o] = (__bf16)c;
          else cbuf[o] = c;
        }
      }
      lds_barrier();
    }
  }
}

// =====================================================================================
// backward recurrence. Per reverse step: cell phase (dz_t of the lane's own cells), then
// dh_{t-1} = U dz_t on MFMA (the serial chain) and, off the chain,
//   DZ: the dz_t tile -> HBM (fp32 [T+1][Mp][4H]); the weight gradients and dx are then ONE
//       parallel pass over all T*Mp rows (lstm_grads_rows): folding them into this kernel
//       lengthens every step of the serial chain and pushes H = 32 past the VGPR budget.
//   DX: dx^T = W dz_t^T tile -> HBM (frozen-weight input gradients, e.g. integrated gradients).
// dhout: [T][Mp][H] (or [Mp][H] for the last step only). Skipped stores go to time row T.
#ifndef TMW_D16
#define TMW_D16 4        // ring depth (reverse steps) of lstm_tm_bwd_wg_kernel's streams, H = 16
#endif
#ifndef TMW_D32
#define TMW_D32 6        // H = 32 (T = 337 micro: 642 -> 555 us from 4 to 6)
#endif
#ifndef TMB_PACKED_Z
// backward: dz / x images stored as packed dwords after a lane-pair exchange (1) instead of 16-bit stores
// (0). The 16-bit stores conflict 2-way, but the exchanges cost more: 1 measured slower (SoilNet 3.29 vs
// 3.14 ms, IG 5.86 vs 5.67 ms per call, profiles/r6_packed_z_ab.txt)
#define TMB_PACKED_Z 0
#endif
__device__ __forceinline__ unsigned __bf16_bits(__bf16 v) {
  return (unsigned)__builtin_bit_cast(unsigned short, v);
}
#ifndef TMB_ZSWZ
#define TMB_ZSWZ 1       // swizzled dz tile in the backward (A/B: 0)
#endif
#ifndef TMW_SKIP
#define TMW_SKIP 0       // (timing experiments only, wrong results: 1 no weight MFMAs, 2 no x / h streams,
#endif                   //  4 no transposed dz copy; T = 337 micro, H = 16: 368 -> 297 / 310 / 352 us)   // 4 bf16 (v_mfma_f32_16x16x16_bf16 operand)

// WG (H <= 32 layers of many tiles, e.g. SoilNet's 418): the weight gradients ride in the
// recurrence instead of a separate pass over the dz / x / h streams. Per reverse step and wave w
// (gate rows 16w .. 16w + 15):
//   dW^T | db += dz_t^T [x_t | 1]   and   dU^T += dz_t^T h_{t-1}
// as v_mfma_f32_16x16x32_bf16 over a PAIR of steps (K = 2 x the tile's 16 sequences; issued every
// other step, which halved their cost on the serial step against one 16x16x16 MFMA per step): dz^T
// comes from a column-major copy of the step's dz tile the cell phase writes next to the row-major
// one, x_t and h_{t-1} are streamed through the same kind of register ring as the saved state and
// staged transposed (bf16) beside it; four image buffers (step & 3), since the pair's older step is
// read while the faster waves already write the next one. The partial tiles stay in VGPRs for all T steps and leave once per workgroup as one
// split record of the weight-gradient pass's layout (lstm_grads_body.h: [tile][cb][DT + HT][4]
// [64][4]), summed over the tiles by the same fixed-order reduction. dz itself never reaches HBM.
// RG (recompute gates): the forward saved no gates (lstm_tm_fwd SG = false). Each step's i, f, g, o
// are recomputed here from x_t and h_{t-1} - the forward's own bf16 operands, fragments, bias and MFMA
// order, so the pre-activations are bitwise the forward's - one step ahead, in the MFMA phase of the
// step before (off the serial chain: they depend on saved data only). x_t / h_{t-1} come through the
// same register rings as the WG streams and are staged row-major ([sequence][channel], the forward's B
// operand layout) into a double buffer.
// UP (un-pool on load): the layer's output went through MaxPooling1D(P) (valid, stride P) and dhout is
// the POOLED gradient [T / P][Mp][H] with the pool's byte argmax pidx of the same shape; the dh stream
// reads pooled granule floor(t / P) and its 4 argmax bytes and keeps the components whose argmax is
// t mod P (zero past the last window), as maxpool1d_bwd would have written them at full resolution -
// that kernel and its full-resolution dh round trip through HBM are gone.
template <int H, int KX, int GR, int D, bool DZ, bool DX, bool LAST, bool WG = false, bool RG = false,
          bool UP = false, bool XB = false, bool HB = false>
__device__ __forceinline__ void lstm_tm_bwd_body(
    const float* __restrict__ dhout, const __bf16* __restrict__ gbuf, const float* __restrict__ cbuf,
    const float* __restrict__ W, const float* __restrict__ U, float* __restrict__ dx, __bf16* __restrict__ dz,
    int Mp, int T, int Din, int Dw, int tile, int ntiles, const float* __restrict__ xw = nullptr,
    const float* __restrict__ hw = nullptr, float* __restrict__ wsr = nullptr,
    const float* __restrict__ bias = nullptr, const unsigned char* __restrict__ pidx = nullptr, int P = 1) {
  static_assert(!(UP && LAST), "un-pooling needs a per-step gradient");
  using C = TMC<H>;
  constexpr int CPL = C::CPL, NW = C::NW, NT = C::NT, G4 = C::G4, KB = C::KB;
  static_assert(!WG || (CPL == 1 && NT == 16 * H && G4 == 16 * NW && GR == 4), "fused weight gradients: H <= 64");
  static_assert(!RG || (CPL == 1 && NT == 16 * H && GR == 4), "recomputed gates: H <= 64, 16-byte x granules");
  constexpr bool XS = WG || RG;                   // x_t / h_{t-1} streams
  constexpr int NXB = KX * 2;                     // din blocks of dx^T (16 rows each)
  constexpr int TX = (NXB + NW - 1) / NW;         // dx tiles per wave
  static_assert(16 * G4 / 4 == NT, "one dz float4 granule per thread");
  // LDS pitches chosen with a model of the gfx950 bank rules (MI355X_MICROARCH.md §LDS: ds_write_b32 /
  // ds_read_b32 bank = dword mod 32 per 32-lane group, ds_read_b128 four 16-lane groups over 64 banks):
  // dz rows G4 + 16 bf16, dx rows 32 KX + 1 floats (the dx^T stores of a wave - 16 sequences x 4
  // quads - landed on 2 banks with a 32-float pitch: 16-way), x / h staging rows + 16 bf16
  constexpr int ZSP = G4 + 16, DXP = DX ? 32 * KX + 1 : 1;
  __shared__ __attribute__((aligned(16))) __bf16 zs[2][16][ZSP];        // dz row-major (B of U dz^T, W dz^T)
  // dz element e of sequence c sits at zs[.][c][zsw(c, e)]: 16-byte chunk index XOR bit 2 of the sequence
  // (scripts/lds_model/zs_swizzle.py: with the G4 + 16 pitch the cell phase's 16-bit stores were 4-way)
  auto zsw = [](int c, int e) { return TMB_ZSWZ ? e ^ (((c >> 2) & 1) << 3) : e; };
  __shared__ __attribute__((aligned(16))) float dhs[2][16][C::HP];      // dh_out tile
  __shared__ __attribute__((aligned(16))) float dxs[2][16][DXP];        // dx tile

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave index in an SGPR
  const int col = lane & 15, quad = lane >> 4;
  const int row0 = tile * 16;

  for (int i = tid; i < 2 * 16 * C::HP; i += NT) (&dhs[0][0][0])[i] = 0.f;

  // fused weight gradients (WG): transposed bf16 images [row][sequence] of dz_t, [x_t | 1] and h_{t-1}
  constexpr int XR = WG ? 32 * KX + 16 : 1;        // x image rows: channels, the bias row, zero rows
  constexpr int DTM = WG ? 2 * KX + 1 : 1;         // dW^T din blocks (incl. the bias row), upper bound
  constexpr int HTW = WG ? H / 16 : 1;             // dU^T k blocks
  constexpr int NB = WG ? 4 : 1, RP = 24;          // image buffers, row pitch (48 B: 16-byte aligned rows)
  __shared__ __attribute__((aligned(16))) __bf16 zT[NB][WG ? G4 : 1][RP];
  __shared__ __attribute__((aligned(16))) __bf16 xT[NB][XR][RP];
  __shared__ __attribute__((aligned(16))) __bf16 hT[NB][WG ? H : 1][RP];
  const int dtw = (Dw + 16) / 16;                  // din blocks of this layer (record layout DT)
  f32x4_t accW[DTM], accU[HTW];
  if constexpr (WG) {
    for (int i = tid; i < NB * XR * RP; i += NT) {
      const int dn = (i / RP) % XR;
      (&xT[0][0][0])[i] = (__bf16)(dn == Dw ? 1.f : 0.f);
    }
#pragma unroll
    for (int d = 0; d < DTM; ++d) accW[d] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < HTW; ++k) accU[k] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  }

  // A fragments of U (dh_rec) and W (dx^T): tile row `col` of cell group gi is unit
  // 4 gi + (col >> 2) when col % 4 == 0 and zero otherwise -> acc[0] is the lane's own cell
  bf16x8_t ufr[CPL][KB];
  int unit[CPL];
#pragma unroll
  for (int cc = 0; cc < CPL; ++cc) {
    const int gi = w + NW * cc;
    unit[cc] = 4 * gi + quad;
    const int au = 4 * gi + (col >> 2);
#pragma unroll
    for (int s = 0; s < KB; ++s) {
      bf16x8_t v;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float val = U[(size_t)au * G4 + 32 * s + 8 * quad + j];
        v[j] = (__bf16)(val * ((col & 3) == 0 ? 1.0f : 0.0f));
      }
      ufr[cc][s] = v;
    }
  }
  // WL (H = 64: 16 waves, 128 VGPRs each): the dx A fragments are read from an LDS image of W^T
  // instead of living in 32 VGPRs; in registers they pushed the body into 16-23 VGPRs of spills,
  // whose scratch reloads sat on the serial step
  constexpr bool WL = DX && H == 64;
  constexpr bool WRG = DX && !WL;
  __shared__ __attribute__((aligned(16))) __bf16 wls[WL ? 32 * KX : 1][WL ? G4 + 8 : 8];
  if constexpr (WL) {
    for (int i = tid; i < 32 * KX * G4; i += NT) {
      const int dn = i / G4, g = i % G4;
      wls[dn][g] = (__bf16)(dn < Dw ? W[(size_t)dn * G4 + g] : 0.f);
    }
  }
  bf16x8_t wfr[WRG ? TX : 1][WRG ? KB : 1];
  if constexpr (WRG) {
#pragma unroll
    for (int q = 0; q < TX; ++q) {
      const int xb = w + NW * q;
      const int din = 16 * xb + col;
#pragma unroll
      for (int s = 0; s < KB; ++s) {
        bf16x8_t v;
#pragma unroll
        for (int j = 0; j < 8; ++j)
          v[j] = (__bf16)(W[(size_t)min(din, Dw - 1) * G4 + 32 * s + 8 * quad + j] * ((xb < NXB && din < Dw) ? 1.0f : 0.0f));
        wfr[q][s] = v;
      }
    }
  }

  // ---- streams. internal state (per lane, ring over reverse steps): gates, c_t
  uint2 rg[CPL][RG ? 1 : D];                      // packed bf16 gates (not saved under RG)
  // c_t ring: under RG the forward saved c in bf16 (TM_RG_BF16C), kept raw here and widened where used
  using CT = std::conditional_t<RG && TM_RG_BF16C, __bf16, float>;
  CT rc[CPL][D];
  auto idx = [&](int tt, int cc) { return ((((size_t)tt * ntiles + tile) * NW + w) * CPL + cc) * 64 + lane; };
#define GQ_TMB_LOAD_STATE(J, SS)                                                    \
  {                                                                                 \
    const int tt_ = max(T - 1 - (SS), 0);                                           \
    _Pragma("unroll") for (int cc = 0; cc < CPL; ++cc) {                            \
      const size_t o_ = idx(tt_, cc);                                               \
      if constexpr (!RG) rg[cc][J] = *reinterpret_cast<const uint2*>(gbuf + o_ * 4); \
      rc[cc][J] = reinterpret_cast<const CT*>(cbuf)[o_];                            \
    }                                                                               \
  }
  // Streams: every wave loads and stages granule (tid mod n) of each contiguous tile (no
  // branch around memory ops, see the forward). dh: [16][H] float4 granules.
  constexpr int n_gd = 16 * H / 4;
  const int gd = (tid % n_gd) * 4;
  const float* dbase = dhout + (size_t)row0 * H + gd;
  const size_t dstep = LAST ? 0 : (size_t)Mp * H;
  const unsigned* ibase = UP ? reinterpret_cast<const unsigned*>(pidx + (size_t)row0 * H + gd) : nullptr;
  const int Ts = UP ? T / P : 0;
  // t / P as a multiply-high (exact for t * P < 2^32); P == 1 is the identity (its magic would wrap)
  const unsigned pmag = (UP && P > 1) ? 0xFFFFFFFFu / (unsigned)P + 1u : 0u;
  float4 rd[D];
  auto dh_tile = [&](int j, int t) -> float4 { (void)t; return rd[j]; };
  // dz storer: one float4 granule of the [16][4H] tile per thread
  const int gz_seq = tid / (G4 / 4), gz_c = (tid % (G4 / 4)) * 4;
  __bf16* zbase = dz + (size_t)(row0 + gz_seq) * G4 + gz_c;
  const size_t zstep = (size_t)Mp * G4;
  // dx storer over [16][Din] granules of GR floats (lanes past the tile rewrite granule 0)
  const int n_gx = 16 * Din / GR;
  const int gx = (tid % n_gx) * GR;
  const int gx_seq = gx / Din, gx_k = gx % Din;
  const size_t xstep = (size_t)Mp * Din;
  float* sbase = dx + (size_t)row0 * Din + gx;
  // WG streams: XG consecutive floats of the [16][Din] x_t tile (threads past the tile repeat it)
  // and element tid of the [16][H] h_{t-1} tile, in rings over reverse steps like the saved state
  constexpr int XG = XS ? (16 * 32 * KX / NT > 1 ? 16 * 32 * KX / NT : 1) : 1;
  static_assert(XG <= 4, "x stream granule");
  // XB / HB: x / h_{t-1} are bf16 (a recompute-gates pair's layer-A output, TM_RG_BF16H)
  std::conditional_t<XB, GranuleH<XG>, Granule<XG>> wx[XS ? D : 1];
  std::conditional_t<HB, __bf16, float> wh[XS ? D : 1];
  const int wxe = (tid * XG) % (16 * Din);
  const int wx_seq = wxe / Din, wx_k = wxe % Din;
  const auto wxb = reinterpret_cast<std::conditional_t<XB, const __bf16*, const float*>>(xw) + (size_t)row0 * Din + wxe;
  const auto whb = reinterpret_cast<std::conditional_t<HB, const __bf16*, const float*>>(hw) + (size_t)row0 * H + tid;
  const size_t whstep = (size_t)Mp * H;
#define GQ_TMB_LOAD_W(J, SS)                                                        \
  if constexpr (XS && !(TMW_SKIP & 2)) {                                                               \
    const int tt_ = max(T - 1 - (SS), 0);                                           \
    wx[J].load(wxb + (size_t)tt_ * xstep);                                          \
    wh[J] = whb[(size_t)max(tt_ - 1, 0) * whstep];                                  \
  }

  // RG: the forward's A fragments (rows permuted: tile row `col` = gate (col & 3) of unit 4 w + (col >> 2)),
  // bias, and the row-major bf16 x_t / h_{t-1} double buffers
  constexpr int KSH = C::KSH;
  __shared__ __attribute__((aligned(16))) __bf16 xrs[RG ? 2 : 1][16][RG ? 32 * KX + 16 : 8];
  __shared__ __attribute__((aligned(16))) __bf16 hrs[RG ? 2 : 1][16][RG ? C::KPH + 16 : 8];
  bf16x8_t fu[RG ? KSH : 1], fw[RG ? KX : 1];
  f32x4_t fb4 = {0.f, 0.f, 0.f, 0.f};
  if constexpr (RG) {
    for (int i = tid; i < 2 * 16 * (32 * KX + 16); i += NT) (&xrs[0][0][0])[i] = (__bf16)0.0f;
    for (int i = tid; i < 2 * 16 * (C::KPH + 16); i += NT) (&hrs[0][0][0])[i] = (__bf16)0.0f;
    const int au = 4 * w + (col >> 2), ag = col & 3;
#pragma unroll
    for (int s = 0; s < KSH; ++s) {
      bf16x8_t v;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int k = 32 * s + 8 * quad + j;
        v[j] = (__bf16)(U[min(k, H - 1) * G4 + ag * H + au] * (k < H ? 1.0f : 0.0f));
      }
      fu[s] = v;
    }
#pragma unroll
    for (int s = 0; s < KX; ++s) {
      bf16x8_t v;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int k = 32 * s + 8 * quad + j;
        v[j] = (__bf16)(W[min(k, Dw - 1) * G4 + ag * H + au] * (k < Dw ? 1.0f : 0.0f));
      }
      fw[s] = v;
    }
    const int u = 4 * w + quad;
    fb4 = f32x4_t{bias[u], bias[H + u], bias[2 * H + u], bias[3 * H + u]};
  }
  // x_tt and h_{tt-1} of ring slot J into buffer b (h_{-1} = 0)
  auto rg_stage = [&](int b, int J, int tt) {
    if constexpr (RG) {
      if constexpr (XG % 2 == 0 && TMB_PACKED_Z) {   // channel pairs as dwords (wx_k is even)
#pragma unroll
        for (int q = 0; q < XG; q += 2)
          *reinterpret_cast<unsigned*>(&xrs[b][wx_seq][wx_k + q]) =
              __bf16_bits(wx[J].bf(q)) | (__bf16_bits(wx[J].bf(q + 1)) << 16);
      } else {
#pragma unroll
        for (int q = 0; q < XG; ++q) xrs[b][wx_seq][wx_k + q] = wx[J].bf(q);
      }
      hrs[b][tid / H][tid % H] = (__bf16)((float)wh[J] * (tt >= 1 ? 1.f : 0.f));
    }
  };
  // pre-activations from buffer b: exactly the forward's two MFMA chains (x part from the bias)
  auto rg_pre = [&](int b) -> f32x4_t {
    f32x4_t ax = fb4, ah = {0.f, 0.f, 0.f, 0.f};
    if constexpr (RG) {
#pragma unroll
      for (int s = 0; s < KX; ++s) {
        const bf16x8_t bx = *reinterpret_cast<const bf16x8_t*>(&xrs[b][col][32 * s + 8 * quad]);
        ax = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fw[s], bx, ax, 0, 0, 0);
      }
#pragma unroll
      for (int s = 0; s < KSH; ++s) {
        const bf16x8_t bh = *reinterpret_cast<const bf16x8_t*>(&hrs[b][col][32 * s + 8 * quad]);
        ah = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fu[s], bh, ah, 0, 0, 0);
      }
    }
    return ax + ah;
  };

  // reverse step s <-> time t = T-1-s. Streams for step s are loaded D steps ahead.
#define GQ_TMB_LOAD_D(J, SS)                                                                \
  if constexpr (UP) {                                                                       \
    const int tt_ = max(T - 1 - (SS), 0);                                                   \
    const int st_ = P > 1 ? (int)__umulhi((unsigned)tt_, pmag) : tt_;                      \
    const int sc_ = min(st_, Ts - 1);                                                       \
    float4 v_ = *reinterpret_cast<const float4*>(dbase + (size_t)sc_ * dstep);              \
    const unsigned id_ = ibase[(size_t)sc_ * dstep / 4];                                    \
    const unsigned ph_ = st_ < Ts ? (unsigned)(tt_ - st_ * P) : 0xffu + 1u;                 \
    v_.x = (id_ & 0xffu) == ph_ ? v_.x : 0.f;                                               \
    v_.y = ((id_ >> 8) & 0xffu) == ph_ ? v_.y : 0.f;                                        \
    v_.z = ((id_ >> 16) & 0xffu) == ph_ ? v_.z : 0.f;                                       \
    v_.w = (id_ >> 24) == ph_ ? v_.w : 0.f;                                                 \
    rd[J] = v_;                                                                             \
  } else {                                                                                  \
    const int tt_ = max(T - 1 - (SS), 0);                                                   \
    float4 v_ = *reinterpret_cast<const float4*>(dbase + (size_t)tt_ * dstep);              \
    if (LAST) {                                                                             \
      const float m_ = (SS) == 0 ? 1.f : 0.f;                                               \
      v_.x *= m_; v_.y *= m_; v_.z *= m_; v_.w *= m_;                                       \
    }                                                                                       \
    rd[J] = v_;                                                                             \
  }
#pragma unroll
  for (int j = 0; j < D; ++j) {
    GQ_TMB_LOAD_STATE(j, j)
    GQ_TMB_LOAD_D(j, j)
    GQ_TMB_LOAD_W(j, j)
  }
  __syncthreads();
  // stage step 0 (t = T-1) tiles
  *reinterpret_cast<float4*>(&dhs[0][gd / H][gd % H]) = dh_tile(0, T - 1);
  GQ_TMB_LOAD_D(0, D)
  rg_stage(0, 0, T - 1);
  float dc[CPL], dhr[CPL], dhn[CPL];
#pragma unroll
  for (int cc = 0; cc < CPL; ++cc) dc[cc] = dhr[cc] = 0.f;
  __syncthreads();
  // (RG) gates of the step to come: pre-activations from the MFMA phase of the step before, activated
  // at the end of that phase (after its dx / weight-gradient MFMAs have covered the MFMA latency)
  auto rg_act = [&](const f32x4_t& a) {
    return make_float4(sigmoidf_fast(a[0]), sigmoidf_fast(a[1]), tanhf_fast(a[2]), sigmoidf_fast(a[3]));
  };
  f32x4_t pre = rg_pre(0);
  float4 gn = make_float4(0.f, 0.f, 0.f, 0.f);
  if constexpr (RG) gn = rg_act(pre);
  // dh_out of the step to come, read from LDS one step early (right after the barrier that
  // published it) so the cell phase does not wait on an LDS round trip
#pragma unroll
  for (int cc = 0; cc < CPL; ++cc) dhn[cc] = dhs[0][col][unit[cc]];

  for (int s0 = 0; s0 < T; s0 += D) {
#pragma unroll
    for (int j = 0; j < D; ++j) {
      const int s = s0 + j;
      const int t = T - 1 - s;
      const int p = s & 1;
      const int jn = (j + 1 == D) ? 0 : j + 1;
      // ---------------- cell phase
#pragma unroll
      for (int cc = 0; cc < CPL; ++cc) {
        const int u = unit[cc];
        const float cp = (float)rc[cc][jn] * (t > 0 ? 1.f : 0.f);      // c_{t-1}
        const float dh = dhn[cc] + dhr[cc];
        float4 g4;
        if constexpr (RG)
          g4 = gn;
        else
          g4 = gates_unpack(rg[cc][j]);
        const float tc = tanhf_fast((float)rc[cc][j]);
        const float dct = dc[cc] + dh * g4.w * (1.f - tc * tc);
        dc[cc] = dct * g4.y;
        const __bf16 z0 = (__bf16)(dct * g4.z * g4.x * (1.f - g4.x));
        const __bf16 z1 = (__bf16)(dct * cp * g4.y * (1.f - g4.y));
        const __bf16 z2 = (__bf16)(dct * g4.x * (1.f - g4.z * g4.z));
        const __bf16 z3 = (__bf16)(dh * tc * g4.w * (1.f - g4.w));
        if constexpr (CPL == 1 && TMB_PACKED_Z) {
          // dword stores instead of 16-bit ones (two lanes writing the two halves of one dword was a
          // 2-way bank conflict on every dz store: ~1/3 of the LDS cycles of the H = 16 backward were
          // conflicts). zs: units u, u + 1 (quads q, q ^ 1 = lanes l, l ^ 16) share a dword; the even quad
          // stores gates 0, 1, the odd one gates 2, 3, after one exchange of packed gate pairs. zT:
          // sequences col, col ^ 1 (lanes l, l ^ 1) share a dword; the same split by col parity.
          const unsigned b0 = __bf16_bits(z0), b1 = __bf16_bits(z1), b2 = __bf16_bits(z2), b3 = __bf16_bits(z3);
          const unsigned lo = b0 | (b1 << 16), hi = b2 | (b3 << 16);
          const bool qo = quad & 1;
          const unsigned rq = (unsigned)__shfl_xor((int)(qo ? lo : hi), 16, 64);   // partner unit's pair
          const int gq = qo ? 2 : 0, ub = u & ~1;
          const unsigned mq0 = qo ? b2 : b0, mq1 = qo ? b3 : b1;                    // my gates gq, gq + 1
          const unsigned w0 = qo ? ((rq & 0xffffu) | (mq0 << 16)) : (mq0 | (rq << 16));
          const unsigned w1 = qo ? ((rq >> 16) | (mq1 << 16)) : (mq1 | (rq & 0xffff0000u));
          *reinterpret_cast<unsigned*>(&zs[p][col][zsw(col, gq * H + ub)]) = w0;
          *reinterpret_cast<unsigned*>(&zs[p][col][zsw(col, (gq + 1) * H + ub)]) = w1;
          if constexpr (WG && !(TMW_SKIP & 4)) {
            const bool co = col & 1;
            const unsigned rc2 = (unsigned)__shfl_xor((int)(co ? lo : hi), 1, 64);  // partner sequence's pair
            const int gc = co ? 2 : 0, cb = col & ~1;
            const unsigned mc0 = co ? b2 : b0, mc1 = co ? b3 : b1;
            const unsigned v0 = co ? ((rc2 & 0xffffu) | (mc0 << 16)) : (mc0 | (rc2 << 16));
            const unsigned v1 = co ? ((rc2 >> 16) | (mc1 << 16)) : (mc1 | (rc2 & 0xffff0000u));
            *reinterpret_cast<unsigned*>(&zT[s & 3][gc * H + u][cb]) = v0;
            *reinterpret_cast<unsigned*>(&zT[s & 3][(gc + 1) * H + u][cb]) = v1;
          }
        } else {
          zs[p][col][zsw(col, 0 * H + u)] = z0;
          zs[p][col][zsw(col, 1 * H + u)] = z1;
          zs[p][col][zsw(col, 2 * H + u)] = z2;
          zs[p][col][zsw(col, 3 * H + u)] = z3;
          if constexpr (WG && !(TMW_SKIP & 4)) {
            zT[s & 3][0 * H + u][col] = z0;
            zT[s & 3][1 * H + u][col] = z1;
            zT[s & 3][2 * H + u][col] = z2;
            zT[s & 3][3 * H + u][col] = z3;
          }
        }
      }
      if constexpr (WG && !(TMW_SKIP & 2)) {   // stage [x_t | 1] and h_{t-1} of this step, refill the slots
        const float hm = t >= 1 ? 1.f : 0.f;
#pragma unroll
        for (int q = 0; q < XG; ++q) {
          const int dn = wx_k + q;
          xT[s & 3][dn][wx_seq] = dn < Dw ? wx[j].bf(q) : (__bf16)(dn == Dw ? 1.f : 0.f);
        }
        hT[s & 3][tid % H][tid / H] = (__bf16)((float)wh[j] * hm);
      }
      rg_stage((s + 1) & 1, jn, t - 1);            // (RG) x_{t-1}, h_{t-2}: the next step's gates
      GQ_TMB_LOAD_W(j, s + D)
      GQ_TMB_LOAD_STATE(j, s + D)
      *reinterpret_cast<float4*>(&dhs[p ^ 1][gd / H][gd % H]) = dh_tile(jn, t - 1);   // dh tile of step s+1
      GQ_TMB_LOAD_D(jn, s + 1 + D)
      lds_barrier();
#pragma unroll
      for (int cc = 0; cc < CPL; ++cc) dhn[cc] = dhs[p ^ 1][col][unit[cc]];   // next step's dh_out
      // ---------------- MFMA phase
      // (a) serial chain: dh_{t-1} = U dz_t
#pragma unroll
      for (int cc = 0; cc < CPL; ++cc) {
        f32x4_t a0 = {0.f, 0.f, 0.f, 0.f}, a1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int k = 0; k < KB; ++k) {
          const bf16x8_t bz = *reinterpret_cast<const bf16x8_t*>(&zs[p][col][zsw(col, 32 * k + 8 * quad)]);
          if (k & 1) a1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ufr[cc][k], bz, a1, 0, 0, 0);
          else a0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ufr[cc][k], bz, a0, 0, 0, 0);
        }
        dhr[cc] = a0[0] + a1[0];
      }
      if constexpr (RG) pre = rg_pre((s + 1) & 1);   // next step's gates, behind the serial chain
      // (a') weight gradients of the step pair (s - 1, s) at odd s, or of the last step alone
      // (K lanes of the missing older step zeroed); the unrolled chunk's pad steps add nothing
      if (WG && !(TMW_SKIP & 1) && t >= 0 && ((s & 1) || t == 0)) {
        const int half = quad >> 1, so = 8 * (quad & 1);      // K = 8 quad + i -> (step of the pair, sequence)
        const int bk = half ? (s & 3) : ((s - 1) & 3);
        const bool live = half || (s & 1);
        const bf16x8_t zero8 = {};
        // (both operands of a dead half are zeroed: its buffers may hold anything, NaN patterns too)
        bf16x8_t az = *reinterpret_cast<const bf16x8_t*>(&zT[bk][16 * w + col][so]);
        az = live ? az : zero8;
#pragma unroll
        for (int d = 0; d < DTM; ++d)
          if (d < dtw) {                            // wave-uniform, no global memory access inside
            bf16x8_t bx = *reinterpret_cast<const bf16x8_t*>(&xT[bk][16 * d + col][so]);
            bx = live ? bx : zero8;
            accW[d] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(az, bx, accW[d], 0, 0, 0);
          }
#pragma unroll
        for (int k = 0; k < HTW; ++k) {
          bf16x8_t bh = *reinterpret_cast<const bf16x8_t*>(&hT[bk][16 * k + col][so]);
          bh = live ? bh : zero8;
          accU[k] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(az, bh, accU[k], 0, 0, 0);
        }
      }
      // (b) dz tile of this step -> HBM as bf16 (its exact values: the MFMAs above consumed
      // these bf16 values; steps past t = 0 pad the unrolled chunk: scratch row)
      if constexpr (DZ) {
        const uint2 zv = *reinterpret_cast<const uint2*>(&zs[p][gz_seq][zsw(gz_seq, gz_c)]);
        const int tz = t >= 0 ? t : T;
        *reinterpret_cast<uint2*>(zbase + (size_t)tz * zstep) = zv;
      }
      // (c) previous step's dx tile -> HBM (written by all waves before this barrier)
      if constexpr (DX) {
        const int ts = (s >= 1 && s <= T) ? t + 1 : T;
#pragma unroll
        for (int q = 0; q < GR; ++q) sbase[(size_t)ts * xstep + q] = dxs[p ^ 1][gx_seq][gx_k + q];
      }
      // (d) dx^T = W dz^T for this step (steps past t = 0 only pad the unrolled chunk and
      // must not overwrite the t = 0 tile the epilogue stores; no memory op in the branch)
      if (DX && t >= 0) {
#pragma unroll
        for (int q = 0; q < TX; ++q) {
          const int xb = w + NW * q;
          if (xb < NXB) {                           // wave-uniform
            f32x4_t a = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int k = 0; k < KB; ++k) {
              const bf16x8_t bz = *reinterpret_cast<const bf16x8_t*>(&zs[p][col][zsw(col, 32 * k + 8 * quad)]);
              bf16x8_t wa;
              if constexpr (WL) wa = *reinterpret_cast<const bf16x8_t*>(&wls[16 * xb + col][32 * k + 8 * quad]);
              else wa = wfr[q][k];
              a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa, bz, a, 0, 0, 0);
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) dxs[p][col][16 * xb + 4 * quad + r] = a[r];
          }
        }
      }
      if constexpr (RG) gn = rg_act(pre);           // the next step's gates
    }
  }
  __syncthreads();
  if constexpr (DX) {   // dx tile of t = 0
    const int pl = (T - 1) & 1;
#pragma unroll
    for (int q = 0; q < GR; ++q) sbase[q] = dxs[pl][gx_seq][gx_k + q];
  }
  if constexpr (WG) {   // this tile's split record: wave w = column block w / 4, record wave w % 4
    const int cb = w >> 2, wr = w & 3;
    float* rec = wsr + ((size_t)tile * (G4 / 64) + cb) * (size_t)(dtw + HTW) * 1024;
#pragma unroll
    for (int d = 0; d < DTM; ++d)
      if (d < dtw) *reinterpret_cast<f32x4_t*>(rec + ((size_t)(d * 4 + wr) * 64 + lane) * 4) = accW[d];
#pragma unroll
    for (int k = 0; k < HTW; ++k)
      *reinterpret_cast<f32x4_t*>(rec + ((size_t)((dtw + k) * 4 + wr) * 64 + lane) * 4) = accU[k];
  }
#undef GQ_TMB_LOAD_STATE
#undef GQ_TMB_LOAD_D
#undef GQ_TMB_LOAD_W
}

template <int H, int KX, int GR, int D, bool DZ, bool DX, bool LAST, bool RG = false, bool UP = false,
          bool XB = false, bool HB = false>
__global__ __launch_bounds__(TMC<H>::NT) void lstm_tm_bwd_kernel(
    const float* __restrict__ dhout, const __bf16* __restrict__ gbuf, const float* __restrict__ cbuf,
    const float* __restrict__ W, const float* __restrict__ U, float* __restrict__ dx, __bf16* __restrict__ dz,
    int Mp, int T, int Din, int Dw, const float* __restrict__ x = nullptr, const float* __restrict__ h = nullptr,
    const float* __restrict__ bias = nullptr, const unsigned char* __restrict__ pidx = nullptr, int P = 1) {
  lstm_tm_bwd_body<H, KX, GR, D, DZ, DX, LAST, false, RG, UP, XB, HB>(dhout, gbuf, cbuf, W, U, dx, dz, Mp, T, Din,
                                                                      Dw, blockIdx.x, gridDim.x, x, h, nullptr, bias,
                                                                      pidx, P);
}

template <int H, int KX, int D, bool DX, bool LAST, bool RG = false, bool UP = false, bool XB = false, bool HB = false>
__global__ __launch_bounds__(TMC<H>::NT) void lstm_tm_bwd_wg_kernel(
    const float* __restrict__ dhout, const __bf16* __restrict__ gbuf, const float* __restrict__ cbuf,
    const float* __restrict__ W, const float* __restrict__ U, float* __restrict__ dx, const float* __restrict__ x,
    const float* __restrict__ h, float* __restrict__ ws, int Mp, int T, int Din, int Dw,
    const float* __restrict__ bias = nullptr, const unsigned char* __restrict__ pidx = nullptr, int P = 1) {
  lstm_tm_bwd_body<H, KX, 4, D, false, DX, LAST, true, RG, UP, XB, HB>(dhout, gbuf, cbuf, W, U, dx, nullptr, Mp, T,
                                                                       Din, Dw, blockIdx.x, gridDim.x, x, h, ws, bias,
                                                                       pidx, P);
}

// =====================================================================================
// Horizontal fusion of the backward: one launch = the reverse recurrence of layer L (the
// serial critical path, workgroups [0, ntiles)) + the weight-gradient pass of the layer
// processed just before it (extra 256-thread workgroups) + the split reduction of the layer
// before that. The weight-gradient work used to run after each recurrence on the same
// stream; here it fills the idle CUs while the next recurrence runs (separate streams were
// measured slower: cross-stream event waits). Extra waves of a recurrence-sized workgroup
// exit at once (s_barrier only counts live waves).
static constexpr int PIPE_RED_KB = 8;     // slot blocks per reduce workgroup (lstm_grads_reduce_multi)


template <int HR, int HG, int DT>
__global__ __launch_bounds__(TMC<HR>::NT) void lstm_tm_bwd_dual_kernel(
    const float* __restrict__ dh, const __bf16* __restrict__ g, const float* __restrict__ c,
    const float* __restrict__ W, const float* __restrict__ U, __bf16* __restrict__ dz, int Mp, int T, int Dw,
    int ntiles, GradJob gj, RedJob rj) {
  constexpr int D = HR >= 64 ? 2 : 4;
  const int b = blockIdx.x;
  if (b < ntiles) {
    lstm_tm_bwd_body<HR, 1, 1, D, true, false, false>(dh, g, c, W, U, nullptr, dz, Mp, T, Dw, Dw, b, ntiles);
    return;
  }
  if (threadIdx.x >= 256) return;
  const int gb = b - ntiles;
  if (gb < gj.nblocks) {
    if constexpr (HG > 0)
      {
      __shared__ __attribute__((aligned(16))) char gsm[GradsLds<HG, DT>::BYTES];
      lstm_grads_body<HG, DT, 4>(gj.dz, gj.x, gj.h, gj.W, nullptr, gj.ws, gj.rows, gj.period, gj.hshift, gj.Din,
                                 gj.ldx, 0, gj.Din, gj.xg, gj.x_elems, gb % gj.ncb, gb / gj.ncb, gj.ncb, gj.splits, gsm);
    }
    return;
  }
  const int rb = gb - gj.nblocks;
  if (rb < rj.nblocks) {
    if (rj.kb > 1)     // many slots: KB slot blocks per workgroup
      lstm_grads_reduce_multi<PIPE_RED_KB>(rj.ws, rj.splits, rj.RC, rj.ncb, rj.DT, rj.HT, rj.Din, rj.H, rj.dW, rj.db,
                                           rj.dU, rb, rj.nf);
    else               // few slots, many splits: one slot block per workgroup, 4 add chains per lane
      lstm_grads_reduce_body(rj.ws, rj.splits, rj.RC, nullptr, rj.ncb, rj.DT, rj.HT, rj.Din, rj.H, rj.dW, rj.db,
                             rj.dU, rb, 0, 1, rj.nf);
  }
}

// =====================================================================================
// host side
// GNNQC_TM_RECDX=0: multi-column-block layers take dx from weight-gradient slabs + their sum
// (the earlier layout) instead of from the recurrence
static bool tm_rec_dx() {       // read per call (host side of a launch; tests toggle it)
  const char* e = std::getenv("GNNQC_TM_RECDX");
  return !(e != nullptr && e[0] == '0');
}

// Weight gradients inside the backward recurrence (lstm_tm_bwd_wg_kernel) for layers of at least
// GNNQC_TM_FUSED_WGRAD_MIN_TILES 16-sequence tiles (default 64: with few tiles the separate pass
// spreads the rows over the whole GPU, the recurrence's workgroups cannot); GNNQC_TM_FUSED_WGRAD=0
// turns it off. Read per call (tests switch them).
static bool tm_fused_wgrad(int H, int Din, int gr, int ntiles) {
  const char* e = std::getenv("GNNQC_TM_FUSED_WGRAD");
  if (e != nullptr && e[0] == '0') return false;
  const char* m = std::getenv("GNNQC_TM_FUSED_WGRAD_MIN_TILES");
  const int min_tiles = m != nullptr ? std::atoi(m) : 64;
  return (H == 16 || H == 32) && gr == 4 && Din <= 64 && ntiles >= min_tiles;
}

static int tm_granule(int Din, const void* x) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(x);
  if (Din % 4 == 0 && a % 16 == 0) return 4;
  if (Din % 2 == 0 && a % 8 == 0) return 2;
  return 1;
}

// H in {16, 32}: one cell per lane, 4 / 8 waves, comfortably inside the VGPR budget of the
// fused backward (U and W fragments + stream rings + weight-gradient accumulators). Larger
// hidden sizes keep the seq-major kernels of lstm.hip / lstm_grads.hip. The per-step
// x tile must fit the loader lanes and Din + 1 (bias row) must fit 128.
static bool tm_supported(int H, int Din, int gr) {
  if (H != 16 && H != 32 && H != 64) return false;
  if (Din < 1 || Din > 127) return false;
  return 16 * Din / gr <= 16 * H;
}

// recompute-gates backward (lstm_tm_bwd_body RG): one cell per lane with the x / h streams of the
// fused weight-gradient kernel (H <= 32, Din <= 64, 16-byte x granules)
static bool tm_rg_ok(int H, int gr) { return (H == 16 || H == 32) && gr == 4; }

// (MaxPooling1D fused into the recurrences - running max + argmax in the forward, un-pooling on
// load in the backward - was measured slower on both shapes: CML 0.766 vs 0.713 ms, SoilNet 3.920 vs
// 3.894 ms; profiles/r3_bench_soilnet_poolfusion.json. Pooling runs as pool.hip kernels.)
template <int H, bool TRAIN, int KX, int GR>
static void tm_fwd_cfg(int ntiles, const float* x, const float* W, const float* U, const float* b, float* h, __bf16* g,
                       float* c, int Mp, int T, int Din, int Dw, hipStream_t st) {
  constexpr int D = 6;
  if (TRAIN && g == nullptr)      // recompute-gates backward: c only
    hipLaunchKernelGGL((lstm_tm_fwd_kernel<H, TRAIN, KX, GR, D, false>), dim3(ntiles), dim3(TMC<H>::NT), 0, st, x, W,
                       U, b, h, g, c, Mp, T, Din, Dw);
  else
    hipLaunchKernelGGL((lstm_tm_fwd_kernel<H, TRAIN, KX, GR, D>), dim3(ntiles), dim3(TMC<H>::NT), 0, st, x, W, U, b,
                       h, g, c, Mp, T, Din, Dw);
}

template <int H, int KX, int GR, bool DZF, bool DXF, bool LAST>
static void tm_bwd_cfg(int ntiles, const float* dh, const __bf16* g, const float* c, const float* W, const float* U,
                       float* dx, __bf16* dz, int Mp, int T, int Din, int Dw, hipStream_t st,
                       const unsigned char* pidx = nullptr, int P = 0) {
  constexpr int D = H >= 64 ? 2 : 4;        // H = 64: 16 waves x 128 VGPRs, shorter state rings
  if constexpr (!LAST && GR == 4) {
    if (pidx != nullptr) {                  // un-pool on load (the pooled dh of a fused layer + pool)
      hipLaunchKernelGGL((lstm_tm_bwd_kernel<H, KX, GR, D, DZF, DXF, LAST, false, true>), dim3(ntiles),
                         dim3(TMC<H>::NT), 0, st, dh, g, c, W, U, dx, dz, Mp, T, Din, Dw, nullptr, nullptr, nullptr,
                         pidx, P);
      return;
    }
  }
  TORCH_CHECK(pidx == nullptr, "lstm_tm_bwd: un-pooling takes a per-step gradient and 16-byte granules");
  hipLaunchKernelGGL((lstm_tm_bwd_kernel<H, KX, GR, D, DZF, DXF, LAST>), dim3(ntiles), dim3(TMC<H>::NT), 0, st, dh, g,
                     c, W, U, dx, dz, Mp, T, Din, Dw);
}

#define GQ_TM_H_DISPATCH(HV, ...)                                  \
  switch (HV) {                                                    \
    case 16: { constexpr int HH = 16; __VA_ARGS__; break; }        \
    case 32: { constexpr int HH = 32; __VA_ARGS__; break; }        \
    case 64: { constexpr int HH = 64; __VA_ARGS__; break; }        \
    default: TORCH_CHECK(false, "lstm_tm: hidden size must be 16, 32 or 64");  \
  }
// layer pairs run 2 x H/4 waves in one workgroup: H <= 32
#define GQ_TM2_H_DISPATCH(HV, ...)                                 \
  switch (HV) {                                                    \
    case 16: { constexpr int HH = 16; __VA_ARGS__; break; }        \
    case 32: { constexpr int HH = 32; __VA_ARGS__; break; }        \
    default: TORCH_CHECK(false, "lstm_tm2: hidden size must be 16 or 32");  \
  }
#define GQ_TM_KX_DISPATCH(KXN, ...)                                \
  {                                                                \
    const int kx_ = (KXN);                                         \
    if (kx_ == 1) { constexpr int KXX = 1; __VA_ARGS__; }          \
    else if (kx_ == 2) { constexpr int KXX = 2; __VA_ARGS__; }     \
    else { constexpr int KXX = 4; __VA_ARGS__; }                   \
  }
#define GQ_TM_GR_DISPATCH(GRV, ...)                                \
  {                                                                \
    if (GRV == 4) { constexpr int GRR = 4; __VA_ARGS__; }          \
    else if (GRV == 2) { constexpr int GRR = 2; __VA_ARGS__; }     \
    else { constexpr int GRR = 1; __VA_ARGS__; }                   \
  }

// x: [T, Mp, Din] time-major; W: [Dw, 4H] with Dw <= Din (x channels >= Dw must be zero, e.g. the
// alignment padding of a 19-channel input to 20). Returns [h (T,Mp,H), gates (state), c (state)].
// store_gates = false (train): the gates state is empty and the backward recomputes the gates
// (lstm_tm_bwd with an empty g; H <= 32, 16-byte x granules: tm_rg_ok).
std::vector<at::Tensor> lstm_tm_fwd(const at::Tensor& x, const at::Tensor& W, const at::Tensor& U,
                                    const at::Tensor& b, bool train, bool store_gates) {
  check_f32_cuda(x, "x");
  check_f32_cuda(W, "W");
  check_f32_cuda(U, "U");
  check_f32_cuda(b, "b");
  TORCH_CHECK(x.dim() == 3, "lstm_tm_fwd: x must be [T, Mp, Din]");
  const int T = (int)x.size(0), Mp = (int)x.size(1), Din = (int)x.size(2), H = (int)U.size(0);
  TORCH_CHECK(Mp % 16 == 0 && Mp > 0 && T > 0, "lstm_tm_fwd: Mp must be a positive multiple of 16");
  const int Dw = (int)W.size(0);
  TORCH_CHECK(U.size(1) == 4 * H && Dw >= 1 && Dw <= Din && W.size(1) == 4 * H && b.numel() == 4 * H,
              "lstm_tm_fwd: weight shapes");
  const int gr = tm_granule(Din, x.data_ptr());
  TORCH_CHECK(tm_supported(H, Din, gr), "lstm_tm_fwd: unsupported (H, Din) = (", H, ", ", Din, ")");
  TORCH_CHECK(store_gates || !train || tm_rg_ok(H, gr), "lstm_tm_fwd: recomputed gates need H <= 32, Din % 4 == 0");
  c10::DeviceGuard guard(x.device());
  auto opt = x.options();
  // one extra (scratch) time row: stores of steps that have nothing to store land there
  at::Tensor h = at::empty({T + 1, Mp, H}, opt);
  at::Tensor g = (train && store_gates) ? at::empty({T + 1, Mp, H, 4}, opt.dtype(at::kBFloat16))
                                        : at::empty({0}, opt.dtype(at::kBFloat16));
  const bool cbf = train && !store_gates && TM_RG_BF16C;     // (recompute-gates c in bf16)
  at::Tensor c = train ? at::empty({T + 1, Mp, H}, cbf ? opt.dtype(at::kBFloat16) : opt) : at::empty({0}, opt);
  const int ntiles = Mp / 16;
  auto st = stream();
  __bf16* gp = (train && store_gates) ? bf16_ptr(g) : nullptr;
  float* cp = train ? reinterpret_cast<float*>(c.data_ptr()) : nullptr;
  GQ_TM_H_DISPATCH(H, GQ_TM_KX_DISPATCH((Din + 31) / 32, GQ_TM_GR_DISPATCH(gr,
      if (train) tm_fwd_cfg<HH, true, KXX, GRR>(ntiles, x.data_ptr<float>(), W.data_ptr<float>(), U.data_ptr<float>(),
                                                b.data_ptr<float>(), h.data_ptr<float>(), gp, cp, Mp, T, Din, Dw, st);
      else tm_fwd_cfg<HH, false, KXX, GRR>(ntiles, x.data_ptr<float>(), W.data_ptr<float>(), U.data_ptr<float>(),
                                           b.data_ptr<float>(), h.data_ptr<float>(), gp, cp, Mp, T, Din, Dw, st))));
  GQ_LAUNCH_CHECK();
  return {h.narrow(0, 0, T), g, c};
}

// Pair forward (lstm_tm2_fwd_kernel): x [T, Mp, Din]; A: W [Dw <= Din, 4H], B: W [H, 4H].
// Returns [hA, gA, cA, hB, gB, cB] with the layouts of lstm_tm_fwd.
// pool > 0: MaxPooling1D(pool) of hB in the same launch; two more outputs [pooled (T/pool, Mp, H), argmax
// bytes (same shape)]
std::vector<at::Tensor> lstm_tm2_fwd(const at::Tensor& x, const at::Tensor& WA, const at::Tensor& UA,
                                     const at::Tensor& bA, const at::Tensor& WB, const at::Tensor& UB,
                                     const at::Tensor& bB, bool train, bool store_gates, int64_t pool) {
  for (const at::Tensor* t : {&x, &WA, &UA, &bA, &WB, &UB, &bB}) check_f32_cuda(*t, "lstm_tm2_fwd operand");
  TORCH_CHECK(x.dim() == 3, "lstm_tm2_fwd: x must be [T, Mp, Din]");
  const int T = (int)x.size(0), Mp = (int)x.size(1), Din = (int)x.size(2), H = (int)UA.size(0);
  const int Dw = (int)WA.size(0);
  TORCH_CHECK(Mp % 16 == 0 && Mp > 0 && T > 0, "lstm_tm2_fwd: Mp must be a positive multiple of 16");
  TORCH_CHECK(UA.size(1) == 4 * H && Dw >= 1 && Dw <= Din && WA.size(1) == 4 * H && bA.numel() == 4 * H,
              "lstm_tm2_fwd: layer A weight shapes");
  TORCH_CHECK(UB.size(0) == H && UB.size(1) == 4 * H && WB.size(0) == H && WB.size(1) == 4 * H && bB.numel() == 4 * H,
              "lstm_tm2_fwd: layer B must be H -> H with the same H");
  const int gr = tm_granule(Din, x.data_ptr());
  TORCH_CHECK(H <= 32 && tm_supported(H, Din, gr), "lstm_tm2_fwd: unsupported (H, Din) = (", H, ", ", Din, ")");
  TORCH_CHECK(store_gates || !train || tm_rg_ok(H, gr), "lstm_tm2_fwd: recomputed gates need Din % 4 == 0");
  const bool sg = train && store_gates;
  c10::DeviceGuard guard(x.device());
  auto opt = x.options();
  auto mk = [&](bool state, int last) {
    return state ? (train ? at::empty({T + 1, Mp, H, last}, opt) : at::empty({0}, opt)) : at::empty({T + 1, Mp, H}, opt);
  };
  at::Tensor hA = (train && !sg && TM_RG_BF16H) ? at::empty({T + 1, Mp, H}, opt.dtype(at::kBFloat16)) : mk(false, 0);
  at::Tensor hB = mk(false, 0);
  at::Tensor gA = sg ? at::empty({T + 1, Mp, H, 4}, opt.dtype(at::kBFloat16)) : at::empty({0}, opt.dtype(at::kBFloat16));
  at::Tensor gB = sg ? at::empty({T + 1, Mp, H, 4}, opt.dtype(at::kBFloat16)) : at::empty({0}, opt.dtype(at::kBFloat16));
  const bool cbf = train && !sg && TM_RG_BF16C;              // (recompute-gates c in bf16)
  const auto copt = cbf ? opt.dtype(at::kBFloat16) : opt;
  at::Tensor cA = train ? at::empty({T + 1, Mp, H}, copt) : at::empty({0}, opt);
  at::Tensor cB = train ? at::empty({T + 1, Mp, H}, copt) : at::empty({0}, opt);
  const int ntiles = Mp / 16;
  auto st = stream();
  __bf16* PG[2] = {sg ? bf16_ptr(gA) : nullptr, sg ? bf16_ptr(gB) : nullptr};
  float* P[4] = {nullptr, train ? reinterpret_cast<float*>(cA.data_ptr()) : nullptr, nullptr,
                 train ? reinterpret_cast<float*>(cB.data_ptr()) : nullptr};
  at::Tensor pooled, pidx;
  const TmPool pl = tm_pool_outputs((int)pool, T, Mp, H, opt, pooled, pidx);
#define GQ_TM2_LAUNCH2(HH, TR, KXX, GRR, SGV, PLV)                                                              \
  hipLaunchKernelGGL((lstm_tm2_fwd_kernel<HH, TR, KXX, GRR, 6, SGV, PLV>), dim3(ntiles), dim3(2 * TMC<HH>::NT), 0,  \
                     st, x.data_ptr<float>(), WA.data_ptr<float>(), UA.data_ptr<float>(), bA.data_ptr<float>(),    \
                     WB.data_ptr<float>(), UB.data_ptr<float>(), bB.data_ptr<float>(), reinterpret_cast<float*>(hA.data_ptr()), PG[0], \
                     P[1], hB.data_ptr<float>(), PG[1], P[3], Mp, T, Din, Dw, pl.P, pl.out, pl.idx)
#define GQ_TM2_LAUNCH(HH, TR, KXX, GRR, SGV)                                                                    \
  do { if (pl.P > 0) GQ_TM2_LAUNCH2(HH, TR, KXX, GRR, SGV, true); else GQ_TM2_LAUNCH2(HH, TR, KXX, GRR, SGV, false); } \
  while (0)
  GQ_TM2_H_DISPATCH(H, GQ_TM_KX_DISPATCH((Din + 31) / 32, GQ_TM_GR_DISPATCH(gr,
      if (sg) GQ_TM2_LAUNCH(HH, true, KXX, GRR, true); else if (train) GQ_TM2_LAUNCH(HH, true, KXX, GRR, false);
      else GQ_TM2_LAUNCH(HH, false, KXX, GRR, true))));
#undef GQ_TM2_LAUNCH
#undef GQ_TM2_LAUNCH2
  GQ_LAUNCH_CHECK();
  return {hA.narrow(0, 0, T), gA, cA, hB.narrow(0, 0, T), gB, cB, pooled, pidx};
}

// ---- pipelined backward (see lstm_tm_bwd_dual_kernel)
static constexpr int PIPE_MAX_SPLITS = 512;     // one reduction group: the reduce fits one launch

// workspace of a pending weight-gradient job: [splits][ncb][(DT + HT) fragments][1024] fp32
at::Tensor lstm_grads_job_ws(const at::Tensor& dz, const at::Tensor& x, const at::Tensor& W, int64_t H) {
  check_f32_cuda(W, "W");
  const int Dw = (int)W.size(0);
  const long rows = x.numel() / x.size(-1);
  const int ncb = lstm_grads_col_blocks((int)H);
  const long ntiles = (rows + 31) / 32;
  // row tiles per split: each split writes a whole record (all column blocks) once, so few tiles
  // per split multiply the record traffic (written here, re-read by the reduction)
  static const int tps = [] {
    const char* e = std::getenv("GNNQC_GRADS_TPS");
    return e != nullptr ? std::max(1, std::atoi(e)) : 4;   // 4: best of 2 / 4 / 8 / 16 on the CML step
  }();
  const int splits = (int)std::max<long>(1, std::min<long>({(ntiles + tps - 1) / tps, (long)std::max(64, 2048 / ncb),
                                                            (long)PIPE_MAX_SPLITS}));
  const int DT = (Dw + 1 + 15) / 16, HT = (int)H / 16;
  c10::DeviceGuard guard(x.device());
  return at::empty({(long)splits * ncb * (DT + HT) * 1024}, x.options());
}

static bool grads_job_ok(const at::Tensor& x, int Dw) {
  const int ldx = (int)x.stride(-2);
  return ldx % 4 == 0 && ldx >= Dw && ldx <= 144 && reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0 &&
         (Dw + 1 + 15) / 16 <= 5 && x.stride(-1) == 1;
}

// rec: dh [T, Mp, H] (empty: no recurrence); job (gz empty: none): dz / x / h / W of the layer
// whose weight gradients to compute, with its row mapping (period, hshift) and workspace;
// reduce (rws empty: none): a job whose gradient pass already ran. Returns the rec's dz.
at::Tensor lstm_tm_bwd_pipe(const at::Tensor& dh, const at::Tensor& g, const at::Tensor& c, const at::Tensor& W,
                            const at::Tensor& U, int64_t T, const at::Tensor& gz, const at::Tensor& gx,
                            const at::Tensor& gh, const at::Tensor& gW, int64_t g_period, int64_t g_hshift,
                            const at::Tensor& gws, const at::Tensor& rws, const at::Tensor& rW, at::Tensor rdW,
                            at::Tensor rdU, at::Tensor rdb) {
  const bool rec = dh.numel() > 0, job = gz.numel() > 0, red = rws.numel() > 0;
  const at::Tensor& ref = rec ? dh : (job ? gz : rws);
  c10::DeviceGuard guard(ref.device());
  int HR = 16, Mp = 0, ntiles = 0, Dw = 1;
  at::Tensor dz = at::empty({0}, ref.options());
  if (rec) {
    for (const at::Tensor* t : {&dh, &c, &W, &U}) check_f32_cuda(*t, "lstm_tm_bwd_pipe operand");
    check_gates_cuda(g);
    HR = (int)U.size(0);
    Mp = (int)dh.size(1);
    TORCH_CHECK(dh.dim() == 3 && dh.size(0) == T && dh.size(2) == HR && Mp % 16 == 0, "lstm_tm_bwd_pipe: dh shape");
    TORCH_CHECK(g.numel() == (long)(T + 1) * Mp * HR * 4 && c.numel() == (long)(T + 1) * Mp * HR,
                "lstm_tm_bwd_pipe: saved state shapes");
    TORCH_CHECK(HR == 16 || HR == 32 || HR == 64, "lstm_tm_bwd_pipe: hidden size");
    ntiles = Mp / 16;
    Dw = (int)W.size(0);
    dz = at::empty({T + 1, Mp, 4 * HR}, dh.options().dtype(at::kBFloat16));
  }
  GradJob gj{};
  at::Tensor gz_b;
  int HG = 0, DTG = 1;
  if (job) {
    check_dz_cuda(gz);
    for (const at::Tensor* t : {&gh, &gW, &gws}) check_f32_cuda(*t, "lstm_tm_bwd_pipe job operand");
    // the job bodies read bf16 dz; an fp32 dz (sequence-major lstm_bwd) is rounded here exactly as
    // the grads body would round it when staging, so the result is the same
    if (!dz_bf16(gz)) gz_b = gz.to(at::kBFloat16);
    TORCH_CHECK(gx.is_cuda() && gx.scalar_type() == at::kFloat, "lstm_tm_bwd_pipe: job x");
    HG = (int)gW.size(1) / 4;
    const int gDw = (int)gW.size(0);
    TORCH_CHECK(grads_job_ok(gx, gDw), "lstm_tm_bwd_pipe: job x layout");
    DTG = (gDw + 1 + 15) / 16;
    gj.dz = gz_b.defined() ? gz_b.data_ptr() : gz.data_ptr();
    gj.x = gx.data_ptr<float>();
    gj.h = gh.data_ptr<float>();
    gj.W = gW.data_ptr<float>();
    gj.ws = gws.data_ptr<float>();
    gj.ldx = (int)gx.stride(-2);
    gj.rows = gx.numel() / gx.size(-1);
    gj.period = g_period;
    gj.hshift = g_hshift;
    gj.x_elems = (long)(gx.storage().nbytes() / sizeof(float)) - gx.storage_offset();
    gj.Din = gDw;
    gj.xg = (int)((32L * gj.ldx / 4 + 255) / 256);
    gj.ncb = lstm_grads_col_blocks(HG);
    const long RC = (long)(DTG + HG / 16) * 1024 * gj.ncb;
    gj.splits = (int)(gws.numel() / RC);
    TORCH_CHECK(gj.splits >= 1 && gj.splits <= PIPE_MAX_SPLITS && gws.numel() == gj.splits * RC,
                "lstm_tm_bwd_pipe: job workspace size");
    gj.nblocks = gj.ncb * gj.splits;
  }
  RedJob rj{};
  if (red) {
    for (const at::Tensor* t : {&rws, &rW}) check_f32_cuda(*t, "lstm_tm_bwd_pipe reduce operand");
    for (at::Tensor* t : {&rdW, &rdU, &rdb}) check_f32_cuda(*t, "lstm_tm_bwd_pipe reduce gradient");
    rj.H = (int)rW.size(1) / 4;
    rj.Din = (int)rW.size(0);
    rj.DT = (rj.Din + 1 + 15) / 16;
    rj.HT = rj.H / 16;
    rj.ncb = lstm_grads_col_blocks(rj.H);
    rj.RC = (rj.DT + rj.HT) * 1024 * rj.ncb;
    rj.splits = (int)(rws.numel() / rj.RC);
    TORCH_CHECK(rj.splits >= 1 && rj.splits <= PIPE_MAX_SPLITS && rws.numel() == (long)rj.splits * rj.RC,
                "lstm_tm_bwd_pipe: reduce workspace size");
    TORCH_CHECK(rdW.numel() == rW.numel() && rdU.numel() == (long)rj.H * 4 * rj.H && rdb.numel() == 4 * rj.H,
                "lstm_tm_bwd_pipe: reduce gradient buffers");
    rj.ws = rws.data_ptr<float>();
    rj.dW = rdW.data_ptr<float>();
    rj.dU = rdU.data_ptr<float>();
    rj.db = rdb.data_ptr<float>();
    rj.nf = chain_ctl(rws.get_device()) + 7;
    // the wide form once the one-block-per-16-slots grid would exceed a few waves of workgroups
    rj.kb = (rj.RC + 15) / 16 > 1024 ? PIPE_RED_KB : 1;
    rj.nblocks = (rj.RC + 16 * rj.kb - 1) / (16 * rj.kb);
  }
  const int nblk = ntiles + gj.nblocks + rj.nblocks;
  if (nblk == 0) return dz;
  TORCH_CHECK(!job || HG == HR || HG == 2 * HR || !rec, "lstm_tm_bwd_pipe: job hidden size must be H or 2H of the rec");
  const __bf16* PG = rec ? bf16_ptr(g) : nullptr;
  const float* P[5] = {rec ? dh.data_ptr<float>() : nullptr, nullptr,
                       rec ? c.data_ptr<float>() : nullptr, rec ? W.data_ptr<float>() : nullptr,
                       rec ? U.data_ptr<float>() : nullptr};
  __bf16* dzp = rec ? bf16_ptr(dz) : nullptr;
  auto st = stream();
#define GQ_PIPE_LAUNCH(HRV, HGV, DTV)                                                                          \
  hipLaunchKernelGGL((lstm_tm_bwd_dual_kernel<HRV, HGV, DTV>), dim3(nblk), dim3(TMC<HRV>::NT), 0, st, P[0], PG,    \
                     P[2], P[3], P[4], dzp, Mp, (int)T, Dw, ntiles, gj, rj)
#define GQ_PIPE_DT(HRV, HGV)                                                                                   \
  switch (DTG) {                                                                                               \
    case 1: GQ_PIPE_LAUNCH(HRV, HGV, 1); break;                                                                \
    case 2: GQ_PIPE_LAUNCH(HRV, HGV, 2); break;                                                                \
    case 3: GQ_PIPE_LAUNCH(HRV, HGV, 3); break;                                                                \
    case 4: GQ_PIPE_LAUNCH(HRV, HGV, 4); break;                                                                \
    default: GQ_PIPE_LAUNCH(HRV, HGV, 5); break;                                                               \
  }
#define GQ_PIPE_H(HRV)                                                                                         \
  if (!job) GQ_PIPE_LAUNCH(HRV, 0, 1);                                                                         \
  else if (HG == HRV) { GQ_PIPE_DT(HRV, HRV) }                                                                 \
  else { GQ_PIPE_DT(HRV, 2 * HRV) }
  if (!rec) {                   // flush launch: 256-thread workgroups; job of any hidden size
    if (!job) GQ_PIPE_LAUNCH(16, 0, 1);
    else if (HG == 16) { GQ_PIPE_DT(16, 16) }
    else if (HG == 32) { GQ_PIPE_DT(16, 32) }
    else if (HG == 64) { GQ_PIPE_DT(32, 64) }
    else { GQ_PIPE_DT(64, 128) }
  } else if (HR == 16) {
    GQ_PIPE_H(16)
  } else if (HR == 32) {
    GQ_PIPE_H(32)
  } else {
    GQ_PIPE_H(64)
  }
#undef GQ_PIPE_H
#undef GQ_PIPE_DT
#undef GQ_PIPE_LAUNCH
  GQ_LAUNCH_CHECK();
  return dz;
}

// ---- all pending weight-gradient jobs in ONE launch, then all reductions in ONE launch
// (after the chain backward, whose recurrences leave no per-layer launch to hide them in)
static constexpr int MULTI_MAX = 12;
struct MultiGrad {
  GradJob j[MULTI_MAX];
  int start[MULTI_MAX + 1];
  int key[MULTI_MAX];              // HG * 8 + DT
  int n;
  int gcn_nb;                      // > 0: blocks [0, gcn_nb) run the fused GCN backward (gcn_fused.h)
  GcnBwdJob gcn;
  int gcn_coef;                    // 1: those blocks run the coefficient form (gcn_coef_bwd_body) instead
  GcnCoefJob gcnc;
};
struct MultiRed {
  RedJob j[MULTI_MAX];
  int start[MULTI_MAX + 1];
  int n;
  int* nf;                         // non-finite gradient flag (chain control word 7)
};

__global__ __launch_bounds__(256) void lstm_grads_multi_kernel(MultiGrad M) {
  __shared__ __attribute__((aligned(16))) char smem[GradsLds<128, 5>::BYTES];   // the largest instance
  static_assert(GcnBwdLds<2, 16>::BYTES <= GradsLds<128, 5>::BYTES, "GCN job LDS");
  if ((int)blockIdx.x < M.gcn_nb) {                      // the GCN backward's workgroups
    const int gb = blockIdx.x;
    if (M.gcn_coef) gcn_coef_bwd_body<2, 16>(M.gcnc, gb);
    else if (M.gcn.key == 2 * 64 + 16)                     // (the CML configuration)
      gcn_fused_bwd_body<2, 16>(M.gcn, gb % M.gcn.B, gb / M.gcn.B, smem);
    return;
  }
  const int b = blockIdx.x - M.gcn_nb;
  int k = 0;
  while (k + 1 < M.n && b >= M.start[k + 1]) ++k;        // uniform
  const GradJob gj = M.j[k];                              // by value: scalar loads, no scratch copy
  const int gb = b - M.start[k];
#define GQ_MG(HG, DT)                                                                                    \
  case HG * 8 + DT:                                                                                      \
    lstm_grads_body<HG, DT, 4>(gj.dz, gj.x, gj.h, gj.W, nullptr, gj.ws, gj.rows, gj.period, gj.hshift, gj.Din, \
                               gj.ldx, 0, gj.Din, gj.xg, gj.x_elems, gb % gj.ncb, gb / gj.ncb, gj.ncb, gj.splits, \
                               smem);                                                                    \
    break;
#define GQ_MG_H(HG) GQ_MG(HG, 1) GQ_MG(HG, 2) GQ_MG(HG, 3) GQ_MG(HG, 4) GQ_MG(HG, 5)
  switch (M.key[k]) {
    GQ_MG_H(16) GQ_MG_H(32) GQ_MG_H(64) GQ_MG_H(128)
    default: break;
  }
#undef GQ_MG_H
#undef GQ_MG
}

__global__ __launch_bounds__(256) void lstm_grads_reduce_multi_kernel(MultiRed M) {
  const int b = blockIdx.x;
  int k = 0;
  while (k + 1 < M.n && b >= M.start[k + 1]) ++k;
  const RedJob rj = M.j[k];
  if (rj.kb > 1)
    lstm_grads_reduce_multi<PIPE_RED_KB>(rj.ws, rj.splits, rj.RC, rj.ncb, rj.DT, rj.HT, rj.Din, rj.H, rj.dW, rj.db,
                                         rj.dU, b - M.start[k], M.nf);
  else
    lstm_grads_reduce_body(rj.ws, rj.splits, rj.RC, nullptr, rj.ncb, rj.DT, rj.HT, rj.Din, rj.H, rj.dW, rj.db,
                           rj.dU, b - M.start[k], 0, 1, M.nf);
}

// gcn_fused.hip: the fused GCN backward's job (run here as extra workgroups)
GcnBwdJob gcn_bwd_job(const at::Tensor& dh, int64_t c_off, const at::Tensor& series, const at::Tensor& shift,
                      const at::Tensor& scale, const at::Tensor& win_group, const at::Tensor& win_center,
                      const at::Tensor& win_valid, const at::Tensor& group_anom_pos, const at::Tensor& pw,
                      const at::Tensor& wids, const at::Tensor& table, const c10::optional<at::Tensor>& cursor,
                      int64_t tb, int64_t seq_len, bool time_norm, const at::Tensor& S, const at::Tensor& st,
                      const at::Tensor& W, const at::Tensor& bias, const at::Tensor& alpha, const at::Tensor& dW,
                      const at::Tensor& dgamma, const at::Tensor& dbeta, const at::Tensor& dalpha, int& nblocks);

GcnCoefJob gcn_coef_job(const at::Tensor& dh, int64_t c_off, const at::Tensor& coef, const at::Tensor& S,
                        const at::Tensor& st, const at::Tensor& W, const at::Tensor& bias, const at::Tensor& dW,
                        const at::Tensor& dgamma, const at::Tensor& dbeta, const at::Tensor& dalpha);

// grads of jobs (dz, x, h, W, period, hshift, ws) then reductions of rjobs (ws, W, dW, dU, db):
// a reduce job may be one of this call's grads jobs (stream order runs the grads first).
// gcn_t / gcn_i (optional): the arguments of gcn_fused_bwd - [dh, series, shift, scale, win_group,
// win_center, win_valid, group_anom_pos, pw, wids, table, cursor (empty: none), S, st, W, bias,
// alpha, dW, dgamma, dbeta, dalpha] / [c_off, tb, seq_len, time_norm] - run as extra workgroups of
// the gradient launch (both only need the chain backward's results; the CML configuration,
// Cin = 2, F = 16, only: every instantiation would raise the launch's register allocation).
void lstm_grads_multi(at::TensorList gz, at::TensorList gx, at::TensorList gh, at::TensorList gW,
                      at::IntArrayRef period, at::IntArrayRef hshift, at::TensorList gws, at::TensorList rws,
                      at::TensorList rW, at::TensorList rdW, at::TensorList rdU, at::TensorList rdb,
                      at::TensorList gcn_t, at::IntArrayRef gcn_i) {
  const int ng = (int)gz.size(), nr = (int)rws.size();
  TORCH_CHECK(ng <= MULTI_MAX && nr <= MULTI_MAX && (int)gx.size() == ng && (int)gh.size() == ng &&
                  (int)gW.size() == ng && (int)period.size() == ng && (int)hshift.size() == ng &&
                  (int)gws.size() == ng && (int)rW.size() == nr && (int)rdW.size() == nr && (int)rdU.size() == nr &&
                  (int)rdb.size() == nr, "lstm_grads_multi: job lists");
  TORCH_CHECK((gcn_t.size() == 0 && gcn_i.size() == 0) || (gcn_t.size() == 21 && gcn_i.size() == 4) ||
                  (gcn_t.size() == 10 && gcn_i.size() == 1), "lstm_grads_multi: gcn job lists");
  TORCH_CHECK(gcn_t.size() == 0 || ng > 0, "lstm_grads_multi: a GCN job rides on a gradient launch");
  if (ng + nr == 0) return;
  c10::DeviceGuard guard(ng ? gz[0].device() : rws[0].device());
  auto st = stream();
  if (ng) {
    MultiGrad M{};
    M.n = ng;
    if (gcn_t.size() == 10) {        // coefficient form: [dh, coef, S, st, W, b, dW, dgamma, dbeta, dalpha] / [c_off]
      M.gcnc = gcn_coef_job(gcn_t[0], gcn_i[0], gcn_t[1], gcn_t[2], gcn_t[3], gcn_t[4], gcn_t[5], gcn_t[6], gcn_t[7],
                            gcn_t[8], gcn_t[9]);
      M.gcn_coef = 1;
      M.gcn_nb = M.gcnc.nblocks;
    } else if (gcn_t.size() > 0) {
      const c10::optional<at::Tensor> cur = gcn_t[11].numel() > 0 ? c10::optional<at::Tensor>(gcn_t[11]) : c10::nullopt;
      M.gcn = gcn_bwd_job(gcn_t[0], gcn_i[0], gcn_t[1], gcn_t[2], gcn_t[3], gcn_t[4], gcn_t[5], gcn_t[6], gcn_t[7],
                          gcn_t[8], gcn_t[9], gcn_t[10], cur, gcn_i[1], gcn_i[2], gcn_i[3] != 0, gcn_t[12], gcn_t[13],
                          gcn_t[14], gcn_t[15], gcn_t[16], gcn_t[17], gcn_t[18], gcn_t[19], gcn_t[20], M.gcn_nb);
      TORCH_CHECK(M.gcn.key == 2 * 64 + 16, "lstm_grads_multi: the GCN job takes 2 input / 16 output channels");
    }
    int nb = 0;
    // job bodies read bf16 dz: an fp32 one (sequence-major lstm_bwd) is rounded once here, as the
    // body would round it when staging (same result); stream-ordered, so the temporaries may go
    std::vector<at::Tensor> zb(ng);
    for (int k = 0; k < ng; ++k) {
      check_dz_cuda(gz[k]);
      zb[k] = dz_bf16(gz[k]) ? gz[k] : gz[k].to(at::kBFloat16);
      for (const at::Tensor* t : {&gh[k], &gW[k], &gws[k]}) check_f32_cuda(*t, "lstm_grads_multi operand");
      TORCH_CHECK(gx[k].is_cuda() && gx[k].scalar_type() == at::kFloat, "lstm_grads_multi: x");
      const int HG = (int)gW[k].size(1) / 4, Dw = (int)gW[k].size(0);
      TORCH_CHECK(HG == 16 || HG == 32 || HG == 64 || HG == 128, "lstm_grads_multi: hidden size");
      TORCH_CHECK(grads_job_ok(gx[k], Dw), "lstm_grads_multi: x layout");
      const int DT = (Dw + 1 + 15) / 16;
      GradJob& j = M.j[k];
      j.dz = zb[k].data_ptr();
      j.x = gx[k].data_ptr<float>();
      j.h = gh[k].data_ptr<float>();
      j.W = gW[k].data_ptr<float>();
      j.ws = gws[k].data_ptr<float>();
      j.ldx = (int)gx[k].stride(-2);
      j.rows = gx[k].numel() / gx[k].size(-1);
      j.period = period[k];
      j.hshift = hshift[k];
      j.x_elems = (long)(gx[k].storage().nbytes() / sizeof(float)) - gx[k].storage_offset();
      j.Din = Dw;
      j.xg = (int)((32L * j.ldx / 4 + 255) / 256);
      j.ncb = lstm_grads_col_blocks(HG);
      const long RC = (long)(DT + HG / 16) * 1024 * j.ncb;
      j.splits = (int)(gws[k].numel() / RC);
      TORCH_CHECK(j.splits >= 1 && j.splits <= PIPE_MAX_SPLITS && gws[k].numel() == j.splits * RC,
                  "lstm_grads_multi: workspace size");
      j.nblocks = j.ncb * j.splits;
      M.key[k] = HG * 8 + DT;
      M.start[k] = nb;
      nb += j.nblocks;
    }
    M.start[ng] = nb;
    hipLaunchKernelGGL(lstm_grads_multi_kernel, dim3(M.gcn_nb + nb), dim3(256), 0, st, M);
    GQ_LAUNCH_CHECK();
  }
  if (nr) {
    MultiRed R{};
    R.n = nr;
    R.nf = chain_ctl(rws[0].get_device()) + 7;
    int nb = 0;
    for (int k = 0; k < nr; ++k) {
      RedJob& r = R.j[k];
      r.H = (int)rW[k].size(1) / 4;
      r.Din = (int)rW[k].size(0);
      r.DT = (r.Din + 1 + 15) / 16;
      r.HT = r.H / 16;
      r.ncb = lstm_grads_col_blocks(r.H);
      r.RC = (r.DT + r.HT) * 1024 * r.ncb;
      r.splits = (int)(rws[k].numel() / r.RC);
      TORCH_CHECK(r.splits >= 1 && r.splits <= PIPE_MAX_SPLITS && rws[k].numel() == (long)r.splits * r.RC,
                  "lstm_grads_multi: reduce workspace size");
      TORCH_CHECK(rdW[k].numel() == rW[k].numel() && rdU[k].numel() == (long)r.H * 4 * r.H &&
                      rdb[k].numel() == 4 * r.H, "lstm_grads_multi: gradient buffers");
      r.ws = rws[k].data_ptr<float>();
      r.dW = rdW[k].data_ptr<float>();
      r.dU = rdU[k].data_ptr<float>();
      r.db = rdb[k].data_ptr<float>();
      r.kb = (r.RC + 15) / 16 > 1024 ? PIPE_RED_KB : 1;    // wide jobs: KB slot blocks per workgroup
      r.nblocks = (r.RC + 16 * r.kb - 1) / (16 * r.kb);
      R.start[k] = nb;
      nb += r.nblocks;
    }
    R.start[nr] = nb;
    hipLaunchKernelGGL(lstm_grads_reduce_multi_kernel, dim3(nb), dim3(256), 0, st, R);
    GQ_LAUNCH_CHECK();
  }
}

// Switch for the deferred split reductions (common.h defer_reduce_mode); returns the previous value.
bool lstm_defer_reduce(bool flag) {
  const bool old = defer_reduce_mode();
  defer_reduce_mode() = flag;
  return old;
}

// Every queued split reduction (lstm_grads_rows under defer_reduce_mode) in one launch per
// MULTI_MAX jobs: each job's slot blocks are workgroups of lstm_grads_reduce_multi_kernel, so the
// layers' reductions (7 launches of 9-36 us on the SoilNet step, all of them a tail of idle CUs)
// run side by side. Same fixed summation order per slot as the per-layer reduce: deterministic.
// Returns the number of reductions run.
int64_t lstm_reduce_flush() {
  auto& q = deferred_reds();
  const int n = (int)q.size();
  for (int k0 = 0; k0 < n; k0 += MULTI_MAX) {
    const int kn = std::min(MULTI_MAX, n - k0);
    MultiRed R{};
    R.n = kn;
    R.nf = chain_ctl(c10::hip::current_device()) + 7;
    int nb = 0;
    for (int k = 0; k < kn; ++k) {
      const DeferredRed& d = q[k0 + k];
      RedJob& r = R.j[k];
      r.H = d.H;
      r.Din = d.Din;
      r.DT = (r.Din + 1 + 15) / 16;
      r.HT = r.H / 16;
      r.ncb = lstm_grads_col_blocks(r.H);
      r.RC = (r.DT + r.HT) * 1024 * r.ncb;
      r.splits = d.splits;
      TORCH_CHECK(d.ws.numel() >= (long)r.splits * r.RC, "lstm_reduce_flush: workspace size");
      r.ws = d.ws.data_ptr<float>();
      r.dW = d.dW;
      r.dU = d.dU;
      r.db = d.db;
      r.kb = (r.RC + 15) / 16 > 1024 ? PIPE_RED_KB : 1;
      r.nblocks = (r.RC + 16 * r.kb - 1) / (16 * r.kb);
      R.start[k] = nb;
      nb += r.nblocks;
    }
    R.start[kn] = nb;
    c10::DeviceGuard guard(q[k0].ws.device());
    hipLaunchKernelGGL(lstm_grads_reduce_multi_kernel, dim3(nb), dim3(256), 0, stream(), R);
    GQ_LAUNCH_CHECK();
  }
  q.clear();       // workspaces return to the caching allocator in stream order
  return n;
}

// Weight gradients (+ dx) of one time-major layer from its dz (lstm_grads_rows): accumulates
// dW, dU, db; returns dx [T, Mp, Din] if need_dx.
at::Tensor lstm_tm_grads(const at::Tensor& dz, const at::Tensor& x, const at::Tensor& h, const at::Tensor& W,
                         at::Tensor dW, at::Tensor dU, at::Tensor db, bool need_dx) {
  check_dz_cuda(dz);
  for (const at::Tensor* t : {&x, &h, &W}) check_f32_cuda(*t, "lstm_tm_grads operand");
  for (const at::Tensor* t : {&dW, &dU, &db}) check_f32_cuda(*t, "lstm_tm_grads gradient");
  const int T = (int)x.size(0), Mp = (int)x.size(1), Din = (int)x.size(2), H = (int)h.size(2);
  const int Dw = (int)W.size(0);
  TORCH_CHECK(dz.size(0) >= T && dz.size(1) == Mp && dz.size(2) == 4 * H && h.size(0) == T && h.size(1) == Mp,
              "lstm_tm_grads: shapes");
  TORCH_CHECK(Dw <= Din && dW.numel() == (long)Dw * 4 * H && dU.numel() == (long)H * 4 * H && db.numel() == 4 * H,
              "lstm_tm_grads: gradient buffer shapes");
  c10::DeviceGuard guard(x.device());
  const long rows = (long)T * Mp;
  const int ncb = lstm_grads_col_blocks(H);
  // padding channels (>= Dw) are written as zeros by the kernel (their W rows are masked)
  at::Tensor dx = need_dx ? at::empty({ncb, T, Mp, Din}, x.options()) : at::empty({0}, x.options());
  lstm_grads_rows(dz.data_ptr(), dz_bf16(dz), x.data_ptr<float>(), h.data_ptr<float>(), W.data_ptr<float>(),
                  need_dx ? dx.data_ptr<float>() : nullptr, dW.data_ptr<float>(), dU.data_ptr<float>(),
                  db.data_ptr<float>(), rows, rows, Mp, H, Dw, Din, rows * Din, Din, rows * Din, stream());
  if (!need_dx) return dx;
  return ncb == 1 ? dx[0] : dx.sum(0);
}

at::Tensor maxpool1d_bwd(const at::Tensor& dy, const at::Tensor& idx, int64_t T, int64_t p);   // pool.hip

// dh: [T, Mp, H] (or [Mp, H] when only the last step has a gradient). Returns dx [T, Mp, Din]
// (empty if !need_dx) and accumulates dW, dU, db when they are non-empty. An empty g (the forward ran
// with store_gates = false) selects the recompute-gates backward, which needs the bias b.
// pidx / pool (optional): the layer's output went through MaxPooling1D(pool) and dh is the POOLED
// gradient [T / pool, Mp, H] with the pool's byte argmax pidx (un-pooled on load, lstm_tm_bwd_body UP).
at::Tensor lstm_tm_bwd(const at::Tensor& dh, const at::Tensor& g, const at::Tensor& c, const at::Tensor& x,
                       const at::Tensor& h, const at::Tensor& W, const at::Tensor& U, const at::Tensor& b,
                       at::Tensor dW, at::Tensor dU, at::Tensor db, bool need_dx,
                       const c10::optional<at::Tensor>& pidx_opt, int64_t pool) {
  const at::Tensor* ops[] = {&dh, &W, &U, &b};
  for (const at::Tensor* t : ops) check_f32_cuda(*t, "lstm_tm_bwd operand");
  const bool rg = g.numel() == 0;
  // x / h in bf16: a recompute-gates pair's layer-A output (TM_RG_BF16H) as layer B's x or layer A's h
  const bool xb = x.scalar_type() == at::kBFloat16, hb = h.scalar_type() == at::kBFloat16;
  if (!xb) check_f32_cuda(x, "lstm_tm_bwd x");
  if (!hb) check_f32_cuda(h, "lstm_tm_bwd h");
  TORCH_CHECK(((!xb && !hb) || rg) && !(xb && hb) && x.is_cuda() && h.is_cuda(),
              "lstm_tm_bwd: bf16 x or h only from a recompute-gates pair forward");
  const float* xptr = reinterpret_cast<const float*>(x.data_ptr());
  const auto fopt = x.options().dtype(at::kFloat);   // (fp32 outputs / workspaces whatever x's dtype)
  const float* hptr = reinterpret_cast<const float*>(h.data_ptr());
  if (!rg) check_gates_cuda(g);
  // (recompute gates: c_t saved in bf16 by the forward, TM_RG_BF16C)
  TORCH_CHECK(c.is_cuda() && c.is_contiguous() &&
                  c.scalar_type() == ((rg && TM_RG_BF16C) ? at::kBFloat16 : at::kFloat),
              "lstm_tm_bwd: c must be the forward's saved state (", (rg && TM_RG_BF16C) ? "bf16" : "fp32", ")");
  const float* cptr = reinterpret_cast<const float*>(c.data_ptr());
  const int T = (int)x.size(0), Mp = (int)x.size(1), Din = (int)x.size(2), H = (int)U.size(0);
  const int Dw = (int)W.size(0);
  TORCH_CHECK(Dw >= 1 && Dw <= Din && W.size(1) == 4 * H && b.numel() == 4 * H, "lstm_tm_bwd: W / b shape");
  const bool last = dh.dim() == 2;
  const bool up = pidx_opt.has_value() && pidx_opt->defined() && pidx_opt->numel() > 0;
  const unsigned char* pidx = nullptr;
  const int P = up ? (int)pool : 1;
  if (up) {
    TORCH_CHECK(!last && P >= 1 && P <= 255 && T / P >= 1, "lstm_tm_bwd: pool size 1..255 <= T, per-step gradient");
    TORCH_CHECK(pidx_opt->is_cuda() && pidx_opt->scalar_type() == at::kByte && pidx_opt->is_contiguous() &&
                    pidx_opt->sizes() == dh.sizes(), "lstm_tm_bwd: pidx must be a contiguous uint8 tensor shaped like dh");
    pidx = pidx_opt->data_ptr<uint8_t>();
  }
  TORCH_CHECK(last ? (dh.size(0) == Mp && dh.size(1) == H)
                   : (dh.size(0) == (up ? T / P : T) && dh.size(1) == Mp && dh.size(2) == H), "lstm_tm_bwd: dh shape");
  TORCH_CHECK(dh.is_contiguous(), "lstm_tm_bwd: dh must be contiguous");
  TORCH_CHECK((rg || g.numel() == (long)(T + 1) * Mp * H * 4) && c.numel() == (long)(T + 1) * Mp * H &&
                  h.numel() == (long)T * Mp * H, "lstm_tm_bwd: saved state shapes");
  const bool wg = dW.numel() > 0;
  if (wg) {
    const at::Tensor* gs[] = {&dW, &dU, &db};
    for (const at::Tensor* t : gs) check_f32_cuda(*t, "lstm_tm_bwd grad");
    TORCH_CHECK(dW.numel() == (long)Dw * 4 * H && dU.numel() == (long)H * 4 * H && db.numel() == 4 * H,
                "lstm_tm_bwd: gradient buffer shapes");
  }
  const int gr = tm_granule(Din, x.data_ptr());
  TORCH_CHECK(tm_supported(H, Din, gr), "lstm_tm_bwd: unsupported shape");
  TORCH_CHECK(!rg || (tm_rg_ok(H, gr) && Din <= 64 && h.is_contiguous() && x.is_contiguous()),
              "lstm_tm_bwd: recomputed gates need H <= 32, Din <= 64, contiguous 16-byte aligned x / h");
  c10::DeviceGuard guard(x.device());
  const int ntiles = Mp / 16;
  auto st = stream();
  const int ncb_w = lstm_grads_col_blocks(H);
  __bf16* gptr = rg ? nullptr : bf16_ptr(g);
  if (wg && (rg || tm_fused_wgrad(H, Din, gr, ntiles))) {
    // weight gradients inside the recurrence: one split record per tile, then the reduction
    const int DT = (Dw + 1 + 15) / 16, RC = (DT + H / 16) * 1024 * ncb_w;
    const int NG = std::max(1, ntiles / 512);
    at::Tensor ws = at::empty({(long)ntiles * RC + (NG > 1 ? (long)NG * RC : 0L)}, fopt);
    at::Tensor dx = need_dx ? at::empty({T + 1, Mp, Din}, fopt) : at::empty({0}, fopt);
    if (need_dx) TORCH_CHECK(tm_granule(Din, dx.data_ptr()) >= gr, "lstm_tm_bwd: dx alignment");
    TORCH_CHECK(reinterpret_cast<uintptr_t>(h.data_ptr()) % 4 == 0 && h.is_contiguous(), "lstm_tm_bwd: h layout");
#define GQ_TM_WG_CALL4(DXV, LASTV, RGV, UPV, XBV, HBV)                                                         \
  hipLaunchKernelGGL((lstm_tm_bwd_wg_kernel<HH, KXX, HH == 16 ? TMW_D16 : TMW_D32, DXV, LASTV, RGV, UPV, XBV, HBV>), \
                     dim3(ntiles), dim3(TMC<HH>::NT), 0, st, dh.data_ptr<float>(), gptr, cptr,                   \
                     W.data_ptr<float>(), U.data_ptr<float>(), need_dx ? dx.data_ptr<float>() : nullptr,         \
                     xptr, hptr, ws.data_ptr<float>(), Mp, T, Din, Dw, b.data_ptr<float>(), pidx, P)
#define GQ_TM_WG_CALL3(DXV, LASTV, RGV, UPV)                                                                   \
  do { if constexpr (RGV) { if (xb) { GQ_TM_WG_CALL4(DXV, LASTV, RGV, UPV, true, false); break; }                \
                            if (hb) { GQ_TM_WG_CALL4(DXV, LASTV, RGV, UPV, false, true); break; } }              \
       GQ_TM_WG_CALL4(DXV, LASTV, RGV, UPV, false, false); } while (0)
#define GQ_TM_WG_CALL2(DXV, LASTV, RGV)                                                                        \
  do { if constexpr (!LASTV) { if (up) { GQ_TM_WG_CALL3(DXV, LASTV, RGV, true); break; } }                      \
       GQ_TM_WG_CALL3(DXV, LASTV, RGV, false); } while (0)
#define GQ_TM_WG_CALL(DXV, LASTV) \
  do { if (rg) GQ_TM_WG_CALL2(DXV, LASTV, true); else GQ_TM_WG_CALL2(DXV, LASTV, false); } while (0)
#define GQ_TM_WG_KX(...)                                                                                        \
  if ((Din + 31) / 32 == 1) { constexpr int KXX = 1; __VA_ARGS__; }                                             \
  else { constexpr int KXX = 2; __VA_ARGS__; }
    switch (H) {
      case 16: { constexpr int HH = 16;
        GQ_TM_WG_KX(if (need_dx) { if (last) GQ_TM_WG_CALL(true, true); else GQ_TM_WG_CALL(true, false); }
                    else { if (last) GQ_TM_WG_CALL(false, true); else GQ_TM_WG_CALL(false, false); }) break; }
      default: { constexpr int HH = 32;
        GQ_TM_WG_KX(if (need_dx) { if (last) GQ_TM_WG_CALL(true, true); else GQ_TM_WG_CALL(true, false); }
                    else { if (last) GQ_TM_WG_CALL(false, true); else GQ_TM_WG_CALL(false, false); }) break; }
    }
#undef GQ_TM_WG_KX
#undef GQ_TM_WG_CALL
#undef GQ_TM_WG_CALL2
#undef GQ_TM_WG_CALL3
#undef GQ_TM_WG_CALL4
    GQ_LAUNCH_CHECK();
    lstm_grads_reduce_records(ws, H, Dw, ntiles, dW.data_ptr<float>(), dU.data_ptr<float>(), db.data_ptr<float>(), st);
    return need_dx ? dx.narrow(0, 0, T) : dx;
  }
  TORCH_CHECK(!rg || !wg, "lstm_tm_bwd: recomputed gates with weight gradients take the fused kernel");
  if (wg && need_dx && ncb_w > 1 && tm_rec_dx()) {
    // several gate-column blocks: the weight-gradient pass could only produce dx as ncb partial
    // slabs plus a slab sum (ncb + 2 dx-sized passes); the recurrence computes dx^T = W dz^T
    // itself instead (its MFMA phase has the whole 4H dz tile in LDS) and writes dx once.
    at::Tensor dz = at::empty({T + 1, Mp, 4 * H}, fopt.dtype(at::kBFloat16));
    at::Tensor dx = at::empty({T + 1, Mp, Din}, fopt);
    TORCH_CHECK(tm_granule(Din, dx.data_ptr()) >= gr, "lstm_tm_bwd: dx alignment");
#define GQ_TM_BWD_CALL2(LASTV)                                                                              \
  tm_bwd_cfg<HH, KXX, GRR, true, true, LASTV>(ntiles, dh.data_ptr<float>(), bf16_ptr(g), c.data_ptr<float>(), \
                                              W.data_ptr<float>(), U.data_ptr<float>(), dx.data_ptr<float>(),  \
                                              bf16_ptr(dz), Mp, T, Din, Dw, st, pidx, P)
    GQ_TM_H_DISPATCH(H, GQ_TM_KX_DISPATCH((Din + 31) / 32, GQ_TM_GR_DISPATCH(gr,
        if (last) GQ_TM_BWD_CALL2(true); else GQ_TM_BWD_CALL2(false))));
#undef GQ_TM_BWD_CALL2
    GQ_LAUNCH_CHECK();
    const long rows = (long)T * Mp;
    lstm_grads_rows(dz.data_ptr(), 1, x.data_ptr<float>(), h.data_ptr<float>(), W.data_ptr<float>(), nullptr,
                    dW.data_ptr<float>(), dU.data_ptr<float>(), db.data_ptr<float>(), rows, rows, Mp, H, Dw, Din,
                    rows * Din, Din, rows * Din, st);
    return dx.narrow(0, 0, T);
  }
  if (wg) {
    // recurrence -> dz (bf16), then dW/dU/db (+ dx) in one pass over T*Mp rows. (A pooled gradient
    // is un-pooled to full resolution first: this path's recurrence is instantiated without UP.)
    const at::Tensor dhf = up ? maxpool1d_bwd(dh.view({1, T / P, (long)Mp * H}), pidx_opt->view({1, T / P, (long)Mp * H}),
                                              T, P).view({T, Mp, H})
                              : dh;
    at::Tensor dz = at::empty({T + 1, Mp, 4 * H}, fopt.dtype(at::kBFloat16));
    GQ_TM_H_DISPATCH(H,
        if (last) tm_bwd_cfg<HH, 1, 1, true, false, true>(ntiles, dhf.data_ptr<float>(), bf16_ptr(g),
              c.data_ptr<float>(), W.data_ptr<float>(), U.data_ptr<float>(), nullptr, bf16_ptr(dz), Mp, T, Din, Dw, st);
        else tm_bwd_cfg<HH, 1, 1, true, false, false>(ntiles, dhf.data_ptr<float>(), bf16_ptr(g),
              c.data_ptr<float>(), W.data_ptr<float>(), U.data_ptr<float>(), nullptr, bf16_ptr(dz), Mp, T, Din, Dw, st));
    GQ_LAUNCH_CHECK();
    const long rows = (long)T * Mp;
    const int ncb = lstm_grads_col_blocks(H);
    // dx keeps the x layout (Din channels); padding channels (>= Dw) get zero gradient
    at::Tensor dx = need_dx ? at::empty({ncb, T, Mp, Din}, fopt) : at::empty({0}, fopt);
    lstm_grads_rows(dz.data_ptr(), 1, x.data_ptr<float>(), h.data_ptr<float>(), W.data_ptr<float>(),
                    need_dx ? dx.data_ptr<float>() : nullptr, dW.data_ptr<float>(), dU.data_ptr<float>(),
                    db.data_ptr<float>(), rows, rows, Mp, H, Dw, Din, rows * Din, Din, rows * Din, st);
    if (!need_dx) return dx;
    return ncb == 1 ? dx[0] : dx.sum(0);
  }
  at::Tensor dx = at::empty({T + 1, Mp, Din}, fopt);
  TORCH_CHECK(tm_granule(Din, dx.data_ptr()) >= gr, "lstm_tm_bwd: dx alignment");
  if (rg) {      // frozen weights (integrated gradients), gates recomputed: H <= 32, GR = 4
#define GQ_TM_RG_CALL3(LASTV, UPV, XBV, HBV)                                                                   \
  hipLaunchKernelGGL((lstm_tm_bwd_kernel<HH, KXX, 4, 4, false, true, LASTV, true, UPV, XBV, HBV>), dim3(ntiles),  \
                     dim3(TMC<HH>::NT), 0, st, dh.data_ptr<float>(), nullptr, cptr,                                \
                     W.data_ptr<float>(), U.data_ptr<float>(), dx.data_ptr<float>(), nullptr, Mp, T, Din, Dw,     \
                     xptr, hptr, b.data_ptr<float>(), pidx, P)
#define GQ_TM_RG_CALL2(LASTV, UPV)                                                                             \
  do { if (xb) { GQ_TM_RG_CALL3(LASTV, UPV, true, false); break; }                                             \
       if (hb) { GQ_TM_RG_CALL3(LASTV, UPV, false, true); break; }                                             \
       GQ_TM_RG_CALL3(LASTV, UPV, false, false); } while (0)
#define GQ_TM_RG_CALL(LASTV) \
  do { if constexpr (!LASTV) { if (up) { GQ_TM_RG_CALL2(LASTV, true); break; } } GQ_TM_RG_CALL2(LASTV, false); } while (0)
    GQ_TM2_H_DISPATCH(H, if ((Din + 31) / 32 == 1) { constexpr int KXX = 1; if (last) GQ_TM_RG_CALL(true); else GQ_TM_RG_CALL(false); }
                         else { constexpr int KXX = 2; if (last) GQ_TM_RG_CALL(true); else GQ_TM_RG_CALL(false); });
#undef GQ_TM_RG_CALL
#undef GQ_TM_RG_CALL2
#undef GQ_TM_RG_CALL3
    GQ_LAUNCH_CHECK();
    return dx.narrow(0, 0, T);
  }
#define GQ_TM_BWD_CALL(LASTV)                                                                               \
  tm_bwd_cfg<HH, KXX, GRR, false, true, LASTV>(ntiles, dh.data_ptr<float>(), gptr,                 \
                                               c.data_ptr<float>(), W.data_ptr<float>(), U.data_ptr<float>(), \
                                               dx.data_ptr<float>(), nullptr, Mp, T, Din, Dw, st, pidx, P)
  GQ_TM_H_DISPATCH(H, GQ_TM_KX_DISPATCH((Din + 31) / 32, GQ_TM_GR_DISPATCH(gr,
      if (last) GQ_TM_BWD_CALL(true); else GQ_TM_BWD_CALL(false))));
#undef GQ_TM_BWD_CALL
  GQ_LAUNCH_CHECK();
  return dx.narrow(0, 0, T);
}

}  // namespace gq

TORCH_LIBRARY_IMPL(gnnqc, CUDA, m) {
  m.impl("lstm_tm_fwd", &gq::lstm_tm_fwd);
  m.impl("lstm_tm2_fwd", &gq::lstm_tm2_fwd);
  m.impl("lstm_tm_grads", &gq::lstm_tm_grads);
  m.impl("lstm_tm_bwd_pipe", &gq::lstm_tm_bwd_pipe);
  m.impl("lstm_grads_job_ws", &gq::lstm_grads_job_ws);
  m.impl("lstm_grads_multi", &gq::lstm_grads_multi);
  m.impl("lstm_tm_bwd", &gq::lstm_tm_bwd);
}
