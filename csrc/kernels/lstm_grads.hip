// Fused LSTM weight / input gradients for gfx950 (backward).
//
// After the BPTT kernel has produced dz = dL/dz_t for every (sequence, step) row,
// all remaining LSTM gradients are contractions over those rows:
//   dW = x^T dz   [Din, 4H]      dU = h_{t-1}^T dz  [H, 4H]      db = 1^T dz  [4H]
//   dx = dz W^T   [rows, Din]
// hipBLASLt runs the first three as K = B*T (~23k CML, ~2.3M SoilNet) skinny GEMMs with
// poor tile choices; here ONE kernel streams each 32-row tile of (dz, x, h_{t-1}) through
// LDS once and feeds all four products to v_mfma_f32_16x16x32_bf16:
//   * grid = (gate-unit column blocks of 64) x (row splits); a workgroup keeps its
//     dW^T / dU^T / db partial tiles in registers across all its row tiles, writes them
//     once to a workspace, and a reduce kernel adds the split sums to the gradient
//     buffers (these can be the optimiser's flat gradient views: no AccumulateGrad pass);
//   * db rides along as an extra constant-1 input channel of x (row Din of dW^T);
//   * dx^T = W dz^T uses W as register-resident A fragments; with one column
//     block (H <= 16) dx is stored directly, otherwise accumulated atomically.
#include "common.h"
#include "lstm_grads_body.h"

#include <cstdlib>
#include <type_traits>

namespace gq {

int* chain_ctl(int dev);   // lstm_chain.hip: the device's chain control words

std::vector<DeferredRed>& deferred_reds() {
  static std::vector<DeferredRed> v;
  return v;
}

template <int H, int DT, int GRX, typename ZT>
__global__ __launch_bounds__(256) void lstm_grads_kernel(
    const void* __restrict__ dz, const float* __restrict__ x, const float* __restrict__ hseq,
    const float* __restrict__ W, float* __restrict__ dx, float* __restrict__ ws, long rows, long period,
    long hshift, int Din, int ldx, long dx_cb_stride, int lddx, int xg, long x_elems) {
  __shared__ __attribute__((aligned(16))) char smem[GradsLds<H, DT>::BYTES];
  // the column blocks of a row split share its x / h_{t-1} tiles: keep them on one XCD
#ifndef GQ_GRADS_NO_XCD
  const int v = xcd_group_remap(blockIdx.x + gridDim.x * blockIdx.y, gridDim.x * gridDim.y, gridDim.x);
#else
  const int v = blockIdx.x + gridDim.x * blockIdx.y;      // (A/B: dispatch order)
#endif
  lstm_grads_body<H, DT, GRX, false, ZT>(dz, x, hseq, W, dx, ws, rows, period, hshift, Din, ldx, dx_cb_stride, lddx,
                                         xg, x_elems, v % gridDim.x, v / gridDim.x, gridDim.x, gridDim.y, smem);
}

__global__ __launch_bounds__(256) void lstm_grads_reduce_kernel(const float* __restrict__ ws, int splits, int RC,
                                                                float* __restrict__ ws2, int ncb, int DT, int HT,
                                                                int Din, int H, float* __restrict__ dW,
                                                                float* __restrict__ db, float* __restrict__ dU,
                                                                int* nf) {
  lstm_grads_reduce_body(ws, splits, RC, ws2, ncb, DT, HT, Din, H, dW, db, dU, blockIdx.x, blockIdx.y, gridDim.y, nf);
}

__global__ __launch_bounds__(256) void lstm_grads_reduce_final_kernel(const float* __restrict__ ws2, int NG, int RC,
                                                                      int ncb, int DT, int HT, int Din, int H,
                                                                      float* __restrict__ dW, float* __restrict__ db,
                                                                      float* __restrict__ dU, int* nf) {
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < RC; e += gridDim.x * blockDim.x) {
    float s = 0.f;
    for (int g = 0; g < NG; ++g) s += ws2[(size_t)g * RC + e];
    grads_add(s, e, ncb, DT, HT, Din, H, dW, db, dU, nf);
  }
}

template <int H, typename ZT>
void launch_grads_h(int DT, int grx, dim3 grid, hipStream_t st, const void* dz, const float* x, const float* h,
                    const float* W, float* dx, float* ws, long rows, long period, long hshift, int Din, int ldx,
                    long dx_cb_stride, int lddx, int xg, long x_elems) {
  switch (DT) {
#define GQ_DT(D)                                                                                              \
  case D:                                                                                                     \
    if (grx == 4)                                                                                             \
      hipLaunchKernelGGL((lstm_grads_kernel<H, D, 4, ZT>), grid, dim3(256), 0, st, dz, x, h, W, dx, ws, rows, \
                         period, hshift, Din, ldx, dx_cb_stride, lddx, xg, x_elems);                          \
    else                                                                                                      \
      hipLaunchKernelGGL((lstm_grads_kernel<H, D, 1, ZT>), grid, dim3(256), 0, st, dz, x, h, W, dx, ws, rows, \
                         period, hshift, Din, ldx, dx_cb_stride, lddx, xg, x_elems);                          \
    break;
    GQ_DT(1) GQ_DT(2) GQ_DT(3) GQ_DT(4) GQ_DT(5) GQ_DT(6) GQ_DT(7) GQ_DT(8) GQ_DT(9)
#undef GQ_DT
    default:
      TORCH_CHECK(false, "gnnqc lstm_grads: input width ", Din, " too large (max 143)");
  }
}

void lstm_grads_reduce_records(const at::Tensor& ws_t, int H, int Din, int splits, float* dW, float* dU, float* db,
                               hipStream_t st);

// Flat-row launcher shared by the sequence-major (lstm_grads) and time-major (lstm_tm_bwd)
// paths: row r of dz / x / dx has h_{t-1} at row r - hshift when r % period >= hshift.
// x rows have pitch ldx, dx rows pitch lddx; only the first Din (= rows of W) channels are used.
//   sequence-major [M,T,C]: period = T, hshift = 1;  time-major [T,Mp,C]: period = T*Mp, hshift = Mp.
void lstm_grads_rows(const void* dz, int zbf, const float* x, const float* hseq, const float* W, float* dx,
                     float* dW, float* dU, float* db, long rows, long period, long hshift, int H, int Din, int ldx,
                     long dx_cb_stride, int lddx, long x_elems, hipStream_t st) {
  if (rows == 0) return;
  TORCH_CHECK(ldx >= Din && ldx <= 144, "gnnqc lstm_grads: x row pitch ", ldx, " (Din ", Din, ")");
  const int ncb = (4 * H) / GR_CB;
  const long ntiles = (rows + GR_ROWS - 1) / GR_ROWS;
  // ~2 tiles per workgroup for small row counts (latency: everything in flight at once),
  // ~2 workgroups per CU for large ones: each split writes a (DT + HT) x 4H record that the
  // reduction reads back, so more splits cost record traffic (SoilNet, 8.5k sequences x 12-37
  // steps: budget 2048 / 1024 / 512 / 256 -> 2.986 / 2.950 / 2.919 / 3.060 ms per step,
  // profiles/r6_grads_budget_ab.txt). The split count depends only on the shape and the reduce
  // kernel sums in a fixed order: bitwise reproducible in every mode.
  static const int wg_budget = [] {            // workgroups per pass (A/B: GNNQC_GRADS_WG)
    const char* e = std::getenv("GNNQC_GRADS_WG");
    return e != nullptr ? std::max(256, std::atoi(e)) : 512;
  }();
  const int splits = (int)std::max<long>(1, std::min<long>((ntiles + 1) / 2, std::max(64, wg_budget / ncb)));
  const int DT = (Din + 1 + 15) / 16;
  const int HT = H / 16;
  const int grx = (ldx % 4 == 0 && reinterpret_cast<uintptr_t>(x) % 16 == 0) ? 4 : 1;
  const int xg = (int)((GR_ROWS * (long)ldx / grx + 255) / 256);
  const int RC = (DT + HT) * 1024 * ncb;          // floats per split record (all column blocks)
  const int NG = std::max(1, splits / 512);       // split groups of the reduction
  auto ws_t = at::empty({(long)splits * RC + (NG > 1 ? (long)NG * RC : 0L)},
                        at::TensorOptions().dtype(at::kFloat).device(at::kCUDA, c10::hip::current_device()));
  float* ws = ws_t.data_ptr<float>();
  float* ws2 = ws + (size_t)splits * RC;
  dim3 grid(ncb, splits);
#define GQ_GR_H(HH)                                                                                              \
  case HH:                                                                                                       \
    if (zbf)                                                                                                     \
      launch_grads_h<HH, __bf16>(DT, grx, grid, st, dz, x, hseq, W, dx, ws, rows, period, hshift, Din, ldx,      \
                                 dx_cb_stride, lddx, xg, x_elems);                                               \
    else                                                                                                         \
      launch_grads_h<HH, float>(DT, grx, grid, st, dz, x, hseq, W, dx, ws, rows, period, hshift, Din, ldx,       \
                                dx_cb_stride, lddx, xg, x_elems);                                                \
    break;
  switch (H) {
    GQ_GR_H(16) GQ_GR_H(32) GQ_GR_H(64) GQ_GR_H(128)
    default: TORCH_CHECK(false, "gnnqc lstm_grads: unsupported hidden size ", H);
  }
#undef GQ_GR_H
  GQ_LAUNCH_CHECK();
  lstm_grads_reduce_records(ws_t, H, Din, splits, dW, dU, db, st);
}

// Sum `splits` split records ([split][cb][DT + HT][4][64][4] floats, ws_t also holding the NG group
// sums past them when splits > 512) into dW / dU / db: deferred to lstm_reduce_flush in deferred
// mode, else one reduce launch (+ the group-sum launch).
void lstm_grads_reduce_records(const at::Tensor& ws_t, int H, int Din, int splits, float* dW, float* dU, float* db,
                               hipStream_t st) {
  const int ncb = (4 * H) / GR_CB;
  const int DT = (Din + 1 + 15) / 16;
  const int HT = H / 16;
  const int RC = (DT + HT) * 1024 * ncb;
  const int NG = std::max(1, splits / 512);
  TORCH_CHECK(ws_t.numel() >= (long)splits * RC + (NG > 1 ? (long)NG * RC : 0L), "lstm_grads: split records");
  if (defer_reduce_mode()) {                      // summed by lstm_reduce_flush with the other layers'
    deferred_reds().push_back(DeferredRed{ws_t, H, Din, splits, dW, dU, db});
    return;
  }
  float* ws = ws_t.data_ptr<float>();
  float* ws2 = ws + (size_t)splits * RC;
  // every weight-gradient reduction raises the non-finite flag (chain control word 7) that the
  // flag-driven Adam (adam_flagged) decides from
  int* nf = chain_ctl(c10::hip::current_device()) + 7;
  hipLaunchKernelGGL(lstm_grads_reduce_kernel, dim3((RC + 15) / 16, NG), dim3(256), 0, st, ws, splits, RC, ws2, ncb,
                     DT, HT, Din, H, dW, db, dU, nf);
  GQ_LAUNCH_CHECK();
  if (NG > 1) {
    hipLaunchKernelGGL(lstm_grads_reduce_final_kernel, dim3(std::min((RC + 255) / 256, 1024)), dim3(256), 0, st, ws2,
                       NG, RC, ncb, DT, HT, Din, H, dW, db, dU, nf);
    GQ_LAUNCH_CHECK();
  }
}

// ---------------------------------------------------------------------------------------
// dx = dz W^T on its own (no LDS): for a 16-row tile and a 16-wide din tile, the MFMA B
// operand (rows x gate-units, K-contiguous per lane) is 8 consecutive floats of one dz row
// and the A operand (din x gate-units) 8 consecutive floats of one W row, so both come
// straight from global memory / registers; the C tile's 4 consecutive din values per lane
// leave as one float4. All 4H gate-units are contracted in one workgroup: no per-column-
// block slabs and no slab sum. Used when the weight-gradient pass runs on a side stream
// (off the critical path) while this kernel feeds the next layer's recurrence.
template <int H, int RW, int NDT, typename ZT>   // RW: waves sharing one 16-row tile; NDT: din tiles per wave
__global__ __launch_bounds__(256) void lstm_dx_kernel(const void* __restrict__ dzv, const float* __restrict__ W,
                                                      float* __restrict__ dx, long rows, int Dw, int lddx) {
  const ZT* __restrict__ dz = reinterpret_cast<const ZT*>(dzv);
  constexpr int G4 = 4 * H, KS = G4 / 32, TPB = 4 / RW;     // row tiles per workgroup pass
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int col = lane & 15, quad = lane >> 4;
  const int wr = w / RW, wd = w % RW;                       // row-tile slot, din-tile phase
  bf16x8_t wa[NDT][KS];
#pragma unroll
  for (int d = 0; d < NDT; ++d) {
    const int din = 16 * (wd + RW * d) + col;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const float4 a = *reinterpret_cast<const float4*>(W + (size_t)min(din, Dw - 1) * G4 + 32 * ks + 8 * quad);
      const float4 b = *reinterpret_cast<const float4*>(W + (size_t)min(din, Dw - 1) * G4 + 32 * ks + 8 * quad + 4);
      const float m = din < Dw ? 1.f : 0.f;
      wa[d][ks] = bf16x8_t{(__bf16)(a.x * m), (__bf16)(a.y * m), (__bf16)(a.z * m), (__bf16)(a.w * m),
                           (__bf16)(b.x * m), (__bf16)(b.y * m), (__bf16)(b.z * m), (__bf16)(b.w * m)};
    }
  }
  const long ntiles = (rows + 15) / 16;
  for (long t = (long)blockIdx.x * TPB + wr; t < ntiles; t += (long)gridDim.x * TPB) {
    const long r = t * 16 + col;
    const long rc = min(r, rows - 1);
    bf16x8_t bz[KS];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      if constexpr (std::is_same<ZT, __bf16>::value) {
        bz[ks] = *reinterpret_cast<const bf16x8_t*>(dz + (size_t)rc * G4 + 32 * ks + 8 * quad);
      } else {
        const float4 a = *reinterpret_cast<const float4*>(dz + (size_t)rc * G4 + 32 * ks + 8 * quad);
        const float4 b = *reinterpret_cast<const float4*>(dz + (size_t)rc * G4 + 32 * ks + 8 * quad + 4);
        bz[ks] = bf16x8_t{(__bf16)a.x, (__bf16)a.y, (__bf16)a.z, (__bf16)a.w,
                          (__bf16)b.x, (__bf16)b.y, (__bf16)b.z, (__bf16)b.w};
      }
    }
#pragma unroll
    for (int d = 0; d < NDT; ++d) {
      const int din0 = 16 * (wd + RW * d) + 4 * quad;
      f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[d][ks], bz[ks], acc, 0, 0, 0);
      // lane holds dx[r][din0 .. din0+3]; columns Dw .. lddx-1 (layout padding) get zeros
      if (r < rows && din0 < lddx) {
        float* o = dx + (size_t)r * lddx + din0;
        if (din0 + 4 <= lddx) {
          *reinterpret_cast<float4*>(o) = make_float4(acc[0], acc[1], acc[2], acc[3]);
        } else {
          for (int q = 0; q < lddx - din0; ++q) o[q] = acc[q];
        }
      }
    }
  }
}

// dz: [>= rows, 4H] fp32 (or bf16: zbf) rows; W: [Dw, 4H]; out: [rows, lddx] (lddx >= Dw, multiple of 4).
// Narrow inputs (1-2 din tiles) give each wave its own row tile instead of a din tile that
// is then thrown away: no redundant dz loads, 2-4 row tiles per workgroup pass.
void lstm_dx_rows(const void* dz, int zbf, const float* W, float* dx, long rows, int H, int Dw, int lddx,
                  hipStream_t st) {
  if (rows == 0) return;
  const int ndin = (lddx + 15) / 16;
  TORCH_CHECK(ndin <= 8, "lstm_dx: input width ", lddx, " > 128");
  const int rw = ndin >= 3 ? 4 : ndin;
  const int ndt = (ndin + rw - 1) / rw;
  const long ngroups = ((rows + 15) / 16 + (4 / rw) - 1) / (4 / rw);
  // every wave converts its W fragments (KS x 2 float4 rows per din tile: 32 KB per wave at H = 128)
  // once and then walks row tiles: wide layers cap the grid so that setup is amortised over several
  // tiles (at one tile per wave, H = 128 re-read ~640 MB of W through L2 on the SoilNet step)
  const long cap = H >= 128 ? 1024 : (H >= 64 ? 2048 : 8192);
  const int grid = (int)std::max<long>(1, std::min<long>(ngroups, cap));
#define GQ_DX(HH, RWV, ND)                                                                                          \
  do {                                                                                                              \
    if (zbf) hipLaunchKernelGGL((lstm_dx_kernel<HH, RWV, ND, __bf16>), dim3(grid), dim3(256), 0, st, dz, W, dx,     \
                                rows, Dw, lddx);                                                                    \
    else hipLaunchKernelGGL((lstm_dx_kernel<HH, RWV, ND, float>), dim3(grid), dim3(256), 0, st, dz, W, dx, rows,    \
                            Dw, lddx);                                                                              \
  } while (0)
#define GQ_DX_H(HH)                                                                            \
  case HH:                                                                                     \
    if (rw == 1) GQ_DX(HH, 1, 1); else if (rw == 2) GQ_DX(HH, 2, 1);                           \
    else if (ndt == 1) GQ_DX(HH, 4, 1); else GQ_DX(HH, 4, 2);                                  \
    break;
  switch (H) {
    GQ_DX_H(16) GQ_DX_H(32) GQ_DX_H(64) GQ_DX_H(128)
    default: TORCH_CHECK(false, "lstm_dx: unsupported hidden size ", H);
  }
#undef GQ_DX_H
#undef GQ_DX
  GQ_LAUNCH_CHECK();
}

// dx = dz[:rows] W^T into a fresh [rows / lead, lead, lddx] tensor (shape taken from `like`).
at::Tensor lstm_dx(const at::Tensor& dz, const at::Tensor& W, const at::Tensor& like) {
  check_dz_cuda(dz);
  check_f32_cuda(W, "W");
  const int G4 = (int)W.size(1), H = G4 / 4, Dw = (int)W.size(0);
  TORCH_CHECK(dz.size(-1) == G4, "lstm_dx: dz / W gate widths differ");
  const int lddx = (int)like.size(-1);
  TORCH_CHECK(lddx >= Dw && lddx % 4 == 0, "lstm_dx: output width must be >= W rows and a multiple of 4");
  const long rows = like.numel() / lddx;
  TORCH_CHECK(dz.numel() / G4 >= rows, "lstm_dx: dz has too few rows");
  c10::DeviceGuard guard(dz.device());
  at::Tensor dx = at::empty(like.sizes(), like.options().dtype(at::kFloat));
  lstm_dx_rows(dz.data_ptr(), dz_bf16(dz), W.data_ptr<float>(), dx.data_ptr<float>(), rows, H, Dw, lddx, stream());
  return dx;
}

int lstm_grads_col_blocks(int H) { return (4 * H) / GR_CB; }

// (A one-pass dx = dz W^T over all 4H gate-units instead of ncb slabs + their sum was measured
// slower on the SoilNet step - 5.016 vs 4.944 ms - and removed; the time-major layers now take dx
// from their recurrence instead, lstm_tm.hip tm_rec_dx.)

// dz [M(p),T,4H] from lstm_bwd; x [M,T,Din] (unit inner stride, row stride ldx);
// hseq [M,T,H]; W [Din,4H]. dW/dU/db are ACCUMULATED into (pass zeroed or existing
// gradient buffers). Returns dx [M,T,Din] if need_dx (else an empty tensor).
at::Tensor lstm_grads(const at::Tensor& dz, const at::Tensor& x, const at::Tensor& hseq, const at::Tensor& W,
                      at::Tensor dW, at::Tensor dU, at::Tensor db, bool need_dx) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kFloat && x.dim() == 3 && x.stride(2) == 1 &&
                  x.stride(0) == x.size(1) * x.stride(1), "x must be [M,T,Din] float32 with unit inner stride");
  check_f32_cuda(hseq, "hseq");
  check_f32_cuda(W, "W");
  check_f32_cuda(dW, "dW");
  check_f32_cuda(dU, "dU");
  check_f32_cuda(db, "db");
  check_dz_cuda(dz);
  TORCH_CHECK(dz.stride(2) == 1 && dz.stride(1) == dz.size(2) &&
                  dz.stride(0) == dz.size(1) * dz.size(2), "dz must be a contiguous [M,T,4H] row block");
  const int M = x.size(0), T = x.size(1), Din = x.size(2), H = hseq.size(2);
  TORCH_CHECK(dz.size(0) == M && dz.size(1) == T && dz.size(2) == 4 * H, "dz shape");
  TORCH_CHECK(hseq.size(0) == M && hseq.size(1) == T, "hseq shape");
  TORCH_CHECK(W.size(0) == Din && W.size(1) == 4 * H && dW.sizes() == W.sizes() && dU.size(0) == H &&
                  dU.size(1) == 4 * H && db.numel() == 4 * H, "gradient buffer shapes");
  TORCH_CHECK(Din + 1 <= 9 * 16, "gnnqc lstm_grads: input width ", Din, " too large (max 143)");
  c10::DeviceGuard guard(x.device());
  const int ncb = lstm_grads_col_blocks(H);
  // dx = dz W^T contracts over all 4H gate-units: with a few column blocks each block writes its
  // partial product to its own slab (plain stores), summed below; with 4+ (H >= 64) the slabs
  // would cost ncb + 2 dx-sized passes, so one lstm_dx pass over dz produces dx instead
  const bool onepass = need_dx && ncb >= 4 && Din % 4 == 0 && Din <= 128;
  at::Tensor dx = need_dx ? at::empty({onepass ? 1 : ncb, M, T, Din}, x.options()) : at::empty({0}, x.options());
  const long rows = (long)M * T;
  if (rows == 0) return need_dx ? dx.sum(0) : dx;
  lstm_grads_rows(dz.data_ptr(), dz_bf16(dz), x.data_ptr<float>(), hseq.data_ptr<float>(), W.data_ptr<float>(),
                  (need_dx && !onepass) ? dx.data_ptr<float>() : nullptr, dW.data_ptr<float>(), dU.data_ptr<float>(),
                  db.data_ptr<float>(), rows, T, 1, H, Din, x.stride(1), rows * Din, Din,
                  (long)(x.storage().nbytes() / sizeof(float)) - x.storage_offset(), stream());
  if (!need_dx) return dx;
  if (onepass) {
    lstm_dx_rows(dz.data_ptr(), dz_bf16(dz), W.data_ptr<float>(), dx.data_ptr<float>(), rows, H, Din, Din, stream());
    return dx[0];
  }
  return ncb == 1 ? dx[0] : dx.sum(0);
}

}  // namespace gq

TORCH_LIBRARY_IMPL(gnnqc, CUDA, m) {
  m.impl("lstm_grads", &gq::lstm_grads);
  m.impl("lstm_dx", &gq::lstm_dx);
}
