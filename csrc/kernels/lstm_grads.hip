// Fused LSTM weight / input gradients for gfx950 (backward).
//
// After the BPTT kernel has produced dz = dL/dz_t for every (sequence, step) row,
// all remaining LSTM gradients are contractions over those rows:
//   dW = x^T dz   [Din, 4H]      dU = h_{t-1}^T dz  [H, 4H]      db = 1^T dz  [4H]
//   dx = dz W^T   [rows, Din]
// hipBLASLt runs the first three as K = B*T (~23k) skinny GEMMs with poor tile
// choices; here ONE kernel streams each 32-row tile of (dz, x, h_{t-1}) through
// LDS once and feeds all four products to v_mfma_f32_16x16x32_bf16:
//   * grid = (gate-unit column blocks of 64) x (row splits); a workgroup keeps its
//     dW^T / dU^T / db partial tiles in registers across all its row tiles and adds
//     them to the gradient buffers with one fp32 atomic per element at the end
//     (these can be the optimiser's flat gradient views: no AccumulateGrad pass);
//   * db rides along as an extra constant-1 input channel of x (row Din of dW^T);
//   * dx^T = W dz^T uses W as register-resident A fragments; with one column
//     block (H <= 16) dx is stored directly, otherwise accumulated atomically.
#include "common.h"

namespace gq {

constexpr int GR_ROWS = 32;         // rows (sequence, step) per tile = MFMA K
constexpr int GR_CB = 64;           // gate-units per column block (4 waves x 16)
constexpr int GR_LDR = GR_ROWS + 8; // padded LDS row length (bf16) of transposed images

template <int H, int DT>            // DT = ceil((Din + 1) / 16) din tiles (incl. the bias channel)
__global__ __launch_bounds__(256) void lstm_grads_kernel(
    const float* __restrict__ dz, const float* __restrict__ x, const float* __restrict__ hseq,
    const float* __restrict__ W, float* __restrict__ dx, float* __restrict__ dW, float* __restrict__ dU,
    float* __restrict__ db, long rows, long period, long hshift, int Din, int ldx, long dx_cb_stride, int lddx) {
  constexpr int G4 = 4 * H;
  constexpr int HT = H / 16;        // k tiles of dU
  constexpr int DP = DT * 16;       // padded din (incl. bias channel)
  __shared__ __attribute__((aligned(16))) __bf16 dzT[GR_CB][GR_LDR];          // [gu][row]
  __shared__ __attribute__((aligned(16))) __bf16 dzR[GR_ROWS][GR_CB + 8];     // [row][gu]
  __shared__ __attribute__((aligned(16))) __bf16 xT[DP][GR_LDR];             // [din][row]
  __shared__ __attribute__((aligned(16))) __bf16 hT[H][GR_LDR];              // [k][row]

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int w = tid >> 6;
  const int col = lane & 15;
  const int quad = lane >> 4;
  const int cb = blockIdx.x;               // column block: gate-units [cb*64, cb*64+64)
  const int gu0 = cb * GR_CB;
  const long ntiles = (rows + GR_ROWS - 1) / GR_ROWS;

  f32x4_t accW[DT], accU[HT];
#pragma unroll
  for (int d = 0; d < DT; ++d) accW[d] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int k = 0; k < HT; ++k) accU[k] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  // dx work items of this wave: (din tile, row tile) pairs, 2 row tiles per 32 rows
  constexpr int DXT = (DP + 15) / 16 * 2;
  // A fragments of W for dx^T = W dz^T: rows = din, k = gate-units of this block
  bf16x8_t wa[(DXT + 3) / 4][2];
#pragma unroll
  for (int i = 0; i < (DXT + 3) / 4; ++i) {
    const int item = w + 4 * i;
    const int dtile = item >> 1;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8_t v;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int din = dtile * 16 + col;
        const int gu = gu0 + 32 * ks + 8 * quad + j;
        v[j] = (__bf16)(W[(size_t)min(din, Din - 1) * G4 + gu] * ((item < DXT && din < Din) ? 1.f : 0.f));
      }
      wa[i][ks] = v;
    }
  }

  for (long tile = blockIdx.y; tile < ntiles; tile += gridDim.y) {
    const long r0 = tile * GR_ROWS;
    // ---- stage dz (both orientations), x^T (+ ones channel) and h_{t-1}^T as bf16
    for (int e = tid; e < GR_ROWS * (GR_CB / 4); e += 256) {
      const int rr = e / (GR_CB / 4);
      const int c4 = (e % (GR_CB / 4)) * 4;
      const long r = min(r0 + rr, rows - 1);
      float4 v = *reinterpret_cast<const float4*>(dz + (size_t)r * G4 + gu0 + c4);
      const float m = (r0 + rr < rows) ? 1.f : 0.f;
      const __bf16 b0 = (__bf16)(v.x * m), b1 = (__bf16)(v.y * m), b2 = (__bf16)(v.z * m), b3 = (__bf16)(v.w * m);
      typedef __bf16 bf16x4_t __attribute__((ext_vector_type(4)));
      *reinterpret_cast<bf16x4_t*>(&dzR[rr][c4]) = bf16x4_t{b0, b1, b2, b3};
      dzT[c4 + 0][rr] = b0;
      dzT[c4 + 1][rr] = b1;
      dzT[c4 + 2][rr] = b2;
      dzT[c4 + 3][rr] = b3;
    }
    for (int e = tid; e < GR_ROWS * DP; e += 256) {
      const int rr = e / DP;
      const int d = e % DP;
      const long r = r0 + rr;
      const bool ok = r < rows;
      const long rc = min(r, rows - 1);
      float v = x[(size_t)rc * ldx + min(d, Din - 1)];
      v = d < Din ? v : (d == Din ? 1.f : 0.f);
      xT[d][rr] = (__bf16)(ok ? v : 0.f);
    }
    for (int e = tid; e < GR_ROWS * H; e += 256) {
      const int rr = e / H;
      const int k = e % H;
      const long r = r0 + rr;
      const long rc = min(r, rows - 1);
      const float v = hseq[(size_t)max(rc - hshift, 0L) * H + k];   // h_{t-1}: hshift rows back
      hT[k][rr] = (__bf16)((r < rows && rc % period >= hshift) ? v : 0.f);
    }
    __syncthreads();
    // ---- dW^T (wave w: gate-units [16w,16w+16) of the block) and dU^T
    const bf16x8_t az = *reinterpret_cast<const bf16x8_t*>(&dzT[16 * w + col][8 * quad]);
#pragma unroll
    for (int d = 0; d < DT; ++d) {
      const bf16x8_t bx = *reinterpret_cast<const bf16x8_t*>(&xT[16 * d + col][8 * quad]);
      accW[d] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(az, bx, accW[d], 0, 0, 0);
    }
#pragma unroll
    for (int k = 0; k < HT; ++k) {
      const bf16x8_t bh = *reinterpret_cast<const bf16x8_t*>(&hT[16 * k + col][8 * quad]);
      accU[k] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(az, bh, accU[k], 0, 0, 0);
    }
    // ---- dx^T tiles: item = (din tile, row tile)
    if (dx != nullptr) {
#pragma unroll
      for (int i = 0; i < (DXT + 3) / 4; ++i) {
        const int item = w + 4 * i;
        if (item < DXT) {   // wave-uniform
          const int dtile = item >> 1, rt = item & 1;
          f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int ks = 0; ks < 2; ++ks) {
            const bf16x8_t bz = *reinterpret_cast<const bf16x8_t*>(&dzR[16 * rt + col][32 * ks + 8 * quad]);
            acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[i][ks], bz, acc, 0, 0, 0);
          }
          const long r = r0 + 16 * rt + col;
          if (r < rows) {
            float* o = dx + cb * dx_cb_stride + (size_t)r * lddx;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              const int din = dtile * 16 + 4 * quad + q;
              if (din < Din) {
                o[din] = acc[q];
              }
            }
          }
        }
      }
    }
    __syncthreads();
  }
  // ---- flush partial weight gradients. The C tiles hold [gate-unit][din|k] with
  // the gate-unit on 4 rows per lane; transpose them through LDS so that every
  // atomic wave-instruction adds 64 consecutive gate-units (256 contiguous bytes:
  // the full-rate shape; one lane per row would run ~17x slower).
  __shared__ float fl[DP + H][GR_CB + 1];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int c = 16 * w + 4 * quad + q;
#pragma unroll
    for (int d = 0; d < DT; ++d) fl[16 * d + col][c] = accW[d][q];
#pragma unroll
    for (int k = 0; k < HT; ++k) fl[DP + 16 * k + col][c] = accU[k][q];
  }
  __syncthreads();
  for (int e = tid; e < (DP + H) * GR_CB; e += 256) {
    const int row = e / GR_CB, c = e % GR_CB;
    const float v = fl[row][c];
    if (row < Din) atomicAdd(dW + (size_t)row * G4 + gu0 + c, v);
    else if (row == Din) atomicAdd(db + gu0 + c, v);
    else if (row >= DP) atomicAdd(dU + (size_t)(row - DP) * G4 + gu0 + c, v);
  }
}

template <int H>
void launch_grads_h(int DT, dim3 grid, hipStream_t st, const float* dz, const float* x, const float* h,
                    const float* W, float* dx, float* dW, float* dU, float* db, long rows, long period, long hshift,
                    int Din, int ldx, long dx_cb_stride, int lddx) {
  switch (DT) {
#define GQ_DT(D)                                                                                              \
  case D:                                                                                                     \
    hipLaunchKernelGGL((lstm_grads_kernel<H, D>), grid, dim3(256), 0, st, dz, x, h, W, dx, dW, dU, db, rows, period, \
                       hshift, Din, ldx, dx_cb_stride, lddx);                                                           \
    break;
    GQ_DT(1) GQ_DT(2) GQ_DT(3) GQ_DT(4) GQ_DT(5) GQ_DT(6) GQ_DT(7) GQ_DT(8) GQ_DT(9)
#undef GQ_DT
    default:
      TORCH_CHECK(false, "gnnqc lstm_grads: input width ", Din, " too large (max 143)");
  }
}

// Flat-row launcher shared by the sequence-major (lstm_grads) and time-major (lstm_tm_bwd)
// paths: row r of dz / x / dx has h_{t-1} at row r - hshift when r % period >= hshift.
// x rows have pitch ldx, dx rows pitch lddx; only the first Din (= rows of W) channels are used.
//   sequence-major [M,T,C]: period = T, hshift = 1;  time-major [T,Mp,C]: period = T*Mp, hshift = Mp.
void lstm_grads_rows(const float* dz, const float* x, const float* hseq, const float* W, float* dx, float* dW,
                     float* dU, float* db, long rows, long period, long hshift, int H, int Din, int ldx,
                     long dx_cb_stride, int lddx, hipStream_t st) {
  if (rows == 0) return;
  const int ncb = (4 * H) / GR_CB;
  const long ntiles = (rows + GR_ROWS - 1) / GR_ROWS;
  // enough workgroups to fill the chip, few enough that the final atomics stay cheap
  const int splits = deterministic_mode() ? 1 : (int)std::max<long>(1, std::min<long>(ntiles, std::max(32, 256 / ncb)));
  dim3 grid(ncb, splits);
  const int DT = (Din + 1 + 15) / 16;
#define GQ_GR_H(HH)                                                                                              \
  case HH:                                                                                                       \
    launch_grads_h<HH>(DT, grid, st, dz, x, hseq, W, dx, dW, dU, db, rows, period, hshift, Din, ldx, dx_cb_stride, \
                       lddx);                                                                                    \
    break;
  switch (H) {
    GQ_GR_H(16) GQ_GR_H(32) GQ_GR_H(64) GQ_GR_H(128)
    default: TORCH_CHECK(false, "gnnqc lstm_grads: unsupported hidden size ", H);
  }
#undef GQ_GR_H
  GQ_LAUNCH_CHECK();
}

int lstm_grads_col_blocks(int H) { return (4 * H) / GR_CB; }

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
  TORCH_CHECK(dz.is_cuda() && dz.scalar_type() == at::kFloat && dz.stride(2) == 1 && dz.stride(1) == dz.size(2) &&
                  dz.stride(0) == dz.size(1) * dz.size(2), "dz must be a contiguous [M,T,4H] row block");
  const int M = x.size(0), T = x.size(1), Din = x.size(2), H = hseq.size(2);
  TORCH_CHECK(dz.size(0) == M && dz.size(1) == T && dz.size(2) == 4 * H, "dz shape");
  TORCH_CHECK(hseq.size(0) == M && hseq.size(1) == T, "hseq shape");
  TORCH_CHECK(W.size(0) == Din && W.size(1) == 4 * H && dW.sizes() == W.sizes() && dU.size(0) == H &&
                  dU.size(1) == 4 * H && db.numel() == 4 * H, "gradient buffer shapes");
  TORCH_CHECK(Din + 1 <= 9 * 16, "gnnqc lstm_grads: input width ", Din, " too large (max 143)");
  c10::DeviceGuard guard(x.device());
  const int ncb = lstm_grads_col_blocks(H);
  // dx = dz W^T contracts over all 4H gate-units: with several column blocks each
  // block writes its partial product to its own slab (plain stores), summed below
  at::Tensor dx = need_dx ? at::empty({ncb, M, T, Din}, x.options()) : at::empty({0}, x.options());
  const long rows = (long)M * T;
  if (rows == 0) return need_dx ? dx.sum(0) : dx;
  lstm_grads_rows(dz.data_ptr<float>(), x.data_ptr<float>(), hseq.data_ptr<float>(), W.data_ptr<float>(),
                  need_dx ? dx.data_ptr<float>() : nullptr, dW.data_ptr<float>(), dU.data_ptr<float>(),
                  db.data_ptr<float>(), rows, T, 1, H, Din, x.stride(1), rows * Din, Din, stream());
  if (!need_dx) return dx;
  return ncb == 1 ? dx[0] : dx.sum(0);
}

}  // namespace gq

TORCH_LIBRARY_IMPL(gnnqc, CUDA, m) { m.impl("lstm_grads", &gq::lstm_grads); }
