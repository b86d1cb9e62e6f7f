// Shared device helpers for the gnnqc gfx950 kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <ATen/ATen.h>
#include <ATen/hip/HIPContext.h>
#include <c10/core/DeviceGuard.h>
#include <torch/library.h>

#include <vector>

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef float f32x16_t __attribute__((ext_vector_type(16)));

namespace gq {

__device__ __forceinline__ float sigmoidf_fast(float x) {
  return __builtin_amdgcn_rcpf(1.0f + __expf(-x));
}
__device__ __forceinline__ float tanhf_fast(float x) {
  // tanh(x) = 2*sigmoid(2x) - 1 ; saturates correctly for |x| -> inf
  return 2.0f * __builtin_amdgcn_rcpf(1.0f + __expf(-2.0f * x)) - 1.0f;
}

// Workgroup barrier that orders LDS traffic only. __syncthreads() also drains
// vmcnt (outstanding global loads AND stores on CDNA4), which in a persistent
// recurrence turns every step into a full HBM round trip; prefetched loads and
// fire-and-forget stores must be allowed to stay in flight across the step.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// Virtual block index for hardware block L of an N-block launch such that the `group` virtual
// blocks g * group ... g * group + group - 1 run on ONE XCD (blocks are dealt round-robin over the
// 8 XCDs: L and L + 8 share one). For launches whose groups re-read the same tiles (e.g. the
// column blocks of one row split): each XCD's L2 then serves the re-reads instead of all 8 XCDs
// fetching the tile from HBM. Identity unless N is a multiple of 8 * group.
__device__ __forceinline__ int xcd_group_remap(int L, int N, int group) {
  if (group <= 1 || N % (8 * group) != 0) return L;
  const int x = L & 7, k = L >> 3;      // the k-th block dealt to x's XCD
  return ((k / group) * 8 + x) * group + k % group;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

inline hipStream_t stream() { return at::hip::getCurrentHIPStream().stream(); }

// Deterministic mode: kernels whose cross-workgroup reductions use float
// atomics launch a single workgroup per output block instead, so every gradient element
// receives exactly one atomic (onto zero) and training is bitwise reproducible.
// Slower; for debugging / reproducibility runs. Set via gnnqc.ops.set_deterministic.
inline bool& deterministic_mode() {
  static bool v = false;
  return v;
}

// Deferred weight-gradient reductions (direct-accumulation training steps whose layers run the
// per-layer backward, e.g. SoilNet's 418-tile recurrences): while set, lstm_grads_rows queues its
// split reduction (workspace + destination buffers) instead of launching it, and
// lstm_reduce_flush (lstm_tm.hip) runs every queued one in ONE launch at the end of the backward.
// Set per call by gnnqc.ops.lstm, only when the gradient buffers are the optimiser's own.
inline bool& defer_reduce_mode() {
  static bool v = false;
  return v;
}
struct DeferredRed {
  at::Tensor ws;                 // [splits][RC] split records (kept alive until the flush)
  int H, Din, splits;
  float* dW;
  float* dU;
  float* db;
};
std::vector<DeferredRed>& deferred_reds();      // lstm_grads.hip

#define GQ_CHECK(cond, msg) TORCH_CHECK(cond, "gnnqc: ", msg)
#define GQ_LAUNCH_CHECK() do { hipError_t e__ = hipGetLastError(); TORCH_CHECK(e__ == hipSuccess, "gnnqc kernel launch failed: ", hipGetErrorString(e__)); } while (0)

inline void check_f32_cuda(const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), "gnnqc: ", name, " must be a GPU tensor");
  TORCH_CHECK(t.scalar_type() == at::kFloat, "gnnqc: ", name, " must be float32");
  TORCH_CHECK(t.is_contiguous(), "gnnqc: ", name, " must be contiguous");
}

// LSTM gate gradients dz: bf16 from the time-major recurrences (they are bf16 values already: the
// recurrence stages them through bf16 LDS for its MFMAs), fp32 from the sequence-major lstm_bwd
inline void check_dz_cuda(const at::Tensor& t) {
  TORCH_CHECK(t.is_cuda(), "gnnqc: dz must be a GPU tensor");
  TORCH_CHECK(t.scalar_type() == at::kFloat || t.scalar_type() == at::kBFloat16, "gnnqc: dz must be float32 or bfloat16");
  TORCH_CHECK(t.is_contiguous(), "gnnqc: dz must be contiguous");
}
inline int dz_bf16(const at::Tensor& t) { return t.scalar_type() == at::kBFloat16 ? 1 : 0; }
// saved LSTM gates of the time-major recurrences: bf16 [.., 4] (lstm_tm_common.h gates_pack)
inline void check_gates_cuda(const at::Tensor& t) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kBFloat16 && t.is_contiguous(),
              "gnnqc: saved LSTM gates must be a contiguous bfloat16 GPU tensor");
}
inline __bf16* bf16_ptr(const at::Tensor& t) {
  TORCH_CHECK(t.scalar_type() == at::kBFloat16, "gnnqc: expected a bfloat16 tensor");
  return reinterpret_cast<__bf16*>(t.data_ptr<at::BFloat16>());
}

}  // namespace gq
