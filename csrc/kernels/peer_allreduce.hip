// One-shot peer all-reduce of the flat gradient buffer over xGMI.
//
// RCCL's ring all-reduce moves a 753 KB buffer in 2 (N-1) latency-bound steps. On an MI355X node
// every GPU has a direct xGMI link to each of the other seven, so a small buffer is reduced in
// ONE step instead: every rank publishes its gradients in a registered region, the ranks signal
// each other with a flag store into each peer's region, and every rank then reads all N copies
// over its links at once and sums them in a fixed rank order (bit-identical on every rank).
//
// Region of one rank (uncached device memory, exported with hipIpcGetMemHandle, opened by the peers):
//   data[2][cap] floats   double buffer by launch parity: launch k writes data[k & 1] while a
//                         slow peer may still be reading data[(k - 1) & 1]; launch k + 1 on this
//                         rank only starts after every peer has signalled launch k, i.e. after
//                         every peer finished launch k - 1, so data[(k + 1) & 1] is free again.
//   flags[MAXR][16] ints  flags[p][0] = last launch number rank p has published (written by p)
//   ctl[16] ints          local: [0] launch counter, [1] arrival ticket, [2] spin timeout flag
// Ordering: data stores -> system-scope release fence (L2 write-back) -> flag stores into every
// peer's region; the reader acquires each flag at system scope and reads peer data with 16-byte
// loads that bypass L1 and L2 (sc0 sc1; no stale lines from two launches ago). The region is
// uncached device memory where the driver allows it. Every spin is bounded: a workgroup that
// gives up rejects the step (non-finite flag word 7 + a NaN in its slice), sets ctl[2] and exits;
// the host all-reduces ctl[2] at the epoch end and raises on every rank. It never hangs the device.
// Verified bitwise against RCCL / gloo with two ranks on ONE GPU only (tests/test_dp_gpu.py):
// between different GPUs over xGMI it is unverified (no multi-GPU box was available).
#include "common.h"

#include <cstring>

namespace gq {

constexpr int PEER_MAXR = 8;
constexpr int PEER_FLAG_PITCH = 16;   // ints: one 64-byte line per flag
constexpr long PEER_SPIN_LIMIT = 1L << 27;   // ~10 s of s_sleep polling: a stalled peer host, not a bug

struct PeerArgs {
  float* g;                       // local flat gradients: in = this rank's, out = scale * sum
  float* base[PEER_MAXR];         // every rank's region (this rank's own pointer at [rank])
  int* ctl;                       // this rank's ctl words
  int* ext;                       // the device's chain control words: [2] = reject this step
  long n, cap;
  int rank, world;
  float scale;
};

__device__ __forceinline__ int* peer_flags(float* base, long cap) { return reinterpret_cast<int*>(base + 2 * cap); }

typedef unsigned peer_u32x4 __attribute__((ext_vector_type(4)));

// 16-byte loads that bypass this GPU's L1 and L2 (sc0 sc1): a peer's region is written by the
// peer over xGMI, so a line cached here from an earlier launch would be stale
__device__ __forceinline__ __amdgpu_buffer_rsrc_t peer_rsrc(const float* p, long nfloats) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p), (short)0, (int)(nfloats * 4), 0x00020000);
}
__device__ __forceinline__ float4 peer_ld16(__amdgpu_buffer_rsrc_t r, long i4) {
  const peer_u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)(i4 * 16), 0, 1 | 16);
  return make_float4(__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z), __uint_as_float(v.w));
}

template <int W>
__global__ __launch_bounds__(256) void peer_allreduce_kernel(PeerArgs A) {
  const int tid = threadIdx.x;
  const int G = gridDim.x;
  // every workgroup reads the launch number before it arrives; the last arrival advances it
  const int k = __hip_atomic_load(A.ctl + 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const int par = k & 1;
  const long n4 = A.n / 4;
  // ---- publish this rank's gradients (float4 slices; tail by the last workgroup)
  float* mine = A.base[A.rank] + par * A.cap;
  for (long i = blockIdx.x * 256L + tid; i < n4; i += (long)G * 256)
    reinterpret_cast<float4*>(mine)[i] = reinterpret_cast<const float4*>(A.g)[i];
  for (long i = n4 * 4 + blockIdx.x * 256L + tid; i < A.n; i += (long)G * 256) mine[i] = A.g[i];
  __threadfence_system();
  __syncthreads();
  __shared__ int go;
  if (tid == 0) {
    const int ticket = __hip_atomic_fetch_add(A.ctl + 1, 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (ticket == G - 1) {           // all slices are out: tell every rank (incl. this one)
      __hip_atomic_store(A.ctl + 1, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __threadfence_system();
      for (int p = 0; p < W; ++p)
        __hip_atomic_store(peer_flags(A.base[p], A.cap) + A.rank * PEER_FLAG_PITCH, k + 1, __ATOMIC_RELEASE,
                           __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_store(A.ctl + 0, k + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    // wait for every rank's launch k (bounded)
    int ok = 1;
    int* fl = peer_flags(A.base[A.rank], A.cap);
    for (int p = 0; p < W && ok; ++p) {
      long spins = 0;
      while (__hip_atomic_load(fl + p * PEER_FLAG_PITCH, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < k + 1) {
        __builtin_amdgcn_s_sleep(2);
        if (++spins > PEER_SPIN_LIMIT) {
          ok = 0;
          break;
        }
      }
    }
    if (!ok) {
      // ANY workgroup that gave up rejects the whole step on this rank: it raises the non-finite
      // gradient flag (ext[7], read by adam_flagged; adam_guarded scans g) and leaves a NaN in the
      // first element of its own, never-reduced slice (so an unguarded update shows it too). The
      // timeout is recorded in this region's own control word (ctl[2], not the chain-timeout word),
      // which the host all-reduces at the epoch end and raises on every rank: a peer timeout is
      // fatal for the job, since the ranks' parameters may now differ.
      __hip_atomic_store(A.ctl + 2, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (A.ext != nullptr) __hip_atomic_store(A.ext + 7, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const long i0 = blockIdx.x * 256L * 4;
      if (i0 < A.n) A.g[i0] = __builtin_nanf("");
    }
    go = ok;
  }
  __syncthreads();
  if (!go) return;
  // ---- sum all ranks' copies in rank order: per thread one float4 from each of the W regions,
  // all W loads in flight before the first add (bit-identical on every rank)
  __amdgpu_buffer_rsrc_t rs[W];
#pragma unroll
  for (int p = 0; p < W; ++p) rs[p] = peer_rsrc(A.base[p] + par * A.cap, A.cap);
  for (long i = blockIdx.x * 256L + tid; i < n4; i += (long)G * 256) {
    float4 v[W];
#pragma unroll
    for (int p = 0; p < W; ++p) v[p] = peer_ld16(rs[p], i);
    float4 s = v[0];
#pragma unroll
    for (int p = 1; p < W; ++p) {
      s.x += v[p].x;
      s.y += v[p].y;
      s.z += v[p].z;
      s.w += v[p].w;
    }
    reinterpret_cast<float4*>(A.g)[i] = make_float4(s.x * A.scale, s.y * A.scale, s.z * A.scale, s.w * A.scale);
  }
  for (long i = n4 * 4 + blockIdx.x * 256L + tid; i < A.n; i += (long)G * 256) {
    float s = 0.f;
#pragma unroll
    for (int p = 0; p < W; ++p)
      s += __uint_as_float(__hip_atomic_load(reinterpret_cast<const unsigned*>(A.base[p] + par * A.cap) + i,
                                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
    A.g[i] = s * A.scale;
  }
}

// region: data[2][cap] + flags[PEER_MAXR][16] + ctl[16] (zeroed)
at::Tensor peer_region_alloc(int64_t cap) {
  TORCH_CHECK(cap > 0 && cap % 4 == 0, "peer_region_alloc: capacity must be a positive multiple of 4 floats");
  const int dev = c10::hip::current_device();
  c10::DeviceGuard guard(c10::Device(c10::kCUDA, dev));
  const size_t bytes = (2 * (size_t)cap + PEER_MAXR * PEER_FLAG_PITCH + 16) * sizeof(float);
  void* p = nullptr;
  // uncached device memory: the flags and data are written by peers over xGMI and polled / read
  // here (coarse-grained hipMalloc memory would let this GPU's L2 keep stale lines); plain
  // hipMalloc only if the driver refuses the flag
  if (hipExtMallocWithFlags(&p, bytes, hipDeviceMallocUncached) != hipSuccess || p == nullptr) {
    (void)hipGetLastError();
    TORCH_CHECK(hipMalloc(&p, bytes) == hipSuccess, "peer_region_alloc: hipMalloc failed");
  }
  TORCH_CHECK(hipMemset(p, 0, bytes) == hipSuccess, "peer_region_alloc: hipMemset failed");
  TORCH_CHECK(hipDeviceSynchronize() == hipSuccess, "peer_region_alloc: sync failed");
  return at::from_blob(p, {(long)(bytes / sizeof(float))}, [](void* q) { (void)hipFree(q); },
                       at::TensorOptions().dtype(at::kFloat).device(at::kCUDA, dev));
}

at::Tensor peer_ipc_handle(const at::Tensor& region) {
  hipIpcMemHandle_t h;
  TORCH_CHECK(hipIpcGetMemHandle(&h, region.data_ptr()) == hipSuccess, "peer_ipc_handle: hipIpcGetMemHandle failed");
  at::Tensor out = at::empty({(long)sizeof(h)}, at::TensorOptions().dtype(at::kByte));
  std::memcpy(out.data_ptr<uint8_t>(), &h, sizeof(h));
  return out;
}

int64_t peer_ipc_open(const at::Tensor& handle) {
  TORCH_CHECK(handle.numel() == (long)sizeof(hipIpcMemHandle_t) && handle.scalar_type() == at::kByte &&
                  !handle.is_cuda(), "peer_ipc_open: expected the 64-byte host handle of peer_ipc_handle");
  hipIpcMemHandle_t h;
  std::memcpy(&h, handle.data_ptr<uint8_t>(), sizeof(h));
  void* p = nullptr;
  TORCH_CHECK(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess) == hipSuccess,
              "peer_ipc_open: hipIpcOpenMemHandle failed");
  return reinterpret_cast<int64_t>(p);
}

void peer_ipc_close(int64_t ptr) { (void)hipIpcCloseMemHandle(reinterpret_cast<void*>(ptr)); }

// g (float32, contiguous, n <= cap): replaced by scale * (sum over ranks); bases: every rank's
// region address in this process (own region at [rank]); ctl = region tail (own)
int* chain_ctl(int dev);   // lstm_chain.hip: the device's chain control words

void peer_allreduce(at::Tensor g, at::IntArrayRef bases, at::Tensor region, int64_t rank, int64_t cap,
                    double scale) {
  check_f32_cuda(g, "g");
  const int world = (int)bases.size();
  TORCH_CHECK(world >= 1 && world <= PEER_MAXR && rank >= 0 && rank < world, "peer_allreduce: 1..8 ranks");
  TORCH_CHECK(g.numel() <= cap && region.numel() >= 2 * cap + PEER_MAXR * PEER_FLAG_PITCH + 16,
              "peer_allreduce: buffer larger than the registered region");
  TORCH_CHECK(reinterpret_cast<int64_t>(region.data_ptr()) == bases[rank], "peer_allreduce: own region mismatch");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(g.data_ptr()) % 16 == 0, "peer_allreduce: g must be 16-byte aligned");
  PeerArgs A{};
  A.g = g.data_ptr<float>();
  for (int p = 0; p < world; ++p) A.base[p] = reinterpret_cast<float*>(bases[p]);
  A.ctl = reinterpret_cast<int*>(region.data_ptr<float>() + 2 * cap + PEER_MAXR * PEER_FLAG_PITCH);
  A.n = g.numel();
  A.cap = cap;
  A.rank = (int)rank;
  A.world = world;
  A.scale = (float)scale;
  A.ext = chain_ctl(g.get_device());
  c10::DeviceGuard guard(g.device());
  // few workgroups: the copy / sum is link-bound, and every workgroup must be co-resident for the
  // arrival ticket (<= 64 x 256 threads always are)
  const int grid = (int)std::max<long>(1, std::min<long>(64, (A.n / 4 + 255) / 256));
#define GQ_PEER_W(WW) case WW: hipLaunchKernelGGL(peer_allreduce_kernel<WW>, dim3(grid), dim3(256), 0, stream(), A); break;
  switch (world) {
    GQ_PEER_W(1) GQ_PEER_W(2) GQ_PEER_W(3) GQ_PEER_W(4) GQ_PEER_W(5) GQ_PEER_W(6) GQ_PEER_W(7) GQ_PEER_W(8)
    default: TORCH_CHECK(false, "peer_allreduce: 1..8 ranks");
  }
#undef GQ_PEER_W
  GQ_LAUNCH_CHECK();
}

}  // namespace gq

// catch-all kernels (setup ops without device tensors; the all-reduce checks its operands itself)
TORCH_LIBRARY_FRAGMENT(gnnqc, m) {
  m.def("peer_region_alloc(int cap) -> Tensor", &gq::peer_region_alloc);
  m.def("peer_ipc_handle(Tensor region) -> Tensor", &gq::peer_ipc_handle);
  m.def("peer_ipc_open(Tensor handle) -> int", &gq::peer_ipc_open);
  m.def("peer_ipc_close(int ptr) -> ()", &gq::peer_ipc_close);
  m.def("peer_allreduce(Tensor(a!) g, int[] bases, Tensor region, int rank, int cap, float scale) -> ()",
        &gq::peer_allreduce);
}
