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
constexpr int PEER_SLICES = 1024;            // fused reduce + Adam: 1024-float slices (one per workgroup)

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

// region: data[2][cap] + flags[PEER_MAXR][16] + ctl[16] + slice flags[2][PEER_MAXR][PEER_SLICES] (zeroed)
at::Tensor peer_region_alloc(int64_t cap) {
  TORCH_CHECK(cap > 0 && cap % 4 == 0, "peer_region_alloc: capacity must be a positive multiple of 4 floats");
  const int dev = c10::hip::current_device();
  c10::DeviceGuard guard(c10::Device(c10::kCUDA, dev));
  const size_t bytes = (2 * (size_t)cap + PEER_MAXR * PEER_FLAG_PITCH + 16 + 2 * PEER_MAXR * PEER_SLICES) * sizeof(float);
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

// ---------------------------------------------------------------------------------------------
// Peer reduction FUSED into the flag-driven Adam update (adam.hip adam_flagged): ONE launch and one
// pass over the gradients per step instead of the all-reduce kernel followed by the optimiser.
// Workgroup b owns slice b (256 float4 = 1024 floats) end to end:
//   1. reads its slice of this rank's gradients, publishes it in data[k & 1] of its own region, and
//      (after a system-scope release) stores 2 (k + 1) + bad into slice flag [k & 1][rank][b] of
//      EVERY rank's region, bad = this rank rejects the step (LSTM chain timeout ext[2], a gradient
//      producer's non-finite flag ext[7], or a NaN poison in g[0]);
//   2. lanes 0..W-1 poll the W flags of slice b in its own region (bounded, system-scope acquire);
//      the step is rejected on EVERY rank if any rank's bit is set (all ranks see the same bits);
//   3. sums the W copies of the slice in rank order with cache-bypassing 16-byte loads (bit-identical
//      on every rank) and applies Adam to the slice (gscale folds the 1 / world mean in), skipping
//      non-finite elements (counted in state[5], identical on every rank);
//   4. an arrival ticket (ctl[1]; release from a slice that timed out, acquire by the last arrival);
//      the last arrival clears g[0] and the flags, advances the launch counter ctl[0], the step
//      counter and the batch cursor.
// Slices need no grid-wide barrier: a slice flag of launch k is only overwritten by launch k + 2 of
// its writer, which cannot start before this rank has finished launch k (it needs this rank's flags
// of launch k + 1); data[k & 1] likewise. Every wait is bounded: a timed-out slice rejects the step
// on this rank (no parameter of the slice changes), sets ctl[2] (the host raises at the epoch end).
// The slices of the timed-out launch that did not time out have updated already (undoing them would
// need a grid-wide barrier in every launch); from the next launch on, the sticky ctl[2] rejects the
// step on every rank (see ``sticky``), so the ranks stop at the same state until the job stops.
template <int W>
__global__ __launch_bounds__(256) void adam_peer_kernel(PeerArgs A, float* __restrict__ p, float* __restrict__ m,
                                                        float* __restrict__ v, const float* __restrict__ lr_p,
                                                        float* __restrict__ step_p, float b1, float b2, float eps,
                                                        float gscale, float wd, int* __restrict__ state,
                                                        long* __restrict__ cursor, long cursor_mod) {
  const int tid = threadIdx.x;
  const int b = blockIdx.x;
  float* __restrict__ g = A.g;
  int* __restrict__ ext = A.ext;
  const int k = __hip_atomic_load(A.ctl + 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const int par = k & 1;
  const float step0 = __hip_atomic_load(step_p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const int timeout = __hip_atomic_load(ext + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const int nonfin = __hip_atomic_load(ext + 7, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const float g0 = __hip_atomic_load(g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  // ctl[2] is sticky (only the host clears it): after a peer spin timeout in an earlier launch this
  // rank rejects, and through its flag bit makes EVERY rank reject, every later step, so no rank
  // trains on while another holds the partial update of the timed-out launch (the host raises on
  // every rank at the epoch end; the job resumes from its last checkpoint)
  const int sticky = __hip_atomic_load(A.ctl + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const int bad = (timeout != 0 || nonfin != 0 || sticky != 0 || !isfinite(g0)) ? 1 : 0;
  const long n4 = A.n / 4;
  const long i = (long)b * 256 + tid;
  // ---- 1. publish
  float4 gg = make_float4(0.f, 0.f, 0.f, 0.f);
  if (i < n4) gg = reinterpret_cast<const float4*>(g)[i];
  float* mine = A.base[A.rank] + par * A.cap;
  if (i < n4) reinterpret_cast<float4*>(mine)[i] = gg;
  const long it = n4 * 4 + i;                     // (n % 4 tail: slice 0's threads, one element each)
  float gt = 0.f;
  if (b == 0 && it < A.n) {
    gt = g[it];
    mine[it] = gt;
  }
  __threadfence_system();
  __syncthreads();
  const int fval = 2 * (k + 1) + bad;
  if (tid < W) {
    int* fl = peer_flags(A.base[tid], A.cap) + PEER_MAXR * PEER_FLAG_PITCH + 16;   // slice flags of rank tid
    __hip_atomic_store(fl + (par * PEER_MAXR + A.rank) * PEER_SLICES + b, fval, __ATOMIC_RELEASE,
                       __HIP_MEMORY_SCOPE_SYSTEM);
  }
  // ---- 2. wait for every rank's slice b (lane q polls rank q's flag in this rank's region)
  __shared__ int sbad, sok;
  if (tid == 0) {
    sbad = 0;
    sok = 1;
  }
  __syncthreads();
  if (tid < W) {
    const int* fl = peer_flags(A.base[A.rank], A.cap) + PEER_MAXR * PEER_FLAG_PITCH + 16 +
                    (par * PEER_MAXR + tid) * PEER_SLICES + b;
    long spins = 0;
    int f;
    while ((f = __hip_atomic_load(fl, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM)) < 2 * (k + 1)) {
      __builtin_amdgcn_s_sleep(2);
      if (++spins > PEER_SPIN_LIMIT) break;
    }
    if (f < 2 * (k + 1)) {
      atomicExch(&sok, 0);
      __hip_atomic_store(A.ctl + 2, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else if (f & 1) {
      atomicExch(&sbad, 1);
    }
  }
  __syncthreads();
  const bool ok = sok != 0 && sbad == 0;
  // ---- 3. rank-order sum + Adam on the slice
  int skipped = 0;
  if (i < n4) {
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
    if (sok) {
      float4 vv[W];
#pragma unroll
      for (int q = 0; q < W; ++q) vv[q] = peer_ld16(peer_rsrc(A.base[q] + par * A.cap, A.cap), i);
      s = vv[0];
#pragma unroll
      for (int q = 1; q < W; ++q) {
        s.x += vv[q].x;
        s.y += vv[q].y;
        s.z += vv[q].z;
        s.w += vv[q].w;
      }
    }
    if (ok) {
      float4 pp = reinterpret_cast<const float4*>(p)[i];
      float4 mm = reinterpret_cast<const float4*>(m)[i];
      float4 vq = reinterpret_cast<const float4*>(v)[i];
      const float step = step0 + 1.0f;
      const float alpha = *lr_p * sqrtf(1.0f - powf(b2, step)) / (1.0f - powf(b1, step));
#define GQ_ADAMP_LANE(c)                                          \
      if (isfinite(s.c)) {                                        \
        const float gc = s.c * gscale + wd * pp.c;                \
        mm.c = b1 * mm.c + (1.f - b1) * gc;                       \
        vq.c = b2 * vq.c + (1.f - b2) * gc * gc;                  \
        pp.c -= alpha * mm.c / (sqrtf(vq.c) + eps);               \
      } else {                                                    \
        ++skipped;                                                \
      }
      GQ_ADAMP_LANE(x) GQ_ADAMP_LANE(y) GQ_ADAMP_LANE(z) GQ_ADAMP_LANE(w)
#undef GQ_ADAMP_LANE
      reinterpret_cast<float4*>(p)[i] = pp;
      reinterpret_cast<float4*>(m)[i] = mm;
      reinterpret_cast<float4*>(v)[i] = vq;
    }
    // g[0] is cleared by the last arrival only (every workgroup read it above)
    if (i == 0) {
      g[1] = 0.f;
      g[2] = 0.f;
      g[3] = 0.f;
    } else {
      reinterpret_cast<float4*>(g)[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
  if (b == 0 && it < A.n) {
    g[it] = 0.f;
    if (ok) {
      float st = 0.f;
#pragma unroll
      for (int q = 0; q < W; ++q)
        st += __uint_as_float(__hip_atomic_load(reinterpret_cast<const unsigned*>(A.base[q] + par * A.cap) + it,
                                                __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
      if (isfinite(st)) {
        const float step = step0 + 1.0f;
        const float alpha = *lr_p * sqrtf(1.0f - powf(b2, step)) / (1.0f - powf(b1, step));
        const float gc = st * gscale + wd * p[it];
        m[it] = b1 * m[it] + (1.f - b1) * gc;
        v[it] = b2 * v[it] + (1.f - b2) * gc * gc;
        p[it] -= alpha * m[it] / (sqrtf(v[it]) + eps);
      } else {
        ++skipped;
      }
    }
  }
  if (skipped) atomicAdd(state + 5, skipped);
  // ---- 4. arrival ticket; the last arrival finishes the step's bookkeeping. A workgroup whose wait
  // timed out stored ctl[2] (lanes < W: the wave of tid 0) and arrives with a RELEASE ticket; the
  // last arrival acquires after its ticket (the relaxed tickets in between continue the release
  // sequence), so it sees every timeout before it decides. Slices that did not time out keep the
  // relaxed ticket: a release there would drain the slice's update stores first (~6 us, adam.hip).
  __shared__ int last;
  __builtin_amdgcn_s_barrier();
  if (tid == 0) {
    const int ticket = sok ? __hip_atomic_fetch_add(A.ctl + 1, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                           : __hip_atomic_fetch_add(A.ctl + 1, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    last = ticket == (int)gridDim.x - 1;
  }
  lds_barrier();
  if (!last || tid != 0) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  __hip_atomic_store(A.ctl + 1, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(A.ctl + 0, k + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  g[0] = 0.f;
  // (a slice that timed out rejected only itself on this rank: count the step as rejected too)
  const bool all_ok = ok && __hip_atomic_load(A.ctl + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0;
  if (all_ok) step_p[0] = step0 + 1.0f;
  else __hip_atomic_fetch_add(state + 3, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(state + 2, all_ok ? 1 : 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (timeout) {
    __hip_atomic_store(ext + 2, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_fetch_add(ext + 3, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (nonfin) __hip_atomic_store(ext + 7, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (cursor != nullptr) cursor[0] = (cursor[0] + 1) % cursor_mod;
}

// p / g / m / v: the flat optimiser buffers (g = this rank's gradients, cleared); state / cursor as
// adam_flagged; bases / region / rank / cap as peer_allreduce. Returns false (nothing launched) when
// the buffer has more slices than the region's slice flags (the caller then runs the two kernels).
bool adam_peer(at::Tensor p, at::Tensor g, at::Tensor m, at::Tensor v, const at::Tensor& lr, at::Tensor step,
               double b1, double b2, double eps, double gscale, double wd, at::Tensor state,
               const c10::optional<at::Tensor>& cursor, int64_t cursor_mod, at::IntArrayRef bases,
               at::Tensor region, int64_t rank, int64_t cap) {
  const at::Tensor* ops[] = {&p, &g, &m, &v, &lr, &step};
  for (const at::Tensor* t : ops) check_f32_cuda(*t, "adam_peer operand");
  const int world = (int)bases.size();
  TORCH_CHECK(world >= 1 && world <= PEER_MAXR && rank >= 0 && rank < world, "adam_peer: 1..8 ranks");
  const long n = p.numel();
  TORCH_CHECK(n >= 4 && g.numel() == n && m.numel() == n && v.numel() == n, "adam_peer: size mismatch");
  TORCH_CHECK(n <= cap && region.numel() >= 2 * cap + PEER_MAXR * PEER_FLAG_PITCH + 16 + 2 * PEER_MAXR * PEER_SLICES,
              "adam_peer: buffer larger than the registered region");
  TORCH_CHECK(reinterpret_cast<int64_t>(region.data_ptr()) == bases[rank], "adam_peer: own region mismatch");
  for (const at::Tensor* t : {&p, &g, &m, &v})
    TORCH_CHECK(reinterpret_cast<uintptr_t>(t->data_ptr()) % 16 == 0, "adam_peer: buffers must be 16-byte aligned");
  TORCH_CHECK(state.is_cuda() && state.scalar_type() == at::kInt && state.numel() >= 6 && state.is_contiguous(),
              "adam_peer: state must be int32[>=6] on the device");
  long* cp = nullptr;
  if (cursor.has_value() && cursor->defined()) {
    TORCH_CHECK(cursor->is_cuda() && cursor->scalar_type() == at::kLong && cursor->numel() >= 1 && cursor_mod >= 1,
                "adam_peer: cursor int64[1], cursor_mod >= 1");
    cp = cursor->data_ptr<int64_t>();
  }
  const long grid = std::max<long>(1, (n / 4 + 255) / 256);
  TORCH_CHECK(n % 4 < 256, "adam_peer: tail");
  if (grid > PEER_SLICES) return false;
  PeerArgs A{};
  A.g = g.data_ptr<float>();
  for (int q = 0; q < world; ++q) A.base[q] = reinterpret_cast<float*>(bases[q]);
  A.ctl = reinterpret_cast<int*>(region.data_ptr<float>() + 2 * cap + PEER_MAXR * PEER_FLAG_PITCH);
  A.n = n;
  A.cap = cap;
  A.rank = (int)rank;
  A.world = world;
  A.scale = 1.f;
  A.ext = chain_ctl(g.get_device());
  c10::DeviceGuard guard(g.device());
#define GQ_ADAMP_W(WW)                                                                                         \
  case WW:                                                                                                     \
    hipLaunchKernelGGL(adam_peer_kernel<WW>, dim3((int)grid), dim3(256), 0, stream(), A, p.data_ptr<float>(),  \
                       m.data_ptr<float>(), v.data_ptr<float>(), lr.data_ptr<float>(), step.data_ptr<float>(), \
                       (float)b1, (float)b2, (float)eps, (float)gscale, (float)wd, state.data_ptr<int>(), cp,   \
                       cursor_mod);                                                                            \
    break;
  switch (world) {
    GQ_ADAMP_W(1) GQ_ADAMP_W(2) GQ_ADAMP_W(3) GQ_ADAMP_W(4) GQ_ADAMP_W(5) GQ_ADAMP_W(6) GQ_ADAMP_W(7) GQ_ADAMP_W(8)
    default: TORCH_CHECK(false, "adam_peer: 1..8 ranks");
  }
#undef GQ_ADAMP_W
  GQ_LAUNCH_CHECK();
  return true;
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
  m.def("adam_peer(Tensor(a!) p, Tensor(b!) g, Tensor(c!) m, Tensor(d!) v, Tensor lr, Tensor(e!) step, float b1, "
        "float b2, float eps, float gscale, float wd, Tensor(f!) state, Tensor(g!)? cursor, int cursor_mod, int[] bases, "
        "Tensor region, int rank, int cap) -> bool", &gq::adam_peer);
}
