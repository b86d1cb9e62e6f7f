// Single-launch Adam over the flat fp32 parameter buffer.
//
// The reference uses Keras Adam (jit_compile XLA; beta1 .9, beta2 .999, eps 1e-7,
// libs/fit_model.py:71-74). Keras' update rule is the "epsilon hat" form:
//   m = b1 m + (1-b1) g ; v = b2 v + (1-b2) g^2
//   p -= lr * sqrt(1-b2^t)/(1-b1^t) * m / (sqrt(v) + eps)
// All trainables live in one contiguous buffer (parameters are views into it) so
// the optimiser is one kernel and the DP gradient all-reduce is one collective;
// grad_scale folds the 1/world averaging in. lr and step are device tensors so the
// launch can be captured in a HIP graph and replayed with a changing schedule.
#include "common.h"

namespace gq {

// zero_g: the gradient buffer is cleared once read (the next step's backward accumulates onto
// zeros; the trainer then launches no separate zero-fill per step), also for a skipped step.
__global__ void adam_kernel(float* __restrict__ p, float* __restrict__ g, float* __restrict__ m,
                            float* __restrict__ v, const float* __restrict__ lr_p, const float* __restrict__ step_p,
                            long n, float b1, float b2, float eps, float gscale, float wd,
                            const int* __restrict__ ok_p, int zero_g) {
  const long n4 = n / 4;
  const long stride = (long)gridDim.x * blockDim.x;
  if (ok_p != nullptr && *ok_p == 0) {         // non-finite gradients: skip the whole update
    if (zero_g) {
      for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4; i += stride)
        reinterpret_cast<float4*>(g)[i] = make_float4(0.f, 0.f, 0.f, 0.f);
      for (long i = n4 * 4 + blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += stride) g[i] = 0.f;
    }
    return;
  }
  const float step = *step_p;
  const float lr = *lr_p;
  const float bc1 = 1.0f - powf(b1, step);
  const float bc2 = 1.0f - powf(b2, step);
  const float alpha = lr * sqrtf(bc2) / bc1;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 gg = reinterpret_cast<const float4*>(g)[i];
    if (zero_g) reinterpret_cast<float4*>(g)[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    float4 pp = reinterpret_cast<float4*>(p)[i];
    float4 mm = reinterpret_cast<float4*>(m)[i];
    float4 vv = reinterpret_cast<float4*>(v)[i];
#define GQ_ADAM_LANE(c)                                         \
    {                                                           \
      float gc = gg.c * gscale + wd * pp.c;                     \
      mm.c = b1 * mm.c + (1.f - b1) * gc;                       \
      vv.c = b2 * vv.c + (1.f - b2) * gc * gc;                  \
      pp.c -= alpha * mm.c / (sqrtf(vv.c) + eps);               \
    }
    GQ_ADAM_LANE(x) GQ_ADAM_LANE(y) GQ_ADAM_LANE(z) GQ_ADAM_LANE(w)
#undef GQ_ADAM_LANE
    reinterpret_cast<float4*>(p)[i] = pp;
    reinterpret_cast<float4*>(m)[i] = mm;
    reinterpret_cast<float4*>(v)[i] = vv;
  }
  for (long i = n4 * 4 + blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += stride) {
    float gc = g[i] * gscale + wd * p[i];
    if (zero_g) g[i] = 0.f;
    m[i] = b1 * m[i] + (1.f - b1) * gc;
    v[i] = b2 * v[i] + (1.f - b2) * gc * gc;
    p[i] -= alpha * m[i] / (sqrtf(v[i]) + eps);
  }
}

__global__ void nonfinite_kernel(const float* __restrict__ x, long n, int* out) {
  int bad = 0;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    bad += !isfinite(x[i]);
  // wave-level reduce then one atomic per wave
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) bad += __shfl_xor(bad, o, 64);
  if ((threadIdx.x & 63) == 0 && bad) atomicAdd(out, bad);
}

// Non-finite gradient guard, graph-capturable: every workgroup counts
// non-finite entries of g into state[0]; the last workgroup to finish (ticket state[1])
// publishes ok = (count == 0) in state[2], advances the optimiser step counter only for
// a good step, counts skipped steps in state[3] and re-arms state[0..1] for the next
// launch. The Adam kernel then reads state[2]. No host synchronisation anywhere.
// ext (optional): the LSTM chain kernels' control words (lstm_chain.hip). ext[2] is set when a
// chain consumer's bounded spin timed out in this step - its activations / gradients then came
// from stale data, so the step is rejected like a non-finite one; the flag is cleared and
// counted in ext[3] (the host raises on it at epoch end).
__global__ void grad_guard_kernel(const float* __restrict__ g, long n, int* __restrict__ state,
                                  float* __restrict__ step, int* __restrict__ ext) {
  int bad = 0;
  const long n4 = n / 4, stride = (long)gridDim.x * blockDim.x;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4; i += stride) {
    const float4 v = reinterpret_cast<const float4*>(g)[i];
    bad += !isfinite(v.x) + !isfinite(v.y) + !isfinite(v.z) + !isfinite(v.w);
  }
  for (long i = n4 * 4 + blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += stride) bad += !isfinite(g[i]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) bad += __shfl_xor(bad, o, 64);
  __shared__ int wsum[16];
  if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = bad;
  __syncthreads();
  if (threadIdx.x == 0) {
    int tot = 0;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) tot += wsum[w];
    if (tot) atomicAdd(&state[0], tot);
    __threadfence();
    const int ticket = atomicAdd(&state[1], 1);
    if (ticket == (int)gridDim.x - 1) {          // last workgroup: all counts are in
      const int cnt = atomicAdd(&state[0], 0);
      int stale = 0;
      if (ext != nullptr) {
        stale = atomicExch(&ext[2], 0);
        if (stale) atomicAdd(&ext[3], 1);
        atomicExch(&ext[7], 0);                  // producer flag (adam_flagged): the scan covers it
      }
      const int ok = cnt == 0 && stale == 0;
      state[2] = ok;
      if (ok) step[0] += 1.0f;
      else state[3] += 1;
      state[0] = 0;
      state[1] = 0;
      __threadfence();
    }
  }
}

void grad_guard(const at::Tensor& g, at::Tensor state, at::Tensor step, const c10::optional<at::Tensor>& ext) {
  check_f32_cuda(g, "g");
  check_f32_cuda(step, "step");
  TORCH_CHECK(state.is_cuda() && state.scalar_type() == at::kInt && state.numel() >= 4 && state.is_contiguous(),
              "grad_guard: state must be int32[4] on the device");
  TORCH_CHECK((reinterpret_cast<uintptr_t>(g.data_ptr()) % 16) == 0, "grad_guard: g must be 16-byte aligned");
  c10::DeviceGuard guard(g.device());
  const long n = g.numel();
  const int grid = (int)std::max<long>(1, std::min<long>((n / 4 + 255) / 256, 128));
  int* ep = nullptr;
  if (ext.has_value() && ext->defined()) {
    TORCH_CHECK(ext->is_cuda() && ext->scalar_type() == at::kInt && ext->numel() >= 4 && ext->get_device() == g.get_device(),
                "grad_guard: ext must be int32[4] on the gradient's device");
    ep = ext->data_ptr<int>();
  }
  hipLaunchKernelGGL(grad_guard_kernel, dim3(grid), dim3(256), 0, stream(), g.data_ptr<float>(), n,
                     state.data_ptr<int>(), step.data_ptr<float>(), ep);
  GQ_LAUNCH_CHECK();
}

void adam_step(at::Tensor p, at::Tensor g, at::Tensor m, at::Tensor v, const at::Tensor& lr,
               const at::Tensor& step, double b1, double b2, double eps, double gscale, double wd,
               const c10::optional<at::Tensor>& ok, bool zero_grad) {
  const at::Tensor* ops[] = {&p, &g, &m, &v, &lr, &step};
  for (const at::Tensor* t : ops) check_f32_cuda(*t, "adam operand");
  if (ok.has_value())
    TORCH_CHECK(ok->is_cuda() && ok->scalar_type() == at::kInt && ok->numel() >= 4, "adam: guard state int32[4]");
  const long n = p.numel();
  TORCH_CHECK(g.numel() == n && m.numel() == n && v.numel() == n, "adam: size mismatch");
  TORCH_CHECK((reinterpret_cast<uintptr_t>(p.data_ptr()) % 16) == 0 && (reinterpret_cast<uintptr_t>(g.data_ptr()) % 16) == 0,
              "adam: buffers must be 16-byte aligned");
  c10::DeviceGuard guard(p.device());
  const int block = 256;
  const int grid = (int)std::max<long>(1, std::min<long>((n / 4 + block - 1) / block, 1024));
  hipLaunchKernelGGL(adam_kernel, dim3(grid), dim3(block), 0, stream(), p.data_ptr<float>(), g.data_ptr<float>(),
                     m.data_ptr<float>(), v.data_ptr<float>(), lr.data_ptr<float>(), step.data_ptr<float>(), n,
                     (float)b1, (float)b2, (float)eps, (float)gscale, (float)wd,
                     ok.has_value() ? ok->data_ptr<int>() + 2 : nullptr, zero_grad ? 1 : 0);
  GQ_LAUNCH_CHECK();
}

// Guard + Adam in ONE launch (was grad_guard then adam_kernel): every workgroup loads its share of
// g into registers and counts non-finite entries; arrival ticket state[1]; the last arrival
// decides ok (no non-finite value, no chain timeout in ext[2]), advances the step counter for
// a good step, re-arms the counters and bumps the generation word state[4]; every workgroup
// waits for the generation to move (all are co-resident: grid <= resident capacity, checked
// on the host; bounded spin) and then applies the update from registers, or only clears g.
// cursor (optional): the device batch cursor of multi-step graphs, advanced mod cursor_mod.
template <int K>
__global__ __launch_bounds__(256) void adam_guarded_kernel(
    float* __restrict__ p, float* __restrict__ g, float* __restrict__ m, float* __restrict__ v,
    const float* __restrict__ lr_p, float* __restrict__ step_p, long n, float b1, float b2, float eps, float gscale,
    float wd, int* __restrict__ state, int* __restrict__ ext, long* __restrict__ cursor, long cursor_mod) {
  __shared__ int wsum[4];
  __shared__ int okf;
  const int tid = threadIdx.x;
  const long n4 = n / 4, stride = (long)gridDim.x * blockDim.x;
  const long i0 = blockIdx.x * (long)blockDim.x + tid;
  __shared__ int gen_s;
  __shared__ float step_s;
  // state[4] = 2 * generation + ok of the last decision. Thread 0 reads it and the step counter
  // with ACQUIRE loads before its arrival ticket: they complete before the ticket is issued, so
  // the last arrival (which changes both only after every ticket) cannot overtake them.
  if (tid == 0) {
    gen_s = __hip_atomic_load(state + 4, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
    step_s = __hip_atomic_load(step_p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
  }
  float4 gg[K], pq[K], mq[K], vq[K];
  float gt = 0.f;
  int bad = 0;
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const long i = i0 + k * stride;
    const bool in = i < n4;
    gg[k] = in ? reinterpret_cast<const float4*>(g)[i] : make_float4(0.f, 0.f, 0.f, 0.f);
    // p / m / v are loaded now too: their latency overlaps the grid-wide decision below
    pq[k] = in ? reinterpret_cast<const float4*>(p)[i] : make_float4(0.f, 0.f, 0.f, 0.f);
    mq[k] = in ? reinterpret_cast<const float4*>(m)[i] : make_float4(0.f, 0.f, 0.f, 0.f);
    vq[k] = in ? reinterpret_cast<const float4*>(v)[i] : make_float4(0.f, 0.f, 0.f, 0.f);
    bad += !isfinite(gg[k].x) + !isfinite(gg[k].y) + !isfinite(gg[k].z) + !isfinite(gg[k].w);
  }
  const long it = n4 * 4 + i0;                   // (n % 4 tail: one element per thread at most)
  if (it < n) {
    gt = g[it];
    bad += !isfinite(gt);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) bad += __shfl_xor(bad, o, 64);
  if ((tid & 63) == 0) wsum[tid >> 6] = bad;
  __syncthreads();
  if (tid == 0) {
    const int gen0 = gen_s;
    const float step0 = step_s;
    const int tot = (wsum[0] + wsum[1]) + (wsum[2] + wsum[3]);
    // ONE atomic carries both the arrival (low 16 bits) and "this workgroup saw a non-finite
    // value" (high bits): the last arrival learns everything from the value it gets back
    const int old = __hip_atomic_fetch_add(state + 1, 1 + (tot ? 65536 : 0), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    int ok;
    if ((old & 0xffff) == (int)gridDim.x - 1) {  // last arrival
      const int nbad = (old >> 16) + (tot ? 1 : 0);
      int stale = 0;
      if (ext != nullptr) {
        stale = __hip_atomic_exchange(ext + 2, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (stale) __hip_atomic_fetch_add(ext + 3, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(ext + 7, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // (the scan covers it)
      }
      ok = nbad == 0 && stale == 0;
      if (ok) step_p[0] = step0 + 1.0f;
      else __hip_atomic_fetch_add(state + 3, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(state + 1, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(state + 2, ok, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(state + 4, ((gen0 >> 1) + 1) * 2 + ok, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      int spins = 0, gv;
      while ((gv = __hip_atomic_load(state + 4, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) == gen0) {
        __builtin_amdgcn_s_sleep(2);
        if (++spins > (1 << 22)) break;          // never expected (co-resident grid)
      }
      if (gv != gen0) {
        ok = gv & 1;
      } else {
        // the decision never arrived (the grid was not co-resident): this workgroup's slice is
        // left unchanged while others may update theirs - a partial step. Count it in state[6];
        // the trainer raises on it at epoch end (FlatOptimizer.check_update).
        ok = 0;
        __hip_atomic_fetch_add(state + 6, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    okf = ok;
  }
  __syncthreads();
  const float step0 = step_s;
  if (!okf) {                                    // rejected step: parameters untouched, g cleared
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const long i = i0 + k * stride;
      if (i < n4) reinterpret_cast<float4*>(g)[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    if (it < n) g[it] = 0.f;
  } else {
    const float step = step0 + 1.0f;
    const float lr = *lr_p;
    const float alpha = lr * sqrtf(1.0f - powf(b2, step)) / (1.0f - powf(b1, step));
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const long i = i0 + k * stride;
      if (i >= n4) break;
      reinterpret_cast<float4*>(g)[i] = make_float4(0.f, 0.f, 0.f, 0.f);
      float4 pp = pq[k], mm = mq[k], vv = vq[k];
#define GQ_ADAM_LANE(c)                                         \
      {                                                         \
        float gc = gg[k].c * gscale + wd * pp.c;                \
        mm.c = b1 * mm.c + (1.f - b1) * gc;                     \
        vv.c = b2 * vv.c + (1.f - b2) * gc * gc;                \
        pp.c -= alpha * mm.c / (sqrtf(vv.c) + eps);             \
      }
      GQ_ADAM_LANE(x) GQ_ADAM_LANE(y) GQ_ADAM_LANE(z) GQ_ADAM_LANE(w)
#undef GQ_ADAM_LANE
      reinterpret_cast<float4*>(p)[i] = pp;
      reinterpret_cast<float4*>(m)[i] = mm;
      reinterpret_cast<float4*>(v)[i] = vv;
    }
    if (it < n) {
      g[it] = 0.f;
      const float gc = gt * gscale + wd * p[it];
      m[it] = b1 * m[it] + (1.f - b1) * gc;
      v[it] = b2 * v[it] + (1.f - b2) * gc * gc;
      p[it] -= alpha * m[it] / (sqrtf(v[it]) + eps);
    }
  }
  if (cursor != nullptr && blockIdx.x == 0 && tid == 0) cursor[0] = (cursor[0] + 1) % cursor_mod;
}

// capacity of the co-resident grid (blocks of 256 threads) for adam_guarded_kernel<K>
template <int K>
static int adam_guarded_capacity(int dev) {
  static int cap[64] = {0};
  if (cap[dev] == 0) {
    hipDeviceProp_t prop;
    TORCH_CHECK(hipGetDeviceProperties(&prop, dev) == hipSuccess, "adam_guarded: device properties");
    int occ = 0;
    TORCH_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, reinterpret_cast<const void*>(&adam_guarded_kernel<K>),
                                                           256, 0) == hipSuccess, "adam_guarded: occupancy");
    cap[dev] = std::max(1, occ * prop.multiProcessorCount);
  }
  return cap[dev];
}

// Returns false (nothing launched) when the buffer is too large for one co-resident grid with
// <= 8 float4 per thread; the caller then runs grad_guard + adam_step.
bool adam_guarded(at::Tensor p, at::Tensor g, at::Tensor m, at::Tensor v, const at::Tensor& lr, at::Tensor step,
                  double b1, double b2, double eps, double gscale, double wd, at::Tensor state,
                  const c10::optional<at::Tensor>& ext, const c10::optional<at::Tensor>& cursor, int64_t cursor_mod) {
  const at::Tensor* ops[] = {&p, &g, &m, &v, &lr, &step};
  for (const at::Tensor* t : ops) check_f32_cuda(*t, "adam operand");
  TORCH_CHECK(state.is_cuda() && state.scalar_type() == at::kInt && state.numel() >= 7 && state.is_contiguous(),
              "adam_guarded: state must be int32[>=7] on the device");
  const long n = p.numel();
  TORCH_CHECK(g.numel() == n && m.numel() == n && v.numel() == n, "adam: size mismatch");
  TORCH_CHECK((reinterpret_cast<uintptr_t>(p.data_ptr()) % 16) == 0 && (reinterpret_cast<uintptr_t>(g.data_ptr()) % 16) == 0 &&
                  (reinterpret_cast<uintptr_t>(m.data_ptr()) % 16) == 0 && (reinterpret_cast<uintptr_t>(v.data_ptr()) % 16) == 0,
              "adam: buffers must be 16-byte aligned");
  int* ep = nullptr;
  if (ext.has_value() && ext->defined()) {
    TORCH_CHECK(ext->is_cuda() && ext->scalar_type() == at::kInt && ext->numel() >= 4, "adam_guarded: ext int32[4]");
    ep = ext->data_ptr<int>();
  }
  long* cp = nullptr;
  if (cursor.has_value() && cursor->defined()) {
    TORCH_CHECK(cursor->is_cuda() && cursor->scalar_type() == at::kLong && cursor->numel() >= 1 && cursor_mod >= 1,
                "adam_guarded: cursor int64[1], cursor_mod >= 1");
    cp = cursor->data_ptr<int64_t>();
  }
  c10::DeviceGuard guard(p.device());
  const int dev = p.get_device();
  const long n4 = std::max<long>(1, (n / 4 + 255) / 256);      // 256-thread blocks at one float4 each
#define GQ_ADAM_G(KK)                                                                                        \
  {                                                                                                          \
    const int grid = (int)((n4 + KK - 1) / KK);                                                              \
    if (grid <= adam_guarded_capacity<KK>(dev) && (long)grid * 256 > n % 4) {                                \
      hipLaunchKernelGGL(adam_guarded_kernel<KK>, dim3(grid), dim3(256), 0, stream(), p.data_ptr<float>(),    \
                         g.data_ptr<float>(), m.data_ptr<float>(), v.data_ptr<float>(), lr.data_ptr<float>(), \
                         step.data_ptr<float>(), n, (float)b1, (float)b2, (float)eps, (float)gscale, (float)wd, \
                         state.data_ptr<int>(), ep, cp, cursor_mod);                                          \
      GQ_LAUNCH_CHECK();                                                                                     \
      return true;                                                                                           \
    }                                                                                                        \
  }
  GQ_ADAM_G(1) GQ_ADAM_G(2) GQ_ADAM_G(4) GQ_ADAM_G(8)
#undef GQ_ADAM_G
  return false;
}

// Adam with the step decision taken from FLAGS instead of a grid-wide scan of g: every kernel that
// writes this step's gradients (the CML training step: time4 / head, the LSTM weight-gradient
// reduction, the fused GCN backward) raises ext[7] when a value it adds is not finite; the LSTM
// chain raises ext[2] on a spin timeout; in data parallel, chain_poison turns either flag into a
// NaN in g[0] before the all-reduce, so every rank sees it there. Every workgroup reads ext[2],
// ext[7] and g[0] BEFORE its arrival ticket, and only the last arrival clears them (and g[0], which
// the update otherwise leaves to it), so all workgroups take the same decision without waiting for
// each other: no co-residency assumption, no spin (adam_guarded's grid-wide barrier cost ~8 us).
// A gradient element that is not finite although no producer flagged (fp32 overflow of a sum of
// finite parts) leaves its parameter and slots untouched and is counted in state[5].
__global__ __launch_bounds__(256) void adam_flagged_kernel(
    float* __restrict__ p, float* __restrict__ g, float* __restrict__ m, float* __restrict__ v,
    const float* __restrict__ lr_p, float* __restrict__ step_p, long n, float b1, float b2, float eps, float gscale,
    float wd, int* __restrict__ state, int* __restrict__ ext, long* __restrict__ cursor, long cursor_mod) {
  const int tid = threadIdx.x;
  const float step0 = __hip_atomic_load(step_p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const int timeout = __hip_atomic_load(ext + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const int nonfin = __hip_atomic_load(ext + 7, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const float g0 = __hip_atomic_load(g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const bool ok = timeout == 0 && nonfin == 0 && isfinite(g0);
  const long n4 = n / 4;
  const long i = blockIdx.x * (long)blockDim.x + tid;
  int skipped = 0;
  if (i < n4) {
    float4 gg = reinterpret_cast<const float4*>(g)[i];
    if (ok) {
      float4 pp = reinterpret_cast<const float4*>(p)[i];
      float4 mm = reinterpret_cast<const float4*>(m)[i];
      float4 vv = reinterpret_cast<const float4*>(v)[i];
      const float step = step0 + 1.0f;
      const float alpha = *lr_p * sqrtf(1.0f - powf(b2, step)) / (1.0f - powf(b1, step));
#define GQ_ADAMF_LANE(c)                                          \
      if (isfinite(gg.c)) {                                       \
        const float gc = gg.c * gscale + wd * pp.c;               \
        mm.c = b1 * mm.c + (1.f - b1) * gc;                       \
        vv.c = b2 * vv.c + (1.f - b2) * gc * gc;                  \
        pp.c -= alpha * mm.c / (sqrtf(vv.c) + eps);               \
      } else {                                                    \
        ++skipped;                                                \
      }
      GQ_ADAMF_LANE(x) GQ_ADAMF_LANE(y) GQ_ADAMF_LANE(z) GQ_ADAMF_LANE(w)
#undef GQ_ADAMF_LANE
      reinterpret_cast<float4*>(p)[i] = pp;
      reinterpret_cast<float4*>(m)[i] = mm;
      reinterpret_cast<float4*>(v)[i] = vv;
    }
    // g[0] stays until the last arrival clears it (every workgroup reads it first): the first
    // float4's owner never stores lane x, so the last arrival's clear is the only write of g[0]
    // (a store of the old value here could land after that clear)
    if (i == 0) {
      g[1] = 0.f;
      g[2] = 0.f;
      g[3] = 0.f;
    } else {
      reinterpret_cast<float4*>(g)[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
  const long it = n4 * 4 + i;                    // (n % 4 tail: one element per thread at most)
  if (it < n) {
    const float gt = g[it];
    g[it] = 0.f;
    if (ok && isfinite(gt)) {
      const float step = step0 + 1.0f;
      const float alpha = *lr_p * sqrtf(1.0f - powf(b2, step)) / (1.0f - powf(b1, step));
      const float gc = gt * gscale + wd * p[it];
      m[it] = b1 * m[it] + (1.f - b1) * gc;
      v[it] = b2 * v[it] + (1.f - b2) * gc * gc;
      p[it] -= alpha * m[it] / (sqrtf(v[it]) + eps);
    } else if (ok) {
      ++skipped;
    }
  }
  if (skipped) atomicAdd(state + 5, skipped);
  __shared__ int last;
  // Every thread's reads of the flags / g[0] have returned (their values decided `ok` above), so a
  // plain s_barrier (no vmcnt drain of this workgroup's stores) and a relaxed ticket suffice: the
  // last arrival's clears cannot overtake a read that has completed. (An acq_rel ticket or
  // __syncthreads() here waited for every store of the update: ~6 us.)
  __builtin_amdgcn_s_barrier();
  if (tid == 0) last = __hip_atomic_fetch_add(state + 1, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                       (int)gridDim.x - 1;
  lds_barrier();
  if (!last || tid != 0) return;
  __hip_atomic_store(state + 1, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  g[0] = 0.f;
  if (ok) step_p[0] = step0 + 1.0f;
  else __hip_atomic_fetch_add(state + 3, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(state + 2, ok ? 1 : 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (timeout) {
    __hip_atomic_store(ext + 2, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_fetch_add(ext + 3, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (nonfin) __hip_atomic_store(ext + 7, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (cursor != nullptr) cursor[0] = (cursor[0] + 1) % cursor_mod;
}

void adam_flagged(at::Tensor p, at::Tensor g, at::Tensor m, at::Tensor v, const at::Tensor& lr, at::Tensor step,
                  double b1, double b2, double eps, double gscale, double wd, at::Tensor state, at::Tensor ext,
                  const c10::optional<at::Tensor>& cursor, int64_t cursor_mod) {
  const at::Tensor* ops[] = {&p, &g, &m, &v, &lr, &step};
  for (const at::Tensor* t : ops) check_f32_cuda(*t, "adam operand");
  TORCH_CHECK(state.is_cuda() && state.scalar_type() == at::kInt && state.numel() >= 6 && state.is_contiguous(),
              "adam_flagged: state must be int32[>=6] on the device");
  TORCH_CHECK(ext.is_cuda() && ext.scalar_type() == at::kInt && ext.numel() >= 8, "adam_flagged: ext int32[8]");
  const long n = p.numel();
  TORCH_CHECK(n >= 4 && g.numel() == n && m.numel() == n && v.numel() == n, "adam: size mismatch");
  TORCH_CHECK((reinterpret_cast<uintptr_t>(p.data_ptr()) % 16) == 0 && (reinterpret_cast<uintptr_t>(g.data_ptr()) % 16) == 0 &&
                  (reinterpret_cast<uintptr_t>(m.data_ptr()) % 16) == 0 && (reinterpret_cast<uintptr_t>(v.data_ptr()) % 16) == 0,
              "adam: buffers must be 16-byte aligned");
  long* cp = nullptr;
  if (cursor.has_value() && cursor->defined()) {
    TORCH_CHECK(cursor->is_cuda() && cursor->scalar_type() == at::kLong && cursor->numel() >= 1 && cursor_mod >= 1,
                "adam_flagged: cursor int64[1], cursor_mod >= 1");
    cp = cursor->data_ptr<int64_t>();
  }
  c10::DeviceGuard guard(p.device());
  const long work = std::max<long>(n / 4, n % 4);
  const int grid = (int)((work + 255) / 256);
  hipLaunchKernelGGL(adam_flagged_kernel, dim3(grid), dim3(256), 0, stream(), p.data_ptr<float>(), g.data_ptr<float>(),
                     m.data_ptr<float>(), v.data_ptr<float>(), lr.data_ptr<float>(), step.data_ptr<float>(), n,
                     (float)b1, (float)b2, (float)eps, (float)gscale, (float)wd, state.data_ptr<int>(),
                     ext.data_ptr<int>(), cp, cursor_mod);
  GQ_LAUNCH_CHECK();
}

at::Tensor nonfinite_count(const at::Tensor& x) {
  check_f32_cuda(x, "x");
  c10::DeviceGuard guard(x.device());
  at::Tensor out = at::zeros({1}, x.options().dtype(at::kInt));
  const long n = x.numel();
  const int grid = (int)std::max<long>(1, std::min<long>((n + 255) / 256, 1024));
  hipLaunchKernelGGL(nonfinite_kernel, dim3(grid), dim3(256), 0, stream(), x.data_ptr<float>(), n,
                     out.data_ptr<int>());
  GQ_LAUNCH_CHECK();
  return out;
}

// Data parallel: a chain spin timeout on ONE rank must reject the step on EVERY rank. Before the
// gradient all-reduce, a rank whose chain timed out (ext[2] != 0) writes NaN into g[0]; the SUM
// spreads it and every rank's guard skips the step (the local guard still counts the timeout).
// ext[7] (a gradient producer saw a non-finite value, adam_flagged) poisons the same way.
__global__ void chain_poison_kernel(float* __restrict__ g, const int* __restrict__ ext) {
  if (threadIdx.x == 0 && (__hip_atomic_load(ext + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0 ||
                           __hip_atomic_load(ext + 7, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0))
    g[0] = __builtin_nanf("");
}

void chain_poison(at::Tensor g, const at::Tensor& ext) {
  check_f32_cuda(g, "g");
  TORCH_CHECK(ext.is_cuda() && ext.scalar_type() == at::kInt && ext.numel() >= 8 && ext.get_device() == g.get_device(),
              "chain_poison: ext must be int32[8] on the gradient's device");
  TORCH_CHECK(g.numel() >= 1, "chain_poison: empty gradient buffer");
  c10::DeviceGuard guard(g.device());
  hipLaunchKernelGGL(chain_poison_kernel, dim3(1), dim3(64), 0, stream(), g.data_ptr<float>(), ext.data_ptr<int>());
  GQ_LAUNCH_CHECK();
}

}  // namespace gq

TORCH_LIBRARY_IMPL(gnnqc, CUDA, m) {
  m.impl("chain_poison", &gq::chain_poison);
  m.impl("adam_step", &gq::adam_step);
  m.impl("nonfinite_count", &gq::nonfinite_count);
  m.impl("grad_guard", &gq::grad_guard);
  m.impl("adam_guarded", &gq::adam_guarded);
  m.impl("adam_flagged", &gq::adam_flagged);
}
