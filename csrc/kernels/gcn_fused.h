// Device-side pieces of the fused CML GCN (gcn_fused.hip) shared with the LSTM weight-gradient
// launch (lstm_tm.hip lstm_grads_multi), which runs the GCN backward as extra workgroups: the two
// are independent (both only need the chain backward's outputs), and one launch of both overlaps
// them on the otherwise idle CUs instead of running them back to back.
#pragma once
#include "common.h"

#include <vector>

namespace gq {

int* chain_ctl(int dev);   // lstm_chain.hip: word 7 = a gradient producer saw a non-finite value

constexpr int GF_MAX_CIN = 4;
constexpr int GF_ROW_MAX = 128;        // N * Cin floats per staged row
constexpr int GF_RPP = 64;             // rows per pass (4 threads per row, 256 threads)

struct GfData {                        // the resident window store (gnnqc.data.store.DeviceStore)
  const float* series;                 // [G][Ttot][N][C]
  const float* shift;                  // [G][Tn][N][C]
  const float* scale;
  const long* wg;                      // window -> group
  const long* wc;                      // window -> centre time index
  const uint8_t* wv;                   // [nwin][N] node valid
  const float* wlab;                   // [nwin] label
  const long* gap;                     // [G] flagged node position
  const double* mom;                   // [nwin][nstat] (gcn_window_prep)
  const float* pw;                     // [nwin][N]
  const long* wids;                    // [B] ids, or
  const long* table;                   // [nrows][B] + cursor
  const long* cursor;
  long nrows;
  int Ttot, Tn, N, tb, T, time_norm;
};

__device__ __forceinline__ const long* gf_ids(const GfData& D, int B) {
  return D.cursor != nullptr ? D.table + (D.cursor[0] % D.nrows) * B : D.wids;
}

// ---- step kernels. A workgroup owns `rows` consecutive steps of ONE sample's window. Every load
// of a pass is issued before the first wait (the slab of series values, the node tables, the
// parameters, the batch's moment records, the upstream gradient): one memory round trip after the
// id -> window chain, instead of one per dependent stage.
constexpr int GF_SLAB = 4096;          // floats of series staged per pass (16 per thread)
constexpr int GF_SPT = GF_SLAB / 256;

__device__ __forceinline__ int gf_rows_per_pass(int NC) { return min(GF_RPP, GF_SLAB / NC); }

// issue the loads of rows [t0, t0 + nr) of a window (contiguous NC floats per row) into registers
__device__ __forceinline__ void gf_slab_load(const float* __restrict__ src, int n, float (&v)[GF_SPT]) {
#pragma unroll
  for (int u = 0; u < GF_SPT; ++u) {
    const int i = threadIdx.x + 256 * u;
    v[u] = i < n ? src[i] : 0.f;
  }
}

// normalise the loaded values into sx[n] (element i: node (i % NC) / Cin, channel i % Cin)
template <int Cin>
__device__ __forceinline__ void gf_slab_park(const float (&v)[GF_SPT], int n, int NC, const float* svm,
                                             const float* ssh, const float* ssc, float* sx) {
  int e = threadIdx.x % NC;
  const int step = 256 % NC;
#pragma unroll
  for (int u = 0; u < GF_SPT; ++u) {
    const int i = threadIdx.x + 256 * u;
    if (i < n) sx[i] = (v[u] - ssh[e]) * ssc[e] * svm[e / Cin];
    e += step;
    if (e >= NC) e -= NC;
  }
}

// ---- backward (training): workgroup (bx, by) of the (B, ny) grid, 256 threads; parameter
// gradients added with float atomics
struct GcnBwdJob {
  GfData D;
  int B, Mp, Dh, c_off, rows, ny, key;             // key = Cin * 64 + F (lstm_grads_multi dispatch)
  const float* dh;
  const double* Sg;
  const float* st;
  const float* W;
  const float* bias;
  const float* alpha;
  float* dW;
  float* dgamma;
  float* dbeta;
  float* dalpha;
  int* nf;                                         // chain control word 7 (non-finite gradient)
};

// The closed form of gcn_glue.hip gcn_bwd_finalize_kernel (training) for feature f, applied to the
// raw partial sums tot = (A = sum dy, Z = sum dy z, P = sum da y[y <= 0], Q_k = sum x_k dy) of any
// subset of the rows (it is linear in them), added with float atomics; a non-finite contribution
// raises the step's non-finite flag (chain control word 7)
template <int Cin, int F>
__device__ __forceinline__ void gcn_bwd_apply(const float (&tot)[3 + Cin], int f, const double* __restrict__ Sg,
                                              const float* __restrict__ st, const float* __restrict__ W,
                                              const float* __restrict__ bias, float* dW, float* dgamma, float* dbeta,
                                              float* dalpha, int* nf) {
  const float mu = st[f], inv = st[F + f], scf = st[2 * F + f];
  const float A = tot[0], Z = tot[1], P = tot[2];
  const float dg = inv * (Z - mu * A);
  bool fin = isfinite(A) && isfinite(dg) && isfinite(P);
  atomicAdd(dbeta + f, A);
  atomicAdd(dgamma + f, dg);
  atomicAdd(dalpha + f, P);
  const double n = fmax(Sg[Cin + Cin * Cin], 1.0);
  const double bf = bias[f];
#pragma unroll
  for (int k = 0; k < Cin; ++k) {
    double s2w = 0.0;
#pragma unroll
    for (int l = 0; l < Cin; ++l) s2w += Sg[Cin + k * Cin + l] * (double)W[l * F + f];
    const double s1 = Sg[k];
    const double sxx = inv * (s2w + s1 * (bf - mu));
    const float d = (float)(scf * (tot[3 + k] - s1 * A / n - sxx * dg / n));
    fin = fin && isfinite(d);
    atomicAdd(dW + k * F + f, d);
  }
  if (!fin) __hip_atomic_store(nf, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ---- the backward coefficients (gcn_fused_fwd_kernel COEF) as a side job: one workgroup of
// blockDim.x threads (a multiple of 256) per sample row b of [0, Mp), all T steps, from the store and
// the BatchNorm statistics st [4][F] (mu, inv, scale, shift) the forward kernel wrote. Run by spare
// workgroups of the LSTM chain forward launch (its stages leave most CUs idle), or on its own.
struct GcnCoefFwdJob {
  GfData D;
  int B, Mp, on;
  const float* st;
  const float* W;
  const float* bias;
  const float* alpha;
  float* coef;                                     // [T][Mp][(3 + Cin) F]
};

constexpr int GCF_LDS_FLOATS = 16384;              // staged slab (64 KB): rows per pass = this / (N Cin)

struct GcnCoefFwdLds {
  static constexpr int BYTES = (GCF_LDS_FLOATS + 4 * GF_ROW_MAX) * 4;
};

// ---- the whole training-step forward as PRODUCER workgroups of the LSTM chain forward launch
// (lstm_chain.hip): one workgroup (blockDim.x threads, a multiple of 256, F / 4 threads per row) per
// sample row b of [0, Mp), all T steps. The arithmetic of gcn_fused_fwd_kernel (the batch's moment
// records summed in one fixed order - the same in every workgroup -, the BatchNorm prep, the
// node-pooled PReLU output, the flagged series) plus, when coef != nullptr, the backward
// coefficients of gcn_coef_fwd_body. Each time-major input row goes to `out` (fp32, read by the
// backward) and, when gout != nullptr, to the tagged granule stream gout ({value, tag | t} per
// element), which the chain's first stage streams like a stage-to-stage hand-off: it starts on the
// first steps while later rows are still being produced, instead of after a separate forward
// launch and its tail. y / y_mask / wid leave through agent-scope stores and the workgroup then
// counts itself in *done (the chain's head waits for every producer before it reads the labels).
struct GcnProdJob {
  GfData D;
  int B, Mp, Cp, on;
  const float* W;
  const float* bias;
  const float* gamma;
  const float* beta;
  const float* alpha;
  float* rmean;
  float* rvar;
  float momentum, eps;
  float* out;                                      // [T][Mp][Cp]
  unsigned long long* gout;                        // [T][Mp][Cp] tagged granules (nullptr: none)
  double* Sout;                                    // [nstat]
  float* st;                                       // [4][F]: mu, inv, scale, shift
  float* y;                                        // [B]
  float* ym;                                       // [B]
  long* wid;                                       // [B]
  float* coef;                                     // [T][Mp][(3 + Cin) F] (nullptr: none)
};

struct GcnProdLds {
  static constexpr int PRM = (GF_MAX_CIN + 2) * 32;   // floats: W', b', alpha per feature
  static constexpr int BYTES = (GCF_LDS_FLOATS + 4 * GF_ROW_MAX + PRM) * 4 + 17 * 32 * 8;
};

__device__ __forceinline__ void gf_st_granule(unsigned long long* p, float v, unsigned tag) {
  __hip_atomic_store(p, ((unsigned long long)tag << 32) | __float_as_uint(v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}

template <int Cin, int F>
__device__ __forceinline__ void gcn_prod_body(const GcnProdJob& J, int b, unsigned tagb, int* done, char* smem,
                                              long long* mark = nullptr) {
  constexpr int NA = 3 + Cin, nstat = Cin + Cin * Cin + 1, QPR = F / 4;
  constexpr int SPT = 12;                                              // staged floats per thread and pass
  static_assert(F % 4 == 0 && (Cin + 2) * F <= GcnProdLds::PRM && nstat <= 32, "producer layout");
  const GfData& D = J.D;
  const int tid = threadIdx.x, nthr = blockDim.x, N = D.N, T = D.T, NC = N * Cin;
  const int lane = tid & 63, wv = tid >> 6, nwv = nthr >> 6;
  float* sx = reinterpret_cast<float*>(smem);                         // [GCF_LDS_FLOATS]
  float* svm = sx + GCF_LDS_FLOATS;                                    // [GF_ROW_MAX] x 4
  float* spw = svm + GF_ROW_MAX;
  float* ssh = spw + GF_ROW_MAX;
  float* ssc = ssh + GF_ROW_MAX;
  float* prm = ssc + GF_ROW_MAX;                                       // [Cin + 2][F]
  double* dred = reinterpret_cast<double*>(prm + GcnProdLds::PRM);     // [16][32] + S [32]
  double* S = dred + 16 * 32;
  const long* ids = gf_ids(D, J.B);
  const long wraw = b < J.B ? ids[b] : -1;
  const bool live = wraw >= 0;
  const long w = live ? wraw : 0;
  const long g = D.wg[w], c0 = D.wc[w];
  const long tn = D.time_norm ? c0 : 0;
  const float* src = D.series + (g * D.Ttot + (c0 - D.tb)) * (long)NC;
  // thread -> (row lane rl, feature quad fq); rows per pass: the LDS slab, the row lanes and the
  // register staging (SPT floats per thread) all hold them
  const int fq = tid % QPR, rl = tid / QPR, rlanes = nthr / QPR;
  const int RP = max(1, min(min(GCF_LDS_FLOATS, SPT * nthr) / NC, rlanes));
  // ---- phase A: every load before the first wait (the first pass's series slab, the node tables,
  // the parameters, the batch's moment records): one memory round trip after id -> window
  float v[SPT];
  auto load_slab = [&](int p0, int n) {
#pragma unroll
    for (int u = 0; u < SPT; ++u) {
      const int i = tid + nthr * u;
      v[u] = live && i < n ? src[(long)p0 * NC + i] : 0.f;
    }
  };
  load_slab(0, min(RP, T) * NC);
  float pv[Cin + 6];
  if (tid < F) {
#pragma unroll
    for (int k = 0; k < Cin; ++k) pv[k] = J.W[k * F + tid];
    pv[Cin] = J.bias[tid];
    pv[Cin + 1] = J.gamma[tid];
    pv[Cin + 2] = J.beta[tid];
    pv[Cin + 3] = J.alpha[tid];
    pv[Cin + 4] = J.rmean[tid];
    pv[Cin + 5] = J.rvar[tid];
  }
  float nv = 0.f, npw = 0.f, nsh = 0.f, nsc = 0.f;
  if (tid < N) {
    nv = live && D.wv[w * N + tid] ? 1.f : 0.f;
    npw = live ? D.pw[w * N + tid] : 0.f;
  }
  if (tid < NC) {
    nsh = D.shift[(g * D.Tn + tn) * (long)NC + tid];
    nsc = D.scale[(g * D.Tn + tn) * (long)NC + tid];
  }
  double mv[nstat];
#pragma unroll
  for (int i = 0; i < nstat; ++i) mv[i] = 0.0;
  for (int k = tid; k < J.B; k += nthr) {          // the batch's moments: B window records
    const long wk = ids[k];
    if (wk >= 0) {
#pragma unroll
      for (int i = 0; i < nstat; ++i) mv[i] += D.mom[wk * nstat + i];
    }
  }
  // ---- phase B
  if (tid < N) {
    svm[tid] = nv;
    spw[tid] = npw;
  }
  if (tid < NC) {
    ssh[tid] = nsh;
    ssc[tid] = nsc;
  }
#pragma unroll
  for (int i = 0; i < nstat; ++i) {
    double sv = mv[i];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) sv += __shfl_xor(sv, o, 64);
    if (lane == 0) dred[wv * 32 + i] = sv;
  }
  __syncthreads();
  if (mark != nullptr && tid == 0) mark[0] = (long long)__builtin_amdgcn_s_memrealtime();
  if (tid < nstat) {                               // fixed order: identical in every workgroup
    double sv = 0.0;
    for (int k = 0; k < nwv; ++k) sv += dred[k * 32 + tid];
    S[tid] = sv;
  }
  auto park = [&](int n) {                         // normalise the staged values into sx
#pragma unroll
    for (int u = 0; u < SPT; ++u) {
      const int i = tid + nthr * u;
      if (i < n) {
        const int e = i % NC;
        sx[i] = (v[u] - ssh[e]) * ssc[e] * svm[e / Cin];
      }
    }
  };
  park(min(RP, T) * NC);
  __syncthreads();
  if (tid < F) {                                   // BatchNorm (training statistics) folded into W', b'
    const double cnt = fmax(S[Cin + Cin * Cin], 1.0);
    double ex[Cin];
#pragma unroll
    for (int k = 0; k < Cin; ++k) ex[k] = S[k] / cnt;
    double m = pv[Cin], vv = 0.0;
#pragma unroll
    for (int k = 0; k < Cin; ++k) {
      m += ex[k] * (double)pv[k];
#pragma unroll
      for (int l = 0; l < Cin; ++l) vv += (double)pv[k] * (S[Cin + k * Cin + l] / cnt - ex[k] * ex[l]) * (double)pv[l];
    }
    const float mu = (float)m, var = (float)fmax(vv, 0.0);
    const float inv = rsqrtf(var + J.eps);
    const float sc = pv[Cin + 1] * inv;
    const float sh = pv[Cin + 2] - mu * sc;
#pragma unroll
    for (int k = 0; k < Cin; ++k) prm[k * F + tid] = pv[k] * sc;
    prm[Cin * F + tid] = pv[Cin] * sc + sh;
    prm[(Cin + 1) * F + tid] = pv[Cin + 3];
    if (b == 0) {
      J.st[tid] = mu;
      J.st[F + tid] = inv;
      J.st[2 * F + tid] = sc;
      J.st[3 * F + tid] = sh;
      J.rmean[tid] = pv[Cin + 4] * J.momentum + mu * (1.f - J.momentum);
      J.rvar[tid] = pv[Cin + 5] * J.momentum + var * (1.f - J.momentum);
    }
  }
  if (b == 0 && tid < nstat) J.Sout[tid] = S[tid];
  __syncthreads();
  if (mark != nullptr && tid == 0) mark[1] = (long long)__builtin_amdgcn_s_memrealtime();
  float pwk[Cin][4], pb[4], pal[4], rwk[Cin][4], rb[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int f = 4 * fq + j;
#pragma unroll
    for (int k = 0; k < Cin; ++k) {
      pwk[k][j] = prm[k * F + f];
      rwk[k][j] = J.W[k * F + f];
    }
    pb[j] = prm[Cin * F + f];
    pal[j] = prm[(Cin + 1) * F + f];
    rb[j] = J.bias[f];
  }
  const long apl = D.gap[g];
  const int ap = apl < 0 ? 0 : (int)apl;
  for (int p0 = 0; p0 < T; p0 += RP) {
    const int nr = min(RP, T - p0);
    if (p0 > 0) {                                  // (more rows than one pass: stage the next slab)
      load_slab(p0, nr * NC);
      __syncthreads();                             // previous pass's LDS reads are done
      park(nr * NC);
      __syncthreads();
    }
    // the pooled outputs first (the chain's first stage streams them), the coefficients after
    for (int rr = rl; rr < nr; rr += rlanes) {
      const int t = p0 + rr;
      float acc[4] = {0.f, 0.f, 0.f, 0.f};
      const float* xr = sx + rr * NC;
      for (int n = 0; n < N; ++n) {
        const float wn = spw[n];
        float xv[Cin];
#pragma unroll
        for (int k = 0; k < Cin; ++k) xv[k] = xr[n * Cin + k];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          float yv = pb[j];
#pragma unroll
          for (int k = 0; k < Cin; ++k) yv += xv[k] * pwk[k][j];
          acc[j] += wn * (yv > 0.f ? yv : pal[j] * yv);
        }
      }
      const long ro = ((long)t * J.Mp + b) * J.Cp;
      if (J.gout != nullptr) {
        const unsigned tag = tagb | (unsigned)t;
#pragma unroll
        for (int j = 0; j < 4; ++j) gf_st_granule(J.gout + ro + Cin + 4 * fq + j, acc[j], tag);
        if (fq == 0)
#pragma unroll
          for (int k = 0; k < Cin; ++k) gf_st_granule(J.gout + ro + k, xr[ap * Cin + k], tag);
        for (int c = Cin + F + fq; c < J.Cp; c += QPR) gf_st_granule(J.gout + ro + c, 0.f, tag);
      }
      float* o = J.out + ro;
      *reinterpret_cast<float4*>(o + Cin + 4 * fq) = make_float4(acc[0], acc[1], acc[2], acc[3]);
      if (fq == 0)
#pragma unroll
        for (int k = 0; k < Cin; ++k) o[k] = xr[ap * Cin + k];
      for (int c = Cin + F + fq; c < J.Cp; c += QPR) o[c] = 0.f;
    }
    if (mark != nullptr && p0 == 0 && tid == 0) mark[2] = (long long)__builtin_amdgcn_s_memrealtime();
    if (J.coef != nullptr)
      for (int rr = rl; rr < nr; rr += rlanes) {
        const int t = p0 + rr;
        float cf[NA][4];
#pragma unroll
        for (int a = 0; a < NA; ++a)
#pragma unroll
          for (int j = 0; j < 4; ++j) cf[a][j] = 0.f;
        const float* xr = sx + rr * NC;
        for (int n = 0; n < N; ++n) {
          const float wn = spw[n];
          float xv[Cin];
#pragma unroll
          for (int k = 0; k < Cin; ++k) xv[k] = xr[n * Cin + k];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            float yv = pb[j], z = rb[j];
#pragma unroll
            for (int k = 0; k < Cin; ++k) {
              yv += xv[k] * pwk[k][j];
              z += xv[k] * rwk[k][j];
            }
            const bool pos = yv > 0.f;
            const float dp = pos ? wn : pal[j] * wn;
            cf[0][j] += dp;
            cf[1][j] += dp * z;
            cf[2][j] += pos ? 0.f : wn * yv;
#pragma unroll
            for (int k = 0; k < Cin; ++k) cf[3 + k][j] += dp * xv[k];
          }
        }
        float* co = J.coef + ((long)t * J.Mp + b) * (NA * F) + 4 * fq;
#pragma unroll
        for (int a = 0; a < NA; ++a)
          *reinterpret_cast<float4*>(co + a * F) = make_float4(cf[a][0], cf[a][1], cf[a][2], cf[a][3]);
      }
  }
  // ---- the labels (agent scope), then this workgroup's arrival (the chain's head waits for all)
  if (tid == 0 && b < J.B) {
    __hip_atomic_store(reinterpret_cast<unsigned*>(J.y + b), __float_as_uint(live ? D.wlab[w] : 0.f),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(reinterpret_cast<unsigned*>(J.ym + b), __float_as_uint(live ? 1.f : 0.f), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(reinterpret_cast<unsigned long long*>(J.wid + b), (unsigned long long)wraw, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  }
  if (tid == 0 && done != nullptr) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // (the label stores are acknowledged)
    __hip_atomic_fetch_add(done, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// host: jobs left by gcn_fused_fwd for the next chain forward launch (gcn_fused.hip): the
// coefficient side job, or the whole forward as producer workgroups (prod)
struct GcnPending {
  GcnCoefFwdJob job;
  std::vector<at::Tensor> keep;
  GcnProdJob prod;
  std::vector<at::Tensor> pkeep;
};
bool gcn_coef_side_mode();
GcnPending& gcn_pending(int dev);
bool gcn_coef_take(int dev, GcnCoefFwdJob& job, std::vector<at::Tensor>& keep);
bool gcn_coef_flush_dev(int dev);
bool gcn_prod_take(int dev, GcnProdJob& job, std::vector<at::Tensor>& keep);
bool gcn_prod_flush_dev(int dev);

template <int Cin, int F>
__device__ __forceinline__ void gcn_coef_fwd_body(const GcnCoefFwdJob& J, int b, char* smem) {
  constexpr int NA = 3 + Cin;
  static_assert(F % 4 == 0, "feature quads");
  const GfData& D = J.D;
  const int tid = threadIdx.x, nthr = blockDim.x, N = D.N, T = D.T, NC = N * Cin;
  float* sx = reinterpret_cast<float*>(smem);                       // [GCF_LDS_FLOATS]
  float* svm = sx + GCF_LDS_FLOATS;                                  // [GF_ROW_MAX] x 4
  float* spw = svm + GF_ROW_MAX;
  float* ssh = spw + GF_ROW_MAX;
  float* ssc = ssh + GF_ROW_MAX;
  const long wraw = b < J.B ? gf_ids(D, J.B)[b] : -1;
  if (wraw < 0) {                                   // padding sample / row: zero coefficients
    for (long i = tid; i < (long)T * NA * F; i += nthr) {
      const long t = i / (NA * F);
      J.coef[(t * J.Mp + b) * (NA * F) + i % (NA * F)] = 0.f;
    }
    return;
  }
  const long w = wraw, g = D.wg[w], c0 = D.wc[w];
  const long tn = D.time_norm ? c0 : 0;
  if (tid < N) {
    svm[tid] = D.wv[w * N + tid] ? 1.f : 0.f;
    spw[tid] = D.pw[w * N + tid];
  }
  if (tid < NC) {
    ssh[tid] = D.shift[(g * D.Tn + tn) * (long)NC + tid];
    ssc[tid] = D.scale[(g * D.Tn + tn) * (long)NC + tid];
  }
  // thread -> (row lane rl, feature quad fq): F / 4 quads per row
  constexpr int QPR = F / 4;
  const int fq = tid % QPR, rl = tid / QPR, rlanes = nthr / QPR;
  float rw[Cin][4], rb[4], scv[4], shv[4], al[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int f = 4 * fq + j;
#pragma unroll
    for (int k = 0; k < Cin; ++k) rw[k][j] = J.W[k * F + f];
    rb[j] = J.bias[f];
    scv[j] = J.st[2 * F + f];
    shv[j] = J.st[3 * F + f];
    al[j] = J.alpha[f];
  }
  const float* src = D.series + (g * D.Ttot + (c0 - D.tb)) * (long)NC;
  const int RP = max(1, min(GCF_LDS_FLOATS / NC, rlanes));
  __syncthreads();
  for (int p0 = 0; p0 < T; p0 += RP) {
    const int nr = min(RP, T - p0);
    if (p0 > 0) __syncthreads();                  // previous pass's LDS reads are done
    for (int i = tid; i < nr * NC; i += nthr) {
      const int e = i % NC;
      sx[i] = (src[(long)p0 * NC + i] - ssh[e]) * ssc[e] * svm[e / Cin];
    }
    __syncthreads();
    for (int rr = rl; rr < nr; rr += rlanes) {
      float cf[NA][4];
#pragma unroll
      for (int a = 0; a < NA; ++a)
#pragma unroll
        for (int j = 0; j < 4; ++j) cf[a][j] = 0.f;
      const float* xr = sx + rr * NC;
      for (int n = 0; n < N; ++n) {
        const float wn = spw[n];
        float xv[Cin];
#pragma unroll
        for (int k = 0; k < Cin; ++k) xv[k] = xr[n * Cin + k];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          float z = rb[j];
#pragma unroll
          for (int k = 0; k < Cin; ++k) z += xv[k] * rw[k][j];
          const float yv = z * scv[j] + shv[j];
          const bool pos = yv > 0.f;
          const float dp = pos ? wn : al[j] * wn;
          cf[0][j] += dp;
          cf[1][j] += dp * z;
          cf[2][j] += pos ? 0.f : wn * yv;
#pragma unroll
          for (int k = 0; k < Cin; ++k) cf[3 + k][j] += dp * xv[k];
        }
      }
      float* co = J.coef + ((long)(p0 + rr) * J.Mp + b) * (NA * F) + 4 * fq;
#pragma unroll
      for (int a = 0; a < NA; ++a)
        *reinterpret_cast<float4*>(co + a * F) = make_float4(cf[a][0], cf[a][1], cf[a][2], cf[a][3]);
    }
  }
}

template <int Cin, int F>
struct GcnBwdLds {
  static constexpr int BYTES = (4 * GF_ROW_MAX + GF_SLAB + 4 * (3 + Cin) * F) * 4;
};

// smem: GcnBwdLds<Cin, F>::BYTES of LDS, 16-byte aligned (the caller's buffer: a kernel that
// holds several instantiations reserves the largest one, not their sum)
template <int Cin, int F>
__device__ __forceinline__ void gcn_fused_bwd_body(const GcnBwdJob J, int bx, int by, char* smem) {
  constexpr int FQ = F / 4;
  constexpr int NA = 3 + Cin;
  const GfData& D = J.D;
  const int B = J.B, Mp = J.Mp, Dh = J.Dh, c_off = J.c_off, rows = J.rows;
  const float* __restrict__ dh = J.dh;
  const double* __restrict__ Sg = J.Sg;
  const float* __restrict__ st = J.st;
  const float* __restrict__ W = J.W;
  const float* __restrict__ bias = J.bias;
  const float* __restrict__ alpha = J.alpha;
  float* __restrict__ dW = J.dW;
  float* __restrict__ dgamma = J.dgamma;
  float* __restrict__ dbeta = J.dbeta;
  float* __restrict__ dalpha = J.dalpha;
  int* __restrict__ nf = J.nf;
  const int b = bx, tid = threadIdx.x, N = D.N, T = D.T;
  const int t0 = by * rows, t1 = min(T, t0 + rows);
  float* sx = reinterpret_cast<float*>(smem);                       // [GF_SLAB]
  float* svm = sx + GF_SLAB;                                          // [GF_ROW_MAX] x 4
  float* spw = svm + GF_ROW_MAX;
  float* ssh = spw + GF_ROW_MAX;
  float* ssc = ssh + GF_ROW_MAX;
  auto red = reinterpret_cast<float (*)[NA][F]>(ssc + GF_ROW_MAX);   // [4][NA][F]
  const int NC = N * Cin;
  const int RP = gf_rows_per_pass(NC);
  const int r = tid >> 2, q = tid & 3, f0 = q * FQ;
  // ---- phase A: all loads (the upstream gradient and the parameters do not depend on the ids)
  float gv[FQ];
  {
    const int t = t0 + r;
    const float* dr = dh + ((long)min(t, T - 1) * Mp + b) * Dh + c_off + f0;
#pragma unroll
    for (int j = 0; j < FQ; ++j) gv[j] = (r < min(RP, t1 - t0)) ? dr[j] : 0.f;
  }
  float wk[Cin][FQ], bb[FQ], sc[FQ], sh[FQ], al[FQ];
#pragma unroll
  for (int j = 0; j < FQ; ++j) {
    const int f = f0 + j;
#pragma unroll
    for (int k = 0; k < Cin; ++k) wk[k][j] = W[k * F + f];
    bb[j] = bias[f];
    sc[j] = st[2 * F + f];
    sh[j] = st[3 * F + f];
    al[j] = alpha[f];
  }
  const long* ids = gf_ids(D, B);
  const long wraw = ids[b];
  if (wraw < 0) return;                           // padding sample: no contribution (uniform exit)
  const long w = wraw;
  const long g = D.wg[w], c0 = D.wc[w];
  const long tn = D.time_norm ? c0 : 0;
  float nv = 0.f, npw = 0.f, nsh = 0.f, nsc = 0.f;
  if (tid < N) {
    nv = D.wv[w * N + tid] ? 1.f : 0.f;
    npw = D.pw[w * N + tid];
  }
  if (tid < NC) {
    nsh = D.shift[(g * D.Tn + tn) * (long)NC + tid];
    nsc = D.scale[(g * D.Tn + tn) * (long)NC + tid];
  }
  float v[GF_SPT];
  const float* src = D.series + (g * D.Ttot + (c0 - D.tb)) * (long)NC;
  int nr = min(RP, t1 - t0);
  gf_slab_load(src + (long)t0 * NC, nr * NC, v);
  // ---- phase B
  if (tid < N) {
    svm[tid] = nv;
    spw[tid] = npw;
  }
  if (tid < NC) {
    ssh[tid] = nsh;
    ssc[tid] = nsc;
  }
  __syncthreads();
  gf_slab_park<Cin>(v, nr * NC, NC, svm, ssh, ssc, sx);
  __syncthreads();
  float acc[NA][FQ];
#pragma unroll
  for (int a = 0; a < NA; ++a)
#pragma unroll
    for (int j = 0; j < FQ; ++j) acc[a][j] = 0.f;
  for (int p0 = t0; p0 < t1; p0 += RP) {
    if (p0 != t0) {
      nr = min(RP, t1 - p0);
      gf_slab_load(src + (long)p0 * NC, nr * NC, v);
      __syncthreads();
      gf_slab_park<Cin>(v, nr * NC, NC, svm, ssh, ssc, sx);
      __syncthreads();
      if (r < nr) {
        const float* dr = dh + ((long)(p0 + r) * Mp + b) * Dh + c_off + f0;
#pragma unroll
        for (int j = 0; j < FQ; ++j) gv[j] = dr[j];
      }
    }
    if (r < nr) {
      const float* xr = sx + r * NC;
      for (int n = 0; n < N; ++n) {
        const float wn = spw[n];                  // 0 for masked / unpooled nodes: no contribution
        float xv[Cin];
#pragma unroll
        for (int k = 0; k < Cin; ++k) xv[k] = xr[n * Cin + k];
#pragma unroll
        for (int j = 0; j < FQ; ++j) {
          float z = bb[j];
#pragma unroll
          for (int k = 0; k < Cin; ++k) z += xv[k] * wk[k][j];
          const float yv = z * sc[j] + sh[j];
          const float da = wn * gv[j];
          const bool pos = yv > 0.f;
          const float dy = pos ? da : al[j] * da;
          acc[0][j] += dy;
          acc[1][j] += dy * z;
          acc[2][j] += pos ? 0.f : da * yv;
#pragma unroll
          for (int k = 0; k < Cin; ++k) acc[3 + k][j] += xv[k] * dy;
        }
      }
    }
  }
  // reduce over the workgroup's rows: lanes with equal q (stride 4) inside the wave, then 4 waves
  const int lane = tid & 63, wv = tid >> 6;
#pragma unroll
  for (int a = 0; a < NA; ++a)
#pragma unroll
    for (int j = 0; j < FQ; ++j) {
      float x = acc[a][j];
#pragma unroll
      for (int o = 32; o >= 4; o >>= 1) x += __shfl_xor(x, o, 64);
      if (lane < 4) red[wv][a][lane * FQ + j] = x;
    }
  __syncthreads();
  if (tid >= F) return;
  const int f = tid;
  float tot[NA];
#pragma unroll
  for (int a = 0; a < NA; ++a) tot[a] = (red[0][a][f] + red[1][a][f]) + (red[2][a][f] + red[3][a][f]);
  gcn_bwd_apply<Cin, F>(tot, f, Sg, st, W, bias, dW, dgamma, dbeta, dalpha, nf);
}

// ---- backward from the forward's coefficients (gcn_fused_fwd_kernel COEF): the partial sums are
// sum over rows of dh[row][c_off + f] * coef[row][a][f], a streaming dot product over [T * Mp] rows.
// Workgroup bx of nblocks (256 threads: 16 rows x 16 features per pass, F = 16) sums its row range
// and adds the closed form of its partial with float atomics.
struct GcnCoefJob {
  const float* dh;                                 // [>= T][Mp][Dh]
  const float* coef;                               // [T][Mp][(3 + Cin) F]
  long rows;                                       // T * Mp
  int Dh, c_off, nblocks, key;                     // key = Cin * 64 + F
  const double* Sg;
  const float* st;
  const float* W;
  const float* bias;
  float* dW;
  float* dgamma;
  float* dbeta;
  float* dalpha;
  int* nf;
};

template <int Cin, int F>
__device__ __forceinline__ void gcn_coef_bwd_body(const GcnCoefJob& J, int bx) {
  constexpr int NA = 3 + Cin, RPP = 256 / F;
  static_assert(256 % F == 0 && F <= 64 && 64 % F == 0, "rows per pass");
  __shared__ float red[4][NA][F];
  const int tid = threadIdx.x, f = tid % F, rl = tid / F;
  const long per = (J.rows + J.nblocks - 1) / J.nblocks;
  const long r0 = (long)bx * per, r1 = min(J.rows, r0 + per);
  float acc[NA];
#pragma unroll
  for (int a = 0; a < NA; ++a) acc[a] = 0.f;
  long r = r0 + rl;
  for (; r + 3 * RPP < r1; r += 4 * RPP) {         // four rows in flight per thread
    float g[4], c[4][NA];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const long ru = r + u * RPP;
      g[u] = J.dh[ru * J.Dh + J.c_off + f];
#pragma unroll
      for (int a = 0; a < NA; ++a) c[u][a] = J.coef[ru * (NA * F) + a * F + f];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int a = 0; a < NA; ++a) acc[a] += g[u] * c[u][a];
  }
  for (; r < r1; r += RPP) {
    const float g = J.dh[r * J.Dh + J.c_off + f];
#pragma unroll
    for (int a = 0; a < NA; ++a) acc[a] += g * J.coef[r * (NA * F) + a * F + f];
  }
  const int lane = tid & 63, wv = tid >> 6;
#pragma unroll
  for (int a = 0; a < NA; ++a) {
    float x = acc[a];
#pragma unroll
    for (int o = 32; o >= F; o >>= 1) x += __shfl_xor(x, o, 64);
    if (lane < F) red[wv][a][lane] = x;
  }
  __syncthreads();
  if (tid >= F) return;
  float tot[NA];
#pragma unroll
  for (int a = 0; a < NA; ++a) tot[a] = (red[0][a][f] + red[1][a][f]) + (red[2][a][f] + red[3][a][f]);
  gcn_bwd_apply<Cin, F>(tot, f, J.Sg, J.st, J.W, J.bias, J.dW, J.dgamma, J.dbeta, J.dalpha, J.nf);
}

}  // namespace gq
