// Device-side pieces of the fused CML GCN (gcn_fused.hip) shared with the LSTM weight-gradient
// launch (lstm_tm.hip lstm_grads_multi), which runs the GCN backward as extra workgroups: the two
// are independent (both only need the chain backward's outputs), and one launch of both overlaps
// them on the otherwise idle CUs instead of running them back to back.
#pragma once
#include "common.h"

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
  // the closed form of gcn_glue.hip gcn_bwd_finalize_kernel (training), applied to this partial
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

}  // namespace gq
