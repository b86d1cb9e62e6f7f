// Training-step GeneralConv + BatchNorm + PReLU + node pooling, fused with the window gather
// (SURVEY §2.2 K1 + K2 + K12; reference: spektral GeneralConv at libs/create_model.py:184-189,
// timeseries_pooling :8-41, Concatenate :223, the window parse libs/preprocessing_functions.py:566-666).
//
// The generic path is three launches before the LSTM chain: batch_gather (cut + normalise the
// windows into x [B,T,N,C]), gcn_prep (per-sample pooling weights + fp64 moments of x, the last
// workgroup sums them and preps BatchNorm) and gcn_pool_fwd (x -> the time-major LSTM input).
// Everything gcn_prep computes per sample depends only on the WINDOW (its normalised series, its
// node mask, its group's adjacency), not on the model, so it is computed once per store
// (gcn_window_prep: moments [nwin][nstat] fp64 + pooling weights [nwin][N]). A training step then
// needs ONE launch: every workgroup sums the batch's B moment records in a fixed order (the same
// order in every workgroup: identical, deterministic statistics, no cross-workgroup hand-off),
// preps BatchNorm for itself, cuts its rows of ONE window straight from the resident series into
// LDS and writes the time-major LSTM input [T][Mp][Cp] = [flagged series | pooled | 0 pad].
// Workgroup (0, 0) also writes S / st for the backward and applies the Keras running-stat update.
//
// Backward (gcn_fused_bwd): the closed-form BatchNorm/PReLU/pooling parameter gradient is LINEAR
// in the per-row partial sums (A = sum dy, Z = sum dy z, P = sum da y[y<=0], Q_k = sum x_k dy), so
// every workgroup maps its own partial sums to dW, dgamma, dbeta, dalpha contributions and adds them
// with float atomics: no partial-record workspace and no finalize launch (not bitwise
// reproducible: the deterministic mode keeps the generic path).
#include "gcn_fused.h"

namespace gq {

// ---- per-window precompute: one workgroup per window
template <int Cin>
__global__ __launch_bounds__(256) void gcn_window_prep_kernel(GfData D, const float* __restrict__ gadj,
                                                              int agg_mean, int pool, int nwin,
                                                              double* __restrict__ mom, float* __restrict__ pw) {
  constexpr int nstat = Cin + Cin * Cin + 1;
  const int w = blockIdx.x, tid = threadIdx.x, N = D.N;
  extern __shared__ float sh_[];      // vm [N], coef [N]
  float* svm = sh_;
  float* coef = sh_ + N;
  __shared__ float red[4];
  __shared__ double dred[4][nstat];
  const long g = D.wg[w];
  for (int n = tid; n < N; n += 256) svm[n] = D.wv[(long)w * N + n] ? 1.f : 0.f;
  __syncthreads();
  // pooling weights (gcn_glue.hip gcn_prep_kernel, on the masked group adjacency)
  const float* A = gadj + g * (long)N * N;
  float ms = 0.f;
  for (int i = tid; i < N; i += 256) ms += svm[i];
  ms = wave_sum(ms);
  if ((tid & 63) == 0) red[tid >> 6] = ms;
  __syncthreads();
  ms = red[0] + red[1] + red[2] + red[3];
  const long ap = D.gap[g];
  for (int i = tid; i < N; i += 256) {
    float p;
    if (pool == 0) p = svm[i] / fmaxf(ms, 1.f);
    else if (pool == 1) p = svm[i];
    else p = (i == (ap < 0 ? 0 : ap)) ? 1.f : 0.f;
    float c = p;
    if (agg_mean && p != 0.f) {
      float deg = 0.f;
      for (int j = 0; j < N; ++j) deg += A[(long)i * N + j] * svm[i] * svm[j];
      c = p / fmaxf(deg, 1.f);
    }
    coef[i] = c;
  }
  __syncthreads();
  for (int j = tid; j < N; j += 256) {
    float s = 0.f;
    for (int i = 0; i < N; ++i) s += coef[i] * (A[(long)i * N + j] * svm[i] * svm[j]);
    pw[(long)w * N + j] = s;
  }
  // fp64 moments of the window's normalised values over its T x N rows (masked rows: zeros)
  const int NC = N * Cin;
  const long c0 = D.wc[w];
  const float* src = D.series + (g * D.Ttot + (c0 - D.tb)) * (long)NC;
  const long tn = D.time_norm ? c0 : 0;
  const float* shp = D.shift + (g * D.Tn + tn) * (long)NC;
  const float* scp = D.scale + (g * D.Tn + tn) * (long)NC;
  double acc[nstat];
#pragma unroll
  for (int i = 0; i < nstat; ++i) acc[i] = 0.0;
  const int R = D.T * N;
  for (int r = tid; r < R; r += 256) {
    const int n = r % N;
    const float m = svm[n];
    float xv[Cin];
#pragma unroll
    for (int k = 0; k < Cin; ++k) {
      const int e = n * Cin + k;
      xv[k] = (src[(long)r * Cin + k] - shp[e]) * scp[e] * m;
    }
#pragma unroll
    for (int k = 0; k < Cin; ++k) {
      const float mx = m * xv[k];
      acc[k] += mx;
#pragma unroll
      for (int l = 0; l < Cin; ++l) acc[Cin + k * Cin + l] += (double)mx * xv[l];
    }
    acc[nstat - 1] += m;
  }
  const int lane = tid & 63, wv = tid >> 6;
#pragma unroll
  for (int i = 0; i < nstat; ++i) {
    double v = acc[i];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if (lane == 0) dred[wv][i] = v;
  }
  __syncthreads();
  if (tid < nstat) mom[(long)w * nstat + tid] = (dred[0][tid] + dred[1][tid]) + (dred[2][tid] + dred[3][tid]);
}

// ---- forward: grid (Mp, NY), 256 threads
// COEF (training): also the backward coefficients of every (t, sample, feature f), written to
// coef [T][Mp][NA][F] (NA = 3 + Cin), with dpos_n = w_n (y_nf > 0 ? 1 : alpha_f) over the nodes n:
//   c0 = sum dpos_n, c1 = sum dpos_n z_nf, c2 = sum_{y_nf <= 0} w_n y_nf, c3+k = sum dpos_n x_nk
// (z = x W + b before BatchNorm, y after it). The parameter gradient's partial sums of
// gcn_fused_bwd_body are these times the pooled channel's upstream gradient dh[t][b][f], so the
// backward becomes a streaming dot product (gcn_coef_bwd_body) with no window gather, slab staging
// or per-node recompute behind the LSTM backward.
template <int Cin, int F, bool COEF>
__global__ __launch_bounds__(256) void gcn_fused_fwd_kernel(
    GfData D, int B, int Mp, int Cp, int rows, const float* __restrict__ W, const float* __restrict__ bias,
    const float* __restrict__ gamma, const float* __restrict__ beta, const float* __restrict__ alpha,
    float* __restrict__ rmean, float* __restrict__ rvar, int training, float momentum, float eps,
    float* __restrict__ out, double* __restrict__ Sout, float* __restrict__ st, float* __restrict__ y,
    float* __restrict__ ym, long* __restrict__ wid_out, float* __restrict__ coef) {
  constexpr int nstat = Cin + Cin * Cin + 1;
  constexpr int FQ = F / 4;
  constexpr int Ca = Cin;
  constexpr int NA = 3 + Cin;
  const int b = blockIdx.x, tid = threadIdx.x, N = D.N, T = D.T;
  const int t0 = blockIdx.y * rows, t1 = min(T, t0 + rows);
  if (b >= B) {                                   // padding sequences of the time-major input: zeros
    for (int t = t0; t < t1; ++t) {
      for (int c = tid; c < Cp; c += 256) out[((long)t * Mp + b) * Cp + c] = 0.f;
      if constexpr (COEF)
        for (int c = tid; c < NA * F; c += 256) coef[((long)t * Mp + b) * (NA * F) + c] = 0.f;
    }
    return;
  }
  __shared__ double dred[4][nstat];
  __shared__ double S[nstat];
  __shared__ float prm[Cin + 2][F];             // W' = W * scale, b' = b * scale + shift, alpha
  __shared__ float svm[GF_ROW_MAX], spw[GF_ROW_MAX], ssh[GF_ROW_MAX], ssc[GF_ROW_MAX];
  __shared__ __attribute__((aligned(16))) float sx[GF_SLAB];
  const int NC = N * Cin;
  const int RP = gf_rows_per_pass(NC);
  // ---- phase A: all loads
  const long* ids = gf_ids(D, B);
  const long wraw = ids[b];
  const long w = wraw < 0 ? 0 : wraw;
  const float live = wraw >= 0 ? 1.f : 0.f;
  const long g = D.wg[w], c0 = D.wc[w];
  const long tn = D.time_norm ? c0 : 0;
  float pv[Cin + 6];                              // this thread's parameter column (tid < F)
  if (tid < F) {
#pragma unroll
    for (int k = 0; k < Cin; ++k) pv[k] = W[k * F + tid];
    pv[Cin] = bias[tid];
    pv[Cin + 1] = gamma[tid];
    pv[Cin + 2] = beta[tid];
    pv[Cin + 3] = alpha[tid];
    pv[Cin + 4] = rmean[tid];
    pv[Cin + 5] = rvar[tid];
  }
  float nv = 0.f, npw = 0.f, nsh = 0.f, nsc = 0.f;
  if (tid < N) {
    nv = D.wv[w * N + tid] ? live : 0.f;
    npw = D.pw[w * N + tid] * live;
  }
  if (tid < NC) {
    nsh = D.shift[(g * D.Tn + tn) * (long)NC + tid];
    nsc = D.scale[(g * D.Tn + tn) * (long)NC + tid];
  }
  double mv[nstat];
#pragma unroll
  for (int i = 0; i < nstat; ++i) mv[i] = 0.0;
  if (training) {                                 // the batch's moments: B window records
    for (int k = tid; k < B; k += 256) {
      const long wk = ids[k];
      if (wk >= 0) {
#pragma unroll
        for (int i = 0; i < nstat; ++i) mv[i] += D.mom[wk * nstat + i];
      }
    }
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
  if (training) {                                 // fixed-order reduction: identical in every workgroup
    const int lane = tid & 63, wv = tid >> 6;
#pragma unroll
    for (int i = 0; i < nstat; ++i) {
      double sv = mv[i];
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) sv += __shfl_xor(sv, o, 64);
      if (lane == 0) dred[wv][i] = sv;
    }
  }
  __syncthreads();
  if (training && tid < nstat) S[tid] = (dred[0][tid] + dred[1][tid]) + (dred[2][tid] + dred[3][tid]);
  gf_slab_park<Cin>(v, nr * NC, NC, svm, ssh, ssc, sx);
  __syncthreads();
  if (tid < F) {
    float mu, var;
    if (training) {
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
      mu = (float)m;
      var = (float)fmax(vv, 0.0);
    } else {
      mu = pv[Cin + 4];
      var = pv[Cin + 5];
    }
    const float inv = rsqrtf(var + eps);
    const float sc = pv[Cin + 1] * inv;
    const float sh = pv[Cin + 2] - mu * sc;
#pragma unroll
    for (int k = 0; k < Cin; ++k) prm[k][tid] = pv[k] * sc;
    prm[Cin][tid] = pv[Cin] * sc + sh;
    prm[Cin + 1][tid] = pv[Cin + 3];
    if (b == 0 && blockIdx.y == 0) {
      st[tid] = mu;
      st[F + tid] = inv;
      st[2 * F + tid] = sc;
      st[3 * F + tid] = sh;
      if (training) {
        rmean[tid] = pv[Cin + 4] * momentum + mu * (1.f - momentum);
        rvar[tid] = pv[Cin + 5] * momentum + var * (1.f - momentum);
      }
    }
  }
  if (b == 0 && blockIdx.y == 0 && training && tid < nstat) Sout[tid] = S[tid];
  if (blockIdx.y == 0 && tid == 0) {
    y[b] = D.wlab[w] * live;
    ym[b] = live;
    wid_out[b] = wraw;
  }
  __syncthreads();
  const long apl = D.gap[g];
  const int ap = apl < 0 ? 0 : (int)apl;
  const int r = tid >> 2, q = tid & 3, f0 = q * FQ;
  float pwk[Cin][FQ], pb[FQ], pal[FQ];
  float rwk[COEF ? Cin : 1][FQ], rb[FQ];           // COEF: the raw W, b (z before BatchNorm)
#pragma unroll
  for (int j = 0; j < FQ; ++j) {
#pragma unroll
    for (int k = 0; k < Cin; ++k) pwk[k][j] = prm[k][f0 + j];
    pb[j] = prm[Cin][f0 + j];
    pal[j] = prm[Cin + 1][f0 + j];
    if constexpr (COEF) {
#pragma unroll
      for (int k = 0; k < Cin; ++k) rwk[k][j] = W[k * F + f0 + j];
      rb[j] = bias[f0 + j];
    }
  }
  for (int p0 = t0; p0 < t1; p0 += RP) {
    if (p0 != t0) {                               // (more rows than one pass: stage the next slab)
      nr = min(RP, t1 - p0);
      gf_slab_load(src + (long)p0 * NC, nr * NC, v);
      __syncthreads();
      gf_slab_park<Cin>(v, nr * NC, NC, svm, ssh, ssc, sx);
      __syncthreads();
    }
    for (int rr = r; rr < nr; rr += 64) {
      const int t = p0 + rr;
      float acc[FQ];
      float cf[COEF ? NA : 1][FQ];
#pragma unroll
      for (int j = 0; j < FQ; ++j) {
        acc[j] = 0.f;
#pragma unroll
        for (int a = 0; a < (COEF ? NA : 1); ++a) cf[a][j] = 0.f;
      }
      const float* xr = sx + rr * NC;
      for (int n = 0; n < N; ++n) {
        const float wn = spw[n];
        float xv[Cin];
#pragma unroll
        for (int k = 0; k < Cin; ++k) xv[k] = xr[n * Cin + k];
#pragma unroll
        for (int j = 0; j < FQ; ++j) {
          float yv = pb[j];
#pragma unroll
          for (int k = 0; k < Cin; ++k) yv += xv[k] * pwk[k][j];
          const bool pos = yv > 0.f;
          acc[j] += wn * (pos ? yv : pal[j] * yv);
          if constexpr (COEF) {
            float z = rb[j];
#pragma unroll
            for (int k = 0; k < Cin; ++k) z += xv[k] * rwk[k][j];
            const float dp = pos ? wn : pal[j] * wn;
            cf[0][j] += dp;
            cf[1][j] += dp * z;
            cf[2][j] += pos ? 0.f : wn * yv;
#pragma unroll
            for (int k = 0; k < Cin; ++k) cf[3 + k][j] += dp * xv[k];
          }
        }
      }
      float* o = out + ((long)t * Mp + b) * Cp;
      if (q < Ca) o[q] = xr[ap * Cin + q];
#pragma unroll
      for (int j = 0; j < FQ; ++j) o[Ca + f0 + j] = acc[j];
      for (int c = Ca + F + q; c < Cp; c += 4) o[c] = 0.f;
      if constexpr (COEF) {
        float* co = coef + ((long)t * Mp + b) * (NA * F) + f0;
#pragma unroll
        for (int a = 0; a < NA; ++a) {
          if constexpr (FQ == 4) {
            *reinterpret_cast<float4*>(co + a * F) = make_float4(cf[a][0], cf[a][1], cf[a][2], cf[a][3]);
          } else {
#pragma unroll
            for (int j = 0; j < FQ; ++j) co[a * F + j] = cf[a][j];
          }
        }
      }
    }
  }
}

// ---- backward (training): grid (B, NY), 256 threads (body in gcn_fused.h: it also runs as extra
// workgroups of the LSTM weight-gradient launch, lstm_tm.hip lstm_grads_multi)
template <int Cin, int F>
__global__ __launch_bounds__(256) void gcn_fused_bwd_kernel(GcnBwdJob J) {
  __shared__ __attribute__((aligned(16))) char smem[GcnBwdLds<Cin, F>::BYTES];
  gcn_fused_bwd_body<Cin, F>(J, blockIdx.x, blockIdx.y, smem);
}

// ------------------------------------------------------------------ host
static GfData gf_data(const at::Tensor& series, const at::Tensor& shift, const at::Tensor& scale,
                      const at::Tensor& win_group, const at::Tensor& win_center, const at::Tensor& win_valid,
                      const at::Tensor& win_label, const at::Tensor& group_anom_pos, const at::Tensor& mom,
                      const at::Tensor& pw, const at::Tensor& wids, const at::Tensor& table,
                      const c10::optional<at::Tensor>& cursor, int64_t tb, int64_t seq_len, bool time_norm, int& B) {
  check_f32_cuda(series, "series");
  check_f32_cuda(shift, "shift");
  check_f32_cuda(scale, "scale");
  TORCH_CHECK(series.dim() == 4 && shift.dim() == 4 && scale.sizes() == shift.sizes(), "gcn_fused: store shapes");
  TORCH_CHECK(win_group.scalar_type() == at::kLong && win_center.scalar_type() == at::kLong &&
                  group_anom_pos.scalar_type() == at::kLong && win_valid.scalar_type() == at::kByte &&
                  win_valid.is_contiguous(), "gcn_fused: index tables");
  GfData D{};
  D.series = series.data_ptr<float>();
  D.shift = shift.data_ptr<float>();
  D.scale = scale.data_ptr<float>();
  D.wg = win_group.data_ptr<long>();
  D.wc = win_center.data_ptr<long>();
  D.wv = win_valid.data_ptr<uint8_t>();
  D.gap = group_anom_pos.data_ptr<long>();
  D.Ttot = (int)series.size(1);
  D.Tn = (int)shift.size(1);
  D.N = (int)series.size(2);
  D.tb = (int)tb;
  D.T = (int)seq_len;
  D.time_norm = time_norm ? 1 : 0;
  TORCH_CHECK(win_valid.size(1) == D.N, "gcn_fused: win_valid must be [nwin, N]");
  const int C = (int)series.size(3);
  TORCH_CHECK(C >= 1 && C <= GF_MAX_CIN && D.N * C <= GF_ROW_MAX, "gcn_fused: N * C must be <= 128, C <= 4");
  if (win_label.numel() > 0) {
    check_f32_cuda(win_label, "win_label");
    TORCH_CHECK(win_label.dim() == 1, "gcn_fused: per-window labels (flagged-sensor windows)");
    D.wlab = win_label.data_ptr<float>();
  }
  if (mom.numel() > 0) {
    TORCH_CHECK(mom.is_cuda() && mom.scalar_type() == at::kDouble && mom.is_contiguous() &&
                    mom.size(1) == C + C * C + 1, "gcn_fused: moments [nwin, nstat] fp64");
    D.mom = mom.data_ptr<double>();
  }
  if (pw.numel() > 0) {
    check_f32_cuda(pw, "pool weights");
    TORCH_CHECK(pw.size(1) == D.N, "gcn_fused: pool weights [nwin, N]");
    D.pw = pw.data_ptr<float>();
  }
  if (cursor.has_value() && cursor->defined()) {
    TORCH_CHECK(table.dim() == 2 && table.scalar_type() == at::kLong && table.is_contiguous() && table.is_cuda(),
                "gcn_fused: table must be a contiguous int64 [rows, B] device tensor");
    TORCH_CHECK(cursor->scalar_type() == at::kLong && cursor->numel() >= 1 && cursor->is_cuda(),
                "gcn_fused: cursor must be int64[1] on the device");
    B = (int)table.size(1);
    D.table = table.data_ptr<long>();
    D.cursor = cursor->data_ptr<long>();
    D.nrows = table.size(0);
  } else if (wids.numel() > 0 || wids.dim() == 1) {
    TORCH_CHECK(wids.scalar_type() == at::kLong && wids.is_contiguous() && wids.is_cuda(), "gcn_fused: wids int64");
    B = (int)wids.size(0);
    D.wids = wids.data_ptr<long>();
    D.nrows = 1;
  }
  TORCH_CHECK(B >= 0 && B <= 4096, "gcn_fused: batch size");
  return D;
}

// workgroups per sample (ny) and steps per workgroup (rows): one staging pass per workgroup
static void gf_grid(int T, int NC, int& ny, int& rows) {
  const int rp = std::min(GF_RPP, GF_SLAB / NC);
  ny = std::max(1, std::min(16, (T + rp - 1) / rp));
  rows = (T + ny - 1) / ny;
}

#define GQ_GF_CIN(CIN_RT, ...)                                 \
  switch (CIN_RT) {                                            \
    case 1: { constexpr int CIN = 1; __VA_ARGS__; } break;     \
    case 2: { constexpr int CIN = 2; __VA_ARGS__; } break;     \
    case 3: { constexpr int CIN = 3; __VA_ARGS__; } break;     \
    case 4: { constexpr int CIN = 4; __VA_ARGS__; } break;     \
    default: TORCH_CHECK(false, "gcn_fused: 1..4 input channels"); \
  }
#define GQ_GF_F(F_RT, ...)                                     \
  switch (F_RT) {                                              \
    case 8: { constexpr int FF = 8; __VA_ARGS__; } break;      \
    case 16: { constexpr int FF = 16; __VA_ARGS__; } break;    \
    case 32: { constexpr int FF = 32; __VA_ARGS__; } break;    \
    default: TORCH_CHECK(false, "gcn_fused: 8, 16 or 32 output channels"); \
  }

// [moments [nwin, nstat] fp64, pool weights [nwin, N]] of every window of the store
std::vector<at::Tensor> gcn_window_prep(const at::Tensor& series, const at::Tensor& shift, const at::Tensor& scale,
                                        const at::Tensor& win_group, const at::Tensor& win_center,
                                        const at::Tensor& win_valid, const at::Tensor& group_adj,
                                        const at::Tensor& group_anom_pos, int64_t tb, int64_t seq_len,
                                        bool time_norm, bool agg_mean, int64_t pool) {
  int B = 0;
  const at::Tensor e = series.new_zeros(0);
  GfData D = gf_data(series, shift, scale, win_group, win_center, win_valid, e, group_anom_pos, e, e,
                     e.to(at::kLong), e.to(at::kLong), c10::nullopt, tb, seq_len, time_norm, B);
  check_f32_cuda(group_adj, "group_adj");
  TORCH_CHECK(pool >= 0 && pool <= 2, "gcn_window_prep: pool 0 mean, 1 sum, 2 selection");
  const int C = (int)series.size(3);
  const long nwin = win_group.size(0);
  c10::DeviceGuard guard(series.device());
  at::Tensor mom = at::empty({nwin, C + C * C + 1}, series.options().dtype(at::kDouble));
  at::Tensor pw = at::empty({nwin, D.N}, series.options());
  if (nwin > 0)
    GQ_GF_CIN(C, hipLaunchKernelGGL(gcn_window_prep_kernel<CIN>, dim3(nwin), dim3(256), 2 * D.N * sizeof(float),
                                    stream(), D, group_adj.data_ptr<float>(), agg_mean ? 1 : 0, (int)pool, (int)nwin,
                                    mom.data_ptr<double>(), pw.data_ptr<float>()));
  GQ_LAUNCH_CHECK();
  return {mom, pw};
}

// returns [h [T, Mp, Cp], S [nstat] fp64 (training), st [4, F], y [B], y_mask [B], wid [B]]
std::vector<at::Tensor> gcn_fused_fwd(const at::Tensor& series, const at::Tensor& shift, const at::Tensor& scale,
                                      const at::Tensor& win_group, const at::Tensor& win_center,
                                      const at::Tensor& win_valid, const at::Tensor& win_label,
                                      const at::Tensor& group_anom_pos, const at::Tensor& mom, const at::Tensor& pw,
                                      const at::Tensor& wids, const at::Tensor& table,
                                      const c10::optional<at::Tensor>& cursor, int64_t tb, int64_t seq_len,
                                      bool time_norm, const at::Tensor& W, const at::Tensor& bias,
                                      const at::Tensor& gamma, const at::Tensor& beta, const at::Tensor& alpha,
                                      at::Tensor rmean, at::Tensor rvar, bool training, double momentum, double eps,
                                      int64_t Mp, int64_t Cp, bool with_coef, bool defer) {
  int B = 0;
  GfData D = gf_data(series, shift, scale, win_group, win_center, win_valid, win_label, group_anom_pos, mom, pw,
                     wids, table, cursor, tb, seq_len, time_norm, B);
  TORCH_CHECK(D.wlab != nullptr && D.pw != nullptr && (!training || D.mom != nullptr), "gcn_fused_fwd: tables");
  for (const at::Tensor* t : {&W, &bias, &gamma, &beta, &alpha, (const at::Tensor*)&rmean, (const at::Tensor*)&rvar})
    check_f32_cuda(*t, "gcn_fused_fwd parameter");
  const int C = (int)series.size(3), F = (int)W.size(1);
  TORCH_CHECK(W.size(0) == C && bias.numel() == F && gamma.numel() == F && beta.numel() == F && alpha.numel() == F &&
                  rmean.numel() == F && rvar.numel() == F, "gcn_fused_fwd: parameter shapes");
  TORCH_CHECK(Mp >= B && Mp % 16 == 0 && Cp >= C + F && Cp % 4 == 0, "gcn_fused_fwd: Mp / Cp");
  c10::DeviceGuard guard(series.device());
  auto fo = series.options();
  const int T = (int)seq_len;
  at::Tensor out = at::empty({T, Mp, Cp}, fo);
  at::Tensor S = at::empty({training ? C + C * C + 1 : 0}, fo.dtype(at::kDouble));
  at::Tensor st = at::empty({4, F}, fo);
  at::Tensor y = at::empty({B}, fo), ym = at::empty({B}, fo);
  at::Tensor wid = at::empty({B}, win_group.options());
  int ny, rows;
  gf_grid(T, D.N * C, ny, rows);
  // (the coefficient form: the CML configuration, 2 inputs / 16 features, training only). Side mode
  // (default): the coefficients are left to spare workgroups of the next LSTM chain forward launch
  // (gcn_coef_take), which runs while this kernel's output is consumed; else this kernel writes them.
  const bool want = with_coef && training && C == 2 && F == 16;
  at::Tensor coef = at::empty({want ? T : 0, want ? Mp : 0, (3 + C) * F}, fo);
  if (defer && training && C == 2 && F == 16 && T < 4096) {
    // producer mode: no launch here; the next LSTM chain forward launch runs this forward as producer
    // workgroups (gcn_prod_body) that stream its input to the chain's first stage (gcn_prod_flush
    // runs it on its own if another consumer comes first)
    at::Tensor gout = at::empty({T, Mp, Cp}, fo.dtype(at::kLong));
    GcnPending& pd = gcn_pending(series.get_device());
    TORCH_CHECK(!pd.prod.on, "gcn_fused_fwd: a deferred forward is still pending");
    GcnProdJob& J = pd.prod;
    J = GcnProdJob{};
    J.D = D;
    J.B = B;
    J.Mp = (int)Mp;
    J.Cp = (int)Cp;
    J.on = 1;
    J.W = W.data_ptr<float>();
    J.bias = bias.data_ptr<float>();
    J.gamma = gamma.data_ptr<float>();
    J.beta = beta.data_ptr<float>();
    J.alpha = alpha.data_ptr<float>();
    J.rmean = rmean.data_ptr<float>();
    J.rvar = rvar.data_ptr<float>();
    J.momentum = (float)momentum;
    J.eps = (float)eps;
    J.out = out.data_ptr<float>();
    J.gout = reinterpret_cast<unsigned long long*>(gout.data_ptr<int64_t>());
    J.Sout = S.data_ptr<double>();
    J.st = st.data_ptr<float>();
    J.y = y.data_ptr<float>();
    J.ym = ym.data_ptr<float>();
    J.wid = wid.data_ptr<long>();
    J.coef = want ? coef.data_ptr<float>() : nullptr;
    pd.pkeep = {out, gout, S, st, y, ym, wid, coef, W, bias, gamma, beta, alpha, rmean, rvar, series, shift, scale,
                win_group, win_center, win_valid, win_label, group_anom_pos, mom, pw, wids, table};
    if (cursor.has_value() && cursor->defined()) pd.pkeep.push_back(*cursor);
    return {out, S, st, y, ym, wid, coef};
  }
  const bool side = want && gcn_coef_side_mode();
  const bool cf = want && !side;
#define GQ_GF_FWD(CINV, FV, CFV)                                                                                      \
  hipLaunchKernelGGL((gcn_fused_fwd_kernel<CINV, FV, CFV>), dim3(Mp, ny), dim3(256), 0, stream(), D, B, (int)Mp,      \
      (int)Cp, rows, W.data_ptr<float>(), bias.data_ptr<float>(), gamma.data_ptr<float>(), beta.data_ptr<float>(),    \
      alpha.data_ptr<float>(), rmean.data_ptr<float>(), rvar.data_ptr<float>(), training ? 1 : 0, (float)momentum,     \
      (float)eps, out.data_ptr<float>(), training ? S.data_ptr<double>() : nullptr, st.data_ptr<float>(),             \
      y.data_ptr<float>(), ym.data_ptr<float>(), wid.data_ptr<long>(), cf ? coef.data_ptr<float>() : nullptr)
  if (cf) GQ_GF_FWD(2, 16, true);
  else GQ_GF_CIN(C, GQ_GF_F(F, GQ_GF_FWD(CIN, FF, false)));
#undef GQ_GF_FWD
  GQ_LAUNCH_CHECK();
  if (side) {
    // a job left pending by an earlier forward (no chain forward took it: e.g. a second micro-batch
    // forward before the first backward) runs now, or its coefficient tensor would never be written
    gcn_coef_flush_dev(series.get_device());
    GcnPending& pd = gcn_pending(series.get_device());
    pd.job = GcnCoefFwdJob{};
    pd.job.D = D;
    pd.job.B = B;
    pd.job.Mp = (int)Mp;
    pd.job.on = 1;
    pd.job.st = st.data_ptr<float>();
    pd.job.W = W.data_ptr<float>();
    pd.job.bias = bias.data_ptr<float>();
    pd.job.alpha = alpha.data_ptr<float>();
    pd.job.coef = coef.data_ptr<float>();
    // (the tensors the job reads or writes stay referenced until it has been launched)
    pd.keep = {coef, st, W, bias, alpha, series, shift, scale, win_group, win_center, win_valid, pw, wids, table};
    if (cursor.has_value() && cursor->defined()) pd.keep.push_back(*cursor);
  }
  return {out, S, st, y, ym, wid, coef};
}

// ---- pending coefficient side job (per device)
bool gcn_coef_side_mode() {
  const char* e = std::getenv("GNNQC_GCN_COEF_SIDE");
  return e == nullptr || std::atoi(e) != 0;
}

GcnPending& gcn_pending(int dev) {
  static GcnPending slots[64];
  TORCH_CHECK(dev >= 0 && dev < 64, "gcn_fused: device index");
  return slots[dev];
}

// the pending job of the current device, handed to a launch that runs it (chain forward); clears it
bool gcn_coef_take(int dev, GcnCoefFwdJob& job, std::vector<at::Tensor>& keep) {
  GcnPending& pd = gcn_pending(dev);
  if (!pd.job.on) return false;
  job = pd.job;
  keep.insert(keep.end(), pd.keep.begin(), pd.keep.end());
  pd.job.on = 0;
  pd.keep.clear();
  return true;
}

__global__ __launch_bounds__(1024) void gcn_coef_fwd_kernel(GcnCoefFwdJob J) {
  __shared__ __attribute__((aligned(16))) char smem[GcnCoefFwdLds::BYTES];
  gcn_coef_fwd_body<2, 16>(J, blockIdx.x, smem);
}

// the pending producer job of the current device, handed to the chain forward launch; clears it
bool gcn_prod_take(int dev, GcnProdJob& job, std::vector<at::Tensor>& keep) {
  GcnPending& pd = gcn_pending(dev);
  if (!pd.prod.on) return false;
  job = pd.prod;
  keep.insert(keep.end(), pd.pkeep.begin(), pd.pkeep.end());
  pd.prod.on = 0;
  pd.pkeep.clear();
  return true;
}

template <int Cin, int F>
__global__ __launch_bounds__(1024) void gcn_prod_kernel(GcnProdJob J) {
  __shared__ __attribute__((aligned(16))) char smem[GcnProdLds::BYTES];
  gcn_prod_body<Cin, F>(J, blockIdx.x, 0u, nullptr, smem);
}

// run a pending deferred forward on its own (no chain forward launch took it); returns whether
// there was one. The granule stream is not written (nothing streams it).
bool gcn_prod_flush_dev(int dev) {
  GcnProdJob J{};
  std::vector<at::Tensor> keep;
  if (!gcn_prod_take(dev, J, keep)) return false;
  J.gout = nullptr;
  hipLaunchKernelGGL((gcn_prod_kernel<2, 16>), dim3(J.Mp), dim3(1024), 0, stream(), J);
  GQ_LAUNCH_CHECK();
  return true;
}

bool gcn_prod_flush(const at::Tensor& like) {
  TORCH_CHECK(like.is_cuda(), "gcn_prod_flush: a GPU tensor names the device");
  c10::DeviceGuard guard(like.device());
  return gcn_prod_flush_dev(like.get_device());
}

// run the pending coefficient side job of device ``dev`` on its own; returns whether there was one
bool gcn_coef_flush_dev(int dev) {
  GcnCoefFwdJob J{};
  std::vector<at::Tensor> keep;
  if (!gcn_coef_take(dev, J, keep)) return false;
  hipLaunchKernelGGL(gcn_coef_fwd_kernel, dim3(J.Mp), dim3(1024), 0, stream(), J);
  GQ_LAUNCH_CHECK();
  return true;
}

// run the pending coefficient job on its own (nothing consumed it: no chain forward in between);
// returns whether there was one (a pending deferred forward, which writes the coefficients too, runs
// first)
bool gcn_coef_flush(const at::Tensor& like) {
  TORCH_CHECK(like.is_cuda(), "gcn_coef_flush: a GPU tensor names the device");
  c10::DeviceGuard guard(like.device());
  if (gcn_prod_flush_dev(like.get_device())) return true;
  return gcn_coef_flush_dev(like.get_device());
}

// The training backward's job (gcn_fused_bwd_body): adds dW, dgamma, dbeta, dalpha (float atomics)
// from dh [T, Mp, Dh] channels [c_off, c_off + F). (db is zero in training: BatchNorm removes the
// bias.) nblocks = B * ny workgroups (0: nothing to do). Shared with lstm_grads_multi (lstm_tm.hip).
GcnBwdJob gcn_bwd_job(const at::Tensor& dh, int64_t c_off, const at::Tensor& series, const at::Tensor& shift,
                      const at::Tensor& scale, const at::Tensor& win_group, const at::Tensor& win_center,
                      const at::Tensor& win_valid, const at::Tensor& group_anom_pos, const at::Tensor& pw,
                      const at::Tensor& wids, const at::Tensor& table, const c10::optional<at::Tensor>& cursor,
                      int64_t tb, int64_t seq_len, bool time_norm, const at::Tensor& S, const at::Tensor& st,
                      const at::Tensor& W, const at::Tensor& bias, const at::Tensor& alpha, const at::Tensor& dW,
                      const at::Tensor& dgamma, const at::Tensor& dbeta, const at::Tensor& dalpha, int& nblocks) {
  int B = 0;
  const at::Tensor e = series.new_zeros(0);
  GcnBwdJob J{};
  J.D = gf_data(series, shift, scale, win_group, win_center, win_valid, e, group_anom_pos, e, pw, wids, table, cursor,
                tb, seq_len, time_norm, B);
  check_f32_cuda(dh, "dh");
  for (const at::Tensor* t : {&st, &W, &bias, &alpha, &dW, &dgamma, &dbeta, &dalpha})
    check_f32_cuda(*t, "gcn_fused_bwd operand");
  const int C = (int)series.size(3), F = (int)W.size(1);
  TORCH_CHECK(C >= 1 && C <= GF_MAX_CIN && (F == 8 || F == 16 || F == 32), "gcn_fused_bwd: 1..4 input, 8/16/32 output channels");
  TORCH_CHECK(S.is_cuda() && S.scalar_type() == at::kDouble && S.numel() == C + C * C + 1, "gcn_fused_bwd: S");
  TORCH_CHECK(dh.dim() == 3 && dh.size(0) == seq_len && dh.size(1) >= B && dh.size(2) >= c_off + F,
              "gcn_fused_bwd: dh [T, Mp, Dh]");
  TORCH_CHECK(dW.numel() == (long)C * F && dgamma.numel() == F && dbeta.numel() == F && dalpha.numel() == F &&
                  st.numel() == 4 * F, "gcn_fused_bwd: gradient shapes");
  int ny, rows;
  gf_grid((int)seq_len, J.D.N * C, ny, rows);
  J.B = B;
  J.Mp = (int)dh.size(1);
  J.Dh = (int)dh.size(2);
  J.c_off = (int)c_off;
  J.rows = rows;
  J.ny = ny;
  J.key = C * 64 + F;
  J.dh = dh.data_ptr<float>();
  J.Sg = S.data_ptr<double>();
  J.st = st.data_ptr<float>();
  J.W = W.data_ptr<float>();
  J.bias = bias.data_ptr<float>();
  J.alpha = alpha.data_ptr<float>();
  J.dW = dW.data_ptr<float>();
  J.dgamma = dgamma.data_ptr<float>();
  J.dbeta = dbeta.data_ptr<float>();
  J.dalpha = dalpha.data_ptr<float>();
  J.nf = chain_ctl(series.get_device()) + 7;
  nblocks = B * ny;
  return J;
}

// The coefficient-form backward's job: dh [>= T, Mp, Dh] channels [c_off, c_off + F) against coef
// [T, Mp, (3 + Cin) F] of gcn_fused_fwd(with_coef); nblocks workgroups of 256 threads.
GcnCoefJob gcn_coef_job(const at::Tensor& dh, int64_t c_off, const at::Tensor& coef, const at::Tensor& S,
                        const at::Tensor& st, const at::Tensor& W, const at::Tensor& bias, const at::Tensor& dW,
                        const at::Tensor& dgamma, const at::Tensor& dbeta, const at::Tensor& dalpha) {
  check_f32_cuda(dh, "dh");
  check_f32_cuda(coef, "coef");
  for (const at::Tensor* t : {&st, &W, &bias, &dW, &dgamma, &dbeta, &dalpha}) check_f32_cuda(*t, "gcn_coef_bwd operand");
  const int C = (int)W.size(0), F = (int)W.size(1);
  TORCH_CHECK(C == 2 && F == 16, "gcn_coef_bwd: the CML configuration (2 inputs, 16 features)");
  TORCH_CHECK(coef.dim() == 3 && coef.size(2) == (3 + C) * F, "gcn_coef_bwd: coef [T, Mp, (3 + Cin) F]");
  const long T = coef.size(0), Mp = coef.size(1);
  TORCH_CHECK(dh.dim() == 3 && dh.size(0) >= T && dh.size(1) == Mp && dh.size(2) >= c_off + F,
              "gcn_coef_bwd: dh [>= T, Mp, Dh] with the coefficients' T and Mp");
  TORCH_CHECK(S.is_cuda() && S.scalar_type() == at::kDouble && S.numel() == C + C * C + 1, "gcn_coef_bwd: S");
  TORCH_CHECK(dW.numel() == (long)C * F && dgamma.numel() == F && dbeta.numel() == F && dalpha.numel() == F &&
                  st.numel() == 4 * F, "gcn_coef_bwd: gradient shapes");
  GcnCoefJob J{};
  J.dh = dh.data_ptr<float>();
  J.coef = coef.data_ptr<float>();
  J.rows = T * Mp;
  J.Dh = (int)dh.size(2);
  J.c_off = (int)c_off;
  // ~180 rows per workgroup (the CML step: 128 workgroups over 23k rows): every workgroup's loads
  // are one short burst, and 128 x 80 atomics onto 80 gradients stay cheap
  J.nblocks = (int)std::max<long>(1, std::min<long>(256, (J.rows + 179) / 180));
  J.key = C * 64 + F;
  J.Sg = S.data_ptr<double>();
  J.st = st.data_ptr<float>();
  J.W = W.data_ptr<float>();
  J.bias = bias.data_ptr<float>();
  J.dW = dW.data_ptr<float>();
  J.dgamma = dgamma.data_ptr<float>();
  J.dbeta = dbeta.data_ptr<float>();
  J.dalpha = dalpha.data_ptr<float>();
  J.nf = chain_ctl(dh.get_device()) + 7;
  return J;
}

__global__ __launch_bounds__(256) void gcn_coef_bwd_kernel(GcnCoefJob J) { gcn_coef_bwd_body<2, 16>(J, blockIdx.x); }

void gcn_coef_bwd(const at::Tensor& dh, int64_t c_off, const at::Tensor& coef, const at::Tensor& S,
                  const at::Tensor& st, const at::Tensor& W, const at::Tensor& bias, at::Tensor dW, at::Tensor dgamma,
                  at::Tensor dbeta, at::Tensor dalpha) {
  c10::DeviceGuard guard(dh.device());
  const GcnCoefJob J = gcn_coef_job(dh, c_off, coef, S, st, W, bias, dW, dgamma, dbeta, dalpha);
  if (J.rows > 0) hipLaunchKernelGGL(gcn_coef_bwd_kernel, dim3(J.nblocks), dim3(256), 0, stream(), J);
  GQ_LAUNCH_CHECK();
}

void gcn_fused_bwd(const at::Tensor& dh, int64_t c_off, const at::Tensor& series, const at::Tensor& shift,
                   const at::Tensor& scale, const at::Tensor& win_group, const at::Tensor& win_center,
                   const at::Tensor& win_valid, const at::Tensor& group_anom_pos, const at::Tensor& pw,
                   const at::Tensor& wids, const at::Tensor& table, const c10::optional<at::Tensor>& cursor, int64_t tb,
                   int64_t seq_len, bool time_norm, const at::Tensor& S, const at::Tensor& st, const at::Tensor& W,
                   const at::Tensor& bias, const at::Tensor& alpha, at::Tensor dW, at::Tensor dgamma, at::Tensor dbeta,
                   at::Tensor dalpha) {
  c10::DeviceGuard guard(series.device());
  int nb = 0;
  const GcnBwdJob J = gcn_bwd_job(dh, c_off, series, shift, scale, win_group, win_center, win_valid, group_anom_pos,
                                  pw, wids, table, cursor, tb, seq_len, time_norm, S, st, W, bias, alpha, dW, dgamma,
                                  dbeta, dalpha, nb);
  const int C = (int)series.size(3), F = (int)W.size(1);
  if (nb > 0)
    GQ_GF_CIN(C, GQ_GF_F(F, hipLaunchKernelGGL((gcn_fused_bwd_kernel<CIN, FF>), dim3(J.B, J.ny), dim3(256), 0,
                                               stream(), J)));
  GQ_LAUNCH_CHECK();
}

}  // namespace gq

TORCH_LIBRARY_IMPL(gnnqc, CUDA, m) {
  m.impl("gcn_window_prep", &gq::gcn_window_prep);
  m.impl("gcn_fused_fwd", &gq::gcn_fused_fwd);
  m.impl("gcn_fused_bwd", &gq::gcn_fused_bwd);
  m.impl("gcn_coef_bwd", &gq::gcn_coef_bwd);
  m.impl("gcn_coef_flush", &gq::gcn_coef_flush);
  m.impl("gcn_prod_flush", &gq::gcn_prod_flush);
}
