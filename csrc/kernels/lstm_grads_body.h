// Device bodies of the LSTM weight-gradient pass (lstm_grads.hip) and its split reduction,
// shared with lstm_tm.hip, whose backward launches can carry them as extra workgroups.
#pragma once
#include "common.h"

#include <type_traits>

namespace gq {

constexpr int GR_ROWS = 32;         // rows (sequence, step) per tile = MFMA K
constexpr int GR_CB = 64;           // gate-units per column block (4 waves x 16)
constexpr int GR_LDR = GR_ROWS + 8; // padded LDS row length (bf16) of transposed images
// Staging map of the per-tile register images: GR_SEQ_FAST = 1 gives consecutive lanes consecutive
// row pairs of ONE channel / gate-unit quad, so the packed (rows 2p, 2p + 1) stores into the
// transposed images hit consecutive dwords (with consecutive lanes on consecutive channels the 32
// lanes of a ds_write_b32 group land on 2-4 banks: 8- to 16-way, scripts/lds_model/grads.py), but
// the global loads then read 16 rows x 16-32 B per wave instead of whole rows. Measured slightly
// slower (SoilNet 2.737 vs 2.724 ms, profiles/r6_grads_stage_map_ab.txt): off.
#ifndef GR_SEQ_FAST
#define GR_SEQ_FAST 0
#endif

// a weight-gradient pass (lstm_grads_body) and its split reduction as kernel-argument records
struct GradJob {
  const void* dz;                   // bf16 (GradJob consumers instantiate the bf16 body only)
  const float* x;
  const float* h;
  const float* W;
  float* ws;
  long rows, period, hshift, x_elems;
  int Din, ldx, xg, ncb, splits, nblocks;
};

struct RedJob {
  const float* ws;
  float* dW;
  float* db;
  float* dU;
  int* nf;                // non-finite gradient flag (chain control word 7, read by adam_flagged)
  int splits, RC, ncb, DT, HT, Din, H, nblocks, kb;
};

// One workgroup = (column block cb of 64 gate-units, row split s); it walks the row tiles
// s, s + splits, ... with a one-tile register prefetch: tile i+1's dz / x / h_{t-1} loads are
// issued before tile i's MFMAs and only waited for when tile i+1 is staged (LDS-only
// barriers, so the loads stay in flight across them). Every tile's x and h rows are ONE
// contiguous span (flat rows), streamed in GRX-float granules. The weight-gradient partial
// tiles stay in VGPRs and are written once per workgroup, in MFMA-fragment order, to a
// workspace that lstm_grads_reduce_kernel sums over the splits (fixed order, plain
// read-modify-write into the gradient buffers: deterministic, no float atomics).
// (device body: cb / split / ncbv / splits are the virtual block coordinates, so the same code
// runs as its own kernel or as extra workgroups of a recurrence launch; needs 256 threads)
// LDS of one body instance (the caller owns the buffer: a kernel holding several instances
// then reserves the largest one instead of their sum)
template <int H, int DT>
struct GradsLds {
  static constexpr int DZT = GR_CB * GR_LDR * 2;
  static constexpr int DZR = GR_ROWS * (GR_CB + 8) * 2;
  static constexpr int XT = DT * 16 * GR_LDR * 2;
  static constexpr int HT = H * GR_LDR * 2;
  static constexpr int BYTES = DZT + DZR + XT + HT;
};

// agent-scope (sc1, write-through) store of 16 bytes as two untorn 8-byte halves
__device__ __forceinline__ void st4_sc1(float* p, f32x4_t v) {
  unsigned long long* q = reinterpret_cast<unsigned long long*>(p);
  __hip_atomic_store(q, ((unsigned long long)__float_as_uint(v[1]) << 32) | __float_as_uint(v[0]), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(q + 1, ((unsigned long long)__float_as_uint(v[3]) << 32) | __float_as_uint(v[2]), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ float ld_sc1(const float* p) {
  return __uint_as_float(__hip_atomic_load(reinterpret_cast<const unsigned*>(p), __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT));
}

// CH (chained: extra workgroups of the backward chain kernel): no dx, and the split record is
// stored write-through (sc1) for a reduction inside the same launch that reads it with sc1 loads
// ZT: dz element type - bf16 (the time-major recurrences: 8 B per 4 gate-units, exact, since the
// MFMAs consume bf16 either way) or fp32 (the sequence-major lstm_bwd). A compile-time choice: a
// runtime branch around the prefetch loads made hipcc drain the load ring at the join (measured:
// the SoilNet weight-gradient passes 20-25 % slower).
template <int H, int DT, int GRX, bool CH = false, typename ZT = __bf16>
__device__ __forceinline__ void lstm_grads_body(
    const void* __restrict__ dzv, const float* __restrict__ x, const float* __restrict__ hseq,
    const float* __restrict__ W, float* __restrict__ dx, float* __restrict__ ws, long rows, long period,
    long hshift, int Din, int ldx, long dx_cb_stride, int lddx, int xg, long x_elems, int cb, int split,
    int ncbv, int splits, char* __restrict__ smem) {
  constexpr bool ZBF = std::is_same<ZT, __bf16>::value;
  const ZT* __restrict__ dz = reinterpret_cast<const ZT*>(dzv);
  constexpr int G4 = 4 * H;
  constexpr int HT = H / 16;        // k tiles of dU
  constexpr int DP = DT * 16;       // padded din (incl. bias channel)
  constexpr int XGM = (GR_ROWS * 144 / GRX + 255) / 256;   // max x granules per thread
  // h_{t-1} staging items: (row pair, 4-unit quad) -> 16 * H / 4 items, two float4 loads each
  constexpr int HG = (GR_ROWS / 2 * H / 4 + 255) / 256;    // items per thread
  using L = GradsLds<H, DT>;
  static_assert(L::DZT % 16 == 0 && L::DZR % 16 == 0 && L::XT % 16 == 0, "grads LDS layout");
  auto dzT = reinterpret_cast<__bf16 (*)[GR_LDR]>(smem);                              // [gu][row]
  auto dzR = reinterpret_cast<__bf16 (*)[GR_CB + 8]>(smem + L::DZT);                  // [row][gu]
  auto xT = reinterpret_cast<__bf16 (*)[GR_LDR]>(smem + L::DZT + L::DZR);             // [din][row]
  auto hT = reinterpret_cast<__bf16 (*)[GR_LDR]>(smem + L::DZT + L::DZR + L::XT);     // [k][row]

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int w = tid >> 6;
  const int col = lane & 15;
  const int quad = lane >> 4;
  const int gu0 = cb * GR_CB;                // column block: gate-units [cb*64, cb*64+64)
  const long ntiles = (rows + GR_ROWS - 1) / GR_ROWS;
  const long nmine = split < ntiles ? (ntiles - 1 - split) / splits + 1 : 0;

  for (int e = tid; e < DP * GR_LDR; e += 256) (&xT[0][0])[e] = (__bf16)0.f;   // channels > Din stay 0

  f32x4_t accW[DT], accU[HT];
#pragma unroll
  for (int d = 0; d < DT; ++d) accW[d] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int k = 0; k < HT; ++k) accU[k] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  // dx work items of this wave: (din tile, row tile) pairs, 2 row tiles per 32 rows
  constexpr int DXT = (DP + 15) / 16 * 2;
  bf16x8_t wa[CH ? 1 : (DXT + 3) / 4][2];
#pragma unroll
  for (int i = 0; i < (CH ? 0 : (DXT + 3) / 4); ++i) {
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

  // ---- per-tile register images (prefetch ring of depth 1)
  float4 rz[2];                     // dz: rows 2 (tid/16) and 2 (tid/16) + 1, gate-units 4*(tid%16) ..
  // x: GRX == 4 -> items (row pair, 4-channel quad), two float4 each (packed bf16x2 staging);
  // GRX == 1 (unaligned rows) -> single floats of the contiguous [32][ldx] span
  constexpr int XGP = (GR_ROWS / 2 * 144 / 4 + 255) / 256;   // max pair items per thread
  float rx[GRX == 4 ? 1 : XGM][GRX];
  float4 rxp[GRX == 4 ? XGP : 1][2];
  float4 rh[HG][2];                 // h_{t-1}: rows 2p and 2p + 1 of unit quad c (item = p * H/4 + c)
  const int zr = GR_SEQ_FAST ? (tid & 15) : (tid >> 4), zc = (GR_SEQ_FAST ? (tid >> 4) : (tid & 15)) * 4;
  // (x / h_{t-1} items: row pair and channel quad of item `it`)
  auto it_pair = [&](int it, int nq) { return GR_SEQ_FAST ? (it & 15) : it / nq; };
  auto it_quad = [&](int it, int nq) { return GR_SEQ_FAST ? (it >> 4) : it % nq; };
  const long xspan = (long)GR_ROWS * ldx;
  // x_elems: floats readable from x (a strided view may end before rows * ldx)
  const long xlast = (x_elems - GRX) / GRX * GRX, hlast = rows * (long)H - 4;
  auto load_tile = [&](long tile) {
    const long r0 = tile * GR_ROWS;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const long r = min(r0 + 2 * zr + q, rows - 1);
      if constexpr (ZBF) {
        const uint2 u = *reinterpret_cast<const uint2*>(dz + (size_t)r * G4 + gu0 + zc);
        rz[q] = make_float4(__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u),
                            __uint_as_float(u.y << 16), __uint_as_float(u.y & 0xffff0000u));
      } else {
        rz[q] = *reinterpret_cast<const float4*>(dz + (size_t)r * G4 + gu0 + zc);
      }
    }
    // granule offsets are clamped into the tile's span (idle lanes re-read a line already
    // being fetched instead of the next tile's data) and into the array (rows past the end
    // and h_{t-1} of a period's first step are masked when staged)
    if constexpr (GRX == 4) {
      const int nq = ldx / 4, nit = GR_ROWS / 2 * nq;
#pragma unroll
      for (int i = 0; i < XGP; ++i) {
        if (i < xg) {                             // kernel argument: a scalar (uniform) branch
          const int it = min(tid + 256 * i, nit - 1);
          const long o = (r0 + 2 * it_pair(it, nq)) * ldx + 4 * it_quad(it, nq);
          rxp[i][0] = *reinterpret_cast<const float4*>(x + min(o, xlast));
          rxp[i][1] = *reinterpret_cast<const float4*>(x + min(o + ldx, xlast));
        }
      }
    } else {
#pragma unroll
      for (int i = 0; i < XGM; ++i) {
        if (i < xg) {                             // kernel argument: a scalar (uniform) branch
          const long o = min(r0 * ldx + min((long)(tid + 256 * i) * GRX, xspan - GRX), xlast);
          rx[i][0] = x[o];
        }
      }
    }
#pragma unroll
    for (int i = 0; i < HG; ++i) {
      const int it = min(tid + 256 * i, GR_ROWS / 2 * H / 4 - 1);     // (idle lanes re-read the last item)
      const long o = (r0 - hshift + 2 * it_pair(it, H / 4)) * H + 4 * it_quad(it, H / 4);
      rh[i][0] = *reinterpret_cast<const float4*>(hseq + min(max(o, 0L), hlast));
      rh[i][1] = *reinterpret_cast<const float4*>(hseq + min(max(o + H, 0L), hlast));
    }
  };
  auto stage_tile = [&](long tile) {
    const long r0 = tile * GR_ROWS;
    {
      // a lane holds rows 2 zr and 2 zr + 1 of its 4 gate-units: the transposed image gets one
      // packed bf16x2 (4-byte) store per gate-unit instead of two 2-byte stores into a shared
      // dword (LDS bank conflicts dominated this staging: rocprofv3 SQ_LDS_BANK_CONFLICT)
      typedef __bf16 bf16x4_t __attribute__((ext_vector_type(4)));
      typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
      const int rr = 2 * zr;
      const float m0 = (r0 + rr < rows) ? 1.f : 0.f, m1 = (r0 + rr + 1 < rows) ? 1.f : 0.f;
      const bf16x4_t a = bf16x4_t{(__bf16)(rz[0].x * m0), (__bf16)(rz[0].y * m0), (__bf16)(rz[0].z * m0),
                                  (__bf16)(rz[0].w * m0)};
      const bf16x4_t b = bf16x4_t{(__bf16)(rz[1].x * m1), (__bf16)(rz[1].y * m1), (__bf16)(rz[1].z * m1),
                                  (__bf16)(rz[1].w * m1)};
      if constexpr (!CH) {
        if (dx != nullptr) {   // (uniform) the row-major copy feeds only the dx products
          *reinterpret_cast<bf16x4_t*>(&dzR[rr][zc]) = a;
          *reinterpret_cast<bf16x4_t*>(&dzR[rr + 1][zc]) = b;
        }
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) *reinterpret_cast<bf16x2_t*>(&dzT[zc + j][rr]) = bf16x2_t{a[j], b[j]};
    }
    if constexpr (GRX == 4) {
      typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
      const int nq = ldx / 4, nit = GR_ROWS / 2 * nq;
#pragma unroll
      for (int i = 0; i < XGP; ++i) {
        const int it = tid + 256 * i;
        if (i < xg && it < nit) {                 // one packed bf16x2 (rows 2p, 2p + 1) per channel
          const int rr = 2 * it_pair(it, nq), d0 = 4 * it_quad(it, nq);
          const float ma = (r0 + rr < rows) ? 1.f : 0.f, mb = (r0 + rr + 1 < rows) ? 1.f : 0.f;
          const float a[4] = {rxp[i][0].x, rxp[i][0].y, rxp[i][0].z, rxp[i][0].w};
          const float b[4] = {rxp[i][1].x, rxp[i][1].y, rxp[i][1].z, rxp[i][1].w};
#pragma unroll
          for (int q = 0; q < 4; ++q)
            if (d0 + q < Din)
              *reinterpret_cast<bf16x2_t*>(&xT[d0 + q][rr]) = bf16x2_t{(__bf16)(a[q] * ma), (__bf16)(b[q] * mb)};
        }
      }
    } else {
#pragma unroll
      for (int i = 0; i < XGM; ++i) {
        const long g = (long)(tid + 256 * i) * GRX;
        if (i < xg && g < xspan) {                // xg: wave-uniform (kernel argument)
          const int rr = (int)(g / ldx), d0 = (int)(g % ldx);
          const float m = (r0 + rr < rows) ? 1.f : 0.f;
          if (d0 < Din) xT[d0][rr] = (__bf16)(rx[i][0] * m);
        }
      }
    }
    if (tid < GR_ROWS) xT[Din][tid] = (__bf16)((r0 + tid < rows) ? 1.f : 0.f);   // bias channel
#pragma unroll
    for (int i = 0; i < HG; ++i) {
      // one packed bf16x2 (rows 2p, 2p + 1) per unit: conflict-free across a wave's lanes
      const int it = tid + 256 * i;
      if (it < GR_ROWS / 2 * H / 4) {
        const int rr = 2 * it_pair(it, H / 4), k0 = 4 * it_quad(it, H / 4);
        const long ra = r0 + rr, rb = ra + 1;
        const float ma = (ra < rows && ra % period >= hshift) ? 1.f : 0.f;
        const float mb = (rb < rows && rb % period >= hshift) ? 1.f : 0.f;
        typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
        *reinterpret_cast<bf16x2_t*>(&hT[k0 + 0][rr]) = bf16x2_t{(__bf16)(rh[i][0].x * ma), (__bf16)(rh[i][1].x * mb)};
        *reinterpret_cast<bf16x2_t*>(&hT[k0 + 1][rr]) = bf16x2_t{(__bf16)(rh[i][0].y * ma), (__bf16)(rh[i][1].y * mb)};
        *reinterpret_cast<bf16x2_t*>(&hT[k0 + 2][rr]) = bf16x2_t{(__bf16)(rh[i][0].z * ma), (__bf16)(rh[i][1].z * mb)};
        *reinterpret_cast<bf16x2_t*>(&hT[k0 + 3][rr]) = bf16x2_t{(__bf16)(rh[i][0].w * ma), (__bf16)(rh[i][1].w * mb)};
      }
    }
  };

  if (nmine > 0) load_tile(split);
  for (long i = 0; i < nmine; ++i) {
    const long tile = split + i * splits;
    lds_barrier();                                // previous tile's LDS reads are done
    stage_tile(tile);
    load_tile(min(tile + splits, ntiles - 1));    // prefetch (the last one is a harmless reload)
    lds_barrier();
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
    if constexpr (!CH) if (dx != nullptr) {
      const long r0 = tile * GR_ROWS;
#pragma unroll
      for (int ii = 0; ii < (DXT + 3) / 4; ++ii) {
        const int item = w + 4 * ii;
        if (item < DXT) {   // wave-uniform
          const int dtile = item >> 1, rt = item & 1;
          f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int ks = 0; ks < 2; ++ks) {
            const bf16x8_t bz = *reinterpret_cast<const bf16x8_t*>(&dzR[16 * rt + col][32 * ks + 8 * quad]);
            acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[ii][ks], bz, acc, 0, 0, 0);
          }
          const long r = r0 + 16 * rt + col;
          if (r < rows) {
            float* o = dx + cb * dx_cb_stride + (size_t)r * lddx;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              const int din = dtile * 16 + 4 * quad + q;
              if (din < lddx) o[din] = acc[q];   // columns Din .. lddx-1: zero (W rows masked)
            }
          }
        }
      }
    }
  }
  // ---- partial tiles -> workspace record of this workgroup, fragment order (float4 per lane)
  float* rec = ws + ((size_t)split * ncbv + cb) * (size_t)(DT + HT) * 1024;
#pragma unroll
  for (int d = 0; d < DT; ++d) {
    float* o = rec + ((size_t)(d * 4 + w) * 64 + lane) * 4;
    if constexpr (CH) st4_sc1(o, accW[d]);
    else *reinterpret_cast<f32x4_t*>(o) = accW[d];
  }
#pragma unroll
  for (int k = 0; k < HT; ++k) {
    float* o = rec + ((size_t)((DT + k) * 4 + w) * 64 + lane) * 4;
    if constexpr (CH) st4_sc1(o, accU[k]);
    else *reinterpret_cast<f32x4_t*>(o) = accU[k];
  }
}

// Reduction of the per-split records in a fixed order (deterministic):
//   reduce: workgroup = 16 consecutive record slots x 16 split lanes (x NG split groups in
//           grid.y); split lane l of group g sums splits g*16 + l, + 16*NG, ...; the 16 lane
//           partials are combined through LDS. With NG == 1 (up to 512 splits) the result is
//           added to the gradient buffers directly, else it goes to ws2[g][slot] and
//   final:  thread = record slot sums its NG group sums and adds them.
// Adding: one writer per element, plain read-modify-write into dW [Din,4H] / db / dU [H,4H].
// nf (optional): raised when a sum is not finite (adam_flagged reads it instead of scanning g)
__device__ __forceinline__ void grads_add(float s, int e, int ncb, int DT, int HT, int Din, int H,
                                          float* __restrict__ dW, float* __restrict__ db, float* __restrict__ dU,
                                          int* nf = nullptr) {
  if (nf != nullptr && !isfinite(s)) __hip_atomic_store(nf, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const int R = (DT + HT) * 1024;
  const int G4 = 4 * H;
  // record layout: [split][cb][DT + HT fragments][4 waves][64 lanes][4]
  const int cb = e / R, slot = e % R;
  const int q = slot & 3, lane = (slot >> 2) & 63, w = (slot >> 8) & 3, j = slot >> 10;
  const int colr = lane & 15, quad = lane >> 4;
  const int gu = cb * GR_CB + 16 * w + 4 * quad + q;
  if (j < DT) {
    const int din = 16 * j + colr;
    if (din < Din) dW[(size_t)din * G4 + gu] += s;
    else if (din == Din) db[gu] += s;
  } else {
    const int k = 16 * (j - DT) + colr;
    if (k < H) dU[(size_t)k * G4 + gu] += s;
  }
}

__device__ __forceinline__ void lstm_grads_reduce_body(const float* __restrict__ ws, int splits, int RC,
                                                       float* __restrict__ ws2, int ncb, int DT, int HT, int Din,
                                                       int H, float* __restrict__ dW, float* __restrict__ db,
                                                       float* __restrict__ dU, int bx, int g, int NG,
                                                       int* nf = nullptr) {
  // 16 consecutive slots (64 B per split row) x 16 split lanes (measured faster than 8 x 32)
  __shared__ float red[16][17];
  const int sl = threadIdx.x & 15, l = threadIdx.x >> 4;
  const int slot = min(bx * 16 + sl, RC - 1);
  const int stride = 16 * NG;
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  int sp = g * 16 + l;
  for (; sp + 3 * stride < splits; sp += 4 * stride) {
    a0 += ws[(size_t)sp * RC + slot];
    a1 += ws[(size_t)(sp + stride) * RC + slot];
    a2 += ws[(size_t)(sp + 2 * stride) * RC + slot];
    a3 += ws[(size_t)(sp + 3 * stride) * RC + slot];
  }
  for (; sp < splits; sp += stride) a0 += ws[(size_t)sp * RC + slot];
  red[l][sl] = (a0 + a1) + (a2 + a3);
  __syncthreads();
  if (threadIdx.x < 16 && bx * 16 + sl < RC) {
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) s += red[k][sl];
    if (NG == 1) grads_add(s, slot, ncb, DT, HT, Din, H, dW, db, dU, nf);
    else ws2[(size_t)g * RC + slot] = s;
  }
}

// Reduction for the pipelined backward (lstm_tm_bwd_dual_kernel): one workgroup reduces KB
// slot blocks (16 slots each) at once, so all KB x (splits / 16) loads of a thread are in
// flight together and the job needs KB times fewer workgroups (they are as wide as the
// recurrence's, so their count, not their bytes, bounded the one-block-per-16-slots form).
// Fixed summation order: deterministic. Splits <= PIPE_MAX_SPLITS, added directly.
template <int KB>
__device__ __forceinline__ void lstm_grads_reduce_multi(const float* __restrict__ ws, int splits, int RC, int ncb,
                                                        int DT, int HT, int Din, int H, float* __restrict__ dW,
                                                        float* __restrict__ db, float* __restrict__ dU, int bx,
                                                        int* nf = nullptr) {
  __shared__ float red[KB][16][17];
  const int sl = threadIdx.x & 15, l = threadIdx.x >> 4;
  int slot[KB];
  float a[KB];
#pragma unroll
  for (int k = 0; k < KB; ++k) {
    slot[k] = min((bx * KB + k) * 16 + sl, RC - 1);
    a[k] = 0.f;
  }
  for (int sp = l; sp < splits; sp += 16) {
    const float* r = ws + (size_t)sp * RC;
#pragma unroll
    for (int k = 0; k < KB; ++k) a[k] += r[slot[k]];
  }
#pragma unroll
  for (int k = 0; k < KB; ++k) red[k][l][sl] = a[k];
  __syncthreads();
  if (threadIdx.x < 16 * KB) {
    const int k = threadIdx.x >> 4;
    const int e = (bx * KB + k) * 16 + sl;
    if (e < RC) {
      float s = 0.f;
#pragma unroll
      for (int j = 0; j < 16; ++j) s += red[k][j][sl];
      grads_add(s, e, ncb, DT, HT, Din, H, dW, db, dU, nf);
    }
  }
}

}  // namespace gq
