// Cross-CU layer pipeline for the forward of a time-major LSTM stack (gfx950).
//
// The per-layer forward kernels (lstm_tm.hip) run one after another: with the CML batch a
// recurrence occupies 8 of the 256 CUs, and the stack's six recurrences (plus three pool
// launches) are a serial sum. Sequences never mix across layers, so tile j of layer k+1
// only needs tile j of layer k - and only up to the step it is at. This kernel runs all
// layers of the stack at once: workgroup (stage s, tile j) computes layer s of tile j on
// its own CU and consumes layer s-1's output AS IT IS PRODUCED, a few steps behind.
//
// Hand-off (MI355X_MICROARCH.md "Workgroup dispatch ... inter-workgroup visibility", R2
// granules): the producer writes every output element a second time as an 8-byte
// {value, tag} granule with an agent-scope (sc1, write-through) store; the consumer's
// prefetch ring loads granules with agent-scope (sc1, L1-bypassing) loads and checks the
// tag (launch epoch | time index) when it stages x_t into LDS; a wave whose granules are not
// there yet re-polls (bounded; a timeout sets a flag instead of hanging). The producer
// never waits, the consumer only when it catches up. An 8-byte granule is written and read
// untorn, so no fence or flag ordering is needed.
//
// The launch epoch lives in device memory (ctl[0]) and is advanced by the last workgroup
// to finish, so HIP-graph replays get fresh tags and stale granules of an earlier launch
// at the same address never match. All workgroups must be co-resident (grid <= 256 of
// 1024-thread workgroups, checked on the host): a consumer spins only on producers that
// are already running. Workgroups of stage s for tile j have the same blockIdx % 8, so
// under the observed round-robin placement one tile's whole stack shares an XCD (speed only).
//
// A MaxPooling1D(3) between two stages is done by the CONSUMER while staging its input
// (three granules per element, max + first-max argmax byte): the producer's own per-step
// pooling lengthened its serial chain by ~110 ns per step (58 -> 78 us for the first pooled
// CML layer), while the consumer, running at a third of the producer's step rate, has slack.
// Each stage also writes everything the per-layer kernels write (h, gate / cell state for
// the backward, pooled output + argmax bytes), so the backward is unchanged.
#include "chain_head.h"
#include "common.h"
#include "gcn_fused.h"
#include "lstm_grads_body.h"
#include "lstm_tm_common.h"

#include <cstdlib>
#include <type_traits>

namespace gq {

typedef unsigned long long u64x2_t __attribute__((ext_vector_type(2)));
typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));

static constexpr int CHAIN_MAX = 8;
static constexpr int CHAIN_SPIN = 1 << 20;
// granule ring depth of a non-pooling consumer: an sc1 load of a line another CU wrote
// through to memory takes microseconds under load, D steps of ~0.33 us each must cover it.
// D, LEAD1 and CHAINB_LEAD (below) from a same-box sweep of compile-time variants
// (scripts/build_chain_variants.py, scripts/gpu_ab_chain.sh; CML step, ms): D = 6 / LEAD 2 / 2:
// 0.3099 0.3092; D = 5: 0.3105; D = 4: 0.3072 0.3070; D = 3: 0.3055; D = 8: 0.3121; D = 4 with
// CHAINB_LEAD 1: 0.3025; D = 4 with both leads 1: 0.3021 0.3022 0.3006 (kept); D = 3 with both
// leads 1: 0.3044 0.2999. A shorter ring lets each consumer start sooner behind its producer.
#ifndef CHAIN_D
#define CHAIN_D 4
#endif
#ifndef CHAIN_D3
#define CHAIN_D3 2           // ring of a pooling (PIN = 3) consumer: it runs at a third of the rate
#endif                       // (2 vs 3: 0.2982 0.2994 vs 0.3022 0.3027 ms/step; the backward rings at 3
                             // instead of 4 and LEAD3 = 0 were slower: 0.3054 0.3057, 0.3043)
#ifndef CHAIN_LEAD1
#define CHAIN_LEAD1 1
#endif
#ifndef CHAIN_D0
#define CHAIN_D0 6           // x prefetch depth of stage 0 (its input is complete before the launch)
#endif
#ifndef CHAIN_LD16
#define CHAIN_LD16 0         // 1: one 16-byte buffer load per granule pair (measured: stale reads, ~4.5k re-polls per launch)
#endif
#ifndef CHAIN_DEFER_LD
#define CHAIN_DEFER_LD 1     // I/O waves issue their next loads a step after staging (see the I/O loops)
#endif
#ifndef CHAIN_W_SLEEP
#define CHAIN_W_SLEEP 0      // chain_wait back-off: s_sleep argument (x 64 clocks) per nap unit (8 / 8: 0.284 ms/step,
#endif
#ifndef CHAIN_W_NAPMAX
#define CHAIN_W_NAPMAX 1     //   2 / 4: 0.278, 0 / 1: 0.275-0.277: lane 0's load latency paces the poll) and the largest nap
#endif
#ifndef CHAIN_RP_NAPMAX
#define CHAIN_RP_NAPMAX 16   // bulk re-poll of a stale tile: largest nap (s_sleep 2 units) between rounds
#endif
#ifndef CHAIN_H64_CPL2
#define CHAIN_H64_CPL2 1     // H = 64 forward stages: two cells per lane on 8 compute waves (see ChainCfg)
#endif
#ifndef CHAIN_PRIO
#define CHAIN_PRIO 2         // s_setprio of the compute waves of a stage with I/O waves
#endif
#ifndef CHAIN_LEAD3
#define CHAIN_LEAD3 1
#endif

struct ChainStage {
  const float* x;                    // stage 0: fp32 input [T][Mp][Din]
  const unsigned long long* xin;     // stages > 0: tagged input stream [T][Mp][Din]
  const float* W;
  const float* U;
  const float* b;
  float* h;                          // [T+1][Mp][H] (row T: scratch)
  __bf16* g;                         // train: [T+1][tiles][NW][CPL][64][4] packed bf16 gates
  float* c;
  unsigned long long* sout;          // tagged output stream [To][Mp][H] (nullptr: last stage)
  float* pout;                       // last stage only: own pooled output [T/P][Mp][H] (P > 0)
  unsigned* iout;
  float* pin_out;                    // PIN > 1: the pooled input [T][Mp][Din] + argmax bytes,
  unsigned char* pin_idx;            //   written here (the producer publishes unpooled h)
  long long* prof;                   // profiling (GNNQC_CHAIN_PROF=1): tile 0's per-step phase clocks
  int H, T, Din, Dw, KX, P, PIN;
};

struct ChainT4 {
  const unsigned long long* xin;     // the last chain stage's granule stream [>= 3 T][Mp][Din]
  const float* W;                    // [Dw][512]
  const float* U;                    // [128][512]
  const float* b;                    // [512]
  float* h;                          // [T][Mp][128]
  float* g;                          // train: [T][tiles][8][4][64][4] fp32 gates (time4_head.hip t4_sidx)
  float* c;                          // train: [T][tiles][8][4][64][2] (c_t, c_{t-1})
  float* pin_out;                    // pooled input [T][Mp][Din]: the chain stage's pooled output
  unsigned char* pin_idx;            //   and its argmax bytes
  int T, Din, Dw, on;
  ChainHead hd;
  float* hb;                         // train: the head backward precomputed here ([ntiles][16][128]
                                     // dh_{T-1} | records, dL/dloss = 1; nullptr: the backward runs it)
};

struct ChainArgs {
  ChainStage st[CHAIN_MAX];
  int ns, ntiles, nt8, Mp;
  int* ctl;                          // [0] epoch, [1] finished workgroups, [2] spin timeout seen
  long long* trace;                  // [blocks][2] start / end s_memrealtime (100 MHz) of the last launch
  // extra workgroups past the stages (the chain leaves most CUs idle): build the time4 kernel's
  // A-fragment image (lstm_tm_common.h t4_pack_one) from pkU / pkW into pk
  const float* pkU;
  const float* pkW;
  bf16x8_t* pk;
  int pkDw;
  int npk;                           // packing workgroups
  ChainT4 t4;                        // t4.on: time4 + head as one more stage (blocks [ns nt8, (ns + 1) nt8))
  // side job on the idle CUs: the GCN backward's coefficients (gcn_fused.h gcn_coef_fwd_body), one
  // workgroup per sample row; it only reads the store and writes its own buffer, nothing waits on it
  GcnCoefFwdJob cf;
  // gp.on: the GCN forward itself as producer workgroups (gcn_prod_body), one per sample row; the
  // first stage streams their tagged granules (st[0].xin) and the head waits for all of them
  // (ctl[10] counts them) before it reads the labels they write
  GcnProdJob gp;
};
static_assert(sizeof(ChainArgs) <= 4096, "chain forward kernel arguments");

__device__ __forceinline__ unsigned long long ld_granule(const unsigned long long* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ void st_granule(unsigned long long* p, float v, unsigned tag) {
  __hip_atomic_store(p, ((unsigned long long)tag << 32) | __float_as_uint(v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}

// slow path: lane 0 alone polls (its granule) with a growing back-off, then the wave checks
// every lane's granule. (All 64 lanes of every waiting wave polling back-to-back loaded the
// memory system enough to slow the running stages' own streams severalfold.)
template <bool INL>
__device__ __forceinline__ unsigned long long chain_wait_body(const unsigned long long* p, unsigned want, int* ctl);
#ifdef CHAIN_WAIT_INLINE
__device__ __forceinline__
#else
__device__ __noinline__
#endif
unsigned long long chain_wait(const unsigned long long* p, unsigned want, int* ctl) {
  return chain_wait_body<false>(p, want, ctl);
}
// inlined form for the forward I/O waves: a call in their step loop made the compiler drain vmcnt
// at the tag checks (the whole x ring waited for each step)
__device__ __forceinline__ unsigned long long chain_wait_inl(const unsigned long long* p, unsigned want, int* ctl) {
  return chain_wait_body<true>(p, want, ctl);
}
template <bool INL>
__device__ __forceinline__ unsigned long long chain_wait_body(const unsigned long long* p, unsigned want, int* ctl) {
  unsigned long long v = 0;
  const bool l0 = (threadIdx.x & 63) == 0;
#ifdef GQ_CHAIN_PROF
  if (l0) __hip_atomic_fetch_add(ctl + 9, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // re-polls (diagnostics)
#endif
  int nap = 1;
  // ctl[6] != 0: a debug spin limit (tests force a timeout with it)
  const int lim0 = __hip_atomic_load(ctl + 6, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const int lim = lim0 > 0 ? lim0 : CHAIN_SPIN;
  for (int it = 0; it < lim; ++it) {
    unsigned t0 = want;
    if (l0) t0 = (unsigned)(ld_granule(p) >> 32);
    if ((unsigned)__builtin_amdgcn_readfirstlane((int)t0) == want) {
      v = ld_granule(p);
      if (__builtin_amdgcn_ballot_w64((unsigned)(v >> 32) != want) == 0) return v;
    }
    for (int k = 0; k < nap; ++k) __builtin_amdgcn_s_sleep(CHAIN_W_SLEEP);
    nap = min(nap * 2, CHAIN_W_NAPMAX);
  }
  __hip_atomic_store(ctl + 2, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return v;
}

// one thread: wait (bounded, back-off) until the counter *p reaches n; the hand-off data behind it
// is read with agent-scope loads. A timeout flags the step (ctl[2]) as the granule waits do.
__device__ __forceinline__ void chain_wait_count(const int* p, int n, int* ctl) {
  const int lim0 = __hip_atomic_load(ctl + 6, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const int lim = lim0 > 0 ? lim0 : CHAIN_SPIN;
  int nap = 1;
  for (int it = 0; it < lim; ++it) {
    if (__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= n) return;
    for (int k = 0; k < nap; ++k) __builtin_amdgcn_s_sleep(CHAIN_W_SLEEP);
    nap = min(nap * 2, CHAIN_W_NAPMAX);
  }
  __hip_atomic_store(ctl + 2, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Per-step phase clocks of tile 0 (s_memtime: shader clock ticks) into pr[step][8] for the first
// CHAIN_PROF_STEPS steps; pr is workgroup-uniform (nullptr: off). Compiled in only with
// -DGQ_CHAIN_PROF (GNNQC_CHAIN_PROF_BUILD=1 at build time): even when off, the marks' clock reads
// and conditional stores kept the compiler from overlapping the step phases (chain forward 107 ->
// 131 us, backward 124 -> 155 us, measured).
static constexpr int CHAIN_PROF_STEPS = 64;
#ifdef GQ_CHAIN_PROF
__device__ __forceinline__ void chain_mark(long long* pr, int step, int k) {
  if (pr != nullptr && threadIdx.x == 0 && step < CHAIN_PROF_STEPS)
    pr[step * 8 + k] = (long long)__builtin_amdgcn_s_memtime();
}
// (the same from lane 0 of the calling wave: the forward's I/O waves)
__device__ __forceinline__ void chain_mark_wave(long long* pr, int step, int k) {
  if (pr != nullptr && (threadIdx.x & 63) == 0 && step < CHAIN_PROF_STEPS)
    pr[step * 8 + k] = (long long)__builtin_amdgcn_s_memtime();
}
#else
__device__ __forceinline__ void chain_mark(long long*, int, int) {}
__device__ __forceinline__ void chain_mark_wave(long long*, int, int) {}
#endif

// Tag base of a launch: (epoch mod (2^20 - 1)) + 1 in the high 20 bits of the 32-bit tag, the
// time index (< 4096) in the low 12. Never 0, so a zeroed granule (fresh or reused memory)
// can never pass as a valid one, whatever the epoch counter has wrapped to.
__device__ __forceinline__ unsigned chain_tag_base(unsigned E) { return ((E % 0xFFFFFu) + 1u) << 12; }

// One layer of one tile: lstm_tm_fwd_kernel's step with the x ring fed either from global memory
// (stage 0) or from the previous stage's granule stream (SRC), the output also published as granules.
// LDS of one stage (carved from the kernel's one buffer: the stage bodies must not each
// reserve their own static arrays)
template <int H, int KX>
struct ChainLds {
  static constexpr int HS = 2 * 16 * (TMC<H>::KPH + 8) * 2;
  static constexpr int XS = 2 * 16 * (32 * KX + 8) * 2;
  static constexpr int HF = 2 * 16 * TMC<H>::HP * 4;
  // (stages with a publisher wave: H <= 32, and H = 64 in its two-cells-per-lane layout) the cells'
  // packed gates and c of two steps
  static constexpr bool PUB = H <= 32 || CHAIN_H64_CPL2;
  static constexpr int GS = PUB ? 2 * 16 * H * 8 : 0;
  static constexpr int CS = PUB ? 2 * 16 * H * 4 : 0;
  static constexpr int BYTES = HS + XS + HF + GS + CS;
};
constexpr int chain_max2(int a, int b) { return a > b ? a : b; }
static constexpr int CHAIN_LDS_STAGE = chain_max2(chain_max2(ChainLds<64, 2>::BYTES, ChainLds<32, 2>::BYTES),
                                                  ChainLds<16, 2>::BYTES);

// Gate scaling: sigmoid(z) = 1 / (1 + 2^(-z log2 e)), tanh(z) = 2 / (1 + 2^(-2 z log2 e)) - 1, one
// v_exp_f32 each after one multiply. (Folding the scale into the bf16 weight fragments saved the
// multiplies but rounded W log2(e) instead of W: the kernels' rounding no longer matched the other
// LSTM kernels' and the numerics oracle, so the weights stay unscaled.)
__device__ __forceinline__ float chain_gate_scale(int ag) { return ag == 2 ? -2.8853900817779268f : -1.4426950408889634f; }

// Roles of a stage workgroup. H = 16 / 32: waves [0, NW) compute the cells and store their own
// outputs straight from registers (h, the granule that publishes it, the packed gates and c for the
// backward); they issue no global load, so no s_waitcnt vmcnt ever waits on their write-through
// stores. D more waves (the I/O waves) take turns streaming x: I/O wave k loads the whole [16][Din]
// tile of every step s = k (mod D) D steps ahead and, in step s - 1, waits for it (its own loads
// only: a plain vmcnt(0)), checks the tags (re-polls a stale granule), max-pools PIN consecutive
// steps (writing the pooled input and the argmax bytes for the backward) and writes x_s into the
// LDS tile of the next step. (A register ring of D slots in one wave was the first form: the
// compiler's wait insertion drained the whole ring at the top of every unrolled round.) For a last
// stage that pools its own output, I/O wave 0 pools h from the fp32 LDS tile. One LDS barrier per
// step. H = 64 fills a 1024-thread workgroup with compute waves: there every thread also streams x
// through a D-slot register ring, as one role.
// (only when they fit the 1024-thread workgroup and a lane's share of one step's tile - ngl granules
// of pin steps each - stays within 24 registers pairs; else every thread streams, as for H = 64)
__host__ __device__ constexpr int chain_io_waves(int nt, int d, int ngl = 1, int pin = 1) {
  return nt + 64 * d + 64 <= 1024 && ngl * pin <= 12 ? d : 0;   // (+ the publisher wave)
}
// a pooling consumer (pin = 3 granules per element) splits each step's tile over two I/O waves
// (and so does a 64-channel input of an H = 64 stage, 8 granule pairs per lane in one wave: its I/O
// waves' registers spilled; with two waves per step the ring is 3 steps deep to fit the workgroup)
__host__ __device__ constexpr int chain_io_group(int pin, int kx = 1, int h = 16) {
  return pin > 1 || (h == 64 && kx == 2 && CHAIN_H64_CPL2) ? 2 : 1;
}
__host__ __device__ constexpr int chain_stage_d(int h, int kx, int d) {
  return h == 64 && kx == 2 && CHAIN_H64_CPL2 && d > 3 ? 3 : d;
}
// threads of a stage workgroup that run the stage (compute + I/O waves + the publisher)
__host__ __device__ constexpr int chain_live_threads(int nt, int d, int kx, bool src, int pin, int h = 16) {
  return nt + 64 * chain_io_waves(nt, d * chain_io_group(pin, kx, h),
                                  (16 * 32 * kx / (src ? 2 : 4) + 64 * chain_io_group(pin, kx, h) - 1) /
                                      (64 * chain_io_group(pin, kx, h)),
                                  pin) +
         (chain_io_waves(nt, d * chain_io_group(pin, kx, h),
                         (16 * 32 * kx / (src ? 2 : 4) + 64 * chain_io_group(pin, kx, h) - 1) /
                             (64 * chain_io_group(pin, kx, h)),
                         pin) > 0 ? 64 : 0);
}

// Compute layout of a forward chain stage: one cell per lane (as TMC), except H = 64, which runs two
// cells per lane on 8 compute waves so that the I/O waves and the publisher fit the 1024-thread
// workgroup too (with 16 compute waves every thread streamed its own x granules and stored its own
// outputs, and its loads waited behind its write-through stores). The saved gates / c keep the
// one-cell-per-lane layout of the backward (cell (wave gi, lane), gi = compute wave + NW * cc).
template <int H>
struct ChainCfg {
  static constexpr int CPL = (H == 64 && CHAIN_H64_CPL2) ? 2 : 1;
  static constexpr int NW = H / 4 / CPL, NT = 64 * NW, G4 = 4 * H;
  static constexpr int KSH = TMC<H>::KSH, KPH = TMC<H>::KPH, HP = TMC<H>::HP;
  static constexpr int NWV = H / 4, NCELL = 64 * NWV;     // the saved-state layout's waves / cells per tile
};

template <int H, bool TRAIN, int KX, int D, bool SRC, int PIN>
__device__ __forceinline__ void chain_stage(const ChainStage& S, int tile, int ntiles, int Mp, unsigned tagb,
                                            int* ctl, char* smem) {
  using C = ChainCfg<H>;
  constexpr int NW = C::NW, NT = C::NT, G4 = C::G4, CPL = C::CPL, NWV = C::NWV, NCELL = C::NCELL;
  constexpr int KPX = 32 * KX;
  // elements per streamed granule: stage 0 reads float4 of x; a stream consumer reads two adjacent
  // 8-byte {value, tag} granules with one 16-byte load (each half is one whole granule)
  constexpr int GR = SRC ? 2 : 4;
  constexpr int G = chain_io_group(PIN, KX, H);  // I/O waves sharing one step's tile
  constexpr int NIOW = chain_io_waves(NT, D * G, (16 * KPX / GR + 64 * G - 1) / (64 * G), PIN);   // (0: none)
  constexpr bool IOW = NIOW > 0;
  constexpr int NIO = IOW ? 64 * G : NT;         // threads streaming one step's tile
  constexpr int NSLOT = IOW ? 1 : D;             // x slots per streaming thread
  // granules per streaming lane: I/O waves cover the largest tile the template allows; without
  // them every thread streams one granule (the host requires 16 Din / GR <= NT then)
  constexpr int NGL = IOW ? (16 * KPX / GR + NIO - 1) / NIO : 1;
  using L = ChainLds<H, KX>;
  static_assert(L::BYTES <= CHAIN_LDS_STAGE && L::HS % 16 == 0 && L::XS % 16 == 0, "chain LDS layout");
  auto hs = reinterpret_cast<__bf16 (*)[16][C::KPH + 8]>(smem);
  auto xs = reinterpret_cast<__bf16 (*)[16][KPX + 8]>(smem + L::HS);
  auto hf = reinterpret_cast<float (*)[16][C::HP]>(smem + L::HS + L::XS);
  auto gst = reinterpret_cast<uint2 (*)[NCELL]>(smem + L::HS + L::XS + L::HF);            // [2][cells] (IOW)
  auto cst = reinterpret_cast<float (*)[NCELL]>(smem + L::HS + L::XS + L::HF + L::GS);   // [2][cells] (IOW)

  const int T = S.T, Din = S.Din, Dw = S.Dw, P = S.P;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int col = lane & 15, quad = lane >> 4;
  const int row0 = tile * 16;
  const size_t hstep = (size_t)Mp * H;
  const int To = P > 0 ? T / P : T;      // (P > 0 only without a consumer stage)

  constexpr int NTL = NT + 64 * NIOW + (IOW ? 64 : 0);   // live threads (the rest exited)
  for (int i = tid; i < 2 * 16 * (C::KPH + 8); i += NTL) (&hs[0][0][0])[i] = (__bf16)0.0f;
  for (int i = tid; i < 2 * 16 * (KPX + 8); i += NTL) (&xs[0][0][0])[i] = (__bf16)0.0f;

  // ---- x streaming: lane iot of a streaming wave / thread block owns granules iot + NIO j of the
  // contiguous [16][Din] tile (mod n_gx: duplicate lanes load and write the same values; no branch
  // around a load - the compiler drains vmcnt at the join of one)
  const bool compute = w < NW;
  const int iow = IOW ? (w - NW) / G : 0;        // I/O wave group (IOW): steps s = iow (mod D)
  const int iot = IOW ? ((w - NW) % G) * 64 + lane : tid;
  const int n_gx = 16 * Din / GR;
  const size_t xstep = (size_t)Mp * Din;
  // per granule: its element offset in the tile (32 bits; the tile of step tx starts at element
  // (tx Mp + row0) Din) and its LDS byte offset in the bf16 x tile
  int goff[NGL], loff[NGL];
#pragma unroll
  for (int j = 0; j < NGL; ++j) {
    const int gx = min(iot + NIO * j, n_gx - 1) * GR;
    goff[j] = gx;
    loff[j] = ((gx / Din) * (KPX + 8) + gx % Din) * 2;
  }
  const size_t xbase = (size_t)row0 * Din;
  char* xsb = reinterpret_cast<char*>(&xs[0][0][0]);
  constexpr int XBUF = 16 * (KPX + 8) * 2;       // bytes of one x tile buffer
  // (x granules as whole vectors: a float[4] ring was split into scalars and the compiler copied
  // lanes of a just-issued load into the loop-carried registers - an immediate vmcnt wait for the
  // full memory latency in every staging step)
  f32x4_t xr[NSLOT][NGL];
  u64x2_t xq[NSLOT][NGL][PIN];
  // (SRC: L1-bypassing 16-byte buffer loads of the granule stream; byte offsets < 2^32, host-checked)
  const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<unsigned long long*>(SRC ? S.xin : nullptr), (short)0, 0x7fffffff, 0x00020000);
  auto load_x = [&](int r, int tx) {
#pragma unroll
    for (int q = 0; q < (SRC ? PIN : 1); ++q) {
      const size_t tb = xbase + (size_t)(SRC ? PIN * tx + q : tx) * xstep;
#pragma unroll
      for (int j = 0; j < NGL; ++j) {
        if constexpr (SRC) {
#if CHAIN_LD16
          const u32x4_t v = __builtin_amdgcn_raw_buffer_load_b128(xrs, (int)((tb + goff[j]) * 8), 0, 16);
          xq[r][j][q] = u64x2_t{((unsigned long long)v.y << 32) | v.x, ((unsigned long long)v.w << 32) | v.z};
#else
          xq[r][j][q] = u64x2_t{ld_granule(S.xin + tb + goff[j]), ld_granule(S.xin + tb + goff[j] + 1)};
#endif
        } else {
          xr[r][j] = *reinterpret_cast<const f32x4_t*>(S.x + tb + goff[j]);
        }
      }
    }
  };
  auto stage_x = [&](int buf, int r, int tx) {
    if constexpr (SRC) {
      // every granule's tag first (one ballot), the re-poll only on a miss
      bool bad = false;
#pragma unroll
      for (int j = 0; j < NGL; ++j)
#pragma unroll
        for (int q = 0; q < PIN; ++q) {
          const unsigned want = tagb | (unsigned)(PIN * tx + q);
          bad |= (unsigned)(xq[r][j][q].x >> 32) != want || (unsigned)(xq[r][j][q].y >> 32) != want;
        }
      if (__builtin_amdgcn_ballot_w64(bad) != 0) {
        // re-poll: every granule of the tile re-loaded AT ONCE per round (one memory round trip a
        // round, not one per granule), short back-off, bounded (a timeout flags the step)
#ifdef GQ_CHAIN_PROF
        if (lane == 0) __hip_atomic_fetch_add(ctl + 9, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#endif
        const int lim0 = __hip_atomic_load(ctl + 6, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int lim = lim0 > 0 ? lim0 : CHAIN_SPIN;
        int nap = 1;
        for (int it = 0;; ++it) {
#pragma unroll
          for (int q = 0; q < PIN; ++q) {
            const size_t tb = xbase + (size_t)(PIN * tx + q) * xstep;
#pragma unroll
            for (int j = 0; j < NGL; ++j)
              xq[r][j][q] = u64x2_t{ld_granule(S.xin + tb + goff[j]), ld_granule(S.xin + tb + goff[j] + 1)};
          }
          bad = false;
#pragma unroll
          for (int j = 0; j < NGL; ++j)
#pragma unroll
            for (int q = 0; q < PIN; ++q) {
              const unsigned want = tagb | (unsigned)(PIN * tx + q);
              bad |= (unsigned)(xq[r][j][q].x >> 32) != want || (unsigned)(xq[r][j][q].y >> 32) != want;
            }
          if (__builtin_amdgcn_ballot_w64(bad) == 0) break;
          if (it >= lim) {
            __hip_atomic_store(ctl + 2, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            break;
          }
          for (int k = 0; k < nap; ++k) __builtin_amdgcn_s_sleep(2);
          nap = min(nap * 2, CHAIN_RP_NAPMAX);
        }
      }
      const size_t po = xbase + (size_t)tx * xstep;
#pragma unroll
      for (int j = 0; j < NGL; ++j) {
        float m0 = __uint_as_float((unsigned)xq[r][j][0].x), m1 = __uint_as_float((unsigned)xq[r][j][0].y);
        if constexpr (PIN > 1) {
          unsigned a0 = 0, a1 = 0;
#pragma unroll
          for (int q = 1; q < PIN; ++q) {
            const float v0 = __uint_as_float((unsigned)xq[r][j][q].x), v1 = __uint_as_float((unsigned)xq[r][j][q].y);
            if (v0 > m0) { m0 = v0; a0 = q; }
            if (v1 > m1) { m1 = v1; a1 = q; }
          }
          *reinterpret_cast<float2*>(S.pin_out + po + goff[j]) = make_float2(m0, m1);
          *reinterpret_cast<unsigned short*>(S.pin_idx + po + goff[j]) = (unsigned short)(a0 | (a1 << 8));
        }
        *reinterpret_cast<bf16x2_t*>(xsb + buf * XBUF + loff[j]) = bf16x2_t{(__bf16)m0, (__bf16)m1};
      }
    } else {
#pragma unroll
      for (int j = 0; j < NGL; ++j) {
        // GR = 4 consecutive channels of one sequence (Din % 4 == 0): one 8-byte LDS write
        const bf16x4_t v = __builtin_convertvector(xr[r][j], bf16x4_t);
        *reinterpret_cast<bf16x4_t*>(xsb + buf * XBUF + loff[j]) = v;
      }
    }
  };

  // ---- compute role: fragments of the pre-scaled gate weights, one cell (unit, sequence) per lane
  const int wc = compute ? w : 0;
  const int ag = col & 3;
  int unit[CPL];
  bf16x8_t ufr[CPL][C::KSH], wfr[CPL][KX];
  f32x4_t bias4[CPL];
#pragma unroll
  for (int cc = 0; cc < CPL; ++cc) {
    const int gi = wc + NW * cc;                 // (the cell group: a one-cell-per-lane wave)
    const int au = 4 * gi + (col >> 2);
    unit[cc] = 4 * gi + quad;
    bias4[cc] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    if (compute) {
#pragma unroll
      for (int s = 0; s < C::KSH; ++s) {
        bf16x8_t v;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int k = 32 * s + 8 * quad + j;
          v[j] = (__bf16)(S.U[min(k, H - 1) * G4 + ag * H + au] * (k < H ? 1.0f : 0.0f));
        }
        ufr[cc][s] = v;
      }
#pragma unroll
      for (int s = 0; s < KX; ++s) {
        bf16x8_t v;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int k = 32 * s + 8 * quad + j;
          v[j] = (__bf16)(S.W[min(k, Dw - 1) * G4 + ag * H + au] * (k < Dw ? 1.0f : 0.0f));
        }
        wfr[cc][s] = v;
      }
      const int u = unit[cc];
      bias4[cc] = f32x4_t{S.b[u], S.b[H + u], S.b[2 * H + u], S.b[3 * H + u]};
    }
  }
  // this lane's output elements (sequence row0 + col, unit) in the [T][Mp][H] streams
  float* hp[CPL];
  unsigned long long* sp[CPL];
  __bf16* gp[CPL];
  float* cp[CPL];
  const size_t gstride = (size_t)ntiles * NWV * 64;
#pragma unroll
  for (int cc = 0; cc < CPL; ++cc) {
    const size_t hoff = (size_t)(row0 + col) * H + unit[cc];
    hp[cc] = S.h + hoff;
    sp[cc] = S.sout != nullptr ? S.sout + hoff : nullptr;
    gp[cc] = S.g + (((size_t)tile * NWV + wc + NW * cc) * 64 + lane) * 4;
    cp[cc] = S.c + ((size_t)tile * NWV + wc + NW * cc) * 64 + lane;
  }
  const bool publish = S.sout != nullptr;
  const bool own_pool = P > 0;

  // ---- a last stage that pools its own output: the pooling lanes (I/O wave 0, or the first 16 H / 4
  // threads) own float4 granules of the [16][H] tile
  constexpr int n_gh = 16 * H / 4;
  constexpr int NPT = IOW ? 64 : NT;             // pooling threads (the publisher wave, or every thread)
  constexpr int NPL = (n_gh + NPT - 1) / NPT;
  PoolAcc pool[NPL];
  const bool publisher = IOW && w == NW + NIOW;
  const bool pooler = IOW ? publisher : wave_uniform(tid < n_gh);
  auto pool_step = [&](int tp) {           // h_tp from hf[tp & 1]
#pragma unroll
    for (int q = 0; q < NPL; ++q) {
      const int gh = (((IOW ? lane : tid) + NPT * q) % n_gh) * 4;
      const float4 v = *reinterpret_cast<const float4*>(&hf[tp & 1][gh / H][gh % H]);
      pool[q].step(v, tp, P, To, S.pout, S.iout, (size_t)row0 * H + gh, hstep);
    }
  };

  // ---- prologue: x_0 in LDS buffer 0, the first D steps' loads in flight
  const bool streamer = IOW ? (!compute && !publisher) : true;
  if (streamer) {
    if constexpr (SRC) {
      // start once the producer is D + LEAD (input) steps ahead: the loads then find their
      // granules. (Starting at once left every load stale: each of the first D steps then paid a
      // full re-poll round trip, ~12 us of lag per stage.)
      constexpr int LEAD = PIN > 1 ? CHAIN_LEAD3 : CHAIN_LEAD1;
      const int tw = min(D + LEAD, T - 1);
      (void)chain_wait(S.xin + xbase + goff[0] + 1 + (size_t)(PIN * tw + PIN - 1) * xstep,
                       tagb | (unsigned)(PIN * tw + PIN - 1), ctl);
    }
    if constexpr (IOW) {
      load_x(0, min(iow, T - 1));            // I/O wave k: x_k
    } else {
#pragma unroll
      for (int r = 0; r < D; ++r) load_x(r, min(r, T - 1));
    }
  }
  __syncthreads();
  if (IOW ? (streamer && iow == 0) : streamer) {
    stage_x(0, 0, 0);
    if (!IOW || !CHAIN_DEFER_LD) load_x(0, min(D, T - 1));
  }
  float c[CPL];
#pragma unroll
  for (int cc = 0; cc < CPL; ++cc) c[cc] = 0.f;
  __syncthreads();

  long long* pr = (S.prof != nullptr && tile == 0) ? S.prof : nullptr;
  // the compute step of time t (reads xs[p], hs[p]; writes hs[p ^ 1], the outputs)
  auto compute_step = [&](int t, auto IO, int rn) {
    constexpr bool DOI = decltype(IO)::value;
    const int p = t & 1;
    chain_mark(pr, t, 0);
    f32x4_t acc[CPL];
#pragma unroll
    for (int cc = 0; cc < CPL; ++cc) {
      f32x4_t accx = bias4[cc], acch = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < KX; ++s) {
        const bf16x8_t bx = *reinterpret_cast<const bf16x8_t*>(&xs[p][col][32 * s + 8 * quad]);
        accx = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wfr[cc][s], bx, accx, 0, 0, 0);
      }
#pragma unroll
      for (int s = 0; s < C::KSH; ++s) {
        const bf16x8_t bh = *reinterpret_cast<const bf16x8_t*>(&hs[p][col][32 * s + 8 * quad]);
        acch = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ufr[cc][s], bh, acch, 0, 0, 0);
      }
      acc[cc] = accx + acch;
    }
    chain_mark(pr, t, 1);
    if constexpr (DOI) {                 // (H = 64: every thread also streams x through its ring)
      stage_x(p ^ 1, rn, min(t + 1, T - 1));
      load_x(rn, min(t + 1 + D, T - 1));
    }
#pragma unroll
    for (int cc = 0; cc < CPL; ++cc) {
      const f32x4_t a = acc[cc];
      const int u = unit[cc], cell = (wc + NW * cc) * 64 + lane;
      const float iv = __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(chain_gate_scale(0) * a[0]));
      const float fv = __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(chain_gate_scale(1) * a[1]));
      const float gv = 2.0f * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(chain_gate_scale(2) * a[2])) - 1.0f;
      const float ov = __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(chain_gate_scale(3) * a[3]));
      c[cc] = fv * c[cc] + iv * gv;
      const float rc = __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-2.8853900817779268f * c[cc]));
      const float hv = (2.0f * ov) * rc - ov;            // o tanh(c)
      hs[p ^ 1][col][u] = (__bf16)hv;
      // the granule that publishes h_t goes out at once, from registers (write-through: the consumer
      // polls it); the bulk outputs (h, packed gates, c) are staged in LDS for the publisher wave, whose
      // wide contiguous stores keep the CU's vector-memory path free for the consumer-side loads
      if (publish) st_granule(sp[cc] + (size_t)t * hstep, hv, tagb | (unsigned)t);
      if constexpr (IOW) {
        hf[p][col][u] = hv;
        if constexpr (TRAIN) {
          gst[p][cell] = gates_pack(iv, fv, gv, ov);
          cst[p][cell] = c[cc];
        }
      } else {
        if (own_pool) hf[p][col][u] = hv;
        hp[cc][(size_t)t * hstep] = hv;
        if constexpr (TRAIN) {
          *reinterpret_cast<uint2*>(gp[cc] + (size_t)t * gstride * 4) = gates_pack(iv, fv, gv, ov);
          cp[cc][(size_t)t * gstride] = c[cc];
        }
      }
    }
    chain_mark(pr, t, 2);
  };
  // publisher wave: step tp's h tile, gates and c from LDS buffer tp & 1 with 16-byte stores; a whole
  // [16][H] row block of the time-major streams is contiguous. (Publishing the granules from here as
  // well, a step later with 16-byte write-through buffer stores, timed out: consumers never saw them.)
  auto publish_step = [&](int tp) {
    const int pb = tp & 1;
    const size_t tile_off = ((size_t)tp * Mp + row0) * H;
#pragma unroll
    for (int q = lane; q < 16 * H / 4; q += 64) {
      const int e = 4 * q;
      *reinterpret_cast<float4*>(S.h + tile_off + e) = *reinterpret_cast<const float4*>(&hf[pb][e / H][e % H]);
    }
    if constexpr (TRAIN) {
      const size_t cell0 = ((size_t)tp * ntiles + tile) * NCELL;      // this tile's cells of step tp
#pragma unroll
      for (int q = lane; q < NCELL / 2; q += 64)
        *reinterpret_cast<uint4*>(S.g + (cell0 + 2 * q) * 4) = *reinterpret_cast<const uint4*>(&gst[pb][2 * q]);
#pragma unroll
      for (int q = lane; q < NCELL / 4; q += 64)
        *reinterpret_cast<float4*>(S.c + cell0 + 4 * q) = *reinterpret_cast<const float4*>(&cst[pb][4 * q]);
    }
    if (own_pool) pool_step(tp);
  };
  using yes = std::true_type;
  using no = std::false_type;
  if constexpr (IOW) {
    if (compute) {
      if (CHAIN_PRIO > 0) __builtin_amdgcn_s_setprio(CHAIN_PRIO);   // the serial cell math issues first on a shared SIMD
      for (int t = 0; t < T; ++t) {
        compute_step(t, no{}, 0);
        lds_barrier();
        chain_mark(pr, t, 3);
      }
      __builtin_amdgcn_s_setprio(0);
    } else if (publisher) {
      for (int t = 0; t < T; ++t) {
        if (t >= 1) publish_step(t - 1);
        chain_mark_wave(pr, t, 7);         // (the publisher reaches the step barrier)
        lds_barrier();
      }
      publish_step(T - 1);
    } else {
      // I/O wave k stages the steps s = k (mod D): x_{t+1} in step t, then loads x_{t+1+D}
      // the group's next loads are issued at the top of the step AFTER its staging step (right after
      // that barrier, beside the compute waves' cell math) instead of before the barrier they would
      // hold up; they still land D - 1 steps ahead of their use
      int kt = (iow + D - 1) % D;        // steps until this wave's turn: t = kt, kt + D, ...
      int next_ld = iow == 0 ? D : -1;   // (group 0 staged x_0 in the prologue)
      for (int t = 0; t < T; ++t) {
        if (CHAIN_DEFER_LD && next_ld >= 0) {
          load_x(0, min(next_ld, T - 1));
          next_ld = -1;
        }
        if (kt == 0 && t + 1 < T) {
          if (iot == 0) chain_mark_wave(pr, t, 4);
          stage_x((t + 1) & 1, 0, t + 1);
          if (iot == 0) chain_mark_wave(pr, t, 5);
          if (CHAIN_DEFER_LD) next_ld = t + 1 + D;
          else load_x(0, min(t + 1 + D, T - 1));
          if (iot == 0) chain_mark_wave(pr, t, 6);
        }
        kt = kt == 0 ? D - 1 : kt - 1;
        lds_barrier();
      }
    }
  } else {
    for (int t0 = 0; t0 < T; t0 += D) {
#pragma unroll
      for (int r = 0; r < D; ++r) {
        const int t = t0 + r;
        if (t >= T) break;               // (uniform: the last round of the ring may be partial)
        compute_step(t, yes{}, (r + 1 == D) ? 0 : r + 1);
        if (own_pool && pooler && t >= 1) pool_step(t - 1);
        lds_barrier();
        chain_mark(pr, t, 3);
      }
    }
  }
  if constexpr (!IOW) {
    if (own_pool && pooler) pool_step(T - 1);
  }
}

// ---- time4 (H = 128, the CML TimeLayer's last layer, last state only) + head + weighted BCE as one
// more consumer stage of the forward chain (lstm_chain_head_fwd). As its own launch
// (time4_head.hip) it could only start once the whole chain had drained, and its six steps plus
// the head (~22 us) ran serially behind it. Here one workgroup per tile consumes the last chain
// stage's UNPOOLED granules, max-pools them (MaxPooling1D(3); the pooled input and the argmax
// bytes are written for the backward) and runs each step as soon as its three input steps are
// published; the head and the loss follow the last step. 1024 threads with two cells per lane
// (the chain kernel's launch bounds give a lane 128 VGPRs; the standalone kernel's four cells per
// lane need 256). time4_head.hip's saved-state layouts (h; fp32 gates and (c_t, c_{t-1}) in its
// t4_sidx order) are kept, so its backward is unchanged.
struct ChainT4Lds {
  static constexpr int HS = 2 * 16 * (128 + 8) * 2;       // bf16 h_{t-1} (double buffer)
  static constexpr int XS = 2 * 16 * (64 + 8) * 2;        // bf16 x_t (double buffer)
  static constexpr int HL = 16 * (128 + 4) * 4;           // fp32 h_{T-1} for the head
  static constexpr int DHT = 16 * (128 + 4) * 4;          // precomputed head backward: dh_{T-1}
  // (the head backward's dh tile and scratch follow the head forward's, whose weight images it reuses)
  static constexpr int HF = ChainHeadFwdLds<128>::BYTES;
  static constexpr int HB = DHT + ChainHeadBwdLds<128>::BYTES - (128 + CH_HU) * CH_WP * 4;   // (no weight images)
  static constexpr int BYTES = HS + XS + HL + HF + HB;
};

template <bool TRAIN>
__device__ __forceinline__ void chain_t4_stage(const ChainT4 Q, int tile, int ntiles, int Mp, unsigned tagb, int* ctl,
                                               char* smem) {
  constexpr int H = 128, G4 = 4 * H, NW = 16, CPL = 2, KX = 2, KSH = H / 32, HPB = H + 8, XP = 64 + 8;
  static_assert(ChainT4Lds::HS % 16 == 0 && ChainT4Lds::XS % 16 == 0 && ChainT4Lds::HL % 16 == 0, "t4 LDS layout");
  auto hs = reinterpret_cast<__bf16 (*)[16][HPB]>(smem);
  auto xs = reinterpret_cast<__bf16 (*)[16][XP]>(smem + ChainT4Lds::HS);
  float* hl = reinterpret_cast<float*>(smem + ChainT4Lds::HS + ChainT4Lds::XS);
  const int T = Q.T, Din = Q.Din, Dw = Q.Dw;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int col = lane & 15, quad = lane >> 4;
  const int row0 = tile * 16;

  for (int i = tid; i < 2 * 16 * HPB; i += 1024) (&hs[0][0][0])[i] = (__bf16)0.0f;
  for (int i = tid; i < 2 * 16 * XP; i += 1024) (&xs[0][0][0])[i] = (__bf16)0.0f;
  // input element of this thread: (sequence er, channel ek) of the [16][Din] tile; threads past
  // the tile re-load the last element (every lane of a waiting wave must hold a real granule)
  const int n_el = 16 * Din;
  const bool own = tid < n_el;
  const int el = min(tid, n_el - 1), er = el / Din, ek = el % Din;
  const size_t xstep = (size_t)Mp * Din, xoff = (size_t)(row0 + er) * Din + ek;
  unsigned long long xq[3];
  auto load_x = [&](int tx) {
#pragma unroll
    for (int r = 0; r < 3; ++r) xq[r] = ld_granule(Q.xin + xoff + (size_t)(3 * tx + r) * xstep);
  };
  // the first input's granules are requested before the weight gathers (their latency overlaps)
  load_x(0);

  // weights -> permuted A fragments (as chain_stage) straight from global memory: the gathers'
  // latency is hidden behind the wait for the first input
  bf16x8_t ufr[CPL][KSH], wfr[CPL][KX];
  f32x4_t bias4[CPL];
  int unit[CPL];
#pragma unroll
  for (int cc = 0; cc < CPL; ++cc) {
    const int gi = w + NW * cc;
    const int au = 4 * gi + (col >> 2), ag = col & 3;
    unit[cc] = 4 * gi + quad;
#pragma unroll
    for (int s = 0; s < KSH; ++s) {
      bf16x8_t v;
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = (__bf16)Q.U[(32 * s + 8 * quad + j) * G4 + ag * H + au];
      ufr[cc][s] = v;
    }
#pragma unroll
    for (int s = 0; s < KX; ++s) {
      bf16x8_t v;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int k = 32 * s + 8 * quad + j;
        v[j] = (__bf16)(Q.W[min(k, Dw - 1) * G4 + ag * H + au] * (k < Dw ? 1.0f : 0.0f));
      }
      wfr[cc][s] = v;
    }
    const int u = unit[cc];
    bias4[cc] = f32x4_t{Q.b[u], Q.b[H + u], Q.b[2 * H + u], Q.b[3 * H + u]};
  }

  // x_tx = MaxPool(3) of the producer's h at 3 tx .. 3 tx + 2 (first maximum wins, its byte kept)
  auto stage_x = [&](int buf, int tx) {
    bool bad = false;
#pragma unroll
    for (int r = 0; r < 3; ++r) bad |= (unsigned)(xq[r] >> 32) != (tagb | (unsigned)(3 * tx + r));
    if (__builtin_amdgcn_ballot_w64(bad) != 0) {
      // re-poll all three granules at once, inline (a call to chain_wait here made the compiler keep
      // live registers in scratch around it: two scratch reloads in every step of this loop)
      const int lim0 = __hip_atomic_load(ctl + 6, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int lim = lim0 > 0 ? lim0 : CHAIN_SPIN;
      for (int it = 0;; ++it) {
        __builtin_amdgcn_s_sleep(1);
#pragma unroll
        for (int r = 0; r < 3; ++r) xq[r] = ld_granule(Q.xin + xoff + (size_t)(3 * tx + r) * xstep);
        bad = false;
#pragma unroll
        for (int r = 0; r < 3; ++r) bad |= (unsigned)(xq[r] >> 32) != (tagb | (unsigned)(3 * tx + r));
        if (__builtin_amdgcn_ballot_w64(bad) == 0) break;
        if (it >= lim) {
          __hip_atomic_store(ctl + 2, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
      }
    }
    float m = __uint_as_float((unsigned)xq[0]);
    unsigned arg = 0;
#pragma unroll
    for (int r = 1; r < 3; ++r) {
      const float v = __uint_as_float((unsigned)xq[r]);
      if (v > m) { m = v; arg = r; }
    }
    if (own) {
      Q.pin_out[xoff + (size_t)tx * xstep] = m;
      Q.pin_idx[xoff + (size_t)tx * xstep] = (unsigned char)arg;
      xs[buf][er][ek] = (__bf16)m;
    }
  };

  __syncthreads();                                // LDS zeroed
  stage_x(0, 0);
  if (T > 1) load_x(1);
  float c[CPL];
#pragma unroll
  for (int cc = 0; cc < CPL; ++cc) c[cc] = 0.f;
  __syncthreads();

  for (int t = 0; t < T; ++t) {
    const int p = t & 1;
    f32x4_t acc[CPL];
#pragma unroll
    for (int cc = 0; cc < CPL; ++cc) {
      f32x4_t accx = bias4[cc], acch = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < KX; ++s) {
        const bf16x8_t bx = *reinterpret_cast<const bf16x8_t*>(&xs[p][col][32 * s + 8 * quad]);
        accx = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wfr[cc][s], bx, accx, 0, 0, 0);
      }
#pragma unroll
      for (int s = 0; s < KSH; ++s) {
        const bf16x8_t bh = *reinterpret_cast<const bf16x8_t*>(&hs[p][col][32 * s + 8 * quad]);
        acch = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ufr[cc][s], bh, acch, 0, 0, 0);
      }
      acc[cc] = accx + acch;
    }
    if (wave_uniform(t + 1 < T)) {
      stage_x(p ^ 1, t + 1);
      if (wave_uniform(t + 2 < T)) load_x(t + 2);
    }
#pragma unroll
    for (int cc = 0; cc < CPL; ++cc) {
      const float iv = sigmoidf_fast(acc[cc][0]);
      const float fv = sigmoidf_fast(acc[cc][1]);
      const float gv = tanhf_fast(acc[cc][2]);
      const float ov = sigmoidf_fast(acc[cc][3]);
      const float cold = c[cc];
      c[cc] = fv * cold + iv * gv;
      const float hv = ov * tanhf_fast(c[cc]);
      const int u = unit[cc];
      hs[p ^ 1][col][u] = (__bf16)hv;
      Q.h[((size_t)t * Mp + row0 + col) * H + u] = hv;
      if (t == T - 1) hl[col * (H + 4) + u] = hv;
      if constexpr (TRAIN) {
        const int gi = w + NW * cc;                 // time4_head.hip's (wave, cell) of this cell
        const size_t o = ((((size_t)t * ntiles + tile) * 8 + (gi & 7)) * 4 + (gi >> 3)) * 64 + lane;
        *reinterpret_cast<float4*>(Q.g + o * 4) = make_float4(iv, fv, gv, ov);
        *reinterpret_cast<float2*>(Q.c + o * 2) = make_float2(c[cc], cold);
      }
    }
    lds_barrier();
  }
  __syncthreads();
}

__device__ __forceinline__ void chain_finish(int* ctl, int nblk) {
  if (threadIdx.x == 0) {
    const int old = __hip_atomic_fetch_add(ctl + 1, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (old == nblk - 1) {            // last workgroup: next launch gets a new epoch
      __hip_atomic_store(ctl + 1, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(ctl + 10, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // (GCN producers)
      __hip_atomic_fetch_add(ctl, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

static constexpr int CHAIN_LDS = ChainT4Lds::BYTES > CHAIN_LDS_STAGE ? ChainT4Lds::BYTES : CHAIN_LDS_STAGE;

template <bool TRAIN>
__global__ __launch_bounds__(1024) void lstm_chain_fwd_kernel(ChainArgs A) {
  const int nblk = gridDim.x;
  __shared__ __attribute__((aligned(16))) char smem[CHAIN_LDS];
  if ((int)blockIdx.x >= A.ns * A.nt8) {
    int r = (int)blockIdx.x - A.ns * A.nt8;
    if (A.t4.on) {
      if (r < A.nt8) {                            // time4 + head stage of tile r
        if (r < A.ntiles) {
          if (threadIdx.x == 0) A.trace[2 * blockIdx.x] = (long long)__builtin_amdgcn_s_memrealtime();
          const unsigned tagb = chain_tag_base((unsigned)__hip_atomic_load(A.ctl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
          // the head's weight images go to LDS first: this workgroup then waits ~60 us for its first
          // input anyway (the chain's stages are all far behind), and the head runs right after the
          // last time4 step
          constexpr int HOFF = ChainT4Lds::HS + ChainT4Lds::XS + ChainT4Lds::HL;
          float* hW1 = ch_head_fwd_weights<128>(smem + HOFF);
          ch_stage_weights<128>(A.t4.hd, hW1, hW1 + 128 * CH_WP);
          if (A.gp.on) {                          // the labels come from this launch's GCN producers
            if (threadIdx.x == 0) chain_wait_count(A.ctl + 10, A.gp.Mp, A.ctl);
            __syncthreads();
          }
          chain_t4_stage<TRAIN>(A.t4, r, A.ntiles, A.Mp, tagb, A.ctl, smem);
          long long* mk = blockIdx.x < 64 ? A.trace + 512 + blockIdx.x : nullptr;   // (trace: phase ends)
          if (mk != nullptr && threadIdx.x == 0) mk[0] = (long long)__builtin_amdgcn_s_memrealtime();
          if (threadIdx.x >= 64 * CH_NW) return;    // the head runs on 8 waves (the rest exit)
          const bool pre = TRAIN && A.t4.hb != nullptr;
          chain_head_fwd<128>(A.t4.hd, r, A.ntiles, reinterpret_cast<const float*>(smem + ChainT4Lds::HS + ChainT4Lds::XS),
                              smem + HOFF, true, !pre);
          if (mk != nullptr && threadIdx.x == 0) mk[64] = (long long)__builtin_amdgcn_s_memrealtime();
          if constexpr (TRAIN) {
            if (A.t4.hb != nullptr) {
              // the head backward, here instead of at the start of the backward launch (it only needs
              // this launch's outputs; dL/dloss = 1, scaled there): the backward's time4 stage then
              // starts its reverse steps at once (the head backward was ~12 us of its critical path)
              __syncthreads();
              constexpr int OFF = HOFF + ChainT4Lds::HF;   // (after the head forward's scratch and weights)
              float* dhs = reinterpret_cast<float*>(smem + OFF);
              ChainHead hb = A.t4.hd;
              hb.gpart = A.t4.hb + (size_t)A.ntiles * 16 * 128;
              chain_head_bwd<128>(hb, reinterpret_cast<const float*>(smem + ChainT4Lds::HS + ChainT4Lds::XS), r, A.ntiles,
                                  dhs, smem + OFF + ChainT4Lds::DHT, 132, true, false, CH_NW, hW1, hW1 + 128 * CH_WP);
              for (int e = ch_tid(); e < 16 * 128; e += 64 * CH_NW)
                A.t4.hb[((size_t)r * 16 + e / 128) * 128 + e % 128] = dhs[(e / 128) * 132 + e % 128];
              // the loss hand-off last: its stores' acknowledgement wait then overlaps nothing it delays
              chain_head_fwd_handoff<128>(A.t4.hd, r, A.ntiles, smem + HOFF);
            }
          }
          __syncthreads();
          if (threadIdx.x == 0) A.trace[2 * blockIdx.x + 1] = (long long)__builtin_amdgcn_s_memrealtime();
        }
        chain_finish(A.ctl, nblk);
        return;
      }
      r -= A.nt8;
    }
    if (r < A.npk) {
      const int f = r * 1024 + (int)threadIdx.x;  // packing workgroups
      if (A.pk != nullptr && f < T4PK_ALL) t4_pack_one(f, A.pkU, A.pkW, A.pkDw, A.pk);
    } else if (A.cf.on && r - A.npk < A.cf.Mp) {  // GCN backward coefficients of sample row r - npk
      gcn_coef_fwd_body<2, 16>(A.cf, r - A.npk, smem);
    } else if (A.gp.on && r - A.npk - (A.cf.on ? A.cf.Mp : 0) < A.gp.Mp) {   // GCN forward producer
      // (trace: start / end at [2 blockIdx]; rows < 32: phase A loads in / BatchNorm prepped / the
      // first pass's rows stored at [640 + 4 row + 0..2])
      if (threadIdx.x == 0 && blockIdx.x < 256) A.trace[2 * blockIdx.x] = (long long)__builtin_amdgcn_s_memrealtime();
      const unsigned E = (unsigned)__hip_atomic_load(A.ctl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int row = r - A.npk - (A.cf.on ? A.cf.Mp : 0);
      gcn_prod_body<2, 16>(A.gp, row, chain_tag_base(E), A.ctl + 10, smem, row < 32 ? A.trace + 640 + 4 * row : nullptr);
      if (threadIdx.x == 0 && blockIdx.x < 256) A.trace[2 * blockIdx.x + 1] = (long long)__builtin_amdgcn_s_memrealtime();
    }
    chain_finish(A.ctl, nblk);
    return;
  }
  const int s = blockIdx.x / A.nt8, tile = blockIdx.x % A.nt8;
  if (s >= A.ns || tile >= A.ntiles) {
    chain_finish(A.ctl, nblk);
    return;
  }
  if (threadIdx.x == 0) A.trace[2 * blockIdx.x] = (long long)__builtin_amdgcn_s_memrealtime();
  const unsigned E = (unsigned)__hip_atomic_load(A.ctl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const unsigned tagb = chain_tag_base(E);
  // (a local copy: field-wise scalar loads of the kernel arguments; a reference into the by-value
  // argument array made the compiler copy the whole array to scratch)
  const ChainStage S = A.st[s];
  const int H = S.H, KX = S.KX;
  const bool src = s > 0 || A.gp.on;              // (stage 0 then streams the GCN producers' granules)
#define GQ_CHAIN_BODY(HH, KXX, DD, SRCV, PINV)                                          \
  {                                                                                     \
    constexpr int DS = chain_stage_d(HH, KXX, DD);                                      \
    if (threadIdx.x >= chain_live_threads(ChainCfg<HH>::NT, DS, KXX, SRCV, PINV, HH)) return; \
    chain_stage<HH, TRAIN, KXX, DS, SRCV, PINV>(S, tile, A.ntiles, A.Mp, tagb, A.ctl, smem); \
  }
#ifdef CHAIN_KX1_ONLY      // (A/B probe: no 33-64-channel stage bodies in the kernel; such chains fail)
#define GQ_CHAIN_SRC(HH, PINV, DD) if (KX == 1) GQ_CHAIN_BODY(HH, 1, DD, true, PINV)
#define GQ_CHAIN_KX(HH)                                                                 \
  if (src) { if (S.PIN == 3) { GQ_CHAIN_SRC(HH, 3, CHAIN_D3) } else { GQ_CHAIN_SRC(HH, 1, CHAIN_D) } } \
  else { if (KX == 1) GQ_CHAIN_BODY(HH, 1, CHAIN_D0, false, 1) }
#else
#define GQ_CHAIN_SRC(HH, PINV, DD)                                                      \
  if (KX == 1) GQ_CHAIN_BODY(HH, 1, DD, true, PINV) else GQ_CHAIN_BODY(HH, 2, DD, true, PINV)
#define GQ_CHAIN_KX(HH)                                                                 \
  if (src) { if (S.PIN == 3) { GQ_CHAIN_SRC(HH, 3, CHAIN_D3) } else { GQ_CHAIN_SRC(HH, 1, CHAIN_D) } } \
  else { if (KX == 1) GQ_CHAIN_BODY(HH, 1, CHAIN_D0, false, 1) else GQ_CHAIN_BODY(HH, 2, CHAIN_D0, false, 1) }
#endif
  if (H == 16) GQ_CHAIN_KX(16)
  else if (H == 32) GQ_CHAIN_KX(32)
  else GQ_CHAIN_KX(64)
#undef GQ_CHAIN_KX
#undef GQ_CHAIN_SRC
#undef GQ_CHAIN_BODY
  __syncthreads();
  if (threadIdx.x == 0) A.trace[2 * blockIdx.x + 1] = (long long)__builtin_amdgcn_s_memrealtime();
  chain_finish(A.ctl, nblk);
}

// =====================================================================================
// backward chain: the layers' reverse recurrences, top layer first. Stage k's dx (the
// gradient of the layer below's output, un-pooled by the CONSUMER with the forward's argmax
// bytes when a MaxPooling1D sits between them) is handed off as granules like the forward's
// h; every stage also writes its dz [T+1][Mp][4H] for the weight-gradient pass. The last
// stage writes its dx as plain fp32 (the GCN backward's input).
struct ChainBStage {
  const float* dh;                   // stage 0: fp32 gradient of the layer's (pooled) output [Ts][Mp][H]
  const unsigned long long* din;     // stages > 0: tagged dx stream of the stage above [Ts][Mp][H]
  const unsigned char* pidx;         // P > 0: argmax bytes of the pool after this layer [Ts][Mp][H]
  const __bf16* g;
  const float* c;
  const float* W;
  const float* U;
  __bf16* dz;                        // [T+1][Mp][4H] bf16 (the exact MFMA operand values)
  unsigned long long* sout;          // tagged dx stream [T+1][Mp][Din] (nullptr: last stage)
  float* dx;                         // last stage: fp32 dx [T][Mp][Din]
  long long* trace_mid;              // profiling: time the step loop starts
  long long* prof;                   // profiling (GNNQC_CHAIN_PROF=1): tile 0's per-step phase clocks
  // producer-side un-pooling (uidx != nullptr): the MaxPooling1D(uP) between this stage's input and the
  // stage below is undone HERE - its argmax bytes [T][Mp][Din] are staged in LDS once and every dx
  // element is published as uP full-resolution granules (value at the argmax step, 0 elsewhere) into a
  // [uT][Mp][Din] stream, so the stage below (punp = 1) streams plain dh with no argmax load or select
  // on its recurrence
  const unsigned char* uidx;
  int uP, uT, punp;
  int H, T, Din, Dw, KX, P, Ts;
};

// time4's backward (with the head backward and the loss gradient as its prologue) as the first
// stage of the backward launch (lstm_chain_head_bwd): it publishes dx - the gradient of the
// chain's pooled top output - as granules, so the top chain stage starts after time4's first
// reverse step instead of after the whole time4_head_bwd launch (~26 us).
struct ChainT4B {
  const float* h;                    // time4's h [T][Mp][128] (h_{T-1} feeds the head)
  const float* g;                    // saved gates, fp32 (time4_head.hip t4_sidx layout)
  const float* c;                    // saved (c_t, c_{t-1})
  const bf16x8_t* pk;                // the forward's fragment image of (W, U) (lstm_chain_head_fwd)
  const float* hb;                   // the forward's precomputed head backward (ChainT4::hb) or nullptr
  __bf16* dz;                        // [T+1][Mp][512] bf16 (the weight-gradient pass's input)
  unsigned long long* sout;          // dx granule stream [T][Mp][Din]
  int T, Din, Dw, on;
  ChainHead hd;
};

struct ChainBArgs {
  ChainBStage st[CHAIN_MAX];
  int ns, ntiles, nt8, Mp;
  int* ctl;
  long long* trace;
  ChainT4B t4;                       // t4.on: blocks [ns nt8, (ns + 1) nt8) run time4's backward
};
static_assert(sizeof(ChainBArgs) <= 4096, "chain backward kernel arguments");

// LDS pitches of the backward stages (bf16 dz rows G4 + ZPAD, fp32 dx rows 32 KX + XPAD), chosen with
// scripts/lds_model as in lstm_tm.hip's backward: with a 32-float dx pitch the dx wave's dx^T stores
// (16 sequences x 4 quads per wave) fell on 2 banks of ds_write_b32's 32 (16-way); 33 leaves 2-way
#ifndef CHAINB_ZPAD
#define CHAINB_ZPAD 16
#endif
#ifndef CHAINB_XPAD
#define CHAINB_XPAD 1
#endif
#ifndef CHAINB_ZSWZ
#define CHAINB_ZSWZ 0    // swizzled dz tile: same-box CML 0.2477 vs 0.2459 ms unswizzled (profiles/r6_zs_swizzle_ab.txt)
#endif
template <int H, int KX>
struct ChainBLds {
  static constexpr bool WL = H >= 32;             // W^T fragments of dx from LDS (VGPR budget)
  static constexpr int ZS = 2 * 16 * (4 * H + CHAINB_ZPAD) * 2;
  static constexpr int DH = 2 * 16 * TMC<H>::HP * 4;
  static constexpr int DX = 2 * 16 * (32 * KX + CHAINB_XPAD) * 4;
  static constexpr int WB = WL ? 2 * KX * 16 * (4 * H + 8) * 2 : 0;
  static constexpr int BYTES = ZS + DH + DX + WB;
};
// H >= 32 stages split the two per-step products over K (chain_bwd_stage, SK): every wave runs a
// full 16-row MFMA tile of dh_rec^T = U dz^T / dx^T = W dz^T over a K slice and the partial tiles
// meet in LDS (dpart / xpart, a second barrier per step). The one-tile-per-wave layout (each wave
// owning its own four units: 12 of every 16 A rows zero) issued 4x the MFMAs and made those stages
// MFMA-pipe bound (H = 64: ~0.4 us of a 1.3 us step in the products alone, measured).
template <int H, int KX>
struct ChainBLdsSK {
  static constexpr int NW = TMC<H>::NW, UT = H / 16, KG = NW / UT, NXB = 2 * KX, KXG = NW / NXB;
  static constexpr int ZS = 2 * 16 * (4 * H + CHAINB_ZPAD) * 2;
  static constexpr int DH = 2 * 16 * TMC<H>::HP * 4;
  static constexpr int DP = KG * 16 * TMC<H>::HP * 4;
  static constexpr int XPP = 32 * KX + 4;              // xpart row pitch
  static constexpr int XP = 2 * KXG * 16 * XPP * 4;
  static constexpr int BYTES = ZS + DH + DP + XP;
};
constexpr int chainb_max(int a, int b) { return a > b ? a : b; }
static constexpr int CHAINB_LDS_STAGE =
    chainb_max(chainb_max(ChainBLds<64, 2>::BYTES, ChainBLdsSK<64, 1>::BYTES),
               chainb_max(ChainBLdsSK<64, 2>::BYTES, chainb_max(ChainBLdsSK<32, 1>::BYTES, ChainBLdsSK<32, 2>::BYTES)));

struct ChainT4BLds {
  static constexpr int DHT = 16 * 132 * 4;                 // dh_{T-1} from the head
  static constexpr int ZS = 16 * (512 + 8) * 2;            // bf16 dz tile
  static constexpr int DN = 2 * 16 * 132 * 4;              // dh_rec partials of the two K halves
  static constexpr int DXP = 4 * 16 * 68 * 4;              // dx partials of the four K quarters
  static constexpr int STEP = ZS + DN + DXP;
  static constexpr int HEAD = ChainHeadBwdLds<128>::BYTES; // the head prologue's scratch (same bytes)
  static constexpr int BYTES = DHT + (STEP > HEAD ? STEP : HEAD);
};
static constexpr int CHAINB_LDS = ChainT4BLds::BYTES > CHAINB_LDS_STAGE ? ChainT4BLds::BYTES : CHAINB_LDS_STAGE;

#ifndef CHAINB_LEAD
#define CHAINB_LEAD 1
#endif
#ifndef CHAINB_IO
#define CHAINB_IO 0          // 1: H = 16 stages as compute / rotating I/O / publisher waves (chain_bwd_stage_io);
                             // measured slower (bottom stages end 123 / 140 vs 113 / 117 us, bench 0.307 vs
                             // 0.286 ms/step): the I/O waves' staging and load issue hold up the step barrier
#endif
#ifndef CHAINB_DXW
#define CHAINB_DXW 1         // H = 16 stages: dx = W dz by a dedicated wave (not by compute waves 0 / 1 between
                             // the step's MFMA and the next cell phase, which put it on the recurrence's path)
#endif
#ifndef CHAINB_PUBBATCH
#define CHAINB_PUBBATCH 4    // backward publisher: LDS reads of this many dx elements per lane, then their stores
#endif
#ifndef CHAINB_NPUB
#define CHAINB_NPUB 4        // publisher waves per H <= 32 stage (each publishes every NPUB-th 64-element slice;
                             // same-box chain bwd 156.8 / 136.9 / 133.0 / 130.0 us for 1 / 2 / 3 / 4)
#endif
#ifndef CHAINB_PUBPRIO
#define CHAINB_PUBPRIO 2     // s_setprio of the backward publisher and dz waves (same-box A/B: chain bwd 127.3 -> 124.2 us, bench 0.2626 -> 0.2596 ms)
#endif
#ifndef CHAINB_DXPRIO
#define CHAINB_DXPRIO 2      // s_setprio of the backward dx wave (same-box A/B: chain bwd 124.0 -> 122.2 us, bench 0.2589 -> 0.2562 ms)
#endif
#ifndef CHAINB_PUNPOOL
#define CHAINB_PUNPOOL 0     // 1: producer-side un-pooling (ChainBStage::uidx). Off: against the round-5 baseline
                             // build on one box it measured chain bwd 121.4 (on) / 123.9 (compiled in, off) vs 115.9 us
#endif
#ifndef CHAINB_DZW
#define CHAINB_DZW 1         // 1: a dz wave stores each step's dz tile (else the publisher wave does)
#endif
#ifndef CHAINB_G
#define CHAINB_G 2           // waves per backward I/O group: 2 = one for the cell records, one for dh
#endif
// ring depths (reverse steps of prefetch) per hidden size
#ifndef CHAINB_D16
#define CHAINB_D16 4
#endif
#ifndef CHAINB_D32
#define CHAINB_D32 4
#endif
#ifndef CHAINB_D64
#define CHAINB_D64 2
#endif
// threads of a backward stage workgroup: compute waves (+ the publisher wave when it fits, + the dx
// wave of the split-free H = 16 stages)
__host__ __device__ constexpr bool chainb_dxw(int h) {
  return CHAINB_DXW && h < 32 && TMC<16>::NT + 64 * CHAINB_NPUB + 64 <= 1024;
}
// (+ the dz wave: the step's dz tile leaves from its own wave, beside the publisher's dx granules)
// publisher waves of a stage (0: H = 64, whose compute waves fill the workgroup)
__host__ __device__ constexpr int chainb_npub(int h, int nt) {
  return nt + 64 > 1024 ? 0
       : chainb_max(1, CHAINB_NPUB < (1024 - nt - (chainb_dxw(h) ? 64 : 0) - 64) / 64
                           ? CHAINB_NPUB : (1024 - nt - (chainb_dxw(h) ? 64 : 0) - 64) / 64);
}
__host__ __device__ constexpr bool chainb_dzw(int h, int nt) {
  return CHAINB_DZW && chainb_npub(h, nt) > 0 && nt + 64 * chainb_npub(h, nt) + 64 + (chainb_dxw(h) ? 64 : 0) <= 1024;
}
__host__ __device__ constexpr int chainb_live_threads(int h, int nt) {
  return nt + 64 * chainb_npub(h, nt) + (chainb_dxw(h) ? 64 : 0) + (chainb_dzw(h, nt) ? 64 : 0);
}

// lstm_tm_bwd_body (DZ + DX) with one dh element per lane from the stage above's stream
// (or, stage 0, from global memory), un-pooled on load, and dx published element-wise.
template <int H, int KX, int D, bool SRC, bool UP, bool XO>
__device__ __forceinline__ void chain_bwd_stage(const ChainBStage S, int tile, int ntiles, int Mp, unsigned tagb,
                                                int* ctl, char* smem) {
  using C = TMC<H>;
  constexpr int CPL = C::CPL, NW = C::NW, NT = C::NT, G4 = C::G4, KB = C::KB;
  constexpr int NXB = KX * 2;
  constexpr int TX = (NXB + NW - 1) / NW;
  constexpr bool SK = H >= 32;                     // split-K products (ChainBLdsSK)
  static_assert(CPL == 1 && 16 * H == NT, "one dh element per lane");
  using L = ChainBLds<H, KX>;
  using LK = ChainBLdsSK<H, KX>;
  constexpr int UT = LK::UT, KG = LK::KG, KXG = LK::KXG, KPG = SK ? KB / KG : 1, KPX = SK ? KB / KXG : 1;
  static_assert(!SK || (NW % UT == 0 && KB % KG == 0 && NW % NXB == 0 && KB % KXG == 0), "split-K tiling");
  static_assert(L::BYTES <= CHAINB_LDS_STAGE && LK::BYTES <= CHAINB_LDS_STAGE && L::ZS % 16 == 0 && L::DH % 16 == 0,
                "chain bwd LDS layout");
  auto zs = reinterpret_cast<__bf16 (*)[16][G4 + CHAINB_ZPAD]>(smem);
  // dz element e of sequence c at zs[.][c][chz(c, e)]: 16-byte chunk XOR bit 2 of the sequence (as lstm_tm.hip)
  auto chz = [](int c, int e) { return CHAINB_ZSWZ ? e ^ (((c >> 2) & 1) << 3) : e; };
  auto dhs = reinterpret_cast<float (*)[16][C::HP]>(smem + L::ZS);
  auto dxs = reinterpret_cast<float (*)[16][32 * KX + CHAINB_XPAD]>(smem + L::ZS + L::DH);
  auto wl = reinterpret_cast<__bf16 (*)[16][G4 + 8]>(smem + L::ZS + L::DH + L::DX);
  auto dpart = reinterpret_cast<float (*)[16][C::HP]>(smem + LK::ZS + LK::DH);                      // [KG]
  auto xpart = reinterpret_cast<float (*)[KXG][16][LK::XPP]>(smem + LK::ZS + LK::DH + LK::DP);      // [2][KXG]

  const int T = S.T, Din = S.Din, Dw = S.Dw, P = S.P, Ts = S.Ts;
  // source kind and un-pooling are template parameters: with run-time branches around the
  // ring loads the compiler drained the whole prefetch ring (vmcnt(0)) every D steps
  const int tid = threadIdx.x, lane = tid & 63;
  // Publisher wave (a spare wave of the 1024-thread workgroup, H < 64): it alone stores the
  // dx granules. The write-through (sc1) stores are acknowledged only after the memory
  // round trip and the vector-memory counter retires in order, so in a compute wave every
  // wait for a ring load also waited for the stores issued before it (~2 us per step, 6x the
  // step time). The publisher joins the same barriers and reads the dx tile from LDS.
  const int row0 = tile * 16;
  constexpr bool PUBW = NT + 64 <= 1024;
  constexpr int NPUB = chainb_npub(H, NT);
  constexpr bool DXW = !SK && chainb_dxw(H);
  constexpr bool DZW = PUBW && chainb_dzw(H, NT);
  static_assert(PUBW == (NPUB > 0), "publisher waves");
  static_assert(!DXW || PUBW, "the dx wave hands its tiles to the publisher");
  if constexpr (DZW) {
    // dz wave: after step s's barrier (the second one of the step, SK: its first), the dz tile of step s
    // from zs[s & 1] (held until step s + 2's cell phase) -> HBM with 16-byte stores
    if (tid >= NT + 64 * NPUB + (DXW ? 64 : 0)) {
      if (CHAINB_PUBPRIO > 0) __builtin_amdgcn_s_setprio(CHAINB_PUBPRIO);
      const int nsteps = (T + D - 1) / D * D;
      __syncthreads();
      __syncthreads();
      for (int s = 0; s < nsteps; ++s) {
        lds_barrier();
        if (s < T) {
          const int pb = s & 1;
          __bf16* zt = S.dz + ((size_t)(T - 1 - s) * Mp + row0) * G4;
#pragma unroll
          for (int q = lane; q < 16 * G4 / 8; q += 64) {
            const int e = 8 * q;
            *reinterpret_cast<uint4*>(zt + e) = *reinterpret_cast<const uint4*>(&zs[pb][e / G4][chz(e / G4, e % G4)]);
          }
        }
        if constexpr (SK) lds_barrier();
      }
      __syncthreads();
      return;
    }
  }
  if constexpr (DXW) {
    // dx wave: after step s's barrier, dx^T = W dz^T of that step from zs[s & 1] into dxs[s & 1]
    // (the publisher stores it after the next barrier, as before). It joins barrier s + 1 only once
    // done, and zs[s & 1] is rewritten only in step s + 2's cell phase (after barrier s + 1), so the
    // compute waves go from their dh_rec MFMA straight to the next cell phase.
    if (tid >= NT + 64 * NPUB) {
      if (CHAINB_DXPRIO > 0) __builtin_amdgcn_s_setprio(CHAINB_DXPRIO);
      const int col = lane & 15, quad = lane >> 4;
      bf16x8_t wx[NXB][KB];
#pragma unroll
      for (int xb = 0; xb < NXB; ++xb) {
        const int din = 16 * xb + col;
#pragma unroll
        for (int k = 0; k < KB; ++k) {
          bf16x8_t v;
#pragma unroll
          for (int j = 0; j < 8; ++j)
            v[j] = (__bf16)(S.W[(size_t)min(din, Dw - 1) * G4 + 32 * k + 8 * quad + j] * (din < Dw ? 1.f : 0.f));
          wx[xb][k] = v;
        }
      }
      const int nsteps = (T + D - 1) / D * D;
      __syncthreads();
      __syncthreads();
      for (int s = 0; s < nsteps; ++s) {
        lds_barrier();
        if (s < T) {
          const int p = s & 1;
          bf16x8_t bz[KB];
#pragma unroll
          for (int k = 0; k < KB; ++k) bz[k] = *reinterpret_cast<const bf16x8_t*>(&zs[p][col][chz(col, 32 * k + 8 * quad)]);
#pragma unroll
          for (int xb = 0; xb < NXB; ++xb) {
            f32x4_t a = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int k = 0; k < KB; ++k) a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wx[xb][k], bz[k], a, 0, 0, 0);
#pragma unroll
            for (int r = 0; r < 4; ++r) dxs[p][col][16 * xb + 4 * quad + r] = a[r];
          }
          chain_mark_wave((S.prof != nullptr && tile == 0) ? S.prof : nullptr, s, 6);   // (dx tile in LDS)
        }
      }
      __syncthreads();
      return;
    }
  }
  if constexpr (PUBW) {
    if (tid >= NT) {
      if (CHAINB_PUBPRIO > 0) __builtin_amdgcn_s_setprio(CHAINB_PUBPRIO);
      const int nsteps = (T + D - 1) / D * D;
      const int nx = 16 * Din;
      const size_t xstep = (size_t)Mp * Din;
      // publisher wave pj of NPUB publishes the 64-element slices pj, pj + NPUB, ... of each dx tile
      const int pj = (tid - NT) >> 6;
      constexpr int ESTR = 64 * (NPUB > 0 ? NPUB : 1);
      const int dq = ESTR / Din, dr = ESTR % Din;
      // producer-side un-pooling: this tile's argmax bytes of all T steps in LDS (loaded before the
      // publisher's first store, so no load of it waits behind its write-through stores), and the
      // full-resolution steps past the last pooling window published as zeros up front (the stage
      // below needs them first)
      constexpr int UPOFF = ((SK ? LK::BYTES : L::BYTES) + 15) / 16 * 16;
      unsigned char* ub = reinterpret_cast<unsigned char*>(smem + UPOFF);
      const bool unp = CHAINB_PUNPOOL && XO && S.uidx != nullptr;
      if (unp) {
        const int nw4 = T * 16 * Din / 4;
        for (int i = tid - NT; i < nw4; i += ESTR) {
          const int e = 4 * i, ts = e / (16 * Din), r = e % (16 * Din);
          *reinterpret_cast<unsigned*>(ub + e) =
              *reinterpret_cast<const unsigned*>(S.uidx + ((size_t)ts * Mp + row0) * Din + r);
        }
        for (int tt = T * S.uP; tt < S.uT; ++tt)
          for (int e = tid - NT; e < nx; e += ESTR)
            st_granule(S.sout + (size_t)row0 * Din + e + (size_t)tt * xstep, 0.f, tagb | (unsigned)tt);
      }
      // LDS reads of CHAINB_PUBBATCH elements per lane first, then their stores: a read -> wait -> store
      // loop per element paid one LDS round trip per element on the publisher's step (16 Din / 64 =
      // Din / 4 elements per lane, the same count on every lane since Din % 4 == 0). (All Din / 4 at
      // once, up to 16, pushed the kernel from 32 to 176 bytes of scratch: chain bwd 133 -> 258 us.)
      constexpr int PUBN = CHAINB_PUBBATCH > 0 ? CHAINB_PUBBATCH : 1;   // elements per lane per batch
      auto publish = [&](int buf, int ts) {
        const unsigned tag = tagb | (unsigned)ts;
        for (int e0 = 64 * pj; e0 < nx; e0 += ESTR * PUBN) {
        const int niter = min((nx - e0 + ESTR - 1) / ESTR, PUBN);
        float vv[PUBN];
        unsigned bb[PUBN];
        int row = (lane + e0) / Din, k = (lane + e0) % Din;
#pragma unroll
        for (int i = 0; i < PUBN; ++i) {
          if (i < niter) {                          // wave-uniform
            if constexpr (SK) {
              float v = 0.f;
#pragma unroll
              for (int g = 0; g < KXG; ++g) v += xpart[buf][g][row][k];
              vv[i] = v;
            } else {
              vv[i] = dxs[buf][row][k];
            }
            bb[i] = unp ? (unsigned)ub[(ts * 16 + row) * Din + k] : 0u;
          }
          row += dq;
          k += dr;
          if (k >= Din) { k -= Din; ++row; }
        }
#pragma unroll
        for (int i = 0; i < PUBN; ++i) {
          if (i < niter) {
            const int e = e0 + lane + ESTR * i;
            if (unp) {
              for (int qq = 0; qq < S.uP; ++qq) {
                const int tt = ts * S.uP + qq;
                st_granule(S.sout + (size_t)row0 * Din + e + (size_t)tt * xstep, bb[i] == (unsigned)qq ? vv[i] : 0.f,
                           tagb | (unsigned)tt);
              }
            } else {
              const size_t o = (size_t)row0 * Din + e + (size_t)ts * xstep;
              if constexpr (XO) st_granule(S.sout + o, vv[i], tag);
              else S.dx[o] = vv[i];
            }
          }
        }
        }
      };
      // ... and the step's dz tile (16-byte stores from LDS; zs[s & 1] holds it from the barrier
      // that follows step s's cell phase until the cell phase of step s + 2): the compute waves then
      // issue only loads, so their waits are for their own loads alone
      auto store_dz = [&](int ss) {
        const int pb = ss & 1;
        __bf16* zt = S.dz + ((size_t)(T - 1 - ss) * Mp + row0) * G4;
#pragma unroll
        for (int q = lane; q < 16 * G4 / 8; q += 64) {
          const int e = 8 * q;
          *reinterpret_cast<uint4*>(zt + e) = *reinterpret_cast<const uint4*>(&zs[pb][e / G4][chz(e / G4, e % G4)]);
        }
      };
      __syncthreads();
      __syncthreads();
      if constexpr (SK) {            // two barriers per step; step s's dx tile is complete after the second
        for (int s = 0; s < nsteps; ++s) {
          lds_barrier();
          if (!DZW && s < T) store_dz(s);
          lds_barrier();
          if (s < T) publish(s & 1, T - 1 - s);
        }
        __syncthreads();
      } else {
        long long* prw = (S.prof != nullptr && tile == 0 && pj == 0) ? S.prof : nullptr;
        for (int s = 0; s < nsteps; ++s) {
          lds_barrier();
          const int t = T - 1 - s;
          if (!DZW && s < T) store_dz(s);
          if (s >= 1 && s <= T) publish((s - 1) & 1, t + 1);
          if (s < T) chain_mark_wave(prw, s, 7);   // (the publisher's work of the step is issued)
        }
        __syncthreads();
        publish((T - 1) & 1, 0);
      }
      return;
    }
  }
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int col = lane & 15, quad = lane >> 4;

  for (int i = tid; i < 2 * 16 * C::HP; i += NT) (&dhs[0][0][0])[i] = 0.f;

  const int unit = 4 * w + quad;
  // SK: wave w owns unit tile ut over K slice kg of dh_rec^T, din tile xt over K slice kx of dx^T
  const int ut = w % UT, kg = w / UT, xt = w % NXB, kx = w / NXB;
  bf16x8_t ufr[SK ? KPG : KB];
  bf16x8_t ufk[SK ? KPX : 1];                      // (SK: the W fragments of this wave's dx slice)
  if constexpr (SK) {
#pragma unroll
    for (int q = 0; q < KPG; ++q) {
      bf16x8_t v;
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = (__bf16)S.U[(size_t)(16 * ut + col) * G4 + 32 * (kg * KPG + q) + 8 * quad + j];
      ufr[q] = v;
    }
    const int din = 16 * xt + col;
#pragma unroll
    for (int q = 0; q < KPX; ++q) {
      bf16x8_t v;
#pragma unroll
      for (int j = 0; j < 8; ++j)
        v[j] = (__bf16)(S.W[(size_t)min(din, Dw - 1) * G4 + 32 * (kx * KPX + q) + 8 * quad + j] * (din < Dw ? 1.f : 0.f));
      ufk[q] = v;
    }
  } else {
    const int au = 4 * w + (col >> 2);
#pragma unroll
    for (int s = 0; s < KB; ++s) {
      bf16x8_t v;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float val = S.U[(size_t)au * G4 + 32 * s + 8 * quad + j];
        v[j] = (__bf16)(val * ((col & 3) == 0 ? 1.f : 0.f));
      }
      ufr[s] = v;
    }
  }
  bf16x8_t wfr[(L::WL || SK || DXW) ? 1 : TX][(L::WL || SK || DXW) ? 1 : KB];
  if constexpr (SK || DXW) {
  } else if constexpr (L::WL) {     // W^T blocks [NXB][16 din][4H] in LDS (unrolled: all loads in flight)
    static_assert((NXB * 16 * G4) % NT == 0, "W staging trip count");
#pragma unroll
    for (int it = 0; it < NXB * 16 * G4 / NT; ++it) {
      const int i = tid + it * NT;
      const int xb = i / (16 * G4), r = (i / G4) % 16, k = i % G4;
      const int din = 16 * xb + r;
      wl[xb][r][k] = (__bf16)(S.W[(size_t)min(din, Dw - 1) * G4 + k] * (din < Dw ? 1.f : 0.f));   // no branch
    }
  } else {
#pragma unroll
    for (int q = 0; q < TX; ++q) {
      const int xb = w + NW * q;
      const int din = 16 * xb + col;
#pragma unroll
      for (int s = 0; s < KB; ++s) {
        bf16x8_t v;
#pragma unroll
        for (int j = 0; j < 8; ++j)
          v[j] = (__bf16)(S.W[(size_t)min(din, Dw - 1) * G4 + 32 * s + 8 * quad + j] *
                          ((xb < NXB && din < Dw) ? 1.f : 0.f));
        wfr[q][s] = v;
      }
    }
  }

  // forward state ring (gates, c_t) and the dh element ring, D reverse steps ahead
  uint2 rg[D];                       // packed bf16 gates
  float rc[D];
  unsigned long long rq[D];
  unsigned ri[D];
  auto sidx = [&](int tt) { return ((((size_t)tt * ntiles + tile) * NW + w)) * 64 + lane; };
  // tt / P as a multiply-high with the magic floor(2^32 / P) + 1 (exact for tt * P < 2^32; here
  // tt < 4096, P <= 255): the per-step integer divisions by the run-time pool size cost the
  // un-pooling stages ~160 shader clocks per step on the dh staging (phase table, round 5)
  // un-pooling stages; the magic of P == 1 would be 2^32, which wraps to 0, so that pool size
  // (a chain that ends in MaxPooling1D(1)) takes the identity instead
  const unsigned pmag = (UP && P > 1) ? 0xFFFFFFFFu / (unsigned)P + 1u : 0u;
  auto divp = [&](int tt) { return P > 1 ? (int)__umulhi((unsigned)tt, pmag) : tt; };
  // source time of the dh of time tt (-1: past the last pooling window -> zero gradient)
  auto src_t = [&](int tt) {
    if constexpr (UP) return tt < Ts * P ? divp(tt) : -1;
    else return tt;
  };
  const size_t eoff = (size_t)row0 * H + tid;        // this lane's dh element in a [Mp][H] row block
  const size_t hstep = (size_t)Mp * H;
  auto load = [&](int J, int SS) {
    const int tt = max(T - 1 - SS, 0);
    const size_t o = sidx(tt);
    rg[J] = *reinterpret_cast<const uint2*>(S.g + o * 4);
    rc[J] = S.c[o];
    const int st = max(src_t(tt), 0);
    if constexpr (SRC) rq[J] = ld_granule(S.din + eoff + (size_t)st * hstep);
    else rq[J] = (unsigned long long)__float_as_uint(S.dh[eoff + (size_t)st * hstep]);
    if constexpr (UP) ri[J] = (unsigned)S.pidx[eoff + (size_t)st * hstep];
    else ri[J] = 0u;
  };
  // dh of time tt from ring slot J (tag-checked for a stream source)
  auto stage_dh = [&](int J, int tt) -> float {
    const int st = tt >= 0 ? src_t(tt) : -1;
    if constexpr (SRC) {
      const bool bad = st >= 0 && (unsigned)(rq[J] >> 32) != (tagb | (unsigned)st);
      if (__builtin_amdgcn_ballot_w64(bad) != 0)
        rq[J] = chain_wait(S.din + eoff + (size_t)max(st, 0) * hstep, tagb | (unsigned)max(st, 0), ctl);
    }
    const float v = __uint_as_float((unsigned)rq[J]);
    bool keep = st >= 0;
    if constexpr (UP) keep = keep && ri[J] == (unsigned)(tt - st * P);
    return keep ? v : 0.f;
  };
  // dz storer (one float4 granule of the [16][4H] tile per thread)
  const int gz_seq = tid / (G4 / 4), gz_c = (tid % (G4 / 4)) * 4;
  __bf16* zbase = S.dz + (size_t)(row0 + gz_seq) * G4 + gz_c;
  const size_t zstep = (size_t)Mp * G4;
  // dx: element e of the [16][Din] tile per lane, NQ passes (Din <= 64), clamped duplicates
  // instead of a branch; XO: publish granules, else (bottom stage) plain fp32
  constexpr int NQ = (16 * 64 + NT - 1) / NT;
  const int nx = 16 * Din;
  const size_t xstep = (size_t)Mp * Din;
  int xrow[NQ], xk[NQ], xo[NQ];
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    const int e = min(tid + q * NT, nx - 1);
    xrow[q] = e / Din;
    xk[q] = e % Din;
    xo[q] = row0 * Din + e;
  }
  auto store_dx = [&](int buf, int ts, unsigned tag) {
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      float v;
      if constexpr (SK) {
        v = 0.f;
#pragma unroll
        for (int g = 0; g < KXG; ++g) v += xpart[buf][g][xrow[q]][xk[q]];
      } else {
        v = dxs[buf][xrow[q]][xk[q]];
      }
      const size_t o = (size_t)xo[q] + (size_t)ts * xstep;
      if constexpr (XO) st_granule(S.sout + o, v, tag);
      else S.dx[o] = v;
    }
  };

  if constexpr (SRC) {    // start once the stage above is D + LEAD steps ahead (see the forward)
    int tw = T - 1 - (D + CHAINB_LEAD);
    tw = max(tw, 0);
    const int st = src_t(tw);
    if (st >= 0) (void)chain_wait(S.din + eoff + (size_t)st * hstep, tagb | (unsigned)st, ctl);
  }
#pragma unroll
  for (int j = 0; j < D; ++j) load(j, j);
  __syncthreads();
  dhs[0][tid / H][tid % H] = stage_dh(0, T - 1);
  load(0, D);
  float dc = 0.f, dhr = 0.f, dhn;
  __syncthreads();
  dhn = dhs[0][col][unit];
  if (tid == 0 && S.trace_mid) S.trace_mid[blockIdx.x] = (long long)__builtin_amdgcn_s_memrealtime();

  long long* pr = (S.prof != nullptr && tile == 0) ? S.prof : nullptr;
  for (int s0 = 0; s0 < T; s0 += D) {
#pragma unroll
    for (int j = 0; j < D; ++j) {
      const int s = s0 + j;
      const int t = T - 1 - s;
      const int p = s & 1;
      const int jn = (j + 1 == D) ? 0 : j + 1;
      chain_mark(pr, s, 0);
      {
        const float cp = rc[jn] * (t > 0 ? 1.f : 0.f);
        const float dh = dhn + dhr;
        const float4 g4 = gates_unpack(rg[j]);
        const float tc = tanhf_fast(rc[j]);
        const float dct = dc + dh * g4.w * (1.f - tc * tc);
        dc = dct * g4.y;
        zs[p][col][chz(col, 0 * H + unit)] = (__bf16)(dct * g4.z * g4.x * (1.f - g4.x));
        zs[p][col][chz(col, 1 * H + unit)] = (__bf16)(dct * cp * g4.y * (1.f - g4.y));
        zs[p][col][chz(col, 2 * H + unit)] = (__bf16)(dct * g4.x * (1.f - g4.z * g4.z));
        zs[p][col][chz(col, 3 * H + unit)] = (__bf16)(dh * tc * g4.w * (1.f - g4.w));
      }
      {   // state of step s + D and the dh of step s + 1 (time t - 1)
        const int tt = max(T - 1 - (s + D), 0);
        const size_t o = sidx(tt);
        rg[j] = *reinterpret_cast<const uint2*>(S.g + o * 4);
        rc[j] = S.c[o];
      }
      chain_mark(pr, s, 1);
      dhs[p ^ 1][tid / H][tid % H] = stage_dh(jn, t - 1);
      chain_mark(pr, s, 2);
      {
        const int tt = max(T - 1 - (s + 1 + D), 0);
        const int st = max(src_t(tt), 0);
        if constexpr (SRC) rq[jn] = ld_granule(S.din + eoff + (size_t)st * hstep);
        else rq[jn] = (unsigned long long)__float_as_uint(S.dh[eoff + (size_t)st * hstep]);
        if constexpr (UP) ri[jn] = (unsigned)S.pidx[eoff + (size_t)st * hstep];
        else ri[jn] = 0u;
      }
      lds_barrier();
      chain_mark(pr, s, 3);
      dhn = dhs[p ^ 1][col][unit];
      if constexpr (SK) {   // partial products of this wave's K slices -> LDS
        f32x4_t a = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int q = 0; q < KPG; ++q) {
          const bf16x8_t bz = *reinterpret_cast<const bf16x8_t*>(&zs[p][col][chz(col, 32 * (kg * KPG + q) + 8 * quad)]);
          a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ufr[q], bz, a, 0, 0, 0);
        }
        f32x4_t b = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int q = 0; q < KPX; ++q) {
          const bf16x8_t bz = *reinterpret_cast<const bf16x8_t*>(&zs[p][col][chz(col, 32 * (kx * KPX + q) + 8 * quad)]);
          b = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ufk[q], bz, b, 0, 0, 0);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          dpart[kg][col][16 * ut + 4 * quad + r] = a[r];
          xpart[p][kx][col][16 * xt + 4 * quad + r] = b[r];
        }
      } else {   // serial chain: dh_{t-1} = U dz_t
        f32x4_t a0 = {0.f, 0.f, 0.f, 0.f}, a1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int k = 0; k < KB; ++k) {
          const bf16x8_t bz = *reinterpret_cast<const bf16x8_t*>(&zs[p][col][chz(col, 32 * k + 8 * quad)]);
          if (k & 1) a1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ufr[k], bz, a1, 0, 0, 0);
          else a0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ufr[k], bz, a0, 0, 0, 0);
        }
        dhr = a0[0] + a1[0];
#ifdef GQ_CHAIN_PROF
        if (pr != nullptr) asm volatile("" ::"v"(dhr));
#endif
      }
      chain_mark(pr, s, 4);
      if constexpr (!PUBW) {   // dz tile -> HBM (weight-gradient pass; else the publisher stores it)
        const uint2 zv = *reinterpret_cast<const uint2*>(&zs[p][gz_seq][chz(gz_seq, gz_c)]);
        const int tz = t >= 0 ? t : T;
        *reinterpret_cast<uint2*>(zbase + (size_t)tz * zstep) = zv;
      }
      {   // previous step's dx tile (time t + 1) -> stream / HBM; steps outside write row T
        const int ts = (s >= 1 && s <= T) ? t + 1 : T;
        if constexpr (!PUBW) store_dx(p ^ 1, ts, tagb | (unsigned)ts);
      }
      if constexpr (SK) {   // the partial tiles meet: dh_{t-1} of this lane's cell
        lds_barrier();
        float sdh = 0.f;
#pragma unroll
        for (int g = 0; g < KG; ++g) sdh += dpart[g][col][unit];
        dhr = sdh;
      } else if (!DXW && t >= 0) {   // dx^T = W dz^T of this step (DXW: the dx wave's)
#pragma unroll
        for (int q = 0; q < TX; ++q) {
          const int xb = w + NW * q;
          if (xb < NXB) {
            f32x4_t a = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int k = 0; k < KB; ++k) {
              const bf16x8_t bz = *reinterpret_cast<const bf16x8_t*>(&zs[p][col][chz(col, 32 * k + 8 * quad)]);
              bf16x8_t wa;
              if constexpr (L::WL) wa = *reinterpret_cast<const bf16x8_t*>(&wl[xb][col][32 * k + 8 * quad]);
              else wa = wfr[q][k];
              a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa, bz, a, 0, 0, 0);
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) dxs[p][col][16 * xb + 4 * quad + r] = a[r];
          }
        }
      }
      chain_mark(pr, s, 5);
    }
  }
  __syncthreads();
  if constexpr (!PUBW) store_dx((T - 1) & 1, 0, tagb);     // dx tile of t = 0
}

// The H = 16 reverse recurrence (the bottom layers' 181 steps: the backward's critical path) with the
// forward's role split. Compute waves: per step, the cell's gate gradients from LDS inputs only (the
// packed gates, c_t and c_{t-1} as one 16-byte record, dh from the stage above), dz to LDS, one
// barrier, dh_rec = U dz and dx = W dz by MFMA from LDS; no global memory access at all. D rotating
// I/O waves: wave k stages the records and the (tag-checked, un-pooled) dh tile of every step
// s = k (mod D), loaded D steps ahead, with 16-byte loads of the tile's contiguous cell block. A
// publisher wave stores each step's dz tile (16-byte stores) and publishes its dx, one step later.
template <int H>
struct ChainBIoLds {
  static constexpr int ZS = 2 * 16 * (4 * H + 8) * 2;
  static constexpr int DH = 2 * 16 * TMC<H>::HP * 4;
  static constexpr int DX = 2 * 16 * 32 * 2 * 4;          // dx tiles (KX <= 2)
  static constexpr int RC = 2 * TMC<H>::NT * 16;          // {gates, c_t, c_{t-1}} records
  static constexpr int BYTES = ZS + DH + DX + RC;
};
__host__ __device__ constexpr int chainb_io_threads(int nt, int d) { return nt + 64 * d * CHAINB_G + 64; }
template <int V>
struct ChIc { static constexpr int value = V; };

template <int H, int KX, int D, bool SRC, bool UP, bool XO>
__device__ __forceinline__ void chain_bwd_stage_io(const ChainBStage S, int tile, int ntiles, int Mp, unsigned tagb,
                                                   int* ctl, char* smem) {
  using C = TMC<H>;
  constexpr int NW = C::NW, NT = C::NT, G4 = C::G4, KB = C::KB;
  constexpr int NXB = KX * 2;
  constexpr int TX = (NXB + NW - 1) / NW;
  static_assert(C::CPL == 1 && 16 * H == NT && NT % 256 == 0, "one dh element per compute lane");
  constexpr int CPLN = NT / 64;                     // cells per I/O lane (whole tile per I/O wave)
  static_assert(CPLN % 4 == 0 || CPLN == 4, "I/O lanes move cells four at a time");
  using L = ChainBIoLds<H>;
  static_assert(L::BYTES <= CHAINB_LDS_STAGE, "chain bwd I/O LDS layout");
  auto zs = reinterpret_cast<__bf16 (*)[16][G4 + 8]>(smem);
  auto dhs = reinterpret_cast<float (*)[16][C::HP]>(smem + L::ZS);
  auto dxs = reinterpret_cast<float (*)[16][32 * KX]>(smem + L::ZS + L::DH);
  auto rec = reinterpret_cast<uint4 (*)[NT]>(smem + L::ZS + L::DH + L::DX);

  const int T = S.T, Din = S.Din, Dw = S.Dw, P = S.P, Ts = S.Ts;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int col = lane & 15, quad = lane >> 4;
  const int row0 = tile * 16;
  constexpr int G = CHAINB_G;
  static_assert(G == 1 || G == 2, "backward I/O group: one wave, or a record wave and a dh wave");
  const bool compute = w < NW;
  const bool publisher = w == NW + D * G;
  const int iow = (w - NW) / G;                     // I/O group: steps s = iow (mod D)
  const int sub = (w - NW) % G;                     // (G = 2: 0 loads the cell records, 1 the dh tile)
  constexpr int NTL = chainb_io_threads(NT, D);
  for (int i = tid; i < 2 * 16 * C::HP; i += NTL) (&dhs[0][0][0])[i] = 0.f;
  const size_t hstep = (size_t)Mp * H;
  const size_t zstep = (size_t)Mp * G4;
  const size_t xstep = (size_t)Mp * Din;
  // source time of the dh of time tt (-1: past the last pooling window -> zero gradient)
  auto src_t = [&](int tt) {
    if constexpr (UP) return tt < Ts * P ? tt / P : -1;
    else return tt;
  };
  long long* pr = (S.prof != nullptr && tile == 0) ? S.prof : nullptr;

  // ---------------------------------------------------------------- I/O waves
  // one slot: this tile's 4 cells x {gates (2 x 16 B), c_t, c_{t-1}} and 2 dh pairs (+ argmax bytes)
  constexpr int NDP = NT / 2 / 64;                  // dh pairs per lane
  uint4 sg[CPLN / 2];
  float4 sc[CPLN / 4], scp[CPLN / 4];
  u64x2_t sq[NDP];
  unsigned short si[NDP];
  // (SB: 0 = records only, 1 = dh only, 2 = both; a compile-time choice so no branch sits between a
  // wave's loads and their use)
  auto io_load = [&](auto sbc, int ss) {            // the inputs of reverse step ss
    constexpr int SB = decltype(sbc)::value;
    const int tt = max(T - 1 - ss, 0);
    const size_t cell0 = ((size_t)tt * ntiles + tile) * NT;
    const size_t cellp = ((size_t)max(tt - 1, 0) * ntiles + tile) * NT;
    // (lane's cells: groups of four, 4 (lane + 64 q) + i; gates of a group = two 16-byte halves)
    if constexpr (SB != 1) {
#pragma unroll
      for (int q = 0; q < CPLN / 2; ++q)
        sg[q] = *reinterpret_cast<const uint4*>(S.g + (cell0 + 4 * (lane + 64 * (q / 2)) + 2 * (q % 2)) * 4);
#pragma unroll
      for (int q = 0; q < CPLN / 4; ++q) {
        sc[q] = *reinterpret_cast<const float4*>(S.c + cell0 + 4 * (lane + 64 * q));
        scp[q] = *reinterpret_cast<const float4*>(S.c + cellp + 4 * (lane + 64 * q));
      }
    }
    const int st = max(src_t(tt), 0);
#pragma unroll
    for (int q = 0; q < (SB != 0 ? NDP : 0); ++q) {
      const size_t e = (size_t)row0 * H + 2 * (lane + 64 * q) + (size_t)st * hstep;
      if constexpr (SRC) sq[q] = u64x2_t{ld_granule(S.din + e), ld_granule(S.din + e + 1)};
      else {
        const float2 v = *reinterpret_cast<const float2*>(S.dh + e);
        sq[q] = u64x2_t{(unsigned long long)__float_as_uint(v.x), (unsigned long long)__float_as_uint(v.y)};
      }
      if constexpr (UP) si[q] = *reinterpret_cast<const unsigned short*>(S.pidx + e);
      else si[q] = 0;
    }
  };
  auto io_stage = [&](auto sbc, int buf, int ss) {  // step ss's records and dh tile -> LDS buffer buf
    constexpr int SB = decltype(sbc)::value;
    const int tt = T - 1 - ss;
    const int st = src_t(tt);
    if constexpr (SRC && SB != 0) {
      bool bad = false;
#pragma unroll
      for (int q = 0; q < NDP; ++q)
        bad |= st >= 0 && ((unsigned)(sq[q].x >> 32) != (tagb | (unsigned)st) || (unsigned)(sq[q].y >> 32) != (tagb | (unsigned)st));
      if (__builtin_amdgcn_ballot_w64(bad) != 0) {   // re-poll the whole tile at once (bounded)
        const int lim0 = __hip_atomic_load(ctl + 6, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int lim = lim0 > 0 ? lim0 : CHAIN_SPIN;
        int nap = 1;
        for (int it = 0;; ++it) {
#pragma unroll
          for (int q = 0; q < NDP; ++q) {
            const size_t e = (size_t)row0 * H + 2 * (lane + 64 * q) + (size_t)max(st, 0) * hstep;
            sq[q] = u64x2_t{ld_granule(S.din + e), ld_granule(S.din + e + 1)};
          }
          bad = false;
#pragma unroll
          for (int q = 0; q < NDP; ++q)
            bad |= (unsigned)(sq[q].x >> 32) != (tagb | (unsigned)st) || (unsigned)(sq[q].y >> 32) != (tagb | (unsigned)st);
          if (__builtin_amdgcn_ballot_w64(bad) == 0) break;
          if (it >= lim) {
            __hip_atomic_store(ctl + 2, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            break;
          }
          for (int k = 0; k < nap; ++k) __builtin_amdgcn_s_sleep(2);
          nap = min(nap * 2, CHAIN_RP_NAPMAX);
        }
      }
    }
    const unsigned ph = UP ? (unsigned)(tt % P) : 0u;
#pragma unroll
    for (int q = 0; q < (SB != 0 ? NDP : 0); ++q) {
      const int e = 2 * (lane + 64 * q);
      const float v0 = __uint_as_float((unsigned)sq[q].x), v1 = __uint_as_float((unsigned)sq[q].y);
      const bool k0 = st >= 0 && (!UP || (si[q] & 0xffu) == ph), k1 = st >= 0 && (!UP || (si[q] >> 8) == ph);
      *reinterpret_cast<float2*>(&dhs[buf][e / H][e % H]) = make_float2(k0 ? v0 : 0.f, k1 ? v1 : 0.f);
    }
    const float cm = tt > 0 ? 1.f : 0.f;
#pragma unroll
    for (int q = 0; q < (SB != 1 ? CPLN / 4 : 0); ++q) {
      const int c0 = 4 * (lane + 64 * q);
      const uint4 ga = sg[2 * q], gb = sg[2 * q + 1];
      rec[buf][c0 + 0] = make_uint4(ga.x, ga.y, __float_as_uint(sc[q].x), __float_as_uint(scp[q].x * cm));
      rec[buf][c0 + 1] = make_uint4(ga.z, ga.w, __float_as_uint(sc[q].y), __float_as_uint(scp[q].y * cm));
      rec[buf][c0 + 2] = make_uint4(gb.x, gb.y, __float_as_uint(sc[q].z), __float_as_uint(scp[q].z * cm));
      rec[buf][c0 + 3] = make_uint4(gb.z, gb.w, __float_as_uint(sc[q].w), __float_as_uint(scp[q].w * cm));
    }
  };

  // ---------------------------------------------------------------- compute state
  const int unit = 4 * w + quad;
  const int au = 4 * w + (col >> 2);
  bf16x8_t ufr[KB];
  bf16x8_t wfr[TX][KB];
  if (compute) {
#pragma unroll
    for (int k = 0; k < KB; ++k) {
      bf16x8_t v;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float val = S.U[(size_t)au * G4 + 32 * k + 8 * quad + j];
        v[j] = (__bf16)(val * ((col & 3) == 0 ? 1.f : 0.f));
      }
      ufr[k] = v;
    }
#pragma unroll
    for (int q = 0; q < TX; ++q) {
      const int xb = w + NW * q;
      const int din = 16 * xb + col;
#pragma unroll
      for (int k = 0; k < KB; ++k) {
        bf16x8_t v;
#pragma unroll
        for (int j = 0; j < 8; ++j)
          v[j] = (__bf16)(S.W[(size_t)min(din, Dw - 1) * G4 + 32 * k + 8 * quad + j] *
                          ((xb < NXB && din < Dw) ? 1.f : 0.f));
        wfr[q][k] = v;
      }
    }
  }

  // ---------------------------------------------------------------- prologue
  // run f with this I/O wave's share as a compile-time constant
  auto io_dispatch = [&](auto f) {
    if constexpr (G == 1) f(ChIc<2>{});
    else if (sub == 0) f(ChIc<0>{});
    else f(ChIc<1>{});
  };
  if (!compute && !publisher) {
    if constexpr (SRC) {    // start once the stage above is D + LEAD steps ahead (see the forward)
      const int tw = max(T - 1 - (D + CHAINB_LEAD), 0);
      const int st = src_t(tw);
      if (st >= 0) (void)chain_wait(S.din + (size_t)row0 * H + (size_t)st * hstep, tagb | (unsigned)st, ctl);
    }
    io_dispatch([&](auto sbc) { io_load(sbc, min(iow, T - 1)); });
  }
  __syncthreads();
  if (!compute && !publisher && iow == 0) {
    io_dispatch([&](auto sbc) {
      io_stage(sbc, 0, 0);
      if (!CHAIN_DEFER_LD) io_load(sbc, min(D, T - 1));
    });
  }
  __syncthreads();
  if (tid == 0 && S.trace_mid) S.trace_mid[blockIdx.x] = (long long)__builtin_amdgcn_s_memrealtime();

  if (compute) {
    if (CHAIN_PRIO > 0) __builtin_amdgcn_s_setprio(CHAIN_PRIO);
    float dc = 0.f, dhr = 0.f;
    for (int s = 0; s < T; ++s) {
      const int t = T - 1 - s;
      const int p = s & 1;
      chain_mark(pr, s, 0);
      {   // cell: gate gradients of (unit, sequence col) at time t
        const uint4 r4 = rec[p][w * 64 + lane];
        const float dh = dhs[p][col][unit] + dhr;
        const float4 g4 = gates_unpack(make_uint2(r4.x, r4.y));
        const float ct = __uint_as_float(r4.z), cp = __uint_as_float(r4.w);
        const float tc = tanhf_fast(ct);
        const float dct = dc + dh * g4.w * (1.f - tc * tc);
        dc = dct * g4.y;
        zs[p][col][0 * H + unit] = (__bf16)(dct * g4.z * g4.x * (1.f - g4.x));
        zs[p][col][1 * H + unit] = (__bf16)(dct * cp * g4.y * (1.f - g4.y));
        zs[p][col][2 * H + unit] = (__bf16)(dct * g4.x * (1.f - g4.z * g4.z));
        zs[p][col][3 * H + unit] = (__bf16)(dh * tc * g4.w * (1.f - g4.w));
      }
      chain_mark(pr, s, 1);
      lds_barrier();
      chain_mark(pr, s, 2);
      {   // dh_{t-1} = U dz_t (the serial chain), then dx^T = W dz^T
        f32x4_t a0 = {0.f, 0.f, 0.f, 0.f}, a1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int k = 0; k < KB; ++k) {
          const bf16x8_t bz = *reinterpret_cast<const bf16x8_t*>(&zs[p][col][32 * k + 8 * quad]);
          if (k & 1) a1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ufr[k], bz, a1, 0, 0, 0);
          else a0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ufr[k], bz, a0, 0, 0, 0);
        }
        dhr = a0[0] + a1[0];     // (U^T rows with (col & 3) == 0: element 0 is this lane's unit)
      }
      chain_mark(pr, s, 3);
#pragma unroll
      for (int q = 0; q < TX; ++q) {
        const int xb = w + NW * q;
        if (xb < NXB) {
          f32x4_t a = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int k = 0; k < KB; ++k) {
            const bf16x8_t bz = *reinterpret_cast<const bf16x8_t*>(&zs[p][col][32 * k + 8 * quad]);
            a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wfr[q][k], bz, a, 0, 0, 0);
          }
#pragma unroll
          for (int r = 0; r < 4; ++r) dxs[p][col][16 * xb + 4 * quad + r] = a[r];
        }
      }
      chain_mark(pr, s, 4);
    }
    __builtin_amdgcn_s_setprio(0);
  } else if (publisher) {
    // after barrier s: step s's dz tile is complete (compute only reads it until barrier s + 1) and
    // step s - 1's dx tile too (written after barrier s - 1)
    auto store_dz = [&](int ss) {
      const int tz = T - 1 - ss;
      const int pb = ss & 1;
      __bf16* zt = S.dz + ((size_t)tz * Mp + row0) * G4;
#pragma unroll
      for (int q = lane; q < 16 * G4 / 8; q += 64) {
        const int e = 8 * q;
        *reinterpret_cast<uint4*>(zt + e) = *reinterpret_cast<const uint4*>(&zs[pb][e / G4][e % G4]);
      }
    };
    auto publish = [&](int ss) {            // step ss's dx tile
      const int tz = T - 1 - ss;
      const int pb = ss & 1;
      const unsigned tag = tagb | (unsigned)tz;
      const size_t xo = ((size_t)tz * Mp + row0) * Din;
      for (int e = lane; e < 16 * Din; e += 64) {
        const float v = dxs[pb][e / Din][e % Din];
        if constexpr (XO) st_granule(S.sout + xo + e, v, tag);
        else S.dx[xo + e] = v;
      }
    };
    for (int s = 0; s < T; ++s) {
      lds_barrier();
      store_dz(s);
      if (s >= 1) publish(s - 1);
    }
    __syncthreads();
    publish(T - 1);
    return;
  } else {
    io_dispatch([&](auto sbc) {
      const bool mk = lane == 0 && sub == G - 1;      // (phase marks: the dh wave, which tag-checks)
      int kt = (iow + D - 1) % D;           // steps until this group's turn
      int next_ld = iow == 0 ? D : -1;      // (deferred loads: see the forward's I/O loop)
      for (int s = 0; s < T; ++s) {
        if (CHAIN_DEFER_LD && next_ld >= 0) {
          io_load(sbc, min(next_ld, T - 1));
          next_ld = -1;
        }
        if (kt == 0 && s + 1 < T) {
          if (mk) chain_mark_wave(pr, s, 5);
          io_stage(sbc, (s + 1) & 1, s + 1);
          if (mk) chain_mark_wave(pr, s, 6);
          if (CHAIN_DEFER_LD) next_ld = s + 1 + D;
          else io_load(sbc, min(s + 1 + D, T - 1));
          if (mk) chain_mark_wave(pr, s, 7);
        }
        kt = kt == 0 ? D - 1 : kt - 1;
        lds_barrier();
      }
    });
  }
  __syncthreads();
}

// time4's backward on one 16-sequence tile with 1024 threads: the head backward (chain_head.h,
// waves 8..15 repeating waves 0..7), then the reverse recurrence with two cells per lane:
// dh_rec^T = U dz^T with wave w on unit tile w % 8 over K half w / 8, dx^T = W dz^T with din tile
// w % 4 over K quarter w / 4 (partials summed through LDS), dz -> HBM, dx -> granules (tag =
// pooled time of the chain's top layer). Then this tile's share of the head-gradient reduction.
__device__ __forceinline__ void chain_t4_bwd_stage(const ChainT4B Q, int tile, int ntiles, int Mp, unsigned tagb,
                                                   char* smem, long long* mk = nullptr) {
  constexpr int H = 128, G4 = 4 * H, NW = 16, CPL = 2, HP = H + 4, ZP = G4 + 8, XP = 68;
  using L = ChainT4BLds;
  static_assert(L::DHT % 16 == 0 && L::ZS % 16 == 0 && L::DN % 16 == 0, "t4 backward LDS layout");
  float* dhT = reinterpret_cast<float*>(smem);
  char* rs = smem + L::DHT;
  auto zs = reinterpret_cast<__bf16 (*)[ZP]>(rs);
  auto dhn = reinterpret_cast<float (*)[16][HP]>(rs + L::ZS);
  auto dxp = reinterpret_cast<float (*)[16][XP]>(rs + L::ZS + L::DN);
  const int T = Q.T, Din = Q.Din, Dw = Q.Dw;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int col = lane & 15, quad = lane >> 4;
  const int row0 = tile * 16;

  int unit[CPL];
  size_t so[CPL];                                  // this cell's index in time4's state layout (t = 0)
#pragma unroll
  for (int cc = 0; cc < CPL; ++cc) {
    const int gi = w + NW * cc;
    unit[cc] = 4 * gi + quad;
    so[cc] = (((size_t)tile * 8 + (gi & 7)) * 4 + (gi >> 3)) * 64 + lane;
  }
  const size_t sstep = (size_t)ntiles * 8 * 4 * 64;
  // forward state ring (2 reverse steps), refilled right after the cell phase that used a slot
  float4 rg[2][CPL];
  float2 rcs[2][CPL];
  auto load_slot = [&](int j, int t) {
    const size_t tc = (size_t)max(t, 0);
#pragma unroll
    for (int cc = 0; cc < CPL; ++cc) {
      const size_t o = tc * sstep + so[cc];
      rg[j][cc] = *reinterpret_cast<const float4*>(Q.g + o * 4);
      rcs[j][cc] = *reinterpret_cast<const float2*>(Q.c + o * 2);
    }
  };
  load_slot(0, T - 1);
  load_slot(1, T - 2);
  if (Q.hb != nullptr) {                           // precomputed by the forward (dL/dloss = 1): scale
    const float gl = Q.hd.dloss[0];
    for (int e = tid; e < 16 * H; e += 1024) dhT[(e / H) * HP + e % H] = gl * Q.hb[((size_t)tile * 16 + e / H) * H + e % H];
  } else {
    chain_head_bwd<H>(Q.hd, Q.h + (size_t)(T - 1) * Mp * H, tile, ntiles, dhT, rs);
  }
  // weight fragments (after the head prologue: live through it they would crowd its registers),
  // from the forward's lane-contiguous fragment image (time4_head.hip's backward layout: wave
  // w' < 8 holds unit tile w' over the full K, and din tile w' % 4 over gate-column half w' / 4)
  const int ut = w & 7, kh = w >> 3, dt = w & 3, kq = w >> 2;
  bf16x8_t ufr[8], wfr[4];
  {
    const bf16x8_t* pu = Q.pk + T4PK_N + (size_t)ut * 16 * 64 + lane;
    const bf16x8_t* pw = Q.pk + T4PK_N + T4PK_BU + (size_t)(dt + 4 * (kq >> 1)) * 8 * 64 + lane;
#pragma unroll
    for (int s = 0; s < 8; ++s) ufr[s] = pu[(8 * kh + s) * 64];
#pragma unroll
    for (int s = 0; s < 4; ++s) wfr[s] = pw[(4 * (kq & 1) + s) * 64];
  }
  __syncthreads();                                 // the head scratch becomes the step tiles
  if (mk != nullptr && tid == 0) mk[0] = (long long)__builtin_amdgcn_s_memrealtime();   // (trace: head done)
  // dx element of this thread (threads past the [16][Din] tile re-read the last one, no store)
  const int nx = 16 * Din;
  const bool ownx = tid < nx;
  const int ex = min(tid, nx - 1), er = ex / Din, ek = ex % Din;
  const size_t xstep = (size_t)Mp * Din, xoff = (size_t)(row0 + er) * Din + ek;
  const int zq = tid >> 6, zc = (tid & 63) * 8;    // dz store: 8 bf16 of the [16][512] tile
  float dc[CPL], dhr[CPL];
#pragma unroll
  for (int cc = 0; cc < CPL; ++cc) dc[cc] = dhr[cc] = 0.f;
  for (int s0 = 0; s0 < T; s0 += 2) {
#pragma unroll
  for (int j = 0; j < 2; ++j) {                   // (static ring slot: a dynamic index spilled the ring)
    const int s = s0 + j;
    if (s >= T) break;
    const int t = T - 1 - s;
#pragma unroll
    for (int cc = 0; cc < CPL; ++cc) {
      const int u = unit[cc];
      const float dh = dhr[cc] + (s == 0 ? dhT[col * HP + u] : 0.f);
      const float4 g = rg[j][cc];
      const float cprev = rcs[j][cc].y;            // (0 at t = 0: the forward's initial state)
      const float tc = tanhf_fast(rcs[j][cc].x);
      const float dct = dc[cc] + dh * g.w * (1.f - tc * tc);
      dc[cc] = dct * g.y;
      zs[col][0 * H + u] = (__bf16)(dct * g.z * g.x * (1.f - g.x));
      zs[col][1 * H + u] = (__bf16)(dct * cprev * g.y * (1.f - g.y));
      zs[col][2 * H + u] = (__bf16)(dct * g.x * (1.f - g.z * g.z));
      zs[col][3 * H + u] = (__bf16)(dh * tc * g.w * (1.f - g.w));
    }
    load_slot(j, t - 2);
    lds_barrier();
    *reinterpret_cast<uint4*>(Q.dz + ((size_t)t * Mp + row0 + zq) * G4 + zc) = *reinterpret_cast<const uint4*>(&zs[zq][zc]);
    {
      f32x4_t a0 = {0.f, 0.f, 0.f, 0.f}, a1 = a0, b0 = a0, b1 = a0;
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const bf16x8_t bz = *reinterpret_cast<const bf16x8_t*>(&zs[col][32 * (8 * kh + q) + 8 * quad]);
        if (q & 1) a1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ufr[q], bz, a1, 0, 0, 0);
        else a0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ufr[q], bz, a0, 0, 0, 0);
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const bf16x8_t bz = *reinterpret_cast<const bf16x8_t*>(&zs[col][32 * (4 * kq + q) + 8 * quad]);
        if (q & 1) b1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wfr[q], bz, b1, 0, 0, 0);
        else b0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wfr[q], bz, b0, 0, 0, 0);
      }
      const f32x4_t a = a0 + a1, b = b0 + b1;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        dhn[kh][col][16 * ut + 4 * quad + r] = a[r];
        dxp[kq][col][16 * dt + 4 * quad + r] = b[r];
      }
    }
    lds_barrier();
#pragma unroll
    for (int cc = 0; cc < CPL; ++cc) dhr[cc] = dhn[0][col][unit[cc]] + dhn[1][col][unit[cc]];
    const float v = (dxp[0][er][ek] + dxp[1][er][ek]) + (dxp[2][er][ek] + dxp[3][er][ek]);
    if (ownx) st_granule(Q.sout + xoff + (size_t)t * xstep, v, tagb | (unsigned)t);
  }
  }
  if (mk != nullptr && tid == 0) mk[64] = (long long)__builtin_amdgcn_s_memrealtime();  // (trace: steps done)
  if (Q.hb != nullptr) {
    ChainHead hd = Q.hd;
    hd.gpart = const_cast<float*>(Q.hb) + (size_t)ntiles * 16 * H;
    chain_head_bwd_reduce<H>(hd, tile, ntiles, true, Q.hd.dloss[0]);
  } else {
    chain_head_bwd_reduce<H>(Q.hd, tile, ntiles);
  }
}

__global__ __launch_bounds__(1024) void lstm_chain_bwd_kernel(ChainBArgs A) {
  const int nblk = gridDim.x;
  __shared__ __attribute__((aligned(16))) char smem[CHAINB_LDS];
  const int s = blockIdx.x / A.nt8, tile = blockIdx.x % A.nt8;
  if (s == A.ns && A.t4.on && tile < A.ntiles) {  // time4 + head backward of this tile
    if (threadIdx.x == 0) A.trace[2 * blockIdx.x] = (long long)__builtin_amdgcn_s_memrealtime();
    const unsigned tagb = chain_tag_base((unsigned)__hip_atomic_load(A.ctl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    chain_t4_bwd_stage(A.t4, tile, A.ntiles, A.Mp, tagb, smem, blockIdx.x < 64 ? A.trace + 512 + blockIdx.x : nullptr);
    __syncthreads();
    if (threadIdx.x == 0) A.trace[2 * blockIdx.x + 1] = (long long)__builtin_amdgcn_s_memrealtime();
    chain_finish(A.ctl, nblk);
    return;
  }
  if (s >= A.ns || tile >= A.ntiles) {
    chain_finish(A.ctl, nblk);
    return;
  }
  if (threadIdx.x == 0) A.trace[2 * blockIdx.x] = (long long)__builtin_amdgcn_s_memrealtime();
  const unsigned E = (unsigned)__hip_atomic_load(A.ctl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const unsigned tagb = chain_tag_base(E);
  // the stage record is loaded field by field from the kernel arguments (scalar loads): a
  // reference into the by-value argument array made the compiler copy the whole array to
  // scratch and read every field from there inside the step loop
  const ChainBStage S = A.st[s];
  const int H = S.H, KX = S.KX;
  const bool src = s > 0 || A.t4.on;              // (stage 0 then reads time4's dx granules)
#define GQ_CHAINB_BODY3(HH, KXX, DD, SRCV, UPV, XOV)                                    \
  {                                                                                     \
    if constexpr (HH == 16 && CHAINB_IO) {                                              \
      if (threadIdx.x >= chainb_io_threads(TMC<HH>::NT, DD)) return;                    \
      chain_bwd_stage_io<HH, KXX, DD, SRCV, UPV, XOV>(S, tile, A.ntiles, A.Mp, tagb, A.ctl, smem); \
    } else {                                                                            \
      if (threadIdx.x >= chainb_live_threads(HH, TMC<HH>::NT)) return;                   \
      chain_bwd_stage<HH, KXX, DD, SRCV, UPV, XOV>(S, tile, A.ntiles, A.Mp, tagb, A.ctl, smem); \
    }                                                                                   \
  }
#define GQ_CHAINB_BODY2(HH, KXX, DD, SRCV, UPV)                                         \
  if (!SRCV || S.sout) GQ_CHAINB_BODY3(HH, KXX, DD, SRCV, UPV, true)                    \
  else GQ_CHAINB_BODY3(HH, KXX, DD, SRCV, UPV, false)
#define GQ_CHAINB_BODY(HH, KXX, DD)                                                     \
  {                                                                                     \
    if (src) { if (S.P > 0 && !S.punp) { GQ_CHAINB_BODY2(HH, KXX, DD, true, true) }    \
               else { GQ_CHAINB_BODY2(HH, KXX, DD, true, false) } }                     \
    else { if (S.P > 0) { GQ_CHAINB_BODY3(HH, KXX, DD, false, true, true) }             \
           else { GQ_CHAINB_BODY3(HH, KXX, DD, false, false, true) } }                  \
  }
#ifdef CHAINB_ONLY
  { GQ_CHAINB_BODY3(CHAINB_ONLY, CHAINB_KX, CHAINB_DONLY, CHAINB_SRC, CHAINB_UP, true) }
#else
  if (H == 16) { if (KX == 1) GQ_CHAINB_BODY(16, 1, CHAINB_D16) else GQ_CHAINB_BODY(16, 2, CHAINB_D16) }
  else if (H == 32) { if (KX == 1) GQ_CHAINB_BODY(32, 1, CHAINB_D32) else GQ_CHAINB_BODY(32, 2, CHAINB_D32) }
  else { if (KX == 1) GQ_CHAINB_BODY(64, 1, CHAINB_D64) else GQ_CHAINB_BODY(64, 2, CHAINB_D64) }
#endif
#undef GQ_CHAINB_BODY
#undef GQ_CHAINB_BODY2
#undef GQ_CHAINB_BODY3
  __syncthreads();
  if (threadIdx.x == 0) A.trace[2 * blockIdx.x + 1] = (long long)__builtin_amdgcn_s_memrealtime();
  chain_finish(A.ctl, nblk);
}

// ---------------------------------------------------------------------------------------
// host
static long long* chain_trace_buf(int dev) {
  static long long* tr[64] = {nullptr};
  // [0, 512): per-workgroup start / end; [512, 768): stage-loop start (backward)
  if (!tr[dev]) TORCH_CHECK(hipMalloc(&tr[dev], 3 * 256 * sizeof(long long)) == hipSuccess,
                            "lstm_chain: trace");
  return tr[dev];
}

// tile 0's per-step phase clocks [CHAIN_MAX stages][CHAIN_PROF_STEPS][8] of the last launch with
// GNNQC_CHAIN_PROF=1 (forward and backward use the same buffer)
static long long* chain_prof_buf(int dev);
// zero the phase-clock buffer before a profiled launch: a stage with fewer than CHAIN_PROF_STEPS
// steps (or fewer marks) than the previous launch's would otherwise leave that launch's rows behind
// (the round-4 table's backward rows 0-1 and m6 columns were such leftovers)
static void chain_prof_clear(int dev) {
  long long* pb = chain_prof_buf(dev);
  if (pb != nullptr)
    TORCH_CHECK(hipMemsetAsync(pb, 0, CHAIN_MAX * CHAIN_PROF_STEPS * 8 * sizeof(long long), stream()) == hipSuccess,
                "chain prof clear");
}
static long long* chain_prof_buf(int dev) {
#ifdef GQ_CHAIN_PROF
  static const bool on = [] {
    const char* e = std::getenv("GNNQC_CHAIN_PROF");
    return e != nullptr && e[0] == '1';
  }();
#else
  const bool on = false;
#endif
  if (!on) return nullptr;
  static long long* pb[64] = {nullptr};
  if (!pb[dev]) {
    TORCH_CHECK(hipMalloc(&pb[dev], CHAIN_MAX * CHAIN_PROF_STEPS * 8 * sizeof(long long)) == hipSuccess, "chain prof");
    TORCH_CHECK(hipMemset(pb[dev], 0, CHAIN_MAX * CHAIN_PROF_STEPS * 8 * sizeof(long long)) == hipSuccess, "chain prof");
  }
  return pb[dev];
}

at::Tensor lstm_chain_prof(const at::Tensor& like) {
  c10::DeviceGuard guard(like.device());
  long long* p = chain_prof_buf(like.get_device());
  TORCH_CHECK(p != nullptr, "lstm_chain_prof: build with GNNQC_CHAIN_PROF_BUILD=1 and set GNNQC_CHAIN_PROF=1 "
                            "before the first chain launch");
  at::Tensor o = at::empty({CHAIN_MAX, CHAIN_PROF_STEPS, 8}, like.options().dtype(at::kLong));
  TORCH_CHECK(hipMemcpyAsync(o.data_ptr<int64_t>(), p, o.numel() * sizeof(long long), hipMemcpyDeviceToDevice,
                             stream()) == hipSuccess, "lstm_chain_prof");
  return o;
}

int* chain_ctl(int dev) {
  static int* ctl[64] = {nullptr};
  TORCH_CHECK(dev >= 0 && dev < 64, "lstm_chain: device index");
  if (!ctl[dev]) {
    hipStreamCaptureStatus cs;
    TORCH_CHECK(hipStreamIsCapturing(stream(), &cs) == hipSuccess && cs == hipStreamCaptureStatusNone,
                "lstm_chain: first use must not be inside a graph capture");
    int* p = nullptr;
    TORCH_CHECK(hipMalloc(&p, 16 * sizeof(int)) == hipSuccess, "lstm_chain: control word allocation");
    const int init[16] = {1, 0};     // epoch 1; [4], [5]: head tickets; [8]: head backward reduce arrivals
    TORCH_CHECK(hipMemcpy(p, init, sizeof(init), hipMemcpyHostToDevice) == hipSuccess, "lstm_chain: init");
    ctl[dev] = p;
  }
  return ctl[dev];
}

// Workgroups of the chain kernels that can be resident at once on this device: the CU count
// of the device (a partitioned MI355X exposes fewer) times the occupancy of the 1024-thread
// chain kernels (with their LDS and VGPR use). Every workgroup of a chain launch must be
// resident, or consumers spin on producers that are never scheduled.
static int chain_capacity(int dev) {
  static int cap[64] = {0};
  TORCH_CHECK(dev >= 0 && dev < 64, "lstm_chain: device index");
  if (cap[dev] == 0) {
    hipDeviceProp_t prop;
    TORCH_CHECK(hipGetDeviceProperties(&prop, dev) == hipSuccess, "lstm_chain: device properties");
    int occ = 1 << 30;
    const void* kernels[] = {reinterpret_cast<const void*>(&lstm_chain_fwd_kernel<true>),
                             reinterpret_cast<const void*>(&lstm_chain_fwd_kernel<false>),
                             reinterpret_cast<const void*>(&lstm_chain_bwd_kernel)};
    for (const void* k : kernels) {
      int n = 0;
      TORCH_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k, 1024, 0) == hipSuccess,
                  "lstm_chain: occupancy query");
      occ = std::min(occ, n);
    }
    cap[dev] = std::max(0, occ) * prop.multiProcessorCount;
  }
  return cap[dev];
}

int64_t lstm_chain_capacity(const at::Tensor& like) {
  TORCH_CHECK(like.is_cuda(), "lstm_chain_capacity: a GPU tensor names the device");
  return chain_capacity(like.get_device());
}

// The device's chain control words as an int32[16] view (no copy): [epoch, finished workgroups,
// spin-timeout flag, timeouts consumed by the gradient guard, time4/head kernel tickets (2),
// debug spin limit (0: default), a gradient producer saw a non-finite value, head backward
// reduce arrivals, 0...]. The optimiser's update reads and clears the flags inside the captured
// step (a timed-out or non-finite step is skipped, never applied).
at::Tensor lstm_chain_ctl(const at::Tensor& like) {
  TORCH_CHECK(like.is_cuda(), "lstm_chain_ctl: a GPU tensor names the device");
  c10::DeviceGuard guard(like.device());
  int* p = chain_ctl(like.get_device());
  return at::from_blob(p, {16}, like.options().dtype(at::kInt));
}

// x [T, Mp, Din] (Din % 4 == 0, 16-B aligned); per stage W [Dw, 4H], U [H, 4H], b [4H];
// pool[s] > 0: MaxPooling1D(pool[s]) after stage s. Returns per stage [h, g, c, pooled, idx].
// time4 + head as a chain stage (lstm_chain_head_fwd): its weights, the head and the loss inputs
struct T4Host {
  const at::Tensor* b;
  at::TensorList head;
  const at::Tensor* y;
  const at::Tensor* mask;
  int64_t M;
  double alpha1, alpha2, w0, w1;
  at::Tensor sums, hist;
};

// time4_head.hip: the forward head arguments (weights, labels, metric accumulators, ticket)
void t4_head_fwd_args(ChainHead& hd, at::TensorList head, const at::Tensor& y, const at::Tensor& mask, int64_t M,
                      int Mp, double alpha1, double alpha2, double w0, double w1, const at::Tensor& sums,
                      const at::Tensor& hist, at::Tensor& logits, at::Tensor& loss, at::Tensor& part);

static std::vector<at::Tensor> chain_fwd_impl(const at::Tensor& x, at::TensorList W, at::TensorList U,
                                              at::TensorList b, at::IntArrayRef pool, bool train, const at::Tensor* pkW,
                                              const at::Tensor* pkU, const T4Host* t4 = nullptr);

std::vector<at::Tensor> lstm_chain_fwd(const at::Tensor& x, at::TensorList W, at::TensorList U, at::TensorList b,
                                       at::IntArrayRef pool, bool train) {
  return chain_fwd_impl(x, W, U, b, pool, train, nullptr, nullptr);
}

// The chain forward, whose spare workgroups also build the time4 kernel's fragment image of
// (Wt4 [Din, 512], Ut4 [128, 512]); the image is appended to the result.
std::vector<at::Tensor> lstm_chain_fwd_pack(const at::Tensor& x, at::TensorList W, at::TensorList U,
                                            at::TensorList b, at::IntArrayRef pool, bool train, const at::Tensor& Wt4,
                                            const at::Tensor& Ut4) {
  return chain_fwd_impl(x, W, U, b, pool, train, &Wt4, &Ut4);
}

// The chain forward with time4 (Wt4 [Din, 512], Ut4 [128, 512], bt4 [512], last state only) and the
// classifier head + weighted BCE (head = [W1, b1, W2, b2, W3, b3], y / mask [M]) as one more stage
// consuming the last chain stage's output, which must be max-pooled by 3 (chain_t4_stage). Returns
// lstm_chain_fwd_pack's result followed by [h4 [T4, Mp, 128], g4, c4, logits [M], loss [1]] (the
// outputs of time4_head_fwd); with sums / hist non-empty the metric accumulators are updated.
std::vector<at::Tensor> lstm_chain_head_fwd(const at::Tensor& x, at::TensorList W, at::TensorList U, at::TensorList b,
                                            at::IntArrayRef pool, bool train, const at::Tensor& Wt4,
                                            const at::Tensor& Ut4, const at::Tensor& bt4, at::TensorList head,
                                            const at::Tensor& y, const at::Tensor& mask, int64_t M, double alpha1,
                                            double alpha2, double w0, double w1, at::Tensor sums, at::Tensor hist) {
  T4Host h4{&bt4, head, &y, &mask, M, alpha1, alpha2, w0, w1, sums, hist};
  return chain_fwd_impl(x, W, U, b, pool, train, &Wt4, &Ut4, &h4);
}

static std::vector<at::Tensor> chain_fwd_impl(const at::Tensor& x, at::TensorList W, at::TensorList U,
                                              at::TensorList b, at::IntArrayRef pool, bool train, const at::Tensor* pkW,
                                              const at::Tensor* pkU, const T4Host* t4) {
  check_f32_cuda(x, "x");
  const int ns = (int)W.size();
  TORCH_CHECK(ns >= 1 && ns <= CHAIN_MAX && (int)U.size() == ns && (int)b.size() == ns && (int)pool.size() == ns,
              "lstm_chain: stage lists");
  TORCH_CHECK(x.dim() == 3 && x.is_contiguous(), "lstm_chain: x must be a contiguous [T, Mp, Din]");
  const int Mp = (int)x.size(1);
  TORCH_CHECK(Mp % 16 == 0, "lstm_chain: Mp must be a multiple of 16");
  const int ntiles = Mp / 16, nt8 = (ntiles + 7) / 8 * 8;
  TORCH_CHECK(ns * nt8 <= chain_capacity(x.get_device()), "lstm_chain: ", ns * nt8,
              " workgroups cannot all be resident on this device");
  TORCH_CHECK(x.size(2) % 4 == 0 && reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0,
              "lstm_chain: x channels must be float4 granules");
  c10::DeviceGuard guard(x.device());
  auto opt = x.options();
  ChainArgs A{};
  A.ns = ns;
  A.ntiles = ntiles;
  A.nt8 = nt8;
  A.Mp = Mp;
  A.ctl = chain_ctl(x.get_device());
  A.trace = chain_trace_buf(x.get_device());
  chain_prof_clear(x.get_device());
  std::vector<at::Tensor> out;
  at::Tensor prev_stream;
  int T = (int)x.size(0), Din = (int)x.size(2);
  for (int s = 0; s < ns; ++s) {
    for (const at::Tensor* t : {&W[s], &U[s], &b[s]}) check_f32_cuda(*t, "lstm_chain weight");
    const int H = (int)U[s].size(0), Dw = (int)W[s].size(0);
    TORCH_CHECK(H == 16 || H == 32 || H == 64, "lstm_chain: hidden size ", H);
    TORCH_CHECK(W[s].size(1) == 4 * H && U[s].size(1) == 4 * H && b[s].numel() == 4 * H, "lstm_chain: weights");
    TORCH_CHECK(Dw <= Din && Din <= 64 && (s == 0 || Din <= H), "lstm_chain: stage ", s, " input width ", Din);
    TORCH_CHECK(T >= 1 && T < 4096, "lstm_chain: sequence length");
    const int P = (int)pool[s];
    const bool last = s + 1 == ns && t4 == nullptr;   // (time4 consumes the last chain stage)
    TORCH_CHECK(last || P == 0 || P == 3, "lstm_chain: pools between stages must be 3 (got ", P, ")");
    TORCH_CHECK(t4 == nullptr || s + 1 < ns || P == 3, "lstm_chain_head_fwd: the last chain stage must pool by 3");
    ChainStage& S = A.st[s];
    S.x = s == 0 ? x.data_ptr<float>() : nullptr;
    S.xin = s == 0 ? nullptr : reinterpret_cast<const unsigned long long*>(prev_stream.data_ptr<int64_t>());
    S.W = W[s].data_ptr<float>();
    S.U = U[s].data_ptr<float>();
    S.b = b[s].data_ptr<float>();
    at::Tensor h = at::empty({T + 1, Mp, H}, opt);
    at::Tensor g = train ? at::empty({T + 1, Mp, H, 4}, opt.dtype(at::kBFloat16)) : at::empty({0}, opt);
    at::Tensor c = train ? at::empty({T + 1, Mp, H}, opt) : at::empty({0}, opt);
    at::Tensor pooled, pidx;
    const TmPool pl = tm_pool_outputs(P, T, Mp, H, opt, pooled, pidx);
    const int To = P > 0 ? T / P : T;
    TORCH_CHECK(To >= 1, "lstm_chain: pooled length");
    // the stream carries the UNPOOLED h: a pooling consumer pools it (and writes pooled / pidx)
    at::Tensor so = !last ? at::empty({T, Mp, H}, opt.dtype(at::kLong)) : at::Tensor();
    S.h = h.data_ptr<float>();
    S.g = train ? bf16_ptr(g) : nullptr;
    S.c = train ? c.data_ptr<float>() : nullptr;
    S.sout = so.defined() ? reinterpret_cast<unsigned long long*>(so.data_ptr<int64_t>()) : nullptr;
    S.pout = last ? pl.out : nullptr;
    S.iout = last ? pl.idx : nullptr;
    S.P = last ? P : 0;
    if (!last && P > 0 && s + 1 < ns) {          // the next stage pools this stage's output
      A.st[s + 1].pin_out = pooled.data_ptr<float>();
      A.st[s + 1].pin_idx = pidx.data_ptr<uint8_t>();
    } else if (!last && P > 0) {                 // ... or time4 does
      A.t4.pin_out = pooled.data_ptr<float>();
      A.t4.pin_idx = pidx.data_ptr<uint8_t>();
    }
    S.H = H;
    S.T = T;
    S.Din = Din;
    S.Dw = Dw;
    S.KX = (Din + 31) / 32;
    S.PIN = s > 0 ? std::max(1, (int)pool[s - 1]) : 1;
    // a stage without I/O waves (H = 64) streams one granule per thread (chain_stage NGL)
    TORCH_CHECK(H < 64 || 16 * Din / (s == 0 ? 4 : 2) <= 64 * TMC<64>::NW, "lstm_chain: stage ", s, " input tile");
    TORCH_CHECK(s == 0 || (long)T * Mp * Din * 8 < (1L << 31), "lstm_chain: stage ", s, " input stream too large");
    TORCH_CHECK(s == 0 || Din % 2 == 0, "lstm_chain: stage ", s, " input width must be even");
    TORCH_CHECK(s > 0 || Din % 4 == 0, "lstm_chain: the input width must be a multiple of 4");
    {
      long long* pb = chain_prof_buf(x.get_device());
      S.prof = pb != nullptr ? pb + (size_t)s * CHAIN_PROF_STEPS * 8 : nullptr;
    }
    out.insert(out.end(), {h.narrow(0, 0, T), g, c, pooled, pidx});
    if (so.defined()) out.push_back(so);        // kept alive until the launch is enqueued
    prev_stream = so;
    T = To;
    Din = H;
  }
  int nblk = ns * nt8;
  std::vector<at::Tensor> t4out;
  at::Tensor hb_t;
  if (t4 != nullptr) {
    TORCH_CHECK(pkW != nullptr && pkU != nullptr, "lstm_chain_head_fwd: time4 weights");
    check_f32_cuda(*t4->b, "bt4");
    const int Dw4 = (int)pkW->size(0);
    TORCH_CHECK(T >= 1 && T <= 16, "lstm_chain_head_fwd: time4 sequence length 1..16 (got ", T, ")");
    TORCH_CHECK(Din <= 64 && Dw4 >= 1 && Dw4 <= Din && t4->b->numel() == 512, "lstm_chain_head_fwd: time4 input width");
    ChainT4& Q = A.t4;
    Q.on = 1;
    Q.xin = reinterpret_cast<const unsigned long long*>(prev_stream.data_ptr<int64_t>());
    Q.W = pkW->data_ptr<float>();
    Q.U = pkU->data_ptr<float>();
    Q.b = t4->b->data_ptr<float>();
    at::Tensor h4 = at::empty({T, Mp, 128}, opt);
    at::Tensor g4 = train ? at::empty({(long)T * Mp * 128 * 4}, opt) : at::empty({0}, opt);
    at::Tensor c4 = train ? at::empty({(long)T * Mp * 128 * 2}, opt) : at::empty({0}, opt);
    Q.h = h4.data_ptr<float>();
    Q.g = train ? g4.data_ptr<float>() : nullptr;
    Q.c = train ? c4.data_ptr<float>() : nullptr;
    Q.T = T;
    Q.Din = Din;
    Q.Dw = Dw4;
    at::Tensor logits, loss, part;
    t4_head_fwd_args(Q.hd, t4->head, *t4->y, *t4->mask, t4->M, Mp, t4->alpha1, t4->alpha2, t4->w0, t4->w1, t4->sums,
                     t4->hist, logits, loss, part);
    t4out = {h4, g4, c4, logits, loss, part};
    // the head backward precomputed by this launch (GNNQC_HEAD_BWD_IN_FWD=0: the backward runs it)
    const char* hbe = std::getenv("GNNQC_HEAD_BWD_IN_FWD");
    if (train && !(hbe != nullptr && hbe[0] == '0')) {
      hb_t = at::empty({(long)ntiles * 16 * 128 + (long)ntiles * ChainHeadRec<128>::PITCH}, opt);
      Q.hb = hb_t.data_ptr<float>();
    } else {
      hb_t = at::empty({0}, opt);
    }
    nblk += nt8;
  }
  at::Tensor pk;
  if (pkW != nullptr) {
    check_f32_cuda(*pkW, "Wt4");
    check_f32_cuda(*pkU, "Ut4");
    TORCH_CHECK(pkU->size(0) == 128 && pkU->size(1) == 512 && pkW->size(1) == 512 && pkW->size(0) <= 64,
                "lstm_chain_fwd_pack: time4 weights must be [<=64, 512] and [128, 512]");
    pk = at::empty({(long)T4PK_ALL * 4}, opt);                // 16 B per fragment (forward + backward)
    A.pkU = pkU->data_ptr<float>();
    A.pkW = pkW->data_ptr<float>();
    A.pkDw = (int)pkW->size(0);
    A.pk = reinterpret_cast<bf16x8_t*>(pk.data_ptr<float>());
    A.npk = (T4PK_ALL + 1023) / 1024;
    nblk += A.npk;
    TORCH_CHECK(nblk <= chain_capacity(x.get_device()), "lstm_chain: ", nblk,
                " workgroups cannot all be resident on this device");
  }
  // a deferred GCN forward (gcn_fused_fwd defer) whose output is this launch's input runs as
  // producer workgroups of this launch (the first stage streams their granules, the head waits for
  // their labels); any other pending one runs on its own first
  std::vector<at::Tensor> gp_keep;
  {
    const int dev = x.get_device();
    const GcnProdJob& P = gcn_pending(dev).prod;
    if (P.on) {
      const int H0 = A.st[0].H, Din0 = A.st[0].Din;
      const bool mine = train && t4 != nullptr && P.out == x.data_ptr<float>() && P.Mp == Mp &&
                        P.Cp == Din0 && P.D.T == (int)x.size(0) && Din0 % 2 == 0 &&
                        (H0 < 64 || 16 * Din0 / 2 <= 64 * TMC<64>::NW) &&
                        (long)P.D.T * Mp * Din0 * 8 < (1L << 31) && nblk + P.Mp <= chain_capacity(dev);
      if (mine) {
        static_assert(GcnProdLds::BYTES <= CHAIN_LDS, "GCN producer LDS");
        gcn_prod_take(dev, A.gp, gp_keep);
        A.st[0].xin = A.gp.gout;
        nblk += A.gp.Mp;
      } else {
        gcn_prod_flush_dev(dev);
      }
    }
  }
  // a pending GCN coefficient job (gcn_fused_fwd, side mode) rides on this launch when its
  // workgroups fit the co-resident grid as well; else it stays pending (gcn_coef_flush runs it)
  std::vector<at::Tensor> cf_keep;
  if (gcn_pending(x.get_device()).job.on && train &&
      nblk + gcn_pending(x.get_device()).job.Mp <= chain_capacity(x.get_device())) {
    static_assert(GcnCoefFwdLds::BYTES <= CHAIN_LDS, "coefficient job LDS");
    gcn_coef_take(x.get_device(), A.cf, cf_keep);
    nblk += A.cf.Mp;
  }
  if (train)
    hipLaunchKernelGGL(lstm_chain_fwd_kernel<true>, dim3(nblk), dim3(1024), 0, stream(), A);
  else
    hipLaunchKernelGGL(lstm_chain_fwd_kernel<false>, dim3(nblk), dim3(1024), 0, stream(), A);
  GQ_LAUNCH_CHECK();
  // drop the stream buffers from the result (the caching allocator orders their reuse)
  std::vector<at::Tensor> res;
  for (auto& t : out)
    if (t.scalar_type() != at::kLong) res.push_back(t);
  if (pk.defined()) res.push_back(pk);
  if (hb_t.defined()) res.push_back(hb_t);        // (headed launch: [.., pk, hb, h4, g4, c4, logits, loss])
  for (int i = 0; i < 5 && i < (int)t4out.size(); ++i) res.push_back(t4out[i]);
  return res;
}

// Backward of a chain, stages listed TOP layer first. dh: gradient of the top layer's output
// (pooled if pool[0] > 0); per stage the forward's g / c, W, U, the argmax bytes of the pool
// after the layer (empty if none) and pool size; x_width[s]: channels of the layer's input
// layout. Returns [dz_0 .. dz_{n-1}, dx of the bottom layer].
static std::vector<at::Tensor> chain_bwd_setup(ChainBArgs& A, std::vector<at::Tensor>& keep, const at::Tensor& dh,
                                               at::TensorList g, at::TensorList c, at::TensorList W, at::TensorList U,
                                               at::TensorList pidx, at::IntArrayRef pool, at::IntArrayRef x_width,
                                               at::IntArrayRef T_in, int extra_blocks);

std::vector<at::Tensor> lstm_chain_bwd(const at::Tensor& dh, at::TensorList g, at::TensorList c, at::TensorList W,
                                       at::TensorList U, at::TensorList pidx, at::IntArrayRef pool,
                                       at::IntArrayRef x_width, at::IntArrayRef T_in) {
  ChainBArgs A{};
  std::vector<at::Tensor> keep;
  auto res = chain_bwd_setup(A, keep, dh, g, c, W, U, pidx, pool, x_width, T_in, 0);
  hipLaunchKernelGGL(lstm_chain_bwd_kernel, dim3(A.ns * A.nt8), dim3(1024), 0, stream(), A);
  GQ_LAUNCH_CHECK();
  return res;
}

// time4_head.hip: the backward head arguments (weights, labels, dloss, gradient sinks, tickets)
void t4_head_bwd_args(ChainHead& hd, at::TensorList head, const at::Tensor& y, const at::Tensor& mask, int64_t M,
                      int Mp, double alpha1, double alpha2, double w0, double w1, const at::Tensor& dloss,
                      at::TensorList hgrads, at::Tensor& gpart);

// lstm_chain_bwd with time4 + the head as its first stage (chain_t4_bwd_stage): dloss [1]; x4 the
// pooled top chain output (time4's input, [T4, Mp, Din]); h4 / g4 / c4 time4's saved forward state
// (lstm_chain_head_fwd / time4_head_fwd); Wt4 / Ut4 its weights and pk their fragment image (the
// forward's last result); head = [W1, b1, W2, b2, W3, b3]
// with their gradients hgrads (accumulated); then the chain stages, TOP layer first, as for
// lstm_chain_bwd (the top one must pool by 3). Returns [dz4 [T4 + 1, Mp, 512], dz_0 .. dz_{n-1}, dx].
std::vector<at::Tensor> lstm_chain_head_bwd(const at::Tensor& dloss, const at::Tensor& x4, const at::Tensor& h4,
                                            const at::Tensor& g4, const at::Tensor& c4, const at::Tensor& Wt4,
                                            const at::Tensor& Ut4, const at::Tensor& pk, const at::Tensor& hb,
                                            at::TensorList head, const at::Tensor& y,
                                            const at::Tensor& mask, int64_t M, double alpha1, double alpha2, double w0,
                                            double w1, at::TensorList hgrads, at::TensorList g, at::TensorList c,
                                            at::TensorList W, at::TensorList U, at::TensorList pidx,
                                            at::IntArrayRef pool, at::IntArrayRef x_width, at::IntArrayRef T_in) {
  check_f32_cuda(x4, "x4");
  for (const at::Tensor* t : {&dloss, &h4, &g4, &c4, &Wt4, &Ut4}) check_f32_cuda(*t, "lstm_chain_head_bwd operand");
  TORCH_CHECK(x4.dim() == 3 && x4.is_contiguous(), "lstm_chain_head_bwd: x4 must be a contiguous [T4, Mp, Din]");
  const int T4 = (int)x4.size(0), Mp = (int)x4.size(1), Din = (int)x4.size(2), Dw = (int)Wt4.size(0);
  TORCH_CHECK(T4 >= 1 && T4 <= 16 && Din <= 64 && Dw >= 1 && Dw <= Din && Wt4.size(1) == 512 && Ut4.size(0) == 128 &&
                  Ut4.size(1) == 512, "lstm_chain_head_bwd: time4 shapes");
  TORCH_CHECK(dloss.numel() == 1, "lstm_chain_head_bwd: dloss must be a scalar");
  TORCH_CHECK(h4.numel() == (long)T4 * Mp * 128 && g4.numel() == (long)T4 * Mp * 128 * 4 && c4.numel() == (long)T4 * Mp * 128 * 2,
              "lstm_chain_head_bwd: time4 saved state shapes");
  TORCH_CHECK(pool.size() >= 1 && pool[0] == 3, "lstm_chain_head_bwd: the top chain stage must pool by 3");
  ChainBArgs A{};
  std::vector<at::Tensor> keep;
  c10::DeviceGuard guard(x4.device());
  auto opt = x4.options();
  at::Tensor so = at::empty({T4, Mp, Din}, opt.dtype(at::kLong));      // time4's dx granules
  auto res = chain_bwd_setup(A, keep, x4, g, c, W, U, pidx, pool, x_width, T_in, (Mp / 16 + 7) / 8 * 8);
  A.st[0].dh = nullptr;
  A.st[0].din = reinterpret_cast<const unsigned long long*>(so.data_ptr<int64_t>());
  ChainT4B& Q = A.t4;
  Q.on = 1;
  Q.h = h4.data_ptr<float>();
  Q.g = g4.data_ptr<float>();
  Q.c = c4.data_ptr<float>();
  TORCH_CHECK(pk.is_cuda() && pk.is_contiguous() && pk.nbytes() == (size_t)T4PK_ALL * 16,
              "lstm_chain_head_bwd: pk must be the forward's full fragment image");
  Q.pk = reinterpret_cast<const bf16x8_t*>(pk.data_ptr());
  if (hb.numel() > 0) {
    check_f32_cuda(hb, "lstm_chain_head_bwd hb");
    TORCH_CHECK(hb.numel() == (long)(Mp / 16) * 16 * 128 + (long)(Mp / 16) * ChainHeadRec<128>::PITCH,
                "lstm_chain_head_bwd: hb must be the forward's precomputed head backward");
    Q.hb = hb.data_ptr<float>();
  } else {
    Q.hb = nullptr;
  }
  at::Tensor dz4 = at::empty({T4 + 1, Mp, 512}, opt.dtype(at::kBFloat16));
  Q.dz = bf16_ptr(dz4);
  Q.sout = reinterpret_cast<unsigned long long*>(so.data_ptr<int64_t>());
  Q.T = T4;
  Q.Din = Din;
  Q.Dw = Dw;
  at::Tensor gpart;
  t4_head_bwd_args(Q.hd, head, y, mask, M, Mp, alpha1, alpha2, w0, w1, dloss, hgrads, gpart);
  hipLaunchKernelGGL(lstm_chain_bwd_kernel, dim3((A.ns + 1) * A.nt8), dim3(1024), 0, stream(), A);
  GQ_LAUNCH_CHECK();
  res.insert(res.begin(), dz4);
  return res;
}

static std::vector<at::Tensor> chain_bwd_setup(ChainBArgs& A, std::vector<at::Tensor>& keep, const at::Tensor& dh,
                                               at::TensorList g, at::TensorList c, at::TensorList W, at::TensorList U,
                                               at::TensorList pidx, at::IntArrayRef pool, at::IntArrayRef x_width,
                                               at::IntArrayRef T_in, int extra_blocks) {
  check_f32_cuda(dh, "dh");
  const int ns = (int)W.size();
  TORCH_CHECK(ns >= 1 && ns <= CHAIN_MAX && (int)U.size() == ns && (int)g.size() == ns && (int)c.size() == ns &&
                  (int)pidx.size() == ns && (int)pool.size() == ns && (int)x_width.size() == ns &&
                  (int)T_in.size() == ns, "lstm_chain_bwd: stage lists");
  TORCH_CHECK(dh.dim() == 3 && dh.is_contiguous(), "lstm_chain_bwd: dh must be a contiguous [Ts, Mp, H]");
  const int Mp = (int)dh.size(1);
  TORCH_CHECK(Mp % 16 == 0, "lstm_chain_bwd: Mp");
  const int ntiles = Mp / 16, nt8 = (ntiles + 7) / 8 * 8;
  TORCH_CHECK(ns * nt8 + extra_blocks <= chain_capacity(dh.get_device()), "lstm_chain_bwd: ", ns * nt8 + extra_blocks,
              " workgroups cannot all be resident on this device");
  c10::DeviceGuard guard(dh.device());
  auto opt = dh.options();
  A.ns = ns;
  A.ntiles = ntiles;
  A.nt8 = nt8;
  A.Mp = Mp;
  A.ctl = chain_ctl(dh.get_device());
  A.trace = chain_trace_buf(dh.get_device());
  chain_prof_clear(dh.get_device());
  std::vector<at::Tensor> dzs;
  at::Tensor dx, prev;
  for (int s = 0; s < ns; ++s) {
    const int H = (int)U[s].size(0), Dw = (int)W[s].size(0), T = (int)T_in[s], Din = (int)x_width[s];
    const int P = (int)pool[s];
    TORCH_CHECK(H == 16 || H == 32 || H == 64, "lstm_chain_bwd: hidden size ", H);
    TORCH_CHECK(Dw <= Din && Din <= 64 && Din % 4 == 0 && T >= 1 && T < 4096, "lstm_chain_bwd: stage ", s, " shape");
    for (const at::Tensor* t : {&c[s], &W[s], &U[s]}) check_f32_cuda(*t, "lstm_chain_bwd operand");
    check_gates_cuda(g[s]);
    TORCH_CHECK(g[s].numel() == (long)(T + 1) * Mp * H * 4 && c[s].numel() == (long)(T + 1) * Mp * H,
                "lstm_chain_bwd: saved state shapes");
    const int Ts = P > 0 ? T / P : T;
    if (s == 0) {
      TORCH_CHECK(dh.size(0) == Ts && dh.size(2) == H, "lstm_chain_bwd: dh shape");
    } else {
      TORCH_CHECK((int)x_width[s - 1] == H, "lstm_chain_bwd: stage ", s, " output width");
      TORCH_CHECK((int)T_in[s - 1] == Ts, "lstm_chain_bwd: lengths");
    }
    if (P > 0) {
      TORCH_CHECK(pidx[s].numel() == (long)Ts * Mp * H && pidx[s].scalar_type() == at::kByte,
                  "lstm_chain_bwd: argmax bytes");
    }
    ChainBStage& S = A.st[s];
    S.dh = s == 0 ? dh.data_ptr<float>() : nullptr;
    S.din = s == 0 ? nullptr : reinterpret_cast<const unsigned long long*>(prev.data_ptr<int64_t>());
    S.pidx = P > 0 ? pidx[s].data_ptr<uint8_t>() : nullptr;
    S.g = bf16_ptr(g[s]);
    S.c = c[s].data_ptr<float>();
    S.W = W[s].data_ptr<float>();
    S.U = U[s].data_ptr<float>();
    at::Tensor dz = at::empty({T + 1, Mp, 4 * H}, opt.dtype(at::kBFloat16));
    S.dz = bf16_ptr(dz);
    dzs.push_back(dz);
    const bool last = s + 1 == ns && ns > 1;     // (a single stage publishes: profiling)
    // producer-side un-pooling of the stage below's input pool (ChainBStage::uidx)
    S.uidx = nullptr;
    S.uP = 0;
    S.uT = 0;
    S.punp = s > 0 ? A.st[s - 1].uidx != nullptr : 0;
    int sT = T;                                  // rows of this stage's dx stream
    if (!last && s + 1 < ns && pool[s + 1] > 0) {
      static const bool on = [] {
        const char* e = std::getenv("GNNQC_CHAINB_PUNPOOL");
        return CHAINB_PUNPOOL && (e == nullptr || std::atoi(e) != 0);
      }();
      const int Hs = H, KXs = (Din + 31) / 32;
      const int stage_bytes = Hs >= 32 ? (KXs == 1 ? (Hs == 32 ? ChainBLdsSK<32, 1>::BYTES : ChainBLdsSK<64, 1>::BYTES)
                                                   : (Hs == 32 ? ChainBLdsSK<32, 2>::BYTES : ChainBLdsSK<64, 2>::BYTES))
                                       : (KXs == 1 ? ChainBLds<16, 1>::BYTES : ChainBLds<16, 2>::BYTES);
      const long ub = (long)T * 16 * Din;
      const int uT = (int)T_in[s + 1];
      // (the publisher wave un-pools: H = 64 stages fill the workgroup with compute waves and store dx themselves)
      if (on && 16 * H + 64 <= 1024 && (stage_bytes + 15) / 16 * 16 + ub <= CHAINB_LDS && (long)uT * Mp * Din * 8 < (1L << 31) &&
          T * (int)pool[s + 1] <= uT) {
        TORCH_CHECK(pidx[s + 1].numel() == (long)T * Mp * Din && pidx[s + 1].scalar_type() == at::kByte,
                    "lstm_chain_bwd: argmax bytes of stage ", s + 1);
        S.uidx = pidx[s + 1].data_ptr<uint8_t>();
        S.uP = (int)pool[s + 1];
        S.uT = uT;
        sT = uT;
      }
    }
    if (!last) {
      at::Tensor so = at::empty({sT + 1, Mp, Din}, opt.dtype(at::kLong));
      S.sout = reinterpret_cast<unsigned long long*>(so.data_ptr<int64_t>());
      S.dx = nullptr;
      keep.push_back(so);
      prev = so;
    } else {
      dx = at::empty({T + 1, Mp, Din}, opt);
      S.sout = nullptr;
      S.dx = dx.data_ptr<float>();
    }
    S.H = H;
    S.T = T;
    S.Din = Din;
    S.Dw = Dw;
    S.KX = (Din + 31) / 32;
    S.P = P;
    S.Ts = Ts;
    S.trace_mid = A.trace + 512;
    {
      long long* pb = chain_prof_buf(dh.get_device());
      S.prof = pb != nullptr ? pb + (size_t)s * CHAIN_PROF_STEPS * 8 : nullptr;
    }
  }
  dzs.push_back(dx.defined() ? dx.narrow(0, 0, (int)T_in[ns - 1]) : at::empty({0}, opt));
  return dzs;
}

// [epoch, finished, timeout flag, 0] of this device's chain control words (tests)
at::Tensor lstm_chain_status(const at::Tensor& like) {
  c10::DeviceGuard guard(like.device());
  int* p = chain_ctl(like.get_device());
  // [0] epoch, [1] finished workgroups, [2] spin timeout, [3] rejected steps, .., [9] consumer re-polls
  at::Tensor o = at::empty({12}, like.options().dtype(at::kInt));
  TORCH_CHECK(hipMemcpyAsync(o.data_ptr<int>(), p, 12 * sizeof(int), hipMemcpyDeviceToDevice, stream()) == hipSuccess,
              "lstm_chain_status");
  return o;
}

// [blocks, 2] start / end timestamps (s_memrealtime ticks) of the last chain launch (profiling)
at::Tensor lstm_chain_trace(const at::Tensor& like) {
  c10::DeviceGuard guard(like.device());
  long long* p = chain_trace_buf(like.get_device());
  at::Tensor o = at::empty({3 * 256}, like.options().dtype(at::kLong));
  TORCH_CHECK(hipMemcpyAsync(o.data_ptr<int64_t>(), p, o.numel() * sizeof(long long), hipMemcpyDeviceToDevice,
                             stream()) == hipSuccess, "lstm_chain_trace");
  return o;
}

}  // namespace gq

TORCH_LIBRARY_IMPL(gnnqc, CUDA, m) {
  m.impl("lstm_chain_fwd", &gq::lstm_chain_fwd);
  m.impl("lstm_chain_fwd_pack", &gq::lstm_chain_fwd_pack);
  m.impl("lstm_chain_head_fwd", &gq::lstm_chain_head_fwd);
  m.impl("lstm_chain_status", &gq::lstm_chain_status);
  m.impl("lstm_chain_capacity", &gq::lstm_chain_capacity);
  m.impl("lstm_chain_ctl", &gq::lstm_chain_ctl);
  m.impl("lstm_chain_trace", &gq::lstm_chain_trace);
  m.impl("lstm_chain_prof", &gq::lstm_chain_prof);
  m.impl("lstm_chain_bwd", &gq::lstm_chain_bwd);
  m.impl("lstm_chain_head_bwd", &gq::lstm_chain_head_bwd);
}
