// One whole LearnedSimulator.predict_positions (learned_simulator.py:413-438)
// in ONE launch, for graphs of up to 8,192 particles at hidden 64 and
// nmlp_layers 1 (the C1 headline: 2,000 particles, r = 15, L = 5; the Taylor
// bars' 4,800 / 6,400 / 8,000 with two 16-item node sub-tiles per workgroup):
//   radius graph (torch_cluster.radius via radius_graph, :116-117)
//   -> Encoder (graph_network.py:86-96, features :231-316)
//   -> L x InteractionNetwork (graph_network.py:150-222, edge-latent doubling)
//   -> Decoder (:321-333) -> Euler integrator (learned_simulator.py:381-411)
//   (+ the rollout window shift, evaluate.py:136-139).
//
// Why one launch.  At C1 the whole step is ~7 GFLOP of fp32 MFMA work, 45 us
// of a 256-CU chip's time at the 1/4 MFMA occupancy one wave per SIMD
// reaches, and the per-layer launch sequence paid, per layer, a kernel
// boundary, a grid-wide ramp, and a weight staging pass that no other work
// overlapped.  Here workgroup t owns receivers
// [t*nt, t*nt + nt) for the whole step and stays resident (grid <= 256, one
// workgroup per CU by its LDS size).  Layer k of tile t needs only layer k's
// node halves u_k, v_k of the tiles its senders live in, so instead of a grid
// barrier every tile publishes a per-tile phase counter after writing its
// rows and every consumer waits on the counters of ITS sender tiles only
// (dataflow: a slow tile delays its dependents, not the chip).  While a tile
// waits, the next layer's weights are already in flight.
//
// Hand-off protocol (cdna_hip_programming.md Guideline 16, MI355X_MICROARCH.md
// "visibility", table row 1: one workgroup per CU, hipMalloc memory): every
// handed-off byte (u_k / v_k rows) is stored write-through (sc1) and drained
// (s_waitcnt vmcnt(0) in every storing wave, then a workgroup barrier); ONE
// lane then stores the tile's counter with an agent-scope atomic (sc1 store).
// The consumer's wave 0 polls the counters relaxed (sc1 loads); the other
// waves pass a workgroup barrier after the match; EVERY load of handed-off
// rows is an sc1 buffer load (no L1), so no acquire fence is needed.  Each
// layer's u/v go to their own buffers (written once per step), so there is
// no write-after-read hazard between tiles at different layers; x and the
// edge latent e0 of a tile's own edges never leave its LDS.  Counters are
// zeroed by the driver at the start of every call; phase p of step s is
// epoch0 + p + 1 with epoch0 = s (L + 1).  Every spin is bounded: a tile that
// times out records it in an error word and finishes (results are then
// garbage): sgnn_step_check returns SGNN_ERR_STEP_TIMEOUT for that call, and
// the Python wrappers raise SgnnError.
#include <map>
#include <mutex>
#include <tuple>
#include <type_traits>

#include "common.h"
#include "fwd16.h"
#include "sgnn_internal.h"
#include "step16.h"

#include "fwd16_dev.h"

namespace {

using sgnn::Step16Args;
using sgnn::Lay16;

typedef __attribute__((address_space(1))) uint32_t gu32;

constexpr int kPollLimit = 1 << 21;   // ~1 s of polling: a hang becomes an error word
constexpr int kMaxGrid = sgnn::kStep16MaxGrid;
using sgnn::kStepFlagErr;
using sgnn::kStepFlagStride;

SGNN_DEV f32x4 ld4_sc1(__amdgpu_buffer_rsrc_t rs, int voff) {
  typedef int i32x4 __attribute__((ext_vector_type(4)));
  return __builtin_bit_cast(f32x4, __builtin_bit_cast(i32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, voff, 0, 16)));
}
SGNN_DEV void st4_sc1(__amdgpu_buffer_rsrc_t rs, int voff, f32x4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), rs, voff, 0, 16);
}

// LDS carve (floats), shared with the host's size query.  A tile of nt <= 16 receivers is one 16-item
// node sub-tile, nt <= 32 two (NSUB).
constexpr int kMaxNT = sgnn::kStep16MaxNT;
struct Carve {
  int sw0, sw1, svec, sxw, sxv, scratch, xs, dbuf, region, ints, total;  // float offsets / count
  int region_floats;
  int list_cap;  // radius phase: candidate slots (4 waves x Q, Q = round64(n / 4) at most)
};
SGNN_HOST_DEV inline Carve carve(int n, int dim, int nt, int cap, bool e0g) {
  Carve c{};
  const int nsub = (nt + 15) / 16;
  int o = 0;
  c.sw0 = o; o += H * LDX;        // edge W1e (x 2^k), LDS image [H][LDX]
  c.sw1 = o; o += H * LDX;        // edge W2
  c.svec = o; o += 4 * H;         // edge b2, gamma, beta
  c.sxw = o; o += H * LDX;        // Encoder.edge_fn W2
  c.sxv = o; o += 4 * H;          // Encoder.edge_fn b1, b2, gamma, beta
  c.scratch = o; o += 4 * 16 * nsub * LDX;  // per-wave receiver sums; node-phase exchange buffers
  c.xs = o; o += 16 * nsub * LDX;  // x rows of the tile's nodes (resident for the step)
  c.dbuf = o; o += 2 * KQ * 64 * 4;  // donated pre-wait products (EdgePhase::plan)
  // the radius phase's candidate list ([dim][list_cap] positions + [list_cap] ids) overlays everything
  // before `ints` (nothing else there is live yet); the region after dbuf holds the e0 rows (unless in HBM)
  c.list_cap = 4 * ((((n + 3) / 4) + 63) & ~63);
  const int e0f = e0g ? 0 : nt * cap * LDX, listf = (dim + 1) * c.list_cap - o;
  c.region_floats = e0f > listf ? e0f : (listf > 0 ? listf : 0);
  c.region = o; o += (c.region_floats + 3) & ~3;
  // lsend, lrecv [round16(nt*cap)] each, nbr [nt*cap]; deg [32]; pre [36]; mask [8]; kw [4][64]; deps [256] +
  // count; example offsets [kStep16MaxEx + 1]; receiver positions [3][32]; box [8]; segment counts [4]
  c.ints = o;
  o += 2 * ((nt * cap + 15) & ~15) + nt * cap + kMaxNT + kMaxNT + 4 + 8 + 4 * 64 + sgnn::kStep16MaxGrid + 4 +
       sgnn::kStep16MaxEx + 4 + 3 * kMaxNT + 8 + 4;
  c.total = (o + 3) & ~3;
  return c;
}

// Experiment builds (-DSGNN_PROBE, tools/exp_probe_step16.py): per-wave s_memtime marks at the phase
// boundaries, [workgroup][wave][64] into the buffer set by sgnn_set_probe16.  Slots: 0 start, 1 radius done,
// 2 encoder done; layer k < 5 at 3 + 8 k + (0 start, 1 node weights requested, 2 published, 3 pre-wait done,
// 4 wait done, 5 edge phase done, 6 node tail done, 7 end); layer 1's halves at 48 + (0 gathers issued,
// 1.. after each), its node phase at 52 (sums read), 53 (first Linear); 56 positions staged, 58 weights in
// LDS, 59 tile CSR built.
#ifdef SGNN_PROBE
__device__ uint64_t* g_probe16;
SGNN_DEV void mark(int slot) {
  const uint64_t t = __builtin_amdgcn_s_memtime();
  if (g_probe16 && lane_id() == 0 && slot >= 0 && slot < 64)
    g_probe16[((int64_t)blockIdx.x * kWaves16 + wave_id()) * 64 + slot] = t;
}
#else
SGNN_DEV void mark(int) {}
#endif

// Hand-off check build (-DSGNN_HANDOFF_CHECK, tools/exp_handoff.py).  Buffer g_hc
// (sgnn_set_handoff_check): [0] hash mismatches, [1] tag mismatches, [2] printed lines, [3] final checks
// run, [4..15] spare; then tags [L][n][4]: for every node-half row it stores, the producing wave b
// writes the phase its rows are published with (epoch0 + buffer + 1, sc1, drained with the rows);
// then hashes [grid][L][kHcHalves][64][2]: per gathered half and lane, a hash of the u and of the v
// row words as the consumer used them.  Consumers compare the tags of every row they gather (sender
// and receiver) with the phase they polled for; at the end of the kernel every tile publishes a final
// phase, waits for its sender tiles to reach it, re-gathers every half of every layer and compares the
// hashes: a row read before its producer's stores had landed differs from the settled value.
#ifdef SGNN_HANDOFF_CHECK
__device__ uint32_t* g_hc;
constexpr int kHcHalves = sgnn::kStep16MaxNT * sgnn::kStep16MaxCap / 16;
SGNN_DEV uint32_t* hc_tags() { return g_hc + 16; }
SGNN_DEV uint32_t* hc_hash(const Step16Args& a) { return g_hc + 16 + (int64_t)a.L * a.n * 4; }
SGNN_DEV uint32_t hc_mix(uint32_t h, f32x4 v) {
#pragma unroll
  for (int c = 0; c < 4; ++c) h = (h ^ __builtin_bit_cast(uint32_t, v[c])) * 16777619u;
  return h;
}
// the reports are out-of-line calls: printf inlined into the unrolled layer code made the check build's
// compile take 15+ minutes
__attribute__((noinline)) __device__ void hc_report_tag(int wg, int k, int b, int l, int e, int r, int rt, uint32_t r0,
                                                       uint32_t r1, uint32_t r2, uint32_t r3, int s, int st, uint32_t s0,
                                                       uint32_t s1, uint32_t s2, uint32_t s3, uint32_t ep) {
  atomicAdd(g_hc + 1, 1u);
  if (atomicAdd(g_hc + 2, 1u) < 48u)
    printf("SGNN-HANDOFF tag: wg %d layer %d wave %d lane %d edge %d recv %d (tile %d) tags %u %u %u %u "
           "send %d (tile %d) tags %u %u %u %u, polled for %u\n", wg, k, b, l, e, r, rt, r0, r1, r2, r3, s, st, s0,
           s1, s2, s3, ep);
}
__attribute__((noinline)) __device__ void hc_report_stale(int wg, int k, int b, int l, int e, int Et, int r, int rt,
                                                         int bu, int s, int st, int bv) {
  atomicAdd(g_hc, 1u);
  if (atomicAdd(g_hc + 2, 1u) < 48u)
    printf("SGNN-HANDOFF stale: wg %d layer %d wave %d lane %d edge %d (of %d) recv %d (tile %d)%s send %d "
           "(tile %d)%s\n", wg, k, b, l, e, Et, r, rt, bu ? " STALE" : "", s, st, bv ? " STALE" : "");
}
#endif

// Per-tile counters of the sender tiles `deps` (up to 256, all requested at once).  Every wave polls for
// itself (no workgroup barrier after the match): `issue` requests the counters early -- before the
// wave's last pre-wait product, so their round trip overlaps it -- and `wait` checks them and polls
// on until they match.
struct TilePoll {
  uint32_t v[kMaxGrid / 64], w[kMaxGrid / 64];
  SGNN_DEV static void read(uint32_t (&x)[kMaxGrid / 64], const int32_t* deps, int ndeps, const uint32_t* flags,
                            uint32_t epoch, int lane) {
#pragma unroll
    for (int q = 0; q < kMaxGrid / 64; ++q)
      x[q] = lane + 64 * q < ndeps
                 ? __hip_atomic_load((const gu32*)(flags + deps[lane + 64 * q] * kStepFlagStride), __ATOMIC_RELAXED,
                                     __HIP_MEMORY_SCOPE_AGENT)
                 : epoch;
  }
  SGNN_DEV static bool ok(const uint32_t (&x)[kMaxGrid / 64], uint32_t epoch) {
    bool r = true;
#pragma unroll
    for (int q = 0; q < kMaxGrid / 64; ++q) r = r && x[q] >= epoch;
    return __all(r);
  }
  // two early reads, one product apart: the later one usually sees counters the earlier missed
  SGNN_DEV void issue(const int32_t* deps, int ndeps, const uint32_t* flags, uint32_t epoch, int lane) {
    read(v, deps, ndeps, flags, epoch, lane);
  }
  SGNN_DEV void issue2(const int32_t* deps, int ndeps, const uint32_t* flags, uint32_t epoch, int lane) {
    read(w, deps, ndeps, flags, epoch, lane);
  }
  SGNN_DEV void wait(const int32_t* deps, int ndeps, uint32_t* flags, uint32_t epoch, int lane, int limit) {
    if (limit < 0 && lane == 0)  // test hook (sgnn_step_ws.step_poll_limit < 0): the error path
      __hip_atomic_store((gu32*)(flags + kStepFlagErr), epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (ok(v, epoch) || ok(w, epoch)) return;
    // two polls in flight: each check waits only for the older one, so the counters are sampled twice
    // per round trip
    read(v, deps, ndeps, flags, epoch, lane);
    for (int it = 0;; it += 2) {
      read(w, deps, ndeps, flags, epoch, lane);
      if (ok(v, epoch)) break;
      read(v, deps, ndeps, flags, epoch, lane);
      if (ok(w, epoch)) break;
      if (it >= limit) {
        if (lane == 0)
          __hip_atomic_store((gu32*)(flags + kStepFlagErr), epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
  }
};

// Every storing wave drains its sc1 stores, then one lane publishes the phase.  skew > 0 (test knob,
// sgnn_step_ws.step_skew): that lane first sleeps 0..7 x skew rounds of s_sleep 16 (~0.4 us each), a
// tile- and phase-dependent count, so tiles run the hand-off under uneven load.
SGNN_DEV void publish(uint32_t* flags, int tile, uint32_t epoch, int skew) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    if (skew > 0) {
      const uint32_t h = ((uint32_t)tile * 2654435761u) ^ (epoch * 40503u);
      const int rounds = (int)((h >> 28) & 7u) * skew;
      for (int r = 0; r < rounds; ++r) __builtin_amdgcn_s_sleep(16);
    }
    __hip_atomic_store((gu32*)(flags + tile * kStepFlagStride), epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// Sum over the lanes j, j + 16, j + 32, j + 48 (the column groups holding one item's units): two
// cross-row swaps on the VALU instead of two LDS permute round trips.
SGNN_DEV float xg_sum(float v) {
  // v_permlane32_swap / v_permlane16_swap exchange lanes between two registers (both written): with
  // both holding v, their sum is the sum over lanes l and l ^ 32, then l and l ^ 16.  Inline: this
  // compiler's builtins for them return the first register twice.  s_nop: VALU -> permlane hazards.
  float p = v, q = v;
  asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1\n\ts_nop 1" : "+v"(p), "+v"(q));
  v = p + q;
  p = v;
  q = v;
  asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1\n\ts_nop 1" : "+v"(p), "+v"(q));
  return p + q;
}
// LayerNorm statistics of full rows held as in ln_stats (two-pass, biased variance, eps 1e-5)
SGNN_DEV void ln_stats_x(const f32x4 (&r)[KQ], float& mean, float& rstd) {
  f32x4 p = (r[0] + r[1]) + (r[2] + r[3]);
  mean = xg_sum((p[0] + p[1]) + (p[2] + p[3])) * (1.0f / H);
  f32x4 v = zero4();
#pragma unroll
  for (int q = 0; q < KQ; ++q) {
    const f32x4 d = r[q] - mean;
    v += d * d;
  }
  rstd = __builtin_amdgcn_rsqf(xg_sum((v[0] + v[1]) + (v[2] + v[3])) * (1.0f / H) + 1e-5f);
}

// Node update of the tile's NS 16-item sub-tiles (item rows 16 s + j; `cnt` valid rows in all) from the
// first Linear's post-ReLU outputs h[s]: last Linear, LayerNorm, + residual xo -> x (LDS rows xs), then u, v
// of the next layer (mode 0, sc1 rows) or decoder + integrator + window shift (mode 1).  Same arithmetic
// as fwd16.hip node_tail.  The kernel runs it once per 16-item sub-tile (NS = 1); NS > 1 would take the
// sub-tiles through each exchange together (sub-tile s's exchange buffers: scratch rows 48 s .. 48 s + 47),
// the round-5 experiment DESIGN.md section 8.1 records and that is not shipped.
template <int NS>
SGNN_DEV void xchg_n(float* buf, int sstride, int j, int ucol, int g, const f32x4 (&v)[NS], f32x4 (&out)[NS][KQ]) {
#pragma unroll
  for (int s = 0; s < NS; ++s) st4(buf + s * sstride + j * LDX + ucol, v[s]);
  __syncthreads();
#pragma unroll
  for (int s = 0; s < NS; ++s)
#pragma unroll
    for (int q = 0; q < KQ; ++q) out[s][q] = ld4(buf + s * sstride + j * LDX + 16 * q + 4 * g);
}

template <int MODE, int NS>
SGNN_DEV void step_tail(const Step16Args& a, const NodeW<2, MODE>& W, float* scratch, float* xs, int64_t i0, int cnt,
                        const f32x4 (&h)[NS], const f32x4 (&xo)[NS], int b, int j, int g, __amdgpu_buffer_rsrc_t ru,
                        __amdgpu_buffer_rsrc_t rv, int kk) {
  (void)kk;  // the node-half buffer written (mode 0): the check build's tags
  constexpr int SB = 48 * LDX;
  const int ucol = 16 * b + 4 * g;
  f32x4 hr[NS][KQ], yr[NS][KQ], xnr[NS][KQ], y[NS], xn[NS];
  xchg_n<NS>(scratch, SB, j, ucol, g, h, hr);
#pragma unroll
  for (int s = 0; s < NS; ++s) y[s] = mm(W.vb2, W.w2, hr[s]);
  xchg_n<NS>(scratch + 16 * LDX, SB, j, ucol, g, y, yr);
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    float mean, rstd;
    ln_stats_x(yr[s], mean, rstd);
#pragma unroll
    for (int c = 0; c < 4; ++c) xn[s][c] = (y[s][c] - mean) * rstd * W.vg[c] + W.vbb[c] + xo[s][c];  // LN + :176
  }
  xchg_n<NS>(xs, 16 * LDX, j, ucol, g, xn, xnr);
  if constexpr (MODE == 0) {
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const int64_t i = i0 + 16 * s + j;
      const bool valid = 16 * s + j < cnt;
      const f32x4 u = mm(W.vba, W.wa, xnr[s]);
      const f32x4 v = mm(zero4(), W.wb, xnr[s]);
      const int off = valid ? (int)i * (H * 4) + ucol * 4 : kBufDrop;
      st4_sc1(ru, off, u);
      st4_sc1(rv, off, v);
#ifdef SGNN_HANDOFF_CHECK
      if (g_hc && valid && g == 0)
        __hip_atomic_store((gu32*)(hc_tags() + ((int64_t)kk * a.n + i) * 4 + b), a.epoch0 + (uint32_t)kk + 1u,
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#endif
    }
  } else {
    f32x4 hd[NS], hdr[NS][KQ];
#pragma unroll
    for (int s = 0; s < NS; ++s) hd[s] = relu4(mm(W.vba, W.wa, xnr[s]));
    xchg_n<NS>(scratch + 2 * 16 * LDX, SB, j, ucol, g, hd, hdr);
    const int D = a.dim;
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const int64_t i = i0 + 16 * s + j;
      const bool valid = 16 * s + j < cnt;
      if (b == 0) {
        const f32x4 o = mm(W.vbo, W.wb, hdr[s]);  // lanes g == 0 hold outputs 0..3
        if (valid && g == 0) {
#pragma unroll
          for (int c = 0; c < 4; ++c)
            if (c <= D) a.pred[i * (D + 1) + c] = comp(o, c);
          const float* p = a.pos_seq + i * a.T * D;  // learned_simulator.py:398-411
#pragma unroll
          for (int c = 0; c < 3; ++c) {
            if (c >= D) break;
            const float acc = __fadd_rn(__fmul_rn(comp(o, c), a.acc_std[c]), a.acc_mean[c]);
            const float pT = p[(a.T - 1) * D + c], pT1 = p[(a.T - 2) * D + c];
            const float np = __fadd_rn(pT, __fadd_rn(__fsub_rn(pT, pT1), acc));
            a.next_pos[i * D + c] = np;
            if (a.window_out) a.window_out[(i * a.T + a.T - 1) * D + c] = np;
          }
        }
      } else if (b == 1 && g == 0 && valid && a.window_out) {  // evaluate.py:136-139
        const float* p = a.pos_seq + i * a.T * D;
        float* w = a.window_out + i * a.T * D;
        for (int k = 0; k < (a.T - 1) * D; ++k) w[k] = p[k + D];
      }
    }
  }
}

// Sum of v over the 16 lanes of each row (DPP: xor 1, xor 2, half mirror, mirror); every lane of the
// row ends with the same value.
template <int C>
SGNN_DEV float dppf(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), C, 0xf, 0xf, false));
}
SGNN_DEV float row_sum16(float v) {
  v += dppf<0xB1>(v);
  v += dppf<0x4E>(v);
  v += dppf<0x141>(v);
  v += dppf<0x140>(v);
  return v;
}

// Edge bias b2 / gamma / beta of the lane's units 16 t + j (the swapped-operand layout below).
struct EdgeVec {
  float b2[KQ], ga[KQ], be[KQ];
};

// The LayerNorm + receiver sums of one half's y in four parts: 0 means, 1 deviations + variances,
// 2 scales + incidence + messages, 3 the 16 aggregation MFMAs.  (Interleaving them with the next
// half's MFMAs gains nothing: f32 MFMA occupies most of the SIMD's VALU, tools/exp/mfma_valu_overlap.hip.)
// With two node sub-tiles (NSUB 2: receivers i0 .. i0 + 31) the incidence has a block per sub-tile, and a
// half runs the MFMAs of the blocks its receivers hit (one, or two for the half that straddles).
template <int NSUB>
struct LnAgg {
  f32x4 d[KQ], mu, var;
  float sb[NSUB][4];
  bool hit[NSUB];
  SGNN_DEV void part(int p, const f32x4 (&y)[KQ], f32x4 (&agg)[NSUB][KQ], const EdgeVec& ev, const int32_t* lrecv,
                     int hs, int Et, int i0, int j, int g) {
    if (p == 0) {  // two-pass statistics per edge 4 g + c (torch: biased variance, eps 1e-5)
      mu = (y[0] + y[1]) + (y[2] + y[3]);
#pragma unroll
      for (int c = 0; c < 4; ++c) mu[c] = row_sum16(mu[c]) * (1.0f / H);
    } else if (p == 1) {
      var = zero4();
#pragma unroll
      for (int t = 0; t < KQ; ++t) {
        d[t] = y[t] - mu;
        var += d[t] * d[t];
      }
#pragma unroll
      for (int c = 0; c < 4; ++c) var[c] = row_sum16(var[c]);
    } else if (p == 2) {
      f32x4 rs;
#pragma unroll
      for (int c = 0; c < 4; ++c) rs[c] = __builtin_amdgcn_rsqf(var[c] * (1.0f / H) + 1e-5f);
      // B: lane (col j, k = g) supplies S[edge 4 g + s][recv i0 + j] for step s = 0..3
      typedef int i32x4 __attribute__((ext_vector_type(4)));
      const i32x4 rv = *reinterpret_cast<const i32x4*>(lrecv + hs + 4 * g);
#pragma unroll
      for (int s = 0; s < NSUB; ++s) {
#pragma unroll
        for (int s2 = 0; s2 < 4; ++s2) sb[s][s2] = (hs + 4 * g + s2 < Et && rv[s2] - i0 - 16 * s == j) ? 1.0f : 0.0f;
        if constexpr (NSUB > 1) hit[s] = __ballot(sb[s][0] + sb[s][1] + sb[s][2] + sb[s][3] != 0.0f) != 0ull;
      }
#pragma unroll
      for (int t = 0; t < KQ; ++t) d[t] = d[t] * rs * ev.ga[t] + ev.be[t];  // m (A: lane (unit j, k = g))
    } else {
#pragma unroll
      for (int s = 0; s < NSUB; ++s) {
        if (NSUB > 1 && !hit[s]) continue;
#pragma unroll
        for (int s2 = 0; s2 < 4; ++s2)  // the four accumulators in turn: no dependent back-to-back MFMAs
#pragma unroll
          for (int t = 0; t < KQ; ++t) agg[s][t] = mfma16(d[t][s2], sb[s][s2], agg[s][t]);
      }
    }
  }
};

// The last Linear of the edge MLP, its LayerNorm and the receiver sums of one
// 16-edge half, with no transposition through LDS.  The Linear runs with its
// operands swapped (mm_full<true>): lane (j, g) receives y[unit 16 t + j][edge
// 4 g + c], so each edge's LayerNorm statistics (graph_network.py:197-198) are
// an in-lane sum over t plus a 16-lane row sum, and the LayerNorm'd messages m
// are already the A operand of
//   agg[unit][recv] += m[unit][edge] S[edge][recv],   S = the half's 0/1 receiver incidence
// (16 v_mfma_f32_16x16x4_f32, B = S built from the half's receiver ids): the
// segmented sum runs on the matrix cores and the wave's aggregates stay in
// registers across its halves.  Receiver r of the tile is column r - i0 (< 16);
// padding edges have S = 0 (their rows are clamped copies, finite).
// lin2: ReLU + the Linear (y, before the LayerNorm); the LnAgg parts finish a half.
SGNN_DEV void lin2_init(const f32x4 (&acc)[KQ], f32x4 (&x)[KQ], f32x4 (&y)[KQ], const EdgeVec& ev) {
#pragma unroll
  for (int t = 0; t < KQ; ++t) {
    x[t] = relu4(acc[t]);
    y[t] = f32x4{ev.b2[t], ev.b2[t], ev.b2[t], ev.b2[t]};
  }
}

// halves per wave whose W1e e0 product runs before the wait (2 / 4 measured: C1 r = 15 +13 % / -1 %,
// t8000 +4 % / 0)
constexpr int kPre = 3;
// The tile publishes the node halves its previous stage stored after this many of those products: the
// drain of the write-through stores overlaps them (after the second / third product: C1 r = 15 +11 / +13 us)
constexpr int kPubAt = 1;
static_assert(kPubAt >= 0 && kPubAt <= kPre, "publish point within the pre-wait");

// The edge MLP of a layer, split around the wait for the sender tiles.  Wave b
// takes the 16-edge halves b, b + 4, ... of the compacted tile CSR.  The first
// Linear on cat[x_i, x_j, e] is u[recv] + v[send] + 2^k W1_e e0 (graph_network.py:
// 197): its e0 part needs no other tile's data, so `prewait` forms it for the
// wave's first kPre halves BEFORE the wait (and, FIRST, runs the edge features +
// Encoder.edge_fn for every half and keeps the e0 rows), and `postwait` adds the
// gathered u / v rows, runs the last Linear + LayerNorm and the receiver sums
// (half_agg, on the matrix cores).
template <int NSUB>
struct EdgePhase {
  const Step16Args& a;
  const float *sw0, *sw1, *svec, *sxw, *sxv;
  float *sums, *e0l;
  const int32_t *lsend, *lrecv;
  int Et, i0, b, j, g, l;
  f32x4 pre[kPre][KQ];
  bool e0_hbm = false;        // e0l is the tile's HBM block (E0G), not LDS
  int hc_k = 0, hc_slot = 0;  // check build: the layer, and the workgroup's slot in the hash table
  uint32_t hc_ep = 0;         // check build: the phase the gathered rows were polled for

  // Encoder.edge_fn of one half from its endpoints' positions -> x (e0), rows kept in e0l
  SGNN_DEV void encode(f32x4 (&x)[KQ], const float (&xw1)[KQ], const float (&ps)[3], const float (&pr)[3], int hs,
                       bool ev) const {
    // edge features (p_s - p_r) / R and their norm (learned_simulator.py:299-312)
    float f[4] = {0.0f, 0.0f, 0.0f, 0.0f}, ss = 0.0f;
#pragma unroll
    for (int c = 0; c < 3; ++c)
      if (c < a.dim) {
        const float dd = __fdiv_rn(__fsub_rn(ps[c], pr[c]), a.radius);
        f[c] = dd;
        ss = __fadd_rn(ss, __fmul_rn(dd, dd));
      }
    const float nrm = sqrtf(ss);
    if (a.dim == 1) f[1] = nrm; else if (a.dim == 2) f[2] = nrm; else f[3] = nrm;
    const float fg = g == 0 ? f[0] : g == 1 ? f[1] : g == 2 ? f[2] : f[3];
    // Linear(dim + 1, H) -> ReLU -> Linear(H, H) -> LayerNorm (graph_network.py:92-96)
    f32x4 hx[KQ], y[KQ];
#pragma unroll
    for (int t = 0; t < KQ; ++t) {
      hx[t] = relu4(mfma16(xw1[t], fg, ld4(sxv + 16 * t + 4 * g)));
      y[t] = ld4(sxv + H + 16 * t + 4 * g);
    }
    mm_full(y, sxw, hx, j, g);
    float mu, rs;
    ln_stats_x(y, mu, rs);
    const int e = hs + j;
#pragma unroll
    for (int t = 0; t < KQ; ++t) {
      const f32x4 ga = ld4(sxv + 2 * H + 16 * t + 4 * g), be = ld4(sxv + 3 * H + 16 * t + 4 * g);
#pragma unroll
      for (int c = 0; c < 4; ++c) x[t][c] = (y[t][c] - mu) * rs * ga[c] + be[c];
      if (ev) st4(e0l + e * LDX + 16 * t + 4 * g, x[t]);
    }
  }

  SGNN_DEV void ld_e0(f32x4 (&x)[KQ], int hs) const {
    const int e = hs + j, ec = e < Et ? e : Et - 1;
#pragma unroll
    for (int q = 0; q < KQ; ++q) x[q] = ld4(e0l + ec * LDX + 16 * q + 4 * g);
  }

  // before the wait: (FIRST) e0 of every half; W1e e0 of the first kPre halves
  // Balance of the pre-wait products: with NH halves in the tile, F = NH / 4 full rounds and r = NH % 4
  // in {1, 2} (and F < kPre), waves b < r own F + 1 halves and the others F.  Then wave r + i (i < r)
  // forms the W1e e0 product of wave i's last half (its first product, into dbuf before the publish
  // barrier; FIRST: it also encodes that half's e0 rows), so every wave runs at most F + 1 products
  // before the wait and the owner reads the donated one after it.
  int F = 0, r = 0;
  bool donor = false, owner_d = false, donates = false;
  int NH = 0;   // the tile's 16-edge halves
  int hd = -1;
  float* dbuf = nullptr;   // [2][KQ][64] f32x4 donated products
  SGNN_DEV void plan(float* dbuf_) {
    NH = (Et + 15) / 16;
    F = NH / 4;
    r = NH % 4;
    const bool don = (r == 1 || r == 2) && F + 1 <= kPre;
    donates = don;  // (workgroup-uniform: from the tile's half count)
    owner_d = don && b < r;
    donor = don && b >= r && b - r < r;
    hd = donor ? 16 * (kWaves16 * F + (b - r)) : -1;
    dbuf = dbuf_;
  }
  // the wave's k-th product / encode item: the donated half first (donor), then its own halves;
  // -1 skips an own half whose product runs on the donor, -2 ends the list
  SGNN_DEV int item_half(int k) const {
    int m = k;
    if (donor) {
      if (k == 0) return hd;
      m = k - 1;
    }
    const int hs = 16 * b + 16 * kWaves16 * m;
    if (hs >= Et) return -2;
    if (owner_d && m == F) return -1;
    return hs;
  }

  // hook(s) runs before the wave's product slot s (s = 0 .. kPre - 1) and hook(kPre) after the last: the
  // caller publishes and requests the node weights there, between the products.  Slot s holds item s;
  // its product goes to pre[s] (own half m = s), or (DONOR) slot 0's to dbuf and slot s's (own half
  // m = s - 1) to pre[s - 1].
  template <bool FIRST, bool DONOR, class Hook>
  SGNN_DEV void prewait(const float (&xw1)[KQ], Hook&& hook) {
    const float* pos = a.pos_last ? a.pos_last : a.pos_seq + (int64_t)(a.T - 1) * a.dim;
    const int pstride = a.pos_last ? a.dim : a.T * a.dim;
    float ps_n[3] = {0.0f, 0.0f, 0.0f}, pr_n[3] = {0.0f, 0.0f, 0.0f};
    auto load_pos = [&](int hs) {
      const int e = hs + j, ec = e < Et ? e : Et - 1;
      const int rr = lrecv[ec], ss = lsend[ec];
#pragma unroll
      for (int c = 0; c < 3; ++c)
        if (c < a.dim) {
          ps_n[c] = pos[(int64_t)ss * pstride + c];
          pr_n[c] = pos[(int64_t)rr * pstride + c];
        }
    };
    auto next_item = [&](int k) {  // the next item to encode from k on (-2: none)
      int h = item_half(k);
      while (h == -1) h = item_half(++k);
      return h;
    };
    auto encode_item = [&](f32x4 (&x)[KQ], int hs, int k) {
      float ps[3], pr[3];
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        ps[c] = ps_n[c];
        pr[c] = pr_n[c];
      }
      const int hn = next_item(k + 1);
      if (hn >= 0) load_pos(hn);
      encode(x, xw1, ps, pr, hs, hs + j < Et);
    };
    if (FIRST) {
      const int h0 = next_item(0);
      if (h0 >= 0) load_pos(h0);
    }
    // e0 rows in HBM (two node sub-tiles): the next item's rows are requested before this item's product,
    // so their L2 round trip hides under its MFMAs (LDS rows need no lookahead)
    f32x4 xn[KQ];
    if constexpr (!FIRST) {
      if (e0_hbm) {
        const int h0 = next_item(0);
        if (h0 >= 0) ld_e0(xn, h0);
      }
    }
#pragma unroll
    for (int sl = 0; sl < kPre; ++sl) {
      hook(sl);
      const int hs = item_half(sl);
      if (hs < 0) continue;
      f32x4 x[KQ];
      if constexpr (FIRST) {
        encode_item(x, hs, sl);
      } else if (e0_hbm) {
#pragma unroll
        for (int q = 0; q < KQ; ++q) x[q] = xn[q];
        int hn = -2;
#pragma unroll
        for (int k = sl + 1; k < kPre; ++k) {
          const int h = item_half(k);
          if (h >= 0) {
            hn = h;
            break;
          }
          if (h == -2) break;
        }
        if (hn >= 0) ld_e0(xn, hn);
      } else {
        ld_e0(x, hs);
      }
      constexpr int kLast = kPre - 1;
      f32x4(&dst)[KQ] = pre[DONOR ? (sl == 0 ? kLast : sl - 1) : sl];
#pragma unroll
      for (int t = 0; t < KQ; ++t) dst[t] = zero4();
      mm_full(dst, sw0, x, j, g);
      if (DONOR && sl == 0) {
#pragma unroll
        for (int t = 0; t < KQ; ++t) st4(dbuf + (((b - r) * KQ + t) * 64 + l) * 4, dst[t]);
      }
    }
    hook(kPre);
    if constexpr (FIRST) {  // the rest of the items: e0 rows only
      for (int k = kPre;; ++k) {
        const int hs = item_half(k);
        if (hs == -2) break;
        if (hs < 0) continue;
        f32x4 x[KQ];
        encode_item(x, hs, k);
      }
      // Tiles whose e0 rows live in HBM (two node sub-tiles): the rows are no hand-off.  Every e0 row is
      // stored and later loaded by the same lane of the same wave (a padding lane reloads row Et - 1, stored
      // by its own wave in the same instruction), and a half's 16 rows are 16 x 272 B = 34 whole 128-B
      // lines at a 128-B aligned offset, so no line is written by two waves.  This drain is therefore not
      // an ordering requirement: it is a leftover mitigation from the round-5 merged node-phase experiment
      // (where the e0 path was ruled out as that failure's cause), measured neutral.
      if (e0_hbm) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }

  // after the wait: + u[recv] + v[send], ReLU, last Linear, LayerNorm, receiver sums (half_agg);
  // the wave's receiver aggregates are stored to its rows of `sums` at the end
  SGNN_DEV void postwait(__amdgpu_buffer_rsrc_t ru, __amdgpu_buffer_rsrc_t rv, bool probe = false) {
    f32x4 agg[NSUB][KQ];
#pragma unroll
    for (int s = 0; s < NSUB; ++s)
#pragma unroll
      for (int t = 0; t < KQ; ++t) agg[s][t] = zero4();
    // the raw u / v rows of the next half stay in flight across the current half's MFMAs: summing them
    // here would put a wait for the loads just issued in front of those MFMAs
    f32x4 gu[KQ], gv[KQ];
#ifdef SGNN_HANDOFF_CHECK
    uint32_t tg_r[4], tg_s[4];
    int hc_r = 0, hc_s = 0;
#endif
    auto gather = [&](int hs) {  // clamped: harmless past the end
      const int e = hs + j, ec = e < Et ? e : Et - 1;
      int r = lrecv[ec], s = lsend[ec];
      SGNN_BOUNDS(r, 0, a.n, "step16 gathered receiver");
      SGNN_BOUNDS(s, 0, a.n, "step16 gathered sender");
#pragma unroll
      for (int t = 0; t < KQ; ++t) {
        gu[t] = ld4_sc1(ru, r * (H * 4) + (16 * t + 4 * g) * 4);
        gv[t] = ld4_sc1(rv, s * (H * 4) + (16 * t + 4 * g) * 4);
      }
#ifdef SGNN_HANDOFF_CHECK
      hc_r = r;
      hc_s = s;
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        if (!g_hc) break;
        tg_r[w] = __hip_atomic_load((const gu32*)(hc_tags() + ((int64_t)hc_k * a.n + r) * 4 + w), __ATOMIC_RELAXED,
                                    __HIP_MEMORY_SCOPE_AGENT);
        tg_s[w] = __hip_atomic_load((const gu32*)(hc_tags() + ((int64_t)hc_k * a.n + s) * 4 + w), __ATOMIC_RELAXED,
                                    __HIP_MEMORY_SCOPE_AGENT);
      }
#endif
    };
    // check build: the rows of half hs as used (tags against the polled phase, hashes for the final check)
    auto note = [&](int hs) {
#ifdef SGNN_HANDOFF_CHECK
      if (!g_hc) return;
      uint32_t hu = 2166136261u, hv = 2166136261u;
#pragma unroll
      for (int t = 0; t < KQ; ++t) {
        hu = hc_mix(hu, gu[t]);
        hv = hc_mix(hv, gv[t]);
      }
      const int64_t slot = (((int64_t)hc_slot * a.L + hc_k) * kHcHalves + hs / 16) * 64 + l;
      hc_hash(a)[2 * slot] = hu;
      hc_hash(a)[2 * slot + 1] = hv;
      if (hs + j < Et) {
        bool bad = false;
#pragma unroll
        for (int w = 0; w < 4; ++w) bad = bad || tg_r[w] != hc_ep || tg_s[w] != hc_ep;
        if (bad)
          hc_report_tag((int)blockIdx.x, hc_k, b, l, hs + j, hc_r, hc_r / a.nt, tg_r[0], tg_r[1], tg_r[2], tg_r[3], hc_s,
                        hc_s / a.nt, tg_s[0], tg_s[1], tg_s[2], tg_s[3], hc_ep);
      }
#else
      (void)hs;
#endif
    };
    EdgeVec ev;
#pragma unroll
    for (int t = 0; t < KQ; ++t) {
      ev.b2[t] = svec[16 * t + j];
      ev.ga[t] = svec[H + 16 * t + j];
      ev.be[t] = svec[2 * H + 16 * t + j];
    }
    LnAgg<NSUB> la;
    auto finish = [&](const f32x4 (&acc)[KQ], int hs) {  // ReLU -> last Linear -> LayerNorm -> sums
      f32x4 x[KQ], y[KQ];
      lin2_init(acc, x, y, ev);
      mm_full<true>(y, sw1, x, j, g);
#pragma unroll
      for (int p = 0; p < 4; ++p) la.part(p, y, agg, ev, lrecv, hs, Et, i0, j, g);
    };
    const int npre = donor ? kPre - 1 : kPre;  // own halves whose product ran before the wait
    int hs = 16 * b;
    if (hs < Et) gather(hs);
    if (probe) mark(48);
#pragma unroll
    for (int m = 0; m < kPre; ++m) {
      if (hs >= Et) break;
      f32x4 acc[KQ];
      note(hs);
      if (owner_d && m == F) {   // formed by the donor wave (published with the barrier before the wait)
#pragma unroll
        for (int t = 0; t < KQ; ++t) acc[t] = ld4(dbuf + ((b * KQ + t) * 64 + l) * 4) + (gu[t] + gv[t]);
      } else if (m < npre) {
#pragma unroll
        for (int t = 0; t < KQ; ++t) acc[t] = pre[m][t] + (gu[t] + gv[t]);
      } else {
        f32x4 x[KQ];
        ld_e0(x, hs);
#pragma unroll
        for (int t = 0; t < KQ; ++t) acc[t] = gu[t] + gv[t];
        mm_full(acc, sw0, x, j, g);
      }
      gather(hs + 16 * kWaves16);
      finish(acc, hs);
      if (probe) mark(49 + m);
      hs += 16 * kWaves16;
    }
    for (; hs < Et; hs += 16 * kWaves16) {   // halves past kPre: the e0 product here
      f32x4 x[KQ], acc[KQ];
      ld_e0(x, hs);
      note(hs);
#pragma unroll
      for (int t = 0; t < KQ; ++t) acc[t] = gu[t] + gv[t];
      gather(hs + 16 * kWaves16);
      mm_full(acc, sw0, x, j, g);
      finish(acc, hs);
    }
#pragma unroll
    for (int s = 0; s < NSUB; ++s)
#pragma unroll
      for (int t = 0; t < KQ; ++t) st4(sums + (16 * s + j) * LDX + 16 * t + 4 * g, agg[s][t]);
  }
};

// Stage an edge MLP's LDS images: W1e (columns 2H..3H of W1, x scale) and W2 + vectors.
// Up to four H-vectors, one element per thread (wave b holds vector b): requested with the matrices, so
// the LDS images are written without a load round trip of their own.
struct VecStage {
  float v;
  SGNN_DEV void load(const float* p0, const float* p1, const float* p2, const float* p3) {
    const int b = threadIdx.x / 64;
    const float* p = b == 0 ? p0 : b == 1 ? p1 : b == 2 ? p2 : p3;
    v = p ? p[threadIdx.x & 63] : 0.0f;
  }
  SGNN_DEV void store(float* dst, int nvec) const {
    if ((int)threadIdx.x < nvec * H) dst[threadIdx.x] = v;
  }
};
static_assert(kBlock16 == 4 * H, "VecStage: one element per thread");

struct EdgeStage {
  f32x4 w1e[kStagePer], w2[kStagePer];
  VecStage vec;
  SGNN_DEV void load(const Lay16& L) {
    stage_w64_load(w1e, L.ew1 + 2 * H, 3 * H);
    stage_w64_load(w2, L.ew2, H);
    vec.load(L.eb2, L.eg, L.ebb, nullptr);
  }
  SGNN_DEV void store(float* sw0, float* sw1, float* svec, float scale) const {
    stage_w64_store(sw0, w1e, scale);
    stage_w64_store(sw1, w2, 1.0f);
    vec.store(svec, 3);
  }
};

// Layer k's weights by a constant index per case: indexing the kernel-argument
// array with a runtime k would copy the whole argument block to scratch.
SGNN_DEV Lay16 lay_at(const Step16Args& a, int k) {
  switch (k) {
    case 0: return a.lay[0];
    case 1: return a.lay[1];
    case 2: return a.lay[2];
    case 3: return a.lay[3];
    case 4: return a.lay[4];
    case 5: return a.lay[5];
    case 6: return a.lay[6];
    case 7: return a.lay[7];
    case 8: return a.lay[8];
    default: return a.lay[9];
  }
}
static_assert(sgnn::kStep16MaxL == 10, "lay_at covers every layer");

SGNN_DEV Node16Args node_args(const Step16Args& a, const Lay16& L, const Lay16* next) {
  Node16Args nd{};
  nd.w1 = L.nw1; nd.b1 = L.nb1; nd.w2 = L.nw2; nd.b2 = L.nb2; nd.g = L.ng; nd.bb = L.nbb;
  if (next) {
    nd.we = next->ew1; nd.be = next->eb1;
  } else {
    nd.wd1 = a.d_w1; nd.bd1 = a.d_b1; nd.wd2 = a.d_w2; nd.bd2 = a.d_b2;
  }
  nd.dim = a.dim;
  return nd;
}

// One interaction layer of the tile: wait for the sender tiles' u_k / v_k,
// edge phase, receiver sums, node phase, publish u_{k+1} / v_{k+1}, stage the
// next layer's edge weights.
template <bool FIRST, int MODE, bool E0G, int NSUB, int PUB>
SGNN_DEV void step_layer(const Step16Args& a, int k, float* lds, const Carve& cv, const float (&xw1)[KQ],
                         const int32_t* deps, int ndeps, const int32_t* lsend, const int32_t* lrecv, int Et, int i0,
                         int cnt, int b, int j, int g, int l, int tile) {
  float* sw0 = lds + cv.sw0;
  float* sw1 = lds + cv.sw1;
  float* svec = lds + cv.svec;
  float* scratch = lds + cv.scratch;
  float* xs = lds + cv.xs;
  const int64_t nH = (int64_t)a.n * H;
  // e0 rows of the tile's edges: LDS, or (graphs whose tile does not fit) a per-tile HBM block behind
  // the layers' node halves -- written and read by this workgroup only
  float* e0l = E0G ? a.uvl + 2 * a.L * nH + (int64_t)tile * a.ecap_t * LDX : lds + cv.region;
  const __amdgpu_buffer_rsrc_t ru = buf_rsrc(a.uvl + (2 * k) * nH), rv = buf_rsrc(a.uvl + (2 * k + 1) * nH);
  const Lay16 Lk = lay_at(a, k), Ln = lay_at(a, MODE == 0 ? k + 1 : k);
  // this layer's node weights (VGPR-resident) are requested first: the W1e e0 products and the wait
  // for the sender tiles hide their latency (this layer's edge weights were staged in LDS before the
  // previous layer published)
  const int ps = k < 5 ? 3 + 8 * k : -1;  // probe slots of this layer
  mark(ps);
  NodeW<2, MODE> W;
  const Node16Args nd = node_args(a, Lk, MODE == 0 ? &Ln : nullptr);
  float* sums = scratch + b * 16 * NSUB * LDX;
  EdgePhase<NSUB> ep{a, sw0, sw1, svec, lds + cv.sxw, lds + cv.sxv, sums, e0l, lsend, lrecv, Et, i0, b, j, g, l};
  ep.e0_hbm = E0G;
  ep.hc_k = k;
  ep.hc_slot = (int)blockIdx.x;
  ep.hc_ep = a.epoch0 + (uint32_t)k + 1;
  mark(ps < 0 ? -1 : ps + 1);
  // Between the pre-wait products: publish phase k + 1 (u_k / v_k, stored by the previous stage; the
  // drain of those write-through stores overlaps the first product), then request this layer's node
  // weights (VGPR-resident) in three parts, so neither the drain nor the load issue stalls the MFMAs.
  const uint32_t ep_k = a.epoch0 + (uint32_t)k + 1;
  TilePoll poll;
  // The publish point PUB: after the first product (1), so the drain of the write-through stores overlaps
  // it -- or, in tiles of at most one half per wave, whose layer is a latency chain through the sender
  // tiles' flags, before any product (0): the kernel picks per tile (k_step16)
  constexpr int pub_at = PUB;
  auto hook = [&](int m) {
    if (m == pub_at) {
      publish(a.flags, tile, ep_k, a.skew);
      mark(ps < 0 ? -1 : ps + 2);
      W.load_first(nd, b, j, g);
    }
    // publishing before the first product: the donated products (dbuf, written in the donors' slot 0)
    // need a barrier of their own before any owner reads them after its wait
    if (pub_at == 0 && m == 1 && ep.donates) __syncthreads();
    if (m == (pub_at + 1 < kPre ? pub_at + 1 : kPre)) W.load_mid(nd, b, j, g);
    if (m == kPre - 1) poll.issue(deps, ndeps, a.flags, ep_k, l);
    if (m == kPre) poll.issue2(deps, ndeps, a.flags, ep_k, l);
    if (m == (pub_at + 2 < kPre ? pub_at + 2 : kPre)) W.load_out(nd, b, j, g);
  };
  ep.plan(lds + cv.dbuf);
  if (ep.donor) ep.template prewait<FIRST, true>(xw1, hook);
  else ep.template prewait<FIRST, false>(xw1, hook);
  mark(ps < 0 ? -1 : ps + 3);
  poll.wait(deps, ndeps, a.flags, ep_k, l, a.poll_limit);
  // Guideline 16 (every load of the handed-off rows is an sc1 buffer load): no acquire instruction, but
  // this wave-scope fence keeps the compiler from moving those loads above the poll
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  mark(ps < 0 ? -1 : ps + 4);
  ep.postwait(ru, rv, k == 1);
  mark(ps < 0 ? -1 : ps + 5);
  __syncthreads();
  // the next layer's edge weights: requested now, staged in LDS before this layer publishes
  EdgeStage nxt;
  if (MODE == 0) nxt.load(Ln);
  // receiver sums of sub-tile s: the four waves' partial rows 16 s + j of their blocks
  constexpr int kWaveRows = 16 * NSUB;
  auto sum_rows = [&](f32x4 (&ag)[KQ], int s) {
#pragma unroll
    for (int q = 0; q < KQ; ++q) {
      ag[q] = ld4(scratch + (16 * s + j) * LDX + 16 * q + 4 * g);
#pragma unroll
      for (int w = 1; w < kWaves16; ++w) ag[q] += ld4(scratch + (w * kWaveRows + 16 * s + j) * LDX + 16 * q + 4 * g);
    }
  };
  f32x4 ag[KQ], xr[KQ];
  sum_rows(ag, 0);
#pragma unroll
  for (int q = 0; q < KQ; ++q) xr[q] = ld4(xs + j * LDX + 16 * q + 4 * g);
  f32x4 xo = ld4(xs + j * LDX + 16 * b + 4 * g);
  // sub-tile 1's sums move to rows the exchange buffers (rows 0 .. 47) leave alone: wave 3's block
  float* ag1 = scratch + 3 * kWaveRows * LDX;
  if constexpr (NSUB > 1) {
    f32x4 t1[KQ];
    sum_rows(t1, 1);
    __syncthreads();
#pragma unroll
    for (int q = 0; q < KQ; ++q) st4(ag1 + j * LDX + 16 * q + 4 * g, t1[q]);
  }
  __syncthreads();  // the exchange buffers alias the sums
  if (k == 1) mark(52);
  // u_{k+1} / v_{k+1} (mode 0); the decoder needs none
  const __amdgpu_buffer_rsrc_t ru1 = buf_rsrc(a.uvl + (MODE == 0 ? 2 * k + 2 : 0) * nH),
                               rv1 = buf_rsrc(a.uvl + (MODE == 0 ? 2 * k + 3 : 0) * nH);
#pragma unroll
  for (int s = 0; s < NSUB; ++s) {
    if (s > 0) {  // (sub-tile 1's rows: written by no exchange of sub-tile 0)
#pragma unroll
      for (int q = 0; q < KQ; ++q) {
        ag[q] = ld4(ag1 + j * LDX + 16 * q + 4 * g);
        xr[q] = ld4(xs + (16 * s + j) * LDX + 16 * q + 4 * g);
      }
      xo = ld4(xs + (16 * s + j) * LDX + 16 * b + 4 * g);
    }
    const f32x4 h[1] = {relu4(mm_cat(W.vb1, W.w1a, ag, W.w1x, xr))};  // graph_network.py:220
    if (k == 1 && s == 0) mark(53);
    const f32x4 xo1[1] = {xo};
    step_tail<MODE, 1>(a, W, scratch, xs + 16 * s * LDX, i0 + 16 * s, cnt - 16 * s, h, xo1, b, j, g, ru1, rv1, k + 1);
  }
  mark(ps < 0 ? -1 : ps + 6);
  if constexpr (MODE == 0) {
    nxt.store(sw0, sw1, svec, (float)(2 << k));  // W1e x 2^(k+1): exact
    __syncthreads();  // the next layer's pre-wait reads the staged weights; it publishes u_{k+1} / v_{k+1}
  }
  mark(ps < 0 ? -1 : ps + 7);
}

#ifdef SGNN_HANDOFF_CHECK
// Check build, after the last layer: every workgroup publishes a final phase (epoch0 + L + 1: no layer
// uses it, the next step starts at epoch0 + L + 2) in its own slot and waits until EVERY slot holds it
// (all workgroups resident; a grid barrier, once), so every node-half row of the step has settled.
// Then each wave re-gathers every half it used in every layer (sc1 loads) and compares the hashes.
SGNN_DEV void hc_final(const Step16Args& a, int tile, const int32_t* lsend, const int32_t* lrecv, int Et, int b,
                       int j, int g, int l) {
  if (a.poll_limit < 0 || !g_hc) return;  // the forced-timeout test hook / no buffer: nothing to check
  const uint32_t fin = a.epoch0 + (uint32_t)a.L + 1u;
  publish(a.flags, tile, fin, 0);
  const int G = (int)gridDim.x;
  for (int it = 0; it < (1 << 22); ++it) {
    bool ok = true;
    for (int t = l; t < G; t += 64)
      ok = ok && __hip_atomic_load((const gu32*)(a.flags + t * kStepFlagStride), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= fin;
    if (__all(ok)) break;
    __builtin_amdgcn_s_sleep(2);
  }
  if (threadIdx.x == 0) atomicAdd(g_hc + 3, 1u);
  const int64_t nH = (int64_t)a.n * H;
  for (int k = 0; k < a.L; ++k) {
    const __amdgpu_buffer_rsrc_t ru = buf_rsrc(a.uvl + (2 * k) * nH), rv = buf_rsrc(a.uvl + (2 * k + 1) * nH);
    for (int hs = 16 * b; hs < Et; hs += 16 * kWaves16) {
      const int e = hs + j, ec = e < Et ? e : Et - 1;
      const int r = lrecv[ec], s = lsend[ec];
      uint32_t hu = 2166136261u, hv = 2166136261u;
#pragma unroll
      for (int t = 0; t < KQ; ++t) {
        hu = hc_mix(hu, ld4_sc1(ru, r * (H * 4) + (16 * t + 4 * g) * 4));
        hv = hc_mix(hv, ld4_sc1(rv, s * (H * 4) + (16 * t + 4 * g) * 4));
      }
      const int64_t slot = (((int64_t)blockIdx.x * a.L + k) * kHcHalves + hs / 16) * 64 + l;
      const bool bu = hu != hc_hash(a)[2 * slot], bv = hv != hc_hash(a)[2 * slot + 1];
      if (bu || bv) hc_report_stale((int)blockIdx.x, k, b, l, e, Et, r, r / a.nt, bu, s, s / a.nt, bv);
    }
  }
}
#endif

template <int DIM, int KQF, bool E0G, int NSUB>
__global__ __launch_bounds__(kBlock16) __attribute__((amdgpu_waves_per_eu(1))) void k_step16(Step16Args a_) {
  // every access through the kernel-argument segment itself (scalar loads): binding a reference to
  // the by-value parameter would copy its 1.3 KB to scratch first
  (void)a_;
  const Step16Args& a = *(const Step16Args*)(const __attribute__((address_space(4))) Step16Args*)
                             __builtin_amdgcn_kernarg_segment_ptr();
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int l = lane_id(), j = l & 15, g = l >> 4, b = wave_id();
  // The tile this workgroup owns.  tile_order 1: XCD-contiguous tiles -- blocks
  // b, b + 8, ... share an XCD under the dispatch order and take consecutive tiles, so the sender tiles of a
  // tile (its lattice neighbours) mostly share its L2: XCD x (= b mod 8) owns G / 8 (+1 for x < G mod 8)
  // consecutive tiles, a bijection.  EVERY use of the tile index (publish slot, dependency list, e0 block)
  // takes this one value (step_layer's `tile` argument); placement is a speed matter only.
  const bool xcd_order = a.tile_order != 0;
  const int xq = (int)gridDim.x / 8, xr = (int)gridDim.x % 8, xc = (int)blockIdx.x % 8;
  const int tile = xcd_order ? xc * xq + min(xc, xr) + (int)blockIdx.x / 8 : (int)blockIdx.x;
  const int nt = a.nt, cap = a.cap, n = a.n;
  const int i0 = tile * nt;
  const int cnt = min(nt, n - i0);
  const Carve cv = carve(n, DIM, nt, cap, E0G);
  int32_t* ints = reinterpret_cast<int32_t*>(lds + cv.ints);
  int32_t* lsend = ints;
  int32_t* lrecv = lsend + ((nt * cap + 15) & ~15);   // 16-B aligned rows: half_agg reads int4s
  int32_t* nbr_l = lrecv + ((nt * cap + 15) & ~15);
  int32_t* ldeg = nbr_l + nt * cap;
  int32_t* lpre = ldeg + kMaxNT;
  uint32_t* mask = reinterpret_cast<uint32_t*>(lpre + kMaxNT + 4);
  int32_t* kw_all = reinterpret_cast<int32_t*>(mask + 8);
  int32_t* deps = kw_all + 4 * 64;       // the sender tiles of this tile's edges, compacted
  int32_t* ndeps_l = deps + kMaxGrid;
  int32_t* exs = ndeps_l + 4;            // example offsets (ex_ptr)
  float* rp = reinterpret_cast<float*>(exs + sgnn::kStep16MaxEx + 4);  // [3][32] the tile's receivers' positions
  float* box = rp + 3 * kMaxNT;          // the receivers' bounding box grown by the margin: lo [3], hi [3]
  int32_t* segn = reinterpret_cast<int32_t*>(box + 8);  // kept candidates per wave segment

  mark(0);
  if (threadIdx.x < 8) mask[threadIdx.x] = 0u;

  // ---- radius graph of the tile's receivers (torch_cluster's rule: first `cap` in-range senders of
  // the receiver's example in ascending index, strict <; learned_simulator.py:116-117) --------------
  // the tile's node features (learned_simulator.py:256-290): their raw inputs are requested first and
  // combined after the radius search, so the loads complete under it
  const int nvel = (a.T - 1) * DIM;
  float fr0[NSUB][KQF][4], fr1[NSUB][KQF][4], vmean[DIM], vstd[DIM];
  int64_t ptype[NSUB];
#pragma unroll
  for (int d = 0; d < DIM; ++d) {
    vmean[d] = a.vel_mean[d];
    vstd[d] = a.vel_std[d];
  }
#pragma unroll
  for (int s = 0; s < NSUB; ++s) {
    const int64_t ic = 16 * s + j < cnt ? (int64_t)(i0 + 16 * s + j) : (int64_t)i0;
    const float* p = a.pos_seq + ic * a.T * DIM;
#pragma unroll
    for (int q = 0; q < KQF; ++q)
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int f = 16 * q + 4 * g + c, t = f / DIM, cc = f - t * DIM;
        fr0[s][q][c] = f < nvel ? p[(t + 1) * DIM + cc] : f == nvel ? p[(a.T - 1) * DIM] : 0.0f;
        fr1[s][q][c] = f < nvel ? p[t * DIM + cc] : 0.0f;
      }
    ptype[s] = a.use_emb ? a.types[ic] : 0;
  }
  // the window's last frame (or the previous step's contiguous next_pos)
  const float* src = a.pos_last ? a.pos_last : a.pos_seq + (int64_t)(a.T - 1) * DIM;
  const int pstride = a.pos_last ? DIM : a.T * DIM;
  const int n_ex = a.n_ex;
  // one example (the rollout benches): the candidates are [0, n) without waiting for ex_ptr, so the first
  // filter batch's positions are requested now, under the receivers' box and the weight loads (used below
  // only if ex_ptr confirms [0, n))
  constexpr int kBatch = 8;  // 64-candidate chunks whose loads are in flight together (16: neutral to +1 %)
  const int Q1 = (((a.n + 3) >> 2) + 63) & ~63;
  const bool pre_ok = n_ex == 1 && b * Q1 < a.n;
  float pre[kBatch][DIM];
  if (pre_ok) {
    const int s0 = b * Q1, s1 = min(s0 + Q1, a.n);
#pragma unroll
    for (int u = 0; u < kBatch; ++u) {
      const int jj = min(s0 + 64 * u + l, s1 - 1);
#pragma unroll
      for (int d = 0; d < DIM; ++d) pre[u][d] = src[(int64_t)jj * pstride + d];
    }
  }
  {  // example offsets; wave 0: the receivers' positions and their bounding box, grown by the margin
    const int64_t exv = (int)threadIdx.x <= n_ex ? a.ex_ptr[threadIdx.x] : 0;
    if (b == 0) {
      float lo[DIM], hi[DIM];
#pragma unroll
      for (int d = 0; d < DIM; ++d) {
        const float v = src[(int64_t)(i0 + min(l, cnt - 1)) * pstride + d];
        if (l < cnt) rp[d * kMaxNT + l] = v;
        lo[d] = v;
        hi[d] = v;
      }
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1)
#pragma unroll
        for (int d = 0; d < DIM; ++d) {
          lo[d] = fminf(lo[d], __shfl_xor(lo[d], o, 64));
          hi[d] = fmaxf(hi[d], __shfl_xor(hi[d], o, 64));
        }
      // |p_j - p_i|^2 < r^2 in fp32 implies |p_j,d - p_i,d| < r (1 + 2^-22) + one ulp of the coordinates:
      // 1e-3 r + 1e-6 |p| covers both with room (a wider box only keeps more candidates; radius_small.h)
      float mag = 0.0f;
#pragma unroll
      for (int d = 0; d < DIM; ++d) mag = fmaxf(mag, fmaxf(fabsf(lo[d]), fabsf(hi[d])));
      const float m = 1.001f * a.radius + 1e-6f * (mag + 1.0f);
      if (l == 0)
#pragma unroll
        for (int d = 0; d < DIM; ++d) {
          box[d] = lo[d] - m;
          box[3 + d] = hi[d] + m;
        }
    }
    if ((int)threadIdx.x <= n_ex) exs[threadIdx.x] = (int32_t)exv;
  }

  if (a.use_emb) {  // :287-290 type embedding
#pragma unroll
    for (int s = 0; s < NSUB; ++s)
#pragma unroll
      for (int q = 0; q < KQF; ++q)
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const int f = 16 * q + 4 * g + c;
          if (f > nvel && f < nvel + 1 + a.emb_dim) fr0[s][q][c] = a.emb_w[ptype[s] * a.emb_dim + (f - nvel - 1)];
        }
  }
  // weights of layer 0's edge MLP and of Encoder.edge_fn (LDS images after the radius search), issued after
  // the positions (loads complete in order) and in flight during the radius queries; Encoder.node_fn's
  // (VGPR-resident) follow the queries, under the LDS staging and the tile CSR
  EdgeStage st0;
  st0.load(a.lay[0]);
  f32x4 sx[kStagePer];
  stage_w64_load(sx, a.xe_w2, H);
  VecStage sxv;
  sxv.load(a.xe_b1, a.xe_b2, a.xe_g, a.xe_bb);
  NodeW<2, 0> E;
  f32x4 w1f[KQF];
  f32x4 vb1;
  auto load_encoder = [&]() {
    Node16Args nd{};
    nd.w2 = a.xn_w2; nd.b2 = a.xn_b2; nd.g = a.xn_g; nd.bb = a.xn_bb;
    nd.we = a.lay[0].ew1; nd.be = a.lay[0].eb1; nd.dim = DIM;
    E.load_tail(nd, b, j, g);
    const int urow = 16 * b + j;
#pragma unroll
    for (int q = 0; q < KQF; ++q)
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int f = 16 * q + 4 * g + c;
        w1f[q][c] = f < a.feat ? a.xn_w1[(int64_t)urow * a.feat + f] : 0.0f;
      }
    vb1 = ld4(a.xn_b1 + 16 * b + 4 * g);
  };
  __syncthreads();
  // the candidates: the examples of the tile's receivers, [jb, je), kept when inside the box.  Wave w
  // filters the contiguous quarter [jb + w Q, jb + (w + 1) Q) into its own segment of the list, so the
  // segments in order are ascending in index (the scan below takes them in order).
  float* cp = lds;                                                   // [DIM][list_cap] positions
  int32_t* cid = reinterpret_cast<int32_t*>(lds + DIM * cv.list_cap);  // [list_cap] indices
  auto example_of = [&](int i) {  // largest e with ex_ptr[e] <= i
    int lo = 0, hi = n_ex - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (exs[mid] <= i) lo = mid; else hi = mid - 1;
    }
    return lo;
  };
  const int cjb = exs[example_of(i0)], cje = exs[example_of(i0 + cnt - 1) + 1];
  const int Q = (((cje - cjb + 3) >> 2) + 63) & ~63;
  {
    float blo[DIM], bhi[DIM];
#pragma unroll
    for (int d = 0; d < DIM; ++d) {
      blo[d] = box[d];
      bhi[d] = box[3 + d];
    }
    const int s0 = cjb + b * Q, s1 = min(s0 + Q, cje);
    int kept = 0;
    const bool use_pre = pre_ok && cjb == 0 && cje == a.n;   // then s0 = b Q1, s1 = min(s0 + Q1, n) as above
    for (int base = s0; base < s1; base += 64 * kBatch) {
      float pc[kBatch][DIM];
      if (use_pre && base == s0) {
#pragma unroll
        for (int u = 0; u < kBatch; ++u)
#pragma unroll
          for (int d = 0; d < DIM; ++d) pc[u][d] = pre[u][d];
      } else {
#pragma unroll
        for (int u = 0; u < kBatch; ++u) {
          const int jj = min(base + 64 * u + l, s1 - 1);
#pragma unroll
          for (int d = 0; d < DIM; ++d) pc[u][d] = src[(int64_t)jj * pstride + d];
        }
      }
#pragma unroll
      for (int u = 0; u < kBatch; ++u) {
        const int jj = base + 64 * u + l;
        bool in = jj < s1;
#pragma unroll
        for (int d = 0; d < DIM; ++d) in = in && pc[u][d] >= blo[d] && pc[u][d] <= bhi[d];
        const uint64_t bal = __ballot(in);
        if (in) {
          const int slot = b * Q + kept + (int)__popcll(bal & ((1ull << l) - 1ull));
          SGNN_BOUNDS(slot, 0, cv.list_cap, "step16 candidate slot");
#pragma unroll
          for (int d = 0; d < DIM; ++d) cp[d * cv.list_cap + slot] = pc[u][d];
          cid[slot] = jj;
        }
        kept += (int)__popcll(bal);
      }
    }
    if (l == 0) segn[b] = kept;
  }
  __syncthreads();
  mark(56);  // probe: candidates staged
  {
    int32_t* kw = kw_all + b * 64;
    const float r2 = a.r2;  // a local: the LDS stores below would make the compiler re-load the argument
    const int loop = a.loop;
    int sn[kWaves16];
#pragma unroll
    for (int w = 0; w < kWaves16; ++w) sn[w] = segn[w];
    for (int rl = b; rl < cnt; rl += kWaves16) {
      const int i = i0 + rl;
      const int ex = example_of(i);
      const int jb = exs[ex], je = exs[ex + 1];
      float pi[DIM];
#pragma unroll
      for (int d = 0; d < DIM; ++d) pi[d] = rp[d * kMaxNT + rl];
      int c = 0;
      // four 64-candidate chunks per round: their LDS reads are in flight together, then the chunks
      // are taken in index order (the first `cap` in range are kept; a round may test up to three
      // chunks past the cap, harmlessly)
      constexpr int kRound = 4;
      for (int w = 0; w < kWaves16 && c < cap; ++w) {
        const int wn = sn[w], wb = w * Q;
        for (int base = 0; base < wn && c < cap; base += 64 * kRound) {
          float pc[kRound][DIM];
          int id[kRound];
#pragma unroll
          for (int u = 0; u < kRound; ++u) {
            const int kk = wb + min(base + 64 * u + l, wn - 1);
#pragma unroll
            for (int d = 0; d < DIM; ++d) pc[u][d] = cp[d * cv.list_cap + kk];
            id[u] = cid[kk];
          }
#pragma unroll
          for (int u = 0; u < kRound; ++u) {
            float s = 0.0f;  // fp32, dims summed in order, no contraction (oracle rule)
#pragma unroll
            for (int d = 0; d < DIM; ++d) {
#pragma clang fp contract(off)
              const float t = __fsub_rn(pc[u][d], pi[d]);
              s = __fadd_rn(s, __fmul_rn(t, t));
            }
            const bool in = base + 64 * u + l < wn && id[u] >= jb && id[u] < je && s < r2;
            const uint64_t bal = __ballot(in);
            const int slot = c + (int)__popcll(bal & ((1ull << l) - 1ull));
            if (in && slot < cap) kw[slot] = id[u];
            c += (int)__popcll(bal);
          }
        }
      }
      wave_lds_sync();
      c = min(c, cap);
      int top = l < c ? kw[l] : INT32_MAX;
      if (!loop) {  // torch_cluster: K+1 first-by-index, then the self loop dropped
        const uint64_t self = __ballot(l < c && top == i);
        if (self) {
          const int at = __ffsll((long long)self) - 1;
          const int nx = __shfl(top, (l + 1) & 63, 64);
          if (l >= at) top = (l + 1 < c) ? nx : INT32_MAX;
          c -= 1;
        }
      }
      if (l < c) nbr_l[rl * cap + l] = top;
      if (l == 0) ldeg[rl] = c;
      wave_lds_sync();
    }
  }
  __syncthreads();  // the candidate list overlays the weights' LDS images
  mark(1);
  load_encoder();
  // LDS images of the staged weights (requested before the radius phase)
  st0.store(lds + cv.sw0, lds + cv.sw1, lds + cv.svec, 1.0f);
  stage_w64_store(lds + cv.sxw, sx, 1.0f);
  sxv.store(lds + cv.sxv, 4);
  __syncthreads();
  mark(58);  // probe: weights in LDS
  // tile CSR (receiver-sorted, senders ascending) from the kept lists; sender-tile mask
  if (b == 0) {
    const int dg = l < cnt ? ldeg[l] : 0;
    int incl = dg;
#pragma unroll
    for (int o = 1; o < kMaxNT; o <<= 1) {
      const int t = __shfl_up(incl, o, 64);
      if (l >= o) incl += t;
    }
    if (l < kMaxNT) lpre[l + 1] = incl;
    if (l == 0) lpre[0] = 0;
    if (a.deg_out && l < cnt) a.deg_out[i0 + l] = dg;
  }
  __syncthreads();
  const int Et = lpre[cnt];
  for (int t = threadIdx.x; t < cnt * cap; t += kBlock16) {
    const int k = t / cap, q = t - k * cap;
    if (q < ldeg[k]) {
      int32_t sv = nbr_l[k * cap + q];
      SGNN_BOUNDS(sv, 0, n, "step16 sender");
      int e = lpre[k] + q;
      SGNN_BOUNDS(e, 0, nt * cap, "step16 tile edge");
      lsend[e] = sv;
      lrecv[e] = i0 + k;
      const int st = sv / nt;
      atomicOr(&mask[st >> 5], 1u << (st & 31));
      if (a.nbr_out) a.nbr_out[(int64_t)(i0 + k) * cap + q] = sv;
    }
  }
  __syncthreads();
  mark(59);  // probe: CSR built
  if (b == 0) {  // the mask as a list (wave_lds_sync-free: one wave, in order)
    int base = 0;
    for (int t0 = 0; t0 < (int)gridDim.x; t0 += 64) {
      const int t = t0 + l;
      const bool on = t < (int)gridDim.x && ((mask[t >> 5] >> (t & 31)) & 1u);
      const uint64_t bal = __ballot(on);
      if (on) {
        int slot = base + (int)__popcll(bal & ((1ull << l) - 1ull));
        SGNN_BOUNDS(slot, 0, kMaxGrid, "step16 dependency list");
        deps[slot] = t;
      }
      base += (int)__popcll(bal);
    }
    if (l == 0) *ndeps_l = base;
  }

  // ---- Encoder.node_fn of the tile's nodes (features: learned_simulator.py:256-290) -> x0 (LDS),
  // u_0 / v_0 (published as phase 1) ------------------------------------------------------------
  float xw1[KQ] = {0.0f, 0.0f, 0.0f, 0.0f};  // Encoder.edge_fn W1 [H][dim + 1]: unit 16 t + j, k = g
#pragma unroll
  for (int t = 0; t < KQ; ++t) xw1[t] = g <= DIM ? a.xe_w1[(16 * t + j) * (DIM + 1) + g] : 0.0f;
  f32x4 eh[NSUB], ez[NSUB];
#pragma unroll
  for (int s = 0; s < NSUB; ++s) {
    f32x4 xf[KQF];
#pragma unroll
    for (int q = 0; q < KQF; ++q)
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int f = 16 * q + 4 * g + c, t = f / DIM, cc = f - t * DIM;
        float val = fr0[s][q][c];  // embedding, or 0 past the features
        if (f < nvel) {  // learned_simulator.py:258,272-278 normalised velocity history
          float mn = vmean[0], sd = vstd[0];
#pragma unroll
          for (int d = 1; d < DIM; ++d)
            if (cc == d) {
              mn = vmean[d];
              sd = vstd[d];
            }
          val = __fdiv_rn(__fsub_rn(__fsub_rn(fr0[s][q][c], fr1[s][q][c]), mn), sd);
        } else if (f == nvel) {  // :282-284 wall distance
          val = __fdiv_rn(fminf(fmaxf(__fadd_rn(fr0[s][q][c], 2.0f), 0.0f), a.wall_max), a.wall_div);
        }
        xf[q][c] = val;
      }
    eh[s] = relu4(mm(vb1, w1f, xf));
    ez[s] = zero4();
  }
#pragma unroll
  for (int s = 0; s < NSUB; ++s) {
    const f32x4 h1[1] = {eh[s]}, x1[1] = {ez[s]};
    step_tail<0, 1>(a, E, lds + cv.scratch, lds + cv.xs + 16 * s * LDX, i0 + 16 * s, cnt - 16 * s, h1, x1, b, j, g,
                    buf_rsrc(a.uvl), buf_rsrc(a.uvl + (int64_t)n * H), 0);
  }
  mark(2);  // u_0 / v_0 are published by layer 0's pre-wait

  // ---- the interaction layers ------------------------------------------------------------------
  const int ndeps = *ndeps_l;
  // the publish point (step_layer): before the first pre-wait product where the waves hold at most one
  // half each (a layer of such tiles is a latency chain through the sender tiles' flags: C1 r = 0.6
  // 64.9 -> 61.6 us per step), after it otherwise (its drain then overlaps the product: publishing first
  // there cost 0.5-1.6 %); same-box A/Bs, DESIGN.md section 5
  auto layers = [&](auto pub) {
    constexpr int P = decltype(pub)::value;
    step_layer<true, 0, E0G, NSUB, P>(a, 0, lds, cv, xw1, deps, ndeps, lsend, lrecv, Et, i0, cnt, b, j, g, l, tile);
    for (int k = 1; k < a.L - 1; ++k)
      step_layer<false, 0, E0G, NSUB, P>(a, k, lds, cv, xw1, deps, ndeps, lsend, lrecv, Et, i0, cnt, b, j, g, l,
                                         tile);
    step_layer<false, 1, E0G, NSUB, P>(a, a.L - 1, lds, cv, xw1, deps, ndeps, lsend, lrecv, Et, i0, cnt, b, j, g, l,
                                       tile);
  };
  if (Et <= 16 * kWaves16) layers(std::integral_constant<int, 0>{});
  else layers(std::integral_constant<int, kPubAt>{});
#ifdef SGNN_HANDOFF_CHECK
  hc_final(a, tile, lsend, lrecv, Et, b, j, g, l);
#endif
}

}  // namespace

namespace sgnn {

size_t step16_lds_bytes(const Step16Args& a) {
  if (a.nt < 1 || a.nt > kStep16MaxNT || a.cap < 1 || a.cap > kStep16MaxCap || a.dim < 1 || a.dim > 3) return 0;
  return sizeof(float) * (size_t)carve(a.n, a.dim, a.nt, a.cap, a.e0_hbm != 0).total;
}

namespace {
using Step16Kernel = void (*)(Step16Args);

// The kernel variant for these arguments (null when none applies).
Step16Kernel step16_kernel(const Step16Args& a) {
  const int kqf = (a.feat + 15) / 16;
  if (kqf < 1 || kqf > 3 || a.dim < 1 || a.dim > 3) return nullptr;
#define SGNN_S16(D_, G_, S_) \
  return kqf == 1 ? k_step16<D_, 1, G_, S_> : kqf == 2 ? k_step16<D_, 2, G_, S_> : k_step16<D_, 3, G_, S_>
  if (a.nt > 16) {  // two node sub-tiles: the tile's e0 rows never fit next to them
    if (!a.e0_hbm) return nullptr;
    if (a.dim == 1) SGNN_S16(1, true, 2);
    if (a.dim == 2) SGNN_S16(2, true, 2);
    SGNN_S16(3, true, 2);
  }
  if (a.e0_hbm) {
    if (a.dim == 1) SGNN_S16(1, true, 1);
    if (a.dim == 2) SGNN_S16(2, true, 1);
    SGNN_S16(3, true, 1);
  }
  if (a.dim == 1) SGNN_S16(1, false, 1);
  if (a.dim == 2) SGNN_S16(2, false, 1);
  SGNN_S16(3, false, 1);
#undef SGNN_S16
}

// at least 81 KB: one workgroup per CU whatever the shape (the hand-off protocol's measured form)
size_t step16_lds_request(const Step16Args& a) { return std::max<size_t>(step16_lds_bytes(a), 81 * 1024); }
}  // namespace

int64_t step16_resident(const Step16Args& a) {
  const Step16Kernel kern = step16_kernel(a);
  const size_t lds = step16_lds_bytes(a);
  if (!kern || lds == 0 || lds > kStep16MaxLds) return 0;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  // the occupancy query per (device, variant, LDS request), once
  static std::mutex mu;
  static std::map<std::tuple<int, const void*, size_t>, int64_t> cache;
  const auto key = std::make_tuple(dev, reinterpret_cast<const void*>(kern), step16_lds_request(a));
  std::lock_guard<std::mutex> lk(mu);
  const auto it = cache.find(key);
  if (it != cache.end()) return it->second;
  int cus = 0, per_cu = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)kStep16MaxLds);
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void*>(kern), kBlock16,
                                                   std::get<2>(key)) != hipSuccess)
    return 0;
  return cache[key] = (int64_t)per_cu * cus;
}

int step16_launch(const Step16Args& a_in, hipStream_t s) {
  Step16Args a = a_in;
  if (a.poll_limit == 0) a.poll_limit = kPollLimit;
  const size_t lds = step16_lds_bytes(a);
  const int64_t grid = ((int64_t)a.n + a.nt - 1) / a.nt;
  if (lds == 0 || lds > kStep16MaxLds || grid < 1 || grid > kStep16MaxGrid || a.L < 2 || a.L > kStep16MaxL ||
      a.ecap_t != a.nt * a.cap)
    return set_error(SGNN_ERR_UNSUPPORTED, "step16: shape outside the one-launch step");
  const Step16Kernel kern = step16_kernel(a);
  if (!kern) return set_error(SGNN_ERR_UNSUPPORTED, "step16: more than 48 node features");
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)kStep16MaxLds);
  hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(kBlock16), step16_lds_request(a), s, a);
  return check_launch("step16");
}

}  // namespace sgnn

#ifdef SGNN_HANDOFF_CHECK
extern "C" int sgnn_set_handoff_check(uint32_t* buf) {
  return hipMemcpyToSymbol(HIP_SYMBOL(g_hc), &buf, sizeof(buf)) == hipSuccess ? 0 : 3;
}
#endif

#ifdef SGNN_PROBE
extern "C" int sgnn_set_probe16(uint64_t* buf) {
  return hipMemcpyToSymbol(HIP_SYMBOL(g_probe16), &buf, sizeof(buf)) == hipSuccess ? 0 : 3;
}
#endif
