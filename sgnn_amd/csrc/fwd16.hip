// Inference node layer for H = 64 on v_mfma_f32_16x16x4_f32 (gfx950).
//
// Replaces, per InteractionNetwork, the node half of
// sgnn/single_scale/graph_network.py:201-222 (node MLP on cat[aggr, x] + LN),
// the residual of :176, and either the next layer's edge-MLP node halves
// (u = W1_i x + b1, v = W1_j x, see epd_fwd.hip) or the Decoder (:321-333)
// with the Euler integrator of learned_simulator.py:381-411.
//
// Shape of the work (why this kernel exists next to k_node_layer): per node
// the chain is 4-5 dependent Linear layers of H x 2H / H x H; with 32 nodes
// per wave and all H units in one wave (k_node_layer) a 2k-particle graph has
// 63 waves on 1,024 SIMDs and each walks 320 dependent 64-cycle MFMAs.  Here a
// workgroup owns 16 nodes and its 4 waves split the H = 64 output units (16
// each), so every Linear is 16 (K = 64) or 32 (K = 128) 32-cycle MFMAs per
// wave, a 2k graph runs on 500 waves, and the weights of a wave's 16 output
// rows live in VGPRs for the whole launch (no LDS staging pass).
//
// Layout ("items on lanes", 16x16x4): lane l = (item j = l & 15, group g =
// l >> 4).  D[unit][item]: lane holds units 16 b + 4 g + (0..3) of item j
// (b = wave).  A Linear's K order is 16 q + 4 g + c for the c-th component of
// the q-th float4, so both operands are float4 rows: W[16 b + j][16 q + 4 g ..]
// and In[j][16 q + 4 g ..].  Between Linears the waves exchange their unit
// blocks through LDS ([16 items][H + 4]) with one barrier.
#include "common.h"
#include "fwd16.h"
#include "radius_small.h"
#include "sgnn_internal.h"

#include "fwd16_dev.h"

namespace {


template <int NL, int MODE>
SGNN_DEV void node_tail(const Node16Args& a, const NodeW<NL, MODE>& W, float (*bufs)[16 * LDX], int64_t i,
                        bool valid, f32x4 h, f32x4 xo, int b, int j, int g);

template <int NL, int MODE>
SGNN_DEV void node_tile(const Node16Args& a, const NodeW<NL, MODE>& W, float (*bufs)[16 * LDX], int64_t i,
                        bool valid, const f32x4 (&ag)[KQ], const f32x4 (&xr)[KQ], f32x4 xo, int b, int j,
                        int g) {
  const f32x4 h = relu4(mm_cat(W.vb1, W.w1a, ag, W.w1x, xr));  // graph_network.py:220
  node_tail<NL, MODE>(a, W, bufs, i, valid, h, xo, b, j, g);
}

// From the first Linear's post-ReLU output h (own units) on: (middle Linear),
// last Linear, LayerNorm, + xo (residual; zero in the encoder) -> x_out, then
// u/v (mode 0) or decoder + integrator (mode 1).
template <int NL, int MODE>
SGNN_DEV void node_tail(const Node16Args& a, const NodeW<NL, MODE>& W, float (*bufs)[16 * LDX], int64_t i,
                        bool valid, f32x4 h, f32x4 xo, int b, int j, int g) {
  const int ucol = 16 * b + 4 * g;
  f32x4 hr[KQ], yr[KQ];
  xchg(bufs[0], j, ucol, g, h, hr);
  f32x4 y;
  if constexpr (NL == 3) {
    f32x4 mr[KQ];
    xchg(bufs[1], j, ucol, g, relu4(mm(W.vbm, W.wm, hr)), mr);
    y = mm(W.vb2, W.w2, mr);
  } else {
    y = mm(W.vb2, W.w2, hr);
  }
  xchg(bufs[2], j, ucol, g, y, yr);
  float mean, rstd;
  ln_stats(yr, mean, rstd);
  f32x4 xn;
#pragma unroll
  for (int c = 0; c < 4; ++c) xn[c] = (y[c] - mean) * rstd * W.vg[c] + W.vbb[c] + xo[c];  // LN (+ :176 residual)
  if (valid && a.x_out) st4(a.x_out + i * H + ucol, xn);
  f32x4 xnr[KQ];
  xchg(bufs[3], j, ucol, g, xn, xnr);
  if constexpr (MODE == 0) {
    const f32x4 u = mm(W.vba, W.wa, xnr);
    const f32x4 v = mm(zero4(), W.wb, xnr);
    if (valid) {
      st4(a.u + i * H + ucol, u);
      st4(a.v + i * H + ucol, v);
    }
  } else {
    f32x4 hdr[KQ];
    xchg(bufs[4], j, ucol, g, relu4(mm(W.vba, W.wa, xnr)), hdr);
    if constexpr (NL == 3) {
      f32x4 hd2r[KQ];
      xchg(bufs[5], j, ucol, g, relu4(mm(W.vbmd, W.wmd, hdr)), hd2r);
#pragma unroll
      for (int q = 0; q < KQ; ++q) hdr[q] = hd2r[q];
    }
    const int D = a.dim;
    if (b == 0) {
      const f32x4 o = mm(W.vbo, W.wb, hdr);  // lanes g == 0 hold outputs 0..3
      if (valid && g == 0) {
#pragma unroll
        for (int c = 0; c < 4; ++c)
          if (c <= D) a.pred[i * (D + 1) + c] = comp(o, c);
        if (a.pos_seq) {  // learned_simulator.py:398-411
          const float* p = a.pos_seq + i * a.T * D;
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
      }
    } else if (b == 1 && g == 0 && valid && a.pos_seq && a.window_out) {  // evaluate.py:136-139
      const float* p = a.pos_seq + i * a.T * D;
      float* w = a.window_out + i * a.T * D;
      for (int k = 0; k < (a.T - 1) * D; ++k) w[k] = p[k + D];
    }
  }
}

template <int NL, int MODE>
__global__ __launch_bounds__(kBlock16) void k_node16(Node16Args a) {
  __shared__ float xb[kBufs][16 * LDX];
  const int l = lane_id(), j = l & 15, g = l >> 4, b = wave_id();
  NodeW<NL, MODE> W;
  W.load(a, b, j, g);
  for (int64_t tile = blockIdx.x; tile * 16 < a.n; tile += gridDim.x) {
    const int64_t i = tile * 16 + j;
    const bool valid = i < a.n;
    f32x4 ag[KQ], xr[KQ], xo;
    load_agg16(ag, a, valid ? i : a.n - 1, g);
    load_x16(a, valid ? i : 0, b, g, xr, xo);
    node_tile<NL, MODE>(a, W, xb, i, valid, ag, xr, xo, b, j, g);
  }
}

// ---------------------------------------------------------------------------
// Fused layer (edge MLP -> receiver sums in LDS -> node update), see fwd16.h.


// WPE: waves per SIMD the register allocation is sized for -- 2 (<= 256
// VGPRs, two workgroups per CU) or 1 (the whole register file, no spills) for
// grids of <= 256 workgroups, which hold one workgroup per CU anyway.
template <int NL, int MODE, bool FIRST, int WPE = 2>
__global__ __launch_bounds__(kBlock16) __attribute__((amdgpu_waves_per_eu(WPE))) void k_layer16(sgnn::Layer16Args a) {
  // LDS: edge MLP weights (W1e pre-scaled by 2^k, exact) and per-wave
  // receiver sums; the node phase's exchange buffers alias the sums (barriers
  // separate the phases).  FIRST adds the edge encoder's last Linear.
  constexpr int NW = NL == 3 ? 3 : 2;
  constexpr int NB = (NL == 3 || MODE == 1) ? kBufs : 4;  // node_tail touches buffers 0, 2, 3 at NL 2, mode 0
  __shared__ float sw[NW][H * LDX];
  __shared__ float svec[4][H];                    // b2, gamma, beta, bm
  __shared__ float scratch[NB * 16 * LDX];  // per-wave receiver sums; = xb in the node phase
  __shared__ float sxw[FIRST ? H * LDX : 4];      // encoder W2 (FIRST)
  __shared__ float sxv[FIRST ? 4 : 1][H];         // encoder b1, b2, gamma, beta (FIRST)
  __shared__ int32_t lsend[FIRST ? 16 * 32 : 1], lrecv[FIRST ? 16 * 32 : 1];  // lists mode: the tile's CSR
  __shared__ int32_t lpre[FIRST ? 17 : 1], lred[FIRST ? kWaves16 : 1];
  static_assert(NB >= kWaves16, "the per-wave sums fit the node buffers");
  float* sums_all = scratch;
  auto xb = reinterpret_cast<float (*)[16 * LDX]>(scratch);
  const Node16Args& nd = a.nd;
  const int l = lane_id(), j = l & 15, g = l >> 4, b = wave_id();
  const int NT = a.nt;
  // the first tile's edge range and first half are requested before the
  // weight staging, so their dependent loads overlap it
  int64_t tile = blockIdx.x;
  int32_t ea = 0, eb = 0;
  int r_n = 0, s_n = 0;
  f32x4 x_n[KQ], uv_n[KQ];
  float ps_n[3] = {0.0f, 0.0f, 0.0f}, pr_n[3] = {0.0f, 0.0f, 0.0f};
  const bool lists = FIRST && a.l_deg != nullptr;
  auto load_half = [&](int32_t hs) {  // indices, e0 row (FIRST: both positions), u[recv] + v[send]
    const int32_t e = hs + j;
    const int32_t ec = e < eb ? e : eb - 1;
    if (FIRST && lists) {
      r_n = lrecv[ec - ea];
      s_n = lsend[ec - ea];
    } else {
      r_n = a.recv[ec];
      s_n = a.send[ec];
    }
    SGNN_BOUNDS(r_n, 0, nd.n, "layer16 receiver");
    SGNN_BOUNDS(s_n, 0, nd.n, "layer16 sender");
    if constexpr (FIRST) {
#pragma unroll
      for (int c = 0; c < 3; ++c)
        if (c < a.dim) {
          ps_n[c] = a.pos[(int64_t)s_n * a.pos_stride + c];
          pr_n[c] = a.pos[(int64_t)r_n * a.pos_stride + c];
        }
    } else {
#pragma unroll
      for (int q = 0; q < KQ; ++q) x_n[q] = ld_e0_edge(a.e0t, ec, q, g);
    }
#pragma unroll
    for (int t = 0; t < KQ; ++t)
      uv_n[t] = ld4(a.u_in + (int64_t)r_n * H + 16 * t + 4 * g) + ld4(a.v_in + (int64_t)s_n * H + 16 * t + 4 * g);
  };
  // lists mode (FIRST, one tile per workgroup): the tile's CSR rows from the
  // radius search's padded lists -- row start = sum of deg over the earlier
  // rows (a workgroup reduction), the rows compacted into LDS and written out
  auto build_tile_csr = [&](int64_t i0) {
    const int cnt = (int)min<int64_t>(NT, nd.n - i0);
    int part = 0;
    for (int64_t k = threadIdx.x; k < i0; k += kBlock16) part += a.l_deg[k];
    const int dg = b == 0 && l < cnt ? a.l_deg[i0 + l] : 0;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) part += __shfl_xor(part, o, 64);
    if (l == 0) lred[b] = part;
    __syncthreads();
    if (b == 0) {
      int base = 0;
#pragma unroll
      for (int w = 0; w < kWaves16; ++w) base += lred[w];
      int incl = dg;
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) {
        const int t = __shfl_up(incl, o, 64);
        if (l >= o) incl += t;
      }
      if (l < 16) lpre[l + 1] = base + incl;
      if (l == 0) lpre[0] = base;
    }
    __syncthreads();
    const int base = lpre[0];
    for (int t = threadIdx.x; t < cnt * a.l_cap; t += kBlock16) {
      const int k = t / a.l_cap, q = t - k * a.l_cap;
      const int r0 = lpre[k];
      if (q < lpre[k + 1] - r0) {
        int32_t sv = a.l_nbr[(i0 + k) * a.l_cap + q];
        SGNN_BOUNDS(sv, 0, nd.n, "layer16 padded-list sender");
        int slot = r0 - base + q;
        SGNN_BOUNDS(slot, 0, 16 * 32, "layer16 tile CSR slot");
        lsend[slot] = sv;
        lrecv[slot] = (int32_t)(i0 + k);
        a.send_out[r0 + q] = sv;
        a.recv_out[r0 + q] = (int32_t)(i0 + k);
      }
    }
    if (threadIdx.x < cnt) a.rowptr_out[i0 + threadIdx.x] = lpre[threadIdx.x];
    if (threadIdx.x == 0 && i0 + cnt == nd.n) a.rowptr_out[nd.n] = lpre[cnt];
    __syncthreads();
    ea = base;
    eb = lpre[cnt];
  };
  auto start_tile = [&](int64_t tl) {
    const int64_t i0 = tl * NT;
    if (FIRST && lists) {
      build_tile_csr(i0);
    } else {
      ea = nd.rowptr[i0];
      eb = nd.rowptr[min<int64_t>(i0 + NT, nd.n)];
    }
    if (ea + 16 * b < eb) load_half(ea + 16 * b);
  };
  f32x4 st0[kStagePer], st1[kStagePer], st2[kStagePer];
  stage_w64_load(st0, a.ewe, 3 * H);
  if (NL == 3) stage_w64_load(st1, a.ewm, H);
  stage_w64_load(st2, a.ew2, H);
  if (tile * NT < nd.n) start_tile(tile);
  stage_w64_store(sw[0], st0, a.e_scale);
  if (NL == 3) stage_w64_store(sw[1], st1, 1.0f);
  stage_w64_store(sw[NW - 1], st2, 1.0f);
  stage_vec(svec[0], a.eb2, H, H);
  stage_vec(svec[1], a.eg, H, H);
  stage_vec(svec[2], a.ebb, H, H);
  stage_vec(svec[3], a.ebm, H, H);
  float xw1[KQ] = {0.0f, 0.0f, 0.0f, 0.0f};  // FIRST: encoder W1 [H][dim + 1], unit 16 t + j, k = g
  if constexpr (FIRST) {
    f32x4 sx[kStagePer];
    stage_w64_load(sx, a.xw2, H);
    stage_w64_store(sxw, sx, 1.0f);
    stage_vec(sxv[0], a.xb1, H, H);
    stage_vec(sxv[1], a.xb2, H, H);
    stage_vec(sxv[2], a.xg, H, H);
    stage_vec(sxv[3], a.xbb, H, H);
#pragma unroll
    for (int t = 0; t < KQ; ++t) xw1[t] = g <= a.dim ? a.xw1[(16 * t + j) * (a.dim + 1) + g] : 0.0f;
  }
  NodeW<NL, MODE> NWt;
  NWt.load(nd, b, j, g);
  float* sums = sums_all + b * 16 * LDX;
  for (; tile * NT < nd.n; tile += gridDim.x) {
    __syncthreads();  // staging done / the previous node phase no longer reads the scratch
#pragma unroll
    for (int q = 0; q < KQ; ++q) st4(sums + j * LDX + 16 * q + 4 * g, zero4());
    const int64_t i0 = tile * NT;
    const int64_t i = i0 + j;
    const bool valid = j < NT && i < nd.n;
    f32x4 xr[KQ], xo;  // the node phase's x rows, requested now
    load_x16(nd, valid ? i : 0, b, g, xr, xo);
    // edge phase: wave b takes the 16-edge halves b, b + 4, ... of the tile's
    // receivers' (contiguous) edge range, all H units per wave, no barriers
    for (int32_t hs = ea + 16 * b; hs < eb; hs += 16 * kWaves16) {
      const bool ev = hs + j < eb;
      const int r = r_n;
      f32x4 x[KQ], acc[KQ];
      float ps[3], pr[3];
#pragma unroll
      for (int q = 0; q < KQ; ++q) {
        x[q] = x_n[q];
        acc[q] = uv_n[q];
      }
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        ps[c] = ps_n[c];
        pr[c] = pr_n[c];
      }
      if (hs + 16 * kWaves16 < eb) load_half(hs + 16 * kWaves16);
      if constexpr (FIRST) {
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
        // Encoder.edge_fn: Linear(dim + 1, H) -> ReLU -> Linear(H, H) -> LayerNorm
        f32x4 hx[KQ], y[KQ];
#pragma unroll
        for (int t = 0; t < KQ; ++t) {
          hx[t] = relu4(mfma16(xw1[t], fg, ld4(sxv[0] + 16 * t + 4 * g)));
          y[t] = ld4(sxv[1] + 16 * t + 4 * g);
        }
        mm_full(y, sxw, hx, j, g);
        float mu, rs;
        ln_stats(y, mu, rs);
        const int32_t e = hs + j;
        float* et = a.e0t_out + (int64_t)(e >> 5) * (32 * H);
#pragma unroll
        for (int t = 0; t < KQ; ++t) {
          const f32x4 ga = ld4(sxv[2] + 16 * t + 4 * g), be = ld4(sxv[3] + 16 * t + 4 * g);
#pragma unroll
          for (int c = 0; c < 4; ++c) x[t][c] = (y[t][c] - mu) * rs * ga[c] + be[c];
          if (ev) {  // e0 for the later layers, 32-edge tiled layout (ld_e0_edge's address)
            const int tt = t >> 1, gg = 2 * (t & 1) + (g >> 1), hh = g & 1;
            st4(et + (tt * 4 + gg) * 256 + ((e & 31) + 32 * hh) * 4, x[t]);
          }
        }
      }
      // first Linear: u[recv] + v[send] + 2^k W1_e e0 (graph_network.py:197 on cat[x_i, x_j, e])
      mm_full(acc, sw[0], x, j, g);
#pragma unroll
      for (int t = 0; t < KQ; ++t) x[t] = relu4(acc[t]);
      if constexpr (NL == 3) {
#pragma unroll
        for (int t = 0; t < KQ; ++t) acc[t] = ld4(svec[3] + 16 * t + 4 * g);
        mm_full(acc, sw[1], x, j, g);
#pragma unroll
        for (int t = 0; t < KQ; ++t) x[t] = relu4(acc[t]);
      }
#pragma unroll
      for (int t = 0; t < KQ; ++t) acc[t] = ld4(svec[0] + 16 * t + 4 * g);
      mm_full(acc, sw[NW - 1], x, j, g);
      float mu, rs;
      ln_stats(acc, mu, rs);
      f32x4 m[KQ];
#pragma unroll
      for (int t = 0; t < KQ; ++t) {
        const f32x4 ga = ld4(svec[1] + 16 * t + 4 * g), be = ld4(svec[2] + 16 * t + 4 * g);
#pragma unroll
        for (int c = 0; c < 4; ++c) m[t][c] = (acc[t][c] - mu) * rs * ga[c] + be[c];
      }
      // receiver runs of the half (recv sorted along the 16-lane rows):
      // segmented inclusive scan with DPP row shifts, then the last lane of
      // each run adds its total to the receiver's row of this wave's sums
      const int rk = ev ? r : -1 - j;  // padding lanes: runs of their own
#pragma unroll
      for (int d = 1; d < 16; d <<= 1) {
        const int pr = dpp_row_shr(rk, d, INT32_MIN);
#pragma unroll
        for (int t = 0; t < KQ; ++t)
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            const float pv = __int_as_float(dpp_row_shr(__float_as_int(m[t][c]), d, 0));
            m[t][c] = pr == rk ? m[t][c] + pv : m[t][c];
          }
      }
      const int rn = dpp_row_shl1(rk, INT32_MIN);
      if (ev && rn != rk) {
        float* dst = sums + (r - (int)i0) * LDX + 4 * g;
#pragma unroll
        for (int t = 0; t < KQ; ++t) st4(dst + 16 * t, ld4(dst + 16 * t) + m[t]);
      }
    }
    __syncthreads();
    if ((tile + gridDim.x) * NT < nd.n) start_tile(tile + gridDim.x);  // overlaps the node phase
    // node phase: the messages summed over the waves in a fixed order
    f32x4 ag[KQ];
#pragma unroll
    for (int q = 0; q < KQ; ++q) {
      ag[q] = ld4(sums_all + j * LDX + 16 * q + 4 * g);
#pragma unroll
      for (int w = 1; w < kWaves16; ++w) ag[q] += ld4(sums_all + w * 16 * LDX + j * LDX + 16 * q + 4 * g);
    }
    __syncthreads();  // the node buffers alias the sums
    node_tile<NL, MODE>(nd, NWt, xb, i, valid, ag, xr, xo, b, j, g);
  }
}

// ---------------------------------------------------------------------------
// Encoders (inference).

// The encoder's weights of one wave's 16 output rows (resident for the launch).
template <int NL, int KQF>
struct EncNodeW {
  NodeW<NL, 0> W;
  f32x4 w1f[KQF];  // first Linear [H][feat] (feat not a multiple of 4: scalar loads)
  f32x4 vb1;
  SGNN_DEV void load(const sgnn::EncNode16Args& a, int b, int j, int g) {
    const int urow = 16 * b + j, ucol = 16 * b + 4 * g;
    W.load_tail(a.nd, b, j, g);
#pragma unroll
    for (int q = 0; q < KQF; ++q)
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int f = 16 * q + 4 * g + c;
        w1f[q][c] = f < a.feat ? a.w1[(int64_t)urow * a.feat + f] : 0.0f;
      }
    vb1 = ld4(a.b1 + ucol);
  }
};

// Node features -> Encoder.node_fn -> x0, u, v of the 16 nodes of `tile`
// (a tile past the end runs with every row invalid: the barriers of node_tail
// stay matched across the waves that share `xb`).
template <int NL, int KQF>
SGNN_DEV void enc_node16_tile(const sgnn::EncNode16Args& a, const EncNodeW<NL, KQF>& E, float (*xb)[16 * LDX],
                              int64_t tile, int b, int j, int g) {
  const Node16Args& nd = a.nd;
  const int D = a.dim, nvel = (a.T - 1) * D;
  const int64_t i = tile * 16 + j;
  const bool valid = i < nd.n;
  const int64_t ic = valid ? i : nd.n - 1;
  const float* p = a.pos_seq + ic * a.T * D;
  f32x4 xf[KQF];
#pragma unroll
  for (int q = 0; q < KQF; ++q)
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int f = 16 * q + 4 * g + c;
      float val = 0.0f;
      if (f < nvel) {  // learned_simulator.py:258,272-278 normalised velocity history
        const int t = f / D, cc = f - t * D;
        const float vel = __fsub_rn(p[(t + 1) * D + cc], p[t * D + cc]);
        val = __fdiv_rn(__fsub_rn(vel, a.vel_mean[cc]), a.vel_std[cc]);
      } else if (f == nvel) {  // :282-284 wall distance
        val = __fdiv_rn(fminf(fmaxf(__fadd_rn(p[(a.T - 1) * D], 2.0f), 0.0f), a.wall_max), a.wall_div);
      } else if (a.use_emb && f < nvel + 1 + a.emb_dim) {  // :287-290 type embedding
        val = a.emb_w[a.types[ic] * a.emb_dim + (f - nvel - 1)];
      }
      xf[q][c] = val;
    }
  const f32x4 h = relu4(mm(E.vb1, E.w1f, xf));
  node_tail<NL, 0>(nd, E.W, xb, i, valid, h, zero4(), b, j, g);
}

template <int NL, int KQF>
__global__ __launch_bounds__(kBlock16) void k_enc_node16(sgnn::EncNode16Args a) {
  __shared__ float xb[kBufs][16 * LDX];
  const int l = lane_id(), j = l & 15, g = l >> 4, b = wave_id();
  EncNodeW<NL, KQF> E;
  E.load(a, b, j, g);
  for (int64_t tile = blockIdx.x; tile * 16 < a.nd.n; tile += gridDim.x) enc_node16_tile<NL, KQF>(a, E, xb, tile, b, j, g);
}

// The small-graph radius search (radius_small.h) and the node encoder in ONE
// launch: the two are independent (the encoder reads only the position
// window), and each alone is a few microseconds of latency on a fraction of
// the chip.  Workgroups [0, rgrid) run the radius body; the others run the
// encoder with two 16-node tiles per workgroup (waves 0-3 and 4-7, each half
// with its own exchange buffers).
template <int DIM, int NL, int KQF>
__global__ __launch_bounds__(sgnn::kSmallBlock) void k_radius_enc16(sgnn::RadiusSmallArgs r, sgnn::EncNode16Args a,
                                                                    int rgrid) {
  extern __shared__ float lds[];
  if ((int)blockIdx.x < rgrid) {
    sgnn::radius_small_body<DIM>(r, lds, blockIdx.x, rgrid);
    return;
  }
  const int l = lane_id(), j = l & 15, g = l >> 4, w = wave_id(), half = w >> 2, b = w & 3;
  auto xb = reinterpret_cast<float (*)[16 * LDX]>(lds) + half * kBufs;
  EncNodeW<NL, KQF> E;
  E.load(a, b, j, g);
  const int64_t pairs = gridDim.x - rgrid;
  for (int64_t pr = blockIdx.x - rgrid; pr * 32 < a.nd.n; pr += pairs) enc_node16_tile<NL, KQF>(a, E, xb, 2 * pr + half, b, j, g);
}

}  // namespace

namespace sgnn {

int node16_launch(const Node16Args& a, int mode, int nl, hipStream_t s) {
  if (a.n <= 0) return SGNN_OK;
  const int64_t tiles = (a.n + 15) / 16;
  const unsigned grid = (unsigned)std::min<int64_t>(tiles, 256 * 4);
  if (mode == 0 && nl == 2) hipLaunchKernelGGL((k_node16<2, 0>), dim3(grid), dim3(kBlock16), 0, s, a);
  else if (mode == 0) hipLaunchKernelGGL((k_node16<3, 0>), dim3(grid), dim3(kBlock16), 0, s, a);
  else if (nl == 2) hipLaunchKernelGGL((k_node16<2, 1>), dim3(grid), dim3(kBlock16), 0, s, a);
  else hipLaunchKernelGGL((k_node16<3, 1>), dim3(grid), dim3(kBlock16), 0, s, a);
  return check_launch("node_layer16");
}

int layer16_launch(const Layer16Args& a, int mode, int nl, hipStream_t s, bool first) {
  if (a.nd.n <= 0) return SGNN_OK;
  if (a.nt < 1 || a.nt > 16) return set_error(SGNN_ERR_INVALID, "layer16: nodes per tile must be 1..16");
  if (first && (mode != 0 || nl != 2))
    return set_error(SGNN_ERR_UNSUPPORTED, "layer16: the fused edge encoder needs nmlp_layers 1 and a later layer");
  const int64_t tiles = (a.nd.n + a.nt - 1) / a.nt;
  const unsigned grid = (unsigned)std::min<int64_t>(tiles, 512);
  if (a.l_deg && (!first || tiles > 512 || a.l_cap < 1 || a.l_cap > 32 || !a.l_nbr || !a.rowptr_out ||
                  !a.send_out || !a.recv_out))
    return set_error(SGNN_ERR_INVALID, "layer16: CSR from the padded lists needs the first layer, <= 512 tiles, "
                                       "cap <= 32");
  // one workgroup per CU: the whole register file (no spills; C1 r = 15 0.1222 -> 0.1184 ms/step,
  // r = 0.6 0.0845 -> 0.081)
  // (measured slower past 256 workgroups, one per CU in two rounds: 4,800 particles 0.155 -> 0.173,
  // 8,000 0.217 -> 0.242 ms/step)
  if (grid <= 256) {
    if (first) hipLaunchKernelGGL((k_layer16<2, 0, true, 1>), dim3(grid), dim3(kBlock16), 0, s, a);
    else if (mode == 0 && nl == 2) hipLaunchKernelGGL((k_layer16<2, 0, false, 1>), dim3(grid), dim3(kBlock16), 0, s, a);
    else if (mode == 0) hipLaunchKernelGGL((k_layer16<3, 0, false, 1>), dim3(grid), dim3(kBlock16), 0, s, a);
    else if (nl == 2) hipLaunchKernelGGL((k_layer16<2, 1, false, 1>), dim3(grid), dim3(kBlock16), 0, s, a);
    else hipLaunchKernelGGL((k_layer16<3, 1, false, 1>), dim3(grid), dim3(kBlock16), 0, s, a);
    return check_launch("layer16");
  }
  if (first) hipLaunchKernelGGL((k_layer16<2, 0, true>), dim3(grid), dim3(kBlock16), 0, s, a);
  else if (mode == 0 && nl == 2) hipLaunchKernelGGL((k_layer16<2, 0, false>), dim3(grid), dim3(kBlock16), 0, s, a);
  else if (mode == 0) hipLaunchKernelGGL((k_layer16<3, 0, false>), dim3(grid), dim3(kBlock16), 0, s, a);
  else if (nl == 2) hipLaunchKernelGGL((k_layer16<2, 1, false>), dim3(grid), dim3(kBlock16), 0, s, a);
  else hipLaunchKernelGGL((k_layer16<3, 1, false>), dim3(grid), dim3(kBlock16), 0, s, a);
  return check_launch("layer16");
}

int enc_node16_launch(const EncNode16Args& a, int nl, hipStream_t s) {
  if (a.nd.n <= 0) return SGNN_OK;
  const int kqf = (a.feat + 15) / 16;
  if (kqf > 3) return set_error(SGNN_ERR_UNSUPPORTED, "encode_nodes16: more than 48 node features");
  const unsigned grid = (unsigned)std::min<int64_t>((a.nd.n + 15) / 16, 256 * 4);
#define SGNN_ENC16(NL_, KQF_) hipLaunchKernelGGL((k_enc_node16<NL_, KQF_>), dim3(grid), dim3(kBlock16), 0, s, a)
  if (nl == 2) {
    if (kqf == 1) SGNN_ENC16(2, 1); else if (kqf == 2) SGNN_ENC16(2, 2); else SGNN_ENC16(2, 3);
  } else {
    if (kqf == 1) SGNN_ENC16(3, 1); else if (kqf == 2) SGNN_ENC16(3, 2); else SGNN_ENC16(3, 3);
  }
#undef SGNN_ENC16
  return check_launch("encode_nodes16");
}

int radius_enc16_launch(const RadiusSmallArgs& r, const EncNode16Args& a, int nl, hipStream_t s, bool csr) {
  const int kqf = (a.feat + 15) / 16;
  if (kqf > 3) return set_error(SGNN_ERR_UNSUPPORTED, "encode_nodes16: more than 48 node features");
  if (r.n != a.nd.n) return set_error(SGNN_ERR_INVALID, "radius_enc16: particle counts differ");
  // one workgroup per CU: at ~186 VGPRs (the encoder's resident weights) a CU holds one 8-wave
  // workgroup, so a grid past 256 would run a second round; the radius queries (cheap next to the
  // position staging every workgroup pays) take the CUs the encoder's 32-node pairs leave
#ifndef SGNN_MERGE_EGRID
#define SGNN_MERGE_EGRID 128
#endif
  const int egrid = (int)std::min<int64_t>((a.nd.n + 31) / 32, SGNN_MERGE_EGRID);
  const int rgrid = (int)std::max<int64_t>(1, std::min<int64_t>((r.n + 7) / 8, 256 - egrid));
  const size_t lds = std::max(radius_small_lds(r.n, r.dim), sizeof(float) * 2 * kBufs * 16 * LDX);
  auto go = [&](auto kern) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)std::max(radius_small_lds(kSmallN, 3), sizeof(float) * 2 * kBufs * 16 * LDX));
    hipLaunchKernelGGL(kern, dim3((unsigned)(rgrid + egrid)), dim3(kSmallBlock), lds, s, r, a, rgrid);
  };
#define SGNN_RE16(D_)                                                   \
  do {                                                                  \
    if (nl == 2) {                                                      \
      if (kqf == 1) go(k_radius_enc16<D_, 2, 1>);                       \
      else if (kqf == 2) go(k_radius_enc16<D_, 2, 2>);                  \
      else go(k_radius_enc16<D_, 2, 3>);                                \
    } else {                                                            \
      if (kqf == 1) go(k_radius_enc16<D_, 3, 1>);                       \
      else if (kqf == 2) go(k_radius_enc16<D_, 3, 2>);                  \
      else go(k_radius_enc16<D_, 3, 3>);                                \
    }                                                                   \
  } while (0)
  if (r.dim == 1) SGNN_RE16(1);
  else if (r.dim == 2) SGNN_RE16(2);
  else SGNN_RE16(3);
#undef SGNN_RE16
  int st = check_launch("radius_enc16");
  if (st || !csr) return st;
  return radius_small_csr(r, s);
}

}  // namespace sgnn
