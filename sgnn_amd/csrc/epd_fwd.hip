// Encode-Process-Decode forward for gfx950 (fp32 MFMA v_mfma_f32_32x32x2_f32).
//
// Replaces, per step, the PyG/torch op chain of
//   sgnn/single_scale/learned_simulator.py:231-316 (features),
//   sgnn/single_scale/graph_network.py:86-96 (Encoder), :150-222 (L x
//   InteractionNetwork), :321-333 (Decoder) and learned_simulator.py:381-411
//   (Euler integrator)
// with 2 + 2L launches:
//   k_encode_nodes  features -> node MLP+LN -> x0, and layer-0 u/v
//   k_encode_edges  edge features -> edge MLP+LN -> e0 (tiled layout)
//   per layer k:
//     k_edge_layer  gather u[recv] + v[send] + 2^k W1e e0 -> ReLU -> W2 -> LN
//                   -> wave-segmented sum over the receiver-sorted CSR
//     k_node_layer  [agg, x] -> MLP+LN -> residual, then the NEXT layer's
//                   u/v projections, or (last layer) decoder + integrator.
//
// The edge MLP's first Linear is split by input block (x_i | x_j | e):
// W1 [x_i; x_j; e] = (W1_i x)[recv] + (W1_j x)[send] + W1_e e, so the two
// node blocks are computed once per NODE (u, v) instead of once per edge:
// the per-edge work drops from 3H^2+H^2 to H^2+H^2 multiply-adds.
#include "common.h"
#include "../../include/sgnn.h"
#include "sgnn_internal.h"
#include "fwd16.h"
#include "radius_small.h"

namespace {

constexpr int kBlock = 256;  // 4 waves; each wave owns 32 items at a time
constexpr int kWaves = kBlock / 64;

struct EncNodeArgs {
  const float* pos_seq;
  int64_t n;
  int T, dim;
  const int64_t* types;
  const float* emb_w;
  int emb_dim, use_emb;
  const float* vel_mean;
  const float* vel_std;
  float radius;
  int feat;  // number of real node features
  const float *w1, *b1, *w2, *b2, *g, *bb;  // encoder node MLP (w2/b2 = LAST Linear)
  const float *wm, *bm;                     // middle Linear (nlin = 3) or null
  float wall_max, wall_div;                 // clamp(x+2, 0, wall_max) / wall_div
  const float *we, *be;                     // edge0 W1 [H][3H], b1
  float *x0, *u, *v;
  sgnn_saves sv;
  const float* feat_in;  // explicit node features [n][feat] (EncodeProcessDecode.forward) or null
};

template <int TH, bool G = false>
SGNN_DEV void store_uv(const float* Wi, const float* Wj, const float* b1e, int ldh,
                       const f32x16 (&x)[TH], float* u_row, float* v_row, bool valid) {
  f32x16 acc[TH];
  acc_bias<TH>(acc, b1e);
  mfma_from_acc<TH, TH, G>(acc, Wi, ldh, 0, x);
  if (valid) store_row_clayout<TH>(u_row, acc);
  acc_bias<TH>(acc, nullptr);
  mfma_from_acc<TH, TH, G>(acc, Wj, ldh, 0, x);
  if (valid) store_row_clayout<TH>(v_row, acc);
}

// GI / GJ: W1e_i / W1e_j read from L2 (buffer loads) instead of an LDS image.
template <int TH, bool GI, bool GJ>
SGNN_DEV void store_uv2(const float* Wi, int ldi, const float* Wj, int ldj, const float* b1e,
                        const f32x16 (&x)[TH], float* u_row, float* v_row, bool valid) {
  f32x16 acc[TH];
  acc_bias<TH>(acc, b1e);
  mfma_from_acc<TH, TH, GI>(acc, Wi, ldi, 0, x);
  if (valid) store_row_clayout<TH>(u_row, acc);
  acc_bias<TH>(acc, nullptr);
  mfma_from_acc<TH, TH, GJ>(acc, Wj, ldj, 0, x);
  if (valid) store_row_clayout<TH>(v_row, acc);
}

template <int TH, int TKF, bool TRAIN, int NL>
__global__ __launch_bounds__(kBlock) void k_encode_nodes(EncNodeArgs a) {
  constexpr bool GW = TH > 2;  // H = 128: weights read from L2 (460 KB/layer > LDS)
  constexpr int H = 32 * TH, ldf = 32 * TKF + 4;
  constexpr int ldh = GW ? H : H + 4, ldwe = GW ? 3 * H : H + 4;
  extern __shared__ float lds[];
  float* W1 = lds;
  float* sW = W1 + H * ldf;
  const float* W2 = GW ? a.w2 : sW;
  const float* Wi = GW ? a.we : sW + H * ldh;
  const float* Wj = GW ? a.we + H : sW + 2 * H * ldh;
  float* b1 = GW ? sW : sW + 3 * H * ldh;
  float* b2 = b1 + H;
  float* g = b2 + H;
  float* bb = g + H;
  float* b1e = bb + H;
  float* bm = b1e + H;
  stage_matrix(W1, ldf, a.w1, a.feat, H, a.feat, H, 32 * TKF);
  if (NL == 3) stage_vec(bm, a.bm, H, H);
  if (!GW) {
    stage_matrix(sW, ldh, a.w2, H, H, H, H, H);
    stage_matrix(sW + H * ldh, ldh, a.we, 3 * H, H, H, H, H);
    stage_matrix(sW + 2 * H * ldh, ldh, a.we + H, 3 * H, H, H, H, H);
  }
  stage_vec(b1, a.b1, H, H);
  stage_vec(b2, a.b2, H, H);
  stage_vec(g, a.g, H, H);
  stage_vec(bb, a.bb, H, H);
  stage_vec(b1e, a.be, H, H);
  __syncthreads();
  const int l = lane_id(), j = l & 31, h = l >> 5, w = wave_id();
  const int nvel = (a.T - 1) * a.dim;
  for (int64_t blk = blockIdx.x; blk * (32 * kWaves) < a.n; blk += gridDim.x) {
    const int64_t node0 = blk * (32 * kWaves) + 32 * w;
    if (node0 >= a.n) continue;
    const int64_t i = node0 + j;
    const bool valid = i < a.n;
    const int64_t ic = valid ? i : a.n - 1;
    const float* p = a.feat_in ? nullptr : a.pos_seq + ic * a.T * a.dim;
    f32x16 xf[TKF];
#pragma unroll
    for (int tk = 0; tk < TKF; ++tk)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int f = 32 * tk + crow(r, h);
        float val = 0.0f;
        if (a.feat_in) {  // explicit features (graph_network.py:403 Encoder input)
          if (f < a.feat) val = a.feat_in[ic * a.feat + f];
        } else if (f < nvel) {  // learned_simulator.py:258,272-278
          const int t = f / a.dim, c = f - t * a.dim;
          const float vel = __fsub_rn(p[(t + 1) * a.dim + c], p[t * a.dim + c]);
          val = __fdiv_rn(__fsub_rn(vel, a.vel_mean[c]), a.vel_std[c]);
        } else if (f == nvel) {  // :282-284
          val = __fdiv_rn(fminf(fmaxf(__fadd_rn(p[(a.T - 1) * a.dim], 2.0f), 0.0f), a.wall_max),
                          a.wall_div);
        } else if (a.use_emb && f < nvel + 1 + a.emb_dim) {  // :287-290
          val = a.emb_w[a.types[ic] * a.emb_dim + (f - nvel - 1)];
        }
        xf[tk][r] = val;
      }
    f32x16 hacc[TH];
    acc_bias<TH>(hacc, b1);
    mfma_from_acc<TH, TKF>(hacc, W1, ldf, 0, xf);
    acc_relu<TH>(hacc);
    if (TRAIN && valid) store_row_clayout<TH>(a.sv.h + i * H, hacc);
    f32x16 y[TH], h2[TH];
    mlp_tail<TH, NL, TH, GW>(y, h2, hacc, a.wm, H, bm, W2, ldh, b2);
    if (TRAIN && NL == 3 && valid) store_row_clayout<TH>(a.sv.h2 + i * H, h2);
    if (TRAIN) {
      f32x16 yh[TH];
      float rs;
      acc_layernorm_save<TH>(y, g, bb, yh, rs);
      if (valid) {
        store_row_clayout<TH>(a.sv.yhat + i * H, yh);
        if (h == 0) a.sv.rstd[i] = rs;
      }
    } else {
      acc_layernorm<TH>(y, g, bb);
    }
    if (valid) store_row_clayout<TH>(a.x0 + i * H, y);
    store_uv<TH, GW>(Wi, Wj, b1e, ldwe, y, a.u + i * H, a.v + i * H, valid);
  }
}

struct EncEdgeArgs {
  const float* pos;
  int64_t stride;
  int dim;
  float radius;
  const int32_t *rowptr, *send, *recv;
  int64_t n;
  const float *w1, *b1, *w2, *b2, *g, *bb;
  float* e0t;
  sgnn_saves sv;
  const float *wm, *bm;
  const float* efeat_in;  // explicit edge features [E][fe] in COO order, or null
  const int32_t* perm;    // CSR position -> COO edge id (with efeat_in)
  int fe;
};

template <int TH, bool TRAIN, int NL>
__global__ __launch_bounds__(kBlock) void k_encode_edges(EncEdgeArgs a) {
  constexpr bool GW = TH > 2;
  constexpr int H = 32 * TH, ldh = GW ? H : H + 4, ld1 = 5;
  extern __shared__ float lds[];
  float* W1 = lds;
  float* sW = W1 + H * ld1;
  const float* W2 = GW ? a.w2 : sW;
  float* b1 = GW ? sW : sW + H * ldh;
  float* b2 = b1 + H;
  float* g = b2 + H;
  float* bb = g + H;
  float* bm = bb + H;
  stage_matrix(W1, ld1, a.w1, a.dim + 1, H, a.dim + 1, H, 4);
  if (NL == 3) stage_vec(bm, a.bm, H, H);
  if (!GW) stage_matrix(sW, ldh, a.w2, H, H, H, H, H);
  stage_vec(b1, a.b1, H, H);
  stage_vec(b2, a.b2, H, H);
  stage_vec(g, a.g, H, H);
  stage_vec(bb, a.bb, H, H);
  __syncthreads();
  const int64_t E = a.rowptr[a.n];
  const int64_t ntiles = (E + 31) / 32;
  const int l = lane_id(), j = l & 31, h = l >> 5;
  const int64_t gw = (int64_t)blockIdx.x * kWaves + wave_id();
  const int64_t nw = (int64_t)gridDim.x * kWaves;
  for (int64_t tile = gw; tile < ntiles; tile += nw) {
    const int64_t e = tile * 32 + j;
    const int64_t ec = e < E ? e : E - 1;
    float f[4] = {0.0f, 0.0f, 0.0f, 0.0f};
    if (a.efeat_in) {  // explicit features (graph_network.py:403 Encoder input)
      const int64_t src = a.perm[ec];
      for (int c = 0; c < a.fe; ++c) f[c] = a.efeat_in[src * a.fe + c];
    } else {
      int64_t s = a.send[ec], r = a.recv[ec];
      SGNN_BOUNDS(s, 0, a.n, "encode_edges sender");
      SGNN_BOUNDS(r, 0, a.n, "encode_edges receiver");
      float ss = 0.0f;
      for (int c = 0; c < a.dim; ++c) {  // learned_simulator.py:299-312
        const float d = __fdiv_rn(__fsub_rn(a.pos[s * a.stride + c], a.pos[r * a.stride + c]), a.radius);
        f[c] = d;
        ss = __fadd_rn(ss, __fmul_rn(d, d));
      }
      f[a.dim] = sqrtf(ss);
    }
    f32x16 hacc[TH];
    acc_bias<TH>(hacc, b1);
    mfma_step<TH>(hacc, W1, ld1, h, h ? f[1] : f[0]);
    mfma_step<TH>(hacc, W1, ld1, 2 + h, h ? f[3] : f[2]);
    acc_relu<TH>(hacc);
    f32x16 y[TH], h2[TH];
    mlp_tail<TH, NL, TH, GW>(y, h2, hacc, a.wm, H, bm, W2, ldh, b2);
    if (TRAIN && NL == 3) store_tiled<TH>(a.sv.h2 + tile * (32 * H), h2);
    if (TRAIN) {
      f32x16 yh[TH];
      float rs;
      acc_layernorm_save<TH>(y, g, bb, yh, rs);
      store_tiled<TH>(a.sv.yhat + tile * (32 * H), yh);
      if (h == 0 && e < E) a.sv.rstd[e] = rs;
    } else {
      acc_layernorm<TH>(y, g, bb);
    }
    float* dst = a.e0t + tile * (32 * H) + l * 4;
#pragma unroll
    for (int t = 0; t < TH; ++t)
#pragma unroll
      for (int gg = 0; gg < 4; ++gg) {
        f32x4 v4;
#pragma unroll
        for (int c = 0; c < 4; ++c) v4[c] = y[t][4 * gg + c];
        st4(dst + (t * 4 + gg) * 256, v4);
      }
  }
}

struct EdgeLayerArgs {
  const float *u, *v, *e0t;
  float e_scale;
  const int32_t *rowptr, *send, *recv;
  int64_t n;
  const float *we, *w2, *b2, *g, *bb;  // we = edge W1 + 2H (ld 3H); w2 = LAST Linear
  float *agg, *cin, *cout;
  sgnn_saves sv;
  const float *wm, *bm;
};

template <int TH, bool TRAIN, int NL>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(TH > 2 ? 1 : 2)))
void k_edge_layer(EdgeLayerArgs a) {
  // W1e always sits in LDS (67.6 KB at H = 128, next to the per-wave sum
  // buffers); the last (and middle) Linear is an LDS image at H = 64 and
  // read from L2 at H = 128.
  constexpr bool GW = TH > 2;
  constexpr int H = 32 * TH, ldh = H + 4;            // ldh: LDS image leading dim
  constexpr int ldw2 = GW ? H : ldh;
  extern __shared__ float lds[];
  float* sW = lds;
  const float* We = sW;
  const float* W2 = GW ? a.w2 : sW + H * ldh;
  float* b2 = sW + (GW ? 1 : 2) * H * ldh;
  float* g = b2 + H;
  float* bb = g + H;
  float* bm = bb + H;
  float* mbuf = bm + (NL == 3 ? H : 0);  // per wave [32][ldh]
  if (NL == 3) stage_vec(bm, a.bm, H, H);
  // W1e staged pre-scaled by 2^k: (2^k W1e) e0 == W1e (2^k e0) bit for bit
  // (power-of-two scaling is exact), so the MFMA operands need no scaling.
  stage_matrix(sW, ldh, a.we, 3 * H, H, H, H, H, a.e_scale);
  if (!GW) stage_matrix(sW + H * ldh, ldh, a.w2, H, H, H, H, H);
  stage_vec(b2, a.b2, H, H);
  stage_vec(g, a.g, H, H);
  stage_vec(bb, a.bb, H, H);
  __syncthreads();
  const int l = lane_id(), j = l & 31, h = l >> 5, w = wave_id();
  float* ml = mbuf + w * 32 * ldh;
  const int64_t E = a.rowptr[a.n];
  const int64_t ntiles = (E + 31) / 32;
  // Tile order: XCD-aware grid stride.  Workgroups are dealt round-robin over
  // the 8 XCDs (blocks b and b + 8 share one L2); the logical id
  // (b % 8) * (nwg / 8) + b / 8 gives each XCD's waves a contiguous band of
  // consecutive tiles per round, so the u[recv] / v[send] rows a band gathers
  // (receivers and their lattice neighbours) stay in that XCD's L2 instead of
  // being fetched by all eight.  (Needs nwg % 8 == 0; the host rounds the grid.)
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int lg = (nwg % 8 == 0) ? (bid % 8) * (nwg / 8) + bid / 8 : bid;
  const int64_t nw = (int64_t)nwg * kWaves;
  const int64_t t_begin = (int64_t)lg * kWaves + w, t_end = ntiles;
  // Software pipeline: the next tile's indices and e0 are loaded while this
  // tile computes, and this tile's u[recv] / v[send] gathers are issued before
  // its W1e e0 product and added after it (the gather latency hides behind
  // its MFMAs).  H = 128 runs one workgroup per CU (LDS), so the wave may use
  // the whole register file for the prefetched operands.
  constexpr bool PF = true;
  int rv_n = 0, s_n = 0, nb_n = -1;  // int32: no widening right after the load
  f32x4 xg_n[TH * 4];
  auto fetch = [&](int64_t t) {
    const int64_t b = t * 32, ee = b + j;
    const int64_t ecc = ee < E ? ee : E - 1;
    rv_n = a.recv[ecc];
    s_n = a.send[ecc];
    SGNN_BOUNDS(rv_n, 0, a.n, "edge_layer receiver");
    SGNN_BOUNDS(s_n, 0, a.n, "edge_layer sender");
    // receivers around the tile: lane 0 reads the one before, lane 1 the one
    // after, as one divergent load (a uniform-address load goes to an SGPR at
    // once -- a wait on every gather in flight); read back with readlane
    const bool has = j == 0 ? b > 0 : b + 32 < E;
    nb_n = has ? a.recv[j == 0 ? b - 1 : b + 32] : -1;
    const float* src = a.e0t + t * (32 * H) + l * 4;
#pragma unroll
    for (int q = 0; q < TH * 4; ++q) xg_n[q] = ld4(src + q * 256);
  };
  if (PF && t_begin < t_end) fetch(t_begin);
  // drain the first tile's loads: the waitcnt pass merges this preheader
  // state into the loop header and would otherwise make every iteration wait
  // for its own freshly issued prefetch
  __builtin_amdgcn_s_waitcnt(0);
  for (int64_t tile = t_begin; tile < t_end; tile += nw) {
    const int64_t base = tile * 32;
    const int64_t e = base + j;
    const bool valid = e < E;
    if (!PF) fetch(tile);
    const int rv = rv_n, nb = nb_n;
    const int s = s_n;
    f32x4 xg[TH * 4];
#pragma unroll
    for (int q = 0; q < TH * 4; ++q) xg[q] = xg_n[q];
    f32x16 hacc[TH];
    if constexpr (PF) {
      f32x16 ur[TH], vr[TH];
      load_row_clayout<TH>(ur, a.u + (int64_t)rv * H);
      load_row_clayout<TH>(vr, a.v + (int64_t)s * H);
      if (tile + nw < t_end) fetch(tile + nw);
      zero_acc_regs<TH>(hacc);
      mfma_from_groups<TH, TH, false>(hacc, We, ldh, 0, xg, 1.0f);
#pragma unroll
      for (int t = 0; t < TH; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) hacc[t][r] += ur[t][r] + vr[t][r];
    } else {
      load_row_clayout<TH>(hacc, a.u + (int64_t)rv * H);
      add_row_clayout<TH>(hacc, a.v + (int64_t)s * H);
      mfma_from_groups<TH, TH, false>(hacc, We, ldh, 0, xg, 1.0f);
    }
    acc_relu<TH>(hacc);
    if (TRAIN) store_tiled<TH>(a.sv.h + tile * (32 * H), hacc);
    f32x16 y[TH], h2[TH];
    mlp_tail<TH, NL, TH, GW>(y, h2, hacc, a.wm, H, bm, W2, ldw2, b2);
    if (TRAIN && NL == 3 && a.sv.h2) store_tiled<TH>(a.sv.h2 + tile * (32 * H), h2);
    if (TRAIN) {
      f32x16 yh[TH];
      float rs;
      acc_layernorm_save<TH>(y, g, bb, yh, rs);
      if (a.sv.yhat) store_tiled<TH>(a.sv.yhat + tile * (32 * H), yh);   // (NULL: recomputed in the backward)
      if (h == 0 && valid) a.sv.rstd[e] = rs;
    } else {
      acc_layernorm<TH>(y, g, bb);
    }
#pragma unroll
    for (int t = 0; t < TH; ++t)
#pragma unroll
      for (int gg = 0; gg < 4; ++gg) {
        f32x4 v4;
#pragma unroll
        for (int c = 0; c < 4; ++c) v4[c] = y[t][4 * gg + c];
        st4(ml + j * ldh + 32 * t + 8 * gg + 4 * h, v4);
      }
    wave_lds_sync();
    // wave-segmented sum over the receiver-sorted CSR: lane = latent unit
    const int nvalid = (E - base) < 32 ? (int)(E - base) : 32;
    segment_sum_store<TH>(ml, ldh, rv, nvalid, base, tile, __builtin_amdgcn_readlane(nb, 0),
                          __builtin_amdgcn_readlane(nb, 1), a.agg, a.cin, a.cout);
    wave_lds_sync();
  }
}

struct NodeLayerArgs {
  const float *x_in, *agg, *cin, *cout;
  const int32_t* rowptr;
  int64_t n;
  const float *w1, *b1, *w2, *b2, *g, *bb;  // node MLP
  // mode 0: next-layer projections
  const float *we, *be;
  float *u, *v;
  // mode 1: decoder + integrator
  const float *wd1, *bd1, *wd2, *bd2;
  const float* pos_seq;
  int T, dim;
  const float *acc_mean, *acc_std;
  float *pred, *next_pos, *window_out;
  float* x_out;
  sgnn_saves sv;
  const float *wm, *bm;    // node MLP middle Linear (nlin = 3)
  const float *wdm, *bdm;  // decoder middle Linear (nlin = 3)
};

template <int TH>
SGNN_DEV void load_agg(f32x16 (&a)[TH], const NodeLayerArgs& p, int64_t i) {
  constexpr int H = 32 * TH;
  const int32_t r0 = p.rowptr[i], r1 = p.rowptr[i + 1];
  if (r1 <= r0) {
#pragma unroll
    for (int t = 0; t < TH; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) a[t][r] = 0.0f;
    return;
  }
  const int32_t t0 = r0 >> 5, t1 = (r1 - 1) >> 5;
  if (t0 == t1) {
    load_row_clayout<TH>(a, p.agg + i * H);
  } else {
    // head partial + every later tile's partial (a segment longer than 32
    // edges leaves whole-tile sums in cin of the tiles it spans)
    load_row_clayout<TH>(a, p.cout + (int64_t)t0 * H);
    for (int32_t t = t0 + 1; t <= t1; ++t) add_row_clayout<TH>(a, p.cin + (int64_t)t * H);
  }
}

template <int TH, int MODE, bool TRAIN, int NL>
__global__ __launch_bounds__(kBlock) void k_node_layer(NodeLayerArgs a) {
  constexpr bool GW = TH > 2;
  constexpr int H = 32 * TH, ldh = H + 4;
  constexpr int ld2 = GW ? 2 * H : 2 * H + 4, ldw2 = GW ? H : ldh;
  constexpr int lda = GW ? (MODE == 0 ? 3 * H : H) : ldh;
  extern __shared__ float lds[];
  float* sW = lds;
  // LDS: [W1 | W2 | Wa | decoder W2 (mode 1, 32 rows)] for H = 64 (70.5 / 79.2
  // KB: two workgroups per CU); the next layer's W1e_j (mode 0) is read from L2
  // at both widths.  H = 128: only the padded decoder W2.
  const float* W1 = GW ? a.w1 : sW;
  const float* W2 = GW ? a.w2 : sW + H * ld2;
  const float* Wa = GW ? (MODE == 0 ? a.we : a.wd1) : sW + H * ld2 + H * ldh;
  float* sWb = GW ? sW : sW + H * ld2 + 2 * H * ldh;  // mode 1: decoder W2 (32 rows)
  const float* Wb = MODE == 0 ? a.we + H : sWb;
  const int ldb = MODE == 0 ? 3 * H : ldh;
  float* b1 = MODE == 0 ? sWb : sWb + 32 * ldh;
  float* b2 = b1 + H;
  float* g = b2 + H;
  float* bb = g + H;
  float* ba = bb + H;  // mode 0: b1e   mode 1: decoder b1
  float* bd2 = ba + H;  // mode 1: decoder b2 (32)
  float* bm = bd2 + 32;  // nlin 3: node MLP middle bias
  float* bdm = bm + H;   // nlin 3: decoder middle bias
  if (NL == 3) {
    stage_vec(bm, a.bm, H, H);
    if (MODE == 1) stage_vec(bdm, a.bdm, H, H);
  }
  if (!GW) {
    stage_matrix(sW, ld2, a.w1, 2 * H, H, 2 * H, H, 2 * H);
    stage_matrix(sW + H * ld2, ldh, a.w2, H, H, H, H, H);
  }
  if (MODE == 0) {
    if (!GW) stage_matrix(sW + H * ld2 + H * ldh, ldh, a.we, 3 * H, H, H, H, H);
    stage_vec(ba, a.be, H, H);
  } else {
    if (!GW) stage_matrix(sW + H * ld2 + H * ldh, ldh, a.wd1, H, H, H, H, H);
    stage_matrix(sWb, ldh, a.wd2, H, a.dim + 1, H, 32, H);
    stage_vec(ba, a.bd1, H, H);
    stage_vec(bd2, a.bd2, a.dim + 1, 32);
  }
  stage_vec(b1, a.b1, H, H);
  stage_vec(b2, a.b2, H, H);
  stage_vec(g, a.g, H, H);
  stage_vec(bb, a.bb, H, H);
  __syncthreads();
  const int l = lane_id(), j = l & 31, h = l >> 5, w = wave_id();
  for (int64_t blk = blockIdx.x; blk * (32 * kWaves) < a.n; blk += gridDim.x) {
    const int64_t node0 = blk * (32 * kWaves) + 32 * w;
    if (node0 >= a.n) continue;
    const int64_t i = node0 + j;
    const bool valid = i < a.n;
    const int64_t ic = valid ? i : a.n - 1;
    f32x16 ag[TH], x[TH];
    load_agg<TH>(ag, a, ic);
    if (TRAIN && valid) store_row_clayout<TH>(a.sv.agg + i * H, ag);
    load_row_clayout<TH>(x, a.x_in + ic * H);
    f32x16 hacc[TH];
    acc_bias<TH>(hacc, b1);
    mfma_from_acc<TH, TH, GW>(hacc, W1, ld2, 0, ag);   // graph_network.py:220 cat([aggr, x])
    mfma_from_acc<TH, TH, GW>(hacc, W1, ld2, H, x);
    acc_relu<TH>(hacc);
    if (TRAIN && valid) store_row_clayout<TH>(a.sv.h + i * H, hacc);
    f32x16 y[TH], h2[TH];
    mlp_tail<TH, NL, TH, GW>(y, h2, hacc, a.wm, H, bm, W2, ldw2, b2);
    if (TRAIN && NL == 3 && valid) store_row_clayout<TH>(a.sv.h2 + i * H, h2);
    if (TRAIN) {
      f32x16 yh[TH];
      float rs;
      acc_layernorm_save<TH>(y, g, bb, yh, rs);
      if (valid) {
        store_row_clayout<TH>(a.sv.yhat + i * H, yh);
        if (h == 0) a.sv.rstd[i] = rs;
      }
    } else {
      acc_layernorm<TH>(y, g, bb);
    }
#pragma unroll
    for (int t = 0; t < TH; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) x[t][r] = y[t][r] + x[t][r];  // :176 residual
    if (valid && a.x_out) store_row_clayout<TH>(a.x_out + i * H, x);
    if (MODE == 0) {
      store_uv2<TH, GW, true>(Wa, lda, Wb, ldb, ba, x, a.u + i * H, a.v + i * H, valid);
    } else {
      f32x16 hd[TH];
      acc_bias<TH>(hd, ba);
      mfma_from_acc<TH, TH, GW>(hd, Wa, lda, 0, x);
      acc_relu<TH>(hd);
      if (TRAIN && valid) store_row_clayout<TH>(a.sv.hd + i * H, hd);
      f32x16 o[1], hd2[TH];
      mlp_tail<TH, NL, 1>(o, hd2, hd, a.wdm, H, bdm, Wb, ldh, bd2);
      if (TRAIN && NL == 3 && valid) store_row_clayout<TH>(a.sv.hd2 + i * H, hd2);
      if (valid && h == 0 && !a.pos_seq) {  // decoder output only (EncodeProcessDecode.forward)
        for (int c = 0; c <= a.dim; ++c) a.pred[i * (a.dim + 1) + c] = o[0][c];
      } else if (valid && h == 0) {  // lanes with h == 0 hold units 0..3 in registers 0..3
        const int D = a.dim;
        for (int c = 0; c <= D; ++c) a.pred[i * (D + 1) + c] = o[0][c];
        const float* p = a.pos_seq + i * a.T * D;
        for (int c = 0; c < D; ++c) {  // learned_simulator.py:398-411
          const float acc = __fadd_rn(__fmul_rn(o[0][c], a.acc_std[c]), a.acc_mean[c]);
          const float pT = p[(a.T - 1) * D + c], pT1 = p[(a.T - 2) * D + c];
          const float vel = __fsub_rn(pT, pT1);
          const float np = __fadd_rn(pT, __fadd_rn(vel, acc));
          a.next_pos[i * D + c] = np;
          if (a.window_out) a.window_out[(i * a.T + a.T - 1) * D + c] = np;
        }
      } else if (valid && a.window_out) {  // evaluate.py:136-139 window shift
        const float* p = a.pos_seq + i * a.T * a.dim;
        float* q = a.window_out + i * a.T * a.dim;
        for (int k = 0; k < (a.T - 1) * a.dim; ++k) q[k] = p[k + a.dim];
      }
    }
  }
}

// ---------------------------------------------------------------------------
int check_mlp(const sgnn_mlp* m, int in_dim, int hidden, int out_dim, bool need_ln,
              const char* what) {
  if (!m || !m->w1 || !m->b1 || !m->w2 || !m->b2)
    return sgnn::set_error(SGNN_ERR_INVALID, what);
  if (m->nlin != 2 && m->nlin != 3)
    return sgnn::set_error(SGNN_ERR_UNSUPPORTED, "MLPs must have 2 or 3 Linear layers (nmlp_layers 1 or 2)");
  if (m->nlin == 3 && (!m->w3 || !m->b3)) return sgnn::set_error(SGNN_ERR_INVALID, what);
  if ((in_dim >= 0 && m->in_dim != in_dim) || m->hidden != hidden || m->out_dim != out_dim)
    return sgnn::set_error(SGNN_ERR_INVALID, what);
  if (need_ln && (!m->ln_g || !m->ln_b)) return sgnn::set_error(SGNN_ERR_INVALID, what);
  return SGNN_OK;
}

const float* last_w(const sgnn_mlp* m) { return m->nlin == 3 ? m->w3 : m->w2; }
const float* last_b(const sgnn_mlp* m) { return m->nlin == 3 ? m->b3 : m->b2; }
const float* mid_w(const sgnn_mlp* m) { return m->nlin == 3 ? m->w2 : nullptr; }
const float* mid_b(const sgnn_mlp* m) { return m->nlin == 3 ? m->b2 : nullptr; }

template <typename K>
void set_lds(K kernel, size_t bytes) {
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kernel),
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
}

template <typename K, typename A>
void launch1(K k, unsigned grid, size_t lds, hipStream_t s, const A& a) {
  set_lds(k, lds);
  hipLaunchKernelGGL(k, dim3(grid), dim3(kBlock), lds, s, a);
}

constexpr size_t kLdsMax = 160 * 1024;

bool want_saves(const sgnn_saves* sv) { return sv != nullptr && sv->yhat != nullptr; }

template <int TH, int TKF, int NL>
void go_encode_nodes(bool train, unsigned grid, size_t lds, hipStream_t s, const EncNodeArgs& a) {
  if (train) return launch1(k_encode_nodes<TH, TKF, true, NL>, grid, lds, s, a);
  launch1(k_encode_nodes<TH, TKF, false, NL>, grid, lds, s, a);
}

template <int TH, int NL>
void go_encode_edges(bool train, unsigned grid, size_t lds, hipStream_t s, const EncEdgeArgs& a) {
  if (train) return launch1(k_encode_edges<TH, true, NL>, grid, lds, s, a);
  launch1(k_encode_edges<TH, false, NL>, grid, lds, s, a);
}

template <int TH, int NL>
void go_edge_layer(bool train, unsigned grid, size_t lds, hipStream_t s, const EdgeLayerArgs& a) {
  if (train) return launch1(k_edge_layer<TH, true, NL>, grid, lds, s, a);
  launch1(k_edge_layer<TH, false, NL>, grid, lds, s, a);
}

template <int TH, int MODE, int NL>
void go_node_layer(bool train, unsigned grid, size_t lds, hipStream_t s, const NodeLayerArgs& a) {
  if (train) return launch1(k_node_layer<TH, MODE, true, NL>, grid, lds, s, a);
  launch1(k_node_layer<TH, MODE, false, NL>, grid, lds, s, a);
}

}  // namespace

extern "C" int64_t sgnn_edge_latent_floats(int64_t edge_cap, int32_t hidden) {
  return ((edge_cap + 31) / 32) * 32 * (int64_t)hidden;
}

#define SGNN_DISPATCH_H_NL(H, NL, CALL)                                   \
  do {                                                                    \
    if ((H) == 64 && (NL) == 2) { constexpr int TH_ = 2, NL_ = 2; CALL; } \
    else if ((H) == 64) { constexpr int TH_ = 2, NL_ = 3; CALL; }         \
    else if ((NL) == 2) { constexpr int TH_ = 4, NL_ = 2; CALL; }         \
    else { constexpr int TH_ = 4, NL_ = 3; CALL; }                        \
  } while (0)

static int check_train(bool train, const sgnn_mlp* m, const sgnn_saves* sv, const char* what) {
  if (train && m->nlin == 3 && !sv->h2) return sgnn::set_error(SGNN_ERR_INVALID, what);
  return SGNN_OK;
}

namespace sgnn {

// sgnn_encode_nodes; with fuse_radius, the small-graph radius search those
// arguments describe is launched too (in the same launch as the inference
// encoder when that takes the 16-node path, else just before it).
int encode_nodes_impl(const float* pos_seq, int64_t n, int32_t T, int32_t dim, const int64_t* types,
                      const float* emb_w, int32_t emb_dim, int32_t use_emb, const float* vel_mean,
                      const float* vel_std, float wall_max, float wall_div, const sgnn_mlp* enc,
                      const sgnn_mlp* edge0, float* x0, float* u, float* v, const sgnn_saves* saves,
                      void* stream, const RadiusSmallArgs* fuse_radius, bool defer_csr, bool* csr_pending) {
  if (csr_pending) *csr_pending = false;
  if (n <= 0) return SGNN_OK;
  if (!pos_seq || !vel_mean || !vel_std || !x0 || !u || !v || T < 2 || dim < 1 || dim > 3)
    return set_error(SGNN_ERR_INVALID, "encode_nodes: bad arguments");
  if (!enc) return set_error(SGNN_ERR_INVALID, "encode_nodes: enc");
  const int H = enc->hidden;
  const int feat = (T - 1) * dim + 1 + (use_emb ? emb_dim : 0);
  int st = check_mlp(enc, feat, H, H, true, "encode_nodes: encoder MLP shape");
  if (!st) st = check_mlp(edge0, 3 * H, H, H, true, "encode_nodes: edge0 MLP shape");
  if (st) return st;
  if (use_emb && (!types || !emb_w)) return set_error(SGNN_ERR_INVALID, "encode_nodes: embedding");
  if (H != 64 && H != 128) return set_error(SGNN_ERR_UNSUPPORTED, "encode_nodes: hidden must be 64 or 128");
  EncNodeArgs a{pos_seq, n, T, dim, types, emb_w, emb_dim, use_emb, vel_mean, vel_std, wall_max,
                feat, enc->w1, enc->b1, last_w(enc), last_b(enc), enc->ln_g, enc->ln_b,
                mid_w(enc), mid_b(enc), wall_max, wall_div, edge0->w1, edge0->b1, x0, u, v, {}};
  const bool train = want_saves(saves);
  if ((st = check_train(train, enc, saves, "encode_nodes: nmlp_layers = 2 training needs saves->h2"))) return st;
  if (train) {
    if (!saves->h || !saves->rstd) return set_error(SGNN_ERR_INVALID, "encode_nodes: saves");
    a.sv = *saves;
  }
  if (!train && H == 64 && feat <= 48) {  // inference: 16-node tiles, units split over 4 waves (fwd16.hip)
    sgnn::EncNode16Args b{};
    b.nd.n = n; b.nd.wm = mid_w(enc); b.nd.bm = mid_b(enc); b.nd.w2 = last_w(enc); b.nd.b2 = last_b(enc);
    b.nd.g = enc->ln_g; b.nd.bb = enc->ln_b; b.nd.we = edge0->w1; b.nd.be = edge0->b1;
    b.nd.u = u; b.nd.v = v; b.nd.x_out = x0;
    b.pos_seq = pos_seq; b.T = T; b.dim = dim; b.types = types; b.emb_w = emb_w; b.emb_dim = emb_dim;
    b.use_emb = use_emb; b.vel_mean = vel_mean; b.vel_std = vel_std; b.wall_max = wall_max;
    b.wall_div = wall_div; b.feat = feat; b.w1 = enc->w1; b.b1 = enc->b1;
    if (fuse_radius) {
      const bool defer = defer_csr && csr_pending;
      st = sgnn::radius_enc16_launch(*fuse_radius, b, enc->nlin, static_cast<hipStream_t>(stream), !defer);
      if (!st && defer) *csr_pending = true;
      return st;
    }
    return sgnn::enc_node16_launch(b, enc->nlin, static_cast<hipStream_t>(stream));
  }
  if (fuse_radius && (st = radius_small_launch(*fuse_radius, static_cast<hipStream_t>(stream)))) return st;
  const unsigned grid = persistent_grid(n, 32 * kWaves, 2);
  const int tkf = (feat + 31) / 32;
  const size_t lds = sizeof(float) * (size_t)(H * (32 * tkf + 4) + (H == 64 ? 3 * H * (H + 4) : 0) + 6 * H);
  if (lds > kLdsMax) return set_error(SGNN_ERR_UNSUPPORTED, "encode_nodes: too many features");
  if (tkf > 3 || (tkf == 3 && H != 64))
    return set_error(SGNN_ERR_UNSUPPORTED, "encode_nodes: too many node features");
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (tkf == 1) SGNN_DISPATCH_H_NL(H, enc->nlin, (go_encode_nodes<TH_, 1, NL_>(train, grid, lds, s, a)));
  else if (tkf == 2) SGNN_DISPATCH_H_NL(H, enc->nlin, (go_encode_nodes<TH_, 2, NL_>(train, grid, lds, s, a)));
  else {
    if (enc->nlin == 2) go_encode_nodes<2, 3, 2>(train, grid, lds, s, a);
    else go_encode_nodes<2, 3, 3>(train, grid, lds, s, a);
  }
  return check_launch("encode_nodes");
}

}  // namespace sgnn

extern "C" int sgnn_encode_nodes(const float* pos_seq, int64_t n, int32_t T, int32_t dim,
                                 const int64_t* types, const float* emb_w, int32_t emb_dim,
                                 int32_t use_emb, const float* vel_mean, const float* vel_std,
                                 float wall_max, float wall_div, const sgnn_mlp* enc,
                                 const sgnn_mlp* edge0, float* x0, float* u, float* v,
                                 const sgnn_saves* saves, void* stream) {
  return sgnn::encode_nodes_impl(pos_seq, n, T, dim, types, emb_w, emb_dim, use_emb, vel_mean, vel_std, wall_max,
                                 wall_div, enc, edge0, x0, u, v, saves, stream, nullptr, false, nullptr);
}

extern "C" int sgnn_encode_edges(const float* pos, int64_t pos_stride, int32_t dim, float radius,
                                 const int32_t* rowptr, const int32_t* send, const int32_t* recv,
                                 int64_t n, int64_t edge_cap, const sgnn_mlp* enc, float* e0t,
                                 const sgnn_saves* saves, void* stream) {
  using namespace sgnn;
  if (n <= 0 || edge_cap <= 0) return SGNN_OK;
  if (!pos || !rowptr || !send || !recv || !e0t || dim < 1 || dim > 3)
    return set_error(SGNN_ERR_INVALID, "encode_edges: bad arguments");
  if (!enc) return set_error(SGNN_ERR_INVALID, "encode_edges: enc");
  const int H = enc->hidden;
  int st = check_mlp(enc, dim + 1, H, H, true, "encode_edges: encoder MLP shape");
  if (st) return st;
  if (H != 64 && H != 128) return set_error(SGNN_ERR_UNSUPPORTED, "encode_edges: hidden must be 64 or 128");
  EncEdgeArgs a{pos, pos_stride, dim, radius, rowptr, send, recv, n, enc->w1, enc->b1,
                last_w(enc), last_b(enc), enc->ln_g, enc->ln_b, e0t, {}, mid_w(enc), mid_b(enc)};
  const bool train = want_saves(saves);
  if ((st = check_train(train, enc, saves, "encode_edges: nmlp_layers = 2 training needs saves->h2"))) return st;
  if (train) {
    if (!saves->rstd) return set_error(SGNN_ERR_INVALID, "encode_edges: saves");
    a.sv = *saves;
  }
  const unsigned grid = persistent_grid(edge_cap, 32 * kWaves, 4);
  const size_t lds = sizeof(float) * (size_t)(H * 5 + (H == 64 ? H * (H + 4) : 0) + 5 * H);
  hipStream_t s = static_cast<hipStream_t>(stream);
  SGNN_DISPATCH_H_NL(H, enc->nlin, (go_encode_edges<TH_, NL_>(train, grid, lds, s, a)));
  return check_launch("encode_edges");
}

extern "C" int sgnn_edge_layer(const float* u, const float* v, const float* e0t, float e_scale,
                               const int32_t* rowptr, const int32_t* send, const int32_t* recv,
                               int64_t n, int64_t edge_cap, const sgnn_mlp* edge_fn, float* agg,
                               float* cin, float* cout, const sgnn_saves* saves, void* stream) {
  using namespace sgnn;
  if (n <= 0 || edge_cap <= 0) return SGNN_OK;
  if (!u || !v || !e0t || !rowptr || !send || !recv || !agg || !cin || !cout || !edge_fn)
    return set_error(SGNN_ERR_INVALID, "edge_layer: null pointer");
  const int H = edge_fn->hidden;
  int st = check_mlp(edge_fn, 3 * H, H, H, true, "edge_layer: edge MLP shape");
  if (st) return st;
  if (H != 64 && H != 128) return set_error(SGNN_ERR_UNSUPPORTED, "edge_layer: hidden must be 64 or 128");
  EdgeLayerArgs a{u, v, e0t, e_scale, rowptr, send, recv, n, edge_fn->w1 + 2 * H, last_w(edge_fn),
                  last_b(edge_fn), edge_fn->ln_g, edge_fn->ln_b, agg, cin, cout, {},
                  mid_w(edge_fn), mid_b(edge_fn)};
  // training saves; at hidden 128 with nmlp_layers 2, yhat and h2 may both be NULL (the backward recomputes
  // them from h: include/sgnn.h, sgnn_saves)
  const bool train = saves != nullptr && (saves->yhat != nullptr || saves->h != nullptr);
  const bool rc = train && !saves->yhat;
  if (rc && !(H == 128 && edge_fn->nlin == 3 && !saves->h2))
    return set_error(SGNN_ERR_INVALID, "edge_layer: saves->yhat NULL only at hidden 128, nmlp_layers 2, with h2 NULL");
  if (!rc && (st = check_train(train, edge_fn, saves, "edge_layer: nmlp_layers = 2 training needs saves->h2")))
    return st;
  if (train) {
    if (!saves->h || !saves->rstd) return set_error(SGNN_ERR_INVALID, "edge_layer: saves");
    a.sv = *saves;
  }
  const size_t lds = sizeof(float) * (size_t)((H == 64 ? 2 : 1) * H * (H + 4) + 4 * H + kWaves * 32 * (H + 4));
  unsigned grid = persistent_grid(edge_cap, 32 * kWaves, H == 64 ? 2 : 1);  // workgroups per CU LDS allows
  if (grid >= 8) grid &= ~7u;  // a multiple of 8 for the XCD-aware tile order
  hipStream_t s = static_cast<hipStream_t>(stream);
  SGNN_DISPATCH_H_NL(H, edge_fn->nlin, (go_edge_layer<TH_, NL_>(train, grid, lds, s, a)));
  return check_launch("edge_layer");
}

static int node_layer_common(NodeLayerArgs& a, const sgnn_mlp* node_fn, int mode, int dec_nlin,
                             const sgnn_saves* saves, void* stream) {
  using namespace sgnn;
  const int H = node_fn ? node_fn->hidden : 0;
  int st = check_mlp(node_fn, 2 * H, H, H, true, "node_layer: node MLP shape");
  if (st) return st;
  if (H != 64 && H != 128) return set_error(SGNN_ERR_UNSUPPORTED, "node_layer: hidden must be 64 or 128");
  if (mode == 1 && dec_nlin != node_fn->nlin)
    return set_error(SGNN_ERR_UNSUPPORTED, "node_layer_decode: decoder and node MLP depths differ");
  a.w1 = node_fn->w1; a.b1 = node_fn->b1; a.w2 = last_w(node_fn); a.b2 = last_b(node_fn);
  a.wm = mid_w(node_fn); a.bm = mid_b(node_fn);
  a.g = node_fn->ln_g; a.bb = node_fn->ln_b;
  const bool train = want_saves(saves);
  if ((st = check_train(train, node_fn, saves, "node_layer: nmlp_layers = 2 training needs saves->h2"))) return st;
  if (train) {
    if (!saves->h || !saves->rstd || !saves->agg || (mode == 1 && (!saves->hd || !a.x_out)) ||
        (mode == 1 && dec_nlin == 3 && !saves->hd2))
      return set_error(SGNN_ERR_INVALID, "node_layer: saves");
    a.sv = *saves;
  }
  // inference, small graphs: 16-node tiles, output units split over 4 waves (fwd16.hip); from ~10k
  // nodes up the 32-node one-wave tiles below are faster (C2 50k: 36 vs 45 us per layer)
  if (!train && H == 64 && a.n <= 8192) {
    sgnn::Node16Args b{a.x_in, a.agg, a.cin, a.cout, a.rowptr, a.n, a.w1, a.b1, a.wm, a.bm, a.w2, a.b2,
                       a.g, a.bb, a.we, a.be, a.u, a.v, a.wd1, a.bd1, a.wdm, a.bdm, a.wd2, a.bd2,
                       a.pos_seq, a.T, a.dim, a.acc_mean, a.acc_std, a.pred, a.next_pos,
                       a.window_out, a.x_out};
    return sgnn::node16_launch(b, mode, node_fn->nlin, static_cast<hipStream_t>(stream));
  }
  const size_t vec = 5 * H + 32 + 2 * H;
  const size_t dec_w2 = mode == 1 ? 32 * (H + 4) : 0;  // padded decoder last Linear
  const size_t lds = sizeof(float) * (H == 64 ? H * (2 * H + 4) + 2 * H * (H + 4) + dec_w2 + vec
                                              : dec_w2 + vec);
  const unsigned grid = persistent_grid(a.n, 32 * kWaves, 2);
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (mode == 0) SGNN_DISPATCH_H_NL(H, node_fn->nlin, (go_node_layer<TH_, 0, NL_>(train, grid, lds, s, a)));
  else SGNN_DISPATCH_H_NL(H, node_fn->nlin, (go_node_layer<TH_, 1, NL_>(train, grid, lds, s, a)));
  return check_launch("node_layer");
}

extern "C" int sgnn_node_layer(const float* x_in, const float* agg, const float* cin,
                               const float* cout, const int32_t* rowptr, int64_t n,
                               const sgnn_mlp* node_fn, const sgnn_mlp* next_edge, float* x_out,
                               float* u, float* v, const sgnn_saves* saves, void* stream) {
  using namespace sgnn;
  if (n <= 0) return SGNN_OK;
  if (!x_in || !agg || !cin || !cout || !rowptr || !x_out || !u || !v || !next_edge)
    return set_error(SGNN_ERR_INVALID, "node_layer: null pointer");
  const int H = node_fn ? node_fn->hidden : 0;
  int st = check_mlp(next_edge, 3 * H, H, H, true, "node_layer: next edge MLP shape");
  if (st) return st;
  NodeLayerArgs a{};
  a.x_in = x_in; a.agg = agg; a.cin = cin; a.cout = cout; a.rowptr = rowptr; a.n = n;
  a.we = next_edge->w1; a.be = next_edge->b1; a.u = u; a.v = v; a.x_out = x_out;
  return node_layer_common(a, node_fn, 0, 0, saves, stream);
}

extern "C" int sgnn_node_layer_decode(const float* x_in, const float* agg, const float* cin,
                                      const float* cout, const int32_t* rowptr, int64_t n,
                                      const sgnn_mlp* node_fn, const sgnn_mlp* decoder,
                                      const float* pos_seq, int32_t T, int32_t dim,
                                      const float* acc_mean, const float* acc_std, float* x_out,
                                      float* pred, float* next_pos, float* window_out,
                                      const sgnn_saves* saves, void* stream) {
  using namespace sgnn;
  if (n <= 0) return SGNN_OK;
  if (!x_in || !agg || !cin || !cout || !rowptr || !pred || dim < 1 || dim > 3 ||
      (pos_seq && (!acc_mean || !acc_std || !next_pos || T < 2)))
    return set_error(SGNN_ERR_INVALID, "node_layer_decode: bad arguments");
  const int H = node_fn ? node_fn->hidden : 0;
  int st = check_mlp(decoder, H, H, dim + 1, false, "node_layer_decode: decoder MLP shape");
  if (st) return st;
  NodeLayerArgs a{};
  a.x_in = x_in; a.agg = agg; a.cin = cin; a.cout = cout; a.rowptr = rowptr; a.n = n;
  a.wd1 = decoder->w1; a.bd1 = decoder->b1; a.wd2 = last_w(decoder); a.bd2 = last_b(decoder);
  a.wdm = mid_w(decoder); a.bdm = mid_b(decoder);
  a.pos_seq = pos_seq; a.T = T; a.dim = dim; a.acc_mean = acc_mean; a.acc_std = acc_std;
  a.pred = pred; a.next_pos = next_pos; a.window_out = window_out; a.x_out = x_out;
  if (window_out && window_out == pos_seq)
    return set_error(SGNN_ERR_INVALID, "node_layer_decode: window_out aliases pos_seq");
  return node_layer_common(a, node_fn, 1, decoder->nlin, saves, stream);
}

// ---------------------------------------------------------------------------
// EncodeProcessDecode.forward(x, edge_index, edge_features) on explicit
// features (graph_network.py:388-406): the encoders read given feature rows
// instead of deriving them from positions.
extern "C" int sgnn_encode_node_features(const float* x, int64_t n, int32_t feat,
                                         const sgnn_mlp* enc, const sgnn_mlp* edge0, float* x0,
                                         float* u, float* v, void* stream) {
  using namespace sgnn;
  if (n <= 0) return SGNN_OK;
  if (!x || !x0 || !u || !v || !enc || feat < 1) return set_error(SGNN_ERR_INVALID, "encode_node_features: bad arguments");
  const int H = enc->hidden;
  int st = check_mlp(enc, feat, H, H, true, "encode_node_features: encoder MLP shape");
  if (!st) st = check_mlp(edge0, 3 * H, H, H, true, "encode_node_features: edge0 MLP shape");
  if (st) return st;
  if (H != 64 && H != 128) return set_error(SGNN_ERR_UNSUPPORTED, "encode_node_features: hidden must be 64 or 128");
  EncNodeArgs a{nullptr, n, 2, 1, nullptr, nullptr, 0, 0, nullptr, nullptr, 0.0f, feat, enc->w1,
                enc->b1, last_w(enc), last_b(enc), enc->ln_g, enc->ln_b, mid_w(enc), mid_b(enc),
                0.0f, 1.0f, edge0->w1, edge0->b1, x0, u, v, {}, x};
  const unsigned grid = persistent_grid(n, 32 * kWaves, 2);
  const int tkf = (feat + 31) / 32;
  const size_t lds = sizeof(float) * (size_t)(H * (32 * tkf + 4) + (H == 64 ? 3 * H * (H + 4) : 0) + 6 * H);
  if (tkf > 3 || (tkf == 3 && H != 64) || lds > kLdsMax)
    return set_error(SGNN_ERR_UNSUPPORTED, "encode_node_features: too many node features");
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (tkf == 1) SGNN_DISPATCH_H_NL(H, enc->nlin, (go_encode_nodes<TH_, 1, NL_>(false, grid, lds, s, a)));
  else if (tkf == 2) SGNN_DISPATCH_H_NL(H, enc->nlin, (go_encode_nodes<TH_, 2, NL_>(false, grid, lds, s, a)));
  else if (enc->nlin == 2) go_encode_nodes<2, 3, 2>(false, grid, lds, s, a);
  else go_encode_nodes<2, 3, 3>(false, grid, lds, s, a);
  return check_launch("encode_node_features");
}

extern "C" int sgnn_encode_edge_features(const float* e, int32_t fe, const int32_t* perm,
                                         const int32_t* rowptr, int64_t n, int64_t edge_cap,
                                         const sgnn_mlp* enc, float* e0t, void* stream) {
  using namespace sgnn;
  if (n <= 0 || edge_cap <= 0) return SGNN_OK;
  if (!e || !perm || !rowptr || !e0t || !enc || fe < 1 || fe > 4)
    return set_error(SGNN_ERR_INVALID, "encode_edge_features: bad arguments (1 <= fe <= 4)");
  const int H = enc->hidden;
  int st = check_mlp(enc, fe, H, H, true, "encode_edge_features: encoder MLP shape");
  if (st) return st;
  if (H != 64 && H != 128) return set_error(SGNN_ERR_UNSUPPORTED, "encode_edge_features: hidden must be 64 or 128");
  EncEdgeArgs a{nullptr, 0, fe - 1, 1.0f, rowptr, nullptr, nullptr, n, enc->w1, enc->b1,
                last_w(enc), last_b(enc), enc->ln_g, enc->ln_b, e0t, {}, mid_w(enc), mid_b(enc),
                e, perm, fe};
  const unsigned grid = persistent_grid(edge_cap, 32 * kWaves, 4);
  const size_t lds = sizeof(float) * (size_t)(H * 5 + (H == 64 ? H * (H + 4) : 0) + 5 * H);
  hipStream_t s = static_cast<hipStream_t>(stream);
  SGNN_DISPATCH_H_NL(H, enc->nlin, (go_encode_edges<TH_, NL_>(false, grid, lds, s, a)));
  return check_launch("encode_edge_features");
}

// ---------------------------------------------------------------------------
// Fused InteractionNetwork layer (inference, H = 64): edge MLP + receiver sums
// + node update in one launch (fwd16.hip k_layer16).
static int layer_common(sgnn::Layer16Args& L, const sgnn_mlp* edge_fn, const sgnn_mlp* node_fn, int mode,
                        int dec_nlin, void* stream, bool first = false) {
  using namespace sgnn;
  const int H = node_fn ? node_fn->hidden : 0;
  int st = check_mlp(node_fn, 2 * H, H, H, true, "interaction_layer: node MLP shape");
  if (!st) st = check_mlp(edge_fn, 3 * H, H, H, true, "interaction_layer: edge MLP shape");
  if (st) return st;
  if (H != 64) return set_error(SGNN_ERR_UNSUPPORTED, "interaction_layer: fused layer needs hidden 64");
  if (edge_fn->nlin != node_fn->nlin || (mode == 1 && dec_nlin != node_fn->nlin))
    return set_error(SGNN_ERR_UNSUPPORTED, "interaction_layer: MLP depths differ");
  Node16Args& a = L.nd;
  a.w1 = node_fn->w1; a.b1 = node_fn->b1; a.w2 = last_w(node_fn); a.b2 = last_b(node_fn);
  a.wm = mid_w(node_fn); a.bm = mid_b(node_fn); a.g = node_fn->ln_g; a.bb = node_fn->ln_b;
  L.ewe = edge_fn->w1 + 2 * H; L.ewm = mid_w(edge_fn); L.ebm = mid_b(edge_fn);
  L.ew2 = last_w(edge_fn); L.eb2 = last_b(edge_fn); L.eg = edge_fn->ln_g; L.ebb = edge_fn->ln_b;
  // nodes per workgroup tile: ~400 workgroups, 8..16 nodes each -- fewer, fatter workgroups pay
  // the per-workgroup weight loads less often, and more than 512 (two per CU) would run in two
  // rounds (measured, tools/exp_layer16.py: C1 r = 15 21.4 -> 18.6-19.9 us at 8 nodes vs 4,
  // r = 0.6 17.9 -> 11.8 us; 4,800 particles best at 12, 8,000 at 16)
  L.nt = (int)std::min<int64_t>(16, std::max<int64_t>(8, (a.n + 399) / 400));
#ifdef SGNN_EXPERIMENT
  if (const char* e = getenv("SGNN_NT")) L.nt = std::min(16, std::max(8, atoi(e)));  // tools/exp_layer16.py builds
#endif
  return layer16_launch(L, mode, node_fn->nlin, static_cast<hipStream_t>(stream), first);
}

extern "C" int sgnn_interaction_layer(const float* x_in, const float* u_in, const float* v_in,
                                      const float* e0t, float e_scale, const int32_t* rowptr,
                                      const int32_t* send, const int32_t* recv, int64_t n,
                                      const sgnn_mlp* edge_fn, const sgnn_mlp* node_fn,
                                      const sgnn_mlp* next_edge, float* x_out, float* u_out,
                                      float* v_out, void* stream) {
  using namespace sgnn;
  if (n <= 0) return SGNN_OK;
  if (!x_in || !u_in || !v_in || !e0t || !rowptr || !send || !recv || !x_out || !u_out || !v_out ||
      !next_edge || u_out == u_in || v_out == v_in)
    return set_error(SGNN_ERR_INVALID, "interaction_layer: bad arguments (u/v out must not alias u/v in)");
  const int H = node_fn ? node_fn->hidden : 0;
  int st = check_mlp(next_edge, 3 * H, H, H, true, "interaction_layer: next edge MLP shape");
  if (st) return st;
  Layer16Args L{};
  L.nd.x_in = x_in; L.nd.rowptr = rowptr; L.nd.n = n; L.nd.we = next_edge->w1; L.nd.be = next_edge->b1;
  L.nd.u = u_out; L.nd.v = v_out; L.nd.x_out = x_out;
  L.u_in = u_in; L.v_in = v_in; L.e0t = e0t; L.e_scale = e_scale; L.send = send; L.recv = recv;
  return layer_common(L, edge_fn, node_fn, 0, 0, stream);
}

extern "C" int sgnn_interaction_layer_decode(const float* x_in, const float* u_in, const float* v_in,
                                             const float* e0t, float e_scale, const int32_t* rowptr,
                                             const int32_t* send, const int32_t* recv, int64_t n,
                                             const sgnn_mlp* edge_fn, const sgnn_mlp* node_fn,
                                             const sgnn_mlp* decoder, const float* pos_seq, int32_t T,
                                             int32_t dim, const float* acc_mean, const float* acc_std,
                                             float* pred, float* next_pos, float* window_out,
                                             void* stream) {
  using namespace sgnn;
  if (n <= 0) return SGNN_OK;
  if (!x_in || !u_in || !v_in || !e0t || !rowptr || !send || !recv || !pred || dim < 1 || dim > 3 ||
      (pos_seq && (!acc_mean || !acc_std || !next_pos || T < 2)))
    return set_error(SGNN_ERR_INVALID, "interaction_layer_decode: bad arguments");
  if (window_out && window_out == pos_seq)
    return set_error(SGNN_ERR_INVALID, "interaction_layer_decode: window_out aliases pos_seq");
  const int H = node_fn ? node_fn->hidden : 0;
  int st = check_mlp(decoder, H, H, dim + 1, false, "interaction_layer_decode: decoder MLP shape");
  if (st) return st;
  Layer16Args L{};
  L.nd.x_in = x_in; L.nd.rowptr = rowptr; L.nd.n = n;
  L.nd.wd1 = decoder->w1; L.nd.bd1 = decoder->b1; L.nd.wd2 = last_w(decoder); L.nd.bd2 = last_b(decoder);
  L.nd.wdm = mid_w(decoder); L.nd.bdm = mid_b(decoder);
  L.nd.pos_seq = pos_seq; L.nd.T = T; L.nd.dim = dim; L.nd.acc_mean = acc_mean; L.nd.acc_std = acc_std;
  L.nd.pred = pred; L.nd.next_pos = next_pos; L.nd.window_out = window_out; L.nd.x_out = nullptr;
  L.u_in = u_in; L.v_in = v_in; L.e0t = e0t; L.e_scale = e_scale; L.send = send; L.recv = recv;
  return layer_common(L, edge_fn, node_fn, 1, decoder->nlin, stream);
}

namespace sgnn {

int interaction_layer_encode_impl(const float* pos, int64_t pos_stride, int32_t dim, float radius,
                                  const sgnn_mlp* enc_edge, float* e0t, const float* x_in, const float* u_in,
                                  const float* v_in, const int32_t* rowptr, const int32_t* send,
                                  const int32_t* recv, int64_t n, const sgnn_mlp* edge_fn, const sgnn_mlp* node_fn,
                                  const sgnn_mlp* next_edge, float* x_out, float* u_out, float* v_out, void* stream,
                                  const RadiusSmallArgs* lists) {
  if (n <= 0) return SGNN_OK;
  if (lists && (lists->n != n || lists->rowptr != rowptr || lists->send != send || lists->recv != recv))
    return set_error(SGNN_ERR_INVALID, "interaction_layer_encode: lists describe another graph");
  if (!pos || dim < 1 || dim > 3 || !(radius > 0.0f) || !e0t || !x_in || !u_in || !v_in || !rowptr || !send ||
      !recv || !x_out || !u_out || !v_out || !next_edge || u_out == u_in || v_out == v_in)
    return set_error(SGNN_ERR_INVALID, "interaction_layer_encode: bad arguments");
  const int H = node_fn ? node_fn->hidden : 0;
  int st = check_mlp(enc_edge, dim + 1, H, H, true, "interaction_layer_encode: edge encoder MLP shape");
  if (!st) st = check_mlp(next_edge, 3 * H, H, H, true, "interaction_layer_encode: next edge MLP shape");
  if (st) return st;
  if (enc_edge->nlin != 2 || node_fn->nlin != 2)
    return set_error(SGNN_ERR_UNSUPPORTED, "interaction_layer_encode: nmlp_layers 1 only");
  Layer16Args L{};
  L.nd.x_in = x_in; L.nd.rowptr = rowptr; L.nd.n = n; L.nd.we = next_edge->w1; L.nd.be = next_edge->b1;
  L.nd.u = u_out; L.nd.v = v_out; L.nd.x_out = x_out;
  L.u_in = u_in; L.v_in = v_in; L.e0t = e0t; L.e_scale = 1.0f; L.send = send; L.recv = recv;
  L.pos = pos; L.pos_stride = pos_stride; L.dim = dim; L.radius = radius;
  L.xw1 = enc_edge->w1; L.xb1 = enc_edge->b1; L.xw2 = enc_edge->w2; L.xb2 = enc_edge->b2;
  L.xg = enc_edge->ln_g; L.xbb = enc_edge->ln_b; L.e0t_out = e0t;
  if (lists) {
    L.l_deg = lists->deg; L.l_nbr = lists->nbr; L.l_cap = lists->cap;
    L.rowptr_out = lists->rowptr; L.send_out = lists->send; L.recv_out = lists->recv;
  }
  return layer_common(L, edge_fn, node_fn, 0, 0, stream, true);
}

}  // namespace sgnn

extern "C" int sgnn_interaction_layer_encode(const float* pos, int64_t pos_stride, int32_t dim, float radius,
                                             const sgnn_mlp* enc_edge, float* e0t, const float* x_in,
                                             const float* u_in, const float* v_in, const int32_t* rowptr,
                                             const int32_t* send, const int32_t* recv, int64_t n,
                                             const sgnn_mlp* edge_fn, const sgnn_mlp* node_fn,
                                             const sgnn_mlp* next_edge, float* x_out, float* u_out,
                                             float* v_out, void* stream) {
  return sgnn::interaction_layer_encode_impl(pos, pos_stride, dim, radius, enc_edge, e0t, x_in, u_in, v_in, rowptr,
                                             send, recv, n, edge_fn, node_fn, next_edge, x_out, u_out, v_out,
                                             stream, nullptr);
}
