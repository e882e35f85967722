// Backward of the Encode-Process-Decode training step for gfx950.
//
// Reverse-mode of sgnn/single_scale/learned_simulator.py:440-491
// (predict_accelerations) + train.py:257-268 (loss), i.e. what
// loss.backward() computes through PyG/torch autograd, as 3L + 4 fused
// launches (L = message-passing layers):
//   k_dec_bwd       loss -> d pred -> Decoder backward -> g_L = dL/dx_L
//   k_node_bwd(k)   node MLP + LayerNorm + residual backward -> d agg_k, dx_k'
//   k_edge_bwd(k)   edge MLP + LayerNorm backward from d agg_k[recv]:
//                   dh (ReLU-masked) -> segment sums dU (receiver CSR),
//                   dh rows for dV, dE0 += 2^k W1e^T dh
//   k_uv_bwd64(k)   g_k = dx_k' + W1i^T dU + W1j^T dV  (dV gathered through
//                   the sender-sorted transpose CSR, deterministic)
//   k_enc_node_bwd, k_enc_edge_bwd   Encoder MLPs
//   k_reduce_slabs  weight gradients
// Weight gradients are outer products summed over items (nodes / edges):
// each 4-wave workgroup stages 128 items of both operands in LDS
// ([item][unit] images) and every wave accumulates one 32x32 output tile
// with v_mfma_f32_32x32x2_f32 using the items as the k dimension.  Per-WG
// partials go to a slab; k_reduce_slabs sums the slabs in fixed order, so
// gradients are bitwise reproducible run to run (no float atomics).
#include "common.h"
#include "../../include/sgnn.h"
#include "sgnn_internal.h"

namespace {

constexpr int kBlock = 256;
constexpr int kWaves = 4;
constexpr int kChunk = 32 * kWaves;  // items per workgroup iteration

SGNN_DEV int clamp_items(int64_t remaining) {
  return remaining <= 0 ? 0 : (remaining >= 32 ? 32 : (int)remaining);
}

template <int TH>
SGNN_DEV void zero(f32x16 (&x)[TH]) {
#pragma unroll
  for (int t = 0; t < TH; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) x[t][r] = 0.0f;
}

template <int TH>
SGNN_DEV void zero_if(f32x16 (&x)[TH], bool pred) {
  if (pred) zero<TH>(x);
}

// lane = unit: sum over the first nvalid items of a wave's LDS slice
// (every image row past nvalid holds zeros, so all 32 rows are summed: four
// independent partial sums over an unrolled loop instead of a dependent
// load-add chain of runtime length)
SGNN_DEV float lane_sum(const float* slice, int ld, int nvalid, int unit) {
  (void)nvalid;
  float s0 = 0.0f, s1 = 0.0f, s2 = 0.0f, s3 = 0.0f;
#pragma unroll
  for (int it = 0; it < 32; it += 4) {
    s0 += slice[it * ld + unit];
    s1 += slice[(it + 1) * ld + unit];
    s2 += slice[(it + 2) * ld + unit];
    s3 += slice[(it + 3) * ld + unit];
  }
  return (s0 + s1) + (s2 + s3);
}

template <int TH>
SGNN_DEV void lane_sums(float (&acc)[TH / 2 > 0 ? TH / 2 : 1], const float* slice, int ld,
                        int nvalid) {
  constexpr int UPL = (32 * TH) / 64 > 0 ? (32 * TH) / 64 : 1;
#pragma unroll
  for (int q = 0; q < UPL; ++q) {
    const int u = lane_id() + 64 * q;
    if (u < 32 * TH) acc[q] += lane_sum(slice, ld, nvalid, u);
  }
}

// Resolve a receiver-CSR row sum (agg or dU) for node i from rows + carries.
template <int TH>
SGNN_DEV void load_resolved(f32x16 (&a)[TH], const float* rows, const float* cin,
                            const float* cout, const int32_t* rowptr, int64_t i) {
  constexpr int H = 32 * TH;
  const int32_t r0 = rowptr[i], r1 = rowptr[i + 1];
  if (r1 <= r0) {
    zero<TH>(a);
    return;
  }
  const int32_t t0 = r0 >> 5, t1 = (r1 - 1) >> 5;
  if (t0 == t1) {
    load_row_clayout<TH>(a, rows + i * H);
  } else {
    load_row_clayout<TH>(a, cout + (int64_t)t0 * H);  // segments may span > 2 tiles
    for (int32_t t = t0 + 1; t <= t1; ++t) add_row_clayout<TH>(a, cin + (int64_t)t * H);
  }
}

// Each wave owns output tiles w, w+4, ... of a [32*TU x 32*TV] gradient.
template <int NT>
SGNN_DEV void outer_tiles(f32x16 (&acc)[NT], int TU, int TV, const float* A, int lda, int abase,
                          const float* B, int ldb, int bbase) {
  const int w = wave_id();
#pragma unroll
  for (int q = 0; q < NT; ++q) {
    const int tile = w + kWaves * q;
    if (tile < TU * TV) {
      const int tu = tile / TV, tv = tile - tu * TV;
      mfma_outer<kChunk>(acc[q], A, lda, abase + 32 * tu, B, ldb, bbase + 32 * tv);
    }
  }
}

template <int NT>
SGNN_DEV void store_outer(float* dst, int ld, int TU, int TV, const f32x16 (&acc)[NT]) {
  const int w = wave_id();
#pragma unroll
  for (int q = 0; q < NT; ++q) {
    const int tile = w + kWaves * q;
    if (tile < TU * TV) {
      const int tu = tile / TV, tv = tile - tu * TV;
      store_tile_rowmajor(dst + (32 * tu) * ld + 32 * tv, ld, acc[q]);
    }
  }
}

template <int NT>
SGNN_DEV void zero_acc(f32x16 (&acc)[NT]) {
#pragma unroll
  for (int q = 0; q < NT; ++q)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[q][r] = 0.0f;
}

// per-wave lane-unit vector partial -> slab row (wave w)
template <int TH>
SGNN_DEV void store_lane_vec(float* dst, const float (&acc)[TH / 2 > 0 ? TH / 2 : 1]) {
  constexpr int H = 32 * TH;
  constexpr int UPL = H / 64 > 0 ? H / 64 : 1;
  const int w = wave_id(), l = lane_id();
#pragma unroll
  for (int q = 0; q < UPL; ++q)
    if (l + 64 * q < H) dst[w * H + l + 64 * q] = acc[q];
}

#define LANEVEC(name) float name[TH / 2 > 0 ? TH / 2 : 1] = {}
template <int TH>
using LaneVec = float[TH / 2 > 0 ? TH / 2 : 1];

// acc[t][u] += sum_k W[k][u] x[k]: the input gradient of a Linear layer
// (dIn = W^T dOut).  LDS mode (GW = false): w is a staged W^T image [u][k]
// with leading dim ld.  Global mode (GW, H = 128 where the images do not fit
// next to the item buffers): w is the row-major torch weight [k][u] itself
// (ld = its row length), read transposed from L2 — consecutive lanes read
// consecutive u, so every load is two 128-B segments.
template <int TH, int TK, bool GW>
SGNN_DEV void matvec_t(f32x16 (&acc)[TH], const float* w, int ld, const f32x16 (&x)[TK]) {
  if constexpr (!GW) {
    mfma_from_acc<TH, TK>(acc, w, ld, 0, x);
  } else {
    // Buffer loads: per-lane part of the address in one VGPR, the row in a
    // scalar offset, the 32-unit tile in the immediate.  (Plain pointers make
    // the compiler hoist 32*TH*TK 64-bit addresses out of the item loop.)
    const int l = lane_id() & 31, h = lane_id() >> 5;
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(w), (short)0, 0x7ffffff0, 0x00020000);
    const int voff = 4 * (4 * h * ld + l);
    if constexpr (TH < 4) {
      // H = 64 (k_uv_bwd64: two waves per SIMD hide the round trip; the prefetch registers spilled
      // there, C2 training +0.5-1 %, profiles/r06_ab_gw_prefetch.txt): one group at a time
#pragma unroll
      for (int s = 0; s < 4 * TK; ++s)
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          float wv[TH];
#pragma unroll
          for (int t = 0; t < TH; ++t)
            wv[t] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
                rs, voff + 128 * t, 4 * (32 * (s >> 2) + 8 * (s & 3) + c) * ld, 0));
#pragma unroll
          for (int t = 0; t < TH; ++t) acc[t] = mfma32(wv[t], x[s >> 2][4 * (s & 3) + c], acc[t]);
        }
      return;
    }
    // H = 128 (one wave per SIMD): one k-group (4 k-steps x TH tiles) of weights in flight ahead of the
    // group being multiplied (the compiler's own schedule waited one L2 round trip per TH MFMAs); same
    // products, same order
    constexpr int NG = 4 * TK;
    float wv[2][4][TH];
    auto fetch = [&](float (&dst)[4][TH], int s) {
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int soff = 4 * (32 * (s >> 2) + 8 * (s & 3) + c) * ld;
#pragma unroll
        for (int t = 0; t < TH; ++t)
          dst[c][t] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, voff + 128 * t, soff, 0));
      }
    };
    fetch(wv[0], 0);
#pragma unroll
    for (int s = 0; s < NG; ++s) {
      if (s + 1 < NG) fetch(wv[(s + 1) & 1], s + 1);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int t = 0; t < TH; ++t) acc[t] = mfma32(wv[s & 1][c][t], x[s >> 2][4 * (s & 3) + c], acc[t]);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
}

// Per-wave item images in LDS: the workgroup's [128 items][units] operands of
// the weight-gradient outer products.
struct Imgs {
  float *bufA, *bufB, *sA, *sB;
  int lda, ldb, j;
};

SGNN_DEV Imgs make_imgs(float* bufA, int lda, float* bufB, int ldb) {
  const int w = wave_id();
  return Imgs{bufA, bufB, bufA + w * 32 * lda, bufB + w * 32 * ldb, lda, ldb, lane_id() & 31};
}

template <int TH>
SGNN_DEV void relu_mask(f32x16 (&d)[TH], const f32x16 (&act)[TH], bool valid) {
#pragma unroll
  for (int t = 0; t < TH; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) d[t][r] = (valid && act[t][r] > 0.0f) ? d[t][r] : 0.0f;
}

// Backward of one hidden Linear + the ReLU in front of it:
//   dW += dy (x) act, db += dy, dact = (W^T dy) * [act > 0]
// (act = post-ReLU input of the layer, zeroed for invalid items).
template <int TH, bool GW, int NT>
SGNN_DEV void hidden_linear_bwd(const f32x16 (&dy)[TH], const f32x16 (&act)[TH], const float* w,
                                int ld, bool valid, int nvalid, const Imgs& im, f32x16 (&acc)[NT],
                                LaneVec<TH>& s_b, f32x16 (&dact)[TH]) {
  lds_store_items<TH>(im.sA, im.lda, im.j, dy);
  lds_store_items<TH>(im.sB, im.ldb, im.j, act);
  wave_lds_sync();
  lane_sums<TH>(s_b, im.sA, im.lda, nvalid);
  __syncthreads();
  outer_tiles<NT>(acc, TH, TH, im.bufA, im.lda, 0, im.bufB, im.ldb, 0);
  __syncthreads();
  zero<TH>(dact);
  matvec_t<TH, TH, GW>(dact, w, ld, dy);
  relu_mask<TH>(dact, act, valid);
}

// Backward of LN(LAST(relu(MID(h1)))) (NL = 3) or LN(LAST(h1)) (NL = 2)
// from dm = dL/d(LN output): LayerNorm affine sums, last (+ middle) Linear
// weight/bias gradients, and dh1 = dL/d(pre-ReLU first hidden).
template <int TH, int NL, bool GW, int NT>
SGNN_DEV void ln_mlp_tail_bwd(const f32x16 (&dm_in)[TH], const f32x16 (&yh_in)[TH], float rs,
                              const float* gam, const f32x16 (&h1)[TH], const f32x16 (&h2)[TH],
                              const float* wl, int ldl, const float* wm, int ldm, bool valid,
                              int nvalid, const Imgs& im, f32x16 (&acc_wl)[NT],
                              f32x16 (&acc_wm)[NT], LaneVec<TH>& s_db, LaneVec<TH>& s_dg,
                              LaneVec<TH>& s_dbl, LaneVec<TH>& s_dbm, f32x16 (&dh1)[TH]) {
  f32x16 dm[TH], dy[TH];
#pragma unroll
  for (int t = 0; t < TH; ++t) dm[t] = dm_in[t];
  zero_if<TH>(dm, !valid);
  acc_layernorm_bwd<TH>(dm, yh_in, rs, gam, dy);
  zero_if<TH>(dy, !valid);
  {
    // d beta = sum dm, d gamma = sum dm * yhat (graph_network.py:148 LayerNorm)
    f32x16 t2[TH];
#pragma unroll
    for (int t = 0; t < TH; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) t2[t][r] = valid ? yh_in[t][r] * dm[t][r] : 0.0f;
    lds_store_items<TH>(im.sA, im.lda, im.j, dm);
    lds_store_items<TH>(im.sB, im.ldb, im.j, t2);
    wave_lds_sync();
    lane_sums<TH>(s_db, im.sA, im.lda, nvalid);
    lane_sums<TH>(s_dg, im.sB, im.ldb, nvalid);
    wave_lds_sync();
  }
  if constexpr (NL == 3) {
    f32x16 d2[TH];
    hidden_linear_bwd<TH, GW, NT>(dy, h2, wl, ldl, valid, nvalid, im, acc_wl, s_dbl, d2);
    hidden_linear_bwd<TH, GW, NT>(d2, h1, wm, ldm, valid, nvalid, im, acc_wm, s_dbm, dh1);
  } else {
    hidden_linear_bwd<TH, GW, NT>(dy, h1, wl, ldl, valid, nvalid, im, acc_wl, s_dbl, dh1);
  }
}

// Slab layouts (floats; W = kWaves partial rows per vector).  Matrices first,
// then vectors; kept in sync with training.py's reduction table.
struct SlabLayout {
  int64_t total, vb;
};

SGNN_HOST_DEV inline int64_t slab_nmat_floats(int kind, int64_t H, int64_t fpad, int nl) {
  const int64_t mid = nl == 3 ? H * H : 0;
  switch (kind) {
    case SGNN_SLAB_EDGE: return 2 * H * H + mid;            // dWl | dW1e | dWm
    case SGNN_SLAB_NODE: return 3 * H * H + mid;            // dWl | dW1[H][2H] | dWm
    case SGNN_SLAB_UV: return 2 * H * H;                    // dW1[H][2H] (i | j)
    case SGNN_SLAB_DECODER: return 32 * H + H * H + mid;    // dWl[32][H] | dW1 | dWm
    case SGNN_SLAB_ENC_NODE: return H * H + H * fpad + mid; // dWl | dW1[H][fpad] | dWm
    case SGNN_SLAB_ENC_EDGE: return H * H + H * 32 + mid;   // dWl | dW1[H][32] | dWm
    default: return -1;
  }
}

SGNN_HOST_DEV inline int64_t slab_nvec_floats(int kind, int64_t H, int nl) {
  const int64_t W = kWaves, mid = nl == 3 ? W * H : 0;
  switch (kind) {
    case SGNN_SLAB_EDGE: return 3 * W * H + mid;                  // dbl dg db | dbm
    case SGNN_SLAB_NODE: return 4 * W * H + mid;                  // db1 dbl dg db | dbm
    case SGNN_SLAB_UV: return W * H;                              // db1
    case SGNN_SLAB_DECODER: return W * 32 + W * H + W * 8 + mid;  // dbl[32] db1 loss[8] | dbm
    case SGNN_SLAB_ENC_NODE: return 4 * W * H + mid + 32 * H;     // db1 dbl dg db | dbm | G[32][H]
    case SGNN_SLAB_ENC_EDGE: return 4 * W * H + mid;              // db1 dbl dg db | dbm
    default: return -1;
  }
}

// ===========================================================================
// Edge layer backward
struct EdgeBwdArgs {
  const float* dagg;
  const int32_t *rowptr, *send, *recv;
  int64_t n;
  const float *hs, *hs2, *yh, *rstd, *e0t;
  float e_scale;
  const float *wl, *wm, *we, *gamma;  // we = edge W1 + 2H (ld 3H)
  float *du, *cin, *cout, *dh_rows, *de0t;
  int de0_accumulate;
  float* slab;
  int64_t slab_stride;
  // hidden 128, nlin 3 with yh == NULL: the middle / last Linear's biases (the forward's h2 and yhat are
  // recomputed from h in k_edge_items instead of saved)
  const float *bm = nullptr, *bl = nullptr;
};

// W1E: this layer's dE0 / dW1e products run in-layer (de0t != NULL, the
// multi-scale path); single-scale H = 64 training leaves them to
// k_edge_latent_grad, so that variant carries no dW1e accumulator or e0 image.
template <int TH, int NL, bool W1E>
__global__ __launch_bounds__(kBlock) void k_edge_bwd(EdgeBwdArgs a) {
  constexpr bool GW = TH > 2;
  constexpr int H = 32 * TH, ldh = H + 4;
  constexpr int ldl = GW ? H : ldh, lde = GW ? 3 * H : ldh;
  extern __shared__ float lds[];
  float* p = lds;
  const float* WlT = a.wl;
  const float* WmT = a.wm;
  const float* WeT = a.we;
  if (!GW) {
    stage_matrix_t(p, ldh, a.wl, H, H, H, H, H);
    WlT = p;
    p += H * ldh;
    if (W1E) {  // only the in-layer dE0 product needs W1e^T (the host sizes LDS to match)
      stage_matrix_t(p, ldh, a.we, 3 * H, H, H, H, H);
      WeT = p;
      p += H * ldh;
    }
    if (NL == 3) {
      stage_matrix_t(p, ldh, a.wm, H, H, H, H, H);
      WmT = p;
      p += H * ldh;
    }
  }
  float* gam = p;
  float* bufA = gam + H;
  float* bufB = bufA + kChunk * ldh;
  stage_vec(gam, a.gamma, H, H);
  __syncthreads();
  const Imgs im = make_imgs(bufA, ldh, bufB, ldh);
  const int j = im.j, w = wave_id();
  constexpr int NT = (TH * TH + kWaves - 1) / kWaves;
  f32x16 acc_wl[NT], acc_wm[NT], acc_w1[NT];
  zero_acc<NT>(acc_wl);
  zero_acc<NT>(acc_wm);
  zero_acc<NT>(acc_w1);
  LANEVEC(s_dbl);
  LANEVEC(s_dbm);
  LANEVEC(s_dg);
  LANEVEC(s_db);
  const int64_t E = a.rowptr[a.n];
  const int64_t nchunks = (E + kChunk - 1) / kChunk;
  const int64_t G = gridDim.x;
  // The chunk's inputs are loaded one chunk ahead (its receiver ids two
  // ahead, so the d agg row gather never waits on them): the gathers and the
  // tiled saves of chunk c + G are in flight while chunk c computes.
  auto recv_of = [&](int64_t c) -> int {
    const int64_t base = (c * kWaves + w) * 32, e = base + j;
    return (c < nchunks && base < E) ? a.recv[e < E ? e : E - 1] : 0;
  };
  auto fetch = [&](int64_t c, int rv, f32x16 (&dm)[TH], f32x16 (&yh)[TH], f32x16 (&h1)[TH],
                   f32x16 (&h2)[TH], float& rs, int& prv, int& nxt) {
    const int64_t tile = c * kWaves + w, base = tile * 32, e = base + j;
    if (c < nchunks && base < E) {  // tiles past the last valid one are not allocated
      load_row_clayout<TH>(dm, a.dagg + (int64_t)rv * H);
      load_tiled<TH>(yh, a.yh + tile * (32 * H));
      load_tiled<TH>(h1, a.hs + tile * (32 * H));
      if (NL == 3) load_tiled<TH>(h2, a.hs2 + tile * (32 * H));
      rs = a.rstd[e < E ? e : E - 1];
      // receivers around the tile: lane 0 reads the one before, lane 1 the
      // one after, as one divergent load (a uniform-address load would be
      // read into an SGPR at once -- a wait on every prefetch in flight);
      // segment_sum_store takes them with readlane
      const int64_t q = j == 0 ? base - 1 : base + 32;
      const bool has = j == 0 ? base > 0 : base + 32 < E;
      prv = has ? a.recv[has ? q : base] : -1;
      nxt = prv;
    } else {
      zero<TH>(dm);
      zero<TH>(yh);
      zero<TH>(h1);
      if (NL == 3) zero<TH>(h2);
      rs = 0.0f;
      prv = nxt = -1;
    }
  };
  f32x16 dm[TH], yh[TH], h1[TH], h2[TH];
  float rs;
  int prv, nxt;
  int rv = recv_of(blockIdx.x);
  fetch(blockIdx.x, rv, dm, yh, h1, h2, rs, prv, nxt);
  int rv_n = recv_of(blockIdx.x + G);
  // drain the first chunk's loads: the waitcnt pass merges this preheader
  // state into the loop header and would otherwise make every iteration wait
  // for its own freshly issued prefetch
  __builtin_amdgcn_s_waitcnt(0);
  for (int64_t c = blockIdx.x; c < nchunks; c += G) {
    const int64_t tile = c * kWaves + w, base = tile * 32, e = base + j;
    const int nvalid = clamp_items(E - base);
    const bool valid = e < E;
    f32x16 dm_n[TH], yh_n[TH], h1_n[TH], h2_n[TH];
    float rs_n;
    int prv_n, nxt_n;
    fetch(c + G, rv_n, dm_n, yh_n, h1_n, h2_n, rs_n, prv_n, nxt_n);
    const int rv_n2 = recv_of(c + 2 * G);
    zero_if<TH>(h1, !valid);
    if (NL == 3) zero_if<TH>(h2, !valid);
    f32x16 dh[TH];
    ln_mlp_tail_bwd<TH, NL, GW, NT>(dm, yh, rs, gam, h1, h2, WlT, ldl, WmT, ldl, valid, nvalid, im,
                                    acc_wl, acc_wm, s_db, s_dg, s_dbl, s_dbm, dh);
    f32x16 e0[TH];
    zero<TH>(e0);
    if (W1E && nvalid > 0) {
      // dE0 += 2^k W1e^T dh (the edge latent feeding layer k is 2^k e0)
      f32x16 de[TH];
      zero<TH>(de);
      matvec_t<TH, TH, GW>(de, WeT, lde, dh);
      float* dtile = a.de0t + tile * (32 * H);
      if (a.de0_accumulate & 1) {
        f32x16 old[TH];
        load_tiled<TH>(old, dtile);
#pragma unroll
        for (int t = 0; t < TH; ++t)
#pragma unroll
          for (int r = 0; r < 16; ++r) de[t][r] = old[t][r] + de[t][r] * a.e_scale;
      } else {
#pragma unroll
        for (int t = 0; t < TH; ++t)
#pragma unroll
          for (int r = 0; r < 16; ++r) de[t][r] *= a.e_scale;
      }
      store_tiled<TH>(dtile, de);
    }
    // !W1E: sgnn_edge_latent_grad forms dE0 and dW1e of this layer
    constexpr bool w1e_here = W1E;
    store_row_clayout_if<TH>(buf_rsrc(a.dh_rows + base * H), j * (4 * H), valid, dh);
    if (w1e_here) {
      if (nvalid > 0) {
        load_tiled<TH>(e0, a.e0t + tile * (32 * H));
        zero_if<TH>(e0, !valid);
      }
      lds_store_items<TH>(im.sA, ldh, j, dh);
      lds_store_items<TH>(im.sB, ldh, j, e0);
      __syncthreads();
      outer_tiles<NT>(acc_w1, TH, TH, bufA, ldh, 0, bufB, ldh, 0);  // dW1e = sum dh (x) e0
      __syncthreads();
    }
    // dU: receiver segment sums of dh (overwrites dh)
    segment_sum_rows<TH>(dh, rv, valid, __builtin_amdgcn_readlane(prv, 0), __builtin_amdgcn_readlane(nxt, 1),
                         tile, a.du, a.cin, a.cout);
#pragma unroll
    for (int t = 0; t < TH; ++t) {
      dm[t] = dm_n[t];
      yh[t] = yh_n[t];
      h1[t] = h1_n[t];
      if (NL == 3) h2[t] = h2_n[t];
    }
    rs = rs_n;
    prv = prv_n;
    nxt = nxt_n;
    rv = rv_n;
    rv_n = rv_n2;
  }
  float* slab = a.slab + blockIdx.x * a.slab_stride;
  store_outer<NT>(slab, H, TH, TH, acc_wl);
  if (W1E) store_outer<NT>(slab + H * H, H, TH, TH, acc_w1);
  if (NL == 3) store_outer<NT>(slab + 2 * H * H, H, TH, TH, acc_wm);
  float* v = slab + slab_nmat_floats(SGNN_SLAB_EDGE, H, 0, NL);
  store_lane_vec<TH>(v, s_dbl);
  store_lane_vec<TH>(v + kWaves * H, s_dg);
  store_lane_vec<TH>(v + 2 * kWaves * H, s_db);
  if (NL == 3) store_lane_vec<TH>(v + 3 * kWaves * H, s_dbm);
}

// ---------------------------------------------------------------------------
// The single-scale training variant at H = 64 (NL = 2, dE0 / dW1e left to the
// latent pass), sized for TWO workgroups per CU: LDS = Wl^T (16 KB) + the two
// [128 items][64] item images (32 KB each) = 80 KB, with no row padding --
// rows are XOR-swizzled in 16-B groups instead (swz) -- and LayerNorm gamma
// read from L2; <= 256 VGPRs.  Two independent workgroups per CU interleave
// one's MFMA phases with the other's LayerNorm / gather / segment-sum phases,
// which a single 4-wave workgroup (1 wave per SIMD) runs back to back.
SGNN_DEV int swz(int r, int u) { return r * 64 + (u ^ ((r & 15) << 2)); }

// 0 from an opaque move: per-lane offsets derived from it are recomputed at
// each use instead of being hoisted out of the caller's chunk loop, where the
// unrolled helpers below would otherwise keep dozens of address VGPRs live.
SGNN_DEV int opaque_zero() {
  int z;
  asm volatile("v_mov_b32 %0, 0" : "=v"(z));
  return z;
}

// scale * W^T of a [64 out k][64 in u] block (leading dim ldw, 16-B aligned)
// into a swizzled [u][k] image: four float4 loads per thread issued
// together, then written transposed.
SGNN_DEV void swz_stage_wt(float* wt, const float* w, int ldw, float scale) {
  static_assert(kBlock == 256, "W staging: 16 floats per thread");
  const int t = threadIdx.x, u0 = 4 * (t & 15), k0 = t >> 4;
  f32x4 wv[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) wv[i] = ld4(w + (k0 + 16 * i) * ldw + u0) * scale;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int c = 0; c < 4; ++c) wt[swz(u0 + c, k0 + 16 * i)] = wv[i][c];
}

// Item-on-lane register tile -> swizzled [item][64] image row `item`.
SGNN_DEV void swz_store_items(float* img, int item, const f32x16 (&x)[2]) {
  const int h = lane_id() >> 5;
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      f32x4 v;
#pragma unroll
      for (int c = 0; c < 4; ++c) v[c] = x[t][4 * g + c];
      st4(img + swz(item, 32 * t + 8 * g + 4 * h), v);
    }
}

// Column sums of a wave's 32 swizzled image rows (rows past nvalid hold
// zeros) with 16-B reads: lane L reads unit group L & 15 of rows
// (L >> 4) + 4k, then a butterfly over the four row phases.  Every lane ends
// with units 4 (L & 15) + c.  Row (L >> 4) + 4k has XOR term
// 4 (L >> 4) + 16 (k & 3): four per-lane offsets, the row in the immediate.
SGNN_DEV f32x4 swz_col_sums(const float* slice) {
  const int L = lane_id(), ug = L & 15, ro = L >> 4;
  const int cc = ro * 64 + ((4 * ug) ^ (4 * ro));
  f32x4 s0 = {0.0f, 0.0f, 0.0f, 0.0f}, s1 = s0;
#pragma unroll
  for (int k = 0; k < 8; k += 2) {
    s0 += ld4(slice + (cc ^ (16 * (k & 3))) + 256 * k);
    s1 += ld4(slice + (cc ^ (16 * ((k + 1) & 3))) + 256 * (k + 1));
  }
  s0 += s1;
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    s0[c] += __shfl_xor(s0[c], 16, 64);
    s0[c] += __shfl_xor(s0[c], 32, 64);
  }
  return s0;
}

// mfma_outer over the 128 items of two swizzled images (one 32x32 tile).
// Row 2s + h has (row & 15) = 2(s & 7) + h, so its XOR term is 8(s & 7) ^ 4h:
// eight per-lane column offsets per operand, the row in the immediate.
SGNN_DEV void swz_outer(f32x16& acc, const float* A, int ua, const float* B, int vb) {
  constexpr int G = 4, NS = kChunk / 2;
  const int l = (lane_id() & 31) + opaque_zero(), h = lane_id() >> 5;
  const int ca = h * 64 + ((ua + l) ^ (4 * h)), cb = h * 64 + ((vb + l) ^ (4 * h));
  auto ra = [&](int s) { return A[(ca ^ (8 * (s & 7))) + 128 * s]; };
  auto rb = [&](int s) { return B[(cb ^ (8 * (s & 7))) + 128 * s]; };
  float a0[G], b0[G], a1[G], b1[G];
#pragma unroll
  for (int i = 0; i < G; ++i) {
    a0[i] = ra(i);
    b0[i] = rb(i);
  }
#pragma unroll
  for (int s = 0; s < NS; s += 2 * G) {
#pragma unroll
    for (int i = 0; i < G; ++i) {
      a1[i] = ra(s + G + i);
      b1[i] = rb(s + G + i);
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < G; ++i) acc = mfma32(a0[i], b0[i], acc);
    if (s + 2 * G < NS) {
#pragma unroll
      for (int i = 0; i < G; ++i) {
        a0[i] = ra(s + 2 * G + i);
        b0[i] = rb(s + 2 * G + i);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < G; ++i) acc = mfma32(a1[i], b1[i], acc);
  }
}

// acc[t][u] += sum_k W[k][u] x[k] with W^T staged swizzled ([u][k] image)
SGNN_DEV void swz_matvec_t(f32x16 (&acc)[2], const float* wt, const f32x16 (&x)[2]) {
  const int l = lane_id() & 31, h = lane_id() >> 5;
#pragma unroll
  for (int tk = 0; tk < 2; ++tk)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      f32x4 w[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) w[t] = ld4(wt + swz(32 * t + l, 32 * tk + 8 * g + 4 * h));
#pragma unroll
      for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int t = 0; t < 2; ++t) acc[t] = mfma32(w[t][c], x[tk][4 * g + c], acc[t]);
    }
}

// DW1E: this layer's dW1e = sum_e dh (x) e0 as well (the caller's
// de0_accumulate bit 1), through the same two item images after the dWl
// product: one more outer product per chunk instead of a separate
// k_edge_w1e_grad launch that re-reads the dh rows.
template <bool DW1E>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(2)))
void k_edge_bwd64(EdgeBwdArgs a) {
  constexpr int TH = 2, H = 64;
  extern __shared__ float lds[];
  float* wt = lds;                  // Wl^T [u][k]
  float* bufA = wt + H * H;         // [128 items][64]
  float* bufB = bufA + kChunk * H;
  swz_stage_wt(wt, a.wl, H, 1.0f);
  __syncthreads();
  const int w = wave_id(), l = lane_id(), j = l & 31;
  float* sA = bufA + w * 32 * H;    // this wave's rows (w*32 + j; (row & 15) == (j & 15))
  float* sB = bufB + w * 32 * H;
  const int tu = w >> 1, tv = w & 1;   // the wave's dWl tile
  f32x16 acc, acc_e;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = acc_e[r] = 0.0f;
  f32x4 s_dbl = {0.0f, 0.0f, 0.0f, 0.0f}, s_dg = s_dbl, s_db = s_dbl;   // units 4 (lane & 15) + c
  const int64_t E = a.rowptr[a.n];
  const int64_t nchunks = (E + kChunk - 1) / kChunk;
  for (int64_t c = blockIdx.x; c < nchunks; c += gridDim.x) {
    const int64_t tile = c * kWaves + w, base = tile * 32, e = base + j;
    const int nvalid = clamp_items(E - base);
    const bool valid = e < E;
    f32x16 dm[TH], yh[TH], h1[TH];
    float rs = 0.0f;
    int rv = 0, nb = -1;
    if (nvalid > 0) {  // tiles past the last valid one are not allocated
      const int64_t ec = valid ? e : E - 1;
      rv = a.recv[ec];
      load_row_clayout<TH>(dm, a.dagg + (int64_t)rv * H);
      load_tiled<TH>(yh, a.yh + tile * (32 * H));
      load_tiled<TH>(h1, a.hs + tile * (32 * H));
      rs = a.rstd[ec];
      // receivers around the tile: lane 0 the one before, lane 1 the one after
      const int64_t q = j == 0 ? base - 1 : base + 32;
      const bool has = j == 0 ? base > 0 : base + 32 < E;
      nb = has ? a.recv[has ? q : base] : -1;
    } else {
      zero<TH>(dm);
      zero<TH>(yh);
      zero<TH>(h1);
    }
    zero_if<TH>(dm, !valid);
    zero_if<TH>(h1, !valid);
    // LayerNorm backward (graph_network.py:148), its affine sums
    f32x16 dy[TH];
    acc_layernorm_bwd<TH>(dm, yh, rs, a.gamma, dy);
    zero_if<TH>(dy, !valid);
#pragma unroll
    for (int t = 0; t < TH; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) yh[t][r] *= dm[t][r];   // dgamma terms (dm = 0 off the edges)
    swz_store_items(sA, j, dm);
    swz_store_items(sB, j, yh);
    wave_lds_sync();
    s_db += swz_col_sums(sA);
    s_dg += swz_col_sums(sB);
    wave_lds_sync();
    // last Linear: dWl += dy (x) h1, dbl += dy, dh = (Wl^T dy) * [h1 > 0]
    swz_store_items(sA, j, dy);
    swz_store_items(sB, j, h1);
    wave_lds_sync();
    s_dbl += swz_col_sums(sA);
    __syncthreads();
    swz_outer(acc, bufA, 32 * tu, bufB, 32 * tv);
    __syncthreads();
    f32x16 dh[TH];
    zero<TH>(dh);
    swz_matvec_t(dh, wt, dy);
    relu_mask<TH>(dh, h1, valid);
    store_row_clayout_if<TH>(buf_rsrc(a.dh_rows + base * H), j * (4 * H), valid, dh);
    if constexpr (DW1E) {
      // dW1e += dh (x) e0 (the 2^k of the latent is applied in the slab reduction)
      f32x16 e0[TH];
      if (nvalid > 0) load_tiled<TH>(e0, a.e0t + tile * (32 * H));
      else zero<TH>(e0);
      zero_if<TH>(e0, !valid);
      swz_store_items(sA, j, dh);
      swz_store_items(sB, j, e0);
      __syncthreads();
      swz_outer(acc_e, bufA, 32 * tu, bufB, 32 * tv);
      __syncthreads();
    }
    segment_sum_rows<TH>(dh, rv, valid, __builtin_amdgcn_readlane(nb, 0), __builtin_amdgcn_readlane(nb, 1),
                         tile, a.du, a.cin, a.cout);
  }
  float* slab = a.slab + blockIdx.x * a.slab_stride;
  store_tile_rowmajor(slab + (32 * tu) * H + 32 * tv, H, acc);
  if constexpr (DW1E) store_tile_rowmajor(slab + H * H + (32 * tu) * H + 32 * tv, H, acc_e);
  float* v = slab + slab_nmat_floats(SGNN_SLAB_EDGE, H, 0, 2);
  if (l < 16) {
    st4(v + w * H + 4 * l, s_dbl);
    st4(v + kWaves * H + w * H + 4 * l, s_dg);
    st4(v + 2 * kWaves * H + w * H + 4 * l, s_db);
  }
}


// ===========================================================================
// Node layer backward (graph_network.py:201-222 + residual :176)
struct NodeBwdArgs {
  const float* g;  // dL/dx_out
  int64_t n;
  const float *yh, *rstd, *hn, *hn2, *agg, *x;
  const float *w1, *wl, *wm, *gamma;
  float *dagg, *dxp;
  float* slab;
  int64_t slab_stride;
};

template <int TH, int NL>
__global__ __launch_bounds__(kBlock) void k_node_bwd(NodeBwdArgs a) {
  constexpr bool GW = TH > 2;
  constexpr int H = 32 * TH, ldh = H + 4;
  constexpr int ldl = GW ? H : ldh, ld1 = GW ? 2 * H : ldh;
  extern __shared__ float lds[];
  float* p = lds;
  const float* WlT = a.wl;
  const float* WmT = a.wm;
  const float* W1T = a.w1;  // W1T[i][k] = W1[k][i], i < 2H
  if (!GW) {
    stage_matrix_t(p, ldh, a.wl, H, H, H, H, H);
    WlT = p;
    p += H * ldh;
    stage_matrix_t(p, ldh, a.w1, 2 * H, H, 2 * H, H, 2 * H);
    W1T = p;
    p += 2 * H * ldh;
    if (NL == 3) {
      stage_matrix_t(p, ldh, a.wm, H, H, H, H, H);
      WmT = p;
      p += H * ldh;
    }
  }
  // agg / x halves of W1^T: LDS rows 0..H-1 / H..2H-1; global columns 0.. / H..
  const float* W1aT = W1T;
  const float* W1xT = GW ? a.w1 + H : W1T + H * ldh;
  float* gam = p;
  float* bufA = gam + H;
  float* bufB = bufA + kChunk * ldh;
  stage_vec(gam, a.gamma, H, H);
  __syncthreads();
  const Imgs im = make_imgs(bufA, ldh, bufB, ldh);
  const int j = im.j, w = wave_id();
  constexpr int NT = (TH * TH + kWaves - 1) / kWaves;
  f32x16 acc_wl[NT], acc_wm[NT], acc_w1a[NT], acc_w1x[NT];
  zero_acc<NT>(acc_wl);
  zero_acc<NT>(acc_wm);
  zero_acc<NT>(acc_w1a);
  zero_acc<NT>(acc_w1x);
  LANEVEC(s_dbl);
  LANEVEC(s_dbm);
  LANEVEC(s_dg);
  LANEVEC(s_db);
  LANEVEC(s_db1);
  const int64_t nchunks = (a.n + kChunk - 1) / kChunk;
  for (int64_t c = blockIdx.x; c < nchunks; c += gridDim.x) {
    const int64_t i = c * kChunk + w * 32 + j;
    const int nvalid = clamp_items(a.n - (c * kChunk + w * 32));
    const bool valid = i < a.n;
    const int64_t ic = valid ? i : a.n - 1;
    f32x16 gi[TH], yh[TH], h1[TH], h2[TH], dh[TH];
    load_row_clayout<TH>(gi, a.g + ic * H);
    zero_if<TH>(gi, !valid);
    load_row_clayout<TH>(yh, a.yh + ic * H);
    load_row_clayout<TH>(h1, a.hn + ic * H);
    zero_if<TH>(h1, !valid);
    if (NL == 3) {
      load_row_clayout<TH>(h2, a.hn2 + ic * H);
      zero_if<TH>(h2, !valid);
    }
    ln_mlp_tail_bwd<TH, NL, GW, NT>(gi, yh, a.rstd[ic], gam, h1, h2, WlT, ldl, WmT, ldl, valid,
                                    nvalid, im, acc_wl, acc_wm, s_db, s_dg, s_dbl, s_dbm, dh);
    {
      f32x16 ag[TH];
      load_row_clayout<TH>(ag, a.agg + ic * H);
      zero_if<TH>(ag, !valid);
      lds_store_items<TH>(im.sA, ldh, j, dh);
      lds_store_items<TH>(im.sB, ldh, j, ag);
      wave_lds_sync();
      lane_sums<TH>(s_db1, im.sA, ldh, nvalid);
      __syncthreads();
      outer_tiles<NT>(acc_w1a, TH, TH, bufA, ldh, 0, bufB, ldh, 0);  // dW1[:, :H] = dh (x) agg
      __syncthreads();
    }
    {
      f32x16 xx[TH];
      load_row_clayout<TH>(xx, a.x + ic * H);
      zero_if<TH>(xx, !valid);
      lds_store_items<TH>(im.sB, ldh, j, xx);
      __syncthreads();
      outer_tiles<NT>(acc_w1x, TH, TH, bufA, ldh, 0, bufB, ldh, 0);  // dW1[:, H:] = dh (x) x
      __syncthreads();
    }
    // d agg = W1[:, :H]^T dh ; dx' = g + W1[:, H:]^T dh
    f32x16 o[TH];
    zero<TH>(o);
    matvec_t<TH, TH, GW>(o, W1aT, ld1, dh);
    if (valid) store_row_clayout<TH>(a.dagg + i * H, o);
    matvec_t<TH, TH, GW>(gi, W1xT, ld1, dh);
    if (valid) store_row_clayout<TH>(a.dxp + i * H, gi);
  }
  float* slab = a.slab + blockIdx.x * a.slab_stride;
  store_outer<NT>(slab, H, TH, TH, acc_wl);
  store_outer<NT>(slab + H * H, 2 * H, TH, TH, acc_w1a);
  store_outer<NT>(slab + H * H + H, 2 * H, TH, TH, acc_w1x);
  if (NL == 3) store_outer<NT>(slab + 3 * H * H, H, TH, TH, acc_wm);
  float* v = slab + slab_nmat_floats(SGNN_SLAB_NODE, H, 0, NL);
  store_lane_vec<TH>(v, s_db1);
  store_lane_vec<TH>(v + kWaves * H, s_dbl);
  store_lane_vec<TH>(v + 2 * kWaves * H, s_dg);
  store_lane_vec<TH>(v + 3 * kWaves * H, s_db);
  if (NL == 3) store_lane_vec<TH>(v + 4 * kWaves * H, s_dbm);
}

// ===========================================================================
// u/v projections backward: g = dx' + W1i^T dU + W1j^T dV
struct UvBwdArgs {
  const float* dxp;
  const float *du, *cin, *cout;
  const int32_t* rowptr;
  const float* dh_rows;
  const int32_t *tptr, *tperm;
  const float* x;
  int64_t n;
  const float* w1;  // edge W1 [H][3H]
  float* g;
  float* slab;
  int64_t slab_stride;
};

// H = 64 variant sized for two workgroups per CU (512 workgroups: every
// 128-node chunk of a 50k graph resident at once instead of 1.5 rounds at
// one per CU): Wi^T as a swizzled 16 KB LDS image, Wj^T read from L2, the two
// unpadded swizzled item images (64 KB) -- 80 KB -- and <= 256 VGPRs.
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(2)))
void k_uv_bwd64(UvBwdArgs a) {
  constexpr int TH = 2, H = 64;
  extern __shared__ float lds[];
  float* wi = lds;                  // Wi^T [u][k]
  float* bufA = wi + H * H;         // [128 items][64]
  float* bufB = bufA + kChunk * H;
  swz_stage_wt(wi, a.w1, 3 * H, 1.0f);
  __syncthreads();
  const int w = wave_id(), l = lane_id(), j = l & 31;
  float* sA = bufA + w * 32 * H;
  float* sB = bufB + w * 32 * H;
  const int tu = w >> 1, tv = w & 1;
  f32x16 acc_i, acc_j;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc_i[r] = acc_j[r] = 0.0f;
  f32x4 s_db1 = {0.0f, 0.0f, 0.0f, 0.0f};   // units 4 (lane & 15) + c
  const int64_t nchunks = (a.n + kChunk - 1) / kChunk;
  for (int64_t c = blockIdx.x; c < nchunks; c += gridDim.x) {
    const int64_t i = c * kChunk + w * 32 + j;
    const bool valid = i < a.n;
    const int64_t ic = valid ? i : a.n - 1;
    f32x16 du[TH], dv[TH], xx[TH], gg[TH];
    load_resolved<TH>(du, a.du, a.cin, a.cout, a.rowptr, ic);
    zero<TH>(dv);
    for (int32_t t = a.tptr[ic], t1 = a.tptr[ic + 1]; t < t1; ++t)
      add_row_clayout<TH>(dv, a.dh_rows + (int64_t)a.tperm[t] * H);
    zero_if<TH>(du, !valid);
    zero_if<TH>(dv, !valid);
    load_row_clayout<TH>(xx, a.x + ic * H);
    zero_if<TH>(xx, !valid);
    load_row_clayout<TH>(gg, a.dxp + ic * H);
    // g = dx' + W1i^T dU + W1j^T dV  (graph_network.py:197 on cat[x_i, x_j, e])
    swz_matvec_t(gg, wi, du);
    matvec_t<TH, TH, true>(gg, a.w1 + H, 3 * H, dv);
    if (valid) store_row_clayout<TH>(a.g + i * H, gg);
    swz_store_items(sA, j, du);
    swz_store_items(sB, j, xx);
    wave_lds_sync();
    s_db1 += swz_col_sums(sA);
    __syncthreads();
    swz_outer(acc_i, bufA, 32 * tu, bufB, 32 * tv);   // dW1[:, 0:H] = dU (x) x
    __syncthreads();
    swz_store_items(sA, j, dv);
    __syncthreads();
    swz_outer(acc_j, bufA, 32 * tu, bufB, 32 * tv);   // dW1[:, H:2H] = dV (x) x
    __syncthreads();
  }
  float* slab = a.slab + blockIdx.x * a.slab_stride;
  store_tile_rowmajor(slab + (32 * tu) * 2 * H + 32 * tv, 2 * H, acc_i);
  store_tile_rowmajor(slab + H + (32 * tu) * 2 * H + 32 * tv, 2 * H, acc_j);
  if (l < 16) st4(slab + 2 * H * H + w * H + 4 * l, s_db1);
}

// matvec_t's global (L2) mode at H = 64 with one 16-unit k-group of weights
// in flight at a time (the unbatched form keeps all 64 loads live: spills at
// the 256-register budget of two waves per SIMD).
SGNN_DEV void gw_matvec_t64(f32x16 (&acc)[2], const float* w, int ld, const f32x16 (&x)[2]) {
  const int l = (lane_id() & 31) + opaque_zero(), h = lane_id() >> 5;
  const __amdgpu_buffer_rsrc_t rs = weight_rsrc(w);
  const int voff = 4 * (4 * h * ld + l);
#pragma unroll
  for (int tk = 0; tk < 2; ++tk)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      float wv[4][2];
#pragma unroll
      for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int t = 0; t < 2; ++t)
          wv[c][t] = __uint_as_float(
              __builtin_amdgcn_raw_buffer_load_b32(rs, voff + 128 * t, 4 * (32 * tk + 8 * g + c) * ld, 0));
#pragma unroll
      for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int t = 0; t < 2; ++t) acc[t] = mfma32(wv[c][t], x[tk][4 * g + c], acc[t]);
      __builtin_amdgcn_sched_barrier(0);
    }
}

// Node MLP backward at H = 64, NL = 2, sized for two workgroups per CU like
// k_edge_bwd64 / k_uv_bwd64: Wl^T swizzled in LDS (16 KB), W1^T's agg and x
// halves read from L2, two unpadded swizzled item images (64 KB) -- 80 KB --
// and <= 256 VGPRs (g is read again for dx' instead of kept live).
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(2)))
void k_node_bwd64(NodeBwdArgs a) {
  constexpr int TH = 2, H = 64;
  extern __shared__ float lds[];
  float* wl = lds;                  // Wl^T [u][k]
  float* bufA = wl + H * H;
  float* bufB = bufA + kChunk * H;
  swz_stage_wt(wl, a.wl, H, 1.0f);
  __syncthreads();
  const int w = wave_id(), l = lane_id(), j = l & 31;
  float* sA = bufA + w * 32 * H;
  float* sB = bufB + w * 32 * H;
  const int tu = w >> 1, tv = w & 1;
  f32x16 acc_wl, acc_wa, acc_wx;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc_wl[r] = acc_wa[r] = acc_wx[r] = 0.0f;
  f32x4 s_db1 = {0.0f, 0.0f, 0.0f, 0.0f}, s_dbl = s_db1, s_dg = s_db1, s_db = s_db1;
  const int64_t nchunks = (a.n + kChunk - 1) / kChunk;
  for (int64_t c = blockIdx.x; c < nchunks; c += gridDim.x) {
    const int64_t i = c * kChunk + w * 32 + j;
    const bool valid = i < a.n;
    const int64_t ic = valid ? i : a.n - 1;
    f32x16 dy[TH], h1[TH];
    {
      f32x16 gi[TH], yh[TH];
      load_row_clayout<TH>(gi, a.g + ic * H);
      zero_if<TH>(gi, !valid);
      load_row_clayout<TH>(yh, a.yh + ic * H);
      // LayerNorm backward (graph_network.py:219 LayerNorm) and its affine sums
      acc_layernorm_bwd<TH>(gi, yh, a.rstd[ic], a.gamma, dy);
      zero_if<TH>(dy, !valid);
#pragma unroll
      for (int t = 0; t < TH; ++t) yh[t] *= gi[t];
      swz_store_items(sA, j, gi);
      swz_store_items(sB, j, yh);
      wave_lds_sync();
      s_db += swz_col_sums(sA);
      s_dg += swz_col_sums(sB);
      wave_lds_sync();
    }
    load_row_clayout<TH>(h1, a.hn + ic * H);   // after the LayerNorm part: fewer rows live at once
    zero_if<TH>(h1, !valid);
    // last Linear: dWl += dy (x) h1, dbl += dy, dh = (Wl^T dy) * [h1 > 0]
    swz_store_items(sA, j, dy);
    swz_store_items(sB, j, h1);
    wave_lds_sync();
    s_dbl += swz_col_sums(sA);
    __syncthreads();
    swz_outer(acc_wl, bufA, 32 * tu, bufB, 32 * tv);
    __syncthreads();
    f32x16 dh[TH];
    zero<TH>(dh);
    swz_matvec_t(dh, wl, dy);
    relu_mask<TH>(dh, h1, valid);
    // first Linear on cat[agg, x] (graph_network.py:220): dW1 += dh (x) [agg, x], db1 += dh
    {
      f32x16 ag[TH];
      load_row_clayout<TH>(ag, a.agg + ic * H);
      zero_if<TH>(ag, !valid);
      swz_store_items(sA, j, dh);
      swz_store_items(sB, j, ag);
      wave_lds_sync();
      s_db1 += swz_col_sums(sA);
      __syncthreads();
      swz_outer(acc_wa, bufA, 32 * tu, bufB, 32 * tv);
      __syncthreads();
    }
    {
      f32x16 xx[TH];
      load_row_clayout<TH>(xx, a.x + ic * H);
      zero_if<TH>(xx, !valid);
      swz_store_items(sB, j, xx);
      __syncthreads();
      swz_outer(acc_wx, bufA, 32 * tu, bufB, 32 * tv);
      __syncthreads();
    }
    // d agg = W1[:, :H]^T dh ; dx' = g + W1[:, H:]^T dh (residual graph_network.py:176)
    f32x16 o[TH];
    zero<TH>(o);
    gw_matvec_t64(o, a.w1, 2 * H, dh);
    if (valid) store_row_clayout<TH>(a.dagg + i * H, o);
    load_row_clayout<TH>(o, a.g + ic * H);
    gw_matvec_t64(o, a.w1 + H, 2 * H, dh);
    if (valid) store_row_clayout<TH>(a.dxp + i * H, o);
  }
  float* slab = a.slab + blockIdx.x * a.slab_stride;
  store_tile_rowmajor(slab + (32 * tu) * H + 32 * tv, H, acc_wl);
  store_tile_rowmajor(slab + H * H + (32 * tu) * 2 * H + 32 * tv, 2 * H, acc_wa);
  store_tile_rowmajor(slab + H * H + H + (32 * tu) * 2 * H + 32 * tv, 2 * H, acc_wx);
  float* v = slab + slab_nmat_floats(SGNN_SLAB_NODE, H, 0, 2);
  if (l < 16) {
    st4(v + w * H + 4 * l, s_db1);
    st4(v + kWaves * H + w * H + 4 * l, s_dbl);
    st4(v + 2 * kWaves * H + w * H + 4 * l, s_dg);
    st4(v + 3 * kWaves * H + w * H + 4 * l, s_db);
  }
}

// ===========================================================================
// Loss (train.py:257-268) + Decoder / prediction-head backward
// (graph_network.py:321-333, multi_scale_gnn.py:275; no LayerNorm)
struct DecBwdArgs {
  const float* pred;      // [n][D+1]
  const float* pos_seq;   // noisy input window [n][T][D]
  const float* next_pos;  // [n][D]
  const float* noise;     // [n][T][D] or null
  const float* next_strain;  // [n]
  const float *acc_mean, *acc_std;
  int64_t n;
  int T, D;
  float w_pos, w_strain, inv_count;
  const float* dpred;
  const float *hd, *hd2, *x;
  const float *wd1, *wdm, *wdl;
  float* g;
  float* slab;
  int64_t slab_stride;
};

template <int TH, int NL>
__global__ __launch_bounds__(kBlock) void k_dec_bwd(DecBwdArgs a) {
  constexpr bool GW = TH > 2;
  constexpr int H = 32 * TH, ldh = H + 4, ldo = 32 + 4;
  constexpr int ld1 = GW ? H : ldh;
  extern __shared__ float lds[];
  float* WlT = lds;                 // [H][ldo]: WlT[i][k] = Wdl[k][i], k < 32 (D+1 valid)
  float* p = WlT + H * ldo;
  stage_matrix_t(WlT, ldo, a.wdl, H, a.D + 1, H, 32, H);
  const float* W1T = a.wd1;
  const float* WmT = a.wdm;
  if (!GW) {
    stage_matrix_t(p, ldh, a.wd1, H, H, H, H, H);
    W1T = p;
    p += H * ldh;
    if (NL == 3) {
      stage_matrix_t(p, ldh, a.wdm, H, H, H, H, H);
      WmT = p;
      p += H * ldh;
    }
  }
  float* bufA = p;
  float* bufB = bufA + kChunk * ldh;
  __syncthreads();
  const Imgs im = make_imgs(bufA, ldh, bufB, ldh);
  const int l = lane_id(), j = im.j, h = l >> 5, w = wave_id();
  constexpr int NT2 = (TH + kWaves - 1) / kWaves;     // [32 x H] last layer
  constexpr int NT = (TH * TH + kWaves - 1) / kWaves;
  f32x16 acc_wl[NT2], acc_wm[NT], acc_w1[NT];
  zero_acc<NT2>(acc_wl);
  zero_acc<NT>(acc_wm);
  zero_acc<NT>(acc_w1);
  float s_dbl = 0.0f;  // lane = output unit (< 32)
  LANEVEC(s_db1);
  LANEVEC(s_dbm);
  float loss_acc[5] = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f};  // total, x, y, z, strain
  const int64_t nchunks = (a.n + kChunk - 1) / kChunk;
  for (int64_t c = blockIdx.x; c < nchunks; c += gridDim.x) {
    const int64_t i = c * kChunk + w * 32 + j;
    const int nvalid = clamp_items(a.n - (c * kChunk + w * 32));
    const bool valid = i < a.n;
    const int64_t ic = valid ? i : a.n - 1;
    f32x16 dp[1];
    zero<1>(dp);
    if (valid && h == 0 && a.dpred) {
      for (int cc = 0; cc <= a.D; ++cc) dp[0][cc] = a.dpred[ic * (a.D + 1) + cc];
    } else if (valid && h == 0) {
      const int D = a.D, T = a.T;
      const float* pp = a.pos_seq + ic * T * D;
      float tot = 0.0f;
      for (int cc = 0; cc < D; ++cc) {  // learned_simulator.py:479-481, :509-517
        const float nz = a.noise ? a.noise[(ic * T + T - 1) * D + cc] : 0.0f;
        const float nxt = __fadd_rn(a.next_pos[ic * D + cc], nz);
        const float prev = pp[(T - 1) * D + cc];
        const float pvel = __fsub_rn(prev, pp[(T - 2) * D + cc]);
        const float acc = __fsub_rn(__fsub_rn(nxt, prev), pvel);
        const float tgt = __fdiv_rn(__fsub_rn(acc, a.acc_mean[cc]), a.acc_std[cc]);
        const float d = a.pred[ic * (D + 1) + cc] - tgt;
        dp[0][cc] = 2.0f * a.w_pos * d * a.inv_count;
        tot += d * d;
        loss_acc[1 + cc] += d * d;
      }
      const float ds = a.pred[ic * (D + 1) + D] - a.next_strain[ic];
      dp[0][D] = 2.0f * a.w_strain * ds * a.inv_count;
      loss_acc[0] += a.w_pos * tot + a.w_strain * ds * ds;
      loss_acc[4] += ds * ds;
    }
    constexpr int ldp = 32 + 4;
    f32x16 h1[TH], h2[TH], hl[TH];
    load_row_clayout<TH>(h1, a.hd + ic * H);
    zero_if<TH>(h1, !valid);
    if (NL == 3) {
      load_row_clayout<TH>(h2, a.hd2 + ic * H);
      zero_if<TH>(h2, !valid);
    }
#pragma unroll
    for (int t = 0; t < TH; ++t) hl[t] = NL == 3 ? h2[t] : h1[t];
    {
      // d pred image (32 units) and hl image for dWl = dpred (x) hl
      f32x4 v;
#pragma unroll
      for (int gq = 0; gq < 4; ++gq) {
#pragma unroll
        for (int cc = 0; cc < 4; ++cc) v[cc] = dp[0][4 * gq + cc];
        st4(bufA + (w * 32 + j) * ldp + 8 * gq + 4 * h, v);
      }
      lds_store_items<TH>(im.sB, ldh, j, hl);
      wave_lds_sync();
      if (l < 32) s_dbl += lane_sum(bufA + w * 32 * ldp, ldp, nvalid, l);
      __syncthreads();
      outer_tiles<NT2>(acc_wl, 1, TH, bufA, ldp, 0, bufB, ldh, 0);
      __syncthreads();
    }
    f32x16 dh[TH];
    zero<TH>(dh);
    mfma_from_acc<TH, 1>(dh, WlT, ldo, 0, dp);
    relu_mask<TH>(dh, hl, valid);
    if constexpr (NL == 3) {
      f32x16 d1[TH];
      hidden_linear_bwd<TH, GW, NT>(dh, h1, WmT, ld1, valid, nvalid, im, acc_wm, s_dbm, d1);
#pragma unroll
      for (int t = 0; t < TH; ++t) dh[t] = d1[t];
    }
    f32x16 xx[TH];
    load_row_clayout<TH>(xx, a.x + ic * H);
    zero_if<TH>(xx, !valid);
    lds_store_items<TH>(im.sA, ldh, j, dh);
    lds_store_items<TH>(im.sB, ldh, j, xx);
    wave_lds_sync();
    lane_sums<TH>(s_db1, im.sA, ldh, nvalid);
    __syncthreads();
    outer_tiles<NT>(acc_w1, TH, TH, bufA, ldh, 0, bufB, ldh, 0);
    __syncthreads();
    f32x16 gg[TH];
    zero<TH>(gg);
    matvec_t<TH, TH, GW>(gg, W1T, ld1, dh);
    if (valid) store_row_clayout<TH>(a.g + i * H, gg);
  }
  float* slab = a.slab + blockIdx.x * a.slab_stride;
  store_outer<NT2>(slab, H, 1, TH, acc_wl);           // [32][H] (rows >= D+1 are zero)
  store_outer<NT>(slab + 32 * H, H, TH, TH, acc_w1);  // [H][H]
  if (NL == 3) store_outer<NT>(slab + 32 * H + H * H, H, TH, TH, acc_wm);
  float* v = slab + slab_nmat_floats(SGNN_SLAB_DECODER, H, 0, NL);
  if (l < 32) v[w * 32 + l] = s_dbl;
  store_lane_vec<TH>(v + kWaves * 32, s_db1);
  // loss partials: reduce over lanes, one row of 8 per wave
  float* lp = v + kWaves * 32 + kWaves * H;
#pragma unroll
  for (int q = 0; q < 5; ++q) {
    float s = loss_acc[q];
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    if (l == 0) lp[w * 8 + q] = s;
  }
  if (NL == 3) store_lane_vec<TH>(lp + kWaves * 8, s_dbm);
}

// ===========================================================================
// Encoder node MLP backward (graph_network.py:86-90; multi_scale_gnn.py:241)
struct EncNodeBwdArgs {
  const float* g;
  const float* pos_seq;
  int64_t n;
  int T, dim, feat;
  const float *vel_mean, *vel_std;
  float wall_max, wall_div;
  const float *h1, *h2, *yh, *rstd;
  const float *wl, *wm, *gamma;
  float* slab;
  int64_t slab_stride;
  const int64_t* types;  // particle types (use_emb) -> embedding features + per-type dh sums
  const float* emb_w;
  int emb_dim, use_emb;
  float* dh_out;         // > 32 types: dh rows [n][H] out (k_type_sums forms G) instead of the one-hot G
};

template <int TH, int TKF, int NL>
__global__ __launch_bounds__(kBlock) void k_enc_node_bwd(EncNodeBwdArgs a) {
  constexpr bool GW = TH > 2;
  constexpr int H = 32 * TH, ldh = H + 4, ldf = 32 * TKF + 4;
  constexpr int ldl = GW ? H : ldh;
  constexpr int ldb = ldh > ldf ? ldh : ldf;
  extern __shared__ float lds[];
  float* p = lds;
  const float* WlT = a.wl;
  const float* WmT = a.wm;
  if (!GW) {
    stage_matrix_t(p, ldh, a.wl, H, H, H, H, H);
    WlT = p;
    p += H * ldh;
    if (NL == 3) {
      stage_matrix_t(p, ldh, a.wm, H, H, H, H, H);
      WmT = p;
      p += H * ldh;
    }
  }
  float* gam = p;
  float* bufA = gam + H;
  float* bufB = bufA + kChunk * ldh;  // rows of max(ldh, ldf)
  stage_vec(gam, a.gamma, H, H);
  __syncthreads();
  const Imgs im = make_imgs(bufA, ldh, bufB, ldb);
  const int l = lane_id(), j = im.j, h = l >> 5, w = wave_id();
  constexpr int NT = (TH * TH + kWaves - 1) / kWaves;
  constexpr int NT1 = (TH * TKF + kWaves - 1) / kWaves;
  constexpr int NTG = (TH + kWaves - 1) / kWaves;
  f32x16 acc_wl[NT], acc_wm[NT], acc_w1[NT1], acc_g[NTG];
  zero_acc<NT>(acc_wl);
  zero_acc<NT>(acc_wm);
  zero_acc<NT1>(acc_w1);
  zero_acc<NTG>(acc_g);
  LANEVEC(s_db1);
  LANEVEC(s_dbl);
  LANEVEC(s_dbm);
  LANEVEC(s_dg);
  LANEVEC(s_db);
  const int nvel = (a.T - 1) * a.dim;
  const int64_t nchunks = (a.n + kChunk - 1) / kChunk;
  for (int64_t c = blockIdx.x; c < nchunks; c += gridDim.x) {
    const int64_t i = c * kChunk + w * 32 + j;
    const int nvalid = clamp_items(a.n - (c * kChunk + w * 32));
    const bool valid = i < a.n;
    const int64_t ic = valid ? i : a.n - 1;
    f32x16 gi[TH], yh[TH], h1[TH], h2[TH], dh[TH];
    load_row_clayout<TH>(gi, a.g + ic * H);
    load_row_clayout<TH>(yh, a.yh + ic * H);
    load_row_clayout<TH>(h1, a.h1 + ic * H);
    zero_if<TH>(h1, !valid);
    if (NL == 3) {
      load_row_clayout<TH>(h2, a.h2 + ic * H);
      zero_if<TH>(h2, !valid);
    }
    ln_mlp_tail_bwd<TH, NL, GW, NT>(gi, yh, a.rstd[ic], gam, h1, h2, WlT, ldl, WmT, ldl, valid,
                                    nvalid, im, acc_wl, acc_wm, s_db, s_dg, s_dbl, s_dbm, dh);
    // node features recomputed exactly as the forward (learned_simulator.py:272-284,
    // multi_scale_simulator.py:176-196)
    f32x16 xf[TKF];
    const float* pp = a.pos_seq + ic * a.T * a.dim;
#pragma unroll
    for (int tk = 0; tk < TKF; ++tk)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int f = 32 * tk + crow(r, h);
        float val = 0.0f;
        if (valid && f < nvel) {
          const int t = f / a.dim, cc = f - t * a.dim;
          const float vel = __fsub_rn(pp[(t + 1) * a.dim + cc], pp[t * a.dim + cc]);
          val = __fdiv_rn(__fsub_rn(vel, a.vel_mean[cc]), a.vel_std[cc]);
        } else if (valid && f == nvel) {
          val = __fdiv_rn(fminf(fmaxf(__fadd_rn(pp[(a.T - 1) * a.dim], 2.0f), 0.0f), a.wall_max),
                          a.wall_div);
        } else if (valid && a.use_emb && f < nvel + 1 + a.emb_dim) {  // :287-290
          val = a.emb_w[a.types[ic] * a.emb_dim + (f - nvel - 1)];
        }
        xf[tk][r] = val;
      }
    lds_store_items<TH>(im.sA, ldh, j, dh);
    lds_store_items<TKF>(im.sB, ldb, j, xf);
    wave_lds_sync();
    lane_sums<TH>(s_db1, im.sA, ldh, nvalid);
    __syncthreads();
    outer_tiles<NT1>(acc_w1, TH, TKF, bufA, ldh, 0, bufB, ldb, 0);
    __syncthreads();
    if (a.dh_out && valid) store_row_clayout<TH>(a.dh_out + i * H, dh);
    if (a.use_emb && !a.dh_out) {
      // G[type][u] += dh[u] over this type's nodes (one-hot (x) dh); the
      // embedding gradient is G . W1[:, emb columns] (sgnn_embedding_grad)
      const int ty = valid ? (int)a.types[ic] : -1;
      f32x16 oh[1];
#pragma unroll
      for (int r = 0; r < 16; ++r) oh[0][r] = crow(r, h) == ty ? 1.0f : 0.0f;
      lds_store_items<1>(im.sB, ldb, j, oh);
      __syncthreads();
      outer_tiles<NTG>(acc_g, 1, TH, bufB, ldb, 0, bufA, ldh, 0);
      __syncthreads();
    }
  }
  float* slab = a.slab + blockIdx.x * a.slab_stride;
  store_outer<NT>(slab, H, TH, TH, acc_wl);
  store_outer<NT1>(slab + H * H, 32 * TKF, TH, TKF, acc_w1);
  if (NL == 3) store_outer<NT>(slab + H * H + H * 32 * TKF, H, TH, TH, acc_wm);
  float* v = slab + slab_nmat_floats(SGNN_SLAB_ENC_NODE, H, 32 * TKF, NL);
  store_lane_vec<TH>(v, s_db1);
  store_lane_vec<TH>(v + kWaves * H, s_dbl);
  store_lane_vec<TH>(v + 2 * kWaves * H, s_dg);
  store_lane_vec<TH>(v + 3 * kWaves * H, s_db);
  if (NL == 3) store_lane_vec<TH>(v + 4 * kWaves * H, s_dbm);
  store_outer<NTG>(v + (NL == 3 ? 5 : 4) * kWaves * H, H, 1, TH, acc_g);  // G [32][H]
}

// ===========================================================================
// Encoder edge MLP backward (graph_network.py:92-96; multi_scale_gnn.py:247-258)
// from dE0
struct EncEdgeBwdArgs {
  const float* de0t;
  const float* pos;
  int64_t stride;
  int dim;
  float radius;
  const int32_t *rowptr, *send, *recv;
  int64_t n;
  const float *h2, *yh, *rstd;
  const float *w1, *b1, *wl, *wm, *gamma;
  float* slab;
  int64_t slab_stride;
};

template <int TH, int NL>
__global__ __launch_bounds__(kBlock) void k_enc_edge_bwd(EncEdgeBwdArgs a) {
  constexpr bool GW = TH > 2;
  constexpr int H = 32 * TH, ldh = H + 4, ld1 = 5, ldf = 32 + 4;
  constexpr int ldl = GW ? H : ldh;
  extern __shared__ float lds[];
  float* W1 = lds;
  float* p = W1 + H * ld1;
  stage_matrix(W1, ld1, a.w1, a.dim + 1, H, a.dim + 1, H, 4);
  const float* WlT = a.wl;
  const float* WmT = a.wm;
  if (!GW) {
    stage_matrix_t(p, ldh, a.wl, H, H, H, H, H);
    WlT = p;
    p += H * ldh;
    if (NL == 3) {
      stage_matrix_t(p, ldh, a.wm, H, H, H, H, H);
      WmT = p;
      p += H * ldh;
    }
  }
  float* b1 = p;
  float* gam = b1 + H;
  float* bufA = gam + H;
  float* bufB = bufA + kChunk * ldh;
  stage_vec(b1, a.b1, H, H);
  stage_vec(gam, a.gamma, H, H);
  __syncthreads();
  const Imgs im = make_imgs(bufA, ldh, bufB, ldh);
  const int l = lane_id(), j = im.j, h = l >> 5, w = wave_id();
  constexpr int NT = (TH * TH + kWaves - 1) / kWaves;
  constexpr int NT1 = (TH + kWaves - 1) / kWaves;
  f32x16 acc_wl[NT], acc_wm[NT], acc_w1[NT1];
  zero_acc<NT>(acc_wl);
  zero_acc<NT>(acc_wm);
  zero_acc<NT1>(acc_w1);
  LANEVEC(s_db1);
  LANEVEC(s_dbl);
  LANEVEC(s_dbm);
  LANEVEC(s_dg);
  LANEVEC(s_db);
  const int64_t E = a.rowptr[a.n];
  const int64_t nchunks = (E + kChunk - 1) / kChunk;
  for (int64_t c = blockIdx.x; c < nchunks; c += gridDim.x) {
    const int64_t tile = c * kWaves + w, base = tile * 32, e = base + j;
    const int nvalid = clamp_items(E - base);
    const bool valid = e < E;
    const int64_t ec = valid ? e : (E > 0 ? E - 1 : 0);
    f32x16 dm[TH], yh[TH], h1[TH], h2[TH], fx[1];
    float rs = 0.0f;
    zero<TH>(dm);
    zero<TH>(yh);
    zero<TH>(h1);
    zero<TH>(h2);
    zero<1>(fx);
    if (nvalid > 0) {
      load_tiled<TH>(dm, a.de0t + tile * (32 * H));
      load_tiled<TH>(yh, a.yh + tile * (32 * H));
      if (NL == 3) load_tiled<TH>(h2, a.h2 + tile * (32 * H));
      rs = a.rstd[ec];
      // recompute edge features and the first hidden layer (cheap: K = dim+1)
      const int64_t s = a.send[ec], r = a.recv[ec];
      float f[4] = {0.0f, 0.0f, 0.0f, 0.0f};
      float ss = 0.0f;
      for (int cc = 0; cc < a.dim; ++cc) {
        const float d = __fdiv_rn(__fsub_rn(a.pos[s * a.stride + cc], a.pos[r * a.stride + cc]), a.radius);
        f[cc] = d;
        ss = __fadd_rn(ss, __fmul_rn(d, d));
      }
      f[a.dim] = sqrtf(ss);
      acc_bias<TH>(h1, b1);
      mfma_step<TH>(h1, W1, ld1, h, h ? f[1] : f[0]);
      mfma_step<TH>(h1, W1, ld1, 2 + h, h ? f[3] : f[2]);
      acc_relu<TH>(h1);
      if (valid && h == 0) {
#pragma unroll
        for (int cc = 0; cc < 4; ++cc) fx[0][cc] = f[cc];
      }
    }
    zero_if<TH>(h1, !valid);
    zero_if<TH>(h2, !valid);
    f32x16 dh[TH];
    ln_mlp_tail_bwd<TH, NL, GW, NT>(dm, yh, rs, gam, h1, h2, WlT, ldl, WmT, ldl, valid, nvalid,
                                    im, acc_wl, acc_wm, s_db, s_dg, s_dbl, s_dbm, dh);
    lds_store_items<TH>(im.sA, ldh, j, dh);
    lds_store_items<1>(bufB + w * 32 * ldf, ldf, j, fx);
    wave_lds_sync();
    lane_sums<TH>(s_db1, im.sA, ldh, nvalid);
    __syncthreads();
    outer_tiles<NT1>(acc_w1, TH, 1, bufA, ldh, 0, bufB, ldf, 0);
    __syncthreads();
  }
  float* slab = a.slab + blockIdx.x * a.slab_stride;
  store_outer<NT>(slab, H, TH, TH, acc_wl);
  store_outer<NT1>(slab + H * H, 32, TH, 1, acc_w1);
  if (NL == 3) store_outer<NT>(slab + H * H + H * 32, H, TH, TH, acc_wm);
  float* v = slab + slab_nmat_floats(SGNN_SLAB_ENC_EDGE, H, 0, NL);
  store_lane_vec<TH>(v, s_db1);
  store_lane_vec<TH>(v + kWaves * H, s_dbl);
  store_lane_vec<TH>(v + 2 * kWaves * H, s_dg);
  store_lane_vec<TH>(v + 3 * kWaves * H, s_db);
  if (NL == 3) store_lane_vec<TH>(v + 4 * kWaves * H, s_dbm);
}

// Encoder edge MLP backward at H = 64, NL = 2 (the single-scale training
// configuration), sized like k_edge_bwd64 for TWO workgroups per CU: Wl^T
// swizzled in LDS (16 KB) + two unpadded swizzled [128 items][64] images
// (64 KB) = 80 KB, W1 / b1 / gamma read from L2, <= 256 VGPRs.  Per 128-edge
// chunk: LayerNorm backward from dE0, dWl = sum dy (x) h1 (one 32x32 tile per
// wave), dh = (Wl^T dy) * [h1 > 0], then dW1 = sum dh (x) f over the edge
// features f (dim + 1 <= 4 of a 32-column tile; the two 32-unit tiles are
// split over the waves by item halves and summed once at the end) and
// db1 = sum dh.  h1 is recomputed from the positions as the forward did.
SGNN_DEV void swz_store_feat(float* img, int item, f32x4 f) {
  const int h = lane_id() >> 5;
#pragma unroll
  for (int q = 0; q < 4; ++q) {  // half h writes column groups 4 (2q + h) .. +3 of columns 0..31
    const int g = 2 * q + h;
    st4(img + swz(item, 4 * g), g == 0 ? f : f32x4{0.0f, 0.0f, 0.0f, 0.0f});
  }
}

// swz_outer over the item steps [s0, s0 + 32) (items 2 s0 .. 2 s0 + 63).
SGNN_DEV void swz_outer_half(f32x16& acc, const float* A, int ua, const float* B, int vb, int s0) {
  constexpr int G = 4, NS = kChunk / 4;
  const int l = (lane_id() & 31) + opaque_zero(), h = lane_id() >> 5;
  const int ca = h * 64 + ((ua + l) ^ (4 * h)), cb = h * 64 + ((vb + l) ^ (4 * h));
  auto ra = [&](int s) { return A[(ca ^ (8 * (s & 7))) + 128 * s]; };
  auto rb = [&](int s) { return B[(cb ^ (8 * (s & 7))) + 128 * s]; };
#pragma unroll
  for (int s = 0; s < NS; s += G) {
    float a[G], b[G];
#pragma unroll
    for (int i = 0; i < G; ++i) {
      a[i] = ra(s0 + s + i);
      b[i] = rb(s0 + s + i);
    }
#pragma unroll
    for (int i = 0; i < G; ++i) acc = mfma32(a[i], b[i], acc);
  }
}

__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(2)))
void k_enc_edge_bwd64(EncEdgeBwdArgs a) {
  constexpr int TH = 2, H = 64;
  extern __shared__ float lds[];
  float* wt = lds;                  // Wl^T [u][k]
  float* bufA = wt + H * H;         // [128 items][64]
  float* bufB = bufA + kChunk * H;
  swz_stage_wt(wt, a.wl, H, 1.0f);
  __syncthreads();
  const int w = wave_id(), l = lane_id(), j = l & 31, h = l >> 5;
  float* sA = bufA + w * 32 * H;
  float* sB = bufB + w * 32 * H;
  const int tu = w >> 1, tv = w & 1;   // the wave's dWl tile
  const int t1 = w & 1, ih = w >> 1;   // its dW1 tile (units 32 t1 ..) and item half
  const int nf = a.dim + 1;
  f32x16 acc, acc1;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    acc[r] = 0.0f;
    acc1[r] = 0.0f;
  }
  f32x4 s_dbl = {0.0f, 0.0f, 0.0f, 0.0f}, s_dg = s_dbl, s_db = s_dbl, s_db1 = s_dbl;
  const int64_t E = a.rowptr[a.n];
  const int64_t nchunks = (E + kChunk - 1) / kChunk;
  for (int64_t c = blockIdx.x; c < nchunks; c += gridDim.x) {
    const int64_t tile = c * kWaves + w, base = tile * 32, e = base + j;
    const int nvalid = clamp_items(E - base);
    const bool valid = e < E;
    f32x16 dm[TH], yh[TH], h1[TH];
    float rs = 0.0f;
    f32x4 fx = {0.0f, 0.0f, 0.0f, 0.0f};
    zero<TH>(dm);
    zero<TH>(yh);
    zero<TH>(h1);
    if (nvalid > 0) {  // tiles past the last valid one are not allocated
      const int64_t ec = valid ? e : E - 1;
      load_tiled<TH>(dm, a.de0t + tile * (32 * H));
      load_tiled<TH>(yh, a.yh + tile * (32 * H));
      rs = a.rstd[ec];
      // edge features (learned_simulator.py:299-312) and the first hidden layer, as the forward
      const int64_t snd = a.send[ec], rcv = a.recv[ec];
      float f[4] = {0.0f, 0.0f, 0.0f, 0.0f};
      float ss = 0.0f;
      for (int cc = 0; cc < a.dim; ++cc) {
        const float d = __fdiv_rn(__fsub_rn(a.pos[snd * a.stride + cc], a.pos[rcv * a.stride + cc]), a.radius);
        f[cc] = d;
        ss = __fadd_rn(ss, __fmul_rn(d, d));
      }
      f[a.dim] = sqrtf(ss);
      acc_bias<TH>(h1, a.b1);
#pragma unroll
      for (int st = 0; st < 2; ++st) {  // K = 4 in two 32x32x2 steps: k = 2 st + h
        const int k = 2 * st + h;
        const float b = st == 0 ? (h ? f[1] : f[0]) : (h ? f[3] : f[2]);
#pragma unroll
        for (int t = 0; t < TH; ++t) {
          const float wv = k < nf ? a.w1[(32 * t + j) * nf + k] : 0.0f;
          h1[t] = mfma32(wv, b, h1[t]);
        }
      }
      acc_relu<TH>(h1);
      if (valid) fx = f32x4{f[0], f[1], f[2], f[3]};
    }
    zero_if<TH>(dm, !valid);
    zero_if<TH>(h1, !valid);
    // LayerNorm backward (graph_network.py:92-96 encoder LN), its affine sums
    f32x16 dy[TH];
    acc_layernorm_bwd<TH>(dm, yh, rs, a.gamma, dy);
    zero_if<TH>(dy, !valid);
#pragma unroll
    for (int t = 0; t < TH; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) yh[t][r] *= dm[t][r];
    swz_store_items(sA, j, dm);
    swz_store_items(sB, j, yh);
    wave_lds_sync();
    s_db += swz_col_sums(sA);
    s_dg += swz_col_sums(sB);
    wave_lds_sync();
    // last Linear: dWl += dy (x) h1, dbl += dy, dh = (Wl^T dy) * [h1 > 0]
    swz_store_items(sA, j, dy);
    swz_store_items(sB, j, h1);
    wave_lds_sync();
    s_dbl += swz_col_sums(sA);
    __syncthreads();
    swz_outer(acc, bufA, 32 * tu, bufB, 32 * tv);
    __syncthreads();
    f32x16 dh[TH];
    zero<TH>(dh);
    swz_matvec_t(dh, wt, dy);
    relu_mask<TH>(dh, h1, valid);
    // first Linear: dW1 += dh (x) f, db1 += dh
    swz_store_items(sA, j, dh);
    swz_store_feat(sB, j, fx);
    wave_lds_sync();
    s_db1 += swz_col_sums(sA);
    __syncthreads();
    swz_outer_half(acc1, bufA, 32 * t1, bufB, 0, 32 * ih);
    __syncthreads();
  }
  // the item halves of each dW1 tile: waves 2, 3 hand theirs to waves 0, 1 (fixed order)
  if (w >= 2) store_tile_rowmajor(bufA + (w - 2) * 32 * 32, 32, acc1);
  __syncthreads();
  float* slab = a.slab + blockIdx.x * a.slab_stride;
  if (w < 2) {
    const int hh = l >> 5;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc1[r] += bufA[w * 32 * 32 + crow(r, hh) * 32 + j];
    store_tile_rowmajor(slab + H * H + (32 * t1) * 32, 32, acc1);
  }
  store_tile_rowmajor(slab + (32 * tu) * H + 32 * tv, H, acc);
  float* v = slab + slab_nmat_floats(SGNN_SLAB_ENC_EDGE, H, 0, 2);
  if (l < 16) {
    st4(v + w * H + 4 * l, s_db1);
    st4(v + kWaves * H + w * H + 4 * l, s_dbl);
    st4(v + 2 * kWaves * H + w * H + 4 * l, s_dg);
    st4(v + 3 * kWaves * H + w * H + 4 * l, s_db);
  }
}

// ===========================================================================
// Hidden 128: per-item chains and weight-gradient GEMMs in separate launches.
// In the fused form every wave would hold 3-4 [128 x 128] weight-gradient
// accumulators (192-256 registers) next to the per-item state, which does not
// fit the 512-entry register file without spilling.  At H = 128 the per-item
// kernels (wave-independent, no workgroup barriers) therefore write the
// pre-activation gradients (dy, d2, dh) to scratch, and k_wgrad_half forms every
// dW = sum_items A (x) B (plus the bias sums = column sums of A) as a split-K
// MFMA GEMM over LDS-staged 128-item chunks, into the same slab layouts.

template <int TH>
SGNN_DEV void wave_colsum(LaneVec<TH>& acc, float* slice, const f32x16 (&x)[TH], int nvalid) {
  constexpr int ldh = 32 * TH + 4;
  lds_store_items<TH>(slice, ldh, lane_id() & 31, x);
  wave_lds_sync();
  lane_sums<TH>(acc, slice, ldh, nvalid);
  wave_lds_sync();
}

struct WgradOp {
  const float *A, *B;
  int a_tiled, b_tiled;  // 1: 32-item tiled layout; 0: row-major with leading dim a_ld / b_ld
  int a_ld, b_ld;
  float* dst;            // workgroup-0 slab + matrix offset
  int dst_ld;
  float* colsum;         // workgroup-0 slab + [W][32*TU] vector offset, or null
  int64_t slab_stride, nitems;
  const int32_t* nitems_dev;  // if set: nitems = *nitems_dev (edge count = rowptr[n])
  // extents in floats (from A, B, dst, colsum): what the bounds-checked build (SGNN_DEBUG_BOUNDS) tests
  // every operand load and slab store against
  int64_t a_len, b_len, dst_len, colsum_len;
};

// Weight-gradient GEMM dW = sum_items A (x) B for 128-row gradients (TU = 4),
// split over two workgroups per slab: workgroup b < nslab forms rows [0, 64)
// and b + nslab rows [64, 128) of slab b's gradient over the same item range,
// from 64-item chunks.  The two images (A half 17 KB + B 34 KB) let two
// workgroups share a CU; the next chunk's operands are loaded into registers
// while the current chunk's MFMAs run.  (Round 2's one-workgroup-per-slab form
// with 128-item chunks -- 135 KB of images, staging and MFMAs serialised --
// ran at 0.27 of fp32 MFMA peak per C5 launch.)
constexpr int kHalfChunk = 64;

// One 64-item chunk of U units (starting at unit u0 of a USRC-unit operand) in
// registers: thread t holds float4 groups t, t + 256, ... (NPT of them), so the
// next chunk's loads are in flight during this chunk's MFMAs.
template <int U, int NTH>
struct ChunkRegs {
  static constexpr int NPT = kHalfChunk * U / 4 / NTH;
  f32x4 v[NPT];
};

template <int U, int USRC, int NTH>
SGNN_DEV void fetch_sub(ChunkRegs<U, NTH>& r, const float* src, int tiled, int ld, int u0, int64_t item0,
                        int64_t nitems, int64_t len) {
  (void)len;
  constexpr int per_tile = (U / 32) * 4 * 64;   // float4 groups per 32-item tile (tiled layout)
  constexpr int Q = U / 4;
  const int g0 = (u0 / 32) * 4;
#pragma unroll
  for (int k = 0; k < ChunkRegs<U, NTH>::NPT; ++k) {
    const int idx = threadIdx.x + k * NTH;
    f32x4 v = {0.0f, 0.0f, 0.0f, 0.0f};
    if (tiled) {
      const int q = idx / per_tile, rem = idx - q * per_tile;
      const int grp = rem >> 6, lane = rem & 63;
      const int64_t t0 = item0 + q * 32;
      if (t0 + (lane & 31) < nitems) {
        int64_t off = (t0 / 32) * (32 * USRC) + (g0 + grp) * 256 + lane * 4;
        SGNN_BOUNDS(off, 0, len - 3, "wgrad tiled operand");
        v = ld4(src + off);
      }
    } else {
      const int item = idx / Q, quad = idx - item * Q;
      if (item0 + item < nitems) {
        int64_t off = (item0 + item) * ld + u0 + 4 * quad;
        SGNN_BOUNDS(off, 0, len - 3, "wgrad row operand");
        v = ld4(src + off);
      }
    }
    r.v[k] = v;
  }
}

// The registers of fetch_sub as an LDS image [item][unit] (ld U + 4).
template <int U, int NTH>
SGNN_DEV void put_sub(float* img, const ChunkRegs<U, NTH>& r, int tiled) {
  constexpr int ldi = U + 4, per_tile = (U / 32) * 4 * 64, Q = U / 4;
#pragma unroll
  for (int k = 0; k < ChunkRegs<U, NTH>::NPT; ++k) {
    const int idx = threadIdx.x + k * NTH;
    int item, unit;
    if (tiled) {
      const int q = idx / per_tile, rem = idx - q * per_tile;
      const int grp = rem >> 6, lane = rem & 63;
      item = q * 32 + (lane & 31);
      unit = 32 * (grp >> 2) + 8 * (grp & 3) + 4 * (lane >> 5);
    } else {
      item = idx / Q;
      unit = 4 * (idx - item * Q);
    }
    int o = item * ldi + unit;
    SGNN_BOUNDS(o, 0, kHalfChunk * ldi - 3, "wgrad LDS image");
    st4(img + o, r.v[k]);
  }
}

// TAG only names the launch for the profiler: 1 = the edge layer's weight gradients (bench.py reads
// their per-launch bytes from the rocprofv3 summary), 0 = every other caller.  NWV waves per
// workgroup: 8 at 128 x 128 (one output tile per wave, four waves per SIMD across the two
// workgroups of a CU, so one wave's loads wait under three others' MFMAs), 4 at 128 x 32.
template <int TV, int TAG, int NWV>
__global__ __launch_bounds__(64 * NWV) __attribute__((amdgpu_waves_per_eu(NWV / 2)))
void k_wgrad_half(WgradOp op, int nslab) {
  constexpr int NTH = 64 * NWV;
  constexpr int AU = 64, BU = 32 * TV, lda = AU + 4, ldb = BU + 4;
  constexpr int TU = 2, NT = (TU * TV + NWV - 1) / NWV;
  constexpr int RPW = kHalfChunk / NWV;   // items per wave in the column sums
  extern __shared__ float lds[];
  float* imA = lds;
  float* imB = imA + kHalfChunk * lda;
  const int l = lane_id(), w = (int)threadIdx.x / 64;
  const int half = blockIdx.x >= (unsigned)nslab ? 1 : 0;
  const int slab = (int)blockIdx.x - half * nslab;
  f32x16 acc[NT];
  zero_acc<NT>(acc);
  float cs = 0.0f;
  const int64_t nitems = op.nitems_dev ? (int64_t)*op.nitems_dev : op.nitems;
  const int64_t nch = (nitems + kHalfChunk - 1) / kHalfChunk;
  const int64_t c0 = nch * slab / nslab, c1 = nch * (slab + 1) / nslab;
  ChunkRegs<AU, NTH> ra;
  ChunkRegs<BU, NTH> rb;
  if (c0 < c1) {
    fetch_sub<AU, 128, NTH>(ra, op.A, op.a_tiled, op.a_ld, AU * half, c0 * kHalfChunk, nitems, op.a_len);
    fetch_sub<BU, BU, NTH>(rb, op.B, op.b_tiled, op.b_ld, 0, c0 * kHalfChunk, nitems, op.b_len);
  }
  for (int64_t c = c0; c < c1; ++c) {
    put_sub<AU, NTH>(imA, ra, op.a_tiled);
    put_sub<BU, NTH>(imB, rb, op.b_tiled);
    __syncthreads();
    if (c + 1 < c1) {   // the next chunk's loads fly under this chunk's MFMAs
      fetch_sub<AU, 128, NTH>(ra, op.A, op.a_tiled, op.a_ld, AU * half, (c + 1) * kHalfChunk, nitems, op.a_len);
      fetch_sub<BU, BU, NTH>(rb, op.B, op.b_tiled, op.b_ld, 0, (c + 1) * kHalfChunk, nitems, op.b_len);
    }
#pragma unroll
    for (int q = 0; q < NT; ++q) {
      const int tile = w + NWV * q;
      if (tile < TU * TV) {
        const int tu = tile / TV, tv = tile - tu * TV;
        mfma_outer<kHalfChunk>(acc[q], imA, lda, 32 * tu, imB, ldb, 32 * tv);
      }
    }
    if (op.colsum) {
      const float* sl = imA + w * RPW * lda;
#pragma unroll
      for (int it = 0; it < RPW; ++it) cs += sl[it * lda + l];
    }
    __syncthreads();
  }
#pragma unroll
  for (int q = 0; q < NT; ++q) {
    const int tile = w + NWV * q;
    if (tile < TU * TV) {
      const int tu = tile / TV, tv = tile - tu * TV;
      const int64_t o = slab * op.slab_stride + (int64_t)(AU * half + 32 * tu) * op.dst_ld + 32 * tv;
#ifdef SGNN_DEBUG_BOUNDS
      int64_t hi = o + 31 * (int64_t)op.dst_ld + 31;   // the tile's last element
      SGNN_BOUNDS(hi, 0, op.dst_len, "wgrad slab tile");
#endif
      store_tile_rowmajor(op.dst + o, op.dst_ld, acc[q]);
    }
  }
  if (op.colsum) {
    // kWaves partial rows per slab: waves w and w + 4 (NWV = 8) add theirs through LDS, in that order
    if constexpr (NWV > kWaves) {
      if (w >= kWaves) lds[(w - kWaves) * 64 + l] = cs;
      __syncthreads();
      if (w < kWaves) cs += lds[w * 64 + l];
    }
    if (w < kWaves) {
      int64_t o = slab * op.slab_stride + w * 128 + AU * half + l;
      SGNN_BOUNDS(o, 0, op.colsum_len, "wgrad column sums");
      op.colsum[o] = cs;
    }
  }
}

// The 128 x 128 weight-gradient GEMM with ONE workgroup per slab forming all 128 rows: the B operand of a
// chunk is read from HBM once instead of once per row half (k_wgrad_half: A + 2 B per chunk; C5's edge
// GEMMs ran at ~4.4 TB/s).  Sixteen waves (four per SIMD, as two k_wgrad_half workgroups), one 32 x 32
// output tile each; the [64 items][128 + 4] images of A and B (67.6 KB).  Same products in the same order
// as k_wgrad_half (every tile over the chunk's 64 items in order, chunks in order; the column sums by
// waves 0-7 over the same item partition, waves w and w + 4 added in that order), so the slabs are
// bit-identical to the half-row form.
template <int TAG>
__global__ __launch_bounds__(1024) void k_wgrad_full(WgradOp op, int nslab) {
  constexpr int NWV = 16, NTH = 64 * NWV;
  constexpr int U = 128, ld = U + 4;
  constexpr int RPW = kHalfChunk / 8;     // items per column-sum wave (waves 0-7, as k_wgrad_half)
  extern __shared__ float lds[];
  float* imA = lds;
  float* imB = imA + kHalfChunk * ld;
  const int l = lane_id(), w = (int)threadIdx.x / 64;
  const int slab = (int)blockIdx.x;
  const int tu = w >> 2, tv = w & 3;
  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.0f;
  float cs0 = 0.0f, cs1 = 0.0f;
  const int64_t nitems = op.nitems_dev ? (int64_t)*op.nitems_dev : op.nitems;
  const int64_t nch = (nitems + kHalfChunk - 1) / kHalfChunk;
  const int64_t c0 = nch * slab / nslab, c1 = nch * (slab + 1) / nslab;
  ChunkRegs<U, NTH> ra, rb;
  if (c0 < c1) {
    fetch_sub<U, U, NTH>(ra, op.A, op.a_tiled, op.a_ld, 0, c0 * kHalfChunk, nitems, op.a_len);
    fetch_sub<U, U, NTH>(rb, op.B, op.b_tiled, op.b_ld, 0, c0 * kHalfChunk, nitems, op.b_len);
  }
  for (int64_t c = c0; c < c1; ++c) {
    put_sub<U, NTH>(imA, ra, op.a_tiled);
    put_sub<U, NTH>(imB, rb, op.b_tiled);
    __syncthreads();
    if (c + 1 < c1) {   // the next chunk's loads fly under this chunk's MFMAs
      fetch_sub<U, U, NTH>(ra, op.A, op.a_tiled, op.a_ld, 0, (c + 1) * kHalfChunk, nitems, op.a_len);
      fetch_sub<U, U, NTH>(rb, op.B, op.b_tiled, op.b_ld, 0, (c + 1) * kHalfChunk, nitems, op.b_len);
    }
    mfma_outer<kHalfChunk>(acc, imA, ld, 32 * tu, imB, ld, 32 * tv);
    if (op.colsum && w < 8) {
      const float* sl = imA + w * RPW * ld;
#pragma unroll
      for (int it = 0; it < RPW; ++it) {
        cs0 += sl[it * ld + l];
        cs1 += sl[it * ld + 64 + l];
      }
    }
    __syncthreads();
  }
  {
    const int64_t o = slab * op.slab_stride + (int64_t)(32 * tu) * op.dst_ld + 32 * tv;
#ifdef SGNN_DEBUG_BOUNDS
    int64_t hi = o + 31 * (int64_t)op.dst_ld + 31;
    SGNN_BOUNDS(hi, 0, op.dst_len, "wgrad slab tile");
#endif
    store_tile_rowmajor(op.dst + o, op.dst_ld, acc);
  }
  if (op.colsum) {
    if (w >= kWaves && w < 8) {
      lds[(w - kWaves) * 128 + l] = cs0;
      lds[(w - kWaves) * 128 + 64 + l] = cs1;
    }
    __syncthreads();
    if (w < kWaves) {
      cs0 += lds[w * 128 + l];
      cs1 += lds[w * 128 + 64 + l];
      int64_t o = slab * op.slab_stride + w * 128 + l;
      SGNN_BOUNDS(o, 0, op.colsum_len - 64, "wgrad column sums");
      op.colsum[o] = cs0;
      op.colsum[o + 64] = cs1;
    }
  }
}

// ---- edge layer, H = 128 ---------------------------------------------------
struct EdgeItemsArgs {
  EdgeBwdArgs b;
  float *dy_out, *d2_out;  // tiled scratch
  float* h2_out;           // tiled scratch: the recomputed h2 (b.yh == NULL), B operand of dW_last
};

// (templated on TH; at H = 64 the fused k_edge_bwd measured faster: the
// split's GEMMs are load-latency bound there, 285 vs 175 us at C2)
template <int TH, int NL>
__global__ __launch_bounds__(kBlock) void k_edge_items(EdgeItemsArgs p) {
  constexpr bool GW = TH > 2;  // H = 64: weight images in LDS
  constexpr int H = 32 * TH, ldh = H + 4;
  constexpr int ldl = GW ? H : ldh, lde = GW ? 3 * H : ldh;
  const EdgeBwdArgs& a = p.b;
  extern __shared__ float lds[];
  float* q = lds;
  const float* WlT = a.wl;
  const float* WmT = a.wm;
  const float* WeT = a.we;
  if (!GW) {
    stage_matrix_t(q, ldh, a.wl, H, H, H, H, H);
    WlT = q;
    q += H * ldh;
    stage_matrix_t(q, ldh, a.we, 3 * H, H, H, H, H);
    WeT = q;
    q += H * ldh;
    if (NL == 3) {
      stage_matrix_t(q, ldh, a.wm, H, H, H, H, H);
      WmT = q;
      q += H * ldh;
    }
  }
  float* gam = q;
  stage_vec(gam, a.gamma, H, H);
  // H = 128: the last Linear's W^T image fits in the LDS the wave slices leave (kItemsLdsW): one of the
  // per-tile products reads LDS instead of L2
  float* wlt = gam + H + kWaves * 32 * ldh;
  if (GW) stage_matrix_t(wlt, ldh, a.wl, H, H, H, H, H);
  // recompute mode (round 6; hidden 128, nlin 3, a.yh == NULL): the forward's h2 = relu(Wm h1 + bm) and
  // yhat = LN-normalised(Wl h2 + bl) are formed again from the saved h1 with the forward's own functions
  // (mlp_tail, acc_layernorm_save: same operands, same MFMA order, so bit for bit the forward's values),
  // instead of being saved: two [E][H] tensors less per block (C5: ~6 GB per block)
  const bool rc = GW && NL == 3 && a.yh == nullptr;
  float* vbm = wlt + H * ldh;
  float* vbl = vbm + H;
  if (rc) {
    stage_vec(vbm, a.bm, H, H);
    stage_vec(vbl, a.bl, H, H);
  }
  const float* hs2 = rc ? p.h2_out : a.hs2;
  __syncthreads();
  const int l = lane_id(), j = l & 31, w = wave_id();
  float* sl = gam + H + w * 32 * ldh;
  LANEVEC(s_dg);
  LANEVEC(s_db);
  const int64_t E = a.rowptr[a.n];
  const int64_t ntiles = (E + 31) / 32;
  const int64_t nw = (int64_t)gridDim.x * kWaves;
  for (int64_t tile = (int64_t)blockIdx.x * kWaves + w; tile < ntiles; tile += nw) {
    const int64_t base = tile * 32, e = base + j;
    const int nvalid = clamp_items(E - base);
    const bool valid = e < E;
    const int64_t ec = valid ? e : E - 1;
    const int rv = a.recv[ec];
    // receivers around the tile (lane 0: before, lane 1: after; one divergent load, readlane at use)
    const bool has = j == 0 ? base > 0 : base + 32 < E;
    const int nb = has ? a.recv[j == 0 ? base - 1 : base + 32] : -1;
    f32x16 dy[TH];
    {
      f32x16 dm[TH], yh[TH];
      load_row_clayout<TH>(dm, a.dagg + (int64_t)rv * H);
      zero_if<TH>(dm, !valid);
      if constexpr (GW && NL == 3) {
        if (rc) {
          f32x16 h1[TH], h2r[TH], y[TH];
          load_tiled<TH>(h1, a.hs + tile * (32 * H));
          mlp_tail<TH, 3, TH, true>(y, h2r, h1, a.wm, H, vbm, a.wl, H, vbl);
          float rs_fwd;
          acc_layernorm_save<TH>(y, gam, gam, yh, rs_fwd);   // (the affine output y is not used)
          store_tiled<TH>(p.h2_out + tile * (32 * H), h2r);
        } else {
          load_tiled<TH>(yh, a.yh + tile * (32 * H));
        }
      } else {
        load_tiled<TH>(yh, a.yh + tile * (32 * H));
      }
      acc_layernorm_bwd<TH>(dm, yh, a.rstd[ec], gam, dy);
      zero_if<TH>(dy, !valid);
      wave_colsum<TH>(s_db, sl, dm, nvalid);
#pragma unroll
      for (int t = 0; t < TH; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) yh[t][r] = valid ? yh[t][r] * dm[t][r] : 0.0f;
      wave_colsum<TH>(s_dg, sl, yh, nvalid);
    }
    store_tiled<TH>(p.dy_out + tile * (32 * H), dy);
    f32x16 dh[TH];
    zero<TH>(dh);
    if constexpr (NL == 3) {
      f32x16 d2[TH], act[TH];
      zero<TH>(d2);
      matvec_t<TH, TH, false>(d2, GW ? wlt : WlT, ldh, dy);
      load_tiled<TH>(act, hs2 + tile * (32 * H));   // (recompute mode: stored by this lane just above)
      relu_mask<TH>(d2, act, valid);
      store_tiled<TH>(p.d2_out + tile * (32 * H), d2);
      matvec_t<TH, TH, GW>(dh, WmT, ldl, d2);
    } else {
      matvec_t<TH, TH, false>(dh, GW ? wlt : WlT, ldh, dy);
    }
    {
      f32x16 act[TH];
      load_tiled<TH>(act, a.hs + tile * (32 * H));
      relu_mask<TH>(dh, act, valid);
    }
    {
      f32x16 de[TH];
      zero<TH>(de);
      matvec_t<TH, TH, GW>(de, WeT, lde, dh);
      float* dtile = a.de0t + tile * (32 * H);
      if (a.de0_accumulate & 1) {
        f32x16 old[TH];
        load_tiled<TH>(old, dtile);
#pragma unroll
        for (int t = 0; t < TH; ++t)
#pragma unroll
          for (int r = 0; r < 16; ++r) de[t][r] = old[t][r] + de[t][r] * a.e_scale;
      } else {
#pragma unroll
        for (int t = 0; t < TH; ++t)
#pragma unroll
          for (int r = 0; r < 16; ++r) de[t][r] *= a.e_scale;
      }
      store_tiled<TH>(dtile, de);
    }
    if (valid) store_row_clayout<TH>(a.dh_rows + e * H, dh);
    lds_store_items<TH>(sl, ldh, j, dh);
    wave_lds_sync();
    segment_sum_store<TH>(sl, ldh, rv, nvalid, base, tile, __builtin_amdgcn_readlane(nb, 0),
                          __builtin_amdgcn_readlane(nb, 1), a.du, a.cin, a.cout);
    wave_lds_sync();
  }
  float* v = a.slab + blockIdx.x * a.slab_stride + slab_nmat_floats(SGNN_SLAB_EDGE, H, 0, NL);
  store_lane_vec<TH>(v + kWaves * H, s_dg);
  store_lane_vec<TH>(v + 2 * kWaves * H, s_db);
}

// ---- node layer, H = 128 ---------------------------------------------------
struct NodeItemsArgs {
  NodeBwdArgs b;
  float *dy_out, *d2_out, *dh_out;  // row-major [n][H] scratch
};

template <int NL>
__global__ __launch_bounds__(kBlock) void k_node_items(NodeItemsArgs p) {
  constexpr int TH = 4, H = 128, ldh = H + 4;
  const NodeBwdArgs& a = p.b;
  extern __shared__ float lds[];
  float* gam = lds;
  stage_vec(gam, a.gamma, H, H);
  float* wlt = gam + H + kWaves * 32 * ldh;   // the last Linear's W^T image (kItemsLdsW)
  stage_matrix_t(wlt, ldh, a.wl, H, H, H, H, H);
  __syncthreads();
  const int l = lane_id(), j = l & 31, w = wave_id();
  float* sl = gam + H + w * 32 * ldh;
  LANEVEC(s_dg);
  LANEVEC(s_db);
  const int64_t ntiles = (a.n + 31) / 32;
  const int64_t nw = (int64_t)gridDim.x * kWaves;
  for (int64_t tile = (int64_t)blockIdx.x * kWaves + w; tile < ntiles; tile += nw) {
    const int64_t i = tile * 32 + j;
    const int nvalid = clamp_items(a.n - tile * 32);
    const bool valid = i < a.n;
    const int64_t ic = valid ? i : a.n - 1;
    f32x16 gi[TH], dy[TH];
    load_row_clayout<TH>(gi, a.g + ic * H);
    zero_if<TH>(gi, !valid);
    {
      f32x16 yh[TH];
      load_row_clayout<TH>(yh, a.yh + ic * H);
      acc_layernorm_bwd<TH>(gi, yh, a.rstd[ic], gam, dy);
      zero_if<TH>(dy, !valid);
      wave_colsum<TH>(s_db, sl, gi, nvalid);
#pragma unroll
      for (int t = 0; t < TH; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) yh[t][r] = valid ? yh[t][r] * gi[t][r] : 0.0f;
      wave_colsum<TH>(s_dg, sl, yh, nvalid);
    }
    if (valid) store_row_clayout<TH>(p.dy_out + i * H, dy);
    f32x16 dh[TH];
    zero<TH>(dh);
    if constexpr (NL == 3) {
      f32x16 d2[TH], act[TH];
      zero<TH>(d2);
      matvec_t<TH, TH, false>(d2, wlt, ldh, dy);
      load_row_clayout<TH>(act, a.hn2 + ic * H);
      relu_mask<TH>(d2, act, valid);
      if (valid) store_row_clayout<TH>(p.d2_out + i * H, d2);
      matvec_t<TH, TH, true>(dh, a.wm, H, d2);
    } else {
      matvec_t<TH, TH, false>(dh, wlt, ldh, dy);
    }
    {
      f32x16 act[TH];
      load_row_clayout<TH>(act, a.hn + ic * H);
      relu_mask<TH>(dh, act, valid);
    }
    if (valid) store_row_clayout<TH>(p.dh_out + i * H, dh);
    f32x16 o[TH];
    zero<TH>(o);
    matvec_t<TH, TH, true>(o, a.w1, 2 * H, dh);
    if (valid) store_row_clayout<TH>(a.dagg + i * H, o);
    matvec_t<TH, TH, true>(gi, a.w1 + H, 2 * H, dh);
    if (valid) store_row_clayout<TH>(a.dxp + i * H, gi);
  }
  float* v = a.slab + blockIdx.x * a.slab_stride + slab_nmat_floats(SGNN_SLAB_NODE, H, 0, NL);
  store_lane_vec<TH>(v + 2 * kWaves * H, s_dg);
  store_lane_vec<TH>(v + 3 * kWaves * H, s_db);
}

// ---- u/v projections, H = 128 ------------------------------------------------
struct UvItemsArgs {
  UvBwdArgs b;
  float *du_out, *dv_out;  // row-major [n][H]
};

__global__ __launch_bounds__(kBlock) void k_uv_items(UvItemsArgs p) {
  constexpr int TH = 4, H = 128;
  const UvBwdArgs& a = p.b;
  const int l = lane_id(), j = l & 31, w = wave_id();
  const int64_t ntiles = (a.n + 31) / 32;
  const int64_t nw = (int64_t)gridDim.x * kWaves;
  for (int64_t tile = (int64_t)blockIdx.x * kWaves + w; tile < ntiles; tile += nw) {
    const int64_t i = tile * 32 + j;
    const bool valid = i < a.n;
    const int64_t ic = valid ? i : a.n - 1;
    f32x16 du[TH], dv[TH], gg[TH];
    load_resolved<TH>(du, a.du, a.cin, a.cout, a.rowptr, ic);
    zero<TH>(dv);
    for (int32_t t = a.tptr[ic], t1 = a.tptr[ic + 1]; t < t1; ++t)
      add_row_clayout<TH>(dv, a.dh_rows + (int64_t)a.tperm[t] * H);
    load_row_clayout<TH>(gg, a.dxp + ic * H);
    matvec_t<TH, TH, true>(gg, a.w1, 3 * H, du);
    matvec_t<TH, TH, true>(gg, a.w1 + H, 3 * H, dv);
    if (valid) {
      store_row_clayout<TH>(a.g + i * H, gg);
      store_row_clayout<TH>(p.du_out + i * H, du);
      store_row_clayout<TH>(p.dv_out + i * H, dv);
    }
  }
}

// ---- edge encoder, H = 128 ---------------------------------------------------
struct EncEdgeItemsArgs {
  EncEdgeBwdArgs b;
  float *dy_out, *d2_out, *dh_out, *h1_out;  // tiled scratch
  float* f_out;                              // [E][32] edge features (units >= dim+1 zero)
};

template <int NL>
__global__ __launch_bounds__(kBlock) void k_enc_edge_items(EncEdgeItemsArgs p) {
  constexpr int TH = 4, H = 128, ldh = H + 4, ld1 = 5;
  const EncEdgeBwdArgs& a = p.b;
  extern __shared__ float lds[];
  float* W1 = lds;
  float* b1 = W1 + H * ld1;
  float* gam = b1 + H;
  stage_matrix(W1, ld1, a.w1, a.dim + 1, H, a.dim + 1, H, 4);
  stage_vec(b1, a.b1, H, H);
  stage_vec(gam, a.gamma, H, H);
  __syncthreads();
  const int l = lane_id(), j = l & 31, h = l >> 5, w = wave_id();
  float* sl = gam + H + w * 32 * ldh;
  LANEVEC(s_dg);
  LANEVEC(s_db);
  const int64_t E = a.rowptr[a.n];
  const int64_t ntiles = (E + 31) / 32;
  const int64_t nw = (int64_t)gridDim.x * kWaves;
  for (int64_t tile = (int64_t)blockIdx.x * kWaves + w; tile < ntiles; tile += nw) {
    const int64_t base = tile * 32, e = base + j;
    const int nvalid = clamp_items(E - base);
    const bool valid = e < E;
    const int64_t ec = valid ? e : E - 1;
    f32x16 dy[TH];
    {
      f32x16 dm[TH], yh[TH];
      load_tiled<TH>(dm, a.de0t + tile * (32 * H));
      zero_if<TH>(dm, !valid);
      load_tiled<TH>(yh, a.yh + tile * (32 * H));
      acc_layernorm_bwd<TH>(dm, yh, a.rstd[ec], gam, dy);
      zero_if<TH>(dy, !valid);
      wave_colsum<TH>(s_db, sl, dm, nvalid);
#pragma unroll
      for (int t = 0; t < TH; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) yh[t][r] = valid ? yh[t][r] * dm[t][r] : 0.0f;
      wave_colsum<TH>(s_dg, sl, yh, nvalid);
    }
    store_tiled<TH>(p.dy_out + tile * (32 * H), dy);
    // recompute edge features and the first hidden layer (K = dim+1)
    const int64_t s = a.send[ec], r = a.recv[ec];
    float f[4] = {0.0f, 0.0f, 0.0f, 0.0f};
    float ss = 0.0f;
    for (int cc = 0; cc < a.dim; ++cc) {
      const float d = __fdiv_rn(__fsub_rn(a.pos[s * a.stride + cc], a.pos[r * a.stride + cc]), a.radius);
      f[cc] = d;
      ss = __fadd_rn(ss, __fmul_rn(d, d));
    }
    f[a.dim] = sqrtf(ss);
    if (valid && h == 0) {
      f32x4 v = {f[0], f[1], f[2], f[3]};
      st4(p.f_out + e * 32, v);
      const f32x4 z = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
      for (int q = 1; q < 8; ++q) st4(p.f_out + e * 32 + 4 * q, z);
    }
    f32x16 h1[TH];
    acc_bias<TH>(h1, b1);
    mfma_step<TH>(h1, W1, ld1, h, h ? f[1] : f[0]);
    mfma_step<TH>(h1, W1, ld1, 2 + h, h ? f[3] : f[2]);
    acc_relu<TH>(h1);
    zero_if<TH>(h1, !valid);
    store_tiled<TH>(p.h1_out + tile * (32 * H), h1);
    f32x16 dh[TH];
    zero<TH>(dh);
    if constexpr (NL == 3) {
      f32x16 d2[TH], act[TH];
      zero<TH>(d2);
      matvec_t<TH, TH, true>(d2, a.wl, H, dy);
      load_tiled<TH>(act, a.h2 + tile * (32 * H));
      relu_mask<TH>(d2, act, valid);
      store_tiled<TH>(p.d2_out + tile * (32 * H), d2);
      matvec_t<TH, TH, true>(dh, a.wm, H, d2);
    } else {
      matvec_t<TH, TH, true>(dh, a.wl, H, dy);
    }
    relu_mask<TH>(dh, h1, valid);
    store_tiled<TH>(p.dh_out + tile * (32 * H), dh);
  }
  float* v = a.slab + blockIdx.x * a.slab_stride + slab_nmat_floats(SGNN_SLAB_ENC_EDGE, H, 0, NL);
  store_lane_vec<TH>(v + 2 * kWaves * H, s_dg);
  store_lane_vec<TH>(v + 3 * kWaves * H, s_db);
}

// ===========================================================================
// Slab reduction: out[r][c] = scale * sum_g sum_q slab_g[off + q*rep + r*ld + c].
// Block = 32 consecutive output elements (the C-ABI's block_start unit).
// Descriptors whose rows are 16-B aligned (ncols, ld, offsets, strides all
// multiples of 4): 8 lanes x float4 cover the 32 elements and the 256 threads
// are 32 slab groups, each summing slabs g = q, q+32, ... with 4 independent
// float4 accumulators (16-B loads: 4x the bytes per load instruction of the
// scalar form).  Otherwise 32 lanes x 1 float and 8 slab groups.  The group
// partials are added in a fixed order through LDS: deterministic.
__global__ __launch_bounds__(256) void k_reduce_slabs(const sgnn_reduce_desc* descs,
                                                      const int32_t* block_start, int ndesc) {
  __shared__ float part[32][33];
  int lo = 0, hi = ndesc - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (block_start[mid] <= (int)blockIdx.x) lo = mid; else hi = mid - 1;
  }
  const sgnn_reduce_desc d = descs[lo];
  const int64_t total = (int64_t)d.nrows * d.ncols;
  const int64_t blk0 = (int64_t)(blockIdx.x - block_start[lo]) * 32;
  const bool vec = ((d.ncols | d.src_ld | d.offset | d.slab_stride | d.rep_stride) & 3) == 0 &&
                   (reinterpret_cast<uintptr_t>(d.src) & 15) == 0;
  int ngroups;
  if (vec) {
    ngroups = 32;
    const int e4 = threadIdx.x & 7, q = threadIdx.x >> 3;
    const int64_t idx = blk0 + 4 * e4;  // ncols % 4 == 0: a float4 never straddles a row or the end
    f32x4 s0 = {0.0f, 0.0f, 0.0f, 0.0f}, s1 = s0, s2 = s0, s3 = s0;
    if (idx < total) {
      const int r = (int)(idx / d.ncols), cc = (int)(idx - (int64_t)r * d.ncols);
      const float* base = d.src + d.offset + (int64_t)r * d.src_ld + cc;
      for (int k = 0; k < d.nrep; ++k) {
        const float* p = base + (int64_t)k * d.rep_stride;
        int g = q;
        for (; g + 96 < d.nslab; g += 128) {
          s0 += ld4(p + (int64_t)g * d.slab_stride);
          s1 += ld4(p + (int64_t)(g + 32) * d.slab_stride);
          s2 += ld4(p + (int64_t)(g + 64) * d.slab_stride);
          s3 += ld4(p + (int64_t)(g + 96) * d.slab_stride);
        }
        for (; g < d.nslab; g += 32) s0 += ld4(p + (int64_t)g * d.slab_stride);
      }
    }
    const f32x4 t = (s0 + s1) + (s2 + s3);
#pragma unroll
    for (int c = 0; c < 4; ++c) part[q][4 * e4 + c] = t[c];
  } else {
    ngroups = 8;
    const int e = threadIdx.x & 31, q = threadIdx.x >> 5;
    const int64_t idx = blk0 + e;
    float s[8] = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
    if (idx < total) {
      const int r = (int)(idx / d.ncols), cc = (int)(idx - (int64_t)r * d.ncols);
      const float* base = d.src + d.offset + (int64_t)r * d.src_ld + cc;
      for (int k = 0; k < d.nrep; ++k) {
        const float* p = base + (int64_t)k * d.rep_stride;
        int g = q;
        for (; g + 56 < d.nslab; g += 64) {
#pragma unroll
          for (int u = 0; u < 8; ++u) s[u] += p[(int64_t)(g + 8 * u) * d.slab_stride];
        }
        for (; g < d.nslab; g += 8) s[0] += p[(int64_t)g * d.slab_stride];
      }
    }
    part[q][e] = ((s[0] + s[1]) + (s[2] + s[3])) + ((s[4] + s[5]) + (s[6] + s[7]));
  }
  __syncthreads();
  const int64_t idx = blk0 + threadIdx.x;
  if (threadIdx.x < 32 && idx < total) {
    float t = 0.0f;
    for (int k = 0; k < ngroups; ++k) t += part[k][threadIdx.x];
    const int r = (int)(idx / d.ncols), cc = (int)(idx - (int64_t)r * d.ncols);
    float* o = d.dst + (int64_t)r * d.dst_ld + cc;
    *o = d.accumulate ? *o + t * d.scale : t * d.scale;
  }
}

// ===========================================================================
// Sender-sorted transpose of the receiver CSR (for dV): tptr[s] .. tptr[s+1]
// lists the edge ids with sender s in ascending order (deterministic).
__global__ __launch_bounds__(256) void k_tcsr_count(const int32_t* rowptr, int64_t n,
                                                    const int32_t* send, int32_t* cnt) {
  const int64_t E = rowptr[n];
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < E;
       e += (int64_t)gridDim.x * blockDim.x)
    atomicAdd(&cnt[send[e]], 1);
}

__global__ __launch_bounds__(256) void k_tcsr_fill(const int32_t* rowptr, int64_t n,
                                                   const int32_t* send, const int32_t* tptr,
                                                   int32_t* fill, int32_t* raw) {
  const int64_t E = rowptr[n];
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < E;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int32_t s = send[e];
    raw[tptr[s] + atomicAdd(&fill[s], 1)] = (int32_t)e;
  }
}

// one wave per sender segment: rank = number of smaller edge ids in the segment
__global__ __launch_bounds__(256) void k_tcsr_sort(const int32_t* tptr, int64_t n,
                                                   const int32_t* raw, int32_t* perm) {
  const int64_t s = (int64_t)blockIdx.x * (blockDim.x >> 6) + wave_id();
  if (s >= n) return;
  const int lane = lane_id();
  const int32_t b = tptr[s], len = tptr[s + 1] - b;
  for (int q = lane; q < len; q += 64) {
    const int32_t key = raw[b + q];
    int rank = 0;
    for (int t = 0; t < len; ++t) rank += raw[b + t] < key;
    perm[b + rank] = key;
  }
}

template <typename K>
void set_lds(K kernel, size_t bytes) {
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kernel),
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
}

template <typename K, typename A>
void launch_bwd(K kernel, int nslab, size_t lds, void* stream, const A& a) {
  set_lds(kernel, lds);
  hipLaunchKernelGGL(kernel, dim3((unsigned)nslab), dim3(kBlock), lds,
                     static_cast<hipStream_t>(stream), a);
}

template <int TU, int TV, int TAG = 0>
void run_wgrad(const WgradOp& op, int nslab, void* stream) {
  static_assert(TU == 4, "weight-gradient GEMMs of 128-row gradients (the H = 128 backward)");
#ifndef SGNN_WGRAD_FULL
#define SGNN_WGRAD_FULL 1
#endif
  if (SGNN_WGRAD_FULL && TV == 4) {   // 128 x 128: one full-row workgroup (16 waves) per slab
    const size_t lds = 4 * (size_t)kHalfChunk * 2 * (128 + 4);
    auto kern = k_wgrad_full<TAG>;
    set_lds(kern, lds);
    hipLaunchKernelGGL(kern, dim3((unsigned)nslab), dim3(1024), lds, static_cast<hipStream_t>(stream), op, nslab);
    return;
  }
  // two half-row workgroups per slab, two per CU
  constexpr int NWV = TV == 4 ? 8 : 4;
  const size_t lds = 4 * (size_t)kHalfChunk * ((64 + 4) + (32 * TV + 4));
  auto kern = k_wgrad_half<TV, TAG, NWV>;
  set_lds(kern, lds);
  hipLaunchKernelGGL(kern, dim3((unsigned)(2 * nslab)), dim3(64 * NWV), lds, static_cast<hipStream_t>(stream), op,
                     nslab);
}

// a_len / b_len: the operands' extents in floats; the slab region holds nslab x slab_stride floats.
WgradOp wg(const float* A, int a_tiled, int a_ld, int64_t a_len, const float* B, int b_tiled, int b_ld,
           int64_t b_len, float* slab, int64_t mat_off, int dst_ld, int64_t vec_off, int64_t slab_stride,
           int nslab, int64_t nitems, const int32_t* nitems_dev) {
  const int64_t slab_len = (int64_t)nslab * slab_stride;
  return WgradOp{A, B, a_tiled, b_tiled, a_ld, b_ld, slab + mat_off, dst_ld,
                 vec_off >= 0 ? slab + vec_off : nullptr, slab_stride, nitems, nitems_dev,
                 a_len, b_len, slab_len - mat_off, vec_off >= 0 ? slab_len - vec_off : 0};
}

constexpr size_t kItemsLds = 4 * (128 + (size_t)kWaves * 32 * (128 + 4));  // gamma + wave slices
constexpr size_t kItemsLdsW = kItemsLds + 4 * (size_t)128 * (128 + 4) + 4 * 2 * 128;  // + the last Linear's
                                                                                       // W^T image + bm, bl

// LDS bytes per kind: weight images (H = 64 only) + vectors + the two
// [128 items][H+4] operand images of the outer products.
size_t bwd_lds(int kind, int H, int tkf, int nl) {
  const size_t ldh = H + 4, chunk = kChunk;
  const bool gw = H > 64;
  const size_t img = gw ? 0 : H * ldh;        // one staged H x H weight image
  const size_t mid = nl == 3 ? img : 0;
  const size_t bufs = 2 * chunk * ldh;
  switch (kind) {
    case SGNN_SLAB_EDGE: return 4 * (2 * img + mid + H + bufs);
    case SGNN_SLAB_NODE: return 4 * (3 * img + mid + H + bufs);
    case SGNN_SLAB_DECODER: return 4 * (H * 36 + img + mid + bufs);
    case SGNN_SLAB_ENC_NODE: {
      const size_t ldb = std::max<size_t>(ldh, 32 * tkf + 4);
      return 4 * (img + mid + H + chunk * ldh + chunk * ldb);
    }
    case SGNN_SLAB_ENC_EDGE: return 4 * (H * 5 + img + mid + 2 * H + bufs);
    default: return 0;
  }
}

int check_bwd_mlp(const sgnn_mlp* m, const char* what) {
  if (!m || !m->w1 || !m->w2) return sgnn::set_error(SGNN_ERR_INVALID, what);
  if (m->hidden != 64 && m->hidden != 128)
    return sgnn::set_error(SGNN_ERR_UNSUPPORTED, "backward: hidden must be 64 or 128");
  if (m->nlin != 2 && m->nlin != 3)
    return sgnn::set_error(SGNN_ERR_UNSUPPORTED, "backward: MLPs must have 2 or 3 Linear layers");
  if (m->nlin == 3 && !m->w3) return sgnn::set_error(SGNN_ERR_INVALID, what);
  return SGNN_OK;
}

const float* last_w(const sgnn_mlp* m) { return m->nlin == 3 ? m->w3 : m->w2; }
const float* mid_w(const sgnn_mlp* m) { return m->nlin == 3 ? m->w2 : nullptr; }
const float* last_b(const sgnn_mlp* m) { return m->nlin == 3 ? m->b3 : m->b2; }
const float* mid_b(const sgnn_mlp* m) { return m->nlin == 3 ? m->b2 : nullptr; }

#define SGNN_BWD_DISPATCH(H, NL, CALL)                                    \
  do {                                                                    \
    if ((H) == 64 && (NL) == 2) { constexpr int TH_ = 2, NL_ = 2; CALL; } \
    else if ((H) == 64) { constexpr int TH_ = 2, NL_ = 3; CALL; }         \
    else if ((NL) == 2) { constexpr int TH_ = 4, NL_ = 2; CALL; }         \
    else { constexpr int TH_ = 4, NL_ = 3; CALL; }                        \
  } while (0)

}  // namespace

// ---------------------------------------------------------------------------
extern "C" int64_t sgnn_bwd_slab_floats(int32_t kind, int32_t hidden, int32_t feat, int32_t nlin) {
  if (kind < 0 || kind > SGNN_SLAB_ENC_EDGE || (nlin != 2 && nlin != 3) || hidden <= 0) return -1;
  const int64_t fpad = 32 * ((feat + 31) / 32);
  int64_t f = slab_nmat_floats(kind, hidden, fpad, nlin) + slab_nvec_floats(kind, hidden, nlin);
  // the slab stride an odd multiple of 256 B: the slab reduction reads one 128-B segment from each of
  // 512 slabs at a time, and strides that are multiples of 2-4 KB (round 5's) pile those reads onto few
  // HBM channels.  Same-box A/B, ms/step: C2 training 1.937 -> 1.911, C3 1.919 -> 1.910, C5 494.5 -> 492.4
  // (profiles/r06_ab_slab_stride.txt)
  f = 64 * ((f + 63) / 64);
  if ((f / 64) % 2 == 0) f += 64;
  return f;
}

extern "C" int64_t sgnn_bwd_scratch_floats(int32_t kind, int32_t hidden, int64_t nitems, int32_t nlin) {
  if (hidden != 128) return 0;
  const int64_t H = hidden, pad = 32 * ((nitems + 31) / 32);
  (void)nlin;
  switch (kind) {
    case SGNN_SLAB_EDGE: return 3 * pad * H;                // dy, d2, recomputed h2 (tiled)
    case SGNN_SLAB_NODE: return 3 * nitems * H;             // dy, d2, dh
    case SGNN_SLAB_UV: return 2 * nitems * H;               // dU, dV
    case SGNN_SLAB_ENC_EDGE: return 4 * pad * H + pad * 32; // dy, d2, dh, h1 (tiled) + features
    default: return 0;
  }
}

extern "C" int sgnn_edge_layer_bwd(const float* dagg, const int32_t* rowptr, const int32_t* send,
                                   const int32_t* recv, int64_t n, const sgnn_saves* saves,
                                   const float* e0t, float e_scale, const sgnn_mlp* edge_fn,
                                   float* du, float* cin, float* cout, float* dh_rows, float* de0t,
                                   int32_t de0_accumulate, float* slab, int32_t nslab,
                                   float* scratch, int64_t edge_cap, void* stream) {
  using namespace sgnn;
  if (!edge_fn || !dagg || !rowptr || !send || !recv || !saves || !saves->h ||
      !saves->rstd || !e0t || !du || !cin || !cout || !dh_rows || !slab || nslab < 1 || n <= 0 ||
      (!de0t && edge_fn->hidden == 128))
    return set_error(SGNN_ERR_INVALID, "edge_layer_bwd: bad arguments");
  int st = check_bwd_mlp(edge_fn, "edge_layer_bwd: edge MLP");
  if (st) return st;
  // recompute mode: yhat and h2 both NULL, hidden 128 with nlin 3 only (include/sgnn.h, sgnn_saves)
  const bool rc = !saves->yhat;
  if (rc && !(edge_fn->hidden == 128 && edge_fn->nlin == 3 && !saves->h2))
    return set_error(SGNN_ERR_INVALID, "edge_layer_bwd: saves->yhat NULL only at hidden 128, nlin 3, with h2 NULL");
  if (!rc && edge_fn->nlin == 3 && !saves->h2) return set_error(SGNN_ERR_INVALID, "edge_layer_bwd: saves->h2");
  const int H = edge_fn->hidden;
  if (H == 64 && n * H * 4 >= (int64_t)kBufRecords)
    return set_error(SGNN_ERR_UNSUPPORTED, "edge_layer_bwd: at most 8M nodes per launch at H = 64");
  EdgeBwdArgs a{dagg, rowptr, send, recv, n, saves->h, saves->h2, saves->yhat, saves->rstd, e0t,
                e_scale, last_w(edge_fn), mid_w(edge_fn), edge_fn->w1 + 2 * H, edge_fn->ln_g, du,
                cin, cout, dh_rows, de0t, de0_accumulate, slab,
                sgnn_bwd_slab_floats(SGNN_SLAB_EDGE, H, 0, edge_fn->nlin)};
  if (rc) {
    a.bm = mid_b(edge_fn);
    a.bl = last_b(edge_fn);
  }
  if (H == 128) {
    if (!scratch || edge_cap < 1) return set_error(SGNN_ERR_INVALID, "edge_layer_bwd: H=128 needs scratch");
    const int nl = edge_fn->nlin;
    const int64_t pad = 32 * ((edge_cap + 31) / 32);
    EdgeItemsArgs p{a, scratch, scratch + pad * H, scratch + 2 * pad * H};
    const int64_t tl = pad * H;   // floats of one tiled [edge_cap][H] array
    const int64_t vb = slab_nmat_floats(SGNN_SLAB_EDGE, H, 0, nl), W = kWaves, ss = a.slab_stride;
    const int32_t* Edev = rowptr + n;
    const float* hl = nl == 3 ? (rc ? p.h2_out : saves->h2) : saves->h;
    if (nl == 3) launch_bwd(k_edge_items<4, 3>, nslab, kItemsLdsW, stream, p);
    else launch_bwd(k_edge_items<4, 2>, nslab, kItemsLdsW, stream, p);
    run_wgrad<4, 4, 1>(wg(p.dy_out, 1, 0, tl, hl, 1, 0, tl, slab, 0, H, vb, ss, nslab, 0, Edev), nslab, stream);
    run_wgrad<4, 4, 1>(wg(dh_rows, 0, H, edge_cap * H, e0t, 1, 0, tl, slab, H * H, H, -1, ss, nslab, 0, Edev), nslab,
                       stream);
    if (nl == 3)
      run_wgrad<4, 4, 1>(wg(p.d2_out, 1, 0, tl, saves->h, 1, 0, tl, slab, 2 * H * H, H, vb + 3 * W * H, ss, nslab, 0, Edev),
                      nslab, stream);
    return check_launch("edge_layer_bwd");
  }
  if (H == 64 && edge_fn->nlin == 2 && !de0t) {  // single-scale training: two workgroups per CU
    if (de0_accumulate & 2) launch_bwd(k_edge_bwd64<true>, nslab, 4 * (size_t)(H * H + 2 * kChunk * H), stream, a);
    else launch_bwd(k_edge_bwd64<false>, nslab, 4 * (size_t)(H * H + 2 * kChunk * H), stream, a);
    return check_launch("edge_layer_bwd");
  }
  const size_t lds = bwd_lds(SGNN_SLAB_EDGE, H, 0, edge_fn->nlin) - (de0t ? 0 : 4 * (size_t)H * (H + 4));
  if (de0t) SGNN_BWD_DISPATCH(H, edge_fn->nlin, (launch_bwd(k_edge_bwd<TH_, NL_, true>, nslab, lds, stream, a)));
  else SGNN_BWD_DISPATCH(H, edge_fn->nlin, (launch_bwd(k_edge_bwd<TH_, NL_, false>, nslab, lds, stream, a)));
  return check_launch("edge_layer_bwd");
}

extern "C" int sgnn_node_layer_bwd(const float* g, int64_t n, const sgnn_saves* saves,
                                   const float* x_in, const sgnn_mlp* node_fn, float* dagg,
                                   float* dxp, float* slab, int32_t nslab, float* scratch,
                                   void* stream) {
  using namespace sgnn;
  if (!node_fn || !g || !saves || !saves->yhat || !saves->rstd || !saves->h || !saves->agg ||
      !x_in || !dagg || !dxp || !slab || nslab < 1 || n <= 0)
    return set_error(SGNN_ERR_INVALID, "node_layer_bwd: bad arguments");
  int st = check_bwd_mlp(node_fn, "node_layer_bwd: node MLP");
  if (st) return st;
  if (node_fn->nlin == 3 && !saves->h2) return set_error(SGNN_ERR_INVALID, "node_layer_bwd: saves->h2");
  const int H = node_fn->hidden;
  NodeBwdArgs a{g, n, saves->yhat, saves->rstd, saves->h, saves->h2, saves->agg, x_in, node_fn->w1,
                last_w(node_fn), mid_w(node_fn), node_fn->ln_g, dagg, dxp, slab,
                sgnn_bwd_slab_floats(SGNN_SLAB_NODE, H, 0, node_fn->nlin)};
  if (H == 128) {
    if (!scratch) return set_error(SGNN_ERR_INVALID, "node_layer_bwd: H=128 needs scratch");
    const int nl = node_fn->nlin;
    NodeItemsArgs p{a, scratch, scratch + n * H, scratch + 2 * n * H};
    const int64_t nH = n * H;
    if (nl == 3) launch_bwd(k_node_items<3>, nslab, kItemsLdsW, stream, p);
    else launch_bwd(k_node_items<2>, nslab, kItemsLdsW, stream, p);
    const int64_t vb = slab_nmat_floats(SGNN_SLAB_NODE, H, 0, nl), W = kWaves, ss = a.slab_stride;
    const float* hl = nl == 3 ? saves->h2 : saves->h;
    run_wgrad<4, 4>(wg(p.dy_out, 0, H, nH, hl, 0, H, nH, slab, 0, H, vb + W * H, ss, nslab, n, nullptr), nslab, stream);
    run_wgrad<4, 4>(wg(p.dh_out, 0, H, nH, saves->agg, 0, H, nH, slab, H * H, 2 * H, vb, ss, nslab, n, nullptr), nslab,
                    stream);
    run_wgrad<4, 4>(wg(p.dh_out, 0, H, nH, x_in, 0, H, nH, slab, H * H + H, 2 * H, -1, ss, nslab, n, nullptr), nslab,
                    stream);
    if (nl == 3)
      run_wgrad<4, 4>(wg(p.d2_out, 0, H, nH, saves->h, 0, H, nH, slab, 3 * H * H, H, vb + 4 * W * H, ss, nslab, n, nullptr),
                      nslab, stream);
    return check_launch("node_layer_bwd");
  }
  if (H == 64 && node_fn->nlin == 2) {  // two workgroups per CU
    launch_bwd(k_node_bwd64, nslab, 4 * (size_t)(H * H + 2 * kChunk * H), stream, a);
    return check_launch("node_layer_bwd");
  }
  const size_t lds = bwd_lds(SGNN_SLAB_NODE, H, 0, node_fn->nlin);
  SGNN_BWD_DISPATCH(H, node_fn->nlin, (launch_bwd(k_node_bwd<TH_, NL_>, nslab, lds, stream, a)));
  return check_launch("node_layer_bwd");
}

extern "C" int sgnn_uv_bwd(const float* dxp, const float* du, const float* cin, const float* cout,
                           const int32_t* rowptr, const float* dh_rows, const int32_t* tptr,
                           const int32_t* tperm, const float* x_in, int64_t n,
                           const sgnn_mlp* edge_fn, float* g, float* slab, int32_t nslab,
                           float* scratch, void* stream) {
  using namespace sgnn;
  if (!edge_fn || !dxp || !du || !cin || !cout || !rowptr || !dh_rows || !tptr || !tperm ||
      !x_in || !g || !slab || nslab < 1 || n <= 0)
    return set_error(SGNN_ERR_INVALID, "uv_bwd: bad arguments");
  int st = check_bwd_mlp(edge_fn, "uv_bwd: edge MLP");
  if (st) return st;
  const int H = edge_fn->hidden;
  UvBwdArgs a{dxp, du, cin, cout, rowptr, dh_rows, tptr, tperm, x_in, n, edge_fn->w1, g, slab,
              sgnn_bwd_slab_floats(SGNN_SLAB_UV, H, 0, edge_fn->nlin)};
  if (H == 128) {
    if (!scratch) return set_error(SGNN_ERR_INVALID, "uv_bwd: H=128 needs scratch");
    UvItemsArgs p{a, scratch, scratch + n * H};
    const int64_t nH = n * H;
    launch_bwd(k_uv_items, nslab, 0, stream, p);
    const int64_t ss = a.slab_stride;
    run_wgrad<4, 4>(wg(p.du_out, 0, H, nH, x_in, 0, H, nH, slab, 0, 2 * H, 2 * H * H, ss, nslab, n, nullptr), nslab,
                    stream);
    run_wgrad<4, 4>(wg(p.dv_out, 0, H, nH, x_in, 0, H, nH, slab, H, 2 * H, -1, ss, nslab, n, nullptr), nslab, stream);
    return check_launch("uv_bwd");
  }
  launch_bwd(k_uv_bwd64, nslab, 4 * (size_t)(H * H + 2 * kChunk * H), stream, a);
  return check_launch("uv_bwd");
}

extern "C" int sgnn_decoder_loss_bwd(const float* pred, const float* pos_seq,
                                     const float* next_pos, const float* noise,
                                     const float* next_strain, const float* acc_mean,
                                     const float* acc_std, int64_t n, int32_t T, int32_t dim,
                                     float w_pos, float w_strain, float inv_count,
                                     const float* dpred, const sgnn_saves* saves,
                                     const float* x_last, const sgnn_mlp* decoder, float* g,
                                     float* slab, int32_t nslab, void* stream) {
  using namespace sgnn;
  if (!decoder || !pred || !saves || !saves->hd || !x_last || !g || !slab || nslab < 1 || n <= 0 ||
      T < 2 || dim < 1 || dim > 3 ||
      (!dpred && (!pos_seq || !next_pos || !next_strain || !acc_mean || !acc_std)))
    return set_error(SGNN_ERR_INVALID, "decoder_loss_bwd: bad arguments");
  int st = check_bwd_mlp(decoder, "decoder_loss_bwd: decoder MLP");
  if (st) return st;
  if (decoder->nlin == 3 && !saves->hd2) return set_error(SGNN_ERR_INVALID, "decoder_loss_bwd: saves->hd2");
  const int H = decoder->hidden;
  if (decoder->out_dim != dim + 1) return set_error(SGNN_ERR_INVALID, "decoder_loss_bwd: out dim");
  DecBwdArgs a{pred, pos_seq, next_pos, noise, next_strain, acc_mean, acc_std, n, T, dim,
               w_pos, w_strain, inv_count, dpred, saves->hd, saves->hd2, x_last, decoder->w1,
               mid_w(decoder), last_w(decoder), g, slab,
               sgnn_bwd_slab_floats(SGNN_SLAB_DECODER, H, 0, decoder->nlin)};
  const size_t lds = bwd_lds(SGNN_SLAB_DECODER, H, 0, decoder->nlin);
  SGNN_BWD_DISPATCH(H, decoder->nlin, (launch_bwd(k_dec_bwd<TH_, NL_>, nslab, lds, stream, a)));
  return check_launch("decoder_loss_bwd");
}

namespace {
constexpr int kTypeSumNodes = 256;   // nodes per k_type_sums workgroup
constexpr int kMaxTypes = 256;

// G[t][u] = sum over nodes i of type t of dh[i][u], deterministic: workgroup b
// sums its node range in ascending order into LDS (thread u owns column u, so
// no two threads touch one word), partials [b][t][u] are then summed over b in
// ascending order by k_type_sums_reduce.
__global__ __launch_bounds__(128) void k_type_sums(const float* dh, const int64_t* types, int64_t n, int H,
                                                   int ntypes, float* partial) {
  extern __shared__ float acc[];   // [ntypes][H]
  for (int q = threadIdx.x; q < ntypes * H; q += blockDim.x) acc[q] = 0.0f;
  __syncthreads();
  const int64_t i0 = (int64_t)blockIdx.x * kTypeSumNodes, i1 = min(i0 + kTypeSumNodes, n);
  for (int u = threadIdx.x; u < H; u += blockDim.x)
    for (int64_t i = i0; i < i1; ++i) {
      const int64_t t = types[i];
      if (t >= 0 && t < ntypes) acc[t * H + u] += dh[i * H + u];
    }
  __syncthreads();
  for (int q = threadIdx.x; q < ntypes * H; q += blockDim.x)
    partial[(int64_t)blockIdx.x * ntypes * H + q] = acc[q];
}

__global__ __launch_bounds__(256) void k_type_sums_reduce(const float* partial, int nblk, int count, float* G) {
  const int q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= count) return;
  float s = 0.0f;
  for (int b = 0; b < nblk; ++b) s += partial[(int64_t)b * count + q];
  G[q] = s;
}
}  // namespace

extern "C" size_t sgnn_type_sums_workspace_bytes(int64_t n, int32_t hidden, int32_t ntypes) {
  const int64_t nblk = (n + kTypeSumNodes - 1) / kTypeSumNodes;
  return sizeof(float) * ((size_t)n * hidden + (size_t)nblk * ntypes * hidden);
}

static int encode_nodes_bwd_impl(const float* g, const float* pos_seq, int64_t n, int32_t T, int32_t dim,
                                 const int64_t* types, const float* emb_w, int32_t emb_dim, int32_t ntypes,
                                 int32_t use_emb, const float* vel_mean, const float* vel_std, float wall_max,
                                 float wall_div, const sgnn_saves* saves, const sgnn_mlp* enc, float* slab,
                                 int32_t nslab, void* stream, float* dh_out) {
  using namespace sgnn;
  if (!enc || !g || !pos_seq || !vel_mean || !vel_std || !saves || !saves->h || !saves->yhat ||
      !saves->rstd || !slab || nslab < 1 || n <= 0)
    return set_error(SGNN_ERR_INVALID, "encode_nodes_bwd: bad arguments");
  int st = check_bwd_mlp(enc, "encode_nodes_bwd: encoder MLP");
  if (st) return st;
  if (enc->nlin == 3 && !saves->h2) return set_error(SGNN_ERR_INVALID, "encode_nodes_bwd: saves->h2");
  const int H = enc->hidden;
  const int feat = (T - 1) * dim + 1 + (use_emb ? emb_dim : 0);
  if (enc->in_dim != feat) return set_error(SGNN_ERR_INVALID, "encode_nodes_bwd: encoder input width");
  if (use_emb && (!types || !emb_w || ntypes < 1 || ntypes > (dh_out ? kMaxTypes : 32)))
    return set_error(SGNN_ERR_UNSUPPORTED, dh_out ? "encode_nodes_bwd: embeddings need types, weights, ntypes <= 256"
                                                  : "encode_nodes_bwd: embeddings need types, weights, ntypes <= 32 "
                                                    "(sgnn_encode_nodes_bwd_typed: <= 256)");
  const int tkf = (feat + 31) / 32;
  EncNodeBwdArgs a{g, pos_seq, n, T, dim, feat, vel_mean, vel_std, wall_max, wall_div, saves->h,
                   saves->h2, saves->yhat, saves->rstd, last_w(enc), mid_w(enc), enc->ln_g, slab,
                   sgnn_bwd_slab_floats(SGNN_SLAB_ENC_NODE, H, feat, enc->nlin), types, emb_w,
                   use_emb ? emb_dim : 0, use_emb, dh_out};
  const size_t lds = bwd_lds(SGNN_SLAB_ENC_NODE, H, tkf, enc->nlin);
  if (tkf == 1) {
    SGNN_BWD_DISPATCH(H, enc->nlin, (launch_bwd(k_enc_node_bwd<TH_, 1, NL_>, nslab, lds, stream, a)));
  } else if (tkf == 2) {
    SGNN_BWD_DISPATCH(H, enc->nlin, (launch_bwd(k_enc_node_bwd<TH_, 2, NL_>, nslab, lds, stream, a)));
  } else {
    return set_error(SGNN_ERR_UNSUPPORTED, "encode_nodes_bwd: > 64 node features");
  }
  return check_launch("encode_nodes_bwd");
}

extern "C" int sgnn_encode_nodes_bwd(const float* g, const float* pos_seq, int64_t n, int32_t T,
                                     int32_t dim, const int64_t* types, const float* emb_w,
                                     int32_t emb_dim, int32_t ntypes, int32_t use_emb,
                                     const float* vel_mean, const float* vel_std,
                                     float wall_max, float wall_div, const sgnn_saves* saves,
                                     const sgnn_mlp* enc, float* slab, int32_t nslab,
                                     void* stream) {
  return encode_nodes_bwd_impl(g, pos_seq, n, T, dim, types, emb_w, emb_dim, ntypes, use_emb, vel_mean, vel_std,
                               wall_max, wall_div, saves, enc, slab, nslab, stream, nullptr);
}

extern "C" int sgnn_encode_nodes_bwd_typed(const float* g, const float* pos_seq, int64_t n, int32_t T,
                                           int32_t dim, const int64_t* types, const float* emb_w,
                                           int32_t emb_dim, int32_t ntypes, const float* vel_mean,
                                           const float* vel_std, float wall_max, float wall_div,
                                           const sgnn_saves* saves, const sgnn_mlp* enc, float* slab,
                                           int32_t nslab, float* G, void* workspace, void* stream) {
  using namespace sgnn;
  if (!G || !workspace || !enc) return set_error(SGNN_ERR_INVALID, "encode_nodes_bwd_typed: bad arguments");
  const int H = enc->hidden;
  float* dh = static_cast<float*>(workspace);
  int st = encode_nodes_bwd_impl(g, pos_seq, n, T, dim, types, emb_w, emb_dim, ntypes, 1, vel_mean, vel_std,
                                 wall_max, wall_div, saves, enc, slab, nslab, stream, dh);
  if (st) return st;
  if ((size_t)ntypes * H * sizeof(float) > 160 * 1024)
    return set_error(SGNN_ERR_UNSUPPORTED, "encode_nodes_bwd_typed: ntypes x hidden > 40960");
  const int nblk = (int)((n + kTypeSumNodes - 1) / kTypeSumNodes);
  float* partial = dh + n * H;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const size_t lds = sizeof(float) * (size_t)ntypes * H;
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(k_type_sums), hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)lds);
  hipLaunchKernelGGL(k_type_sums, dim3(nblk), dim3(128), lds, s, dh, types, n, H, ntypes, partial);
  const int count = ntypes * H;
  hipLaunchKernelGGL(k_type_sums_reduce, dim3((count + 255) / 256), dim3(256), 0, s, partial, nblk, count, G);
  return check_launch("encode_nodes_bwd_typed");
}

extern "C" int sgnn_encode_edges_bwd(const float* de0t, const float* pos, int64_t pos_stride,
                                     int32_t dim, float radius, const int32_t* rowptr,
                                     const int32_t* send, const int32_t* recv, int64_t n,
                                     const sgnn_saves* saves, const sgnn_mlp* enc, float* slab,
                                     int32_t nslab, float* scratch, int64_t edge_cap,
                                     void* stream) {
  using namespace sgnn;
  if (!enc || !de0t || !pos || !rowptr || !send || !recv || !saves || !saves->yhat ||
      !saves->rstd || !slab || nslab < 1 || n <= 0)
    return set_error(SGNN_ERR_INVALID, "encode_edges_bwd: bad arguments");
  int st = check_bwd_mlp(enc, "encode_edges_bwd: encoder MLP");
  if (st) return st;
  if (enc->nlin == 3 && !saves->h2) return set_error(SGNN_ERR_INVALID, "encode_edges_bwd: saves->h2");
  const int H = enc->hidden;
  EncEdgeBwdArgs a{de0t, pos, pos_stride, dim, radius, rowptr, send, recv, n, saves->h2,
                   saves->yhat, saves->rstd, enc->w1, enc->b1, last_w(enc), mid_w(enc), enc->ln_g,
                   slab, sgnn_bwd_slab_floats(SGNN_SLAB_ENC_EDGE, H, 0, enc->nlin)};
  if (H == 128) {
    if (!scratch || edge_cap < 1) return set_error(SGNN_ERR_INVALID, "encode_edges_bwd: H=128 needs scratch");
    const int nl = enc->nlin;
    const int64_t pad = 32 * ((edge_cap + 31) / 32);
    EncEdgeItemsArgs p{a, scratch, scratch + pad * H, scratch + 2 * pad * H, scratch + 3 * pad * H,
                       scratch + 4 * pad * H};
    const int64_t tl = pad * H;
    const size_t lds = kItemsLds + 4 * (size_t)(128 * 5 + 128);
    if (nl == 3) launch_bwd(k_enc_edge_items<3>, nslab, lds, stream, p);
    else launch_bwd(k_enc_edge_items<2>, nslab, lds, stream, p);
    const int64_t vb = slab_nmat_floats(SGNN_SLAB_ENC_EDGE, H, 0, nl), W = kWaves, ss = a.slab_stride;
    const int32_t* Edev = rowptr + n;
    const float* hl = nl == 3 ? saves->h2 : p.h1_out;
    run_wgrad<4, 4>(wg(p.dy_out, 1, 0, tl, hl, 1, 0, tl, slab, 0, H, vb + W * H, ss, nslab, 0, Edev), nslab, stream);
    run_wgrad<4, 1>(wg(p.dh_out, 1, 0, tl, p.f_out, 0, 32, pad * 32, slab, H * H, 32, vb, ss, nslab, 0, Edev), nslab,
                    stream);
    if (nl == 3)
      run_wgrad<4, 4>(wg(p.d2_out, 1, 0, tl, p.h1_out, 1, 0, tl, slab, H * H + H * 32, H, vb + 4 * W * H, ss, nslab, 0,
                         Edev),
                      nslab, stream);
    return check_launch("encode_edges_bwd");
  }
  if (H == 64 && enc->nlin == 2 && dim <= 3) {  // single-scale training: two workgroups per CU
    launch_bwd(k_enc_edge_bwd64, nslab, 4 * (size_t)(H * H + 2 * kChunk * H), stream, a);
    return check_launch("encode_edges_bwd");
  }
  const size_t lds = bwd_lds(SGNN_SLAB_ENC_EDGE, H, 0, enc->nlin);
  SGNN_BWD_DISPATCH(H, enc->nlin, (launch_bwd(k_enc_edge_bwd<TH_, NL_>, nslab, lds, stream, a)));
  return check_launch("encode_edges_bwd");
}

extern "C" int sgnn_reduce_slabs(const sgnn_reduce_desc* descs_dev, const int32_t* block_start,
                                 int32_t ndesc, int32_t nblocks, void* stream) {
  using namespace sgnn;
  if (!descs_dev || !block_start || ndesc < 1 || nblocks < 1)
    return set_error(SGNN_ERR_INVALID, "reduce_slabs: bad arguments");
  hipLaunchKernelGGL(k_reduce_slabs, dim3((unsigned)nblocks), dim3(256), 0,
                     static_cast<hipStream_t>(stream), descs_dev, block_start, ndesc);
  return check_launch("reduce_slabs");
}

extern "C" size_t sgnn_transpose_workspace_bytes(int64_t n, int64_t edge_cap) {
  return sizeof(int32_t) * (size_t)(2 * (n + 1) + edge_cap) + 3 * 256 + 65536;
}

extern "C" int sgnn_transpose_csr(const int32_t* rowptr, const int32_t* send, int64_t n,
                                  int64_t edge_cap, void* workspace, int32_t* tptr,
                                  int32_t* tperm, void* stream) {
  using namespace sgnn;
  if (!rowptr || !send || !workspace || !tptr || !tperm || n <= 0 || edge_cap < 1)
    return set_error(SGNN_ERR_INVALID, "transpose_csr: bad arguments");
  hipStream_t s = static_cast<hipStream_t>(stream);
  char* p = static_cast<char*>(workspace);
  auto take = [&](size_t bytes) {
    char* r = p;
    p += (bytes + 255) & ~size_t(255);
    return r;
  };
  int32_t* cnt = reinterpret_cast<int32_t*>(take(sizeof(int32_t) * 2 * (n + 1)));
  int32_t* fill = cnt + (n + 1);
  int32_t* raw = reinterpret_cast<int32_t*>(take(sizeof(int32_t) * edge_cap));
  int32_t* partials = reinterpret_cast<int32_t*>(take(65536 - 512));
  (void)hipMemsetAsync(cnt, 0, sizeof(int32_t) * 2 * (n + 1), s);
  const unsigned g = (unsigned)std::min<int64_t>((edge_cap + 255) / 256, 2048);
  hipLaunchKernelGGL(k_tcsr_count, dim3(g), dim3(256), 0, s, rowptr, n, send, cnt);
  int st = scan_exclusive(cnt, tptr, n + 1, partials, s);
  if (st) return st;
  hipLaunchKernelGGL(k_tcsr_fill, dim3(g), dim3(256), 0, s, rowptr, n, send, tptr, fill, raw);
  hipLaunchKernelGGL(k_tcsr_sort, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, s, tptr, n, raw,
                     tperm);
  return check_launch("transpose_csr");
}

namespace {
// dEmb[t][c] (+)= sum_u G[t][u] W1[u][col0 + c]   (G = per-type sums of dh)
__global__ __launch_bounds__(256) void k_embedding_grad(const float* G, int ntypes, int H,
                                                        const float* w1, int ld, int col0,
                                                        int emb_dim, float* demb, int accumulate) {
  for (int idx = blockIdx.x * blockDim.x + threadIdx.x; idx < ntypes * emb_dim;
       idx += gridDim.x * blockDim.x) {
    const int t = idx / emb_dim, c = idx - t * emb_dim;
    float s = 0.0f;
    for (int u = 0; u < H; ++u) s += G[t * H + u] * w1[(int64_t)u * ld + col0 + c];
    demb[idx] = accumulate ? demb[idx] + s : s;
  }
}
}  // namespace

extern "C" int sgnn_embedding_grad(const float* G, int32_t ntypes, int32_t hidden, const float* w1,
                                   int32_t w1_ld, int32_t col0, int32_t emb_dim, float* demb,
                                   int32_t accumulate, void* stream) {
  using namespace sgnn;
  if (!G || !w1 || !demb || ntypes < 1 || ntypes > 256 || hidden < 1 || emb_dim < 1)
    return set_error(SGNN_ERR_INVALID, "embedding_grad: bad arguments");
  hipLaunchKernelGGL(k_embedding_grad, dim3((ntypes * emb_dim + 255) / 256), dim3(256), 0,
                     static_cast<hipStream_t>(stream), G, ntypes, hidden, w1, w1_ld, col0, emb_dim,
                     demb, accumulate);
  return check_launch("embedding_grad");
}

// ---------------------------------------------------------------------------
// dE0 = sum_k scale_k W1e_k^T dh_k over the interaction layers sharing one
// encoded edge latent (the input of layer k is scale_k e0, scale_k = 2^k):
// one streaming pass over the edges after the layer backwards, instead of a
// read-modify-write of dE0 inside every layer's edge backward.
namespace {
constexpr int kMaxLatentLayers = 9;
struct EdgeLatentGradArgs {
  const float* dh[kMaxLatentLayers];   // [E][H] rows per layer
  const float* we[kMaxLatentLayers];   // edge W1 + 2H per layer (ld 3H)
  float* slab[kMaxLatentLayers];       // SLAB_EDGE slab arena of each layer
  float scale[kMaxLatentLayers];
  int nlayers;
  const int32_t* rowptr;
  int64_t n;
  const float* e0t;
  float* de0t;
  int64_t slab_stride;
};

// One pass over the edges after the layer backwards (H = 64), per 128-edge
// chunk: e0 (loaded once) as an LDS item image, then for every layer k the
// dh_k rows (next layer's prefetched under this one's MFMAs):
//   dE0  += (2^k W1e_k^T) dh_k                (register MFMAs)
//   dW1e_k += sum_items dh_k (x) e0           (LDS images, items as k;
//                                              2^k applied in the slab reduction)
// The W1e_k^T images sit in LDS for L <= 5 (GW = false), else are read from L2.
// DE / DW select the two halves: the dW1e-only variant (L = 1) runs per layer
// on a side stream as soon as that layer's dh is written, the dE0-only pass
// afterwards carries no item images and no barriers.
template <int TH, int L, bool GW, bool DE = true, bool DW = true>
__global__ __launch_bounds__(kBlock) void k_edge_latent_grad(EdgeLatentGradArgs a) {
  constexpr int H = 32 * TH, ldh = H + 4;
  constexpr int NT = (TH * TH + kWaves - 1) / kWaves;
  extern __shared__ float lds[];
  float* bufA = lds;                  // dh_k item image
  float* bufB = bufA + kChunk * ldh;  // e0 item image
  float* wimg = DW ? bufB + kChunk * ldh : lds;  // 2^k W1e_k^T (GW = false)
  if constexpr (DE && !GW) {
#pragma unroll
    for (int k = 0; k < L; ++k) stage_matrix_t(wimg + k * H * ldh, ldh, a.we[k], 3 * H, H, H, H, H, a.scale[k]);
  }
  __syncthreads();
  const Imgs im = make_imgs(bufA, ldh, bufB, ldh);
  const int w = wave_id(), j = im.j;
  f32x16 acc[L][NT];
  if constexpr (DW) {
#pragma unroll
    for (int k = 0; k < L; ++k) zero_acc<NT>(acc[k]);
  }
  const int64_t E = a.rowptr[a.n];
  const int64_t nchunks = (E + kChunk - 1) / kChunk;
  for (int64_t c = blockIdx.x; c < nchunks; c += gridDim.x) {
    const int64_t tile = c * kWaves + w, base = tile * 32, e = base + j;
    const int nvalid = clamp_items(E - base);
    const bool valid = e < E;
    const int64_t ec = valid ? e : E - 1;
    f32x16 de[TH], cur[TH], nxt[TH], e0[TH];
    zero<TH>(de);
    zero<TH>(e0);
    zero<TH>(cur);
    if (nvalid > 0) {  // tiles past the last valid one are not allocated
      if (DW) load_tiled<TH>(e0, a.e0t + tile * (32 * H));
      load_row_clayout<TH>(cur, a.dh[0] + ec * H);
    }
    if constexpr (DW) {
      zero_if<TH>(e0, !valid);
      lds_store_items<TH>(im.sB, ldh, j, e0);
    }
#pragma unroll
    for (int k = 0; k < L; ++k) {
      if (k + 1 < L && nvalid > 0) load_row_clayout<TH>(nxt, a.dh[k + 1] + ec * H);  // prefetch
      zero_if<TH>(cur, !valid);
      if (DW) lds_store_items<TH>(im.sA, ldh, j, cur);
      if constexpr (!DE) {
      } else if constexpr (GW) {
#pragma unroll
        for (int t = 0; t < TH; ++t)
#pragma unroll
          for (int r = 0; r < 16; ++r) cur[t][r] *= a.scale[k];   // 2^k: exact
        matvec_t<TH, TH, true>(de, a.we[k], 3 * H, cur);
      } else {
        mfma_from_acc<TH, TH>(de, wimg + k * H * ldh, ldh, 0, cur);
      }
      if constexpr (DW) {
        __syncthreads();
        outer_tiles<NT>(acc[k], TH, TH, bufA, ldh, 0, bufB, ldh, 0);
        __syncthreads();
      }
      if (k + 1 < L) {
#pragma unroll
        for (int t = 0; t < TH; ++t) cur[t] = nvalid > 0 ? nxt[t] : cur[t];
      }
    }
    if (DE && nvalid > 0) store_tiled<TH>(a.de0t + tile * (32 * H), de);
  }
  if constexpr (DW) {
#pragma unroll
    for (int k = 0; k < L; ++k)
      store_outer<NT>(a.slab[k] + blockIdx.x * a.slab_stride + H * H, H, TH, TH, acc[k]);
  }
}

// dW1e_k = sum_e dh_k[e] (x) e0[e] for one layer (H = 64), streamed: every
// wave's next 32 edges (dh_k rows and the e0 tile, both contiguous) load into
// registers while the current chunk's outer product runs, so the launch is
// one HBM stream under the MFMAs instead of load -> barrier -> MFMA rounds.
// (Folding this layer's dE0 term in as well -- dE0 += 2^k W1e_k^T dh_k per
// layer on the side stream -- measured slower: the W1e^T image keeps it at
// one workgroup per CU and the dE0 read-modify-write per layer moves more
// bytes than k_edge_de0's single pass.)
template <int TH>
__global__ __launch_bounds__(kBlock) void k_edge_w1e_grad(EdgeLatentGradArgs a) {
  constexpr int H = 32 * TH, ldh = H + 4;
  constexpr int NT = (TH * TH + kWaves - 1) / kWaves;
  extern __shared__ float lds[];
  float* bufA = lds;                  // dh_k item image
  float* bufB = bufA + kChunk * ldh;  // e0 item image
  const Imgs im = make_imgs(bufA, ldh, bufB, ldh);
  const int w = wave_id(), j = im.j;
  f32x16 acc[NT];
  zero_acc<NT>(acc);
  const int64_t E = a.rowptr[a.n];
  const int64_t nchunks = (E + kChunk - 1) / kChunk, G = gridDim.x;
  auto fetch = [&](int64_t c, f32x16 (&e0)[TH], f32x16 (&dh)[TH]) {
    const int64_t tile = c * kWaves + w, base = tile * 32, e = base + j;
    if (c < nchunks && base < E) {  // tiles past the last valid one are not allocated
      load_tiled<TH>(e0, a.e0t + tile * (32 * H));
      load_row_clayout<TH>(dh, a.dh[0] + (e < E ? e : E - 1) * H);
    } else {
      zero<TH>(e0);
      zero<TH>(dh);
    }
  };
  f32x16 e0[TH], dh[TH];
  fetch(blockIdx.x, e0, dh);
  // drain the first chunk's loads here: the waitcnt pass merges this
  // preheader state into the loop header and would otherwise make every
  // iteration wait for its own freshly issued prefetch
  __builtin_amdgcn_s_waitcnt(0);
  for (int64_t c = blockIdx.x; c < nchunks; c += G) {
    f32x16 e0n[TH], dhn[TH];
    fetch(c + G, e0n, dhn);
    const bool valid = (c * kWaves + w) * 32 + j < E;
    zero_if<TH>(e0, !valid);
    zero_if<TH>(dh, !valid);
    lds_store_items<TH>(im.sA, ldh, j, dh);
    lds_store_items<TH>(im.sB, ldh, j, e0);
    __syncthreads();
    outer_tiles<NT>(acc, TH, TH, bufA, ldh, 0, bufB, ldh, 0);
    __syncthreads();
#pragma unroll
    for (int t = 0; t < TH; ++t) {
      e0[t] = e0n[t];
      dh[t] = dhn[t];
    }
  }
  store_outer<NT>(a.slab[0] + blockIdx.x * a.slab_stride + H * H, H, TH, TH, acc);
}

// dE0 = sum_k 2^k W1e_k^T dh_k over L <= 5 layers (H = 64): the L swizzled
// 64x64 images of 2^k W1e_k^T fill exactly 80 KB of LDS, so two 8-wave
// workgroups share a CU (4 waves per SIMD); no item images and no barriers in
// the loop -- every wave owns whole 32-edge tiles (grid-stride over waves)
// and prefetches layer k+1's dh rows under layer k's 64 MFMAs.
constexpr int kDe0Waves = 8;   // 512-thread workgroups: 4 waves per SIMD at <= 128 VGPRs

template <int L>
__global__ __launch_bounds__(64 * kDe0Waves) __attribute__((amdgpu_waves_per_eu(4)))
void k_edge_de0(EdgeLatentGradArgs a) {
  constexpr int TH = 2, H = 64;
  extern __shared__ float lds[];
  if (threadIdx.x < kBlock) {
#pragma unroll
    for (int k = 0; k < L; ++k) swz_stage_wt(lds + k * H * H, a.we[k], 3 * H, a.scale[k]);
  }
  __syncthreads();
  const int j = lane_id() & 31;
  const int64_t E = a.rowptr[a.n];
  const int64_t ntiles = (E + 31) / 32, nw = (int64_t)gridDim.x * kDe0Waves;
  for (int64_t tile = (int64_t)blockIdx.x * kDe0Waves + wave_id(); tile < ntiles; tile += nw) {
    const int64_t e = tile * 32 + j, ec = e < E ? e : E - 1;
    f32x16 de[TH], cur[TH], nxt[TH];
    zero<TH>(de);
    load_row_clayout<TH>(cur, a.dh[0] + ec * H);
#pragma unroll
    for (int k = 0; k < L; ++k) {
      if (k + 1 < L) load_row_clayout<TH>(nxt, a.dh[k + 1] + ec * H);
      zero_if<TH>(cur, e >= E);
      swz_matvec_t(de, lds + k * H * H, cur);
      if (k + 1 < L) {
#pragma unroll
        for (int t = 0; t < TH; ++t) cur[t] = nxt[t];
      }
      __builtin_amdgcn_sched_barrier(0);   // one layer's rows in flight, not all L
    }
    store_tiled<TH>(a.de0t + tile * (32 * H), de);
  }
}

// DE / DW: both halves (one pass), dE0 only (no item images), or dW1e only
// (L = 1, one layer per launch).
template <int L, bool DE, bool DW>
void launch_latent(const EdgeLatentGradArgs& a, int nslab, void* stream) {
  constexpr int H = 64, ldh = H + 4;
  constexpr bool GW = L > 5;
  const size_t lds = 4 * (size_t)((DW ? 2 * kChunk * ldh : 0) + (GW || !DE ? 0 : L * H * ldh));
  launch_bwd(k_edge_latent_grad<2, L, GW, DE, DW>, nslab, lds, stream, a);
}

template <int L>
void launch_latent(const EdgeLatentGradArgs& a, int nslab, void* stream, bool dw) {
  if (dw) return launch_latent<L, true, true>(a, nslab, stream);
  if constexpr (L <= 5) {   // dE0 only: the 80 KB two-workgroups-per-CU pass
    const size_t lds = 4 * (size_t)L * 64 * 64;
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(k_edge_de0<L>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(k_edge_de0<L>, dim3((unsigned)nslab), dim3(64 * kDe0Waves), lds,
                       static_cast<hipStream_t>(stream), a);
    return;
  }
  launch_latent<L, true, false>(a, nslab, stream);
}
}  // namespace

extern "C" int sgnn_edge_latent_grad(const float* const* dh_rows, const sgnn_mlp* edge_fns,
                                     const float* scales, int32_t nlayers, const int32_t* rowptr,
                                     int64_t n, int64_t edge_cap, const float* e0t, float* de0t,
                                     float* const* slabs, int32_t nslab, void* stream) {
  using namespace sgnn;
  if (!dh_rows || !edge_fns || !scales || !rowptr || !e0t || (!de0t && !slabs) || nslab < 1 ||
      nlayers < 1 || n <= 0 || edge_cap < 1)
    return set_error(SGNN_ERR_INVALID, "edge_latent_grad: bad arguments");
  const int H = edge_fns[0].hidden;
  if (H != 64) return set_error(SGNN_ERR_UNSUPPORTED, "edge_latent_grad: hidden 64 only (128 accumulates in-layer)");
  if (nlayers > kMaxLatentLayers)
    return set_error(SGNN_ERR_UNSUPPORTED, "edge_latent_grad: at most 9 layers share an edge latent");
  EdgeLatentGradArgs a{};
  for (int k = 0; k < nlayers; ++k) {
    if (!dh_rows[k] || !edge_fns[k].w1 || edge_fns[k].hidden != H || (slabs && !slabs[k]) ||
        edge_fns[k].nlin != edge_fns[0].nlin)
      return set_error(SGNN_ERR_INVALID, "edge_latent_grad: layer arguments");
    a.dh[k] = dh_rows[k];
    a.we[k] = edge_fns[k].w1 + 2 * H;
    a.slab[k] = slabs ? slabs[k] : nullptr;
    a.scale[k] = scales[k];
  }
  a.nlayers = nlayers;
  a.rowptr = rowptr;
  a.n = n;
  a.e0t = e0t;
  a.de0t = de0t;
  a.slab_stride = sgnn_bwd_slab_floats(SGNN_SLAB_EDGE, H, 0, edge_fns[0].nlin);
  if (!de0t) {  // dW1e only: one launch per layer
    for (int k = 0; k < nlayers; ++k) {
      EdgeLatentGradArgs b = a;
      b.dh[0] = a.dh[k];
      b.we[0] = a.we[k];
      b.slab[0] = a.slab[k];
      b.scale[0] = a.scale[k];
      b.nlayers = 1;
      launch_bwd(k_edge_w1e_grad<2>, nslab, 4 * (size_t)(2 * kChunk * (H + 4)), stream, b);
    }
    return check_launch("edge_latent_grad");
  }
  const bool dw = slabs != nullptr;
  switch (nlayers) {
    case 1: launch_latent<1>(a, nslab, stream, dw); break;
    case 2: launch_latent<2>(a, nslab, stream, dw); break;
    case 3: launch_latent<3>(a, nslab, stream, dw); break;
    case 4: launch_latent<4>(a, nslab, stream, dw); break;
    case 5: launch_latent<5>(a, nslab, stream, dw); break;
    case 6: launch_latent<6>(a, nslab, stream, dw); break;
    case 7: launch_latent<7>(a, nslab, stream, dw); break;
    case 8: launch_latent<8>(a, nslab, stream, dw); break;
    default: launch_latent<9>(a, nslab, stream, dw); break;
  }
  return check_launch("edge_latent_grad");
}

