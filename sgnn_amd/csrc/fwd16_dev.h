// Device helpers of the H = 64 items-on-lanes kernels on v_mfma_f32_16x16x4_f32
// (fwd16.hip: node layer / fused layer / encoder; step16.hip: the one-launch
// step).  Layout: see fwd16.hip.
#pragma once
#include "common.h"
#include "fwd16.h"

namespace {

using sgnn::Node16Args;

constexpr int H = 64;
constexpr int KQ = H / 16;          // float4 groups per lane for K = H
constexpr int LDX = H + 4;          // LDS exchange row stride (floats)
constexpr int kWaves16 = H / 16;    // one wave per 16-unit output block
constexpr int kBlock16 = 64 * kWaves16;
constexpr int kBufs = 6;            // distinct exchange buffers per node tile

SGNN_DEV f32x4 mfma16(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

SGNN_DEV f32x4 zero4() { return f32x4{0.0f, 0.0f, 0.0f, 0.0f}; }

SGNN_DEV f32x4 relu4(f32x4 v) {
#pragma unroll
  for (int c = 0; c < 4; ++c) v[c] = fmaxf(v[c], 0.0f);
  return v;
}

// w[q] = W[row][col0 + 16 q + 4 g .. +3] (zero when !ok)
template <int Q>
SGNN_DEV void load_wrow(f32x4 (&w)[Q], const float* W, int ld, int row, int col0, int g, bool ok = true) {
#pragma unroll
  for (int q = 0; q < Q; ++q) w[q] = ok ? ld4(W + (int64_t)row * ld + col0 + 16 * q + 4 * g) : zero4();
}

// init + sum_k W[own unit][k] X[item][k], K = 16 Q, two accumulator chains
// (the dependent-accumulator latency is 40 cycles against 32 of issue).
template <int Q>
SGNN_DEV f32x4 mm(f32x4 init, const f32x4 (&w)[Q], const f32x4 (&x)[Q]) {
  f32x4 a0 = init, a1 = zero4();
#pragma unroll
  for (int q = 0; q < Q; q += 2)
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      a0 = mfma16(w[q][c], x[q][c], a0);
      if (q + 1 < Q) a1 = mfma16(w[q + 1][c], x[q + 1][c], a1);
    }
  return a0 + a1;
}

// init + W_a agg + W_x x (the node MLP's first Linear on cat[aggr, x]).
SGNN_DEV f32x4 mm_cat(f32x4 init, const f32x4 (&wa)[KQ], const f32x4 (&xa)[KQ], const f32x4 (&wx)[KQ],
                      const f32x4 (&xx)[KQ]) {
  f32x4 a0 = init, a1 = zero4();
#pragma unroll
  for (int q = 0; q < KQ; ++q)
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      a0 = mfma16(wa[q][c], xa[q][c], a0);
      a1 = mfma16(wx[q][c], xx[q][c], a1);
    }
  return a0 + a1;
}

// Publish this wave's unit block of 16 items, read back the full rows.
SGNN_DEV void xchg(float* buf, int j, int ucol, int g, f32x4 v, f32x4 (&out)[KQ]) {
  st4(buf + j * LDX + ucol, v);
  __syncthreads();
#pragma unroll
  for (int q = 0; q < KQ; ++q) out[q] = ld4(buf + j * LDX + 16 * q + 4 * g);
}

// Two-pass LayerNorm statistics of the full rows (torch: biased variance, eps 1e-5).
SGNN_DEV void ln_stats(const f32x4 (&r)[KQ], float& mean, float& rstd) {
  float p[4] = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
  for (int q = 0; q < KQ; ++q)
#pragma unroll
    for (int c = 0; c < 4; ++c) p[c] += r[q][c];
  float s = (p[0] + p[1]) + (p[2] + p[3]);
  s += __shfl_xor(s, 16, 64);
  s += __shfl_xor(s, 32, 64);
  mean = s * (1.0f / H);
#pragma unroll
  for (int c = 0; c < 4; ++c) p[c] = 0.0f;
#pragma unroll
  for (int q = 0; q < KQ; ++q)
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const float d = r[q][c] - mean;
      p[c] += d * d;
    }
  float v = (p[0] + p[1]) + (p[2] + p[3]);
  v += __shfl_xor(v, 16, 64);
  v += __shfl_xor(v, 32, 64);
  rstd = 1.0f / sqrtf(v * (1.0f / H) + 1e-5f);
}

// Aggregated messages of node i (full row in B layout): the edge layer left
// either the whole row in agg or, for a receiver whose edges straddle 32-edge
// tiles, a head partial in cout and whole-tile partials in cin.
SGNN_DEV void load_agg16(f32x4 (&ag)[KQ], const Node16Args& a, int64_t i, int g) {
  const int32_t r0 = a.rowptr[i], r1 = a.rowptr[i + 1];
  if (r1 <= r0) {
#pragma unroll
    for (int q = 0; q < KQ; ++q) ag[q] = zero4();
    return;
  }
  const int32_t t0 = r0 >> 5, t1 = (r1 - 1) >> 5;
  const float* src = t0 == t1 ? a.agg + i * H : a.cout + (int64_t)t0 * H;
#pragma unroll
  for (int q = 0; q < KQ; ++q) ag[q] = ld4(src + 16 * q + 4 * g);
  for (int32_t t = t0 + 1; t <= t1; ++t)
#pragma unroll
    for (int q = 0; q < KQ; ++q) ag[q] += ld4(a.cin + (int64_t)t * H + 16 * q + 4 * g);
}

SGNN_DEV float comp(f32x4 v, int c) { return c == 0 ? v[0] : c == 1 ? v[1] : c == 2 ? v[2] : v[3]; }

// Node-side weights of one wave's 16 output rows (node MLP, then the next
// edge MLP's node halves or the decoder), resident for the whole launch.
template <int NL, int MODE>
struct NodeW {
  f32x4 w1a[KQ], w1x[KQ], wm[KQ], w2[KQ], wa[KQ], wmd[KQ], wb[KQ];
  f32x4 vb1, vb2, vg, vbb, vbm, vba, vbmd, vbo;
  SGNN_DEV void load(const Node16Args& a, int b, int j, int g) {
    const int urow = 16 * b + j, ucol = 16 * b + 4 * g;
    load_wrow(w1a, a.w1, 2 * H, urow, 0, g);
    load_wrow(w1x, a.w1, 2 * H, urow, H, g);
    vb1 = ld4(a.b1 + ucol);
    load_tail(a, b, j, g);
  }
  // everything after the first Linear (the encoder supplies its own first Linear)
  SGNN_DEV void load_tail(const Node16Args& a, int b, int j, int g) {
    load_mid(a, b, j, g);
    load_out(a, b, j, g);
  }
  // the first Linear only / the node MLP's tail / the next edge MLP's node halves or the decoder: three
  // parts the one-launch step requests at different points
  SGNN_DEV void load_first(const Node16Args& a, int b, int j, int g) {
    const int urow = 16 * b + j, ucol = 16 * b + 4 * g;
    load_wrow(w1a, a.w1, 2 * H, urow, 0, g);
    load_wrow(w1x, a.w1, 2 * H, urow, H, g);
    vb1 = ld4(a.b1 + ucol);
  }
  SGNN_DEV void load_mid(const Node16Args& a, int b, int j, int g) {
    const int urow = 16 * b + j, ucol = 16 * b + 4 * g;
    if (NL == 3) load_wrow(wm, a.wm, H, urow, 0, g);
    load_wrow(w2, a.w2, H, urow, 0, g);
    vb2 = ld4(a.b2 + ucol);
    vg = ld4(a.g + ucol);
    vbb = ld4(a.bb + ucol);
    vbm = NL == 3 ? ld4(a.bm + ucol) : zero4();
  }
  SGNN_DEV void load_out(const Node16Args& a, int b, int j, int g) {
    const int urow = 16 * b + j, ucol = 16 * b + 4 * g;
    vbmd = zero4();
    vbo = zero4();
    if (MODE == 0) {  // next edge MLP: u = W1_i x + b1 (cols 0..H), v = W1_j x (cols H..2H)
      load_wrow(wa, a.we, 3 * H, urow, 0, g);
      load_wrow(wb, a.we, 3 * H, urow, H, g);
      vba = ld4(a.be + ucol);
    } else {          // decoder: H -> H (-> H) -> dim + 1, no LayerNorm
      load_wrow(wa, a.wd1, H, urow, 0, g);
      vba = ld4(a.bd1 + ucol);
      if (NL == 3) {
        load_wrow(wmd, a.wdm, H, urow, 0, g);
        vbmd = ld4(a.bdm + ucol);
      }
      load_wrow(wb, a.wd2, H, j, 0, g, j <= a.dim);  // output rows 0..dim of a 16-row tile
#pragma unroll
      for (int c = 0; c < 4; ++c) vbo[c] = 4 * g + c <= a.dim ? a.bd2[4 * g + c] : 0.0f;
    }
  }
};

// The node update of 16 items (node i on lane row j; `valid` false on padding
// rows) from their aggregated messages `ag` (full rows): node MLP + LN +
// residual -> x_out, then u/v (mode 0) or decoder + integrator (mode 1).
// bufs: kBufs exchange buffers [16][LDX] (every wave of the workgroup calls).
// x rows of the 16 items (B layout) and this wave's own units (residual).
SGNN_DEV void load_x16(const Node16Args& a, int64_t ic, int b, int g, f32x4 (&xr)[KQ], f32x4& xo) {
#pragma unroll
  for (int q = 0; q < KQ; ++q) xr[q] = ld4(a.x_in + ic * H + 16 * q + 4 * g);
  xo = ld4(a.x_in + ic * H + 16 * b + 4 * g);
}

// e0 of edge e, units 16 q + 4 g .. +3 (32-edge MFMA-C-layout tiles)
SGNN_DEV f32x4 ld_e0_edge(const float* e0t, int64_t e, int q, int g) {
  const int64_t tile = e >> 5;
  const int item = (int)(e & 31);
  const int t = q >> 1, gg = 2 * (q & 1) + (g >> 1), hh = g & 1;
  return ld4(e0t + tile * (32 * H) + (t * 4 + gg) * 256 + (item + 32 * hh) * 4);
}

// Row-local (16-lane) DPP shifts: lane j of a row receives lane j - d (shr)
// or j + 1 (shl 1); lanes without a source keep `fill`.
template <int D>
SGNN_DEV int dpp_shr_c(int v, int fill) {
  return __builtin_amdgcn_update_dpp(fill, v, 0x110 + D, 0xf, 0xf, false);
}
SGNN_DEV int dpp_row_shr(int v, int d, int fill) {
  return d == 1 ? dpp_shr_c<1>(v, fill) : d == 2 ? dpp_shr_c<2>(v, fill) : d == 4 ? dpp_shr_c<4>(v, fill)
                                                                                  : dpp_shr_c<8>(v, fill);
}
SGNN_DEV int dpp_row_shl1(int v, int fill) { return __builtin_amdgcn_update_dpp(fill, v, 0x101, 0xf, 0xf, false); }

// One Linear over all H units of 16 items held as 4 unit tiles (lane (j, g):
// units 16 t + 4 g + c of item j in acc[t][c]); A rows from an LDS image
// [H][LDX]; B = x (the same tile layout: tile q supplies k = 16 q + 4 g + c).
// Four independent accumulator chains, so the MFMAs issue back to back.
// TR: the same products with the operands swapped, y^T = x^T W^T: lane (j, g) then holds
// y[unit 16 t + j][item 4 g + c] (units on the lane's row position, items on its column group).
template <bool TR = false>
SGNN_DEV void mm_full(f32x4 (&acc)[KQ], const float* Wl, const f32x4 (&x)[KQ], int j, int g) {
  f32x4 w[2][KQ];  // the A rows of k-group q + 1 are read while group q multiplies
#pragma unroll
  for (int t = 0; t < KQ; ++t) w[0][t] = ld4(Wl + (16 * t + j) * LDX + 4 * g);
#pragma unroll
  for (int q = 0; q < KQ; ++q) {
    if (q + 1 < KQ) {
#pragma unroll
      for (int t = 0; t < KQ; ++t) w[(q + 1) & 1][t] = ld4(Wl + (16 * t + j) * LDX + 16 * (q + 1) + 4 * g);
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int t = 0; t < KQ; ++t)
        acc[t] = TR ? mfma16(x[q][c], w[q & 1][t][c], acc[t]) : mfma16(w[q & 1][t][c], x[q][c], acc[t]);
    __builtin_amdgcn_sched_barrier(0);
  }
}

// Stage a [H][H] weight block (row stride ldg, optional scale) into an LDS
// image [H][LDX] in two parts: float4 loads into registers, later the LDS
// stores (loads issued first, so the stores wait on one memory latency and
// later-issued loads stay in flight).
constexpr int kStagePer = H * H / 4 / kBlock16;
SGNN_DEV void stage_w64_load(f32x4 (&v)[kStagePer], const float* src, int ldg) {
#pragma unroll
  for (int k = 0; k < kStagePer; ++k) {
    const int idx = threadIdx.x + k * kBlock16, r = idx / (H / 4), c = (idx % (H / 4)) * 4;
    v[k] = ld4(src + (int64_t)r * ldg + c);
  }
}
SGNN_DEV void stage_w64_store(float* dst, const f32x4 (&v)[kStagePer], float scale) {
#pragma unroll
  for (int k = 0; k < kStagePer; ++k) {
    const int idx = threadIdx.x + k * kBlock16, r = idx / (H / 4), c = (idx % (H / 4)) * 4;
    st4(dst + r * LDX + c, v[k] * scale);
  }
}

}  // namespace
