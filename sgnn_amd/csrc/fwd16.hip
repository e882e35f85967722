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
#include "sgnn_internal.h"

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

template <int NL, int MODE>
__global__ __launch_bounds__(kBlock16) void k_node16(Node16Args a) {
  __shared__ float xb[kBufs][16 * LDX];
  const int l = lane_id(), j = l & 15, g = l >> 4, b = wave_id();
  const int urow = 16 * b + j;      // the W row this lane feeds as the A operand
  const int ucol = 16 * b + 4 * g;  // the 4 output units this lane holds in D
  // weights of this wave's 16 output rows, resident for the whole launch
  f32x4 w1a[KQ], w1x[KQ], wm[KQ], w2[KQ], wa[KQ], wmd[KQ], wb[KQ];
  load_wrow(w1a, a.w1, 2 * H, urow, 0, g);
  load_wrow(w1x, a.w1, 2 * H, urow, H, g);
  if (NL == 3) load_wrow(wm, a.wm, H, urow, 0, g);
  load_wrow(w2, a.w2, H, urow, 0, g);
  const f32x4 vb1 = ld4(a.b1 + ucol), vb2 = ld4(a.b2 + ucol);
  const f32x4 vg = ld4(a.g + ucol), vbb = ld4(a.bb + ucol);
  const f32x4 vbm = NL == 3 ? ld4(a.bm + ucol) : zero4();
  f32x4 vba, vbmd = zero4(), vbo = zero4();
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
  float* bh = xb[0];
  float* bm = xb[1];
  float* by = xb[2];
  float* bx = xb[3];
  float* bd = xb[4];
  float* bd2 = xb[5];
  for (int64_t tile = blockIdx.x; tile * 16 < a.n; tile += gridDim.x) {
    const int64_t i = tile * 16 + j;
    const bool valid = i < a.n;
    const int64_t ic = valid ? i : a.n - 1;
    f32x4 ag[KQ], xr[KQ];
    load_agg16(ag, a, ic, g);
#pragma unroll
    for (int q = 0; q < KQ; ++q) xr[q] = ld4(a.x_in + ic * H + 16 * q + 4 * g);
    const f32x4 xo = ld4(a.x_in + ic * H + ucol);  // residual: own units
    f32x4 hr[KQ], yr[KQ];
    const f32x4 h = relu4(mm_cat(vb1, w1a, ag, w1x, xr));  // graph_network.py:220
    xchg(bh, j, ucol, g, h, hr);
    f32x4 y;
    if constexpr (NL == 3) {
      f32x4 mr[KQ];
      xchg(bm, j, ucol, g, relu4(mm(vbm, wm, hr)), mr);
      y = mm(vb2, w2, mr);
    } else {
      y = mm(vb2, w2, hr);
    }
    xchg(by, j, ucol, g, y, yr);
    float mean, rstd;
    ln_stats(yr, mean, rstd);
    f32x4 xn;
#pragma unroll
    for (int c = 0; c < 4; ++c) xn[c] = (y[c] - mean) * rstd * vg[c] + vbb[c] + xo[c];  // LN, :176 residual
    if (valid && a.x_out) st4(a.x_out + i * H + ucol, xn);
    f32x4 xnr[KQ];
    xchg(bx, j, ucol, g, xn, xnr);
    if constexpr (MODE == 0) {
      const f32x4 u = mm(vba, wa, xnr);
      const f32x4 v = mm(zero4(), wb, xnr);
      if (valid) {
        st4(a.u + i * H + ucol, u);
        st4(a.v + i * H + ucol, v);
      }
    } else {
      f32x4 hdr[KQ];
      xchg(bd, j, ucol, g, relu4(mm(vba, wa, xnr)), hdr);
      if constexpr (NL == 3) {
        f32x4 hd2r[KQ];
        xchg(bd2, j, ucol, g, relu4(mm(vbmd, wmd, hdr)), hd2r);
#pragma unroll
        for (int q = 0; q < KQ; ++q) hdr[q] = hd2r[q];
      }
      const int D = a.dim;
      if (b == 0) {
        const f32x4 o = mm(vbo, wb, hdr);  // lanes g == 0 hold outputs 0..3
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

}  // namespace sgnn
