// Shared device helpers for the sgnn gfx950 kernels.
//
// MFMA convention used everywhere ("items on lanes"):
//   D[unit][item] = sum_k W[unit][k] * In[item][k]      (v_mfma_f32_32x32x2_f32)
// A operand (lane l) = W[unit0 + (l&31)][kappa(s, l>>5)]  -- read from LDS
// B operand (lane l) = In[item0 + (l&31)][kappa(s, l>>5)] -- per-lane register
// D/C layout: lane l holds item (l&31); register r of tile t holds unit
//   32 t + crow(r, l>>5), crow(r, h) = (r&3) + 8 (r>>2) + 4 h.
// Because every item sits on one lane with its units in registers, an
// accumulator is directly the B operand of the next product (the k order is
// the crow permutation; the W read uses the same permutation), a row-wise
// LayerNorm is a register sum plus one lane^32 exchange, and nothing crosses
// LDS between the two Linear layers of an MLP.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

#define SGNN_DEV __device__ __forceinline__

// Debug builds (-DSGNN_DEBUG_BOUNDS, tools/exp_debug_bounds.py): index checks on the graph paths that
// print the violation (device printf, no trap) and clamp the index so the run continues; no code in
// product builds.
#ifdef SGNN_DEBUG_BOUNDS
#define SGNN_BOUNDS(idx, lo, hi, what)                                                               \
  do {                                                                                              \
    if ((int64_t)(idx) < (int64_t)(lo) || (int64_t)(idx) >= (int64_t)(hi)) {                         \
      printf("SGNN-BOUNDS %s: %lld outside [%lld, %lld) at %s:%d block %d\n", what, (long long)(idx),  \
             (long long)(lo), (long long)(hi), __FILE__, __LINE__, (int)blockIdx.x);                   \
      idx = (int64_t)(idx) < (int64_t)(lo) ? (lo) : (hi) - 1;                                         \
    }                                                                                               \
  } while (0)
#else
#define SGNN_BOUNDS(idx, lo, hi, what) \
  do {                                 \
  } while (0)
#endif
#define SGNN_HOST_DEV __host__ __device__

SGNN_DEV int lane_id() { return threadIdx.x & 63; }

// Wave index within the workgroup as a provably wave-uniform (SGPR) value:
// tile / item bookkeeping derived from it stays on the scalar unit (scalar
// loads of uniform indices, s_cbranch on uniform conditions) instead of 64-bit
// VALU arithmetic and exec-mask branches (hipcc treats threadIdx.x >> 6 as
// divergent).
SGNN_DEV int wave_id() { return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); }

SGNN_DEV int crow(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

SGNN_DEV f32x16 mfma32(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

SGNN_DEV f32x4 ld4(const float* p) { return *reinterpret_cast<const f32x4*>(p); }
SGNN_DEV void st4(float* p, f32x4 v) { *reinterpret_cast<f32x4*>(p) = v; }

SGNN_DEV float wave_xor32(float v) { return __shfl_xor(v, 32, 64); }

// Copy a [rows x cols] row-major global matrix (leading dim ldg) into LDS
// with leading dimension lds_ld, zero-filling rows >= rows_valid and columns
// >= cols_valid up to [rows_pad x cols_pad].  Optional scale.
SGNN_DEV void stage_matrix(float* lds, int lds_ld, const float* g, int ldg, int rows_valid,
                           int cols_valid, int rows_pad, int cols_pad, float scale = 1.0f) {
  const int total = rows_pad * cols_pad;
  for (int idx = threadIdx.x; idx < total; idx += blockDim.x) {
    const int r = idx / cols_pad, c = idx - r * cols_pad;
    float v = 0.0f;
    if (r < rows_valid && c < cols_valid) v = g[(int64_t)r * ldg + c] * scale;
    lds[r * lds_ld + c] = v;
  }
}

SGNN_DEV void stage_vec(float* lds, const float* g, int n_valid, int n_pad) {
  for (int idx = threadIdx.x; idx < n_pad; idx += blockDim.x)
    lds[idx] = (g != nullptr && idx < n_valid) ? g[idx] : 0.0f;
}

// acc[t] += W[32t + lane][kappa] * b for one k-step; W rows in LDS with
// leading dim ld, k offset `koff` already including the lane-half term.
template <int TH>
SGNN_DEV void mfma_step(f32x16 (&acc)[TH], const float* wl, int ld, int koff, float b) {
  const int l = lane_id() & 31;
#pragma unroll
  for (int t = 0; t < TH; ++t) acc[t] = mfma32(wl[(32 * t + l) * ld + koff], b, acc[t]);
}

// Buffer resource over a global weight matrix: loads take the per-lane part
// of the address in one VGPR, the uniform part in a scalar offset and the
// immediate (plain pointers make the compiler hoist one 64-bit address per
// unrolled load out of the item loop and spill them).
SGNN_DEV __amdgpu_buffer_rsrc_t weight_rsrc(const float* w) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(w), (short)0, 0x7ffffff0, 0x00020000);
}

SGNN_DEV f32x4 buf_ld4(__amdgpu_buffer_rsrc_t rs, int voff, int soff) {
  typedef int i32x4 __attribute__((ext_vector_type(4)));
  const i32x4 v = __builtin_bit_cast(i32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, voff, soff, 0));
  return __builtin_bit_cast(f32x4, v);
}

// W rows for one (t, k-group) product step: LDS image or global (G) matrix.
template <int TH, bool G>
struct WRows {
  const float* w;
  int ld;
  __amdgpu_buffer_rsrc_t rs;
  int voff;
  SGNN_DEV WRows(const float* w_, int ld_) : w(w_), ld(ld_) {
    const int l = lane_id() & 31, h = lane_id() >> 5;
    if constexpr (G) {
      rs = weight_rsrc(w_);
      voff = 4 * (l * ld_ + 4 * h);
    } else {
      voff = l * ld_ + 4 * h;
    }
  }
  // units 32t + lane, k = kb .. kb+3 (+4h)
  SGNN_DEV f32x4 get(int t, int kb) const {
    if constexpr (G) return buf_ld4(rs, voff, 4 * (32 * t * ld + kb));
    else return ld4(w + voff + 32 * t * ld + kb);
  }
};

// Product with the B operand in C layout (a previous accumulator X, TK
// tiles): acc[t] += sum_{k} W[32t+lane][k] X[k][item] over K = 32*TK units.
// G: W is a global (L2-resident) matrix, otherwise an LDS image.
template <int TH, int TK, bool G = false>
SGNN_DEV void mfma_from_acc(f32x16 (&acc)[TH], const float* wl, int ld, int kbase,
                            const f32x16 (&x)[TK]) {
  const WRows<TH, G> W(wl, ld);
  if constexpr (G) {
    // Global (L2) weights: the next k-group's rows are requested before this group's 4 TH MFMAs, so
    // each group's load latency hides under the previous group's products (the compiler's own
    // schedule issued every group's loads right in front of its MFMAs and waited on them: one L2
    // round trip per 16 MFMAs).  Same products in the same order: bit-identical results.
    constexpr int NG = 4 * TK;
    f32x4 w[2][TH];
#pragma unroll
    for (int t = 0; t < TH; ++t) w[0][t] = W.get(t, kbase);
#pragma unroll
    for (int s = 0; s < NG; ++s) {
      const int tk = s >> 2, g = s & 3;
      if (s + 1 < NG) {
#pragma unroll
        for (int t = 0; t < TH; ++t) w[(s + 1) & 1][t] = W.get(t, kbase + 32 * ((s + 1) >> 2) + 8 * ((s + 1) & 3));
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int c = 0; c < 4; ++c) {
#pragma unroll
        for (int t = 0; t < TH; ++t) acc[t] = mfma32(w[s & 1][t][c], x[tk][4 * g + c], acc[t]);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    return;
  }
#pragma unroll
  for (int tk = 0; tk < TK; ++tk) {
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      f32x4 w[TH];
#pragma unroll
      for (int t = 0; t < TH; ++t) w[t] = W.get(t, kbase + 32 * tk + 8 * g);
#pragma unroll
      for (int c = 0; c < 4; ++c) {
#pragma unroll
        for (int t = 0; t < TH; ++t) acc[t] = mfma32(w[t][c], x[tk][4 * g + c], acc[t]);
      }
    }
  }
}

// Same, but the B operand comes as float4 groups in the C-layout order that
// the caller loads from memory: xg[tk*4+g] holds units 32tk+8g+4h+(0..3).
template <int TH, int TK, bool G = false>
SGNN_DEV void mfma_from_groups(f32x16 (&acc)[TH], const float* wl, int ld, int kbase,
                               const f32x4 (&xg)[TK * 4], float scale) {
  const WRows<TH, G> W(wl, ld);
#pragma unroll
  for (int tk = 0; tk < TK; ++tk) {
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      f32x4 w[TH];
#pragma unroll
      for (int t = 0; t < TH; ++t) w[t] = W.get(t, kbase + 32 * tk + 8 * g);
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const float b = xg[tk * 4 + g][c] * scale;
#pragma unroll
        for (int t = 0; t < TH; ++t) acc[t] = mfma32(w[t][c], b, acc[t]);
      }
    }
  }
}

// Initialise acc with a per-unit bias (LDS vector, may be null -> 0).
// (one null test per call, then 16-B LDS reads: registers 4g..4g+3 of a tile
// hold the contiguous units 32t + 8g + 4h + 0..3)
template <int TH>
SGNN_DEV void acc_bias(f32x16 (&acc)[TH], const float* bias_lds) {
  const int h = lane_id() >> 5;
  if (bias_lds == nullptr) {
#pragma unroll
    for (int t = 0; t < TH; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[t][r] = 0.0f;
    return;
  }
#pragma unroll
  for (int t = 0; t < TH; ++t)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const f32x4 b = ld4(bias_lds + 32 * t + 8 * g + 4 * h);
#pragma unroll
      for (int c = 0; c < 4; ++c) acc[t][4 * g + c] = b[c];
    }
}

template <int TH>
SGNN_DEV void zero_acc_regs(f32x16 (&acc)[TH]) {
#pragma unroll
  for (int t = 0; t < TH; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = 0.0f;
}

template <int TH>
SGNN_DEV void acc_relu(f32x16 (&acc)[TH]) {
#pragma unroll
  for (int t = 0; t < TH; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = fmaxf(acc[t][r], 0.0f);
}

// Row-wise sums of one item's 32*TH units (lane pair l, l^32): four
// independent partial sums (short dependency chains), then the lane^32 half.
template <int TH>
SGNN_DEV float row_sum(const f32x16 (&x)[TH]) {
  float p[4] = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
  for (int t = 0; t < TH; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) p[r & 3] += x[t][r];
  const float s = (p[0] + p[1]) + (p[2] + p[3]);
  return s + wave_xor32(s);
}

template <int TH>
SGNN_DEV float row_sum_sq_dev(const f32x16 (&x)[TH], float mean) {
  float p[4] = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
  for (int t = 0; t < TH; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float d = x[t][r] - mean;
      p[r & 3] += d * d;
    }
  const float s = (p[0] + p[1]) + (p[2] + p[3]);
  return s + wave_xor32(s);
}

// Row-wise LayerNorm over the 32*TH units of each item (one lane pair), eps
// 1e-5, two-pass mean / biased variance as torch.nn.LayerNorm.
template <int TH>
SGNN_DEV void acc_layernorm(f32x16 (&acc)[TH], const float* gamma_lds, const float* beta_lds) {
  const int h = lane_id() >> 5;
  constexpr float inv_n = 1.0f / (32.0f * TH);
  const float mean = row_sum<TH>(acc) * inv_n;
  const float v = row_sum_sq_dev<TH>(acc, mean);
  const float rstd = 1.0f / sqrtf(v * inv_n + 1e-5f);
#pragma unroll
  for (int t = 0; t < TH; ++t)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const f32x4 ga = ld4(gamma_lds + 32 * t + 8 * g + 4 * h);
      const f32x4 be = ld4(beta_lds + 32 * t + 8 * g + 4 * h);
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int r = 4 * g + c;
        acc[t][r] = (acc[t][r] - mean) * rstd * ga[c] + be[c];
      }
    }
}

// Load a node-major row (row-major [N][32*TH]) in C layout into f32x16 regs.
template <int TH>
SGNN_DEV void load_row_clayout(f32x16 (&x)[TH], const float* row) {
  const int h = lane_id() >> 5;
#pragma unroll
  for (int t = 0; t < TH; ++t)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const f32x4 v = ld4(row + 32 * t + 8 * g + 4 * h);
#pragma unroll
      for (int c = 0; c < 4; ++c) x[t][4 * g + c] = v[c];
    }
}

template <int TH>
SGNN_DEV void add_row_clayout(f32x16 (&x)[TH], const float* row) {
  const int h = lane_id() >> 5;
#pragma unroll
  for (int t = 0; t < TH; ++t)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const f32x4 v = ld4(row + 32 * t + 8 * g + 4 * h);
#pragma unroll
      for (int c = 0; c < 4; ++c) x[t][4 * g + c] += v[c];
    }
}

template <int TH>
SGNN_DEV void store_row_clayout(float* row, const f32x16 (&x)[TH]) {
  const int h = lane_id() >> 5;
#pragma unroll
  for (int t = 0; t < TH; ++t)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      f32x4 v;
#pragma unroll
      for (int c = 0; c < 4; ++c) v[c] = x[t][4 * g + c];
      st4(row + 32 * t + 8 * g + 4 * h, v);
    }
}

// Predicated stores without branches: lanes that must not write get a
// buffer offset past num_records and the hardware drops their write.  A loop
// whose stores are all of this kind issues the same number of memory
// instructions on every path, so the compiler's wait counts for loads
// prefetched before them stay exact (a data-dependent number of stores makes
// every later wait a full drain).
constexpr uint32_t kBufRecords = 0x7ffffff0u;   // bytes addressable from a resource base
constexpr int kBufDrop = 0x7ffffff0;            // voffset of a dropped lane
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

SGNN_DEV __amdgpu_buffer_rsrc_t buf_rsrc(const float* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), (short)0, kBufRecords, 0x00020000);
}

// row + (units of an items-on-lanes register tile): store_row_clayout where
// `on`, a dropped write elsewhere.  voff = the row's byte offset from rs.
template <int TH>
SGNN_DEV void store_row_clayout_if(__amdgpu_buffer_rsrc_t rs, int voff, bool on, const f32x16 (&x)[TH]) {
  const int h = lane_id() >> 5;
  const int v0 = on ? voff + 16 * h : kBufDrop;
#pragma unroll
  for (int t = 0; t < TH; ++t)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      u32x4 d;
#pragma unroll
      for (int c = 0; c < 4; ++c) d[c] = __float_as_uint(x[t][4 * g + c]);
      __builtin_amdgcn_raw_buffer_store_b128(d, rs, on ? v0 + 4 * (32 * t + 8 * g) : kBufDrop, 0, 0);
    }
}

template <int CTRL, int ROWS = 0xf>
SGNN_DEV int dpp_i(int v, int fill) { return __builtin_amdgcn_update_dpp(fill, v, CTRL, ROWS, 0xf, false); }

// Receiver segment sums of one 32-edge tile held items on lanes (lane (j, h)
// = edge j of the tile, units 32t + 8g + 4h + c; recv sorted, rv = recv of
// lane's edge, valid = edge < E), with segment_sum_store's carry contract:
// a run that starts and ends in the tile -> rows[recv]; one that starts here
// and continues (nxt == recv of edge 31) -> cout[tile]; one that began in an
// earlier tile (prv == its recv) -> cin[tile].  The sums come from a
// segmented inclusive scan along the edges with DPP (row shifts 1-8 inside
// the 16-lane rows, then row_bcast:15 into the second row of each half; the
// sortedness makes "same receiver d edges back" the whole segment test), and
// the last edge of each run stores (branch-free, see store_row_clayout_if).
// x is overwritten by the scan.
template <int TH>
SGNN_DEV void segment_sum_rows(f32x16 (&x)[TH], int rv, bool valid, int prv, int nxt, int64_t tile,
                               float* rows, float* cin, float* cout) {
  constexpr int H = 32 * TH;
  const int l = lane_id(), j = l & 31;
  const int rk = valid ? rv : -1 - j;  // invalid edges: runs of their own
  auto step = [&](int pr, auto shift) {
#pragma unroll
    for (int t = 0; t < TH; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float pv = __int_as_float(shift(__float_as_int(x[t][r])));
        x[t][r] = pr == rk ? x[t][r] + pv : x[t][r];
      }
  };
  step(dpp_i<0x111>(rk, INT32_MIN), [](int v) { return dpp_i<0x111>(v, 0); });
  step(dpp_i<0x112>(rk, INT32_MIN), [](int v) { return dpp_i<0x112>(v, 0); });
  step(dpp_i<0x114>(rk, INT32_MIN), [](int v) { return dpp_i<0x114>(v, 0); });
  step(dpp_i<0x118>(rk, INT32_MIN), [](int v) { return dpp_i<0x118>(v, 0); });
  step(dpp_i<0x142, 0xa>(rk, INT32_MIN), [](int v) { return dpp_i<0x142, 0xa>(v, 0); });
  const int rn = __builtin_amdgcn_ds_bpermute(((l + 1) & 63) << 2, rk);
  const bool writer = valid && (j == 31 || rn != rk);
  const bool starts = rv != prv, cont = j == 31 && nxt == rv;
  store_row_clayout_if<TH>(buf_rsrc(rows), rv * (4 * H), writer && starts && !cont, x);
  store_row_clayout_if<TH>(buf_rsrc(cout + tile * H), 0, writer && starts && cont, x);
  store_row_clayout_if<TH>(buf_rsrc(cin + tile * H), 0, writer && !starts, x);
}

// LayerNorm that also returns the normalised value yhat and 1/std per item
// (saved by the training forward for the LayerNorm backward).
template <int TH>
SGNN_DEV void acc_layernorm_save(f32x16 (&acc)[TH], const float* gamma_lds, const float* beta_lds,
                                 f32x16 (&yhat)[TH], float& rstd_out) {
  const int h = lane_id() >> 5;
  constexpr float inv_n = 1.0f / (32.0f * TH);
  const float mean = row_sum<TH>(acc) * inv_n;
  const float v = row_sum_sq_dev<TH>(acc, mean);
  const float rstd = 1.0f / sqrtf(v * inv_n + 1e-5f);
  rstd_out = rstd;
#pragma unroll
  for (int t = 0; t < TH; ++t)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const f32x4 ga = ld4(gamma_lds + 32 * t + 8 * g + 4 * h);
      const f32x4 be = ld4(beta_lds + 32 * t + 8 * g + 4 * h);
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int r = 4 * g + c;
        const float yh = (acc[t][r] - mean) * rstd;
        yhat[t][r] = yh;
        acc[t][r] = yh * ga[c] + be[c];
      }
    }
}

// LayerNorm backward for one item per lane pair (units in registers):
//   g = dout * gamma;  dy = rstd * (g - mean(g) - yhat * mean(g * yhat)).
template <int TH>
SGNN_DEV void acc_layernorm_bwd(const f32x16 (&dout)[TH], const f32x16 (&yhat)[TH], float rstd,
                                const float* gamma_lds, f32x16 (&dy)[TH]) {
  const int h = lane_id() >> 5;
  constexpr float inv_n = 1.0f / (32.0f * TH);
  float p1[4] = {0.0f, 0.0f, 0.0f, 0.0f}, p2[4] = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
  for (int t = 0; t < TH; ++t)
#pragma unroll
    for (int gq = 0; gq < 4; ++gq) {
      const f32x4 ga = ld4(gamma_lds + 32 * t + 8 * gq + 4 * h);
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int r = 4 * gq + c;
        const float g = dout[t][r] * ga[c];
        dy[t][r] = g;
        p1[r & 3] += g;
        p2[r & 3] += g * yhat[t][r];
      }
    }
  float s1 = (p1[0] + p1[1]) + (p1[2] + p1[3]);
  float s2 = (p2[0] + p2[1]) + (p2[2] + p2[3]);
  s1 += wave_xor32(s1);
  s2 += wave_xor32(s2);
  const float m1 = s1 * inv_n, m2 = s2 * inv_n;
#pragma unroll
  for (int t = 0; t < TH; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) dy[t][r] = rstd * (dy[t][r] - m1 - yhat[t][r] * m2);
}

// Tiled per-32-item layout used for edge tensors: tile base + (t*4+g)*256 +
// lane*4 holds units 32t+8g+4h+(0..3) of item (lane&31).
template <int TH>
SGNN_DEV void load_tiled(f32x16 (&x)[TH], const float* tile_base) {
  const float* p = tile_base + lane_id() * 4;
#pragma unroll
  for (int t = 0; t < TH; ++t)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const f32x4 v = ld4(p + (t * 4 + g) * 256);
#pragma unroll
      for (int c = 0; c < 4; ++c) x[t][4 * g + c] = v[c];
    }
}

template <int TH>
SGNN_DEV void store_tiled(float* tile_base, const f32x16 (&x)[TH]) {
  float* p = tile_base + lane_id() * 4;
#pragma unroll
  for (int t = 0; t < TH; ++t)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      f32x4 v;
#pragma unroll
      for (int c = 0; c < 4; ++c) v[c] = x[t][4 * g + c];
      st4(p + (t * 4 + g) * 256, v);
    }
}

// Write an item-on-lane register tile into an LDS image [item][unit] (ld).
template <int TH>
SGNN_DEV void lds_store_items(float* img, int ld, int item, const f32x16 (&x)[TH]) {
  const int h = lane_id() >> 5;
#pragma unroll
  for (int t = 0; t < TH; ++t)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      f32x4 v;
#pragma unroll
      for (int c = 0; c < 4; ++c) v[c] = x[t][4 * g + c];
      st4(img + item * ld + 32 * t + 8 * g + 4 * h, v);
    }
}

// Outer-product accumulation over items from two LDS images [item][unit]:
//   acc[u][v] += sum_{item < nitems} A[item][ua + u] * B[item][vb + v]
// for one 32x32 output tile (u, v in 0..31): MFMA with the items as k.
// NITEMS is a compile-time multiple of 32: the LDS operands are read in
// batches of G k-steps one batch ahead of the MFMAs that consume them (the
// compiler's own schedule waited on every read pair: LDS latency per MFMA).
template <int NITEMS>
SGNN_DEV void mfma_outer(f32x16& acc, const float* A, int lda, int ua, const float* B, int ldb,
                         int vb) {
  static_assert(NITEMS % 32 == 0, "items per outer product: multiple of 32");
  constexpr int G = 8, NS = NITEMS / 2;   // k-steps per batch, k-steps
  const int l = lane_id() & 31, h = lane_id() >> 5;
  const float* pa = A + h * lda + ua + l;
  const float* pb = B + h * ldb + vb + l;
  float a0[G], b0[G], a1[G], b1[G];
#pragma unroll
  for (int i = 0; i < G; ++i) {
    a0[i] = pa[2 * i * lda];
    b0[i] = pb[2 * i * ldb];
  }
#pragma unroll
  for (int s = 0; s < NS; s += 2 * G) {
#pragma unroll
    for (int i = 0; i < G; ++i) {
      a1[i] = pa[2 * (s + G + i) * lda];
      b1[i] = pb[2 * (s + G + i) * ldb];
    }
    __builtin_amdgcn_sched_barrier(0);   // keep the reads ahead of the MFMAs
#pragma unroll
    for (int i = 0; i < G; ++i) acc = mfma32(a0[i], b0[i], acc);
    if (s + 2 * G < NS) {
#pragma unroll
      for (int i = 0; i < G; ++i) {
        a0[i] = pa[2 * (s + 2 * G + i) * lda];
        b0[i] = pb[2 * (s + 2 * G + i) * ldb];
      }
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < G; ++i) acc = mfma32(a1[i], b1[i], acc);
  }
}

// Store a 32x32 C-layout accumulator tile (rows u, cols = lane) into a
// row-major matrix region dst[u * ld + v] (v = lane&31).
SGNN_DEV void store_tile_rowmajor(float* dst, int ld, const f32x16& acc) {
  const int l = lane_id() & 31, h = lane_id() >> 5;
#pragma unroll
  for (int r = 0; r < 16; ++r) dst[crow(r, h) * ld + l] = acc[r];
}

SGNN_DEV void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Stage a [rows x cols] row-major global matrix TRANSPOSED into LDS:
// lds[c * ld + r] = g[r * ldg + c] (r < rows_valid, c < cols_valid, zero pad).
SGNN_DEV void stage_matrix_t(float* lds, int ld, const float* g, int ldg, int rows_valid,
                             int cols_valid, int rows_pad, int cols_pad, float scale = 1.0f) {
  const int total = rows_pad * cols_pad;
  if (rows_valid == rows_pad && cols_valid == cols_pad && (cols_pad & 3) == 0 && (ldg & 3) == 0 &&
      (reinterpret_cast<uintptr_t>(g) & 15) == 0) {
    // unpadded, 16-B aligned weights: float4 loads, four per thread in flight
    // (the scalar loop below waits on one load per element)
    const int q4 = cols_pad >> 2, nq = rows_pad * q4, B = blockDim.x;
    for (int b = threadIdx.x; b < nq; b += 4 * B) {
      f32x4 v[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int idx = b + i * B, r = idx / q4, c4 = idx - r * q4;
        if (idx < nq) v[i] = ld4(g + (int64_t)r * ldg + 4 * c4) * scale;
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int idx = b + i * B, r = idx / q4, c4 = idx - r * q4;
        if (idx < nq) {
#pragma unroll
          for (int c = 0; c < 4; ++c) lds[(4 * c4 + c) * ld + r] = v[i][c];
        }
      }
    }
    return;
  }
  for (int idx = threadIdx.x; idx < total; idx += blockDim.x) {
    const int r = idx / cols_pad, c = idx - r * cols_pad;
    float v = 0.0f;
    if (r < rows_valid && c < cols_valid) v = g[(int64_t)r * ldg + c] * scale;
    lds[c * ld + r] = v;
  }
}

// Tail of an MLP after its first ReLU: y = LAST(relu(MID(h))) for 3 Linear
// layers (nmlp_layers = 2), y = LAST(h) for 2 (nmlp_layers = 1).
// h2 receives the second hidden (NL = 3; untouched for NL = 2) for the
// training saves.
// The middle weights Wm are always global; Wl is global when GL.
template <int TH, int NL, int TO, bool GL = false>
SGNN_DEV void mlp_tail(f32x16 (&y)[TO], f32x16 (&h2)[TH], const f32x16 (&h)[TH], const float* Wm,
                       int ldm, const float* bm_lds, const float* Wl, int ldl, const float* bl_lds) {
  if constexpr (NL == 3) {
    acc_bias<TH>(h2, bm_lds);
    mfma_from_acc<TH, TH, true>(h2, Wm, ldm, 0, h);
    acc_relu<TH>(h2);
    acc_bias<TO>(y, bl_lds);
    mfma_from_acc<TO, TH, GL>(y, Wl, ldl, 0, h2);
  } else {
    acc_bias<TO>(y, bl_lds);
    mfma_from_acc<TO, TH, GL>(y, Wl, ldl, 0, h);
  }
}

template <int TH, int NL, int TO, bool GL = false>
SGNN_DEV void mlp_tail(f32x16 (&y)[TO], const f32x16 (&h)[TH], const float* Wm, int ldm,
                       const float* bm_lds, const float* Wl, int ldl, const float* bl_lds) {
  f32x16 h2[TH];
  mlp_tail<TH, NL, TO, GL>(y, h2, h, Wm, ldm, bm_lds, Wl, ldl, bl_lds);
}

// Segment sum over the receiver-sorted CSR of a wave's 32-item LDS slice
// (lane = unit) with tile carries (same contract as the forward edge layer).
// The 32 rows are read up front; whether a segment starts / ends its
// receiver's row follows from the neighbouring receivers (prev_recv = recv of
// the edge before the tile, next_recv = of the edge after it, -1 if none), so
// no rowptr loads sit on the serial path.
template <int TH>
SGNN_DEV void segment_sum_store(const float* slice, int ld, int rv, int nvalid, int64_t base,
                                int64_t tile, int prev_recv, int next_recv, float* dst_rows,
                                float* cin, float* cout) {
  constexpr int H = 32 * TH;
  constexpr int UPL = H / 64 > 0 ? H / 64 : 1;
  const int l = lane_id();
  float vals[UPL][32];
#pragma unroll
  for (int q = 0; q < UPL; ++q)
#pragma unroll
    for (int jj = 0; jj < 32; ++jj) vals[q][jj] = (l + 64 * q < H) ? slice[jj * ld + l + 64 * q] : 0.0f;
  float acc[UPL];
#pragma unroll
  for (int q = 0; q < UPL; ++q) acc[q] = 0.0f;
  bool starts_row = true;  // does the open segment start its receiver's row?
#pragma unroll
  for (int jj = 0; jj < 32; ++jj) {
    if (jj < nvalid) {
#pragma unroll
      for (int q = 0; q < UPL; ++q) acc[q] += vals[q][jj];
      const int rr = __builtin_amdgcn_readlane(rv, jj);
      if (jj == 0) starts_row = prev_recv != rr;
      const int nx = (jj + 1 < nvalid) ? __builtin_amdgcn_readlane(rv, jj + 1) : (jj == 31 ? next_recv : -1);
      if (nx != rr) {
        const bool ends_row = true;  // the next edge belongs to another receiver (or none)
        float* dst = starts_row && ends_row ? dst_rows + (int64_t)rr * H
                   : starts_row ? cout + tile * H : cin + tile * H;
        (void)ends_row;
#pragma unroll
        for (int q = 0; q < UPL; ++q) {
          if (l + 64 * q < H) dst[l + 64 * q] = acc[q];
          acc[q] = 0.0f;
        }
        starts_row = true;
      }
    }
  }
  // an open segment at the tile end continues into the next tile
  if (nvalid == 32) {
    const int rr = __builtin_amdgcn_readlane(rv, 31);
    if (next_recv == rr) {
      float* dst = starts_row ? cout + tile * H : cin + tile * H;
#pragma unroll
      for (int q = 0; q < UPL; ++q)
        if (l + 64 * q < H) dst[l + 64 * q] = acc[q];
    }
  }
}
