// Width-generic building blocks (any latent / hidden / edge widths, any
// nmlp_layers): the reference's build_mlp (graph_network.py:7-45) on rows
// gathered from up to three sources, the receiver sums of MessagePassing
// (aggr='add', graph_network.py:136), and the feature construction of
// LearnedSimulator._encoder_preprocessor (learned_simulator.py:231-316).
//
// These serve the shapes the MFMA kernels are not instantiated for (hidden
// widths other than 64 / 128, latent_dim != mlp_hidden_dim, nedge_out !=
// latent_dim) and the reference's per-module forwards on explicit tensors
// (Encoder / InteractionNetwork / Processor / Decoder, G2M / M2M / M2G
// blocks).  Plain fp32 FMA, one dot product per thread with the input rows
// staged in LDS: correct for every width, not the fast path -- the H = 64 /
// 128 kernels are.
#include "../../include/sgnn.h"
#include "common.h"
#include "sgnn_internal.h"

namespace {

constexpr int kRows = 8;      // rows per workgroup tile
constexpr int kGBlock = 256;

struct GSrc {
  const float* p;
  const int32_t* idx;  // row r reads p[(idx ? idx[r] : r) * ld + c]
  int64_t ld;
  int dim;
  float scale;
};

struct RowsArgs {
  GSrc src[3];
  int nsrc;
  int64_t n;
  int nlin;
  const float* w[3];
  const float* b[3];
  int dims[4];  // dims[0] = sum of source widths; dims[k + 1] = out width of Linear k
  const float *ln_g, *ln_b;
  const float* residual;  // out += residual[r] (after the LayerNorm), ld = dims[nlin]
  float* out;
  int maxd;
};

__global__ __launch_bounds__(kGBlock) void k_rows_mlp(RowsArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  float* buf0 = lds;
  float* buf1 = lds + kRows * a.maxd;
  const int tid = threadIdx.x;
  for (int64_t r0 = (int64_t)blockIdx.x * kRows; r0 < a.n; r0 += (int64_t)gridDim.x * kRows) {
    const int nr = (int)min<int64_t>(kRows, a.n - r0);
    const int din = a.dims[0];
    for (int p = tid; p < nr * din; p += kGBlock) {
      const int r = p / din;
      int c = p - r * din;
      int s = 0;
      while (c >= a.src[s].dim) c -= a.src[s++].dim;
      const GSrc& g = a.src[s];
      const int64_t row = g.idx ? g.idx[r0 + r] : r0 + r;
      buf0[r * a.maxd + p - r * din] = g.p[row * g.ld + c] * g.scale;
    }
    __syncthreads();
    float* in = buf0;
    float* out = buf1;
    for (int k = 0; k < a.nlin; ++k) {
      const int K = a.dims[k], U = a.dims[k + 1];
      const bool last = k == a.nlin - 1;
      const float* W = a.w[k];
      for (int p = tid; p < nr * U; p += kGBlock) {
        const int r = p / U, u = p - r * U;
        const float* x = in + r * a.maxd;
        const float* wr = W + (int64_t)u * K;
        float acc = a.b[k] ? a.b[k][u] : 0.0f;
        for (int c = 0; c < K; ++c) acc = fmaf(wr[c], x[c], acc);
        out[r * a.maxd + u] = last ? acc : fmaxf(acc, 0.0f);
      }
      __syncthreads();
      float* t = in;
      in = out;
      out = t;
    }
    // LayerNorm (biased variance, eps 1e-5) + residual: one wave per row
    const int U = a.dims[a.nlin];
    const int lane = lane_id(), w = wave_id();
    for (int r = w; r < nr; r += kGBlock / 64) {
      const float* y = in + r * a.maxd;
      float mean = 0.0f, rstd = 1.0f;
      if (a.ln_g) {
        float s = 0.0f;
        for (int u = lane; u < U; u += 64) s += y[u];
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) s += __shfl_xor(s, o, 64);
        mean = s / U;
        float v = 0.0f;
        for (int u = lane; u < U; u += 64) {
          const float d = y[u] - mean;
          v += d * d;
        }
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
        rstd = 1.0f / sqrtf(v / U + 1e-5f);
      }
      for (int u = lane; u < U; u += 64) {
        float o = a.ln_g ? (y[u] - mean) * rstd * a.ln_g[u] + a.ln_b[u] : y[u];
        if (a.residual) o += a.residual[(r0 + r) * U + u];
        a.out[(r0 + r) * U + u] = o;
      }
    }
    __syncthreads();
  }
}

// agg[i][c] = sum over p in [rowptr[i], rowptr[i+1]) of m[perm ? perm[p] : p][c], in CSR order.
__global__ __launch_bounds__(kGBlock) void k_segment_sum(const float* m, const int32_t* rowptr, const int32_t* perm,
                                                        int64_t n, int width, float* agg) {
  const int64_t total = n * width;
  for (int64_t t = (int64_t)blockIdx.x * kGBlock + threadIdx.x; t < total; t += (int64_t)gridDim.x * kGBlock) {
    const int64_t i = t / width;
    const int c = (int)(t - i * width);
    float s = 0.0f;
    for (int32_t p = rowptr[i]; p < rowptr[i + 1]; ++p) s += m[(int64_t)(perm ? perm[p] : p) * width + c];
    agg[t] = s;
  }
}

// LearnedSimulator._encoder_preprocessor's node features (learned_simulator.py:256-290).
__global__ __launch_bounds__(kGBlock) void k_node_features(const float* pos_seq, int64_t n, int T, int dim,
                                                          const int64_t* types, const float* emb_w, int emb_dim,
                                                          int use_emb, const float* vel_mean, const float* vel_std,
                                                          float wall_max, float wall_div, int feat, float* out) {
  const int64_t total = n * feat;
  const int nvel = (T - 1) * dim;
  for (int64_t t = (int64_t)blockIdx.x * kGBlock + threadIdx.x; t < total; t += (int64_t)gridDim.x * kGBlock) {
    const int64_t i = t / feat;
    const int f = (int)(t - i * feat);
    const float* p = pos_seq + i * T * dim;
    float v = 0.0f;
    if (f < nvel) {
      const int k = f / dim, c = f - k * dim;
      v = __fdiv_rn(__fsub_rn(__fsub_rn(p[(k + 1) * dim + c], p[k * dim + c]), vel_mean[c]), vel_std[c]);
    } else if (f == nvel) {
      v = __fdiv_rn(fminf(fmaxf(__fadd_rn(p[(T - 1) * dim], 2.0f), 0.0f), wall_max), wall_div);
    } else if (use_emb) {
      v = emb_w[types[i] * emb_dim + (f - nvel - 1)];
    }
    out[t] = v;
  }
}

// Edge features (p_s - p_r) / R and their norm (learned_simulator.py:299-312), CSR order.
__global__ __launch_bounds__(kGBlock) void k_edge_features(const float* pos, int64_t stride, int dim, float radius,
                                                          const int32_t* send, const int32_t* recv,
                                                          const int32_t* rowptr, int64_t n, float* out) {
  const int64_t E = rowptr[n];
  for (int64_t e = (int64_t)blockIdx.x * kGBlock + threadIdx.x; e < E; e += (int64_t)gridDim.x * kGBlock) {
    const float* ps = pos + (int64_t)send[e] * stride;
    const float* pr = pos + (int64_t)recv[e] * stride;
    float ss = 0.0f;
    for (int c = 0; c < dim; ++c) {
      const float d = __fdiv_rn(__fsub_rn(ps[c], pr[c]), radius);
      out[e * (dim + 1) + c] = d;
      ss = __fadd_rn(ss, __fmul_rn(d, d));
    }
    out[e * (dim + 1) + dim] = sqrtf(ss);
  }
}

unsigned grid_for(int64_t items, int64_t per_wg) {
  return (unsigned)std::max<int64_t>(1, std::min<int64_t>((items + per_wg - 1) / per_wg, 2048));
}

}  // namespace

extern "C" int sgnn_rows_mlp(const sgnn_rows_src* srcs, int32_t nsrc, int64_t n, const sgnn_mlp* mlp,
                             const float* residual, float* out, void* stream) {
  using namespace sgnn;
  if (n <= 0) return SGNN_OK;
  if (!srcs || nsrc < 1 || nsrc > 3 || !mlp || !out || !mlp->w1 || !mlp->w2 || (mlp->nlin == 3 && !mlp->w3))
    return set_error(SGNN_ERR_INVALID, "rows_mlp: bad arguments");
  if (mlp->nlin < 2 || mlp->nlin > 3) return set_error(SGNN_ERR_UNSUPPORTED, "rows_mlp: 2 or 3 Linear layers");
  RowsArgs a{};
  int din = 0;
  for (int s = 0; s < nsrc; ++s) {
    if (!srcs[s].data || srcs[s].dim < 1 || srcs[s].ld < srcs[s].dim)
      return set_error(SGNN_ERR_INVALID, "rows_mlp: bad row source");
    a.src[s] = GSrc{srcs[s].data, srcs[s].index, srcs[s].ld, srcs[s].dim, srcs[s].scale};
    din += srcs[s].dim;
  }
  if (din != mlp->in_dim) return set_error(SGNN_ERR_INVALID, "rows_mlp: source widths != MLP input width");
  a.nsrc = nsrc;
  a.n = n;
  a.nlin = mlp->nlin;
  a.w[0] = mlp->w1; a.b[0] = mlp->b1;
  if (mlp->nlin == 2) {
    a.w[1] = mlp->w2; a.b[1] = mlp->b2;
  } else {
    a.w[1] = mlp->w2; a.b[1] = mlp->b2; a.w[2] = mlp->w3; a.b[2] = mlp->b3;
  }
  a.dims[0] = din;
  for (int k = 1; k < mlp->nlin; ++k) a.dims[k] = mlp->hidden;
  a.dims[mlp->nlin] = mlp->out_dim;
  a.ln_g = mlp->ln_g; a.ln_b = mlp->ln_b;
  if ((a.ln_g == nullptr) != (a.ln_b == nullptr)) return set_error(SGNN_ERR_INVALID, "rows_mlp: half a LayerNorm");
  a.residual = residual;
  a.out = out;
  a.maxd = std::max({din, mlp->hidden, mlp->out_dim});
  const size_t lds = sizeof(float) * 2 * kRows * (size_t)a.maxd;
  if (lds > 160 * 1024) return set_error(SGNN_ERR_UNSUPPORTED, "rows_mlp: rows wider than the LDS tile");
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(k_rows_mlp), hipFuncAttributeMaxDynamicSharedMemorySize,
                            160 * 1024);
  hipLaunchKernelGGL(k_rows_mlp, dim3(grid_for(n, kRows)), dim3(kGBlock), lds, static_cast<hipStream_t>(stream), a);
  return check_launch("rows_mlp");
}

extern "C" int sgnn_segment_sum(const float* m, const int32_t* rowptr, const int32_t* perm, int64_t n, int32_t width,
                                float* agg, void* stream) {
  using namespace sgnn;
  if (n <= 0) return SGNN_OK;
  if (!m || !rowptr || !agg || width < 1) return set_error(SGNN_ERR_INVALID, "segment_sum: bad arguments");
  hipLaunchKernelGGL(k_segment_sum, dim3(grid_for(n * width, kGBlock)), dim3(kGBlock), 0,
                     static_cast<hipStream_t>(stream), m, rowptr, perm, n, width, agg);
  return check_launch("segment_sum");
}

extern "C" int sgnn_node_features(const float* pos_seq, int64_t n, int32_t T, int32_t dim, const int64_t* types,
                                  const float* emb_w, int32_t emb_dim, int32_t use_emb, const float* vel_mean,
                                  const float* vel_std, float wall_max, float wall_div, float* out, void* stream) {
  using namespace sgnn;
  if (n <= 0) return SGNN_OK;
  if (!pos_seq || !out || T < 2 || dim < 1 || dim > 3 || !vel_mean || !vel_std || (use_emb && (!types || !emb_w)))
    return set_error(SGNN_ERR_INVALID, "node_features: bad arguments");
  const int feat = (T - 1) * dim + 1 + (use_emb ? emb_dim : 0);
  hipLaunchKernelGGL(k_node_features, dim3(grid_for(n * feat, kGBlock)), dim3(kGBlock), 0,
                     static_cast<hipStream_t>(stream), pos_seq, n, T, dim, types, emb_w, emb_dim, use_emb, vel_mean,
                     vel_std, wall_max, wall_div, feat, out);
  return check_launch("node_features");
}

extern "C" int sgnn_edge_features(const float* pos, int64_t pos_stride, int32_t dim, float radius,
                                  const int32_t* rowptr, const int32_t* send, const int32_t* recv, int64_t n,
                                  int64_t edge_cap, float* out, void* stream) {
  using namespace sgnn;
  if (n <= 0) return SGNN_OK;
  if (!pos || !rowptr || !send || !recv || !out || dim < 1 || dim > 3 || !(radius > 0.0f))
    return set_error(SGNN_ERR_INVALID, "edge_features: bad arguments");
  hipLaunchKernelGGL(k_edge_features, dim3(grid_for(edge_cap, kGBlock)), dim3(kGBlock), 0,
                     static_cast<hipStream_t>(stream), pos, pos_stride, dim, radius, send, recv, rowptr, n, out);
  return check_launch("edge_features");
}
