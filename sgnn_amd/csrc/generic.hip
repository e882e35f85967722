// The feature construction of LearnedSimulator._encoder_preprocessor
// (learned_simulator.py:231-316) on explicit tensors: node features (velocity
// history, wall distance, type embedding) and edge features (normalised
// displacement and its norm) of a CSR graph.  The width-generic path
// (sgnn_amd/autograd.py over autograd.hip) feeds them to the modules at shapes
// the fused encoders are not built for.
#include "../../include/sgnn.h"
#include "common.h"
#include "sgnn_internal.h"

namespace {

constexpr int kGBlock = 256;

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
