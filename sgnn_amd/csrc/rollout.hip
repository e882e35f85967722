// Host-side step / rollout drivers: one C-ABI call issues a whole
// LearnedSimulator.predict_positions (learned_simulator.py:413-438) or a whole
// autoregressive rollout (evaluate.py:117-145), so the per-kernel cost on the
// host is a hipLaunchKernel (~µs) instead of a Python ctypes round trip.
#include "../../include/sgnn.h"
#include "sgnn_internal.h"
#include "radius_small.h"

extern "C" int sgnn_predict_positions(const sgnn_epd* m, const sgnn_step_in* in, const float* pos_seq,
                                      const sgnn_step_ws* ws, float* pred, float* next_pos,
                                      float* window_out, void* stream) {
  using namespace sgnn;
  if (!m || !in || !pos_seq || !ws || !pred || !next_pos || m->nlayers < 1 || !m->edge || !m->node)
    return set_error(SGNN_ERR_INVALID, "predict_positions: bad arguments");
  const int64_t n = in->n;
  const int T = in->T, d = in->dim;
  // radius graph on the most recent frame (learned_simulator.py:116-117); graphs of <= 2,560
  // particles launch its search together with the node encoder (independent work, one launch whose
  // grid fits the 256 CUs once: C1 0.1275 -> 0.1239 ms/step; measured slower at 4,800 / 8,000
  // particles, 0.156 -> 0.167 / 0.217 -> 0.268, where the radius search needs more workgroups)
  constexpr int64_t kMergeMaxN = 2560;
  RadiusSmallArgs ra{};
  const bool small = n <= kMergeMaxN && radius_small_plan(pos_seq + (int64_t)(T - 1) * d, (int64_t)T * d, n, d, in->ex_ptr,
                                       in->n_ex, in->radius, in->K, 1, ws->radius_ws, ws->rowptr, ws->send,
                                       ws->recv, ws->edge_cap, &ra);
  // small graphs at hidden 64: one fused launch per layer (u/v ping-pong), the first one with the
  // edge encoder folded in (nmlp_layers 1) -- and, after the merged radius + encoder launch, with the
  // CSR built from the radius search's padded lists (no separate compaction launch)
  const bool fused = ws->u2 && ws->v2 && m->node[0].hidden == 64 && n <= 8192;
  const bool enc_in_layer0 = fused && m->nlayers > 1 && m->enc_edge->nlin == 2 && m->node[0].nlin == 2;
  bool csr_pending = false;
  int st = SGNN_OK;
  if (!small) {
    st = sgnn_radius_graph(pos_seq + (int64_t)(T - 1) * d, (int64_t)T * d, n, d, in->ex_ptr, in->n_ex,
                           in->radius, in->K, 1, ws->radius_ws, ws->rowptr, ws->send, ws->recv,
                           ws->edge_cap, stream);
    if (st) return st;
  }
  st = encode_nodes_impl(pos_seq, n, T, d, in->types, in->emb_w, in->emb_dim, in->use_emb, in->vel_mean,
                         in->vel_std, in->wall_max, in->wall_div, m->enc_node, &m->edge[0], ws->x_a, ws->u,
                         ws->v, nullptr, stream, small ? &ra : nullptr, small && enc_in_layer0, &csr_pending);
  if (st) return st;
  const float* last = pos_seq + (int64_t)(T - 1) * d;
  float* x_in = ws->x_a;
  float* x_out = ws->x_b;
  float scale = 1.0f;
  // larger graphs keep the edge / node kernel pair (more workgroups, no per-workgroup weight staging
  // per node tile)
  if (!enc_in_layer0) {
    st = sgnn_encode_edges(last, (int64_t)T * d, d, in->radius, ws->rowptr, ws->send, ws->recv, n,
                           ws->edge_cap, m->enc_edge, ws->e0t, nullptr, stream);
    if (st) return st;
  }
  if (fused) {
    float *u_in = ws->u, *v_in = ws->v, *u_out = ws->u2, *v_out = ws->v2;
    for (int k = 0; k < m->nlayers; ++k, scale *= 2.0f) {
      if (k == 0 && enc_in_layer0) {
        st = interaction_layer_encode_impl(last, (int64_t)T * d, d, in->radius, m->enc_edge, ws->e0t, x_in, u_in,
                                           v_in, ws->rowptr, ws->send, ws->recv, n, &m->edge[0], &m->node[0],
                                           &m->edge[1], x_out, u_out, v_out, stream, csr_pending ? &ra : nullptr);
        std::swap(x_in, x_out);
        std::swap(u_in, u_out);
        std::swap(v_in, v_out);
      } else if (k < m->nlayers - 1) {
        st = sgnn_interaction_layer(x_in, u_in, v_in, ws->e0t, scale, ws->rowptr, ws->send, ws->recv, n,
                                    &m->edge[k], &m->node[k], &m->edge[k + 1], x_out, u_out, v_out, stream);
        std::swap(x_in, x_out);
        std::swap(u_in, u_out);
        std::swap(v_in, v_out);
      } else {
        st = sgnn_interaction_layer_decode(x_in, u_in, v_in, ws->e0t, scale, ws->rowptr, ws->send, ws->recv,
                                           n, &m->edge[k], &m->node[k], m->dec, pos_seq, T, d, in->acc_mean,
                                           in->acc_std, pred, next_pos, window_out, stream);
      }
      if (st) return st;
    }
    return SGNN_OK;
  }
  for (int k = 0; k < m->nlayers; ++k, scale *= 2.0f) {
    st = sgnn_edge_layer(ws->u, ws->v, ws->e0t, scale, ws->rowptr, ws->send, ws->recv, n, ws->edge_cap,
                         &m->edge[k], ws->agg, ws->cin, ws->cout, nullptr, stream);
    if (st) return st;
    if (k < m->nlayers - 1) {
      st = sgnn_node_layer(x_in, ws->agg, ws->cin, ws->cout, ws->rowptr, n, &m->node[k], &m->edge[k + 1],
                           x_out, ws->u, ws->v, nullptr, stream);
      float* t = x_in;
      x_in = x_out;
      x_out = t;
    } else {
      st = sgnn_node_layer_decode(x_in, ws->agg, ws->cin, ws->cout, ws->rowptr, n, &m->node[k], m->dec,
                                  pos_seq, T, d, in->acc_mean, in->acc_std, nullptr, pred, next_pos,
                                  window_out, nullptr, stream);
    }
    if (st) return st;
  }
  return SGNN_OK;
}

extern "C" int sgnn_rollout(const sgnn_epd* m, const sgnn_step_in* in, float* win_a, float* win_b,
                            const sgnn_step_ws* ws, int32_t nsteps, float* out_pos, float* out_pred,
                            void* stream) {
  using namespace sgnn;
  if (!win_a || !win_b || win_a == win_b || !out_pos || !out_pred || nsteps < 0)
    return set_error(SGNN_ERR_INVALID, "rollout: bad arguments");
  const int64_t n = in ? in->n : 0;
  const int d = in ? in->dim : 0;
  for (int32_t k = 0; k < nsteps; ++k) {
    float* cur = (k & 1) ? win_b : win_a;
    float* nxt = (k & 1) ? win_a : win_b;
    const int st = sgnn_predict_positions(m, in, cur, ws, out_pred + (int64_t)k * n * (d + 1),
                                          out_pos + (int64_t)k * n * d, nxt, stream);
    if (st) return st;
  }
  return SGNN_OK;
}
