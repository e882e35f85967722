// Inference-path node kernels on v_mfma_f32_16x16x4_f32 (fwd16.hip): shared
// between the translation units that dispatch to them.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace sgnn {

struct RadiusSmallArgs;  // radius_small.h

// One InteractionNetwork node update (graph_network.py:201-222) + residual
// (:176), followed by the NEXT layer's edge-MLP node halves u, v (mode 0) or
// the decoder + Euler integrator (mode 1, learned_simulator.py:381-411).
struct Node16Args {
  const float *x_in, *agg, *cin, *cout;
  const int32_t* rowptr;
  int64_t n;
  const float *w1, *b1, *wm, *bm, *w2, *b2, *g, *bb;  // node MLP (wm/bm: nmlp_layers = 2)
  // mode 0: next edge MLP's first Linear [H][3H] and bias
  const float *we, *be;
  float *u, *v;
  // mode 1: decoder (wdm/bdm: nmlp_layers = 2) + integrator
  const float *wd1, *bd1, *wdm, *bdm, *wd2, *bd2;
  const float* pos_seq;
  int T, dim;
  const float *acc_mean, *acc_std;
  float *pred, *next_pos, *window_out;
  float* x_out;
};

// Launches the H = 64 kernel (nl = Linear layers per MLP, 2 or 3).
int node16_launch(const Node16Args& a, int mode, int nl, hipStream_t stream);

// One whole InteractionNetwork layer (graph_network.py:150-222) in ONE launch:
// a workgroup owns `nt` consecutive receivers, runs the edge MLP over all of
// their incoming edges (a contiguous range of the receiver-sorted CSR), sums
// the messages in LDS, and applies the node update of node16 to them.  Reads
// u_in / v_in (this layer's node halves), writes nd.u / nd.v (the next
// layer's) -- distinct buffers, since other workgroups still gather u_in.
struct Layer16Args {
  Node16Args nd;
  const float *u_in, *v_in, *e0t;
  float e_scale;
  const int32_t *send, *recv;
  const float *ewe, *ewm, *ebm, *ew2, *eb2, *eg, *ebb;  // edge MLP (ewe = W1 + 2H, ld 3H)
  int nt;
  // first layer only (first = true): Encoder.edge_fn fused in -- e0 of every
  // edge from the positions (learned_simulator.py:299-312, graph_network.py:
  // 92-96; nmlp_layers = 1), used at once and written to e0t_out for the
  // later layers
  const float* pos;  // most recent frame, particle i at pos + i * pos_stride
  int64_t pos_stride;
  int dim;
  float radius;
  const float *xw1, *xb1, *xw2, *xb2, *xg, *xbb;
  float* e0t_out;
  // first layer, optional: the radius search's padded lists (l_deg [n], l_nbr
  // [n][l_cap]) instead of the CSR -- every workgroup builds its tile's CSR
  // rows in LDS and writes them (rowptr / send / recv above) for the later
  // layers; needs one tile per workgroup (tiles <= 512)
  const int32_t *l_deg, *l_nbr;
  int l_cap;
  int32_t *rowptr_out, *send_out, *recv_out;
};

int layer16_launch(const Layer16Args& a, int mode, int nl, hipStream_t stream, bool first = false);

// Encoder, node side (learned_simulator.py:256-290 features -> Encoder.node_fn,
// graph_network.py:86-90) + the first layer's u/v; nd carries the encoder's
// tail Linear(s)/LayerNorm, edge0's first Linear (we, be), x_out = x0, u, v.
struct EncNode16Args {
  Node16Args nd;
  const float* pos_seq;
  int T, dim;
  const int64_t* types;
  const float* emb_w;
  int emb_dim, use_emb;
  const float *vel_mean, *vel_std;
  float wall_max, wall_div;
  int feat;
  const float *w1, *b1;  // encoder first Linear [H][feat]
};
int enc_node16_launch(const EncNode16Args& a, int nl, hipStream_t stream);
// The small-graph radius search and this encoder in one launch (they are
// independent), followed by the radius graph's CSR launch.
int radius_enc16_launch(const RadiusSmallArgs& r, const EncNode16Args& a, int nl, hipStream_t stream,
                        bool csr = true);

}  // namespace sgnn
