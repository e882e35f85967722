// Inference-path node kernels on v_mfma_f32_16x16x4_f32 (fwd16.hip): shared
// between the translation units that dispatch to them.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace sgnn {

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

}  // namespace sgnn
