// One LearnedSimulator.predict_positions step in ONE launch (step16.hip):
// shared between the step driver (rollout.hip) and the kernel.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace sgnn {

constexpr int kStep16MaxL = 10;     // interaction layers carried in the kernel arguments
constexpr int kStep16MaxNT = 32;    // receivers per workgroup (one or two 16-item node sub-tiles)
constexpr int kStep16MaxCap = 64;   // neighbour cap (K, +1 without self loops)
constexpr int kStep16MaxGrid = 256; // one workgroup per CU, every workgroup resident
constexpr int kStep16MaxEx = 64;    // examples in the batch (their offsets are staged in LDS)
constexpr size_t kStep16MaxLds = 160 * 1024;
// Phase counters: one per workgroup, kStepFlagStride words apart (16 = 64 B: no two tiles' counters share
// a 128-B line half, so a publish does not disturb the polls of the neighbouring tiles' consumers), and
// the error word at the fixed index kStepFlagErr.  sgnn_step_ws.step_flags holds kStepFlagWords words.
#ifndef SGNN_FLAG_STRIDE
#define SGNN_FLAG_STRIDE 16
#endif
constexpr int kStepFlagStride = SGNN_FLAG_STRIDE;
constexpr int kStepFlagErr = kStep16MaxGrid * 16;
constexpr int kStepFlagWords = kStepFlagErr + 32;
static_assert(kStepFlagStride >= 1 && kStepFlagStride <= 16, "flag stride");
static_assert(kStepFlagWords == 4128 && kStepFlagErr == 4096, "include/sgnn.h SGNN_STEP_FLAG_WORDS / _ERR");

// Weights of one InteractionNetwork (nmlp_layers 1): edge_fn = Linear(3H, H) ->
// ReLU -> Linear(H, H) -> LayerNorm, node_fn = Linear(2H, H) -> ReLU ->
// Linear(H, H) -> LayerNorm (graph_network.py:139-148), torch [out][in].
struct Lay16 {
  const float *ew1, *eb1, *ew2, *eb2, *eg, *ebb;
  const float *nw1, *nb1, *nw2, *nb2, *ng, *nbb;
};

struct Step16Args {
  // inputs (learned_simulator.py:413-438): window [n][T][dim], examples
  const float* pos_seq;
  const float* pos_last;  // optional: the window's last frame as a contiguous [n][dim] copy (rollout steps > 0)
  int n, T, dim;
  const int64_t* ex_ptr;
  int n_ex;
  float radius, r2;
  int cap, loop;  // kept neighbours per receiver (K, or K + 1 then the self loop dropped)
  const int64_t* types;
  const float* emb_w;
  int emb_dim, use_emb, feat;
  const float *vel_mean, *vel_std, *acc_mean, *acc_std;
  float wall_max, wall_div;
  // weights
  int L;
  Lay16 lay[kStep16MaxL];
  const float *xn_w1, *xn_b1, *xn_w2, *xn_b2, *xn_g, *xn_bb;  // Encoder.node_fn
  const float *xe_w1, *xe_b1, *xe_w2, *xe_b2, *xe_g, *xe_bb;  // Encoder.edge_fn
  const float *d_w1, *d_b1, *d_w2, *d_b2;                    // Decoder
  // workspace
  float* uvl;          // [L][2][n][H]: layer k's node halves u_k, v_k (written once per step), then (e0_hbm)
                       // [grid][ecap_t][H + 4] e0 rows of each tile's edges
  int e0_hbm;          // e0 rows in HBM instead of LDS (tiles whose edges do not fit next to the weights)
  uint32_t* flags;     // [grid] per-tile phase counters + [grid] error word, zeroed per call
  uint32_t epoch0;     // phase counter base of this step within the call
  int nt;              // receivers per workgroup
  int ecap_t;          // edge rows per workgroup (nt * cap)
  int32_t *deg_out, *nbr_out;  // optional: the radius graph as padded lists [n], [n][cap]
  int poll_limit;      // polls per wait before the error word is set (< 0: test hook, set it at the first wait)
  int skew;            // test knob (sgnn_step_ws.step_skew): tile-dependent sleep before each publish, 0 = off
  int tile_order;      // 0: tile = workgroup index; 1: XCD-contiguous tiles (k_step16)
  // outputs
  float *pred, *next_pos, *window_out;
};

// LDS bytes the kernel needs for these arguments (0 when it does not apply).
size_t step16_lds_bytes(const Step16Args& a);
// Workgroups of this launch's kernel variant the device holds at once (CUs x occupancy per CU).
int64_t step16_resident(const Step16Args& a);
// Launches the kernel (a.nt / a.ecap_t set by the caller; grid = ceil(n / nt)).
int step16_launch(const Step16Args& a, hipStream_t s);

}  // namespace sgnn
