/*
 * sgnn.h — C-ABI of libsgnn_hip.so, the MI355X (gfx950) implementation of
 * sgnn's single-scale LearnedSimulator hot path.
 *
 * Every entry point takes plain device pointers, sizes and a hipStream_t
 * (passed as void* so the header needs no HIP include), launches
 * asynchronously on that stream, never synchronises, never allocates, and
 * returns an sgnn_status.  All buffers are owned by the caller.  Float data
 * is fp32; graph indices are int32 (N*K < 2^31).  Weights are passed in
 * torch.nn.Linear layout [out][in], row-major.
 *
 * Reference interfaces each group replaces are cited per function
 * (paths relative to the xrkong/sgnn repository root).
 */
#ifndef SGNN_H_
#define SGNN_H_

#include <stddef.h>
#include <stdint.h>

/* ABI revision of this header; sgnn_abi_version() returns the library's.  6: sgnn_step_ws starts with
 * struct_size (checked by every entry point that takes it), step_flags is SGNN_STEP_FLAG_WORDS long. */
#define SGNN_ABI_VERSION 6
/* Size of sgnn_step_ws.step_flags in 32-bit words, and the index of its error word (bindings that do not
 * include this header ask sgnn_step_flag_words()). */
#define SGNN_STEP_FLAG_WORDS 4128
#define SGNN_STEP_FLAG_ERR 4096

#ifdef __cplusplus
extern "C" {
#endif

typedef enum sgnn_status {
  SGNN_OK = 0,
  SGNN_ERR_INVALID = 1,     /* bad pointer / size / dimension */
  SGNN_ERR_UNSUPPORTED = 2, /* shape this build has no kernel for (e.g. hidden != 64/128) */
  SGNN_ERR_HIP = 3,         /* a HIP launch failed; see sgnn_last_error() */
  SGNN_ERR_STEP_TIMEOUT = 4 /* sgnn_step_check: a workgroup of the one-launch step gave up waiting for
                               its sender tiles; that call's outputs are invalid */
} sgnn_status;

/* One build_mlp(...) (+ optional LayerNorm) parameter set,
 * sgnn/single_scale/graph_network.py:7-45 and :86-96 / :139-148 (and the
 * multi-scale copy, multi_scale_gnn.py:26-64).  nlin = number of Linear layers
 * = nmlp_layers + 1, 2 or 3: w1 [hidden][in_dim]; nlin 2: w2 [out_dim][hidden];
 * nlin 3: w2 [hidden][hidden] (middle) and w3 [out_dim][hidden].  ln_g/ln_b
 * may be NULL (Decoder / prediction head have no LayerNorm). */
typedef struct sgnn_mlp {
  const float* w1; const float* b1;
  const float* w2; const float* b2;
  const float* ln_g; const float* ln_b;
  int32_t in_dim, hidden, out_dim, nlin;
  const float* w3; const float* b3;
} sgnn_mlp;

/* Optional activation saves of the training forward (NULL pointer / NULL
 * struct = inference).  Edge tensors use the 32-edge tiled layout of e0t;
 * node tensors are row-major [N][H]; rstd is one float per item.
 * sgnn_edge_layer / sgnn_edge_layer_bwd at hidden 128 with nlin 3: yhat and h2
 * may both be NULL (h and rstd given) -- the backward then forms them again
 * from h with the forward's own arithmetic (bit-identical), two [E][H] tensors
 * less per layer; its scratch (sgnn_bwd_scratch_floats) holds the recomputed h2. */
typedef struct sgnn_saves {
  float* h;     /* post-ReLU hidden of the MLP's first Linear */
  float* yhat;  /* LayerNorm-normalised (pre-affine) output */
  float* rstd;  /* LayerNorm 1/std per item */
  float* agg;   /* node layers: resolved aggregate [N][H] */
  float* hd;    /* node_layer_decode: decoder hidden [N][H] */
  float* h2;    /* nlin = 3: post-ReLU hidden of the middle Linear */
  float* hd2;   /* node_layer_decode, nlin = 3: decoder second hidden [N][H] */
} sgnn_saves;

const char* sgnn_version(void);
const char* sgnn_last_error(void);
int32_t sgnn_abi_version(void);     /* SGNN_ABI_VERSION the library was built with */
int32_t sgnn_step_flag_words(void); /* SGNN_STEP_FLAG_WORDS the library was built with */

/* ---------------------------------------------------------------------------
 * Neighbour search.  Replaces torch_geometric.nn.radius_graph(x, r, batch,
 * loop, max_num_neighbors) -> torch_cluster.radius, called at
 * sgnn/single_scale/learned_simulator.py:116-117 (batch ids :104-106).
 * Output is a receiver-sorted CSR: for receiver i (query), senders
 * send[rowptr[i] .. rowptr[i+1]) ascending, each with ||p_j - p_i||^2 < r^2
 * (fp32, dims summed in order), same example (ex_ptr), at most K kept
 * (first K ascending; K+1 then self dropped when loop == 0).  recv[e] = i.
 * The reference's edge_index = [send ; recv] (int64) in the same order.
 * Capacity: edge_cap >= n * (loop ? K : K + 1); K + !loop <= 64.
 * pos: particle i at pos + i * pos_stride (so the last frame of a [N,T,d]
 * sequence can be passed without a copy).  ex_ptr: device int64 [n_ex+1].
 * workspace: sgnn_radius_workspace_bytes(n, K, loop) bytes, 256-B aligned.
 * ------------------------------------------------------------------------- */
size_t sgnn_radius_workspace_bytes(int64_t n, int32_t K, int32_t loop);
int sgnn_radius_graph(const float* pos, int64_t pos_stride, int64_t n, int32_t dim,
                      const int64_t* ex_ptr, int32_t n_ex, float radius, int32_t K,
                      int32_t loop, void* workspace, int32_t* rowptr, int32_t* send,
                      int32_t* recv, int64_t edge_cap, void* stream);

/* Static graphs (multi-scale g2m/m2m/m2g edges, sgnn/multi_scale/
 * multi_scale_graph.py:193-281, consumed by multi_scale_gnn.py:277-325):
 * COO edge_index rows (src = edge_index[0] = sender, dst = edge_index[1] =
 * receiver, int64, values in [0, n)) -> receiver-sorted CSR, stable (edges of
 * one receiver keep their original order = PyG's scatter-add order).
 * rowptr [n+1], send/recv [E]. */
size_t sgnn_coo_workspace_bytes(int64_t n, int64_t E);
int sgnn_coo_to_csr(const int64_t* src, const int64_t* dst, int64_t E, int64_t n, void* workspace,
                    int32_t* rowptr, int32_t* send, int32_t* recv, int32_t* perm, void* stream);
/* perm (optional, [E]): CSR position -> original COO edge id. */

/* EncodeProcessDecode.forward(x, edge_index, edge_features) on explicit
 * features (graph_network.py:388-406; MultiScaleGNN.forward
 * multi_scale_gnn.py:262-326): the encoders read given rows instead of
 * deriving features from positions.  x: [n][feat] row-major; e: [E][fe] in the
 * COO order of edge_index, read through perm from sgnn_coo_to_csr.  The rest
 * of the chain is unchanged (sgnn_edge_layer / sgnn_node_layer /
 * sgnn_node_layer_decode with pos_seq = NULL: decoder output only). */
int sgnn_encode_node_features(const float* x, int64_t n, int32_t feat, const sgnn_mlp* enc,
                              const sgnn_mlp* edge0, float* x0, float* u, float* v, void* stream);
int sgnn_encode_edge_features(const float* e, int32_t fe, const int32_t* perm,
                              const int32_t* rowptr, int64_t n, int64_t edge_cap,
                              const sgnn_mlp* enc, float* e0t, void* stream);

/* ---------------------------------------------------------------------------
 * Feature construction on explicit tensors (generic.hip): the node and edge
 * features of _encoder_preprocessor (learned_simulator.py:231-316) for the
 * width-generic path (the fused encoders compute them on the fly).
 * ------------------------------------------------------------------------- */
/* Node features [n][(T-1)*dim + 1 (+ emb_dim)] (learned_simulator.py:256-290; wall as sgnn_encode_nodes). */
int sgnn_node_features(const float* pos_seq, int64_t n, int32_t T, int32_t dim, const int64_t* types,
                       const float* emb_w, int32_t emb_dim, int32_t use_emb, const float* vel_mean,
                       const float* vel_std, float wall_max, float wall_div, float* out, void* stream);
/* Edge features [E][dim+1] in CSR order (learned_simulator.py:299-312), E = rowptr[n]. */
int sgnn_edge_features(const float* pos, int64_t pos_stride, int32_t dim, float radius,
                       const int32_t* rowptr, const int32_t* send, const int32_t* recv, int64_t n,
                       int64_t edge_cap, float* out, void* stream);

/* ---------------------------------------------------------------------------
 * Encoder, node side: node features of LearnedSimulator._encoder_preprocessor
 * (learned_simulator.py:256-290: normalised velocity history, wall distance
 * clamp(x+2, 0, wall_max) / wall_div — single scale: (R, 1), learned_simulator.py:
 * 282-284; multi scale: (R_g, R_g), multi_scale_simulator.py:190-193 —,
 * optional type embedding) fused with Encoder.node_fn
 * (graph_network.py:86-90, :111) and with the receiver/sender projections of
 * the first InteractionNetwork's edge MLP:
 *   u = x0 W1[:, 0:H]^T + b1,  v = x0 W1[:, H:2H]^T   (W1 of edge0)
 * pos_seq: [n][T][dim].  types/emb_w only read when use_emb != 0.
 * ------------------------------------------------------------------------- */
int sgnn_encode_nodes(const float* pos_seq, int64_t n, int32_t T, int32_t dim,
                      const int64_t* types, const float* emb_w, int32_t emb_dim,
                      int32_t use_emb, const float* vel_mean, const float* vel_std,
                      float wall_max, float wall_div, const sgnn_mlp* enc,
                      const sgnn_mlp* edge0, float* x0, float* u, float* v,
                      const sgnn_saves* saves, void* stream);

/* Encoder, edge side: edge features (learned_simulator.py:299-312:
 * (p_s - p_r)/R and its norm) fused with Encoder.edge_fn (graph_network.py:
 * 92-96).  Output e0 in the tiled layout (sgnn_edge_tile_floats(H) floats per
 * 32-edge tile) that sgnn_edge_layer reads. */
int64_t sgnn_edge_latent_floats(int64_t edge_cap, int32_t hidden);
int sgnn_encode_edges(const float* pos, int64_t pos_stride, int32_t dim, float radius,
                      const int32_t* rowptr, const int32_t* send, const int32_t* recv,
                      int64_t n, int64_t edge_cap, const sgnn_mlp* enc, float* e0t,
                      const sgnn_saves* saves, void* stream);

/* ---------------------------------------------------------------------------
 * Processor, edge half of one InteractionNetwork (graph_network.py:150-199):
 *   m_e  = LN(W2 relu(u[recv] + v[send] + e_scale * W1[:, 2H:3H] e0_e) + b2)
 *   agg_i = sum over edges e with recv == i of m_e   (aggr='add', :136)
 * e_scale = 2^k reproduces the edge-latent doubling (update returns the input
 * edge features, :176/:222); it is applied to the staged W1e (exact for a
 * power of two, the only values the reference produces).  agg rows whose edges straddle a 32-edge tile
 * are left in cin/cout ([ceil(edge_cap/32)][H] each); sgnn_node_layer*
 * resolves them (deterministic, no atomics).
 * ------------------------------------------------------------------------- */
int sgnn_edge_layer(const float* u, const float* v, const float* e0t, float e_scale,
                    const int32_t* rowptr, const int32_t* send, const int32_t* recv,
                    int64_t n, int64_t edge_cap, const sgnn_mlp* edge_fn, float* agg,
                    float* cin, float* cout, const sgnn_saves* saves, void* stream);

/* Processor, node half (graph_network.py:201-222 and the residual :176):
 *   x_out = x_in + LN(W2 relu(W1 [agg, x_in] + b1) + b2)
 * fused with the next layer's projections (u, v as sgnn_encode_nodes). */
int sgnn_node_layer(const float* x_in, const float* agg, const float* cin, const float* cout,
                    const int32_t* rowptr, int64_t n, const sgnn_mlp* node_fn,
                    const sgnn_mlp* next_edge, float* x_out, float* u, float* v,
                    const sgnn_saves* saves, void* stream);

/* Last processor node half fused with the Decoder (graph_network.py:321-333,
 * no LayerNorm) and LearnedSimulator._decoder_postprocessor
 * (learned_simulator.py:381-411, Euler with dt = 1):
 *   pred = decoder(x_out) [n][dim+1];  a = pred[:, :dim] * acc_std + acc_mean
 *   next_pos = p_T + ((p_T - p_{T-1}) + a)          (pos_seq [n][T][dim])
 * x_out may be NULL (inference).  If window_out is not NULL it receives the
 * next input window of the autoregressive rollout, cat([pos_seq[:, 1:],
 * next_pos[:, None]], 1) (sgnn/single_scale/evaluate.py:136-139). */
int sgnn_node_layer_decode(const float* x_in, const float* agg, const float* cin,
                           const float* cout, const int32_t* rowptr, int64_t n,
                           const sgnn_mlp* node_fn, const sgnn_mlp* decoder,
                           const float* pos_seq, int32_t T, int32_t dim,
                           const float* acc_mean, const float* acc_std, float* x_out,
                           float* pred, float* next_pos, float* window_out,
                           const sgnn_saves* saves, void* stream);

/* One whole InteractionNetwork.forward (graph_network.py:150-222, inference,
 * hidden 64) in ONE launch: edge half + receiver sums + node half as above,
 * without the agg/cin/cout round trip -- each workgroup owns a run of
 * consecutive receivers and all of their (contiguous) CSR edges.  u_in/v_in
 * are this layer's node halves, u_out/v_out receive the next layer's (they
 * must be different buffers: other workgroups still read u_in/v_in).
 * Replaces the pair sgnn_edge_layer + sgnn_node_layer(_decode). */
int sgnn_interaction_layer(const float* x_in, const float* u_in, const float* v_in,
                           const float* e0t, float e_scale, const int32_t* rowptr,
                           const int32_t* send, const int32_t* recv, int64_t n,
                           const sgnn_mlp* edge_fn, const sgnn_mlp* node_fn,
                           const sgnn_mlp* next_edge, float* x_out, float* u_out, float* v_out,
                           void* stream);
int sgnn_interaction_layer_decode(const float* x_in, const float* u_in, const float* v_in,
                                  const float* e0t, float e_scale, const int32_t* rowptr,
                                  const int32_t* send, const int32_t* recv, int64_t n,
                                  const sgnn_mlp* edge_fn, const sgnn_mlp* node_fn,
                                  const sgnn_mlp* decoder, const float* pos_seq, int32_t T,
                                  int32_t dim, const float* acc_mean, const float* acc_std,
                                  float* pred, float* next_pos, float* window_out, void* stream);

/* sgnn_interaction_layer for the FIRST layer with Encoder.edge_fn folded in
 * (graph_network.py:92-96, learned_simulator.py:299-312; nmlp_layers 1): e0 of
 * every edge is computed from the positions (most recent frame at pos + i *
 * pos_stride) inside the layer, used at once, and written to e0t for the
 * later layers -- replaces sgnn_encode_edges + sgnn_interaction_layer(k = 0). */
int sgnn_interaction_layer_encode(const float* pos, int64_t pos_stride, int32_t dim, float radius,
                                  const sgnn_mlp* enc_edge, float* e0t, const float* x_in,
                                  const float* u_in, const float* v_in, const int32_t* rowptr,
                                  const int32_t* send, const int32_t* recv, int64_t n,
                                  const sgnn_mlp* edge_fn, const sgnn_mlp* node_fn,
                                  const sgnn_mlp* next_edge, float* x_out, float* u_out, float* v_out,
                                  void* stream);

/* ---------------------------------------------------------------------------
 * Whole-step drivers.  One call = one LearnedSimulator.predict_positions
 * (learned_simulator.py:413-438: radius graph, encoders, L interaction
 * layers, decoder, Euler) or a whole autoregressive rollout (evaluate.py:
 * 117-145: the window shift is fused into the decoder kernel), issued from C
 * so the host cost per kernel is one hipLaunchKernel. */
typedef struct sgnn_epd {
  int32_t nlayers;
  const sgnn_mlp* enc_node;
  const sgnn_mlp* enc_edge;
  const sgnn_mlp* edge; /* [nlayers] InteractionNetwork edge_fn */
  const sgnn_mlp* node; /* [nlayers] InteractionNetwork node_fn */
  const sgnn_mlp* dec;
} sgnn_epd;

typedef struct sgnn_step_in {
  int64_t n;
  int32_t T, dim;
  const int64_t* ex_ptr; /* [n_ex+1] example offsets (nparticles_per_example) */
  int32_t n_ex;
  float radius;
  int32_t K; /* max_num_neighbors (20) */
  const int64_t* types;
  const float* emb_w;
  int32_t emb_dim, use_emb;
  const float *vel_mean, *vel_std, *acc_mean, *acc_std;
  float wall_max, wall_div; /* clamp(x + 2, 0, wall_max) / wall_div */
} sgnn_step_in;

typedef struct sgnn_step_ws { /* device buffers of one (n, T, dim, H, K) shape */
  int64_t struct_size; /* = sizeof(sgnn_step_ws); any other value: SGNN_ERR_INVALID (a caller built against
                          another revision of this header) */
  void* radius_ws;
  int32_t *rowptr, *send, *recv;
  int64_t edge_cap;
  float *e0t, *x_a, *x_b, *u, *v, *agg, *cin, *cout;
  float *u2, *v2; /* [n][H] second node-half buffers: with both set, H = 64 and n <= 8192 each
                     layer runs as ONE sgnn_interaction_layer launch (u/v ping-pong); else two */
  /* Optional, the one-launch step (hidden 64, nmlp_layers 1, n <= 8192, 2 <= nlayers <= 10):
   * with all three set, a whole step is ONE kernel launch (radius graph, encoders, every layer,
   * decoder, integrator; sgnn_step_path() says whether it applies).  The radius graph then stays
   * in the kernel's LDS: rowptr/send/recv are not written, step_deg receives each receiver's
   * neighbour count. */
  float* uvl;           /* nlayers*2*n*H + (n+32)*K*(H+4) floats: every layer's node halves u_k, v_k
                           ([nlayers][2][n][H]), then room for the edge latents of tiles too large for
                           the kernel's LDS */
  uint32_t* step_flags; /* [SGNN_STEP_FLAG_WORDS] per-workgroup phase counters (64 B apart) + error word
                           at [SGNN_STEP_FLAG_ERR] (zeroed per call) */
  int32_t* step_deg;    /* [n] neighbours kept per receiver */
  int32_t step_poll_limit; /* 0: default (~1 s of polling per wait before the error word is set);
                              < 0: test hook, every tile records a timeout at its first wait */
  int32_t step_skew;       /* test knob, 0 = off: before each phase publish, workgroup t sleeps a
                              tile- and phase-dependent 0..7 x step_skew rounds of ~0.4 us, so tiles
                              hand off under uneven load (results must not change) */
} sgnn_step_ws;

int sgnn_predict_positions(const sgnn_epd* model, const sgnn_step_in* in, const float* pos_seq,
                           const sgnn_step_ws* ws, float* pred, float* next_pos, float* window_out,
                           void* stream);
/* 1 when sgnn_predict_positions / sgnn_rollout run these arguments as the one-launch step, 0 when
 * they run the per-kernel sequence; (*nt, *grid) = receivers per workgroup and workgroups. */
int sgnn_step_path(const sgnn_epd* model, const sgnn_step_in* in, const sgnn_step_ws* ws, int32_t* nt,
                   int32_t* grid);
/* Co-residency.  The one-launch step hands data between its workgroups through per-tile counters, so
 * every workgroup of a launch must be resident at once (grid <= CUs x the kernel's occupancy, checked
 * per call).  Within this process a call takes the one-launch path only when no one-launch step of an
 * earlier call on ANOTHER stream of the device may still be running (else it runs the per-kernel
 * sequence: same results).  Across processes nothing can be checked: two one-launch steps sharing the
 * device's CUs can each hold CUs the other's waiting tiles need; their bounded waits then expire and
 * the error word is set.  sgnn_step_check reads that word once the call's work is done (it
 * synchronises `stream`, the one entry point that does) and returns SGNN_ERR_STEP_TIMEOUT when set --
 * the caller must treat that call's outputs as invalid.  The Python wrappers call it after every
 * predict_positions / rollout (learned_simulator.py:413-438, evaluate.py:117-145 sync on .cpu() too).
 * Processes that share one device (e.g. data-parallel ranks on one GPU) should opt out: a workspace
 * without the one-launch buffers (uvl / step_flags / step_deg NULL; in Python StepWorkspace(one_launch=
 * False), or SGNN_ONE_LAUNCH=0 in the environment) always runs the per-kernel sequence. */
int sgnn_step_check(const sgnn_step_ws* ws, void* stream);
/* Steps alternate win_a -> win_b -> win_a ...; step k writes out_pred[k][n][dim+1]
 * (normalised acceleration + strain) and out_pos[k][n][dim]. */
int sgnn_rollout(const sgnn_epd* model, const sgnn_step_in* in, float* win_a, float* win_b,
                 const sgnn_step_ws* ws, int32_t nsteps, float* out_pos, float* out_pred,
                 void* stream);
/* Teacher-forced ("one_step") rollout, evaluate.py:136-145 with inference_mode == "one_step": step k
 * predicts from the current window exactly as sgnn_rollout does, then the next window is
 * cat([window[:, 1:], gt_k]) -- the ground-truth position of step k, not the prediction (:140-143).
 * gt_k[i][c] = gt[k * gt_ld_t + i * gt_ld_n + c] (the reference's position[:, T:] is [n][steps][dim]:
 * gt_ld_n = steps * dim, gt_ld_t = dim).  Outputs as sgnn_rollout. */
int sgnn_rollout_one_step(const sgnn_epd* model, const sgnn_step_in* in, float* win_a, float* win_b,
                          const sgnn_step_ws* ws, int32_t nsteps, const float* gt, int64_t gt_ld_n,
                          int64_t gt_ld_t, float* out_pos, float* out_pred, void* stream);

/* ---------------------------------------------------------------------------
 * Training backward: reverse of predict_accelerations (learned_simulator.py:
 * 440-491) + the loss of train.py:257-268, i.e. what loss.backward() does
 * through PyG/torch autograd.  Call order per step (L layers):
 *   sgnn_transpose_csr (sender-sorted CSR for dV; once per graph)
 *   sgnn_decoder_loss_bwd                 -> g = dL/dx_L
 *   for k = L-1 .. 0:
 *     sgnn_node_layer_bwd(k, g)           -> dagg, dx'
 *     sgnn_edge_layer_bwd(k, dagg)        -> dU (+carries), dh rows, dE0
 *     sgnn_uv_bwd(k, dx', dU, dh)         -> g = dL/dx_k
 *   sgnn_encode_nodes_bwd(g), sgnn_encode_edges_bwd(dE0)
 *   sgnn_reduce_slabs                     -> parameter gradients
 * Each *_bwd launches `nslab` persistent workgroups and writes one partial
 * slab of sgnn_bwd_slab_floats(kind, H, feat, nlin) floats per workgroup.
 * Slab layouts (row-major, W = 4 waves per workgroup, vectors as W partial
 * rows; Wl = last Linear, Wm = middle Linear (nlin = 3 only, appended), W1 =
 * first):
 *   EDGE    : dWl[H][H] | dW1e[H][H] (x 2^k in the reduce) | dWm |
 *             dbl, dgamma, dbeta [W][H] | dbm
 *   NODE    : dWl[H][H] | dW1[H][2H] | dWm | db1, dbl, dgamma, dbeta [W][H] | dbm
 *   UV      : dW1[:, 0:2H] as [H][2H] | db1 [W][H]
 *   DECODER : dWl[32][H] (rows > dim zero) | dW1[H][H] | dWm | dbl [W][32] |
 *             db1 [W][H] | loss [W][8] = (total, x, y, z, strain) sums of
 *             squared errors | dbm [W][H]
 *   ENC_NODE: dWl[H][H] | dW1[H][32*ceil(F/32)] | dWm | db1, dbl, dgamma, dbeta [W][H] | dbm |
 *             G[32][H] (per-particle-type sums of dh; zero without embeddings)
 *   ENC_EDGE: dWl[H][H] | dW1[H][32] | dWm | db1, dbl, dgamma, dbeta [W][H] | dbm
 * Hidden 64 or 128, nlin 2 or 3 (nmlp_layers 1 or 2).  Saved activations come
 * through struct sgnn_saves as the training forward wrote them.
 * ------------------------------------------------------------------------- */
enum { SGNN_SLAB_EDGE = 0, SGNN_SLAB_NODE = 1, SGNN_SLAB_UV = 2, SGNN_SLAB_DECODER = 3,
       SGNN_SLAB_ENC_NODE = 4, SGNN_SLAB_ENC_EDGE = 5 };
int64_t sgnn_bwd_slab_floats(int32_t kind, int32_t hidden, int32_t feat, int32_t nlin);
/* Hidden 128 runs each of the EDGE / NODE / UV / ENC_EDGE backwards as a
 * per-item kernel that writes pre-activation gradients to `scratch` plus
 * split-K MFMA GEMMs for the weight gradients (same slab layouts).  scratch
 * must hold sgnn_bwd_scratch_floats(kind, hidden, nitems, nlin) floats, nitems
 * = edge_cap (edge kinds) or n (node kinds); 0 (scratch unused) for hidden 64.
 * One scratch buffer may serve every call on the same stream. */
int64_t sgnn_bwd_scratch_floats(int32_t kind, int32_t hidden, int64_t nitems, int32_t nlin);

/* out[r*dst_ld + c] (+)= scale * sum_{g<nslab} sum_{q<nrep}
 *                         src[g*slab_stride + offset + q*rep_stride + r*src_ld + c] */
typedef struct sgnn_reduce_desc {
  const float* src; float* dst;
  int64_t slab_stride, offset, rep_stride;
  int32_t nslab, nrep, src_ld, nrows, ncols, dst_ld, accumulate;
  float scale;
} sgnn_reduce_desc;
/* block_start[d] = sum_{d' < d} ceil(nrows*ncols / 32) (device int32 [ndesc]);
 * nblocks = the total.  Deterministic (fixed summation order). */
int sgnn_reduce_slabs(const sgnn_reduce_desc* descs_dev, const int32_t* block_start,
                      int32_t ndesc, int32_t nblocks, void* stream);

size_t sgnn_transpose_workspace_bytes(int64_t n, int64_t edge_cap);
int sgnn_transpose_csr(const int32_t* rowptr, const int32_t* send, int64_t n, int64_t edge_cap,
                       void* workspace, int32_t* tptr, int32_t* tperm, void* stream);

/* dpred != NULL: use it as dL/dpred [n][dim+1] (autograd path) instead of the
 * fused loss gradient 2*w*(pred - target)*inv_count of train.py:257-268. */
/* saves: hd (+ hd2 for nlin 3) as node_layer_decode wrote them. */
int sgnn_decoder_loss_bwd(const float* pred, const float* pos_seq, const float* next_pos,
                          const float* noise, const float* next_strain, const float* acc_mean,
                          const float* acc_std, int64_t n, int32_t T, int32_t dim, float w_pos,
                          float w_strain, float inv_count, const float* dpred,
                          const sgnn_saves* saves, const float* x_last, const sgnn_mlp* decoder,
                          float* g, float* slab, int32_t nslab, void* stream);
/* saves: yhat, rstd, h, agg (+ h2) as node_layer wrote them. */
int sgnn_node_layer_bwd(const float* g, int64_t n, const sgnn_saves* saves, const float* x_in,
                        const sgnn_mlp* node_fn, float* dagg, float* dxp, float* slab,
                        int32_t nslab, float* scratch, void* stream);
/* saves: h, yhat, rstd (+ h2) as edge_layer wrote them.  With de0t: this
 * layer's dE0 term is written (de0_accumulate bit 0: added) and its dW1e
 * formed in-layer.  de0t = NULL (H = 64): both are left to
 * sgnn_edge_latent_grad, except that de0_accumulate bit 1 (value 2) at
 * nmlp_layers 1 forms this layer's dW1e in the kernel (slab dW1e block), so
 * only the dE0 pass remains. */
int sgnn_edge_layer_bwd(const float* dagg, const int32_t* rowptr, const int32_t* send,
                        const int32_t* recv, int64_t n, const sgnn_saves* saves, const float* e0t,
                        float e_scale, const sgnn_mlp* edge_fn, float* du, float* cin,
                        float* cout, float* dh_rows, float* de0t, int32_t de0_accumulate,
                        float* slab, int32_t nslab, float* scratch, int64_t edge_cap,
                        void* stream);
/* dE0 = sum_k scales[k] W1e_k^T dh_k (edge_fns[k].w1 columns 2H..3H) over
 * nlayers layers that share one encoded edge latent, from each layer's dh
 * rows [E][H] (the dh_rows output of sgnn_edge_layer_bwd, one buffer per
 * layer), plus each layer's dW1e = sum_e dh_k (x) e0 into the dW1e block of
 * its SLAB_EDGE slabs (slabs[k], nslab workgroups, the same arena
 * sgnn_edge_layer_bwd wrote; the 2^k factor is applied by the slab
 * reduction as for the in-layer product).  With it, sgnn_edge_layer_bwd is
 * called with de0t = NULL (H = 64, nlayers <= 9) and skips both products.
 * Writes de0t in the tiled layout of e0.  Either half may be skipped:
 * slabs = NULL forms dE0 only; de0t = NULL forms the dW1e blocks only (one
 * launch per layer, so a layer's dW1e can run on a second stream as soon as
 * its dh rows exist). */
int sgnn_edge_latent_grad(const float* const* dh_rows, const sgnn_mlp* edge_fns,
                          const float* scales, int32_t nlayers, const int32_t* rowptr, int64_t n,
                          int64_t edge_cap, const float* e0t, float* de0t, float* const* slabs,
                          int32_t nslab, void* stream);
int sgnn_uv_bwd(const float* dxp, const float* du, const float* cin, const float* cout,
                const int32_t* rowptr, const float* dh_rows, const int32_t* tptr,
                const int32_t* tperm, const float* x_in, int64_t n, const sgnn_mlp* edge_fn,
                float* g, float* slab, int32_t nslab, float* scratch, void* stream);
/* Wall feature as sgnn_encode_nodes: clamp(x + 2, 0, wall_max) / wall_div.
 * saves: h, yhat, rstd (+ h2). */
int sgnn_encode_nodes_bwd(const float* g, const float* pos_seq, int64_t n, int32_t T,
                          int32_t dim, const int64_t* types, const float* emb_w, int32_t emb_dim,
                          int32_t ntypes, int32_t use_emb, const float* vel_mean,
                          const float* vel_std, float wall_max, float wall_div,
                          const sgnn_saves* saves, const sgnn_mlp* enc, float* slab,
                          int32_t nslab, void* stream);
/* The same for more than 32 particle types (up to 256; ntypes x hidden <=
 * 40960): the per-type sums G[ntypes][H] of the encoder's first-layer
 * gradient are not kept in the slab but formed from per-node dh rows by a
 * deterministic two-pass type sum (fixed node order per 256-node block, then
 * fixed block order) and written to G; the slab's G block is left unused.
 * workspace: sgnn_type_sums_workspace_bytes(n, hidden, ntypes) bytes.
 * Replaces the same autograd path as sgnn_encode_nodes_bwd with an
 * nn.Embedding(ntypes, emb) of any size (learned_simulator.py:51-52). */
int sgnn_encode_nodes_bwd_typed(const float* g, const float* pos_seq, int64_t n, int32_t T,
                                int32_t dim, const int64_t* types, const float* emb_w, int32_t emb_dim,
                                int32_t ntypes, const float* vel_mean, const float* vel_std,
                                float wall_max, float wall_div, const sgnn_saves* saves,
                                const sgnn_mlp* enc, float* slab, int32_t nslab, float* G,
                                void* workspace, void* stream);
size_t sgnn_type_sums_workspace_bytes(int64_t n, int32_t hidden, int32_t ntypes);
/* Particle-type embedding gradient (learned_simulator.py:287-290 under
 * autograd): the ENC_NODE slab's trailing G[32][H] block (per-type sums of the
 * encoder's first-layer gradient, reduced) times the embedding columns of
 * W1: dEmb[t][c] (+)= sum_u G[t][u] W1[u][col0 + c]. */
int sgnn_embedding_grad(const float* G, int32_t ntypes, int32_t hidden, const float* w1,
                        int32_t w1_ld, int32_t col0, int32_t emb_dim, float* demb,
                        int32_t accumulate, void* stream);
/* saves: yhat, rstd (+ h2); the first hidden is recomputed. */
int sgnn_encode_edges_bwd(const float* de0t, const float* pos, int64_t pos_stride, int32_t dim,
                          float radius, const int32_t* rowptr, const int32_t* send,
                          const int32_t* recv, int64_t n, const sgnn_saves* saves,
                          const sgnn_mlp* enc, float* slab, int32_t nslab, float* scratch,
                          int64_t edge_cap, void* stream);

/* Random-walk training noise (noise_utils.py:4-39) and the noisy window
 * (learned_simulator.py:467) in one pass: velocity increments
 * N(0, (std_last/sqrt(T-1))^2) from a Philox4x32-10 stream keyed by seed
 * and counted by the global particle index (offset + i: `offset` = index of
 * this call's first particle in the data-parallel batch), cumsum twice, noise[n][T][dim] with noise[:,0] = 0,
 * noisy = pos_seq + noise.  The distribution of the reference's CPU-generator
 * draw, not its bit stream. */
int sgnn_random_walk_noise(const float* pos_seq, int64_t n, int32_t T, int32_t dim,
                           float noise_std_last_step, uint64_t seed, uint64_t offset, float* noise,
                           float* noisy, void* stream);

/* Fused Adam over a flat fp32 buffer; same update as torch.optim.Adam
 * (amsgrad=False, weight_decay=0) used by train.py:199,271-273. step >= 1. */
int sgnn_adam_step(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, int64_t n,
                   float lr, float beta1, float beta2, float eps, int64_t step, void* stream);

/* ---------------------------------------------------------------------------
 * Width-generic differentiable building blocks (autograd.hip).  The
 * reference's modules are differentiable at any widths and depths
 * (build_mlp, graph_network.py:7-45; Encoder / InteractionNetwork / Processor /
 * Decoder forwards :98, :150, :276, :324; G2M / M2M / M2G blocks,
 * multi_scale_gnn.py:84, :132, :179): these are the forward and backward
 * pieces the Python autograd Functions (sgnn_amd/autograd.py) compose for
 * every shape the fused MFMA kernels are not built for.  Everything is
 * deterministic: no float atomics, fixed summation orders.
 * ------------------------------------------------------------------------- */
/* C[M][N] (ldc) = op(A) op(B) (+ C when accumulate) (+ bias[n]) (then ReLU when relu), fp32 on the
 * MFMA cores (v_mfma_f32_32x32x2_f32, exact fp32 products).  op(A) = A stored [M][K] (lda), or A^T with
 * A stored [K][M] (trans_a); op(B) = B stored [K][N] (ldb), or B^T with B stored [N][K] (trans_b).
 * Long K is split over workgroups whose partial tiles are summed in split order in `workspace`
 * (sgnn_gemm_workspace_bytes(M, N, K) bytes; the split depends on the shape only). */
size_t sgnn_gemm_workspace_bytes(int64_t M, int64_t N, int64_t K);
int sgnn_gemm(int32_t trans_a, int32_t trans_b, int64_t M, int64_t N, int64_t K, const float* A, int64_t lda,
              const float* B, int64_t ldb, const float* bias, int32_t relu, float* C, int64_t ldc,
              int32_t accumulate, void* workspace, size_t workspace_bytes, void* stream);
/* LayerNorm over rows of `width` (torch: biased variance, eps 1e-5, affine), out = LN(x) (+ residual);
 * yhat [n][width] / rstd [n] receive the normalised rows and 1/std when not NULL. */
int sgnn_layernorm(const float* x, int64_t n, int32_t width, const float* gamma, const float* beta,
                   const float* residual, float* out, float* yhat, float* rstd, void* stream);
/* dx = rstd (g - mean(g) - yhat mean(g yhat)), g = dout * gamma (per row). */
int sgnn_layernorm_bwd(const float* dout, const float* yhat, const float* rstd, const float* gamma, int64_t n,
                       int32_t width, float* dx, void* stream);
/* out[c] (+)= sum_r x[r][c] (* mul[r][c]) over the n rows, in row order per 256-row block, blocks in order
 * (workspace: sgnn_colsum_workspace_bytes(n, width)). */
size_t sgnn_colsum_workspace_bytes(int64_t n, int32_t width);
int sgnn_colsum(const float* x, int64_t ldx, const float* mul, int64_t ldm, int64_t n, int32_t width, float* out,
                int32_t accumulate, void* workspace, size_t workspace_bytes, void* stream);
/* dy[r][c] = y[r][c] > 0 ? dy[r][c] : 0 (ReLU backward on the saved post-activation rows). */
int sgnn_relu_bwd(float* dy, int64_t ldd, const float* y, int64_t ldy, int64_t n, int32_t width, void* stream);
/* out[r][0:width] (ld_out) = scale * src[index ? index[r] : r][0:width] (ld_src): one column block of a
 * concatenation of gathered rows (cat([x_i, x_j, e]), graph_network.py:197). */
int sgnn_gather_rows(const float* src, int64_t ld_src, int32_t width, const int32_t* index, int64_t nrows,
                     float scale, float* out, int64_t ld_out, void* stream);
/* out[i][0:width] (+)= scale * sum over p in [rowptr[i], rowptr[i+1]) of src[perm ? perm[p] : p][0:width], in
 * CSR order: the receiver sums of aggr='add' (graph_network.py:136) and the backward of a row gather. */
int sgnn_segment_sum_cols(const float* src, int64_t ld_src, int32_t width, const int32_t* rowptr,
                          const int32_t* perm, int64_t n, float scale, float* out, int64_t ld_out,
                          int32_t accumulate, void* stream);
/* Explicit edge latent rows e [E][width] (COO order; ld) -> the tiled e0t layout sgnn_edge_layer reads
 * (width a multiple of 32; CSR position p reads row perm[p] of sgnn_coo_to_csr; tiles padded with zeros up
 * to edge_cap).  InteractionNetwork.forward(x, edge_index, e) on the fused kernels (graph_network.py:150). */
int sgnn_edge_rows_to_tiles(const float* e, int64_t ld, int32_t width, const int32_t* perm, const int32_t* rowptr,
                            int64_t n, int64_t edge_cap, float* e0t, void* stream);
/* The inverse, for the module-level block backward (InteractionNetwork.forward under autograd,
 * graph_network.py:150): out[perm[p]][0:width] (+ when accumulate) = scale * tile position p of e0t for
 * p < num_edges (= rowptr[n]; the edge-latent gradient dE0 back in the caller's COO row order). */
int sgnn_edge_tiles_to_rows(const float* e0t, int32_t width, const int32_t* perm, const int32_t* rowptr, int64_t n,
                            int64_t num_edges, float scale, float* out, int64_t ld, int32_t accumulate, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* SGNN_H_ */
