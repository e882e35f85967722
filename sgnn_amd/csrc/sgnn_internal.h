// Host-side helpers shared by the sgnn translation units.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "../../include/sgnn.h"

namespace sgnn {

int set_error(int status, const char* msg);
int check_launch(const char* where);
struct RadiusSmallArgs;  // radius_small.h
// sgnn_encode_nodes, optionally with the small-graph radius search launched
// alongside (epd_fwd.hip).
int encode_nodes_impl(const float* pos_seq, int64_t n, int32_t T, int32_t dim, const int64_t* types,
                      const float* emb_w, int32_t emb_dim, int32_t use_emb, const float* vel_mean,
                      const float* vel_std, float wall_max, float wall_div, const sgnn_mlp* enc,
                      const sgnn_mlp* edge0, float* x0, float* u, float* v, const sgnn_saves* saves,
                      void* stream, const RadiusSmallArgs* fuse_radius, bool defer_csr = false,
                      bool* csr_pending = nullptr);
// sgnn_interaction_layer_encode; with lists (the radius search's padded lists
// whose CSR is still to be built), the layer builds and writes the CSR itself.
int interaction_layer_encode_impl(const float* pos, int64_t pos_stride, int32_t dim, float radius,
                                  const sgnn_mlp* enc_edge, float* e0t, const float* x_in, const float* u_in,
                                  const float* v_in, const int32_t* rowptr, const int32_t* send,
                                  const int32_t* recv, int64_t n, const sgnn_mlp* edge_fn, const sgnn_mlp* node_fn,
                                  const sgnn_mlp* next_edge, float* x_out, float* u_out, float* v_out, void* stream,
                                  const RadiusSmallArgs* lists);
int scan_exclusive(const int32_t* in, int32_t* out, int64_t len, int32_t* partials,
                   hipStream_t stream);

// Number of workgroups to launch for a grid-stride kernel: enough to fill
// the 256 CUs `per_cu` times, never more than the work needs.
inline unsigned persistent_grid(int64_t work_items, int64_t items_per_wg, int per_cu) {
  const int64_t need = (work_items + items_per_wg - 1) / items_per_wg;
  const int64_t cap = 256LL * per_cu;
  return (unsigned)std::max<int64_t>(1, std::min(need, cap));
}

}  // namespace sgnn
