// Host-side step / rollout drivers: one C-ABI call issues a whole
// LearnedSimulator.predict_positions (learned_simulator.py:413-438) or a whole
// autoregressive rollout (evaluate.py:117-145), so the per-kernel cost on the
// host is a hipLaunchKernel (~µs) instead of a Python ctypes round trip.
#include "../../include/sgnn.h"
#include "sgnn_internal.h"
#include "radius_small.h"
#include "step16.h"

#include <stdio.h>

#include <mutex>

namespace {

// An MLP of nmlp_layers 1 with these widths (and a LayerNorm when `ln`).
bool mlp16(const sgnn_mlp* m, int in_dim, int out_dim, bool ln) {
  return m && m->nlin == 2 && m->w1 && m->b1 && m->w2 && m->b2 && m->in_dim == in_dim && m->hidden == 64 &&
         m->out_dim == out_dim && (!ln || (m->ln_g && m->ln_b));
}

int device_cus() {
  static int cus = 0;
  if (cus == 0) {
    int dev = 0;
    hipDeviceProp_t p{};
    cus = (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&p, dev) == hipSuccess) ? p.multiProcessorCount
                                                                                              : -1;
  }
  return cus;
}

// The one-launch step's arguments when it applies to this call (step16.hip):
// hidden 64, nmlp_layers 1 everywhere, 2..10 layers, n <= 8192 particles, a
// grid of <= one workgroup per CU, and the kernel's LDS under 160 KB.
// a workspace struct from a caller built against this header revision (include/sgnn.h struct_size)
bool ws_ok(const sgnn_step_ws* ws) { return ws && ws->struct_size == (int64_t)sizeof(sgnn_step_ws); }

bool step16_plan(const sgnn_epd* m, const sgnn_step_in* in, const float* pos_seq, const sgnn_step_ws* ws,
                 float* pred, float* next_pos, float* window_out, sgnn::Step16Args* out) {
  using namespace sgnn;
  if (!m || !in || !ws_ok(ws) || !ws->uvl || !ws->step_flags || !ws->step_deg) return false;
  const int L = m->nlayers;
  const int64_t n = in->n;
  const int d = in->dim, T = in->T;
  const int cap = in->K;  // predict_positions keeps self loops (learned_simulator.py:75,117)
  if (L < 2 || L > kStep16MaxL || n < 1 || n > kStep16MaxGrid * kStep16MaxNT || d < 1 || d > 3 || T < 2 ||
      cap < 1 || cap > kStep16MaxCap || in->n_ex < 1 || in->n_ex > kStep16MaxEx || !in->ex_ptr ||
      !(in->radius > 0.0f))
    return false;
  const int feat = (T - 1) * d + 1 + (in->use_emb ? in->emb_dim : 0);
  if (feat > 48 || !mlp16(m->enc_node, feat, 64, true) || !mlp16(m->enc_edge, d + 1, 64, true) ||
      !mlp16(m->dec, 64, d + 1, false))
    return false;
  for (int k = 0; k < L; ++k)
    if (!mlp16(&m->edge[k], 3 * 64, 64, true) || !mlp16(&m->node[k], 2 * 64, 64, true)) return false;
  Step16Args a{};
  a.n = (int)n; a.T = T; a.dim = d; a.ex_ptr = in->ex_ptr; a.n_ex = in->n_ex;
  a.radius = in->radius; a.r2 = in->radius * in->radius; a.cap = cap; a.loop = 1;
  a.types = in->types; a.emb_w = in->emb_w; a.emb_dim = in->emb_dim; a.use_emb = in->use_emb; a.feat = feat;
  a.vel_mean = in->vel_mean; a.vel_std = in->vel_std; a.acc_mean = in->acc_mean; a.acc_std = in->acc_std;
  a.wall_max = in->wall_max; a.wall_div = in->wall_div;
  a.L = L;
  for (int k = 0; k < L; ++k) {
    const sgnn_mlp &e = m->edge[k], &v = m->node[k];
    a.lay[k] = Lay16{e.w1, e.b1, e.w2, e.b2, e.ln_g, e.ln_b, v.w1, v.b1, v.w2, v.b2, v.ln_g, v.ln_b};
  }
  const sgnn_mlp *xn = m->enc_node, *xe = m->enc_edge, *dc = m->dec;
  a.xn_w1 = xn->w1; a.xn_b1 = xn->b1; a.xn_w2 = xn->w2; a.xn_b2 = xn->b2; a.xn_g = xn->ln_g; a.xn_bb = xn->ln_b;
  a.xe_w1 = xe->w1; a.xe_b1 = xe->b1; a.xe_w2 = xe->w2; a.xe_b2 = xe->b2; a.xe_g = xe->ln_g; a.xe_bb = xe->ln_b;
  a.d_w1 = dc->w1; a.d_b1 = dc->b1; a.d_w2 = dc->w2; a.d_b2 = dc->b2;
  a.uvl = ws->uvl; a.flags = ws->step_flags; a.deg_out = ws->step_deg; a.nbr_out = nullptr;
  a.pos_seq = pos_seq; a.pred = pred; a.next_pos = next_pos; a.window_out = window_out;
  // receivers per workgroup: 8 up to 2,048 particles (C1: 250 workgroups), then as many as keep
  // the grid at one workgroup per CU (up to 32: the Taylor bars' 4,800 / 6,400 / 8,000 at 19 / 25 / 32)
  const int64_t cus = std::min<int64_t>(device_cus(), kStep16MaxGrid);
  if (cus < 1) return false;
  a.nt = (int)std::max<int64_t>(8, (n + cus - 1) / cus);
  if (a.nt > kStep16MaxNT || (n + a.nt - 1) / a.nt > cus) return false;
  a.ecap_t = a.nt * cap;
  a.e0_hbm = a.nt > 16 ? 1 : 0;   // two node sub-tiles: their e0 rows live in HBM
  a.poll_limit = ws->step_poll_limit;
  a.skew = ws->step_skew;
  // XCD-contiguous tiles: a tile's sender tiles then mostly share its XCD's L2 (HBM/MALL traffic
  // C1 r = 15 20.1 -> 16.7 MB per launch).  With the phase counters 64 B apart it is as fast as the
  // dispatch order or faster at every size (profiles/r05_ab_flag_stride.txt, r05_ab_xcd_all_sizes.txt);
  // with packed counters it was slower on some boxes (the counters of a tile's neighbours shared a
  // line its producers kept writing: r05_ab_dispatch_order_packed_flags.txt)
  a.tile_order = 1;
  size_t lds = step16_lds_bytes(a);
  if (lds > kStep16MaxLds && !a.e0_hbm) {  // the tile's e0 rows do not fit in LDS: keep them in HBM (ws->uvl's tail)
    a.e0_hbm = 1;
    lds = step16_lds_bytes(a);
  }
  if (lds == 0 || lds > kStep16MaxLds) return false;
  // co-residency: every workgroup of the launch must be on the device at once (include/sgnn.h)
  if (step16_resident(a) < (n + a.nt - 1) / a.nt) return false;
  *out = a;
  return true;
}

constexpr size_t kStepFlagBytes = sgnn::kStepFlagWords * sizeof(uint32_t);
constexpr int kMaxDevices = 64;

// In-process co-residency guard (include/sgnn.h, "Co-residency"): per device, the stream and an event
// recorded after the last call that ran the one-launch step.  A call holds the lock while it decides
// and launches, so two host threads cannot both launch one-launch steps on different streams.
struct Step16Guard {
  hipStream_t stream = nullptr;
  hipEvent_t done = nullptr;
};
std::mutex g_guard_mu;
Step16Guard g_guard[kMaxDevices];

class Step16Call {
 public:
  explicit Step16Call(hipStream_t s) : lk_(g_guard_mu), s_(s) {
    if (hipGetDevice(&dev_) != hipSuccess || dev_ < 0 || dev_ >= kMaxDevices) {
      dev_ = -1;
      return;
    }
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    capturing_ = hipStreamIsCapturing(s, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone;
    // (no event query while capturing: the graph's replays are ordered on their own stream)
    const Step16Guard& g = g_guard[dev_];
    allow_ = capturing_ || !g.done || g.stream == s || hipEventQuery(g.done) != hipErrorNotReady;
  }
  bool allow() const { return allow_ && dev_ >= 0; }
  // after the call's launches: remember them if any was a one-launch step
  void launched_step16() {
    if (dev_ < 0 || capturing_) return;
    Step16Guard& g = g_guard[dev_];
    if (!g.done && hipEventCreateWithFlags(&g.done, hipEventDisableTiming) != hipSuccess) {
      g.done = nullptr;
      return;
    }
    if (hipEventRecord(g.done, s_) == hipSuccess) g.stream = s_;
  }

 private:
  std::lock_guard<std::mutex> lk_;
  hipStream_t s_;
  int dev_ = -1;
  bool capturing_ = false, allow_ = false;
};

}  // namespace

extern "C" int sgnn_step_path(const sgnn_epd* m, const sgnn_step_in* in, const sgnn_step_ws* ws, int32_t* nt,
                              int32_t* grid) {
  sgnn::Step16Args a{};
  float dummy = 0.0f;
  const bool one = step16_plan(m, in, &dummy, ws, &dummy, &dummy, nullptr, &a);
  if (nt) *nt = one ? a.nt : 0;
  if (grid) *grid = one ? (int32_t)((a.n + a.nt - 1) / a.nt) : 0;
  return one ? 1 : 0;
}

// One predict_positions; `step` = index of this step within the call (the
// one-launch step's phase counters are zeroed at step 0 and count on).
// pos_last: optional contiguous copy of pos_seq's last frame (a rollout's previous next_pos).
// allow16: the call's co-residency guard lets it use the one-launch step; *used16 is set when it did.
static int predict_impl(const sgnn_epd* m, const sgnn_step_in* in, const float* pos_seq, const sgnn_step_ws* ws,
                        float* pred, float* next_pos, float* window_out, void* stream, int32_t step,
                        const float* pos_last, bool allow16, bool* used16) {
  using namespace sgnn;
  if (!m || !in || !pos_seq || !ws || !pred || !next_pos || m->nlayers < 1 || !m->edge || !m->node)
    return set_error(SGNN_ERR_INVALID, "predict_positions: bad arguments");
  if (!ws_ok(ws))
    return set_error(SGNN_ERR_INVALID, "predict_positions: sgnn_step_ws.struct_size != sizeof(sgnn_step_ws) "
                                       "(caller built against another include/sgnn.h revision)");
  if (window_out && window_out == pos_seq)
    return set_error(SGNN_ERR_INVALID, "predict_positions: window_out aliases pos_seq");
  hipStream_t s = static_cast<hipStream_t>(stream);
  Step16Args sa{};
  if (allow16 && step16_plan(m, in, pos_seq, ws, pred, next_pos, window_out, &sa)) {
    // the phase counters and the error word start from zero in every call
    if (step == 0 && hipMemsetAsync(ws->step_flags, 0, kStepFlagBytes, s) != hipSuccess)
      return check_launch("predict_positions: zeroing the step counters");
    sa.epoch0 = (uint32_t)step * (uint32_t)(m->nlayers + 1);
    sa.pos_last = pos_last;
    *used16 = true;
    return step16_launch(sa, s);
  }
  // the per-kernel sequence: clear a previous call's error word so sgnn_step_check reads this call's
  if (step == 0 && ws->step_flags &&
      hipMemsetAsync(ws->step_flags + kStepFlagErr, 0, sizeof(uint32_t), s) != hipSuccess)
    return check_launch("predict_positions: clearing the step error word");
  const int64_t n = in->n;
  const int T = in->T, d = in->dim;
  // radius graph on the most recent frame (learned_simulator.py:116-117); graphs of <= 2,560
  // particles launch its search together with the node encoder (independent work, one launch whose
  // grid fits the 256 CUs once: C1 0.1275 -> 0.1239 ms/step; measured slower at 4,800 / 8,000
  // particles, 0.156 -> 0.167 / 0.217 -> 0.268, where the radius search needs more workgroups)
#ifndef SGNN_MERGE_MAX_N
#define SGNN_MERGE_MAX_N 8192
#endif
  constexpr int64_t kMergeMaxN = SGNN_MERGE_MAX_N;
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

extern "C" int sgnn_predict_positions(const sgnn_epd* m, const sgnn_step_in* in, const float* pos_seq,
                                      const sgnn_step_ws* ws, float* pred, float* next_pos,
                                      float* window_out, void* stream) {
  Step16Call call(static_cast<hipStream_t>(stream));
  bool used16 = false;
  const int st = predict_impl(m, in, pos_seq, ws, pred, next_pos, window_out, stream, 0, nullptr, call.allow(),
                              &used16);
  if (used16) call.launched_step16();
  return st;
}

extern "C" int sgnn_rollout(const sgnn_epd* m, const sgnn_step_in* in, float* win_a, float* win_b,
                            const sgnn_step_ws* ws, int32_t nsteps, float* out_pos, float* out_pred,
                            void* stream) {
  using namespace sgnn;
  if (!win_a || !win_b || win_a == win_b || !out_pos || !out_pred || nsteps < 0)
    return set_error(SGNN_ERR_INVALID, "rollout: bad arguments");
  const int64_t n = in ? in->n : 0;
  const int d = in ? in->dim : 0;
  Step16Call call(static_cast<hipStream_t>(stream));
  bool used16 = false;
  int st = SGNN_OK;
  for (int32_t k = 0; k < nsteps && st == SGNN_OK; ++k) {
    float* cur = (k & 1) ? win_b : win_a;
    float* nxt = (k & 1) ? win_a : win_b;
    // step k's window ends with step k-1's prediction, already contiguous in out_pos; every step of
    // the call takes the path its first step took
    st = predict_impl(m, in, cur, ws, out_pred + (int64_t)k * n * (d + 1), out_pos + (int64_t)k * n * d, nxt,
                      stream, k, k > 0 ? out_pos + (int64_t)(k - 1) * n * d : nullptr, call.allow() && (k == 0 || used16),
                      &used16);
  }
  if (used16) call.launched_step16();
  return st;
}

namespace {
// one_step rollout (evaluate.py:140-143): the next window's last frame is the ground-truth position of
// the step, win[i][T-1][:] = gt[i * gt_ld + c] (the predicted frame the decoder shifted in is replaced)
__global__ void k_teacher_frame(float* win, int64_t n, int T, int d, const float* gt, int64_t gt_ld) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n * d) return;
  const int64_t i = t / d;
  const int c = (int)(t - i * d);
  win[(i * T + T - 1) * d + c] = gt[i * gt_ld + c];
}
}  // namespace

extern "C" int sgnn_rollout_one_step(const sgnn_epd* m, const sgnn_step_in* in, float* win_a, float* win_b,
                                     const sgnn_step_ws* ws, int32_t nsteps, const float* gt, int64_t gt_ld_n,
                                     int64_t gt_ld_t, float* out_pos, float* out_pred, void* stream) {
  using namespace sgnn;
  if (!in || !win_a || !win_b || win_a == win_b || !out_pos || !out_pred || nsteps < 0 || (nsteps > 0 && !gt) ||
      gt_ld_n < in->dim || gt_ld_t < 0)
    return set_error(SGNN_ERR_INVALID, "rollout_one_step: bad arguments");
  const int64_t n = in->n;
  const int d = in->dim, T = in->T;
  hipStream_t s = static_cast<hipStream_t>(stream);
  Step16Call call(s);
  bool used16 = false;
  int st = SGNN_OK;
  for (int32_t k = 0; k < nsteps && st == SGNN_OK; ++k) {
    float* cur = (k & 1) ? win_b : win_a;
    float* nxt = (k & 1) ? win_a : win_b;
    // the window's last frame is ground truth from step 1 on: read from the window itself (no pos_last)
    st = predict_impl(m, in, cur, ws, out_pred + (int64_t)k * n * (d + 1), out_pos + (int64_t)k * n * d, nxt,
                      stream, k, nullptr, call.allow() && (k == 0 || used16), &used16);
    if (st == SGNN_OK && k + 1 < nsteps && n > 0) {
      const int64_t tot = n * d;
      hipLaunchKernelGGL(k_teacher_frame, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, nxt, n, T, d,
                         gt + (int64_t)k * gt_ld_t, gt_ld_n);
      st = check_launch("rollout_one_step: ground-truth frame");
    }
  }
  if (used16) call.launched_step16();
  return st;
}

extern "C" int sgnn_step_check(const sgnn_step_ws* ws, void* stream) {
  using namespace sgnn;
  if (!ws_ok(ws)) return set_error(SGNN_ERR_INVALID, "step_check: bad arguments (or sgnn_step_ws.struct_size)");
  if (!ws->step_flags) return SGNN_OK;
  hipStream_t s = static_cast<hipStream_t>(stream);
  uint32_t word = 0;
  if (hipMemcpyAsync(&word, ws->step_flags + kStepFlagErr, sizeof(word), hipMemcpyDeviceToHost, s) != hipSuccess ||
      hipStreamSynchronize(s) != hipSuccess)
    return check_launch("step_check: reading the step error word");
  if (word != 0) {
    char msg[256];
    snprintf(msg, sizeof(msg),
             "one-launch step: a workgroup timed out waiting for its sender tiles (phase %u); this call's "
             "outputs are invalid (another one-launch step shared the device's CUs?)", word);
    return set_error(SGNN_ERR_STEP_TIMEOUT, msg);
  }
  return SGNN_OK;
}
