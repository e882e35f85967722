// Small-graph radius search body (n <= kSmallN), shared by k_radius_small
// (radius.hip) and the merged radius + node-encoder launch (fwd16.hip).
//
// Every workgroup stages the whole position array in LDS (coalesced, SoA),
// and one wave per query walks the candidates of the query's example IN
// ASCENDING INDEX, 64 per step, straight out of LDS; it keeps the in-range
// ones in order and stops as soon as it holds `cap` of them --
// torch_cluster's CUDA rule (first K in ascending index, strict <, as reached
// by sgnn/single_scale/learned_simulator.py:116-117) needs no sort and no
// merge in this order.  Writes the padded lists nbr [n][cap] and deg [n].
#pragma once
#include "common.h"
#include "sgnn_internal.h"

namespace sgnn {

constexpr int kSmallN = 8192;
constexpr int kSmallBlock = 512;  // 8 query waves per workgroup
constexpr int kRadiusMaxCap = 64;  // neighbour cap K (+1 without self loops): one kept slot per lane

struct RadiusSmallArgs {
  const float* pos;
  int64_t stride;
  int n, dim;
  const int64_t* ex_ptr;
  int n_ex;
  float r2;
  int cap, loop;
  int32_t *nbr, *deg;              // padded lists (workspace)
  int32_t *rowptr, *send, *recv;   // CSR outputs
};

// LDS bytes of the body: positions [DIM][n] + the per-wave kept lists.
inline size_t radius_small_lds(int n, int dim) {
  return sizeof(float) * (size_t)n * dim + sizeof(int32_t) * (kSmallBlock / 64) * kRadiusMaxCap;
}

// Launches k_csr_small (deg -> rowptr, padded lists -> receiver-sorted CSR);
// the lists must have been written by an earlier launch on `s`.
int radius_small_csr(const RadiusSmallArgs& a, hipStream_t s);
// Both launches of the small path (radius.hip).
int radius_small_launch(const RadiusSmallArgs& a, hipStream_t s);
// Fills *out when sgnn_radius_graph would take the small path with these
// arguments (same meaning as its parameters); false otherwise.
bool radius_small_plan(const float* pos, int64_t pos_stride, int64_t n, int32_t dim, const int64_t* ex_ptr,
                       int32_t n_ex, float radius, int32_t K, int32_t loop, void* workspace, int32_t* rowptr,
                       int32_t* send, int32_t* recv, int64_t edge_cap, RadiusSmallArgs* out);

// Queries blk, blk + nblk, ... in waves of 8 (workgroup of kSmallBlock threads).
// lds: radius_small_lds(n, DIM) bytes.
template <int DIM>
SGNN_DEV void radius_small_body(const RadiusSmallArgs& a, float* lds, int blk, int nblk) {
  const int n = a.n;
  float* sp = lds;  // [DIM][n] SoA
  int32_t* kept_all = reinterpret_cast<int32_t*>(lds + (size_t)n * DIM);
  for (int t = threadIdx.x; t < n * DIM; t += kSmallBlock) {
    const int i = t / DIM, d = t - i * DIM;
    sp[d * n + i] = a.pos[(int64_t)i * a.stride + d];
  }
  __syncthreads();
  const int lane = lane_id(), w = wave_id();
  int32_t* kw = kept_all + w * kRadiusMaxCap;
  const int cap = a.cap;
  for (int i = blk * (kSmallBlock / 64) + w; i < n; i += nblk * (kSmallBlock / 64)) {
    int lo = 0, hi = a.n_ex - 1;  // example of i: largest b with ex_ptr[b] <= i
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (a.ex_ptr[mid] <= i) lo = mid; else hi = mid - 1;
    }
    const int jb = (int)a.ex_ptr[lo], je = (int)a.ex_ptr[lo + 1];
    float pi[DIM];
#pragma unroll
    for (int d = 0; d < DIM; ++d) pi[d] = sp[d * n + i];
    int cnt = 0;
    for (int base = jb; base < je && cnt < cap; base += 64) {
      const int j = base + lane;
      bool in = false;
      if (j < je) {
        float s = 0.0f;  // fp32, dims summed in order, no contraction (oracle rule)
#pragma unroll
        for (int d = 0; d < DIM; ++d) {
          const float t = __fsub_rn(sp[d * n + j], pi[d]);
          s = __fadd_rn(s, __fmul_rn(t, t));
        }
        in = s < a.r2;
      }
      const uint64_t bal = __ballot(in);
      const int slot = cnt + (int)__popcll(bal & ((1ull << lane) - 1ull));
      if (in && slot < cap) kw[slot] = j;
      cnt += (int)__popcll(bal);
    }
    wave_lds_sync();
    cnt = min(cnt, cap);
    int top = lane < cnt ? kw[lane] : INT32_MAX;
    if (!a.loop) {  // torch_cluster: K+1 first-by-index, then drop the self loop
      const uint64_t self = __ballot(lane < cnt && top == i);
      if (self) {
        const int at = __ffsll((long long)self) - 1;
        const int nxt = __shfl(top, (lane + 1) & 63, 64);
        if (lane >= at) top = (lane + 1 < cnt) ? nxt : INT32_MAX;
        cnt -= 1;
      }
    }
    if (lane < cnt) {
      SGNN_BOUNDS(top, 0, a.n, "radius(small) neighbour");
      a.nbr[(int64_t)i * cap + lane] = top;
    }
    if (lane == 0) a.deg[i] = cnt;
    wave_lds_sync();
  }
}

}  // namespace sgnn
