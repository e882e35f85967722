// Small-graph radius search body (n <= kSmallN), shared by k_radius_small
// (radius.hip) and the merged radius + node-encoder launch (fwd16.hip).
//
// Workgroup b owns a contiguous run of queries.  It first filters the
// candidates of their examples against the run's bounding box grown by the
// radius (coalesced loads, kept in ascending index in LDS: positions SoA +
// ids), then one wave per query walks that list IN ASCENDING INDEX, 64 per
// step, keeps the in-range ones in order and stops as soon as it holds `cap`
// of them -- torch_cluster's CUDA rule (first K in ascending index, strict <,
// as reached by sgnn/single_scale/learned_simulator.py:116-117) needs no sort
// and no merge in this order.  The box is conservative (every in-range pair
// passes it under fp32 rounding), so the list holds every candidate the
// exact test can accept: the graph is the brute force's bit for bit, and a
// run of spatially close queries (consecutive lattice indices) walks a few
// dozen candidates instead of all n.  Writes the padded lists nbr [n][cap]
// and deg [n].
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

constexpr int kSmallChunks = kSmallN / 64 / (kSmallBlock / 64);  // 64-candidate chunks per wave, at most

// LDS bytes of the body: candidate positions [DIM][n] + ids [n], the per-wave kept lists, the chunk
// offsets and the box partials.
inline size_t radius_small_lds(int n, int dim) {
  return sizeof(float) * (size_t)n * (dim + 1) + sizeof(int32_t) * (kSmallBlock / 64) * kRadiusMaxCap +
         sizeof(int32_t) * (kSmallN / 64 + 4) + sizeof(float) * (kSmallBlock / 64) * 8;
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

// Queries [blk * per, (blk + 1) * per) of workgroup blk (of nblk), per = ceil(n / nblk); waves of 8
// (workgroup of kSmallBlock threads).  lds: radius_small_lds(n, DIM) bytes.
template <int DIM>
SGNN_DEV void radius_small_body(const RadiusSmallArgs& a, float* lds, int blk, int nblk) {
  const int n = a.n;
  const int lane = lane_id(), w = wave_id();
  constexpr int kW = kSmallBlock / 64;
  const int per = (n + nblk - 1) / nblk;
  const int q0 = min(n, blk * per), q1 = min(n, q0 + per);
  float* cp = lds;                                                  // [DIM][n] candidate positions
  int32_t* cid = reinterpret_cast<int32_t*>(lds + (size_t)n * DIM);  // [n] candidate ids
  int32_t* kept_all = cid + n;                                      // [kW][kRadiusMaxCap]
  int32_t* coff = kept_all + kW * kRadiusMaxCap;                    // [n / 64 + 1] chunk offsets
  float* red = reinterpret_cast<float*>(coff + kSmallN / 64 + 4);   // [kW][2 DIM] box partials
  // the run's bounding box (lanes over queries, then waves)
  float lo[DIM], hi[DIM];
#pragma unroll
  for (int d = 0; d < DIM; ++d) {
    lo[d] = INFINITY;
    hi[d] = -INFINITY;
  }
  for (int i = q0 + (int)threadIdx.x; i < q1; i += kSmallBlock)
#pragma unroll
    for (int d = 0; d < DIM; ++d) {
      const float v = a.pos[(int64_t)i * a.stride + d];
      lo[d] = fminf(lo[d], v);
      hi[d] = fmaxf(hi[d], v);
    }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1)
#pragma unroll
    for (int d = 0; d < DIM; ++d) {
      lo[d] = fminf(lo[d], __shfl_xor(lo[d], o, 64));
      hi[d] = fmaxf(hi[d], __shfl_xor(hi[d], o, 64));
    }
  if (lane == 0)
#pragma unroll
    for (int d = 0; d < DIM; ++d) {
      red[w * 2 * DIM + d] = lo[d];
      red[w * 2 * DIM + DIM + d] = hi[d];
    }
  __syncthreads();
  float mag = 0.0f;
#pragma unroll
  for (int d = 0; d < DIM; ++d) {
    for (int k = 0; k < kW; ++k) {
      lo[d] = fminf(lo[d], red[k * 2 * DIM + d]);
      hi[d] = fmaxf(hi[d], red[k * 2 * DIM + DIM + d]);
    }
    mag = fmaxf(mag, fmaxf(fabsf(lo[d]), fabsf(hi[d])));
  }
  // margin: |p_j - p_i|^2 < r^2 in fp32 implies |p_j,d - p_i,d| < r (1 + 2^-22) + one ulp of the
  // coordinates; 1e-3 r + 1e-6 |p| covers both with room (a wider box only keeps more candidates)
  const float r = sqrtf(a.r2);
  const float m = 1.001f * r + 1e-6f * (mag + 1.0f);
  // candidates: the examples of the run's queries, [jb, je)
  int jb = 0, je = 0;
  if (q0 < q1) {
    int lo_e = 0, hi_e = a.n_ex - 1;
    while (lo_e < hi_e) {
      const int mid = (lo_e + hi_e + 1) >> 1;
      if (a.ex_ptr[mid] <= q0) lo_e = mid; else hi_e = mid - 1;
    }
    jb = (int)a.ex_ptr[lo_e];
    lo_e = 0;
    hi_e = a.n_ex - 1;
    while (lo_e < hi_e) {
      const int mid = (lo_e + hi_e + 1) >> 1;
      if (a.ex_ptr[mid] <= q1 - 1) lo_e = mid; else hi_e = mid - 1;
    }
    je = (int)a.ex_ptr[lo_e + 1];
  }
  // pass 1: wave w filters chunks w, w + 8, ... (positions kept in registers), counts per chunk
  const int nch = (je - jb + 63) / 64;
  float pj[kSmallChunks][DIM];
  bool inb[kSmallChunks];
#pragma unroll
  for (int c = 0; c < kSmallChunks; ++c) {
    const int ch = w + kW * c;
    const int j = jb + 64 * ch + lane;
    inb[c] = false;
    if (ch < nch && j < je) {
#pragma unroll
      for (int d = 0; d < DIM; ++d) pj[c][d] = a.pos[(int64_t)j * a.stride + d];
    }
  }
#pragma unroll
  for (int c = 0; c < kSmallChunks; ++c) {
    const int ch = w + kW * c;
    if (ch >= nch) break;
    const int j = jb + 64 * ch + lane;
    bool in = j < je;
#pragma unroll
    for (int d = 0; d < DIM; ++d) in = in && pj[c][d] >= lo[d] - m && pj[c][d] <= hi[d] + m;
    inb[c] = in;
    const int cnt = (int)__popcll(__ballot(in));
    if (lane == 0) coff[ch] = cnt;
  }
  __syncthreads();
  if (w == 0) {  // exclusive scan of the chunk counts (nch <= 128)
    int run = 0;
    for (int c0 = 0; c0 < nch; c0 += 64) {
      const int c = c0 + lane;
      const int v = c < nch ? coff[c] : 0;
      int incl = v;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const int t = __shfl_up(incl, o, 64);
        if (lane >= o) incl += t;
      }
      if (c < nch) coff[c] = run + incl - v;
      run += __shfl(incl, 63, 64);
    }
    if (lane == 0) coff[nch] = run;
  }
  __syncthreads();
  // pass 2: the kept candidates in ascending index
#pragma unroll
  for (int c = 0; c < kSmallChunks; ++c) {
    const int ch = w + kW * c;
    if (ch >= nch) break;
    const uint64_t bal = __ballot(inb[c]);
    if (inb[c]) {
      const int slot = coff[ch] + (int)__popcll(bal & ((1ull << lane) - 1ull));
      cid[slot] = jb + 64 * ch + lane;
#pragma unroll
      for (int d = 0; d < DIM; ++d) cp[d * n + slot] = pj[c][d];
    }
  }
  __syncthreads();
  const int total = coff[nch];
  int32_t* kw = kept_all + w * kRadiusMaxCap;
  const int cap = a.cap;
  for (int i = q0 + w; i < q1; i += kW) {
    int lo_e = 0, hi_e = a.n_ex - 1;  // example of i: largest b with ex_ptr[b] <= i
    while (lo_e < hi_e) {
      const int mid = (lo_e + hi_e + 1) >> 1;
      if (a.ex_ptr[mid] <= i) lo_e = mid; else hi_e = mid - 1;
    }
    const int ib = (int)a.ex_ptr[lo_e], ie = (int)a.ex_ptr[lo_e + 1];
    float pi[DIM];
#pragma unroll
    for (int d = 0; d < DIM; ++d) pi[d] = a.pos[(int64_t)i * a.stride + d];
    int cnt = 0;
    for (int base = 0; base < total && cnt < cap; base += 64) {
      const int k = base + lane;
      bool in = false;
      int j = 0;
      if (k < total) {
        j = cid[k];
        float s = 0.0f;  // fp32, dims summed in order, no contraction (oracle rule)
#pragma unroll
        for (int d = 0; d < DIM; ++d) {
#pragma clang fp contract(off)
          const float t = __fsub_rn(cp[d * n + k], pi[d]);
          s = __fadd_rn(s, __fmul_rn(t, t));
        }
        in = j >= ib && j < ie && s < a.r2;
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
