// Radius-graph neighbour search for gfx950 (replaces torch_cluster.radius as
// reached by sgnn/single_scale/learned_simulator.py:116-117).
//
// Small graphs (n <= 8192): k_radius_small (every workgroup stages all
// positions in LDS; one wave per query scans its example in ascending index
// and stops at the cap) + k_csr_small (scan + compaction): two launches.
//
// Large graphs (no host sync, capturable in a hipGraph):
//   0. k_bbox             per-block bounding boxes of the finite coordinates; zeroes
//                         the cell histogram (no memset launch)
//   1. k_cell_assign      particle -> (example, dense cell of side 1.01 r, grown
//                         x2 until the grid fits the workspace); histogram
//   2. scan               cell counts -> cell starts
//   3. k_cell_scatter     counting sort into cell order + a cell-ordered copy
//                         of the positions (x, y, z, id)
//   4. k_radius_query_lds LDS spatial binning: a workgroup per tile of 64
//                         cells of one grid row stages the 3^(d-1) neighbour
//                         row spans with coalesced float4 loads; one lane per
//                         particle keeps the cap smallest in-range ids
//                         (torch_cluster's CUDA rule: first K in ascending
//                         index).  Writes deg and a padded list.
//   5. scan               deg -> rowptr (rowptr[n] = E, left on the device)
//   6. k_compact          padded lists -> receiver-sorted CSR (send, recv)
#include "common.h"
#include "../../include/sgnn.h"
#include "sgnn_internal.h"
#include "radius_small.h"

namespace {

constexpr int kScanItems = 8;
constexpr int kScanBlock = 256;
constexpr int kScanTile = kScanItems * kScanBlock;  // 2048 elements per block

__global__ __launch_bounds__(kScanBlock) void k_scan_block(const int32_t* in, int32_t* out,
                                                           int64_t len, int32_t* partials) {
  __shared__ int32_t wsum[kScanBlock / 64];
  const int64_t base = (int64_t)blockIdx.x * kScanTile + (int64_t)threadIdx.x * kScanItems;
  int32_t v[kScanItems];
  int32_t s = 0;
#pragma unroll
  for (int k = 0; k < kScanItems; ++k) {
    const int64_t i = base + k;
    v[k] = i < len ? in[i] : 0;
    s += v[k];
  }
  const int lane = threadIdx.x & 63, w = wave_id();
  int32_t incl = s;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int32_t t = __shfl_up(incl, o, 64);
    if (lane >= o) incl += t;
  }
  if (lane == 63) wsum[w] = incl;
  __syncthreads();
  int32_t woff = 0;
  for (int k = 0; k < w; ++k) woff += wsum[k];
  int32_t run = woff + incl - s;
#pragma unroll
  for (int k = 0; k < kScanItems; ++k) {
    const int64_t i = base + k;
    if (i < len) out[i] = run;
    run += v[k];
  }
  if (threadIdx.x == blockDim.x - 1) partials[blockIdx.x] = woff + incl;
}

// Adds the exclusive prefix of the block totals: each block reduces the
// totals of the blocks before it itself (<= 8192 of them), so the totals need
// no scan launch of their own.
__global__ __launch_bounds__(kScanBlock) void k_scan_add(int32_t* out, int64_t len,
                                                         const int32_t* partials) {
  __shared__ int32_t wsum[kScanBlock / 64];
  int32_t s = 0;
  for (int b = threadIdx.x; b < (int)blockIdx.x; b += blockDim.x) s += partials[b];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  if (lane_id() == 0) wsum[wave_id()] = s;
  __syncthreads();
  int32_t add = 0;
#pragma unroll
  for (int k = 0; k < kScanBlock / 64; ++k) add += wsum[k];
  const int64_t base = (int64_t)blockIdx.x * kScanTile;
  for (int k = threadIdx.x; k < kScanTile; k += blockDim.x) {
    const int64_t i = base + k;
    if (i < len) out[i] += add;
  }
}

// ---------------------------------------------------------------------------
// Dense cell grid derived on the device from the particles' bounding box, so
// no host sync: the three cells of one grid row (dx = -1..1) are contiguous in
// cell order, a 2D query walks 3 spans (3D: 9) of the cell-sorted id array.
struct Grid {  // 28 bytes, stored at bbox + 8 (8 words reserved)
  float lo[3];
  float inv_cell;
  int g[3];
};

static_assert(sizeof(Grid) <= 32, "Grid must fit the 8 reserved words");

// order-preserving float <-> uint so atomicMax/Min work on zero-initialised words
SGNN_DEV uint32_t f2ord(float f) {
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
SGNN_DEV float ord2f(uint32_t o) {
  return __uint_as_float((o & 0x80000000u) ? (o & 0x7FFFFFFFu) : ~o);
}

// bbox words: [0..2] = ~ord(min_d) (max of the complement = min), [3..5] =
// ord(max_d) (0: no finite value); the derived Grid lives at bbox + 8.

// Every thread derives the same grid from the bbox (identical float ops).
SGNN_DEV Grid make_grid(const uint32_t (&bbox)[6], int dim, int n_ex, float cell0, int64_t max_cells) {
  Grid G;
  float lo[3] = {0.f, 0.f, 0.f}, hi[3] = {0.f, 0.f, 0.f};
  for (int d = 0; d < 3; ++d) {
    if (d < dim && bbox[d] != 0u && bbox[3 + d] != 0u) {
      lo[d] = ord2f(~bbox[d]);
      hi[d] = ord2f(bbox[3 + d]);
    }
    G.lo[d] = lo[d];
  }
  float cell = cell0;
  for (int it = 0; it < 64; ++it) {
    int64_t tot = n_ex;
    for (int d = 0; d < 3; ++d) {
      const float ext = (hi[d] - lo[d]) / cell;
      G.g[d] = d < dim ? (int)fminf(ext, 1.0e7f) + 1 : 1;
      tot *= G.g[d];
    }
    if (tot <= max_cells) break;
    cell *= 2.0f;
  }
  G.inv_cell = 1.0f / cell;
  return G;
}

// Per-block bounding-box partials (no atomics, nothing to initialise): block
// b writes its 6 words to bboxp[8 b ..]; k_cell_assign reduces them.  The
// blocks also zero the cell histogram words (count, fill) the later kernels
// accumulate into, so the pipeline needs no memset launch.
template <int DIM>
__global__ __launch_bounds__(256) void k_bbox(const float* pos, int64_t stride, int64_t n, uint32_t* bboxp,
                                              int32_t* zero, int64_t nzero) {
  __shared__ uint32_t red[6][4];
  uint32_t v[6] = {0, 0, 0, 0, 0, 0};
  const int64_t gsz = (int64_t)gridDim.x * blockDim.x, gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (int64_t i = gid; i < nzero; i += gsz) zero[i] = 0;
  for (int64_t i = gid; i < n; i += gsz) {
#pragma unroll
    for (int d = 0; d < DIM; ++d) {
      const float x = pos[i * stride + d];
      if (isfinite(x)) {
        const uint32_t o = f2ord(x);
        v[d] = max(v[d], ~o);
        v[3 + d] = max(v[3 + d], o);
      }
    }
  }
  const int lane = threadIdx.x & 63, w = wave_id();
#pragma unroll
  for (int k = 0; k < 6; ++k) {
    uint32_t a = v[k];
    for (int o = 32; o > 0; o >>= 1) a = max(a, (uint32_t)__shfl_xor((int)a, o, 64));
    if (lane == 0) red[k][w] = a;
  }
  __syncthreads();
  if (threadIdx.x < 6) {
    uint32_t a = 0;
    for (int k = 0; k < (int)(blockDim.x >> 6); ++k) a = max(a, red[threadIdx.x][k]);
    bboxp[8 * blockIdx.x + threadIdx.x] = a;
  }
}

SGNN_DEV int cell_of(float x, float lo, float inv_cell, int g) {
  float q = floorf((x - lo) * inv_cell);
  if (!(q == q)) q = 0.0f;
  q = fminf(fmaxf(q, 0.0f), (float)(g - 1));
  return (int)q;
}

SGNN_DEV float dist2_ordered(const float* a, const float* b, int dim) {
  // fp32, dims summed in order, no contraction: matches the oracle / golden rule.
  float s = 0.0f;
  for (int d = 0; d < dim; ++d) {
#pragma clang fp contract(off)
    const float t = __fsub_rn(a[d], b[d]);
    s = __fadd_rn(s, __fmul_rn(t, t));
  }
  return s;
}

// Atomic add of 1 per active lane to counter[key], wave-aggregated where it
// pays: coarse cells put a whole wave's particles in one or two cells, where
// per-lane atomics serialise on one address, so a key shared by >= 4 lanes
// takes one atomic for its group; once the leading group is small (fine cells:
// ~1-2 particles per cell and wave-distinct keys) the remaining lanes issue
// their own atomics in one instruction instead of one serial round trip per key.
// Returns the lane's slot = old counter value + its rank among same-key lanes.
SGNN_DEV int32_t wave_aggregated_inc(int32_t* counter, int32_t key, bool active) {
  const int lane = lane_id();
  uint64_t remaining = __ballot(active);
  int32_t slot = 0;
  for (int it = 0; remaining && it < 4; ++it) {
    const int leader = __ffsll((unsigned long long)remaining) - 1;
    const int32_t lkey = __shfl(key, leader, 64);
    const uint64_t grp = __ballot(active && key == lkey) & remaining;
    if (__popcll(grp) < 4) break;
    int32_t base = 0;
    if (lane == leader) base = atomicAdd(&counter[lkey], (int32_t)__popcll(grp));
    base = __shfl(base, leader, 64);
    if ((grp >> lane) & 1ull) slot = base + (int32_t)__popcll(grp & ((1ull << lane) - 1ull));
    remaining &= ~grp;
  }
  if ((remaining >> lane) & 1ull) slot = atomicAdd(&counter[key], 1);
  return slot;
}

// DIM is a template parameter: with a runtime dimension loop the compiler kept
// the Grid in LDS and issued the coordinate loads one after another (measured
// 25 us vs 4 us for 50k particles, tools/bench_assign.hip).
// Every block reduces k_bbox's partials and derives the grid (identical float
// ops in every block); block 0 also stores it at bbox + 8 for the query.
template <int DIM>
__global__ __launch_bounds__(256) void k_cell_assign(const float* pos, int64_t stride, int64_t n,
                                                     const int64_t* ex_ptr, int n_ex,
                                                     const uint32_t* bboxp, int nbb, float cell0,
                                                     int64_t max_cells, uint32_t* bbox, int32_t* cell_of_p,
                                                     int32_t* ex_of, int32_t* count) {
  __shared__ Grid sG;
  const int64_t i0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool active = i0 < n;
  const int64_t i = active ? i0 : n - 1;
  float x[DIM];
#pragma unroll
  for (int d = 0; d < DIM; ++d) x[d] = pos[i * stride + d];
  if (threadIdx.x < 64) {  // wave 0: lane L takes partials L, L + 64 (nbb <= 128), then a butterfly
    uint32_t v[6] = {0, 0, 0, 0, 0, 0};
    for (int k = threadIdx.x; k < nbb; k += 64)
#pragma unroll
      for (int c = 0; c < 6; ++c) v[c] = max(v[c], bboxp[8 * k + c]);
#pragma unroll
    for (int c = 0; c < 6; ++c)
      for (int o = 32; o > 0; o >>= 1) v[c] = max(v[c], (uint32_t)__shfl_xor((int)v[c], o, 64));
    if (threadIdx.x == 0) {
      sG = make_grid(v, DIM, n_ex, cell0, max_cells);
      if (blockIdx.x == 0) *reinterpret_cast<Grid*>(bbox + 8) = sG;
    }
  }
  __syncthreads();
  const Grid G = sG;
  int lo = 0, hi = n_ex - 1;  // largest b with ex_ptr[b] <= i
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (ex_ptr[mid] <= i) lo = mid; else hi = mid - 1;
  }
  int c[3] = {0, 0, 0};
#pragma unroll
  for (int d = 0; d < DIM; ++d) c[d] = cell_of(x[d], G.lo[d], G.inv_cell, G.g[d]);
  const int32_t key = (int32_t)((((int64_t)lo * G.g[2] + c[2]) * G.g[1] + c[1]) * G.g[0] + c[0]);
  if (active) {
    cell_of_p[i] = key;
    ex_of[i] = lo;
    // histogram only: a non-returning atomic (the slot is taken in k_cell_scatter)
    __hip_atomic_fetch_add(&count[key], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

template <int DIM>
__global__ __launch_bounds__(256) void k_cell_scatter(int64_t n, const int32_t* cell_of_p,
                                                      const int32_t* start, int32_t* fill,
                                                      int32_t* order, const float* pos, int64_t stride,
                                                      f32x4* cpos) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool active = i < n;
  const int32_t b = active ? cell_of_p[i] : 0;
  const int32_t slot = wave_aggregated_inc(fill, b, active);
  if (active) {
    const int32_t at = start[b] + slot;
    order[at] = (int32_t)i;
    if (cpos) {  // cell-ordered copy (x, y, z, id): the LDS-binned query stages contiguous spans of it
      f32x4 v = {0.0f, 0.0f, 0.0f, __int_as_float((int)i)};
#pragma unroll
      for (int d = 0; d < DIM; ++d) v[d] = pos[i * stride + d];
      cpos[at] = v;
    }
  }
}

// ---------------------------------------------------------------------------
// LDS-binned query (large graphs): a workgroup owns a tile of kTX consecutive
// cells of one grid row (same example, z, y).  Its candidates -- the
// 3^(dim-1) neighbour rows over cells [x0 - 1, x0 + kTX] -- are contiguous
// spans of the cell-ordered copy `cpos`, staged once into LDS with coalesced
// float4 loads together with the cell starts of those spans; every particle of
// the tile's own cells is then one lane, which walks its 3^dim neighbour
// cells out of LDS and keeps the `cap` smallest in-range ids in a sorted
// register list (torch_cluster's rule: first K by ascending index).  A tile
// whose candidates overflow the LDS capacity reads the same spans from HBM.
constexpr int kTX = 64;
constexpr int kQBlock = 256;
constexpr int kLdsCand = 3072;   // staged candidates (48 KB of float4)
// register-list lengths of the query kernel: 32 covers the reference's caps
// (20, 24, +1 without self loops); 64 serves caps 33..64 (torch_cluster's
// default max_num_neighbors = 32 with loop = False asks for 33)
template <int MAXCAP>
SGNN_DEV void sorted_insert(int (&top)[MAXCAP], int x) {
  // keep top[] ascending: x shifts the larger entries one slot up
#pragma unroll
  for (int s = MAXCAP - 1; s > 0; --s) {
    const int lo = top[s - 1];
    top[s] = x < lo ? lo : (x < top[s] ? x : top[s]);
  }
  top[0] = x < top[0] ? x : top[0];
}

template <int DIM, int kMaxCap>
__global__ __launch_bounds__(kQBlock) void k_radius_query_lds(
    const f32x4* cpos, const int32_t* start, const uint32_t* bbox, int n_ex, float r2, int cap, int loop,
    int32_t* nbr, int32_t* deg, int64_t n) {
  __shared__ f32x4 cand[kLdsCand];
  __shared__ int32_t cstart[9][kTX + 3];  // cell starts of each neighbour row's span (+ end)
  __shared__ int32_t seg_base[9 + 1];   // + the total
  __shared__ int32_t seg_g0[9];           // global index of each span's first candidate
  const Grid G = *reinterpret_cast<const Grid*>(bbox + 8);
  const int tiles_x = (G.g[0] + kTX - 1) / kTX;
  const int64_t ntiles = (int64_t)n_ex * G.g[2] * G.g[1] * tiles_x;
  constexpr int NR = DIM == 3 ? 9 : (DIM == 2 ? 3 : 1);
  if (threadIdx.x == 0 && blockIdx.x == 0) deg[n] = 0;  // scan sentinel -> rowptr[n] = E
  for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int64_t row = tile / tiles_x;  // row = (ex * g2 + cz) * g1 + cy
    const int x0 = (int)(tile - row * tiles_x) * kTX;
    const int x1 = min(x0 + kTX, G.g[0]);                     // own cells [x0, x1)
    const int xa = max(x0 - 1, 0), xb = min(x1, G.g[0] - 1);  // span cells [xa, xb]
    const int nspan = xb - xa + 1;
    const int cy = (int)(row % G.g[1]);
    const int cz = (int)((row / G.g[1]) % G.g[2]);
    __syncthreads();  // the previous tile's LDS is no longer read
    for (int q = threadIdx.x; q < NR * (kTX + 3); q += blockDim.x) {
      const int rq = q / (kTX + 3), c = q - rq * (kTX + 3);
      const int dz = DIM == 3 ? rq / 3 - 1 : 0, dy = DIM >= 2 ? rq % 3 - 1 : 0;
      const bool ok = cy + dy >= 0 && cy + dy < G.g[1] && cz + dz >= 0 && cz + dz < G.g[2];
      const int64_t rk = (row + (int64_t)dz * G.g[1] + dy) * G.g[0];
      if (c <= nspan) cstart[rq][c] = ok ? start[rk + xa + c] : 0;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      int tot = 0;
      for (int rq = 0; rq < NR; ++rq) {
        seg_base[rq] = tot;
        seg_g0[rq] = cstart[rq][0];
        tot += cstart[rq][nspan] - cstart[rq][0];
      }
      seg_base[NR] = tot;
    }
    __syncthreads();
    const bool staged = seg_base[NR] <= kLdsCand;
    if (staged) {
      for (int rq = 0; rq < NR; ++rq) {
        const int len = cstart[rq][nspan] - cstart[rq][0];
        for (int t = threadIdx.x; t < len; t += blockDim.x) cand[seg_base[rq] + t] = cpos[seg_g0[rq] + t];
      }
    }
    __syncthreads();
    // queries: the particles of the own cells (center row = index NR / 2)
    const int rc = NR / 2;
    const int qa = cstart[rc][x0 - xa], qb = cstart[rc][x1 - xa];
    for (int qi = qa + threadIdx.x; qi < qb; qi += blockDim.x) {
      const f32x4 me = staged ? cand[seg_base[rc] + (qi - seg_g0[rc])] : cpos[qi];
      const int i = __float_as_int(me[3]);
      const int cx = cell_of(me[0], G.lo[0], G.inv_cell, G.g[0]);
      int top[kMaxCap];
#pragma unroll
      for (int s = 0; s < kMaxCap; ++s) top[s] = INT32_MAX;
      int cnt = 0;
      for (int rq = 0; rq < NR; ++rq) {
        const int ca = max(cx - 1, xa) - xa, cb = min(cx + 1, xb) - xa;  // span-relative cells
        const int ja = cstart[rq][ca] - seg_g0[rq], jb = cstart[rq][cb + 1] - seg_g0[rq];
        for (int t = ja; t < jb; ++t) {
          const f32x4 c = staged ? cand[seg_base[rq] + t] : cpos[seg_g0[rq] + t];
          float s = 0.0f;  // fp32, dims summed in order, no contraction (oracle rule)
#pragma unroll
          for (int d = 0; d < DIM; ++d) {
#pragma clang fp contract(off)
            const float u = __fsub_rn(c[d], me[d]);
            s = __fadd_rn(s, __fmul_rn(u, u));
          }
          if (s < r2) {
            const int j = __float_as_int(c[3]);
            ++cnt;
            if (j < top[kMaxCap - 1]) sorted_insert(top, j);
          }
        }
      }
      cnt = min(cnt, cap);
      int32_t* out = nbr + (int64_t)i * cap;
      int w = 0;
      bool self_dropped = false;
#pragma unroll
      for (int s = 0; s < kMaxCap; ++s) {
        if (s < cnt) {
          const int v = top[s];
          if (!loop && v == i && !self_dropped) {  // torch_cluster: K+1 first-by-index, then drop self
            self_dropped = true;
          } else {
            out[w] = v;
            ++w;
          }
        }
      }
      deg[i] = w;
    }
  }
}

__global__ __launch_bounds__(256) void k_compact(int64_t n, int cap, const int32_t* nbr,
                                                 const int32_t* deg, const int32_t* rowptr,
                                                 int32_t* send, int32_t* recv) {
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t i = g / cap;
  const int t = (int)(g - i * cap);
  if (i >= n || t >= deg[i]) return;
  const int32_t e = rowptr[i] + t;
  send[e] = nbr[g];
  recv[e] = (int32_t)i;
}

// ---------------------------------------------------------------------------
// Small-graph path (n <= kSmallN, e.g. the 2k-particle Taylor bar): two
// launches instead of the cell pipeline's eleven (body in radius_small.h).
using sgnn::kSmallBlock;
using sgnn::kSmallN;

template <int DIM>
__global__ __launch_bounds__(kSmallBlock) void k_radius_small(sgnn::RadiusSmallArgs a) {
  extern __shared__ float lds[];
  sgnn::radius_small_body<DIM>(a, lds, blockIdx.x, gridDim.x);
}

// deg -> rowptr (exclusive scan, rowptr[n] = E) and the padded lists ->
// receiver-sorted CSR.  n <= kSmallN: every workgroup scans all of deg in LDS
// (8 rows per thread) -- cheaper than a grid-wide scan's extra launches --
// then copies the rows of its own 32-row slice (thread = (row, slot), slots
// t and t + 32 for caps up to 64); workgroup 0 writes rowptr.
__global__ __launch_bounds__(1024) void k_csr_small(int n, int cap, const int32_t* nbr,
                                                    const int32_t* deg, int32_t* rowptr,
                                                    int32_t* send, int32_t* recv) {
  __shared__ int32_t wsum[16];
  __shared__ int32_t srow[kSmallN + 1];
  const int base = threadIdx.x * 8;
  int32_t v[8], s = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    v[k] = base + k < n ? deg[base + k] : 0;
    s += v[k];
  }
  const int lane = lane_id(), w = wave_id();
  int32_t incl = s;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int32_t t = __shfl_up(incl, o, 64);
    if (lane >= o) incl += t;
  }
  if (lane == 63) wsum[w] = incl;
  __syncthreads();
  int32_t run = incl - s;
  for (int k = 0; k < w; ++k) run += wsum[k];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    if (base + k <= n) srow[base + k] = run;  // index n gets E (items past n add 0)
    run += v[k];
  }
  if (base + 8 == n) srow[n] = run;  // n == 8192: index n lies past every thread's range
  __syncthreads();
  if (blockIdx.x == 0)
    for (int i = threadIdx.x; i <= n; i += blockDim.x) rowptr[i] = srow[i];
  const int i = blockIdx.x * 32 + (threadIdx.x >> 5), t = threadIdx.x & 31;
  if (i < n) {
    const int r0 = srow[i], dg = srow[i + 1] - r0;
    for (int tt = t; tt < dg; tt += 32) {
      send[r0 + tt] = nbr[i * cap + tt];
      recv[r0 + tt] = i;
    }
  }
}

constexpr int kBboxBlocks = 128;

struct RadiusWs {
  uint32_t nbuckets;  // cell capacity (cells of all examples)
  int32_t *count, *fill, *start, *bucket_of, *ex_of, *order, *nbr, *deg, *partials;
  uint32_t *bbox, *bboxp;
  f32x4* cpos;  // [n] cell-ordered (x, y, z, id)
  size_t bytes;
};

size_t align_up(size_t x) { return (x + 255) & ~size_t(255); }

RadiusWs radius_layout(int64_t n, int32_t K, int32_t loop, void* base) {
  RadiusWs w{};
  uint32_t m = 1024;
  while ((int64_t)m < 2 * n) m <<= 1;
  w.nbuckets = m;
  const int cap = K + (loop ? 0 : 1);
  const int64_t nparts = std::max<int64_t>((m + 1 + kScanTile - 1) / kScanTile,
                                           (n + 1 + kScanTile - 1) / kScanTile) + 1;
  char* p = static_cast<char*>(base);
  size_t off = 0;
  auto take = [&](int64_t count) {
    int32_t* r = reinterpret_cast<int32_t*>(p + off);
    off += align_up(sizeof(int32_t) * (size_t)count);
    return r;
  };
  w.count = take(2 * (int64_t)m + 2);  // count[m+1], fill[m+1]: zeroed by k_bbox
  w.fill = w.count + m + 1;
  w.bbox = reinterpret_cast<uint32_t*>(take(16));                 // Grid at + 8
  w.bboxp = reinterpret_cast<uint32_t*>(take(8 * kBboxBlocks));   // k_bbox per-block partials
  w.start = take(m + 1);
  w.bucket_of = take(n);
  w.ex_of = take(n);
  w.order = take(n);
  w.cpos = reinterpret_cast<f32x4*>(take(4 * n));
  w.nbr = take(n * cap);
  w.deg = take(n + 1);
  w.partials = take(nparts);
  w.bytes = off;
  return w;
}

}  // namespace

namespace sgnn {

int scan_exclusive(const int32_t* in, int32_t* out, int64_t len, int32_t* partials,
                   hipStream_t stream) {
  if (len <= 0) return SGNN_OK;
  const int64_t nb = (len + kScanTile - 1) / kScanTile;
  if (nb > 8192) return set_error(SGNN_ERR_UNSUPPORTED, "scan: more than 16M elements");
  hipLaunchKernelGGL(k_scan_block, dim3((unsigned)nb), dim3(kScanBlock), 0, stream, in, out, len,
                     partials);
  if (nb > 1)
    hipLaunchKernelGGL(k_scan_add, dim3((unsigned)nb), dim3(kScanBlock), 0, stream, out, len,
                       partials);
  return check_launch("scan");
}

}  // namespace sgnn

namespace sgnn {

int radius_small_csr(const RadiusSmallArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(k_csr_small, dim3((unsigned)((a.n + 31) / 32)), dim3(1024), 0, s, a.n, a.cap, a.nbr,
                     a.deg, a.rowptr, a.send, a.recv);
  return check_launch("radius_graph(small csr)");
}

int radius_small_launch(const RadiusSmallArgs& a, hipStream_t s) {
  const unsigned grid = (unsigned)std::min<int64_t>((a.n + 7) / 8, 512);
  auto go = [&](auto kern) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)radius_small_lds(kSmallN, 3));
    hipLaunchKernelGGL(kern, dim3(grid), dim3(kSmallBlock), radius_small_lds(a.n, a.dim), s, a);
  };
  if (a.dim == 1) go(k_radius_small<1>);
  else if (a.dim == 2) go(k_radius_small<2>);
  else go(k_radius_small<3>);
  return radius_small_csr(a, s);
}

// The small path's arguments (workspace layout included) when sgnn_radius_graph
// would take it with these arguments; false otherwise (validation left to it).
bool radius_small_plan(const float* pos, int64_t pos_stride, int64_t n, int32_t dim, const int64_t* ex_ptr,
                       int32_t n_ex, float radius, int32_t K, int32_t loop, void* workspace, int32_t* rowptr,
                       int32_t* send, int32_t* recv, int64_t edge_cap, RadiusSmallArgs* out) {
  const int cap = K + (loop ? 0 : 1);
  if (n < 1 || n > kSmallN || dim < 1 || dim > 3 || n_ex < 1 || K < 1 || !(radius > 0.0f) || cap > 32 ||
      edge_cap < n * cap || !pos || !ex_ptr || !workspace || !rowptr || !send || !recv)
    return false;
  RadiusWs w = radius_layout(n, K, loop, workspace);
  *out = RadiusSmallArgs{pos, pos_stride, (int)n, dim, ex_ptr, n_ex, radius * radius, cap, loop, w.nbr, w.deg,
                         rowptr, send, recv};
  return true;
}

}  // namespace sgnn

extern "C" size_t sgnn_radius_workspace_bytes(int64_t n, int32_t K, int32_t loop) {
  return radius_layout(n, K, loop, nullptr).bytes;
}

extern "C" int sgnn_radius_graph(const float* pos, int64_t pos_stride, int64_t n, int32_t dim,
                                 const int64_t* ex_ptr, int32_t n_ex, float radius, int32_t K,
                                 int32_t loop, void* workspace, int32_t* rowptr, int32_t* send,
                                 int32_t* recv, int64_t edge_cap, void* stream_) {
  using namespace sgnn;
  hipStream_t stream = static_cast<hipStream_t>(stream_);
  const int cap = K + (loop ? 0 : 1);
  if (n < 0 || dim < 1 || dim > 3 || n_ex < 1 || K < 1 || !(radius > 0.0f))
    return set_error(SGNN_ERR_INVALID, "radius_graph: bad n/dim/n_ex/K/radius");
  if (cap > kRadiusMaxCap) return set_error(SGNN_ERR_UNSUPPORTED, "radius_graph: K (+1 without loop) > 64");
  if (edge_cap < n * cap) return set_error(SGNN_ERR_INVALID, "radius_graph: edge_cap < n*cap");
  if (n > (int64_t)1 << 26) return set_error(SGNN_ERR_UNSUPPORTED, "radius_graph: n > 2^26");
  if (n == 0) {
    (void)hipMemsetAsync(rowptr, 0, sizeof(int32_t), stream);
    return check_launch("radius_graph(n=0)");
  }
  if (!pos || !ex_ptr || !workspace || !rowptr || !send || !recv)
    return set_error(SGNN_ERR_INVALID, "radius_graph: null pointer");
  RadiusWs w = radius_layout(n, K, loop, workspace);
  const float r2 = radius * radius;
  if (n <= kSmallN) {  // small graphs: brute force over LDS in index order, two launches
    const RadiusSmallArgs a{pos, pos_stride, (int)n, dim, ex_ptr, n_ex, r2, cap, loop, w.nbr, w.deg,
                            rowptr, send, recv};
    return radius_small_launch(a, stream);
  }
  if ((int64_t)n_ex > (int64_t)w.nbuckets)
    return set_error(SGNN_ERR_UNSUPPORTED, "radius_graph: more examples than cell capacity (2n)");
  const float cell0 = radius * 1.01f;  // margin keeps |dp| < r inside +-1 cell under rounding
  const int64_t max_cells = w.nbuckets;
  const unsigned nblk = (unsigned)((n + 255) / 256);
  const unsigned bblk = std::min<unsigned>(nblk, kBboxBlocks);
#define SGNN_DIM_LAUNCH(K, GRID, ...)                                                                 \
  do {                                                                                             \
    if (dim == 1) hipLaunchKernelGGL(K<1>, dim3(GRID), dim3(256), 0, stream, __VA_ARGS__);          \
    else if (dim == 2) hipLaunchKernelGGL(K<2>, dim3(GRID), dim3(256), 0, stream, __VA_ARGS__);     \
    else hipLaunchKernelGGL(K<3>, dim3(GRID), dim3(256), 0, stream, __VA_ARGS__);                   \
  } while (0)
  SGNN_DIM_LAUNCH(k_bbox, bblk, pos, pos_stride, n, w.bboxp, w.count, 2 * (int64_t)w.nbuckets + 2);
  SGNN_DIM_LAUNCH(k_cell_assign, nblk, pos, pos_stride, n, ex_ptr, n_ex, w.bboxp, (int)bblk, cell0, max_cells,
                  w.bbox, w.bucket_of, w.ex_of, w.count);
  int st = scan_exclusive(w.count, w.start, (int64_t)w.nbuckets + 1, w.partials, stream);
  if (st) return st;
  SGNN_DIM_LAUNCH(k_cell_scatter, nblk, n, w.bucket_of, w.start, w.fill, w.order, pos, pos_stride, w.cpos);
#undef SGNN_DIM_LAUNCH
  // LDS-binned query over cell tiles (persistent grid: the tile count lives on the device)
  // about one tile per workgroup at lattice densities (~1.5 particles per cell, 64-cell tiles)
  const unsigned qgrid = (unsigned)std::min<int64_t>(std::max<int64_t>((n + 63) / 64, 1), 4096);
  auto query = [&](auto kern) {
    hipLaunchKernelGGL(kern, dim3(qgrid), dim3(kQBlock), 0, stream, w.cpos, w.start, w.bbox, n_ex, r2, cap, loop,
                       w.nbr, w.deg, n);
  };
  if (cap <= 32) {
    if (dim == 1) query(k_radius_query_lds<1, 32>);
    else if (dim == 2) query(k_radius_query_lds<2, 32>);
    else query(k_radius_query_lds<3, 32>);
  } else {
    if (dim == 1) query(k_radius_query_lds<1, kRadiusMaxCap>);
    else if (dim == 2) query(k_radius_query_lds<2, kRadiusMaxCap>);
    else query(k_radius_query_lds<3, kRadiusMaxCap>);
  }
  st = scan_exclusive(w.deg, rowptr, n + 1, w.partials, stream);
  if (st) return st;
  const int64_t tot = n * cap;
  hipLaunchKernelGGL(k_compact, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, stream, n, cap,
                     w.nbr, w.deg, rowptr, send, recv);
  return check_launch("radius_graph");
}

// ---------------------------------------------------------------------------
// Static graphs (multi-scale g2m / m2m / m2g, sgnn/multi_scale/
// multi_scale_graph.py:193-281): COO edge_index [2][E] (int64, row 0 =
// sender j, row 1 = receiver i, PyG flow source_to_target) -> the receiver-
// sorted CSR the layer kernels consume.  Stable: within a receiver, edges keep
// their original order, i.e. the order PyG's scatter-add sums them in.
namespace {

__global__ __launch_bounds__(256) void k_coo_count(const int64_t* dst, int64_t E, int32_t* cnt) {
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < E;
       e += (int64_t)gridDim.x * blockDim.x)
    atomicAdd(&cnt[dst[e]], 1);
}

__global__ __launch_bounds__(256) void k_coo_fill(const int64_t* dst, int64_t E, const int32_t* ptr,
                                                  int32_t* fill, int32_t* raw) {
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < E;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t d = dst[e];
    raw[ptr[d] + atomicAdd(&fill[d], 1)] = (int32_t)e;
  }
}

// one wave per receiver: rank = number of smaller edge ids in its segment
__global__ __launch_bounds__(256) void k_coo_sort(const int32_t* ptr, int64_t n, const int32_t* raw,
                                                  const int64_t* src, const int64_t* dst,
                                                  int32_t* send, int32_t* recv, int32_t* perm) {
  const int64_t i = (int64_t)blockIdx.x * (blockDim.x >> 6) + wave_id();
  if (i >= n) return;
  const int lane = threadIdx.x & 63;
  const int32_t b = ptr[i], len = ptr[i + 1] - b;
  for (int q = lane; q < len; q += 64) {
    const int32_t key = raw[b + q];
    int rank = 0;
    for (int t = 0; t < len; ++t) rank += raw[b + t] < key;
    send[b + rank] = (int32_t)src[key];
    recv[b + rank] = (int32_t)dst[key];
    if (perm) perm[b + rank] = key;
  }
}

}  // namespace

extern "C" size_t sgnn_coo_workspace_bytes(int64_t n, int64_t E) {
  return sizeof(int32_t) * (size_t)(2 * (n + 1) + E) + 3 * 256 + 65536;
}

extern "C" int sgnn_coo_to_csr(const int64_t* src, const int64_t* dst, int64_t E, int64_t n,
                               void* workspace, int32_t* rowptr, int32_t* send, int32_t* recv,
                               int32_t* perm, void* stream_) {
  using namespace sgnn;
  hipStream_t s = static_cast<hipStream_t>(stream_);
  if (n <= 0 || E < 0 || !rowptr || !workspace || (E > 0 && (!src || !dst || !send || !recv)))
    return set_error(SGNN_ERR_INVALID, "coo_to_csr: bad arguments");
  if (E >= ((int64_t)1 << 31)) return set_error(SGNN_ERR_UNSUPPORTED, "coo_to_csr: E >= 2^31");
  char* p = static_cast<char*>(workspace);
  auto take = [&](size_t bytes) {
    char* r = p;
    p += (bytes + 255) & ~size_t(255);
    return r;
  };
  int32_t* cnt = reinterpret_cast<int32_t*>(take(sizeof(int32_t) * 2 * (n + 1)));
  int32_t* fill = cnt + (n + 1);
  int32_t* raw = reinterpret_cast<int32_t*>(take(sizeof(int32_t) * (E > 0 ? E : 1)));
  int32_t* partials = reinterpret_cast<int32_t*>(take(65536 - 512));
  (void)hipMemsetAsync(cnt, 0, sizeof(int32_t) * 2 * (n + 1), s);
  const unsigned g = (unsigned)std::max<int64_t>(1, std::min<int64_t>((E + 255) / 256, 2048));
  if (E > 0) hipLaunchKernelGGL(k_coo_count, dim3(g), dim3(256), 0, s, dst, E, cnt);
  int st = scan_exclusive(cnt, rowptr, n + 1, partials, s);
  if (st) return st;
  if (E > 0) {
    hipLaunchKernelGGL(k_coo_fill, dim3(g), dim3(256), 0, s, dst, E, rowptr, fill, raw);
    hipLaunchKernelGGL(k_coo_sort, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, s, rowptr, n, raw,
                       src, dst, send, recv, perm);
  }
  return check_launch("coo_to_csr");
}
