// Radius-graph neighbour search for gfx950 (replaces torch_cluster.radius as
// reached by sgnn/single_scale/learned_simulator.py:116-117).
//
// Pipeline (5-9 launches, no host sync, capturable in a hipGraph):
//   1. k_cell_assign   particle -> (example, cell = floor(p / (1.01 r))) ->
//                      hash bucket; histogram with one atomic per particle
//   2. scan            bucket counts -> bucket starts
//   3. k_cell_scatter  counting-sort particle ids into bucket order
//   4. k_radius_query  one wave per query particle: walks the 3^d neighbour
//                      cells (each a contiguous bucket span, 64 candidates per
//                      wave step, coalesced id loads), keeps in-range
//                      same-example candidates, and maintains the `cap`
//                      smallest sender ids with a 64-lane bitonic sort +
//                      merge in registers (torch_cluster's CUDA rule: first K
//                      in ascending index).  Writes deg and a padded list.
//   5. scan            deg -> rowptr (rowptr[n] = E, left on the device)
//   6. k_compact       padded lists -> receiver-sorted CSR (send, recv)
#include "common.h"
#include "../../include/sgnn.h"
#include "sgnn_internal.h"

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
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
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

// Exclusive scan of up to 1024*8 block totals in one block.
__global__ __launch_bounds__(1024) void k_scan_partials(int32_t* partials, int nb) {
  __shared__ int32_t wsum[16];
  const int base = threadIdx.x * 8;
  int32_t v[8], s = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    v[k] = base + k < nb ? partials[base + k] : 0;
    s += v[k];
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
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
  for (int k = 0; k < 8; ++k) {
    if (base + k < nb) partials[base + k] = run;
    run += v[k];
  }
}

__global__ __launch_bounds__(kScanBlock) void k_scan_add(int32_t* out, int64_t len,
                                                         const int32_t* partials) {
  const int32_t add = partials[blockIdx.x];
  const int64_t base = (int64_t)blockIdx.x * kScanTile;
  for (int k = threadIdx.x; k < kScanTile; k += blockDim.x) {
    const int64_t i = base + k;
    if (i < len) out[i] += add;
  }
}

SGNN_DEV int cell_coord(float x, float inv_cell) {
  float q = floorf(x * inv_cell);
  if (!(q == q)) q = 0.0f;
  q = fminf(fmaxf(q, -1048576.0f), 1048576.0f);
  return (int)q;
}

SGNN_DEV uint32_t cell_hash(int cx, int cy, int cz, int ex, uint32_t mask) {
  uint32_t h = (uint32_t)cx * 0x9E3779B1u + (uint32_t)cy * 0x85EBCA77u + (uint32_t)cz * 0xC2B2AE3Du +
               (uint32_t)ex * 0x27D4EB2Fu;
  h ^= h >> 15;
  h *= 0x2C1B3C6Du;
  h ^= h >> 12;
  h *= 0x297A2D39u;
  h ^= h >> 15;
  return h & mask;
}

SGNN_DEV float dist2_ordered(const float* a, const float* b, int dim) {
  // fp32, dims summed in order, no contraction: matches the oracle / golden rule.
  float s = 0.0f;
  for (int d = 0; d < dim; ++d) {
    const float t = __fsub_rn(a[d], b[d]);
    s = __fadd_rn(s, __fmul_rn(t, t));
  }
  return s;
}

__global__ __launch_bounds__(256) void k_cell_assign(const float* pos, int64_t stride, int64_t n,
                                                     int dim, const int64_t* ex_ptr, int n_ex,
                                                     float inv_cell, uint32_t mask,
                                                     int32_t* bucket_of, int32_t* ex_of,
                                                     int32_t* count) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  int lo = 0, hi = n_ex - 1;  // largest b with ex_ptr[b] <= i
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (ex_ptr[mid] <= i) lo = mid; else hi = mid - 1;
  }
  const float* p = pos + i * stride;
  const int cx = cell_coord(p[0], inv_cell);
  const int cy = dim > 1 ? cell_coord(p[1], inv_cell) : 0;
  const int cz = dim > 2 ? cell_coord(p[2], inv_cell) : 0;
  const uint32_t b = cell_hash(cx, cy, cz, lo, mask);
  bucket_of[i] = (int32_t)b;
  ex_of[i] = lo;
  atomicAdd(&count[b], 1);
}

__global__ __launch_bounds__(256) void k_cell_scatter(int64_t n, const int32_t* bucket_of,
                                                      const int32_t* start, int32_t* fill,
                                                      int32_t* order) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int32_t b = bucket_of[i];
  order[start[b] + atomicAdd(&fill[b], 1)] = (int32_t)i;
}

SGNN_DEV int bitonic_sort64(int key, int lane) {
#pragma unroll
  for (int k = 2; k <= 64; k <<= 1) {
#pragma unroll
    for (int j = k >> 1; j > 0; j >>= 1) {
      const int other = __shfl_xor(key, j, 64);
      const bool up = (lane & k) == 0;
      const bool lower = (lane & j) == 0;
      key = (lower == up) ? min(key, other) : max(key, other);
    }
  }
  return key;
}

SGNN_DEV int bitonic_merge64(int key, int lane) {
#pragma unroll
  for (int j = 32; j > 0; j >>= 1) {
    const int other = __shfl_xor(key, j, 64);
    key = ((lane & j) == 0) ? min(key, other) : max(key, other);
  }
  return key;
}

__global__ __launch_bounds__(256) void k_radius_query(
    const float* pos, int64_t stride, int64_t n, int dim, float r2, float inv_cell,
    uint32_t mask, const int32_t* ex_of, const int32_t* start, const int32_t* order, int cap,
    int loop, int32_t* nbr, int32_t* deg) {
  const int lane = threadIdx.x & 63;
  const int64_t i = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (i == 0 && lane == 0) deg[n] = 0;  // scan sentinel -> rowptr[n] = E
  if (i >= n) return;
  float pi[3] = {0.0f, 0.0f, 0.0f};
  for (int d = 0; d < dim; ++d) pi[d] = pos[i * stride + d];
  const int ex = ex_of[i];
  int ci[3] = {cell_coord(pi[0], inv_cell), dim > 1 ? cell_coord(pi[1], inv_cell) : 0,
               dim > 2 ? cell_coord(pi[2], inv_cell) : 0};
  int top = INT32_MAX;  // lanes [0, cnt) hold the kept ids, ascending
  int cnt = 0;
  const int zr = dim > 2 ? 1 : 0, yr = dim > 1 ? 1 : 0;
  for (int dz = -zr; dz <= zr; ++dz)
    for (int dy = -yr; dy <= yr; ++dy)
      for (int dx = -1; dx <= 1; ++dx) {
        const int tc[3] = {ci[0] + dx, ci[1] + dy, ci[2] + dz};
        const uint32_t b = cell_hash(tc[0], tc[1], tc[2], ex, mask);
        const int s0 = start[b], s1 = start[b + 1];
        for (int base = s0; base < s1; base += 64) {
          const int t = base + lane;
          int key = INT32_MAX;
          if (t < s1) {
            const int j = order[t];
            if (ex_of[j] == ex) {
              float pj[3] = {0.0f, 0.0f, 0.0f};
              for (int d = 0; d < dim; ++d) pj[d] = pos[(int64_t)j * stride + d];
              bool same_cell = true;
              for (int d = 0; d < dim; ++d) same_cell &= cell_coord(pj[d], inv_cell) == tc[d];
              if (same_cell && dist2_ordered(pj, pi, dim) < r2) key = j;
            }
          }
          if (cnt >= cap) {
            const int kth = __shfl(top, cap - 1, 64);
            if (key >= kth) key = INT32_MAX;
          }
          const unsigned long long bal = __ballot(key != INT32_MAX);
          if (bal) {
            const int nnew = __popcll(bal);
            key = bitonic_sort64(key, lane);
            const int other = __shfl(key, 63 - lane, 64);
            top = bitonic_merge64(min(top, other), lane);
            if (lane >= cap) top = INT32_MAX;
            cnt = min(cnt + nnew, cap);
          }
        }
      }
  if (!loop) {  // torch_cluster: K+1 nearest-by-index, then drop the self loop
    const unsigned long long self = __ballot(lane < cnt && top == (int)i);
    if (self) {
      const int at = __ffsll((long long)self) - 1;
      const int nxt = __shfl(top, (lane + 1) & 63, 64);
      if (lane >= at) top = (lane + 1 < cnt) ? nxt : INT32_MAX;
      cnt -= 1;
    }
  }
  if (lane < cnt) nbr[i * cap + lane] = top;
  if (lane == 0) deg[i] = cnt;
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

struct RadiusWs {
  uint32_t nbuckets;
  int32_t *count, *fill, *start, *bucket_of, *ex_of, *order, *nbr, *deg, *partials;
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
  w.count = take(2 * (int64_t)m + 2);  // count[m+1] and fill[m+1]: one memset
  w.fill = w.count + m + 1;
  w.start = take(m + 1);
  w.bucket_of = take(n);
  w.ex_of = take(n);
  w.order = take(n);
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
  if (nb > 1) {
    hipLaunchKernelGGL(k_scan_partials, dim3(1), dim3(1024), 0, stream, partials, (int)nb);
    hipLaunchKernelGGL(k_scan_add, dim3((unsigned)nb), dim3(kScanBlock), 0, stream, out, len,
                       partials);
  }
  return check_launch("scan");
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
  if (cap > 32) return set_error(SGNN_ERR_UNSUPPORTED, "radius_graph: K (+1 without loop) > 32");
  if (edge_cap < n * cap) return set_error(SGNN_ERR_INVALID, "radius_graph: edge_cap < n*cap");
  if (n > (int64_t)1 << 26) return set_error(SGNN_ERR_UNSUPPORTED, "radius_graph: n > 2^26");
  if (n == 0) {
    (void)hipMemsetAsync(rowptr, 0, sizeof(int32_t), stream);
    return check_launch("radius_graph(n=0)");
  }
  if (!pos || !ex_ptr || !workspace || !rowptr || !send || !recv)
    return set_error(SGNN_ERR_INVALID, "radius_graph: null pointer");
  RadiusWs w = radius_layout(n, K, loop, workspace);
  const float cell = radius * 1.01f;  // margin keeps |dp| < r inside +-1 cell under rounding
  const float inv_cell = 1.0f / cell;
  const float r2 = radius * radius;
  const unsigned nblk = (unsigned)((n + 255) / 256);
  (void)hipMemsetAsync(w.count, 0, sizeof(int32_t) * (2 * (size_t)w.nbuckets + 2), stream);
  hipLaunchKernelGGL(k_cell_assign, dim3(nblk), dim3(256), 0, stream, pos, pos_stride, n, dim,
                     ex_ptr, n_ex, inv_cell, w.nbuckets - 1, w.bucket_of, w.ex_of, w.count);
  int st = scan_exclusive(w.count, w.start, (int64_t)w.nbuckets + 1, w.partials, stream);
  if (st) return st;
  hipLaunchKernelGGL(k_cell_scatter, dim3(nblk), dim3(256), 0, stream, n, w.bucket_of, w.start,
                     w.fill, w.order);
  hipLaunchKernelGGL(k_radius_query, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, stream, pos,
                     pos_stride, n, dim, r2, inv_cell, w.nbuckets - 1, w.ex_of, w.start, w.order,
                     cap, loop, w.nbr, w.deg);
  st = scan_exclusive(w.deg, rowptr, n + 1, w.partials, stream);
  if (st) return st;
  const int64_t tot = n * cap;
  hipLaunchKernelGGL(k_compact, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, stream, n, cap,
                     w.nbr, w.deg, rowptr, send, recv);
  return check_launch("radius_graph");
}
