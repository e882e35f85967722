/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load this; the product path never does.
 *
 * CPU restatement of the neighbour search the reference reaches through
 * `torch_geometric.nn.radius_graph(positions, r=R, batch=batch_ids,
 * loop=True, max_num_neighbors=20)` (sgnn/single_scale/learned_simulator.py:
 * 104-117) -> torch_cluster.radius (third-party, un-vendored; torch_cluster
 * 1.6.x as pinned only by README.md:23 "data.pyg.org/whl/torch-2.5.0+cu118").
 *
 * Semantics restated (torch_cluster's CUDA kernel):
 *   for each query i (ascending), candidates j of the SAME example in
 *   ascending index, hit iff sum_d (x_j[d]-x_i[d])^2 < r*r evaluated in fp32
 *   with the dims summed in order (no FMA contraction: build with
 *   -ffp-contract=off); keep the first `cap` hits where cap = K if loop else
 *   K+1, then drop the self hit when loop == 0.  Output: receiver-sorted edge
 *   list, senders ascending; edge_index = [sender j ; receiver i].
 * Pinned against tests/golden/*.npz (generated from the reference).
 *
 * Two implementations, same result:
 *   oracle_radius_bruteforce  O(N^2) per example - the literal rule
 *   oracle_radius_cells       uniform cell list + per-query ascending sort,
 *                             the complexity class of torch_cluster's CPU
 *                             KD-tree path (used as the CPU baseline).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

static float d2_fp32(const float* a, const float* b, int dim) {
  float s = 0.0f;
  for (int d = 0; d < dim; ++d) {
    float t = a[d] - b[d];
    float sq = t * t;
    s = s + sq;
  }
  return s;
}

static int cmp_i64(const void* a, const void* b) {
  int64_t x = *(const int64_t*)a, y = *(const int64_t*)b;
  return (x > y) - (x < y);
}

/* returns number of edges written, or -1 if `max_edges` would overflow */
int64_t oracle_radius_bruteforce(const float* pos, int64_t n, int dim, const int64_t* ex_ptr,
                                 int n_ex, float r, int K, int loop, int64_t* send,
                                 int64_t* recv, int64_t max_edges) {
  const float r2 = r * r;
  const int cap = loop ? K : K + 1;
  int64_t e = 0;
  for (int ex = 0; ex < n_ex; ++ex) {
    for (int64_t i = ex_ptr[ex]; i < ex_ptr[ex + 1]; ++i) {
      int taken = 0;
      for (int64_t j = ex_ptr[ex]; j < ex_ptr[ex + 1] && taken < cap; ++j) {
        if (d2_fp32(pos + j * dim, pos + i * dim, dim) < r2) {
          ++taken;
          if (!loop && j == i) continue;
          if (e >= max_edges) return -1;
          send[e] = j;
          recv[e] = i;
          ++e;
        }
      }
    }
  }
  (void)n;
  return e;
}

int64_t oracle_radius_cells(const float* pos, int64_t n, int dim, const int64_t* ex_ptr,
                            int n_ex, float r, int K, int loop, int64_t* send, int64_t* recv,
                            int64_t max_edges) {
  const float r2 = r * r;
  const int cap = loop ? K : K + 1;
  int64_t e = 0;
  int64_t* hits = NULL;
  int64_t hits_cap = 0;
  for (int ex = 0; ex < n_ex; ++ex) {
    const int64_t b = ex_ptr[ex], m = ex_ptr[ex + 1] - b;
    if (m <= 0) continue;
    double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (int64_t i = 0; i < m; ++i)
      for (int d = 0; d < dim; ++d) {
        double v = pos[(b + i) * dim + d];
        if (v < lo[d]) lo[d] = v;
        if (v > hi[d]) hi[d] = v;
      }
    double cell = r > 0 ? (double)r : 1.0;
    int64_t g[3] = {1, 1, 1}, ncell;
    for (;;) {
      ncell = 1;
      for (int d = 0; d < dim; ++d) {
        double ext = hi[d] - lo[d];
        g[d] = (isfinite(ext) ? (int64_t)(ext / cell) : 0) + 1;
        ncell *= g[d];
      }
      if (ncell <= 8 * m + 64) break;
      cell *= 2.0;
    }
    int64_t* cid = (int64_t*)malloc(sizeof(int64_t) * m);
    int64_t* start = (int64_t*)calloc(ncell + 1, sizeof(int64_t));
    int64_t* order = (int64_t*)malloc(sizeof(int64_t) * m);
    for (int64_t i = 0; i < m; ++i) {
      int64_t c = 0;
      for (int d = dim - 1; d >= 0; --d) {
        double v = pos[(b + i) * dim + d];
        int64_t q = isfinite(v) ? (int64_t)((v - lo[d]) / cell) : 0;
        if (q < 0) q = 0;
        if (q >= g[d]) q = g[d] - 1;
        c = c * g[d] + q;
      }
      cid[i] = c;
      start[c + 1]++;
    }
    for (int64_t c = 0; c < ncell; ++c) start[c + 1] += start[c];
    {
      int64_t* fill = (int64_t*)calloc(ncell, sizeof(int64_t));
      for (int64_t i = 0; i < m; ++i) order[start[cid[i]] + fill[cid[i]]++] = i;
      free(fill);
    }
    for (int64_t i = 0; i < m; ++i) {
      int64_t nh = 0;
      int64_t q[3] = {0, 0, 0};
      {
        int64_t c = cid[i];
        for (int d = 0; d < dim; ++d) { q[d] = c % g[d]; c /= g[d]; }
      }
      int64_t lo3[3] = {0, 0, 0}, hi3[3] = {0, 0, 0};
      for (int d = 0; d < dim; ++d) {
        lo3[d] = q[d] > 0 ? q[d] - 1 : 0;
        hi3[d] = q[d] + 1 < g[d] ? q[d] + 1 : g[d] - 1;
      }
      for (int64_t z = lo3[2]; z <= hi3[2]; ++z)
        for (int64_t y = lo3[1]; y <= hi3[1]; ++y)
          for (int64_t x = lo3[0]; x <= hi3[0]; ++x) {
            int64_t c = x + g[0] * (y + g[1] * z);
            for (int64_t t = start[c]; t < start[c + 1]; ++t) {
              int64_t j = order[t];
              if (d2_fp32(pos + (b + j) * dim, pos + (b + i) * dim, dim) < r2) {
                if (nh == hits_cap) {
                  hits_cap = hits_cap ? 2 * hits_cap : 256;
                  hits = (int64_t*)realloc(hits, sizeof(int64_t) * hits_cap);
                }
                hits[nh++] = j;
              }
            }
          }
      qsort(hits, (size_t)nh, sizeof(int64_t), cmp_i64);
      if (nh > cap) nh = cap;
      for (int64_t t = 0; t < nh; ++t) {
        if (!loop && hits[t] == i) continue;
        if (e >= max_edges) { free(cid); free(start); free(order); free(hits); return -1; }
        send[e] = b + hits[t];
        recv[e] = b + i;
        ++e;
      }
    }
    free(cid);
    free(start);
    free(order);
  }
  free(hits);
  (void)n;
  return e;
}
