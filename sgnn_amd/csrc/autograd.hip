// Width-generic differentiable building blocks (include/sgnn.h, "Width-generic
// differentiable building blocks"): an MFMA fp32 GEMM with a fused bias / ReLU
// epilogue and deterministic split-K, LayerNorm forward / backward, column
// sums, the ReLU mask, and the row gathers / CSR segment sums a message-passing
// block and its backward are made of.  sgnn_amd/autograd.py composes them into
// torch.autograd.Functions: build_mlp (+ LayerNorm) of any widths and depth
// (graph_network.py:7-45), the edge gather cat([x_i, x_j, e]) (:197) and the
// receiver sum (aggr='add', :136) -- so every module of the reference is
// differentiable on the GPU at every shape, not only at the widths the fused
// kernels are instantiated for.
#include "../../include/sgnn.h"
#include "common.h"
#include "sgnn_internal.h"

namespace {

constexpr int kTile = 64;    // output tile (M and N) per workgroup
constexpr int kKc = 16;      // K per LDS stage (8 MFMAs of k = 2)
constexpr int kLdT = kTile + 4;
constexpr int kGemmThreads = 256;
constexpr int kMaxSplit = 64;
constexpr int kEw = 256;     // threads of the elementwise kernels

struct GemmArgs {
  const float *A, *B, *bias;
  int64_t lda, ldb, ldc, M, N, K;
  float* C;
  float* part;   // split-K partial tiles [split][M][N] (null: one split, epilogue in place)
  int ta, tb, relu, accumulate;
  int64_t nkc;   // K chunks of kKc
};

// op(A)[m][k] and op(B)[k][n] into LDS as As[k][m], Bs[k][n] (zero outside the matrix).  Each thread
// moves four elements along the operand's contiguous dimension.
SGNN_DEV void stage_a(float* As, const GemmArgs& g, int64_t m0, int64_t k0) {
  const int t = threadIdx.x;
  if (!g.ta) {  // A [M][K]: k contiguous
    const int m = t >> 2, kq = (t & 3) * 4;
    const int64_t gm = m0 + m;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int64_t gk = k0 + kq + c;
      As[(kq + c) * kLdT + m] = (gm < g.M && gk < g.K) ? g.A[gm * g.lda + gk] : 0.0f;
    }
  } else {      // A stored [K][M]: m contiguous
    const int k = t >> 4, mq = (t & 15) * 4;
    const int64_t gk = k0 + k;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int64_t gm = m0 + mq + c;
      As[k * kLdT + mq + c] = (gm < g.M && gk < g.K) ? g.A[gk * g.lda + gm] : 0.0f;
    }
  }
}

SGNN_DEV void stage_b(float* Bs, const GemmArgs& g, int64_t n0, int64_t k0) {
  const int t = threadIdx.x;
  if (!g.tb) {  // B [K][N]: n contiguous
    const int k = t >> 4, nq = (t & 15) * 4;
    const int64_t gk = k0 + k;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int64_t gn = n0 + nq + c;
      Bs[k * kLdT + nq + c] = (gn < g.N && gk < g.K) ? g.B[gk * g.ldb + gn] : 0.0f;
    }
  } else {      // B stored [N][K]: k contiguous
    const int n = t >> 2, kq = (t & 3) * 4;
    const int64_t gn = n0 + n;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int64_t gk = k0 + kq + c;
      Bs[(kq + c) * kLdT + n] = (gn < g.N && gk < g.K) ? g.B[gn * g.ldb + gk] : 0.0f;
    }
  }
}

SGNN_DEV float epilogue(const GemmArgs& g, float v, int64_t m, int64_t n) {
  if (g.accumulate) v += g.C[m * g.ldc + n];
  if (g.bias) v += g.bias[n];
  return g.relu ? fmaxf(v, 0.0f) : v;
}

// Workgroup (bx, by, split): the 64 x 64 tile of C at (bx * 64, by * 64) over this split's K chunks.
// Waves in a 2 x 2 grid, each one 32 x 32 accumulator: lane l holds column (l & 31), register r row
// crow(r, l >> 5) (common.h).
__global__ __launch_bounds__(kGemmThreads) void k_gemm(GemmArgs g) {
  __shared__ float As[kKc * kLdT];
  __shared__ float Bs[kKc * kLdT];
  const int l = lane_id(), w = wave_id();
  const int wm = w >> 1, wn = w & 1;
  // row tiles on grid.x (2^31 - 1: edge-row GEMMs of any graph), column tiles on grid.y
  const int64_t m0 = (int64_t)blockIdx.x * kTile, n0 = (int64_t)blockIdx.y * kTile;
  const int split = blockIdx.z, nsplit = gridDim.z;
  const int64_t c0 = g.nkc * split / nsplit, c1 = g.nkc * (split + 1) / nsplit;
  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.0f;
  for (int64_t c = c0; c < c1; ++c) {
    stage_a(As, g, m0, c * kKc);
    stage_b(Bs, g, n0, c * kKc);
    __syncthreads();
#pragma unroll
    for (int s = 0; s < kKc / 2; ++s) {
      const int k = 2 * s + (l >> 5);
      acc = mfma32(As[k * kLdT + wm * 32 + (l & 31)], Bs[k * kLdT + wn * 32 + (l & 31)], acc);
    }
    __syncthreads();
  }
  const int64_t n = n0 + wn * 32 + (l & 31);
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int64_t m = m0 + wm * 32 + crow(r, l >> 5);
    if (m >= g.M || n >= g.N) continue;
    if (g.part) g.part[((int64_t)split * g.M + m) * g.N + n] = acc[r];
    else g.C[m * g.ldc + n] = epilogue(g, acc[r], m, n);
  }
}

// Split-K partials summed in split order, then the epilogue.
__global__ __launch_bounds__(kEw) void k_gemm_reduce(GemmArgs g, int nsplit) {
  const int64_t total = g.M * g.N;
  for (int64_t t = (int64_t)blockIdx.x * kEw + threadIdx.x; t < total; t += (int64_t)gridDim.x * kEw) {
    float v = 0.0f;
    for (int s = 0; s < nsplit; ++s) v += g.part[(int64_t)s * total + t];
    const int64_t m = t / g.N, n = t - m * g.N;
    g.C[m * g.ldc + n] = epilogue(g, v, m, n);
  }
}

// Splits of K for this shape: enough workgroups to fill the chip (~2 per CU), each split >= 4 K chunks.
int gemm_splits(int64_t M, int64_t N, int64_t K) {
  const int64_t tiles = ((M + kTile - 1) / kTile) * ((N + kTile - 1) / kTile);
  const int64_t nkc = (K + kKc - 1) / kKc;
  int64_t s = (512 + tiles - 1) / tiles;
  s = std::min<int64_t>(s, std::max<int64_t>(1, nkc / 4));
  return (int)std::max<int64_t>(1, std::min<int64_t>(s, kMaxSplit));
}

unsigned ew_grid(int64_t items) {
  return (unsigned)std::max<int64_t>(1, std::min<int64_t>((items + kEw - 1) / kEw, 4096));
}

// One wave per row: mean, biased variance (two passes over the row), affine, residual.
__global__ __launch_bounds__(kEw) void k_layernorm(const float* x, int64_t n, int width, const float* gamma,
                                                   const float* beta, const float* residual, float* out, float* yhat,
                                                   float* rstd_out) {
  const int l = lane_id();
  const int64_t nw = (int64_t)gridDim.x * (kEw / 64);
  for (int64_t r = (int64_t)blockIdx.x * (kEw / 64) + wave_id(); r < n; r += nw) {
    const float* y = x + r * width;
    float s = 0.0f;
    for (int c = l; c < width; c += 64) s += y[c];
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) s += __shfl_xor(s, o, 64);
    const float mean = s / width;
    float v = 0.0f;
    for (int c = l; c < width; c += 64) {
      const float d = y[c] - mean;
      v += d * d;
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
    const float rstd = 1.0f / sqrtf(v / width + 1e-5f);
    for (int c = l; c < width; c += 64) {
      const float yh = (y[c] - mean) * rstd;
      if (yhat) yhat[r * width + c] = yh;
      float o = yh * gamma[c] + beta[c];
      if (residual) o += residual[r * width + c];
      out[r * width + c] = o;
    }
    if (rstd_out && l == 0) rstd_out[r] = rstd;
  }
}

__global__ __launch_bounds__(kEw) void k_layernorm_bwd(const float* dout, const float* yhat, const float* rstd,
                                                       const float* gamma, int64_t n, int width, float* dx) {
  const int l = lane_id();
  const int64_t nw = (int64_t)gridDim.x * (kEw / 64);
  for (int64_t r = (int64_t)blockIdx.x * (kEw / 64) + wave_id(); r < n; r += nw) {
    float sg = 0.0f, sgy = 0.0f;
    for (int c = l; c < width; c += 64) {
      const float gc = dout[r * width + c] * gamma[c];
      sg += gc;
      sgy += gc * yhat[r * width + c];
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
      sg += __shfl_xor(sg, o, 64);
      sgy += __shfl_xor(sgy, o, 64);
    }
    const float mg = sg / width, mgy = sgy / width, rs = rstd[r];
    for (int c = l; c < width; c += 64) {
      const float gc = dout[r * width + c] * gamma[c];
      dx[r * width + c] = rs * (gc - mg - yhat[r * width + c] * mgy);
    }
  }
}

constexpr int kColRows = 256;   // rows per column-sum block

// partial[b][c] = sum over rows [b * 256, b * 256 + 256) in order of x[r][c] (* mul[r][c])
__global__ __launch_bounds__(kEw) void k_colsum_part(const float* x, int64_t ldx, const float* mul, int64_t ldm,
                                                     int64_t n, int width, float* partial) {
  const int64_t r0 = (int64_t)blockIdx.x * kColRows, r1 = min(r0 + kColRows, n);
  for (int c = threadIdx.x; c < width; c += kEw) {
    float s = 0.0f;
    for (int64_t r = r0; r < r1; ++r) s += mul ? x[r * ldx + c] * mul[r * ldm + c] : x[r * ldx + c];
    partial[(int64_t)blockIdx.x * width + c] = s;
  }
}

__global__ __launch_bounds__(kEw) void k_colsum_reduce(const float* partial, int64_t nblk, int width, float* out,
                                                       int accumulate) {
  for (int c = blockIdx.x * kEw + threadIdx.x; c < width; c += gridDim.x * kEw) {
    float s = 0.0f;
    for (int64_t b = 0; b < nblk; ++b) s += partial[b * width + c];
    out[c] = accumulate ? out[c] + s : s;
  }
}

__global__ __launch_bounds__(kEw) void k_relu_bwd(float* dy, int64_t ldd, const float* y, int64_t ldy, int64_t n,
                                                  int width) {
  const int64_t total = n * width;
  for (int64_t t = (int64_t)blockIdx.x * kEw + threadIdx.x; t < total; t += (int64_t)gridDim.x * kEw) {
    const int64_t r = t / width, c = t - r * width;
    if (!(y[r * ldy + c] > 0.0f)) dy[r * ldd + c] = 0.0f;
  }
}

__global__ __launch_bounds__(kEw) void k_gather_rows(const float* src, int64_t ld_src, int width, const int32_t* index,
                                                     int64_t nrows, float scale, float* out, int64_t ld_out) {
  const int64_t total = nrows * width;
  for (int64_t t = (int64_t)blockIdx.x * kEw + threadIdx.x; t < total; t += (int64_t)gridDim.x * kEw) {
    const int64_t r = t / width, c = t - r * width;
    const int64_t row = index ? (int64_t)index[r] : r;
    out[r * ld_out + c] = scale * src[row * ld_src + c];
  }
}

__global__ __launch_bounds__(kEw) void k_segment_sum_cols(const float* src, int64_t ld_src, int width,
                                                          const int32_t* rowptr, const int32_t* perm, int64_t n,
                                                          float scale, float* out, int64_t ld_out, int accumulate) {
  const int64_t total = n * width;
  for (int64_t t = (int64_t)blockIdx.x * kEw + threadIdx.x; t < total; t += (int64_t)gridDim.x * kEw) {
    const int64_t i = t / width, c = t - i * width;
    float s = 0.0f;
    for (int32_t p = rowptr[i]; p < rowptr[i + 1]; ++p) s += src[(int64_t)(perm ? perm[p] : p) * ld_src + c];
    float* o = out + i * ld_out + c;
    *o = accumulate ? *o + scale * s : scale * s;
  }
}

// Edge rows [E][width] (COO order, read through the receiver-CSR permutation) -> the 32-edge tiled
// layout of e0t (include/sgnn.h, sgnn_encode_edges): CSR position p holds unit u of its edge at
// tile (p / 32), group 4 (u / 32) + (u % 32) / 8, lane (p % 32) + 32 ((u % 8) / 4), float u % 4.
__global__ __launch_bounds__(kEw) void k_rows_to_tiles(const float* e, int64_t ld, int width, const int32_t* perm,
                                                       const int32_t* rowptr, int64_t n, int64_t cap_items,
                                                       float* e0t) {
  const int64_t E = rowptr[n];
  const int64_t total = cap_items * width;
  for (int64_t t = (int64_t)blockIdx.x * kEw + threadIdx.x; t < total; t += (int64_t)gridDim.x * kEw) {
    const int64_t p = t / width;
    const int u = (int)(t - p * width), uu = u & 31;
    const float v = p < E ? e[(int64_t)(perm ? perm[p] : p) * ld + u] : 0.0f;
    const int64_t tile = p >> 5;
    const int grp = 4 * (u >> 5) + (uu >> 3), lane = (int)(p & 31) + 32 * ((uu >> 2) & 1);
    e0t[tile * 32 * width + grp * 256 + lane * 4 + (uu & 3)] = v;
  }
}

// The inverse: tile position p (< E) -> row perm[p] of out (+)= scale * its units (the edge-latent
// gradient of a module-level block backward back in the caller's COO order).
__global__ __launch_bounds__(kEw) void k_tiles_to_rows(const float* e0t, int width, const int32_t* perm,
                                                       const int32_t* rowptr, int64_t n, int64_t num_edges,
                                                       float scale, float* out, int64_t ld, int accumulate) {
  // the device edge count, bounded by the host's: `out` / `perm` are sized by num_edges
  const int64_t E = min((int64_t)rowptr[n], num_edges);
  const int64_t total = E * width;
  for (int64_t t = (int64_t)blockIdx.x * kEw + threadIdx.x; t < total; t += (int64_t)gridDim.x * kEw) {
    const int64_t p = t / width;
    const int u = (int)(t - p * width), uu = u & 31;
    const int64_t tile = p >> 5;
    const int grp = 4 * (u >> 5) + (uu >> 3), lane = (int)(p & 31) + 32 * ((uu >> 2) & 1);
    const float v = scale * e0t[tile * 32 * width + grp * 256 + lane * 4 + (uu & 3)];
    float* o = out + (int64_t)(perm ? perm[p] : p) * ld + u;
    *o = accumulate ? *o + v : v;
  }
}

}  // namespace

extern "C" int sgnn_edge_tiles_to_rows(const float* e0t, int32_t width, const int32_t* perm, const int32_t* rowptr,
                                       int64_t n, int64_t num_edges, float scale, float* out, int64_t ld,
                                       int32_t accumulate, void* stream) {
  using namespace sgnn;
  if (!rowptr || !e0t || width < 32 || width % 32 != 0 || ld < width || n < 0 || num_edges < 0 ||
      (num_edges > 0 && !out))
    return set_error(SGNN_ERR_INVALID, "edge_tiles_to_rows: bad arguments");
  if (num_edges == 0) return SGNN_OK;
  hipLaunchKernelGGL(k_tiles_to_rows, dim3(ew_grid(num_edges * width)), dim3(kEw), 0, static_cast<hipStream_t>(stream),
                     e0t, width, perm, rowptr, n, num_edges, scale, out, ld, accumulate ? 1 : 0);
  return check_launch("edge_tiles_to_rows");
}

extern "C" int sgnn_edge_rows_to_tiles(const float* e, int64_t ld, int32_t width, const int32_t* perm,
                                       const int32_t* rowptr, int64_t n, int64_t edge_cap, float* e0t, void* stream) {
  using namespace sgnn;
  if (!rowptr || !e0t || width < 32 || width % 32 != 0 || edge_cap < 1 || (ld < width) || n < 0)
    return set_error(SGNN_ERR_INVALID, "edge_rows_to_tiles: bad arguments");
  const int64_t cap_items = 32 * ((edge_cap + 31) / 32);
  hipLaunchKernelGGL(k_rows_to_tiles, dim3(ew_grid(cap_items * width)), dim3(kEw), 0, static_cast<hipStream_t>(stream),
                     e, ld, width, perm, rowptr, n, cap_items, e0t);
  return check_launch("edge_rows_to_tiles");
}

extern "C" size_t sgnn_gemm_workspace_bytes(int64_t M, int64_t N, int64_t K) {
  if (M <= 0 || N <= 0 || K <= 0) return 0;
  const int s = gemm_splits(M, N, K);
  return s > 1 ? sizeof(float) * (size_t)s * (size_t)M * (size_t)N : 0;
}

extern "C" int sgnn_gemm(int32_t trans_a, int32_t trans_b, int64_t M, int64_t N, int64_t K, const float* A,
                         int64_t lda, const float* B, int64_t ldb, const float* bias, int32_t relu, float* C,
                         int64_t ldc, int32_t accumulate, void* workspace, size_t workspace_bytes, void* stream) {
  using namespace sgnn;
  if (M < 0 || N < 0 || K < 0 || !C || ldc < N) return set_error(SGNN_ERR_INVALID, "gemm: bad arguments");
  if (M == 0 || N == 0) return SGNN_OK;
  if (K > 0 && (!A || !B || lda < (trans_a ? M : K) || ldb < (trans_b ? K : N)))
    return set_error(SGNN_ERR_INVALID, "gemm: bad operand");
  if ((N + kTile - 1) / kTile > 65535 || (M + kTile - 1) / kTile > INT32_MAX)
    return set_error(SGNN_ERR_UNSUPPORTED, "gemm: more than 4M columns");
  hipStream_t s = static_cast<hipStream_t>(stream);
  GemmArgs g{A, B, bias, lda, ldb, ldc, M, N, K, C, nullptr, trans_a ? 1 : 0, trans_b ? 1 : 0, relu ? 1 : 0,
             accumulate ? 1 : 0, (K + kKc - 1) / kKc};
  const int nsplit = K > 0 ? gemm_splits(M, N, K) : 1;
  if (nsplit > 1) {
    if (!workspace || workspace_bytes < sgnn_gemm_workspace_bytes(M, N, K))
      return set_error(SGNN_ERR_INVALID, "gemm: workspace smaller than sgnn_gemm_workspace_bytes");
    g.part = static_cast<float*>(workspace);
  }
  const dim3 grid((unsigned)((M + kTile - 1) / kTile), (unsigned)((N + kTile - 1) / kTile), (unsigned)nsplit);
  hipLaunchKernelGGL(k_gemm, grid, dim3(kGemmThreads), 0, s, g);
  if (nsplit > 1) hipLaunchKernelGGL(k_gemm_reduce, dim3(ew_grid(M * N)), dim3(kEw), 0, s, g, nsplit);
  return check_launch("gemm");
}

extern "C" int sgnn_layernorm(const float* x, int64_t n, int32_t width, const float* gamma, const float* beta,
                              const float* residual, float* out, float* yhat, float* rstd, void* stream) {
  using namespace sgnn;
  if (n <= 0) return SGNN_OK;
  if (!x || !gamma || !beta || !out || width < 1) return set_error(SGNN_ERR_INVALID, "layernorm: bad arguments");
  hipLaunchKernelGGL(k_layernorm, dim3(ew_grid(n * 64)), dim3(kEw), 0, static_cast<hipStream_t>(stream), x, n,
                     width, gamma, beta, residual, out, yhat, rstd);
  return check_launch("layernorm");
}

extern "C" int sgnn_layernorm_bwd(const float* dout, const float* yhat, const float* rstd, const float* gamma,
                                  int64_t n, int32_t width, float* dx, void* stream) {
  using namespace sgnn;
  if (n <= 0) return SGNN_OK;
  if (!dout || !yhat || !rstd || !gamma || !dx || width < 1)
    return set_error(SGNN_ERR_INVALID, "layernorm_bwd: bad arguments");
  hipLaunchKernelGGL(k_layernorm_bwd, dim3(ew_grid(n * 64)), dim3(kEw), 0, static_cast<hipStream_t>(stream), dout,
                     yhat, rstd, gamma, n, width, dx);
  return check_launch("layernorm_bwd");
}

extern "C" size_t sgnn_colsum_workspace_bytes(int64_t n, int32_t width) {
  if (n <= 0 || width <= 0) return 0;
  return sizeof(float) * (size_t)((n + kColRows - 1) / kColRows) * (size_t)width;
}

extern "C" int sgnn_colsum(const float* x, int64_t ldx, const float* mul, int64_t ldm, int64_t n, int32_t width,
                           float* out, int32_t accumulate, void* workspace, size_t workspace_bytes, void* stream) {
  using namespace sgnn;
  if (width < 1 || !out) return set_error(SGNN_ERR_INVALID, "colsum: bad arguments");
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (n <= 0) {
    if (!accumulate && hipMemsetAsync(out, 0, sizeof(float) * width, s) != hipSuccess)
      return check_launch("colsum: zero");
    return SGNN_OK;
  }
  if (!x || ldx < width || (mul && ldm < width) || !workspace ||
      workspace_bytes < sgnn_colsum_workspace_bytes(n, width))
    return set_error(SGNN_ERR_INVALID, "colsum: bad operand or workspace");
  const int64_t nblk = (n + kColRows - 1) / kColRows;
  float* part = static_cast<float*>(workspace);
  hipLaunchKernelGGL(k_colsum_part, dim3((unsigned)nblk), dim3(kEw), 0, s, x, ldx, mul, ldm, n, width, part);
  hipLaunchKernelGGL(k_colsum_reduce, dim3((unsigned)((width + kEw - 1) / kEw)), dim3(kEw), 0, s, part, nblk, width,
                     out, accumulate ? 1 : 0);
  return check_launch("colsum");
}

extern "C" int sgnn_relu_bwd(float* dy, int64_t ldd, const float* y, int64_t ldy, int64_t n, int32_t width,
                             void* stream) {
  using namespace sgnn;
  if (n <= 0) return SGNN_OK;
  if (!dy || !y || width < 1 || ldd < width || ldy < width) return set_error(SGNN_ERR_INVALID, "relu_bwd: bad arguments");
  hipLaunchKernelGGL(k_relu_bwd, dim3(ew_grid(n * width)), dim3(kEw), 0, static_cast<hipStream_t>(stream), dy, ldd, y,
                     ldy, n, width);
  return check_launch("relu_bwd");
}

extern "C" int sgnn_gather_rows(const float* src, int64_t ld_src, int32_t width, const int32_t* index, int64_t nrows,
                                float scale, float* out, int64_t ld_out, void* stream) {
  using namespace sgnn;
  if (nrows <= 0) return SGNN_OK;
  if (!src || !out || width < 1 || ld_src < width || ld_out < width)
    return set_error(SGNN_ERR_INVALID, "gather_rows: bad arguments");
  hipLaunchKernelGGL(k_gather_rows, dim3(ew_grid(nrows * width)), dim3(kEw), 0, static_cast<hipStream_t>(stream), src,
                     ld_src, width, index, nrows, scale, out, ld_out);
  return check_launch("gather_rows");
}

extern "C" int sgnn_segment_sum_cols(const float* src, int64_t ld_src, int32_t width, const int32_t* rowptr,
                                     const int32_t* perm, int64_t n, float scale, float* out, int64_t ld_out,
                                     int32_t accumulate, void* stream) {
  using namespace sgnn;
  if (n <= 0) return SGNN_OK;
  if (!src || !rowptr || !out || width < 1 || ld_src < width || ld_out < width)
    return set_error(SGNN_ERR_INVALID, "segment_sum_cols: bad arguments");
  hipLaunchKernelGGL(k_segment_sum_cols, dim3(ew_grid(n * width)), dim3(kEw), 0, static_cast<hipStream_t>(stream), src,
                     ld_src, width, rowptr, perm, n, scale, out, ld_out, accumulate ? 1 : 0);
  return check_launch("segment_sum_cols");
}
